// oracle/oracle_capi.cpp -- C entry points of the CPU oracle, for tests/ and
// bench.py's cpu_baseline leg only (loaded with ctypes).  TEST INFRASTRUCTURE:
// never linked into the product.  See oracle.hpp for what is restated and the
// "parity unpinned" status.
#include "oracle.hpp"
#include "oracle_exact.hpp"

#include <chrono>
#include <cstdio>
#include <exception>

using namespace lzo;

extern "C" {

// Full 3-approximation (p = 1 semantics).  out: 2*cap uint32 (src,len pairs).
// stats (optional, 16 x uint32): size_sss, has_runs, num_lpf, len_lpf_phr,
//   num_gaps, patt_lens[5], roll_threshold, log2_size_h.
// Returns number of factors, or -1 on error / capacity overflow.
int64_t oracle_factorize_approx(uint8_t* T, uint64_t n, int phr_mode, uint32_t rk_seed,
                                uint32_t* out, uint64_t cap, uint32_t* stats) {
    try {
        uint64_t k = 0;
        bool overflow = false;
        approx_stats st;
        factorize_approximate(T, (u32)n, phr_mode, rk_seed, [&](factor f) {
            if (k < cap) { out[2 * k] = f.src; out[2 * k + 1] = f.len; } else overflow = true;
            k++;
        }, &st);
        if (stats) {
            stats[0] = st.size_sss; stats[1] = st.has_runs; stats[2] = st.num_lpf;
            stats[3] = st.len_lpf_phr; stats[4] = st.num_gaps;
            for (int i = 0; i < 5; i++) stats[5 + i] = st.patt_lens[i];
            stats[10] = st.roll_threshold; stats[11] = st.log2_size_h;
        }
        return overflow ? -1 : (int64_t)k;
    } catch (const std::exception& e) {
        std::fprintf(stderr, "oracle error: %s\n", e.what());
        return -1;
    }
}

// The p-thread CPU-baseline leg's stream (LPF in p partitions, the reference's racy parallel
// greedy where lz77_sss.hpp:467-474 selects it): for the validity tests of the timing leg only.
// *par = 1 when the parallel greedy ran.  Returns the factor count, -1 on error / overflow.
int64_t oracle_factorize_p(uint8_t* T, uint64_t n, int p, uint32_t rk_seed, uint32_t* out, uint64_t cap, int* par) {
    try {
        const int prev = omp_get_max_threads();
        omp_set_num_threads(std::max(1, p));
        uint64_t k = 0;
        bool overflow = false;
        approx_stats st;
        factorize_approximate(T, (u32)n, lpf_opt, rk_seed, [&](factor f) {
            if (k < cap) { out[2 * k] = f.src; out[2 * k + 1] = f.len; } else overflow = true;
            k++;
        }, &st, 1, std::max(1, p));
        omp_set_num_threads(prev);
        if (par) *par = st.greedy_parallel;
        return overflow ? -1 : (int64_t)k;
    } catch (const std::exception& e) {
        std::fprintf(stderr, "oracle error: %s\n", e.what());
        return -1;
    }
}

// pos_t = uint64_t form (lz77_sss<uint64_t>): out 2*cap uint64 pairs, stats 12 x uint64.
int64_t oracle_factorize_approx64(uint8_t* T, uint64_t n, int phr_mode, uint32_t rk_seed, int fact_mode,
                                  uint64_t* out, uint64_t cap, uint64_t* stats) {
    try {
        uint64_t k = 0;
        bool overflow = false;
        approx_stats st;
        factorize_approximate<u64>(T, (u64)n, phr_mode, rk_seed, [&](factor_t<u64> f) {
            if (k < cap) { out[2 * k] = f.src; out[2 * k + 1] = f.len; } else overflow = true;
            k++;
        }, &st, fact_mode);
        if (stats) {
            stats[0] = st.size_sss; stats[1] = st.has_runs; stats[2] = st.num_lpf;
            stats[3] = st.len_lpf_phr; stats[4] = st.num_gaps;
            for (int i = 0; i < 5; i++) stats[5 + i] = st.patt_lens[i];
            stats[10] = st.roll_threshold; stats[11] = st.log2_size_h;
        }
        return overflow ? -1 : (int64_t)k;
    } catch (const std::exception& e) {
        std::fprintf(stderr, "oracle error: %s\n", e.what());
        return -1;
    }
}

// One block of the sharded greedy (oracle.hpp greedy_block).  table: the carried table
// (pos + 1; uint32 entries, or uint64 for wide), table_entries its length (0: empty, the
// block sizes it; the needed length is returned in *table_entries when it differs).
// state: [start, idxpos, end] in, [exit_start, exit_idxpos] out in state[3..4].
// Returns the factor count (out: 2*cap uint64), -1 on overflow, -2 if the table is too small.
int64_t oracle_greedy_block(uint8_t* T, uint64_t n, int phr_mode, uint32_t rk_seed, int wide, uint64_t* state,
                            void* table, uint64_t* table_entries, uint64_t* out, uint64_t cap) {
    try {
        uint64_t k = 0;
        bool overflow = false;
        auto run = [&](auto zero) -> int64_t {
            using Q = decltype(zero);
            std::vector<Q> H;
            Q* tab = (Q*)table;
            if (*table_entries) H.assign(tab, tab + *table_entries);
            Q es = 0, ei = 0;
            greedy_block<Q>(T, (Q)n, phr_mode, rk_seed, (Q)state[0], (Q)state[1], (Q)state[2], H, es, ei,
                            [&](factor_t<Q> f) {
                                if (k < cap) { out[2 * k] = f.src; out[2 * k + 1] = f.len; } else overflow = true;
                                k++;
                            });
            state[3] = es;
            state[4] = ei;
            if (H.size() != *table_entries) {
                const bool fits = tab && H.size() <= *table_entries;
                *table_entries = H.size();
                if (!fits) return -2;
            }
            std::copy(H.begin(), H.end(), tab);
            return overflow ? -1 : (int64_t)k;
        };
        return wide ? run((u64)0) : run((u32)0);
    } catch (const std::exception& e) {
        std::fprintf(stderr, "oracle error: %s\n", e.what());
        return -3;
    }
}

// SSS with 64-bit positions and the LPF_opt phrases of pos_t = uint64_t (tests)
int64_t oracle_sss64(const uint8_t* T, uint64_t n, uint64_t* out, uint64_t cap, int* has_runs) {
    bool hr = false;
    std::vector<u64> S = compute_sss<u64>(T, n, hr);
    if (has_runs) *has_runs = hr;
    if (S.size() > cap) return -1;
    std::copy(S.begin(), S.end(), out);
    return (int64_t)S.size();
}
int64_t oracle_lpf_opt64(const uint8_t* T, uint64_t n, uint64_t* out, uint64_t cap) {
    lce_structure<u64> L;
    L.build(T, n);
    auto P = build_lpf_opt(T, n, L);
    if (P.size() > cap) return -1;
    for (size_t k = 0; k < P.size(); k++) { out[3 * k] = P[k].beg; out[3 * k + 1] = P[k].end; out[3 * k + 2] = P[k].src; }
    return (int64_t)P.size();
}

// fact_mode = skip_phrases (gapped stream).  Returns the record count or -1.
int64_t oracle_factorize_skip(uint8_t* T, uint64_t n, int phr_mode, uint32_t* out, uint64_t cap) {
    try {
        uint64_t k = 0;
        bool overflow = false;
        factorize_approximate(T, (u32)n, phr_mode, 42, [&](factor f) {
            if (k < cap) { out[2 * k] = f.src; out[2 * k + 1] = f.len; } else overflow = true;
            k++;
        }, nullptr, 2);
        return overflow ? -1 : (int64_t)k;
    } catch (const std::exception& e) {
        std::fprintf(stderr, "oracle error: %s\n", e.what());
        return -1;
    }
}

// Exact greedy LZ77 (factorize_exact restatement, oracle.hpp).  Returns z or -1 (cap too small).
int64_t oracle_factorize_exact(const uint8_t* T, uint64_t n, uint32_t* out, uint64_t cap) {
    std::vector<factor> F = factorize_exact(T, n);
    if (F.size() > cap) return -1;
    for (size_t k = 0; k < F.size(); k++) { out[2 * k] = F[k].src; out[2 * k + 1] = F[k].len; }
    return (int64_t)F.size();
}
// Same, timed (cpu_baseline of the exact mode): factor count, seconds.
int64_t oracle_factorize_exact_timed(const uint8_t* T, uint64_t n, double* seconds) {
    const double t0 = omp_get_wtime();
    std::vector<factor> F = factorize_exact(T, n);
    *seconds = omp_get_wtime() - t0;
    return (int64_t)F.size();
}

// The reference's exact transform restated (oracle_exact.hpp): factorize_exact<greedy, lpf_opt,
// with_samples (mode 1) | without_samples (mode 2)> at p threads (p = 1: the deterministic stream).
// Returns z or -1 (cap too small / error).
int64_t oracle_factorize_exact_smpl(uint8_t* T, uint64_t n, int mode, int p, uint32_t* out, uint64_t cap) {
    try {
        if (n >= 0xFFFFFFF0ull) return -1;
        std::vector<factor> F = factorize_exact_smpl(T, (u32)n, mode, p);
        if (F.size() > cap) return -1;
        for (size_t k = 0; k < F.size(); k++) { out[2 * k] = F[k].src; out[2 * k + 1] = F[k].len; }
        return (int64_t)F.size();
    } catch (const std::exception& e) {
        std::fprintf(stderr, "oracle error: %s\n", e.what());
        return -1;
    }
}
// Same, timed (cpu_baseline of bench.py --mode exact): factor count; seconds for the whole call and
// for its approximation stage.
int64_t oracle_factorize_exact_smpl_timed(uint8_t* T, uint64_t n, int mode, int p, double* seconds,
                                          double* seconds_aprx) {
    try {
        if (n >= 0xFFFFFFF0ull) return -1;
        const double t0 = omp_get_wtime();
        std::vector<factor> F = factorize_exact_smpl(T, (u32)n, mode, p, seconds_aprx);
        *seconds = omp_get_wtime() - t0;
        return (int64_t)F.size();
    } catch (const std::exception& e) {
        std::fprintf(stderr, "oracle error: %s\n", e.what());
        return -1;
    }
}

// Factor count and wall time only (cpu_baseline); also returns an FNV-1a hash of the stream.
int64_t oracle_factorize_timed(uint8_t* T, uint64_t n, int phr_mode, uint32_t rk_seed,
                               double* seconds, uint64_t* stream_hash) {
    uint64_t k = 0, h = 1469598103934665603ull;
    auto t0 = std::chrono::steady_clock::now();
    factorize_approximate(T, (u32)n, phr_mode, rk_seed, [&](factor f) {
        k++;
        uint32_t w[2] = {f.src, f.len};
        const uint8_t* p = (const uint8_t*)w;
        for (int i = 0; i < 8; i++) { h ^= p[i]; h *= 1099511628211ull; }
    });
    auto t1 = std::chrono::steady_clock::now();
    if (seconds) *seconds = std::chrono::duration<double>(t1 - t0).count();
    if (stream_hash) *stream_hash = h;
    return (int64_t)k;
}

// The CPU baseline at p threads: every OpenMP stage of the
// restatement on p threads, and for p > 1 the LPF phrases in p partitions
// (lpf_opt.cpp:46-56).  The greedy emitter stays sequential: the reference's parallel
// gap index (lz77_sss.hpp:470-474, run-free texts only) is not restated.  Timing only.
int64_t oracle_factorize_timed_p(uint8_t* T, uint64_t n, int phr_mode, uint32_t rk_seed, int p,
                                 double* seconds, uint64_t* stream_hash, int* par) {
    const int prev = omp_get_max_threads();
    omp_set_num_threads(std::max(1, p));
    uint64_t k = 0, h = 1469598103934665603ull;
    approx_stats st;
    auto t0 = std::chrono::steady_clock::now();
    factorize_approximate(T, (u32)n, phr_mode, rk_seed, [&](factor f) {
        k++;
        uint32_t w[2] = {f.src, f.len};
        const uint8_t* q = (const uint8_t*)w;
        for (int i = 0; i < 8; i++) { h ^= q[i]; h *= 1099511628211ull; }
    }, &st, 1, std::max(1, p));
    auto t1 = std::chrono::steady_clock::now();
    omp_set_num_threads(prev);
    if (par) *par = st.greedy_parallel;
    if (seconds) *seconds = std::chrono::duration<double>(t1 - t0).count();
    if (stream_hash) *stream_hash = h;
    return (int64_t)k;
}

// The same CPU baseline with pos_t = uint64_t (configs[3]'s chr19-style text past 4 GiB): every
// OpenMP stage on p threads, LPF in p partitions, the greedy sequential unless lz77_sss.hpp:467-474
// selects the reference's parallel one.  Timing only.
int64_t oracle_factorize_timed_p64(uint8_t* T, uint64_t n, int phr_mode, uint32_t rk_seed, int p,
                                   double* seconds, uint64_t* stream_hash, int* par) {
    try {
        const int prev = omp_get_max_threads();
        omp_set_num_threads(std::max(1, p));
        uint64_t k = 0, h = 1469598103934665603ull;
        approx_stats st;
        auto t0 = std::chrono::steady_clock::now();
        factorize_approximate<u64>(T, (u64)n, phr_mode, rk_seed, [&](factor_t<u64> f) {
            k++;
            const uint64_t w[2] = {f.src, f.len};
            const uint8_t* q = (const uint8_t*)w;
            for (int i = 0; i < 16; i++) { h ^= q[i]; h *= 1099511628211ull; }
        }, &st, 1, std::max(1, p));
        auto t1 = std::chrono::steady_clock::now();
        omp_set_num_threads(prev);
        if (par) *par = st.greedy_parallel;
        if (seconds) *seconds = std::chrono::duration<double>(t1 - t0).count();
        if (stream_hash) *stream_hash = h;
        return (int64_t)k;
    } catch (const std::exception& e) {
        std::fprintf(stderr, "oracle error: %s\n", e.what());
        return -1;
    }
}

// SSS only.  Returns |S| (or -1 if cap too small); *has_runs set.
int64_t oracle_sss(const uint8_t* T, uint64_t n, uint32_t* out, uint64_t cap, int* has_runs) {
    bool hr = false;
    std::vector<u32> S = compute_sss(T, n, hr);
    if (has_runs) *has_runs = hr;
    if (S.size() > cap) return -1;
    std::copy(S.begin(), S.end(), out);
    return (int64_t)S.size();
}

// Q membership by brute force for j in [0, n-tau] (tests).  q: n-tau+1 bytes.
void oracle_q_bruteforce(const uint8_t* T, uint64_t n, uint8_t* q) {
    if (n < TAU) return;
    for (u64 j = 0; j + TAU <= n; j++) q[j] = q_bruteforce(T, j);
}
// Phi' (tests): phi[j] for j in [0, n-tau], SSS_INF = 2^32-1 for Q
void oracle_phi(const uint8_t* T, uint64_t n, uint64_t* phi) {
    if (n < TAU) return;
    const u32 bp = pow32((u32)SSS_BASE, TAU);
    u32 fp = 0;
    for (u64 k = 0; k < TAU; k++) fp = fp * (u32)SSS_BASE + T[k];
    for (u64 j = 0; j + TAU <= n; j++) {
        phi[j] = q_bruteforce(T, j) ? SSS_INF : fp;
        if (j + TAU < n) fp = fp * (u32)SSS_BASE + T[j + TAU] - bp * T[j];
    }
}

// SA_S / ISA_S / LCP_S (tests).  Each array has cap entries.
int64_t oracle_sa_s(const uint8_t* T, uint64_t n, uint32_t* S, uint32_t* SA, uint32_t* LCP, uint64_t cap) {
    lce_structure<> L;
    L.build(T, n);
    if (L.s() > cap) return -1;
    std::copy(L.S.begin(), L.S.end(), S);
    std::copy(L.SA.begin(), L.SA.end(), SA);
    std::copy(L.LCP.begin(), L.LCP.end(), LCP);
    return L.s();
}

// Exact LCE for query pairs (tests).
void oracle_lce(const uint8_t* T, uint64_t n, const uint32_t* qi, const uint32_t* qj, uint64_t nq, uint32_t* out) {
    lce_structure<> L;
    L.build(T, n);
    for (u64 k = 0; k < nq; k++) out[k] = (u32)L.lce(qi[k], qj[k]);
}

// LPF phrase list after build_LPF_opt (tests); out: 3*cap (beg,end,src)
int64_t oracle_lpf_opt(const uint8_t* T, uint64_t n, uint32_t* out, uint64_t cap) {
    lce_structure<> L;
    L.build(T, n);
    auto P = build_lpf_opt(T, n, L);
    if (P.size() > cap) return -1;
    for (size_t k = 0; k < P.size(); k++) { out[3 * k] = P[k].beg; out[3 * k + 1] = P[k].end; out[3 * k + 2] = P[k].src; }
    return (int64_t)P.size();
}

void oracle_decode(const uint32_t* f, uint64_t nf, uint8_t* out, uint64_t n) {
    decode(reinterpret_cast<const factor*>(f), nf, out, n);
}

void oracle_gap_bases(uint32_t rk_seed, uint64_t* out5) {
    auto b = gap_bases(rk_seed);
    for (int i = 0; i < 5; i++) out5[i] = b[i];
}

int oracle_num_threads(void) {
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}

}  // extern "C"
