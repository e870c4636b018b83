// greedy.hip -- the gap-filling factor emitter (factorize_greedy,
// include/lz77_sss/algorithms/approximate/factorize/greedy.cpp:34-140 with
// longest_prev_occ, factorize/common.cpp:33-61, and the single-slot hash
// index rolling_hash_index_107, data_structures/rolling_hash_index_107.hpp:33-172),
// reproduced exactly for num_threads = 1.
//
// The reference walks gaps sequentially against a hash table H that every
// visited gap position writes (5 Karp-Rabin fingerprints mod 2^107-1).  A
// query at position q only ever reads "the last position inserted into slot
// s before q".  So, for a GIVEN set I of inserted positions, all lookups are
// fixed by one stable radix sort of the (slot, position) entries of I.  The
// engine therefore iterates:
//
//   1. speculate I (initially: every gap position [phrase end, next phrase beg])
//   2. k_slots + radix sort + k_occ  -> occ5[q][x] for every q in I
//   3. k_walk (DRY): every walk segment (a gap walk + the LPF factors up to
//      the next gap) runs in parallel from its assumed start state
//   4. the host links segments into the chain starting at position 0; unknown
//      start states become new segments (speculatively, all at once)
//   5. I' = positions actually inserted along the chain.  I' == I means every
//      lookup used in the chain was exact -> k_walk (WRITE) emits the factors.
//      Otherwise I <- I' and repeat.
//
// The last 64 positions (the text tail, where the reference's stale / zeroed
// fingerprints and conditional inserts live, rolling_hash_index_107.hpp:80-150)
// are walked by one thread (k_tail) with an exact local model of the table.
#include "../include/engine.h"
#include "../include/lce_dev.h"

#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <array>
#include <cmath>
#include <cstring>
#include <limits>
#include <random>
#include <unordered_map>

namespace lz {

// ---------------------------------------------------------------------------
// 107-bit Mersenne arithmetic (rolling_hash.hpp uses mersenne::mod, absent
// upstream; canonical residues in [0, 2^107-1))
static constexpr u128 P107 = ((u128)1 << 107) - 1;
__host__ __device__ static inline u128 mod107(u128 x) {
    x = (x & P107) + (x >> 107);
    x = (x & P107) + (x >> 107);
    return x >= P107 ? x - P107 : x;
}
static u128 mulmod107_host(u128 a, u128 b) {
    u128 r = 0;
    for (int bit = 106; bit >= 0; bit--) {
        r = mod107(r << 1);
        if ((b >> bit) & 1) r = mod107(r + a);
    }
    return r;
}
static u128 powmod107_host(u128 b, u64 e) {
    u128 r = 1;
    while (e) {
        if (e & 1) r = mulmod107_host(r, b);
        b = mulmod107_host(b, b);
        e >>= 1;
    }
    return r;
}

struct gap_cfg {
    u32 n, nt;          // text length, start of the tail region
    u32 lens[5];
    u64 base[5];
    u32 thr;            // roll_threshold
    u32 mask;           // slot mask (2^k - 1)
    const u128* negpow; // [5][256]: -(o * b^len) mod P
};

__device__ __forceinline__ u128 kr_roll(u128 fp, u64 b, u128 negpow_out, u32 in) {
    return mod107(fp * b + mod107((u128)in + negpow_out));
}
// Phi_x(T[q..q+len)) mod P, direct evaluation (roll-ins only)
__device__ __forceinline__ u128 kr_direct(const u8* T, u64 q, u32 len, u64 b) {
    u128 fp = 0;
    for (u32 j = 0; j < len; j++) fp = mod107(fp * b + T[q + j]);
    return fp;
}

// ---------------------------------------------------------------------------
// 2. entries of I: one thread per chunk of an interval
struct ichunk { u32 q0, q1, rank0; };

__global__ void k_slots(const u8* __restrict__ T, gap_cfg G, const ichunk* __restrict__ chunks, u32 nch,
                        u32* __restrict__ keys, u32* __restrict__ vals, u32* __restrict__ ipos) {
    const u64 c = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= nch) return;
    const ichunk ch = chunks[c];
    u128 fp[5];
#pragma unroll
    for (int x = 0; x < 5; x++) fp[x] = kr_direct(T, ch.q0, G.lens[x], G.base[x]);
    for (u32 q = ch.q0; q < ch.q1; q++) {
        const u32 rank = ch.rank0 + (q - ch.q0);
        ipos[rank] = q;
#pragma unroll
        for (int x = 4; x >= 0; x--) {
            const u32 e = 5 * rank + (4 - x);
            keys[e] = (u32)((u64)fp[x] & G.mask);
            vals[e] = e;
        }
        if (q + 1 < ch.q1) {
#pragma unroll
            for (int x = 0; x < 5; x++)
                fp[x] = kr_roll(fp[x], G.base[x], G.negpow[x * 256 + T[q]], T[q + G.lens[x]]);
        }
    }
}

__global__ void k_occ(const u32* __restrict__ skeys, const u32* __restrict__ svals, const u32* __restrict__ ipos,
                      u64 m, u32* __restrict__ occ5) {
    const u64 t = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= m) return;
    const u32 e = svals[t];
    u32 o = NONE;
    if (t > 0 && skeys[t - 1] == skeys[t]) o = ipos[svals[t - 1] / 5];
    occ5[e] = o;
}

// ---------------------------------------------------------------------------
// 3. walks
struct walk_ctx {
    const u8* T;
    gap_cfg G;
    const u32* P;        // phrases (beg,end,src) + sentinel
    const u32* occ5;
    const u32* istart;   // interval starts of I (sorted)
    const u32* iend;     // interval ends (exclusive)
    const u32* irank;    // rank of istart
    u32 nint;
    lce_view L;
    // tail-model support
    const u32* skeys;    // sorted slot keys
    const u32* svals;
    const u32* ipos;
    u64 nentries;
};

__device__ __forceinline__ u32 interval_rank(const walk_ctx& W, u32 q, int& hint) {
    // interval containing q; hint caches the last one
    if (hint >= 0 && q >= W.istart[hint] && q < W.iend[hint]) return W.irank[hint] + (q - W.istart[hint]);
    u32 lo = 0, hi = W.nint;
    while (lo < hi) {
        u32 mid = (lo + hi) >> 1;
        if (W.istart[mid] <= q) lo = mid + 1; else hi = mid;
    }
    if (lo == 0) return NONE;
    const u32 k = lo - 1;
    if (q >= W.iend[k]) return NONE;
    hint = (int)k;
    return W.irank[k] + (q - W.istart[k]);
}

template <bool WRITE>
__device__ void walk_segment(const walk_ctx& W, seg_in in, seg_out& out, u32* fout) {
    const u8* T = W.T;
    const u32 n = W.G.n, nt = W.G.nt;
    const u32* P = W.P;
    u32 i = in.start, p = in.p, idx = in.idxpos, zm = in.zmask;
    u32 nf = 0, ns = 0, flags = 0, e = in.start;
    int hint = -1;
    out.next = n;
    u64 guard = 0;
    const u64 guard_max = 4ull * n + 1024;
    auto emit = [&](u32 src, u32 len) {
        if (WRITE) { fout[2 * nf] = src; fout[2 * nf + 1] = len; }
        nf++;
    };
    auto query = [&](u32 q, u32& fsrc, u32& flen) {
        fsrc = T[q];
        flen = 0;
        const u32 rk = interval_rank(W, q, hint);
        if (rk == NONE) return;  // q not in I: speculation miss, fixed by the next round
        for (int x = 4; x >= 0; x--) {
            const u32 occ = W.occ5[5 * (u64)rk + (4 - x)];
            if (occ != NONE && occ < q && T[occ] == T[q]) {
                flen = (u32)dev_lce(W.L, occ, q);
                fsrc = occ;
                return;
            }
        }
    };
    for (;;) {
        u32 gap_end = P[3 * p];
        if (i < gap_end) {
            if (idx < i) {
                if (i - idx > W.G.thr) {  // reinit (only matters in the tail region)
                    zm = 0;
                    for (int x = 0; x < 5; x++) zm |= ((u64)i + W.G.lens[x] >= n) ? (1u << x) : 0u;
                }
                idx = i;
            }
            do {
                if (i >= nt) { flags |= 1; out.flags = flags; return; }
                if (++guard > guard_max || i > n) { out.flags = flags | 4; return; }
                u32 fsrc, flen;
                query(i, fsrc, flen);
                idx = i + 1;
                i += flen ? flen : 1;
                if (i > gap_end) {
                    if (i <= P[3 * p + 1]) {
                        flen -= i - gap_end;
                        i = gap_end;
                    } else {
                        do { p++; } while (P[3 * p + 1] <= i);
                        gap_end = P[3 * p];
                    }
                }
                emit(fsrc, flen);
                if (idx < i) idx = i;
            } while (i < gap_end);
            e = i;
        }
        if (i == n) break;
        const u32 exc = i - gap_end;
        u32 lsrc = P[3 * p + 2] + exc, llen = (P[3 * p + 1] - P[3 * p]) - exc;
        if (idx == i) {
            if (i >= nt) { flags |= 1; out.flags = flags; return; }
            u32 fsrc, flen;
            query(i, fsrc, flen);
            idx = i + 1;
            if (ns < 4) out.single[ns] = i; else flags |= 2;
            ns++;
            if (flen > llen) { lsrc = fsrc; llen = flen; }
        }
        emit(lsrc, llen);
        i += llen;
        if (++guard > guard_max || i > n || llen == 0) { out.flags = flags | 4; return; }
        while (P[3 * p + 1] <= i) p++;
        if (i < P[3 * p]) { out.next = i; break; }
    }
    out.e = e;
    out.nfact = nf;
    out.idxpos = idx;
    out.zmask = zm;
    out.nsingle = ns;
    out.flags = flags;
}

template <bool WRITE>
__global__ void k_walk(walk_ctx W, const seg_in* __restrict__ segs, const u32* __restrict__ ids, u32 nseg,
                       seg_out* __restrict__ outs, const u64* __restrict__ offs, u32* __restrict__ fact) {
    const u64 t = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= nseg) return;
    const u32 g = ids ? ids[t] : (u32)t;
    seg_out o;
    o.flags = 0;
    o.e = segs[g].start;
    o.nfact = 0;
    walk_segment<WRITE>(W, segs[g], o, WRITE ? fact + 2 * offs[t] : nullptr);
    if (!WRITE) outs[g] = o;
}

// ---------------------------------------------------------------------------
// exact single-thread walk from a segment start to the end of the text,
// modelling the table in the tail region (last 64 positions)
struct tail_ins { u32 slot, pos; };
constexpr int TAIL_CAP = 64 * 5 + 8;

__device__ u32 last_global_in_slot(const walk_ctx& W, u32 slot) {
    // last entry with key == slot in the sorted key array
    u64 lo = 0, hi = W.nentries;
    while (lo < hi) {
        u64 mid = (lo + hi) >> 1;
        if (W.skeys[mid] <= slot) lo = mid + 1; else hi = mid;
    }
    if (lo == 0 || W.skeys[lo - 1] != slot) return NONE;
    return W.ipos[W.svals[lo - 1] / 5];
}

__global__ void k_tail(walk_ctx W, seg_in in, u32* __restrict__ fact, u64 off, u64* __restrict__ count_out,
                       u32* __restrict__ ins_out /* [start, e) + singles, cap 8 */) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    const u8* T = W.T;
    const u32 n = W.G.n, nt = W.G.nt;
    const u32* P = W.P;
    tail_ins loc[TAIL_CAP];
    int nloc = 0;
    u32 i = in.start, p = in.p, idx = in.idxpos, zm = in.zmask;
    u64 nf = 0;
    int hint = -1;
    u32 nins = 0;
    auto fp_slot = [&](u32 q, int x) -> u32 {
        const u32 len = W.G.lens[x];
        if (zm >> x & 1) return 0;
        const u64 qq = ((u64)q + len <= n) ? q : (n >= len ? n - len : 0);
        if ((u64)len > n) return 0;
        return (u32)((u64)kr_direct(T, qq, len, W.G.base[x]) & W.G.mask);
    };
    auto lookup = [&](u32 q, int x, u32 slot) -> u32 {
        for (int k = nloc - 1; k >= 0; k--)
            if (loc[k].slot == slot) return loc[k].pos;
        if (q < nt) {
            const u32 rk = interval_rank(W, q, hint);
            return rk == NONE ? NONE : W.occ5[5 * (u64)rk + (4 - x)];
        }
        return last_global_in_slot(W, slot);
    };
    auto insert = [&](u32 q, u32 slot) {
        if (nloc < TAIL_CAP) loc[nloc++] = {slot, q};
    };
    auto query = [&](u32 q, u32& fsrc, u32& flen) {
        fsrc = T[q];
        flen = 0;
        bool hit = false;
        for (int x = 4; x >= 0; x--) {
            if (!hit) {
                const u32 slot = (q >= nt) ? fp_slot(q, x) : 0;
                const u32 occ = lookup(q, x, slot);
                if (q >= nt) insert(q, slot);
                if (occ != NONE && occ < q && T[occ] == T[q]) {
                    flen = (u32)dev_lce(W.L, occ, q);
                    fsrc = occ;
                    hit = true;
                }
            } else if (q >= nt && (u64)q + W.G.lens[x] < n) {
                insert(q, fp_slot(q, x));
            }
        }
    };
    auto advance_to = [&](u32 target) {
        for (; idx < target; idx++)
            if (idx >= nt)
                for (int x = 0; x < 5; x++)
                    if ((u64)idx + W.G.lens[x] < n) insert(idx, fp_slot(idx, x));
    };
    auto emit = [&](u32 src, u32 len) {
        fact[2 * (off + nf)] = src;
        fact[2 * (off + nf) + 1] = len;
        nf++;
    };
    // inserted intervals below the tail region (the only ones the speculated
    // set I has to contain): recorded as [a, b) pairs, capacity 8
    auto record = [&](u32 a, u32 b) {
        if (a >= nt || a >= b) return;
        if (nins > 0 && ins_out[2 * (nins - 1) + 1] >= a) {
            ins_out[2 * (nins - 1) + 1] = max(ins_out[2 * (nins - 1) + 1], b);
            return;
        }
        if (nins < 8) { ins_out[2 * nins] = a; ins_out[2 * nins + 1] = b; nins++; }
        else count_out[2] = 1;  // overflow (cannot happen: see DESIGN.md 4.5)
    };
    count_out[2] = 0;
    u64 guard = 0;
    for (;;) {
        if (++guard > 4ull * n + 1024 || i > n) { count_out[2] = 2; break; }
        u32 gap_end = P[3 * p];
        if (i < gap_end) {
            if (idx < i) {
                if (i - idx > W.G.thr) {
                    zm = 0;
                    for (int x = 0; x < 5; x++) zm |= ((u64)i + W.G.lens[x] >= n) ? (1u << x) : 0u;
                }
                idx = i;  // roll: fingerprints advance, nothing inserted
            }
            const u32 walk_start = i;
            do {
                u32 fsrc, flen;
                query(i, fsrc, flen);
                idx = i + 1;
                i += flen ? flen : 1;
                if (i > gap_end) {
                    if (i <= P[3 * p + 1]) {
                        flen -= i - gap_end;
                        i = gap_end;
                    } else {
                        do { p++; } while (P[3 * p + 1] <= i);
                        advance_to(gap_end);
                        gap_end = P[3 * p];
                    }
                }
                emit(fsrc, flen);
                advance_to(i);
            } while (i < gap_end);
            record(walk_start, i);
        }
        if (i == n) break;
        const u32 exc = i - gap_end;
        u32 lsrc = P[3 * p + 2] + exc, llen = (P[3 * p + 1] - P[3 * p]) - exc;
        if (idx == i) {
            u32 fsrc, flen;
            query(i, fsrc, flen);
            idx = i + 1;
            record(i, i + 1);
            if (flen > llen) { lsrc = fsrc; llen = flen; }
        }
        emit(lsrc, llen);
        i += llen;
        while (P[3 * p + 1] <= i) p++;
    }
    count_out[0] = nf;
    count_out[1] = nins;
}

// ---------------------------------------------------------------------------
// host side
struct gap_params_h {
    std::array<u32, 5> patt_lens{};
    u32 roll_threshold = 0;
    u32 log2_size_h = 0;
};

// lz77_sss.hpp:99-122, 425-461 and rolling_hash_index_107.hpp:59-70 (pos_t =
// uint32_t, malloc_count_peak() - malloc_count_current() == 0)
static gap_params_h choose_gap_params(u32 n, u32 num_lpf, u32 len_lpf_phr, u32 num_gaps) {
    static const std::array<std::pair<double, std::array<u32, 5>>, 10> table{{
        {6, {2, 3, 4, 5, 6}}, {8, {2, 3, 4, 6, 8}}, {12, {2, 3, 4, 8, 12}}, {16, {2, 4, 6, 9, 16}},
        {32, {2, 4, 6, 10, 20}}, {64, {2, 4, 7, 12, 28}}, {128, {2, 4, 8, 16, 36}},
        {256, {2, 5, 10, 20, 42}}, {1024, {2, 6, 12, 24, 48}},
        {std::numeric_limits<double>::max(), {2, 8, 16, 32, 64}}}};
    gap_params_h g;
    const u32 len_gaps = n - len_lpf_phr;
    const double rel_len_gaps = len_gaps / (double)n;
    const double avg_gap_len = len_gaps / (double)num_gaps;
    const double avg_lpf_phr_len = len_lpf_phr / (double)num_lpf;
    const u64 target = std::min<u64>(1ull << 30, std::max<u64>({1ull << 20, 0ull, (u64)((n / 3.0) * rel_len_gaps)}));
    const double guess = std::min<double>({avg_gap_len, avg_lpf_phr_len, 8.0 * std::pow(128, 1.0 - rel_len_gaps)});
    for (auto& [thr, lens] : table)
        if (guess <= thr) { g.patt_lens = lens; break; }
    u32 rt = 0;
    for (int j = 0; j < 5; j++) rt += g.patt_lens[j];
    g.roll_threshold = rt / 5;
    const int64_t rk_bytes = (int64_t)(80 + 16 * 256 * 256) * 5;  // rk_prime<107>::byte_size() * 5
    const int64_t min_index_size = std::max<u32>(1u << 20, (u32)(n * 0.1)) / sizeof(u32);
    const int64_t max_index_size = (1ll << 30) / (int64_t)sizeof(u32);
    const int64_t target_entries = std::max<int64_t>(0, (int64_t)target - rk_bytes) / (int64_t)sizeof(u32);
    const uint64_t target_size_h = std::min<int64_t>(max_index_size, std::max<int64_t>(min_index_size, target_entries));
    g.log2_size_h = (u8)std::round(std::log2(target_size_h));
    return g;
}

// phrase statistics (approximate/common.cpp:98-157, p = 1)
__global__ void k_phrase_info(const u32* __restrict__ P, u32 m, u32 n, u32* __restrict__ acc) {
    const u64 k = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= m) return;
    const u32 b = P[3 * k], e = P[3 * k + 1];
    atomicAdd(&acc[0], e - b);
    u32 gaps = 0;
    if (k == 0 ? b > 0 : b > P[3 * (k - 1) + 1]) gaps++;
    if (k == m - 1 && e < n) gaps++;
    if (gaps) atomicAdd(&acc[1], gaps);
}

struct interval { u32 a, b; };  // [a, b)

static void normalize(std::vector<interval>& v) {
    std::sort(v.begin(), v.end(), [](const interval& x, const interval& y) { return x.a < y.a || (x.a == y.a && x.b < y.b); });
    std::vector<interval> out;
    for (auto& x : v) {
        if (x.b <= x.a) continue;
        if (!out.empty() && x.a <= out.back().b) out.back().b = std::max(out.back().b, x.b);
        else out.push_back(x);
    }
    v.swap(out);
}
static void clip(std::vector<interval>& v, u32 nt) {
    for (auto& x : v) { x.a = std::min(x.a, nt); x.b = std::min(x.b, nt); }
    normalize(v);
}

u64 engine::factorize_greedy(const u8* T, u32 rk_seed, int log2_override) {
    const u32 N = (u32)n;
    const u32 m = num_phr;  // phrases; P[m] = sentinel
    u32* P = lpf.get((u64)(m + 1) * 3);
    {
        const u32 sent[3] = {N, N + 1, 0};
        LZ_HIP(hipMemcpyAsync(P + 3 * (u64)m, sent, 12, hipMemcpyHostToDevice, st));
    }
    // ---- phrase statistics -> parameters
    u32 num_lpf = m, len_lpf_phr = 0, num_gaps = 1;
    if (m > 0) {
        u32* acc = counters.get(16);
        LZ_HIP(hipMemsetAsync(acc, 0, 8, st));
        k_phrase_info<<<cdiv(m, 256), 256, 0, st>>>(P, m, N, acc);
        u32 h[2];
        LZ_HIP(hipMemcpyAsync(h, acc, 8, hipMemcpyDeviceToHost, st));
        LZ_HIP(hipStreamSynchronize(st));
        len_lpf_phr = h[0];
        num_gaps = h[1];
    }
    gap_params_h gp = choose_gap_params(N, num_lpf, len_lpf_phr, num_gaps);
    if (log2_override > 0) gp.log2_size_h = (u32)log2_override;
    // bases: rk_prime::random64(257, 2^20-1) from mt19937_64(rk_seed) (rolling_hash.hpp:127-130)
    std::array<u64, 5> bases;
    {
        std::mt19937_64 g(rk_seed);
        for (int i = 0; i < 5; i++) bases[i] = std::uniform_int_distribution<u64>(257, (1ull << 20) - 1)(g);
    }
    std::vector<u128> negpow(5 * 256);
    for (int x = 0; x < 5; x++) {
        const u128 bp = powmod107_host(bases[x], gp.patt_lens[x]);
        const u128 nb = (P107 - bp) % P107;
        negpow[x * 256] = 0;
        for (int o = 1; o < 256; o++) negpow[x * 256 + o] = mod107(negpow[x * 256 + o - 1] + nb);
    }
    u128* d_negpow = (u128*)tmp_greedy.get(5 * 256 * sizeof(u128));
    LZ_HIP(hipMemcpyAsync(d_negpow, negpow.data(), 5 * 256 * sizeof(u128), hipMemcpyHostToDevice, st));

    stats.assign(24, 0);
    stats[0] = s; stats[1] = has_runs; stats[2] = num_lpf; stats[3] = len_lpf_phr; stats[4] = num_gaps;
    for (int x = 0; x < 5; x++) stats[5 + x] = gp.patt_lens[x];
    stats[10] = gp.roll_threshold; stats[11] = gp.log2_size_h;

    gap_cfg G{};
    G.n = N;
    G.nt = N > 64 ? N - 64 : 0;
    for (int x = 0; x < 5; x++) { G.lens[x] = gp.patt_lens[x]; G.base[x] = bases[x]; }
    G.thr = gp.roll_threshold;
    G.mask = (u32)((1ull << gp.log2_size_h) - 1);
    G.negpow = d_negpow;

    // host copy of phrases (segment bookkeeping)
    std::vector<u32> hP((u64)(m + 1) * 3);
    LZ_HIP(hipMemcpyAsync(hP.data(), P, hP.size() * 4, hipMemcpyDeviceToHost, st));
    LZ_HIP(hipStreamSynchronize(st));
    auto first_phrase_after = [&](u32 i) -> u32 {  // smallest k with P[k].end > i
        u32 lo = 0, hi = m;
        while (lo < hi) {
            u32 mid = (lo + hi) >> 1;
            if (hP[3 * mid + 1] <= i) lo = mid + 1; else hi = mid;
        }
        return lo;
    };
    u32 zmask0 = 0;
    for (int x = 0; x < 5; x++) zmask0 |= (G.lens[x] >= N) ? (1u << x) : 0u;  // reinit(0) at construction

    // ---- default segments and I_0
    std::vector<u32> starts;   // segment start positions (sorted, unique)
    std::vector<interval> I;
    {
        u32 prev_end = 0;
        for (u32 k = 0; k <= m; k++) {
            const u32 b = hP[3 * k], e = hP[3 * k + 1];
            if (prev_end < b) {
                starts.push_back(prev_end);
                I.push_back({prev_end, std::min(b + 1, N)});
            }
            prev_end = std::max(prev_end, e);
        }
        if (starts.empty() || starts[0] != 0) starts.insert(starts.begin(), 0u);
    }
    clip(I, G.nt);

    dbuf<seg_in>& d_segs = seg_in_buf;
    dbuf<seg_out>& d_outs = seg_out_buf;
    std::vector<seg_in> hsegs;
    std::vector<seg_out> houts;
    u64 total_fact = 0;
    int outer = 0, rounds_total = 0;
    for (;; outer++) {
        if (outer > 64) throw error(-6, "greedy speculation did not converge");
        // ---- 2. entries of I -> sort -> occ5
        std::vector<ichunk> chunks;
        std::vector<u32> h_is, h_ie, h_ir;
        u64 nI = 0;
        for (auto& iv : I) {
            h_is.push_back(iv.a); h_ie.push_back(iv.b); h_ir.push_back((u32)nI);
            for (u32 q = iv.a; q < iv.b; q += 1024) {
                const u32 q1 = std::min<u32>(iv.b, q + 1024);
                chunks.push_back({q, q1, (u32)(nI + (q - iv.a))});
            }
            nI += iv.b - iv.a;
        }
        if (5 * nI >= (1ull << 32)) throw error(-1, "gap region too large for 32-bit entry ids");
        const u64 ne = 5 * nI;
        u32* d_is = ist.get(h_is.size() + 1);
        u32* d_ie = iend.get(h_ie.size() + 1);
        u32* d_ir = irank.get(h_ir.size() + 1);
        if (!h_is.empty()) {
            LZ_HIP(hipMemcpyAsync(d_is, h_is.data(), h_is.size() * 4, hipMemcpyHostToDevice, st));
            LZ_HIP(hipMemcpyAsync(d_ie, h_ie.data(), h_ie.size() * 4, hipMemcpyHostToDevice, st));
            LZ_HIP(hipMemcpyAsync(d_ir, h_ir.data(), h_ir.size() * 4, hipMemcpyHostToDevice, st));
        }
        ichunk* d_ch = (ichunk*)chunk_buf.get(std::max<size_t>(1, chunks.size()) * sizeof(ichunk));
        if (!chunks.empty())
            LZ_HIP(hipMemcpyAsync(d_ch, chunks.data(), chunks.size() * sizeof(ichunk), hipMemcpyHostToDevice, st));
        u32* keys = ekeys.get(ne + 1), *vals = evals.get(ne + 1);
        u32* skeys = ekeys2.get(ne + 1), *svals = evals2.get(ne + 1);
        u32* ipos = ipos_buf.get(nI + 1);
        u32* occ5 = occ_buf.get(ne + 1);
        if (!chunks.empty()) {
            k_slots<<<cdiv(chunks.size(), 64), 64, 0, st>>>(T, G, d_ch, (u32)chunks.size(), keys, vals, ipos);
            size_t tb = 0;
            LZ_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, keys, skeys, vals, svals, (int)ne, 0,
                                                      (int)gp.log2_size_h, st));
            u8* t = scan_tmp.get(tb);
            LZ_HIP(hipcub::DeviceRadixSort::SortPairs(t, tb, keys, skeys, vals, svals, (int)ne, 0,
                                                      (int)gp.log2_size_h, st));
            k_occ<<<cdiv(ne, 256), 256, 0, st>>>(skeys, svals, ipos, ne, occ5);
        }
        walk_ctx W{};
        W.T = T;
        W.G = G;
        W.P = P;
        W.occ5 = occ5;
        W.istart = d_is;
        W.iend = d_ie;
        W.irank = d_ir;
        W.nint = (u32)h_is.size();
        W.L = view(T);
        W.skeys = skeys;
        W.svals = svals;
        W.ipos = ipos;
        W.nentries = ne;

        // ---- 3./4. walk all known segments, link the chain, add missing starts
        std::unordered_map<u32, u32> id_of;
        hsegs.clear();
        for (u32 a : starts) {
            id_of[a] = (u32)hsegs.size();
            hsegs.push_back({a, first_phrase_after(a), a, zmask0});
        }
        houts.assign(hsegs.size(), seg_out{});
        std::vector<u32> todo(hsegs.size());
        for (u32 g = 0; g < todo.size(); g++) todo[g] = g;
        std::vector<u32> chain;
        bool tail_reached = false;
        for (int round = 0;; round++) {
            rounds_total++;
            if (round > 256) throw error(-6, "greedy segment linking did not converge");
            // walk the todo segments (compact arrays: dbuf growth does not preserve contents)
            if (!todo.empty()) {
                std::vector<seg_in> tin(todo.size());
                for (size_t t = 0; t < todo.size(); t++) tin[t] = hsegs[todo[t]];
                seg_in* ds = d_segs.get(todo.size());
                seg_out* dout = d_outs.get(todo.size());
                LZ_HIP(hipMemcpyAsync(ds, tin.data(), tin.size() * sizeof(seg_in), hipMemcpyHostToDevice, st));
                k_walk<false><<<cdiv(todo.size(), 64), 64, 0, st>>>(W, ds, nullptr, (u32)todo.size(), dout, nullptr, nullptr);
                LZ_HIP(hipGetLastError());
                std::vector<seg_out> tout(todo.size());
                LZ_HIP(hipMemcpyAsync(tout.data(), dout, tout.size() * sizeof(seg_out), hipMemcpyDeviceToHost, st));
                LZ_HIP(hipStreamSynchronize(st));
                for (size_t t = 0; t < todo.size(); t++) houts[todo[t]] = tout[t];
            }
            // link from position 0
            chain.clear();
            tail_reached = false;
            std::vector<u32> missing;
            u32 g = id_of.at(0);
            u32 idxp = 0, zm = zmask0;
            bool complete = true;
            for (;;) {
                if (chain.size() > hsegs.size()) throw error(-6, "greedy: segment chain has a cycle");
                chain.push_back(g);
                hsegs[g].idxpos = idxp;  // exact inputs of chain segments (used by the tail walk)
                hsegs[g].zmask = zm;
                const seg_out& o = houts[g];
                if (o.flags & 2) throw error(-6, "greedy: too many LPF-start queries in one segment");
                if (o.flags & 4) throw error(-6, "greedy: walk guard tripped (internal error)");
                if (o.flags & 1) { tail_reached = true; break; }
                if (o.next >= N) break;
                idxp = o.idxpos;
                zm = o.zmask;
                auto it = id_of.find(o.next);
                if (it == id_of.end()) { complete = false; break; }
                g = it->second;
            }
            if (debug_enabled())
                std::fprintf(stderr, "[lz77sss-debug] greedy outer=%d round=%d segs=%zu chain=%zu complete=%d tail=%d\n",
                             outer, round, hsegs.size(), chain.size(), (int)complete, (int)tail_reached);
            if (complete) break;
            // speculatively add every unknown next state
            todo.clear();
            for (u32 h = 0; h < houts.size(); h++) {
                const seg_out& o = houts[h];
                if ((o.flags & 1) || o.next >= N) continue;
                if (id_of.count(o.next)) continue;
                const u32 a = o.next;
                id_of[a] = (u32)hsegs.size();
                todo.push_back((u32)hsegs.size());
                hsegs.push_back({a, first_phrase_after(a), a, zmask0});
                houts.push_back(seg_out{});
                missing.push_back(a);
            }
            if (missing.empty()) throw error(-6, "greedy: chain broken without new states");
        }
        // ---- tail: exact single-thread walk from the first chain segment in the tail region
        u64 tail_count = 0;
        std::vector<interval> tail_ins;
        u64 chain_fact = 0;
        size_t nchain = chain.size() - (tail_reached ? 1 : 0);
        for (size_t c = 0; c < nchain; c++) chain_fact += houts[chain[c]].nfact;
        u64* d_cnt = (u64*)counters64.get(4);
        u32* d_tins = tail_ins_buf.get(16);
        const u64 tail_bound = tail_reached ? (u64)N - hsegs[chain.back()].start + 1 : 0;
        u32* fo = fact.get(2 * (chain_fact + tail_bound) + 2);
        if (tail_reached) {
            const seg_in tin = hsegs[chain.back()];
            k_tail<<<1, 64, 0, st>>>(W, tin, fo, chain_fact, d_cnt, d_tins);
            LZ_HIP(hipGetLastError());
            u64 hc[3];
            u32 hti[16];
            LZ_HIP(hipMemcpyAsync(hc, d_cnt, 24, hipMemcpyDeviceToHost, st));
            LZ_HIP(hipMemcpyAsync(hti, d_tins, 64, hipMemcpyDeviceToHost, st));
            LZ_HIP(hipStreamSynchronize(st));
            if (hc[2]) throw error(-6, "greedy tail: insert overflow or guard tripped");
            tail_count = hc[0];
            for (u64 k = 0; k < hc[1]; k++) tail_ins.push_back({hti[2 * k], hti[2 * k + 1]});
        }
        // ---- 5. actual insert set along the chain
        std::vector<interval> I2 = tail_ins;
        for (size_t c = 0; c < nchain; c++) {
            const seg_in& si = hsegs[chain[c]];
            const seg_out& o = houts[chain[c]];
            I2.push_back({si.start, o.e});
            for (u32 k = 0; k < o.nsingle && k < 4; k++) I2.push_back({o.single[k], o.single[k] + 1});
        }
        clip(I2, G.nt);
        bool same = I2.size() == I.size();
        for (size_t k = 0; same && k < I.size(); k++) same = I2[k].a == I[k].a && I2[k].b == I[k].b;
        if (!same) {
            I.swap(I2);
            starts.clear();
            for (auto& sg : hsegs) starts.push_back(sg.start);
            std::sort(starts.begin(), starts.end());
            starts.erase(std::unique(starts.begin(), starts.end()), starts.end());
            continue;
        }
        // ---- write pass for the chain segments (before the tail segment)
        if (nchain) {
            std::vector<u64> offs(nchain);
            std::vector<u32> ids(nchain);
            u64 o = 0;
            for (size_t c = 0; c < nchain; c++) { offs[c] = o; o += houts[chain[c]].nfact; ids[c] = chain[c]; }
            u64* doffs = seg_offs.get(nchain);
            std::vector<seg_in> cin(nchain);
            for (size_t c = 0; c < nchain; c++) cin[c] = hsegs[chain[c]];
            seg_in* ds = d_segs.get(nchain);
            LZ_HIP(hipMemcpyAsync(ds, cin.data(), nchain * sizeof(seg_in), hipMemcpyHostToDevice, st));
            LZ_HIP(hipMemcpyAsync(doffs, offs.data(), nchain * 8, hipMemcpyHostToDevice, st));
            k_walk<true><<<cdiv(nchain, 64), 64, 0, st>>>(W, ds, nullptr, (u32)nchain, nullptr, doffs, fo);
            LZ_HIP(hipGetLastError());
        }
        total_fact = chain_fact + tail_count;
        break;
    }
    stats[12] = outer + 1;
    stats[13] = rounds_total;
    stats[14] = stats_fallback_lanes;
    return total_fact;
}

}  // namespace lz
