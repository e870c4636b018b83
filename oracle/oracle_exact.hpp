// ============================================================================
//  oracle/oracle_exact.hpp -- CPU restatement of the reference's exact transform:
//  factorize_exact<greedy, lpf_opt, with_samples | without_samples,
//  decomposed_static_weighted_square_grid> (lz77_sss.hpp:318-341, 600-666).
//
//  TEST INFRASTRUCTURE ONLY (like oracle.hpp): tests/, smoke() and the cpu_baseline leg of
//  bench.py --mode exact use it as the checker / the timed CPU path; the product never does.
//
//  What is restated, with the reference lines each part follows:
//   * the sample set C from the approximate factors, literally (common.cpp:34-88: C[0] = 0, then
//     for every approximate phrase but the first the phrase ends accumulated from 0 -- the first
//     phrase's length is not added, so a sample lies on the last character of each phrase --
//     with a sample every delta positions inside), delta = min(n / z_aprx, 256)
//     (lz77_sss.hpp:326), and the parallel sections (common.cpp:48-75, 16 per thread);
//   * PA_C / SA_C: the sample ids sorted by cmp_sample_lex<LEFT / RIGHT>
//     (sample_index.hpp:261-286, 316-344), the left contexts compared over lce_l_64 capped at
//     delta plus the next character, the right ones by the exact LCE; ips4o -> std::stable_sort
//     (the shim that makes the tie order deterministic);
//   * the sampled pattern lengths of both directions (construction.cpp build_samples:
//     LCX arrays, the rank-interpolated lengths, the short lengths added while cheap), and the
//     interval samples per sampled length keyed by a Rabin-Karp fingerprint of the pattern
//     (construction.cpp, queries.cpp sxa_interval; a 61-bit Mersenne hash here, every lookup
//     verified by an LCE so a collision falls back to a search -- the intervals are exact
//     either way, as the reference's LCE-checked equality makes them);
//   * extend_left / extend_right / interpolate (queries.cpp): exact XA intervals of a pattern,
//     found here by binary search inside the sampled interval of the longest sampled length
//     below the pattern's (the reference's narrowing; only speed depends on how);
//   * P, Pi, Psi (common.cpp:114-182) and the decomposed static weighted square grid
//     (decomposed_range.hpp, static_weighted_square_grid.hpp: per first character, windows of
//     16 384 ranks, points sorted by (window, weight), lighter_point_in_range's visit order:
//     contained windows row by row by their lightest point, then the border windows' points in
//     weight order);
//   * intersect (common.cpp:258-358: the Pi / Psi scan below 4 096 ranks, else the grid; the
//     source is the found point's sample minus lce_l - 1, kept only when strictly longer);
//   * transform_to_exact_with_samples / extend_right_with_samples (with_samples.cpp:31-240)
//     and transform_to_exact_without_samples (without_samples.cpp:31-152), with the
//     reference's exponential / binary search helpers (utils.hpp:326-471): the probe order
//     decides which point supplies a source, so it is followed call by call.
//  The approximate factors and the LCE are the oracle's own (oracle.hpp).  At p = 1 the output
//  is the reference's stream under the pinned choices above (the reference itself cannot be
//  built here: parity unpinned); at p > 1 the sections restart the greedy parse
//  (timing only).
// ============================================================================
#pragma once
#include "oracle.hpp"


namespace lzo {

// ---------------------------------------------------------------------------
// the reference's search helpers (utils.hpp:326-471), restated
template <class V, class I, class F>
static inline I xs_min_geq(V v, I l, I r, F at) {
    while (l != r) {
        const I m = l + (r - l) / 2;
        if (v <= at(m)) r = m;
        else l = m + 1;
    }
    return l;
}
template <class V, class I, class F>
static inline I xs_max_lt(V v, I l, I r, F at) {
    while (l != r) {
        const I m = l + (r - l) / 2 + 1;
        if (at(m) < v) l = m;
        else r = m - 1;
    }
    return l;
}
template <class V, class I, class F>
static inline I xs_max_geq(V v, I l, I r, F at) {
    while (l != r) {
        const I m = l + (r - l) / 2 + 1;
        if (at(m) >= v) l = m;
        else r = m - 1;
    }
    return l;
}
template <class V, class I, class F>
static inline I xs_max_leq(V v, I l, I r, F at) {
    while (l != r) {
        const I m = l + (r - l) / 2 + 1;
        if (at(m) <= v) l = m;
        else r = m - 1;
    }
    return l;
}
// exp_search_max_geq<val, pos, RIGHT>: probes left + 1, left + 3, left + 7, ... while they hold,
// then a binary search over the last step
template <class V, class I, class F>
static inline I xs_exp_max_geq_right(V v, I l, I r, F at) {
    if (r == l) return l;
    I step = 1;
    l += step;
    while (at(l) >= v) {
        step *= 2;
        if (r < step || r - step < l) {
            step = r - l + 1;
            l = r + 1;
            break;
        }
        l += step;
    }
    return xs_max_geq<V, I>(v, (I)(l - step), (I)(l - 1), at);
}

// ---------------------------------------------------------------------------
// Rabin-Karp substring fingerprints (role of rabin_karp_substring<31>: a prefix fingerprint every
// 16 characters, the rest rolled on demand), here mod 2^61 - 1 with a fixed base
struct rk61 {
    static constexpr u64 M = (1ull << 61) - 1;
    static constexpr u64 B = 0x1F3D5B79ull;
    static constexpr u32 RATE = 16;
    const u8* T = nullptr;
    u64 n = 0;
    std::vector<u64> pre;   // H(T[0 .. 16k))
    std::vector<u64> pw;    // B^k, k < PW_N
    static constexpr u64 PW_N = 1u << 20;
    static u64 mul(u64 a, u64 b) {
        const u128 x = (u128)a * b;
        u64 r = (u64)(x & M) + (u64)(x >> 61);
        return r >= M ? r - M : r;
    }
    static u64 add(u64 a, u64 b) { u64 r = a + b; return r >= M ? r - M : r; }
    u64 bpow(u64 e) const {
        if (e < PW_N) return pw[e];
        u64 r = 1, b = B;
        while (e) { if (e & 1) r = mul(r, b); b = mul(b, b); e >>= 1; }
        return r;
    }
    void build(const u8* T_, u64 n_, int p) {
        T = T_;
        n = n_;
        pw.resize(PW_N);
        pw[0] = 1;
        for (u64 k = 1; k < PW_N; k++) pw[k] = mul(pw[k - 1], B);
        const u64 nb = n / RATE + 1;
        pre.assign(nb + 1, 0);
        // per block hash of 16 characters, then a sequential prefix combination
        std::vector<u64> blk(nb, 0);
#pragma omp parallel for num_threads(p) schedule(static)
        for (u64 b = 0; b < nb; b++) {
            u64 h = 0;
            const u64 e = std::min<u64>(n, (b + 1) * RATE);
            for (u64 i = b * RATE; i < e; i++) h = add(mul(h, B), (u64)T[i] + 1);
            blk[b] = h;
        }
        const u64 b16 = pw[RATE];
        for (u64 b = 0; b < nb; b++) pre[b + 1] = add(mul(pre[b], b16), blk[b]);
    }
    u64 prefix(u64 x) const {  // H(T[0 .. x))
        const u64 b = x / RATE;
        u64 h = pre[b];
        for (u64 i = b * RATE; i < x; i++) h = add(mul(h, B), (u64)T[i] + 1);
        return h;
    }
    u64 sub(u64 a, u64 len) const {  // H(T[a .. a + len))
        const u64 hb = prefix(a + len), ha = mul(prefix(a), bpow(len));
        return hb >= ha ? hb - ha : hb + M - ha;
    }
};

// open-addressing map fingerprint -> packed interval (role of tsl::sparse_set in the reference's
// interval samples; 16 B per slot, load <= 1/2).  A key collision of two patterns keeps the first
// pattern's interval: every lookup is verified against the text, so the second one falls back to
// a search
struct fp_map {
    std::vector<u64> key, val;
    u64 mask = 0;
    static constexpr u64 EMPTY = ~0ull;
    void init(u64 n) {
        u64 cap = 16;
        while (cap < 2 * n + 2) cap <<= 1;
        key.assign(cap, EMPTY);
        val.assign(cap, 0);
        mask = cap - 1;
    }
    static u64 mix(u64 k) { k ^= k >> 31; k *= 0x9E3779B97F4A7C15ull; return k ^ (k >> 29); }
    void put(u64 k, u64 v) {
        if (k == EMPTY) k = 0;
        for (u64 h = mix(k) & mask;; h = (h + 1) & mask) {
            if (key[h] == EMPTY) { key[h] = k; val[h] = v; return; }
            if (key[h] == k) return;
        }
    }
    bool get(u64 k, u64& v) const {
        if (key.empty()) return false;
        if (k == EMPTY) k = 0;
        for (u64 h = mix(k) & mask;; h = (h + 1) & mask) {
            if (key[h] == EMPTY) return false;
            if (key[h] == k) { v = val[h]; return true; }
        }
    }
};

// ---------------------------------------------------------------------------
enum exact_transf { ex_naive = 0, ex_with_samples = 1, ex_without_samples = 2 };

struct exact_smpl {
    static constexpr u32 MAX_DELTA = 256;            // lz77_sss.hpp:83
    static constexpr u32 RANGE_SCAN = 4096;          // lz77_sss.hpp:85 range_scan_threshold
    static constexpr u32 SECT_PER_THR = 16;          // lz77_sss.hpp:94
    static constexpr u32 WIN = 16384;                // static_weighted_square_grid.hpp default
    static constexpr u32 NO = 0xFFFFFFFFu;
    enum { LEFT = 0, RIGHT = 1 };

    const u8* T = nullptr;
    u32 n = 0;
    const lce_structure<u32>* L = nullptr;
    int p = 1;
    u32 delta = 0, za = 0;
    std::vector<factor> Fa;   // the approximate factors
    std::vector<u32> C;        // samples
    u32 c = 0;
    struct sect_t { u32 beg, phr; };
    std::vector<sect_t> sect;
    std::vector<u32> XA[2];   // PA_C, SA_C: sample ids in order
    std::vector<u32> RK[2];   // rank of each sample in them
    std::vector<u32> Pi, Psi;
    std::vector<u32> lens[2];  // sampled pattern lengths
    rk61 rk;
    std::vector<fp_map> ivs[2];  // per sampled length index: fp -> b << 32 | e
    // the decomposed grid
    std::array<u32, 257> CS{};
    struct point { u32 x, y, w; };
    struct grid_t {
        u32 width = 0;
        std::vector<point> pts;
        std::vector<u32> beg;  // width^2 + 1 window starts in pts
    };
    std::vector<grid_t> grid;  // per first character

    u32 rlce(u32 i, u32 j) const { return (u32)L->lce(i, j); }
    // cmp_lex<dir> (sample_index.hpp:261-274)
    template <int dir>
    bool cmp_lex(u32 i, u32 j, u32 l) const {
        if (i == j) return false;
        if constexpr (dir == LEFT) {
            if (l > std::min(i, j)) return i < j;
            return T[i - l] < T[j - l];
        } else {
            if ((u64)std::max(i, j) + l == n) return i > j;
            return T[i + l] < T[j + l];
        }
    }
    // lce<dir> of two text positions, the left one capped (lce_l_64 semantics)
    template <int dir>
    u32 lce(u32 i, u32 j, u32 cap) const {
        if constexpr (dir == LEFT) return lce_left<u32>(T, i, j, cap);
        else return rlce(i, j);
    }

    // ---- C and the sections (common.cpp:34-88)
    void build_c() {
        C.clear();
        C.reserve(za + n / std::max<u32>(delta, 1) + 2);
        C.push_back(0);
        // (the reference's split needs z_aprx >= the section count; short inputs use one section)
        const u32 nsect = (p == 1 || za < 4u * (u32)p * SECT_PER_THR) ? 1u : (u32)p * SECT_PER_THR;
        sect.assign(nsect + 1, sect_t{0, 0});
        sect[nsect] = {n, za};
        u32 phr_nxt = za / nsect, s = 1;
        u32 end_cur = 0, end_lst = 0;
        for (u32 phr = 1; phr < za; phr++) {
            const u32 smpl_lst0 = end_cur;
            u32 smpl_lst = smpl_lst0;
            end_cur += std::max<u32>(1, Fa[phr].len);
            while (end_cur - smpl_lst > delta) {
                smpl_lst += delta;
                C.push_back(smpl_lst);
            }
            C.push_back(end_cur);
            if (phr == phr_nxt) {
                sect[s++] = {end_lst + 1, phr};
                phr_nxt = s == nsect ? za : (s * (za / nsect));
            }
            end_lst = end_cur;
        }
        c = (u32)C.size();
    }

    // ---- PA_C / SA_C (sample_index.hpp:316-344) and the sampled lengths (construction.cpp)
    template <int dir>
    void sort_xa() {
        std::vector<u32>& X = XA[dir];
        X.resize(c);
        for (u32 i = 0; i < c; i++) X[i] = i;
        auto cmp = [&](u32 a, u32 b) {
            if (a == b) return false;
            return cmp_lex<dir>(C[a], C[b], lce<dir>(C[a], C[b], delta));
        };
#ifdef _OPENMP
        if (p > 1) __gnu_parallel::stable_sort(X.begin(), X.end(), cmp);
        else std::stable_sort(X.begin(), X.end(), cmp);
#else
        std::stable_sort(X.begin(), X.end(), cmp);
#endif
        RK[dir].resize(c);
        for (u32 i = 0; i < c; i++) RK[dir][X[i]] = i;
    }
    template <bool IsLeft>
    bool pos_in_T(u32 q, u32 offs) const { return IsLeft ? q >= offs : (u64)q + offs < n; }

    template <int dir>
    void build_samples(u32 max_smpl_len) {
        const std::vector<u32>& X = XA[dir];
        std::vector<u32> LCX(c + 1, 0);
#pragma omp parallel for num_threads(p) schedule(static)
        for (u64 i = 1; i < c; i++) LCX[i] = lce<dir>(C[X[i - 1]], C[X[i]], delta);
        std::vector<u32> srt(LCX.begin(), LCX.begin() + c);
        std::sort(srt.begin(), srt.end());
        auto at = [&](u32 i) { return srt[i]; };
        max_smpl_len = std::min<u32>(srt[c - 1], max_smpl_len);
        const u32 rng_min = xs_min_geq<u32, u32>(3u, 0u, c - 1, at);
        const u32 rng_max = xs_min_geq<u32, u32>(max_smpl_len, 0u, c - 1, at);
        const double max_num_samples = 2.0 * c;
        const double rng = (double)rng_max - (double)rng_min;
        std::vector<u32>& pl = lens[dir];
        pl = {1, 2};
        ivs[dir].assign(2, {});
        if (rng_min >= rng_max) return;
        u64 num = std::min<u64>((u64)max_smpl_len - 2,
                                2 + (u64)std::floor((2.0 * max_num_samples) / (double)(rng_min + rng_max)));
        std::vector<u32> ranks(std::max<u64>(num, 3), 0);
        for (u64 i = 2; i < num; i++) {
            const double rel = (double)(i - 1) / (double)(num - 2);
            const u32 rnk = (u32)std::floor((double)rng_min + rel * rng);
            const u32 len = std::max(srt[rnk], pl.back() + 1);
            if (len > max_smpl_len) break;
            pl.push_back(len);
            ranks[i] = xs_min_geq<u32, u32>(len, 0u, c - 1, at);
        }
        const u32 max_add = (u32)(max_num_samples * 0.2);
        if (ranks[2] < max_add) {
            u32 added = 0;
            for (u32 len = 3; true; len++) {
                if (std::find(pl.begin(), pl.end(), len) != pl.end()) continue;
                const u32 rnk = xs_min_geq<u32, u32>(len, 0u, c - 1, at);
                if (len > max_smpl_len || added + rnk > max_add) break;
                added += rnk;
                pl.insert(pl.begin() + (len - 1), len);
            }
        }
        // interval samples: per sampled length >= 3 (index >= 2) the XA interval of every pattern
        // of that length that begins a sample's context, keyed by the pattern's fingerprint
        const u32 npl = (u32)pl.size();
        ivs[dir].assign(npl, {});
        LCX[c] = 0;
        // one table per length, filled in parallel (each from its own boundaries)
#pragma omp parallel for num_threads(p) schedule(dynamic, 1)
        for (u32 j = 2; j < npl; j++) {
            const u32 len = pl[j];
            u64 cnt = 0;
            for (u32 i = 1; i <= c; i++) cnt += LCX[i] < len;
            ivs[dir][j].init(cnt);
            u32 b = 0;
            for (u32 i = 1; i <= c; i++) {
                if (LCX[i] >= len) continue;
                const u32 q = C[X[i - 1]];
                if (pos_in_T<dir == LEFT>(q, len - 1)) ivs[dir][j].put(fp<dir>(q, len), (u64)b << 32 | (i - 1));
                b = i;
            }
        }
    }
    // fingerprint of the pattern of length len at q (LEFT: ending at q; RIGHT: starting at q)
    template <int dir>
    u64 fp(u32 q, u32 len) const { return dir == LEFT ? rk.sub((u64)q + 1 - len, len) : rk.sub(q, len); }

    // ---- exact XA intervals
    // leftward LCE with lce_l_64's semantics (min(cap, min(i, j) + 1, equal characters going
    // left)), eight characters per step
    static u32 lce_left_w(const u8* T_, u32 i, u32 j, u32 cap) {
        const u32 cp = std::min<u32>(cap, std::min(i, j) + 1);
        if (i == j) return cp;
        u32 k = 0;
        while (k + 8 <= cp) {
            u64 x, y;
            std::memcpy(&x, T_ + (i - k - 7), 8);
            std::memcpy(&y, T_ + (j - k - 7), 8);
            if (x != y) return k + (u32)(std::countl_zero(x ^ y) >> 3);
            k += 8;
        }
        while (k < cp && T_[i - k] == T_[j - k]) k++;
        return k;
    }
    // LCE of the pattern at q with the context of sample position s, at least `skip` known equal,
    // at most len
    template <int dir>
    u32 pat_lce(u32 q, u32 s, u32 skip, u32 len) const {
        if (skip >= len) return len;
        if constexpr (dir == LEFT) {
            return skip + lce_left_w(T, q - skip, s - skip, len - skip);
        } else {
            // (the reference compares up to 3 tau characters directly; the same value, found here
            // through the LCE structure once the first 64 characters agree)
            const u32 rest = len - skip, head = std::min<u32>(rest, 64);
            const u32 k = (u32)naive_lce(T, n, (u64)q + skip, (u64)s + skip, head);
            if (k < head || rest == head) return skip + k;
            return std::min<u32>(rlce(q, s), len);
        }
    }
    // [b, e] of the ranks in [lo, hi] whose contexts begin with the pattern (empty: b > e), when
    // the answer holds [in_b, in_e] (a longer pattern's interval; in_b > in_e: none): the
    // reference's binary searches with the common prefix of both search bounds skipped
    template <int dir>
    std::pair<u32, u32> search_iv(u32 q, u32 len, u32 lo, u32 hi, u32 in_b = 1, u32 in_e = 0) const {
        const std::vector<u32>& X = XA[dir];
        auto side = [&](u32 m, u32 skip, u32& l) -> int {  // 0: match, -1: context smaller, +1: larger
            const u32 sp = C[X[m]];
            l = pat_lce<dir>(q, sp, skip, len);
            if (l >= len) return 0;
            return cmp_lex<dir>(sp, q, l) ? -1 : 1;
        };
        const bool inner = in_b <= in_e;
        // first rank in [lo, hi + 1) that is not smaller (inside [lo, in_b] when inner)
        u32 l = lo, r = inner ? in_b : hi + 1, ll = 0, lr = inner ? len : 0;
        while (l < r) {
            const u32 m = l + (r - l) / 2;
            u32 lm;
            if (side(m, std::min(ll, lr), lm) < 0) { l = m + 1; ll = lm; }
            else { r = m; lr = lm; }
        }
        const u32 b = l;
        // (rank b matches iff a probe set r to it with a full match; inner: in_b matches)
        if (!inner && (b > hi || lr < len)) return {1, 0};
        // first rank that is larger, after the matching rank b (or the inner interval)
        l = inner ? in_e + 1 : b + 1;
        r = hi + 1;
        ll = len;
        lr = 0;
        while (l < r) {
            const u32 m = l + (r - l) / 2;
            u32 lm;
            if (side(m, std::min(ll, lr), lm) <= 0) { l = m + 1; ll = lm; }
            else { r = m; lr = lm; }
        }
        if (b >= l) return {1, 0};
        return {b, l - 1};
    }
    // the interval of the pattern of length len at q inside [lo, hi] (a shorter pattern's interval,
    // or everything) holding [in_b, in_e]: the sampled interval of the longest sampled length <= len
    // (queries.cpp extend: its interval samples; the interval itself when len is sampled), narrowed
    // by binary search
    template <int dir>
    std::pair<u32, u32> interval(u32 q, u32 len, u32 lo = 0, u32 hi = NO, u32 in_b = 1, u32 in_e = 0) const {
        if (hi == NO) hi = c - 1;
        if (len == 0) return {lo, hi};
        if constexpr (dir == LEFT) {
            if ((u64)q + 1 < len) return {1, 0};
        } else {
            if ((u64)q + len > n) return {1, 0};
        }
        const std::vector<u32>& pl = lens[dir];
        const u32 x = xs_max_leq<u32, u32>(len, 0u, (u32)pl.size() - 1, [&](u32 k) { return pl[k]; });
        if (x >= 2 && pl[x] <= len) {
            u64 v;
            if (!ivs[dir][x].get(fp<dir>(q, pl[x]), v)) return {1, 0};  // (the shorter pattern begins no context)
            const u32 b = (u32)(v >> 32), e = (u32)v;
            u32 l0;
            if (pat_lce<dir>(q, C[XA[dir][b]], 0, pl[x]) >= pl[x]) {
                (void)l0;
                if (pl[x] == len) return {b, e};
                lo = std::max(lo, b);
                hi = std::min(hi, e);
            }  // (else a fingerprint collision: searched in the given range)
        }
        if (lo > hi) return {1, 0};
        return search_iv<dir>(q, len, lo, hi, in_b, in_e);
    }

    // ---- P, Pi, Psi and the decomposed square grid (common.cpp:114-182, decomposed_range.hpp,
    // static_weighted_square_grid.hpp)
    void build_points() {
        Pi.resize(c);
        Psi.resize(c);
        for (u32 x = 0; x < c; x++) Pi[x] = RK[RIGHT][XA[LEFT][x]];
        for (u32 y = 0; y < c; y++) Psi[y] = RK[LEFT][XA[RIGHT][y]];
        CS.fill(0);
        for (u32 i = 0; i < c; i++) CS[T[C[i]] + 1]++;
        for (int ch = 1; ch <= 256; ch++) CS[ch] += CS[ch - 1];
        grid.assign(256, grid_t{});
        std::array<std::vector<point>, 256> pc;
        for (u32 i = 0; i < c; i++) {
            const u8 ch = T[C[i]];
            pc[ch].push_back(point{RK[LEFT][i] - CS[ch], RK[RIGHT][i] - CS[ch], i});
        }
        for (int ch = 0; ch < 256; ch++) {
            const u32 frq = CS[ch + 1] - CS[ch];
            if (!frq) continue;
            grid_t& G = grid[ch];
            G.width = (frq + WIN - 1) / WIN;
            const u64 nw = (u64)G.width * G.width;
            auto widx = [&](const point& pt) -> u64 { return (u64)G.width * (pt.y / WIN) + pt.x / WIN; };
            std::vector<point>& P = pc[ch];
            std::sort(P.begin(), P.end(), [&](const point& a, const point& b) {
                const u64 wa = widx(a), wb = widx(b);
                return wa == wb ? a.w < b.w : wa < wb;
            });
            G.beg.assign(nw + 1, 0);
            for (const point& pt : P) G.beg[widx(pt) + 1]++;
            for (u64 k = 0; k < nw; k++) G.beg[k + 1] += G.beg[k];
            G.pts = std::move(P);
        }
    }
    // lighter_point_in_range (static_weighted_square_grid.hpp): the visit order decides the point
    bool grid_query(u8 ch, u32 weight, u32 x1, u32 x2, u32 y1, u32 y2, point& out) const {
        const grid_t& G = grid[ch];
        x1 -= CS[ch]; x2 -= CS[ch]; y1 -= CS[ch]; y2 -= CS[ch];
        const u32 xw1 = x1 / WIN, xw2 = x2 / WIN, yw1 = y1 / WIN, yw2 = y2 / WIN;
        const u32 xi1 = xw1 + (x1 % WIN != 0), yi1 = yw1 + (y1 % WIN != 0);
        const u32 xi2 = xw2 + (x2 % WIN == WIN - 1), yi2 = yw2 + (y2 % WIN == WIN - 1);
        const bool contained = xi1 < xi2 && yi1 < yi2;
        auto wid = [&](u32 xw, u32 yw) -> u64 { return (u64)G.width * yw + xw; };
        if (contained) {
            for (u32 yw = yi1; yw < yi2; yw++)
                for (u32 xw = xi1; xw < xi2; xw++) {
                    const u64 k = wid(xw, yw);
                    if (G.beg[k + 1] > G.beg[k]) {
                        const point& pt = G.pts[G.beg[k]];
                        if (pt.w < weight) { out = pt; return true; }
                    }
                }
        }
        for (u32 yw = yw1; yw <= yw2; yw++) {
            const bool yc = contained && yi1 <= yw && yw < yi2;
            for (u32 xw = xw1; xw <= xw2;) {
                if (yc && xw == xi1) { xw = xi2; continue; }
                const u64 k = wid(xw, yw);
                for (u32 t = G.beg[k]; t < G.beg[k + 1]; t++) {
                    const point& pt = G.pts[t];
                    if (pt.w >= weight) break;
                    if (x1 <= pt.x && pt.x <= x2 && y1 <= pt.y && pt.y <= y2) { out = pt; return true; }
                }
                xw++;
            }
        }
        return false;
    }

    // ---- intersect (common.cpp:258-358)
    static void adjust_xc(const std::vector<u32>& C_, u32 c_, u32& xc, u32 pos) {
        while (xc < c_ && C_[xc] < pos) xc++;
        while (xc > 0 && C_[xc - 1] >= pos) xc--;
    }
    bool intersect(u32 pb, u32 pe, u32 sb, u32 se, u32 i, u32 j, u32 lce_l, u32 lce_r, u32& xc, factor& f,
                   bool naive) const {
        (void)i;
        bool res = false;
        u32 py = 0;
        const u32 pa_rng = pe - pb + 1, sa_rng = se - sb + 1;
        adjust_xc(C, c, xc, j);
        if (!naive && std::min(pa_rng, sa_rng) <= RANGE_SCAN) {
            if (pa_rng <= sa_rng) {
                for (u32 x = pb; x <= pe; x++)
                    if (XA[LEFT][x] < xc && sb <= Pi[x] && Pi[x] <= se) { py = Pi[x]; res = true; break; }
            } else {
                for (u32 y = sb; y <= se; y++)
                    if (XA[RIGHT][y] < xc && pb <= Psi[y] && Psi[y] <= pe) { py = y; res = true; break; }
            }
        } else {
            point pt;
            res = grid_query(T[j], xc, pb, pe, sb, se, pt);
            if (res) py = pt.y + CS[T[j]];
        }
        if (res) {
            const u32 l = lce_l + lce_r - 1;
            if (l > f.len) {
                f.len = l;
                f.src = C[XA[RIGHT][py]] - lce_l + 1;
            }
        }
        return res;
    }

    // ---- extend_right_with_samples (with_samples.cpp:34-122).  The interval's lce values of the
    // reference only steer which of two exact procedures computes an interval, so only the
    // intervals are kept
    void extend_right_with_samples(u32 pb, u32 pe, u32 i, u32 j, u32 e, u32& xc, factor& f) const {
        const std::vector<u32>& sl = lens[RIGHT];
        const int nsl = (int)sl.size();
        const u32 lce_r_min = f.len < j - i ? 0 : (i + f.len - j);
        const u32 lce_l = (j - i) + 1;
        const int16_t x_min = xs_max_leq<u32, int16_t>(lce_r_min, (int16_t)0, (int16_t)(nsl - 1),
                                                        [&](int16_t x) { return sl[x]; });
        const int16_t x_max = xs_max_leq<u32, int16_t>(e - j, x_min, (int16_t)(nsl - 1), [&](int16_t x) { return sl[x]; });
        std::pair<u32, u32> sa_iv{1, 0}, sa_nxt{1, 0};
        u32 lce_r = 0, lce_r_nxt = 0;
        const int16_t x_res = xs_exp_max_geq_right<bool, int16_t>(true, (int16_t)(x_min - 1), x_max, [&](int16_t x) {
            const u32 lt = sl[x];
            const auto iv = interval<RIGHT>(j, lt);
            if (iv.first <= iv.second) {
                if (intersect(pb, pe, iv.first, iv.second, i, j, lce_l, lt, xc, f, false)) {
                    sa_iv = iv;
                    lce_r = lt;
                    return true;
                }
                sa_nxt = iv;
            }
            lce_r_nxt = lt;
            return false;
        });
        if (x_res < x_min || (x_res < x_max && sl[x_res + 1] < lce_r_min)) return;
        // (qc_right = the interval of lce_r; the probes below compute exact intervals, whether by
        // extend_right or by interpolate_right between qc_right and qc_right_nxt)
        // (the search keeps the last found interval -- every later probe is longer, its interval
        // inside -- and the last interval that found no point -- every later probe is shorter, its
        // interval around it: the narrowing of extend_right / interpolate_right)
        const u32 lce_r_max = lce_r_nxt == 0 ? e - j : (lce_r_nxt - 1);
        std::pair<u32, u32> sup = lce_r ? sa_iv : std::pair<u32, u32>{0, c - 1};
        auto fnc = [&](u32 lt) -> bool {
            const auto iv = interval<RIGHT>(j, lt, sup.first, sup.second, sa_nxt.first, sa_nxt.second);
            if (iv.first <= iv.second) {
                if (intersect(pb, pe, iv.first, iv.second, i, j, lce_l, lt, xc, f, false)) {
                    sup = iv;
                    return true;
                }
                sa_nxt = iv;
            }
            return false;
        };
        if (lce_r_nxt == 0) xs_exp_max_geq_right<bool, u32>(true, lce_r, lce_r_max, fnc);
        else xs_max_geq<bool, u32>(true, lce_r, lce_r_max, fnc);
    }

    // ---- the transforms
    template <class OUT>
    void section_with_samples(u32 sct, OUT&& out) const {
        const u32 b = sect[sct].beg, e = sect[sct + 1].beg;
        u32 fi = sect[sct].phr;
        factor fa = Fa[fi++];
        u32 beg_nxt = b + std::max<u32>(1, fa.len);
        u32 xc = xs_min_geq<u32, u32>(b, 0u, c - 1, [&](u32 x) { return C[x]; });
        const std::vector<u32>& ll = lens[LEFT];
        std::vector<u8> smpld(delta + 1, 0);
        for (u32 len : ll)
            if (len <= delta) smpld[len] = 1;
        for (u32 i = b; i < e;) {
            while (beg_nxt <= i) {
                fa = Fa[fi++];
                beg_nxt += std::max<u32>(1, fa.len);
            }
            factor f = fa;
            if (f.len != 0) {
                const u32 cut = f.len - (beg_nxt - i);
                f.len -= cut;
                f.src += cut;
            }
            const u32 max_k = std::min<u32>(delta, e - i);
            for (u32 x = 0; x < ll.size(); x++) {
                const u32 k = ll[x] - 1;
                if (k >= max_k) break;
                const u32 j = i + k;
                const auto iv = interval<LEFT>(j, k + 1);
                if (iv.first <= iv.second) extend_right_with_samples(iv.first, iv.second, i, j, e, xc, f);
            }
            for (u32 k = 2; k < max_k; k++) {
                const u32 lce_l = k + 1;
                if (smpld[lce_l]) continue;
                const u32 j = i + k;
                const auto iv = interval<LEFT>(j, lce_l);
                if (iv.first <= iv.second) extend_right_with_samples(iv.first, iv.second, i, j, e, xc, f);
            }
            if (f.len > e - i) f.len = e - i;
            out(f);
            i += std::max<u32>(1, f.len);
        }
    }
    template <class OUT>
    void section_without_samples(u32 sct, bool naive, OUT&& out) const {
        const u32 b = sect[sct].beg, e = sect[sct + 1].beg;
        u32 fi = sect[sct].phr;
        factor fa = Fa[fi++];
        u32 beg_nxt = b + std::max<u32>(1, fa.len);
        u32 xc = xs_min_geq<u32, u32>(b, 0u, c - 1, [&](u32 x) { return C[x]; });
        for (u32 i = b; i < e;) {
            while (beg_nxt <= i) {
                fa = Fa[fi++];
                beg_nxt += std::max<u32>(1, fa.len);
            }
            // (naive, naive.cpp:57: a literal to start from, no approximate lower bound)
            factor f = naive ? factor{T[i], 0} : fa;
            const u32 max_j = std::min<u32>(e, i + delta);
            if (f.len != 0) {
                const u32 cut = f.len - (beg_nxt - i);
                f.len -= cut;
                f.src += cut;
            }
            for (u32 j = i; j < max_j; j++) {
                const u32 lce_l = (j - i) + 1;
                const auto pa = interval<LEFT>(j, lce_l);
                if (pa.first > pa.second) continue;
                const u32 lce_r_min = f.len < j - i ? 0 : (i + f.len - j);
                const u32 lce_r_max = e - j;
                std::pair<u32, u32> sup{0, c - 1}, nxt{1, 0};
                xs_exp_max_geq_right<bool, u32>(true, lce_r_min, lce_r_max, [&](u32 lt) {
                    const auto iv = interval<RIGHT>(j, lt, sup.first, sup.second, nxt.first, nxt.second);
                    if (iv.first <= iv.second) {
                        if (intersect(pa.first, pa.second, iv.first, iv.second, i, j, lce_l, lt, xc, f, naive)) {
                            sup = iv;
                            return true;
                        }
                        nxt = iv;
                    }
                    return false;
                });
            }
            out(f);
            i += std::max<u32>(1, f.len);
        }
    }

    // the whole transform: approximate factors in, exact factors out (in text order)
    void run(const u8* T_, u32 n_, const lce_structure<u32>& L_, std::vector<factor>&& aprx, int p_, int mode,
             std::vector<factor>& outF) {
        T = T_;
        n = n_;
        L = &L_;
        p = std::max(1, p_);
        Fa = std::move(aprx);
        za = (u32)Fa.size();
        outF.clear();
        if (n == 0) return;
        delta = std::min<u32>(n / za, MAX_DELTA);
        build_c();
        sort_xa<LEFT>();
        sort_xa<RIGHT>();
        if (mode == ex_with_samples) {
            rk.build(T, n, p);
            // get_max_smpl_len_right (lz77_sss.hpp:124-127) of the approximate compression ratio
            const double cr = n / (double)za;
            const u32 msr = (u32)std::llround(cr * (1.0 + 0.5 * std::exp(-cr / 1000.0)));
            build_samples<LEFT>(delta);
            build_samples<RIGHT>(msr);
        } else {
            lens[LEFT] = {1, 2};
            lens[RIGHT] = {1, 2};
            ivs[LEFT].assign(2, {});
            ivs[RIGHT].assign(2, {});
        }
        build_points();
        const u32 nsect = (u32)sect.size() - 1;
        std::vector<std::vector<factor>> part(nsect);
#pragma omp parallel for num_threads(p) schedule(dynamic, 1)
        for (u64 s = 0; s < nsect; s++) {
            auto put = [&](factor f) { part[s].push_back(f); };
            if (mode == ex_with_samples) section_with_samples((u32)s, put);
            else section_without_samples((u32)s, mode == ex_naive, put);
        }
        for (auto& v : part) outF.insert(outF.end(), v.begin(), v.end());
    }
};

// factorize_exact<greedy, lpf_opt, mode> at p threads: the 3-approximation (oracle.hpp, p = 1
// stream for p = 1; LPF in p partitions otherwise, timing only), then the transform
static inline std::vector<factor> factorize_exact_smpl(u8* T, u32 n, int mode, int p, double* t_aprx = nullptr) {
    std::vector<factor> Fa;
    lce_structure<u32> L;
    const double t0 = omp_get_wtime();
    if (n) factorize_approximate<u32>(T, n, lpf_opt, 42, [&](factor f) { Fa.push_back(f); }, nullptr, 1, std::max(1, p), &L);
    if (t_aprx) *t_aprx = omp_get_wtime() - t0;
    std::vector<factor> F;
    exact_smpl X;
    X.run(T, n, L, std::move(Fa), p, mode, F);
    return F;
}

}  // namespace lzo
