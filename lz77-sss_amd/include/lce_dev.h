// lce_dev.h -- exact longest-common-extension queries on the device.
// Role of lce::ds::lce_sss::lce / lce_lr (patched-files/external/lce/include/
// ds/lce_sss.hpp:102-177): naive comparison of up to 3*tau bytes, then the
// successor sync positions and an RMQ over the LCP of the suffix-sorted sync
// positions.  Unlike the reference (which asserts the K&K lemma in its
// "case 1"), the unsynchronized case is resolved by a bounded comparison, so
// every value returned is the exact LCE.
#pragma once
#include "lz77sss_internal.h"

namespace LZ_NS {

constexpr int MAX_LV = 32;
constexpr u32 LCP_SAT = 0xFFFFFFFFu;  // stored LCP values saturate here (pos_t = uint64_t only)

// Periodic runs seen by the Q anchors (csrc/sss.hip): for anchor t (position
// 128t) whose window T[128t..128t+340) has smallest period p <= 170: p[t] = p,
// hi[t] = exclusive end and lo[t] = start of the maximal p-periodic run that
// contains the window (hi = 0 / lo = ~0 when unknown); p[t] = 0 otherwise.
// Long naive comparisons skip through runs with them: once 512 equal bytes
// end inside runs of the same period on both sides, the two strings stay
// equal until the first of the runs ends, and differ right there if the run
// ends are at different offsets.
struct run_tab {
    const u8* p = nullptr;
    const pos_t* hi = nullptr;
    const pos_t* lo = nullptr;
    // Per-block run records from the SSS pass (csrc/sss.hip k_sss_runs + k_blk_runinfo): for a
    // 512-byte block b that is p-extendable (T[z] == T[z+p] for z in [512b, 512b+512)),
    //   re[b] = end << 16 | exact << 8 | p,  rs[b] = start << 16 | exact << 8 | p
    // where [start, end) is the p-periodic run holding it (the end exact or a lower bound, the
    // start exact or an upper bound); 0 for other blocks.  One load per side of a skip.
    const u64* re = nullptr;
    const u64* rs = nullptr;
    u64 nbk = 0;
    unsigned long long* dbg = nullptr;  // LZ77SSS_LCE_DEBUG: step / skip counters (engine::lce_dbg)
};
__device__ __forceinline__ void lce_count(const run_tab& R, int c) {
    if (R.dbg) atomicAdd(R.dbg + c, 1ull);
}
// One side of a run skip.  Forward: T[x-512..x) matched; the run around x - 1 must hold
// [x - 340, x) -- from the block records (the block holding x - 1, or the one before it whose
// run may end inside x - 1's block) or else from the Q-anchor table (the anchor of x - 340,
// whose probe [a, a + 340) lies inside the matched bytes; its end is exact when known).
// Output: e = the run's end, exact or a lower bound.  Backward: T[x..x+512) matched, the run
// around x holds [x, x + 340); output its start (exact or an upper bound).
__device__ __forceinline__ bool run_side_fwd(const run_tab& R, u64 x, u64& e, bool& xe) {
    if (R.re) {
        const u64 b = (x - 1) >> 9;
        const u64 v0 = R.re[b], u0 = R.rs[b], v1 = b ? R.re[b - 1] : 0, u1 = b ? R.rs[b - 1] : 0;
        if ((v0 & 255) && (u0 >> 16) + 340 <= x && (v0 >> 16) >= x) {
            e = v0 >> 16;
            xe = (v0 >> 8) & 1;
            return true;
        }
        if ((v1 & 255) && (u1 >> 16) + 340 <= x && (v1 >> 16) >= x) {
            e = v1 >> 16;
            xe = (v1 >> 8) & 1;
            return true;
        }
    }
    if (R.p) {
        const u64 a = (x - 340) >> 7;
        if (R.p[a]) {
            const u64 hi = R.hi[a];  // 0: unknown
            if (hi >= x) {
                e = hi;
                xe = true;
                return true;
            }
        }
    }
    return false;
}
__device__ __forceinline__ bool run_side_bwd(const run_tab& R, u64 x, u64& s0, bool& xs) {
    if (R.re) {
        const u64 b = x >> 9;
        const bool nx = b + 1 < R.nbk;
        const u64 v0 = R.re[b], u0 = R.rs[b], v1 = nx ? R.re[b + 1] : 0, u1 = nx ? R.rs[b + 1] : 0;
        if ((u0 & 255) && (u0 >> 16) <= x && (v0 >> 16) >= x + 340) {
            s0 = u0 >> 16;
            xs = (u0 >> 8) & 1;
            return true;
        }
        if ((u1 & 255) && (u1 >> 16) <= x && (v1 >> 16) >= x + 340) {
            s0 = u1 >> 16;
            xs = (u1 >> 8) & 1;
            return true;
        }
    }
    if (R.p) {
        const u64 a = (x + 127) >> 7;
        if (R.p[a]) {
            const u64 lo = R.lo[a];  // RUN_LO_UNKNOWN: larger than every position
            if (lo <= x) {
                s0 = lo;
                xs = true;
                return true;
            }
        }
    }
    return false;
}
// T[x-512..x) == T[y-512..y), both inside periodic runs (run_side_fwd).  The two periods px,
// py may differ: the runs share [x - 340, x) ~ [y - 340, y), 340 >= px + py bytes, so both
// have the period gcd(px, py) there and, being px- resp. py-periodic, everywhere (Fine-Wilf).
// Returns 0: no skip; 1: equal for *d more bytes (go on comparing from there); 2: they differ
// exactly at *d (the run that ends first ends exactly there, the other goes on)
__device__ __forceinline__ int run_skip_fwd(const run_tab& R, u64 x, u64 y, u64& d) {
    u64 ex, ey;
    bool xx, xy;
    if (!run_side_fwd(R, x, ex, xx) || !run_side_fwd(R, y, ey, xy)) return 0;
    const u64 dx = ex - x, dy = ey - y;
    d = min(dx, dy);
    return (dx != dy && (dx < dy ? xx : xy)) ? 2 : 1;
}
// T[x..x+512) == T[y..y+512): the same going left
__device__ __forceinline__ int run_skip_bwd(const run_tab& R, u64 x, u64 y, u64& d) {
    u64 sx, sy;
    bool xx, xy;
    if (!run_side_bwd(R, x, sx, xx) || !run_side_bwd(R, y, sy, xy)) return 0;
    const u64 dx = x - sx, dy = y - sy;
    d = min(dx, dy);
    return (dx != dy && (dx < dy ? xx : xy)) ? 2 : 1;
}

// exact LCE of T[i..] and T[j..], at most lim (caller guarantees i+lim, j+lim <= n)
__device__ inline u64 dev_lce_fwd(const u8* T, const run_tab& R, u64 i, u64 j, u64 lim) {
    u64 k = 0;
    lce_count(R, 0);
    u64 nst = 0;
    while (k < lim) {
        const u64 step = min<u64>(lim - k, 512);
        lce_count(R, 1);
        if (R.dbg && ++nst > R.dbg[4]) atomicMax(R.dbg + 4, nst);
        const u64 c = dev_naive_lce(T, i + k, j + k, step);
        k += c;
        if (c < step || k >= lim) return min(k, lim);
        if (!(R.p || R.re) || k < 512) continue;  // no run table: plain comparison of the next 512 bytes
        u64 dj;
        if (const int sk = run_skip_fwd(R, i + k, j + k, dj)) {  // T[x-512..x) == T[y-512..y)
            lce_count(R, sk == 2 ? 3 : 2);
            if (k + dj >= lim) return lim;
            k += dj;
            if (sk == 2) return k;
        }
    }
    return lim;
}
// wave-cooperative dev_lce_fwd: all 64 lanes call it with the same arguments and
// get the same result; 512 bytes are compared per step (8 per lane)
__device__ inline u64 wave_lce_fwd(const u8* T, const run_tab& R, u64 i, u64 j, u64 lim, u32 lane) {
    u64 k = 0;
    while (k < lim) {
        const u64 step = min<u64>(lim - k, 512);
        const u64 off = 8 * lane;
        bool diff = false;
        if (off < step) {
            u64 x = ldu64(T + i + k + off), y = ldu64(T + j + k + off);
            const u64 r = step - off;
            if (r < 8) { const u64 msk = (1ull << (8 * r)) - 1; x &= msk; y &= msk; }
            diff = x != y;
        }
        const u64 bal = __ballot(diff);
        if (bal) {
            const u64 fo = k + 8 * (u64)__builtin_ctzll(bal);
            const u64 x = ldu64(T + i + fo), y = ldu64(T + j + fo);
            return fo + (__builtin_ctzll(x ^ y) >> 3);
        }
        k += step;
        if (k >= lim) return min(k, lim);
        if (!(R.p || R.re) || k < 512) continue;
        u64 dj;
        if (const int sk = run_skip_fwd(R, i + k, j + k, dj)) {
            if (k + dj >= lim) return lim;
            k += dj;
            if (sk == 2) return k;
        }
    }
    return lim;
}
// #equal chars going left from i and j (T[i-t] == T[j-t]), at most lim <= min(i,j)+1
__device__ __forceinline__ u64 dev_naive_lce_left(const u8* T, u64 i, u64 j, u64 lim) {
    u64 k = 0;
    while (k + 32 <= lim) {  // 32 bytes per memory round trip (dev_naive_lce)
        u64 x[4], y[4];
#pragma unroll
        for (int t = 0; t < 4; t++) {
            x[t] = ldu64(T + (i - k - 8 * t - 7));
            y[t] = ldu64(T + (j - k - 8 * t - 7));
        }
#pragma unroll
        for (int t = 0; t < 4; t++)
            if (x[t] != y[t]) return k + 8 * t + (__builtin_clzll(x[t] ^ y[t]) >> 3);
        k += 32;
    }
    while (k + 8 <= lim) {
        const u64 x = ldu64(T + (i - k - 7)), y = ldu64(T + (j - k - 7));
        if (x != y) return k + (__builtin_clzll(x ^ y) >> 3);
        k += 8;
    }
    while (k < lim && T[i - k] == T[j - k]) k++;
    return k;
}
__device__ inline u64 dev_lce_bwd(const u8* T, const run_tab& R, u64 i, u64 j, u64 lim) {
    u64 k = 0;
    lce_count(R, 5);
    while (k < lim) {
        const u64 step = min<u64>(lim - k, 512);
        lce_count(R, 6);
        const u64 c = dev_naive_lce_left(T, i - k, j - k, step);
        k += c;
        if (c < step || k >= lim) return min(k, lim);
        if (!(R.p || R.re) || k < 512) continue;  // no run table: plain comparison of the next 512 bytes
        u64 dj;
        if (const int sk = run_skip_bwd(R, i - k + 1, j - k + 1, dj)) {  // T[x..x+512) == T[y..y+512)
            lce_count(R, 7);
            if (k + dj >= lim) return lim;
            k += dj;
            if (sk == 2) return k;
        }
    }
    return lim;
}

struct lce_view {
    const u8* T;
    u64 n;
    u32 s;
    const pos_t* S;
    const u32* ISA;
    const u32* succ;  // bucket (x >> 9) -> first sync index with S >= bucket*512
    u32 nlev;
    const u32* rmq[MAX_LV];
    run_tab R;
};

__device__ __forceinline__ u32 dev_succ(const lce_view& L, u64 x) {
    u32 k = L.succ[x >> 9];
    while (k < L.s && L.S[k] < x) k++;
    return k;
}
// min LCP over ranks (a, b], a < b
__device__ __forceinline__ u32 dev_rmq(const lce_view& L, u32 a, u32 b) {
    const u32 l = a + 1, len = b - a;
    const u32 lv = 31 - __builtin_clz(len);
    const u32* t = L.rmq[lv];
    return min(t[l], t[b + 1 - (1u << lv)]);
}
__device__ __forceinline__ u64 dev_lce_sync(const lce_view& L, u32 ka, u32 kb) {
    u32 a = L.ISA[ka], b = L.ISA[kb];
    if (a > b) { u32 t = a; a = b; b = t; }
    return dev_rmq(L, a, b);
}
__device__ __forceinline__ u64 dev_lce(const lce_view& L, u64 i, u64 j) {
    if (i == j) return L.n - i;
    const u64 l = min(i, j), r = max(i, j);
    const u64 lmax = L.n - r, local = min<u64>(64, lmax);
    // a short naive probe settles most queries; longer ones go straight to the
    // successor sync positions (the reference compares 3*tau bytes first; the
    // result is the same exact LCE)
    u64 c = dev_naive_lce(L.T, l, r, local);
    if (c < local || c == lmax) return c;
    const u32 kl = dev_succ(L, l), kr = dev_succ(L, r);
    if (kl == L.s || kr == L.s) return c + dev_lce_fwd(L.T, L.R, l + c, r + c, lmax - c);
    const u64 dl = L.S[kl] - l, dr = L.S[kr] - r;
    if (dl == dr) {
        if (dl > c) {
            const u64 e = dev_lce_fwd(L.T, L.R, l + c, r + c, dl - c);
            if (e < dl - c) return c + e;
        }
        const u64 v = dev_lce_sync(L, kl, kr);
        if (sizeof(pos_t) > 4 && v == LCP_SAT)  // saturated LCP: finish by comparison
            return dl + v + dev_lce_fwd(L.T, L.R, l + dl + v, r + dl + v, lmax - dl - v);
        return dl + v;
    }
    const u64 bound = min(min(dl, dr) + 2 * TAU - 1, lmax);
    if (bound > c) c += dev_lce_fwd(L.T, L.R, l + c, r + c, bound - c);
    return c;
}

// leftward LCE, exact semantics of lce_l_64 (include/lz77_sss/algorithms/lce_l.hpp:33-83):
// min(cap', #equal chars going left from i and j), cap' = min(cap, min(i,j)+1)
__device__ __forceinline__ pos_t dev_lce_left(const u8* T, const run_tab& R, pos_t i, pos_t j, pos_t cap) {
    const pos_t cp = min(cap, (pos_t)(min(i, j) + 1));
    if (i == j) return cp;
    return (pos_t)dev_lce_bwd(T, R, i, j, cp);
}

}  // namespace LZ_NS
