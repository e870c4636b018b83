// lce_dev.h -- exact longest-common-extension queries on the device.
// Role of lce::ds::lce_sss::lce / lce_lr (patched-files/external/lce/include/
// ds/lce_sss.hpp:102-177): naive comparison of up to 3*tau bytes, then the
// successor sync positions and an RMQ over the LCP of the suffix-sorted sync
// positions.  Unlike the reference (which asserts the K&K lemma in its
// "case 1"), the unsynchronized case is resolved by a bounded comparison, so
// every value returned is the exact LCE.
#pragma once
#include "lz77sss_internal.h"

namespace lz {

constexpr int MAX_LV = 32;

struct lce_view {
    const u8* T;
    u64 n;
    u32 s;
    const u32* S;
    const u32* ISA;
    const u32* succ;  // bucket (x >> 9) -> first sync index with S >= bucket*512
    u32 nlev;
    const u32* rmq[MAX_LV];
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
    const u64 lmax = L.n - r, local = min<u64>(3 * TAU, lmax);
    u64 c = dev_naive_lce(L.T, l, r, local);
    if (c < local || c == lmax) return c;
    const u32 kl = dev_succ(L, l), kr = dev_succ(L, r);
    if (kl == L.s || kr == L.s) return c + dev_naive_lce(L.T, l + c, r + c, lmax - c);
    const u64 dl = L.S[kl] - l, dr = L.S[kr] - r;
    if (dl == dr) {
        if (dl > c) {
            const u64 e = dev_naive_lce(L.T, l + c, r + c, dl - c);
            if (e < dl - c) return c + e;
        }
        return dl + dev_lce_sync(L, kl, kr);
    }
    const u64 bound = min(min(dl, dr) + 2 * TAU - 1, lmax);
    if (bound > c) c += dev_naive_lce(L.T, l + c, r + c, bound - c);
    return c;
}

// leftward LCE, exact semantics of lce_l_64 (include/lz77_sss/algorithms/lce_l.hpp:33-83):
// min(cap', #equal chars going left from i and j), cap' = min(cap, min(i,j)+1)
__device__ __forceinline__ u32 dev_lce_left(const u8* T, u32 i, u32 j, u32 cap) {
    const u32 cp = min(cap, min(i, j) + 1);
    if (i == j) return cp;
    u32 k = 0;
    // 8 bytes at a time while possible
    while (k + 8 <= cp) {
        const u64 x = ldu64(T + (i - k - 7)), y = ldu64(T + (j - k - 7));
        if (x != y) return k + (__builtin_clzll(x ^ y) >> 3);
        k += 8;
    }
    while (k < cp && T[i - k] == T[j - k]) k++;
    return k;
}

}  // namespace lz
