// sa_s.hip -- suffix order of the sync positions and the LCE structure
// (roles of lce_classic_for_sss: gsaca_for_lce + ISA + Kasai LCP + rmq_n,
// patched-files/external/lce/include/ds/lce_classic_for_sss.hpp:36-142, and
// of pred_index / reduce_fps_3tau_lexicographic, lce_sss.hpp:68-83; those
// sources are absent upstream).
//
// SA_S is the TRUE suffix order of the sync positions:
//   key_k = T[S[k] .. S[k] + max(3tau, S[k+1]-S[k]+2tau))  (last key: to n)
//   R_0   = lexicographic rank of key_k            (comparison merge sort)
//   R_h+1 = rank of (R_h[k], R_h[k+2^h])            (radix sort, prefix doubling)
// until all ranks are distinct.  LCP between SA-neighbours comes from binary
// lifting over the stored R_h levels plus one bounded key comparison.
#include "../include/engine.h"
#include "../include/lce_dev.h"

#include <hipcub/hipcub.hpp>
#include <rocprim/rocprim.hpp>

namespace lz {

__global__ void k_key_len(const u32* __restrict__ S, u32 s, u64 n, u32* __restrict__ KL) {
    const u64 k = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= s) return;
    const u64 beg = S[k];
    u64 len = (k + 1 < s) ? max<u64>(3 * TAU, (u64)S[k + 1] - S[k] + 2 * TAU) : n - beg;
    KL[k] = (u32)min<u64>(len, n - beg);
}

__device__ __forceinline__ int dev_key_cmp(const u8* T, const u32* S, const u32* KL, u32 a, u32 b) {
    const u64 la = KL[a], lb = KL[b], m = min(la, lb);
    const u64 c = dev_naive_lce(T, S[a], S[b], m);
    if (c < m) return T[(u64)S[a] + c] < T[(u64)S[b] + c] ? -1 : 1;
    return la < lb ? -1 : (la > lb ? 1 : 0);
}

struct key_less {
    const u8* T;
    const u32* S;
    const u32* KL;
    __device__ bool operator()(const u32& a, const u32& b) const { return dev_key_cmp(T, S, KL, a, b) < 0; }
};

__global__ void k_iota(u32* __restrict__ x, u32 m) {
    const u64 k = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (k < m) x[k] = (u32)k;
}
__global__ void k_key_diff(const u8* T, const u32* S, const u32* KL, const u32* __restrict__ idx, u32 s,
                           u32* __restrict__ flag) {
    const u64 t = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= s) return;
    flag[t] = (t == 0) ? 1u : (dev_key_cmp(T, S, KL, idx[t - 1], idx[t]) != 0 ? 1u : 0u);
}
__global__ void k_scatter_rank(const u32* __restrict__ idx, const u32* __restrict__ rank, u32 s, u32* __restrict__ R) {
    const u64 t = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (t < s) R[idx[t]] = rank[t];
}
__global__ void k_pack_pairs(const u32* __restrict__ R, u32 s, u32 h, u32 bits, u64* __restrict__ kv,
                             u32* __restrict__ idx) {
    const u64 k = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= s) return;
    const u64 r2 = (k + h < s) ? R[k + h] : 0;
    kv[k] = ((u64)R[k] << bits) | r2;
    idx[k] = (u32)k;
}
__global__ void k_pair_diff(const u64* __restrict__ kv, u32 s, u32* __restrict__ flag) {
    const u64 t = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= s) return;
    flag[t] = (t == 0 || kv[t] != kv[t - 1]) ? 1u : 0u;
}
__global__ void k_sa_from_rank(const u32* __restrict__ R, u32 s, u32* __restrict__ SA, u32* __restrict__ ISA) {
    const u64 k = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= s) return;
    const u32 r = R[k] - 1;
    SA[r] = (u32)k;
    ISA[k] = r;
}

struct rank_levels {
    u32 nlev;
    const u32* R[MAX_LV];
};

// LCP[r] = LCE(S[SA[r-1]], S[SA[r]]), r >= 1; LCP[0] = 0
__global__ void k_lcp(const u8* __restrict__ T, u64 n, const u32* __restrict__ S, const u32* __restrict__ KL,
                      const u32* __restrict__ SA, u32 s, rank_levels RL, u32* __restrict__ LCP) {
    const u64 r = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= s) return;
    if (r == 0) { LCP[0] = 0; return; }
    const u32 a = SA[r - 1], b = SA[r];
    u64 c = 0;
    for (int lv = (int)RL.nlev - 1; lv >= 0; lv--) {
        const u64 w = 1ull << lv;
        if (a + c < s && b + c < s && RL.R[lv][a + c] == RL.R[lv][b + c]) c += w;
    }
    u64 v;
    if (a + c >= s) v = n - S[a];
    else if (b + c >= s) v = n - S[b];
    else {
        const u32 ka = (u32)(a + c), kb = (u32)(b + c);
        const u64 m = min(KL[ka], KL[kb]);
        v = ((u64)S[ka] - S[a]) + dev_naive_lce(T, S[ka], S[kb], m);
    }
    LCP[r] = (u32)v;
}

__global__ void k_min_level(const u32* __restrict__ prev, u32 cnt, u32 half, u32* __restrict__ out) {
    const u64 k = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (k < cnt) out[k] = min(prev[k], prev[k + half]);
}

__global__ void k_succ_table(const u32* __restrict__ S, u32 s, u64 nb, u32* __restrict__ tab) {
    const u64 bkt = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (bkt >= nb) return;
    const u64 x = bkt << 9;
    u32 lo = 0, hi = s;
    while (lo < hi) {
        u32 mid = (lo + hi) >> 1;
        if ((u64)S[mid] < x) lo = mid + 1; else hi = mid;
    }
    tab[bkt] = lo;
}

static void scan_incl(u32* in, u32* out, u32 m, dbuf<u8>& tmp, hipStream_t st) {
    size_t tb = 0;
    LZ_HIP(hipcub::DeviceScan::InclusiveSum(nullptr, tb, in, out, (int)m, st));
    u8* t = tmp.get(tb);
    LZ_HIP(hipcub::DeviceScan::InclusiveSum(t, tb, in, out, (int)m, st));
}

void engine::build_sa_s(const u8* T) {
    nlev_rank = 0;
    if (s == 0) return;
    const u32* dS = S.p;
    u32* KL = key_len.get(s);
    const unsigned g = cdiv(s, 256);
    k_key_len<<<g, 256, 0, st>>>(dS, s, n, KL);
    // ---- R_0: comparison merge sort of the keys
    u32* idx_in = u32a.get(s);
    u32* idx = u32b.get(s);
    k_iota<<<g, 256, 0, st>>>(idx_in, s);
    {
        size_t tb = 0;
        key_less cmp{T, dS, KL};
        LZ_HIP(rocprim::merge_sort(nullptr, tb, idx_in, idx, (size_t)s, cmp, st));
        u8* t = scan_tmp.get(tb);
        LZ_HIP(rocprim::merge_sort(t, tb, idx_in, idx, (size_t)s, cmp, st));
    }
    u32* flag = u32c.get(s);
    u32* rank = u32d.get(s);
    k_key_diff<<<g, 256, 0, st>>>(T, dS, KL, idx, s, flag);
    scan_incl(flag, rank, s, scan_tmp, st);
    u32* R0 = rank_lv[0].get(s);
    k_scatter_rank<<<g, 256, 0, st>>>(idx, rank, s, R0);
    nlev_rank = 1;
    u32 maxr = rd1(rank + s - 1, st);
    // ---- prefix doubling over the sequence of key ranks
    u32 bits = 1;
    while (bits < 32 && (1ull << bits) <= s) bits++;
    u64* kv = u64a.get(s);
    u64* kv2 = u64b.get(s);
    while (maxr < s) {
        if (nlev_rank >= MAX_LV) throw error(-6, "prefix doubling did not converge");
        const u32 h = 1u << (nlev_rank - 1);
        const u32* R = rank_lv[nlev_rank - 1].p;
        k_pack_pairs<<<g, 256, 0, st>>>(R, s, h, bits, kv, idx_in);
        size_t tb = 0;
        LZ_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, kv, kv2, idx_in, idx, (int)s, 0, (int)(2 * bits), st));
        u8* t = scan_tmp.get(tb);
        LZ_HIP(hipcub::DeviceRadixSort::SortPairs(t, tb, kv, kv2, idx_in, idx, (int)s, 0, (int)(2 * bits), st));
        k_pair_diff<<<g, 256, 0, st>>>(kv2, s, flag);
        scan_incl(flag, rank, s, scan_tmp, st);
        u32* Rn = rank_lv[nlev_rank].get(s);
        k_scatter_rank<<<g, 256, 0, st>>>(idx, rank, s, Rn);
        nlev_rank++;
        maxr = rd1(rank + s - 1, st);
    }
    k_sa_from_rank<<<g, 256, 0, st>>>(rank_lv[nlev_rank - 1].p, s, SA.get(s), ISA.get(s));
    LZ_HIP(hipGetLastError());
}

void engine::build_lcp_rmq(const u8* T) {
    nlev_rmq = 0;
    const u64 nb = (n >> 9) + 2;
    u32* tab = succ_tab.get(nb);
    k_succ_table<<<cdiv(nb, 256), 256, 0, st>>>(S.p, s, nb, tab);
    if (s == 0) return;
    const unsigned g = cdiv(s, 256);
    rank_levels RL{};
    RL.nlev = nlev_rank;
    for (u32 i = 0; i < nlev_rank; i++) RL.R[i] = rank_lv[i].p;
    u32* L0 = lcp_rmq[0].get(s);
    k_lcp<<<g, 256, 0, st>>>(T, n, S.p, key_len.p, SA.p, s, RL, L0);
    nlev_rmq = 1;
    for (u32 lv = 1; (1ull << lv) <= s; lv++) {
        const u32 cnt = s - (1u << lv) + 1;
        u32* out = lcp_rmq[lv].get(cnt);
        k_min_level<<<cdiv(cnt, 256), 256, 0, st>>>(lcp_rmq[lv - 1].p, cnt, 1u << (lv - 1), out);
        nlev_rmq = lv + 1;
    }
    LZ_HIP(hipGetLastError());
}

lce_view engine::view(const u8* T) const {
    lce_view L{};
    L.T = T;
    L.n = n;
    L.s = s;
    L.S = S.p;
    L.ISA = ISA.p;
    L.succ = succ_tab.p;
    L.nlev = nlev_rmq;
    for (u32 i = 0; i < nlev_rmq; i++) L.rmq[i] = lcp_rmq[i].p;
    return L;
}

}  // namespace lz
