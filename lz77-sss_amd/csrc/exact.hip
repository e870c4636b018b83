// exact.hip -- exact greedy LZ77 on the device (role of
// lz77_sss<>::factorize_exact<greedy, lpf_opt, transf_mode, range_ds_t, tau>,
// include/lz77_sss/lz77_sss.hpp:188-200 and 333-357; transform_to_exact/*.cpp).
//
// The reference refines its 3-approximation with sampled sources until every
// factor is a longest previous factor, so the factor LENGTHS of its exact mode
// are the canonical greedy LZ77 ones (at p = 1).  Its sources depend on the
// sample index and the range structure's visit order; here they follow one
// fixed rule instead:
//
//   SA       suffix array of T by prefix doubling (7-character keys, then
//            rank pairs, device radix sort per round)
//   PSV/NSV  for rank r: nearest ranks left / right whose suffix starts
//            earlier in T (min-tree over SA, descended per rank)
//   LPF(p)   = max(LCE(p, SA[psv]), LCE(p, SA[nsv])) with the device LCE of
//            lce_dev.h (Crochemore-Ilie); source = the candidate with the
//            longer LCE, the smaller text position on ties
//   factors  p_0 = 0, p_{k+1} = p_k + max(1, LPF(p_k)); a copy {src, LPF} when
//            LPF >= 1, else the literal {T[p], 0}
//
// The greedy chain is resolved with chunk speculation: one walk per chunk of
// XCH positions from the chunk start marks the positions it visits; a single
// thread then follows the real chain from chunk to chunk, walking only until
// it meets a marked position (the walks converge, after which the chunk's
// speculative exit is the real one); a counting walk and a writing walk per
// visited chunk emit the factors in order.
#include "../../include/lz77sss.h"
#include "../include/engine.h"

#include <hipcub/hipcub.hpp>

namespace lz {

// ---------------------------------------------------------------------------
// suffix array by prefix doubling
// initial key: the first SA_K0 = 7 characters in base 257 with c + 1 per
// character and 0 past the end, so a suffix shorter than 7 sorts before every
// suffix it is a proper prefix of (257^7 < 2^57)
constexpr u32 SA_K0 = 7;
__global__ void k_sa_init(const u8* __restrict__ T, u64 n, u64* __restrict__ key, u32* __restrict__ idx) {
    const u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const u64 x = ldu64(T + i);
    u64 k = 0;
#pragma unroll
    for (u32 j = 0; j < SA_K0; j++) k = k * 257 + (i + j < n ? ((x >> (8 * j)) & 255) + 1 : 0);
    key[i] = k;
    idx[i] = (u32)i;
}
__global__ void k_sa_flags(const u64* __restrict__ skey, u64 n, u32* __restrict__ flag) {
    const u64 t = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (t < n) flag[t] = (t == 0 || skey[t] != skey[t - 1]) ? 1u : 0u;
}
__global__ void k_sa_scatter(const u32* __restrict__ sidx, const u32* __restrict__ rank, u64 n, u32* __restrict__ R) {
    const u64 t = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (t < n) R[sidx[t]] = rank[t];
}
// ranks are 1-based; a suffix ending before i + h pairs with rank 0 (shorter sorts first)
__global__ void k_sa_pairs(const u32* __restrict__ R, u64 n, u64 h, u32 bits, u64* __restrict__ key,
                           u32* __restrict__ idx) {
    const u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    key[i] = ((u64)R[i] << bits) | (i + h < n ? R[i + h] : 0u);
    idx[i] = (u32)i;
}

// ---------------------------------------------------------------------------
// min-tree over SA (level 0 = SA itself; level k halves level k-1)
struct min_tree {
    const u32* lv[MAX_LV];
    u64 sz[MAX_LV];
    u32 nlev;
};
__global__ void k_tree_level(const u32* __restrict__ prev, u64 psz, u32* __restrict__ out, u64 sz) {
    const u64 j = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= sz) return;
    const u32 a = prev[2 * j], b = 2 * j + 1 < psz ? prev[2 * j + 1] : NONE;
    out[j] = min(a, b);
}
// nearest rank left of r whose SA value is < v (NONE if none)
__device__ u32 tree_prev(const min_tree& M, u64 r, u32 v) {
    u64 i = r;
    u32 k = 0;
    for (;;) {
        if (i == 0) return NONE;
        if ((i & 1) && M.lv[k][i - 1] < v) {
            i = i - 1;
            break;
        }
        i >>= 1;
        k++;
        if (k >= M.nlev) return NONE;
    }
    while (k > 0) {  // rightmost leaf < v below (k, i)
        const u64 c = 2 * i + 1;
        k--;
        i = (c < M.sz[k] && M.lv[k][c] < v) ? c : c - 1;
    }
    return (u32)i;
}
// nearest rank right of r whose SA value is < v (NONE if none)
__device__ u32 tree_next(const min_tree& M, u64 r, u32 v) {
    u64 i = r;
    u32 k = 0;
    for (;;) {
        if (!(i & 1) && i + 1 < M.sz[k] && M.lv[k][i + 1] < v) {
            i = i + 1;
            break;
        }
        i >>= 1;
        k++;
        if (k >= M.nlev || M.sz[k] <= 1) return NONE;
    }
    while (k > 0) {  // leftmost leaf < v below (k, i)
        const u64 c = 2 * i;
        k--;
        i = (M.lv[k][c] < v) ? c : c + 1;
    }
    return (u32)i;
}

// LPF and source of every position (one thread per rank)
__global__ void k_lpf_exact(lce_view L, const u32* __restrict__ SA, min_tree M, u32* __restrict__ lpf,
                            u32* __restrict__ src) {
    const u64 r = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= L.n) return;
    const u32 p = SA[r];
    const u32 ps = tree_prev(M, r, p), ns = tree_next(M, r, p);
    const u32 a = ps != NONE ? SA[ps] : NONE, b = ns != NONE ? SA[ns] : NONE;
    const u64 la = a != NONE ? dev_lce(L, a, p) : 0, lb = b != NONE ? dev_lce(L, b, p) : 0;
    const bool pick_a = la > lb || (la == lb && a < b);
    const u64 len = pick_a ? la : lb;
    lpf[p] = (u32)len;
    src[p] = len ? (pick_a ? a : b) : (u32)L.T[p];
}

// ---------------------------------------------------------------------------
// greedy chain by chunk speculation
constexpr u32 XCH = 1u << 18;  // positions per chunk (a multiple of 32)
__device__ __forceinline__ u32 step_len(const u32* lpf, u32 p) { return max(1u, lpf[p]); }
// speculative walk from the chunk start: marks visited positions, records the exit
__global__ void k_chain_spec(const u32* __restrict__ lpf, u64 n, u32 nch, u32* __restrict__ mark,
                             u32* __restrict__ spec_exit) {
    const u64 c = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= nch) return;
    const u64 lo = c * XCH, hi = min<u64>(n, lo + XCH);
    u64 p = lo;
    u32 word = 0, wi = (u32)(lo >> 5);
    while (p < hi) {
        const u32 w = (u32)(p >> 5);
        if (w != wi) {
            mark[wi] = word;
            for (u32 x = wi + 1; x < w; x++) mark[x] = 0;
            wi = w;
            word = 0;
        }
        word |= 1u << (p & 31);
        p += step_len(lpf, (u32)p);
    }
    const u32 wend = (u32)((hi + 31) >> 5);
    if (wi < wend) mark[wi] = word;
    for (u32 x = wi + 1; x < wend; x++) mark[x] = 0;
    spec_exit[c] = (u32)min<u64>(p, 0xFFFFFFFFull);
}
// the real chain, chunk by chunk (one thread): entry[c] = first chain position
// in chunk c (NONE if the chain jumps over it)
__global__ void k_chain_resolve(const u32* __restrict__ lpf, u64 n, u32 nch, const u32* __restrict__ mark,
                                const u32* __restrict__ spec_exit, u32* __restrict__ entry) {
    if (blockIdx.x != 0 || threadIdx.x != 0) return;
    u64 E = 0;
    for (u32 c = 0; c < nch; c++) {
        const u64 hi = min<u64>(n, (u64)(c + 1) * XCH);
        if (E >= hi) {
            entry[c] = NONE;
            continue;
        }
        entry[c] = (u32)E;
        u64 p = E;
        while (p < hi && !((mark[p >> 5] >> (p & 31)) & 1)) p += step_len(lpf, (u32)p);
        E = p < hi ? (u64)spec_exit[c] : p;  // merged with the speculative walk, or left the chunk
    }
}
// factors of each visited chunk: count (out == nullptr) or write at off[c]
__global__ void k_chain_emit(const u8* __restrict__ T, const u32* __restrict__ lpf, const u32* __restrict__ src,
                             u64 n, u32 nch, const u32* __restrict__ entry, u32* __restrict__ cnt,
                             const u64* __restrict__ off, u32* __restrict__ out) {
    const u64 c = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= nch) return;
    const u32 e = entry[c];
    if (e == NONE) {
        if (!out) cnt[c] = 0;
        return;
    }
    const u64 hi = min<u64>(n, (c + 1) * (u64)XCH);
    u64 p = e, k = out ? off[c] : 0;
    u32 z = 0;
    while (p < hi) {
        const u32 len = lpf[p];
        if (out) {
            out[2 * k] = src[p];
            out[2 * k + 1] = len;
            k++;
        }
        z++;
        p += max(1u, len);
    }
    if (!out) cnt[c] = z;
}

static u64 excl_scan_u32to64(const u32* cnt, u64* off, u32 m, dbuf<u8>& tmp, dbuf<u64>& wide, hipStream_t st);

void engine::build_sa_full(const u8* T) {
    if (n >= (1ull << 31)) throw error(LZ77SSS_EINVAL, "exact mode: n must be < 2^31 (radix sort item count)");
    const unsigned g = cdiv(n, 256);
    u64* key = x_key.get(n);
    u64* key2 = x_key2.get(n);
    u32* idx = x_idx.get(n);
    u32* idx2 = x_idx2.get(n);
    u32* R = x_rank.get(n);
    u32* flag = x_flag.get(n);
    u32* rank = x_lpf.get(n);  // scratch until the LPF pass
    k_sa_init<<<g, 256, 0, st>>>(T, n, key, idx);
    u32 bits = 1;
    while (bits < 32 && (1ull << bits) <= n) bits++;
    for (u64 h = 0;; h = h ? 2 * h : SA_K0) {
        if (h) k_sa_pairs<<<g, 256, 0, st>>>(R, n, h, bits, key, idx);
        const int eb = h ? (int)(2 * bits) : 57;
        size_t tb = 0;
        LZ_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, key, key2, idx, idx2, (int)n, 0, eb, st));
        u8* t = scan_tmp.get(tb);
        LZ_HIP(hipcub::DeviceRadixSort::SortPairs(t, tb, key, key2, idx, idx2, (int)n, 0, eb, st));
        k_sa_flags<<<g, 256, 0, st>>>(key2, n, flag);
        size_t tb2 = 0;
        LZ_HIP(hipcub::DeviceScan::InclusiveSum(nullptr, tb2, flag, rank, (int)n, st));
        u8* t2 = scan_tmp.get(tb2);
        LZ_HIP(hipcub::DeviceScan::InclusiveSum(t2, tb2, flag, rank, (int)n, st));
        k_sa_scatter<<<g, 256, 0, st>>>(idx2, rank, n, R);
        x_rounds++;
        if (rd1(rank + n - 1, st) == n) break;
        if (h > n) throw error(LZ77SSS_EINTERNAL, "exact mode: prefix doubling did not converge");
    }
    sa_full = idx2;  // sorted suffix starts (x_idx2)
    LZ_HIP(hipGetLastError());
}

u64 engine::factorize_exact(bool log) {
    LZ_HIP(hipSetDevice(device));
    if (n > 0xFFFFFFF0ull) throw error(LZ77SSS_EINVAL, "n too large for pos_t = uint32_t");
    num_fact = 0;
    stats.assign(24, 0);
    x_rounds = 0;
    if (n == 0) return 0;
    timer.begin(st);
    // LCE structure of the approximate path (SSS, SA_S, LCP/RMQ over S)
    build_sss(d_text);
    timer.mark("sss");
    build_sa_s(d_text);
    timer.mark("sa_s");
    build_lcp_rmq(d_text);
    timer.mark("lcp_rmq");
    build_sa_full(d_text);
    timer.mark("sa_full");
    // min-tree over SA
    min_tree M{};
    M.lv[0] = sa_full;
    M.sz[0] = n;
    M.nlev = 1;
    {
        u64 total = 0;
        for (u64 sz = n; sz > 1; sz = (sz + 1) / 2) total += (sz + 1) / 2;
        u32* buf = x_tree.get(total + 1);
        u64 o = 0;
        for (u64 sz = (n + 1) / 2; M.nlev < (u32)MAX_LV; sz = (sz + 1) / 2) {
            M.lv[M.nlev] = buf + o;
            M.sz[M.nlev] = sz;
            k_tree_level<<<cdiv(sz, 256), 256, 0, st>>>(M.lv[M.nlev - 1], M.sz[M.nlev - 1], buf + o, sz);
            o += sz;
            M.nlev++;
            if (sz == 1) break;
        }
    }
    u32* lpfa = x_lpf.get(n);
    u32* srca = x_src.get(n);
    k_lpf_exact<<<cdiv(n, 256), 256, 0, st>>>(view(d_text), sa_full, M, lpfa, srca);
    LZ_HIP(hipGetLastError());
    timer.mark("lpf_exact");
    // greedy chain
    const u32 nch = (u32)((n + XCH - 1) / XCH);
    u32* mark = x_mark.get(n / 32 + 2);
    u32* sexit = x_chunk.get(3 * (u64)nch + 3);
    u32* entry = sexit + nch + 1;
    u32* cnt = entry + nch + 1;
    k_chain_spec<<<cdiv(nch, 64), 64, 0, st>>>(lpfa, n, nch, mark, sexit);
    k_chain_resolve<<<1, 64, 0, st>>>(lpfa, n, nch, mark, sexit, entry);
    k_chain_emit<<<cdiv(nch, 64), 64, 0, st>>>(d_text, lpfa, srca, n, nch, entry, cnt, nullptr, nullptr);
    u64* off = x_off.get((u64)nch + 1);
    const u64 z = excl_scan_u32to64(cnt, off, nch, scan_tmp, x_wide, st);
    u32* F = fact.get(2 * z + 2);
    k_chain_emit<<<cdiv(nch, 64), 64, 0, st>>>(d_text, lpfa, srca, n, nch, entry, cnt, off, F);
    LZ_HIP(hipGetLastError());
    timer.mark("greedy_exact");
    LZ_HIP(hipStreamSynchronize(st));
    num_fact = z;
    stats[0] = s;
    stats[1] = has_runs;
    stats[18] = x_rounds;  // prefix-doubling rounds of the full suffix array
    if (log) {
        for (auto& [name, ms] : timer.read()) std::fprintf(stderr, "[lz77sss] %-12s %9.3f ms\n", name.c_str(), ms);
        std::fprintf(stderr, "[lz77sss] exact: n=%llu factors=%llu doubling rounds=%u\n", (unsigned long long)n,
                     (unsigned long long)z, x_rounds);
    }
    return z;
}

__global__ void k_widen(const u32* __restrict__ a, u32 m, u64* __restrict__ b) {
    const u64 k = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (k <= m) b[k] = k < m ? a[k] : 0;
}
// exclusive scan of m u32 counts into m+1 u64 offsets; returns the total
static u64 excl_scan_u32to64(const u32* cnt, u64* off, u32 m, dbuf<u8>& tmp, dbuf<u64>& wide, hipStream_t st) {
    u64* w = wide.get((u64)m + 1);
    k_widen<<<cdiv((u64)m + 1, 256), 256, 0, st>>>(cnt, m, w);
    size_t tb = 0;
    LZ_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, w, off, (int)(m + 1), st));
    u8* t = tmp.get(tb);
    LZ_HIP(hipcub::DeviceScan::ExclusiveSum(t, tb, w, off, (int)(m + 1), st));
    return rd1(off + m, st);
}

}  // namespace lz
