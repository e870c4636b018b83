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
//   LCP      of SA neighbours in text order (Kasai lower bounds, chunked;
//            chunk starts and long extensions by the device LCE of lce_dev.h)
//   LPF(p)   = max(LCE(p, SA[psv]), LCE(p, SA[nsv])) (Crochemore-Ilie), each
//            LCE the minimum of LCP over the rank range, read off a min-tree
//            over LCP along the PSV/NSV descent; source = the candidate with
//            the longer LCE, the smaller text position on ties
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
// ranks are head ranks: R[i] = 1 + position in SA of the first suffix of i's
// group (0 = past the end, so a suffix ending before i + h sorts first);
// singletons keep their final position, so only suffixes in groups of >= 2
// (the active list A, kept in SA order) take part in later rounds
__global__ void k_sa_pairs(const u32* __restrict__ R, u64 n, const u32* __restrict__ A, u64 m, u64 h, u32 bits,
                           u64* __restrict__ key, u32* __restrict__ idx) {
    const u64 j = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= m) return;
    const u32 i = A[j];
    key[j] = ((u64)R[i] << bits) | (i + h < n ? R[i + h] : 0u);
    idx[j] = i;
}
// first-of-run markers for the max-scans: sub-groups (whole key) and groups (key >> gbits)
__global__ void k_sa_marks(const u64* __restrict__ skey, u64 m, u32 gbits, u32* __restrict__ sm,
                           u32* __restrict__ gm) {
    const u64 t = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= m) return;
    sm[t] = (t == 0 || skey[t] != skey[t - 1]) ? (u32)t : 0u;
    gm[t] = (t == 0 || (skey[t] >> gbits) != (skey[t - 1] >> gbits)) ? (u32)t : 0u;
}
struct max_op {
    __device__ __forceinline__ u32 operator()(const u32& a, const u32& b) const { return a > b ? a : b; }
};
// sorted active item t: SA position, new head rank, stays active iff its sub-group has >= 2 members
__global__ void k_sa_update(const u64* __restrict__ skey, const u32* __restrict__ sidx, u64 m, u32 gbits,
                            const u32* __restrict__ sfirst, const u32* __restrict__ gfirst, u32* __restrict__ SA,
                            u32* __restrict__ R, u8* __restrict__ act) {
    const u64 t = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= m) return;
    const u64 g0 = gbits >= 64 ? 0 : (skey[t] >> gbits) - 1;  // group head position (round 0: one group at 0)
    const u64 pos = g0 + t - gfirst[t];
    const u64 head = g0 + sfirst[t] - gfirst[t];
    SA[pos] = sidx[t];
    R[sidx[t]] = (u32)(head + 1);
    const bool first = sfirst[t] == t;
    const bool last = t + 1 == m || skey[t + 1] != skey[t];
    act[t] = (first && last) ? 0 : 1;
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
// Nearest rank left of r whose SA value is < v (NONE if none), and through
// *lce the LCE of the two suffixes = min LCP[psv+1 .. r].  The climb rejects
// left siblings whose SA minimum is >= v and the descent skips right children
// the same way; those nodes tile (psv, r), so their LCP-tree minima (same
// shape, tree C) give the LCE without touching the text.
__device__ u32 tree_prev(const min_tree& M, const min_tree& C, u64 r, u32 v, u32* lce) {
    u64 i = r;
    u32 k = 0, acc = C.lv[0][r];
    for (;;) {
        if (i == 0) return NONE;
        if (i & 1) {
            if (M.lv[k][i - 1] < v) {
                i = i - 1;
                break;
            }
            acc = min(acc, C.lv[k][i - 1]);
        }
        i >>= 1;
        k++;
        if (k >= M.nlev) return NONE;
    }
    while (k > 0) {  // rightmost leaf < v below (k, i)
        const u64 c = 2 * i + 1;
        k--;
        if (c < M.sz[k] && M.lv[k][c] < v) {
            i = c;
        } else {
            if (c < M.sz[k]) acc = min(acc, C.lv[k][c]);
            i = c - 1;
        }
    }
    *lce = acc;
    return (u32)i;
}
// Nearest rank right of r whose SA value is < v (NONE if none); *lce = min LCP[r+1 .. nsv].
__device__ u32 tree_next(const min_tree& M, const min_tree& C, u64 r, u32 v, u32* lce) {
    u64 i = r;
    u32 k = 0, acc = NONE;
    for (;;) {
        if (!(i & 1) && i + 1 < M.sz[k]) {
            if (M.lv[k][i + 1] < v) {
                i = i + 1;
                break;
            }
            acc = min(acc, C.lv[k][i + 1]);
        }
        i >>= 1;
        k++;
        if (k >= M.nlev || M.sz[k] <= 1) return NONE;
    }
    while (k > 0) {  // leftmost leaf < v below (k, i)
        const u64 c = 2 * i;
        k--;
        if (M.lv[k][c] < v) {
            i = c;
        } else {
            acc = min(acc, C.lv[k][c]);
            i = c + 1;
        }
    }
    *lce = min(acc, C.lv[0][i]);
    return (u32)i;
}

// LCP[r] = LCE(SA[r-1], SA[r]) in text order (Kasai: PLCP[i] >= PLCP[i-1] - 1),
// one thread per chunk of PLCP_CH positions; the chunk's first value and any
// extension past 64 bytes come from the SSS-backed device LCE
constexpr u32 PLCP_CH = 64;
__global__ void k_plcp(lce_view L, const u32* __restrict__ R, const u32* __restrict__ SA, u32* __restrict__ LCP) {
    const u64 i0 = ((u64)blockIdx.x * blockDim.x + threadIdx.x) * PLCP_CH;
    if (i0 >= L.n) return;
    const u64 i1 = min<u64>(L.n, i0 + PLCP_CH);
    u64 h = 0;
    bool exact = false;  // h is a valid lower bound carried from i-1
    for (u64 i = i0; i < i1; i++) {
        const u32 r = R[i] - 1;
        if (r == 0) {
            LCP[0] = 0;
            exact = false;
            continue;
        }
        const u64 prev = SA[r - 1];
        if (!exact) {
            h = dev_lce(L, prev, i);
        } else {
            h = h ? h - 1 : 0;
            const u64 lim = L.n - max<u64>(i, prev);
            if (h < lim) {
                const u64 step = min<u64>(64, lim - h);
                const u64 c = dev_naive_lce(L.T, prev + h, i + h, step);
                h += c;
                if (c == step && h < lim) h += dev_lce(L, prev + h, i + h);
            }
        }
        LCP[r] = (u32)h;
        exact = true;
    }
}

// LPF and source of every position (one thread per rank)
__global__ void k_lpf_exact(lce_view L, const u32* __restrict__ SA, min_tree M, min_tree C, u32* __restrict__ lpf,
                            u32* __restrict__ src) {
    const u64 r = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= L.n) return;
    const u32 p = SA[r];
    u32 la = 0, lb = 0;
    const u32 ps = tree_prev(M, C, r, p, &la), ns = tree_next(M, C, r, p, &lb);
    const u32 a = ps != NONE ? SA[ps] : NONE, b = ns != NONE ? SA[ns] : NONE;
    if (a == NONE) la = 0;
    if (b == NONE) lb = 0;
    const bool pick_a = la > lb || (la == lb && a < b);
    const u32 len = pick_a ? la : lb;
    lpf[p] = len;
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
    u64* key = x_key.get(n);
    u64* key2 = x_key2.get(n);
    u32* idx = x_idx.get(n);   // active list / sort values
    u32* idx2 = x_idx2.get(n); // sorted values
    u32* SA = x_sa.get(n);
    u32* R = x_rank.get(n);
    u32* sm = x_flag.get(n);
    u32* gm = x_lpf.get(n);    // scratch until the LPF pass
    u32* sf = x_src.get(n);    // scratch until the LPF pass
    u32* gf = x_lcp.get(n);    // scratch until the LCP pass
    u8* act = (u8*)x_mark.get(n / 4 + 1);
    u32 bits = 1;
    while (bits < 32 && (1ull << bits) <= n) bits++;
    u32* A = idx;   // active list (SA order)
    u32* B = idx2;  // sort values / next active list
    k_sa_init<<<cdiv(n, 256), 256, 0, st>>>(T, n, key, A);
    u64 m = n;
    for (u64 h = 0; m > 0; h = h ? 2 * h : SA_K0) {
        if (h > n) throw error(LZ77SSS_EINTERNAL, "exact mode: prefix doubling did not converge");
        const unsigned g = cdiv(m, 256);
        u32 *vin = A, *vout = B;  // round 0: iota in A, sorted into B
        if (h) {
            k_sa_pairs<<<g, 256, 0, st>>>(R, n, A, m, h, bits, key, B);
            vin = B;
            vout = A;
        }
        const int eb = h ? (int)(2 * bits) : 57;
        size_t tb = 0;
        LZ_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, key, key2, vin, vout, (int)m, 0, eb, st));
        u8* t = scan_tmp.get(tb);
        LZ_HIP(hipcub::DeviceRadixSort::SortPairs(t, tb, key, key2, vin, vout, (int)m, 0, eb, st));
        const u32 gbits = h ? bits : 64;
        k_sa_marks<<<g, 256, 0, st>>>(key2, m, gbits >= 64 ? 63 : gbits, sm, gm);
        size_t tb2 = 0;
        LZ_HIP(hipcub::DeviceScan::InclusiveScan(nullptr, tb2, sm, sf, max_op{}, (int)m, st));
        u8* t2 = scan_tmp.get(tb2);
        LZ_HIP(hipcub::DeviceScan::InclusiveScan(t2, tb2, sm, sf, max_op{}, (int)m, st));
        if (h) {
            LZ_HIP(hipcub::DeviceScan::InclusiveScan(t2, tb2, gm, gf, max_op{}, (int)m, st));
        } else {
            LZ_HIP(hipMemsetAsync(gf, 0, m * 4, st));
        }
        k_sa_update<<<g, 256, 0, st>>>(key2, vout, m, gbits, sf, gf, SA, R, act);
        // next active list (SA order): members of sub-groups of >= 2, into the other buffer
        u32* nxt = vout == A ? B : A;
        u32* cnt = counters.get(16);
        size_t tb3 = 0;
        LZ_HIP(hipcub::DeviceSelect::Flagged(nullptr, tb3, vout, act, nxt, cnt + 4, (int)m, st));
        u8* t3 = scan_tmp.get(tb3);
        LZ_HIP(hipcub::DeviceSelect::Flagged(t3, tb3, vout, act, nxt, cnt + 4, (int)m, st));
        const u64 m_prev = m;
        m = rd1(cnt + 4, st);
        if (debug_enabled()) std::fprintf(stderr, "[lz77sss-debug] sa_full round h=%llu items=%llu -> active %llu\n",
                                          (unsigned long long)h, (unsigned long long)m_prev, (unsigned long long)m);
        A = nxt;
        B = nxt == idx ? idx2 : idx;
        x_rounds++;
    }
    sa_full = SA;
    LZ_HIP(hipGetLastError());
}

u64 engine::factorize_exact(bool log) {
    LZ_HIP(hipSetDevice(device));
    if (n > 0xFFFFFFF0ull) throw error(LZ77SSS_EINVAL, "n too large for pos_t = uint32_t");
    num_fact = 0;
    last_fact_mode = LZ77SSS_GREEDY;
    stats.assign(28, 0);
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
    // LCP of SA neighbours, then min-trees over SA and LCP
    const lce_view LV = view(d_text);
    u32* lcp = x_lcp.get(n);
    k_plcp<<<cdiv(cdiv(n, PLCP_CH), 256), 256, 0, st>>>(LV, x_rank.p, sa_full, lcp);
    min_tree M{}, C{};
    M.lv[0] = sa_full;
    C.lv[0] = lcp;
    M.sz[0] = C.sz[0] = n;
    M.nlev = C.nlev = 1;
    {
        u64 total = 0;
        for (u64 sz = n; sz > 1; sz = (sz + 1) / 2) total += (sz + 1) / 2;
        u32* buf = x_tree.get(total + 1);
        u32* lbuf = x_ltree.get(total + 1);
        u64 o = 0;
        for (u64 sz = (n + 1) / 2; M.nlev < (u32)MAX_LV; sz = (sz + 1) / 2) {
            const u32 k = M.nlev;
            M.lv[k] = buf + o;
            C.lv[k] = lbuf + o;
            M.sz[k] = C.sz[k] = sz;
            k_tree_level<<<cdiv(sz, 256), 256, 0, st>>>(M.lv[k - 1], M.sz[k - 1], buf + o, sz);
            k_tree_level<<<cdiv(sz, 256), 256, 0, st>>>(C.lv[k - 1], C.sz[k - 1], lbuf + o, sz);
            o += sz;
            M.nlev = C.nlev = k + 1;
            if (sz == 1) break;
        }
    }
    u32* lpfa = x_lpf.get(n);
    u32* srca = x_src.get(n);
    k_lpf_exact<<<cdiv(n, 256), 256, 0, st>>>(LV, sa_full, M, C, lpfa, srca);
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
