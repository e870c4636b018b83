// lnf.hip -- the LPF/LNF phrase mode (factorize_approximate<greedy, lpf_lnf_opt>,
// config 3): every PSV/NSV phrase of the text and every PGV/NGV phrase of the
// reversed text, deduplicated by "same diagonal as the last phrase of the
// stream", then the greedy phrase selection.  Restates, for p = 1:
//   build_PGV_NGV_S            nxv_pxv.cpp:94-156
//   build_LNF_all / LPF_all    approximate/lpf_lnf/lpf_lnf.cpp:31-249
//   greedy_phrase_selection    approximate/common.cpp:31-96 (ips4o -> stable order)
//   in-place reversal          lz77_sss.hpp:385-393 (here: a reversed device copy)
//
// Device formulation:
//   * candidates per sync index and stream side are independent; the dedupe
//     state of a stream is "the last pushed phrase", so the pushed phrases form
//     a path: next(i) = first valid j > i not skipped by i, which is either the
//     end of i's equal-diagonal run or the first j whose start reaches i's end
//     (binary search) -> pointer doubling from the first valid candidate;
//   * phrases keep the reference's push order through sequence slots and a
//     stable radix sort on (beg asc, end desc);
//   * the selection loop's next choice depends only on the current phrase c
//     (X(c) = first phrase starting after end(c), and the first argmax of end
//     over [0, X(c)) by a prefix max-scan), so it is pointer doubling again; the
//     loop's window start only matters for its last-phrase quirk
//     (common.cpp:58-75) and is recovered by a max-scan along the path.
#include "../include/engine.h"
#include "../include/prim.h"
#include "../include/lce_dev.h"

#include <hipcub/hipcub.hpp>

namespace LZ_NS {

__global__ void k_reverse(const u8* __restrict__ T, u64 n, u8* __restrict__ R) {
    for (u64 i = gtid(); i < n; i += gstride()) R[i] = T[n - 1 - i];
}
__global__ void k_sa_lvl(const u32* __restrict__ prev, u32 cnt, u32 half, int want_max, u32* __restrict__ out) {
    const u64 k = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (k < cnt) out[k] = want_max ? max(prev[k], prev[k + half]) : min(prev[k], prev[k + half]);
}
struct sa_levels {
    u32 nlev;
    const u32* L[MAX_LV];
};
// smaller (want_max = 0: PSV/NSV) or greater (1: PGV/NGV) previous/next value of SA over ranks
__global__ void k_pnv(const u32* __restrict__ SA, u32 s, sa_levels M, int want_max, u32* __restrict__ PV,
                      u32* __restrict__ NV) {
    const u64 r = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= s) return;
    const u32 v = SA[r];
    auto blocked = [&](u32 x) { return want_max ? x < v : x > v; };  // a run of such values is skipped
    u64 pos = r;
    for (int lv = (int)M.nlev - 1; lv >= 0; lv--) {
        const u64 w = 1ull << lv;
        if (pos >= w && blocked(M.L[lv][pos - w])) pos -= w;
    }
    PV[r] = pos == 0 ? s : (u32)(pos - 1);
    pos = r + 1;
    for (int lv = (int)M.nlev - 1; lv >= 0; lv--) {
        const u64 w = 1ull << lv;
        if (pos + w <= s && blocked(M.L[lv][pos])) pos += w;
    }
    NV[r] = pos >= s ? s : (u32)pos;
}

// candidate record per (sync index, side): valid, diag, end, beg, src
// (positions are pos_t: the pos_t = uint64_t build serves lz77_sss<uint64_t>::factorize_approximate
// <greedy, lpf_lnf_opt>, lz77_sss.hpp:384-396 instantiated with either pos_t)
constexpr int AREC = 5;
__global__ void k_all_candidates(lce_view L, const u32* __restrict__ SA, const u32* __restrict__ PV,
                                 const u32* __restrict__ NV, int lnf, int opt, pos_t* __restrict__ rec) {
    const u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    const u32 s = L.s;
    if (i >= s) return;
    const pos_t Si = L.S[i];
    const u32 r = L.ISA[i];
    for (int side = 0; side < 2; side++) {
        pos_t* o = rec + (2 * i + side) * AREC;
        const u32 nb = side ? NV[r] : PV[r];
        if (nb == s) { o[0] = 0; continue; }
        pos_t src = L.S[SA[nb]], beg = Si;
        const pos_t diag = lnf ? src - beg : beg - src;
        const pos_t end = Si + (pos_t)dev_lce(L, src, Si);
        if (opt && src != 0 && Si != 0) {
            const pos_t l = dev_lce_left(L.T, L.R, src - 1, Si - 1, POS_NONE);
            beg -= l;
            src -= l;
        }
        o[0] = (end - beg > 1) ? 1u : 2u;  // 1 valid, 2 exists but too short (no state change)
        o[1] = diag;
        o[2] = end;
        o[3] = beg;
        o[4] = src;
    }
}
__global__ void k_side_flags(const pos_t* __restrict__ rec, u32 s, int side, u32* __restrict__ f) {
    const u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < s) f[i] = rec[(2 * i + side) * AREC] == 1u;
}
__global__ void k_side_compact(const pos_t* __restrict__ rec, const pos_t* __restrict__ S, u32 s, int side,
                               const u32* __restrict__ off, u32* __restrict__ V, pos_t* __restrict__ bV,
                               pos_t* __restrict__ dV, pos_t* __restrict__ eV) {
    const u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= s) return;
    const pos_t* r = rec + (2 * i + side) * AREC;
    if (r[0] != 1u) return;
    const u32 k = off[i];
    V[k] = (u32)i;
    bV[k] = S[i];
    dV[k] = r[1];
    eV[k] = r[2];
}
__global__ void k_diag_change(const pos_t* __restrict__ dV, u32 nv, u32* __restrict__ chg) {
    const u64 k = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (k < nv) chg[k] = (k == 0 || dV[k] != dV[k - 1]) ? 1u : 0u;
}
__global__ void k_run_starts(const u32* __restrict__ chg, const u32* __restrict__ rid, u32 nv, u32* __restrict__ rstart) {
    const u64 k = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (k < nv && chg[k]) rstart[rid[k] - 1] = (u32)k;
}
// next pushed candidate after k (nv = none)
__global__ void k_stream_next(const pos_t* __restrict__ bV, const pos_t* __restrict__ eV, const u32* __restrict__ rid,
                              const u32* __restrict__ rstart, u32 nruns, u32 nv, u32* __restrict__ nxt) {
    const u64 k = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (k > nv) return;
    if (k == nv) { nxt[nv] = nv; return; }
    const u32 nd = rid[k] < nruns ? rstart[rid[k]] : nv;  // first later candidate on another diagonal
    u32 lo = (u32)k + 1, hi = nd;                          // first one starting at or after end(k)
    const pos_t e = eV[k];
    while (lo < hi) {
        const u32 mid = (lo + hi) >> 1;
        if (bV[mid] < e) lo = mid + 1; else hi = mid;
    }
    nxt[k] = lo;
}
__global__ void k_jmp(const u32* __restrict__ prev, u32 m, u32* __restrict__ out) {
    const u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < m) out[i] = prev[prev[i]];
}
__global__ void k_expand2(const u32* __restrict__ C, u32 cnt, const u32* __restrict__ J, u32* __restrict__ out) {
    const u64 m = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (m >= cnt) return;
    const u32 c = C[m];
    out[2 * m] = c;
    out[2 * m + 1] = J[c];
}
__global__ void k_mark_nodes(const u32* __restrict__ C, u32 cnt, u32 term, u32* __restrict__ mark) {
    const u64 m = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (m < cnt && C[m] < term) mark[C[m]] = 1;
}
// pushed phrase of stream candidate k -> sequence slot (forward coordinates)
__global__ void k_stream_emit(const pos_t* __restrict__ rec, const u32* __restrict__ V, const u32* __restrict__ mark,
                              u32 nv, int side, int lnf, pos_t N, u64 slot_base, pos_t* __restrict__ slots,
                              u32* __restrict__ sflag) {
    const u64 k = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= nv || !mark[k]) return;
    const u32 i = V[k];
    const pos_t* r = rec + (2 * (u64)i + side) * AREC;
    pos_t b = r[3], e = r[2], sr = r[4];
    if (lnf) {  // reversed coordinates -> forward (lpf_lnf.cpp: n - end, n - beg, n - (src + len))
        const pos_t len = e - b;
        const pos_t fb = N - e, fe = N - b, fs = N - (sr + len);
        b = fb;
        e = fe;
        sr = fs;
    }
    const u64 slot = slot_base + 2 * (u64)i + side;
    slots[3 * slot] = b;
    slots[3 * slot + 1] = e;
    slots[3 * slot + 2] = sr;
    sflag[slot] = 1;
}
// sort keys of the merged phrases: (beg asc, end desc), stable -> push order.  32-bit
// positions pack both into one key; 64-bit ones are sorted twice (~end, then beg: LSD order)
__global__ void k_slot_compact(const pos_t* __restrict__ slots, const u32* __restrict__ sflag, const u32* __restrict__ off,
                               u64 nslots, pos_t* __restrict__ P, u64* __restrict__ keys, u32* __restrict__ vals) {
    const u64 t = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= nslots || !sflag[t]) return;
    const u32 o = off[t];
    const pos_t b = slots[3 * t], e = slots[3 * t + 1];
    P[3 * (u64)o] = b;
    P[3 * (u64)o + 1] = e;
    P[3 * (u64)o + 2] = slots[3 * t + 2];
    if constexpr (sizeof(pos_t) == 4) keys[o] = ((u64)b << 32) | (u64)(0xFFFFFFFFu - e);
    else keys[o] = ~(u64)e;
    vals[o] = o;
}
__global__ void k_beg_keys(const pos_t* __restrict__ P, const u32* __restrict__ idx, u32 p, u64* __restrict__ keys) {
    const u64 t = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (t < p) keys[t] = P[3 * (u64)idx[t]];
}
__global__ void k_gather3(const pos_t* __restrict__ P, const u32* __restrict__ idx, u32 p, pos_t* __restrict__ Q) {
    const u64 t = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= p) return;
    const u32 j = idx[t];
    Q[3 * t] = P[3 * (u64)j];
    Q[3 * t + 1] = P[3 * (u64)j + 1];
    Q[3 * t + 2] = P[3 * (u64)j + 2];
}
// selection: pm[k] = (end, first index) max over [0, k]; the larger end wins, ties the smaller index
struct end_key {
    pos_t e;
    u32 t;
};
struct end_max {
    __device__ __forceinline__ end_key operator()(const end_key& a, const end_key& b) const {
        return (a.e > b.e || (a.e == b.e && a.t < b.t)) ? a : b;
    }
};
__global__ void k_end_keys(const pos_t* __restrict__ Q, u32 p, end_key* __restrict__ ek) {
    const u64 t = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (t < p) ek[t] = end_key{Q[3 * t + 1], (u32)t};
}
__device__ __forceinline__ u32 first_beg_after(const pos_t* Q, u32 p, pos_t e) {  // first t with beg > e
    u32 lo = 0, hi = p;
    while (lo < hi) {
        const u32 mid = (lo + hi) >> 1;
        if (Q[3 * mid] <= e) lo = mid + 1; else hi = mid;
    }
    return lo;
}
__global__ void k_select_next(const pos_t* __restrict__ Q, const end_key* __restrict__ pm, u32 p, u32* __restrict__ nxt,
                              u32* __restrict__ X) {
    const u64 c = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (c > p) return;
    if (c == p) { nxt[p] = p; return; }
    const pos_t ec = Q[3 * c + 1];
    const u32 x = first_beg_after(Q, p, ec);
    X[c] = x;
    const end_key best = pm[x - 1];  // x > c >= 0 since beg_c < end_c
    nxt[c] = best.e > ec ? best.t : x;
}
// i_T of the selection loop along the chain: j_{t+1} = max(j_t, X(c_t) - t - 1)
__global__ void k_window_terms(const u32* __restrict__ chain, const u32* __restrict__ X, u32 len, int64_t* __restrict__ y) {
    const u64 t = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (t < len) y[t] = (int64_t)X[chain[t]] - (int64_t)t - 1;
}
__global__ void k_first_ge_end0(const pos_t* __restrict__ Q, u32 p, u32* __restrict__ out) {
    const u64 t = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    block_min(out, t >= 1 && t < p && Q[3 * t + 1] >= Q[1] ? (u32)t : 0xFFFFFFFFu);
}
// trimmed output phrases along the selection chain
__global__ void k_select_emit(const pos_t* __restrict__ Q, const u32* __restrict__ chain, u32 len,
                              pos_t* __restrict__ outP, u32* __restrict__ keep) {
    const u64 t = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= len) return;
    const u32 c = chain[t];
    const pos_t b = Q[3 * (u64)c];
    pos_t e = Q[3 * (u64)c + 1];
    if (t + 1 < len) e = min(e, Q[3 * (u64)chain[t + 1]]);
    outP[3 * t] = b;
    outP[3 * t + 1] = e;
    outP[3 * t + 2] = Q[3 * (u64)c + 2];
    keep[t] = (t + 1 == len || e > b) ? 1u : 0u;
}
__global__ void k_compact_keep(const pos_t* __restrict__ P, const u32* __restrict__ keep, const u32* __restrict__ off,
                               u32 len, pos_t* __restrict__ out) {
    const u64 t = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= len || !keep[t]) return;
    const u32 o = off[t];
    out[3 * (u64)o] = P[3 * t];
    out[3 * (u64)o + 1] = P[3 * t + 1];
    out[3 * (u64)o + 2] = P[3 * t + 2];
}

__global__ void k_marked_positions(const u32* __restrict__ marks, const u32* __restrict__ off, u32 p,
                                   u32* __restrict__ out) {
    const u64 t = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (t < p && marks[t]) out[off[t]] = (u32)t;
}
__global__ void k_set1(u32* p, u32 v) { *p = v; }

// exclusive scan (off[m] = total)
static u32 xscan(u32* cnt, u32* off, u64 m, dbuf<u8>& tmp, hipStream_t st) {
    excl_sum_total(cnt, off, m, tmp, st);
    return rd1(off + m, st);
}

// nodes on the path from 0 through nxt (m nodes, terminal m-1): marks[k] = 1
void engine::path_marks(u32 m, u32* nxt0, u32* marks) {
    u32 lv = 0;
    while ((1ull << lv) < m) lv++;
    u32* J[MAX_LV + 1];
    J[0] = nxt0;
    for (u32 t = 1; t <= lv; t++) {
        J[t] = jump[t].get(m);
        k_jmp<<<cdiv(m, 256), 256, 0, st>>>(J[t - 1], m, J[t]);
    }
    u32* C = u32a.get(2ull << lv);
    u32* C2 = u32b.get(2ull << lv);
    LZ_HIP(hipMemsetAsync(C, 0, 4, st));
    u32 cnt = 1;
    for (int t = (int)lv - 1; t >= 0; t--) {
        k_expand2<<<cdiv(cnt, 256), 256, 0, st>>>(C, cnt, J[t], C2);
        std::swap(C, C2);
        cnt *= 2;
    }
    LZ_HIP(hipMemsetAsync(marks, 0, (size_t)m * 4, st));
    k_mark_nodes<<<cdiv(cnt, 256), 256, 0, st>>>(C, cnt, m - 1, marks);
}

// the pushed phrases of one sync-index pass (LNF on the reversed text: lnf = 1)
void engine::all_phrases(const u8* T, int lnf, int opt, u64 slot_base, pos_t* slots, u32* sflag) {
    if (s == 0) return;
    const unsigned g = cdiv(s, 256);
    sa_levels M{};
    M.L[0] = SA.p;
    M.nlev = 1;
    for (u32 lv = 1; (1ull << lv) <= s; lv++) {
        const u32 cnt = s - (1u << lv) + 1;
        u32* out = sa_min[lv].get(cnt);
        k_sa_lvl<<<cdiv(cnt, 256), 256, 0, st>>>(M.L[lv - 1], cnt, 1u << (lv - 1), lnf, out);
        M.L[lv] = out;
        M.nlev = lv + 1;
    }
    k_pnv<<<g, 256, 0, st>>>(SA.p, s, M, lnf, PSV.get(s), NSV.get(s));
    pos_t* rec = cand.get((u64)s * 2 * AREC);
    k_all_candidates<<<g, 256, 0, st>>>(view(T), SA.p, PSV.p, NSV.p, lnf, opt, rec);
    for (int side = 0; side < 2; side++) {
        u32* f = u32c.get(s + 1);
        u32* off = u32d.get(s + 1);
        k_side_flags<<<g, 256, 0, st>>>(rec, s, side, f);
        const u32 nv = xscan(f, off, s, scan_tmp, st);
        if (!nv) continue;
        u32* V = l_V.get(nv + 1);
        pos_t* bV = l_b.get(nv + 1);
        pos_t* dV = l_d.get(nv + 1);
        pos_t* eV = l_e.get(nv + 1);
        k_side_compact<<<g, 256, 0, st>>>(rec, S.p, s, side, off, V, bV, dV, eV);
        u32* chg = u32c.get(nv + 1);
        u32* rid = u32d.get(nv + 1);
        k_diag_change<<<cdiv(nv, 256), 256, 0, st>>>(dV, nv, chg);
        {
            size_t tb = 0;
            LZ_HIP(hipcub::DeviceScan::InclusiveSum(nullptr, tb, chg, rid, (int)nv, st));
            u8* t = scan_tmp.get(tb);
            LZ_HIP(hipcub::DeviceScan::InclusiveSum(t, tb, chg, rid, (int)nv, st));
        }
        const u32 nruns = rd1(rid + nv - 1, st);
        u32* rstart = l_r.get(nruns + 1);
        k_run_starts<<<cdiv(nv, 256), 256, 0, st>>>(chg, rid, nv, rstart);
        u32* nxt = jump[0].get(nv + 1);
        k_stream_next<<<cdiv(nv + 1, 256), 256, 0, st>>>(bV, eV, rid, rstart, nruns, nv, nxt);
        u32* marks = u32e.get(nv + 1);
        path_marks(nv + 1, nxt, marks);
        k_stream_emit<<<cdiv(nv, 256), 256, 0, st>>>(rec, V, marks, nv, side, lnf, (pos_t)n, slot_base, slots, sflag);
        LZ_HIP(hipGetLastError());
    }
}

// phr_mode lpf_lnf_opt (opt = 1) / lpf_lnf_naive (opt = 0): phrases in lpf + num_phr
void engine::build_lpf_lnf(int opt) {
    const u64 N = n;
    if (!d_text_rev) {
        LZ_HIP(hipMalloc(&d_text_rev, max_n + TEXT_PAD));
        LZ_HIP(hipMemsetAsync(d_text_rev, 0, max_n + TEXT_PAD, st));
    }
    k_reverse<<<capped_grid(N, 256), 256, 0, st>>>(d_text, N, d_text_rev);
    // LNF phrases of the reversed text (lz77_sss.hpp:385-393)
    build_sss(d_text_rev);
    build_sa_s(d_text_rev);
    build_lcp_rmq(d_text_rev);
    timer.mark("lnf_structures");
    const u64 s_rev = s;
    u32* sf_l = l_sflag_lnf.get(2 * s_rev + 1);
    pos_t* sl_l = l_slots_lnf.get(3 * (2 * s_rev + 1));
    LZ_HIP(hipMemsetAsync(sf_l, 0, (2 * s_rev + 1) * 4, st));
    all_phrases(d_text_rev, 1, opt, 0, sl_l, sf_l);
    timer.mark("lnf_phrases");
    // LPF phrases of the text
    build_sss(d_text);
    build_sa_s(d_text);
    build_lcp_rmq(d_text);
    timer.mark("lpf_structures");
    const u64 nsl = 2 * s_rev + 2 * (u64)s;
    u32* sflag = l_sflag.get(nsl + 1);
    pos_t* slots = l_slots.get(3 * (nsl + 1));
    LZ_HIP(hipMemsetAsync(sflag, 0, (nsl + 1) * 4, st));
    if (s_rev) {
        LZ_HIP(hipMemcpyAsync(sflag, sf_l, 2 * s_rev * 4, hipMemcpyDeviceToDevice, st));
        LZ_HIP(hipMemcpyAsync(slots, sl_l, 3 * 2 * s_rev * sizeof(pos_t), hipMemcpyDeviceToDevice, st));
    }
    all_phrases(d_text, 0, opt, 2 * s_rev, slots, sflag);
    timer.mark("lpf_phrases");
    // merge in push order, stable sort by (beg asc, end desc)
    u32* off = l_off.get(nsl + 1);
    const u32 p = xscan(sflag, off, nsl, scan_tmp, st);
    num_phr = 0;
    if (p == 0) {
        lpf.get(3);
        return;
    }
    pos_t* P = l_P.get(3 * (u64)p);
    u64* keys = u64a.get(p);
    u64* keys2 = u64b.get(p);
    u32* vals = l_V.get(p);
    u32* vals2 = l_V2.get(p);
    k_slot_compact<<<cdiv(nsl, 256), 256, 0, st>>>(slots, sflag, off, nsl, P, keys, vals);
    {
        size_t tb = 0;
        LZ_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, keys, keys2, vals, vals2, (int)p, 0, 64, st));
        u8* t = scan_tmp.get(tb);
        LZ_HIP(hipcub::DeviceRadixSort::SortPairs(t, tb, keys, keys2, vals, vals2, (int)p, 0, 64, st));
        if constexpr (sizeof(pos_t) > 4) {  // second (stable) pass on beg
            k_beg_keys<<<cdiv(p, 256), 256, 0, st>>>(P, vals2, p, keys);
            LZ_HIP(hipcub::DeviceRadixSort::SortPairs(t, tb, keys, keys2, vals2, vals, (int)p, 0, 64, st));
            std::swap(vals, vals2);
        }
    }
    pos_t* Q = l_Q.get(3 * (u64)p);
    k_gather3<<<cdiv(p, 256), 256, 0, st>>>(P, vals2, p, Q);
    // selection (approximate/common.cpp:31-96)
    end_key* ek = (end_key*)u64a.get(2 * (u64)p);
    end_key* pm = (end_key*)u64b.get(2 * (u64)p);
    k_end_keys<<<cdiv(p, 256), 256, 0, st>>>(Q, p, ek);
    {
        size_t tb = 0;
        LZ_HIP(hipcub::DeviceScan::InclusiveScan(nullptr, tb, ek, pm, end_max{}, (int)p, st));
        u8* t = scan_tmp.get(tb);
        LZ_HIP(hipcub::DeviceScan::InclusiveScan(t, tb, ek, pm, end_max{}, (int)p, st));
    }
    u32* nxt = jump[0].get(p + 1);
    u32* X = l_X.get(p + 1);
    k_select_next<<<cdiv(p + 1, 256), 256, 0, st>>>(Q, pm, p, nxt, X);
    u32* marks = u32e.get(p + 1);
    path_marks(p + 1, nxt, marks);
    // chain in order = marked phrases by index (the path is increasing)
    u32* coff = l_coff.get(p + 1);
    const u32 len = xscan(marks, coff, p, scan_tmp, st);
    u32* chain = l_r.get(len + 2);
    k_marked_positions<<<cdiv(p, 256), 256, 0, st>>>(marks, coff, p, chain);
    // the loop's last-phrase quirk: window start of the final step
    u32 len2 = len;
    {
        u32* d_i0 = counters.get(16);
        k_set1<<<1, 1, 0, st>>>(d_i0, p);
        k_first_ge_end0<<<cdiv(p, 256), 256, 0, st>>>(Q, p, d_i0);
        const u32 i0 = rd1(d_i0, st);
        int64_t iT = i0;
        if (len >= 2 && i0 < p) {
            int64_t* y = (int64_t*)tmp_bytes.get((u64)len * 8);
            int64_t* ym = (int64_t*)l_tmp64.get(len);
            k_window_terms<<<cdiv(len - 1, 256), 256, 0, st>>>(chain, X, len - 1, y);
            size_t tb = 0;
            LZ_HIP(hipcub::DeviceReduce::Max(nullptr, tb, y, ym, (int)(len - 1), st));
            u8* t = scan_tmp.get(tb);
            LZ_HIP(hipcub::DeviceReduce::Max(t, tb, y, ym, (int)(len - 1), st));
            const int64_t jm = rd1(ym, st);
            iT = std::max<int64_t>((int64_t)i0, jm) + (int64_t)(len - 1);
        }
        const u32 cT = rd1(chain + len - 1, st);
        if (i0 < p && iT == (int64_t)p - 1 && cT != p - 1) {
            k_set1<<<1, 1, 0, st>>>(chain + len, p - 1);
            len2 = len + 1;
        }
    }
    pos_t* outP = l_P.get(3 * (u64)len2);
    u32* keep = u32c.get(len2 + 1);
    k_select_emit<<<cdiv(len2, 256), 256, 0, st>>>(Q, chain, len2, outP, keep);
    u32* koff = u32d.get(len2 + 1);
    num_phr = xscan(keep, koff, len2, scan_tmp, st);
    pos_t* dst = lpf.get((u64)(num_phr + 1) * 3);
    k_compact_keep<<<cdiv(len2, 256), 256, 0, st>>>(outP, keep, koff, len2, dst);
    LZ_HIP(hipGetLastError());
    timer.mark("phrase_selection");
}

}  // namespace LZ_NS
