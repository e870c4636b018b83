// lpf.hip -- LPF candidate phrases at sync positions (build_LPF_opt,
// include/lz77_sss/algorithms/approximate/lpf_lnf/lpf_opt.cpp:33-157, p = 1)
// and the phrase statistics (get_phrase_info, approximate/common.cpp:98-157).
//
//  1. PSV/NSV over SA_S (nxv_pxv.cpp:33-92) by descending a min sparse table
//     over SA_S (the reference uses a sequential stack).
//  2. Per sync index i, both candidates (source, end = S[i] + LCE_R, and the
//     left extension LCE_L up to the largest cap the sequential loop could
//     ever apply: S[i]-S[i-1]).
//  3. The loop's skip chain (lpf_opt.cpp:61-63) is a linked list: the next
//     processed index after i depends only on E_i = max candidate end, so the
//     processed set is the path from index 0, found by pointer doubling; the
//     running max_end is an exclusive max-scan of E over that path.
//  4. Phrases are then formed independently per processed index and compacted
//     in text order.
#include "../include/engine.h"
#include "../include/prim.h"
#include "../include/lce_dev.h"

#include <hipcub/hipcub.hpp>

namespace LZ_NS {

__global__ void k_sa_min_level(const u32* __restrict__ prev, u32 cnt, u32 half, u32* __restrict__ out) {
    const u64 k = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (k < cnt) out[k] = min(prev[k], prev[k + half]);
}
__global__ void k_sa_min_level2(const u32* __restrict__ prev, u32 cnt1, u32 half, u32* __restrict__ out1, u32 cnt2,
                                u32* __restrict__ out2) {
    const u64 k = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= cnt1) return;
    const u32 a = min(prev[k], prev[k + half]);
    out1[k] = a;
    if (k < cnt2) out2[k] = min(a, min(prev[k + 2 * half], prev[k + 3 * half]));
}

struct sa_min_levels {
    u32 nlev;
    const u32* L[MAX_LV];
};

// PSV[r] = max r' < r with SA[r'] < SA[r] (or s); NSV[r] = min r' > r with SA[r'] < SA[r] (or s)
__global__ void k_psv_nsv(const u32* __restrict__ SA, u32 s, sa_min_levels M, u32* __restrict__ PSV,
                          u32* __restrict__ NSV) {
    const u64 r = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= s) return;
    const u32 v = SA[r];
    u64 pos = r;
    for (int lv = (int)M.nlev - 1; lv >= 0; lv--) {
        const u64 w = 1ull << lv;
        if (pos >= w && M.L[lv][pos - w] > v) pos -= w;
    }
    PSV[r] = pos == 0 ? s : (u32)(pos - 1);
    pos = r + 1;
    for (int lv = (int)M.nlev - 1; lv >= 0; lv--) {
        const u64 w = 1ull << lv;
        if (pos + w <= s && M.L[lv][pos] > v) pos += w;
    }
    NSV[r] = pos >= s ? s : (u32)pos;
}

// candidate record per sync index: [srcP, endP, lP, srcN, endN, lN, hasP|hasN<<1, E]
constexpr int CREC = 8;

// two lanes per sync index (adjacent: side 0 = PSV, side 1 = NSV), each with its own LCE pair,
// combined by a shuffle: the LCEs are dependent load chains, and one lane doing both sides
// left 54 K indices (rr) on 848 waves
__global__ void k_lpf_candidates(lce_view L, const u32* __restrict__ SA, const u32* __restrict__ PSV,
                                 const u32* __restrict__ NSV, pos_t* __restrict__ cand) {
    const u64 t = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    const u64 i = t >> 1;
    const int side = (int)(t & 1);
    const u32 s = L.s;
    pos_t src = 0, end = 0, l = 0;
    int has = 0;
    pos_t Si = 0;
    if (i < s) {
        const pos_t* S = L.S;
        const u32 r = L.ISA[i];
        Si = S[i];
        const pos_t capmax = i >= 2 ? Si - S[i - 1] : Si;
        const u32 nb = side == 0 ? PSV[r] : NSV[r];
        if (nb != s) {
            src = S[SA[nb]];
            end = Si + (pos_t)dev_lce(L, src, Si);
            if (src != 0 && Si != 0) l = dev_lce_left(L.T, L.R, src - 1, Si - 1, capmax);
            has = 1;
        }
    }
    const pos_t o_src = __shfl_xor(src, 1), o_end = __shfl_xor(end, 1), o_l = __shfl_xor(l, 1);
    const int o_has = __shfl_xor(has, 1);
    if (i >= s || side) return;
    pos_t rec[CREC] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (has) {
        rec[0] = src;
        rec[1] = end;
        rec[2] = l;
    }
    if (o_has) {
        rec[3] = o_src;
        rec[4] = o_end;
        rec[5] = o_l;
    }
    rec[6] = (pos_t)(has | (o_has << 1));
    rec[7] = max(has ? end : (pos_t)0, o_has ? o_end : (pos_t)0);
#pragma unroll
    for (int x = 0; x < CREC; x++) cand[i * CREC + x] = rec[x];
}

// next processed index after i (lpf_opt.cpp:61-63): max(i+1, last k: S[k] <= E_i)
__global__ void k_next(const pos_t* __restrict__ S, u32 s, const pos_t* __restrict__ cand, u32* __restrict__ nxt) {
    const u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (i > s) return;
    if (i == s) { nxt[s] = s; return; }
    const pos_t E = cand[i * CREC + 7];
    u32 nx = (u32)i + 1;
    if (i + 1 < s && S[i + 1] <= E) {
        u32 lo = (u32)i + 1, hi = s;  // last k with S[k] <= E: first k with S[k] > E, minus 1
        while (lo < hi) {
            u32 mid = (lo + hi) >> 1;
            if (S[mid] <= E) lo = mid + 1; else hi = mid;
        }
        nx = lo - 1;
        if (nx < i + 1) nx = (u32)i + 1;
    }
    nxt[i] = nx;
}
__global__ void k_jump(const u32* __restrict__ prev, u32 m, u32* __restrict__ out) {
    const u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < m) out[i] = prev[prev[i]];
}
// two doubling levels per launch: out1 = prev o prev, out2 = out1 o out1
__global__ void k_jump2(const u32* __restrict__ prev, u32 m, u32* __restrict__ out1, u32* __restrict__ out2) {
    const u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    const u32 b = prev[prev[i]];
    out1[i] = b;
    out2[i] = prev[prev[b]];
}
// top-down path expansion: out[2m] = C[m], out[2m+1] = J[C[m]]
__global__ void k_expand(const u32* __restrict__ C, u32 cnt, const u32* __restrict__ J, u32* __restrict__ out) {
    const u64 m = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (m >= cnt) return;
    const u32 c = C[m];
    out[2 * m] = c;
    out[2 * m + 1] = J[c];
}
// two expansion levels per launch (J = level t, J1 = level t - 1)
__global__ void k_expand2l(const u32* __restrict__ C, u32 cnt, const u32* __restrict__ J, const u32* __restrict__ J1,
                           u32* __restrict__ out) {
    const u64 m = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (m >= cnt) return;
    const u32 c = C[m], d = J[c];
    out[4 * m] = c;
    out[4 * m + 1] = J1[c];
    out[4 * m + 2] = d;
    out[4 * m + 3] = J1[d];
}
__global__ void k_mark(const u32* __restrict__ C, u32 cnt, u32 s, u32* __restrict__ mark) {
    const u64 m = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (m < cnt && C[m] < s) mark[C[m]] = 1;
}
__global__ void k_masked_E(const pos_t* __restrict__ cand, const u32* __restrict__ mark, u32 s, pos_t* __restrict__ Em) {
    const u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < s) Em[i] = mark[i] ? cand[i * CREC + 7] : (pos_t)0;
}

// phrase of a processed index given lst_end (lpf_opt.cpp:65-144)
__global__ void k_phrase(const pos_t* __restrict__ S, u32 s, const pos_t* __restrict__ cand, const u32* __restrict__ mark,
                         const pos_t* __restrict__ lst, pos_t* __restrict__ ph, u32* __restrict__ push) {
    const u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= s) return;
    u32 pu = 0;
    pos_t pb = 0, pe = 0, ps = 0;
    if (mark[i]) {
        const pos_t* c = cand + i * CREC;
        const pos_t lst_end = lst[i];
        const pos_t Si = S[i];
        const u32 has = (u32)c[6];
        for (int side = 0; side < 2; side++) {
            if (!(has >> side & 1)) continue;
            pos_t src = c[side * 3 + 0];
            const pos_t end = c[side * 3 + 1];
            if (end > lst_end) {
                pos_t beg = Si;
                if (Si > lst_end && src != 0 && Si != 0) {
                    const pos_t l = min(c[side * 3 + 2], (pos_t)(Si - lst_end));
                    beg -= l;
                    src -= l;
                }
                if (beg < lst_end) {
                    const pos_t exc = lst_end - beg;
                    beg += exc;
                    src += exc;
                }
                if (side == 0) {
                    if (end - beg > 1) { pb = beg; pe = end; ps = src; }
                } else {
                    if (end - beg > pe - pb) { pb = beg; pe = end; ps = src; }
                }
            }
            if (side == 1 && pe - pb > 1) pu = 1;  // pushed only in the NSV branch (lpf_opt.cpp:138-140)
        }
    }
    ph[i * 3 + 0] = pb;
    ph[i * 3 + 1] = pe;
    ph[i * 3 + 2] = ps;
    push[i] = pu;
}
__global__ void k_compact3(const pos_t* __restrict__ ph, const u32* __restrict__ push, const u32* __restrict__ off,
                           u32 s, pos_t* __restrict__ out) {
    const u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= s || !push[i]) return;
    const u32 o = off[i];
    out[o * 3 + 0] = ph[i * 3 + 0];
    out[o * 3 + 1] = ph[i * 3 + 1];
    out[o * 3 + 2] = ph[i * 3 + 2];
}

// after k_compact3: the phrase count m (from the last push offset), the sentinel {n, n+1, 0}
// at P[m], and the greedy's phrase statistics (total phrase length, gaps: approximate/common.cpp
// get_phrase_info as k_phrase_info) -- so one host read gives all three
__global__ void k_phrase_finish(pos_t* __restrict__ P, const u32* __restrict__ push, const u32* __restrict__ off, u32 s,
                                pos_t n, u64* __restrict__ acc) {
    const u32 m = off[s - 1] + push[s - 1];
    const u64 k = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    u64 len = 0, gaps = 0;
    if (k < m) {
        const pos_t b = P[3 * k], e = P[3 * k + 1];
        len = e - b;
        if (k == 0 ? b > 0 : b > P[3 * (k - 1) + 1]) gaps++;
        if (k == m - 1 && e < n) gaps++;
    }
    if (k == 0) {
        acc[2] = m;
        P[3 * (u64)m] = n;
        P[3 * (u64)m + 1] = n + 1;
        P[3 * (u64)m + 2] = 0;
    }
    block_add64(&acc[0], len);
    block_add64(&acc[1], gaps);
}

struct max_op {
    __device__ pos_t operator()(const pos_t& a, const pos_t& b) const { return a > b ? a : b; }
};

// ---------------------------------------------------------------------------
// build_LPF_naive (lpf_lnf/lpf_naive.cpp:33-110, p = 1): the longer PSV/NSV
// candidate (strictly longer replaces) at every sync index the previous pushed
// phrase does not cover; next(i) = first j > i with S[j] >= S[i] + len_i
// (lpf_naive.cpp:104-108), so the processed indices are again a path from 0.
// cand2[i] = (src, len)
__global__ void k_lpf_naive_cand(lce_view L, const u32* __restrict__ SA, const u32* __restrict__ PSV,
                                 const u32* __restrict__ NSV, pos_t* __restrict__ cand2) {
    const u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    const u32 s = L.s;
    if (i >= s) return;
    const u32 r = L.ISA[i];
    const pos_t Si = L.S[i];
    pos_t src = 0, len = 0;
#pragma unroll
    for (int side = 0; side < 2; side++) {
        const u32 nb = side == 0 ? PSV[r] : NSV[r];
        if (nb == s) continue;
        const pos_t sc = L.S[SA[nb]];
        const pos_t lc = (pos_t)dev_lce(L, sc, Si);
        if (lc > len) {
            src = sc;
            len = lc;
        }
    }
    cand2[2 * i] = src;
    cand2[2 * i + 1] = len;
}
__global__ void k_next_naive(const pos_t* __restrict__ S, u32 s, const pos_t* __restrict__ cand2, u32* __restrict__ nxt) {
    const u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (i > s) return;
    if (i == s) { nxt[s] = s; return; }
    const u64 E = (u64)S[i] + cand2[2 * i + 1];
    u32 lo = (u32)i + 1, hi = s;  // first k > i with S[k] >= E (s if none)
    while (lo < hi) {
        const u32 mid = (lo + hi) >> 1;
        if ((u64)S[mid] < E) lo = mid + 1; else hi = mid;
    }
    nxt[i] = lo;
}
__global__ void k_phrase_naive(const pos_t* __restrict__ S, u32 s, const pos_t* __restrict__ cand2,
                               const u32* __restrict__ mark, pos_t* __restrict__ ph, u32* __restrict__ push) {
    const u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= s) return;
    const pos_t len = cand2[2 * i + 1];
    const bool pu = mark[i] && len > 0;
    ph[i * 3 + 0] = S[i];
    ph[i * 3 + 1] = S[i] + len;
    ph[i * 3 + 2] = cand2[2 * i];
    push[i] = pu ? 1u : 0u;
}

// SA min levels 1.. (two per launch where both exist) into M.L; returns the level count
static u32 sa_min_levels_build(hipStream_t st, const u32* SA, u32 s, dbuf<u32>* sa_min, sa_min_levels& M) {
    M.L[0] = SA;
    u32 nl = 1;
    for (u32 lv = 1; (1ull << lv) <= s;) {
        const u32 cnt = s - (1u << lv) + 1;
        u32* out = sa_min[lv].get(cnt);
        const u32* prev = lv == 1 ? SA : sa_min[lv - 1].p;
        M.L[lv] = out;
        if ((2ull << lv) <= s) {
            const u32 cnt2 = s - (2u << lv) + 1;
            u32* out2 = sa_min[lv + 1].get(cnt2);
            k_sa_min_level2<<<cdiv(cnt, 256), 256, 0, st>>>(prev, cnt, 1u << (lv - 1), out, cnt2, out2);
            M.L[lv + 1] = out2;
            nl = lv + 2;
            lv += 2;
        } else {
            k_sa_min_level<<<cdiv(cnt, 256), 256, 0, st>>>(prev, cnt, 1u << (lv - 1), out);
            nl = lv + 1;
            lv += 1;
        }
    }
    M.nlev = nl;
    return nl;
}
// jump levels 1 .. T_lv - 1 over jump[0] (m nodes; level T_lv is never read by the expansion)
static void jump_levels_build(hipStream_t st, u32 m, u32 T_lv, dbuf<u32>* jump) {
    for (u32 t = 1; t < T_lv;) {
        if (t + 1 < T_lv) {
            k_jump2<<<cdiv(m, 256), 256, 0, st>>>(jump[t - 1].p, m, jump[t].get(m), jump[t + 1].get(m));
            t += 2;
        } else {
            k_jump<<<cdiv(m, 256), 256, 0, st>>>(jump[t - 1].p, m, jump[t].get(m));
            t += 1;
        }
    }
}
// top-down expansion of the path from node 0 over jump[0 .. T_lv - 1]: C (2^T_lv entries) in order
static u32* path_expand(hipStream_t st, u32 T_lv, dbuf<u32>* jump, u32* C, u32* C2) {
    u64 cnt = 1;
    int t = (int)T_lv - 1;
    while (t >= 0) {
        if (t >= 1) {
            k_expand2l<<<cdiv(cnt, 256), 256, 0, st>>>(C, (u32)cnt, jump[t].p, jump[t - 1].p, C2);
            cnt *= 4;
            t -= 2;
        } else {
            k_expand<<<cdiv(cnt, 256), 256, 0, st>>>(C, (u32)cnt, jump[t].p, C2);
            cnt *= 2;
            t -= 1;
        }
        std::swap(C, C2);
    }
    return C;
}

// PSV/NSV over SA_S into the engine's PSV / NSV buffers
void engine::psv_nsv_s() {
    const unsigned g = cdiv(s, 256);
    sa_min_levels M{};
    sa_min_levels_build(st, SA.p, s, sa_min, M);
    k_psv_nsv<<<g, 256, 0, st>>>(SA.p, s, M, PSV.get(s), NSV.get(s));
}

// path of processed indices from 0 along nxt (pointer doubling + top-down expansion) -> mark[i] = 1
void engine::mark_path(u32* mark) {
    const u32 m = s + 1;
    u32 T_lv = 0;
    while ((1ull << T_lv) < m) T_lv++;
    jump_levels_build(st, m, T_lv, jump);
    u32* C = u32a.get(4ull << T_lv);
    u32* C2 = u32b.get(4ull << T_lv);
    LZ_HIP(hipMemsetAsync(C, 0, 4, st));
    C = path_expand(st, T_lv, jump, C, C2);
    const u32 cnt = 1u << T_lv;
    LZ_HIP(hipMemsetAsync(mark, 0, (size_t)s * 4, st));
    k_mark<<<cdiv(cnt, 256), 256, 0, st>>>(C, cnt, s, mark);
}

void engine::build_lpf_naive(const u8* T) {
    num_phr = 0;
    if (s == 0) return;
    const unsigned g = cdiv(s, 256);
    psv_nsv_s();
    pos_t* cd = cand.get((u64)s * 2);
    k_lpf_naive_cand<<<g, 256, 0, st>>>(view(T), SA.p, PSV.p, NSV.p, cd);
    k_next_naive<<<cdiv(s + 1, 256), 256, 0, st>>>(S.p, s, cd, jump[0].get(s + 1));
    u32* mark = u32c.get(s);
    mark_path(mark);
    pos_t* ph3 = p_ph3.get((u64)s * 3);
    u32* push = u32d.get(s);
    k_phrase_naive<<<g, 256, 0, st>>>(S.p, s, cd, mark, ph3, push);
    u32* off = mark;  // mark no longer needed
    scan_dev(push, off, s, s, 0u, 0u, op_sum{}, true, scan_tmp, st);
    {
        const auto [lo, lp] = rd2(off + s - 1, push + s - 1, st);
        num_phr = lo + lp;
    }
    pos_t* out = lpf.get((u64)(num_phr + 1) * 3);
    k_compact3<<<g, 256, 0, st>>>(ph3, push, off, s, out);
    LZ_HIP(hipGetLastError());
}

void engine::build_lpf_opt(const u8* T) {
    num_phr = 0;
    if (s == 0) return;
    const unsigned g = cdiv(s, 256);
    // 1. PSV/NSV
    {
        sa_min_levels M{};
        sa_min_levels_build(st, SA.p, s, sa_min, M);
        k_psv_nsv<<<g, 256, 0, st>>>(SA.p, s, M, PSV.get(s), NSV.get(s));
    }
    // (lean mode: each table goes as soon as it has been read, so the phase's peak is not the sum
    // of all of them: the sparse table over SA here, the doubling levels and the expansion
    // buffers after the expansion, PSV / NSV after the candidates)
    auto drop = [&](auto&... b) {
        if (!lean) return;
        LZ_HIP(hipStreamSynchronize(st));  // (the launches that read them have run)
        (b.release(), ...);
    };
    for (auto& b : sa_min) drop(b);
    // 2. candidates
    pos_t* cd = cand.get((u64)s * CREC);
    k_lpf_candidates<<<cdiv(2ull * s, 256), 256, 0, st>>>(view(T), SA.p, PSV.p, NSV.p, cd);
    // 3. skip chain: pointer doubling over next[], nodes 0..s (s = end)
    const u32 m = s + 1;
    u32 T_lv = 0;
    while ((1ull << T_lv) < m) T_lv++;
    k_next<<<cdiv(m, 256), 256, 0, st>>>(S.p, s, cd, jump[0].get(m));
    jump_levels_build(st, m, T_lv, jump);
    u32* C = u32a.get(4ull << T_lv);
    u32* C2 = u32b.get(4ull << T_lv);
    u32* mark = u32c.get(s);
    u64* acc = counters64.get(16) + 2;  // [2] total length, [3] gaps, [4] m (factorize_greedy's slots)
    fills({{C, 4, 0u}, {mark, (u64)s * 4, 0u}, {acc, 16, 0u}});  // (none is read before its use below)
    C = path_expand(st, T_lv, jump, C, C2);
    const u32 cnt = 1u << T_lv;
    k_mark<<<cdiv(cnt, 256), 256, 0, st>>>(C, cnt, s, mark);
    drop(PSV, NSV, u32a, u32b);
    for (auto& b : jump) drop(b);
    // running max_end before each processed index
    pos_t* Em = p_Em.get(s);
    k_masked_E<<<g, 256, 0, st>>>(cd, mark, s, Em);
    pos_t* lst = p_lst.get(s);
    scan_dev(Em, lst, s, s, (pos_t)0, (pos_t)0, op_max{}, true, scan_tmp, st);
    // 4. phrases + compaction
    pos_t* ph3 = p_ph3.get((u64)s * 3);
    u32* push = u32d.get(s);
    k_phrase<<<g, 256, 0, st>>>(S.p, s, cd, mark, lst, ph3, push);
    u32* off = mark;  // mark no longer needed after k_phrase
    scan_dev(push, off, s, s, 0u, 0u, op_sum{}, true, scan_tmp, st);
    // compaction for the bound s, then the count, sentinel and the greedy's phrase statistics in
    // one pass and one host read (the emitter reuses them: phr_info)
    pos_t* out = lpf.get((u64)(s + 1) * 3);
    k_compact3<<<g, 256, 0, st>>>(ph3, push, off, s, out);
    k_phrase_finish<<<cdiv((u64)s + 1, 256), 256, 0, st>>>(out, push, off, s, (pos_t)n, acc);
    LZ_HIP(hipGetLastError());
    u64 h3[3];
    hread rb(st);
    rb.add(h3, (const u64*)acc, 3);
    rb.sync();
    num_phr = (u32)h3[2];
    phr_info = {true, h3[0], h3[1]};
}

}  // namespace LZ_NS
