// decode.hip -- LZ77 decode on the device (the host
// decode is lz77_sss<>::decode, algorithms/common.cpp:31-54).
//
// Position p of the output is covered by factor fid[p] (starts scattered, then
// a max-scan).  A literal position resolves to itself; a copied position points
// at its source src + (p - start) < p.  Pointer jumping on these references
// reaches a literal in ceil(log2(chain depth)) rounds; the byte is that
// literal's factor source.  Self-overlapping copies are folded into their first
// period, so every reference leaves its factor and the depth is counted in
// factors, not positions.
#include "../../include/lz77sss.h"
#include "../include/engine.h"
#include "../include/prim.h"

namespace LZ_NS {

// (the per-factor and per-position kernels loop over a capped grid: n and z pass 2^32 with
// pos_t = uint64_t, GRID_CAP in lz77sss_internal.h)
__global__ void k_dec_lens(const pos_t* __restrict__ F, u64 nf, u64* __restrict__ len) {
    for (u64 f = gtid(); f < nf; f += gstride()) len[f] = F[2 * f + 1] ? F[2 * f + 1] : 1u;
}
__global__ void k_dec_heads(const u64* __restrict__ start, u64 nf, u64 n, u32* __restrict__ head) {
    for (u64 f = gtid(); f < nf; f += gstride())
        if (start[f] < n) head[start[f]] = (u32)f;
}
struct max_u32 {
    __device__ __forceinline__ u32 operator()(const u32& a, const u32& b) const { return a > b ? a : b; }
};
// ref[p]: p for literals, the source position for copies; err on a forward reference
__global__ void k_dec_refs(const pos_t* __restrict__ F, const u64* __restrict__ start, const u32* __restrict__ fid, u64 n,
                           pos_t* __restrict__ ref, u32* __restrict__ err) {
    for (u64 p = gtid(); p < n; p += gstride()) {
        const u32 f = fid[p];
        const pos_t len = F[2 * (u64)f + 1];
        if (len == 0) { ref[p] = (pos_t)p; continue; }
        const pos_t src = F[2 * (u64)f], st = (pos_t)start[f];
        if (src >= st) { atomicOr(err, 1u); ref[p] = (pos_t)p; continue; }  // only on an invalid stream
        // a self-overlapping copy (distance d < len) is d-periodic: fold the offset
        // into the first period so the reference lands before the factor start
        const pos_t d = st - src;
        pos_t off = (pos_t)(p - st);
        if (off >= d) off %= d;
        ref[p] = src + off;
    }
}
// one pointer-jumping round.  Grid-stride over a fixed grid so that the change
// flag costs one atomic per block: millions of same-address atomics (even one
// per wave) serialize at ~10 ns each.
constexpr unsigned DEC_GRID = 4096;
__global__ void __launch_bounds__(256) k_dec_jump(const pos_t* __restrict__ ref, u64 n, pos_t* __restrict__ out,
                                                  u32* __restrict__ changed) {
    __shared__ u32 any;
    if (threadIdx.x == 0) any = 0;
    __syncthreads();
    bool ch = false;
    const u64 stride = (u64)gridDim.x * blockDim.x;
    u64 p = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    for (; p + 3 * stride < n; p += 4 * stride) {  // 4 independent gathers in flight per lane
        pos_t r[4], rr[4];
#pragma unroll
        for (int k = 0; k < 4; k++) r[k] = ref[p + k * stride];
#pragma unroll
        for (int k = 0; k < 4; k++) rr[k] = ref[r[k]];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            out[p + k * stride] = rr[k];
            ch |= rr[k] != r[k];
        }
    }
    for (; p < n; p += stride) {
        const pos_t r = ref[p];
        const pos_t rr = ref[r];
        out[p] = rr;
        ch |= rr != r;
    }
    if (ch) any = 1;
    __syncthreads();
    if (threadIdx.x == 0 && any) atomicOr(changed, 1u);
}
__global__ void k_dec_bytes(const pos_t* __restrict__ F, const u32* __restrict__ fid, const pos_t* __restrict__ ref, u64 n,
                            const u8* __restrict__ cmp, u8* __restrict__ out, u32* __restrict__ mism) {
    for (u64 p = gtid(); p < n; p += gstride()) {
        const u8 c = (u8)F[2 * (u64)fid[ref[p]]];
        if (out) out[p] = c;
        if (cmp && cmp[p] != c) atomicAdd(mism, 1u);  // only on a failed round trip
    }
}

// decodes nf factors (device array, 2 x u32 each) of a text of length n; writes
// the text to out (device, may be null) and, when cmp is given, counts the
// positions where it differs from cmp.  Returns the mismatch count, or throws
// on an invalid stream (lengths not summing to n, forward references).
u64 engine::decode_device(const pos_t* F, u64 nf, u64 n_out, u8* out, const u8* cmp) {
    if (n_out == 0) {
        if (nf) throw error(LZ77SSS_EINVAL, "factors for an empty text");
        return 0;
    }
    if (nf == 0 || nf > n_out) throw error(LZ77SSS_EINVAL, "factor count does not fit the text length");
    if (n_out > POS_MAX_N) throw error(LZ77SSS_EINVAL, "n too large for pos_t");
    if (nf >= (1ull << 32)) throw error(LZ77SSS_EINVAL, "too many factors for the device decode (factor ids are 32-bit)");
    // starts in 64 bits: lengths of an invalid stream may sum past 2^32 (the sum check must see it)
    u64* len = dec_len64.get(nf + 1);
    u64* start = dec_start64.get(nf + 1);
    k_dec_lens<<<capped_grid(nf, 256), 256, 0, st>>>(F, nf, len);
    LZ_HIP(hipMemsetAsync(len + nf, 0, 8, st));
    excl_sum64(len, start, (u64)0, nf + 1, scan_tmp, st);
    if (rd1(start + nf, st) != n_out) throw error(LZ77SSS_EINVAL, "factor lengths do not sum to n");
    u32* head = dec_fid.get(n_out);
    u32* fid = dec_fid2.get(n_out);
    LZ_HIP(hipMemsetAsync(head, 0, n_out * 4, st));
    k_dec_heads<<<capped_grid(nf, 256), 256, 0, st>>>(start, nf, n_out, head);
    incl_scan64(head, fid, n_out, max_u32{}, scan_tmp, st);
    pos_t* ref = dec_ref.get(n_out);
    pos_t* ref2 = dec_ref2.get(n_out);
    u32* flags = counters.get(16);
    LZ_HIP(hipMemsetAsync(flags, 0, 8, st));
    k_dec_refs<<<capped_grid(n_out, 256), 256, 0, st>>>(F, start, fid, n_out, ref, flags);
    if (rd1(flags, st)) throw error(LZ77SSS_EINVAL, "factor source not before its position");
    dec_rounds = 0;
    for (int round = 0; round < 40; round++) {
        dec_rounds++;
        LZ_HIP(hipMemsetAsync(flags + 1, 0, 4, st));
        k_dec_jump<<<std::min<u64>(cdiv(n_out, 256), DEC_GRID), 256, 0, st>>>(ref, n_out, ref2, flags + 1);
        std::swap(ref, ref2);
        if (!rd1(flags + 1, st)) break;
    }
    LZ_HIP(hipMemsetAsync(flags + 2, 0, 4, st));
    k_dec_bytes<<<capped_grid(n_out, 256), 256, 0, st>>>(F, fid, ref, n_out, cmp, out, flags + 2);
    LZ_HIP(hipGetLastError());
    return cmp ? rd1(flags + 2, st) : 0;
}

// ---------------------------------------------------------------------------
// Verification of a factor stream against the text it encodes, without decoding it:
// decode(F) == T holds iff the lengths sum to n and every position p of every factor
// (start st, source src) satisfies  literal: T[p] == (u8)src;  copy: src < st and
// T[p] == T[src + (p - st)]  (induction over p: the decoder's out[src + p - st] is
// out at an earlier position, which equals T there).  So the check reads the text
// twice (position and source) and needs only the factor starts (8 B per factor), not
// the 24 B per position of decode_device: a 50 GiB factorization is verified in HBM.
// One workgroup per VB-position block: the factors covering it are f0..f1 (binary
// searches of the starts); their in-block starts are marked in LDS and an inclusive
// max-scan gives every position its factor.
constexpr u32 VB_T = 256, VB_PER = 16, VB = VB_T * VB_PER;
__global__ __launch_bounds__(VB_T) void k_verify_blocks(const pos_t* __restrict__ F, const u64* __restrict__ start,
                                                         u64 nf, u64 n, const u8* __restrict__ T,
                                                         unsigned long long* __restrict__ bad) {  // [0] count, [1] first
    __shared__ u16 fl[VB];
    __shared__ u64 s_f0;
    __shared__ u32 s_wmax[VB_T / 64];
    const u64 nblk = (n + VB - 1) / VB;
    for (u64 blk = blockIdx.x; blk < nblk; blk += gridDim.x) {  // (block-uniform loop: barriers inside)
    const u64 b0 = blk * VB;
    const u64 b1 = min(n, b0 + VB);
    if (threadIdx.x == 0) {
        u64 lo = 0, hi = nf;  // last factor with start <= b0
        while (hi - lo > 1) {
            const u64 mid = (lo + hi) >> 1;
            if (start[mid] <= b0) lo = mid; else hi = mid;
        }
        s_f0 = lo;
    }
    for (u32 k = threadIdx.x; k < VB; k += VB_T) fl[k] = 0;
    __syncthreads();
    const u64 f0 = s_f0;
    // factors starting inside the block: at most VB of them, in order from f0 + 1
    for (u64 f = f0 + 1 + threadIdx.x; f < nf && start[f] < b1; f += VB_T) fl[start[f] - b0] = (u16)(f - f0);
    __syncthreads();
    // inclusive max-scan of fl: VB_PER consecutive entries per thread, then a block scan
    const u32 base = threadIdx.x * VB_PER;
    u32 m = 0;
    for (u32 k = 0; k < VB_PER; k++) m = max(m, (u32)fl[base + k]);  // (fl[0] = 0: f0 covers b0)
    const u32 lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    u32 incl = m;
    for (u32 o = 1; o < 64; o <<= 1) {
        const u32 y = __shfl_up(incl, o, 64);
        if (lane >= o) incl = max(incl, y);
    }
    if (lane == 63) s_wmax[wv] = incl;
    __syncthreads();
    u32 carry = 0;
    for (u32 w = 0; w < wv; w++) carry = max(carry, s_wmax[w]);
    // exclusive prefix: the waves before this one, then the lanes before this one
    const u32 ex = (u32)__shfl_up(incl, 1, 64);
    u32 run = max(carry, lane ? ex : 0u);
    u32 cnt = 0;
    u64 first = ~0ull;
    for (u32 k = 0; k < VB_PER; k++) {
        const u64 p = b0 + base + k;
        const u32 c0 = cnt;
        run = max(run, (u32)fl[base + k]);
        if (p >= b1) break;
        const u64 f = f0 + run;
        const pos_t src = F[2 * f], len = F[2 * f + 1];
        const u8 c = T[p];
        if (len == 0) {
            cnt += (p != start[f] || c != (u8)src) ? 1u : 0u;
        } else {
            const u64 st = start[f];
            cnt += ((u64)src >= st || T[(u64)src + (p - st)] != c) ? 1u : 0u;
        }
        if (cnt != c0 && first == ~0ull) first = p;
    }
    for (int o = 32; o > 0; o >>= 1) {
        cnt += __shfl_down(cnt, o, 64);
        first = min(first, (u64)__shfl_down(first, o, 64));
    }
    if (lane == 0 && cnt) {
        atomicAdd(bad, (unsigned long long)cnt);
        atomicMin(bad + 1, (unsigned long long)first);
    }
    __syncthreads();  // fl / s_f0 / s_wmax are rewritten by the next block of the loop
    }
}

// LZ77SSS_DEBUG_VERIFY: every LPF phrase (beg, end, src) copies equal bytes and its source lies
// before it; [0] bad phrases, [1] the first bad phrase index
__global__ void k_verify_phrases(const pos_t* __restrict__ P, u64 m, const u8* __restrict__ T,
                                 unsigned long long* __restrict__ bad) {
    const u64 k = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    bool b = false;
    if (k < m) {
        const pos_t beg = P[3 * k], end = P[3 * k + 1], src = P[3 * k + 2];
        b = end <= beg || src >= beg || dev_naive_lce(T, src, beg, end - beg) != (u64)(end - beg) ||
            (k > 0 && beg < P[3 * (k - 1) + 1]);
    }
    if (b) {
        atomicAdd(bad, 1ull);
        atomicMin(bad + 1, (unsigned long long)k);
    }
}
// LZ77SSS_DEBUG_VERIFY: SA_S order and LCP against bounded direct comparisons (2^20 bytes);
// [0] bad LCP, [1] bad order, [2] first bad rank; the successor table against a binary search
__global__ void k_verify_sa_lcp(const u8* __restrict__ T, u64 n, const pos_t* __restrict__ S, const u32* __restrict__ SA,
                                const u32* __restrict__ LCP, u32 s, unsigned long long* __restrict__ bad) {
    const u64 r = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (r == 0 || r >= s) return;
    const u64 a = S[SA[r - 1]], b = S[SA[r]];
    const u64 lim = min<u64>(1ull << 20, n - max(a, b));
    const u64 l = dev_naive_lce(T, a, b, lim);
    const bool bl = l < lim && LCP[r] != (u32)l;
    const bool bo = l < lim && !(T[a + l] < T[b + l]);
    if (bl) atomicAdd(bad, 1ull);
    if (bo) atomicAdd(bad + 1, 1ull);
    if (bl || bo) atomicMin(bad + 2, (unsigned long long)r);
}
__global__ void k_verify_succ(const pos_t* __restrict__ S, u32 s, const u32* __restrict__ succ, u64 nb,
                              unsigned long long* __restrict__ bad) {
    const u64 bkt = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (bkt >= nb) return;
    const u32 k = succ[bkt];
    const u64 x = bkt << 9;
    const bool ok = k <= s && (k == s || (u64)S[k] >= x) && (k == 0 || (u64)S[k - 1] < x);
    if (!ok) {
        atomicAdd(bad + 3, 1ull);
        atomicMin(bad + 4, (unsigned long long)bkt);
    }
}
void engine::debug_verify_lce(const char* what) {
    unsigned long long* bad = (unsigned long long*)counters64.get(24) + 18;
    LZ_HIP(hipMemsetAsync(bad, 0, 48, st));
    LZ_HIP(hipMemsetAsync(bad + 2, 0xFF, 8, st));
    LZ_HIP(hipMemsetAsync(bad + 4, 0xFF, 8, st));
    if (s > 1) k_verify_sa_lcp<<<cdiv(s, 256), 256, 0, st>>>(d_text, n, S.p, SA.p, lcp_rmq[0].p, s, bad);
    const u64 nb = (n >> 9) + 2;
    k_verify_succ<<<cdiv(nb, 256), 256, 0, st>>>(S.p, s, succ_tab.p, nb, bad);
    u64 h[6];
    LZ_HIP(hipMemcpyAsync(h, bad, 48, hipMemcpyDeviceToHost, st));
    LZ_HIP(hipStreamSynchronize(st));
    std::fprintf(stderr, "[lz77sss-verify] %s: |S|=%u bad LCP=%llu bad order=%llu first rank=%lld; succ buckets=%llu bad=%llu first=%lld\n",
                 what, s, (unsigned long long)h[0], (unsigned long long)h[1], (long long)h[2], (unsigned long long)nb,
                 (unsigned long long)h[3], (long long)h[4]);
}
void engine::debug_verify_phrases(const char* what) {
    unsigned long long* bad = (unsigned long long*)counters64.get(24) + 18;
    LZ_HIP(hipMemsetAsync(bad, 0, 8, st));
    LZ_HIP(hipMemsetAsync(bad + 1, 0xFF, 8, st));
    if (num_phr) k_verify_phrases<<<cdiv(num_phr, 256), 256, 0, st>>>(lpf.p, num_phr, d_text, bad);
    const auto [cnt, first] = rd2((const u64*)bad, (const u64*)bad + 1, st);
    pos_t ph[3] = {0, 0, 0};
    if (cnt) LZ_HIP(hipMemcpy(ph, lpf.p + 3 * first, sizeof(ph), hipMemcpyDeviceToHost));
    std::fprintf(stderr, "[lz77sss-verify] %s: phrases=%u bad=%llu first=%llu (beg=%llu end=%llu src=%llu)\n", what,
                 num_phr, (unsigned long long)cnt, (unsigned long long)(cnt ? first : 0), (unsigned long long)ph[0],
                 (unsigned long long)ph[1], (unsigned long long)ph[2]);
}

u64 engine::verify_factors(const pos_t* F, u64 nf, u64 n_out, const u8* T, u64* first_bad) {
    if (first_bad) *first_bad = ~0ull;
    if (n_out == 0) return nf ? 1 : 0;
    if (nf == 0) return n_out;
    u64* len = dec_len64.get(nf + 1);
    u64* start = dec_start64.get(nf + 1);
    k_dec_lens<<<capped_grid(nf, 256), 256, 0, st>>>(F, nf, len);
    LZ_HIP(hipMemsetAsync(len + nf, 0, 8, st));
    excl_sum64(len, start, (u64)0, nf + 1, scan_tmp, st);
    if (rd1(start + nf, st) != n_out) throw error(LZ77SSS_EINVAL, "factor lengths do not sum to n");
    unsigned long long* bad = (unsigned long long*)counters64.get(24) + 16;  // (0..15: the greedy's slots)
    LZ_HIP(hipMemsetAsync(bad, 0, 8, st));
    LZ_HIP(hipMemsetAsync(bad + 1, 0xFF, 8, st));
    k_verify_blocks<<<capped_grid(n_out, VB), VB_T, 0, st>>>(F, start, nf, n_out, T, bad);
    LZ_HIP(hipGetLastError());
    const auto [cnt, first] = rd2((const u64*)bad, (const u64*)bad + 1, st);
    if (first_bad) *first_bad = first;
    return cnt;
}

}  // namespace LZ_NS
