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

__global__ void k_dec_lens(const pos_t* __restrict__ F, u64 nf, u64* __restrict__ len) {
    const u64 f = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (f < nf) len[f] = F[2 * f + 1] ? F[2 * f + 1] : 1u;
}
__global__ void k_dec_heads(const u64* __restrict__ start, u64 nf, u64 n, u32* __restrict__ head) {
    const u64 f = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (f < nf && start[f] < n) head[start[f]] = (u32)f;
}
struct max_u32 {
    __device__ __forceinline__ u32 operator()(const u32& a, const u32& b) const { return a > b ? a : b; }
};
// ref[p]: p for literals, the source position for copies; err on a forward reference
__global__ void k_dec_refs(const pos_t* __restrict__ F, const u64* __restrict__ start, const u32* __restrict__ fid, u64 n,
                           pos_t* __restrict__ ref, u32* __restrict__ err) {
    const u64 p = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n) return;
    const u32 f = fid[p];
    const pos_t len = F[2 * (u64)f + 1];
    if (len == 0) { ref[p] = (pos_t)p; return; }
    const pos_t src = F[2 * (u64)f], st = (pos_t)start[f];
    if (src >= st) { atomicOr(err, 1u); ref[p] = (pos_t)p; return; }  // only on an invalid stream
    // a self-overlapping copy (distance d < len) is d-periodic: fold the offset
    // into the first period so the reference lands before the factor start
    const pos_t d = st - src;
    pos_t off = (pos_t)(p - st);
    if (off >= d) off %= d;
    ref[p] = src + off;
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
    const u64 p = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n) return;
    const u8 c = (u8)F[2 * (u64)fid[ref[p]]];
    if (out) out[p] = c;
    if (cmp && cmp[p] != c) atomicAdd(mism, 1u);  // only on a failed round trip
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
    k_dec_lens<<<cdiv(nf, 256), 256, 0, st>>>(F, nf, len);
    LZ_HIP(hipMemsetAsync(len + nf, 0, 8, st));
    excl_sum64(len, start, (u64)0, nf + 1, scan_tmp, st);
    if (rd1(start + nf, st) != n_out) throw error(LZ77SSS_EINVAL, "factor lengths do not sum to n");
    u32* head = dec_fid.get(n_out);
    u32* fid = dec_fid2.get(n_out);
    LZ_HIP(hipMemsetAsync(head, 0, n_out * 4, st));
    k_dec_heads<<<cdiv(nf, 256), 256, 0, st>>>(start, nf, n_out, head);
    incl_scan64(head, fid, n_out, max_u32{}, scan_tmp, st);
    pos_t* ref = dec_ref.get(n_out);
    pos_t* ref2 = dec_ref2.get(n_out);
    u32* flags = counters.get(16);
    LZ_HIP(hipMemsetAsync(flags, 0, 8, st));
    k_dec_refs<<<cdiv(n_out, 256), 256, 0, st>>>(F, start, fid, n_out, ref, flags);
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
    k_dec_bytes<<<cdiv(n_out, 256), 256, 0, st>>>(F, fid, ref, n_out, cmp, out, flags + 2);
    LZ_HIP(hipGetLastError());
    return cmp ? rd1(flags + 2, st) : 0;
}

}  // namespace LZ_NS
