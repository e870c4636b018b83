// ssszip.hip -- the "gapped" container of ssszip on the device (role of
// encode_gapped, cli/ssszip.cpp:119-177, over the skip_phrases stream of
// factorize_skip_gaps, approximate/factorize/skip_gaps.cpp:31-61; vbyte codes as
// include/lz77_sss/misc/vbyte.hpp:62-84).
//
// Layout: 1 byte is_64_bit (0: pos_t = uint32_t), 8 bytes n (little endian), then
// records.  A phrase of length >= 64, or any phrase not preceded by a gap, is
// written as vbyte(i - src) vbyte(len) (i = its text position); gap records and
// shorter phrases that follow a gap merge into one gap, written before the next
// written phrase (and at the end) as vbyte(gap length) vbyte(0) + the raw gap bytes.
//
// The encoder's state (inside a gap or not) is a 2-state automaton whose transition
// per record is "set", "clear" or "keep": it is the value of the last record that is
// not a keep (a max-scan of indices).  Text positions, gap starts and the output
// offsets are scans; every record then writes its bytes independently.
#include "../../include/lz77sss.h"
#include "../include/engine.h"
#include "../include/prim.h"

#include <hipcub/hipcub.hpp>

namespace lz {

constexpr u32 SSZ_MIN_LPF = 64;  // min_lpf_len, cli/ssszip.cpp:37

__device__ __forceinline__ u32 vb_len(u64 x) {
    u32 k = 1;
    while (x >>= 7) k++;
    return k;
}
__device__ __forceinline__ u64 vb_put(u8* o, u64 x) {
    u64 k = 0;
    do {
        u8 b = (u8)(x & 127u);
        x >>= 7;
        if (x) b |= 128u;
        o[k++] = b;
    } while (x);
    return k;
}

// adv = text advance of record r; dec = r + 1 for records that set or clear the gap state
__global__ void k_ssz_prep(const u32* __restrict__ F, u64 z, u64* __restrict__ adv, u32* __restrict__ dec) {
    const u64 r = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= z) return;
    const u32 src = F[2 * r], len = F[2 * r + 1];
    adv[r] = len ? len : src;
    dec[r] = (len == 0 || len >= SSZ_MIN_LPF) ? (u32)(r + 1) : 0u;
}
struct max_u32_op {
    __device__ __forceinline__ u32 operator()(const u32& a, const u32& b) const { return a > b ? a : b; }
};
struct max_u64_op {
    __device__ __forceinline__ u64 operator()(const u64& a, const u64& b) const { return a > b ? a : b; }
};
// merged[r]: record r belongs to a gap (state before r from the last set/clear record)
__global__ void k_ssz_merged(const u32* __restrict__ F, u64 z, const u32* __restrict__ lastdec, u8* __restrict__ merged,
                             u64* __restrict__ rs, const u64* __restrict__ pos) {
    const u64 r = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= z) return;
    const u32 len = F[2 * r + 1];
    const u32 j = r ? lastdec[r - 1] : 0u;
    const bool gap_before = j && F[2 * (u64)(j - 1) + 1] == 0;
    const bool m = len == 0 || (len < SSZ_MIN_LPF && gap_before);
    merged[r] = m;
    // a gap run starts at a merged record whose predecessor is not merged (a gap record)
    rs[r] = (m && !gap_before) ? pos[r] + 1 : 0;
}
// bytes of record r: written phrases (with the flush of the gap before them)
__global__ void k_ssz_size(const u32* __restrict__ F, u64 z, const u8* __restrict__ merged,
                           const u64* __restrict__ runst, const u64* __restrict__ pos, u64* __restrict__ sz) {
    const u64 r = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= z) return;
    if (merged[r]) { sz[r] = 0; return; }
    const u32 src = F[2 * r], len = F[2 * r + 1];
    u64 b = vb_len(pos[r] - src) + vb_len(len);
    if (r && merged[r - 1]) {
        const u64 glen = pos[r] - (runst[r - 1] - 1);
        b += vb_len(glen) + 1 + glen;
    }
    sz[r] = b;
}
// headers of every written record; the raw gap bytes by k_ssz_copy
__global__ void k_ssz_write(const u32* __restrict__ F, u64 z, const u8* __restrict__ merged,
                            const u64* __restrict__ runst, const u64* __restrict__ pos, const u64* __restrict__ off,
                            u8* __restrict__ out) {
    const u64 r = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= z || merged[r]) return;
    const u32 src = F[2 * r], len = F[2 * r + 1];
    u8* o = out + 9 + off[r];
    if (r && merged[r - 1]) {
        const u64 glen = pos[r] - (runst[r - 1] - 1);
        o += vb_put(o, glen);
        *o++ = 0;
        o += glen;  // raw bytes: k_ssz_copy
    }
    o += vb_put(o, pos[r] - src);
    vb_put(o, len);
}
// one workgroup per written record that flushes a gap: copy the gap's text bytes
__global__ void k_ssz_copy(const u8* __restrict__ T, u64 z, const u8* __restrict__ merged,
                           const u64* __restrict__ runst, const u64* __restrict__ pos, const u64* __restrict__ off,
                           u8* __restrict__ out) {
    const u64 r = blockIdx.x;
    if (r == 0 || merged[r] || !merged[r - 1]) return;
    const u64 beg = runst[r - 1] - 1, glen = pos[r] - beg;
    u8* o = out + 9 + off[r] + vb_len(glen) + 1;
    for (u64 k = threadIdx.x; k < glen; k += blockDim.x) o[k] = T[beg + k];
}
// the gap still open at the end of the stream (and the header)
__global__ void k_ssz_tail(const u8* __restrict__ T, u64 n, u64 z, const u8* __restrict__ merged,
                           const u64* __restrict__ runst, u64 off_end, u8* __restrict__ out) {
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        out[0] = 0;  // is_64_bit
        for (int k = 0; k < 8; k++) out[1 + k] = (u8)(n >> (8 * k));
    }
    if (!z || !merged[z - 1]) return;
    const u64 beg = runst[z - 1] - 1, glen = n - beg;
    u8* o = out + 9 + off_end;
    const u64 h = vb_len(glen) + 1;
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        const u64 k = vb_put(o, glen);
        o[k] = 0;
    }
    for (u64 k = (u64)blockIdx.x * blockDim.x + threadIdx.x; k < glen; k += (u64)gridDim.x * blockDim.x)
        o[h + k] = T[beg + k];
}

u64 engine::ssszip_gapped() {
    const u64 z = num_fact;
    const u32* F = fact.p;
    u64 total = 9;
    const unsigned g = cdiv(z, 256);
    u64* adv = x_off.get(4 * (z + 1));  // adv, pos, rs, runst
    u64* pos = adv + (z + 1);
    u64* rs = pos + (z + 1);
    u64* runst = rs + (z + 1);
    u32* dec = x_idx.get(2 * (z + 1));
    u32* lastdec = dec + (z + 1);
    u8* merged = (u8*)x_mark.get(z / 4 + 2);
    u64* sz = x_wide.get(2 * (z + 1));
    u64* off = sz + (z + 1);
    u64 off_end = 0, tail = 0;
    if (z) {
        k_ssz_prep<<<g, 256, 0, st>>>(F, z, adv, dec);
        excl_sum64(adv, pos, (u64)0, z, scan_tmp, st);
        incl_scan64(dec, lastdec, z, max_u32_op{}, scan_tmp, st);
        k_ssz_merged<<<g, 256, 0, st>>>(F, z, lastdec, merged, rs, pos);
        incl_scan64(rs, runst, z, max_u64_op{}, scan_tmp, st);
        k_ssz_size<<<g, 256, 0, st>>>(F, z, merged, runst, pos, sz);
        LZ_HIP(hipMemsetAsync(sz + z, 0, 8, st));
        excl_sum64(sz, off, (u64)0, z + 1, scan_tmp, st);
        off_end = rd1(off + z, st);
        u8 mlast = 0;
        u64 rlast = 0;
        LZ_HIP(hipMemcpyAsync(&mlast, merged + z - 1, 1, hipMemcpyDeviceToHost, st));
        LZ_HIP(hipMemcpyAsync(&rlast, runst + z - 1, 8, hipMemcpyDeviceToHost, st));
        LZ_HIP(hipStreamSynchronize(st));
        if (mlast) {
            const u64 glen = n - (rlast - 1);
            u64 h = 1;
            for (u64 x = glen; x >>= 7;) h++;
            tail = h + 1 + glen;
        }
    }
    total += off_end + tail;
    u8* out = ssz_out.get(total);
    if (z) {
        k_ssz_write<<<g, 256, 0, st>>>(F, z, merged, runst, pos, off, out);
        k_ssz_copy<<<(unsigned)z, 256, 0, st>>>(d_text, z, merged, runst, pos, off, out);
    }
    k_ssz_tail<<<std::max<unsigned>(1, cdiv(tail, 256 * 16)), 256, 0, st>>>(d_text, n, z, merged, runst, off_end, out);
    LZ_HIP(hipGetLastError());
    LZ_HIP(hipStreamSynchronize(st));
    ssz_size = total;
    return total;
}

}  // namespace lz
