// prim.h -- device-wide scans with 64-bit item counts (rocprim takes size_t
// sizes; hipcub's DeviceScan takes int, which wraps past 2^31 items).
#pragma once
#include "lz77sss_internal.h"

#include <rocprim/device/device_scan.hpp>

namespace lz {

// out[k] = init + sum in[0..k), k < m
template <class I, class O, class T>
inline void excl_sum64(I in, O out, T init, u64 m, dbuf<u8>& tmp, hipStream_t st) {
    size_t tb = 0;
    LZ_HIP(rocprim::exclusive_scan(nullptr, tb, in, out, init, (size_t)m, rocprim::plus<T>(), st));
    u8* t = tmp.get(std::max<size_t>(tb, 1));
    LZ_HIP(rocprim::exclusive_scan(t, tb, in, out, init, (size_t)m, rocprim::plus<T>(), st));
}
// out[k] = op(in[0..k]), k < m
template <class I, class O, class Op>
inline void incl_scan64(I in, O out, u64 m, Op op, dbuf<u8>& tmp, hipStream_t st) {
    size_t tb = 0;
    LZ_HIP(rocprim::inclusive_scan(nullptr, tb, in, out, (size_t)m, op, st));
    u8* t = tmp.get(std::max<size_t>(tb, 1));
    LZ_HIP(rocprim::inclusive_scan(t, tb, in, out, (size_t)m, op, st));
}

// ---------------------------------------------------------------------------
// Scans of small arrays (the per-phrase, per-stripe, per-segment and sync-set counts of a
// factorization: often a few hundred to 64 Ki items) in ONE launch of one workgroup: rocprim's
// decoupled-lookback scan costs a state-init kernel and a scan kernel (and the host round trip
// of its temp-size query pattern) per call, which on the headline text is most of a scan's time.
// in == out is allowed; items at or past `mr` read as the identity (the total of a count array
// then lands at out[m - 1 + excl] without a memset of the pad entry).
constexpr u32 SCAN_SMALL_T = 1024;
constexpr u64 SCAN_SMALL_MAX = 1u << 16;
struct op_sum {
    template <class T>
    __device__ __forceinline__ T operator()(T a, T b) const { return a + b; }
};
struct op_min {
    template <class T>
    __device__ __forceinline__ T operator()(T a, T b) const { return a < b ? a : b; }
};
struct op_max {
    template <class T>
    __device__ __forceinline__ T operator()(T a, T b) const { return a > b ? a : b; }
};
template <class T, class Op>
__global__ __launch_bounds__(SCAN_SMALL_T) void k_scan_small(const T* in, T* out, u32 m, u32 mr, T init, T id, Op op,
                                                              int excl) {
    __shared__ T s_w[SCAN_SMALL_T / 64];
    const u32 t = threadIdx.x, lane = t & 63, wv = t >> 6;
    const u32 per = (m + SCAN_SMALL_T - 1) / SCAN_SMALL_T;
    const u32 b = min(m, t * per), e = min(m, b + per);
    T tot = id;
    for (u32 i = b; i < e; i++) tot = op(tot, i < mr ? in[i] : id);
    T incl = tot;
    for (u32 o = 1; o < 64; o <<= 1) {
        const T y = __shfl_up(incl, o, 64);
        if (lane >= o) incl = op(y, incl);
    }
    if (lane == 63) s_w[wv] = incl;
    __syncthreads();
    T run = init;
    for (u32 w = 0; w < wv; w++) run = op(run, s_w[w]);
    const T ex = __shfl_up(incl, 1, 64);
    if (lane) run = op(run, ex);
    for (u32 i = b; i < e; i++) {
        const T x = i < mr ? in[i] : id;
        if (excl) {
            out[i] = run;
            run = op(run, x);
        } else {
            run = op(run, x);
            out[i] = run;
        }
    }
}
// out[k] = init op in[0..k) (exclusive) or in[0..k] (inclusive), k < m; in[k] = id for k >= mr
template <class T, class Op>
inline void scan_dev(const T* in, T* out, u64 m, u64 mr, T init, T id, Op op, bool excl, dbuf<u8>& tmp, hipStream_t st) {
    if (m == 0) return;
    if (m <= SCAN_SMALL_MAX) {
        k_scan_small<T, Op><<<1, SCAN_SMALL_T, 0, st>>>(in, out, (u32)m, (u32)std::min(mr, m), init, id, op, excl ? 1 : 0);
        LZ_HIP(hipGetLastError());
        return;
    }
    if (mr < m) LZ_HIP(hipMemsetAsync(const_cast<T*>(in) + mr, 0, (m - mr) * sizeof(T), st));  // (sums only: id == 0)
    size_t tb = 0;
    if (excl) {
        LZ_HIP(rocprim::exclusive_scan(nullptr, tb, in, out, init, (size_t)m, op, st));
        u8* t = tmp.get(std::max<size_t>(tb, 1));
        LZ_HIP(rocprim::exclusive_scan(t, tb, in, out, init, (size_t)m, op, st));
    } else {
        LZ_HIP(rocprim::inclusive_scan(nullptr, tb, in, out, (size_t)m, op, st));
        u8* t = tmp.get(std::max<size_t>(tb, 1));
        LZ_HIP(rocprim::inclusive_scan(t, tb, in, out, (size_t)m, op, st));
    }
}
// exclusive sum over m + 1 items of a count array cnt[0..m) (off[m] = total; cnt[m] is not read
// on the small path, zeroed on the large one)
template <class T>
inline void excl_sum_total(T* cnt, T* off, u64 m, dbuf<u8>& tmp, hipStream_t st) {
    scan_dev(cnt, off, m + 1, m, (T)0, (T)0, op_sum{}, true, tmp, st);
}
template <class T>
inline void incl_sum(const T* in, T* out, u64 m, dbuf<u8>& tmp, hipStream_t st) {
    scan_dev(in, out, m, m, (T)0, (T)0, op_sum{}, false, tmp, st);
}

}  // namespace lz
