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
// Device scans with 64-bit item counts behind one call (rocprim: hipcub's DeviceScan takes int).
// (A one-workgroup scan for arrays of up to 64 Ki items was measured against rocprim's
// decoupled-lookback scan, tools/microbench/scancheck.hip: 4.6-14 us against 2.8-6.6 us per call
// back to back, so rocprim stays.)  in == out is allowed.
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
// out[k] = init op in[0..k) (exclusive) or in[0..k] (inclusive: init must be the identity id), k < m;
// in[k] = id for k >= mr (sums only: the pad is zeroed)
template <class T, class Op>
inline void scan_dev(const T* in, T* out, u64 m, u64 mr, T init, T id, Op op, bool excl, dbuf<u8>& tmp, hipStream_t st) {
    (void)id;
    if (m == 0) return;
    if (mr < m) LZ_HIP(hipMemsetAsync(const_cast<T*>(in) + mr, 0, (m - mr) * sizeof(T), st));
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
// exclusive sum over m + 1 items of a count array cnt[0..m) (off[m] = total; cnt[m] is zeroed)
template <class T>
inline void excl_sum_total(T* cnt, T* off, u64 m, dbuf<u8>& tmp, hipStream_t st) {
    scan_dev(cnt, off, m + 1, m, (T)0, (T)0, op_sum{}, true, tmp, st);
}
template <class T>
inline void incl_sum(const T* in, T* out, u64 m, dbuf<u8>& tmp, hipStream_t st) {
    scan_dev(in, out, m, m, (T)0, (T)0, op_sum{}, false, tmp, st);
}

}  // namespace lz
