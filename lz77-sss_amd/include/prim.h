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

}  // namespace lz
