// msort_dev.h -- comparison merge sort of u32 item ids on the device (runs of RUN items
// by insertion sort, then merge-path passes that double the run width).  Used where the
// order needs a comparator that reads the text (LCE): SA_S tie groups (csrc/sa_s.hip)
// and the sample orders PA / SA of the exact-smpl path (csrc/smpl.hip).
#pragma once
#include "lz77sss_internal.h"

namespace LZ_NS {

constexpr u32 MS_RUN = 8;
constexpr u32 MS_MPT = 8;  // outputs per thread in a merge pass
template <class C>
__global__ void k_msort_runs(const u32* __restrict__ in, u32* __restrict__ out, u32 d, C cmp) {
    const u64 b = ((u64)blockIdx.x * blockDim.x + threadIdx.x) * MS_RUN;
    if (b >= d) return;
    const u32 m = (u32)min<u64>(MS_RUN, d - b);
    u32 v[MS_RUN];
    for (u32 i = 0; i < m; i++) v[i] = in[b + i];
    for (u32 i = 1; i < m; i++) {
        const u32 x = v[i];
        int j = (int)i - 1;
        while (j >= 0 && cmp(x, v[j])) { v[j + 1] = v[j]; j--; }
        v[j + 1] = x;
    }
    for (u32 i = 0; i < m; i++) out[b + i] = v[i];
}
template <class C>
__global__ void k_msort_merge(const u32* __restrict__ in, u32* __restrict__ out, u32 d, u32 w, C cmp) {
    const u64 p0 = ((u64)blockIdx.x * blockDim.x + threadIdx.x) * MS_MPT;
    if (p0 >= d) return;
    const u64 base = p0 / (2ull * w) * (2ull * w);
    const u64 a0 = base, a1 = min<u64>(base + w, d), b0 = a1, b1 = min<u64>(base + 2ull * w, d);
    const u64 la = a1 - a0, lb = b1 - b0;
    const u64 diag = p0 - base;
    // merge path: i items from A, diag - i from B; A wins ties (stable)
    u64 lo = diag > lb ? diag - lb : 0, hi = min(diag, la);
    while (lo < hi) {
        const u64 mid = (lo + hi) >> 1;
        // take A[mid] before B[diag-1-mid] iff !(B < A)
        if (!cmp(in[b0 + diag - 1 - mid], in[a0 + mid])) lo = mid + 1; else hi = mid;
    }
    u64 i = lo, j = diag - lo;
    const u64 pend = min<u64>(p0 + MS_MPT, b1);
    for (u64 p = p0; p < pend; p++) {
        bool takeA;
        if (i >= la) takeA = false;
        else if (j >= lb) takeA = true;
        else takeA = !cmp(in[b0 + j], in[a0 + i]);
        out[p] = takeA ? in[a0 + i++] : in[b0 + j++];
    }
}
// sorts `a` (d items) stably; `tmp` has room for d items; result left in `a`
template <class C>
static void merge_sort_u32(u32* a, u32* tmp, u32 d, C cmp, hipStream_t st) {
    if (d <= 1) return;
    k_msort_runs<<<(unsigned)((((u64)d + MS_RUN - 1) / MS_RUN + 255) / 256), 256, 0, st>>>(a, tmp, d, cmp);
    u32* src = tmp;
    u32* dst = a;
    for (u64 w = MS_RUN; w < d; w *= 2) {
        k_msort_merge<<<(unsigned)((((u64)d + MS_MPT - 1) / MS_MPT + 255) / 256), 256, 0, st>>>(src, dst, d, (u32)w,
                                                                                              cmp);
        std::swap(src, dst);
    }
    if (src != a) LZ_HIP(hipMemcpyAsync(a, src, (size_t)d * 4, hipMemcpyDeviceToDevice, st));
    LZ_HIP(hipGetLastError());
}

}  // namespace LZ_NS
