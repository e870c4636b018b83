// scancheck.hip -- scan_dev (include/prim.h) against a host
// scan: sums / min / max, exclusive / inclusive, in place, pad items (mr < m), u32 and u64.
//   hipcc -O2 --offload-arch=gfx950 -std=c++20 -I../../lz77-sss_amd/include scancheck.hip -o scancheck
#include "lz77sss_internal.h"
#include "prim.h"

#include <cstdio>
#include <random>
#include <vector>

using namespace lz;

template <class T, class Op, class HostOp>
static int check(u64 m, u64 mr, bool excl, bool inplace, T init, T id, Op op, HostOp hop, dbuf<u8>& tmp, hipStream_t st) {
    std::mt19937_64 g(m * 7 + mr);
    std::vector<T> h(m), want(m), got(m);
    for (u64 i = 0; i < m; i++) h[i] = (T)(g() % 1000);
    T run = excl ? init : id;
    if (!excl) run = init;
    for (u64 i = 0; i < m; i++) {
        const T x = i < mr ? h[i] : id;
        if (excl) { want[i] = run; run = hop(run, x); }
        else { run = hop(run, x); want[i] = run; }
    }
    T *d_in, *d_out;
    LZ_HIP(hipMalloc(&d_in, m * sizeof(T) + 8));
    LZ_HIP(hipMalloc(&d_out, m * sizeof(T) + 8));
    LZ_HIP(hipMemcpy(d_in, h.data(), m * sizeof(T), hipMemcpyHostToDevice));
    scan_dev(d_in, inplace ? d_in : d_out, m, mr, init, id, op, excl, tmp, st);
    LZ_HIP(hipStreamSynchronize(st));
    LZ_HIP(hipMemcpy(got.data(), inplace ? d_in : d_out, m * sizeof(T), hipMemcpyDeviceToHost));
    (void)hipFree(d_in);
    (void)hipFree(d_out);
    u64 bad = 0;
    for (u64 i = 0; i < m; i++) bad += got[i] != want[i];
    if (bad) std::printf("FAIL m=%llu mr=%llu excl=%d inplace=%d size=%zu: %llu bad\n", (unsigned long long)m,
                         (unsigned long long)mr, excl, inplace, sizeof(T), (unsigned long long)bad);
    return bad ? 1 : 0;
}

int main() {
    hipStream_t st;
    LZ_HIP(hipStreamCreate(&st));
    dbuf<u8> tmp;
    int fails = 0, runs = 0;
    const u64 sizes[] = {1, 2, 63, 64, 65, 1023, 1024, 1025, 4096, 54283, 32767, 32768, 32769, 65535, 65536, 65537, 200000};
    for (u64 m : sizes) {
        for (int e = 0; e < 2; e++)
            for (int ip = 0; ip < 2; ip++) {
                const u64 mr = m > 1 && e ? m - 1 : m;  // a pad item (the count arrays' total slot)
                fails += check<u32>(m, mr, e, ip, 0u, 0u, op_sum{}, [](u32 a, u32 b) { return a + b; }, tmp, st);
                fails += check<u64>(m, mr, e, ip, (u64)(e ? 5 : 0), (u64)0, op_sum{}, [](u64 a, u64 b) { return a + b; }, tmp, st);
                fails += check<u32>(m, m, e, ip, 0xFFFFFFFFu, 0xFFFFFFFFu, op_min{},
                                    [](u32 a, u32 b) { return a < b ? a : b; }, tmp, st);
                fails += check<u64>(m, m, e, ip, (u64)0, (u64)0, op_max{}, [](u64 a, u64 b) { return a > b ? a : b; },
                                    tmp, st);
                runs += 4;
            }
    }
    // timing: one-launch scan vs rocprim at the sizes of the headline step's count scans
    for (u64 m : {530ull, 21596ull, 32769ull, 54283ull}) {
        u32* d;
        LZ_HIP(hipMalloc(&d, (m + 1) * 4));
        LZ_HIP(hipMemset(d, 1, (m + 1) * 4));
        hipEvent_t a, b;
        LZ_HIP(hipEventCreate(&a));
        LZ_HIP(hipEventCreate(&b));
        for (int pass = 0; pass < 2; pass++) {
            scan_dev(d, d, m, m, 0u, 0u, op_sum{}, true, tmp, st);  // warm
            LZ_HIP(hipEventRecord(a, st));
            for (int r = 0; r < 20; r++) scan_dev(d, d, m, m, 0u, 0u, op_sum{}, true, tmp, st);
            LZ_HIP(hipEventRecord(b, st));
            LZ_HIP(hipEventSynchronize(b));
            float ms = 0;
            LZ_HIP(hipEventElapsedTime(&ms, a, b));
            size_t tb = 0;
            LZ_HIP(rocprim::exclusive_scan(nullptr, tb, d, d, 0u, (size_t)m, op_sum{}, st));
            u8* t = tmp.get(tb);
            LZ_HIP(hipEventRecord(a, st));
            for (int r = 0; r < 20; r++) LZ_HIP(rocprim::exclusive_scan(t, tb, d, d, 0u, (size_t)m, op_sum{}, st));
            LZ_HIP(hipEventRecord(b, st));
            LZ_HIP(hipEventSynchronize(b));
            float ms2 = 0;
            LZ_HIP(hipEventElapsedTime(&ms2, a, b));
            if (pass) std::printf("m=%llu: scan_dev %.1f us, rocprim %.1f us per scan\n", (unsigned long long)m, ms * 50.f,
                                  ms2 * 50.f);
        }
        (void)hipFree(d);
    }
    std::printf("scancheck: %d of %d cases failed\n", fails, runs);
    return fails ? 1 : 0;
}
