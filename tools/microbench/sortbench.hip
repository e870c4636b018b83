// radix-sort configuration probe for the greedy base sort: 54.6M (slot, entry) pairs,
// slot < 2^25, entries = iota (stable order within a slot)
#include <hip/hip_runtime.h>
#include <cstring>
#include <rocprim/device/device_radix_sort.hpp>
#include <cstdio>
#include <vector>
#include <cstdint>
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1);} } while (0)
using u32 = uint32_t;
__global__ void gen(u32* k, u32* v, size_t m, u32 mask) {
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    uint64_t x = i * 0x9E3779B97F4A7C15ull; x ^= x >> 29; x *= 0xBF58476D1CE4E5B9ull; x ^= x >> 32;
    // 10% of entries in 64 hot slots (repetitive text)
    u32 s = (u32)x & mask;
    if ((x >> 40) % 10 == 0) s = (u32)((x >> 50) & 63) * 977;
    k[i] = s; v[i] = (u32)i;
}
template <class Cfg>
float run(const char* name, u32* k, u32* v, u32* k2, u32* v2, size_t m, int bits, std::vector<u32>* ref) {
    size_t tb = 0;
    CK(rocprim::radix_sort_pairs<Cfg>(nullptr, tb, k, k2, v, v2, m, 0, bits));
    void* t; CK(hipMalloc(&t, tb));
    hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    for (int w = 0; w < 2; w++) CK(rocprim::radix_sort_pairs<Cfg>(t, tb, k, k2, v, v2, m, 0, bits));
    CK(hipEventRecord(a));
    const int R = 10;
    for (int r = 0; r < R; r++) CK(rocprim::radix_sort_pairs<Cfg>(t, tb, k, k2, v, v2, m, 0, bits));
    CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
    float ms; CK(hipEventElapsedTime(&ms, a, b));
    std::vector<u32> h(m);
    CK(hipMemcpy(h.data(), v2, m * 4, hipMemcpyDeviceToHost));
    bool ok = true;
    if (ref->empty()) *ref = h; else ok = (h == *ref);
    printf("%-40s %8.3f ms  %s\n", name, ms / R, ok ? "ok" : "MISMATCH");
    CK(hipFree(t));
    return ms / R;
}
int main() {
    const size_t m = 54594560; const int bits = 25;
    u32 *k, *v, *k2, *v2;
    CK(hipMalloc(&k, m * 4)); CK(hipMalloc(&v, m * 4)); CK(hipMalloc(&k2, m * 4)); CK(hipMalloc(&v2, m * 4));
    gen<<<(m + 255) / 256, 256>>>(k, v, m, (1u << bits) - 1);
    CK(hipDeviceSynchronize());
    std::vector<u32> ref;
    using namespace rocprim;
    run<default_config>("default", k, v, k2, v2, m, bits, &ref);
#define OS(BS, IPT, RB, ALG) \
    run<radix_sort_config<default_config, default_config, radix_sort_onesweep_config<kernel_config<256, 12>, kernel_config<BS, IPT>, RB, block_radix_rank_algorithm::ALG>>>( \
        "onesweep bs=" #BS " ipt=" #IPT " rb=" #RB " " #ALG, k, v, k2, v2, m, bits, &ref)
    OS(256, 12, 8, default_algorithm); OS(256, 16, 8, default_algorithm); OS(512, 8, 8, match);
    OS(256, 12, 9, match); OS(256, 16, 9, match); OS(512, 12, 9, match);
    OS(256, 12, 10, match); OS(512, 8, 10, match); OS(256, 16, 11, match);
    OS(128, 12, 9, default_algorithm);
    return 0;
}
