// radix-sort configuration probe for the genome base sort: 1.31G (slot, entry) pairs,
// uniform slot < 2^25, values = a counting iterator (entry ids), as greedy.hip
#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/iterator/counting_iterator.hpp>
#include <cstdio>
#include <cstdint>
#include <vector>
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1);} } while (0)
using u32 = uint32_t;
__global__ void gen(u32* k, size_t m, u32 mask) {
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    uint64_t x = i * 0x9E3779B97F4A7C15ull; x ^= x >> 29; x *= 0xBF58476D1CE4E5B9ull; x ^= x >> 32;
    k[i] = (u32)x & mask;
}
__global__ void chk(const u32* v, size_t m, const u32* ref, unsigned long long* bad) {
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < m && v[i] != ref[i]) atomicAdd(bad, 1ull);
}
template <class Cfg>
void run(const char* name, u32* k, u32* k2, u32* v2, u32* ref, size_t m, int bits) {
    size_t tb = 0;
    const rocprim::counting_iterator<u32> ids(0);
    CK(rocprim::radix_sort_pairs<Cfg>(nullptr, tb, k, k2, ids, v2, m, 0, bits));
    void* t; CK(hipMalloc(&t, tb));
    hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    CK(rocprim::radix_sort_pairs<Cfg>(t, tb, k, k2, ids, v2, m, 0, bits));
    CK(hipEventRecord(a));
    const int R = 3;
    for (int r = 0; r < R; r++) CK(rocprim::radix_sort_pairs<Cfg>(t, tb, k, k2, ids, v2, m, 0, bits));
    CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
    float ms; CK(hipEventElapsedTime(&ms, a, b));
    unsigned long long* bad; CK(hipMalloc(&bad, 8)); CK(hipMemset(bad, 0, 8));
    if (ref) chk<<<(m + 255) / 256, 256>>>(v2, m, ref, bad);
    unsigned long long hb = 0; CK(hipMemcpy(&hb, bad, 8, hipMemcpyDeviceToHost));
    printf("%-44s %9.3f ms  %s\n", name, ms / R, hb ? "MISMATCH" : "ok");
    fflush(stdout);
    CK(hipFree(t)); CK(hipFree(bad));
}
int main() {
    const size_t m = 1312213715; const int bits = 25;
    u32 *k, *k2, *v2, *ref;
    CK(hipMalloc(&k, m * 4)); CK(hipMalloc(&k2, m * 4)); CK(hipMalloc(&v2, m * 4)); CK(hipMalloc(&ref, m * 4));
    gen<<<(m + 255) / 256, 256>>>(k, m, (1u << bits) - 1);
    CK(hipDeviceSynchronize());
    using namespace rocprim;
    run<default_config>("default", k, k2, ref, nullptr, m, bits);
#define OS(BS, IPT, RB, ALG) \
    run<radix_sort_config<default_config, default_config, radix_sort_onesweep_config<kernel_config<256, 12>, kernel_config<BS, IPT>, RB, block_radix_rank_algorithm::ALG>>>( \
        "onesweep bs=" #BS " ipt=" #IPT " rb=" #RB " " #ALG, k, k2, v2, ref, m, bits)
    OS(256, 12, 8, default_algorithm); OS(512, 8, 8, match);
    OS(256, 12, 9, match); OS(256, 16, 9, match); OS(512, 12, 9, match);
    OS(256, 12, 10, match); OS(512, 8, 10, match); OS(256, 16, 11, match);
    return 0;
}
