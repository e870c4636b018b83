// sortcheck.hip -- correctness of the device radix sorts the SA_S build uses (hipcub
// DeviceRadixSort::SortPairs, u64 keys on a bit range, u32 values) at sizes past 2^26 items:
// sortedness, stability (equal keys keep their value order) and key/value pairing.
//   hipcc -O2 --offload-arch=gfx950 -std=c++20 sortcheck.hip -o sortcheck && ./sortcheck 100000000 54
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e = (x);                                                          \
        if (e != hipSuccess) {                                                       \
            std::printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__);     \
            std::exit(2);                                                            \
        }                                                                            \
    } while (0)

__global__ void k_init(uint64_t* k, uint32_t* v, uint64_t n, uint32_t bits, uint64_t seed) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint64_t x = i * 0x9E3779B97F4A7C15ull + seed;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    x ^= x >> 31;
    // few distinct high parts: many equal keys (stability matters)
    k[i] = bits >= 64 ? x : (x & ((1ull << bits) - 1)) & ~((1ull << (bits / 2)) - 1);
    v[i] = (uint32_t)i;
}
__global__ void k_check(const uint64_t* kin, const uint64_t* k, const uint32_t* v, uint64_t n,
                        unsigned long long* bad) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    if (kin[v[i]] != k[i]) atomicAdd(bad, 1ull);                                   // pairing
    if (i && k[i - 1] > k[i]) atomicAdd(bad + 1, 1ull);                             // order
    if (i && k[i - 1] == k[i] && v[i - 1] > v[i]) atomicAdd(bad + 2, 1ull);         // stability
}

__global__ void k_counts(uint32_t* c, uint64_t n) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) c[i] = 1u + (uint32_t)((i * 2654435761u) >> 30);
}
__global__ void k_cmp(const uint32_t* a, const uint32_t* b, uint64_t n, unsigned long long* bad) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n && a[i] != b[i]) atomicAdd(bad, 1ull);
}

int main(int argc, char** argv) {
    const uint64_t n = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 100000000ull;
    const uint32_t bits = argc > 2 ? (uint32_t)std::atoi(argv[2]) : 54;
    uint64_t *k, *k2;
    uint32_t *v, *v2;
    unsigned long long* bad;
    CK(hipMalloc(&k, n * 8));
    CK(hipMalloc(&k2, n * 8));
    CK(hipMalloc(&v, n * 4));
    CK(hipMalloc(&v2, n * 4));
    CK(hipMalloc(&bad, 24));
    CK(hipMemset(bad, 0, 24));
    const unsigned g = (unsigned)((n + 255) / 256);
    k_init<<<g, 256>>>(k, v, n, bits, 12345);
    size_t tb = 0;
    CK(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, k, k2, v, v2, (int)n, 0, (int)bits));
    void* t;
    CK(hipMalloc(&t, tb));
    CK(hipcub::DeviceRadixSort::SortPairs(t, tb, k, k2, v, v2, (int)n, 0, (int)bits));
    k_check<<<g, 256>>>(k, k2, v2, n, bad);
    unsigned long long h[3];
    CK(hipMemcpy(h, bad, 24, hipMemcpyDeviceToHost));
    std::printf("n=%llu bits=%u temp=%zu: bad pairing=%llu order=%llu stability=%llu\n", (unsigned long long)n, bits,
                tb, h[0], h[1], h[2]);
    // in-place vs out-of-place inclusive sum of u32 counts (the SA_S piece offsets scan in place)
    uint32_t* c = v;
    uint32_t* c2 = v2;
    k_counts<<<g, 256>>>(c, n);
    size_t tb2 = 0;
    CK(hipcub::DeviceScan::InclusiveSum(nullptr, tb2, c, c2, (int)n));
    void* t2;
    CK(hipMalloc(&t2, tb2));
    CK(hipcub::DeviceScan::InclusiveSum(t2, tb2, c, c2, (int)n));  // out of place
    CK(hipcub::DeviceScan::InclusiveSum(t2, tb2, c, c, (int)n));   // in place
    CK(hipMemset(bad, 0, 24));
    k_cmp<<<g, 256>>>(c, c2, n, bad);
    CK(hipMemcpy(h, bad, 24, hipMemcpyDeviceToHost));
    std::printf("n=%llu in-place inclusive scan: %llu entries differ from the out-of-place scan\n",
                (unsigned long long)n, h[0]);
    return (h[0] || h[1] || h[2]) ? 1 : 0;
}
