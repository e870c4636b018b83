// Internal declarations shared by the host/device sources of liblz77sss_hip.so.
#pragma once
#define LZ77SSS_API __attribute__((visibility("default")))

#ifdef __HIPCC__
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdint>
#include <cstdio>
#include <chrono>
#include <cstdlib>
#include <stdexcept>
#include <string>
#include <vector>

namespace lz {

using u8 = uint8_t;
using u16 = uint16_t;
using u32 = uint32_t;
using u64 = uint64_t;
using u128 = unsigned __int128;

constexpr u32 TAU = 512;
constexpr u32 QL = TAU / 3;  // period bound of Q (170)
constexpr u32 QM = 2 * QL;   // anchor probe length (340)
constexpr u32 QA = 128;      // anchor stride
constexpr u64 P61 = (1ull << 61) - 1;
constexpr u32 INF32 = 0xFFFFFFFFu;  // Phi' of Q windows (and of windows hashing to 2^32-1)
constexpr u32 SSS_BASE = 296819;  // odd: invertible mod 2^32
constexpr u64 INF64 = ~0ull;
constexpr u32 NONE = 0xFFFFFFFFu;
// zero bytes allocated past n in the HBM text buffer: lets vector loads and
// the SSS lane streams run past the end without bounds checks
constexpr u64 TEXT_PAD = 64 * 1024;

// A dispatch's grid size is a 32-bit count of work-items (the HSA kernel dispatch packet), so a
// launch of 2^32 or more threads wraps around silently and covers only part of its domain (a
// wave-per-item kernel over more than 2^26 items, a thread-per-byte kernel over more than 4 GiB).
// Kernels whose domain can reach that loop over a capped grid (grid-stride), GRID_CAP blocks.
constexpr uint64_t GRID_CAP = 1ull << 20;
#ifdef __HIPCC__
__device__ __forceinline__ uint64_t gtid() { return (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; }
__device__ __forceinline__ uint64_t gstride() { return (uint64_t)gridDim.x * blockDim.x; }
#endif

// wall clock in ms (debug laps)
inline double now_ms() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

inline bool debug_enabled() {
    static int v = -1;
    if (v < 0) {
        const char* e = std::getenv("LZ77SSS_DEBUG");
        v = (e && *e && *e != '0') ? 1 : 0;
    }
    return v == 1;
}

// Block-aggregated counters.  The compiler already folds a uniform-address
// atomic into one per wave, but a device-scope atomic still costs ~10 ns and
// same-address ones serialize: a kernel with millions of waves pays seconds
// (the first decode: 16M wave atomics, 190 ms per round).  These helpers issue
// one atomic per workgroup; every thread of the block must call them.
// Needs blockDim.x <= 1024.
__device__ inline u32 block_count_claim(u32* ctr, bool pred) {
    __shared__ u32 s_wc[16], s_base;
    const u32 lane = threadIdx.x & 63, wv = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
    const u64 m = __ballot(pred);
    if (lane == 0) s_wc[wv] = (u32)__popcll(m);
    __syncthreads();
    if (threadIdx.x == 0) {
        u32 tot = 0;
        for (u32 w = 0; w < nw; w++) {
            const u32 c = s_wc[w];
            s_wc[w] = tot;
            tot += c;
        }
        s_base = tot ? atomicAdd(ctr, tot) : 0;
    }
    __syncthreads();
    const u32 r = s_base + s_wc[wv] + (u32)__popcll(m & ((1ull << lane) - 1));
    __syncthreads();  // s_wc / s_base reusable by a following call
    return r;
}
// adds v (per thread) to *acc with one atomic per workgroup
__device__ inline void block_add(u32* acc, u32 v) {
    __shared__ u32 s_sum;
    if (threadIdx.x == 0) s_sum = 0;
    __syncthreads();
    for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
    if ((threadIdx.x & 63) == 0 && v) atomicAdd(&s_sum, v);
    __syncthreads();
    if (threadIdx.x == 0 && s_sum) atomicAdd(acc, s_sum);
    __syncthreads();
}

// *acc = min(*acc, v over the block) with one atomic per workgroup
__device__ inline void block_min(u32* acc, u32 v) {
    __shared__ u32 s_min;
    if (threadIdx.x == 0) s_min = 0xFFFFFFFFu;
    __syncthreads();
    for (int o = 32; o > 0; o >>= 1) v = min(v, (u32)__shfl_down(v, o, 64));
    if ((threadIdx.x & 63) == 0 && v != 0xFFFFFFFFu) atomicMin(&s_min, v);
    __syncthreads();
    if (threadIdx.x == 0 && s_min != 0xFFFFFFFFu) atomicMin(acc, s_min);
    __syncthreads();
}

// 64-bit forms of block_add / block_min (sums and positions past 2^32)
__device__ inline void block_add64(u64* acc, u64 v) {
    __shared__ u64 s_sum64;
    if (threadIdx.x == 0) s_sum64 = 0;
    __syncthreads();
    for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
    if ((threadIdx.x & 63) == 0 && v) atomicAdd((unsigned long long*)&s_sum64, (unsigned long long)v);
    __syncthreads();
    if (threadIdx.x == 0 && s_sum64) atomicAdd((unsigned long long*)acc, (unsigned long long)s_sum64);
    __syncthreads();
}
__device__ inline void block_min64(u64* acc, u64 v) {
    __shared__ u64 s_min64;
    if (threadIdx.x == 0) s_min64 = ~0ull;
    __syncthreads();
    for (int o = 32; o > 0; o >>= 1) v = min(v, (u64)__shfl_down(v, o, 64));
    if ((threadIdx.x & 63) == 0 && v != ~0ull) atomicMin((unsigned long long*)&s_min64, (unsigned long long)v);
    __syncthreads();
    if (threadIdx.x == 0 && s_min64 != ~0ull) atomicMin((unsigned long long*)acc, (unsigned long long)s_min64);
    __syncthreads();
}

struct error : std::runtime_error {
    int code;
    error(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

#define LZ_HIP(x)                                                                                  \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess)                                                                      \
            throw ::lz::error(-3, std::string(#x) + ": " + hipGetErrorString(e_) + " @" __FILE__ ":" \
                                      + std::to_string(__LINE__));                                 \
    } while (0)

// device bytes held by dbufs in this process, and their peak (the "peak memory consumption"
// line of a logged factorization, lz77_sss.hpp:345-353)
inline std::atomic<uint64_t> g_dev_bytes{0}, g_dev_peak{0};
// the peak since the last phase mark (phase_timer: device bytes held per phase)
inline std::atomic<uint64_t> g_phase_peak{0};
inline void dev_bytes_add(int64_t b) {
    const uint64_t v = g_dev_bytes.fetch_add((uint64_t)b) + (uint64_t)b;
    uint64_t pk = g_dev_peak.load();
    while (b > 0 && v > pk && !g_dev_peak.compare_exchange_weak(pk, v)) {}
    uint64_t pp = g_phase_peak.load();
    while (b > 0 && v > pp && !g_phase_peak.compare_exchange_weak(pp, v)) {}
}

// grow-only device buffer
template <class T>
struct dbuf {
    T* p = nullptr;
    size_t cap = 0;
    dbuf() = default;
    dbuf(const dbuf&) = delete;
    dbuf& operator=(const dbuf&) = delete;
    T* get(size_t n) {
        if (n > cap) {
            const size_t c = std::max<size_t>(n, cap + cap / 4);
            if (p) {
                LZ_HIP(hipFree(p));
                dev_bytes_add(-(int64_t)(cap * sizeof(T)));
            }
            p = nullptr;
            cap = 0;
            LZ_HIP(hipMalloc(&p, std::max<size_t>(c, 1) * sizeof(T)));
            cap = c;
            dev_bytes_add((int64_t)(cap * sizeof(T)));
        }
        return p;
    }
    // grow keeping the first `keep` elements (stream-ordered copy on st)
    T* grow_keep(size_t n, size_t keep, hipStream_t st) {
        if (n <= cap) return p;
        T* q = nullptr;
        const size_t c = std::max<size_t>(n, cap + cap / 2);
        LZ_HIP(hipMalloc(&q, c * sizeof(T)));
        dev_bytes_add((int64_t)(c * sizeof(T)));
        if (p && keep) LZ_HIP(hipMemcpyAsync(q, p, keep * sizeof(T), hipMemcpyDeviceToDevice, st));
        if (p) {
            LZ_HIP(hipStreamSynchronize(st));
            LZ_HIP(hipFree(p));
            dev_bytes_add(-(int64_t)(cap * sizeof(T)));
        }
        p = q;
        cap = c;
        return p;
    }
    void release() {
        if (p) {
            (void)hipFree(p);
            dev_bytes_add(-(int64_t)(cap * sizeof(T)));
        }
        p = nullptr;
        cap = 0;
    }
    ~dbuf() { release(); }
};

// ---------------------------------------------------------------------------
// device helpers
__device__ __forceinline__ u64 mod61_canon(u64 x) {  // x < 2^62
    u64 c = (x & P61) + (x >> 61);
    return c >= P61 ? c - P61 : c;
}
// unaligned 8-byte little-endian load from global memory
__device__ __forceinline__ u64 ldu64(const u8* p) {
    u64 a = (u64)(uintptr_t)p;
    const u64* q = (const u64*)(a & ~7ull);
    u32 sh = (u32)(a & 7) * 8;
    u64 lo = q[0];
    if (!sh) return lo;
    u64 hi = q[1];
    return (lo >> sh) | (hi << (64 - sh));
}
// forward LCE of T[a..] and T[b..], at most lim bytes (caller guarantees
// a+lim, b+lim <= n + TEXT_PAD)
__device__ __forceinline__ u64 dev_naive_lce(const u8* T, u64 a, u64 b, u64 lim) {
    u64 k = 0;
    // 32 bytes per round: the eight loads of a round are issued before any compare (one memory
    // round trip instead of four; a long comparison is latency-bound)
    while (k + 32 <= lim) {
        u64 x[4], y[4];
#pragma unroll
        for (int t = 0; t < 4; t++) {
            x[t] = ldu64(T + a + k + 8 * t);
            y[t] = ldu64(T + b + k + 8 * t);
        }
#pragma unroll
        for (int t = 0; t < 4; t++)
            if (x[t] != y[t]) return k + 8 * t + (__builtin_ctzll(x[t] ^ y[t]) >> 3);
        k += 32;
    }
    while (k + 8 <= lim) {
        u64 x = ldu64(T + a + k), y = ldu64(T + b + k);
        if (x != y) return k + (__builtin_ctzll(x ^ y) >> 3);
        k += 8;
    }
    while (k < lim && T[a + k] == T[b + k]) k++;
    return k;
}

}  // namespace lz

// The approximate-factorization pipeline is compiled twice (Makefile): once with
// pos_t = uint32_t in namespace lz, and once with -DLZ_POS64, pos_t = uint64_t in
// namespace lz64 (lz77_sss<pos_t> with pos_t in {uint32_t, uint64_t},
// include/lz77_sss/lz77_sss.hpp:72-75).  Text positions and lengths are pos_t;
// sync indices, ranks, segment and entry ids stay 32-bit.
#ifdef LZ_POS64
#define LZ_NS lz64
namespace lz64 {
using namespace lz;
using pos_t = uint64_t;
}  // namespace lz64
#else
#define LZ_NS lz
namespace lz {
using pos_t = uint32_t;
}  // namespace lz
#endif
namespace LZ_NS {
constexpr pos_t POS_NONE = ~(pos_t)0;
constexpr u64 POS_MAX_N = sizeof(pos_t) == 4 ? 0xFFFFFFF0ull : (1ull << 40);  // largest supported n
}  // namespace LZ_NS
#endif
