// Streaming shapes for k_sss_runs' run crossing (tools/microbench; not product code):
// a 1 GiB text of period-1 runs, every 512-byte block checked for a period-p break the way the
// crossing loop does it.  Variants differ in blocks per wave, chunk depth and load width, to
// find what the crossing's HBM rate is bound by.
//   hipcc -O3 --offload-arch=gfx950 stream_runs.hip -o stream_runs && ./stream_runs
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <vector>
typedef uint64_t u64;
typedef uint32_t u32;
typedef uint8_t u8;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("hip error %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

// plain read: every wave sums 16-byte loads over its span (the HBM read ceiling of this shape)
template <int UNROLL>
__global__ __launch_bounds__(256) void k_read(const uint4* __restrict__ T, u64 n16, u64 per_wave, u32* out) {
    const u32 lane = threadIdx.x & 63;
    const u64 w = (u64)blockIdx.x * 4 + (threadIdx.x >> 6);
    const u64 a = w * per_wave, b = min(n16, a + per_wave);
    u32 acc = 0;
    for (u64 i = a + lane; i < b; i += 64 * UNROLL) {
        uint4 v[UNROLL];
#pragma unroll
        for (int u = 0; u < UNROLL; u++) v[u] = T[min(i + 64 * u, n16 - 1)];
#pragma unroll
        for (int u = 0; u < UNROLL; u++) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

// the crossing shape: one wave per span of NB blocks, chunks of CH blocks (8-byte lane loads)
// staged through an LDS ring of RS blocks, DEPTH chunks in flight; per block one p-shifted
// compare from the ring and a ballot (the first break ends the wave's count)
template <u32 NB, u32 CH, u32 RS, u32 DEPTH>
__global__ __launch_bounds__(256) void k_cross(const unsigned char* __restrict__ T, u64 nblk_total, u32 p,
                                               u32* __restrict__ out) {
    __shared__ u64 s_ring[4][RS * 64];
    const u32 lane = threadIdx.x & 63;
    u64* ring = s_ring[threadIdx.x >> 6];
    const u64 w = (u64)blockIdx.x * 4 + (u32)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const u64 b0 = w * NB;
    if (b0 >= nblk_total) return;
    auto load8 = [&](u64 k) -> u64 { return *(const u64*)(T + (b0 + k) * 512 + 8 * lane); };
    u64 R[DEPTH][CH];
#pragma unroll
    for (u32 d = 0; d < DEPTH; d++)
#pragma unroll
        for (u32 e = 0; e < CH; e++) R[d][e] = load8(d * CH + e);
    u32 brk = 0;
    const u32 ol = lane + (p >> 3), sh = 8 * (p & 7);
    for (u32 c = 0; c < NB; c += CH) {
        // the oldest chunk into the ring, the next one loading
#pragma unroll
        for (u32 e = 0; e < CH; e++) ring[((c + e) % RS) * 64 + lane] = R[0][e];
#pragma unroll
        for (u32 d = 0; d + 1 < DEPTH; d++)
#pragma unroll
            for (u32 e = 0; e < CH; e++) R[d][e] = R[d + 1][e];
#pragma unroll
        for (u32 e = 0; e < CH; e++) R[DEPTH - 1][e] = load8(c + DEPTH * CH + e);
        __builtin_amdgcn_wave_barrier();
        if (c == 0) continue;  // block c - CH .. c - 1 checked once their successor chunk is in
        u64 acc = 0;
#pragma unroll
        for (u32 j = 0; j < CH; j++) {
            const u32 k = c - CH + j;
            const u32 o = (k % RS) * 64;
            const u64 lo = ring[(o + ol) % (RS * 64)], hi = ring[(o + ol + 1) % (RS * 64)];
            const u64 d = ring[o + lane] ^ (sh ? ((lo >> sh) | (hi << (64 - sh))) : lo);
            acc |= d;
        }
        if (__ballot(acc != 0)) brk++;
    }
    if (lane == 0 && brk) atomicAdd(out, brk);
}

extern "C" int64_t lz77sss_gen_random_repetitive(uint32_t, uint32_t, uint32_t, double, double, uint8_t*, uint64_t);

// k_sss_pure's shape: a per-stripe state word read first (HSTATE), the period of block 1 found
// by a candidate search before the stream (PSEARCH: here by one ballot per shift, as a cost
// stand-in), an exit at the first chunk with a break (EXIT)
template <bool HSTATE, bool PSEARCH, bool EXIT>
__global__ __launch_bounds__(256) void k_pure_like(const unsigned char* __restrict__ T, u64 nstripes,
                                                   const u64* __restrict__ hitw, u32* __restrict__ out) {
    constexpr u32 CH = 8, RS = 16;
    __shared__ u64 s_ring[4][RS * 64];
    const u32 lane = threadIdx.x & 63;
    u64* ring = s_ring[threadIdx.x >> 6];
    const u64 w = (u64)blockIdx.x * 4 + (u32)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    if (w + 1 >= nstripes) return;
    if (HSTATE && !(hitw[3 * w + 2] >> 63)) return;
    const unsigned char* Tw = T + w * 32768ull + 8 * lane;
    auto load8 = [&](u32 k) -> u64 { return *(const u64*)(Tw + (u64)k * 512); };
    u64 R0[CH], R1[CH];
#pragma unroll
    for (u32 e = 0; e < CH; e++) R0[e] = load8(e);
#pragma unroll
    for (u32 e = 0; e < CH; e++) R1[e] = load8(CH + e);
    u32 P = 2, ol = lane, sh = 16, brk = 0;
#pragma unroll
    for (u32 g = 0; g <= 9; g++) {
        const u32 c = CH * g;
        if (g <= 8) {
#pragma unroll
            for (u32 e = 0; e < CH; e++) ring[((c + e) % RS) * 64 + lane] = R0[e];
#pragma unroll
            for (u32 e = 0; e < CH; e++) R0[e] = R1[e];
            if (g + 2 <= 8) {
#pragma unroll
                for (u32 e = 0; e < CH; e++) R1[e] = load8(c + 2 * CH + e);
            }
        }
        __builtin_amdgcn_wave_barrier();
        if (g == 0) {
            if (PSEARCH) {
                P = 0;
                for (u32 q = 1; q <= 170 && !P; q++) {
                    const u32 o = 64 + lane + (q >> 3), s2 = 8 * (q & 7);
                    const u64 lo = ring[o], hi = ring[o + 1];
                    const u64 v = s2 ? ((lo >> s2) | (hi << (64 - s2))) : lo;
                    if (!__ballot(v != ring[64 + lane])) P = q;
                }
                if (!P) return;
                ol = lane + (P >> 3);
                sh = 8 * (P & 7);
            }
            continue;
        }
        u64 acc = 0;
#pragma unroll
        for (u32 j = 0; j < CH; j++) {
            const u32 k = c - CH + j;
            if (k > 65) break;
            const u32 o = (k % RS) * 64;
            const u64 lo = ring[(o + ol) % (RS * 64)], hi = ring[(o + ol + 1) % (RS * 64)];
            acc |= ring[o + lane] ^ (sh ? ((lo >> sh) | (hi << (64 - sh))) : lo);
        }
        if (__ballot(acc != 0)) {
            if (EXIT) return;
            brk++;
        }
    }
    if (lane == 0) out[16 + (w & 1023)] = 1u + brk;
}


// --- k_sss_pure (round-6 v1) as in csrc/sss.hip, with switches: PS = period search of block 1 by
// candidates (else P = 2), HW = per-stripe state word first
__device__ __forceinline__ u64 shfl64(u64 v, u32 src) {
    return ((u64)(u32)__shfl((int)(u32)(v >> 32), (int)src, 64) << 32) | (u32)__shfl((int)(u32)v, (int)src, 64);
}
template <int CTRL, int ROWM = 0xF>
__device__ __forceinline__ u32 dpp(u32 old, u32 v) {
    return (u32)__builtin_amdgcn_update_dpp((int)old, (int)v, CTRL, ROWM, 0xF, false);
}
__device__ __forceinline__ u64 shifted8(u64 Bx, u64 By, u32 p, u32 lane) {
    const u32 q = p >> 3, sh = 8 * (p & 7);
    const u32 src = (lane + q) & 63;
    const u64 a = shfl64(Bx, src), c = shfl64(By, src);
    const u64 w0 = lane + q >= 64 ? c : a;
    if (!sh) return w0;
    u64 w1 = ((u64)dpp<0x130>(0u, (u32)(w0 >> 32)) << 32) | dpp<0x130>(0u, (u32)w0);
    if (lane == 63)
        w1 = ((u64)(u32)__builtin_amdgcn_readlane((int)(u32)(By >> 32), (int)q) << 32) |
             (u32)__builtin_amdgcn_readlane((int)(u32)By, (int)q);
    return (w0 >> sh) | (w1 << (64 - sh));
}
__device__ __forceinline__ u32 smallest_period(u64 Bx, u64 By, u32 lane) {
    const u64 A = ((u64)(u32)__builtin_amdgcn_readlane((int)(u32)(Bx >> 32), 0) << 32) |
                  (u32)__builtin_amdgcn_readlane((int)(u32)Bx, 0);
    const u32 j0 = (3 * lane + 1) >> 3;
    const u64 w0 = shfl64(Bx, j0 & 63), w1 = shfl64(Bx, (j0 + 1) & 63), w2 = shfl64(Bx, (j0 + 2) & 63);
    u64 m[3];
#pragma unroll
    for (u32 k = 0; k < 3; k++) {
        const u32 q = 3 * lane + 1 + k, r = q - 8 * j0;
        const u64 v = r == 0 ? w0 : r < 8 ? (w0 >> (8 * r)) | (w1 << (64 - 8 * r))
                                 : r == 8 ? w1 : (w1 >> (8 * (r - 8))) | (w2 << (64 - 8 * (r - 8)));
        m[k] = __ballot(q <= 170 && v == A);
    }
    for (;;) {
        u32 best = 0xFFFFu;
#pragma unroll
        for (u32 k = 0; k < 3; k++)
            if (m[k]) best = min(best, 3u * (u32)__builtin_ctzll(m[k]) + 1 + k);
        if (best > 170) return 0;
        m[(best - 1) % 3] &= ~(1ull << ((best - 1) / 3));
        if (!__ballot(shifted8(Bx, By, best, lane) != Bx)) return best;
    }
}
template <bool PS, bool HW, u32 WPG>
__global__ __launch_bounds__(64 * WPG) void k_pure_v1(const unsigned char* __restrict__ T, u64 nstripes,
                                                       const u64* __restrict__ hitw, u32* __restrict__ out) {
    constexpr u32 PR_CH = 8, PR_RS = 16;
    __shared__ u64 s_ring[WPG][PR_RS * 64];
    const u32 lane = threadIdx.x & 63;
    u64* ring = s_ring[threadIdx.x >> 6];
    const u64 w = (u64)blockIdx.x * WPG + (u32)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    if (w + 1 >= nstripes) return;
    if (HW && !(hitw[3 * w + 2] >> 63)) return;
    const unsigned char* Tw = T + w * 32768ull + 8 * lane;
    auto load8 = [&](u32 k) -> u64 { return *(const u64*)(Tw + (u64)k * 512); };
    u64 Q[3][PR_CH];
#pragma unroll
    for (u32 d = 0; d < 2; d++)
#pragma unroll
        for (u32 e = 0; e < PR_CH; e++) Q[d][e] = load8(d * PR_CH + e);
    u32 P = 2, ol = lane, sh = 16;
#pragma unroll
    for (u32 g = 0; g <= 9; g++) {
        const u32 c = PR_CH * g;
        if (g + 2 <= 8) {
#pragma unroll
            for (u32 e = 0; e < PR_CH; e++) Q[(g + 2) % 3][e] = load8(c + 2 * PR_CH + e);
        }
        if (g <= 8) {
#pragma unroll
            for (u32 e = 0; e < PR_CH; e++) ring[((c + e) % PR_RS) * 64 + lane] = Q[g % 3][e];
        }
        __builtin_amdgcn_wave_barrier();
        if (g == 0) {
            if (PS) {
                P = smallest_period(ring[64 + lane], ring[128 + lane], lane);
                if (!P) return;
                ol = lane + (P >> 3);
                sh = 8 * (P & 7);
            }
            continue;
        }
        u64 acc = 0;
#pragma unroll
        for (u32 j = 0; j < PR_CH; j++) {
            const u32 k = c - PR_CH + j;
            if (k > 65) break;
            const u32 o = (k % PR_RS) * 64;
            const u64 lo = ring[(o + ol) % (PR_RS * 64)], hi = ring[(o + ol + 1) % (PR_RS * 64)];
            acc |= ring[o + lane] ^ (sh ? ((lo >> sh) | (hi << (64 - sh))) : lo);
        }
        if (__ballot(acc != 0)) return;
    }
    if (lane == 0) out[16 + (w & 1023)] = P;
}

// k_cross with k_sss_pure's features one at a time: EXIT at the first chunk with a break, HW state
// word first, PADB extra ring blocks of LDS (fewer workgroups per CU), NCHK blocks checked
template <bool EXIT, bool HW, u32 PADB, u32 NCHK>
__global__ __launch_bounds__(256) void k_cross2(const unsigned char* __restrict__ T, u64 nstripes, u32 p,
                                                const u64* __restrict__ hitw, u32* __restrict__ out) {
    constexpr u32 CH = 8, RS = 16, DEPTH = 2;
    __shared__ u64 s_ring[4][(RS + PADB) * 64];
    const u32 lane = threadIdx.x & 63;
    u64* ring = s_ring[threadIdx.x >> 6];
    const u64 w = (u64)blockIdx.x * 4 + (u32)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    if (w + 1 >= nstripes) return;
    if (HW && !(hitw[3 * w + 2] >> 63)) return;
    const u64 b0 = w * 64;
    auto load8 = [&](u64 k) -> u64 { return *(const u64*)(T + (b0 + k) * 512 + 8 * lane); };
    u64 R[DEPTH][CH];
#pragma unroll
    for (u32 d = 0; d < DEPTH; d++)
#pragma unroll
        for (u32 e = 0; e < CH; e++) R[d][e] = load8(d * CH + e);
    u32 brk = 0;
    const u32 ol = lane + (p >> 3), sh = 8 * (p & 7);
    for (u32 c = 0; c < NCHK + CH; c += CH) {
#pragma unroll
        for (u32 e = 0; e < CH; e++) ring[((c + e) % RS) * 64 + lane] = R[0][e];
#pragma unroll
        for (u32 d = 0; d + 1 < DEPTH; d++)
#pragma unroll
            for (u32 e = 0; e < CH; e++) R[d][e] = R[d + 1][e];
#pragma unroll
        for (u32 e = 0; e < CH; e++) R[DEPTH - 1][e] = load8(c + DEPTH * CH + e);
        __builtin_amdgcn_wave_barrier();
        if (c == 0) continue;
        u64 acc = 0;
#pragma unroll
        for (u32 j = 0; j < CH; j++) {
            const u32 k = c - CH + j;
            if (k >= NCHK) break;
            const u32 o = (k % RS) * 64;
            const u64 lo = ring[(o + ol) % (RS * 64)], hi = ring[(o + ol + 1) % (RS * 64)];
            acc |= ring[o + lane] ^ (sh ? ((lo >> sh) | (hi << (64 - sh))) : lo);
        }
        if (__ballot(acc != 0)) {
            if (EXIT) return;
            brk++;
        }
    }
    if (lane == 0 && brk) atomicAdd(out, brk);
}

// --- run_scan of csrc/sss.hip (k_sss_runs' phase 1) alone, in a lean kernel (copied verbatim)
constexpr u32 TAU = 512;
constexpr u32 QL = 170;
constexpr u32 RM_CH = 8;
__device__ __forceinline__ u32 run_scan(const u8* __restrict__ Tw, u64* __restrict__ ring, u32 rs, u32 lane,
                                        u32& mreg, u32& m64, u32& m65) {
    auto load8 = [&](u32 k) -> u64 { return *(const u64*)(Tw + (u64)k * TAU); };
    // two chunk buffers, each refilled right after it is stored (no register copies: a copy of a
    // loading register waits for its load), so two chunks stay in flight
    u64 A[RM_CH], B[RM_CH];
    auto load_to = [&](u64* X, u32 k0) {
        // (in issue order: the scheduler may not interleave two chunks' loads, or a wait for the
        // older chunk would drain the younger one too)
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (u32 e = 0; e < RM_CH; e++) X[e] = load8(k0 + e);
        __builtin_amdgcn_sched_barrier(0);
    };
    auto store_from = [&](const u64* X, u32 k0) {
#pragma unroll
        for (u32 e = 0; e < RM_CH; e++) ring[((k0 + e) % rs) * 64 + lane] = X[e];
    };
    u32 P0 = 0, P = 0, ol = 0, sh = 0, nsearch = 0;
    bool pure = true;
    auto put = [&](u32 k, u32 m) {
        if (k < 64) mreg = lane == k ? m : mreg;
        else if (k == 64) m64 = m;
        else m65 = m;
    };
    // blocks k0 .. k0 + 7 (<= 65) against their bytes P ahead; a chunk with a break block by block
    auto check = [&](u32 k0) {
        u64 acc = 0;
        if (P) {
            // (no branch per block: the 24 ring reads issue together, blocks past 65 are masked)
#pragma unroll
            for (u32 j = 0; j < RM_CH; j++) {
                const u32 k = k0 + j, o = (k % rs) * 64;
                const u64 lo = ring[(o + ol) % (rs * 64)], hi = ring[(o + ol + 1) % (rs * 64)];
                const u64 keep = k <= 65 ? ~0ull : 0ull;
                acc |= (ring[o + lane] ^ (sh ? ((lo >> sh) | (hi << (64 - sh))) : lo)) & keep;
            }
        }
        if (P && !__ballot(acc != 0)) {
            mreg = (lane >= k0 && lane < k0 + RM_CH) ? P : mreg;
            if (k0 == 64) m64 = m65 = P;
            return;
        }
        pure = false;
        for (u32 j = 0; j < RM_CH; j++) {
            const u32 k = k0 + j;
            if (k > 65) break;
            const u32 o = (k % rs) * 64;
            const u64 x = ring[o + lane];
            u64 d = ~0ull;
            if (P) {
                const u64 lo = ring[(o + ol) % (rs * 64)], hi = ring[(o + ol + 1) % (rs * 64)];
                d = x ^ (sh ? ((lo >> sh) | (hi << (64 - sh))) : lo);
            }
            u32 mk = P;
            if (__ballot(d != 0)) {
                mk = 0;
                if (nsearch < 8) {  // a run of another period, or none (bounded searches per stripe)
                    nsearch++;
                    const u32 P2 = smallest_period(x, ring[((k + 1) % rs) * 64 + lane], lane);
                    if (P2) {
                        P = mk = P2;
                        ol = lane + (P >> 3);
                        sh = 8 * (P & 7);
                    }
                }
            }
            put(k, mk);
        }
    };
    load_to(A, 0);
    load_to(B, RM_CH);
    store_from(A, 0);
    load_to(A, 2 * RM_CH);
    __builtin_amdgcn_wave_barrier();
    // the period of block 1 (blocks 1, 2 in the ring)
    P0 = P = smallest_period(ring[64 + lane], ring[128 + lane], lane);
    pure = P0 != 0;
    ol = lane + (P >> 3);
    sh = 8 * (P & 7);
    // step c: chunk c into the ring, chunk c + 16 loading, chunk c - 8 checked (blocks 0 .. 65; the
    // steps are unconditional -- a skipped store leaves a loading register to be overwritten, and
    // the compiler then drains every load -- so chunks up to 80 are stored and loads reach block
    // 103, inside the text pad for every stripe but the last)
    for (u32 c = RM_CH; c <= 72; c += 2 * RM_CH) {
        store_from(B, c);
        load_to(B, c + 2 * RM_CH);
        __builtin_amdgcn_wave_barrier();
        check(c - RM_CH);
        store_from(A, c + RM_CH);
        load_to(A, c + 3 * RM_CH);
        __builtin_amdgcn_wave_barrier();
        check(c);
    }
    return pure ? P0 : 0u;
}


template <u32 RSLX, int WPG>
__global__ __launch_bounds__(64 * WPG) void k_scan_only(const unsigned char* __restrict__ T, u64 nstripes,
                                                        const u64* __restrict__ hitw, u32* __restrict__ out) {
    __shared__ u64 s_ring[WPG][RSLX * 64];
    const u32 lane = threadIdx.x & 63;
    u64* ring = s_ring[threadIdx.x >> 6];
    const u64 w = (u64)blockIdx.x * WPG + (u32)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    if (w + 1 >= nstripes) return;
    if (!(hitw[3 * w + 2] >> 63)) return;
    u32 mp = 0, m64 = 0, m65 = 0;
    const u32 P0 = run_scan(T + w * 32768ull + 8 * lane, ring, RSLX, lane, mp, m64, m65);
    if (lane == 0 && (P0 == 0x12345 || m64 == 0x12345)) out[3] = mp;
    if (P0 && lane == 0) out[16 + (w & 1023)] = P0;
}

// run_scan with its parts switched: PS period search (else P = 2), MAP map recording, SLOW the
// per-block path on a dirty chunk (else exit), BUF 1 = two named buffers + sched barriers, 0 = R[2]
// with copies (k_cross2's form)
template <bool PS, bool MAP, bool SLOW, int BUF>
__device__ __forceinline__ u32 run_scan_t(const u8* __restrict__ Tw, u64* __restrict__ ring, u32 lane, u32& mreg,
                                          u32& m64, u32& m65) {
    constexpr u32 rs = 16;
    auto load8 = [&](u32 k) -> u64 { return *(const u64*)(Tw + (u64)k * TAU); };
    u32 P0 = 0, P = 2, ol = lane, sh = 16, nsearch = 0;
    bool pure = true, stop = false;
    auto put = [&](u32 k, u32 m) {
        if (k < 64) mreg = lane == k ? m : mreg;
        else if (k == 64) m64 = m;
        else m65 = m;
    };
    auto check = [&](u32 k0) {
        u64 acc = 0;
#pragma unroll
        for (u32 j = 0; j < RM_CH; j++) {
            const u32 k = k0 + j, o = (k % rs) * 64;
            const u64 lo = ring[(o + ol) % (rs * 64)], hi = ring[(o + ol + 1) % (rs * 64)];
            const u64 keep = k <= 65 ? ~0ull : 0ull;
            acc |= (ring[o + lane] ^ (sh ? ((lo >> sh) | (hi << (64 - sh))) : lo)) & keep;
        }
        if (!__ballot(acc != 0)) {
            if (MAP) {
                mreg = (lane >= k0 && lane < k0 + RM_CH) ? P : mreg;
                if (k0 == 64) m64 = m65 = P;
            }
            return;
        }
        pure = false;
        if (!SLOW) { stop = true; return; }
        for (u32 j = 0; j < RM_CH; j++) {
            const u32 k = k0 + j;
            if (k > 65) break;
            const u32 o = (k % rs) * 64;
            const u64 x = ring[o + lane];
            const u64 lo = ring[(o + ol) % (rs * 64)], hi = ring[(o + ol + 1) % (rs * 64)];
            const u64 d = x ^ (sh ? ((lo >> sh) | (hi << (64 - sh))) : lo);
            u32 mk = P;
            if (__ballot(d != 0)) {
                mk = 0;
                if (nsearch < 8) {
                    nsearch++;
                    const u32 P2 = smallest_period(x, ring[((k + 1) % rs) * 64 + lane], lane);
                    if (P2) {
                        P = mk = P2;
                        ol = lane + (P >> 3);
                        sh = 8 * (P & 7);
                    }
                }
            }
            put(k, mk);
        }
    };
    if (BUF == 1) {
        u64 A[RM_CH], B[RM_CH];
        auto load_to = [&](u64* X, u32 k0) {
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (u32 e = 0; e < RM_CH; e++) X[e] = load8(k0 + e);
            __builtin_amdgcn_sched_barrier(0);
        };
        auto store_from = [&](const u64* X, u32 k0) {
#pragma unroll
            for (u32 e = 0; e < RM_CH; e++) ring[((k0 + e) % rs) * 64 + lane] = X[e];
        };
        load_to(A, 0);
        load_to(B, RM_CH);
        store_from(A, 0);
        load_to(A, 2 * RM_CH);
        __builtin_amdgcn_wave_barrier();
        if (PS) {
            P0 = P = smallest_period(ring[64 + lane], ring[128 + lane], lane);
            ol = lane + (P >> 3);
            sh = 8 * (P & 7);
            if (!P) return 0;
        } else P0 = 2;
        for (u32 c = RM_CH; c <= 72; c += 2 * RM_CH) {
            store_from(B, c);
            load_to(B, c + 2 * RM_CH);
            __builtin_amdgcn_wave_barrier();
            check(c - RM_CH);
            if (stop) return 0;
            store_from(A, c + RM_CH);
            load_to(A, c + 3 * RM_CH);
            __builtin_amdgcn_wave_barrier();
            check(c);
            if (stop) return 0;
        }
    } else {
        u64 R[2][RM_CH];
#pragma unroll
        for (u32 d = 0; d < 2; d++)
#pragma unroll
            for (u32 e = 0; e < RM_CH; e++) R[d][e] = load8(d * RM_CH + e);
        for (u32 c = 0; c < 66 + RM_CH; c += RM_CH) {
#pragma unroll
            for (u32 e = 0; e < RM_CH; e++) ring[((c + e) % rs) * 64 + lane] = R[0][e];
#pragma unroll
            for (u32 e = 0; e < RM_CH; e++) R[0][e] = R[1][e];
#pragma unroll
            for (u32 e = 0; e < RM_CH; e++) R[1][e] = load8(c + 2 * RM_CH + e);
            __builtin_amdgcn_wave_barrier();
            if (c == 0) {
                if (PS) {
                    P0 = P = smallest_period(ring[64 + lane], ring[128 + lane], lane);
                    ol = lane + (P >> 3);
                    sh = 8 * (P & 7);
                    if (!P) return 0;
                } else P0 = 2;
                continue;
            }
            check(c - RM_CH);
            if (stop) return 0;
        }
    }
    return pure ? P0 : 0u;
}
template <bool PS, bool MAP, bool SLOW, int BUF>
__global__ __launch_bounds__(256) void k_scan_t(const unsigned char* __restrict__ T, u64 nstripes,
                                                const u64* __restrict__ hitw, u32* __restrict__ out) {
    __shared__ u64 s_ring[4][16 * 64];
    const u32 lane = threadIdx.x & 63;
    u64* ring = s_ring[threadIdx.x >> 6];
    const u64 w = (u64)blockIdx.x * 4 + (u32)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    if (w + 1 >= nstripes) return;
    if (!(hitw[3 * w + 2] >> 63)) return;
    u32 mp = 0, m64 = 0, m65 = 0;
    const u32 P0 = run_scan_t<PS, MAP, SLOW, BUF>(T + w * 32768ull + 8 * lane, ring, lane, mp, m64, m65);
    if (lane == 0 && (P0 == 0x12345 || m64 == 0x12345)) out[3] = mp;
    if (P0 && lane == 0) out[16 + (w & 1023)] = P0;
}

// cross2 grown step by step toward run_scan: PSX period search at the first chunk, MAPX map entries
// in the fast path, SLOWX per-block path on a dirty chunk, FUN branch-free funnel shift
template <bool PSX, bool MAPX, bool SLOWX, bool FUN>
__global__ __launch_bounds__(256) void k_grow(const unsigned char* __restrict__ T, u64 nstripes,
                                              const u64* __restrict__ hitw, u32* __restrict__ out) {
    constexpr u32 CH = 8, RS = 16, DEPTH = 2, NCHK = 66;
    __shared__ u64 s_ring[4][RS * 64];
    const u32 lane = threadIdx.x & 63;
    u64* ring = s_ring[threadIdx.x >> 6];
    const u64 w = (u64)blockIdx.x * 4 + (u32)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    if (w + 1 >= nstripes) return;
    if (!(hitw[3 * w + 2] >> 63)) return;
    const u64 b0 = w * 64;
    auto load8 = [&](u64 k) -> u64 { return *(const u64*)(T + (b0 + k) * 512 + 8 * lane); };
    u64 R[DEPTH][CH];
#pragma unroll
    for (u32 d = 0; d < DEPTH; d++)
#pragma unroll
        for (u32 e = 0; e < CH; e++) R[d][e] = load8(d * CH + e);
    u32 p = 2, P0 = 2, nsearch = 0, mreg = 0, m64 = 0, m65 = 0;
    bool pure = true;
    u32 ol = lane + (p >> 3), sh = 8 * (p & 7);
    auto shifted = [&](u64 lo, u64 hi) -> u64 {
        if (FUN) return (lo >> sh) | ((hi << 1) << (63 - sh));
        return sh ? ((lo >> sh) | (hi << (64 - sh))) : lo;
    };
    for (u32 c = 0; c < NCHK + CH; c += CH) {
#pragma unroll
        for (u32 e = 0; e < CH; e++) ring[((c + e) % RS) * 64 + lane] = R[0][e];
#pragma unroll
        for (u32 d = 0; d + 1 < DEPTH; d++)
#pragma unroll
            for (u32 e = 0; e < CH; e++) R[d][e] = R[d + 1][e];
#pragma unroll
        for (u32 e = 0; e < CH; e++) R[DEPTH - 1][e] = load8(c + DEPTH * CH + e);
        __builtin_amdgcn_wave_barrier();
        if (c == 0) {
            if (PSX) {
                P0 = p = smallest_period(ring[64 + lane], ring[128 + lane], lane);
                if (!p) return;
                ol = lane + (p >> 3);
                sh = 8 * (p & 7);
            }
            continue;
        }
        u64 acc = 0;
        const u32 k0 = c - CH;
#pragma unroll
        for (u32 j = 0; j < CH; j++) {
            const u32 k = k0 + j;
            if (k >= NCHK) break;
            const u32 o = (k % RS) * 64;
            const u64 lo = ring[(o + ol) % (RS * 64)], hi = ring[(o + ol + 1) % (RS * 64)];
            acc |= ring[o + lane] ^ shifted(lo, hi);
        }
        if (__ballot(acc != 0)) {
            pure = false;
            if (!SLOWX) return;
            for (u32 j = 0; j < CH; j++) {
                const u32 k = k0 + j;
                if (k >= NCHK) break;
                const u32 o = (k % RS) * 64;
                const u64 x = ring[o + lane];
                const u64 lo = ring[(o + ol) % (RS * 64)], hi = ring[(o + ol + 1) % (RS * 64)];
                u32 mk = p;
                if (__ballot((x ^ shifted(lo, hi)) != 0)) {
                    mk = 0;
                    if (nsearch < 8) {
                        nsearch++;
                        const u32 P2 = smallest_period(x, ring[((k + 1) % RS) * 64 + lane], lane);
                        if (P2) {
                            p = mk = P2;
                            ol = lane + (p >> 3);
                            sh = 8 * (p & 7);
                        }
                    }
                }
                if (k < 64) mreg = lane == k ? mk : mreg;
                else if (k == 64) m64 = mk;
                else m65 = mk;
            }
        } else if (MAPX) {
            mreg = (lane >= k0 && lane < k0 + CH) ? p : mreg;
            if (k0 == 64) m64 = m65 = p;
        }
    }
    if (lane == 0 && (m64 == 0x12345 || m65 == 0x12345)) out[3] = mreg;
    if (pure && lane == 0) out[16 + (w & 1023)] = P0;  // (no same-address atomics: they serialize)
}

int main() {
    const u64 n = 1ull << 30, pad = 1 << 20;
    std::vector<unsigned char> h(n + pad, 0);
    // period-1 runs of 100 000 bytes, a fresh byte each
    for (u64 i = 0; i < n; i++) h[i] = (unsigned char)(1 + (i / 100000) % 251);
    unsigned char* d;
    u32* out;
    CK(hipMalloc(&d, n + pad));
    CK(hipMalloc(&out, 8192));
    CK(hipMemcpy(d, h.data(), n + pad, hipMemcpyHostToDevice));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    auto timeit = [&](const char* name, auto launch) {
        for (int r = 0; r < 3; r++) launch();
        CK(hipEventRecord(a));
        const int R = 10;
        for (int r = 0; r < R; r++) launch();
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        ms /= R;
        printf("%-44s %8.1f us  %6.2f TB/s\n", name, ms * 1e3, n / (ms * 1e-3) / 1e12);
        return 0;
    };
    const u64 n16 = n / 16;
    for (u64 per : {2048ull, 8192ull, 32768ull}) {
        const u64 waves = (n16 + per - 1) / per;
        char nm[64];
        snprintf(nm, 64, "read x4 per_wave=%llu B", (unsigned long long)per * 16);
        timeit(nm, [&] { k_read<4><<<(unsigned)((waves + 3) / 4), 256>>>((const uint4*)d, n16, per, out); });
    }
    const u64 nbt = n / 512;
#define CROSS(NB, CH, RS, DEPTH)                                                                           \
    timeit("cross NB=" #NB " CH=" #CH " RS=" #RS " DEPTH=" #DEPTH, [&] {                                   \
        k_cross<NB, CH, RS, DEPTH><<<(unsigned)((nbt / NB + 3) / 4), 256>>>(d, nbt, 1, out);              \
    });
    CROSS(64, 8, 16, 1)
    CROSS(64, 8, 16, 2)
    CROSS(64, 8, 16, 3)
    CROSS(256, 8, 16, 1)
    CROSS(256, 8, 16, 2)
    CROSS(64, 4, 8, 2)
    CROSS(64, 4, 8, 4)
    CROSS(256, 4, 8, 4)
    CROSS(64, 16, 32, 1)
    // the rr text (random_repetitive_string(2^30), knobs 0.5 / 0.05, seed 42): period-2 runs
    if (lz77sss_gen_random_repetitive((u32)n, (u32)n, 42, 0.5, 0.05, h.data(), n) != (int64_t)n) return 1;
    CK(hipMemcpy(d, h.data(), n, hipMemcpyHostToDevice));
    const u64 ns = (n - 1024) / 32768 + 1;
    std::vector<u64> hw(3 * ns, 1ull << 63);
    u64* dhw;
    CK(hipMalloc(&dhw, 24 * ns));
    CK(hipMemcpy(dhw, hw.data(), 24 * ns, hipMemcpyHostToDevice));
    printf("-- rr text\n");
    timeit("cross p=2 NB=64 CH=8 RS=16 DEPTH=2 (rr)", [&] { k_cross<64, 8, 16, 2><<<(unsigned)((nbt / 64 + 3) / 4), 256>>>(d, nbt, 2, out); });
#define PURE(H, PS, EX) timeit("pure_like hstate=" #H " psearch=" #PS " exit=" #EX, [&] { k_pure_like<H, PS, EX><<<(unsigned)((ns + 3) / 4), 256>>>(d, ns, dhw, out); });
    PURE(false, false, false)
    PURE(true, false, false)
    PURE(false, true, false)
    PURE(false, false, true)
    PURE(true, true, true)
#define V1(PS, HW, WPG) timeit("pure_v1 psearch=" #PS " hitw=" #HW " wpg=" #WPG, [&] { k_pure_v1<PS, HW, WPG><<<(unsigned)((ns + WPG - 1) / WPG), 64 * WPG>>>(d, ns, dhw, out); });
    V1(true, true, 4)
    V1(false, true, 4)
    V1(true, false, 4)
    V1(false, false, 4)
    V1(true, true, 1)
    V1(true, true, 2)
    timeit("cross p=2 NB=64 CH=8 RS=16 DEPTH=2 (rr, again)", [&] { k_cross<64, 8, 16, 2><<<(unsigned)((nbt / 64 + 3) / 4), 256>>>(d, nbt, 2, out); });
#define C2(EX, HW, PAD, NC) timeit("cross2 exit=" #EX " hitw=" #HW " pad=" #PAD " nchk=" #NC, [&] { k_cross2<EX, HW, PAD, NC><<<(unsigned)((ns + 3) / 4), 256>>>(d, ns, 2, dhw, out); });
    C2(false, false, 0, 64)
    C2(true, false, 0, 64)
    C2(false, true, 0, 64)
    C2(false, false, 4, 64)
    C2(false, false, 0, 66)
    C2(true, true, 0, 66)
    timeit("scan_only rs=16 wpg=4", [&] { k_scan_only<16, 4><<<(unsigned)((ns + 3) / 4), 256>>>(d, ns, dhw, out); });
    timeit("scan_only rs=16 wpg=1", [&] { k_scan_only<16, 1><<<(unsigned)ns, 64>>>(d, ns, dhw, out); });
    timeit("cross2 exit hitw 66 (again)", [&] { k_cross2<true, true, 0, 66><<<(unsigned)((ns + 3) / 4), 256>>>(d, ns, 2, dhw, out); });
#define ST(PS, MAP, SLOW, BUF) timeit("scan_t ps=" #PS " map=" #MAP " slow=" #SLOW " buf=" #BUF, [&] { k_scan_t<PS, MAP, SLOW, BUF><<<(unsigned)((ns + 3) / 4), 256>>>(d, ns, dhw, out); });
    ST(false, false, false, 0)
    ST(false, false, false, 1)
    ST(true, false, false, 0)
    ST(false, true, false, 0)
    ST(false, false, true, 0)
    ST(true, true, true, 0)
    ST(true, true, true, 1)
#define GR(A, B, C, D) timeit("grow ps=" #A " map=" #B " slow=" #C " fun=" #D, [&] { k_grow<A, B, C, D><<<(unsigned)((ns + 3) / 4), 256>>>(d, ns, dhw, out); });
    GR(false, false, false, false)
    GR(true, false, false, false)
    GR(true, true, false, false)
    GR(true, true, true, false)
    GR(true, true, true, true)
    GR(false, false, false, true)
    return 0;
}
