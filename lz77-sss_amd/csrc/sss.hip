// sss.hip -- kernel 1: the tau-synchronizing set (role of
// lce::rolling_hash::sss<pos_t,tau>, called at
// patched-files/external/lce/include/ds/lce_sss.hpp:53; its source is absent
// upstream, the definition pinned here is DESIGN.md section 4.1):
//
//   Phi(j)  = KR fingerprint of T[j..j+tau) mod 2^31-1 (base SSS_BASE)
//   Q       = { j : T[j..j+tau) has a period <= floor(tau/3) }
//   S       = { i <= n-2tau : min Phi'[i..i+tau] < inf at i or at i+tau }
//
// Launches:
//   k_q_anchors  -- per anchor a (every 128 positions) the smallest period <= 170
//                   of T[a..a+340), the Q interval it induces on (a-128, a], and
//                   the local extent of the periodic run (run table, lce_dev.h)
//   k_run_elems + 2 scans + k_run_finish -- exact run ends/starts along chains
//   k_sss_stream -- one wave per stripe of 16384 decisions, walked in 512-blocks
//                   with bytes, prefix hashes and Phi' in registers: lane Horner +
//                   wave scan, 7 rolls per lane, van Herk minima by lane-local
//                   and wave scans, ordered per-stripe output
//   k_sss_fallback -- exact slow path for stripes with more than SCAP outputs
//   k_sss_compact-- per-stripe outputs -> sorted S
#include "../include/engine.h"

#include <hipcub/hipcub.hpp>


namespace lz {

// ---------------------------------------------------------------------------
// Q anchors.  A workgroup of 256 lanes covers anchors tb-1 .. tb+254 (lane i ->
// anchor tb-1+i) and owns tb .. tb+252; the three halo anchors give the owned
// ones their neighbours' periods.  Text [a(tb-1) - 256, a(tb+254) + 1024) is
// staged in LDS.
constexpr int QT_THREADS = 256;
constexpr int QT_OWN = QT_THREADS - 3;                  // owned anchors per workgroup
constexpr int QT_LDS = QT_THREADS * (int)QA + 256 + 1024;
constexpr u32 RUN_HCAP = 640;                           // local run extension: [a-256, a+640)
constexpr u32 RUN_LCAP = 256;

__global__ __launch_bounds__(QT_THREADS) void k_q_anchors(const u8* __restrict__ T, u64 n, u64 nanch,
                                                          u16* __restrict__ qinfo, u32* __restrict__ any_q,
                                                          u8* __restrict__ run_p, u32* __restrict__ run_hi,
                                                          u32* __restrict__ run_lo, u8* __restrict__ run_cap) {
    // LDS text with one pad word per 128 bytes: the anchors of a wave sit 128 bytes
    // apart, so unpadded their accesses would all hit the same bank
    __shared__ __attribute__((aligned(16))) u32 b32[QT_LDS / 4 + QT_LDS / 128 + 2];
    __shared__ u8 s_p1[QT_THREADS], s_c[QT_THREADS], s_p[QT_THREADS];
    __shared__ u32 s_anyq;
    const int i = (int)threadIdx.x;
    const int64_t tb = (int64_t)blockIdx.x * QT_OWN;
    const int64_t base = (tb - 1) * (int64_t)QA - 256;  // LDS offset 0
    {
        // all global loads first (one round trip), then the LDS writes.  Loads are
        // unconditional: out-of-range lanes read the zero padding at T + n (a guarded
        // or zeroed load becomes a branch with its own s_waitcnt)
        constexpr int NL = (QT_THREADS * (int)QA) / (QT_THREADS * 16);  // 8 full rounds
        constexpr int TAIL = QT_LDS - NL * QT_THREADS * 16;              // 1280 bytes
        static_assert(TAIL > 0 && TAIL <= QT_THREADS * 16, "one tail round");
        auto src = [&](int x) -> const uint4* {
            const int64_t g = base + x;
            const bool okr = g >= 0 && (u64)g + 16 <= n + TEXT_PAD;
            return (const uint4*)(T + (okr ? (u64)g : n));
        };
        uint4 v[NL + 1];
#pragma unroll
        for (int r = 0; r < NL; r++) v[r] = *src(i * 16 + r * QT_THREADS * 16);
        v[NL] = *src(i * 16 < TAIL ? NL * QT_THREADS * 16 + i * 16 : -(1 << 20));
        auto put = [&](int x, uint4 q) {
            const int w = (x >> 2) + (x >> 7);
            b32[w] = q.x;
            b32[w + 1] = q.y;
            b32[w + 2] = q.z;
            b32[w + 3] = q.w;
        };
#pragma unroll
        for (int r = 0; r < NL; r++) put(i * 16 + r * QT_THREADS * 16, v[r]);
        if (i * 16 < TAIL) put(NL * QT_THREADS * 16 + i * 16, v[NL]);
    }
    if (i == 0) s_anyq = 0;
    __syncthreads();
    // LDS accessors on offsets o = position - base
    auto word = [&](int w) -> u32 { return b32[w + (w >> 5)]; };
    auto byte = [&](int o) -> u32 { return (word(o >> 2) >> (8 * (o & 3))) & 255u; };
    // first o in [h, cap) with T[o] != T[o+p] (cap if none)
    auto ext_fwd = [&](int h, int cap, int p) -> int {
        for (; h < cap && (h & 3); h++)
            if (byte(h) != byte(h + p)) return h;
        int q = (h + p) >> 2;
        const u32 sh = (u32)((h + p) & 3);
        u32 lo = word(q);
        for (; h < cap; h += 4) {
            const u32 hi = word(q + 1);
            u32 d = word(h >> 2) ^ __builtin_amdgcn_alignbyte(hi, lo, sh);
            const int rem = cap - h;
            if (rem < 4) d &= (1u << (8 * rem)) - 1;
            if (d) return h + (__builtin_ctz(d) >> 3);
            lo = hi;
            q++;
        }
        return cap;
    };
    // smallest l' in [cap, l] with T[o] == T[o+p] for all o in [l', l)
    auto ext_bwd = [&](int l, int cap, int p) -> int {
        for (; l > cap && (l & 3); l--)
            if (byte(l - 1) != byte(l - 1 + p)) return l;
        if (l >= cap + 4) {
            int q = (l - 4 + p) >> 2;
            const u32 sh = (u32)((l + p) & 3);
            u32 hi = word(q + 1);
            for (; l >= cap + 4; l -= 4) {
                const u32 lo = word(q);
                const u32 d = word((l - 4) >> 2) ^ __builtin_amdgcn_alignbyte(hi, lo, sh);
                if (d) return l - 4 + ((31 - __builtin_clz(d)) >> 3) + 1;
                hi = lo;
                q--;
            }
        }
        for (; l > cap && byte(l - 1) == byte(l - 1 + p); l--) {
        }
        return l;
    };

    // ---- 1. candidate periods of the probe T[a..a+340): a 4-byte filter (fully
    // unrolled: mask word and bit of each candidate are compile-time constants)
    const int64_t t = tb - 1 + i;
    const int oa = i * (int)QA + 256;  // LDS offset of the anchor
    const u64 a = (u64)t * QA;
    const bool probe_ok = t >= 0 && (u64)t < nanch && a + QM <= n;
    u32 cm[6] = {0, 0, 0, 0, 0, 0};  // bit pp-1
    if (probe_ok) {
        const u32 w0 = word(oa >> 2);
        u32 dprev = w0;
#pragma unroll
        for (int k = 0; k <= (int)(QL / 4); k++) {
            const u32 dnext = word((oa >> 2) + k + 1);
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const u32 pp = 4 * k + r;
                if (pp >= 1 && pp <= QL && __builtin_amdgcn_alignbyte(dnext, dprev, r) == w0)
                    cm[(pp - 1) >> 5] |= 1u << ((pp - 1) & 31);
            }
            dprev = dnext;
        }
    }
    u32 p1 = 0;
    for (int wi = 0; wi < 6 && !p1; wi++)
        if (cm[wi]) p1 = 32 * wi + __builtin_ctz(cm[wi]) + 1;
    // ---- 2. shift-p1 agreement over the anchor's own 128 bytes; a probe that
    // agrees over its whole chunk is verified from its two successors' chunks
    // when they test the same shift (inside a run: every anchor), so each byte
    // of a run is compared about once instead of 340/128 times
    const int c = p1 ? ext_fwd(oa, oa + (int)QA, (int)p1) - oa : 0;
    s_p1[i] = (u8)p1;
    s_c[i] = (u8)c;
    __syncthreads();
    u32 per = 0;
    if (p1) {
        const int need = (int)(QM - p1);  // bytes of the probe that must agree with shift p1
        int f = -1;                       // first disagreement of shift p1 (offset from a), -1: none
        if (c < min(need, (int)QA)) {
            f = c;
        } else {
            const bool s1 = i + 1 < QT_THREADS && s_p1[i + 1] == p1;
            const bool s2 = need <= 2 * (int)QA || (i + 2 < QT_THREADS && s_p1[i + 2] == p1);
            if (s1 && s2) {
                if (s_c[i + 1] < min(need - (int)QA, (int)QA)) f = (int)QA + s_c[i + 1];
                else if (need > 2 * (int)QA && s_c[i + 2] < need - 2 * (int)QA) f = 2 * (int)QA + s_c[i + 2];
            } else {
                const int e = ext_fwd(oa + (int)QA, oa + need, (int)p1);
                if (e < oa + need) f = e - oa;
            }
        }
        if (f < 0) {
            per = p1;
        } else {
            // p1 is the smallest candidate and T[a..a+f+p1) has period p1, so by
            // Fine-Wilf a period pp <= f of the probe would share gcd(p1, pp) = p1
            // with it, and every multiple of p1 up to f disagrees at f - pp + p1:
            // only candidates pp > f remain (at run ends this skips ~85 full checks)
            cm[(p1 - 1) >> 5] &= ~(1u << ((p1 - 1) & 31));
            for (int wi = 0; wi < 6; wi++) {
                const int lo = 32 * wi + 1;  // candidate of bit 0
                if (f + 1 >= lo + 32) cm[wi] = 0;
                else if (f + 1 > lo) cm[wi] &= ~0u << (f + 1 - lo);
            }
            for (int wi = 0; wi < 6 && !per;) {
                if (!cm[wi]) {
                    wi++;
                    continue;
                }
                const u32 pp = 32 * wi + __builtin_ctz(cm[wi]) + 1;
                if (ext_fwd(oa + 4, oa + (int)(QM - pp), (int)pp) == oa + (int)(QM - pp)) per = pp;
                cm[wi] &= cm[wi] - 1;
            }
        }
    }
    s_p[i] = (u8)per;
    __syncthreads();

    // ---- 3. owned anchors: Q interval on (a-128, a] and the local run extent
    if (i >= 1 && i <= QT_OWN && (u64)t < nanch) {
        u16 res = 0xFF00;  // empty interval
        u32 rp = 0, rhi = 0, rlo = 0;
        u8 rcap = 0;
        const u32 p = per;
        if (p) {
            // neighbours with the same period: their windows overlap this one by >= 212 >= p
            // bytes, so the union is p-periodic and the extensions are known without scanning
            const bool contb = s_p[i - 1] == p, contf = s_p[i + 1] == p;
            const bool contf2 = contf && s_p[i + 2] == p;
            const u64 hi_cap = min(a + TAU - p, n - p), lo_cap = a >= 127 ? a - 127 : 0;
            const int o_hicap = (int)((int64_t)hi_cap - base), o_locap = (int)((int64_t)lo_cap - base);
            const int o_hi = contf2 ? o_hicap : ext_fwd(oa + (int)(QM - p), o_hicap, (int)p);
            const int o_lo = contb ? o_locap : ext_bwd(oa, o_locap, (int)p);
            const u64 hi = (u64)(base + o_hi), lo = (u64)(base + o_lo);
            // Q on (a-128, a]: j >= lo, j + tau - p <= hi, j <= n - tau
            const int64_t jlo = (int64_t)lo;
            int64_t jhi = min((int64_t)a, (int64_t)hi + (int64_t)p - (int64_t)TAU);
            jhi = min(jhi, (int64_t)n - (int64_t)TAU);
            if (jlo <= jhi) {
                const int64_t r0 = (int64_t)a - 127;  // rel(j) = j - r0 in [0,127]
                res = (u16)(((jlo - r0) << 8) | (jhi - r0));
                s_anyq = 1;
            }
            // local extent of the p-periodic run around the window (for run-skipping LCE);
            // inside a chain of same-period anchors the values only need to mark the chain
            rp = p;
            if (contf) {
                rhi = (u32)(a + RUN_HCAP);
                rcap |= 1;
            } else {
                const u64 h2_cap = min(a + RUN_HCAP - p, n - p);
                const u64 h2 = hi < hi_cap ? hi : (u64)(base + ext_fwd(o_hi, (int)((int64_t)h2_cap - base), (int)p));
                rhi = (u32)(h2 + p);
                rcap |= h2 == a + RUN_HCAP - p ? 1 : 0;
            }
            if (contb) {
                rlo = (u32)(a >= RUN_LCAP ? a - RUN_LCAP : a - QA);
                rcap |= 2;
            } else {
                const u64 l2_cap = a >= RUN_LCAP ? a - RUN_LCAP : 0;
                const u64 l2 = (lo > lo_cap) ? lo : (u64)(base + ext_bwd(o_lo, (int)((int64_t)l2_cap - base), (int)p));
                rlo = (u32)l2;
                rcap |= (l2 == a - RUN_LCAP && a >= RUN_LCAP) ? 2 : 0;
            }
        }
        qinfo[t] = res;
        run_p[t] = (u8)rp;
        run_hi[t] = rhi;
        run_lo[t] = rlo;
        run_cap[t] = rcap;
    }
    __syncthreads();
    // one atomic per block: same-address atomics from every anchor serialize
    if (i == 0 && s_anyq) atomicOr(any_q, 1u);
}

// run chains: anchor t continues into t+1 (same run) when both have period p
// and t's run covers t+1's window; a chain's exact hi is its last anchor's local
// hi (exact unless capped), its exact lo its first anchor's local lo.
__global__ void k_run_elems(const u8* __restrict__ rp, const u32* __restrict__ rhi, const u32* __restrict__ rlo,
                            const u8* __restrict__ rcap, u64 na, u64* __restrict__ ehi_rev, u64* __restrict__ elo) {
    const u64 t = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= na) return;
    const u32 p = rp[t];
    const u64 a = t * QA;
    const bool cont_f = p && t + 1 < na && rp[t + 1] == p && (u64)rhi[t] >= a + QA + QM;
    const bool cont_b = p && t >= 1 && rp[t - 1] == p && (u64)rlo[t] + QA <= a;
    u64 vh = 0, vl = 0xFFFFFFFFull;
    if (p) {
        vh = (!cont_f && (rcap[t] & 1)) ? 0 : rhi[t];
        vl = (!cont_b && (rcap[t] & 2)) ? 0xFFFFFFFFull : rlo[t];
    }
    ehi_rev[na - 1 - t] = ((u64)(!cont_f) << 63) | vh;
    elo[t] = ((u64)(!cont_b) << 63) | vl;
}
struct last_marked {
    __device__ __forceinline__ u64 operator()(const u64& x, const u64& y) const { return (y >> 63) ? y : x; }
};
__global__ void k_run_finish(const u64* __restrict__ shi_rev, const u64* __restrict__ slo, u64 na,
                             u32* __restrict__ rhi, u32* __restrict__ rlo) {
    const u64 t = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= na) return;
    rhi[t] = (u32)shi_rev[na - 1 - t];
    rlo[t] = (u32)slo[t];
}

// canonical x mod (2^31 - 1) for x < 2^63
__device__ __forceinline__ u32 red31(u64 x) {
    u64 r = (x & P31) + (x >> 31);
    r = (r & P31) + (r >> 31);
    return (u32)(r >= P31 ? r - P31 : r);
}
__device__ __forceinline__ u32 mulmod31(u32 a, u32 c) { return red31((u64)a * c); }
// canonical x mod (2^31 - 1) for x < 2^51 (one fold: the high part fits 20 bits)
__device__ __forceinline__ u32 red31s(u64 x) {
    const u32 lo = (u32)x, hi = (u32)(x >> 32);
    const u32 r = (lo & (u32)P31) + __builtin_amdgcn_alignbit(hi, lo, 31);
    return r >= (u32)P31 ? r - (u32)P31 : r;
}

// ---------------------------------------------------------------------------
// main pass, streaming form: one wave per stripe of SD = 32 x 512 decisions,
// walked block by block with everything in registers (no LDS, no barriers).
// Lane L owns positions s_k + 8L .. s_k + 8L + 7 of every 512-block k.
//
//   bytes   8 per lane and block (one coalesced 512-byte load per wave),
//           prefetched two blocks ahead
//   hashes  H(s_k + 8L) (prefix hash relative to the stripe start) from a
//           lane Horner over 8 bytes + a 6-step wave scan of affine maps;
//           Phi(s_k + 8L) = H(s_k+1 + 8L) - H(s_k + 8L) * b^512, then 7 rolls
//   minima  van Herk / Gil-Werman with 512-blocks: for decision block c the
//           wave holds Phi'(block c) and Phi'(block c+1) in registers;
//           m_i = min(suffix_c, prefix_c+1) from lane-local scans + wave scans
//   output  i in S  <=>  m_i < inf and (Phi'(i) == m_i or Phi'(i+512) == m_i),
//           ordered per stripe (capacity SCAP, exact fallback beyond)
constexpr int SNB = 32;                       // decision blocks per stripe
constexpr int SD = SNB * (int)TAU;            // decisions per stripe (16384)
constexpr int SCAP = 512;                     // sync positions per stripe before the fallback
constexpr int SWAVES = 4;                     // independent waves per workgroup

struct sss_pow2 {
    u32 pw8[8];    // b^(7 - e)
    u32 b8, ib8;   // b^8 and its inverse mod P31
    u32 b512;      // b^512 = b^tau
    u32 bn;        // P - b^tau
};

// canonical x mod (2^31 - 1) for x < 2^32
__device__ __forceinline__ u32 canon31(u32 r) { return min(r, r - (u32)P31); }
// < 2^32 and congruent to x mod P31, for x < 2^62; canon31 of it is canonical
// (a fold of a product of two canonical values never reaches 2 P31)
__device__ __forceinline__ u32 fold31(u64 x) {
    return ((u32)x & (u32)P31) + __builtin_amdgcn_alignbit((u32)(x >> 32), (u32)x, 31);
}
__device__ __forceinline__ u32 mm31(u32 a, u32 c) { return canon31(fold31((u64)a * c)); }
__device__ __forceinline__ u32 addm31(u32 a, u32 c) { return canon31(a + c); }
__device__ __forceinline__ u32 subm31(u32 a, u32 c) { return canon31(a + (u32)P31 - c); }

// wave scans by DPP (gfx9 row shifts + row broadcasts; no LDS round trips)
template <int CTRL, int ROWM = 0xF>
__device__ __forceinline__ u32 dpp(u32 old, u32 v) {
    return (u32)__builtin_amdgcn_update_dpp((int)old, (int)v, CTRL, ROWM, 0xF, false);
}
__device__ __forceinline__ u32 wave_prefix_min(u32 v) {  // inclusive, over lanes <= L
    v = min(v, dpp<0x111>(INF32, v));
    v = min(v, dpp<0x112>(INF32, v));
    v = min(v, dpp<0x114>(INF32, v));
    v = min(v, dpp<0x118>(INF32, v));
    v = min(v, dpp<0x142, 0xA>(INF32, v));
    v = min(v, dpp<0x143, 0xC>(INF32, v));
    return v;
}
__device__ __forceinline__ u32 wave_prefix_addm31(u32 v) {  // inclusive sums mod P31
    v = addm31(v, dpp<0x111>(0, v));
    v = addm31(v, dpp<0x112>(0, v));
    v = addm31(v, dpp<0x114>(0, v));
    v = addm31(v, dpp<0x118>(0, v));
    v = addm31(v, dpp<0x142, 0xA>(0, v));
    v = addm31(v, dpp<0x143, 0xC>(0, v));
    return v;
}
__device__ __forceinline__ u32 wave_suffix_min(u32 v, u32 lane) {  // inclusive, over lanes >= L
    v = min(v, dpp<0x101>(INF32, v));
    v = min(v, dpp<0x102>(INF32, v));
    v = min(v, dpp<0x104>(INF32, v));
    v = min(v, dpp<0x108>(INF32, v));
    const u32 r1 = (u32)__builtin_amdgcn_readlane((int)v, 16), r2 = (u32)__builtin_amdgcn_readlane((int)v, 32),
              r3 = (u32)__builtin_amdgcn_readlane((int)v, 48);
    const u32 a1 = min(r2, r3), a0 = min(r1, a1);
    return min(v, lane < 16 ? a0 : lane < 32 ? a1 : lane < 48 ? r3 : INF32);
}

__global__ __launch_bounds__(64 * SWAVES) void k_sss_stream(const u8* __restrict__ T, u64 n, u64 last_i,
                                                           const u16* __restrict__ qinfo, u64 nstripes,
                                                           u32* __restrict__ s_out, u32* __restrict__ s_cnt,
                                                           u32* __restrict__ s_flag, u32* __restrict__ any_flag,
                                                           u32 b, sss_pow2 PW) {
    const u32 lane = threadIdx.x & 63;
    const u64 w = (u64)blockIdx.x * SWAVES + (threadIdx.x >> 6);
    if (w >= nstripes) return;  // whole wave
    const u64 i0 = w * (u64)SD;
    const u64 jmax = n - TAU;                  // last position with a full window (n >= 2 tau here)
    const u64 ilim = min<u64>(last_i - i0, (u64)SD - 1);  // decisions i0 + u, u <= ilim
    // per-lane powers: pwl = b^(8 lane), ipw = b^(-8 (lane + 1))
    u32 pwl = 1, ipw = PW.ib8;
    {
        u32 f = PW.b8, g = PW.ib8;
        for (int d = 0; d < 6; d++) {
            if (lane & (1u << d)) {
                pwl = mm31(pwl, f);
                ipw = mm31(ipw, g);
            }
            f = mm31(f, f);
            g = mm31(g, g);
        }
    }
    auto load8 = [&](u64 k) -> u64 { return *(const u64*)(T + i0 + k * TAU + 8 * lane); };
    // A_k(lane) = H(s_k + 8 lane) b^(-8 lane) for block k from its bytes, where H
    // is the prefix hash from the stripe start: with g = h8(lane) b^(-8(lane+1)),
    // A = carry + (exclusive prefix sum of g), a plain DPP sum scan mod P31.
    // carry = H(s_k) in, H(s_k+1) = b^512 (carry + sum of all g) out
    auto block_hash = [&](u64 bytes, u32& carry) -> u32 {
        const u32 lo = (u32)bytes, hi = (u32)(bytes >> 32);
        u64 acc = 0;
#pragma unroll
        for (int e = 0; e < 8; e++) {
            const u32 c = ((e < 4 ? lo : hi) >> (8 * (e & 3))) & 255u;
            acc += (u64)c * PW.pw8[e];
        }
        const u32 g = mm31(canon31(fold31(acc)), ipw);
        const u32 G = wave_prefix_addm31(g);
        const u32 A = addm31(carry, subm31(G, g));
        carry = mm31(addm31(carry, (u32)__builtin_amdgcn_readlane((int)G, 63)), PW.b512);
        return A;
    };
    // Phi'(s_k + 8 lane + e), e < 8, into v
    auto phi_block = [&](u64 k, u32 h0, u32 h1, u64 bo, u64 bi, u16 q0, u16 q1, u32* v) {
        // Phi(s_k + 8 lane) = H(s_k+1 + 8 lane) - H(s_k + 8 lane) b^512 = b^(8 lane) (A_k+1 - A_k b^512)
        u32 fp = mm31(subm31(h1, mm31(h0, PW.b512)), pwl);
        const u32 olo = (u32)bo, ohi = (u32)(bo >> 32), ilo = (u32)bi, ihi = (u32)(bi >> 32);
#pragma unroll
        for (int e = 0; e < 8; e++) {
            v[e] = fp;
            if (e < 7) {
                const u32 in = ((e < 4 ? ilo : ihi) >> (8 * (e & 3))) & 255u;
                const u32 out = ((e < 4 ? olo : ohi) >> (8 * (e & 3))) & 255u;
                fp = canon31(fold31((u64)fp * b + in + (u64)out * PW.bn));
            }
        }
        const u64 j0 = i0 + k * TAU + 8 * lane;
        const bool endblk = i0 + k * TAU + TAU - 1 > jmax;
        if (__builtin_expect(__ballot(q0 != 0xFF00 || q1 != 0xFF00) != 0 || endblk, 0)) {
            const u64 ta = (j0 + 127) >> 7;
#pragma unroll
            for (int e = 0; e < 8; e++) {
                const u64 j = j0 + e;
                if (j > jmax) {
                    v[e] = INF32;
                } else {
                    const u64 t = (j + 127) >> 7;
                    const u16 qi = t == ta ? q0 : q1;
                    const u32 rel = (u32)(j + 127 - (t << 7));
                    if (rel >= (u32)(qi >> 8) && rel <= (u32)(qi & 255)) v[e] = INF32;
                }
            }
        }
    };
    auto loadq = [&](u64 k, u16& q0, u16& q1) {
        const u64 j0 = i0 + k * TAU + 8 * lane;
        const u64 ta = (j0 + 127) >> 7;
        q0 = q1 = 0xFF00;
        if (j0 <= jmax) {
            q0 = qinfo[ta];
            if ((j0 & 127) == 0 && j0 + 1 <= jmax) q1 = qinfo[ta + 1];
        }
    };

    // prologue: H for blocks 0 and 1, Phi'(block 0)
    u32 carry = 0;
    u64 B0 = load8(0), B1 = load8(1), B2 = load8(2);
    u16 qa0, qa1, qb0, qb1;
    loadq(0, qa0, qa1);
    loadq(1, qb0, qb1);
    const u32 H0 = block_hash(B0, carry);
    u32 H1 = block_hash(B1, carry);
    u32 x[8], y[8];
    phi_block(0, H0, H1, B0, B1, qa0, qa1, x);
    u32 nout = 0;       // outputs of this stripe so far (uniform)
    u32* out = s_out + w * SCAP;
    const u32 nblk = (u32)min<u64>((u64)SNB, ilim / TAU + 1);
    for (u32 c = 0; c < nblk; c++) {
        // block c+2: bytes (prefetched), hash; block c+1: Phi'
        const u64 B3 = load8(c + 3);  // prefetch (the text pad covers the stripe's end)
        u16 qc0, qc1;
        loadq(c + 2, qc0, qc1);
        const u32 H2 = block_hash(B2, carry);
        phi_block(c + 1, H1, H2, B1, B2, qb0, qb1, y);
        // window minima for decisions of block c
        u32 sx[8], py[8];
        sx[7] = x[7];
#pragma unroll
        for (int e = 6; e >= 0; e--) sx[e] = min(x[e], sx[e + 1]);
        py[0] = y[0];
#pragma unroll
        for (int e = 1; e < 8; e++) py[e] = min(py[e - 1], y[e]);
        const u32 sufL = wave_suffix_min(sx[0], lane), preL = wave_prefix_min(py[7]);
        const u32 suf_after = dpp<0x130>(INF32, sufL);   // wave_shl:1 -> lane + 1 (63: inf)
        const u32 pre_before = dpp<0x138>(INF32, preL);  // wave_shr:1 -> lane - 1 (0: inf)
        const u32 g = min(suf_after, pre_before);
        u32 mk = 0;
#pragma unroll
        for (int e = 0; e < 8; e++) {
            const u32 m = min(min(sx[e], g), py[e]);
            if (m != INF32 && (x[e] == m || y[e] == m)) mk |= 1u << e;
        }
        if (c * TAU + TAU - 1 > ilim) {  // last block of the last stripe
            const int64_t keep = (int64_t)ilim - (int64_t)(c * TAU + 8 * lane) + 1;  // decisions of this lane kept
            mk &= keep <= 0 ? 0u : keep >= 8 ? 0xFFu : (1u << keep) - 1;
        }
        // ordered output: rank = sum of popc over lower lanes (4 ballots on the bits of popc)
        const u64 anyb = __ballot(mk != 0);
        if (anyb) {
            const u32 pc = __popc(mk);
            u32 rank = 0, tot = 0;
#pragma unroll
            for (int bit = 0; bit < 4; bit++) {
                const u64 bb = __ballot((pc >> bit) & 1);
                rank += (u32)__popcll(bb & ((1ull << lane) - 1)) << bit;
                tot += (u32)__popcll(bb) << bit;
            }
            u32 o = nout + rank;
            for (u32 mm = mk; mm; mm &= mm - 1) {
                if (o < (u32)SCAP) out[o] = (u32)(i0 + c * TAU + 8 * lane + __builtin_ctz(mm));
                o++;
            }
            nout += tot;
        }
        // shift the pipeline
#pragma unroll
        for (int e = 0; e < 8; e++) x[e] = y[e];
        H1 = H2;
        B1 = B2;
        B2 = B3;
        qb0 = qc0;
        qb1 = qc1;
    }
    if (lane == 0) {
        s_cnt[w] = nout;
        s_flag[w] = nout > (u32)SCAP;
        if (nout > (u32)SCAP) atomicOr(any_flag, 1u);
    }
}

// Exact slow path for stripes whose output buffer overflowed: one workgroup
// recomputes the stripe's Phi' values and the window minima directly.
__global__ __launch_bounds__(256) void k_sss_fallback(const u8* __restrict__ T, u64 n, u64 last_i,
                                                      const u16* __restrict__ qinfo, const u32* __restrict__ lanes,
                                                      u64* __restrict__ scratch, u8* __restrict__ member,
                                                      u32* __restrict__ ovf_out, u32* __restrict__ lane_cnt, u32 b,
                                                      u64 bpow) {
    const u64 lane = lanes[blockIdx.x];
    const u64 i0 = lane * SD;
    const u64 i_end = min(i0 + SD, last_i + 1);
    const u64 j_end = min(i0 + SD + TAU - 1, n - TAU);
    u64* v = scratch + (u64)blockIdx.x * (SD + TAU);
    u8* mem = member + (u64)blockIdx.x * SD;
    if (threadIdx.x == 0) {
        u64 fp = 0;
        for (u64 k = 0; k < TAU; k++) fp = (fp * b + T[i0 + k]) % P31;
        for (u64 j = i0; j <= j_end; j++) {
            const u64 t = (j + 127) >> 7;
            const u16 qi = qinfo[t];
            const u32 rel = (u32)(j + 127 - (t << 7));
            v[j - i0] = (rel >= (u32)(qi >> 8) && rel <= (u32)(qi & 255)) ? INF64 : fp;
            if (j < j_end) fp = (fp * b + T[j + TAU] + (P31 - bpow) * T[j]) % P31;
        }
    }
    __syncthreads();
    for (u64 i = i0 + threadIdx.x; i < i_end; i += blockDim.x) {
        u64 m = INF64;
        for (u64 x = 0; x <= TAU; x++) m = min(m, v[i - i0 + x]);
        mem[i - i0] = (m != INF64 && (v[i - i0] == m || v[i - i0 + TAU] == m));
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        u32 c = 0;
        for (u64 i = i0; i < i_end; i++)
            if (mem[i - i0]) ovf_out[(u64)blockIdx.x * SD + c++] = (u32)i;
        lane_cnt[lane] = c;
    }
}

__global__ void k_sss_compact(const u32* __restrict__ lane_out, const u32* __restrict__ lane_cnt,
                              const u32* __restrict__ lane_off, const u32* __restrict__ lane_flag,
                              const u32* __restrict__ ovf_slot, const u32* __restrict__ ovf_out, u64 nlanes,
                              u32* __restrict__ S) {
    const u64 lane = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (lane >= nlanes) return;
    const u32 c = lane_cnt[lane], o = lane_off[lane];
    const u32* src = lane_flag[lane] ? ovf_out + (u64)ovf_slot[lane] * SD : lane_out + lane * SCAP;
    for (u32 x = 0; x < c; x++) S[o + x] = src[x];
}

static u64 pow31_host(u64 b, u64 e) {
    u64 r = 1;
    while (e) {
        if (e & 1) r = r * b % P31;
        b = b * b % P31;
        e >>= 1;
    }
    return r;
}

void engine::build_sss(const u8* T) {
    s = 0;
    has_runs = false;
    runs_valid = false;
    sss_kernel_ms = 0;
    if (n < 2 * (u64)TAU) return;
    const u64 last_i = n - 2 * TAU;
    const u64 nanch = (n - TAU) / QA + 2;
    u16* qi = q_info.get(nanch);
    u32* ctr = counters.get(16);
    LZ_HIP(hipMemsetAsync(ctr, 0, 16 * sizeof(u32), st));
    u8* rp = run_p.get(nanch);
    u32* rhi = run_hi.get(nanch);
    u32* rlo = run_lo.get(nanch);
    u8* rcap = tmp_bytes.get(nanch);
    k_q_anchors<<<cdiv(nanch, QT_OWN), QT_THREADS, 0, st>>>(T, n, nanch, qi, ctr + 0, rp, rhi, rlo, rcap);
    LZ_HIP(hipGetLastError());
    {
        u64* ea = run_scan_a.get(2 * nanch);
        u64* eb = run_scan_b.get(2 * nanch);
        k_run_elems<<<cdiv(nanch, 256), 256, 0, st>>>(rp, rhi, rlo, rcap, nanch, ea, ea + nanch);
        size_t tb = 0;
        LZ_HIP(hipcub::DeviceScan::InclusiveScan(nullptr, tb, ea, eb, last_marked{}, (int)nanch, st));
        u8* t = scan_tmp.get(tb);
        LZ_HIP(hipcub::DeviceScan::InclusiveScan(t, tb, ea, eb, last_marked{}, (int)nanch, st));
        LZ_HIP(hipcub::DeviceScan::InclusiveScan(t, tb, ea + nanch, eb + nanch, last_marked{}, (int)nanch, st));
        k_run_finish<<<cdiv(nanch, 256), 256, 0, st>>>(eb, eb + nanch, nanch, rhi, rlo);
        LZ_HIP(hipGetLastError());
        runs_valid = true;
    }

    const u64 nlanes = last_i / SD + 1;  // stripes
    u32* lo = lane_out.get(nlanes * SCAP);
    u32* lc = lane_cnt.get(nlanes + 1);
    u32* lf = lane_flag.get(nlanes);
    sss_pow2 PW;
    {
        auto mm = [](u64 x, u64 y) { return x * y % P31; };
        (void)mm;
        PW.b8 = (u32)pow31_host(SSS_BASE, 8);
        PW.ib8 = (u32)pow31_host(PW.b8, P31 - 2);  // Fermat inverse
        for (int e = 0; e < 8; e++) PW.pw8[e] = (u32)pow31_host(SSS_BASE, 7 - e);
        PW.b512 = (u32)pow31_host(SSS_BASE, TAU);
        PW.bn = (u32)((P31 - PW.b512) % P31);
    }
    const u64 bpow = PW.b512;
    hipEvent_t e0, e1;
    LZ_HIP(hipEventCreate(&e0));
    LZ_HIP(hipEventCreate(&e1));
    LZ_HIP(hipEventRecord(e0, st));
    k_sss_stream<<<cdiv(nlanes, SWAVES), 64 * SWAVES, 0, st>>>(T, n, last_i, qi, nlanes, lo, lc, lf, ctr + 1,
                                                               (u32)SSS_BASE, PW);
    LZ_HIP(hipGetLastError());
    LZ_HIP(hipEventRecord(e1, st));

    u32 h_ctr[2];
    LZ_HIP(hipMemcpyAsync(h_ctr, ctr, 2 * sizeof(u32), hipMemcpyDeviceToHost, st));
    LZ_HIP(hipStreamSynchronize(st));
    float ms = 0;
    LZ_HIP(hipEventElapsedTime(&ms, e0, e1));
    sss_kernel_ms = ms;
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    has_runs = h_ctr[0] != 0;

    // overflowing tiles -> exact slow path
    u32* ovf_slot = u32c.get(nlanes);
    u32* ovf_out = nullptr;
    if (h_ctr[1]) {
        std::vector<u32> hf(nlanes);
        LZ_HIP(hipMemcpy(hf.data(), lf, nlanes * sizeof(u32), hipMemcpyDeviceToHost));
        std::vector<u32> lanes, slot(nlanes, 0);
        for (u64 l = 0; l < nlanes; l++)
            if (hf[l]) { slot[l] = (u32)lanes.size(); lanes.push_back((u32)l); }
        u32* d_lanes = u32d.get(lanes.size());
        LZ_HIP(hipMemcpy(d_lanes, lanes.data(), lanes.size() * 4, hipMemcpyHostToDevice));
        LZ_HIP(hipMemcpy(ovf_slot, slot.data(), nlanes * 4, hipMemcpyHostToDevice));
        u64* scratch = u64a.get(lanes.size() * (SD + TAU));
        u8* member = tmp_bytes.get(lanes.size() * SD);
        ovf_out = u32b.get(lanes.size() * SD);
        k_sss_fallback<<<(unsigned)lanes.size(), 256, 0, st>>>(T, n, last_i, qi, d_lanes, scratch, member, ovf_out,
                                                               lc, (u32)SSS_BASE, bpow);
        LZ_HIP(hipGetLastError());
        stats_fallback_lanes = lanes.size();
    } else {
        ovf_out = lo;  // unused
        stats_fallback_lanes = 0;
    }

    // exclusive scan of lane counts -> offsets; total = |S|
    u32* off = u32a.get(nlanes + 1);
    size_t tb = 0;
    LZ_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, lc, off, (int)(nlanes + 1), st));
    u8* tmp = tmp_bytes.get(std::max<size_t>(tb, tmp_bytes.cap));
    LZ_HIP(hipMemsetAsync(lc + nlanes, 0, sizeof(u32), st));
    LZ_HIP(hipcub::DeviceScan::ExclusiveSum(tmp, tb, lc, off, (int)(nlanes + 1), st));
    s = rd1(off + nlanes, st);
    u32* dS = S.get((u64)s + 1);
    k_sss_compact<<<cdiv(nlanes, 256), 256, 0, st>>>(lo, lc, off, lf, ovf_slot, ovf_out, nlanes, dS);
    LZ_HIP(hipGetLastError());
}

}  // namespace lz
