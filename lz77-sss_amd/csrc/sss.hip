// sss.hip -- kernel 1: the tau-synchronizing set (role of
// lce::rolling_hash::sss<pos_t,tau>, called at
// patched-files/external/lce/include/ds/lce_sss.hpp:53; its source is absent
// upstream, the definition pinned here is DESIGN.md section 4.1):
//
//   Phi(j)  = KR fingerprint of T[j..j+tau) mod 2^61-1 (base SSS_BASE)
//   Q       = { j : T[j..j+tau) has a period <= floor(tau/3) }
//   S       = { i <= n-2tau : min Phi'[i..i+tau] < inf at i or at i+tau }
//
// Launches:
//   k_q_anchors  -- per anchor a (every 128 positions) the smallest period <= 170
//                   of T[a..a+340), the Q interval it induces on (a-128, a], and
//                   the local extent of the periodic run (run table, lce_dev.h)
//   k_run_elems + 2 scans + k_run_finish -- exact run ends/starts along chains
//   k_sss_tile   -- one workgroup per tile of 7168 decisions: bytes staged once
//                   in LDS, prefix-hash scan + rolls give Phi', van Herk minima
//                   over 512-blocks in registers, ordered per-tile output
//   k_sss_fallback -- exact slow path for tiles with more than TCAP outputs
//   k_sss_compact-- per-tile outputs -> sorted S
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

// ---------------------------------------------------------------------------
// main pass: one workgroup per tile of TL decisions i in [t0, t0+TL)
//
//   bytes   T[t0 .. t0+8192)             staged once in LDS (coalesced uint4)
//   hashes  Phi(j), j in [t0, t0+7680)   prefix-hash scan over 512 threads x 16
//                                        bytes, then 15 rolls per thread
//   minima  m_i = min Phi'[i..i+512]     van Herk / Gil-Werman with 512-blocks:
//                                        m_i = min(suffix_c[o], prefix_c+1[o]),
//                                        both from wave scans held in registers
//   output  i in S  <=>  m_i < inf and (Phi'(i) == m_i or Phi'(i+512) == m_i)
constexpr int TL = 7168;            // decisions per tile (14 blocks of 512)
constexpr int TB = TL + 2 * TAU;    // staged bytes = 8192 = 512 threads x 16
constexpr int TP = TL + TAU;        // Phi' values per tile = 7680 (15 blocks)
constexpr int TWG = 512;            // threads per tile
constexpr int TCAP = 256;           // sync positions per tile before the exact fallback
static_assert(TB == TWG * 16, "tile bytes must be 16 per thread");

struct sss_pow {
    u32 scan[6];   // b^(16 * 2^d)
    u32 pw16[64];  // b^(16 k)
    u32 b1024;     // b^1024 (one wave of bytes)
    u32 b512;      // b^512 = b^tau
    u32 bn;        // P - b^tau
};

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
__device__ __forceinline__ u32 shfl_up32(u32 v, u32 d) { return __shfl_up(v, d, 64); }
__device__ __forceinline__ u32 shfl_down32(u32 v, u32 d) { return __shfl_down(v, d, 64); }

__global__ __launch_bounds__(TWG, 3) void k_sss_tile(const u8* __restrict__ T, u64 n, u64 last_i,
                                                     const u16* __restrict__ qinfo, u32* __restrict__ tile_out,
                                                     u32* __restrict__ tile_cnt, u32* __restrict__ tile_flag,
                                                     u32* __restrict__ any_flag, u32 b, sss_pow PW) {
    __shared__ __attribute__((aligned(16))) u8 s_t[TB + 16];
    __shared__ u32 s_h[TWG + 1];
    __shared__ u32 s_phi[TP + TP / 16];  // padded: index u + u/16 (bank spread)
    __shared__ u32 s_wt[TWG / 64];
    __shared__ u32 s_bc[TL / 512];
    const u32 tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const u64 t0 = (u64)blockIdx.x * TL;

    // 1. stage the tile's bytes (zero padded past n + TEXT_PAD)
    {
        const u64 g = t0 + 16ull * tid;
        uint4 v = {0, 0, 0, 0};
        if (g + 16 <= n + TEXT_PAD) v = *(const uint4*)(T + g);
        *(uint4*)&s_t[16 * tid] = v;
        if (tid == 0) *(uint4*)&s_t[TB] = uint4{0, 0, 0, 0};
    }
    __syncthreads();
    // 2. prefix hashes at every 16-byte boundary
    const uint4 mine = *(const uint4*)&s_t[16 * tid];
    const u32 mw[4] = {mine.x, mine.y, mine.z, mine.w};
    u32 h = 0;
#pragma unroll
    for (int k = 0; k < 16; k++) h = red31s((u64)h * b + ((mw[k >> 2] >> (8 * (k & 3))) & 255u));
    u32 inc = h;
#pragma unroll
    for (int d = 0; d < 6; d++) {
        const u32 left = shfl_up32(inc, 1u << d);
        if (lane >= (1u << d)) inc = red31((u64)left * PW.scan[d] + inc);
    }
    u32 exc = shfl_up32(inc, 1);
    if (lane == 0) exc = 0;
    if (lane == 63) s_wt[wv] = inc;
    __syncthreads();
    u32 hw = 0;  // prefix hash of the bytes before this wave
    for (u32 v = 0; v < wv; v++) hw = red31((u64)hw * PW.b1024 + s_wt[v]);
    const u32 hl = red31((u64)hw * PW.pw16[lane] + exc);
    s_h[tid] = hl;
    if (tid == TWG - 1) s_h[TWG] = red31((u64)hl * PW.scan[0] + h);
    __syncthreads();
    // 3. Phi'(u) for u in [16 tid, 16 tid + 16), u < TP
    if (16 * tid < (u32)TP) {
        // Phi(u0) = H(u0 + 512) - H(u0) * b^512
        u32 fp = red31((u64)s_h[tid + 32] + (P31 - mulmod31(hl, PW.b512)));
        const u64 j0 = t0 + 16ull * tid;
        const u64 jmax = n >= TAU ? n - TAU : 0;  // last position with a full window
        const u64 ta = (j0 + 127) >> 7;
        u16 q0 = 0xFF00, q1 = 0xFF00;
        if (j0 <= jmax) {
            q0 = qinfo[ta];
            if (((j0 + 15 + 127) >> 7) != ta && j0 + 15 <= jmax) q1 = qinfo[ta + 1];
        }
        const uint4 ahead = *(const uint4*)&s_t[16 * tid + TAU];
        const u32 aw[4] = {ahead.x, ahead.y, ahead.z, ahead.w};
        const bool noq = q0 == 0xFF00 && q1 == 0xFF00 && j0 + 15 <= jmax;  // common case: no Q, no end
#pragma unroll
        for (int k = 0; k < 16; k++) {
            const u32 u = 16 * tid + k;
            const u64 j = j0 + k;
            u32 v = fp;
            if (!noq) {
                if (j > jmax) {
                    v = INF32;
                } else {
                    const u64 t = (j + 127) >> 7;
                    const u16 qi = t == ta ? q0 : q1;
                    const u32 rel = (u32)(j + 127 - (t << 7));
                    if (rel >= (u32)(qi >> 8) && rel <= (u32)(qi & 255)) v = INF32;
                }
            }
            s_phi[u + (u >> 4)] = v;
            if (k < 15) {
                const u32 in = (aw[k >> 2] >> (8 * (k & 3))) & 255u, out = (mw[k >> 2] >> (8 * (k & 3))) & 255u;
                fp = red31s((u64)fp * b + in + (u64)out * PW.bn);
            }
        }
    }
    __syncthreads();
    // 4. window minima: wave w handles block pairs (c, c+1) for c = w, w + 8 (c < 14)
    const u32 ilim = last_i >= t0 ? (u32)min<u64>(last_i - t0, (u64)TL) : 0u;  // decisions u <= ilim
    const bool any_i = last_i >= t0;
    u32 masks[2] = {0, 0};
    for (int r = 0; r < 2; r++) {
        const u32 c = wv + 8 * r;
        if (c >= (u32)(TL / 512)) break;
        u32 x[8], y[8];
#pragma unroll
        for (int e = 0; e < 8; e++) {
            const u32 ux = c * 512 + 8 * lane + e, uy = ux + 512;
            x[e] = s_phi[ux + (ux >> 4)];
            y[e] = s_phi[uy + (uy >> 4)];
        }
        // suffix minima of block c, prefix minima of block c+1
        u32 sx[8], py[8];
        sx[7] = x[7];
#pragma unroll
        for (int e = 6; e >= 0; e--) sx[e] = min(x[e], sx[e + 1]);
        py[0] = y[0];
#pragma unroll
        for (int e = 1; e < 8; e++) py[e] = min(py[e - 1], y[e]);
        // lanes after this one (suffix) / before it (prefix)
        u32 sufL = sx[0], preL = py[7];
#pragma unroll
        for (int d = 0; d < 6; d++) {
            const u32 dn = shfl_down32(sufL, 1u << d);
            if (lane + (1u << d) < 64) sufL = min(sufL, dn);
            const u32 up = shfl_up32(preL, 1u << d);
            if (lane >= (1u << d)) preL = min(preL, up);
        }
        u32 suf_after = shfl_down32(sufL, 1), pre_before = shfl_up32(preL, 1);
        if (lane == 63) suf_after = INF32;
        if (lane == 0) pre_before = INF32;
        u32 mk = 0;
#pragma unroll
        for (int e = 0; e < 8; e++) {
            const u32 m = min(min(sx[e], suf_after), min(pre_before, py[e]));
            if (m != INF32 && (x[e] == m || y[e] == m) && any_i && c * 512 + 8 * lane + e <= ilim) mk |= 1u << e;
        }
        masks[r] = mk;
        u32 cnt = __popc(mk);
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) cnt += __shfl_xor(cnt, d, 64);
        if (lane == 0) s_bc[c] = cnt;
    }
    __syncthreads();
    // 5. ordered output: block offsets, then lane offsets inside the block
    u32 tot = 0;
    for (int c = 0; c < TL / 512; c++) tot += s_bc[c];
    for (int r = 0; r < 2; r++) {
        const u32 c = wv + 8 * r;
        if (c >= (u32)(TL / 512)) break;
        u32 boff = 0;
        for (u32 cc = 0; cc < c; cc++) boff += s_bc[cc];
        const u32 mk = masks[r];
        const u32 pc = __popc(mk);
        u32 incl = pc;
#pragma unroll
        for (int d = 0; d < 6; d++) {
            const u32 up = __shfl_up(incl, 1u << d, 64);
            if (lane >= (1u << d)) incl += up;
        }
        u32 o = boff + incl - pc;
        for (int e = 0; e < 8; e++)
            if (mk & (1u << e)) {
                if (o < (u32)TCAP) tile_out[(u64)blockIdx.x * TCAP + o] = (u32)(t0 + c * 512 + 8 * lane + e);
                o++;
            }
    }
    if (tid == 0) {
        tile_cnt[blockIdx.x] = tot;
        tile_flag[blockIdx.x] = tot > (u32)TCAP;
        if (tot > (u32)TCAP) atomicOr(any_flag, 1u);
    }
}

// Exact slow path for tiles whose output buffer overflowed: one workgroup
// recomputes the tile's Phi' values and the window minima directly.
__global__ __launch_bounds__(256) void k_sss_fallback(const u8* __restrict__ T, u64 n, u64 last_i,
                                                      const u16* __restrict__ qinfo, const u32* __restrict__ lanes,
                                                      u64* __restrict__ scratch, u8* __restrict__ member,
                                                      u32* __restrict__ ovf_out, u32* __restrict__ lane_cnt, u32 b,
                                                      u64 bpow) {
    const u64 lane = lanes[blockIdx.x];
    const u64 i0 = lane * TL;
    const u64 i_end = min(i0 + TL, last_i + 1);
    const u64 j_end = min(i0 + TL + TAU - 1, n - TAU);
    u64* v = scratch + (u64)blockIdx.x * (TL + TAU);
    u8* mem = member + (u64)blockIdx.x * TL;
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
            if (mem[i - i0]) ovf_out[(u64)blockIdx.x * TL + c++] = (u32)i;
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
    const u32* src = lane_flag[lane] ? ovf_out + (u64)ovf_slot[lane] * TL : lane_out + lane * TCAP;
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

    const u64 nlanes = last_i / TL + 1;  // tiles
    u32* lo = lane_out.get(nlanes * TCAP);
    u32* lc = lane_cnt.get(nlanes + 1);
    u32* lf = lane_flag.get(nlanes);
    sss_pow PW;
    {
        auto mm = [](u64 x, u64 y) { return x * y % P31; };
        u64 b16 = pow31_host(SSS_BASE, 16);
        for (int d = 0; d < 6; d++) { PW.scan[d] = (u32)b16; b16 = mm(b16, b16); }
        PW.pw16[0] = 1;
        const u64 p16 = pow31_host(SSS_BASE, 16);
        for (int k = 1; k < 64; k++) PW.pw16[k] = (u32)mm(PW.pw16[k - 1], p16);
        PW.b1024 = (u32)pow31_host(SSS_BASE, 1024);
        PW.b512 = (u32)pow31_host(SSS_BASE, TAU);
        PW.bn = (u32)((P31 - PW.b512) % P31);
    }
    const u64 bpow = PW.b512;
    hipEvent_t e0, e1;
    LZ_HIP(hipEventCreate(&e0));
    LZ_HIP(hipEventCreate(&e1));
    LZ_HIP(hipEventRecord(e0, st));
    k_sss_tile<<<(unsigned)nlanes, TWG, 0, st>>>(T, n, last_i, qi, lo, lc, lf, ctr + 1, (u32)SSS_BASE, PW);
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
        u64* scratch = u64a.get(lanes.size() * (TL + TAU));
        u8* member = tmp_bytes.get(lanes.size() * TL);
        ovf_out = u32b.get(lanes.size() * TL);
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
