// sss.hip -- kernel 1: the tau-synchronizing set (role of
// lce::rolling_hash::sss<pos_t,tau>, called at
// patched-files/external/lce/include/ds/lce_sss.hpp:53; its source is absent
// upstream, the definition pinned here is DESIGN.md section 4.1):
//
//   Phi(j)  = sum_k T[j+k] b^(tau-1-k) mod 2^32, b = SSS_BASE (a polynomial
//             Karp-Rabin hash over Z/2^32, not over a prime: DESIGN.md 4.1 states
//             what that choice costs on hash-adversarial text)
//   Q       = { j : T[j..j+tau) has a period <= floor(tau/3) }
//   Phi'(j) = INF (2^32-1) for j in Q, else Phi(j)
//   S       = { i <= n-2tau : m_i != INF and m_i in {Phi'(i), Phi'(i+tau)} },
//             m_i = min Phi'[i..i+tau]
//
// Launches:
//   k_q_anchors  -- per anchor a (every 128 positions) the smallest period <= 170
//                   of T[a..a+340), the Q interval it induces on (a-128, a], and
//                   the local extent of the periodic run (run table, lce_dev.h)
//   k_run_elems + 2 scans + k_run_finish -- exact run ends/starts along chains
//   k_sss_stream -- one wave per stripe of 32768 decisions, walked in 512-blocks
//                   with bytes, prefix hashes and Phi' in registers: lane Horner +
//                   wave scan, 7 rolls per lane, van Herk minima by lane-local
//                   and wave scans, ordered per-stripe output
//   k_sss_fallback -- exact workgroup-parallel path for stripes with more than SCAP outputs
//   k_sss_compact-- per-stripe outputs -> sorted S
#include "../../include/lz77sss.h"
#include "../include/engine.h"
#include "../include/prim.h"

#include <hipcub/hipcub.hpp>

#include <cstdlib>
#include <vector>


namespace LZ_NS {

// ---------------------------------------------------------------------------
// Q anchors.  A workgroup of QT_THREADS lanes (128 by default) covers anchors
// tb-1 .. tb+QT_THREADS-2 (lane i -> anchor tb-1+i) and owns QT_OWN = QT_THREADS-3 of
// them (tb .. tb+QT_OWN-1); the three halo anchors give the owned ones their
// neighbours' periods.  Text [a(tb-1) - 256, a(tb+QT_THREADS-2) + 1024) is staged in LDS.
constexpr int SNB = 64;                       // decision blocks per stripe (k_sss_stream)
constexpr int SD = SNB * (int)TAU;            // decisions per stripe (32768)
#ifndef LZ_QT_THREADS
#define LZ_QT_THREADS 128  // k_q_anchors workgroup (anchors per tile + 3 halo); rr: 256 -> 623 us, 128 -> 576 us, 64 -> 580 us
#endif
constexpr int QT_THREADS = LZ_QT_THREADS;
constexpr int QT_OWN = QT_THREADS - 3;                  // owned anchors per workgroup
constexpr int QT_LDS = QT_THREADS * (int)QA + 256 + 1024;
constexpr u32 RUN_HCAP = 640;                           // local run extension: [a-256, a+640)
constexpr u32 RUN_LCAP = 256;

// tiles: the tiles to compute (tile = 253 owned anchors; nullptr = tile blockIdx.x);
// sflag/slist/scnt (optional): stripes whose decisions see a Q window of an owned
// anchor are appended once to slist (the exact re-run of build_sss)
__global__ __launch_bounds__(QT_THREADS) void k_q_anchors(const u8* __restrict__ T, u64 n, u64 nanch,
                                                          u16* __restrict__ qinfo, u32* __restrict__ any_q,
                                                          u8* __restrict__ run_p, pos_t* __restrict__ run_hi,
                                                          pos_t* __restrict__ run_lo, u8* __restrict__ run_cap,
                                                          const u32* __restrict__ tiles, u32* __restrict__ sflag,
                                                          u32* __restrict__ slist, u32* __restrict__ scnt,
                                                          u64 nstripes) {
    // LDS text with one pad word per 128 bytes: the anchors of a wave sit 128 bytes
    // apart, so unpadded their accesses would all hit the same bank
    __shared__ __attribute__((aligned(16))) u32 b32[QT_LDS / 4 + QT_LDS / 128 + 2];
    __shared__ u8 s_p1[QT_THREADS], s_c[QT_THREADS], s_p[QT_THREADS];
    __shared__ u32 s_anyq, s_mark[4];
    const int i = (int)threadIdx.x;
    const int64_t tb = (int64_t)(tiles ? tiles[blockIdx.x] : blockIdx.x) * QT_OWN;
    // stripes a Q window of this tile can reach: decisions (a - 640, a] of owned anchors a
    const int64_t w_lo = max<int64_t>(0, (tb * (int64_t)QA - 639) / SD);
    const int64_t base = (tb - 1) * (int64_t)QA - 256;  // LDS offset 0
    {
        // all global loads first (one round trip), then the LDS writes.  Loads are
        // unconditional: out-of-range lanes read the zero padding at T + n (a guarded
        // or zeroed load becomes a branch with its own s_waitcnt)
        constexpr int NR = (QT_LDS + QT_THREADS * 16 - 1) / (QT_THREADS * 16);  // load rounds (last partial)
        auto src = [&](int x) -> const uint4* {
            const int64_t g = base + x;
            const bool okr = g >= 0 && (u64)g + 16 <= n + TEXT_PAD;
            return (const uint4*)(T + (okr ? (u64)g : n));
        };
        uint4 v[NR];
#pragma unroll
        for (int r = 0; r < NR; r++) {
            const int x = i * 16 + r * QT_THREADS * 16;
            v[r] = *src(x < QT_LDS ? x : -(1 << 20));
        }
        auto put = [&](int x, uint4 q) {
            const int w = (x >> 2) + (x >> 7);
            b32[w] = q.x;
            b32[w + 1] = q.y;
            b32[w + 2] = q.z;
            b32[w + 3] = q.w;
        };
#pragma unroll
        for (int r = 0; r < NR; r++) {
            const int x = i * 16 + r * QT_THREADS * 16;
            if (x < QT_LDS) put(x, v[r]);
        }
    }
    if (i == 0) s_anyq = 0;
    if (i < 4) s_mark[i] = 0;
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
    // candidates of the words k >= kbeg (fully unrolled; the guard is uniform or a lane mask)
    auto filt_words = [&](int kbeg) {
        const u32 w0 = word(oa >> 2);
#pragma unroll
        for (int k = 0; k <= (int)(QL / 4); k++) {
            if (k < kbeg) continue;
            const u32 dprev = word((oa >> 2) + k), dnext = word((oa >> 2) + k + 1);
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const u32 pp = 4 * k + r;
                if (pp >= 1 && pp <= QL && __builtin_amdgcn_alignbyte(dnext, dprev, r) == w0)
                    cm[(pp - 1) >> 5] |= 1u << ((pp - 1) & 31);
            }
        }
    };
    // the smallest candidate first: groups of 4 words until every probe of the wave has one
    // (inside runs of small period after a few words); the rest only where p1 fails
    int kdone = (int)(QL / 4) + 1;
    if (probe_ok) {
        const u32 w0 = word(oa >> 2);
#pragma unroll
        for (int g = 0; g <= (int)(QL / 4); g += 4) {
#pragma unroll
            for (int k = g; k < g + 4 && k <= (int)(QL / 4); k++) {
                const u32 dprev = word((oa >> 2) + k), dnext = word((oa >> 2) + k + 1);
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    const u32 pp = 4 * k + r;
                    if (pp >= 1 && pp <= QL && __builtin_amdgcn_alignbyte(dnext, dprev, r) == w0)
                        cm[(pp - 1) >> 5] |= 1u << ((pp - 1) & 31);
                }
            }
            if (g + 4 <= (int)(QL / 4) && !__ballot((cm[0] | cm[1] | cm[2] | cm[3] | cm[4] | cm[5]) == 0)) {
                kdone = g + 4;
                break;
            }
        }
    }
    u32 p1 = 0;
    for (int wi = 0; wi < 6 && !p1; wi++)
        if (cm[wi]) p1 = 32 * wi + __builtin_ctz(cm[wi]) + 1;
    // ---- 2. shift-p1 agreement over the anchor's own 128 bytes; a probe that
    // agrees over its whole chunk is verified from its two successors' chunks
    // when they test the same shift (inside a run: every anchor), so each byte
    // of a run is compared about once instead of 340/128 times
    // agreement of shift p1 over the anchor's own 128 bytes, 16 bytes per step (oa is
    // word aligned): inside a run every anchor runs the whole chunk, so the LDS loads
    // of a step are issued together and the exit test is taken once per 4 words
    auto chunk_agree = [&](int p) -> int {
        const int w0 = oa >> 2;
        const int q0 = (oa + p) >> 2;
        const u32 sh = (u32)(p & 3);
        u32 lo = word(q0);
#pragma unroll 1
        for (int k = 0; k < (int)QA / 4; k += 4) {
            u32 a[4], b[5];
#pragma unroll
            for (int j = 0; j < 4; j++) {
                a[j] = word(w0 + k + j);
                b[j + 1] = word(q0 + k + j + 1);
            }
            b[0] = lo;
            u32 d[4];
            bool any = false;
#pragma unroll
            for (int j = 0; j < 4; j++) {
                d[j] = a[j] ^ __builtin_amdgcn_alignbyte(b[j + 1], b[j], sh);
                any |= d[j] != 0;
            }
            if (any) {
#pragma unroll
                for (int j = 0; j < 4; j++)
                    if (d[j]) return 4 * (k + j) + (__builtin_ctz(d[j]) >> 3);
            }
            lo = b[4];
        }
        return (int)QA;
    };
    const int c = p1 ? chunk_agree((int)p1) : 0;
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
            if (kdone <= (int)(QL / 4)) filt_words(kdone);  // the candidates past the early stop
            cm[(p1 - 1) >> 5] &= ~(1u << ((p1 - 1) & 31));
            for (int wi = 0; wi < 6; wi++) {
                const int lo = 32 * wi + 1;  // candidate of bit 0
                if (f + 1 >= lo + 32) cm[wi] = 0;
                else if (f + 1 > lo) cm[wi] &= ~0u << (f + 1 - lo);
            }
            // a period pp must also agree where earlier shifts disagreed: test the
            // disagreement of p1 (f) and of the last rejected candidate (g) first, so
            // candidates in a run broken by a single character cost O(1), not a scan
            int g = f;
            for (int wi = 0; wi < 6 && !per;) {
                if (!cm[wi]) {
                    wi++;
                    continue;
                }
                const u32 pp = 32 * wi + __builtin_ctz(cm[wi]) + 1;
                cm[wi] &= cm[wi] - 1;
                const int lim = (int)(QM - pp);  // offsets x < lim are compared (x >= 4 after the filter)
                if ((f < lim && byte(oa + f) != byte(oa + f + (int)pp)) ||
                    (g < lim && byte(oa + g) != byte(oa + g + (int)pp)))
                    continue;
                const int e = ext_fwd(oa + 4, oa + lim, (int)pp);
                if (e == oa + lim) per = pp;
                else g = e - oa;
            }
        }
    }
    s_p[i] = (u8)per;
    __syncthreads();

    // ---- 3. owned anchors: Q interval on (a-128, a] and the local run extent
    if (i >= 1 && i <= QT_OWN && (u64)t < nanch) {
        u16 res = 0xFF00;  // empty interval
        u32 rp = 0;
        pos_t rhi = 0, rlo = 0;
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
                if (sflag) {  // decisions [j - 512, j] for j in (a - 128, a]: stripes of (a - 640, a]
                    const int64_t wa = max<int64_t>(0, ((int64_t)a - 639) / SD), wb = (int64_t)a / SD;
                    for (int64_t w = wa; w <= wb; w++) s_mark[w - w_lo] = 1;
                }
            }
            // local extent of the p-periodic run around the window (for run-skipping LCE);
            // inside a chain of same-period anchors the values only need to mark the chain
            rp = p;
            if (contf) {
                rhi = (pos_t)(a + RUN_HCAP);
                rcap |= 1;
            } else {
                const u64 h2_cap = min(a + RUN_HCAP - p, n - p);
                const u64 h2 = hi < hi_cap ? hi : (u64)(base + ext_fwd(o_hi, (int)((int64_t)h2_cap - base), (int)p));
                rhi = (pos_t)(h2 + p);
                rcap |= h2 == a + RUN_HCAP - p ? 1 : 0;
            }
            if (contb) {
                rlo = (pos_t)(a >= RUN_LCAP ? a - RUN_LCAP : a - QA);
                rcap |= 2;
            } else {
                const u64 l2_cap = a >= RUN_LCAP ? a - RUN_LCAP : 0;
                const u64 l2 = (lo > lo_cap) ? lo : (u64)(base + ext_bwd(o_lo, (int)((int64_t)l2_cap - base), (int)p));
                rlo = (pos_t)l2;
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
    // (and none once the flag is visible: on run-heavy text every block has a Q window)
    if (i == 0 && s_anyq && __hip_atomic_load(any_q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u)
        atomicOr(any_q, 1u);
    if (sflag && i < 4 && s_mark[i] && (u64)(w_lo + i) < nstripes && atomicOr(&sflag[w_lo + i], 1u) == 0u)
        slist[atomicAdd(scnt, 1u)] = (u32)(w_lo + i);
}

// run chains: anchor t continues into t+1 (same run) when both have period p
// and t's run covers t+1's window; a chain's exact hi is its last anchor's local
// hi (exact unless capped), its exact lo its first anchor's local lo.
// an unknown run start reads as larger than every position (lce_dev.h: "lo > x" skips the jump)
constexpr u64 RUN_LO_UNKNOWN = sizeof(pos_t) == 4 ? 0xFFFFFFFFull : (1ull << 62);
// element e of the run-chain scans is anchor t(e): e itself, or with a tile list the
// anchors of the listed (sorted) tiles back to back.  Chains never cross a tile that
// is not listed (its anchors have period 0), so the scans over the concatenation are
// exact.  Elements past the last anchor are chain ends with unknown values.
__device__ __forceinline__ u64 run_elem_anchor(const u32* __restrict__ tiles, u64 e) {
    return tiles ? (u64)tiles[e / QT_OWN] * QT_OWN + e % QT_OWN : e;
}
// chain keys: kend_rev[m-1-e] = e at a chain end (else ~0), kstart[e] = e + 1 at a
// chain start (else 0); an inclusive min-scan over kend_rev and a max-scan over kstart
// give every element its chain's last and first element
__global__ void k_run_keys(const u8* __restrict__ rp, const pos_t* __restrict__ rhi, const pos_t* __restrict__ rlo,
                           u64 na, const u32* __restrict__ tiles, u64 m, u32* __restrict__ kend_rev,
                           u32* __restrict__ kstart) {
    const u64 e = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= m) return;
    const u64 t = run_elem_anchor(tiles, e);
    bool cont_f = false, cont_b = false;
    if (t < na) {
        const u32 p = rp[t];
        const u64 a = t * QA;
        cont_f = p && t + 1 < na && rp[t + 1] == p && (u64)rhi[t] >= a + QA + QM;
        cont_b = p && t >= 1 && rp[t - 1] == p && (u64)rlo[t] + QA <= a;
    }
    kend_rev[m - 1 - e] = cont_f ? 0xFFFFFFFFu : (u32)e;
    kstart[e] = cont_b ? 0u : (u32)e + 1;
}
// exact run ends / starts: the chain's last anchor's local hi (unknown = 0 when capped) and
// its first anchor's local lo (unknown when capped).  In place: an end (start) anchor
// rewrites its own entry by the same rule, so reading it before or after gives one value.
__global__ void k_run_apply(const u32* __restrict__ send_rev, const u32* __restrict__ sstart, const u8* __restrict__ rp,
                            const u8* __restrict__ rcap, u64 na, const u32* __restrict__ tiles, u64 m,
                            pos_t* __restrict__ rhi, pos_t* __restrict__ rlo) {
    const u64 e = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= m) return;
    const u64 t = run_elem_anchor(tiles, e);
    if (t >= na || !rp[t]) return;
    const u64 te = run_elem_anchor(tiles, send_rev[m - 1 - e]), ts = run_elem_anchor(tiles, sstart[e] - 1);
    const pos_t hi = (rcap[te] & 1) ? (pos_t)0 : rhi[te];
    const pos_t lo = (rcap[ts] & 2) ? (pos_t)RUN_LO_UNKNOWN : rlo[ts];
    rhi[t] = hi;
    rlo[t] = lo;
}

// ---------------------------------------------------------------------------
// main pass, streaming form: one wave per stripe of SD = SNB x 512 decisions,
// walked block by block with everything in registers (no LDS, no barriers).
// Lane L owns positions s_k + 8L .. s_k + 8L + 7 of every 512-block k.
// All fingerprint arithmetic is mod 2^32 (plain wrapping u32 multiply-adds).
//
//   bytes   8 per lane and block (one coalesced 512-byte load per wave),
//           prefetched two blocks ahead
//   hashes  prefix hash Hp(x) from the stripe start: lane Horner over its 8
//           bytes, lane starts from a DPP sum scan of h8(L) b^(-8(L+1))
//           (b odd, so b^-1 exists mod 2^32); Phi(j) = Hp(j+512) - b^512 Hp(j)
//   minima  van Herk / Gil-Werman with 512-blocks: for decision block c the
//           wave holds Phi'(block c) and Phi'(block c+1) in registers;
//           m_i = min(suffix_c, prefix_c+1) from lane-local scans + wave scans
//   output  i in S  <=>  m_i != INF and min(Phi'(i), Phi'(i+512)) == m_i
//           (m_i <= both, so this is "either equals m_i"; the INF test folds into
//           a clamp of the cross-lane minimum); decisions come out as 8 wave
//           masks, compacted in position order by a wave scan of per-lane counts
//
// Two instantiations:
//   PASS1  every stripe, Q assumed empty (Phi' = Phi), plus the periodicity filter
//          of every block (sss_filter); a stripe with a confirmed filter hit stops
//          computing S (it is re-run) and only filters its remaining blocks
//   QSKIP  the exact re-run of the stripes listed by build_sss, with the Q
//          intervals of k_q_anchors; blocks entirely inside Q skip their hashing
//          and minima
#ifndef SSS_VAR
#define SSS_VAR 0  // timing experiments only (tools/sss_variants.sh); 0 = the product kernel
#endif
constexpr int SCAP = 1024;                    // sync positions per stripe before the fallback
constexpr int SWAVES = 4;                     // independent waves per workgroup
constexpr int FA_LANES = 22;                  // candidate lanes per filter anchor (4 shifts each)

struct sss_pow32 {
    u32 pwb[8];    // b^e, e < 8
    u32 b8, ib8;   // b^8 and b^-8 (mod 2^32)
    u32 B;         // b^512 = b^tau
};

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
__device__ __forceinline__ u32 wave_prefix_add(u32 v) {  // inclusive sums mod 2^32
    v += dpp<0x111>(0, v);
    v += dpp<0x112>(0, v);
    v += dpp<0x114>(0, v);
    v += dpp<0x118>(0, v);
    v += dpp<0x142, 0xA>(0, v);
    v += dpp<0x143, 0xC>(0, v);
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

// one v_min3_u32 (the compiler otherwise re-associates the clamp into every decision)
__device__ __forceinline__ u32 min3u(u32 a, u32 b, u32 c) {
    u32 r;
    asm("v_min3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}

// Periodicity filter of one 512-block (PASS1), on the bytes the wave already holds
// (lane L: bytes 8L..8L+7 as B).  Filter anchors A0 = block start and A1 = +256; bit
// r of the (uniform) result is set when T[A_r .. A_r + 16) recurs at a shift in
// [84, 171].  No false negatives: a tau-window with a period p <= 170 has the period
// kp in (85, 170] (a multiple of p) and contains [A, A + 186) for its filter anchor A
// in [j, j + 256), so T[A..A+16) recurs at A + kp.  Lane l < 22 of half h tests the 4
// shifts 84 + 4l + k of A_h (its bytes gathered from 2-3 lanes by ds_bpermute); an
// 8-byte repeat (about one block in 400 on ACGT text) is confirmed on bytes 8..15, and a 16-byte
// repeat at shift d in [86, 170] on the whole stretch a Q window would force: T[A..A+186-d) ==
// T[A+d..A+186) (the window holds [A, A+186) and has the period d; shifts 84, 85 and 171 are never
// such a multiple).  The chance 16-byte repeats of a random ACGT text then pass only at d close to
// 170, where the stretch is short (all inside the block: A + 186 <= 442, compared from the
// registers by cross-lane moves).
// 8 bytes at byte offset 8 lane + p of the 1024-byte concatenation [Bx, By] of two blocks in
// registers (p <= 170): the lane's words lane + p/8 and lane + p/8 + 1, by cross-lane moves
__device__ __forceinline__ u64 shfl64(u64 v, u32 src) {
    return ((u64)(u32)__shfl((int)(u32)(v >> 32), (int)src, 64) << 32) | (u32)__shfl((int)(u32)v, (int)src, 64);
}
// the same from the blocks' word rotations a = shfl64(Bx, (lane + p/8) & 63), c = shfl64(By, ...)
// (a streaming caller rotates every block once and uses it for two blocks)
__device__ __forceinline__ u64 shifted8_rot(u64 a, u64 c, u64 By, u32 p, u32 lane) {
    const u32 q = p >> 3, sh = 8 * (p & 7);
    const u64 w0 = lane + q >= 64 ? c : a;
    if (!sh) return w0;
    // word lane + q + 1: lane + 1's w0; for lane 63 word 64 + q, i.e. By's lane q
    u64 w1 = ((u64)dpp<0x130>(0u, (u32)(w0 >> 32)) << 32) | dpp<0x130>(0u, (u32)w0);
    if (lane == 63)
        w1 = ((u64)(u32)__builtin_amdgcn_readlane((int)(u32)(By >> 32), (int)q) << 32) |
             (u32)__builtin_amdgcn_readlane((int)(u32)By, (int)q);
    return (w0 >> sh) | (w1 << (64 - sh));
}
__device__ __forceinline__ u64 shifted8(u64 Bx, u64 By, u32 p, u32 lane) {
    const u32 src = (lane + (p >> 3)) & 63;
    return shifted8_rot(shfl64(Bx, src), shfl64(By, src), By, p, lane);
}
__device__ __forceinline__ u32 sss_filter(u64 B, u32 lane) {
    const u32 lo = (u32)B, hi = (u32)(B >> 32);
    const u32 li = lane & 31, grp = lane >> 5;
    // anchor bytes of the lane's half (lane 0 or 32)
    const int la = (int)(lane & 32u);
    const u64 A = (u64)(u32)__shfl((int)hi, la, 64) << 32 | (u32)__shfl((int)lo, la, 64);
    // x0 = 84 + 4 li (+ 256 grp): the hi word of lane 10 + li/2 (li even) or the lo word of
    // lane 11 + li/2 (li odd)
    const bool ev = (li & 1) == 0;
    const int l0 = (int)((grp << 5) + 10 + (li >> 1) + (li & 1));
    const u32 s0l = (u32)__shfl((int)lo, l0, 64), s0h = (u32)__shfl((int)hi, l0, 64);
    const u32 s1l = (u32)__shfl((int)lo, l0 + 1, 64), s1h = (u32)__shfl((int)hi, l0 + 1, 64);
    const u32 d0 = ev ? s0h : s0l, d1 = ev ? s1l : s0h, d2 = ev ? s1h : s1l;
    // any 8-byte repeat among the 4 shifts of the candidate lanes (wave masks, no per-lane bits)
    u64 any = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const u64 w = (u64)__builtin_amdgcn_alignbyte(d2, d1, k) << 32 | __builtin_amdgcn_alignbyte(d1, d0, k);
        any |= __ballot(w == A);
    }
    if (!(any & 0x003FFFFF003FFFFFull)) return 0;  // candidate lanes li < FA_LANES (22)
    static_assert(FA_LANES == 22, "candidate lane mask");
    // rare: confirm on bytes 8..15
    const u32 cl = grp ? (u32)__builtin_amdgcn_readlane((int)lo, 33) : (u32)__builtin_amdgcn_readlane((int)lo, 1);
    const u32 ch = grp ? (u32)__builtin_amdgcn_readlane((int)hi, 33) : (u32)__builtin_amdgcn_readlane((int)hi, 1);
    const u32 s2l = (u32)__shfl((int)lo, l0 + 2, 64), s2h = (u32)__shfl((int)hi, l0 + 2, 64);
    const u32 d3 = ev ? s2l : s1h, d4 = ev ? s2h : s2l;
    u32 hk = 0;  // the lane's shifts (bit k: d = 84 + 4 li + k) with a 16-byte repeat
#pragma unroll
    for (int k = 0; k < 4; k++)
        hk |= (__builtin_amdgcn_alignbyte(d1, d0, k) == (u32)A && __builtin_amdgcn_alignbyte(d2, d1, k) == (u32)(A >> 32) &&
               __builtin_amdgcn_alignbyte(d3, d2, k) == cl && __builtin_amdgcn_alignbyte(d4, d3, k) == ch)
                  ? 1u << k : 0u;
    if (li >= (u32)FA_LANES) hk = 0;
    u32 res = 0;
    // (a confirmed half drops its other candidate lanes at once: on run-heavy text every even shift
    // of a period-2 run is a candidate, and skipping them one by one cost ~600 SALU per block)
    for (u64 hm = __ballot(hk != 0); hm;) {
        const u32 L = (u32)__builtin_ctzll(hm);
        const u32 g = L >> 5;
        hm &= hm - 1;
        const u64 x = shfl64(B, (32 * g + lane) & 63);  // bytes A + 8 lane .. + 7
        for (u32 bits = (u32)__builtin_amdgcn_readlane((int)hk, (int)L); bits; bits &= bits - 1) {
            const u32 d = 84 + 4 * (L & 31) + (u32)__builtin_ctz(bits);
            if (d < 86 || d > 170) continue;
            const u32 len = 186 - d, o = 8 * lane;  // <= 100 bytes: lanes 0..12
            const u32 q = (32 * g + (d >> 3) + lane) & 63, sh = 8 * (d & 7);
            const u64 y0 = shfl64(B, q), y1 = shfl64(B, (q + 1) & 63);
            u64 y = sh ? (y0 >> sh) | (y1 << (64 - sh)) : y0, xx = x;
            bool bad = false;
            if (o < len) {
                if (len - o < 8) {
                    const u64 m = (1ull << (8 * (len - o))) - 1;
                    xx &= m;
                    y &= m;
                }
                bad = xx != y;
            }
            if (!__ballot(bad)) {
                res |= 1u << g;
                hm &= g ? 0ull : 0xFFFFFFFF00000000ull;
                break;
            }
        }
    }
    return res;
}

// The smallest period q <= 170 of a 512-byte block Bx (lane L: bytes 8L .. 8L + 7) whose next
// block is By: the smallest q with T[z] == T[z + q] for the block's 512 positions (0: none).  A
// period of the block is a shift at which its first 8 bytes recur, so only those shifts are
// verified, in increasing order (lane L finds the recurrences at q = 3L + 1 .. 3L + 3 from its
// words j0 .. j0 + 2; one ballot per verified candidate instead of one per shift)
__device__ __forceinline__ u32 smallest_period(u64 Bx, u64 By, u32 lane) {
    const u64 A = ((u64)(u32)__builtin_amdgcn_readlane((int)(u32)(Bx >> 32), 0) << 32) |
                  (u32)__builtin_amdgcn_readlane((int)(u32)Bx, 0);
    const u32 j0 = (3 * lane + 1) >> 3;
    const u64 w0 = shfl64(Bx, j0 & 63), w1 = shfl64(Bx, (j0 + 1) & 63), w2 = shfl64(Bx, (j0 + 2) & 63);
    u64 m[3];
#pragma unroll
    for (u32 k = 0; k < 3; k++) {
        const u32 q = 3 * lane + 1 + k, r = q - 8 * j0;  // r <= 9
        const u64 v = r == 0 ? w0 : r < 8 ? (w0 >> (8 * r)) | (w1 << (64 - 8 * r))
                                 : r == 8 ? w1 : (w1 >> (8 * (r - 8))) | (w2 << (64 - 8 * (r - 8)));
        m[k] = __ballot(q <= QL && v == A);
    }
    for (;;) {
        u32 best = 0xFFFFu;
#pragma unroll
        for (u32 k = 0; k < 3; k++)
            if (m[k]) best = min(best, 3u * (u32)__builtin_ctzll(m[k]) + 1 + k);
        if (best > QL) return 0;
        m[(best - 1) % 3] &= ~(1ull << ((best - 1) / 3));
        if (!__ballot(shifted8(Bx, By, best, lane) != Bx)) return best;
    }
}

// Run scan of a stripe pass 1 stopped (the first phase of k_sss_runs): blocks 0 .. 65 streamed
// through the wave's LDS ring (chunks of 8 blocks; three register buffers, the loads of chunk g + 2
// issued before chunk g is stored, so 16 blocks stay in flight through each store's wait; the loop
// is unrolled, so nothing is copied -- a copy of a loading register waits for its load), each
// compared with its bytes P ahead, P = the smallest period <= 170 of block 1 (0: none).  Returns
// whether all 66 blocks have it (a pure run: every window of the stripe's decisions P-periodic, in
// Q, none of its decisions in S); clean = the blocks before the first chunk with a break (they all
// have the period P).  Stops at the first such chunk.  Full stripes only
// (loads reach block 71: inside the text pad for every stripe but the last).
// (tools/microbench/stream_runs.hip k_pure_v1: this loop alone reads the 1 GiB rr text at 5.6 TB/s)
constexpr u32 RM_CH = 8;
__device__ __forceinline__ bool run_scan(const u8* __restrict__ Tw, u64* __restrict__ ring, u32 rs, u32 lane,
                                         u32& P, u32& clean) {
    auto load8 = [&](u32 k) -> u64 { return *(const u64*)(Tw + (u64)k * TAU); };
    u64 Q[3][RM_CH];
#pragma unroll
    for (u32 d = 0; d < 2; d++)
#pragma unroll
        for (u32 e = 0; e < RM_CH; e++) Q[d][e] = load8(d * RM_CH + e);
    u32 ol = 0, sh = 0;
    P = 0;
    clean = 0;
#pragma unroll
    for (u32 g = 0; g <= 9; g++) {
        const u32 c = RM_CH * g;
        if (g + 2 <= 8) {
#pragma unroll
            for (u32 e = 0; e < RM_CH; e++) Q[(g + 2) % 3][e] = load8(c + 2 * RM_CH + e);
        }
        if (g <= 8) {
#pragma unroll
            for (u32 e = 0; e < RM_CH; e++) ring[((c + e) % rs) * 64 + lane] = Q[g % 3][e];
        }
        __builtin_amdgcn_wave_barrier();
        if (g == 0) {
            // the period of block 1 (blocks 1, 2 in the ring)
            P = smallest_period(ring[64 + lane], ring[128 + lane], lane);
            if (!P) return false;
            ol = lane + (P >> 3);
            sh = 8 * (P & 7);
            continue;
        }
        u64 acc = 0;
#pragma unroll
        for (u32 j = 0; j < RM_CH; j++) {
            const u32 k = c - RM_CH + j;
            if (k > 65) break;
            const u32 o = (k % rs) * 64;
            const u64 lo = ring[(o + ol) % (rs * 64)], hi = ring[(o + ol + 1) % (rs * 64)];
            acc |= ring[o + lane] ^ (sh ? ((lo >> sh) | (hi << (64 - sh))) : lo);
        }
        if (__ballot(acc != 0)) return false;
        clean = min(c, 66u);
    }
    return true;
}

template <bool QSKIP, bool PASS1>
__global__ __launch_bounds__(64 * SWAVES, 5) void k_sss_stream(const u8* __restrict__ T, u64 n, u64 last_i,
                                                           const u16* __restrict__ qinfo, u64 nstripes,
                                                           pos_t* __restrict__ s_out, u32* __restrict__ s_cnt,
                                                           u32* __restrict__ s_flag, u32* __restrict__ ovf_ctr,
                                                           u32 b, sss_pow32 PW, u32 scap, u64* __restrict__ hitw,
                                                           u16* __restrict__ q_init, u8* __restrict__ rp_init,
                                                           const u32* __restrict__ list,
                                                           const u32* __restrict__ list_cnt,
                                                           u8* __restrict__ blk_p, u16* __restrict__ blk_fo,
                                                           u16* __restrict__ blk_lo, u64 nbk,
                                                           u32* __restrict__ mark_flag, u32* __restrict__ tot) {
    const u32 lane = threadIdx.x & 63;
    // the stripe index is wave-uniform: keep it (and every address derived from it) in SGPRs
    const u64 wi = (u64)blockIdx.x * SWAVES + (u32)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    u64 w = wi;
    if (list) {
        if (wi >= *list_cnt) return;  // whole wave
        w = list[wi];
    } else if (wi >= nstripes) {
        return;
    }
    const u64 i0 = w * (u64)SD;
    const u64 jmax = n - TAU;                  // last position with a full window (n >= 2 tau here)
    const u64 ilim = min<u64>(last_i - i0, (u64)SD - 1);  // decisions i0 + u, u <= ilim
    const u32 nblk = (u32)min<u64>((u64)SNB, ilim / TAU + 1);
    // blocks k >= kend hold positions past the last full window (jmax): k TAU + TAU - 1 > jmax - i0
    const u32 kend = (u32)min<u64>((jmax + 1 - i0) / TAU, 0xFFFFFFFFull);
    // PASS1 filter state: hit bits per filter anchor (block k < 64: bit k of hw[r]; blocks 64, 65
    // of the last stripe: bits 2(k - 64) + r of hw2), confirmed hit in a decision block
    u64 hw0 = 0, hw1 = 0, hw2 = 0;
    bool dirty = false;
    auto filt = [&](u32 k, u64 Bk) {
#if SSS_VAR == 1
        return;
#endif
        // (filter anchors past jmax + 255 have no full window: the zero padding past n is periodic)
        const u64 a0 = i0 + (u64)k * TAU;
        const u32 f = sss_filter(Bk, lane) & ((a0 <= jmax + 255 ? 1u : 0u) | (a0 + 256 <= jmax + 255 ? 2u : 0u));
        // branch-free (a conditional target makes the compiler spill the words to scratch)
        const u64 lowk = k < 64 ? 1ull << (k & 63) : 0ull;
        hw0 |= (f & 1) ? lowk : 0ull;
        hw1 |= (f & 2) ? lowk : 0ull;
        hw2 |= k >= 64 ? (u64)f << ((2 * k) & 63) : 0ull;  // blocks 64, 65: bits 0..3
        // (a hit in the two halo blocks is left to the Q-anchor chain: stopping the stripe sends its
        // 64 blocks through k_sss_runs' slow path on one wave, 130 us for one stray hit on the
        // genome-like text against about 60 us of the chain)
        if (f && k < nblk) dirty = true;
    };
    u32 nout = 0;  // outputs of this stripe so far (uniform)
#if SSS_VAR == 2
    u32 vacc = 0;
#endif
    {
        // per-lane powers: pwl = b^(8 lane), ibl = b^(-8 (lane + 1))
        u32 pwl = 1, ibl = PW.ib8;
        {
            u32 f = PW.b8, g = PW.ib8;
            for (int d = 0; d < 6; d++) {
                if (lane & (1u << d)) {
                    pwl *= f;
                    ibl *= g;
                }
                f *= f;
                g *= g;
            }
        }
        const u32 nB = 0u - PW.B;
        auto load8 = [&](u64 k) -> u64 { return *(const u64*)(T + i0 + k * TAU + 8 * lane); };
        // Hp(s_k + 8 lane + e), e < 8, into h; carry = Hp(s_k) in, Hp(s_k+1) out (uniform)
        auto block_prefix = [&](u64 bytes, u32& carry, u32* h) {
            const u32 lo = (u32)bytes, hi = (u32)(bytes >> 32);
#if SSS_VAR == 3
            for (int e = 0; e < 8; e++) h[e] = (e < 4 ? lo : hi) + carry + e;
            carry += lo;
            return;
#endif
            u32 c[8], loc[8];
#pragma unroll
            for (int e = 0; e < 8; e++) c[e] = ((e < 4 ? lo : hi) >> (8 * (e & 3))) & 255u;
            loc[0] = 0;
#pragma unroll
            for (int e = 1; e < 8; e++) loc[e] = loc[e - 1] * b + c[e - 1];
            const u32 h8 = loc[7] * b + c[7];
            const u32 g = h8 * ibl;
            const u32 G = wave_prefix_add(g);
            const u32 hl = (carry + (G - g)) * pwl;  // Hp(s_k + 8 lane)
            h[0] = hl;
#pragma unroll
            for (int e = 1; e < 8; e++) h[e] = hl * PW.pwb[e] + loc[e];
            carry = (carry + (u32)__builtin_amdgcn_readlane((int)G, 63)) * PW.B;
        };
        // block k lies entirely in Q (every window T[j..j+512) is periodic): its Phi' is
        // INF at all 512 positions.  Uniform test on the anchors' intervals: anchor 0
        // must cover rel 127 (offset 0), anchors 1-3 all of rel 0..127, anchor 4 rel 0..126
        auto fullq = [&](uint4 q) -> bool {
            const u32 a0 = q.x & 0xFFFFu, a4 = q.z & 0xFFFFu;
            const bool m0 = (a0 >> 8) <= 127u && (a0 & 255u) >= 127u;
            const bool m1 = (q.x >> 24) == 0u && ((q.x >> 16) & 255u) >= 127u;
            const bool m2 = (q.y >> 8 & 255u) == 0u && (q.y & 255u) >= 127u;
            const bool m3 = (q.y >> 24) == 0u && ((q.y >> 16) & 255u) >= 127u;
            const bool m4 = (a4 >> 8) == 0u && (a4 & 255u) >= 126u;
            return m0 && m1 && m2 && m3 && m4;
        };
        // all-Q test of a block (uniform; one per block, carried from step to step)
        auto allq = [&](uint4 q) -> bool {
            if constexpr (!QSKIP) return false;
            const bool anyq = (q.x != 0xFF00FF00u) || (q.y != 0xFF00FF00u) || ((q.z & 0xFFFFu) != 0xFF00u);
            return __builtin_amdgcn_readfirstlane((int)anyq) && fullq(q);
        };
        // Phi'(s_k + 8 lane + e) from the prefix hashes of blocks k and k+1 (INF for Q
        // windows and past the last full window).  q holds the Q intervals of the block's
        // 5 anchors (s_k/128 + 0..4), loaded by the whole wave as one scalar load: the
        // per-lane test runs only when one of them is non-empty
        auto phi_block = [&](u64 k, const u32* h0, const u32* h1, uint4 q, u32* v) {
            const bool anyq = (q.x != 0xFF00FF00u) || (q.y != 0xFF00FF00u) || ((q.z & 0xFFFFu) != 0xFF00u);
#pragma unroll
            for (int e = 0; e < 8; e++) v[e] = h0[e] * nB + h1[e];
            const bool endblk = (u32)k >= kend;
            if (__builtin_amdgcn_readfirstlane((int)(anyq || endblk))) {
                // anchor r (0..4) of the block covers offsets (128r - 128, 128r]; its Q interval
                // [lo, hi] (rel = offset + 127 - 128r) is an offset interval, uniform per block:
                // the lane ORs the part that meets its 8 positions into an INF mask
                const int o = (int)(8 * lane);
                const u32 qa[5] = {q.x & 0xFFFFu, q.x >> 16, q.y & 0xFFFFu, q.y >> 16, q.z & 0xFFFFu};
                u32 bits = 0;
#pragma unroll
                for (int r = 0; r < 5; r++) {
                    const int lo = (int)(qa[r] >> 8), hi = min((int)(qa[r] & 255u), 127);
                    if (lo <= hi) {  // uniform
                        const int l = max(128 * r - 127 + lo - o, 0), h = min(128 * r - 127 + hi - o, 7);
                        if (l <= h) bits |= ((2u << h) - 1u) & ~((1u << l) - 1u);
                    }
                }
                if (endblk) {  // positions past the last full window
                    const u64 j0 = i0 + k * TAU + (u64)o;
                    const u64 keep = jmax >= j0 ? min<u64>(jmax - j0 + 1, 8) : 0;
                    bits |= 0xFFu & ~((1u << keep) - 1u);
                }
#pragma unroll
                for (int e = 0; e < 8; e++) v[e] |= 0u - ((bits >> e) & 1u);
            }
        };
        auto phi_or_inf = [&](bool full, u64 k, const u32* h0, const u32* h1, uint4 q, u32* v) {
            if (full) {
#pragma unroll
                for (int e = 0; e < 8; e++) v[e] = INF32;
            } else {
                phi_block(k, h0, h1, q, v);
            }
        };
        // Q intervals of the anchors of block k (uniform address: a scalar load); PASS1
        // assumes Q empty
        auto loadq = [&](u64 k) -> uint4 {
            if constexpr (PASS1) return make_uint4(0xFF00FF00u, 0xFF00FF00u, 0xFF00FF00u, 0xFF00FF00u);
            return *(const uint4*)(qinfo + ((i0 + k * TAU) >> 7));
        };

        // prologue: Hp for blocks 0 and 1, Phi'(block 0)
        u32 carry = 0;
        const u64 B0 = load8(0), B1 = load8(1);
        // bytes of blocks c + 2 .. c + 5 in flight at step c (four blocks ahead: a lone wave at the
        // kernel's tail otherwise waits on every load)
        u64 Ba = load8(2), Bb = load8(3), Bc = load8(4), Bd = load8(5);
        const uint4 qa = loadq(0);
        uint4 qb = loadq(1);
        u32 hA[8], hB[8], xA[8], xB[8];
        if constexpr (PASS1) {
            filt(0, B0);
            filt(1, B1);
        }
        // a stripe with a hit in its decision blocks is re-run; it stops here and build_sss
        // marks all of its anchors' tiles for the exact Q pass (k_sss_runs settles
        // most such stripes first)
        if (dirty) goto stripe_done;
        block_prefix(B0, carry, hA);
        block_prefix(B1, carry, hB);
        bool fA = allq(qa), fB = false;
        bool fq = allq(qb);  // all-Q flag of the block whose Phi' the next step computes
        bool hvalid = true;  // the prefix hash carry continues the last computed block
        phi_or_inf(fA, 0, hA, hB, qa, xA);
        pos_t* out = s_out + w * SCAP;
        // one decision block: x = Phi'(block c) (in), y = Phi'(block c+1) (out),
        // h0 = Hp(block c+1) (in), h1 <- Hp(block c+2); B = bytes of block c+2
        // Phi(j) = Hp(j+512) - b^512 Hp(j) does not depend on where the prefix hash starts
        // (the start's contribution cancels): the prefix hash of block k is needed only when
        // block k-1 or k is not all Q, and restarts from 0 after skipped blocks
        auto step = [&](u32 c, const u32* x, u32* y, const u32* h0, u32* h1, u64 B, uint4& qn, bool fx, bool& fy,
                        uint4 qc /* Q intervals of block c + 2 */) {
            const bool f1 = fq, f2 = allq(qc);
            if (!(f1 && f2)) {
                if (!hvalid) carry = 0;
                block_prefix(B, carry, h1);
            }
            hvalid = !(f1 && f2);
            phi_or_inf(f1, c + 1, h0, h1, qn, y);
            fy = f1;
            fq = f2;
            qn = qc;
            // both blocks all INF: every window minimum is INF, no decision of block c is in S
            if (fx && fy) return;
#if SSS_VAR == 2
            for (int e = 0; e < 8; e++) vacc ^= x[e] + y[e];
            return;
#endif
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
            // clamped to INF-1: then min(x, y) == m' <=> (min(x, y) == m and m != INF), as m <= min(x, y)
            const u32 g = min(min(suf_after, pre_before), INF32 - 1);
            // decisions: M[e] = wave mask of lanes whose position 8 lane + e is in S
            u64 M[8];
            u64 U = 0;
#pragma unroll
            for (int e = 0; e < 8; e++) {
                M[e] = __ballot(min(x[e], y[e]) == min3u(sx[e], g, py[e]));
                U |= M[e];
            }
            if (U) {
                // ordered emission: per-lane bit sets from the masks, a wave scan of their
                // counts gives each lane its slot (positions ascend with lane, then e)
                u32 mb = 0;
#pragma unroll
                for (int e = 0; e < 8; e++) mb |= __builtin_amdgcn_inverse_ballot_w64(M[e]) ? (1u << e) : 0u;
                const u64 rem = ilim - (u64)c * TAU;  // decisions of this block: offsets <= rem
                if (rem < (u64)TAU - 1) {
                    const int lim = (int)rem - (int)(8 * lane);  // keep e <= lim
                    mb = lim < 0 ? 0u : lim >= 7 ? mb : (mb & ((2u << lim) - 1u));
                }
                const u32 cnt = (u32)__popc(mb);
                const pos_t base = (pos_t)(i0 + c * TAU + 8 * lane);
                if (!__ballot(cnt > 1)) {
                    // usual case (sparse S): at most one output per lane, slot = lanes below with one
                    const u64 has = __ballot(cnt != 0);
                    const u32 o = nout + (u32)__builtin_amdgcn_mbcnt_hi((u32)(has >> 32),
                                                                        __builtin_amdgcn_mbcnt_lo((u32)has, 0u));
                    if (cnt && o < (u32)SCAP) out[o] = base + (pos_t)__builtin_ctz(mb);
                    nout += (u32)__popcll(has);
                } else {
                    const u32 incl = wave_prefix_add(cnt);
                    u32 o = nout + incl - cnt;
                    for (u32 m = mb; m; m &= m - 1) {
                        if (o < (u32)SCAP) out[o] = base + (pos_t)__builtin_ctz(m);
                        o++;
                    }
                    nout += (u32)__builtin_amdgcn_readlane((int)incl, 63);
                }
            }
        };
        // PASS1 filters block c + 2 at step c (blocks 0 .. nblk + 1 in all: windows of the
        // stripe's decisions reach two blocks past its end); a hit in a decision block ends
        // the stripe (it is re-run)
        for (u32 c = 0; c < nblk; c += 2) {
            const u64 N0 = load8(c + 6);  // prefetch (the text pad covers the stripe's end)
            if constexpr (PASS1) {
                filt(c + 2, Ba);
                if (dirty) break;
            }
            step(c, xA, xB, hB, hA, Ba, qb, fA, fB, loadq(c + 2));
            if (c + 1 >= nblk) break;
            const u64 N1 = load8(c + 7);
            if constexpr (PASS1) {
                filt(c + 3, Bb);
                if (dirty) break;
            }
            step(c + 1, xB, xA, hA, hB, Bb, qb, fB, fA, loadq(c + 3));
            Ba = Bc;
            Bb = Bd;
            Bc = N0;
            Bd = N1;
        }
    }
stripe_done:
#if SSS_VAR == 2
    if (vacc == 0x9e3779b9u) nout++;
#endif
    if constexpr (PASS1) {
        if (lane == 0) {
            hitw[3 * w] = hw0;
            hitw[3 * w + 1] = hw1;
            hitw[3 * w + 2] = hw2 | (dirty ? 1ull << 63 : 0ull);
            // filter hits of a stripe that runs on (halo blocks): their tiles need the Q-anchor pass
            // (the stopped stripes are k_sss_runs' to report); one flag, no atomic once it is set
            if (!dirty && (hw0 | hw1 | hw2) && __hip_atomic_load(mark_flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u)
                atomicOr(mark_flag, 1u);
        }
        // (the Q intervals and periods of the anchors are not cleared here: build_sss clears
        // them only when some tile needs the Q-anchor pass, or a stripe the fallback)
        // the per-block run records start out unknown (k_sss_runs writes the stripes it
        // settles); the last stripe also clears the blocks past its own, up to nbk inclusive
        {
            const u64 gk = w * (u64)SNB + lane;
            if (gk <= nbk) {
                blk_p[gk] = 0;
                blk_fo[gk] = 0;
                blk_lo[gk] = 0;
            }
            if (w + 1 == nstripes) {
                for (u64 g2 = gk + 64; g2 <= nbk; g2 += 64) {
                    blk_p[g2] = 0;
                    blk_fo[g2] = 0;
                    blk_lo[g2] = 0;
                }
            }
        }
        if (dirty) nout = 0;  // re-run
    }
    if (lane == 0) {
        const u32 fl = nout > scap ? 1u : 0u;
        const u32 old = PASS1 ? 0u : s_flag[w];
        // |S| as 64 partial sums (same-address atomics from every stripe would serialize); a re-run
        // replaces the stripe's earlier count
        const u32 dn = nout - (PASS1 ? 0u : s_cnt[w]);
        if (dn) atomicAdd(tot + (w & 63), dn);
        s_cnt[w] = nout;
        s_flag[w] = fl;
        if (fl != old) atomicAdd(ovf_ctr, fl ? 1u : 0xFFFFFFFFu);
    }
}

// ---------------------------------------------------------------------------
// k_sss_runs: the exact sync set of the stripes pass 1 stopped (a confirmed filter hit in a
// decision block), in one pass over the stripe when its periodic windows lie in runs.
//
// For a period p, a p-break is a position z with T[z] != T[z+p]; a window T[j..j+512) is
// p-periodic iff it holds no p-break in [j, j+511-p].  A window in Q (period q <= 170) that is
// not p-periodic holds no p-periodic stretch of p + 170 bytes: such a stretch has the periods p
// and q and is longer than p + q - gcd(p, q), so gcd(p, q) is one of its periods (Fine-Wilf);
// as it covers q consecutive bytes of the window, the window has the period gcd(p, q) | p and
// would be p-periodic.  With the period p of the current run every window of a block is
//   p-periodic                       -> in Q
//   holding a p-periodic stretch of p + 170 bytes -> not in Q
//   without a hit of its filter anchor (sss_filter has no false negatives) -> not in Q
// and the windows none of this settles (at a change of period) are classified again with the
// smallest period of the first of them.  A stripe that still has unsettled windows is left to
// the exact Q-anchor path (k_q_anchors + the QSKIP re-run).  Run-heavy text (rr: nearly every
// window periodic, periods 1..170) is thereby settled in this one pass.  The kernel also writes
// the per-block run records of the LCE (lce_dev.h run_tab::bp).

// bit e <=> byte e of d is nonzero
__device__ __forceinline__ u32 byte_mask8(u64 d) {
    auto m4 = [](u32 x) -> u32 {
        u32 t = x | (x >> 4);
        t |= t >> 2;
        t |= t >> 1;
        t &= 0x01010101u;
        return ((t * 0x00204081u) >> 21) & 0xFu;  // bytes 0..3 -> bits 21..24
    };
    return m4((u32)d) | (m4((u32)(d >> 32)) << 4);
}
__device__ __forceinline__ u32 mask_le(int t) { return t < 0 ? 0u : t >= 7 ? 0xFFu : ((2u << t) - 1u); }        // e <= t
__device__ __forceinline__ u32 mask_ge(int t) { return t <= 0 ? 0xFFu : t > 7 ? 0u : ((0xFFu << t) & 0xFFu); }  // e >= t

// Classification of the windows j = 8 lane + e of a block k with the period p, from the
// p-differences T[z] ^ T[z+p] of the lane's positions in blocks k (pd0) and k + 1 (pd1).
// Returns the lane's mask of p-periodic windows; *u = the windows it does not settle.
// Positions are block-relative; a window's p-breaks lie in [j, j + 511 - p].
__device__ u32 q_classify(u64 pd0, u64 pd1, u32 p, u32 lane, u32& u) {
    constexpr u32 NB = 1u << 12;  // no p-break
    const u32 m0 = byte_mask8(pd0), m1 = byte_mask8(pd1);
    const u32 b0 = 8 * lane, b1 = 512 + 8 * lane;
    const int hb0 = m0 ? 31 - __builtin_clz(m0) : -1, hb1 = m1 ? 31 - __builtin_clz(m1) : -1;
    const u32 f0 = m0 ? b0 + __builtin_ctz(m0) : NB, f1 = m1 ? b1 + __builtin_ctz(m1) : NB;
    const u32 S1 = wave_suffix_min(f1, lane);
    const u32 S0n = dpp<0x130>(NB, wave_suffix_min(f0, lane)), S1n = dpp<0x130>(NB, S1);
    const u32 F1 = (u32)__builtin_amdgcn_readlane((int)S1, 0);
    const u32 nx0 = min(S0n, F1), nx1 = S1n;  // first p-break past the lane's positions in block k / k+1
    // a p-break followed by 170 positions without one (a p-periodic stretch of p + 170 bytes
    // after it): only a lane's highest p-break can be one
    const u32 la0 = (m0 && nx0 >= b0 + (u32)hb0 + 171u) ? b0 + (u32)hb0 : NB;
    const u32 la1 = (m1 && nx1 >= b1 + (u32)hb1 + 171u) ? b1 + (u32)hb1 : NB;
    const u32 SL0n = dpp<0x130>(NB, wave_suffix_min(la0, lane));
    const u32 L1 = (u32)__builtin_amdgcn_readlane((int)wave_suffix_min(la1, lane), 0);
    const u32 R = min(SL0n, L1);  // the first such p-break past the lane's positions
    const int ip = (int)p, rb = (int)b0;
    const u32 above = hb0 < 0 ? 0xFFu : ((0xFFu << (hb0 + 1)) & 0xFFu);   // no p-break of the lane in [e, 8)
    const u32 per = above & mask_le((int)nx0 - rb - 512 + ip);             // none in [j, j + 511 - p]
    const u32 longA = above & mask_le((int)nx0 - rb - 170);                // none in [j, j + 169]
    const u32 longB = (la0 != NB ? mask_le(hb0) : 0u) | mask_ge((int)R - rb - 341 + ip);  // one at z <= j + 341 - p
    u = ~per & ~(longA | longB) & 0xFFu;
    return per;
}
// the smallest period q <= 170 of the window T[j..j+512) (0: none): T[z] == T[z + q] for z in
// [j, j + 512 - q).  Candidates are the shifts at which the window's first 8 bytes recur (as in
// smallest_period), each verified by one masked compare of the window's words (lane L: bytes
// 8L .. 8L + 7) against the shifted ones
__device__ u32 find_period(const u8* __restrict__ T, u64 j, u32 lane) {
    const u64 W = ldu64(T + j + 8 * lane), W2 = ldu64(T + j + TAU + 8 * lane);
    const u64 A = ((u64)(u32)__builtin_amdgcn_readlane((int)(u32)(W >> 32), 0) << 32) |
                  (u32)__builtin_amdgcn_readlane((int)(u32)W, 0);
    const u32 j0 = (3 * lane + 1) >> 3;
    const u64 w0 = shfl64(W, j0 & 63), w1 = shfl64(W, (j0 + 1) & 63), w2 = shfl64(W, (j0 + 2) & 63);
    u64 m[3];
#pragma unroll
    for (u32 k = 0; k < 3; k++) {
        const u32 q = 3 * lane + 1 + k, r = q - 8 * j0;  // r <= 9
        const u64 v = r == 0 ? w0 : r < 8 ? (w0 >> (8 * r)) | (w1 << (64 - 8 * r))
                                 : r == 8 ? w1 : (w1 >> (8 * (r - 8))) | (w2 << (64 - 8 * (r - 8)));
        m[k] = __ballot(q <= QL && v == A);
    }
    for (;;) {
        u32 q = 0xFFFFu;
#pragma unroll
        for (u32 k = 0; k < 3; k++)
            if (m[k]) q = min(q, 3u * (u32)__builtin_ctzll(m[k]) + 1 + k);
        if (q > QL) return 0;
        m[(q - 1) % 3] &= ~(1ull << ((q - 1) / 3));
        const u32 len = TAU - q, o = 8 * lane;
        u64 a = W, c = shifted8(W, W2, q, lane);
        bool bad = false;
        if (o < len) {
            if (len - o < 8) {
                const u64 mk = (1ull << (8 * (len - o))) - 1;
                a &= mk;
                c &= mk;
            }
            bad = a != c;
        }
        if (!__ballot(bad)) return q;
    }
}
// first / last nonzero byte of a wave's 512 p-differences (block offsets), -1 if none
__device__ __forceinline__ int first_diff(u64 d) {
    const u64 b = __ballot(d != 0);
    if (!b) return -1;
    const u32 L = (u32)__builtin_ctzll(b);
    const u64 v = ((u64)(u32)__builtin_amdgcn_readlane((int)(u32)(d >> 32), (int)L) << 32) |
                  (u32)__builtin_amdgcn_readlane((int)(u32)d, (int)L);
    return (int)(8 * L + (__builtin_ctzll(v) >> 3));
}
__device__ __forceinline__ int last_diff(u64 d) {
    const u64 b = __ballot(d != 0);
    if (!b) return -1;
    const u32 L = 63u - (u32)__builtin_clzll(b);
    const u64 v = ((u64)(u32)__builtin_amdgcn_readlane((int)(u32)(d >> 32), (int)L) << 32) |
                  (u32)__builtin_amdgcn_readlane((int)(u32)d, (int)L);
    return (int)(8 * L + ((63 - __builtin_clzll(v)) >> 3));
}

// (113 VGPRs = 4 waves per SIMD; bounding it to the 5 its LDS allows spills 17 VGPRs and was
// slower on rr: 0.518 vs 0.483 ms for the SSS kernels, tools/gpu_r03b.sh)
// (one wave per workgroup: a workgroup's slot is held until its slowest wave ends, and a stripe
// with run boundaries walks several times longer than a pure run)
constexpr int RWAVES = 1;
__global__ __launch_bounds__(64 * RWAVES) __attribute__((amdgpu_waves_per_eu(4))) void k_sss_runs(const u8* __restrict__ T, u64 n, u64 last_i, u64 nstripes,
                                                        pos_t* __restrict__ s_out, u32* __restrict__ s_cnt,
                                                        u32* __restrict__ s_flag, u32* __restrict__ ovf_ctr, u32 b,
                                                        sss_pow32 PW, u32 scap, u64* __restrict__ hitw,
                                                        u8* __restrict__ blk_p, u16* __restrict__ blk_fo,
                                                        u16* __restrict__ blk_lo, u64 nbk, u32* __restrict__ any_q,
                                                        u32* __restrict__ dbg, u32* __restrict__ tot,
                                                        u32* __restrict__ prof, int scan) {
    // a ring of RSL blocks per wave in LDS: the bytes at offset p of a block are two aligned word
    // reads (the block after it follows in the ring).  The text arrives RCH blocks at a time in
    // registers, loaded one chunk ahead (a register rotation per block would make every load
    // wait for the one before: one load in flight)
    constexpr u32 RSL = 16, RCH = 8;
    __shared__ u64 s_ring[RWAVES][RSL * 64];
    const u32 lane = threadIdx.x & 63;
    u64* ring = s_ring[threadIdx.x >> 6];
    const u64 w = (u64)blockIdx.x * RWAVES + (u32)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    if (w >= nstripes) return;
    if (!(hitw[3 * w + 2] >> 63)) return;  // settled by pass 1
    const u64 t_start = prof ? (u64)clock64() : 0;  // LZ77SSS_RUNS_PROF: per-stripe clocks and counts
    u32 n_phi = 0, n_cross = 0;
    const u64 i0 = w * (u64)SD;
    // phase 1 (full stripes but the last): the run scan.  A pure run is settled here with the
    // records and flags the walk below would produce for it (block 0: period P, first break
    // unknown; blocks 1 .. 63: period P, no break; some window in Q; no sync position); any other
    // stripe keeps its run map for the walk's crossings
    const bool map_ok = scan && w + 1 < nstripes;
    u32 mp = 0, m64 = 0, m65 = 0;
    if (map_ok) {
        u32 P0, clean;
        const bool pure = run_scan(T + i0 + 8 * lane, ring, RSL, lane, P0, clean);
        // the run map for the walk's crossings: the blocks before `clean` have the period P0
        mp = lane < clean ? P0 : 0u;
        m64 = clean > 64 ? P0 : 0u;
        m65 = clean > 65 ? P0 : 0u;
        if (pure) {
            const u64 gk = w * (u64)SNB + lane;  // < nbk (not the last stripe)
            blk_p[gk] = (u8)P0;
            blk_fo[gk] = lane ? (u16)0xFFFFu : (u16)0;
            blk_lo[gk] = 0;
            if (prof && lane == 0) {
                prof[4 * w] = (u32)t_start;
                prof[4 * w + 1] = 0;
            }
            if (lane == 0) {
                hitw[3 * w] = 0;
                hitw[3 * w + 1] = 0;
                hitw[3 * w + 2] = 1ull << 62;  // settled
                if (__hip_atomic_load(any_q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u) atomicOr(any_q, 1u);
                if (__hip_atomic_load(any_q + 4, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u) atomicOr(any_q + 4, 1u);
            }
            return;
        }
        __builtin_amdgcn_wave_barrier();  // (the walk's prologue refills the ring)
    }
    const u64 jmax = n - TAU;
    const u64 ilim = min<u64>(last_i - i0, (u64)SD - 1);
    const u32 nblk = (u32)min<u64>((u64)SNB, ilim / TAU + 1);
    const u32 kend = (u32)min<u64>((jmax + 1 - i0) / TAU, 0xFFFFFFFFull);
    const u64 gk0 = i0 / TAU;
    u32 pwl = 1, ibl = PW.ib8;
    {
        u32 f = PW.b8, g = PW.ib8;
        for (int d = 0; d < 6; d++) {
            if (lane & (1u << d)) {
                pwl *= f;
                ibl *= g;
            }
            f *= f;
            g *= g;
        }
    }
    const u32 nB = 0u - PW.B;
    auto load8 = [&](u64 k) -> u64 { return *(const u64*)(T + i0 + k * TAU + 8 * lane); };
    // (other lanes read the words: a wavefront fence orders the writes before their reads)
    auto ring_sync = [&]() {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    };
    // bytes at offset 8 lane + p of block k (blocks k, k + 1 in the ring)
    auto ring_shift = [&](u32 k, u32 p) -> u64 {
        const u32 o = (k % RSL) * 64 + lane + (p >> 3), sh = 8 * (p & 7);
        const u64 lo = ring[o % (RSL * 64)];
        if (!sh) return lo;
        const u64 hi = ring[(o + 1) % (RSL * 64)];
        return (lo >> sh) | (hi << (64 - sh));
    };
    auto block_prefix = [&](u64 bytes, u32& carry, u32* h) {
        const u32 lo = (u32)bytes, hi = (u32)(bytes >> 32);
        u32 c[8], loc[8];
#pragma unroll
        for (int e = 0; e < 8; e++) c[e] = ((e < 4 ? lo : hi) >> (8 * (e & 3))) & 255u;
        loc[0] = 0;
#pragma unroll
        for (int e = 1; e < 8; e++) loc[e] = loc[e - 1] * b + c[e - 1];
        const u32 h8 = loc[7] * b + c[7];
        const u32 g = h8 * ibl;
        const u32 G = wave_prefix_add(g);
        const u32 hl = (carry + (G - g)) * pwl;
        h[0] = hl;
#pragma unroll
        for (int e = 1; e < 8; e++) h[e] = hl * PW.pwb[e] + loc[e];
        carry = (carry + (u32)__builtin_amdgcn_readlane((int)G, 63)) * PW.B;
    };
    auto valid_mask = [&](u32 k) -> u32 {
        if (k < kend) return 0xFFu;
        const u64 j0 = i0 + (u64)k * TAU + 8 * lane;
        return jmax >= j0 ? mask_le((int)min<u64>(jmax - j0, 7)) : 0u;
    };
    // filter anchor hits of window j = 8 lane + e of a block: A0, A1 of the block (bits 0, 1),
    // A0 of the next (bit 2)
    auto hit_mask = [&](u32 hits) -> u32 {
        if (lane == 0) return ((hits & 1) ? 1u : 0u) | ((hits & 2) ? 0xFEu : 0u);
        if (lane < 32) return (hits & 2) ? 0xFFu : 0u;
        if (lane == 32) return ((hits & 2) ? 1u : 0u) | ((hits & 4) ? 0xFEu : 0u);
        return (hits & 4) ? 0xFFu : 0u;
    };
    // the smallest p <= 170 with T[z] == T[z+p] for every z of ring block k (bytes Bx), 0 if none
    auto block_period = [&](u32 k, u64 Bx) -> u32 { return smallest_period(Bx, ring[((k + 1) % RSL) * 64 + lane], lane); };

    u32 p = 1;  // the period of the current run
    bool fail = false, anyq = false;
    u32 nout = 0;
    u32 n_cls = 0, n_find = 0;  // slow classifications, period searches (debug counters)
    pos_t* out = s_out + w * SCAP;
    // run records of the stripe's blocks, lane k holding block k's (stored together at the end):
    // the period when the block is p-extendable (rp), the first break in it of the period in
    // effect before it (rf: the exact end of the previous block's run), at a segment start the
    // last break of its period in the block before (rl: the exact start of its run).  Offsets + 1;
    // 0 = unknown, 0xFFFF = no such break (lce_dev.h run_tab)
    u32 rp = 0, rf = 0, rl = 0, prev_rec = 0;
    auto put_rec = [&](u32 k, bool ext, int fo, int lo) {
        const u32 rec = ext ? p : 0u;
        const u32 f = fo == -2 ? 0u : fo < 0 ? 0xFFFFu : (u32)(fo + 1);
        if (lane == k) {
            rp = rec;
            rf = f;
            if (lo >= -1) rl = lo < 0 ? 0xFFFFu : (u32)(lo + 1);
        }
        prev_rec = rec;
    };
    // last break of period p in ring block k - 1 (block k follows): the exact start of a new run
    auto seg_lo = [&](u32 k, u64 Bprev) -> int { return last_diff(Bprev ^ ring_shift(k - 1, p)); };

    // Q mask of block k (bytes B0k, B1k of blocks k, k + 1; ring holds k .. k + 2; p-differences
    // pd0, pd1 of blocks k, k + 1 for the current period, updated when it changes), slow path
    auto classify = [&](u32 k, u64 B0k, u64 B1k, u64& pd0, u64& pd1) -> u32 {
        const u32 vm = valid_mask(k);
        u32 u;
        n_cls++;
        u32 q = q_classify(pd0, pd1, p, lane, u);
        u &= vm;
        if (__ballot(u != 0)) {
            const u32 h = sss_filter(B0k, lane) | ((sss_filter(B1k, lane) & 1u) << 2);
            u &= hit_mask(h);
            // a change of period: classify again with the smallest period of block k + 1 (where
            // the windows of block k end), then of block k, then of the first unsettled window;
            // the period that settles them is kept for the blocks after
            // The third try's period search also decides the first unsettled window exactly
            // (find_period: 0 = not in Q, else in Q).  More tries settle few more stripes and cost
            // far more (12 tries: k_sss_runs 320 -> 546 us on the 1 GiB repetitive text, 31 -> 24
            // stripes left to the Q-anchor path)
            constexpr int MAX_TRY = 3;
            for (int t = 0; t < MAX_TRY && __ballot(u != 0); t++) {
                u32 p2;
                if (t == 0) {
                    p2 = block_period(k + 1, B1k);
                } else if (t == 1) {
                    p2 = block_period(k, B0k);
                } else {
                    const u64 ub = __ballot(u != 0);
                    const u32 L = (u32)__builtin_ctzll(ub);
                    const u32 e = (u32)__builtin_ctz((u32)__builtin_amdgcn_readlane((int)u, (int)L));
                    p2 = find_period(T, i0 + (u64)k * TAU + 8 * L + e, lane);
                    if (lane == L) {
                        u &= ~(1u << e);
                        if (p2) q |= 1u << e;
                    }
                }
                n_find++;
                if (!p2 || p2 == p) continue;
                const u64 qd0 = B0k ^ ring_shift(k, p2), qd1 = B1k ^ ring_shift(k + 1, p2);
                u32 u2;
                q |= q_classify(qd0, qd1, p2, lane, u2);
                u &= u2;
                p = p2;
                pd0 = qd0;
                pd1 = qd1;
            }
            if (__ballot(u != 0)) fail = true;
        }
        q &= vm;
        if (__ballot(q != 0)) anyq = true;
        return q;
    };
    auto phi = [&](u32 k, const u32* h0, const u32* h1, u32 q, u32* v) {
#pragma unroll
        for (int e = 0; e < 8; e++) v[e] = h0[e] * nB + h1[e];
        u32 bits = q;
        if (k >= kend) {
            const u64 j0 = i0 + (u64)k * TAU + 8 * lane;
            const u64 keep = jmax >= j0 ? min<u64>(jmax - j0 + 1, 8) : 0;
            bits |= 0xFFu & ~((1u << keep) - 1u);
        }
#pragma unroll
        for (int e = 0; e < 8; e++) v[e] |= 0u - ((bits >> e) & 1u);
    };

    // prologue: blocks 0 .. RSL - 1 in the ring, the chunk after them loading (blocks past
    // nblk + 4 are never read: the text pad covers up to there); block 0 classified, Phi'(0).
    // Iteration c reads ring blocks c .. c + 3
    u64 R[RCH];
    auto load_chunk = [&](u32 k0) {
#pragma unroll
        for (u32 e = 0; e < RCH; e++) R[e] = load8(k0 + e);  // unconditional (in the pad): no phi copies
    };
    auto store_chunk = [&](u32 k0) {
#pragma unroll
        for (u32 e = 0; e < RCH; e++) ring[((k0 + e) % RSL) * 64 + lane] = R[e];
    };
    load_chunk(0);
    store_chunk(0);
    load_chunk(RCH);
    store_chunk(RCH);
    load_chunk(RSL);
    ring_sync();
    auto ring_blk = [&](u32 k) -> u64 { return ring[(k % RSL) * 64 + lane]; };
    u64 Bk1 = ring_blk(1);
    u64 pdk = ring_blk(0) ^ ring_shift(0, 1), pdk1 = Bk1 ^ ring_shift(1, 1);
    bool z1 = __ballot(pdk1 != 0) != 0;
    u32 hc[8], hn[8], x[8], y[8];  // Hp of block c+1 (hc), of block c+2 (hn); Phi' of blocks c, c+1
    u32 carry = 0;
    int hk = -1;  // the block whose Hp is in hc (prefix hashes continue from carry after it)
    bool fx;
    {
        const u64 B0 = ring_blk(0);
        const bool z0 = __ballot(pdk != 0) != 0;
        u32 q0 = 0xFFu;
        fx = !z0 && !z1;
        if (!fx) {
            q0 = classify(0, B0, Bk1, pdk, pdk1);
            z1 = __ballot(pdk1 != 0) != 0;
        } else if (i0 <= jmax) {
            anyq = true;
        }
        put_rec(0, __ballot(pdk != 0) == 0, -2, -2);
        if (!fx) {
            block_prefix(B0, carry, hc);
            block_prefix(Bk1, carry, hn);
            phi(0, hc, hn, q0, x);
#pragma unroll
            for (int e = 0; e < 8; e++) hc[e] = hn[e];
            hk = 1;
        }
    }
    const bool fail_pro = fail;  // block 0 unsettled
    // the ring and the loading chunk as after refill(c), for a crossing that jumped to c
    auto seek = [&](u32 c) {
        const u32 cb = c & ~(RCH - 1);
        load_chunk(cb);
        store_chunk(cb);
        load_chunk(cb + RCH);
        store_chunk(cb + RCH);
        load_chunk(cb + 2 * RCH);
        ring_sync();
    };
    auto refill = [&](u32 c) {
        if (c % RCH == 0 && c) {
            // blocks c + RCH .. c + 2 RCH - 1 replace c - RCH .. c - 1 (read no more); the next
            // chunk loads for RCH iterations
            store_chunk(c + RCH);
            load_chunk(c + 2 * RCH);
            ring_sync();
        }
    };
    u32 c = 0;
    for (; c < nblk && !fail; c++) {
        refill(c);
        u32 k = c + 1;
        bool z0;
        if (fx && !z1) {
            // the run goes on while block c + 2 has no p-break: every window of block c + 1
            // p-periodic, no decision of block c in S (Phi'(c), Phi'(c + 1) all INF); those
            // blocks are recorded together with the run's period (a tight loop: one p-difference
            // per block)
            const u32 cs = c;
            const u32 ol = lane + (p >> 3), sh = 8 * (p & 7);
            u64 d;
            // RB blocks per round: their ring reads are issued together and the first dirty one
            // found from the ballots (one LDS round trip per RB blocks instead of per block).  At c
            // the ring holds blocks c - c % 8 .. c - c % 8 + 15, so blocks c + 2 .. c + RB + 2 are
            // in it; the refills of the blocks crossed run after the reads
            constexpr u32 RB = 6;
            static_assert(RB + 2 <= RSL - RCH, "run-crossing batch must stay inside the ring");
            auto pdiff = [&](u32 k) -> u64 {  // p-differences of ring block k
                const u32 o = (k % RSL) * 64;
                const u64 lo = ring[(o + ol) % (RSL * 64)], hi = ring[(o + ol + 1) % (RSL * 64)];
                return ring[o + lane] ^ (sh ? ((lo >> sh) | (hi << (64 - sh))) : lo);
            };
            for (;;) {
                if (map_ok) {
                    // the run map: blocks whose entry is p have the period p, so the run goes on
                    // up to the first other one (t) without reading them; jump when that saves a
                    // chunk of loads (the blocks from t on are compared below as before)
                    const u64 cm = __ballot(mp == p);
                    const u32 from = c + 2;
                    u32 t = from;
                    if (from < 64) {
                        const u64 nc = ~cm & (~0ull << from);
                        t = nc ? (u32)__builtin_ctzll(nc) : 64u;
                    }
                    if (t == 64 && m64 == p) t = 65;
                    if (t == 65 && m65 == p) t = 66;
                    const u32 jt = min(t - 2, nblk);
                    if (jt >= c + RCH) {
                        n_cross += jt - c;
                        c = jt;
                        seek(c);
                        if (c >= nblk) break;
                    }
                }
                u32 f = RB;  // first block of the round with a p-break (uniform)
#pragma unroll
                for (u32 j = 0; j < RB; j++)
                    if (__ballot(pdiff(c + 2 + j) != 0) && f == RB) f = j;
                const u32 lim = nblk - c;  // >= 1
                const u32 adv = min(f, lim);
                if (f < lim) d = pdiff(c + 2 + f);  // (read again: no array of RB values held live)
                for (u32 j = 1; j <= adv; j++) refill(c + j);
                c += adv;
                n_cross += adv;
                if (f < RB || c >= nblk) break;
            }
            if (c > cs) {
                if (lane > cs && lane <= c) {
                    rp = p;
                    rf = 0xFFFFu;
                }
                prev_rec = p;
                hk = -1;
                if (i0 + (u64)(cs + 1) * TAU <= jmax) anyq = true;
            }
            if (c >= nblk) break;
            k = c + 1;
            Bk1 = ring_blk(k + 1);
            pdk = 0;  // block k: clean
            z0 = false;
            pdk1 = d;
            z1 = true;
        } else {
            Bk1 = ring_blk(k + 1);
            pdk = pdk1;
            z0 = z1;
            pdk1 = Bk1 ^ ring_shift(k + 1, p);
            z1 = __ballot(pdk1 != 0) != 0;
        }
        const u64 Bk = ring_blk(k);
        const int fok = z0 ? first_diff(pdk) : -1;  // before a change of period: the end of the last run
        bool allk = !z0 && !z1;  // no p-break in blocks k, k + 1: every window of block k is p-periodic
        u32 qk = 0xFFu;
        if (!allk) {
            qk = classify(k, Bk, Bk1, pdk, pdk1);
            z1 = __ballot(pdk1 != 0) != 0;
        } else if (i0 + (u64)k * TAU <= jmax) {
            anyq = true;
        }
        if (fail) break;
        const bool ext = __ballot(pdk != 0) == 0;
        put_rec(k, ext, fok, (ext && p != prev_rec) ? seg_lo(k, ring_blk(c)) : -2);
        // Phi'(block k)
        if (!allk) {
            if (hk != (int)k) {  // restart the prefix hash at block k (Phi is origin-free)
                carry = 0;
                block_prefix(Bk, carry, hc);
            }
            block_prefix(Bk1, carry, hn);
            phi(k, hc, hn, qk, y);
#pragma unroll
            for (int e = 0; e < 8; e++) hc[e] = hn[e];
            hk = (int)k + 1;
            n_phi++;
        }
        // decisions of block c from Phi'(c) = x and Phi'(c+1) = y
        if (!(fx && allk)) {
            u32 xx[8], yy[8];
#pragma unroll
            for (int e = 0; e < 8; e++) {
                xx[e] = fx ? INF32 : x[e];
                yy[e] = allk ? INF32 : y[e];
            }
            u32 sx[8], py[8];
            sx[7] = xx[7];
#pragma unroll
            for (int e = 6; e >= 0; e--) sx[e] = min(xx[e], sx[e + 1]);
            py[0] = yy[0];
#pragma unroll
            for (int e = 1; e < 8; e++) py[e] = min(py[e - 1], yy[e]);
            const u32 sufL = wave_suffix_min(sx[0], lane), preL = wave_prefix_min(py[7]);
            const u32 suf_after = dpp<0x130>(INF32, sufL);
            const u32 pre_before = dpp<0x138>(INF32, preL);
            const u32 g = min(min(suf_after, pre_before), INF32 - 1);
            u64 M[8];
            u64 U = 0;
#pragma unroll
            for (int e = 0; e < 8; e++) {
                M[e] = __ballot(min(xx[e], yy[e]) == min3u(sx[e], g, py[e]));
                U |= M[e];
            }
            if (U) {
                u32 mb = 0;
#pragma unroll
                for (int e = 0; e < 8; e++) mb |= __builtin_amdgcn_inverse_ballot_w64(M[e]) ? (1u << e) : 0u;
                const u64 rem = ilim - (u64)c * TAU;
                if (rem < (u64)TAU - 1) {
                    const int lim = (int)rem - (int)(8 * lane);
                    mb = lim < 0 ? 0u : lim >= 7 ? mb : (mb & ((2u << lim) - 1u));
                }
                const u32 cnt = (u32)__popc(mb);
                const pos_t base = (pos_t)(i0 + (u64)c * TAU + 8 * lane);
                const u32 incl = wave_prefix_add(cnt);
                u32 o = nout + incl - cnt;
                for (u32 m = mb; m; m &= m - 1) {
                    if (o < (u32)SCAP) out[o] = base + (pos_t)__builtin_ctz(m);
                    o++;
                }
                nout += (u32)__builtin_amdgcn_readlane((int)incl, 63);
            }
        }
#pragma unroll
        for (int e = 0; e < 8; e++) x[e] = y[e];
        fx = allk;
    }
    if (fail) {
        // the exact Q-anchor path takes the stripe; its remaining blocks still get their run
        // records (the LCE consults them on both sides of a comparison)
        const u32 k0 = fail_pro ? 1u : c + 1;
        u64 Bq = ring_blk(k0 - 1), B0x = ring_blk(k0), B1x = ring_blk(k0 + 1);
        for (u32 kk = k0; kk < (u32)SNB; kk++) {
            if (kk > k0) {
                Bq = B0x;
                B0x = B1x;
                B1x = load8(kk + 1);
            }
            u64 pd = B0x ^ shifted8(B0x, B1x, p, lane);
            // the first break of the period of the record before (a run's exact end): the failed
            // block's classification may have left p at another period already
            const u32 pr = prev_rec ? prev_rec : p;
            const int fo = first_diff(pr == p ? pd : B0x ^ shifted8(B0x, B1x, pr, lane));
            if (__ballot(pd != 0)) {
                const u32 p2 = smallest_period(B0x, B1x, lane);
                if (p2) {
                    p = p2;
                    pd = 0;
                }
            }
            const bool ext = __ballot(pd != 0) == 0;
            put_rec(kk, ext, fo, (ext && p != prev_rec) ? last_diff(Bq ^ shifted8(Bq, B0x, p, lane)) : -2);
        }
    }
    // the stripe's run records, one store per lane
    if (gk0 + lane < nbk) {
        blk_p[gk0 + lane] = (u8)rp;
        blk_fo[gk0 + lane] = (u16)rf;
        blk_lo[gk0 + lane] = (u16)rl;
    }
    // some block has a record: the segment kernels run (one flag for the text, no atomic once set)
    if (__ballot(gk0 + lane < nbk && rp != 0) && lane == 0 &&
        __hip_atomic_load(any_q + 4, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u)
        atomicOr(any_q + 4, 1u);
    // a stripe whose sync set overflows goes to the exact path too (k_sss_fallback reads the Q
    // intervals of k_q_anchors)
    const bool ovf = !fail && nout > scap;
    if (ovf) fail = true;
    if (prof && lane == 0) {
        const u64 t_end = clock64();
        prof[4 * w] = (u32)t_start;
        prof[4 * w + 1] = (u32)(t_end - t_start);
        prof[4 * w + 2] = min(n_cls, 0xFFFFu) | (min(n_find, 0xFFFFu) << 16) | (fail ? 0x80000000u : 0u);
        prof[4 * w + 3] = min(n_phi, 0xFFFFu) | (min(n_cross, 0xFFFFu) << 16);
    }
    if (lane == 0) {
        if (dbg) {  // (same-address atomics from every wave serialize: debug runs only)
            atomicAdd(dbg + 0, n_cls);
            atomicAdd(dbg + 1, n_find);
            atomicAdd(dbg + 2, fail ? 1u : 0u);
            atomicAdd(dbg + 3, ovf ? 1u : 0u);
        }
        if (fail) {  // left to the Q-anchor path (still forced)
            if (__hip_atomic_load(any_q + 5, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u) atomicOr(any_q + 5, 1u);
            return;
        }
        hitw[3 * w] = 0;
        hitw[3 * w + 1] = 0;
        hitw[3 * w + 2] = 1ull << 62;  // settled here
        // one flag for the whole text: no atomic once it is visible
        if (anyq && __hip_atomic_load(any_q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u) atomicOr(any_q, 1u);
        const u32 fl = nout > scap ? 1u : 0u;
        const u32 old = s_flag[w];
        if (nout) atomicAdd(tot + (w & 63), nout);  // |S| partial sums (pass 1 counted 0 here)
        s_cnt[w] = nout;
        s_flag[w] = fl;
        if (fl != old) atomicAdd(ovf_ctr, fl ? 1u : 0xFFFFFFFFu);
    }
}
// The per-block run records (pass 1 clears them, k_sss_runs writes the stripes it runs on; the
// clearing stores cost nothing measurable beside pass 1's work, where gating every read by the
// stripe's state made the segment kernels 11 us slower on the 1 GiB repetitive text)
struct blk_recs {
    const u8* bp;
    const u16* fo;
    const u16* lo;
    __device__ __forceinline__ u32 p(u64 b) const { return bp[b]; }
    __device__ __forceinline__ u32 f(u64 b) const { return fo[b]; }
    __device__ __forceinline__ u32 l(u64 b) const { return lo[b]; }
};
// per-block run end / start packed for one-load lookups (lce_dev.h run_tab::re / rs): the
// segment's end made exact by the first break of its period in the block after it (fo), its
// start by the last break in the block before it (lo); offsets + 1, 0 = unknown, 0xFFFF = none
// in that block (a bound one block further)
__global__ void k_blk_runinfo(blk_recs B, const pos_t* __restrict__ ser, const pos_t* __restrict__ ss, u64 nbk,
                              u64* __restrict__ re, u64* __restrict__ rs) {
    const u64 b = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= nbk) return;
    const u64 p = B.p(b);
    if (!p) {
        re[b] = 0;
        rs[b] = 0;
        return;
    }
    const u64 se = ser[nbk - 1 - b], eb = se >> 9;
    u64 e = se + p, xe = 0;
    if (eb < nbk) {
        const u32 f = B.f(eb);
        if (f == 0xFFFFu) e = se + TAU + p;
        else if (f) { e = se + (f - 1) + p; xe = 1; }
    }
    const u64 s0 = ss[b], sb = s0 >> 9;
    u64 st = s0, xs = 0;
    if (sb) {
        const u32 l = B.l(sb);
        if (l == 0xFFFFu) st = s0 - TAU;
        else if (l) { st = s0 - TAU + l; xs = 1; }
    }
    re[b] = (e << 16) | (xe << 8) | p;
    rs[b] = (st << 16) | (xs << 8) | p;
}
// Run-record segments (maximal runs of consecutive blocks with the same nonzero period) in
// two launches: k_blk_seg_tiles finds per tile of BT_TILE blocks its first segment end
// (first block b with !cont_f(b)) and last segment start (last b with !cont_b(b)); then
// k_blk_seg_info computes every block's segment end/start inside its tile by LDS scans,
// resolves segments that cross tile boundaries through the tile table (a wave-parallel
// search over 64 tiles per step) and writes the packed records.  Same values as the
// marker + min/max-scan formulation (k_blk_marks + two device scans + k_blk_runinfo).
constexpr u32 BT_T = 1024, BT_PER = 4, BT_TILE = BT_T * BT_PER;
constexpr u64 BT_NONE = ~0ull;
__device__ __forceinline__ bool blk_cont_f(const blk_recs& B, u64 nbk, u64 b) {
    const u32 p = B.p(b);
    return p && b + 1 < nbk && B.p(b + 1) == p;
}
__device__ __forceinline__ bool blk_cont_b(const blk_recs& B, u64 b) {
    const u32 p = B.p(b);
    return p && b > 0 && B.p(b - 1) == p;
}
__global__ __launch_bounds__(BT_T) void k_blk_seg_tiles(blk_recs bp, u64 nbk, u64* __restrict__ tfe,
                                                        u64* __restrict__ tls) {
    __shared__ u64 s_e[BT_T / 64], s_s[BT_T / 64];
    const u32 t = threadIdx.x, lane = t & 63, wv = t >> 6;
    const u64 t0 = (u64)blockIdx.x * BT_TILE;
    u64 fe = BT_NONE, ls = BT_NONE;
    for (u32 k = 0; k < BT_PER; k++) {
        const u64 b = t0 + (u64)k * BT_T + t;
        if (b >= nbk) break;
        if (fe == BT_NONE && !blk_cont_f(bp, nbk, b)) fe = b;
        if (!blk_cont_b(bp, b)) ls = b;
    }
    for (int o = 32; o >= 1; o >>= 1) {
        const u64 a = __shfl_xor(fe, o), c = __shfl_xor(ls, o);
        fe = min(fe, a);
        ls = (ls == BT_NONE) ? c : (c == BT_NONE ? ls : max(ls, c));
    }
    if (lane == 0) {
        s_e[wv] = fe;
        s_s[wv] = ls;
    }
    __syncthreads();
    if (t == 0) {
        u64 e = BT_NONE, l = BT_NONE;
        for (u32 k = 0; k < BT_T / 64; k++) {
            e = min(e, s_e[k]);
            if (s_s[k] != BT_NONE) l = (l == BT_NONE) ? s_s[k] : max(l, s_s[k]);
        }
        tfe[blockIdx.x] = e;
        tls[blockIdx.x] = l;
    }
}
__global__ __launch_bounds__(BT_T) void k_blk_seg_info(blk_recs bp, u64 nbk,
                                                       const u64* __restrict__ tfe, const u64* __restrict__ tls,
                                                       u64 ntile, u64* __restrict__ re, u64* __restrict__ rs) {
    // the tile's 64 groups of 64 blocks: per group the ballot masks of its segment ends
    // (!cont_f) and starts (!cont_b); a block's segment end is the first end at or after it (in
    // its group, else in the first later group that has one, else past the tile: s_after), its
    // start the last start at or before it.  One barrier, no scans (the LDS Hillis-Steele form
    // took 38-42 us on the 1 GiB repetitive text)
    static_assert(BT_TILE == 64 * 64, "64 groups of 64 blocks per tile");
    __shared__ u64 s_em[64], s_bm[64];
    __shared__ u64 s_after, s_before;
    const u32 t = threadIdx.x, lane = t & 63, wv = t >> 6;
    const u64 tile = blockIdx.x, t0 = tile * BT_TILE;
    const u64 tn = min<u64>(BT_TILE, nbk - t0);
    constexpr u32 GPW = BT_TILE / BT_T;  // groups per wave (4)
    u32 pv[GPW];
#pragma unroll
    for (u32 k = 0; k < GPW; k++) {
        const u32 g = wv * GPW + k, i = g * 64 + lane;
        const u64 b = t0 + i;
        const bool in = i < tn;
        const u32 p = in ? bp.p(b) : 0u;
        pv[k] = p;
        const bool cf = in && p && b + 1 < nbk && bp.p(b + 1) == p;
        const bool cb = in && p && b > 0 && bp.p(b - 1) == p;
        const u64 em = __ballot(in && !cf), bm = __ballot(in && !cb);
        if (lane == 0) {
            s_em[g] = em;
            s_bm[g] = bm;
        }
    }
    // the first segment end at or after the next tile, the last segment start before this
    // tile (wave 0 / wave 1 search the tile table 64 tiles per step)
    if (t < 64) {
        u64 r = BT_NONE;
        for (u64 base = tile + 1; base < ntile; base += 64) {
            const u64 x = base + lane < ntile ? tfe[base + lane] : BT_NONE;
            const u64 bal = __ballot(x != BT_NONE);
            if (bal) {
                const u32 L = (u32)__builtin_ctzll(bal);
                r = __shfl(x, (int)L);
                break;
            }
        }
        if (lane == 0) s_after = r;
    } else if (t < 128) {
        u64 r = BT_NONE;
        for (u64 top = tile; top > 0;) {
            const u64 lo_t = top >= 64 ? top - 64 : 0;
            const u64 idx = lo_t + lane;
            const u64 x = idx < top ? tls[idx] : BT_NONE;
            const u64 bal = __ballot(x != BT_NONE);
            if (bal) {
                const u32 L = 63u - (u32)__builtin_clzll(bal);
                r = __shfl(x, (int)L);
                break;
            }
            top = lo_t;
        }
        if (lane == 0) s_before = r;
    }
    __syncthreads();
    const u64 em_l = s_em[lane], bm_l = s_bm[lane];
    const u64 ge = __ballot(em_l != 0), gb = __ballot(bm_l != 0);  // groups holding an end / a start
#pragma unroll
    for (u32 k = 0; k < GPW; k++) {
        const u32 g = wv * GPW + k, i = g * 64 + lane;
        if (i >= tn) break;
        const u64 b = t0 + i;
        const u64 p = pv[k];
        if (!p) {
            re[b] = 0;
            rs[b] = 0;
            continue;
        }
        u64 eb;
        const u64 me = s_em[g] >> lane;  // ends at or after the block in its group
        if (me) {
            eb = b + (u64)__builtin_ctzll(me);
        } else {
            const u64 nx = g < 63 ? ge & (~0ull << (g + 1)) : 0ull;
            if (nx) {
                const u32 g2 = (u32)__builtin_ctzll(nx);
                eb = t0 + (u64)g2 * 64 + (u64)__builtin_ctzll(s_em[g2]);
            } else {
                eb = s_after;  // always found: the last block ends every segment
            }
        }
        u64 sb0;
        const u64 mb = s_bm[g] & (lane == 63 ? ~0ull : ((2ull << lane) - 1));  // starts at or before it
        if (mb) {
            sb0 = t0 + (u64)g * 64 + (63u - (u32)__builtin_clzll(mb));
        } else {
            const u64 pr = gb & ((1ull << g) - 1);
            if (pr) {
                const u32 g2 = 63u - (u32)__builtin_clzll(pr);
                sb0 = t0 + (u64)g2 * 64 + (63u - (u32)__builtin_clzll(s_bm[g2]));
            } else {
                sb0 = s_before;  // always found: block 0 starts every segment
            }
        }
        const u64 se = (eb + 1) * TAU, ebn = eb + 1;
        u64 e = se + p, xe = 0;
        if (ebn < nbk) {
            const u32 f = bp.f(ebn);
            if (f == 0xFFFFu) e = se + TAU + p;
            else if (f) { e = se + (f - 1) + p; xe = 1; }
        }
        const u64 s0 = sb0 * TAU, sb = sb0;
        u64 st = s0, xs = 0;
        if (sb) {
            const u32 l = bp.l(sb);
            if (l == 0xFFFFu) st = s0 - TAU;
            else if (l) { st = s0 - TAU + l; xs = 1; }
        }
        re[b] = (e << 16) | (xe << 8) | p;
        rs[b] = (st << 16) | (xs << 8) | p;
    }
}
// run-record segment markers: ends (stored reversed, for a min-scan) and starts (max-scan)
__global__ void k_blk_marks(blk_recs B, u64 nbk, pos_t* __restrict__ end_rev, pos_t* __restrict__ beg) {
    const u64 b = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= nbk) return;
    const bool cont_f = blk_cont_f(B, nbk, b), cont_b = blk_cont_b(B, b);
    end_rev[nbk - 1 - b] = cont_f ? (pos_t)~(pos_t)0 : (pos_t)((b + 1) * TAU);
    beg[b] = cont_b ? (pos_t)0 : (pos_t)(b * TAU);
}

// Per stripe: the re-run list starts with the stripes whose own blocks had a confirmed
// filter hit; per tile of 253 anchors: marked when a filter anchor A with A/128 in
// [first anchor, last anchor + 1] was hit (a window in Q with exact anchor a has its
// filter anchor in [a, a + 255]); the anchors past the last stripe's own ones (tail)
// start out empty.
__global__ void k_sss_marks(const u64* __restrict__ hitw, u64 nstripes, u64 ntiles, u64 tpad, u64 nanch,
                            u8* __restrict__ tflag, u32* __restrict__ sflag, u32* __restrict__ slist,
                            u32* __restrict__ scnt, u64 t_tail, u64 q_end, u16* __restrict__ qinfo,
                            u8* __restrict__ run_p) {
    const u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < nstripes) {
        // forced: pass 1 stopped the stripe and k_sss_runs could not settle it (bit 63); settled by
        // k_sss_runs (bit 62): exact already, never appended to the re-run by k_q_anchors
        const bool forced = (hitw[3 * i + 2] >> 63) != 0, settled = ((hitw[3 * i + 2] >> 62) & 1) != 0;
        sflag[i] = (forced || settled) ? 1u : 0u;
        if (forced) slist[atomicAdd(scnt, 1u)] = (u32)i;
    }
    if (i < ntiles) {
        // filter anchor f (position 256 f) of stripe f >> 7, block (f & 127) >> 1, half f & 1
        const u64 flo = (QT_OWN * i + 1) / 2, fhi = (QT_OWN * i + QT_OWN) / 2;
        bool d = false;
        for (u64 w = flo >> 7; w <= (fhi >> 7) && !d; w++) {
            const u64 ra = max<u64>(flo, w << 7) - (w << 7), rb = min<u64>(fhi, (w << 7) + 127) - (w << 7);
            if (w < nstripes) {
                // bits k with 2k + r in [ra, rb]
                auto mask = [](u64 lo, u64 hi) -> u64 {  // bits lo..hi (empty if lo > hi)
                    if (lo > hi) return 0;
                    return (hi >= 63 ? ~0ull : ((2ull << hi) - 1)) & ~((1ull << lo) - 1);
                };
                const u64 m0 = mask((ra + 1) / 2, rb / 2);
                const u64 m1 = rb >= 1 ? mask(ra / 2, (rb - 1) / 2) : 0;
                d = ((hitw[3 * w] & m0) | (hitw[3 * w + 1] & m1)) != 0;
            } else if (w == nstripes && nstripes) {
                // blocks 64, 65 of the last stripe: bits f - 128 w of its third word
                const u64 hi = min<u64>(rb, 3);
                if (ra <= hi) {
                    const u64 m = ((2ull << hi) - 1) & ~((1ull << ra) - 1);
                    d = (hitw[3 * (nstripes - 1) + 2] & m) != 0;
                }
            }
        }
        // a forced stripe w stopped filtering at its first hit: every anchor whose Q windows
        // its blocks 0..65 could hold, [256 w - 1, 256 w + 262) (to the end for the last)
        const u64 t0 = QT_OWN * i, t1 = t0 + QT_OWN;
        const u64 apw = SD / QA;
        for (u64 w = t0 >= apw + 262 ? (t0 - 262) / apw : 0; !d && w < nstripes && w * apw <= t1; w++) {
            if (!(hitw[3 * w + 2] >> 63)) continue;
            const u64 lo = w ? w * apw - 1 : 0, hi = w + 1 == nstripes ? ~0ull : w * apw + apw + 6;
            d = lo < t1 && t0 < hi;
        }
        tflag[i] = d ? 1 : 0;
    } else if (i < tpad) {
        tflag[i] = 0;
    }
    if (t_tail + i < q_end) {
        qinfo[t_tail + i] = 0xFF00;
        if (t_tail + i < nanch) run_p[t_tail + i] = 0;
    }
}

// one workgroup: the sorted list of set flags (tiles to compute).  flag is padded with
// zeros to a multiple of 16 * 1024 bytes; each thread owns a run of 16-byte words.
// Flag bytes (0/1) -> the sorted list of flagged indices.  Block b owns the 16-byte
// words [1024 b, 1024 b + 1024) (16 Ki flags; one word per thread): k_flag_count
// writes the block's count, k_flag_list adds the counts of the blocks before it (a
// workgroup-parallel sum) and writes its indices in order.  (One workgroup over all the
// flags took 43 us for the 67 K tiles of a 1 GiB run-heavy text.)
constexpr u32 FL_T = 1024;
__device__ __forceinline__ u32 flag_word_count(const u8* __restrict__ flag, u64 nwords, u64 w, uint4& v) {
    v = w < nwords ? ((const uint4*)flag)[w] : make_uint4(0u, 0u, 0u, 0u);
    return __popc(v.x) + __popc(v.y) + __popc(v.z) + __popc(v.w);  // flags are 0/1 bytes
}
__global__ __launch_bounds__(FL_T) void k_flag_count(const u8* __restrict__ flag, u64 nwords, u32* __restrict__ bcnt) {
    __shared__ u32 s_w[FL_T / 64];
    const u32 t = threadIdx.x;
    uint4 v;
    u32 c = flag_word_count(flag, nwords, (u64)blockIdx.x * FL_T + t, v);
    c = wave_prefix_add(c);
    if ((t & 63) == 63) s_w[t >> 6] = c;
    __syncthreads();
    if (t == 0) {
        u32 tot = 0;
        for (u32 k = 0; k < FL_T / 64; k++) tot += s_w[k];
        bcnt[blockIdx.x] = tot;
    }
}
__global__ __launch_bounds__(FL_T) void k_flag_list(const u8* __restrict__ flag, u64 nwords, const u32* __restrict__ bcnt,
                                                    u32* __restrict__ list, u32* __restrict__ cnt) {
    __shared__ u32 s_w[FL_T / 64];
    __shared__ u32 s_part[FL_T / 64];
    __shared__ u32 s_base;
    const u32 t = threadIdx.x, lane = t & 63, wv = t >> 6;
    const u64 w = (u64)blockIdx.x * FL_T + t;
    {
        // the counts of the blocks before this one, summed by the whole workgroup (a 2^40-byte
        // text has ~4 K blocks: a one-thread sum per block would be quadratic in total)
        u32 b = 0;
        for (u32 k = t; k < blockIdx.x; k += FL_T) b += bcnt[k];
        for (int o = 32; o >= 1; o >>= 1) b += __shfl_xor(b, o);
        if (lane == 0) s_part[wv] = b;
        __syncthreads();
        if (t == 0) {
            u32 tot = 0;
            for (u32 k = 0; k < FL_T / 64; k++) tot += s_part[k];
            s_base = tot;
            if (blockIdx.x + 1 == gridDim.x) *cnt = tot + bcnt[blockIdx.x];
        }
    }
    uint4 v;
    const u32 c = flag_word_count(flag, nwords, w, v);
    const u32 incl = wave_prefix_add(c);
    if (lane == 63) s_w[wv] = incl;
    __syncthreads();
    if (t == 0) {
        u32 tot = s_base;
        for (u32 k = 0; k < FL_T / 64; k++) {
            const u32 x = s_w[k];
            s_w[k] = tot;
            tot += x;
        }
    }
    __syncthreads();
    u32 o = s_w[wv] + incl - c;
    const u32 wd[4] = {v.x, v.y, v.z, v.w};
    for (int q = 0; q < 4; q++)
        for (u32 b = wd[q]; b; b &= b - 1) list[o++] = (u32)(w * 16 + 4 * q + (__builtin_ctz(b) >> 3));
}

// Exact path for stripes whose output buffer overflowed (dense sync sets, e.g.
// hash-adversarial text): one 256-thread workgroup per stripe, everything
// parallel.  (1) Phi' of the stripe's windows: thread t hashes a contiguous run
// of ~130 windows (one direct 512-byte hash, then rolls), Q windows -> INF;
// (2) van Herk / Gil-Werman 512-block prefix and suffix minima (one thread per
// block and direction); (3) m_i = min(suf[i], pre[i + 511], Phi'[i + 512]) and the
// membership test per decision; (4) ordered compaction: each thread owns 128
// consecutive decisions, a block scan of their counts gives the offsets.
constexpr int FB_T = 256;
constexpr int FB_DEC = SD / FB_T;  // decisions per thread (128)
__global__ __launch_bounds__(FB_T) void k_sss_fallback(const u8* __restrict__ T, u64 n, u64 last_i,
                                                       const u16* __restrict__ qinfo, const u32* __restrict__ lanes,
                                                       u32* __restrict__ scratch, pos_t* __restrict__ ovf_out,
                                                       u32* __restrict__ lane_cnt, u32 b, u32 bpow) {
    __shared__ u32 s_cnt[FB_T];
    const u64 lane = lanes[blockIdx.x];
    const u64 i0 = lane * SD;
    const u64 i_end = min(i0 + SD, last_i + 1);
    const u64 j_end = min(i0 + SD + TAU - 1, n - TAU);  // last window needed (a full one)
    const u64 L = j_end - i0 + 1;
    const u32 t = threadIdx.x;
    u32* v = scratch + (u64)blockIdx.x * 3 * (SD + TAU);
    u32* pre = v + (SD + TAU);
    u32* suf = pre + (SD + TAU);
    {
        const u64 C = (L + FB_T - 1) / FB_T;
        const u64 a = min<u64>(L, t * C), e = min<u64>(L, a + C);
        if (a < e) {
            u32 fp = 0;
            for (u64 k = 0; k < TAU; k++) fp = fp * b + T[i0 + a + k];
            for (u64 r = a; r < e; r++) {
                const u64 j = i0 + r;
                const u64 q = (j + 127) >> 7;
                const u16 qi = qinfo[q];
                const u32 rel = (u32)(j + 127 - (q << 7));
                v[r] = (rel >= (u32)(qi >> 8) && rel <= (u32)(qi & 255)) ? INF32 : fp;
                if (r + 1 < e) fp = fp * b + T[j + TAU] - bpow * T[j];
            }
        }
    }
    __syncthreads();
    {
        const u64 nblk = (L + TAU - 1) / TAU;
        for (u64 k = t; k < 2 * nblk; k += FB_T) {
            const u64 blk = k >> 1, a = blk * TAU, e = min<u64>(L, a + TAU);
            if (k & 1) {
                u32 m = INF32;
                for (u64 r = e; r > a; r--) suf[r - 1] = m = min(m, v[r - 1]);
            } else {
                u32 m = INF32;
                for (u64 r = a; r < e; r++) pre[r] = m = min(m, v[r]);
            }
        }
    }
    __syncthreads();
    u32 mask[FB_DEC / 32];
    u32 c = 0;
    const u64 d0 = (u64)t * FB_DEC;
#pragma unroll
    for (int w = 0; w < FB_DEC / 32; w++) {
        u32 bits = 0;
        for (int k = 0; k < 32; k++) {
            const u64 r = d0 + 32 * w + k;
            if (i0 + r >= i_end) break;
            const u32 m = min(min(suf[r], pre[r + TAU - 1]), v[r + TAU]);
            if (m != INF32 && (v[r] == m || v[r + TAU] == m)) bits |= 1u << k;
        }
        mask[w] = bits;
        c += __popc(bits);
    }
    s_cnt[t] = c;
    __syncthreads();
    if (t == 0) {
        u32 tot = 0;
        for (int k = 0; k < FB_T; k++) {
            const u32 x = s_cnt[k];
            s_cnt[k] = tot;
            tot += x;
        }
        lane_cnt[lane] = tot;
    }
    __syncthreads();
    u32 o = s_cnt[t];
    pos_t* out = ovf_out + (u64)blockIdx.x * SD;
#pragma unroll
    for (int w = 0; w < FB_DEC / 32; w++)
        for (u32 bits = mask[w]; bits; bits &= bits - 1) out[o++] = (pos_t)(i0 + d0 + 32 * w + __builtin_ctz(bits));
}

// one wave per stripe, its outputs copied by the 64 lanes (coalesced; one thread per stripe
// copying its ~128 outputs alone took 48 us on a 1 GiB genome-like text)
__global__ void k_sss_compact(const pos_t* __restrict__ lane_out, const u32* __restrict__ lane_cnt,
                              const u32* __restrict__ lane_off, const u32* __restrict__ lane_flag,
                              const u32* __restrict__ ovf_slot, const pos_t* __restrict__ ovf_out, u64 nlanes,
                              pos_t* __restrict__ S) {
    const u32 lane = threadIdx.x & 63;
    for (u64 w = gtid() >> 6; w < nlanes; w += gstride() >> 6) {
        const u32 c = lane_cnt[w], o = lane_off[w];
        const pos_t* src = lane_flag[w] ? ovf_out + (u64)ovf_slot[w] * SD : lane_out + w * SCAP;
        for (u32 x = lane; x < c; x += 64) S[(u64)o + x] = src[x];
    }
}

// Compaction with the offsets found in the kernel (no overflowing stripe): workgroup b copies the
// outputs of stripes [64 b, 64 b + 64), its base the sum of all earlier stripes' counts (read by
// the whole workgroup from L2, 32 loads per thread at most at 1 GiB); the block's outputs are one
// contiguous range of S, copied by all threads (an output finds its stripe by a binary search
// over the block's 64 offsets)
constexpr u32 CC_T = 1024, CC_SPB = 64;
__global__ __launch_bounds__(CC_T) void k_sss_compact_scan(const pos_t* __restrict__ lane_out,
                                                           const u32* __restrict__ lane_cnt, u64 nlanes,
                                                           pos_t* __restrict__ S) {
    __shared__ u32 s_part[CC_T / 64];
    __shared__ u32 s_off[CC_SPB + 1];
    const u32 t = threadIdx.x, lane = t & 63, wv = t >> 6;
    const u64 w0 = (u64)blockIdx.x * CC_SPB;
    u32 sum = 0;
#pragma unroll 8
    for (u64 k = t; k < w0; k += CC_T) sum += lane_cnt[k];
    for (int o = 32; o >= 1; o >>= 1) sum += __shfl_xor(sum, o, 64);
    if (lane == 0) s_part[wv] = sum;
    const u32 c = t < CC_SPB && w0 + t < nlanes ? lane_cnt[w0 + t] : 0u;
    __syncthreads();
    if (t < CC_SPB) {  // wave 0: the block's offsets (relative), s_off[64] = its total
        const u32 inc = wave_prefix_add(c);
        s_off[t] = inc - c;
        if (t == CC_SPB - 1) s_off[CC_SPB] = inc;
    }
    u32 base = 0;
    for (u32 k = 0; k < CC_T / 64; k++) base += s_part[k];
    __syncthreads();
    const u32 tot = s_off[CC_SPB];
    for (u32 j = t; j < tot; j += CC_T) {
        u32 lo = 0, hi = CC_SPB - 1;  // the last stripe k with s_off[k] <= j
        while (lo < hi) {
            const u32 mid = (lo + hi + 1) >> 1;
            if (s_off[mid] <= j) lo = mid;
            else hi = mid - 1;
        }
        S[(u64)base + j] = lane_out[(w0 + lo) * SCAP + (j - s_off[lo])];
    }
}

// exclusive scan of the stripe counts in one workgroup (off[m] = the total): one launch where the
// pad fill and rocprim's scan took three (about 15 us of the phase on a 1 GiB text).  Wave w holds
// the chunks w, w + 16, ... of 64 counts in registers (all loads issued at once: a loop of
// dependent load-scan steps took 25-60 us), their totals are scanned across the workgroup
constexpr u32 CS_T = 1024, CS_CPW = 64, CS_MAX = CS_T * CS_CPW;
__global__ __launch_bounds__(CS_T) void k_count_scan(const u32* __restrict__ cnt, u64 m, u32* __restrict__ off) {
    __shared__ u32 s_c[CS_T];
    __shared__ u32 s_w[CS_T / 64];
    const u32 t = threadIdx.x, lane = t & 63, wv = t >> 6;
    const u32 nch = (u32)((m + 63) / 64);
    u32 x[CS_CPW];
#pragma unroll
    for (u32 k = 0; k < CS_CPW; k++) {
        const u64 i = ((u64)(wv + 16 * k)) * 64 + lane;
        x[k] = i < m ? cnt[i] : 0u;
    }
#pragma unroll
    for (u32 k = 0; k < CS_CPW; k++) {
        const u32 c = wv + 16 * k;
        if (c < nch) {  // (uniform)
            x[k] = wave_prefix_add(x[k]);  // inclusive, per chunk
            if (lane == 63) s_c[c] = x[k];
        }
    }
    __syncthreads();
    const u32 v = t < nch ? s_c[t] : 0u;
    const u32 incl = wave_prefix_add(v);
    if (lane == 63) s_w[wv] = incl;
    __syncthreads();
    if (t < 64) {
        const u32 y = t < CS_T / 64 ? s_w[t] : 0u;
        const u32 iy = wave_prefix_add(y);
        if (t < CS_T / 64) s_w[t] = iy - y;
    }
    __syncthreads();
    if (t < nch) s_c[t] = s_w[wv] + incl - v;  // chunk bases
    __syncthreads();
#pragma unroll
    for (u32 k = 0; k < CS_CPW; k++) {
        const u32 c = wv + 16 * k;
        if (c < nch) {
            const u64 i = (u64)c * 64 + lane;
            const u32 ex = (u32)__shfl_up((int)x[k], 1, 64);  // the inclusive sum of the lane before
            if (i < m) off[i] = s_c[c] + (lane ? ex : 0u);
            if (c + 1 == nch && lane == 63) off[m] = s_c[c] + x[k];
        }
    }
}

static u32 pow32_host(u32 b, u64 e) {
    u32 r = 1;
    while (e) {
        if (e & 1) r *= b;
        b *= b;
        e >>= 1;
    }
    return r;
}

// run chains of the anchors (all, or the anchors of a sorted tile list): exact run
// ends/starts along chains by two last-marked scans
void engine::run_chains(u64 nanch, const u32* tiles, u64 m) {
    if (!m) {
        runs_valid = true;
        return;
    }
    // the chain keys are u32 element indices + 1 (k_run_keys); the scans take size_t counts
    if (m >= 0xFFFFFFFFull) throw error(LZ77SSS_EINVAL, "too many anchors for the run-chain scans (u32 chain keys)");
    u32* ka = (u32*)run_scan_a.get(m);  // 2 x m u32
    u32* kb = (u32*)run_scan_b.get(m);
    k_run_keys<<<cdiv(m, 256), 256, 0, st>>>(run_p.p, run_hi.p, run_lo.p, nanch, tiles, m, ka, ka + m);
    scan_dev(ka, kb, m, m, 0xFFFFFFFFu, 0xFFFFFFFFu, op_min{}, false, scan_tmp, st);
    scan_dev(ka + m, kb + m, m, m, 0u, 0u, op_max{}, false, scan_tmp, st);
    k_run_apply<<<cdiv(m, 256), 256, 0, st>>>(kb, kb + m, run_p.p, tmp_bytes.p, nanch, tiles, m, run_hi.p, run_lo.p);
    LZ_HIP(hipGetLastError());
    runs_valid = true;
}

// Q anchors and the periodic-run table of every anchor (an externally built sync set
// needs them for the LCE); returns whether some window is in Q
bool engine::build_q_runs(const u8* T) {
    runs_valid = false;
    brk_valid = false;
    if (n < 2 * (u64)TAU) return false;
    const u64 nanch = (n - TAU) / QA + 2;
    u16* qi = q_info.get(nanch + 64);
    u32* ctr = counters.get(16);
    LZ_HIP(hipMemsetAsync(ctr, 0, 16 * sizeof(u32), st));
    u8* rp = run_p.get(nanch);
    pos_t* rhi = run_hi.get(nanch);
    pos_t* rlo = run_lo.get(nanch);
    u8* rcap = tmp_bytes.get(nanch);
    k_q_anchors<<<cdiv(nanch, QT_OWN), QT_THREADS, 0, st>>>(T, n, nanch, qi, ctr + 0, rp, rhi, rlo, rcap, nullptr,
                                                           nullptr, nullptr, nullptr, 0);
    LZ_HIP(hipGetLastError());
    run_chains(nanch, nullptr, nanch);
    return rd1(ctr, st) != 0;
}

// The sync set:
//   1. k_sss_stream<PASS1> over every stripe with Q assumed empty + the periodicity filter
//   2. k_sss_marks / k_flag_list: the tiles of anchors the filter hit (sorted), the stripes
//      forced into the re-run; one host read of the tile count
//   3. k_q_anchors on those tiles only (exact Q intervals + run table there; it appends the
//      stripes whose decisions see a Q window), run chains over them
//   4. k_sss_stream<QSKIP> re-runs the listed stripes exactly
//   5. per-stripe counts -> offsets (one host read: |S|, overflow, any Q), fallback for
//      overflowing stripes (rare), compaction
void engine::build_sss(const u8* T) {
    s = 0;
    has_runs = false;
    sss_kernel_ms = 0;
    sss_ev_pending = false;
    sss_kernel_bytes = 0;
    runs_valid = false;
    stats_fallback_lanes = 0;
    stats_sss_tiles = 0;
    brk_valid = false;
    if (n < 2 * (u64)TAU) return;
    const u64 last_i = n - 2 * TAU;
    const u64 nanch = (n - TAU) / QA + 2;
    const u64 nlanes = last_i / SD + 1;  // stripes
    const u64 ntiles = cdiv(nanch, QT_OWN);
    u16* qi = q_info.get(nanch + 64);  // k_sss_stream reads 8 anchors per block, up to 2 blocks past n
    u8* rp = run_p.get(nanch);
    pos_t* rhi = run_hi.get(nanch);
    pos_t* rlo = run_lo.get(nanch);
    u8* rcap = tmp_bytes.get(nanch);
    u32* ctr = counters.get(16);
    // ctr: any Q, overflowing stripes, tiles, re-run stripes, any block record, marks needed;
    // 8..11: k_sss_runs counters.  tot: |S| as 64 partial sums (stripe w adds to w & 63)
    u32* tot = sss_tot.get(64);
    fills({{ctr, 12 * sizeof(u32), 0u}, {tot, 64 * sizeof(u32), 0u}});
    pos_t* lo = lane_out.get(nlanes * SCAP);
    u32* lc = lane_cnt.get(nlanes + 1);
    u32* lf = lane_flag.get(nlanes);
    u64* hw = sss_hitw.get(3 * nlanes);
    const u64 tpad = (ntiles + 16 * 1024 - 1) / (16 * 1024) * (16 * 1024);  // k_flag_list reads 16-byte words
    u8* tfl = sss_tflag.get(tpad);
    u32* tl = sss_tiles.get(ntiles);
    u32* sfl = sss_sflag.get(nlanes);
    u32* sl = sss_slist.get(nlanes);
    sss_pow32 PW;
    for (int e = 0; e < 8; e++) PW.pwb[e] = pow32_host(SSS_BASE, e);
    PW.b8 = pow32_host(SSS_BASE, 8);
    PW.ib8 = pow32_host(PW.b8, (1ull << 31) - 1);  // b8^(2^31 - 1) = b8^-1 (odd units mod 2^32 have order | 2^30)
    PW.B = pow32_host(SSS_BASE, TAU);
    const u32 bpow = PW.B;
    // test knob: a lower overflow threshold sends more stripes down the exact fallback
    const char* scap_env = std::getenv("LZ77SSS_TEST_SCAP");
    const u32 scap = scap_env ? (u32)std::min<long>(SCAP, std::max<long>(0, std::atol(scap_env))) : (u32)SCAP;
    if (!sss_ev0)
        for (hipEvent_t* e : {&sss_ev0, &sss_ev1, &sss_evA, &sss_evB}) LZ_HIP(hipEventCreate(e));
    sss_ev_pending = false;
    LZ_HIP(hipEventRecord(sss_ev0, st));
    // per-block run records (0: unknown), cleared by pass 1
    const u64 nbk = (n + TAU - 1) / TAU;
    u8* bp = blk_p.get(nbk + 1);
    u16* bfo = blk_fo.get(nbk + 1);
    u16* blo = blk_lo.get(nbk + 1);
    const bool runs_kernel = !std::getenv("LZ77SSS_NO_RUNS_KERNEL");  // test knob: every stopped stripe through the Q-anchor path
    // test knob: pure runs through k_sss_runs as well (pass 1 does not settle them)
    const bool pure_runs = runs_kernel && !std::getenv("LZ77SSS_NO_PURE_RUNS");
    k_sss_stream<false, true><<<cdiv(nlanes, SWAVES), 64 * SWAVES, 0, st>>>(
        T, n, last_i, qi, nlanes, lo, lc, lf, ctr + 1, (u32)SSS_BASE, PW, scap, hw, qi, rp, nullptr, nullptr, bp, bfo,
        blo, nbk, ctr + 5, tot);
    LZ_HIP(hipGetLastError());
    // the stripes pass 1 stopped: settled in one pass where their periodic windows are runs
    // (k_sss_runs), which also writes the per-block run records of the LCE
    // LZ77SSS_RUNS_PROF: per-stripe clocks and counters of k_sss_runs, summarized on stderr
    u32* runs_prof = nullptr;
    if (std::getenv("LZ77SSS_RUNS_PROF")) {
        runs_prof = (u32*)u64a.get(2 * nlanes + 2);
        LZ_HIP(hipMemsetAsync(runs_prof, 0, 16 * nlanes, st));
    }
    if (runs_kernel)
        k_sss_runs<<<cdiv(nlanes, RWAVES), 64 * RWAVES, 0, st>>>(T, n, last_i, nlanes, lo, lc, lf, ctr + 1,
                                                                (u32)SSS_BASE, PW, scap, hw, bp, bfo, blo, nbk, ctr + 0,
                                                                debug_enabled() ? ctr + 8 : nullptr, tot, runs_prof,
                                                                pure_runs ? 1 : 0);
    LZ_HIP(hipGetLastError());
    // one read: any Q window, overflowing stripes, does any block have a run record, does any tile
    // need the Q-anchor pass (a hit in a stripe pass 1 ran through, or a stripe k_sss_runs could not
    // settle); |S| as 64 partial sums (final unless the Q-anchor pass re-runs stripes)
    u32 hc[6], htot[64];
    LZ_HIP(hipEventRecord(sss_evA, st));
    {
        hread rb(st);
        rb.add(hc, (const u32*)ctr, 6);
        rb.add(htot, (const u32*)tot, 64);
        rb.sync();
    }
    const u32 need_marks = hc[5], any_rec = hc[4];
    if (runs_prof) {
        std::vector<u32> hp4(4 * nlanes);
        LZ_HIP(hipMemcpy(hp4.data(), runs_prof, 16 * nlanes, hipMemcpyDeviceToHost));
        std::vector<std::pair<u32, u64>> dur;
        u64 t0 = ~0ull, sum_phi = 0, sum_cross = 0, sum_cls = 0;
        for (u64 w = 0; w < nlanes; w++)
            if (hp4[4 * w + 1]) {
                dur.push_back({hp4[4 * w + 1], w});
                t0 = std::min<u64>(t0, hp4[4 * w]);
                sum_phi += hp4[4 * w + 3] & 0xFFFF;
                sum_cross += hp4[4 * w + 3] >> 16;
                sum_cls += hp4[4 * w + 2] & 0xFFFF;
            }
        std::sort(dur.begin(), dur.end());
        const size_t m = dur.size();
        std::fprintf(stderr, "[lz77sss-runs-prof] stripes run %zu of %llu: blocks hashed %llu crossed %llu classifications %llu\n", m,
                     (unsigned long long)nlanes, (unsigned long long)sum_phi, (unsigned long long)sum_cross, (unsigned long long)sum_cls);
        if (m) {
            std::fprintf(stderr, "[lz77sss-runs-prof] clocks p50 %u p90 %u p99 %u max %u\n", dur[m / 2].first, dur[m * 9 / 10].first,
                         dur[m * 99 / 100].first, dur[m - 1].first);
            for (size_t i = m; i > 0 && i + 12 > m; i--) {
                const u64 w = dur[i - 1].second;
                std::fprintf(stderr, "[lz77sss-runs-prof]   stripe %llu: clocks %u start %llu cls %u find %u fail %u hashed %u crossed %u\n",
                             (unsigned long long)w, hp4[4 * w + 1], (unsigned long long)(hp4[4 * w] - (u32)t0), hp4[4 * w + 2] & 0xFFFF,
                             (hp4[4 * w + 2] >> 16) & 0x7FFF, hp4[4 * w + 2] >> 31, hp4[4 * w + 3] & 0xFFFF, hp4[4 * w + 3] >> 16);
            }
        }
    }
    LZ_HIP(hipEventRecord(sss_evB, st));
    u32 ndirty = 0;
    // the per-anchor Q intervals and run periods start out empty when something reads them (the
    // Q-anchor pass and its re-run, the fallback); pass 1 no longer clears them (25 MB of stores
    // per GiB that only run-free or settled texts skipped reading)
    bool anchors_cleared = false;
    auto clear_anchors = [&]() {
        if (anchors_cleared) return;
        fills({{qi, 2 * (nanch + 64), 0xFF00FF00u}, {rp, nanch, 0u}});
        anchors_cleared = true;
    };
    if (need_marks || !runs_kernel) {
        clear_anchors();
        // tiles the filter marked (the stopped stripes k_sss_runs settled have no hit bits left)
        const u64 nblk_last = std::min<u64>(SNB, (last_i - (nlanes - 1) * SD) / TAU + 1);
        const u64 t_tail = (nlanes - 1) * (SD / QA) + 4 * nblk_last, q_end = nanch + 64;
        const u64 nthr = std::max<u64>(std::max<u64>(nlanes, tpad), q_end - t_tail);
        k_sss_marks<<<cdiv(nthr, 256), 256, 0, st>>>(hw, nlanes, ntiles, tpad, nanch, tfl, sfl, sl, ctr + 3, t_tail,
                                                    q_end, qi, rp);
        const u64 nfw = (ntiles + 15) / 16;  // 16-byte flag words (the flag array is padded to tpad)
        const unsigned nfb = cdiv(nfw, FL_T);
        u32* fc = sss_fcnt.get(nfb);
        k_flag_count<<<nfb, FL_T, 0, st>>>(tfl, nfw, fc);
        k_flag_list<<<nfb, FL_T, 0, st>>>(tfl, nfw, fc, tl, ctr + 2);
        LZ_HIP(hipGetLastError());
        ndirty = rd1(ctr + 2, st);
    }
    stats_sss_tiles = ndirty;
    if (debug_enabled()) {
        u32 dc[4];
        LZ_HIP(hipMemcpy(dc, ctr + 8, 16, hipMemcpyDeviceToHost));
        std::fprintf(stderr, "[lz77sss-debug] sss: k_sss_runs slow classifications=%u period searches=%u unsettled stripes=%u (overflowing %u) tiles=%u\n",
                     dc[0], dc[1], dc[2], dc[3], ndirty);
    }
    if (ndirty) {
        k_q_anchors<<<ndirty, QT_THREADS, 0, st>>>(T, n, nanch, qi, ctr + 0, rp, rhi, rlo, rcap, tl, sfl, sl, ctr + 3,
                                                   nlanes);
        LZ_HIP(hipGetLastError());
        run_chains(nanch, tl, (u64)ndirty * QT_OWN);
        // a marked tile spans at most 3 stripes' decision ranges (its anchors' Q windows reach
        // 639 decisions back); the forced stripes each meet a marked tile
        const u64 maxw = std::min<u64>(nlanes, 4ull * ndirty + 4);
        k_sss_stream<true, false><<<cdiv(maxw, SWAVES), 64 * SWAVES, 0, st>>>(
            T, n, last_i, qi, nlanes, lo, lc, lf, ctr + 1, (u32)SSS_BASE, PW, scap, nullptr, nullptr, nullptr, sl,
            ctr + 3, nullptr, nullptr, nullptr, 0, nullptr, tot);
        LZ_HIP(hipGetLastError());
    }
    runs_valid = ndirty != 0;  // the anchor run table: period 0 outside the marked tiles (none: not read)
    brk_valid = false;
    if (any_rec) {
        // run-record segments -> packed per-block run end / start (two launches)
        const u64 ntile = (nbk + BT_TILE - 1) / BT_TILE;
        u64* tt = (u64*)blk_mk.get(4 * ntile + 4);  // 2 x ntile u64 (the buffer is pos_t-typed)
        const blk_recs BR{bp, bfo, blo};
        k_blk_seg_tiles<<<(unsigned)ntile, BT_T, 0, st>>>(BR, nbk, tt, tt + ntile);
        k_blk_seg_info<<<(unsigned)ntile, BT_T, 0, st>>>(BR, nbk, tt, tt + ntile, ntile, blk_re.get(nbk),
                                                         blk_rs.get(nbk));
        LZ_HIP(hipGetLastError());
        if (std::getenv("LZ77SSS_BLK_CHECK") && nbk < 0x7FFFFFFFull) {
            // test knob: the marker + min/max-scan formulation, compared entry by entry
            pos_t* mk = (pos_t*)u64a.get(2 * nbk + 2);
            pos_t* ser = (pos_t*)u64b.get(nbk + 1);
            pos_t* bss = (pos_t*)u32e.get(2 * nbk + 2);
            k_blk_marks<<<cdiv(nbk, 256), 256, 0, st>>>(BR, nbk, mk, mk + nbk);
            size_t tb = 0, tb2 = 0;
            LZ_HIP(hipcub::DeviceScan::InclusiveScan(nullptr, tb, mk, ser, hipcub::Min(), (int)nbk, st));
            LZ_HIP(hipcub::DeviceScan::InclusiveScan(nullptr, tb2, mk + nbk, bss, hipcub::Max(), (int)nbk, st));
            u8* t = scan_tmp.get(std::max(tb, tb2));
            LZ_HIP(hipcub::DeviceScan::InclusiveScan(t, tb, mk, ser, hipcub::Min(), (int)nbk, st));
            LZ_HIP(hipcub::DeviceScan::InclusiveScan(t, tb2, mk + nbk, bss, hipcub::Max(), (int)nbk, st));
            u64* re2 = (u64*)u32d.get(4 * nbk + 4);
            u64* rs2 = re2 + nbk;
            k_blk_runinfo<<<cdiv(nbk, 256), 256, 0, st>>>(BR, ser, bss, nbk, re2, rs2);
            std::vector<u64> a(2 * nbk), c(2 * nbk);
            LZ_HIP(hipMemcpyAsync(a.data(), blk_re.p, 8 * nbk, hipMemcpyDeviceToHost, st));
            LZ_HIP(hipMemcpyAsync(a.data() + nbk, blk_rs.p, 8 * nbk, hipMemcpyDeviceToHost, st));
            LZ_HIP(hipMemcpyAsync(c.data(), re2, 16 * nbk, hipMemcpyDeviceToHost, st));
            LZ_HIP(hipStreamSynchronize(st));
            for (u64 i = 0; i < 2 * nbk; i++)
                if (a[i] != c[i]) throw error(LZ77SSS_EINTERNAL, "run-record check: tile kernels differ from the scan form");
        }
        brk_nbk = nbk;
        brk_valid = true;
        if (const char* dp = std::getenv("LZ77SSS_DUMP_RUNS")) {
            // debug knob: the raw records (period, first break, last break) and the packed
            // end / start words, as five consecutive arrays of nbk entries
            std::vector<u8> hp(nbk);
            std::vector<u16> hf(nbk), hl(nbk);
            std::vector<u64> he(nbk), hs(nbk);
            LZ_HIP(hipStreamSynchronize(st));
            LZ_HIP(hipMemcpy(hp.data(), bp, nbk, hipMemcpyDeviceToHost));
            LZ_HIP(hipMemcpy(hf.data(), bfo, 2 * nbk, hipMemcpyDeviceToHost));
            LZ_HIP(hipMemcpy(hl.data(), blo, 2 * nbk, hipMemcpyDeviceToHost));
            LZ_HIP(hipMemcpy(he.data(), blk_re.p, 8 * nbk, hipMemcpyDeviceToHost));
            LZ_HIP(hipMemcpy(hs.data(), blk_rs.p, 8 * nbk, hipMemcpyDeviceToHost));
            if (FILE* f = std::fopen(dp, "wb")) {
                std::fwrite(hp.data(), 1, nbk, f);
                std::fwrite(hf.data(), 2, nbk, f);
                std::fwrite(hl.data(), 2, nbk, f);
                std::fwrite(he.data(), 8, nbk, f);
                std::fwrite(hs.data(), 8, nbk, f);
                std::fclose(f);
            }
        }
        if (debug_enabled()) {
            std::vector<u8> hb(nbk);
            LZ_HIP(hipMemcpy(hb.data(), bp, nbk, hipMemcpyDeviceToHost));
            u64 cnt[4] = {0, 0, 0, 0}, seg = 0;
            for (u64 i = 0; i < nbk; i++) {
                cnt[hb[i] == 0 ? 0 : hb[i] == 1 ? 1 : hb[i] <= 16 ? 2 : 3]++;
                if (hb[i] && (i == 0 || hb[i - 1] != hb[i])) seg++;
            }
            std::fprintf(stderr, "[lz77sss-debug] sss: run records: blocks=%llu none=%llu p1=%llu p2-16=%llu p17+=%llu segments=%llu\n",
                         (unsigned long long)nbk, (unsigned long long)cnt[0], (unsigned long long)cnt[1],
                         (unsigned long long)cnt[2], (unsigned long long)cnt[3], (unsigned long long)seg);
            if (nbk <= 64) {
                std::vector<u16> hf(nbk), hl(nbk);
                std::vector<u64> hre(nbk), hrs(nbk);
                LZ_HIP(hipMemcpy(hf.data(), bfo, 2 * nbk, hipMemcpyDeviceToHost));
                LZ_HIP(hipMemcpy(hl.data(), blo, 2 * nbk, hipMemcpyDeviceToHost));
                LZ_HIP(hipMemcpy(hre.data(), blk_re.p, 8 * nbk, hipMemcpyDeviceToHost));
                LZ_HIP(hipMemcpy(hrs.data(), blk_rs.p, 8 * nbk, hipMemcpyDeviceToHost));
                for (u64 i = 0; i < nbk; i++)
                    std::fprintf(stderr, "[lz77sss-debug]   block %llu: p=%u fo=%u lo=%u run end=%llu start=%llu\n",
                                 (unsigned long long)i, hb[i], hf[i], hl[i], (unsigned long long)(hre[i] >> 16),
                                 (unsigned long long)(hrs[i] >> 16));
            }
        }
    }

    u32 hp[3];
    u32 total = 0;
    for (u32 v : htot) total += v;
    u32* off = u32a.get(nlanes + 1);
    auto scan_counts = [&]() {
        if (nlanes <= CS_MAX) k_count_scan<<<1, CS_T, 0, st>>>(lc, nlanes, off);
        else excl_sum_total(lc, off, nlanes, scan_tmp, st);
    };
    if (!ndirty && !hc[1]) {
        // the usual case: the counts are final and nothing overflowed, so |S| is known and the
        // compaction finds the stripes' offsets itself (no scan launch, no second read)
        has_runs = hc[0] != 0;
        if (total >= 0x7FFFFFFFu) throw error(LZ77SSS_EINVAL, "sync set of 2^31 or more positions (split the text)");
        s = total;
        sss_kernel_bytes = n + sizeof(pos_t) * (u64)s;
        pos_t* dS = S.get((u64)s + 1);
        k_sss_compact_scan<<<cdiv(nlanes, CC_SPB), CC_T, 0, st>>>(lo, lc, nlanes, dS);
        LZ_HIP(hipGetLastError());
        LZ_HIP(hipEventRecord(sss_ev1, st));  // sss_kernel_ms: the two windows (engine.h sss_ms)
        sss_ev_pending = true;
        return;
    }
    // exclusive scan of stripe counts -> offsets; total = |S|
    scan_counts();
    {
        hread rb(st);
        rb.add(hp, (const u32*)ctr, 2);
        rb.add(hp + 2, (const u32*)(off + nlanes));
        rb.sync();
    }
    has_runs = hp[0] != 0;
    total = hp[2];

    // overflowing stripes -> exact workgroup-parallel path
    u32* ovf_slot = u32c.get(nlanes);
    pos_t* ovf_out = lo;  // unused unless some stripe overflowed
    if (hp[1]) {
        std::vector<u32> hf(nlanes);
        LZ_HIP(hipMemcpy(hf.data(), lf, nlanes * sizeof(u32), hipMemcpyDeviceToHost));
        std::vector<u32> lanes, slot(nlanes, 0);
        for (u64 l = 0; l < nlanes; l++)
            if (hf[l]) { slot[l] = (u32)lanes.size(); lanes.push_back((u32)l); }
        u32* d_lanes = u32d.get(lanes.size());
        LZ_HIP(hipMemcpy(d_lanes, lanes.data(), lanes.size() * 4, hipMemcpyHostToDevice));
        LZ_HIP(hipMemcpy(ovf_slot, slot.data(), nlanes * 4, hipMemcpyHostToDevice));
        u32* scratch = (u32*)u64a.get((lanes.size() * 3 * (SD + TAU) + 1) / 2);
        ovf_out = sss_ovf.get(lanes.size() * SD);
        clear_anchors();  // (Q intervals: empty outside the marked tiles)
        k_sss_fallback<<<(unsigned)lanes.size(), FB_T, 0, st>>>(T, n, last_i, qi, d_lanes, scratch, ovf_out, lc,
                                                                (u32)SSS_BASE, bpow);
        LZ_HIP(hipGetLastError());
        stats_fallback_lanes = lanes.size();
        scan_counts();
        total = rd1(off + nlanes, st);
    }
    // |S| feeds hipcub/rocprim item counts (int) in SA_S and LPF: a sync set this large would
    // need > 2^31 entries (about 2^39 text bytes of random-like text, past one GPU's HBM)
    if (total >= 0x7FFFFFFFu) throw error(LZ77SSS_EINVAL, "sync set of 2^31 or more positions (split the text)");
    s = total;
    sss_kernel_bytes = n + sizeof(pos_t) * (u64)s;
    pos_t* dS = S.get((u64)s + 1);
    k_sss_compact<<<capped_grid(nlanes * 64, 256), 256, 0, st>>>(lo, lc, off, lf, ovf_slot, ovf_out, nlanes, dS);
    LZ_HIP(hipGetLastError());
    LZ_HIP(hipEventRecord(sss_ev1, st));  // (this path's second window also holds its reads)
    sss_ev_pending = true;
}

// ---------------------------------------------------------------------------
// pos_t = uint64_t sync set of a decision range (lce_sss.hpp:53 instantiated with
// pos_t = uint64_t, lz77_sss.hpp:72-75).  Phi and Q are functions of window contents
// only, so S n [b, e) is the sync set of the view T[b, e + 2tau - 1), whose last
// decision is e - 1: the range is walked in windows of `window` decisions through
// build_sss on such views (a 2tau-1 byte halo each), and the positions are widened to
// 64 bits with the view offset plus `base` added.  The same halo is what a rank of a
// sharded job holds: it loads T[b_r, e_r + 2tau - 1) and passes
// base = b_r.
__global__ void k_lower_bound_u32(const pos_t* __restrict__ S, u32 s, u32 x, u32* __restrict__ out) {
    u32 lo = 0, hi = s;
    while (lo < hi) {
        const u32 mid = (lo + hi) >> 1;
        if (S[mid] < x) lo = mid + 1; else hi = mid;
    }
    *out = lo;
}
__global__ void k_sss_widen(const pos_t* __restrict__ S, u32 s, const u32* __restrict__ skip, u64 add,
                            u64* __restrict__ out) {
    const u32 k0 = *skip;
    const u64 k = (u64)blockIdx.x * blockDim.x + threadIdx.x + k0;
    if (k >= s) return;
    out[k - k0] = (u64)S[k] + add;
}

void engine::build_sss_range(u64 first, u64 end, u64 base, u64 window) {
    s64 = 0;
    has_runs64 = false;
    stats_sss_windows = 0;
    if (n < 2 * (u64)TAU) return;
    end = std::min<u64>(end, n - 2 * TAU + 1);
    if (first >= end) return;
    if (window == 0) window = 1ull << 30;
    window = std::max<u64>(4096, (window + 4095) & ~4095ull);  // view starts stay 256-byte aligned
    if (window > (1ull << 31)) throw error(LZ77SSS_EINVAL, "window must be at most 2^31 decisions");
    const u64 n_full = n;
    u32* ctr = counters.get(16) + 12;  // build_sss clears and uses the first two
    u64 b = first & ~255ull;  // aligned view start; decisions in [b, first) are dropped
    double kms = 0;
    u64 kbytes = 0;
    try {
        while (b < end) {
            const u64 e = std::min(end, b + window);
            n = e - b + 2 * TAU - 1;  // the view: its last decision is e - 1
            build_sss(d_text + b);
            kms += sss_ms();
            kbytes += sss_kernel_bytes;
            has_runs64 |= has_runs;
            stats_sss_windows++;
            const u32 x = first > b ? (u32)(first - b) : 0u;
            k_lower_bound_u32<<<1, 1, 0, st>>>(S.p, s, x, ctr);
            const u32 skip = x ? rd1(ctr, st) : 0u;
            const u64 cnt = (u64)s - skip;
            u64* out = S64.grow_keep(s64 + cnt + 1, s64, st);
            if (cnt) k_sss_widen<<<cdiv(cnt, 256), 256, 0, st>>>(S.p, s, ctr, b + base, out + s64);
            LZ_HIP(hipGetLastError());
            s64 += cnt;
            b = e;
        }
    } catch (...) {
        n = n_full;
        throw;
    }
    n = n_full;
    sss_kernel_ms = kms / (double)stats_sss_windows;  // per launch, averaged over the windows
    sss_kernel_bytes = kbytes / stats_sss_windows;
    // the u32 structures now describe the last view, not the text
    s = 0;
    runs_valid = false;
    brk_valid = false;
    LZ_HIP(hipStreamSynchronize(st));
}

}  // namespace LZ_NS
