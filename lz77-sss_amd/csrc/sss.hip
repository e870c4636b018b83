// sss.hip -- kernel 1: the tau-synchronizing set (role of
// lce::rolling_hash::sss<pos_t,tau>, called at
// patched-files/external/lce/include/ds/lce_sss.hpp:53; its source is absent
// upstream, the definition pinned here is DESIGN.md section 4.1):
//
//   Phi(j)  = KR fingerprint of T[j..j+tau) mod 2^61-1 (base SSS_BASE)
//   Q       = { j : T[j..j+tau) has a period <= floor(tau/3) }
//   S       = { i <= n-2tau : min Phi'[i..i+tau] < inf at i or at i+tau }
//
// Three launches:
//   k_q_anchors  -- per anchor a (every 128 positions) the smallest period <= 170
//                   of T[a..a+340) and the Q interval it induces on (a-128, a]
//   k_sss_main   -- lanes stream contiguous 4 KiB segments; text is staged
//                   through LDS in coalesced 128-B rows; per lane a rolling
//                   61-bit Karp-Rabin hash feeds a monotone deque (LDS) that
//                   decides "forward-window minimum" (A) and "backward-window
//                   minimum" (B); i in S <=> A(i) or B(i+tau)
//   k_sss_compact-- per-lane outputs -> sorted S
#include "../include/engine.h"

#include <hipcub/hipcub.hpp>

namespace lz {

// ---------------------------------------------------------------------------
// Q anchors
constexpr int QT_ANCH = 128;                 // anchors per workgroup
constexpr int QT_SPAN = QT_ANCH * QA;        // 16384 positions
constexpr int QT_LDS = QT_SPAN + 256 + 1024; // [A0-256, A0+16384+1024)
constexpr u32 RUN_HCAP = 640;                // local run extension: [a-256, a+640)
constexpr u32 RUN_LCAP = 256;

__global__ __launch_bounds__(128) void k_q_anchors(const u8* __restrict__ T, u64 n, u64 nanch,
                                                   u16* __restrict__ qinfo, u32* __restrict__ any_q,
                                                   u8* __restrict__ run_p, u32* __restrict__ run_hi,
                                                   u32* __restrict__ run_lo, u8* __restrict__ run_cap) {
    __shared__ __attribute__((aligned(16))) u8 buf[QT_LDS];
    const u64 A0 = (u64)blockIdx.x * QT_SPAN;
    const int64_t base = (int64_t)A0 - 256;
    for (int x = threadIdx.x * 16; x < QT_LDS; x += 128 * 16) {
        int64_t g = base + x;
        uint4 v = {0, 0, 0, 0};
        if (g >= 0 && (u64)g + 16 <= n + TEXT_PAD) v = *(const uint4*)(T + g);
        *(uint4*)&buf[x] = v;
    }
    __syncthreads();
    const u64 t = (u64)blockIdx.x * QT_ANCH + threadIdx.x;
    if (t >= nanch) return;
    const u64 a = t * QA;
    u16 res = 0xFF00;  // empty interval
    u32 rp = 0, rhi = 0, rlo = 0;
    u8 rcap = 0;
    if (a + QM <= n) {
        const int la = (int)(a - base);  // multiple of 4
        const u32* b32 = (const u32*)buf;
        const u32 w0 = b32[la >> 2];
        u32 p = 0;
        u32 dprev = w0;
        for (int k = 0; k <= (int)(QL / 4) && !p; k++) {
            u32 dnext = b32[(la >> 2) + k + 1];
#pragma unroll
            for (int r = 0; r < 4; r++) {
                u32 pp = 4 * k + r;
                if (!p && pp >= 1 && pp <= QL) {
                    u32 w = __builtin_amdgcn_alignbyte(dnext, dprev, r);
                    if (w == w0) {
                        bool ok = true;
                        for (u32 x = 4; x < QM - pp; x++)
                            if (buf[la + x] != buf[la + pp + x]) { ok = false; break; }
                        if (ok) p = pp;
                    }
                }
            }
            dprev = dnext;
        }
        if (p) {
            u64 hi = a + QM - p;
            const u64 hi_cap = min(a + TAU - p, n - p);
            while (hi < hi_cap && buf[hi - base] == buf[hi + p - base]) hi++;
            const u64 lo_cap = a >= 127 ? a - 127 : 0;
            u64 lo = a;
            while (lo > lo_cap && buf[lo - 1 - base] == buf[lo - 1 + p - base]) lo--;
            // Q on (a-128, a]: j >= lo, j + tau - p <= hi, j <= n - tau
            int64_t jlo = (int64_t)lo;
            int64_t jhi = min((int64_t)a, (int64_t)hi + (int64_t)p - (int64_t)TAU);
            jhi = min(jhi, (int64_t)n - (int64_t)TAU);
            if (jlo <= jhi) {
                int64_t r0 = (int64_t)a - 127;  // rel(j) = j - r0 in [0,127]
                res = (u16)(((jlo - r0) << 8) | (jhi - r0));
                atomicOr(any_q, 1u);
            }
            // local extent of the p-periodic run around the window (for run-skipping LCE)
            u64 h2 = hi;
            const u64 h2_cap = min(a + RUN_HCAP - p, n - p);
            while (h2 < h2_cap && buf[h2 - base] == buf[h2 + p - base]) h2++;
            u64 l2 = lo;
            const u64 l2_cap = a >= RUN_LCAP ? a - RUN_LCAP : 0;
            while (l2 > l2_cap && buf[l2 - 1 - base] == buf[l2 - 1 + p - base]) l2--;
            rp = p;
            rhi = (u32)(h2 + p);
            rlo = (u32)l2;
            rcap = (h2 == a + RUN_HCAP - p ? 1 : 0) | (l2 == a - RUN_LCAP && a >= RUN_LCAP ? 2 : 0);
        }
    }
    qinfo[t] = res;
    run_p[t] = (u8)rp;
    run_hi[t] = rhi;
    run_lo[t] = rlo;
    run_cap[t] = rcap;
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
// main pass
constexpr int SL = 4096;     // sync candidates per lane
constexpr int NLW = 256;     // lanes per workgroup
constexpr int CH = 128;      // staging chunk (bytes per lane row)
constexpr int RSB = CH + 16; // LDS row stride (conflict-free ds_read_b128)
constexpr int DQ = 32;       // deque capacity per lane
constexpr int LCAP = 128;    // per-lane output capacity
constexpr int NCH = (SL + 2 * TAU) / CH;

struct lane_state {
    u64 fp;
    u64 front_val, back_val;
    u32 front_pos, cnt, h;
    u64 last_emit;
    u32 nout, flag;
};

__global__ __launch_bounds__(256, 1) void k_sss_main(const u8* __restrict__ T, u64 n, u64 last_i,
                                                     const u16* __restrict__ qinfo, u32* __restrict__ lane_out,
                                                     u32* __restrict__ lane_cnt, u32* __restrict__ lane_flag,
                                                     u32* __restrict__ any_flag, u32 b, u64 bn) {
    __shared__ __attribute__((aligned(16))) u8 s_in[NLW * RSB];
    __shared__ __attribute__((aligned(16))) u8 s_out[NLW * RSB];
    __shared__ u64 s_dqv[DQ * NLW];
    __shared__ u16 s_dqp[DQ * NLW];
    const int tid = threadIdx.x;
    const u64 lane = (u64)blockIdx.x * NLW + tid;
    const u64 wg_i0 = (u64)blockIdx.x * NLW * SL;
    const u64 i0 = lane * SL;
    const bool active = i0 <= last_i;
    const u64 i_end = active ? min(i0 + SL, last_i + 1) : i0;
    const u64 j_end = active ? min(i0 + SL + TAU - 1, n - TAU) : 0;
    const u64 kend = active ? j_end - i0 + TAU : 0;
    const u32 bn_lo = (u32)bn, bn_hi = (u32)(bn >> 32);

    u64 fp = 0, front_val = 0, back_val = 0, last_emit = INF64;
    u32 front_pos = 0, cnt = 0, h = 0, nout = 0, flag = 0;
    u64 cur_anchor = INF64;
    u32 qs = 255, qe = 0;
    u32* myout = lane_out + lane * LCAP;

    auto emit = [&](u64 i) {
        if (last_emit == INF64 || i > last_emit) {
            if (nout < LCAP) myout[nout] = (u32)i; else flag = 1;
            nout++;
            last_emit = i;
        }
    };

    for (int c = 0; c < NCH; c++) {
        __syncthreads();
#pragma unroll
        for (int r = 0; r < (NLW * CH / 16) / NLW; r++) {
            const int piece = r * NLW + tid;
            const int row = piece >> 3, col = (piece & 7) * 16;
            const u64 rowi0 = wg_i0 + (u64)row * SL;
            const u64 g = rowi0 + (u64)c * CH + col;
            uint4 vin = {0, 0, 0, 0}, vout = {0, 0, 0, 0};
            if (rowi0 <= last_i) {
                vin = *(const uint4*)(T + g);
                if (c * CH >= (int)TAU) vout = *(const uint4*)(T + g - TAU);
            }
            *(uint4*)&s_in[row * RSB + col] = vin;
            *(uint4*)&s_out[row * RSB + col] = vout;
        }
        __syncthreads();
        if (!active) continue;
        for (int qd = 0; qd < CH / 16; qd++) {
            const uint4 vi = *(const uint4*)&s_in[tid * RSB + qd * 16];
            const uint4 vo = *(const uint4*)&s_out[tid * RSB + qd * 16];
            const u32 wi4[4] = {vi.x, vi.y, vi.z, vi.w}, wo4[4] = {vo.x, vo.y, vo.z, vo.w};
#pragma unroll
            for (int w = 0; w < 4; w++) {
#pragma unroll
                for (int kk = 0; kk < 4; kk++) {
                    const u32 k = c * CH + qd * 16 + w * 4 + kk;
                    const u32 in = (wi4[w] >> (8 * kk)) & 255u, out = (wo4[w] >> (8 * kk)) & 255u;
                    // fp <- fp*b + in - out*b^tau  (lazy mod 2^61-1, fp < 2^62)
                    const u32 lo = (u32)fp, hi = (u32)(fp >> 32);
                    u64 a0 = (u64)lo * b + in;
                    a0 += (u64)bn_lo * out;
                    u64 a1 = (u64)hi * b + (a0 >> 32);
                    a1 += (u64)bn_hi * out;
                    fp = ((((a1 << 32) | (u32)a0)) & P61) + (a1 >> 29);
                    if (k + 1 < TAU || k >= kend) continue;
                    const u64 j = i0 + k - TAU + 1;
                    const u32 jo = (u32)(j - i0);
                    const u64 t = (j + 127) >> 7;
                    if (t != cur_anchor) {
                        cur_anchor = t;
                        const u16 qi = qinfo[t];
                        qs = qi >> 8;
                        qe = qi & 255;
                    }
                    const u32 rel = (u32)(j + 127 - (t << 7));
                    const u64 v = (rel >= qs && rel <= qe) ? INF64 : mod61_canon(fp);
                    // 1. expiry of the front: it survived (f, f+tau] -> A(f)
                    if (cnt && front_pos + TAU + 1 == jo) {
                        const u64 f = i0 + front_pos;
                        if (f < i_end) emit(f);
                        h = (h + 1) & (DQ - 1);
                        cnt--;
                        if (cnt) {
                            front_val = s_dqv[h * NLW + tid];
                            front_pos = s_dqp[h * NLW + tid];
                        }
                    }
                    // 2. B(j): v <= min of the previous tau values -> i = j - tau
                    if (v != INF64 && jo >= TAU && (cnt == 0 || v <= front_val)) {
                        const u64 i = j - TAU;
                        if (i < i_end) emit(i);
                    }
                    // 3. pop larger values from the back
                    while (cnt && back_val > v) {
                        cnt--;
                        if (cnt) back_val = s_dqv[((h + cnt - 1) & (DQ - 1)) * NLW + tid];
                    }
                    // 4. push
                    if (v != INF64) {
                        if (cnt == DQ) {
                            flag = 1;
                        } else {
                            const u32 e = (h + cnt) & (DQ - 1);
                            s_dqv[e * NLW + tid] = v;
                            s_dqp[e * NLW + tid] = (u16)jo;
                            cnt++;
                            back_val = v;
                            if (cnt == 1) { front_val = v; front_pos = jo; }
                        }
                    }
                }
            }
        }
    }
    if (active) {
        for (u32 x = 0; x < cnt; x++) {
            const u64 f = i0 + s_dqp[((h + x) & (DQ - 1)) * NLW + tid];
            if (f < i_end) emit(f);
        }
        lane_cnt[lane] = nout;
        lane_flag[lane] = flag;
        if (flag) atomicOr(any_flag, 1u);
    } else if (lane < (u64)gridDim.x * NLW) {
        lane_cnt[lane] = 0;
        lane_flag[lane] = 0;
    }
}

// Exact slow path for lanes whose deque or output buffer overflowed: one
// workgroup recomputes the lane's Phi' values and the window minima directly.
__global__ __launch_bounds__(256) void k_sss_fallback(const u8* __restrict__ T, u64 n, u64 last_i,
                                                      const u16* __restrict__ qinfo, const u32* __restrict__ lanes,
                                                      u64* __restrict__ scratch, u8* __restrict__ member,
                                                      u32* __restrict__ ovf_out, u32* __restrict__ lane_cnt, u32 b,
                                                      u64 bpow) {
    const u64 lane = lanes[blockIdx.x];
    const u64 i0 = lane * SL;
    const u64 i_end = min(i0 + SL, last_i + 1);
    const u64 j_end = min(i0 + SL + TAU - 1, n - TAU);
    u64* v = scratch + (u64)blockIdx.x * (SL + TAU);
    u8* mem = member + (u64)blockIdx.x * SL;
    if (threadIdx.x == 0) {
        u64 fp = 0;
        for (u64 k = 0; k < TAU; k++) fp = mod61_canon(((u64)((u128)fp * b % P61)) + T[i0 + k]);
        for (u64 j = i0; j <= j_end; j++) {
            const u64 t = (j + 127) >> 7;
            const u16 qi = qinfo[t];
            const u32 rel = (u32)(j + 127 - (t << 7));
            v[j - i0] = (rel >= (u32)(qi >> 8) && rel <= (u32)(qi & 255)) ? INF64 : fp;
            if (j < j_end) {
                u128 x = (u128)fp * b + T[j + TAU] + (u128)(P61 - bpow) * T[j];
                fp = (u64)(x % P61);
            }
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
            if (mem[i - i0]) ovf_out[(u64)blockIdx.x * SL + c++] = (u32)i;
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
    const u32* src = lane_flag[lane] ? ovf_out + (u64)ovf_slot[lane] * SL : lane_out + lane * LCAP;
    for (u32 x = 0; x < c; x++) S[o + x] = src[x];
}

static u64 pow61_host(u64 b, u64 e) {
    u64 r = 1;
    while (e) {
        if (e & 1) r = (u64)((u128)r * b % P61);
        b = (u64)((u128)b * b % P61);
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
    k_q_anchors<<<cdiv(nanch, QT_ANCH), QT_ANCH, 0, st>>>(T, n, nanch, qi, ctr + 0, rp, rhi, rlo, rcap);
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

    const u64 nlanes_need = last_i / SL + 1;
    const unsigned nwg = cdiv(nlanes_need, NLW);
    const u64 nlanes = (u64)nwg * NLW;
    u32* lo = lane_out.get(nlanes * LCAP);
    u32* lc = lane_cnt.get(nlanes + 1);
    u32* lf = lane_flag.get(nlanes);
    const u64 bpow = pow61_host(SSS_BASE, TAU);
    const u64 bn = (P61 - bpow) % P61;
    hipEvent_t e0, e1;
    LZ_HIP(hipEventCreate(&e0));
    LZ_HIP(hipEventCreate(&e1));
    LZ_HIP(hipEventRecord(e0, st));
    k_sss_main<<<nwg, NLW, 0, st>>>(T, n, last_i, qi, lo, lc, lf, ctr + 1, (u32)SSS_BASE, bn);
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

    // overflow lanes -> exact slow path
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
        u64* scratch = u64a.get(lanes.size() * (SL + TAU));
        u8* member = tmp_bytes.get(lanes.size() * SL);
        ovf_out = u32b.get(lanes.size() * SL);
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
