// engine.hip -- session lifetime, phase orchestration and the C-ABI
// (include/lz77sss.h).  The orchestration mirrors
// factorizer::factorize / compute_approximation (include/lz77_sss/lz77_sss.hpp:285-491)
// for fact_mode = greedy, phr_mode = lpf_opt, p = 1.
#include "../../include/lz77sss.h"
#include "../include/engine.h"
#include "../include/engine_if.h"

#include <hipcub/hipcub.hpp>

#include <chrono>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>

namespace LZ_NS {

void engine::init(int dev, u64 maxn) {
    device = dev;
    int cnt = 0;
    if (hipGetDeviceCount(&cnt) != hipSuccess || cnt <= 0) throw error(LZ77SSS_ENODEV, "no HIP device available");
    if (dev < 0 || dev >= cnt) throw error(LZ77SSS_EINVAL, "invalid device ordinal");
    LZ_HIP(hipSetDevice(dev));
    hipDeviceProp_t prop;
    LZ_HIP(hipGetDeviceProperties(&prop, dev));
    if (std::string(prop.gcnArchName).find("gfx950") == std::string::npos)
        throw error(LZ77SSS_ENODEV, std::string("device is not gfx950: ") + prop.gcnArchName);
    LZ_HIP(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    max_n = maxn;
    LZ_HIP(hipMalloc(&d_text, max_n + TEXT_PAD));
    LZ_HIP(hipMemsetAsync(d_text, 0, max_n + TEXT_PAD, st));
    LZ_HIP(hipHostMalloc(&h_pin, 256, hipHostMallocDefault));
    for (auto& e : ev_pin) LZ_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    LZ_HIP(hipStreamSynchronize(st));
}

void engine::load(const u8* h_text, u64 n_) {
    if (n_ > max_n) throw error(LZ77SSS_EINVAL, "text larger than the session capacity");
    LZ_HIP(hipSetDevice(device));
    n = n_;
    runs_valid = false;
    brk_valid = false;
    if (n) LZ_HIP(hipMemcpyAsync(d_text, h_text, n, hipMemcpyHostToDevice, st));
    LZ_HIP(hipMemsetAsync(d_text + n, 0, TEXT_PAD, st));
    LZ_HIP(hipStreamSynchronize(st));
}

void engine::destroy() {
    for (hipEvent_t* e : {&sss_ev0, &sss_ev1, &sss_evA, &sss_evB}) {
        if (*e) (void)hipEventDestroy(*e);
        *e = nullptr;
    }
    if (d_text) (void)hipFree(d_text);
    if (d_text_rev) (void)hipFree(d_text_rev);
    d_text = d_text_rev = nullptr;
    if (h_pin) (void)hipHostFree(h_pin);
    h_pin = nullptr;
    for (auto& e : ev_pin)
        if (e) (void)hipEventDestroy(e), e = nullptr;
    if (st) (void)hipStreamDestroy(st);
    st = nullptr;
}

// fact_mode = skip_phrases: the gapped stream of factorize_skip_gaps
// (approximate/factorize/skip_gaps.cpp:31-61): {beg of the first phrase, 0}, then
// per phrase {src, len} followed by {gap length, 0} when the next phrase (or the
// sentinel {n, n+1, 0}) starts after its end
struct fill_batch {
    u8* p[engine::FILL_MAX];
    u64 bytes[engine::FILL_MAX];
    u32 pat[engine::FILL_MAX];
};
// blockIdx.y = the fill; 32-bit stores over the aligned words, then the tail bytes
__global__ void k_fills(fill_batch B) {
    const u32 f = blockIdx.y;
    u8* p = B.p[f];
    const u64 nb = B.bytes[f];
    const u32 pat = B.pat[f];
    const u64 head = ((4 - ((uintptr_t)p & 3)) & 3) < nb ? ((4 - ((uintptr_t)p & 3)) & 3) : nb;
    const u64 nw = (nb - head) / 4;
    const u64 t0 = (u64)blockIdx.x * blockDim.x + threadIdx.x, str = (u64)gridDim.x * blockDim.x;
    u32* w = (u32*)(p + head);
    const u32 rot = 8 * (u32)(((uintptr_t)p + head) & 3);  // (0: the words are aligned)
    const u32 wp = rot ? (pat >> rot) | (pat << (32 - rot)) : pat;
    for (u64 k = t0; k < nw; k += str) w[k] = wp;
    if (t0 < head) p[t0] = (u8)(pat >> (8 * ((uintptr_t)(p + t0) & 3)));
    const u64 tail0 = head + 4 * nw;
    if (t0 < nb - tail0) p[tail0 + t0] = (u8)(pat >> (8 * ((uintptr_t)(p + tail0 + t0) & 3)));
}
void engine::fills(std::initializer_list<fill_op> ops) {
    fill_batch B{};
    u32 nf = 0;
    u64 wmax = 0;
    for (const fill_op& o : ops) {
        if (!o.bytes || !o.p) continue;
        if (nf == (u32)FILL_MAX) throw error(LZ77SSS_EINTERNAL, "fills: too many");
        B.p[nf] = (u8*)o.p;
        B.bytes[nf] = o.bytes;
        B.pat[nf] = o.pat;
        wmax = std::max<u64>(wmax, o.bytes / 4 + 4);
        nf++;
    }
    if (!nf) return;
    const u32 gx = (u32)std::min<u64>(std::max<u64>(1, cdiv(wmax, 256)), 2048);
    k_fills<<<dim3(gx, nf), 256, 0, st>>>(B);
    LZ_HIP(hipGetLastError());
}

__global__ void k_skip_counts(const pos_t* __restrict__ P, u32 m, u32* __restrict__ cnt) {
    const u64 k = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (k > m) return;
    cnt[k] = k == m ? 1u : 1u + (P[3 * (k + 1)] > P[3 * k + 1] ? 1u : 0u);  // slot m: the leading gap record
}
__global__ void k_skip_write(const pos_t* __restrict__ P, u32 m, const u32* __restrict__ off, pos_t* __restrict__ F) {
    const u64 k = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (k > m) return;
    if (k == m) {
        F[0] = P[0];  // beg of the first phrase (or n: the sentinel)
        F[1] = 0;
        return;
    }
    const u64 o = 1 + off[k];
    const pos_t beg = P[3 * k], end = P[3 * k + 1], src = P[3 * k + 2], nb = P[3 * (k + 1)];
    F[2 * o] = src;
    F[2 * o + 1] = end - beg;
    if (nb > end) {
        F[2 * o + 2] = nb - end;
        F[2 * o + 3] = 0;
    }
}
u64 engine::emit_skip_phrases() {
    const u32 m = num_phr;
    pos_t* P = lpf.get((u64)(m + 1) * 3);
    const pos_t sent[3] = {(pos_t)n, (pos_t)n + 1, 0};
    LZ_HIP(hipMemcpyAsync(P + 3 * (u64)m, sent, sizeof(sent), hipMemcpyHostToDevice, st));
    LZ_HIP(hipStreamSynchronize(st));  // sent is a stack array
    u32* cnt = u32a.get((u64)m + 2);
    u32* off = u32b.get((u64)m + 2);
    k_skip_counts<<<cdiv((u64)m + 1, 256), 256, 0, st>>>(P, m, cnt);
    size_t tb = 0;
    LZ_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, cnt, off, (int)(m + 1), st));
    u8* t = scan_tmp.get(tb);
    LZ_HIP(hipcub::DeviceScan::ExclusiveSum(t, tb, cnt, off, (int)(m + 1), st));
    const u32 last = rd1(off + m, st);  // records of the m phrases (slot m is the leading record)
    const u64 z = (u64)last + 1;
    pos_t* F = fact.get(2 * z + 2);
    k_skip_write<<<cdiv((u64)m + 1, 256), 256, 0, st>>>(P, m, off, F);
    LZ_HIP(hipGetLastError());
    return z;
}

void engine::prepare_phrases(int phr_mode, bool external_sss) {
    const bool dbg = debug_enabled();
    const char* lean_env = std::getenv("LZ77SSS_LEAN");
    const bool lean_mode = lean_env ? lean_env[0] != '0' : n >= (1ull << 33);
    lean = lean_mode;
    if (lean_mode) {
        release_greedy_buffers();  // the last call's emitter buffers go before the phases grow
        timer.mark("release");     // (the phases after it report peaks without those buffers)
    }
    phr_info.valid = false;
    if (std::getenv("LZ77SSS_LCE_DEBUG") && !lce_dbg) {
        LZ_HIP(hipMalloc(&lce_dbg, 8 * sizeof(unsigned long long)));
        LZ_HIP(hipMemset(lce_dbg, 0, 8 * sizeof(unsigned long long)));
    }
    auto trace = [&](const char* what) {
        if (!dbg) return;
        LZ_HIP(hipStreamSynchronize(st));
        std::fprintf(stderr, "[lz77sss-debug] done %s (|S|=%u phrases=%u)\n", what, s, num_phr);
        if (lce_dbg) {
            unsigned long long c[8];
            LZ_HIP(hipMemcpy(c, lce_dbg, sizeof(c), hipMemcpyDeviceToHost));
            LZ_HIP(hipMemset(lce_dbg, 0, sizeof(c)));
            std::fprintf(stderr, "[lz77sss-debug]   lce fwd calls=%llu steps=%llu skips=%llu exact=%llu max_steps=%llu | bwd calls=%llu steps=%llu skips=%llu\n",
                         c[0], c[1], c[2], c[3], c[4], c[5], c[6], c[7]);
        }
    };
    if (phr_mode == LZ77SSS_LPF_OPT || phr_mode == LZ77SSS_LPF_NAIVE) {
        if (external_sss) {
            build_q_runs(d_text);  // the LCE's run table; S came from set_sss
        } else {
            build_sss(d_text);
        }
        timer.mark("sss");
        trace("sss");
        build_sa_s(d_text);
        timer.mark("sa_s");
        trace("sa_s");
        build_lcp_rmq(d_text);
        timer.mark("lcp_rmq");
        trace("lcp_rmq");
        if (std::getenv("LZ77SSS_DEBUG_VERIFY")) debug_verify_lce("sa_s + lcp");
        if (phr_mode == LZ77SSS_LPF_OPT) build_lpf_opt(d_text);
        else build_lpf_naive(d_text);
        timer.mark("lpf");
        trace("lpf");
        if (std::getenv("LZ77SSS_DEBUG_VERIFY")) debug_verify_phrases("lpf");
    } else {
        if (external_sss) throw error(LZ77SSS_EINVAL, "an external sync set needs phr_mode lpf_opt or lpf_naive");
        build_lpf_lnf(phr_mode == LZ77SSS_LPF_LNF_OPT ? 1 : 0);
        trace("lpf_lnf");
    }
    // large texts: the phases' own scratch goes back before the emitter allocates its base set
    // (grow-only buffers otherwise keep every phase's peak: 2.5 GiB of 288 GiB were left free
    // after a 50 GiB factorization in round 4).  Small texts keep them for the next call.
    if (lean_mode) release_phase_scratch();
}

// the emitter's buffers of the last call (lean mode, before the phases of the next one grow)
void engine::release_greedy_buffers() {
    fact.release(); tmp_greedy.release(); chunk_buf.release(); chunk_buf2.release(); rem_buf.release();
    add_keys32.release(); add_pos.release(); dirty_in.release(); dirty_out.release(); dirty_sorted.release();
    tmp_greedy2.release(); tmp_greedy3.release(); add_keys.release(); add_keys2.release();
    seg_in_buf.release(); seg_out_buf.release(); seg_ids.release(); irank.release(); ekeys.release();
    evals.release(); ekeys2.release(); evals2.release(); occ_buf.release(); ist.release(); iend.release();
    ipos_buf.release(); iposr_buf.release(); tail_ins_buf.release(); seg_offs.release();
    g_sin.release(); g_sout.release(); g_valid.release(); g_cs.release(); g_tailc.release();
    g_succ.release(); g_seg_at.release(); g_ids.release(); g_chain.release(); g_dist[0].release(); g_dist[1].release();
    g_cbv.release(); g_bmI.release(); g_bmI2.release(); g_bmIb.release(); g_bmT.release();
    g_tmp1.release(); g_tmp2.release(); g_tmp3.release(); g_tmp4.release(); g_tmp5.release(); g_tmp6.release();
    g_tmp7.release(); g_tmp8.release(); g_ark.release(); g_ast.release(); g_aen.release(); g_offs.release();
    g_predk.release(); g_wk.release(); g_ids2.release(); g_brev.release(); g_bsum.release(); g_bincl.release();
    g_pbtmp.release(); g_pbcur.release(); g_pbm.release(); g_pwp.release(); g_pcnt.release(); g_sdk.release();
    g_dstart.release(); g_pflag.release(); g_bstart.release(); g_abeg.release(); g_abeg2.release(); g_bmA.release();
    g_x32.release(); g_xpos.release(); g_stash.release(); g_H.release(); g_Hs.release(); g_hsused.release();
    g_hsave.release(); g_htrue.release(); g_specbad.release(); fact_acc.release(); g_cut.release();
    g_xk.release(); g_xk2.release(); g_ls_h.release(); g_ls_g.release(); g_lng.release(); g_pbw.release();
    num_fact = 0;  // (the factors went with fact; the callers set last_fact_mode when they write new ones)
    negpow_key = {};  // the influence tables lived in tmp_greedy
    negpow_dev = nullptr;
    seg_at_clean = false;
    seg_at_n = 0;
}

// the buffers the phases before the emitter use only while they run: the SSS pass's stripe
// outputs, filter words, tile lists and run-record inputs, SA_S's rank levels and sort scratch,
// LPF's sparse tables over SA, PSV/NSV, candidates and pointer-doubling levels, the shared scratch.  Kept: the text, S, SA / ISA / LCP and its RMQ
// levels, the successor table, the run tables and block records (the LCE's view), the phrases.
void engine::release_phase_scratch() {
    lane_out.release(); lane_cnt.release(); lane_flag.release(); sss_ovf.release();
    sss_hitw.release(); sss_tflag.release(); sss_tiles.release(); sss_sflag.release(); sss_slist.release();
    sss_fcnt.release(); sss_tot.release(); q_info.release();
    blk_p.release(); blk_fo.release(); blk_lo.release(); blk_mk.release(); blk_ser.release(); blk_ss.release();
    run_scan_a.release(); run_scan_b.release(); S64.release(); s64 = 0;
    for (auto& b : rank_lv) b.release();
    nlev_rank = 0;
    for (auto& b : sa_min) b.release();
    for (auto& b : jump) b.release();  // (the emitter's segment linking grows its own levels again)
    PSV.release(); NSV.release(); cand.release(); p_Em.release(); p_lst.release(); p_ph3.release();
    key_len.release(); sa_tmp1.release(); sa_tmp2.release(); sa_tmp3.release();
    tmp_bytes.release(); tmp_bytes2.release(); tmp_bytes3.release(); scan_tmp.release();
    u64a.release(); u64b.release(); u32a.release(); u32b.release(); u32c.release(); u32d.release(); u32e.release();
    stats_released_scratch++;
}

void engine::set_sss(const pos_t* S_any, u64 count, bool runs) {
    LZ_HIP(hipSetDevice(device));
    // the same bound as build_sss: SA_S / LPF pass item counts to hipcub / rocprim as int
    if (count >= 0x7FFFFFFFull) throw error(LZ77SSS_EINVAL, "sync set too large");
    pos_t* d = S.get(count + 1);
    if (count) LZ_HIP(hipMemcpyAsync(d, S_any, count * sizeof(pos_t), hipMemcpyDefault, st));
    LZ_HIP(hipStreamSynchronize(st));
    s = (u32)count;
    has_runs = runs;
}

u64 engine::factorize(int phr_mode, u32 rk_seed, int log2_override, bool log, int fact_mode) {
    LZ_HIP(hipSetDevice(device));
    if (phr_mode < LZ77SSS_LPF_NAIVE || phr_mode > LZ77SSS_LPF_LNF_OPT) throw error(LZ77SSS_EINVAL, "unsupported phrase mode");
    if (n > POS_MAX_N)
        throw error(LZ77SSS_EINVAL, sizeof(pos_t) == 4 ? "n too large for pos_t = uint32_t" : "n too large");
    num_fact = 0;
    last_fact_mode = fact_mode;
    stats.assign(28, 0);
    if (n == 0) return 0;
    const auto t_start = std::chrono::steady_clock::now();
    const u64 peak0 = g_dev_bytes.load();
    if (log) g_dev_peak.store(peak0);
    timer.begin(st);
    prepare_phrases(phr_mode, false);
    if (fact_mode == LZ77SSS_SKIP_PHRASES) {
        num_fact = emit_skip_phrases();
        timer.mark("skip_phrases");
    } else {
        num_fact = factorize_greedy(d_text, rk_seed, log2_override);
        timer.mark("greedy");
    }
    if (std::getenv("LZ77SSS_DEBUG_VERIFY") && fact_mode != LZ77SSS_SKIP_PHRASES) {
        u64 first = 0;
        const u64 bad = verify_factors(fact.p, num_fact, n, d_text, &first);
        std::fprintf(stderr, "[lz77sss-verify] factors: z=%llu bad positions=%llu first=%llu\n",
                     (unsigned long long)num_fact, (unsigned long long)bad, (unsigned long long)first);
    }
    if (debug_enabled()) std::fprintf(stderr, "[lz77sss-debug] done greedy (|S|=%u phrases=%u)\n", s, num_phr);
    stream_wait(st);
    if (log) {
        for (auto& [name, ms] : timer.read()) std::fprintf(stderr, "[lz77sss] %-10s %9.3f ms\n", name.c_str(), ms);
        std::fprintf(stderr, "[lz77sss] n=%llu |S|=%u phrases=%u factors=%llu outer=%llu rounds=%llu\n",
                     (unsigned long long)n, s, num_phr, (unsigned long long)num_fact,
                     (unsigned long long)stats[12], (unsigned long long)stats[13]);
        if (fact_mode != LZ77SSS_SKIP_PHRASES) log_summary(t_start);
    }
    return num_fact;
}

// the summary a logged factorization prints (lz77_sss.hpp:345-353, formats of
// misc/utils.hpp:54-96); peak memory = the session's peak device bytes + n (the text)
static std::string fmt_time(u64 ns) {
    if (ns > 10000000000ull) return std::to_string(ns / 1000000000) + " s";
    if (ns > 10000000ull) return std::to_string(ns / 1000000) + " ms";
    if (ns > 10000ull) return std::to_string(ns / 1000) + " us";
    return std::to_string(ns) + " ns";
}
static std::string fmt_size(u64 B) {
    if (B > 10000000000ull) return std::to_string(B / 1000000000) + " GB";
    if (B > 10000000ull) return std::to_string(B / 1000000) + " MB";
    if (B > 10000ull) return std::to_string(B / 1000) + " KB";
    return std::to_string(B) + " B";
}
void engine::log_summary(std::chrono::steady_clock::time_point t_start) const {
    const u64 ns = (u64)std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t_start).count();
    const double comp_ratio = n / (double)std::max<u64>(1, num_fact);
    const double tp = 1000.0 * (double)n / (double)std::max<u64>(1, ns);
    std::printf("num. of factors: %llu\n", (unsigned long long)num_fact);
    std::printf("input length / num. of factors: %s\n", std::to_string(comp_ratio).c_str());
    std::printf("total time: %s\n", fmt_time(ns).c_str());
    std::printf("throughput: %s MB/s\n", std::to_string(tp).c_str());
    std::printf("peak memory consumption: %s\n", fmt_size(g_dev_peak.load() + n).c_str());
    std::fflush(stdout);
}

// the two halves of lz77sss_session_prepare / _greedy_block (a block of a sharded run)
static u64 block_prepare(engine& E, int phr_mode, bool external_sss, int log2_override) {
    LZ_HIP(hipSetDevice(E.device));
    if (phr_mode != LZ77SSS_LPF_OPT && phr_mode != LZ77SSS_LPF_NAIVE)
        throw error(LZ77SSS_EINVAL, "a sharded factorization needs phr_mode lpf_opt or lpf_naive");
    if (E.n > POS_MAX_N) throw error(LZ77SSS_EINVAL, "n too large for pos_t");
    E.num_fact = 0;
    E.last_fact_mode = LZ77SSS_GREEDY;
    E.stats.assign(28, 0);
    E.spec_track = false;
    E.timer.begin(E.st);
    E.prepare_phrases(phr_mode, external_sss);
    const u64 ent = E.n ? E.carried_entries(log2_override) : 1;
    E.g_Hs.get(ent);
    LZ_HIP(hipStreamSynchronize(E.st));
    return ent * sizeof(pos_t);
}
static u64 block_run(engine& E, u32 rk_seed, int log2_override, u64* st) {
    LZ_HIP(hipSetDevice(E.device));
    greedy_block b;
    b.start = (pos_t)st[0];
    b.idxpos = (pos_t)st[1];
    b.zmask = (u32)st[2];
    b.carried = (st[3] & 1) != 0;
    b.seed = (st[3] & 2) != 0;
    b.end = (pos_t)st[4];
    E.timer.begin(E.st);
    E.last_fact_mode = LZ77SSS_GREEDY;
    E.num_fact = E.n ? E.factorize_greedy(E.d_text, rk_seed, log2_override, &b) : 0;
    E.timer.mark("greedy");
    LZ_HIP(hipStreamSynchronize(E.st));
    st[5] = b.exit_start;
    st[6] = b.exit_idxpos;
    st[7] = b.exit_zmask;
    return E.num_fact;
}

}  // namespace LZ_NS

#ifdef LZ_POS64
// ===========================================================================
// the pos_t = uint64_t engine behind the C-ABI's 64-bit sessions (engine_if.h)
// ===========================================================================
namespace lz64 {
struct engine64_impl final : lz::engine_if {
    engine E;
    ~engine64_impl() override { E.destroy(); }
    int device() const override { return E.device; }
    u64 n() const override { return E.n; }
    u64 max_n() const override { return E.max_n; }
    u8* text() override { return E.d_text; }
    hipStream_t stream() override { return E.st; }
    void set_n(u64 n) override { E.n = n; }
    void load(const u8* t, u64 n) override { E.load(t, n); }
    u64 factorize(int phr, u32 seed, int log2, bool log, int fact_mode) override {
        return E.factorize(phr, seed, log2, log, fact_mode);
    }
    u64 num_fact() const override { return E.num_fact; }
    const u64* factors() const override { return E.fact.p; }
    u64* factors_buf(u64 nf) override { return E.fact.get(2 * nf + 2); }
    u64 decode(const u64* F, u64 nf, u64 n_out, u8* d_out, bool cmp) override {
        return E.decode_device(F, nf, n_out, d_out, cmp ? E.d_text : nullptr);
    }
    u8* dec_out(u64 n) override { return E.dec_out.get(n); }
    u64 verify(u64* first_bad) override {
        E.check_verifiable();
        const u64 bad = E.verify_factors(E.fact.p, E.num_fact, E.n, E.d_text, first_bad);
        LZ_HIP(hipStreamSynchronize(E.st));
        return bad;
    }
    void sss(u64* size, int* has_runs) override {
        LZ_HIP(hipSetDevice(E.device));
        E.build_sss(E.d_text);
        LZ_HIP(hipStreamSynchronize(E.st));
        *size = E.s;
        *has_runs = E.has_runs;
    }
    u64 sss_size() const override { return E.s; }
    const u64* sss_ptr() const override { return E.S.p; }
    void sss_range(u64 first, u64 end, u64 base, u64 window, u64* size, int* has_runs) override {
        LZ_HIP(hipSetDevice(E.device));
        E.build_sss_range(first, end, base, window);
        *size = E.s64;
        *has_runs = E.has_runs64;
    }
    u64 range_size() const override { return E.s64; }
    const u64* range_ptr() const override { return E.S64.p; }
    u64 num_phr() const override { return E.num_phr; }
    const u64* lpf_ptr() const override { return E.lpf.p; }
    const u32* sa_ptr() const override { return E.SA.p; }
    const u32* lcp_ptr() const override { return E.lcp_rmq[0].p; }
    std::vector<u64>& stats() override { return E.stats; }
    lz::phase_timer& timer() override { return E.timer; }
    double sss_kernel_ms() const override { return E.sss_ms(); }
    u64 sss_kernel_bytes() const override { return E.sss_kernel_bytes; }
    u32 dec_rounds() const override { return E.dec_rounds; }
    void set_sss(const u64* S_any, u64 count, bool runs) override { E.set_sss(S_any, count, runs); }
    u64 prepare(int phr_mode, bool external_sss, int log2_override) override {
        return block_prepare(E, phr_mode, external_sss, log2_override);
    }
    void* carried_table() override { return E.g_Hs.p; }
    u64 carried_bytes() const override { return E.g_Hs.cap * sizeof(pos_t); }
    u64 greedy_block(u32 rk_seed, int log2_override, u64* st) override { return block_run(E, rk_seed, log2_override, st); }
    void spec_begin(int part, u64 base) override { E.spec_begin(part, base); }
    int spec_resolve(const void* true_tab, u64 bytes, int parts) override {
        return E.spec_resolve(true_tab, bytes, parts);
    }
};
}  // namespace lz64
namespace lz {
engine_if* make_engine64(int dev, u64 maxn) {
    auto* p = new lz64::engine64_impl();
    try {
        p->E.init(dev, maxn);
    } catch (...) {
        delete p;
        throw;
    }
    return p;
}
}  // namespace lz
#else
// ===========================================================================
// C-ABI
// ===========================================================================
struct lz77sss_session {
    lz::engine E;                          // pos_t = uint32_t sessions
    std::unique_ptr<lz::engine_if> E64;    // pos_t = uint64_t sessions (lz77sss_session_create64)
    bool range64 = false;                  // E64: the last sync set came from sss_range
};

static thread_local std::string g_err;

template <class F>
static int guarded(F&& f) {
    try {
        f();
        return LZ77SSS_OK;
    } catch (const lz::error& e) {
        g_err = e.what();
        return e.code;
    } catch (const std::bad_alloc&) {
        g_err = "out of memory";
        return LZ77SSS_ENOMEM;
    } catch (const std::exception& e) {
        g_err = e.what();
        return LZ77SSS_EINTERNAL;
    }
}
static void need32(lz77sss_session* s, const char* what) {
    if (s->E64) throw lz::error(LZ77SSS_EINVAL, std::string(what) + " is not available on a pos_t = uint64_t session");
}

extern "C" {

LZ77SSS_API const char* lz77sss_last_error(void) { return g_err.c_str(); }

LZ77SSS_API int lz77sss_device_count(void) {
    int c = 0;
    if (hipGetDeviceCount(&c) != hipSuccess) return 0;
    return c;
}

LZ77SSS_API void lz77sss_default_params(lz77sss_params* prm) {
    if (!prm) return;
    std::memset(prm, 0, sizeof(*prm));
    prm->phr_mode = LZ77SSS_LPF_OPT;
    prm->fact_mode = LZ77SSS_GREEDY;
    prm->tau = 512;
    prm->rk_seed = 42;
    prm->index_log2_size = 0;
    prm->device = 0;
    prm->log = 0;
    prm->num_threads = 0;
}

static void check_params(const lz77sss_params* prm) {
    if (!prm) throw lz::error(LZ77SSS_EINVAL, "params is NULL");
    if (prm->tau != 512) throw lz::error(LZ77SSS_EINVAL, "only tau = 512 is supported");
    if (prm->fact_mode != LZ77SSS_GREEDY && prm->fact_mode != LZ77SSS_SKIP_PHRASES)
        throw lz::error(LZ77SSS_EINVAL, "supported fact_modes: greedy, skip_phrases");
    if (prm->phr_mode < LZ77SSS_LPF_NAIVE || prm->phr_mode > LZ77SSS_LPF_LNF_OPT)
        throw lz::error(LZ77SSS_EINVAL, "unsupported phr_mode");
    if (prm->index_log2_size < 0 || prm->index_log2_size > 30) throw lz::error(LZ77SSS_EINVAL, "bad index_log2_size");
}

// factorize_exact<greedy, lpf_opt, transf_mode, range_ds_t, tau> (lz77_sss.hpp:188-200)
static void check_exact_params(const lz77sss_params* prm, int transf_mode) {
    if (!prm) throw lz::error(LZ77SSS_EINVAL, "params is NULL");
    if (prm->tau != 512) throw lz::error(LZ77SSS_EINVAL, "only tau = 512 is supported");
    if (prm->fact_mode != LZ77SSS_GREEDY) throw lz::error(LZ77SSS_EINVAL, "exact mode requires fact_mode = greedy");
    if (prm->phr_mode != LZ77SSS_LPF_OPT && prm->phr_mode != LZ77SSS_LPF_LNF_OPT)
        throw lz::error(LZ77SSS_EINVAL, "unsupported phr_mode");
    if (transf_mode < LZ77SSS_TRANSF_NAIVE || transf_mode > LZ77SSS_TRANSF_FULL_SA)
        throw lz::error(LZ77SSS_EINVAL, "unsupported transf_mode");
}

LZ77SSS_API int lz77sss_session_create(int device, uint64_t max_n, lz77sss_session** out) {
    if (!out) return LZ77SSS_EINVAL;
    *out = nullptr;
    lz77sss_session* s = new (std::nothrow) lz77sss_session();
    if (!s) return LZ77SSS_ENOMEM;
    int rc = guarded([&] { s->E.init(device, max_n); });
    if (rc) {
        s->E.destroy();
        delete s;
        return rc;
    }
    *out = s;
    return LZ77SSS_OK;
}

LZ77SSS_API int lz77sss_session_create64(int device, uint64_t max_n, lz77sss_session** out) {
    if (!out) return LZ77SSS_EINVAL;
    *out = nullptr;
    lz77sss_session* s = new (std::nothrow) lz77sss_session();
    if (!s) return LZ77SSS_ENOMEM;
    int rc = guarded([&] { s->E64.reset(lz::make_engine64(device, max_n)); });
    if (rc) {
        delete s;
        return rc;
    }
    *out = s;
    return LZ77SSS_OK;
}

LZ77SSS_API int lz77sss_session_is64(const lz77sss_session* s) { return s && s->E64 ? 1 : 0; }

LZ77SSS_API int lz77sss_session_load(lz77sss_session* s, const uint8_t* text, uint64_t n) {
    if (!s || (!text && n)) return LZ77SSS_EINVAL;
    return guarded([&] {
        if (s->E64) s->E64->load(text, n);
        else s->E.load(text, n);
    });
}

LZ77SSS_API int lz77sss_session_factorize(lz77sss_session* s, const lz77sss_params* prm, uint64_t* num_factors) {
    if (!s) return LZ77SSS_EINVAL;
    return guarded([&] {
        check_params(prm);
        s->range64 = false;
        uint64_t z = s->E64 ? s->E64->factorize(prm->phr_mode, prm->rk_seed, prm->index_log2_size, prm->log != 0,
                                                 prm->fact_mode)
                            : s->E.factorize(prm->phr_mode, prm->rk_seed, prm->index_log2_size, prm->log != 0,
                                             prm->fact_mode);
        if (num_factors) *num_factors = z;
    });
}

LZ77SSS_API int lz77sss_session_factorize_exact(lz77sss_session* s, const lz77sss_params* prm, int transf_mode,
                                                uint64_t* num_factors) {
    if (!s) return LZ77SSS_EINVAL;
    return guarded([&] {
        need32(s, "session_factorize_exact");
        check_exact_params(prm, transf_mode);
        // the reference's transforms run the sample-index path (csrc/smpl.hip); FULL_SA the
        // full suffix array (csrc/exact.hip)
        uint64_t z = transf_mode == LZ77SSS_TRANSF_FULL_SA
                         ? s->E.factorize_exact(prm->log != 0)
                         : s->E.factorize_exact_smpl(transf_mode, prm->phr_mode, prm->rk_seed, prm->index_log2_size,
                                                     prm->log != 0);
        if (num_factors) *num_factors = z;
    });
}

LZ77SSS_API int lz77sss_session_get_factors(lz77sss_session* s, lz77sss_factor32* out, uint64_t cap) {
    if (!s) return LZ77SSS_EINVAL;
    return guarded([&] {
        need32(s, "get_factors (32-bit layout)");
        if (!out && s->E.num_fact) throw lz::error(LZ77SSS_EINVAL, "out is NULL");
        if (cap < s->E.num_fact) throw lz::error(LZ77SSS_EINVAL, "output capacity too small");
        if (s->E.num_fact)
            LZ_HIP(hipMemcpy(out, s->E.fact.p, s->E.num_fact * sizeof(lz77sss_factor32), hipMemcpyDeviceToHost));
    });
}

// the 10-byte serialized pos_t = uint64_t factor of lz77_sss.hpp:149-173 is a storage
// format; in memory a factor is {uint64_t src, uint64_t len} (lz77_sss.hpp:129-147)
LZ77SSS_API int lz77sss_session_get_factors64(lz77sss_session* s, lz77sss_factor64* out, uint64_t cap) {
    if (!s) return LZ77SSS_EINVAL;
    return guarded([&] {
        const uint64_t z = s->E64 ? s->E64->num_fact() : s->E.num_fact;
        if (!out && z) throw lz::error(LZ77SSS_EINVAL, "out is NULL");
        if (cap < z) throw lz::error(LZ77SSS_EINVAL, "output capacity too small");
        if (!z) return;
        if (s->E64) {
            LZ_HIP(hipMemcpy(out, s->E64->factors(), z * sizeof(lz77sss_factor64), hipMemcpyDeviceToHost));
        } else {
            std::vector<lz77sss_factor32> tmp(z);
            LZ_HIP(hipMemcpy(tmp.data(), s->E.fact.p, z * sizeof(lz77sss_factor32), hipMemcpyDeviceToHost));
            for (uint64_t k = 0; k < z; k++) out[k] = lz77sss_factor64{tmp[k].src, tmp[k].len};
        }
    });
}

// decode on the device: the factors of the last factorize call (already in HBM)
LZ77SSS_API int lz77sss_session_decode(lz77sss_session* s, uint8_t* out, uint64_t cap, uint64_t* mismatches) {
    if (!s) return LZ77SSS_EINVAL;
    return guarded([&] {
        if (s->E64) {
            lz::engine_if& E = *s->E64;
            LZ_HIP(hipSetDevice(E.device()));
            if (out && cap < E.n()) throw lz::error(LZ77SSS_EINVAL, "output capacity too small");
            lz::u8* d_out = out && E.n() ? E.dec_out(E.n()) : nullptr;
            E.timer().begin(E.stream());
            const uint64_t bad = E.decode(E.factors(), E.num_fact(), E.n(), d_out, mismatches != nullptr);
            E.timer().mark("decode");
            if (E.stats().size() > 18) E.stats()[18] = E.dec_rounds();
            if (mismatches) *mismatches = bad;
            if (d_out) LZ_HIP(hipMemcpyAsync(out, d_out, E.n(), hipMemcpyDeviceToHost, E.stream()));
            LZ_HIP(hipStreamSynchronize(E.stream()));
            return;
        }
        lz::engine& E = s->E;
        LZ_HIP(hipSetDevice(E.device));
        if (out && cap < E.n) throw lz::error(LZ77SSS_EINVAL, "output capacity too small");
        lz::u8* d_out = out && E.n ? E.dec_out.get(E.n) : nullptr;
        E.timer.begin(E.st);
        const uint64_t bad = E.decode_device(E.fact.p, E.num_fact, E.n, d_out, mismatches ? E.d_text : nullptr);
        E.timer.mark("decode");
        if (E.stats.size() > 18) E.stats[18] = E.dec_rounds;
        if (mismatches) *mismatches = bad;
        if (d_out) LZ_HIP(hipMemcpyAsync(out, d_out, E.n, hipMemcpyDeviceToHost, E.st));
        LZ_HIP(hipStreamSynchronize(E.st));
    });
}

// the factors of the last factorization checked against the loaded text in HBM (csrc/decode.hip
// verify_factors): the decode round trip without materialising the decoded text
LZ77SSS_API int lz77sss_session_verify(lz77sss_session* s, uint64_t* bad_positions, uint64_t* first_bad) {
    if (!s || !bad_positions) return LZ77SSS_EINVAL;
    return guarded([&] {
        if (s->E64) {
            LZ_HIP(hipSetDevice(s->E64->device()));
            *bad_positions = s->E64->verify(first_bad);
            return;
        }
        lz::engine& E = s->E;
        E.check_verifiable();
        LZ_HIP(hipSetDevice(E.device));
        *bad_positions = E.verify_factors(E.fact.p, E.num_fact, E.n, E.d_text, first_bad);
        LZ_HIP(hipStreamSynchronize(E.st));
    });
}

LZ77SSS_API int lz77sss_session_sss(lz77sss_session* s, uint64_t* size_sss, int* has_runs) {
    if (!s) return LZ77SSS_EINVAL;
    return guarded([&] {
        if (s->E64) {
            uint64_t sz = 0;
            int hr = 0;
            s->E64->sss(&sz, &hr);
            s->range64 = false;
            if (size_sss) *size_sss = sz;
            if (has_runs) *has_runs = hr;
            return;
        }
        LZ_HIP(hipSetDevice(s->E.device));
        s->E.build_sss(s->E.d_text);
        LZ_HIP(hipStreamSynchronize(s->E.st));
        if (size_sss) *size_sss = s->E.s;
        if (has_runs) *has_runs = s->E.has_runs;
    });
}

LZ77SSS_API int lz77sss_session_sss_range(lz77sss_session* s, uint64_t first, uint64_t end, uint64_t base,
                                          uint64_t window, uint64_t* size_sss, int* has_runs) {
    if (!s) return LZ77SSS_EINVAL;
    return guarded([&] {
        if (s->E64) {
            uint64_t cnt = 0;
            int hr = 0;
            s->E64->sss_range(first, end, base, window, &cnt, &hr);
            s->range64 = true;
            if (size_sss) *size_sss = cnt;
            if (has_runs) *has_runs = hr;
            return;
        }
        LZ_HIP(hipSetDevice(s->E.device));
        s->E.build_sss_range(first, end, base, window);
        if (size_sss) *size_sss = s->E.s64;
        if (has_runs) *has_runs = s->E.has_runs64;
    });
}

// 64-bit sync set: of the last sss_range call (32-bit session) or of the last sss /
// factorize call (64-bit session)
static void sss64_src(lz77sss_session* s, const uint64_t*& p, uint64_t& cnt) {
    if (s->E64 && s->range64) {
        p = s->E64->range_ptr();
        cnt = s->E64->range_size();
    } else if (s->E64) {
        p = s->E64->sss_ptr();
        cnt = s->E64->sss_size();
    } else {
        p = s->E.S64.p;
        cnt = s->E.s64;
    }
}

LZ77SSS_API int lz77sss_session_get_sss64(lz77sss_session* s, uint64_t* out, uint64_t cap) {
    if (!s) return LZ77SSS_EINVAL;
    return guarded([&] {
        const uint64_t* p;
        uint64_t cnt;
        sss64_src(s, p, cnt);
        if (!out && cnt) throw lz::error(LZ77SSS_EINVAL, "out is NULL");
        if (cap < cnt) throw lz::error(LZ77SSS_EINVAL, "output capacity too small");
        if (cnt) LZ_HIP(hipMemcpy(out, p, cnt * 8, hipMemcpyDeviceToHost));
    });
}

LZ77SSS_API int lz77sss_session_copy_sss64_device(lz77sss_session* s, void* dst, uint64_t cap) {
    if (!s) return LZ77SSS_EINVAL;
    return guarded([&] {
        const uint64_t* p;
        uint64_t cnt;
        sss64_src(s, p, cnt);
        if (!dst && cnt) throw lz::error(LZ77SSS_EINVAL, "dst is NULL");
        if (cap < cnt) throw lz::error(LZ77SSS_EINVAL, "output capacity too small");
        const int dev = s->E64 ? s->E64->device() : s->E.device;
        hipStream_t st = s->E64 ? s->E64->stream() : s->E.st;
        LZ_HIP(hipSetDevice(dev));
        if (cnt) LZ_HIP(hipMemcpyAsync(dst, p, cnt * 8, hipMemcpyDeviceToDevice, st));
        LZ_HIP(hipStreamSynchronize(st));
    });
}

// device-to-device copy of the last factorization in the session's own layout
// ({u32 src, u32 len} or {u64 src, u64 len} per factor): the emission step of a
// sharded run gathers these bytes over RCCL without a host round trip
LZ77SSS_API int lz77sss_session_copy_factors_device(lz77sss_session* s, void* dst, uint64_t cap_bytes,
                                                    uint64_t* bytes) {
    if (!s) return LZ77SSS_EINVAL;
    return guarded([&] {
        const uint64_t z = s->E64 ? s->E64->num_fact() : s->E.num_fact;
        const uint64_t nb = z * (s->E64 ? sizeof(lz77sss_factor64) : sizeof(lz77sss_factor32));
        if (bytes) *bytes = nb;
        if (!dst) {
            if (cap_bytes) throw lz::error(LZ77SSS_EINVAL, "dst is NULL");
            return;
        }
        if (cap_bytes < nb) throw lz::error(LZ77SSS_EINVAL, "output capacity too small");
        const int dev = s->E64 ? s->E64->device() : s->E.device;
        hipStream_t st = s->E64 ? s->E64->stream() : s->E.st;
        const void* src = s->E64 ? (const void*)s->E64->factors() : (const void*)s->E.fact.p;
        LZ_HIP(hipSetDevice(dev));
        if (nb) LZ_HIP(hipMemcpyAsync(dst, src, nb, hipMemcpyDefault, st));
        LZ_HIP(hipStreamSynchronize(st));
    });
}

// chr19-style text in HBM: byte p of the text is a function of (p, seed) only
__device__ __forceinline__ lz::u64 gen_mix(lz::u64 x) {  // splitmix64 finalizer
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}
__global__ void k_gen_genome(lz::u8* __restrict__ out, lz::u64 n, lz::u64 offset, lz::u64 base_len,
                             lz::u64 mut_thr, lz::u64 seed) {
    for (lz::u64 i0 = lz::gtid() * 16; i0 < n; i0 += lz::gstride() * 16) {
    lz::u32 w[4] = {0, 0, 0, 0};
    for (int k = 0; k < 16 && i0 + k < n; k++) {
        const lz::u64 p = offset + i0 + k;
        const lz::u64 q = p % base_len;
        lz::u32 c = (lz::u32)(gen_mix(q ^ (seed << 40)) >> 62);
        if (p >= base_len) {
            const lz::u64 h = gen_mix(p ^ (seed * 0xD6E8FEB86659FD93ull) ^ 0x5851F42D4C957F2Dull);
            if (h < mut_thr) c = (c + 1 + (lz::u32)((h >> 7) % 3)) & 3;
        }
        w[k >> 2] |= (lz::u32)"ACGT"[c] << (8 * (k & 3));
    }
    if (i0 + 16 <= n) {
        *(uint4*)(out + i0) = make_uint4(w[0], w[1], w[2], w[3]);
    } else {
        for (int k = 0; i0 + k < n; k++) out[i0 + k] = (lz::u8)(w[k >> 2] >> (8 * (k & 3)));
    }
    }
}

LZ77SSS_API int lz77sss_session_gen_genome(lz77sss_session* s, uint64_t n, uint64_t base_len, double mut_rate,
                                           uint32_t seed, uint64_t offset) {
    if (!s || base_len == 0 || !(mut_rate >= 0.0 && mut_rate <= 1.0)) return LZ77SSS_EINVAL;
    return guarded([&] {
        const int dev = s->E64 ? s->E64->device() : s->E.device;
        const uint64_t cap = s->E64 ? s->E64->max_n() : s->E.max_n;
        lz::u8* text = s->E64 ? s->E64->text() : s->E.d_text;
        hipStream_t st = s->E64 ? s->E64->stream() : s->E.st;
        if (n > cap) throw lz::error(LZ77SSS_EINVAL, "text larger than the session capacity");
        LZ_HIP(hipSetDevice(dev));
        if (s->E64) s->E64->set_n(n);
        else s->E.n = n;
        const lz::u64 thr = mut_rate >= 1.0 ? ~0ull : (lz::u64)(mut_rate * 18446744073709551616.0);
        if (n) k_gen_genome<<<lz::capped_grid((n + 15) / 16, 256), 256, 0, st>>>(text, n, offset, base_len, thr, seed);
        LZ_HIP(hipGetLastError());
        LZ_HIP(hipMemsetAsync(text + n, 0, lz::TEXT_PAD, st));
        LZ_HIP(hipStreamSynchronize(st));
    });
}

// Huffman factor container of the last greedy / exact factorization (csrc/huffman.hip)
LZ77SSS_API int lz77sss_session_huffman(lz77sss_session* s, uint8_t* out, uint64_t cap, uint64_t* size) {
    if (!s) return LZ77SSS_EINVAL;
    return guarded([&] {
        need32(s, "huffman");
        lz::engine& E = s->E;
        if (E.last_fact_mode == LZ77SSS_SKIP_PHRASES)
            throw lz::error(LZ77SSS_EINVAL, "the Huffman container holds a factorization, not a skip_phrases stream");
        LZ_HIP(hipSetDevice(E.device));
        const uint64_t b = E.huffman_container();
        if (size) *size = b;
        if (out) {
            if (cap < b) throw lz::error(LZ77SSS_EINVAL, "output capacity too small");
            LZ_HIP(hipMemcpy(out, E.hf_out.p, b, hipMemcpyDeviceToHost));
        }
    });
}

// ssszip's gapped container of the last skip_phrases factorization (csrc/ssszip.hip)
LZ77SSS_API int lz77sss_session_ssszip_gapped(lz77sss_session* s, uint8_t* out, uint64_t cap, uint64_t* size) {
    if (!s) return LZ77SSS_EINVAL;
    return guarded([&] {
        need32(s, "ssszip_gapped");
        lz::engine& E = s->E;
        if (E.last_fact_mode != LZ77SSS_SKIP_PHRASES)
            throw lz::error(LZ77SSS_EINVAL, "ssszip_gapped needs a preceding factorize with fact_mode = skip_phrases");
        LZ_HIP(hipSetDevice(E.device));
        const uint64_t b = E.ssszip_gapped();
        if (size) *size = b;
        if (out) {
            if (cap < b) throw lz::error(LZ77SSS_EINVAL, "output capacity too small");
            LZ_HIP(hipMemcpy(out, E.ssz_out.p, b, hipMemcpyDeviceToHost));
        }
    });
}

LZ77SSS_API int lz77sss_session_get_sss(lz77sss_session* s, uint32_t* out, uint64_t cap) {
    if (!s) return LZ77SSS_EINVAL;
    return guarded([&] {
        need32(s, "get_sss (32-bit positions)");
        if (cap < s->E.s) throw lz::error(LZ77SSS_EINVAL, "output capacity too small");
        if (s->E.s) LZ_HIP(hipMemcpy(out, s->E.S.p, (size_t)s->E.s * 4, hipMemcpyDeviceToHost));
    });
}

LZ77SSS_API int lz77sss_session_get_sa_s(lz77sss_session* s, uint32_t* sa, uint32_t* lcp, uint64_t cap) {
    if (!s) return LZ77SSS_EINVAL;
    return guarded([&] {
        const uint64_t cnt = s->E64 ? s->E64->sss_size() : s->E.s;
        if (cap < cnt) throw lz::error(LZ77SSS_EINVAL, "output capacity too small");
        if (!cnt) return;
        const uint32_t* psa = s->E64 ? s->E64->sa_ptr() : s->E.SA.p;
        const uint32_t* plcp = s->E64 ? s->E64->lcp_ptr() : s->E.lcp_rmq[0].p;
        if (sa) LZ_HIP(hipMemcpy(sa, psa, (size_t)cnt * 4, hipMemcpyDeviceToHost));
        if (lcp) LZ_HIP(hipMemcpy(lcp, plcp, (size_t)cnt * 4, hipMemcpyDeviceToHost));
    });
}

LZ77SSS_API int lz77sss_session_get_lpf(lz77sss_session* s, uint32_t* out3, uint64_t cap, uint64_t* count) {
    if (!s) return LZ77SSS_EINVAL;
    return guarded([&] {
        need32(s, "get_lpf (32-bit positions)");
        if (count) *count = s->E.num_phr;
        if (!out3) return;
        if (cap < s->E.num_phr) throw lz::error(LZ77SSS_EINVAL, "output capacity too small");
        if (s->E.num_phr) LZ_HIP(hipMemcpy(out3, s->E.lpf.p, (size_t)s->E.num_phr * 12, hipMemcpyDeviceToHost));
    });
}

LZ77SSS_API int lz77sss_session_get_lpf64(lz77sss_session* s, uint64_t* out3, uint64_t cap, uint64_t* count) {
    if (!s) return LZ77SSS_EINVAL;
    return guarded([&] {
        const uint64_t m = s->E64 ? s->E64->num_phr() : s->E.num_phr;
        if (count) *count = m;
        if (!out3 || !m) return;
        if (cap < m) throw lz::error(LZ77SSS_EINVAL, "output capacity too small");
        if (s->E64) {
            LZ_HIP(hipMemcpy(out3, s->E64->lpf_ptr(), (size_t)m * 24, hipMemcpyDeviceToHost));
        } else {
            std::vector<uint32_t> tmp(3 * m);
            LZ_HIP(hipMemcpy(tmp.data(), s->E.lpf.p, (size_t)m * 12, hipMemcpyDeviceToHost));
            for (uint64_t k = 0; k < 3 * m; k++) out3[k] = tmp[k];
        }
    });
}

LZ77SSS_API int lz77sss_session_phase_times(lz77sss_session* s, double* ms, const char** names, int cap) {
    if (!s) return LZ77SSS_EINVAL;
    int k = 0;
    int rc = guarded([&] {
        static thread_local std::vector<std::string> keep;
        auto v = s->E64 ? s->E64->timer().read() : s->E.timer.read();
        keep.clear();
        for (auto& x : v) keep.push_back(x.first);
        for (auto& x : v) {
            if (k >= cap) break;
            if (ms) ms[k] = x.second;
            if (names) names[k] = keep[k].c_str();
            k++;
        }
    });
    return rc ? rc : k;
}

// device memory per phase, in the order of lz77sss_session_phase_times
LZ77SSS_API int lz77sss_session_phase_mem(lz77sss_session* s, uint64_t* held, uint64_t* peak, uint64_t* hbm_free,
                                          int cap) {
    if (!s) return LZ77SSS_EINVAL;
    const lz::phase_timer& t = s->E64 ? s->E64->timer() : s->E.timer;
    int k = 0;
    for (size_t i = 1; i < t.mem.size() && k < cap; i++, k++) {
        if (held) held[k] = t.mem[i].held;
        if (peak) peak[k] = t.mem[i].peak;
        if (hbm_free) hbm_free[k] = t.mem[i].hbm_free;
    }
    return k;
}

LZ77SSS_API int lz77sss_session_stats(lz77sss_session* s, uint64_t* out, int cap) {
    if (!s || !out) return LZ77SSS_EINVAL;
    const std::vector<uint64_t>& st = s->E64 ? s->E64->stats() : s->E.stats;
    int k = 0;
    for (; k < cap && k < (int)st.size(); k++) out[k] = st[k];
    return k;
}

LZ77SSS_API int lz77sss_session_sss_kernel_time(lz77sss_session* s, double* ms, uint64_t* bytes) {
    if (!s) return LZ77SSS_EINVAL;
    if (ms) *ms = s->E64 ? s->E64->sss_kernel_ms() : s->E.sss_ms();
    if (bytes) *bytes = s->E64 ? s->E64->sss_kernel_bytes() : s->E.sss_kernel_bytes;
    return LZ77SSS_OK;
}

LZ77SSS_API void lz77sss_session_destroy(lz77sss_session* s) {
    if (!s) return;
    s->E64.reset();
    s->E.destroy();
    delete s;
}

// ---- sharded factorization: sync set by text block + all-gather, the
// phrases on every rank, the greedy chain block by block in rank order
__global__ void k_narrow_u32(const uint64_t* __restrict__ in, uint64_t m, uint32_t* __restrict__ out) {
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k < m) out[k] = (uint32_t)in[k];
}

LZ77SSS_API int lz77sss_session_set_sss(lz77sss_session* s, const uint64_t* S, uint64_t count, int has_runs) {
    if (!s || (!S && count)) return LZ77SSS_EINVAL;
    return guarded([&] {
        if (s->E64) return s->E64->set_sss(S, count, has_runs != 0);
        lz::engine& E = s->E;
        LZ_HIP(hipSetDevice(E.device));
        if (count && E.n > 0xFFFFFFF0ull) throw lz::error(LZ77SSS_EINVAL, "n too large for pos_t = uint32_t");
        lz::u64* tmp = E.u64a.get(count + 1);
        if (count) LZ_HIP(hipMemcpyAsync(tmp, S, count * 8, hipMemcpyDefault, E.st));
        lz::u32* narrow = E.u32e.get(count + 1);
        if (count) k_narrow_u32<<<lz::cdiv(count, 256), 256, 0, E.st>>>(tmp, count, narrow);
        LZ_HIP(hipStreamSynchronize(E.st));
        E.set_sss(narrow, count, has_runs != 0);
    });
}

LZ77SSS_API int lz77sss_session_prepare(lz77sss_session* s, const lz77sss_params* prm, int external_sss,
                                        uint64_t* carried_bytes) {
    if (!s) return LZ77SSS_EINVAL;
    return guarded([&] {
        check_params(prm);
        const uint64_t b = s->E64 ? s->E64->prepare(prm->phr_mode, external_sss != 0, prm->index_log2_size)
                                  : lz::block_prepare(s->E, prm->phr_mode, external_sss != 0, prm->index_log2_size);
        if (carried_bytes) *carried_bytes = b;
    });
}

LZ77SSS_API int lz77sss_session_carried_copy(lz77sss_session* s, void* buf, uint64_t bytes, int to_session) {
    if (!s || (!buf && bytes)) return LZ77SSS_EINVAL;
    return guarded([&] {
        void* tab = s->E64 ? s->E64->carried_table() : (void*)s->E.g_Hs.p;
        const uint64_t cap = s->E64 ? s->E64->carried_bytes() : s->E.g_Hs.cap * sizeof(lz::pos_t);
        if (!tab) throw lz::error(LZ77SSS_EINVAL, "no carried table: call lz77sss_session_prepare first");
        if (bytes > cap) throw lz::error(LZ77SSS_EINVAL, "carried table smaller than the copy");
        const int dev = s->E64 ? s->E64->device() : s->E.device;
        hipStream_t st = s->E64 ? s->E64->stream() : s->E.st;
        LZ_HIP(hipSetDevice(dev));
        if (bytes) {
            if (to_session) LZ_HIP(hipMemcpyAsync(tab, buf, bytes, hipMemcpyDefault, st));
            else LZ_HIP(hipMemcpyAsync(buf, tab, bytes, hipMemcpyDefault, st));
        }
        LZ_HIP(hipStreamSynchronize(st));
    });
}

LZ77SSS_API int lz77sss_session_greedy_block(lz77sss_session* s, const lz77sss_params* prm, lz77sss_block* blk,
                                             uint64_t* num_factors) {
    if (!s || !blk) return LZ77SSS_EINVAL;
    return guarded([&] {
        check_params(prm);
        // reserved = 1: seed the table from the gap positions before start (a speculative lead-in)
        uint64_t st[8] = {blk->start, blk->idxpos, blk->zmask,
                          (uint64_t)(blk->carried != 0) | (blk->reserved == 1 && !blk->carried ? 2u : 0u), blk->end, 0,
                          0, 0};
        const uint64_t z = s->E64 ? s->E64->greedy_block(prm->rk_seed, prm->index_log2_size, st)
                                  : lz::block_run(s->E, prm->rk_seed, prm->index_log2_size, st);
        blk->exit_start = st[5];
        blk->exit_idxpos = st[6];
        blk->exit_zmask = (uint32_t)st[7];
        if (num_factors) *num_factors = z;
    });
}

LZ77SSS_API int lz77sss_session_spec_begin(lz77sss_session* s, int part, uint64_t block_start) {
    if (!s || part < 0 || part >= LZ77SSS_SPEC_MAX_PARTS) return LZ77SSS_EINVAL;
    return guarded([&] {
        if (s->E64) s->E64->spec_begin(part, block_start);
        else s->E.spec_begin(part, block_start);
    });
}

LZ77SSS_API int lz77sss_session_spec_resolve(lz77sss_session* s, const void* true_table, uint64_t bytes, int parts,
                                             int* accepted_parts) {
    if (!s || !true_table || !accepted_parts || parts < 0 || parts > LZ77SSS_SPEC_MAX_PARTS) return LZ77SSS_EINVAL;
    return guarded([&] {
        *accepted_parts = s->E64 ? s->E64->spec_resolve(true_table, bytes, parts)
                                 : s->E.spec_resolve(true_table, bytes, parts);
    });
}

}  // extern "C"
// one-shot: upload, factorize, stream the factors to the callback in text order
template <class FACT, class EMIT>
static int one_shot(const uint8_t* text, uint64_t n, const lz77sss_params* prm, EMIT emit, void* user, bool wide,
                    bool exact, int transf_mode) {
    if ((!text && n) || !emit) return LZ77SSS_EINVAL;
    lz77sss_session* s = nullptr;
    int rc = guarded([&] {
        if (exact) check_exact_params(prm, transf_mode);
        else check_params(prm);
    });
    if (rc) return rc;
    rc = (wide && !exact) ? lz77sss_session_create64(prm->device, n, &s) : lz77sss_session_create(prm->device, n, &s);
    if (rc) return rc;
    rc = lz77sss_session_load(s, text, n);
    uint64_t z = 0;
    if (!rc) rc = exact ? lz77sss_session_factorize_exact(s, prm, transf_mode, &z) : lz77sss_session_factorize(s, prm, &z);
    if (!rc && z) {
        std::vector<FACT> buf;
        rc = guarded([&] { buf.resize(z); });
        if (!rc) {
            if constexpr (sizeof(FACT) == 16) rc = lz77sss_session_get_factors64(s, buf.data(), z);
            else rc = lz77sss_session_get_factors(s, buf.data(), z);
        }
        const uint64_t B = 1 << 16;
        for (uint64_t o = 0; !rc && o < z; o += B) {
            if (emit(buf.data() + o, std::min(B, z - o), user) != 0) {
                g_err = "emit callback aborted";
                rc = LZ77SSS_ECALLBACK;
            }
        }
    }
    lz77sss_session_destroy(s);
    return rc;
}

extern "C" {
LZ77SSS_API int lz77sss_factorize_approx_u32(const uint8_t* text, uint64_t n, const lz77sss_params* prm,
                                             lz77sss_emit_fn emit, void* user) {
    return one_shot<lz77sss_factor32>(text, n, prm, emit, user, false, false, 0);
}

LZ77SSS_API int lz77sss_factorize_approx_u64(const uint8_t* text, uint64_t n, const lz77sss_params* prm,
                                             lz77sss_emit64_fn emit, void* user) {
    return one_shot<lz77sss_factor64>(text, n, prm, emit, user, true, false, 0);
}

LZ77SSS_API int lz77sss_factorize_exact_u32(const uint8_t* text, uint64_t n, const lz77sss_params* prm,
                                            int transf_mode, lz77sss_emit_fn emit, void* user) {
    return one_shot<lz77sss_factor32>(text, n, prm, emit, user, false, true, transf_mode);
}

LZ77SSS_API int lz77sss_factorize_exact_u64(const uint8_t* text, uint64_t n, const lz77sss_params* prm,
                                            int transf_mode, lz77sss_emit64_fn emit, void* user) {
    return one_shot<lz77sss_factor64>(text, n, prm, emit, user, true, true, transf_mode);
}

// decode on a device: upload, pointer-jumping decode (csrc/decode.hip), download
LZ77SSS_API int lz77sss_decode_u32_device(const lz77sss_factor32* f, uint64_t nf, uint8_t* out, uint64_t n,
                                          int device) {
    if ((!f && nf) || (!out && n)) return LZ77SSS_EINVAL;
    lz77sss_session* s = nullptr;
    int rc = lz77sss_session_create(device, n, &s);
    if (rc) return rc;
    rc = guarded([&] {
        lz::engine& E = s->E;
        lz::u32* F = E.fact.get(2 * nf + 2);
        if (nf) LZ_HIP(hipMemcpyAsync(F, f, nf * sizeof(lz77sss_factor32), hipMemcpyHostToDevice, E.st));
        lz::u8* d_out = n ? E.dec_out.get(n) : nullptr;
        E.decode_device(F, nf, n, d_out, nullptr);
        if (n) LZ_HIP(hipMemcpyAsync(out, d_out, n, hipMemcpyDeviceToHost, E.st));
        LZ_HIP(hipStreamSynchronize(E.st));
    });
    lz77sss_session_destroy(s);
    return rc;
}

LZ77SSS_API int lz77sss_decode_u64_device(const lz77sss_factor64* f, uint64_t nf, uint8_t* out, uint64_t n,
                                          int device) {
    if ((!f && nf) || (!out && n)) return LZ77SSS_EINVAL;
    lz77sss_session* s = nullptr;
    int rc = lz77sss_session_create64(device, n, &s);
    if (rc) return rc;
    rc = guarded([&] {
        lz::engine_if& E = *s->E64;
        lz::u64* F = E.factors_buf(nf);
        if (nf) LZ_HIP(hipMemcpyAsync(F, f, nf * sizeof(lz77sss_factor64), hipMemcpyHostToDevice, E.stream()));
        lz::u8* d_out = n ? E.dec_out(n) : nullptr;
        E.decode(F, nf, n, d_out, false);
        if (n) LZ_HIP(hipMemcpyAsync(out, d_out, n, hipMemcpyDeviceToHost, E.stream()));
        LZ_HIP(hipStreamSynchronize(E.stream()));
    });
    lz77sss_session_destroy(s);
    return rc;
}

}  // extern "C"
// decode: algorithms/common.cpp:31-54 (sequential; forward byte copy allows overlap)
template <class FACT>
static int host_decode(const FACT* f, uint64_t nf, uint8_t* out, uint64_t n) {
    if ((!f && nf) || (!out && n)) return LZ77SSS_EINVAL;
    uint64_t pos = 0, k = 0;
    while (pos < n && k < nf) {
        const FACT x = f[k++];
        if (x.len == 0) {
            out[pos++] = (uint8_t)x.src;
        } else {
            if ((uint64_t)x.src >= pos || x.len > n - pos) {
                g_err = "invalid factor during decode";
                return LZ77SSS_EINVAL;
            }
            for (uint64_t i = 0; i < x.len; i++) out[pos + i] = out[x.src + i];
            pos += x.len;
        }
    }
    if (pos != n) {
        g_err = "factors do not cover the output length";
        return LZ77SSS_EINVAL;
    }
    return LZ77SSS_OK;
}

extern "C" {
LZ77SSS_API int lz77sss_decode_u32(const lz77sss_factor32* f, uint64_t nf, uint8_t* out, uint64_t n) {
    return host_decode(f, nf, out, n);
}

LZ77SSS_API int lz77sss_decode_u64(const lz77sss_factor64* f, uint64_t nf, uint8_t* out, uint64_t n) {
    return host_decode(f, nf, out, n);
}

}  // extern "C"
#endif  // LZ_POS64
