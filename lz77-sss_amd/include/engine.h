// engine.h -- the device-resident LZ77-SSS engine (one per session / GPU).
// Data layout in HBM is documented in DESIGN.md section 5.
#pragma once
#include <initializer_list>
#include "../../include/lz77sss.h"
#include "lz77sss_internal.h"
#include "lce_dev.h"
#include "timer.h"

#include <array>
#include <cstdlib>
#include <cstring>
#include <string>
#include <utility>
#include <vector>

namespace LZ_NS {

struct lpf3 { pos_t beg, end, src; };
struct smpl_view;  // csrc/smpl.hip

// greedy walk segments (csrc/greedy.hip)
// walk segment input: start position, first phrase index, gap-index state, and
// the position at or after which the gap walk stops (a chunk boundary; n = none)
struct seg_in { pos_t start; u32 p; pos_t idxpos; u32 zmask; pos_t lim; };
constexpr int SEG_NBND = 16;  // factor starts recorded per gap walk (chunk convergence)
struct seg_out {
    pos_t next;      // start of the next gap (or n)
    pos_t e;         // end of this segment's gap walk (positions [start, e) inserted)
    u32 nfact;
    pos_t idxpos;    // gap index position after the segment
    u32 zmask;
    u32 nsingle;     // extra inserted positions (LPF-start queries)
    pos_t single[4];
    u32 flags;       // 1: reached the tail region, 2: single overflow
    u32 nbnd;        // recorded factor starts of the first gap walk
    pos_t bnd[SEG_NBND];
};

// the greedy chain over a text block [start, end) (csrc/greedy.hip): the
// exact chain state at start in, the state at the first hand-over point >= end out; the
// carried table (g_Hs: last insert per slot before the block, pos + 1) in and out
struct greedy_block {
    pos_t start = 0, idxpos = 0;
    u32 zmask = 0;
    bool carried = false;  // g_Hs holds the inserts before start (else it is zeroed)
    bool seed = false;     // (not carried) seed g_Hs from the gap positions before start (a lead-in)
    pos_t end = 0;
    pos_t exit_start = 0, exit_idxpos = 0;
    u32 exit_zmask = 0;
};

struct engine {
    int device = 0;
    hipStream_t st = nullptr;
    u64 max_n = 0, n = 0;
    u8* d_text = nullptr;  // n + TEXT_PAD bytes (zero padded)
    u8* d_text_rev = nullptr;  // reversed copy for LPF/LNF modes (lazily allocated)

    // ---- string synchronizing set ----
    dbuf<u16> q_info;          // per anchor: Q interval (start<<8 | end) of (a-128, a]
    dbuf<pos_t> lane_out;      // per-stripe sync positions (k_sss_stream)
    dbuf<u32> lane_cnt, lane_flag;
    dbuf<pos_t> sss_ovf;       // fallback outputs
    dbuf<pos_t> S;             // sync positions (sorted)
    dbuf<u32> counters;        // small scratch counters
    u32 s = 0;
    bool has_runs = false;
    // dominant kernel (SSS phase) duration: HIP events recorded around the phase's kernels, read
    // when asked (sss_ms), so the phase needs no synchronization of its own for them
    // Two windows: pass 1 .. k_sss_runs, and after the phase's one host read the rest through the
    // compaction (the read's round trip is not kernel time)
    mutable double sss_kernel_ms = 0;
    hipEvent_t sss_ev0 = nullptr, sss_ev1 = nullptr, sss_evA = nullptr, sss_evB = nullptr;
    mutable bool sss_ev_pending = false;
    double sss_ms() const {
        if (sss_ev_pending) {
            float a = 0, b = 0;
            LZ_HIP(hipEventSynchronize(sss_ev1));
            LZ_HIP(hipEventElapsedTime(&a, sss_ev0, sss_evA));
            LZ_HIP(hipEventElapsedTime(&b, sss_evB, sss_ev1));
            sss_kernel_ms = (double)a + (double)b;
            sss_ev_pending = false;
        }
        return sss_kernel_ms;
    }
    u64 sss_kernel_bytes = 0;  // its algorithmic bytes (text + 4|S|) per launch
    u64 stats_fallback_lanes = 0;
    dbuf<u8> run_p;            // periodic-run table per Q anchor (lce_dev.h run_tab)
    dbuf<pos_t> run_hi, run_lo;
    dbuf<u64> run_scan_a, run_scan_b;
    bool runs_valid = false;
    // pos_t = uint64_t sync set of a decision range (build_sss_range): any n, windowed
    dbuf<u64> S64;
    u64 s64 = 0;
    bool has_runs64 = false;
    u64 stats_sss_windows = 0;
    // filter pass of build_sss: hit words per stripe, marked tiles, re-run stripes
    dbuf<u64> sss_hitw;
    dbuf<u8> sss_tflag;
    dbuf<u32> sss_tiles, sss_sflag, sss_slist, sss_fcnt;
    u64 stats_sss_tiles = 0;
    // per-block run records (lce_dev.h run_tab::bp / ser / ss): the period of every
    // p-extendable 512-byte block (k_sss_runs), segment ends / starts by two scans
    dbuf<u8> blk_p;
    dbuf<u16> blk_fo, blk_lo;
    dbuf<pos_t> blk_mk, blk_ser, blk_ss;
    dbuf<u32> sss_tot;  // |S| partial sums of the stripe kernels (csrc/sss.hip)
    dbuf<u64> blk_re, blk_rs;  // packed per-block run end / start (lce_dev.h run_tab::re / rs)
    u64 brk_nbk = 0;
    bool brk_valid = false;
    bool no_blkrec = std::getenv("LZ77SSS_NO_BLKREC") != nullptr;  // test knob: LCE without the block records
    unsigned long long* lce_dbg = nullptr;  // LZ77SSS_LCE_DEBUG: device counters of dev_lce_fwd / bwd
    run_tab runs() const {
        run_tab R;
        if (runs_valid) { R.p = run_p.p; R.hi = run_hi.p; R.lo = run_lo.p; }
        if (brk_valid && !no_blkrec) {
            R.re = blk_re.p;
            R.rs = blk_rs.p;
            R.nbk = brk_nbk;
        }
        R.dbg = lce_dbg;
        return R;
    }

    // ---- suffix order of sync positions / LCE ----
    dbuf<u32> SA, ISA, LCP;
    dbuf<pos_t> key_len;
    dbuf<u32> rank_lv[MAX_LV];       // R_h per doubling level (for LCP binary lifting)
    dbuf<u32> lcp_rmq[MAX_LV];       // sparse table levels over LCP
    u32 nlev_rank = 0, nlev_rmq = 0;
    u32 rank_step = 2;  // SA_S prefix doubling: ranks per radix key (level lv spans rank_step^lv)
    dbuf<u32> succ_tab;              // bucket -> first sync index with S >= bucket*512
    dbuf<u8> tmp_bytes, tmp_bytes2, tmp_bytes3, scan_tmp;
    dbuf<u64> u64a, u64b;
    dbuf<u32> sa_tmp1, sa_tmp2, sa_tmp3;
    u64 stats_sa_distinct = 0, stats_sa_ties = 0;
    dbuf<u32> u32a, u32b, u32c, u32d, u32e;

    // ---- LPF phrases ----
    dbuf<u32> sa_min[MAX_LV];        // sparse table over SA (PSV/NSV)
    dbuf<u32> jump[MAX_LV];          // pointer-doubling tables (skip chain)
    dbuf<u32> PSV, NSV;
    dbuf<pos_t> cand;                // per sync index candidate data
    dbuf<pos_t> p_Em, p_lst, p_ph3;  // running max_end scan and phrase scratch (csrc/lpf.hip)
    dbuf<pos_t> lpf;                 // phrases as (beg,end,src) triples + sentinel
    u32 num_phr = 0;
    // the emitter's phrase statistics (total phrase length, gaps), when the phrase builder already
    // computed them and wrote the sentinel (build_lpf_opt); any other phrase source clears it
    struct { bool valid; u64 len, gaps; } phr_info{false, 0, 0};

    // ---- greedy ----
    dbuf<pos_t> fact;                // output factors (src,len) pairs
    dbuf<u8> tmp_greedy, chunk_buf, chunk_buf2, rem_buf;
    dbuf<u32> add_keys32;
    dbuf<pos_t> add_pos, dirty_in, dirty_out, dirty_sorted;
    dbuf<u8> tmp_greedy2, tmp_greedy3;
    dbuf<u64> add_keys, add_keys2;
    dbuf<seg_in> seg_in_buf;
    dbuf<seg_out> seg_out_buf;
    dbuf<u32> seg_ids, irank, ekeys, evals, ekeys2, evals2, occ_buf;
    dbuf<pos_t> ist, iend, ipos_buf, iposr_buf, tail_ins_buf;
    dbuf<u64> seg_offs, counters64;
    // device-resident greedy orchestration (csrc/greedy.hip)
    dbuf<seg_in> g_sin;
    dbuf<seg_out> g_sout;
    dbuf<u8> g_valid, g_cs, g_tailc;
    bool seg_at_clean = false;  // g_seg_at is all NONE
    u64 seg_at_n = 0;
    dbuf<u32> g_succ, g_seg_at, g_ids, g_chain, g_dist[2];
    dbuf<pos_t> g_cbv;
    dbuf<u32> g_bmI, g_bmI2, g_bmIb, g_bmT;
    dbuf<u32> g_tmp1, g_tmp2, g_tmp3, g_tmp4, g_tmp5, g_tmp6, g_tmp7, g_tmp8, g_ark;
    dbuf<pos_t> g_ast, g_aen;
    dbuf<u64> g_offs;
    // LPF/LNF mode (csrc/lnf.hip)
    dbuf<u32> l_V, l_V2, l_X, l_coff, l_r, l_sflag_lnf, l_sflag, l_off;
    dbuf<pos_t> l_b, l_d, l_e, l_slots_lnf, l_slots, l_P, l_Q;
    dbuf<u64> l_tmp64;
    dbuf<u32> g_predk, g_wk, g_ids2;
    dbuf<u32> g_brev;
    dbuf<u64> g_bsum, g_bincl, g_pbtmp;
    dbuf<u32> g_pbcur;  // predecessor bucket scatter
    dbuf<u32> g_pbm, g_pwp, g_pcnt, g_sdk, g_dstart, g_pflag;  // dense slot ids of the base set  // per-block bitmap counts and their inclusive scan
    dbuf<u32> g_bstart, g_abeg, g_abeg2, g_bmA, g_x32;
    dbuf<pos_t> g_xpos;
    dbuf<pos_t> g_stash;  // per segment: factors of its last speculative walk (csrc/greedy.hip STASH_CAP)
    std::array<u64, 10> negpow_key{};  // (bases, pattern lengths) of the influence tables in tmp_greedy
    const void* negpow_dev = nullptr;
    dbuf<pos_t> g_H;    // materialized gap-index table of the sequential completion
    dbuf<pos_t> g_Hs;   // greedy windows: last insert per slot before the window (pos + 1)
    // speculative blocks of a sharded run, walked as consecutive parts: the
    // table each part started from (part 0: the speculated entry table), per part the
    // entry-table slots its lookups used, the true entry table when it arrives
    bool spec_track = false;
    int spec_part = 0;
    u64 spec_base = 0, spec_m = 0;  // block start; table slots
    dbuf<u32> g_hsused;
    dbuf<pos_t> g_hsave, g_htrue;
    dbuf<u32> g_specbad;
    void spec_begin(int part, u64 base);
    int spec_resolve(const void* true_tab, u64 bytes, int parts);
    dbuf<pos_t> fact_acc;  // greedy windows: the stream so far
    dbuf<u8> g_cut;     // chain_cut + completion counters
    dbuf<u64> g_xk, g_xk2;
    dbuf<u32> g_ls_h, g_ls_g;  // LSD base sort: digit counts per tile and their scans (csrc/greedy.hip)
    dbuf<u32> g_lng;           // long chain ranges for k_chain_inserts_long
    dbuf<u32> g_pbw;           // presence words with their ranks, packed (the LSD sort's dense-id map)
    // exact mode (csrc/exact.hip)
    dbuf<u64> x_key, x_key2, x_off, x_wide;
    dbuf<u32> x_idx, x_idx2, x_sa, x_rank, x_flag, x_tree, x_ltree, x_lcp, x_lpf, x_src, x_mark, x_chunk;
    const u32* sa_full = nullptr;    // suffix array of the text (x_sa) after build_sa_full
    u32 x_rounds = 0;
    // exact-smpl mode (csrc/smpl.hip): approximate factors, samples, PA / SA, grid, RKS,
    // exact-smpl (csrc/smpl.hip): samples, PA / SA orders, grid, phrase tasks
    dbuf<u32> e_afact, e_afst, e_tmp1, e_tmp2, e_C, e_PA, e_SA, e_PAR, e_SAR, e_Pi, e_Psi, e_CS;
    dbuf<u32> e_alpha;  // exact-smpl: the character codes of the sort keys and the text's character flags
    dbuf<u32> e_preL, e_preR, e_wblk;  // exact-smpl: first ranks per 16-bit key prefix (PA, SA); first sample per 256-block
    dbuf<u64> e_cyc;  // exact-smpl debug counters (LZ77SSS_SMPL_PROF)
    dbuf<u32> e_gx, e_gy, e_gw, e_cell, e_adjL, e_adjR;
    dbuf<u32> e_rst[18];  // exact-smpl: row sparse tables of the grid cells' lightest weights
    // exact-smpl source pass: the reference's grid (16384-rank windows), the phrase starts, the
    // sampled left pattern lengths of with_samples
    dbuf<u32> e_CS2, e_gx2, e_gy2, e_gw2, e_cell2, e_fpos, e_vis, e_twk, e_fwk;
    dbuf<u32> e_rst2[18];
    dbuf<u32> e_ivmin[MAX_LV], e_ivminL[MAX_LV];  // sparse-table minima of the SA / PA adjacent LCEs (interval ends)
    dbuf<u64> e_kSA, e_kPA;                      // 16-byte context keys by SA / PA rank
    dbuf<u32> e_wPA[MAX_LV], e_wSA[MAX_LV];      // minima of the PA / SA weights per sparse-table level
    dbuf<u32> e_tpos, e_tlen, e_tsrc, e_thop, e_tkeys, e_tvals;
    dbuf<u64> e_key, e_key2, e_key3;
    // device decode (csrc/decode.hip)
    dbuf<u32> dec_fid, dec_fid2;
    dbuf<pos_t> dec_ref, dec_ref2;
    dbuf<u64> dec_len64, dec_start64;
    dbuf<u8> dec_out;
    u32 dec_rounds = 0;
    u64 num_fact = 0;
    int last_fact_mode = -1;  // fact_mode of the last factorize call (-1: none yet)
    // lz77sss_session_verify checks the factors in HBM against the text in HBM: a factorization must
    // exist and be one (a skip_phrases stream is not).  Loading another text keeps the factors, so
    // the check then reports where they do not reproduce it (tests corrupt the text this way)
    void check_verifiable() const {
        if (last_fact_mode == -1) throw error(LZ77SSS_EINVAL, "no factorization in the session to verify");
        if (last_fact_mode == LZ77SSS_SKIP_PHRASES)
            throw error(LZ77SSS_EINVAL, "a skip_phrases stream is not a factorization (nothing to verify)");
    }
    dbuf<u8> ssz_out;         // ssszip gapped container (csrc/ssszip.hip)
    dbuf<u8> hf_tabs, hf_words, hf_out;  // Huffman factor container (csrc/huffman.hip)
    u64 ssz_size = 0;
    std::vector<u64> stats;

    phase_timer timer;

    // pinned read-back slots (64 x u32; sa_s uses the first, build_sss 32..) + events
    u32* h_pin = nullptr;
    hipEvent_t ev_pin[2] = {nullptr, nullptr};

    // several buffer fills in one launch (k_fills, csrc/engine.hip): a rocclr fill costs about 5 us
    // of launch and gap however small the buffer, and a call has tens of them.  A fill writes the
    // 32-bit pattern `pat` over `bytes` bytes (a byte value v: pat = v * 0x01010101; 16-bit
    // patterns repeat in both halves); at most FILL_MAX per launch, in any order (they must not
    // overlap)
    struct fill_op { void* p; u64 bytes; u32 pat; };
    static constexpr int FILL_MAX = 8;
    void fills(std::initializer_list<fill_op> ops);
    void init(int dev, u64 maxn);
    void load(const u8* h_text, u64 n_);
    void destroy();

    // pipeline phases (each enqueues on `st`)
    void build_sss(const u8* T);
    bool build_q_runs(const u8* T);     // Q anchors + periodic-run table only
    void run_chains(u64 nanch, const u32* tiles, u64 m);  // exact run ends along anchor chains
    void set_sss(const pos_t* S_any, u64 count, bool runs);  // an externally built (sharded) sync set
    void build_sss_range(u64 first, u64 end, u64 base, u64 window);  // csrc/sss.hip
    void build_sa_s(const u8* T);
    void build_lcp_rmq(const u8* T);
    void build_lpf_opt(const u8* T);
    void build_lpf_naive(const u8* T);  // lpf_naive mode (csrc/lpf.hip)
    void psv_nsv_s();
    void mark_path(u32* mark);
    void build_lpf_lnf(int opt);  // csrc/lnf.hip
    void all_phrases(const u8* T, int lnf, int opt, u64 slot_base, pos_t* slots, u32* sflag);
    void path_marks(u32 m, u32* nxt0, u32* marks);
    u64 factorize_greedy(const u8* T, u32 rk_seed, int log2_override, greedy_block* blk = nullptr);
    u64 factorize(int phr_mode, u32 rk_seed, int log2_override, bool log, int fact_mode = 1);
    void log_summary(std::chrono::steady_clock::time_point t_start) const;  // lz77_sss.hpp:345-353
    void prepare_phrases(int phr_mode, bool external_sss);  // the phases before the emitter
    void release_phase_scratch();                           // (large texts, LZ77SSS_LEAN: engine.hip)
    void release_greedy_buffers();
    bool lean = false;  // this call releases scratch as it goes (prepare_phrases)
    u64 stats_released_scratch = 0;
    u64 carried_entries(int log2_override);                 // slots of the gap index (carried table size)
    u64 emit_skip_phrases();  // fact_mode = skip_phrases (csrc/engine.hip)
    u64 ssszip_gapped();      // csrc/ssszip.hip
    u64 huffman_container();  // csrc/huffman.hip
    void build_sa_full(const u8* T);
    u64 factorize_exact(bool log);  // csrc/exact.hip (full suffix array, LZ77SSS_TRANSF_FULL_SA)
    u64 factorize_exact_smpl(int transf_mode, int phr_mode, u32 rk_seed, int log2_override, bool log);  // csrc/smpl.hip
    void build_adjacent(smpl_view& V);                                                                 // csrc/smpl.hip
    u64 decode_device(const pos_t* F, u64 nf, u64 n_out, u8* out, const u8* cmp);
    u64 verify_factors(const pos_t* F, u64 nf, u64 n_out, const u8* T, u64* first_bad = nullptr);  // csrc/decode.hip
    void debug_verify_phrases(const char* what);  // LZ77SSS_DEBUG_VERIFY (csrc/decode.hip)
    void debug_verify_lce(const char* what);
    lce_view view(const u8* T) const;
};

// small host helpers: device values the host needs (counts, sizes, states).  A read-back is a
// round trip the whole pipeline waits on, so it is made as short as the hardware allows: one tiny
// kernel copies every requested value into host-coherent pinned memory (mapped into the device
// address space) and then writes a sequence number there; the host spins on that word.  Against
// hipMemcpyAsync per value + hipStreamSynchronize this saves a copy launch per value and the
// runtime's wait-and-wake (LZ77SSS_NO_SPIN selects the copy + synchronize form for A/B runs).
struct sync_slot {
    u8* h = nullptr;  // host pointer (fine-grained, coherent)
    u8* d = nullptr;  // the same memory as the device sees it
    u32 seq = 0;
    bool spin = std::getenv("LZ77SSS_NO_SPIN") == nullptr;
    sync_slot() {
        if (hipHostMalloc((void**)&h, 8192, hipHostMallocMapped | hipHostMallocPortable | hipHostMallocCoherent) != hipSuccess) {
            h = nullptr;
            return;
        }
        if (hipHostGetDevicePointer((void**)&d, h, 0) != hipSuccess) d = h;
        std::memset(h, 0, 8192);
    }
    ~sync_slot() {
        if (h) (void)hipHostFree(h);
    }
};
// (a slot whose pinned allocation failed has h == nullptr: hread then uses the copy +
// synchronize form instead of failing every entry point)
inline sync_slot& host_slot() {
    static thread_local sync_slot s;
    return s;
}
struct hread_job {
    const u8* src[16];
    u32 off[16], bytes[16];
    u32 n, seq;
};
// copies the requested values into the slot as 8-byte words (sequence number << 32 | 4 value
// bytes): a word is complete when the host sees its sequence number, so no fence orders the
// payload before a flag (a system-scope fence writes back the whole L2 first: 60 us after the
// bitmap fills of the greedy setup)
static __global__ __launch_bounds__(64) void k_hread(hread_job J, u64* __restrict__ dst) {
    if (J.n == 0 && threadIdx.x == 0)  // a plain wait: one word
        __hip_atomic_store(&dst[0], (u64)J.seq << 32, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    for (u32 i = 0; i < J.n; i++) {
        const u32* src = (const u32*)J.src[i];
        for (u32 w = threadIdx.x; w < J.bytes[i] / 4; w += 64)
            __hip_atomic_store(&dst[J.off[i] / 4 + w], ((u64)J.seq << 32) | src[w], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}
// waits until the nw words from word w0 carry sequence number seq (the stream's error state is
// checked while spinning), then unpacks them into out
inline void spin_wait(sync_slot& S, u32 seq, u64 w0, u64 nw, u32* out, hipStream_t st) {
    volatile u64* W = (volatile u64*)S.h + w0;
    u64 done = 0;
    for (u64 it = 1;; it++) {
        while (done < nw) {
            const u64 v = W[done];
            if ((u32)(v >> 32) != seq) break;
            out[done++] = (u32)v;
        }
        if (done == nw) return;
        if ((it & 255) == 0) {
            const hipError_t e = hipStreamQuery(st);
            if (e == hipSuccess) {
                for (; done < nw; done++) {
                    const u64 v = W[done];
                    if ((u32)(v >> 32) != seq) throw error(-6 /* LZ77SSS_EINTERNAL */, "read-back: stream idle but a value never arrived");
                    out[done] = (u32)v;
                }
                return;
            }
            if (e != hipErrorNotReady) LZ_HIP(e);
        }
        __builtin_ia32_pause();
    }
}
// several device values of any small types with one round trip: add() records, sync() copies
// them all (the values as of sync(): nothing enqueued between may change them) and waits
struct hread {
    hipStream_t st;
    sync_slot& S;
    size_t off = 0;  // payload bytes so far (4 per 8-byte slot word)
    struct item { void* dst; const void* src; size_t off, bytes; };
    item items[16];
    int n = 0;
    u32 tmp[1024];
    explicit hread(hipStream_t s) : st(s), S(host_slot()) {}
    template <class T>
    void add(T* dst, const T* src, size_t count = 1) {
        static_assert(sizeof(T) % 4 == 0, "read-back values are whole 4-byte words");
        const size_t b = sizeof(T) * count;
        if (off + b > 4 * 1024 || n == 16) throw error(-6 /* LZ77SSS_EINTERNAL */, "hread: staging slot full");
        items[n++] = {dst, src, off, b};
        off += b;
    }
    void sync() {
        if (S.spin && S.h) {
            hread_job J{};
            for (int k = 0; k < n; k++) {
                J.src[k] = (const u8*)items[k].src;
                J.off[k] = (u32)items[k].off;
                J.bytes[k] = (u32)items[k].bytes;
            }
            J.n = (u32)n;
            J.seq = ++S.seq;
            if (J.seq == 0) J.seq = S.seq = 1;  // (0: the slot's initial contents)
            k_hread<<<1, 64, 0, st>>>(J, (u64*)S.d);
            LZ_HIP(hipGetLastError());
            spin_wait(S, J.seq, 0, n ? off / 4 : 1, tmp, st);
        } else {
            for (int k = 0; k < n; k++)
                LZ_HIP(hipMemcpyAsync((u8*)tmp + items[k].off, items[k].src, items[k].bytes, hipMemcpyDeviceToHost, st));
            LZ_HIP(hipStreamSynchronize(st));
        }
        for (int k = 0; k < n; k++) std::memcpy(items[k].dst, (const u8*)tmp + items[k].off, items[k].bytes);
        n = 0;
        off = 0;
    }
};
template <class T>
static inline T rd1(const T* dptr, hipStream_t st) {
    T v;
    hread rb(st);
    rb.add(&v, dptr);
    rb.sync();
    return v;
}
// two device values with one synchronization
template <class T>
static inline std::pair<T, T> rd2(const T* a, const T* b, hipStream_t st) {
    T v[2];
    hread rb(st);
    rb.add(&v[0], a);
    rb.add(&v[1], b);
    rb.sync();
    return {v[0], v[1]};
}
// everything enqueued on st so far has completed (the spin form of hipStreamSynchronize)
inline void stream_wait(hipStream_t st) {
    hread rb(st);
    rb.sync();
}
static inline unsigned cdiv(u64 a, u64 b) { return (unsigned)((a + b - 1) / b); }
// blocks of a grid-stride launch over `items` work-items (at least 1, at most GRID_CAP)
static inline unsigned capped_grid(u64 items, u64 threads) {
    return (unsigned)std::min<u64>(std::max<u64>((items + threads - 1) / threads, 1), GRID_CAP);
}

}  // namespace LZ_NS
