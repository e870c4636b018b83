/*
 * lz77sss.h -- C-ABI of liblz77sss_hip.so, the MI355X-native LZ77-SSS engine.
 *
 * This is the drop-in boundary for the reference's approximate-factorization
 * path.  Each entry point names the reference interface it replaces
 * (paths relative to LukasNalbach/lz77-sss):
 *
 *   lz77sss_factorize_approx_u32  <- lz77_sss<uint32_t>::factorize_approximate
 *                                    <fact_mode, phr_mode, tau>(input, n, output, params)
 *                                    include/lz77_sss/lz77_sss.hpp:176-186
 *   lz77sss_factorize_approx_u64  <- lz77_sss<uint64_t>::factorize_approximate (same lines;
 *                                    pos_t = uint64_t per lz77_sss.hpp:72-75, selected by the CLI
 *                                    for n > 2^32 - 1, cli/lz77_sss_3_aprx.cpp:73-83)
 *   lz77sss_factorize_exact_u32   <- lz77_sss<uint32_t>::factorize_exact
 *                                    <fact_mode, phr_mode, transf_mode, range_ds_t, tau>(input, n, output, params)
 *                                    include/lz77_sss/lz77_sss.hpp:188-200,333-357
 *   lz77sss_decode_u32            <- lz77_sss<uint32_t>::decode(fact_it, out_it, n)
 *                                    include/lz77_sss/lz77_sss.hpp:202-203,
 *                                    include/lz77_sss/algorithms/common.cpp:31-54
 *   lz77sss_factorize_exact_u64,
 *   lz77sss_decode_u64            <- the same with pos_t = uint64_t
 *   lz77sss_factor32              <- lz77_sss<uint32_t>::factor {src, len}
 *                                    include/lz77_sss/lz77_sss.hpp:129-147 (8-byte layout;
 *                                    literal <=> len == 0, src = (uint8_t)char)
 *   lz77sss_factor64              <- lz77_sss<uint64_t>::factor {src, len} (in memory; its
 *                                    10-byte stream form, lz77_sss.hpp:149-173, is written by
 *                                    lz77sss_serialize_factors64)
 *   lz77sss_params                <- struct parameters {num_threads, log}
 *                                    include/lz77_sss/lz77_sss.hpp:67-70, plus the knobs the
 *                                    reference leaves to std::random_device / malloc_count
 *
 * The session API keeps the text resident in HBM (bench / repeated calls);
 * the one-shot API uploads, factorizes and streams factors to a callback in
 * text order, batched, on the calling thread (the reference calls `output`
 * once per factor on the calling thread: greedy.cpp:91,127).
 *
 * Errors: every function returns 0 on success or a negative LZ77SSS_E* code
 * and never throws across the ABI; lz77sss_last_error() gives a message.
 * There is no CPU fallback: without a usable gfx950 device every compute
 * entry point fails with LZ77SSS_ENODEV.
 */
#ifndef LZ77SSS_H
#define LZ77SSS_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* enum phrase_mode, lz77_sss.hpp:48-53 (same numeric values) */
enum { LZ77SSS_LPF_NAIVE = 0, LZ77SSS_LPF_LNF_NAIVE = 1, LZ77SSS_LPF_OPT = 2, LZ77SSS_LPF_LNF_OPT = 3 };
/* enum factorize_mode, lz77_sss.hpp:55-59 (same numeric values) */
enum { LZ77SSS_GREEDY_NAIVE = 0, LZ77SSS_GREEDY = 1, LZ77SSS_SKIP_PHRASES = 2 };

/* enum transform_mode, lz77_sss.hpp:60-64 (same numeric values); FULL_SA is a device
 * extension (not a reference mode): the lengths from LPF over the full suffix array */
enum { LZ77SSS_TRANSF_NAIVE = 0, LZ77SSS_TRANSF_WITH_SAMPLES = 1, LZ77SSS_TRANSF_WITHOUT_SAMPLES = 2,
       LZ77SSS_TRANSF_FULL_SA = 3 };

enum {
    LZ77SSS_OK = 0,
    LZ77SSS_EINVAL = -1,      /* bad argument (unsupported mode, tau, n too large for pos_t) */
    LZ77SSS_ENODEV = -2,      /* no HIP device / HIP runtime error at init */
    LZ77SSS_EHIP = -3,        /* HIP runtime error during a launch / copy */
    LZ77SSS_ENOMEM = -4,      /* device or host allocation failed */
    LZ77SSS_ECALLBACK = -5,   /* the emit callback returned non-zero (output aborted) */
    LZ77SSS_EINTERNAL = -6    /* internal consistency check failed */
};

typedef struct { uint32_t src; uint32_t len; } lz77sss_factor32;
typedef struct { uint64_t src; uint64_t len; } lz77sss_factor64;

typedef struct {
    int32_t phr_mode;        /* default LZ77SSS_LPF_OPT, lz77_sss.hpp:77 */
    int32_t fact_mode;       /* default LZ77SSS_GREEDY, lz77_sss.hpp:78; LZ77SSS_SKIP_PHRASES gives
                                the gapped stream of factorize_skip_gaps (skip_gaps.cpp:31-61):
                                {first phrase start, 0}, then {src, len} per LPF phrase, each
                                followed by {gap length, 0} when the next phrase starts later */
    uint32_t tau;            /* default 512, lz77_sss.hpp:82 (only 512 is supported) */
    uint32_t rk_seed;        /* seeds the 5 gap-index rk_prime<107> bases (replaces the
                                std::random_device of rolling_hash.hpp:127-130) */
    int32_t index_log2_size; /* 0 = the reference formula with malloc_count == 0
                                (lz77_sss.hpp:117-122, rolling_hash_index_107.hpp:59-70) */
    int32_t device;          /* HIP device ordinal */
    int32_t log;             /* parameters::log: print per-phase times to stderr */
    uint16_t num_threads;    /* parameters::num_threads; accepted for API parity -- the
                                output is always the p = 1 factorization */
} lz77sss_params;

/* Fills defaults (the reference's template defaults + rk_seed = 42). */
void lz77sss_default_params(lz77sss_params* prm);

/* Batched, in-order factor sink.  Return 0 to continue, non-zero to abort. */
typedef int (*lz77sss_emit_fn)(const lz77sss_factor32* batch, uint64_t count, void* user);
typedef int (*lz77sss_emit64_fn)(const lz77sss_factor64* batch, uint64_t count, void* user);

/* One-shot: factorize text[0..n) (host memory).  LPF/LNF modes do NOT modify
 * `text` (the reference reverses the caller's buffer in place and restores
 * it, lz77_sss.hpp:385-393; here the reversal happens in HBM).  No padding
 * past n is required. */
int lz77sss_factorize_approx_u32(const uint8_t* text, uint64_t n, const lz77sss_params* prm,
                                 lz77sss_emit_fn emit, void* user);
/* The same with pos_t = uint64_t: any n up to 2^40 (texts past 2^32 - 16 bytes need this
 * one).  The gap index is sized by the reference's formula for 8-byte entries
 * (rolling_hash_index_107.hpp:59-70), so the stream is the reference's pos_t = uint64_t
 * stream, which differs from the uint32_t one in general.  Every phr_mode (lpf_naive,
 * lpf_lnf_naive, lpf_opt, lpf_lnf_opt). */
int lz77sss_factorize_approx_u64(const uint8_t* text, uint64_t n, const lz77sss_params* prm,
                                 lz77sss_emit64_fn emit, void* user);

/* One-shot exact factorization (greedy LZ77: every factor is a longest previous
 * factor; a copy {src, len >= 1} or the literal {char, 0} when the character is
 * new).  The factor lengths are the canonical greedy LZ77 ones, as the
 * reference's exact modes produce at p = 1.  transf_mode naive, with_samples and
 * without_samples run the reference's exact-smpl path on the device (csrc/smpl.hip:
 * the 3-approximation, the sample index over its phrase ends and delta-samples, the
 * decomposed weighted square grid, and per order keyed insertion ranks over adjacent-LCE
 * and weight sparse tables, which answer every interval query with_samples' interval
 * samples would; lz77_sss.hpp:558-709, transform_to_exact/{naive,with_samples,without_samples}.cpp); their sources are
 * the reference's: of the factors of the final length, the first the transform's visit order
 * meets, its point from the Pi / Psi scan or the reference's own 16384-rank grid (a source pass
 * after the chain; with PA / SA ties in sample order, the stable-sort reading of the
 * reference's ips4o).  LZ77SSS_TRANSF_FULL_SA computes the
 * same lengths from LPF over the full suffix array of the text (csrc/exact.hip; 44 B
 * per character, n < 2^31) with the PSV/NSV source rule.  The sample-index modes require
 * n < 2^32 - 16 and fewer than 2^31 samples (z_aprx + n/delta; LZ77SSS_EINVAL otherwise). */
int lz77sss_factorize_exact_u32(const uint8_t* text, uint64_t n, const lz77sss_params* prm, int transf_mode,
                                lz77sss_emit_fn emit, void* user);
/* pos_t = uint64_t form of the exact factorization: the factors are widened to lz77sss_factor64,
 * the computation runs on a pos_t = uint32_t session, so the limits of the _u32 form apply
 * (sample-index modes n < 2^32 - 16, FULL_SA n < 2^31). */
int lz77sss_factorize_exact_u64(const uint8_t* text, uint64_t n, const lz77sss_params* prm, int transf_mode,
                                lz77sss_emit64_fn emit, void* user);

/* Decode nf factors into out[0..n) (host memory), algorithms/common.cpp:31-54. */
int lz77sss_decode_u32(const lz77sss_factor32* factors, uint64_t nf, uint8_t* out, uint64_t n);

/* Same, decoded on `device` (csrc/decode.hip: pointer jumping over source
 * references, O(n log depth) work).  Stricter than the host decode: the factor
 * lengths must sum to exactly n. */
int lz77sss_decode_u32_device(const lz77sss_factor32* factors, uint64_t nf, uint8_t* out, uint64_t n, int device);
int lz77sss_decode_u64(const lz77sss_factor64* factors, uint64_t nf, uint8_t* out, uint64_t n);
int lz77sss_decode_u64_device(const lz77sss_factor64* factors, uint64_t nf, uint8_t* out, uint64_t n, int device);
/* The reference's pos_t = uint64_t factor stream (lz77_sss.hpp:149-173): 5 bytes src, 5
 * bytes len, little endian; out holds 10 * nf bytes.  Returns LZ77SSS_EINVAL if a value
 * needs more than 40 bits. */
int lz77sss_serialize_factors64(const lz77sss_factor64* factors, uint64_t nf, uint8_t* out);
int lz77sss_deserialize_factors64(const uint8_t* in, uint64_t nf, lz77sss_factor64* factors);

/* ---- device-resident session (text stays in HBM across calls) ---- */
typedef struct lz77sss_session lz77sss_session;

/* Creates a session on `device` able to hold texts of up to max_n bytes (pos_t = uint32_t:
 * n <= 2^32 - 16). */
int lz77sss_session_create(int device, uint64_t max_n, lz77sss_session** out);
/* A pos_t = uint64_t session (lz77_sss<uint64_t>): any n up to 2^40.  Supports load,
 * gen_genome, factorize (every phr_mode; greedy / skip_phrases), verify, get_factors64,
 * decode, sss, get_sss64, get_sa_s, get_lpf64, phase_times, stats, sss_kernel_time;
 * the 32-bit accessors and the exact / LNF / container entry points return LZ77SSS_EINVAL. */
int lz77sss_session_create64(int device, uint64_t max_n, lz77sss_session** out);
int lz77sss_session_is64(const lz77sss_session* s);
/* Copies text[0..n) host -> HBM (not part of the timed factorization). */
int lz77sss_session_load(lz77sss_session* s, const uint8_t* text, uint64_t n);
/* Factorizes the loaded text; factors stay in HBM. */
int lz77sss_session_factorize(lz77sss_session* s, const lz77sss_params* prm, uint64_t* num_factors);
/* Exact factorization of the loaded text (see lz77sss_factorize_exact_u32); factors stay in HBM. */
int lz77sss_session_factorize_exact(lz77sss_session* s, const lz77sss_params* prm, int transf_mode,
                                    uint64_t* num_factors);
/* Copies the factors HBM -> host (cap >= num_factors). */
int lz77sss_session_get_factors(lz77sss_session* s, lz77sss_factor32* out, uint64_t cap);
/* 64-bit factors (any session; a 32-bit session's factors are widened). */
int lz77sss_session_get_factors64(lz77sss_session* s, lz77sss_factor64* out, uint64_t cap);
/* Decodes the factors of the last factorize call on the device.  out (host,
 * cap >= n) may be NULL; when mismatches is given it receives the number of
 * positions where the decoded text differs from the loaded one (0 = round trip
 * holds), without leaving HBM.  Timed as phase "decode". */
int lz77sss_session_decode(lz77sss_session* s, uint8_t* out, uint64_t cap, uint64_t* mismatches);
/* Checks the factors of the last factorization against the loaded text without decoding
 * them (a 50 GiB stream needs no n-sized decode buffers): *bad_positions = the number of
 * positions whose factor does not reproduce the text (a literal with another byte, a copy
 * from a position >= its own, a copied byte that differs); 0 <=> decode(F) == T; first_bad
 * (may be NULL) the smallest such position (UINT64_MAX if none).  Fails with LZ77SSS_EINVAL
 * when the lengths do not sum to n, when the session holds no factorization yet, and after a
 * skip_phrases call (its gapped stream is not a factorization). */
int lz77sss_session_verify(lz77sss_session* s, uint64_t* bad_positions, uint64_t* first_bad);
/* Runs only the string-synchronizing-set pass (kernel 1) on the loaded text. */
int lz77sss_session_sss(lz77sss_session* s, uint64_t* size_sss, int* has_runs);
/* Copies the sync set of the last sss/factorize call HBM -> host. */
int lz77sss_session_get_sss(lz77sss_session* s, uint32_t* out, uint64_t cap);
/* pos_t = uint64_t sync set (lce::rolling_hash::sss<uint64_t, tau>, called at
 * patched-files/external/lce/include/ds/lce_sss.hpp:53 with the pos_t of
 * lz77_sss.hpp:72-75): S n [first, end) of the loaded text, any n, computed in
 * windows of `window` decisions (0 = 2^30, rounded up to a multiple of 4096, at
 * most 2^31) with a 2*tau-1 byte halo each; end is clamped to n - 2*tau + 1.
 * Positions are reported + base: a rank of a sharded job loads its block
 * T[b_r, e_r + 2*tau - 1), passes [0, e_r - b_r) and base = b_r, and the
 * concatenation over ranks in rank order is the sync set of T.
 * The result stays in HBM until get_sss64 / copy_sss64_device. */
int lz77sss_session_sss_range(lz77sss_session* s, uint64_t first, uint64_t end, uint64_t base, uint64_t window,
                              uint64_t* size_sss, int* has_runs);
int lz77sss_session_get_sss64(lz77sss_session* s, uint64_t* out, uint64_t cap);  /* also a 64-bit session's S */
/* Device-to-device copy of the sss_range result into `dst`, a device buffer on the
 * session's device (e.g. a collective's send buffer); cap in elements. */
int lz77sss_session_copy_sss64_device(lz77sss_session* s, void* dst, uint64_t cap);
/* Copy of the last factorization (factorize / greedy_block) in the session's own
 * layout -- lz77sss_factor32 for a 32-bit session, lz77sss_factor64 for a 64-bit
 * one -- to `dst` (host or device memory; device-to-device for a collective's send
 * buffer, the emission step of SURVEY.md 8e).  *bytes receives the size; dst NULL
 * with cap_bytes 0 only queries it.  Replaces reading lz77_sss::factorize's output
 * vector (lz77_sss.hpp:259-282) on the rank that emits it. */
int lz77sss_session_copy_factors_device(lz77sss_session* s, void* dst, uint64_t cap_bytes, uint64_t* bytes);
/* Fills the session text with n bytes of a chr19-style text generated in HBM: a
 * random ACGT block of base_len bytes, repeated, each copy byte mutated to another
 * base with probability mut_rate -- every byte a function of (position, seed), so
 * any block of it can be generated alone (the C4 input, without a host copy). */
int lz77sss_session_gen_genome(lz77sss_session* s, uint64_t n, uint64_t base_len, double mut_rate, uint32_t seed,
                               uint64_t offset);
/* ssszip's gapped container of the last factorize call, which must have used
 * fact_mode = LZ77SSS_SKIP_PHRASES (encode_gapped, cli/ssszip.cpp:119-177, vbyte
 * codes of misc/vbyte.hpp:62-84, min_lpf_len 64 of cli/ssszip.cpp:37): built in HBM;
 * *size = its byte length; out (host, cap >= *size) may be NULL to query the size. */
int lz77sss_session_ssszip_gapped(lz77sss_session* s, uint8_t* out, uint64_t cap, uint64_t* size);
/* The Huffman factor container of the last factorization (huff_writer,
 * include/lz77_sss/misc/huffman.hpp:318-375, as written by
 * cli/lz77_sss_3_aprx.cpp:71-85): 5 bytes n, then per block of 2^14 factors an
 * Elias-delta count, two 66-symbol length-limited Huffman tables and the coded
 * factors.  Built in HBM; out (host) may be NULL to query *size. */
int lz77sss_session_huffman(lz77sss_session* s, uint8_t* out, uint64_t cap, uint64_t* size);
/* Copies SA_S / LCP_S (suffix order of the sync positions) of the last call. */
int lz77sss_session_get_sa_s(lz77sss_session* s, uint32_t* sa, uint32_t* lcp, uint64_t cap);
/* Copies the LPF phrase list (beg,end,src triples) of the last factorize call. */
int lz77sss_session_get_lpf(lz77sss_session* s, uint32_t* out3, uint64_t cap, uint64_t* count);
int lz77sss_session_get_lpf64(lz77sss_session* s, uint64_t* out3, uint64_t cap, uint64_t* count);
/* Per-phase times (ms, hipEvent-timed) of the last call; returns the count. */
int lz77sss_session_phase_times(lz77sss_session* s, double* ms, const char** names, int cap);
/* Device memory per phase of the last call, in the order of lz77sss_session_phase_times: the
 * bytes the process's engine buffers held when the phase was enqueued (held), their peak during the
 * phase (peak), and the GPU's free memory then (hbm_free: hipMemGetInfo at the call's start, later
 * phases derived from the process's allocations since; every phase queried when LZ77SSS_PHASE_MEM is
 * set).  held / peak are process-wide: with several sessions in one process they count all of them.
 * A lean call (texts of 8 GiB and more) starts with a "release" phase that frees the last call's
 * emitter buffers, so the later peaks do not include them.  The text itself (n + 64 KiB) is not in
 * held/peak.  Returns the number of phases (or a negative error). */
int lz77sss_session_phase_mem(lz77sss_session* s, uint64_t* held, uint64_t* peak, uint64_t* hbm_free, int cap);
/* Statistics of the last factorize call: [size_sss, has_runs, num_lpf, len_lpf_phr,
 * num_gaps, patt_lens[5], roll_threshold, log2_size_h, greedy_rounds, fixups, ...]; after an
 * exact-smpl call 24..28 = samples, delta, phrase tasks, chunks << 32 | doubling levels, and 1 when
 * the sources follow the reference's visit order. */
int lz77sss_session_stats(lz77sss_session* s, uint64_t* out, int cap);
void lz77sss_session_destroy(lz77sss_session* s);

/* ---- sharded factorization ----
 * One text, N ranks (one session per rank, the whole text loaded on each):
 *   1. rank r: lz77sss_session_sss_range on its text block, all-gather the blocks' sync
 *      sets in rank order, lz77sss_session_set_sss with the gathered set;
 *   2. every rank: lz77sss_session_prepare(external_sss = 1) -- SA_S, LCP, LCE and the
 *      phrases (replicated), and the gap-index parameters;
 *   3. in rank order: rank r receives the chain state and the carried table from r - 1
 *      (lz77sss_session_carried_copy into its session), runs lz77sss_session_greedy_block
 *      on [state.start, b_{r+1}) and sends exit state + carried table to r + 1;
 *   4. the ranks' factors concatenated in rank order are the factorization of the text
 *      (bit-identical to one lz77sss_session_factorize of the whole text). */
typedef struct {
    uint64_t start;       /* in: chain position where the block's walk starts (0 on rank 0) */
    uint64_t idxpos;      /* in: gap-index position at start (0 on rank 0) */
    uint32_t zmask;       /* in: zeroed-fingerprint mask (0 on every rank but a text shorter than 65) */
    int32_t carried;      /* in: 1 = the session's carried table holds the inserts before start */
    uint64_t end;         /* in: block end: n (last rank) or <= n - 4160 */
    uint64_t exit_start;  /* out: the next block's start (the first hand-over point >= end) */
    uint64_t exit_idxpos; /* out */
    uint32_t exit_zmask;  /* out */
    uint32_t reserved;    /* in: 1 (with carried = 0) = start from the table of the gap positions before
                             start (the lead-in of a speculative block); else 0 */
} lz77sss_block;
/* Loads an externally computed sync set (host or device pointer, 64-bit positions). */
int lz77sss_session_set_sss(lz77sss_session* s, const uint64_t* S, uint64_t count, int has_runs);
/* Phases before the greedy emitter; *carried_bytes = size of the carried table. */
int lz77sss_session_prepare(lz77sss_session* s, const lz77sss_params* prm, int external_sss,
                            uint64_t* carried_bytes);
/* Carried table <-> buf (host or device memory): to_session = 1 loads it, 0 reads it. */
int lz77sss_session_carried_copy(lz77sss_session* s, void* buf, uint64_t bytes, int to_session);
/* The greedy chain of one block; its factors replace the session's factors. */
int lz77sss_session_greedy_block(lz77sss_session* s, const lz77sss_params* prm, lz77sss_block* blk,
                                 uint64_t* num_factors);
/* Speculative blocks (no reference counterpart: the reference's chain is one
 * sequential loop, greedy.cpp:46-134).  A speculative block starting at block_start is walked
 * as consecutive parts 0, 1, ... (one greedy_block each, each from the previous one's exit
 * state).  spec_begin(part): the next greedy_block is part `part`; part 0 starts from the
 * carried table now in the session (a speculated entry table).  The session keeps the table
 * each part started from and records which entry-table slots each part's lookups use.
 * spec_resolve: given the true entry table (host or device, `bytes` as
 * lz77sss_session_prepare reported), *accepted_parts = the number of leading parts all of whose
 * used slots agree: those parts' factors and exit states are the true ones.  The carried table
 * becomes the writes of the accepted parts over the true entry table -- the table to re-walk
 * the rest of the block with, from the exit state of the last accepted part (or the true
 * entry state), or the exit table when every part was accepted.  The caller compares the
 * chain states (parts = 0 rejects everything: the carried table becomes the true one). */
#define LZ77SSS_SPEC_MAX_PARTS 16
int lz77sss_session_spec_begin(lz77sss_session* s, int part, uint64_t block_start);
int lz77sss_session_spec_resolve(lz77sss_session* s, const void* true_table, uint64_t bytes, int parts,
                                 int* accepted_parts);

/* Average duration (ms) of the dominant kernel (SSS main pass) over the
 * last call, measured with hipEvents on its own stream; bytes = algorithmic
 * bytes of that launch (n + 4|S|). */
int lz77sss_session_sss_kernel_time(lz77sss_session* s, double* ms, uint64_t* bytes);

/* ---- synthetic inputs (tests / bench) ---- */
/* random_repetitive_string (utils.hpp:579-640) with a seed instead of
 * std::random_device; knobs < 0 are drawn as in the reference. */
int64_t lz77sss_gen_random_repetitive(uint32_t min_size, uint32_t max_size, uint32_t seed,
                                      double rep_knob, double run_knob, uint8_t* out, uint64_t cap);
/* chr19-style: random ACGT base block repeated with point mutations. */
int64_t lz77sss_gen_genome(uint64_t n, uint64_t base_len, double mut_rate, uint32_t seed, uint8_t* out);
/* The text of lz77sss_session_gen_genome (position-hashed), generated on the host. */
int lz77sss_gen_genome_pos(uint64_t n, uint64_t base_len, double mut_rate, uint32_t seed, uint64_t offset,
                           uint8_t* out);

const char* lz77sss_last_error(void);
/* Number of visible HIP devices (0 if none); does not create a context. */
int lz77sss_device_count(void);

#ifdef __cplusplus
}
#endif
#endif /* LZ77SSS_H */
