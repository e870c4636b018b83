// engine_if.h -- the C-ABI's view of the pos_t = uint64_t engine (namespace lz64,
// compiled from the same sources with -DLZ_POS64).  The C-ABI itself is built
// once, with the pos_t = uint32_t engine; 64-bit sessions go through this interface.
#pragma once
#include "lz77sss_internal.h"
#include "timer.h"

#include <vector>

namespace lz {

struct engine_if {
    virtual ~engine_if() = default;
    virtual int device() const = 0;
    virtual u64 n() const = 0;
    virtual u64 max_n() const = 0;
    virtual u8* text() = 0;                  // HBM text (n + TEXT_PAD bytes)
    virtual hipStream_t stream() = 0;
    virtual void set_n(u64 n) = 0;
    virtual void load(const u8* t, u64 n) = 0;
    virtual u64 factorize(int phr_mode, u32 rk_seed, int log2_override, bool log, int fact_mode) = 0;
    virtual u64 num_fact() const = 0;
    virtual const u64* factors() const = 0;  // device, (src, len) pairs
    virtual u64* factors_buf(u64 nf) = 0;    // device buffer for nf factors (decode input)
    virtual u64 decode(const u64* F, u64 nf, u64 n_out, u8* d_out, bool cmp_with_text) = 0;
    virtual u8* dec_out(u64 n) = 0;
    virtual u64 verify(u64* first_bad) = 0;  // the factors against the loaded text (csrc/decode.hip)
    virtual void sss(u64* size, int* has_runs) = 0;
    virtual u64 sss_size() const = 0;
    virtual const u64* sss_ptr() const = 0;
    // sync set of a decision range (build_sss_range), kept apart from the text's own S
    virtual void sss_range(u64 first, u64 end, u64 base, u64 window, u64* size, int* has_runs) = 0;
    virtual u64 range_size() const = 0;
    virtual const u64* range_ptr() const = 0;
    virtual u64 num_phr() const = 0;
    virtual const u64* lpf_ptr() const = 0;  // (beg, end, src) triples
    virtual const u32* sa_ptr() const = 0;
    virtual const u32* lcp_ptr() const = 0;
    virtual std::vector<u64>& stats() = 0;
    virtual phase_timer& timer() = 0;
    virtual double sss_kernel_ms() const = 0;
    virtual u64 sss_kernel_bytes() const = 0;
    virtual u32 dec_rounds() const = 0;
    // sharded factorization (rank-ordered greedy blocks)
    virtual void set_sss(const u64* S_any, u64 count, bool runs) = 0;
    virtual u64 prepare(int phr_mode, bool external_sss, int log2_override) = 0;  // returns carried-table bytes
    virtual void* carried_table() = 0;
    virtual u64 carried_bytes() const = 0;   // capacity of the carried table
    virtual u64 greedy_block(u32 rk_seed, int log2_override, u64* state /* start, idxpos, zmask, carried, end,
                                                                        exit_start, exit_idxpos, exit_zmask */) = 0;
    virtual void spec_begin(int part, u64 base) = 0;
    virtual int spec_resolve(const void* true_tab, u64 bytes, int parts) = 0;
};

// defined in the LZ_POS64 compilation of csrc/engine.hip; throws lz::error
engine_if* make_engine64(int dev, u64 maxn);

}  // namespace lz
