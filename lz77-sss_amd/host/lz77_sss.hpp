// lz77_sss.hpp -- drop-in C++ host mirror of the reference's static template API
// (include/lz77_sss/lz77_sss.hpp:48-203 of LukasNalbach/lz77-sss) over the
// C-ABI of liblz77sss_hip.so (include/lz77sss.h).
//
// A caller of
//     lz77_sss<pos_t>::factorize_approximate<greedy, lpf_opt, 512>(T, n, out, {.num_threads = p});
//     lz77_sss<uint32_t>::factorize_exact<greedy, lpf_opt, with_samples>(T, n, out);
//     lz77_sss<uint32_t>::decode(fact_it, out_it, n);
// keeps its code and links against the HIP library instead.  Differences:
//   * the factorization runs on an MI355X (device `parameters::device`) with the
//     p = 1 output stream of the reference (num_threads is accepted and ignored);
//   * errors surface as lz77_sss_error (the reference only asserts); no CPU fallback;
//   * pos_t = uint32_t (n < 2^32) or uint64_t (any n up to 2^40; the pos_t = uint64_t
//     engine, lz77sss_factorize_approx_u64); the factor layout is the reference's
//     `factor{pos_t src, len}` (literal <=> len == 0, src = the byte), streamed as 8
//     or 5 + 5 bytes (lz77_sss.hpp:149-173);
//   * the input is not modified (the reference's LPF/LNF modes reverse it in place
//     and restore it, lz77_sss.hpp:385-393).
#pragma once

#include <cstdint>
#include <istream>
#include <ostream>
#include <stdexcept>
#include <string>
#include <type_traits>
#include <vector>

#include "../../include/lz77sss.h"

enum phrase_mode { lpf_naive, lpf_lnf_naive, lpf_opt, lpf_lnf_opt };   // lz77_sss.hpp:48-53
enum factorize_mode { greedy_naive, greedy, skip_phrases };            // lz77_sss.hpp:55-59
enum transform_mode { naive, with_samples, without_samples };          // lz77_sss.hpp:60-64

// Range structures of the reference's exact modes (data_structures/*_range/*.hpp):
// accepted as template arguments for source compatibility.  The device exact-smpl
// path (csrc/smpl.hip) always builds the default, a decomposed static weighted
// square grid (decomposed_range.hpp:78-166, static_weighted_square_grid.hpp:67-185);
// the factor lengths are the canonical greedy LZ77 ones whichever structure is
// named, the sources those of the default structure's visit order.
template <typename> struct static_weighted_kd_tree {};
template <typename> struct static_weighted_square_grid {};
template <typename> struct static_weighted_striped_square {};
template <typename> struct dynamic_square_grid {};
template <typename> struct semi_dynamic_square_grid {};
template <typename> struct decomposed_static_weighted_square_grid {};
template <typename> struct decomposed_static_weighted_kd_tree {};
template <typename> struct decomposed_semi_dynamic_square_grid {};

// lz77_sss.hpp:67-70, plus the device-side knobs of this implementation
struct parameters {
    uint16_t num_threads = 0;  // accepted for source compatibility (p = 1 semantics)
    bool log = false;          // phase timings on stderr
    int device = 0;            // HIP device ordinal
    uint32_t rk_seed = 42;     // seed of the gap-index Karp-Rabin bases (rolling_hash.hpp:127-130)
};

struct lz77_sss_error : std::runtime_error {
    int code;
    lz77_sss_error(int c, const std::string& what) : std::runtime_error(what), code(c) {}
};

template <typename pos_t = uint32_t>
class lz77_sss {
    static_assert(std::is_same_v<pos_t, uint32_t> || std::is_same_v<pos_t, uint64_t>,
                  "pos_t is uint32_t or uint64_t (lz77_sss.hpp:72-75)");
    static constexpr bool wide = std::is_same_v<pos_t, uint64_t>;
    using cfactor = std::conditional_t<wide, lz77sss_factor64, lz77sss_factor32>;

    static void check(int rc) {
        if (rc != LZ77SSS_OK) {
            const char* m = lz77sss_last_error();
            throw lz77_sss_error(rc, std::string("lz77sss: ") + (m ? m : "error"));
        }
    }

  public:
    static constexpr phrase_mode default_phr_mode = lpf_opt;
    static constexpr factorize_mode default_fact_mode = greedy;
    static constexpr transform_mode default_transf_mode = without_samples;
    template <typename sidx_t> using default_range_ds_t = decomposed_static_weighted_square_grid<sidx_t>;
    static constexpr uint64_t default_tau = 512;

    struct factor {  // lz77_sss.hpp:129-147 (same layout as lz77sss_factor32 / lz77sss_factor64)
        pos_t src;
        pos_t len;
        pos_t length() const { return len > 1 ? len : 1; }
        static constexpr pos_t size_of() { return wide ? 10 : 8; }
        // the reference's stream form: 8 bytes (uint32_t), 5 + 5 bytes little endian (uint64_t)
        friend std::ostream& operator<<(std::ostream& out, const factor& f) {
            if constexpr (!wide) {
                out.write(reinterpret_cast<const char*>(&f), 8);
            } else {
                out.write(reinterpret_cast<const char*>(&f.src), 5);
                out.write(reinterpret_cast<const char*>(&f.len), 5);
            }
            return out;
        }
        friend std::istream& operator>>(std::istream& in, factor& f) {
            if constexpr (!wide) {
                in.read(reinterpret_cast<char*>(&f), 8);
            } else {
                f.src = f.len = 0;
                in.read(reinterpret_cast<char*>(&f.src), 5);
                in.read(reinterpret_cast<char*>(&f.len), 5);
            }
            return in;
        }
    };
    static_assert(sizeof(factor) == sizeof(cfactor));

    // lz77_sss.hpp:176-186: factors are handed to `output` by value, in text order,
    // on the calling thread.
    template <factorize_mode fact_mode = default_fact_mode, phrase_mode phr_mode = default_phr_mode,
              uint64_t tau = default_tau, typename char_t, typename output_fnc_t>
    static void factorize_approximate(char_t* input, pos_t input_size, output_fnc_t output, parameters params = {}) {
        static_assert(sizeof(char_t) == 1, "byte alphabet only (lz77_sss.hpp:287)");
        lz77sss_params p;
        lz77sss_default_params(&p);
        p.phr_mode = static_cast<int32_t>(phr_mode);
        p.fact_mode = static_cast<int32_t>(fact_mode);
        p.tau = static_cast<uint32_t>(tau);
        p.rk_seed = params.rk_seed;
        p.device = params.device;
        p.log = params.log ? 1 : 0;
        p.num_threads = params.num_threads;
        struct ctx_t {
            output_fnc_t* out;
        } ctx{&output};
        auto emit = [](const cfactor* batch, uint64_t count, void* user) -> int {
            auto* c = static_cast<ctx_t*>(user);
            for (uint64_t k = 0; k < count; k++) (*c->out)(factor{(pos_t)batch[k].src, (pos_t)batch[k].len});
            return 0;
        };
        if constexpr (wide)
            check(lz77sss_factorize_approx_u64(reinterpret_cast<const uint8_t*>(input), input_size, &p, emit, &ctx));
        else
            check(lz77sss_factorize_approx_u32(reinterpret_cast<const uint8_t*>(input), input_size, &p, emit, &ctx));
    }

    // lz77_sss.hpp:188-200: exact factorization.  Every transf_mode of the reference
    // (naive, with_samples, without_samples, lz77_sss.hpp:616-661) runs the sample-index
    // transform on the device (csrc/smpl.hip); with_samples adds the Rabin-Karp prefix
    // fingerprints and the interval samples (transform_to_exact/with_samples.cpp:31-240).
    // Lengths are the canonical greedy LZ77 ones; see include/lz77sss.h for the sources.
    template <factorize_mode fact_mode = default_fact_mode, phrase_mode phr_mode = default_phr_mode,
              transform_mode transf_mode = default_transf_mode,
              template <typename> typename range_ds_t = default_range_ds_t, uint64_t tau = default_tau,
              typename char_t, typename output_fnc_t>
    static void factorize_exact(char_t* input, pos_t input_size, output_fnc_t output, parameters params = {}) {
        static_assert(sizeof(char_t) == 1, "byte alphabet only (lz77_sss.hpp:287)");
        static_assert(fact_mode != skip_phrases, "lz77_sss.hpp:333");
        lz77sss_params p;
        lz77sss_default_params(&p);
        p.phr_mode = static_cast<int32_t>(phr_mode);
        p.fact_mode = static_cast<int32_t>(fact_mode);
        p.tau = static_cast<uint32_t>(tau);
        p.device = params.device;
        p.log = params.log ? 1 : 0;
        p.num_threads = params.num_threads;
        struct ctx_t {
            output_fnc_t* out;
        } ctx{&output};
        auto emit = [](const cfactor* batch, uint64_t count, void* user) -> int {
            auto* c = static_cast<ctx_t*>(user);
            for (uint64_t k = 0; k < count; k++) (*c->out)(factor{(pos_t)batch[k].src, (pos_t)batch[k].len});
            return 0;
        };
        if constexpr (wide)
            check(lz77sss_factorize_exact_u64(reinterpret_cast<const uint8_t*>(input), input_size, &p,
                                              static_cast<int>(transf_mode), emit, &ctx));
        else
            check(lz77sss_factorize_exact_u32(reinterpret_cast<const uint8_t*>(input), input_size, &p,
                                              static_cast<int>(transf_mode), emit, &ctx));
    }

    // lz77_sss.hpp:202-203 (algorithms/common.cpp:31-54): sequential host decode
    template <typename fact_it_t, typename out_it_t>
    static void decode(fact_it_t fact_it, out_it_t out_it, pos_t output_size) {
        std::vector<uint8_t> buf(output_size);
        std::vector<cfactor> fs;
        for (uint64_t pos = 0; pos < output_size;) {
            const factor f = *fact_it;
            ++fact_it;
            fs.push_back({f.src, f.len});
            pos += f.length();
        }
        if constexpr (wide) check(lz77sss_decode_u64(fs.data(), fs.size(), buf.data(), output_size));
        else check(lz77sss_decode_u32(fs.data(), fs.size(), buf.data(), output_size));
        for (uint64_t i = 0; i < output_size; i++) *out_it++ = static_cast<char>(buf[i]);
    }
};
