// Synthetic input generators (host C++).  Not on the hot path; used by tests
// and bench.py to build inputs of BASELINE.json's configs.
//
//  * lz77sss_gen_random_repetitive restates random_repetitive_string
//    (include/lz77_sss/misc/utils.hpp:579-640) with std::random_device replaced
//    by a seed (utils.hpp:581-582), and optional pinned knobs
//    repetition_repetitiveness / run_repetitiveness (drawn U(0,1) at
//    utils.hpp:591-592 when the argument is < 0).  Uses libstdc++'s
//    distributions exactly as the reference does, so a given seed reproduces
//    the string the reference would produce for that random_device value.
//  * lz77sss_gen_genome: a "chr19-style" text: a random ACGT
//    base block, repeated with independent point mutations per copy.
#include "../include/lz77sss_internal.h"

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <random>

extern "C" {

LZ77SSS_API int64_t lz77sss_gen_random_repetitive(uint32_t min_size, uint32_t max_size, uint32_t seed,
                                                  double rep_knob, double run_knob,
                                                  uint8_t* out, uint64_t cap) {
    std::mt19937 mt(seed);
    std::uniform_real_distribution<double> prob_distrib(0.0, 1.0);
    std::uniform_int_distribution<int> char_distrib(-128, 127);
    // random_log_uniform_size (utils.hpp:569-577)
    std::uniform_real_distribution<double> log_distrib(std::log((double)std::max<uint64_t>(1, min_size)),
                                                       std::log((double)std::max<uint64_t>(1, max_size)));
    uint32_t target = (uint32_t)std::clamp<uint64_t>((uint64_t)std::llround(std::exp(log_distrib(mt))), min_size, max_size);
    double rep = prob_distrib(mt);
    double run = prob_distrib(mt);
    if (rep_knob >= 0) rep = rep_knob;
    if (run_knob >= 0) run = run_knob;
    std::uniform_int_distribution<uint32_t> rep_len_distrib(1, std::max((rep * target) / 100, 1.0));
    std::uniform_int_distribution<uint32_t> run_len_distrib(1, std::max((run * target) / 200, 1.0));
    std::discrete_distribution<int> op_distrib({2 - (rep + run), rep, run});
    if (target > cap) return -1;
    uint64_t sz = 0;
    out[sz++] = (uint8_t)(char)char_distrib(mt);
    while (sz < target) {
        switch (op_distrib(mt)) {
            case 0: out[sz++] = (uint8_t)(char)char_distrib(mt); break;
            case 1: {
                uint32_t len = std::min<uint32_t>(target - (uint32_t)sz, rep_len_distrib(mt));
                uint32_t src = std::uniform_int_distribution<uint32_t>(0, (uint32_t)sz - 1)(mt);
                for (uint32_t i = 0; i < len; i++) { out[sz] = out[src + i]; sz++; }
                break;
            }
            case 2: {
                uint32_t len = std::min<uint32_t>(target - (uint32_t)sz, run_len_distrib(mt));
                uint8_t c = (uint8_t)(char)char_distrib(mt);
                for (uint32_t i = 0; i < len; i++) out[sz++] = c;
                break;
            }
        }
    }
    return (int64_t)sz;
}

// genome-like: base block of `base_len` uniform ACGT, then copies of the base
// with each character replaced (by a different base letter) with probability
// mut_rate.  Deterministic in seed (mt19937_64, raw draws only).
LZ77SSS_API int64_t lz77sss_gen_genome(uint64_t n, uint64_t base_len, double mut_rate, uint32_t seed, uint8_t* out) {
    static const char acgt[4] = {'A', 'C', 'G', 'T'};
    std::mt19937_64 g(seed);
    base_len = std::min(base_len, n);
    for (uint64_t i = 0; i < base_len; i++) out[i] = (uint8_t)acgt[g() >> 62];
    const uint64_t thr = (uint64_t)(mut_rate * 18446744073709551615.0);
    for (uint64_t i = base_len; i < n; i++) {
        uint8_t c = out[i % base_len];
        if (g() < thr) {
            int k = 0;
            while (acgt[k] != (char)c) k++;
            k = (k + 1 + (int)(g() % 3)) & 3;
            c = (uint8_t)acgt[k];
        }
        out[i] = c;
    }
    return (int64_t)n;
}

}  // extern "C"
