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
#include "../../include/lz77sss.h"
#include "../include/lz77sss_internal.h"

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <random>
#include <thread>
#include <vector>

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

// the position-hashed chr19-style text of lz77sss_session_gen_genome, on the host
// (same bytes: byte p is a function of (p, seed) only), so the oracle can check a
// text the device generated in HBM
static inline uint64_t gen_mix_host(uint64_t x) {  // splitmix64 finalizer
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}
LZ77SSS_API int lz77sss_gen_genome_pos(uint64_t n, uint64_t base_len, double mut_rate, uint32_t seed, uint64_t offset,
                                       uint8_t* out) {
    if ((!out && n) || base_len == 0 || !(mut_rate >= 0.0 && mut_rate <= 1.0)) return LZ77SSS_EINVAL;
    const uint64_t thr = mut_rate >= 1.0 ? ~0ull : (uint64_t)(mut_rate * 18446744073709551616.0);
    auto part = [&](uint64_t a, uint64_t b) {
        for (uint64_t i = a; i < b; i++) {
            const uint64_t p = offset + i;
            uint32_t c = (uint32_t)(gen_mix_host((p % base_len) ^ ((uint64_t)seed << 40)) >> 62);
            if (p >= base_len) {
                const uint64_t h = gen_mix_host(p ^ ((uint64_t)seed * 0xD6E8FEB86659FD93ull) ^ 0x5851F42D4C957F2Dull);
                if (h < thr) c = (c + 1 + (uint32_t)((h >> 7) % 3)) & 3;
            }
            out[i] = (uint8_t)"ACGT"[c];
        }
    };
    const uint64_t nt = std::max<uint64_t>(1, std::min<uint64_t>(16, std::thread::hardware_concurrency()));
    std::vector<std::thread> th;
    const uint64_t chunk = (n + nt - 1) / nt;
    for (uint64_t t = 0; t < nt; t++) {
        const uint64_t a = std::min(n, t * chunk), b = std::min(n, a + chunk);
        if (a < b) th.emplace_back(part, a, b);
    }
    for (auto& x : th) x.join();
    return LZ77SSS_OK;
}

}  // extern "C"

// lz77_sss<uint64_t>::factor stream form (include/lz77_sss/lz77_sss.hpp:149-173): the low
// 5 bytes of src, then of len, little endian
extern "C" __attribute__((visibility("default"))) int lz77sss_serialize_factors64(const lz77sss_factor64* f,
                                                                                 uint64_t nf, uint8_t* out) {
    if ((!f || !out) && nf) return LZ77SSS_EINVAL;
    for (uint64_t k = 0; k < nf; k++) {
        if ((f[k].src >> 40) || (f[k].len >> 40)) return LZ77SSS_EINVAL;
        for (int b = 0; b < 5; b++) {
            out[10 * k + b] = (uint8_t)(f[k].src >> (8 * b));
            out[10 * k + 5 + b] = (uint8_t)(f[k].len >> (8 * b));
        }
    }
    return LZ77SSS_OK;
}
extern "C" __attribute__((visibility("default"))) int lz77sss_deserialize_factors64(const uint8_t* in, uint64_t nf,
                                                                                   lz77sss_factor64* f) {
    if ((!f || !in) && nf) return LZ77SSS_EINVAL;
    for (uint64_t k = 0; k < nf; k++) {
        uint64_t s = 0, l = 0;
        for (int b = 0; b < 5; b++) {
            s |= (uint64_t)in[10 * k + b] << (8 * b);
            l |= (uint64_t)in[10 * k + 5 + b] << (8 * b);
        }
        f[k] = lz77sss_factor64{s, l};
    }
    return LZ77SSS_OK;
}
