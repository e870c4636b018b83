// Uses the C++ mirror of the reference API exactly as the reference's own test
// does (tests/test_lz77_sss.cpp:73-82: decode(factorize(T)) == T), on
// random_repetitive_string(10^4, 2*10^5) texts with seeds 1..N.
// Exit status: 0 = all round trips equal, 2 = no device (error surfaced, no fallback), 1 = mismatch.
#include "../../lz77-sss_amd/host/lz77_sss.hpp"

#include <cstdio>
#include <cstring>
#include <sstream>
#include <string>
#include <vector>

template <typename pos_t>
static int run(int nseeds) {
    using lz = lz77_sss<pos_t>;
    for (int seed = 1; seed <= nseeds; seed++) {
        std::vector<uint8_t> buf(200000 + 16);
        const int64_t n = lz77sss_gen_random_repetitive(10000, 200000, seed, -1.0, -1.0, buf.data(), 200000);
        if (n < 0) return 1;
        std::string T(reinterpret_cast<char*>(buf.data()), (size_t)n);
        std::vector<typename lz::factor> F;
        try {
            lz::template factorize_approximate<greedy, lpf_opt>(T.data(), (pos_t)n, [&](typename lz::factor f) { F.push_back(f); });
        } catch (const lz77_sss_error& e) {
            std::printf("error %d: %s\n", e.code, e.what());
            return e.code == LZ77SSS_ENODEV ? 2 : 1;
        }
        std::string D;
        lz::decode(F.begin(), std::back_inserter(D), (pos_t)n);
        if (D != T) {
            std::printf("seed %d: round trip FAILED\n", seed);
            return 1;
        }
        // exact mode, as tests/test_lz77_sss.cpp:95-133 of the reference (round trip only), for
        // every transform_mode of lz77_sss.hpp:60-64 (with_samples: configs[4]); the lengths are the
        // canonical greedy LZ77 ones, so all three streams have the same factor count
        size_t zx[3] = {0, 0, 0};
        std::vector<typename lz::factor> FX;
        auto check_exact = [&](int k, const char* name) -> int {
            std::string DX;
            lz::decode(FX.begin(), std::back_inserter(DX), (pos_t)n);
            if (DX != T || FX.size() > F.size()) {
                std::printf("seed %d: exact %s round trip FAILED\n", seed, name);
                return 1;
            }
            zx[k] = FX.size();
            FX.clear();
            return 0;
        };
        auto sink = [&](typename lz::factor f) { FX.push_back(f); };
        lz::template factorize_exact<greedy, lpf_opt, without_samples, decomposed_semi_dynamic_square_grid>(
            T.data(), (pos_t)n, sink);
        if (check_exact(0, "without_samples")) return 1;
        lz::template factorize_exact<greedy, lpf_opt, with_samples>(T.data(), (pos_t)n, sink);
        if (check_exact(1, "with_samples")) return 1;
        lz::template factorize_exact<greedy, lpf_opt, naive, decomposed_static_weighted_kd_tree>(T.data(), (pos_t)n,
                                                                                               sink);
        if (check_exact(2, "naive")) return 1;
        if (zx[0] != zx[1] || zx[0] != zx[2]) {
            std::printf("seed %d: exact factor counts differ across transform modes\n", seed);
            return 1;
        }
        // LPF/LNF phrases (configs[2], lz77_sss.hpp:384-396; either pos_t)
        {
            std::vector<typename lz::factor> FL;
            lz::template factorize_approximate<greedy, lpf_lnf_opt>(T.data(), (pos_t)n,
                                                                    [&](typename lz::factor f) { FL.push_back(f); });
            std::string DL;
            lz::decode(FL.begin(), std::back_inserter(DL), (pos_t)n);
            if (DL != T) {
                std::printf("seed %d: lpf_lnf_opt round trip FAILED\n", seed);
                return 1;
            }
        }
        // the factor stream form (lz77_sss.hpp:149-173): write and read back
        std::stringstream ss;
        for (auto& f : F) ss << f;
        if (ss.str().size() != F.size() * (size_t)lz::factor::size_of()) return 1;
        for (auto& f : F) {
            typename lz::factor g{};
            ss >> g;
            if (g.src != f.src || g.len != f.len) return 1;
        }
        std::printf("pos_t=%zu seed %d: n=%lld z=%zu z_exact=%zu ok\n", 8 * sizeof(pos_t), seed, (long long)n, F.size(),
                    zx[0]);
    }
    return 0;
}

int main(int argc, char** argv) {
    const int nseeds = argc > 1 ? std::atoi(argv[1]) : 4;
    const int a = run<uint32_t>(nseeds);
    if (a) return a;
    return run<uint64_t>(nseeds);
}
