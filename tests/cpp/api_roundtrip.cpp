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
        // exact mode, as tests/test_lz77_sss.cpp:95-133 of the reference (round trip only)
        std::vector<typename lz::factor> FX;
        lz::template factorize_exact<greedy, lpf_opt, without_samples, decomposed_semi_dynamic_square_grid>(
            T.data(), (pos_t)n, [&](typename lz::factor f) { FX.push_back(f); });
        std::string DX;
        lz::decode(FX.begin(), std::back_inserter(DX), (pos_t)n);
        if (DX != T || FX.size() > F.size()) {
            std::printf("seed %d: exact round trip FAILED\n", seed);
            return 1;
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
                    FX.size());
    }
    return 0;
}

int main(int argc, char** argv) {
    const int nseeds = argc > 1 ? std::atoi(argv[1]) : 4;
    const int a = run<uint32_t>(nseeds);
    if (a) return a;
    return run<uint64_t>(nseeds);
}
