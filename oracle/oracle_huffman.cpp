// oracle_huffman.cpp -- TEST INFRASTRUCTURE ONLY (linked into liboracle.so).
// Sequential restatement of the Huffman factor container of
// include/lz77_sss/misc/huffman.hpp (bit_writer :41-93, put_elias_delta :153-160,
// huffman::build_from_freq/build_codes/write_table :177-300, huff_writer :318-375):
// 5 bytes n (LE); per block of 2^14 factors an Elias-delta count, two 66-entry
// 4-bit code-length tables, then per factor code(lb) + payload.  The reference file
// cannot be compiled here (it needs std::byteswap, GCC >= 12), so this restatement
// plus the decoder below (huff_factor_iterator :377-436) pin the format by round trip.
#include <algorithm>
#include <array>
#include <cstdint>
#include <cstring>
#include <queue>
#include <vector>

namespace {

constexpr uint32_t SIG = 66, BLK = 1u << 14, MAXL = 15;

struct bits_out {
    std::vector<uint8_t> b;
    uint64_t nbit = 0;
    void put(uint64_t x, uint32_t n) {  // n low bits of x, most significant first
        for (uint32_t k = n; k-- > 0;) {
            if ((nbit & 7) == 0) b.push_back(0);
            if ((x >> k) & 1) b.back() |= (uint8_t)(0x80u >> (nbit & 7));
            nbit++;
        }
    }
};
struct bits_in {
    const uint8_t* b;
    uint64_t nbytes, p = 0;
    uint64_t get(uint32_t n) {
        uint64_t x = 0;
        for (uint32_t k = 0; k < n; k++, p++) x = (x << 1) | (p / 8 < nbytes ? (b[p / 8] >> (7 - p % 8)) & 1 : 0);
        return x;
    }
};
uint32_t bw(uint64_t x) { return x ? 64 - __builtin_clzll(x) : 0; }

struct code_t {
    std::array<uint32_t, SIG> len{}, code{};
};
void canonical(code_t& c) {
    std::array<uint64_t, MAXL + 1> cnt{}, next{};
    for (uint32_t s = 0; s < SIG; s++)
        if (c.len[s]) cnt[c.len[s]]++;
    uint64_t v = 0;
    for (uint32_t l = 1; l <= MAXL; l++) next[l] = v = (v + cnt[l - 1]) << 1;
    for (uint32_t s = 0; s < SIG; s++)
        if (c.len[s]) c.code[s] = (uint32_t)next[c.len[s]]++;
}
code_t build(const std::array<uint64_t, SIG>& f) {
    code_t c;
    std::vector<uint64_t> used;
    for (uint32_t s = 0; s < SIG; s++)
        if (f[s]) used.push_back(s);
    if (used.size() == 1) c.len[used[0]] = 1;
    if (used.size() > 1) {
        // Huffman tree on a min-heap of (weight, node id); ties by node id
        std::vector<std::array<uint64_t, 3>> kids;  // internal nodes: {left, right, -}
        const uint64_t leaves = used.size();
        std::priority_queue<std::pair<uint64_t, uint64_t>, std::vector<std::pair<uint64_t, uint64_t>>,
                            std::greater<>> h;
        for (uint64_t i = 0; i < leaves; i++) h.push({f[used[i]], i});
        while (h.size() > 1) {
            auto a = h.top();
            h.pop();
            auto b = h.top();
            h.pop();
            kids.push_back({a.second, b.second, 0});
            h.push({a.first + b.first, leaves + kids.size() - 1});
        }
        std::vector<uint64_t> depth(leaves + kids.size(), 0);
        for (uint64_t u = leaves + kids.size(); u-- > leaves;) {  // parents before children
            depth[kids[u - leaves][0]] = depth[u] + 1;
            depth[kids[u - leaves][1]] = depth[u] + 1;
        }
        // clip to MAXL, repair the Kraft sum from the longest non-empty length < MAXL
        std::array<uint64_t, MAXL + 2> bl{};
        for (uint64_t i = 0; i < leaves; i++) bl[std::min<uint64_t>(std::max<uint64_t>(1, depth[i]), MAXL)]++;
        uint64_t kraft = 0;
        for (uint32_t l = 1; l <= MAXL; l++) kraft += bl[l] << (MAXL - l);
        while (kraft > (1ull << MAXL)) {
            uint32_t l = MAXL - 1;
            while (l >= 1 && bl[l] == 0) l--;
            bl[l]--;
            bl[l + 1]++;
            kraft -= 1ull << (MAXL - l - 1);
        }
        // longest lengths to the rarest symbols (std::sort: the reference's tie order)
        std::sort(used.begin(), used.end(), [&](uint64_t a, uint64_t b) { return f[a] < f[b]; });
        uint64_t k = 0;
        for (uint32_t l = MAXL; l >= 1; l--)
            for (uint64_t j = 0; j < bl[l]; j++) c.len[used[k++]] = l;
    }
    canonical(c);
    return c;
}
void elias(bits_out& o, uint64_t x) {
    const uint32_t lx = bw(x), ll = bw(lx);
    o.put(0, ll - 1);
    o.put(lx, ll);
    o.put(x, lx - 1);
}

}  // namespace

extern "C" int64_t oracle_huffman(const uint32_t* F, uint64_t z, uint64_t n, uint8_t* out, uint64_t cap) {
    bits_out o;
    uint64_t pos = 0;
    for (uint64_t b0 = 0; b0 < z; b0 += BLK) {
        const uint64_t b1 = std::min<uint64_t>(z, b0 + BLK);
        std::vector<std::pair<uint64_t, uint64_t>> e;  // (val, len)
        for (uint64_t r = b0; r < b1; r++) {
            const uint32_t src = F[2 * r], len = F[2 * r + 1];
            if (len == 0) e.push_back({src & 255u, 0}), pos += 1;
            else e.push_back({pos - src, len}), pos += len;
        }
        std::array<uint64_t, SIG> hl{}, hd{};
        for (auto& x : e) {
            hl[x.second ? bw(x.second) : 0]++;
            if (x.second) hd[bw(x.first)]++;
        }
        const code_t L = build(hl), D = build(hd);
        elias(o, e.size());
        for (uint32_t s = 0; s < SIG; s++) o.put(L.len[s], 4);
        for (uint32_t s = 0; s < SIG; s++) o.put(D.len[s], 4);
        for (auto& x : e) {
            const uint32_t lb = x.second ? bw(x.second) : 0;
            o.put(L.code[lb], L.len[lb]);
            if (!lb) {
                o.put(x.first, 8);
            } else {
                o.put(x.second, lb - 1);
                const uint32_t db = bw(x.first);
                o.put(D.code[db], D.len[db]);
                o.put(x.first, db - 1);
            }
        }
    }
    const uint64_t total = 5 + o.b.size();
    if (out && cap >= total) {
        for (int k = 0; k < 5; k++) out[k] = (uint8_t)(n >> (8 * k));
        if (!o.b.empty()) std::memcpy(out + 5, o.b.data(), o.b.size());
    }
    return (int64_t)total;
}

// decoder: factors (src, len) from the container; returns the factor count or -1
extern "C" int64_t oracle_huffman_decode(const uint8_t* in, uint64_t nbytes, uint32_t* F, uint64_t cap) {
    if (nbytes < 5) return -1;
    uint64_t n = 0;
    for (int k = 0; k < 5; k++) n |= (uint64_t)in[k] << (8 * k);
    bits_in r{in + 5, nbytes - 5};
    uint64_t pos = 0, z = 0;
    while (pos < n) {
        uint64_t zeros = 0;
        while (r.get(1) == 0) {
            if (++zeros > 64) return -1;
        }
        const uint64_t lx = (1ull << zeros) | r.get((uint32_t)zeros);
        const uint64_t cnt = lx <= 1 ? lx : ((1ull << (lx - 1)) | r.get((uint32_t)(lx - 1)));
        code_t L, D;
        for (uint32_t s = 0; s < SIG; s++) L.len[s] = (uint32_t)r.get(4);
        for (uint32_t s = 0; s < SIG; s++) D.len[s] = (uint32_t)r.get(4);
        canonical(L);
        canonical(D);
        auto sym = [&](const code_t& c) -> int64_t {
            uint64_t v = 0;
            for (uint32_t l = 1; l <= MAXL; l++) {
                v = (v << 1) | r.get(1);
                for (uint32_t s = 0; s < SIG; s++)
                    if (c.len[s] == l && c.code[s] == v) return s;
            }
            return -1;
        };
        for (uint64_t k = 0; k < cnt && pos < n; k++) {
            const int64_t lb = sym(L);
            if (lb < 0 || z >= cap) return -1;
            if (lb == 0) {
                F[2 * z] = (uint32_t)r.get(8);
                F[2 * z + 1] = 0;
                pos += 1;
            } else {
                const uint64_t len = (1ull << (lb - 1)) | r.get((uint32_t)(lb - 1));
                const int64_t db = sym(D);
                if (db <= 0) return -1;
                const uint64_t dist = (1ull << (db - 1)) | r.get((uint32_t)(db - 1));
                F[2 * z] = (uint32_t)(pos - dist);
                F[2 * z + 1] = (uint32_t)len;
                pos += len;
            }
            z++;
        }
    }
    return (int64_t)z;
}
