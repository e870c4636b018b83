// huffman.hip -- the Huffman factor container of the encoder CLIs (role of
// huff_writer, include/lz77_sss/misc/huffman.hpp:318-375, used by
// cli/lz77_sss_3_aprx.cpp:71-85) built from the factors in HBM.
//
// Container: 5 bytes n (little endian), then one MSB-first bit stream.  Factors
// are cut into blocks of 2^14; factor f at text position i is the entry
// (val, len) = (byte, 0) for a literal, (i - src, len) otherwise.  Per block:
// Elias-delta(#entries), two 66-symbol code-length tables (4 bits each) for the
// length classes lb = bit_width(len) (0 = literal) and distance classes
// db = bit_width(val), then per entry code(lb) + (literal: 8-bit byte |
// len without its top bit + code(db) + val without its top bit).  Code lengths are
// length-limited (15) Huffman lengths with canonical codes (huffman.hpp:177-300).
//
// Device: entry classes and per-block class histograms (one workgroup per block,
// LDS counters); host: the 2 x 66-symbol codes of every block (a few hundred
// symbols of work per block); device: bit length of every entry, a scan for the
// bit offsets, and every entry ORs its fields into the big-endian 32-bit words it
// spans (fields are <= 32 bits: at most two words).
#include "../../include/lz77sss.h"
#include "../include/engine.h"
#include "../include/prim.h"

#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <array>
#include <queue>

namespace lz {

constexpr u32 HF_SIGMA = 66;
constexpr u32 HF_BLOCK = 1u << 14;
constexpr u32 HF_MAXLEN = 15;

__device__ __forceinline__ u32 bitw(u64 x) { return x ? 64u - (u32)__builtin_clzll(x) : 0u; }

// per entry: val, class lb, class db, text position (pos scan below)
__global__ void k_hf_adv(const u32* __restrict__ F, u64 z, u64* __restrict__ adv) {
    const u64 r = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (r < z) adv[r] = F[2 * r + 1] ? F[2 * r + 1] : 1u;
}
// one workgroup per block: class histograms
__global__ __launch_bounds__(256) void k_hf_hist(const u32* __restrict__ F, u64 z, const u64* __restrict__ pos,
                                                 u32* __restrict__ hist) {
    __shared__ u32 h[2 * HF_SIGMA];
    const u64 b = blockIdx.x;
    for (u32 k = threadIdx.x; k < 2 * HF_SIGMA; k += 256) h[k] = 0;
    __syncthreads();
    const u64 r0 = b * HF_BLOCK, r1 = min<u64>(z, r0 + HF_BLOCK);
    for (u64 r = r0 + threadIdx.x; r < r1; r += 256) {
        const u32 len = F[2 * r + 1];
        if (len == 0) {
            atomicAdd(&h[0], 1u);
        } else {
            atomicAdd(&h[bitw(len)], 1u);
            atomicAdd(&h[HF_SIGMA + bitw(pos[r] - F[2 * r])], 1u);
        }
    }
    __syncthreads();
    for (u32 k = threadIdx.x; k < 2 * HF_SIGMA; k += 256) hist[b * 2 * HF_SIGMA + k] = h[k];
}
struct hf_tab {  // per block: [lenclass code | dist code] lengths and codes
    u8 ll[HF_SIGMA], dl[HF_SIGMA];
    u32 lc[HF_SIGMA], dc[HF_SIGMA];
    u32 hdr_bits;  // Elias delta + the two tables
    u32 nent;
};
__global__ void k_hf_bits(const u32* __restrict__ F, u64 z, const u64* __restrict__ pos, const hf_tab* __restrict__ tab,
                          u64* __restrict__ bits) {
    const u64 r = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= z) return;
    const hf_tab& t = tab[r / HF_BLOCK];
    const u32 len = F[2 * r + 1];
    u64 b = (r % HF_BLOCK == 0) ? t.hdr_bits : 0;
    if (len == 0) {
        b += t.ll[0] + 8;
    } else {
        const u32 lb = bitw(len), db = bitw(pos[r] - F[2 * r]);
        b += t.ll[lb] + (lb - 1) + t.dl[db] + (db - 1);
    }
    bits[r] = b;
}
// OR v (nb <= 32 bits, MSB first) into the big-endian bit stream at bit offset o
__device__ __forceinline__ void hf_put(u32* w, u64 o, u32 v, u32 nb) {
    if (!nb) return;
    const u64 x = ((u64)(nb == 32 ? v : (v & ((1u << nb) - 1u)))) << (64 - nb - (o & 31));
    atomicOr(&w[o >> 5], (u32)(x >> 32));
    if ((u32)x) atomicOr(&w[(o >> 5) + 1], (u32)x);
}
__device__ __forceinline__ u64 hf_elias(u32* w, u64 o, u64 x) {
    const u32 lx = bitw(x), ll = bitw(lx);
    hf_put(w, o, 0, ll - 1);
    o += ll - 1;
    hf_put(w, o, lx, ll);
    o += ll;
    hf_put(w, o, (u32)x, lx - 1);
    return o + lx - 1;
}
__global__ void k_hf_write(const u32* __restrict__ F, u64 z, const u64* __restrict__ pos, const hf_tab* __restrict__ tab,
                           const u64* __restrict__ off, u32* __restrict__ words) {
    const u64 r = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= z) return;
    const hf_tab& t = tab[r / HF_BLOCK];
    u64 o = off[r];
    if (r % HF_BLOCK == 0) {
        o = hf_elias(words, o, t.nent);
        for (u32 s = 0; s < HF_SIGMA; s++, o += 4) hf_put(words, o, t.ll[s], 4);
        for (u32 s = 0; s < HF_SIGMA; s++, o += 4) hf_put(words, o, t.dl[s], 4);
    }
    const u32 src = F[2 * r], len = F[2 * r + 1];
    if (len == 0) {
        hf_put(words, o, t.lc[0], t.ll[0]);
        hf_put(words, o + t.ll[0], src & 255u, 8);
        return;
    }
    const u64 val = pos[r] - src;
    const u32 lb = bitw(len), db = bitw(val);
    hf_put(words, o, t.lc[lb], t.ll[lb]);
    o += t.ll[lb];
    hf_put(words, o, len, lb - 1);
    o += lb - 1;
    hf_put(words, o, t.dc[db], t.dl[db]);
    o += t.dl[db];
    hf_put(words, o, (u32)val, db - 1);
}
__global__ void k_hf_bytes(const u32* __restrict__ words, u64 nbytes, u64 n, u8* __restrict__ out) {
    const u64 k = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (k < 5) out[k] = (u8)(n >> (8 * k));
    if (k < nbytes) out[5 + k] = (u8)(words[k >> 2] >> (8 * (3 - (k & 3))));
}

// ---- host: length-limited Huffman lengths + canonical codes of one alphabet
// (huffman.hpp:177-300: depths from a min-heap on (weight, node), lengths clipped at
// 15 and repaired to the Kraft bound from the longest side, then re-assigned by
// ascending frequency from the longest length down; canonical codes by length, then
// symbol)
static void hf_code(const u32* freq, u8* len, u32* code) {
    std::vector<u32> used;
    for (u32 s = 0; s < HF_SIGMA; s++) {
        len[s] = 0;
        code[s] = 0;
        if (freq[s]) used.push_back(s);
    }
    if (used.size() == 1) len[used[0]] = 1;
    if (used.size() > 1) {
        struct node { u64 w; u32 l, r, sym; };
        const u32 none = ~0u;
        std::vector<node> nd;
        using item = std::pair<u64, u64>;
        std::priority_queue<item, std::vector<item>, std::greater<item>> pq;
        for (u32 s : used) {
            nd.push_back({freq[s], none, none, s});
            pq.push({freq[s], nd.size() - 1});
        }
        while (pq.size() > 1) {
            const item a = pq.top();
            pq.pop();
            const item b = pq.top();
            pq.pop();
            nd.push_back({a.first + b.first, (u32)a.second, (u32)b.second, none});
            pq.push({a.first + b.first, nd.size() - 1});
        }
        std::array<u32, HF_SIGMA> depth{};
        std::vector<std::pair<u32, u32>> stk{{(u32)pq.top().second, 0u}};
        while (!stk.empty()) {
            const auto [u, d] = stk.back();
            stk.pop_back();
            if (nd[u].sym != none) {
                depth[nd[u].sym] = std::max(1u, d);
            } else {
                stk.push_back({nd[u].l, d + 1});
                stk.push_back({nd[u].r, d + 1});
            }
        }
        std::array<u64, HF_MAXLEN + 2> bl{};
        for (u32 s : used) bl[std::min(depth[s], HF_MAXLEN)]++;
        u64 kraft = 0;
        for (u32 l = 1; l <= HF_MAXLEN; l++) kraft += bl[l] << (HF_MAXLEN - l);
        while (kraft > (1ull << HF_MAXLEN)) {
            u32 l = HF_MAXLEN - 1;
            while (l >= 1 && bl[l] == 0) l--;
            bl[l]--;
            bl[l + 1]++;
            kraft -= 1ull << (HF_MAXLEN - l - 1);
        }
        std::sort(used.begin(), used.end(), [&](u32 a, u32 b) { return freq[a] < freq[b]; });
        u32 idx = 0;
        for (u32 l = HF_MAXLEN; l >= 1; l--)
            for (u64 k = 0; k < bl[l]; k++) len[used[idx++]] = (u8)l;
    }
    std::array<u32, HF_MAXLEN + 1> cnt{}, next{};
    for (u32 s = 0; s < HF_SIGMA; s++)
        if (len[s]) cnt[len[s]]++;
    u32 c = 0;
    for (u32 l = 1; l <= HF_MAXLEN; l++) {
        c = (c + cnt[l - 1]) << 1;
        next[l] = c;
    }
    for (u32 s = 0; s < HF_SIGMA; s++)
        if (len[s]) code[s] = next[len[s]]++;
}
static u32 bitw_host(u64 x) { return x ? 64u - (u32)__builtin_clzll(x) : 0u; }

u64 engine::huffman_container() {
    const u64 z = num_fact;
    const u32* F = fact.p;
    const u64 nblk = (z + HF_BLOCK - 1) / HF_BLOCK;
    const unsigned g = cdiv(z, 256);
    u64* adv = x_off.get(3 * (z + 1));
    u64* pos = adv + (z + 1);
    u64* off = pos + (z + 1);
    u64* bits = x_wide.get(z + 1);
    u64 total_bits = 0;
    std::vector<hf_tab> ht(std::max<u64>(1, nblk));
    if (z) {
        k_hf_adv<<<g, 256, 0, st>>>(F, z, adv);
        excl_sum64(adv, pos, (u64)0, z, scan_tmp, st);
        u32* hist = x_idx.get(nblk * 2 * HF_SIGMA);
        k_hf_hist<<<(unsigned)nblk, 256, 0, st>>>(F, z, pos, hist);
        std::vector<u32> hh(nblk * 2 * HF_SIGMA);
        LZ_HIP(hipMemcpyAsync(hh.data(), hist, hh.size() * 4, hipMemcpyDeviceToHost, st));
        LZ_HIP(hipStreamSynchronize(st));
        for (u64 b = 0; b < nblk; b++) {
            hf_tab& T = ht[b];
            hf_code(&hh[b * 2 * HF_SIGMA], T.ll, T.lc);
            hf_code(&hh[b * 2 * HF_SIGMA + HF_SIGMA], T.dl, T.dc);
            T.nent = (u32)std::min<u64>(HF_BLOCK, z - b * HF_BLOCK);
            const u32 lx = bitw_host(T.nent), ll = bitw_host(lx);
            T.hdr_bits = (ll - 1) + ll + (lx - 1) + 2 * 4 * HF_SIGMA;
        }
        hf_tab* dt = (hf_tab*)hf_tabs.get(nblk * sizeof(hf_tab));
        LZ_HIP(hipMemcpyAsync(dt, ht.data(), nblk * sizeof(hf_tab), hipMemcpyHostToDevice, st));
        k_hf_bits<<<g, 256, 0, st>>>(F, z, pos, dt, bits);
        LZ_HIP(hipMemsetAsync(bits + z, 0, 8, st));
        excl_sum64(bits, off, (u64)0, z + 1, scan_tmp, st);
        total_bits = rd1(off + z, st);
        const u64 nw = total_bits / 32 + 2;
        u32* words = (u32*)hf_words.get(nw * 4);
        LZ_HIP(hipMemsetAsync(words, 0, nw * 4, st));
        k_hf_write<<<g, 256, 0, st>>>(F, z, pos, dt, off, words);
        LZ_HIP(hipStreamSynchronize(st));  // dt / ht stay valid until here
    }
    const u64 nbytes = (total_bits + 7) / 8;
    u8* out = hf_out.get(nbytes + 5);
    const u32* words = z ? (const u32*)hf_words.p : nullptr;
    k_hf_bytes<<<cdiv(std::max<u64>(nbytes, 5), 256), 256, 0, st>>>(words, nbytes, n, out);
    LZ_HIP(hipGetLastError());
    LZ_HIP(hipStreamSynchronize(st));
    return nbytes + 5;
}

}  // namespace lz
