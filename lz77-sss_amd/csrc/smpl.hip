// smpl.hip -- exact LZ77 through a sample index on the device: the exact-smpl path of
// configs[4] (lz77_sss<>::factorizer::exact_factorizer, include/lz77_sss/lz77_sss.hpp:558-709;
// transform_to_exact/{common,naive,without_samples,with_samples}.cpp; the sample index of
// data_structures/sample_index/{sample_index.hpp,construction.cpp,queries.cpp}; the
// decomposed static weighted square grid of decomposed_range.hpp and
// static_weighted_range/static_weighted_square_grid.hpp).
//
// Pipeline, everything resident in HBM:
//   approx   the 3-approximation (greedy + lpf_opt, engine::factorize); its factors
//            are kept for the lower bounds of without_samples / with_samples
//   C        samples: 0, the last position of every approximate phrase and every
//            delta-th position inside it, delta = min(n / z, 256) (common.cpp:34-88,
//            lz77_sss.hpp:326); consecutive samples are at most delta apart
//   PA, SA   sample ids by left context (at most delta + 1 characters, lce_l_64
//            semantics) and by suffix (sample_index.hpp:317-353): a radix sort by a
//            64-bit key packing as many characters as the text's alphabet allows, then a
//            comparison merge sort whose comparator falls back to the text (leftward LCE /
//            the SSS-backed LCE of lce_dev.h)
//   points   (x = PA rank, y = SA rank, weight = sample id); Pi, Psi (common.cpp:114-182)
//   grid     per first character (decomposed_range.hpp:82-130) cells of >= SG_WIN ranks per side
//            ranks, points sorted by (cell, weight) (static_weighted_square_grid.hpp:67-104)
//   orders   per order (PA, SA): 16-byte context keys by rank, the adjacent LCEs
//            (construction.cpp:118-129) with sparse-table minima, and sparse-table minima
//            of the weights.  They replace with_samples' interval samples
//            (construction.cpp:108-305): any interval of any pattern length comes from one
//            insertion rank by binary lifting, and the nearest lighter samples in SA order
//            bound every right extension
//   phrases  one wave per phrase start i; lane j in [i, i + delta) finds the PA interval
//            of T[i..j] (extend_left, queries.cpp:67-275) and the longest right extension
//            lce_r whose SA interval holds a point lighter than the first sample >= j
//            (intersect, common.cpp:258-358: the lightest point of either interval on the
//            lane, else the Pi / Psi scan below SCAN_T ranks or the grid, for the whole wave
//            one query at a time); the wave keeps the longest, the smallest j on ties
//   chain    chunk walks: one wave per chunk of SMPL_CHUNK approximate phrases walks the
//            greedy chain from the chunk's first phrase start (a task per phrase, in a hash
//            table) until it meets another walk's task or passes its chunk end; bridges walk on
//            from every chunk exit until they meet a task; the chain from position 0 is then
//            marked in order by pointer doubling + top-down expansion over the successor tasks
//
// Lengths are the canonical greedy LZ77 lengths (every leftmost occurrence of a phrase
// contains a sample within its first delta characters: DESIGN.md 4.8); the three transform
// modes give the same lengths (naive skips the approximate lower bound).  Sources are the
// lighter points found, not the reference's visit order (whose PA / SA tie order comes from
// an unstable parallel sort).
#include "../../include/lz77sss.h"
#include "../include/engine.h"
#include "../include/msort_dev.h"

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <vector>

#include <hipcub/hipcub.hpp>

namespace LZ_NS {

// LZ_SMPL_CHECK (debug builds only, tools/build_check.sh): every array index of the phrase
// searches and walks is checked against its array's size; the first violation is recorded in
// g_smpl_chk (site, index, limit) and the index replaced by 0, so the kernel completes and the
// host prints the site
#ifdef LZ_SMPL_CHECK
__device__ u32* g_smpl_chk;
__device__ u64 g_smpl_lim[8];  // c, ncell, nblk, za, n + pad, hash slots, task capacity, ncell2
__device__ __forceinline__ u64 smpl_ck(u64 idx, u64 lim, u32 site) {
    if (idx < lim) return idx;
    u32* ck = g_smpl_chk;
    if (ck && atomicCAS(ck, 0u, site) == 0u) {
        ck[1] = (u32)idx;
        ck[2] = (u32)(idx >> 32);
        ck[3] = (u32)lim;
        ck[4] = (u32)(lim >> 32);
    }
    return 0;
}
#define CK(idx, lim, site) smpl_ck((u64)(idx), (u64)(lim), (site))
#define LIM(k) g_smpl_lim[k]
// every phase synchronised and named on stderr: a fault then names its phase
#define SMPL_STAGE(name)                                                                    \
    do {                                                                                    \
        const hipError_t e_ = hipStreamSynchronize(st);                                     \
        std::fprintf(stderr, "[lz77sss] smpl stage %s: %s\n", name, hipGetErrorString(e_)); \
        LZ_HIP(e_);                                                                         \
    } while (0)
#else
#define CK(idx, lim, site) (idx)
#define LIM(k) 0
#define SMPL_STAGE(name) ((void)0)
#endif

constexpr u32 SMPL_MAX_DELTA = 256;  // lz77_sss.hpp:81 max_delta
constexpr u32 SCAN_T = 1024;         // lz77_sss.hpp:83 range_scan_threshold (4096 on a CPU core)
constexpr u32 SMALL_T = 32;          // intersect queries scanned by their own lane (no wave round trip)
#ifndef LZ_SG_WIN
#define LZ_SG_WIN 2048
#endif
constexpr u32 SG_WIN = LZ_SG_WIN;    // smallest grid cell width in ranks (the reference: 16384 on a CPU core)
constexpr u32 SG_GMAX = 512;         // cells per side at most: wider blocks get wider cells
constexpr u32 RST_MAX = 18;          // row sparse-table levels at most (2^17 cells per side)
constexpr u32 RG_WIN = 16384;        // the reference's window width (static_weighted_square_grid.hpp:69)
constexpr u32 RG_SCAN = 4096;        // the reference's range_scan_threshold (lz77_sss.hpp:85)
constexpr u32 SWPB = 4;              // waves per workgroup of the phrase kernels
#ifndef SMPL_OCC
#define SMPL_OCC 6                   // waves per SIMD the walk kernels are register-bounded for: the walks
                                     // are bound by L2-miss traffic, more waves in flight beat the spills
                                     // (genome 1 GiB k_chunk_walks: 4 -> 981 ms, 5 -> 922, 6 -> 832, 7 -> 860,
                                     // 8 -> 883)
#endif
constexpr u32 SMPL_CHUNK = 1024;     // approximate phrases per chunk walk at most
constexpr u32 SMPL_WALKS = 16384;    // chunk walks wanted

// ---------------------------------------------------------------------------
// rank intervals of an order by its adjacent LCEs (mn[0][r] = LCE of ranks r - 1, r) and their
// sparse-table minima (mn[l][i] = min adj[i .. i + 2^l)): an interval's ends by binary lifting
// (iv_around); a linear scan took seconds on repetitive text, where one interval spans millions
// of samples
struct iv_levels { const u32* mn[MAX_LV]; u32 nlv; };

// ---------------------------------------------------------------------------
// device view
struct smpl_view {
    lce_view L;
    const u32* C;            // samples (increasing)
    u32 c;
    u32 delta;
    const u32* PA;           // sample id by PA rank
    const u32* SA;           // sample id by SA rank
    const u32* Pi;           // SA rank of PA rank x
    const u32* Psi;          // PA rank of SA rank y
    const u32* CS;           // [257] first rank per first character
    const u32* gcb;          // [257] first cell per character
    const u32* gwd;          // [256] grid width per character (cells per side)
    const u32* gwin;         // [256] cell width in ranks per character
    const u32* cell;         // [ncells + 1] first point per cell
    const u32* rst[RST_MAX]; // per row of cells: min weight over cells [x, x + 2^k) of the row
    const u32* gx;           // points by (cell, weight): PA rank, SA rank, weight
    const u32* gy;
    const u32* gw;
    const u32* afst;         // approximate phrase starts [za + 1]
    const u32* afact;        // approximate factors (src, len)
    u32 za;
    int mode;                // LZ77SSS_TRANSF_*
    u32 small_t;             // intersect queries with a side of at most this many ranks run on their own lane
    u32 scan_t;              // the wave scans a side of at most this many ranks (else the grid)
    u32 lane_scan;           // a lane scans PA intervals of fewer ranks for the answer
    iv_levels sM;            // SA order: adjacent sample-suffix LCEs (sM.mn[0][r] = LCE of ranks r - 1, r) and their
                             // sparse-table minima; the SA interval of any right extension by binary lifting
    iv_levels pM;            // PA order: the same over the left contexts (capped at delta)
    const u32* PAR;          // PA / SA rank of a sample id
    const u32* SAR;
    const u32* wPA[MAX_LV];  // sparse-table minima of the weights (sample ids) by PA rank: min PA[x .. x + 2^k)
    const u32* wSA[MAX_LV];  // the same by SA rank (level 0: PA / SA themselves)
    u32 wlv;                 // levels
    const u32* pre[2];       // PA / SA: the first rank per value of a context's first 16 key bits [65537]
    const u8* code;          // the characters' codes in the sort keys
    u32 kbits_ch;            // bits per character in the sort keys
    u32 kc[2];               // characters per sort key (PA, SA)
    const u32* wblk;         // the first sample index x with C[x] >= 256 b, per 256-position block b
    const ulonglong2* kSA;   // context keys by SA rank (key_right) and by PA rank (key_left)
    const ulonglong2* kPA;
    unsigned long long* cyc;  // debug (LZ77SSS_SMPL_PROF): per-section clock and query counters, or null
    u32 prof_split;           // debug: phrases before / after this position counted apart
};

// ---- comparisons of a pattern (text position pp) with sample contexts -----------------
// left: T[pp - len + 1 .. pp] against the context ending at pm; the LCE starts from a
// known lower bound offs (queries.cpp lce_offs); returns the LCE (capped at len)
__device__ __forceinline__ u32 lce_left_offs(const smpl_view& V, u32 pm, u32 pp, u32 offs, u32 len) {
    if (min(pm, pp) < offs) return offs;
    return offs + (u32)dev_lce_left(V.L.T, V.L.R, pm - offs, pp - offs, len - offs);
}
// cmp_lex<LEFT>(pm, pp, l) (sample_index.hpp:256-267): the sample context sorts first
__device__ __forceinline__ bool less_left(const smpl_view& V, u32 pm, u32 pp, u32 l) {
    if (pm == pp) return false;
    if (l > min(pm, pp)) return pm < pp;
    return V.L.T[pm - l] < V.L.T[pp - l];
}
__device__ __forceinline__ u32 lce_right_offs(const smpl_view& V, u32 pm, u32 pp, u32 offs) {
    if ((u64)max(pm, pp) + offs >= V.L.n) return offs;
    if (pm == pp) return (u32)(V.L.n - pp);
    return offs + (u32)dev_lce(V.L, (u64)pm + offs, (u64)pp + offs);
}
__device__ __forceinline__ bool less_right(const smpl_view& V, u32 pm, u32 pp, u32 l) {
    if (pm == pp) return false;
    if ((u64)max(pm, pp) + l >= V.L.n) return pm > pp;
    return V.L.T[(u64)pm + l] < V.L.T[(u64)pp + l];
}

// ---- intersect (common.cpp:258-358), one query of the wave at a time -----------------
// For every lane with q: is there a point with x in [xb, xe], y in [yb, ye] and weight < W?
// (all ranks inside the block of first character ch).  py = its SA rank.
__device__ void wave_intersect(const smpl_view& V, bool q, u32 xb, u32 xe, u32 yb, u32 ye, u32 W, u32 ch, bool& found,
                               u32& py, u32 lane) {
    found = false;
    // queries with a small side (at most SMALL_T ranks) scan it on their own lane, in the order
    // the cooperative scan below uses (ascending ranks of the smaller side: the same point)
    bool qq = q;
    if (q && V.mode != LZ77SSS_TRANSF_NAIVE) {
        const u32 rx = xe - xb + 1, ry = ye - yb + 1;
        if (min(rx, ry) <= V.small_t) {
            qq = false;
            if (rx <= ry) {
                for (u32 x = xb; x <= xe; x++) {
                    const u32 yy = V.Pi[CK(x, LIM(0), 1)];
                    if (V.PA[CK(x, LIM(0), 2)] < W && yy >= yb && yy <= ye) {
                        found = true;
                        py = yy;
                        break;
                    }
                }
            } else {
                for (u32 yy = yb; yy <= ye; yy++) {
                    const u32 xx = V.Psi[CK(yy, LIM(0), 3)];
                    if (V.SA[CK(yy, LIM(0), 4)] < W && xx >= xb && xx <= xe) {
                        found = true;
                        py = yy;
                        break;
                    }
                }
            }
        }
    }
    u64 pend = __ballot(qq);
    while (pend) {
        const int L = __builtin_ctzll(pend);
        pend &= pend - 1;
        const u32 qxb = __builtin_amdgcn_readlane(xb, L), qxe = __builtin_amdgcn_readlane(xe, L);
        const u32 qyb = __builtin_amdgcn_readlane(yb, L), qye = __builtin_amdgcn_readlane(ye, L);
        const u32 qW = __builtin_amdgcn_readlane(W, L), qch = __builtin_amdgcn_readlane(ch, L);
        bool f = false;
        u32 y = 0;
        const u32 rx = qxe - qxb + 1, ry = qye - qyb + 1;
        if (V.mode != LZ77SSS_TRANSF_NAIVE && min(rx, ry) <= V.scan_t) {
            // scan the smaller interval through Pi / Psi
            if (rx <= ry) {
                for (u32 base = qxb; base <= qxe; base += 64) {
                    const u32 x = base + lane;
                    u32 yy = 0;
                    bool ok = false;
                    if (x <= qxe) {
                        yy = V.Pi[CK(x, LIM(0), 5)];
                        ok = V.PA[CK(x, LIM(0), 6)] < qW && yy >= qyb && yy <= qye;
                    }
                    const u64 bal = __ballot(ok);
                    if (bal) {
                        f = true;
                        y = __builtin_amdgcn_readlane(yy, __builtin_ctzll(bal));
                        break;
                    }
                }
            } else {
                for (u32 base = qyb; base <= qye; base += 64) {
                    const u32 yy = base + lane;
                    bool ok = false;
                    if (yy <= qye) {
                        const u32 xx = V.Psi[CK(yy, LIM(0), 3)];
                        ok = V.SA[CK(yy, LIM(0), 7)] < qW && xx >= qxb && xx <= qxe;
                    }
                    const u64 bal = __ballot(ok);
                    if (bal) {
                        f = true;
                        y = base + (u32)__builtin_ctzll(bal);
                        break;
                    }
                }
            }
        } else {
            // the grid of character qch (static_weighted_square_grid.hpp:116-185): the contained
            // cells through row sparse tables of their lightest weights (a lane per row), the
            // border cells a lane each (their points in weight order up to the first heavy one)
            const u32 r0 = V.CS[qch], gw = V.gwd[qch], cb = V.gcb[qch], win = V.gwin[qch];
            const u32 x1 = qxb - r0, x2 = qxe - r0, y1 = qyb - r0, y2 = qye - r0;
            const u32 xw1 = x1 / win, xw2 = x2 / win, yw1 = y1 / win, yw2 = y2 / win;
            const u32 xi1 = xw1 + (x1 % win != 0), yi1 = yw1 + (y1 % win != 0);
            const u32 xi2 = xw2 + (x2 % win == win - 1), yi2 = yw2 + (y2 % win == win - 1);
            const bool inner = xi1 < xi2 && yi1 < yi2;
            if (inner) {
                const u32 wx = xi2 - xi1, k = 31 - __builtin_clz(wx);
                const u32* R = V.rst[k];
                for (u32 base = yi1; base < yi2 && !f; base += 64) {
                    const u32 row = base + lane;
                    bool ok = false;
                    if (row < yi2) {
                        const u32 o = cb + row * gw;
                        ok = min(R[CK(o + xi1, LIM(1) + 1, 8)], R[CK(o + xi2 - (1u << k), LIM(1) + 1, 9)]) < qW;
                    }
                    const u64 bal = __ballot(ok);
                    if (bal) {
                        // the row's first cell with a lighter point: its lightest point
                        const u32 row1 = base + (u32)__builtin_ctzll(bal), o = cb + row1 * gw;
                        for (u32 xb = xi1; xb < xi2; xb += 64) {
                            const u32 cx = xb + lane;
                            const bool hit = cx < xi2 && V.rst[0][CK(o + cx, LIM(1) + 1, 10)] < qW;
                            const u64 hb = __ballot(hit);
                            if (hb) {
                                const u32 cid = o + xb + (u32)__builtin_ctzll(hb);
                                y = V.gy[CK(V.cell[CK(cid, LIM(1) + 1, 11)], LIM(0), 12)];
                                f = true;
                                break;
                            }
                        }
                    }
                }
            }
            if (!f) {
                // border cells in the reference's row-major order (the first cell in it with a
                // point decides which point answers): the full row yw1 (< yi1), the cells xw1
                // (< xi1) and xw2 (>= xi2) of each inner row, the full row yw2 (>= yi2); every
                // cell row by row when there is no inner part
                const u32 nx = xw2 - xw1 + 1, ny = yw2 - yw1 + 1;
                const bool full = !inner;
                const u32 top = full ? ny : (yw1 < yi1 ? 1u : 0u), bot = full ? 0u : (yw2 >= yi2 ? 1u : 0u);
                const u32 lc = (!full && xw1 < xi1) ? 1u : 0u, rc = (!full && xw2 >= xi2) ? 1u : 0u;
                const u32 nin = full ? 0u : yi2 - yi1, sides = lc + rc;
                const u32 ntop = top * nx, nmid = sides * nin, nb = ntop + nmid + bot * nx;
                for (u32 base = 0; base < nb && !f; base += 64) {
                    const u32 t = base + lane;
                    bool ok = false;
                    u32 yy = 0;
                    if (t < nb) {
                        u32 cx, cy;
                        if (t < ntop) {
                            cy = yw1 + t / nx;
                            cx = xw1 + t % nx;
                        } else if (t < ntop + nmid) {
                            const u32 u = t - ntop, s = u % sides;
                            cy = yi1 + u / sides;
                            cx = (lc && s == 0) ? xw1 : xw2;
                        } else {
                            cy = yw2;
                            cx = xw1 + (t - ntop - nmid);
                        }
                        const u32 cid = cb + cy * gw + cx;
                        const u32 p1 = V.cell[CK(cid + 1, LIM(1) + 1, 13)];
                        for (u32 q = V.cell[CK(cid, LIM(1) + 1, 14)]; q < p1; q++) {
                            if (V.gw[CK(q, LIM(0), 15)] >= qW) break;
                            const u32 xx = V.gx[CK(q, LIM(0), 16)], y3 = V.gy[CK(q, LIM(0), 16)];
                            if (xx >= qxb && xx <= qxe && y3 >= qyb && y3 <= qye) {
                                ok = true;
                                yy = y3;
                                break;
                            }
                        }
                    }
                    const u64 bal = __ballot(ok);
                    if (bal) {
                        f = true;
                        y = __builtin_amdgcn_readlane(yy, __builtin_ctzll(bal));
                    }
                }
            }
        }
        if ((int)lane == L) {
            found = f;
            py = y;
        }
    }
}

// ---- context keys ------------------------------------------------------------------------
// 15 context bytes and their count in 16: the right key of p holds T[p .. p + 15) (zero past n)
// big-endian in its top 15 bytes and min(n - p, 15) in its low byte; the left key T[p], T[p - 1],
// .., T[p - 14] (zero before 0) and min(p + 1, 15).  Two keys give the contexts' common prefix
// below 15 and their order (key_lcp / key_less_at), so most steps of an insertion search are
// one 16-byte load with no text access.
__device__ __forceinline__ ulonglong2 key_right(const u8* T, u64 n, u64 p) {
    ulonglong2 k;
    if (p + 16 <= n) {
        k.x = __builtin_bswap64(ldu64(T + p));
        k.y = (__builtin_bswap64(ldu64(T + p + 8)) & ~0xFFull) | 15u;
        return k;
    }
    u64 h = 0, l = 0;
    for (u32 t = 0; t < 15; t++) {
        const u64 b = p + t < n ? T[p + t] : 0u;
        if (t < 8) h |= b << (56 - 8 * t);
        else l |= b << (56 - 8 * (t - 8));
    }
    k.x = h;
    k.y = l | (n - p < 15 ? n - p : 15ull);
    return k;
}
__device__ __forceinline__ ulonglong2 key_left(const u8* T, u64 p) {
    ulonglong2 k;
    if (p >= 15) {
        k.x = ldu64(T + p - 7);                        // T[p] in the top byte .. T[p - 7]
        k.y = (ldu64(T + p - 15) & ~0xFFull) | 15u;    // T[p - 8] .. T[p - 14]
        return k;
    }
    u64 h = 0, l = 0;
    for (u32 t = 0; t < 15; t++) {
        const u64 b = t <= p ? T[p - t] : 0u;
        if (t < 8) h |= b << (56 - 8 * t);
        else l |= b << (56 - 8 * (t - 8));
    }
    k.x = h;
    k.y = l | (p + 1 < 15 ? p + 1 : 15ull);
    return k;
}
// the common prefix of the two contexts, or 15 when both hold 15 equal bytes (the rest unknown)
__device__ __forceinline__ u32 key_lcp(const ulonglong2& a, const ulonglong2& b) {
    const u64 x = a.x ^ b.x, y = (a.y ^ b.y) & ~0xFFull;
    const u32 d = x ? (u32)(__builtin_clzll(x) >> 3) : (y ? 8u + (u32)(__builtin_clzll(y) >> 3) : 15u);
    return min(d, (u32)min(a.y & 0xFF, b.y & 0xFF));
}
__device__ __forceinline__ u32 key_byte(const ulonglong2& a, u32 e) {
    return (u32)((e < 8 ? a.x >> (56 - 8 * e) : a.y >> (56 - 8 * (e - 8))) & 0xFF);
}
// context a sorts before b, given their common prefix e < 15: a shorter context is smaller
__device__ __forceinline__ bool key_less_at(const ulonglong2& a, const ulonglong2& b, u32 e) {
    const u32 ca = (u32)(a.y & 0xFF), cb = (u32)(b.y & 0xFF);
    if (e < ca && e < cb) return key_byte(a, e) < key_byte(b, e);
    return e == ca && e < cb;
}
__global__ void k_ctx_keys(const u8* __restrict__ T, u64 n, const u32* __restrict__ C, const u32* __restrict__ X, u32 c,
                           int left, ulonglong2* __restrict__ out) {
    const u64 r = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= c) return;
    const u32 pm = C[X[r]];
    out[r] = left ? key_left(T, pm) : key_right(T, n, pm);
}

// min of the adjacent LCEs over ranks [a, b] (a <= b)
__device__ __forceinline__ u32 adj_min(const iv_levels& M, u32 a, u32 b) {
    const u32 k = 31 - __builtin_clz(b - a + 1);
    return min(M.mn[k][CK(a, k ? LIM(0) - (1u << k) + 1 : LIM(0) + 1, 20)],
               M.mn[k][CK(b + 1 - (1u << k), k ? LIM(0) - (1u << k) + 1 : LIM(0) + 1, 21)]);
}
// LCE of the sample suffix at SA rank y with the suffix whose insertion rank is rs (LCEs hlo /
// hhi with ranks rs - 1 / rs)
__device__ __forceinline__ u32 lce_of_rank(const iv_levels& M, u32 y, u32 rs, u32 hlo, u32 hhi) {
    if (y < rs) return y + 1 == rs ? hlo : min(hlo, adj_min(M, y + 1, rs - 1));
    return y == rs ? hhi : min(hhi, adj_min(M, rs + 1, y));
}
// the lightest point (smallest sample id) with rank in [a, b] of an order (PA: V.wPA, SA: V.wSA)
__device__ __forceinline__ u32 min_weight(const u32* const* Wl, u32 a, u32 b) {
    const u32 k = 31 - __builtin_clz(b - a + 1);
    return min(Wl[k][CK(a, k ? LIM(0) - (1u << k) + 1 : LIM(0), 22)], Wl[k][CK(b + 1 - (1u << k), k ? LIM(0) - (1u << k) + 1 : LIM(0), 23)]);
}


// the rank interval [b, e] around insertion rank rs whose LCEs with the pattern are >= len
// (hlo / hhi: the LCEs of ranks rs - 1 / rs): the four adjacent LCEs either side first (most
// intervals of a phrase search are a few ranks wide), then binary lifting (iv_begin / iv_end),
// both ends' loads issued together
__device__ __forceinline__ void iv_around(const iv_levels& M, u32 c, u32 rs, u32 hlo, u32 hhi, u32 len, u32& b,
                                          u32& e) {
    const u32* a = M.mn[0];
    const bool db = hlo >= len, de = hhi >= len;  // the interval reaches below / above rs
    b = rs;
    e = rs - 1;
    u32 vb[4], ve[4];
#pragma unroll
    for (u32 t = 0; t < 4; t++) {
        vb[t] = db && t + 1 <= rs - 1 ? a[CK(rs - 1 - t, LIM(0) + 1, 24)] : 0u;  // adj[r] links ranks r - 1, r
        ve[t] = de && rs + 1 + t <= c ? a[CK(rs + 1 + t, LIM(0) + 1, 25)] : 0u;
    }
    bool lb = db, le = de;  // still extending
    if (db) b = rs - 1;
    if (de) e = rs;
#pragma unroll
    for (u32 t = 0; t < 4; t++) {
        if (lb) {
            if (vb[t] < len) lb = false;
            else b = rs - 2 - t;
        }
        if (le) {
            if (ve[t] < len) le = false;
            else e = rs + 1 + t;
        }
    }
    // b: adj[b + 1 .. rs - 1] >= len so far; e: adj[rs + 1 .. e] >= len so far
    for (int l = (int)M.nlv - 1; l >= 0 && (lb || le); l--) {
        const u32 w = 1u << l;
        const bool tb = lb && b >= w, te = le && e + 1 + w <= c;
        u32 x = 0, y = 0;
        if (tb) x = M.mn[l][CK(b + 1 - w, l ? LIM(0) - w + 1 : LIM(0) + 1, 26)];
        if (te) y = M.mn[l][CK(e + 1, l ? LIM(0) - w + 1 : LIM(0) + 1, 27)];
        if (tb && x >= len) b -= w;
        if (te && y >= len) e += w;
    }
}

// what is known about position j, whatever phrase it serves: the insertion ranks of its left
// context (PA, capped at delta) and of its suffix (SA) with the LCEs of their neighbours, the
// first sample W at or after j, and of the nearest SA ranks either side of rsR holding a sample
// lighter than W (the earlier sample suffixes sharing the most with the suffix at j) the one with
// the larger LCE uA (no earlier sample shares more)
struct pos_info {
    u32 rsL, hloL, hhiL;
    u32 rsR, hloR, hhiR;
    u32 w;
    u32 yA, uA;
};
__device__ __forceinline__ void key_step(const ulonglong2& km, const ulonglong2& kp, u32 D, bool left, u32& lm,
                                         bool& ls, bool& text) {
    const u32 el = key_lcp(km, kp);
    text = false;
    if (left && el >= D) {
        lm = D;
        ls = false;
    } else if (el < 15) {
        lm = el;
        ls = key_less_at(km, kp, el);
    } else {
        text = true;  // 15 equal bytes: the text decides
    }
}
// the range of first-16-bit values of the sort keys (k_smpl_keys: kc characters of `bits` bits)
// of the contexts that agree with the context at p on its first characters: all the key's
// characters in 16 bits, at most D of a left context (the comparator looks no further)
__device__ __forceinline__ void ctx_pre16(const smpl_view& V, u64 p, bool left, u32 D, u32& vlo, u32& vhi) {
    const u32 bits = V.kbits_ch, kc = left ? V.kc[0] : V.kc[1];
    const u32 q = min(kc, (16 + bits - 1) / bits), qa = left ? min(q, D) : q, qb = qa * bits;
    u32 v = 0;
    for (u32 t = 0; t < qa; t++) {
        u32 d;
        if (left) d = p >= (u64)t ? V.code[V.L.T[CK(p - t, LIM(4), 28)]] : 0u;
        else d = p + t < V.L.n ? V.code[V.L.T[CK(p + t, LIM(4), 29)]] : 0u;
        v = (v << bits) | d;
    }
    if (qb >= 16) {
        vlo = vhi = v >> (qb - 16);
    } else {
        vlo = v << (16 - qb);
        vhi = vlo | ((1u << (16 - qb)) - 1);
    }
}
// one comparison of an insertion search: the LCE lm of the context at rank m with the pattern
// (capped at D on the left) and whether it sorts below the pattern; keys first, the text past 15
// equal bytes (lower bound hb)
template <bool LEFT>
__device__ __forceinline__ void rank_cmp(const smpl_view& V, u32 j, u32 D, const ulonglong2& km, const ulonglong2& kp,
                                         u32 m, u32 hb, u32& lm, bool& ls) {
    bool text;
    key_step(km, kp, D, LEFT, lm, ls, text);
    if (text) {
        const u32 pm = V.C[CK((LEFT ? V.PA : V.SA)[CK(m, LIM(0), 30)], LIM(0), 31)];
        if (LEFT) {
            lm = lce_left_offs(V, pm, j, max(hb, 15u), D);
            ls = lm < D && less_left(V, pm, j, lm);
        } else {
            lm = lce_right_offs(V, pm, j, max(hb, 15u));
            ls = less_right(V, pm, j, lm);
        }
    }
}
// the three binary searches (PA / SA insertion ranks, W) advance together, one load each per
// step: the insertion searches inside the ranks of the pattern's first 16 key bits (V.pre), W
// inside the samples of j's 256-position block (V.wblk); then the two nearest-lighter searches
// together
template <bool PROF>
__device__ void pos_probe(const smpl_view& V, u32 j, u32 D, u32 cb, u32 ce, pos_info& P, u64* cy) {
    const u8* T = V.L.T;
    u64 t0 = PROF ? clock64() : 0;
    if constexpr (PROF) cy[13] += __popcll(__ballot(true));
    const ulonglong2 kpL = key_left(T, j), kpR = key_right(T, V.L.n, j);
    u32 vL0, vL1, vR0, vR1;
    ctx_pre16(V, j, true, D, vL0, vL1);
    ctx_pre16(V, j, false, 0, vR0, vR1);
    const u32 bL = V.pre[0][CK(vL0, 65537, 32)], eL = V.pre[0][CK(vL1 + 1, 65537, 33)], bR = V.pre[1][CK(vR0, 65537, 34)],
              eR = V.pre[1][CK(vR1 + 1, 65537, 35)];  // in [cb, ce]
    u32 lW = V.wblk[CK(j >> 8, LIM(2), 36)], hW = V.wblk[CK((j >> 8) + 1, LIM(2), 37)];
    // one rank more either side (inside the character's block): the search then compares the
    // pattern with both neighbours of its insertion rank, whose LCEs it returns
    u32 lL = bL > cb ? bL - 1 : bL, rL = eL < ce ? eL + 1 : eL, hlL = 1, hrL = 1;
    u32 lR = bR > cb ? bR - 1 : bR, rR = eR < ce ? eR + 1 : eR, hlR = 1, hrR = 1;
    P.hloL = P.hhiL = P.hloR = P.hhiR = 0;
    while (lL < rL || lR < rR || lW < hW) {
        const bool aL = lL < rL, aR = lR < rR, aW = lW < hW;
        const u32 mL = lL + (rL - lL) / 2, mR = lR + (rR - lR) / 2, mW = (lW + hW) >> 1;
        ulonglong2 kL = make_ulonglong2(0, 0), kR = make_ulonglong2(0, 0);
        u32 cW = 0;
        if (aL) kL = V.kPA[CK(mL, LIM(0), 38)];
        if (aR) kR = V.kSA[CK(mR, LIM(0), 39)];
        if (aW) cW = V.C[CK(mW, LIM(0) + 1, 40)];
        if (aL) {
            u32 lm;
            bool ls;
            rank_cmp<true>(V, j, D, kL, kpL, mL, min(hlL, hrL), lm, ls);
            if (ls) {
                lL = mL + 1;
                hlL = P.hloL = lm;
            } else {
                rL = mL;
                hrL = P.hhiL = lm;
            }
        }
        if (aR) {
            u32 lm;
            bool ls;
            rank_cmp<false>(V, j, D, kR, kpR, mR, min(hlR, hrR), lm, ls);
            if (ls) {
                lR = mR + 1;
                hlR = P.hloR = lm;
            } else {
                rR = mR;
                hrR = P.hhiR = lm;
            }
        }
        if (aW) {
            if (cW < j) lW = mW + 1;
            else hW = mW;
        }
        if constexpr (PROF) cy[12]++;
    }
    if constexpr (PROF) {
        const u64 t = clock64();
        cy[8] += t - t0;
        t0 = t;
    }
    P.rsL = lL;
    P.rsR = lR;
    P.w = lW;  // the first sample index x with C[x] >= j (adjust_xc, common.cpp:184-196)
    // nearest lighter ranks, both sides at once: the four ranks either side first, then blocks
    // of 2^l ranks over the weight minima, l growing while the blocks hold no lighter sample
    // and falling once one does (2 log d steps for a lighter sample d ranks away)
    const u32 c = V.c, rs = lR, W = lW;
    u32 vb[4], vf[4];
#pragma unroll
    for (u32 t = 0; t < 4; t++) {
        vb[t] = t < rs ? V.SA[CK(rs - 1 - t, LIM(0), 41)] : NONE;
        vf[t] = rs + t < c ? V.SA[CK(rs + t, LIM(0), 42)] : NONE;
    }
    u32 yb = NONE, yf = NONE;
#pragma unroll
    for (int t = 3; t >= 0; t--) {
        if (vb[t] < W) yb = rs - 1 - t;
        if (vf[t] < W) yf = rs + t;
    }
    bool sb = yb == NONE && rs > 4, sf = yf == NONE && rs + 4 < c;
    u32 pb = rs - 4, pf = rs + 4;  // ranks [pb, rs) / [rs, pf) hold no lighter sample
    int lb = 2, lf = 2;            // block levels
    bool ub_ = true, uf_ = true;   // growing
    const int top = (int)V.wlv - 1;
    while (sb || sf) {
        const u32 wb = 1u << max(lb, 0), wf = 1u << max(lf, 0);
        const bool tb = sb && lb >= 0 && lb <= top && pb >= wb, tf = sf && lf >= 0 && lf <= top && pf + wf <= c;
        u32 x = 0, y = 0;
        if (tb) x = V.wSA[lb][CK(pb - wb, lb ? LIM(0) - wb + 1 : LIM(0), 43)];
        if (tf) y = V.wSA[lf][CK(pf, lf ? LIM(0) - wf + 1 : LIM(0), 44)];
        if (sb) {
            if (tb && x >= W) {
                pb -= wb;
                if (ub_ && lb < top) lb++;
                else if (!ub_) lb--;
            } else if (ub_) {
                ub_ = false;
                lb--;
            } else {
                lb--;
            }
            if (lb < 0) sb = false;
        }
        if (sf) {
            if (tf && y >= W) {
                pf += wf;
                if (uf_ && lf < top) lf++;
                else if (!uf_) lf--;
            } else if (uf_) {
                uf_ = false;
                lf--;
            } else {
                lf--;
            }
            if (lf < 0) sf = false;
        }
        if constexpr (PROF) cy[11]++;
    }
    if (yb == NONE && rs > 4) yb = pb == 0 ? NONE : pb - 1;
    if (yf == NONE && rs + 4 < c) yf = pf >= c ? NONE : pf;
    if constexpr (PROF) cy[9] += clock64() - t0;
    u32 ub = 0, uf = 0;
    if (yb != NONE) ub = lce_of_rank(V.sM, yb, rs, P.hloR, P.hhiR);
    if (yf != NONE) uf = lce_of_rank(V.sM, yf, rs, P.hloR, P.hhiR);
    if (uf > ub) {
        P.yA = yf;
        P.uA = uf;
    } else {
        P.yA = yb;
        P.uA = ub;

    }
}

// the walk's memory of the positions of the last phrase's first window (base .. base + 63, a
// lane each): the next phrase starts less than 64 positions later and takes them over by a lane
// shift (pos_info depends on the position only)
struct lane_cache {
    u32 base;     // NONE: empty
    u32 ak;       // the approximate phrase holding the last phrase start, or NONE
    pos_info P;   // valid if has
    bool has;
};

constexpr u32 BISECT_T = 128;   // right-extension bounds this close are bisected at once
constexpr u32 LANE_SCAN = 32;  // PA intervals scanned whole on the lane

// ---- one exact phrase at i (transform_to_exact_{naive,without_samples,with_samples}) --
// executed by a whole wave; returns (src, len) in every lane.
// Lane j in [i, i + delta) (64 at a time) looks for the longest phrase T[i .. j + x) whose
// occurrence contains a sample at j: the PA interval of T[i .. j] (the sample contexts that end
// with it; extend<LEFT>, queries.cpp:67-275) and, for right extensions x, the SA interval of
// T[j .. j + x) (extend<RIGHT>; with_samples narrows both by interval samples,
// with_samples.cpp:35-122), then a point in both lighter than the first sample >= j
// (intersect, common.cpp:258-358).  Both intervals come from the insertion ranks of j's
// context / suffix (pos_probe, once per position of a walk) and the adjacent LCEs around them
// (binary lifting over V.pM / V.sM): the same rank sets the reference's LCE binary searches
// find, so every decision is the same.  x is bounded by the nearest lighter samples in SA order
// (no earlier sample shares more with the suffix at j), starts from the best witness among
// them and the lightest point of the PA interval, then runs the largest candidate, an
// exponential search and bisection; the predicate is monotone in x, so the result is the
// reference's whatever the probe order.
template <bool PROF>
__device__ void wave_phrase(const smpl_view& V, u32 i, u32& f_src, u32& f_len, u32& f_k, u32 lane, lane_cache& K,
                            u64* cy) {
    const u32 n = (u32)V.L.n;
    const u32 e = n;  // one section: p = 1
    const u8* T = V.L.T;
    // PROF (LZ77SSS_SMPL_PROF): clocks and counts per walk in cy, printed by factorize_exact_smpl
    u64 ct = PROF ? clock64() : 0;
    auto tick = [&](int k) {
        if constexpr (PROF) {
            const u64 t = clock64();
            cy[k] += t - ct;
            ct = t;
        }
    };
    // lower bound: the approximate phrase covering i, cut at i (without_samples.cpp:64-77)
    f_src = T[i];
    f_len = 0;
    f_k = NONE;  // the phrase's j - i when a sample-anchored factor beats the lower bound
    if (V.mode != LZ77SSS_TRANSF_NAIVE) {
        // largest k with afst[k] <= i: the walk's last one and the 63 after it first
        u32 lo = 0, hi = V.za;
        if (K.ak != NONE) {
            const u32 k = K.ak + 1 + lane;
            const u64 bal = __ballot(k < V.za && V.afst[CK(k, LIM(3) + 1, 45)] <= i);
            lo = K.ak + (u32)__popcll(bal);  // afst increases: the lanes below i are a prefix
            if (bal != ~0ull) hi = lo + 1;
        }
        while (hi - lo > 1) {
            const u32 m = (lo + hi) >> 1;
            if (V.afst[CK(m, LIM(3) + 1, 46)] <= i) lo = m; else hi = m;
        }
        K.ak = lo;
        const u32 alen = V.afact[CK(2 * lo + 1, 2 * LIM(3), 47)];
        if (alen != 0) {
            const u32 nxt = V.afst[CK(lo + 1, LIM(3) + 1, 48)];
            const u32 cut = alen - (nxt - i);
            f_len = alen - cut;
            f_src = V.afact[2 * lo] + cut;
        }
    }
    const u32 max_j = min<u32>(e, i + V.delta);
    const u32 D = V.delta;  // left contexts: pattern lengths j - i + 1 <= delta
    {
        // the cached window shifted to start at i
        const u32 d = (K.base != NONE && i >= K.base && i - K.base < 64) ? i - K.base : 64u;
        const u32 sl = (lane + d) & 63;
        const bool h = __shfl((int)K.has, sl, 64) != 0;
        K.P.rsL = __shfl(K.P.rsL, sl, 64);
        K.P.hloL = __shfl(K.P.hloL, sl, 64);
        K.P.hhiL = __shfl(K.P.hhiL, sl, 64);
        K.P.rsR = __shfl(K.P.rsR, sl, 64);
        K.P.hloR = __shfl(K.P.hloR, sl, 64);
        K.P.hhiR = __shfl(K.P.hhiR, sl, 64);
        K.P.w = __shfl(K.P.w, sl, 64);
        K.P.yA = __shfl(K.P.yA, sl, 64);
        K.P.uA = __shfl(K.P.uA, sl, 64);
        K.has = lane + d < 64 && h;
        K.base = i;
    }
    for (u32 j0 = i; j0 < max_j; j0 += 64) {
        const u32 j = j0 + lane;
        const bool act = j < max_j;
        const bool first = j0 == i;  // the window the cache holds
        const u32 lce_l = j - i + 1;
        const u32 ch = act ? T[j] : 0u;
        const u32 cb = V.CS[ch], ce = V.CS[ch + 1];
        pos_info P{};
        const bool have = act && ce > cb;
        if (have) {
            if (first && K.has) {
                P = K.P;
            } else {
                pos_probe<PROF>(V, j, D, cb, ce, P, cy);
                if (first) {
                    K.P = P;
                    K.has = true;
                }
            }
        }
        // PA interval of T[i..j]: the ranks around j's insertion rank whose contexts share lce_l
        u32 xb = 0, xe = 0;
        const bool okl = have && (P.hloL >= lce_l || P.hhiL >= lce_l);
        tick(0);
        if (okl) iv_around(V.pM, V.c, P.rsL, P.hloL, P.hhiL, lce_l, xb, xe);
        tick(14);
        // right extensions: max lce_r in [lce_r_min, e - j] with a lighter point
        const u32 lrmin = (f_len < j - i) ? 0u : (i + f_len - j);
        const u32 lrmax = e - j;
        u32 lo = lrmin, hi = lrmax + 1, step = 1;
        bool bin = false;
        bool run = okl && lo < lrmax;
        const u32 rs = P.rsR, h_lo = P.hloR, h_hi = P.hhiR, W = P.w, yA = P.yA, uA = P.uA;
        // no sample before j shares more than uA characters with the suffix at j
        hi = min(hi, uA + 1);
        if (hi - lo <= 1) run = false;
        u32 best_y = 0;
        bool got = false, top = true;
        // the answer is the largest LCE with j of a lighter sample whose context ends with
        // T[i..j].  Few such contexts (a PA interval below LANE_SCAN ranks): all of them, on the
        // lane.  Else the nearest lighter sample in SA order, whose LCE bounds the answer, when
        // its context ends with T[i..j]; the probes below finish between the bounds.
        bool done = !run;
        if (run) {
            if (xe - xb < V.lane_scan) {
                for (u32 x = xb; x <= xe; x++) {
                    if (V.PA[CK(x, LIM(0), 50)] < W) {
                        const u32 y = V.Pi[CK(x, LIM(0), 51)], l = lce_of_rank(V.sM, y, rs, h_lo, h_hi);
                        if (l > lo) {
                            lo = l;
                            best_y = y;
                            got = true;
                        }
                    }
                }
                done = true;
            } else if (yA == NONE || uA <= lo) {
                done = true;  // no lighter sample shares more than lo
            } else {
                const u32 xx = V.PAR[CK(V.SA[CK(yA, LIM(0), 52)], LIM(0), 53)];
                if (xx >= xb && xx <= xe) {
                    lo = uA;
                    best_y = yA;
                    got = true;
                    done = true;
                }
            }
        }
        if (run) {
            if (!done) {
                // the lightest point of the PA interval is a witness up to its LCE
                const u32 s0 = min_weight(V.wPA, xb, xe);
                if (s0 < W) {
                    const u32 y0 = V.SAR[CK(s0, LIM(0), 54)], l0 = lce_of_rank(V.sM, y0, rs, h_lo, h_hi);
                    if (l0 > lo) {
                        lo = l0;
                        best_y = y0;
                        got = true;
                    }
                }
            }
            if (done || hi - lo <= 1) run = false;
        }
        tick(1);
        while (__ballot(run)) {
            u32 x = 0, nb = 0, ne = 0;
            bool cand = false;
            if (run) {
                // the largest possible x first (its intervals are the narrowest, and it is often
                // the answer), then bisection between the witness and the failed probes when they
                // are at most BISECT_T apart (its probes stay well above lo, where the intervals
                // are narrow), else an exponential search up from lo first: the predicate is
                // monotone in x, so the answer is the reference's upward exponential search's
                x = top ? hi - 1 : bin ? lo + (hi - lo) / 2 : min(lo + step, hi - 1);
                cand = h_lo >= x || h_hi >= x;
                if (cand) iv_around(V.sM, V.c, rs, h_lo, h_hi, x, nb, ne);
            }
            tick(7);
            if constexpr (PROF) {
                cy[3]++;
                cy[4] += __popcll(__ballot(cand && min(xe - xb, ne - nb) + 1 > V.small_t));
                cy[5] += __popcll(__ballot(cand));
            }
            bool f;
            u32 py;
            wave_intersect(V, cand, xb, xe, nb, ne, W, ch, f, py, lane);
            tick(2);
            if (run) {
                if (cand && f) {
                    lo = lce_of_rank(V.sM, py, rs, h_lo, h_hi);  // >= x: the point is a witness up to it
                    best_y = py;
                    got = true;
                    if (!bin && !top) step *= 2;
                } else {
                    hi = x;
                    if (!top || hi - lo <= BISECT_T) bin = true;
                }
                top = false;
                if (hi - lo <= 1) run = false;
            }
            // a lane whose longest possible phrase (lce_l + hi - 2) cannot beat the wave's
            // best confirmed one (longer, or as long at a smaller j) or f stops searching; the
            // winner is never stopped and its search is unchanged, so the result is the same
            u32 bl = got ? lce_l + lo - 1 : 0u, bjj = got ? j : 0xFFFFFFFFu;
            for (int o = 32; o >= 1; o >>= 1) {
                const u32 l2 = __shfl_xor(bl, o, 64), j2 = __shfl_xor(bjj, o, 64);
                if (l2 > bl || (l2 == bl && j2 < bjj)) {
                    bl = l2;
                    bjj = j2;
                }
            }
            if (run) {
                const u32 ub = lce_l + hi - 2;
                if (ub <= f_len || ub < bl || (ub == bl && j > bjj)) run = false;
            }
        }
        // the longest of the wave (the smallest j on ties) improves f (intersect: lce > f.len)
        u32 len = got ? lce_l + lo - 1 : 0u;
        u32 src = got ? V.C[CK(V.SA[CK(best_y, LIM(0), 55)], LIM(0), 56)] - lce_l + 1 : 0u;
        u32 bj = got ? j : 0xFFFFFFFFu;
        for (int o = 32; o >= 1; o >>= 1) {
            const u32 l2 = __shfl_xor(len, o, 64), s2 = __shfl_xor(src, o, 64), j2 = __shfl_xor(bj, o, 64);
            if (l2 > len || (l2 == len && j2 < bj)) {
                len = l2;
                src = s2;
                bj = j2;
            }
        }
        if (len > f_len) {
            f_len = len;
            f_src = src;
            f_k = bj - i;  // the smallest j reaching len (its lane is never stopped early)
        }
    }
    if (f_len > e - i) f_len = e - i;
    if constexpr (PROF) cy[6]++;
}

// ---------------------------------------------------------------------------
// construction kernels
__global__ void k_afst_len(const u32* __restrict__ F, u32 za, u32* __restrict__ out) {
    const u64 k = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (k < za) out[k] = max(1u, F[2 * k + 1]);
    else if (k == za) out[k] = 0;
}
// samples per approximate phrase k >= 1: ceil(len / delta); 1 for phrase 0 (C[0] = 0)
__global__ void k_smpl_count(const u32* __restrict__ F, u32 za, u32 delta, u32* __restrict__ cnt) {
    const u64 k = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (k > za) return;
    if (k == za) { cnt[k] = 0; return; }
    if (k == 0) { cnt[k] = 1; return; }
    const u32 g = max(1u, F[2 * k + 1]);
    cnt[k] = (g + delta - 1) / delta;
}
__global__ void k_smpl_fill(const u32* __restrict__ F, const u32* __restrict__ afst, u32 za, u32 delta,
                            const u32* __restrict__ off, u32* __restrict__ C) {
    const u64 k = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= za) return;
    if (k == 0) { C[0] = 0; return; }
    // end_cur before phrase k = afst[k] - 1 (common.cpp:59-70 sums the lengths of phrases 1..k)
    const u32 g = max(1u, F[2 * k + 1]);
    const u32 prev = afst[k] - 1, cnt = (g + delta - 1) / delta;
    u32 o = off[k];
    for (u32 m = 1; m < cnt; m++) C[o++] = prev + m * delta;
    C[o] = prev + g;
}
// 57-bit keys: 7 characters (c + 1, 0 past the text) going left from C (PA) or right (SA)
// the characters the text uses (one flag per byte value)
__global__ void k_text_alpha(const u8* __restrict__ T, u64 n, u32* __restrict__ used) {
    __shared__ u32 f[256];
    f[threadIdx.x] = 0;
    __syncthreads();
    const u64 nw = n / 16;
    for (u64 k = (u64)blockIdx.x * blockDim.x + threadIdx.x; k < nw; k += (u64)gridDim.x * blockDim.x) {
        const uint4 v = ((const uint4*)T)[k];
        const u32 w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int q = 0; q < 4; q++)
#pragma unroll
            for (int b = 0; b < 4; b++) f[(w[q] >> (8 * b)) & 0xFF] = 1;
    }
    for (u64 k = nw * 16 + (u64)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += (u64)gridDim.x * blockDim.x)
        f[T[k]] = 1;
    __syncthreads();
    if (f[threadIdx.x]) used[threadIdx.x] = 1;
}
// sort keys of the sample contexts: kc characters of `bits` bits each (the character's rank in
// the text's alphabet), the first one in the top bits; past the text's end (right) or start
// (left) the code 0, the smallest character's, so that a shorter context never gets a larger key
// than a context it is a prefix of (key order implies context order; equal keys go to the
// comparator).  Left contexts take at most cap + 1 characters, all the comparator looks at.
__global__ void k_smpl_keys(const u8* __restrict__ T, u64 n, const u32* __restrict__ C, u32 c, int left,
                            const u8* __restrict__ code, u32 bits, u32 kc, u64* __restrict__ key, u32* __restrict__ id) {
    const u64 k = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= c) return;
    const u64 p = C[k];
    u64 v = 0;
    for (u32 t = 0; t < kc; t++) {
        u64 d;
        if (left) d = p >= (u64)t ? code[T[p - t]] : 0u;
        else d = p + t < n ? code[T[p + t]] : 0u;
        v = (v << bits) | d;
    }
    key[k] = v;
    id[k] = (u32)k;
}
// the first 16 bits of a sort key of kbits bits
__device__ __forceinline__ u32 key_pre16(u64 key, u32 kbits) {
    return kbits >= 16 ? (u32)(key >> (kbits - 16)) : (u32)(key << (16 - kbits));
}
// out[u] = the first rank whose sorted key starts with 16 bits >= u, u in [0, 65536]
__global__ void k_pre_table(const u64* __restrict__ sorted, u32 c, u32 kbits, u32* __restrict__ out) {
    const u32 u = blockIdx.x * blockDim.x + threadIdx.x;
    if (u > 65536) return;
    u32 lo = 0, hi = c;
    while (lo < hi) {
        const u32 m = (lo + hi) >> 1;
        if (key_pre16(sorted[m], kbits) < u) lo = m + 1; else hi = m;
    }
    out[u] = lo;
}
// out[b] = the first sample index x with C[x] >= 256 b (b in [0, nblk)); consecutive samples
// are at most delta <= 256 apart, so each sample fills at most two blocks
__global__ void k_wblk(const u32* __restrict__ C, u32 c, u64 nblk, u32* __restrict__ out) {
    const u64 x = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (x >= c) return;
    const u64 b0 = x == 0 ? 0 : ((u64)C[x - 1] >> 8) + 1, b1 = (u64)C[x] >> 8;
    for (u64 b = b0; b <= b1 && b < nblk; b++) out[b] = (u32)x;
    if (x == c - 1)
        for (u64 b = b1 + 1; b < nblk; b++) out[b] = c;
}
struct smpl_less {
    lce_view L;
    const u32* C;
    const u64* key;  // by sample id
    u32 cap;         // left: delta (the compared context is cap + 1 characters)
    int left;
    __device__ bool operator()(const u32& a, const u32& b) const {
        if (a == b) return false;
        const u64 ka = key[a], kb = key[b];
        if (ka != kb) return ka < kb;
        const u32 pa = C[a], pb = C[b];
        if (left) {
            const u32 l = (u32)dev_lce_left(L.T, L.R, pa, pb, cap);
            if (l > min(pa, pb)) return pa < pb;
            const u8 ca = L.T[pa - l], cb = L.T[pb - l];
            if (ca != cb) return ca < cb;
            return a < b;  // equal on cap + 1 characters
        }
        return suffix_less(pa, pb);
    }
    // the suffix order of two text positions (dev_lce's cases): when both meet their next sync
    // positions at the same offset d with equal text before them, the order is that of the sync
    // suffixes (ISA), with no LCP range minimum and no text read after it
    __device__ bool suffix_less(u64 i, u64 j) const {
        const u64 l = min(i, j), r = max(i, j);
        const u64 lmax = L.n - r, local = min<u64>(64, lmax);
        u64 c = dev_naive_lce(L.T, l, r, local);
        if (c < local || c == lmax) {
            if (r + c >= L.n) return i > j;
            return L.T[i + c] < L.T[j + c];
        }
        const u32 kl = dev_succ(L, l), kr = dev_succ(L, r);
        if (kl != L.s && kr != L.s) {
            const u64 dl = L.S[kl] - l, dr = L.S[kr] - r;
            if (dl == dr && (sizeof(pos_t) == 4)) {
                if (dl > c) {
                    const u64 e = dev_lce_fwd(L.T, L.R, l + c, r + c, dl - c);
                    if (e < dl - c) {
                        const u64 m = c + e;
                        return L.T[i + m] < L.T[j + m];
                    }
                }
                // equal up to the sync positions S[kl] = l + d, S[kr] = r + d
                const u32 a = L.ISA[kl], b = L.ISA[kr];
                return (i == l) ? a < b : b < a;
            }
        }
        const u64 e = dev_lce(L, i, j);
        if (r + e >= L.n) return i > j;
        return L.T[i + e] < L.T[j + e];
    }
};
__global__ void k_rank_of(const u32* __restrict__ X, u32 c, u32* __restrict__ R) {
    const u64 r = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (r < c) R[X[r]] = (u32)r;
}
__global__ void k_pi_psi(const u32* __restrict__ PA, const u32* __restrict__ SA, const u32* __restrict__ PAR,
                         const u32* __restrict__ SAR, u32 c, u32* __restrict__ Pi, u32* __restrict__ Psi) {
    const u64 r = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= c) return;
    Pi[r] = SAR[PA[r]];
    Psi[r] = PAR[SA[r]];
}
__global__ void k_char_hist(const u8* __restrict__ T, const u32* __restrict__ C, u32 c, u32* __restrict__ hist) {
    __shared__ u32 h[256];
    h[threadIdx.x] = 0;
    __syncthreads();
    for (u64 k = (u64)blockIdx.x * blockDim.x + threadIdx.x; k < c; k += (u64)gridDim.x * blockDim.x)
        atomicAdd(&h[T[C[k]]], 1u);
    __syncthreads();
    if (h[threadIdx.x]) atomicAdd(&hist[threadIdx.x], h[threadIdx.x]);
}
// grid cell of sample id k and its sort key (cell << 32 | weight)
__global__ void k_grid_keys(const u8* __restrict__ T, const u32* __restrict__ C, u32 c, const u32* __restrict__ PAR,
                            const u32* __restrict__ SAR, const u32* __restrict__ CS, const u32* __restrict__ gcb,
                            const u32* __restrict__ gwd, const u32* __restrict__ gwin, u64* __restrict__ key,
                            u32* __restrict__ id) {
    const u64 k = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= c) return;
    const u32 ch = T[C[k]];
    const u32 r0 = CS[ch];
    const u32 cx = (PAR[k] - r0) / gwin[ch], cy = (SAR[k] - r0) / gwin[ch];
    key[k] = ((u64)(gcb[ch] + cy * gwd[ch] + cx) << 32) | (u32)k;
    id[k] = (u32)k;
}
__global__ void k_grid_points(const u64* __restrict__ skey, const u32* __restrict__ PAR, const u32* __restrict__ SAR,
                              u32 c, u32* __restrict__ gx, u32* __restrict__ gy, u32* __restrict__ gw,
                              u32* __restrict__ cell, u32 ncell) {
    const u64 t = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (t > c) return;
    // cell[x] = first point of a cell >= x: point t starts the cells after point t - 1's
    // cell up to its own (each cell written once)
    const u32 lo = t == 0 ? 0u : (u32)(skey[t - 1] >> 32) + 1;
    const u32 hi = t == c ? ncell : (u32)(skey[t] >> 32);
    for (u32 x = lo; x <= hi; x++) cell[x] = (u32)t;
    if (t < c) {
        const u32 k = (u32)skey[t];
        gx[t] = PAR[k];
        gy[t] = SAR[k];
        gw[t] = k;
    }
}
// lightest weight per cell (cells sorted by weight inside; INF when empty) = row level 0
__global__ void k_cell_min(const u32* __restrict__ cell, const u32* __restrict__ gw, u32 ncell, u32* __restrict__ out) {
    const u64 t = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= ncell) return;
    const u32 p0 = cell[t];
    out[t] = cell[t + 1] > p0 ? gw[p0] : 0xFFFFFFFFu;
}
// row level k from k - 1: cells x of a row with x + 2^k <= gw (the others are never read)
__global__ void k_cell_rowmin(const u32* __restrict__ prev, const u32* __restrict__ cgw, const u32* __restrict__ cgcb,
                              u32 ncell, u32 half, u32* __restrict__ out) {
    const u64 t = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= ncell) return;
    // the character block of cell t (<= 256 blocks, binary search)
    u32 lo = 0, hi = 256;
    while (hi - lo > 1) {
        const u32 m = (lo + hi) >> 1;
        if (cgcb[m] <= t) lo = m; else hi = m;
    }
    const u32 gw = cgw[lo];
    const u32 x = gw ? (u32)((t - cgcb[lo]) % gw) : 0u;
    out[t] = x + half < gw ? min(prev[t], prev[t + half]) : prev[t];
}

// adjacent context LCEs of an order (LCP_S / LCS_S of construction.cpp:118-129)
__global__ void k_adj_lce(lce_view L, const u32* __restrict__ C, const u32* __restrict__ X, u32 c, u32 cap, int left,
                          u32* __restrict__ out) {
    const u64 r = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (r > c) return;
    if (r == 0 || r == c) { out[r] = 0; return; }
    const u32 a = C[X[r - 1]], b = C[X[r]];
    out[r] = left ? (u32)dev_lce_left(L.T, L.R, a, b, cap) : (u32)min<u64>(dev_lce(L, a, b), 0xFFFFFFFFull);
}
// sparse-table level of the adjacent LCEs: out[k] = min(prev[k], prev[k + half])
__global__ void k_iv_min_level(const u32* __restrict__ prev, u64 cnt, u64 half, u32* __restrict__ out) {
    const u64 k = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (k < cnt) out[k] = min(prev[k], prev[k + half]);
}

// ---------------------------------------------------------------------------
// chain kernels: task table (position -> phrase), a hash map position -> task id
struct task_tab {
    u32* pos;
    u32* len;
    u32* src;
    u32* hop;
    u32* wk;     // the phrase's j - i (wave_phrase f_k): where the source pass starts
    u32* keys;   // position + 1, 0 empty
    u32* vals;   // task id
    u32 mask;
    u32 cap;     // task capacity
    u32* ntask;  // counter
};
__device__ __forceinline__ u32 thash(u32 p) { return (p * 0x9E3779B1u) ^ (p >> 15); }
// inserts p; returns the new task id, or NONE if p was present (or the table is full)
__device__ u32 task_insert(task_tab& Tt, u32 p, u32 hop) {
    u32 h = thash(p);
    for (u32 probe = 0; probe <= Tt.mask; probe++, h++) {
        const u32 old = atomicCAS(&Tt.keys[h & Tt.mask], 0u, p + 1);
        if (old == p + 1) return NONE;
        if (old == 0) {
            const u32 id = atomicAdd(Tt.ntask, 1u);
            if (id >= Tt.cap) {
                Tt.vals[h & Tt.mask] = NONE;
                return NONE;
            }
            Tt.pos[id] = p;
            Tt.hop[id] = hop;
            Tt.len[id] = NONE;
            Tt.vals[h & Tt.mask] = id;
            return id;
        }
    }
    return NONE;
}
__device__ u32 task_find(const task_tab& Tt, u32 p) {
    u32 h = thash(p);
    for (u32 probe = 0; probe <= Tt.mask; probe++, h++) {
        const u32 k = Tt.keys[h & Tt.mask];
        if (k == 0) return NONE;
        if (k == p + 1) return Tt.vals[h & Tt.mask];
    }
    return NONE;
}
// ---- the chain by chunk walks + bridges (replaces one hop per launch) ----------------
// Chunk k's wave walks the greedy chain from its first approximate phrase, inserting a task per phrase, until it
// meets a task another walk inserted (merged) or passes its chunk end (its exit is kept).
// A bridge walks from every exit until it meets a task.  Every task's successor position
// then holds a task (a walk inserts it, finds it, or hands it to a bridge), so the chain
// from position 0 lies in the table; it is marked by pointer doubling.
template <bool PROF>
__device__ __forceinline__ u32 wave_walk(const smpl_view& V, task_tab& Tt, u64 p, u64 stop, u32 lane, u32* __restrict__ full,
                                         u32& nph, u64* cy) {
    const u64 n = V.L.n;
    lane_cache K{NONE, NONE, pos_info{}, false};
    for (;;) {
        if (p >= n) return NONE;
        if (p >= stop) return (u32)p;
        u32 t = NONE;
        if (lane == 0) {
            t = task_insert(Tt, (u32)p, 0);
            if (t == NONE && task_find(Tt, (u32)p) == NONE) atomicOr(full, 1u);  // table full
        }
        t = (u32)__shfl((int)t, 0);
        if (t == NONE) return NONE;  // merged (or out of room: reported)
        u32 src, len, wk;
        wave_phrase<PROF>(V, (u32)p, src, len, wk, lane, K, cy);
        nph++;
        if (lane == 0) {
            Tt.src[t] = src;
            Tt.len[t] = len;
            Tt.wk[t] = wk;
        }
        p += max(1u, len);
    }
}
// PROF (LZ77SSS_SMPL_PROF): per walk its clock ticks and phrase count in prof, the section
// clocks and counts summed into V.cyc (walks starting before / at or after V.prof_split apart)
template <bool PROF>
__device__ __forceinline__ void walk_prof(const smpl_view& V, u64 start, u64 t0, u32 nph, const u64* cy, u32 lane,
                                          u32* __restrict__ slot) {
    if (lane != 0) return;
    slot[0] = (u32)(wall_clock64() - t0);
    slot[1] = nph;
    const u32 bank = start < V.prof_split ? 0 : 16;
    for (int k = 0; k < 16; k++) atomicAdd(&V.cyc[bank + k], (unsigned long long)cy[k]);
}
// Chunk k starts at approximate phrase k * cp (so every walk has about cp phrases to parse,
// whatever the text's local compressibility) and ends at phrase (k + 1) * cp.
template <bool PROF>
__global__ __launch_bounds__(64 * SWPB, SMPL_OCC) void k_chunk_walks(const smpl_view V, task_tab Tt, u32 cp, u32 nch,
                                                          u32* __restrict__ ex, u32* __restrict__ full,
                                                          u32* __restrict__ prof) {
    const u32 lane = threadIdx.x & 63;
    const u32 k = blockIdx.x * SWPB + (threadIdx.x >> 6);
    if (k >= nch) return;
    const u64 a = (u64)k * cp, b = min<u64>(V.za, a + cp);
    const u64 t0 = PROF ? wall_clock64() : 0;
    u32 nph = 0;
    u64 cy[16] = {};
    const u64 start = V.afst[a];
    const u32 e = wave_walk<PROF>(V, Tt, start, V.afst[b], lane, full, nph, cy);
    if (lane == 0) ex[k] = e;
    if constexpr (PROF) walk_prof<PROF>(V, start, t0, nph, cy, lane, prof + 2 * (u64)k);
}
template <bool PROF>
__global__ __launch_bounds__(64 * SWPB, SMPL_OCC) void k_bridge_walks(const smpl_view V, task_tab Tt, u32 nch,
                                                           const u32* __restrict__ ex, u32* __restrict__ full,
                                                           u32* __restrict__ prof) {
    const u32 lane = threadIdx.x & 63;
    const u32 k = blockIdx.x * SWPB + (threadIdx.x >> 6);
    if (k >= nch || ex[k] == NONE) return;
    const u64 t0 = PROF ? wall_clock64() : 0;
    u32 nph = 0;
    u64 cy[16] = {};
    wave_walk<PROF>(V, Tt, ex[k], ~0ull, lane, full, nph, cy);
    if constexpr (PROF) walk_prof<PROF>(V, ex[k], t0, nph, cy, lane, prof + 2 * (u64)k);
}
// successor task of every task (ntask = the end); a missing successor is reported
__global__ void k_task_next(task_tab Tt, u32 ntask, u32 n, u32* __restrict__ nxt, u32* __restrict__ bad) {
    const u64 t = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (t > ntask) return;
    if (t == ntask) { nxt[t] = ntask; return; }
    const u64 q = (u64)Tt.pos[t] + max(1u, Tt.len[t]);
    u32 r = ntask;
    if (q < n) {
        r = task_find(Tt, (u32)q);
        if (r == NONE || r >= ntask) { atomicOr(bad, 1u); r = ntask; }
    }
    nxt[t] = r;
}
__global__ void k_tjump(const u32* __restrict__ prev, u32 m, u32* __restrict__ out) {
    const u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < m) out[i] = prev[prev[i]];
}
__global__ void k_texpand(const u32* __restrict__ C, u64 cnt, const u32* __restrict__ J, u32* __restrict__ out) {
    const u64 m = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (m >= cnt) return;
    const u32 c = C[m];
    out[2 * m] = c;
    out[2 * m + 1] = J[c];
}
__global__ void k_troot(task_tab Tt, u32* __restrict__ C, u32 ntask) {
    const u32 r = task_find(Tt, 0u);
    C[0] = r == NONE ? ntask : r;
}
// the path from the root in order: its length (first end marker) and its factors
__global__ void k_path_len(const u32* __restrict__ C, u64 cnt, u32 ntask, u32* __restrict__ z) {
    const u64 m = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (m < cnt && C[m] == ntask && (m == 0 || C[m - 1] != ntask)) *z = (u32)m;
}
__global__ void k_path_emit(task_tab Tt, const u32* __restrict__ C, u32 z, u32* __restrict__ F, u32* __restrict__ wk) {
    const u64 m = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (m >= z) return;
    const u32 t = C[m];
    F[2 * m] = Tt.src[t];
    F[2 * m + 1] = Tt.len[t];
    wk[m] = Tt.wk[t];
}

// ---------------------------------------------------------------------------
// the source pass: the reference's source for every phrase of the chain.  The lengths are the
// canonical ones whatever the probe order; the source is not: the reference keeps the first
// factor it finds of the final length (intersect, common.cpp:341-346: only a strictly longer one
// replaces f), so it is
//   * the approximate phrase cut at i when that is already as long (without_samples.cpp:64-77,
//     with_samples.cpp:146-160; naive starts from a literal, naive.cpp:57),
//   * else the point that intersect returns for the first j in the transform's visit order whose
//     intervals (T[i..j] in PA order, T[j..i+len) in SA order) hold a point lighter than the
//     first sample >= j: j ascending (naive.cpp:60, without_samples.cpp:79), with_samples the
//     sampled left lengths first, then the others (with_samples.cpp:162-185); intersect's point
//     comes from the Pi / Psi scan below RG_SCAN ranks or the reference's grid
//     (static_weighted_square_grid.hpp:116-185), both in their visit order (wave_intersect
//     over a view holding the reference's grid).
__global__ void k_fact_len1(const u32* __restrict__ F, u32 z, u32* __restrict__ out) {
    const u64 m = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (m < z) out[m] = max(1u, F[2 * m + 1]);
    else if (m == z) out[m] = 0;
}
// histogram of the adjacent left-context LCEs in PA order, LCX[0 .. c) (LCX[0] = 0; values <= delta)
__global__ void k_adj_hist(const u32* __restrict__ adj, u32 c, u32* __restrict__ hist) {
    __shared__ u32 h[SMPL_MAX_DELTA + 1];
    for (u32 t = threadIdx.x; t <= SMPL_MAX_DELTA; t += blockDim.x) h[t] = 0;
    __syncthreads();
    for (u64 k = (u64)blockIdx.x * blockDim.x + threadIdx.x; k < c; k += (u64)gridDim.x * blockDim.x)
        atomicAdd(&h[min(adj[k], SMPL_MAX_DELTA)], 1u);
    __syncthreads();
    for (u32 t = threadIdx.x; t <= SMPL_MAX_DELTA; t += blockDim.x)
        if (h[t]) atomicAdd(&hist[t], h[t]);
}
// One lane per phrase.  The walk's phrase search kept, of the j reaching the final length, the
// smallest (wk = j - i; NONE when the lower bound was kept, whose source is the reference's
// already): the reference's first j in ascending order (naive, without_samples).  with_samples
// visits the sampled left lengths first, so a sampled k in (wk, kmax) reaching the length comes
// before wk: those are tried in ascending order, then wk (a sampled wk is the answer itself).
// Each try is one position probe, two interval liftings and one intersect of the wave.
__global__ __launch_bounds__(64 * SWPB) void k_ref_sources(const smpl_view V, u32* __restrict__ F,
                                                           const u32* __restrict__ pos, const u32* __restrict__ wk,
                                                           u32 z, const u32* __restrict__ smpld,
                                                           u32* __restrict__ miss) {
    const u32 lane = threadIdx.x & 63;
    const u64 m = ((u64)blockIdx.x * SWPB + (threadIdx.x >> 6)) * 64 + lane;
    const u32 n = (u32)V.L.n;
    const bool ws = V.mode == LZ77SSS_TRANSF_WITH_SAMPLES;
    u32 i = 0, M = 0, k0 = NONE, kmax = 0;
    if (m < z) {
        k0 = wk[m];
        if (k0 != NONE) {
            i = pos[m];
            M = F[2 * m + 1];
            kmax = min(min(V.delta, n - i), M);
        }
    }
    // the lane's next candidate: with_samples' sampled k above k0 first (ascending), then k0
    bool pend = k0 != NONE;
    u32 k = k0;
    bool after = false;  // k0 itself has been reached (the last candidate)
    if (pend && ws && !smpld[k0 + 1]) {
        u32 t = k0 + 1;
        while (t < kmax && !smpld[t + 1]) t++;
        if (t < kmax) k = t;
        else after = true;
    } else {
        after = true;
    }
    while (__ballot(pend)) {
        const u32 j = i + k;
        const u32 ch = pend ? V.L.T[j] : 0u;
        const u32 cb = V.CS[ch], ce = V.CS[ch + 1];
        pos_info P{};
        const bool have = pend && ce > cb;
        if (have) pos_probe<false>(V, j, V.delta, cb, ce, P, nullptr);
        const u32 lce_l = k + 1, lce_r = M - k;
        u32 xb = 1, xe = 0, nb = 1, ne = 0;
        const bool okl = have && (P.hloL >= lce_l || P.hhiL >= lce_l);
        const bool okr = have && (P.hloR >= lce_r || P.hhiR >= lce_r);
        if (okl) iv_around(V.pM, V.c, P.rsL, P.hloL, P.hhiL, lce_l, xb, xe);
        if (okr) iv_around(V.sM, V.c, P.rsR, P.hloR, P.hhiR, lce_r, nb, ne);
        const bool cand = okl && okr;
        bool f = false;
        u32 py = 0;
        wave_intersect(V, cand, xb, xe, nb, ne, P.w, ch, f, py, lane);
        if (pend) {
            if (cand && f) {
                F[2 * m] = V.C[V.SA[py]] - lce_l + 1;
                pend = false;
            } else if (after) {
                atomicAdd(miss, 1u);  // (k0 reaches the length: cannot happen)
                pend = false;
            } else {
                u32 t = k + 1;
                while (t < kmax && !smpld[t + 1]) t++;
                if (t < kmax) {
                    k = t;
                } else {
                    k = k0;
                    after = true;
                }
            }
        }
    }
}

// with_samples' sampled left pattern lengths (construction.cpp build_samples<LEFT>, max length
// delta) from the histogram of LCX[0 .. c) (the adjacent left-context LCEs in PA order, <= delta):
// the rank-interpolated lengths between the ranks of 3 and of the longest, then the short lengths
// added while their ranks sum below 0.2 x 2c.  smpld[len] = 1 for every sampled length.
static void sampled_left_lengths(const u32* hist, u32 c, u32 delta, u32* smpld) {
    u64 cum[SMPL_MAX_DELTA + 2];  // cum[v] = number of values < v
    cum[0] = 0;
    for (u32 v = 0; v <= SMPL_MAX_DELTA; v++) cum[v + 1] = cum[v] + hist[v];
    // the binary searches of the reference over the sorted values: the first index in [0, c - 1]
    // whose value is >= v (c - 1 when none is)
    auto rank_geq = [&](u32 v) -> u32 { return (u32)std::min<u64>(cum[std::min<u32>(v, SMPL_MAX_DELTA + 1)], c - 1); };
    auto at = [&](u64 r) -> u32 {
        u32 v = 0;
        while (v < SMPL_MAX_DELTA && cum[v + 1] <= r) v++;
        return v;
    };
    std::vector<u32> pl{1, 2};
    const u32 msl = std::min<u32>(at(c - 1), delta);
    const u32 rng_min = rank_geq(3), rng_max = rank_geq(msl);
    if (rng_min < rng_max) {
        const double max_num = 2.0 * c, rng = (double)rng_max - (double)rng_min;
        const u64 num = std::min<u64>((u64)msl - 2, 2 + (u64)std::floor((2.0 * max_num) / (double)(rng_min + rng_max)));
        std::vector<u32> ranks(std::max<u64>(num, 3), 0);
        for (u64 i = 2; i < num; i++) {
            const double rel = (double)(i - 1) / (double)(num - 2);
            const u32 rnk = (u32)std::floor((double)rng_min + rel * rng);
            const u32 len = std::max(at(rnk), pl.back() + 1);
            if (len > msl) break;
            pl.push_back(len);
            ranks[i] = rank_geq(len);
        }
        const u32 max_add = (u32)(max_num * 0.2);
        if (ranks[2] < max_add) {
            u32 added = 0;
            for (u32 len = 3; true; len++) {
                if (std::find(pl.begin(), pl.end(), len) != pl.end()) continue;
                const u32 rnk = rank_geq(len);
                if (len > msl || added + rnk > max_add) break;
                added += rnk;
                pl.push_back(len);
            }
        }
    }
    for (u32 len : pl)
        if (len <= SMPL_MAX_DELTA) smpld[len] = 1;
}

u64 engine::factorize_exact_smpl(int transf_mode, int phr_mode, u32 rk_seed, int log2_override, bool log) {
    LZ_HIP(hipSetDevice(device));
    if (n > 0xFFFFFFF0ull) throw error(LZ77SSS_EINVAL, "n too large for pos_t = uint32_t");
    const auto t_start = std::chrono::steady_clock::now();
    if (log) g_dev_peak.store(g_dev_bytes.load());
    // the 3-approximation (compute_approximation, lz77_sss.hpp:324)
    const u64 za64 = factorize(phr_mode, rk_seed, log2_override, false, LZ77SSS_GREEDY);
    SMPL_STAGE("approx");
    num_fact = 0;
    last_fact_mode = LZ77SSS_GREEDY;
    if (n == 0) return 0;
    const u32 delta = (u32)std::min<u64>(n / za64, SMPL_MAX_DELTA);
    // hipcub scans / radix sorts below take int item counts, and the sample offsets are u32:
    // c <= za + n / delta samples (one per phrase end, one per delta inside a phrase) must stay
    // below 2^31 (low-compressibility texts past about 2 GiB reach it)
    if (za64 + n / std::max<u32>(delta, 1) + 1 >= 0x7FFFFFFFull)
        throw error(LZ77SSS_EINVAL, "exact-smpl: more than 2^31 samples (za + n/delta); text too incompressible");
    const u32 za = (u32)za64;
    u32* afact = e_afact.get(2 * (u64)za + 2);
    LZ_HIP(hipMemcpyAsync(afact, fact.p, (size_t)za * 8, hipMemcpyDeviceToDevice, st));
    // approximate phrase starts
    u32* afst = e_afst.get((u64)za + 2);
    {
        u32* lens = e_tmp1.get((u64)za + 2);
        k_afst_len<<<cdiv((u64)za + 1, 256), 256, 0, st>>>(afact, za, lens);
        size_t tb = 0;
        LZ_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, lens, afst, (int)(za + 1), st));
        u8* t = scan_tmp.get(tb);
        LZ_HIP(hipcub::DeviceScan::ExclusiveSum(t, tb, lens, afst, (int)(za + 1), st));
    }
    // samples C (build_c, common.cpp:34-88)
    u32 c;
    {
        u32* cnt = e_tmp1.get((u64)za + 2);
        u32* off = e_tmp2.get((u64)za + 2);
        k_smpl_count<<<cdiv((u64)za + 1, 256), 256, 0, st>>>(afact, za, delta, cnt);
        size_t tb = 0;
        LZ_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, cnt, off, (int)(za + 1), st));
        u8* t = scan_tmp.get(tb);
        LZ_HIP(hipcub::DeviceScan::ExclusiveSum(t, tb, cnt, off, (int)(za + 1), st));
        c = rd1(off + za, st);
        u32* C = e_C.get((u64)c + 1);
        k_smpl_fill<<<cdiv(za, 256), 256, 0, st>>>(afact, afst, za, delta, off, C);
    }
    u32* C = e_C.p;
    timer.mark("smpl_set"); SMPL_STAGE("smpl_set");
    const lce_view LV = view(d_text);
    // PA / SA (sample_index.hpp:317-353): radix sort by as many characters as 64 bits hold in
    // the text's alphabet (32 of a 4-letter text), merge sort by the text
    u32 bits = 1, kc_max = 64, kc_side[2] = {0, 0};
    u8* code = (u8*)e_alpha.get(64 + 256);
    {
        u32* used = (u32*)code + 64;
        LZ_HIP(hipMemsetAsync(used, 0, 1024, st));
        k_text_alpha<<<std::min<u64>(std::max<u64>(1, cdiv(n / 16, 256)), 2048), 256, 0, st>>>(d_text, n, used);
        u32 hu[256];
        LZ_HIP(hipMemcpyAsync(hu, used, 1024, hipMemcpyDeviceToHost, st));
        LZ_HIP(hipStreamSynchronize(st));
        u8 hc[256];
        u32 sigma = 0;
        for (int ch = 0; ch < 256; ch++) {
            hc[ch] = (u8)sigma;
            sigma += hu[ch] ? 1u : 0u;
        }
        while ((1u << bits) < sigma) bits++;
        kc_max = 64 / bits;
        LZ_HIP(hipMemcpyAsync(code, hc, 256, hipMemcpyHostToDevice, st));
        LZ_HIP(hipStreamSynchronize(st));  // (hc lives in this block)
    }
    u32* PA = e_PA.get(c);
    u32* SA = e_SA.get(c);
    u32* PAR = e_PAR.get(c);
    u32* SAR = e_SAR.get(c);
    {
        u64* key = e_key.get(c);
        u64* key2 = e_key2.get(c);
        u64* keyid = e_key3.get(c);
        u32* id = e_tmp1.get(c);
        u32* tmp = e_tmp2.get(c);
        for (int left = 1; left >= 0; left--) {
            u32* X = left ? PA : SA;
            const u32 kc = left ? std::min<u32>(kc_max, delta + 1) : kc_max;
            k_smpl_keys<<<cdiv(c, 256), 256, 0, st>>>(d_text, n, C, c, left, code, bits, kc, key, id);
            LZ_HIP(hipMemcpyAsync(keyid, key, (size_t)c * 8, hipMemcpyDeviceToDevice, st));
            const int kbits = (int)(bits * kc);
            size_t tb = 0;
            LZ_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, key, key2, id, X, (int)c, 0, kbits, st));
            u8* t = scan_tmp.get(tb);
            LZ_HIP(hipcub::DeviceRadixSort::SortPairs(t, tb, key, key2, id, X, (int)c, 0, kbits, st));
            SMPL_STAGE(left ? "radix PA" : "radix SA");
            merge_sort_u32(X, tmp, c, smpl_less{LV, C, keyid, delta, left}, st);
            SMPL_STAGE(left ? "merge PA" : "merge SA");
            k_rank_of<<<cdiv(c, 256), 256, 0, st>>>(X, c, left ? PAR : SAR);
            k_pre_table<<<cdiv(65537, 256), 256, 0, st>>>(key2, c, (u32)kbits, (left ? e_preL : e_preR).get(65537));
            kc_side[left ? 0 : 1] = kc;
        }
    }
    u32* Pi = e_Pi.get(c);
    u32* Psi = e_Psi.get(c);
    k_pi_psi<<<cdiv(c, 256), 256, 0, st>>>(PA, SA, PAR, SAR, c, Pi, Psi);
    timer.mark("smpl_index"); SMPL_STAGE("smpl_index");
    // the decomposed grid (decomposed_range.hpp:82-130, static_weighted_square_grid.hpp:67-104)
    u32 hh[256];
    {
        u32* hist = e_tmp1.get(256);
        LZ_HIP(hipMemsetAsync(hist, 0, 1024, st));
        k_char_hist<<<std::min<unsigned>(cdiv(c, 256), 1024), 256, 0, st>>>(d_text, C, c, hist);
        LZ_HIP(hipMemcpyAsync(hh, hist, 1024, hipMemcpyDeviceToHost, st));
        LZ_HIP(hipStreamSynchronize(st));
    }
    // one grid per character block: the phrase searches' (cells of at least SG_WIN ranks, at most
    // SG_GMAX per side) or, with ref = true, the reference's own (windows of exactly RG_WIN ranks,
    // div_ceil(frq, RG_WIN) per side) for the source pass.  Returns false when the cells would
    // take more than max_bytes.
    struct grid_set {
        const u32* cs;  // [CS 257 | first cell 257 | cells per side 256 | cell width 256]
        const u32* cell;
        const u32* gx;
        const u32* gy;
        const u32* gw;
        const u32* rst[RST_MAX];
        u32 ncell;
    };
    auto build_grid = [&](bool ref, dbuf<u32>& cs_b, dbuf<u32>& gx_b, dbuf<u32>& gy_b, dbuf<u32>& gw_b,
                          dbuf<u32>& cell_b, dbuf<u32>* rst_b, u64 max_bytes, grid_set& G) -> bool {
        u32 hCS[257], hgcb[257], hgwd[256], hwin[256];
        u64 ncell64 = 0;
        u32 wmax = 1;
        hCS[0] = 0;
        hgcb[0] = 0;
        for (int ch = 0; ch < 256; ch++) {
            hCS[ch + 1] = hCS[ch] + hh[ch];
            if (ref) {
                hgwd[ch] = (hh[ch] + RG_WIN - 1) / RG_WIN;
                hwin[ch] = RG_WIN;
            } else {
                hgwd[ch] = std::min<u32>((hh[ch] + SG_WIN - 1) / SG_WIN, SG_GMAX);
                hwin[ch] = hgwd[ch] ? (hh[ch] + hgwd[ch] - 1) / hgwd[ch] : SG_WIN;
            }
            ncell64 += (u64)hgwd[ch] * hgwd[ch];
            if (ncell64 >= 0xFFFFFFF0ull) return false;
            hgcb[ch + 1] = (u32)ncell64;
            wmax = std::max(wmax, hgwd[ch]);
        }
        u32 nlv = 1;  // row levels k with 2^k <= the widest row
        while (nlv < RST_MAX && (2ull << (nlv - 1)) <= wmax) nlv++;
        if ((2ull << (nlv - 1)) <= wmax) return false;
        const u32 ncell = (u32)ncell64;
        if ((u64)(ncell + 1) * 4 * (nlv + 1) > max_bytes) return false;
        u32* dCS = cs_b.get(257 + 257 + 256 + 256);
        LZ_HIP(hipMemcpyAsync(dCS, hCS, 257 * 4, hipMemcpyHostToDevice, st));
        LZ_HIP(hipMemcpyAsync(dCS + 257, hgcb, 257 * 4, hipMemcpyHostToDevice, st));
        LZ_HIP(hipMemcpyAsync(dCS + 514, hgwd, 256 * 4, hipMemcpyHostToDevice, st));
        LZ_HIP(hipMemcpyAsync(dCS + 770, hwin, 256 * 4, hipMemcpyHostToDevice, st));
        LZ_HIP(hipStreamSynchronize(st));  // (the host arrays live in this frame)
        u32* gx = gx_b.get(c);
        u32* gy = gy_b.get(c);
        u32* gw = gw_b.get(c);
        u32* cell = cell_b.get((u64)ncell + 1);
        {
            u64* key = e_key.get(c);
            u64* key2 = e_key2.get(c);
            u32* id = e_tmp1.get(c);
            u32* id2 = e_tmp2.get(c);
            k_grid_keys<<<cdiv(c, 256), 256, 0, st>>>(d_text, C, c, PAR, SAR, dCS, dCS + 257, dCS + 514, dCS + 770,
                                                      key, id);
            size_t tb = 0;
            LZ_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, key, key2, id, id2, (int)c, 0, 64, st));
            u8* t = scan_tmp.get(tb);
            LZ_HIP(hipcub::DeviceRadixSort::SortPairs(t, tb, key, key2, id, id2, (int)c, 0, 64, st));
            k_grid_points<<<cdiv((u64)c + 1, 256), 256, 0, st>>>(key2, PAR, SAR, c, gx, gy, gw, cell, ncell);
        }
        // row sparse tables over the cells' lightest weights (levels 0 .. nlv - 1)
        u32* lv0 = rst_b[0].get((u64)ncell + 1);
        if (ncell) k_cell_min<<<cdiv(ncell, 256), 256, 0, st>>>(cell, gw, ncell, lv0);
        G.rst[0] = lv0;
        for (u32 k = 1; k < nlv; k++) {
            u32* out = rst_b[k].get((u64)ncell + 1);
            if (ncell)
                k_cell_rowmin<<<cdiv(ncell, 256), 256, 0, st>>>(rst_b[k - 1].p, dCS + 514, dCS + 257, ncell,
                                                                 1u << (k - 1), out);
            G.rst[k] = out;
        }
        for (u32 k = nlv; k < RST_MAX; k++) G.rst[k] = nullptr;
        G.cs = dCS;
        G.ncell = ncell;
        G.cell = cell;
        G.gx = gx;
        G.gy = gy;
        G.gw = gw;
        return true;
    };
    grid_set G1{};
    if (!build_grid(false, e_CS, e_gx, e_gy, e_gw, e_cell, e_rst, ~0ull, G1))
        throw error(LZ77SSS_EINTERNAL, "exact-smpl: grid too large");
    auto set_grid = [](smpl_view& W, const grid_set& G) {
        W.CS = G.cs;
        W.gcb = G.cs + 257;
        W.gwd = G.cs + 514;
        W.gwin = G.cs + 770;
        for (u32 k = 0; k < RST_MAX; k++) W.rst[k] = G.rst[k];
        W.cell = G.cell;
        W.gx = G.gx;
        W.gy = G.gy;
        W.gw = G.gw;
    };
    timer.mark("smpl_grid"); SMPL_STAGE("smpl_grid");
    smpl_view V{};
    V.L = LV;
    V.C = C;
    V.c = c;
    V.delta = delta;
    V.PA = PA;
    V.SA = SA;
    V.Pi = Pi;
    V.Psi = Psi;
    V.PAR = PAR;
    V.SAR = SAR;
    V.pre[0] = e_preL.p;
    V.pre[1] = e_preR.p;
    V.code = code;
    V.kbits_ch = bits;
    V.kc[0] = kc_side[0];
    V.kc[1] = kc_side[1];
    {
        const u64 nblk = (n >> 8) + 2;
        u32* wb = e_wblk.get(nblk);
        k_wblk<<<cdiv(c, 256), 256, 0, st>>>(C, c, nblk, wb);
        V.wblk = wb;
    }
    set_grid(V, G1);
    V.afst = afst;
    V.afact = afact;
    V.za = za;
    V.mode = transf_mode;
    V.small_t = SMALL_T;
    if (const char* e = std::getenv("LZ77SSS_SMPL_SMALL")) V.small_t = (u32)std::max(0L, std::atol(e));
    V.lane_scan = LANE_SCAN;
    if (const char* e = std::getenv("LZ77SSS_SMPL_LSCAN")) V.lane_scan = (u32)std::max(0L, std::atol(e));
    V.scan_t = SCAN_T;
    if (const char* e = std::getenv("LZ77SSS_SMPL_SCAN")) V.scan_t = (u32)std::max(0L, std::atol(e));
    build_adjacent(V);
    V.cyc = nullptr;
    if (std::getenv("LZ77SSS_SMPL_PROF")) {
        V.cyc = (unsigned long long*)e_cyc.get(32);
        LZ_HIP(hipMemsetAsync(V.cyc, 0, 256, st));
        const char* sp = std::getenv("LZ77SSS_SMPL_PROF_SPLIT");
        V.prof_split = sp ? (u32)std::atoll(sp) : 0u;
    }
    // the chain (chunk walks + bridges, then the path from position 0 by pointer doubling).
    // Chunks hold cp approximate phrases each (the walks re-synchronise with the true chain
    // within a few phrases, so longer chunks leave less to the bridges); cut by phrase count, not
    // bytes, so a low-compressibility stretch (short phrases) does not give a few walks most of
    // the work; at least SMPL_WALKS walks (four per wave slot of the chip) while cp >= 32
#ifdef LZ_SMPL_CHECK
    static u32* s_chk = nullptr;
    if (!s_chk) LZ_HIP(hipMalloc(&s_chk, 64));
    LZ_HIP(hipMemsetAsync(s_chk, 0, 64, st));
    LZ_HIP(hipMemcpyToSymbolAsync(HIP_SYMBOL(g_smpl_chk), &s_chk, sizeof(s_chk), 0, hipMemcpyHostToDevice, st));
    u64 lims[8] = {c, G1.ncell, (n >> 8) + 2, za, n + TEXT_PAD, 0, 0, 0};
    LZ_HIP(hipMemcpyToSymbolAsync(HIP_SYMBOL(g_smpl_lim), lims, sizeof(lims), 0, hipMemcpyHostToDevice, st));
    LZ_HIP(hipStreamSynchronize(st));
    auto chk_report = [&](const char* where) {
        u32 h[5];
        LZ_HIP(hipMemcpy(h, s_chk, sizeof(h), hipMemcpyDeviceToHost));
        std::fprintf(stderr, "[lz77sss] smpl check %s: %s site %u index %llu limit %llu\n", where, h[0] ? "FAIL" : "ok",
                     h[0], (unsigned long long)h[1] | ((unsigned long long)h[2] << 32),
                     (unsigned long long)h[3] | ((unsigned long long)h[4] << 32));
    };
#endif
    u32 cp = (u32)std::max<u64>(32, std::min<u64>(SMPL_CHUNK, za / SMPL_WALKS));
    if (const char* e = std::getenv("LZ77SSS_SMPL_CHUNK")) cp = (u32)std::max(1L, std::atol(e));
    const u32 nch = (u32)(((u64)za + cp - 1) / cp);
    // task capacity: the chain (z <= z_approx) plus the walks before they merge; a full
    // table is detected and the walks rerun with four times the room
    u64 tcap64 = std::min<u64>(0x7FFFFFF0ull, 3 * (u64)za + 64 * (u64)nch + 65536);
    const bool prof_on = std::getenv("LZ77SSS_SMPL_PROF") != nullptr;
    u32* prof = prof_on ? e_tmp2.get(4 * (u64)nch + 4) : nullptr;
    task_tab Tt{};
    u32* ctr = counters.get(16);
    u32* full = ctr + 9;
    u32* bad = ctr + 10;
    u32* zp = ctr + 11;
    u32* ex = e_tmp1.get((u64)nch + 1);
    u32 hc[2];
    for (int attempt = 0;; attempt++) {
        const u32 tcap = (u32)tcap64;
        u32 hsz = 1;
        while (hsz < 2ull * tcap) hsz <<= 1;
        Tt.pos = e_tpos.get(tcap);
        Tt.len = e_tlen.get(tcap);
        Tt.src = e_tsrc.get(tcap);
        Tt.hop = e_thop.get(tcap);
        Tt.wk = e_twk.get(tcap);
        Tt.keys = e_tkeys.get(hsz);
        Tt.vals = e_tvals.get(hsz);
        Tt.mask = hsz - 1;
        Tt.cap = tcap;
        Tt.ntask = ctr + 8;
        LZ_HIP(hipMemsetAsync(Tt.keys, 0, (size_t)hsz * 4, st));
        LZ_HIP(hipMemsetAsync(ctr + 8, 0, 16, st));
        if (prof) LZ_HIP(hipMemsetAsync(prof, 0, (4 * (size_t)nch + 4) * 4, st));
        if (prof) k_chunk_walks<true><<<cdiv(nch, SWPB), 64 * SWPB, 0, st>>>(V, Tt, cp, nch, ex, full, prof);
        else k_chunk_walks<false><<<cdiv(nch, SWPB), 64 * SWPB, 0, st>>>(V, Tt, cp, nch, ex, full, nullptr);
        LZ_HIP(hipGetLastError());
        timer.mark("smpl_tasks"); SMPL_STAGE("smpl_tasks");
        if (prof) k_bridge_walks<true><<<cdiv(nch, SWPB), 64 * SWPB, 0, st>>>(V, Tt, nch, ex, full, prof + 2 * (u64)nch);
        else k_bridge_walks<false><<<cdiv(nch, SWPB), 64 * SWPB, 0, st>>>(V, Tt, nch, ex, full, nullptr);
        LZ_HIP(hipGetLastError());
        LZ_HIP(hipMemcpyAsync(hc, ctr + 8, 8, hipMemcpyDeviceToHost, st));
        LZ_HIP(hipStreamSynchronize(st));
        if (!hc[1] && hc[0] < tcap) break;
        if (attempt >= 3 || tcap64 >= 0x7FFFFFF0ull) throw error(LZ77SSS_EINTERNAL, "exact-smpl: task table full");
        tcap64 = std::min<u64>(0x7FFFFFF0ull, 4 * tcap64);
    }
    const u32 ntask = hc[0];
#ifdef LZ_SMPL_CHECK
    chk_report("walks");
#endif
    if (V.cyc) {
        u64 hcy[32];
        LZ_HIP(hipMemcpy(hcy, V.cyc, 256, hipMemcpyDeviceToHost));
        for (int bank = 0; bank < 2; bank++) {
            const u64* h = hcy + 16 * bank;
            const double tot = (double)(h[0] + h[1] + h[2] + h[7] + h[14]) + 1e-9, ph = (double)std::max<u64>(1, h[6]);
            std::fprintf(stderr,
                         "[lz77sss] smpl %s %u: phrases=%llu clocks/phrase=%.0f: position probes %.1f%% (searches "
                         "%.1f%%, %.1f steps; lighter %.1f%%, %.1f steps; %.1f lanes/phrase), PA interval %.1f%%, "
                         "witnesses %.1f%%, probe intervals %.1f%%, intersect %.1f%%; probes/phrase=%.2f "
                         "queries/probe=%.2f coop queries/probe=%.2f (left to the wave %.2f)\n",
                         bank ? "at/after" : "before", V.prof_split, (unsigned long long)h[6], tot / ph,
                         100 * h[0] / tot, 100 * h[8] / tot, (double)h[12] / ph, 100 * h[9] / tot, (double)h[11] / ph,
                         (double)h[13] / ph, 100 * h[14] / tot, 100 * h[1] / tot, 100 * h[7] / tot, 100 * h[2] / tot,
                         h[3] / ph, (double)h[5] / std::max<u64>(1, h[3]), (double)h[4] / std::max<u64>(1, h[3]),
                         (double)h[15] / std::max<u64>(1, h[3]));
        }
    }
    if (prof) {
        // per-walk profile (wall clock at 100 MHz): the slowest walks and the phrase totals
        std::vector<u32> hp(4 * (size_t)nch);
        LZ_HIP(hipMemcpy(hp.data(), prof, hp.size() * 4, hipMemcpyDeviceToHost));
        for (int br = 0; br < 2; br++) {
            std::vector<u32> tk(nch);
            u64 ph = 0, sum = 0;
            u32 mph = 0;
            for (u32 k = 0; k < nch; k++) {
                tk[k] = hp[2 * ((u64)br * nch + k)];
                const u32 q = hp[2 * ((u64)br * nch + k) + 1];
                ph += q;
                mph = std::max(mph, q);
                sum += tk[k];
            }
            std::vector<u32> s2 = tk;
            std::sort(s2.begin(), s2.end());
            const u32 kmax = (u32)(std::max_element(tk.begin(), tk.end()) - tk.begin());
            std::fprintf(stderr,
                         "[lz77sss] smpl %s: walks=%u phrases=%llu max_phrases=%u ticks sum=%.1f ms p50=%.1f us "
                         "p99=%.1f us max=%.1f us (walk %u, %u phrases, at %u)\n",
                         br ? "bridges" : "chunks", nch, (unsigned long long)ph, mph, sum / 1e5, s2[nch / 2] / 100.0,
                         s2[(u64)nch * 99 / 100] / 100.0, s2.back() / 100.0, kmax, hp[2 * ((u64)br * nch + kmax) + 1],
                         br ? 0u : kmax * cp);
        }
    }
    timer.mark("smpl_bridges"); SMPL_STAGE("smpl_bridges");
    // the path from the task at position 0: pointer doubling + top-down expansion (in order)
    u32 T_lv = 0;
    while ((1ull << T_lv) < (u64)ntask + 1) T_lv++;
    if (T_lv >= MAX_LV) throw error(LZ77SSS_EINTERNAL, "exact-smpl: too many tasks");
    k_task_next<<<cdiv((u64)ntask + 1, 256), 256, 0, st>>>(Tt, ntask, (u32)n, jump[0].get((u64)ntask + 1), bad);
    for (u32 t = 1; t < T_lv; t++)
        k_tjump<<<cdiv((u64)ntask + 1, 256), 256, 0, st>>>(jump[t - 1].p, ntask + 1, jump[t].get((u64)ntask + 1));
    u32* PC = e_tmp2.get(2ull << T_lv);
    u32* C2 = e_thop.get(2ull << T_lv);  // (task hops are not used by the chain)
    k_troot<<<1, 1, 0, st>>>(Tt, PC, ntask);
    u64 cnt = 1;
    for (int t = (int)T_lv - 1; t >= 0; t--) {
        k_texpand<<<cdiv(cnt, 256), 256, 0, st>>>(PC, cnt, jump[t].p, C2);
        std::swap(PC, C2);
        cnt *= 2;
    }
    LZ_HIP(hipMemcpyAsync(zp, &cnt, 4, hipMemcpyHostToDevice, st));  // no end marker: the path fills C
    k_path_len<<<cdiv(cnt, 256), 256, 0, st>>>(PC, cnt, ntask, zp);
    LZ_HIP(hipMemcpyAsync(hc, bad, 8, hipMemcpyDeviceToHost, st));
    LZ_HIP(hipStreamSynchronize(st));
    if (hc[0]) throw error(LZ77SSS_EINTERNAL, "exact-smpl: a task without its successor");
    const u64 z = hc[1];
    u32* F = fact.get(2 * z + 2);
    u32* FWK = e_fwk.get(z + 1);
    if (z) k_path_emit<<<cdiv(z, 256), 256, 0, st>>>(Tt, PC, (u32)z, F, FWK);
    LZ_HIP(hipGetLastError());
    LZ_HIP(hipStreamSynchronize(st));
    const u32 rounds = nch, walks = T_lv;
    timer.mark("smpl_chain"); SMPL_STAGE("smpl_chain");
    // the reference's sources (k_ref_sources) over its own grid, built now that the walks are
    // done; LZ77SSS_SMPL_OWN_SOURCES=1 keeps the phrase searches' witnesses (valid, not the
    // reference's), as does a reference grid that would not fit in half the free memory
    bool ref_src = false;
    if (z && !std::getenv("LZ77SSS_SMPL_OWN_SOURCES")) {
        size_t free_b = 0, tot_b = 0;
        LZ_HIP(hipMemGetInfo(&free_b, &tot_b));
        grid_set G2{};
        if (build_grid(true, e_CS2, e_gx2, e_gy2, e_gw2, e_cell2, e_rst2, (u64)free_b / 2, G2)) {
            smpl_view V2 = V;
            set_grid(V2, G2);
#ifdef LZ_SMPL_CHECK
            lims[1] = std::max(G1.ncell, G2.ncell);
            LZ_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_smpl_lim), lims, sizeof(lims)));
#endif
            V2.scan_t = RG_SCAN;
            V2.cyc = nullptr;
            u32* vis = e_vis.get(2 * (SMPL_MAX_DELTA + 1));
            u32 hsm[SMPL_MAX_DELTA + 1] = {};
            if (transf_mode == LZ77SSS_TRANSF_WITH_SAMPLES) {
                u32* hist = vis + SMPL_MAX_DELTA + 1;
                LZ_HIP(hipMemsetAsync(hist, 0, (SMPL_MAX_DELTA + 1) * 4, st));
                k_adj_hist<<<std::min<unsigned>(cdiv(c, 256), 1024), 256, 0, st>>>(V.pM.mn[0], c, hist);
                u32 hh2[SMPL_MAX_DELTA + 1];
                LZ_HIP(hipMemcpyAsync(hh2, hist, sizeof(hh2), hipMemcpyDeviceToHost, st));
                LZ_HIP(hipStreamSynchronize(st));
                sampled_left_lengths(hh2, c, delta, hsm);
            }
            LZ_HIP(hipMemcpyAsync(vis, hsm, sizeof(hsm), hipMemcpyHostToDevice, st));
            // phrase starts: exclusive sum of max(1, len)
            u32* lens = e_tmp1.get(z + 1);
            u32* fpos = e_fpos.get(z + 1);
            k_fact_len1<<<cdiv(z + 1, 256), 256, 0, st>>>(F, (u32)z, lens);
            size_t tb = 0;
            LZ_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, lens, fpos, (int)(z + 1), st));
            u8* t = scan_tmp.get(tb);
            LZ_HIP(hipcub::DeviceScan::ExclusiveSum(t, tb, lens, fpos, (int)(z + 1), st));
            u32* miss = ctr + 12;
            LZ_HIP(hipMemsetAsync(miss, 0, 4, st));
            k_ref_sources<<<cdiv(cdiv(z, 64), SWPB), 64 * SWPB, 0, st>>>(V2, F, fpos, FWK, (u32)z, vis, miss);
            LZ_HIP(hipGetLastError());
            u32 hm = 0;
            LZ_HIP(hipMemcpyAsync(&hm, miss, 4, hipMemcpyDeviceToHost, st));
            LZ_HIP(hipStreamSynchronize(st));
            if (hm) throw error(LZ77SSS_EINTERNAL, "exact-smpl: a phrase without a source in the reference's order");
            ref_src = true;
#ifdef LZ_SMPL_CHECK
            chk_report("sources");
#endif
        }
        timer.mark("smpl_sources"); SMPL_STAGE("smpl_sources");
    }
    num_fact = z;
    stats.resize(29, 0);
    stats[28] = ref_src ? 1 : 0;  // the sources follow the reference's visit order
    stats[24] = c;
    stats[25] = delta;
    stats[26] = ntask;
    stats[27] = ((u64)rounds << 32) | walks;  // chunks, doubling levels
    if (log) {
        for (auto& [name, ms] : timer.read()) std::fprintf(stderr, "[lz77sss] %-12s %9.3f ms\n", name.c_str(), ms);
        std::fprintf(stderr, "[lz77sss] exact-smpl: n=%llu approx=%u samples=%u delta=%u tasks=%llu chunks=%u levels=%u factors=%llu\n",
                     (unsigned long long)n, za, c, delta, (unsigned long long)stats[26], rounds, walks,
                     (unsigned long long)z);
        log_summary(t_start);
    }
    return z;
}

// the phrase searches' structures per order (PA: left contexts, SA: suffixes): the 16-byte
// context keys by rank, the adjacent LCEs (LCS_S / LCP_S of construction.cpp:118-129; left
// capped at delta) and their sparse-table minima
void engine::build_adjacent(smpl_view& V) {
    const u32 c = V.c;
    for (int side = 0; side < 2; side++) {
        const bool left = side == 0;
        const u32* X = left ? V.PA : V.SA;
        ulonglong2* keys = (ulonglong2*)(left ? e_kPA : e_kSA).get(2 * (u64)c + 2);
        k_ctx_keys<<<cdiv(c, 256), 256, 0, st>>>(d_text, n, V.C, X, c, left, keys);
        iv_levels M{};
        u32* adj = (left ? e_adjL : e_adjR).get((u64)c + 1);
        k_adj_lce<<<cdiv((u64)c + 1, 256), 256, 0, st>>>(V.L, V.C, X, c, V.delta, left, adj);
        M.mn[0] = adj;
        M.nlv = 1;
        dbuf<u32>* lv = left ? e_ivminL : e_ivmin;
        while ((2ull << (M.nlv - 1)) <= c && M.nlv < (u32)MAX_LV) {
            const u64 half = 1ull << (M.nlv - 1), cnt = (u64)c - 2 * half + 1;
            u32* out = lv[M.nlv].get(cnt);
            k_iv_min_level<<<cdiv(cnt, 256), 256, 0, st>>>(M.mn[M.nlv - 1], cnt, half, out);
            M.mn[M.nlv++] = out;
        }
        if (left) {
            V.pM = M;
            V.kPA = keys;
        } else {
            V.sM = M;
            V.kSA = keys;
        }
    }
    // minima of the weights (sample ids) by PA / SA rank
    V.wPA[0] = V.PA;
    V.wSA[0] = V.SA;
    V.wlv = 1;
    while ((2ull << (V.wlv - 1)) <= c && V.wlv < (u32)MAX_LV) {
        const u64 half = 1ull << (V.wlv - 1), cnt = (u64)c - 2 * half + 1;
        u32* o1 = e_wPA[V.wlv].get(cnt);
        u32* o2 = e_wSA[V.wlv].get(cnt);
        k_iv_min_level<<<cdiv(cnt, 256), 256, 0, st>>>(V.wPA[V.wlv - 1], cnt, half, o1);
        k_iv_min_level<<<cdiv(cnt, 256), 256, 0, st>>>(V.wSA[V.wlv - 1], cnt, half, o2);
        V.wPA[V.wlv] = o1;
        V.wSA[V.wlv] = o2;
        V.wlv++;
    }
    LZ_HIP(hipGetLastError());
    timer.mark("smpl_adj"); SMPL_STAGE("smpl_adj");
}

}  // namespace LZ_NS
