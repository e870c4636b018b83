// smpl.hip -- exact LZ77 through a sample index on the device: the exact-smpl path of
// configs[4] (lz77_sss<>::factorizer::exact_factorizer, include/lz77_sss/lz77_sss.hpp:558-709;
// transform_to_exact/{common,naive,without_samples,with_samples}.cpp; the sample index of
// data_structures/sample_index/{sample_index.hpp,construction.cpp,queries.cpp}; the
// Rabin-Karp substring fingerprints of data_structures/rabin_karp_substring.hpp; the
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
//            57-bit key of 7 characters, then a comparison merge sort whose comparator
//            falls back to the text (leftward LCE / the SSS-backed LCE of lce_dev.h)
//   points   (x = PA rank, y = SA rank, weight = sample id); Pi, Psi (common.cpp:114-182)
//   grid     per first character (decomposed_range.hpp:82-130) cells of >= SG_WIN ranks per side
//            ranks, points sorted by (cell, weight) (static_weighted_square_grid.hpp:67-104)
//   RKS      prefix fingerprints mod 2^31 - 1 every RKS_RATE characters
//            (rabin_karp_substring.hpp:77-172); with_samples: hash tables of the PA / SA
//            intervals of the sampled pattern lengths (construction.cpp:108-305)
//   phrases  one wave per phrase start i; lane j in [i, i + delta) finds the PA interval
//            of T[i..j] (extend_left, queries.cpp:67-275) and the longest right extension
//            lce_r whose SA interval holds a point lighter than the first sample >= j
//            (exp/binary search over lce_r, intersect of common.cpp:258-358, decided for
//            the whole wave one query at a time: the Pi / Psi scan below SCAN_T ranks,
//            the grid above); the wave keeps the longest, the smallest j on ties
//   chain    chunk walks: one wave per chunk of ~32 approximate phrases walks the greedy
//            chain from the chunk start (a task per phrase, in a hash table) until it meets
//            another walk's task or passes its chunk end; bridges walk on from every chunk
//            exit until they meet a task; the chain from position 0 is then marked in order
//            by pointer doubling + top-down expansion over the successor tasks
//
// Lengths are the canonical greedy LZ77 lengths (every leftmost occurrence of a phrase
// contains a sample within its first delta characters: DESIGN.md 4.8); sources are the
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

constexpr u32 SMPL_MAX_DELTA = 256;  // lz77_sss.hpp:81 max_delta
constexpr u32 SCAN_T = 4096;         // lz77_sss.hpp:83 range_scan_threshold
constexpr u32 SMALL_T = 32;          // intersect queries scanned by their own lane (no wave round trip)
#ifndef LZ_SG_WIN
#define LZ_SG_WIN 2048
#endif
constexpr u32 SG_WIN = LZ_SG_WIN;    // smallest grid cell width in ranks (the reference: 16384 on a CPU core)
constexpr u32 SG_GMAX = 512;         // cells per side at most: wider blocks get wider cells
constexpr u32 SG_LV = 10;            // row sparse-table levels (2^9 = SG_GMAX / 1)
constexpr u32 RKS_RATE = 16;         // lz77_sss.hpp:82 rks_sample_rate
constexpr u32 RKS_P = 0x7FFFFFFFu;   // Mersenne prime 2^31 - 1 (rabin_karp_substring<31>)
constexpr u32 RKS_B = 0x2545F491u % RKS_P;  // fixed base (the reference draws one per run)
constexpr u32 SWPB = 4;              // waves per workgroup of the phrase kernels
constexpr u32 NSMPL = 24;            // sampled pattern lengths per side at most (with_samples)

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
    const u32* rst[SG_LV];   // per row of cells: min weight over cells [x, x + 2^k) of the row
    const u32* gx;           // points by (cell, weight): PA rank, SA rank, weight
    const u32* gy;
    const u32* gw;
    const u32* afst;         // approximate phrase starts [za + 1]
    const u32* afact;        // approximate factors (src, len)
    u32 za;
    int mode;                // LZ77SSS_TRANSF_*
    u32 small_t;             // intersect queries with a side of at most this many ranks run on their own lane
    // with_samples: RKS + interval samples
    const u32* rks;          // fps[k] = fp(T[0 .. k * RKS_RATE))
    const u32* pw_lo;        // b^e, e <= sq
    const u32* pw_hi;        // b^(sq * e)
    u32 sq;
    const u64* hkey;         // interval hash: (side << 63 | len idx << 40 | fp) + 1, 0 empty
    const u64* hval;         // (b << 32 | e)
    u64 hmask;
    u32 nlen[2];             // sampled lengths per side (0 = LEFT, 1 = RIGHT), the first two are 1, 2
    u32 slen[2][NSMPL];
};

__device__ __forceinline__ u32 mod31(u64 v) {
    v = (v >> 31) + (v & RKS_P);
    v = (v >> 31) + (v & RKS_P);
    return (u32)(v >= RKS_P ? v - RKS_P : v);
}
__device__ __forceinline__ u32 rks_pow(const smpl_view& V, u64 e) {
    return mod31((u64)V.pw_hi[e / V.sq] * V.pw_lo[e % V.sq]);
}
// fingerprint of T[0 .. x) (rabin_karp_substring.hpp:223-230)
__device__ __forceinline__ u32 rks_upto(const smpl_view& V, u64 x) {
    const u64 blk = x / RKS_RATE;
    u32 fp = V.rks[blk];
    for (u64 p = blk * RKS_RATE; p < x; p++) fp = mod31((u64)fp * RKS_B + V.L.T[p]);
    return fp;
}
// fingerprint of T[pos .. pos + len) (rabin_karp_substring.hpp:232-239)
__device__ __forceinline__ u32 rks_sub(const smpl_view& V, u64 pos, u64 len) {
    const u32 a = mod31((u64)rks_upto(V, pos) * rks_pow(V, len)), b = rks_upto(V, pos + len);
    return b >= a ? b - a : RKS_P - (a - b);
}

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

// extend (queries.cpp:67-275 without interval samples): the ranks [b, e] of the order
// (left: PA, right: SA) whose sample contexts match the pattern at pp of length len,
// searched inside [b, e] whose contexts share lb / le characters with the pattern at
// the two ends.  Returns false if none matches.
template <bool LEFT>
__device__ bool extend_iv(const smpl_view& V, u32 pp, u32 len, u32& b, u32& e, u32& lb, u32& le) {
    const u32* X = LEFT ? V.PA : V.SA;
    auto lce_at = [&](u32 r, u32 offs) -> u32 {
        const u32 pm = V.C[X[r]];
        if (LEFT) return lce_left_offs(V, pm, pp, offs, len);
        return min(lce_right_offs(V, pm, pp, offs), max(len, offs));
    };
    auto less_at = [&](u32 r, u32 l) -> bool {
        const u32 pm = V.C[X[r]];
        return LEFT ? less_left(V, pm, pp, l) : less_right(V, pm, pp, l);
    };
    if (lb < len) lb = lce_at(b, lb);
    if (le < len) le = (e == b) ? lb : lce_at(e, le);
    // first matching rank: l "less than the pattern", r "matching or greater"
    u32 nb, nlb;
    if (lb >= len) {
        nb = b;
        nlb = lb;
    } else {
        if (!less_at(b, lb)) return false;              // every rank greater
        if (le < len && less_at(e, le)) return false;   // every rank less
        u32 l = b, r = e, ll = lb, lr = le;
        while (r - l > 1) {
            const u32 m = l + (r - l) / 2;
            const u32 lm = lce_at(m, min(ll, lr));
            if (lm < len && less_at(m, lm)) {
                l = m;
                ll = lm;
            } else {
                r = m;
                lr = lm;
            }
        }
        if (lr < len) return false;
        nb = r;
        nlb = lr;
    }
    // last matching rank: l matching, r not
    u32 ne, nle;
    if (le >= len) {
        ne = e;
        nle = le;
    } else {
        u32 l = nb, r = e, ll = nlb, lr = le;
        while (r - l > 1) {
            const u32 m = l + (r - l) / 2;
            const u32 lm = lce_at(m, min(ll, lr));
            if (lm >= len) {
                l = m;
                ll = lm;
            } else {
                r = m;
                lr = lm;
            }
        }
        ne = l;
        nle = ll;
    }
    b = nb;
    e = ne;
    lb = nlb;
    le = nle;
    return true;
}

// interval samples (sxa_interval, queries.cpp:31-65): the interval of the sampled length
// index k at pp, by fingerprint, verified against the interval's first sample
template <bool LEFT>
__device__ bool sampled_iv(const smpl_view& V, u32 k, u32 pp, u32 fp, u32& b, u32& e) {
    const u32 len = V.slen[LEFT ? 0 : 1][k];
    const u64 key = (((u64)(LEFT ? 0 : 1) << 63) | ((u64)k << 40) | fp) + 1;
    u64 h = (key * 0x9E3779B97F4A7C15ull) >> 20;
    for (u32 probe = 0; probe <= V.hmask; probe++, h++) {
        const u64 kk = V.hkey[h & V.hmask];
        if (kk == 0) return false;
        if (kk != key) continue;
        const u64 v = V.hval[h & V.hmask];
        const u32 rb = (u32)(v >> 32), re = (u32)v;
        const u32 pm = V.C[(LEFT ? V.PA : V.SA)[rb]];
        const u32 l = LEFT ? lce_left_offs(V, pm, pp, 0, len) : min(lce_right_offs(V, pm, pp, 0), len);
        if (l >= len) {
            b = rb;
            e = re;
            return true;
        }
    }
    return false;
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
                    const u32 yy = V.Pi[x];
                    if (V.PA[x] < W && yy >= yb && yy <= ye) {
                        found = true;
                        py = yy;
                        break;
                    }
                }
            } else {
                for (u32 yy = yb; yy <= ye; yy++) {
                    const u32 xx = V.Psi[yy];
                    if (V.SA[yy] < W && xx >= xb && xx <= xe) {
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
        if (V.mode != LZ77SSS_TRANSF_NAIVE && min(rx, ry) <= SCAN_T) {
            // scan the smaller interval through Pi / Psi
            if (rx <= ry) {
                for (u32 base = qxb; base <= qxe; base += 64) {
                    const u32 x = base + lane;
                    u32 yy = 0;
                    bool ok = false;
                    if (x <= qxe) {
                        yy = V.Pi[x];
                        ok = V.PA[x] < qW && yy >= qyb && yy <= qye;
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
                        const u32 xx = V.Psi[yy];
                        ok = V.SA[yy] < qW && xx >= qxb && xx <= qxe;
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
                        ok = min(R[o + xi1], R[o + xi2 - (1u << k)]) < qW;
                    }
                    const u64 bal = __ballot(ok);
                    if (bal) {
                        // the row's first cell with a lighter point: its lightest point
                        const u32 row1 = base + (u32)__builtin_ctzll(bal), o = cb + row1 * gw;
                        for (u32 xb = xi1; xb < xi2; xb += 64) {
                            const u32 cx = xb + lane;
                            const bool hit = cx < xi2 && V.rst[0][o + cx] < qW;
                            const u64 hb = __ballot(hit);
                            if (hb) {
                                const u32 cid = o + xb + (u32)__builtin_ctzll(hb);
                                y = V.gy[V.cell[cid]];
                                f = true;
                                break;
                            }
                        }
                    }
                }
            }
            if (!f) {
                // border cells: full rows yw1 (< yi1) and yw2 (>= yi2) when not inner, and the
                // columns xw1 (< xi1) and xw2 (>= xi2) of the inner rows (every cell when there
                // is no inner part)
                const u32 nx = xw2 - xw1 + 1, ny = yw2 - yw1 + 1;
                const bool full = !inner;
                const u32 top = full ? ny : (yw1 < yi1 ? 1u : 0u), bot = full ? 0u : (yw2 >= yi2 ? 1u : 0u);
                const u32 lc = (!full && xw1 < xi1) ? 1u : 0u, rc = (!full && xw2 >= xi2) ? 1u : 0u;
                const u32 nin = full ? 0u : yi2 - yi1;
                const u32 nrow = (top + bot) * nx, ncol = (lc + rc) * nin, nb = nrow + ncol;
                for (u32 base = 0; base < nb && !f; base += 64) {
                    const u32 t = base + lane;
                    bool ok = false;
                    u32 yy = 0;
                    if (t < nb) {
                        u32 cx, cy;
                        if (t < nrow) {
                            const u32 r = t / nx;
                            cy = r < top ? yw1 + r : yw2;
                            cx = xw1 + t % nx;
                        } else {
                            const u32 u = t - nrow, side = lc ? u / nin : 1u;
                            cy = yi1 + u % nin;
                            cx = side == 0 ? xw1 : xw2;
                        }
                        const u32 cid = cb + cy * gw + cx;
                        const u32 p1 = V.cell[cid + 1];
                        for (u32 q = V.cell[cid]; q < p1; q++) {
                            if (V.gw[q] >= qW) break;
                            const u32 xx = V.gx[q], y3 = V.gy[q];
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

// first sample index x with C[x] >= j (adjust_xc, common.cpp:184-196)
__device__ __forceinline__ u32 first_sample_geq(const smpl_view& V, u32 j) {
    u32 lo = 0, hi = V.c;
    while (lo < hi) {
        const u32 m = (lo + hi) >> 1;
        if (V.C[m] < j) lo = m + 1; else hi = m;
    }
    return lo;
}

// ---- one exact phrase at i (transform_to_exact_{naive,without_samples,with_samples}) --
// executed by a whole wave; returns (src, len) in every lane
__device__ void wave_phrase(const smpl_view& V, u32 i, u32& f_src, u32& f_len, u32 lane) {
    const u32 n = (u32)V.L.n;
    const u32 e = n;  // one section: p = 1
    const u8* T = V.L.T;
    // lower bound: the approximate phrase covering i, cut at i (without_samples.cpp:64-77)
    f_src = T[i];
    f_len = 0;
    if (V.mode != LZ77SSS_TRANSF_NAIVE) {
        u32 lo = 0, hi = V.za;  // largest k with afst[k] <= i
        while (hi - lo > 1) {
            const u32 m = (lo + hi) >> 1;
            if (V.afst[m] <= i) lo = m; else hi = m;
        }
        const u32 alen = V.afact[2 * lo + 1];
        if (alen != 0) {
            const u32 nxt = V.afst[lo + 1];
            const u32 cut = alen - (nxt - i);
            f_len = alen - cut;
            f_src = V.afact[2 * lo] + cut;
        }
    }
    const u32 max_j = min<u32>(e, i + V.delta);
    for (u32 j0 = i; j0 < max_j; j0 += 64) {
        const u32 j = j0 + lane;
        const bool act = j < max_j;
        const u32 lce_l = j - i + 1;
        const u32 ch = act ? T[j] : 0u;
        // PA interval of T[i..j] (extend_left; with_samples: the sampled lengths by fingerprint)
        u32 xb = V.CS[ch], xe = V.CS[ch + 1] - 1, xlb = 1, xle = 1;
        bool okl = act && V.CS[ch + 1] > V.CS[ch];
        if (okl && lce_l > 1) {
            if (V.mode == LZ77SSS_TRANSF_WITH_SAMPLES) {
                // the longest sampled length <= lce_l narrows the search (extend<LEFT> with samples)
                u32 k = 0;
                while (k + 1 < V.nlen[0] && V.slen[0][k + 1] <= lce_l) k++;
                if (k >= 2) {
                    u32 b2, e2;
                    const u32 L0 = V.slen[0][k];
                    if (sampled_iv<true>(V, k, j, rks_sub(V, j + 1 - L0, L0), b2, e2)) {
                        xb = b2;
                        xe = e2;
                        xlb = xle = L0;
                    } else {
                        okl = false;
                    }
                }
            }
            if (okl) okl = extend_iv<true>(V, j, lce_l, xb, xe, xlb, xle);
        }
        // right extensions: max lce_r in [lce_r_min, e - j] with a lighter point (exp search,
        // then binary search; common.cpp intersect decides each probe)
        const u32 lrmin = (f_len < j - i) ? 0u : (i + f_len - j);
        const u32 lrmax = e - j;
        u32 lo = lrmin, hi = lrmax + 1, step = 1;
        bool bin = false;
        bool run = okl && lo < lrmax;
        u32 yb = V.CS[ch], ye = V.CS[ch + 1] - 1, ylb = 1, yle = 1;
        const u32 W = act ? first_sample_geq(V, j) : 0u;
        u32 best_y = 0;
        bool got = false;
        while (__ballot(run)) {
            u32 x = 0, nb = yb, ne = ye, nlb = ylb, nle = yle;
            bool cand = false;
            if (run) {
                x = bin ? lo + (hi - lo) / 2 : min(lo + step, hi - 1);
                cand = true;
                if (V.mode == LZ77SSS_TRANSF_WITH_SAMPLES) {
                    // extend_right_with_samples (with_samples.cpp:35-122): the longest sampled
                    // length <= x beyond the known match narrows the interval by fingerprint
                    u32 k = 0;
                    while (k + 1 < V.nlen[1] && V.slen[1][k + 1] <= x) k++;
                    const u32 L1 = V.slen[1][k];
                    if (k >= 2 && L1 > min(nlb, nle)) {
                        u32 b2, e2;
                        if (sampled_iv<false>(V, k, j, rks_sub(V, j, L1), b2, e2)) {
                            nb = b2;
                            ne = e2;
                            nlb = nle = L1;
                        } else {
                            cand = false;
                        }
                    }
                }
                if (cand) cand = extend_iv<false>(V, j, x, nb, ne, nlb, nle);
            }
            bool f;
            u32 py;
            wave_intersect(V, cand, xb, xe, nb, ne, W, ch, f, py, lane);
            if (run) {
                if (cand && f) {
                    lo = x;
                    yb = nb;
                    ye = ne;
                    ylb = nlb;
                    yle = nle;
                    best_y = py;
                    got = true;
                    if (!bin) step *= 2;
                } else {
                    hi = x;
                    bin = true;
                }
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
        u32 src = got ? V.C[V.SA[best_y]] - lce_l + 1 : 0u;
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
        }
    }
    if (f_len > e - i) f_len = e - i;
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
__global__ void k_smpl_keys(const u8* __restrict__ T, u64 n, const u32* __restrict__ C, u32 c, int left,
                            u64* __restrict__ key, u32* __restrict__ id) {
    const u64 k = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= c) return;
    const u64 p = C[k];
    u64 v = 0;
    for (int t = 0; t < 7; t++) {
        u64 d;
        if (left) d = p >= (u64)t ? (u64)T[p - t] + 1 : 0;
        else d = p + t < n ? (u64)T[p + t] + 1 : 0;
        v = v * 257 + d;
    }
    key[k] = v;
    id[k] = (u32)k;
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
        const u64 l = dev_lce(L, pa, pb);
        if ((u64)max(pa, pb) + l >= L.n) return pa > pb;
        return L.T[pa + l] < L.T[pb + l];
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

// RKS block fingerprints: (fp(T[16k .. 16k + 16)), b^len) per block, then an inclusive scan
// with the concatenation (fa, pa) . (fb, pb) = (fa pb + fb, pa pb) (rabin_karp_substring.hpp:205-208)
__global__ void k_rks_blocks(const u8* __restrict__ T, u64 n, u64 nb, u64* __restrict__ out) {
    const u64 k = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= nb) return;
    u32 fp = 0, pw = 1;
    for (u64 p = k * RKS_RATE; p < (k + 1) * RKS_RATE && p < n; p++) {
        fp = mod31((u64)fp * RKS_B + T[p]);
        pw = mod31((u64)pw * RKS_B);
    }
    out[k] = ((u64)pw << 32) | fp;
}
struct rks_cat {
    __device__ u64 operator()(const u64& a, const u64& b) const {
        const u32 fa = (u32)a, pa = (u32)(a >> 32), fb = (u32)b, pb = (u32)(b >> 32);
        return ((u64)mod31((u64)pa * pb) << 32) | mod31((u64)fa * pb + fb);
    }
};
__global__ void k_rks_shift(const u64* __restrict__ incl, u64 nb, u32* __restrict__ fps) {
    const u64 k = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (k <= nb) fps[k] = k == 0 ? 0u : (u32)incl[k - 1];
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
// interval samples of one sampled length (construction.cpp:265-305): every maximal rank
// interval whose adjacent LCEs are >= len, keyed by the fingerprint of its context
// the interval's end: the last e with adj[r + 1 .. e] >= len, by binary lifting over the
// sparse-table minima of adj (levels mn[l][i] = min adj[i .. i + 2^l)); a linear scan took
// seconds on repetitive text, where one interval spans millions of samples
struct iv_levels { const u32* mn[MAX_LV]; u32 nlv; };
__device__ __forceinline__ u32 iv_end(const iv_levels& M, const u32* adj, u32 c, u32 r, u32 len) {
    u64 pos = (u64)r + 1;  // adj[r + 1 .. pos) are all >= len
    for (int l = (int)M.nlv - 1; l >= 0; l--) {
        const u64 w = 1ull << l;
        if (pos + w <= c && M.mn[l][pos] >= len) pos += w;
    }
    return (u32)(pos - 1);
}
__global__ void k_iv_min_level(const u32* __restrict__ prev, u64 cnt, u64 half, u32* __restrict__ out) {
    const u64 k = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (k < cnt) out[k] = min(prev[k], prev[k + half]);
}
__global__ void k_iv_insert(const smpl_view V, const u32* __restrict__ X, const u32* __restrict__ adj, u32 c,
                            int left, u32 k, u32 len, u64* __restrict__ hkey, u64* __restrict__ hval, u64 hmask,
                            iv_levels M) {
    const u64 r = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= c) return;
    if (r > 0 && adj[r] >= len) return;  // not an interval start
    const u32 e = iv_end(M, adj, c, (u32)r, len);
    const u32 pm = V.C[X[r]];
    if (left ? pm + 1 < len : (u64)pm + len > V.L.n) return;  // context shorter than len
    const u32 fp = left ? rks_sub(V, pm + 1 - len, len) : rks_sub(V, pm, len);
    const u64 key = (((u64)(left ? 0 : 1) << 63) | ((u64)k << 40) | fp) + 1;
    u64 h = (key * 0x9E3779B97F4A7C15ull) >> 20;
    for (;; h++) {
        const u64 old = atomicCAS((unsigned long long*)&hkey[h & hmask], 0ull, (unsigned long long)key);
        if (old == 0) {
            hval[h & hmask] = ((u64)r << 32) | e;
            return;
        }
    }
}

// ---------------------------------------------------------------------------
// chain kernels: task table (position -> phrase), a hash map position -> task id
struct task_tab {
    u32* pos;
    u32* len;
    u32* src;
    u32* hop;
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
// Chunk k's wave walks the greedy chain from k * CS, inserting a task per phrase, until it
// meets a task another walk inserted (merged) or passes its chunk end (its exit is kept).
// A bridge walks from every exit until it meets a task.  Every task's successor position
// then holds a task (a walk inserts it, finds it, or hands it to a bridge), so the chain
// from position 0 lies in the table; it is marked by pointer doubling.
__device__ __forceinline__ u32 wave_walk(const smpl_view& V, task_tab& Tt, u64 p, u64 stop, u32 lane, u32* __restrict__ full) {
    const u64 n = V.L.n;
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
        u32 src, len;
        wave_phrase(V, (u32)p, src, len, lane);
        if (lane == 0) {
            Tt.src[t] = src;
            Tt.len[t] = len;
        }
        p += max(1u, len);
    }
}
__global__ __launch_bounds__(64 * SWPB) void k_chunk_walks(const smpl_view V, task_tab Tt, u64 CS, u32 nch,
                                                          u32* __restrict__ ex, u32* __restrict__ full) {
    const u32 lane = threadIdx.x & 63;
    const u32 k = blockIdx.x * SWPB + (threadIdx.x >> 6);
    if (k >= nch) return;
    const u32 e = wave_walk(V, Tt, (u64)k * CS, min<u64>(V.L.n, (u64)(k + 1) * CS), lane, full);
    if (lane == 0) ex[k] = e;
}
__global__ __launch_bounds__(64 * SWPB) void k_bridge_walks(const smpl_view V, task_tab Tt, u32 nch,
                                                           const u32* __restrict__ ex, u32* __restrict__ full) {
    const u32 lane = threadIdx.x & 63;
    const u32 k = blockIdx.x * SWPB + (threadIdx.x >> 6);
    if (k >= nch || ex[k] == NONE) return;
    wave_walk(V, Tt, ex[k], ~0ull, lane, full);
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
__global__ void k_path_emit(task_tab Tt, const u32* __restrict__ C, u32 z, u32* __restrict__ F) {
    const u64 m = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (m >= z) return;
    const u32 t = C[m];
    F[2 * m] = Tt.src[t];
    F[2 * m + 1] = Tt.len[t];
}

// ---------------------------------------------------------------------------
// host side
static u32 pow31_host(u64 b, u64 e) {
    u64 r = 1 % RKS_P, x = b % RKS_P;
    while (e) {
        if (e & 1) r = r * x % RKS_P;
        x = x * x % RKS_P;
        e >>= 1;
    }
    return (u32)r;
}

u64 engine::factorize_exact_smpl(int transf_mode, int phr_mode, u32 rk_seed, int log2_override, bool log) {
    LZ_HIP(hipSetDevice(device));
    if (n > 0xFFFFFFF0ull) throw error(LZ77SSS_EINVAL, "n too large for pos_t = uint32_t");
    const auto t_start = std::chrono::steady_clock::now();
    if (log) g_dev_peak.store(g_dev_bytes.load());
    // the 3-approximation (compute_approximation, lz77_sss.hpp:324)
    const u64 za64 = factorize(phr_mode, rk_seed, log2_override, false, LZ77SSS_GREEDY);
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
    timer.mark("smpl_set");
    const lce_view LV = view(d_text);
    // PA / SA (sample_index.hpp:317-353): radix sort by 7 characters, merge sort by the text
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
            k_smpl_keys<<<cdiv(c, 256), 256, 0, st>>>(d_text, n, C, c, left, key, id);
            LZ_HIP(hipMemcpyAsync(keyid, key, (size_t)c * 8, hipMemcpyDeviceToDevice, st));
            size_t tb = 0;
            LZ_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, key, key2, id, X, (int)c, 0, 57, st));
            u8* t = scan_tmp.get(tb);
            LZ_HIP(hipcub::DeviceRadixSort::SortPairs(t, tb, key, key2, id, X, (int)c, 0, 57, st));
            merge_sort_u32(X, tmp, c, smpl_less{LV, C, keyid, delta, left}, st);
            k_rank_of<<<cdiv(c, 256), 256, 0, st>>>(X, c, left ? PAR : SAR);
        }
    }
    u32* Pi = e_Pi.get(c);
    u32* Psi = e_Psi.get(c);
    k_pi_psi<<<cdiv(c, 256), 256, 0, st>>>(PA, SA, PAR, SAR, c, Pi, Psi);
    timer.mark("smpl_index");
    // the decomposed grid (decomposed_range.hpp:82-130, static_weighted_square_grid.hpp:67-104)
    u32 hCS[257], hgcb[257], hgwd[256], hwin[256];
    u32* dCS = e_CS.get(257 + 257 + 256 + 256);
    {
        u32* hist = e_tmp1.get(256);
        LZ_HIP(hipMemsetAsync(hist, 0, 1024, st));
        k_char_hist<<<std::min<unsigned>(cdiv(c, 256), 1024), 256, 0, st>>>(d_text, C, c, hist);
        u32 hh[256];
        LZ_HIP(hipMemcpyAsync(hh, hist, 1024, hipMemcpyDeviceToHost, st));
        LZ_HIP(hipStreamSynchronize(st));
        hCS[0] = 0;
        hgcb[0] = 0;
        for (int ch = 0; ch < 256; ch++) {
            hCS[ch + 1] = hCS[ch] + hh[ch];
            // cells of at least SG_WIN ranks, at most SG_GMAX per side
            hgwd[ch] = std::min<u32>((hh[ch] + SG_WIN - 1) / SG_WIN, SG_GMAX);
            hwin[ch] = hgwd[ch] ? (hh[ch] + hgwd[ch] - 1) / hgwd[ch] : SG_WIN;
            hgcb[ch + 1] = hgcb[ch] + hgwd[ch] * hgwd[ch];
        }
        LZ_HIP(hipMemcpyAsync(dCS, hCS, 257 * 4, hipMemcpyHostToDevice, st));
        LZ_HIP(hipMemcpyAsync(dCS + 257, hgcb, 257 * 4, hipMemcpyHostToDevice, st));
        LZ_HIP(hipMemcpyAsync(dCS + 514, hgwd, 256 * 4, hipMemcpyHostToDevice, st));
        LZ_HIP(hipMemcpyAsync(dCS + 770, hwin, 256 * 4, hipMemcpyHostToDevice, st));
    }
    const u32 ncell = hgcb[256];
    u32* gx = e_gx.get(c);
    u32* gy = e_gy.get(c);
    u32* gw = e_gw.get(c);
    u32* cell = e_cell.get((u64)ncell + 1);
    {
        u64* key = e_key.get(c);
        u64* key2 = e_key2.get(c);
        u32* id = e_tmp1.get(c);
        u32* id2 = e_tmp2.get(c);
        k_grid_keys<<<cdiv(c, 256), 256, 0, st>>>(d_text, C, c, PAR, SAR, dCS, dCS + 257, dCS + 514, dCS + 770, key,
                                                  id);
        size_t tb = 0;
        LZ_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, key, key2, id, id2, (int)c, 0, 64, st));
        u8* t = scan_tmp.get(tb);
        LZ_HIP(hipcub::DeviceRadixSort::SortPairs(t, tb, key, key2, id, id2, (int)c, 0, 64, st));
        k_grid_points<<<cdiv((u64)c + 1, 256), 256, 0, st>>>(key2, PAR, SAR, c, gx, gy, gw, cell, ncell);
    }
    // row sparse tables over the cells' lightest weights (levels 0 .. SG_LV - 1)
    const u32* rst[SG_LV];
    {
        u32* lv0 = e_rst[0].get((u64)ncell + 1);
        if (ncell) k_cell_min<<<cdiv(ncell, 256), 256, 0, st>>>(cell, gw, ncell, lv0);
        rst[0] = lv0;
        for (u32 k = 1; k < SG_LV; k++) {
            u32* out = e_rst[k].get((u64)ncell + 1);
            if (ncell)
                k_cell_rowmin<<<cdiv(ncell, 256), 256, 0, st>>>(e_rst[k - 1].p, dCS + 514, dCS + 257, ncell, 1u << (k - 1),
                                                                 out);
            rst[k] = out;
        }
    }
    timer.mark("smpl_grid");
    smpl_view V{};
    V.L = LV;
    V.C = C;
    V.c = c;
    V.delta = delta;
    V.PA = PA;
    V.SA = SA;
    V.Pi = Pi;
    V.Psi = Psi;
    V.CS = dCS;
    V.gcb = dCS + 257;
    V.gwd = dCS + 514;
    V.gwin = dCS + 770;
    for (u32 k = 0; k < SG_LV; k++) V.rst[k] = rst[k];
    V.cell = cell;
    V.gx = gx;
    V.gy = gy;
    V.gw = gw;
    V.afst = afst;
    V.afact = afact;
    V.za = za;
    V.mode = transf_mode;
    V.small_t = SMALL_T;
    if (const char* e = std::getenv("LZ77SSS_SMPL_SMALL")) V.small_t = (u32)std::max(0L, std::atol(e));
    V.nlen[0] = V.nlen[1] = 0;
    if (transf_mode == LZ77SSS_TRANSF_WITH_SAMPLES) build_interval_samples(V, n, za64);
    // the chain (chunk walks + bridges, then the path from position 0 by pointer doubling).
    // Chunks hold about 32 approximate phrases each (the walks re-synchronise with the true
    // chain within a few phrases).
    const u64 CS = std::max<u64>(256, std::min<u64>(1ull << 26, 32 * (n / std::max<u64>(1, za64))));
    const u32 nch = (u32)((n + CS - 1) / CS);
    // task capacity: the chain (z <= z_approx) plus the walks before they merge; a full
    // table is detected and the walks rerun with four times the room
    u64 tcap64 = std::min<u64>(0x7FFFFFF0ull, 3 * (u64)za + 64 * (u64)nch + 65536);
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
        Tt.keys = e_tkeys.get(hsz);
        Tt.vals = e_tvals.get(hsz);
        Tt.mask = hsz - 1;
        Tt.cap = tcap;
        Tt.ntask = ctr + 8;
        LZ_HIP(hipMemsetAsync(Tt.keys, 0, (size_t)hsz * 4, st));
        LZ_HIP(hipMemsetAsync(ctr + 8, 0, 16, st));
        k_chunk_walks<<<cdiv(nch, SWPB), 64 * SWPB, 0, st>>>(V, Tt, CS, nch, ex, full);
        LZ_HIP(hipGetLastError());
        timer.mark("smpl_tasks");
        k_bridge_walks<<<cdiv(nch, SWPB), 64 * SWPB, 0, st>>>(V, Tt, nch, ex, full);
        LZ_HIP(hipGetLastError());
        LZ_HIP(hipMemcpyAsync(hc, ctr + 8, 8, hipMemcpyDeviceToHost, st));
        LZ_HIP(hipStreamSynchronize(st));
        if (!hc[1] && hc[0] < tcap) break;
        if (attempt >= 3 || tcap64 >= 0x7FFFFFF0ull) throw error(LZ77SSS_EINTERNAL, "exact-smpl: task table full");
        tcap64 = std::min<u64>(0x7FFFFFF0ull, 4 * tcap64);
    }
    const u32 ntask = hc[0];
    timer.mark("smpl_bridges");
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
    if (z) k_path_emit<<<cdiv(z, 256), 256, 0, st>>>(Tt, PC, (u32)z, F);
    LZ_HIP(hipGetLastError());
    LZ_HIP(hipStreamSynchronize(st));
    const u32 rounds = nch, walks = T_lv;
    timer.mark("smpl_chain");
    num_fact = z;
    stats.resize(28, 0);
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

// interval samples of with_samples (build_xa_s_1_2_intervals + build_samples,
// construction.cpp:31-305): the RKS prefix fingerprints, adjacent context LCEs of PA and SA,
// the sampled pattern lengths (quantiles of the adjacent LCEs), one hash entry per interval
void engine::build_interval_samples(smpl_view& V, u64 nn, u64 za) {
    // RKS (rabin_karp_substring.hpp:77-172)
    const u64 nb = (nn + RKS_RATE - 1) / RKS_RATE;
    u32* fps = e_rks.get(nb + 2);
    {
        u64* blk = e_key.get(nb + 1);
        u64* incl = e_key2.get(nb + 1);
        k_rks_blocks<<<cdiv(nb, 256), 256, 0, st>>>(d_text, nn, nb, blk);
        rks_cat op{};
        size_t tb = 0;
        LZ_HIP(hipcub::DeviceScan::InclusiveScan(nullptr, tb, blk, incl, op, (int)nb, st));
        u8* t = scan_tmp.get(tb);
        LZ_HIP(hipcub::DeviceScan::InclusiveScan(t, tb, blk, incl, op, (int)nb, st));
        k_rks_shift<<<cdiv(nb + 1, 256), 256, 0, st>>>(incl, nb, fps);
    }
    // the last block is partial: fps[nb] must be fp(T[0..n)); fp(T[0..16 nb)) with zero
    // padding differs, so rks_upto never reads fps[nb] past n (x / 16 <= (n - 1) / 16 < nb
    // for x < n; x = n reads fps[n / 16] only when n % 16 == 0, where it is exact)
    u32 sq = 1;
    while ((u64)sq * sq < nn + 1) sq++;
    std::vector<u32> lo(sq + 1), hi(sq + 2);
    lo[0] = 1;
    for (u32 e = 1; e <= sq; e++) lo[e] = (u32)((u64)lo[e - 1] * RKS_B % RKS_P);
    hi[0] = 1;
    for (u32 e = 1; e <= sq + 1; e++) hi[e] = (u32)((u64)hi[e - 1] * lo[sq] % RKS_P);
    u32* dpw = e_rkspw.get(2 * (u64)sq + 4);
    LZ_HIP(hipMemcpyAsync(dpw, lo.data(), (sq + 1) * 4, hipMemcpyHostToDevice, st));
    LZ_HIP(hipMemcpyAsync(dpw + sq + 1, hi.data(), (sq + 2) * 4, hipMemcpyHostToDevice, st));
    V.rks = fps;
    V.pw_lo = dpw;
    V.pw_hi = dpw + sq + 1;
    V.sq = sq;
    // adjacent LCEs and sampled lengths per side
    const u32 c = V.c;
    const u64 max_smpl_right = (u64)std::llround((double)nn / za * (1.0 + 0.5 * std::exp(-(double)nn / za / 1000.0)));
    // the adjacent LCEs are sorted on the device (a radix sort of c - 1 keys) and only the
    // sorted column goes to the host for the quantile picks (a host sort took 0.6 s per side
    // on the genome-like text's 2^24+ samples)
    std::vector<u32> srth[2];
    u32* adj[2] = {e_adjL.get((u64)c + 1), e_adjR.get((u64)c + 1)};
    u32* srtd = e_adjS.get((u64)c + 1);
    for (int side = 0; side < 2; side++) {
        k_adj_lce<<<cdiv((u64)c + 1, 256), 256, 0, st>>>(V.L, V.C, side == 0 ? V.PA : V.SA, c, V.delta, side == 0,
                                                        adj[side]);
        srth[side].resize(c > 1 ? (size_t)c - 1 : 0);
        if (c > 1) {
            size_t tb = 0;
            LZ_HIP(hipcub::DeviceRadixSort::SortKeys(nullptr, tb, adj[side] + 1, srtd, (int)(c - 1), 0, 32, st));
            u8* t = scan_tmp.get(tb);
            LZ_HIP(hipcub::DeviceRadixSort::SortKeys(t, tb, adj[side] + 1, srtd, (int)(c - 1), 0, 32, st));
            LZ_HIP(hipMemcpyAsync(srth[side].data(), srtd, ((size_t)c - 1) * 4, hipMemcpyDeviceToHost, st));
            LZ_HIP(hipStreamSynchronize(st));  // srtd is reused by the other side
        }
    }
    u64 total_iv = 0;
    for (int side = 0; side < 2; side++) {
        // construction.cpp:136-199: quantiles of the sorted adjacent LCEs in [3, max]
        const std::vector<u32>& srt = srth[side];
        const u64 maxlen = side == 0 ? V.delta : std::min<u64>(srt.empty() ? 0 : srt.back(), max_smpl_right);
        V.slen[side][0] = 1;
        V.slen[side][1] = 2;
        u32 k = 2;
        if (!srt.empty() && maxlen > 3) {
            const u64 rmin = std::lower_bound(srt.begin(), srt.end(), 3u) - srt.begin();
            const u64 rmax = std::lower_bound(srt.begin(), srt.end(), (u32)maxlen) - srt.begin();
            if (rmin < rmax) {
                const u64 want = std::min<u64>(NSMPL, std::min<u64>(maxlen - 2, 2 + (u64)std::floor(4.0 * c / (double)(rmin + rmax))));
                for (u64 q = 2; q < want && k < NSMPL; q++) {
                    const double rel = (q - 1) / (double)(want - 2);
                    const u64 rk = (u64)std::floor(rmin + rel * (double)(rmax - rmin));
                    const u32 len = std::max<u32>(srt[std::min<u64>(rk, srt.size() - 1)], V.slen[side][k - 1] + 1);
                    if (len > maxlen) break;
                    V.slen[side][k++] = len;
                }
            }
        }
        V.nlen[side] = k;
        for (u32 q = 2; q < k; q++) {
            const u32 len = V.slen[side][q];
            total_iv += 1 + (u64)(std::upper_bound(srt.begin(), srt.end(), len - 1) - srt.begin());
        }
    }
    u64 hs = 1024;
    while (hs < 2 * total_iv + 1024) hs <<= 1;
    u64* hkey = e_hkey.get(hs);
    u64* hval = e_hval.get(hs);
    LZ_HIP(hipMemsetAsync(hkey, 0, hs * 8, st));
    V.hkey = hkey;
    V.hval = hval;
    V.hmask = hs - 1;
    for (int side = 0; side < 2; side++) {
        // sparse-table minima of adj[0 .. c) (level 0 is adj itself) for the interval ends
        iv_levels M{};
        M.mn[0] = adj[side];
        M.nlv = 1;
        while ((2ull << (M.nlv - 1)) <= c && M.nlv < (u32)MAX_LV) {
            const u64 half = 1ull << (M.nlv - 1), cnt = (u64)c - 2 * half + 1;
            u32* out = e_ivmin[M.nlv].get(cnt);
            k_iv_min_level<<<cdiv(cnt, 256), 256, 0, st>>>(M.mn[M.nlv - 1], cnt, half, out);
            M.mn[M.nlv++] = out;
        }
        for (u32 q = 2; q < V.nlen[side]; q++)
            k_iv_insert<<<cdiv(c, 256), 256, 0, st>>>(V, side == 0 ? V.PA : V.SA, adj[side], c, side == 0, q,
                                                     V.slen[side][q], hkey, hval, hs - 1, M);
    }
    LZ_HIP(hipGetLastError());
    timer.mark("smpl_ivs");
}

}  // namespace LZ_NS
