// sa_s.hip -- suffix order of the sync positions and the LCE structure
// (roles of lce_classic_for_sss: gsaca_for_lce + ISA + Kasai LCP + rmq_n,
// patched-files/external/lce/include/ds/lce_classic_for_sss.hpp:36-142, and
// of pred_index / reduce_fps_3tau_lexicographic, lce_sss.hpp:68-83; those
// sources are absent upstream).
//
// SA_S is the TRUE suffix order of the sync positions:
//   key_k = T[S[k] .. S[k] + max(3tau, S[k+1]-S[k]+2tau))  (last key: to n)
//   R_0   = lexicographic rank of key_k            (comparison merge sort)
//   R_h+1 = rank of (R_h[k], R_h[k+2^h])            (radix sort, prefix doubling)
// until all ranks are distinct.  LCP between SA-neighbours comes from binary
// lifting over the stored R_h levels plus one bounded key comparison.
#include "../include/engine.h"
#include "../include/prim.h"
#include "../include/lce_dev.h"
#include "../include/msort_dev.h"

#include <hipcub/hipcub.hpp>

namespace LZ_NS {

__global__ void k_key_len(const pos_t* __restrict__ S, u32 s, u64 n, pos_t* __restrict__ KL) {
    const u64 k = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= s) return;
    const u64 beg = S[k];
    u64 len = (k + 1 < s) ? max<u64>(3 * TAU, (u64)S[k + 1] - S[k] + 2 * TAU) : n - beg;
    KL[k] = (pos_t)min<u64>(len, n - beg);
}

__device__ __forceinline__ int dev_key_cmp(const u8* T, const pos_t* S, const pos_t* KL, u32 a, u32 b) {
    const u64 la = KL[a], lb = KL[b], m = min(la, lb);
    const u64 c = dev_naive_lce(T, S[a], S[b], m);
    if (c < m) return T[(u64)S[a] + c] < T[(u64)S[b] + c] ? -1 : 1;
    return la < lb ? -1 : (la > lb ? 1 : 0);
}

struct key_less {
    const u8* T;
    const pos_t* S;
    const pos_t* KL;
    __device__ bool operator()(const u32& a, const u32& b) const { return dev_key_cmp(T, S, KL, a, b) < 0; }
};

__global__ void k_iota(u32* __restrict__ x, u32 m) {
    const u64 k = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (k < m) x[k] = (u32)k;
}
__global__ void k_key_diff(const u8* T, const pos_t* S, const pos_t* KL, const u32* __restrict__ idx, u32 s,
                           u32* __restrict__ flag) {
    const u64 t = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= s) return;
    flag[t] = (t == 0) ? 1u : (dev_key_cmp(T, S, KL, idx[t - 1], idx[t]) != 0 ? 1u : 0u);
}
__global__ void k_scatter_rank(const u32* __restrict__ idx, const u32* __restrict__ rank, u32 s, u32* __restrict__ R) {
    const u64 t = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (t < s) R[idx[t]] = rank[t];
}
// the q ranks R[k], R[k+h], .., R[k+(q-1)h] (0 past the end) as one radix key: the
// next level ranks rank-string prefixes q times as long (q = 64 / bits, at most 4)
__global__ void k_pack_pairs(const u32* __restrict__ R, u32 s, u64 h, u32 bits, u32 q, u64* __restrict__ kv,
                             u32* __restrict__ idx) {
    const u64 k = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= s) return;
    u64 key = R[k];
    for (u32 j = 1; j < q; j++) key = (key << bits) | ((k + j * h < s) ? R[k + j * h] : 0u);
    kv[k] = key;
    idx[k] = (u32)k;
}
__global__ void k_pair_diff(const u64* __restrict__ kv, u32 s, u32* __restrict__ flag) {
    const u64 t = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= s) return;
    flag[t] = (t == 0 || kv[t] != kv[t - 1]) ? 1u : 0u;
}
__global__ void k_sa_from_rank(const u32* __restrict__ R, u32 s, u32* __restrict__ SA, u32* __restrict__ ISA) {
    const u64 k = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= s) return;
    const u32 r = R[k] - 1;
    SA[r] = (u32)k;
    ISA[k] = r;
}

struct rank_levels {
    u32 nlev, step;  // level lv ranks prefixes of step^lv key ranks
    const u32* R[MAX_LV];
};

// LCP[r] = LCE(S[SA[r-1]], S[SA[r]]), r >= 1; LCP[0] = 0
__global__ void k_lcp(const u8* __restrict__ T, u64 n, const pos_t* __restrict__ S, const pos_t* __restrict__ KL,
                      const u32* __restrict__ SA, u32 s, rank_levels RL, run_tab R, u32* __restrict__ LCP) {
    const u64 r = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= s) return;
    if (r == 0) { LCP[0] = 0; return; }
    const u32 a = SA[r - 1], b = SA[r];
    u64 c = 0;
    u64 w = 1;  // span of the top level
    for (u32 lv = 1; lv < RL.nlev; lv++) w *= RL.step;
    // the top level ranks are all distinct; below level lv + 1 the common prefix left is
    // shorter than step * w: at most step - 1 steps of w per level
    for (int lv = (int)RL.nlev - 1; lv >= 0; lv--, w /= RL.step) {
        for (u32 t = 1; t < RL.step; t++) {
            if (a + c < s && b + c < s && RL.R[lv][a + c] == RL.R[lv][b + c]) c += w;
            else break;
        }
    }
    u64 v;
    if (a + c >= s) v = n - S[a];
    else if (b + c >= s) v = n - S[b];
    else {
        const u32 ka = (u32)(a + c), kb = (u32)(b + c);
        const u64 m = min(KL[ka], KL[kb]);
        v = ((u64)S[ka] - S[a]) + dev_lce_fwd(T, R, S[ka], S[kb], m);
    }
    LCP[r] = (u32)min<u64>(v, LCP_SAT);
}

__global__ void k_min_level(const u32* __restrict__ prev, u32 cnt, u32 half, u32* __restrict__ out) {
    const u64 k = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (k < cnt) out[k] = min(prev[k], prev[k + half]);
}
// two sparse-table levels per launch (lv from lv - 1 and lv + 1 from lv - 1: half the launches)
__global__ void k_min_level2(const u32* __restrict__ prev, u32 cnt1, u32 half, u32* __restrict__ out1, u32 cnt2,
                             u32* __restrict__ out2) {
    const u64 k = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= cnt1) return;
    const u32 a = min(prev[k], prev[k + half]);
    out1[k] = a;
    if (k < cnt2) out2[k] = min(a, min(prev[k + 2 * half], prev[k + 3 * half]));
}

__global__ void k_succ_table(const pos_t* __restrict__ S, u32 s, u64 nb, u32* __restrict__ tab) {
    const u64 bkt = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (bkt >= nb) return;
    const u64 x = bkt << 9;
    u32 lo = 0, hi = s;
    while (lo < hi) {
        u32 mid = (lo + hi) >> 1;
        if ((u64)S[mid] < x) lo = mid + 1; else hi = mid;
    }
    tab[bkt] = lo;
}

// ---------------------------------------------------------------------------
// key deduplication (exact: hash groups are verified by full comparison)
__device__ __forceinline__ u64 mix64(u64 z) {
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}
// h(key) = mix(len) + sum over its 8-byte words w of mix(word_w) * R^w (mod 2^64, R odd).
// The sum splits over pieces, so a key is cut into KH_CHUNK-byte pieces hashed by
// different waves and added atomically: long keys (gaps of MBs inside periodic runs)
// do not serialize on one wave.  A piece inside a p-periodic run (run table, lce_dev.h)
// has a word sequence of period L = p / gcd(p, 8): its sum is the first L terms times
// geometric series in R^L, so run-heavy text is hashed without reading the runs.
// k_key_prep sets H = mix(len) and the piece counts.
constexpr u32 KH_CHUNK = 16384;
constexpr u32 KH_WAVES = 16384;
constexpr u64 KH_R = 0x9e3779b97f4a7c15ull;  // odd
constexpr u64 kh_pow_host(u64 e) {
    u64 r = 1, b = KH_R;
    while (e) { if (e & 1) r *= b; b *= b; e >>= 1; }
    return r;
}
constexpr u64 KH_R64 = kh_pow_host(64);
__device__ __forceinline__ u64 kh_pow(u64 e) {  // R^e mod 2^64
    u64 r = 1, b = KH_R;
    while (e) {
        if (e & 1) r *= b;
        b *= b;
        e >>= 1;
    }
    return r;
}
// (one launch: the key lengths (k_key_len's rule), H = mix(len), the piece counts, idx = iota)
__global__ void k_key_prep(const pos_t* __restrict__ S, u32 s, u64 n, pos_t* __restrict__ KL, u64* __restrict__ H,
                           u32* __restrict__ CC, u32* __restrict__ idx) {
    const u64 k = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= s) return;
    const u64 beg = S[k];
    const u64 len = min<u64>((k + 1 < s) ? max<u64>(3 * TAU, (u64)S[k + 1] - beg + 2 * TAU) : n - beg, n - beg);
    KL[k] = (pos_t)len;
    H[k] = mix64(len ^ 0xd6e8feb86659fd93ull);
    CC[k] = (u32)max<u64>(1, (len + KH_CHUNK - 1) / KH_CHUNK);
    idx[k] = (u32)k;
}
// OFF = inclusive scan of the piece counts; wave w hashes pieces [w*per, (w+1)*per)
__global__ __launch_bounds__(256) void k_key_hash(const u8* __restrict__ T, const pos_t* __restrict__ S,
                                                  const pos_t* __restrict__ KL, const u32* __restrict__ OFF, u32 s,
                                                  run_tab R, u64* __restrict__ H) {
    const u32 wave = (u32)(((u64)blockIdx.x * blockDim.x + threadIdx.x) >> 6);
    const u32 lane = threadIdx.x & 63;
    const u32 total = OFF[s - 1];
    const u32 per = (total + KH_WAVES - 1) / KH_WAVES;
    u32 c = wave * per;
    const u32 cend = min(total, c + per);
    if (c >= cend) return;
    // key holding piece c: first k with OFF[k] > c
    u32 lo = 0, hi = s - 1;
    while (lo < hi) {
        const u32 mid = (lo + hi) >> 1;
        if (OFF[mid] > c) hi = mid; else lo = mid + 1;
    }
    u32 k = lo;
    for (; c < cend; c++) {
        while (OFF[k] <= c) k++;
        const u32 first = k ? OFF[k - 1] : 0;
        const u64 beg = S[k], len = KL[k];
        const u64 b0 = (u64)(c - first) * KH_CHUNK, b1 = min<u64>(len, b0 + KH_CHUNK);
        u64 h = 0;
        u32 pp = 0;  // period of a run holding the whole piece (and the word after it), else 0
        if (b1 == b0 + KH_CHUNK && b1 + 8 <= len) {
            const u64 x0 = beg + b0;
            // a piece inside a p-periodic stretch of the block run records
            if (R.re) {
                const u64 bb = (x0 + 511) >> 9;
                const u64 v = R.re[bb], u = R.rs[bb];
                if ((v & 255) && (u >> 16) <= x0 && (v >> 16) >= x0 + KH_CHUNK + 8) pp = (u32)(v & 255);
            }
            if (!pp && R.p) {
                const u64 t = (x0 + 127) >> 7;
                const u32 p = R.p[t];
                if (p && (u64)R.lo[t] <= x0 && (u64)R.hi[t] >= x0 + KH_CHUNK + 8) pp = p;
            }
        }
        if (pp) {
            const u32 L = pp / min(pp & (0u - pp), 8u), NW = KH_CHUNK / 8;
            const u64 RL = kh_pow(L), Rw0 = kh_pow(b0 / 8);
            const u32 K = NW / L, rem = NW % L;  // words j < rem recur K + 1 times, the others K
            u64 g0 = 0, q = 1;  // g0 = sum_{i<K} RL^i, q = RL^K
            {
                u64 base = RL, e = K, acc = 0, pw = 1;  // geometric sum by binary doubling
                u64 sb = 1;                            // sum_{i<2^b} base^i for the current bit block
                while (e) {
                    if (e & 1) { acc += sb * pw; pw *= base; }
                    sb += sb * base;
                    base *= base;
                    e >>= 1;
                }
                g0 = acc;
                q = pw;
            }
            const u64 g1 = g0 + q;
            for (u32 j = lane; j < L; j += 64) {
                const u64 x = ldu64(T + beg + b0 + 8ull * j);
                h += mix64(x) * Rw0 * kh_pow(j) * (j < rem ? g1 : g0);
            }
        } else {
            u64 pw = kh_pow(b0 / 8 + lane);
            for (u64 w = b0 / 8 + lane; 8 * w < b1; w += 64) {
                u64 x = ldu64(T + beg + 8 * w);
                const u64 rem = len - 8 * w;
                if (rem < 8) x &= (1ull << (8 * rem)) - 1;
                h += mix64(x) * pw;
                pw *= KH_R64;
            }
        }
        for (int o = 32; o >= 1; o >>= 1) h += __shfl_xor(h, o);
        if (lane == 0 && b0 < b1) atomicAdd((unsigned long long*)&H[k], (unsigned long long)h);
    }
}
// big-endian 8-byte word i of a key (zero past its end): radix keys of the presort
__device__ __forceinline__ u64 key_word_be(const u8* T, u64 beg, u64 len, u32 i) {
    const u64 off = 8ull * i;
    if (off >= len) return 0;
    u64 x = ldu64(T + beg + off);
    const u64 r = len - off;
    if (r < 8) x &= (1ull << (8 * r)) - 1;
    return __builtin_bswap64(x);
}
__global__ void k_word_keys(const u8* __restrict__ T, const pos_t* __restrict__ S, const pos_t* __restrict__ KL,
                            const u32* __restrict__ v, u32 d, u32 i, u64* __restrict__ key) {
    const u64 t = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (t < d) key[t] = key_word_be(T, S[v[t]], KL[v[t]], i);
}
// wave-parallel exact comparison of two keys (all 64 lanes must call it)
__device__ int wave_key_cmp(const u8* T, const run_tab& R, const pos_t* S, const pos_t* KL, u32 a, u32 b, u32 lane) {
    const u64 la = KL[a], lb = KL[b], m = min(la, lb);
    const u64 pa = S[a], pb = S[b];
    const u64 c = wave_lce_fwd(T, R, pa, pb, m, lane);
    if (c < m) return T[pa + c] < T[pb + c] ? -1 : 1;
    return la < lb ? -1 : (la > lb ? 1 : 0);
}
// flags: new group where the hash changes; exact check of equal-hash neighbours
__global__ __launch_bounds__(256) void k_group_verify(const u8* T, run_tab R, const pos_t* S, const pos_t* KL,
                                                      const u64* __restrict__ Hs, const u32* __restrict__ idx,
                                                      u32 s, u32* __restrict__ flag, u32* __restrict__ collide) {
    const u32 lane = threadIdx.x & 63;
    for (u64 t = gtid() >> 6; t < s; t += gstride() >> 6) {  // one wave per key (grid-stride: s * 64 threads)
        if (t == 0 || Hs[t] != Hs[t - 1]) {
            if (lane == 0) flag[t] = 1;
            continue;
        }
        const int c = wave_key_cmp(T, R, S, KL, idx[t - 1], idx[t], lane);
        if (lane == 0) {
            flag[t] = 0;
            if (c != 0) atomicOr(collide, 1u);
        }
    }
}
__global__ void k_reps(const u32* __restrict__ flag, const u32* __restrict__ grp, const u32* __restrict__ idx, u32 s,
                       u32* __restrict__ rep) {
    const u64 t = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (t < s && flag[t]) rep[grp[t] - 1] = idx[t];
}
// distinct keys are radix-sorted by their first PRESORT_WORDS big-endian words
// (LSD: one stable 64-bit radix pass per word); keys equal on that prefix form
// tie segments finished by exact wave comparisons below
constexpr u32 PRESORT_WORDS = 4;
__global__ void k_prefix_ties(const u8* __restrict__ T, const pos_t* __restrict__ S, const pos_t* __restrict__ KL,
                              const u32* __restrict__ srt, u32 d, u8* __restrict__ tie) {
    const u64 r = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= d) return;
    if (r == 0) { tie[0] = 0; return; }
    const u32 a = srt[r - 1], b = srt[r];
    bool eq = true;
    for (u32 i = 0; i < PRESORT_WORDS && eq; i++)
        eq = key_word_be(T, S[a], KL[a], i) == key_word_be(T, S[b], KL[b], i);
    tie[r] = eq ? 1 : 0;
}
// Tie segments (keys equal on the presort prefix) are finished by a merge sort in
// which every comparison is done by a whole wave (64 lanes x 8 bytes per step).
// Items hold key ids, segment k occupies [sbeg[k], sbeg[k+1]).
// A pass of width w merges, inside every segment, neighbouring sorted blocks of
// w items (local offsets).  Each wave produces opw = min(16, 2w) outputs of one
// merge; uoff is the exclusive scan of the per-segment wave counts, so passes
// cost O(members) and only log2(longest segment) passes run.
__global__ void k_seg_units(const u32* __restrict__ sbeg, u32 nseg, u32 opw, u32* __restrict__ units) {
    const u64 k = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (k < nseg) units[k] = (sbeg[k + 1] - sbeg[k] + opw - 1) / opw;
    if (k == nseg) units[k] = 0;  // exclusive scan over nseg + 1 -> uoff[nseg] = total
}
__global__ __launch_bounds__(256) void k_segmerge(const u8* T, run_tab R, const pos_t* S, const pos_t* KL,
                                                  const u32* __restrict__ sbeg, const u32* __restrict__ uoff, u32 nseg,
                                                  u32 nunits, const u32* __restrict__ in, u32* __restrict__ out, u32 w,
                                                  u32 opw) {
    const u32 lane = threadIdx.x & 63;
    const u32 nu = min(nunits, uoff[nseg]);  // nunits: launch bound, uoff[nseg]: exact count
    for (u64 uu = gtid() >> 6; uu < nu; uu += gstride() >> 6) {  // one wave per output run (grid-stride)
    const u32 unit = (u32)uu;
    u32 lo = 0, hi = nseg;  // last k with uoff[k] <= unit
    while (hi - lo > 1) {
        const u32 mid = (lo + hi) >> 1;
        if (uoff[mid] <= unit) lo = mid; else hi = mid;
    }
    const u32 k = lo, o = sbeg[k], L = sbeg[k + 1] - o;
    const u64 p0 = (u64)(unit - uoff[k]) * opw;
    const u64 base = p0 / (2ull * w) * (2ull * w);
    const u64 a0 = o + base, a1 = o + min<u64>(base + w, L), b0 = a1, b1 = o + min<u64>(base + 2ull * w, L);
    const u64 la = a1 - a0, lb = b1 - b0, diag = p0 - base;
    u64 l2 = diag > lb ? diag - lb : 0, h2 = min(diag, la);
    while (l2 < h2) {
        const u64 mid = (l2 + h2) >> 1;
        if (!(wave_key_cmp(T, R, S, KL, in[b0 + diag - 1 - mid], in[a0 + mid], lane) < 0)) l2 = mid + 1; else h2 = mid;
    }
    u64 i = l2, j = diag - l2;
    const u64 pend = min<u64>(o + p0 + opw, b1);
    for (u64 p = o + p0; p < pend; p++) {
        bool takeA;
        if (i >= la) takeA = false;
        else if (j >= lb) takeA = true;
        else takeA = !(wave_key_cmp(T, R, S, KL, in[b0 + j], in[a0 + i], lane) < 0);
        const u32 v = takeA ? in[a0 + i++] : in[b0 + j++];
        if (lane == 0) out[p] = v;
    }
    }
}
// ranks in a tie segment (tie with the previous or the next rank) and segment starts
__global__ void k_tie_member(const u8* __restrict__ tie, u32 d, u8* __restrict__ member, u8* __restrict__ start) {
    const u64 r = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= d) return;
    const bool nx = r + 1 < d && tie[r + 1];
    member[r] = (tie[r] || nx) ? 1 : 0;
    start[r] = (!tie[r] && nx) ? 1 : 0;
}
__global__ void k_gather_u8(const u8* __restrict__ src, const u32* __restrict__ pos, u32 m, u8* __restrict__ dst) {
    const u64 t = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (t < m) dst[t] = src[pos[t]];
}
// sbeg[nseg] = mt; len[k] = sbeg[k+1] - sbeg[k]
__global__ void k_seg_lens(u32* __restrict__ sbeg, u32 nseg, u32 mt, u32* __restrict__ len) {
    const u64 k = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (k == 0) sbeg[nseg] = mt;
    if (k < nseg) len[k] = (k + 1 < nseg ? sbeg[k + 1] : mt) - sbeg[k];
}
__global__ void k_gather_u32(const u32* __restrict__ src, const u32* __restrict__ pos, u32 m, u32* __restrict__ dst) {
    const u64 t = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (t < m) dst[t] = src[pos[t]];
}
__global__ void k_scatter_u32(const u32* __restrict__ src, const u32* __restrict__ pos, u32 m, u32* __restrict__ dst) {
    const u64 t = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (t < m) dst[pos[t]] = src[t];
}
__global__ void k_rank_of_group(const u32* __restrict__ srt_grp, u32 d, u32* __restrict__ rank_of) {
    const u64 r = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (r < d) rank_of[srt_grp[r]] = (u32)r + 1;
}
__global__ void k_r0_from_groups(const u32* __restrict__ idx, const u32* __restrict__ grp, const u32* __restrict__ rank_of,
                                 u32 s, u32* __restrict__ R0) {
    const u64 t = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (t < s) R0[idx[t]] = rank_of[grp[t] - 1];
}
__global__ void k_map_rep_to_group(const u32* __restrict__ srt_key, u32 d, const u32* __restrict__ key_to_grp,
                                   u32* __restrict__ srt_grp) {
    const u64 r = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (r < d) srt_grp[r] = key_to_grp[srt_key[r]];
}
__global__ void k_key_to_grp(const u32* __restrict__ flag, const u32* __restrict__ grp, const u32* __restrict__ idx,
                             u32 s, u32* __restrict__ key_to_grp) {
    const u64 t = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (t < s && flag[t]) key_to_grp[idx[t]] = grp[t] - 1;
}

// (stable comparison merge sort of u32 items: include/msort_dev.h)
// debug builds of the phase: synchronize and name the step that faulted
#define SA_DBG(what)                                                                  \
    do {                                                                              \
        if (debug_enabled()) {                                                        \
            hipError_t se_ = hipStreamSynchronize(st);                                \
            const double t_ = now_ms();                                               \
            fprintf(stderr, "[sa_s] %-16s %s %8.3f ms\n", what, se_ == hipSuccess ? "ok" : hipGetErrorString(se_), \
                    t_ - sa_dbg_t);                                                   \
            sa_dbg_t = t_;                                                            \
            LZ_HIP(se_);                                                              \
        }                                                                             \
    } while (0)
static void scan_incl(u32* in, u32* out, u32 m, dbuf<u8>& tmp, hipStream_t st) {
    incl_sum(in, out, m, tmp, st);  // (include/prim.h: one launch up to 64 Ki items)
}

void engine::build_sa_s(const u8* T) {
    double sa_dbg_t = now_ms();
    (void)sa_dbg_t;
    nlev_rank = 0;
    if (s == 0) return;
    const pos_t* dS = S.p;
    pos_t* KL = key_len.get(s);
    const unsigned g = cdiv(s, 256);
    // ---- R_0: lexicographic rank of the keys (equal keys share a rank)
    u32* idx_in = u32a.get(s);
    u32* idx = u32b.get(s);
    u32* flag = u32c.get(s);
    u32* rank = u32d.get(s);
    u32* R0 = rank_lv[0].get(s);
    bool done_r0 = false;
    {
        // 1. group identical keys by a wave-parallel hash, verified exactly
        u64* H = u64a.get(s);
        u64* Hs = u64b.get(s);
        u32* CC = u32e.get(s);
        k_key_prep<<<g, 256, 0, st>>>(dS, s, n, KL, H, CC, idx_in);
        scan_incl(CC, CC, s, scan_tmp, st);
        k_key_hash<<<KH_WAVES * 64 / 256, 256, 0, st>>>(T, dS, KL, CC, s, runs(), H);
        SA_DBG("key hash");
        size_t tb = 0;
        LZ_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, H, Hs, idx_in, idx, (int)s, 0, 64, st));
        u8* t = scan_tmp.get(tb);
        LZ_HIP(hipcub::DeviceRadixSort::SortPairs(t, tb, H, Hs, idx_in, idx, (int)s, 0, 64, st));
        u32* ctr = counters.get(16);
        LZ_HIP(hipMemsetAsync(ctr + 2, 0, 4, st));
        SA_DBG("hash sort");
        k_group_verify<<<capped_grid((u64)s * 64, 256), 256, 0, st>>>(T, runs(), dS, KL, Hs, idx, s, flag, ctr + 2);
        scan_incl(flag, rank, s, scan_tmp, st);  // rank[t] = group id + 1
        const auto [collide, d] = rd2(ctr + 2, rank + s - 1, st);
        if (debug_enabled()) fprintf(stderr, "[sa_s] s=%u collide=%u\n", s, collide);
        if (!collide) {
            u32* rep = sa_tmp1.get(d);
            k_reps<<<g, 256, 0, st>>>(flag, rank, idx, s, rep);
            // 2. sort distinct keys: bounded comparison, then exact wave sort of bounded ties
            u32* srt = rep;
            SA_DBG("reps");
            {
                u32* v2 = sa_tmp2.get(d);
                u64* wk = u64b.get(2 * (u64)d);  // sorted hashes no longer needed
                u64* wk2 = wk + d;
                // double buffers: the sort alternates between the two halves, no copy per word
                hipcub::DoubleBuffer<u64> kb(wk, wk2);
                hipcub::DoubleBuffer<u32> vb(srt, v2);
                size_t tb2 = 0;
                LZ_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, tb2, kb, vb, (int)d, 0, 64, st));
                u8* t2 = scan_tmp.get(tb2);
                for (int i = (int)PRESORT_WORDS - 1; i >= 0; i--) {
                    k_word_keys<<<cdiv(d, 256), 256, 0, st>>>(T, dS, KL, vb.Current(), d, (u32)i, kb.Current());
                    LZ_HIP(hipcub::DeviceRadixSort::SortPairs(t2, tb2, kb, vb, (int)d, 0, 64, st));
                }
                if (vb.Current() != srt)
                    LZ_HIP(hipMemcpyAsync(srt, vb.Current(), (size_t)d * 4, hipMemcpyDeviceToDevice, st));
            }
            SA_DBG("presort");
            u8* tie = tmp_bytes.get(d);
            k_prefix_ties<<<cdiv(d, 256), 256, 0, st>>>(T, dS, KL, srt, d, tie);
            if (debug_enabled()) fprintf(stderr, "[sa_s] distinct=%u sorted\n", d);
            // members of tie segments (ranks r whose key ties with r-1 or r+1, in order) and the
            // segment offsets, on the device: flags, two flagged selections, a max-reduction
            u8* mflag = tmp_bytes2.get(2 * (u64)d + 2);
            u8* sflag = mflag + d + 1;
            k_tie_member<<<cdiv(d, 256), 256, 0, st>>>(tie, d, mflag, sflag);
            u32* dpos = sa_tmp3.get(d);
            u32* cnt4 = counters.get(16) + 8;
            {
                size_t tb = 0;
                hipcub::CountingInputIterator<u32> it0(0);
                LZ_HIP(hipcub::DeviceSelect::Flagged(nullptr, tb, it0, mflag, dpos, cnt4, (int)d, st));
                u8* tq = scan_tmp.get(tb);
                LZ_HIP(hipcub::DeviceSelect::Flagged(tq, tb, it0, mflag, dpos, cnt4, (int)d, st));
            }
            const u32 mt = rd1(cnt4, st);
            u32 nseg = 0, maxl = 0;
            u32* dsb = u32e.get(2 * (u64)mt + 4);
            if (mt) {
                u8* sf2 = tmp_bytes3.get(mt);
                k_gather_u8<<<cdiv(mt, 256), 256, 0, st>>>(sflag, dpos, mt, sf2);
                size_t tb = 0;
                hipcub::CountingInputIterator<u32> it0(0);
                LZ_HIP(hipcub::DeviceSelect::Flagged(nullptr, tb, it0, sf2, dsb, cnt4 + 1, (int)mt, st));
                u8* tq = scan_tmp.get(tb);
                LZ_HIP(hipcub::DeviceSelect::Flagged(tq, tb, it0, sf2, dsb, cnt4 + 1, (int)mt, st));
                nseg = rd1(cnt4 + 1, st);
                u32* seglen = dsb + nseg + 1;
                k_seg_lens<<<cdiv(nseg + 1, 256), 256, 0, st>>>(dsb, nseg, mt, seglen);
                size_t tb2 = 0;
                LZ_HIP(hipcub::DeviceReduce::Max(nullptr, tb2, seglen, cnt4 + 2, (int)nseg, st));
                u8* tq2 = scan_tmp.get(tb2);
                LZ_HIP(hipcub::DeviceReduce::Max(tq2, tb2, seglen, cnt4 + 2, (int)nseg, st));
                maxl = rd1(cnt4 + 2, st);
            }
            if (debug_enabled()) fprintf(stderr, "[sa_s] tie segments=%u members=%u longest=%u\n", nseg, mt, maxl);
            if (mt) {
                u32* it_a = (u32*)u64a.get(mt);  // hashes no longer needed
                u32* it_b = it_a + mt;
                u32* units = dsb + nseg + 1;
                k_gather_u32<<<cdiv(mt, 256), 256, 0, st>>>(srt, dpos, mt, it_a);
                u32* uoff = sa_tmp1.p == srt ? sa_tmp2.get(nseg + 1) : sa_tmp1.get(nseg + 1);
                // output runs per wave: up to 16, fewer while that leaves under 16 Ki waves -- a
                // latency chain of wave comparisons per run (rr, 54 K keys: sa_s 1.57 -> 1.34 ms at
                // 4; genome, millions of tie members: 16, 4 costs +0.4 ms; LZ77SSS_SEGMERGE_OPW forces)
                u64 opw_cap = 16;
                while (opw_cap > 4 && mt / opw_cap < 16384) opw_cap /= 2;
                if (const char* e = std::getenv("LZ77SSS_SEGMERGE_OPW")) opw_cap = std::max<u64>(1, std::strtoull(e, nullptr, 10));
                u32 opw_prev = 0;
                for (u64 w = 1; w < maxl; w *= 2) {
                    const u32 opw = (u32)std::min<u64>(opw_cap, 2 * w);  // short output runs: more waves on long segments
                    // no host read-back: launch for the upper bound cdiv(members, opw) + segments; the
                    // unit offsets depend on opw only (it saturates at opw_cap after a few passes)
                    if (opw != opw_prev) {
                        k_seg_units<<<cdiv(nseg + 1, 256), 256, 0, st>>>(dsb, nseg, opw, units);
                        scan_dev(units, uoff, (u64)nseg + 1, (u64)nseg + 1, 0u, 0u, op_sum{}, true, scan_tmp, st);
                        opw_prev = opw;
                    }
                    const u32 nunits = cdiv(mt, opw) + nseg;
                    k_segmerge<<<capped_grid((u64)nunits * 64, 256), 256, 0, st>>>(T, runs(), dS, KL, dsb, uoff, nseg, nunits,
                                                                            it_a, it_b, (u32)w, opw);
                    std::swap(it_a, it_b);
                    SA_DBG("segmerge");
                }
                k_scatter_u32<<<cdiv(mt, 256), 256, 0, st>>>(it_a, dpos, mt, srt);
                SA_DBG("tie scatter");
                LZ_HIP(hipGetLastError());
            }
            stats_sa_ties = nseg;
            // 3. ranks: sorted distinct keys -> groups -> every key
            u32* key_to_grp = idx_in;  // free now
            k_key_to_grp<<<g, 256, 0, st>>>(flag, rank, idx, s, key_to_grp);
            u32* srt_grp = sa_tmp2.p;  // merge scratch, free now
            k_map_rep_to_group<<<cdiv(d, 256), 256, 0, st>>>(srt, d, key_to_grp, srt_grp);
            u32* rank_of = srt;  // sorted reps consumed by k_map_rep_to_group (stream order)
            k_rank_of_group<<<cdiv(d, 256), 256, 0, st>>>(srt_grp, d, rank_of);
            k_r0_from_groups<<<g, 256, 0, st>>>(idx, rank, rank_of, s, R0);
            SA_DBG("r0");
            stats_sa_distinct = d;
            done_r0 = true;
        }
    }
    if (!done_r0) {
        // hash collision between different keys: exact comparison sort of all keys
        k_iota<<<g, 256, 0, st>>>(idx, s);
        merge_sort_u32(idx, idx_in, s, key_less{T, dS, KL}, st);
        k_key_diff<<<g, 256, 0, st>>>(T, dS, KL, idx, s, flag);
        scan_incl(flag, rank, s, scan_tmp, st);
        k_scatter_rank<<<g, 256, 0, st>>>(idx, rank, s, R0);
    }
    nlev_rank = 1;
    u32 maxr = done_r0 ? (u32)stats_sa_distinct : rd1(rank + s - 1, st);
    // ---- prefix doubling over the sequence of key ranks
    u32 bits = 1;
    while (bits < 32 && (1ull << bits) <= s) bits++;
    // ranks per radix key: a small sync set (repetitive text) packs 3-4 ranks into the
    // 64-bit key and needs half the rounds, each a chain of small sort launches
    const u32 q = std::min<u32>(4, 64 / bits);
    rank_step = q;
    u64* kv = u64a.get(s);
    u64* kv2 = u64b.get(s);
    // every round's max rank goes to pinned memory behind its launches, and is read
    // only after the NEXT round is enqueued: the device never idles on the host's
    // convergence test.  The round after convergence is redundant but harmless (all
    // ranks distinct: the same head ranks again, one more level for the LCP lifting).
    int pending = -1;  // slot of the last round whose max rank is in flight
    while (maxr < s) {
        if (nlev_rank >= MAX_LV) throw error(-6, "prefix doubling did not converge");
        u64 h = 1;
        for (u32 l = 1; l < nlev_rank; l++) h *= q;
        const u32* R = rank_lv[nlev_rank - 1].p;
        k_pack_pairs<<<g, 256, 0, st>>>(R, s, h, bits, q, kv, idx_in);
        size_t tb = 0;
        LZ_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, kv, kv2, idx_in, idx, (int)s, 0, (int)(q * bits), st));
        u8* t = scan_tmp.get(tb);
        LZ_HIP(hipcub::DeviceRadixSort::SortPairs(t, tb, kv, kv2, idx_in, idx, (int)s, 0, (int)(q * bits), st));
        k_pair_diff<<<g, 256, 0, st>>>(kv2, s, flag);
        scan_incl(flag, rank, s, scan_tmp, st);
        u32* Rn = rank_lv[nlev_rank].get(s);
        k_scatter_rank<<<g, 256, 0, st>>>(idx, rank, s, Rn);
        SA_DBG("doubling");
        const int slot = (int)(nlev_rank & 1);
        LZ_HIP(hipMemcpyAsync(h_pin + slot, rank + s - 1, 4, hipMemcpyDeviceToHost, st));
        LZ_HIP(hipEventRecord(ev_pin[slot], st));
        nlev_rank++;
        if (pending >= 0) {
            LZ_HIP(hipEventSynchronize(ev_pin[pending]));
            if (h_pin[pending] >= s) break;  // converged one round ago
        }
        pending = slot;
    }
    LZ_HIP(hipGetLastError());
    k_sa_from_rank<<<g, 256, 0, st>>>(rank_lv[nlev_rank - 1].p, s, SA.get(s), ISA.get(s));
    LZ_HIP(hipGetLastError());
}

void engine::build_lcp_rmq(const u8* T) {
    nlev_rmq = 0;
    const u64 nb = (n >> 9) + 2;
    u32* tab = succ_tab.get(nb);
    k_succ_table<<<cdiv(nb, 256), 256, 0, st>>>(S.p, s, nb, tab);
    if (s == 0) return;
    const unsigned g = cdiv(s, 256);
    rank_levels RL{};
    RL.nlev = nlev_rank;
    RL.step = rank_step;
    for (u32 i = 0; i < nlev_rank; i++) RL.R[i] = rank_lv[i].p;
    u32* L0 = lcp_rmq[0].get(s);
    k_lcp<<<g, 256, 0, st>>>(T, n, S.p, key_len.p, SA.p, s, RL, runs(), L0);
    nlev_rmq = 1;
    for (u32 lv = 1; (1ull << lv) <= s;) {
        const u32 cnt = s - (1u << lv) + 1;
        u32* out = lcp_rmq[lv].get(cnt);
        if ((2ull << lv) <= s) {
            const u32 cnt2 = s - (2u << lv) + 1;
            k_min_level2<<<cdiv(cnt, 256), 256, 0, st>>>(lcp_rmq[lv - 1].p, cnt, 1u << (lv - 1), out, cnt2,
                                                         lcp_rmq[lv + 1].get(cnt2));
            nlev_rmq = lv + 2;
            lv += 2;
        } else {
            k_min_level<<<cdiv(cnt, 256), 256, 0, st>>>(lcp_rmq[lv - 1].p, cnt, 1u << (lv - 1), out);
            nlev_rmq = lv + 1;
            lv += 1;
        }
    }
    LZ_HIP(hipGetLastError());
}

lce_view engine::view(const u8* T) const {
    lce_view L{};
    L.T = T;
    L.n = n;
    L.s = s;
    L.S = S.p;
    L.ISA = ISA.p;
    L.succ = succ_tab.p;
    L.nlev = nlev_rmq;
    for (u32 i = 0; i < nlev_rmq; i++) L.rmq[i] = lcp_rmq[i].p;
    L.R = runs();
    return L;
}

}  // namespace LZ_NS
