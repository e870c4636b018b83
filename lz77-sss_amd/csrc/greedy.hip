// greedy.hip -- the gap-filling factor emitter (factorize_greedy,
// include/lz77_sss/algorithms/approximate/factorize/greedy.cpp:34-140 with
// longest_prev_occ, factorize/common.cpp:33-61, and the single-slot hash
// index rolling_hash_index_107, data_structures/rolling_hash_index_107.hpp:33-172),
// reproduced exactly for num_threads = 1.
//
// The reference walks gaps sequentially against a hash table H that every
// visited gap position writes (5 Karp-Rabin fingerprints mod 2^107-1).  A
// query at q only ever reads "the last position inserted into slot s before
// q".  For a GIVEN set I of inserted positions every lookup is therefore
// fixed by a stable radix sort of the (slot, position) entries of I.  The
// engine speculates I and iterates to a fixed point:
//
//   base   : one full sort of the entries of a base set I_b
//   delta  : I = I_b - R + A with R a bitmap over I_b and A a small sorted
//            list of (slot, position, order) keys; lookups honour both
//   walks  : a walk segment = one gap walk + the LPF factors up to the next
//            gap; all segments run in parallel from their assumed start
//   link   : the host links segments into the chain from position 0; unknown
//            start states become new segments (speculatively, all at once)
//   check  : I' = positions the chain actually inserted.  I' == I  =>  every
//            lookup of the chain was exact -> a WRITE walk emits the factors.
//            Otherwise only the segments holding the next same-slot insert
//            after a changed position are re-walked (dirty), and I <- I'.
//
// The last 64 positions (where the reference's stale / zeroed fingerprints and
// conditional inserts live, rolling_hash_index_107.hpp:80-150) are walked by
// one thread (k_tail) with an exact local model of the table.
#include "../../include/lz77sss.h"
#include "../include/engine.h"
#include "../include/prim.h"
#include "../include/lce_dev.h"

#include <hipcub/hipcub.hpp>
#include <rocprim/block/block_radix_sort.hpp>
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/iterator/counting_iterator.hpp>

#include <algorithm>
#include <array>
#include <chrono>
#include <cmath>
#include <cstring>
#include <limits>
#include <random>
#include <unordered_map>

namespace LZ_NS {

// ---------------------------------------------------------------------------
// 107-bit Mersenne arithmetic (rolling_hash.hpp relies on mersenne::mod, absent
// upstream; residues are canonical in [0, 2^107-1))
static constexpr u128 P107 = ((u128)1 << 107) - 1;
__host__ __device__ static inline u128 mod107(u128 x) {
    x = (x & P107) + (x >> 107);
    x = (x & P107) + (x >> 107);
    return x >= P107 ? x - P107 : x;
}
static u128 mulmod107_host(u128 a, u128 b) {
    u128 r = 0;
    for (int bit = 106; bit >= 0; bit--) {
        r = mod107(r << 1);
        if ((b >> bit) & 1) r = mod107(r + a);
    }
    return r;
}
static u128 powmod107_host(u128 b, u64 e) {
    u128 r = 1;
    while (e) {
        if (e & 1) r = mulmod107_host(r, b);
        b = mulmod107_host(b, b);
        e >>= 1;
    }
    return r;
}

struct gap_cfg {
    pos_t n, nt;        // text length, start of the tail region
    u32 lens[5];
    u64 base[5];
    u32 thr;            // roll_threshold
    u32 mask;           // slot mask (2^k - 1)
    const u128* negpow; // [5][256]: -(o * b^len) mod P
};

// fp * b + negpow_out + in mod P, canonical: fp, negpow_out < P, b < 2^20, so the sum is below
// 2^128 and one 64 x 64 product with its high half, one 43-bit x 20-bit product and two folds at
// bit 107 replace the generic 128-bit product and the inner reduction (k_slots is VALU-bound on
// these rolls)
__device__ __forceinline__ u128 kr_roll(u128 fp, u64 b, u128 negpow_out, u32 in) {
    constexpr u64 M43 = (1ull << 43) - 1;
    const u64 lo = (u64)fp, hi = (u64)(fp >> 64);
    const u64 clo = (u64)negpow_out, chi = (u64)(negpow_out >> 64);
    u64 xlo = lo * b;
    u64 xhi = __umul64hi(lo, b) + hi * b;
    const u64 t = xlo + clo;
    u64 carry = t < xlo ? 1u : 0u;
    const u64 t2 = t + in;
    carry += t2 < t ? 1u : 0u;
    xlo = t2;
    xhi += chi + carry;
#pragma unroll
    for (int f = 0; f < 2; f++) {  // x = (x mod 2^107) + (x >> 107)
        const u64 q = xhi >> 43;
        xhi &= M43;
        const u64 s2 = xlo + q;
        xhi += s2 < xlo ? 1u : 0u;
        xlo = s2;
    }
    if (xhi == M43 && xlo == ~0ull) return 0;  // x == P
    return ((u128)xhi << 64) | xlo;
}
// Phi_x(T[q..q+len)) mod P by direct evaluation (roll-ins only)
__device__ __forceinline__ u128 kr_direct(const u8* T, u64 q, u32 len, u64 b) {
    u128 fp = 0;
    for (u32 j = 0; j < len; j++) fp = kr_roll(fp, b, 0, T[q + j]);
    return fp;
}

// ---------------------------------------------------------------------------
// entries: e = 5*rank + (4 - x); entries of one position are generated in the
// order of longest_prev_occ (x = 4 .. 0)
struct ichunk { pos_t q0, q1; u32 rank0; };

// one thread per (chunk, x): the 5 fingerprint chains of a chunk run on 5 adjacent
// lanes (5x the threads of a chunk-per-thread walk for latency hiding).  A workgroup
// holds SL_CH chunks; every SL_K positions the entries (and positions) go through LDS and
// leave as runs of 5 SL_K contiguous entries per chunk: written straight from the lanes,
// the 4-byte stores 5 chunk lengths apart wrote 4.4x the key bytes to HBM (PMC
// WRITE_SIZE, rr: 1.2 GB for 0.27 GB).
constexpr u32 SL_CH = 64, SL_K = 16, SL_T = 5 * SL_CH;
__global__ __launch_bounds__(SL_T) void k_slots(const u8* __restrict__ T, gap_cfg G, const ichunk* __restrict__ chunks,
                                                u32 nch, u32* __restrict__ keys, u32* __restrict__ vals,
                                                pos_t* __restrict__ ipos, u8* __restrict__ pf = nullptr) {
    __shared__ u32 s_key[SL_CH * SL_K * 5];
    __shared__ pos_t s_pos[SL_CH * SL_K];
    __shared__ ichunk s_ch[SL_CH];
    __shared__ u32 s_maxlen;
    const u32 tid = threadIdx.x;
    const u64 c0 = (u64)blockIdx.x * SL_CH;
    const u32 cl = tid / 5, ord = tid - 5 * cl;  // lanes of a chunk: x = 4, 3, 2, 1, 0 (entry order)
    const int x = 4 - (int)ord;
    if (tid == 0) s_maxlen = 0;
    __syncthreads();
    if (tid < SL_CH) {
        ichunk c{0, 0, 0};
        if (c0 + tid < nch) c = chunks[c0 + tid];
        s_ch[tid] = c;
        atomicMax(&s_maxlen, (u32)(c.q1 - c.q0));
    }
    __syncthreads();
    const ichunk ch = s_ch[cl];
    const bool act = c0 + cl < nch;
    const u32 len = G.lens[x];
    const u64 b = G.base[x];
    const u128* np = G.negpow + x * 256;
    u128 fp = act ? kr_direct(T, ch.q0, len, b) : (u128)0;
    const u32 maxlen = s_maxlen;
    for (u32 k0 = 0; k0 < maxlen; k0 += SL_K) {
        // fingerprints of positions q0 + k0 .. + SL_K into LDS
        for (u32 j = 0; j < SL_K; j++) {
            const pos_t q = ch.q0 + k0 + j;
            if (!act || q >= ch.q1) break;
            const u32 key = (u32)((u64)fp & G.mask);
            s_key[(cl * SL_K + j) * 5 + ord] = key;
            if (x == 4) s_pos[cl * SL_K + j] = q;
            if (q + 1 < ch.q1) fp = kr_roll(fp, b, np[T[q]], T[q + len]);
        }
        __syncthreads();
        // per chunk: entries 5 (rank0 + k0) .. + 5 min(SL_K, left), contiguous
        for (u32 idx = tid; idx < SL_CH * SL_K * 5; idx += SL_T) {
            const u32 c = idx / (SL_K * 5), r = idx - c * (SL_K * 5);
            const ichunk cc = s_ch[c];
            if (c0 + c >= nch) continue;
            const u64 left = (u64)(cc.q1 - cc.q0);
            if (k0 >= left || r >= 5 * min<u64>(SL_K, left - k0)) continue;
            const u64 e = 5ull * (cc.rank0 + k0) + r;
            const u32 key = s_key[idx];
            keys[e] = key;
            if (vals) vals[e] = (u32)e;
            // slot presence (dense ids): plain stores, a hot slot is read far more often.  Here, off
            // the fingerprint chains: in the roll loop the test's load stalled every step of a chain
            if (pf && !pf[key]) pf[key] = 1;
        }
        if (ipos) {
            for (u32 idx = tid; idx < SL_CH * SL_K; idx += SL_T) {
                const u32 c = idx / SL_K, j = idx - c * SL_K;
                const ichunk cc = s_ch[c];
                if (c0 + c >= nch || (u64)k0 + j >= (u64)(cc.q1 - cc.q0)) continue;
                ipos[cc.rank0 + k0 + j] = s_pos[idx];
            }
        }
        __syncthreads();
    }
}
// dense slot ids: a repetitive text hashes its gap positions into few distinct slots
// (rr 1 GiB: 6 091 of 2^25), so sorting dense ids needs 2 radix passes instead of 4.
// Presence as one byte per slot written with plain stores (idempotent: hot slots cost
// no atomics), packed into a bitmap with per-word popcounts; id = rank of the slot.
__global__ void k_presence_pack(const u8* __restrict__ pf, u64 nw, u32* __restrict__ pbm, u32* __restrict__ c) {
    const u64 w = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= nw) return;
    const uint4* q = (const uint4*)(pf + 32 * w);
    const uint4 a = q[0], b = q[1];
    const u32 v[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    u32 bits = 0;
#pragma unroll
    for (int j = 0; j < 8; j++)
#pragma unroll
        for (int k = 0; k < 4; k++) bits |= ((v[j] >> (8 * k)) & 1u) << (4 * j + k);
    pbm[w] = bits;
    c[w] = __popc(bits);
}
__device__ __forceinline__ u32 slot_rank(const u32* pbm, const u32* pwp, u32 k) {
    return pwp[k >> 5] + __popc(pbm[k >> 5] & ((1u << (k & 31)) - 1u));
}
// four keys per thread (16-byte load and store, eight independent table reads in
// flight): one key per thread left the pass latency-bound (rr: 1.9 TB/s)
__global__ void k_dense_keys(const u32* __restrict__ keys, u64 m, const u32* __restrict__ pbm,
                             const u32* __restrict__ pwp, u32* __restrict__ dk) {
    const u64 q = (u64)blockIdx.x * blockDim.x + threadIdx.x;  // quad
    if (4 * q + 3 < m) {
        const uint4 k = *(const uint4*)(keys + 4 * q);
        *(uint4*)(dk + 4 * q) = make_uint4(slot_rank(pbm, pwp, k.x), slot_rank(pbm, pwp, k.y),
                                           slot_rank(pbm, pwp, k.z), slot_rank(pbm, pwp, k.w));
    } else {
        for (u64 e = 4 * q; e < m; e++) dk[e] = slot_rank(pbm, pwp, keys[e]);
    }
}
// pred5[e] = pv[t] for the permutation e = svals[t] without a radix sort by e: bucket
// b holds the 2^PB_SH consecutive ids [b << PB_SH, (b+1) << PB_SH), so its size is known;
// pass 1 moves (e, pv) pairs into their buckets (per tile: an LDS histogram, one global
// atomic per non-empty bucket, LDS cursors), pass 2 scatters each bucket's pairs inside
// its own 1 MiB window of pred5 (L2-local writes)
#ifndef LZ_PB_SH
#define LZ_PB_SH 18
#endif
constexpr u32 PB_SH = LZ_PB_SH;
static_assert(((1ull << 32) >> PB_SH) <= (1u << 14), "k_pb_move's LDS histogram holds 2^14 buckets");
constexpr int PB_T = 1024;
__global__ void k_pb_init(u32* __restrict__ cursor, u32 nb) {
    const u32 b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b < nb) cursor[b] = b << PB_SH;
}
// (the sorted-order predecessor of entry svals[t] is svals[t-1] when skeys[t-1] == skeys[t],
// computed here instead of in a pass of its own)
__global__ __launch_bounds__(PB_T) void k_pb_move(const u32* __restrict__ svals, const u32* __restrict__ skeys, u64 m,
                                                  u64 tile, u32 nb, u32* __restrict__ cursor, u64* __restrict__ tmp) {
    __shared__ u32 h[1u << 14];  // nb <= 2^32 >> PB_SH
    const int tid = (int)threadIdx.x;
    for (u32 b = tid; b < nb; b += PB_T) h[b] = 0;
    __syncthreads();
    const u64 t0 = (u64)blockIdx.x * tile, t1 = min(m, t0 + tile);
    for (u64 t = t0 + tid; t < t1; t += PB_T) atomicAdd(&h[svals[t] >> PB_SH], 1u);
    __syncthreads();
    for (u32 b = tid; b < nb; b += PB_T)
        if (h[b]) h[b] = atomicAdd(&cursor[b], h[b]);
    __syncthreads();
    for (u64 t = t0 + tid; t < t1; t += PB_T) {
        const u32 e = svals[t];
        const u32 pv = (t > 0 && skeys[t - 1] == skeys[t]) ? svals[t - 1] : NONE;
        const u32 p = atomicAdd(&h[e >> PB_SH], 1u);
        tmp[p] = ((u64)e << 32) | pv;
    }
}
// XCD-aware: workgroups are dispatched round-robin over the 8 XCDs, so consecutive logical
// blocks (the same bucket's 1 MiB window of pred5) are given to workgroups of one XCD, whose L2
// then merges the window's scattered 4-byte writes instead of eight L2s writing partial lines
constexpr u32 N_XCD = 8;
__global__ void k_pb_apply(const u64* __restrict__ tmp, u64 m, u32* __restrict__ pred5) {
    const u32 per = gridDim.x / N_XCD;  // grid: a multiple of N_XCD
    const u64 lb = (u64)(blockIdx.x % N_XCD) * per + blockIdx.x / N_XCD;
    const u64 i = lb * blockDim.x + threadIdx.x;
    if (i >= m) return;
    const u64 x = tmp[i];
    pred5[x >> 32] = (u32)x;
}
// k_pred and k_dense_heads in one pass over the sorted dense ids
__global__ void k_pred_heads(const u32* __restrict__ sdk, const u32* __restrict__ svals, u64 m, u32 D,
                             u32* __restrict__ pred5, u32* __restrict__ dstart) {
    const u64 t = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (t > m) return;
    if (t == m) { dstart[D] = (u32)m; return; }
    const bool head = t == 0 || sdk[t - 1] != sdk[t];
    if (head) dstart[sdk[t]] = (u32)t;
    if (pred5) pred5[svals[t]] = head ? NONE : svals[t - 1];
}
// first sorted index of every dense id (all ids occur), dstart[D] = m; four keys per thread
__global__ void k_dense_heads(const u32* __restrict__ sdk, u64 m, u32 D, u32* __restrict__ dstart) {
    const u64 t = 4 * ((u64)blockIdx.x * blockDim.x + threadIdx.x);
    if (t == 0) dstart[D] = (u32)m;
    if (t >= m) return;
    u32 k[4];
    if (t + 3 < m) {
        const uint4 q = *(const uint4*)(sdk + t);
        k[0] = q.x; k[1] = q.y; k[2] = q.z; k[3] = q.w;
    } else {
        for (u64 j = 0; j < 4; j++) k[j] = t + j < m ? sdk[t + j] : NONE;
    }
    u32 prev = t ? sdk[t - 1] : NONE;
#pragma unroll
    for (u32 j = 0; j < 4; j++) {
        if (t + j < m && k[j] != prev) dstart[k[j]] = (u32)(t + j);
        prev = k[j];
    }
}
// slot -> first sorted index with slot >= s: the start of the next present slot's id
// four slots per thread (one presence word, a 16-byte store)
__global__ void k_bstart_rank(const u32* __restrict__ pbm, const u32* __restrict__ pwp,
                              const u32* __restrict__ dstart, u32 nslots, u32 D, u32* __restrict__ bstart) {
    const u64 x = 4 * ((u64)blockIdx.x * blockDim.x + threadIdx.x);
    if (x + 3 < nslots) {
        const u32 w = pbm[x >> 5], r0 = pwp[x >> 5], sh = (u32)x & 31;  // x, x + 3 share the word
        const u32 below = w & ((1u << sh) - 1u);
        const u32 r = r0 + __popc(below);
        const u32 b0 = (w >> sh) & 1u, b1 = (w >> (sh + 1)) & 1u, b2 = (w >> (sh + 2)) & 1u;
        *(uint4*)(bstart + x) = make_uint4(dstart[r], dstart[r + b0], dstart[r + b0 + b1], dstart[r + b0 + b1 + b2]);
    } else {
        for (u64 y = x; y <= nslots; y++) bstart[y] = dstart[y < nslots ? slot_rank(pbm, pwp, (u32)y) : D];
    }
}
// predecessor entry within the same slot (base set)
__global__ void k_pred(const u32* __restrict__ skeys, const u32* __restrict__ svals, u64 m, u32* __restrict__ pred5) {
    const u64 t = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= m) return;
    pred5[svals[t]] = (t > 0 && skeys[t - 1] == skeys[t]) ? svals[t - 1] : NONE;
}
// bucket tables over slots: bucket[s] = first sorted index with slot >= s (bucket[nslots] = m)
struct key_u32 { const u32* k; __device__ u32 operator()(u64 t) const { return k[t]; } };
struct key_u64 { const u64* k; __device__ u32 operator()(u64 t) const { return (u32)(k[t] >> 35); } };
// dense bucket tables without per-thread fill loops (skewed slot sets leave long
// empty ranges): every run head t of slot k writes t at reversed index nslots - k,
// an inclusive min-scan over the reversed array fills the empty slots with the
// next non-empty slot's start, k_unreverse restores slot order
template <class K>
__global__ void k_bucket_heads(K key, u64 m, u32 nslots, u32* __restrict__ rev) {
    const u64 t = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (t > m) return;
    if (t == m) { rev[0] = (u32)m; return; }
    const u32 k = key(t);
    if (t == 0 || key(t - 1) != k) rev[nslots - k] = (u32)t;
}
__global__ void k_unreverse(const u32* __restrict__ rev, u32 nslots, u32* __restrict__ bucket) {
    const u64 x = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (x <= nslots) bucket[x] = rev[nslots - x];
}
struct min_u32_op {
    __device__ __forceinline__ u32 operator()(const u32& a, const u32& b) const { return a < b ? a : b; }
};
template <class K>
__global__ void k_bucket_search(K key, u64 m, u32 nslots, u32* __restrict__ bucket) {
    const u64 sl = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (sl > nslots) return;
    u64 lo = 0, hi = m;
    while (lo < hi) {
        const u64 mid = (lo + hi) >> 1;
        if (key(mid) < sl) lo = mid + 1; else hi = mid;
    }
    bucket[sl] = (u32)lo;
}
// predecessor in sorted order (NONE at a slot boundary), to be sorted back by entry id
__global__ void k_pred_sorted(const u32* __restrict__ skeys, const u32* __restrict__ svals, u64 m, u32* __restrict__ pv) {
    const u64 t = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (t < m) pv[t] = (t > 0 && skeys[t - 1] == skeys[t]) ? svals[t - 1] : NONE;
}
// added entries -> 64-bit keys (slot << 35 | x << 3 | order); x = the position for
// pos_t = uint32_t, the entry's rank in its (position-ordered) list for pos_t = uint64_t
// (ranks are monotone in position, so the key order is the same)
__global__ void k_pack_added(const u32* __restrict__ keys, const pos_t* __restrict__ ipos, u64 m, u64* __restrict__ out) {
    const u64 e = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= m) return;
    const u64 x = sizeof(pos_t) == 4 ? (u64)ipos[e / 5] : e / 5;
    out[e] = ((u64)keys[e] << 35) | (x << 3) | (e % 5);
}
__global__ void k_set_rem(u8* __restrict__ rem, const u32* __restrict__ ranks, u64 m, u8 v) {
    const u64 k = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (k < m) rem[ranks[k]] = v;
}

// factors a speculative walk keeps per segment (seg_tab::stash): the final emission copies
// them instead of re-walking the chain (genome: 20.6 factors per chain segment on average)
constexpr u32 STASH_CAP = 32;
constexpr u32 SEG_NO_STASH = 0x100;  // seg_out::flags: an aliased segment whose stash is incomplete

// ---------------------------------------------------------------------------
struct walk_ctx {
    const u8* T;
    gap_cfg G;
    const pos_t* P;      // phrases (beg,end,src) + sentinel
    // base set
    const pos_t* istart; // interval starts (sorted)
    const pos_t* iend;   // interval ends (exclusive)
    const u32* irank;    // rank of istart
    u32 nint;
    const u32* keys;     // slot of entry e (position order)
    const u32* skeys;    // sorted slots
    const u32* svals;    // entry ids in sorted order
    const u32* pred5;    // predecessor entry in the same slot
    const pos_t* ipos;   // rank -> position
    const pos_t* iposr;  // ipos | POS_RFLAG when the rank is removed (one load per pred step), or null
    u64 nentries;
    const u32* bstart;   // slot -> first sorted base entry (nslots + 1)
    // delta
    const u8* rem;       // removed base ranks
    const u64* akeys;    // sorted added keys (main list)
    u64 nadd;
    const u32* abeg;     // slot -> first added key (nslots + 1)
    const pos_t* apos;   // positions of the main list (rank -> position, pos_t = uint64_t keys)
    u64 napos;
    const u64* akeys2;   // sorted added keys (extra list, positions joined after the main build)
    u64 nadd2;
    const u32* abeg2;
    const pos_t* apos2;
    u64 napos2;
    const u32* bmI;      // current insert set (membership of added positions)
    pos_t bmoff;         // text position of bit 0 of the window bitmaps (a multiple of 32)
    const pos_t* Hs;     // window mode: slot -> last insert before the window (POS_NONE), or null
    u32* hs_used;        // speculative block: bitmap of the slots whose entry-table value a lookup used
    pos_t blk_start;     //   (values below the block start come from the entry table)
    int use_pred;        // base lookups via pred5 (else bucket search)
    lce_view L;
};

constexpr pos_t POS_RFLAG = (pos_t)1 << (8 * sizeof(pos_t) - 1);  // iposr: removed (texts below 2^31 / 2^63)
__device__ __forceinline__ u32 base_rank(const walk_ctx& W, pos_t q, int& hint) {
    if (hint >= 0) {
        if (q >= W.istart[hint] && q < W.iend[hint]) return W.irank[hint] + (u32)(q - W.istart[hint]);
        // a walk moves forward: the query after an LPF phrase is usually in the next interval
        const int h1 = hint + 1;
        if ((u32)h1 < W.nint && q >= W.istart[h1] && q < W.iend[h1]) {
            hint = h1;
            return W.irank[h1] + (u32)(q - W.istart[h1]);
        }
    }
    u32 lo = 0, hi = W.nint;
    while (lo < hi) {
        const u32 mid = (lo + hi) >> 1;
        if (W.istart[mid] <= q) lo = mid + 1; else hi = mid;
    }
    if (lo == 0) return NONE;
    const u32 k = lo - 1;
    if (q >= W.iend[k]) return NONE;
    hint = (int)k;
    return W.irank[k] + (u32)(q - W.istart[k]);
}
__device__ __forceinline__ pos_t occ_max(pos_t a, pos_t b) {
    if (a == POS_NONE) return b;
    if (b == POS_NONE) return a;
    return max(a, b);
}
__device__ __forceinline__ pos_t occ_min(pos_t a, pos_t b) {
    if (a == POS_NONE) return b;
    if (b == POS_NONE) return a;
    return min(a, b);
}
// last base entry strictly before (slot, q, ord) in processing order, skipping removed
__device__ pos_t base_last_before(const walk_ctx& W, u32 slot, pos_t q, u32 ord) {
    const u64 beg = W.bstart[slot], end = W.bstart[slot + 1];
    // within [beg, end) entries are in (position, order) order: first >= (q, ord)
    u64 lo = beg, hi = end;
    while (lo < hi) {
        const u64 mid = (lo + hi) >> 1;
        const u32 e = W.svals[mid];
        const pos_t pq = W.ipos[e / 5];
        const u32 po = e % 5;
        if (pq < q || (pq == q && po < ord)) lo = mid + 1; else hi = mid;
    }
    for (u64 t = lo; t > beg; t--) {
        const u32 rk = W.svals[t - 1] / 5;
        if (!W.rem[rk] || W.ipos[rk] == q) return W.ipos[rk];
    }
    return POS_NONE;
}
__device__ __forceinline__ bool in_I(const walk_ctx& W, pos_t q) {
    const pos_t r = q - W.bmoff;
    return (W.bmI[r >> 5] >> (r & 31)) & 1;
}
// key field of position q in an added list: q itself (u32) or the number of list
// positions below q (u64; first_ge) / at or below q (!first_ge)
__device__ __forceinline__ u64 added_x(const pos_t* apos, u64 na, pos_t q, bool first_ge) {
    if (sizeof(pos_t) == 4) return (u64)q + (first_ge ? 0 : 1);
    u64 lo = 0, hi = na;
    while (lo < hi) {
        const u64 mid = (lo + hi) >> 1;
        if (first_ge ? apos[mid] < q : apos[mid] <= q) lo = mid + 1; else hi = mid;
    }
    return lo;
}
__device__ __forceinline__ pos_t added_pos(const pos_t* apos, u64 key) {
    const u64 x = (key >> 3) & 0xFFFFFFFFull;
    return sizeof(pos_t) == 4 ? (pos_t)x : apos[x];
}
__device__ pos_t added_last_before_1(const walk_ctx& W, const u64* ak, const u32* ab, const pos_t* apos, u64 na,
                                     u32 slot, pos_t q, u32 ord) {
    // rank keys (pos_t = uint64_t): when q is not in the list, the entries of rank
    // lower_bound(q) lie after q whatever their order, so the search key takes order 0
    const u64 x = added_x(apos, na, q, true);
    const u32 o = (sizeof(pos_t) == 4 || (x < na && apos[x] == q)) ? ord : 0u;
    const u64 key = ((u64)slot << 35) | (x << 3) | o;
    u64 lo = ab[slot], hi = ab[slot + 1];  // first >= key
    const u64 beg = lo;
    while (lo < hi) {
        const u64 mid = (lo + hi) >> 1;
        if (ak[mid] < key) lo = mid + 1; else hi = mid;
    }
    for (u64 t = lo; t > beg; t--) {
        const pos_t pq = added_pos(apos, ak[t - 1]);
        if (pq == q || in_I(W, pq)) return pq;
    }
    return POS_NONE;
}
__device__ pos_t added_last_before(const walk_ctx& W, u32 slot, pos_t q, u32 ord) {
    pos_t r = POS_NONE;
    if (W.nadd) r = added_last_before_1(W, W.akeys, W.abeg, W.apos, W.napos, slot, q, ord);
    if (W.nadd2) r = occ_max(r, added_last_before_1(W, W.akeys2, W.abeg2, W.apos2, W.napos2, slot, q, ord));
    return r;
}
// last insert into the slot before the window (the carried table holds pos + 1, 0 = none)
__device__ __forceinline__ pos_t carried(const walk_ctx& W, u32 slot) {
    const pos_t h = W.Hs[slot];
    if (W.hs_used && (h == 0 || h - 1 < W.blk_start)) atomicOr(&W.hs_used[slot >> 5], 1u << (slot & 31));
    return h ? h - 1 : POS_NONE;
}
// H[slot of (q,x)] just before longest_prev_occ's advance_and_get_occ<x> at q
__device__ pos_t lookup(const walk_ctx& W, pos_t q, int x, int& hint) {
    const u32 ord = 4 - x;
    const u32 rk = base_rank(W, q, hint);
    u32 slot;
    pos_t cb;
    if (rk != NONE) {
        const u32 e = 5 * rk + ord;
        slot = W.keys[e];
        if (W.use_pred && W.iposr) {
            u32 p = W.pred5[e];
            pos_t v = p == NONE ? 0 : W.iposr[p / 5];
            while (p != NONE && (v & POS_RFLAG) && (v & ~POS_RFLAG) != q) {
                p = W.pred5[p];
                if (p != NONE) v = W.iposr[p / 5];
            }
            cb = p == NONE ? POS_NONE : (v & ~POS_RFLAG);
        } else if (W.use_pred) {
            u32 p = W.pred5[e];
            while (p != NONE && W.rem[p / 5] && W.ipos[p / 5] != q) p = W.pred5[p];
            cb = p == NONE ? POS_NONE : W.ipos[p / 5];
        } else {
            // entries of a bucket are in ascending entry order: locate e, then walk back
            const u64 beg = W.bstart[slot];
            u64 lo = beg, hi = W.bstart[slot + 1];
            while (lo < hi) {
                const u64 mid = (lo + hi) >> 1;
                if (W.svals[mid] < e) lo = mid + 1; else hi = mid;
            }
            cb = POS_NONE;
            for (u64 t = lo; t > beg; t--) {
                const u32 r2 = W.svals[t - 1] / 5;
                if (!W.rem[r2] || W.ipos[r2] == q) { cb = W.ipos[r2]; break; }
            }
        }
    } else {
        slot = (u32)((u64)kr_direct(W.T, q, W.G.lens[x], W.G.base[x]) & W.G.mask);
        cb = base_last_before(W, slot, q, ord);
    }
    const pos_t r = occ_max(cb, added_last_before(W, slot, q, ord));
    return (r == POS_NONE && W.Hs) ? carried(W, slot) : r;  // inserts of earlier windows are all older
}

// ---------------------------------------------------------------------------
// walks
template <bool WRITE>
__device__ void walk_segment(const walk_ctx& W, seg_in in, seg_out* __restrict__ og, pos_t* fout) {
    // outputs go straight to the table entry og (the bnd/single lists are indexed
    // dynamically: a local copy of seg_out would live in scratch memory)
    const u8* T = W.T;
    const pos_t n = W.G.n, nt = W.G.nt;
    const pos_t* P = W.P;
    pos_t i = in.start, idx = in.idxpos, e = in.start, next = n;
    u32 p = in.p, zm = in.zmask;
    u32 nf = 0, ns = 0, flags = 0, nb = 0;
    bool first_gap = true;
    int hint = -1;
    u64 guard = 0;
    const u64 guard_max = 4ull * n + 1024;
    auto finish = [&]() {
        if (WRITE) return;
        og->next = next;
        og->e = e;
        og->nfact = nf;
        og->idxpos = idx;
        og->zmask = zm;
        og->nsingle = ns;
        og->flags = flags;
        og->nbnd = nb;
    };
    auto emit = [&](pos_t src, pos_t len) {
        if (WRITE || (fout && nf < STASH_CAP)) { fout[2 * nf] = src; fout[2 * nf + 1] = len; }
        nf++;
    };
    auto query = [&](pos_t q, pos_t& fsrc, pos_t& flen) {
        fsrc = T[q];
        flen = 0;
        for (int x = 4; x >= 0; x--) {
            const pos_t occ = lookup(W, q, x, hint);
            if (occ != POS_NONE && occ < q && T[occ] == T[q]) {
                flen = (pos_t)dev_lce(W.L, occ, q);
                fsrc = occ;
                return;
            }
        }
    };
    for (;;) {
        pos_t gap_end = P[3 * p];
        if (i < gap_end) {
            if (idx < i) {
                if (i - idx > W.G.thr) {  // reinit (matters only in the tail region)
                    zm = 0;
                    for (int x = 0; x < 5; x++) zm |= ((u64)i + W.G.lens[x] >= n) ? (1u << x) : 0u;
                }
                idx = i;
            }
            do {
                // the tail test comes first: a chunk walk that stopped at its boundary on a
                // factor start >= nt would hand the tail walk a start past the positions its
                // last factor advanced over in the tail region (conditional inserts,
                // rolling_hash_index_107.hpp:121-127), which the tail model then never sees
                if (i >= nt) { flags |= 1; finish(); return; }
                if (i >= in.lim) {  // chunk boundary reached: stop at the next factor start
                    next = i;
                    e = i;
                    finish();
                    return;
                }
                if (++guard > guard_max || i > n) { flags |= 4; finish(); return; }
                if (!WRITE && first_gap && nb < SEG_NBND) og->bnd[nb++] = i;
                pos_t fsrc, flen;
                query(i, fsrc, flen);
                idx = i + 1;
                i += flen ? flen : 1;
                if (i > gap_end) {
                    if (i <= P[3 * p + 1]) {
                        flen -= i - gap_end;
                        i = gap_end;
                    } else {
                        do { p++; } while (P[3 * p + 1] <= i);
                        gap_end = P[3 * p];
                    }
                }
                emit(fsrc, flen);
                if (idx < i) idx = i;
            } while (i < gap_end);
            e = i;
        }
        first_gap = false;
        if (i == n) break;
        const pos_t exc = i - gap_end;
        pos_t lsrc = P[3 * p + 2] + exc, llen = (P[3 * p + 1] - P[3 * p]) - exc;
        if (idx == i) {
            if (i >= nt) { flags |= 1; finish(); return; }
            pos_t fsrc, flen;
            query(i, fsrc, flen);
            idx = i + 1;
            if (ns < 4) { if (!WRITE) og->single[ns] = i; } else flags |= 2;
            ns++;
            if (flen > llen) { lsrc = fsrc; llen = flen; }
        }
        emit(lsrc, llen);
        i += llen;
        if (++guard > guard_max || i > n || llen == 0) { flags |= 4; finish(); return; }
        while (P[3 * p + 1] <= i) p++;
        if (i < P[3 * p]) { next = i; break; }
    }
    finish();
}

// successor insert (next position of the same slot after y) in the current set:
// the only query whose lookup can change when y joins or leaves I
__global__ void k_dirty(walk_ctx W, const pos_t* __restrict__ ys, u64 m, pos_t* __restrict__ out) {
    const u64 k = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= m) return;
    const pos_t y = ys[k];
#pragma unroll 1
    for (int x = 0; x < 5; x++) {
        const u32 slot = (u32)((u64)kr_direct(W.T, y, W.G.lens[x], W.G.base[x]) & W.G.mask);
        pos_t best = POS_NONE;
        const u64 bend = W.bstart[slot + 1];
        u64 lo = W.bstart[slot], hi = bend;  // first entry after (slot, y)
        while (lo < hi) {
            const u64 mid = (lo + hi) >> 1;
            if (W.ipos[W.svals[mid] / 5] <= y) lo = mid + 1; else hi = mid;
        }
        for (u64 t = lo; t < bend; t++) {
            const u32 rk = W.svals[t] / 5;
            if (!W.rem[rk]) { best = W.ipos[rk]; break; }
        }
        for (int li = 0; li < 2; li++) {
            const u64* ak = li ? W.akeys2 : W.akeys;
            const u32* ab = li ? W.abeg2 : W.abeg;
            const pos_t* ap = li ? W.apos2 : W.apos;
            if (!(li ? W.nadd2 : W.nadd)) continue;
            const u64 key = ((u64)slot << 35) | (added_x(ap, li ? W.napos2 : W.napos, y, false) << 3);
            u64 a = ab[slot], b = ab[slot + 1];
            const u64 aend = b;
            while (a < b) {
                const u64 mid = (a + b) >> 1;
                if (ak[mid] < key) a = mid + 1; else b = mid;
            }
            for (; a < aend; a++) {
                const pos_t pq = added_pos(ap, ak[a]);
                if (in_I(W, pq)) { best = occ_min(best, pq); break; }
            }
        }
        out[5 * k + x] = best;
    }
}

// incremental delta: y joined (flag 1) or left (flag 0) I; base positions flip
// their removed bit, others are reported as additions to maintain on the host
__global__ void k_flip(walk_ctx W, const pos_t* __restrict__ ys, const u8* __restrict__ joined, u64 m,
                       u8* __restrict__ rem, u8* __restrict__ in_base) {
    const u64 k = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= m) return;
    int hint = -1;
    const u32 rk = base_rank(W, ys[k], hint);
    in_base[k] = rk != NONE;
    if (rk != NONE) {
        rem[rk] = joined[k] ? 0 : 1;
        if (W.iposr) ((pos_t*)W.iposr)[rk] = W.ipos[rk] | (joined[k] ? (pos_t)0 : POS_RFLAG);
    }
}
// ---------------------------------------------------------------------------
// exact single-thread walk from a segment start to the end of the text, with
// a local model of the inserts in the tail region (last 64 positions)
struct tail_ins { u32 slot; pos_t pos; };
constexpr int TAIL_CAP = 64 * 5 + 8;

__global__ void k_tail(walk_ctx W, seg_in in, pos_t* __restrict__ fact, u64 off, u64* __restrict__ count_out,
                       pos_t* __restrict__ ins_out /* [a, b) pairs below the tail region, cap 8 */) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    const u8* T = W.T;
    const pos_t n = W.G.n, nt = W.G.nt;
    const pos_t* P = W.P;
    tail_ins loc[TAIL_CAP];
    int nloc = 0;
    pos_t i = in.start, idx = in.idxpos;
    u32 p = in.p, zm = in.zmask;
    u64 nf = 0;
    int hint = -1;
    u32 nins = 0;
    auto fp_slot = [&](pos_t q, int x) -> u32 {
        const u32 len = W.G.lens[x];
        if ((zm >> x & 1) || (u64)len > n) return 0;
        const u64 qq = ((u64)q + len <= n) ? q : n - len;
        return (u32)((u64)kr_direct(T, qq, len, W.G.base[x]) & W.G.mask);
    };
    auto tail_lookup = [&](u32 slot) -> pos_t {
        for (int k = nloc - 1; k >= 0; k--)
            if (loc[k].slot == slot) return loc[k].pos;
        // every base / added entry lies below nt
        const pos_t r = occ_max(base_last_before(W, slot, nt, 0), added_last_before(W, slot, nt, 0));
        return (r == POS_NONE && W.Hs) ? carried(W, slot) : r;
    };
    auto insert = [&](pos_t q, u32 slot) {
        if (nloc < TAIL_CAP) loc[nloc++] = {slot, q};
    };
    auto query = [&](pos_t q, pos_t& fsrc, pos_t& flen) {
        fsrc = T[q];
        flen = 0;
        bool hit = false;
        for (int x = 4; x >= 0; x--) {
            if (q < nt) {
                if (hit) continue;
                const pos_t occ = lookup(W, q, x, hint);
                if (occ != POS_NONE && occ < q && T[occ] == T[q]) {
                    flen = (pos_t)dev_lce(W.L, occ, q);
                    fsrc = occ;
                    hit = true;
                }
            } else if (!hit) {
                const u32 slot = fp_slot(q, x);
                const pos_t occ = tail_lookup(slot);
                insert(q, slot);  // advance_and_get_occ always inserts
                if (occ != POS_NONE && occ < q && T[occ] == T[q]) {
                    flen = (pos_t)dev_lce(W.L, occ, q);
                    fsrc = occ;
                    hit = true;
                }
            } else if ((u64)q + W.G.lens[x] < n) {
                insert(q, fp_slot(q, x));  // advance<x> inserts only if cur_pos + len < n
            }
        }
    };
    auto advance_to = [&](pos_t target) {
        for (; idx < target; idx++)
            if (idx >= nt)
                for (int x = 0; x < 5; x++)
                    if ((u64)idx + W.G.lens[x] < n) insert(idx, fp_slot(idx, x));
    };
    auto emit = [&](pos_t src, pos_t len) {
        fact[2 * (off + nf)] = src;
        fact[2 * (off + nf) + 1] = len;
        nf++;
    };
    auto record = [&](pos_t a, pos_t b) {
        b = min(b, nt);
        if (a >= b) return;
        if (nins > 0 && ins_out[2 * (nins - 1) + 1] >= a) {
            ins_out[2 * (nins - 1) + 1] = max(ins_out[2 * (nins - 1) + 1], b);
            return;
        }
        if (nins < 8) { ins_out[2 * nins] = a; ins_out[2 * nins + 1] = b; nins++; }
        else count_out[2] = 1;
    };
    count_out[2] = 0;
    u64 guard = 0;
    for (;;) {
        if (++guard > 4ull * n + 1024 || i > n) { count_out[2] = 2; break; }
        pos_t gap_end = P[3 * p];
        if (i < gap_end) {
            if (idx < i) {
                if (i - idx > W.G.thr) {
                    zm = 0;
                    for (int x = 0; x < 5; x++) zm |= ((u64)i + W.G.lens[x] >= n) ? (1u << x) : 0u;
                }
                idx = i;  // roll: fingerprints advance, nothing inserted
            }
            const pos_t walk_start = i;
            do {
                pos_t fsrc, flen;
                query(i, fsrc, flen);
                idx = i + 1;
                i += flen ? flen : 1;
                if (i > gap_end) {
                    if (i <= P[3 * p + 1]) {
                        flen -= i - gap_end;
                        i = gap_end;
                    } else {
                        do { p++; } while (P[3 * p + 1] <= i);
                        advance_to(gap_end);
                        gap_end = P[3 * p];
                    }
                }
                emit(fsrc, flen);
                advance_to(i);
            } while (i < gap_end);
            record(walk_start, i);
        }
        if (i == n) break;
        const pos_t exc = i - gap_end;
        pos_t lsrc = P[3 * p + 2] + exc, llen = (P[3 * p + 1] - P[3 * p]) - exc;
        if (idx == i) {
            pos_t fsrc, flen;
            query(i, fsrc, flen);
            idx = i + 1;
            record(i, i + 1);
            if (flen > llen) { lsrc = fsrc; llen = flen; }
        }
        emit(lsrc, llen);
        i += llen;
        while (P[3 * p + 1] <= i) p++;
    }
    count_out[0] = nf;
    count_out[1] = nins;
}

// ---------------------------------------------------------------------------
// Bounded-cost completion: the reference loop itself (greedy.cpp:46-134 with
// longest_prev_occ, factorize/common.cpp:33-61) on one thread, against a
// materialized single-slot table H and the literal rolling_hash_index_107
// semantics (reinit / roll / advance / advance_and_get_occ, including stale and
// zeroed fingerprints at the text end, rolling_hash_index_107.hpp:80-150).  It
// starts from an exact chain state (a segment start whose predecessors were all
// exact) with H holding the last insert per slot below that state, so its output
// continues the confirmed prefix.  Used when the speculation does not reach its
// fixed point within the round budget, or a walk reports an internal overflow.
__device__ __forceinline__ void atomic_max_pos(pos_t* a, pos_t v) {
    if constexpr (sizeof(pos_t) == 4) atomicMax((u32*)a, (u32)v);
    else atomicMax((unsigned long long*)a, (unsigned long long)v);
}
__global__ void k_h_fill(const u8* __restrict__ T, gap_cfg G, const u32* __restrict__ bm, pos_t off, pos_t y,
                         pos_t* __restrict__ H) {
    const u64 w = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (off + w * 32 >= y) return;
    u32 bits = bm[w];
    while (bits) {
        const pos_t q = off + (pos_t)(32 * w) + (pos_t)__builtin_ctz(bits);
        bits &= bits - 1;
        if (q >= y) break;
        // confirmed inserts lie below the tail region: all 5 fingerprints are full windows
        for (int x = 0; x < 5; x++)
            atomic_max_pos(&H[(u32)((u64)kr_direct(T, q, G.lens[x], G.base[x]) & G.mask)], q + 1);
    }
}
__global__ void k_h_fix(pos_t* __restrict__ H, u64 m) {  // pos + 1 (0 = none) -> pos (POS_NONE)
    const u64 k = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (k < m) H[k] = H[k] ? H[k] - 1 : POS_NONE;
}
__global__ void k_h_unfix(const pos_t* __restrict__ H, u64 m, pos_t* __restrict__ Hs) {  // pos -> pos + 1
    const u64 k = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (k < m) Hs[k] = H[k] == POS_NONE ? 0 : H[k] + 1;
}
// out: [0] factors, [1] guard tripped, [2] exit position (>= stop), [3] index position there
__global__ void k_seq_walk(const u8* __restrict__ T, gap_cfg G, const pos_t* __restrict__ P, lce_view L,
                           pos_t* __restrict__ H, seg_in in, pos_t stop, pos_t* __restrict__ fact, u64 off,
                           u64* __restrict__ out, u32* __restrict__ hs_used, pos_t blk_start) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    const pos_t n = G.n;
    u128 fp[5];
    pos_t cur = in.idxpos;
    for (int x = 0; x < 5; x++) {  // fingerprint state at cur
        const u32 len = G.lens[x];
        if (((in.zmask >> x) & 1) || len > n) fp[x] = 0;
        else fp[x] = kr_direct(T, (u64)cur + len <= n ? cur : n - len, len, G.base[x]);
    }
    auto slot_of = [&](int x) -> u32 { return (u32)((u64)fp[x] & G.mask); };
    auto roll1 = [&](int x) {
        if ((u64)cur + G.lens[x] < n) fp[x] = kr_roll(fp[x], G.base[x], G.negpow[x * 256 + T[cur]], T[cur + G.lens[x]]);
    };
    auto roll = [&]() {
        for (int x = 0; x < 5; x++) roll1(x);
        cur++;
    };
    auto reinit = [&](pos_t pos) {
        cur = pos;
        for (int x = 0; x < 5; x++) fp[x] = ((u64)pos + G.lens[x] < n) ? kr_direct(T, pos, G.lens[x], G.base[x]) : 0;
    };
    auto advance = [&]() {
        for (int x = 0; x < 5; x++)
            if ((u64)cur + G.lens[x] < n) {
                H[slot_of(x)] = cur;
                roll1(x);
            }
        cur++;
    };
    auto longest_prev_occ = [&](pos_t pos, pos_t& fsrc, pos_t& flen) {
        fsrc = T[pos];
        flen = 0;
        for (int x = 4; x >= 0; x--) {
            if (flen == 0) {  // advance_and_get_occ<x>: always inserts
                const u32 sl = slot_of(x);
                const pos_t occ = H[sl];
                if (hs_used && (occ == POS_NONE || occ < blk_start)) atomicOr(&hs_used[sl >> 5], 1u << (sl & 31));
                H[sl] = cur;
                roll1(x);
                if (occ < pos && T[occ] == T[pos]) {
                    flen = (pos_t)dev_lce(L, occ, pos);
                    fsrc = occ;
                }
            } else if ((u64)cur + G.lens[x] < n) {  // advance<x>
                H[slot_of(x)] = cur;
                roll1(x);
            }
        }
        cur++;
    };
    u64 nf = 0, guard = 0;
    auto emit = [&](pos_t src, pos_t len) {
        fact[2 * (off + nf)] = src;
        fact[2 * (off + nf) + 1] = len;
        nf++;
    };
    pos_t i = in.start;
    u32 p = in.p;
    out[1] = 0;
    out[2] = n;
    for (;;) {
        if (++guard > 4ull * n + 1024 || i > n) { out[1] = 1; break; }
        pos_t gap_end = P[3 * p];
        // window end: hand over at a gap start or a gap-walk factor start >= stop (the
        // segment walks' boundaries), before the index rolls to it
        if (i >= stop && i < gap_end) { out[2] = i; break; }
        if (i < gap_end) {
            if (cur < i) {
                if (i - cur <= G.thr) {
                    do roll(); while (cur < i);
                } else {
                    reinit(i);
                }
            }
            bool stopped = false;
            do {
                if (i >= stop) { stopped = true; break; }
                pos_t fsrc, flen;
                longest_prev_occ(i, fsrc, flen);
                i += flen ? flen : 1;
                if (i > gap_end) {
                    if (i <= P[3 * p + 1]) {
                        flen -= i - gap_end;
                        i = gap_end;
                    } else {
                        do { p++; } while (P[3 * p + 1] <= i);
                        while (cur < gap_end) advance();
                        gap_end = P[3 * p];
                    }
                }
                emit(fsrc, flen);
                while (cur < i) advance();
            } while (i < gap_end);
            if (stopped) { out[2] = i; break; }
        }
        if (i == n) break;
        const pos_t exc = i - gap_end;
        pos_t lsrc = P[3 * p + 2] + exc, llen = (P[3 * p + 1] - P[3 * p]) - exc;
        if (cur == i) {
            pos_t fsrc, flen;
            longest_prev_occ(i, fsrc, flen);
            if (flen > llen) { lsrc = fsrc; llen = flen; }
        }
        emit(lsrc, llen);
        i += llen;
        while (P[3 * p + 1] <= i) p++;
    }
    out[0] = nf;
    out[3] = cur;
}
// first set bit of a bitmap (~0 if none), one atomic per workgroup
__global__ void k_first_bit(const u32* __restrict__ bm, u64 nw, pos_t off, u64* __restrict__ out) {
    const u64 w = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    const u64 v = (w < nw && bm[w]) ? off + 32 * w + (u64)__builtin_ctz(bm[w]) : ~0ull;
    block_min64(out, v);
}

// phrase statistics (approximate/common.cpp:98-157, p = 1)
__global__ void k_phrase_info(const pos_t* __restrict__ P, u32 m, pos_t n, u64* __restrict__ acc) {
    const u64 k = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    u64 len = 0, gaps = 0;
    if (k < m) {
        const pos_t b = P[3 * k], e = P[3 * k + 1];
        len = e - b;
        if (k == 0 ? b > 0 : b > P[3 * (k - 1) + 1]) gaps++;
        if (k == m - 1 && e < n) gaps++;
    }
    block_add64(&acc[0], len);
    block_add64(&acc[1], gaps);
}

// ---------------------------------------------------------------------------
// host side
struct gap_params_h {
    std::array<u32, 5> patt_lens{};
    u32 roll_threshold = 0;
    u32 log2_size_h = 0;
};

// lz77_sss.hpp:99-122, 425-461 and rolling_hash_index_107.hpp:59-70 (the entry
// counts depend on sizeof(pos_t); malloc_count_peak() - malloc_count_current() == 0)
static gap_params_h choose_gap_params(pos_t n, u64 num_lpf, pos_t len_lpf_phr, u64 num_gaps) {
    static const std::array<std::pair<double, std::array<u32, 5>>, 10> table{{
        {6, {2, 3, 4, 5, 6}}, {8, {2, 3, 4, 6, 8}}, {12, {2, 3, 4, 8, 12}}, {16, {2, 4, 6, 9, 16}},
        {32, {2, 4, 6, 10, 20}}, {64, {2, 4, 7, 12, 28}}, {128, {2, 4, 8, 16, 36}},
        {256, {2, 5, 10, 20, 42}}, {1024, {2, 6, 12, 24, 48}},
        {std::numeric_limits<double>::max(), {2, 8, 16, 32, 64}}}};
    gap_params_h g;
    const pos_t len_gaps = n - len_lpf_phr;
    const double rel_len_gaps = len_gaps / (double)n;
    const double avg_gap_len = len_gaps / (double)num_gaps;
    const double avg_lpf_phr_len = len_lpf_phr / (double)num_lpf;
    const u64 target = std::min<u64>(1ull << 30, std::max<u64>({1ull << 20, 0ull, (u64)((n / 3.0) * rel_len_gaps)}));
    const double guess = std::min<double>({avg_gap_len, avg_lpf_phr_len, 8.0 * std::pow(128, 1.0 - rel_len_gaps)});
    for (auto& [thr, lens] : table)
        if (guess <= thr) { g.patt_lens = lens; break; }
    u32 rt = 0;
    for (int j = 0; j < 5; j++) rt += g.patt_lens[j];
    g.roll_threshold = rt / 5;
    const int64_t rk_bytes = (int64_t)(80 + 16 * 256 * 256) * 5;  // rk_prime<107>::byte_size() * 5
    const int64_t min_index_size = (int64_t)(std::max<pos_t>(1u << 20, (pos_t)(n * 0.1)) / sizeof(pos_t));
    const int64_t max_index_size = (1ll << 30) / (int64_t)sizeof(pos_t);
    const int64_t target_entries = std::max<int64_t>(0, (int64_t)target - rk_bytes) / (int64_t)sizeof(pos_t);
    const uint64_t target_size_h = std::min<int64_t>(max_index_size, std::max<int64_t>(min_index_size, target_entries));
    g.log2_size_h = (u8)std::round(std::log2(target_size_h));
    return g;
}

// ---------------------------------------------------------------------------
// device-resident segment table and orchestration (engine::factorize_greedy)
constexpr u32 PENDING = 0xFFFFFFFEu;  // seg_at entry being created in this pass

struct seg_tab {
    seg_in* sin;
    seg_out* sout;
    u8* valid;       // output exact for the current lookup state
    u32* succ;       // id of the segment starting at sout.next (NONE = unknown)
    u32* seg_at;     // text position - segoff -> segment id (NONE / PENDING)
    pos_t segoff;    // window start
    u32* nseg;       // device counter
    u32 cap;
    const pos_t* cbv;  // chunk boundaries (sorted)
    u32 ncb;
    const pos_t* P;  // phrases (beg, end, src) + sentinel
    u32 m;
    pos_t N;         // end of the window: a segment whose next start is >= N ends the chain
    u32 zmask0;
    u32* err;        // bit 1: table full, 2: too many LPF-start queries, 4: walk guard
    pos_t* stash;    // per segment: the first STASH_CAP factors of its last walk (src, len)
};


__device__ __forceinline__ u32 first_phrase_after(const pos_t* P, u32 m, pos_t a) {  // smallest k: end_k > a
    u32 lo = 0, hi = m;
    while (lo < hi) {
        const u32 mid = (lo + hi) >> 1;
        if (P[3 * mid + 1] <= a) lo = mid + 1; else hi = mid;
    }
    return lo;
}
__device__ __forceinline__ pos_t upper_cb(const seg_tab& S, pos_t a) {  // first chunk boundary > a (N if none)
    u32 lo = 0, hi = S.ncb;
    while (lo < hi) {
        const u32 mid = (lo + hi) >> 1;
        if (S.cbv[mid] <= a) lo = mid + 1; else hi = mid;
    }
    return lo < S.ncb ? S.cbv[lo] : S.N;
}
__device__ __forceinline__ seg_in make_seg_in(const seg_tab& S, pos_t a) {
    return seg_in{a, first_phrase_after(S.P, S.m, a), a, S.zmask0, upper_cb(S, a)};
}

// default segments: one per gap (phrase k's gap [end_{k-1}, beg_k)) + chunk
// boundaries inside long gaps; also the initial speculation I_0 and the base
// superset (gaps + the LPF-start query position, + interiors of short phrases)
__device__ __forceinline__ void gap_of(const pos_t* P, u32 k, pos_t& a, pos_t& b) {
    a = k ? P[3 * (k - 1) + 1] : 0;
    b = P[3 * k];
}
__device__ __forceinline__ u32 gap_chunks(pos_t a, pos_t b, u32 CH) {
    return (b > a && b - a > 2 * (pos_t)CH) ? (u32)((b - a - CH / 2 - 1) / CH) : 0;
}
// gap k clipped to the window [lo, hi)
__device__ __forceinline__ void gap_in(const pos_t* P, u32 k, pos_t lo, pos_t hi, pos_t& a, pos_t& b) {
    gap_of(P, k, a, b);
    a = max(a, lo);
    b = min(b, hi);
}
// chunk boundaries stay below the tail region (cmax = nt): a chunk walk starting inside
// it would walk tail positions without the tail model's stale-fingerprint semantics
__global__ void k_gap_counts(const pos_t* __restrict__ P, u32 m, u32 CH, pos_t lo, pos_t hi, pos_t cmax,
                             u32* __restrict__ nsegs, u32* __restrict__ ncbs) {
    const u64 k = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (k > m) return;
    pos_t a, b;
    gap_in(P, (u32)k, lo, hi, a, b);
    u32 K = gap_chunks(a, b, CH);
    if (K) K = min(K, a < cmax ? (u32)((cmax - a - 1) / CH) : 0u);  // boundaries a + t CH < cmax
    nsegs[k] = (a < b) ? 1 + K : 0;
    ncbs[k] = K;
}
// item id (a chunk boundary or a segment) -> its gap: the k with off[k] <= id < off[k+1]
// (off = exclusive scan over the m + 1 gaps; a gap without items repeats its offset).
// One thread per item: a long gap (repetitive text: 10^5 chunks in one gap) is spread
// over the grid instead of being walked by one thread or wave
__device__ __forceinline__ u32 item_gap(const u32* __restrict__ off, u32 m, u32 id) {
    u32 lo = 0, hi = m + 1;
    while (hi - lo > 1) {
        const u32 mid = (lo + hi) >> 1;
        if (off[mid] <= id) lo = mid; else hi = mid;
    }
    return lo;
}
__global__ void k_gap_cbv(const pos_t* __restrict__ P, u32 m, u32 CH, pos_t lo, pos_t hi, const u32* __restrict__ cb_off,
                          u32 ncb, pos_t* __restrict__ cbv) {
    const u64 id = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (id >= ncb) return;
    const u32 k = item_gap(cb_off, m, (u32)id);
    pos_t a, b;
    gap_in(P, k, lo, hi, a, b);
    cbv[id] = a + (pos_t)((u32)id - cb_off[k] + 1) * CH;
}
__global__ void k_gap_segs(seg_tab S, u32 CH, const u32* __restrict__ seg_off, u32 nseg) {
    const u64 id = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (id >= nseg) return;
    const u32 k = item_gap(seg_off, S.m, (u32)id);
    pos_t a, b;
    gap_in(S.P, k, S.segoff, S.N, a, b);
    const pos_t x = a + (pos_t)((u32)id - seg_off[k]) * CH;
    S.sin[id] = seg_in{x, k, x, S.zmask0, upper_cb(S, x)};
    S.valid[id] = 0;
    S.succ[id] = NONE;
    S.seg_at[x - S.segoff] = (u32)id;
}
// bitmaps over text positions (bit q of word q >> 5)
__device__ __forceinline__ void bm_set_range(u32* bm, pos_t a, pos_t b) {  // [a, b)
    while (a < b) {
        const u64 w = a >> 5;
        const u32 lo = a & 31, hi = (u32)min<u64>(32u, lo + (u64)(b - a));
        const u32 mask = (hi == 32 ? 0xFFFFFFFFu : ((1u << hi) - 1)) & ~((1u << lo) - 1);
        atomicOr(&bm[w], mask);
        a += hi - lo;
    }
}
// one wave sets [a, b): lanes stride over the 32-bit words
__device__ __forceinline__ void bm_set_range_wave(u32* bm, pos_t a, pos_t b, u32 lane) {
    if (a >= b) return;
    const u64 w0 = a >> 5, w1 = (b - 1) >> 5;
    for (u64 w = w0 + lane; w <= w1; w += 64) {
        u32 mask = 0xFFFFFFFFu;
        if (w == w0) mask &= ~((1u << (a & 31)) - 1);
        if (w == w1 && (b & 31)) mask &= (1u << (b & 31)) - 1;
        atomicOr(&bm[w], mask);
    }
}
// I_0 and the base superset over the window [lo, hi) (relative to off): every gap
// [a_k, b_k) plus its LPF-start query position b_k, and the interiors of phrases of at
// most 48 bytes.  The gap parts are set per default segment (one wave each: at most 2 CH
// positions), the rest per phrase (one thread: at most 48 positions)
__global__ void k_gap_bitmaps(seg_tab S, u32 nseg, pos_t N, pos_t nt, pos_t hi, pos_t off, u32* __restrict__ bmI,
                              u32* __restrict__ bmSup) {
    const u32 lane = threadIdx.x & 63;
    for (u64 id = gtid() >> 6; id < nseg; id += gstride() >> 6) {  // one wave per segment (grid-stride)
    // the segment table (k_gap_segs) holds each segment's start and gap; a segment ends
    // where the next one of its gap starts, the last one at the (clipped) gap end
    const seg_in g = S.sin[id];
    const u32 k = g.p;
    pos_t a, b;
    gap_in(S.P, k, S.segoff, S.N, a, b);
    const pos_t x0 = g.start;
    const bool more = id + 1 < nseg && S.sin[id + 1].p == k;
    const pos_t x1 = min(more ? S.sin[id + 1].start : b, min(min(N, nt), hi));
    if (x0 < x1) {
        bm_set_range_wave(bmI, x0 - off, x1 - off, lane);
        bm_set_range_wave(bmSup, x0 - off, x1 - off, lane);
    }
    }
}
__global__ void k_gap_bitmaps_phr(const pos_t* __restrict__ P, u32 m, pos_t N, pos_t nt, pos_t lo, pos_t hi, pos_t off,
                                  u32* __restrict__ bmI, u32* __restrict__ bmSup) {
    const u64 k = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (k > m) return;
    pos_t a, b;
    gap_of(P, (u32)k, a, b);
    if (a < b && b >= lo && b < min(min(N, nt), hi)) {  // the query position past the gap
        const pos_t q = b - off;
        atomicOr(&bmI[q >> 5], 1u << (q & 31));
        atomicOr(&bmSup[q >> 5], 1u << (q & 31));
    }
    if (k < m) {
        const pos_t pb = max(P[3 * k], lo), pe = min(min(P[3 * k + 1], nt), hi);
        if (P[3 * k + 1] - P[3 * k] <= 48 && pb < pe) bm_set_range(bmSup, pb - off, pe - off);
    }
}
__global__ void k_bm_xor(const u32* __restrict__ a, const u32* __restrict__ b, u64 nw, u32* __restrict__ x) {
    const u64 w = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (w < nw) x[w] = a[w] ^ b[w];
}
__global__ void k_bm_andnot(const u32* __restrict__ a, const u32* __restrict__ b, u64 nw, u32* __restrict__ x) {
    const u64 w = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (w < nw) x[w] = a[w] & ~b[w];
}
__global__ void k_bm_or(const u32* __restrict__ a, const u32* __restrict__ b, u64 nw, u32* __restrict__ x) {
    const u64 w = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (w < nw) x[w] = a[w] | b[w];
}
// Bitmap -> positions lists without per-word count arrays: a block of 256 lanes owns
// BMB = 2048 words (8 per lane); pass 1 writes per-block counts of the marked bits
// (two masks packed in one u64: hi = mask A, lo = mask B), one scan over the ~nw/2048
// block counts gives every block its offsets, pass 2 recomputes the lane counts, scans
// them in LDS and writes the positions in order.  Replaces two full-length (nw) count
// arrays and their device-wide scans.
constexpr u32 BMB_T = 256, BMB_W = 8, BMB = BMB_T * BMB_W;
// masks of word w: runs (A = run starts, B = run ends) or set bits (A = a & ~b, B unused)
struct bm_runs {
    const u32* bm;
    __device__ __forceinline__ void masks(u64 w, u32& a, u32& b) const {
        const u32 x = bm[w], prev = w ? (bm[w - 1] >> 31) : 0u;
        const u32 sh = (x << 1) | prev;
        a = x & ~sh;
        b = ~x & sh;
    }
};
struct bm_bits {
    const u32* bm;
    const u32* notbm;  // optional: bits of bm not in notbm
    __device__ __forceinline__ void masks(u64 w, u32& a, u32& b) const {
        a = bm[w] & (notbm ? ~notbm[w] : ~0u);
        b = 0;
    }
};
template <class M>
__global__ __launch_bounds__(BMB_T) void k_bmb_count(M mk, u64 nw, u64* __restrict__ bsum) {
    __shared__ u64 red[BMB_T / 64];
    const u64 w0 = (u64)blockIdx.x * BMB + threadIdx.x;
    u32 ca = 0, cb = 0;
#pragma unroll
    for (u32 r = 0; r < BMB_W; r++) {
        const u64 w = w0 + (u64)r * BMB_T;
        if (w < nw) {
            u32 a, b;
            mk.masks(w, a, b);
            ca += __popc(a);
            cb += __popc(b);
        }
    }
    u64 v = ((u64)ca << 32) | cb;
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0) bsum[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}
// pass 2, coalesced: in round r lane l owns word w0 + 256 r + l; the lanes' counts of
// a round are scanned across the block (wave scan + 4 wave totals in LDS), so the
// outputs stay in word order
template <class M, class OUT>
__global__ __launch_bounds__(BMB_T) void k_bmb_write(M mk, u64 nw, const u64* __restrict__ bincl, OUT out, pos_t off) {
    __shared__ u64 wsum[BMB_T / 64];
    const u32 l = threadIdx.x, lane = l & 63, wv = l >> 6;
    u64 base = blockIdx.x ? bincl[blockIdx.x - 1] : 0ull;
    // a block without marked bits writes nothing (uniform exit; sparse bitmaps of
    // repetitive text skip almost every block instead of 8 scan rounds each)
    if (bincl[blockIdx.x] == base) return;
    for (u32 r = 0; r < BMB_W; r++) {
        const u64 w = (u64)blockIdx.x * BMB + (u64)r * BMB_T + l;
        u32 a = 0, b = 0;
        if (w < nw) mk.masks(w, a, b);
        const u64 mine = ((u64)__popc(a) << 32) | __popc(b);
        u64 inc = mine;  // inclusive wave scan
        for (u32 d = 1; d < 64; d <<= 1) {
            const u64 v = __shfl_up(inc, d);
            if (lane >= d) inc += v;
        }
        if (lane == 63) wsum[wv] = inc;
        __syncthreads();
        u64 pre = 0, tot = 0;
#pragma unroll
        for (u32 k = 0; k < BMB_T / 64; k++) {
            const u64 x = wsum[k];
            if (k < wv) pre += x;
            tot += x;
        }
        const u64 o = base + pre + inc - mine;
        u32 oa = (u32)(o >> 32), ob = (u32)o;
        while (a) { out.a(oa++, off + (pos_t)(32 * w + __builtin_ctz(a)), w); a &= a - 1; }
        while (b) { out.b(ob++, off + (pos_t)(32 * w + __builtin_ctz(b))); b &= b - 1; }
        base += tot;
        __syncthreads();  // wsum reused by the next round
    }
}
struct out_runs {
    pos_t* st;
    pos_t* en;
    __device__ __forceinline__ void a(u32 o, pos_t p, u64) const { st[o] = p; }
    __device__ __forceinline__ void b(u32 o, pos_t p) const { en[o] = p; }
};
struct out_list {  // positions + a flag bit from a second bitmap
    pos_t* pos;
    u8* flag;
    const u32* flagbm;
    __device__ __forceinline__ void a(u32 o, pos_t p, u64 w) const {
        pos[o] = p;
        if (flag) flag[o] = (flagbm[w] >> (p & 31)) & 1;  // offsets are multiples of 32
    }
    __device__ __forceinline__ void b(u32, pos_t) const {}
};
// totals of the two masks; bincl holds the inclusive block scan afterwards
template <class M>
static u64 bmb_scan(M mk, u64 nw, dbuf<u64>& bs, dbuf<u64>& bi, dbuf<u8>& tmp, hipStream_t st) {
    const u64 nblk = std::max<u64>(1, (nw + BMB - 1) / BMB);
    u64* s = bs.get(nblk);
    u64* incl = bi.get(nblk);
    k_bmb_count<<<(unsigned)nblk, BMB_T, 0, st>>>(mk, nw, s);
    size_t tb = 0;
    LZ_HIP(hipcub::DeviceScan::InclusiveSum(nullptr, tb, s, incl, (int)nblk, st));
    u8* t = tmp.get(tb);
    LZ_HIP(hipcub::DeviceScan::InclusiveSum(t, tb, s, incl, (int)nblk, st));
    return rd1(incl + nblk - 1, st);
}
// intervals -> chunks of <= ch positions with ranks (rank0 = exclusive scan of
// lengths).  Short chunks keep k_slots (one thread per chunk, a direct
// fingerprint of <= 64 bytes per pattern, then rolls) wide on the device: the
// chunk length is 128, or 32 when that leaves fewer than ~2^18 chunks.
constexpr u32 SLOT_CHUNK_LONG = 128, SLOT_CHUNK_SHORT = 32;
__global__ void k_iv_chunk_counts(const pos_t* __restrict__ st, const pos_t* __restrict__ en, u32 ni, u32* __restrict__ nch,
                                  u32* __restrict__ nch_short, u32* __restrict__ len, u32 short_len) {
    const u64 k = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= ni) return;
    const u32 l = (u32)(en[k] - st[k]);  // intervals hold < 2^32 / 5 positions (entry ids are 32-bit)
    len[k] = l;
    nch[k] = (l + SLOT_CHUNK_LONG - 1) / SLOT_CHUNK_LONG;
    nch_short[k] = (l + short_len - 1) / short_len;
}
// one thread per chunk; its interval by binary search over the chunk offsets
__global__ void k_iv_chunks(const pos_t* __restrict__ st, const pos_t* __restrict__ en, u32 ni, const u32* __restrict__ choff,
                            u32 nch, u32 chl, const u32* __restrict__ rank, ichunk* __restrict__ ch) {
    const u64 c = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= nch) return;
    u32 lo = 0, hi = ni;  // last k with choff[k] <= c (every interval has >= 1 chunk)
    while (hi - lo > 1) {
        const u32 mid = (lo + hi) >> 1;
        if (choff[mid] <= c) lo = mid; else hi = mid;
    }
    const pos_t q = st[lo] + (pos_t)(c - choff[lo]) * chl;
    ch[c] = ichunk{q, min(en[lo], (pos_t)(q + chl)), rank[lo] + (u32)(q - st[lo])};
}
// rem[r] = base position r not in I
__global__ void k_rem_from_bm(const pos_t* __restrict__ ipos, u64 nb, const u32* __restrict__ bmI, pos_t off,
                              u8* __restrict__ rem, pos_t* __restrict__ iposr) {
    const u64 r = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= nb) return;
    const pos_t p = ipos[r], q = p - off;
    const bool in = (bmI[q >> 5] >> (q & 31)) & 1;
    rem[r] = in ? 0 : 1;
    if (iposr) iposr[r] = p | (in ? (pos_t)0 : POS_RFLAG);
}

// walks over a list of segment ids (outputs in the table; WRITE: factors at offs)
// waves per SIMD the walk kernel is compiled for (its loads are dependent chains:
// occupancy hides their latency; fewer registers cost a few spilled bytes)
#ifndef LZ_WALK_WAVES
#define LZ_WALK_WAVES 8
#endif
template <bool WRITE>
__global__ __launch_bounds__(64, LZ_WALK_WAVES) void k_walk(walk_ctx W, seg_tab S, const u32* __restrict__ ids, u32 cnt, const u64* __restrict__ offs,
                       pos_t* __restrict__ fact) {
    const u64 t = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= cnt) return;
    const u32 g = ids[t];
    seg_out* og = WRITE ? nullptr : S.sout + g;
    if (WRITE && S.stash) {
        // the segment's last walk is exact for the final insert set: copy its stashed factors
        const u32 nf = S.sout[g].nfact;
        if (nf <= STASH_CAP && !(S.sout[g].flags & SEG_NO_STASH)) {
            const pos_t* src = S.stash + (u64)g * 2 * STASH_CAP;
            pos_t* dst = fact + 2 * offs[t];
            for (u32 k = 0; k < 2 * nf; k++) dst[k] = src[k];
            return;
        }
    }
    walk_segment<WRITE>(W, S.sin[g], og, WRITE ? fact + 2 * offs[t] : (S.stash ? S.stash + (u64)g * 2 * STASH_CAP : nullptr));
    if (!WRITE) {
        const u32 fl = og->flags;
        if (fl & 2) atomicOr(S.err, 2u);
        if (fl & 4) atomicOr(S.err, 4u);
        S.valid[g] = 1;
        S.succ[g] = NONE;
    }
}
// expected walk length of a segment (its first gap stretch), to group similar walks in a wave
__global__ void k_walk_keys(seg_tab S, const u32* __restrict__ ids, u32 cnt, u32* __restrict__ keys) {
    const u64 t = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= cnt) return;
    const seg_in si = S.sin[ids[t]];
    const pos_t ge = min(S.P[3 * si.p], si.lim);
    keys[t] = ge > si.start ? (u32)min<u64>(ge - si.start, 0xFFFFFFFFull) : 0u;
}
__global__ void k_todo(seg_tab S, u32 nseg, u32* __restrict__ ids, u32* __restrict__ cnt) {
    const u64 g = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    const bool todo = g < nseg && !S.valid[g];
    const u32 slot = block_count_claim(cnt, todo);
    if (todo) ids[slot] = (u32)g;
}
// claim the segment starting at x (created by this thread iff *mine)
__device__ u32 seg_claim(const seg_tab& S, pos_t x, bool& mine) {
    mine = false;
    const u32 old = atomicCAS(&S.seg_at[x - S.segoff], NONE, PENDING);
    if (old != NONE) return old;
    const u32 id = atomicAdd(S.nseg, 1u);
    if (id >= S.cap) {
        atomicOr(S.err, 1u);
        atomicExch(&S.seg_at[x - S.segoff], NONE);
        return NONE;
    }
    mine = true;
    return id;
}
// link every valid segment to the segment starting at its next state; unknown
// next states become alias segments (the real chain enters a valid chunk walk
// at one of its recorded factor starts) or fresh segments to walk
__global__ void k_link(seg_tab S, u32 nseg) {
    const u64 g = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= nseg || !S.valid[g] || S.succ[g] != NONE) return;
    const seg_out& o = S.sout[g];
    if ((o.flags & 1) || o.next >= S.N) return;
    const pos_t x = o.next;
    const u32 s = S.seg_at[x - S.segoff];
    if (s == PENDING) return;
    if (s != NONE) { S.succ[g] = s; return; }
    // alias into the chunk walk that covers x?
    u32 src = NONE, k_at = 0;
    {
        u32 lo = 0, hi = S.ncb;  // last boundary <= x
        while (lo < hi) {
            const u32 mid = (lo + hi) >> 1;
            if (S.cbv[mid] <= x) lo = mid + 1; else hi = mid;
        }
        if (lo > 0 && S.cbv[lo - 1] < x) {
            const u32 gc = S.seg_at[S.cbv[lo - 1] - S.segoff];
            if (gc < S.cap) {
                if (!S.valid[gc]) return;  // the chunk walk is stale: walked next round, link again
                const seg_out& oc = S.sout[gc];
                for (u32 k = 1; k < oc.nbnd; k++)
                    if (oc.bnd[k] == x) { src = gc; k_at = k; break; }
            }
        }
    }
    bool mine;
    const u32 id = seg_claim(S, x, mine);
    if (!mine) return;  // another thread creates it; resolved by the next link pass
    S.sin[id] = make_seg_in(S, x);
    S.succ[id] = NONE;
    if (src != NONE) {
        seg_out oa = S.sout[src];
        const u32 nf_src = oa.nfact;
        oa.nfact -= k_at;
        oa.nbnd = 0;
        if (S.stash) {
            // the alias's factors are the chunk walk's from factor k_at on: copy them when the
            // chunk walk kept all of its factors, else the final emission walks the alias
            if (nf_src <= STASH_CAP) {
                const pos_t* a = S.stash + (u64)src * 2 * STASH_CAP + 2 * k_at;
                pos_t* d = S.stash + (u64)id * 2 * STASH_CAP;
                for (u32 k = 0; k < 2 * oa.nfact; k++) d[k] = a[k];
            } else {
                oa.flags |= SEG_NO_STASH;
            }
        }
        S.sout[id] = oa;
        S.valid[id] = 1;
    } else {
        S.valid[id] = 0;
    }
    __threadfence();
    atomicExch(&S.seg_at[x - S.segoff], id);
    S.succ[g] = id;
}
// sparse reset of the position -> segment map (every entry set was a segment start)
__global__ void k_seg_at_clear(seg_tab S, u32 nseg) {
    const u64 g = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (g < nseg) S.seg_at[S.sin[g].start - S.segoff] = NONE;
}
// pointer doubling along succ: J = terminal-or-successor, D = hops
__global__ void k_jump0(seg_tab S, u32 nseg, u32* __restrict__ J, u32* __restrict__ D) {
    const u64 g = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= nseg) return;
    bool term = !S.valid[g] || S.succ[g] >= S.cap;
    if (!term) {
        const seg_out& o = S.sout[g];
        term = (o.flags & 1) || o.next >= S.N;
    }
    J[g] = term ? (u32)g : S.succ[g];
    D[g] = term ? 0 : 1;
}
__global__ void k_jumpk(const u32* __restrict__ J, const u32* __restrict__ D, u32 nseg, u32* __restrict__ J2,
                        u32* __restrict__ D2) {
    const u64 g = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= nseg) return;
    const u32 j = J[g];
    J2[g] = J[j];
    D2[g] = D[g] + D[j];
}
// two doubling levels per launch: J1 = J o J, J2 = J1 o J1, D2 = D + D o J + D o J1 + D o J o J1
__global__ void k_jumpk2(const u32* __restrict__ J, const u32* __restrict__ D, u32 nseg, u32* __restrict__ J1,
                         u32* __restrict__ J2, u32* __restrict__ D2) {
    const u64 g = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= nseg) return;
    const u32 a = J[g], b = J[a], c = J[b], d = J[c];
    J1[g] = b;
    J2[g] = d;
    D2[g] = D[g] + D[a] + D[b] + D[c];
}
struct chain_status { u32 term, hops, valid, flags; pos_t next; u32 err, nseg; };
__global__ void k_chain_status(seg_tab S, const u32* __restrict__ J, const u32* __restrict__ D, u32 c0,
                               chain_status* out) {
    const u32 t = J[c0];
    chain_status c{};
    c.term = t;
    c.hops = D[c0];
    c.valid = S.valid[t];
    c.flags = S.sout[t].flags;
    c.next = S.sout[t].next;
    c.err = *S.err;
    c.nseg = *S.nseg;
    *out = c;
}
// chain[k] = k-th successor of segment 0 (binary lifting over the stored levels)
struct jump_levels { const u32* J[MAX_LV]; u32 nlv; };
__global__ void k_chain_expand(jump_levels JL, u32 len, u32 c0, u32* __restrict__ chain) {
    const u64 k = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= len) return;
    u32 g = c0;
    for (u32 l = 0; l < JL.nlv; l++)
        if ((k >> l) & 1) g = JL.J[l][g];
    chain[k] = g;
}
// I' bitmap: what the chain inserted below nt ([start, e) + LPF-start queries)
// (clipped to the window's bitmap range [off, hi), hi <= nt)
// the range words [w0, w1] of chain node g ([start, min(e, hi)) relative to off) and the masks of its
// end words
__device__ __forceinline__ bool chain_range(const seg_tab& S, u32 g, pos_t hi, pos_t off, pos_t& x0, pos_t& x1) {
    const pos_t a = S.sin[g].start, b = min(S.sout[g].e, hi);
    x0 = a - off;
    x1 = b - off;
    return a < b;
}
__device__ __forceinline__ u32 range_mask(u64 w, pos_t x0, pos_t x1) {
    const u64 w0 = x0 >> 5, w1 = (x1 - 1) >> 5;
    u32 mask = 0xFFFFFFFFu;
    if (w == w0) mask &= ~((1u << (x0 & 31)) - 1);
    if (w == w1 && (x1 & 31)) mask &= (1u << (x1 & 31)) - 1;
    return mask;
}
// one wave per chain node: its gap walk range and single inserts into bm; a node whose range is
// longer than long_words (0: none) is appended to `lng` (count lng[0], ranges from lng + 2) for
// k_chain_inserts_long.  outside: inserted positions not in bmI (duplicates only add: 0 iff none)
__global__ void k_chain_inserts(seg_tab S, const u32* __restrict__ chain, u32 cnt, pos_t hi, pos_t off,
                                u32* __restrict__ bm, const u32* __restrict__ bmI = nullptr, u32* __restrict__ outside = nullptr,
                                u32 long_words = 0, u32* __restrict__ lng = nullptr, u32 lng_cap = 0) {
    const u32 lane = threadIdx.x & 63;
    u32 c = 0;
    for (u64 k = gtid() >> 6; k < cnt; k += gstride() >> 6) {  // one wave per chain node (grid-stride)
        const u32 g = chain[k];
        const seg_out& o = S.sout[g];
        pos_t x0, x1;
        if (chain_range(S, g, hi, off, x0, x1)) {
            const u64 w0 = x0 >> 5, w1 = (x1 - 1) >> 5;
            bool here = true;
            if (long_words && w1 - w0 >= long_words) {
                // the overflow decision comes from lane 0's own atomic result: a plain load of
                // lng[1] may hit a stale L1 line while the atomics are performed in L2
                u32 ovf = 0;
                if (lane == 0) {
                    const u32 slot = atomicAdd(lng, 1u);
                    if (slot < lng_cap) {
                        ((u64*)(lng + 2))[2 * slot] = x0;
                        ((u64*)(lng + 2))[2 * slot + 1] = x1;
                    } else {
                        ovf = 1;
                        atomicOr(lng + 1, 1u);  // list full: handled here (lng[1] for the host / debug)
                    }
                }
                here = __shfl(ovf, 0, 64) != 0;
            }
            if (here) {
                // loads first, atomics after: an atomic without return still counts against the
                // load counter, so a load behind it would wait for its round trip
                if (outside)
                    for (u64 w = w0 + lane; w <= w1; w += 64) c += __popc(range_mask(w, x0, x1) & ~bmI[w]);
                for (u64 w = w0 + lane; w <= w1; w += 64) atomicOr(&bm[w], range_mask(w, x0, x1));
            }
        }
        if (lane < o.nsingle && lane < 4 && o.single[lane] < hi) {
            const pos_t r = o.single[lane] - off;
            if (outside) c += ((bmI[r >> 5] >> (r & 31)) & 1) ? 0u : 1u;
            atomicOr(&bm[r >> 5], 1u << (r & 31));
        }
    }
    if (outside) {
        for (int o2 = 32; o2 > 0; o2 >>= 1) c += __shfl_down(c, o2, 64);
        if (lane == 0 && c) atomicAdd(outside, c);
    }
}
// the listed long ranges, every thread of the grid on each
__global__ void k_chain_inserts_long(const u32* __restrict__ lng, u32 lng_cap, u32* __restrict__ bm, const u32* __restrict__ bmI,
                                     u32* __restrict__ outside) {
    u32 c = 0;
    const u32 nl = min(lng[0], lng_cap);
    for (u32 k = 0; k < nl; k++) {
        const pos_t x0 = (pos_t)((const u64*)(lng + 2))[2 * k], x1 = (pos_t)((const u64*)(lng + 2))[2 * k + 1];
        const u64 w0 = x0 >> 5, w1 = (x1 - 1) >> 5;
        for (u64 w = w0 + gtid(); w <= w1; w += gstride()) {
            const u32 mask = range_mask(w, x0, x1);
            if (outside) c += __popc(mask & ~bmI[w]);
            atomicOr(&bm[w], mask);
        }
    }
    if (outside) block_add(outside, c);
}
// I within I': base ranks in I (rem = 0) whose position the chain did not insert -> *missing
__global__ void k_subset_check(const pos_t* __restrict__ ipos, const u8* __restrict__ rem, u64 nb, const u32* __restrict__ bm2,
                               pos_t off, u32* __restrict__ missing) {
    const u64 r = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    bool miss = false;
    if (r < nb && !rem[r]) {
        const pos_t q = ipos[r] - off;
        miss = !((bm2[q >> 5] >> (q & 31)) & 1);
    }
    if (__any(miss) && (threadIdx.x & 63) == __ffsll((unsigned long long)__ballot(miss)) - 1) atomicAdd(missing, 1u);
}
// the window's entry segment: the exact chain state handed over by the previous window
// (a default segment starting there takes it over); *c0 = its id
__global__ void k_entry_seg(seg_tab S, pos_t start, pos_t idxpos, u32 zmask, u32* __restrict__ c0,
                            seg_in* __restrict__ entry_out) {
    u32 g = S.seg_at[start - S.segoff];
    if (g == NONE) {
        g = atomicAdd(S.nseg, 1u);
        S.seg_at[start - S.segoff] = g;
    }
    seg_in in = make_seg_in(S, start);
    in.idxpos = idxpos;
    in.zmask = zmask;
    S.sin[g] = in;
    S.valid[g] = 0;
    S.succ[g] = NONE;
    *c0 = g;
    *entry_out = in;
}
// window exit: the chain's last segment stopped at a start >= the window end
__global__ void k_exit_state(seg_tab S, u32 term, seg_in* __restrict__ out) {
    const seg_out& o = S.sout[term];
    seg_in x{};
    x.start = o.next;
    x.idxpos = o.idxpos;
    x.zmask = o.zmask;
    *out = x;
}
// carried table (pos + 1, 0 = none): every insert of the window's chain, for the next window
__global__ void k_h_export(const u8* __restrict__ T, gap_cfg G, seg_tab S, const u32* __restrict__ chain, u32 cnt,
                           pos_t* __restrict__ Hs) {
    const u32 lane = threadIdx.x & 63;
    auto put = [&](pos_t q) {
        for (int x = 0; x < 5; x++)
            atomic_max_pos(&Hs[(u32)((u64)kr_direct(T, q, G.lens[x], G.base[x]) & G.mask)], q + 1);
    };
    for (u64 k = gtid() >> 6; k < cnt; k += gstride() >> 6) {  // one wave per chain node (grid-stride)
        const u32 g = chain[k];
        const seg_out& o = S.sout[g];
        const pos_t a = S.sin[g].start;
        for (pos_t q = a + lane; q < o.e; q += 64) put(q);
        if (lane < o.nsingle && lane < 4) put(o.single[lane]);
    }
}
// the lead-in table of a speculative block: the speculated insert set of
// [0, upto) -- every gap position and the query position past each gap, as the first
// speculation of the one-GPU engine -- as the last insert per slot (pos + 1)
constexpr u32 SEED_CH = 128;
__global__ void k_seed_counts(const pos_t* __restrict__ P, u32 m, pos_t upto, u32* __restrict__ cnt) {
    const u64 k = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (k > m) return;
    pos_t a, b;
    gap_of(P, (u32)k, a, b);
    b = min(b, upto);
    cnt[k] = b > a ? (u32)((b - a + SEED_CH - 1) / SEED_CH) : 0u;
}
__global__ void k_seed_slots(const u8* __restrict__ T, gap_cfg G, const pos_t* __restrict__ P, u32 m, pos_t upto,
                             const u32* __restrict__ off, u32 nch, pos_t* __restrict__ Hs) {
    const u64 t = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= 5ull * nch) return;
    const u32 c = (u32)(t / 5);
    const int x = (int)(t - 5ull * c);
    u32 lo = 0, hi = m + 1;  // the gap holding chunk c: last k with off[k] <= c
    while (hi - lo > 1) {
        const u32 mid = (lo + hi) >> 1;
        if (off[mid] <= c) lo = mid; else hi = mid;
    }
    pos_t a, b;
    gap_of(P, lo, a, b);
    b = min(b, upto);
    const pos_t q0 = a + (pos_t)(c - off[lo]) * SEED_CH, q1 = min(b, q0 + SEED_CH);
    const u32 len = G.lens[x];
    const u64 base = G.base[x];
    const u128* np = G.negpow + x * 256;
    u128 fp = kr_direct(T, q0, len, base);
    for (pos_t q = q0; q < q1; q++) {
        if ((u64)q + len < (u64)G.n) atomic_max_pos(&Hs[(u32)((u64)fp & G.mask)], q + 1);
        if (q + 1 < q1) fp = kr_roll(fp, base, np[T[q]], T[q + len]);
    }
}
__global__ void k_seed_queries(const u8* __restrict__ T, gap_cfg G, const pos_t* __restrict__ P, u32 m, pos_t upto,
                               pos_t* __restrict__ Hs) {
    const u64 t = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= 5ull * (m + 1)) return;
    const u32 k = (u32)(t / 5);
    const int x = (int)(t - 5ull * k);
    pos_t a, b;
    gap_of(P, k, a, b);
    if (a < b && b < upto && (u64)b + G.lens[x] < (u64)G.n)
        atomic_max_pos(&Hs[(u32)((u64)kr_direct(T, b, G.lens[x], G.base[x]) & G.mask)], b + 1);
}
// speculative blocks: bad[0] = the first part whose lookups used a slot where the
// speculated entry table and the true one differ (atomicMin; starts at the number of parts)
__global__ void k_spec_check(const u32* __restrict__ used, int parts, u64 nw, const pos_t* __restrict__ spec,
                             const pos_t* __restrict__ tru, u64 nslots, u32* __restrict__ bad) {
    const u64 k = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= nslots) return;
    const bool differs = spec[k] != tru[k];
    bool any = false;
    for (int p = 0; p < parts; ++p)
        if ((used[(u64)p * nw + (k >> 5)] >> (k & 31)) & 1u) {
            if (differs) atomicMin(bad, (u32)p);
            any = true;
            break;
        }
    if (any && bad[1] != 0xFFFFFFFFu) {  // debug counters (bad[1] = ~0: off): used slots, differing ones
        atomicAdd(bad + 1, 1u);
        if (differs) {
            atomicAdd(bad + 2, 1u);
            const u32 x = atomicAdd(bad + 3, 1u);  // up to 8 examples (slot, speculated, true) from bad + 4
            if (x < 8) {
                u64* ex = (u64*)(bad + 4) + 3 * x;
                ex[0] = k;
                ex[1] = (u64)spec[k];
                ex[2] = (u64)tru[k];
            }
        }
    }
}
// the carried table for the rest: the speculative block's writes (values > its start) over the true table
__global__ void k_spec_merge(pos_t* __restrict__ Hs, const pos_t* __restrict__ tru, u64 nslots, pos_t blk_start) {
    const u64 k = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= nslots) return;
    const pos_t h = Hs[k];
    if (!(h != 0 && h - 1 >= blk_start)) Hs[k] = tru[k];
}
// completion start: the last chain node whose start is <= y0 (the first position where
// the speculated insert set and the chain's differ): every lookup of its predecessors
// happened below y0, so its start state is exact (index state from its predecessor)
struct chain_cut { u32 k, pad; seg_in in; };
__global__ void k_chain_cut(seg_tab S, const u32* __restrict__ chain, u32 nall, const u64* __restrict__ y0p,
                            seg_in entry, chain_cut* __restrict__ out) {
    const u64 y0 = *y0p;
    chain_cut c{};
    if (nall == 0 || y0 <= entry.start) {
        c.k = 0;
        c.in = entry;
        *out = c;
        return;
    }
    u32 lo = 0, hi = nall;  // first k with start > y0
    while (lo < hi) {
        const u32 mid = (lo + hi) >> 1;
        if (S.sin[chain[mid]].start <= y0) lo = mid + 1; else hi = mid;
    }
    c.k = lo - 1;  // chain[0] starts at the window entry <= y0
    c.in = S.sin[chain[c.k]];
    if (c.k > 0) {
        const seg_out& pv = S.sout[chain[c.k - 1]];
        c.in.idxpos = pv.idxpos;
        c.in.zmask = pv.zmask;
    } else {
        c.in = entry;
    }
    *out = c;
}
__global__ void k_set_pairs(const pos_t* __restrict__ pairs, u32 np, pos_t off, u32* __restrict__ bm,
                            const u32* __restrict__ bmI = nullptr, u32* __restrict__ outside = nullptr) {
    const u64 k = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (k < np && pairs[2 * k] >= off) {
        pos_t a = pairs[2 * k] - off;
        const pos_t b = pairs[2 * k + 1] - off;
        u32 c = 0;
        while (a < b) {
            const u64 w = a >> 5;
            const u32 lo = a & 31, hi = (u32)min<u64>(32u, lo + (u64)(b - a));
            const u32 mask = (hi == 32 ? 0xFFFFFFFFu : ((1u << hi) - 1)) & ~((1u << lo) - 1);
            atomicOr(&bm[w], mask);
            if (outside) c += __popc(mask & ~bmI[w]);
            a += hi - lo;
        }
        if (outside && c) atomicAdd(outside, c);
    }
}
__global__ void k_chain_nfact(seg_tab S, const u32* __restrict__ chain, u32 cnt, u64* __restrict__ nf) {
    const u64 k = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (k < cnt) nf[k] = S.sout[chain[k]].nfact;
}
// a walked segment is stale iff a dirty position lies in its covered range
__global__ void k_stale(seg_tab S, u32 nseg, const pos_t* __restrict__ dirty, u64 nd) {
    const u64 g = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= nseg || !S.valid[g]) return;
    const seg_out& o = S.sout[g];
    const pos_t a = S.sin[g].start, b = (o.flags & 1) ? S.N : max(o.next, (pos_t)(o.e + 1));
    u64 l = 0, h = nd;
    while (l < h) {
        const u64 mid = (l + h) >> 1;
        if (dirty[mid] < a) l = mid + 1; else h = mid;
    }
    if (l < nd && dirty[l] <= b) {
        S.valid[g] = 0;
        S.succ[g] = NONE;
    }
}
// segments whose cached successor became invalid keep the id (the table entry is re-walked in place)
__global__ void k_invalidate_all(seg_tab S, u32 nseg) {
    const u64 g = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= nseg) return;
    S.valid[g] = 0;
    S.succ[g] = NONE;
}

__global__ void k_set_u32x2(u32* p, u32 a, u32 b) {
    p[0] = a;
    p[1] = b;
}
__global__ void k_put3(pos_t* p, pos_t a, pos_t b, pos_t c) {
    p[0] = a;
    p[1] = b;
    p[2] = c;
}
__global__ void k_sum_u8(const u8* __restrict__ f, u64 m, u32* __restrict__ acc) {
    const u64 k = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    block_add(acc, k < m && !f[k] ? 1u : 0u);
}
// exclusive scan of cnt[0..m) into off[0..m] (off[m] = total); cnt needs m+1 entries
template <class T>
static void excl_scan_nr(T* cnt, T* off, u64 m, dbuf<u8>& tmp, hipStream_t st) {  // total left at off[m]
    excl_sum_total(cnt, off, m, tmp, st);  // (include/prim.h: one launch up to 64 Ki items)
}
template <class T>
static T excl_scan(T* cnt, T* off, u64 m, dbuf<u8>& tmp, hipStream_t st) {
    excl_scan_nr(cnt, off, m, tmp, st);
    return rd1(off + m, st);
}

// LZ77SSS_LSD_CHECK: first index where two u32 arrays differ (atomic min), and the count
__global__ void k_first_diff_u32(const u32* __restrict__ a, const u32* __restrict__ b, u64 m, u64* __restrict__ out) {
    const u64 t = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (t < m && a[t] != b[t]) {
        atomicMin((unsigned long long*)&out[0], (unsigned long long)t);
        atomicAdd((unsigned long long*)&out[1], 1ull);
    }
}
// ---------------------------------------------------------------------------
// LSD radix sort of the base entries (key = slot or dense slot id, value = entry id) by
// reduce-then-scan: per digit a histogram pass over the tiles of its input, a
// scan, a scatter pass.  A tile is block-sorted in LDS on its digit and leaves as
// contiguous runs per digit (coalesced); pass 0 reads the raw slots (the dense-id map is
// applied on the fly: no separate key array), the last pass writes only the entry ids plus
// the first sorted index of every key (atomic min per key and tile).  Against rocprim's
// onesweep on the dense rr keys (a dense-key pass, two passes writing keys and ids, a
// predecessor/head pass): 32 instead of about 52 bytes per entry moved.
constexpr u32 LS_T = 256, LS_IPT = 8, LS_TILE = LS_T * LS_IPT, LS_DB = 7, LS_NB = 1u << LS_DB, LS_MAXP = 5;
struct ls_dense {  // pass-0 key of entry e: the dense id of its slot
    const u32* keys;
    const u64* pbw;  // per presence word: rank of its first slot << 32 | the word (one load per key)
    __device__ __forceinline__ u32 operator()(u64 e) const {
        const u32 k = keys[e];
        const u64 w = pbw[k >> 5];
        return (u32)(w >> 32) + __popc((u32)w & ((1u << (k & 31)) - 1u));
    }
};
__global__ void k_pack_pbw(const u32* __restrict__ pbm, const u32* __restrict__ pwp, u64 nw, u64* __restrict__ pbw) {
    const u64 w = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (w < nw) pbw[w] = ((u64)pwp[w] << 32) | pbm[w];
}
struct ls_plain {
    const u32* keys;
    __device__ __forceinline__ u32 operator()(u64 e) const { return keys[e]; }
};
// h[d] += number of lanes of the wave holding digit d: one LDS atomic per distinct digit of the
// wave (the same-address atomics of a hot digit otherwise serialize lane by lane: rr's dense keys
// are few per tile, 176 us per histogram pass)
__device__ __forceinline__ void wave_agg_add(u32* h, u32 d, bool valid) {
    const u32 lane = threadIdx.x & 63;
    u64 todo = __ballot(valid);
    while (todo) {
        const int leader = __ffsll((long long)todo) - 1;
        const u32 dl = __shfl(d, leader, 64);
        const u64 same = __ballot(valid && d == dl);
        if (lane == (u32)leader) atomicAdd(&h[dl], (u32)__popcll(same));
        todo &= ~same;
    }
}
// H[digit * ntile + tile]: counts of digit `pass` per tile of this pass's input (the tiles of pass
// p > 0 are tiles of pass p - 1's output, so every pass counts its own input)
// AGG: wave-aggregated atomics, for inputs sorted on the lower digits (few distinct digits per
// wave); the unsorted first pass keeps plain atomics (aggregation measured slower there)
template <class KF, bool AGG>
__global__ __launch_bounds__(LS_T) void k_ls_hist(KF kf, u64 m, u32 pass, u32 ntile, u32* __restrict__ H) {
    __shared__ u32 hw[LS_T / 64][LS_NB];  // per-wave histograms: same-address atomics only within a wave
    for (u32 i = threadIdx.x; i < LS_NB * (LS_T / 64); i += LS_T) (&hw[0][0])[i] = 0;
    __syncthreads();
    u32* h = hw[threadIdx.x >> 6];
    const u64 t0 = (u64)blockIdx.x * LS_TILE;
    const u32 sh = pass * LS_DB;
    for (u32 i = 0; i < LS_IPT; i++) {
        const u64 e = t0 + (u64)i * LS_T + threadIdx.x;
        const bool valid = e < m;
        const u32 d = valid ? (kf(e) >> sh) & (LS_NB - 1) : 0u;
        if (AGG) wave_agg_add(h, d, valid);
        else if (valid) atomicAdd(&h[d], 1u);
    }
    __syncthreads();
    for (u32 i = threadIdx.x; i < LS_NB; i += LS_T) {
        u32 t = 0;
#pragma unroll
        for (u32 w = 0; w < LS_T / 64; w++) t += hw[w][i];
        H[(u64)i * ntile + blockIdx.x] = t;
    }
}
// one pass: items of tile `blockIdx` (pass 0: key kf(e), value e; later: kin / vin), sorted in LDS on
// digit `pass`, written at G[digit] + (rank within the digit).  LAST: values only, plus
// head[key] = min sorted index of the key
template <class KF, bool FIRST, bool LAST>
__global__ __launch_bounds__(LS_T) void k_ls_scatter(KF kf, const u32* __restrict__ kin, const u32* __restrict__ vin, u64 m,
                                                     u32 pass, u32 ntile, const u32* __restrict__ G, u32* __restrict__ kout,
                                                     u32* __restrict__ vout, u32* __restrict__ head) {
    using bsort = rocprim::block_radix_sort<u32, LS_T, LS_IPT, u32>;
    __shared__ union {
        typename bsort::storage_type sort;
        struct { u32 dig[LS_TILE]; u32 start[LS_NB]; u32 base[LS_NB]; } w;
    } sm;
    const u64 t0 = (u64)blockIdx.x * LS_TILE;
    u32 k[LS_IPT], v[LS_IPT];
#pragma unroll
    for (u32 i = 0; i < LS_IPT; i++) {
        const u64 e = t0 + (u64)threadIdx.x * LS_IPT + i;
        if (e < m) {
            k[i] = FIRST ? kf(e) : kin[e];
            v[i] = FIRST ? (u32)e : vin[e];
        } else {
            k[i] = 0xFFFFFFFFu;  // past the end: sorts after every item of the top digit
            v[i] = NONE;
        }
    }
    const u32 b0 = pass * LS_DB;
    bsort().sort_to_striped(k, v, sm.sort, b0, min(b0 + LS_DB, 32u));
    __syncthreads();
    // sorted position j = i * LS_T + tid; the first position of every digit in the tile
    const u32 nvalid = (u32)min<u64>(LS_TILE, m - t0);
#pragma unroll
    for (u32 i = 0; i < LS_IPT; i++) sm.w.dig[i * LS_T + threadIdx.x] = (k[i] >> b0) & (LS_NB - 1);
    __syncthreads();
#pragma unroll
    for (u32 i = 0; i < LS_IPT; i++) {
        const u32 j = i * LS_T + threadIdx.x;
        const u32 d = sm.w.dig[j];
        if (j < nvalid && (j == 0 || sm.w.dig[j - 1] != d)) sm.w.start[d] = j;
    }
    for (u32 d = threadIdx.x; d < LS_NB; d += LS_T) sm.w.base[d] = G[(u64)d * ntile + blockIdx.x];
    __syncthreads();
#pragma unroll
    for (u32 i = 0; i < LS_IPT; i++) {
        const u32 j = i * LS_T + threadIdx.x;
        if (j >= nvalid) break;
        const u32 d = sm.w.dig[j];
        const u32 pos = sm.w.base[d] + (j - sm.w.start[d]);
        vout[pos] = v[i];
        if (!LAST) kout[pos] = k[i];
    }
    if (LAST && head) {
        // the first item of every key in this tile (sorted by the whole key: the earlier passes
        // ordered the tile's input by the lower digits)
        __syncthreads();
#pragma unroll
        for (u32 i = 0; i < LS_IPT; i++) sm.w.dig[i * LS_T + threadIdx.x] = k[i];
        __syncthreads();
#pragma unroll
        for (u32 i = 0; i < LS_IPT; i++) {
            const u32 j = i * LS_T + threadIdx.x;
            if (j >= nvalid) break;
            if (j == 0 || sm.w.dig[j - 1] != k[i]) {
                const u32 d = (k[i] >> b0) & (LS_NB - 1);
                atomicMin(&head[k[i]], sm.w.base[d] + (j - sm.w.start[d]));
            }
        }
    }
}

// one pass by ballot ranking instead of a block sort: the tile's items (striped, in input
// order) go round by round; in a round every wave groups its lanes by digit (one ballot per
// distinct digit: few on these skewed keys), the per-wave digit counts in LDS give each item
// its rank behind the earlier waves of the round and the earlier rounds (running per-digit
// bases), and the item is written straight from registers.  Stable; no LDS exchange.
template <class KF, bool FIRST, bool LAST>
__global__ __launch_bounds__(LS_T) void k_ls_rank(KF kf, const u32* __restrict__ kin, const u32* __restrict__ vin, u64 m,
                                                  u32 pass, u32 ntile, const u32* __restrict__ G, u32* __restrict__ kout,
                                                  u32* __restrict__ vout) {
    __shared__ u32 s_base[LS_NB];
    __shared__ u32 s_wc[LS_T / 64][LS_NB];
    const u32 lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (u32 d = threadIdx.x; d < LS_NB; d += LS_T) s_base[d] = G[(u64)d * ntile + blockIdx.x];
    for (u32 d = lane; d < LS_NB; d += 64) s_wc[w][d] = 0;
    const u64 t0 = (u64)blockIdx.x * LS_TILE;
    const u32 b0 = pass * LS_DB;
    u32 k[LS_IPT], v[LS_IPT];
#pragma unroll
    for (u32 i = 0; i < LS_IPT; i++) {
        const u64 e = t0 + (u64)i * LS_T + threadIdx.x;
        k[i] = v[i] = 0;
        if (e < m) {
            k[i] = FIRST ? kf(e) : kin[e];
            v[i] = FIRST ? (u32)e : vin[e];
        }
    }
    __syncthreads();
#pragma unroll
    for (u32 i = 0; i < LS_IPT; i++) {
        const bool valid = t0 + (u64)i * LS_T + threadIdx.x < m;
        const u32 d = (k[i] >> b0) & (LS_NB - 1);
        u64 todo = __ballot(valid);
        u32 below = 0;
        while (todo) {
            const int leader = __ffsll((long long)todo) - 1;
            const u32 dl = __shfl(d, leader, 64);
            const u64 same = __ballot(valid && d == dl);
            if (valid && d == dl) below = (u32)__popcll(same & ((1ull << lane) - 1));
            if (lane == (u32)leader) s_wc[w][dl] = (u32)__popcll(same);
            todo &= ~same;
        }
        __syncthreads();
        u32 pos = 0;
        if (valid) {
            pos = s_base[d] + below;
            for (u32 w2 = 0; w2 < w; w2++) pos += s_wc[w2][d];
        }
        __syncthreads();
        for (u32 dd = threadIdx.x; dd < LS_NB; dd += LS_T) {
            u32 t = 0;
#pragma unroll
            for (u32 w2 = 0; w2 < LS_T / 64; w2++) {
                t += s_wc[w2][dd];
                s_wc[w2][dd] = 0;
            }
            s_base[dd] += t;
        }
        if (valid) {
            vout[pos] = v[i];
            if (kout) kout[pos] = k[i];
        }
        __syncthreads();
    }
}

// gap-index slot count (the carried table's entries) of the current phrases
u64 engine::carried_entries(int log2_override) {
    const pos_t N = (pos_t)n;
    const u32 m = num_phr;
    pos_t* P = lpf.get((u64)(m + 1) * 3);
    k_put3<<<1, 1, 0, st>>>(P + 3 * (u64)m, N, N + 1, 0);
    u64 num_gaps = 1;
    pos_t len_lpf_phr = 0;
    if (m > 0) {
        u64* acc = counters64.get(16) + 2;
        LZ_HIP(hipMemsetAsync(acc, 0, 16, st));
        k_phrase_info<<<cdiv(m, 256), 256, 0, st>>>(P, m, N, acc);
        u64 h2[2];
        hread rb(st);
        rb.add(h2, acc, 2);
        rb.sync();
        len_lpf_phr = (pos_t)h2[0];
        num_gaps = h2[1];
    }
    gap_params_h gp = choose_gap_params(N, m, len_lpf_phr, num_gaps);
    if (log2_override > 0) gp.log2_size_h = (u32)log2_override;
    return 1ull << gp.log2_size_h;
}

u64 engine::factorize_greedy(const u8* T, u32 rk_seed, int log2_override, greedy_block* blk) {
    const bool dbg = debug_enabled();
    double t_mark = now_ms();
    auto lap = [&](const char* what) {
        if (!dbg) return;
        LZ_HIP(hipStreamSynchronize(st));
        const double t = now_ms();
        std::fprintf(stderr, "[lz77sss-debug]   %-28s %9.3f ms\n", what, t - t_mark);
        t_mark = t;
    };
    const pos_t N = (pos_t)n;
    const u32 m = num_phr;  // phrases; P[m] = sentinel
    pos_t* P = lpf.get((u64)(m + 1) * 3);
    // ---- phrase statistics -> parameters (lz77_sss.hpp:420-461)
    u64 num_lpf = m, num_gaps = 1;
    pos_t len_lpf_phr = 0;
    if (!phr_info.valid) k_put3<<<1, 1, 0, st>>>(P + 3 * (u64)m, N, N + 1, 0);
    if (phr_info.valid && m > 0) {
        len_lpf_phr = (pos_t)phr_info.len;  // (build_lpf_opt: statistics and sentinel done)
        num_gaps = phr_info.gaps;
    } else if (m > 0) {
        u64* acc = counters64.get(16) + 2;
        LZ_HIP(hipMemsetAsync(acc, 0, 16, st));
        k_phrase_info<<<cdiv(m, 256), 256, 0, st>>>(P, m, N, acc);
        u64 h2[2];
        hread rb(st);
        rb.add(h2, acc, 2);
        rb.sync();
        len_lpf_phr = (pos_t)h2[0];
        num_gaps = h2[1];
    }
    gap_params_h gp = choose_gap_params(N, num_lpf, len_lpf_phr, num_gaps);
    if (log2_override > 0) gp.log2_size_h = (u32)log2_override;
    // bases: rk_prime::random64(257, 2^20-1) from mt19937_64(rk_seed) (rolling_hash.hpp:127-130)
    std::array<u64, 5> bases;
    {
        std::mt19937_64 g(rk_seed);
        for (int i = 0; i < 5; i++) bases[i] = std::uniform_int_distribution<u64>(257, (1ull << 20) - 1)(g);
    }
    // the influence tables depend only on (bases, pattern lengths): uploaded once per change
    u128* d_negpow = (u128*)tmp_greedy.get(5 * 256 * sizeof(u128));
    {
        std::array<u64, 10> key;
        for (int x = 0; x < 5; x++) { key[x] = bases[x]; key[5 + x] = gp.patt_lens[x]; }
        if (key != negpow_key || d_negpow != negpow_dev) {
            std::vector<u128> negpow(5 * 256);
            for (int x = 0; x < 5; x++) {
                const u128 bp = powmod107_host(bases[x], gp.patt_lens[x]);
                const u128 nbp = (P107 - bp) % P107;
                negpow[x * 256] = 0;
                for (int o = 1; o < 256; o++) negpow[x * 256 + o] = mod107(negpow[x * 256 + o - 1] + nbp);
            }
            LZ_HIP(hipMemcpyAsync(d_negpow, negpow.data(), 5 * 256 * sizeof(u128), hipMemcpyHostToDevice, st));
            LZ_HIP(hipStreamSynchronize(st));  // (the host vector goes out of scope)
            negpow_key = key;
            negpow_dev = d_negpow;
        }
    }

    stats.assign(28, 0);
    stats[0] = s; stats[1] = has_runs; stats[2] = num_lpf; stats[3] = len_lpf_phr; stats[4] = num_gaps;
    for (int x = 0; x < 5; x++) stats[5 + x] = gp.patt_lens[x];
    stats[10] = gp.roll_threshold; stats[11] = gp.log2_size_h;

    gap_cfg G{};
    G.n = N;
    G.nt = N > 64 ? N - 64 : 0;
    for (int x = 0; x < 5; x++) { G.lens[x] = gp.patt_lens[x]; G.base[x] = bases[x]; }
    G.thr = gp.roll_threshold;
    G.mask = (u32)((1ull << gp.log2_size_h) - 1);
    G.negpow = d_negpow;
    u32 zmask0 = 0;
    for (int x = 0; x < 5; x++) zmask0 |= (G.lens[x] >= N) ? (1u << x) : 0u;  // reinit(0) at construction
    // test knobs of the chain-insert kernels, read once per call: a small long-range list and a
    // short "long" range make the overflow path run
    const u32 knob_lng_cap = [] {
        const char* e = std::getenv("LZ77SSS_TEST_LNG_CAP");
        return e ? (u32)std::max<long>(0, std::atol(e)) : 0xFFFFFFFFu;
    }();
    const u32 knob_long_words = [] {
        const char* e = std::getenv("LZ77SSS_TEST_LONG_WORDS");
        return e ? (u32)std::max<long>(1, std::atol(e)) : 2048u;
    }();
    const char* ch_env = std::getenv("LZ77SSS_GAP_CHUNK");  // tuning knob (walk length per segment)
    const u32 CH = std::getenv("LZ77SSS_NO_CHUNK") ? 0x0FFFFFFFu : ch_env ? (u32)std::max(16, std::atoi(ch_env)) : 512u;
    const char* mo_env = std::getenv("LZ77SSS_GREEDY_MAX_OUTER");  // test knob (0: sequential only)
    const int max_outer = mo_env ? std::max(0, std::atoi(mo_env)) : 256;
    const u64 nslots_all = (u64)G.mask + 1;
    const char* psm = std::getenv("LZ77SSS_PRED_SORTED_MIN");
    const u64 pred_sorted_min = psm ? std::strtoull(psm, nullptr, 10) : (1ull << 27);

    // ---- windows: the chain is walked window by window; a window gets the
    // exact chain state at its start and the table of the last insert per slot before it
    // (pos + 1, 0 = none), and hands both on.  Windows bound the gap-index entry ids
    // (32-bit) and every position-indexed structure to the window's span.  One window
    // covers the text unless its base set would not fit (or LZ77SSS_GREEDY_WINDOW asks).
    const u64 est_base = (u64)(N - len_lpf_phr) + 49ull * (m + 1);  // gap positions + queries + short phrases
    u64 WS = N;
    if (const char* we = std::getenv("LZ77SSS_GREEDY_WINDOW")) {
        WS = std::max<u64>(4096, std::strtoull(we, nullptr, 10));
    } else if (est_base * 5 >= (1ull << 31)) {
        // windows of ~2^31 / 10 base positions (uniform gap density assumed; a window whose base
        // set still overflows the ids fails loudly below)
        WS = std::max<u64>(1ull << 20, (u64)((double)N * ((double)(1ull << 31) / 10.0) / (double)est_base));
    }
    // a block of a sharded factorization: [blk->start, blk->end) from the given chain state
    const pos_t target_end = blk ? blk->end : N;
    if (blk && (blk->end > N || blk->start >= blk->end || (blk->end < N && (u64)blk->end + 4096 > (u64)G.nt)))
        throw error(LZ77SSS_EINVAL, "greedy block: need start < end and end == n or end <= n - 4160");
    const bool multi = WS < (u64)N;
    const bool carry = multi || blk;
    pos_t* Hs = nullptr;
    if (carry) {
        if (blk && blk->carried && g_Hs.cap < nslots_all)
            throw error(LZ77SSS_EINVAL, "greedy block: carried table not loaded (size it with carried_entries)");
        Hs = g_Hs.get(nslots_all);
        if (!(blk && blk->carried)) LZ_HIP(hipMemsetAsync(Hs, 0, nslots_all * sizeof(pos_t), st));
    }
    if (blk && !blk->carried && blk->seed && blk->start > 0) {
        // a lead-in of a speculative block: the table seeded from the gap positions before it
        u32* cnt = g_tmp1.get(m + 2);
        u32* off = g_tmp2.get(m + 2);
        k_seed_counts<<<cdiv(m + 1, 256), 256, 0, st>>>(P, m, blk->start, cnt);
        const u32 nch = excl_scan(cnt, off, m + 1, scan_tmp, st);
        if (nch) k_seed_slots<<<cdiv(5ull * nch, 256), 256, 0, st>>>(T, G, P, m, blk->start, off, nch, Hs);
        k_seed_queries<<<cdiv(5ull * (m + 1), 256), 256, 0, st>>>(T, G, P, m, blk->start, Hs);
        LZ_HIP(hipGetLastError());
    }
    if (blk && spec_track && nslots_all > spec_m)
        throw error(LZ77SSS_EINVAL, "speculative block: the carried table changed size since spec_begin");
    seg_in entry{0, 0, 0, zmask0, N};
    if (blk) {
        entry.start = blk->start;
        entry.idxpos = blk->idxpos;
        entry.zmask = blk->zmask;
    }
    u64 total_fact = 0, walked_all = 0;
    int outer_all = 0, rounds_all = 0, nwin = 0;
    u32 nseg_last = 0, nseg0_all = 0;
    lce_view Lv = view(T);
    // a non-last window (or block) whose chain reaches the tail region (a gap factor
    // longer than the >= 4096 positions left after the window end) is walked again as the
    // last window: the tail model needs every insert in the tail region before its start
    bool force_last = false;

    for (;;) {
        const pos_t a = entry.start;
        // the window [a, bw): non-last windows end below the tail region (nt) and leave >= 4096 positions
        pos_t bw = force_last ? N : target_end;
        if (!force_last && WS < (u64)(target_end - a) && (u64)a + WS + 4096 <= (u64)G.nt) bw = (pos_t)(a + WS);
        const bool last = bw == N;
        bool redo = false;
        const pos_t off = a & ~(pos_t)31;  // bitmap origin (word aligned)
        const u64 nw = (u64)(bw - off) / 32 + 2;  // bitmap words (a zero word past the end)
        const unsigned gw = cdiv(nw, 256);
        const unsigned bmb_blocks = (unsigned)std::max<u64>(1, (nw + BMB - 1) / BMB);
        const pos_t hi_ins = std::min<pos_t>(bw, G.nt);  // inserts recorded in the window bitmaps: [a, hi_ins)

        // ---- default segments: gaps (clipped to the window) + chunk boundaries of long gaps
        u32* cnt_seg = g_tmp1.get(m + 2);
        u32* cnt_cb = g_tmp2.get(m + 2);
        u32* off_seg = g_tmp3.get(m + 2);
        u32* off_cb = g_tmp4.get(m + 2);
        k_gap_counts<<<cdiv(m + 1, 256), 256, 0, st>>>(P, m, CH, a, bw, G.nt, cnt_seg, cnt_cb);
        excl_scan_nr(cnt_seg, off_seg, m + 1, scan_tmp, st);
        excl_scan_nr(cnt_cb, off_cb, m + 1, scan_tmp, st);
        u32 nseg0, ncb;
        {
            hread rb(st);
            rb.add(&nseg0, off_seg + m + 1);
            rb.add(&ncb, off_cb + m + 1);
            rb.sync();
        }
        pos_t* cbv = g_cbv.get(ncb + 1);
        if (ncb) k_gap_cbv<<<cdiv(ncb, 256), 256, 0, st>>>(P, m, CH, a, bw, off_cb, ncb, cbv);
        u32 cap = nseg0 + nseg0 / 2 + (1u << 16);
        seg_tab S{};
        auto bind_tab = [&]() {
            S.sin = g_sin.p; S.sout = g_sout.p; S.valid = g_valid.p; S.succ = g_succ.p; S.cap = cap;
            S.stash = g_stash.p;
        };
        g_sin.get(cap); g_sout.get(cap); g_valid.get(cap); g_succ.get(cap);
        g_stash.get((u64)cap * 2 * STASH_CAP);
        bind_tab();
        {
            // the position -> segment map is cleared sparsely after each window (k_seg_at_clear);
            // a fresh or reallocated map, or one left dirty by a failed call, is cleared densely
            const u64 span = (u64)(bw - a) + 1;
            u32* prev = g_seg_at.p;
            S.seg_at = g_seg_at.get(span);
            if (S.seg_at != prev || !seg_at_clean || seg_at_n < span) {
                LZ_HIP(hipMemsetAsync(S.seg_at, 0xFF, g_seg_at.cap * 4, st));
                seg_at_n = g_seg_at.cap;
            }
            seg_at_clean = false;
        }
        S.segoff = a;
        S.nseg = (u32*)counters64.get(16);  // [0] nseg/err, [1] c0, [2..3] phrase info, [4..] entry seg_in
        S.err = S.nseg + 1;
        k_set_u32x2<<<1, 1, 0, st>>>(S.nseg, nseg0, 0);
        S.cbv = cbv; S.ncb = ncb; S.P = P; S.m = m; S.N = bw; S.zmask0 = zmask0;
        if (nseg0) k_gap_segs<<<cdiv(nseg0, 256), 256, 0, st>>>(S, CH, off_seg, nseg0);
        u32* d_c0 = (u32*)(counters64.p + 1);
        static_assert(sizeof(seg_in) <= 12 * sizeof(u64), "entry slot");
        seg_in* d_entry = (seg_in*)(counters64.p + 4);
        k_entry_seg<<<1, 1, 0, st>>>(S, a, entry.idxpos, entry.zmask, d_c0, d_entry);
        // bitmaps: I (current speculation), I' (what the chain inserted), Ib (base set), scratch
        u32* bmI = g_bmI.get(nw);
        u32* bmI2 = g_bmI2.get(nw);
        u32* bmIb = g_bmIb.get(nw);
        u32* bmT = g_bmT.get(nw);
        // the superset goes straight into Ib (the first base set); the scratch bitmap is
        // always fully overwritten before it is read
        fills({{bmI, nw * 4, 0u}, {bmIb, nw * 4, 0u}});
        if (nseg0)
            k_gap_bitmaps<<<capped_grid((u64)nseg0 * 64, 256), 256, 0, st>>>(S, nseg0, N, G.nt, hi_ins, off, bmI, bmIb);
        k_gap_bitmaps_phr<<<cdiv(m + 1, 256), 256, 0, st>>>(P, m, N, G.nt, a, hi_ins, off, bmI, bmIb);
        u32 hn[2];
        u32 c0 = 0;
        // the exact entry of the window as the completion path sees it
        seg_in entry_in;
        {
            hread rb(st);
            rb.add(hn, S.nseg, 2);
            rb.add(&c0, d_c0);
            rb.add(&entry_in, d_entry);
            rb.sync();
        }
        const u32 nseg_init = hn[0];
        lap("greedy setup");

        walk_ctx W{};
        W.T = T;
        W.G = G;
        W.P = P;
        W.L = Lv;
        W.bmoff = off;
        W.Hs = Hs;
        // speculative part: its bitmap of used entry-table slots; values below the
        // speculative block's start come from that table (earlier parts' writes do not)
        W.hs_used = (blk && spec_track) ? g_hsused.p + (u64)spec_part * (spec_m / 32 + 1) : nullptr;
        W.blk_start = blk ? (spec_track ? (pos_t)spec_base : blk->start) : 0;

        // window exit (the chain state at the first handover point >= bw) and the carried table
        seg_in exit_in{};
        // ---- bounded completion (k_seq_walk): the chain prefix [0, k*) is written by the
        // segment walks, the rest of the window by the exact sequential walk from chain node k*
        u64* d_sq = (u64*)g_cut.get(sizeof(chain_cut) + 256);
        chain_cut* d_cutp = (chain_cut*)(d_sq + 8);
        u64* d_y0 = d_sq + 6;
        auto seq_complete = [&](const u32* chain, u32 nall, const u64* offs, const u32* ins_bm, bool from_entry) -> u64 {
            if (from_entry) LZ_HIP(hipMemsetAsync(d_y0, 0, 8, st));
            k_chain_cut<<<1, 1, 0, st>>>(S, chain, from_entry ? 0u : nall, d_y0, entry_in, d_cutp);
            chain_cut cut;
            {
                hread rb(st);
                rb.add(&cut, (const chain_cut*)d_cutp);
                rb.sync();
            }
            const u64 offk = cut.k ? rd1(offs + cut.k, st) : 0;
            pos_t* fo = fact.get(2 * (offk + (u64)(N - cut.in.start) + 2) + 2);
            if (cut.k) {
                k_walk<true><<<cdiv(cut.k, 64), 64, 0, st>>>(W, S, chain, cut.k, offs, fo);
                LZ_HIP(hipGetLastError());
            }
            pos_t* H = g_H.get((u64)nslots_all);
            if (Hs) LZ_HIP(hipMemcpyAsync(H, Hs, nslots_all * sizeof(pos_t), hipMemcpyDeviceToDevice, st));
            else LZ_HIP(hipMemsetAsync(H, 0, nslots_all * sizeof(pos_t), st));
            if (cut.in.start > off && ins_bm)
                k_h_fill<<<cdiv(((u64)(cut.in.start - off) + 31) / 32, 256), 256, 0, st>>>(T, G, ins_bm, off, cut.in.start,
                                                                                         H);
            k_h_fix<<<cdiv(nslots_all, 256), 256, 0, st>>>(H, nslots_all);
            k_seq_walk<<<1, 64, 0, st>>>(T, G, P, Lv, H, cut.in, last ? N + 1 : bw, fo, offk, d_sq, W.hs_used,
                                         W.blk_start);
            LZ_HIP(hipGetLastError());
            u64 hc[4];
            {
                hread rb(st);
                rb.add(hc, (const u64*)d_sq, 4);
                rb.sync();
            }
            if (hc[1]) throw error(-6, "greedy: sequential completion guard tripped (internal error)");
            if (!last && hc[2] >= (u64)G.nt) {
                redo = true;  // the hand-over point lies in the tail region
                return 0;
            }
            if (!last) {
                exit_in.start = (pos_t)hc[2];
                exit_in.idxpos = (pos_t)hc[3];
                exit_in.zmask = 0;  // below the tail region no fingerprint is zeroed
                k_h_unfix<<<cdiv(nslots_all, 256), 256, 0, st>>>(H, nslots_all, Hs);
            }
            stats[19] = 1;
            stats[20] = cut.in.start;
            lap("sequential completion");
            return offk + hc[0];
        };

        // ---- base set (entries sorted by slot) and delta
        u64 nb = 0;
        const u32 nslots = G.mask + 1;
        auto build_buckets = [&](auto key, u64 mk, dbuf<u32>& bk) {
            u32* b = bk.get((u64)nslots + 1);
            if (mk * 16 >= nslots) {
                u32* rev = g_brev.get(2 * ((u64)nslots + 1));
                u32* scn = rev + nslots + 1;
                LZ_HIP(hipMemsetAsync(rev, 0xFF, ((u64)nslots + 1) * 4, st));
                k_bucket_heads<<<cdiv(mk + 1, 256), 256, 0, st>>>(key, mk, nslots, rev);
                size_t tb = 0;
                LZ_HIP(hipcub::DeviceScan::InclusiveScan(nullptr, tb, rev, scn, min_u32_op{}, (int)(nslots + 1), st));
                u8* t = scan_tmp.get(tb);
                LZ_HIP(hipcub::DeviceScan::InclusiveScan(t, tb, rev, scn, min_u32_op{}, (int)(nslots + 1), st));
                k_unreverse<<<cdiv((u64)nslots + 1, 256), 256, 0, st>>>(scn, nslots, b);
            } else {
                k_bucket_search<<<cdiv((u64)nslots + 1, 256), 256, 0, st>>>(key, mk, nslots, b);
            }
        };
        // runs of a bitmap -> intervals (st, en), ranks, chunks for k_slots
        auto runs_to_chunks = [&](const u32* bm, dbuf<pos_t>& dst, dbuf<pos_t>& den, dbuf<u32>& drk, dbuf<u8>& dch,
                                  u32& ni, u64& npos, u32& nch) -> ichunk* {
            const u64 tot = bmb_scan(bm_runs{bm}, nw, g_bsum, g_bincl, scan_tmp, st);
            ni = (u32)(tot >> 32);  // run starts (= run ends)
            pos_t* ra = dst.get(ni + 1);
            pos_t* rb = den.get(ni + 1);
            k_bmb_write<<<bmb_blocks, BMB_T, 0, st>>>(bm_runs{bm}, nw, g_bincl.p, out_runs{ra, rb}, off);
            u32* len = g_tmp5.get(ni + 1);
            u32* nc = g_tmp6.get(ni + 1);
            u32* rk = drk.get(ni + 1);
            u32* choff = g_tmp7.get(ni + 1);
            npos = 0;
            nch = 0;
            u32 chl = SLOT_CHUNK_LONG;
            if (ni) {
                u32* ncs = g_tmp8.get(ni + 1);
                // short chunks (test/tuning knob LZ77SSS_SLOT_CHUNK, <= SLOT_CHUNK_LONG)
                const char* sce = std::getenv("LZ77SSS_SLOT_CHUNK");
                const u32 scl = sce ? std::max(8u, std::min<u32>(SLOT_CHUNK_LONG, (u32)std::atoi(sce))) : SLOT_CHUNK_SHORT;
                k_iv_chunk_counts<<<cdiv(ni, 256), 256, 0, st>>>(ra, rb, ni, nc, ncs, len, scl);
                npos = excl_scan(len, rk, ni, scan_tmp, st);
                if (npos < (u64)SLOT_CHUNK_LONG << (std::getenv("LZ77SSS_SLOT_CHUNK_SH") ? std::atoi(std::getenv("LZ77SSS_SLOT_CHUNK_SH")) : 18)) chl = scl;
                nch = excl_scan(chl == SLOT_CHUNK_LONG ? nc : ncs, choff, ni, scan_tmp, st);
            }
            ichunk* ch = (ichunk*)dch.get(std::max<u64>(1, nch) * sizeof(ichunk));
            if (nch) k_iv_chunks<<<cdiv(nch, 256), 256, 0, st>>>(ra, rb, ni, choff, nch, chl, rk, ch);
            return ch;
        };
        // LSD sort of m entries on `bits` key bits (pass-0 keys from kf0): entry ids to vout, the first
        // sorted index of every key to head (pre-set to NONE); ka / va: scratch for the middle passes
        auto lsd_sort = [&](auto kf0, u64 m, u32 bits, u32* ka, u32* va, u32* vout, u32* head, u32 nkeys) {
            const u32 npass = std::max<u32>(1, (bits + LS_DB - 1) / LS_DB);
            if (npass > LS_MAXP) throw error(-6, "lsd_sort: too many key bits");
            const u32 ntile = cdiv(m, LS_TILE);
            const u64 per = (u64)LS_NB * ntile;
            u32* H = g_ls_h.get(per + 1);
            u32* Gs = g_ls_g.get(per + 1);
            // the first pass (entry order: many distinct digits per wave) block-sorts its tiles, the
            // later ones (inputs sorted on the lower digits: few per wave) rank by ballots
            // (rr 13-bit dense keys: pass 0 278 vs 369 us, pass 1 167 vs 284 us); LZ77SSS_LS_BLOCKSORT /
            // LZ77SSS_LS_RANK force either for every pass
            const bool all_bs = std::getenv("LZ77SSS_LS_BLOCKSORT") != nullptr, all_rk = std::getenv("LZ77SSS_LS_RANK") != nullptr;
            auto use_bsort = [&](u32 p) { return all_bs || (!all_rk && p == 0); };
            const bool bsort = use_bsort(npass - 1);  // the last pass: heads in the block-sort kernel
            // ping-pong: pass p reads what pass p - 1 wrote (the ranking form writes the last pass's
            // keys too, for the key heads)
            const bool kb1 = npass > 2 || (head && !bsort && npass > 1);
            u32 *kb[2] = {ka, kb1 ? g_predk.get(m + 1) : nullptr}, *vb[2] = {va, npass > 2 ? g_ids2.get(m + 1) : nullptr};
            u32* klast = nullptr;
            for (u32 p = 0; p < npass; p++) {
                const bool first = p == 0, lastp = p + 1 == npass;
                u32 *ko = kb[p & 1], *vo = lastp ? vout : vb[p & 1];
                const u32 *ki = kb[(p + 1) & 1], *vi = vb[(p + 1) & 1];
                const ls_plain kp{ki};
                if (first) k_ls_hist<decltype(kf0), false><<<ntile, LS_T, 0, st>>>(kf0, m, p, ntile, H);
                else k_ls_hist<ls_plain, true><<<ntile, LS_T, 0, st>>>(kp, m, p, ntile, H);
                excl_sum64(H, Gs, 0u, per, scan_tmp, st);
                if (use_bsort(p)) {
                    if (first && lastp)
                        k_ls_scatter<decltype(kf0), true, true><<<ntile, LS_T, 0, st>>>(kf0, ki, vi, m, p, ntile, Gs, ko, vo, head);
                    else if (first)
                        k_ls_scatter<decltype(kf0), true, false><<<ntile, LS_T, 0, st>>>(kf0, ki, vi, m, p, ntile, Gs, ko, vo, head);
                    else if (lastp)
                        k_ls_scatter<ls_plain, false, true><<<ntile, LS_T, 0, st>>>(kp, ki, vi, m, p, ntile, Gs, ko, vo, head);
                    else
                        k_ls_scatter<ls_plain, false, false><<<ntile, LS_T, 0, st>>>(kp, ki, vi, m, p, ntile, Gs, ko, vo, head);
                } else {
                    u32* kw = (lastp && !head) ? nullptr : ko;
                    if (lastp) klast = kw;
                    if (first && lastp)
                        k_ls_rank<decltype(kf0), true, true><<<ntile, LS_T, 0, st>>>(kf0, ki, vi, m, p, ntile, Gs, kw, vo);
                    else if (first)
                        k_ls_rank<decltype(kf0), true, false><<<ntile, LS_T, 0, st>>>(kf0, ki, vi, m, p, ntile, Gs, kw, vo);
                    else if (lastp)
                        k_ls_rank<ls_plain, false, true><<<ntile, LS_T, 0, st>>>(kp, ki, vi, m, p, ntile, Gs, kw, vo);
                    else
                        k_ls_rank<ls_plain, false, false><<<ntile, LS_T, 0, st>>>(kp, ki, vi, m, p, ntile, Gs, kw, vo);
                }
            }
            if (head && !bsort) k_dense_heads<<<cdiv(cdiv(m + 1, 4), 256), 256, 0, st>>>(klast, m, nkeys, head);
            LZ_HIP(hipGetLastError());
        };
        // base sets this large get their predecessors in sorted order and moved back to
        // entry order in buckets (random 4-byte scatters over the whole array are slower)
        auto build_base = [&](const u32* bm) {
            if (bm != bmIb) LZ_HIP(hipMemcpyAsync(bmIb, bm, nw * 4, hipMemcpyDeviceToDevice, st));
            u32 ni, nch;
            ichunk* ch = runs_to_chunks(bmIb, ist, iend, irank, chunk_buf, ni, nb, nch);
            if (dbg) {
                std::fprintf(stderr, "[lz77sss-debug] greedy base: intervals=%u positions=%llu chunks=%u slots=2^%u\n", ni,
                             (unsigned long long)nb, nch, gp.log2_size_h);
                pos_t r[4] = {0, 0, 0, 0};
                if (ni) {
                    LZ_HIP(hipMemcpy(r, ist.p, sizeof(pos_t) * std::min<u32>(ni, 2), hipMemcpyDeviceToHost));
                    LZ_HIP(hipMemcpy(r + 2, iend.p, sizeof(pos_t) * std::min<u32>(ni, 2), hipMemcpyDeviceToHost));
                }
                std::fprintf(stderr, "[lz77sss-debug] greedy base: window [%llu, %llu) off=%llu nw=%llu runs %llu-%llu %llu-%llu\n",
                             (unsigned long long)a, (unsigned long long)bw, (unsigned long long)off,
                             (unsigned long long)nw, (unsigned long long)r[0], (unsigned long long)r[2],
                             (unsigned long long)r[1], (unsigned long long)r[3]);
            }
            lap("base intervals");
            if (5 * nb >= (1ull << 32))
                throw error(-1, "gap region of a greedy window too large for 32-bit entry ids (set LZ77SSS_GREEDY_WINDOW)");
            const u64 ne5 = 5 * nb;
            u32* keys = ekeys.get(ne5 + 1);
            u32* vals = evals.get(ne5 + 1);
            u32* skeys = ekeys2.get(ne5 + 1);
            u32* svals = evals2.get(ne5 + 1);
            pos_t* ipos = ipos_buf.get(nb + 1);
            u32* pred5 = occ_buf.get(ne5 + 1);
            u8* rem = rem_buf.get(nb + 1);
            bool dense = false, ls = false;
            u32 D = 0, dense_bits = 0;
            const u64 npw = ((u64)nslots + 31) / 32;
            u32* pbm = g_pbm.get(npw + 1);
            u32* pwp = g_pwp.get(npw + 1);
            // distinct slots -> dense ids when that saves radix passes (tried below 2^28 entries:
            // a base set that large comes from a non-repetitive text, whose slots are all in use);
            // k_slots marks the present slots
            const bool try_dense = nch && ne5 < (1ull << 28) && !std::getenv("LZ77SSS_NO_DENSE");
            u8* pf = try_dense ? (u8*)g_pflag.get(npw * 8) : nullptr;
            fills({{rem, nb + 1, 0u}, {pf, pf ? npw * 32 : 0, 0u}});
            if (nch) {
                k_slots<<<cdiv(nch, SL_CH), SL_T, 0, st>>>(T, G, ch, nch, keys, nullptr, ipos, pf);
                lap("base slots");
                if (try_dense) {
                    u32* pcnt = g_pcnt.get(npw + 1);
                    k_presence_pack<<<cdiv(npw, 256), 256, 0, st>>>(pf, npw, pbm, pcnt);
                    D = excl_scan(pcnt, pwp, npw, scan_tmp, st);
                    u32 dbits = 1;
                    while (dbits < 32 && (1ull << dbits) < D) dbits++;
                    dense = (dbits + 7) / 8 < (gp.log2_size_h + 7) / 8;
                    dense_bits = dbits;
                }
                u32* sk_in = keys;
                u32 sbits = gp.log2_size_h;
                // dense ids and bucket-search lookups (no predecessors): the LSD sort over the raw
                // slots, dense-id map fused into its first pass, entry ids and dense-id starts out
                ls = dense && !W.use_pred && !std::getenv("LZ77SSS_NO_LSD");
                if (ls) {
                    u32* dstart = g_dstart.get((u64)D + 2);
                    fills({{dstart, (u64)D * 4, ~0u}, {dstart + D, 4, (u32)ne5}, {dstart + D + 1, 4, 0u}});
                    u64* pbw = (u64*)g_pbw.get(2 * npw);
                    k_pack_pbw<<<cdiv(npw, 256), 256, 0, st>>>(pbm, pwp, npw, pbw);
                    lsd_sort(ls_dense{keys, pbw}, ne5, dense_bits, skeys, vals, svals, dstart, D);
                    if (std::getenv("LZ77SSS_LSD_CHECK")) {
                        // the rocprim path into scratch, compared entry by entry
                        u32* dk = g_sdk.get(ne5 + 1);
                        u32* ck = g_predk.get(ne5 + 1);
                        u32* cv = g_ids2.get(ne5 + 1);
                        k_dense_keys<<<cdiv(cdiv(ne5, 4), 256), 256, 0, st>>>(keys, ne5, pbm, pwp, dk);
                        size_t tb = 0;
                        const rocprim::counting_iterator<u32> ids(0);
                        LZ_HIP(rocprim::radix_sort_pairs(nullptr, tb, dk, ck, ids, cv, (size_t)ne5, 0u, dense_bits, st));
                        u8* t = scan_tmp.get(tb);
                        LZ_HIP(rocprim::radix_sort_pairs(t, tb, dk, ck, ids, cv, (size_t)ne5, 0u, dense_bits, st));
                        u32* ds2 = g_pcnt.get(std::max<u64>(npw + 1, (u64)D + 2));
                        k_pred_heads<<<cdiv(ne5 + 1, 256), 256, 0, st>>>(ck, cv, ne5, D, nullptr, ds2);
                        u64* r = (u64*)g_cut.get(sizeof(chain_cut) + 256) + 20;
                        const u64 init[4] = {~0ull, 0, ~0ull, 0};
                        LZ_HIP(hipMemcpyAsync(r, init, 32, hipMemcpyHostToDevice, st));
                        k_first_diff_u32<<<cdiv(ne5, 256), 256, 0, st>>>(svals, cv, ne5, r);
                        k_first_diff_u32<<<cdiv((u64)D + 1, 256), 256, 0, st>>>(dstart, ds2, (u64)D + 1, r + 2);
                        u64 h[4];
                        LZ_HIP(hipMemcpyAsync(h, r, 32, hipMemcpyDeviceToHost, st));
                        LZ_HIP(hipStreamSynchronize(st));
                        std::fprintf(stderr, "[lz77sss-lsd-check] m=%llu D=%u bits=%u: svals diff=%llu first=%lld, dstart diff=%llu first=%lld\n",
                                     (unsigned long long)ne5, D, dense_bits, (unsigned long long)h[1], (long long)h[0],
                                     (unsigned long long)h[3], (long long)h[2]);
                        if (h[1] || h[3]) {
                            u32 a[8], b[8];
                            const u64 f = h[1] ? std::min<u64>(h[0], ne5 - 8) : 0;
                            LZ_HIP(hipMemcpy(a, svals + f, 32, hipMemcpyDeviceToHost));
                            LZ_HIP(hipMemcpy(b, cv + f, 32, hipMemcpyDeviceToHost));
                            for (int q = 0; q < 8; q++) std::fprintf(stderr, "  [%llu] lsd %u rocprim %u\n", (unsigned long long)(f + q), a[q], b[q]);
                        }
                    }
                    if (dbg)
                        std::fprintf(stderr, "[lz77sss-debug] greedy base: %u distinct slots, LSD sort on %u bits\n", D,
                                     dense_bits);
                } else if (dense) {
                    // (a transform iterator mapping the ids inside the sort was slower: rr sort
                    // passes +234 us against this pass's 211 us)
                    k_dense_keys<<<cdiv(cdiv(ne5, 4), 256), 256, 0, st>>>(keys, ne5, pbm, pwp, skeys);
                    sk_in = skeys;
                    skeys = g_sdk.get(ne5 + 1);
                    sbits = dense_bits;
                }
                if (!ls) {
                    if (dbg)
                        std::fprintf(stderr, "[lz77sss-debug] greedy base: %u distinct slots, %s sort on %u bits\n", D,
                                     dense ? "dense-id" : "slot", sbits);
                    size_t tb = 0;
                    // values = entry ids: a counting iterator, so the ids are never written or read
                    const rocprim::counting_iterator<u32> ids(0);
                    LZ_HIP(rocprim::radix_sort_pairs(nullptr, tb, sk_in, skeys, ids, svals, (size_t)ne5, 0u, sbits, st));
                    u8* t = scan_tmp.get(tb);
                    LZ_HIP(rocprim::radix_sort_pairs(t, tb, sk_in, skeys, ids, svals, (size_t)ne5, 0u, sbits, st));
                    if (dense && ne5 < pred_sorted_min) {
                        // predecessors and dense-id starts in one pass (buckets below reuse dstart)
                        k_pred_heads<<<cdiv(ne5 + 1, 256), 256, 0, st>>>(skeys, svals, ne5, D, W.use_pred ? pred5 : nullptr,
                                                                          g_dstart.get((u64)D + 1));
                    } else if (W.use_pred && ne5 < pred_sorted_min) {
                        k_pred<<<cdiv(ne5, 256), 256, 0, st>>>(skeys, svals, ne5, pred5);
                    } else if (W.use_pred) {
                        // pred5[e] = predecessor of entry e in its slot: the sorted-order predecessors
                        // moved back to entry order (a random scatter of 4-byte writes is ~3x slower)
                        if (std::getenv("LZ77SSS_PRED_RADIX")) {  // reference path: radix sort by entry id
                            u32* pv = vals;  // the unsorted values are no longer needed
                            k_pred_sorted<<<cdiv(ne5, 256), 256, 0, st>>>(skeys, svals, ne5, pv);
                            u32* kdump = g_predk.get(ne5 + 1);
                            int eb = 1;
                            while (eb < 32 && (1ull << eb) < ne5) eb++;
                            size_t tb2 = 0;
                            LZ_HIP(rocprim::radix_sort_pairs(nullptr, tb2, svals, kdump, pv, pred5, (size_t)ne5, 0u,
                                                             (unsigned)eb, st));
                            u8* t2 = scan_tmp.get(tb2);
                            LZ_HIP(rocprim::radix_sort_pairs(t2, tb2, svals, kdump, pv, pred5, (size_t)ne5, 0u, (unsigned)eb,
                                                             st));
                        } else {
                            const u32 nbk = (u32)((ne5 + (1ull << PB_SH) - 1) >> PB_SH);
                            u32* cursor = g_pbcur.get(nbk + 1);
                            u64* tmp = g_pbtmp.get(ne5);
                            const u32 ntile = (u32)std::min<u64>(1024, cdiv(ne5, PB_T));
                            const u64 tile = (ne5 + ntile - 1) / ntile;
                            k_pb_init<<<cdiv(nbk, 256), 256, 0, st>>>(cursor, nbk);
                            k_pb_move<<<ntile, PB_T, 0, st>>>(svals, skeys, ne5, tile, nbk, cursor, tmp);
                            k_pb_apply<<<cdiv(cdiv(ne5, 256), N_XCD) * N_XCD, 256, 0, st>>>(tmp, ne5, pred5);
                        }
                    }
                }
            }
            lap("base sort + pred");
            if (dense) {
                u32* dstart = g_dstart.get((u64)D + 1);
                if (ne5 >= pred_sorted_min && !ls)
                    k_dense_heads<<<cdiv(cdiv(ne5 + 1, 4), 256), 256, 0, st>>>(skeys, ne5, D, dstart);
                k_bstart_rank<<<cdiv(cdiv((u64)nslots + 1, 4), 256), 256, 0, st>>>(pbm, pwp, dstart, nslots, D,
                                                                          g_bstart.get((u64)nslots + 1));
            } else {
                build_buckets(key_u32{skeys}, ne5, g_bstart);
            }
            W.istart = ist.p; W.iend = iend.p; W.irank = irank.p; W.nint = ni;
            W.keys = keys; W.skeys = skeys; W.svals = svals; W.pred5 = pred5; W.ipos = ipos; W.nentries = ne5;
            W.bstart = g_bstart.p;
            W.rem = rem; W.akeys = nullptr; W.nadd = 0; W.akeys2 = nullptr; W.nadd2 = 0;
            // removed flags packed into the positions (the flag bit is above every position)
            W.iposr = (W.use_pred && (u64)N < (u64)POS_RFLAG && !std::getenv("LZ77SSS_NO_IPOSR"))
                          ? iposr_buf.get(nb + 1) : nullptr;
            lap("base buckets");
        };
        // added entries: positions of I outside the base set.  The main list is
        // rebuilt rarely (membership of its positions is read from the I bitmap);
        // positions that join later and are missing from it go to the small extra list.
        u32* bmA = g_bmA.get(nw);
        u64 na_main = 0;
        bool bmA_zero = false;  // the main list is empty and bmA was not computed (I within the base set)
        // I_fresh: I was set by set_state(true) and not changed since (I lies within the base set), so
        // I' == I is decided by two checks over the chain's inserts and the base ranks (i_cnt[0]:
        // inserts outside I, i_cnt[1]: positions of I not inserted) instead of a full-length xor and count
        bool I_fresh = false;
        u32* i_cnt = counters.get(16) + 12;
        auto build_list = [&](const u32* bm, dbuf<u32>& k32, dbuf<pos_t>& kpos, dbuf<u64>& ka, dbuf<u64>& kb,
                              dbuf<u32>& bucket, const u64*& keys_out, u64& nkeys, const u32*& bk_out,
                              const pos_t*& apos_out, u64& napos_out) -> u64 {
            u32 ni, nch;
            u64 na;
            ichunk* ch = runs_to_chunks(bm, g_ast, g_aen, g_ark, chunk_buf2, ni, na, nch);
            nkeys = 0;
            keys_out = nullptr;
            apos_out = nullptr;
            napos_out = 0;
            if (!na) return 0;
            u32* akey32 = k32.get(5 * na);
            pos_t* apos = kpos.get(na);
            apos_out = apos;
            napos_out = na;
            k_slots<<<cdiv(nch, SL_CH), SL_T, 0, st>>>(T, G, ch, nch, akey32, nullptr, apos);
            u64* ak = ka.get(5 * na);
            u64* ak2 = kb.get(5 * na);
            k_pack_added<<<cdiv(5 * na, 256), 256, 0, st>>>(akey32, apos, 5 * na, ak);
            size_t tb = 0;
            LZ_HIP(rocprim::radix_sort_keys(nullptr, tb, ak, ak2, (size_t)(5 * na), 0u, 63u, st));
            u8* t = scan_tmp.get(tb);
            LZ_HIP(rocprim::radix_sort_keys(t, tb, ak, ak2, (size_t)(5 * na), 0u, 63u, st));
            keys_out = ak2;
            nkeys = 5 * na;
            build_buckets(key_u64{ak2}, 5 * na, bucket);
            bk_out = bucket.p;
            return na;
        };
        auto rebuild_main = [&]() {
            bmA_zero = false;
            k_bm_andnot<<<gw, 256, 0, st>>>(bmI, bmIb, nw, bmA);
            na_main = build_list(bmA, add_keys32, add_pos, add_keys, add_keys2, g_abeg, W.akeys, W.nadd, W.abeg, W.apos,
                                 W.napos);
            W.nadd2 = 0;
            W.akeys2 = nullptr;
        };
        auto rebuild_added = [&](bool main_list) {
            if (main_list) return rebuild_main();
            k_bm_andnot<<<gw, 256, 0, st>>>(bmI, bmIb, nw, bmT);
            if (!bmA_zero) k_bm_andnot<<<gw, 256, 0, st>>>(bmT, bmA, nw, bmT);
            const u64 nx = build_list(bmT, g_x32, g_xpos, g_xk, g_xk2, g_abeg2, W.akeys2, W.nadd2, W.abeg2, W.apos2,
                                      W.napos2);
            if (nx * 4 > na_main + (1u << 16)) rebuild_main();
        };
        // rem + added for the current I; within_base: I is a subset of the base set (the first
        // speculation, or a base rebuilt as I' u I_b), so no position is added and the main list
        // (I - I_b, a full-length bitmap pass and a count) is empty without computing it
        auto set_state = [&](bool within_base) {
            W.bmI = bmI;
            I_fresh = within_base;
            if (nb)
                k_rem_from_bm<<<cdiv(nb, 256), 256, 0, st>>>(W.ipos, nb, bmI, off, (u8*)W.rem, (pos_t*)W.iposr);
            if (!within_base) return rebuild_added(true);
            bmA_zero = true;
            na_main = 0;
            W.akeys = nullptr; W.nadd = 0; W.abeg = nullptr; W.apos = nullptr; W.napos = 0;
            W.akeys2 = nullptr; W.nadd2 = 0;
        };
        // same-slot predecessors (pred5) pay for their scatter when the walks make many
        // lookups: short gaps (many factors per gap position).  Texts with few, long gaps
        // (long factors, few lookups) search the buckets instead.  LZ77SSS_PRED /
        // LZ77SSS_NO_PRED force either path (tests).
        W.use_pred = std::getenv("LZ77SSS_PRED") ? 1
                     : std::getenv("LZ77SSS_NO_PRED") ? 0
                     : ((u64)(N - len_lpf_phr) < 4096ull * (u64)std::max<u64>(1, num_gaps)) ? 1 : 0;

        // ---- walk + link until the chain from the window entry is complete, then check I
        u32 nseg = nseg_init;
        u32* ids = g_ids.get(cap);
        u32* d_cnt = counters.get(16);
        chain_status cs{};
        chain_status* d_cs = (chain_status*)g_cs.get(sizeof(chain_status));
        jump_levels JL{};
        u64 wfact = 0, walked_total = 0;
        int outer = 0, rounds_total = 0;
        if (max_outer == 0) {
            wfact = seq_complete(nullptr, 0, nullptr, nullptr, true);
        } else {
            build_base(bmIb);  // superset: gaps + short phrase interiors
            set_state(true);
            bool restart_seq = false;  // a walk overflowed or linking ran away: complete from the entry
            for (;; outer++) {
                for (int round = 0;; round++) {
                    rounds_total++;
                    if (round > 100000) { restart_seq = true; break; }
                    LZ_HIP(hipMemsetAsync(d_cnt, 0, 4, st));
                    k_todo<<<cdiv(nseg, 256), 256, 0, st>>>(S, nseg, ids, d_cnt);
                    const u32 ntodo = rd1(d_cnt, st);
                    const u32* wids = ids;
                    if (ntodo >= (1u << 16)) {  // sort the walks by expected length: less divergence per wave
                        u32* wk = g_wk.get(2ull * ntodo);
                        u32* ids2 = g_ids2.get(ntodo);
                        k_walk_keys<<<cdiv(ntodo, 256), 256, 0, st>>>(S, ids, ntodo, wk);
                        size_t tb = 0;
                        LZ_HIP(rocprim::radix_sort_pairs_desc(nullptr, tb, wk, wk + ntodo, ids, ids2, (size_t)ntodo, 0u,
                                                              32u, st));
                        u8* t = scan_tmp.get(tb);
                        LZ_HIP(rocprim::radix_sort_pairs_desc(t, tb, wk, wk + ntodo, ids, ids2, (size_t)ntodo, 0u, 32u,
                                                              st));
                        wids = ids2;
                    }
                    if (ntodo) {
                        k_walk<false><<<cdiv(ntodo, 64), 64, 0, st>>>(W, S, wids, ntodo, nullptr, nullptr);
                        LZ_HIP(hipGetLastError());
                        walked_total += ntodo;
                    }
                    lap("walk");
                    for (;;) {  // link; grow the table when full
                        k_link<<<cdiv(nseg, 256), 256, 0, st>>>(S, nseg);
                        u32 h2[2];
                        {
                            hread rb(st);
                            rb.add(h2, (const u32*)S.nseg, 2);
                            rb.sync();
                        }
                        if (!(h2[1] & 1)) { nseg = h2[0]; break; }
                        const u32 ncap = cap * 2;
                        g_sin.grow_keep(ncap, cap, st); g_sout.grow_keep(ncap, cap, st);
                        g_stash.grow_keep((u64)ncap * 2 * STASH_CAP, (u64)cap * 2 * STASH_CAP, st);
                        g_valid.grow_keep(ncap, cap, st); g_succ.grow_keep(ncap, cap, st);
                        g_ids.get(ncap);
                        ids = g_ids.p;
                        cap = ncap;
                        bind_tab();
                        const u32 fix[2] = {cap < h2[0] ? cap : h2[0], h2[1] & ~1u};
                        LZ_HIP(hipMemcpyAsync(S.nseg, fix, 8, hipMemcpyHostToDevice, st));
                        LZ_HIP(hipStreamSynchronize(st));
                    }
                    // pointer doubling along succ from every segment
                    u32* D0 = g_dist[0].get(nseg);
                    u32* D1 = g_dist[1].get(nseg);
                    k_jump0<<<cdiv(nseg, 256), 256, 0, st>>>(S, nseg, jump[0].get(nseg), D0);
                    u32 nlv = 1;
                    while ((1ull << (nlv - 1)) < nseg) {
                        if (nlv + 1 >= (u32)MAX_LV) throw error(-6, "greedy: too many jump levels");
                        if ((1ull << nlv) < nseg) {  // two levels in one launch
                            k_jumpk2<<<cdiv(nseg, 256), 256, 0, st>>>(jump[nlv - 1].p, D0, nseg, jump[nlv].get(nseg),
                                                                      jump[nlv + 1].get(nseg), D1);
                            nlv += 2;
                        } else {
                            k_jumpk<<<cdiv(nseg, 256), 256, 0, st>>>(jump[nlv - 1].p, D0, nseg, jump[nlv].get(nseg),
                                                                     D1);
                            nlv++;
                        }
                        std::swap(D0, D1);
                    }
                    JL.nlv = nlv;
                    for (u32 l = 0; l < nlv; l++) JL.J[l] = jump[l].p;
                    k_chain_status<<<1, 1, 0, st>>>(S, jump[nlv - 1].p, D0, c0, d_cs);
                    {
                        hread rb(st);
                        rb.add(&cs, (const chain_status*)d_cs);
                        rb.sync();
                    }
                    lap("link");
                    if (cs.err & 6) { restart_seq = true; break; }  // 2: LPF-start query overflow, 4: walk guard
                    if (dbg)
                        std::fprintf(stderr,
                                     "[lz77sss-debug] greedy window=%d outer=%d round=%d segs=%u walked=%u chain=%u valid=%u "
                                     "flags=%u\n",
                                     nwin, outer, round, nseg, ntodo, cs.hops + 1, cs.valid, cs.flags);
                    if (cs.valid && ((cs.flags & 1) || cs.next >= bw)) break;
                }
                if (restart_seq) {
                    wfact = seq_complete(nullptr, 0, nullptr, nullptr, true);
                    break;
                }
                // ---- the chain, its factor offsets, the tail
                const bool tail = cs.flags & 1;
                if (tail && !last) {
                    redo = true;
                    break;
                }
                const u32 nall = cs.hops + 1, nchain = nall - (tail ? 1u : 0u);
                u32* chain = g_chain.get(nall + 1);
                k_chain_expand<<<cdiv(nall, 256), 256, 0, st>>>(JL, nall, c0, chain);
                u64* nf = seg_offs.get(nall + 2);
                u64* offs = g_offs.get(nall + 2);
                u64 chain_fact = 0;
                if (nchain) {
                    k_chain_nfact<<<cdiv(nchain, 256), 256, 0, st>>>(S, chain, nchain, nf);
                    chain_fact = excl_scan(nf, offs, nchain, scan_tmp, st);
                }
                u64 tail_count = 0, tail_bound = 0;
                pos_t tail_pairs[16];
                u64 hc[3] = {0, 0, 0};
                if (tail) {
                    seg_in tin;
                    seg_out prev{};
                    {
                        hread rb(st);
                        rb.add(&tin, (const seg_in*)(g_sin.p + cs.term));
                        u32 pg = 0;
                        if (nall >= 2) rb.add(&pg, (const u32*)(chain + nall - 2));
                        rb.sync();
                        if (nall >= 2) {
                            rb.add(&prev, (const seg_out*)(g_sout.p + pg));
                            rb.sync();
                        }
                    }
                    if (nall >= 2) {  // exact chain state entering the tail walk
                        tin.idxpos = prev.idxpos;
                        tin.zmask = prev.zmask;
                    } else {
                        tin.idxpos = entry_in.idxpos;
                        tin.zmask = entry_in.zmask;
                    }
                    if (dbg)
                        std::fprintf(stderr, "[lz77sss-debug] greedy tail entry: start=%llu p=%u idxpos=%llu zmask=%u lim=%llu nall=%u\n",
                                     (unsigned long long)tin.start, tin.p, (unsigned long long)tin.idxpos, tin.zmask,
                                     (unsigned long long)tin.lim, nall);
                    tail_bound = (u64)N - tin.start + 1;
                    pos_t* fo = fact.get(2 * (chain_fact + tail_bound) + 2);
                    u64* d_tc = (u64*)g_tailc.get(4 * sizeof(u64));
                    pos_t* d_tins = tail_ins_buf.get(16);
                    k_tail<<<1, 64, 0, st>>>(W, tin, fo, chain_fact, d_tc, d_tins);
                    LZ_HIP(hipGetLastError());
                    {
                        hread rb(st);
                        rb.add(hc, (const u64*)d_tc, 3);
                        rb.add(tail_pairs, (const pos_t*)d_tins, 16);
                        rb.sync();
                    }
                    if (hc[2]) throw error(-6, "greedy tail: insert overflow or guard tripped");
                    tail_count = hc[0];
                    lap("tail");
                } else {
                    fact.get(2 * chain_fact + 2);
                }
                // ---- the insert set the chain actually produced vs the speculation
                const bool fast = I_fresh && !std::getenv("LZ77SSS_NO_FAST_CHECK");
                // a long gap is walked by one wave: with few chain nodes, the long ranges go to the
                // whole grid instead
                constexpr u32 LNG_CAP = 1024;
                u32* lng = nchain ? (u32*)g_lng.get(2 + 4 * LNG_CAP) : nullptr;
                fills({{bmI2, nw * 4, 0u}, {fast ? i_cnt : nullptr, 8, 0u}, {lng, 8, 0u}});
                if (nchain) {
                    // test knobs: a small list and a short "long" range make the overflow path run
                    const u32 lng_cap = std::min(LNG_CAP, knob_lng_cap);
                    const u32 long_words = knob_long_words;
                    k_chain_inserts<<<capped_grid((u64)nchain * 64, 256), 256, 0, st>>>(S, chain, nchain, hi_ins, off, bmI2,
                                                                                     bmI, fast ? i_cnt : nullptr, long_words,
                                                                                     lng, lng_cap);
                    k_chain_inserts_long<<<1024, 256, 0, st>>>(lng, lng_cap, bmI2, bmI, fast ? i_cnt : nullptr);
                }
                if (tail && hc[1]) {
                    pos_t* d_tins = tail_ins_buf.p;
                    k_set_pairs<<<1, 64, 0, st>>>(d_tins, (u32)hc[1], off, bmI2, bmI, fast ? i_cnt : nullptr);
                }
                bool same = false;
                if (fast) {
                    // I' == I  <=>  no insert outside I  and  every position of I (all base ranks
                    // not removed: I lies within the base set) inserted
                    if (nb) k_subset_check<<<cdiv(nb, 256), 256, 0, st>>>(W.ipos, W.rem, nb, bmI2, off, i_cnt + 1);
                    u32 ic[2];
                    hread rb(st);
                    rb.add(ic, (const u32*)i_cnt, 2);
                    rb.sync();
                    same = ic[0] == 0 && ic[1] == 0;
                    if (dbg)
                        std::fprintf(stderr, "[lz77sss-debug] greedy fast check: inserts outside I=%u, waves with I positions "
                                     "not inserted=%u -> %s\n", ic[0], ic[1], same ? "equal" : "full check");
                }
                u64 ny = 0;
                if (!same) {
                    k_bm_xor<<<gw, 256, 0, st>>>(bmI2, bmI, nw, bmT);
                    ny = bmb_scan(bm_bits{bmT, nullptr}, nw, g_bsum, g_bincl, scan_tmp, st) >> 32;
                }
                lap("insert set");
                if (ny == 0 && dbg && std::getenv("LZ77SSS_DEBUG_JUMP")) {
                    // which phrases the converged chain rolled over (interior in I), by log2 length
                    std::vector<u32> hb(nw);
                    std::vector<pos_t> hp(3 * ((u64)m + 1));
                    LZ_HIP(hipStreamSynchronize(st));
                    LZ_HIP(hipMemcpy(hb.data(), bmI, nw * 4, hipMemcpyDeviceToHost));
                    LZ_HIP(hipMemcpy(hp.data(), P, hp.size() * sizeof(pos_t), hipMemcpyDeviceToHost));
                    u64 tot[2][40] = {}, jmp[2][40] = {}, jpos[2][40] = {};
                    pos_t prev_end = 0;
                    for (u32 k = 0; k < m; k++) {
                        const pos_t b0 = hp[3 * k], b1 = hp[3 * k + 1];
                        const int g = b0 > prev_end ? 1 : 0;
                        prev_end = b1;
                        if (b0 < a || b1 >= hi_ins || b1 - b0 < 4) continue;
                        int lg = 0;
                        while (((pos_t)2 << lg) <= b1 - b0) lg++;
                        const pos_t q = b0 + (b1 - b0) / 2 - off;
                        tot[g][lg]++;
                        if ((hb[q >> 5] >> (q & 31)) & 1) { jmp[g][lg]++; jpos[g][lg] += b1 - b0; }
                    }
                    for (int g = 0; g < 2; g++)
                        for (int lg = 0; lg < 40; lg++)
                            if (tot[g][lg])
                                std::fprintf(stderr, "[lz77sss-debug] jump %s len 2^%d: phrases=%llu rolled=%llu pos=%llu\n",
                                             g ? "after-gap" : "adjacent", lg, (unsigned long long)tot[g][lg],
                                             (unsigned long long)jmp[g][lg], (unsigned long long)jpos[g][lg]);
                }
                if (ny == 0) {
                    // every lookup of the chain was exact: emit the factors
                    if (nchain) {
                        k_walk<true><<<cdiv(nchain, 64), 64, 0, st>>>(W, S, chain, nchain, offs, fact.p);
                        LZ_HIP(hipGetLastError());
                        lap("write");
                    }
                    if (!last) {
                        seg_in* d_ex = (seg_in*)(d_sq + 16);
                        k_exit_state<<<1, 1, 0, st>>>(S, cs.term, d_ex);
                        hread rb(st);
                        rb.add(&exit_in, (const seg_in*)d_ex);
                        k_h_export<<<capped_grid((u64)nchain * 64, 256), 256, 0, st>>>(T, G, S, chain, nchain, Hs);
                        rb.sync();
                    }
                    wfact = chain_fact + tail_count;
                    break;
                }
                if (outer + 1 >= max_outer) {
                    // round budget spent: the chain is exact up to the first changed position
                    LZ_HIP(hipMemsetAsync(d_y0, 0xFF, 8, st));
                    k_first_bit<<<gw, 256, 0, st>>>(bmT, nw, off, d_y0);
                    wfact = seq_complete(chain, nall, offs, bmI2, false);
                    break;
                }
                // positions that joined (flag 1) or left (0) I
                pos_t* d_y = dirty_in.get(ny + 1);
                u8* d_j = (u8*)tmp_greedy2.get(2 * ny + 2);
                k_bmb_write<<<bmb_blocks, BMB_T, 0, st>>>(bm_bits{bmT, nullptr}, nw, g_bincl.p, out_list{d_y, d_j, bmI2},
                                                          off);
                // many positions outside the base set: rebuild it as I' u I_b, re-walk everything
                const u64 outside = bmb_scan(bm_bits{bmI2, bmIb}, nw, g_bsum, g_bincl, scan_tmp, st) >> 32;
                if (outside * 8 > nb) {
                    k_bm_or<<<gw, 256, 0, st>>>(bmI2, bmIb, nw, bmT);
                    std::swap(g_bmI.p, g_bmI2.p), std::swap(g_bmI.cap, g_bmI2.cap);
                    bmI = g_bmI.p;
                    bmI2 = g_bmI2.p;
                    build_base(bmT);
                    set_state(true);
                    k_invalidate_all<<<cdiv(nseg, 256), 256, 0, st>>>(S, nseg);
                    if (dbg) std::fprintf(stderr, "[lz77sss-debug] greedy rebuild: outside=%llu\n", (unsigned long long)outside);
                    continue;
                }
                if (ny > nseg) {
                    // too many changes for dirty tracking to pay off: new state, re-walk everything
                    std::swap(g_bmI.p, g_bmI2.p), std::swap(g_bmI.cap, g_bmI2.cap);
                    bmI = g_bmI.p;
                    bmI2 = g_bmI2.p;
                    set_state(false);
                    k_invalidate_all<<<cdiv(nseg, 256), 256, 0, st>>>(S, nseg);
                    lap("delta (full)");
                    if (dbg)
                        std::fprintf(stderr, "[lz77sss-debug] greedy delta (full): changed=%llu outside=%llu\n",
                                     (unsigned long long)ny, (unsigned long long)outside);
                    continue;
                }
                // dirty = changed positions + their same-slot successors before and after the update
                pos_t* d_d = dirty_out.get(11 * ny + 1);
                LZ_HIP(hipMemcpyAsync(d_d, d_y, ny * sizeof(pos_t), hipMemcpyDeviceToDevice, st));
                k_dirty<<<cdiv(ny, 64), 64, 0, st>>>(W, d_y, ny, d_d + ny);
                k_flip<<<cdiv(ny, 256), 256, 0, st>>>(W, d_y, d_j, ny, (u8*)W.rem, d_j + ny);
                I_fresh = false;
                std::swap(g_bmI.p, g_bmI2.p), std::swap(g_bmI.cap, g_bmI2.cap);
                bmI = g_bmI.p;
                bmI2 = g_bmI2.p;
                LZ_HIP(hipMemsetAsync(d_cnt, 0, 4, st));
                k_sum_u8<<<cdiv(ny, 256), 256, 0, st>>>(d_j + ny, ny, d_cnt);
                W.bmI = bmI;
                if (rd1(d_cnt, st)) rebuild_added(false);
                k_dirty<<<cdiv(ny, 64), 64, 0, st>>>(W, d_y, ny, d_d + 6 * ny);
                pos_t* d_ds = dirty_sorted.get(11 * ny + 1);
                {
                    constexpr unsigned PB = 8 * sizeof(pos_t);
                    size_t tb = 0;
                    LZ_HIP(rocprim::radix_sort_keys(nullptr, tb, d_d, d_ds, (size_t)(11 * ny), 0u, PB, st));
                    u8* t = scan_tmp.get(tb);
                    LZ_HIP(rocprim::radix_sort_keys(t, tb, d_d, d_ds, (size_t)(11 * ny), 0u, PB, st));
                }
                k_stale<<<cdiv(nseg, 256), 256, 0, st>>>(S, nseg, d_ds, 11 * ny);
                lap("delta + dirty");
                if (dbg)
                    std::fprintf(stderr, "[lz77sss-debug] greedy delta: changed=%llu outside=%llu\n", (unsigned long long)ny,
                                 (unsigned long long)outside);
            }
        }
        k_seg_at_clear<<<cdiv(nseg, 256), 256, 0, st>>>(S, nseg);
        seg_at_clean = true;
        if (redo) {
            if (dbg) std::fprintf(stderr, "[lz77sss-debug] greedy window %d reaches the tail region: walked again as the last\n", nwin);
            force_last = true;
            stats[19] = 0;
            stats[23]++;
            continue;
        }
        outer_all += max_outer == 0 ? 0 : outer + 1;
        rounds_all += rounds_total;
        walked_all += walked_total;
        nseg_last = nseg;
        nseg0_all += nseg0;
        nwin++;
        // the window's factors: fact[0, wfact); appended to the stream when there are several windows
        if (carry) {
            pos_t* acc = fact_acc.grow_keep(2 * (total_fact + wfact) + 2, 2 * total_fact, st);
            if (wfact)
                LZ_HIP(hipMemcpyAsync(acc + 2 * total_fact, fact.p, 2 * wfact * sizeof(pos_t), hipMemcpyDeviceToDevice, st));
        }
        total_fact += wfact;
        if (last) {
            entry.start = N;
            break;
        }
        entry = exit_in;
        if (dbg)
            std::fprintf(stderr, "[lz77sss-debug] greedy window %d done: factors=%llu next=%llu\n", nwin - 1,
                         (unsigned long long)wfact, (unsigned long long)entry.start);
        if (entry.start >= target_end) break;
    }
    if (blk) {
        blk->exit_start = entry.start;
        blk->exit_idxpos = entry.idxpos;
        blk->exit_zmask = entry.zmask;
    }
    if (carry) {
        // the stream: fact_acc becomes fact
        std::swap(fact.p, fact_acc.p);
        std::swap(fact.cap, fact_acc.cap);
    }
    stats[12] = outer_all;
    stats[13] = rounds_all;
    stats[14] = stats_fallback_lanes;
    stats[15] = walked_all;
    stats[16] = nseg_last;
    stats[17] = nseg0_all;
    stats[21] = nwin;
    stats[22] = stats_sss_tiles;  // anchor tiles the SSS filter marked (exact Q pass)
    return total_fact;
}

// ---------------------------------------------------------------------------
// speculative blocks of a sharded run, walked as consecutive parts.  spec_begin
// snapshots the carried table part `part` starts from (part 0: the speculated entry table) and
// tracks the entry-table slots its lookups use; spec_resolve compares them, part by part, with the
// true entry table (host or device memory).  A part all of whose used slots agree -- and whose
// predecessors' did -- saw at every lookup the value the true table holds, so its factors, exit
// state and inserts are the true ones.  The carried table becomes the writes of the accepted parts
// over the true entry table: the table the caller re-walks the rest with (or passes on).
void engine::spec_begin(int part, u64 base) {
    LZ_HIP(hipSetDevice(device));
    const u64 m = g_Hs.cap;
    if (!m || !g_Hs.p) throw error(LZ77SSS_EINVAL, "speculative block: no carried table (prepare first)");
    if (part == 0) {
        spec_m = m;
        spec_base = base;
    } else if (!spec_track || part != spec_part + 1 || base != spec_base || m != spec_m) {
        throw error(LZ77SSS_EINVAL, "speculative block: parts must follow each other from part 0");
    }
    const u64 nw = m / 32 + 1;
    // every part keeps a snapshot of the whole carried table: on a pos_t = uint64_t session with a
    // 2^28-slot index that is 2 GiB per part, so the part count is bounded by free HBM (the caller
    // stops speculating on ENOMEM; the parts walked so far stay valid)
    const u64 need = (u64)(part + 1) * m * sizeof(pos_t) + (u64)(part + 1) * nw * 4;
    const u64 have = g_hsave.cap * sizeof(pos_t) + g_hsused.cap * 4;
    if (need > have) {
        size_t fr = 0, tot = 0;
        LZ_HIP(hipMemGetInfo(&fr, &tot));
        if ((u64)fr < need - have + (1ull << 30))
            throw error(LZ77SSS_ENOMEM, "speculative block: no HBM left for another part snapshot");
    }
    pos_t* sv = g_hsave.grow_keep((u64)(part + 1) * m, (u64)part * m, st);
    u32* used = g_hsused.grow_keep((u64)(part + 1) * nw, (u64)part * nw, st);
    LZ_HIP(hipMemcpyAsync(sv + (u64)part * m, g_Hs.p, m * sizeof(pos_t), hipMemcpyDeviceToDevice, st));
    LZ_HIP(hipMemsetAsync(used + (u64)part * nw, 0, nw * 4, st));
    spec_part = part;
    spec_track = true;
}
int engine::spec_resolve(const void* true_tab, u64 bytes, int parts) {
    LZ_HIP(hipSetDevice(device));
    const bool tracked = spec_track && parts > 0;
    spec_track = false;
    const u64 m = bytes / sizeof(pos_t);
    if (!true_tab || !m || m > g_Hs.cap) throw error(LZ77SSS_EINVAL, "speculative block: bad true table");
    if (tracked && (parts > spec_part + 1 || m > spec_m))
        throw error(LZ77SSS_EINVAL, "speculative block: more parts than were walked");
    pos_t* tru = g_htrue.get(m);
    LZ_HIP(hipMemcpyAsync(tru, true_tab, m * sizeof(pos_t), hipMemcpyDefault, st));
    int acc = 0;
    if (tracked) {
        u32* bad = g_specbad.get(4 + 2 * 3 * 8);
        const bool dbg = debug_enabled() || std::getenv("LZ77SSS_SPEC_DEBUG");
        const u32 init[4] = {(u32)parts, dbg ? 0u : 0xFFFFFFFFu, 0, 0};
        LZ_HIP(hipMemcpyAsync(bad, init, 16, hipMemcpyHostToDevice, st));
        k_spec_check<<<cdiv(m, 256), 256, 0, st>>>(g_hsused.p, parts, spec_m / 32 + 1, g_hsave.p, tru, m, bad);
        u32 hb[3];
        LZ_HIP(hipMemcpyAsync(hb, bad, 12, hipMemcpyDeviceToHost, st));
        LZ_HIP(hipStreamSynchronize(st));
        acc = (int)hb[0];
        if (dbg)
            std::fprintf(stderr,
                         "[lz77sss] speculative block at %llu: %u entry-table slots used, %u differ; %d of %d parts "
                         "accepted\n",
                         (unsigned long long)spec_base, hb[1], hb[2], acc, parts);
        if (dbg && hb[2]) {
            u64 ex[24];
            LZ_HIP(hipMemcpy(ex, bad + 4, sizeof(ex), hipMemcpyDeviceToHost));
            for (u32 x = 0; x < std::min<u32>(hb[2], 8); x++)
                std::fprintf(stderr, "[lz77sss]   slot %llu: speculated %lld, true %lld (positions + 1)\n",
                             (unsigned long long)ex[3 * x], (long long)ex[3 * x + 1], (long long)ex[3 * x + 2]);
        }
    }
    if (tracked && acc < parts)  // the table the first rejected part started from
        LZ_HIP(hipMemcpyAsync(g_Hs.p, g_hsave.p + (u64)acc * spec_m, m * sizeof(pos_t), hipMemcpyDeviceToDevice, st));
    if (tracked && acc > 0) k_spec_merge<<<cdiv(m, 256), 256, 0, st>>>(g_Hs.p, tru, m, (pos_t)spec_base);
    else LZ_HIP(hipMemcpyAsync(g_Hs.p, tru, m * sizeof(pos_t), hipMemcpyDeviceToDevice, st));
    LZ_HIP(hipGetLastError());
    LZ_HIP(hipStreamSynchronize(st));
    return acc;
}

}  // namespace LZ_NS
