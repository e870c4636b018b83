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
#include "../include/engine.h"
#include "../include/lce_dev.h"

#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <array>
#include <chrono>
#include <cmath>
#include <cstring>
#include <limits>
#include <random>
#include <unordered_map>

namespace lz {

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
    u32 n, nt;          // text length, start of the tail region
    u32 lens[5];
    u64 base[5];
    u32 thr;            // roll_threshold
    u32 mask;           // slot mask (2^k - 1)
    const u128* negpow; // [5][256]: -(o * b^len) mod P
};

__device__ __forceinline__ u128 kr_roll(u128 fp, u64 b, u128 negpow_out, u32 in) {
    return mod107(fp * b + mod107((u128)in + negpow_out));
}
// Phi_x(T[q..q+len)) mod P by direct evaluation (roll-ins only)
__device__ __forceinline__ u128 kr_direct(const u8* T, u64 q, u32 len, u64 b) {
    u128 fp = 0;
    for (u32 j = 0; j < len; j++) fp = mod107(fp * b + T[q + j]);
    return fp;
}

// ---------------------------------------------------------------------------
// entries: e = 5*rank + (4 - x); entries of one position are generated in the
// order of longest_prev_occ (x = 4 .. 0)
struct ichunk { u32 q0, q1, rank0; };

__global__ void k_slots(const u8* __restrict__ T, gap_cfg G, const ichunk* __restrict__ chunks, u32 nch,
                        u32* __restrict__ keys, u32* __restrict__ vals, u32* __restrict__ ipos) {
    const u64 c = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= nch) return;
    const ichunk ch = chunks[c];
    u128 fp[5];
#pragma unroll
    for (int x = 0; x < 5; x++) fp[x] = kr_direct(T, ch.q0, G.lens[x], G.base[x]);
    for (u32 q = ch.q0; q < ch.q1; q++) {
        const u32 rank = ch.rank0 + (q - ch.q0);
        if (ipos) ipos[rank] = q;
#pragma unroll
        for (int x = 4; x >= 0; x--) {
            const u32 e = 5 * rank + (4 - x);
            keys[e] = (u32)((u64)fp[x] & G.mask);
            if (vals) vals[e] = e;
        }
        if (q + 1 < ch.q1) {
#pragma unroll
            for (int x = 0; x < 5; x++)
                fp[x] = kr_roll(fp[x], G.base[x], G.negpow[x * 256 + T[q]], T[q + G.lens[x]]);
        }
    }
}
// predecessor entry within the same slot (base set)
__global__ void k_pred(const u32* __restrict__ skeys, const u32* __restrict__ svals, u64 m, u32* __restrict__ pred5) {
    const u64 t = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= m) return;
    pred5[svals[t]] = (t > 0 && skeys[t - 1] == skeys[t]) ? svals[t - 1] : NONE;
}
// added entries -> 64-bit keys (slot << 35 | pos << 3 | order)
__global__ void k_pack_added(const u32* __restrict__ keys, const u32* __restrict__ ipos, u64 m, u64* __restrict__ out) {
    const u64 e = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= m) return;
    out[e] = ((u64)keys[e] << 35) | ((u64)ipos[e / 5] << 3) | (e % 5);
}
__global__ void k_set_rem(u8* __restrict__ rem, const u32* __restrict__ ranks, u64 m, u8 v) {
    const u64 k = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (k < m) rem[ranks[k]] = v;
}

// ---------------------------------------------------------------------------
struct walk_ctx {
    const u8* T;
    gap_cfg G;
    const u32* P;        // phrases (beg,end,src) + sentinel
    // base set
    const u32* istart;   // interval starts (sorted)
    const u32* iend;     // interval ends (exclusive)
    const u32* irank;    // rank of istart
    u32 nint;
    const u32* keys;     // slot of entry e (position order)
    const u32* skeys;    // sorted slots
    const u32* svals;    // entry ids in sorted order
    const u32* pred5;    // predecessor entry in the same slot
    const u32* ipos;     // rank -> position
    u64 nentries;
    // delta
    const u8* rem;       // removed base ranks
    const u64* akeys;    // sorted added keys
    u64 nadd;
    lce_view L;
};

__device__ __forceinline__ u32 base_rank(const walk_ctx& W, u32 q, int& hint) {
    if (hint >= 0 && q >= W.istart[hint] && q < W.iend[hint]) return W.irank[hint] + (q - W.istart[hint]);
    u32 lo = 0, hi = W.nint;
    while (lo < hi) {
        const u32 mid = (lo + hi) >> 1;
        if (W.istart[mid] <= q) lo = mid + 1; else hi = mid;
    }
    if (lo == 0) return NONE;
    const u32 k = lo - 1;
    if (q >= W.iend[k]) return NONE;
    hint = (int)k;
    return W.irank[k] + (q - W.istart[k]);
}
__device__ __forceinline__ u32 occ_max(u32 a, u32 b) {
    if (a == NONE) return b;
    if (b == NONE) return a;
    return max(a, b);
}
__device__ __forceinline__ u32 occ_min(u32 a, u32 b) {
    if (a == NONE) return b;
    if (b == NONE) return a;
    return min(a, b);
}
// last base entry strictly before (slot, q, ord) in processing order, skipping removed
__device__ u32 base_last_before(const walk_ctx& W, u32 slot, u32 q, u32 ord) {
    u64 lo = 0, hi = W.nentries;  // first index with key > slot
    while (lo < hi) {
        const u64 mid = (lo + hi) >> 1;
        if (W.skeys[mid] <= slot) lo = mid + 1; else hi = mid;
    }
    const u64 end = lo;
    lo = 0;
    hi = end;  // first index with key >= slot
    while (lo < hi) {
        const u64 mid = (lo + hi) >> 1;
        if (W.skeys[mid] < slot) lo = mid + 1; else hi = mid;
    }
    const u64 beg = lo;
    // within [beg, end) entries are in (position, order) order: first >= (q, ord)
    lo = beg;
    hi = end;
    while (lo < hi) {
        const u64 mid = (lo + hi) >> 1;
        const u32 e = W.svals[mid];
        const u32 pq = W.ipos[e / 5], po = e % 5;
        if (pq < q || (pq == q && po < ord)) lo = mid + 1; else hi = mid;
    }
    for (u64 t = lo; t > beg; t--) {
        const u32 rk = W.svals[t - 1] / 5;
        if (!W.rem[rk] || W.ipos[rk] == q) return W.ipos[rk];
    }
    return NONE;
}
__device__ u32 added_last_before(const walk_ctx& W, u32 slot, u32 q, u32 ord) {
    if (!W.nadd) return NONE;
    const u64 key = ((u64)slot << 35) | ((u64)q << 3) | ord;
    u64 lo = 0, hi = W.nadd;  // first >= key
    while (lo < hi) {
        const u64 mid = (lo + hi) >> 1;
        if (W.akeys[mid] < key) lo = mid + 1; else hi = mid;
    }
    if (lo == 0) return NONE;
    const u64 k = W.akeys[lo - 1];
    if ((k >> 35) != slot) return NONE;
    return (u32)((k >> 3) & 0xFFFFFFFFull);
}
// H[slot of (q,x)] just before longest_prev_occ's advance_and_get_occ<x> at q
__device__ u32 lookup(const walk_ctx& W, u32 q, int x, int& hint) {
    const u32 ord = 4 - x;
    const u32 rk = base_rank(W, q, hint);
    u32 slot, cb;
    if (rk != NONE) {
        const u32 e = 5 * rk + ord;
        slot = W.keys[e];
        u32 p = W.pred5[e];
        while (p != NONE && W.rem[p / 5] && W.ipos[p / 5] != q) p = W.pred5[p];
        cb = p == NONE ? NONE : W.ipos[p / 5];
    } else {
        slot = (u32)((u64)kr_direct(W.T, q, W.G.lens[x], W.G.base[x]) & W.G.mask);
        cb = base_last_before(W, slot, q, ord);
    }
    return occ_max(cb, added_last_before(W, slot, q, ord));
}

// ---------------------------------------------------------------------------
// walks
template <bool WRITE>
__device__ void walk_segment(const walk_ctx& W, seg_in in, seg_out& out, u32* fout) {
    const u8* T = W.T;
    const u32 n = W.G.n, nt = W.G.nt;
    const u32* P = W.P;
    u32 i = in.start, p = in.p, idx = in.idxpos, zm = in.zmask;
    u32 nf = 0, ns = 0, flags = 0, e = in.start, nb = 0;
    bool first_gap = true;
    int hint = -1;
    out.next = n;
    out.nbnd = 0;
    u64 guard = 0;
    const u64 guard_max = 4ull * n + 1024;
    auto emit = [&](u32 src, u32 len) {
        if (WRITE) { fout[2 * nf] = src; fout[2 * nf + 1] = len; }
        nf++;
    };
    auto query = [&](u32 q, u32& fsrc, u32& flen) {
        fsrc = T[q];
        flen = 0;
        for (int x = 4; x >= 0; x--) {
            const u32 occ = lookup(W, q, x, hint);
            if (occ != NONE && occ < q && T[occ] == T[q]) {
                flen = (u32)dev_lce(W.L, occ, q);
                fsrc = occ;
                return;
            }
        }
    };
    for (;;) {
        u32 gap_end = P[3 * p];
        if (i < gap_end) {
            if (idx < i) {
                if (i - idx > W.G.thr) {  // reinit (matters only in the tail region)
                    zm = 0;
                    for (int x = 0; x < 5; x++) zm |= ((u64)i + W.G.lens[x] >= n) ? (1u << x) : 0u;
                }
                idx = i;
            }
            do {
                if (i >= in.lim) {  // chunk boundary reached: stop at the next factor start
                    out.next = i;
                    out.e = i;
                    out.nfact = nf;
                    out.idxpos = idx;
                    out.zmask = zm;
                    out.nsingle = ns;
                    out.flags = flags;
                    out.nbnd = nb;
                    return;
                }
                if (i >= nt) { out.flags = flags | 1; out.nbnd = nb; return; }
                if (++guard > guard_max || i > n) { out.flags = flags | 4; return; }
                if (first_gap && nb < SEG_NBND) out.bnd[nb++] = i;
                u32 fsrc, flen;
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
        const u32 exc = i - gap_end;
        u32 lsrc = P[3 * p + 2] + exc, llen = (P[3 * p + 1] - P[3 * p]) - exc;
        if (idx == i) {
            if (i >= nt) { out.flags = flags | 1; return; }
            u32 fsrc, flen;
            query(i, fsrc, flen);
            idx = i + 1;
            if (ns < 4) out.single[ns] = i; else flags |= 2;
            ns++;
            if (flen > llen) { lsrc = fsrc; llen = flen; }
        }
        emit(lsrc, llen);
        i += llen;
        if (++guard > guard_max || i > n || llen == 0) { out.flags = flags | 4; return; }
        while (P[3 * p + 1] <= i) p++;
        if (i < P[3 * p]) { out.next = i; break; }
    }
    out.e = e;
    out.nfact = nf;
    out.idxpos = idx;
    out.zmask = zm;
    out.nsingle = ns;
    out.flags = flags;
    out.nbnd = nb;
}

template <bool WRITE>
__global__ void k_walk(walk_ctx W, const seg_in* __restrict__ segs, u32 nseg, seg_out* __restrict__ outs,
                       const u64* __restrict__ offs, u32* __restrict__ fact) {
    const u64 t = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= nseg) return;
    seg_out o;
    o.flags = 0;
    o.e = segs[t].start;
    o.nfact = 0;
    o.nsingle = 0;
    walk_segment<WRITE>(W, segs[t], o, WRITE ? fact + 2 * offs[t] : nullptr);
    if (!WRITE) outs[t] = o;
}

// successor insert (next position of the same slot after y) in the current set:
// the only query whose lookup can change when y joins or leaves I
__global__ void k_dirty(walk_ctx W, const u32* __restrict__ ys, u64 m, u32* __restrict__ out) {
    const u64 k = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= m) return;
    const u32 y = ys[k];
#pragma unroll 1
    for (int x = 0; x < 5; x++) {
        const u32 slot = (u32)((u64)kr_direct(W.T, y, W.G.lens[x], W.G.base[x]) & W.G.mask);
        u32 best = NONE;
        u64 lo = 0, hi = W.nentries;  // first entry after (slot, y)
        while (lo < hi) {
            const u64 mid = (lo + hi) >> 1;
            const u32 key = W.skeys[mid];
            const u32 pq = W.ipos[W.svals[mid] / 5];
            if (key < slot || (key == slot && pq <= y)) lo = mid + 1; else hi = mid;
        }
        for (u64 t = lo; t < W.nentries && W.skeys[t] == slot; t++) {
            const u32 rk = W.svals[t] / 5;
            if (!W.rem[rk]) { best = W.ipos[rk]; break; }
        }
        if (W.nadd) {
            const u64 key = ((u64)slot << 35) | ((u64)(y + 1) << 3);
            u64 a = 0, b = W.nadd;
            while (a < b) {
                const u64 mid = (a + b) >> 1;
                if (W.akeys[mid] < key) a = mid + 1; else b = mid;
            }
            if (a < W.nadd && (W.akeys[a] >> 35) == slot) best = occ_min(best, (u32)((W.akeys[a] >> 3) & 0xFFFFFFFFull));
        }
        out[5 * k + x] = best;
    }
}

// incremental delta: y joined (flag 1) or left (flag 0) I; base positions flip
// their removed bit, others are reported as additions to maintain on the host
__global__ void k_flip(walk_ctx W, const u32* __restrict__ ys, const u8* __restrict__ joined, u64 m,
                       u8* __restrict__ rem, u8* __restrict__ in_base) {
    const u64 k = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= m) return;
    int hint = -1;
    const u32 rk = base_rank(W, ys[k], hint);
    in_base[k] = rk != NONE;
    if (rk != NONE) rem[rk] = joined[k] ? 0 : 1;
}
// rem[r] = (base position r is not in I); I given as sorted disjoint intervals
__global__ void k_rem_from_set(const u32* __restrict__ ipos, u64 nb, const u32* __restrict__ ia,
                               const u32* __restrict__ ib, u32 ni, u8* __restrict__ rem) {
    const u64 r = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= nb) return;
    const u32 q = ipos[r];
    u32 lo = 0, hi = ni;
    while (lo < hi) {
        const u32 mid = (lo + hi) >> 1;
        if (ia[mid] <= q) lo = mid + 1; else hi = mid;
    }
    rem[r] = (lo == 0 || q >= ib[lo - 1]) ? 1 : 0;
}
// a walked segment is stale iff a dirty position lies in its covered range
__global__ void k_stale(const u32* __restrict__ lo, const u32* __restrict__ hi, u64 nseg,
                        const u32* __restrict__ dirty, u64 nd, u8* __restrict__ stale) {
    const u64 g = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= nseg) return;
    const u32 a = lo[g], b = hi[g];
    u64 l = 0, h = nd;
    while (l < h) {
        const u64 mid = (l + h) >> 1;
        if (dirty[mid] < a) l = mid + 1; else h = mid;
    }
    stale[g] = (l < nd && dirty[l] <= b) ? 1 : 0;
}

// ---------------------------------------------------------------------------
// exact single-thread walk from a segment start to the end of the text, with
// a local model of the inserts in the tail region (last 64 positions)
struct tail_ins { u32 slot, pos; };
constexpr int TAIL_CAP = 64 * 5 + 8;

__global__ void k_tail(walk_ctx W, seg_in in, u32* __restrict__ fact, u64 off, u64* __restrict__ count_out,
                       u32* __restrict__ ins_out /* [a, b) pairs below the tail region, cap 8 */) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    const u8* T = W.T;
    const u32 n = W.G.n, nt = W.G.nt;
    const u32* P = W.P;
    tail_ins loc[TAIL_CAP];
    int nloc = 0;
    u32 i = in.start, p = in.p, idx = in.idxpos, zm = in.zmask;
    u64 nf = 0;
    int hint = -1;
    u32 nins = 0;
    auto fp_slot = [&](u32 q, int x) -> u32 {
        const u32 len = W.G.lens[x];
        if ((zm >> x & 1) || (u64)len > n) return 0;
        const u64 qq = ((u64)q + len <= n) ? q : n - len;
        return (u32)((u64)kr_direct(T, qq, len, W.G.base[x]) & W.G.mask);
    };
    auto tail_lookup = [&](u32 slot) -> u32 {
        for (int k = nloc - 1; k >= 0; k--)
            if (loc[k].slot == slot) return loc[k].pos;
        // every base / added entry lies below nt
        return occ_max(base_last_before(W, slot, nt, 0), added_last_before(W, slot, nt, 0));
    };
    auto insert = [&](u32 q, u32 slot) {
        if (nloc < TAIL_CAP) loc[nloc++] = {slot, q};
    };
    auto query = [&](u32 q, u32& fsrc, u32& flen) {
        fsrc = T[q];
        flen = 0;
        bool hit = false;
        for (int x = 4; x >= 0; x--) {
            if (q < nt) {
                if (hit) continue;
                const u32 occ = lookup(W, q, x, hint);
                if (occ != NONE && occ < q && T[occ] == T[q]) {
                    flen = (u32)dev_lce(W.L, occ, q);
                    fsrc = occ;
                    hit = true;
                }
            } else if (!hit) {
                const u32 slot = fp_slot(q, x);
                const u32 occ = tail_lookup(slot);
                insert(q, slot);  // advance_and_get_occ always inserts
                if (occ != NONE && occ < q && T[occ] == T[q]) {
                    flen = (u32)dev_lce(W.L, occ, q);
                    fsrc = occ;
                    hit = true;
                }
            } else if ((u64)q + W.G.lens[x] < n) {
                insert(q, fp_slot(q, x));  // advance<x> inserts only if cur_pos + len < n
            }
        }
    };
    auto advance_to = [&](u32 target) {
        for (; idx < target; idx++)
            if (idx >= nt)
                for (int x = 0; x < 5; x++)
                    if ((u64)idx + W.G.lens[x] < n) insert(idx, fp_slot(idx, x));
    };
    auto emit = [&](u32 src, u32 len) {
        fact[2 * (off + nf)] = src;
        fact[2 * (off + nf) + 1] = len;
        nf++;
    };
    auto record = [&](u32 a, u32 b) {
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
        u32 gap_end = P[3 * p];
        if (i < gap_end) {
            if (idx < i) {
                if (i - idx > W.G.thr) {
                    zm = 0;
                    for (int x = 0; x < 5; x++) zm |= ((u64)i + W.G.lens[x] >= n) ? (1u << x) : 0u;
                }
                idx = i;  // roll: fingerprints advance, nothing inserted
            }
            const u32 walk_start = i;
            do {
                u32 fsrc, flen;
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
        const u32 exc = i - gap_end;
        u32 lsrc = P[3 * p + 2] + exc, llen = (P[3 * p + 1] - P[3 * p]) - exc;
        if (idx == i) {
            u32 fsrc, flen;
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

// phrase statistics (approximate/common.cpp:98-157, p = 1)
__global__ void k_phrase_info(const u32* __restrict__ P, u32 m, u32 n, u32* __restrict__ acc) {
    const u64 k = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= m) return;
    const u32 b = P[3 * k], e = P[3 * k + 1];
    atomicAdd(&acc[0], e - b);
    u32 gaps = 0;
    if (k == 0 ? b > 0 : b > P[3 * (k - 1) + 1]) gaps++;
    if (k == m - 1 && e < n) gaps++;
    if (gaps) atomicAdd(&acc[1], gaps);
}

// ---------------------------------------------------------------------------
// host side
struct gap_params_h {
    std::array<u32, 5> patt_lens{};
    u32 roll_threshold = 0;
    u32 log2_size_h = 0;
};

// lz77_sss.hpp:99-122, 425-461 and rolling_hash_index_107.hpp:59-70 (pos_t =
// uint32_t, malloc_count_peak() - malloc_count_current() == 0)
static gap_params_h choose_gap_params(u32 n, u32 num_lpf, u32 len_lpf_phr, u32 num_gaps) {
    static const std::array<std::pair<double, std::array<u32, 5>>, 10> table{{
        {6, {2, 3, 4, 5, 6}}, {8, {2, 3, 4, 6, 8}}, {12, {2, 3, 4, 8, 12}}, {16, {2, 4, 6, 9, 16}},
        {32, {2, 4, 6, 10, 20}}, {64, {2, 4, 7, 12, 28}}, {128, {2, 4, 8, 16, 36}},
        {256, {2, 5, 10, 20, 42}}, {1024, {2, 6, 12, 24, 48}},
        {std::numeric_limits<double>::max(), {2, 8, 16, 32, 64}}}};
    gap_params_h g;
    const u32 len_gaps = n - len_lpf_phr;
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
    const int64_t min_index_size = std::max<u32>(1u << 20, (u32)(n * 0.1)) / sizeof(u32);
    const int64_t max_index_size = (1ll << 30) / (int64_t)sizeof(u32);
    const int64_t target_entries = std::max<int64_t>(0, (int64_t)target - rk_bytes) / (int64_t)sizeof(u32);
    const uint64_t target_size_h = std::min<int64_t>(max_index_size, std::max<int64_t>(min_index_size, target_entries));
    g.log2_size_h = (u8)std::round(std::log2(target_size_h));
    return g;
}

struct interval { u32 a, b; };  // [a, b)
using ivec = std::vector<interval>;

static void normalize(ivec& v) {
    std::sort(v.begin(), v.end(), [](const interval& x, const interval& y) { return x.a < y.a || (x.a == y.a && x.b < y.b); });
    ivec out;
    out.reserve(v.size());
    for (auto& x : v) {
        if (x.b <= x.a) continue;
        if (!out.empty() && x.a <= out.back().b) out.back().b = std::max(out.back().b, x.b);
        else out.push_back(x);
    }
    v.swap(out);
}
static void clip(ivec& v, u32 nt) {
    for (auto& x : v) { x.a = std::min(x.a, nt); x.b = std::min(x.b, nt); }
    normalize(v);
}
// a \ b for normalized interval lists
static ivec subtract(const ivec& a, const ivec& b) {
    ivec out;
    size_t j = 0;
    for (auto x : a) {
        u32 cur = x.a;
        while (j < b.size() && b[j].b <= cur) j++;
        for (size_t k = j; k < b.size() && b[k].a < x.b; k++) {
            if (b[k].a > cur) out.push_back({cur, b[k].a});
            cur = std::max(cur, b[k].b);
            if (cur >= x.b) break;
        }
        if (cur < x.b) out.push_back({cur, x.b});
    }
    return out;
}
static u64 total_len(const ivec& v) {
    u64 t = 0;
    for (auto& x : v) t += x.b - x.a;
    return t;
}

static double now_ms() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

u64 engine::factorize_greedy(const u8* T, u32 rk_seed, int log2_override) {
    const bool dbg = debug_enabled();
    double t_mark = now_ms();
    auto lap = [&](const char* what) {
        if (!dbg) return;
        LZ_HIP(hipStreamSynchronize(st));
        const double t = now_ms();
        std::fprintf(stderr, "[lz77sss-debug]   %-28s %9.3f ms\n", what, t - t_mark);
        t_mark = t;
    };
    const u32 N = (u32)n;
    const u32 m = num_phr;  // phrases; P[m] = sentinel
    u32* P = lpf.get((u64)(m + 1) * 3);
    {
        const u32 sent[3] = {N, N + 1, 0};
        LZ_HIP(hipMemcpyAsync(P + 3 * (u64)m, sent, 12, hipMemcpyHostToDevice, st));
    }
    // ---- phrase statistics -> parameters (lz77_sss.hpp:420-461)
    u32 num_lpf = m, len_lpf_phr = 0, num_gaps = 1;
    if (m > 0) {
        u32* acc = counters.get(16);
        LZ_HIP(hipMemsetAsync(acc, 0, 8, st));
        k_phrase_info<<<cdiv(m, 256), 256, 0, st>>>(P, m, N, acc);
        u32 h[2];
        LZ_HIP(hipMemcpyAsync(h, acc, 8, hipMemcpyDeviceToHost, st));
        LZ_HIP(hipStreamSynchronize(st));
        len_lpf_phr = h[0];
        num_gaps = h[1];
    }
    gap_params_h gp = choose_gap_params(N, num_lpf, len_lpf_phr, num_gaps);
    if (log2_override > 0) gp.log2_size_h = (u32)log2_override;
    // bases: rk_prime::random64(257, 2^20-1) from mt19937_64(rk_seed) (rolling_hash.hpp:127-130)
    std::array<u64, 5> bases;
    {
        std::mt19937_64 g(rk_seed);
        for (int i = 0; i < 5; i++) bases[i] = std::uniform_int_distribution<u64>(257, (1ull << 20) - 1)(g);
    }
    std::vector<u128> negpow(5 * 256);
    for (int x = 0; x < 5; x++) {
        const u128 bp = powmod107_host(bases[x], gp.patt_lens[x]);
        const u128 nbp = (P107 - bp) % P107;
        negpow[x * 256] = 0;
        for (int o = 1; o < 256; o++) negpow[x * 256 + o] = mod107(negpow[x * 256 + o - 1] + nbp);
    }
    u128* d_negpow = (u128*)tmp_greedy.get(5 * 256 * sizeof(u128));
    LZ_HIP(hipMemcpyAsync(d_negpow, negpow.data(), 5 * 256 * sizeof(u128), hipMemcpyHostToDevice, st));

    stats.assign(24, 0);
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

    std::vector<u32> hP((u64)(m + 1) * 3);
    LZ_HIP(hipMemcpyAsync(hP.data(), P, hP.size() * 4, hipMemcpyDeviceToHost, st));
    LZ_HIP(hipStreamSynchronize(st));
    auto first_phrase_after = [&](u32 i) -> u32 {  // smallest k with P[k].end > i
        u32 lo = 0, hi = m;
        while (lo < hi) {
            const u32 mid = (lo + hi) >> 1;
            if (hP[3 * mid + 1] <= i) lo = mid + 1; else hi = mid;
        }
        return lo;
    };
    u32 zmask0 = 0;
    for (int x = 0; x < 5; x++) zmask0 |= (G.lens[x] >= N) ? (1u << x) : 0u;  // reinit(0) at construction

    // ---- segments (flat arrays; ids in creation order)
    // Long gaps are cut into chunks of GAP_CHUNK positions: a segment's gap walk
    // stops at the first factor start at or after the next chunk boundary.  Every
    // gap position is inserted whatever the factor boundaries are, so a chunk
    // walk started at its boundary is exact from the first factor start it
    // shares with the real chain (the chain enters through an alias segment).
    const u32 GAP_CHUNK = std::getenv("LZ77SSS_NO_CHUNK") ? 0xFFFFFFF : 512;
    std::vector<u32> cbv;  // chunk boundaries (sorted)
    std::vector<seg_in> hsegs;
    std::vector<seg_out> houts;
    std::vector<u8> valid;       // output exact for the current lookup state
    std::vector<u32> seg_next;   // cached id of the segment starting at houts.next (NONE = unknown)
    std::unordered_map<u32, u32> seg_at;  // start -> id
    auto add_segment = [&](u32 a) {
        auto it = std::upper_bound(cbv.begin(), cbv.end(), a);
        const u32 lim = it == cbv.end() ? N : *it;
        seg_at[a] = (u32)hsegs.size();
        hsegs.push_back({a, first_phrase_after(a), a, zmask0, lim});
        houts.push_back(seg_out{});
        valid.push_back(0);
        seg_next.push_back(NONE);
    };
    auto find_seg = [&](u32 a) -> u32 {
        auto it = seg_at.find(a);
        return it == seg_at.end() ? NONE : it->second;
    };
    u64 n_alias = 0;
    // segment starting at x: existing, or an alias entering a valid chunk walk at one
    // of its recorded factor starts; NONE otherwise (*blocked: the chunk walk is stale)
    auto resolve = [&](u32 x, bool* blocked) -> u32 {
        u32 g = find_seg(x);
        if (g != NONE) return g;
        auto it = std::upper_bound(cbv.begin(), cbv.end(), x);
        if (it == cbv.begin()) return NONE;
        const u32 c = *(it - 1);
        const u32 gc = find_seg(c);
        if (gc == NONE) return NONE;
        if (!valid[gc]) {
            if (blocked) *blocked = true;
            return NONE;
        }
        const seg_out& oc = houts[gc];
        for (u32 k = 1; k < oc.nbnd; k++) {
            if (oc.bnd[k] != x) continue;
            seg_out oa = oc;
            oa.nfact -= k;
            oa.nbnd = 0;
            add_segment(x);
            g = (u32)hsegs.size() - 1;
            houts[g] = oa;
            valid[g] = 1;
            n_alias++;
            return g;
        }
        return NONE;
    };
    // default segments and I_0 (every gap + the LPF-start query that follows it)
    ivec I;
    {
        u32 prev_end = 0;
        std::vector<u32> starts;
        for (u32 k = 0; k <= m; k++) {
            const u32 b = hP[3 * k], e = hP[3 * k + 1];
            if (prev_end < b) {
                starts.push_back(prev_end);
                if (b - prev_end > 2 * (u64)GAP_CHUNK)
                    for (u32 c = prev_end + GAP_CHUNK; c + GAP_CHUNK / 2 < b; c += GAP_CHUNK) cbv.push_back(c);
                I.push_back({prev_end, std::min(b + 1, N)});
            }
            prev_end = std::max(prev_end, e);
        }
        if (starts.empty() || starts[0] != 0) starts.insert(starts.begin(), 0);  // phrases begin at >= 1
        for (u32 a : starts) add_segment(a);
        for (u32 c : cbv) add_segment(c);
    }
    clip(I, G.nt);
    // base superset: the speculated gaps plus the interiors of short phrases,
    // where walk overruns insert (greedy.cpp:69-78); those start "removed"
    ivec Isup = I;
    for (u32 k = 0; k < m; k++) {
        const u32 b = hP[3 * k], e = hP[3 * k + 1];
        if (e - b <= 48) Isup.push_back({b, e});
    }
    clip(Isup, G.nt);
    lap("greedy setup");

    // ---- base build
    ivec Ib;
    std::vector<u32> h_is, h_ie, h_ir;
    u64 nb = 0, ne = 0;
    walk_ctx W{};
    W.T = T;
    W.G = G;
    W.P = P;
    W.L = view(T);
    auto build_base = [&](const ivec& Inew) {
        Ib = Inew;
        h_is.clear(); h_ie.clear(); h_ir.clear();
        std::vector<ichunk> chunks;
        nb = 0;
        for (auto& iv : Ib) {
            h_is.push_back(iv.a); h_ie.push_back(iv.b); h_ir.push_back((u32)nb);
            for (u32 q = iv.a; q < iv.b; q += 1024)
                chunks.push_back({q, std::min<u32>(iv.b, q + 1024), (u32)(nb + (q - iv.a))});
            nb += iv.b - iv.a;
        }
        if (5 * nb >= (1ull << 32)) throw error(-1, "gap region too large for 32-bit entry ids");
        ne = 5 * nb;
        u32* d_is = ist.get(h_is.size() + 1);
        u32* d_ie = iend.get(h_ie.size() + 1);
        u32* d_ir = irank.get(h_ir.size() + 1);
        if (!h_is.empty()) {
            LZ_HIP(hipMemcpyAsync(d_is, h_is.data(), h_is.size() * 4, hipMemcpyHostToDevice, st));
            LZ_HIP(hipMemcpyAsync(d_ie, h_ie.data(), h_ie.size() * 4, hipMemcpyHostToDevice, st));
            LZ_HIP(hipMemcpyAsync(d_ir, h_ir.data(), h_ir.size() * 4, hipMemcpyHostToDevice, st));
        }
        ichunk* d_ch = (ichunk*)chunk_buf.get(std::max<size_t>(1, chunks.size()) * sizeof(ichunk));
        if (!chunks.empty())
            LZ_HIP(hipMemcpyAsync(d_ch, chunks.data(), chunks.size() * sizeof(ichunk), hipMemcpyHostToDevice, st));
        u32* keys = ekeys.get(ne + 1);
        u32* vals = evals.get(ne + 1);
        u32* skeys = ekeys2.get(ne + 1);
        u32* svals = evals2.get(ne + 1);
        u32* ipos = ipos_buf.get(nb + 1);
        u32* pred5 = occ_buf.get(ne + 1);
        u8* rem = rem_buf.get(nb + 1);
        LZ_HIP(hipMemsetAsync(rem, 0, nb + 1, st));
        if (!chunks.empty()) {
            k_slots<<<cdiv(chunks.size(), 64), 64, 0, st>>>(T, G, d_ch, (u32)chunks.size(), keys, vals, ipos);
            size_t tb = 0;
            LZ_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, keys, skeys, vals, svals, (int)ne, 0,
                                                      (int)gp.log2_size_h, st));
            u8* t = scan_tmp.get(tb);
            LZ_HIP(hipcub::DeviceRadixSort::SortPairs(t, tb, keys, skeys, vals, svals, (int)ne, 0,
                                                      (int)gp.log2_size_h, st));
            k_pred<<<cdiv(ne, 256), 256, 0, st>>>(skeys, svals, ne, pred5);
        }
        W.istart = d_is; W.iend = d_ie; W.irank = d_ir; W.nint = (u32)h_is.size();
        W.keys = keys; W.skeys = skeys; W.svals = svals; W.pred5 = pred5; W.ipos = ipos; W.nentries = ne;
        W.rem = rem; W.akeys = nullptr; W.nadd = 0;
        lap("base build (slots+sort+pred)");
    };
    std::vector<u32> A_pos;  // sorted positions of I outside the base set
    // rebuild the added-entry list from A_pos
    auto rebuild_added = [&]() {
        W.nadd = 0;
        W.akeys = nullptr;
        if (A_pos.empty()) return;
        std::vector<ichunk> chunks;
        u64 na = 0;
        for (size_t k = 0; k < A_pos.size();) {
            size_t j = k + 1;
            while (j < A_pos.size() && A_pos[j] == A_pos[j - 1] + 1 && j - k < 1024) j++;
            chunks.push_back({A_pos[k], A_pos[j - 1] + 1, (u32)na});
            na += j - k;
            k = j;
        }
        ichunk* d_ch = (ichunk*)chunk_buf2.get(chunks.size() * sizeof(ichunk));
        LZ_HIP(hipMemcpyAsync(d_ch, chunks.data(), chunks.size() * sizeof(ichunk), hipMemcpyHostToDevice, st));
        u32* akey32 = add_keys32.get(5 * na);
        u32* apos = add_pos.get(na);
        k_slots<<<cdiv(chunks.size(), 64), 64, 0, st>>>(T, G, d_ch, (u32)chunks.size(), akey32, nullptr, apos);
        u64* ak = add_keys.get(5 * na);
        u64* ak2 = add_keys2.get(5 * na);
        k_pack_added<<<cdiv(5 * na, 256), 256, 0, st>>>(akey32, apos, 5 * na, ak);
        size_t tb = 0;
        LZ_HIP(hipcub::DeviceRadixSort::SortKeys(nullptr, tb, ak, ak2, (int)(5 * na), 0, 63, st));
        u8* t = scan_tmp.get(tb);
        LZ_HIP(hipcub::DeviceRadixSort::SortKeys(t, tb, ak, ak2, (int)(5 * na), 0, 63, st));
        W.akeys = ak2;
        W.nadd = 5 * na;
    };
    // full state for I (I must be a subset of the base set here)
    auto set_state = [&](const ivec& Iset) {
        std::vector<u32> ia(Iset.size()), ib(Iset.size());
        for (size_t k = 0; k < Iset.size(); k++) { ia[k] = Iset[k].a; ib[k] = Iset[k].b; }
        u32* d_a = dirty_in.get(ia.size() + 1);
        u32* d_b = dirty_out.get(ib.size() + 1);
        if (!ia.empty()) {
            LZ_HIP(hipMemcpyAsync(d_a, ia.data(), ia.size() * 4, hipMemcpyHostToDevice, st));
            LZ_HIP(hipMemcpyAsync(d_b, ib.data(), ib.size() * 4, hipMemcpyHostToDevice, st));
        }
        if (nb) k_rem_from_set<<<cdiv(nb, 256), 256, 0, st>>>(W.ipos, nb, d_a, d_b, (u32)ia.size(), (u8*)W.rem);
        A_pos.clear();
        rebuild_added();
        LZ_HIP(hipStreamSynchronize(st));
    };

    build_base(Isup);
    set_state(I);
    std::vector<seg_in> tin;
    std::vector<seg_out> tout;
    auto walk_ids = [&](const std::vector<u32>& ids) {
        if (ids.empty()) return;
        tin.resize(ids.size());
        for (size_t t = 0; t < ids.size(); t++) tin[t] = hsegs[ids[t]];
        seg_in* ds = seg_in_buf.get(ids.size());
        seg_out* dout = seg_out_buf.get(ids.size());
        LZ_HIP(hipMemcpyAsync(ds, tin.data(), tin.size() * sizeof(seg_in), hipMemcpyHostToDevice, st));
        k_walk<false><<<cdiv(ids.size(), 64), 64, 0, st>>>(W, ds, (u32)ids.size(), dout, nullptr, nullptr);
        LZ_HIP(hipGetLastError());
        tout.resize(ids.size());
        LZ_HIP(hipMemcpyAsync(tout.data(), dout, tout.size() * sizeof(seg_out), hipMemcpyDeviceToHost, st));
        LZ_HIP(hipStreamSynchronize(st));
        for (size_t t = 0; t < ids.size(); t++) {
            const u32 g = ids[t];
            houts[g] = tout[t];
            valid[g] = 1;
            seg_next[g] = NONE;
            if (houts[g].flags & 2) throw error(-6, "greedy: too many LPF-start queries in one segment");
            if (houts[g].flags & 4) throw error(-6, "greedy: walk guard tripped (internal error)");
        }
    };

    std::vector<u32> chain;
    bool tail_reached = false;
    std::vector<u32> todo;
    for (u32 g = 0; g < hsegs.size(); g++) todo.push_back(g);
    u64 total_fact = 0;
    int outer = 0, rounds_total = 0;
    u64 walked_total = 0;
    for (;; outer++) {
        if (outer > 500) throw error(-6, "greedy speculation did not converge");
        // ---- walk + link until the chain from position 0 is complete and exact
        for (int round = 0;; round++) {
            rounds_total++;
            if (round > 100000) throw error(-6, "greedy segment linking did not converge");
            walk_ids(todo);
            walked_total += todo.size();
            lap("walk");
            todo.clear();
            chain.clear();
            tail_reached = false;
            u32 g = find_seg(0);
            u32 idxp = 0, zm = zmask0;
            bool complete = true;
            for (;;) {
                if (chain.size() > hsegs.size()) throw error(-6, "greedy: segment chain has a cycle");
                if (!valid[g]) { todo.push_back(g); complete = false; break; }
                chain.push_back(g);
                hsegs[g].idxpos = idxp;  // exact inputs of chain segments (used by the tail walk)
                hsegs[g].zmask = zm;
                const seg_out& o = houts[g];
                if (o.flags & 1) { tail_reached = true; break; }
                if (o.next >= N) break;
                idxp = o.idxpos;
                zm = o.zmask;
                u32 nx = seg_next[g];
                if (nx == NONE) {
                    bool blocked = false;
                    nx = resolve(o.next, &blocked);
                    seg_next[g] = nx;
                    if (blocked) todo.push_back(g);  // a stale chunk walk: re-walk the invalid ones
                }
                if (nx == NONE) { complete = false; break; }
                g = nx;
            }
            lap("link");
            if (dbg)
                std::fprintf(stderr,
                             "[lz77sss-debug] greedy outer=%d round=%d segs=%zu chain=%zu complete=%d tail=%d |I|=%llu "
                             "adds=%llu rems=%zu\n",
                             outer, round, hsegs.size(), chain.size(), (int)complete, (int)tail_reached,
                             (unsigned long long)total_len(I), (unsigned long long)(W.nadd / 5), A_pos.size());
            if (complete) break;
            if (!todo.empty()) {
                // batch: re-walk every stale segment, not only the one the link stopped at
                todo.clear();
                for (u32 h = 0; h < hsegs.size(); h++)
                    if (!valid[h]) todo.push_back(h);
                continue;
            }
            // speculatively create every unknown next state of current segments
            std::vector<u32> fresh;
            for (u32 h = 0; h < houts.size(); h++) {
                if (!valid[h]) continue;
                const seg_out& o = houts[h];
                if ((o.flags & 1) || o.next >= N || seg_next[h] != NONE) continue;
                bool blocked = false;
                if (resolve(o.next, &blocked) != NONE || blocked) continue;
                fresh.push_back(o.next);
            }
            std::sort(fresh.begin(), fresh.end());
            fresh.erase(std::unique(fresh.begin(), fresh.end()), fresh.end());
            if (fresh.empty()) throw error(-6, "greedy: chain broken without new states");
            for (u32 a : fresh) {
                todo.push_back((u32)hsegs.size());
                add_segment(a);
            }
        }
        // ---- tail: exact single-thread walk from the chain segment that enters the tail region
        u64 tail_count = 0;
        ivec tail_ins;
        u64 chain_fact = 0;
        const size_t nchain = chain.size() - (tail_reached ? 1 : 0);
        for (size_t c = 0; c < nchain; c++) chain_fact += houts[chain[c]].nfact;
        const u64 tail_bound = tail_reached ? (u64)N - hsegs[chain.back()].start + 1 : 0;
        u32* fo = fact.get(2 * (chain_fact + tail_bound) + 2);
        if (tail_reached) {
            u64* d_cnt = counters64.get(4);
            u32* d_tins = tail_ins_buf.get(16);
            k_tail<<<1, 64, 0, st>>>(W, hsegs[chain.back()], fo, chain_fact, d_cnt, d_tins);
            LZ_HIP(hipGetLastError());
            u64 hc[3];
            u32 hti[16];
            LZ_HIP(hipMemcpyAsync(hc, d_cnt, 24, hipMemcpyDeviceToHost, st));
            LZ_HIP(hipMemcpyAsync(hti, d_tins, 64, hipMemcpyDeviceToHost, st));
            LZ_HIP(hipStreamSynchronize(st));
            if (hc[2]) throw error(-6, "greedy tail: insert overflow or guard tripped");
            tail_count = hc[0];
            for (u64 k = 0; k < hc[1]; k++) tail_ins.push_back({hti[2 * k], hti[2 * k + 1]});
            lap("tail");
        }
        // ---- the insert set the chain actually produced
        ivec I2 = tail_ins;
        I2.reserve(tail_ins.size() + 2 * nchain);
        for (size_t c = 0; c < nchain; c++) {
            const seg_in& si = hsegs[chain[c]];
            const seg_out& o = houts[chain[c]];
            I2.push_back({si.start, o.e});
            for (u32 k = 0; k < o.nsingle && k < 4; k++) I2.push_back({o.single[k], o.single[k] + 1});
        }
        clip(I2, G.nt);
        bool same = I2.size() == I.size();
        for (size_t k = 0; same && k < I.size(); k++) same = I2[k].a == I[k].a && I2[k].b == I[k].b;
        lap("insert set");
        if (same) {
            // ---- every lookup of the chain was exact: emit the factors
            if (nchain) {
                std::vector<u64> offs(nchain);
                std::vector<seg_in> cin(nchain);
                u64 o = 0;
                for (size_t c = 0; c < nchain; c++) { offs[c] = o; o += houts[chain[c]].nfact; cin[c] = hsegs[chain[c]]; }
                u64* doffs = seg_offs.get(nchain);
                seg_in* ds = seg_in_buf.get(nchain);
                LZ_HIP(hipMemcpyAsync(ds, cin.data(), nchain * sizeof(seg_in), hipMemcpyHostToDevice, st));
                LZ_HIP(hipMemcpyAsync(doffs, offs.data(), nchain * 8, hipMemcpyHostToDevice, st));
                k_walk<true><<<cdiv(nchain, 64), 64, 0, st>>>(W, ds, (u32)nchain, nullptr, doffs, fo);
                LZ_HIP(hipGetLastError());
                lap("write");
            }
            total_fact = chain_fact + tail_count;
            break;
        }
        // ---- I changed: the positions that joined (1) or left (0) it
        const ivec joined_iv = subtract(I2, I), left_iv = subtract(I, I2);
        std::vector<u32> ys;
        std::vector<u8> yj;
        for (auto& iv : joined_iv)
            for (u32 q = iv.a; q < iv.b; q++) { ys.push_back(q); yj.push_back(1); }
        for (auto& iv : left_iv)
            for (u32 q = iv.a; q < iv.b; q++) { ys.push_back(q); yj.push_back(0); }
        I.swap(I2);
        const u64 outside = total_len(subtract(I, Ib));
        if (outside * 50 > nb) {
            // many positions outside the base set: rebuild it as I u I_b, re-walk everything
            ivec Inew = I;
            Inew.insert(Inew.end(), Ib.begin(), Ib.end());
            normalize(Inew);
            build_base(Inew);
            set_state(I);
            std::fill(valid.begin(), valid.end(), 0);
            todo.clear();
            for (u32 g = 0; g < hsegs.size(); g++) todo.push_back(g);
            if (dbg) std::fprintf(stderr, "[lz77sss-debug] greedy rebuild: outside=%llu\n", (unsigned long long)outside);
            continue;
        }
        // dirty = changed positions + their same-slot successors before and after the update
        const u64 ny = ys.size();
        u32* d_y = dirty_in.get(ny + 1);
        u8* d_j = (u8*)tmp_greedy2.get(2 * ny + 2);
        u32* d_d = dirty_out.get(11 * ny + 1);
        LZ_HIP(hipMemcpyAsync(d_y, ys.data(), ny * 4, hipMemcpyHostToDevice, st));
        LZ_HIP(hipMemcpyAsync(d_j, yj.data(), ny, hipMemcpyHostToDevice, st));
        LZ_HIP(hipMemcpyAsync(d_d, d_y, ny * 4, hipMemcpyDeviceToDevice, st));
        k_dirty<<<cdiv(ny, 64), 64, 0, st>>>(W, d_y, ny, d_d + ny);
        k_flip<<<cdiv(ny, 256), 256, 0, st>>>(W, d_y, d_j, ny, (u8*)W.rem, d_j + ny);
        std::vector<u8> inb(ny);
        LZ_HIP(hipMemcpyAsync(inb.data(), d_j + ny, ny, hipMemcpyDeviceToHost, st));
        LZ_HIP(hipStreamSynchronize(st));
        bool a_changed = false;
        {
            std::vector<u32> add, del;
            for (u64 k = 0; k < ny; k++)
                if (!inb[k]) (yj[k] ? add : del).push_back(ys[k]);
            if (!add.empty() || !del.empty()) {
                a_changed = true;
                std::sort(add.begin(), add.end());
                std::sort(del.begin(), del.end());
                std::vector<u32> tmp;
                std::set_difference(A_pos.begin(), A_pos.end(), del.begin(), del.end(), std::back_inserter(tmp));
                A_pos.clear();
                std::merge(tmp.begin(), tmp.end(), add.begin(), add.end(), std::back_inserter(A_pos));
            }
        }
        if (a_changed) rebuild_added();
        k_dirty<<<cdiv(ny, 64), 64, 0, st>>>(W, d_y, ny, d_d + 6 * ny);
        // sort dirty positions (NONE entries sort last and are ignored)
        u32* d_ds = dirty_sorted.get(11 * ny + 1);
        {
            size_t tb = 0;
            LZ_HIP(hipcub::DeviceRadixSort::SortKeys(nullptr, tb, d_d, d_ds, (int)(11 * ny), 0, 32, st));
            u8* t = scan_tmp.get(tb);
            LZ_HIP(hipcub::DeviceRadixSort::SortKeys(t, tb, d_d, d_ds, (int)(11 * ny), 0, 32, st));
        }
        // staleness of every walked segment
        const u64 ns = hsegs.size();
        std::vector<u32> lo(ns), hi(ns);
        for (u64 g = 0; g < ns; g++) {
            lo[g] = hsegs[g].start;
            hi[g] = (houts[g].flags & 1) ? N : std::max(houts[g].next, houts[g].e + 1);
        }
        u32* d_lo = seg_lo.get(ns);
        u32* d_hi = seg_hi.get(ns);
        u8* d_st = (u8*)tmp_greedy3.get(ns);
        LZ_HIP(hipMemcpyAsync(d_lo, lo.data(), ns * 4, hipMemcpyHostToDevice, st));
        LZ_HIP(hipMemcpyAsync(d_hi, hi.data(), ns * 4, hipMemcpyHostToDevice, st));
        k_stale<<<cdiv(ns, 256), 256, 0, st>>>(d_lo, d_hi, ns, d_ds, 11 * ny, d_st);
        std::vector<u8> stale(ns);
        LZ_HIP(hipMemcpyAsync(stale.data(), d_st, ns, hipMemcpyDeviceToHost, st));
        LZ_HIP(hipStreamSynchronize(st));
        todo.clear();
        for (u64 g = 0; g < ns; g++) {
            if (stale[g]) valid[g] = 0;
            if (!valid[g]) todo.push_back((u32)g);
        }
        lap("delta + dirty");
        if (dbg)
            std::fprintf(stderr, "[lz77sss-debug] greedy delta: changed=%llu outside=%zu rewalk=%zu\n",
                         (unsigned long long)ny, A_pos.size(), todo.size());
    }
    stats[12] = outer + 1;
    stats[13] = rounds_total;
    stats[14] = stats_fallback_lanes;
    stats[15] = walked_total;
    stats[16] = n_alias;
    stats[17] = cbv.size();
    return total_fact;
}

}  // namespace lz
