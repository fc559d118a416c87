// sh_stack.hip — arrival-order stack engine for partitioned
//   every e1=S[f1] -> e2=S[x.a op e1.a] within W          (C2)
//
// StreamPreStateProcessor.java:325-403 (break-early expiry, then processAndReturn
// over the pending list in creation order) with `every` on the start state makes
// every partial independent: partial i (an event passing f1) is consumed by the
// first later event q of its key with x_q op y_i (y_i = the same attribute of i),
// unless ts_q - ts_i > W expired it first. When the ordering term compares one
// attribute with itself, a key's pending partials form a monotone stack: a
// consumer pops exactly the entries it beats, which sit on top (for `>` the stack
// is non-increasing from the bottom up: every survivor of q is >= x_q = y_q and q
// is pushed on top of them), and expiry drops entries from the bottom (creation
// order is time order). The rows of a consumer are its popped entries in creation
// order. No key sort, no segment, no walk back.
//
// Layout of the work (gfx950: 256 CUs in 8 XCDs, 160 KiB LDS per CU):
//  * the stream is cut into n_chunks arrival chunks; the keys into G = 2, 4 or 8
//    groups (key & (G - 1)); workgroup (chunk, group) runs on one CU with the
//    stacks of its <= SK_KPW keys in LDS (a ring of SK_D entries per key: the
//    ordering value and the timestamp as a 16-bit offset; deeper entries spill to
//    a per-key stack in HBM, touched by ~0.04% of the events on C2). The G
//    workgroups of a chunk sit on one XCD, so the chunk's columns come from HBM
//    once and from that XCD's L2 for the other groups.
//  * a chunk first replays its halo (the events within W before it, found by a
//    parallel search of the timestamps) without output, so its stacks start
//    exact: a partial older than the halo is expired for every event of the chunk.
//  * per sub-tile of 1,024 * EPL arrival events: every wave loads its contiguous
//    64 * EPL events (coalesced rows), keeps its group's events and sends each to
//    the wave that owns its key (local key & 15) through a per-wave LDS queue, in
//    arrival order (ranks from wave ballots and returning LDS atomics; two
//    workgroup barriers per sub-tile). Each wave then processes its queue in
//    batches of 64: the k-th event of a key within the batch runs in round k, so
//    the events of one round touch distinct keys; an event loads its key's whole
//    ring (16 LDS reads issued together), expires, pops and pushes in registers.
//  * pass 1 writes each event's count (u8) and the sub-tile totals (ttot); an
//    exclusive scan turns them into each sub-tile's first row; pass 2 replays the
//    chunk and writes each consumer's rows at sub-tile base + the prefix of the
//    counts before it (the producer waves scan the counts of their rows).
// HBM bytes per event (C2): pass 1 reads ts 8 + key 4 + price 4 and writes the
// count 1; pass 2 reads them again + the count + volume 8 and writes 32 B per row.
#include <hip/hip_runtime.h>
#include <stdlib.h>

#include "../../include/sh_query.h"
#include "sh_device.h"
#include "sh_rows.h"
#include "sh_vm.h"
#include "sh_wave.h"

#define SK_TPB 1024
#define SK_NW (SK_TPB / 64)  // waves: a key's owner wave is its local key & 15
#define SK_D 8               // ring entries per key in LDS
#define SK_KPW 2500          // keys per workgroup at most
#define SK_CAPW 160          // queue entries per owner wave and sub-tile (64 expected)
#define SK_OFF_BITS 13       // q2: event offset in the sub-tile | row offset << 13
#define SK_ROWS_LIM (1u << (32 - SK_OFF_BITS))

static_assert(SK_NW == 16, "16 owner waves");

struct SkLds {
    uint32_t y[SK_D][SK_KPW];         // ring entries: order key of the ordering value
    uint16_t t[SK_D][SK_KPW];         // ... timestamp - tb
    uint16_t h[SK_KPW];               // bottom (3 bits) | count << 3 (4) | spilled << 7 (9)
    uint16_t spt[SK_KPW];             // timestamp of the newest spilled entry
    uint32_t qx[SK_NW * SK_CAPW];     // queue: order key of the ordering value
    uint32_t q1[SK_NW * SK_CAPW];     // ts - tb | wave-local key << 16 | NaN << 30 | open << 31
    uint32_t q2[SK_NW * SK_CAPW];     // offset in the sub-tile | row offset << 13 (pass 2)
    uint32_t wcnt[SK_NW][SK_NW];      // [producer wave][owner wave]: queued events
    uint32_t wrow[SK_NW];             // pass 2: rows of each producer wave's events
    uint32_t wsum[SK_NW];             // pass 1: matches of each owner wave's events
    unsigned long long sa, sz;        // halo search bounds
};
static_assert(sizeof(SkLds) <= 163840, "LDS");

// order keys: a float's IEEE bits (or an int) as an unsigned integer of the same
// order -- positive floats get the sign bit set, negative ones are inverted -- so
// every comparison of the ordering term is one unsigned compare, branch-free
__device__ __forceinline__ uint32_t sk_key(uint32_t bits, bool f32) {
    return f32 ? ((bits & 0x80000000u) ? ~bits : (bits | 0x80000000u)) : (bits ^ 0x80000000u);
}
__device__ __forceinline__ uint32_t sk_unkey(uint32_t k, bool f32) {
    return f32 ? ((k & 0x80000000u) ? (k & 0x7FFFFFFFu) : ~k) : (k ^ 0x80000000u);
}

// the opening filter's fast form: each term compares a 4-byte column (the ordering
// one or the prefetched one) with a constant through order keys
__device__ __forceinline__ bool sk_open_fast(const shk_plan& P, uint32_t x, uint32_t l0) {
    bool ok = true;
    for (int k = 0; k < P.n_terms; k++) {
        const uint32_t v = P.f_col[k] ? l0 : x;
        const bool f = P.f_f32[k] != 0;
        const bool nan = f && (v & 0x7FFFFFFFu) > 0x7F800000u;
        uint32_t kv = sk_key(v, f);
        kv = (f && kv == 0x7FFFFFFFu) ? 0x80000000u : kv;  // -0.0 compares as +0.0
        const uint32_t kc = P.f_ckey[k];
        const bool r = (P.f_lt[k] && kv < kc) || (P.f_eq[k] && kv == kc) || (P.f_gt[k] && kv > kc);
        ok = ok && (nan ? P.f_nan[k] != 0 : r);
    }
    return ok;
}

// the opening filter (f1 and the e1-only terms of f2) on event e, as terms_pass:
// the general form, evaluated by k_stk_open into a bit per event when the terms
// have no fast form (keeps the VM's code out of the matcher)
__device__ __forceinline__ bool sk_open_gen(const shk_plan& P, int64_t e) {
    for (int k = 0; k < P.n_terms; k++) {
        const shp_term T = P.terms[k];
        VmVal l, r;
        l.t = T.ltype;
        l.null = 0;
        l.b = bk_raw(P.tl[k], e, T.ltype);
        if (T.rkind == 1) {
            r.t = T.ctype;
            r.null = 0;
            r.b = T.c;
        } else {
            r.t = T.rtype;
            r.null = 0;
            r.b = bk_raw(P.tr[k], e, T.rtype);
            if (T.rkind == 2) {
                VmVal c;
                c.t = T.ctype;
                c.null = 0;
                c.b = T.c;
                r = vm_arith(T.aop, T.atype, r, c);
                if (r.null) return false;
            }
        }
        if (!vm_cmp(T.op, T.dom, l, r)) return false;
    }
    return true;
}

// one bit per event: the opening filter's general form (64 events per word)
__global__ void __launch_bounds__(256) k_stk_open(shk_plan P) {
    const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const bool ok = e < P.n && sk_open_gen(P, e);
    const uint64_t m = __ballot(ok);
    if ((threadIdx.x & 63) == 0 && e < P.n) const_cast<uint64_t*>(P.omask)[e >> 6] = m;
}

// a key's spilled entries are written by one lane and read back by another lane of
// the same wave in a later round: both sides go to L2 (agent-scope relaxed atomics
// bypass the CU's L1, whose copy of a reused slot would otherwise be stale)
__device__ __forceinline__ uint64_t sk_spill_load(const uint64_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void sk_spill_store(uint64_t* p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// value of a select entry of a row: the consumed partial's ordering value (y) or
// the consumer's attribute (preloaded)
__device__ __forceinline__ int64_t sk_yraw(uint32_t y, int type) {
    return type == SH_T_FLOAT ? (int64_t)y : (int64_t)(int32_t)y;
}

// XCD-aware (chunk, group) of this workgroup: workgroups are dealt round-robin
// to the 8 XCDs, so the G groups of a chunk take consecutive slots of one XCD
__device__ __forceinline__ void sk_place(const shk_plan& P, int* c, int* g) {
    const int xcd = (int)(blockIdx.x & 7u), slot = (int)(blockIdx.x >> 3);
    *c = xcd * P.cpx + (slot >> P.gshift);
    *g = slot & ((1 << P.gshift) - 1);
}

// first event of the halo of a chunk starting at cb: the first index with
// ts >= ts[cb] - W (timestamps are non-decreasing), at most one chunk back
// (else SHB_F_HALO); a 1,024-ary search over the timestamps
__device__ int64_t sk_halo(const shk_plan& P, SkLds& L, int64_t cb) {
    if (cb == 0) return 0;
    const int64_t T = P.ts[cb] - P.within;
    int64_t a = cb - P.chunk < 0 ? 0 : cb - P.chunk;
    if (P.ts[a] >= T) {
        if (a > 0 && threadIdx.x == 0) atomicOr(P.flag, SHB_F_HALO);
        return a;
    }
    int64_t z = cb;  // ts[a] < T <= ts[z]
    while (z - a > 1) {
        const int64_t step = (z - a + SK_TPB - 1) / SK_TPB;
        if (threadIdx.x == 0) {
            L.sa = (unsigned long long)a;
            L.sz = (unsigned long long)z;
        }
        __syncthreads();
        const int64_t p = a + step * (int64_t)(threadIdx.x + 1);
        if (p < z) {
            if (P.ts[p] >= T) atomicMin(&L.sz, (unsigned long long)p);
            else atomicMax(&L.sa, (unsigned long long)p);
        }
        __syncthreads();
        a = (int64_t)L.sa;
        z = (int64_t)L.sz;
        __syncthreads();
    }
    return z;
}

template <int PASS, int EPL, int MODE, int NO>
__global__ void __launch_bounds__(SK_TPB, 1) k_stk(shk_plan P, shb_out O, shb_cols OC, uint64_t seq_base,
                                                  uint64_t* __restrict__ out_seq, int64_t* __restrict__ out_vals,
                                                  int64_t out_cap) {
    __shared__ SkLds L;
    constexpr int SUB = SK_TPB * EPL;
    static_assert(SUB <= (1 << SK_OFF_BITS), "offsets");
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
    int c, g;
    sk_place(P, &c, &g);
    if (c >= P.n_chunks) return;
    const int64_t cb = (int64_t)c * P.chunk;
    const int64_t ce = cb + P.chunk < P.n ? cb + P.chunk : P.n;
    if (cb >= ce) return;
    if (PASS == 2 && __hip_atomic_load(P.flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0)
        return;  // pass 1 refused the run: the host takes another engine
    const int G = 1 << P.gshift;
    int64_t h;
    if (PASS == 1) {
        h = sk_halo(P, L, cb);
        if (g == 0 && threadIdx.x == 0) P.hstart[c] = h;
    } else {
        h = P.hstart[c];
    }
    const int64_t hb = (h / SUB) * SUB;
    const int64_t tb = P.ts[hb];
    for (int i = threadIdx.x; i < P.kpw; i += SK_TPB) L.h[i] = 0;
    const uint32_t W = (uint32_t)P.within;
    const bool f32 = P.dom == DOM_F32;

    // the producer's events of sub-tile s0: row i holds s0 + w * 64 * EPL + 64 i + lane,
    // loaded one sub-tile ahead (with the predecessor of row 0, the prefetched
    // filter operands and, pass 2, the sub-tile's first row)
    int32_t kk[EPL];
    uint32_t xx[EPL];
    int64_t tt[EPL];
    uint32_t cc[EPL];
    uint32_t la[EPL];
    uint64_t om[EPL];
    int64_t tpr = INT64_MIN;
    uint32_t rows_next = 0;
    auto load = [&](int64_t s0) {
        const int64_t e0 = s0 + (int64_t)w * (64 * EPL) + lane;
        tpr = (e0 > hb && e0 - 1 < ce) ? P.ts[e0 - 1] : INT64_MIN;
        if (PASS == 2 && s0 >= cb) rows_next = P.ttot[s0 / SUB];
#pragma unroll
        for (int i = 0; i < EPL; i++) {
            const int64_t e = e0 + 64 * i;
            const bool v = e < ce;
            kk[i] = v ? P.keys[e] : -1;
            xx[i] = v ? ((const uint32_t*)P.xcol)[e] : 0u;
            tt[i] = v ? P.ts[e] : tb;
            cc[i] = (PASS == 2 && v && s0 >= cb) ? (uint32_t)P.cnt[e] : 0u;
            la[i] = (P.pre[0] >= 0 && v) ? ((const uint32_t*)P.tl[P.pre[0]])[e] : 0u;
            om[i] = (P.omask && v) ? P.omask[e >> 6] : 0ull;  // (rows are 64-aligned)
        }
    };
    load(hb);
    unsigned long long pc_prod = 0, pc_queue = 0, pc_proc = 0, pc0 = 0, n_batch = 0, n_round = 0, n_ev = 0;
    int64_t prev_sub = -1;  // pass 1: the last sub-tile whose totals wait in wsum
    for (int64_t s0 = hb; s0 < ce; s0 += SUB) {
        const bool emit = s0 >= cb;
        if (P.prof) pc0 = clock64();
        // ---- producer: own events, their owner wave and rank
        if (lane < SK_NW) L.wcnt[w][lane] = 0u;
        uint32_t rk[EPL], qa[EPL], qb[EPL], qc[EPL];
        int bn[EPL];
        uint32_t rr[EPL];
        uint32_t flag = 0;
        uint32_t rcarry = 0;
#pragma unroll
        for (int i = 0; i < EPL; i++) {
            const int64_t e = s0 + (int64_t)w * (64 * EPL) + 64 * i + lane;
            const bool v = e < ce;
            const int32_t k = kk[i];
            if (v && k >= P.nkeys) flag |= SHB_F_KEY;
            const bool own = v && k >= 0 && k < P.nkeys && (k & (G - 1)) == g;
            const int64_t dt = tt[i] - tb;
            if (v && (dt < 0 || dt > 65535)) flag |= SHB_F_TS;
            {
                // timestamps never go back: the previous event is lane - 1, the last of
                // the previous row, or (row 0, lane 0) the previous wave's last event
                const int64_t up = __shfl(tt[i], lane > 0 ? lane - 1 : 0);
                const int64_t pv = lane > 0 ? up : (i > 0 ? __shfl(tt[i > 0 ? i - 1 : 0], 63) : tpr);
                if (v && pv > tt[i]) flag |= SHB_F_MONO;
            }
            const uint32_t lk = own ? (uint32_t)k >> P.gshift : 0u;
            const int b = (int)(lk & 15u);
            bn[i] = own ? b : -1;
            // a NaN consumer takes nothing and never opens a partial
            const bool xnan = f32 && (xx[i] & 0x7FFFFFFFu) > 0x7F800000u;
            bool open = false;
            if (own && !xnan) {
                if (P.fast_open) open = sk_open_fast(P, xx[i], la[i]);
                else open = (om[i] >> lane) & 1ull;
            }
            qa[i] = sk_key(xx[i], f32) ^ P.kflip;
            qb[i] = (uint32_t)dt | ((lk >> 4) << 16) | (xnan ? 0x40000000u : 0u) | (open ? 0x80000000u : 0u);
            qc[i] = (uint32_t)(e - s0);
            if (PASS == 1 && emit && v && !(k >= 0 && k < P.nkeys) && g == 0) P.cnt[e] = 0;
            // rank among this wave's earlier events of the same owner wave
            uint64_t peers = __ballot(own);
#pragma unroll
            for (int bb = 0; bb < 4; bb++) {
                const bool bit = (b >> bb) & 1;
                const uint64_t m = __ballot(own && bit);
                peers &= bit ? m : ~m;
            }
            const uint32_t r = (uint32_t)__popcll(peers & lt);
            uint32_t old = 0u;
            if (own && r == 0) old = atomicAdd(&L.wcnt[w][b], (uint32_t)__popcll(peers));
            const int ld = own ? (int)__ffsll((unsigned long long)peers) - 1 : lane;
            rk[i] = (uint32_t)__shfl((int)old, ld) + r;
            if (PASS == 2) {
                // rows of the events before this one in the wave's run (arrival order)
                const uint32_t ci = emit ? cc[i] : 0u;
                const uint32_t inc = shw_incl_scan(ci);
                rr[i] = rcarry + inc - ci;
                rcarry += shw_last(inc);
            }
        }
        if (flag) atomicOr(P.flag, (int)flag);
        if (PASS == 2 && lane == 0) L.wrow[w] = rcarry;
        if (P.prof) {
            const unsigned long long t = clock64();
            pc_prod += t - pc0;
            pc0 = t;
        }
        __syncthreads();  // A: queue counts and row totals of the sub-tile are in
        if (PASS == 1 && threadIdx.x == 0 && prev_sub >= 0) {
            uint32_t s = 0;
#pragma unroll
            for (int q = 0; q < SK_NW; q++) s += L.wsum[q];
            if (s) atomicAdd(&P.ttot[prev_sub], s);
        }
        prev_sub = emit ? s0 / SUB : -1;
        // queue positions: owner b's region, after the earlier producer waves' events
        {
            uint32_t pb = 0;
            if (lane < SK_NW)
                for (int q = 0; q < w; q++) pb += L.wcnt[q][lane];
            uint32_t rbase = 0;
            if (PASS == 2)
                for (int q = 0; q < w; q++) rbase += L.wrow[q];
#pragma unroll
            for (int i = 0; i < EPL; i++) {
                const int b = bn[i];
                const uint32_t pos = (uint32_t)__shfl((int)pb, b < 0 ? 0 : b) + rk[i];
                if (b >= 0) {
                    if (pos >= SK_CAPW) {
                        atomicOr(P.flag, SHK_F_QUEUE);
                    } else {
                        const int qi = b * SK_CAPW + (int)pos;
                        L.qx[qi] = qa[i];
                        L.q1[qi] = qb[i];
                        uint32_t q2 = qc[i];
                        if (PASS == 2) {
                            const uint32_t ro = rbase + rr[i];
                            if (ro >= SK_ROWS_LIM) atomicOr(P.flag, SHK_F_ROWS);
                            q2 |= ro << SK_OFF_BITS;
                        }
                        L.q2[qi] = q2;
                    }
                }
            }
        }
        // this wave's queue length (sum over the producer waves)
        uint32_t nq = lane < SK_NW ? L.wcnt[lane][w] : 0u;
        nq = shw_last(shw_incl_scan(nq));
        if (nq > SK_CAPW) nq = SK_CAPW;
        const uint64_t rows0 = (PASS == 2 && emit) ? (uint64_t)rows_next : 0ull;
        __syncthreads();  // B: queues complete
        if (P.prof) {
            const unsigned long long t = clock64();
            pc_queue += t - pc0;
            pc0 = t;
        }
        if (s0 + SUB < ce) load(s0 + SUB);  // next sub-tile in flight during the queue
        // ---- owner: the wave's queue in batches of 64, the k-th event of a key in round k
        uint32_t msum = 0;
        n_ev += nq;
        for (uint32_t base = 0; base < nq; base += 64) {
            const uint32_t idx = base + (uint32_t)lane;
            const bool act = idx < nq;
            const int qi = w * SK_CAPW + (int)(act ? idx : 0u);
            const uint32_t x = L.qx[qi], a1 = L.q1[qi], a2 = L.q2[qi];
            const uint32_t wl = (a1 >> 16) & 0xFFu;
            uint64_t peers = __ballot(act);
#pragma unroll
            for (int bb = 0; bb < 8; bb++) {
                const bool bit = (wl >> bb) & 1u;
                const uint64_t m = __ballot(act && bit);
                peers &= bit ? m : ~m;
            }
            const uint32_t rank = (uint32_t)__popcll(peers & lt);
            const int64_t j = s0 + (int64_t)(a2 & ((1u << SK_OFF_BITS) - 1u));
            const uint32_t lk = (wl << 4) | (uint32_t)w;
            // consumer-side select values, loaded before the rounds
            int64_t v1[NO > 0 ? NO : 1];
            if (PASS == 2 && NO > 0) {
                const int32_t key = (int32_t)((lk << P.gshift) | (uint32_t)g);
#pragma unroll
                for (int o = 0; o < (NO > 0 ? NO : 1); o++) {
                    v1[o] = 0;
                    if (O.kind[o] != 1 || !act || !emit) continue;
                    if (O.src[o] == P.xcol) v1[o] = sk_yraw(sk_unkey(x ^ P.kflip, f32), O.type[o]);
                    else if (O.src[o] == (const void*)P.keys) v1[o] = (int64_t)key;
                    else v1[o] = bk_raw(O.src[o], j, O.type[o]);
                }
            }
            n_batch++;
            for (uint32_t rd = 0; __ballot(act && rank >= rd) != 0ull; rd++) {
                n_round++;
                if (!(act && rank == rd)) continue;
                // the key's ring: all entries at once (one LDS latency)
                const uint32_t hw = L.h[lk];
                uint32_t y[SK_D];
                uint32_t tv[SK_D];
#pragma unroll
                for (int s = 0; s < SK_D; s++) {
                    y[s] = L.y[s][lk];
                    tv[s] = L.t[s][lk];
                }
                uint32_t b = hw & 7u, n = (hw >> 3) & 15u, sc = hw >> 7;
                const uint32_t now = a1 & 0xFFFFu;
                const uint32_t full = n ? ((1u << n) - 1u) : 0u;
                uint32_t live = ((full << b) | (full >> (SK_D - b))) & 0xFFu;
                // expiry from the bottom (creation order is time order)
                uint32_t E = 0;
#pragma unroll
                for (int s = 0; s < SK_D; s++)
                    E |= (((live >> s) & 1u) && ((now - tv[s]) & 0xFFFFu) > W) ? (1u << s) : 0u;
                if (E) {
                    const uint32_t ne = (uint32_t)__popc(E);
                    b = (b + ne) & 7u;
                    n -= ne;
                    live &= ~E;
                    sc = 0;  // spilled entries are older than an expired one
                }
                // the entries x beats: the top of the stack (order keys; -0.0 as +0.0)
                const uint32_t cx = x == P.zk1 ? P.zk0 : x;
                if (a1 & 0x40000000u) live = 0;  // a NaN consumer
                uint32_t K = 0;
#pragma unroll
                for (int s = 0; s < SK_D; s++) {
                    const uint32_t cy = y[s] == P.zk1 ? P.zk0 : y[s];
                    K |= (((live >> s) & 1u) && (cx > cy || (P.ge && cx == cy))) ? (1u << s) : 0u;
                }
                const uint32_t k = (uint32_t)__popc(K);
                n -= k;
                // below an emptied ring: the spilled entries (HBM)
                uint64_t* spl = P.spill + ((uint64_t)blockIdx.x * (uint64_t)P.kpw + lk) * (uint64_t)P.spill_cap;
                uint32_t ks = 0;  // spilled entries popped (rows); `sc` may also drop to 0 by expiry
                uint32_t slo = sc;  // the popped spilled entries are slots [slo, slo + ks)
                if (n == 0 && sc > 0 && !(a1 & 0x40000000u)) {
                    while (sc > 0) {
                        const uint64_t ev = sk_spill_load(spl + sc - 1);
                        if (((now - (uint32_t)(ev >> 32)) & 0xFFFFu) > W) {
                            sc = 0;  // this one and every older spilled entry expired
                            break;
                        }
                        const uint32_t cy = (uint32_t)ev == P.zk1 ? P.zk0 : (uint32_t)ev;
                        if (!(cx > cy || (P.ge && cx == cy))) break;
                        sc--;
                        ks++;
                        slo = sc;
                    }
                }
                const uint32_t total = ks + k;
                if (PASS == 1) {
                    if (emit) {
                        if (total > 255u) atomicOr(P.flag, SHB_F_COUNT);
                        P.cnt[j] = (uint8_t)(total > 255u ? 255u : total);
                        msum += total;
                    }
                } else if (emit && total) {
                    // rows in creation order: the spilled entries, then the ring's
                    const int64_t r0 = (int64_t)rows0 + (int64_t)(a2 >> SK_OFF_BITS);
                    const uint64_t seq = seq_base + (uint64_t)j;
                    const int32_t key = (int32_t)((lk << P.gshift) | (uint32_t)g);
                    auto put = [&](int64_t row, uint32_t yv) {
                        if (row >= out_cap) return;  // the host reports SH_E_MORE
                        if (NO > 0) {
                            int64_t v[NO > 0 ? NO : 1];
#pragma unroll
                            for (int o = 0; o < (NO > 0 ? NO : 1); o++)
                                v[o] = O.kind[o] == SHB_OUT_KIND_Y ? sk_yraw(sk_unkey(yv ^ P.kflip, f32), O.type[o])
                                                                   : v1[o];
                            bk_store<MODE, NO>(OC, row, v, seq, out_seq, out_vals);
                        } else {
                            const int no = O.n_out;
                            if (MODE == SHB_OUT_PACKED) {
                                uint32_t* rp = (uint32_t*)OC.rows + row * OC.rw;
                                rp[0] = (uint32_t)seq;
                                rp[1] = (uint32_t)(seq >> 32);
                                for (int q = 2; q < OC.rw; q++) rp[q] = 0u;
                            } else if (out_seq) {
                                out_seq[row] = seq;
                            }
                            for (int o = 0; o < no; o++) {
                                int64_t vv;
                                if (O.kind[o] == SHB_OUT_KIND_Y) vv = sk_yraw(sk_unkey(yv ^ P.kflip, f32), O.type[o]);
                                else if (O.src[o] == P.xcol) vv = sk_yraw(sk_unkey(x ^ P.kflip, f32), O.type[o]);
                                else if (O.src[o] == (const void*)P.keys) vv = (int64_t)key;
                                else vv = bk_raw(O.src[o], j, O.type[o]);
                                if (MODE == SHB_OUT_PACKED) {
                                    uint32_t* rp = (uint32_t*)OC.rows + row * OC.rw + OC.woff[o];
                                    rp[0] = OC.colw[o] == 1 ? (uint32_t)(uint8_t)vv : (uint32_t)vv;
                                    if (OC.colw[o] == 8) rp[1] = (uint32_t)((uint64_t)vv >> 32);
                                } else if (MODE == SHB_OUT_COLS) {
                                    bk_put(OC.cols[o], OC.colw[o], row, vv);
                                } else if (out_vals) {
                                    out_vals[row * no + o] = vv;
                                }
                            }
                        }
                    };
                    for (uint32_t q = 0; q < ks; q++) put(r0 + q, (uint32_t)sk_spill_load(spl + slo + q));
                    uint32_t Km = K;
                    while (Km) {
                        const uint32_t s = (uint32_t)__ffs(Km) - 1u;
                        Km &= Km - 1u;
                        uint32_t yv = y[0];
#pragma unroll
                        for (int u = 1; u < SK_D; u++) yv = s == (uint32_t)u ? y[u] : yv;
                        // logical index above the new top
                        const uint32_t li = (s - b) & 7u;
                        put(r0 + (int64_t)ks + (int64_t)(li - n), yv);
                    }
                }
                // push: a full ring spills its bottom entry first
                if (a1 >> 31) {
                    if (n == SK_D) {
                        if (sc > 0 && ((now - (uint32_t)L.spt[lk]) & 0xFFFFu) > W) sc = 0;
                        if (sc >= (uint32_t)P.spill_cap) {
                            atomicOr(P.flag, SHK_F_SPILL);
                        } else {
                            uint32_t yb = y[0], tbb = tv[0];
#pragma unroll
                            for (int u = 1; u < SK_D; u++) {
                                yb = b == (uint32_t)u ? y[u] : yb;
                                tbb = b == (uint32_t)u ? tv[u] : tbb;
                            }
                            sk_spill_store(spl + sc, (uint64_t)yb | ((uint64_t)tbb << 32));
                            sc++;
                            L.spt[lk] = (uint16_t)tbb;
                        }
                        b = (b + 1u) & 7u;
                        n = SK_D - 1;
                    }
                    const uint32_t s = (b + n) & 7u;
                    L.y[s][lk] = x;
                    L.t[s][lk] = (uint16_t)now;
                    n++;
                }
                L.h[lk] = (uint16_t)(b | (n << 3) | (sc << 7));
            }
        }
        if (PASS == 1) {
            msum = shw_last(shw_incl_scan(msum));
            if (lane == 0) L.wsum[w] = emit ? msum : 0u;
        }
        if (P.prof) pc_proc += clock64() - pc0;
    }
    if (P.prof && lane == 0) {
        // clock ticks per phase summed over the waves: producer, queue hand-off
        // (both barriers' waits included), owner processing
        atomicAdd(P.prof + 0, pc_prod);
        atomicAdd(P.prof + 1, pc_queue);
        atomicAdd(P.prof + 2, pc_proc);
        atomicAdd(P.prof + 3, n_batch);
        atomicAdd(P.prof + 4, n_round);
        atomicAdd(P.prof + 5, n_ev);
    }
    if (PASS == 1) {
        __syncthreads();
        if (threadIdx.x == 0 && prev_sub >= 0) {
            uint32_t s = 0;
#pragma unroll
            for (int q = 0; q < SK_NW; q++) s += L.wsum[q];
            if (s) atomicAdd(&P.ttot[prev_sub], s);
        }
    }
}

static int sk_ok() { return hipGetLastError() == hipSuccess ? 0 : -3; }

static unsigned sk_grid(const shk_plan* P) { return 8u * (unsigned)P->cpx << P->gshift; }

extern "C" int shk_max_keys(void) { return SK_KPW; }

extern "C" int shk_open_bits(const shk_plan* P, void* stream) {
    if (!P->omask) return -1;
    hipLaunchKernelGGL(k_stk_open, dim3((unsigned)((P->n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, *P);
    return sk_ok();
}

extern "C" int shk_count(const shk_plan* P, void* stream) {
    hipStream_t st = (hipStream_t)stream;
    if (P->kpw > SK_KPW || P->gshift < 1 || P->gshift > 3) return -1;
    const shb_out O{};
    const shb_cols OC{};
    switch (P->gshift) {
        case 1: hipLaunchKernelGGL((k_stk<1, 2, SHB_OUT_RAW, 0>), dim3(sk_grid(P)), dim3(SK_TPB), 0, st, *P, O, OC, 0ull,
                                   nullptr, nullptr, 0ll); break;
        case 2: hipLaunchKernelGGL((k_stk<1, 4, SHB_OUT_RAW, 0>), dim3(sk_grid(P)), dim3(SK_TPB), 0, st, *P, O, OC, 0ull,
                                   nullptr, nullptr, 0ll); break;
        default: hipLaunchKernelGGL((k_stk<1, 8, SHB_OUT_RAW, 0>), dim3(sk_grid(P)), dim3(SK_TPB), 0, st, *P, O, OC,
                                    0ull, nullptr, nullptr, 0ll); break;
    }
    return sk_ok();
}

template <int EPL, int MODE, int NO>
static void sk_emit_launch(const shk_plan* P, const shb_out* O, const shb_cols& OC, uint64_t seq_base,
                           uint64_t* out_seq, int64_t* out_vals, int64_t out_cap, hipStream_t st) {
    hipLaunchKernelGGL((k_stk<2, EPL, MODE, NO>), dim3(sk_grid(P)), dim3(SK_TPB), 0, st, *P, *O, OC, seq_base, out_seq,
                       out_vals, out_cap);
}

template <int EPL>
static void sk_emit_mode(const shk_plan* P, const shb_out* O, const shb_cols* OC, uint64_t seq_base,
                         uint64_t* out_seq, int64_t* out_vals, int64_t out_cap, hipStream_t st) {
    // the packed four-value row of C2 unrolled; every other layout by descriptors
    if (OC && OC->use == SHB_OUT_PACKED) {
        if (O->n_out == 4) sk_emit_launch<EPL, SHB_OUT_PACKED, 4>(P, O, *OC, seq_base, out_seq, out_vals, out_cap, st);
        else sk_emit_launch<EPL, SHB_OUT_PACKED, 0>(P, O, *OC, seq_base, out_seq, out_vals, out_cap, st);
    } else if (OC && OC->use == SHB_OUT_COLS) {
        sk_emit_launch<EPL, SHB_OUT_COLS, 0>(P, O, *OC, seq_base, out_seq, out_vals, out_cap, st);
    } else if (O->n_out == 4) {
        sk_emit_launch<EPL, SHB_OUT_RAW, 4>(P, O, shb_cols{}, seq_base, out_seq, out_vals, out_cap, st);
    } else {
        sk_emit_launch<EPL, SHB_OUT_RAW, 0>(P, O, shb_cols{}, seq_base, out_seq, out_vals, out_cap, st);
    }
}

extern "C" int shk_emit(const shk_plan* P, const shb_out* O, const shb_cols* OC, uint64_t seq_base,
                        uint64_t* out_seq, int64_t* out_vals, int64_t out_cap, void* stream) {
    hipStream_t st = (hipStream_t)stream;
    if (P->kpw > SK_KPW || P->gshift < 1 || P->gshift > 3) return -1;
    if (OC && OC->use == SHB_OUT_PACKED && (OC->rw % 4 || OC->rw > 2 + 2 * SHB_MAX_OUT + 2)) return -1;
    switch (P->gshift) {
        case 1: sk_emit_mode<2>(P, O, OC, seq_base, out_seq, out_vals, out_cap, st); break;
        case 2: sk_emit_mode<4>(P, O, OC, seq_base, out_seq, out_vals, out_cap, st); break;
        default: sk_emit_mode<8>(P, O, OC, seq_base, out_seq, out_vals, out_cap, st); break;
    }
    return sk_ok();
}
