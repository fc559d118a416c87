// sh_stack.hip — the stack matcher of the bucketed window engine for partitioned
//   every e1=S[f1] -> e2=S[x.a op e1.a] within W          (C2)
//
// StreamPreStateProcessor.java:325-403 (break-early expiry, then processAndReturn
// over the pending list in creation order) with `every` on the start state makes
// every partial independent: partial i (an event passing f1) is consumed by the
// first later event q of its key with x_q op y_i (y_i = the same attribute of i),
// unless ts_q - ts_i > W expired it first. When the ordering term compares one
// attribute with itself, a key's pending partials form a monotone stack: a
// consumer takes exactly the entries it beats, which sit on top (for `>` the stack
// never increases upwards: every survivor of q is >= x_q and q goes on top), and
// expiry drops entries from the bottom (creation order is time order). A
// consumer's rows are its popped entries in creation order.
//
// This matcher can replace the sort-and-walk one (shb_match, hipRTC) between the
// two kernels of sh_bucket.hip (opt-in, SH_STACK=1: on C2 at 100M it takes 3.7 ms
// where shb_match takes 2.1, DESIGN.md "stack matcher"): k_bk_scatter has put
// every arrival tile in key-bucket order (b = key & 255; per event the packed word
// (ts - tbase) << kb | key >> 8 and the staged ordering column), k_bk_emit writes
// the ordered rows from what this kernel leaves: the counts (cnt, at the slots),
// the e1 values (match stream ms[0]), each (tile, bucket) segment's first match
// position (mstart) and the per-tile totals (ttot).
//
// One wave per (bucket, run of tiles), four buckets of one run per workgroup:
//  * a wave reads its bucket's events of the run's tiles (after the halo tiles the
//    window reaches, replayed without output) as one stream in arrival order, in
//    batches of SK_B events (the next batch's loads in flight while the current
//    one runs);
//  * lane k owns local key k (a bucket holds <= 64 keys): its stack's head (ring
//    bottom and count, top value, bottom timestamp, spilled count) in registers,
//    its ring of SK_D entries in an LDS column no other lane touches, deeper
//    entries spilled to a per-key stack in HBM. Six ballots per 64 events sort the
//    batch by key in LDS (stable: each key's events stay in arrival order), and
//    each owner then runs its events: expire the bottom, take the entries the
//    event beats, stage their values, push the event if it opens. A batch costs as
//    many steps as its busiest key has events; every step reads one LDS word pair
//    whose address is known a step ahead, and the second entries from the top and
//    the bottom are read speculatively with it;
//  * then, lanes over events: the counts' prefix gives every event its first
//    match-stream position, each tile's first event of the bucket records the
//    segment's position (mstart), and lanes over the staged values write them out.
// No segment table, no walk back, no workgroup barrier.
#include <hip/hip_runtime.h>

#include "../../include/sh_query.h"
#include "sh_device.h"
#include "sh_wave.h"

#define SK_WPB 4        // waves (buckets) per workgroup
#define SK_D 8          // ring entries per key in LDS
#define SK_KEYS 64      // local keys of a bucket, at most (kb <= 6)
#define SK_B 256        // events of a batch
#define SK_RUNT 256     // tiles of a run and its halo, at most
#define SK_STG 384      // staged matches of a batch, at most (else SHB_F_COUNT)

struct SkWave {
    uint32_t y[SK_D][SK_KEYS];   // ring entries: order keys (column k: key k's ring)
    uint32_t t[SK_D][SK_KEYS];   // ... packed timestamps (ts - tbase)
    union {
        uint2 sw[SK_B];          // the batch by key: packed word, order key (^ kflip)
        uint32_t pre[SK_B];      // then each event's first match-stream position
    } u;
    uint32_t bg[SK_B];           // tile << 13 | slot of each event (arrival order)
    uint32_t stv[SK_STG];        // staged values of the batch's matches (order keys)
    uint16_t stt[SK_STG];        // their event (arrival index in the batch) | row << 8
    uint16_t so[SK_B];           // each sorted entry: arrival index | opens << 8 | NaN << 9
    uint8_t cntb[SK_B];          // each event's matches (<= 255, else SHB_F_COUNT)
    uint32_t cum[SK_RUNT + 1];   // stream position of each tile's first event of the bucket
    uint16_t lo[SK_RUNT];        // the bucket's start in each tile's bucket order
    uint32_t sn;                 // staged values so far
};

// order keys: a float's IEEE bits (or an int) as an unsigned integer of the same
// order -- positive floats get the sign bit set, negative ones are inverted -- so
// every operator becomes one unsigned compare
template <bool F32>
__device__ __forceinline__ uint32_t sk_key(uint32_t bits) {
    return F32 ? ((bits & 0x80000000u) ? ~bits : (bits | 0x80000000u)) : (bits ^ 0x80000000u);
}
template <bool F32>
__device__ __forceinline__ uint32_t sk_unkey(uint32_t k) {
    return F32 ? ((k & 0x80000000u) ? (k & 0x7FFFFFFFu) : ~k) : (k ^ 0x80000000u);
}

// the opening filter: terms on the ordering column against constants, through
// order keys (-0.0 as +0.0; NaN: every compare false but !=)
__device__ __forceinline__ bool sk_open(const shk_params& K, uint32_t x) {
    bool ok = true;
#pragma unroll
    for (int k = 0; k < SHK_MAX_TERMS; k++) {
        if (k >= K.n_terms) break;
        const bool f = K.f_f32[k] != 0;
        const bool nan = f && (x & 0x7FFFFFFFu) > 0x7F800000u;
        uint32_t kv = f ? sk_key<true>(x) : sk_key<false>(x);
        kv = (f && kv == 0x7FFFFFFFu) ? 0x80000000u : kv;
        const uint32_t kc = K.f_ckey[k];
        const bool r = (K.f_lt[k] && kv < kc) || (K.f_eq[k] && kv == kc) || (K.f_gt[k] && kv > kc);
        ok = ok && (nan ? K.f_nan[k] != 0 : r);
    }
    return ok;
}

// a key's spilled entries are written and read back by its owner lane: through L2
// (agent-scope relaxed atomics skip the L1)
__device__ __forceinline__ uint64_t sk_spill_load(const uint64_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void sk_spill_store(uint64_t* p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ void sk_wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <bool F32>
__global__ void __launch_bounds__(64 * SK_WPB, 2) k_bk_stk(shb_plan P, shk_params K) {
    __shared__ SkWave Ls[SK_WPB];
    const int lane = (int)(threadIdx.x & 63u), wv = (int)(threadIdx.x >> 6);
    SkWave& L = Ls[wv];
    // workgroups are dealt round-robin to the 8 XCDs: XCD x takes bucket groups
    // [8x, 8x + 8) of each run (whose tiles' columns its L2 then holds)
    const int xcd = (int)(blockIdx.x & 7u), slot = (int)(blockIdx.x >> 3);
    const int run = slot >> 3;
    const int b = (((xcd << 3) | (slot & 7)) * SK_WPB) + wv;
    const int A = run * K.run_tiles;
    if (A >= P.nt) return;
    const int E = A + K.run_tiles < P.nt ? A + K.run_tiles : P.nt;
    const int kb = P.kb;
    const uint32_t kmask = (1u << kb) - 1u;
    const uint32_t W = (uint32_t)P.within;
    const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
    const bool owner = (lane >> kb) == 0;  // lane `lane` owns local key `lane`
    const int h0 = P.hstart[A];
    const int nt = E - h0;  // tiles of the pass
    uint32_t flag = 0u;
    // the halo is complete for a consumer at packed time `now` iff every event
    // before it is older than the window: now > tpre[h0] - tbase + W (hlim <= now)
    uint32_t hlim = 0u;
    if (h0 > 0) {
        const int64_t hl = P.tpre[h0] - P.tbase + P.within + 1;
        hlim = hl <= 0 ? 0u : (hl >= 0xFFFFFFFFll ? 0xFFFFFFFFu : (uint32_t)hl);
    }
    if (nt > SK_RUNT) {
        if (lane == 0) atomicOr(P.flag, SHB_F_HALO);
        return;
    }
    // the bucket's segment of every tile (transposed starts) -> stream positions
    uint32_t carry = 0u;
    for (int i0 = 0; i0 < nt; i0 += 64) {
        const int i = i0 + lane;
        uint32_t l0 = 0u, c = 0u;
        if (i < nt) {
            l0 = P.tofft[(int64_t)b * P.tstride + h0 + i];
            c = (uint32_t)P.tofft[(int64_t)(b + 1) * P.tstride + h0 + i] - l0;
            L.lo[i] = (uint16_t)l0;
        }
        const uint32_t inc = shw_incl_scan(c);
        if (i < nt) L.cum[i] = carry + inc - c;
        carry += shw_last(inc);
    }
    const uint32_t nev = carry;  // events of the pass
    if (lane == 0) {
        L.cum[nt] = nev;
        L.sn = 0u;
    }
    // the run's region of the match stream: a partial is consumed once, and the
    // partials the run's consumers take are events of the pass
    uint32_t mpos = 0u;
    if (K.want_ms) {
        if (lane == 0) mpos = atomicAdd(P.ms_ctr, nev);
        mpos = (uint32_t)__shfl((int)mpos, 0);
    }
    const uint32_t* __restrict__ xs = (const uint32_t*)P.st_dst[0];
    uint32_t* __restrict__ ms = (uint32_t*)P.ms[0];
    // key `lane`'s spill stack (HBM)
    uint64_t* const spl = K.spill + (((uint64_t)blockIdx.x * SK_WPB + wv) * SK_KEYS + lane) * (uint64_t)K.spill_cap;
    const uint32_t gA = (uint32_t)A << SHB_TILE_SHIFT;  // the first emitting slot index
    sk_wave_sync();
    const uint32_t fem = L.cum[A - h0];                  // ... and stream position

    // a batch's loads: stream position -> tile (binary search of cum) -> slot
    uint32_t rw[SK_B / 64], rx[SK_B / 64], rg[SK_B / 64];
    auto issue = [&](uint32_t fb) {
#pragma unroll
        for (int j = 0; j < SK_B / 64; j++) {
            const uint32_t f = fb + (uint32_t)(j * 64 + lane);
            rw[j] = rx[j] = rg[j] = 0u;
            if (f < nev) {
                int lo = 0, hi = nt - 1;  // the last tile whose start is <= f
                while (lo < hi) {
                    const int mid = (lo + hi + 1) >> 1;
                    if (L.cum[mid] <= f) lo = mid;
                    else hi = mid - 1;
                }
                const uint32_t g = ((uint32_t)(h0 + lo) << SHB_TILE_SHIFT) + L.lo[lo] + (f - L.cum[lo]);
                rg[j] = g;
                rw[j] = P.w0[g];
                rx[j] = xs[g];
            }
        }
    };
    // key `lane`'s stack head: ring bottom and count, spilled entries, latest
    // timestamp, top value, bottom timestamp, newest spilled timestamp
    uint32_t o_bo = 0u, o_c = 0u, o_sc = 0u, o_last = 0u, o_ytop = 0u, o_tbot = 0u, o_spt = 0u;
    // diagnostics (SH_BK_PROFILE): clock ticks per phase and counts, per wave
    const bool prof = P.prof != nullptr;
    unsigned long long pt = prof ? clock64() : 0ull, pr[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#define SK_TICK(i)                                 \
    if (prof) {                                    \
        const unsigned long long t2_ = clock64();  \
        pr[i] += t2_ - pt;                         \
        pt = t2_;                                  \
    }
    SK_TICK(0);
    issue(0u);
    SK_TICK(1);
    uint32_t prevT = 0xFFFFFFFFu;  // the last tile whose segment position is recorded
    for (uint32_t fb = 0; fb < nev; fb += SK_B) {
        const uint32_t fe = fb + SK_B < nev ? fb + SK_B : nev;
        const uint32_t ethr = fem <= fb ? 0u : (fem - fb < SK_B ? fem - fb : SK_B);  // first emitting event
        // the batch by key, stable: each owner's events [kst, kst + kn) in arrival order
        uint64_t mk[SK_B / 64];
        uint32_t kn = 0u;
#pragma unroll
        for (int j = 0; j < SK_B / 64; j++) {
            const bool act = fb + (uint32_t)(j * 64 + lane) < fe;
            const uint32_t kk = rw[j] & kmask;
            uint64_t m = __ballot(act);
            for (int bb = 0; bb < kb; bb++) {
                const uint64_t bm = __ballot(act && ((kk >> bb) & 1u));
                m &= ((lane >> bb) & 1) ? bm : ~bm;
            }
            mk[j] = owner ? m : 0ull;
            kn += (uint32_t)__popcll(mk[j]);
        }
        const uint32_t kst = shw_incl_scan(kn) - kn;
        uint32_t krun = kst;  // the owner's next sorted position
#pragma unroll
        for (int j = 0; j < SK_B / 64; j++) {
            const bool act = fb + (uint32_t)(j * 64 + lane) < fe;
            const int kk = (int)(rw[j] & kmask);
            const uint32_t base = (uint32_t)__shfl((int)krun, kk);
            const uint32_t plo = (uint32_t)__shfl((int)(uint32_t)mk[j], kk);
            const uint32_t phi = (uint32_t)__shfl((int)(uint32_t)(mk[j] >> 32), kk);
            const uint64_t peers = ((uint64_t)phi << 32) | plo;
            if (act) {
                const uint32_t d = base + (uint32_t)__popcll(peers & lt);
                const uint32_t xr = rx[j];
                const bool nan = F32 && (xr & 0x7FFFFFFFu) > 0x7F800000u;
                const bool open = !nan && sk_open(K, xr);
                L.u.sw[d] = make_uint2(rw[j], sk_key<F32>(xr) ^ K.kflip);
                L.so[d] = (uint16_t)((j * 64 + lane) | (open ? 0x100 : 0) | (nan ? 0x200 : 0));
                L.bg[j * 64 + lane] = rg[j];
            }
            krun += (uint32_t)__popcll(mk[j]);
        }
        sk_wave_sync();
        SK_TICK(2);
        if (fb + SK_B < nev) issue(fb + SK_B);
        SK_TICK(1);
        // the owners run their events (the next entry's words read a step ahead),
        // as many steps as the busiest key has events
        uint32_t nmax = kn;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) nmax = max(nmax, (uint32_t)__shfl_xor((int)nmax, d));
        const uint32_t kl = kn ? kst + kn - 1u : kst;  // the owner's last entry
        uint2 vn = L.u.sw[kst < SK_B ? kst : SK_B - 1];
        uint32_t on = L.so[kst < SK_B ? kst : SK_B - 1];
        for (uint32_t s = 0; s < nmax; s++) {
            const uint2 v = vn;
            uint32_t o = on;
            {
                const uint32_t sx = kst + s + 1u < kl ? kst + s + 1u : kl;
                vn = L.u.sw[sx];
                on = L.so[sx];
            }
            if (s < kn) {
                // speculative: the second entries from the bottom and from the top
                const uint32_t tsec = L.t[(o_bo + 1u) & (SK_D - 1)][lane];
                const uint32_t ysec = L.y[(o_bo + o_c - 2u) & (SK_D - 1)][lane];
                const uint32_t w = v.x, x = v.y;
                const bool open = (o & 0x100u) != 0u, nan = (o & 0x200u) != 0u;
                o &= 0xFFu;
                const bool emit = o >= ethr;
                const uint32_t now = w >> kb;
                flag |= (emit && now < hlim) ? (uint32_t)SHB_F_HALO : 0u;
                flag |= now < o_last ? (uint32_t)SHB_F_MONO : 0u;
                o_last = now;
                const uint32_t cx = x == K.zk1 ? K.zk0 : x;
                // expiry from the bottom (spilled entries are older still): one entry
                // by the speculative read, more (rare) by a walk
                const bool ex1 = o_c > 0u && now - o_tbot > W;
                o_sc = ex1 ? 0u : o_sc;
                o_bo = ex1 ? ((o_bo + 1u) & (SK_D - 1)) : o_bo;
                o_tbot = ex1 ? tsec : o_tbot;
                o_c = ex1 ? o_c - 1u : o_c;
                if (ex1 && o_c > 0u && now - o_tbot > W) {
                    do {
                        o_bo = (o_bo + 1u) & (SK_D - 1);
                        o_tbot = L.t[o_bo][lane];
                    } while (--o_c > 0u && now - o_tbot > W);
                }
                // the entries x beats: the top of the stack (top and second in registers)
                const uint32_t ytop = o_ytop;
                const uint32_t c0 = ytop == K.zk1 ? K.zk0 : ytop;
                const uint32_t c1 = ysec == K.zk1 ? K.zk0 : ysec;
                const bool b0 = !nan && o_c > 0u && (cx > c0 || (K.ge && cx == c0));
                const bool b1 = b0 && o_c > 1u && (cx > c1 || (K.ge && cx == c1));
                uint32_t kp = (b0 ? 1u : 0u) + (b1 ? 1u : 0u);
                o_ytop = (b0 && !b1 && o_c > 1u) ? ysec : o_ytop;
                if (b1 && o_c > 2u) {
                    for (;;) {
                        const uint32_t yv = L.y[(o_bo + o_c - 1u - kp) & (SK_D - 1)][lane];
                        const uint32_t cy = yv == K.zk1 ? K.zk0 : yv;
                        if (!(cx > cy || (K.ge && cx == cy))) {
                            o_ytop = yv;  // the new top
                            break;
                        }
                        if (++kp == o_c) break;
                    }
                }
                // below an emptied ring: the spilled entries
                uint32_t ks = 0u, slo = o_sc;
                if (kp == o_c && o_sc > 0u && !nan) {
                    while (o_sc > 0u) {
                        const uint64_t ev = sk_spill_load(spl + o_sc - 1u);
                        if (now - (uint32_t)(ev >> 32) > W) {
                            o_sc = 0u;  // it and every older spilled entry expired
                            break;
                        }
                        const uint32_t cy = (uint32_t)ev == K.zk1 ? K.zk0 : (uint32_t)ev;
                        if (!(cx > cy || (K.ge && cx == cy))) break;
                        o_sc--;
                        ks++;
                        slo = o_sc;
                    }
                }
                const uint32_t tot = emit ? ks + kp : 0u;
                flag |= tot > 255u ? (uint32_t)SHB_F_COUNT : 0u;
                L.cntb[o] = (uint8_t)(tot > 255u ? 255u : tot);
                // stage the values in creation order: spilled ones, then the ring's
                if (K.want_ms && tot > 0u) {
                    const uint32_t sb =
                        __hip_atomic_fetch_add(&L.sn, tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
                    if (sb + tot > SK_STG) {
                        flag |= SHB_F_COUNT;
                    } else {
                        const uint32_t r0 = sb + ks;
                        if (kp) {
                            L.stv[r0 + kp - 1u] = ytop;
                            L.stt[r0 + kp - 1u] = (uint16_t)(o | ((ks + kp - 1u) << 8));
                        }
                        if (kp >= 2u) {
                            L.stv[r0 + kp - 2u] = ysec;
                            L.stt[r0 + kp - 2u] = (uint16_t)(o | ((ks + kp - 2u) << 8));
                        }
                        if (kp >= 3u || ks) {
                            for (uint32_t q = 0; q < ks; q++) {
                                L.stv[sb + q] = (uint32_t)sk_spill_load(spl + slo + q);
                                L.stt[sb + q] = (uint16_t)(o | (q << 8));
                            }
                            for (uint32_t q = 0; q + 2u < kp; q++) {
                                L.stv[r0 + q] = L.y[(o_bo + o_c - kp + q) & (SK_D - 1)][lane];
                                L.stt[r0 + q] = (uint16_t)(o | ((ks + q) << 8));
                            }
                        }
                    }
                }
                o_c -= kp;
                // push: a full ring spills its bottom entry first
                if (open) {
                    if (o_c == SK_D) {
                        if (o_sc > 0u && now - o_spt > W) o_sc = 0u;
                        if (o_sc >= (uint32_t)K.spill_cap) {
                            flag |= SHK_F_SPILL;
                        } else {
                            sk_spill_store(spl + o_sc, (uint64_t)L.y[o_bo][lane] | ((uint64_t)o_tbot << 32));
                            o_spt = o_tbot;
                            o_sc++;
                        }
                        o_bo = (o_bo + 1u) & (SK_D - 1);
                        o_c = SK_D - 1;
                        o_tbot = L.t[o_bo][lane];
                    }
                    const uint32_t sl = (o_bo + o_c) & (SK_D - 1);
                    L.y[sl][lane] = x;
                    L.t[sl][lane] = now;
                    o_tbot = o_c == 0u ? now : o_tbot;
                    o_c++;
                    o_ytop = x;
                }
            }
        }
        if (prof) pr[7] += nmax;
        sk_wave_sync();
        SK_TICK(4);
        if (prof) pr[6]++;
        // lanes over events: counts, positions, each tile's segment
#pragma unroll
        for (int j = 0; j < SK_B / 64; j++) {
            const uint32_t e = (uint32_t)(j * 64 + lane);
            const bool act = fb + e < fe;
            const uint32_t tot = act ? (uint32_t)L.cntb[e] : 0u;
            const uint32_t g = act ? L.bg[e] : 0u;
            const bool emit = act && e >= ethr;
            const uint32_t incm = shw_incl_scan(tot);
            const uint32_t excl = incm - tot;
            L.u.pre[e] = mpos + excl;
            if (emit) P.cnt[g] = (uint8_t)tot;
            // per tile of the block: its first lane records the segment's position
            // (the tile's first event of the bucket) and adds the segment's matches
            const uint32_t T = g >> SHB_TILE_SHIFT;
            const uint32_t Tp = (uint32_t)__shfl((int)T, lane > 0 ? lane - 1 : 0);
            const bool seg = emit && (lane == 0 || T != Tp);
            const uint64_t fm = __ballot(seg);
            const uint64_t after = lane == 63 ? 0ull : fm & ~((2ull << lane) - 1ull);
            const int lastl = after ? (int)__builtin_ctzll(after) - 1 : 63;
            const uint32_t tend = (uint32_t)__shfl((int)incm, lastl);
            if (seg) {
                if (lane != 0 || T != prevT) P.mstart[(int64_t)T * SHB_NB + b] = mpos + excl;
                if (tend > excl) atomicAdd(&P.ttot[T], tend - excl);
            }
            if (fm) prevT = (uint32_t)__shfl((int)T, 63 - __builtin_clzll(fm));
            mpos += shw_last(incm);
        }
        sk_wave_sync();
        // lanes over the staged values: into the match stream
        if (K.want_ms) {
            const uint32_t nst = L.sn < SK_STG ? L.sn : SK_STG;
            for (uint32_t s = (uint32_t)lane; s < nst; s += 64) {
                const uint32_t tg = L.stt[s];
                ms[L.u.pre[tg & 0xFFu] + (tg >> 8)] = sk_unkey<F32>(L.stv[s] ^ K.kflip);
            }
        }
        sk_wave_sync();
        if (lane == 0) L.sn = 0u;
        SK_TICK(5);
    }
#undef SK_TICK
    if (prof && lane == 0)
        for (int i = 0; i < 8; i++) atomicAdd(P.prof + i, pr[i]);
    if (flag) atomicOr(P.flag, (int)flag);
}

extern "C" int shk_match(const shb_plan* P, const shk_params* K, void* stream) {
    if (P->kb > 6 || P->n_staged < 1 || P->st_width[0] != 4 || K->run_tiles < 1 ||
        K->run_tiles > SK_RUNT - SHB_HMAX || K->n_terms < 0 || K->n_terms > SHK_MAX_TERMS || K->spill_cap < 1 ||
        (K->want_ms && P->ms_width[0] != 4))
        return -1;
    const int runs = (P->nt + K->run_tiles - 1) / K->run_tiles;
    // 64 workgroups of 4 buckets per run: XCD x holds bucket groups 8x .. 8x + 7
    const unsigned grid = (unsigned)runs * (SHB_NB / SK_WPB);
    if (K->dom == DOM_F32)
        hipLaunchKernelGGL(k_bk_stk<true>, dim3(grid), dim3(64 * SK_WPB), 0, (hipStream_t)stream, *P, *K);
    else
        hipLaunchKernelGGL(k_bk_stk<false>, dim3(grid), dim3(64 * SK_WPB), 0, (hipStream_t)stream, *P, *K);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

extern "C" int shk_max_run_tiles(void) { return SK_RUNT - SHB_HMAX; }
extern "C" int shk_spill_keys(void) { return SK_KEYS * SK_WPB; }
