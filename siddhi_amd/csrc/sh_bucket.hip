// sh_bucket.hip — bucketed window engine: the data movement around the hipRTC
// matcher (shb_match, sh_jit.cpp) for partitioned
//   every e1=S[f1] -> e2=S[f2(e1,e2)] within W        (C2)
//
// A partial opened at event i is consumed at the first later event j of its
// key with f2(i, j) while ts_j - ts_i <= W (StreamPreStateProcessor.java:325-403:
// break-early expiry then processAndReturn, every event a consumer candidate).
// The reference walks one global per-query pending list per event; here:
//
//  k_bk_scatter per arrival tile T (8,192 events): stable reorder by key bucket
//               (b = key & 255) inside the tile's own region, moving only the
//               packed (ts | local key) word and the columns the matcher reads;
//               ranks from wave ballots (sh_wave.h), staged through LDS so the
//               tile is written as one contiguous run; the bucket starts of the
//               tile (toff) and each event's slot (sp)
//  shb_match    (hipRTC) per (bucket, run of tiles): the bucket's segment of
//               each tile plus halo tiles covering the window, gathered into LDS;
//               per-consumer walk back over its key -> partials consumed per
//               event (u8, at the event's slot), their e1-side select values
//               (match stream, one region per pass), each (tile, bucket)
//               segment's first match position, matches per tile (atomics)
//  (scan)       tile totals -> each tile's first row
//  k_bk_emit    per arrival tile: counts by slot -> positions, arrival-order
//               scan, ordered rows (trigger seq + select values)
//
// HBM bytes per event (C2): scatter 16 read / 10 written, matcher ~9 read +
// 1 + the match stream written, emitter ~19 read + the rows; no global
// histogram or segment scan.
#include <hip/hip_runtime.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/sh_query.h"
#include "sh_device.h"
#include "sh_nfa.h"
#include "sh_rows.h"
#include "sh_wave.h"

#define BK_TPB 512
#define BK_ITEMS (SHB_TILE / BK_TPB)

static_assert(BK_ITEMS == 16, "tile / threads");


// XCD-aware tile order: workgroups are dealt round-robin to the 8 XCDs, so
// block `bid` takes tile (bid % 8) * per + bid / 8 and each XCD walks a
// contiguous run of arrival tiles; the (bucket, tile) segments of neighbouring
// tiles share cache lines (partial-line writes of the scatter, count and
// match-stream gathers of the emitter) and now meet in the same L2. -1: none.
__device__ __forceinline__ int bk_tile(int nt) {
    const int per = (nt + 7) >> 3;
    const int t = (int)(blockIdx.x & 7u) * per + (int)(blockIdx.x >> 3);
    return t < nt ? t : -1;
}
static inline unsigned bk_grid(int nt) { return 8u * (unsigned)((nt + 7) >> 3); }


// ---------------------------------------------------------------- partition
// One arrival tile per workgroup, reordered stably by key bucket into the
// tile's own region (tile-local: no histogram pass, no global scan, and every
// write of the tile is one contiguous run): the packed word (ts - tbase) << kb |
// key >> 8 and the staged columns at T * TILE + slot, the slot of every event
// (sp, arrival order: the emitter finds an event's count and match-stream
// position through it) and the tile's bucket starts (toff).
template <int MINW, int TPB>
__global__ void __launch_bounds__(TPB, MINW) k_bk_scatter(const int32_t* __restrict__ keys,
                                                          const int64_t* __restrict__ ts, int32_t nkeys, shb_plan P) {
    constexpr int SC_ITEMS = SHB_TILE / TPB;  // events per lane
    __shared__ uint32_t wcnt[TPB / 64][256];
    __shared__ uint32_t tstart[256];
    __shared__ uint32_t ws[TPB / 64];
    __shared__ uint32_t stage[SHB_TILE];
    __shared__ int64_t s_tmx[TPB / 64];
    const int T = bk_tile(P.nt);
    if (T < 0) return;
    const int64_t b0 = (int64_t)T << SHB_TILE_SHIFT;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int c = threadIdx.x; c < (TPB / 64) * 256; c += TPB) (&wcnt[0][0])[c] = 0u;
    __syncthreads();
    // the keys and timestamps of the tile are loaded up front (one HBM round
    // trip); the packed word is formed in registers
    int32_t key[SC_ITEMS];
    uint32_t rw[SC_ITEMS], wp[SC_ITEMS];
    const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
    {
        int64_t tv[SC_ITEMS];
        const int64_t e0 = b0 + (int64_t)w * (64 * SC_ITEMS) + lane;
        if (b0 + SHB_TILE <= P.n) {
            // a full tile: unpredicated loads at immediate offsets from two bases
            const int32_t* __restrict__ pk = keys + e0;
            const int64_t* __restrict__ pt = ts + e0;
#pragma unroll
            for (int j = 0; j < SC_ITEMS; j++) {
                key[j] = pk[j * 64];
                tv[j] = pt[j * 64];
            }
        } else {
#pragma unroll
            for (int j = 0; j < SC_ITEMS; j++) {
                const int64_t i = e0 + j * 64;
                const bool in = i < P.n;
                key[j] = in ? keys[i] : -1;
                tv[j] = in ? ts[i] : P.tbase;
            }
        }
        const int64_t lim = (int64_t)1 << (32 - P.kb);
        bool bad = false, badk = false;
        int64_t tmx = INT64_MIN;
#pragma unroll
        for (int j = 0; j < SC_ITEMS; j++) {
            const int64_t dt = tv[j] - P.tbase;
            if (key[j] >= nkeys) badk = true;
            if (key[j] >= 0 && !P.no_ts && (dt < 0 || dt >= lim)) bad = true;
            if (key[j] >= 0 && tv[j] > tmx) tmx = tv[j];
            wp[j] = P.no_ts ? ((uint32_t)key[j] >> 8) : (((uint32_t)dt << P.kb) | ((uint32_t)key[j] >> 8));
            rw[j] = key[j] >= 0 ? ((uint32_t)key[j] & (SHB_NB - 1)) << 16 : ~0u;
        }
        if (bad) atomicOr(P.flag, SHB_F_TS);
        if (badk) atomicOr(P.flag, SHB_F_KEY);
        // the tile's latest timestamp (the matcher's halo check)
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) {
            const int64_t y = __shfl_xor(tmx, o);
            tmx = y > tmx ? y : tmx;
        }
        if (lane == 0) s_tmx[w] = tmx;
        if (threadIdx.x == 0) P.tfirst[T] = tv[0];
    }
    // each wave ranks its own contiguous 1,024 events (16 rounds of 64): the
    // rank of an event among the wave's same-bucket events before it, from 8
    // ballots per round; the leader lane of each bucket group adds the group to
    // the wave's running count with a returning LDS atomic and the group reads
    // its base from the leader
    {
        uint32_t old[SC_ITEMS];
#pragma unroll
        for (int j = 0; j < SC_ITEMS; j++) {
            const bool valid = rw[j] != ~0u;
            const uint32_t d = (rw[j] >> 16) & (SHB_NB - 1);
            uint64_t peers = __ballot(valid);
#pragma unroll
            for (int bb = 0; bb < 8; bb++) {
                const bool bit = (d >> bb) & 1u;
                const uint64_t m = __ballot(valid && bit);
                peers &= bit ? m : ~m;
            }
            const uint32_t r = (uint32_t)__popcll(peers & lt);
            old[j] = 0u;
            if (valid && r == 0) old[j] = atomicAdd(&wcnt[w][d], (uint32_t)__popcll(peers));
            // rank | leader lane << 8 | bucket << 16 (~0u: no key)
            rw[j] = valid ? (r | ((uint32_t)(__ffsll((unsigned long long)peers) - 1) << 8) | (d << 16)) : ~0u;
        }
#pragma unroll
        for (int j = 0; j < SC_ITEMS; j++) {
            const uint32_t ld = rw[j] == ~0u ? (uint32_t)lane : (rw[j] >> 8) & 63u;
            const uint32_t base = (uint32_t)__shfl((int)old[j], (int)ld);
            if (rw[j] != ~0u) rw[j] = ((base + (rw[j] & 0xFFu)) & 0xFFFFu) | (rw[j] & 0xFF0000u);  // wave rank | bucket << 16
        }
    }
    __syncthreads();
    // per bucket: the waves' exclusive offsets, then the buckets' starts
    uint32_t nvalid;
    {
        uint32_t tot = 0;
        if (threadIdx.x < 256) {
#pragma unroll
            for (int q = 0; q < TPB / 64; q++) {
                const uint32_t c = wcnt[q][threadIdx.x];
                wcnt[q][threadIdx.x] = tot;
                tot += c;
            }
        }
        const uint32_t ex = shw_block_excl<TPB>(threadIdx.x < 256 ? tot : 0u, ws, &nvalid);
        if (threadIdx.x < 256) {
            tstart[threadIdx.x] = ex;
            P.toff[(int64_t)T * SHB_TOFF + threadIdx.x] = (uint16_t)ex;
        }
        if (threadIdx.x == 256) P.toff[(int64_t)T * SHB_TOFF + 256] = (uint16_t)nvalid;
        if (threadIdx.x == 0) {
            int64_t m = s_tmx[0];
#pragma unroll
            for (int q = 1; q < TPB / 64; q++) m = s_tmx[q] > m ? s_tmx[q] : m;
            P.tpre[T] = m;
        }
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < SC_ITEMS; j++) {
        const bool valid = rw[j] != ~0u;
        const uint32_t d = (rw[j] >> 16) & (SHB_NB - 1);
        rw[j] = valid ? tstart[d] + wcnt[w][d] + (rw[j] & 0xFFFFu) : ~0u;  // the event's slot
        const int64_t i = b0 + (int64_t)w * (64 * SC_ITEMS) + j * 64 + lane;
        if (i < P.n) P.sp[i] = (uint16_t)rw[j];
        if (valid) stage[rw[j]] = wp[j];
    }
    __syncthreads();
    const int64_t ob = (int64_t)T << SHB_TILE_SHIFT;
#define BK_WRITE_OUT(TY, DST, EXPR)                                                  \
    {                                                                                \
        _Pragma("unroll 4") for (int m = 0; m < SC_ITEMS; m++) {                     \
            const uint32_t l = (uint32_t)(m * TPB + threadIdx.x);                 \
            if (l < nvalid) ((TY*)(DST))[EXPR(ob + l)] = (TY)stage[l];               \
        }                                                                            \
        __syncthreads();                                                             \
    }
#define BK_ID(x) (x)
#define BK_LO(x) (2 * (x))
#define BK_HI(x) (2 * (x) + 1)
    BK_WRITE_OUT(uint32_t, P.w0, BK_ID);
    for (int c = 0; c < P.n_staged; c++) {
        const int wd = P.st_width[c];
        const int halves = wd == 8 ? 2 : 1;
        for (int hh = 0; hh < halves; hh++) {
#pragma unroll
            for (int j = 0; j < SC_ITEMS; j++) {
                if (rw[j] == ~0u) continue;
                const int64_t i = b0 + (int64_t)w * (64 * SC_ITEMS) + j * 64 + lane;
                uint32_t v;
                if (wd == 8) v = ((const uint32_t*)P.st_src[c])[2 * i + hh];
                else if (wd == 4) v = ((const uint32_t*)P.st_src[c])[i];
                else v = ((const uint8_t*)P.st_src[c])[i];
                stage[rw[j]] = v;
            }
            __syncthreads();
            if (wd == 8) {
                if (hh == 0) BK_WRITE_OUT(uint32_t, P.st_dst[c], BK_LO)
                else BK_WRITE_OUT(uint32_t, P.st_dst[c], BK_HI)
            } else if (wd == 4) {
                BK_WRITE_OUT(uint32_t, P.st_dst[c], BK_ID)
            } else {
                BK_WRITE_OUT(uint8_t, P.st_dst[c], BK_ID)
            }
        }
    }
#undef BK_WRITE_OUT
#undef BK_ID
#undef BK_LO
#undef BK_HI
}

// ---------------------------------------------------------------- emitter
// Per arrival tile, 8 waves of 1,024 consecutive events each:
//  1. the tile's counts in its bucket order (one 16-byte load per thread) ->
//     their exclusive prefix pfx[slot] (LDS): an event of bucket d at slot s has
//     count pfx[s+1] - pfx[s] and match-stream position mstart[T][d] + pfx[s] -
//     pfx[toff[d]] (the matcher wrote each (tile, bucket) segment's matches
//     contiguously, in arrival order)
//  2. per wave: the counts and positions of its events (registers), its total
//  3. per half-wave-block of 512 events: a DPP scan gives each event its first
//     row; the wave's row map (row -> event) is filled and lane t writes rows t,
//     t + 64, ... (consecutive lanes, consecutive rows: coalesced stores); the
//     consumer-side values are read by arrival index, the e1-side values from
//     the match stream
#define BK_EHALF 512   // events of one row-map pass of a wave
#define BK_PFX_BITS 24  // pfx words: prefix in the low bits, the slot's bucket above
#define BK_PFX_MASK ((1u << BK_PFX_BITS) - 1u)
#define BK_NOSLOT 0xFFFFFFFFu
#define BK_EROWS 1024  // rows the wave's map holds per pass (more: event-parallel writes)

// select value o of a row (raw 8-byte form; kind 0: by match-stream position, 1: by event)
#define BK_VAL(o, i, mp, row) bk_raw(O.src[o], O.kind[o] == 1 ? (i) : (mp), O.type[o])


// the select values of a row (NO > 0: unrolled, the descriptors in scalar registers)
template <int NO>
__device__ __forceinline__ void bk_vals(const shb_out& O, int64_t i, int64_t mp, int64_t row, int64_t* v) {
#pragma unroll
    for (int o = 0; o < NO; o++) v[o] = BK_VAL(o, i, mp, row);
}


template <int MODE, int NO>
__device__ __forceinline__ void bk_row(const shb_out& O, const shb_cols& OC, const int32_t* o_kind,
                                       const int32_t* o_type, const void* const* o_src, int64_t row, int64_t i,
                                       int64_t mp, uint64_t seq, uint64_t* __restrict__ out_seq,
                                       int64_t* __restrict__ out_vals) {
    if (NO > 0) {
        int64_t v[NO > 0 ? NO : 1];
        bk_vals<NO>(O, i, mp, row, v);
        bk_store<MODE, NO>(OC, row, v, seq, out_seq, out_vals);
        return;
    }
    // any number of values: the descriptors from LDS, one value at a time
    const int no = O.n_out;
    if (MODE == SHB_OUT_PACKED) {
        uint32_t* r = (uint32_t*)OC.rows + row * OC.rw;
        r[0] = (uint32_t)seq;
        r[1] = (uint32_t)(seq >> 32);
        for (int k = 2; k < OC.rw; k++) r[k] = 0u;
    } else if (out_seq) {
        out_seq[row] = seq;
    }
    for (int o = 0; o < no; o++) {
        const int64_t v = bk_raw(o_src[o], o_kind[o] == 1 ? i : mp, o_type[o]);
        if (MODE == SHB_OUT_PACKED) {
            uint32_t* r = (uint32_t*)OC.rows + row * OC.rw + OC.woff[o];
            r[0] = OC.colw[o] == 1 ? (uint32_t)(uint8_t)v : (uint32_t)v;
            if (OC.colw[o] == 8) r[1] = (uint32_t)((uint64_t)v >> 32);
        } else if (MODE == SHB_OUT_COLS) {
            bk_put(OC.cols[o], OC.colw[o], row, v);
        } else if (out_vals) {
            out_vals[row * no + o] = v;
        }
    }
}

// rows per lane whose loads are issued before their stores (the template's RU:
// 4 or 6; a half of 512 events has ~290 rows on C2, one round of 6 x 64 rows)

template <int MODE, int NO, int BK_RU, int BK_OCC = 4>
__global__ void __launch_bounds__(BK_TPB, BK_OCC) k_bk_emit(shb_plan P, shb_out O, shb_cols OC, uint64_t seq_base,
                                                    uint64_t* __restrict__ out_seq, int64_t* __restrict__ out_vals,
                                                    int64_t out_cap) {
    // the slot prefix (phases 1-2) and the row maps (phase 3) share storage: phase 3
    // starts after the barrier that ends every wave's phase 2 (42 KB instead of 75:
    // three workgroups per CU when the registers allow)
    // LM (6 waves per SIMD, <= 80 VGPRs): the wave's 1,024 match-stream positions go
    // to LDS once (emp holds both halves) instead of living in registers through the
    // row loop, and a half's row map holds 512 rows (more: the event-parallel path)
    constexpr bool LM = BK_OCC >= 6;
    constexpr int EROWS = LM ? 512 : BK_EROWS;
    constexpr int EMPW = LM ? 2 * BK_EHALF : BK_EHALF;
    constexpr int BK_MAPW = (BK_TPB / 64) * (EROWS / 2 + EMPW + BK_EHALF / 2);
    __shared__ uint32_t pool[(SHB_TILE + 1) > BK_MAPW ? (SHB_TILE + 1) : BK_MAPW];
    uint32_t* const pfx = pool;
    uint16_t(*const rmap)[EROWS] = (uint16_t(*)[EROWS])pool;
    uint32_t(*const emp)[EMPW] = (uint32_t(*)[EMPW])(pool + (BK_TPB / 64) * (EROWS / 2));
    uint16_t(*const ero)[BK_EHALF] =
        (uint16_t(*)[BK_EHALF])(pool + (BK_TPB / 64) * (EROWS / 2 + EMPW));
    __shared__ uint32_t ms0[SHB_NB];
    __shared__ uint16_t to[SHB_NB + 1];
    __shared__ uint32_t wtot[BK_TPB / 64], ws[BK_TPB / 64];
    __shared__ int32_t o_kind[SHB_MAX_OUT], o_type[SHB_MAX_OUT];
    __shared__ const void* o_src[SHB_MAX_OUT];
    __shared__ uint32_t s_tb;
    constexpr int NV = NO > 0 ? NO : 1;
    const int T = bk_tile(P.nt);
    if (T < 0) return;
    const int64_t b0 = (int64_t)T << SHB_TILE_SHIFT;
    const int tile_n = (int)((P.n - b0) < SHB_TILE ? (P.n - b0) : SHB_TILE);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (threadIdx.x <= SHB_NB) to[threadIdx.x] = P.toff[(int64_t)T * SHB_TOFF + threadIdx.x];
    if (threadIdx.x < SHB_NB) ms0[threadIdx.x] = P.mstart[(int64_t)T * SHB_NB + threadIdx.x];
    if (threadIdx.x == 0) s_tb = P.ttot[T];
    if (NO == 0 && threadIdx.x < SHB_MAX_OUT) {
#pragma unroll
        for (int o = 0; o < SHB_MAX_OUT; o++)
            if (o == (int)threadIdx.x) {
                o_kind[o] = O.kind[o];
                o_type[o] = O.type[o];
                o_src[o] = O.src[o];
            }
    }
    // the events of this wave (arrival order): their slots, loaded up front (the
    // bucket of a slot follows from the tile's bucket starts: no key read)
    uint32_t sl[BK_ITEMS];
    {
        const int l0 = w * (64 * BK_ITEMS) + lane;
#pragma unroll
        for (int j = 0; j < BK_ITEMS; j++) {
            const int l = l0 + j * 64;
            sl[j] = l < tile_n ? (uint32_t)P.sp[b0 + l] : BK_NOSLOT;
        }
    }
    // 1. counts in the tile's bucket order -> pfx (loaded with the events; the
    // slots past the tile's valid events are masked below). Each word holds the
    // exclusive prefix (< 2^21: 8,192 counts of at most 255) and, in its top 8
    // bits, the slot's bucket: a thread's 16 consecutive slots find theirs by one
    // binary search over the bucket starts and a forward walk
    {
        const int s0 = threadIdx.x * 16;
        const uint4 q = *(const uint4*)(P.cnt + b0 + s0);
        __syncthreads();
        const int nv = to[SHB_NB];
        uint32_t c[16];
        const uint32_t wd[4] = {q.x, q.y, q.z, q.w};
        uint32_t sum = 0;
#pragma unroll
        for (int k = 0; k < 16; k++) {
            c[k] = (s0 + k < nv) ? (wd[k >> 2] >> (8 * (k & 3))) & 0xFFu : 0u;
            sum += c[k];
        }
        uint32_t tot;
        uint32_t off = shw_block_excl<BK_TPB>(sum, ws, &tot);
        int d = 0;  // the last bucket whose start is <= s0
        {
            int lo = 0, hi = SHB_NB - 1;
            while (lo < hi) {
                const int mid = (lo + hi + 1) >> 1;
                if ((int)to[mid] <= s0) lo = mid;
                else hi = mid - 1;
            }
            d = lo;
        }
#pragma unroll
        for (int k = 0; k < 16; k++) {
            while (d < SHB_NB - 1 && (int)to[d + 1] <= s0 + k) d++;
            pfx[s0 + k] = off | ((uint32_t)d << BK_PFX_BITS);
            off += c[k];
        }
        if (threadIdx.x == 0) pfx[SHB_TILE] = tot;
        __syncthreads();
    }
    // 2. counts (4 packed per register) and match-stream positions of the wave's events
    uint32_t cp[BK_ITEMS / 4];
    uint32_t mp[BK_ITEMS];
    uint32_t mine = 0;
#pragma unroll
    for (int j = 0; j < BK_ITEMS; j++) {
        uint32_t c = 0;
        mp[j] = 0u;
        if (sl[j] != BK_NOSLOT) {
            const uint32_t s = sl[j];
            const uint32_t pw = pfx[s];
            const uint32_t d = pw >> BK_PFX_BITS;
            const uint32_t ps = pw & BK_PFX_MASK;
            c = (pfx[s + 1] & BK_PFX_MASK) - ps;
            mp[j] = ms0[d] + ps - (pfx[to[d]] & BK_PFX_MASK);
        }
        if ((j & 3) == 0) cp[j >> 2] = 0u;
        cp[j >> 2] |= c << (8 * (j & 3));
        mine += c;
    }
    {
        const uint32_t wsum = shw_last(shw_incl_scan(mine));
        if (lane == 0) wtot[w] = wsum;
    }
    __syncthreads();
    if (LM) {
#pragma unroll
        for (int j = 0; j < BK_ITEMS; j++) emp[w][j * 64 + lane] = mp[j];
    }
    uint64_t rb = s_tb;  // this wave's first row
    for (int q = 0; q < w; q++) rb += wtot[q];
    // 3. rows, one half (512 events) at a time
#pragma unroll
    for (int hf = 0; hf < BK_ITEMS / 8; hf++) {
        uint32_t carry = 0;
        uint32_t ro8[8];
#pragma unroll
        for (int jj = 0; jj < 8; jj++) {
            const int j = hf * 8 + jj;
            const uint32_t c = (cp[j >> 2] >> (8 * (j & 3))) & 0xFFu;
            const uint32_t incl = shw_incl_scan(c);
            const uint32_t ro = carry + incl - c;
            if (!LM) ro8[jj] = ro;
            const int e = jj * 64 + lane;
            if (!LM) emp[w][e] = mp[j];
            ero[w][e] = (uint16_t)ro;
            for (uint32_t k = 0; k < c; k++)
                if (ro + k < EROWS) rmap[w][ro + k] = (uint16_t)e;
            carry += shw_last(incl);
        }
        const uint32_t R = carry;
        const int64_t ib = b0 + (int64_t)w * (64 * BK_ITEMS) + hf * BK_EHALF;  // arrival index of event 0 of the half
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const int eo = LM ? hf * BK_EHALF : 0;  // the half's first entry of emp
        if (R <= EROWS) {
            // row-parallel: lane t writes rows t, t + 64, ... (consecutive lanes,
            // consecutive rows); BK_RU rows' loads go out before their stores
            if (NO > 0) {
                for (uint32_t t0 = 0; t0 < R; t0 += 64 * BK_RU) {
                    int64_t v[BK_RU][NV];
                    int64_t ii[BK_RU];
                    bool ok[BK_RU];
#pragma unroll
                    for (int u = 0; u < BK_RU; u++) {
                        const uint32_t t = t0 + u * 64 + lane;
                        ok[u] = t < R && (int64_t)rb + t < out_cap;  // (past out_cap: the host reports SH_E_MORE)
                        ii[u] = ib;
                        if (ok[u]) {
                            const int e = rmap[w][t];
                            const uint32_t k = t - ero[w][e];
                            ii[u] = ib + e;
                            bk_vals<NV>(O, ii[u], (int64_t)emp[w][eo + e] + k, (int64_t)rb + t, v[u]);
                        }
                    }
#pragma unroll
                    for (int u = 0; u < BK_RU; u++)
                        if (ok[u])
                            bk_store<MODE, NV>(OC, (int64_t)rb + t0 + u * 64 + lane, v[u],
                                                           seq_base + (uint64_t)ii[u], out_seq, out_vals);
                }
            } else {
                for (uint32_t t = lane; t < R; t += 64) {
                    const int e = rmap[w][t];
                    const uint32_t k = t - ero[w][e];
                    const int64_t i = ib + e;
                    const int64_t row = (int64_t)rb + t;
                    if (row >= out_cap) continue;  // the host reports SH_E_MORE
                    bk_row<MODE, NO>(O, OC, o_kind, o_type, o_src, row, i, (int64_t)emp[w][eo + e] + k,
                                     seq_base + (uint64_t)i, out_seq, out_vals);
                }
            }
        } else {
            // a dense half (more rows than the map holds): each event writes its rows
            // (LM: its first row from the same scan again, not kept in registers)
            uint32_t carry2 = 0;
#pragma unroll
            for (int jj = 0; jj < 8; jj++) {
                const int j = hf * 8 + jj;
                const uint32_t c = (cp[j >> 2] >> (8 * (j & 3))) & 0xFFu;
                const int64_t i = ib + jj * 64 + lane;
                uint32_t ro = 0;
                if (LM) {
                    const uint32_t incl = shw_incl_scan(c);
                    ro = carry2 + incl - c;
                    carry2 += shw_last(incl);
                } else {
                    ro = ro8[jj];
                }
                for (uint32_t k = 0; k < c; k++) {
                    const int64_t row = (int64_t)rb + ro + k;
                    if (row >= out_cap) break;
                    bk_row<MODE, NO>(O, OC, o_kind, o_type, o_src, row, i,
                                     (int64_t)(LM ? emp[w][j * 64 + lane] : mp[j]) + k,
                                     seq_base + (uint64_t)i, out_seq, out_vals);
                }
            }
        }
        rb += R;
        // the map is rewritten by the next half: this wave's reads come first
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
}

// ---------------------------------------------------------------- halo bound
// hstart[T] <- the first halo tile of a matcher pass whose chunk starts at tile
// T: tile T - 1, and before it every tile whose successor starts within W of
// tile T's first event (for streams in time order, every tile that can hold an
// event the window reaches), at most SHB_HMAX. One thread per tile.
__global__ void __launch_bounds__(256) k_bk_halo(const int64_t* __restrict__ tfirst, int32_t* __restrict__ hstart,
                                                 int32_t nt, int64_t within) {
    const int t = blockIdx.x * 256 + threadIdx.x;
    if (t >= nt) return;
    const int64_t ta = tfirst[t];
    const int64_t tlim = ta < INT64_MIN + within ? INT64_MIN : ta - within;
    int h = t > 0 ? 1 : 0;
    while (h < t && h < SHB_HMAX && tfirst[t - h] >= tlim) h++;
    hstart[t] = t - h;
}

// tpre[T] <- the latest timestamp of the tiles before T (exclusive prefix max,
// INT64_MIN for tile 0): the matcher's proof that a walk leaving its key's run
// saw every event of the key inside the window. One workgroup, each thread a
// contiguous run of tiles (independent loads), one LDS scan.
__global__ void __launch_bounds__(1024) k_bk_tpre(int64_t* __restrict__ tpre, int32_t nt) {
    __shared__ int64_t s[1024];
    const int per = (nt + 1023) / 1024;
    const int t0 = threadIdx.x * per;
    int64_t m = INT64_MIN;
    for (int t = t0; t < t0 + per && t < nt; t++) m = tpre[t] > m ? tpre[t] : m;
    s[threadIdx.x] = m;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {
        const int64_t y = threadIdx.x >= (unsigned)o ? s[threadIdx.x - o] : INT64_MIN;
        __syncthreads();
        if (y > s[threadIdx.x]) s[threadIdx.x] = y;
        __syncthreads();
    }
    int64_t run = threadIdx.x ? s[threadIdx.x - 1] : INT64_MIN;  // tiles before t0
    for (int t = t0; t < t0 + per && t < nt; t++) {
        const int64_t v = tpre[t];
        tpre[t] = run;
        run = v > run ? v : run;
    }
}

// ---------------------------------------------------------------- sequence carry
// The rise-and-fall sequence `every e1=S, e2=S[f2(x, e1)]+, e3=S[f3(x, e2[last])]`
// (nf_query.s3; SEQUENCE semantics make each key's state ONE partial: k_seq3s in
// sh_nfa.hip states the per-event step, CountPreStateProcessor.java:52-193,
// StreamPreStateProcessor.java:325-403). Per event x of a key:
//   hit = (a last e2 exists) && f3(x, last)   -> one match (e1, last, x)
//   else if (an e1 exists) && f2(x, e1)       -> last = x (the e2 run grows)
//   else                                      -> e1 = x, no last (every: a new start)
// The sequence has no window, so a key's state runs over the whole stream. One
// workgroup per key bucket walks the bucket's segments of every tile in order,
// in chunks of at most S3B_CH events, with the state of each of its keys in LDS:
// a chunk is sorted stably by local key (two 6-bit passes of wave ballots), the
// first event of each key run steps through the run, and the chunk's matches go
// out in arrival order: count 0/1 at the event's slot, the e1 / last values in
// the slot range of the event's (tile, bucket) segment (at most one match per
// event, so the segment's slots hold its matches), the segment's first match
// position and the tile's matches. k_bk_emit then writes the ordered rows.
#define S3B_TPB 1024
#define S3B_CH 4096
#define S3B_NR (S3B_CH / S3B_TPB)
#define S3B_NK 4096  // local keys per bucket (kb <= 12)
#define S3B_W (S3B_TPB / 64)

__device__ __forceinline__ NfVal s3b_val(uint32_t b, int t) {
    NfVal v;
    v.t = (uint8_t)t;
    v.null = 0;
    v.b = t == SH_T_INT ? (int64_t)(int32_t)b : (int64_t)b;
    return v;
}

// one stable multisplit pass over 6 bits of the local key: the chunk positions
// in `in` order (identity when in == nullptr) -> `out`
__device__ __forceinline__ void s3b_sort_pass(const uint32_t* __restrict__ c_key, const uint16_t* in,
                                              uint16_t* out, int L, int sh, uint32_t (*wc)[64], uint32_t* ws) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
    for (int c = threadIdx.x; c < S3B_W * 64; c += S3B_TPB) (&wc[0][0])[c] = 0u;
    __syncthreads();
    uint32_t rk[S3B_NR], dg[S3B_NR], ix[S3B_NR];
#pragma unroll
    for (int r = 0; r < S3B_NR; r++) {
        const int pos = (w * S3B_NR + r) * 64 + lane;  // wave w owns positions [w * 256, w * 256 + 256)
        const bool valid = pos < L;
        ix[r] = valid ? (in ? (uint32_t)in[pos] : (uint32_t)pos) : 0u;
        const uint32_t d = valid ? (c_key[ix[r]] >> sh) & 63u : 0u;
        uint64_t peers = __ballot(valid);
#pragma unroll
        for (int bb = 0; bb < 6; bb++) {
            const bool bit = (d >> bb) & 1u;
            const uint64_t m = __ballot(valid && bit);
            peers &= bit ? m : ~m;
        }
        const uint32_t r_ = (uint32_t)__popcll(peers & lt);
        const uint32_t base = valid ? wc[w][d] : 0u;
        if (valid && r_ == 0) wc[w][d] = base + (uint32_t)__popcll(peers);
        rk[r] = valid ? base + r_ : ~0u;
        dg[r] = d;
    }
    __syncthreads();
    // (digit, wave) exclusive offsets: thread t = digit * 16 + wave
    {
        const int d = threadIdx.x >> 4, q = threadIdx.x & 15;
        uint32_t tot;
        const uint32_t ex = shw_block_excl<S3B_TPB>(wc[q][d], ws, &tot);
        __syncthreads();
        wc[q][d] = ex;
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < S3B_NR; r++)
        if (rk[r] != ~0u) out[wc[w][dg[r]] + rk[r]] = (uint16_t)ix[r];
    __syncthreads();
}

// one stable multisplit pass over the low 8 bits of the local key (kb <= 8: the whole
// key in one pass instead of two 6-bit ones); wc8: S3B_W x 256 counters
__device__ __forceinline__ void s3b_sort_pass8(const uint32_t* __restrict__ c_key, uint16_t* out, int L,
                                               uint32_t (*wc8)[256], uint32_t* ws) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
    for (int c = threadIdx.x; c < S3B_W * 256; c += S3B_TPB) (&wc8[0][0])[c] = 0u;
    __syncthreads();
    uint32_t rk[S3B_NR], dg[S3B_NR];
#pragma unroll
    for (int r = 0; r < S3B_NR; r++) {
        const int pos = (w * S3B_NR + r) * 64 + lane;  // wave w owns positions [w * 256, w * 256 + 256)
        const bool valid = pos < L;
        const uint32_t d = valid ? c_key[pos] & 255u : 0u;
        uint64_t peers = __ballot(valid);
#pragma unroll
        for (int bb = 0; bb < 8; bb++) {
            const bool bit = (d >> bb) & 1u;
            const uint64_t m = __ballot(valid && bit);
            peers &= bit ? m : ~m;
        }
        const uint32_t r_ = (uint32_t)__popcll(peers & lt);
        const uint32_t base = valid ? wc8[w][d] : 0u;
        if (valid && r_ == 0) wc8[w][d] = base + (uint32_t)__popcll(peers);
        rk[r] = valid ? base + r_ : ~0u;
        dg[r] = d;
    }
    __syncthreads();
    // (digit, wave) exclusive offsets, digit-major: thread t takes digit t / 4, waves
    // 4 (t % 4) .. 4 (t % 4) + 3
    {
        const int d = threadIdx.x >> 2, q0 = (threadIdx.x & 3) * 4;
        uint32_t v[4], sum = 0;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            v[k] = wc8[q0 + k][d];
            sum += v[k];
        }
        uint32_t tot;
        uint32_t ex = shw_block_excl<S3B_TPB>(sum, ws, &tot);
        __syncthreads();
#pragma unroll
        for (int k = 0; k < 4; k++) {
            wc8[q0 + k][d] = ex;
            ex += v[k];
        }
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < S3B_NR; r++)
        if (rk[r] != ~0u) out[wc8[w][dg[r]] + rk[r]] = (uint16_t)((w * S3B_NR + r) * 64 + lane);
    __syncthreads();
}

__global__ void __launch_bounds__(S3B_TPB) k_s3b(shb_plan P, shb_s3 S) {
    __shared__ uint32_t st_e1[S3B_NK], st_last[S3B_NK];
    __shared__ uint8_t st_f[S3B_NK];  // bit 0: an e1, bit 1: a last e2
    __shared__ uint32_t c_key[S3B_CH], c_val[S3B_CH];
    __shared__ uint16_t o_a[S3B_CH], o_b[S3B_CH];
    __shared__ uint32_t m_v0[S3B_CH], m_v1[S3B_CH];
    __shared__ uint16_t m_pre[S3B_CH];  // 0/1 per event, then its exclusive prefix over the chunk
    __shared__ uint32_t wc[S3B_W][64];
    __shared__ uint32_t ws[S3B_W];
    __shared__ uint32_t seg_p[SHB_CT_MAX + 1], seg_g[SHB_CT_MAX];
    __shared__ uint8_t seg_of[S3B_CH / 32];
    const int b = blockIdx.x;
    const int kb = P.kb;
    const uint32_t kmask = (1u << kb) - 1u;
    const int t = S.type;
    for (int k = threadIdx.x; k < S3B_NK; k += S3B_TPB) st_f[k] = 0;
    const uint32_t* __restrict__ gcol = (const uint32_t*)P.st_dst[0];
    uint32_t warm = 0u;  // the warming reads, consumed by an empty asm at the end
    unsigned long long t_prev = wall_clock64();
#define S3B_PROF(ph)                                                                 \
    if (P.prof && threadIdx.x == 0) {                                                \
        const unsigned long long t_now = wall_clock64();                             \
        atomicAdd(&P.prof[ph], t_now - t_prev);                                      \
        t_prev = t_now;                                                              \
    }
    for (int a = 0; a < P.nt;) {
        __syncthreads();
        // the bucket's segments of tiles [a, a + SHB_CT_MAX), their prefix
        const int nseg = P.nt - a < SHB_CT_MAX ? P.nt - a : SHB_CT_MAX;
        uint32_t len = 0u, g = 0u;
        if ((int)threadIdx.x < nseg) {
            const int T = a + (int)threadIdx.x;
            const uint32_t lo = P.tofft[(int64_t)b * P.tstride + T], hi = P.tofft[(int64_t)(b + 1) * P.tstride + T];
            len = hi - lo;
            g = ((uint32_t)T << SHB_TILE_SHIFT) + lo;
        }
        {
            uint32_t tot;
            const uint32_t pre = shw_block_excl<S3B_TPB>(len, ws, &tot);
            if ((int)threadIdx.x < nseg) {
                seg_p[threadIdx.x] = pre;
                seg_g[threadIdx.x] = g;
            }
            if ((int)threadIdx.x == nseg) seg_p[nseg] = tot;
        }
        __syncthreads();
        // this chunk: tiles [a, a + ne), at most S3B_CH events
        const int ne = __syncthreads_count((int)threadIdx.x < nseg && seg_p[threadIdx.x + 1] <= S3B_CH);
        if (ne == 0) {
            if (threadIdx.x == 0) atomicOr(P.flag, SHB_F_SPAN);
            return;  // (uniform) the host reruns on the general engine
        }
        const int L = (int)seg_p[ne];
        // the next chunk's bucket starts, loaded now and used after the sort (the
        // warming reads of its segments then overlap this chunk's walk)
        uint32_t nlo = 0u, nhi = 0u;
        const int Tn = a + ne + (int)threadIdx.x;
        if (S.warm && (int)threadIdx.x < SHB_CT_MAX && Tn < P.nt) {
            nlo = P.tofft[(int64_t)b * P.tstride + Tn];
            nhi = P.tofft[(int64_t)(b + 1) * P.tstride + Tn];
        }
        for (int j = (int)threadIdx.x; j * 32 < L; j += S3B_TPB) {
            const uint32_t e = (uint32_t)j * 32u;
            int lo = 0, hi = ne - 1;
            while (lo < hi) {
                const int mid = (lo + hi + 1) >> 1;
                if (seg_p[mid] <= e) lo = mid;
                else hi = mid - 1;
            }
            seg_of[j] = (uint8_t)lo;
        }
        __syncthreads();
#define S3B_GIDX(i, out) { int sg_ = seg_of[(i) >> 5]; while (seg_p[sg_ + 1] <= (uint32_t)(i)) sg_++; \
    out = seg_g[sg_] + ((uint32_t)(i) - seg_p[sg_]); }
        // the chunk's events (arrival order inside the bucket)
#pragma unroll
        for (int k = 0; k < S3B_NR; k++) {
            const int i = k * S3B_TPB + (int)threadIdx.x;
            if (i < L) {
                uint32_t gi;
                S3B_GIDX(i, gi)
                c_key[i] = P.w0[gi] & kmask;
                c_val[i] = gcol[gi];
            }
        }
        __syncthreads();
        S3B_PROF(0)
        // stable sort by local key
        const uint16_t* srt;
        if (kb <= 6) {
            s3b_sort_pass(c_key, nullptr, o_a, L, 0, wc, ws);
            srt = o_a;
        } else {
            s3b_sort_pass(c_key, nullptr, o_a, L, 0, wc, ws);
            s3b_sort_pass(c_key, o_a, o_b, L, 6, wc, ws);
            srt = o_b;
        }
        S3B_PROF(1)
        if (nhi > nlo) {
            const uint32_t g = ((uint32_t)Tn << SHB_TILE_SHIFT) + nlo;
            warm ^= P.w0[g] ^ gcol[g];
            if (nhi - nlo > 32u) warm ^= P.w0[g + 32u] ^ gcol[g + 32u];
        }
        // the first event of each key run steps through the run
        for (int q = threadIdx.x; q < L; q += S3B_TPB) {
            const uint32_t ci = srt[q];
            const uint32_t key = c_key[ci];
            if (q > 0 && c_key[srt[q - 1]] == key) continue;
            uint32_t f = st_f[key], e1b = st_e1[key], lastb = st_last[key];
            // a float attribute compared as float both times (C3's shape): the compares
            // without the generic value / domain dispatch -- k_s3b 3.69 -> 2.78 ms
            // (profiles/r6_c3_s3b_f32_ab.txt)
            const bool f32 = t == SH_T_FLOAT && S.dom2 == DOM_F32 && S.dom3 == DOM_F32;
            for (int r = q; r < L; r++) {
                const uint32_t cr = r == q ? ci : srt[r];
                if (r > q && c_key[cr] != key) break;
                const uint32_t xb = c_val[cr];
                bool hit, grow;
                if (f32) {
                    const float x = __uint_as_float(xb);
                    hit = (f & 2u) && nf_cmp_op<float>(S.op3, x, __uint_as_float(lastb));
                    grow = !hit && (f & 1u) && nf_cmp_op<float>(S.op2, x, __uint_as_float(e1b));
                } else {
                    const NfVal x = s3b_val(xb, t);
                    hit = (f & 2u) && nf_cmp(S.op3, S.dom3, x, s3b_val(lastb, t));
                    grow = !hit && (f & 1u) && nf_cmp(S.op2, S.dom2, x, s3b_val(e1b, t));
                }
                m_pre[cr] = hit ? 1 : 0;
                if (hit) {  // (the outputs read the values of matching events only)
                    m_v0[cr] = e1b;
                    m_v1[cr] = lastb;
                }
                if (grow) {
                    f |= 2u;
                    lastb = xb;
                } else {
                    f = 1u;
                    e1b = xb;
                }
            }
            st_f[key] = (uint8_t)f;
            st_e1[key] = e1b;
            st_last[key] = lastb;
        }
        __syncthreads();
        S3B_PROF(2)
        // matches: exclusive prefix over the chunk in arrival order (4 per thread)
        uint32_t total;
        {
            const int p0 = (int)threadIdx.x * S3B_NR;
            uint32_t v[S3B_NR], sum = 0;
#pragma unroll
            for (int q = 0; q < S3B_NR; q++) {
                v[q] = p0 + q < L ? (uint32_t)m_pre[p0 + q] : 0u;
                sum += v[q];
            }
            uint32_t off = shw_block_excl<S3B_TPB>(sum, ws, &total);
#pragma unroll
            for (int q = 0; q < S3B_NR; q++) {
                if (p0 + q < L) {
                    uint32_t gi;
                    S3B_GIDX(p0 + q, gi)
                    P.cnt[gi] = (uint8_t)v[q];
                    m_pre[p0 + q] = (uint16_t)off;
                }
                off += v[q];
            }
        }
        __syncthreads();
        // per tile: its segment's matches start at the segment's first slot
        for (int sg = threadIdx.x; sg < ne; sg += S3B_TPB) {
            const uint32_t x0 = seg_p[sg], x1 = seg_p[sg + 1];
            const uint32_t q0 = x0 < (uint32_t)L ? (uint32_t)m_pre[x0] : total;
            const uint32_t q1 = x1 < (uint32_t)L ? (uint32_t)m_pre[x1] : total;
            const int T = a + sg;
            P.mstart[(int64_t)T * SHB_NB + b] = seg_g[sg];
            if (q1 > q0) atomicAdd(&P.ttot[T], q1 - q0);
        }
        // the matches' e1 / last values, compact inside their segment's slots
        for (int i = threadIdx.x; i < L; i += S3B_TPB) {
            const uint32_t pre = m_pre[i];
            const uint32_t nxt = i + 1 < L ? (uint32_t)m_pre[i + 1] : total;
            if (nxt == pre) continue;
            int sg = seg_of[i >> 5];
            while (seg_p[sg + 1] <= (uint32_t)i) sg++;
            const uint32_t s0 = seg_p[sg];
            const uint32_t q0 = s0 < (uint32_t)L ? (uint32_t)m_pre[s0] : total;
            const int64_t dst = (int64_t)seg_g[sg] + (pre - q0);
            for (int m = 0; m < S.n_ms; m++) ((uint32_t*)P.ms[m])[dst] = S.ms_slot[m] == 0 ? m_v0[i] : m_v1[i];
        }
#undef S3B_GIDX
        S3B_PROF(3)
        a += ne;
    }
#undef S3B_PROF
    if (S.warm) asm volatile("" ::"v"(warm));
}

// ---------------------------------------------------------------- aggregate carry
// Select-clause aggregators of the bucketed window engine (C2 select variant ii):
// one running value per partition key and output, added in the reference's order
// -- the key's matches in trigger order, each consumer's matches in partial
// creation order (AttributeAggregatorExecutor state per partition key;
// SumAttributeAggregatorExecutor.java:167-185: sum(int|long) -> long with Java
// wrap-around, sum(float|double) -> double, value += (double) x;
// AvgAttributeAggregatorExecutor.java:145-155: the double sum / count;
// count() -> long). One workgroup per key bucket walks the bucket's segments of
// every tile in order (chunks of at most AGC_CH events), with every local key's
// running values in LDS: per chunk the events' counts (cnt, at their slots) give
// each consumer its rows -- a prefix over the chunk, and the match-stream position
// mstart[T][b] + the prefix inside its (tile, bucket) segment; the e1-side
// arguments of the chunk's rows are gathered into LDS; a stable sort by local key
// puts each key's consumers together in arrival order and the first consumer of
// each key run adds them all in sequence, writing the running values by match-
// stream position (k_bk_emit writes them into the rows). No exactness proof is
// needed: the additions are the reference's own sequence.
#define AGC_TPB 1024
#define AGC_CH 4096
#define AGC_NR (AGC_CH / AGC_TPB)
#define AGC_ROWS 8192  // rows of a chunk whose e1-side arguments fit LDS (more: SHB_F_AGG)

__device__ __forceinline__ int64_t agc_load(const void* p, int64_t i, int type) {
    return (type == SH_T_LONG || type == SH_T_DOUBLE) ? ((const int64_t*)p)[i] : (int64_t)((const uint32_t*)p)[i];
}

// one running value: sum(int|long) in long, the rest in double (bits)
__device__ __forceinline__ void agc_add(int kind, int type, int64_t& acc, int64_t x) {
    if (kind == SH_AGG_SUM && (type == SH_T_INT || type == SH_T_LONG)) {
        const int64_t v = type == SH_T_INT ? (int64_t)(int32_t)x : x;
        acc = (int64_t)((uint64_t)acc + (uint64_t)v);
        return;
    }
    double d;
    switch (type) {
        case SH_T_INT: d = (double)(int32_t)x; break;
        case SH_T_LONG: d = (double)x; break;
        case SH_T_FLOAT: d = (double)__uint_as_float((uint32_t)x); break;
        default: d = __longlong_as_double(x);
    }
    acc = __double_as_longlong(__longlong_as_double(acc) + d);
}

__global__ void __launch_bounds__(AGC_TPB) k_bk_aggc(shb_plan P, shb_aggc A) {
    __shared__ int64_t st_acc[SHB_MAX_AGG][256];
    __shared__ int64_t st_cnt[256];
    __shared__ uint32_t c_key[AGC_CH];   // local key | count << 16
    __shared__ uint16_t c_pre[AGC_CH];   // the consumer's first row in the chunk
    __shared__ uint32_t c_mp[AGC_CH];    // ... and its match-stream position
    __shared__ int64_t c_e2w[AGC_CH];    // e2-side argument, column 0 (any width)
    __shared__ uint32_t c_e2n[AGC_CH];   // e2-side argument, column 1 (4-byte)
    __shared__ uint32_t r_e1[AGC_ROWS];  // e1-side argument per row of the chunk
    __shared__ uint16_t o_a[AGC_CH], o_b[AGC_CH];
    __shared__ uint32_t wc[AGC_TPB / 64][64];
    __shared__ uint32_t ws[AGC_TPB / 64];
    __shared__ uint32_t seg_p[SHB_CT_MAX + 1], seg_g[SHB_CT_MAX];
    __shared__ uint8_t seg_of[AGC_CH / 32];
    const int b = blockIdx.x;
    const int kb = P.kb;
    const uint32_t kmask = (1u << kb) - 1u;
    for (int k = threadIdx.x; k < 256; k += AGC_TPB) {
        st_cnt[k] = 0;
        for (int o = 0; o < SHB_MAX_AGG; o++) st_acc[o][k] = 0;  // 0 == long 0 == double +0.0
    }
    const void* e1src = A.e1_col >= 0 ? P.ms[A.e1_col] : nullptr;
    const void* e2src = A.e2_col[0] >= 0 ? P.st_dst[A.e2_col[0]] : nullptr;
    const void* e2srn = A.e2_col[1] >= 0 ? P.st_dst[A.e2_col[1]] : nullptr;
    unsigned long long t_prev = wall_clock64();
#define AGC_PROF(ph)                                                                 \
    if (P.prof && threadIdx.x == 0) {                                                \
        const unsigned long long t_now = wall_clock64();                             \
        atomicAdd(&P.prof[8 + (ph)], t_now - t_prev);                                \
        t_prev = t_now;                                                              \
    }
    for (int a = 0; a < P.nt;) {
        __syncthreads();
        const int nseg = P.nt - a < SHB_CT_MAX ? P.nt - a : SHB_CT_MAX;
        uint32_t len = 0u, g = 0u;
        if ((int)threadIdx.x < nseg) {
            const int T = a + (int)threadIdx.x;
            const uint32_t lo = P.tofft[(int64_t)b * P.tstride + T], hi = P.tofft[(int64_t)(b + 1) * P.tstride + T];
            len = hi - lo;
            g = ((uint32_t)T << SHB_TILE_SHIFT) + lo;
        }
        {
            uint32_t tot;
            const uint32_t pre = shw_block_excl<AGC_TPB>(len, ws, &tot);
            if ((int)threadIdx.x < nseg) {
                seg_p[threadIdx.x] = pre;
                seg_g[threadIdx.x] = g;
            }
            if ((int)threadIdx.x == nseg) seg_p[nseg] = tot;
        }
        __syncthreads();
        const int ne = __syncthreads_count((int)threadIdx.x < nseg && seg_p[threadIdx.x + 1] <= AGC_CH);
        if (ne == 0) {
            if (threadIdx.x == 0) atomicOr(P.flag, SHB_F_AGG);
            return;  // (uniform) the host runs the post-pass instead
        }
        const int L = (int)seg_p[ne];
        for (int j = (int)threadIdx.x; j * 32 < L; j += AGC_TPB) {
            const uint32_t e = (uint32_t)j * 32u;
            int lo = 0, hi = ne - 1;
            while (lo < hi) {
                const int mid = (lo + hi + 1) >> 1;
                if (seg_p[mid] <= e) lo = mid;
                else hi = mid - 1;
            }
            seg_of[j] = (uint8_t)lo;
        }
        __syncthreads();
        AGC_PROF(0)
        // the chunk's consumers (arrival order inside the bucket): key, count, e2 argument
        uint32_t cc[AGC_NR];
        int sgi[AGC_NR];
#pragma unroll
        for (int k = 0; k < AGC_NR; k++) {
            const int i = (int)threadIdx.x * AGC_NR + k;  // 4 consecutive events per thread
            cc[k] = 0u;
            sgi[k] = 0;
            if (i < L) {
                int sg = seg_of[i >> 5];
                while (seg_p[sg + 1] <= (uint32_t)i) sg++;
                sgi[k] = sg;
                const uint32_t gi = seg_g[sg] + ((uint32_t)i - seg_p[sg]);
                cc[k] = P.cnt[gi];
                c_key[i] = (P.w0[gi] & kmask) | (cc[k] << 16);
                if (e2src) c_e2w[i] = agc_load(e2src, gi, A.e2_type[0]);
                if (e2srn) c_e2n[i] = ((const uint32_t*)e2srn)[gi];
            }
        }
        // rows: exclusive prefix over the chunk
        uint32_t total;
        {
            uint32_t sum = 0;
#pragma unroll
            for (int k = 0; k < AGC_NR; k++) sum += cc[k];
            uint32_t off = shw_block_excl<AGC_TPB>(sum, ws, &total);
#pragma unroll
            for (int k = 0; k < AGC_NR; k++) {
                const int i = (int)threadIdx.x * AGC_NR + k;
                if (i < L) c_pre[i] = (uint16_t)off;
                off += cc[k];
            }
        }
        if (total > AGC_ROWS) {
            if (threadIdx.x == 0) atomicOr(P.flag, SHB_F_AGG);
            return;  // (uniform: total is the block sum)
        }
        __syncthreads();
        AGC_PROF(1)
        // match-stream positions (the segment's first match + the prefix inside it)
        // and the e1-side arguments of the rows
#pragma unroll
        for (int k = 0; k < AGC_NR; k++) {
            const int i = (int)threadIdx.x * AGC_NR + k;
            if (i >= L) continue;
            const int sg = sgi[k];
            const uint32_t mp = P.mstart[(int64_t)(a + sg) * SHB_NB + b] + c_pre[i] - c_pre[seg_p[sg]];
            c_mp[i] = mp;
            if (e1src)
                for (uint32_t q = 0; q < cc[k]; q++) r_e1[c_pre[i] + q] = (uint32_t)((const uint32_t*)e1src)[mp + q];
        }
        __syncthreads();
        AGC_PROF(2)
        // stable sort by local key (kb <= 8: 6 bits, then the high bits)
        const uint16_t* srt = o_a;
        s3b_sort_pass(c_key, nullptr, o_a, L, 0, wc, ws);  // (digits of the low 12 bits: the key)
        if (kb > 6) {
            s3b_sort_pass(c_key, o_a, o_b, L, 6, wc, ws);
            srt = o_b;
        }
        AGC_PROF(3)
        // the first consumer of each key run adds the run's rows in sequence
        for (int q = threadIdx.x; q < L; q += AGC_TPB) {
            const uint32_t ci = srt[q];
            const uint32_t key = c_key[ci] & 0xFFFFu;
            if (q > 0 && (c_key[srt[q - 1]] & 0xFFFFu) == key) continue;
            int64_t acc[SHB_MAX_AGG];
#pragma unroll
            for (int o = 0; o < SHB_MAX_AGG; o++) acc[o] = st_acc[o][key];
            int64_t n = st_cnt[key];
            for (int r = q; r < L; r++) {
                const uint32_t cr = r == q ? ci : srt[r];
                const uint32_t kw = c_key[cr];
                if (r > q && (kw & 0xFFFFu) != key) break;
                const uint32_t c = kw >> 16;
                const uint32_t r0 = c_pre[cr], mp = c_mp[cr];
                const int64_t x2 = e2src ? c_e2w[cr] : 0;
                const int64_t x3 = e2srn ? (int64_t)c_e2n[cr] : 0;
                for (uint32_t m = 0; m < c; m++) {
                    n++;
                    const int64_t x1 = e1src ? (int64_t)r_e1[r0 + m] : 0;
#pragma unroll
                    for (int o = 0; o < SHB_MAX_AGG; o++) {
                        if (o >= A.n) break;
                        const int kind = A.kind[o];
                        int64_t v;
                        if (kind == SH_AGG_COUNT) {
                            v = n;
                        } else {
                            const int sd = A.side[o];
                            agc_add(kind, sd == 0 ? A.e1_type : A.e2_type[sd - 1], acc[o],
                                    sd == 0 ? x1 : (sd == 1 ? x2 : x3));
                            v = kind == SH_AGG_AVG
                                    ? __double_as_longlong(__longlong_as_double(acc[o]) / (double)n)
                                    : acc[o];
                        }
                        ((int64_t*)A.out[o])[(int64_t)mp + m] = v;
                    }
                }
            }
#pragma unroll
            for (int o = 0; o < SHB_MAX_AGG; o++) st_acc[o][key] = acc[o];
            st_cnt[key] = n;
        }
        __syncthreads();
        AGC_PROF(4)
        a += ne;
    }
#undef AGC_PROF
}

// the aggregate carry with the additions in parallel (k_bk_aggp, the default carry):
// the chunk's consumers sorted by local key as in k_bk_aggc, then their rows in that
// order -- each key's rows of the chunk one contiguous run, in the reference's order --
// get a block-wide segmented prefix per output plus the key's running value from the
// earlier chunks. Exact by construction: sum(int | long) adds in 64-bit two's
// complement (Java's long wrap-around); the double additions (sum of float / double,
// avg of any type) run on 64-bit fixed point -- units of 2^-24 for float / double
// arguments, of 1 for int / long -- and every addend and every running value must be
// an integer number of units below 2^53 in magnitude, so each of Java's sequential
// double additions is exact and equals this sum (SumAttributeAggregatorExecutor.java
// :167-185, AvgAttributeAggregatorExecutor.java:145-155); a row that fails the test
// sets SHB_F_AGG and the host takes the post-pass.
#define AGP_ROWS 8192
#define AGP_LIM 9007199254740992.0  // 2^53

// output o's mode: 0 long wrap-around sum, 1 fixed-point double sum (avg: / count), 2 count
__device__ __forceinline__ int agp_mode(const shb_aggc& A, int o, int* type) {
    const int kind = A.kind[o];
    if (kind == SH_AGG_COUNT) return 2;
    const int sd = A.side[o];
    *type = sd == 0 ? A.e1_type : A.e2_type[sd - 1];
    if (kind == SH_AGG_SUM && (*type == SH_T_INT || *type == SH_T_LONG)) return 0;
    return 1;
}

// an addend in the output's units; false: not an exact fixed-point value
__device__ __forceinline__ bool agp_units(int mode, int type, int64_t x, int64_t* u) {
    if (mode == 0) {
        *u = type == SH_T_INT ? (int64_t)(int32_t)x : x;
        return true;
    }
    double d;
    switch (type) {
        case SH_T_INT: d = (double)(int32_t)x; break;
        case SH_T_LONG: d = (double)x; break;
        case SH_T_FLOAT: d = (double)__uint_as_float((uint32_t)x); break;
        default: d = __longlong_as_double(x);
    }
    if (type == SH_T_FLOAT || type == SH_T_DOUBLE) d *= 16777216.0;  // 2^24: exact
    if (!(d == d) || fabs(d) >= AGP_LIM || d != trunc(d)) return false;
    *u = (int64_t)d;
    return true;
}

__global__ void __launch_bounds__(AGC_TPB) k_bk_aggp(shb_plan P, shb_aggc A) {
    __shared__ int64_t st_acc[SHB_MAX_AGG][256];
    __shared__ int64_t st_cnt[256];
    __shared__ uint32_t c_key[AGC_CH];   // local key | count << 16
    __shared__ uint16_t c_pre[AGC_CH];   // the consumer's first row in the chunk (arrival order)
    __shared__ uint32_t c_mp[AGC_CH];    // ... its match-stream position
    __shared__ uint32_t c_gi[AGC_CH];    // ... its slot
    __shared__ uint16_t o_a[AGC_CH];
    __shared__ uint16_t rs[AGC_CH + 1];  // sorted consumer -> its first row in key order
    __shared__ uint16_t run_q[257];      // key run -> its first sorted consumer
    __shared__ int s_nruns;
    __shared__ uint16_t rq[AGP_ROWS];    // row in key order -> its sorted consumer
    __shared__ uint32_t wc8[AGC_TPB / 64][256];
    __shared__ uint32_t ws[AGC_TPB / 64];
    __shared__ uint32_t seg_p[SHB_CT_MAX + 1], seg_g[SHB_CT_MAX];
    __shared__ uint8_t seg_of[AGC_CH / 32];
    __shared__ int s_bad;
    const int b = blockIdx.x;
    const int kb = P.kb;
    const uint32_t kmask = (1u << kb) - 1u;
    const int lane = (int)(threadIdx.x & 63u), wv = (int)(threadIdx.x >> 6);
    for (int k = threadIdx.x; k < 256; k += AGC_TPB) {
        st_cnt[k] = 0;
        for (int o = 0; o < SHB_MAX_AGG; o++) st_acc[o][k] = 0;
    }
    if (threadIdx.x == 0) s_bad = 0;
    const uint32_t* e1src = A.e1_col >= 0 ? (const uint32_t*)P.ms[A.e1_col] : nullptr;
    const void* e2src = A.e2_col[0] >= 0 ? P.st_dst[A.e2_col[0]] : nullptr;
    const uint32_t* e2srn = A.e2_col[1] >= 0 ? (const uint32_t*)P.st_dst[A.e2_col[1]] : nullptr;
    unsigned long long t_prev = wall_clock64();
#define AGP_PROF(ph)                                                                 \
    if (P.prof && threadIdx.x == 0) {                                                \
        const unsigned long long t_now = wall_clock64();                             \
        atomicAdd(&P.prof[8 + (ph)], t_now - t_prev);                                \
        t_prev = t_now;                                                              \
    }
    for (int a = 0; a < P.nt;) {
        __syncthreads();
        const int nseg = P.nt - a < SHB_CT_MAX ? P.nt - a : SHB_CT_MAX;
        uint32_t len = 0u, g = 0u;
        if ((int)threadIdx.x < nseg) {
            const int T = a + (int)threadIdx.x;
            const uint32_t lo = P.tofft[(int64_t)b * P.tstride + T], hi = P.tofft[(int64_t)(b + 1) * P.tstride + T];
            len = hi - lo;
            g = ((uint32_t)T << SHB_TILE_SHIFT) + lo;
        }
        {
            uint32_t tot;
            const uint32_t pre = shw_block_excl<AGC_TPB>(len, ws, &tot);
            if ((int)threadIdx.x < nseg) {
                seg_p[threadIdx.x] = pre;
                seg_g[threadIdx.x] = g;
            }
            if ((int)threadIdx.x == nseg) seg_p[nseg] = tot;
        }
        __syncthreads();
        const int ne = __syncthreads_count((int)threadIdx.x < nseg && seg_p[threadIdx.x + 1] <= AGC_CH);
        if (ne == 0) {
            if (threadIdx.x == 0) atomicOr(P.flag, SHB_F_AGG);
            return;  // (uniform) the host runs the post-pass instead
        }
        const int L = (int)seg_p[ne];
        for (int j = (int)threadIdx.x; j * 32 < L; j += AGC_TPB) {
            const uint32_t e = (uint32_t)j * 32u;
            int lo = 0, hi = ne - 1;
            while (lo < hi) {
                const int mid = (lo + hi + 1) >> 1;
                if (seg_p[mid] <= e) lo = mid;
                else hi = mid - 1;
            }
            seg_of[j] = (uint8_t)lo;
        }
        __syncthreads();
        // the chunk's consumers (arrival order inside the bucket): key, count, slot
        uint32_t cc[AGC_NR], ms0[AGC_NR];
        int sgi[AGC_NR];
#pragma unroll
        for (int k = 0; k < AGC_NR; k++) {
            const int i = (int)threadIdx.x * AGC_NR + k;  // 4 consecutive events per thread
            cc[k] = 0u;
            sgi[k] = 0;
            ms0[k] = 0u;
            if (i < L) {
                int sg = seg_of[i >> 5];
                while (seg_p[sg + 1] <= (uint32_t)i) sg++;
                sgi[k] = sg;
                const uint32_t gi = seg_g[sg] + ((uint32_t)i - seg_p[sg]);
                ms0[k] = P.mstart[(int64_t)(a + sg) * SHB_NB + b];
                cc[k] = P.cnt[gi];
                c_key[i] = (P.w0[gi] & kmask) | (cc[k] << 16);
                c_gi[i] = gi;
            }
        }
        uint32_t total;
        {
            uint32_t sum = 0;
#pragma unroll
            for (int k = 0; k < AGC_NR; k++) sum += cc[k];
            uint32_t off = shw_block_excl<AGC_TPB>(sum, ws, &total);
#pragma unroll
            for (int k = 0; k < AGC_NR; k++) {
                const int i = (int)threadIdx.x * AGC_NR + k;
                if (i < L) c_pre[i] = (uint16_t)off;
                off += cc[k];
            }
        }
        if (total > AGP_ROWS) {
            if (threadIdx.x == 0) atomicOr(P.flag, SHB_F_AGG);
            return;  // (uniform: total is the block sum)
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < AGC_NR; k++) {
            const int i = (int)threadIdx.x * AGC_NR + k;
            if (i >= L) continue;
            c_mp[i] = ms0[k] + c_pre[i] - c_pre[seg_p[sgi[k]]];
        }
        __syncthreads();
        AGP_PROF(0)
        // stable sort by local key (kb <= 8: 6 bits, then the high bits)
        const uint16_t* srt = o_a;
        s3b_sort_pass8(c_key, o_a, L, wc8, ws);
        AGP_PROF(1)
        // rows in key order: each sorted consumer's first row, the row -> consumer map,
        // and the key runs (one per local key present: <= 256)
        {
            uint32_t c4[AGC_NR], sum = 0, nst = 0, stb = 0;
#pragma unroll
            for (int k = 0; k < AGC_NR; k++) {
                const int q = (int)threadIdx.x * AGC_NR + k;
                c4[k] = 0u;
                if (q < L) {
                    const uint32_t kw = c_key[srt[q]];
                    c4[k] = kw >> 16;
                    if (q == 0 || (c_key[srt[q - 1]] & 0xFFFFu) != (kw & 0xFFFFu)) {
                        stb |= 1u << k;
                        nst++;
                    }
                }
                sum += c4[k];
            }
            uint32_t tot2, nr;
            uint32_t off = shw_block_excl<AGC_TPB>(sum, ws, &tot2);
            uint32_t ro = shw_block_excl<AGC_TPB>(nst, ws, &nr);
#pragma unroll
            for (int k = 0; k < AGC_NR; k++) {
                const int q = (int)threadIdx.x * AGC_NR + k;
                if (q < L) {
                    rs[q] = (uint16_t)off;
                    for (uint32_t m = 0; m < c4[k]; m++) rq[off + m] = (uint16_t)q;
                    if (stb >> k & 1u) run_q[ro++] = (uint16_t)q;
                }
                off += c4[k];
            }
            if (threadIdx.x == 0) {
                run_q[nr] = (uint16_t)L;
                s_nruns = (int)nr;
            }
            rs[L] = (uint16_t)total;  // (L <= AGC_CH: the sentinel slot)
        }
        __syncthreads();
        AGP_PROF(2)
        // one wave per key run: 64 rows at a time, the count from the row's place in the
        // run, every sum an inclusive wave prefix on top of the key's running value
        {
            const int nruns = s_nruns;
            int type[SHB_MAX_AGG], mode[SHB_MAX_AGG];
#pragma unroll
            for (int o = 0; o < SHB_MAX_AGG; o++) {
                type[o] = SH_T_INT;
                mode[o] = o < A.n ? agp_mode(A, o, &type[o]) : 2;
            }
            bool bad = false;
            for (int ri = wv; ri < nruns; ri += AGC_TPB / 64) {
                const int q0 = run_q[ri], q1 = run_q[ri + 1];
                const int R0 = rs[q0], R1 = rs[q1];
                const uint32_t key = c_key[srt[q0]] & 0xFFFFu;
                int64_t acc[SHB_MAX_AGG];
#pragma unroll
                for (int o = 0; o < SHB_MAX_AGG; o++) acc[o] = st_acc[o][key];
                const int64_t n0 = st_cnt[key];
                for (int r0 = R0; r0 < R1; r0 += 64) {
                    const int r = r0 + lane;
                    const bool ok = r < R1;
                    uint32_t mp = 0u, gi = 0u, wp = 0u;
                    int64_t x1 = 0, x2 = 0, x3 = 0;
                    if (ok) {
                        const uint32_t q = rq[r];
                        const uint32_t cr = srt[q];
                        const uint32_t m = (uint32_t)(r - rs[q]);
                        mp = c_mp[cr] + m;
                        wp = mp;
                        gi = c_gi[cr];
                        if (e1src) x1 = (int64_t)e1src[mp];
                        if (e2src) x2 = agc_load(e2src, gi, A.e2_type[0]);
                        if (e2srn) x3 = (int64_t)e2srn[gi];
                    }
                    const int64_t n = n0 + (r + 1 - R0);
#pragma unroll
                    for (int o = 0; o < SHB_MAX_AGG; o++) {
                        if (o >= A.n) break;
                        int64_t* out = (int64_t*)A.out[o];
                        if (mode[o] == 2) {
                            if (ok) out[wp] = n;
                            continue;
                        }
                        const int sd = A.side[o];
                        int64_t u = 0;
                        if (ok) bad |= !agp_units(mode[o], type[o], sd == 0 ? x1 : (sd == 1 ? x2 : x3), &u);
                        u = (int64_t)shw_incl_scan64((uint64_t)u);
                        const int64_t v = (int64_t)((uint64_t)acc[o] + (uint64_t)u);
                        if (ok) {
                            if (mode[o] == 0) {
                                out[wp] = v;
                            } else {
                                double d = (double)v;
                                bad |= fabs(d) >= AGP_LIM;
                                if (type[o] == SH_T_FLOAT || type[o] == SH_T_DOUBLE) d *= 5.9604644775390625e-08;  // 2^-24: exact
                                if (A.kind[o] == SH_AGG_AVG) d = d / (double)n;
                                out[wp] = __double_as_longlong(d);
                            }
                        }
                        acc[o] = (int64_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)((uint64_t)v >> 32), 63) << 32) |
                                           (uint32_t)__builtin_amdgcn_readlane((int)v, 63));  // (rows past the run add 0)
                    }
                }
                if (lane == 0) {
#pragma unroll
                    for (int o = 0; o < SHB_MAX_AGG; o++) st_acc[o][key] = acc[o];
                    st_cnt[key] = n0 + (R1 - R0);
                }
            }
            if (bad) s_bad = 1;
        }
        __syncthreads();
        if (s_bad) {
            if (threadIdx.x == 0) atomicOr(P.flag, SHB_F_AGG);
            return;  // (uniform: read after the barrier) the host takes the post-pass
        }
        AGP_PROF(3)
        a += ne;
    }
#undef AGP_PROF
}

// ---------------------------------------------------------------- launches
static int bk_ok() { return hipGetLastError() == hipSuccess ? 0 : -3; }

// the tiles' bucket starts transposed (bucket-major): a matcher workgroup reads its
// bucket's starts over ~180 tiles as one contiguous run instead of one cache line
// per tile (64 tiles per workgroup, staged in LDS)
#define TT_T 64
__global__ void __launch_bounds__(256) k_bk_toff_t(const uint16_t* __restrict__ toff, int nt,
                                                   uint16_t* __restrict__ tofft, int stride) {
    __shared__ uint16_t s[TT_T][SHB_NB + 2];
    const int T0 = (int)blockIdx.x * TT_T;
    for (int i = threadIdx.x; i < TT_T * (SHB_NB + 1); i += 256) {
        const int t = i / (SHB_NB + 1), b = i - t * (SHB_NB + 1);
        s[t][b] = T0 + t < nt ? toff[(int64_t)(T0 + t) * SHB_TOFF + b] : (uint16_t)0;
    }
    __syncthreads();
    for (int i = threadIdx.x; i < (SHB_NB + 1) * TT_T; i += 256) {
        const int b = i / TT_T, t = i - b * TT_T;
        if (T0 + t < nt) tofft[(int64_t)b * stride + T0 + t] = s[t][b];
    }
}

extern "C" int shb_partition(const int32_t* keys, const int64_t* ts, int32_t nkeys, shb_plan* P, void* stream) {
    hipStream_t st = (hipStream_t)stream;
    // 1,024 threads, 8 events per lane: 61 VGPRs, 8 waves per SIMD (0.64 vs 0.79 ms on C2
    // for 512 threads x 16 events at 94 VGPRs, profiles/r4_c2_scatter_ab.txt)
    hipLaunchKernelGGL((k_bk_scatter<2, 1024>), dim3(bk_grid(P->nt)), dim3(1024), 0, st, keys, ts, nkeys, *P);
    if (bk_ok()) return -3;
    if (P->tstride < P->nt) return -1;
    hipLaunchKernelGGL(k_bk_toff_t, dim3((P->nt + TT_T - 1) / TT_T), dim3(256), 0, st, (const uint16_t*)P->toff, P->nt,
                       P->tofft, P->tstride);
    if (!P->no_ts) {
        hipLaunchKernelGGL(k_bk_halo, dim3((P->nt + 255) / 256), dim3(256), 0, st, P->tfirst, P->hstart, P->nt,
                           P->within);
        hipLaunchKernelGGL(k_bk_tpre, dim3(1), dim3(1024), 0, st, P->tpre, P->nt);
    }
    return bk_ok();
}

// matches per arrival tile (the matcher's atomics) -> each tile's first row;
// ttot[nt] = the total
extern "C" int shb_finish(shb_plan* P, uint32_t* scan_tmp, void* stream) {
    return shd_exclusive_scan(P->ttot, P->ttot, (int64_t)P->nt + 1, scan_tmp, stream);
}

extern "C" int shb_s3_carry(const shb_plan* P, const shb_s3* S, void* stream) {
    if (P->kb > 12 || P->n_staged < 1 || P->st_width[0] != 4) return -1;
    hipLaunchKernelGGL(k_s3b, dim3(SHB_NB), dim3(S3B_TPB), 0, (hipStream_t)stream, *P, *S);
    return bk_ok();
}

extern "C" int shb_agg_carry(const shb_plan* P, const shb_aggc* A, void* stream) {
    static_assert(AGC_TPB == S3B_TPB && AGC_CH == S3B_CH, "the sort pass shape");
    if (P->kb > 8 || A->n < 1 || A->n > SHB_MAX_AGG) return -1;
    if (A->parallel)
        hipLaunchKernelGGL(k_bk_aggp, dim3(SHB_NB), dim3(AGC_TPB), 0, (hipStream_t)stream, *P, *A);
    else
        hipLaunchKernelGGL(k_bk_aggc, dim3(SHB_NB), dim3(AGC_TPB), 0, (hipStream_t)stream, *P, *A);
    return bk_ok();
}

// rows per lane and round of the 6-waves-per-SIMD form (LM: match-stream positions
// in LDS, <= 80 VGPRs): the most that compile without spilling VGPRs; 0 = that form
// does not fit (more values per row: the 4-waves form below)
template <int MODE, int NO>
constexpr int bk_ru_lm() {
    return NO == 0 ? 4
         : MODE == SHB_OUT_COLS ? (NO <= 2 ? 4 : 0)
                                : (NO <= 3 ? 4 : NO == 4 ? 3 : NO == 5 ? 2 : 0);
}

template <int MODE, int NO>
static void bk_emit_launch(const shb_plan* P, const shb_out* O, const shb_cols& OC, uint64_t seq_base,
                           uint64_t* out_seq, int64_t* out_vals, int64_t out_cap, void* stream) {
    // 6 waves per SIMD where the row loop fits 80 VGPRs (profiles/r6_emit6_ab.txt):
    // C2 (packed, 4 values) emit 1.47 -> 1.26 ms at 3 rows per lane, C3 (raw, 3
    // values) 0.85 -> 0.75. Six values or more stay at 4 waves: C2 + aggregates at 6
    // waves (1 row per lane) was 2.35 -> 2.31 ms but fetched 10.2 GB past L2 instead
    // of 7.6 (its running values by match-stream position thrash L2 harder)
    constexpr int RL = bk_ru_lm<MODE, NO>();
    if constexpr (RL > 0) {
        hipLaunchKernelGGL((k_bk_emit<MODE, NO, RL, 6>), dim3(bk_grid(P->nt)), dim3(BK_TPB), 0, (hipStream_t)stream,
                           *P, *O, OC, seq_base, out_seq, out_vals, out_cap);
        return;
    }
    // otherwise 4 waves per SIMD: 6 rows per lane and round up to 4 values (1.505 vs
    // 1.526 ms for 4 on C2, profiles/r4_c2_emit_ru_ab.txt), fewer beyond: as many as
    // fit 128 VGPRs without spilling
    constexpr int RU = (NO >= 1 && NO <= 4) ? (MODE == SHB_OUT_COLS && NO == 4 ? 4 : 6)
                                            : (MODE == SHB_OUT_RAW ? (NO <= 6 ? 4 : 3)
                                                                   : (MODE == SHB_OUT_PACKED ? (NO <= 6 ? 4 : (NO == 7 ? 2 : 1))
                                                                                             : (NO <= 5 ? 2 : 1)));
    hipLaunchKernelGGL((k_bk_emit<MODE, NO, RU>), dim3(bk_grid(P->nt)), dim3(BK_TPB), 0, (hipStream_t)stream, *P,
                       *O, OC, seq_base, out_seq, out_vals, out_cap);
}

template <int MODE>
static void bk_emit_width(const shb_plan* P, const shb_out* O, const shb_cols& OC, uint64_t seq_base,
                          uint64_t* out_seq, int64_t* out_vals, int64_t out_cap, void* stream) {
    switch (O->n_out) {
        case 1: bk_emit_launch<MODE, 1>(P, O, OC, seq_base, out_seq, out_vals, out_cap, stream); break;
        case 2: bk_emit_launch<MODE, 2>(P, O, OC, seq_base, out_seq, out_vals, out_cap, stream); break;
        case 3: bk_emit_launch<MODE, 3>(P, O, OC, seq_base, out_seq, out_vals, out_cap, stream); break;
        case 4: bk_emit_launch<MODE, 4>(P, O, OC, seq_base, out_seq, out_vals, out_cap, stream); break;
        case 5: bk_emit_launch<MODE, 5>(P, O, OC, seq_base, out_seq, out_vals, out_cap, stream); break;
        case 6: bk_emit_launch<MODE, 6>(P, O, OC, seq_base, out_seq, out_vals, out_cap, stream); break;
        case 7: bk_emit_launch<MODE, 7>(P, O, OC, seq_base, out_seq, out_vals, out_cap, stream); break;
        case 8: bk_emit_launch<MODE, 8>(P, O, OC, seq_base, out_seq, out_vals, out_cap, stream); break;
        default: bk_emit_launch<MODE, 0>(P, O, OC, seq_base, out_seq, out_vals, out_cap, stream); break;
    }
}

extern "C" int shb_emit(const shb_plan* P, const shb_out* O, const shb_cols* OC, uint64_t seq_base,
                        uint64_t* out_seq, int64_t* out_vals, int64_t out_cap, void* stream) {
    if (OC && OC->use == SHB_OUT_PACKED) {
        if (OC->rw % 4 || OC->rw > 2 + 2 * SHB_MAX_OUT + 2) return -1;
        bk_emit_width<SHB_OUT_PACKED>(P, O, *OC, seq_base, out_seq, out_vals, out_cap, stream);
    } else if (OC && OC->use == SHB_OUT_COLS) {
        bk_emit_width<SHB_OUT_COLS>(P, O, *OC, seq_base, out_seq, out_vals, out_cap, stream);
    } else {
        bk_emit_width<SHB_OUT_RAW>(P, O, shb_cols{}, seq_base, out_seq, out_vals, out_cap, stream);
    }
    return bk_ok();
}

// ---------------------------------------------------------------- typed columns
// raw 8-byte rows -> typed columns, for engines that write rows
__global__ void __launch_bounds__(256) k_narrow_rows(const int64_t* __restrict__ vals, int32_t n_out, int64_t m,
                                                     shb_cols OC) {
    const int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (r >= m) return;
    for (int o = 0; o < n_out; o++) bk_put(OC.cols[o], OC.colw[o], r, vals[r * n_out + o]);
}

extern "C" int shd_narrow_rows(const int64_t* vals, int32_t n_out, int64_t m, void* const* cols, const int32_t* w,
                               void* stream) {
    if (m <= 0) return 0;
    if (n_out > SHB_MAX_OUT) return -1;
    shb_cols OC;
    memset(&OC, 0, sizeof(OC));
    for (int o = 0; o < n_out; o++) {
        OC.cols[o] = cols[o];
        OC.colw[o] = w[o];
    }
    hipLaunchKernelGGL(k_narrow_rows, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, (hipStream_t)stream, vals, n_out,
                       m, OC);
    return bk_ok();
}

// raw rows (the engines that write 8-byte words) -> the caller's packed rows:
// one row per thread, built in registers and stored as whole 16-byte pieces
// (bk_pack); NO == 0: any number of values, word by word
template <int NO>
__global__ void __launch_bounds__(256) k_pack_rows(const uint64_t* __restrict__ seq, const int64_t* __restrict__ vals,
                                                   int32_t n_out, int64_t m, shb_cols OC) {
    const int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (r >= m) return;
    if (NO > 0) {
        int64_t v[NO > 0 ? NO : 1];
#pragma unroll
        for (int o = 0; o < NO; o++) v[o] = vals[r * NO + o];
        bk_pack<NO>(OC, r, v, seq[r]);
        return;
    }
    uint32_t* row = (uint32_t*)OC.rows + r * OC.rw;
    const uint64_t q = seq[r];
    row[0] = (uint32_t)q;
    row[1] = (uint32_t)(q >> 32);
    for (int k = 2; k < OC.rw; k++) row[k] = 0u;
    for (int o = 0; o < n_out; o++) {
        const int64_t v = vals[r * n_out + o];
        row[OC.woff[o]] = OC.colw[o] == 1 ? (uint32_t)(uint8_t)v : (uint32_t)v;
        if (OC.colw[o] == 8) row[OC.woff[o] + 1] = (uint32_t)((uint64_t)v >> 32);
    }
}

extern "C" int shd_pack_rows(const uint64_t* seq, const int64_t* vals, int32_t n_out, int64_t m, const int32_t* w,
                             const int32_t* woff, int32_t rw, void* rows, void* stream) {
    if (m <= 0) return 0;
    if (n_out > SHB_MAX_OUT) return -1;
    shb_cols OC;
    memset(&OC, 0, sizeof(OC));
    OC.use = SHB_OUT_PACKED;
    OC.rw = rw;
    OC.rows = rows;
    for (int o = 0; o < n_out; o++) {
        OC.colw[o] = w[o];
        OC.woff[o] = woff[o];
    }
    const dim3 g((unsigned)((m + 255) / 256));
    hipStream_t st = (hipStream_t)stream;
    switch (n_out) {
        case 1: hipLaunchKernelGGL(k_pack_rows<1>, g, dim3(256), 0, st, seq, vals, n_out, m, OC); break;
        case 2: hipLaunchKernelGGL(k_pack_rows<2>, g, dim3(256), 0, st, seq, vals, n_out, m, OC); break;
        case 3: hipLaunchKernelGGL(k_pack_rows<3>, g, dim3(256), 0, st, seq, vals, n_out, m, OC); break;
        case 4: hipLaunchKernelGGL(k_pack_rows<4>, g, dim3(256), 0, st, seq, vals, n_out, m, OC); break;
        case 5: hipLaunchKernelGGL(k_pack_rows<5>, g, dim3(256), 0, st, seq, vals, n_out, m, OC); break;
        case 6: hipLaunchKernelGGL(k_pack_rows<6>, g, dim3(256), 0, st, seq, vals, n_out, m, OC); break;
        case 7: hipLaunchKernelGGL(k_pack_rows<7>, g, dim3(256), 0, st, seq, vals, n_out, m, OC); break;
        case 8: hipLaunchKernelGGL(k_pack_rows<8>, g, dim3(256), 0, st, seq, vals, n_out, m, OC); break;
        default: hipLaunchKernelGGL(k_pack_rows<0>, g, dim3(256), 0, st, seq, vals, n_out, m, OC); break;
    }
    return bk_ok();
}
