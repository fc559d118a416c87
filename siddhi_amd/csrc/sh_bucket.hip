// sh_bucket.hip — bucketed window engine: the data movement around the hipRTC
// matcher (shb_match, sh_jit.cpp) for partitioned
//   every e1=S[f1] -> e2=S[f2(e1,e2)] within W        (C2)
//
// A partial opened at event i is consumed at the first later event j of its
// key with f2(i, j) while ts_j - ts_i <= W (StreamPreStateProcessor.java:325-403:
// break-early expiry then processAndReturn, every event a consumer candidate).
// The reference walks one global per-query pending list per event; here:
//
//  k_bk_hist    arrival tile T x key bucket b counts (b = key & 255)
//  (scan)       -> base[b][T]: where tile T's events of bucket b land
//  k_bk_scatter stable partition of the stream into 256 buckets, moving only
//               the packed (ts | local key) word and the columns the matcher
//               reads; tiles are ranked with wave ballots (sh_wave.h) and
//               staged through LDS so every bucket run is written contiguously
//  shb_match    (hipRTC) per bucket chunk + halo in LDS: per-consumer walk back
//               over its key -> partials consumed per event (u8, bucket order),
//               their e1-side select values (match stream), prefix sums at the
//               (bucket, tile) segment starts
//  k_bk_cum / k_bk_ttot  matches before each segment / per arrival tile
//  k_bk_emit    per arrival tile: re-rank the tile's events by bucket, gather
//               each consumer's count and match-stream position, scan in arrival
//               order and write the ordered rows (trigger seq + select values)
//
// HBM bytes per event: hist 4 + scatter 16 read / 8 written (C2) + matcher 8
// + emitter 16 + the match rows; no pass moves the event row more than once.
#include <hip/hip_runtime.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/sh_query.h"
#include "sh_device.h"
#include "sh_wave.h"

#define BK_TPB 512
#define BK_ITEMS (SHB_TILE / BK_TPB)
#define BK_ROWMAP 2048  // rows per 512-event block written row-parallel

static_assert(BK_ITEMS == 16, "tile / threads");

// raw 8-byte value of a column element (the VmVal bits sh_vm.h load_attr forms)
__device__ __forceinline__ int64_t bk_raw(const void* p, int64_t i, int type) {
    switch (type) {
        case SH_T_LONG:
        case SH_T_DOUBLE: return ((const int64_t*)p)[i];
        case SH_T_FLOAT: return (int64_t)((const uint32_t*)p)[i];
        case SH_T_BOOL: return ((const uint8_t*)p)[i] ? 1 : 0;
        default: return (int64_t)((const int32_t*)p)[i];
    }
}

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

// one typed output column element (sh_device_run.d_out_cols): natural width
__device__ __forceinline__ void bk_put(void* col, int w, int64_t row, int64_t v) {
    if (w == 8) ((int64_t*)col)[row] = v;
    else if (w == 4) ((uint32_t*)col)[row] = (uint32_t)v;
    else ((uint8_t*)col)[row] = (uint8_t)v;
}

// ---------------------------------------------------------------- histogram
__global__ void __launch_bounds__(BK_TPB) k_bk_hist(const int32_t* __restrict__ keys, int64_t n, int32_t nkeys,
                                                    int32_t nt, uint32_t* __restrict__ cnt,
                                                    int32_t* __restrict__ flag) {
    __shared__ uint32_t h[SHB_NB];
    const int T = bk_tile(nt);
    if (T < 0) return;
    if (threadIdx.x < SHB_NB) h[threadIdx.x] = 0u;
    __syncthreads();
    const int64_t b0 = (int64_t)T << SHB_TILE_SHIFT;
    bool bad = false;
#pragma unroll 4
    for (int j = 0; j < BK_ITEMS; j++) {
        const int64_t i = b0 + j * BK_TPB + threadIdx.x;
        if (i < n) {
            const int32_t k = keys[i];
            if (k >= nkeys) bad = true;
            else if (k >= 0) atomicAdd(&h[k & (SHB_NB - 1)], 1u);
        }
    }
    if (bad) atomicOr(flag, SHB_F_KEY);
    __syncthreads();
    if (threadIdx.x < SHB_NB) cnt[(int64_t)threadIdx.x * nt + T] = h[threadIdx.x];
    if (T == 0 && threadIdx.x == 0) cnt[(int64_t)SHB_NB * nt] = 0u;
}

// ---------------------------------------------------------------- partition
template <int MINW>
__global__ void __launch_bounds__(BK_TPB, MINW) k_bk_scatter(const int32_t* __restrict__ keys,
                                                          const int64_t* __restrict__ ts, shb_plan P) {
    __shared__ uint32_t wcnt[BK_TPB / 64][256];
    __shared__ uint32_t tstart[256], gbase[256];
    __shared__ uint32_t ws[BK_TPB / 64];
    __shared__ uint32_t stage[SHB_TILE];
    __shared__ uint8_t dig[SHB_TILE];
    const int T = bk_tile(P.nt);
    if (T < 0) return;
    const int64_t b0 = (int64_t)T << SHB_TILE_SHIFT;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int c = threadIdx.x; c < (BK_TPB / 64) * 256; c += BK_TPB) (&wcnt[0][0])[c] = 0u;
    if (threadIdx.x < 256) gbase[threadIdx.x] = P.base[(int64_t)threadIdx.x * P.nt + T];
    __syncthreads();
    // the keys and timestamps of the tile are loaded up front (one HBM round
    // trip); the packed word (ts - tbase) << kb | key >> 8 is formed in registers
    int32_t key[BK_ITEMS];
    // (staged columns are loaded after the packed words are written: prefetching
    // them as well spills registers at two workgroups per CU)
    uint32_t rw[BK_ITEMS], wp[BK_ITEMS];
    const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
    {
        int64_t tv[BK_ITEMS];
        const int64_t e0 = b0 + (int64_t)w * (64 * BK_ITEMS) + lane;
        if (b0 + SHB_TILE <= P.n) {
            // a full tile: unpredicated loads at immediate offsets from two bases
            const int32_t* __restrict__ pk = keys + e0;
            const int64_t* __restrict__ pt = ts + e0;
#pragma unroll
            for (int j = 0; j < BK_ITEMS; j++) {
                key[j] = pk[j * 64];
                tv[j] = pt[j * 64];
            }
        } else {
#pragma unroll
            for (int j = 0; j < BK_ITEMS; j++) {
                const int64_t i = e0 + j * 64;
                const bool in = i < P.n;
                key[j] = in ? keys[i] : -1;
                tv[j] = in ? ts[i] : P.tbase;
            }
        }
        const int64_t lim = (int64_t)1 << (32 - P.kb);
        bool bad = false;
#pragma unroll
        for (int j = 0; j < BK_ITEMS; j++) {
            const int64_t dt = tv[j] - P.tbase;
            if (key[j] >= 0 && (dt < 0 || dt >= lim)) bad = true;
            wp[j] = ((uint32_t)dt << P.kb) | ((uint32_t)key[j] >> 8);
            // the key is not needed past this point: bucket << 16 (~0u: no key)
            rw[j] = key[j] >= 0 ? ((uint32_t)key[j] & (SHB_NB - 1)) << 16 : ~0u;
        }
        if (bad) atomicOr(P.flag, SHB_F_TS);
    }
    // each wave ranks its own contiguous 1,024 events (16 rounds of 64): the
    // rank of an event among the wave's same-bucket events before it, from 8
    // ballots per round and the wave's running counts (no block barrier)
    // the leader lane of each bucket group adds the group to the wave's running
    // count with a returning LDS atomic (the rounds' atomics issue back to back);
    // the group reads its base from the leader afterwards
    {
        uint32_t old[BK_ITEMS];
#pragma unroll
        for (int j = 0; j < BK_ITEMS; j++) {
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
        for (int j = 0; j < BK_ITEMS; j++) {
            const uint32_t ld = rw[j] == ~0u ? (uint32_t)lane : (rw[j] >> 8) & 63u;
            const uint32_t base = (uint32_t)__shfl((int)old[j], (int)ld);
            if (rw[j] != ~0u) rw[j] = ((base + (rw[j] & 0xFFu)) & 0xFFFFu) | (rw[j] & 0xFF0000u);  // wave rank | bucket << 16
        }
    }
    __syncthreads();
    // per bucket: the waves' exclusive offsets and the tile total, then the
    // buckets' starts
    uint32_t nvalid;
    {
        uint32_t tot = 0;
        if (threadIdx.x < 256) {
#pragma unroll
            for (int q = 0; q < BK_TPB / 64; q++) {
                const uint32_t c = wcnt[q][threadIdx.x];
                wcnt[q][threadIdx.x] = tot;
                tot += c;
            }
        }
        const uint32_t ex = shw_block_excl<BK_TPB>(threadIdx.x < 256 ? tot : 0u, ws, &nvalid);
        if (threadIdx.x < 256) tstart[threadIdx.x] = ex;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < BK_ITEMS; j++) {
        const bool valid = rw[j] != ~0u;
        const uint32_t d = (rw[j] >> 16) & (SHB_NB - 1);
        const uint32_t r = valid ? wcnt[w][d] + (rw[j] & 0xFFFFu) : 0u;  // rank among the tile's bucket-d events
        rw[j] = valid ? tstart[d] + r : ~0u;                  // the event's slot in the staged tile
        if (valid) dig[rw[j]] = (uint8_t)d;
        // the emitter restores arrival order from this rank (no re-ranking there)
        const int64_t i = b0 + (int64_t)w * (64 * BK_ITEMS) + j * 64 + lane;
        if (i < P.n) P.rk[i] = (uint16_t)r;
    }
#pragma unroll
    for (int j = 0; j < BK_ITEMS; j++)
        if (rw[j] != ~0u) stage[rw[j]] = wp[j];
    __syncthreads();
#define BK_WRITE_OUT(T, DST, EXPR)                                                   \
    {                                                                                \
        _Pragma("unroll 4") for (int m = 0; m < BK_ITEMS; m++) {                     \
            const uint32_t l = (uint32_t)(m * BK_TPB + threadIdx.x);                 \
            if (l < nvalid) {                                                        \
                const uint32_t d = dig[l];                                           \
                ((T*)(DST))[EXPR(gbase[d] + l - tstart[d])] = (T)stage[l];           \
            }                                                                        \
        }                                                                            \
        __syncthreads();                                                             \
    }
#define BK_ID(x) (x)
#define BK_LO(x) (2u * (x))
#define BK_HI(x) (2u * (x) + 1u)
    BK_WRITE_OUT(uint32_t, P.w0, BK_ID);
    for (int c = 0; c < P.n_staged; c++) {
        const int wd = P.st_width[c];
        const int halves = wd == 8 ? 2 : 1;
        for (int hh = 0; hh < halves; hh++) {
#pragma unroll
            for (int j = 0; j < BK_ITEMS; j++) {
                if (rw[j] == ~0u) continue;
                const int64_t i = b0 + (int64_t)w * (64 * BK_ITEMS) + j * 64 + lane;
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

// ---------------------------------------------------------------- segment sums
// cum[b][T] = matches of bucket b before the start of its tile-T segment: the
// scanned chunk totals (ctot, exclusive over chunk ids) + the matcher's
// within-chunk prefix at the segment start (psum)
__device__ __forceinline__ int64_t bk_gch(uint32_t bs, int b, uint32_t ch) {
    return (int64_t)(bs / SHB_CH) + ch + b;
}

__global__ void __launch_bounds__(256) k_bk_cum(shb_plan P) {
    const int b = blockIdx.x;
    const uint32_t bs = P.base[(int64_t)b * P.nt];
    const uint32_t nb = P.base[(int64_t)(b + 1) * P.nt] - bs;
    const uint32_t nch = (nb + SHB_CH - 1) / SHB_CH;
    const uint32_t c0 = P.ctot[bk_gch(bs, b, 0)];
    const uint32_t tot = P.ctot[bk_gch(bs, b, nch)] - c0;
    uint32_t* row = P.cum + (int64_t)b * (P.nt + 1);
    for (int T = threadIdx.x; T < P.nt; T += 256) {
        const uint32_t x = P.base[(int64_t)b * P.nt + T] - bs;
        row[T] = x >= nb ? tot : P.ctot[bk_gch(bs, b, x / SHB_CH)] - c0 + P.psum[(int64_t)b * P.nt + T];
    }
    if (threadIdx.x == 0) row[P.nt] = tot;
}

// matches per arrival tile: sum over buckets of the tile's segment
__global__ void __launch_bounds__(256) k_bk_ttot(shb_plan P) {
    const int64_t T = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (T > P.nt) return;
    if (T == P.nt) {
        P.ttot[T] = 0u;
        return;
    }
    uint32_t s = 0;
    for (int b = 0; b < SHB_NB; b++) {
        const uint32_t* row = P.cum + (int64_t)b * (P.nt + 1);
        s += row[T + 1] - row[T];
    }
    P.ttot[T] = s;
}

// ---------------------------------------------------------------- emitter
// per event (registers): bucket d | count << 8 | rank << 16, and its
// match-stream position; the select list lives in LDS (uniform per output)
// COLS: typed output columns (OC.cols), else raw 8-byte rows; NO: the select width
// (1..8: unrolled, the descriptors in scalar registers; 0: any width, a loop)
template <bool COLS, int NO>
__global__ void __launch_bounds__(BK_TPB) k_bk_emit(const int32_t* __restrict__ keys, shb_plan P, shb_out O,
                                                    shb_cols OC, uint64_t seq_base, uint64_t* __restrict__ out_seq,
                                                    int64_t* __restrict__ out_vals, int64_t out_cap) {
    __shared__ uint32_t run[256], lstart[256], segx[256], bstart[256], psum[256];
    __shared__ uint32_t ws[BK_TPB / 64];
    __shared__ uint32_t S[SHB_TILE];
    __shared__ int32_t o_kind[SHB_MAX_OUT], o_type[SHB_MAX_OUT];
    __shared__ const void* o_src[SHB_MAX_OUT];
    __shared__ uint16_t evmap[2 * BK_ROWMAP];
    __shared__ uint32_t blk_mpos[2 * BK_TPB];
    __shared__ uint32_t s_tot;
    const int T = bk_tile(P.nt);
    if (T < 0) return;
    const int64_t b0 = (int64_t)T << SHB_TILE_SHIFT;
    const int tile_n = (int)((P.n - b0) < SHB_TILE ? (P.n - b0) : SHB_TILE);
    if (threadIdx.x < 256) {
        const int b = threadIdx.x;
        run[b] = 0u;
        const uint32_t bs = P.base[(int64_t)b * P.nt];
        bstart[b] = bs;
        segx[b] = P.base[(int64_t)b * P.nt + T] - bs;
        psum[b] = P.psum[(int64_t)b * P.nt + T];
    }
    if (threadIdx.x < SHB_MAX_OUT) {
#pragma unroll
        for (int o = 0; o < SHB_MAX_OUT; o++)
            if (o == (int)threadIdx.x) {
                o_kind[o] = O.kind[o];
                o_type[o] = O.type[o];
                o_src[o] = O.src[o];
            }
    }
    // per event (registers): bucket d | count << 8 | rank << 16 (~0u: no key)
    uint32_t pk[BK_ITEMS];
#pragma unroll
    for (int j = 0; j < BK_ITEMS; j++) {
        const int l = j * BK_TPB + threadIdx.x;
        const int32_t k = (l < tile_n) ? keys[b0 + l] : -1;
        const uint32_t r = (l < tile_n) ? (uint32_t)P.rk[b0 + l] : 0u;
        pk[j] = k >= 0 ? (((uint32_t)k & (SHB_NB - 1)) | (r << 16)) : ~0u;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < BK_ITEMS; j++)
        if (pk[j] != ~0u) atomicAdd(&run[pk[j] & 0xFFu], 1u);
    // counts of the events' consumers, gathered all at once
#pragma unroll
    for (int j = 0; j < BK_ITEMS; j++) {
        if (pk[j] == ~0u) continue;
        const uint32_t d = pk[j] & 0xFFu, r = pk[j] >> 16;
        pk[j] |= (uint32_t)P.cnt[bstart[d] + segx[d] + r] << 8;
    }
    __syncthreads();
    uint32_t nvalid;
    {
        const uint32_t c = threadIdx.x < 256 ? run[threadIdx.x] : 0u;
        const uint32_t ex = shw_block_excl<BK_TPB>(c, ws, &nvalid);
        if (threadIdx.x < 256) lstart[threadIdx.x] = ex;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < BK_ITEMS; j++) {
        if (pk[j] == ~0u) continue;
        const uint32_t d = pk[j] & 0xFFu, r = pk[j] >> 16;
        S[lstart[d] + r] = (pk[j] >> 8) & 0xFFu;
    }
    __syncthreads();
    shw_lds_excl_scan<BK_TPB, BK_ITEMS>(S, (int)nvalid, ws);
    // match-stream position: region of the event's matcher chunk + the prefix
    // inside that chunk (segment start: the matcher's psum; chunk start: 0)
    uint32_t mpos[BK_ITEMS];
#pragma unroll
    for (int j = 0; j < BK_ITEMS; j++) {
        mpos[j] = 0u;
        if (pk[j] == ~0u) continue;
        const uint32_t d = pk[j] & 0xFFu, r = pk[j] >> 16;
        const uint32_t x = segx[d] + r;
        const uint32_t ch = x / SHB_CH;
        const uint32_t hx = (ch * SHB_CH > segx[d]) ? ch * SHB_CH : segx[d];
        const uint32_t wp = S[lstart[d] + r] - S[lstart[d] + (hx - segx[d])] + (hx == segx[d] ? psum[d] : 0u);
        mpos[j] = (uint32_t)(bk_gch(bstart[d], (int)d, ch) * SHB_SPAN) + wp;
    }
    __syncthreads();
    // output offsets: scan of the counts in arrival order
#pragma unroll
    for (int j = 0; j < BK_ITEMS; j++) {
        const int l = j * BK_TPB + threadIdx.x;
        if (l < tile_n) S[l] = pk[j] == ~0u ? 0u : (pk[j] >> 8) & 0xFFu;
    }
    __syncthreads();
    shw_lds_excl_scan<BK_TPB, BK_ITEMS>(S, tile_n, ws);
    const uint32_t tb = P.ttot[T];
    const int no = O.n_out;
    // the rows are written row-parallel, one 1,024-event block at a time: each
    // event enters its rows into the block's row -> event map, then thread t
    // writes row r0 + t (consecutive lanes, consecutive rows: coalesced)
    {
        const int l = tile_n - 1;
        if (l >= 0 && (l & (BK_TPB - 1)) == (int)threadIdx.x) {
            const uint32_t pl = pk[l / BK_TPB];
            s_tot = S[l] + (pl == ~0u ? 0u : (pl >> 8) & 0xFFu);
        }
    }
    __syncthreads();
    // two 512-event blocks at a time: their events enter their rows into the row
    // -> event map, then thread t writes rows r0 + t, r0 + t + 512, ...
    // (consecutive lanes, consecutive rows: coalesced)
#pragma unroll
    for (int j = 0; j < BK_ITEMS; j += 2) {
        const int lb = j * BK_TPB;
        if (lb >= tile_n) break;  // uniform
        const uint32_t r0 = S[lb];
        const uint32_t r1 = lb + 2 * BK_TPB < tile_n ? S[lb + 2 * BK_TPB] : s_tot;
        const uint32_t R = r1 - r0;
        if (R <= 2 * BK_ROWMAP) {
#pragma unroll
            for (int h = 0; h < 2; h++) {
                const int l = lb + h * BK_TPB + threadIdx.x;
                const uint32_t c = (l < tile_n && pk[j + h] != ~0u) ? (pk[j + h] >> 8) & 0xFFu : 0u;
                if (c) {
                    const uint32_t at = S[l] - r0;
                    for (uint32_t k = 0; k < c; k++) evmap[at + k] = (uint16_t)(h * BK_TPB + threadIdx.x);
                }
                blk_mpos[h * BK_TPB + threadIdx.x] = mpos[j + h];
            }
            __syncthreads();
            for (uint32_t t = threadIdx.x; t < R; t += BK_TPB) {
                const int e = evmap[t];
                const int le = lb + e;
                const uint32_t k = r0 + t - S[le];
                const int64_t i = b0 + le;
                const int64_t row = (int64_t)tb + r0 + t;
                if (row >= out_cap) continue;  // the host reports SH_E_MORE
                if (out_seq) out_seq[row] = seq_base + (uint64_t)i;
                if (!out_vals && !COLS) continue;
                // output descriptors straight from the kernel arguments (scalar
                // registers: uniform branches)
                if (NO > 0) {
                    const int64_t mp = (int64_t)blk_mpos[e] + k;
                    int64_t v[NO > 0 ? NO : 1];
#pragma unroll
                    for (int o = 0; o < NO; o++) v[o] = bk_raw(O.src[o], O.kind[o] == 1 ? i : mp, O.type[o]);
                    if (COLS) {
                        // typed columns: consecutive lanes, consecutive elements of each column
#pragma unroll
                        for (int o = 0; o < NO; o++) bk_put(OC.cols[o], OC.colw[o], row, v[o]);
                        continue;
                    }
                    if (NO % 2 == 0) {
                        // a row of NO words as 16-byte stores: consecutive lanes fill whole lines
                        longlong2* dst = (longlong2*)(out_vals + row * NO);
#pragma unroll
                        for (int o = 0; o < NO; o += 2) dst[o / 2] = make_longlong2(v[o], v[o + 1]);
                    } else {
#pragma unroll
                        for (int o = 0; o < NO; o++) out_vals[row * NO + o] = v[o];
                    }
                    continue;
                }
                for (int o = 0; o < no; o++) {
                    const int64_t v = bk_raw(O.src[o], O.kind[o] == 1 ? i : (int64_t)blk_mpos[e] + k, O.type[o]);
                    if (COLS) bk_put(OC.cols[o], OC.colw[o], row, v);
                    else out_vals[row * no + o] = v;
                }
            }
            __syncthreads();
            continue;
        }
        // a dense pair of blocks (more rows than the map holds): event-parallel writes
#pragma unroll
        for (int h = 0; h < 2; h++) {
            const int l = lb + h * BK_TPB + threadIdx.x;
            const uint32_t c = (l < tile_n && pk[j + h] != ~0u) ? (pk[j + h] >> 8) & 0xFFu : 0u;
            if (!c) continue;
            const int64_t i = b0 + l;
            const int64_t row0 = (int64_t)tb + S[l];
            if (row0 + c > out_cap) continue;
            if (out_seq)
                for (uint32_t k = 0; k < c; k++) out_seq[row0 + k] = seq_base + (uint64_t)i;
            if (!out_vals && !COLS) continue;
            for (int o = 0; o < no; o++) {
                const void* src = o_src[o];
                const int ty = o_type[o];
                for (uint32_t k = 0; k < c; k++) {
                    const int64_t v = bk_raw(src, o_kind[o] == 1 ? i : (int64_t)mpos[j + h] + k, ty);
                    if (COLS) bk_put(OC.cols[o], OC.colw[o], row0 + k, v);
                    else out_vals[(row0 + k) * no + o] = v;
                }
            }
        }
    }
}

// ---------------------------------------------------------------- launches
static int bk_ok() { return hipGetLastError() == hipSuccess ? 0 : -3; }

extern "C" int shb_partition(const int32_t* keys, const int64_t* ts, int32_t nkeys, shb_plan* P, uint32_t* scan_tmp,
                             void* stream) {
    hipStream_t st = (hipStream_t)stream;
    const int64_t cells = (int64_t)SHB_NB * P->nt + 1;
    hipLaunchKernelGGL(k_bk_hist, dim3(bk_grid(P->nt)), dim3(BK_TPB), 0, st, keys, P->n, nkeys, P->nt, P->base, P->flag);
    if (bk_ok()) return -3;
    if (shd_exclusive_scan(P->base, P->base, cells, scan_tmp, stream)) return -3;
    // SH_BK_SCAT=1: no occupancy bound on the scatter (more registers, one
    // workgroup per CU); default: 4 waves per SIMD (two workgroups per CU)
    static const int scat = getenv("SH_BK_SCAT") ? atoi(getenv("SH_BK_SCAT")) : 4;
    if (scat == 1)
        hipLaunchKernelGGL(k_bk_scatter<1>, dim3(bk_grid(P->nt)), dim3(BK_TPB), 0, st, keys, ts, *P);
    else
        hipLaunchKernelGGL(k_bk_scatter<4>, dim3(bk_grid(P->nt)), dim3(BK_TPB), 0, st, keys, ts, *P);
    return bk_ok();
}

extern "C" int shb_finish(shb_plan* P, uint32_t* scan_tmp, void* stream) {
    hipStream_t st = (hipStream_t)stream;
    if (shd_exclusive_scan(P->ctot, P->ctot, P->n_gch + 1, scan_tmp, stream)) return -3;
    hipLaunchKernelGGL(k_bk_cum, dim3(SHB_NB), dim3(256), 0, st, *P);
    if (bk_ok()) return -3;
    hipLaunchKernelGGL(k_bk_ttot, dim3((P->nt + 1 + 255) / 256), dim3(256), 0, st, *P);
    if (bk_ok()) return -3;
    return shd_exclusive_scan(P->ttot, P->ttot, (int64_t)P->nt + 1, scan_tmp, stream);
}

template <bool COLS, int NO>
static void bk_emit_launch(const int32_t* keys, const shb_plan* P, const shb_out* O, const shb_cols& OC,
                           uint64_t seq_base, uint64_t* out_seq, int64_t* out_vals, int64_t out_cap, void* stream) {
    hipLaunchKernelGGL((k_bk_emit<COLS, NO>), dim3(bk_grid(P->nt)), dim3(BK_TPB), 0, (hipStream_t)stream, keys, *P, *O,
                       OC, seq_base, out_seq, out_vals, out_cap);
}

template <bool COLS>
static void bk_emit_width(const int32_t* keys, const shb_plan* P, const shb_out* O, const shb_cols& OC,
                          uint64_t seq_base, uint64_t* out_seq, int64_t* out_vals, int64_t out_cap, void* stream) {
    switch (O->n_out) {
        case 1: bk_emit_launch<COLS, 1>(keys, P, O, OC, seq_base, out_seq, out_vals, out_cap, stream); break;
        case 2: bk_emit_launch<COLS, 2>(keys, P, O, OC, seq_base, out_seq, out_vals, out_cap, stream); break;
        case 3: bk_emit_launch<COLS, 3>(keys, P, O, OC, seq_base, out_seq, out_vals, out_cap, stream); break;
        case 4: bk_emit_launch<COLS, 4>(keys, P, O, OC, seq_base, out_seq, out_vals, out_cap, stream); break;
        case 5: bk_emit_launch<COLS, 5>(keys, P, O, OC, seq_base, out_seq, out_vals, out_cap, stream); break;
        case 6: bk_emit_launch<COLS, 6>(keys, P, O, OC, seq_base, out_seq, out_vals, out_cap, stream); break;
        case 7: bk_emit_launch<COLS, 7>(keys, P, O, OC, seq_base, out_seq, out_vals, out_cap, stream); break;
        case 8: bk_emit_launch<COLS, 8>(keys, P, O, OC, seq_base, out_seq, out_vals, out_cap, stream); break;
        default: bk_emit_launch<COLS, 0>(keys, P, O, OC, seq_base, out_seq, out_vals, out_cap, stream); break;
    }
}

extern "C" int shb_emit(const int32_t* keys, const shb_plan* P, const shb_out* O, const shb_cols* OC,
                        uint64_t seq_base, uint64_t* out_seq, int64_t* out_vals, int64_t out_cap, void* stream) {
    if (OC && OC->use)
        bk_emit_width<true>(keys, P, O, *OC, seq_base, out_seq, out_vals, out_cap, stream);
    else
        bk_emit_width<false>(keys, P, O, shb_cols{}, seq_base, out_seq, out_vals, out_cap, stream);
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
