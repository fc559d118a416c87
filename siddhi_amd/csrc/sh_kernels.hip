// sh_kernels.hip — gfx950 kernels of the batch NFA matcher.
//
//  (1) predicate evaluation      : typed postfix VM (vm_eval) run per
//                                  (partial, event) inside the advance kernel
//  (2) radix segment             : k_digit_hist / k_digit_scatter (stable LSD
//                                  radix sort of (key, arrival index), 8-bit
//                                  digits, wave64 ballot ranking) + k_seg_mark
//  (3) per-key state advance     : k_advance, one lane per partition key walks
//                                  its segment in arrival order with the
//                                  pending / new-and-every lists in HBM
//  (4) spawn / compaction        : partial spawn + list compaction in
//                                  k_advance, ordered match placement via an
//                                  exclusive scan of per-event match counts
//  (5) within expiry             : break-early head expiry per event (k_advance)
//
// Semantics follow core/query/input/stream/state/StreamPreStateProcessor.java
// (expireEvents :325-361, updateState :307-323, processAndReturn :363-403),
// StreamPostStateProcessor.java:64-83, the Pattern*ProcessStreamReceiver
// stabilizeStates/eventSequence rules and the executor conversion/null rules.
#include <hip/hip_runtime.h>

#include "../../include/sh_query.h"
#include "sh_device.h"
#include "sh_wave.h"

#include <stdlib.h>
#include <string.h>
#include <type_traits>

#define TPB 256
#define RADIX_ITEMS 16
#define RADIX_TILE (TPB * RADIX_ITEMS)
#define SCAN_ITEMS 4
#define SCAN_TILE (TPB * SCAN_ITEMS)

// ------------------------------------------------------------------ scan
// wave scans: the DPP row-shift / row-broadcast form of sh_wave.h
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) { return shw_incl_scan(v); }

// block-wide exclusive scan of one value per thread; returns block total in *total
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* total) {
    __shared__ uint32_t wsum[TPB / 64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint32_t inc = wave_incl_scan(v);
    if (lane == 63) wsum[w] = inc;
    __syncthreads();
    uint32_t off = 0, tot = 0;
#pragma unroll
    for (int i = 0; i < TPB / 64; i++) {
        uint32_t s = wsum[i];
        if (i < w) off += s;
        tot += s;
    }
    __syncthreads();
    *total = tot;
    return off + inc - v;
}

__global__ void __launch_bounds__(TPB) k_scan_tiles(const uint32_t* __restrict__ in, uint32_t* __restrict__ out,
                                                    int64_t n, uint32_t* __restrict__ tile_sums) {
    const int64_t base = (int64_t)blockIdx.x * SCAN_TILE + (int64_t)threadIdx.x * SCAN_ITEMS;
    uint32_t v[SCAN_ITEMS];
    uint32_t s = 0;
#pragma unroll
    for (int j = 0; j < SCAN_ITEMS; j++) {
        v[j] = (base + j < n) ? in[base + j] : 0u;
        s += v[j];
    }
    uint32_t tot;
    uint32_t off = block_excl_scan(s, &tot);
#pragma unroll
    for (int j = 0; j < SCAN_ITEMS; j++) {
        if (base + j < n) out[base + j] = off;
        off += v[j];
    }
    if (threadIdx.x == 0 && tile_sums) tile_sums[blockIdx.x] = tot;
}

__global__ void __launch_bounds__(TPB) k_scan_add(uint32_t* __restrict__ out, int64_t n,
                                                  const uint32_t* __restrict__ tile_off) {
    const int64_t base = (int64_t)blockIdx.x * SCAN_TILE + (int64_t)threadIdx.x * SCAN_ITEMS;
    const uint32_t add = tile_off[blockIdx.x];
#pragma unroll
    for (int j = 0; j < SCAN_ITEMS; j++)
        if (base + j < n) out[base + j] += add;
}

static int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

extern "C" size_t shd_scan_tmp_words(int64_t n) {
    size_t words = 0;
    int64_t m = ceil_div(n, SCAN_TILE);
    while (m > 1) {
        words += 2 * (size_t)m + 2;
        m = ceil_div(m, SCAN_TILE);
    }
    return words + 4;
}

// exclusive scan of n uint32 (in may equal out); tmp >= shd_scan_tmp_words(n)
extern "C" int shd_exclusive_scan(const uint32_t* in, uint32_t* out, int64_t n, uint32_t* tmp, void* stream) {
    hipStream_t st = (hipStream_t)stream;
    if (n <= 0) return 0;
    int64_t tiles = ceil_div(n, SCAN_TILE);
    if (tiles == 1) {
        hipLaunchKernelGGL(k_scan_tiles, dim3(1), dim3(TPB), 0, st, in, out, n, (uint32_t*)nullptr);
        return hipGetLastError() == hipSuccess ? 0 : -3;
    }
    uint32_t* sums = tmp;
    uint32_t* sums_scanned = tmp + tiles + 1;
    hipLaunchKernelGGL(k_scan_tiles, dim3((unsigned)tiles), dim3(TPB), 0, st, in, out, n, sums);
    int rc = shd_exclusive_scan(sums, sums_scanned, tiles, tmp + 2 * tiles + 2, stream);
    if (rc) return rc;
    hipLaunchKernelGGL(k_scan_add, dim3((unsigned)tiles), dim3(TPB), 0, st, out, n, (const uint32_t*)sums_scanned);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

// ------------------------------------------------------------------ radix segment
// Histogram layout. Global (sub_shift < 0): digit-major, hist[d * ntiles + blk],
// so the exclusive scan orders all blocks by digit. Arrival-tile-major
// (sub_shift >= 0, 2^sub_shift blocks per arrival tile): hist[(tile, d, blk in
// tile)], so the scan keeps every arrival tile in its own region and sorts each
// tile by key: the stable LSD passes then produce (tile, key, arrival) order.
template <int B>
__device__ __forceinline__ int64_t hist_idx(uint32_t d, uint32_t blk, int64_t ntiles, int sub_shift) {
    if (sub_shift < 0) return (int64_t)d * ntiles + blk;
    return ((((int64_t)(blk >> sub_shift)) * (1 << B) + d) << sub_shift) + (blk & ((1u << sub_shift) - 1u));
}

// digit histogram per block (layout: hist_idx); B-bit digits (8, or 10 for two
// passes over 17..20-bit key ranges)
template <int B>
__global__ void __launch_bounds__(TPB) k_digit_hist(const uint32_t* __restrict__ keys, const int32_t* __restrict__ raw,
                                                    uint32_t sentinel, int64_t n, int shift,
                                                    uint32_t* __restrict__ hist, int64_t ntiles, int sub_shift) {
    constexpr int ND = 1 << B;
    __shared__ uint32_t h[ND];
    for (int d = threadIdx.x; d < ND; d += TPB) h[d] = 0;
    __syncthreads();
    const int64_t base = (int64_t)blockIdx.x * RADIX_TILE;
#pragma unroll 4
    for (int j = 0; j < RADIX_ITEMS; j++) {
        int64_t i = base + j * TPB + threadIdx.x;
        if (i < n) {
            uint32_t k;
            if (keys) {
                k = keys[i];
            } else {
                int32_t r = raw ? raw[i] : 0;
                k = r < 0 ? sentinel : (uint32_t)r;
            }
            atomicAdd(&h[(k >> shift) & (ND - 1)], 1u);
        }
    }
    __syncthreads();
    for (int d = threadIdx.x; d < ND; d += TPB) hist[hist_idx<B>(d, blockIdx.x, ntiles, sub_shift)] = h[d];
}

// stable scatter: elements of a tile are ranked in arrival order within their
// digit, staged in LDS in digit order, and written out as contiguous runs per
// digit (coalesced), for the key, the arrival index and every carried column
__device__ __forceinline__ uint32_t load_key(const uint32_t* __restrict__ keys_in, const int32_t* __restrict__ raw,
                                             uint32_t sentinel, int64_t i) {
    if (keys_in) return keys_in[i];
    const int32_t r = raw ? raw[i] : 0;
    return r < 0 ? sentinel : (uint32_t)r;
}

template <int B>
__global__ void __launch_bounds__(TPB, (B <= 8 ? 4 : 3)) k_digit_scatter(const uint32_t* __restrict__ keys_in, const int32_t* __restrict__ raw,
                                                       uint32_t sentinel, const uint32_t* __restrict__ idx_in, int64_t n,
                                                       int shift, const uint32_t* __restrict__ offs, int64_t ntiles,
                                                       uint32_t* __restrict__ keys_out, uint32_t* __restrict__ idx_out,
                                                       shd_payload PL, int sub_shift, int xcd, int counts = 0) {
    // xcd: consecutive tiles go to one XCD (blocks are dealt round-robin over the 8
    // XCDs), so the short per-digit runs neighbouring tiles write into the same digit
    // region meet in one L2 and leave it as whole lines
    int64_t tile = blockIdx.x;
    if (xcd) {
        const int64_t per = (ntiles + 7) >> 3;
        tile = (int64_t)(blockIdx.x & 7u) * per + (blockIdx.x >> 3);
        if (tile >= ntiles) return;
    }
    // every wave owns a contiguous quarter of the tile (items j*64 + lane), so ranking in
    // (j, lane) order inside a wave and then across waves is arrival order: a running
    // count per (wave, digit) bumped by each peer group's leader (returning LDS atomic)
    // replaces a block barrier per item
    constexpr int ND = 1 << B, DPT = ND / TPB;  // digits per thread in the prefix
    constexpr int WAVE_ITEMS = RADIX_TILE / (TPB / 64);
    using dig_t = typename std::conditional<(B <= 8), uint8_t, uint16_t>::type;
    __shared__ uint32_t wcnt[TPB / 64][ND];
    __shared__ uint32_t tstart[ND];
    __shared__ uint32_t gbase[ND];
    __shared__ dig_t dig[RADIX_TILE];
    // 16 KB: 4-byte staging of a whole tile; 8-byte columns go through it as two
    // halves of the tile (values held in registers), so the scatter fits ~26 KB of
    // LDS and five to six workgroups per CU instead of three
    __shared__ __align__(16) uint32_t stage[RADIX_TILE];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint64_t lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    const int64_t base = tile * RADIX_TILE;
    const int64_t wbase = base + (int64_t)w * WAVE_ITEMS + lane;  // element j: wbase + j * 64
    const int64_t tile_n = (n - base) < RADIX_TILE ? (n - base) : RADIX_TILE;
    for (int d = threadIdx.x; d < ND; d += TPB) {
#pragma unroll
        for (int q = 0; q < TPB / 64; q++) wcnt[q][d] = 0;
        if (!counts) gbase[d] = offs[hist_idx<B>(d, (uint32_t)tile, ntiles, sub_shift)];
    }
    if (B == 8 && counts) {
        // offs holds the tiles' digit counts (digit-major, at most SMALL_TILES tiles):
        // the digit's start (scan over the digits' totals) plus the earlier tiles'
        // (8-bit digits: one per thread)
        const uint32_t* c = offs + (int64_t)threadIdx.x * ntiles;
        uint32_t tot = 0, before = 0;
        for (int t = 0; t < (int)ntiles; t++) {
            const uint32_t v = c[t];
            before += t < (int)tile ? v : 0u;
            tot += v;
        }
        uint32_t all;
        gbase[threadIdx.x] = block_excl_scan(tot, &all) + before;
    }
    uint32_t key[RADIX_ITEMS];
#pragma unroll
    for (int j = 0; j < RADIX_ITEMS; j++) {
        const int64_t i = wbase + j * 64;
        key[j] = (i < n) ? load_key(keys_in, raw, sentinel, i) : 0u;
    }
    __syncthreads();
    // wave-local stable rank inside the digit
    uint32_t lp[RADIX_ITEMS];
#pragma unroll
    for (int j = 0; j < RADIX_ITEMS; j++) {
        const bool valid = wbase + j * 64 < n;
        const uint32_t d = (key[j] >> shift) & (ND - 1);
        uint64_t peers = __ballot(valid);
#pragma unroll
        for (int b = 0; b < B; b++) {
            const bool bit = (d >> b) & 1u;
            const uint64_t m = __ballot(valid && bit);
            peers &= bit ? m : ~m;
        }
        uint32_t old = 0;
        const uint32_t rank = __popcll(peers & lt_mask);
        if (valid && rank == 0) old = atomicAdd(&wcnt[w][d], (uint32_t)__popcll(peers));
        const int leader = valid ? __ffsll((unsigned long long)peers) - 1 : lane;
        old = __shfl(old, leader);
        lp[j] = old + rank;
    }
    __syncthreads();
    {
        // per digit: exclusive prefix over the waves, then the tile-local digit starts
        // (thread t owns digits t*DPT .. t*DPT+DPT-1)
        uint32_t loc[DPT], sum = 0;
#pragma unroll
        for (int i = 0; i < DPT; i++) {
            const int d = threadIdx.x * DPT + i;
            uint32_t tot = 0;
#pragma unroll
            for (int q = 0; q < TPB / 64; q++) {
                const uint32_t c = wcnt[q][d];
                wcnt[q][d] = tot;
                tot += c;
            }
            loc[i] = sum;
            sum += tot;
        }
        uint32_t all;
        const uint32_t ex = block_excl_scan(sum, &all);
#pragma unroll
        for (int i = 0; i < DPT; i++) tstart[threadIdx.x * DPT + i] = ex + loc[i];
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < RADIX_ITEMS; j++) {
        if (wbase + j * 64 < n) {
            const uint32_t d = (key[j] >> shift) & (ND - 1);
            lp[j] += tstart[d] + wcnt[w][d];
            dig[lp[j]] = (dig_t)d;
        }
    }
    __syncthreads();
    // write-out through LDS: contiguous runs per digit
#define SH_STAGE_OUT(T, SRCEXPR, DST)                                                           \
    {                                                                                           \
        for (int j = 0; j < RADIX_ITEMS; j++) {                                                 \
            const int64_t i = wbase + j * 64;                                                   \
            if (i < n) stage[lp[j]] = (uint32_t)(SRCEXPR);                                      \
        }                                                                                       \
        __syncthreads();                                                                        \
        for (int m = 0; m < RADIX_ITEMS; m++) {                                                 \
            const int l = m * TPB + threadIdx.x;                                                \
            if (l < tile_n) {                                                                   \
                const uint32_t d = dig[l];                                                      \
                ((T*)(DST))[gbase[d] + (uint32_t)l - tstart[d]] = (T)stage[l];                  \
            }                                                                                   \
        }                                                                                       \
        __syncthreads();                                                                        \
    }
    SH_STAGE_OUT(uint32_t, key[j], keys_out);
    SH_STAGE_OUT(uint32_t, (idx_in ? idx_in[i] : (uint32_t)i), idx_out);
    // PL.pad: the columns are in arrival order and gathered through idx_in (payload
    // carried by the last pass only)
    const bool gather = PL.pad && idx_in;
    for (int c = 0; c < PL.n; c++) {
        if (PL.width[c] == 8) {
            const uint64_t* src = (const uint64_t*)PL.src[c];
            uint64_t* dst = (uint64_t*)PL.dst[c];
            uint64_t v[RADIX_ITEMS];
#pragma unroll
            for (int j = 0; j < RADIX_ITEMS; j++) {
                const int64_t i = wbase + j * 64;
                v[j] = (i < n) ? src[gather ? idx_in[i] : i] : 0ull;
            }
            uint64_t* st64 = (uint64_t*)stage;
            constexpr uint32_t HALF = RADIX_TILE / 2;
            // tile_n <= 0 for the padding tiles of arrival-tile-major order: no rounds
            const uint32_t tn = tile_n > 0 ? (uint32_t)tile_n : 0u;
            for (uint32_t lo = 0; lo < tn; lo += HALF) {  // uniform
#pragma unroll
                for (int j = 0; j < RADIX_ITEMS; j++)
                    if (wbase + j * 64 < n && lp[j] - lo < HALF) st64[lp[j] - lo] = v[j];
                __syncthreads();
#pragma unroll
                for (int m = 0; m < RADIX_ITEMS / 2; m++) {
                    const uint32_t l = lo + m * TPB + threadIdx.x;
                    if (l < tn) {
                        const uint32_t d = dig[l];
                        dst[gbase[d] + l - tstart[d]] = st64[l - lo];
                    }
                }
                __syncthreads();
            }
        } else if (PL.width[c] == 4) {
            const uint32_t* src = (const uint32_t*)PL.src[c];
            SH_STAGE_OUT(uint32_t, src[gather ? idx_in[i] : i], PL.dst[c]);
        } else {
            const uint8_t* src = (const uint8_t*)PL.src[c];
            SH_STAGE_OUT(uint8_t, src[gather ? idx_in[i] : i], PL.dst[c]);
        }
    }
#undef SH_STAGE_OUT
}

// segment starts: flag positions where the (sorted) key changes; sentinel excluded
__global__ void k_seg_flags(const uint32_t* __restrict__ skeys, int64_t n, uint32_t sentinel,
                            uint32_t* __restrict__ flags) {
    int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n) return;
    uint32_t k = skeys ? skeys[p] : 0u;
    bool start = (p == 0) || (skeys && skeys[p - 1] != k);
    flags[p] = (start && k != sentinel) ? 1u : 0u;
}

__global__ void k_seg_compact(const uint32_t* __restrict__ flags, const uint32_t* __restrict__ pos, int64_t n,
                              uint32_t* __restrict__ seg_list, uint32_t* __restrict__ nseg) {
    int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n) return;
    if (flags[p]) seg_list[pos[p]] = (uint32_t)p;
    if (p == n - 1) *nseg = pos[p] + flags[p];
}

#include "sh_vm.h"

// ------------------------------------------------------------------ per-key state
// key block layout (8-byte words):
//   [0] flags: bit0 initialized, bit1 start template pending, bit2 start template in new-and-every
//   [1 .. n]   list counts: word 1+k = pending count of state k | (nae count << 32)
//   off_lists: per state k in 1..n-1: pending[cap] then nae[cap]; record = ts, ts0, rows[n] (u32)
//   off_agg:   per output: dsum, lsum, cnt, mx bits, mx null
struct KeyView {
    uint64_t* base;
    const shp_layout* L;
    __device__ uint64_t* list(int k, int which) const {  // which 0 pending, 1 nae
        return (uint64_t*)((uint8_t*)base + L->off_lists + ((int64_t)(k - 1) * 2 + which) * L->list_bytes);
    }
    __device__ uint64_t* rec(uint64_t* lst, int i) const { return lst + (int64_t)i * L->rec_words; }
    __device__ uint32_t pcount(int k) const { return (uint32_t)base[1 + k]; }
    __device__ uint32_t ncount(int k) const { return (uint32_t)(base[1 + k] >> 32); }
    __device__ void set_counts(int k, uint32_t p, uint32_t n) const { base[1 + k] = (uint64_t)p | ((uint64_t)n << 32); }
};

__device__ __forceinline__ void rec_copy(uint64_t* dst, const uint64_t* src, int words) {
    for (int i = 0; i < words; i++) dst[i] = src[i];
}

struct Emitter {
    const shd_emit* em;
    uint64_t* chunk;
    int64_t used, cap;
    int rec_words;
};

#define EMIT_CHUNK 64

__device__ __forceinline__ uint64_t* emit_slot(Emitter& E) {
    if (E.used == E.cap) {
        unsigned long long at = atomicAdd(E.em->tmp_ctr, (unsigned long long)EMIT_CHUNK);
        if ((int64_t)at + EMIT_CHUNK > E.em->tmp_cap) {
            atomicExch(&E.em->err[1], 1);
            return nullptr;
        }
        E.chunk = E.em->tmp + (int64_t)at * E.rec_words;
        E.used = 0;
        E.cap = EMIT_CHUNK;
    }
    uint64_t* r = E.chunk + E.used * E.rec_words;
    E.used++;
    return r;
}

// QuerySelector.processNoGroupBy / processInBatchNoGroupBy for one match + the
// Sum/Avg/Count/Max/Min aggregators (per partition key, match order)
__device__ void emit_match(const shp_program* __restrict__ P, const KeyView& K, Emitter& E, const uint32_t* rows,
                           const shd_cols* __restrict__ C, uint32_t local_i, uint32_t ordinal, int64_t ts) {
    uint64_t* r = emit_slot(E);
    uint64_t nullmask = 0;
    uint64_t* agg = (uint64_t*)((uint8_t*)K.base + K.L->off_agg);
    for (int o = 0; o < P->n_out; o++) {
        const int aggk = P->out_agg[o];
        VmVal v;
        if (P->out_pc[o] >= 0)
            v = vm_eval(P, P->out_pc[o], P->out_len[o], rows, C);
        else {
            v.null = 0;
            v.b = 1;
            v.t = SH_T_BOOL;
        }
        int64_t outb = v.b;
        bool outnull = v.null;
        if (aggk != SH_AGG_NONE) {
            uint64_t* a = agg + o * 5;
            double dsum = __longlong_as_double((long long)a[0]);
            int64_t lsum = (int64_t)a[1];
            int64_t cnt = (int64_t)a[2];
            switch (aggk) {
                case SH_AGG_SUM:
                    if (!v.null) {
                        if (v.t == SH_T_INT || v.t == SH_T_LONG)
                            lsum += to_i64(v);
                        else
                            dsum = __dadd_rn(dsum, to_f64(v));
                        cnt++;
                    }
                    outnull = false;
                    outb = (P->out_type[o] == SH_T_LONG) ? lsum : f64_bits(dsum);
                    break;
                case SH_AGG_AVG:
                    if (!v.null) {
                        dsum = __dadd_rn(dsum, to_f64(v));
                        cnt++;
                    }
                    outnull = cnt == 0;
                    outb = outnull ? 0 : f64_bits(__ddiv_rn(dsum, (double)cnt));
                    break;
                case SH_AGG_COUNT:
                    cnt++;
                    outnull = false;
                    outb = cnt;
                    break;
                default: {  // MAX / MIN
                    if (!v.null) {
                        VmVal m;
                        m.b = (int64_t)a[3];
                        m.t = v.t;
                        m.null = (uint8_t)a[4];
                        bool better = m.null;
                        if (!better) {
                            const int op = aggk == SH_AGG_MAX ? SH_OP_GT : SH_OP_LT;
                            switch (v.t) {
                                case SH_T_INT: better = cmp_op<int32_t>(op, (int32_t)v.b, (int32_t)m.b); break;
                                case SH_T_LONG: better = cmp_op<int64_t>(op, v.b, m.b); break;
                                case SH_T_FLOAT: better = cmp_op<float>(op, bits_f32(v.b), bits_f32(m.b)); break;
                                default: better = cmp_op<double>(op, bits_f64(v.b), bits_f64(m.b)); break;
                            }
                        }
                        if (better) {
                            a[3] = (uint64_t)v.b;
                            a[4] = 0;
                        }
                    }
                    outnull = a[4] != 0;
                    outb = (int64_t)a[3];
                }
            }
            a[0] = (uint64_t)__double_as_longlong(dsum);
            a[1] = (uint64_t)lsum;
            a[2] = (uint64_t)cnt;
        }
        if (r) r[3 + o] = (uint64_t)outb;
        if (outnull) nullmask |= (1ull << o);
    }
    if (r) {
        r[0] = (uint64_t)local_i | ((uint64_t)ordinal << 32);
        r[1] = (uint64_t)ts;
        r[2] = nullmask;
    }
}

__device__ __forceinline__ bool expired(const uint64_t* rec, int64_t now, int64_t within) {
    const int64_t ts0 = (int64_t)rec[1];
    const int64_t d = ts0 - now;
    return (d < 0 ? -d : d) > within;
}

// ------------------------------------------------------------------ advance kernel
// One lane per key segment: replays StreamPreStateProcessor / StreamPostStateProcessor
// for a PATTERN chain over the key's events in arrival order.
__global__ void __launch_bounds__(TPB) k_advance(const shp_program* __restrict__ P, shp_layout L,
                                                 uint8_t* __restrict__ kstate, shd_batch B,
                                                 const uint32_t* __restrict__ perm, const uint32_t* __restrict__ skeys,
                                                 const uint32_t* __restrict__ seg_list, const uint32_t* __restrict__ nseg,
                                                 const shd_cols* __restrict__ C, shd_emit EM, int32_t nkeys,
                                                 int fast_ok) {
    const uint32_t sidx = blockIdx.x * blockDim.x + threadIdx.x;
    if (sidx >= *nseg) return;
    const uint32_t beg = seg_list[sidx];
    const uint32_t key = skeys ? skeys[beg] : 0u;
    if (key >= (uint32_t)nkeys) {  // key id outside the allocated key state
        atomicExch(&EM.err[0], 2);
        return;
    }
    KeyView K;
    K.base = (uint64_t*)(kstate + (int64_t)key * L.key_bytes);
    K.L = &L;
    const int n = P->n_states;
    const int rw = L.rec_words;
    const int64_t within = P->within_ms;
    Emitter E;
    E.em = &EM;
    E.chunk = nullptr;
    E.used = 0;
    E.cap = 0;
    E.rec_words = 3 + P->n_out;
    uint64_t flags = K.base[0];
    if (!(flags & 1ull)) {
        // initPartition -> StreamPreStateProcessor.init: start template into new-and-every
        flags = 1ull | 4ull;
        for (int k = 1; k < n; k++) K.set_counts(k, 0, 0);
    }
    uint32_t rows[SHP_MAX_STATES];
    for (int64_t p = beg; p < B.n; p++) {
        if (p != beg && skeys && skeys[p] != key) break;
        const uint32_t i = perm ? perm[p] : (uint32_t)p;
        const int64_t t = B.ts[i];
        const int s = B.stream ? B.stream[i] : 0;
        const uint32_t row = B.row ? B.row[i] : B.row_base + i;
        uint32_t nmatch = 0;
        // (5) within expiry on every state (PatternMultiProcessStreamReceiver.stabilizeStates)
        if (within >= 0) {
            for (int k = 1; k < n; k++) {
                uint32_t pc = K.pcount(k), nc = K.ncount(k);
                uint64_t* pl = K.list(k, 0);
                uint32_t e = 0;
                while (e < pc && expired(K.rec(pl, e), t, within)) e++;  // break at first live
                if (e) {
                    for (uint32_t q = e; q < pc; q++) rec_copy(K.rec(pl, q - e), K.rec(pl, q), rw);
                    pc -= e;
                }
                uint64_t* nl = K.list(k, 1);
                uint32_t wpos = 0;
                for (uint32_t q = 0; q < nc; q++) {
                    if (!expired(K.rec(nl, q), t, within)) {
                        if (wpos != q) rec_copy(K.rec(nl, wpos), K.rec(nl, q), rw);
                        wpos++;
                    }
                }
                K.set_counts(k, pc, wpos);
            }
        }
        // updateState for the states this stream drives
        for (int u = 0; u < P->upd_count[s]; u++) {
            const int k = P->upd_state[s][u];
            if (k == 0) {
                if (flags & 4ull) flags = (flags | 2ull) & ~4ull;
                continue;
            }
            uint32_t pc = K.pcount(k), nc = K.ncount(k);
            if (!nc) continue;
            uint64_t* nl = K.list(k, 1);
            // stable insertion sort by StateEvent timestamp (-1 last)
            for (uint32_t a = 1; a < nc; a++) {
                uint64_t tmp[2 + SHP_MAX_STATES / 2 + 1];
                rec_copy(tmp, K.rec(nl, a), rw);
                const int64_t ta = (int64_t)tmp[0];
                int32_t b = (int32_t)a - 1;
                while (b >= 0) {
                    const int64_t tb = (int64_t)K.rec(nl, b)[0];
                    const bool gt = (tb == -1) ? (ta != -1) : (ta != -1 && tb > ta);
                    if (!gt) break;
                    rec_copy(K.rec(nl, b + 1), K.rec(nl, b), rw);
                    b--;
                }
                rec_copy(K.rec(nl, b + 1), tmp, rw);
            }
            if (pc + nc > (uint32_t)L.cap) {
                atomicExch(&EM.err[0], 1);
                nc = L.cap - pc;
            }
            uint64_t* pl = K.list(k, 0);
            for (uint32_t q = 0; q < nc; q++) rec_copy(K.rec(pl, pc + q), K.rec(nl, q), rw);
            K.set_counts(k, pc + nc, 0);
        }
        // processAndReturn in eventSequence order (later states first)
        for (int u = 0; u < P->proc_count[s]; u++) {
            const int k = P->proc_state[s][u];
            if (k == 0) {
                if (!(flags & 2ull)) continue;
                for (int q = 0; q < n; q++) rows[q] = SHD_NULL_ROW;
                rows[0] = row;
                if (!filter_pass(P, 0, rows, C, fast_ok)) continue;
                flags &= ~2ull;                       // template leaves pending (stateChanged)
                if (P->every_start) flags |= 4ull;    // addEveryState: fresh clone into new-and-every
                if (n == 1) {
                    emit_match(P, K, E, rows, C, i, nmatch++, t);
                } else {
                    uint32_t pc = K.pcount(1), nc = K.ncount(1);
                    if (nc >= (uint32_t)L.cap) {
                        atomicExch(&EM.err[0], 1);
                        continue;
                    }
                    uint64_t* r = K.rec(K.list(1, 1), nc);
                    r[0] = (uint64_t)t;   // StateEvent ts := matched event ts
                    r[1] = (uint64_t)t;   // start-state event ts (within)
                    uint32_t* rr = (uint32_t*)(r + 2);
                    for (int q = 0; q < n; q++) rr[q] = rows[q];
                    K.set_counts(1, pc, nc + 1);
                }
                continue;
            }
            uint32_t pc = K.pcount(k);
            if (!pc) continue;
            uint64_t* pl = K.list(k, 0);
            uint32_t w = 0;
            for (uint32_t q = 0; q < pc; q++) {
                uint64_t* r = K.rec(pl, q);
                uint32_t* rr = (uint32_t*)(r + 2);
                for (int z = 0; z < n; z++) rows[z] = rr[z];
                rows[k] = row;
                if (filter_pass(P, k, rows, C, fast_ok)) {
                    if (k == n - 1) {
                        emit_match(P, K, E, rows, C, i, nmatch++, t);
                    } else {
                        uint32_t npc = K.pcount(k + 1), nnc = K.ncount(k + 1);
                        if (nnc >= (uint32_t)L.cap) {
                            atomicExch(&EM.err[0], 1);
                        } else {
                            uint64_t* d = K.rec(K.list(k + 1, 1), nnc);
                            d[0] = (uint64_t)t;
                            d[1] = r[1];
                            uint32_t* dr = (uint32_t*)(d + 2);
                            for (int z = 0; z < n; z++) dr[z] = rows[z];
                            K.set_counts(k + 1, npc, nnc + 1);
                        }
                    }
                } else {
                    if (w != q) rec_copy(K.rec(pl, w), r, rw);
                    w++;
                }
            }
            K.set_counts(k, w, K.ncount(k));
        }
        if (nmatch) EM.match_cnt[i] = nmatch;
    }
    K.base[0] = flags;
    for (int64_t q = E.used; q < E.cap; q++) E.chunk[q * E.rec_words] = ~0ull;  // unused tail
}

// ------------------------------------------------------------------ list capacity growth
// re-lays every key's state from layout `A` into layout `B` (bigger list capacity)
__global__ void k_relayout(const uint8_t* __restrict__ src, shp_layout A, uint8_t* __restrict__ dst, shp_layout B,
                           int32_t nkeys, int32_t n_states, int32_t n_out) {
    const int32_t key = blockIdx.x * blockDim.x + threadIdx.x;
    if (key >= nkeys) return;
    const uint64_t* s = (const uint64_t*)(src + (int64_t)key * A.key_bytes);
    uint64_t* d = (uint64_t*)(dst + (int64_t)key * B.key_bytes);
    for (int w = 0; w < 1 + SHP_MAX_STATES; w++) d[w] = s[w];
    for (int k = 1; k < n_states; k++) {
        const uint32_t cnt[2] = {(uint32_t)s[1 + k], (uint32_t)(s[1 + k] >> 32)};
        for (int which = 0; which < 2; which++) {
            const uint64_t* sl = (const uint64_t*)((const uint8_t*)s + A.off_lists + ((int64_t)(k - 1) * 2 + which) * A.list_bytes);
            uint64_t* dl = (uint64_t*)((uint8_t*)d + B.off_lists + ((int64_t)(k - 1) * 2 + which) * B.list_bytes);
            for (int64_t w = 0; w < (int64_t)cnt[which] * A.rec_words; w++) dl[w] = sl[w];
        }
    }
    const uint64_t* sa = (const uint64_t*)((const uint8_t*)s + A.off_agg);
    uint64_t* da = (uint64_t*)((uint8_t*)d + B.off_agg);
    for (int w = 0; w < n_out * 5; w++) da[w] = sa[w];
}

extern "C" int shd_relayout(const uint8_t* src, const shp_layout* A, uint8_t* dst, const shp_layout* B, int32_t nkeys,
                            int32_t n_states, int32_t n_out, void* stream) {
    if (nkeys <= 0) return 0;
    hipLaunchKernelGGL(k_relayout, dim3((unsigned)ceil_div(nkeys, TPB)), dim3(TPB), 0, (hipStream_t)stream, src, *A,
                       dst, *B, nkeys, n_states, n_out);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

// ------------------------------------------------------------------ ordered placement
__global__ void k_place(const uint64_t* __restrict__ tmp, int64_t nrec, int rec_words, int n_out,
                        const uint32_t* __restrict__ offsets, uint64_t seq_base, uint64_t* __restrict__ out_seq,
                        int64_t* __restrict__ out_ts, int64_t* __restrict__ out_vals, uint8_t* __restrict__ out_nulls) {
    int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= nrec) return;
    const uint64_t* rec = tmp + r * rec_words;
    const uint64_t h = rec[0];
    if (h == ~0ull) return;  // unused slot of a partially filled chunk
    const uint32_t li = (uint32_t)h, ord = (uint32_t)(h >> 32);
    const int64_t dst = (int64_t)offsets[li] + ord;
    if (out_seq) out_seq[dst] = seq_base + li;
    if (out_ts) out_ts[dst] = (int64_t)rec[1];
    for (int o = 0; o < n_out; o++) {
        if (out_vals) out_vals[dst * n_out + o] = (int64_t)rec[3 + o];
        if (out_nulls) out_nulls[dst * n_out + o] = (uint8_t)((rec[2] >> o) & 1);
    }
}

// ------------------------------------------------------------------ host entry points
// XCD-ordered scatter tiles (SH_RADIX_XCD=0 turns it off for A/B runs)
static int radix_xcd() {
    static const int on = [] {
        const char* e = getenv("SH_RADIX_XCD");
        return e && e[0] == '0' ? 0 : 1;
    }();
    return on;
}
// 10-bit digits for 17..20-bit key ranges: opt-in (SH_RADIX10=1). Measured on C3 / C5
// (1M keys): two 10-bit passes 6.9 ms vs three 8-bit passes 6.35 ms for the segment
// phase; a 1024-digit tile needs 64 KB of LDS (2 blocks per CU) and writes runs of ~4
static int radix10() {
    static const int on = [] {
        const char* e = getenv("SH_RADIX10");
        return e && e[0] == '1' ? 1 : 0;
    }();
    return on;
}
static unsigned scatter_grid(int64_t ntiles) { return radix_xcd() ? 8u * (unsigned)((ntiles + 7) >> 3) : (unsigned)ntiles; }
static uint32_t g_bits_for(uint32_t maxkey) {
    uint32_t b = 0;
    while (b < 32 && (maxkey >> b)) b++;
    return b;
}

// Small batches (a send() call of the streaming path, n <= SEG1_MAXN, no carried
// columns): the whole segment in ONE workgroup -- stable LSD passes of 8-bit digits
// in LDS (shw_rank8 ranks each round in element order), then the segment starts --
// instead of ~15 launches (histogram, scans and scatter per pass, flags, scan,
// compaction) that each cost more than the work of a 4,096-event call.
#define SEG1_NT 512
#define SEG1_MAXN 4096
#define SEG1_R (SEG1_MAXN / SEG1_NT)
__global__ void __launch_bounds__(SEG1_NT) k_segment_small(const int32_t* __restrict__ raw, int64_t n, uint32_t sentinel,
                                                           int passes, uint32_t* __restrict__ keys_out,
                                                           uint32_t* __restrict__ idx_out, uint32_t* __restrict__ seg_list,
                                                           uint32_t* __restrict__ nseg) {
    __shared__ uint32_t kA[SEG1_MAXN], kB[SEG1_MAXN];
    __shared__ uint16_t iA[SEG1_MAXN], iB[SEG1_MAXN];
    __shared__ uint32_t wcnt[SEG1_NT / 64][256];
    __shared__ uint32_t run[256], ws[SEG1_NT / 64];
    const int nn = (int)n;
    for (int i = threadIdx.x; i < nn; i += SEG1_NT) {
        const int32_t r = raw[i];
        kA[i] = r < 0 ? sentinel : (uint32_t)r;
        iA[i] = (uint16_t)i;
    }
    uint32_t* kin = kA;
    uint32_t* kout = kB;
    uint16_t* iin = iA;
    uint16_t* iout = iB;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
    for (int ps = 0; ps < passes; ps++) {
        const int shift = 8 * ps;
        for (int i = threadIdx.x; i < (SEG1_NT / 64) * 256; i += SEG1_NT) (&wcnt[0][0])[i] = 0u;
        __syncthreads();
        // each wave ranks its own contiguous SEG1_R rounds of 64 events in order,
        // keeping its running per-digit counts (no block barrier per round)
        uint32_t rk[SEG1_R], dg[SEG1_R];
#pragma unroll
        for (int r = 0; r < SEG1_R; r++) {
            const int i = (wv * SEG1_R + r) * 64 + lane;
            const bool valid = i < nn;
            const uint32_t d = valid ? (kin[i] >> shift) & 0xFFu : 0u;
            uint64_t peers = __ballot(valid);
#pragma unroll
            for (int b = 0; b < 8; b++) {
                const bool bit = (d >> b) & 1u;
                const uint64_t m = __ballot(valid && bit);
                peers &= bit ? m : ~m;
            }
            const uint32_t rr = (uint32_t)__popcll(peers & lt);
            const uint32_t base = valid ? wcnt[wv][d] : 0u;
            if (valid && rr == 0) wcnt[wv][d] = base + (uint32_t)__popcll(peers);
            rk[r] = base + rr;
            dg[r] = valid ? d : 0x100u;
        }
        __syncthreads();
        // (digit, wave) starts: digits in order, waves in order inside a digit
        {
            uint32_t tot_d = 0;
            if (threadIdx.x < 256) {
#pragma unroll
                for (int q = 0; q < SEG1_NT / 64; q++) {
                    const uint32_t c = wcnt[q][threadIdx.x];
                    wcnt[q][threadIdx.x] = tot_d;
                    tot_d += c;
                }
            }
            uint32_t tot;
            const uint32_t ex = shw_block_excl<SEG1_NT>(threadIdx.x < 256 ? tot_d : 0u, ws, &tot);
            if (threadIdx.x < 256) run[threadIdx.x] = ex;
            __syncthreads();
        }
#pragma unroll
        for (int r = 0; r < SEG1_R; r++) {
            const int i = (wv * SEG1_R + r) * 64 + lane;
            if (dg[r] < 0x100u) {
                const uint32_t pos = run[dg[r]] + wcnt[wv][dg[r]] + rk[r];
                kout[pos] = kin[i];
                iout[pos] = iin[i];
            }
        }
        __syncthreads();
        uint32_t* tk = kin;
        kin = kout;
        kout = tk;
        uint16_t* ti = iin;
        iin = iout;
        iout = ti;
    }
    // sorted keys and permutation out; segment starts (a key change, the null-key
    // sentinel excluded) into kout as 0/1 flags, scanned in place
    for (int i = threadIdx.x; i < nn; i += SEG1_NT) {
        const uint32_t k = kin[i];
        keys_out[i] = k;
        idx_out[i] = (uint32_t)iin[i];
        kout[i] = ((i == 0 || kin[i - 1] != k) && k != sentinel) ? 1u : 0u;
    }
    __syncthreads();
    uint32_t flag[SEG1_R];
#pragma unroll
    for (int r = 0; r < SEG1_R; r++) {
        const int i = threadIdx.x * SEG1_R + r;
        flag[r] = i < nn ? kout[i] : 0u;
    }
    const uint32_t total = shw_lds_excl_scan<SEG1_NT, SEG1_R>(kout, nn, ws);
#pragma unroll
    for (int r = 0; r < SEG1_R; r++) {
        const int i = threadIdx.x * SEG1_R + r;
        if (i < nn && flag[r]) seg_list[kout[i]] = (uint32_t)i;
    }
    if (threadIdx.x == 0) *nseg = total;
}

extern "C" int shd_segment_payload(const shd_batch* b, int32_t nkeys, shd_segment_ws* ws, void* stream,
                                   const uint32_t** perm_out, const uint32_t** skeys_out, const shd_payload* carry,
                                   void* const* mid, int tile_shift, int want_segments) {
    hipStream_t st = (hipStream_t)stream;
    const int64_t n = b->n;
    const uint32_t sentinel = (uint32_t)nkeys;
    // arrival tiles of 2^tile_shift events (0: one global segment order)
    const int sub_shift = tile_shift >= 12 ? tile_shift - 12 : -1;
    int64_t ntiles = ceil_div(n, RADIX_TILE);
    if (sub_shift >= 0) ntiles = ceil_div(ntiles, (int64_t)1 << sub_shift) << sub_shift;
    const uint32_t bits = g_bits_for(sentinel);
    static const bool small_on = !(getenv("SH_SEG_SMALL") && getenv("SH_SEG_SMALL")[0] == '0');
    if (small_on && b->keys && n <= SEG1_MAXN && n > 0 && !carry && want_segments && sub_shift < 0 && bits <= 32) {
        // the whole segment in one workgroup (small send() calls)
        const int passes8 = (int)((bits + 7) / 8);
        uint32_t* seg_list = ws->seg_off + 2 * n;
        hipLaunchKernelGGL(k_segment_small, dim3(1), dim3(SEG1_NT), 0, st, b->keys, n, sentinel, passes8, ws->keys_a,
                           ws->idx_a, seg_list, seg_list + n);
        *perm_out = ws->idx_a;
        *skeys_out = ws->keys_a;
        return hipGetLastError() == hipSuccess ? 0 : -3;
    }
    // 17..20-bit key ranges: two passes of 10-bit digits instead of three of 8 (opt-in)
    const int db = (bits > 16 && bits <= 20 && radix10()) ? 10 : 8;
    const int passes = b->keys ? (int)((bits + db - 1) / db) : 0;
    const uint32_t* kin = nullptr;
    const uint32_t* iin = nullptr;
    uint32_t* kout = ws->keys_a;
    uint32_t* iout = ws->idx_a;
    for (int ps = 0; ps < passes; ps++) {
        const int shift = ps * db;
        if (db == 10)
            hipLaunchKernelGGL(k_digit_hist<10>, dim3((unsigned)ntiles), dim3(TPB), 0, st, kin, b->keys, sentinel, n,
                               shift, ws->hist, ntiles, sub_shift);
        else
            hipLaunchKernelGGL(k_digit_hist<8>, dim3((unsigned)ntiles), dim3(TPB), 0, st, kin, b->keys, sentinel, n,
                               shift, ws->hist, ntiles, sub_shift);
        int rc = shd_exclusive_scan(ws->hist, ws->hist, ((int64_t)1 << db) * ntiles, ws->scan_tmp, stream);
        if (rc) return rc;
        // payload ping-pong: pass ps reads the previous pass's output (or the
        // original columns) and writes `mid` (odd distance to the last pass) or
        // the final arrays
        shd_payload PL;
        memset(&PL, 0, sizeof(PL));
        static const bool last_carry = [] {
            const char* e = getenv("SH_SEG_LASTCARRY");
            return e && e[0] == '1';
        }();
        if (carry && last_carry) {
            // the columns travel once, in the last pass, gathered by arrival index
            if (ps == passes - 1) {
                PL = *carry;
                PL.pad = 1;
            }
        } else if (carry) {
            PL = *carry;
            PL.pad = 0;
            const bool last = ps == passes - 1;
            const bool to_mid = ((passes - 1 - ps) & 1) != 0;
            for (int c = 0; c < carry->n; c++) {
                const void* src = (ps == 0) ? carry->src[c] : (((passes - ps) & 1) ? mid[c] : carry->dst[c]);
                PL.src[c] = src;
                PL.dst[c] = last ? carry->dst[c] : (to_mid ? mid[c] : carry->dst[c]);
            }
        }
        if (db == 10)
            hipLaunchKernelGGL(k_digit_scatter<10>, dim3(scatter_grid(ntiles)), dim3(TPB), 0, st, kin, b->keys, sentinel,
                               iin, n, shift, (const uint32_t*)ws->hist, ntiles, kout, iout, PL, sub_shift, radix_xcd());
        else
            hipLaunchKernelGGL(k_digit_scatter<8>, dim3(scatter_grid(ntiles)), dim3(TPB), 0, st, kin, b->keys, sentinel,
                               iin, n, shift, (const uint32_t*)ws->hist, ntiles, kout, iout, PL, sub_shift, radix_xcd());
        kin = kout;
        iin = iout;
        kout = (kout == ws->keys_a) ? ws->keys_b : ws->keys_a;
        iout = (iout == ws->idx_a) ? ws->idx_b : ws->idx_a;
    }
    // kin/iin: sorted keys / permutation (NULL when nothing to sort: single key)
    *perm_out = iin;
    *skeys_out = kin;
    if (!want_segments) return hipGetLastError() == hipSuccess ? 0 : -3;
    uint32_t* flags = ws->seg_off;          // [n]
    uint32_t* pos = ws->seg_off + n;        // [n]
    uint32_t* seg_list = ws->seg_off + 2 * n;  // [n + 1]
    const unsigned g = (unsigned)ceil_div(n, TPB);
    hipLaunchKernelGGL(k_seg_flags, dim3(g), dim3(TPB), 0, st, kin, n, kin ? sentinel : 0xFFFFFFFFu, flags);
    int rc = shd_exclusive_scan(flags, pos, n, ws->scan_tmp, stream);
    if (rc) return rc;
    hipLaunchKernelGGL(k_seg_compact, dim3(g), dim3(TPB), 0, st, (const uint32_t*)flags, (const uint32_t*)pos, n,
                       seg_list, seg_list + n);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

#define SMALL_TILES 16
// stable LSD radix sort of (key, value) pairs by the low `bits` of the key
// (vals NULL: identity); the result lies in the kbuf / vbuf ping-pong buffers,
// which must not alias the inputs
extern "C" int shd_sort_pairs(const uint32_t* keys, const uint32_t* vals, int64_t n, int bits, uint32_t* const* kbuf,
                              uint32_t* const* vbuf, uint32_t* hist, uint32_t* scan_tmp, void* stream,
                              const uint32_t** keys_out, const uint32_t** vals_out) {
    hipStream_t st = (hipStream_t)stream;
    const int64_t ntiles = ceil_div(n, RADIX_TILE);
    const int passes = (bits + 7) / 8;
    const uint32_t* kin = keys;
    const uint32_t* vin = vals;
    shd_payload PL;
    memset(&PL, 0, sizeof(PL));
    for (int ps = 0; ps < passes && n > 0; ps++) {
        const int shift = ps * 8;
        hipLaunchKernelGGL(k_digit_hist<8>, dim3((unsigned)ntiles), dim3(TPB), 0, st, kin, (const int32_t*)nullptr,
                           0xFFFFFFFFu, n, shift, hist, ntiles, -1);
        // a few tiles (a rule run's records): every scatter workgroup sums the counts
        // itself, no scan launches
        // (profiles/r6_c5_sort_small_ab.txt: the record order 0.05 ms faster on C5)
        const bool small = ntiles <= SMALL_TILES;
        if (!small) {
            int rc = shd_exclusive_scan(hist, hist, 256 * ntiles, scan_tmp, stream);
            if (rc) return rc;
        }
        hipLaunchKernelGGL(k_digit_scatter<8>, dim3(scatter_grid(ntiles)), dim3(TPB), 0, st, kin, (const int32_t*)nullptr,
                           0xFFFFFFFFu, vin, n, shift, (const uint32_t*)hist, ntiles, kbuf[ps & 1], vbuf[ps & 1], PL,
                           -1, radix_xcd(), small ? 1 : 0);
        kin = kbuf[ps & 1];
        vin = vbuf[ps & 1];
    }
    *keys_out = kin;
    *vals_out = vin;
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

extern "C" int shd_segment(const shd_batch* b, int32_t nkeys, shd_segment_ws* ws, void* stream,
                           const uint32_t** perm_out, const uint32_t** skeys_out) {
    return shd_segment_payload(b, nkeys, ws, stream, perm_out, skeys_out, nullptr, nullptr, 0, 1);
}

extern "C" int shd_advance(const shp_program* dprog, const shp_layout* lay, uint8_t* kstate, int32_t nkeys,
                           const shd_batch* b, const uint32_t* perm, const uint32_t* skeys, const uint32_t* seg_off,
                           const shd_cols* dcols, const shd_emit* em, void* stream, int fast_ok) {
    hipStream_t st = (hipStream_t)stream;
    const int64_t n = b->n;
    const uint32_t* seg_list = seg_off + 2 * n;
    const uint32_t* nseg = seg_list + n;
    // the segment count is only known on device: size the grid for the worst
    // case (every key present), lanes past *nseg exit at once
    int64_t maxseg = n < (int64_t)nkeys ? n : (int64_t)nkeys;
    if (maxseg < 1) maxseg = 1;
    const unsigned g = (unsigned)ceil_div(maxseg, TPB);
    hipLaunchKernelGGL(k_advance, dim3(g), dim3(TPB), 0, st, dprog, *lay, kstate, *b, perm, skeys, seg_list, nseg,
                       dcols, *em, nkeys, fast_ok);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

extern "C" int shd_emit_place(const shd_emit* em, int32_t n_out, int64_t n_events, uint32_t* offsets,
                              uint32_t* scan_tmp, int64_t n_records, const shd_batch* b, uint64_t* out_seq,
                              int64_t* out_ts, int64_t* out_vals, uint8_t* out_nulls, void* stream) {
    hipStream_t st = (hipStream_t)stream;
    if (n_events > 0) {  // offsets of each event's matches in the ordered output
        int rc = shd_exclusive_scan(em->match_cnt, offsets, n_events, scan_tmp, stream);
        if (rc) return rc;
    }
    const bool any_out = out_seq || out_ts || out_vals || out_nulls;
    if (n_records > 0 && any_out) {
        hipLaunchKernelGGL(k_place, dim3((unsigned)ceil_div(n_records, TPB)), dim3(TPB), 0, st,
                           (const uint64_t*)em->tmp, n_records, 3 + n_out, n_out, (const uint32_t*)offsets,
                           b->seq_base, out_seq, out_ts, out_vals, out_nulls);
    }
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

// ------------------------------------------------------------------ PMC calibration
// Known-byte streams in the access widths the matcher kernels use (4 and 8 bytes
// per lane, coalesced), so FETCH_SIZE / WRITE_SIZE can be scaled by a measured
// factor instead of an assumed one (MI355X_MICROARCH.md, HBM: "other access
// widths are uncalibrated"). Diagnostics only (scripts/pmc_calib.py).
template <typename T>
__global__ void k_cal_read(const T* __restrict__ src, int64_t n, T* __restrict__ sink) {
    T acc = 0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        acc ^= src[i];
    if (acc == (T)0x5A5A5A5A) sink[0] = acc;  // keeps the loads; practically never stores
}
template <typename T>
__global__ void k_cal_write(T* __restrict__ dst, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        dst[i] = (T)i;
}

// kind: 0 read 4 B/lane, 1 read 8 B/lane, 2 write 4 B/lane, 3 write 8 B/lane; bytes of buf
extern "C" int shx_pmc_calibrate(int kind, void* buf, int64_t bytes, void* sink, void* stream) {
    hipStream_t st = (hipStream_t)stream;
    const dim3 g(4096), b(256);
    switch (kind) {
        case 0: hipLaunchKernelGGL(k_cal_read<uint32_t>, g, b, 0, st, (const uint32_t*)buf, bytes / 4, (uint32_t*)sink); break;
        case 1: hipLaunchKernelGGL(k_cal_read<uint64_t>, g, b, 0, st, (const uint64_t*)buf, bytes / 8, (uint64_t*)sink); break;
        case 2: hipLaunchKernelGGL(k_cal_write<uint32_t>, g, b, 0, st, (uint32_t*)buf, bytes / 4); break;
        case 3: hipLaunchKernelGGL(k_cal_write<uint64_t>, g, b, 0, st, (uint64_t*)buf, bytes / 8); break;
        default: return -1;
    }
    return hipGetLastError() == hipSuccess ? 0 : -3;
}
