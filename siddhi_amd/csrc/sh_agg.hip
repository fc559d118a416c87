// sh_agg.hip — select-clause aggregators (sum / avg / count) behind the fast engines.
//
// With aggregators a pattern query's selector keeps one running value per
// partition key and query (AttributeAggregatorExecutor state through the
// partitioned state holder, AttributeAggregatorExecutor.java:52) and emits it
// with every match in match order (a state query's selector sees one state
// event per chunk, QuerySelector.processInBatchNoGroupBy :271-313 keeps it):
//   sum(int|long) -> long  wrap-around long additions
//   sum(float|double), avg(*) -> double: value += (double) x, one double add per
//     match (SumAttributeAggregatorExecutor.java:167-185,
//     AvgAttributeAggregatorExecutor.java:145-155: value / count)
//   count() -> long
// The fast engines (bucketed / window / rise-and-fall / rule set) write the
// aggregator's argument in the aggregate's column; this pass turns the ordered
// rows into the running values.
//
// A chain of double additions is not associative, so the pass first proves it
// does not round: every addend x is an integer multiple of 2^q (q = the lowest
// set bit over all addends) and every running value the reference would form
// is then a multiple of 2^q as well. The sums are taken exactly in 128-bit
// fixed point (any order), and each running value is checked to be exactly
// representable as a double (at most 53 significant bits); when all are, every
// one of the reference's additions was exact and its results equal these bit
// for bit. Otherwise (or with NaN / infinite addends, or a fixed-point range
// over 96 bits) the pass reports "not exact" and the caller reruns the query on
// an engine that adds sequentially.
//
// Pipeline: k_sha_prep (segment id = query * nkeys + key of the trigger event,
// exponent range per column) -> stable radix sort of (segment, row) ->
// k_sha_gather (every aggregate column of a row into sorted order, one row read)
// -> per column: k_sha_tile (segmented inclusive scan of 2,048-row tiles in
// registers + LDS) -> k_sha_carry (one workgroup: segmented scan of the tile
// aggregates) -> k_sha_out (carry-in, exactness check, double conversion)
// -> k_sha_scatter (every column back into its row, one row write).
#include <hip/hip_runtime.h>
#include <string.h>

#include <algorithm>

#include "../../include/sh_query.h"
#include "sh_agg.h"
#include "sh_device.h"

#define SHA_TPB 256
#define SHA_ITEMS 8
#define SHA_TILE (SHA_TPB * SHA_ITEMS)
#define SHA_CARRY_TPB 1024

// 128-bit two's complement fixed point
struct sha_i128 {
    uint64_t lo, hi;
};
__device__ __forceinline__ sha_i128 sha_add(sha_i128 a, sha_i128 b) {
    sha_i128 r;
    r.lo = a.lo + b.lo;
    r.hi = a.hi + b.hi + (r.lo < a.lo ? 1ull : 0ull);
    return r;
}
__device__ __forceinline__ sha_i128 sha_zero() { return sha_i128{0ull, 0ull}; }

// the running value with its segment flag (segmented-scan element): flag = a
// segment starts inside the span, value = the sum since its last start
struct sha_el {
    sha_i128 v;
    int64_t c;
    uint32_t f;
};
__device__ __forceinline__ sha_el sha_comb(const sha_el& a, const sha_el& b) {
    sha_el r;
    r.f = a.f | b.f;
    r.v = b.f ? b.v : sha_add(a.v, b.v);
    r.c = b.f ? b.c : a.c + b.c;
    return r;
}

// decomposition of a double: value = m * 2^e with an odd (or zero) m
__device__ __forceinline__ void sha_split(double d, uint64_t* m, int* e, int* neg) {
    const uint64_t bits = (uint64_t)__double_as_longlong(d);
    const int ef = (int)((bits >> 52) & 0x7FF);
    uint64_t mant = bits & ((1ull << 52) - 1ull);
    int ex;
    if (ef == 0) {
        ex = -1074;
    } else {
        mant |= 1ull << 52;
        ex = ef - 1075;
    }
    if (mant) {
        const int tz = __builtin_ctzll(mant);
        mant >>= tz;
        ex += tz;
    }
    *m = mant;
    *e = ex;
    *neg = (int)(bits >> 63);
}

// the double the reference adds for a raw column value (Float/Integer/Long unboxed to double)
__device__ __forceinline__ double sha_as_double(int64_t raw, int type) {
    switch (type) {
        case SH_T_FLOAT: return (double)__uint_as_float((uint32_t)raw);
        case SH_T_DOUBLE: return __longlong_as_double(raw);
        case SH_T_INT: return (double)(int32_t)raw;
        case SH_T_LONG: return (double)raw;
        default: return 0.0;
    }
}

__device__ __forceinline__ bool sha_fp(const sha_col& c) {
    return c.kind == SH_AGG_AVG || (c.kind == SH_AGG_SUM && (c.arg_type == SH_T_FLOAT || c.arg_type == SH_T_DOUBLE));
}

// ---------------------------------------------------------------- prep
__global__ void __launch_bounds__(SHA_TPB) k_sha_prep(const uint64_t* __restrict__ seq, const int64_t* __restrict__ vals,
                                                      int n_out, int64_t m, const int32_t* __restrict__ query,
                                                      const int32_t* __restrict__ keys, int32_t nkeys,
                                                      uint64_t seq_base, sha_desc D, uint32_t* __restrict__ seg,
                                                      uint32_t* __restrict__ idx, int32_t* __restrict__ range) {
    // grid-stride over the rows with the exponent range per column in registers,
    // then one reduction per workgroup: the range words are a handful of
    // addresses, so per-wave atomics would serialise on them
    int lo[SHA_MAX_COLS], hi[SHA_MAX_COLS], bad[SHA_MAX_COLS];
#pragma unroll
    for (int k = 0; k < SHA_MAX_COLS; k++) {
        lo[k] = 1 << 30;
        hi[k] = -(1 << 30);
        bad[k] = 0;
    }
    for (int64_t r = (int64_t)blockIdx.x * SHA_TPB + threadIdx.x; r < m; r += (int64_t)gridDim.x * SHA_TPB) {
        const int64_t key = keys ? keys[seq[r] - seq_base] : 0;
        const int64_t q = query ? query[r] : 0;
        seg[r] = (uint32_t)(q * nkeys + key);
        idx[r] = (uint32_t)r;
#pragma unroll
        for (int k = 0; k < SHA_MAX_COLS; k++) {
            const sha_col c = D.c[k];
            if (k >= D.n_cols || !sha_fp(c)) continue;
            const double d = sha_as_double(vals[r * n_out + c.col], c.arg_type);
            if (!isfinite(d)) {
                bad[k] = 1;
            } else if (d != 0.0) {
                uint64_t mm;
                int e, ng;
                sha_split(d, &mm, &e, &ng);
                lo[k] = min(lo[k], e);
                hi[k] = max(hi[k], e + 63 - __builtin_clzll(mm));
            }
        }
    }
    __shared__ int s_r[SHA_TPB / 64][SHA_MAX_COLS][3];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
    for (int k = 0; k < SHA_MAX_COLS; k++) {
        if (k >= D.n_cols) continue;
        int l = lo[k], h = hi[k], b = bad[k];
        for (int o = 32; o > 0; o >>= 1) {
            l = min(l, __shfl_xor(l, o));
            h = max(h, __shfl_xor(h, o));
            b |= __shfl_xor(b, o);
        }
        if (lane == 0) {
            s_r[wave][k][0] = l;
            s_r[wave][k][1] = h;
            s_r[wave][k][2] = b;
        }
    }
    __syncthreads();
    const int k = threadIdx.x;
    if (k < D.n_cols && sha_fp(D.c[k])) {
        int l = s_r[0][k][0], h = s_r[0][k][1], b = s_r[0][k][2];
        for (int w = 1; w < SHA_TPB / 64; w++) {
            l = min(l, s_r[w][k][0]);
            h = max(h, s_r[w][k][1]);
            b |= s_r[w][k][2];
        }
        atomicMin(&range[3 * k], l);
        atomicMax(&range[3 * k + 1], h);
        if (b) atomicOr(&range[3 * k + 2], 1);
    }
}

// ---------------------------------------------------------------- scans
// the addend of sorted position p for column c (fixed point at 2^q for doubles), from
// the column's copy in sorted order (sv[p])
__device__ __forceinline__ sha_el sha_load(const int64_t* __restrict__ sv, int64_t p, const sha_col& c, int q) {
    sha_el x;
    x.f = 0;
    x.c = 1;
    x.v = sha_zero();
    const int64_t raw = sv[p];
    if (c.kind == SH_AGG_COUNT) return x;
    if (!sha_fp(c)) {
        // long arithmetic (sum of int / long): the low 64 bits wrap like Java's long
        const int64_t v = c.arg_type == SH_T_INT ? (int64_t)(int32_t)raw : raw;
        x.v.lo = (uint64_t)v;
        x.v.hi = v < 0 ? ~0ull : 0ull;
        return x;
    }
    const double d = sha_as_double(raw, c.arg_type);
    if (d == 0.0) return x;
    uint64_t mm;
    int e, ng;
    sha_split(d, &mm, &e, &ng);
    const int sh = e - q;  // 0 <= sh, sh + bits(mm) <= 96 (checked on the host)
    sha_i128 v;
    if (sh >= 64) {
        v.lo = 0ull;
        v.hi = mm << (sh - 64);
    } else if (sh > 0) {
        v.lo = mm << sh;
        v.hi = mm >> (64 - sh);
    } else {
        v.lo = mm;
        v.hi = 0ull;
    }
    if (ng) {
        v.lo = ~v.lo;
        v.hi = ~v.hi;
        v = sha_add(v, sha_i128{1ull, 0ull});
    }
    x.v = v;
    return x;
}

__device__ __forceinline__ sha_el sha_shfl_up(const sha_el& a, int o) {
    sha_el r;
    r.v.lo = (uint64_t)__shfl_up((long long)a.v.lo, o, 64);
    r.v.hi = (uint64_t)__shfl_up((long long)a.v.hi, o, 64);
    r.c = (int64_t)__shfl_up((long long)a.c, o, 64);
    r.f = (uint32_t)__shfl_up((int)a.f, o, 64);
    return r;
}

// inclusive segmented scan of one element per thread over the workgroup; the
// LDS arrays hold one element per wave
template <int NT>
__device__ __forceinline__ sha_el sha_block_scan(sha_el x, sha_el* wsum) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int o = 1; o < 64; o <<= 1) {
        const sha_el y = sha_shfl_up(x, o);
        if (lane >= o) x = sha_comb(y, x);
    }
    if (lane == 63) wsum[w] = x;
    __syncthreads();
    if (w > 0) {
        sha_el pre = wsum[0];
        for (int i = 1; i < w; i++) pre = sha_comb(pre, wsum[i]);
        x = sha_comb(pre, x);
    }
    __syncthreads();
    return x;
}

// per tile: inclusive segmented scan (sorted order) into out[], the tile's
// aggregate and the tile offset of its first segment start (SHA_TILE: none)
__global__ void __launch_bounds__(SHA_TPB) k_sha_tile(const int64_t* __restrict__ scol,
                                                      const uint32_t* __restrict__ sseg, int64_t m, sha_col c, int q,
                                                      sha_i128* __restrict__ out_v, int64_t* __restrict__ out_c,
                                                      sha_el* __restrict__ tiles, uint32_t* __restrict__ first_head) {
    __shared__ sha_el wsum[SHA_TPB / 64];
    __shared__ uint32_t fh;
    const int64_t t0 = (int64_t)blockIdx.x * SHA_TILE;
    const int64_t p0 = t0 + (int64_t)threadIdx.x * SHA_ITEMS;
    if (threadIdx.x == 0) fh = SHA_TILE;
    __syncthreads();
    sha_el it[SHA_ITEMS];
    sha_el acc;
    acc.f = 0;
    acc.c = 0;
    acc.v = sha_zero();
    uint32_t myfh = SHA_TILE;
#pragma unroll
    for (int j = 0; j < SHA_ITEMS; j++) {
        const int64_t p = p0 + j;
        sha_el x;
        if (p < m) {
            x = sha_load(scol, p, c, q);
            x.f = (p == 0 || sseg[p] != sseg[p - 1]) ? 1u : 0u;
            if (x.f && myfh == SHA_TILE) myfh = (uint32_t)(p - t0);
        } else {
            x.f = 0;
            x.c = 0;
            x.v = sha_zero();
        }
        acc = j == 0 ? x : sha_comb(acc, x);
        it[j] = acc;
    }
    if (myfh != SHA_TILE) atomicMin(&fh, myfh);
    // exclusive prefix of the thread aggregates
    const sha_el inc = sha_block_scan<SHA_TPB>(acc, wsum);
    sha_el pre = sha_shfl_up(inc, 1);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (lane == 0) {
        // the previous wave's last inclusive value
        pre.f = 0;
        pre.c = 0;
        pre.v = sha_zero();
        if (w > 0) {
            pre = wsum[0];
            for (int i = 1; i < w; i++) pre = sha_comb(pre, wsum[i]);
        }
    }
    const bool has_pre = threadIdx.x > 0;
#pragma unroll
    for (int j = 0; j < SHA_ITEMS; j++) {
        const int64_t p = p0 + j;
        if (p >= m) break;
        const sha_el y = has_pre ? sha_comb(pre, it[j]) : it[j];
        out_v[p] = y.v;
        out_c[p] = y.c;
    }
    __syncthreads();
    if (threadIdx.x == SHA_TPB - 1) {
        tiles[blockIdx.x] = inc;
        first_head[blockIdx.x] = fh;
    }
}

// exclusive segmented scan of the tile aggregates (one workgroup)
__global__ void __launch_bounds__(SHA_CARRY_TPB) k_sha_carry(sha_el* __restrict__ tiles, int64_t nt) {
    __shared__ sha_el wsum[SHA_CARRY_TPB / 64];
    const int64_t per = (nt + SHA_CARRY_TPB - 1) / SHA_CARRY_TPB;
    const int64_t b = (int64_t)threadIdx.x * per;
    sha_el acc;
    acc.f = 0;
    acc.c = 0;
    acc.v = sha_zero();
    for (int64_t t = b; t < b + per && t < nt; t++) acc = sha_comb(acc, tiles[t]);
    const sha_el inc = sha_block_scan<SHA_CARRY_TPB>(acc, wsum);
    // exclusive prefix of this thread's run
    sha_el run;
    {
        const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
        sha_el up = sha_shfl_up(inc, 1);
        if (lane == 0) {
            up.f = 0;
            up.c = 0;
            up.v = sha_zero();
            if (w > 0) {
                up = wsum[0];
                for (int i = 1; i < w; i++) up = sha_comb(up, wsum[i]);
            }
        }
        run = up;
        if (threadIdx.x == 0) {
            run.f = 0;
            run.c = 0;
            run.v = sha_zero();
        }
    }
    __syncthreads();
    for (int64_t t = b; t < b + per && t < nt; t++) {
        const sha_el x = tiles[t];
        tiles[t] = run;  // exclusive
        run = sha_comb(run, x);
    }
}

// carry-in, exactness, conversion, write into the row
__global__ void __launch_bounds__(SHA_TPB) k_sha_out(int64_t* __restrict__ scol, int64_t m, sha_col c, int q,
                                                     const sha_i128* __restrict__ in_v, const int64_t* __restrict__ in_c,
                                                     const sha_el* __restrict__ tiles,
                                                     const uint32_t* __restrict__ first_head, int32_t* __restrict__ flag) {
    const int64_t p = (int64_t)blockIdx.x * SHA_TPB + threadIdx.x;
    if (p >= m) return;
    const int64_t t = p / SHA_TILE;
    sha_i128 v = in_v[p];
    int64_t cnt = in_c[p];
    if ((uint32_t)(p - t * SHA_TILE) < first_head[t]) {
        // before the tile's first segment start: the running value carries in
        v = sha_add(tiles[t].v, v);
        cnt += tiles[t].c;
    }
    int64_t out;
    if (c.kind == SH_AGG_COUNT) {
        out = cnt;
    } else if (!sha_fp(c)) {
        out = (int64_t)v.lo;
    } else {
        // exactly representable: at most 53 significant bits
        const bool neg = (int64_t)v.hi < 0;
        sha_i128 a = v;
        if (neg) {
            a.lo = ~a.lo;
            a.hi = ~a.hi;
            a = sha_add(a, sha_i128{1ull, 0ull});
        }
        double d = 0.0;
        if (a.lo | a.hi) {
            int tz;
            uint64_t mlo = a.lo, mhi = a.hi;
            if (mlo) {
                tz = __builtin_ctzll(mlo);
                mlo = (mlo >> tz) | (tz ? (mhi << (64 - tz)) : 0ull);
                mhi = tz ? (mhi >> tz) : mhi;
            } else {
                tz = 64 + __builtin_ctzll(mhi);
                mlo = mhi >> (tz - 64);
                mhi = 0ull;
            }
            if (mhi || mlo >= (1ull << 53)) {
                atomicOr(flag, 1);
                return;
            }
            d = ldexp((double)mlo, q + tz);
            if (neg) d = -d;
        }
        out = c.kind == SH_AGG_AVG ? __double_as_longlong(d / (double)cnt) : __double_as_longlong(d);
    }
    scol[p] = out;
}

// the aggregate columns into sorted order, one row read for all of them (SoA: column k
// at sc + k * m), and back into the rows once every column is done
__global__ void __launch_bounds__(SHA_TPB) k_sha_gather(const int64_t* __restrict__ vals, int n_out,
                                                        const uint32_t* __restrict__ idx, int64_t m, sha_desc D,
                                                        int64_t* __restrict__ sc) {
    const int64_t p = (int64_t)blockIdx.x * SHA_TPB + threadIdx.x;
    if (p >= m) return;
    const int64_t* row = vals + (int64_t)idx[p] * n_out;
    for (int k = 0; k < D.n_cols; k++) sc[(int64_t)k * m + p] = row[D.c[k].col];
}

__global__ void __launch_bounds__(SHA_TPB) k_sha_scatter(int64_t* __restrict__ vals, int n_out,
                                                         const uint32_t* __restrict__ idx, int64_t m, sha_desc D,
                                                         const int64_t* __restrict__ sc) {
    const int64_t p = (int64_t)blockIdx.x * SHA_TPB + threadIdx.x;
    if (p >= m) return;
    int64_t* row = vals + (int64_t)idx[p] * n_out;
    for (int k = 0; k < D.n_cols; k++) row[D.c[k].col] = sc[(int64_t)k * m + p];
}

// ---------------------------------------------------------------- host
extern "C" int64_t sha_scratch_bytes(int64_t m, int n_cols) {
    const int64_t nt = (m + SHA_TILE - 1) / SHA_TILE;
    const int64_t rt = (m + 4095) / 4096;
    // seg, idx, 2 x 2 sort buffers, 128-bit values, counts, tiles, first heads,
    // sort histogram, scan temporaries, exponent ranges, the sorted column copies
    return m * 4 * 6 + m * 16 + m * 8 + nt * (int64_t)sizeof(sha_el) + nt * 4 + 256 * rt * 4 +
           (int64_t)shd_scan_tmp_words(256 * rt) * 4 + 4096 + (int64_t)(n_cols < 1 ? 1 : n_cols) * m * 8 + 256;
}

static int sha_ok() { return hipGetLastError() == hipSuccess ? 0 : -3; }

extern "C" int sha_running(const uint64_t* d_seq, int64_t* d_vals, int32_t n_out, int64_t m, const int32_t* d_query,
                           int32_t n_query, const int32_t* d_keys, int32_t n_keys, uint64_t seq_base,
                           const sha_desc* D, void* d_scratch, void* stream) {
    if (m <= 0 || D->n_cols == 0) return 0;
    if (m >= ((int64_t)1 << 32) || n_out < 1 || !d_seq || !d_vals || !d_scratch) return -1;
    hipStream_t st = (hipStream_t)stream;
    const int64_t nseg = (int64_t)(n_query < 1 ? 1 : n_query) * (n_keys < 1 ? 1 : n_keys);
    if (nseg > ((int64_t)1 << 32)) return -1;
    const int64_t nt = (m + SHA_TILE - 1) / SHA_TILE;
    const int64_t rt = (m + 4095) / 4096;
    uint8_t* p = (uint8_t*)d_scratch;
    auto take = [&](int64_t bytes) {
        uint8_t* r = p;
        p += (bytes + 255) & ~(int64_t)255;
        return (void*)r;
    };
    uint32_t* seg = (uint32_t*)take(m * 4);
    uint32_t* idx = (uint32_t*)take(m * 4);
    uint32_t* kb0 = (uint32_t*)take(m * 4);
    uint32_t* kb1 = (uint32_t*)take(m * 4);
    uint32_t* vb0 = (uint32_t*)take(m * 4);
    uint32_t* vb1 = (uint32_t*)take(m * 4);
    sha_i128* sv = (sha_i128*)take(m * 16);
    int64_t* sc = (int64_t*)take(m * 8);
    sha_el* tiles = (sha_el*)take(nt * (int64_t)sizeof(sha_el));
    uint32_t* fh = (uint32_t*)take(nt * 4);
    uint32_t* hist = (uint32_t*)take(256 * rt * 4);
    uint32_t* stmp = (uint32_t*)take((int64_t)shd_scan_tmp_words(256 * rt) * 4);
    int32_t* range = (int32_t*)take(4 * 3 * SHA_MAX_COLS + 64);
    int64_t* scol = (int64_t*)take((int64_t)D->n_cols * m * 8);
    int32_t h_range[3 * SHA_MAX_COLS];
    for (int k = 0; k < SHA_MAX_COLS; k++) {
        h_range[3 * k] = 1 << 30;
        h_range[3 * k + 1] = -(1 << 30);
        h_range[3 * k + 2] = 0;
    }
    hipMemcpyAsync(range, h_range, sizeof(h_range), hipMemcpyHostToDevice, st);
    hipMemsetAsync(range + 3 * SHA_MAX_COLS, 0, 4, st);
    const unsigned g = (unsigned)((m + SHA_TPB - 1) / SHA_TPB);
    hipLaunchKernelGGL(k_sha_prep, dim3((unsigned)std::min<int64_t>(g, 2048)), dim3(SHA_TPB), 0, st, d_seq, (const int64_t*)d_vals, n_out, m, d_query,
                       d_keys, n_keys, seq_base, *D, seg, idx, range);
    if (sha_ok()) return -3;
    int bits = 0;
    while (bits < 32 && ((int64_t)1 << bits) < nseg) bits++;
    const uint32_t* sseg = seg;
    const uint32_t* sidx = idx;
    uint32_t* kbuf[2] = {kb0, kb1};
    uint32_t* vbuf[2] = {vb0, vb1};
    if (bits > 0 && shd_sort_pairs(seg, idx, m, bits, kbuf, vbuf, hist, stmp, stream, &sseg, &sidx)) return -3;
    hipLaunchKernelGGL(k_sha_gather, dim3(g), dim3(SHA_TPB), 0, st, (const int64_t*)d_vals, n_out, sidx, m, *D, scol);
    hipMemcpyAsync(h_range, range, sizeof(h_range), hipMemcpyDeviceToHost, st);
    if (hipStreamSynchronize(st) != hipSuccess) return -3;
    for (int k = 0; k < D->n_cols; k++) {
        const sha_col c = D->c[k];
        int q = 0;
        const bool fp = c.kind == SH_AGG_AVG || (c.kind == SH_AGG_SUM && (c.arg_type == SH_T_FLOAT || c.arg_type == SH_T_DOUBLE));
        if (fp) {
            if (h_range[3 * k + 2]) return 1;  // NaN / infinite addend
            const int lo = h_range[3 * k], hi = h_range[3 * k + 1];
            if (lo <= hi) {
                if (hi - lo + 1 > 96) return 1;  // fixed-point range
                q = lo;
            }
        }
        int64_t* colk = scol + (int64_t)k * m;
        hipLaunchKernelGGL(k_sha_tile, dim3((unsigned)nt), dim3(SHA_TPB), 0, st, (const int64_t*)colk, sseg, m, c, q,
                           sv, sc, tiles, fh);
        hipLaunchKernelGGL(k_sha_carry, dim3(1), dim3(SHA_CARRY_TPB), 0, st, tiles, nt);
        hipLaunchKernelGGL(k_sha_out, dim3(g), dim3(SHA_TPB), 0, st, colk, m, c, q, (const sha_i128*)sv,
                           (const int64_t*)sc, (const sha_el*)tiles, (const uint32_t*)fh, range + 3 * SHA_MAX_COLS);
        if (sha_ok()) return -3;
    }
    hipLaunchKernelGGL(k_sha_scatter, dim3(g), dim3(SHA_TPB), 0, st, d_vals, n_out, sidx, m, *D,
                       (const int64_t*)scol);
    if (sha_ok()) return -3;
    int32_t inexact = 0;
    hipMemcpyAsync(&inexact, range + 3 * SHA_MAX_COLS, 4, hipMemcpyDeviceToHost, st);
    if (hipStreamSynchronize(st) != hipSuccess) return -3;
    return inexact ? 1 : 0;
}
