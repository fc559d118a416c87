// sh_shard.hip — routing and merging kernels of the key-sharded multi-GPU path
// (include/siddhi_shard.h). HBM-bound integer work, one pass each:
//
//   k_shs_hist    per 16,384-event tile: events per owner rank (LDS histogram)
//   k_shs_pos     per tile: stable position of every event in the owner-major
//                 send buffer (ballot multisplit rank, sh_wave.h)
//   k_shs_pack    event columns + global sequence -> packed records at their
//                 send position (one 32-byte record per C2 event)
//   k_shs_unpack  received records -> columns (coalesced both ways)
//   k_shs_bounds / k_shs_globalize   return route of the owner's match rows
//   k_shs_merge   k-way merge by trigger sequence: each row's output position is
//                 its run index + lower_bound in every other run
#include <hip/hip_runtime.h>
#include <string.h>

#include "../../include/siddhi_hip.h"
#include "../../include/siddhi_shard.h"
#include "sh_device.h"
#include "sh_wave.h"

#define SHS_TPB 1024
#define SHS_TILE_SHIFT 14
#define SHS_TILE (1 << SHS_TILE_SHIFT)
#define SHS_ITEMS (SHS_TILE / SHS_TPB)

__host__ __device__ __forceinline__ uint32_t shs_mix32(uint32_t x) {
    x = (x ^ (x >> 16)) * 0x85EBCA6Bu;
    x = (x ^ (x >> 13)) * 0xC2B2AE35u;
    return x ^ (x >> 16);
}

struct shs_cols {
    const void* src[SHS_MAX_COLS];
    void* dst[SHS_MAX_COLS];
    int64_t base[SHS_MAX_COLS];  // SHS_W_OFF columns: the offsets' base
    int32_t width[SHS_MAX_COLS];
    int32_t n;
    int32_t stride;   // record words
    int32_t compact;  // 1: the sequence number is a 32-bit index into the source slice
    int32_t pad;
};

struct shs_offs {
    int64_t off[SHS_MAX_WORLD + 1];
};

__global__ void __launch_bounds__(SHS_TPB) k_shs_hist(const int32_t* __restrict__ keys, int64_t n, int32_t world,
                                                      int32_t nt, uint32_t* __restrict__ cnt) {
    __shared__ uint32_t h[SHS_MAX_WORLD];
    if (threadIdx.x < SHS_MAX_WORLD) h[threadIdx.x] = 0u;
    __syncthreads();
    const int64_t b0 = (int64_t)blockIdx.x << SHS_TILE_SHIFT;
#pragma unroll 4
    for (int j = 0; j < SHS_ITEMS; j++) {
        const int64_t i = b0 + j * SHS_TPB + threadIdx.x;
        if (i < n) atomicAdd(&h[shs_mix32((uint32_t)keys[i]) % (uint32_t)world], 1u);
    }
    __syncthreads();
    if ((int)threadIdx.x < world) cnt[(int64_t)threadIdx.x * nt + blockIdx.x] = h[threadIdx.x];
    if (blockIdx.x == 0 && threadIdx.x == 0) cnt[(int64_t)world * nt] = 0u;
}

__global__ void __launch_bounds__(SHS_TPB) k_shs_pos(const int32_t* __restrict__ keys, int64_t n, int32_t world,
                                                     int32_t nt, const uint32_t* __restrict__ base,
                                                     uint32_t* __restrict__ pos) {
    __shared__ uint32_t wcnt[SHS_TPB / 64][256];
    __shared__ uint32_t run[256];
    if (threadIdx.x < 256) run[threadIdx.x] = 0u;
    __syncthreads();
    const int64_t b0 = (int64_t)blockIdx.x << SHS_TILE_SHIFT;
    for (int j = 0; j < SHS_ITEMS; j++) {
        const int64_t i = b0 + j * SHS_TPB + threadIdx.x;
        const bool valid = i < n;
        const uint32_t d = valid ? shs_mix32((uint32_t)keys[i]) % (uint32_t)world : 0u;
        const uint32_t r = shw_rank8<SHS_TPB>(d, valid, wcnt, run);
        if (valid) pos[i] = base[(int64_t)d * nt + blockIdx.x] + r;
    }
}

__global__ void k_shs_counts(const uint32_t* __restrict__ base, int32_t world, int32_t nt, uint32_t* __restrict__ out) {
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r <= world) out[r] = base[(int64_t)r * nt];
}

__global__ void k_shs_pack(const uint32_t* __restrict__ pos, int64_t n, shs_cols C, uint64_t seq0,
                           uint32_t* __restrict__ rec) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t* r = rec + (int64_t)pos[i] * C.stride;
    int w = 0;
#pragma unroll
    for (int c = 0; c < SHS_MAX_COLS; c++) {
        if (c >= C.n) break;
        const int wd = C.width[c];
        if (wd == 8) {
            const uint64_t v = ((const uint64_t*)C.src[c])[i];
            r[w] = (uint32_t)v;
            r[w + 1] = (uint32_t)(v >> 32);
            w += 2;
        } else if (wd == SHS_W_OFF) {
            r[w++] = (uint32_t)(((const uint64_t*)C.src[c])[i] - (uint64_t)C.base[c]);
        } else if (wd == 4) {
            r[w++] = ((const uint32_t*)C.src[c])[i];
        } else {
            r[w++] = ((const uint8_t*)C.src[c])[i];
        }
    }
    if (C.compact) {
        r[w] = (uint32_t)i;
        return;
    }
    const uint64_t s = seq0 + (uint64_t)i;
    r[w] = (uint32_t)s;
    r[w + 1] = (uint32_t)(s >> 32);
}

__global__ void k_shs_unpack(const uint32_t* __restrict__ rec, int64_t n, shs_cols C, uint64_t seq0,
                             uint64_t* __restrict__ seq) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t* r = rec + i * C.stride;
    int w = 0;
#pragma unroll
    for (int c = 0; c < SHS_MAX_COLS; c++) {
        if (c >= C.n) break;
        const int wd = C.width[c];
        if (wd == 8) {
            ((uint64_t*)C.dst[c])[i] = (uint64_t)r[w] | ((uint64_t)r[w + 1] << 32);
            w += 2;
        } else if (wd == SHS_W_OFF) {
            ((uint64_t*)C.dst[c])[i] = (uint64_t)C.base[c] + (uint64_t)r[w++];
        } else if (wd == 4) {
            ((uint32_t*)C.dst[c])[i] = r[w++];
        } else {
            ((uint8_t*)C.dst[c])[i] = (uint8_t)r[w++];
        }
    }
    if (seq) seq[i] = C.compact ? seq0 + (uint64_t)r[w] : ((uint64_t)r[w] | ((uint64_t)r[w + 1] << 32));
}

// first index j in [0, m) with a[j] >= v (a ascending)
__device__ __forceinline__ int64_t shs_lower_bound(const uint64_t* a, int64_t lo, int64_t hi, uint64_t v) {
    while (lo < hi) {
        const int64_t mid = lo + ((hi - lo) >> 1);
        if (a[mid] < v)
            lo = mid + 1;
        else
            hi = mid;
    }
    return lo;
}

__global__ void k_shs_bounds(const uint64_t* __restrict__ oseq, int64_t m, uint64_t seq_base, shs_offs S,
                             int32_t world, int64_t* __restrict__ out) {
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r <= world) out[r] = shs_lower_bound(oseq, 0, m, seq_base + (uint64_t)S.off[r]);
}

__global__ void k_shs_globalize(uint64_t* __restrict__ oseq, int64_t m, uint64_t seq_base,
                                const uint64_t* __restrict__ gseq) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j < m) oseq[j] = gseq[oseq[j] - seq_base];
}

__global__ void k_shs_merge(const uint64_t* __restrict__ seq, const int64_t* __restrict__ vals, int32_t n_out,
                            shs_offs R, int32_t n_runs, uint64_t* __restrict__ seq_out,
                            int64_t* __restrict__ vals_out) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= R.off[n_runs]) return;
    int r = 0;
    while (r + 1 < n_runs && R.off[r + 1] <= j) r++;
    const uint64_t s = seq[j];
    int64_t p = j - R.off[r];
    for (int q = 0; q < n_runs; q++)
        if (q != r) p += shs_lower_bound(seq, R.off[q], R.off[q + 1], s) - R.off[q];
    seq_out[p] = s;
    for (int o = 0; o < n_out; o++) vals_out[p * n_out + o] = vals[j * n_out + o];
}

// ---------------------------------------------------------------- C-ABI
static int shs_ok() { return hipGetLastError() == hipSuccess ? SH_OK : SH_E_HIP; }
static int64_t shs_tiles(int64_t n) { return (n + SHS_TILE - 1) >> SHS_TILE_SHIFT; }
static uint32_t shs_blocks(int64_t n, int t) { return (uint32_t)((n + t - 1) / t); }

extern "C" int32_t shs_owner(int32_t key, int32_t world) {
    return world > 0 ? (int32_t)(shs_mix32((uint32_t)key) % (uint32_t)world) : 0;
}

extern "C" int64_t shs_route_scratch_bytes(int64_t n, int32_t world) {
    const int64_t cells = (int64_t)world * shs_tiles(n) + 1;
    // table + counts + the scan's temporaries
    return (cells + SHS_MAX_WORLD + 8 + shd_scan_tmp_words(cells)) * 4;
}

extern "C" int shs_route(const int32_t* d_keys, int64_t n, int32_t world, uint32_t* d_pos, void* d_scratch,
                         int64_t* h_counts, void* stream) {
    if (n < 0 || world < 1 || world > SHS_MAX_WORLD || !h_counts || (n && (!d_keys || !d_pos || !d_scratch)))
        return SH_E_INVALID_ARG;
    if (n >= ((int64_t)1 << 32)) return SH_E_INVALID_ARG;
    hipStream_t st = (hipStream_t)stream;
    if (n == 0) {
        for (int r = 0; r < world; r++) h_counts[r] = 0;
        return SH_OK;
    }
    const int64_t nt = shs_tiles(n);
    const int64_t cells = (int64_t)world * nt + 1;
    uint32_t* table = (uint32_t*)d_scratch;
    uint32_t* counts = table + cells;
    uint32_t* tmp = counts + SHS_MAX_WORLD + 8;
    hipLaunchKernelGGL(k_shs_hist, dim3((uint32_t)nt), dim3(SHS_TPB), 0, st, d_keys, n, world, (int32_t)nt, table);
    if (shs_ok()) return SH_E_HIP;
    if (shd_exclusive_scan(table, table, cells, tmp, stream)) return SH_E_HIP;
    hipLaunchKernelGGL(k_shs_pos, dim3((uint32_t)nt), dim3(SHS_TPB), 0, st, d_keys, n, world, (int32_t)nt, table,
                       d_pos);
    hipLaunchKernelGGL(k_shs_counts, dim3(1), dim3(SHS_MAX_WORLD + 64), 0, st, table, world, (int32_t)nt, counts);
    if (shs_ok()) return SH_E_HIP;
    uint32_t hc[SHS_MAX_WORLD + 1];
    if (hipMemcpyAsync(hc, counts, (size_t)(world + 1) * 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess)
        return SH_E_HIP;
    for (int r = 0; r < world; r++) h_counts[r] = (int64_t)hc[r + 1] - (int64_t)hc[r];
    return SH_OK;
}

static int shs_fill(shs_cols* C, int32_t n_cols, const int32_t* widths, bool compact = false) {
    if (n_cols < 0 || n_cols > SHS_MAX_COLS || (n_cols && !widths)) return SH_E_INVALID_ARG;
    memset(C, 0, sizeof(*C));
    C->n = n_cols;
    C->compact = compact ? 1 : 0;
    int w = 0;
    for (int c = 0; c < n_cols; c++) {
        if (widths[c] != 1 && widths[c] != 4 && widths[c] != 8 && !(compact && widths[c] == SHS_W_OFF))
            return SH_E_INVALID_ARG;
        C->width[c] = widths[c];
        w += widths[c] == 8 ? 2 : 1;
    }
    C->stride = w + (compact ? 1 : 2);
    return SH_OK;
}

extern "C" int32_t shs_record_words(int32_t n_cols, const int32_t* widths) {
    shs_cols C;
    return shs_fill(&C, n_cols, widths) == SH_OK ? C.stride : -1;
}

extern "C" int shs_pack(const uint32_t* d_pos, int64_t n, int32_t n_cols, const void* const* d_cols,
                        const int32_t* widths, uint64_t seq0, uint32_t* d_rec, void* stream) {
    shs_cols C;
    if (shs_fill(&C, n_cols, widths) || n < 0 || (n && (!d_pos || !d_rec))) return SH_E_INVALID_ARG;
    for (int c = 0; c < n_cols; c++) {
        if (!d_cols[c]) return SH_E_INVALID_ARG;
        C.src[c] = d_cols[c];
    }
    if (n == 0) return SH_OK;
    hipLaunchKernelGGL(k_shs_pack, dim3(shs_blocks(n, 256)), dim3(256), 0, (hipStream_t)stream, d_pos, n, C, seq0,
                       d_rec);
    return shs_ok();
}

extern "C" int shs_unpack(const uint32_t* d_rec, int64_t n, int32_t n_cols, void* const* d_cols,
                          const int32_t* widths, uint64_t* d_seq, void* stream) {
    shs_cols C;
    if (shs_fill(&C, n_cols, widths) || n < 0 || (n && !d_rec)) return SH_E_INVALID_ARG;
    for (int c = 0; c < n_cols; c++) {
        if (!d_cols[c]) return SH_E_INVALID_ARG;
        C.dst[c] = d_cols[c];
    }
    if (n == 0) return SH_OK;
    hipLaunchKernelGGL(k_shs_unpack, dim3(shs_blocks(n, 256)), dim3(256), 0, (hipStream_t)stream, d_rec, n, C,
                       (uint64_t)0, d_seq);
    return shs_ok();
}

extern "C" int32_t shs_record_words_compact(int32_t n_cols, const int32_t* widths) {
    shs_cols C;
    return shs_fill(&C, n_cols, widths, true) == SH_OK ? C.stride : -1;
}

extern "C" int shs_pack_compact(const uint32_t* d_pos, int64_t n, int32_t n_cols, const void* const* d_cols,
                                const int32_t* widths, const int64_t* h_base, uint32_t* d_rec, void* stream) {
    shs_cols C;
    if (shs_fill(&C, n_cols, widths, true) || n < 0 || n >= ((int64_t)1 << 32) || (n && (!d_pos || !d_rec)))
        return SH_E_INVALID_ARG;
    for (int c = 0; c < n_cols; c++) {
        if (!d_cols[c] || (widths[c] == SHS_W_OFF && !h_base)) return SH_E_INVALID_ARG;
        C.src[c] = d_cols[c];
        C.base[c] = widths[c] == SHS_W_OFF ? h_base[c] : 0;
    }
    if (n == 0) return SH_OK;
    hipLaunchKernelGGL(k_shs_pack, dim3(shs_blocks(n, 256)), dim3(256), 0, (hipStream_t)stream, d_pos, n, C,
                       (uint64_t)0, d_rec);
    return shs_ok();
}

extern "C" int shs_unpack_compact(const uint32_t* d_rec, int32_t n_cols, void* const* d_cols, const int32_t* widths,
                                  const int64_t* h_src_off, int32_t world, const int64_t* h_src_base,
                                  const uint64_t* h_src_seq0, uint64_t* d_seq, void* stream) {
    shs_cols C;
    if (shs_fill(&C, n_cols, widths, true) || world < 1 || world > SHS_MAX_WORLD || !h_src_off || !h_src_seq0)
        return SH_E_INVALID_ARG;
    // one launch per source rank: its records' bases and first sequence number
    for (int r = 0; r < world; r++) {
        const int64_t a = h_src_off[r], m = h_src_off[r + 1] - a;
        if (m < 0) return SH_E_INVALID_ARG;
        if (m == 0) continue;
        for (int c = 0; c < n_cols; c++) {
            if (!d_cols[c] || (widths[c] == SHS_W_OFF && !h_src_base)) return SH_E_INVALID_ARG;
            const int w = widths[c] == SHS_W_OFF ? 8 : widths[c];
            C.dst[c] = (uint8_t*)d_cols[c] + a * w;
            C.base[c] = widths[c] == SHS_W_OFF ? h_src_base[(int64_t)r * n_cols + c] : 0;
        }
        hipLaunchKernelGGL(k_shs_unpack, dim3(shs_blocks(m, 256)), dim3(256), 0, (hipStream_t)stream,
                           d_rec + a * C.stride, m, C, h_src_seq0[r], d_seq ? d_seq + a : nullptr);
        if (shs_ok()) return SH_E_HIP;
    }
    return SH_OK;
}

extern "C" int shs_rows_home(uint64_t* d_oseq, int64_t m, uint64_t seq_base, const uint64_t* d_gseq,
                             const int64_t* h_src_off, int32_t world, int64_t* h_counts, void* stream) {
    if (m < 0 || world < 1 || world > SHS_MAX_WORLD || !h_src_off || !h_counts || (m && (!d_oseq || !d_gseq)))
        return SH_E_INVALID_ARG;
    hipStream_t st = (hipStream_t)stream;
    if (m == 0) {
        for (int r = 0; r < world; r++) h_counts[r] = 0;
        return SH_OK;
    }
    shs_offs S;
    for (int r = 0; r <= world; r++) S.off[r] = h_src_off[r];
    int64_t* d_b = nullptr;
    if (hipMallocAsync((void**)&d_b, (size_t)(world + 1) * 8, st) != hipSuccess) return SH_E_OOM;
    hipLaunchKernelGGL(k_shs_bounds, dim3(1), dim3(SHS_MAX_WORLD + 64), 0, st, d_oseq, m, seq_base, S, world, d_b);
    hipLaunchKernelGGL(k_shs_globalize, dim3(shs_blocks(m, 256)), dim3(256), 0, st, d_oseq, m, seq_base, d_gseq);
    int64_t hb[SHS_MAX_WORLD + 1];
    const bool ok = shs_ok() == SH_OK &&
                    hipMemcpyAsync(hb, d_b, (size_t)(world + 1) * 8, hipMemcpyDeviceToHost, st) == hipSuccess;
    hipFreeAsync(d_b, st);
    if (!ok || hipStreamSynchronize(st) != hipSuccess) return SH_E_HIP;
    for (int r = 0; r < world; r++) h_counts[r] = hb[r + 1] - hb[r];
    return SH_OK;
}

extern "C" int shs_merge(const uint64_t* d_seq, const int64_t* d_vals, int32_t n_out, const int64_t* h_off,
                         int32_t n_runs, uint64_t* d_seq_out, int64_t* d_vals_out, void* stream) {
    if (n_runs < 1 || n_runs > SHS_MAX_WORLD || !h_off || n_out < 0) return SH_E_INVALID_ARG;
    shs_offs R;
    for (int r = 0; r <= n_runs; r++) R.off[r] = h_off[r];
    const int64_t m = R.off[n_runs];
    if (m <= 0) return SH_OK;
    if (!d_seq || !d_seq_out || (n_out && (!d_vals || !d_vals_out))) return SH_E_INVALID_ARG;
    hipLaunchKernelGGL(k_shs_merge, dim3(shs_blocks(m, 256)), dim3(256), 0, (hipStream_t)stream, d_seq, d_vals, n_out,
                       R, n_runs, d_seq_out, d_vals_out);
    return shs_ok();
}
