// sh_window.hip — the data-parallel "window" engine for two-state patterns
//     every e1=S[f1] -> e2=S[f2(e1, e2)] within W      (configs C1, C2, C5 rules)
//
// For this shape the per-key NFA of StreamPreStateProcessor reduces to: every
// event i of a key with f1(i) opens one partial (the start template is always
// re-armed by `every`, StreamPostStateProcessor.java:77-79); the partial becomes
// pending at the key's next event (updateState, :307-323) and is consumed by the
// first later event j of the key with f2(i, j), unless an event k <= j of the key
// expired it first (|ts_i - ts_k| > W, expireEvents :325-361). With non-decreasing
// timestamps per key the pending list is in creation (= ts) order, so the
// break-early expiry scan removes exactly the over-age partials, and matches at j
// leave in pending (= creation) order. The host checks non-decreasing timestamps
// on the device first (k_ts_check) and falls back to the sequential per-key
// engine (sh_kernels.hip) when they are not.
//
// Every candidate is then independent: one lane per event scans forward in its
// key segment (stable radix segment output) — massively parallel and coalesced.
#include <hip/hip_runtime.h>

#include "../../include/sh_query.h"
#include "sh_device.h"
#include "sh_jit.h"
#include "sh_vm.h"

#include <stdlib.h>
#include <string.h>

#define WTPB 256

static int64_t wceil(int64_t a, int64_t b) { return (a + b - 1) / b; }

__global__ void k_ts_check(const int64_t* __restrict__ ts, const uint32_t* __restrict__ perm,
                           const uint32_t* __restrict__ skeys, int64_t n, uint32_t sentinel, int32_t* __restrict__ flag) {
    for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x + 1; p < n; p += (int64_t)gridDim.x * blockDim.x) {
        const uint32_t k = skeys ? skeys[p] : 0u;
        if (k == sentinel || (skeys && skeys[p - 1] != k)) continue;
        const int64_t a = ts[perm ? perm[p - 1] : p - 1], b = ts[perm ? perm[p] : p];
        if (b < a) atomicExch(flag, 1);
    }
}

// gather a column into key-segment order
template <typename T>
__global__ void k_permute(const T* __restrict__ src, const uint32_t* __restrict__ perm, int64_t n, T* __restrict__ dst) {
    for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < n; p += (int64_t)gridDim.x * blockDim.x)
        dst[p] = src[perm[p]];
}

// build the tile directory of a tile-major segment (pre-zeroed)
__global__ void k_tile_dir(const uint32_t* __restrict__ skeys, int64_t n, int shift, uint32_t K1,
                           uint32_t* __restrict__ ds, uint32_t* __restrict__ de) {
    for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < n; p += (int64_t)gridDim.x * blockDim.x) {
        const uint32_t key = skeys[p];
        const int64_t a = p >> shift;
        const int64_t tb = a << shift;
        const int64_t te = (n < tb + ((int64_t)1 << shift)) ? n : tb + ((int64_t)1 << shift);
        if (p == tb || skeys[p - 1] != key) ds[(size_t)a * K1 + key] = (uint32_t)p;
        if (p == te - 1 || skeys[p + 1] != key) de[(size_t)a * K1 + key] = (uint32_t)(p + 1);
    }
}

// one lane per event: candidate test + forward scan for the consuming event
template <bool FAST>
__global__ void __launch_bounds__(WTPB) k_window(const shp_program* __restrict__ P, const int64_t* __restrict__ sts,
                                                 const uint32_t* __restrict__ skeys, const uint32_t* __restrict__ perm,
                                                 int64_t n, uint32_t sentinel, const shd_cols* __restrict__ C,
                                                 int32_t* __restrict__ match_pos, uint32_t* __restrict__ cnt,
                                                 int fast_ok, int32_t* __restrict__ flag, shd_tiles TL) {
    const int64_t within = P->within_ms;
    const TileDir D = tile_dir(TL);
    for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < n; p += (int64_t)gridDim.x * blockDim.x) {
        const uint32_t key = skeys ? skeys[p] : 0u;
        if (key == sentinel) continue;
        // the reduction to a forward scan needs non-decreasing timestamps per key
        const int64_t pp = key_pred(D, skeys, p, key);
        if (pp >= 0 && sts[p] < sts[pp]) atomicExch(flag, 1);
        uint32_t rows[2];
        rows[0] = (uint32_t)p;
        rows[1] = SHD_NULL_ROW;
        if (FAST) {
            if (!terms_pass2(P, 0, (uint32_t)p, SHD_NULL_ROW, C)) continue;
        } else if (!filter_pass(P, 0, rows, C, fast_ok)) {
            continue;
        }
        const int64_t t0 = sts[p];
        uint32_t a = D.on() ? D.tile(p) : 0u;
        int64_t qend = D.on() ? (int64_t)D.de[D.at(a, key)] : n;
        for (int64_t q = p + 1;; q++) {
            if (q >= qend && !(D.on() && D.next(a, key, q, qend))) break;
            if (skeys && skeys[q] != key) break;
            const int64_t d = sts[q] - t0;
            if ((d < 0 ? -d : d) > within) break;  // expired before event q is matched
            rows[1] = (uint32_t)q;
            const bool pass = FAST ? terms_pass2(P, 1, (uint32_t)p, (uint32_t)q, C) : filter_pass(P, 1, rows, C, fast_ok);
            if (pass) {
                match_pos[p] = (int32_t)q;
                atomicAdd(&cnt[q], 1u);  // key-segment space: neighbouring lanes hit neighbouring words
                break;
            }
        }
    }
}

// per-event match counts back to arrival order (inverse of the segment permutation)
__global__ void k_cnt_scatter(const uint32_t* __restrict__ cnt_s, const uint32_t* __restrict__ perm, int64_t n,
                              uint32_t* __restrict__ cnt) {
    for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < n; q += (int64_t)gridDim.x * blockDim.x)
        cnt[perm[q]] = cnt_s[q];
}

// rank of partial p among the partials consumed by the same event (creation
// order), then the ordered write of the selected attributes
template <bool FAST>
__global__ void __launch_bounds__(WTPB) k_window_place(const shp_program* __restrict__ P, const int64_t* __restrict__ sts,
                                                       const uint32_t* __restrict__ skeys,
                                                       const uint32_t* __restrict__ perm, int64_t n,
                                                       const shd_cols* __restrict__ C,
                                                       const int32_t* __restrict__ match_pos,
                                                       const uint32_t* __restrict__ off, uint64_t seq_base,
                                                       uint64_t* __restrict__ out_seq, int64_t* __restrict__ out_ts,
                                                       int64_t* __restrict__ out_vals, uint8_t* __restrict__ out_nulls,
                                                       int fast_ok, shd_tiles TL) {
    const int64_t within = P->within_ms;
    const int n_out = P->n_out;
    const TileDir D = tile_dir(TL);
    for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < n; p += (int64_t)gridDim.x * blockDim.x) {
        const int32_t q = match_pos[p];
        if (q < 0) continue;
        const uint32_t key = skeys ? skeys[p] : 0u;
        const int64_t tq = sts[q];
        uint32_t rank = 0;
        uint32_t a = D.on() ? D.tile(p) : 0u;
        int64_t rbeg = D.on() ? (int64_t)D.ds[D.at(a, key)] : 0;
        for (int64_t r = p - 1;; r--) {
            if (r < rbeg && !(D.on() && D.prev(a, key, r, rbeg))) break;
            if (skeys && skeys[r] != key) break;
            if (tq - sts[r] > within) break;  // older partials expired before q
            if (match_pos[r] == q) rank++;
        }
        const uint32_t j = perm ? perm[q] : (uint32_t)q;
        const int64_t dst = (int64_t)off[j] + rank;
        if (out_seq) out_seq[dst] = seq_base + j;
        if (out_ts) out_ts[dst] = tq;
        if (FAST) {
            for (int o = 0; o < n_out; o++) {
                const int sl = P->out_slot[o], at = P->out_attr[o];
                const int s = P->state_stream[sl];
                if (out_vals) out_vals[dst * n_out + o] = load_attr(C, s, at, P->attr_type[s][at], sl ? (uint32_t)q : (uint32_t)p);
                if (out_nulls) out_nulls[dst * n_out + o] = 0;
            }
        } else {
            uint32_t rows[2] = {(uint32_t)p, (uint32_t)q};
            for (int o = 0; o < n_out; o++) {
                VmVal v = vm_eval(P, P->out_pc[o], P->out_len[o], rows, C);
                if (out_vals) out_vals[dst * n_out + o] = v.b;
                if (out_nulls) out_nulls[dst * n_out + o] = v.null;
            }
        }
    }
}

static unsigned grid_for(int64_t n) {
    int64_t g = wceil(n, WTPB);
    if (g > 65536 * 4) g = 65536 * 4;
    return (unsigned)(g < 1 ? 1 : g);
}

// Runs the window engine on a segmented single-stream batch whose timestamps and
// columns are already in key-segment order (shd_segment_payload). Returns 0, 1 when
// timestamps decrease inside a key (caller falls back), 2 when out_cap is too
// small, <0 on HIP errors.
extern "C" int shd_window(const shp_program* dprog, const shp_program* hprog, const shd_batch* b, int32_t nkeys,
                          const uint32_t* perm, const uint32_t* skeys, const int64_t* sts, const void* const* scols,
                          shd_window_ws* ws, shd_cols* d_sorted_desc, uint32_t* scan_tmp, uint64_t* out_seq,
                          int64_t* out_ts, int64_t* out_vals, uint8_t* out_nulls, int64_t out_cap,
                          int64_t* n_matches, void* stream, void* ev_mid_, const void* jit_, const shd_tiles* tiles) {
    const shj_window* jit = (const shj_window*)jit_;
    hipEvent_t ev_mid = (hipEvent_t)ev_mid_;
    hipStream_t st = (hipStream_t)stream;
    const int64_t n = b->n;
    const uint32_t sentinel = skeys ? (uint32_t)nkeys : 0xFFFFFFFFu;
    const unsigned g = grid_for(n);
    shd_cols sc;
    memset(&sc, 0, sizeof(sc));
    for (int a = 0; a < hprog->stream_nattr[0]; a++) sc.col[0][a] = scols[a];
    hipMemcpyAsync(d_sorted_desc, &sc, sizeof(sc), hipMemcpyHostToDevice, st);
    hipMemsetAsync(ws->flag, 0, 4, st);
    uint32_t* cnt_s = perm ? ws->cnt_s : ws->cnt;
    const bool fast = hprog->filter_fast[0] && hprog->filter_fast[1] && hprog->out_fast;
    shd_tiles TL;
    memset(&TL, 0, sizeof(TL));
    if (tiles && skeys) TL = *tiles;
    uint32_t tiles_per_xcd = 0, ntiles = 0;
    const unsigned jg = shj_tiles(n, &tiles_per_xcd, &ntiles);
    if (jit && jit->count && jit->emit && skeys && !getenv("SH_NO_EXT")) {
        // consumer-side walk (sh_jit.cpp ExtForm): per-consumer counts straight
        // into arrival order, exclusive scan, then the ordered write
        const shd_cols* dc = d_sorted_desc;
        void* args[] = {(void*)&sts, (void*)&skeys, (void*)&perm, (void*)&n, (void*)&sentinel, (void*)&dc,
                        (void*)&ws->cnt, (void*)&ws->flag, (void*)&tiles_per_xcd, (void*)&ntiles, (void*)&TL};
        if (hipModuleLaunchKernel((hipFunction_t)jit->count, jg, 1, 1, shj_tile_size(), 1, 1, 0, st, args, nullptr) !=
            hipSuccess)
            return -3;
        if (ev_mid) hipEventRecord(ev_mid, st);
        int rc = shd_exclusive_scan(ws->cnt, ws->off, n, scan_tmp, stream);
        if (rc) return rc;
        uint32_t lo = 0, lc = 0;
        int32_t hflag = 0;
        hipMemcpyAsync(&lo, ws->off + (n - 1), 4, hipMemcpyDeviceToHost, st);
        hipMemcpyAsync(&lc, ws->cnt + (n - 1), 4, hipMemcpyDeviceToHost, st);
        hipMemcpyAsync(&hflag, ws->flag, 4, hipMemcpyDeviceToHost, st);
        if (hipStreamSynchronize(st) != hipSuccess) return -3;
        if (hflag) return 1;
        *n_matches = (int64_t)lo + lc;
        if (*n_matches > out_cap) return 2;
        const uint32_t* cnt = ws->cnt;
        const uint32_t* off = ws->off;
        uint64_t seq_base = b->seq_base;
        void* eargs[] = {(void*)&sts,     (void*)&skeys,    (void*)&perm,     (void*)&n,       (void*)&sentinel,
                         (void*)&dc,      (void*)&cnt,      (void*)&off,      (void*)&seq_base, (void*)&out_seq,
                         (void*)&out_ts,  (void*)&out_vals, (void*)&out_nulls, (void*)&tiles_per_xcd,
                         (void*)&ntiles,  (void*)&TL};
        if (*n_matches > 0 &&
            hipModuleLaunchKernel((hipFunction_t)jit->emit, jg, 1, 1, shj_tile_size(), 1, 1, 0, st, eargs, nullptr) !=
                hipSuccess)
            return -3;
        return hipGetLastError() == hipSuccess ? 0 : -3;
    }
    hipMemsetAsync(ws->match_pos, 0xFF, n * 4, st);
    hipMemsetAsync(cnt_s, 0, n * 4, st);
    if (jit) {
        const shd_cols* dc = d_sorted_desc;
        void* args[] = {(void*)&sts,   (void*)&skeys, (void*)&n,     (void*)&sentinel,      (void*)&dc,
                        (void*)&ws->match_pos, (void*)&cnt_s, (void*)&ws->flag, (void*)&tiles_per_xcd,
                        (void*)&ntiles, (void*)&TL};
        if (hipModuleLaunchKernel((hipFunction_t)jit->match, jg, 1, 1, shj_tile_size(), 1, 1, 0, st, args, nullptr) !=
            hipSuccess)
            return -3;
    } else if (fast)
        hipLaunchKernelGGL(k_window<true>, dim3(g), dim3(WTPB), 0, st, dprog, sts, skeys, perm, n, sentinel,
                           (const shd_cols*)d_sorted_desc, ws->match_pos, cnt_s, 1, ws->flag, TL);
    else
        hipLaunchKernelGGL(k_window<false>, dim3(g), dim3(WTPB), 0, st, dprog, sts, skeys, perm, n, sentinel,
                           (const shd_cols*)d_sorted_desc, ws->match_pos, cnt_s, 1, ws->flag, TL);
    if (ev_mid) hipEventRecord(ev_mid, st);
    if (perm) hipLaunchKernelGGL(k_cnt_scatter, dim3(g), dim3(WTPB), 0, st, (const uint32_t*)cnt_s, perm, n, ws->cnt);
    int rc = shd_exclusive_scan(ws->cnt, ws->off, n, scan_tmp, stream);
    if (rc) return rc;
    uint32_t lo = 0, lc = 0;
    int32_t hflag = 0;
    hipMemcpyAsync(&lo, ws->off + (n - 1), 4, hipMemcpyDeviceToHost, st);
    hipMemcpyAsync(&lc, ws->cnt + (n - 1), 4, hipMemcpyDeviceToHost, st);
    hipMemcpyAsync(&hflag, ws->flag, 4, hipMemcpyDeviceToHost, st);
    if (hipStreamSynchronize(st) != hipSuccess) return -3;
    if (hflag) return 1;  // timestamps decrease inside a key: caller falls back
    *n_matches = (int64_t)lo + lc;
    if (*n_matches > out_cap) return 2;
    if (jit) {
        const shd_cols* dc = d_sorted_desc;
        const int32_t* mp = ws->match_pos;
        const uint32_t* off = ws->off;
        uint64_t seq_base = b->seq_base;
        void* args[] = {(void*)&sts,     (void*)&skeys,    (void*)&perm,    (void*)&n,         (void*)&dc,
                        (void*)&mp,      (void*)&off,      (void*)&seq_base, (void*)&out_seq,  (void*)&out_ts,
                        (void*)&out_vals, (void*)&out_nulls, (void*)&tiles_per_xcd, (void*)&ntiles, (void*)&TL};
        if (hipModuleLaunchKernel((hipFunction_t)jit->place, jg, 1, 1, shj_tile_size(), 1, 1, 0, st, args, nullptr) !=
            hipSuccess)
            return -3;
    } else if (fast)
        hipLaunchKernelGGL(k_window_place<true>, dim3(g), dim3(WTPB), 0, st, dprog, sts, skeys, perm, n,
                           (const shd_cols*)d_sorted_desc, (const int32_t*)ws->match_pos, (const uint32_t*)ws->off,
                           b->seq_base, out_seq, out_ts, out_vals, out_nulls, 1, TL);
    else
        hipLaunchKernelGGL(k_window_place<false>, dim3(g), dim3(WTPB), 0, st, dprog, sts, skeys, perm, n,
                           (const shd_cols*)d_sorted_desc, (const int32_t*)ws->match_pos, (const uint32_t*)ws->off,
                           b->seq_base, out_seq, out_ts, out_vals, out_nulls, 1, TL);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

// directory of a tile-major segment (shd_tiles): ds / de hold ntile * K1 words
extern "C" int shd_tile_dir(const uint32_t* skeys, int64_t n, int shift, uint32_t K1, uint32_t ntile, uint32_t* ds,
                            uint32_t* de, void* stream) {
    hipStream_t st = (hipStream_t)stream;
    hipMemsetAsync(ds, 0, (size_t)ntile * K1 * 4, st);
    hipMemsetAsync(de, 0, (size_t)ntile * K1 * 4, st);
    hipLaunchKernelGGL(k_tile_dir, dim3(grid_for(n)), dim3(WTPB), 0, st, skeys, n, shift, K1, ds, de);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}
