// sh_wave.h — wave64 / workgroup scan primitives for gfx950 (CDNA4).
//
// Wave scans use DPP row shifts (row_shr:1,2,4,8 inside each 16-lane row) and the
// GFX9 row broadcasts (row_bcast:15 into rows 1 and 3, row_bcast:31 into rows 2
// and 3): six VALU ops with DPP source modifiers, no LDS and no ds_bpermute.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// DPP controls (GFX9 encoding)
#define SHW_ROW_SHR(n) (0x110 + (n))
#define SHW_ROW_BCAST15 0x142
#define SHW_ROW_BCAST31 0x143

template <int CTRL>
__device__ __forceinline__ uint32_t shw_move(uint32_t v) {
    // lanes without a source keep `old` = 0 (bound_ctrl off, full row / bank masks)
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xF, 0xF, false);
}

// inclusive prefix sum over the 64 lanes of a wave
__device__ __forceinline__ uint32_t shw_incl_scan(uint32_t v) {
    const int lane = threadIdx.x & 63;
    const int rl = lane & 15;
    uint32_t t;
    t = shw_move<SHW_ROW_SHR(1)>(v);
    if (rl >= 1) v += t;
    t = shw_move<SHW_ROW_SHR(2)>(v);
    if (rl >= 2) v += t;
    t = shw_move<SHW_ROW_SHR(4)>(v);
    if (rl >= 4) v += t;
    t = shw_move<SHW_ROW_SHR(8)>(v);
    if (rl >= 8) v += t;
    t = shw_move<SHW_ROW_BCAST15>(v);
    if ((lane & 31) >= 16) v += t;
    t = shw_move<SHW_ROW_BCAST31>(v);
    if (lane >= 32) v += t;
    return v;
}

template <int CTRL>
__device__ __forceinline__ uint64_t shw_move64(uint64_t v) {
    const uint32_t lo = shw_move<CTRL>((uint32_t)v), hi = shw_move<CTRL>((uint32_t)(v >> 32));
    return ((uint64_t)hi << 32) | lo;
}

// inclusive prefix sum of 64-bit values (two's complement: wraps like Java's long)
__device__ __forceinline__ uint64_t shw_incl_scan64(uint64_t v) {
    const int lane = threadIdx.x & 63;
    const int rl = lane & 15;
    uint64_t t;
    t = shw_move64<SHW_ROW_SHR(1)>(v);
    if (rl >= 1) v += t;
    t = shw_move64<SHW_ROW_SHR(2)>(v);
    if (rl >= 2) v += t;
    t = shw_move64<SHW_ROW_SHR(4)>(v);
    if (rl >= 4) v += t;
    t = shw_move64<SHW_ROW_SHR(8)>(v);
    if (rl >= 8) v += t;
    t = shw_move64<SHW_ROW_BCAST15>(v);
    if ((lane & 31) >= 16) v += t;
    t = shw_move64<SHW_ROW_BCAST31>(v);
    if (lane >= 32) v += t;
    return v;
}

// value of lane 63 (the wave total after an inclusive scan)
__device__ __forceinline__ uint32_t shw_last(uint32_t v) { return (uint32_t)__builtin_amdgcn_readlane((int)v, 63); }

// Workgroup exclusive scan of one value per thread (NT threads, NT/64 waves);
// `ws` is NT/64 words of LDS. Returns the exclusive prefix; *total = sum.
template <int NT>
__device__ __forceinline__ uint32_t shw_block_excl(uint32_t v, uint32_t* ws, uint32_t* total) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint32_t inc = shw_incl_scan(v);
    if (lane == 63) ws[w] = inc;
    __syncthreads();
    uint32_t off = 0, tot = 0;
#pragma unroll
    for (int i = 0; i < NT / 64; i++) {
        const uint32_t s = ws[i];
        off += (i < w) ? s : 0u;
        tot += s;
    }
    __syncthreads();
    *total = tot;
    return off + inc - v;
}

// Workgroup exclusive scan of an LDS array a[0..n) in place (n <= NT * PER);
// thread t owns the contiguous run a[t*PER .. t*PER+PER). Returns the total.
template <int NT, int PER>
__device__ __forceinline__ uint32_t shw_lds_excl_scan(uint32_t* a, int n, uint32_t* ws) {
    const int b = threadIdx.x * PER;
    uint32_t v[PER];
    uint32_t s = 0;
#pragma unroll
    for (int i = 0; i < PER; i++) {
        v[i] = (b + i < n) ? a[b + i] : 0u;
        s += v[i];
    }
    uint32_t tot;
    uint32_t off = shw_block_excl<NT>(s, ws, &tot);
#pragma unroll
    for (int i = 0; i < PER; i++) {
        if (b + i < n) a[b + i] = off;
        off += v[i];
    }
    __syncthreads();
    return tot;
}

// Stable multisplit rank for 8-bit digits, one element per thread per round:
// returns (running count of digit d before this round) + (same-digit elements
// of earlier waves in this round) + (same-digit lanes below in this wave), i.e.
// the element's rank among all valid same-digit elements in round order.
// LDS: wcnt[NT/64][256], run[256] (run zeroed by the caller before round 0).
// Peers come from 8 ballots (one per digit bit). NT >= 256.
template <int NT>
__device__ __forceinline__ uint32_t shw_rank8(uint32_t d, bool valid, uint32_t (*wcnt)[256], uint32_t* run) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int i = threadIdx.x; i < (NT / 64) * 256; i += NT) (&wcnt[0][0])[i] = 0u;
    __syncthreads();
    uint64_t peers = __ballot(valid);
#pragma unroll
    for (int b = 0; b < 8; b++) {
        const bool bit = (d >> b) & 1u;
        const uint64_t m = __ballot(valid && bit);
        peers &= bit ? m : ~m;
    }
    const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
    const uint32_t r = (uint32_t)__popcll(peers & lt);
    if (valid && r == 0) wcnt[w][d] = (uint32_t)__popcll(peers);
    __syncthreads();
    if (threadIdx.x < 256) {
        uint32_t acc = run[threadIdx.x];
#pragma unroll
        for (int q = 0; q < NT / 64; q++) {
            const uint32_t c = wcnt[q][threadIdx.x];
            wcnt[q][threadIdx.x] = acc;
            acc += c;
        }
        run[threadIdx.x] = acc;
    }
    __syncthreads();
    const uint32_t res = valid ? wcnt[w][d] + r : 0u;
    __syncthreads();
    return res;
}
