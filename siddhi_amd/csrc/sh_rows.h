// sh_rows.h — one output row in the caller's layout (device side) for the
// bucketed emitter (sh_bucket.hip): raw 8-byte rows + sequence numbers, typed
// natural-width columns, or packed rows.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/sh_query.h"
#include "sh_device.h"

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

// natural width of a select value's column (bk_raw's reads)
__device__ __forceinline__ int bk_width(int type) {
    return (type == SH_T_LONG || type == SH_T_DOUBLE) ? 8 : (type == SH_T_BOOL ? 1 : 4);
}

// one typed output column element (sh_device_run.d_out_cols): natural width
__device__ __forceinline__ void bk_put(void* col, int w, int64_t row, int64_t v) {
    if (w == 8) ((int64_t*)col)[row] = v;
    else if (w == 4) ((uint32_t*)col)[row] = (uint32_t)v;
    else ((uint8_t*)col)[row] = (uint8_t)v;
}

// a packed row (SHB_OUT_PACKED): the trigger sequence number in words 0-1, then
// each select value at its natural width in OC.woff[o] (8-byte values at even
// words), OC.rw words per row (a multiple of 4: whole 16-byte stores). Value o
// sits in words [2 + o, 2 + 2o] (every earlier value one word .. two), so only
// those candidates are tested: the offsets are kernel arguments (scalar), the
// row stays in registers.
template <int NO>
__device__ __forceinline__ void bk_pack(const shb_cols& OC, int64_t row, const int64_t* v, uint64_t seq) {
    constexpr int RW = ((2 + 2 * NO) + 3) & ~3;
    uint4* dst = (uint4*)((uint32_t*)OC.rows + row * OC.rw);
    // one 16-byte store at a time: only its four words live (registers for more rows in flight)
#pragma unroll
    for (int q = 0; q < RW / 4; q++) {
        if (4 * q >= OC.rw) break;
        uint32_t wv[4] = {0u, 0u, 0u, 0u};
        if (q == 0) {
            wv[0] = (uint32_t)seq;
            wv[1] = (uint32_t)(seq >> 32);
        }
#pragma unroll
        for (int o = 0; o < NO; o++) {
            const int wo = OC.woff[o];
            const bool wide = OC.colw[o] == 8;
            const uint32_t lo = OC.colw[o] == 1 ? (uint32_t)(uint8_t)v[o] : (uint32_t)v[o];
            const uint32_t hi = (uint32_t)((uint64_t)v[o] >> 32);
#pragma unroll
            for (int k = 2 + o; k <= 2 + 2 * o && k < RW; k++)
                if (k >= 4 * q && k < 4 * q + 4 && k == wo) wv[k - 4 * q] = lo;
#pragma unroll
            for (int k = 3 + o; k <= 3 + 2 * o && k < RW; k++)
                if (k >= 4 * q && k < 4 * q + 4 && wide && k == wo + 1) wv[k - 4 * q] = hi;
        }
        dst[q] = make_uint4(wv[0], wv[1], wv[2], wv[3]);
    }
}

// one row in the caller's layout (MODE: SHB_OUT_RAW 8-byte words + out_seq,
// SHB_OUT_COLS natural-width columns + out_seq, SHB_OUT_PACKED rows)
template <int MODE, int NO>
__device__ __forceinline__ void bk_store(const shb_cols& OC, int64_t row, const int64_t* v, uint64_t seq,
                                         uint64_t* __restrict__ out_seq, int64_t* __restrict__ out_vals) {
    if (MODE == SHB_OUT_PACKED) {
        bk_pack<NO>(OC, row, v, seq);
        return;
    }
    if (out_seq) out_seq[row] = seq;
    if (MODE == SHB_OUT_COLS) {
#pragma unroll
        for (int o = 0; o < NO; o++) bk_put(OC.cols[o], OC.colw[o], row, v[o]);
    } else if (out_vals) {
        if (NO % 2 == 0) {
            // a row of NO words as 16-byte stores: consecutive lanes fill whole lines
            longlong2* dst = (longlong2*)(out_vals + row * NO);
#pragma unroll
            for (int o = 0; o < NO; o += 2) dst[o / 2] = make_longlong2(v[o], v[o + 1]);
        } else {
#pragma unroll
            for (int o = 0; o < NO; o++) out_vals[row * NO + o] = v[o];
        }
    }
}
