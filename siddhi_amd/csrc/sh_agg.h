// sh_agg.h — running sum / avg / count over an ordered match stream (sh_agg.hip),
// behind the fast engines.
#pragma once
#include <stdint.h>

#define SHA_MAX_COLS 16

// one aggregate output column of the raw rows
struct sha_col {
    int32_t col;       // row position
    int32_t kind;      // SH_AGG_SUM / SH_AGG_AVG / SH_AGG_COUNT
    int32_t arg_type;  // argument type (the raw value the engine wrote there)
    int32_t pad;
};
struct sha_desc {
    int32_t n_cols;
    int32_t pad;
    sha_col c[SHA_MAX_COLS];
};

#ifdef __cplusplus
extern "C" {
#endif
int64_t sha_scratch_bytes(int64_t m, int n_cols);
// d_vals [m x n_out] raw rows in output order (d_seq the trigger sequence numbers,
// d_query the emitting query or NULL): each listed column's argument values
// become the running aggregate per (query, partition key of the trigger event
// = d_keys[seq - seq_base], NULL: one key). 0: done; 1: the double additions
// would round (or NaN / infinite addends): nothing usable was written, run the
// query sequentially; < 0: error.
int sha_running(const uint64_t* d_seq, int64_t* d_vals, int32_t n_out, int64_t m, const int32_t* d_query,
                int32_t n_query, const int32_t* d_keys, int32_t n_keys, uint64_t seq_base, const sha_desc* D,
                void* d_scratch, void* stream);
#ifdef __cplusplus
}
#endif
