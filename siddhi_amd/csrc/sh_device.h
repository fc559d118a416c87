// sh_device.h — host<->kernel structures and launch entry points of the
// gfx950 matcher (implemented in sh_kernels.hip, called from sh_host.cpp).
#pragma once
#include <stddef.h>
#include <stdint.h>

#include "sh_program.h"

#define SHD_NULL_ROW 0xFFFFFFFFu

// Column stores of every stream (device pointers). Lives in device memory;
// kernels take a pointer to it.
struct shd_cols {
    const void* col[SHP_MAX_STREAMS][32];
    const uint8_t* nul[SHP_MAX_STREAMS][32];
};

// One device batch of events in arrival order.
struct shd_batch {
    const int64_t* ts;       // [n]
    const uint8_t* stream;   // [n] or NULL (single stream 0)
    const uint32_t* row;     // [n] row in the stream's column store, or NULL (row = row_base + i)
    const int32_t* keys;     // [n] partition key (dense), -1 = null key; NULL -> key 0
    uint32_t row_base;
    int32_t pad;
    uint64_t seq_base;       // global sequence number of event 0
    int64_t n;
};

// Emission buffers.
struct shd_emit {
    uint64_t* tmp;           // temp records: [cap][3 + n_out] words
    unsigned long long* tmp_ctr;  // atomic record counter
    int64_t tmp_cap;
    uint32_t* match_cnt;     // [n] matches triggered by local event i (pre-zeroed)
    int32_t* err;            // [0]: state overflow, [1]: temp overflow
};

// scratch for the radix segment
struct shd_segment_ws {
    uint32_t* keys_a;
    uint32_t* keys_b;
    uint32_t* idx_a;
    uint32_t* idx_b;
    uint32_t* hist;          // [256 * nblocks]
    uint32_t* scan_tmp;      // scan block sums (3 levels)
    uint32_t* seg_off;       // [3n + 2]: flags, positions, segment list + count
    int64_t cap;
};

// columns carried through the radix segment (moved with their key)
struct shd_payload {
    int32_t n;
    int32_t pad;
    const void* src[8];      // arrival-order columns
    void* dst[8];            // key-segment-order output
    uint8_t width[8];        // 1, 4 or 8 bytes
};

// arrival-tile directory of a tile-major segment: run of key k in tile a is
// [dstart[a*K1+k], dend[a*K1+k]) (empty when equal)
struct shd_tiles {
    const uint32_t* dstart;
    const uint32_t* dend;
    uint32_t K1;             // keys + 1 (the null-key sentinel bucket)
    uint32_t ntile;
    int32_t shift;           // log2 events per tile
    int32_t pad;
};

// scratch of the window engine (sh_window.hip)
struct shd_window_ws {
    int32_t* match_pos;      // [n] consuming position of the partial opened at p, -1 none
    uint32_t* cnt_s;         // [n] matches per event (key-segment position)
    uint32_t* cnt;           // [n] matches per event (arrival index)
    uint32_t* off;           // [n] exclusive scan of cnt
    int32_t* flag;           // [1] non-monotone timestamps seen
};

// ---- bucketed window engine (sh_bucket.hip + the hipRTC matcher shb_match)
// Partitioned `every e1=S[f1] -> e2=S[f2] within W`: each arrival tile of
// SHB_TILE events is stably reordered by key bucket (bucket = key & (SHB_NB-1))
// in its own region (the tile's bucket order: tile-local, no global pass), the
// matcher gathers one bucket's segments of a run of tiles (plus halo tiles that
// cover the window) into LDS and walks each consumer's key back, and the
// emitter restores arrival order per tile.
#define SHB_NB 256
#define SHB_TILE_SHIFT 13
#define SHB_TILE (1 << SHB_TILE_SHIFT)
#define SHB_CH 4096       // chunk (consumer) events of one matcher pass, at most
#define SHB_SPAN 5120     // chunk + halo events staged in LDS, at most
#define SHB_TOFF 264      // u16 stride of a tile's bucket-start row (257 used)
#define SHB_HMAX 64       // halo tiles before a chunk, at most
#define SHB_CT_MAX 160    // tiles per matcher chunk, at most
#define SHB_MAX_STAGED 4
#define SHB_MAX_MS 4
#define SHB_MAX_OUT 16
// flag bits raised on the device (any bit: rerun on the general window path)
#define SHB_F_TS 1        // timestamp outside the packed range
#define SHB_F_KEY 2       // key id >= n_keys
#define SHB_F_MONO 4      // timestamps decrease inside a key
#define SHB_F_COUNT 8     // one consumer takes > 255 partials
#define SHB_F_HALO 16     // a walk reached the halo start
#define SHB_F_SPAN 32     // one tile's bucket segment exceeds a chunk

struct shb_plan {
    int64_t n;
    int64_t tbase;            // packed ts = ts - tbase in the high (32 - kb) bits of w0
    int32_t nt;               // arrival tiles of SHB_TILE events
    int32_t kb;               // local key bits: w0 low bits = key >> log2(SHB_NB)
    int32_t ct;               // arrival tiles per matcher chunk (<= SHB_CT_MAX)
    int32_t n_chunks;         // matcher grid = SHB_NB * n_chunks
    int32_t n_staged;
    int32_t no_ts;            // 1: w0 = the local key alone (no timestamps: the sequence engine)
    const void* st_src[SHB_MAX_STAGED];  // arrival-order columns moved into bucket order
    void* st_dst[SHB_MAX_STAGED];
    int32_t st_width[SHB_MAX_STAGED];
    int32_t n_ms;             // match-stream columns (e1-side select values)
    void* ms[SHB_MAX_MS];     // [n] each, natural width; regions taken per matcher pass
    int32_t ms_width[SHB_MAX_MS];
    const int64_t* ts;        // arrival-order timestamps (tile first timestamps: the halo)
    const int32_t* keys;      // arrival-order partition keys
    uint32_t* w0;             // tiles' bucket order: packed ts | local key
    uint16_t* sp;             // arrival order: the event's slot in its tile's bucket order
    uint16_t* toff;           // [nt][SHB_TOFF]: bucket starts in the tile's bucket order ([256]: valid events)
    uint16_t* tofft;          // the same transposed, [SHB_NB + 1][tstride]: a bucket's starts over the tiles
    int32_t tstride;          // (contiguous for the matchers, which read one bucket over many tiles)
    int32_t pad_t;
    uint8_t* cnt;             // tiles' bucket order: partials consumed per event
    uint32_t* mstart;         // [nt][SHB_NB]: match-stream position of each (tile, bucket) segment's first match
    uint32_t* ttot;           // [nt + 1]: matches per arrival tile -> exclusive scan
    uint32_t* ms_ctr;         // match-stream region allocator
    int64_t* tpre;            // [nt]: latest timestamp of each tile -> of all tiles before it
    int64_t* tfirst;          // [nt]: timestamp of each tile's first event
    int32_t* hstart;          // [nt]: first halo tile of a matcher pass starting at each tile
    int64_t within;           // the window W (ms): halo tiles
    int32_t* flag;
    unsigned long long* prof; // diagnostics (SH_BK_PROFILE): clock ticks per matcher phase, NULL off
};

// select list of the emitter: value o comes from match-stream column idx[o]
// (kind 0) or from the consumer event's attribute idx[o] (kind 1)
struct shb_out {
    int32_t n_out;
    int32_t pad[3];
    int32_t kind[SHB_MAX_OUT];
    int32_t type[SHB_MAX_OUT];    // sh_type: raw-value conversion
    const void* src[SHB_MAX_OUT]; // kind 0: match-stream column, kind 1: consumer column
};

// the rise-and-fall sequence (nf_query.s3) for the bucket-carry engine: every
// operand of f2 / f3 and every e1 / e2[last] select value is one 4-byte attribute
// (staged column 0) of type `type`; ms_slot[m]: match-stream column m holds e1's
// value (slot 0) or the last e2's (slot 1)
struct shb_s3 {
    int32_t type;                 // SH_T_INT or SH_T_FLOAT
    int32_t op2, dom2, op3, dom3;
    int32_t n_ms;
    int32_t ms_slot[2];
    int32_t warm;                 // 1: each chunk warms L2 with the next chunk's segments
};

// select-clause aggregators carried per key by the bucketed engine (k_bk_aggc):
// output o's running value (8-byte raw: long sum / count, double sum / avg) by
// match-stream position, from addends on the e1 side (match-stream column e1_col)
// or the e2 side (staged column e2_col, at the consumer's slot) or none (count())
#define SHB_MAX_AGG 4
#define SHB_F_AGG 64      // a carry chunk's rows overflow its LDS: the post-pass runs
struct shb_aggc {
    int32_t n;
    int32_t e1_col, e1_type;      // match-stream column of the e1-side argument (-1: none; 4-byte)
    int32_t e2_col[2], e2_type[2];  // staged columns of e2-side arguments (-1: none; [1]: 4-byte)
    int32_t kind[SHB_MAX_AGG];    // SH_AGG_SUM / AVG / COUNT
    int32_t side[SHB_MAX_AGG];    // 0: e1, 1: e2 column 0, 2: e2 column 1, 3: none
    void* out[SHB_MAX_AGG];       // [match-stream positions] int64 / double bits
    int32_t parallel;             // 1: k_bk_aggp (segmented prefix, exact fixed point), 0: k_bk_aggc
};

// typed output columns (sh_device_run.d_out_cols) instead of raw 8-byte rows
#define SHB_OUT_RAW 0      // rows of raw 8-byte words (+ the sequence numbers apart)
#define SHB_OUT_COLS 1     // one natural-width column per select value (+ sequence numbers)
#define SHB_OUT_PACKED 2   // packed rows: sequence number, then the values at natural width
struct shb_cols {
    void* cols[SHB_MAX_OUT];      // natural width per select value
    int32_t colw[SHB_MAX_OUT];    // their widths: 8, 4 or 1 bytes
    int32_t use;                  // SHB_OUT_*
    int32_t rw;                   // packed: 4-byte words per row (a multiple of 4)
    int32_t woff[SHB_MAX_OUT];    // packed: word offset of each value in its row
    void* rows;                   // packed: the rows
};

#ifdef __cplusplus
extern "C" {
#endif
// all launches are asynchronous on `stream` (hipStream_t)
size_t shd_scan_tmp_words(int64_t n);
// stable radix segment by (key, arrival): perm / sorted keys (both NULL for an
// unpartitioned batch) and the segment list in ws->seg_off[2n .. 3n] (+ count at [3n])
int shd_segment(const shd_batch* b, int32_t nkeys, shd_segment_ws* ws, void* stream,
                const uint32_t** perm_out, const uint32_t** skeys_out);
// as shd_segment, also moving `carry` columns into key-segment order; `mid`
// holds one intermediate buffer per carried column (multi-pass ping-pong).
// tile_shift >= 12 sorts each arrival tile of 2^tile_shift events by key in its
// own region ((tile, key, arrival) order); want_segments = 0 skips the segment list
int shd_segment_payload(const shd_batch* b, int32_t nkeys, shd_segment_ws* ws, void* stream,
                        const uint32_t** perm_out, const uint32_t** skeys_out, const shd_payload* carry,
                        void* const* mid, int tile_shift, int want_segments);
int shd_advance(const shp_program* dprog, const shp_layout* lay, uint8_t* kstate, int32_t nkeys,
                const shd_batch* b, const uint32_t* perm, const uint32_t* skeys,
                const uint32_t* seg_off, const shd_cols* dcols, const shd_emit* em, void* stream, int fast_ok);
int shd_emit_place(const shd_emit* em, int32_t n_out, int64_t n_events, uint32_t* offsets,
                   uint32_t* scan_tmp, int64_t n_records, const shd_batch* b, uint64_t* out_seq,
                   int64_t* out_ts, int64_t* out_vals, uint8_t* out_nulls, void* stream);
// window engine for `every e1=S[f1] -> e2=S[f2] within W`: 0 ok, 1 = fall back
// (timestamps decrease inside a key), 2 = output capacity too small, <0 error;
// `jit` (const shj_window*, sh_jit.h) selects the hipRTC-specialised kernels
// when non-NULL, else the ahead-of-time ones
int shd_window(const shp_program* dprog, const shp_program* hprog, const shd_batch* b, int32_t nkeys,
               const uint32_t* perm, const uint32_t* skeys, const int64_t* sts, const void* const* scols,
               shd_window_ws* ws, shd_cols* d_sorted_desc, uint32_t* scan_tmp, uint64_t* out_seq,
               int64_t* out_ts, int64_t* out_vals, uint8_t* out_nulls, int64_t out_cap, int64_t* n_matches,
               void* stream, void* ev_mid, const void* jit, const shd_tiles* tiles);
int shd_tile_dir(const uint32_t* skeys, int64_t n, int shift, uint32_t K1, uint32_t ntile, uint32_t* ds,
                 uint32_t* de, void* stream);
int shd_relayout(const uint8_t* src, const shp_layout* A, uint8_t* dst, const shp_layout* B, int32_t nkeys,
                 int32_t n_states, int32_t n_out, void* stream);
int shd_sort_pairs(const uint32_t* keys, const uint32_t* vals, int64_t n, int bits, uint32_t* const* kbuf,
                   uint32_t* const* vbuf, uint32_t* hist, uint32_t* scan_tmp, void* stream,
                   const uint32_t** keys_out, const uint32_t** vals_out);
int shd_exclusive_scan(const uint32_t* in, uint32_t* out, int64_t n, uint32_t* tmp, void* stream);
// bucketed window engine launch steps (sh_bucket.hip), all async on `stream`
int shb_partition(const int32_t* keys, const int64_t* ts, int32_t nkeys, shb_plan* P, void* stream);
int shb_finish(shb_plan* P, uint32_t* scan_tmp, void* stream);
// the rise-and-fall sequence: one workgroup per key bucket carries its keys' state
// across the tiles (after shb_partition with no_ts; before shb_finish)
int shb_s3_carry(const shb_plan* P, const shb_s3* S, void* stream);
// running aggregates per key: one workgroup per key bucket in arrival order (after
// the matcher, before shb_finish / shb_emit)
int shb_agg_carry(const shb_plan* P, const shb_aggc* A, void* stream);
int shb_emit(const shb_plan* P, const shb_out* O, const shb_cols* OC, uint64_t seq_base, uint64_t* out_seq,
             int64_t* out_vals, int64_t out_cap, void* stream);
// raw 8-byte rows [m x n_out] -> typed columns of widths w[o] (8, 4 or 1 bytes)
int shd_narrow_rows(const int64_t* vals, int32_t n_out, int64_t m, void* const* cols, const int32_t* w, void* stream);
// raw rows + sequence numbers -> packed rows (SHB_OUT_PACKED; woff / rw as in shb_cols)
int shd_pack_rows(const uint64_t* seq, const int64_t* vals, int32_t n_out, int64_t m, const int32_t* w,
                  const int32_t* woff, int32_t rw, void* rows, void* stream);
#ifdef __cplusplus
}
#endif
