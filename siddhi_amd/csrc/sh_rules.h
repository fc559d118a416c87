// sh_rules.h — the batch-compiled rule table (config C5) shared by the host
// lowering (sh_host.cpp compile_rules, sh_host_fast.cpp run_rules) and the gfx950 kernels (sh_rules.hip).
#pragma once
#include <stdint.h>

#include "sh_device.h"
#include "sh_program.h"

// one query `every e1=S[f1] -> e2=S[f2(e1, e2)] within W select <projection>`
struct shr_rule {
    int64_t within;                     // ms (the window shape requires `within`)
    int32_t query;                      // query index in the app (junction subscription order)
    int32_t n_out;
    int32_t nt[2];                      // conjuncts of f1 (slot 0) and of f2 (slots 0, 1)
    shp_term t[2][SHP_MAX_TERMS];
    int8_t out_slot[SHP_MAX_OUT];
    int8_t out_attr[SHP_MAX_OUT];
};

struct shr_table {
    int32_t n_rules;
    int32_t ix_attr;                    // indexed slot-0 attribute, -1: no index
    int32_t n_ix;                       // distinct indexed constants
    int32_t n_free;                     // rules without the indexed conjunct
    int32_t attr_type[32];              // stream attribute types
    const shr_rule* rules;              // device [n_rules]
    const int64_t* ix_val;              // device [n_ix], ascending
    const uint32_t* ix_start;           // device [n_ix + 1]
    const uint32_t* ix_rule;            // device rule ids grouped by constant (ascending inside a group)
    const uint32_t* free_rule;          // device [n_free], ascending
};

// the rule set as one image the scan kernel copies into LDS (built by the host when
// it fits): the predicate index, the rule ids per group and without the indexed
// conjunct, per rule its window and term range, and every term
struct shr_meta {
    int64_t within;
    uint16_t toff0, toff1;              // first term of f1 (global part), of f2 (LDS part)
    uint8_t nt0, nt1;
    uint16_t pad;
};
// the image's first `lds` bytes go to LDS: all of it (one 1024-thread workgroup per CU),
// or with SH_RULES_IMG_SPLIT=1 everything but f1's terms (read once per candidate rule),
// so two workgroups fit a CU -- measured slower on C5 (14.5 vs 14.0 ms): the L2 reads
// of f1's terms cost more than the extra occupancy gained
struct shr_img {
    int32_t bytes;                      // image size (multiple of 16), 0: no image
    int32_t lds;                        // bytes staged in LDS (multiple of 16)
    int32_t off_ixv, off_ixs, off_ixr, off_free, off_meta, off_terms1, off_terms0, pad;
    // dense index: (group start, end) per key value in [dense_min, dense_min + dense_n)
    // when the indexed constants span a small range (one LDS read instead of a search)
    int64_t dense_min;
    int32_t dense_n, off_dense;
};
#define SHR_IMG_MAX (144 * 1024)

#ifdef __cplusplus
extern "C" {
#endif
// matches opened at every key-segment position (cnt[p]); flag := 1 when a key's
// timestamps decrease (the window reduction does not hold)
// sts32 (optional): the sorted timestamps as 32-bit offsets from tbase (sts unused)
int shr_count(const shr_table* dT, const int64_t* sts, const uint32_t* skeys, int64_t n, uint32_t sentinel,
              const shd_cols* dC, uint32_t* cnt, int32_t* flag, void* stream, const uint8_t* img = nullptr,
              const shr_img* I = nullptr, const uint32_t* sts32 = nullptr, int64_t tbase = 0);
// the same scan, writing (opening, consuming, rule) records at off[p]
int shr_write(const shr_table* dT, const int64_t* sts, const uint32_t* skeys, int64_t n, uint32_t sentinel,
              const shd_cols* dC, const uint32_t* cnt, const uint32_t* off, uint32_t* rec_p, uint32_t* rec_q,
              uint32_t* rec_r, void* stream, const uint8_t* img = nullptr, const shr_img* I = nullptr,
              const uint32_t* sts32 = nullptr, int64_t tbase = 0);
// PartitionStreamReceiver runs of an arrival-order key array: flags[i] (run
// start), rid[i] (exclusive scan of flags), rfirst[run] (first arrival index);
// run_ids (may be NULL): the caller's run of every event (sh_device_run.d_run)
int shr_run_ids(const int32_t* akeys, const uint32_t* run_ids, int64_t n, int64_t batch, uint32_t* flags,
                uint32_t* rid, uint32_t* rfirst, uint32_t* scan_tmp, void* stream);
// order keys of the records: packed -> k0 = rule << qbits | offset in run,
// k1 = run; else k0 = offset in run, k1 = rule, k2 = run. akeys (the arrival-order
// keys): each run found by walking back from its consuming event, keyed by its first
// arrival index (flags / rid / rfirst unused); a walk longer than 512 events sets
// *long_run and leaves the keys unusable
int shr_keys(const uint32_t* rec_q, const uint32_t* rec_r, int64_t m, const uint32_t* perm, const uint32_t* flags,
             const uint32_t* rid, const uint32_t* rfirst, int64_t batch, int qbits, int packed, uint32_t* k0,
             uint32_t* k1, uint32_t* k2, void* stream,
             const int32_t* akeys = nullptr, const uint32_t* run_ids = nullptr,
             int32_t* long_run = nullptr);
// after the passes by (run, rule, offset) of records taken in any order: each run
// of equal keys (k2 may be NULL) put in rec_p order, in place
int shr_order_ties(uint32_t* order, int64_t m, const uint32_t* k0, const uint32_t* k1, const uint32_t* k2,
                   const uint32_t* rec_p, void* stream);
// gk[i] = key[order[i]], gv[i] = order[i] (order NULL: identity)
int shr_gather(const uint32_t* key, const uint32_t* order, int64_t m, uint32_t* gk, uint32_t* gv, void* stream);
// ordered output rows from the sorted record order
int shr_place(const shr_table* dT, const uint32_t* order, int64_t m, const uint32_t* rec_p, const uint32_t* rec_q,
              const uint32_t* rec_r, const uint32_t* perm, const int64_t* sts, const shd_cols* dC, uint64_t seq_base,
              int n_out, uint64_t* out_seq, int32_t* out_query, int64_t* out_ts, int64_t* out_vals, void* stream,
              const uint32_t* sts32 = nullptr, int64_t tbase = 0);
// sparse partials over arrival order (no key segment; sh_rules.hip): pre[2] (or
// NULL) the attributes f1 reads most on the event's row, loaded with the event; the partials
// (p, r, key) of every event into pr_* (count in *ctr, at most cap written), and
// their count per key (key_cnt[key]++); *flag |= 1 when the run's timestamps
// decrease, 2 when a key is >= nkeys
int shr_sparse_open(const shr_table* dT, const int64_t* ts, const int32_t* akeys, int64_t n, int32_t nkeys,
                    const shd_cols* dC, const uint8_t* img, const shr_img* I, uint32_t* pr_p, uint32_t* pr_r,
                    uint32_t* pr_key, uint32_t* key_cnt, unsigned long long* ctr, int64_t cap,
                    int32_t* flag, const int32_t* pre, void* stream);
// live-partial bitmap of the sparse path: bit (s, key) set when a partial of `key`
// may be consumed by an event of time slice s ([tmin + s << shift, ...)), i.e. it
// opens before the slice ends and expires after it starts. Zeroed by the caller;
// bits == NULL: no bitmap (every event reads its key's list bounds)
struct shr_live {
    uint32_t* bits;   // [nslices][wps]
    int64_t tmin;
    int32_t shift, nslices, wps, pad;
};
// the partials into their keys' lists (key_off: exclusive scan of key_cnt; key_fill:
// zeroed per-key slot counters) and the live bitmap; pre[2] (or NULL) the attributes
// f2 reads most on the consumer's row; the
// consuming event of each (least later event of its key in the window with f2),
// and the (p, q, r) records of the consumed ones (count in *rctr, any order)
int shr_sparse_match(const shr_table* dT, const int64_t* ts, const int32_t* akeys, int64_t n, const shd_cols* dC,
                     const uint8_t* img, const shr_img* I, const uint32_t* pr_p, const uint32_t* pr_r, const uint32_t* pr_key, uint32_t* key_fill,
                     const unsigned long long* ctr, int64_t n_pairs_max, const uint32_t* key_off, uint32_t* l_p,
                     uint32_t* l_r, int64_t* l_te, uint32_t* l_q, uint32_t* rec_p, uint32_t* rec_q, uint32_t* rec_r,
                     unsigned long long* rctr, int64_t rcap, int32_t nkeys, const shr_live* live,
                     const int32_t* pre, void* stream);
// the run's timestamp range (one read-back), and the 32-bit offsets from `base`
int shr_ts_range(const int64_t* ts, int64_t n, int64_t* lo, int64_t* hi, void* scratch16, void* stream);
int shr_ts_to32(const int64_t* ts, int64_t n, int64_t base, uint32_t* t32, void* stream);
#ifdef __cplusplus
}
#endif
