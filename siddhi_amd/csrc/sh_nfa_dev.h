// sh_nfa_dev.h — host <-> kernel interface of the general engine (sh_nfa.hip),
// called from sh_host_nfa.cpp.
#pragma once
#include <stdint.h>

#include "sh_nfa.h"

// emission sink (device pointers)
struct nfd_emit {
    uint64_t* recs;                // [cap][stride] records (sh_nfa.h NF_REC_HDR layout)
    unsigned long long* ctr;       // records handed out (chunked)
    int64_t cap;
    int32_t stride;                // NF_REC_HDR + max n_out
    int32_t pad;
    uint32_t* match_cnt;           // [n] emissions per run-first index (pre-zeroed)
    unsigned* err;                 // OR of nf_err bits
};

// events of one flush in arrival order (device pointers)
struct nfd_events {
    const int64_t* ts;
    const uint8_t* stream;         // NULL: stream 0
    const uint32_t* row;
    const uint32_t* bid;           // send() call id per event, NULL: one call
    const uint32_t* perm;          // key-segment position -> arrival index, NULL: identity
    uint64_t seq_base;
    int64_t batch_events;          // bid == NULL: send() call = arrival index / batch_events (0: one call)
    const int64_t* sts;            // timestamps in key-segment order (NULL: gather ts through perm)
    int32_t sorted_rows;           // 1: column rows are key-segment positions (columns carried by the segment)
    int32_t pad;
    const uint32_t* run;           // caller's PartitionStreamReceiver run per arrival index (sh_device_run.d_run), NULL: none
    const uint32_t* gidx;          // key-sharded push: arrival index -> position in the whole send() call, NULL: identity
};

struct nfd_cand {
    int64_t t;
    uint64_t stamp;
    int32_t key;
    int32_t pad;
};

#ifdef __cplusplus
extern "C" {
#endif
int nfd_run(const nf_table* dT, const nf_cols* dC, uint64_t* kstate, const nfd_events* ev, int64_t n,
            const uint32_t* seg_list, const uint32_t* nseg, const uint32_t* skeys, int32_t nkeys, int64_t max_segments,
            uint64_t tick, int64_t clock, const nfd_emit* em, void* stream);
// the rise-and-fall sequence engine (nf_query.s3) over the key segments, fresh state
int nfd_seq3(const nf_table* dT, const nf_cols* dC, const nfd_events* ev, int64_t n, const uint32_t* seg_list,
             const uint32_t* nseg, const uint32_t* skeys, int32_t nkeys, int64_t max_segments, const nfd_emit* em,
             void* stream, const void* s3_col = nullptr, int compact = 0, int agg = 0, int rw = 0);
// placement of k_seq3s's compact records (loc[cap], then [cap][rw] words over recs;
// wide bit o: output o is a 2-word running aggregate)
int nfd_place_s3(const uint64_t* recs, int64_t cap, int64_t nrec, int n_out, int type, uint64_t seq_base,
                 const uint32_t* offsets, int32_t* out_query, uint64_t* out_seq, int64_t* out_vals, uint32_t* inv,
                 int64_t total, void* stream, int rw, uint32_t wide);
int nfd_start(const nf_table* dT, const nf_cols* dC, uint64_t* kstate, uint64_t tick, int64_t clock,
              const nfd_emit* em, void* stream);
// armed (may be NULL): per-key maybe-registered flags (nf_cols.sched_armed);
// clear_armed: the scan covers the key's only absent processor, so an empty
// queue clears the flag
// rank (may be NULL): per key, its position in the scheduler map's iteration
// order (sh_jmap.h); NULL ranks by registration stamp (one key: unpartitioned)
int nfd_due(const nf_table* dT, int q, int p, const uint64_t* kstate, int32_t nkeys, int64_t now, nfd_cand* cand,
            unsigned long long* ctr, int64_t cap, uint8_t* armed, int clear_armed, const uint64_t* rank,
            void* stream);
// the due pass over the armed-key list (lin, count in device memory) plus the
// keys armed since the last pass (alog, may be NULL); survivors to lout (may be
// NULL: scan only); drop: a drained key leaves the list and clears its flag.
// max_items bounds the launch (grid-stride).
int nfd_due_list(const nf_table* dT, int q, int p, const uint64_t* kstate, const int32_t* lin,
                 const unsigned long long* lin_n, const int32_t* alog, const unsigned long long* alog_n, int64_t now,
                 nfd_cand* cand, unsigned long long* ctr, int64_t cap, uint8_t* armed, int drop, const uint64_t* rank,
                 int32_t* lout, unsigned long long* lout_n, int64_t max_items, void* stream);
// dst[keys[i]] = ranks[i]
int nfd_rank_scatter(const int32_t* keys, const uint64_t* ranks, int64_t n, uint64_t* dst, void* stream);
// device tie-break of a due-key backlog: tmin of the candidates, then per due
// time t (slot t - tmin of `range`) the key with the earliest stamp (-1: none)
// cand[i].stamp = rank[cand[i].key]
int nfd_cand_restamp(nfd_cand* cand, int64_t nc, const uint64_t* rank, void* stream);
int nfd_cand_tmin(const nfd_cand* cand, int64_t nc, unsigned long long* tmin, void* stream);
int nfd_cand_select(const nfd_cand* cand, int64_t nc, int64_t tmin, int64_t range, unsigned long long* slot_stamp,
                    int32_t* slot_key, void* stream);
// seq: trigger sequence number of the rows the timers emit (the next input event's);
// gpos (may be NULL): per selected key its position in the firing order over all
// ranks (key-sharded), which orders its rows and registration stamps
int nfd_timer(const nf_table* dT, const nf_cols* dC, uint64_t* kstate, int q, int p, const int32_t* keys, int32_t nsel,
              int64_t now, uint64_t tick, int64_t clock, uint64_t seq, const nfd_emit* em, void* stream,
              const uint32_t* gpos = nullptr);
int nfd_place(const uint64_t* recs, int64_t nrec, int stride, const uint32_t* offsets, int n_out, int32_t* out_query,
              uint64_t* out_seq, int64_t* out_ts, int64_t* out_vals, uint8_t* out_nulls, uint32_t* inv, int64_t total,
              void* stream);
// [a, a + abytes) and [b, b + bbytes) zeroed in one launch (4-byte multiples)
int nfd_zero2(void* a, int64_t abytes, void* b, int64_t bbytes, void* stream);
// the same for a launch of at most 8,192 records and events, in one workgroup
// (-1: too large, use nfd_place_app)
int nfd_place_app_small(const uint64_t* recs, int64_t nrec, int stride, const uint32_t* counts, int64_t n_idx,
                        int n_out, unsigned long long* base, int32_t* out_query, uint64_t* out_seq, int64_t* out_ts,
                        int64_t* out_vals, uint8_t* out_nulls, void* stream);
// nfd_place appended to device-resident output arrays after *base rows (count on the device)
int nfd_place_app(const uint64_t* recs, int64_t nrec, int stride, const uint32_t* offsets, const uint32_t* counts,
                  int64_t n_idx, int n_out, unsigned long long* base, int32_t* out_query, uint64_t* out_seq,
                  int64_t* out_ts, int64_t* out_vals, uint8_t* out_nulls, uint32_t* inv, void* stream);
int nfd_save(uint64_t* kstate, int64_t key_words, const uint32_t* seg_list, const uint32_t* nseg, const uint32_t* skeys,
             int64_t max_segments, uint64_t* save, int dir, void* stream);
int nfd_save_keys(uint64_t* kstate, int64_t key_words, const int32_t* keys, int32_t nkeys, uint64_t* save, int dir,
                  void* stream);
int nfd_relayout(const nf_table* dA, const nf_table* dB, const uint64_t* src, uint64_t* dst, int32_t nkeys,
                 void* stream);
#ifdef __cplusplus
}
#endif
