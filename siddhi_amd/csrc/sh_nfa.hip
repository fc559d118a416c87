// sh_nfa.hip — gfx950 kernels of the general per-key NFA engine (sh_nfa.h).
//
//   k_nfa_run    one lane per partition-key segment of a flushed batch set
//                (segments come from the radix segment in sh_kernels.hip); the
//                lane replays the key's events through the query processor graph
//                and writes emission records through a chunked sink
//   k_nfa_due    scheduler scan: keys whose FIFO head is due (Scheduler.onTimeChange)
//   k_nfa_timer  one lane per selected key: sendTimerEvents
//   k_nfa_inv / k_nfa_gather  ordered placement of emission records (exclusive scan of
//                counts; row -> record index, then a row-ordered gather)
//   k_nfa_save / k_nfa_load   copy the touched keys' blocks (replay after growth)
//   k_nfa_relayout            re-lays every key block into grown capacities
//
// Latency-bound by design: the parallelism is the number of keys present in a
// flush (C3: 1M keys, C4: 10M keys); per-key work is pointer chasing in the key's
// own arena, which stays L2-resident while its lane runs.
#include <cstdlib>
#include <hip/hip_runtime.h>

#include <algorithm>

#include "sh_nfa.h"
#include "sh_nfa_dev.h"
#include "sh_wave.h"

#define NF_TPB 128
#define NF_SINK_CHUNK 16

struct DevSink {
    uint64_t* buf;
    unsigned long long* ctr;
    int64_t cap;       // records
    int stride;        // words per record
    uint64_t* chunk;
    int used, n;
    __device__ uint64_t* slot(int) {
        if (used == n) {
            unsigned long long at = atomicAdd(ctr, (unsigned long long)NF_SINK_CHUNK);
            if ((int64_t)at + NF_SINK_CHUNK > cap) return nullptr;
            chunk = buf + (int64_t)at * stride;
            used = 0;
            n = NF_SINK_CHUNK;
        }
        uint64_t* r = chunk + (int64_t)used * stride;
        used++;
        return r;
    }
    __device__ void finish() {
        for (int i = used; i < n; i++) chunk[(int64_t)i * stride] = ~0ull;
    }
};

struct DevEvents {
    const int64_t* ts;
    const uint8_t* stream;
    const uint32_t* row;
    const uint32_t* bid;
    const uint32_t* perm;   // key-segment position -> arrival index (NULL: identity)
    uint64_t seq_base;
    int64_t batch_events;
    const int64_t* sts;
    int32_t sorted_rows;
    const uint32_t* run;    // caller's run ids by arrival index (NULL: from adjacency and the send() call)
    const uint32_t* gidx;   // key-sharded push: position of each event in the whole send() call
    __device__ uint32_t at(int64_t k) const { return perm ? perm[k] : (uint32_t)k; }
    __device__ uint32_t pos(int64_t k) const { return gidx ? gidx[at(k)] : at(k); }
};
// the Events interface of nf_process_segment / NfLane::receive
struct DevEv {
    const DevEvents* E;
    // key-segment-ordered copies (sh_run_device) make a lane's reads sequential
    // instead of one gather through perm per event
    __device__ int64_t ts(int64_t k) const { return E->sts ? E->sts[k] : E->ts[E->at(k)]; }
    __device__ uint32_t row(int64_t k) const {
        if (E->sorted_rows) return (uint32_t)k;
        return E->row ? E->row[E->at(k)] : E->at(k);
    }
    __device__ uint64_t seq(int64_t k) const { return E->seq_base + E->pos(k); }
    __device__ int stream(int64_t k) const { return E->stream ? E->stream[E->at(k)] : 0; }
    __device__ uint32_t local(int64_t k) const { return E->pos(k); }
    __device__ uint32_t batch(int64_t k) const {
        return E->bid ? E->bid[E->at(k)] : (E->batch_events ? (uint32_t)(E->at(k) / E->batch_events) : 0u);
    }
    // key-segment position e continues the run that starts at k (e - 1 does)
    __device__ bool joins(int64_t e, int64_t k) const {
        if (E->run) return E->run[E->at(e)] == E->run[E->at(k)];
        return local(e) == local(e - 1) + 1 && batch(e) == batch(k);
    }
};

__device__ inline void lane_init(NfLane<DevSink>& L, const nf_table* T, const nf_cols* C, uint64_t* kb,
                                 DevSink* sink, int64_t clock, int32_t key) {
    L.key = key;
    L.T = T;
    L.C = C;
    L.kb = kb;
    L.sink = sink;
    L.Q = nullptr;
    L.qb = nullptr;
    L.qi = 0;
    L.partitioned = T->partitioned;
    L.in_holder = 0;
    L.h_first = L.h_last = 0;
    L.h_has = 0;
    L.cur_seq = 0;
    L.tag_index = 0;
    L.ordinal = 0;
    L.clock = clock;
    L.stamp = 0;
    L.err = 0;
}

__global__ void __launch_bounds__(NF_TPB) k_nfa_run(const nf_table* __restrict__ T, const nf_cols* __restrict__ C,
                                                    uint64_t* __restrict__ kstate, DevEvents E, int64_t n,
                                                    const uint32_t* __restrict__ seg_list,
                                                    const uint32_t* __restrict__ nseg,
                                                    const uint32_t* __restrict__ skeys, int32_t nkeys, uint64_t tick,
                                                    int64_t clock, nfd_emit EM) {
    const uint32_t sidx = blockIdx.x * blockDim.x + threadIdx.x;
    if (sidx >= *nseg) return;
    const uint32_t beg = seg_list[sidx];
    const uint32_t key = skeys ? skeys[beg] : 0u;
    if (key >= (uint32_t)nkeys) {
        atomicOr(EM.err, (unsigned)NF_E_KEY);
        return;
    }
    int64_t end = beg + 1;
    if (skeys)
        while (end < n && skeys[end] == key) end++;
    else
        end = n;
    DevSink sink;
    sink.buf = EM.recs;
    sink.ctr = EM.ctr;
    sink.cap = EM.cap;
    sink.stride = EM.stride;
    sink.chunk = nullptr;
    sink.used = sink.n = 0;
    NfLane<DevSink> L;
    lane_init(L, T, C, kstate + (int64_t)key * T->key_words, &sink, clock, (int32_t)key);
    DevEv ev{&E};
    nf_process_segment(L, ev, (int64_t)beg, end, tick, EM.match_cnt);
    if (sink.chunk) sink.finish();
    if (L.err) atomicOr(EM.err, L.err);
}

// The rise-and-fall sequence (nf_query.s3, sh_nfa_lower.cpp detect_seq3): one
// lane per key segment, the key's single partial in registers. Per event x:
//   hit = (a last e2 exists) && f3(x, last)        -> emit (e1, last, x)
//   else if f2(x, e1) -> last = x (the e2 run grows)
//   else              -> e1 = x (every: the new start partial)
// Fresh per-key state each run (sh_run_device); emission records and per-event
// counts as k_nfa_run writes them, so k_nfa_place orders the rows.
__device__ __forceinline__ NfVal s3_val(const nf_cols* C, int a, int t, uint32_t row) {
    NfVal v;
    v.t = (uint8_t)t;
    const uint8_t* nm = C->nul[0][a];
    v.null = nm ? nm[row] : 0;
    const void* p = C->col[0][a];
    switch (t) {
        case SH_T_LONG:
        case SH_T_DOUBLE: v.b = ((const int64_t*)p)[row]; break;
        case SH_T_FLOAT: v.b = (int64_t)((const uint32_t*)p)[row]; break;
        case SH_T_BOOL: v.b = ((const uint8_t*)p)[row] ? 1 : 0; break;
        default: v.b = (int64_t)((const int32_t*)p)[row];
    }
    return v;
}

template <int S3_U>
__global__ void __launch_bounds__(NF_TPB) k_seq3(const nf_table* __restrict__ T, const nf_cols* __restrict__ C,
                                                 DevEvents E, int64_t n, const uint32_t* __restrict__ seg_list,
                                                 const uint32_t* __restrict__ nseg,
                                                 const uint32_t* __restrict__ skeys, int32_t nkeys, nfd_emit EM) {
    const uint32_t sidx = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t ns = *nseg;
    if (sidx >= ns) return;
    const uint32_t beg = seg_list[sidx];
    const uint32_t key = skeys ? skeys[beg] : 0u;
    if (key >= (uint32_t)nkeys) {
        atomicOr(EM.err, (unsigned)NF_E_KEY);
        return;
    }
    // segments are listed in order; only the last one may be followed by the
    // null-key run
    int64_t end;
    if (!skeys) {
        end = n;
    } else if (sidx + 1 < ns) {
        end = seg_list[sidx + 1];
    } else {
        end = beg + 1;
        while (end < n && skeys[end] == key) end++;
    }
    const nf_query& Q = T->q[0];
    const bool same2 = Q.s3_e1a == Q.s3_a2 && Q.s3_e1t == Q.s3_t2;  // e1's operand is x's f2 operand
    const bool same3 = Q.s3_la == Q.s3_a3 && Q.s3_lt == Q.s3_t3;
    const bool same23 = Q.s3_a2 == Q.s3_a3 && Q.s3_t2 == Q.s3_t3;  // f2 and f3 read one attribute of x
    DevSink sink;
    sink.buf = EM.recs;
    sink.ctr = EM.ctr;
    sink.cap = EM.cap;
    sink.stride = EM.stride;
    sink.chunk = nullptr;
    sink.used = sink.n = 0;
    DevEv ev{&E};
    bool has_last = false, has_e1 = false;
    uint32_t e1_row = 0, last_row = 0;
    NfVal e1v, lastv;
    e1v.b = lastv.b = 0;
    e1v.t = lastv.t = 0;
    e1v.null = lastv.null = 1;
    bool fail = false;
    for (int64_t k0 = beg; k0 < end && !fail; k0 += S3_U) {
        // the block's operands together (independent loads in flight)
        NfVal x2v[S3_U], x3v[S3_U];
#pragma unroll
        for (int u = 0; u < S3_U; u++) {
            const int64_t k = k0 + u < end ? k0 + u : end - 1;
            const uint32_t row = ev.row(k);
            x2v[u] = s3_val(C, Q.s3_a2, Q.s3_t2, row);
            x3v[u] = same23 ? x2v[u] : s3_val(C, Q.s3_a3, Q.s3_t3, row);
        }
#pragma unroll
        for (int u = 0; u < S3_U; u++) {
            const int64_t k = k0 + u;
            if (k >= end) break;
            const uint32_t row = ev.row(k);
            const bool hit = has_last && !x3v[u].null && !lastv.null && nf_cmp(Q.s3_op3, Q.s3_dom3, x3v[u], lastv);
            if (hit) {
                uint64_t* r = sink.slot(0);
                if (!r) {
                    fail = true;
                    break;
                }
                const uint32_t loc = ev.local(k);
                r[0] = (uint64_t)loc;
                r[1] = (uint64_t)ev.ts(k);
                uint64_t nulls = 0;
                for (int o = 0; o < Q.n_out; o++) {
                    const int sl = Q.s3_out_slot[o];
                    const NfVal v =
                        s3_val(C, Q.s3_out_attr[o], Q.s3_out_type[o], sl == 0 ? e1_row : sl == 1 ? last_row : row);
                    r[NF_REC_HDR + o] = (uint64_t)v.b;
                    if (v.null) nulls |= 1ull << o;
                }
                r[2] = nulls;  // query 0
                r[3] = ev.seq(k);
                EM.match_cnt[loc] = 1;
            }
            if (!hit && has_e1 && !x2v[u].null && !e1v.null && nf_cmp(Q.s3_op2, Q.s3_dom2, x2v[u], e1v)) {
                has_last = true;
                last_row = row;
                lastv = same3 ? x3v[u] : s3_val(C, Q.s3_la, Q.s3_lt, row);
            } else {
                has_last = false;
                has_e1 = true;
                e1_row = row;
                e1v = same2 ? x2v[u] : s3_val(C, Q.s3_e1a, Q.s3_e1t, row);
            }
        }
    }
    if (sink.chunk) sink.finish();
    if (fail) atomicOr(EM.err, (unsigned)NF_E_EMIT);
}

// The same sequence, LDS-staged: when every operand and output reads one 4-byte
// attribute without a null mask (C3), a workgroup owns 256 consecutive key
// segments, one per lane, and walks them in rounds: each round the workgroup
// loads the next S3S_E events of EVERY lane's segment into LDS (value + arrival
// index; 16 threads per 64-byte run) and each lane then steps through its own
// window from LDS. k_seq3's lane-strided loads touch one line per lane per load
// and lose most lines before the lane comes back for the rest.
#define S3S_TPB 256
#define S3S_E 16
#define S3S_LD (S3S_E + 1)  // padded lane stride: the lanes' LDS reads hit distinct banks
__device__ __forceinline__ NfVal s3_bits(uint32_t b, int t) {
    NfVal v;
    v.t = (uint8_t)t;
    v.null = 0;
    v.b = t == SH_T_INT ? (int64_t)(int32_t)b : (int64_t)b;
    return v;
}

// COMPACT: one record slot per key-ordered position (each event triggers at most one
// match) over the emission buffer -- loc[cap] (the trigger's arrival index, ~0u: no
// match; written for every position, coalesced from LDS), then [cap][1 + n_out] words
// (loc again and the raw 4-byte select values) for the positions that matched --
// placed by k_s3_inv / k_s3_gather. No record counter: the generic sink's chunk claims are one atomic on
// a single word per 16 records, which serialises at the L2 (C3: 1.5M claims).
// AGG (COMPACT only): the selector's sum / avg / count run in the lane -- one key's
// matches in trigger order, the reference's own sequence of double additions
// (AttributeAggregatorExecutor state per partition key) -- and the record holds the
// running value (2 words) instead of the argument; rw = record words
#define S3S_MAXO 6
template <bool COMPACT, bool AGG>
__global__ void __launch_bounds__(S3S_TPB) k_seq3s(const nf_table* __restrict__ T, const uint32_t* __restrict__ col,
                                                   const uint32_t* __restrict__ perm, uint64_t seq_base, int64_t n,
                                                   const uint32_t* __restrict__ seg_list,
                                                   const uint32_t* __restrict__ nseg,
                                                   const uint32_t* __restrict__ skeys, int32_t nkeys, nfd_emit EM,
                                                   int rw) {
    __shared__ uint32_t sv[S3S_TPB * S3S_LD], sp[S3S_TPB * S3S_LD];
    __shared__ uint32_t s_b[S3S_TPB], s_e[S3S_TPB];
    __shared__ int64_t s_end;
    const uint32_t ns = *nseg;
    const uint32_t s0 = blockIdx.x * S3S_TPB;
    if (s0 >= ns) {  // uniform per workgroup
        // COMPACT, no keyed event at all: every slot is empty
        if (COMPACT && ns == 0 && blockIdx.x == 0)
            for (int64_t p = threadIdx.x; p < n; p += S3S_TPB) ((uint32_t*)EM.recs)[p] = ~0u;
        return;
    }
    const uint32_t sl = min(s0 + (uint32_t)S3S_TPB, ns) - 1u;  // the workgroup's last segment
    if (threadIdx.x == 0) {
        // segments are listed in order; only the last one may be followed by the
        // null-key run
        int64_t e;
        if (sl + 1u < ns) {
            e = seg_list[sl + 1u];
        } else if (!skeys) {
            e = n;
        } else {
            const uint32_t k = skeys[seg_list[sl]];
            e = (int64_t)seg_list[sl] + 1;
            while (e < n && skeys[e] == k) e++;
        }
        s_end = e;
    }
    __syncthreads();
    const uint32_t P1 = (uint32_t)s_end;
    const uint32_t sidx = s0 + threadIdx.x;
    uint32_t b = P1, e = P1;  // lanes past the last segment: empty
    if (sidx <= sl) {
        b = seg_list[sidx];
        e = sidx < sl ? seg_list[sidx + 1u] : P1;
        if ((skeys ? skeys[b] : 0u) >= (uint32_t)nkeys) {
            atomicOr(EM.err, (unsigned)NF_E_KEY);
            b = e = P1;
        }
    }
    s_b[threadIdx.x] = b;
    s_e[threadIdx.x] = e;
    const nf_query& Q = T->q[0];
    const int t = Q.s3_t2;  // the one attribute's type (checked on the host)
    const int op2 = Q.s3_op2, dom2 = Q.s3_dom2, op3 = Q.s3_op3, dom3 = Q.s3_dom3, no = Q.n_out;
    DevSink sink;
    sink.buf = EM.recs;
    sink.ctr = EM.ctr;
    sink.cap = EM.cap;
    sink.stride = EM.stride;
    sink.chunk = nullptr;
    sink.used = sink.n = 0;
    uint32_t* const rl = (uint32_t*)EM.recs;  // COMPACT: loc per record, then the values
    uint32_t* const rv = rl + EM.cap;
    bool has_last = false, has_e1 = false, fail = false;
    uint32_t e1b = 0, lastb = 0;
    int64_t acc[S3S_MAXO], acnt[S3S_MAXO];  // AGG: running sum (long or double bits) and count per output
#pragma unroll
    for (int o = 0; o < S3S_MAXO; o++) acc[o] = acnt[o] = 0;
    __syncthreads();
    for (uint32_t r0 = 0;; r0 += S3S_E) {
        // every lane's next window, loaded by the whole workgroup
        for (int idx = threadIdx.x; idx < S3S_TPB * S3S_E; idx += S3S_TPB) {
            const int l = idx / S3S_E, j = idx % S3S_E;
            const uint32_t p = s_b[l] + r0 + (uint32_t)j;
            if (p < s_e[l]) {
                sv[l * S3S_LD + j] = col[p];
                sp[l * S3S_LD + j] = perm ? perm[p] : p;
            }
        }
        __syncthreads();
        const uint32_t w0 = b + r0;
        const int cnt = w0 >= e ? 0 : (e - w0 < (uint32_t)S3S_E ? (int)(e - w0) : S3S_E);
        for (int j = 0; j < cnt && !fail; j++) {
            const uint32_t xb = sv[threadIdx.x * S3S_LD + j];
            const NfVal x = s3_bits(xb, t);
            const bool hit = has_last && nf_cmp(op3, dom3, x, s3_bits(lastb, t));
            if (COMPACT) {
                // the slot's record: the trigger's arrival index or ~0u, written back below
                const uint32_t loc = sp[threadIdx.x * S3S_LD + j];
                sv[threadIdx.x * S3S_LD + j] = hit ? loc : ~0u;
                if (hit && !AGG) {
                    // [loc, values]: the gather reads one record in one line
                    uint32_t* r = rv + (int64_t)(w0 + (uint32_t)j) * rw;
                    r[0] = loc;
                    for (int o = 0; o < no; o++) {
                        const int s = Q.s3_out_slot[o];
                        r[1 + o] = s == 0 ? e1b : s == 1 ? lastb : xb;
                    }
                    EM.match_cnt[loc] = 1;
                } else if (hit) {
                    uint32_t* r = rv + (int64_t)(w0 + (uint32_t)j) * rw;
                    r[0] = loc;
                    int wi = 1;
#pragma unroll
                    for (int o = 0; o < S3S_MAXO; o++) {
                        const int ak = o < no ? Q.out_agg[o] : -1;
                        if (ak < 0) continue;
                        const int s = Q.s3_out_slot[o];
                        const uint32_t vb = s == 0 ? e1b : s == 1 ? lastb : xb;
                        if (ak == SH_AGG_NONE) {
                            r[wi++] = vb;
                            continue;
                        }
                        // SumAttributeAggregatorExecutor / AvgAttributeAggregatorExecutor /
                        // CountAttributeAggregatorExecutor on a current event (no nulls here)
                        acnt[o]++;
                        uint64_t ov;
                        if (ak == SH_AGG_COUNT) {
                            ov = (uint64_t)acnt[o];
                        } else if (ak == SH_AGG_SUM && t == SH_T_INT) {
                            acc[o] = (int64_t)((uint64_t)acc[o] + (uint64_t)(int64_t)(int32_t)vb);
                            ov = (uint64_t)acc[o];
                        } else {
                            const double x = t == SH_T_INT ? (double)(int32_t)vb : (double)__uint_as_float(vb);
                            const double d = __longlong_as_double(acc[o]) + x;
                            acc[o] = __double_as_longlong(d);
                            ov = (uint64_t)__double_as_longlong(ak == SH_AGG_AVG ? d / (double)acnt[o] : d);
                        }
                        r[wi] = (uint32_t)ov;
                        r[wi + 1] = (uint32_t)(ov >> 32);
                        wi += 2;
                    }
                    EM.match_cnt[loc] = 1;
                }
            } else if (hit) {
                uint64_t* r = sink.slot(0);
                if (!r) {
                    fail = true;
                    break;
                }
                const uint32_t loc = sp[threadIdx.x * S3S_LD + j];
                r[0] = (uint64_t)loc;
                r[1] = 0;  // the device path places no timestamps
                r[2] = 0;  // no nulls, query 0
                r[3] = seq_base + loc;
                for (int o = 0; o < no; o++) {
                    const int s = Q.s3_out_slot[o];
                    r[NF_REC_HDR + o] = (uint64_t)s3_bits(s == 0 ? e1b : s == 1 ? lastb : xb, t).b;
                }
                EM.match_cnt[loc] = 1;
            }
            if (!hit && has_e1 && nf_cmp(op2, dom2, x, s3_bits(e1b, t))) {
                has_last = true;
                lastb = xb;
            } else {
                has_last = false;
                has_e1 = true;
                e1b = xb;
            }
        }
        // (a barrier too: the write-back and the next round's loads wait for every walk)
        const bool more = __syncthreads_or(w0 + S3S_E < e);
        if (COMPACT) {
            for (int idx = threadIdx.x; idx < S3S_TPB * S3S_E; idx += S3S_TPB) {
                const int l = idx / S3S_E, j = idx % S3S_E;
                const uint32_t p = s_b[l] + r0 + (uint32_t)j;
                if (p < s_e[l]) rl[p] = sv[l * S3S_LD + j];
            }
            __syncthreads();
        }
        if (!more) break;
    }
    // COMPACT: the null-key run after the last segment has no records
    if (COMPACT && sl + 1u == ns)
        for (int64_t p = (int64_t)P1 + threadIdx.x; p < n; p += S3S_TPB) rl[p] = ~0u;
    if (!COMPACT && sink.chunk) sink.finish();
    if (fail) atomicOr(EM.err, (unsigned)NF_E_EMIT);
}

// ordered placement of the compact records (k_nfa_inv / k_nfa_gather for k_seq3s)
__global__ void __launch_bounds__(256) k_s3_inv(const uint32_t* __restrict__ rl, int64_t nrec,
                                                const uint32_t* __restrict__ offsets, uint32_t* __restrict__ inv) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nrec) return;
    const uint32_t loc = rl[i];
    if (loc == ~0u) return;
    inv[offsets[loc]] = (uint32_t)i;  // at most one row per event
}

__global__ void __launch_bounds__(256) k_s3_gather(const uint32_t* __restrict__ rl, const uint32_t* __restrict__ rv,
                                                   const uint32_t* __restrict__ inv, int64_t total, int64_t nrec,
                                                   int n_out, int type, uint64_t seq_base,
                                                   int32_t* __restrict__ out_query, uint64_t* __restrict__ out_seq,
                                                   int64_t* __restrict__ out_vals, int rw, uint32_t wide) {
    const int64_t dst = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (dst >= total) return;
    const uint32_t ix = inv[dst];
    if ((int64_t)ix >= nrec) return;  // no record (an emission overflow, reported through err)
    const uint32_t* r = rv + (int64_t)ix * rw;
    if (out_query) out_query[dst] = 0;
    if (out_seq) out_seq[dst] = seq_base + r[0];
    if (out_vals) {
        // wide bit o: output o is a running aggregate (two words)
        int wi = 1;
        for (int o = 0; o < n_out; o++) {
            if ((wide >> o) & 1u) {
                out_vals[dst * n_out + o] = (int64_t)((uint64_t)r[wi] | ((uint64_t)r[wi + 1] << 32));
                wi += 2;
            } else {
                out_vals[dst * n_out + o] = s3_bits(r[wi++], type).b;
            }
        }
    }
}

extern "C" int nfd_place_s3(const uint64_t* recs, int64_t cap, int64_t nrec, int n_out, int type, uint64_t seq_base,
                            const uint32_t* offsets, int32_t* out_query, uint64_t* out_seq, int64_t* out_vals,
                            uint32_t* inv, int64_t total, void* stream, int rw, uint32_t wide) {
    if (nrec <= 0 || total <= 0) return 0;
    const uint32_t* rl = (const uint32_t*)recs;
    hipMemsetAsync(inv, 0xFF, (size_t)total * 4, (hipStream_t)stream);
    hipLaunchKernelGGL(k_s3_inv, dim3((unsigned)((nrec + 255) / 256)), dim3(256), 0, (hipStream_t)stream, rl, nrec,
                       offsets, inv);
    hipLaunchKernelGGL(k_s3_gather, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, (hipStream_t)stream, rl,
                       rl + cap, (const uint32_t*)inv, total, nrec, n_out, type, seq_base, out_query, out_seq,
                       out_vals, rw, wide);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

// unpartitioned apps: StateStreamRuntime.initPartition at SiddhiAppRuntime.start
__global__ void k_nfa_start(const nf_table* __restrict__ T, const nf_cols* __restrict__ C, uint64_t* __restrict__ kstate,
                            uint64_t tick, int64_t clock, nfd_emit EM) {
    if (blockIdx.x * blockDim.x + threadIdx.x != 0) return;
    NfLane<DevSink> L;
    lane_init(L, T, C, kstate, nullptr, clock, 0);
    L.kb[0] |= 1ull;
    for (int q = 0; q < T->n_queries; q++) {
        L.Q = &T->q[q];
        L.qb = L.kb + L.Q->q_off;
        L.qi = q;
        L.stamp = tick << 32;
        L.init_partition();
    }
    if (L.err) atomicOr(EM.err, L.err);
}

// Scheduler.onTimeChange, first half: every key whose queue head is due
__global__ void __launch_bounds__(256) k_nfa_due(const nf_table* __restrict__ T, int q, int p,
                                                 const uint64_t* __restrict__ kstate, int32_t nkeys, int64_t now,
                                                 nfd_cand* __restrict__ cand, unsigned long long* __restrict__ ctr,
                                                 int64_t cap, uint8_t* __restrict__ armed, int clear_armed,
                                                 const uint64_t* __restrict__ rank) {
    const int32_t key = blockIdx.x * blockDim.x + threadIdx.x;
    if (key >= nkeys) return;
    if (armed && !armed[key]) return;  // never registered since its queues were last empty
    const nf_query& Q = T->q[q];
    const uint64_t* kb = kstate + (int64_t)key * T->key_words;
    const uint64_t* sq = kb + Q.q_off + Q.lay.off_sched + (int64_t)p * (2 + Q.lay.sched_cap);
    const uint32_t head = (uint32_t)sq[0], cnt = (uint32_t)(sq[0] >> 32);
    if (!cnt) {
        if (armed && clear_armed) armed[key] = 0;
        return;
    }
    if (T->partitioned && !(sq[1] >> 63)) return;
    const int64_t t = (int64_t)sq[2 + head];
    if (t > now) return;
    unsigned long long at = atomicAdd(ctr, 1ull);
    if ((int64_t)at >= cap) return;
    cand[at].t = t;
    // position of the key's state in the scheduler map's iteration order
    cand[at].stamp = rank ? rank[key] : (sq[1] & ~(1ull << 63));
    cand[at].key = key;
    cand[at].pad = 0;
}

// The due pass over the armed-key list instead of every key: the list holds
// every key that may have a queued notification (armed flag set), the arm log
// the keys armed since the last pass. Survivors (non-empty queue, or every key
// when `drop` is off) go to lout; a drained key leaves the list and clears its
// flag. Scheduler.onTimeChange's head-peek per state (Scheduler.java:74-99).
__global__ void __launch_bounds__(256) k_nfa_due_list(const nf_table* __restrict__ T, int q, int p,
                                                      const uint64_t* __restrict__ kstate,
                                                      const int32_t* __restrict__ lin,
                                                      const unsigned long long* __restrict__ lin_n,
                                                      const int32_t* __restrict__ alog,
                                                      const unsigned long long* __restrict__ alog_n, int64_t now,
                                                      nfd_cand* __restrict__ cand, unsigned long long* __restrict__ ctr,
                                                      int64_t cap, uint8_t* __restrict__ armed, int drop,
                                                      const uint64_t* __restrict__ rank, int32_t* __restrict__ lout,
                                                      unsigned long long* __restrict__ lout_n) {
    const int64_t n1 = (int64_t)*lin_n, n2 = alog ? (int64_t)*alog_n : 0;
    const nf_query& Q = T->q[q];
    const int lane = threadIdx.x & 63;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    // uniform trip count per wave (ballots below)
    for (int64_t i0 = (int64_t)blockIdx.x * blockDim.x + (threadIdx.x & ~63); i0 < n1 + n2; i0 += stride) {
        const int64_t i = i0 + lane;
        bool keep = false, due = false;
        int32_t key = -1;
        int64_t t = 0;
        uint64_t stamp = 0;
        if (i < n1 + n2) {
            key = i < n1 ? lin[i] : alog[i - n1];
            const uint64_t* kb = kstate + (int64_t)key * T->key_words;
            const uint64_t* sq = kb + Q.q_off + Q.lay.off_sched + (int64_t)p * (2 + Q.lay.sched_cap);
            const uint32_t head = (uint32_t)sq[0], cnt = (uint32_t)(sq[0] >> 32);
            if (!cnt && drop) {
                armed[key] = 0;
            } else {
                keep = true;
                if (cnt && (!T->partitioned || (sq[1] >> 63))) {
                    t = (int64_t)sq[2 + head];
                    due = t <= now;
                    stamp = rank ? rank[key] : (sq[1] & ~(1ull << 63));
                }
            }
        }
        const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
        if (lout) {
            const uint64_t km = __ballot(keep);
            unsigned long long base = 0;
            if (km) {
                const int leader = __ffsll((long long)km) - 1;
                if (lane == leader) base = atomicAdd(lout_n, (unsigned long long)__popcll(km));
                base = __shfl(base, leader);
            }
            if (keep) lout[base + __popcll(km & lt)] = key;
        }
        const uint64_t dm = __ballot(due);
        if (dm) {
            const int leader = __ffsll((long long)dm) - 1;
            unsigned long long base = 0;
            if (lane == leader) base = atomicAdd(ctr, (unsigned long long)__popcll(dm));
            base = __shfl(base, leader);
            const unsigned long long at = base + __popcll(dm & lt);
            if (due && (int64_t)at < cap) {
                cand[at].t = t;
                cand[at].stamp = stamp;
                cand[at].key = key;
                cand[at].pad = 0;
            }
        }
    }
}

// Scheduler.onTimeChange tie-break on the device for a large backlog of due
// keys: the earliest registration stamp per distinct due time (TreeMultimap with
// a zero value comparator keeps one scheduler per time), slot = t - tmin
__global__ void __launch_bounds__(256) k_cand_tmin(const nfd_cand* __restrict__ cand, int64_t nc,
                                                   unsigned long long* __restrict__ tmin) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < nc) atomicMin(tmin, (unsigned long long)cand[i].t);
}

__global__ void __launch_bounds__(256) k_cand_slot(const nfd_cand* __restrict__ cand, int64_t nc, int64_t tmin,
                                                   unsigned long long* __restrict__ slot_stamp) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < nc) atomicMin(&slot_stamp[cand[i].t - tmin], (unsigned long long)cand[i].stamp);
}

__global__ void __launch_bounds__(256) k_cand_pick(const nfd_cand* __restrict__ cand, int64_t nc, int64_t tmin,
                                                   const unsigned long long* __restrict__ slot_stamp,
                                                   int32_t* __restrict__ slot_key) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nc) return;
    const int64_t s = cand[i].t - tmin;
    if (slot_stamp[s] == (unsigned long long)cand[i].stamp) slot_key[s] = cand[i].key;
}

// Scheduler.onTimeChange, second half: sendTimerEvents for each selected key
// (rank = position in due-time order = emission order)
__global__ void __launch_bounds__(NF_TPB) k_nfa_timer(const nf_table* __restrict__ T, const nf_cols* __restrict__ C,
                                                      uint64_t* __restrict__ kstate, int q, int p,
                                                      const int32_t* __restrict__ keys, int32_t nsel, int64_t now,
                                                      uint64_t tick, int64_t clock, uint64_t seq, nfd_emit EM,
                                                      const uint32_t* __restrict__ gpos) {
    const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nsel) return;
    const uint32_t r = gpos ? gpos[i] : (uint32_t)i;  // position in the firing order
    DevSink sink;
    sink.buf = EM.recs;
    sink.ctr = EM.ctr;
    sink.cap = EM.cap;
    sink.stride = EM.stride;
    sink.chunk = nullptr;
    sink.used = sink.n = 0;
    NfLane<DevSink> L;
    lane_init(L, T, C, kstate + (int64_t)keys[i] * T->key_words, &sink, clock, keys[i]);
    L.Q = &T->q[q];
    L.qb = L.kb + L.Q->q_off;
    L.qi = q;
    L.tag_index = (uint32_t)r;
    L.cur_seq = seq;  // rows a timer emits: the next input event's sequence number
    L.stamp = (tick << 32) | (uint64_t)r;
    L.send_timer_events(p, now);
    if (L.ordinal) EM.match_cnt[r] = L.ordinal;
    if (sink.chunk) sink.finish();
    if (L.err) atomicOr(EM.err, L.err);
}

// ordered placement in two passes: the records (grouped by key) scatter only their
// index to the row they own (inv, 4 B per row: the random writes stay small and sit in
// the memory-side cache), then one thread per output row gathers its record and writes
// every output array in row order (coalesced). Unused outputs are NULL.
__global__ void __launch_bounds__(256) k_nfa_inv(const uint64_t* __restrict__ recs, int64_t nrec, int stride,
                                                 const uint32_t* __restrict__ offsets, uint32_t* __restrict__ inv) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nrec) return;
    const uint64_t tag = recs[i * stride];
    if (tag == ~0ull) return;
    inv[(int64_t)offsets[(uint32_t)tag] + (int64_t)(tag >> 32)] = (uint32_t)i;
}

__global__ void __launch_bounds__(256) k_nfa_gather(const uint64_t* __restrict__ recs, const uint32_t* __restrict__ inv,
                                                    int64_t total, int64_t nrec, int stride, int n_out,
                                                    int32_t* __restrict__ out_query, uint64_t* __restrict__ out_seq,
                                                    int64_t* __restrict__ out_ts, int64_t* __restrict__ out_vals,
                                                    uint8_t* __restrict__ out_nulls) {
    const int64_t dst = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (dst >= total) return;
    const uint32_t ix = inv[dst];
    if ((int64_t)ix >= nrec) return;  // no record (an emission overflow, reported through err)
    const uint64_t* r = recs + (int64_t)ix * stride;
    const uint64_t h2 = r[2];
    if (out_query) out_query[dst] = (int)(h2 >> 32);
    if (out_seq) out_seq[dst] = r[3];
    if (out_ts) out_ts[dst] = (int64_t)r[1];
    for (int c = 0; c < n_out; c++) {
        const bool has = c < stride - NF_REC_HDR;
        if (out_vals) out_vals[dst * n_out + c] = has ? (int64_t)r[NF_REC_HDR + c] : 0;
        if (out_nulls) out_nulls[dst * n_out + c] = has ? (uint8_t)((h2 >> c) & 1) : 1;
    }
}

// blocks of the keys touched by this flush <-> compact save area
__global__ void k_nfa_save(const uint64_t* __restrict__ kstate, int64_t key_words, const uint32_t* __restrict__ seg_list,
                           const uint32_t* __restrict__ nseg, const uint32_t* __restrict__ skeys,
                           uint64_t* __restrict__ save, int dir) {
    const uint32_t s = blockIdx.x;
    if (s >= *nseg) return;
    const uint32_t key = skeys ? skeys[seg_list[s]] : 0u;
    uint64_t* kb = (uint64_t*)kstate + (int64_t)key * key_words;
    uint64_t* sv = save + (int64_t)s * key_words;
    for (int64_t w = threadIdx.x; w < key_words; w += blockDim.x) {
        if (dir == 0)
            sv[w] = kb[w];
        else
            kb[w] = sv[w];
    }
}

__global__ void k_nfa_save_keys(uint64_t* __restrict__ kstate, int64_t key_words, const int32_t* __restrict__ keys,
                                uint64_t* __restrict__ save, int dir) {
    const int32_t s = blockIdx.x;
    uint64_t* kb = kstate + (int64_t)keys[s] * key_words;
    uint64_t* sv = save + (int64_t)s * key_words;
    for (int64_t w = threadIdx.x; w < key_words; w += blockDim.x) {
        if (dir == 0)
            sv[w] = kb[w];
        else
            kb[w] = sv[w];
    }
}

// re-lay one key block from table A's layout into table B's (capacities grown)
__global__ void k_nfa_relayout(const nf_table* __restrict__ A, const nf_table* __restrict__ B,
                               const uint64_t* __restrict__ src, uint64_t* __restrict__ dst, int32_t nkeys) {
    const int32_t key = blockIdx.x;
    if (key >= nkeys) return;
    const uint64_t* s0 = src + (int64_t)key * A->key_words;
    uint64_t* d0 = dst + (int64_t)key * B->key_words;
    const int t = threadIdx.x, nt = blockDim.x;
    for (int64_t w = t; w < B->key_words; w += nt) d0[w] = 0;
    __syncthreads();
    if (t == 0) d0[0] = s0[0];
    for (int q = 0; q < A->n_queries; q++) {
        const nf_query& QA = A->q[q];
        const nf_query& QB = B->q[q];
        const uint64_t* s = s0 + QA.q_off;
        uint64_t* d = d0 + QB.q_off;
        for (int w = t; w < NF_QH_WORDS; w += nt) d[w] = s[w];
        for (int w = t; w < QA.n_proc * NF_PS_WORDS; w += nt) d[QB.lay.off_pstate + w] = s[QA.lay.off_pstate + w];
        for (int64_t i = t; i < (int64_t)QA.n_proc * 2 * QA.lay.list_cap; i += nt) {
            const int64_t pl = i / QA.lay.list_cap, e = i % QA.lay.list_cap;
            ((uint32_t*)(d + QB.lay.off_lists))[pl * QB.lay.list_cap + e] = ((const uint32_t*)(s + QA.lay.off_lists))[i];
        }
        for (int w = t; w < nf_agg_words(QA); w += nt) d[QB.lay.off_agg + w] = s[QA.lay.off_agg + w];
        for (int w = t; w < 3 + QA.lay.hold_cap; w += nt) d[QB.lay.off_hold + w] = s[QA.lay.off_hold + w];
        for (int p = 0; p < QA.n_proc; p++) {
            const uint64_t* sq = s + QA.lay.off_sched + (int64_t)p * (2 + QA.lay.sched_cap);
            uint64_t* dq = d + QB.lay.off_sched + (int64_t)p * (2 + QB.lay.sched_cap);
            const uint32_t head = (uint32_t)sq[0], n = (uint32_t)(sq[0] >> 32);
            if (t == 0) {
                dq[0] = (uint64_t)n << 32;
                dq[1] = sq[1];
            }
            for (uint32_t i = t; i < n; i += nt) dq[2 + i] = sq[2 + (head + i) % QA.lay.sched_cap];
        }
        for (int64_t w = t; w < (int64_t)QA.lay.se_cap * QA.lay.se_words; w += nt) d[QB.lay.off_se + w] = s[QA.lay.off_se + w];
        for (int64_t w = t; w < (int64_t)QA.lay.node_cap * 2; w += nt) d[QB.lay.off_node + w] = s[QA.lay.off_node + w];
    }
}

static inline unsigned nf_blocks(int64_t n, int tpb) { return (unsigned)((n + tpb - 1) / tpb); }

extern "C" int nfd_run(const nf_table* dT, const nf_cols* dC, uint64_t* kstate, const nfd_events* ev, int64_t n,
                       const uint32_t* seg_list, const uint32_t* nseg, const uint32_t* skeys, int32_t nkeys,
                       int64_t max_segments, uint64_t tick, int64_t clock, const nfd_emit* em, void* stream) {
    DevEvents E;
    E.ts = ev->ts;
    E.stream = ev->stream;
    E.row = ev->row;
    E.bid = ev->bid;
    E.perm = ev->perm;
    E.seq_base = ev->seq_base;
    E.batch_events = ev->batch_events;
    E.run = ev->run;
    E.gidx = ev->gidx;
    E.sts = ev->sts;
    E.sorted_rows = ev->sorted_rows;
    if (max_segments < 1) max_segments = 1;
    hipLaunchKernelGGL(k_nfa_run, dim3(nf_blocks(max_segments, NF_TPB)), dim3(NF_TPB), 0, (hipStream_t)stream, dT, dC,
                       kstate, E, n, seg_list, nseg, skeys, nkeys, tick, clock, *em);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

extern "C" int nfd_seq3(const nf_table* dT, const nf_cols* dC, const nfd_events* ev, int64_t n,
                        const uint32_t* seg_list, const uint32_t* nseg, const uint32_t* skeys, int32_t nkeys,
                        int64_t max_segments, const nfd_emit* em, void* stream, const void* s3_col, int compact,
                        int agg, int rw) {
    if (s3_col && !ev->gidx) {
        // LDS-staged (the host checked the shape: one 4-byte attribute, no nulls,
        // key-ordered copy in s3_col)
        if (max_segments < 1) max_segments = 1;
        const dim3 g(nf_blocks(max_segments, S3S_TPB)), b(S3S_TPB);
        if (compact && agg)
            hipLaunchKernelGGL((k_seq3s<true, true>), g, b, 0, (hipStream_t)stream, dT, (const uint32_t*)s3_col,
                               ev->perm, ev->seq_base, n, seg_list, nseg, skeys, nkeys, *em, rw);
        else if (compact)
            hipLaunchKernelGGL((k_seq3s<true, false>), g, b, 0, (hipStream_t)stream, dT, (const uint32_t*)s3_col,
                               ev->perm, ev->seq_base, n, seg_list, nseg, skeys, nkeys, *em, rw);
        else
            hipLaunchKernelGGL((k_seq3s<false, false>), g, b, 0, (hipStream_t)stream, dT, (const uint32_t*)s3_col,
                               ev->perm, ev->seq_base, n, seg_list, nseg, skeys, nkeys, *em, rw);
        return hipGetLastError() == hipSuccess ? 0 : -3;
    }
    DevEvents E;
    E.ts = ev->ts;
    E.stream = ev->stream;
    E.row = ev->row;
    E.bid = ev->bid;
    E.perm = ev->perm;
    E.seq_base = ev->seq_base;
    E.batch_events = ev->batch_events;
    E.run = ev->run;
    E.gidx = ev->gidx;
    E.sts = ev->sts;
    E.sorted_rows = ev->sorted_rows;
    if (max_segments < 1) max_segments = 1;
    // events per lane per load block (SH_S3_U: 4 / 8 / 16; measured)
    static const int u = [] {
        const char* e = getenv("SH_S3_U");
        const int v = e ? atoi(e) : 8;
        return v == 4 || v == 16 ? v : 8;
    }();
    const dim3 g(nf_blocks(max_segments, NF_TPB)), b(NF_TPB);
    if (u == 4)
        hipLaunchKernelGGL(k_seq3<4>, g, b, 0, (hipStream_t)stream, dT, dC, E, n, seg_list, nseg, skeys, nkeys, *em);
    else if (u == 16)
        hipLaunchKernelGGL(k_seq3<16>, g, b, 0, (hipStream_t)stream, dT, dC, E, n, seg_list, nseg, skeys, nkeys, *em);
    else
        hipLaunchKernelGGL(k_seq3<8>, g, b, 0, (hipStream_t)stream, dT, dC, E, n, seg_list, nseg, skeys, nkeys, *em);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

extern "C" int nfd_start(const nf_table* dT, const nf_cols* dC, uint64_t* kstate, uint64_t tick, int64_t clock,
                         const nfd_emit* em, void* stream) {
    hipLaunchKernelGGL(k_nfa_start, dim3(1), dim3(64), 0, (hipStream_t)stream, dT, dC, kstate, tick, clock, *em);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

extern "C" int nfd_due(const nf_table* dT, int q, int p, const uint64_t* kstate, int32_t nkeys, int64_t now,
                       nfd_cand* cand, unsigned long long* ctr, int64_t cap, uint8_t* armed, int clear_armed,
                       const uint64_t* rank, void* stream) {
    if (nkeys <= 0) return 0;
    hipLaunchKernelGGL(k_nfa_due, dim3(nf_blocks(nkeys, 256)), dim3(256), 0, (hipStream_t)stream, dT, q, p, kstate,
                       nkeys, now, cand, ctr, cap, armed, clear_armed, rank);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

extern "C" int nfd_due_list(const nf_table* dT, int q, int p, const uint64_t* kstate, const int32_t* lin,
                            const unsigned long long* lin_n, const int32_t* alog, const unsigned long long* alog_n,
                            int64_t now, nfd_cand* cand, unsigned long long* ctr, int64_t cap, uint8_t* armed,
                            int drop, const uint64_t* rank, int32_t* lout, unsigned long long* lout_n,
                            int64_t max_items, void* stream) {
    const int64_t blocks = std::min<int64_t>(std::max<int64_t>(nf_blocks(max_items, 256), 1), 2048);
    hipLaunchKernelGGL(k_nfa_due_list, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, dT, q, p, kstate,
                       lin, lin_n, alog, alog_n, now, cand, ctr, cap, armed, drop, rank, lout, lout_n);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

// the candidates' stamps from the scheduler map's ranks (host-modelled order)
__global__ void k_cand_restamp(nfd_cand* __restrict__ cand, int64_t nc, const uint64_t* __restrict__ rank) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < nc) cand[i].stamp = rank[cand[i].key];
}

extern "C" int nfd_cand_restamp(nfd_cand* cand, int64_t nc, const uint64_t* rank, void* stream) {
    if (nc <= 0) return 0;
    hipLaunchKernelGGL(k_cand_restamp, dim3(nf_blocks(nc, 256)), dim3(256), 0, (hipStream_t)stream, cand, nc, rank);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

extern "C" int nfd_cand_tmin(const nfd_cand* cand, int64_t nc, unsigned long long* tmin, void* stream) {
    if (nc <= 0) return 0;
    hipMemsetAsync(tmin, 0xFF, 8, (hipStream_t)stream);
    hipLaunchKernelGGL(k_cand_tmin, dim3(nf_blocks(nc, 256)), dim3(256), 0, (hipStream_t)stream, cand, nc, tmin);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

__global__ void k_rank_scatter(const int32_t* __restrict__ keys, const uint64_t* __restrict__ ranks, int64_t n,
                               uint64_t* __restrict__ dst) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) dst[keys[i]] = ranks[i];
}

extern "C" int nfd_rank_scatter(const int32_t* keys, const uint64_t* ranks, int64_t n, uint64_t* dst, void* stream) {
    if (n <= 0) return 0;
    hipLaunchKernelGGL(k_rank_scatter, dim3(nf_blocks(n, 256)), dim3(256), 0, (hipStream_t)stream, keys, ranks, n, dst);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

extern "C" int nfd_cand_select(const nfd_cand* cand, int64_t nc, int64_t tmin, int64_t range,
                               unsigned long long* slot_stamp, int32_t* slot_key, void* stream) {
    if (nc <= 0 || range <= 0) return 0;
    hipMemsetAsync(slot_stamp, 0xFF, (size_t)range * 8, (hipStream_t)stream);
    hipMemsetAsync(slot_key, 0xFF, (size_t)range * 4, (hipStream_t)stream);
    hipLaunchKernelGGL(k_cand_slot, dim3(nf_blocks(nc, 256)), dim3(256), 0, (hipStream_t)stream, cand, nc, tmin,
                       slot_stamp);
    hipLaunchKernelGGL(k_cand_pick, dim3(nf_blocks(nc, 256)), dim3(256), 0, (hipStream_t)stream, cand, nc, tmin,
                       slot_stamp, slot_key);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

extern "C" int nfd_timer(const nf_table* dT, const nf_cols* dC, uint64_t* kstate, int q, int p, const int32_t* keys,
                         int32_t nsel, int64_t now, uint64_t tick, int64_t clock, uint64_t seq, const nfd_emit* em,
                         void* stream, const uint32_t* gpos) {
    if (nsel <= 0) return 0;
    hipLaunchKernelGGL(k_nfa_timer, dim3(nf_blocks(nsel, NF_TPB)), dim3(NF_TPB), 0, (hipStream_t)stream, dT, dC,
                       kstate, q, p, keys, nsel, now, tick, clock, seq, *em, gpos);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

extern "C" int nfd_place(const uint64_t* recs, int64_t nrec, int stride, const uint32_t* offsets, int n_out,
                         int32_t* out_query, uint64_t* out_seq, int64_t* out_ts, int64_t* out_vals, uint8_t* out_nulls,
                         uint32_t* inv, int64_t total, void* stream) {
    if (nrec <= 0 || total <= 0) return 0;
    hipMemsetAsync(inv, 0xFF, (size_t)total * 4, (hipStream_t)stream);
    hipLaunchKernelGGL(k_nfa_inv, dim3(nf_blocks(nrec, 256)), dim3(256), 0, (hipStream_t)stream, recs, nrec, stride,
                       offsets, inv);
    hipLaunchKernelGGL(k_nfa_gather, dim3(nf_blocks(total, 256)), dim3(256), 0, (hipStream_t)stream, recs,
                       (const uint32_t*)inv, total, nrec, stride, n_out, out_query, out_seq, out_ts, out_vals, out_nulls);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

// the same placement appended to device-resident output arrays: the launch's rows
// (their count off[n-1] + cnt[n-1] read on the device) go after the *base rows
// already there, then *base grows by them -- no host round trip per launch
__global__ void __launch_bounds__(256) k_nfa_gather_app(const uint64_t* __restrict__ recs,
                                                        const uint32_t* __restrict__ inv, int64_t nrec, int stride,
                                                        int n_out, const uint32_t* __restrict__ off,
                                                        const uint32_t* __restrict__ cnt, int64_t n_idx,
                                                        const unsigned long long* __restrict__ base,
                                                        int32_t* __restrict__ out_query, uint64_t* __restrict__ out_seq,
                                                        int64_t* __restrict__ out_ts, int64_t* __restrict__ out_vals,
                                                        uint8_t* __restrict__ out_nulls) {
    const int64_t dst = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t total = (int64_t)off[n_idx - 1] + cnt[n_idx - 1];
    if (dst >= total) return;
    const uint32_t ix = inv[dst];
    if ((int64_t)ix >= nrec) return;
    const int64_t o = (int64_t)*base + dst;
    const uint64_t* r = recs + (int64_t)ix * stride;
    const uint64_t h2 = r[2];
    out_query[o] = (int)(h2 >> 32);
    out_seq[o] = r[3];
    out_ts[o] = (int64_t)r[1];
    for (int c = 0; c < n_out; c++) {
        const bool has = c < stride - NF_REC_HDR;
        out_vals[o * n_out + c] = has ? (int64_t)r[NF_REC_HDR + c] : 0;
        out_nulls[o * n_out + c] = has ? (uint8_t)((h2 >> c) & 1) : 1;
    }
}

__global__ void k_nfa_app_bump(const uint32_t* __restrict__ off, const uint32_t* __restrict__ cnt, int64_t n_idx,
                               unsigned long long* __restrict__ base) {
    *base += (unsigned long long)off[n_idx - 1] + cnt[n_idx - 1];
}

// two device ranges zeroed in one launch (4-byte multiples): a launch's match
// counts and counter block, or the due pass's counters
__global__ void k_zero2(uint32_t* __restrict__ a, int64_t na, uint32_t* __restrict__ b, int64_t nb) {
    const int64_t n = na > nb ? na : nb;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        if (i < na) a[i] = 0u;
        if (i < nb) b[i] = 0u;
    }
}

extern "C" int nfd_zero2(void* a, int64_t abytes, void* b, int64_t bbytes, void* stream) {
    const int64_t na = abytes / 4, nb = bbytes / 4, n = na > nb ? na : nb;
    if (n <= 0) return 0;
    hipLaunchKernelGGL(k_zero2, dim3(nf_blocks(n, 256) < 1024 ? nf_blocks(n, 256) : 1024), dim3(256), 0,
                       (hipStream_t)stream, (uint32_t*)a, na, (uint32_t*)b, nb);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

// the same appended placement for a small launch in ONE workgroup: the counts'
// scan, the row -> record map and the gather in LDS, the row counter bumped at the
// end (one launch instead of scan, fill, map, gather and bump)
#define NF_PS_TPB 1024
#define NF_PS_MAX 8192
__global__ void __launch_bounds__(NF_PS_TPB) k_nfa_place_small(const uint64_t* __restrict__ recs, int nrec,
                                                              int stride, const uint32_t* __restrict__ counts,
                                                              int n_idx, int n_out, unsigned long long* __restrict__ base,
                                                              int32_t* __restrict__ out_query,
                                                              uint64_t* __restrict__ out_seq,
                                                              int64_t* __restrict__ out_ts,
                                                              int64_t* __restrict__ out_vals,
                                                              uint8_t* __restrict__ out_nulls) {
    __shared__ uint32_t off[NF_PS_MAX];
    __shared__ uint32_t inv[NF_PS_MAX];
    __shared__ uint32_t ws[NF_PS_TPB / 64];
    constexpr int PER = NF_PS_MAX / NF_PS_TPB;
    const int i0 = (int)threadIdx.x * PER;
    uint32_t c[PER], sum = 0;
#pragma unroll
    for (int k = 0; k < PER; k++) {
        c[k] = i0 + k < n_idx ? counts[i0 + k] : 0u;
        sum += c[k];
    }
    uint32_t total;
    uint32_t o = shw_block_excl<NF_PS_TPB>(sum, ws, &total);
#pragma unroll
    for (int k = 0; k < PER; k++) {
        off[i0 + k] = o;
        o += c[k];
    }
    for (uint32_t d = threadIdx.x; d < total; d += NF_PS_TPB) inv[d] = 0xFFFFFFFFu;
    __syncthreads();
    for (int i = threadIdx.x; i < nrec; i += NF_PS_TPB) {
        const uint64_t tag = recs[(int64_t)i * stride];
        if (tag == ~0ull) continue;
        const uint32_t d = off[(uint32_t)tag] + (uint32_t)(tag >> 32);
        if (d < total) inv[d] = (uint32_t)i;
    }
    __syncthreads();
    const int64_t b0 = (int64_t)*base;
    for (uint32_t d = threadIdx.x; d < total; d += NF_PS_TPB) {
        const uint32_t ix = inv[d];
        if (ix >= (uint32_t)nrec) continue;
        const int64_t o2 = b0 + d;
        const uint64_t* r = recs + (int64_t)ix * stride;
        const uint64_t h2 = r[2];
        out_query[o2] = (int)(h2 >> 32);
        out_seq[o2] = r[3];
        out_ts[o2] = (int64_t)r[1];
        for (int cc = 0; cc < n_out; cc++) {
            const bool has = cc < stride - NF_REC_HDR;
            out_vals[o2 * n_out + cc] = has ? (int64_t)r[NF_REC_HDR + cc] : 0;
            out_nulls[o2 * n_out + cc] = has ? (uint8_t)((h2 >> cc) & 1) : 1;
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) *base = (unsigned long long)(b0 + total);
}

extern "C" int nfd_place_app_small(const uint64_t* recs, int64_t nrec, int stride, const uint32_t* counts,
                                   int64_t n_idx, int n_out, unsigned long long* base, int32_t* out_query,
                                   uint64_t* out_seq, int64_t* out_ts, int64_t* out_vals, uint8_t* out_nulls,
                                   void* stream) {
    if (nrec > NF_PS_MAX || n_idx > NF_PS_MAX) return -1;
    if (nrec <= 0 || n_idx <= 0) return 0;
    hipLaunchKernelGGL(k_nfa_place_small, dim3(1), dim3(NF_PS_TPB), 0, (hipStream_t)stream, recs, (int)nrec, stride,
                       counts, (int)n_idx, n_out, base, out_query, out_seq, out_ts, out_vals, out_nulls);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

extern "C" int nfd_place_app(const uint64_t* recs, int64_t nrec, int stride, const uint32_t* offsets,
                             const uint32_t* counts, int64_t n_idx, int n_out, unsigned long long* base,
                             int32_t* out_query, uint64_t* out_seq, int64_t* out_ts, int64_t* out_vals,
                             uint8_t* out_nulls, uint32_t* inv, void* stream) {
    if (nrec <= 0 || n_idx <= 0) return 0;
    hipStream_t st = (hipStream_t)stream;
    hipMemsetAsync(inv, 0xFF, (size_t)nrec * 4, st);
    hipLaunchKernelGGL(k_nfa_inv, dim3(nf_blocks(nrec, 256)), dim3(256), 0, st, recs, nrec, stride, offsets, inv);
    hipLaunchKernelGGL(k_nfa_gather_app, dim3(nf_blocks(nrec, 256)), dim3(256), 0, st, recs, (const uint32_t*)inv, nrec,
                       stride, n_out, offsets, counts, n_idx, (const unsigned long long*)base, out_query, out_seq,
                       out_ts, out_vals, out_nulls);
    hipLaunchKernelGGL(k_nfa_app_bump, dim3(1), dim3(1), 0, st, offsets, counts, n_idx, base);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

extern "C" int nfd_save(uint64_t* kstate, int64_t key_words, const uint32_t* seg_list, const uint32_t* nseg,
                        const uint32_t* skeys, int64_t max_segments, uint64_t* save, int dir, void* stream) {
    if (max_segments < 1) return 0;
    hipLaunchKernelGGL(k_nfa_save, dim3((unsigned)max_segments), dim3(256), 0, (hipStream_t)stream, kstate, key_words,
                       seg_list, nseg, skeys, save, dir);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

extern "C" int nfd_relayout(const nf_table* dA, const nf_table* dB, const uint64_t* src, uint64_t* dst, int32_t nkeys,
                            void* stream) {
    if (nkeys <= 0) return 0;
    hipLaunchKernelGGL(k_nfa_relayout, dim3((unsigned)nkeys), dim3(256), 0, (hipStream_t)stream, dA, dB, src, dst,
                       nkeys);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

extern "C" int nfd_save_keys(uint64_t* kstate, int64_t key_words, const int32_t* keys, int32_t nkeys, uint64_t* save,
                             int dir, void* stream) {
    if (nkeys < 1) return 0;
    hipLaunchKernelGGL(k_nfa_save_keys, dim3((unsigned)nkeys), dim3(256), 0, (hipStream_t)stream, kstate, key_words,
                       keys, save, dir);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}
