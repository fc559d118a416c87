// sh_nfa.h — the general per-key NFA engine of libsiddhi_hip.so.
//
// One lane per partition key replays, over that key's events in arrival order,
// the processor graph StateInputStreamParser builds for a pattern / sequence
// query (core/util/parser/StateInputStreamParser.java:76-408): Stream, Count,
// Logical and Absent pre/post state processors, `every`, `within` expiry,
// Single / Multi / Sequence receivers and the query selector with its
// aggregators. It is the device form of every §8(a) row the data-parallel window
// engine (sh_window.hip) does not cover: Kleene counts (R6), logical and/or
// (R7), sequences (R3 SequenceMulti/Single receivers), absent states and their
// event-time scheduler (R8, R10), multi-query partitions (R-order).
//
// Java object identity is observable on this path:
// next-state forwarding passes the SAME StateEvent, `every` clones are shallow
// (they share StreamEvent chains), Count `addEvent` mutates a shared chain tail,
// logical partners hold the same partials, ComplexEventChunk links events
// through their `next` field. So partials are not value records here: each key
// owns an arena of StateEvent objects and StreamEvent chain nodes in HBM, lists
// hold object ids, clones copy slot references, and unreachable objects are
// reclaimed by a per-key mark-sweep at event boundaries (reachability is what
// the JVM uses too). State holders follow PartitionSyncStateHolder: a pre-state
// whose lists are empty and that is not `initialized` is destroyed when its use
// count returns to 0 (PartitionStateHolder.java:51-65) and re-created fresh.
//
// The code is __host__ __device__: libsiddhi_hip.so runs it in k_nfa
// (sh_nfa.hip), one lane per key segment; tests/nfa_host compiles the same
// header for the CPU so its logic can be diffed against the oracle without a GPU
// (test infrastructure; the product never runs it on the host).
#pragma once
#include <stdint.h>

#include "../../include/sh_query.h"
#include "sh_program.h"

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define NF_HD __host__ __device__
#else
#define NF_HD
#endif
#define NF_INL NF_HD inline

#define NF_MAX_PROC 16
#define NF_MAX_SEQ 48
#define NF_MAX_QUERIES 16
#define NF_MAX_STREAMS 8
#define NF_MAX_ATTRS 32
#define NF_MAX_OUT 16
#define NF_MAX_CODE 2048
#define NF_MAX_CONST 256
#define NF_STACK 24

// pre-state processor kinds
enum nf_kind { NF_K_STREAM = 0, NF_K_COUNT = 1, NF_K_LOGICAL = 2, NF_K_ABSENT = 3 };
// StateEvent / ComplexEvent types (ComplexEvent.Type)
enum nf_evtype { NF_CURRENT = 0, NF_EXPIRED = 1, NF_TIMER = 2, NF_RESET = 3 };

// One pre-state processor and its post-state processor (they are 1:1). Index =
// state id = MetaStateEvent slot = position in StateStreamRuntime's
// preStateProcessor list.
struct nf_proc {
    int8_t kind;            // nf_kind
    int8_t is_start;        // StreamPreStateProcessor.isStartState
    int8_t stream;          // stream feeding this state
    int8_t within_every;    // withinEveryPreStateProcessor (proc) or -1
    int8_t this_last;       // thisLastProcessor (proc whose post marks isEventReturned)
    int8_t partner;         // Logical: partner pre (and its post), -1
    int8_t logical_type;    // SH_E_LOGICAL_AND / SH_E_LOGICAL_OR
    int8_t next_pre;        // post.nextStatePreProcessor, -1
    int8_t next_every_pre;  // post.nextEveryStatePreProcessor, -1
    int8_t callback_pre;    // post.callbackPreStateProcessor (a CountPre), -1
    int8_t to_selector;     // post.nextProcessor is the QuerySelector
    int8_t absent_logical;  // Logical: AbsentLogicalPre/PostStateProcessor (own scheduler)
    int32_t min_count, max_count;
    int64_t waiting;        // Absent / absent logical: waitingTime (ms), -1: no `for`
    int32_t filter_pc, filter_len;  // FilterProcessor between pre and post (-1: none)
};

// the pre owns a Scheduler (AbsentStreamPre / AbsentLogicalPre)
NF_INL bool nf_has_sched(const nf_proc& P) {
    return P.kind == NF_K_ABSENT || (P.kind == NF_K_LOGICAL && P.absent_logical);
}

// Per stream: the ProcessStreamReceiver of this query (StateInputStreamParser.java:91-110)
struct nf_receiver {
    int8_t present;
    int8_t multi;           // Multi (stream used by >1 state) vs Single
    int8_t n_next;          // processCount
    int8_t has_selector;    // querySelector != null
    int8_t next_procs[NF_MAX_PROC];  // nextProcessors (setNext order)
    int8_t event_seq[NF_MAX_PROC];   // eventSequence (reverse of slots)
    int8_t n_for;
    int8_t pad[3];
    int8_t for_stream[NF_MAX_PROC];  // stateProcessorsForStream
};

// per-key, per-query block layout (8-byte words)
struct nf_layout {
    int32_t list_cap;       // pending / new-and-every capacity per pre-state
    int32_t se_cap;         // StateEvent objects
    int32_t node_cap;       // StreamEvent chain nodes
    int32_t hold_cap;       // ReturnEventHolder chunks per run
    int32_t se_words;       // words per StateEvent
    int32_t sched_cap;      // Scheduler toNotify queue capacity
    int32_t group_cap;      // `group by`: aggregator groups per key
    int64_t off_pstate;     // NF_PS_WORDS per proc
    int64_t off_lists;      // per proc: pending[list_cap] then nae[list_cap] (u32 ids)
    int64_t off_agg;        // 5 words per output
    int64_t off_hold;       // retc chunk (2 words) + holder count + hold_cap x (first,last)
    int64_t off_sched;      // per proc: head/count word, registration stamp, sched_cap times
    int64_t off_se;
    int64_t off_node;       // 2 words per node: ts, row | next << 32
    int64_t words;
};

struct nf_query {
    int32_t state_type;     // SH_PATTERN / SH_SEQUENCE
    int32_t n_proc;
    int32_t n_out;
    int32_t contains_agg;
    int64_t within;         // -1: none
    int32_t n_start;
    int32_t n_init, n_reset, n_update;
    int32_t n_startup;      // startup absent pres (partitionCreated)
    int32_t n_sched;        // scheduler-owning pres, in Scheduler creation order
    int8_t sched_seq[NF_MAX_PROC];
    int8_t start_ids[NF_MAX_PROC];
    int8_t init_seq[NF_MAX_SEQ];
    int8_t reset_seq[NF_MAX_SEQ];
    int8_t update_seq[NF_MAX_SEQ];
    int8_t startup[NF_MAX_PROC];
    int8_t slot_stream[NF_MAX_PROC];
    nf_proc proc[NF_MAX_PROC];
    nf_receiver recv[NF_MAX_STREAMS];
    int32_t out_pc[NF_MAX_OUT], out_len[NF_MAX_OUT], out_agg[NF_MAX_OUT], out_type[NF_MAX_OUT];
    // List outputs (out_pc == NF_PC_LIST, SH_OP_MULTI_VAR): slot, chain index, attribute, element type
    int32_t out_mv_slot[NF_MAX_OUT], out_mv_chain[NF_MAX_OUT], out_mv_attr[NF_MAX_OUT], out_mv_type[NF_MAX_OUT];
    int32_t having_pc, having_len;  // QuerySelector havingConditionExecutor (-1: none)
    int32_t n_order, order_desc;    // OrderByEventComparator: attributes, DESC bit per attribute
    int32_t order_pc[SH_MAX_ORDER], order_len[SH_MAX_ORDER];
    int64_t limit, offset;          // QuerySelector limit / offset (-1: none)
    int32_t rate_kind, rate_value;  // OutputRateLimiter (enum sh_rate); its counter: qb[3] >> 32
    int32_t n_group;                // `group by` attributes (aggregator state per group)
    int32_t group_pc[SH_MAX_GROUP], group_len[SH_MAX_GROUP];
    nf_layout lay;
    int64_t q_off;          // word offset of this query's block inside a key block
    // rise-and-fall sequence `every e1=S, e2=S[f2(e2, e1)]+, e3=S[f3(e3, e2[last])]`
    // (no within, one stream): the per-key state reduces to one partial (k_seq3)
    int8_t s3;
    int8_t s3_op2, s3_dom2, s3_op3, s3_dom3;
    int8_t s3_a2, s3_t2, s3_e1a, s3_e1t;      // f2: x.a2 (type t2) op2 e1.e1a (type e1t)
    int8_t s3_a3, s3_t3, s3_la, s3_lt;        // f3: x.a3 (type t3) op3 last.la (type lt)
    int8_t s3_out_slot[NF_MAX_OUT], s3_out_attr[NF_MAX_OUT], s3_out_type[NF_MAX_OUT];
};

struct nf_table {
    int32_t n_queries;
    int32_t n_streams;
    int32_t partitioned;    // all queries in partition 0 (else: all unpartitioned)
    int32_t playback;
    int32_t has_absent;
    int32_t pad;
    int64_t key_words;      // words per key block: 1 header word + every query block
    int32_t stream_nattr[NF_MAX_STREAMS];
    uint32_t attr_used[NF_MAX_STREAMS];  // attributes any filter / select reads (bit per attribute)
    int8_t attr_type[NF_MAX_STREAMS][NF_MAX_ATTRS];
    int32_t n_code, n_const;
    shp_instr code[NF_MAX_CODE];
    int64_t consts[NF_MAX_CONST];
    uint8_t const_null[NF_MAX_CONST];
    uint8_t const_type[NF_MAX_CONST];
    nf_query q[NF_MAX_QUERIES];
};

// column stores the lanes read event attributes from
struct nf_cols {
    const void* col[NF_MAX_STREAMS][NF_MAX_ATTRS];
    const uint8_t* nul[NF_MAX_STREAMS][NF_MAX_ATTRS];
    // per key: set when the key registers a scheduler entry, cleared by the due
    // scan when its queues are empty, so the scan skips keys that never armed one
    // (NULL: every key is scanned)
    uint8_t* sched_armed;
    // keys whose flag went 0 -> 1 since the last due pass (the device due list
    // takes them in, sh_host_nfa.cpp nf_timers); NULL: off
    int32_t* arm_log;
    unsigned long long* arm_ctr;
    uint64_t arm_cap;
    // scheduler-map history of this launch for the host's HashMap-order model
    // (sh_jmap.h): 2 words per record, [0] processing stamp, [1] key | scheduler
    // (query * NF_MAX_PROC + proc) << 32 | kind << 48 (NF_SEV_*); NULL: off
    uint64_t* sev;
    unsigned long long* sev_ctr;
    uint64_t sev_cap;
    // this launch's List values (SH_OP_MULTI_VAR outputs): per list, word 0 the
    // length n, then n raw values, then ceil(n / 64) null-bit words; an output
    // holds the list's word offset. NULL: the app has no List output
    uint64_t* lst;
    unsigned long long* lst_ctr;
    uint64_t lst_cap;
};
#define NF_PC_LIST (-2)  // out_pc of a List output
#define NF_SEV_INSERT 0  // getState added the key (computeIfAbsent)
#define NF_SEV_CALL 1    // getState of a present key (lazy resize only)
#define NF_SEV_REMOVE 2  // queue drained: returnAllStates removes the state

// ------------------------------------------------------------------ layout
#define NF_PS_WORDS 4
// pre-state word 3 bits
#define NF_PS_ALIVE 0x1u
#define NF_PS_INIT 0x2u
#define NF_PS_STARTED 0x4u
#define NF_PS_CHANGED 0x8u
#define NF_PS_SUCCESS 0x10u
#define NF_PS_SRESET 0x20u
#define NF_PS_INACTIVE 0x40u
// query block header words
#define NF_QH_WORDS 4

NF_INL int64_t nf_round_words(int64_t bytes) { return (bytes + 7) / 8; }
// the aggregator region of a query block: the AllPerEvent limiter's held chunk
// (first, last: 2 words), then the aggregators -- 5 words per output, or with
// `group by` a table: a count word + group_cap entries of (value, null) per
// group-by attribute followed by the group's 5 words per output
// (the FirstPerTime limiter's RateLimiterState: outputTime set, outputTime: 2 words)
NF_INL int64_t nf_held_words(const nf_query& q) {
    return q.rate_kind == SH_RATE_ALL_EVENTS || q.rate_kind == SH_RATE_FIRST_TIME ? 2 : 0;
}
NF_INL int64_t nf_group_entry_words(const nf_query& q) { return 2 * (int64_t)q.n_group + (int64_t)q.n_out * 5; }
NF_INL int64_t nf_agg_words_cap(const nf_query& q, int32_t group_cap) {
    return nf_held_words(q) + (q.n_group ? 1 + (int64_t)group_cap * nf_group_entry_words(q) : (int64_t)q.n_out * 5);
}
NF_INL int64_t nf_agg_words(const nf_query& q) { return nf_agg_words_cap(q, q.lay.group_cap); }

// computes `lay` for query q with the given capacities (host side)
NF_INL void nf_set_layout(nf_query& q, int32_t n_slots, int32_t list_cap, int32_t se_cap, int32_t node_cap,
                          int32_t hold_cap, int32_t sched_cap, int32_t group_cap) {
    nf_layout& L = q.lay;
    L.group_cap = group_cap;
    L.list_cap = list_cap;
    L.se_cap = se_cap;
    L.node_cap = node_cap;
    L.hold_cap = hold_cap;
    L.sched_cap = sched_cap;
    L.se_words = 4 + (n_slots + 1) / 2 + q.n_out;
    int64_t w = NF_QH_WORDS;
    L.off_pstate = w;
    w += (int64_t)q.n_proc * NF_PS_WORDS;
    L.off_lists = w;
    w += nf_round_words((int64_t)q.n_proc * 2 * list_cap * 4);
    L.off_agg = w;
    w += nf_agg_words(q);
    L.off_hold = w;
    w += 3 + (int64_t)hold_cap;
    L.off_sched = w;
    w += (int64_t)q.n_proc * (2 + sched_cap);
    L.off_se = w;
    w += (int64_t)se_cap * L.se_words;
    L.off_node = w;
    w += (int64_t)node_cap * 2;
    L.words = w;
}

// ------------------------------------------------------------------ values
struct NfVal {
    int64_t b;
    uint8_t t;
    uint8_t null;
};

NF_INL float nf_f32(int64_t b) {
    union {
        uint32_t u;
        float f;
    } x;
    x.u = (uint32_t)b;
    return x.f;
}
NF_INL double nf_f64(int64_t b) {
    union {
        int64_t u;
        double f;
    } x;
    x.u = b;
    return x.f;
}
NF_INL int64_t nf_bf32(float f) {
    union {
        uint32_t u;
        float f;
    } x;
    x.f = f;
    return (int64_t)x.u;
}
NF_INL int64_t nf_bf64(double d) {
    union {
        int64_t u;
        double f;
    } x;
    x.f = d;
    return x.u;
}
NF_INL int64_t nf_to_i64(const NfVal& v) { return v.t == SH_T_LONG ? v.b : (int64_t)(int32_t)v.b; }
NF_INL float nf_to_f32(const NfVal& v) {
    switch (v.t) {
        case SH_T_INT: return (float)(int32_t)v.b;
        case SH_T_LONG: return (float)v.b;
        case SH_T_FLOAT: return nf_f32(v.b);
        default: return (float)nf_f64(v.b);
    }
}
NF_INL double nf_to_f64(const NfVal& v) {
    switch (v.t) {
        case SH_T_INT: return (double)(int32_t)v.b;
        case SH_T_LONG: return (double)v.b;
        case SH_T_FLOAT: return (double)nf_f32(v.b);
        default: return nf_f64(v.b);
    }
}
// Integer/Long/Float/Double/Boolean.compareTo for OrderByEventComparator (operands share
// the executor's return type): Float.compare orders -0.0 before 0.0 and NaN last
NF_INL int nf_java_compare(const NfVal& x, const NfVal& y) {
    switch (x.t) {
        case SH_T_FLOAT: {
            const float a = nf_f32(x.b), c = nf_f32(y.b);
            if (a < c) return -1;
            if (a > c) return 1;
            const int32_t ia = a != a ? 0x7fc00000 : (int32_t)nf_bf32(a);
            const int32_t ic = c != c ? 0x7fc00000 : (int32_t)nf_bf32(c);
            return ia == ic ? 0 : (ia < ic ? -1 : 1);
        }
        case SH_T_DOUBLE: {
            const double a = nf_f64(x.b), c = nf_f64(y.b);
            if (a < c) return -1;
            if (a > c) return 1;
            const int64_t ia = a != a ? 0x7ff8000000000000ll : nf_bf64(a);
            const int64_t ic = c != c ? 0x7ff8000000000000ll : nf_bf64(c);
            return ia == ic ? 0 : (ia < ic ? -1 : 1);
        }
        case SH_T_BOOL: return (int)(x.b != 0) - (int)(y.b != 0);
        default: {
            const int64_t a = nf_to_i64(x), c = nf_to_i64(y);
            return a < c ? -1 : (a > c ? 1 : 0);
        }
    }
}
template <typename T>
NF_INL bool nf_cmp_op(int op, T a, T b) {
    switch (op) {
        case SH_OP_EQ: return a == b;
        case SH_OP_NE: return a != b;
        case SH_OP_GT: return a > b;
        case SH_OP_GE: return a >= b;
        case SH_OP_LT: return a < b;
        default: return a <= b;
    }
}
// compare executors: Java binary numeric promotion of the unboxed operands
// (core/executor/condition/compare/**); ==/!= on Float/Long compare as double
NF_INL bool nf_cmp(int op, int dom, const NfVal& l, const NfVal& r) {
    switch (dom) {
        case DOM_I32: return nf_cmp_op<int32_t>(op, (int32_t)l.b, (int32_t)r.b);
        case DOM_I64: return nf_cmp_op<int64_t>(op, nf_to_i64(l), nf_to_i64(r));
        case DOM_F32: return nf_cmp_op<float>(op, nf_to_f32(l), nf_to_f32(r));
        case DOM_F64: return nf_cmp_op<double>(op, nf_to_f64(l), nf_to_f64(r));
        case DOM_BOOL: return nf_cmp_op<int>(op, l.b != 0, r.b != 0);
        default: return nf_cmp_op<int32_t>(op, (int32_t)l.b, (int32_t)r.b);
    }
}
NF_INL float nf_fmodf(float a, float b) { return __builtin_fmodf(a, b); }
NF_INL double nf_fmod(double a, double b) { return __builtin_fmod(a, b); }
// math executors (core/executor/math/**): result type fixed at parse time;
// integral and floating x/0, x%0 yield null; Java int/long wrap-around
NF_INL NfVal nf_arith(int aop, int rt, const NfVal& l, const NfVal& r) {
    NfVal o;
    o.t = (uint8_t)rt;
    o.null = 0;
    o.b = 0;
    if (l.null || r.null) {
        o.null = 1;
    } else if (rt == SH_T_INT) {
        const uint32_t a = (uint32_t)l.b, b = (uint32_t)r.b;
        const int32_t sa = (int32_t)a, sb = (int32_t)b;
        int32_t res = 0;
        switch (aop) {
            case SH_OP_ADD: res = (int32_t)(a + b); break;
            case SH_OP_SUB: res = (int32_t)(a - b); break;
            case SH_OP_MUL: res = (int32_t)(a * b); break;
            case SH_OP_DIV:
                if (sb == 0) o.null = 1;
                else res = (sa == INT32_MIN && sb == -1) ? INT32_MIN : sa / sb;
                break;
            default:
                if (sb == 0) o.null = 1;
                else res = (sb == -1) ? 0 : sa % sb;
        }
        o.b = res;
    } else if (rt == SH_T_LONG) {
        const uint64_t a = (uint64_t)nf_to_i64(l), b = (uint64_t)nf_to_i64(r);
        const int64_t sa = (int64_t)a, sb = (int64_t)b;
        int64_t res = 0;
        switch (aop) {
            case SH_OP_ADD: res = (int64_t)(a + b); break;
            case SH_OP_SUB: res = (int64_t)(a - b); break;
            case SH_OP_MUL: res = (int64_t)(a * b); break;
            case SH_OP_DIV:
                if (sb == 0) o.null = 1;
                else res = (sa == INT64_MIN && sb == -1) ? INT64_MIN : sa / sb;
                break;
            default:
                if (sb == 0) o.null = 1;
                else res = (sb == -1) ? 0 : sa % sb;
        }
        o.b = res;
    } else if (rt == SH_T_FLOAT) {
        const float a = nf_to_f32(l), b = nf_to_f32(r);
        float res = 0.f;
        switch (aop) {
            case SH_OP_ADD: res = a + b; break;
            case SH_OP_SUB: res = a - b; break;
            case SH_OP_MUL: res = a * b; break;
            case SH_OP_DIV:
                if (b == 0.0f) o.null = 1;
                else res = a / b;
                break;
            default:
                if (b == 0.0f) o.null = 1;
                else res = nf_fmodf(a, b);
        }
        o.b = nf_bf32(res);
    } else {
        const double a = nf_to_f64(l), b = nf_to_f64(r);
        double res = 0.0;
        switch (aop) {
            case SH_OP_ADD: res = a + b; break;
            case SH_OP_SUB: res = a - b; break;
            case SH_OP_MUL: res = a * b; break;
            case SH_OP_DIV:
                if (b == 0.0) o.null = 1;
                else res = a / b;
                break;
            default:
                if (b == 0.0) o.null = 1;
                else res = nf_fmod(a, b);
        }
        o.b = nf_bf64(res);
    }
    return o;
}

// ------------------------------------------------------------------ emission
// Emission record (words): [0] order tag = run-first local index | ordinal << 32,
// [1] output timestamp, [2] null mask (low 32) | query << 32, [3] trigger seq,
// [4..] raw output values.
#define NF_REC_HDR 4
// row of an empty StreamEvent (`new StreamEvent()` added by an absent logical
// state): every attribute reads as null
#define NF_ROW_NULL 0x7FFFFFFFu

// errors raised by a lane (the host grows the named capacity and replays)
enum nf_err {
    NF_OK = 0,
    NF_E_SE = 1,      // StateEvent arena full
    NF_E_NODE = 2,    // StreamEvent arena full
    NF_E_LIST = 4,    // a pending / new-and-every list full
    NF_E_HOLD = 8,    // ReturnEventHolder list full
    NF_E_SCHED = 16,  // scheduler queue full
    NF_E_EMIT = 32,   // emission buffer full
    NF_E_UNSUP = 64,  // a reference behaviour outside the lowered subset (recursion)
    NF_E_KEY = 128,   // key id out of range
    NF_E_SEV = 256,   // scheduler-history buffer full
    NF_E_LST = 512,   // List-value buffer full
    NF_E_GRP = 1024   // group-by aggregator table of a key full
};

// ------------------------------------------------------------------ the lane
// Sink: NF_HD uint64_t* slot(int words) -> record storage or nullptr (full)
template <class Sink>
struct NfLane {
    const nf_table* T;
    const nf_cols* C;
    uint64_t* kb;            // key block
    Sink* sink;
    // current query
    const nf_query* Q;
    uint64_t* qb;
    int qi;
    int partitioned;
    // transient processing state (thread-local in the reference)
    int in_holder;                   // ReturnEventHolder active (Multi receiver)
    uint32_t h_first, h_last;        // current holder's chunk
    int h_has;
    uint64_t cur_seq;                // trigger sequence of the event being processed
    uint32_t tag_index;              // run's first local index (emission order)
    uint32_t ordinal;                // emissions of this run so far
    int64_t clock;                   // playback clock (TimestampGeneratorImpl)
    uint64_t stamp;                  // processing-order stamp for scheduler registration
    uint32_t err;
    int32_t key;                     // partition key id of kb

    // StreamPostStateProcessor.isEventReturned of every post of the query: a field
    // of the processor object, so it persists across events (query header word 3)
    NF_HD bool returned(int p) const { return (qb[3] >> p) & 1; }
    NF_HD void set_returned(int p, bool v) { qb[3] = v ? (qb[3] | (1ull << p)) : (qb[3] & ~(1ull << p)); }
    // ---------------------------------------------------------- arena access
    NF_HD uint64_t* pst(int p) const { return qb + Q->lay.off_pstate + (int64_t)p * NF_PS_WORDS; }
    NF_HD uint32_t* list(int p, int which) const {
        return (uint32_t*)(qb + Q->lay.off_lists) + ((int64_t)p * 2 + which) * Q->lay.list_cap;
    }
    NF_HD uint64_t* se(uint32_t id) const { return qb + Q->lay.off_se + (int64_t)(id - 1) * Q->lay.se_words; }
    NF_HD uint64_t* node(uint32_t id) const { return qb + Q->lay.off_node + (int64_t)(id - 1) * 2; }
    // pre-state fields
    NF_HD uint32_t ps_flags(int p) const { return (uint32_t)(pst(p)[3] >> 32) & 0xFFFFu; }
    NF_HD void ps_set_flags(int p, uint32_t f) const {
        uint64_t w = pst(p)[3];
        w = (w & ~(0xFFFFull << 32)) | ((uint64_t)(f & 0xFFFFu) << 32);
        pst(p)[3] = w;
    }
    NF_HD bool ps_flag(int p, uint32_t bit) const { return (ps_flags(p) & bit) != 0; }
    NF_HD void ps_setf(int p, uint32_t bit, bool v) const {
        uint32_t f = ps_flags(p);
        ps_set_flags(p, v ? (f | bit) : (f & ~bit));
    }
    NF_HD int32_t ps_use(int p) const { return (int32_t)(int16_t)(pst(p)[3] >> 48); }
    NF_HD void ps_set_use(int p, int32_t u) const {
        uint64_t w = pst(p)[3];
        w = (w & ~(0xFFFFull << 48)) | ((uint64_t)(uint16_t)(int16_t)u << 48);
        pst(p)[3] = w;
    }
    NF_HD uint32_t lcount(int p, int which) const { return (uint32_t)(pst(p)[3] >> (which ? 16 : 0)) & 0xFFFFu; }
    NF_HD void lset(int p, int which, uint32_t n) const {
        const int sh = which ? 16 : 0;
        uint64_t w = pst(p)[3];
        w = (w & ~(0xFFFFull << sh)) | ((uint64_t)(n & 0xFFFFu) << sh);
        pst(p)[3] = w;
    }
    // `cur` chunk (currentStateEventChunk): first | last << 32 in word 1, prev | lret << 32 in word 2
    NF_HD uint32_t* cur(int p) const { return (uint32_t*)(pst(p) + 1); }

    // ---------------------------------------------------------- StateEvent fields
    NF_HD int64_t se_ts(uint32_t s) const { return (int64_t)se(s)[0]; }
    NF_HD void se_set_ts(uint32_t s, int64_t t) const { se(s)[0] = (uint64_t)t; }
    NF_HD uint32_t se_next(uint32_t s) const { return (uint32_t)se(s)[2]; }
    NF_HD void se_set_next(uint32_t s, uint32_t n) const { se(s)[2] = (se(s)[2] & ~0xFFFFFFFFull) | n; }
    NF_HD int se_type(uint32_t s) const { return (int)((se(s)[2] >> 32) & 0xFF); }
    NF_HD void se_set_type(uint32_t s, int t) const {
        se(s)[2] = (se(s)[2] & ~(0xFFull << 32)) | ((uint64_t)(t & 0xFF) << 32);
    }
    NF_HD uint32_t* se_slots(uint32_t s) const { return (uint32_t*)(se(s) + 4); }
    NF_HD uint32_t se_ev(uint32_t s, int slot) const { return se_slots(s)[slot]; }
    NF_HD void se_set_ev(uint32_t s, int slot, uint32_t n) const { se_slots(s)[slot] = n; }
    NF_HD uint64_t* se_out(uint32_t s) const { return se(s) + 4 + (Q->lay.se_words - 4 - Q->n_out); }
    // node fields
    NF_HD int64_t nd_ts(uint32_t n) const { return (int64_t)node(n)[0]; }
    NF_HD uint32_t nd_row(uint32_t n) const { return (uint32_t)node(n)[1] & 0x7FFFFFFFu; }
    NF_HD uint32_t nd_next(uint32_t n) const { return (uint32_t)(node(n)[1] >> 32); }
    NF_HD void nd_set_next(uint32_t n, uint32_t x) const {
        node(n)[1] = (node(n)[1] & 0xFFFFFFFFull) | ((uint64_t)x << 32);
    }

    // ---------------------------------------------------------- allocation
    // query header: [0] se free head | node free head << 32 (ids, 0 = none)
    //               [1] se bump | node bump << 32, [2] se live | node live << 32
    NF_HD uint32_t alloc_se() {
        uint64_t* h = qb;
        uint32_t id = (uint32_t)h[0];
        if (id) {
            h[0] = (h[0] & ~0xFFFFFFFFull) | se_next(id);
        } else {
            uint32_t bump = (uint32_t)h[1];
            if (bump >= (uint32_t)Q->lay.se_cap) {
                err |= NF_E_SE;
                return 0;
            }
            id = bump + 1;
            h[1] = (h[1] & ~0xFFFFFFFFull) | (uint64_t)(bump + 1);
        }
        h[2] += 1;
        return id;
    }
    NF_HD uint32_t alloc_node() {
        uint64_t* h = qb;
        uint32_t id = (uint32_t)(h[0] >> 32);
        if (id) {
            h[0] = (h[0] & 0xFFFFFFFFull) | ((uint64_t)nd_next(id) << 32);
        } else {
            uint32_t bump = (uint32_t)(h[1] >> 32);
            if (bump >= (uint32_t)Q->lay.node_cap) {
                err |= NF_E_NODE;
                return 0;
            }
            id = bump + 1;
            h[1] = (h[1] & 0xFFFFFFFFull) | ((uint64_t)(bump + 1) << 32);
        }
        h[2] += 1ull << 32;
        return id;
    }
    // StateEvent(nslots, nout): ts -1, CURRENT, empty slots, null outputs
    NF_HD uint32_t new_se() {
        uint32_t s = alloc_se();
        if (!s) return 0;
        uint64_t* p = se(s);
        p[0] = (uint64_t)(int64_t)-1;
        p[1] = 0;
        p[2] = 0;
        p[3] = ~0ull;
        for (int w = 4; w < Q->lay.se_words; w++) p[w] = 0;
        return s;
    }
    // StateEventCloner.copyStateEvent (StateEventCloner.java:48-59): shallow slots
    NF_HD uint32_t copy_se(uint32_t src) {
        uint32_t s = alloc_se();
        if (!s) return 0;
        uint64_t* d = se(s);
        const uint64_t* o = se(src);
        d[0] = o[0];
        d[1] = 0;
        d[2] = (uint64_t)se_type(src) << 32;
        d[3] = o[3];
        for (int w = 4; w < Q->lay.se_words; w++) d[w] = o[w];
        return s;
    }
    // StreamEventCloner.copyStreamEvent of the event being processed
    NF_HD uint32_t new_node(int64_t ts, uint32_t row) {
        uint32_t n = alloc_node();
        if (!n) return 0;
        node(n)[0] = (uint64_t)ts;
        node(n)[1] = row;
        return n;
    }

    // ---------------------------------------------------------- holders
    // PartitionSyncStateHolder.getState / returnState (PartitionStateHolder.java:36-72)
    NF_HD void pget(int p) {
        if (!ps_flag(p, NF_PS_ALIVE)) {  // fresh state object
            uint64_t* w = pst(p);
            w[0] = 0;
            w[1] = 0;
            w[2] = 0;
            w[3] = (uint64_t)NF_PS_ALIVE << 32;
        }
        if (partitioned) ps_set_use(p, ps_use(p) + 1);
    }
    NF_HD void pret(int p) {
        if (!partitioned) return;
        const int32_t u = ps_use(p) - 1;
        ps_set_use(p, u);
        if (u == 0 && cur(p)[0] == 0 && lcount(p, 0) == 0 && lcount(p, 1) == 0 && !ps_flag(p, NF_PS_INIT) &&
            !(Q->proc[p].absent_logical && pst(p)[0] != 0))
            ps_setf(p, NF_PS_ALIVE, false);  // canDestroy -> destroyed
    }

    // ---------------------------------------------------------- lists
    NF_HD bool lpush(int p, int which, uint32_t s) {
        uint32_t n = lcount(p, which);
        if (n >= (uint32_t)Q->lay.list_cap) {
            err |= NF_E_LIST;
            return false;
        }
        list(p, which)[n] = s;
        lset(p, which, n + 1);
        return true;
    }
    NF_HD void lerase(int p, int which, uint32_t i) {
        uint32_t n = lcount(p, which);
        uint32_t* l = list(p, which);
        for (uint32_t k = i + 1; k < n; k++) l[k - 1] = l[k];
        lset(p, which, n - 1);
    }
    // eventTimeComparator (StreamPreStateProcessor.java:66-80): -1 sorts last; stable
    NF_HD bool ts_less(uint32_t a, uint32_t b) const {
        const int64_t x = se_ts(a), y = se_ts(b);
        if (x == -1) return false;
        if (y == -1) return true;
        return x < y;
    }
    NF_HD void sort_nae(int p) {
        uint32_t n = lcount(p, 1);
        uint32_t* l = list(p, 1);
        for (uint32_t i = 1; i < n; i++) {
            uint32_t v = l[i];
            int32_t j = (int32_t)i - 1;
            while (j >= 0 && ts_less(v, l[j])) {
                l[j + 1] = l[j];
                j--;
            }
            l[j + 1] = v;
        }
    }
    NF_HD void splice_nae(int p) {  // pending.addAll(nae); nae.clear()
        uint32_t n = lcount(p, 1);
        uint32_t* l = list(p, 1);
        for (uint32_t i = 0; i < n; i++)
            if (!lpush(p, 0, l[i])) break;
        lset(p, 1, 0);
    }

    // ---------------------------------------------------------- chunks
    // ComplexEventChunk (event/ComplexEventChunk.java:32-282) over ids; c[0] first,
    // c[1] last, c[2] prevToLastReturned, c[3] lastReturned
    NF_HD uint32_t last_event(uint32_t evs) {
        uint32_t le = evs;
        while (le && se_next(le) && se_next(le) != evs) le = se_next(le);
        if (le && se_next(le) == evs) se_set_next(le, 0);
        return le;
    }
    NF_HD void ch_add(uint32_t* c, uint32_t evs) {
        if (!c[0])
            c[0] = evs;
        else
            se_set_next(c[1], evs);
        c[1] = last_event(evs);
    }
    NF_HD bool ch_has_next(const uint32_t* c) const {
        if (c[3]) return se_next(c[3]) != 0;
        if (c[2]) return se_next(c[2]) != 0;
        return c[0] != 0;
    }
    NF_HD uint32_t ch_next(uint32_t* c) {
        uint32_t r;
        if (c[3]) {
            r = se_next(c[3]);
            c[2] = c[3];
        } else if (c[2]) {
            r = se_next(c[2]);
        } else {
            r = c[0];
        }
        c[3] = r;
        return r;
    }
    NF_HD void ch_remove(uint32_t* c) {
        if (c[2]) {
            se_set_next(c[2], se_next(c[3]));
        } else {
            c[0] = se_next(c[3]);
            if (!c[0]) c[1] = 0;
        }
        se_set_next(c[3], 0);
        c[3] = 0;
    }
    NF_HD static void ch_clear(uint32_t* c) { c[0] = c[1] = c[2] = c[3] = 0; }
    NF_HD static void ch_reset(uint32_t* c) { c[2] = c[3] = 0; }

    // ---------------------------------------------------------- expressions
    // StateEvent.getStreamEvent(int[] position), event/state/StateEvent.java:138-182
    NF_HD uint32_t chain_at(uint32_t s, int slot, int idx) const {
        uint32_t n = se_ev(s, slot);
        if (!n) return 0;
        if (idx >= 0) {
            for (int i = 1; i <= idx; i++) {
                n = nd_next(n);
                if (!n) return 0;
            }
        } else if (idx == SH_CHAIN_CURRENT) {
            while (nd_next(n)) n = nd_next(n);
        } else if (idx == SH_CHAIN_LAST) {
            if (!nd_next(n)) return 0;
            while (nd_next(nd_next(n))) n = nd_next(n);
        } else {
            int len = 0;
            for (uint32_t x = n; x; x = nd_next(x)) len++;
            int k = len + idx;
            if (k < 0) return 0;
            for (int i = 0; i < k; i++) n = nd_next(n);
        }
        return n;
    }
    NF_HD int64_t load_attr(int s, int a, int type, uint32_t row) const {
        const void* p = C->col[s][a];
        switch (type) {
            case SH_T_LONG: return ((const int64_t*)p)[row];
            case SH_T_FLOAT: return (int64_t)((const uint32_t*)p)[row];
            case SH_T_DOUBLE: return ((const int64_t*)p)[row];
            case SH_T_BOOL: return ((const uint8_t*)p)[row] ? 1 : 0;
            default: return (int64_t)((const int32_t*)p)[row];
        }
    }
    // typed postfix program (QueryRT::eval restated as a stack machine)
    NF_HD NfVal eval(int pc, int len, uint32_t s) const {
        NfVal st[NF_STACK];
        int sp = 0;
        for (int k = 0; k < len; k++) {
            const shp_instr in = T->code[pc + k];
            switch (in.op) {
                case OPC_CONST: {
                    NfVal v;
                    v.b = T->consts[in.x];
                    v.t = T->const_type[in.x];
                    v.null = T->const_null[in.x];
                    st[sp++] = v;
                    break;
                }
                case OPC_VAR: {
                    NfVal v;
                    v.t = in.c;
                    const uint32_t n = chain_at(s, in.a, in.x);
                    if (!n) {
                        v.null = 1;
                        v.b = 0;
                    } else {
                        const int strm = Q->slot_stream[in.a];
                        const uint32_t row = nd_row(n);
                        if (row == NF_ROW_NULL) {
                            v.null = 1;
                            v.b = 0;
                        } else {
                            const uint8_t* nm = C->nul[strm][in.b];
                            v.null = nm ? nm[row] : 0;
                            v.b = load_attr(strm, in.b, in.c, row);
                        }
                    }
                    st[sp++] = v;
                    break;
                }
                case OPC_AND: {
                    NfVal r = st[--sp], l = st[--sp];
                    NfVal o;
                    o.t = SH_T_BOOL;
                    o.null = 0;
                    o.b = (!l.null && l.b && !r.null && r.b) ? 1 : 0;
                    st[sp++] = o;
                    break;
                }
                case OPC_OR: {
                    NfVal r = st[--sp], l = st[--sp];
                    NfVal o;
                    o.t = SH_T_BOOL;
                    o.null = 0;
                    o.b = ((!l.null && l.b) || (!r.null && r.b)) ? 1 : 0;
                    st[sp++] = o;
                    break;
                }
                case OPC_NOT: {
                    NfVal l = st[--sp];
                    NfVal o;
                    o.t = SH_T_BOOL;
                    o.null = 0;
                    o.b = (!l.null && l.b) ? 0 : 1;  // Not(null) = true
                    st[sp++] = o;
                    break;
                }
                case OPC_BOOLV: {
                    NfVal l = st[--sp];
                    NfVal o;
                    o.t = SH_T_BOOL;
                    o.null = 0;
                    o.b = (!l.null && l.b) ? 1 : 0;
                    st[sp++] = o;
                    break;
                }
                case OPC_ISNULL: {
                    NfVal l = st[--sp];
                    NfVal o;
                    o.t = SH_T_BOOL;
                    o.null = 0;
                    o.b = l.null ? 1 : 0;
                    st[sp++] = o;
                    break;
                }
                case OPC_ISNULL_STREAM: {
                    NfVal o;
                    o.t = SH_T_BOOL;
                    o.null = 0;
                    o.b = chain_at(s, in.a, in.x) == 0 ? 1 : 0;
                    st[sp++] = o;
                    break;
                }
                case OPC_CMP: {
                    NfVal r = st[--sp], l = st[--sp];
                    NfVal o;
                    o.t = SH_T_BOOL;
                    o.null = 0;
                    o.b = (!l.null && !r.null && nf_cmp(in.a, in.b, l, r)) ? 1 : 0;
                    st[sp++] = o;
                    break;
                }
                case OPC_ARITH: {
                    NfVal r = st[--sp], l = st[--sp];
                    st[sp++] = nf_arith(in.a, in.b, l, r);
                    break;
                }
                case OPC_SELECT: {
                    NfVal e = st[--sp], t = st[--sp], c = st[--sp];
                    st[sp++] = (!c.null && c.b) ? t : e;
                    break;
                }
                case OPC_CAST: st[sp - 1].t = in.b; break;
                case OPC_OUTPUT: {
                    // HAVING_STATE variable: the selected event's output data
                    NfVal v;
                    v.t = in.c;
                    v.b = (int64_t)se_out(s)[in.b];
                    v.null = (uint8_t)((se(s)[3] >> in.b) & 1u);
                    st[sp++] = v;
                    break;
                }
            }
        }
        return st[sp - 1];
    }

    // ---------------------------------------------------------- processors
    // StreamPreStateProcessor.isExpired (:118-129)
    NF_HD bool is_expired(uint32_t s, int64_t now) const {
        if (Q->within != -1) {
            for (int i = 0; i < Q->n_start; i++) {
                const uint32_t n = se_ev(s, Q->start_ids[i]);
                if (n) {
                    int64_t d = nd_ts(n) - now;
                    if (d < 0) d = -d;
                    if (d > Q->within) return true;
                }
            }
        }
        return false;
    }
    NF_HD void state_changed(int p) {
        pget(p);
        ps_setf(p, NF_PS_CHANGED, true);
        pret(p);
    }
    NF_HD bool pending_empty(int p) {  // getPendingStateEventList().isEmpty() (state returned first)
        if (p < 0) return true;
        pget(p);
        pret(p);
        return lcount(p, 0) == 0;
    }
    NF_HD bool next_is_absent(int p) const {
        const int np = Q->proc[p].next_pre;
        return np >= 0 && nf_has_sched(Q->proc[np]);
    }
    NF_HD bool is_alog(int p) const { return p >= 0 && Q->proc[p].kind == NF_K_LOGICAL && Q->proc[p].absent_logical; }
    // StreamPreStateProcessor.init (:178-194)
    NF_HD void init(int p) {
        const nf_proc& P = Q->proc[p];
        pget(p);
        if (P.is_start && (!ps_flag(p, NF_PS_INIT) || P.next_every_pre >= 0 ||
                           (Q->state_type == SH_SEQUENCE && next_is_absent(p)))) {
            uint32_t s = new_se();
            if (s) add_state(p, s);
            ps_setf(p, NF_PS_INIT, true);
        }
        pret(p);
    }
    // addState (:204-227) and the Count / Logical / Absent overrides.
    // CountPreStateProcessor.addState with minCount 0 calls processMinCountReached,
    // which adds the same StateEvent to the next state (and so on down a chain of
    // min-0 counts): iterative here, with an explicit stack (no device recursion).
    NF_HD void add_state(int p0, uint32_t s) {
        int8_t stk[NF_MAX_PROC + 1];
        int top = 0;
        stk[top++] = (int8_t)p0;
        bool resume = false;  // top frame returns from its nested add_state
        while (top > 0) {
            const int p = stk[top - 1];
            const nf_proc& P = Q->proc[p];
            if (resume) {
                // processMinCountReached, after nextStatePreProcessor.addState
                if (P.next_every_pre >= 0) add_every_state(P.next_every_pre, s);
                ch_clear(cur(p));
                pret(p);
                top--;
                continue;
            }
            pget(p);
            bool nested = false;
            switch (P.kind) {
                case NF_K_COUNT:
                    // CountPreStateProcessor.addState (:114-138)
                    if (Q->state_type == SH_SEQUENCE) {
                        if (lcount(p, 1) == 0) lpush(p, 1, s);
                    } else {
                        lpush(p, 1, s);
                    }
                    if (P.min_count == 0 && !se_ev(s, p)) {
                        uint32_t* c = cur(p);
                        ch_clear(c);
                        ch_add(c, s);
                        // CountPostStateProcessor.processMinCountReached (:66-78)
                        if (P.to_selector) {
                            state_changed(p);
                            ch_reset(c);
                            set_returned(p, true);
                        }
                        if (P.next_pre >= 0 && top <= NF_MAX_PROC) {
                            stk[top++] = (int8_t)P.next_pre;
                            nested = true;
                        } else {
                            if (P.next_every_pre >= 0) add_every_state(P.next_every_pre, s);
                            ch_clear(c);
                        }
                    }
                    break;
                case NF_K_LOGICAL:
                    // AbsentLogicalPreStateProcessor.addState (:78-98): inactive -> no-op
                    if (P.absent_logical && ps_flag(p, NF_PS_INACTIVE)) break;
                    // LogicalPreStateProcessor.addState (:43-66)
                    if (P.is_start || Q->state_type == SH_SEQUENCE) {
                        if (lcount(p, 1) == 0) lpush(p, 1, s);
                        if (P.partner >= 0 && nae_empty(P.partner)) add_to_nae(P.partner, s);
                    } else {
                        lpush(p, 1, s);
                        if (P.partner >= 0) add_to_nae(P.partner, s);
                    }
                    if (P.absent_logical && !P.is_start && P.waiting != -1) {
                        notify_at(p, se_ts(s) + P.waiting);
                        if (is_alog(P.partner)) notify_at(P.partner, se_ts(s) + Q->proc[P.partner].waiting);
                    }
                    break;
                case NF_K_ABSENT:
                    // AbsentStreamPreStateProcessor.addState (:95-114)
                    if (!ps_flag(p, NF_PS_INACTIVE)) {
                        if (Q->state_type == SH_SEQUENCE) {
                            lset(p, 1, 0);
                            lpush(p, 1, s);
                        } else {
                            lpush(p, 1, s);
                        }
                        if (!P.is_start) {
                            const int64_t t = se_ts(s) + P.waiting;
                            pst(p)[0] = (uint64_t)t;
                            notify_at(p, t);
                        }
                    }
                    break;
                default:
                    if (Q->state_type == SH_SEQUENCE) {
                        if (lcount(p, 1) == 0) lpush(p, 1, s);
                    } else {
                        lpush(p, 1, s);
                    }
            }
            if (nested) {
                resume = false;
                continue;
            }
            pret(p);
            top--;
            resume = top > 0;  // every frame below the top is waiting in processMinCountReached
        }
    }
    NF_HD bool nae_empty(int p) {
        pget(p);
        bool r = lcount(p, 1) == 0;
        pret(p);
        return r;
    }
    NF_HD void add_to_nae(int p, uint32_t s) {
        pget(p);
        lpush(p, 1, s);
        pret(p);
    }
    // addEveryState (:229-247; Logical :68-87; Absent :117-131)
    NF_HD void add_every_state(int p, uint32_t src) {
        const nf_proc& P = Q->proc[p];
        uint32_t c = copy_se(src);
        if (!c) return;
        se_set_type(c, NF_CURRENT);
        if (P.absent_logical) {
            // AbsentLogicalPreStateProcessor.addEveryState (:100-118): the last
            // arrived event's time, only this slot and the partner's cleared
            const uint32_t n = se_ev(c, p);
            if (n) se_set_ts(c, nd_ts(n));
            se_set_ev(c, p, 0);
            se_set_ev(c, P.partner, 0);
            pget(p);
            lpush(p, 1, c);
            add_to_nae(P.partner, c);
            pret(p);
            return;
        }
        for (int i = p; i < Q->n_proc; i++) se_set_ev(c, i, 0);
        pget(p);
        lpush(p, 1, c);
        if (P.kind == NF_K_LOGICAL && P.partner >= 0) {
            se_set_ev(c, P.partner, 0);
            add_to_nae(P.partner, c);
        }
        if (P.kind == NF_K_ABSENT) {
            const int64_t t = se_ts(src) + P.waiting;
            pst(p)[0] = (uint64_t)t;
            notify_at(p, t);
        }
        pret(p);
    }
    // resetState (:287-305; Logical :89-108; Absent :133-148)
    NF_HD void reset_state(int p) {
        const nf_proc& P = Q->proc[p];
        pget(p);
        if (P.kind == NF_K_LOGICAL) {
            bool go = P.logical_type == SH_E_LOGICAL_OR;
            if (!go) {
                pget(P.partner);
                pret(P.partner);
                go = lcount(p, 0) == lcount(P.partner, 0);
            }
            if (go) {
                lset(p, 0, 0);
                pget(P.partner);
                pret(P.partner);
                lset(P.partner, 0, 0);
                if (P.is_start && lcount(p, 1) == 0) {
                    if (Q->state_type == SH_SEQUENCE && P.next_every_pre < 0 && !pending_empty(P.next_pre)) {
                        pret(p);
                        return;
                    }
                    init(p);
                }
            }
            pret(p);
            return;
        }
        lset(p, 0, 0);
        const bool absent = P.kind == NF_K_ABSENT;
        if (P.is_start && (absent || lcount(p, 1) == 0)) {
            if (Q->state_type == SH_SEQUENCE && P.next_every_pre < 0 && !pending_empty(P.next_pre)) {
                pret(p);
                return;
            }
            init(p);
        }
        pret(p);
    }
    // updateState (:307-323; Count :181-193; Logical :110-117)
    NF_HD void update_state(int p) {
        const nf_proc& P = Q->proc[p];
        pget(p);
        if (P.kind == NF_K_COUNT && ps_flag(p, NF_PS_SRESET)) {
            ps_setf(p, NF_PS_SRESET, false);
            init(p);
        }
        sort_nae(p);
        splice_nae(p);
        if (P.kind == NF_K_LOGICAL && P.partner >= 0) {
            pget(P.partner);
            sort_nae(P.partner);
            splice_nae(P.partner);
            pret(P.partner);
        }
        pret(p);
    }
    // expireEvents (:325-361)
    NF_HD void expire_events(int p, int64_t now) {
        pget(p);
        uint32_t expired = 0;
        uint32_t* pl = list(p, 0);
        while (lcount(p, 0) > 0) {
            uint32_t s = pl[0];
            if (!is_expired(s, now)) break;
            lerase(p, 0, 0);
            if (se_type(s) != NF_EXPIRED) {
                se_set_type(s, NF_EXPIRED);
                expired = s;
            }
        }
        uint32_t* nl = list(p, 1);
        for (uint32_t i = 0; i < lcount(p, 1);) {
            uint32_t s = nl[i];
            if (is_expired(s, now)) {
                lerase(p, 1, i);
                if (se_type(s) != NF_EXPIRED) {
                    se_set_type(s, NF_EXPIRED);
                    expired = s;
                }
            } else {
                i++;
            }
        }
        const int we = Q->proc[p].within_every;
        if (expired && we >= 0) {
            add_every_state(we, expired);
            update_state(we);
        }
        pret(p);
    }
    // CountPreStateProcessor.startStateReset (:168-179)
    NF_HD void start_state_reset(int p) {
        pget(p);
        ps_setf(p, NF_PS_SRESET, true);
        if (Q->proc[p].callback_pre >= 0) err |= NF_E_UNSUP;  // the reference recurses forever here
        pret(p);
    }
    // StreamPreStateProcessor.process(StateEvent) (:131-142): pre -> [filter] -> post
    NF_HD void process_se(int p, uint32_t s) {
        pget(p);
        uint32_t* c = cur(p);
        ch_add(c, s);
        ch_reset(c);
        ps_setf(p, NF_PS_CHANGED, false);
        const nf_proc& P = Q->proc[p];
        bool go = true;
        if (P.filter_pc >= 0) {
            // FilterProcessor.process (FilterProcessor.java:48-61)
            ch_reset(c);
            while (ch_has_next(c)) {
                uint32_t ev = ch_next(c);
                NfVal r = eval(P.filter_pc, P.filter_len, ev);
                if (r.null || !r.b) ch_remove(c);
            }
            go = c[0] != 0;
        }
        if (go) {
            // PostStateProcessor.process: first event of the chunk, then clear
            ch_reset(c);
            if (ch_has_next(c)) {
                uint32_t e = ch_next(c);
                post_process(p, e, c);
            }
            ch_clear(c);
        }
        ch_reset(c);
        pret(p);
    }
    // StreamPostStateProcessor.process (:64-83)
    NF_HD void stream_post(int p, uint32_t s, uint32_t* c) {
        const nf_proc& P = Q->proc[p];
        state_changed(p);
        const uint32_t n = se_ev(s, p);
        se_set_ts(s, nd_ts(n));
        if (P.to_selector) {
            ch_reset(c);
            set_returned(p, true);
        }
        if (P.next_pre >= 0) add_state(P.next_pre, s);
        if (P.next_every_pre >= 0) add_every_state(P.next_every_pre, s);
        if (P.callback_pre >= 0) start_state_reset(P.callback_pre);
    }
    // CountPostStateProcessor.processMinCountReached (:66-78)
    NF_HD void min_count_reached(int p, uint32_t s, uint32_t* c) {
        const nf_proc& P = Q->proc[p];
        if (P.to_selector) {
            state_changed(p);
            ch_reset(c);
            set_returned(p, true);
        }
        if (P.next_pre >= 0) add_state(P.next_pre, s);
        if (P.next_every_pre >= 0) add_every_state(P.next_every_pre, s);
    }
    NF_HD void post_process(int p, uint32_t s, uint32_t* c) {
        const nf_proc& P = Q->proc[p];
        switch (P.kind) {
            case NF_K_COUNT: {
                // CountPostStateProcessor.process (:39-64)
                uint32_t n = se_ev(s, p);
                int cnt = 1;
                while (nd_next(n)) {
                    cnt++;
                    n = nd_next(n);
                }
                pget(p);
                ps_setf(p, NF_PS_SUCCESS, true);  // successCondition()
                pret(p);
                se_set_ts(s, nd_ts(n));
                if (cnt >= P.min_count) {
                    if (Q->state_type == SH_SEQUENCE) {
                        if (P.next_pre >= 0) add_state(P.next_pre, s);
                        if (cnt != P.max_count) add_state(p, s);
                    } else if (cnt == P.min_count) {
                        min_count_reached(p, s, c);
                    }
                    if (cnt == P.max_count) state_changed(p);
                }
                break;
            }
            case NF_K_LOGICAL: {
                if (P.absent_logical) {
                    // AbsentLogicalPostStateProcessor.process (:37-49): the absent
                    // event arrived
                    state_changed(p);
                    set_returned(p, true);
                    pget(p);
                    pst(p)[0] = (uint64_t)nd_ts(se_ev(s, p));  // updateLastArrivalTime
                    pret(p);
                    break;
                }
                // LogicalPostStateProcessor.process (:59-87)
                if (P.logical_type == SH_E_LOGICAL_AND) {
                    const bool go = is_alog(P.partner) ? partner_can_proceed(P.partner, s) : se_ev(s, P.partner) != 0;
                    if (go)
                        stream_post(p, s, c);
                    else
                        state_changed(p);
                } else {
                    stream_post(p, s, c);
                    if (Q->proc[P.partner].to_selector && P.this_last == P.partner) set_returned(P.partner, true);
                }
                break;
            }
            case NF_K_ABSENT: {
                // AbsentStreamPostStateProcessor.process (:36-56): the absent event
                // arrived -> the partial dies and the wait re-arms
                state_changed(p);
                const uint32_t n = se_ev(s, p);
                se_set_ts(s, nd_ts(n));
                set_returned(p, true);
                if (P.is_start && P.next_every_pre == p) add_every_state(p, s);
                pget(p);
                const int64_t t = nd_ts(n) + P.waiting;
                pst(p)[0] = (uint64_t)t;
                notify_at(p, t);
                pret(p);
                break;
            }
            default: stream_post(p, s, c);
        }
    }
    // processAndReturn (:363-403; Count :52-103; Logical :119-165; Absent :256-274)
    // returns the chunk of returned StateEvents (first id, linked through next)
    NF_HD uint32_t process_and_return(int p, int64_t ts, uint32_t row) {
        const nf_proc& P = Q->proc[p];
        if (P.absent_logical) return alog_process_and_return(p, ts, row);
        uint32_t ret[4] = {0, 0, 0, 0};
        pget(p);
        if (P.kind == NF_K_ABSENT && ps_flag(p, NF_PS_INACTIVE)) {
            pret(p);
            return 0;
        }
        uint32_t* pl = list(p, 0);
        for (uint32_t i = 0; i < lcount(p, 0);) {
            uint32_t s = pl[i];
            if (P.kind == NF_K_COUNT) {
                bool removed = false;
                for (int pos = p + 1; pos <= p + 2; pos++) {
                    if (pos < Q->n_proc && se_ev(s, pos)) {
                        lerase(p, 0, i);
                        removed = true;
                        break;
                    }
                }
                if (removed) continue;
                // StateEvent.addEvent (StateEvent.java:212-222)
                uint32_t ne = new_node(ts, row);
                if (!ne) break;
                uint32_t h = se_ev(s, p);
                if (!h) {
                    se_set_ev(s, p, ne);
                } else {
                    while (nd_next(h)) h = nd_next(h);
                    nd_set_next(h, ne);
                }
                ps_setf(p, NF_PS_SUCCESS, false);
                process_se(p, s);
                const int tl = P.this_last;
                if (returned(tl)) {
                    set_returned(tl, false);
                    ch_add(ret, s);
                }
                bool erased = false;
                if (ps_flag(p, NF_PS_CHANGED)) {
                    lerase(p, 0, i);
                    erased = true;
                }
                if (!ps_flag(p, NF_PS_SUCCESS)) {
                    // StateEvent.removeLastEvent (StateEvent.java:224-236)
                    uint32_t t = se_ev(s, p);
                    if (t) {
                        bool done = false;
                        while (nd_next(t)) {
                            if (!nd_next(nd_next(t))) {
                                nd_set_next(t, 0);
                                done = true;
                                break;
                            }
                            t = nd_next(t);
                        }
                        if (!done) se_set_ev(s, p, 0);
                    }
                    if (Q->state_type == SH_SEQUENCE && !erased) {
                        lerase(p, 0, i);
                        erased = true;
                    }
                }
                if (!erased) i++;
                continue;
            }
            if (P.kind == NF_K_LOGICAL && P.logical_type == SH_E_LOGICAL_OR && se_ev(s, P.partner)) {
                lerase(p, 0, i);
                continue;
            }
            uint32_t ne = new_node(ts, row);
            if (!ne) break;
            se_set_ev(s, p, ne);
            process_se(p, s);
            const int tl = P.this_last;
            if (returned(tl)) {
                set_returned(tl, false);
                ch_add(ret, s);
            }
            if (ps_flag(p, NF_PS_CHANGED)) {
                lerase(p, 0, i);
            } else {
                se_set_ev(s, p, 0);
                if (Q->state_type == SH_PATTERN) {
                    i++;
                } else if (P.kind == NF_K_LOGICAL) {
                    lerase(p, 0, i);
                } else {
                    // SEQUENCE: Stream removes, Absent keeps (removeOnNoStateChange)
                    if (P.kind == NF_K_ABSENT)
                        i++;
                    else
                        lerase(p, 0, i);
                    if (P.kind != NF_K_LOGICAL && P.callback_pre >= 0) start_state_reset(P.callback_pre);
                }
            }
        }
        pret(p);
        if (P.kind == NF_K_ABSENT) return 0;  // AbsentStreamPreStateProcessor returns an empty chunk
        return ret[0];
    }

    // ---------------------------------------------------------- selector
    // QuerySelector.processNoGroupBy / processInBatchNoGroupBy (:161-205, :271-313)
    // with the Sum/Avg/Count/Max/Min aggregators (per partition key)
    // MultiValueVariableFunctionExecutor.execute (MultiValueVariableFunctionExecutor.java:62-70):
    // the attribute of getStreamEvent(position) and of every later event of its
    // chain, into this launch's List buffer; returns the list's word offset
    NF_HD uint64_t collect_list(uint32_t s, int o) {
        const int slot = Q->out_mv_slot[o], a = Q->out_mv_attr[o], ty = Q->out_mv_type[o];
        const uint32_t first = chain_at(s, slot, Q->out_mv_chain[o]);
        uint64_t n = 0;
        for (uint32_t x = first; x; x = nd_next(x)) n++;
        const uint64_t words = 1 + n + (n + 63) / 64;
        if (!C || !C->lst) {
            err |= NF_E_UNSUP;
            return 0;
        }
#if defined(__HIP_DEVICE_COMPILE__)
        const unsigned long long at = atomicAdd(C->lst_ctr, (unsigned long long)words);
#else
        const unsigned long long at = *C->lst_ctr;
        *C->lst_ctr += words;
#endif
        if (at + words > C->lst_cap) {
            err |= NF_E_LST;
            return 0;
        }
        uint64_t* L = C->lst + at;
        L[0] = n;
        for (uint64_t w = 0; w < (n + 63) / 64; w++) L[1 + n + w] = 0;
        const int strm = Q->slot_stream[slot];
        uint64_t i = 0;
        for (uint32_t x = first; x; x = nd_next(x), i++) {
            const uint32_t row = nd_row(x);
            const uint8_t* nm = C->nul[strm][a];
            const bool nul = row == NF_ROW_NULL || (nm && nm[row]);
            L[1 + i] = nul ? 0 : (uint64_t)load_attr(strm, a, ty, row);
            if (nul) L[1 + n + i / 64] |= 1ull << (i % 64);
        }
        return (uint64_t)at;
    }

    // the aggregator words of the state event's group (`group by`): GroupByKeyGenerator's
    // key (the group-by values' toString(), GroupByKeyGenerator.java:60-71) compared as
    // (value, null) pairs with every NaN of a type alike; a new group takes a fresh entry
    NF_HD uint64_t* group_aggs(uint32_t s) {
        uint64_t* tab = qb + Q->lay.off_agg + nf_held_words(*Q);
        const int ng = Q->n_group;
        uint64_t g[2 * SH_MAX_GROUP];
        for (int i = 0; i < ng; i++) {
            const NfVal v = eval(Q->group_pc[i], Q->group_len[i], s);
            uint64_t b = v.null ? 0ull : (uint64_t)v.b;
            if (!v.null && v.t == SH_T_FLOAT && (b & 0x7F800000ull) == 0x7F800000ull && (b & 0x7FFFFFull)) b = 0x7FC00000ull;
            if (!v.null && v.t == SH_T_DOUBLE && (b & 0x7FF0000000000000ull) == 0x7FF0000000000000ull &&
                (b & 0xFFFFFFFFFFFFFull))
                b = 0x7FF8000000000000ull;
            g[2 * i] = b;
            g[2 * i + 1] = v.null ? 1ull : 0ull;
        }
        const int64_t E = nf_group_entry_words(*Q);
        const uint64_t n = tab[0];
        for (uint64_t e = 0; e < n; e++) {
            uint64_t* ent = tab + 1 + e * E;
            bool same = true;
            for (int i = 0; i < 2 * ng && same; i++) same = ent[i] == g[i];
            if (same) return ent + 2 * ng;
        }
        if (n >= (uint64_t)Q->lay.group_cap) {
            err |= NF_E_GRP;
            return nullptr;
        }
        uint64_t* ent = tab + 1 + n * E;
        for (int i = 0; i < 2 * ng; i++) ent[i] = g[i];
        for (int64_t w = 2 * ng; w < E; w++) ent[w] = 0;
        tab[0] = n + 1;
        return ent + 2 * ng;
    }

    NF_HD void populate(uint32_t s) {
        uint64_t* agg = qb + Q->lay.off_agg + nf_held_words(*Q);
        if (Q->n_group && Q->contains_agg) {
            agg = group_aggs(s);
            if (!agg) return;
        }
        uint64_t* out = se_out(s);
        uint64_t mask = se(s)[3];
        for (int o = 0; o < Q->n_out; o++) {
            if (Q->out_pc[o] == NF_PC_LIST) {
                out[o] = collect_list(s, o);
                mask &= ~(1ull << o);
                continue;
            }
            const int ak = Q->out_agg[o];
            if (ak == SH_AGG_NONE) {
                NfVal v = eval(Q->out_pc[o], Q->out_len[o], s);
                out[o] = (uint64_t)v.b;
                mask = v.null ? (mask | (1ull << o)) : (mask & ~(1ull << o));
                continue;
            }
            const bool add = se_type(s) == NF_CURRENT;
            NfVal arg;
            if (Q->out_pc[o] >= 0) {
                arg = eval(Q->out_pc[o], Q->out_len[o], s);
            } else {
                arg.b = 1;
                arg.t = SH_T_BOOL;
                arg.null = 0;
            }
            uint64_t* a = agg + o * 5;
            double dsum = nf_f64((int64_t)a[0]);
            int64_t lsum = (int64_t)a[1];
            int64_t cnt = (int64_t)a[2];
            int64_t rb = 0;
            bool rnull = false;
            switch (ak) {
                case SH_AGG_SUM:
                    if (!arg.null) {
                        if (arg.t == SH_T_INT || arg.t == SH_T_LONG) {
                            lsum += add ? nf_to_i64(arg) : -nf_to_i64(arg);
                        } else {
                            dsum += add ? nf_to_f64(arg) : -nf_to_f64(arg);
                        }
                        cnt += add ? 1 : -1;
                    }
                    if (cnt == 0 && !add) {
                        rnull = true;
                    } else {
                        rb = Q->out_type[o] == SH_T_LONG ? lsum : nf_bf64(dsum);
                    }
                    break;
                case SH_AGG_AVG:
                    if (!arg.null) {
                        dsum += add ? nf_to_f64(arg) : -nf_to_f64(arg);
                        cnt += add ? 1 : -1;
                    }
                    if (cnt == 0)
                        rnull = true;
                    else
                        rb = nf_bf64(dsum / (double)cnt);
                    break;
                case SH_AGG_COUNT:
                    cnt += add ? 1 : -1;
                    rb = cnt;
                    break;
                default: {  // MAX / MIN: the max/min value keeps its own type
                    const bool mnull = a[4] == 0;  // a[4]: 1 = has value
                    if (!arg.null && add) {
                        bool better = mnull;
                        if (!better) {
                            NfVal m;
                            m.b = (int64_t)a[3];
                            m.t = (uint8_t)(a[4] >> 8);
                            m.null = 0;
                            int dom;
                            const int lt = arg.t, rt = m.t;
                            if (lt == SH_T_DOUBLE || rt == SH_T_DOUBLE)
                                dom = DOM_F64;
                            else if (lt == SH_T_FLOAT || rt == SH_T_FLOAT)
                                dom = DOM_F32;
                            else if (lt == SH_T_LONG || rt == SH_T_LONG)
                                dom = DOM_I64;
                            else
                                dom = DOM_I32;
                            better = nf_cmp(ak == SH_AGG_MAX ? SH_OP_GT : SH_OP_LT, dom, arg, m);
                        }
                        if (better) {
                            a[3] = (uint64_t)arg.b;
                            a[4] = 1 | ((uint64_t)arg.t << 8);
                        }
                    }
                    rnull = a[4] == 0;
                    rb = (int64_t)a[3];
                }
            }
            a[0] = (uint64_t)nf_bf64(dsum);
            a[1] = (uint64_t)lsum;
            a[2] = (uint64_t)cnt;
            out[o] = (uint64_t)rb;
            mask = rnull ? (mask | (1ull << o)) : (mask & ~(1ull << o));
        }
        se(s)[3] = mask;
    }
    NF_HD void set_sel_seq(uint32_t s) { se(s)[1] = cur_seq; }
    // havingConditionExecutor.execute (ConditionExpressionExecutor: null is false)
    NF_HD bool having_ok(uint32_t s) const {
        if (Q->having_pc < 0) return true;
        const NfVal v = eval(Q->having_pc, Q->having_len, s);
        return !v.null && v.b;
    }
    // OrderByEventComparator.compare (OrderByEventComparator.java:62-116): nulls after
    // values whatever the direction
    NF_HD int order_compare(uint32_t a, uint32_t b) const {
        for (int i = 0; i < Q->n_order; i++) {
            const NfVal x = eval(Q->order_pc[i], Q->order_len[i], a);
            const NfVal y = eval(Q->order_pc[i], Q->order_len[i], b);
            if (!x.null && !y.null) {
                int r = nf_java_compare(x, y);
                if ((Q->order_desc >> i) & 1) r = -r;
                if (r) return r;
            } else if (!x.null) {
                return -1;
            } else if (!y.null) {
                return 1;
            }
        }
        return 0;
    }
    // QuerySelector.orderEventChunk (:452-483): each run of one event type is sorted
    // with List.sort (stable); here a stable insertion sort of the linked chunk
    NF_HD void order_chunk(uint32_t* c) {
        uint32_t head = 0, tail = 0, run_prev = 0;  // run_prev: node before the current run
        int run_type = -1;
        uint32_t ev = c[0];
        while (ev) {
            const uint32_t nx = se_next(ev);
            se_set_next(ev, 0);
            const int ty = se_type(ev);
            if (ty != run_type) {
                run_type = ty;
                run_prev = tail;
            }
            // first node of the run that orders strictly after ev
            uint32_t prev = run_prev, cur = run_prev ? se_next(run_prev) : head;
            while (cur && order_compare(cur, ev) <= 0) {
                prev = cur;
                cur = se_next(cur);
            }
            se_set_next(ev, cur);
            if (prev)
                se_set_next(prev, ev);
            else
                head = ev;
            if (!cur) tail = ev;
            ev = nx;
        }
        c[0] = head;
        c[1] = tail;
        c[2] = c[3] = 0;
    }
    // QuerySelector.offsetEventChunk (:502-519), insert into: currentOn only
    NF_HD void offset_chunk(uint32_t* c) {
        ch_reset(c);
        int64_t n = 0;
        while (ch_has_next(c)) {
            const uint32_t ev = ch_next(c);
            const int ty = se_type(ev);
            if (ty == NF_CURRENT || ty == NF_EXPIRED) {
                if (Q->offset > n) {
                    if (ty == NF_CURRENT) n++;
                    ch_remove(c);
                } else {
                    break;
                }
            }
        }
    }
    // QuerySelector.limitEventChunk (:485-500), insert into: currentOn only
    NF_HD void limit_chunk(uint32_t* c) {
        ch_reset(c);
        int64_t n = 0;
        while (ch_has_next(c)) {
            const uint32_t ev = ch_next(c);
            const int ty = se_type(ev);
            if (ty == NF_CURRENT || ty == NF_EXPIRED) {
                if (Q->limit > n && ty == NF_CURRENT)
                    n++;
                else
                    ch_remove(c);
            }
        }
    }
    // the query's OutputRateLimiter.process with its counter per partition:
    // FirstPerEventOutputRateLimiter (FirstPerEventOutputRateLimiter.java:47-72) keeps an
    // event when the counter reaches 1 and resets at N (with N = 1 it never resets, as in
    // the reference: only the first event ever passes); LastPerEventOutputRateLimiter
    // (LastPerEventOutputRateLimiter.java:45-68) keeps every N-th current event
    NF_HD void rate_send(uint32_t* c) {
        if (Q->rate_kind == SH_RATE_FIRST_TIME) {
            // FirstPerTimeOutputRateLimiter.process (FirstPerTimeOutputRateLimiter.java:53-75):
            // the chunk's first event passes when the partition's outputTime is unset or
            // outputTime + T <= the playback clock, which becomes the new outputTime
            uint64_t* hw = qb + Q->lay.off_agg;
            if (hw[0] != 0 && (int64_t)(hw[1] + (uint64_t)(int64_t)Q->rate_value) > clock) return;
            hw[0] = 1;
            hw[1] = (uint64_t)clock;
            ch_reset(c);
            const uint32_t ev = ch_next(c);
            ch_remove(c);
            uint32_t out[4] = {0, 0, 0, 0};
            ch_add(out, ev);
            ch_reset(out);
            send_to_callbacks(out);
            return;
        }
        if (Q->rate_kind == SH_RATE_ALL_EVENTS) {
            // AllPerEventOutputRateLimiter.process (AllPerEventOutputRateLimiter.java:48-75): every
            // current / expired event joins the held chunk (key block, after the
            // aggregators); the N-th releases it as one chunk
            uint64_t* hw = qb + Q->lay.off_agg;
            uint32_t held[4] = {(uint32_t)hw[0], (uint32_t)hw[1], 0, 0};
            uint32_t out[4] = {0, 0, 0, 0};
            uint32_t cnt = (uint32_t)(qb[3] >> 32);
            ch_reset(c);
            while (ch_has_next(c)) {
                const uint32_t ev = ch_next(c);
                const int ty = se_type(ev);
                if (ty != NF_CURRENT && ty != NF_EXPIRED) continue;
                ch_remove(c);
                ch_add(held, ev);
                if (++cnt == (uint32_t)Q->rate_value) {
                    ch_add(out, held[0]);
                    ch_clear(held);
                    cnt = 0;
                }
            }
            hw[0] = held[0];
            hw[1] = held[1];
            qb[3] = (qb[3] & 0xFFFFFFFFull) | ((uint64_t)cnt << 32);
            ch_reset(out);
            if (ch_has_next(out)) send_to_callbacks(out);
            return;
        }
        if (Q->rate_kind == SH_RATE_FIRST_EVENTS || Q->rate_kind == SH_RATE_LAST_EVENTS) {
            const bool first = Q->rate_kind == SH_RATE_FIRST_EVENTS;
            uint32_t cnt = (uint32_t)(qb[3] >> 32);
            ch_reset(c);
            while (ch_has_next(c)) {
                const uint32_t ev = ch_next(c);
                if (first) {
                    cnt++;
                    if (cnt == 1u) continue;
                    if (cnt == (uint32_t)Q->rate_value) cnt = 0;
                } else {
                    const int ty = se_type(ev);
                    if ((ty == NF_CURRENT || ty == NF_EXPIRED) && ++cnt == (uint32_t)Q->rate_value) {
                        cnt = 0;
                        continue;
                    }
                }
                ch_remove(c);
            }
            qb[3] = (qb[3] & 0xFFFFFFFFull) | ((uint64_t)cnt << 32);
            ch_reset(c);
            if (!ch_has_next(c)) return;
        }
        send_to_callbacks(c);
    }
    NF_HD void selector_process(uint32_t* c) {
        if (Q->contains_agg) {
            // processInBatchNoGroupBy (QuerySelector.java:271-313): the last event
            // that passes `having` is the chunk's output
            ch_reset(c);
            uint32_t last = 0;
            while (ch_has_next(c)) {
                uint32_t ev = ch_next(c);
                const int ty = se_type(ev);
                if (ty == NF_CURRENT || ty == NF_EXPIRED) {
                    populate(ev);
                    set_sel_seq(ev);
                    if (having_ok(ev) && ty == NF_CURRENT) {
                        ch_remove(c);
                        last = ev;
                    }
                }
            }
            if (last) {
                ch_clear(c);
                ch_add(c, last);
                rate_send(c);
            }
            return;
        }
        ch_reset(c);
        while (ch_has_next(c)) {
            uint32_t ev = ch_next(c);
            const int ty = se_type(ev);
            if (ty == NF_CURRENT || ty == NF_EXPIRED) {
                populate(ev);
                set_sel_seq(ev);
                // insert into: current events only; events failing `having` leave the chunk
                if (ty != NF_CURRENT || !having_ok(ev)) ch_remove(c);
            } else if (ty == NF_TIMER) {
                ch_remove(c);
            }
        }
        if (Q->n_order > 0) order_chunk(c);
        if (Q->offset >= 0) offset_chunk(c);
        if (Q->limit >= 0) limit_chunk(c);
        ch_reset(c);
        if (ch_has_next(c)) rate_send(c);
    }
    // OutputRateLimiter.sendToCallBacks (OutputRateLimiter.java:63-106)
    NF_HD void send_to_callbacks(uint32_t* c) {
        if (in_holder) {
            uint32_t hc[4] = {h_first, h_last, 0, 0};
            ch_add(hc, c[0]);
            h_first = hc[0];
            h_last = hc[1];
            h_has = 1;
            return;
        }
        emit_chunk(c);
    }
    NF_HD void emit_chunk(uint32_t* c) {
        if (!c[0]) return;
        ch_reset(c);
        while (ch_has_next(c)) {
            uint32_t ev = ch_next(c);
            if (se_type(ev) == NF_EXPIRED)
                se_set_type(ev, NF_CURRENT);
            else if (se_type(ev) == NF_RESET)
                ch_remove(c);
        }
        for (uint32_t ev = c[0]; ev; ev = se_next(ev)) {
            uint64_t* r = sink->slot(NF_REC_HDR + Q->n_out);
            const uint32_t ord = ordinal++;
            if (!r) {
                err |= NF_E_EMIT;
                continue;
            }
            r[0] = (uint64_t)tag_index | ((uint64_t)ord << 32);
            r[1] = (uint64_t)se_ts(ev);
            r[2] = (se(ev)[3] & 0xFFFFFFFFull) | ((uint64_t)(uint32_t)qi << 32);
            r[3] = se(ev)[1];
            const uint64_t* o = se_out(ev);
            for (int k = 0; k < Q->n_out; k++) r[NF_REC_HDR + k] = o[k];
        }
    }

    // ---------------------------------------------------------- scheduler
    // Scheduler.notifyAt (util/Scheduler.java:113-127, event-time mode): the key's
    // FIFO queue of notification times for absent pre-state p. Word 1 of the
    // queue marks the key's presence in the scheduler's state map (set by the
    // getState that adds it, cleared when onTimeChange's returnAllStates drops
    // the drained state); every getState is recorded for the host's model of
    // that map's iteration order (sh_jmap.h), which ranks the keys for the
    // one-state-per-due-time pick.
    NF_HD uint64_t* sched(int p) const { return qb + Q->lay.off_sched + (int64_t)p * (2 + Q->lay.sched_cap); }
    NF_HD void sched_record(int p, int kind) {
        if (!C || !C->sev || !partitioned) return;
#if defined(__HIP_DEVICE_COMPILE__)
        const unsigned long long at = atomicAdd(C->sev_ctr, 1ull);
#else
        const unsigned long long at = (*C->sev_ctr)++;
#endif
        if (at >= C->sev_cap) {
            err |= NF_E_SEV;
            return;
        }
        C->sev[2 * at] = stamp;
        C->sev[2 * at + 1] = (uint64_t)(uint32_t)key | ((uint64_t)(qi * NF_MAX_PROC + p) << 32) | ((uint64_t)kind << 48);
    }
    NF_HD void notify_at(int p, int64_t t) {
        uint64_t* q = sched(p);
        uint32_t head = (uint32_t)q[0], n = (uint32_t)(q[0] >> 32);
        if (n >= (uint32_t)Q->lay.sched_cap) {
            err |= NF_E_SCHED;
            return;
        }
        const bool added = !(q[1] >> 63);
        if (added) q[1] = (1ull << 63) | (stamp & ~(1ull << 63));
        sched_record(p, added ? NF_SEV_INSERT : NF_SEV_CALL);
        q[2 + (head + n) % Q->lay.sched_cap] = (uint64_t)t;
        q[0] = (uint64_t)head | ((uint64_t)(n + 1) << 32);
        if (C && C->sched_armed && !C->sched_armed[key]) {
            C->sched_armed[key] = 1;
            if (C->arm_log) {
#if defined(__HIP_DEVICE_COMPILE__)
                const unsigned long long at = atomicAdd(C->arm_ctr, 1ull);
#else
                const unsigned long long at = (*C->arm_ctr)++;
#endif
                if (at < C->arm_cap) C->arm_log[at] = key;  // one entry per key per episode: never full
            }
        }
    }
    NF_HD bool sched_head(int p, int64_t* t) const {
        const uint64_t* q = sched(p);
        uint32_t head = (uint32_t)q[0], n = (uint32_t)(q[0] >> 32);
        if (!n) return false;
        *t = (int64_t)q[2 + head];
        return true;
    }
    NF_HD void sched_pop(int p) {
        uint64_t* q = sched(p);
        uint32_t head = (uint32_t)q[0], n = (uint32_t)(q[0] >> 32);
        if (!n) return;
        head = (head + 1) % Q->lay.sched_cap;
        q[0] = (uint64_t)head | ((uint64_t)(n - 1) << 32);
    }
    // AbsentStreamPreStateProcessor.partitionCreated (:303-314)
    NF_HD void partition_created(int p) {
        const nf_proc& P = Q->proc[p];
        pget(p);
        if (!ps_flag(p, NF_PS_STARTED)) {
            ps_setf(p, NF_PS_STARTED, true);
            if (P.is_start && P.waiting != -1 && !ps_flag(p, NF_PS_INACTIVE)) {
                const int64_t t = clock + P.waiting;
                if (!P.absent_logical) pst(p)[0] = (uint64_t)t;  // AbsentLogical (:333-351): no lastArrivalTime
                notify_at(p, t);
            }
        }
        pret(p);
    }
    // AbsentStreamPreStateProcessor.process(ComplexEventChunk) for a TIMER event
    // at `now` (:150-227)
    NF_HD void process_timer(int p, int64_t now) {
        const nf_proc& P = Q->proc[p];
        if (P.absent_logical) {
            alog_process_timer(p, now);
            return;
        }
        pget(p);
        if (ps_flag(p, NF_PS_INACTIVE)) {
            pret(p);
            return;
        }
        uint32_t retc[4] = {0, 0, 0, 0};
        bool initialize = P.is_start && lcount(p, 1) == 0 && lcount(p, 0) == 0;
        if (initialize && Q->state_type == SH_SEQUENCE && P.next_every_pre < 0 && (int64_t)pst(p)[0] > 0)
            initialize = false;
        if (initialize) {
            uint32_t s = new_se();
            if (s) add_state(p, s);
        } else if (Q->state_type == SH_SEQUENCE && lcount(p, 1) != 0) {
            reset_state(p);
        }
        update_state(p);
        uint32_t* pl = list(p, 0);
        for (uint32_t i = 0; i < lcount(p, 0);) {
            uint32_t ev = pl[i];
            if (is_expired(ev, now)) {
                lerase(p, 0, i);
                if (P.within_every >= 0 && P.next_every_pre != p && P.next_every_pre >= 0)
                    add_every_state(P.next_every_pre, ev);
                continue;
            }
            const int64_t ets = se_ts(ev);
            if ((ets == -1 && now >= (int64_t)pst(p)[0]) || (ets != -1 && now >= ets + P.waiting)) {
                lerase(p, 0, i);
                se_set_ts(ev, now);
                ch_add(retc, ev);
                continue;
            }
            i++;
        }
        if (P.within_every >= 0) update_state(P.within_every);
        const bool not_processed = retc[0] == 0;
        while (ch_has_next(retc)) {
            uint32_t s = ch_next(retc);
            ch_remove(retc);
            absent_send(p, s);
        }
        if (clock > P.waiting + now) pst(p)[0] = (uint64_t)(clock + P.waiting);
        if (not_processed && (int64_t)pst(p)[0] < now) {
            const int64_t t = now + P.waiting;
            pst(p)[0] = (uint64_t)t;
            notify_at(p, t);
        }
        pret(p);
    }
    // AbsentStreamPreStateProcessor.sendEvent (:229-254): straight to the selector
    NF_HD void absent_send(int p, uint32_t s) {
        const nf_proc& P = Q->proc[p];
        if (P.to_selector) {
            uint32_t c[4] = {s, s, 0, 0};
            selector_process(c);
        }
        if (P.next_pre >= 0) add_state(P.next_pre, s);
        if (P.next_every_pre >= 0)
            add_every_state(P.next_every_pre, s);
        else if (P.is_start)
            ps_setf(p, NF_PS_INACTIVE, true);
        if (P.callback_pre >= 0) start_state_reset(P.callback_pre);
    }
    // ---------------------------------------------------------- absent logical
    // AbsentLogicalPreStateProcessor (query/input/stream/state/
    // AbsentLogicalPreStateProcessor.java): a LogicalPre whose element is `not S
    // [for T]`; its state word 0 is lastArrivalTime, INACTIVE is !active.
    // StateEvent.addEvent(slot, new StreamEvent()) (StateEvent.java:212-222)
    NF_HD void add_empty_event(uint32_t s, int slot) {
        const uint32_t ne = new_node(-1, NF_ROW_NULL);
        if (!ne) return;
        uint32_t h = se_ev(s, slot);
        if (!h) {
            se_set_ev(s, slot, ne);
            return;
        }
        while (nd_next(h)) h = nd_next(h);
        nd_set_next(h, ne);
    }
    // :220-228
    NF_HD bool alog_waiting_passed(int p, int64_t now, uint32_t s) const {
        const uint32_t n = se_ev(s, p);
        if (!n) return now >= se_ts(s) + Q->proc[p].waiting;
        return now >= nd_ts(n) + Q->proc[p].waiting;  // re-added by `every`
    }
    // :120-209 (a TIMER event at `now`)
    NF_HD void alog_process_timer(int p, int64_t now) {
        const nf_proc& P = Q->proc[p];
        pget(p);
        if (ps_flag(p, NF_PS_INACTIVE)) {
            pret(p);
            return;
        }
        bool not_processed = true;
        if (now >= (int64_t)pst(p)[0] + P.waiting) {
            if (P.is_start && Q->state_type == SH_SEQUENCE && lcount(p, 1) == 0 && lcount(p, 0) == 0) {
                uint32_t s = new_se();
                if (s) add_state(p, s);
            } else if (Q->state_type == SH_SEQUENCE && lcount(p, 1) != 0) {
                reset_state(p);
            }
            update_state(p);
            uint32_t retc[4] = {0, 0, 0, 0};
            uint32_t expired = 0;
            uint32_t* pl = list(p, 0);
            for (uint32_t i = 0; i < lcount(p, 0);) {
                const uint32_t ev = pl[i];
                if (is_expired(ev, now)) {
                    expired = ev;
                    lerase(p, 0, i);
                    continue;
                }
                if (alog_waiting_passed(p, now, ev)) {
                    lerase(p, 0, i);
                    const bool partner_in = se_ev(ev, P.partner) != 0;
                    if (P.logical_type == SH_E_LOGICAL_OR && !partner_in) {
                        add_empty_event(ev, p);  // OR: the partner never arrived
                        ch_add(retc, ev);
                    } else if (P.logical_type == SH_E_LOGICAL_AND && partner_in) {
                        ch_add(retc, ev);  // AND: the partner arrived but could not send out
                    } else if (P.logical_type == SH_E_LOGICAL_AND) {
                        add_empty_event(ev, p);  // AND: the partner may proceed later
                    }
                    continue;
                }
                i++;
            }
            if (expired && P.within_every >= 0) {
                add_every_state(P.within_every, expired);
                update_state(P.within_every);
            }
            ch_reset(retc);
            not_processed = retc[0] == 0;
            while (ch_has_next(retc)) {
                const uint32_t s = ch_next(retc);
                ch_remove(retc);
                se_set_ts(s, now);
                alog_send(p, s);
            }
            pst(p)[0] = 0;
        }
        if (P.next_every_pre >= 0 || (not_processed && P.is_start)) {
            // every, or an unanswered start state: wait again
            const int64_t lat = (int64_t)pst(p)[0];
            notify_at(p, lat == 0 ? clock + P.waiting : lat + P.waiting);
        }
        pret(p);
    }
    // :230-251
    NF_HD void alog_send(int p, uint32_t s) {
        const nf_proc& P = Q->proc[p];
        if (P.to_selector) {
            uint32_t c[4] = {s, s, 0, 0};
            selector_process(c);
        }
        if (P.next_pre >= 0) add_state(P.next_pre, s);
        if (P.next_every_pre >= 0) {
            add_every_state(P.next_every_pre, s);
        } else if (P.is_start) {
            ps_setf(p, NF_PS_INACTIVE, true);
            if (P.logical_type == SH_E_LOGICAL_OR && is_alog(P.partner)) {
                pget(P.partner);
                ps_setf(P.partner, NF_PS_INACTIVE, true);  // setActive(false)
                pret(P.partner);
            }
        }
        if (P.callback_pre >= 0) start_state_reset(P.callback_pre);
    }
    // :262-320 (returns an empty chunk)
    NF_HD uint32_t alog_process_and_return(int p, int64_t ts, uint32_t row) {
        const nf_proc& P = Q->proc[p];
        pget(p);
        if (ps_flag(p, NF_PS_INACTIVE)) {
            pret(p);
            return 0;
        }
        uint32_t* pl = list(p, 0);
        for (uint32_t i = 0; i < lcount(p, 0);) {
            const uint32_t s = pl[i];
            if (P.logical_type == SH_E_LOGICAL_OR && se_ev(s, P.partner)) {
                lerase(p, 0, i);
                continue;
            }
            const uint32_t cur_ev = se_ev(s, p);
            const uint32_t ne = new_node(ts, row);
            if (!ne) break;
            se_set_ev(s, p, ne);
            process_se(p, s);
            if (P.waiting != -1 ||
                (Q->state_type == SH_SEQUENCE && P.logical_type == SH_E_LOGICAL_AND && P.next_every_pre >= 0))
                se_set_ev(s, p, cur_ev);  // back to the original state
            bool erased = false;
            const int tl = P.this_last;
            if (returned(tl)) {
                // passed the filter: no longer an absence candidate
                set_returned(tl, false);
                lerase(p, 0, i);
                erased = true;
                if (Q->state_type == SH_SEQUENCE) {
                    pget(P.partner);
                    const uint32_t n = lcount(P.partner, 0);
                    const uint32_t* ql = list(P.partner, 0);
                    for (uint32_t k = 0; k < n; k++) {
                        if (ql[k] == s) {
                            lerase(P.partner, 0, k);
                            break;
                        }
                    }
                    pret(P.partner);
                }
            }
            if (!ps_flag(p, NF_PS_CHANGED)) {
                se_set_ev(s, p, cur_ev);
                if (Q->state_type == SH_SEQUENCE && !erased) {
                    lerase(p, 0, i);
                    erased = true;
                }
            }
            if (!erased) i++;
        }
        pret(p);
        return 0;
    }
    // :353-388, asked by the partner's LogicalPostStateProcessor (AND)
    NF_HD bool partner_can_proceed(int p, uint32_t s) {
        const nf_proc& P = Q->proc[p];
        pget(p);
        bool go;
        if (Q->state_type == SH_SEQUENCE && P.next_every_pre < 0 && (int64_t)pst(p)[0] > 0) {
            go = false;
        } else if (P.waiting == -1) {
            // no `for`: proceed while this absent state has not seen its event
            if (P.next_every_pre < 0) {
                go = se_ev(s, p) == 0;
            } else if ((int64_t)pst(p)[0] > 0) {
                go = false;
                pst(p)[0] = 0;
                init(p);
            } else {
                go = true;
            }
        } else {
            go = se_ev(s, p) != 0;
        }
        pret(p);
        return go;
    }

    // Scheduler.sendTimerEvents for this key (Scheduler.java:171-206): every queued
    // notification <= now, in FIFO order
    NF_HD void send_timer_events(int p, int64_t now) {
        int64_t t;
        while (sched_head(p, &t) && t <= now) {
            sched_pop(p);
            process_timer(p, t);
        }
        // SchedulerState.canDestroy: returnAllStates drops the drained state
        if (partitioned && (uint32_t)(sched(p)[0] >> 32) == 0) {
            sched(p)[1] = 0;
            sched_record(p, NF_SEV_REMOVE);
        }
    }

    // ---------------------------------------------------------- receivers
    // PatternMulti/Single, SequenceMulti/Single ProcessStreamReceiver.stabilizeStates
    NF_HD void stabilize(const nf_receiver& R, int64_t ts) {
        for (int p = 0; p < Q->n_proc; p++) expire_events(p, ts);
        if (Q->state_type == SH_SEQUENCE) {
            for (int i = 0; i < Q->n_reset; i++) reset_state(Q->reset_seq[i]);
            for (int i = 0; i < Q->n_update; i++) update_state(Q->update_seq[i]);
        } else if (R.multi) {
            for (int i = 0; i < R.n_for; i++) update_state(R.for_stream[i]);
        } else if (R.n_for > 0) {
            update_state(R.for_stream[0]);
        }
    }
    NF_HD uint32_t* run_retc() const { return (uint32_t*)(qb + Q->lay.off_hold); }
    NF_HD uint32_t* holders() const { return (uint32_t*)(qb + Q->lay.off_hold + 3); }
    NF_HD uint32_t& n_holders() const { return *(uint32_t*)(qb + Q->lay.off_hold + 2); }

    // Single / Multi ProcessStreamReceiver.receive over one same-key run of one
    // stream (SingleProcessStreamReceiver.java:48-73, MultiProcessStreamReceiver.java:155-183)
    template <class Events>
    NF_HD void receive(const nf_receiver& R, const Events& ev, int64_t b, int64_t e) {
        if (!R.multi) {
            uint32_t* retc = run_retc();
            ch_clear(retc);
            const int np = R.next_procs[0];
            for (int64_t k = b; k < e; k++) {
                cur_seq = ev.seq(k);
                stabilize(R, ev.ts(k));
                uint32_t r = process_and_return(np, ev.ts(k), ev.row(k));
                if (r) {
                    for (uint32_t x = r; x; x = se_next(x)) se(x)[1] = cur_seq;
                    ch_add(retc, r);
                }
                if (err) return;
                maybe_gc();
            }
            while (ch_has_next(retc)) {
                uint32_t s = ch_next(retc);
                ch_remove(retc);
                cur_seq = se(s)[1];
                if (R.has_selector) {
                    uint32_t one[4] = {s, s, 0, 0};
                    selector_process(one);
                }
            }
            ch_clear(retc);
            return;
        }
        n_holders() = 0;
        for (int64_t k = b; k < e; k++) {
            cur_seq = ev.seq(k);
            in_holder = 1;
            h_first = h_last = 0;
            h_has = 0;
            stabilize(R, ev.ts(k));
            for (int i = 0; i < R.n_next; i++) {
                const int p = R.next_procs[R.event_seq[i]];
                uint32_t retc[4] = {0, 0, 0, 0};
                uint32_t r = process_and_return(p, ev.ts(k), ev.row(k));
                if (r) ch_add(retc, r);
                if (R.has_selector) {
                    while (ch_has_next(retc)) {
                        uint32_t s = ch_next(retc);
                        ch_remove(retc);
                        uint32_t one[4] = {s, s, 0, 0};
                        selector_process(one);
                    }
                }
                if (h_has) {
                    uint32_t nh = n_holders();
                    if (nh >= (uint32_t)Q->lay.hold_cap / 2) {
                        err |= NF_E_HOLD;
                    } else {
                        holders()[2 * nh] = h_first;
                        holders()[2 * nh + 1] = h_last;
                        n_holders() = nh + 1;
                    }
                    h_first = h_last = 0;
                    h_has = 0;
                }
            }
            in_holder = 0;
            if (err) return;
            maybe_gc();
        }
        for (uint32_t h = 0; h < n_holders(); h++) {
            uint32_t c[4] = {holders()[2 * h], holders()[2 * h + 1], 0, 0};
            emit_chunk(c);
        }
        n_holders() = 0;
    }

    // StateStreamRuntime.initPartition (StateStreamRuntime.java:90-97)
    NF_HD void init_partition() {
        for (int i = 0; i < Q->n_init; i++) init(Q->init_seq[i]);
        for (int i = 0; i < Q->n_startup; i++) partition_created(Q->startup[i]);
    }

    // ---------------------------------------------------------- garbage collection
    // Mark-sweep of the query's arenas at an event boundary (the JVM reclaims by
    // reachability too). Roots: every pre-state's lists and `cur` chunk, the
    // Single receiver's pending return chunk, the Multi receiver's holders.
    // Marks: StateEvent word 2 bit 40, node row word bit 31 (rows < 2^31).
    NF_HD void maybe_gc() {
        const uint64_t* h = qb;
        const uint32_t se_live = (uint32_t)h[2], nd_live = (uint32_t)(h[2] >> 32);
        const uint32_t se_cap = (uint32_t)Q->lay.se_cap, nd_cap = (uint32_t)Q->lay.node_cap;
        if (se_live * 4 < se_cap * 3 && nd_live * 4 < nd_cap * 3) return;
        gc();
    }
    NF_HD void gc() {
        const uint32_t se_bump = (uint32_t)qb[1], nd_bump = (uint32_t)(qb[1] >> 32);
        for (uint32_t i = 1; i <= se_bump; i++) se(i)[2] &= ~(1ull << 40);
        for (uint32_t i = 1; i <= nd_bump; i++) node(i)[1] &= ~(1ull << 31);
        for (int p = 0; p < Q->n_proc; p++) {
            for (int w = 0; w < 2; w++) {
                const uint32_t n = lcount(p, w);
                const uint32_t* l = list(p, w);
                for (uint32_t i = 0; i < n; i++) gc_mark(l[i]);
            }
            const uint32_t* c = cur(p);
            for (int i = 0; i < 4; i++) gc_mark(c[i]);
        }
        const uint32_t* rc = run_retc();
        for (int i = 0; i < 4; i++) gc_mark(rc[i]);
        const uint32_t nh = n_holders();
        for (uint32_t i = 0; i < 2 * nh; i++) gc_mark(holders()[i]);
        if (Q->rate_kind == SH_RATE_ALL_EVENTS) gc_mark((uint32_t)qb[Q->lay.off_agg]);
        if (in_holder) {
            gc_mark(h_first);
            gc_mark(h_last);
        }
        // sweep into fresh free lists
        uint32_t fse = 0, fnd = 0, live_se = 0, live_nd = 0;
        for (uint32_t i = se_bump; i >= 1; i--) {
            if ((se(i)[2] >> 40) & 1) {
                se(i)[2] &= ~(1ull << 40);
                live_se++;
            } else {
                se(i)[2] = (se(i)[2] & ~0xFFFFFFFFull) | fse;
                fse = i;
            }
        }
        for (uint32_t i = nd_bump; i >= 1; i--) {
            if ((node(i)[1] >> 31) & 1) {
                node(i)[1] &= ~(1ull << 31);
                live_nd++;
            } else {
                nd_set_next(i, fnd);
                fnd = i;
            }
        }
        qb[0] = (uint64_t)fse | ((uint64_t)fnd << 32);
        qb[2] = (uint64_t)live_se | ((uint64_t)live_nd << 32);
    }
    NF_HD void gc_mark(uint32_t s) {
        // iterative over the `next` chain; slots' node chains walked inline
        while (s && !((se(s)[2] >> 40) & 1)) {
            se(s)[2] |= 1ull << 40;
            for (int k = 0; k < Q->n_proc; k++) {
                uint32_t n = se_ev(s, k);
                while (n && !((node(n)[1] >> 31) & 1)) {
                    node(n)[1] |= 1ull << 31;
                    n = nd_next(n);
                }
            }
            s = se_next(s);
        }
    }
};

// ------------------------------------------------------------------ segment driver
// Events interface (key-segment position k): ts(k), row(k), seq(k), stream(k),
// local(k) = arrival index inside the flushed batch set, batch(k) = send() call id,
// joins(e, k) = position e continues the same-key run started at k.
//
// PartitionStreamReceiver.receive(Event[]) (core/partition/PartitionStreamReceiver.java:176-272)
// splits a send() call into consecutive same-key runs, lazily inits the key's
// partition (PartitionRuntimeImpl.java:346-364), then hands the run to every
// query of the partition in order. Unpartitioned apps see each send() call
// whole (one key). Emissions of a run carry the run's first arrival index as
// their order tag, so a scan over per-event counts restores the reference's
// global order (R-order).
template <class Sink, class Events>
NF_HD void nf_process_segment(NfLane<Sink>& L, const Events& ev, int64_t beg, int64_t end, uint64_t tick,
                              uint32_t* match_cnt) {
    const nf_table* T = L.T;
    int64_t k = beg;
    while (k < end && !L.err) {
        int64_t e = k + 1;
        while (e < end && ev.joins(e, k)) e++;
        L.tag_index = ev.local(k);
        L.ordinal = 0;
        if (T->partitioned && !(L.kb[0] & 1ull)) {
            L.kb[0] |= 1ull;
            for (int q = 0; q < T->n_queries; q++) {
                L.Q = &T->q[q];
                L.qb = L.kb + L.Q->q_off;
                L.qi = q;
                L.stamp = (tick << 32) | ((uint64_t)ev.local(k) * 2);
                L.init_partition();
            }
        }
        const int s = ev.stream(k);
        for (int q = 0; q < T->n_queries && !L.err; q++) {
            const nf_query* Q = &T->q[q];
            if (!Q->recv[s].present) continue;
            L.Q = Q;
            L.qb = L.kb + Q->q_off;
            L.qi = q;
            L.stamp = (tick << 32) | ((uint64_t)ev.local(k) * 2 + 1);
            L.receive(Q->recv[s], ev, k, e);
        }
        if (L.ordinal && match_cnt) match_cnt[ev.local(k)] = L.ordinal;
        k = e;
    }
}
