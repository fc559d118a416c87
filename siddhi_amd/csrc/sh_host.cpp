// sh_host.cpp — host side of libsiddhi_hip.so: the C-ABI (include/siddhi_hip.h),
// lowering of the app descriptor to the device NFA program, HBM residency of
// event columns and per-key state, and the launch sequence
//   radix segment -> per-key advance -> ordered placement.
//
// The product path has no CPU fallback: without a device every call that
// needs one returns SH_E_NO_DEVICE.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "../../include/siddhi_hip.h"
#include "sh_agg.h"
#include "sh_device.h"
#include "sh_jit.h"
#include "sh_jmap.h"
#include "sh_nfa.h"
#include "sh_nfa_dev.h"
#include "sh_nfa_lower.h"
#include "sh_rules.h"

#define SH_VERSION_STR "siddhi_hip 0.1 (gfx950)"

namespace {

struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
    bool view = false;  // points into another buffer (set_view): never reallocated or freed here
    void set_view(void* at, size_t n) {
        p = at;
        bytes = n;
        view = true;
    }
    int ensure(size_t need) {
        if (need <= bytes) return 0;
        if (view) return SH_E_OOM;
        size_t nb = std::max(need, bytes * 2);
        void* q = nullptr;
        if (hipMalloc(&q, nb) != hipSuccess) return SH_E_OOM;
        if (p) {
            hipMemcpy(q, p, bytes, hipMemcpyDeviceToDevice);
            hipFree(p);
        }
        p = q;
        bytes = nb;
        return 0;
    }
    int ensure_fresh(size_t need) {  // no content preservation
        if (need <= bytes) return 0;
        if (view) return SH_E_OOM;
        if (p) hipFree(p);
        p = nullptr;
        bytes = 0;
        size_t nb = std::max(need, (size_t)4096);
        if (hipMalloc(&p, nb) != hipSuccess) return SH_E_OOM;
        bytes = nb;
        return 0;
    }
    void release() {
        if (p && !view) hipFree(p);
        p = nullptr;
        bytes = 0;
        view = false;
    }
    template <class T>
    T* as() const {
        return (T*)p;
    }
};

// page-locked host staging: async copies from / to it run as plain DMA
// (pageable copies go through the runtime's bounce buffers, ~20 us each)
struct PinBuf {
    void* p = nullptr;
    size_t bytes = 0;
    int ensure(size_t need) {  // no content preservation
        if (need <= bytes) return 0;
        release();
        size_t nb = std::max(need * 2, (size_t)1 << 16);
        if (hipHostMalloc(&p, nb, hipHostMallocDefault) != hipSuccess) {
            p = nullptr;
            return SH_E_OOM;
        }
        bytes = nb;
        return 0;
    }
    void release() {
        if (p) {
            hipDeviceSynchronize();  // an async copy may still read it
            hipHostFree(p);
        }
        p = nullptr;
        bytes = 0;
    }
    template <class T>
    T* as(size_t byte_off = 0) const {
        return (T*)((uint8_t*)p + byte_off);
    }
};

int type_width(int t) {
    switch (t) {
        case SH_T_LONG:
        case SH_T_DOUBLE: return 8;
        case SH_T_BOOL: return 1;
        default: return 4;
    }
}

// ----------------------------------------------------------- lowering
struct Lowering {
    const sh_query_desc* q;
    shp_program P;
    std::string err;
    std::vector<int> chain;  // stream element indices in slot order

    int add_const(int64_t v, int type, int isnull) {
        for (int i = 0; i < P.n_const; i++)
            if (P.consts[i] == v && P.const_type[i] == type && P.const_null[i] == isnull) return i;
        if (P.n_const >= 64) {
            err = "too many constants";
            return -1;
        }
        P.consts[P.n_const] = v;
        P.const_type[P.n_const] = (uint8_t)type;
        P.const_null[P.n_const] = (uint8_t)isnull;
        return P.n_const++;
    }
    bool emit(uint8_t op, uint8_t a, uint8_t b, uint8_t c, int32_t x) {
        if (P.n_code >= SHP_MAX_CODE) {
            err = "expression program too long";
            return false;
        }
        shp_instr& in = P.code[P.n_code++];
        in.op = op;
        in.a = a;
        in.b = b;
        in.c = c;
        in.x = x;
        return true;
    }
    static int dom_for(int op, int lt, int rt) {
        if (lt == SH_T_STRING || rt == SH_T_STRING) return DOM_STR;
        if (lt == SH_T_BOOL || rt == SH_T_BOOL) return DOM_BOOL;
        auto rk = [](int t) {
            switch (t) {
                case SH_T_INT: return 0;
                case SH_T_LONG: return 1;
                case SH_T_FLOAT: return 2;
                default: return 3;
            }
        };
        int r = std::max(rk(lt), rk(rt));
        // Equal/NotEqual FloatLong & LongFloat compare as double
        // (EqualCompareConditionExpressionExecutorFloatLong.java)
        bool fl = (lt == SH_T_FLOAT && rt == SH_T_LONG) || (lt == SH_T_LONG && rt == SH_T_FLOAT);
        if ((op == SH_OP_EQ || op == SH_OP_NE) && fl) r = 3;
        return r == 0 ? DOM_I32 : r == 1 ? DOM_I64 : r == 2 ? DOM_F32 : DOM_F64;
    }
    // postfix emission of an sh_expr tree
    bool gen(int e, int depth) {
        if (e < 0 || e >= q->n_exprs) {
            err = "bad expression index";
            return false;
        }
        if (depth > SHP_MAX_STACK - 2) {
            err = "expression too deep";
            return false;
        }
        const sh_expr& x = q->exprs[e];
        switch (x.op) {
            case SH_OP_CONST: {
                int c = add_const(x.cval, x.type, x.is_null);
                return c >= 0 && emit(OPC_CONST, 0, 0, 0, c);
            }
            case SH_OP_VAR:
                if (x.slot < 0 || x.slot >= P.n_states) {
                    err = "variable slot out of range";
                    return false;
                }
                return emit(OPC_VAR, (uint8_t)x.slot, (uint8_t)x.attr, (uint8_t)x.type, x.chain);
            case SH_OP_IS_NULL_STREAM:
                return emit(OPC_ISNULL_STREAM, (uint8_t)x.slot, 0, 0, x.chain);
            case SH_OP_NOT:
                return gen(x.lhs, depth + 1) && emit(OPC_NOT, 0, 0, 0, 0);
            case SH_OP_BOOL_VAR:
                return gen(x.lhs, depth + 1) && emit(OPC_BOOLV, 0, 0, 0, 0);
            case SH_OP_IS_NULL:
                return gen(x.lhs, depth + 1) && emit(OPC_ISNULL, 0, 0, 0, 0);
            case SH_OP_AND:
            case SH_OP_OR:
                return gen(x.lhs, depth + 1) && gen(x.rhs, depth + 2) &&
                       emit(x.op == SH_OP_AND ? OPC_AND : OPC_OR, 0, 0, 0, 0);
            case SH_OP_EQ:
            case SH_OP_NE:
            case SH_OP_GT:
            case SH_OP_GE:
            case SH_OP_LT:
            case SH_OP_LE: {
                int lt = q->exprs[x.lhs].type, rt = q->exprs[x.rhs].type;
                return gen(x.lhs, depth + 1) && gen(x.rhs, depth + 2) &&
                       emit(OPC_CMP, (uint8_t)x.op, (uint8_t)dom_for(x.op, lt, rt), 0, 0);
            }
            case SH_OP_ADD:
            case SH_OP_SUB:
            case SH_OP_MUL:
            case SH_OP_DIV:
            case SH_OP_MOD:
                return gen(x.lhs, depth + 1) && gen(x.rhs, depth + 2) &&
                       emit(OPC_ARITH, (uint8_t)x.op, (uint8_t)x.type, 0, 0);
            case SH_OP_IF_THEN_ELSE:
                return gen(x.lhs, depth + 1) && gen(x.rhs, depth + 2) && gen(x.third, depth + 3) &&
                       emit(OPC_SELECT, 0, 0, 0, 0) && emit(OPC_CAST, 0, (uint8_t)x.type, 0, 0);
        }
        err = "unsupported expression operator";
        return false;
    }
    // ---- register-only filters: conjunction of `attr op attr|const|attr(aop)const`
    const sh_app_desc* app = nullptr;
    static bool is_var(const sh_expr& x) {
        return x.op == SH_OP_VAR && (x.chain == 0 || x.chain == SH_CHAIN_CURRENT);
    }
    void conjuncts(int e, std::vector<int>& out) {
        const sh_expr& x = q->exprs[e];
        if (x.op == SH_OP_AND) {
            conjuncts(x.lhs, out);
            conjuncts(x.rhs, out);
        } else {
            out.push_back(e);
        }
    }
    // `a.k == b.k` on the attribute that keys the query's partition is always
    // true inside one partition (same key <=> same toString() for these types)
    bool partition_tautology(const sh_expr& c) {
        if (c.op != SH_OP_EQ || q->partition < 0 || !app || !app->partition_attr) return false;
        const sh_expr& l = q->exprs[c.lhs];
        const sh_expr& r = q->exprs[c.rhs];
        if (!is_var(l) || !is_var(r) || l.type != r.type) return false;
        if (!(l.type == SH_T_STRING || l.type == SH_T_INT || l.type == SH_T_LONG || l.type == SH_T_BOOL)) return false;
        const int ns = app->n_streams;
        const int sl = P.state_stream[l.slot], sr = P.state_stream[r.slot];
        return app->partition_attr[q->partition * ns + sl] == l.attr &&
               app->partition_attr[q->partition * ns + sr] == r.attr;
    }
    static int mirror(int op) {
        switch (op) {
            case SH_OP_GT: return SH_OP_LT;
            case SH_OP_GE: return SH_OP_LE;
            case SH_OP_LT: return SH_OP_GT;
            case SH_OP_LE: return SH_OP_GE;
            default: return op;
        }
    }
    bool fast_filter(int root, int k) {
        std::vector<int> cs;
        conjuncts(root, cs);
        int nt = 0;
        for (int e : cs) {
            const sh_expr& c = q->exprs[e];
            if (c.op < SH_OP_EQ || c.op > SH_OP_LE) return false;
            if (partition_tautology(c)) continue;
            if (nt >= SHP_MAX_TERMS) return false;
            int li = c.lhs, ri = c.rhs, op = c.op;
            if (!is_var(q->exprs[li])) {
                std::swap(li, ri);
                op = mirror(op);
            }
            const sh_expr& l = q->exprs[li];
            const sh_expr& r = q->exprs[ri];
            if (!is_var(l)) return false;
            shp_term t;
            memset(&t, 0, sizeof(t));
            t.op = (uint8_t)op;
            t.dom = (uint8_t)dom_for(op, l.type, r.type);
            t.lslot = (uint8_t)l.slot;
            t.lattr = (uint8_t)l.attr;
            t.ltype = (uint8_t)l.type;
            if (is_var(r)) {
                t.rkind = 0;
                t.rslot = (uint8_t)r.slot;
                t.rattr = (uint8_t)r.attr;
                t.rtype = (uint8_t)r.type;
            } else if (r.op == SH_OP_CONST) {
                if (r.is_null) return false;
                t.rkind = 1;
                t.ctype = (uint8_t)r.type;
                t.c = r.cval;
            } else if (r.op == SH_OP_ADD || r.op == SH_OP_SUB || r.op == SH_OP_MUL) {
                const sh_expr& a = q->exprs[r.lhs];
                const sh_expr& b = q->exprs[r.rhs];
                if (!is_var(a) || b.op != SH_OP_CONST || b.is_null) return false;
                t.rkind = 2;
                t.rslot = (uint8_t)a.slot;
                t.rattr = (uint8_t)a.attr;
                t.rtype = (uint8_t)a.type;
                t.aop = (uint8_t)r.op;
                t.atype = (uint8_t)r.type;
                t.ctype = (uint8_t)b.type;
                t.c = b.cval;
            } else {
                return false;
            }
            if (t.ltype == SH_T_OBJECT || t.rtype == SH_T_OBJECT) return false;
            P.terms[k][nt++] = t;
        }
        P.filter_nterms[k] = nt;
        P.filter_fast[k] = 1;
        return true;
    }
    // flatten `Next(...)` chains of stream states, `every` allowed on the start
    // state only (the shapes of configs C1/C2/C5)
    bool flatten(int e, bool first) {
        const sh_state_elem& el = q->elems[e];
        switch (el.kind) {
            case SH_E_NEXT:
                return flatten(el.child0, first) && flatten(el.child1, false);
            case SH_E_EVERY: {
                if (!first || !chain.empty() || q->elems[el.child0].kind != SH_E_STREAM) {
                    err = "device engine: `every` is supported on the start state only";
                    return false;
                }
                P.every_start = 1;
                chain.push_back(el.child0);
                return true;
            }
            case SH_E_STREAM:
                chain.push_back(e);
                return true;
            default:
                err = "device engine: count / logical / absent states are not lowered yet";
                return false;
        }
    }
};

}  // namespace

struct sh_handle {
    std::string err;
    bool has_device = false;
    sh_app_desc app{};
    std::vector<std::vector<int32_t>> stream_types;
    int32_t n_out = 0;
    int32_t partitioned = 0;
    shp_program prog{};
    shp_layout lay{};
    hipStream_t stream = nullptr;      // active stream
    hipStream_t own_stream = nullptr;  // created by sh_compile
    DevBuf d_prog, d_cols_desc, d_kstate, d_err;
    int32_t nkeys_alloc = 0;
    // column stores (streaming path)
    struct Store {
        std::vector<DevBuf> cols, nuls;
        std::vector<bool> has_nul;
        int64_t rows = 0;
    };
    std::vector<Store> stores;
    // staged (pushed, not yet processed) events
    std::vector<int64_t> st_ts;
    std::vector<uint8_t> st_stream;
    std::vector<uint32_t> st_row;
    std::vector<int32_t> st_key;
    int32_t max_key = 0;
    uint64_t seq_next = 0;  // global sequence of the next staged event
    uint64_t seq_staged0 = 0;
    // workspaces
    DevBuf w_ts, w_stream, w_row, w_key, w_keys_a, w_keys_b, w_idx_a, w_idx_b, w_hist, w_scan, w_seg;
    DevBuf w_pstage;  // the general engine's per-call staging (nf_push), one block
    DevBuf w_orows;   // placed rows of a streaming launch, one block (query | seq | ts | values | nulls)
    DevBuf w_cnt, w_off, w_tmp, w_ctr, w_oseq, w_ots, w_ovals, w_onulls, w_oq, w_inv;
    bool dev_want_query = false;  // sh_run_device asked for d_out_query
    const uint32_t* dev_run_ids = nullptr;  // sh_run_device's d_run while it runs the general engine
    bool poisoned = false;  // a failed restore could not put the handle back: every call is refused
    DevBuf v_sts, v_mpos, v_flag, v_cnts, v_mid_ts, v_dir;
    DevBuf v_scol[32], v_mid[32];
    int64_t tmp_cap = 0;
    // drained output queue (host)
    std::vector<int32_t> o_query;
    std::vector<uint64_t> o_seq;
    std::vector<int64_t> o_ts;
    std::vector<int64_t> o_vals;
    std::vector<uint8_t> o_nulls;
    std::vector<uint64_t> o_order;  // key-sharded: per row, launch << 32 | position in the launch
    // deferred rows of streaming launches (single process, no List outputs): each
    // launch's placed rows are appended on the device after the *df_ctr rows already
    // there; they join the host queue above at the next flush (drain / pending /
    // snapshot), so a send() costs no placement round trip. df_ub: an upper bound of
    // the rows held (the launches' record counts), df_stream: the stream they are on.
    DevBuf df_q, df_seq, df_ts, df_vals, df_nulls, df_ctr;
    int64_t df_cap = 0, df_ub = 0;
    hipStream_t df_stream = nullptr;
    int64_t o_read = 0;
    // ---- key-sharded streaming (sh_set_coordinator): the other ranks
    bool coord_on = false;
    sh_coordinator coord{};
    DevBuf w_gidx, n_gpos;
    // ---- List outputs (SH_OP_MULTI_VAR): the launch's device buffer (nf_cols.lst)
    // and the host lists rows hand out (ids l_base ..; valid until the next drain)
    bool has_lists = false;
    DevBuf n_lst, n_lst_ctr;
    int64_t lst_cap = 0;
    std::vector<int64_t> l_vals;
    std::vector<uint8_t> l_nuls;
    std::vector<int64_t> l_start;  // per live list: offset into l_vals (plus one end entry)
    int64_t l_base = 0;            // id of the first live list
    sh_kernel_times times{};
    hipEvent_t ev[6] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};  // [4, 5]: aggregate post-pass
    // hipRTC-specialised window kernels (sh_jit.cpp): 0 untried, 1 loaded, <0 unavailable
    int jit_state = 0;
    shj_window jit{};
    std::string jit_err;
    // ---- general engine (sh_nfa.h): mode 1
    int mode = 0;                 // 0: chain / window engines, 1: general NFA engine
    nf_table* T = nullptr;        // host copy of the NFA table
    DevBuf d_T, d_T_old, d_ncols, n_kstate, n_kstate2, n_save, n_recs, n_ctr, n_err, n_cand, n_sel, n_bid;
    // pinned staging of the streaming path: pin_in = one send() call's uploads,
    // pin_rd = small read-backs + the nf_cols image, pin_out = placed rows
    PinBuf pin_in, pin_rd, pin_out;
    PinBuf pin_stage;  // the general engine's per-call event staging (nf_push)
    DevBuf n_tmin, n_slot_s, n_slot_k;  // device tie-break of due keys
    DevBuf n_armed;                     // per key: may hold a scheduler entry (nf_cols.sched_armed)
    // the armed-key list of the due pass (two buffers, swapped per pass; counts
    // in n_klist_n[0..1]) and the log of keys armed since the last pass
    DevBuf n_klist[2], n_klist_n, n_arm_log, n_arm_ctr;
    int klist_cur = 0;
    double hp_ms[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};  // SH_HOST_PROF: wall time per host phase (printed by sh_destroy)
    int64_t hp_n[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    int seq3_last = 0;                  // the last general-engine run took k_seq3
    bool s3_compact = false;            // ... with k_seq3s's compact records (nfd_place_s3 places them)
    bool s3_agg = false;                // ... whose aggregates ran in the kernel (no post-pass)
    int s3_rw = 0;                      // record words
    uint32_t s3_wide = 0;               // outputs held as 2-word running values
    bool kstate_stale = false;          // key blocks not reset after a k_seq3 run (reset before the next use)
    int s3_type = 0;                    // their values' type (one 4-byte attribute)
    uint64_t s3_seq_base = 0;           // and the run's first trigger sequence number
    bool no_seq3 = false;               // rerun without k_seq3 (aggregates not exact in parallel)
    // scheduler maps' iteration order (sh_jmap.h): host models fed by the
    // launches' getState history, per-key ranks uploaded for the due-key pick
    bool sm_on = false;
    ShSchedModels sm;
    DevBuf n_sev, n_sev_ctr, n_rk_keys, n_rk_vals;
    // the general engine's per-launch counters in one block (one fill, one read-back):
    // record counter n_ctr at 0, error word n_err at 8, history counter n_sev_ctr at 16
    DevBuf n_ctl;
    nf_cols cols_last;          // the column image last uploaded to d_ncols (nf_put_cols)
    bool cols_cached = false;
    std::vector<DevBuf> n_rank;         // by scheduler id, [n_nkeys] u64
    // deferred scheduler history (single process): launches whose records were
    // copied to pin_hist but not yet replayed on the models (nf_sev_flush replays
    // them, in launch order, before the next use of the ranks)
    PinBuf pin_hist;
    int64_t hist_used = 0;                        // records in pin_hist
    std::vector<std::pair<int64_t, int64_t>> sev_pend;  // (first record, records) per launch
    PinBuf pin_sev, pin_rk;
    int64_t sev_cap = 0;
    int caps[6] = {16, 32, 64, 32, 8, 4};  // list, se, node, hold, sched, group
    int32_t n_nkeys = 0;          // key blocks allocated
    int64_t rec_cap = 0;
    int64_t clock = 0;            // TimestampGeneratorImpl current time
    uint64_t tick = 1;            // processing-phase counter (scheduler registration order)
    bool started = false;
    uint32_t batch_id = 0;
    // ---- batch-compiled rule sets (sh_rules.hip): sh_run_device on mode 2, or
    // on any app every query of which is window-shaped
    bool has_rules = false;
    bool r_partitioned = false;
    int32_t r_nout = 0;
    std::vector<shr_rule> r_rules;
    bool r_aggp = false;                 // every rule aggregates (sh_agg.hip post-pass)
    int32_t r_agg[SHP_MAX_OUT] = {0}, r_argt[SHP_MAX_OUT] = {0};
    DevBuf a_q;                          // query per row when the caller wants none
    bool skip_rules = false;             // rerun on the general engine (aggregates not exact in parallel)
    std::vector<int64_t> r_ixval;
    std::vector<uint32_t> r_ixstart, r_ixrule, r_free;
    std::vector<int8_t> r_ixterm;  // per rule: the f1 term its index group implies (-1: none)
    shr_table r_tab{};
    DevBuf rd_rules, rd_ixval, rd_ixstart, rd_ixrule, rd_free, rd_tab;
    DevBuf rd_img;   // the rule set's LDS image (shr_img), when it fits
    DevBuf r_tsr, v_ts32, v_sts32, v_mid_ts32;  // 32-bit timestamp offsets of a rule run (range, arrival, sorted, mid)
    shr_img r_img{};
    DevBuf r_rec, r_keys, r_g, r_sk, r_sv, r_hist, r_scan, r_run;
    // ---- bucketed window engine (sh_bucket.hip + shb_match): 0 untried, 1 loaded, <0 unavailable
    int bk_state = 0;
    int32_t part_attr0 = -1;  // stream-0 attribute keying query 0's partition
    int bk_last = 0;          // 1: the last sh_run_device ran on the bucketed engine
    int s3b_last = 0;         // 1: ... on the sequence bucket-carry engine (k_s3b)
    shj_bucket bk{};
    std::string bk_err;
    DevBuf bk_w0, bk_sp, bk_toff, bk_cnt, bk_mstart, bk_tpre, bk_tfirst, bk_hstart, bk_ttot, bk_flag, bk_prof;
    DevBuf bk_st[SHB_MAX_STAGED], bk_ms[SHB_MAX_MS], bk_agg[SHB_MAX_AGG];
    bool bk_agg_carried = false;  // the last bucketed run carried its aggregates (k_bk_aggc)
    PinBuf bk_rd;
    // typed output columns (sh_device_run.d_out_cols) for engines that write rows
    DevBuf w_colrows;
    bool cols_rows = false;
    // aggregators behind the fast engines (sh_agg.hip): scratch, trigger sequence
    // numbers when the caller wants none, and the last run's path
    DevBuf a_scratch, a_seq;
    int agg_last = 0;  // 1: post-pass done, 2: post-pass not exact -> sequential engine, 3: in the k_seq3s lanes,
                       // 4: carried per key by the bucketed engine (k_bk_aggc)
    std::vector<int32_t> out_types;  // per select position over the queries (-2: types differ)
    uint64_t fp = 0;                 // compiled-program fingerprint (snapshot images)
};

// SH_HOST_PROF: a phase's wall time into h->hp_ms[i] (scope lifetime)
struct HpScope {
    sh_handle* h;
    int i;
    std::chrono::steady_clock::time_point t0;
    HpScope(sh_handle* hh, int ii) : h(getenv("SH_HOST_PROF") ? hh : nullptr), i(ii) {
        if (h) t0 = std::chrono::steady_clock::now();
    }
    ~HpScope() {
        if (!h) return;
        h->hp_ms[i] += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        h->hp_n[i]++;
    }
};

static void set_layout(shp_layout& Y, const shp_program& P, int32_t cap) {
    Y.cap = cap;
    Y.rec_words = 2 + (P.n_states + 1) / 2;
    Y.list_bytes = (int64_t)Y.cap * Y.rec_words * 8;
    Y.off_lists = (int64_t)(1 + SHP_MAX_STATES) * 8;
    Y.off_agg = Y.off_lists + (int64_t)(P.n_states > 1 ? P.n_states - 1 : 0) * 2 * Y.list_bytes;
    Y.key_bytes = Y.off_agg + (int64_t)P.n_out * 5 * 8;
    Y.key_bytes = (Y.key_bytes + 63) & ~63ll;
}

static int fail(sh_handle* h, int code, const std::string& m) {
    if (h) h->err = m;
    return code;
}

static bool device_available() {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return false;
    return n > 0;
}

extern "C" {

const char* sh_version(void) { return SH_VERSION_STR; }

int sh_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

const char* sh_last_error(sh_handle* h) { return h ? h->err.c_str() : "null handle"; }

// chain / window engines: PATTERN chains of stream states in one query
// (k_advance, sh_window.hip); returns SH_E_UNSUPPORTED for anything else
// (errors are reported through h->err; h is only used for that)
static int lower_chain(sh_handle* h, const sh_app_desc* app, int qi, shp_program& Pout) {
    const sh_query_desc& q = app->queries[qi];
    if (q.state_type != SH_PATTERN) return fail(h, SH_E_UNSUPPORTED, "chain engine: sequences go to the general engine");
    Lowering L;
    L.q = &q;
    L.app = app;
    memset(&L.P, 0, sizeof(L.P));
    if (!L.flatten(q.root, true)) return fail(h, SH_E_UNSUPPORTED, L.err);
    shp_program& P = L.P;
    P.n_states = (int32_t)L.chain.size();
    if (P.n_states < 1 || P.n_states > SHP_MAX_STATES)
        return fail(h, SH_E_UNSUPPORTED, "device engine: 1..8 states per pattern");
    P.within_ms = q.within_ms;
    P.n_streams = app->n_streams;
    for (int k = 0; k < P.n_states; k++) {
        const sh_state_elem& el = q.elems[L.chain[k]];
        if (el.slot != k) return fail(h, SH_E_INVALID_ARG, "state slots are not in chain order");
        P.state_stream[k] = el.stream;
    }
    // receivers: PatternSingle updates its only state; PatternMulti updates all
    // states of the stream in setup order and processes them in reverse
    // (PatternMultiProcessStreamReceiver.java:34-51)
    for (int s = 0; s < app->n_streams; s++) {
        int c = 0;
        for (int k = 0; k < P.n_states; k++)
            if (P.state_stream[k] == s) P.upd_state[s][c++] = k;
        P.upd_count[s] = c;
        P.proc_count[s] = c;
        for (int i = 0; i < c; i++) P.proc_state[s][i] = P.upd_state[s][c - 1 - i];
        P.stream_nattr[s] = app->streams[s].n_attrs;
        for (int a = 0; a < app->streams[s].n_attrs; a++) P.attr_type[s][a] = app->streams[s].attr_types[a];
    }
    for (int k = 0; k < P.n_states; k++) {
        const sh_state_elem& el = q.elems[L.chain[k]];
        if (el.filter >= 0) {
            P.filter_pc[k] = P.n_code;
            if (!L.gen(el.filter, 0)) return fail(h, SH_E_UNSUPPORTED, L.err);
            P.filter_len[k] = P.n_code - P.filter_pc[k];
        } else {
            P.filter_pc[k] = -1;
            P.filter_len[k] = 0;
        }
    }
    for (int k = 0; k < P.n_states; k++) {
        const sh_state_elem& el = q.elems[L.chain[k]];
        P.filter_fast[k] = 0;
        if (el.filter >= 0) {
            if (!getenv("SH_DISABLE_FAST_FILTER")) L.fast_filter(el.filter, k);
        } else {
            P.filter_fast[k] = 1;  // no filter: empty conjunction
            P.filter_nterms[k] = 0;
        }
    }
    if (q.n_outputs > SHP_MAX_OUT) return fail(h, SH_E_UNSUPPORTED, "device engine: at most 16 output attributes");
    P.n_out = q.n_outputs;
    P.out_fast = getenv("SH_DISABLE_FAST_FILTER") ? 0 : 1;
    P.agg_post = 0;
    for (int o = 0; o < q.n_outputs; o++) {
        const sh_output_attr& oa = q.outputs[o];
        const bool postable = oa.agg == SH_AGG_SUM || oa.agg == SH_AGG_AVG || oa.agg == SH_AGG_COUNT;
        if (oa.agg == SH_AGG_COUNT && oa.expr < 0) {
            // count(): the row carries any value; the post-pass counts rows
            P.out_slot[o] = 1;
            P.out_attr[o] = 0;
            P.agg_post = 1;
        } else if ((oa.agg != SH_AGG_NONE && !postable) || oa.expr < 0 || !Lowering::is_var(q.exprs[oa.expr])) {
            P.out_fast = 0;
        } else {
            P.out_slot[o] = q.exprs[oa.expr].slot;
            P.out_attr[o] = q.exprs[oa.expr].attr;
            if (oa.agg != SH_AGG_NONE) P.agg_post = 1;
        }
    }
    if (!P.out_fast || getenv("SH_NO_AGG_POST")) P.agg_post = 0;
    for (int o = 0; o < q.n_outputs; o++) {
        const sh_output_attr& oa = q.outputs[o];
        P.out_agg[o] = oa.agg;
        P.out_type[o] = oa.type;
        if (oa.expr >= 0) {
            P.out_pc[o] = P.n_code;
            if (!L.gen(oa.expr, 0)) return fail(h, SH_E_UNSUPPORTED, L.err);
            P.out_len[o] = P.n_code - P.out_pc[o];
            P.out_arg_type[o] = q.exprs[oa.expr].type;
        } else {
            P.out_pc[o] = -1;
            P.out_len[o] = 0;
        }
    }
    // the data-parallel window engine (sh_window.hip) covers
    // `every e1=S[f1] -> e2=S[f2] within W` without aggregators
    {
        bool agg = false;
        for (int o = 0; o < P.n_out; o++) agg |= P.out_agg[o] != SH_AGG_NONE;
        P.window_ok = (P.n_states == 2 && P.every_start && P.within_ms >= 0 && (!agg || P.agg_post) &&
                       P.state_stream[0] == P.state_stream[1] && app->n_streams == 1)
                          ? 1
                          : 0;
        if (getenv("SH_DISABLE_WINDOW")) P.window_ok = 0;
    }
    if (q.partition >= 0) {
        for (int k = 0; k < P.n_states; k++) {
            int s = P.state_stream[k];
            if (!app->partition_streams[q.partition * app->n_streams + s])
                return fail(h, SH_E_UNSUPPORTED, "device engine: every stream of a partitioned query must be keyed");
        }
    }
    Pout = P;
    return SH_OK;
}

// having / order by / limit / offset / output rate limiting need the selector pass of
// the general engine
static bool has_selector_extras(const sh_app_desc* app) {
    for (int32_t q = 0; q < app->n_queries; q++) {
        const sh_query_desc& d = app->queries[q];
        if (d.having >= 0 || d.n_order > 0 || d.limit >= 0 || d.offset >= 0 || d.rate_kind != SH_RATE_NONE ||
            d.n_group > 0)
            return true;
        // a List output (SH_OP_MULTI_VAR) is built by the general engine's selector
        for (int32_t o = 0; o < d.n_outputs; o++)
            if (d.outputs[o].expr >= 0 && d.outputs[o].expr < d.n_exprs && d.exprs[d.outputs[o].expr].op == SH_OP_MULTI_VAR)
                return true;
    }
    return false;
}

static int compile_chain(sh_handle* h, const sh_app_desc* app) {
    if (app->n_queries != 1) return fail(h, SH_E_UNSUPPORTED, "chain engine: one query per app");
    if (has_selector_extras(app))
        return fail(h, SH_E_UNSUPPORTED, "chain engine: having / order by / limit run on the general engine");
    shp_program P;
    int rc = lower_chain(h, app, 0, P);
    if (rc) return rc;
    h->prog = P;
    h->n_out = P.n_out;
    h->partitioned = app->queries[0].partition >= 0;
    h->part_attr0 = (h->partitioned && app->partition_attr)
                        ? app->partition_attr[app->queries[0].partition * app->n_streams + 0]
                        : -1;
    // per-key state layout
    const char* capenv = getenv("SH_PARTIAL_CAP");
    set_layout(h->lay, P, capenv ? atoi(capenv) : 32);

    return SH_OK;
}

// ---- batch-compiled rule sets: every query `every e1=S[f1] -> e2=S[f2] within W`
// with register filters and a projection, all over stream 0 and one partition
static bool ix_term_ok(const shp_term& X) {
    if (X.op != SH_OP_EQ || X.rkind != 1 || X.lslot != 0) return false;
    const bool li = X.ltype == SH_T_INT || X.ltype == SH_T_LONG;
    const bool ci = X.ctype == SH_T_INT || X.ctype == SH_T_LONG;
    if (li && ci) return X.dom == DOM_I32 || X.dom == DOM_I64;
    return X.ltype == X.ctype && (X.ltype == SH_T_STRING || X.ltype == SH_T_BOOL);
}

// index key of a constant, as rule_ix_key (sh_rules.hip) keys attribute values
static int64_t ix_const_key(int type, int64_t c) {
    if (type == SH_T_LONG) return c;
    if (type == SH_T_BOOL) return c != 0;
    return (int64_t)(int32_t)c;
}

static int compile_rules(sh_handle* h, const sh_app_desc* app) {
    if (app->n_queries < 2 || app->n_streams != 1)
        return fail(h, SH_E_UNSUPPORTED, "rule engine: two or more queries over one stream");
    if (has_selector_extras(app))
        return fail(h, SH_E_UNSUPPORTED, "rule engine: having / order by / limit run on the general engine");
    const int part = app->queries[0].partition;
    std::vector<shr_rule> rules(app->n_queries);
    std::unique_ptr<sh_handle> tmp(new sh_handle());
    std::unique_ptr<shp_program> P(new shp_program());
    for (int qi = 0; qi < app->n_queries; qi++) {
        if (lower_chain(tmp.get(), app, qi, *P))
            return fail(h, SH_E_UNSUPPORTED, "rule engine: query " + std::to_string(qi) + ": " + tmp->err);
        if (!P->window_ok || !P->filter_fast[0] || !P->filter_fast[1] || !P->out_fast ||
            app->queries[qi].partition != part)
            return fail(h, SH_E_UNSUPPORTED, "rule engine: query " + std::to_string(qi) +
                                                 " is not `every e1=S[f1] -> e2=S[f2] within W` with register "
                                                 "filters and a projection in the common partition");
        shr_rule& R = rules[qi];
        memset(&R, 0, sizeof(R));
        R.within = P->within_ms;
        R.query = qi;
        R.n_out = P->n_out;
        for (int k = 0; k < 2; k++) {
            R.nt[k] = P->filter_nterms[k];
            for (int t = 0; t < R.nt[k]; t++) R.t[k][t] = P->terms[k][t];
        }
        for (int o = 0; o < P->n_out; o++) {
            R.out_slot[o] = (int8_t)P->out_slot[o];
            R.out_attr[o] = (int8_t)P->out_attr[o];
        }
        // aggregators: one layout for the whole set (the post-pass runs per column
        // over every rule's rows, keyed by (rule, partition key))
        if (qi == 0) {
            h->r_aggp = P->agg_post != 0;
            for (int o = 0; o < SHP_MAX_OUT; o++) {
                h->r_agg[o] = o < P->n_out ? P->out_agg[o] : SH_AGG_NONE;
                h->r_argt[o] = o < P->n_out ? P->out_arg_type[o] : 0;
            }
        } else {
            bool same = (P->agg_post != 0) == h->r_aggp;
            for (int o = 0; o < P->n_out && same; o++)
                same = P->out_agg[o] == h->r_agg[o] && (P->out_agg[o] == SH_AGG_NONE || P->out_arg_type[o] == h->r_argt[o]);
            for (int o = P->n_out; o < SHP_MAX_OUT && same; o++) same = h->r_agg[o] == SH_AGG_NONE;
            if (!same)
                return fail(h, SH_E_UNSUPPORTED, "rule engine: the queries aggregate different select positions");
        }
    }
    // predicate index: the slot-0 attribute most start filters compare for
    // equality with a constant
    const int na = app->streams[0].n_attrs;
    std::vector<int> votes(na, 0);
    for (const shr_rule& R : rules) {
        std::vector<bool> seen(na, false);
        for (int t = 0; t < R.nt[0]; t++) {
            const shp_term& X = R.t[0][t];
            if (ix_term_ok(X) && X.lattr < na && !seen[X.lattr]) {
                seen[X.lattr] = true;
                votes[X.lattr]++;
            }
        }
    }
    int ix = -1;
    for (int a = 0; a < na; a++)
        if (votes[a] > 0 && (ix < 0 || votes[a] > votes[ix])) ix = a;
    std::vector<std::pair<int64_t, uint32_t>> ent;
    h->r_free.clear();
    h->r_ixterm.assign(rules.size(), (int8_t)-1);
    for (uint32_t r = 0; r < (uint32_t)rules.size(); r++) {
        int t = -1;
        for (int k = 0; ix >= 0 && k < rules[r].nt[0]; k++)
            if (ix_term_ok(rules[r].t[0][k]) && rules[r].t[0][k].lattr == ix) {
                t = k;
                break;
            }
        h->r_ixterm[r] = (int8_t)t;
        if (t < 0)
            h->r_free.push_back(r);
        else
            ent.emplace_back(ix_const_key(rules[r].t[0][t].ctype, rules[r].t[0][t].c), r);
    }
    std::sort(ent.begin(), ent.end());
    h->r_ixval.clear();
    h->r_ixstart.clear();
    h->r_ixrule.clear();
    for (size_t i = 0; i < ent.size(); i++) {
        if (i == 0 || ent[i].first != ent[i - 1].first) {
            h->r_ixval.push_back(ent[i].first);
            h->r_ixstart.push_back((uint32_t)i);
        }
        h->r_ixrule.push_back(ent[i].second);
    }
    h->r_ixstart.push_back((uint32_t)ent.size());
    memset(&h->r_tab, 0, sizeof(h->r_tab));
    h->r_tab.n_rules = (int32_t)rules.size();
    h->r_tab.ix_attr = h->r_ixval.empty() ? -1 : ix;
    h->r_tab.n_ix = (int32_t)h->r_ixval.size();
    h->r_tab.n_free = (int32_t)h->r_free.size();
    for (int a = 0; a < na && a < 32; a++) h->r_tab.attr_type[a] = app->streams[0].attr_types[a];
    h->r_nout = 0;
    for (const shr_rule& R : rules) h->r_nout = std::max(h->r_nout, R.n_out);
    h->r_rules.swap(rules);
    h->r_partitioned = part >= 0;
    h->has_rules = true;
    return SH_OK;
}

static int upload_rules(sh_handle* h) {
    const size_t nr = h->r_rules.size();
    if (h->rd_rules.ensure(nr * sizeof(shr_rule)) || h->rd_ixval.ensure(8 * h->r_ixval.size() + 8) ||
        h->rd_ixstart.ensure(4 * h->r_ixstart.size() + 4) || h->rd_ixrule.ensure(4 * h->r_ixrule.size() + 4) ||
        h->rd_free.ensure(4 * h->r_free.size() + 4) || h->rd_tab.ensure(sizeof(shr_table)))
        return fail(h, SH_E_OOM, "hipMalloc failed");
    hipMemcpy(h->rd_rules.p, h->r_rules.data(), nr * sizeof(shr_rule), hipMemcpyHostToDevice);
    if (!h->r_ixval.empty()) hipMemcpy(h->rd_ixval.p, h->r_ixval.data(), 8 * h->r_ixval.size(), hipMemcpyHostToDevice);
    hipMemcpy(h->rd_ixstart.p, h->r_ixstart.data(), 4 * h->r_ixstart.size(), hipMemcpyHostToDevice);
    if (!h->r_ixrule.empty())
        hipMemcpy(h->rd_ixrule.p, h->r_ixrule.data(), 4 * h->r_ixrule.size(), hipMemcpyHostToDevice);
    if (!h->r_free.empty()) hipMemcpy(h->rd_free.p, h->r_free.data(), 4 * h->r_free.size(), hipMemcpyHostToDevice);
    // the LDS image: index values / starts, rule ids, per-rule window + term range, terms
    {
        memset(&h->r_img, 0, sizeof(h->r_img));
        std::vector<uint8_t> img;
        auto sect = [&](size_t bytes) {
            const size_t at = (img.size() + 15) & ~(size_t)15;
            img.resize(at + bytes);
            return at;
        };
        // an indexed rule's equality term on the index attribute holds for every event
        // its group is looked up for (the lookup matched the constant's key exactly),
        // so the image leaves it out (SH_RULES_IXTERM=1 keeps it)
        const bool drop_ix = !(getenv("SH_RULES_IXTERM") && getenv("SH_RULES_IXTERM")[0] == '1');
        auto implied = [&](size_t i) { return drop_ix && i < h->r_ixterm.size() ? (int)h->r_ixterm[i] : -1; };
        size_t nt0 = 0, nt1 = 0;
        for (size_t i = 0; i < nr; i++) {
            const shr_rule& r = h->r_rules[i];
            nt0 += (size_t)r.nt[0] - (implied(i) >= 0 ? 1 : 0);
            nt1 += (size_t)r.nt[1];
        }
        // dense index over a small key range (SH_RULES_DENSE=0: the binary search,
        // whose values and starts are then the only copy of the groups)
        int64_t dmin = 0, drange = 0;
        if (!h->r_ixval.empty() && !(getenv("SH_RULES_DENSE") && getenv("SH_RULES_DENSE")[0] == '0')) {
            dmin = h->r_ixval.front();
            const int64_t r = h->r_ixval.back() - dmin + 1;
            if (r > 0 && r <= 16384) drange = r;
        }
        const size_t o_ixv = sect(drange ? 0 : 8 * h->r_ixval.size());
        const size_t o_ixs = sect(drange ? 0 : 4 * h->r_ixstart.size());
        const size_t o_ixr = sect(4 * h->r_ixrule.size());
        const size_t o_fr = sect(4 * h->r_free.size());
        const size_t o_meta = sect(sizeof(shr_meta) * nr);
        const size_t o_dense = sect(8 * (size_t)drange);
        const size_t o_t1 = sect(sizeof(shp_term) * nt1);
        const size_t lds_split = (img.size() + 15) & ~(size_t)15;
        const size_t o_t0 = sect(sizeof(shp_term) * nt0);
        img.resize((img.size() + 15) & ~(size_t)15);
        const bool split = getenv("SH_RULES_IMG_SPLIT") && getenv("SH_RULES_IMG_SPLIT")[0] == '1';
        const size_t lds = split ? lds_split : img.size();
        static const bool img_on = !(getenv("SH_RULES_IMG") && getenv("SH_RULES_IMG")[0] == '0');
        if (img_on && lds <= SHR_IMG_MAX && nt0 < 65536 && nt1 < 65536) {
            if (!drange) {
                if (!h->r_ixval.empty()) memcpy(&img[o_ixv], h->r_ixval.data(), 8 * h->r_ixval.size());
                memcpy(&img[o_ixs], h->r_ixstart.data(), 4 * h->r_ixstart.size());
            }
            if (!h->r_ixrule.empty()) memcpy(&img[o_ixr], h->r_ixrule.data(), 4 * h->r_ixrule.size());
            if (!h->r_free.empty()) memcpy(&img[o_fr], h->r_free.data(), 4 * h->r_free.size());
            for (size_t g = 0; drange && g < h->r_ixval.size(); g++) {
                const uint32_t e[2] = {h->r_ixstart[g], h->r_ixstart[g + 1]};
                memcpy(&img[o_dense + 8 * (size_t)(h->r_ixval[g] - dmin)], e, 8);
            }
            size_t k0 = 0, k1 = 0;
            for (size_t i = 0; i < nr; i++) {
                const shr_rule& r = h->r_rules[i];
                shr_meta m;
                memset(&m, 0, sizeof(m));
                m.within = r.within;
                m.toff0 = (uint16_t)k0;
                m.toff1 = (uint16_t)k1;
                const int skip = implied(i);
                m.nt0 = (uint8_t)(r.nt[0] - (skip >= 0 ? 1 : 0));
                m.nt1 = (uint8_t)r.nt[1];
                memcpy(&img[o_meta + i * sizeof(shr_meta)], &m, sizeof(m));
                for (int t = 0; t < r.nt[0]; t++) {
                    if (t == skip) continue;
                    memcpy(&img[o_t0 + k0 * sizeof(shp_term)], &r.t[0][t], sizeof(shp_term));
                    k0++;
                }
                for (int t = 0; t < r.nt[1]; t++, k1++)
                    memcpy(&img[o_t1 + k1 * sizeof(shp_term)], &r.t[1][t], sizeof(shp_term));
            }
            if (h->rd_img.ensure(img.size())) return fail(h, SH_E_OOM, "hipMalloc failed");
            hipMemcpy(h->rd_img.p, img.data(), img.size(), hipMemcpyHostToDevice);
            h->r_img.bytes = (int32_t)img.size();
            h->r_img.lds = (int32_t)lds;
            h->r_img.off_ixv = (int32_t)o_ixv;
            h->r_img.off_ixs = (int32_t)o_ixs;
            h->r_img.off_ixr = (int32_t)o_ixr;
            h->r_img.off_free = (int32_t)o_fr;
            h->r_img.off_meta = (int32_t)o_meta;
            h->r_img.off_terms1 = (int32_t)o_t1;
            h->r_img.off_terms0 = (int32_t)o_t0;
            h->r_img.dense_min = dmin;
            h->r_img.dense_n = (int32_t)drange;
            h->r_img.off_dense = (int32_t)o_dense;
        }
    }
    shr_table t = h->r_tab;
    t.rules = h->rd_rules.as<shr_rule>();
    t.ix_val = h->rd_ixval.as<int64_t>();
    t.ix_start = h->rd_ixstart.as<uint32_t>();
    t.ix_rule = h->rd_ixrule.as<uint32_t>();
    t.free_rule = h->rd_free.as<uint32_t>();
    hipMemcpy(h->rd_tab.p, &t, sizeof(t), hipMemcpyHostToDevice);
    return SH_OK;
}

// general engine (sh_nfa.h): every other lowered shape
static int compile_nfa(sh_handle* h, const sh_app_desc* app) {
    nf_table* T = new nf_table();
    std::string err;
    if (nf_lower(app, T, &err)) {
        delete T;
        return fail(h, SH_E_UNSUPPORTED, err);
    }
    const char* capenv = getenv("SH_NFA_CAPS");  // list,se,node,hold,sched (tests: force growth)
    if (capenv) sscanf(capenv, "%d,%d,%d,%d,%d,%d", &h->caps[0], &h->caps[1], &h->caps[2], &h->caps[3], &h->caps[4],
                       &h->caps[5]);
    nf_set_caps(T, h->caps[0], h->caps[1], h->caps[2], h->caps[3], h->caps[4], h->caps[5]);
    h->T = T;
    h->mode = 1;
    int nout = 0;
    for (int q = 0; q < T->n_queries; q++) nout = std::max(nout, T->q[q].n_out);
    h->n_out = nout;
    h->partitioned = T->partitioned;
    for (int q = 0; q < T->n_queries; q++)
        for (int o = 0; o < T->q[q].n_out; o++)
            if (T->q[q].out_pc[o] == NF_PC_LIST) h->has_lists = true;
    if (T->partitioned && T->has_absent && !getenv("SH_NO_MAP_ORDER")) {
        std::vector<int> ids;
        for (int q = 0; q < T->n_queries; q++)
            for (int p = 0; p < T->q[q].n_proc; p++)
                if (nf_has_sched(T->q[q].proc[p])) ids.push_back(q * NF_MAX_PROC + p);
        h->sm_on = true;
        h->sm.init(ids, NF_MAX_QUERIES * NF_MAX_PROC);
        h->n_rank.resize(NF_MAX_QUERIES * NF_MAX_PROC);
    }
    return SH_OK;
}

// FNV-1a over the lowered program as compiled (before any capacity growth):
// snapshot images restore only into a handle compiled from the same app
static uint64_t fnv1a(const void* p, size_t n, uint64_t h = 1469598103934665603ull) {
    const uint8_t* b = (const uint8_t*)p;
    for (size_t i = 0; i < n; i++) h = (h ^ b[i]) * 1099511628211ull;
    return h;
}
static uint64_t program_fingerprint(const sh_handle* h) {
    uint64_t f = fnv1a(&h->mode, sizeof(h->mode));
    if (h->mode == 1 && h->T) return fnv1a(h->T, sizeof(nf_table), f);
    f = fnv1a(&h->prog, sizeof(h->prog), f);
    for (const auto& t : h->stream_types) f = fnv1a(t.data(), t.size() * sizeof(int32_t), f);
    return f;
}

int sh_compile(const sh_app_desc* app, sh_handle** out) {
    if (!app || !out) return SH_E_INVALID_ARG;
    *out = nullptr;
    sh_handle* h = new sh_handle();
    *out = h;
    if (app->version != SH_DESC_VERSION) return fail(h, SH_E_INVALID_ARG, "descriptor version mismatch");
    h->app = *app;
    for (int32_t q = 0; q < app->n_queries; q++)
        for (int32_t o = 0; o < app->queries[q].n_outputs; o++) {
            const int32_t t = app->queries[q].outputs[o].type;
            if ((int32_t)h->out_types.size() <= o) h->out_types.push_back(t);
            else if (h->out_types[o] != t) h->out_types[o] = -2;
        }
    if (app->n_streams < 1 || app->n_streams > SHP_MAX_STREAMS)
        return fail(h, SH_E_UNSUPPORTED, "device engine: 1..8 streams per app");
    for (int s = 0; s < app->n_streams; s++) {
        const sh_stream_def& sd = app->streams[s];
        if (sd.n_attrs > 32) return fail(h, SH_E_UNSUPPORTED, "device engine: at most 32 attributes per stream");
        h->stream_types.emplace_back(sd.attr_types, sd.attr_types + sd.n_attrs);
    }
    int rc = compile_chain(h, app);
    if (rc == SH_E_UNSUPPORTED) {
        const std::string chain_err = h->err;
        const bool rules = compile_rules(h, app) == SH_OK;
        const std::string rules_err = rules ? std::string() : h->err;
        rc = compile_nfa(h, app);
        if (rc && rules) {
            // rule sets beyond the general engine's query table: bulk path only
            rc = SH_OK;
            h->mode = 2;
            h->n_out = h->r_nout;
            h->partitioned = h->r_partitioned;
            h->err.clear();
        } else if (rc) {
            h->err = chain_err + "; " + rules_err + "; " + h->err;
        }
    }
    if (rc) return rc;
    h->fp = program_fingerprint(h);
    h->has_device = device_available();
    if (!h->has_device) return SH_OK;  // compile is host-only; processing needs a device
    hipStreamCreateWithFlags(&h->own_stream, hipStreamNonBlocking);
    h->stream = h->own_stream;
    for (auto& e : h->ev) hipEventCreate(&e);
    if (h->d_prog.ensure(sizeof(shp_program)) || h->d_cols_desc.ensure(sizeof(shd_cols)) || h->d_err.ensure(64))
        return fail(h, SH_E_OOM, "hipMalloc failed");
    hipMemcpy(h->d_prog.p, &h->prog, sizeof(shp_program), hipMemcpyHostToDevice);
    if (h->mode == 1) {
        if (h->d_T.ensure(sizeof(nf_table)) || h->d_ncols.ensure(sizeof(nf_cols)) || h->n_ctl.ensure(256))
            return fail(h, SH_E_OOM, "hipMalloc failed");
        hipMemset(h->n_ctl.p, 0, 256);
        h->n_ctr.set_view(h->n_ctl.as<uint8_t>(), 8);
        h->n_err.set_view(h->n_ctl.as<uint8_t>() + 8, 8);
        h->n_sev_ctr.set_view(h->n_ctl.as<uint8_t>() + 16, 64);
        hipMemcpy(h->d_T.p, h->T, sizeof(nf_table), hipMemcpyHostToDevice);
    }
    if (h->has_rules && upload_rules(h)) return SH_E_OOM;
    h->stores.resize(app->n_streams);
    for (int s = 0; s < app->n_streams; s++) {
        h->stores[s].cols.resize(h->stream_types[s].size());
        h->stores[s].nuls.resize(h->stream_types[s].size());
        h->stores[s].has_nul.assign(h->stream_types[s].size(), false);
    }
    return SH_OK;
}

void sh_destroy(sh_handle* h) {
    if (!h) return;
    if (getenv("SH_HOST_PROF") && h->hp_n[0]) {
        static const char* names[10] = {"push", "timers", "process", "history", "place", "drain",
                                        "hist_copy", "hist_apply", "hist_rank", "hist_records"};
        fprintf(stderr, "[sh host profile]");
        for (int i = 0; i < 9; i++) fprintf(stderr, " %s %.1f ms / %lld", names[i], h->hp_ms[i], (long long)h->hp_n[i]);
        fprintf(stderr, " %s %lld", names[9], (long long)h->hp_n[9]);
        fprintf(stderr, "\n");
    }
    if (h->has_device) {
        hipStreamSynchronize(h->stream);
        h->pin_in.release();
        h->pin_stage.release();
        h->pin_rd.release();
        h->pin_out.release();
        h->pin_hist.release();
        h->n_tmin.release();
        h->n_armed.release();
        h->n_klist[0].release();
        h->n_klist[1].release();
        h->n_klist_n.release();
        h->n_arm_log.release();
        h->n_arm_ctr.release();
        h->n_slot_s.release();
        h->n_slot_k.release();
        h->v_sts.release();
        h->v_mpos.release();
        h->v_flag.release();
        h->v_cnts.release();
        h->v_mid_ts.release();
        h->v_dir.release();
        for (auto& b : h->v_scol) b.release();
        for (auto& b : h->v_mid) b.release();
        DevBuf* bufs[] = {&h->d_prog, &h->d_cols_desc, &h->d_kstate, &h->d_err, &h->w_ts, &h->w_stream, &h->w_row,
                          &h->w_pstage, &h->w_orows,
                          &h->w_key, &h->w_keys_a, &h->w_keys_b, &h->w_idx_a, &h->w_idx_b, &h->w_hist, &h->w_scan,
                          &h->w_seg, &h->w_cnt, &h->w_off, &h->w_tmp, &h->w_ctr, &h->w_oseq, &h->w_ots,
                          &h->w_ovals, &h->w_onulls, &h->w_inv};
        for (DevBuf* b : bufs) b->release();
        DevBuf* nbufs[] = {&h->d_T, &h->d_T_old, &h->d_ncols, &h->n_kstate, &h->n_kstate2, &h->n_save, &h->n_recs,
                           &h->n_ctr, &h->n_err, &h->n_cand, &h->n_sel, &h->n_bid, &h->w_oq,
                           &h->rd_rules, &h->rd_ixval, &h->rd_ixstart, &h->rd_ixrule, &h->rd_free, &h->rd_tab, &h->rd_img,
                           &h->r_tsr, &h->v_ts32, &h->v_sts32, &h->v_mid_ts32,
                           &h->n_ctl,
                           &h->r_rec, &h->r_keys, &h->r_g, &h->r_sk, &h->r_sv, &h->r_hist, &h->r_scan, &h->r_run};
        for (DevBuf* b : nbufs) b->release();
        for (auto& st : h->stores) {
            for (auto& c : st.cols) c.release();
            for (auto& c : st.nuls) c.release();
        }
        for (auto& e : h->ev)
            if (e) hipEventDestroy(e);
        hipStreamDestroy(h->own_stream);
    }
    delete h->T;
    delete h;
}

static int nf_push(sh_handle* h, const sh_batch* b, int64_t r0, const uint32_t* index = nullptr, int64_t call_n = 0,
                   int64_t call_last = 0);
static int nf_start(sh_handle* h);
static int nf_timers(sh_handle* h, int64_t now, bool wall = false);
static int nf_next_due(sh_handle* h, int64_t* out);

static int push_impl(sh_handle* h, const sh_batch* b, const uint32_t* index, int64_t call_n, int64_t call_last) {
    HpScope hp_(h, 0);
    if (h && h->poisoned) return fail(h, SH_E_INVALID_ARG, "handle unusable after a failed restore");
    if (!h || !b) return SH_E_INVALID_ARG;
    if (!h->has_device) return fail(h, SH_E_NO_DEVICE, "no HIP device: the matcher has no CPU fallback");
    if (b->stream < 0 || b->stream >= h->app.n_streams) return fail(h, SH_E_INVALID_ARG, "bad stream index");
    if (b->on_device) return fail(h, SH_E_UNSUPPORTED, "device batches go through sh_run_device");
    if (h->mode == 2)
        return fail(h, SH_E_UNSUPPORTED, "rule sets larger than the general engine's query table run through "
                                         "sh_run_device only");
    if (h->coord_on && !index)
        return fail(h, SH_E_INVALID_ARG, "a key-sharded handle takes its events through sh_push_batch_part");
    if (index) {
        if (!h->coord_on) return fail(h, SH_E_INVALID_ARG, "sh_push_batch_part needs sh_set_coordinator first");
        if (call_n <= 0 || b->n < 0 || b->n > call_n || call_n > 0xFFFFFFFFll)
            return fail(h, SH_E_INVALID_ARG, "bad key-sharded call size");
        for (int64_t i = 0; i < b->n; i++)
            if ((int64_t)index[i] >= call_n || (i && index[i] <= index[i - 1]))
                return fail(h, SH_E_INVALID_ARG, "call positions must ascend below call_n");
        if (b->n == 0) return nf_push(h, b, h->stores[b->stream].rows, index, call_n, call_last);
    }
    if (b->n <= 0) return SH_OK;
    auto& st = h->stores[b->stream];
    const auto& types = h->stream_types[b->stream];
    const int64_t r0 = st.rows;
    size_t pin_need = 0;
    for (size_t a = 0; a < types.size(); a++) pin_need += (size_t)b->n * type_width(types[a]);
    if (h->pin_in.ensure(pin_need)) return fail(h, SH_E_OOM, "pinned staging");
    size_t pin_off = 0;
    bool caller_copy = false;  // a copy reads the caller's memory directly (null masks)
    for (size_t a = 0; a < types.size(); a++) {
        const int w = type_width(types[a]);
        if (st.cols[a].ensure((size_t)(r0 + b->n) * w)) return fail(h, SH_E_OOM, "column store");
        // through pinned staging (the sync below completes the copy before reuse)
        memcpy(h->pin_in.as<void>(pin_off), b->cols[a], (size_t)b->n * w);
        hipMemcpyAsync((uint8_t*)st.cols[a].p + r0 * w, h->pin_in.as<void>(pin_off), b->n * w, hipMemcpyHostToDevice,
                       h->stream);
        pin_off += (size_t)b->n * w;
        const uint8_t* nm = b->nulls ? b->nulls[a] : nullptr;
        if (nm || st.has_nul[a]) {
            if (!st.has_nul[a]) {
                if (st.nuls[a].ensure((size_t)(r0 + b->n))) return fail(h, SH_E_OOM, "null mask");
                hipMemsetAsync(st.nuls[a].p, 0, r0, h->stream);
                st.has_nul[a] = true;
            } else if (st.nuls[a].ensure((size_t)(r0 + b->n))) {
                return fail(h, SH_E_OOM, "null mask");
            }
            if (nm) {
                hipMemcpyAsync((uint8_t*)st.nuls[a].p + r0, nm, b->n, hipMemcpyHostToDevice, h->stream);
                caller_copy = true;
            }
            else
                hipMemsetAsync((uint8_t*)st.nuls[a].p + r0, 0, b->n, h->stream);
        }
    }
    st.rows += b->n;
    // the copies read pin_in, which the general engine's push does not touch (it
    // stages through pin_stage) and which is next written after its syncs; the
    // staged engines reuse pin_in on the next call: complete the copies first
    if (caller_copy || h->mode != 1) hipStreamSynchronize(h->stream);
    if (h->mode == 1) return nf_push(h, b, r0, index, call_n, call_last);
    for (int64_t i = 0; i < b->n; i++) {
        h->st_ts.push_back(b->ts[i]);
        h->st_stream.push_back((uint8_t)b->stream);
        h->st_row.push_back((uint32_t)(r0 + i));
        int32_t k = h->partitioned ? (b->keys ? b->keys[i] : -1) : 0;
        h->st_key.push_back(k);
        if (k + 1 > h->max_key) h->max_key = k + 1;
    }
    h->seq_next += b->n;
    return SH_OK;
}

int sh_push_batch(sh_handle* h, const sh_batch* b) { return push_impl(h, b, nullptr, 0, 0); }

int sh_push_batch_part(sh_handle* h, const sh_batch* b, const uint32_t* index, int64_t call_n, int64_t call_last_ts) {
    if (!h || !b || (b->n > 0 && !index)) return SH_E_INVALID_ARG;
    static const uint32_t none = 0;
    return push_impl(h, b, index ? index : &none, call_n, call_last_ts);
}

int sh_set_coordinator(sh_handle* h, const sh_coordinator* c) {
    if (!h || !c || !c->history || !c->select || !c->min_time) return SH_E_INVALID_ARG;
    if (h->mode != 1)
        return fail(h, SH_E_UNSUPPORTED, "key-sharded streaming coordinates the general engine's schedulers only");
    if (!h->partitioned) return fail(h, SH_E_UNSUPPORTED, "an unpartitioned app does not shard by key");
    if (h->started || h->tick != 1) return fail(h, SH_E_INVALID_ARG, "set the coordinator before sh_start");
    h->coord = *c;
    h->coord_on = true;
    return SH_OK;
}

int sh_set_partition_keys(sh_handle* h, int32_t first_key, int32_t n, const uint16_t* utf16, const int64_t* offsets) {
    if (!h || first_key < 0 || n < 0 || (n && (!utf16 || !offsets))) return SH_E_INVALID_ARG;
    h->sm.set_keys(first_key, n, utf16, offsets);
    return SH_OK;
}

int sh_advance_time(sh_handle* h, int64_t now_ms) {
    if (h && h->poisoned) return fail(h, SH_E_INVALID_ARG, "handle unusable after a failed restore");
    if (!h) return SH_E_INVALID_ARG;
    if (h->mode != 1) return SH_OK;  // the chain / window engines have no timer states
    if (!h->has_device) return fail(h, SH_E_NO_DEVICE, "no HIP device: the matcher has no CPU fallback");
    if (now_ms < h->clock) return SH_OK;  // TimestampGeneratorImpl: time never goes back
    if (!h->started) {
        h->clock = now_ms;
        return SH_OK;  // schedulers exist from SiddhiAppRuntime.start on
    }
    if (!h->app.playback) {
        // wall clock: the clock passes through every queued notify time in order
        for (;;) {
            int64_t t;
            int rc = nf_next_due(h, &t);
            if (rc) return rc;
            if (t > now_ms) break;
            h->clock = std::max(h->clock, t);
            rc = nf_timers(h, h->clock, true);
            if (rc) return rc;
        }
        h->clock = now_ms;
        return SH_OK;
    }
    h->clock = now_ms;
    return nf_timers(h, now_ms);
}

int sh_start(sh_handle* h) {
    if (h && h->poisoned) return fail(h, SH_E_INVALID_ARG, "handle unusable after a failed restore");
    if (!h) return SH_E_INVALID_ARG;
    if (h->mode != 1) return SH_OK;
    if (!h->has_device) return fail(h, SH_E_NO_DEVICE, "no HIP device: the matcher has no CPU fallback");
    return nf_start(h);
}

static int ensure_keys(sh_handle* h, int32_t nkeys) {
    if (nkeys <= h->nkeys_alloc) return 0;
    int32_t nk = std::max(nkeys, h->nkeys_alloc * 2);
    size_t old = (size_t)h->nkeys_alloc * h->lay.key_bytes;
    if (h->d_kstate.ensure((size_t)nk * h->lay.key_bytes)) return SH_E_OOM;
    hipMemsetAsync((uint8_t*)h->d_kstate.p + old, 0, (size_t)nk * h->lay.key_bytes - old, h->stream);
    h->nkeys_alloc = nk;
    return 0;
}

static int ensure_ws(sh_handle* h, int64_t n) {
    // radix blocks of 4096, padded to whole arrival tiles (<= 2^20 events) for
    // the tile-major segment layout
    const int64_t tiles = (n + 4095) / 4096 + 256;
    int rc = 0;
    rc |= h->w_keys_a.ensure_fresh(n * 4);
    rc |= h->w_keys_b.ensure_fresh(n * 4);
    rc |= h->w_idx_a.ensure_fresh(n * 4);
    rc |= h->w_idx_b.ensure_fresh(n * 4);
    // digit histograms: up to 1024 digits per radix block (10-bit passes)
    rc |= h->w_hist.ensure_fresh(1024 * tiles * 4 + 64);
    size_t sw = std::max(shd_scan_tmp_words(1024 * tiles), shd_scan_tmp_words(n));
    rc |= h->w_scan.ensure_fresh(sw * 4 + 64);
    rc |= h->w_seg.ensure_fresh((3 * n + 4) * 4);
    rc |= h->w_cnt.ensure_fresh(n * 4 + 4);
    rc |= h->w_off.ensure_fresh(n * 4 + 4);
    rc |= h->w_ctr.ensure_fresh(64);
    return rc ? SH_E_OOM : 0;
}

// segment -> advance -> place for one device batch; fills outputs into the
// w_o* buffers (or caller-provided device buffers) and returns the match count
static int run_batch(sh_handle* h, const shd_batch& B, int32_t nkeys, const shd_cols& cols, uint64_t* out_seq,
                     int64_t* out_ts, int64_t* out_vals, uint8_t* out_nulls, int64_t out_cap, int64_t* n_matches,
                     bool timed) {
    hipStream_t st = h->stream;
    const int64_t n = B.n;
    if (ensure_ws(h, n)) return fail(h, SH_E_OOM, "workspace");
    hipMemcpyAsync(h->d_cols_desc.p, &cols, sizeof(shd_cols), hipMemcpyHostToDevice, st);
    if (h->tmp_cap < n + (1 << 16)) {
        h->tmp_cap = n + (1 << 16);
        if (h->w_tmp.ensure_fresh((size_t)h->tmp_cap * (3 + h->n_out) * 8)) return fail(h, SH_E_OOM, "emit buffer");
    }
    // keep a copy of the key state: an emit-buffer overflow restores and reruns
    DevBuf backup;
    for (int attempt = 0; attempt < 24; attempt++) {
        const size_t kbytes = (size_t)nkeys * h->lay.key_bytes;
        if (attempt == 0 && !timed) {
            if (backup.ensure_fresh(kbytes)) return fail(h, SH_E_OOM, "state backup");
            hipMemcpyAsync(backup.p, h->d_kstate.p, kbytes, hipMemcpyDeviceToDevice, st);
        }
        hipMemsetAsync(h->w_cnt.p, 0, n * 4, st);
        hipMemsetAsync(h->w_ctr.p, 0, 8, st);
        hipMemsetAsync(h->d_err.p, 0, 8, st);
        if (timed) hipEventRecord(h->ev[0], st);
        shd_segment_ws ws;
        ws.keys_a = h->w_keys_a.as<uint32_t>();
        ws.keys_b = h->w_keys_b.as<uint32_t>();
        ws.idx_a = h->w_idx_a.as<uint32_t>();
        ws.idx_b = h->w_idx_b.as<uint32_t>();
        ws.hist = h->w_hist.as<uint32_t>();
        ws.scan_tmp = h->w_scan.as<uint32_t>();
        ws.seg_off = h->w_seg.as<uint32_t>();
        ws.cap = n;
        const uint32_t* perm = nullptr;
        const uint32_t* skeys = nullptr;
        int rc = shd_segment(&B, nkeys, &ws, st, &perm, &skeys);
        if (rc) return fail(h, SH_E_HIP, "segment launch failed");
        if (timed) hipEventRecord(h->ev[1], st);
        shd_emit em;
        em.tmp = h->w_tmp.as<uint64_t>();
        em.tmp_ctr = h->w_ctr.as<unsigned long long>();
        em.tmp_cap = h->tmp_cap;
        em.match_cnt = h->w_cnt.as<uint32_t>();
        em.err = h->d_err.as<int32_t>();
        bool fast_ok = true;  // register-only filters need null-free columns
        for (int s2 = 0; s2 < SHP_MAX_STREAMS; s2++)
            for (int a = 0; a < 32; a++) fast_ok = fast_ok && cols.nul[s2][a] == nullptr;
        rc = shd_advance(h->d_prog.as<shp_program>(), &h->lay, h->d_kstate.as<uint8_t>(), nkeys, &B, perm, skeys,
                         ws.seg_off, h->d_cols_desc.as<shd_cols>(), &em, st, fast_ok ? 1 : 0);
        if (rc) return fail(h, SH_E_HIP, "advance launch failed");
        if (timed) hipEventRecord(h->ev[2], st);
        int32_t herr[2] = {0, 0};
        unsigned long long nrec = 0;
        hipMemcpyAsync(herr, h->d_err.p, 8, hipMemcpyDeviceToHost, st);
        hipMemcpyAsync(&nrec, h->w_ctr.p, 8, hipMemcpyDeviceToHost, st);
        if (hipStreamSynchronize(st) != hipSuccess) return fail(h, SH_E_HIP, "device error in advance");
        if (herr[0] == 2) return fail(h, SH_E_INVALID_ARG, "partition key id >= n_keys");
        if (herr[0]) {
            // a partial-match list outgrew its capacity: grow every key's lists x4
            // (the reference's lists are unbounded LinkedLists) and rerun the batch
            if (h->lay.cap >= (1 << 20)) return fail(h, SH_E_STATE_OVERFLOW, "partial-match list overflow");
            shp_layout old = h->lay, nl;
            set_layout(nl, h->prog, old.cap * 4);
            DevBuf fresh;
            if (fresh.ensure_fresh((size_t)h->nkeys_alloc * nl.key_bytes)) return fail(h, SH_E_OOM, "state growth");
            if (timed) {
                hipMemsetAsync(fresh.p, 0, (size_t)h->nkeys_alloc * nl.key_bytes, st);
            } else {
                hipMemcpyAsync(h->d_kstate.p, backup.p, kbytes, hipMemcpyDeviceToDevice, st);
                shd_relayout(h->d_kstate.as<uint8_t>(), &old, fresh.as<uint8_t>(), &nl, h->nkeys_alloc,
                             h->prog.n_states, h->n_out, st);
            }
            hipStreamSynchronize(st);
            h->d_kstate.release();
            h->d_kstate = fresh;
            fresh.p = nullptr;
            fresh.bytes = 0;
            h->lay = nl;
            if (!timed) {
                const size_t nkb = (size_t)nkeys * h->lay.key_bytes;
                if (backup.ensure_fresh(nkb)) return fail(h, SH_E_OOM, "state backup");
                hipMemcpyAsync(backup.p, h->d_kstate.p, nkb, hipMemcpyDeviceToDevice, st);
            }
            continue;
        }
        if (herr[1]) {
            // emit buffer too small: restore state, grow, rerun
            if (timed) {
                h->tmp_cap *= 4;
                if (h->w_tmp.ensure_fresh((size_t)h->tmp_cap * (3 + h->n_out) * 8))
                    return fail(h, SH_E_OOM, "emit buffer");
                hipMemsetAsync(h->d_kstate.p, 0, kbytes, st);  // timed runs start from fresh state
                continue;
            }
            hipMemcpyAsync(h->d_kstate.p, backup.p, kbytes, hipMemcpyDeviceToDevice, st);
            h->tmp_cap *= 4;
            if (h->w_tmp.ensure_fresh((size_t)h->tmp_cap * (3 + h->n_out) * 8))
                return fail(h, SH_E_OOM, "emit buffer");
            continue;
        }
        // total matches = sum of per-event counts (<= nrec, chunk tails unused)
        if (timed) hipEventRecord(h->ev[2], st);
        rc = shd_emit_place(&em, h->n_out, n, h->w_off.as<uint32_t>(), h->w_scan.as<uint32_t>(), (int64_t)nrec, &B,
                            nullptr, nullptr, nullptr, nullptr, st);
        (void)rc;
        uint32_t last_off = 0, last_cnt = 0;
        hipMemcpyAsync(&last_off, h->w_off.as<uint32_t>() + (n - 1), 4, hipMemcpyDeviceToHost, st);
        hipMemcpyAsync(&last_cnt, h->w_cnt.as<uint32_t>() + (n - 1), 4, hipMemcpyDeviceToHost, st);
        hipStreamSynchronize(st);
        const int64_t total = (int64_t)last_off + last_cnt;
        *n_matches = total;
        if (total > out_cap) {
            backup.release();
            return SH_E_MORE;
        }
        // placement into the ordered output
        rc = shd_emit_place(&em, h->n_out, 0, h->w_off.as<uint32_t>(), h->w_scan.as<uint32_t>(), (int64_t)nrec, &B,
                            out_seq, out_ts, out_vals, out_nulls, st);
        if (timed) hipEventRecord(h->ev[3], st);
        if (hipStreamSynchronize(st) != hipSuccess) return fail(h, SH_E_HIP, "device error in placement");
        if (timed) {
            hipEventElapsedTime(&h->times.segment_ms, h->ev[0], h->ev[1]);
            hipEventElapsedTime(&h->times.advance_ms, h->ev[1], h->ev[2]);
            hipEventElapsedTime(&h->times.emit_ms, h->ev[2], h->ev[3]);
            hipEventElapsedTime(&h->times.total_ms, h->ev[0], h->ev[3]);
            h->times.advance_launches++;
        }
        backup.release();
        return SH_OK;
    }
    backup.release();
    return fail(h, SH_E_OOM, "emit buffer kept overflowing");
}

// ================================================================ general engine (mode 1)
// sh_nfa.h lanes over the radix segment; emissions are placed by an exclusive
// scan of per-run counts. A lane error (an arena / list / queue / emission
// buffer full) restores the touched keys' blocks, grows the capacity and replays.
// the due scan's key filter (SH_NO_ARMED: scan every key)
static uint8_t* armed_flags(sh_handle* h) {
    static const bool off = getenv("SH_NO_ARMED") != nullptr;
    return off ? nullptr : h->n_armed.as<uint8_t>();
}

static int bits_for(uint64_t v);
static nf_cols nf_store_cols(sh_handle* h) {
    nf_cols c;
    memset(&c, 0, sizeof(c));
    for (int s = 0; s < h->app.n_streams; s++)
        for (size_t a = 0; a < h->stream_types[s].size(); a++) {
            c.col[s][a] = h->stores[s].cols[a].p;
            c.nul[s][a] = h->stores[s].has_nul[a] ? (const uint8_t*)h->stores[s].nuls[a].p : nullptr;
        }
    c.sched_armed = armed_flags(h);
    if (c.sched_armed && h->n_arm_log.p) {
        c.arm_log = h->n_arm_log.as<int32_t>();
        c.arm_ctr = h->n_arm_ctr.as<unsigned long long>();
        c.arm_cap = (uint64_t)h->n_nkeys;
    }
    if (h->sm_on) {
        c.sev = h->n_sev.as<uint64_t>();
        c.sev_ctr = h->n_sev_ctr.as<unsigned long long>();
        c.sev_cap = (uint64_t)h->sev_cap;
    }
    if (h->has_lists && h->n_lst.p) {
        c.lst = h->n_lst.as<uint64_t>();
        c.lst_ctr = h->n_lst_ctr.as<unsigned long long>();
        c.lst_cap = (uint64_t)h->lst_cap;
    }
    return c;
}

// the List buffer of a launch: allocated once (grown on NF_E_LST), counter zeroed
static int nf_lst_ready(sh_handle* h) {
    if (!h->has_lists) return 0;
    if (!h->n_lst.p) {
        h->lst_cap = 1 << 16;
        if (h->n_lst.ensure_fresh((size_t)h->lst_cap * 8) || h->n_lst_ctr.ensure_fresh(64)) return SH_E_OOM;
    }
    return hipMemsetAsync(h->n_lst_ctr.p, 0, 8, h->stream) == hipSuccess ? 0 : SH_E_HIP;
}
static int nf_lst_grow(sh_handle* h) {
    hipStreamSynchronize(h->stream);
    if (h->n_lst.ensure_fresh((size_t)h->lst_cap * 4 * 8)) return SH_E_OOM;
    h->lst_cap *= 4;
    return 0;
}

static int nf_ensure_keys(sh_handle* h, int32_t nkeys) {
    if (nkeys <= h->n_nkeys) return 0;
    const int32_t nk = std::max(nkeys, h->n_nkeys * 2);
    const size_t kb = (size_t)h->T->key_words * 8;
    const size_t old = (size_t)h->n_nkeys * kb, need = (size_t)nk * kb;
    hipStreamSynchronize(h->stream);
    if (h->n_kstate.ensure(need)) return SH_E_OOM;
    hipMemsetAsync((uint8_t*)h->n_kstate.p + old, 0, need - old, h->stream);
    if (h->n_armed.ensure((size_t)nk)) return SH_E_OOM;
    hipMemsetAsync((uint8_t*)h->n_armed.p + h->n_nkeys, 0, (size_t)(nk - h->n_nkeys), h->stream);
    if (h->n_klist[0].ensure((size_t)nk * 4) || h->n_klist[1].ensure((size_t)nk * 4) ||
        h->n_arm_log.ensure((size_t)nk * 4))
        return SH_E_OOM;
    if (!h->n_klist_n.p) {
        if (h->n_klist_n.ensure(16) || h->n_arm_ctr.ensure(8)) return SH_E_OOM;
        hipMemsetAsync(h->n_klist_n.p, 0, 16, h->stream);
        hipMemsetAsync(h->n_arm_ctr.p, 0, 8, h->stream);
    }
    if (h->sm_on)
        for (int s : h->sm.used)
            if (h->n_rank[s].ensure((size_t)nk * 8)) return SH_E_OOM;
    h->n_nkeys = nk;
    return 0;
}

// scheduler-history buffer for a launch processing `events` events / keys
// (zero: clear the counter here; the launch paths clear the whole counter block)
static int nf_sev_ready(sh_handle* h, int64_t events, bool zero = true) {
    if (!h->sm_on) return 0;
    const int64_t need = std::max<int64_t>(4096, 2 * (events + 64) * (int64_t)h->sm.used.size());
    if (need > h->sev_cap) {
        hipStreamSynchronize(h->stream);
        if (h->n_sev.ensure_fresh((size_t)need * 16) || h->n_sev_ctr.ensure_fresh(64)) return SH_E_OOM;
        h->sev_cap = need;
    }
    if (!zero) return 0;
    return hipMemsetAsync(h->n_sev_ctr.p, 0, 8, h->stream) == hipSuccess ? 0 : SH_E_HIP;
}

// the counter block's record counter, error word and history counter, zeroed at once
static void nf_ctl_zero(sh_handle* h) { hipMemsetAsync(h->n_ctl.p, 0, 24, h->stream); }

// replay the launch's getState history on the host models and upload the
// changed ranks (before the next due scan, on the same stream)
// pin_rd slots of the counter block read back after a launch (nf_ctl_read)
enum { PR_CTL = 40 };
// the launch's counter block (records, error, history count) into pin_rd[PR_CTL..+24),
// read with the caller's next sync
static void nf_ctl_read(sh_handle* h) {
    hipMemcpyAsync(h->pin_rd.as<uint8_t>() + PR_CTL, h->n_ctl.p, 24, hipMemcpyDeviceToHost, h->stream);
}
static unsigned nf_ctl_err(sh_handle* h) { return *(const unsigned*)(h->pin_rd.as<uint8_t>() + PR_CTL + 8); }
static int64_t nf_ctl_nrec(sh_handle* h) { return *(const int64_t*)(h->pin_rd.as<uint8_t>() + PR_CTL); }
static int64_t nf_ctl_nsev(sh_handle* h) { return *(const int64_t*)(h->pin_rd.as<uint8_t>() + PR_CTL + 16); }

// the models' ranks after a replay: whole array after a resize, else the touched
// keys (uploaded on the stream, ahead of the next due pass)
static int nf_rank_upload(sh_handle* h) {
    hipStream_t st = h->stream;
    std::vector<int32_t> ks;
    std::vector<uint64_t> vs;
    for (int s : h->sm.used) {
        ShJMap& M = h->sm.maps[s];
        if (M.rerank_all) {
            const int32_t nk = h->n_nkeys;
            if (h->pin_rk.ensure((size_t)nk * 8)) return fail(h, SH_E_OOM, "pinned staging");
            uint64_t* r = h->pin_rk.as<uint64_t>();
            for (int32_t k = 0; k < nk; k++) r[k] = M.present(k) ? M.rank(k) : ~0ull;
            hipMemcpyAsync(h->n_rank[s].p, r, (size_t)nk * 8, hipMemcpyHostToDevice, st);
            if (hipStreamSynchronize(st) != hipSuccess) return fail(h, SH_E_HIP, "rank upload");  // (rare: after a resize)
        } else if (!M.dirty.empty()) {
            ks.clear();
            vs.clear();
            std::sort(M.dirty.begin(), M.dirty.end());
            M.dirty.erase(std::unique(M.dirty.begin(), M.dirty.end()), M.dirty.end());
            for (int32_t k : M.dirty)
                if (M.present(k) && k < h->n_nkeys) {
                    ks.push_back(k);
                    vs.push_back(M.rank(k));
                }
            const size_t m = ks.size();
            if (m) {
                if (h->pin_rk.ensure(m * 12) || h->n_rk_keys.ensure_fresh(m * 4) || h->n_rk_vals.ensure_fresh(m * 8))
                    return fail(h, SH_E_OOM, "rank upload");
                memcpy(h->pin_rk.p, vs.data(), m * 8);
                memcpy(h->pin_rk.as<uint8_t>(m * 8), ks.data(), m * 4);
                hipMemcpyAsync(h->n_rk_vals.p, h->pin_rk.p, m * 8, hipMemcpyHostToDevice, st);
                hipMemcpyAsync(h->n_rk_keys.p, h->pin_rk.as<uint8_t>(m * 8), m * 4, hipMemcpyHostToDevice, st);
                nfd_rank_scatter(h->n_rk_keys.as<int32_t>(), h->n_rk_vals.as<uint64_t>(), (int64_t)m,
                                 h->n_rank[s].as<uint64_t>(), st);
                // no sync: the next launch follows on this stream, and pin_rk is next
                // written after that launch's error read-back has synchronised
            }
        }
        M.rerank_all = false;
        M.dirty.clear();
    }
    return SH_OK;
}

// replay the deferred launches' history (in launch order: a timer launch's
// removals follow its own getState calls, so each launch is one apply) and
// upload the changed ranks; before every use of the ranks or the models
static int nf_sev_flush(sh_handle* h) {
    if (h->sev_pend.empty()) return SH_OK;
    HpScope hp_(h, 3);
    if (hipStreamSynchronize(h->stream) != hipSuccess) return fail(h, SH_E_HIP, "scheduler history");
    {
        HpScope ha_(h, 7);
        for (const auto& pr : h->sev_pend)
            if (!h->sm.apply(h->pin_hist.as<uint64_t>((size_t)pr.first * 16), (size_t)pr.second))
                return fail(h, SH_E_UNSUPPORTED, "more than 2^26 scheduler map bins (keys waiting on one absent state)");
    }
    h->sev_pend.clear();
    h->hist_used = 0;
    HpScope hr_(h, 8);
    return nf_rank_upload(h);
}

// after a launch: its scheduler history. Single process: copied behind the
// launch (no synchronisation) and replayed by nf_sev_flush before the ranks are
// next needed. Key-sharded: exchanged now (the coordinator's history call is a
// collective every rank makes per launch), replayed and uploaded.
// counted: nf_ctl_read ran before the caller's last sync (the history count is in pin_rd)
static int nf_sev_apply(sh_handle* h, bool counted = false) {
    if (!h->sm_on) return SH_OK;
    hipStream_t st = h->stream;
    if (h->pin_sev.ensure(64)) return fail(h, SH_E_OOM, "pinned staging");
    int64_t n;
    {
        HpScope hc_(h, 6);
        if (counted) {
            n = nf_ctl_nsev(h);
        } else {
            hipMemcpyAsync(h->pin_sev.p, h->n_sev_ctr.p, 8, hipMemcpyDeviceToHost, st);
            if (hipStreamSynchronize(st) != hipSuccess) return fail(h, SH_E_HIP, "scheduler history");
            n = (int64_t)*h->pin_sev.as<unsigned long long>();
        }
        h->hp_n[9] += n;
        if (!h->coord_on) {
            if (n == 0) return SH_OK;
            const size_t need = (size_t)(h->hist_used + n) * 16;
            if (need > h->pin_hist.bytes) {
                // grow, keeping the records already copied (their copies must land first)
                if (hipStreamSynchronize(st) != hipSuccess) return fail(h, SH_E_HIP, "scheduler history");
                PinBuf nb;
                if (nb.ensure(need)) return fail(h, SH_E_OOM, "pinned staging");
                if (h->hist_used) memcpy(nb.p, h->pin_hist.p, (size_t)h->hist_used * 16);
                h->pin_hist.release();
                h->pin_hist = nb;
                nb.p = nullptr;
                nb.bytes = 0;
            }
            hipMemcpyAsync(h->pin_hist.as<uint8_t>((size_t)h->hist_used * 16), h->n_sev.p, (size_t)n * 16,
                           hipMemcpyDeviceToHost, st);
            h->sev_pend.emplace_back(h->hist_used, n);
            h->hist_used += n;
            return SH_OK;
        }
        if (h->pin_sev.ensure((size_t)std::max<int64_t>(n, 1) * 16)) return fail(h, SH_E_OOM, "pinned staging");
        if (n) hipMemcpyAsync(h->pin_sev.p, h->n_sev.p, (size_t)n * 16, hipMemcpyDeviceToHost, st);
        if (hipStreamSynchronize(st) != hipSuccess) return fail(h, SH_E_HIP, "scheduler history");
    }
    HpScope hp_(h, 3);
    const uint64_t* recs = h->pin_sev.as<uint64_t>();
    // the launch's history of every rank: the maps model the one state map all
    // keys share (the same launch ticks on every rank keep the stamps comparable)
    const uint64_t* all = nullptr;
    int64_t n_all = 0;
    if (h->coord.history(h->coord.user, recs, n, &all, &n_all) || n_all < 0 || (n_all && !all))
        return fail(h, SH_E_INVALID_ARG, "coordinator: history exchange failed");
    if (n_all == 0) return SH_OK;
    {
        HpScope ha_(h, 7);
        if (!h->sm.apply(all, (size_t)n_all))
            return fail(h, SH_E_UNSUPPORTED, "more than 2^26 scheduler map bins (keys waiting on one absent state)");
    }
    HpScope hr_(h, 8);
    return nf_rank_upload(h);
}

static int nf_upload_table(sh_handle* h) {
    return hipMemcpyAsync(h->d_T.p, h->T, sizeof(nf_table), hipMemcpyHostToDevice, h->stream) == hipSuccess
               ? 0
               : SH_E_HIP;
}

// grow the capacities named by `err` and re-lay every key block
static int nf_grow(sh_handle* h, uint32_t err) {
    int c[6];
    memcpy(c, h->caps, sizeof(c));
    if (err & NF_E_GRP) c[5] *= 2;
    if (err & NF_E_LIST) c[0] *= 2;
    if (err & NF_E_SE) c[1] *= 2;
    if (err & NF_E_NODE) c[2] *= 2;
    if (err & NF_E_HOLD) c[3] *= 2;
    if (err & NF_E_SCHED) c[4] *= 2;
    if (c[0] > 60000 || c[1] > (1 << 22) || c[2] > (1 << 24) || c[3] > (1 << 22) || c[4] > (1 << 20) ||
        c[5] > (1 << 16))
        return fail(h, SH_E_STATE_OVERFLOW, "partial-match state overflow");
    std::unique_ptr<nf_table> old(new nf_table(*h->T));
    nf_set_caps(h->T, c[0], c[1], c[2], c[3], c[4], c[5]);
    memcpy(h->caps, c, sizeof(c));
    hipStream_t st = h->stream;
    if (h->d_T_old.ensure(sizeof(nf_table))) return fail(h, SH_E_OOM, "table");
    hipMemcpyAsync(h->d_T_old.p, old.get(), sizeof(nf_table), hipMemcpyHostToDevice, st);
    nf_upload_table(h);
    if (h->n_nkeys > 0) {
        DevBuf fresh;
        if (fresh.ensure_fresh((size_t)h->n_nkeys * h->T->key_words * 8)) return fail(h, SH_E_OOM, "state growth");
        nfd_relayout(h->d_T_old.as<nf_table>(), h->d_T.as<nf_table>(), h->n_kstate.as<uint64_t>(),
                     fresh.as<uint64_t>(), h->n_nkeys, st);
        if (hipStreamSynchronize(st) != hipSuccess) return fail(h, SH_E_HIP, "relayout");
        h->n_kstate.release();
        h->n_kstate = fresh;
        fresh.p = nullptr;
        fresh.bytes = 0;
    } else {
        hipStreamSynchronize(st);
    }
    return SH_OK;
}

static int nf_ensure_recs(sh_handle* h, int64_t cap) {
    const int stride = NF_REC_HDR + std::max(1, h->n_out);
    if (cap <= h->rec_cap) return 0;
    hipStreamSynchronize(h->stream);
    if (h->n_recs.ensure_fresh((size_t)cap * stride * 8)) return SH_E_OOM;
    h->rec_cap = cap;
    return 0;
}

static nfd_emit nf_emit(sh_handle* h) {
    nfd_emit em;
    em.recs = h->n_recs.as<uint64_t>();
    em.ctr = h->n_ctr.as<unsigned long long>();
    em.cap = h->rec_cap;
    em.stride = NF_REC_HDR + std::max(1, h->n_out);
    em.pad = 0;
    em.match_cnt = h->w_cnt.as<uint32_t>();
    em.err = h->n_err.as<unsigned>();
    return em;
}

// pinned read-back slots (pin_rd): 0 nrec u64, 8 last_off u32, 12 last_cnt u32,
// 16 err u32, 24 due-candidate count u64; the nf_cols image from byte 64
enum { PR_NREC = 0, PR_LOFF = 8, PR_LCNT = 12, PR_ERR = 16, PR_NC = 24, PR_TMIN = 32, PR_COLS = 64 };
// due-key backlogs at least this large are tie-broken on the device when their
// due times span at most kTieBreakSlots milliseconds (SH_TIEBREAK_MIN overrides)
static const int64_t kDeviceTieBreak = [] {
    const char* e = getenv("SH_TIEBREAK_MIN");
    return e ? (int64_t)atoll(e) : (int64_t)4096;
}();
static const int64_t kTieBreakSlots = (int64_t)1 << 22;
static int pin_rd_ready(sh_handle* h) { return h->pin_rd.ensure(PR_COLS + sizeof(nf_cols)); }

// upload the nf_cols image through pinned memory (the caller synchronises the
// stream before the slot is written again)
static void nf_put_cols(sh_handle* h, const nf_cols& cols) {
    // unchanged since the last upload (the common case per call): nothing to copy
    if (h->cols_cached && !memcmp(&h->cols_last, &cols, sizeof(nf_cols))) return;
    memcpy(h->pin_rd.as<nf_cols>(PR_COLS), &cols, sizeof(nf_cols));
    hipMemcpyAsync(h->d_ncols.p, h->pin_rd.as<nf_cols>(PR_COLS), sizeof(nf_cols), hipMemcpyHostToDevice, h->stream);
    h->cols_last = cols;
    h->cols_cached = true;
}

// the deferred rows into the host queue (one sync + one copy per array)
static int nf_app_pull(sh_handle* h) {
    if (h->df_ub == 0) return SH_OK;
    hipStream_t st = h->df_stream;
    unsigned long long n = 0;
    if (hipMemcpyAsync(&n, h->df_ctr.p, 8, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess)
        return fail(h, SH_E_HIP, "deferred rows");
    if ((int64_t)n > h->df_ub) return fail(h, SH_E_HIP, "deferred row count");
    const int no = std::max(1, h->n_out);
    const size_t base = h->o_seq.size();
    h->o_query.resize(base + n);
    h->o_seq.resize(base + n);
    h->o_ts.resize(base + n);
    h->o_vals.resize((base + n) * h->n_out);
    h->o_nulls.resize((base + n) * h->n_out);
    if (n) {
        const size_t b_q = 0, b_seq = ((size_t)n * 4 + 7) / 8 * 8, b_ts = b_seq + (size_t)n * 8,
                     b_v = b_ts + (size_t)n * 8, b_n = b_v + (size_t)n * no * 8, b_end = b_n + (size_t)n * no;
        if (h->pin_out.ensure(b_end)) return fail(h, SH_E_OOM, "pinned staging");
        uint8_t* pb = h->pin_out.as<uint8_t>();
        hipMemcpyAsync(pb + b_q, h->df_q.p, (size_t)n * 4, hipMemcpyDeviceToHost, st);
        hipMemcpyAsync(pb + b_seq, h->df_seq.p, (size_t)n * 8, hipMemcpyDeviceToHost, st);
        hipMemcpyAsync(pb + b_ts, h->df_ts.p, (size_t)n * 8, hipMemcpyDeviceToHost, st);
        if (h->n_out) {
            hipMemcpyAsync(pb + b_v, h->df_vals.p, (size_t)n * no * 8, hipMemcpyDeviceToHost, st);
            hipMemcpyAsync(pb + b_n, h->df_nulls.p, (size_t)n * no, hipMemcpyDeviceToHost, st);
        }
        if (hipStreamSynchronize(st) != hipSuccess) return fail(h, SH_E_HIP, "deferred rows copy");
        memcpy(h->o_query.data() + base, pb + b_q, n * 4);
        memcpy(h->o_seq.data() + base, pb + b_seq, n * 8);
        memcpy(h->o_ts.data() + base, pb + b_ts, n * 8);
        if (h->n_out) {
            memcpy(h->o_vals.data() + base * h->n_out, pb + b_v, n * no * 8);
            memcpy(h->o_nulls.data() + base * h->n_out, pb + b_n, n * no);
        }
    }
    hipMemsetAsync(h->df_ctr.p, 0, 8, st);
    h->df_ub = 0;
    return SH_OK;
}

// a streaming launch's rows appended to the deferred device rows (no sync): the
// scan, the placement and the count stay on the stream; nrec bounds the rows
static int nf_place_deferred(sh_handle* h, int64_t n_idx, int64_t nrec) {
    hipStream_t st = h->stream;
    if (h->df_ub && st != h->df_stream) {
        int rc = nf_app_pull(h);
        if (rc) return rc;
    }
    const int no = std::max(1, h->n_out);
    if (h->df_ub + nrec > h->df_cap) {
        int rc = nf_app_pull(h);
        if (rc) return rc;
        if (nrec > h->df_cap) {
            const int64_t cap = std::max<int64_t>(nrec, (int64_t)1 << 20);
            if (h->df_q.ensure_fresh(cap * 4) || h->df_seq.ensure_fresh(cap * 8) || h->df_ts.ensure_fresh(cap * 8) ||
                h->df_vals.ensure_fresh(cap * no * 8) || h->df_nulls.ensure_fresh(cap * no) ||
                h->df_ctr.ensure_fresh(8))
                return fail(h, SH_E_OOM, "deferred rows");
            h->df_cap = cap;
        }
    }
    if (h->df_ub == 0) hipMemsetAsync(h->df_ctr.p, 0, 8, st);
    if (shd_exclusive_scan(h->w_cnt.as<uint32_t>(), h->w_off.as<uint32_t>(), n_idx, h->w_scan.as<uint32_t>(), st))
        return fail(h, SH_E_HIP, "scan");
    if (h->w_inv.ensure_fresh(nrec * 4)) return fail(h, SH_E_OOM, "placement index");
    if (nfd_place_app(h->n_recs.as<uint64_t>(), nrec, NF_REC_HDR + no, h->w_off.as<uint32_t>(),
                      h->w_cnt.as<uint32_t>(), n_idx, no, h->df_ctr.as<unsigned long long>(), h->df_q.as<int32_t>(),
                      h->df_seq.as<uint64_t>(), h->df_ts.as<int64_t>(), h->df_vals.as<int64_t>(), h->df_nulls.as<uint8_t>(),
                      h->w_inv.as<uint32_t>(), st))
        return fail(h, SH_E_HIP, "placement");
    h->df_ub += nrec;
    h->df_stream = st;
    return SH_OK;
}

// scan the per-index counts, place the records, append them to the host queue
// (or to the caller's device buffers); returns the number of rows
// (launch: the launch's tick, for the key-sharded rows' order tags)
// nrec_known >= 0: the launch's record count, read back with its error word
static int nf_place(sh_handle* h, int64_t n_idx, int64_t* rows_out, uint64_t* d_seq, int64_t* d_vals, int64_t cap,
                    uint64_t launch, int64_t nrec_known) {
    HpScope hp_(h, 4);
    hipStream_t st = h->stream;
    if (!d_seq && !h->coord_on && !h->has_lists && nrec_known >= 0 && !getenv("SH_NO_DEFER_ROWS")) {
        *rows_out = -1;  // not known on the host (the rows are counted on the device)
        return nrec_known ? nf_place_deferred(h, n_idx, nrec_known) : SH_OK;
    }
    if (!d_seq) {
        int rc = nf_app_pull(h);  // host rows go after the deferred ones
        if (rc) return rc;
    }
    if (pin_rd_ready(h)) return fail(h, SH_E_OOM, "pinned staging");
    if (nrec_known < 0) hipMemcpyAsync(h->pin_rd.as<void>(PR_NREC), h->n_ctr.p, 8, hipMemcpyDeviceToHost, st);
    if (shd_exclusive_scan(h->w_cnt.as<uint32_t>(), h->w_off.as<uint32_t>(), n_idx, h->w_scan.as<uint32_t>(), st))
        return fail(h, SH_E_HIP, "scan");
    hipMemcpyAsync(h->pin_rd.as<void>(PR_LOFF), h->w_off.as<uint32_t>() + (n_idx - 1), 4, hipMemcpyDeviceToHost, st);
    hipMemcpyAsync(h->pin_rd.as<void>(PR_LCNT), h->w_cnt.as<uint32_t>() + (n_idx - 1), 4, hipMemcpyDeviceToHost, st);
    if (hipStreamSynchronize(st) != hipSuccess) return fail(h, SH_E_HIP, "device error before placement");
    const unsigned long long nrec =
        nrec_known >= 0 ? (unsigned long long)nrec_known : *h->pin_rd.as<unsigned long long>(PR_NREC);
    const uint32_t last_off = *h->pin_rd.as<uint32_t>(PR_LOFF), last_cnt = *h->pin_rd.as<uint32_t>(PR_LCNT);
    const int64_t total = (int64_t)last_off + last_cnt;
    *rows_out = total;
    if (total == 0) return SH_OK;
    if (h->coord_on && !d_seq) {
        // rows are placed by (position in the launch, ordinal): each row's tag is
        // the position whose count range holds it
        std::vector<uint32_t> cnt((size_t)n_idx);
        hipMemcpy(cnt.data(), h->w_cnt.p, (size_t)n_idx * 4, hipMemcpyDeviceToHost);
        const size_t base = h->o_order.size();
        h->o_order.reserve(base + (size_t)total);
        for (int64_t t = 0; t < n_idx; t++)
            for (uint32_t c = 0; c < cnt[t]; c++) h->o_order.push_back((launch << 32) | (uint64_t)t);
        if ((int64_t)(h->o_order.size() - base) != total) return fail(h, SH_E_HIP, "order tags");
    }
    const int stride = NF_REC_HDR + std::max(1, h->n_out);
    const int no = std::max(1, h->n_out);
    if (h->w_inv.ensure_fresh(total * 4)) return fail(h, SH_E_OOM, "placement index");
    if (d_seq) {  // device-resident output (sh_run_device): seq, values and, when asked, the query
        if (total > cap) return SH_E_MORE;
        if (h->dev_want_query && h->w_oq.ensure_fresh(total * 4)) return fail(h, SH_E_OOM, "output buffers");
        if (h->s3_compact) {
            // one record slot per key-ordered position of the run (n_idx events)
            nfd_place_s3(h->n_recs.as<uint64_t>(), h->rec_cap, n_idx, no, h->s3_type, h->s3_seq_base,
                         h->w_off.as<uint32_t>(), h->dev_want_query ? h->w_oq.as<int32_t>() : nullptr, d_seq, d_vals,
                         h->w_inv.as<uint32_t>(), total, st, h->s3_rw, h->s3_wide);
            return hipStreamSynchronize(st) == hipSuccess ? SH_OK : fail(h, SH_E_HIP, "placement");
        }
        nfd_place(h->n_recs.as<uint64_t>(), (int64_t)nrec, stride, h->w_off.as<uint32_t>(), no,
                  h->dev_want_query ? h->w_oq.as<int32_t>() : nullptr, d_seq, nullptr, d_vals, nullptr,
                  h->w_inv.as<uint32_t>(), total, st);
        return hipStreamSynchronize(st) == hipSuccess ? SH_OK : fail(h, SH_E_HIP, "placement");
    }
    // the rows are placed into one device block laid out like the pinned staging
    // (query | seq | ts | values | nulls) and come back in one copy, then into the host queue
    const size_t b_q = 0, b_seq = b_q + ((size_t)total * 4 + 7) / 8 * 8, b_ts = b_seq + (size_t)total * 8,
                 b_v = b_ts + (size_t)total * 8, b_n = b_v + (size_t)total * no * 8, b_end = b_n + (size_t)total * no;
    if (h->w_orows.ensure_fresh(b_end)) return fail(h, SH_E_OOM, "output buffers");
    uint8_t* ob = h->w_orows.as<uint8_t>();
    nfd_place(h->n_recs.as<uint64_t>(), (int64_t)nrec, stride, h->w_off.as<uint32_t>(), no, (int32_t*)(ob + b_q),
              (uint64_t*)(ob + b_seq), (int64_t*)(ob + b_ts), (int64_t*)(ob + b_v), ob + b_n, h->w_inv.as<uint32_t>(),
              total, st);
    const size_t base = h->o_seq.size();
    h->o_query.resize(base + total);
    h->o_seq.resize(base + total);
    h->o_ts.resize(base + total);
    h->o_vals.resize((base + total) * h->n_out);
    h->o_nulls.resize((base + total) * h->n_out);
    if (h->pin_out.ensure(b_end)) return fail(h, SH_E_OOM, "pinned staging");
    const bool vals = h->n_out && no == h->n_out;
    hipMemcpyAsync(h->pin_out.p, ob, vals ? b_end : b_v, hipMemcpyDeviceToHost, st);
    if (hipStreamSynchronize(st) != hipSuccess) return fail(h, SH_E_HIP, "output copy");
    memcpy(h->o_query.data() + base, h->pin_out.as<void>(b_q), total * 4);
    memcpy(h->o_seq.data() + base, h->pin_out.as<void>(b_seq), total * 8);
    memcpy(h->o_ts.data() + base, h->pin_out.as<void>(b_ts), total * 8);
    if (vals) {
        memcpy(h->o_vals.data() + base * h->n_out, h->pin_out.as<void>(b_v), total * no * 8);
        memcpy(h->o_nulls.data() + base * h->n_out, h->pin_out.as<void>(b_n), total * no);
    }
    if (h->has_lists && vals) {
        // List outputs: the launch's buffer offsets become host list ids
        unsigned long long nw = 0;
        hipMemcpy(&nw, h->n_lst_ctr.p, 8, hipMemcpyDeviceToHost);
        std::vector<uint64_t> L(nw);
        if (nw) hipMemcpy(L.data(), h->n_lst.p, nw * 8, hipMemcpyDeviceToHost);
        if (h->l_start.empty()) h->l_start.push_back(0);
        for (int64_t r = base; r < base + total; r++) {
            const nf_query& Q = h->T->q[h->o_query[r]];
            for (int c = 0; c < Q.n_out; c++) {
                if (Q.out_pc[c] != NF_PC_LIST || h->o_nulls[r * h->n_out + c]) continue;
                const uint64_t off = (uint64_t)h->o_vals[r * h->n_out + c];
                if (off >= nw) return fail(h, SH_E_HIP, "list value out of range");
                const uint64_t len = L[off];
                if (off + 1 + len + (len + 63) / 64 > nw) return fail(h, SH_E_HIP, "list value out of range");
                for (uint64_t i = 0; i < len; i++) {
                    h->l_vals.push_back((int64_t)L[off + 1 + i]);
                    h->l_nuls.push_back((uint8_t)((L[off + 1 + len + i / 64] >> (i % 64)) & 1));
                }
                h->o_vals[r * h->n_out + c] = h->l_base + (int64_t)h->l_start.size() - 1;
                h->l_start.push_back((int64_t)h->l_vals.size());
            }
        }
    }
    return SH_OK;
}

// one or more send() calls resident on the device, processed by k_nfa_run
static int carry_setup(sh_handle* h, const sh_device_run* run, shd_payload* carry, void** mid, int* alias,
                       bool used_only = false, bool with_ts = true);

// `carry` (sh_run_device, single stream): ts and the stream-0 columns are moved
// into key-segment order by the segment, so each lane streams its own events
// gidx / n_idx (key-sharded push): each event's position in the whole send()
// call of n_idx events (match counts and order tags are indexed by it)
static int nf_process(sh_handle* h, const shd_batch& B, int32_t nkeys, const nf_cols& cols_in, uint64_t* d_seq,
                      int64_t* d_vals, int64_t cap, int64_t* n_rows, bool fresh = false, int64_t batch_events = 0,
                      const sh_device_run* carry_run = nullptr, const uint32_t* gidx = nullptr, int64_t n_idx = 0) {
    HpScope hp_(h, 2);
    hipStream_t st = h->stream;
    const int64_t n = B.n;
    if (!gidx) n_idx = n;
    if (ensure_ws(h, std::max(n, n_idx))) return fail(h, SH_E_OOM, "workspace");
    if (nf_ensure_keys(h, nkeys)) return fail(h, SH_E_OOM, "key state");
    if (nf_ensure_recs(h, std::max<int64_t>(h->rec_cap, n + 4096))) return fail(h, SH_E_OOM, "emission buffer");
    nf_cols cols = cols_in;
    cols.sched_armed = armed_flags(h);  // after any key growth above
    if (cols.sched_armed && h->n_arm_log.p) {
        cols.arm_log = h->n_arm_log.as<int32_t>();
        cols.arm_ctr = h->n_arm_ctr.as<unsigned long long>();
        cols.arm_cap = (uint64_t)h->n_nkeys;
    }
    shd_payload carry;
    void* mid[8] = {nullptr};
    int alias = -1;
    const bool sorted_cols = carry_run && B.keys && h->stream_types[0].size() <= 7;
    // the rise-and-fall sequence engine: fresh single-query runs of that shape; its
    // device-resident rows carry no timestamps, so the segment leaves them behind
    const bool s3_shape = fresh && h->T->n_queries == 1 && h->T->q[0].s3 && !h->no_seq3 && !getenv("SH_NO_SEQ3");
    const bool sorted_ts = !(s3_shape && d_seq);
    if (sorted_cols) {
        if (carry_setup(h, carry_run, &carry, mid, &alias, true, sorted_ts)) return fail(h, SH_E_OOM, "sorted columns");
        for (size_t a = 0; a < h->stream_types[0].size(); a++)
            if (a >= 32 || ((h->T->attr_used[0] >> a) & 1u)) cols.col[0][a] = h->v_scol[a].p;
    }
    shd_segment_ws ws;
    ws.keys_a = h->w_keys_a.as<uint32_t>();
    ws.keys_b = h->w_keys_b.as<uint32_t>();
    ws.idx_a = h->w_idx_a.as<uint32_t>();
    ws.idx_b = h->w_idx_b.as<uint32_t>();
    ws.hist = h->w_hist.as<uint32_t>();
    ws.scan_tmp = h->w_scan.as<uint32_t>();
    ws.seg_off = h->w_seg.as<uint32_t>();
    ws.cap = n;
    const uint32_t* perm = nullptr;
    const uint32_t* skeys = nullptr;
    hipEventRecord(h->ev[0], st);
    if (shd_segment_payload(&B, nkeys, &ws, st, &perm, &skeys, sorted_cols ? &carry : nullptr, mid, 0, 1))
        return fail(h, SH_E_HIP, "segment launch failed");
    if (sorted_cols && alias >= 0) cols.col[0][alias] = skeys;
    if (pin_rd_ready(h)) return fail(h, SH_E_OOM, "pinned staging");
    nf_put_cols(h, cols);
    hipEventRecord(h->ev[1], st);
    const uint32_t* seg_list = ws.seg_off + 2 * n;
    const uint32_t* nseg = seg_list + n;
    const int64_t max_seg = std::max<int64_t>(1, std::min<int64_t>(n, nkeys));
    nfd_events E;
    E.ts = B.ts;
    E.stream = B.stream;
    E.row = B.row;
    E.bid = nullptr;  // one send() call per launch (batch 0), or fresh runs' batch_events
    E.perm = perm;
    E.seq_base = B.seq_base;
    E.batch_events = batch_events;
    E.sts = sorted_cols && sorted_ts ? h->v_sts.as<int64_t>() : nullptr;
    // k_seq3's LDS-staged form: every operand and output of the one attribute A
    // (4 bytes, no null mask), read from its key-ordered copy
    const void* s3_col = nullptr;
    if (s3_shape && sorted_cols) {
        const nf_query& Q = h->T->q[0];
        const int A = Q.s3_a2, ty = Q.s3_t2;
        bool ok = (ty == SH_T_FLOAT || ty == SH_T_INT) && A >= 0 && A < (int)h->stream_types[0].size() &&
                  type_width(h->stream_types[0][A]) == 4 && Q.s3_a3 == A && Q.s3_e1a == A && Q.s3_la == A &&
                  Q.s3_t3 == ty && Q.s3_e1t == ty && Q.s3_lt == ty && !cols.nul[0][A];
        // (count() reads no attribute)
        for (int o = 0; o < Q.n_out && ok; o++)
            ok = Q.out_agg[o] == SH_AGG_COUNT || (Q.s3_out_attr[o] == A && Q.s3_out_type[o] == ty);
        const bool staged = !(getenv("SH_S3_STAGED") && getenv("SH_S3_STAGED")[0] == '0');
        if (ok && staged) s3_col = alias == A ? (const void*)skeys : (const void*)cols.col[0][A];
    }
    // its records in the compact form (SH_S3_COMPACT=0: the generic records, for A/B)
    const bool s3_compact_on = !(getenv("SH_S3_COMPACT") && getenv("SH_S3_COMPACT")[0] == '0');
    h->s3_compact = s3_col && d_seq && s3_compact_on;
    h->s3_type = h->T->q[0].s3_t2;
    h->s3_seq_base = B.seq_base;
    // sum / avg / count in the kernel's lanes (each key's matches in trigger order: the
    // reference's own additions), when every aggregate is one of those and the record fits
    {
        const nf_query& Q = h->T->q[0];
        bool agg = h->s3_compact && Q.contains_agg && Q.n_out <= 6 && !getenv("SH_S3_AGG_POST");
        int rw = 1;
        uint32_t wide = 0;
        for (int o = 0; o < Q.n_out; o++) {
            const int ak = Q.out_agg[o];
            if (ak != SH_AGG_NONE && ak != SH_AGG_SUM && ak != SH_AGG_AVG && ak != SH_AGG_COUNT) agg = false;
            const bool w = ak != SH_AGG_NONE;
            rw += w ? 2 : 1;
            if (w) wide |= 1u << o;
        }
        h->s3_agg = agg;
        h->s3_rw = agg ? rw : 1 + std::max(1, Q.n_out);
        h->s3_wide = agg ? wide : 0u;
    }
    E.sorted_rows = sorted_cols ? 1 : 0;
    E.pad = 0;
    E.run = fresh ? h->dev_run_ids : nullptr;
    E.gidx = gidx;
    for (int attempt = 0; attempt < 64; attempt++) {
        const size_t kw = (size_t)h->T->key_words;
        if (!fresh) {
            if (h->n_save.ensure_fresh((size_t)max_seg * kw * 8)) return fail(h, SH_E_OOM, "save area");
            nfd_save(h->n_kstate.as<uint64_t>(), (int64_t)kw, seg_list, nseg, skeys, max_seg, h->n_save.as<uint64_t>(),
                     0, st);
        }
        hipMemsetAsync(h->w_cnt.p, 0, n_idx * 4, st);
        nf_ctl_zero(h);
        if (nf_lst_ready(h)) return fail(h, SH_E_OOM, "list values");
        if (h->has_lists && (cols.lst != h->n_lst.as<uint64_t>() || cols.lst_cap != (uint64_t)h->lst_cap)) {
            cols.lst = h->n_lst.as<uint64_t>();
            cols.lst_ctr = h->n_lst_ctr.as<unsigned long long>();
            cols.lst_cap = (uint64_t)h->lst_cap;
            nf_put_cols(h, cols);
        }
        if (h->sm_on) {
            if (nf_sev_ready(h, n, false)) return fail(h, SH_E_OOM, "scheduler history");
            if (cols.sev != h->n_sev.as<uint64_t>() || cols.sev_cap != (uint64_t)h->sev_cap) {
                // the buffer moved: refresh the column image
                cols = nf_store_cols(h);
                if (sorted_cols) {
                    for (size_t a = 0; a < h->stream_types[0].size(); a++)
                        if (a >= 32 || ((h->T->attr_used[0] >> a) & 1u)) cols.col[0][a] = h->v_scol[a].p;
                    if (alias >= 0) cols.col[0][alias] = skeys;
                }
                nf_put_cols(h, cols);
            }
        }
        nfd_emit em = nf_emit(h);
        // the rise-and-fall sequence engine: fresh single-query runs of that shape
        const bool seq3 = s3_shape;
        h->seq3_last = seq3 ? 1 : 0;
        if (seq3) {
            if (nfd_seq3(h->d_T.as<nf_table>(), h->d_ncols.as<nf_cols>(), &E, n, seg_list, nseg, skeys, nkeys, max_seg,
                         &em, st, s3_col, h->s3_compact ? 1 : 0, h->s3_agg ? 1 : 0, h->s3_rw))
                return fail(h, SH_E_HIP, "k_seq3 launch failed");
        } else if (nfd_run(h->d_T.as<nf_table>(), h->d_ncols.as<nf_cols>(), h->n_kstate.as<uint64_t>(), &E, n,
                           seg_list, nseg, skeys, nkeys, max_seg, h->tick, h->clock, &em, st))
            return fail(h, SH_E_HIP, "k_nfa_run launch failed");
        hipEventRecord(h->ev[2], st);
        nf_ctl_read(h);
        if (hipStreamSynchronize(st) != hipSuccess) return fail(h, SH_E_HIP, "device error in k_nfa_run");
        const unsigned err = nf_ctl_err(h);
        if (!err) {
            h->tick++;
            const int64_t nrec = nf_ctl_nrec(h);
            int src = nf_sev_apply(h, true);
            if (src) return src;
            int rc = nf_place(h, n_idx, n_rows, d_seq, d_vals, cap, h->tick - 1, nrec);
            hipEventElapsedTime(&h->times.segment_ms, h->ev[0], h->ev[1]);
            hipEventElapsedTime(&h->times.advance_ms, h->ev[1], h->ev[2]);
            if (*n_rows >= 0) {
                hipEventRecord(h->ev[3], st);
                hipStreamSynchronize(st);
                hipEventElapsedTime(&h->times.emit_ms, h->ev[2], h->ev[3]);
                hipEventElapsedTime(&h->times.total_ms, h->ev[0], h->ev[3]);
            } else {  // deferred rows: the placement is still on the stream
                h->times.emit_ms = 0.0f;
                hipEventElapsedTime(&h->times.total_ms, h->ev[0], h->ev[2]);
            }
            h->times.advance_launches = attempt + 1;
            return rc;
        }
        if (err & NF_E_KEY) return fail(h, SH_E_INVALID_ARG, "partition key id >= n_keys");
        if (err & NF_E_UNSUP)
            return fail(h, SH_E_UNSUPPORTED, "CountPreStateProcessor.startStateReset recursion (reference overflows)");
        // restore the touched keys (or the fresh state), grow, replay
        if (!fresh)
            nfd_save(h->n_kstate.as<uint64_t>(), (int64_t)kw, seg_list, nseg, skeys, max_seg,
                     h->n_save.as<uint64_t>(), 1, st);
        if (err & NF_E_EMIT) {
            if (nf_ensure_recs(h, h->rec_cap * 4)) return fail(h, SH_E_OOM, "emission buffer");
        }
        if (err & NF_E_SEV) {
            hipStreamSynchronize(st);
            if (h->n_sev.ensure_fresh((size_t)h->sev_cap * 4 * 16)) return fail(h, SH_E_OOM, "scheduler history");
            h->sev_cap *= 4;
        }
        if ((err & NF_E_LST) && nf_lst_grow(h)) return fail(h, SH_E_OOM, "list values");
        if (err & ~(unsigned)(NF_E_EMIT | NF_E_SEV | NF_E_LST)) {
            int rc = nf_grow(h, err);
            if (rc) return rc;
        }
        if (fresh) {
            hipMemsetAsync(h->n_kstate.p, 0, (size_t)nkeys * h->T->key_words * 8, st);
            if (!h->T->partitioned) {
                h->started = false;
                int rc = nf_start(h);
                if (rc) return rc;
            }
        }
    }
    return fail(h, SH_E_STATE_OVERFLOW, "replay limit");
}

// earliest queued notify time over every scheduler and key (INT64_MAX: none;
// key-sharded: over every rank)
static int nf_next_due_local(sh_handle* h, int64_t* out) {
    *out = INT64_MAX;
    if (!h->T->has_absent || h->n_nkeys == 0) return SH_OK;
    if (nf_sev_flush(h)) return SH_E_HIP;
    hipStream_t st = h->stream;
    if (pin_rd_ready(h)) return fail(h, SH_E_OOM, "pinned staging");
    const int32_t nkeys = h->n_nkeys;
    if (h->n_cand.ensure_fresh((size_t)nkeys * sizeof(nfd_cand)) || h->n_tmin.ensure_fresh(8))
        return fail(h, SH_E_OOM, "candidates");
    for (int q = 0; q < h->T->n_queries; q++) {
        for (int si = 0; si < h->T->q[q].n_sched; si++) {
            const int p = h->T->q[q].sched_seq[si];
            hipMemsetAsync(h->n_ctr.p, 0, 8, st);
            nfd_due(h->d_T.as<nf_table>(), q, p, h->n_kstate.as<uint64_t>(), nkeys, INT64_MAX,
                    h->n_cand.as<nfd_cand>(), h->n_ctr.as<unsigned long long>(), nkeys, nullptr, 0, nullptr, st);
            hipMemcpyAsync(h->pin_rd.as<void>(PR_NC), h->n_ctr.p, 8, hipMemcpyDeviceToHost, st);
            if (hipStreamSynchronize(st) != hipSuccess) return fail(h, SH_E_HIP, "k_nfa_due");
            const int64_t nc = (int64_t)*h->pin_rd.as<unsigned long long>(PR_NC);
            if (nc == 0) continue;
            nfd_cand_tmin(h->n_cand.as<nfd_cand>(), nc, h->n_tmin.as<unsigned long long>(), st);
            hipMemcpyAsync(h->pin_rd.as<void>(PR_TMIN), h->n_tmin.p, 8, hipMemcpyDeviceToHost, st);
            if (hipStreamSynchronize(st) != hipSuccess) return fail(h, SH_E_HIP, "k_cand_tmin");
            *out = std::min(*out, (int64_t)*h->pin_rd.as<unsigned long long>(PR_TMIN));
        }
    }
    return SH_OK;
}

static int nf_next_due(sh_handle* h, int64_t* out) {
    int rc = nf_next_due_local(h, out);
    if (rc || !h->coord_on) return rc;
    int64_t g = INT64_MAX;
    if (h->coord.min_time(h->coord.user, *out, &g)) return fail(h, SH_E_INVALID_ARG, "coordinator: min_time failed");
    *out = g;
    return SH_OK;
}

// Scheduler.onTimeChange(now) for every scheduler (absent pre-state) in creation
// order. wall: the EventCaller form outside playback (Scheduler.java:285-300) --
// every due key fires on its own, no collapse of equal due times.
// Key-sharded (coord_on): every rank takes every step (the coordinator calls are
// collectives); the pick runs over all ranks' candidates and the firing order
// positions are global, so registration stamps and row order match one process.
static int nf_timers(sh_handle* h, int64_t now, bool wall) {
    HpScope hp_(h, 1);
    if (!h->T->has_absent) return SH_OK;
    if (h->n_nkeys == 0 && !h->coord_on) return SH_OK;
    hipStream_t st = h->stream;
    if (pin_rd_ready(h)) return fail(h, SH_E_OOM, "pinned staging");
    nf_put_cols(h, nf_store_cols(h));
    bool first_pass = true;
    int n_absent = 0;  // a key's armed flag may be cleared only when it has one scheduler
    for (int q = 0; q < h->T->n_queries; q++)
        for (int p = 0; p < h->T->q[q].n_proc; p++) n_absent += nf_has_sched(h->T->q[q].proc[p]);
    for (int q = 0; q < h->T->n_queries; q++) {
        // Scheduler creation order (the TimestampGenerator's listener order)
        for (int si = 0; si < h->T->q[q].n_sched; si++) {
            const int p = h->T->q[q].sched_seq[si];
            {
                const int frc = nf_sev_flush(h);  // the ranks the due pass reads
                if (frc) return frc;
            }
            const int32_t nkeys = h->n_nkeys;
            unsigned long long nc = 0;
            if (nkeys > 0) {
                // due keys
                if (h->n_cand.ensure_fresh((size_t)nkeys * sizeof(nfd_cand))) return fail(h, SH_E_OOM, "candidates");
                hipMemsetAsync(h->n_ctr.p, 0, 8, st);
                const uint64_t* rank = h->sm_on ? h->n_rank[q * NF_MAX_PROC + p].as<uint64_t>() : nullptr;
                if (armed_flags(h) && h->n_arm_log.p) {
                    // the armed-key list (+ the keys armed since the last pass on the
                    // first scheduler's pass, which also rebuilds the list)
                    unsigned long long* ln = h->n_klist_n.as<unsigned long long>();
                    const int c = h->klist_cur;
                    if (first_pass) {
                        hipMemsetAsync(ln + (c ^ 1), 0, 8, st);
                        nfd_due_list(h->d_T.as<nf_table>(), q, p, h->n_kstate.as<uint64_t>(), h->n_klist[c].as<int32_t>(),
                                     ln + c, h->n_arm_log.as<int32_t>(), h->n_arm_ctr.as<unsigned long long>(), now,
                                     h->n_cand.as<nfd_cand>(), h->n_ctr.as<unsigned long long>(), nkeys, armed_flags(h),
                                     n_absent == 1 ? 1 : 0, rank, h->n_klist[c ^ 1].as<int32_t>(), ln + (c ^ 1),
                                     (int64_t)nkeys, st);
                        hipMemsetAsync(h->n_arm_ctr.p, 0, 8, st);
                        h->klist_cur ^= 1;
                        first_pass = false;
                    } else {
                        nfd_due_list(h->d_T.as<nf_table>(), q, p, h->n_kstate.as<uint64_t>(), h->n_klist[c].as<int32_t>(),
                                     ln + c, nullptr, nullptr, now, h->n_cand.as<nfd_cand>(),
                                     h->n_ctr.as<unsigned long long>(), nkeys, armed_flags(h), 0, rank, nullptr, nullptr,
                                     (int64_t)nkeys, st);
                    }
                } else {
                    nfd_due(h->d_T.as<nf_table>(), q, p, h->n_kstate.as<uint64_t>(), nkeys, now, h->n_cand.as<nfd_cand>(),
                            h->n_ctr.as<unsigned long long>(), nkeys, armed_flags(h), n_absent == 1 ? 1 : 0, rank, st);
                }
                hipMemcpyAsync(h->pin_rd.as<void>(PR_NC), h->n_ctr.p, 8, hipMemcpyDeviceToHost, st);
                if (hipStreamSynchronize(st) != hipSuccess) return fail(h, SH_E_HIP, "k_nfa_due");
                nc = *h->pin_rd.as<unsigned long long>(PR_NC);
            }
            if (nc == 0 && !h->coord_on) continue;
            // TreeMultimap<Long, SchedulerState> with a zero comparator: one key per
            // distinct due time, the first in keyOrder (earliest registration)
            std::vector<int32_t> sel;
            std::vector<uint32_t> gpos;  // key-sharded: firing positions over all ranks
            int64_t n_idx = 0;           // positions in the launch (match counts)
            bool picked = false;
            if (h->coord_on) {
                std::vector<nfd_cand> cs(nc);
                if (nc) hipMemcpy(cs.data(), h->n_cand.p, nc * sizeof(nfd_cand), hipMemcpyDeviceToHost);
                std::vector<int64_t> pos(nc, -1);
                int64_t n_fire = 0;
                static_assert(sizeof(nfd_cand) == sizeof(sh_due_cand), "candidate layout");
                if (h->coord.select(h->coord.user, wall ? 1 : 0, (const sh_due_cand*)cs.data(), (int64_t)nc, pos.data(),
                                    &n_fire))
                    return fail(h, SH_E_INVALID_ARG, "coordinator: select failed");
                if (n_fire == 0) continue;  // every rank skips this launch
                std::vector<std::pair<int64_t, int32_t>> mine;
                for (size_t i = 0; i < cs.size(); i++)
                    if (pos[i] >= 0) {
                        if (pos[i] >= n_fire) return fail(h, SH_E_INVALID_ARG, "coordinator: position out of range");
                        mine.emplace_back(pos[i], cs[i].key);
                    }
                std::sort(mine.begin(), mine.end());
                for (auto& m : mine) {
                    sel.push_back(m.second);
                    gpos.push_back((uint32_t)m.first);
                }
                n_idx = n_fire;
                picked = true;
            }
            if (!picked && (int64_t)nc >= kDeviceTieBreak && !wall) {
                // large backlog of due keys: pick on the device (slot per due time)
                if (h->n_tmin.ensure_fresh(8)) return fail(h, SH_E_OOM, "timer tie-break");
                nfd_cand_tmin(h->n_cand.as<nfd_cand>(), (int64_t)nc, h->n_tmin.as<unsigned long long>(), st);
                hipMemcpyAsync(h->pin_rd.as<void>(PR_TMIN), h->n_tmin.p, 8, hipMemcpyDeviceToHost, st);
                if (hipStreamSynchronize(st) != hipSuccess) return fail(h, SH_E_HIP, "k_cand_tmin");
                const int64_t tmin = (int64_t)*h->pin_rd.as<unsigned long long>(PR_TMIN);
                const int64_t range = now - tmin + 1;
                if (tmin >= 0 && range > 0 && range <= kTieBreakSlots) {
                    if (h->n_slot_s.ensure_fresh((size_t)range * 8) || h->n_slot_k.ensure_fresh((size_t)range * 4) ||
                        h->pin_out.ensure((size_t)range * 4))
                        return fail(h, SH_E_OOM, "timer tie-break");
                    nfd_cand_select(h->n_cand.as<nfd_cand>(), (int64_t)nc, tmin, range,
                                    h->n_slot_s.as<unsigned long long>(), h->n_slot_k.as<int32_t>(), st);
                    hipMemcpyAsync(h->pin_out.p, h->n_slot_k.p, (size_t)range * 4, hipMemcpyDeviceToHost, st);
                    if (hipStreamSynchronize(st) != hipSuccess) return fail(h, SH_E_HIP, "k_cand_select");
                    const int32_t* sk = h->pin_out.as<int32_t>();
                    for (int64_t r = 0; r < range; r++)
                        if (sk[r] >= 0) sel.push_back(sk[r]);
                    picked = true;
                }
            }
            if (!picked) {
                std::vector<nfd_cand> cs(nc);
                hipMemcpy(cs.data(), h->n_cand.p, nc * sizeof(nfd_cand), hipMemcpyDeviceToHost);
                std::sort(cs.begin(), cs.end(), [](const nfd_cand& a, const nfd_cand& b) {
                    if (a.t != b.t) return a.t < b.t;
                    return a.stamp < b.stamp;
                });
                for (size_t i = 0; i < cs.size(); i++)
                    if (wall || i == 0 || cs[i].t != cs[i - 1].t) sel.push_back(cs[i].key);
            }
            const int32_t ns = (int32_t)sel.size();
            if (!h->coord_on) n_idx = ns;
            if (h->n_sel.ensure_fresh((size_t)std::max(ns, 1) * 4) ||
                h->n_save.ensure_fresh((size_t)std::max(ns, 1) * h->T->key_words * 8) ||
                h->n_gpos.ensure_fresh((size_t)std::max(ns, 1) * 4))
                return fail(h, SH_E_OOM, "timer keys");
            if (h->pin_out.ensure((size_t)std::max(ns, 1) * 8)) return fail(h, SH_E_OOM, "pinned staging");
            if (ns) {
                memcpy(h->pin_out.p, sel.data(), (size_t)ns * 4);  // read by the copies before the loop's sync
                hipMemcpyAsync(h->n_sel.p, h->pin_out.p, (size_t)ns * 4, hipMemcpyHostToDevice, st);
                if (h->coord_on) {
                    memcpy(h->pin_out.as<uint8_t>((size_t)ns * 4), gpos.data(), (size_t)ns * 4);
                    hipMemcpyAsync(h->n_gpos.p, h->pin_out.as<uint8_t>((size_t)ns * 4), (size_t)ns * 4,
                                   hipMemcpyHostToDevice, st);
                }
            }
            if (ensure_ws(h, std::max<int64_t>(n_idx, 1))) return fail(h, SH_E_OOM, "workspace");
            if (nf_ensure_recs(h, std::max<int64_t>(h->rec_cap, ns + 4096))) return fail(h, SH_E_OOM, "emission");
            bool counted = false;  // the history count came back with the last error read-back
            for (int attempt = 0;; attempt++) {
                if (attempt > 64) return fail(h, SH_E_STATE_OVERFLOW, "replay limit");
                const size_t kw = (size_t)h->T->key_words;
                hipMemsetAsync(h->w_cnt.p, 0, (size_t)n_idx * 4, st);
                nf_ctl_zero(h);
                {
                    const void* lst0 = h->n_lst.p;
                    if (nf_lst_ready(h)) return fail(h, SH_E_OOM, "list values");
                    if (lst0 != h->n_lst.p) nf_put_cols(h, nf_store_cols(h));
                }
                if (h->sm_on) {
                    const void* sev0 = h->n_sev.p;
                    const int64_t cap0 = h->sev_cap;
                    if (nf_sev_ready(h, ns, false)) return fail(h, SH_E_OOM, "scheduler history");
                    if (sev0 != h->n_sev.p || cap0 != h->sev_cap || attempt > 0) nf_put_cols(h, nf_store_cols(h));
                } else if (attempt > 0) {
                    nf_put_cols(h, nf_store_cols(h));
                }
                if (ns == 0) break;  // key-sharded: another rank fires this launch
                if (h->n_save.ensure_fresh((size_t)ns * kw * 8)) return fail(h, SH_E_OOM, "save area");
                nfd_save_keys(h->n_kstate.as<uint64_t>(), (int64_t)kw, h->n_sel.as<int32_t>(), ns,
                              h->n_save.as<uint64_t>(), 0, st);
                nfd_emit em = nf_emit(h);
                nfd_timer(h->d_T.as<nf_table>(), h->d_ncols.as<nf_cols>(), h->n_kstate.as<uint64_t>(), q, p,
                          h->n_sel.as<int32_t>(), ns, now, h->tick, h->clock, h->seq_next, &em, st,
                          h->coord_on ? h->n_gpos.as<uint32_t>() : nullptr);
                nf_ctl_read(h);
                if (hipStreamSynchronize(st) != hipSuccess) return fail(h, SH_E_HIP, "device error in k_nfa_timer");
                unsigned err = nf_ctl_err(h);
                if (!err) {
                    counted = true;
                    break;
                }
                if (err & NF_E_UNSUP) return fail(h, SH_E_UNSUPPORTED, "startStateReset recursion");
                nfd_save_keys(h->n_kstate.as<uint64_t>(), (int64_t)kw, h->n_sel.as<int32_t>(), ns,
                              h->n_save.as<uint64_t>(), 1, st);
                if (err & NF_E_EMIT && nf_ensure_recs(h, h->rec_cap * 4)) return fail(h, SH_E_OOM, "emission");
                if (err & NF_E_SEV) {
                    hipStreamSynchronize(st);
                    if (h->n_sev.ensure_fresh((size_t)h->sev_cap * 4 * 16)) return fail(h, SH_E_OOM, "history");
                    h->sev_cap *= 4;
                    err &= ~(unsigned)NF_E_SEV;
                }
                if (err & NF_E_LST) {
                    if (nf_lst_grow(h)) return fail(h, SH_E_OOM, "list values");
                    err &= ~(unsigned)NF_E_LST;
                }
                if (err & ~(unsigned)NF_E_EMIT) {
                    int rc = nf_grow(h, err);
                    if (rc) return rc;
                }
            }
            h->tick++;
            {
                int src = nf_sev_apply(h, counted);
                if (src) return src;
            }
            int64_t rows = 0;
            int rc = nf_place(h, n_idx, &rows, nullptr, nullptr, 0, h->tick - 1, counted ? nf_ctl_nrec(h) : -1);
            if (rc) return rc;
        }
    }
    return SH_OK;
}

static int nf_start(sh_handle* h) {
    if (h->started) return SH_OK;
    h->started = true;
    if (h->T->partitioned) return SH_OK;
    if (nf_ensure_keys(h, 1)) return fail(h, SH_E_OOM, "key state");
    const nf_cols cols = nf_store_cols(h);
    hipMemcpyAsync(h->d_ncols.p, &cols, sizeof(nf_cols), hipMemcpyHostToDevice, h->stream);
    h->cols_cached = false;
    hipMemsetAsync(h->n_err.p, 0, 4, h->stream);
    if (nf_ensure_recs(h, 4096)) return fail(h, SH_E_OOM, "emission");
    nfd_emit em = nf_emit(h);
    nfd_start(h->d_T.as<nf_table>(), h->d_ncols.as<nf_cols>(), h->n_kstate.as<uint64_t>(), h->tick, h->clock, &em,
              h->stream);
    unsigned err = 0;
    hipMemcpyAsync(&err, h->n_err.p, 4, hipMemcpyDeviceToHost, h->stream);
    if (hipStreamSynchronize(h->stream) != hipSuccess) return fail(h, SH_E_HIP, "k_nfa_start");
    h->tick++;
    return err ? fail(h, SH_E_STATE_OVERFLOW, "start state overflow") : SH_OK;
}

// InputHandler.send(Event[]) on the general engine: playback clock + due timers
// first (InputHandler.java:85-96), then the batch. index (key-sharded): the
// positions of this rank's events in the whole call of call_n events, whose last
// timestamp is call_last; the rank takes every step of the call even when it owns
// none of its events (the coordinator's exchanges are collectives).
static int nf_push(sh_handle* h, const sh_batch* b, int64_t r0, const uint32_t* index, int64_t call_n,
                   int64_t call_last) {
    if (h->kstate_stale) {
        hipMemsetAsync(h->n_kstate.p, 0, (size_t)h->n_nkeys * h->T->key_words * 8, h->stream);
        h->kstate_stale = false;
        h->started = false;
    }
    if (!h->started) {
        int rc = nf_start(h);
        if (rc) return rc;
    }
    if (h->app.playback) {
        const int64_t last = index ? call_last : b->ts[b->n - 1];
        if (last >= h->clock) {
            h->clock = last;
            int rc = nf_timers(h, last);
            if (rc) return rc;
        }
    }
    const int64_t n = b->n;
    hipStream_t st = h->stream;
    if (index && n == 0) {
        // none of the call's events is ours: the launch still ticks and its
        // (empty) scheduler history joins the others'
        if (h->sm_on && nf_sev_ready(h, 0)) return fail(h, SH_E_OOM, "scheduler history");
        h->tick++;
        int rc = nf_sev_apply(h);
        h->seq_next += call_n;
        h->seq_staged0 = h->seq_next;
        return rc;
    }
    // staged in pinned memory (pin_in; the column copies of this call are complete)
    const size_t o_ts = 0, o_rows = (size_t)n * 8, o_keys = o_rows + (size_t)n * 4, o_sv = o_keys + (size_t)n * 4;
    if (h->pin_stage.ensure(o_sv + (size_t)n)) return fail(h, SH_E_OOM, "pinned staging");
    uint8_t* sv = h->pin_stage.as<uint8_t>(o_sv);
    uint32_t* rows = h->pin_stage.as<uint32_t>(o_rows);
    int32_t* keys = h->pin_stage.as<int32_t>(o_keys);
    memset(sv, (uint8_t)b->stream, (size_t)n);
    memcpy(h->pin_stage.as<int64_t>(o_ts), b->ts, (size_t)n * 8);
    int32_t nk = 1;
    for (int64_t i = 0; i < n; i++) {
        rows[i] = (uint32_t)(r0 + i);
        keys[i] = 0;
        if (h->partitioned) {
            keys[i] = b->keys ? b->keys[i] : -1;
            nk = std::max(nk, keys[i] + 1);
        }
    }
    // one copy: the device staging mirrors pin_stage's layout (ts | rows | keys | stream)
    if (h->w_pstage.ensure_fresh(o_sv + (size_t)n)) return fail(h, SH_E_OOM, "staging");
    hipMemcpyAsync(h->w_pstage.p, h->pin_stage.p, o_sv + (size_t)n, hipMemcpyHostToDevice, st);
    shd_batch B;
    B.ts = h->w_pstage.as<int64_t>();
    B.stream = h->w_pstage.as<uint8_t>() + o_sv;
    B.row = (const uint32_t*)(h->w_pstage.as<uint8_t>() + o_rows);
    B.keys = h->partitioned ? (const int32_t*)(h->w_pstage.as<uint8_t>() + o_keys) : nullptr;
    B.row_base = 0;
    B.pad = 0;
    B.seq_base = h->seq_next;
    B.n = n;
    int64_t nrows = 0;
    const uint32_t* gidx = nullptr;
    if (index) {
        if (h->w_gidx.ensure_fresh((size_t)n * 4)) return fail(h, SH_E_OOM, "staging");
        hipMemcpyAsync(h->w_gidx.p, index, (size_t)n * 4, hipMemcpyHostToDevice, st);
        gidx = h->w_gidx.as<uint32_t>();
    }
    int rc = nf_process(h, B, nk, nf_store_cols(h), nullptr, nullptr, 0, &nrows, false, 0, nullptr, gidx, call_n);
    h->seq_next += index ? call_n : n;
    h->seq_staged0 = h->seq_next;
    return rc;
}

static shd_cols store_cols(sh_handle* h) {
    shd_cols c;
    memset(&c, 0, sizeof(c));
    for (int s = 0; s < h->app.n_streams; s++)
        for (size_t a = 0; a < h->stream_types[s].size(); a++) {
            c.col[s][a] = h->stores[s].cols[a].p;
            c.nul[s][a] = h->stores[s].has_nul[a] ? (const uint8_t*)h->stores[s].nuls[a].p : nullptr;
        }
    return c;
}

// process every staged event
static int flush(sh_handle* h) {
    if (h->mode == 1) return nf_app_pull(h);  // the general engine processes each send() at once
    const int64_t n = (int64_t)h->st_ts.size();
    if (n == 0) return SH_OK;
    if (!h->has_device) return fail(h, SH_E_NO_DEVICE, "no HIP device");
    h->stream = h->own_stream;
    hipStream_t st = h->stream;
    int32_t nkeys = std::max(1, h->max_key);
    if (ensure_keys(h, nkeys)) return fail(h, SH_E_OOM, "key state");
    if (h->w_ts.ensure_fresh(n * 8) || h->w_stream.ensure_fresh(n) || h->w_row.ensure_fresh(n * 4) ||
        h->w_key.ensure_fresh(n * 4))
        return fail(h, SH_E_OOM, "staging");
    hipMemcpyAsync(h->w_ts.p, h->st_ts.data(), n * 8, hipMemcpyHostToDevice, st);
    hipMemcpyAsync(h->w_stream.p, h->st_stream.data(), n, hipMemcpyHostToDevice, st);
    hipMemcpyAsync(h->w_row.p, h->st_row.data(), n * 4, hipMemcpyHostToDevice, st);
    hipMemcpyAsync(h->w_key.p, h->st_key.data(), n * 4, hipMemcpyHostToDevice, st);
    shd_batch B;
    B.ts = h->w_ts.as<int64_t>();
    B.stream = h->w_stream.as<uint8_t>();
    B.row = h->w_row.as<uint32_t>();
    B.keys = h->partitioned ? h->w_key.as<int32_t>() : nullptr;
    B.row_base = 0;
    B.seq_base = h->seq_staged0;
    B.n = n;
    shd_cols cols = store_cols(h);
    int64_t cap = std::max<int64_t>(n, 1024);
    int64_t nm = 0;
    int rc;
    for (;;) {
        if (h->w_oseq.ensure_fresh(cap * 8) || h->w_ots.ensure_fresh(cap * 8) ||
            h->w_ovals.ensure_fresh(cap * std::max(1, h->n_out) * 8) ||
            h->w_onulls.ensure_fresh(cap * std::max(1, h->n_out)))
            return fail(h, SH_E_OOM, "output buffers");
        rc = run_batch(h, B, nkeys, cols, h->w_oseq.as<uint64_t>(), h->w_ots.as<int64_t>(), h->w_ovals.as<int64_t>(),
                       h->w_onulls.as<uint8_t>(), cap, &nm, false);
        if (rc == SH_E_MORE) {
            // the state advanced already; rerunning would double-advance: outputs
            // sized from the count are produced by the placement below instead
            cap = nm;
            if (h->w_oseq.ensure_fresh(cap * 8) || h->w_ots.ensure_fresh(cap * 8) ||
                h->w_ovals.ensure_fresh(cap * std::max(1, h->n_out) * 8) ||
                h->w_onulls.ensure_fresh(cap * std::max(1, h->n_out)))
                return fail(h, SH_E_OOM, "output buffers");
            shd_emit em;
            em.tmp = h->w_tmp.as<uint64_t>();
            em.tmp_ctr = h->w_ctr.as<unsigned long long>();
            em.tmp_cap = h->tmp_cap;
            em.match_cnt = h->w_cnt.as<uint32_t>();
            em.err = h->d_err.as<int32_t>();
            unsigned long long nrec = 0;
            hipMemcpy(&nrec, h->w_ctr.p, 8, hipMemcpyDeviceToHost);
            shd_emit_place(&em, h->n_out, 0, h->w_off.as<uint32_t>(), h->w_scan.as<uint32_t>(), (int64_t)nrec, &B,
                           h->w_oseq.as<uint64_t>(), h->w_ots.as<int64_t>(), h->w_ovals.as<int64_t>(),
                           h->w_onulls.as<uint8_t>(), st);
            hipStreamSynchronize(st);
            rc = SH_OK;
        }
        break;
    }
    if (rc) return rc;
    // D2H into the host output queue
    size_t base = h->o_seq.size();
    h->o_query.resize(base + nm, 0);
    h->o_seq.resize(base + nm);
    h->o_ts.resize(base + nm);
    h->o_vals.resize((base + nm) * h->n_out);
    h->o_nulls.resize((base + nm) * h->n_out);
    if (nm) {
        hipMemcpy(h->o_seq.data() + base, h->w_oseq.p, nm * 8, hipMemcpyDeviceToHost);
        hipMemcpy(h->o_ts.data() + base, h->w_ots.p, nm * 8, hipMemcpyDeviceToHost);
        if (h->n_out) {
            hipMemcpy(h->o_vals.data() + base * h->n_out, h->w_ovals.p, nm * h->n_out * 8, hipMemcpyDeviceToHost);
            hipMemcpy(h->o_nulls.data() + base * h->n_out, h->w_onulls.p, nm * h->n_out, hipMemcpyDeviceToHost);
        }
    }
    h->st_ts.clear();
    h->st_stream.clear();
    h->st_row.clear();
    h->st_key.clear();
    h->seq_staged0 = h->seq_next;
    return SH_OK;
}

int64_t sh_pending(sh_handle* h) {
    if (!h) return SH_E_INVALID_ARG;
    int rc = flush(h);
    if (rc) return rc;
    return (int64_t)h->o_seq.size() - h->o_read;
}

static int drain_impl(sh_handle* h, sh_match_buf* out, uint64_t* order) {
    HpScope hp_(h, 5);
    if (h && h->poisoned) return fail(h, SH_E_INVALID_ARG, "handle unusable after a failed restore");
    if (!h || !out) return SH_E_INVALID_ARG;
    int rc = flush(h);
    if (rc) return rc;
    const int64_t avail = (int64_t)h->o_seq.size() - h->o_read;
    const int64_t k = std::min(avail, out->capacity);
    const int no = out->n_out;
    if (order && h->o_order.size() != h->o_seq.size())
        return fail(h, SH_E_INVALID_ARG, "order tags exist on key-sharded handles only");
    if (h->has_lists && h->l_start.size() > 1) {
        // the lists of rows returned by earlier drains are released now (a
        // handle stays valid until the next drain): keep from the first list the
        // undelivered rows hold
        int64_t keep = h->l_base + (int64_t)h->l_start.size() - 1;
        for (int64_t r = h->o_read; r < (int64_t)h->o_seq.size() && keep > h->l_base; r++) {
            const nf_query& Q = h->T->q[h->o_query[r]];
            for (int c = 0; c < Q.n_out; c++)
                if (Q.out_pc[c] == NF_PC_LIST && !h->o_nulls[r * h->n_out + c])
                    keep = std::min(keep, h->o_vals[r * h->n_out + c]);
        }
        const int64_t drop = keep - h->l_base;
        if (drop > 0) {
            const int64_t cut = h->l_start[drop];
            h->l_vals.erase(h->l_vals.begin(), h->l_vals.begin() + cut);
            h->l_nuls.erase(h->l_nuls.begin(), h->l_nuls.begin() + cut);
            h->l_start.erase(h->l_start.begin(), h->l_start.begin() + drop);
            for (auto& x : h->l_start) x -= cut;
            h->l_base = keep;
        }
    }
    for (int64_t i = 0; i < k; i++) {
        const int64_t r = h->o_read + i;
        if (order) order[i] = h->o_order[r];
        if (out->query) out->query[i] = h->o_query[r];
        if (out->trigger_seq) out->trigger_seq[i] = h->o_seq[r];
        if (out->ts) out->ts[i] = h->o_ts[r];
        for (int c = 0; c < no; c++) {
            const bool has = c < h->n_out;
            if (out->values) out->values[i * no + c] = has ? h->o_vals[r * h->n_out + c] : 0;
            if (out->nulls) out->nulls[i * no + c] = has ? h->o_nulls[r * h->n_out + c] : 1;
        }
    }
    out->count = k;
    h->o_read += k;
    if (h->o_read == (int64_t)h->o_seq.size()) {
        h->o_query.clear();
        h->o_seq.clear();
        h->o_ts.clear();
        h->o_vals.clear();
        h->o_nulls.clear();
        h->o_order.clear();
        h->o_read = 0;
    }
    return avail > k ? SH_E_MORE : SH_OK;
}

int sh_drain(sh_handle* h, sh_match_buf* out) { return drain_impl(h, out, nullptr); }

int64_t sh_list_get(sh_handle* h, int64_t list, int64_t cap, int64_t* values, uint8_t* nulls) {
    if (!h || list < h->l_base || list >= h->l_base + (int64_t)h->l_start.size() - 1) return SH_E_INVALID_ARG;
    const int64_t i = list - h->l_base;
    const int64_t a = h->l_start[i], n = h->l_start[i + 1] - a;
    for (int64_t k = 0; k < n && k < cap; k++) {
        if (values) values[k] = h->l_vals[a + k];
        if (nulls) nulls[k] = h->l_nuls[a + k];
    }
    return n;
}
int sh_drain_ordered(sh_handle* h, sh_match_buf* out, uint64_t* order) { return drain_impl(h, out, order); }

static int bits_for(uint64_t v) {
    int b = 0;
    while (b < 64 && (v >> b)) b++;
    return b;
}

static shd_segment_ws seg_ws(sh_handle* h, int64_t n) {
    shd_segment_ws ws;
    ws.keys_a = h->w_keys_a.as<uint32_t>();
    ws.keys_b = h->w_keys_b.as<uint32_t>();
    ws.idx_a = h->w_idx_a.as<uint32_t>();
    ws.idx_b = h->w_idx_b.as<uint32_t>();
    ws.hist = h->w_hist.as<uint32_t>();
    ws.scan_tmp = h->w_scan.as<uint32_t>();
    ws.seg_off = h->w_seg.as<uint32_t>();
    ws.cap = n;
    return ws;
}

// ts and every column of stream 0 moved into key-segment order by the segment
// A 4-byte column that is the key array itself (the partition attribute, passed
// as the same device buffer) is not carried: its key-segment order is the
// sorted key array (*alias = that attribute, -1 if none). Null-key events
// (sorted to the sentinel bucket) are never read.
static int carry_setup(sh_handle* h, const sh_device_run* run, shd_payload* carry, void** mid, int* alias,
                       bool used_only, bool with_ts) {
    const int64_t n = run->n;
    const int na = (int)h->stream_types[0].size();
    memset(carry, 0, sizeof(*carry));
    *alias = -1;
    int c = 0;
    if (with_ts) {
        if (h->v_sts.ensure_fresh(n * 8) || h->v_mid_ts.ensure_fresh(n * 8)) return SH_E_OOM;
        carry->src[c] = run->d_ts;
        carry->dst[c] = h->v_sts.p;
        carry->width[c] = 8;
        mid[c++] = h->v_mid_ts.p;
    }
    for (int a = 0; a < na; a++) {
        const int w = type_width(h->stream_types[0][a]);
        if (used_only && h->T && a < 32 && !((h->T->attr_used[0] >> a) & 1u)) continue;  // no expression reads it
        if (*alias < 0 && w == 4 && run->d_cols[a] == (const void*)run->d_keys && !getenv("SH_NO_KEY_ALIAS")) {
            *alias = a;
            continue;
        }
        if (h->v_scol[a].ensure_fresh(n * w) || h->v_mid[a].ensure_fresh(n * w)) return SH_E_OOM;
        carry->src[c] = run->d_cols[a];
        carry->dst[c] = h->v_scol[a].p;
        carry->width[c] = (uint8_t)w;
        mid[c++] = h->v_mid[a].p;
    }
    carry->n = c;
    return SH_OK;
}

// log2 of the arrival tile (0: untiled) for a partitioned window run: tiles of
// 2^19 events when the stream spans several and the directory stays small
// (SH_TILE_SHIFT overrides, for tests)
static int tile_shift_for(int64_t n, int32_t nkeys) {
    int shift = 19;
    if (const char* e = getenv("SH_TILE_SHIFT")) shift = atoi(e);
    if (shift < 12 || shift > 24) return 0;
    const int64_t ntile = (n + ((int64_t)1 << shift) - 1) >> shift;
    if (ntile < 2 || ntile * ((int64_t)nkeys + 1) > ((int64_t)1 << 26)) return 0;
    return shift;
}

// batch-compiled rule sets (sh_rules.hip) over HBM-resident columns
static int agg_post(sh_handle* h, sh_device_run* run, int32_t nkeys, const int32_t* d_query, int n_query,
                    const int32_t* agg_kind, const int32_t* arg_type, int n_out);

static int run_rules(sh_handle* h, sh_device_run* run) {
    hipStream_t st = h->stream;
    const int64_t n = run->n;
    const int na = (int)h->stream_types[0].size();
    if (na > 7) return fail(h, SH_E_UNSUPPORTED, "rule engine: at most 7 attributes per stream");
    const bool sorted = h->r_partitioned;
    const int32_t nkeys = sorted ? std::max(1, run->n_keys) : 1;
    if (ensure_ws(h, n) || h->v_flag.ensure_fresh(64)) return fail(h, SH_E_OOM, "workspace");
    h->times = sh_kernel_times{};
    shd_batch B;
    memset(&B, 0, sizeof(B));
    B.ts = run->d_ts;
    B.keys = sorted ? run->d_keys : nullptr;
    B.n = n;
    shd_payload carry;
    void* mid[8] = {nullptr};
    int alias = -1;
    hipEventRecord(h->ev[0], st);
    // SH_RULES_TS32=1: timestamps travel through the segment as 32-bit offsets from
    // the run's first time when its range fits (4 bytes fewer per event and pass).
    // Off by default: on C5 the three passes gained 0.35 ms, the range and
    // conversion passes cost 0.66 ms (profiles/r3_c5_ts32_ab.txt)
    int64_t tlo = 0, thi = 0;
    bool ts32 = false;
    if (sorted && getenv("SH_RULES_TS32") && getenv("SH_RULES_TS32")[0] == '1') {
        if (h->r_tsr.ensure_fresh(64)) return fail(h, SH_E_OOM, "rule workspace");
        if (shr_ts_range(run->d_ts, n, &tlo, &thi, h->r_tsr.p, st)) return fail(h, SH_E_HIP, "timestamp range");
        ts32 = thi >= tlo && (uint64_t)(thi - tlo) <= 0xFFFFFFFFull;
    }
    if (sorted && carry_setup(h, run, &carry, mid, &alias, false, !ts32)) return fail(h, SH_E_OOM, "rule workspace");
    if (ts32) {
        if (h->v_ts32.ensure_fresh((size_t)n * 4) || h->v_sts32.ensure_fresh((size_t)n * 4) ||
            h->v_mid_ts32.ensure_fresh((size_t)n * 4))
            return fail(h, SH_E_OOM, "rule workspace");
        if (shr_ts_to32(run->d_ts, n, tlo, h->v_ts32.as<uint32_t>(), st)) return fail(h, SH_E_HIP, "timestamps");
        carry.src[carry.n] = h->v_ts32.p;
        carry.dst[carry.n] = h->v_sts32.p;
        carry.width[carry.n] = 4;
        mid[carry.n] = h->v_mid_ts32.p;
        carry.n++;
    }
    const uint32_t* sts32 = ts32 ? h->v_sts32.as<uint32_t>() : nullptr;
    shd_segment_ws ws = seg_ws(h, n);
    const uint32_t* perm = nullptr;
    const uint32_t* skeys = nullptr;
    if (shd_segment_payload(&B, nkeys, &ws, st, &perm, &skeys, sorted ? &carry : nullptr, mid, 0, 0))
        return fail(h, SH_E_HIP, "segment launch failed");
    hipEventRecord(h->ev[1], st);
    const int64_t* sts = ts32 ? nullptr : (sorted ? h->v_sts.as<int64_t>() : run->d_ts);
    shd_cols sc;
    memset(&sc, 0, sizeof(sc));
    for (int a = 0; a < na; a++) sc.col[0][a] = sorted ? (const void*)h->v_scol[a].p : run->d_cols[a];
    if (alias >= 0) sc.col[0][alias] = skeys;
    hipMemcpyAsync(h->d_cols_desc.p, &sc, sizeof(sc), hipMemcpyHostToDevice, st);
    const shd_cols* dC = h->d_cols_desc.as<shd_cols>();
    const shr_table* dT = h->rd_tab.as<shr_table>();
    const uint32_t sentinel = sorted ? (uint32_t)nkeys : 0xFFFFFFFFu;
    uint32_t* cnt = h->w_cnt.as<uint32_t>();
    uint32_t* off = h->w_off.as<uint32_t>();
    hipMemsetAsync(h->v_flag.p, 0, 4, st);
    if (shr_count(dT, sts, skeys, n, sentinel, dC, cnt, h->v_flag.as<int32_t>(), st,
                  h->r_img.bytes ? h->rd_img.as<uint8_t>() : nullptr, &h->r_img, sts32, tlo) ||
        shd_exclusive_scan(cnt, off, n, h->w_scan.as<uint32_t>(), st))
        return fail(h, SH_E_HIP, "rule scan launch failed");
    uint32_t lo = 0, lc = 0;
    int32_t flag = 0;
    hipMemcpyAsync(&lo, off + (n - 1), 4, hipMemcpyDeviceToHost, st);
    hipMemcpyAsync(&lc, cnt + (n - 1), 4, hipMemcpyDeviceToHost, st);
    hipMemcpyAsync(&flag, h->v_flag.p, 4, hipMemcpyDeviceToHost, st);
    if (hipStreamSynchronize(st) != hipSuccess) return fail(h, SH_E_HIP, "device error in the rule scan");
    if (flag) return fail(h, SH_E_UNSUPPORTED, "rule engine: timestamps decrease inside a key");
    const int64_t m = (int64_t)lo + lc;
    run->out_count = m;
    if (m > run->out_capacity) return fail(h, SH_E_MORE, "output capacity too small");
    if (m > 0) {
        const int64_t mt = (m + 4095) / 4096;
        const size_t sw = std::max(shd_scan_tmp_words(256 * mt), (size_t)16);
        if (h->r_rec.ensure_fresh((size_t)m * 12) || h->r_keys.ensure_fresh((size_t)m * 12) ||
            h->r_g.ensure_fresh((size_t)m * 8) || h->r_sk.ensure_fresh((size_t)m * 8) ||
            h->r_sv.ensure_fresh((size_t)m * 8) || h->r_hist.ensure_fresh((size_t)256 * mt * 4 + 64) ||
            h->r_scan.ensure_fresh(sw * 4 + 64))
            return fail(h, SH_E_OOM, "match records");
        uint32_t* rec_p = h->r_rec.as<uint32_t>();
        uint32_t* rec_q = rec_p + m;
        uint32_t* rec_r = rec_q + m;
        if (shr_write(dT, sts, skeys, n, sentinel, dC, cnt, off, rec_p, rec_q, rec_r, st,
                      h->r_img.bytes ? h->rd_img.as<uint8_t>() : nullptr, &h->r_img, sts32, tlo))
            return fail(h, SH_E_HIP, "rule write launch failed");
        // PartitionStreamReceiver runs inside each send() call
        const int64_t batch = run->batch_events > 0 ? run->batch_events : 0;
        const uint32_t* flags = nullptr;
        const uint32_t* rid = nullptr;
        const uint32_t* rfirst = nullptr;
        // the runs of the consuming events only, walked back from each record's event
        // (SH_RULES_RUNSCAN=1: flags, scan and first index over every event)
        const bool walk_runs = sorted && !getenv("SH_RULES_RUNSCAN");
        // order key (run, query, consuming event), least significant first; the
        // records are in (opening event, rule) order, which the stable sort keeps
        // among equal keys (creation order of the partials a consumer takes)
        const int64_t runlen = batch > 0 ? std::min(batch, n) : n;
        const int qbits = bits_for((uint64_t)(runlen - 1));
        const int rbits = bits_for((uint64_t)(h->r_rules.size() - 1));
        const int nbits = bits_for((uint64_t)(n - 1));
        const bool packed = qbits + rbits <= 32;
        uint32_t* k0 = h->r_keys.as<uint32_t>();
        uint32_t* k1 = k0 + m;
        uint32_t* k2 = k1 + m;
        bool scan_runs = sorted && !walk_runs;
        if (walk_runs) {
            int32_t* long_run = h->v_flag.as<int32_t>() + 1;
            int32_t lr = 0;
            hipMemsetAsync(long_run, 0, 4, st);
            if (shr_keys(rec_q, rec_r, m, perm, nullptr, nullptr, nullptr, batch, qbits, packed ? 1 : 0, k0, k1, k2,
                         st, run->d_keys, run->d_run, long_run))
                return fail(h, SH_E_HIP, "rule key launch failed");
            hipMemcpyAsync(&lr, long_run, 4, hipMemcpyDeviceToHost, st);
            if (hipStreamSynchronize(st) != hipSuccess) return fail(h, SH_E_HIP, "device error in the rule keys");
            scan_runs = lr != 0;
        }
        if (scan_runs) {
            if (h->r_run.ensure_fresh((size_t)n * 12)) return fail(h, SH_E_OOM, "run ids");
            uint32_t* f = h->r_run.as<uint32_t>();
            if (shr_run_ids(run->d_keys, run->d_run, n, batch, f, f + n, f + 2 * n, h->w_scan.as<uint32_t>(), st))
                return fail(h, SH_E_HIP, "run id launch failed");
            flags = f;
            rid = f + n;
            rfirst = f + 2 * n;
        }
        if ((scan_runs || !walk_runs) &&
            shr_keys(rec_q, rec_r, m, perm, flags, rid, rfirst, batch, qbits, packed ? 1 : 0, k0, k1, k2, st))
            return fail(h, SH_E_HIP, "rule key launch failed");
        const uint32_t* stage_key[3];
        int stage_bits[3];
        int ns = 0;
        if (packed) {
            stage_key[ns] = k0;
            stage_bits[ns++] = qbits + rbits;
        } else {
            stage_key[ns] = k0;
            stage_bits[ns++] = qbits;
            stage_key[ns] = k1;
            stage_bits[ns++] = rbits;
        }
        stage_key[ns] = packed ? k1 : k2;
        stage_bits[ns++] = nbits;
        const uint32_t* order = nullptr;
        uint32_t* gk = h->r_g.as<uint32_t>();
        uint32_t* gv = gk + m;
        uint32_t* kb[2] = {h->r_sk.as<uint32_t>(), h->r_sk.as<uint32_t>() + m};
        uint32_t* vb[2] = {h->r_sv.as<uint32_t>(), h->r_sv.as<uint32_t>() + m};
        for (int s = 0; s < ns; s++) {
            if (stage_bits[s] == 0) continue;
            const uint32_t* ko = nullptr;
            const uint32_t* vo = nullptr;
            if (shr_gather(stage_key[s], order, m, gk, gv, st) ||
                shd_sort_pairs(gk, gv, m, stage_bits[s], kb, vb, h->r_hist.as<uint32_t>(), h->r_scan.as<uint32_t>(),
                               st, &ko, &vo))
                return fail(h, SH_E_HIP, "rule sort launch failed");
            order = vo;
        }
        hipEventRecord(h->ev[2], st);
        if (h->r_aggp) {
            if (!run->d_out_query) {
                if (h->a_q.ensure((size_t)m * 4)) return fail(h, SH_E_OOM, "aggregate query ids");
                run->d_out_query = h->a_q.as<int32_t>();
            }
            if (!run->d_out_seq) {
                if (h->a_seq.ensure((size_t)m * 8)) return fail(h, SH_E_OOM, "aggregate sequence numbers");
                run->d_out_seq = h->a_seq.as<uint64_t>();
            }
        }
        if (shr_place(dT, order, m, rec_p, rec_q, rec_r, perm, sts, dC, 0, std::max(1, h->n_out), run->d_out_seq,
                      run->d_out_query, nullptr, run->d_out_values, st, sts32, tlo))
            return fail(h, SH_E_HIP, "rule placement launch failed");
    } else {
        hipEventRecord(h->ev[2], st);
    }
    hipEventRecord(h->ev[3], st);
    if (hipStreamSynchronize(st) != hipSuccess) return fail(h, SH_E_HIP, "device error in the rule engine");
    hipEventElapsedTime(&h->times.segment_ms, h->ev[0], h->ev[1]);
    hipEventElapsedTime(&h->times.advance_ms, h->ev[1], h->ev[2]);
    hipEventElapsedTime(&h->times.emit_ms, h->ev[2], h->ev[3]);
    hipEventElapsedTime(&h->times.total_ms, h->ev[0], h->ev[3]);
    h->times.advance_launches = 1;
    if (h->r_aggp && m > 0) {
        const int arc = agg_post(h, run, nkeys, run->d_out_query, (int)h->r_rules.size(), h->r_agg, h->r_argt,
                                 std::max(1, h->n_out));
        if (arc < 0) return arc;
        if (arc == 1) return 1;  // not exact in parallel: the caller runs the general engine
    }
    return SH_OK;
}

// bucketed window engine (sh_bucket.hip): partitioned window programs with a
// consumer-side form and a null-free projection; 0 ok, 1 = not applicable or a
// premise failed on the device (the caller runs the general window path),
// SH_E_MORE = output capacity too small (out_count = matches), <0 error
static int run_bucket(sh_handle* h, sh_device_run* run, int32_t nkeys) {
    static const bool off = getenv("SH_DISABLE_BUCKET") != nullptr;
    h->bk_last = 0;
    const shp_program& P = h->prog;
    const int64_t n = run->n;
    if (off || !h->partitioned || nkeys < 1024 || !P.out_fast || n < SHB_TILE) return 1;
    const int kb = std::max(0, bits_for((uint64_t)(nkeys - 1)) - 8);
    if (kb > 8) return 1;
    // select list: e2-side values (and e1's partition attribute, equal to e2's
    // for these types) from the consumer row; other e1-side values ride the match stream
    shb_out O;
    memset(&O, 0, sizeof(O));
    O.n_out = P.n_out;
    int ms[SHB_MAX_MS], n_ms = 0;
    const int part_attr = h->part_attr0;
    for (int o = 0; o < P.n_out; o++) {
        const int a = P.out_attr[o], t = P.attr_type[0][a];
        O.type[o] = t;
        const bool fold = a == part_attr && (t == SH_T_STRING || t == SH_T_INT || t == SH_T_LONG || t == SH_T_BOOL);
        if (P.out_slot[o] == 1 || fold) {
            O.kind[o] = 1;
            O.src[o] = run->d_cols[a];
            continue;
        }
        int m = 0;
        while (m < n_ms && ms[m] != a) m++;
        if (m == n_ms) {
            if (n_ms == SHB_MAX_MS) return 1;
            ms[n_ms++] = a;
        }
        O.kind[o] = 0;
        O.src[o] = (const void*)(intptr_t)m;  // resolved below
    }
    if (h->bk_state == 0) {
        const int lrc = shj_bucket_load(&P, ms, n_ms, &h->bk, &h->bk_err);
        h->bk_state = lrc == 0 ? 1 : (lrc == -1 ? -2 : -1);  // -2: no consumer-side form (not applicable)
    }
    if (h->bk_state != 1) return 1;
    hipStream_t st = h->stream;
    shb_plan B;
    memset(&B, 0, sizeof(B));
    if (n >= ((int64_t)1 << 32) - SHB_TILE) return 1;  // event indices are 32-bit on this engine
    B.n = n;
    B.nt = (int32_t)((n + SHB_TILE - 1) / SHB_TILE);
    B.kb = kb;
    // tiles per matcher chunk: 3,584 events of a bucket at uniform keys (32 per
    // tile), so a chunk and its halo fit the LDS span; denser buckets split
    static const int ct_env = getenv("SH_BK_CT") ? atoi(getenv("SH_BK_CT")) : 0;
    B.ct = ct_env > 0 ? std::min(ct_env, SHB_CT_MAX) : 112;
    B.n_chunks = (B.nt + B.ct - 1) / B.ct;
    const int64_t slots = (int64_t)B.nt * SHB_TILE;  // the tiles' bucket order
    if (ensure_ws(h, std::max<int64_t>(n, (int64_t)B.nt + 1)) || h->bk_w0.ensure_fresh(slots * 4) ||
        h->bk_sp.ensure_fresh(n * 2) || h->bk_toff.ensure_fresh((int64_t)B.nt * SHB_TOFF * 2) ||
        h->bk_cnt.ensure_fresh(slots) || h->bk_mstart.ensure_fresh((int64_t)B.nt * SHB_NB * 4) ||
        h->bk_tpre.ensure_fresh((int64_t)B.nt * 8) || h->bk_tfirst.ensure_fresh((int64_t)B.nt * 8) ||
        h->bk_hstart.ensure_fresh((int64_t)B.nt * 4) || h->bk_ttot.ensure_fresh(((int64_t)B.nt + 1) * 4) ||
        h->bk_flag.ensure_fresh(64) || h->bk_rd.ensure(64))
        return fail(h, SH_E_OOM, "bucket workspace");
    B.n_staged = h->bk.n_staged;
    for (int k = 0; k < B.n_staged; k++) {
        const int a = h->bk.staged_attr[k];
        const int w = type_width(P.attr_type[0][a]);
        if (h->bk_st[k].ensure_fresh(slots * w)) return fail(h, SH_E_OOM, "bucket workspace");
        B.st_src[k] = run->d_cols[a];
        B.st_dst[k] = h->bk_st[k].p;
        B.st_width[k] = w;
    }
    // match stream: one region of SHB_SPAN values per matcher workgroup (its first
    // pass), then a shared tail for further passes; every partial is consumed at
    // most once, so n values suffice for the tail
    B.n_ms = n_ms;
    const int64_t ms_vals = (int64_t)SHB_NB * B.n_chunks * SHB_SPAN + n;
    for (int m = 0; m < n_ms; m++) {
        const int w = type_width(P.attr_type[0][ms[m]]);
        if (h->bk_ms[m].ensure_fresh(ms_vals * w)) return fail(h, SH_E_OOM, "match stream");
        B.ms[m] = h->bk_ms[m].p;
        B.ms_width[m] = w;
    }
    int ms_of[SHB_MAX_OUT];
    for (int o = 0; o < O.n_out; o++) {
        ms_of[o] = O.kind[o] == 0 ? (int)(intptr_t)O.src[o] : -1;
        if (O.kind[o] == 0) O.src[o] = B.ms[ms_of[o]];
    }
    // aggregators carried per key in arrival order (k_bk_aggc: the reference's own
    // additions, no exactness proof): e1-side arguments from one 4-byte match-stream
    // column, e2-side ones from up to two staged columns (one of them 4-byte), count()
    // without one; anything else takes the post-pass (sh_agg.hip)
    shb_aggc AG;
    memset(&AG, 0, sizeof(AG));
    AG.e1_col = AG.e2_col[0] = AG.e2_col[1] = -1;
    bool carry = P.agg_post && !getenv("SH_BK_AGG_POST");
    int agg_of[SHB_MAX_OUT];
    for (int o = 0; o < P.n_out; o++) agg_of[o] = -1;
    for (int o = 0; o < P.n_out && carry; o++) {
        const int ak = P.out_agg[o];
        if (ak == SH_AGG_NONE) continue;
        if (AG.n == SHB_MAX_AGG || (ak != SH_AGG_SUM && ak != SH_AGG_AVG && ak != SH_AGG_COUNT)) {
            carry = false;
            break;
        }
        const int i = AG.n++;
        AG.kind[i] = ak;
        agg_of[o] = i;
        if (ak == SH_AGG_COUNT) {
            AG.side[i] = 3;
            continue;
        }
        const int a = P.out_attr[o], t = P.attr_type[0][a];
        if (t != SH_T_INT && t != SH_T_FLOAT && t != SH_T_LONG && t != SH_T_DOUBLE) {
            carry = false;
            break;
        }
        const int w = type_width(t);
        if (P.out_slot[o] == 0 && ms_of[o] >= 0 && w == 4 && (AG.e1_col < 0 || AG.e1_col == ms_of[o])) {
            AG.e1_col = ms_of[o];
            AG.e1_type = t;
            AG.side[i] = 0;
        } else if (P.out_slot[o] == 1) {
            // the consumer's column at its slot: staged by the partition (the matcher's
            // own staged columns first, then the carry's)
            int k = 0;
            while (k < B.n_staged && (B.st_src[k] != run->d_cols[a])) k++;
            if (k == B.n_staged) {
                if (B.n_staged == SHB_MAX_STAGED || h->bk_st[k].ensure_fresh(slots * w))
                    return B.n_staged == SHB_MAX_STAGED ? 1 : fail(h, SH_E_OOM, "bucket workspace");
                B.st_src[k] = run->d_cols[a];
                B.st_dst[k] = h->bk_st[k].p;
                B.st_width[k] = w;
                B.n_staged++;
            }
            int c = (AG.e2_col[0] == k) ? 0 : (AG.e2_col[1] == k ? 1 : -1);
            if (c < 0) {
                if (AG.e2_col[0] < 0) c = 0;
                else if (AG.e2_col[1] < 0 && w == 4) c = 1;
                else if (AG.e2_col[1] < 0 && type_width(AG.e2_type[0]) == 4) {
                    // keep the 8-byte column in slot 0
                    AG.e2_col[1] = AG.e2_col[0];
                    AG.e2_type[1] = AG.e2_type[0];
                    for (int j = 0; j < i; j++)
                        if (AG.side[j] == 1) AG.side[j] = 2;
                    c = 0;
                } else {
                    carry = false;
                    break;
                }
                AG.e2_col[c] = k;
                AG.e2_type[c] = t;
            }
            AG.side[i] = 1 + c;
        } else {
            carry = false;
        }
    }
    if (carry) {
        for (int i = 0; i < AG.n; i++) {
            if (h->bk_agg[i].ensure_fresh(ms_vals * 8)) return fail(h, SH_E_OOM, "aggregate columns");
            AG.out[i] = h->bk_agg[i].p;
        }
        for (int o = 0; o < O.n_out; o++)
            if (agg_of[o] >= 0) {
                O.kind[o] = 0;
                O.src[o] = AG.out[agg_of[o]];
                O.type[o] = P.out_type[o];
            }
    }
    h->bk_agg_carried = false;
    shb_cols OC;
    memset(&OC, 0, sizeof(OC));
    if (run->d_out_cols && !h->cols_rows && (!P.agg_post || carry)) {
        OC.use = 1;
        for (int o = 0; o < O.n_out; o++) {
            OC.cols[o] = run->d_out_cols[o];
            OC.colw[o] = type_width(O.type[o]);
        }
    }
    B.ts = run->d_ts;
    B.keys = run->d_keys;
    B.w0 = h->bk_w0.as<uint32_t>();
    B.sp = h->bk_sp.as<uint16_t>();
    B.toff = h->bk_toff.as<uint16_t>();
    B.cnt = h->bk_cnt.as<uint8_t>();
    B.mstart = h->bk_mstart.as<uint32_t>();
    B.tpre = h->bk_tpre.as<int64_t>();
    B.tfirst = h->bk_tfirst.as<int64_t>();
    B.hstart = h->bk_hstart.as<int32_t>();
    B.within = std::max<int64_t>(0, P.within_ms);
    B.ttot = h->bk_ttot.as<uint32_t>();
    B.flag = h->bk_flag.as<int32_t>();
    B.ms_ctr = h->bk_flag.as<uint32_t>() + 4;
    static const bool prof = getenv("SH_BK_PROFILE") != nullptr;
    if (prof) {
        if (h->bk_prof.ensure_fresh(128)) return fail(h, SH_E_OOM, "profile");
        hipMemsetAsync(h->bk_prof.p, 0, 128, h->stream);
        B.prof = h->bk_prof.as<unsigned long long>();
    }
    // packed timestamps: ts - tbase in 32 - kb bits, centred on the first event
    hipMemcpyAsync(h->bk_rd.p, run->d_ts, 8, hipMemcpyDeviceToHost, st);
    if (hipStreamSynchronize(st) != hipSuccess) return fail(h, SH_E_HIP, "bucket: timestamp read");
    B.tbase = *h->bk_rd.as<int64_t>() - ((int64_t)1 << (31 - kb));
    hipEventRecord(h->ev[0], st);
    hipMemsetAsync(B.flag, 0, 32, st);  // flag word + match-stream allocator
    hipMemsetAsync(B.ttot, 0, ((int64_t)B.nt + 1) * 4, st);
    if (shb_partition(run->d_keys, run->d_ts, nkeys, &B, st)) return fail(h, SH_E_HIP, "bucket partition launch failed");
    hipEventRecord(h->ev[1], st);
    void* args[] = {&B};
    if (hipModuleLaunchKernel((hipFunction_t)h->bk.match, (unsigned)(SHB_NB * B.n_chunks), 1, 1, 512, 1, 1, 0, st,
                              args, nullptr) != hipSuccess)
        return fail(h, SH_E_HIP, "shb_match launch failed");
    if (carry && shb_agg_carry(&B, &AG, st)) return fail(h, SH_E_HIP, "aggregate carry launch failed");
    if (shb_finish(&B, h->w_scan.as<uint32_t>(), st)) return fail(h, SH_E_HIP, "bucket scan launch failed");
    hipEventRecord(h->ev[2], st);
    if (shb_emit(&B, &O, &OC, 0, run->d_out_seq, run->d_out_values, run->out_capacity, st))
        return fail(h, SH_E_HIP, "bucket emit launch failed");
    hipEventRecord(h->ev[3], st);
    hipMemcpyAsync(h->bk_rd.as<void>(0), B.flag, 4, hipMemcpyDeviceToHost, st);
    hipMemcpyAsync(h->bk_rd.as<void>(8), B.ttot + B.nt, 4, hipMemcpyDeviceToHost, st);
    if (hipStreamSynchronize(st) != hipSuccess) return fail(h, SH_E_HIP, "device error in bucket engine");
    const int32_t flag = *h->bk_rd.as<int32_t>(0);
    const int64_t total = *h->bk_rd.as<uint32_t>(8);
    if (B.prof) {
        unsigned long long pr[16];
        hipMemcpy(pr, B.prof, 128, hipMemcpyDeviceToHost);
        fprintf(stderr, "[shb_match clock ticks, sum over workgroups] load %llu rank %llu walk %llu scan+psum %llu emit %llu\n",
                pr[0], pr[1], pr[2], pr[3], pr[4]);
    }
    if (flag & SHB_F_KEY) return fail(h, SH_E_INVALID_ARG, "partition key id >= n_keys");
    if (flag) return 1;
    run->out_count = total;
    if (total > run->out_capacity) return fail(h, SH_E_MORE, "output capacity too small");
    if (run->d_out_query && total > 0) hipMemsetAsync(run->d_out_query, 0, total * 4, st);
    hipEventElapsedTime(&h->times.segment_ms, h->ev[0], h->ev[1]);
    hipEventElapsedTime(&h->times.advance_ms, h->ev[1], h->ev[2]);
    hipEventElapsedTime(&h->times.emit_ms, h->ev[2], h->ev[3]);
    hipEventElapsedTime(&h->times.total_ms, h->ev[0], h->ev[3]);
    h->times.advance_launches = 1;
    h->bk_last = 1;
    h->bk_agg_carried = carry;
    if (carry) h->agg_last = 4;
    return hipStreamSynchronize(st) == hipSuccess ? SH_OK : fail(h, SH_E_HIP, "bucket engine");
}

// the rise-and-fall sequence on the bucket-carry engine (sh_bucket.hip k_s3b):
// the tile-local bucket partition, one workgroup per bucket carrying its keys'
// state across the stream, the ordered rows by k_bk_emit. 0 ok, 1 = not
// applicable or refused on the device (the caller runs k_seq3s), <0 error
static int run_s3b(sh_handle* h, sh_device_run* run, int32_t nkeys) {
    const bool off = getenv("SH_DISABLE_S3B") != nullptr || getenv("SH_NO_SEQ3") != nullptr;  // (per call: tests A/B it)
    h->s3b_last = 0;
    if (off || !h->partitioned || h->T->n_queries != 1 || !h->T->q[0].s3 || nkeys < 1024 || run->n < SHB_TILE)
        return 1;
    const nf_query& Q = h->T->q[0];
    const int kb = std::max(0, bits_for((uint64_t)(nkeys - 1)) - 8);
    if (kb > 12 || Q.contains_agg) return 1;
    // every operand and select value: one 4-byte attribute A (no null masks on this path)
    const int A = Q.s3_a2, ty = Q.s3_t2;
    if (!(ty == SH_T_FLOAT || ty == SH_T_INT) || A < 0 || A >= (int)h->stream_types[0].size() ||
        type_width(h->stream_types[0][A]) != 4 || Q.s3_a3 != A || Q.s3_e1a != A || Q.s3_la != A || Q.s3_t3 != ty ||
        Q.s3_e1t != ty || Q.s3_lt != ty)
        return 1;
    shb_out O;
    memset(&O, 0, sizeof(O));
    O.n_out = Q.n_out;
    shb_s3 S;
    memset(&S, 0, sizeof(S));
    S.type = ty;
    S.op2 = Q.s3_op2;
    S.dom2 = Q.s3_dom2;
    S.op3 = Q.s3_op3;
    S.dom3 = Q.s3_dom3;
    for (int o = 0; o < Q.n_out; o++) {
        if (Q.s3_out_attr[o] != A || Q.s3_out_type[o] != ty) return 1;
        O.type[o] = ty;
        const int sl = Q.s3_out_slot[o];
        if (sl == 2) {
            O.kind[o] = 1;
            O.src[o] = run->d_cols[A];
            continue;
        }
        int m = 0;
        while (m < S.n_ms && S.ms_slot[m] != sl) m++;
        if (m == S.n_ms) S.ms_slot[S.n_ms++] = sl;
        O.kind[o] = 0;
        O.src[o] = (const void*)(intptr_t)m;  // resolved below
    }
    hipStream_t st = h->stream;
    shb_plan B;
    memset(&B, 0, sizeof(B));
    B.n = run->n;
    B.nt = (int32_t)((run->n + SHB_TILE - 1) / SHB_TILE);
    B.kb = kb;
    B.no_ts = 1;
    const int64_t slots = (int64_t)B.nt * SHB_TILE;
    if (ensure_ws(h, (int64_t)B.nt + 1) || h->bk_w0.ensure_fresh(slots * 4) || h->bk_sp.ensure_fresh(run->n * 2) ||
        h->bk_toff.ensure_fresh((int64_t)B.nt * SHB_TOFF * 2) || h->bk_cnt.ensure_fresh(slots) ||
        h->bk_mstart.ensure_fresh((int64_t)B.nt * SHB_NB * 4) || h->bk_tpre.ensure_fresh((int64_t)B.nt * 8) ||
        h->bk_tfirst.ensure_fresh((int64_t)B.nt * 8) || h->bk_hstart.ensure_fresh((int64_t)B.nt * 4) ||
        h->bk_ttot.ensure_fresh(((int64_t)B.nt + 1) * 4) || h->bk_flag.ensure_fresh(64) || h->bk_rd.ensure(64) ||
        h->bk_st[0].ensure_fresh(slots * 4))
        return fail(h, SH_E_OOM, "sequence workspace");
    B.n_staged = 1;
    B.st_src[0] = run->d_cols[A];
    B.st_dst[0] = h->bk_st[0].p;
    B.st_width[0] = 4;
    // match stream: at most one match per event, in its segment's slots
    B.n_ms = S.n_ms;
    for (int m = 0; m < S.n_ms; m++) {
        if (h->bk_ms[m].ensure_fresh(slots * 4)) return fail(h, SH_E_OOM, "match stream");
        B.ms[m] = h->bk_ms[m].p;
        B.ms_width[m] = 4;
    }
    for (int o = 0; o < O.n_out; o++)
        if (O.kind[o] == 0) O.src[o] = B.ms[(int)(intptr_t)O.src[o]];
    shb_cols OC;
    memset(&OC, 0, sizeof(OC));
    if (run->d_out_cols) {
        OC.use = 1;
        for (int o = 0; o < O.n_out; o++) {
            OC.cols[o] = run->d_out_cols[o];
            OC.colw[o] = 4;
        }
    }
    B.ts = run->d_ts;
    B.keys = run->d_keys;
    B.w0 = h->bk_w0.as<uint32_t>();
    B.sp = h->bk_sp.as<uint16_t>();
    B.toff = h->bk_toff.as<uint16_t>();
    B.cnt = h->bk_cnt.as<uint8_t>();
    B.mstart = h->bk_mstart.as<uint32_t>();
    B.tpre = h->bk_tpre.as<int64_t>();
    B.tfirst = h->bk_tfirst.as<int64_t>();
    B.hstart = h->bk_hstart.as<int32_t>();
    B.ttot = h->bk_ttot.as<uint32_t>();
    B.flag = h->bk_flag.as<int32_t>();
    B.ms_ctr = h->bk_flag.as<uint32_t>() + 4;
    static const bool prof = getenv("SH_BK_PROFILE") != nullptr;
    if (prof) {
        if (h->bk_prof.ensure_fresh(128)) return fail(h, SH_E_OOM, "profile");
        hipMemsetAsync(h->bk_prof.p, 0, 128, st);
        B.prof = h->bk_prof.as<unsigned long long>();
    }
    hipEventRecord(h->ev[0], st);
    hipMemsetAsync(B.flag, 0, 32, st);
    hipMemsetAsync(B.ttot, 0, ((int64_t)B.nt + 1) * 4, st);
    if (shb_partition(run->d_keys, run->d_ts, nkeys, &B, st)) return fail(h, SH_E_HIP, "sequence partition failed");
    hipEventRecord(h->ev[1], st);
    if (shb_s3_carry(&B, &S, st)) return fail(h, SH_E_HIP, "sequence carry launch failed");
    if (shb_finish(&B, h->w_scan.as<uint32_t>(), st)) return fail(h, SH_E_HIP, "sequence scan failed");
    hipEventRecord(h->ev[2], st);
    if (shb_emit(&B, &O, &OC, 0, run->d_out_seq, run->d_out_values, run->out_capacity, st))
        return fail(h, SH_E_HIP, "sequence emit failed");
    hipEventRecord(h->ev[3], st);
    hipMemcpyAsync(h->bk_rd.as<void>(0), B.flag, 4, hipMemcpyDeviceToHost, st);
    hipMemcpyAsync(h->bk_rd.as<void>(8), B.ttot + B.nt, 4, hipMemcpyDeviceToHost, st);
    if (hipStreamSynchronize(st) != hipSuccess) return fail(h, SH_E_HIP, "device error in the sequence engine");
    const int32_t flag = *h->bk_rd.as<int32_t>(0);
    const int64_t total = *h->bk_rd.as<uint32_t>(8);
    if (B.prof) {
        unsigned long long pr[16];
        hipMemcpy(pr, B.prof, 128, hipMemcpyDeviceToHost);
        fprintf(stderr, "[k_s3b clock ticks, sum over workgroups] tables+load %llu sort %llu carry %llu out %llu\n",
                pr[0], pr[1], pr[2], pr[3]);
    }
    if (flag & SHB_F_KEY) return fail(h, SH_E_INVALID_ARG, "partition key id >= n_keys");
    if (flag) return 1;
    run->out_count = total;
    if (total > run->out_capacity) return fail(h, SH_E_MORE, "output capacity too small");
    if (run->d_out_query && total > 0) hipMemsetAsync(run->d_out_query, 0, total * 4, st);
    hipEventElapsedTime(&h->times.segment_ms, h->ev[0], h->ev[1]);
    hipEventElapsedTime(&h->times.advance_ms, h->ev[1], h->ev[2]);
    hipEventElapsedTime(&h->times.emit_ms, h->ev[2], h->ev[3]);
    hipEventElapsedTime(&h->times.total_ms, h->ev[0], h->ev[3]);
    h->times.advance_launches = 1;
    h->s3b_last = 1;
    return hipStreamSynchronize(st) == hipSuccess ? SH_OK : fail(h, SH_E_HIP, "sequence engine");
}

// typed output columns requested: engines that write raw rows write them into a
// workspace that sh_run_device narrows afterwards (the bucketed engine writes
// the columns itself)
static int rows_for_cols(sh_handle* h, sh_device_run* run) {
    if (!run->d_out_cols || h->cols_rows) return SH_OK;
    if (h->w_colrows.ensure((size_t)std::max<int64_t>(1, run->out_capacity) * std::max(1, h->n_out) * 8))
        return fail(h, SH_E_OOM, "typed-column row workspace");
    run->d_out_values = h->w_colrows.as<int64_t>();
    h->cols_rows = true;
    return SH_OK;
}

// the running aggregates of the fast engines' ordered rows (sh_agg.hip): SH_OK,
// 1 = the double additions would round (the caller reruns sequentially), < 0 error
static int agg_post(sh_handle* h, sh_device_run* run, int32_t nkeys, const int32_t* d_query, int n_query,
                    const int32_t* agg_kind, const int32_t* arg_type, int n_out) {
    const int64_t m = run->out_count;
    if (m <= 0) return SH_OK;
    sha_desc D;
    memset(&D, 0, sizeof(D));
    for (int o = 0; o < n_out && D.n_cols < SHA_MAX_COLS; o++)
        if (agg_kind[o] != SH_AGG_NONE) {
            D.c[D.n_cols].col = o;
            D.c[D.n_cols].kind = agg_kind[o];
            D.c[D.n_cols].arg_type = arg_type[o];
            D.n_cols++;
        }
    if (D.n_cols == 0) return SH_OK;
    if (h->a_scratch.ensure((size_t)sha_scratch_bytes(m, D.n_cols))) return fail(h, SH_E_OOM, "aggregate scratch");
    hipEventRecord(h->ev[4], h->stream);
    const int rc = sha_running(run->d_out_seq, run->d_out_values, n_out, m, d_query, n_query,
                               h->partitioned ? run->d_keys : nullptr, h->partitioned ? nkeys : 1, 0, &D,
                               h->a_scratch.p, h->stream);
    if (rc < 0) return fail(h, SH_E_HIP, "aggregate post-pass failed");
    hipEventRecord(h->ev[5], h->stream);
    hipEventSynchronize(h->ev[5]);
    float ms = 0.f;
    hipEventElapsedTime(&ms, h->ev[4], h->ev[5]);
    h->times.emit_ms += ms;
    h->times.total_ms += ms;
    h->agg_last = rc == 0 ? 1 : 2;
    return rc;
}

static int run_device_impl(sh_handle* h, sh_device_run* run) {
    if (!h->has_device) return fail(h, SH_E_NO_DEVICE, "no HIP device");
    if (h->app.n_streams != 1) return fail(h, SH_E_UNSUPPORTED, "sh_run_device: single-stream apps only");
    if (run->n <= 0 || run->n > 0x7FFFFFFFll) return fail(h, SH_E_INVALID_ARG, "sh_run_device: 1 <= n < 2^31");
    // NULL = the default (null) stream, as the header says: the caller's buffers
    // were written there (the handle's own stream is non-blocking and would not
    // wait for them)
    h->stream = (hipStream_t)run->stream;
    if (h->has_rules && (h->mode == 2 || !getenv("SH_DISABLE_RULES"))) {
        const int crc = rows_for_cols(h, run);
        if (crc) return crc;
        int32_t* user_q = run->d_out_query;
        uint64_t* user_seq = run->d_out_seq;
        int rrc = run_rules(h, run);
        if (rrc != 1) return rrc;
        // the aggregates would round in parallel: the general engine adds in sequence
        run->d_out_query = user_q;
        run->d_out_seq = user_seq;
        if (h->mode == 2)
            return fail(h, SH_E_UNSUPPORTED, "rule set aggregates are not exact in parallel and the set is "
                                             "beyond the general engine's query table");
    }
    if (h->mode == 1) {
        const int crc = rows_for_cols(h, run);
        if (crc) return crc;
        // general engine from fresh per-key state; the events arrive as send()
        // calls of run->batch_events
        if (h->T->has_absent) return fail(h, SH_E_UNSUPPORTED, "sh_run_device: absent states need sh_push_batch");
        const int32_t nkeys = h->partitioned ? std::max(1, run->n_keys) : 1;
        if (nf_ensure_keys(h, nkeys)) return fail(h, SH_E_OOM, "key state");
        const nf_query& Q0 = h->T->q[0];
        const bool aggp = h->T->n_queries == 1 && Q0.s3 && Q0.contains_agg;
        if (aggp && !run->d_out_seq) {
            if (h->a_seq.ensure((size_t)std::max<int64_t>(1, run->out_capacity) * 8))
                return fail(h, SH_E_OOM, "aggregate sequence numbers");
            run->d_out_seq = h->a_seq.as<uint64_t>();
        }
        {
            const int src = run_s3b(h, run, nkeys);
            if (src != 1) {
                if (src == SH_OK) h->kstate_stale = true;  // (no key blocks used: reset for a later user)
                return src;
            }
        }
        int rc = SH_OK;
        int64_t rows = 0;
        h->agg_last = 0;
        h->no_seq3 = false;
        for (int pass = 0; pass < 2; pass++) {
            // the rise-and-fall engine keeps no key blocks: their reset waits for a
            // later user (kstate_stale)
            const bool s3_run = h->T->n_queries == 1 && Q0.s3 && !h->no_seq3 && !getenv("SH_NO_SEQ3");
            if (s3_run) {
                h->kstate_stale = true;
            } else {
                hipMemsetAsync(h->n_kstate.p, 0, (size_t)nkeys * h->T->key_words * 8, h->stream);
                h->kstate_stale = false;
            }
            h->started = false;
            rc = nf_start(h);
            if (rc) return rc;
            nf_cols cols;
            memset(&cols, 0, sizeof(cols));
            for (size_t a = 0; a < h->stream_types[0].size(); a++) cols.col[0][a] = run->d_cols[a];
            shd_batch B;
            B.ts = run->d_ts;
            B.stream = nullptr;
            B.row = nullptr;
            B.keys = h->partitioned ? run->d_keys : nullptr;
            B.row_base = 0;
            B.pad = 0;
            B.seq_base = 0;
            B.n = run->n;
            rows = 0;
            h->times = sh_kernel_times{};
            h->dev_want_query = run->d_out_query != nullptr;
            h->dev_run_ids = run->d_run;
            rc = nf_process(h, B, nkeys, cols, run->d_out_seq, run->d_out_values, run->out_capacity, &rows, true,
                            run->batch_events, getenv("SH_NFA_GATHER") ? nullptr : run);
            h->dev_run_ids = nullptr;
            run->out_count = rows;
            if (rc == SH_OK && aggp && h->seq3_last && h->s3_agg) h->agg_last = 3;
            if (rc != SH_OK || !aggp || !h->seq3_last || h->s3_agg) break;
            // k_seq3 wrote the aggregators' arguments: the running values
            int32_t arg_type[NF_MAX_OUT];
            for (int o = 0; o < Q0.n_out; o++) arg_type[o] = Q0.s3_out_type[o];
            const int arc = agg_post(h, run, nkeys, nullptr, 1, Q0.out_agg, arg_type, Q0.n_out);
            if (arc < 0) return arc;
            if (arc == 0) break;
            h->no_seq3 = true;  // not exact: the general engine adds in sequence
        }
        h->no_seq3 = false;
        if (rc == SH_OK && run->d_out_query && rows > 0) {
            hipMemcpyAsync(run->d_out_query, h->w_oq.p, rows * 4, hipMemcpyDeviceToDevice, h->stream);
            hipStreamSynchronize(h->stream);
        }
        return rc;
    }
    const int32_t nkeys = h->partitioned ? std::max(1, run->n_keys) : 1;
    // fresh per-key state
    if (ensure_keys(h, nkeys)) return fail(h, SH_E_OOM, "key state");
    hipMemsetAsync(h->d_kstate.p, 0, (size_t)nkeys * h->lay.key_bytes, h->stream);
    shd_batch B;
    B.ts = run->d_ts;
    B.stream = nullptr;
    B.row = nullptr;
    B.keys = h->partitioned ? run->d_keys : nullptr;
    B.row_base = 0;
    B.seq_base = 0;
    B.n = run->n;
    shd_cols cols;
    memset(&cols, 0, sizeof(cols));
    for (size_t a = 0; a < h->stream_types[0].size(); a++) cols.col[0][a] = run->d_cols[a];
    int64_t nm = 0;
    h->times = sh_kernel_times{};
    h->agg_last = 0;
    // aggregators: the fast engines write raw rows with the arguments, the
    // post-pass turns them into running values (or asks for the sequential engine)
    const bool aggp = h->prog.agg_post != 0;
    bool sequential = false;
    if (aggp) {
        const int crc = rows_for_cols(h, run);
        if (crc) return crc;
        if (!run->d_out_seq) {
            if (h->a_seq.ensure((size_t)std::max<int64_t>(1, run->out_capacity) * 8))
                return fail(h, SH_E_OOM, "aggregate sequence numbers");
            run->d_out_seq = h->a_seq.as<uint64_t>();
        }
    }
    auto finish_agg = [&](int32_t nk) {
        const int arc = agg_post(h, run, nk, nullptr, 1, h->prog.out_agg, h->prog.out_arg_type, h->prog.n_out);
        if (arc == 1) sequential = true;
        return arc;
    };
    if (h->prog.window_ok) {
        const int brc = run_bucket(h, run, nkeys);
        if (brc == SH_OK && aggp && !h->bk_agg_carried) {
            const int arc = finish_agg(nkeys);
            if (arc <= 0) return arc;
        } else if (brc != 1) {
            return brc;
        }
    }
    {
        const int crc = rows_for_cols(h, run);
        if (crc) return crc;
    }
    if (!sequential && h->prog.window_ok && h->stream_types[0].size() <= 7) {
        const int64_t n = run->n;
        hipStream_t st = h->stream;
        if (ensure_ws(h, n)) return fail(h, SH_E_OOM, "workspace");
        const int na = (int)h->stream_types[0].size();
        const bool sorted = h->partitioned;  // unpartitioned: one segment, arrival order
        shd_window_ws wws;
        memset(&wws, 0, sizeof(wws));
        if (h->v_mpos.ensure_fresh(n * 4) || h->v_flag.ensure_fresh(64) || h->v_cnts.ensure_fresh(n * 4))
            return fail(h, SH_E_OOM, "window workspace");
        shd_payload carry;
        void* mid[8] = {nullptr};
        int alias = -1;
        if (sorted && carry_setup(h, run, &carry, mid, &alias)) return fail(h, SH_E_OOM, "window workspace");
        wws.match_pos = h->v_mpos.as<int32_t>();
        wws.cnt_s = h->v_cnts.as<uint32_t>();
        wws.cnt = h->w_cnt.as<uint32_t>();
        wws.off = h->w_off.as<uint32_t>();
        wws.flag = h->v_flag.as<int32_t>();
        // arrival tiles: the sorted order becomes (tile, key, arrival), so the
        // count scatter and the ordered placement touch one tile's output window
        // at a time (L2 / Infinity-Cache resident) instead of the whole stream
        const int tshift = sorted ? tile_shift_for(n, nkeys) : 0;
        hipEventRecord(h->ev[0], st);
        shd_segment_ws ws = seg_ws(h, n);
        const uint32_t* perm = nullptr;
        const uint32_t* skeys = nullptr;
        if (shd_segment_payload(&B, nkeys, &ws, st, &perm, &skeys, sorted ? &carry : nullptr, mid, tshift, 0))
            return fail(h, SH_E_HIP, "segment launch failed");
        shd_tiles TL;
        memset(&TL, 0, sizeof(TL));
        if (tshift) {
            TL.K1 = (uint32_t)nkeys + 1;
            TL.ntile = (uint32_t)((n + ((int64_t)1 << tshift) - 1) >> tshift);
            TL.shift = tshift;
            const size_t words = (size_t)TL.ntile * TL.K1;
            if (h->v_dir.ensure_fresh(words * 8)) return fail(h, SH_E_OOM, "tile directory");
            TL.dstart = h->v_dir.as<uint32_t>();
            TL.dend = h->v_dir.as<uint32_t>() + words;
            if (shd_tile_dir(skeys, n, tshift, TL.K1, TL.ntile, (uint32_t*)TL.dstart, (uint32_t*)TL.dend, st))
                return fail(h, SH_E_HIP, "tile directory launch failed");
        }
        hipEventRecord(h->ev[1], st);
        const int64_t* sts = sorted ? h->v_sts.as<int64_t>() : run->d_ts;
        const void* scols[32];
        for (int a = 0; a < na; a++) scols[a] = sorted ? (const void*)h->v_scol[a].p : run->d_cols[a];
        if (alias >= 0) scols[alias] = skeys;  // the partition column in key-segment order is the sorted key
        if (h->jit_state == 0) {
            if (getenv("SH_DISABLE_JIT")) {
                h->jit_state = -1;
                h->jit_err = "disabled by SH_DISABLE_JIT";
            } else {
                h->jit_state = shj_window_load(&h->prog, &h->jit, &h->jit_err) == 0 ? 1 : -1;
            }
        }
        int wrc = shd_window(h->d_prog.as<shp_program>(), &h->prog, &B, nkeys, perm, skeys, sts, scols, &wws,
                             h->d_cols_desc.as<shd_cols>(), h->w_scan.as<uint32_t>(), run->d_out_seq, nullptr,
                             run->d_out_values, nullptr, run->out_capacity, &nm, st, h->ev[2],
                             h->jit_state == 1 ? &h->jit : nullptr, tshift ? &TL : nullptr);
        hipEventRecord(h->ev[3], st);
        if (hipStreamSynchronize(st) != hipSuccess) return fail(h, SH_E_HIP, "device error in window engine");
        if (wrc < 0) return fail(h, SH_E_HIP, "window engine launch failed");
        run->out_count = nm;
        if (wrc == 2) return fail(h, SH_E_MORE, "output capacity too small");
        if (wrc == 0 && run->d_out_query && nm > 0) hipMemsetAsync(run->d_out_query, 0, nm * 4, st);
        if (wrc == 0) {
            hipEventElapsedTime(&h->times.segment_ms, h->ev[0], h->ev[1]);
            hipEventElapsedTime(&h->times.advance_ms, h->ev[1], h->ev[2]);
            hipEventElapsedTime(&h->times.emit_ms, h->ev[2], h->ev[3]);
            hipEventElapsedTime(&h->times.total_ms, h->ev[0], h->ev[3]);
            h->times.advance_launches = 1;
            if (!aggp) return SH_OK;
            const int arc = finish_agg(nkeys);
            if (arc <= 0) return arc;
        }
        // wrc == 1: timestamps decrease inside a key -> sequential per-key engine
    }
    int rc = run_batch(h, B, nkeys, cols, run->d_out_seq, nullptr, run->d_out_values, nullptr, run->out_capacity,
                       &nm, true);
    run->out_count = nm;
    if (rc == SH_OK && run->d_out_query && nm > 0) {
        hipMemsetAsync(run->d_out_query, 0, nm * 4, h->stream);
        hipStreamSynchronize(h->stream);
    }
    return rc;
}

static int run_device_cols(sh_handle* h, sh_device_run* run);

static_assert(offsetof(sh_device_run, version) == SH_DEVICE_RUN_V1_BYTES, "V1 prefix of sh_device_run");

static int run_device_entry(sh_handle* h, sh_device_run* user, bool v2) {
    if (h && h->poisoned) return fail(h, SH_E_INVALID_ARG, "handle unusable after a failed restore");
    if (!h || !user) return SH_E_INVALID_ARG;
    if (h->has_lists) return fail(h, SH_E_UNSUPPORTED, "List (multi-value) outputs come back through sh_drain");
    // a V1 caller's struct ends before `version`: only its prefix is read
    // the run borrows the caller's stream; the handle's own stream is back for
    // every later call (push, advance, drain), whatever path this one leaves by
    struct StreamGuard {
        sh_handle* h;
        ~StreamGuard() { h->stream = h->own_stream; }
    } guard{h};
    sh_device_run r;
    memset(&r, 0, sizeof(r));
    if (v2) {
        if (user->version != SH_DEVICE_RUN_V2) return fail(h, SH_E_INVALID_ARG, "sh_run_device_v2: version");
        r = *user;
    } else {
        memcpy(&r, user, SH_DEVICE_RUN_V1_BYTES);
    }
    const int rc = run_device_cols(h, &r);
    user->out_count = r.out_count;
    return rc;
}

int sh_run_device(sh_handle* h, sh_device_run* user) { return run_device_entry(h, user, false); }
int sh_run_device_v2(sh_handle* h, sh_device_run* user) { return run_device_entry(h, user, true); }

static int run_device_cols(sh_handle* h, sh_device_run* run) {
    if (!run->d_out_cols) return run_device_impl(h, run);
    // typed columns: one output type per select position across the app's queries
    int32_t w[SHB_MAX_OUT];
    if (h->n_out > SHB_MAX_OUT) return fail(h, SH_E_UNSUPPORTED, "typed columns: too many select values");
    for (int o = 0; o < h->n_out; o++) {
        const int t = o < (int)h->out_types.size() ? h->out_types[o] : SH_T_LONG;
        if (t == -2) return fail(h, SH_E_UNSUPPORTED, "typed columns: queries select different types at one position");
        w[o] = type_width(t);
    }
    int64_t* user_vals = run->d_out_values;
    h->cols_rows = false;
    int rc = run_device_impl(h, run);
    if (h->cols_rows) {
        if (rc == SH_OK && run->out_count > 0) {
            if (shd_narrow_rows(h->w_colrows.as<int64_t>(), h->n_out, run->out_count, run->d_out_cols, w, h->stream) ||
                hipStreamSynchronize(h->stream) != hipSuccess)
                rc = fail(h, SH_E_HIP, "typed-column narrowing failed");
        }
        h->cols_rows = false;
    }
    run->d_out_values = user_vals;
    return rc;
}

// ---- diagnostics of the hipRTC path (not part of the reference-facing ABI)
int shx_jit_status(sh_handle* h) { return h ? h->jit_state : 0; }

// compile-only check of the specialised kernels (no device needed)
int shx_jit_compile(sh_handle* h) {
    if (!h) return SH_E_INVALID_ARG;
    shj_window w;
    std::string err;
    if (!h->prog.window_ok) return fail(h, SH_E_UNSUPPORTED, "not a window-shaped program");
    if (shj_window_compile(&h->prog, &w, &err)) return fail(h, SH_E_HIP, err);
    return SH_OK;
}

// 1: the last sh_run_device ran on the bucketed engine; 0: another engine;
// -1: its matcher could not be built (message in sh_last_error)
int shx_bucket_status(sh_handle* h) {
    if (!h) return 0;
    if (h->bk_state == -2) return 0;  // no consumer-side form: not applicable
    if (h->bk_state < 0) {
        h->err = h->bk_err;
        return -1;
    }
    return h->bk_last;
}

// 1: the last general-engine sh_run_device took the rise-and-fall sequence engine
int shx_seq3_status(sh_handle* h) { return h ? (h->s3b_last ? 2 : h->seq3_last) : 0; }
// aggregators of the last sh_run_device: 0 none on a fast engine, 1 the post-pass
// (sh_agg.hip) formed them, 2 it was not exact and a sequential engine ran
int shx_agg_status(sh_handle* h) { return h ? h->agg_last : 0; }
// 1: the compiled app has the rise-and-fall sequence shape (no device needed)
int shx_seq3_shape(sh_handle* h) { return h && h->T && h->T->n_queries == 1 && h->T->q[0].s3 ? 1 : 0; }

// compile-only check of the bucketed matcher shb_match (no device needed)
int shx_bucket_compile(sh_handle* h, char* buf, int64_t len) {
    if (!h) return SH_E_INVALID_ARG;
    const shp_program& P = h->prog;
    if (!P.window_ok || !P.out_fast) return fail(h, SH_E_UNSUPPORTED, "not a window-shaped projection");
    int ms[SHB_MAX_MS], n_ms = 0;
    for (int o = 0; o < P.n_out; o++) {
        const int a = P.out_attr[o], t = P.attr_type[0][a];
        const bool fold = a == h->part_attr0 && (t == SH_T_STRING || t == SH_T_INT || t == SH_T_LONG || t == SH_T_BOOL);
        if (P.out_slot[o] == 1 || fold) continue;
        int m = 0;
        while (m < n_ms && ms[m] != a) m++;
        if (m == n_ms && n_ms < SHB_MAX_MS) ms[n_ms++] = a;
    }
    std::string src, err;
    if (shj_bucket_source(&P, ms, n_ms, &src)) return fail(h, SH_E_UNSUPPORTED, "no consumer-side form");
    if (buf && len > 0) {
        const int64_t k = std::min<int64_t>(len - 1, (int64_t)src.size());
        memcpy(buf, src.data(), k);
        buf[k] = 0;
    }
    if (shj_bucket_compile(&P, ms, n_ms, &err)) return fail(h, SH_E_HIP, err);
    return SH_OK;
}

int64_t shx_jit_source(sh_handle* h, char* buf, int64_t len) {
    std::string src;
    if (!h || shj_window_source(&h->prog, &src)) return -1;
    if (buf && len > 0) {
        const int64_t k = std::min<int64_t>(len - 1, (int64_t)src.size());
        memcpy(buf, src.data(), k);
        buf[k] = 0;
    }
    return (int64_t)src.size();
}

int sh_last_kernel_times(sh_handle* h, sh_kernel_times* t) {
    if (!h || !t) return SH_E_INVALID_ARG;
    *t = h->times;
    return SH_OK;
}

// ---- snapshot / restore (State.snapshot / restore of the pattern processors,
// StreamPreStateProcessor.java:450-469, driven by SnapshotService.java:90-187,
// 333-430): one opaque, versioned image of everything the matcher carries between
// calls -- partial matches and their events (the column stores they index), the
// schedulers (queues, armed-key lists, HashMap-order models), per-key aggregates,
// the playback clock, sequence counters and undelivered output.
}  // extern "C"

namespace {
const uint32_t kSnapMagic = 0x31534853u;  // "SHS1"
const uint32_t kSnapVersion = 2;  // 2: List values of undelivered rows

struct SnapW {
    std::vector<uint8_t> b;
    bool bad = false;
    void raw(const void* p, size_t n) {
        const uint8_t* q = (const uint8_t*)p;
        b.insert(b.end(), q, q + n);
    }
    template <class T>
    void put(const T& v) {
        raw(&v, sizeof(T));
    }
    template <class T>
    void vec(const std::vector<T>& v) {
        put<uint64_t>(v.size());
        if (!v.empty()) raw(v.data(), v.size() * sizeof(T));
    }
    void dev(const DevBuf& d, size_t n) {
        put<uint64_t>(n);
        if (!n) return;
        if (!d.p || d.bytes < n) {
            bad = true;
            return;
        }
        const size_t at = b.size();
        b.resize(at + n);
        if (hipMemcpy(b.data() + at, d.p, n, hipMemcpyDeviceToHost) != hipSuccess) bad = true;
    }
};

struct SnapR {
    const uint8_t* p;
    size_t n, at = 0;
    bool bad = false;
    bool raw(void* d, size_t k) {
        if (bad || k > n - at) {
            bad = true;
            return false;
        }
        memcpy(d, p + at, k);
        at += k;
        return true;
    }
    template <class T>
    T get() {
        T v{};
        raw(&v, sizeof(T));
        return v;
    }
    template <class T>
    void vec(std::vector<T>& v) {
        const uint64_t k = get<uint64_t>();
        if (bad || k > (n - at) / sizeof(T)) {
            bad = true;
            return;
        }
        v.resize(k);
        if (k) raw(v.data(), k * sizeof(T));
    }
    // restores n bytes into d (grown as needed); returns the byte count
    uint64_t dev(DevBuf& d) {
        const uint64_t k = get<uint64_t>();
        if (bad || k > n - at) {
            bad = true;
            return 0;
        }
        if (!k) return 0;
        if (d.ensure(k) || hipMemcpy(d.p, p + at, k, hipMemcpyHostToDevice) != hipSuccess) bad = true;
        at += k;
        return k;
    }
};

void put_jmap(SnapW& w, const ShJMap& M) {
    w.vec(M.h);
    w.vec(M.nx);
    w.vec(M.pv);
    w.vec(M.pa);
    w.vec(M.lf);
    w.vec(M.rt);
    w.vec(M.fl);
    w.vec(M.code);
    w.vec(M.tab);
    w.put(M.size);
    w.put(M.threshold);
    w.put(M.ord);
    std::vector<int32_t> irr(M.irregular.begin(), M.irregular.end());
    std::sort(irr.begin(), irr.end());
    w.vec(irr);
    w.vec(M.dirty);
    w.put<uint8_t>(M.rerank_all ? 1 : 0);
}

void get_jmap(SnapR& r, ShJMap& M) {
    r.vec(M.h);
    r.vec(M.nx);
    r.vec(M.pv);
    r.vec(M.pa);
    r.vec(M.lf);
    r.vec(M.rt);
    r.vec(M.fl);
    r.vec(M.code);
    r.vec(M.tab);
    M.size = r.get<int32_t>();
    M.threshold = r.get<int32_t>();
    M.ord = r.get<uint64_t>();
    std::vector<int32_t> irr;
    r.vec(irr);
    M.irregular = std::unordered_set<int32_t>(irr.begin(), irr.end());
    r.vec(M.dirty);
    M.rerank_all = r.get<uint8_t>() != 0;
}
}  // namespace

static int snapshot_image(sh_handle* h, SnapW& w) {
    if (h->mode == 2) return fail(h, SH_E_UNSUPPORTED, "snapshot: rule sets run through sh_run_device only");
    int rc = flush(h);  // pending send()s are processed first
    if (rc) return rc;
    if (h->has_device && hipStreamSynchronize(h->stream) != hipSuccess) return fail(h, SH_E_HIP, "snapshot sync");
    w.put(kSnapMagic);
    w.put(kSnapVersion);
    w.put<int32_t>(h->mode);
    w.put(h->fp);
    w.put(h->seq_next);
    w.put(h->seq_staged0);
    w.put(h->max_key);
    w.put(h->clock);
    w.put(h->tick);
    w.put<uint8_t>(h->started ? 1 : 0);
    w.put(h->batch_id);
    w.vec(h->o_query);
    w.vec(h->o_seq);
    w.vec(h->o_ts);
    w.vec(h->o_vals);
    w.vec(h->o_nulls);
    w.put(h->o_read);
    // the List values undelivered rows hold
    w.vec(h->l_vals);
    w.vec(h->l_nuls);
    w.vec(h->l_start);
    w.put(h->l_base);
    w.put<int32_t>((int32_t)h->stores.size());
    for (size_t s = 0; s < h->stores.size(); s++) {
        const auto& st = h->stores[s];
        w.put(st.rows);
        w.put<int32_t>((int32_t)st.cols.size());
        for (size_t a = 0; a < st.cols.size(); a++) {
            w.put<uint8_t>(st.has_nul[a] ? 1 : 0);
            w.dev(st.cols[a], (size_t)st.rows * type_width(h->stream_types[s][a]));
            w.dev(st.nuls[a], st.has_nul[a] ? (size_t)st.rows : 0);
        }
    }
    if (h->mode == 0) {
        w.put(h->lay);
        w.put(h->nkeys_alloc);
        w.dev(h->d_kstate, (size_t)h->nkeys_alloc * h->lay.key_bytes);
    } else {
        w.put(*h->T);
        w.raw(h->caps, sizeof(h->caps));
        w.put(h->n_nkeys);
        w.put<int32_t>(h->klist_cur);
        const size_t nk = (size_t)h->n_nkeys;
        w.dev(h->n_kstate, nk * h->T->key_words * 8);
        w.dev(h->n_armed, nk);
        w.dev(h->n_klist[0], nk ? nk * 4 : 0);
        w.dev(h->n_klist[1], nk ? nk * 4 : 0);
        w.dev(h->n_arm_log, nk ? nk * 4 : 0);
        w.dev(h->n_klist_n, h->n_klist_n.p ? 16 : 0);
        w.dev(h->n_arm_ctr, h->n_arm_ctr.p ? 8 : 0);
        w.put<uint8_t>(h->sm_on ? 1 : 0);
        if (h->sm_on) {
            w.vec(h->sm.chars);
            w.vec(h->sm.off);
            w.vec(h->sm.len);
            w.vec(h->sm.hash);
            w.vec(h->sm.used);
            for (int s : h->sm.used) {
                put_jmap(w, h->sm.maps[s]);
                w.dev(h->n_rank[s], nk * 8);
            }
        }
    }
    if (w.bad) return fail(h, SH_E_HIP, "snapshot: device read-back failed");
    return SH_OK;
}

extern "C" {

int sh_snapshot(sh_handle* h, void* buf, int64_t cap, int64_t* size) {
    if (h && h->coord_on) return fail(h, SH_E_UNSUPPORTED, "snapshots of key-sharded handles are not supported");
    if (h && h->poisoned) return fail(h, SH_E_INVALID_ARG, "handle unusable after a failed restore");
    if (!h || !size || (cap > 0 && !buf)) return SH_E_INVALID_ARG;
    if (h->kstate_stale && h->n_kstate.p) {
        hipMemsetAsync(h->n_kstate.p, 0, (size_t)h->n_nkeys * h->T->key_words * 8, h->stream);
        hipStreamSynchronize(h->stream);
        h->kstate_stale = false;
    }
    if (h->has_device) {
        const int frc = nf_sev_flush(h);  // the models and ranks the image holds
        if (frc) return frc;
    }
    SnapW w;
    const int rc = snapshot_image(h, w);
    if (rc) return rc;
    *size = (int64_t)w.b.size();
    if (!buf || cap < *size) return SH_E_MORE;
    memcpy(buf, w.b.data(), w.b.size());
    return SH_OK;
}

static int restore_image(sh_handle* h, const void* buf, int64_t size);

int sh_restore(sh_handle* h, const void* buf, int64_t size) {
    if (!h || !buf || size <= 0) return SH_E_INVALID_ARG;
    if (h->poisoned) return fail(h, SH_E_INVALID_ARG, "handle unusable after a failed restore");
    if (!h->has_device) return fail(h, SH_E_NO_DEVICE, "no HIP device: the matcher has no CPU fallback");
    for (auto& st : h->stores)
        if (st.rows) return fail(h, SH_E_INVALID_ARG, "restore: the handle has processed events already");
    // the image is applied as it is parsed: keep the handle's own (fresh) image
    // and put it back when the new one turns out damaged, so a failed restore
    // leaves the handle as it was
    SnapW w0;
    int rc = snapshot_image(h, w0);
    if (rc) return rc;
    rc = restore_image(h, buf, size);
    if (rc != SH_OK) {
        const std::string why = h->err;
        if (restore_image(h, w0.b.data(), (int64_t)w0.b.size()) != SH_OK) {
            h->poisoned = true;
            return fail(h, rc, why + " (and the handle could not be reset: " + h->err + "; it refuses further calls)");
        }
        return fail(h, rc, why);
    }
    return SH_OK;
}

static int restore_image(sh_handle* h, const void* buf, int64_t size) {
    SnapR r{(const uint8_t*)buf, (size_t)size};
    if (r.get<uint32_t>() != kSnapMagic || r.get<uint32_t>() != kSnapVersion)
        return fail(h, SH_E_INVALID_ARG, "restore: not a matcher snapshot image of this version");
    if (r.get<int32_t>() != h->mode || r.get<uint64_t>() != h->fp)
        return fail(h, SH_E_INVALID_ARG, "restore: the image was taken from a different app");
    hipStreamSynchronize(h->stream);
    h->seq_next = r.get<uint64_t>();
    h->seq_staged0 = r.get<uint64_t>();
    h->max_key = r.get<int32_t>();
    h->clock = r.get<int64_t>();
    h->tick = r.get<uint64_t>();
    h->started = r.get<uint8_t>() != 0;
    h->batch_id = r.get<uint32_t>();
    r.vec(h->o_query);
    r.vec(h->o_seq);
    r.vec(h->o_ts);
    r.vec(h->o_vals);
    r.vec(h->o_nulls);
    h->o_read = r.get<int64_t>();
    r.vec(h->l_vals);
    r.vec(h->l_nuls);
    r.vec(h->l_start);
    h->l_base = r.get<int64_t>();
    h->st_ts.clear();
    h->st_stream.clear();
    h->st_row.clear();
    h->st_key.clear();
    if (r.get<int32_t>() != (int32_t)h->stores.size()) r.bad = true;
    for (size_t s = 0; s < h->stores.size() && !r.bad; s++) {
        auto& st = h->stores[s];
        st.rows = r.get<int64_t>();
        if (r.get<int32_t>() != (int32_t)st.cols.size()) r.bad = true;
        for (size_t a = 0; a < st.cols.size() && !r.bad; a++) {
            st.has_nul[a] = r.get<uint8_t>() != 0;
            r.dev(st.cols[a]);
            r.dev(st.nuls[a]);
        }
    }
    if (h->mode == 0 && !r.bad) {
        h->lay = r.get<shp_layout>();
        h->nkeys_alloc = r.get<int32_t>();
        r.dev(h->d_kstate);
    } else if (!r.bad) {
        *h->T = r.get<nf_table>();
        r.raw(h->caps, sizeof(h->caps));
        h->n_nkeys = r.get<int32_t>();
        h->klist_cur = r.get<int32_t>();
        r.dev(h->n_kstate);
        r.dev(h->n_armed);
        r.dev(h->n_klist[0]);
        r.dev(h->n_klist[1]);
        r.dev(h->n_arm_log);
        r.dev(h->n_klist_n);
        r.dev(h->n_arm_ctr);
        const bool sm_on = r.get<uint8_t>() != 0;
        if (sm_on != h->sm_on) r.bad = true;
        if (sm_on && !r.bad) {
            r.vec(h->sm.chars);
            r.vec(h->sm.off);
            r.vec(h->sm.len);
            r.vec(h->sm.hash);
            std::vector<int> used;
            r.vec(used);
            if (used != h->sm.used) r.bad = true;
            for (int s : used) {
                if (r.bad) break;
                get_jmap(r, h->sm.maps[s]);
                r.dev(h->n_rank[s]);
            }
        }
        if (!r.bad && nf_upload_table(h)) r.bad = true;
    }
    if (r.bad || r.at != r.n) return fail(h, SH_E_INVALID_ARG, "restore: truncated or inconsistent image");
    if (hipStreamSynchronize(h->stream) != hipSuccess) return fail(h, SH_E_HIP, "restore upload");
    return SH_OK;
}

}  // extern "C"
