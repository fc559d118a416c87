// sh_host.cpp — host side of libsiddhi_hip.so: the C-ABI (include/siddhi_hip.h),
// lowering of the app descriptor to the device NFA program, HBM residency of
// event columns and per-key state, and the launch sequence
//   radix segment -> per-key advance -> ordered placement.
//
// The product path has no CPU fallback: without a device every call that
// needs one returns SH_E_NO_DEVICE.
#include "sh_host_int.h"

#define SH_VERSION_STR "siddhi_hip 0.2 (gfx950; sh_device_run layout 2)"

namespace {

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

static void set_layout(shp_layout& Y, const shp_program& P, int32_t cap) {
    Y.cap = cap;
    Y.rec_words = 2 + (P.n_states + 1) / 2;
    Y.list_bytes = (int64_t)Y.cap * Y.rec_words * 8;
    Y.off_lists = (int64_t)(1 + SHP_MAX_STATES) * 8;
    Y.off_agg = Y.off_lists + (int64_t)(P.n_states > 1 ? P.n_states - 1 : 0) * 2 * Y.list_bytes;
    Y.key_bytes = Y.off_agg + (int64_t)P.n_out * 5 * 8;
    Y.key_bytes = (Y.key_bytes + 63) & ~63ll;
}

int fail(sh_handle* h, int code, const std::string& m) {
    if (h) h->err = m;
    return code;
}

static bool device_available() {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return false;
    return n > 0;
}


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
    if (h->mode == 1 && h->pend.on) nf_settle(h);
    nf_hist_stop(h);
    if (getenv("SH_HOST_PROF") && h->hp_n[0]) {
        static const char* names[SH_HP_N] = {"push",      "timers",     "process",   "history",
                                             "place",     "drain",      "hist_copy", "hist_apply",
                                             "hist_rank", "hist_records", "sync_wait", "pull"};
        fprintf(stderr, "[sh host profile]");
        for (int i = 0; i < SH_HP_N; i++) {
            if (i == 9)
                fprintf(stderr, " %s %lld", names[i], (long long)h->hp_n[i]);
            else
                fprintf(stderr, " %s %.1f ms / %lld", names[i], h->hp_ms[i], (long long)h->hp_n[i]);
        }
        fprintf(stderr, "\n");
    }
    if (h->has_device) {
        hipStreamSynchronize(h->stream);
        h->pin_in.release();
        h->pin_stage.release();
        h->pin_rd.release();
        h->pin_out.release();
        h->pin_hist.release();
        h->pin_sev.release();
        h->pin_rk.release();
        h->pin_cand.release();
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
        if ((size_t)(r0 + b->n) * w > st.cols[a].bytes && h->mode == 1) {
            const int src = nf_settle(h);  // (the store moves: a pending launch reads it)
            if (src) return src;
        }
        if (st.cols[a].ensure((size_t)(r0 + b->n) * w)) return fail(h, SH_E_OOM, "column store");
        // through pinned staging (the sync below completes the copy before reuse)
        memcpy(h->pin_in.as<void>(pin_off), b->cols[a], (size_t)b->n * w);
        hipMemcpyAsync((uint8_t*)st.cols[a].p + r0 * w, h->pin_in.as<void>(pin_off), b->n * w, hipMemcpyHostToDevice,
                       h->stream);
        pin_off += (size_t)b->n * w;
        const uint8_t* nm = b->nulls ? b->nulls[a] : nullptr;
        if (nm || st.has_nul[a]) {
            // the mask moves when it grows: a pending launch reads it (settle first)
            if ((size_t)(r0 + b->n) > st.nuls[a].bytes && h->mode == 1) {
                const int src = nf_settle(h);
                if (src) return src;
            }
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
    if (h->mode == 1) {
        int frc = nf_settle(h);
        if (!frc) frc = nf_sev_flush(h);  // (the replay thread reads the key strings)
        if (frc) return frc;
    }
    if (!h->sm.keys_settable(first_key, n, utf16, offsets))
        return fail(h, SH_E_INVALID_ARG,
                    "sh_set_partition_keys: a key id was used before its string was registered (its scheduler "
                    "map position follows the old string); register strings before the ids appear");
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

int ensure_ws(sh_handle* h, int64_t n) {
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
int flush(sh_handle* h) {
    if (h->mode == 1) {  // the general engine processes each send() at once
        const int src = nf_settle(h);  // (a push's launch may still be pending)
        return src ? src : nf_app_pull(h);
    }
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
            // (the sequence bucket-carry engine writes typed columns / packed rows itself)
            const int src = run_s3b(h, run, nkeys);
            if (src != 1) {
                if (src == SH_OK) h->kstate_stale = true;  // (no key blocks used: reset for a later user)
                return src;
            }
        }
        {
            const int crc = rows_for_cols(h, run);
            if (crc) return crc;
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
        if (h->prog.window_ok && h->out_mode != SHB_OUT_RAW && !h->cols_rows && !getenv("SH_BK_AGG_POST")) {
            // packed rows / typed columns straight from the bucketed engine when its
            // parallel carry takes the batch (the post-pass works on raw rows)
            h->aggp_only = true;
            const int brc = run_bucket(h, run, nkeys);
            h->aggp_only = false;
            if (brc == SH_OK && h->bk_agg_carried) return SH_OK;
            if (brc != SH_OK && brc != 1) return brc;
        }
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
        int brc = run_bucket(h, run, nkeys);
        if (brc == SH_OK && aggp && !h->bk_agg_carried) {
            const int arc = finish_agg(nkeys);
            if (arc <= 0) return arc;
            if (!getenv("SH_BK_AGG_POST")) {
                // the post-pass's additions are not exact in parallel: the bucketed
                // engine again, its carry adding in the reference's sequence
                brc = run_bucket(h, run, nkeys, true);
                if (brc == SH_OK && h->bk_agg_carried) return SH_OK;
                if (brc != SH_OK && brc != 1) return brc;
            }
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
    if (h->mode == 1) {
        const int src = nf_settle(h);  // a streaming push's launch, on the handle's own stream
        if (src) return src;
    }
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
    // a binding built against the 0.1 header (version / pad at offset 88, the
    // typed columns at 96) leaves a small integer where d_out_cols now sits:
    // refuse it rather than write through it
    if (r.d_out_cols && (uintptr_t)r.d_out_cols < 65536)
        return fail(h, SH_E_INVALID_ARG,
                    "sh_run_device: d_out_cols holds a small integer (a caller built against the 0.1 "
                    "sh_device_run layout, version at offset 88?) -- rebuild against this header");
    const int rc = run_device_cols(h, &r);
    user->out_count = r.out_count;
    return rc;
}

int sh_run_device(sh_handle* h, sh_device_run* user) { return run_device_entry(h, user, false); }
int sh_run_device_v2(sh_handle* h, sh_device_run* user) { return run_device_entry(h, user, true); }

// the natural width of every select position (typed columns / packed rows)
static int out_widths(sh_handle* h, int32_t* w, const char* what) {
    if (h->n_out > SHB_MAX_OUT) return fail(h, SH_E_UNSUPPORTED, std::string(what) + ": too many select values");
    for (int o = 0; o < h->n_out; o++) {
        const int t = o < (int)h->out_types.size() ? h->out_types[o] : SH_T_LONG;
        if (t == -2) return fail(h, SH_E_UNSUPPORTED, std::string(what) + ": queries select different types at one position");
        w[o] = type_width(t);
    }
    return SH_OK;
}

// packed rows: the sequence number in words 0-1, each value aligned to its width
// (1-byte values in a 4-byte slot), the row a multiple of 4 words (16 B)
static void packed_layout(const int32_t* w, int n_out, int32_t* woff, int32_t* rw) {
    int pos = 2;
    for (int o = 0; o < n_out; o++) {
        const int wd = w[o] == 8 ? 2 : 1;
        if (wd == 2 && (pos & 1)) pos++;
        woff[o] = pos;
        pos += wd;
    }
    *rw = (pos + 3) & ~3;
}

int sh_packed_row_layout(sh_handle* h, int32_t* offsets, int32_t cap, int32_t* n_out, int32_t* row_bytes) {
    if (!h || !n_out || !row_bytes) return SH_E_INVALID_ARG;
    int32_t w[SHB_MAX_OUT], woff[SHB_MAX_OUT], rw = 0;
    const int rc = out_widths(h, w, "packed rows");
    if (rc) return rc;
    packed_layout(w, h->n_out, woff, &rw);
    for (int o = 0; o < h->n_out && offsets && o < cap; o++) offsets[o] = woff[o] * 4;
    *n_out = h->n_out;
    *row_bytes = rw * 4;
    return SH_OK;
}

static int run_device_cols(sh_handle* h, sh_device_run* run) {
    if (run->out_layout != SH_OUT_RAW && run->out_layout != SH_OUT_PACKED)
        return fail(h, SH_E_INVALID_ARG, "sh_device_run.out_layout");
    const bool packed = run->out_layout == SH_OUT_PACKED;
    if (packed && run->d_out_cols) return fail(h, SH_E_INVALID_ARG, "packed rows and typed columns together");
    if (packed && !run->d_out_values) return fail(h, SH_E_INVALID_ARG, "packed rows: d_out_values is NULL");
    if (!run->d_out_cols && !packed) return run_device_impl(h, run);
    // one output type per select position across the app's queries
    int32_t w[SHB_MAX_OUT];
    {
        const int wrc = out_widths(h, w, packed ? "packed rows" : "typed columns");
        if (wrc) return wrc;
    }
    h->out_mode = packed ? SHB_OUT_PACKED : SHB_OUT_COLS;
    if (packed) {
        for (int o = 0; o < h->n_out; o++) h->pk_w[o] = w[o];
        packed_layout(w, h->n_out, h->pk_woff, &h->pk_rw);
    }
    int64_t* user_vals = run->d_out_values;
    uint64_t* user_seq = run->d_out_seq;
    h->cols_rows = false;
    int rc = run_device_impl(h, run);
    if (h->cols_rows) {
        if (rc == SH_OK && run->out_count > 0) {
            const int64_t m = std::min(run->out_count, run->out_capacity);
            const int crc = packed ? shd_pack_rows(h->w_packseq.as<uint64_t>(), h->w_colrows.as<int64_t>(), h->n_out, m,
                                                   w, h->pk_woff, h->pk_rw, user_vals, h->stream)
                                   : shd_narrow_rows(h->w_colrows.as<int64_t>(), h->n_out, m, run->d_out_cols, w,
                                                     h->stream);
            if (crc || hipStreamSynchronize(h->stream) != hipSuccess)
                rc = fail(h, SH_E_HIP, packed ? "packed-row conversion failed" : "typed-column narrowing failed");
        }
        h->cols_rows = false;
    }
    h->out_mode = SHB_OUT_RAW;
    run->d_out_values = user_vals;
    run->d_out_seq = user_seq;
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

// 1: the last sh_run_device ran on the bucketed engine; 0: another engine; -1: its matcher
// could not be built (message in sh_last_error)
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

int shx_rules_status(sh_handle* h) { return h ? h->rs_last : 0; }

// SH_HOST_PROF phase clocks of a streaming handle (ms and counts, SH_HP_N phases)
int shx_host_profile(sh_handle* h, double* ms, int64_t* n, int cap) {
    if (!h) return 0;
    const int k = cap < SH_HP_N ? cap : SH_HP_N;
    for (int i = 0; i < k; i++) {
        if (ms) ms[i] = h->hp_ms[i];
        if (n) n[i] = h->hp_n[i];
    }
    return SH_HP_N;
}
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
