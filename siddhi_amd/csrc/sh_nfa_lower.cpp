// sh_nfa_lower.cpp — lowers an sh_app_desc (the query-api StateElement trees)
// into the general engine's NFA table (sh_nfa.h). Restates, per query,
// StateInputStreamParser.parseInputStream / parse
// (core/util/parser/StateInputStreamParser.java:76-408):
//   - one receiver per stream: Single if the stream feeds one state, Multi(k)
//     otherwise, eventSequence = slots in reverse (:91-110);
//   - parse() builds the pre/post processor graph: Next links post -> next pre
//     (NextStateElement), Every links the last post back to the first pre and sets
//     withinEvery on the whole sub-tree, Logical creates a partner pair and parses
//     element 2 before element 1 (:350-361), Count wraps a stream state;
//   - StateStreamRuntime.setCommonProcessor: root first's thisLast = root last,
//     setQuerySelector, then setup() wires receivers (StateStreamRuntime.java:38-98);
//   - InnerStateRuntime init/reset/update orders (state/runtime/*.java) become flat
//     sequences of pre-state ids.
// Pure host C++: linked into libsiddhi_hip.so (sh_compile) and into the CPU test
// harness tests/nfa_host.
#include <algorithm>
#include <cstring>
#include <map>
#include <functional>
#include <memory>
#include <string>
#include <vector>

#include "sh_nfa.h"
#include "sh_nfa_lower.h"

namespace {

struct LProc {
    int kind = NF_K_STREAM;
    int stateId = -1;
    bool isStart = false;
    int stream = -1;
    int withinEvery = -1;
    int thisLast = -1;   // proc id
    int partner = -1;    // proc id
    int ltype = 0;
    int nextPre = -1, nextEveryPre = -1, callbackPre = -1;
    bool toSel = false;
    int minc = 0, maxc = 0;
    int64_t waiting = -1;
    int filter = -1;
    bool alog = false;   // AbsentLogicalPreStateProcessor (a Logical pre with its own scheduler)
};

struct LInner {
    enum { BASIC, NEXT, EVERY, LOGICAL } type = BASIC;
    int first = -1, last = -1;  // proc ids
    LInner* a = nullptr;        // NEXT: cur, EVERY: in, LOGICAL: in1
    LInner* b = nullptr;        // NEXT: nxt, LOGICAL: in2
    std::vector<std::pair<int, int>> ssr;  // (stream, proc)
};

struct QueryLowering {
    const sh_app_desc* app;
    const sh_query_desc* q;
    nf_table* T;
    nf_query* Q;
    std::string err;
    std::vector<LProc> procs;
    std::vector<std::unique_ptr<LInner>> inners;
    std::vector<int> pres;       // parse order
    std::vector<int> startup;    // absent pres (partitionCreated order)
    std::vector<int> schedOrder; // scheduler-owning pres in Scheduler creation order
    int slotCounter = 0;
    std::map<int, int> uses;     // stream -> states fed

    LInner* newInner() {
        inners.emplace_back(new LInner());
        return inners.back().get();
    }
    int newProc(int kind) {
        procs.emplace_back();
        procs.back().kind = kind;
        return (int)procs.size() - 1;
    }
    // setNextStatePre (StreamPost / CountPost / LogicalPost)
    void setNextStatePre(int post, int p) {
        LProc& o = procs[post];
        o.nextPre = p;
        if (o.kind == NF_K_COUNT) {
            if (o.isStart && q->state_type == SH_SEQUENCE && o.minc == 0) procs[p].callbackPre = post;
        } else if (o.kind == NF_K_LOGICAL) {
            procs[o.partner].nextPre = p;
        }
    }
    void setNextEveryStatePre(int post, int p) {
        LProc& o = procs[post];
        o.nextEveryPre = p;
        if (o.kind == NF_K_LOGICAL) procs[o.partner].nextEveryPre = p;
    }

    LInner* parse(int ei, int pre, std::vector<int>& list, bool isStart) {
        if (ei < 0 || ei >= q->n_elems) {
            err = "bad state element index";
            return nullptr;
        }
        const sh_state_elem& e = q->elems[ei];
        switch (e.kind) {
            case SH_E_STREAM:
            case SH_E_ABSENT_STREAM: {
                if (e.stream < 0 || e.stream >= app->n_streams) {
                    err = "bad stream index";
                    return nullptr;
                }
                const int stateIndex = slotCounter++;
                if (stateIndex != e.slot) {
                    err = "slot mismatch between descriptor and parse order";
                    return nullptr;
                }
                if (pre < 0) {
                    if (e.kind == SH_E_ABSENT_STREAM) {
                        pre = newProc(NF_K_ABSENT);
                        procs[pre].waiting = e.waiting_ms;
                        startup.push_back(pre);
                        schedOrder.push_back(pre);
                    } else {
                        pre = newProc(NF_K_STREAM);
                    }
                } else if (e.kind == SH_E_ABSENT_STREAM && !procs[pre].alog) {
                    err = "device engine: absent states inside counts are not lowered";
                    return nullptr;
                }
                LProc& P = procs[pre];
                P.stateId = stateIndex;
                P.isStart = isStart;
                P.stream = e.stream;
                P.filter = e.filter;
                P.thisLast = pre;
                uses[e.stream]++;
                LInner* in = newInner();
                in->first = in->last = pre;
                in->ssr.push_back({e.stream, pre});
                list.push_back(pre);
                return in;
            }
            case SH_E_NEXT: {
                LInner* cur = parse(e.child0, -1, list, isStart);
                if (!cur) return nullptr;
                LInner* nxt = parse(e.child1, -1, list, false);
                if (!nxt) return nullptr;
                setNextStatePre(cur->last, nxt->first);
                LInner* ni = newInner();
                ni->type = LInner::NEXT;
                ni->a = cur;
                ni->b = nxt;
                ni->first = cur->first;
                ni->last = nxt->last;
                ni->ssr = cur->ssr;
                ni->ssr.insert(ni->ssr.end(), nxt->ssr.begin(), nxt->ssr.end());
                return ni;
            }
            case SH_E_EVERY: {
                std::vector<int> wl;
                LInner* in = parse(e.child0, -1, wl, isStart);
                if (!in) return nullptr;
                LInner* ev = newInner();
                ev->type = LInner::EVERY;
                ev->a = in;
                ev->first = in->first;
                ev->last = in->last;
                ev->ssr = in->ssr;
                setNextEveryStatePre(ev->last, ev->first);
                for (int p : wl) procs[p].withinEvery = ev->first;
                list.insert(list.end(), wl.begin(), wl.end());
                return ev;
            }
            case SH_E_LOGICAL_AND:
            case SH_E_LOGICAL_OR: {
                if (e.child0 < 0 || e.child1 < 0) {
                    err = "bad logical element";
                    return nullptr;
                }
                const sh_state_elem& e1 = q->elems[e.child0];
                const sh_state_elem& e2 = q->elems[e.child1];
                // an absent element gets AbsentLogicalPre/Post and its own scheduler,
                // element 1's first (StateInputStreamParser.java:289-344)
                const int p1 = newProc(NF_K_LOGICAL);
                const int p2 = newProc(NF_K_LOGICAL);
                const int pe[2] = {p1, p2};
                const sh_state_elem* ee[2] = {&e1, &e2};
                for (int k = 0; k < 2; k++) {
                    if (ee[k]->kind != SH_E_ABSENT_STREAM) continue;
                    procs[pe[k]].alog = true;
                    procs[pe[k]].waiting = ee[k]->waiting_ms;
                    startup.push_back(pe[k]);
                    schedOrder.push_back(pe[k]);
                }
                procs[p1].ltype = procs[p2].ltype = e.kind;
                procs[p1].partner = p2;
                procs[p2].partner = p1;
                LInner* in2 = parse(e.child1, p2, list, isStart);
                if (!in2) return nullptr;
                LInner* in1 = parse(e.child0, p1, list, isStart);
                if (!in1) return nullptr;
                LInner* li = newInner();
                li->type = LInner::LOGICAL;
                li->a = in1;
                li->b = in2;
                li->first = in1->first;
                li->last = in2->last;
                li->ssr = in2->ssr;
                li->ssr.insert(li->ssr.end(), in1->ssr.begin(), in1->ssr.end());
                return li;
            }
            case SH_E_COUNT: {
                const int cp = newProc(NF_K_COUNT);
                procs[cp].minc = e.min_count == SH_ANY ? 0 : e.min_count;
                procs[cp].maxc = e.max_count == SH_ANY ? INT32_MAX : e.max_count;
                LInner* in = parse(e.child0, cp, list, isStart);
                if (!in) return nullptr;
                LInner* ci = newInner();  // CountInnerStateRuntime: same first / last / ssr
                ci->first = in->first;
                ci->last = in->last;
                ci->ssr = in->ssr;
                return ci;
            }
        }
        err = "unknown state element";
        return nullptr;
    }

    // InnerStateRuntime orders
    void initSeq(LInner* n, std::vector<int>& out) {
        switch (n->type) {
            case LInner::NEXT:
                initSeq(n->a, out);
                initSeq(n->b, out);
                return;
            case LInner::EVERY: initSeq(n->a, out); return;
            case LInner::LOGICAL:
                initSeq(n->b, out);
                initSeq(n->a, out);
                return;
            default: out.push_back(n->first);
        }
    }
    void resetSeq(LInner* n, std::vector<int>& out) {
        switch (n->type) {
            case LInner::NEXT:
                resetSeq(n->b, out);
                resetSeq(n->a, out);
                return;
            case LInner::LOGICAL: resetSeq(n->b, out); return;
            default: out.push_back(n->first);  // Every inherits: first processor only
        }
    }
    void updateSeq(LInner* n, std::vector<int>& out) {
        switch (n->type) {
            case LInner::NEXT:
                updateSeq(n->a, out);
                updateSeq(n->b, out);
                return;
            case LInner::LOGICAL: updateSeq(n->b, out); return;
            default: out.push_back(n->first);
        }
    }
    void setQuerySelector(LInner* n) {
        switch (n->type) {
            case LInner::NEXT: setQuerySelector(n->b); return;
            case LInner::EVERY: setQuerySelector(n->a); return;
            case LInner::LOGICAL:
                setQuerySelector(n->b);
                setQuerySelector(n->a);
                return;
            default: procs[n->last].toSel = true;
        }
    }
    // setup(): receiver.setNext(first) + stateProcessorsForStream
    void setup(LInner* n, std::vector<std::pair<int, int>>& order) {
        switch (n->type) {
            case LInner::NEXT:
                setup(n->a, order);
                setup(n->b, order);
                return;
            case LInner::EVERY: setup(n->a, order); return;
            case LInner::LOGICAL:
                setup(n->b, order);
                setup(n->a, order);
                return;
            default: order.push_back(n->ssr[0]);
        }
    }

    // ---------------------------------------------------------- expressions
    int add_const(int64_t v, int type, int isnull) {
        for (int i = 0; i < T->n_const; i++)
            if (T->consts[i] == v && T->const_type[i] == type && T->const_null[i] == isnull) return i;
        if (T->n_const >= NF_MAX_CONST) {
            err = "too many constants";
            return -1;
        }
        T->consts[T->n_const] = v;
        T->const_type[T->n_const] = (uint8_t)type;
        T->const_null[T->n_const] = (uint8_t)isnull;
        return T->n_const++;
    }
    bool emit(uint8_t op, uint8_t a, uint8_t b, uint8_t c, int32_t x) {
        if (T->n_code >= NF_MAX_CODE) {
            err = "expression programs too long";
            return false;
        }
        shp_instr& in = T->code[T->n_code++];
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
        bool fl = (lt == SH_T_FLOAT && rt == SH_T_LONG) || (lt == SH_T_LONG && rt == SH_T_FLOAT);
        if ((op == SH_OP_EQ || op == SH_OP_NE) && fl) r = 3;
        return r == 0 ? DOM_I32 : r == 1 ? DOM_I64 : r == 2 ? DOM_F32 : DOM_F64;
    }
    int max_depth = 0;
    bool gen(int e, int depth) {
        if (e < 0 || e >= q->n_exprs) {
            err = "bad expression index";
            return false;
        }
        if (depth > NF_STACK - 2) {
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
                if (x.slot < 0 || x.slot >= q->n_slots) {
                    err = "variable slot out of range";
                    return false;
                }
                if (x.type == SH_T_OBJECT) {
                    err = "device engine: object attributes are not lowered";
                    return false;
                }
                return emit(OPC_VAR, (uint8_t)x.slot, (uint8_t)x.attr, (uint8_t)x.type, x.chain);
            case SH_OP_IS_NULL_STREAM: return emit(OPC_ISNULL_STREAM, (uint8_t)x.slot, 0, 0, x.chain);
            case SH_OP_NOT: return gen(x.lhs, depth + 1) && emit(OPC_NOT, 0, 0, 0, 0);
            case SH_OP_BOOL_VAR: return gen(x.lhs, depth + 1) && emit(OPC_BOOLV, 0, 0, 0, 0);
            case SH_OP_IS_NULL: return gen(x.lhs, depth + 1) && emit(OPC_ISNULL, 0, 0, 0, 0);
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
            case SH_OP_OUTPUT:
                if (x.attr < 0 || x.attr >= q->n_outputs) {
                    err = "having: output attribute out of range";
                    return false;
                }
                return emit(OPC_OUTPUT, 0, (uint8_t)x.attr, (uint8_t)x.type, 0);
        }
        err = "unsupported expression operator";
        return false;
    }

    // The rise-and-fall sequence (C3's shape):
    //   from every e1=S, e2=S[x.a op2 e1.b]+, e3=S[x.c op3 e2[last].d]
    // SEQUENCE keeps at most one partial per state (StreamPreStateProcessor /
    // CountPreStateProcessor.addState add to an empty new-and-every list only,
    // resetState clears every pending list per event), the e3 match sets slot 2
    // of the shared StateEvent before the count state sees it and drops it
    // (CountPreStateProcessor.java:60-68), and `every` re-arms e1 at every event.
    // Per key this is one partial (e1, last e2) — k_seq3 (sh_nfa.hip) runs it.
    void detect_seq3() {
        Q->s3 = 0;
        if (q->state_type != SH_SEQUENCE || q->within_ms >= 0 || q->n_slots != 3 || q->n_outputs < 1) return;
        // flatten the NEXT chain
        std::vector<int> chain;
        std::function<bool(int)> flat = [&](int e) -> bool {
            if (e < 0 || e >= q->n_elems) return false;
            const sh_state_elem& x = q->elems[e];
            if (x.kind == SH_E_NEXT) return flat(x.child0) && flat(x.child1);
            chain.push_back(e);
            return true;
        };
        if (!flat(q->root) || chain.size() != 3) return;
        const sh_state_elem& ev = q->elems[chain[0]];
        const sh_state_elem& cn = q->elems[chain[1]];
        const sh_state_elem& c3 = q->elems[chain[2]];
        if (ev.kind != SH_E_EVERY || cn.kind != SH_E_COUNT || c3.kind != SH_E_STREAM) return;
        if (ev.child0 < 0 || cn.child0 < 0) return;
        const sh_state_elem& a = q->elems[ev.child0];
        const sh_state_elem& b = q->elems[cn.child0];
        if (a.kind != SH_E_STREAM || b.kind != SH_E_STREAM || a.filter >= 0 || b.filter < 0 || c3.filter < 0) return;
        if (a.slot != 0 || b.slot != 1 || c3.slot != 2 || a.stream != b.stream || b.stream != c3.stream) return;
        if (cn.min_count != 1 || cn.max_count != SH_ANY) return;
        auto var = [&](int e, int slot, bool current_only, int* attr, int* type) {
            if (e < 0 || e >= q->n_exprs) return false;
            const sh_expr& x = q->exprs[e];
            if (x.op != SH_OP_VAR || x.slot != slot || x.type == SH_T_OBJECT) return false;
            if (current_only ? x.chain != SH_CHAIN_CURRENT : (x.chain != 0 && x.chain != SH_CHAIN_CURRENT)) return false;
            *attr = x.attr;
            *type = x.type;
            return true;
        };
        auto mirror = [](int op) {
            switch (op) {
                case SH_OP_GT: return (int)SH_OP_LT;
                case SH_OP_GE: return (int)SH_OP_LE;
                case SH_OP_LT: return (int)SH_OP_GT;
                case SH_OP_LE: return (int)SH_OP_GE;
                default: return op;
            }
        };
        // filter = CMP(x.attr of `self` slot, other slot's attr), either operand order
        auto cmpf = [&](int e, int self, int other, bool other_current, int* op, int* xa, int* xt, int* oa, int* ot) {
            if (e < 0 || e >= q->n_exprs) return false;
            const sh_expr& x = q->exprs[e];
            if (x.op < SH_OP_EQ || x.op > SH_OP_LE) return false;
            if (var(x.lhs, self, false, xa, xt) && var(x.rhs, other, other_current, oa, ot)) {
                *op = x.op;
                return true;
            }
            if (var(x.rhs, self, false, xa, xt) && var(x.lhs, other, other_current, oa, ot)) {
                *op = mirror(x.op);
                return true;
            }
            return false;
        };
        int op2, a2, t2, e1a, e1t, op3, a3, t3, la, lt;
        // the e2 event inside its own filter is the chain's current event
        if (!cmpf(b.filter, 1, 0, false, &op2, &a2, &t2, &e1a, &e1t)) return;
        if (q->exprs[q->exprs[b.filter].lhs].slot == 1 ? q->exprs[q->exprs[b.filter].lhs].chain != SH_CHAIN_CURRENT
                                                       : q->exprs[q->exprs[b.filter].rhs].chain != SH_CHAIN_CURRENT)
            return;
        if (!cmpf(c3.filter, 2, 1, true, &op3, &a3, &t3, &la, &lt)) return;
        if (q->n_outputs > NF_MAX_OUT) return;
        for (int o = 0; o < q->n_outputs; o++) {
            const sh_output_attr& oa = q->outputs[o];
            // sum / avg / count of a plain attribute: the engine writes the argument,
            // the post-pass over the ordered rows forms the running value (sh_agg.hip)
            if (oa.agg == SH_AGG_COUNT && oa.expr < 0) {
                Q->s3_out_slot[o] = 2;
                Q->s3_out_attr[o] = 0;
                Q->s3_out_type[o] = (int8_t)app->streams[c3.stream].attr_types[0];
                continue;
            }
            if (oa.agg != SH_AGG_NONE && oa.agg != SH_AGG_SUM && oa.agg != SH_AGG_AVG && oa.agg != SH_AGG_COUNT) return;
            if (oa.expr < 0) return;
            const sh_expr& x = q->exprs[oa.expr];
            int at, ty;
            if (x.op != SH_OP_VAR || x.slot < 0 || x.slot > 2) return;
            if (!var(oa.expr, x.slot, x.slot == 1, &at, &ty)) return;
            Q->s3_out_slot[o] = (int8_t)x.slot;
            Q->s3_out_attr[o] = (int8_t)at;
            Q->s3_out_type[o] = (int8_t)ty;
        }
        Q->s3_op2 = (int8_t)op2;
        Q->s3_dom2 = (int8_t)dom_for(op2, t2, e1t);
        Q->s3_a2 = (int8_t)a2;
        Q->s3_t2 = (int8_t)t2;
        Q->s3_e1a = (int8_t)e1a;
        Q->s3_e1t = (int8_t)e1t;
        Q->s3_op3 = (int8_t)op3;
        Q->s3_dom3 = (int8_t)dom_for(op3, t3, lt);
        Q->s3_a3 = (int8_t)a3;
        Q->s3_t3 = (int8_t)t3;
        Q->s3_la = (int8_t)la;
        Q->s3_lt = (int8_t)lt;
        Q->s3 = 1;
    }

    bool run() {
        memset(Q, 0, sizeof(*Q));
        Q->state_type = q->state_type;
        Q->within = q->within_ms;
        if (q->n_slots < 1 || q->n_slots > NF_MAX_PROC) {
            err = "device engine: 1..16 states per query";
            return false;
        }
        // receivers: count stream uses first (a pre-pass over the element list)
        std::map<int, int> suse;
        for (int i = 0; i < q->n_elems; i++)
            if (q->elems[i].kind == SH_E_STREAM || q->elems[i].kind == SH_E_ABSENT_STREAM) suse[q->elems[i].stream]++;
        std::vector<int> list;
        LInner* root = parse(q->root, -1, list, true);
        if (!root) return false;
        if ((int)procs.size() != q->n_slots || slotCounter != q->n_slots) {
            err = "state count mismatch";
            return false;
        }
        // proc id -> state id
        std::vector<int> sid(procs.size());
        for (size_t i = 0; i < procs.size(); i++) sid[i] = procs[i].stateId;
        auto S = [&](int p) { return p < 0 ? -1 : sid[p]; };
        procs[root->first].thisLast = root->last;
        setQuerySelector(root);
        if (q->within_ms >= 0)
            for (auto& P : procs)
                if (P.isStart) Q->start_ids[Q->n_start++] = (int8_t)P.stateId;
        std::vector<std::pair<int, int>> order;
        setup(root, order);
        for (auto& kv : suse) {
            nf_receiver& R = Q->recv[kv.first];
            R.present = 1;
            R.n_next = (int8_t)kv.second;
            R.multi = kv.second > 1;
            for (int i = 0; i < NF_MAX_PROC; i++) R.next_procs[i] = -1;
            for (int i = 0; i < kv.second; i++) R.event_seq[i] = (int8_t)(kv.second - 1 - i);
        }
        for (auto& sp : order) {
            nf_receiver& R = Q->recv[sp.first];
            const int p = sp.second;
            if (R.multi) {
                for (int i = 0; i < R.n_next; i++)
                    if (R.next_procs[i] < 0) {
                        R.next_procs[i] = (int8_t)S(p);
                        break;
                    }
                R.has_selector = procs[p].toSel;
            } else {
                R.next_procs[0] = (int8_t)S(p);
                R.has_selector = procs[procs[p].thisLast].toSel;
            }
            R.for_stream[R.n_for++] = (int8_t)S(p);
        }
        std::vector<int> seq;
        initSeq(root, seq);
        Q->n_init = (int)seq.size();
        for (size_t i = 0; i < seq.size(); i++) Q->init_seq[i] = (int8_t)S(seq[i]);
        seq.clear();
        resetSeq(root, seq);
        Q->n_reset = (int)seq.size();
        for (size_t i = 0; i < seq.size(); i++) Q->reset_seq[i] = (int8_t)S(seq[i]);
        seq.clear();
        updateSeq(root, seq);
        Q->n_update = (int)seq.size();
        for (size_t i = 0; i < seq.size(); i++) Q->update_seq[i] = (int8_t)S(seq[i]);
        Q->n_startup = (int)startup.size();
        for (size_t i = 0; i < startup.size(); i++) Q->startup[i] = (int8_t)S(startup[i]);
        Q->n_sched = (int)schedOrder.size();
        for (size_t i = 0; i < schedOrder.size(); i++) Q->sched_seq[i] = (int8_t)S(schedOrder[i]);
        Q->n_proc = (int)procs.size();
        for (auto& P : procs) {
            nf_proc& D = Q->proc[P.stateId];
            D.kind = (int8_t)P.kind;
            D.is_start = P.isStart;
            D.stream = (int8_t)P.stream;
            D.within_every = (int8_t)S(P.withinEvery);
            D.this_last = (int8_t)S(P.thisLast);
            D.partner = (int8_t)S(P.partner);
            D.logical_type = (int8_t)P.ltype;
            D.next_pre = (int8_t)S(P.nextPre);
            D.next_every_pre = (int8_t)S(P.nextEveryPre);
            D.callback_pre = (int8_t)S(P.callbackPre);
            D.to_selector = P.toSel;
            D.min_count = P.minc;
            D.max_count = P.maxc;
            D.waiting = P.waiting;
            D.absent_logical = P.alog;
            Q->slot_stream[P.stateId] = (int8_t)P.stream;
            if (P.filter >= 0) {
                D.filter_pc = T->n_code;
                if (!gen(P.filter, 0)) return false;
                D.filter_len = T->n_code - D.filter_pc;
            } else {
                D.filter_pc = -1;
                D.filter_len = 0;
            }
        }
        if (q->n_outputs > NF_MAX_OUT) {
            err = "device engine: at most 16 output attributes";
            return false;
        }
        // k_seq3 emits without a selector pass
        if (q->having < 0 && q->n_order == 0 && q->limit < 0 && q->offset < 0 && q->rate_kind == SH_RATE_NONE)
            detect_seq3();
        Q->n_out = q->n_outputs;
        for (int o = 0; o < q->n_outputs; o++) {
            const sh_output_attr& oa = q->outputs[o];
            Q->out_agg[o] = oa.agg;
            Q->out_type[o] = oa.type;
            if (oa.agg != SH_AGG_NONE) Q->contains_agg = 1;
            if (oa.expr >= 0 && oa.expr < q->n_exprs && oa.agg == SH_AGG_NONE && q->exprs[oa.expr].op == SH_OP_MULTI_VAR) {
                // a List of the chain's values (MultiValueVariableFunctionExecutor)
                const sh_expr& x = q->exprs[oa.expr];
                if (x.slot < 0 || x.slot >= q->n_slots || x.attr < 0 || x.attr >= NF_MAX_ATTRS) {
                    err = "device engine: bad multi-value variable";
                    return false;
                }
                Q->out_pc[o] = NF_PC_LIST;
                Q->out_len[o] = 0;
                Q->out_mv_slot[o] = x.slot;
                Q->out_mv_chain[o] = x.chain;
                Q->out_mv_attr[o] = x.attr;
                Q->out_mv_type[o] = x.ltype;
                continue;
            }
            if (oa.expr >= 0) {
                Q->out_pc[o] = T->n_code;
                if (!gen(oa.expr, 0)) return false;
                Q->out_len[o] = T->n_code - Q->out_pc[o];
            } else {
                Q->out_pc[o] = -1;
                Q->out_len[o] = 0;
            }
        }
        // GroupByKeyGenerator's executors (the group key of the aggregators' state)
        if (q->n_group < 0 || q->n_group > SH_MAX_GROUP) {
            err = "device engine: at most 4 group-by attributes";
            return false;
        }
        Q->n_group = q->n_group;
        for (int i = 0; i < q->n_group; i++) {
            const int e = q->group_expr[i];
            if (e < 0 || e >= q->n_exprs || q->exprs[e].type == SH_T_OBJECT) {
                err = "device engine: bad group-by attribute";
                return false;
            }
            Q->group_pc[i] = T->n_code;
            if (!gen(e, 0)) return false;
            Q->group_len[i] = T->n_code - Q->group_pc[i];
        }
        Q->having_pc = -1;
        Q->having_len = 0;
        if (q->having >= 0) {
            Q->having_pc = T->n_code;
            if (!gen(q->having, 0)) return false;
            Q->having_len = T->n_code - Q->having_pc;
        }
        if (q->n_order < 0 || q->n_order > SH_MAX_ORDER) {
            err = "order by: 0..4 attributes";
            return false;
        }
        Q->n_order = q->n_order;
        Q->order_desc = q->order_desc;
        for (int i = 0; i < q->n_order; i++) {
            const int e = q->order_expr[i];
            if (e < 0 || e >= q->n_exprs) {
                err = "order by: expression out of range";
                return false;
            }
            const int t = q->exprs[e].type;
            if (t == SH_T_STRING || t == SH_T_OBJECT) {
                err = "order by: string / object attributes need the host's values";
                return false;
            }
            Q->order_pc[i] = T->n_code;
            if (!gen(q->order_expr[i], 0)) return false;
            Q->order_len[i] = T->n_code - Q->order_pc[i];
        }
        Q->limit = q->limit;
        Q->offset = q->offset;
        Q->rate_kind = q->rate_kind;
        Q->rate_value = q->rate_value;
        if (q->rate_kind != SH_RATE_NONE &&
            ((q->rate_kind != SH_RATE_FIRST_EVENTS && q->rate_kind != SH_RATE_LAST_EVENTS &&
              q->rate_kind != SH_RATE_ALL_EVENTS && q->rate_kind != SH_RATE_FIRST_TIME) ||
             q->rate_value < (q->rate_kind == SH_RATE_FIRST_TIME ? 0 : 1))) {
            err = "output rate limiting: `output [first|last|all] every N events` (N >= 1) or `output first every T`";
            return false;
        }
        if (q->rate_kind == SH_RATE_FIRST_TIME && (!app->playback || q->n_group > 0)) {
            // outside playback the limiter reads System.currentTimeMillis(); with group by
            // OutputParser picks FirstGroupByPerTimeOutputRateLimiter
            err = "output first every T: @app:playback apps without group by only";
            return false;
        }
        if (Q->contains_agg && (q->offset > 0 || q->limit == 0)) {
            // processInBatchNoGroupBy would hand an empty chunk to the rate limiter
            err = "aggregating selector with offset > 0 or limit 0 never emits";
            return false;
        }
        return true;
    }
};

}  // namespace

int nf_lower(const sh_app_desc* app, nf_table* T, std::string* err) {
    memset(T, 0, sizeof(*T));
    if (app->n_queries < 1 || app->n_queries > NF_MAX_QUERIES) {
        *err = "device engine: 1..16 queries per app";
        return -1;
    }
    if (app->n_streams < 1 || app->n_streams > NF_MAX_STREAMS) {
        *err = "device engine: 1..8 streams per app";
        return -1;
    }
    T->n_queries = app->n_queries;
    T->n_streams = app->n_streams;
    T->playback = app->playback;
    for (int s = 0; s < app->n_streams; s++) {
        if (app->streams[s].n_attrs > NF_MAX_ATTRS) {
            *err = "device engine: at most 32 attributes per stream";
            return -1;
        }
        T->stream_nattr[s] = app->streams[s].n_attrs;
        for (int a = 0; a < app->streams[s].n_attrs; a++) T->attr_type[s][a] = (int8_t)app->streams[s].attr_types[a];
    }
    // every query in partition 0, or every query unpartitioned
    int np = 0, nu = 0;
    for (int i = 0; i < app->n_queries; i++) {
        if (app->queries[i].partition == 0)
            np++;
        else if (app->queries[i].partition < 0)
            nu++;
    }
    if (np + nu != app->n_queries || (np && nu)) {
        *err = "device engine: all queries in one partition, or none partitioned";
        return -1;
    }
    T->partitioned = np > 0;
    // attributes read by any expression (sh_run_device carries only these through the segment)
    for (int i = 0; i < app->n_queries; i++) {
        const sh_query_desc& qd = app->queries[i];
        std::vector<int> slot_stream(qd.n_slots > 0 ? qd.n_slots : 1, -1);
        for (int e = 0; e < qd.n_elems; e++)
            if ((qd.elems[e].kind == SH_E_STREAM || qd.elems[e].kind == SH_E_ABSENT_STREAM) && qd.elems[e].slot >= 0 &&
                qd.elems[e].slot < qd.n_slots)
                slot_stream[qd.elems[e].slot] = qd.elems[e].stream;
        for (int x = 0; x < qd.n_exprs; x++) {
            const sh_expr& ex = qd.exprs[x];
            if ((ex.op != SH_OP_VAR && ex.op != SH_OP_MULTI_VAR) || ex.slot < 0 || ex.slot >= qd.n_slots || ex.attr < 0 ||
                ex.attr >= 32)
                continue;
            const int st = slot_stream[ex.slot];
            if (st >= 0 && st < NF_MAX_STREAMS) T->attr_used[st] |= 1u << ex.attr;
        }
    }
    for (int i = 0; i < app->n_queries; i++) {
        QueryLowering L;
        L.app = app;
        L.q = &app->queries[i];
        L.T = T;
        L.Q = &T->q[i];
        if (!L.run()) {
            *err = "query " + std::to_string(i) + ": " + L.err;
            return -1;
        }
        if (T->partitioned) {
            for (int p = 0; p < T->q[i].n_proc; p++) {
                const int s = T->q[i].proc[p].stream;
                if (!app->partition_streams[s]) {
                    *err = "device engine: every stream of a partitioned query must be keyed";
                    return -1;
                }
            }
        }
        for (int p = 0; p < T->q[i].n_proc; p++) {
            const nf_proc& P = T->q[i].proc[p];
            if (nf_has_sched(P)) T->has_absent = 1;
            // CountPreStateProcessor.addState with minCount 0 raises the final count
            // post's isEventReturned outside that state's own processing; the flag is
            // consumed by whichever partition key processes the state next, so the
            // result depends on the global cross-key processing order
            if (T->partitioned && P.kind == NF_K_COUNT && P.min_count == 0 && P.to_selector) {
                *err = "query " + std::to_string(i) +
                       ": device engine: a final count state with min 0 inside a partition (cross-key "
                       "isEventReturned hand-off) stays on the reference runtime";
                return -1;
            }
        }
    }
    nf_set_caps(T, 16, 32, 64, 32, 8);
    return 0;
}

void nf_set_caps(nf_table* T, int list_cap, int se_cap, int node_cap, int hold_cap, int sched_cap, int group_cap) {
    int64_t w = 1;  // key header word: bit 0 = partition seen (initPartition done)
    for (int i = 0; i < T->n_queries; i++) {
        nf_query& Q = T->q[i];
        nf_set_layout(Q, Q.n_proc, list_cap, se_cap, node_cap, hold_cap, sched_cap, group_cap);
        Q.q_off = w;
        w += Q.lay.words;
    }
    T->key_words = w;
}
