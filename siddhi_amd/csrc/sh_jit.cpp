// sh_jit.cpp — run-time specialisation of the window engine (sh_window.hip)
// for one compiled query, through hipRTC.
//
// The ahead-of-time window kernels evaluate a query's filters and select list by
// walking the lowered program (shp_term conjunctions or postfix bytecode) on
// every candidate pair; on this path that interpretation — uniform scalar loads
// of the program and branches on operator/type — dominates the kernel. Here the
// same program is printed as straight-line C++ that calls the very same helpers
// (sh_vm.h: vm_cmp, vm_arith and the VmVal conversions, embedded verbatim from
// the device headers), so operator, domain and type arguments are literals and
// fold away, and the result is compiled for gfx950 with the flags of the
// ahead-of-time build (-ffp-contract=off, no denormal flush, correctly rounded
// f32 division: Java arithmetic, bit for bit).
//
// The specialised kernels also stage their tile (and a halo) of the key segment
// in LDS — keys, timestamps and exactly the columns the consuming filter reads —
// so the forward scan of a partial (candidate consumers) and the backward rank
// scan of a match run at LDS latency instead of one dependent global round trip
// per step. Tiles are assigned XCD-major: hardware dispatches workgroup i to XCD
// i % 8, and the mapping below hands each XCD a contiguous run of tiles so a
// tile's halo is the L2-resident tile of the previous workgroup on that XCD.
//
// Semantics are those of k_window / k_window_place (sh_window.hip), which stay
// as the fallback when hipRTC is unavailable or SH_DISABLE_JIT is set.
#include <hip/hip_runtime.h>
#include <hip/hiprtc.h>

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <map>
#include <mutex>
#include <set>
#include <string>
#include <vector>

#include "../../include/sh_query.h"
#include "sh_device.h"
#include "sh_jit.h"
#include "sh_jit_src.inc"

namespace {

int type_width(int t) { return t == SH_T_LONG || t == SH_T_DOUBLE ? 8 : (t == SH_T_BOOL ? 1 : 4); }

// events per workgroup (one lane each) and staged events beyond the tile
// (forward for match, backward for place / the consumer walk); SH_JIT_TILE /
// SH_JIT_HALO override them (tile 64..1024, powers of two; halo 0..1024)
int env_int(const char* name, int def, int lo, int hi) {
    const char* e = getenv(name);
    if (!e) return def;
    const int v = atoi(e);
    return v < lo || v > hi ? def : v;
}
const int kTile = [] {
    const int t = env_int("SH_JIT_TILE", 256, 64, 1024);
    return (t & (t - 1)) ? 256 : t;
}();
const int kHalo = env_int("SH_JIT_HALO", 256, 0, 1024);
// predecessors the bucketed matcher's walk loads and evaluates per block
// (measured on C2: 4 -> 2.04 ms, 8 -> 2.13 ms, 12 -> 2.42 ms per matcher pass)
const int kWalkBlock = env_int("SH_BK_WALK", 4, 2, 16);
// the count walk hands consumers out per lane (SH_BK_DYN=0: every lane of a wave
// walks its consumer to the wave's longest walk)
const int kWalkDyn = env_int("SH_BK_DYN", 1, 0, 1);
// the bucketed matcher's launch bound: minimum workgroups per CU the register
// allocation is sized for (the default 3-KB pass's LDS holds three 512-thread
// workgroups per CU)
const int kMatchMinBlocks = env_int("SH_BK_MINB", 6, 1, 8);
// a matcher pass's LDS span and consumer limit (events; multiples of its 512
// threads, at most SHB_SPAN / SHB_CH): smaller passes take less LDS, so more
// workgroups share a CU, at the price of more halo events per consumer. 3,072 /
// 2,048 measured 4.44 vs 4.63 ms for 5,120 / 4,096 on C2 (profiles/r4_c2_span_ab.txt);
// 2,560 / 2,048 (the pass's 1,792 consumers and ~400 halo events fit) 1.98 vs 2.09 ms
// for the matcher (profiles/r6_c2_span_ab.txt)
const int kSpan = [] {
    const int v = env_int("SH_BK_SPAN", 2560, 1024, SHB_SPAN);
    return v % 512 ? 2560 : v;
}();
const int kChunk = [] {
    const int v = env_int("SH_BK_CH", 2048, 512, SHB_CH);
    return (v % 512 || v > kSpan) ? (kSpan < 2048 ? kSpan : 2048) : v;
}();

int type_width_of(int t) { return t == SH_T_LONG || t == SH_T_DOUBLE ? 8 : (t == SH_T_BOOL ? 1 : 4); }

const char* col_ctype(int t) {
    switch (t) {
        case SH_T_LONG:
        case SH_T_DOUBLE: return "int64_t";
        case SH_T_FLOAT: return "uint32_t";
        case SH_T_BOOL: return "uint8_t";
        default: return "int32_t";
    }
}

// raw VmVal bits of a column element, as load_attr (sh_vm.h) forms them
std::string raw_of(int t, const std::string& v) {
    switch (t) {
        case SH_T_LONG:
        case SH_T_DOUBLE: return "(int64_t)(" + v + ")";
        case SH_T_FLOAT: return "(int64_t)(uint32_t)(" + v + ")";
        case SH_T_BOOL: return "((" + v + ") ? 1ll : 0ll)";
        default: return "(int64_t)(int32_t)(" + v + ")";
    }
}

std::string lit64(int64_t v) {
    char b[64];
    snprintf(b, sizeof(b), "(int64_t)%lldll", (long long)v);
    if (v == INT64_MIN) snprintf(b, sizeof(b), "(int64_t)(-9223372036854775807ll - 1)");
    return b;
}

struct Gen {
    const shp_program& P;
    std::set<int> need[2];  // attributes read per slot (0: partial's event, 1: candidate)
    int tmp = 0;
    explicit Gen(const shp_program& p) : P(p) {}

    std::string var(int slot, int attr) {
        need[slot].insert(attr);
        return "x" + std::to_string(slot) + "_" + std::to_string(attr);
    }

    std::string vmval(const std::string& name, int type, const std::string& bits, const std::string& null) {
        return "VmVal " + name + "; " + name + ".t = " + std::to_string(type) + "; " + name + ".null = " + null +
               "; " + name + ".b = " + bits + ";\n";
    }

    // conjunction of register terms (terms_pass2); `fail` leaves the block
    std::string terms(int k, bool slot1, const std::string& ok) {
        std::string s = "do {\n";
        for (int t = 0; t < P.filter_nterms[k]; t++) {
            const shp_term& T = P.terms[k][t];
            if ((T.lslot && !slot1) || (T.rkind != 1 && T.rslot && !slot1)) {
                s += ok + " = false; break;\n";
                break;
            }
            const std::string l = "l" + std::to_string(tmp), r = "r" + std::to_string(tmp);
            tmp++;
            s += "{\n" + vmval(l, T.ltype, var(T.lslot, T.lattr), "0");
            if (T.rkind == 1) {
                s += vmval(r, T.ctype, lit64(T.c), "0");
            } else {
                s += vmval(r, T.rtype, var(T.rslot, T.rattr), "0");
                if (T.rkind == 2) {
                    const std::string c = "c" + std::to_string(tmp++);
                    s += vmval(c, T.ctype, lit64(T.c), "0");
                    s += r + " = vm_arith(" + std::to_string(T.aop) + ", " + std::to_string(T.atype) + ", " + r +
                         ", " + c + ");\n";
                    s += "if (" + r + ".null) { " + ok + " = false; break; }\n";
                }
            }
            s += "if (!vm_cmp(" + std::to_string(T.op) + ", " + std::to_string(T.dom) + ", " + l + ", " + r + ")) { " +
                 ok + " = false; break; }\n}\n";
        }
        return s + "} while (0);\n";
    }

    // postfix bytecode (vm_eval) as SSA statements; returns the result's name
    std::string bytecode(int pc, int len, bool slot1, std::string& s) {
        std::vector<std::string> st;
        for (int k = 0; k < len; k++) {
            const shp_instr& in = P.code[pc + k];
            const std::string v = "v" + std::to_string(tmp++);
            auto pop = [&]() {
                std::string x = st.back();
                st.pop_back();
                return x;
            };
            switch (in.op) {
                case OPC_CONST:
                    s += vmval(v, P.const_type[in.x], lit64(P.consts[in.x]), P.const_null[in.x] ? "1" : "0");
                    break;
                case OPC_VAR: {
                    const bool valid = (in.a == 0 || slot1) && (in.x == 0 || in.x == SH_CHAIN_CURRENT);
                    s += valid ? vmval(v, in.c, var(in.a, in.b), "0") : vmval(v, in.c, "0", "1");
                    break;
                }
                case OPC_AND: {
                    std::string r = pop(), l = pop();
                    s += vmval(v, SH_T_BOOL,
                               "(!" + l + ".null && " + l + ".b && !" + r + ".null && " + r + ".b) ? 1 : 0", "0");
                    break;
                }
                case OPC_OR: {
                    std::string r = pop(), l = pop();
                    s += vmval(v, SH_T_BOOL,
                               "((!" + l + ".null && " + l + ".b) || (!" + r + ".null && " + r + ".b)) ? 1 : 0", "0");
                    break;
                }
                case OPC_NOT: {
                    std::string l = pop();
                    s += vmval(v, SH_T_BOOL, "(!" + l + ".null && " + l + ".b) ? 0 : 1", "0");
                    break;
                }
                case OPC_BOOLV: {
                    std::string l = pop();
                    s += vmval(v, SH_T_BOOL, "(!" + l + ".null && " + l + ".b) ? 1 : 0", "0");
                    break;
                }
                case OPC_ISNULL: {
                    std::string l = pop();
                    s += vmval(v, SH_T_BOOL, l + ".null ? 1 : 0", "0");
                    break;
                }
                case OPC_ISNULL_STREAM: {
                    const bool valid = (in.a == 0 || slot1) && (in.x == 0 || in.x == SH_CHAIN_CURRENT);
                    s += vmval(v, SH_T_BOOL, valid ? "0" : "1", "0");
                    break;
                }
                case OPC_CMP: {
                    std::string r = pop(), l = pop();
                    s += vmval(v, SH_T_BOOL,
                               "(!" + l + ".null && !" + r + ".null && vm_cmp(" + std::to_string(in.a) + ", " +
                                   std::to_string(in.b) + ", " + l + ", " + r + ")) ? 1 : 0",
                               "0");
                    break;
                }
                case OPC_ARITH: {
                    std::string r = pop(), l = pop();
                    s += "VmVal " + v + " = vm_arith(" + std::to_string(in.a) + ", " + std::to_string(in.b) + ", " + l +
                         ", " + r + ");\n";
                    break;
                }
                case OPC_SELECT: {
                    std::string e = pop(), t = pop(), c = pop();
                    s += "VmVal " + v + " = (!" + c + ".null && " + c + ".b) ? " + t + " : " + e + ";\n";
                    break;
                }
                case OPC_CAST: {
                    std::string l = pop();
                    s += "VmVal " + v + " = " + l + "; " + v + ".t = " + std::to_string(in.b) + ";\n";
                    break;
                }
                default:
                    return "";
            }
            st.push_back(v);
        }
        return st.size() == 1 ? st.back() : "";
    }

    // filter of state k into `bool ok` (declared by the caller, preset true)
    bool filter(int k, bool slot1, const std::string& ok, std::string& s) {
        if (P.filter_fast[k]) {
            s += terms(k, slot1, ok);
            return true;
        }
        if (P.filter_pc[k] < 0) return true;
        std::string body;
        const std::string r = bytecode(P.filter_pc[k], P.filter_len[k], slot1, body);
        if (r.empty()) return false;
        s += "{\n" + body + ok + " = !" + r + ".null && " + r + ".b != 0;\n}\n";
        return true;
    }
};

// loads of the attributes a piece reads, from LDS (staged) or global memory
std::string load_attrs(const shp_program& P, const std::set<int>& attrs, int slot, const std::string& row,
                       const std::set<int>* staged, const std::string& lds_row) {
    std::string s;
    for (int a : attrs) {
        const int t = P.attr_type[0][a];
        const std::string x = "x" + std::to_string(slot) + "_" + std::to_string(a);
        if (staged && staged->count(a))
            s += x + " = " + raw_of(t, "s_c" + std::to_string(a) + "[" + lds_row + "]") + ";\n";
        else
            s += x + " = " + raw_of(t, "c" + std::to_string(a) + "[" + row + "]") + ";\n";
    }
    return s;
}

std::string decl_attrs(const std::set<int>& attrs, int slot) {
    std::string s;
    for (int a : attrs) s += "int64_t x" + std::to_string(slot) + "_" + std::to_string(a) + " = 0;\n";
    return s;
}

std::string col_ptrs(const shp_program& P, const std::set<int>& attrs) {
    std::string s;
    for (int a : attrs) {
        const std::string ct = col_ctype(P.attr_type[0][a]);
        s += "const " + ct + "* __restrict__ c" + std::to_string(a) + " = (const " + ct + "*)C->col[0][" +
             std::to_string(a) + "];\n";
    }
    return s;
}

// ---- consumer-side ("extremum") form of the window reduction
//
// A partial opened at i is consumed at the first later event j of its key with
// f2(i, j), provided ts_j - ts_i <= W (timestamps are non-decreasing per key, so
// no event between them expired it). When f2 is a conjunction of terms on e2
// only, terms on e1 only and at most one ordering comparison X(e2) op Y(e1),
//   i is consumed at j  <=>  f1(i) && f2(i, j) && !(ext_{q in (i, j), q2(q)} X(q) op Y(i))
// with ext = max for > / >= and min for < / <= over the events q strictly
// between i and j that pass the e2-only terms q2 (NaN never compares true and is
// left out). One lane per consumer j walks back over its key's events inside
// the window, keeping ext as it goes; the walk yields the partials j consumes,
// newest first, so counting and ordered placement need no per-partial state.
struct ExtForm {
    std::vector<shp_term> f1, ionly, qonly;
    bool cross = false;
    shp_term ct{};
    bool q_left = true;  // the e2 side is the term's left operand
    int op = 0;          // X(e2) op Y(e1) after mirroring
    int dom = 0;
};

int mirror_op(int op) {
    switch (op) {
        case SH_OP_GT: return SH_OP_LT;
        case SH_OP_GE: return SH_OP_LE;
        case SH_OP_LT: return SH_OP_GT;
        case SH_OP_LE: return SH_OP_GE;
        default: return op;
    }
}

bool ext_form(const shp_program& P, ExtForm& F) {
    if (!P.window_ok) return false;
    for (int k = 0; k < 2; k++)
        if (!P.filter_fast[k] && P.filter_pc[k] >= 0) return false;
    if (P.filter_fast[0])
        for (int t = 0; t < P.filter_nterms[0]; t++) {
            const shp_term& T = P.terms[0][t];
            if (T.lslot || (T.rkind != 1 && T.rslot)) return false;
            F.f1.push_back(T);
        }
    if (P.filter_fast[1])
        for (int t = 0; t < P.filter_nterms[1]; t++) {
            const shp_term& T = P.terms[1][t];
            const bool rconst = T.rkind == 1;
            if (rconst || T.lslot == T.rslot) {
                (T.lslot ? F.qonly : F.ionly).push_back(T);
                continue;
            }
            if (F.cross) return false;  // one ordering comparison across the slots at most
            if (T.op != SH_OP_GT && T.op != SH_OP_GE && T.op != SH_OP_LT && T.op != SH_OP_LE) return false;
            if (T.dom != DOM_I32 && T.dom != DOM_I64 && T.dom != DOM_F32 && T.dom != DOM_F64) return false;
            F.cross = true;
            F.ct = T;
            F.q_left = T.lslot == 1;
            F.op = F.q_left ? T.op : mirror_op(T.op);
            F.dom = T.dom;
        }
    return true;
}

const char* dom_ctype(int dom) {
    switch (dom) {
        case DOM_I32: return "int32_t";
        case DOM_I64: return "int64_t";
        case DOM_F32: return "float";
        default: return "double";
    }
}

std::string dom_conv(int dom, const std::string& v) {
    switch (dom) {
        case DOM_I32: return "(int32_t)" + v + ".b";
        case DOM_I64: return "to_i64(" + v + ")";
        case DOM_F32: return "to_f32(" + v + ")";
        default: return "to_f64(" + v + ")";
    }
}

// statements defining VmVal `name` for one operand of T; slot s reads
// attributes from variables pfx[s]<attr> (recorded in need[s])
struct SideGen {
    std::string pfx[2];
    std::set<int>* need[2];
    int tmp = 0;
    std::string attr(int slot, int a) {
        need[slot]->insert(a);
        return pfx[slot] + std::to_string(a);
    }
    std::string vm(const std::string& name, int type, const std::string& bits) {
        return "VmVal " + name + "; " + name + ".t = " + std::to_string(type) + "; " + name + ".null = 0; " + name +
               ".b = " + bits + ";\n";
    }
    std::string left(const shp_term& T, const std::string& name) { return vm(name, T.ltype, attr(T.lslot, T.lattr)); }
    std::string right(const shp_term& T, const std::string& name) {
        if (T.rkind == 1) return vm(name, T.ctype, lit64(T.c));
        std::string s = vm(name, T.rtype, attr(T.rslot, T.rattr));
        if (T.rkind == 2) {
            const std::string c = name + "c";
            s += vm(c, T.ctype, lit64(T.c));
            s += name + " = vm_arith(" + std::to_string(T.aop) + ", " + std::to_string(T.atype) + ", " + name + ", " +
                 c + ");\n";
        }
        return s;
    }
    // conjunction of terms: clears `ok` when one fails
    std::string terms(const std::vector<shp_term>& ts, const std::string& ok) {
        std::string s;
        for (const shp_term& T : ts) {
            const std::string l = "tl" + std::to_string(tmp), r = "tr" + std::to_string(tmp);
            tmp++;
            s += "if (" + ok + ") {\n" + left(T, l) + right(T, r) + "if (" + r + ".null || !vm_cmp(" +
                 std::to_string(T.op) + ", " + std::to_string(T.dom) + ", " + l + ", " + r + ")) " + ok +
                 " = false;\n}\n";
        }
        return s;
    }
    // the e2 side X and the e1 side Y of the cross term, in the compare domain
    std::string xval(const ExtForm& F, const std::string& out) {
        const std::string v = "xv" + std::to_string(tmp++);
        std::string s = F.q_left ? left(F.ct, v) : right(F.ct, v);
        return s + "const " + dom_ctype(F.dom) + " " + out + " = " + dom_conv(F.dom, v) + ";\n";
    }
    std::string yval(const ExtForm& F, const std::string& out) {
        const std::string v = "yv" + std::to_string(tmp++);
        std::string s = F.q_left ? right(F.ct, v) : left(F.ct, v);
        return s + "const " + dom_ctype(F.dom) + " " + out + " = " + dom_conv(F.dom, v) + ";\n";
    }
};

std::string xcd_tile() {
    return "const uint32_t tile = (blockIdx.x & 7u) * tiles_per_xcd + (blockIdx.x >> 3);\n"
           "if (tile >= ntiles) return;\n"
           "const int64_t b0 = (int64_t)tile * SHJ_TILE;\n";
}

std::string load_set(const shp_program& P, const std::set<int>& attrs, const std::string& pfx, const std::string& row,
                     const std::set<int>* staged, const std::string& lds_row) {
    std::string s;
    for (int a : attrs) {
        const int t = P.attr_type[0][a];
        const std::string x = pfx + std::to_string(a);
        if (staged && staged->count(a))
            s += x + " = " + raw_of(t, "s_c" + std::to_string(a) + "[" + lds_row + "]") + ";\n";
        else
            s += x + " = " + raw_of(t, "c" + std::to_string(a) + "[" + row + "]") + ";\n";
    }
    return s;
}

// shj_count / shj_emit: the consumer-side walk (ExtForm) over a tile of the key
// segment staged in LDS with a backward halo. `outs` writes the select list of
// the partial in x0_* and the consumer in x1_* to row `dst`.
std::string gen_ext(const shp_program& P, const ExtForm& F, const std::string& outs, const std::set<int>& out0,
                    const std::set<int>& out1) {
    std::set<int> need_r, need_q;
    SideGen gq, gi;  // gq: e1 = walked event (x0_), e2 = consumer (x1_); gi: both = walked event
    gq.pfx[0] = "x0_";
    gq.pfx[1] = "x1_";
    gq.need[0] = &need_r;
    gq.need[1] = &need_q;
    gi.pfx[0] = gi.pfx[1] = "x0_";
    gi.need[0] = gi.need[1] = &need_r;
    gi.tmp = 1000;
    const std::string DT = F.cross ? dom_ctype(F.dom) : "int32_t";
    // consumer: e2-only terms and X(consumer)
    std::string qhead = "bool qok = true;\n" + gq.terms(F.qonly, "qok");
    if (F.cross) qhead += "if (qok) {\n" + gq.xval(F, "xq_") + "xq = xq_;\n}\n";
    // walked event as a pending partial
    std::string cand = "bool ok = true;\n" + gq.terms(F.f1, "ok") + gq.terms(F.ionly, "ok");
    if (F.cross)
        cand += "if (ok) {\n" + gq.yval(F, "y") + "ok = cmp_op<" + DT + ">(" + std::to_string(F.op) +
                ", xq, y) && !(hasM && cmp_op<" + DT + ">(" + std::to_string(F.op) + ", M, y));\n}\n";
    else
        cand += "ok = ok && !hasM;\n";
    // walked event as an event between the partial and the consumer
    std::string mid = "bool mk = true;\n" + gi.terms(F.qonly, "mk");
    // once ext has reached X(consumer) no older partial can be consumed (for >:
    // y < X(j) and y >= ext are then disjoint; likewise >=, <, <=): stop there
    std::string stop;
    if (F.cross) {
        const bool mx = F.op == SH_OP_GT || F.op == SH_OP_GE;
        mid += "if (mk) {\n" + gi.xval(F, "xr") + "if (xr == xr && (!hasM || xr " + (mx ? ">" : "<") +
               " M)) M = xr;\nif (xr == xr) hasM = true;\n}\n";
        stop = std::string("    if (xq != xq || (hasM && M ") + (mx ? ">=" : "<=") + " xq)) break;\n";
    } else {
        mid += "if (mk) hasM = true;\n";
        stop = "    if (hasM) break;\n";
    }
    std::set<int> staged = need_r;
    staged.insert(need_q.begin(), need_q.end());
    std::set<int> all = staged;
    all.insert(out0.begin(), out0.end());
    all.insert(out1.begin(), out1.end());
    std::set<int> dec0 = need_r, dec1 = need_q;
    dec0.insert(out0.begin(), out0.end());
    dec1.insert(out1.begin(), out1.end());
    std::set<int> extra0;  // select-list attributes of the partial not read by the walk
    for (int a : out0)
        if (!need_r.count(a)) extra0.insert(a);

    auto head = [&](const std::string& name, const std::string& params) {
        std::string s = "\nextern \"C\" __global__ void __launch_bounds__(SHJ_TILE)\n" + name + "(" + params +
                        ") {\nconst TileDir D = tile_dir(TL);\n__shared__ int64_t s_ts[SHJ_SPAN];\n"
                        "__shared__ uint32_t s_key[SHJ_SPAN];\n";
        for (int a : staged)
            s += "__shared__ " + std::string(col_ctype(P.attr_type[0][a])) + " s_c" + std::to_string(a) +
                 "[SHJ_SPAN];\n";
        s += xcd_tile() + col_ptrs(P, all);
        s += "const int64_t lo = b0 > SHJ_HALO ? b0 - SHJ_HALO : 0;\n"
             "const int64_t hi = (n < b0 + SHJ_TILE) ? n : b0 + SHJ_TILE;\n"
             "for (int i = threadIdx.x; i < SHJ_SPAN; i += SHJ_TILE) {\n"
             "    const int64_t gi = lo + i;\n"
             "    if (gi < hi) {\n        s_ts[i] = sts[gi];\n        s_key[i] = skeys[gi];\n";
        for (int a : staged) s += "        s_c" + std::to_string(a) + "[i] = c" + std::to_string(a) + "[gi];\n";
        s += "    }\n}\n__syncthreads();\nconst int64_t p = b0 + threadIdx.x;\nif (p >= n) return;\n"
             "const uint32_t key = s_key[p - lo];\nconst uint32_t j = perm ? perm[p] : (uint32_t)p;\n";
        return s;
    };
    auto walk = [&](bool count, const std::string& on_consumed) {
        std::string s = "const int64_t tq = s_ts[p - lo];\n" + decl_attrs(dec0, 0) + decl_attrs(dec1, 1) +
                        load_set(P, dec1, "x1_", "p", &staged, "p - lo") + DT + " xq = 0;\n" + qhead +
                        "bool hasM = false;\n" + DT + " M = 0;\n";
        s += R"(uint32_t ta = D.on() ? D.tile(p) : 0u;
int64_t rbeg = D.on() ? (int64_t)D.ds[D.at(ta, key)] : 0;
bool first = true;
for (int64_t r = p - 1;; r--) {
    if (r < rbeg && !(D.on() && D.prev(ta, key, r, rbeg))) break;
    const bool in_lds = r >= lo;
    const uint32_t kr = in_lds ? s_key[r - lo] : skeys[r];
    if (kr != key) break;
    const int64_t tr = in_lds ? s_ts[r - lo] : sts[r];
)";
        if (count) s += "    if (first && tq < tr) atomicExch(flag, 1);\n";
        s += "    first = false;\n    if (tq - tr > SHJ_W || !qok) break;\n";
        s += "    if (in_lds) {\n" + load_set(P, need_r, "x0_", "r", &staged, "r - lo") + "    } else {\n" +
             load_set(P, need_r, "x0_", "r", nullptr, "") + "    }\n";
        s += "    {\n" + cand + "    if (ok) {\n" + on_consumed + "    }\n    }\n";
        s += "    {\n" + mid + "    }\n" + stop + "}\n";
        return s;
    };

    std::string src;
    src += head("shj_count",
                "const int64_t* __restrict__ sts, const uint32_t* __restrict__ skeys, const uint32_t* __restrict__ "
                "perm, int64_t n, uint32_t sentinel, const shd_cols* __restrict__ C, uint32_t* __restrict__ cnt, "
                "int32_t* __restrict__ flag, uint32_t tiles_per_xcd, uint32_t ntiles, shd_tiles TL");
    src += "if (key == sentinel) { cnt[j] = 0u; return; }\nuint32_t c = 0;\n";
    src += walk(true, "        c++;\n");
    src += "cnt[j] = c;\n}\n";

    src += head("shj_emit",
                "const int64_t* __restrict__ sts, const uint32_t* __restrict__ skeys, const uint32_t* __restrict__ "
                "perm, int64_t n, uint32_t sentinel, const shd_cols* __restrict__ C, const uint32_t* __restrict__ "
                "cnt, const uint32_t* __restrict__ off, uint64_t seq_base, uint64_t* __restrict__ out_seq, "
                "int64_t* __restrict__ out_ts, int64_t* __restrict__ out_vals, uint8_t* __restrict__ out_nulls, "
                "uint32_t tiles_per_xcd, uint32_t ntiles, shd_tiles TL");
    src += "if (key == sentinel) return;\nconst uint32_t c = cnt[j];\nif (c == 0u) return;\n"
           "const int64_t base = (int64_t)off[j];\nuint32_t k = 0;\n";
    std::string put = "        const int64_t dst = base + (int64_t)(c - 1u - k);\n        k++;\n"
                      "        if (out_seq) out_seq[dst] = seq_base + j;\n        if (out_ts) out_ts[dst] = tq;\n";
    put += load_set(P, extra0, "x0_", "r", nullptr, "");
    put += outs;
    put += "        if (k == c) break;\n";
    src += walk(false, put);
    src += "}\n";
    return src;
}

// Prints the two specialised kernels of a window-shaped program; false when a
// piece has no straight-line form (the caller keeps the ahead-of-time kernels).
bool generate(const shp_program& P, std::string& src) {
    Gen g(P);
    // ---- match kernel: filters of states 0 and 1
    std::string f0, f1;
    if (!g.filter(0, false, "ok", f0)) return false;
    const std::set<int> a0_f0 = g.need[0];
    g.need[0].clear();
    if (!g.filter(1, true, "ok", f1)) return false;
    std::set<int> a0_m = a0_f0;
    a0_m.insert(g.need[0].begin(), g.need[0].end());
    const std::set<int> a1_m = g.need[1];
    // ---- place kernel: select list
    Gen h(P);
    std::string outs;
    for (int o = 0; o < P.n_out; o++) {
        std::string bits, null;
        if (P.out_fast) {
            bits = h.var(P.out_slot[o] ? 1 : 0, P.out_attr[o]);
            null = "0";
        } else {
            if (P.out_pc[o] < 0) return false;
            std::string body;
            const std::string r = h.bytecode(P.out_pc[o], P.out_len[o], true, body);
            if (r.empty()) return false;
            outs += "{\n" + body;
            bits = r + ".b";
            null = r + ".null";
        }
        if (!P.out_fast) {
            outs += "if (out_vals) out_vals[dst * SHJ_NOUT + " + std::to_string(o) + "] = " + bits + ";\n";
            outs += "if (out_nulls) out_nulls[dst * SHJ_NOUT + " + std::to_string(o) + "] = (uint8_t)" + null + ";\n}\n";
        } else {
            outs += "if (out_vals) out_vals[dst * SHJ_NOUT + " + std::to_string(o) + "] = " + bits + ";\n";
            outs += "if (out_nulls) out_nulls[dst * SHJ_NOUT + " + std::to_string(o) + "] = 0;\n";
        }
    }
    std::set<int> all_m = a0_m;
    all_m.insert(a1_m.begin(), a1_m.end());
    std::set<int> all_p = h.need[0];
    all_p.insert(h.need[1].begin(), h.need[1].end());

    src = SHJ_HEADERS;
    src += "\n#define SHJ_TILE " + std::to_string(kTile) + "\n#define SHJ_HALO " + std::to_string(kHalo) +
           "\n#define SHJ_SPAN (SHJ_TILE + SHJ_HALO)\n#define SHJ_W " + lit64(P.within_ms) + "\n#define SHJ_NOUT " +
           std::to_string(P.n_out) + "\n";

    // ------------------------------------------------------------------ match
    src += R"(
extern "C" __global__ void __launch_bounds__(SHJ_TILE)
shj_match(const int64_t* __restrict__ sts, const uint32_t* __restrict__ skeys, int64_t n, uint32_t sentinel,
          const shd_cols* __restrict__ C, int32_t* __restrict__ match_pos, uint32_t* __restrict__ cnt,
          int32_t* __restrict__ flag, uint32_t tiles_per_xcd, uint32_t ntiles, shd_tiles TL) {
const TileDir D = tile_dir(TL);
__shared__ int64_t s_ts[SHJ_SPAN];
__shared__ uint32_t s_key[SHJ_SPAN];
)";
    for (int a : a1_m)
        src += "__shared__ " + std::string(col_ctype(P.attr_type[0][a])) + " s_c" + std::to_string(a) + "[SHJ_SPAN];\n";
    src += xcd_tile() + col_ptrs(P, all_m);
    src += R"(
const int64_t lim = (n < b0 + SHJ_SPAN) ? n : b0 + SHJ_SPAN;
for (int i = threadIdx.x; i < SHJ_SPAN; i += SHJ_TILE) {
    const int64_t gi = b0 + i;
    if (gi < lim) {
        s_ts[i] = sts[gi];
        s_key[i] = skeys ? skeys[gi] : 0u;
)";
    for (int a : a1_m) src += "        s_c" + std::to_string(a) + "[i] = c" + std::to_string(a) + "[gi];\n";
    src += R"(    }
}
__syncthreads();
const int64_t p = b0 + threadIdx.x;
if (p >= n) return;
const uint32_t key = s_key[threadIdx.x];
if (key == sentinel) return;
const int64_t t0 = s_ts[threadIdx.x];
// the reduction to a forward scan needs non-decreasing timestamps per key
if (D.on()) {
    const int64_t pp = key_pred(D, skeys, p, key);
    if (pp >= 0 && t0 < sts[pp]) atomicExch(flag, 1);
} else if (p > 0) {
    uint32_t kp;
    int64_t tp;
    if (threadIdx.x) { kp = s_key[threadIdx.x - 1]; tp = s_ts[threadIdx.x - 1]; }
    else { kp = skeys ? skeys[p - 1] : 0u; tp = sts[p - 1]; }
    if (kp == key && t0 < tp) atomicExch(flag, 1);
}
)";
    src += decl_attrs(a0_m, 0) + load_attrs(P, a0_m, 0, "p", &a1_m, "threadIdx.x");
    src += "{\nbool ok = true;\n" + f0 + "if (!ok) return;\n}\n";
    src += decl_attrs(a1_m, 1);
    src += R"(uint32_t ta = D.on() ? D.tile(p) : 0u;
int64_t qend = D.on() ? (int64_t)D.de[D.at(ta, key)] : n;
for (int64_t q = p + 1;; q++) {
    if (q >= qend && !(D.on() && D.next(ta, key, q, qend))) break;
    uint32_t kq;
    int64_t tq;
    if (q < lim) {
        const int l = (int)(q - b0);
        kq = s_key[l];
        tq = s_ts[l];
)";
    src += load_attrs(P, a1_m, 1, "q", &a1_m, "l");
    src += "    } else {\n        kq = skeys ? skeys[q] : 0u;\n        tq = sts[q];\n";
    src += load_attrs(P, a1_m, 1, "q", nullptr, "");
    src += R"(    }
    if (kq != key) break;
    const int64_t d = tq - t0;
    if ((d < 0 ? -d : d) > SHJ_W) break;  // expired before event q is matched
    bool ok = true;
)";
    src += f1;
    src += R"(    if (ok) {
        match_pos[p] = (int32_t)q;
        atomicAdd(&cnt[q], 1u);
        break;
    }
}
}
)";

    // ------------------------------------------------------------------ place
    src += R"(
extern "C" __global__ void __launch_bounds__(SHJ_TILE)
shj_place(const int64_t* __restrict__ sts, const uint32_t* __restrict__ skeys, const uint32_t* __restrict__ perm,
          int64_t n, const shd_cols* __restrict__ C, const int32_t* __restrict__ match_pos,
          const uint32_t* __restrict__ off, uint64_t seq_base, uint64_t* __restrict__ out_seq,
          int64_t* __restrict__ out_ts, int64_t* __restrict__ out_vals, uint8_t* __restrict__ out_nulls,
          uint32_t tiles_per_xcd, uint32_t ntiles, shd_tiles TL) {
const TileDir D = tile_dir(TL);
__shared__ int64_t s_ts[SHJ_SPAN];
__shared__ uint32_t s_key[SHJ_SPAN];
__shared__ int32_t s_mp[SHJ_SPAN];
)";
    src += xcd_tile() + col_ptrs(P, all_p);
    src += R"(
const int64_t lo = b0 > SHJ_HALO ? b0 - SHJ_HALO : 0;
const int64_t hi = (n < b0 + SHJ_TILE) ? n : b0 + SHJ_TILE;
for (int i = threadIdx.x; i < SHJ_SPAN; i += SHJ_TILE) {
    const int64_t gi = lo + i;
    if (gi < hi) {
        s_ts[i] = sts[gi];
        s_key[i] = skeys ? skeys[gi] : 0u;
        s_mp[i] = match_pos[gi];
    }
}
__syncthreads();
const int64_t p = b0 + threadIdx.x;
if (p >= n) return;
const int32_t q = s_mp[p - lo];
if (q < 0) return;
const uint32_t key = s_key[p - lo];
const int64_t tq = (q < hi) ? s_ts[q - lo] : sts[q];
uint32_t rank = 0;  // partials of the key consumed by q before this one (creation order)
uint32_t ta = D.on() ? D.tile(p) : 0u;
int64_t rbeg = D.on() ? (int64_t)D.ds[D.at(ta, key)] : 0;
for (int64_t r = p - 1;; r--) {
    if (r < rbeg && !(D.on() && D.prev(ta, key, r, rbeg))) break;
    uint32_t kr;
    int64_t tr;
    int32_t mr;
    if (r >= lo) { kr = s_key[r - lo]; tr = s_ts[r - lo]; mr = s_mp[r - lo]; }
    else { kr = skeys ? skeys[r] : 0u; tr = sts[r]; mr = match_pos[r]; }
    if (kr != key) break;
    if (tq - tr > SHJ_W) break;  // older partials expired before q
    if (mr == q) rank++;
}
const uint32_t j = perm ? perm[q] : (uint32_t)q;
const int64_t dst = (int64_t)off[j] + rank;
if (out_seq) out_seq[dst] = seq_base + j;
if (out_ts) out_ts[dst] = tq;
)";
    src += decl_attrs(h.need[0], 0) + load_attrs(P, h.need[0], 0, "p", nullptr, "");
    src += decl_attrs(h.need[1], 1) + load_attrs(P, h.need[1], 1, "q", nullptr, "");
    src += outs + "}\n";

    // ------------------------------------------------------------------ consumer-side walk
    ExtForm F;
    if (!getenv("SH_NO_EXT") && ext_form(P, F)) src += gen_ext(P, F, outs, h.need[0], h.need[1]);
    return true;
}

// ---- bucketed window engine matcher (sh_bucket.hip drives it)
//
// shb_match: one workgroup per (bucket, chunk): the chunk's SHB_CH events of the
// bucket plus SHB_HALO earlier ones are staged in LDS (packed ts | local key and
// the staged columns), stably re-sorted by local key with ballot ranking, and
// every event of the chunk walks back over its key as a consumer (ExtForm): the
// partials it consumes are counted (u8, bucket order), a scan over the chunk
// places their e1-side select values in the chunk's match-stream region, and the
// prefix at each (bucket, tile) segment start goes to psum for the emitter.
bool gen_bucket(const shp_program& P, const ExtForm& F, const std::vector<int>& ms_attrs, std::vector<int>& staged_out,
                std::string& src) {
    std::set<int> need_r, need_q;
    SideGen gq, gi;
    gq.pfx[0] = "x0_";
    gq.pfx[1] = "x1_";
    gq.need[0] = &need_r;
    gq.need[1] = &need_q;
    gi.pfx[0] = gi.pfx[1] = "x0_";
    gi.need[0] = gi.need[1] = &need_r;
    gi.tmp = 1000;
    const std::string DT = F.cross ? dom_ctype(F.dom) : "int32_t";
    std::string qhead = "bool qok = true;\n" + gq.terms(F.qonly, "qok");
    if (F.cross) qhead += "if (qok) {\n" + gq.xval(F, "xq_") + "xq = xq_;\n}\n";
    std::string cand = "bool ok = true;\n" + gq.terms(F.f1, "ok") + gq.terms(F.ionly, "ok");
    if (F.cross)
        cand += "if (ok) {\n" + gq.yval(F, "y") + "ok = cmp_op<" + DT + ">(" + std::to_string(F.op) +
                ", xq, y) && !(hasM && cmp_op<" + DT + ">(" + std::to_string(F.op) + ", M, y));\n}\n";
    else
        cand += "ok = ok && !hasM;\n";
    std::string mid = "bool mk = true;\n" + gi.terms(F.qonly, "mk");
    // unguarded (straight-line) forms for the predicated fast walk: the guarded
    // blocks only compute values, so they may run for every element
    auto unguard = [](std::string t) {
        for (const char* g : {"if (ok) {", "if (mk) {"}) {
            size_t at;
            while ((at = t.find(g)) != std::string::npos) t.replace(at, strlen(g), "{");
        }
        return t;
    };
    // (a guarded `ok = expr` must become `ok = ok && expr` once unguarded)
    std::string cand_fast = "bool ok = true;\n" + unguard(gq.terms(F.f1, "ok")) + unguard(gq.terms(F.ionly, "ok"));
    if (F.cross)
        cand_fast += "{\n" + unguard(gq.yval(F, "y")) + "ok = ok && cmp_op<" + DT + ">(" + std::to_string(F.op) +
                     ", xq, y) && !(hasM && cmp_op<" + DT + ">(" + std::to_string(F.op) + ", M, y));\n}\n";
    else
        cand_fast += "ok = ok && !hasM;\n";
    std::string mid_fast = "bool mk = true;\n" + unguard(gi.terms(F.qonly, "mk"));
    std::string stop, stop_cond;
    if (F.cross) {
        const bool mx = F.op == SH_OP_GT || F.op == SH_OP_GE;
        mid += "if (mk) {\n" + gi.xval(F, "xr") + "if (xr == xr && (!hasM || xr " + (mx ? ">" : "<") +
               " M)) M = xr;\nif (xr == xr) hasM = true;\n}\n";
        stop_cond = std::string("xq != xq || (hasM && M ") + (mx ? ">=" : "<=") + " xq)";
        mid_fast += "{\n" + unguard(gi.xval(F, "xr")) + "const uint32_t upd = (act && mk && xr == xr) ? 1u : 0u;\nM = (upd && (!hasM || xr " +
                    (mx ? ">" : "<") + " M)) ? xr : M;\nhasM |= upd;\n}\n";
    } else {
        mid += "if (mk) hasM = true;\n";
        mid_fast += "hasM |= (act && mk) ? 1u : 0u;\n";
        stop_cond = "hasM";
    }
    stop = "    if (" + stop_cond + ") { stopped = true; break; }\n";
    std::set<int> staged = need_r;
    staged.insert(need_q.begin(), need_q.end());
    for (int a : ms_attrs) staged.insert(a);
    if (staged.size() > SHB_MAX_STAGED) return false;
    staged_out.assign(staged.begin(), staged.end());
    auto sidx = [&](int a) { return (int)(std::find(staged_out.begin(), staged_out.end(), a) - staged_out.begin()); };
    auto lds = [&](int a) { return "s_a" + std::to_string(a); };
    auto loads = [&](const std::set<int>& attrs, const std::string& pfx, const std::string& row) {
        std::string s;
        for (int a : attrs)
            s += pfx + std::to_string(a) + " = " + raw_of(P.attr_type[0][a], lds(a) + "[" + row + "]") + ";\n";
        return s;
    };
    // the consumer walk back over its key in the sorted span. The first SHB_D
    // predecessors are loaded together (one LDS latency for the common case);
    // a walk that goes on past them continues one event at a time. The count
    // walk records which of the first SHB_D predecessors it consumed (u16 mask,
    // SHB_MOVF: went past SHB_D), so the emit phase rarely walks again.
    auto elem = [&](bool count, const std::string& on_consumed, const std::string& wexpr,
                    const std::string& aexpr) {
        std::string s = "    if (o < 0 || ((" + wexpr + ") & kmask) != key) { ran_off = true; break; }\n"
                        "    const int64_t tr = (int64_t)((" + wexpr + ") >> kb);\n";
        if (count) s += "    if (first && tq < tr) atomicOr(P.flag, SHB_F_MONO);\n";
        s += "    first = false;\n    if (tq - tr > SHJ_W) { stopped = true; break; }\n";
        for (int a : need_r) {
            std::string ae = aexpr;
            size_t at = ae.find("@");
            ae.replace(at, 1, std::to_string(a));
            s += "    x0_" + std::to_string(a) + " = " + raw_of(P.attr_type[0][a], ae) + ";\n";
        }
        s += "    {\n" + cand + "    if (ok) {\n" + on_consumed + "    }\n    }\n";
        s += "    {\n" + mid + "    }\n" + stop;
        return s;
    };
    auto head = [&]() {
        return "const uint32_t wq = s_ws[sp];\nconst uint32_t key = wq & kmask;\n"
               "const int64_t tq = (int64_t)(wq >> kb);\n" +
               decl_attrs(need_r, 0) + decl_attrs(need_q, 1) + loads(need_q, "x1_", "sp") + DT + " xq = 0;\n" +
               qhead + "uint32_t hasM = 0u;\n" + DT + " M = 0;\nuint32_t first = 1u;\n"
               "uint32_t stopped = qok ? 0u : 1u, ran_off = 0u;\n";
    };
    auto slow = [&](bool count, const std::string& on_consumed, const std::string& from) {
        return "for (int o = " + from + "; !stopped && !ran_off; o--) {\n" +
               elem(count, on_consumed, "s_ws[o < 0 ? 0 : o]", "s_a@[o]") + "}\n";
    };
    // the count walk: blocks of SHB_D predecessors, each loaded together and
    // walked with 0/1 word predicates (straight-line vector code: no exec-mask
    // juggling on the CU's shared scalar unit); the block loop runs while any
    // lane of the wave still walks (a uniform exit). Consumed predecessors at
    // distance < 15 go to a 16-bit mask for the emit phase (SHB_MOVF: beyond).
    auto walk_count = [&]() {
        std::string s = head() + "uint32_t mask = 0u;\nuint32_t live = stopped ? 0u : 1u, mono = 0u;\n"
                                 "for (int base = 0; __ballot(live != 0u) != 0ull; base += SHB_D) {\n"
                                 "uint32_t wv[SHB_D];\n";
        for (int a : need_r)
            s += std::string(col_ctype(P.attr_type[0][a])) + " av" + std::to_string(a) + "[SHB_D];\n";
        s += "#pragma unroll\nfor (int u = 0; u < SHB_D; u++) {\n    const int o0 = sp - 1 - base - u;\n"
             "    const int o = o0 < 0 ? 0 : o0;\n    wv[u] = s_ws[o];\n";
        for (int a : need_r) s += "    av" + std::to_string(a) + "[u] = " + lds(a) + "[o];\n";
        s += "}\n#pragma unroll\nfor (int u = 0; u < SHB_D; u++) {\n"
             "    const int step = base + u;\n"
             "    const int o = sp - 1 - step;\n"
             "    const uint32_t same = (o >= 0 && (wv[u] & kmask) == key) ? 1u : 0u;\n"
             "    const int64_t tr = (int64_t)(wv[u] >> kb);\n"
             "    const uint32_t inwin = (tq - tr <= SHJ_W) ? 1u : 0u;\n"
             "    ran_off |= live & (same ^ 1u);\n"
             "    stopped |= live & same & (inwin ^ 1u);\n"
             "    const uint32_t act = live & same & inwin;\n"
             "    mono |= act & first & ((tq < tr) ? 1u : 0u);\n"
             "    first &= act ^ 1u;\n";
        for (int a : need_r)
            s += "    x0_" + std::to_string(a) + " = " + raw_of(P.attr_type[0][a], "av" + std::to_string(a) + "[u]") + ";\n";
        s += "    {\n" + cand_fast +
             "    const uint32_t cons = act & (ok ? 1u : 0u);\n    c_ += cons;\n"
             "    mask |= step < SHB_MSTEPS ? (cons << step) : (cons ? SHB_MOVF : 0u);\n    }\n";
        s += "    {\n" + mid_fast + "    }\n    {\n    const uint32_t st = (act && (" + stop_cond +
             ")) ? 1u : 0u;\n    stopped |= st;\n    live = act & (st ^ 1u);\n    }\n}\n}\n"
             "if (mono) atomicOr(P.flag, SHB_F_MONO);\n";
        s += "if (!stopped && SHB_OFF(tq)) atomicOr(P.flag, SHB_F_HALO);\n";
        return s;
    };
    // the count walk for a floating-point ordering term: ext starts as NaN (no
    // compare with NaN holds, and maxNum/minNum skip a NaN operand), so the
    // `hasM` flag, the NaN tests on X and the per-step premise checks drop out;
    // times compare as the packed 32-bit values (in window: tr >= tq - W)
    const bool fdom = F.cross && (F.dom == DOM_F32 || F.dom == DOM_F64);
    auto walk_count_f = [&]() {
        const bool mx = F.op == SH_OP_GT || F.op == SH_OP_GE;
        const std::string opn = std::to_string(F.op);
        const std::string ext = F.dom == DOM_F32 ? (mx ? "__builtin_fmaxf" : "__builtin_fminf")
                                                 : (mx ? "__builtin_fmax" : "__builtin_fmin");
        std::string cand_f = "bool ok = true;\n" + unguard(gq.terms(F.f1, "ok")) + unguard(gq.terms(F.ionly, "ok")) +
                             "{\n" + unguard(gq.yval(F, "y")) + "ok = ok && cmp_op<" + DT + ">(" + opn +
                             ", xq, y) && !cmp_op<" + DT + ">(" + opn + ", Mx, y);\n}\n";
        std::string mid_f = "bool mk = true;\n" + unguard(gi.terms(F.qonly, "mk")) + "{\n" + unguard(gi.xval(F, "xr")) +
                            "Mx = (act && mk) ? " + ext + "(Mx, xr) : Mx;\n}\n";
        std::string s = head() +
                        "const uint32_t tq32 = wq >> kb;\n"
                        "const uint32_t tlo = tq32 > SHB_WLIM ? tq32 - SHB_WLIM : 0u;\n" + DT +
                        " Mx = " + (F.dom == DOM_F32 ? "__builtin_nanf(\"\")" : "__builtin_nan(\"\")") + ";\n"
                        "uint32_t mask = 0u, cext = 0u, roff = 0u;\n"
                        "uint32_t live = (qok && xq == xq) ? 1u : 0u;\n"
                        "if (live && sp >= 1) {\n"
                        "    const uint32_t wp = s_ws[sp - 1];\n"
                        "    if (((wp ^ wq) & kmask) == 0u && (wp >> kb) > tq32) atomicOr(P.flag, SHB_F_MONO);\n"
                        "}\n"
                        "for (int base = 0; __ballot(live != 0u) != 0ull; base += SHB_D) {\n"
                        "uint32_t wv[SHB_D];\n";
        for (int a : need_r)
            s += std::string(col_ctype(P.attr_type[0][a])) + " av" + std::to_string(a) + "[SHB_D];\n";
        s += "#pragma unroll\nfor (int u = 0; u < SHB_D; u++) {\n    const int o0 = sp - 1 - base - u;\n"
             "    const int o = o0 < 0 ? 0 : o0;\n    wv[u] = s_ws[o];\n";
        for (int a : need_r) s += "    av" + std::to_string(a) + "[u] = " + lds(a) + "[o];\n";
        s += "}\n#pragma unroll\nfor (int u = 0; u < SHB_D; u++) {\n"
             "    const int step = base + u;\n"
             "    const uint32_t same = (u < sp - base && ((wv[u] ^ wq) & kmask) == 0u) ? 1u : 0u;\n"
             "    roff |= live & (same ^ 1u);\n"
             "    const uint32_t act = live & same & ((wv[u] >> kb) >= tlo ? 1u : 0u);\n";
        for (int a : need_r)
            s += "    x0_" + std::to_string(a) + " = " + raw_of(P.attr_type[0][a], "av" + std::to_string(a) + "[u]") + ";\n";
        s += "    {\n" + cand_f +
             "    const uint32_t cons = act & (ok ? 1u : 0u);\n"
             "    if (step < SHB_MSTEPS) mask |= cons << step;\n"
             "    else { cext += cons; mask |= cons ? SHB_MOVF : 0u; }\n    }\n";
        s += "    {\n" + mid_f + "    }\n    live = act & (cmp_op<" + DT + ">(" + (mx ? std::to_string(SH_OP_GE)
                                                                                  : std::to_string(SH_OP_LE)) +
             ", Mx, xq) ? 0u : 1u);\n}\n}\n"
             "c_ = (uint32_t)__popc(mask & ~SHB_MOVF) + cext;\n"
             "if (roff && SHB_OFF(tq32)) atomicOr(P.flag, SHB_F_HALO);\n";
        return s;
    };
    // the same float-domain count walk with work handed out per lane: a wave owns a
    // contiguous range of the chunk's consumers; a lane whose walk ended stores its
    // result and takes the next consumer of the range (ballot rank), so a block of
    // SHB_D steps runs for busy lanes only instead of every lane waiting for the
    // wave's longest walk (C2: mean walk 3.4 steps, p90 9, wave max ~15)
    auto walk_count_f_dyn = [&]() {
        const bool mx = F.op == SH_OP_GT || F.op == SH_OP_GE;
        const std::string opn = std::to_string(F.op);
        const std::string ext = F.dom == DOM_F32 ? (mx ? "__builtin_fmaxf" : "__builtin_fminf")
                                                 : (mx ? "__builtin_fmax" : "__builtin_fmin");
        const std::string nan = F.dom == DOM_F32 ? "__builtin_nanf(\"\")" : "__builtin_nan(\"\")";
        std::string cand_f = "bool ok = true;\n" + unguard(gq.terms(F.f1, "ok")) + unguard(gq.terms(F.ionly, "ok")) +
                             "{\n" + unguard(gq.yval(F, "y")) + "ok = ok && cmp_op<" + DT + ">(" + opn +
                             ", xq, y) && !cmp_op<" + DT + ">(" + opn + ", Mx, y);\n}\n";
        std::string mid_f = "bool mk = true;\n" + unguard(gi.terms(F.qonly, "mk")) + "{\n" + unguard(gi.xval(F, "xr")) +
                            "Mx = (act && mk) ? " + ext + "(Mx, xr) : Mx;\n}\n";
        std::string s =
            "{\n"
            "const int dl_ = (int)(threadIdx.x & 63u), dw_ = (int)(threadIdx.x >> 6);\n"
            "const int per_ = (nc + (SHB_TPB / 64) - 1) / (SHB_TPB / 64);\n"
            "const int c0_ = dw_ * per_ < nc ? dw_ * per_ : nc, c1_ = c0_ + per_ < nc ? c0_ + per_ : nc;\n"
            "const uint64_t dlt_ = dl_ ? (~0ull >> (64 - dl_)) : 0ull;\n"
            "int next_ = c0_, ci = -1, sp = 0, i = 0, base = 0;\n"
            "uint32_t wq = 0u, tlo = 0u, mask = 0u, cext = 0u, roff = 0u, live = 0u;\n" +
            DT + " xq = 0;\n" + DT + " Mx = " + nan + ";\n"
            "for (;;) {\n"
            "    if (ci >= 0 && !live) {\n"
            "        const uint32_t c_ = (uint32_t)__popc(mask & ~SHB_MOVF) + cext;\n"
            "        if (roff && SHB_OFF(wq >> kb)) atomicOr(P.flag, SHB_F_HALO);\n"
            "        if (c_ > 255u) atomicOr(P.flag, SHB_F_COUNT);\n"
            "        s_pre[i - hl] = (uint16_t)(c_ > 255u ? 255u : c_);\n"
            "        s_msk[i - hl] = (uint16_t)mask;\n"
            "        slow_ |= (int)(mask & SHB_MOVF);\n"
            "        ci = -1;\n"
            "    }\n"
            "    const uint64_t im_ = __ballot(ci < 0);\n"
            "    const int r_ = (int)__popcll(im_ & dlt_);\n"
            "    if (ci < 0 && next_ + r_ < c1_) {\n"
            "        ci = next_ + r_;\n"
            "        const uint32_t cw = s_cons[ci];\n"
            "        sp = (int)(cw & 0xFFFFu);\n"
            "        i = hl + (int)(cw >> 16);\n"
            "        wq = s_ws[sp];\n"
            "        const uint32_t tq32 = wq >> kb;\n"
            "        tlo = tq32 > SHB_WLIM ? tq32 - SHB_WLIM : 0u;\n" +
            decl_attrs(need_q, 1) + loads(need_q, "x1_", "sp") + "xq = 0;\n" + qhead +
            "        Mx = " + nan + ";\n"
            "        mask = 0u; cext = 0u; roff = 0u; base = 0;\n"
            "        live = (qok && xq == xq) ? 1u : 0u;\n"
            "        if (live && sp >= 1) {\n"
            "            const uint32_t wp = s_ws[sp - 1];\n"
            "            if (((wp ^ wq) & kmask) == 0u && (wp >> kb) > tq32) atomicOr(P.flag, SHB_F_MONO);\n"
            "        }\n"
            "    }\n"
            "    next_ += (int)__popcll(im_);\n"
            "    if (__ballot(ci >= 0) == 0ull) break;\n"
            "    uint32_t wv[SHB_D];\n";
        for (int a : need_r)
            s += std::string(col_ctype(P.attr_type[0][a])) + " av" + std::to_string(a) + "[SHB_D];\n";
        s += "#pragma unroll\nfor (int u = 0; u < SHB_D; u++) {\n    const int o0 = sp - 1 - base - u;\n"
             "    const int o = o0 < 0 ? 0 : o0;\n    wv[u] = s_ws[o];\n";
        for (int a : need_r) s += "    av" + std::to_string(a) + "[u] = " + lds(a) + "[o];\n";
        s += "}\n" + decl_attrs(need_r, 0) +
             "#pragma unroll\nfor (int u = 0; u < SHB_D; u++) {\n"
             "    const int step = base + u;\n"
             "    const uint32_t same = (u < sp - base && ((wv[u] ^ wq) & kmask) == 0u) ? 1u : 0u;\n"
             "    roff |= live & (same ^ 1u);\n"
             "    const uint32_t act = live & same & ((wv[u] >> kb) >= tlo ? 1u : 0u);\n";
        for (int a : need_r)
            s += "    x0_" + std::to_string(a) + " = " + raw_of(P.attr_type[0][a], "av" + std::to_string(a) + "[u]") + ";\n";
        s += "    {\n" + cand_f +
             "    const uint32_t cons = act & (ok ? 1u : 0u);\n"
             "    if (step < SHB_MSTEPS) mask |= cons << step;\n"
             "    else { cext += cons; mask |= cons ? SHB_MOVF : 0u; }\n    }\n";
        s += "    {\n" + mid_f + "    }\n    live = act & (cmp_op<" + DT + ">(" + (mx ? std::to_string(SH_OP_GE)
                                                                                  : std::to_string(SH_OP_LE)) +
             ", Mx, xq) ? 0u : 1u);\n}\nbase += SHB_D;\n}\n}\n";
        return s;
    };
    auto walk = [&](bool count, const std::string& on_consumed) {
        return head() + slow(count, on_consumed, "sp - 1");
    };
    std::string ms_put;
    for (size_t m = 0; m < ms_attrs.size(); m++) {
        const int a = ms_attrs[m];
        ms_put += "        ((" + std::string(col_ctype(P.attr_type[0][a])) + "*)P.ms[" + std::to_string(m) +
                  "])[dst] = " + lds(a) + "[o];\n";
    }
    (void)sidx;

    src = SHJ_HEADERS;
    const int64_t wlim = P.within_ms < 0 ? 0 : (P.within_ms > 0xFFFFFFFFll ? 0xFFFFFFFFll : P.within_ms);
    src += "\n#define SHJ_W " + lit64(P.within_ms) + "\n#define SHB_WLIM " + std::to_string(wlim) +
           "u\n#define SHB_TPB 512\n#define SHB_D " + std::to_string(kWalkBlock) +
           "\n#define SHB_MOVF 0x8000u\n#define SHB_MSTEPS 15\n"
           "#define SHB_MINB " + std::to_string(kMatchMinBlocks) + "\n"
           "#define SHB_NSEG (SHB_CT_MAX + SHB_HMAX)\n"
           "#define SHB_SPANJ " + std::to_string(kSpan) + "\n#define SHB_CHJ " + std::to_string(kChunk) + "\n" +
           "#define SHB_NR (SHB_SPANJ / SHB_TPB)\nstatic_assert(SHB_SPANJ % SHB_TPB == 0 && SHB_NR * SHB_TPB == SHB_SPANJ && SHB_SPANJ <= SHB_SPAN && SHB_CHJ <= SHB_CH && SHB_CHJ % SHB_TPB == 0, \"span\");\n"
           "static_assert(SHB_NSEG < 256 && SHB_NSEG < SHB_TPB, \"segments\");\n";
    src += R"(
extern "C" __global__ void __launch_bounds__(SHB_TPB, SHB_MINB) shb_match(shb_plan P) {
__shared__ uint32_t s_ws[SHB_SPANJ];
// the chunk's consumers in sorted order: sorted position | (arrival - hl) << 16
__shared__ uint32_t s_cons[SHB_CHJ];
__shared__ uint16_t s_pre[SHB_CHJ];
__shared__ uint32_t u_buf[(SHB_TPB / 64) * 256];  // rank phase: per-wave key counts; then the u16 consumed masks
uint32_t (*const wcnt)[256] = (uint32_t(*)[256])u_buf;
uint16_t* const s_msk = (uint16_t*)u_buf;
static_assert((SHB_TPB / 64) * 256 * 4 >= SHB_CHJ * 2, "masks fit u_buf");
// run: halo events per local key, then their inclusive prefix over the keys
__shared__ uint32_t run[256], tstart[256], ws[SHB_TPB / 64];
// the pass's segments, one per tile from the first halo tile: start in span
// order (exclusive prefix of the lengths, from the table's first tile) and the
// global index of the first event; seg_of[j]: segment of span event 32 j
__shared__ uint32_t seg_p[SHB_NSEG + 1];
__shared__ uint32_t seg_g[SHB_NSEG];
__shared__ uint8_t seg_of[SHB_SPANJ / 32];
__shared__ int s_i[2];
)";
    for (int a : staged_out)
        src += "__shared__ " + std::string(col_ctype(P.attr_type[0][a])) + " " + lds(a) + "[SHB_SPANJ];\n";
    for (size_t k = 0; k < staged_out.size(); k++) {
        const int a = staged_out[k];
        const std::string ct = col_ctype(P.attr_type[0][a]);
        src += "const " + ct + "* __restrict__ g_a" + std::to_string(a) + " = (const " + ct + "*)P.st_dst[" +
               std::to_string(k) + "];\n";
    }
    src += R"(
// consecutive buckets on one XCD (blocks are dealt round-robin to the 8 XCDs):
// neighbouring segments of a tile share cache lines
const int b = (int)((blockIdx.x & 7u) * (SHB_NB / 8) + ((blockIdx.x >> 3) & (SHB_NB / 8 - 1)));
const int A = (int)(blockIdx.x / SHB_NB) * P.ct;
const int E = A + P.ct < P.nt ? A + P.ct : P.nt;
const int kb = P.kb;
const uint32_t kmask = (1u << kb) - 1u;
const int lane = (int)(threadIdx.x & 63u), wv = (int)(threadIdx.x >> 6);
for (int a = A; a < E;) {
__syncthreads();
unsigned long long t_prev = wall_clock64();
#define SHB_PROF(ph) if (P.prof && threadIdx.x == 0) { const unsigned long long t_now = wall_clock64(); atomicAdd(&P.prof[ph], t_now - t_prev); t_prev = t_now; }
// the halo start (k_bk_tpre: tile a - 1 and the tiles before it that the window
// can reach) and the bucket starts of tiles [a - SHB_HMAX, E), loaded together
if (threadIdx.x == 0) s_i[0] = P.hstart[a];
const int Tm = a - SHB_HMAX + (int)threadIdx.x;
uint32_t len = 0u, g = 0u;
if (Tm >= 0 && Tm < E) {
    const uint32_t lo = P.tofft[(int64_t)b * P.tstride + Tm], hi = P.tofft[(int64_t)(b + 1) * P.tstride + Tm];
    len = hi - lo;
    g = ((uint32_t)Tm << SHB_TILE_SHIFT) + lo;

)";
    src += R"(}
__syncthreads();
const int h0 = s_i[0];  // first tile of the segment table
const int nseg = E - h0;
{
    if (Tm < h0) len = 0u;
    uint32_t tot;
    const uint32_t pre = shw_block_excl<SHB_TPB>(len, ws, &tot);
    if (Tm >= h0 && Tm < E) {
        seg_p[Tm - h0] = pre;
        seg_g[Tm - h0] = g;
    }
    if (Tm == E) seg_p[nseg] = tot;
}
__syncthreads();
// this pass: consumers from tiles [a, a + ne), at most SHB_CHJ events; the halo
// from segment sb on (trimmed at the front when it and tile a overflow the span)
const int ta = a - h0;
const uint32_t pa = seg_p[ta];
const int sb = __syncthreads_count((int)threadIdx.x < ta && seg_p[ta + 1] - seg_p[threadIdx.x] > SHB_SPANJ);
const uint32_t sbase = seg_p[sb];
const int ne = __syncthreads_count((int)threadIdx.x >= ta && (int)threadIdx.x < nseg &&
                                   seg_p[threadIdx.x + 1] - pa <= SHB_CHJ &&
                                   seg_p[threadIdx.x + 1] - sbase <= SHB_SPANJ);
if (ne == 0) {
    // tile a's segment alone exceeds a chunk
    if (threadIdx.x == 0) atomicOr(P.flag, SHB_F_SPAN);
    a++;
    continue;
}
const int se = ta + ne;      // one past the pass's last segment
const int hs = h0 + sb;      // the span's first tile (> 0: earlier events exist)
const int L = (int)(seg_p[se] - sbase), hl = (int)(pa - sbase), nc = L - hl;
// a walk that leaves its key's run in the span while still in the window could
// have missed earlier events of the key only if some event before the span is
// as late as the window's start (tpre: the latest timestamp before each tile)
const int64_t tmx_ = hs > 0 ? P.tpre[hs] - P.tbase : INT64_MIN;
#define SHB_OFF(t32) ((int64_t)(t32) - SHJ_W <= tmx_)
for (int j = (int)threadIdx.x; j * 32 < L; j += SHB_TPB) {
    const uint32_t e = sbase + (uint32_t)j * 32u;
    int lo = sb, hi = se - 1;  // the last segment starting at or before e
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (seg_p[mid] <= e) lo = mid;
        else hi = mid - 1;
    }
    seg_of[j] = (uint8_t)lo;
}
__syncthreads();
SHB_PROF(5)
// global index of span event i (segments in span order)
#define SHB_GIDX(i, out) { int sg_ = seg_of[(i) >> 5]; while (seg_p[sg_ + 1] - sbase <= (uint32_t)(i)) sg_++; \
    out = seg_g[sg_] + ((uint32_t)(i) - (seg_p[sg_] - sbase)); }
if (threadIdx.x < 256) run[threadIdx.x] = 0u;
// the span into registers (all loads in flight together): wave v owns the
// contiguous span events [v * SHB_NR * 64, (v + 1) * SHB_NR * 64)
uint32_t wr[SHB_NR];
)";
    for (int a : staged_out)
        src += std::string(col_ctype(P.attr_type[0][a])) + " vr" + std::to_string(a) + "[SHB_NR];\n";
    src += R"(#pragma unroll
for (int k = 0; k < SHB_NR; k++) {
    const int i = (wv * SHB_NR + k) * 64 + lane;
    uint32_t gi = 0u;
    if (i < L) SHB_GIDX(i, gi)
    wr[k] = i < L ? P.w0[gi] : 0u;
)";
    for (int a : staged_out)
        src += "    vr" + std::to_string(a) + "[k] = i < L ? g_a" + std::to_string(a) + "[gi] : 0;\n";
    src += R"(}
for (int c = (int)threadIdx.x; c < (SHB_TPB / 64) * 256; c += SHB_TPB) (&wcnt[0][0])[c] = 0u;
__syncthreads();
SHB_PROF(0)
// stable sort of the span by local key, staged in sorted order (the walks read
// consecutive LDS words): each wave ranks its own events (kb ballots per round,
// running per-key counts of the wave), one block pass combines the waves
uint32_t rw[SHB_NR];
{
    const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
#pragma unroll
    for (int k = 0; k < SHB_NR; k++) {
        const int i = (wv * SHB_NR + k) * 64 + lane;
        const bool valid = i < L;
        const uint32_t d = wr[k] & kmask;
        uint64_t peers = __ballot(valid);
#pragma unroll
        for (int bb = 0; bb < 8; bb++) {
            if (bb < kb) {  // uniform: the local key has kb bits
                const bool bit = (d >> bb) & 1u;
                const uint64_t m = __ballot(valid && bit);
                peers &= bit ? m : ~m;
            }
        }
        const uint32_t r = (uint32_t)__popcll(peers & lt);
        const uint32_t base = valid ? wcnt[wv][d] : 0u;
        rw[k] = valid ? ((base + r) | (d << 16)) : ~0u;
        const uint64_t hal = peers & __ballot(i < hl);  // this round's halo events of key d
        if (valid && r == 0) {
            wcnt[wv][d] = base + (uint32_t)__popcll(peers);
            if (hal) atomicAdd(&run[d], (uint32_t)__popcll(hal));
        }
    }
}
__syncthreads();
{
    uint32_t tot = 0, all;
    if (threadIdx.x < 256) {
#pragma unroll
        for (int q = 0; q < SHB_TPB / 64; q++) {
            const uint32_t c = wcnt[q][threadIdx.x];
            wcnt[q][threadIdx.x] = tot;
            tot += c;
        }
    }
    // one scan for both: span events (low 16 bits) and halo events (high 16 bits) per key
    const uint32_t h = threadIdx.x < 256 ? run[threadIdx.x] : 0u;
    const uint32_t ex = shw_block_excl<SHB_TPB>(threadIdx.x < 256 ? (tot | (h << 16)) : 0u, ws, &all);
    if (threadIdx.x < 256) {
        tstart[threadIdx.x] = ex & 0xFFFFu;
        run[threadIdx.x] = (ex >> 16) + h;
    }
}
__syncthreads();
#pragma unroll
for (int k = 0; k < SHB_NR; k++) {
    if (rw[k] == ~0u) continue;
    const int i = (wv * SHB_NR + k) * 64 + lane;
    const uint32_t d = (rw[k] >> 16) & 0xFFu;
    const int pos = (int)(tstart[d] + wcnt[wv][d] + (rw[k] & 0xFFFFu));
    s_ws[pos] = wr[k];
    // a key's halo events precede its chunk events in sorted order, so the
    // consumer's rank is its position less the halo events of keys <= d
    if (i >= hl) s_cons[pos - (int)run[d]] = (uint32_t)pos | ((uint32_t)(i - hl) << 16);

)";
    for (int a : staged_out) src += "    " + lds(a) + "[pos] = vr" + std::to_string(a) + "[k];\n";
    src += R"(}
__syncthreads();
SHB_PROF(1)
)";
    // slow_: some consumer took a partial beyond the mask's SHB_MSTEPS steps (its
    // match-stream values then come from a second walk)
    src += "int slow_ = 0;\n";
    if (fdom && kWalkDyn) {
        // consumers (chunk events): per-lane work hand-out over each wave's range
        src += "// consumers (chunk events): partials taken per event\n" + walk_count_f_dyn() + "__syncthreads();\n";
    } else {
        src += R"(// consumers (chunk events) in sorted order: partials taken per event
for (int ci = threadIdx.x; ci < nc; ci += SHB_TPB) {
const uint32_t cw = s_cons[ci];
const int sp = (int)(cw & 0xFFFFu), i = hl + (int)(cw >> 16);
uint32_t c_ = 0;
)";
        src += fdom ? walk_count_f() : walk_count();
        src += R"(if (c_ > 255u) atomicOr(P.flag, SHB_F_COUNT);
s_pre[i - hl] = (uint16_t)(c_ > 255u ? 255u : c_);
s_msk[i - hl] = (uint16_t)mask;
slow_ |= (int)(mask & SHB_MOVF);
}
__syncthreads();)";
    }
    src += R"(
SHB_PROF(2)
// the counts to the events' slots; their exclusive prefix over the chunk
// (arrival order inside the bucket)
uint32_t total;
{
    const int p0 = (int)threadIdx.x * (SHB_CHJ / SHB_TPB);
    uint32_t v[SHB_CHJ / SHB_TPB];
    uint32_t sum = 0;
#pragma unroll
    for (int q = 0; q < SHB_CHJ / SHB_TPB; q++) {
        v[q] = (p0 + q < nc) ? (uint32_t)s_pre[p0 + q] : 0u;
        sum += v[q];
    }
    uint32_t off = shw_block_excl<SHB_TPB>(sum, ws, &total);
#pragma unroll
    for (int q = 0; q < SHB_CHJ / SHB_TPB; q++) {
        if (p0 + q < nc) {
            uint32_t gi;
            SHB_GIDX(hl + p0 + q, gi)
            P.cnt[gi] = (uint8_t)v[q];
            s_pre[p0 + q] = (uint16_t)off;
        }
        off += v[q];
    }
}
// the pass's match-stream region: the workgroup's own for its first pass (a
// pass takes at most SHB_SPANJ), taken from the shared tail for any further one
if (a != A && threadIdx.x == 0) s_i[1] = total ? (int)atomicAdd(P.ms_ctr, total) : 0;
__syncthreads();
const int64_t rbase = a == A ? (int64_t)blockIdx.x * SHB_SPAN
                             : (int64_t)gridDim.x * SHB_SPAN + (int64_t)(uint32_t)s_i[1];
// per chunk tile: the first match position of its segment, its matches
for (int t = ta + (int)threadIdx.x; t < se; t += SHB_TPB) {
    const uint32_t x0 = seg_p[t] - pa, x1 = seg_p[t + 1] - pa;
    const uint32_t q0 = x0 < (uint32_t)nc ? (uint32_t)s_pre[x0] : total;
    const uint32_t q1 = x1 < (uint32_t)nc ? (uint32_t)s_pre[x1] : total;
    const int T = h0 + t;
    P.mstart[(int64_t)T * SHB_NB + b] = (uint32_t)rbase + q0;
    if (q1 > q0) atomicAdd(&P.ttot[T], q1 - q0);
}
SHB_PROF(3)
)";
    // one 4-byte match-stream column (C2's e1.price): when no consumer needs the
    // slow walk (which reads s_ws), the values are staged in s_ws in region order
    // and the region goes out as one coalesced run
    const bool stage1 = ms_attrs.size() == 1 && type_width_of(P.attr_type[0][ms_attrs[0]]) == 4;
    if (stage1) {
        const std::string a0 = lds(ms_attrs[0]);
        // (every consumer's LDS words loaded before any value moves: one round
        // trip for the chunk's at most SHB_CHJ / SHB_TPB consumers per thread)
        src += "if (!__syncthreads_or(slow_)) {\n"
               "int sp_[SHB_CHJ / SHB_TPB];\nuint32_t off_[SHB_CHJ / SHB_TPB], m_[SHB_CHJ / SHB_TPB], "
               "nx_[SHB_CHJ / SHB_TPB];\n"
               "#pragma unroll\nfor (int q = 0; q < SHB_CHJ / SHB_TPB; q++) {\n"
               "    const int ci = (int)threadIdx.x + q * SHB_TPB;\n"
               "    const uint32_t cw = ci < nc ? s_cons[ci] : 0u;\n"
               "    const int i = hl + (int)(cw >> 16);\n"
               "    sp_[q] = (int)(cw & 0xFFFFu);\n"
               "    off_[q] = ci < nc ? (uint32_t)s_pre[i - hl] : 0u;\n"
               "    nx_[q] = ci < nc && i + 1 < L ? (uint32_t)s_pre[i + 1 - hl] : total;\n"
               "    m_[q] = ci < nc ? (uint32_t)s_msk[i - hl] : 0u;\n}\n"
               "#pragma unroll\nfor (int q = 0; q < SHB_CHJ / SHB_TPB; q++) {\n"
               "    const uint32_t off = off_[q], cn = nx_[q] - off;\n"
               "    uint32_t m = m_[q], k = 0;\n"
               "    while (m) {\n"
               "        const int o = sp_[q] - __ffs(m);\n"
               "        m &= m - 1u;\n"
               "        s_ws[off + (cn - 1u - k)] = (uint32_t)" + a0 + "[o];\n"
               "        k++;\n"
               "    }\n}\n"
               "__syncthreads();\n"
               "for (int q = threadIdx.x; q < (int)total; q += SHB_TPB) ((uint32_t*)P.ms[0])[rbase + q] = s_ws[q];\n"
               "} else {\n";
    }
    src += R"(// the partials again, their e1-side select values into the region
for (int ci = threadIdx.x; ci < nc; ci += SHB_TPB) {
const uint32_t cw = s_cons[ci];
const int sp = (int)(cw & 0xFFFFu), i = hl + (int)(cw >> 16);
const uint32_t off = s_pre[i - hl];
const uint32_t cn = ((i + 1 < L) ? (uint32_t)s_pre[i + 1 - hl] : total) - off;
if (cn == 0u) continue;
uint32_t k = 0;
)";
    std::string put = "        const int64_t dst = rbase + (int64_t)off + (int64_t)(cn - 1u - k);\n        k++;\n" + ms_put +
                      "        if (k == cn) { stopped = true; break; }\n";
    src += "const uint32_t mk = s_msk[i - hl];\nif (!(mk & SHB_MOVF)) {\n    uint32_t m = mk;\n"
           "    while (m) {\n        const int o = sp - __ffs(m);\n        m &= m - 1u;\n"
           "        const int64_t dst = rbase + (int64_t)off + (int64_t)(cn - 1u - k);\n        k++;\n" +
           ms_put + "    }\n} else {\n" + walk(false, put) + "}\n";
    src += "}\n";
    if (stage1) src += "}\n";
    src += "SHB_PROF(4)\na += ne;\n}\n}\n";

    return true;
}

struct Entry {
    int status = 0;           // 0 ok, <0 failed (message in err)
    std::string err;
    std::vector<char> code;   // gfx950 code object
    hipModule_t mod = nullptr;
    hipFunction_t match = nullptr, place = nullptr, count = nullptr, emit = nullptr;
};

std::mutex g_mu;
std::map<std::string, Entry*> g_cache;  // by generated source; lives for the process

Entry* compile(const std::string& src) {
    std::lock_guard<std::mutex> lk(g_mu);
    auto it = g_cache.find(src);
    if (it != g_cache.end()) return it->second;
    Entry* e = new Entry();
    g_cache[src] = e;
    hiprtcProgram prog;
    if (hiprtcCreateProgram(&prog, src.c_str(), "sh_jit_window.hip", 0, nullptr, nullptr) != HIPRTC_SUCCESS) {
        e->status = -1;
        e->err = "hiprtcCreateProgram failed";
        return e;
    }
    const char* opts[] = {"--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
                          "-fno-gpu-flush-denormals-to-zero", "-fhip-fp32-correctly-rounded-divide-sqrt"};
    const hiprtcResult rc = hiprtcCompileProgram(prog, (int)(sizeof(opts) / sizeof(opts[0])), opts);
    if (rc != HIPRTC_SUCCESS) {
        size_t n = 0;
        hiprtcGetProgramLogSize(prog, &n);
        std::string log(n + 1, '\0');
        hiprtcGetProgramLog(prog, &log[0]);
        e->status = -2;
        e->err = "hipRTC: " + std::string(hiprtcGetErrorString(rc)) + "\n" + log.c_str();
        hiprtcDestroyProgram(&prog);
        return e;
    }
    size_t n = 0;
    hiprtcGetCodeSize(prog, &n);
    e->code.resize(n);
    hiprtcGetCode(prog, e->code.data());
    hiprtcDestroyProgram(&prog);
    return e;
}

}  // namespace

int shj_window_source(const shp_program* hp, std::string* src) {
    if (!hp->window_ok) return -1;
    return generate(*hp, *src) ? 0 : -1;
}

int shj_window_compile(const shp_program* hp, shj_window* out, std::string* err) {
    memset(out, 0, sizeof(*out));
    std::string src;
    if (shj_window_source(hp, &src)) {
        if (err) *err = "no straight-line form";
        return -1;
    }
    Entry* e = compile(src);
    if (e->status) {
        if (err) *err = e->err;
        return e->status;
    }
    out->code = e->code.data();
    out->code_size = e->code.size();
    return 0;
}

int shj_window_load(const shp_program* hp, shj_window* out, std::string* err) {
    int rc = shj_window_compile(hp, out, err);
    if (rc) return rc;
    std::string src;
    shj_window_source(hp, &src);
    std::lock_guard<std::mutex> lk(g_mu);
    Entry* e = g_cache[src];
    if (!e->mod) {
        if (hipModuleLoadData(&e->mod, e->code.data()) != hipSuccess ||
            hipModuleGetFunction(&e->match, e->mod, "shj_match") != hipSuccess ||
            hipModuleGetFunction(&e->place, e->mod, "shj_place") != hipSuccess) {
            if (err) *err = "hipModuleLoadData/GetFunction failed";
            e->mod = nullptr;
            return -3;
        }
        if (hipModuleGetFunction(&e->count, e->mod, "shj_count") != hipSuccess ||
            hipModuleGetFunction(&e->emit, e->mod, "shj_emit") != hipSuccess) {
            e->count = nullptr;
            e->emit = nullptr;
            (void)hipGetLastError();
        }
    }
    out->match = e->match;
    out->place = e->place;
    out->count = e->count;
    out->emit = e->emit;
    return 0;
}

int shj_bucket_load(const shp_program* hp, const int* ms_attrs, int n_ms, shj_bucket* out, std::string* err) {
    memset(out, 0, sizeof(*out));
    ExtForm F;
    if (!hp->window_ok || !ext_form(*hp, F)) {
        if (err) *err = "no consumer-side form";
        return -1;
    }
    std::vector<int> ms(ms_attrs, ms_attrs + n_ms), staged;
    std::string src;
    if (!gen_bucket(*hp, F, ms, staged, src)) {
        if (err) *err = "too many staged columns";
        return -1;
    }
    Entry* e = compile(src);
    if (e->status) {
        if (err) *err = e->err;
        return e->status;
    }
    std::lock_guard<std::mutex> lk(g_mu);
    if (!e->mod) {
        if (hipModuleLoadData(&e->mod, e->code.data()) != hipSuccess ||
            hipModuleGetFunction(&e->match, e->mod, "shb_match") != hipSuccess) {
            if (err) *err = "hipModuleLoadData/GetFunction (shb_match) failed";
            e->mod = nullptr;
            return -3;
        }
    }
    out->match = e->match;
    out->n_staged = (int)staged.size();
    for (size_t k = 0; k < staged.size(); k++) out->staged_attr[k] = staged[k];
    return 0;
}

int shj_bucket_source(const shp_program* hp, const int* ms_attrs, int n_ms, std::string* src) {
    ExtForm F;
    if (!hp->window_ok || !ext_form(*hp, F)) return -1;
    std::vector<int> ms(ms_attrs, ms_attrs + n_ms), staged;
    return gen_bucket(*hp, F, ms, staged, *src) ? 0 : -1;
}

int shj_bucket_compile(const shp_program* hp, const int* ms_attrs, int n_ms, std::string* err) {
    std::string src;
    if (shj_bucket_source(hp, ms_attrs, n_ms, &src)) {
        if (err) *err = "no consumer-side form";
        return -1;
    }
    Entry* e = compile(src);
    if (e->status && err) *err = e->err;
    return e->status;
}

unsigned shj_tiles(int64_t n, uint32_t* tiles_per_xcd, uint32_t* ntiles) {
    const int64_t t = (n + kTile - 1) / kTile;
    *ntiles = (uint32_t)t;
    *tiles_per_xcd = (uint32_t)((t + 7) / 8);
    return *tiles_per_xcd * 8u;
}

int shj_bucket_chunk(void) { return kChunk; }

int shj_tile_size(void) { return kTile; }
