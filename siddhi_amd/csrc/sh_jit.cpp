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

constexpr int kTile = 256;   // events per workgroup (one lane each)
constexpr int kHalo = 256;   // staged events beyond the tile (forward for match, backward for place)

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

std::string xcd_tile() {
    return "const uint32_t tile = (blockIdx.x & 7u) * tiles_per_xcd + (blockIdx.x >> 3);\n"
           "if (tile >= ntiles) return;\n"
           "const int64_t b0 = (int64_t)tile * SHJ_TILE;\n";
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
    return true;
}

struct Entry {
    int status = 0;           // 0 ok, <0 failed (message in err)
    std::string err;
    std::vector<char> code;   // gfx950 code object
    hipModule_t mod = nullptr;
    hipFunction_t match = nullptr, place = nullptr;
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
    }
    out->match = e->match;
    out->place = e->place;
    return 0;
}

unsigned shj_tiles(int64_t n, uint32_t* tiles_per_xcd, uint32_t* ntiles) {
    const int64_t t = (n + kTile - 1) / kTile;
    *ntiles = (uint32_t)t;
    *tiles_per_xcd = (uint32_t)((t + 7) / 8);
    return *tiles_per_xcd * 8u;
}

int shj_tile_size(void) { return kTile; }
