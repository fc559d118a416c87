// sh_vm.h — typed postfix expression VM for filters and select expressions
// (device side). Conversion and null rules of the reference executors:
// core/executor/condition/compare/** (binary numeric promotion; ==/!= on
// Float/Long compare as double), core/executor/condition/{And,Or,Not,IsNull}*,
// core/executor/math/** (null on x/0 and x%0, Java integer wrap-around).
#pragma once
#include <hip/hip_runtime.h>

#include "../../include/sh_query.h"
#include "sh_device.h"

// ------------------------------------------------------------------ expression VM
struct VmVal {
    int64_t b;
    uint8_t t;
    uint8_t null;
};

__device__ __forceinline__ float bits_f32(int64_t b) { return __int_as_float((int32_t)(uint32_t)b); }
__device__ __forceinline__ double bits_f64(int64_t b) { return __longlong_as_double(b); }
__device__ __forceinline__ int64_t f32_bits(float f) { return (int64_t)(uint32_t)__float_as_int(f); }
__device__ __forceinline__ int64_t f64_bits(double d) { return __double_as_longlong(d); }

__device__ __forceinline__ int64_t to_i64(const VmVal& v) {
    return v.t == SH_T_LONG ? v.b : (int64_t)(int32_t)v.b;  // only INT/LONG reach here
}
__device__ __forceinline__ float to_f32(const VmVal& v) {
    switch (v.t) {
        case SH_T_INT: return (float)(int32_t)v.b;
        case SH_T_LONG: return (float)v.b;
        case SH_T_FLOAT: return bits_f32(v.b);
        default: return (float)bits_f64(v.b);
    }
}
__device__ __forceinline__ double to_f64(const VmVal& v) {
    switch (v.t) {
        case SH_T_INT: return (double)(int32_t)v.b;
        case SH_T_LONG: return (double)v.b;
        case SH_T_FLOAT: return (double)bits_f32(v.b);
        default: return bits_f64(v.b);
    }
}

template <typename T>
__device__ __forceinline__ bool cmp_op(int op, T a, T b) {
    switch (op) {
        case SH_OP_EQ: return a == b;
        case SH_OP_NE: return a != b;
        case SH_OP_GT: return a > b;
        case SH_OP_GE: return a >= b;
        case SH_OP_LT: return a < b;
        default: return a <= b;
    }
}


// typed compare in a promotion domain (operands non-null)
__device__ __forceinline__ bool vm_cmp(int op, int dom, const VmVal& l, const VmVal& r) {
    switch (dom) {
        case DOM_I32: return cmp_op<int32_t>(op, (int32_t)l.b, (int32_t)r.b);
        case DOM_I64: return cmp_op<int64_t>(op, to_i64(l), to_i64(r));
        case DOM_F32: return cmp_op<float>(op, to_f32(l), to_f32(r));
        case DOM_F64: return cmp_op<double>(op, to_f64(l), to_f64(r));
        case DOM_BOOL: return cmp_op<int>(op, l.b != 0, r.b != 0);
        default: return cmp_op<int32_t>(op, (int32_t)l.b, (int32_t)r.b);
    }
}

// arithmetic in result type rt (math/{add,subtract,multiply,divide,mod}/*)
__device__ __forceinline__ VmVal vm_arith(int aop, int rt, const VmVal& l, const VmVal& r) {
    VmVal o;
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
        const uint64_t a = (uint64_t)to_i64(l), b = (uint64_t)to_i64(r);
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
        const float a = to_f32(l), b = to_f32(r);
        float res = 0.f;
        switch (aop) {
            case SH_OP_ADD: res = __fadd_rn(a, b); break;
            case SH_OP_SUB: res = __fsub_rn(a, b); break;
            case SH_OP_MUL: res = __fmul_rn(a, b); break;
            case SH_OP_DIV:
                if (b == 0.0f) o.null = 1;
                else res = __fdiv_rn(a, b);
                break;
            default:
                if (b == 0.0f) o.null = 1;
                else res = fmodf(a, b);
        }
        o.b = f32_bits(res);
    } else {
        const double a = to_f64(l), b = to_f64(r);
        double res = 0.0;
        switch (aop) {
            case SH_OP_ADD: res = __dadd_rn(a, b); break;
            case SH_OP_SUB: res = __dsub_rn(a, b); break;
            case SH_OP_MUL: res = __dmul_rn(a, b); break;
            case SH_OP_DIV:
                if (b == 0.0) o.null = 1;
                else res = __ddiv_rn(a, b);
                break;
            default:
                if (b == 0.0) o.null = 1;
                else res = fmod(a, b);
        }
        o.b = f64_bits(res);
    }
    return o;
}

__device__ __forceinline__ int64_t load_attr(const shd_cols* C, int s, int a, int type, uint32_t row) {
    const void* p = C->col[s][a];
    switch (type) {
        case SH_T_LONG: return ((const int64_t*)p)[row];
        case SH_T_FLOAT: return (int64_t)(uint32_t)((const uint32_t*)p)[row];
        case SH_T_DOUBLE: return ((const int64_t*)p)[row];
        case SH_T_BOOL: return ((const uint8_t*)p)[row] ? 1 : 0;
        default: return (int64_t)((const int32_t*)p)[row];
    }
}

// Evaluate `len` instructions at `pc`. rows[slot] = row of the slot's event
// (SHD_NULL_ROW when the slot is empty). Chains are length 1 for stream
// states, so chain index 0 / CURRENT address the event and anything else is null
// (StateEvent.getStreamEvent, StateEvent.java:138-182).
__device__ inline VmVal vm_eval(const shp_program* __restrict__ P, int pc, int len, const uint32_t* rows,
                         const shd_cols* __restrict__ C) {
    VmVal st[SHP_MAX_STACK];
    int sp = 0;
    for (int k = 0; k < len; k++) {
        const shp_instr in = P->code[pc + k];
        switch (in.op) {
            case OPC_CONST: {
                VmVal v;
                v.b = P->consts[in.x];
                v.t = P->const_type[in.x];
                v.null = P->const_null[in.x];
                st[sp++] = v;
                break;
            }
            case OPC_VAR: {
                VmVal v;
                v.t = in.c;
                const uint32_t row = rows[in.a];
                if (row == SHD_NULL_ROW || !(in.x == 0 || in.x == SH_CHAIN_CURRENT)) {
                    v.null = 1;
                    v.b = 0;
                } else {
                    const int s = P->state_stream[in.a];
                    const uint8_t* nm = C->nul[s][in.b];
                    v.null = nm ? nm[row] : 0;
                    v.b = load_attr(C, s, in.b, in.c, row);
                }
                st[sp++] = v;
                break;
            }
            case OPC_AND: {
                VmVal r = st[--sp], l = st[--sp];
                VmVal o;
                o.t = SH_T_BOOL;
                o.null = 0;
                o.b = (!l.null && l.b && !r.null && r.b) ? 1 : 0;
                st[sp++] = o;
                break;
            }
            case OPC_OR: {
                VmVal r = st[--sp], l = st[--sp];
                VmVal o;
                o.t = SH_T_BOOL;
                o.null = 0;
                o.b = ((!l.null && l.b) || (!r.null && r.b)) ? 1 : 0;
                st[sp++] = o;
                break;
            }
            case OPC_NOT: {
                VmVal l = st[--sp];
                VmVal o;
                o.t = SH_T_BOOL;
                o.null = 0;
                o.b = (!l.null && l.b) ? 0 : 1;  // Not(null) = true
                st[sp++] = o;
                break;
            }
            case OPC_BOOLV: {
                VmVal l = st[--sp];
                VmVal o;
                o.t = SH_T_BOOL;
                o.null = 0;
                o.b = (!l.null && l.b) ? 1 : 0;
                st[sp++] = o;
                break;
            }
            case OPC_ISNULL: {
                VmVal l = st[--sp];
                VmVal o;
                o.t = SH_T_BOOL;
                o.null = 0;
                o.b = l.null ? 1 : 0;
                st[sp++] = o;
                break;
            }
            case OPC_ISNULL_STREAM: {
                VmVal o;
                o.t = SH_T_BOOL;
                o.null = 0;
                o.b = (rows[in.a] == SHD_NULL_ROW || !(in.x == 0 || in.x == SH_CHAIN_CURRENT)) ? 1 : 0;
                st[sp++] = o;
                break;
            }
            case OPC_CMP: {
                VmVal r = st[--sp], l = st[--sp];
                VmVal o;
                o.t = SH_T_BOOL;
                o.null = 0;
                o.b = (!l.null && !r.null && vm_cmp(in.a, in.b, l, r)) ? 1 : 0;
                st[sp++] = o;
                break;
            }
            case OPC_ARITH: {
                VmVal r = st[--sp], l = st[--sp];
                st[sp++] = vm_arith(in.a, in.b, l, r);
                break;
            }
            case OPC_SELECT: {
                VmVal e = st[--sp], t = st[--sp], c = st[--sp];
                st[sp++] = (!c.null && c.b) ? t : e;
                break;
            }
            case OPC_CAST: {
                st[sp - 1].t = in.b;
                break;
            }
        }
    }
    return st[sp - 1];
}


// register-only filter: conjunction of shp_term over non-null columns
// (null masks are absent on this path; empty slots compare as null -> false)
__device__ __forceinline__ bool terms_pass(const shp_program* __restrict__ P, int k, const uint32_t* rows,
                                           const shd_cols* __restrict__ C) {
    const int nt = P->filter_nterms[k];
    for (int t = 0; t < nt; t++) {
        const shp_term T = P->terms[k][t];
        const uint32_t lr = rows[T.lslot];
        if (lr == SHD_NULL_ROW) return false;
        VmVal l, r;
        l.t = T.ltype;
        l.null = 0;
        l.b = load_attr(C, P->state_stream[T.lslot], T.lattr, T.ltype, lr);
        if (T.rkind == 1) {
            r.t = T.ctype;
            r.null = 0;
            r.b = T.c;
        } else {
            const uint32_t rr = rows[T.rslot];
            if (rr == SHD_NULL_ROW) return false;
            r.t = T.rtype;
            r.null = 0;
            r.b = load_attr(C, P->state_stream[T.rslot], T.rattr, T.rtype, rr);
            if (T.rkind == 2) {
                VmVal c;
                c.t = T.ctype;
                c.null = 0;
                c.b = T.c;
                r = vm_arith(T.aop, T.atype, r, c);
                if (r.null) return false;
            }
        }
        if (!vm_cmp(T.op, T.dom, l, r)) return false;
    }
    return true;
}

// filter of state k: register path when lowered and no column carries nulls
__device__ __forceinline__ bool filter_pass(const shp_program* __restrict__ P, int k, const uint32_t* rows,
                                            const shd_cols* __restrict__ C, bool fast_ok) {
    if (fast_ok && P->filter_fast[k]) return terms_pass(P, k, rows, C);
    if (P->filter_pc[k] < 0) return true;
    VmVal v = vm_eval(P, P->filter_pc[k], P->filter_len[k], rows, C);
    return !v.null && v.b;
}

// two-slot form for the window engine: rows live in two scalars (no local array,
// no scratch)
__device__ __forceinline__ bool terms_pass2(const shp_program* __restrict__ P, int k, uint32_t r0, uint32_t r1,
                                            const shd_cols* __restrict__ C) {
    const int nt = P->filter_nterms[k];
    for (int t = 0; t < nt; t++) {
        const shp_term T = P->terms[k][t];
        const uint32_t lr = T.lslot ? r1 : r0;
        if (lr == SHD_NULL_ROW) return false;
        VmVal l, r;
        l.t = T.ltype;
        l.null = 0;
        l.b = load_attr(C, P->state_stream[T.lslot], T.lattr, T.ltype, lr);
        if (T.rkind == 1) {
            r.t = T.ctype;
            r.null = 0;
            r.b = T.c;
        } else {
            const uint32_t rr = T.rslot ? r1 : r0;
            if (rr == SHD_NULL_ROW) return false;
            r.t = T.rtype;
            r.null = 0;
            r.b = load_attr(C, P->state_stream[T.rslot], T.rattr, T.rtype, rr);
            if (T.rkind == 2) {
                VmVal c;
                c.t = T.ctype;
                c.null = 0;
                c.b = T.c;
                r = vm_arith(T.aop, T.atype, r, c);
                if (r.null) return false;
            }
        }
        if (!vm_cmp(T.op, T.dom, l, r)) return false;
    }
    return true;
}

// Arrival-tile-major segments (shd_tiles): the events of a key are spread over
// the runs [dstart, dend) of that key in consecutive arrival tiles. A forward
// scan that leaves its run continues at the key's run in the next non-empty
// tile, a backward scan at the previous one; untiled segments keep one run per
// key and the scans stop at the key change.
struct TileDir {
    const uint32_t* ds;
    const uint32_t* de;
    uint32_t K1, ntile;
    int32_t shift;
    __device__ bool on() const { return ds != nullptr; }
    __device__ uint32_t tile(int64_t p) const { return (uint32_t)(p >> shift); }
    __device__ size_t at(uint32_t a, uint32_t key) const { return (size_t)a * K1 + key; }
    // next non-empty run of `key` after tile a (a advances); false when none
    __device__ bool next(uint32_t& a, uint32_t key, int64_t& q, int64_t& qend) const {
        while (++a < ntile) {
            const size_t e = at(a, key);
            const uint32_t s0 = ds[e], e0 = de[e];
            if (e0 > s0) {
                q = s0;
                qend = e0;
                return true;
            }
        }
        return false;
    }
    // previous non-empty run of `key` before tile a (a decreases); false when none
    __device__ bool prev(uint32_t& a, uint32_t key, int64_t& r, int64_t& rbeg) const {
        while (a > 0) {
            a--;
            const size_t e = at(a, key);
            const uint32_t s0 = ds[e], e0 = de[e];
            if (e0 > s0) {
                r = (int64_t)e0 - 1;
                rbeg = s0;
                return true;
            }
        }
        return false;
    }
};

__device__ __forceinline__ TileDir tile_dir(const shd_tiles& T) {
    TileDir d;
    d.ds = T.dstart;
    d.de = T.dend;
    d.K1 = T.K1;
    d.ntile = T.ntile;
    d.shift = T.shift;
    return d;
}

// position of the previous event of p's key (-1: none); the same-key
// predecessor check of the non-decreasing-timestamp premise
__device__ __forceinline__ int64_t key_pred(const TileDir& D, const uint32_t* __restrict__ skeys, int64_t p,
                                            uint32_t key) {
    if (D.on()) {
        uint32_t a = D.tile(p);
        if ((int64_t)D.ds[D.at(a, key)] < p) return p - 1;
        int64_t r, rb;
        return D.prev(a, key, r, rb) ? r : -1;
    }
    if (p == 0 || (skeys && skeys[p - 1] != key)) return -1;
    return p - 1;
}
