// sh_rules.hip — batch-compiled rule sets (config C5): R queries
//     every e1=S[f1_r] -> e2=S[f2_r(e1, e2)] within W_r          r = 0 .. R-1
// over one stream and one `partition with (key of S)` (or none), lowered
// together into one rule table (sh_rules.h) that shares a single radix segment.
//
// Every rule has the window-engine shape (sh_window.hip): with non-decreasing
// timestamps per key, rule r's partial opened at event p (f1_r) is consumed by
// the first later event q of the key with f2_r(p, q), unless ts_q - ts_p > W_r.
// Each query owns its processor state, so rules meet only in the output order:
// PartitionStreamReceiver.receive(Event[]) (core/partition/PartitionStreamReceiver.java:176-216)
// splits a send() call into runs of consecutive same-key events (a null-key event
// is dropped without ending the run) and sends each run to every query of the
// partition in subscription order, and a Multi receiver hands a run's matches to
// the callbacks after the whole run (core/query/input/MultiProcessStreamReceiver.java:95-122).
// A match is therefore ordered by (run, query, consuming event, opening event);
// an unpartitioned app sees each send() call as one run.
//
// Predicate index: the host picks the slot-0 attribute that the most start
// filters compare for equality with an integral / string / bool constant
// (`merchant == M_r`) and groups the rules by that constant; a lane
// binary-searches its event's value and evaluates only the rules of that group
// plus the rules without such a conjunct. Every conjunct is still evaluated, so
// the index only prunes.
//
// Pipeline (sh_host_fast.cpp run_rules): segment (sh_kernels.hip) -> k_rules_scan<0>
// (matches per opening event) -> exclusive scan -> k_rules_scan<1> (records in
// (opening event, rule) order) -> run ids -> k_rules_keys -> stable LSD radix
// sort of the records by (run, query, consuming event) -> k_rules_place.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstring>

#include "../../include/sh_query.h"
#include "sh_device.h"
#include "sh_rules.h"
#include "sh_vm.h"
#include "sh_wave.h"

#define RTPB 256
// a sorted timestamp: 32-bit offsets from tb when the run's range fits (s32), else int64
#define SHR_TS(i) (s32 ? tb + (int64_t)s32[(i)] : sts[(i)])
#define SHR_LDS_IX 2048  // index groups staged in LDS (24 KB)

static unsigned rgrid(int64_t n) {
    int64_t g = (n + RTPB - 1) / RTPB;
    if (g > 65536 * 8) g = 65536 * 8;
    return (unsigned)(g < 1 ? 1 : g);
}

// conjunction of register terms over the two slots (rows in key-segment order)
__device__ __forceinline__ bool rule_terms(const shp_term* __restrict__ T, int nt, uint32_t r0, uint32_t r1,
                                           const shd_cols* __restrict__ C) {
    for (int t = 0; t < nt; t++) {
        const shp_term X = T[t];
        const uint32_t lr = X.lslot ? r1 : r0;
        if (lr == SHD_NULL_ROW) return false;
        VmVal l, r;
        l.t = X.ltype;
        l.null = 0;
        l.b = load_attr(C, 0, X.lattr, X.ltype, lr);
        if (X.rkind == 1) {
            r.t = X.ctype;
            r.null = 0;
            r.b = X.c;
        } else {
            const uint32_t rr = X.rslot ? r1 : r0;
            if (rr == SHD_NULL_ROW) return false;
            r.t = X.rtype;
            r.null = 0;
            r.b = load_attr(C, 0, X.rattr, X.rtype, rr);
            if (X.rkind == 2) {
                VmVal c;
                c.t = X.ctype;
                c.null = 0;
                c.b = X.c;
                r = vm_arith(X.aop, X.atype, r, c);
                if (r.null) return false;
            }
        }
        if (!vm_cmp(X.op, X.dom, l, r)) return false;
    }
    return true;
}

// index key of an attribute value (the host keys the constants the same way)
__device__ __forceinline__ int64_t rule_ix_key(int type, int64_t raw) {
    if (type == SH_T_LONG) return raw;
    if (type == SH_T_BOOL) return raw != 0;
    return (int64_t)(int32_t)raw;
}

// WRITE = 0: matches opened at every key-segment position p -> cnt[p]
// WRITE = 1: the same scan, writing (p, q, rule) records from off[p] on
template <int WRITE>
__global__ void __launch_bounds__(RTPB) k_rules_scan(const shr_table* __restrict__ RT, const int64_t* __restrict__ sts,
                                                     const uint32_t* __restrict__ skeys, int64_t n, uint32_t sentinel,
                                                     const shd_cols* __restrict__ C, uint32_t* __restrict__ cnt,
                                                     const uint32_t* __restrict__ off, uint32_t* __restrict__ rec_p,
                                                     uint32_t* __restrict__ rec_q, uint32_t* __restrict__ rec_r,
                                                     int32_t* __restrict__ flag, const uint32_t* __restrict__ s32,
                                                     int64_t tb) {
    const int ix_attr = RT->ix_attr;
    const int n_ix = RT->n_ix;
    const uint32_t n_free = (uint32_t)RT->n_free;
    // the predicate index in LDS (a lane's binary search is a chain of dependent
    // loads: from LDS instead of L2); the grid is sized so each workgroup stages
    // it once for many events
    __shared__ int64_t s_ixv[SHR_LDS_IX];
    __shared__ uint32_t s_ixs[SHR_LDS_IX + 1];
    const bool lds_ix = ix_attr >= 0 && n_ix <= SHR_LDS_IX;
    if (lds_ix) {
        for (int i = threadIdx.x; i < n_ix; i += blockDim.x) s_ixv[i] = RT->ix_val[i];
        for (int i = threadIdx.x; i <= n_ix; i += blockDim.x) s_ixs[i] = RT->ix_start[i];
    }
    __syncthreads();
    for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < n; p += (int64_t)gridDim.x * blockDim.x) {
        if (WRITE && cnt[p] == 0) continue;
        const uint32_t key = skeys ? skeys[p] : 0u;
        if (key == sentinel) continue;
        const int64_t t0 = SHR_TS(p);
        if (!WRITE && p > 0 && (!skeys || skeys[p - 1] == key) && t0 < SHR_TS(p - 1)) atomicExch(flag, 1);
        uint32_t lo = 0, hi = 0;
        if (ix_attr >= 0) {
            const int ty = RT->attr_type[ix_attr];
            const int64_t x = rule_ix_key(ty, load_attr(C, 0, ix_attr, ty, (uint32_t)p));
            int a = 0, b = n_ix;
            if (lds_ix) {
                while (a < b) {
                    const int m = (a + b) >> 1;
                    if (s_ixv[m] < x)
                        a = m + 1;
                    else
                        b = m;
                }
                if (a < n_ix && s_ixv[a] == x) {
                    lo = s_ixs[a];
                    hi = s_ixs[a + 1];
                }
            } else {
                while (a < b) {
                    const int m = (a + b) >> 1;
                    if (RT->ix_val[m] < x)
                        a = m + 1;
                    else
                        b = m;
                }
                if (a < n_ix && RT->ix_val[a] == x) {
                    lo = RT->ix_start[a];
                    hi = RT->ix_start[a + 1];
                }
            }
        }
        const uint32_t nsel = hi - lo, total = nsel + n_free;
        uint32_t c = 0;
        const uint32_t o = WRITE ? off[p] : 0u;
        for (uint32_t k = 0; k < total; k++) {
            const uint32_t r = k < nsel ? RT->ix_rule[lo + k] : RT->free_rule[k - nsel];
            const shr_rule* R = RT->rules + r;
            if (!rule_terms(R->t[0], R->nt[0], (uint32_t)p, SHD_NULL_ROW, C)) continue;
            const int64_t W = R->within;
            for (int64_t q = p + 1; q < n; q++) {
                if (skeys && skeys[q] != key) break;
                const int64_t d = SHR_TS(q) - t0;
                if (W >= 0 && (d < 0 ? -d : d) > W) break;  // expired before event q is matched
                if (rule_terms(R->t[1], R->nt[1], (uint32_t)p, (uint32_t)q, C)) {
                    if (WRITE) {
                        rec_p[o + c] = (uint32_t)p;
                        rec_q[o + c] = (uint32_t)q;
                        rec_r[o + c] = r;
                    }
                    c++;
                    break;
                }
            }
        }
        if (!WRITE) cnt[p] = c;
    }
}

// the same scan over the rule set's LDS image (shr_img): the index search, the rule
// ids, every term and the stream's column pointers come from LDS, so a lane's chain
// of dependent reads (group -> rule -> terms -> column) stays on chip; one 1024-thread
// workgroup per CU strides over the events
#define RTPB_IMG 1024
__device__ __forceinline__ int64_t rule_attr(const void* const* cols, int a, int type, uint32_t row) {
    const void* p = cols[a];
    switch (type) {
        case SH_T_LONG:
        case SH_T_DOUBLE: return ((const int64_t*)p)[row];
        case SH_T_FLOAT: return (int64_t)(uint32_t)((const uint32_t*)p)[row];
        case SH_T_BOOL: return ((const uint8_t*)p)[row] ? 1 : 0;
        default: return (int64_t)((const int32_t*)p)[row];
    }
}

// the row's attributes a rule set's terms read most, loaded once per event: row
// `slot` (0: the opening event, 1: the consumer) of attribute a[0] / a[1] (-1: none)
struct RowPre {
    int slot;
    int a[2];
    int64_t v[2];
};
__device__ __forceinline__ int64_t rule_attr_pre(const void* const* cols, int a, int type, uint32_t row, int slot,
                                                 const RowPre& R) {
    if (slot == R.slot) {
        if (a == R.a[0]) return R.v[0];
        if (a == R.a[1]) return R.v[1];
    }
    return rule_attr(cols, a, type, row);
}

// terms as rule_terms_img, the preloaded attributes of one row from registers
__device__ __forceinline__ bool rule_terms_pre(const shp_term* T, int nt, uint32_t r0, uint32_t r1,
                                               const void* const* cols, const RowPre& R) {
    for (int t = 0; t < nt; t++) {
        const shp_term X = T[t];
        const uint32_t lr = X.lslot ? r1 : r0;
        if (lr == SHD_NULL_ROW) return false;
        VmVal l, r;
        l.t = X.ltype;
        l.null = 0;
        l.b = rule_attr_pre(cols, X.lattr, X.ltype, lr, X.lslot, R);
        // a float attribute against a double constant (Java compares as double): the
        // same compare without the generic value / domain dispatch
        if (X.rkind == 1 && X.dom == DOM_F64 && X.ltype == SH_T_FLOAT && X.ctype == SH_T_DOUBLE) {
            if (!cmp_op<double>(X.op, (double)__uint_as_float((uint32_t)l.b), __longlong_as_double(X.c))) return false;
            continue;
        }
        if (X.rkind == 1) {
            r.t = X.ctype;
            r.null = 0;
            r.b = X.c;
        } else {
            const uint32_t rr = X.rslot ? r1 : r0;
            if (rr == SHD_NULL_ROW) return false;
            r.t = X.rtype;
            r.null = 0;
            r.b = rule_attr_pre(cols, X.rattr, X.rtype, rr, X.rslot, R);
            if (X.rkind == 2) {
                VmVal c;
                c.t = X.ctype;
                c.null = 0;
                c.b = X.c;
                r = vm_arith(X.aop, X.atype, r, c);
                if (r.null) return false;
            }
        }
        if (!vm_cmp(X.op, X.dom, l, r)) return false;
    }
    return true;
}

__device__ __forceinline__ bool rule_terms_img(const shp_term* T, int nt, uint32_t r0, uint32_t r1,
                                               const void* const* cols) {
    for (int t = 0; t < nt; t++) {
        const shp_term X = T[t];
        const uint32_t lr = X.lslot ? r1 : r0;
        if (lr == SHD_NULL_ROW) return false;
        VmVal l, r;
        l.t = X.ltype;
        l.null = 0;
        l.b = rule_attr(cols, X.lattr, X.ltype, lr);
        if (X.rkind == 1) {
            r.t = X.ctype;
            r.null = 0;
            r.b = X.c;
        } else {
            const uint32_t rr = X.rslot ? r1 : r0;
            if (rr == SHD_NULL_ROW) return false;
            r.t = X.rtype;
            r.null = 0;
            r.b = rule_attr(cols, X.rattr, X.rtype, rr);
            if (X.rkind == 2) {
                VmVal c;
                c.t = X.ctype;
                c.null = 0;
                c.b = X.c;
                r = vm_arith(X.aop, X.atype, r, c);
                if (r.null) return false;
            }
        }
        if (!vm_cmp(X.op, X.dom, l, r)) return false;
    }
    return true;
}

// OCC2: the image fits two workgroups per CU, registers capped for 8 waves per SIMD
template <int WRITE, int OCC2>
__global__ void __launch_bounds__(RTPB_IMG) __attribute__((amdgpu_waves_per_eu(OCC2 ? 8 : 1))) k_rules_scan_img(
    const shr_table* __restrict__ RT, const int64_t* __restrict__ sts, const uint32_t* __restrict__ skeys, int64_t n,
    uint32_t sentinel, const shd_cols* __restrict__ C, uint32_t* __restrict__ cnt, const uint32_t* __restrict__ off,
    uint32_t* __restrict__ rec_p, uint32_t* __restrict__ rec_q, uint32_t* __restrict__ rec_r, int32_t* __restrict__ flag,
    const uint8_t* __restrict__ img, shr_img I, const uint32_t* __restrict__ s32, int64_t tb) {
    extern __shared__ uint4 s_img[];
    __shared__ const void* s_col[32];
    for (int i = threadIdx.x; i < I.lds / 16; i += blockDim.x) s_img[i] = ((const uint4*)img)[i];
    if (threadIdx.x < 32) s_col[threadIdx.x] = C->col[0][threadIdx.x];
    __syncthreads();
    const uint8_t* L = (const uint8_t*)s_img;
    const int64_t* ixv = (const int64_t*)(L + I.off_ixv);
    const uint32_t* ixs = (const uint32_t*)(L + I.off_ixs);
    const uint32_t* ixr = (const uint32_t*)(L + I.off_ixr);
    const uint32_t* fr = (const uint32_t*)(L + I.off_free);
    const shr_meta* meta = (const shr_meta*)(L + I.off_meta);
    const shp_term* terms1 = (const shp_term*)(L + I.off_terms1);           // LDS
    // f1's terms: in LDS when staged, else from the global image (I.lds stops before them)
    const shp_term* terms0 = (const shp_term*)((I.off_terms0 < I.lds ? L : img) + I.off_terms0);
    const int ix_attr = RT->ix_attr;
    const int n_ix = RT->n_ix;
    const uint32_t n_free = (uint32_t)RT->n_free;
    const int ix_ty = ix_attr >= 0 ? RT->attr_type[ix_attr] : 0;
    for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < n; p += (int64_t)gridDim.x * blockDim.x) {
        if (WRITE && cnt[p] == 0) continue;
        const uint32_t key = skeys ? skeys[p] : 0u;
        if (key == sentinel) continue;
        const int64_t t0 = SHR_TS(p);
        if (!WRITE && p > 0 && (!skeys || skeys[p - 1] == key) && t0 < SHR_TS(p - 1)) atomicExch(flag, 1);
        uint32_t lo = 0, hi = 0;
        if (ix_attr >= 0) {
            const int64_t x = rule_ix_key(ix_ty, rule_attr(s_col, ix_attr, ix_ty, (uint32_t)p));
            if (I.dense_n) {
                const int64_t dv = x - I.dense_min;
                if (dv >= 0 && dv < I.dense_n) {
                    const uint2 e = ((const uint2*)(L + I.off_dense))[dv];
                    lo = e.x;
                    hi = e.y;
                }
            } else {
                int a = 0, b = n_ix;
                while (a < b) {
                    const int m = (a + b) >> 1;
                    if (ixv[m] < x)
                        a = m + 1;
                    else
                        b = m;
                }
                if (a < n_ix && ixv[a] == x) {
                    lo = ixs[a];
                    hi = ixs[a + 1];
                }
            }
        }
        const uint32_t nsel = hi - lo, total = nsel + n_free;
        uint32_t c = 0;
        const uint32_t o = WRITE ? off[p] : 0u;
        for (uint32_t k = 0; k < total; k++) {
            const uint32_t r = k < nsel ? ixr[lo + k] : fr[k - nsel];
            const shr_meta M = meta[r];
            if (!rule_terms_img(terms0 + M.toff0, M.nt0, (uint32_t)p, SHD_NULL_ROW, s_col)) continue;
            const shp_term* T1 = terms1 + M.toff1;
            const int64_t W = M.within;
            for (int64_t q = p + 1; q < n; q++) {
                if (skeys && skeys[q] != key) break;
                const int64_t d = SHR_TS(q) - t0;
                if (W >= 0 && (d < 0 ? -d : d) > W) break;  // expired before event q is matched
                if (rule_terms_img(T1, M.nt1, (uint32_t)p, (uint32_t)q, s_col)) {
                    if (WRITE) {
                        rec_p[o + c] = (uint32_t)p;
                        rec_q[o + c] = (uint32_t)q;
                        rec_r[o + c] = r;
                    }
                    c++;
                    break;
                }
            }
        }
        if (!WRITE) cnt[p] = c;
    }
}

template <int WRITE>
static int rules_scan_img(const shr_table* dT, const int64_t* sts, const uint32_t* skeys, int64_t n, uint32_t sentinel,
                          const shd_cols* dC, uint32_t* cnt, const uint32_t* off, uint32_t* rec_p, uint32_t* rec_q,
                          uint32_t* rec_r, int32_t* flag, const uint8_t* img, const shr_img& I, hipStream_t st,
                          const uint32_t* s32, int64_t tb) {
    static int attr_set = 0;  // the dynamic LDS limit, raised once per instantiation
    if (!attr_set) {
        if (hipFuncSetAttribute(reinterpret_cast<const void*>(&k_rules_scan_img<WRITE, 0>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, SHR_IMG_MAX) != hipSuccess ||
            hipFuncSetAttribute(reinterpret_cast<const void*>(&k_rules_scan_img<WRITE, 1>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, SHR_IMG_MAX) != hipSuccess)
            return -3;
        attr_set = 1;
    }
    int64_t g = (n + RTPB_IMG - 1) / RTPB_IMG;
    const int per_cu = (160 * 1024) / (I.lds + 1024);
    const int64_t gmax = 256LL * (per_cu < 1 ? 1 : per_cu);
    if (g > gmax) g = gmax;
    if (g < 1) g = 1;
    static const bool occ_on = !(getenv("SH_RULES_OCC2") && getenv("SH_RULES_OCC2")[0] == '0');
    if (per_cu >= 2 && occ_on)
        hipLaunchKernelGGL((k_rules_scan_img<WRITE, 1>), dim3((unsigned)g), dim3(RTPB_IMG), (size_t)I.lds, st, dT, sts,
                           skeys, n, sentinel, dC, cnt, off, rec_p, rec_q, rec_r, flag, img, I, s32, tb);
    else
        hipLaunchKernelGGL((k_rules_scan_img<WRITE, 0>), dim3((unsigned)g), dim3(RTPB_IMG), (size_t)I.lds, st, dT, sts,
                           skeys, n, sentinel, dC, cnt, off, rec_p, rec_q, rec_r, flag, img, I, s32, tb);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

// start of a PartitionStreamReceiver run: the first keyed event of a send() call,
// or a keyed event whose key differs from the previous keyed event of the call
// (run_ids: the caller's runs, a new id starts a run)
__global__ void k_run_flags(const int32_t* __restrict__ akeys, const uint32_t* __restrict__ run_ids, int64_t n,
                            int64_t batch, uint32_t* __restrict__ flags) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int32_t k = akeys[i];
        uint32_t f = 0;
        if (k >= 0 && run_ids) {
            int64_t j = i - 1;
            while (j >= 0 && akeys[j] < 0) j--;
            f = (j < 0 || run_ids[j] != run_ids[i]) ? 1u : 0u;
        } else if (k >= 0) {
            const int64_t b0 = batch > 0 ? i - i % batch : 0;
            int64_t j = i - 1;
            while (j >= b0 && akeys[j] < 0) j--;
            f = (j < b0 || akeys[j] != k) ? 1u : 0u;
        }
        flags[i] = f;
    }
}

__global__ void k_run_first(const uint32_t* __restrict__ flags, const uint32_t* __restrict__ rid, int64_t n,
                            uint32_t* __restrict__ rfirst) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        if (flags[i]) rfirst[rid[i]] = (uint32_t)i;
}

#define SHR_WALK_MAX 512

__global__ void k_rules_keys(const uint32_t* __restrict__ rec_q, const uint32_t* __restrict__ rec_r, int64_t m,
                             const uint32_t* __restrict__ perm, const uint32_t* __restrict__ flags,
                             const uint32_t* __restrict__ rid, const uint32_t* __restrict__ rfirst, int64_t batch,
                             int qbits, int packed, uint32_t* __restrict__ k0, uint32_t* __restrict__ k1,
                             uint32_t* __restrict__ k2, const int32_t* __restrict__ akeys,
                             const uint32_t* __restrict__ run_ids, int32_t* __restrict__ long_run) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (int64_t)gridDim.x * blockDim.x) {
        const uint32_t q = rec_q[i];
        const uint32_t qa = perm ? perm[q] : q;
        uint32_t run, qoff;
        if (akeys) {
            // the consuming event's PartitionStreamReceiver run, found by walking back
            // from it (the run's first arrival index orders the runs like their ordinal):
            // a keyed event continues the run of the previous keyed event of its call
            // with the same key (or the same caller run id)
            const int32_t key = akeys[qa];
            const int64_t lb = run_ids ? 0 : (batch > 0 ? (int64_t)qa - (int64_t)qa % batch : 0);
            // bounded: a run longer than SHR_WALK_MAX events reports itself and the host
            // redoes the keys from the per-event run scan (no quadratic hot-key walk)
            int64_t first = qa;
            for (;;) {
                int64_t j = first - 1;
                while (j >= lb && akeys[j] < 0 && (int64_t)qa - j <= SHR_WALK_MAX) j--;
                if (j < lb) break;
                if ((int64_t)qa - j > SHR_WALK_MAX) {
                    *long_run = 1;
                    break;
                }
                if (run_ids ? run_ids[j] != run_ids[qa] : akeys[j] != key) break;
                first = j;
            }
            run = (uint32_t)first;
            qoff = qa - (uint32_t)first;
        } else if (flags) {
            run = rid[qa] + flags[qa] - 1u;
            qoff = qa - rfirst[run];
        } else if (batch > 0) {
            run = (uint32_t)(qa / batch);
            qoff = (uint32_t)(qa % batch);
        } else {
            run = 0;
            qoff = qa;
        }
        if (packed) {
            k0[i] = (rec_r[i] << qbits) | qoff;
            k1[i] = run;
        } else {
            k0[i] = qoff;
            k1[i] = rec_r[i];
            k2[i] = run;
        }
    }
}

__global__ void k_gather_key(const uint32_t* __restrict__ key, const uint32_t* __restrict__ order, int64_t m,
                             uint32_t* __restrict__ gk, uint32_t* __restrict__ gv) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (int64_t)gridDim.x * blockDim.x) {
        const uint32_t s = order ? order[i] : (uint32_t)i;
        gk[i] = key[s];
        gv[i] = s;
    }
}

// The records' order without a stage by opening event (records taken in any
// order, sh_sparse): after the stable passes by (run, rule, offset in run), a run
// of equal keys holds partials of one rule that one event consumed together;
// each such run is put in opening-event order (insertion sort by its first
// thread: the runs are short, one record almost always). Equal (run, rule,
// offset) with equal p would be one partial taken twice, so the order is total
// and equals the four-stage sort's.
__device__ __forceinline__ bool tie_eq(const uint32_t* __restrict__ k0, const uint32_t* __restrict__ k1,
                                       const uint32_t* __restrict__ k2, uint32_t a, uint32_t b) {
    return k0[a] == k0[b] && k1[a] == k1[b] && (!k2 || k2[a] == k2[b]);
}

__global__ void k_rules_ties(uint32_t* __restrict__ order, int64_t m, const uint32_t* __restrict__ k0,
                             const uint32_t* __restrict__ k1, const uint32_t* __restrict__ k2,
                             const uint32_t* __restrict__ rec_p) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i + 1 < m; i += (int64_t)gridDim.x * blockDim.x) {
        const uint32_t a = order[i];
        if (!tie_eq(k0, k1, k2, a, order[i + 1])) continue;
        if (i > 0 && tie_eq(k0, k1, k2, a, order[i - 1])) continue;  // not the run's first
        int64_t j = i + 1;
        while (j + 1 < m && tie_eq(k0, k1, k2, a, order[j + 1])) j++;
        // shell sort of order[i..j] by rec_p (gap 1 alone: insertion sort for the
        // usual run of 2-3; the gaps keep a hot key's long run near n log n)
        const int64_t g = j - i + 1;
        int64_t gap = 1;
        while (gap * 9 / 4 + 1 < g) gap = gap * 9 / 4 + 1;
        for (; gap >= 1; gap = gap == 1 ? 0 : (gap * 4) / 9) {
            for (int64_t x = i + gap; x <= j; x++) {
                const uint32_t v = order[x], pv = rec_p[v];
                int64_t y = x - gap;
                while (y >= i && rec_p[order[y]] > pv) {
                    order[y + gap] = order[y];
                    y -= gap;
                }
                order[y + gap] = v;
            }
        }
    }
}

extern "C" int shr_order_ties(uint32_t* order, int64_t m, const uint32_t* k0, const uint32_t* k1, const uint32_t* k2,
                              const uint32_t* rec_p, void* stream) {
    if (m < 2) return 0;
    hipLaunchKernelGGL(k_rules_ties, dim3(rgrid(m)), dim3(RTPB), 0, (hipStream_t)stream, order, m, k0, k1, k2, rec_p);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

__global__ void k_rules_place(const shr_table* __restrict__ RT, const uint32_t* __restrict__ order, int64_t m,
                              const uint32_t* __restrict__ rec_p, const uint32_t* __restrict__ rec_q,
                              const uint32_t* __restrict__ rec_r, const uint32_t* __restrict__ perm,
                              const int64_t* __restrict__ sts, const shd_cols* __restrict__ C, uint64_t seq_base,
                              int n_out, uint64_t* __restrict__ out_seq, int32_t* __restrict__ out_query,
                              int64_t* __restrict__ out_ts, int64_t* __restrict__ out_vals,
                              const uint32_t* __restrict__ s32, int64_t tb) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (int64_t)gridDim.x * blockDim.x) {
        const uint32_t id = order ? order[i] : (uint32_t)i;
        const uint32_t p = rec_p[id], q = rec_q[id];
        const shr_rule* R = RT->rules + rec_r[id];
        if (out_seq) out_seq[i] = seq_base + (perm ? perm[q] : q);
        if (out_query) out_query[i] = R->query;
        if (out_ts) out_ts[i] = SHR_TS(q);
        if (out_vals)
            for (int o = 0; o < n_out; o++) {
                int64_t v = 0;
                if (o < R->n_out) {
                    const int a = R->out_attr[o];
                    v = load_attr(C, 0, a, RT->attr_type[a], R->out_slot[o] ? q : p);
                }
                out_vals[i * n_out + o] = v;
            }
    }
}

static int rules_ok() { return hipGetLastError() == hipSuccess ? 0 : -3; }

// the scans' grid: a few workgroups per CU, each striding over many events (the
// LDS index is staged once per workgroup)
static unsigned sgrid(int64_t n) {
    const unsigned g = rgrid(n);
    return g < 1536u ? g : 1536u;  // 6 per CU (LDS)
}

extern "C" int shr_count(const shr_table* dT, const int64_t* sts, const uint32_t* skeys, int64_t n, uint32_t sentinel,
                         const shd_cols* dC, uint32_t* cnt, int32_t* flag, void* stream, const uint8_t* img,
                         const shr_img* I, const uint32_t* s32, int64_t tb) {
    if (img && I && I->bytes > 0)
        return rules_scan_img<0>(dT, sts, skeys, n, sentinel, dC, cnt, nullptr, nullptr, nullptr, nullptr, flag, img, *I,
                                 (hipStream_t)stream, s32, tb);
    hipLaunchKernelGGL(k_rules_scan<0>, dim3(sgrid(n)), dim3(RTPB), 0, (hipStream_t)stream, dT, sts, skeys, n,
                       sentinel, dC, cnt, (const uint32_t*)nullptr, (uint32_t*)nullptr, (uint32_t*)nullptr,
                       (uint32_t*)nullptr, flag, s32, tb);
    return rules_ok();
}

extern "C" int shr_write(const shr_table* dT, const int64_t* sts, const uint32_t* skeys, int64_t n, uint32_t sentinel,
                         const shd_cols* dC, const uint32_t* cnt, const uint32_t* off, uint32_t* rec_p,
                         uint32_t* rec_q, uint32_t* rec_r, void* stream, const uint8_t* img, const shr_img* I,
                         const uint32_t* s32, int64_t tb) {
    if (img && I && I->bytes > 0)
        return rules_scan_img<1>(dT, sts, skeys, n, sentinel, dC, (uint32_t*)cnt, off, rec_p, rec_q, rec_r, nullptr,
                                 img, *I, (hipStream_t)stream, s32, tb);
    hipLaunchKernelGGL(k_rules_scan<1>, dim3(sgrid(n)), dim3(RTPB), 0, (hipStream_t)stream, dT, sts, skeys, n,
                       sentinel, dC, (uint32_t*)cnt, off, rec_p, rec_q, rec_r, (int32_t*)nullptr, s32, tb);
    return rules_ok();
}

extern "C" int shr_run_ids(const int32_t* akeys, const uint32_t* run_ids, int64_t n, int64_t batch, uint32_t* flags,
                           uint32_t* rid, uint32_t* rfirst, uint32_t* scan_tmp, void* stream) {
    hipStream_t st = (hipStream_t)stream;
    hipLaunchKernelGGL(k_run_flags, dim3(rgrid(n)), dim3(RTPB), 0, st, akeys, run_ids, n, batch, flags);
    int rc = shd_exclusive_scan(flags, rid, n, scan_tmp, stream);
    if (rc) return rc;
    hipLaunchKernelGGL(k_run_first, dim3(rgrid(n)), dim3(RTPB), 0, st, (const uint32_t*)flags, (const uint32_t*)rid,
                       n, rfirst);
    return rules_ok();
}

extern "C" int shr_keys(const uint32_t* rec_q, const uint32_t* rec_r, int64_t m, const uint32_t* perm,
                        const uint32_t* flags, const uint32_t* rid, const uint32_t* rfirst, int64_t batch, int qbits,
                        int packed, uint32_t* k0, uint32_t* k1, uint32_t* k2, void* stream, const int32_t* akeys,
                        const uint32_t* run_ids, int32_t* long_run) {
    if (akeys && !long_run) return 1;
    hipLaunchKernelGGL(k_rules_keys, dim3(rgrid(m)), dim3(RTPB), 0, (hipStream_t)stream, rec_q, rec_r, m, perm, flags,
                       rid, rfirst, batch, qbits, packed, k0, k1, k2, akeys, run_ids, long_run);
    return rules_ok();
}

extern "C" int shr_gather(const uint32_t* key, const uint32_t* order, int64_t m, uint32_t* gk, uint32_t* gv,
                          void* stream) {
    hipLaunchKernelGGL(k_gather_key, dim3(rgrid(m)), dim3(RTPB), 0, (hipStream_t)stream, key, order, m, gk, gv);
    return rules_ok();
}

extern "C" int shr_place(const shr_table* dT, const uint32_t* order, int64_t m, const uint32_t* rec_p,
                         const uint32_t* rec_q, const uint32_t* rec_r, const uint32_t* perm, const int64_t* sts,
                         const shd_cols* dC, uint64_t seq_base, int n_out, uint64_t* out_seq, int32_t* out_query,
                         int64_t* out_ts, int64_t* out_vals, void* stream, const uint32_t* s32, int64_t tb) {
    hipLaunchKernelGGL(k_rules_place, dim3(rgrid(m)), dim3(RTPB), 0, (hipStream_t)stream, dT, order, m, rec_p, rec_q,
                       rec_r, perm, sts, dC, seq_base, n_out, out_seq, out_query, out_ts, out_vals, s32, tb);
    return rules_ok();
}

// the timestamps' range (min, max) of a run, for the 32-bit offsets
__global__ void __launch_bounds__(256) k_ts_range(const int64_t* __restrict__ ts, int64_t n,
                                                  unsigned long long* __restrict__ mm) {
    int64_t lo = INT64_MAX, hi = INT64_MIN;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t t = ts[i];
        lo = t < lo ? t : lo;
        hi = t > hi ? t : hi;
    }
    for (int o = 32; o > 0; o >>= 1) {
        const int64_t l2 = __shfl_xor(lo, o), h2 = __shfl_xor(hi, o);
        lo = l2 < lo ? l2 : lo;
        hi = h2 > hi ? h2 : hi;
    }
    // order-preserving unsigned form of the signed values
    if ((threadIdx.x & 63) == 0) {
        atomicMin(&mm[0], (unsigned long long)lo ^ 0x8000000000000000ull);
        atomicMax(&mm[1], (unsigned long long)hi ^ 0x8000000000000000ull);
    }
}

__global__ void __launch_bounds__(256) k_ts_to32(const int64_t* __restrict__ ts, int64_t n, int64_t base,
                                                 uint32_t* __restrict__ t32) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        t32[i] = (uint32_t)(ts[i] - base);
}

extern "C" int shr_ts_range(const int64_t* ts, int64_t n, int64_t* lo, int64_t* hi, void* scratch, void* stream) {
    hipStream_t st = (hipStream_t)stream;
    unsigned long long init[2] = {~0ull, 0ull};
    hipMemcpyAsync(scratch, init, 16, hipMemcpyHostToDevice, st);
    const unsigned g = n > 0 ? (unsigned)std::min<int64_t>((n + 255) / 256, 4096) : 1u;
    hipLaunchKernelGGL(k_ts_range, dim3(g), dim3(256), 0, st, ts, n, (unsigned long long*)scratch);
    unsigned long long out[2];
    hipMemcpyAsync(out, scratch, 16, hipMemcpyDeviceToHost, st);
    if (hipStreamSynchronize(st) != hipSuccess) return -3;
    *lo = (int64_t)(out[0] ^ 0x8000000000000000ull);
    *hi = (int64_t)(out[1] ^ 0x8000000000000000ull);
    return 0;
}

extern "C" int shr_ts_to32(const int64_t* ts, int64_t n, int64_t base, uint32_t* t32, void* stream) {
    if (n <= 0) return 0;
    hipLaunchKernelGGL(k_ts_to32, dim3((unsigned)std::min<int64_t>((n + 255) / 256, 65536)), dim3(256), 0,
                       (hipStream_t)stream, ts, n, base, t32);
    return rules_ok();
}

// ---------------------------------------------------------------- sparse partials
// The same matches without a key segment, for partitioned rule sets whose start
// filters open few partials (C5: `amount > A and merchant == M` holds for ~2% of
// the events). Every partial (p, r) is independent -- it is consumed by the first
// later event q of its key with |ts_q - ts_p| <= W_r and f2_r(p, q) -- so with
// non-decreasing timestamps (checked over the whole run) the consuming event is
// the least such q:
//   k_sparse_open: per event (arrival order) the index lookup of its candidate
//     rules, the round's (event, rule) pairs expanded in LDS, f1 per pair (one
//     lane each) -> the partials (p, r), appended through an LDS buffer per wave,
//     and per key a count (the partial's slot in its key's list);
//   scan of the per-key counts -> each key's list;
//   k_sparse_place: the partials into their keys' lists, with their expiry time;
//   k_sparse_take: per event q, its key's partials opened before it that are not
//     expired at ts_q and whose f2 holds -> atomicMin of q into the partial;
//   k_sparse_rec: the taken partials -> (p, q, r) records (any order: the host
//     sorts them by p first, which restores the (opening event, rule) order the
//     record sort's stability relies on).
// A run whose timestamps decrease, whose keys leave [0, nkeys), or whose partials
// overflow the buffers (the host reads the count) sets a flag: the host runs the
// key-segment path instead.
#define SPA_TPB 1024
#define SPA_BUF 1024
#define SPA_F_TS 1
#define SPA_F_KEY 2

// the predicate-index group of value x of the indexed attribute: [lo, hi) of ix_rule
__device__ __forceinline__ void spa_group(const shr_table* __restrict__ RT, const uint8_t* __restrict__ img,
                                          const shr_img& I, int64_t x, uint32_t* lo, uint32_t* hi) {
    *lo = *hi = 0;
    if (img && I.dense_n) {
        const int64_t dv = x - I.dense_min;
        if (dv >= 0 && dv < I.dense_n) {
            const uint2 e = ((const uint2*)(img + I.off_dense))[dv];
            *lo = e.x;
            *hi = e.y;
        }
        return;
    }
    const int n_ix = RT->n_ix;
    int a = 0, b = n_ix;
    while (a < b) {
        const int m = (a + b) >> 1;
        if (RT->ix_val[m] < x)
            a = m + 1;
        else
            b = m;
    }
    if (a < n_ix && RT->ix_val[a] == x) {
        *lo = RT->ix_start[a];
        *hi = RT->ix_start[a + 1];
    }
}

#define SPA_U 4  // events per thread and round, their loads issued together

// the rule set as the sparse kernels read it: the LDS image (IMG, shr_img: the
// index, rule ids, windows and terms on chip, like k_rules_scan_img) or the table
// in global memory
struct SpaRules {
    const uint8_t* L;          // LDS image
    const uint8_t* G;          // the whole image (global): f1's terms past I.lds
    const void* const* cols;   // stream-0 column pointers (LDS)
};

template <bool IMG>
__device__ __forceinline__ void spa_stage(const uint8_t* __restrict__ img, const shr_img& I,
                                          const shd_cols* __restrict__ C, uint4* s_img, const void** s_col) {
    if (IMG)
        for (int i = threadIdx.x; i < I.lds / 16; i += blockDim.x) s_img[i] = ((const uint4*)img)[i];
    if (threadIdx.x < 32) s_col[threadIdx.x] = C->col[0][threadIdx.x];
}

// open's image: everything but f2's terms (the host's descriptor for it has f1's
// terms moved down over them: off_terms1 <= off_terms0 and the bytes between the
// image's f2 terms and f1 terms skipped -- I.pad below)
template <bool IMG>
__device__ __forceinline__ void spa_stage_open(const uint8_t* __restrict__ img, const shr_img& I,
                                               const shd_cols* __restrict__ C, uint4* s_img, const void** s_col) {
    if (IMG) {
        const int cut = I.off_terms1 / 16, skip = I.pad / 16;  // (pad: the f2 terms' bytes, a multiple of 16)
        for (int i = threadIdx.x; i < I.lds / 16; i += blockDim.x)
            s_img[i] = ((const uint4*)img)[i < cut ? i : i + skip];
    }
    if (threadIdx.x < 32) s_col[threadIdx.x] = C->col[0][threadIdx.x];
}

// candidate rule group of an index value: [lo, hi) of the rule ids
template <bool IMG>
__device__ __forceinline__ void spa_candidates(const shr_table* __restrict__ RT, const shr_img& I, const SpaRules& S,
                                               const uint8_t* __restrict__ img, int64_t x, uint32_t* lo,
                                               uint32_t* hi) {
    if (!IMG) {
        spa_group(RT, img, I, x, lo, hi);
        return;
    }
    *lo = *hi = 0;
    if (I.dense_n) {
        const int64_t dv = x - I.dense_min;
        if (dv >= 0 && dv < I.dense_n) {
            const uint2 e = ((const uint2*)(S.L + I.off_dense))[dv];
            *lo = e.x;
            *hi = e.y;
        }
        return;
    }
    const int64_t* ixv = (const int64_t*)(S.L + I.off_ixv);
    const uint32_t* ixs = (const uint32_t*)(S.L + I.off_ixs);
    const int n_ix = RT->n_ix;
    int a = 0, b = n_ix;
    while (a < b) {
        const int m = (a + b) >> 1;
        if (ixv[m] < x)
            a = m + 1;
        else
            b = m;
    }
    if (a < n_ix && ixv[a] == x) {
        *lo = ixs[a];
        *hi = ixs[a + 1];
    }
}

template <bool IMG>
__device__ __forceinline__ uint32_t spa_rule_id(const shr_table* __restrict__ RT, const shr_img& I, const SpaRules& S,
                                                uint32_t lo, uint32_t k, uint32_t nsel) {
    if (IMG)
        return k < nsel ? ((const uint32_t*)(S.L + I.off_ixr))[lo + k] : ((const uint32_t*)(S.L + I.off_free))[k - nsel];
    return k < nsel ? RT->ix_rule[lo + k] : RT->free_rule[k - nsel];
}

// f1 of rule r on row p
template <bool IMG>
__device__ __forceinline__ bool spa_f1(const shr_table* __restrict__ RT, const shr_img& I, const SpaRules& S,
                                       const shd_cols* __restrict__ C, uint32_t r, uint32_t p, const RowPre& RP) {
    if (IMG) {
        const shr_meta M = ((const shr_meta*)(S.L + I.off_meta))[r];
        const shp_term* T0 = (const shp_term*)((I.off_terms0 < I.lds ? S.L : S.G) + I.off_terms0) + M.toff0;
        return rule_terms_pre(T0, M.nt0, p, SHD_NULL_ROW, S.cols, RP);
    }
    const shr_rule* R = RT->rules + r;
    return rule_terms(R->t[0], R->nt[0], p, SHD_NULL_ROW, C);
}

// f2 of rule r on (p, q)
template <bool IMG>
__device__ __forceinline__ bool spa_f2(const shr_table* __restrict__ RT, const shr_img& I, const SpaRules& S,
                                       const shd_cols* __restrict__ C, uint32_t r, uint32_t p, uint32_t q,
                                       const RowPre& RP) {
    if (IMG) {
        const shr_meta M = ((const shr_meta*)(S.L + I.off_meta))[r];
        return rule_terms_pre((const shp_term*)(S.L + I.off_terms1) + M.toff1, M.nt1, p, q, S.cols, RP);
    }
    const shr_rule* R = RT->rules + r;
    return rule_terms(R->t[1], R->nt[1], p, q, C);
}

#define SPA_WBUF 192  // partials a wave holds before it appends them (one global atomic per flush)
// (event, candidate rule) pairs of a round expanded in LDS, at most: 1.5 per event
#define SPO_TPB 512  // k_sparse_open's workgroup
template <int TPB>
struct SpaOpen {
    static constexpr int PAIRS = TPB * SPA_U * 3 / 2;
    static constexpr int WBUF = TPB >= 1024 ? SPA_WBUF : 128;
    static constexpr int LDS = 3 * (TPB / 64) * WBUF * 4 + PAIRS * 4 + 512;  // static arrays, bytes (about)
};

template <bool IMG, int OTPB>
__global__ void __launch_bounds__(OTPB) k_sparse_open(const shr_table* __restrict__ RT,
                                                         const int64_t* __restrict__ ts,
                                                         const int32_t* __restrict__ akeys, int64_t n, int32_t nkeys,
                                                         const shd_cols* __restrict__ C,
                                                         const uint8_t* __restrict__ img, shr_img I,
                                                         uint32_t* __restrict__ pr_p, uint32_t* __restrict__ pr_r,
                                                         uint32_t* __restrict__ pr_key, uint32_t* __restrict__ key_cnt,
                                                         unsigned long long* __restrict__ ctr, int64_t cap,
                                                         int32_t* __restrict__ flag, int pa0, int pa1) {
    extern __shared__ uint4 s_img[];
    __shared__ const void* s_col[32];
    // per wave: its pending partials (opening event, rule, key) and their count --
    // waves run independently, no block barrier after the image is staged
    __shared__ uint32_t w_p[OTPB / 64][SpaOpen<OTPB>::WBUF], w_r[OTPB / 64][SpaOpen<OTPB>::WBUF],
        w_k[OTPB / 64][SpaOpen<OTPB>::WBUF];
    __shared__ uint32_t w_fill[OTPB / 64];
    // a round's (event, candidate rule) pairs: rule << 12 | the event's index in the round
    __shared__ uint32_t s_pair[SpaOpen<OTPB>::PAIRS];
    constexpr int SPA_PAIRS = SpaOpen<OTPB>::PAIRS;
    constexpr int SPA_WBUF_ = SpaOpen<OTPB>::WBUF;
    __shared__ uint32_t s_ws[OTPB / 64];
    static_assert(OTPB * SPA_U <= 4096, "12-bit event index in a pair");
    spa_stage_open<IMG>(img, I, C, s_img, s_col);
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
    if (lane == 0) w_fill[wv] = 0u;
    const SpaRules S{(const uint8_t*)s_img, img, s_col};
    const uint32_t n_free = (uint32_t)RT->n_free;
    const int ix_attr = RT->ix_attr;
    const int ix_ty = ix_attr >= 0 ? RT->attr_type[ix_attr] : 0;
    int32_t fl = 0;
    __syncthreads();
    const void* ix_col = ix_attr >= 0 ? s_col[ix_attr] : nullptr;
    // a wave's partials to global: one atomic for the run, then coalesced stores
    auto flush = [&](uint32_t fill) {
        unsigned long long g0 = 0;
        if (lane == 0) g0 = atomicAdd(ctr, (unsigned long long)fill);
        g0 = __shfl(g0, 0);
        for (uint32_t i = lane; i < fill; i += 64) {
            const int64_t g = (int64_t)g0 + i;
            if (g < cap) {
                pr_p[g] = w_p[wv][i];
                pr_r[g] = w_r[wv][i];
                pr_key[g] = w_k[wv][i];
            }
        }
    };
    const int64_t round = (int64_t)OTPB * SPA_U;
    for (int64_t base = (int64_t)blockIdx.x * round; base < n; base += (int64_t)gridDim.x * round) {
        // SPA_U runs of the workgroup's events: ts, key, index value
        int64_t tv[SPA_U], tp[SPA_U];
        int32_t key[SPA_U];
        int64_t xv[SPA_U];
#pragma unroll
        for (int u = 0; u < SPA_U; u++) {
            const int64_t p = base + (int64_t)u * OTPB + threadIdx.x;
            const bool in = p < n;
            tv[u] = in ? ts[p] : 0;
            tp[u] = in && p > 0 ? ts[p - 1] : INT64_MIN;
            key[u] = in ? akeys[p] : -1;
            xv[u] = (in && ix_col) ? rule_ix_key(ix_ty, rule_attr(s_col, ix_attr, ix_ty, (uint32_t)p)) : 0;
        }
        uint32_t lo[SPA_U], hi[SPA_U];
#pragma unroll
        for (int u = 0; u < SPA_U; u++) {
            if (tv[u] < tp[u]) fl |= SPA_F_TS;
            if (key[u] >= nkeys) fl |= SPA_F_KEY;
            lo[u] = hi[u] = 0;
            if (ix_col && key[u] >= 0 && key[u] < nkeys) spa_candidates<IMG>(RT, I, S, img, xv[u], &lo[u], &hi[u]);
        }
        // the pairs of the round, expanded in LDS so that each lane evaluates f1 for
        // one (event, rule) pair: no wave waits for its event with the most candidate
        // rules (C5: ~1 candidate per event, ~5 for a wave's busiest). A round with
        // more pairs than fit expands them in batches of SPA_PAIRS.
        uint32_t tc = 0u;
#pragma unroll
        for (int u = 0; u < SPA_U; u++)
            tc += (key[u] >= 0 && key[u] < nkeys) ? hi[u] - lo[u] + n_free : 0u;
        uint32_t np_;
        const uint32_t at0 = shw_block_excl<OTPB>(tc, s_ws, &np_);
        for (uint32_t b0 = 0; b0 < np_; b0 += SPA_PAIRS) {
            const uint32_t b1 = b0 + SPA_PAIRS;
            uint32_t at = at0;
#pragma unroll
            for (int u = 0; u < SPA_U; u++) {
                const bool live = key[u] >= 0 && key[u] < nkeys;
                const uint32_t total = live ? hi[u] - lo[u] + n_free : 0u;
                const uint32_t nsel = hi[u] - lo[u];
                for (uint32_t k = 0; k < total; k++, at++)
                    if (at >= b0 && at < b1)
                        s_pair[at - b0] = (spa_rule_id<IMG>(RT, I, S, lo[u], k, nsel) << 12) |
                                          (uint32_t)(u * OTPB + (int)threadIdx.x);
            }
            __syncthreads();
            const uint32_t nb = min(np_ - b0, (uint32_t)SPA_PAIRS);
            for (uint32_t q0 = 0; q0 < nb; q0 += OTPB) {
                const uint32_t q = q0 + threadIdx.x;
                bool ok = false;
                uint32_t r = 0u, pp = 0u;
                int32_t kk = 0;
                if (q < nb) {
                    const uint32_t w = s_pair[q];
                    r = w >> 12;
                    pp = (uint32_t)(base + (int64_t)(w & 4095u));
                    // f1's most read attributes of the event (IMG: the terms come from LDS)
                    RowPre rq;
                    rq.slot = 0;
                    rq.a[0] = pa0;
                    rq.a[1] = pa1;
                    rq.v[0] = pa0 >= 0 ? rule_attr(s_col, pa0, RT->attr_type[pa0], pp) : 0;
                    rq.v[1] = pa1 >= 0 ? rule_attr(s_col, pa1, RT->attr_type[pa1], pp) : 0;
                    kk = akeys[pp];
                    ok = spa_f1<IMG>(RT, I, S, C, r, pp, rq);
                }
                const uint64_t m = __ballot(ok);
                if (m == 0ull) continue;
                const uint32_t fill = w_fill[wv];
                const uint32_t wat = fill + (uint32_t)__popcll(m & lt);
                if (ok) {
                    atomicAdd(&key_cnt[kk], 1u);  // (no return: the slot is taken at placement)
                    if (wat < SPA_WBUF_) {
                        w_p[wv][wat] = pp;
                        w_r[wv][wat] = r;
                        w_k[wv][wat] = (uint32_t)kk;
                    } else {
                        const unsigned long long g = atomicAdd(ctr, 1ull);  // (buffer full: straight out)
                        if ((int64_t)g < cap) {
                            pr_p[g] = pp;
                            pr_r[g] = r;
                            pr_key[g] = (uint32_t)kk;
                        }
                    }
                }
                const uint32_t nf = min(fill + (uint32_t)__popcll(m), (uint32_t)SPA_WBUF_);
                if (lane == 0) w_fill[wv] = nf;
                if (nf > SPA_WBUF_ - 64) {
                    flush(nf);
                    if (lane == 0) w_fill[wv] = 0u;
                }
            }
            __syncthreads();  // (the next batch or round rewrites the pairs)
        }
    }
    {
        const uint32_t fill = w_fill[wv];
        if (fill) flush(fill);
    }
    if (fl) atomicOr(flag, fl);
}

__global__ void k_sparse_place(const uint32_t* __restrict__ pr_p, const uint32_t* __restrict__ pr_r,
                               const uint32_t* __restrict__ pr_key, uint32_t* __restrict__ key_fill,
                               const unsigned long long* __restrict__ ctr, const uint32_t* __restrict__ key_off,
                               const shr_table* __restrict__ RT, const int64_t* __restrict__ ts,
                               uint32_t* __restrict__ l_p, uint32_t* __restrict__ l_r, int64_t* __restrict__ l_te,
                               uint32_t* __restrict__ l_q, shr_live LV) {
    const int64_t np = (int64_t)*ctr;
    for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s < np; s += (int64_t)gridDim.x * blockDim.x) {
        const uint32_t p = pr_p[s], r = pr_r[s], key = pr_key[s];  // (np <= the buffers: the host checked the count)
        const uint32_t pos = key_off[key] + atomicAdd(&key_fill[key], 1u);  // (any order inside a key's list)
        const int64_t W = RT->rules[r].within;
        const int64_t t = ts[p];
        const int64_t te = (W < 0 || t > INT64_MAX - W) ? INT64_MAX : t + W;
        l_p[pos] = p;
        l_r[pos] = r;
        l_te[pos] = te;
        l_q[pos] = 0xFFFFFFFFu;
        if (LV.bits) {
            // the slices in which an event can consume it: from its own to its expiry's
            // (the run's timestamps lie in [tmin, tmin + nslices << shift))
            const int64_t s0 = (t - LV.tmin) >> LV.shift;
            const int64_t tend = LV.tmin + ((int64_t)LV.nslices << LV.shift);  // (no overflow: te may be INT64_MAX)
            const int64_t s1 = te >= tend ? LV.nslices - 1 : (te - LV.tmin) >> LV.shift;
            for (int64_t sl = s0; sl <= s1; sl++)
                atomicOr(&LV.bits[sl * LV.wps + (key >> 5)], 1u << (key & 31u));
        }
    }
}

#define SPA_TQ 256  // (event, list entry) pairs a wave queues at a time (k_sparse_take)
template <bool IMG>
__global__ void __launch_bounds__(SPA_TPB) k_sparse_take(const shr_table* __restrict__ RT,
                                                         const int64_t* __restrict__ ts,
                                                         const int32_t* __restrict__ akeys, int64_t n,
                                                         const shd_cols* __restrict__ C,
                                                         const uint8_t* __restrict__ img, shr_img I,
                                                         const uint32_t* __restrict__ key_off,
                                                         const uint32_t* __restrict__ l_p,
                                                         const uint32_t* __restrict__ l_r,
                                                         const int64_t* __restrict__ l_te, uint32_t* __restrict__ l_q,
                                                         shr_live LV, int pa0, int pa1) {
    extern __shared__ uint4 s_img[];
    __shared__ const void* s_col[32];
    __shared__ uint32_t s_tq[SPA_TPB / 64][SPA_TQ], s_tp[SPA_TPB / 64][SPA_TQ];
    spa_stage<IMG>(img, I, C, s_img, s_col);
    __syncthreads();
    const SpaRules S{(const uint8_t*)s_img, img, s_col};
    constexpr int TPB = SPA_TPB;
    const int lane = (int)(threadIdx.x & 63u), wv = (int)(threadIdx.x >> 6);
    const int64_t wb = (int64_t)blockIdx.x, nw = (int64_t)gridDim.x;
    // SPA_U events per thread and round: their key, list bounds and first list
    // entry are loaded together (three dependent random reads per event otherwise)
    const int64_t round = (int64_t)TPB * SPA_U;
    for (int64_t base = wb * round; base < n; base += nw * round) {
        int32_t key[SPA_U];
        int64_t tq[SPA_U];
#pragma unroll
        for (int u = 0; u < SPA_U; u++) {
            const int64_t q = base + (int64_t)u * TPB + threadIdx.x;
            // streaming loads: they do not displace the live bitmap's lines from L2
            // (profiles/r6_c5_take_nt_ab.txt: advance 2.72 -> 2.65 ms)
            key[u] = q < n ? __builtin_nontemporal_load(akeys + q) : -1;
            tq[u] = q < n ? __builtin_nontemporal_load(ts + q) : 0;
        }
        // the live bitmap: an event whose key has no partial that can be consumed in
        // its time slice reads nothing else (a 128 KB slice of bits per 1M keys, in L2)
        if (LV.bits) {
            uint32_t wbits[SPA_U];
#pragma unroll
            for (int u = 0; u < SPA_U; u++) {
                wbits[u] = 0u;
                if (key[u] >= 0) {
                    const int64_t sl = (tq[u] - LV.tmin) >> LV.shift;
                    wbits[u] = LV.bits[sl * LV.wps + ((uint32_t)key[u] >> 5)];
                }
            }
#pragma unroll
            for (int u = 0; u < SPA_U; u++)
                if (key[u] >= 0 && !((wbits[u] >> ((uint32_t)key[u] & 31u)) & 1u)) key[u] = -1;
        }
        uint32_t lo[SPA_U], hi[SPA_U];
#pragma unroll
        for (int u = 0; u < SPA_U; u++) {
            lo[u] = hi[u] = 0;
            if (key[u] >= 0) {
                lo[u] = key_off[key[u]];
                hi[u] = key_off[key[u] + 1];
            }
        }
        // the wave's (event, list entry) pairs of the round into its LDS queue, then one
        // lane per pair: the few events whose key has live partials (~1% on C5) pay the
        // list's dependent reads once per round together, not once per event slot u
        // (C5 advance 2.43 -> 1.61 ms, profiles/r6_c5_take_queue_ab.txt)
        uint32_t off[SPA_U], wtot = 0;
#pragma unroll
        for (int u = 0; u < SPA_U; u++) {
            const uint32_t c = hi[u] - lo[u];
            const uint32_t incl = shw_incl_scan(c);
            off[u] = wtot + incl - c;
            wtot += shw_last(incl);
        }
        for (uint32_t b0 = 0; b0 < wtot; b0 += SPA_TQ) {  // (uniform in the wave)
#pragma unroll
            for (int u = 0; u < SPA_U; u++) {
                // this batch's part of the slot's list only (a hot key's long list costs
                // its length once over all batches, not once per batch)
                const uint32_t q = (uint32_t)(base + (int64_t)u * TPB + threadIdx.x);
                const uint32_t c = hi[u] - lo[u];
                const uint32_t k0 = b0 > off[u] ? b0 - off[u] : 0u;
                const uint32_t e = b0 + SPA_TQ > off[u] ? b0 + SPA_TQ - off[u] : 0u;
                const uint32_t k1 = e < c ? e : c;
                for (uint32_t k = k0; k < k1; k++) {
                    const uint32_t at = off[u] + k;
                    s_tq[wv][at - b0] = q;
                    s_tp[wv][at - b0] = lo[u] + k;
                }
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            const uint32_t nb = wtot - b0 < SPA_TQ ? wtot - b0 : SPA_TQ;
            for (uint32_t j = lane; j < nb; j += 64) {
                const uint32_t q = s_tq[wv][j], pos = s_tp[wv][j];
                const uint32_t p = l_p[pos], r = l_r[pos];
                const int64_t te = l_te[pos], tqq = ts[q];
                if (p >= q || tqq > te) continue;
                RowPre rp;
                rp.slot = 1;
                rp.a[0] = pa0;
                rp.a[1] = pa1;
                rp.v[0] = pa0 >= 0 ? rule_attr(S.cols, pa0, RT->attr_type[pa0], q) : 0;
                rp.v[1] = pa1 >= 0 ? rule_attr(S.cols, pa1, RT->attr_type[pa1], q) : 0;
                if (spa_f2<IMG>(RT, I, S, C, r, p, q, rp)) atomicMin(&l_q[pos], q);
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
    }
}

__global__ void __launch_bounds__(256) k_sparse_rec(const uint32_t* __restrict__ l_p,
                                                    const uint32_t* __restrict__ l_r,
                                                    const uint32_t* __restrict__ l_q,
                                                    const unsigned long long* __restrict__ ctr,
                                                    uint32_t* __restrict__ rec_p, uint32_t* __restrict__ rec_q,
                                                    uint32_t* __restrict__ rec_r, unsigned long long* __restrict__ rctr,
                                                    int64_t rcap) {
    const int64_t np = (int64_t)*ctr;
    const int lane = threadIdx.x & 63;
    const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
    for (int64_t s0 = (int64_t)blockIdx.x * blockDim.x; s0 < np; s0 += (int64_t)gridDim.x * blockDim.x) {
        const int64_t s = s0 + threadIdx.x;
        const bool hit = s < np && l_q[s] != 0xFFFFFFFFu;
        const uint64_t m = __ballot(hit);
        if (m == 0ull) continue;
        unsigned long long b = 0;
        if (lane == __ffsll((unsigned long long)m) - 1) b = atomicAdd(rctr, (unsigned long long)__popcll(m));
        b = __shfl(b, __ffsll((unsigned long long)m) - 1);
        if (hit) {
            const int64_t o = (int64_t)b + __popcll(m & lt);
            if (o < rcap) {
                rec_p[o] = l_p[s];
                rec_q[o] = l_q[s];
                rec_r[o] = l_r[s];
            }
        }
    }
}

// a sparse kernel with the rule image in LDS: its dynamic LDS limit raised once, to
// what its static arrays leave of the CU's 160 KB (a failed call is cleared, so it
// does not surface as the next launch's error)
template <typename K>
static int spa_img_attr(K* kern) {
    hipFuncAttributes fa;
    if (hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(kern)) != hipSuccess) {
        (void)hipGetLastError();
        return 0;
    }
    const int lim = std::min<int>(SHR_IMG_MAX, 160 * 1024 - (int)fa.sharedSizeBytes);
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, lim) !=
        hipSuccess) {
        (void)hipGetLastError();
        return 0;
    }
    return lim;
}

// the rule image fits LDS beside `static_lds` bytes of a kernel's own arrays
static bool spa_img_fits(const uint8_t* img, const shr_img* I, int static_lds) {
    return img && I && I->bytes > 0 && I->lds + static_lds + 256 <= 160 * 1024;
}

extern "C" int shr_sparse_open(const shr_table* dT, const int64_t* ts, const int32_t* akeys, int64_t n, int32_t nkeys,
                               const shd_cols* dC, const uint8_t* img, const shr_img* I, uint32_t* pr_p,
                               uint32_t* pr_r, uint32_t* pr_key, uint32_t* key_cnt,
                               unsigned long long* ctr, int64_t cap, int32_t* flag, const int32_t* pre,
                               void* stream) {
    const int pa0 = pre ? pre[0] : -1, pa1 = pre ? pre[1] : -1;
    // 512-thread workgroups on an image without f2's terms: two per CU, whose block
    // phases overlap (one 1,024-thread workgroup per CU on the whole image: segment
    // 2.17 vs 2.06 ms on C5, profiles/r6_c5_open512_ab.txt)
    shr_img IO;
    memset(&IO, 0, sizeof(IO));
    if (img && I && I->bytes > 0 && !(getenv("SH_SPARSE_IMG") && getenv("SH_SPARSE_IMG")[0] == '0')) {
        IO = *I;
        // f2's terms [off_terms1, off_terms0) left out; f1's terms moved down over them
        const int t1 = I->off_terms0 - I->off_terms1;
        IO.pad = 0;
        if (t1 > 0 && I->off_terms0 < I->lds && t1 % 16 == 0) {
            IO.pad = t1;
            IO.off_terms0 = I->off_terms1;
            IO.lds = I->lds - t1;
        } else if (t1 > 0 && I->off_terms0 >= I->lds) {
            IO.lds = I->off_terms1;  // (f1's terms in global memory: only the f2 terms cut)
        }
    }
    constexpr int T = SPO_TPB;
    const int buf = SpaOpen<T>::LDS;
    static const int lim = spa_img_attr(&k_sparse_open<true, T>);
    const bool use_img = IO.bytes > 0 && spa_img_fits(img, &IO, buf) && IO.lds <= lim;
    int64_t g = (n + T * SPA_U - 1) / (T * SPA_U);
    const int per_cu = use_img ? (160 * 1024) / (IO.lds + buf) : (160 * 1024) / buf;
    const int64_t gmax = 256LL * std::max(1, std::min(per_cu, 4));
    if (g > gmax) g = gmax;  // each workgroup strides over the run (the image staged once, few buffer flushes)
    if (g < 1) g = 1;
    if (use_img)
        hipLaunchKernelGGL((k_sparse_open<true, T>), dim3((unsigned)g), dim3(T), (size_t)IO.lds, (hipStream_t)stream, dT,
                           ts, akeys, n, nkeys, dC, img, IO, pr_p, pr_r, pr_key, key_cnt, ctr, cap, flag, pa0, pa1);
    else
        hipLaunchKernelGGL((k_sparse_open<false, T>), dim3((unsigned)g), dim3(T), 0, (hipStream_t)stream, dT, ts, akeys,
                           n, nkeys, dC, IO.bytes > 0 ? img : (const uint8_t*)nullptr, IO, pr_p, pr_r, pr_key, key_cnt,
                           ctr, cap, flag, pa0, pa1);
    return rules_ok();
}

extern "C" int shr_sparse_match(const shr_table* dT, const int64_t* ts, const int32_t* akeys, int64_t n,
                                const shd_cols* dC, const uint8_t* img, const shr_img* I, const uint32_t* pr_p, const uint32_t* pr_r,
                                const uint32_t* pr_key, uint32_t* key_fill, const unsigned long long* ctr,
                                int64_t n_pairs_max, const uint32_t* key_off, uint32_t* l_p, uint32_t* l_r,
                                int64_t* l_te, uint32_t* l_q, uint32_t* rec_p, uint32_t* rec_q, uint32_t* rec_r,
                                unsigned long long* rctr, int64_t rcap, int32_t nkeys, const shr_live* live,
                                const int32_t* pre, void* stream) {
    const int pa0 = pre ? pre[0] : -1, pa1 = pre ? pre[1] : -1;
    hipStream_t st = (hipStream_t)stream;
    const unsigned gp = rgrid(n_pairs_max);
    shr_live LV;
    memset(&LV, 0, sizeof(LV));
    if (live && live->bits) LV = *live;
    hipLaunchKernelGGL(k_sparse_place, dim3(gp), dim3(RTPB), 0, st, pr_p, pr_r, pr_key, key_fill, ctr, key_off, dT, ts,
                       l_p, l_r, l_te, l_q, LV);
    {
        shr_img none;
        memset(&none, 0, sizeof(none));
        static const int lim = spa_img_attr(&k_sparse_take<true>);
        const int tstat = 2 * (SPA_TPB / 64) * SPA_TQ * 4 + 512;  // the pair queues + the column pointers
        const bool use_img = spa_img_fits(img, I, tstat) && I->lds <= lim &&
                             !(getenv("SH_SPARSE_IMG") && getenv("SH_SPARSE_IMG")[0] == '0');
        int64_t tg = (n + SPA_TPB * SPA_U - 1) / (SPA_TPB * SPA_U);
        const int per_cu = use_img ? (160 * 1024) / (I->lds + tstat) : 2;
        const int64_t gmax = 256LL * std::max(1, std::min(per_cu, 2));
        if (tg > gmax) tg = gmax;
        if (tg < 1) tg = 1;
        // (slicing the keys by XCD measured 7.17 vs 2.94 ms for take on C5, and 512-thread
        // workgroups lost too, profiles/r4_c5_xcd_ab.txt, r5_c5_take512_ab.txt: removed)
        if (use_img)
            hipLaunchKernelGGL((k_sparse_take<true>), dim3((unsigned)tg), dim3(SPA_TPB), (size_t)I->lds, st, dT, ts,
                               akeys, n, dC, img, *I, key_off, (const uint32_t*)l_p, (const uint32_t*)l_r,
                               (const int64_t*)l_te, l_q, LV, pa0, pa1);
        else
            hipLaunchKernelGGL((k_sparse_take<false>), dim3((unsigned)tg), dim3(SPA_TPB), 0, st, dT, ts, akeys, n,
                               dC, (const uint8_t*)nullptr, none, key_off, (const uint32_t*)l_p, (const uint32_t*)l_r,
                               (const int64_t*)l_te, l_q, LV, pa0, pa1);
    }
    hipLaunchKernelGGL(k_sparse_rec, dim3(gp), dim3(256), 0, st, (const uint32_t*)l_p, (const uint32_t*)l_r,
                       (const uint32_t*)l_q, ctr, rec_p, rec_q, rec_r, rctr, rcap);
    return rules_ok();
}
