// sh_host_int.h -- internal to libsiddhi_hip.so: the handle behind the C-ABI
// (include/siddhi_hip.h), its device and pinned buffers, and the host-side
// functions shared by the ABI (sh_host.cpp), the general engine driver
// (sh_host_nfa.cpp), the fast engine drivers (sh_host_fast.cpp) and snapshots
// (sh_host_snap.cpp).
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <atomic>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
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

namespace shh {

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

inline int type_width(int t) {
    switch (t) {
        case SH_T_LONG:
        case SH_T_DOUBLE: return 8;
        case SH_T_BOOL: return 1;
        default: return 4;
    }
}

}  // namespace shh
using shh::DevBuf;
using shh::PinBuf;
using shh::type_width;

#define SH_HP_N 12
// one k_nfa_run launch of the general engine: what its completion and any replay
// need (sh_host_nfa.cpp nf_launch / nf_complete); a streaming push leaves it
// pending (on) until the next call into the handle settles it
struct NfLaunch {
    bool on = false;
    shd_batch B{};
    nfd_events E{};
    nf_cols cols{};
    int64_t n = 0, n_idx = 0, max_seg = 0, cap = 0;
    int32_t nkeys = 0;
    const uint32_t* seg_list = nullptr;
    const uint32_t* nseg = nullptr;
    const uint32_t* skeys = nullptr;
    bool fresh = false, sorted_cols = false, s3_shape = false;
    int alias = -1;
    const void* s3_col = nullptr;
    uint64_t* d_seq = nullptr;
    int64_t* d_vals = nullptr;
    int attempt = 0;
    bool defer = false;     // may be left pending (streaming push, single process)
    bool early = false;     // this attempt's history job was queued at launch (its counter block: ctl)
    const uint8_t* ctl = nullptr;
};

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
    DevBuf w_pstage, w_pstage2;  // the general engine's per-call staging (nf_push), one block; two
    int pst = 0;                 // alternate per call (a call's launch may still read the last one)
    NfLaunch pend;               // a streaming push's launch not yet completed (nf_settle)
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
    PinBuf pin_stage, pin_stage2;  // the general engine's per-call event staging (nf_push), alternating
    DevBuf n_tmin, n_slot_s, n_slot_k;  // device tie-break of due keys
    DevBuf n_armed;                     // per key: may hold a scheduler entry (nf_cols.sched_armed)
    // the armed-key list of the due pass (two buffers, swapped per pass; counts
    // in n_klist_n[0..1]) and the log of keys armed since the last pass
    DevBuf n_klist[2], n_klist_n, n_arm_log, n_arm_ctr;
    int klist_cur = 0;
    // SH_HOST_PROF: wall time per host phase (shx_host_profile; printed by sh_destroy)
    // 0 push, 1 timers, 2 process, 3 history, 4 place, 5 drain, 6 hist_copy, 7 hist_apply,
    // 8 hist_rank, 9 history records (count), 10 blocked in stream syncs, 11 deferred-row pulls
    double hp_ms[SH_HP_N] = {};
    int64_t hp_n[SH_HP_N] = {};
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
    // the replay runs on a host thread (hw_*): a launch's records are queued with
    // an event recorded behind their copy; the thread waits for it and applies the
    // launches in order while this thread goes on (stages and launches the next
    // call); every use of the models joins it first (nf_sev_flush)
    struct HistJob {
        int64_t first, n;
        hipEvent_t ev;
        const uint8_t* ctl;  // (a launch queued before its completion: its counter block, n from it)
    };
    std::thread hw_thread;
    std::mutex hw_mu;
    std::deque<HistJob> hw_q;
    std::atomic<int> hw_pending{0};      // queued or running jobs (the thread and the joins spin on it)
    std::atomic<bool> hw_stop{false};
    std::condition_variable hw_cv;       // (SH_HIST_SPIN=0: the thread sleeps on it between jobs)
    bool hw_spin = true;
    bool hw_fail = false;
    PinBuf pin_ctl2;                     // counter blocks of launches whose history jobs were queued at launch
                                         // (one 32-byte slot per history event, hw_ev)
    hipEvent_t hw_ev[16] = {};
    int hw_ev_next = 0;
    double hw_ms = 0.0;  // the thread's replay time (phase 7 when profiled)
    bool hist_spec = false;  // the last launch's first history records came back with its counters
    std::vector<nfd_cand> pick_slots;  // host pick of the due keys: one slot per due millisecond
    PinBuf pin_sev, pin_rk, pin_cand;
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
    // sparse partials (shr_sparse_*): the partials, per key counts and list starts,
    // the keys' lists (opening event, rule, consuming event, expiry), counters
    DevBuf rs_pr, rs_key, rs_list, rs_ctl, rs_live;
    int rs_last = 0;  // 1: the last rule run took the sparse-partial path
    // ---- bucketed window engine (sh_bucket.hip + shb_match): 0 untried, 1 loaded, <0 unavailable
    int bk_state = 0;
    int32_t part_attr0 = -1;  // stream-0 attribute keying query 0's partition
    int bk_last = 0;          // 1: the last sh_run_device ran on the bucketed engine
    int s3b_last = 0;         // 1: ... on the sequence bucket-carry engine (k_s3b)
    shj_bucket bk{};
    std::string bk_err;
    DevBuf bk_w0, bk_sp, bk_toff, bk_tofft, bk_cnt, bk_mstart, bk_tpre, bk_tfirst, bk_hstart, bk_ttot, bk_flag, bk_prof;
    DevBuf bk_st[SHB_MAX_STAGED], bk_ms[SHB_MAX_MS], bk_agg[SHB_MAX_AGG];
    bool bk_agg_carried = false;  // the last bucketed run carried its aggregates (k_bk_aggc)
    PinBuf bk_rd;
    bool aggp_refused = false;  // run_bucket: k_bk_aggp refused a value once: the post-pass from then on
    bool aggp_only = false;  // run_bucket: k_bk_aggp or nothing (1), the caller's layout kept
    // typed output columns (sh_device_run.d_out_cols) for engines that write rows
    DevBuf w_colrows;
    bool cols_rows = false;
    // the caller's layout of this sh_run_device call (SHB_OUT_*): engines that
    // write it themselves take it, the others write raw rows into w_colrows (and
    // the sequence numbers into w_packseq) for a conversion afterwards
    int out_mode = SHB_OUT_RAW;
    int32_t pk_w[SHB_MAX_OUT], pk_woff[SHB_MAX_OUT], pk_rw = 0;
    DevBuf w_packseq;
    // aggregators behind the fast engines (sh_agg.hip): scratch, trigger sequence
    // numbers when the caller wants none, and the last run's path
    DevBuf a_scratch, a_seq;
    int agg_last = 0;  // 1: post-pass done, 2: post-pass not exact -> sequential engine, 3: in the k_seq3s lanes,
                       // 4: carried per key by the bucketed engine (k_bk_aggc), 5: ... in parallel (k_bk_aggp)
    std::vector<int32_t> out_types;  // per select position over the queries (-2: types differ)
    uint64_t fp = 0;                 // compiled-program fingerprint (snapshot images)
};

// SH_HOST_PROF: a phase's wall time into h->hp_ms[i] (scope lifetime)
struct HpScope {
    sh_handle* h;
    int i;
    std::chrono::steady_clock::time_point t0;
    static bool on() {
        static const bool v = getenv("SH_HOST_PROF") != nullptr;  // (read once per process)
        return v;
    }
    HpScope(sh_handle* hh, int ii) : h(on() ? hh : nullptr), i(ii) {
        if (h) t0 = std::chrono::steady_clock::now();
    }
    ~HpScope() {
        if (!h) return;
        h->hp_ms[i] += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        h->hp_n[i]++;
    }
};

// the scheduler-history replay thread: stop it (sh_destroy)
void nf_hist_stop(sh_handle* h);

// a stream sync of the streaming path (its wait counted as phase 10)
inline hipError_t nf_sync(sh_handle* h, hipStream_t st) {
    HpScope w_(h, 10);
    return hipStreamSynchronize(st);
}

// ---- shared host functions (definitions in the .cpp named in the comment)
// sh_host.cpp
int ensure_ws(sh_handle* h, int64_t n);
int fail(sh_handle* h, int code, const std::string& m);
int flush(sh_handle* h);
// sh_host_nfa.cpp
int nf_launch(sh_handle* h, NfLaunch& L);
int nf_complete(sh_handle* h, NfLaunch& L, int64_t* n_rows);
int nf_settle(sh_handle* h);
int nf_app_pull(sh_handle* h);
int nf_ensure_keys(sh_handle* h, int32_t nkeys);
int nf_next_due(sh_handle* h, int64_t* out);
int nf_process(sh_handle* h, const shd_batch& B, int32_t nkeys, const nf_cols& cols_in, uint64_t* d_seq,
               int64_t* d_vals, int64_t cap, int64_t* n_rows, bool fresh = false, int64_t batch_events = 0,
               const sh_device_run* carry_run = nullptr, const uint32_t* gidx = nullptr, int64_t n_idx = 0);
int nf_push(sh_handle* h, const sh_batch* b, int64_t r0, const uint32_t* index = nullptr, int64_t call_n = 0,
            int64_t call_last = 0);
int nf_sev_flush(sh_handle* h);
int nf_start(sh_handle* h);
int nf_timers(sh_handle* h, int64_t now, bool wall = false);
int nf_upload_table(sh_handle* h);
// sh_host_fast.cpp
int agg_post(sh_handle* h, sh_device_run* run, int32_t nkeys, const int32_t* d_query, int n_query,
             const int32_t* agg_kind, const int32_t* arg_type, int n_out);
int bits_for(uint64_t v);
int carry_setup(sh_handle* h, const sh_device_run* run, shd_payload* carry, void** mid, int* alias,
                bool used_only = false, bool with_ts = true);
int rows_for_cols(sh_handle* h, sh_device_run* run);
// the caller's layout for an engine that writes it itself (typed columns /
// packed rows, unless the rows were sent to the workspace): OC->use = SHB_OUT_RAW otherwise
void direct_layout(sh_handle* h, sh_device_run* run, const int32_t* widths, int n_out, shb_cols* OC);
int run_bucket(sh_handle* h, sh_device_run* run, int32_t nkeys, bool force_carry = false);
int run_rules(sh_handle* h, sh_device_run* run);
int run_s3b(sh_handle* h, sh_device_run* run, int32_t nkeys);
shd_segment_ws seg_ws(sh_handle* h, int64_t n);
int tile_shift_for(int64_t n, int32_t nkeys);

// diagnostics of the engine choices (not part of the reference-facing ABI)
extern "C" {
int shx_jit_status(sh_handle* h);
int shx_jit_compile(sh_handle* h);
int shx_bucket_status(sh_handle* h);
int shx_seq3_status(sh_handle* h);
int shx_agg_status(sh_handle* h);
int shx_rules_status(sh_handle* h);
int shx_host_profile(sh_handle* h, double* ms, int64_t* n, int cap);
int shx_seq3_shape(sh_handle* h);
int shx_bucket_compile(sh_handle* h, char* buf, int64_t len);
int64_t shx_jit_source(sh_handle* h, char* buf, int64_t len);
}
