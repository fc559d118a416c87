// sh_host_nfa.cpp -- the general NFA engine (sh_nfa.h, mode 1) on the host side:
// per-key state and buffers, the launch / replay loop of k_nfa_run, ordered placement
// of its records, the playback / wall-clock scheduler passes (due list, pick, timer
// kernel) and the scheduler maps' HashMap-order models (sh_jmap.h).
#include "sh_host_int.h"

// ================================================================ general engine (mode 1)
// sh_nfa.h lanes over the radix segment; emissions are placed by an exclusive
// scan of per-run counts. A lane error (an arena / list / queue / emission
// buffer full) restores the touched keys' blocks, grows the capacity and replays.
// the due scan's key filter (SH_NO_ARMED: scan every key)
static uint8_t* armed_flags(sh_handle* h) {
    static const bool off = getenv("SH_NO_ARMED") != nullptr;
    return off ? nullptr : h->n_armed.as<uint8_t>();
}

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
    nf_sync(h, h->stream);
    if (h->n_lst.ensure_fresh((size_t)h->lst_cap * 4 * 8)) return SH_E_OOM;
    h->lst_cap *= 4;
    return 0;
}

int nf_ensure_keys(sh_handle* h, int32_t nkeys) {
    if (nkeys <= h->n_nkeys) return 0;
    const int32_t nk = std::max(nkeys, h->n_nkeys * 2);
    const size_t kb = (size_t)h->T->key_words * 8;
    const size_t old = (size_t)h->n_nkeys * kb, need = (size_t)nk * kb;
    nf_sync(h, h->stream);
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
        nf_sync(h, h->stream);
        if (h->n_sev.ensure_fresh((size_t)need * 16) || h->n_sev_ctr.ensure_fresh(64)) return SH_E_OOM;
        h->sev_cap = need;
    }
    if (!zero) return 0;
    return hipMemsetAsync(h->n_sev_ctr.p, 0, 8, h->stream) == hipSuccess ? 0 : SH_E_HIP;
}

// replay the launch's getState history on the host models and upload the
// changed ranks (before the next due scan, on the same stream)
// pin_rd slots of the counter block read back after a launch (nf_ctl_read)
enum { PR_CTL = 40 };
// scheduler-history records copied back speculatively with a launch's counters
// (a launch with more takes a second, event-tracked copy)
static const int64_t kHistSpec = 4096;

// the launch's counter block (records, error, history count) into pin_rd[PR_CTL..+24),
// read with the caller's next sync; single process with scheduler maps: the first
// kHistSpec history records come back in the same sync (h->hist_spec)
static void nf_ctl_read(sh_handle* h) {
    hipMemcpyAsync(h->pin_rd.as<uint8_t>() + PR_CTL, h->n_ctl.p, 24, hipMemcpyDeviceToHost, h->stream);
    h->hist_spec = false;
    static const bool spec_off = getenv("SH_HIST_SPEC") && getenv("SH_HIST_SPEC")[0] == '0';
    if (spec_off || !h->sm_on || h->coord_on || h->sev_cap < kHistSpec) return;
    if ((size_t)(h->hist_used + kHistSpec) * 16 > h->pin_hist.bytes) {
        if (nf_sev_flush(h)) return;  // (the buffer restarts once the thread is idle)
        if (h->pin_hist.ensure((size_t)kHistSpec * 16 * 4)) return;
    }
    hipMemcpyAsync(h->pin_hist.as<uint8_t>((size_t)h->hist_used * 16), h->n_sev.p, (size_t)kHistSpec * 16,
                   hipMemcpyDeviceToHost, h->stream);
    h->hist_spec = true;
}
static const uint8_t* nf_ctl(sh_handle* h) { return h->pin_rd.as<uint8_t>() + PR_CTL; }
static unsigned nf_ctl_err(sh_handle* h) { return *(const unsigned*)(nf_ctl(h) + 8); }
static int64_t nf_ctl_nrec(sh_handle* h) { return *(const int64_t*)nf_ctl(h); }
static int64_t nf_ctl_nsev(sh_handle* h) { return *(const int64_t*)(nf_ctl(h) + 16); }

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
            if (nf_sync(h, st) != hipSuccess) return fail(h, SH_E_HIP, "rank upload");  // (rare: after a resize)
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

// the replay thread: applies queued launches in order, each after its copy's event.
// It spins on the pending count (a condition variable's wake-up cost the launching
// thread ~20 us per launch); a job queued before its launch completed reads its
// record count from the launch's counter block and skips a failed launch (the
// replay queues its own job) or one with more records than came back (the
// completion applies those itself)
static inline void hw_relax(int& spins) {
    if (++spins < 256)
        __builtin_ia32_pause();
    else
        std::this_thread::yield();
}

static void hw_loop(sh_handle* h) {
    for (;;) {
        int spins = 0;
        if (h->hw_spin) {
            while (h->hw_pending.load(std::memory_order_acquire) == 0) {
                if (h->hw_stop.load(std::memory_order_acquire)) return;
                hw_relax(spins);
            }
        } else {
            std::unique_lock<std::mutex> lk(h->hw_mu);
            h->hw_cv.wait(lk, [h] { return h->hw_stop.load() || h->hw_pending.load() != 0; });
            if (h->hw_pending.load() == 0) return;
        }
        sh_handle::HistJob j;
        {
            std::lock_guard<std::mutex> lk(h->hw_mu);
            j = h->hw_q.front();
        }
        const auto t0 = std::chrono::steady_clock::now();
        // polled (a blocking wait would hold the runtime's locks against the
        // launching thread's calls)
        hipError_t q = hipSuccess;
        spins = 0;
        if (j.ev)
            while ((q = hipEventQuery(j.ev)) == hipErrorNotReady) std::this_thread::sleep_for(std::chrono::microseconds(5));
        bool ok = q == hipSuccess;
        int64_t n = j.n;
        if (ok && j.ctl) {
            const unsigned err = *(const unsigned*)(j.ctl + 8);
            const int64_t ns = *(const int64_t*)(j.ctl + 16);
            n = (err || ns > kHistSpec) ? 0 : ns;
        }
        if (ok && n > 0) ok = h->sm.apply(h->pin_hist.as<uint64_t>((size_t)j.first * 16), (size_t)n);
        const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        {
            std::lock_guard<std::mutex> lk(h->hw_mu);
            h->hw_q.pop_front();
            h->hw_ms += ms;
            if (!ok) h->hw_fail = true;
        }
        h->hw_pending.fetch_sub(1, std::memory_order_release);
    }
}

// queue a launch's records [first, first + n) of pin_hist (tracked: their copy is
// on h->stream; ctl: n comes from this counter block once the copy has landed)
static int hw_submit(sh_handle* h, int64_t first, int64_t n, bool tracked, const uint8_t* ctl = nullptr) {
    if (!h->hw_thread.joinable()) {
        for (auto& e : h->hw_ev)
            if (!e && hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess)
                return fail(h, SH_E_HIP, "history events");
        h->hw_stop.store(false);
        h->hw_spin = !(getenv("SH_HIST_SPIN") && getenv("SH_HIST_SPIN")[0] == '0');
        h->hw_thread = std::thread(hw_loop, h);
    }
    {
        // (an event is reused only after its job is done: at most 15 queued)
        int spins = 0;
        while (h->hw_pending.load(std::memory_order_acquire) >= 15) hw_relax(spins);
    }
    hipEvent_t ev = nullptr;  // (untracked: the records are on the host already)
    if (tracked) {
        ev = h->hw_ev[h->hw_ev_next];
        h->hw_ev_next = (h->hw_ev_next + 1) % 16;
        if (hipEventRecord(ev, h->stream) != hipSuccess) return fail(h, SH_E_HIP, "history event");
    }
    {
        std::lock_guard<std::mutex> lk(h->hw_mu);  // (the count under the lock: no lost wake-up)
        h->hw_q.push_back({first, n, ev, ctl});
        h->hw_pending.fetch_add(1, std::memory_order_release);
    }
    if (!h->hw_spin) h->hw_cv.notify_one();
    return SH_OK;
}

void nf_hist_stop(sh_handle* h) {
    if (!h->hw_thread.joinable()) return;
    {
        std::lock_guard<std::mutex> lk(h->hw_mu);
        h->hw_stop.store(true, std::memory_order_release);
    }
    h->hw_cv.notify_all();
    h->hw_thread.join();
    h->hw_pending.store(0);
    h->hw_q.clear();
    for (auto& e : h->hw_ev)
        if (e) {
            hipEventDestroy(e);
            e = nullptr;
        }
}

// wait for the replay thread to apply every queued launch; before every use of
// the models (a due pick, a rank upload, a snapshot, new key strings)
int nf_sev_flush(sh_handle* h) {
    if (!h->hw_thread.joinable()) return SH_OK;
    HpScope hp_(h, 3);
    int spins = 0;
    while (h->hw_pending.load(std::memory_order_acquire) != 0) hw_relax(spins);
    bool bad;
    {
        std::lock_guard<std::mutex> lk(h->hw_mu);
        bad = h->hw_fail;
        h->hw_fail = false;
        h->hp_ms[7] = h->hw_ms;
    }
    h->hist_used = 0;
    if (bad) return fail(h, SH_E_UNSUPPORTED, "more than 2^26 scheduler map bins (keys waiting on one absent state)");
    return SH_OK;
}

// the models' ranks on the device (the device pick of a large due backlog)
static int nf_rank_sync(sh_handle* h) {
    int rc = nf_sev_flush(h);
    if (rc) return rc;
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
            if (nf_sync(h, st) != hipSuccess) return fail(h, SH_E_HIP, "scheduler history");
            n = (int64_t)*h->pin_sev.as<unsigned long long>();
        }
        h->hp_n[9] += n;
        if (!h->coord_on) {
            const bool spec = counted && h->hist_spec;
            h->hist_spec = false;
            if (n == 0) return SH_OK;
            if (spec && n <= kHistSpec) {
                // already on the host (the counters' sync): the thread starts at once
                int qrc = hw_submit(h, h->hist_used, n, false);
                if (qrc) return qrc;
                h->hist_used += n;
                return SH_OK;
            }
            if ((size_t)(h->hist_used + n) * 16 > h->pin_hist.bytes) {
                // grow: once the thread has applied the queued launches, the buffer restarts
                int frc = nf_sev_flush(h);
                if (frc) return frc;
                if (h->pin_hist.ensure((size_t)n * 16)) return fail(h, SH_E_OOM, "pinned staging");
            }
            hipMemcpyAsync(h->pin_hist.as<uint8_t>((size_t)h->hist_used * 16), h->n_sev.p, (size_t)n * 16,
                           hipMemcpyDeviceToHost, st);
            int qrc = hw_submit(h, h->hist_used, n, true);
            if (qrc) return qrc;
            h->hist_used += n;
            return SH_OK;
        }
        if (h->pin_sev.ensure((size_t)std::max<int64_t>(n, 1) * 16)) return fail(h, SH_E_OOM, "pinned staging");
        if (n) hipMemcpyAsync(h->pin_sev.p, h->n_sev.p, (size_t)n * 16, hipMemcpyDeviceToHost, st);
        if (nf_sync(h, st) != hipSuccess) return fail(h, SH_E_HIP, "scheduler history");
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

int nf_upload_table(sh_handle* h) {
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
        if (nf_sync(h, st) != hipSuccess) return fail(h, SH_E_HIP, "relayout");
        h->n_kstate.release();
        h->n_kstate = fresh;
        fresh.p = nullptr;
        fresh.bytes = 0;
    } else {
        nf_sync(h, st);
    }
    return SH_OK;
}

static int nf_ensure_recs(sh_handle* h, int64_t cap) {
    const int stride = NF_REC_HDR + std::max(1, h->n_out);
    if (cap <= h->rec_cap) return 0;
    nf_sync(h, h->stream);
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
    return e ? (int64_t)atoll(e) : (int64_t)65536;
}();
static const int64_t kTieBreakSlots = (int64_t)1 << 22;
// due candidates copied back with their count (a larger backlog takes a second copy)
static const int64_t kCandSpec = 4096;

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
int nf_app_pull(sh_handle* h) {
    if (h->df_ub == 0) return SH_OK;
    HpScope hp_(h, 11);
    hipStream_t st = h->df_stream;
    unsigned long long n = 0;
    if (hipMemcpyAsync(&n, h->df_ctr.p, 8, hipMemcpyDeviceToHost, st) != hipSuccess ||
        nf_sync(h, st) != hipSuccess)
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
        if (nf_sync(h, st) != hipSuccess) return fail(h, SH_E_HIP, "deferred rows copy");
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
    static const bool multi = getenv("SH_PLACE_MULTI") != nullptr;
    if (nrec <= 8192 && n_idx <= 8192 && !multi) {
        // one workgroup: scan, map, gather and the row count in one launch
        if (nfd_place_app_small(h->n_recs.as<uint64_t>(), nrec, NF_REC_HDR + no, h->w_cnt.as<uint32_t>(), n_idx, no,
                                h->df_ctr.as<unsigned long long>(), h->df_q.as<int32_t>(), h->df_seq.as<uint64_t>(),
                                h->df_ts.as<int64_t>(), h->df_vals.as<int64_t>(), h->df_nulls.as<uint8_t>(), st))
            return fail(h, SH_E_HIP, "placement");
        h->df_ub += nrec;
        h->df_stream = st;
        return SH_OK;
    }
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
    if (nf_sync(h, st) != hipSuccess) return fail(h, SH_E_HIP, "device error before placement");
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
            return nf_sync(h, st) == hipSuccess ? SH_OK : fail(h, SH_E_HIP, "placement");
        }
        nfd_place(h->n_recs.as<uint64_t>(), (int64_t)nrec, stride, h->w_off.as<uint32_t>(), no,
                  h->dev_want_query ? h->w_oq.as<int32_t>() : nullptr, d_seq, nullptr, d_vals, nullptr,
                  h->w_inv.as<uint32_t>(), total, st);
        return nf_sync(h, st) == hipSuccess ? SH_OK : fail(h, SH_E_HIP, "placement");
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
    if (nf_sync(h, st) != hipSuccess) return fail(h, SH_E_HIP, "output copy");
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

// `carry` (sh_run_device, single stream): ts and the stream-0 columns are moved
// into key-segment order by the segment, so each lane streams its own events
// gidx / n_idx (key-sharded push): each event's position in the whole send()
// call of n_idx events (match counts and order tags are indexed by it)
int nf_process(sh_handle* h, const shd_batch& B, int32_t nkeys, const nf_cols& cols_in, uint64_t* d_seq,
                      int64_t* d_vals, int64_t cap, int64_t* n_rows, bool fresh, int64_t batch_events,
                      const sh_device_run* carry_run, const uint32_t* gidx, int64_t n_idx) {
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
    NfLaunch& L = h->pend;
    L = NfLaunch{};
    L.B = B;
    L.E = E;
    L.cols = cols;
    L.n = n;
    L.n_idx = n_idx;
    L.nkeys = nkeys;
    L.max_seg = max_seg;
    L.seg_list = seg_list;
    L.nseg = nseg;
    L.skeys = skeys;
    L.fresh = fresh;
    L.sorted_cols = sorted_cols;
    L.alias = alias;
    L.s3_shape = s3_shape;
    L.s3_col = s3_col;
    L.d_seq = d_seq;
    L.d_vals = d_vals;
    L.cap = cap;
    // a streaming push (single process, host rows) leaves the launch's completion --
    // its error word, history and placement -- to the next call into the handle
    // (nf_settle), so the caller prepares the next send() while this one runs
    static const bool no_defer = getenv("SH_NO_DEFER_LAUNCH") != nullptr;
    const bool defer = !no_defer && !d_seq && !fresh && !h->coord_on && !h->has_lists && !sorted_cols;
    L.defer = defer;
    int rc = nf_launch(h, L);
    if (rc) return rc;
    if (defer) {
        L.on = true;
        *n_rows = -1;
        return SH_OK;
    }
    return nf_complete(h, L, n_rows);
}

// one attempt of a k_nfa_run launch: save the touched keys, clear the counters, the
// kernel, and the counter block (+ the first history records) read back behind it
int nf_launch(sh_handle* h, NfLaunch& L) {
    hipStream_t st = h->stream;
    const size_t kw = (size_t)h->T->key_words;
    if (!L.fresh) {
        if (h->n_save.ensure_fresh((size_t)L.max_seg * kw * 8)) return fail(h, SH_E_OOM, "save area");
        nfd_save(h->n_kstate.as<uint64_t>(), (int64_t)kw, L.seg_list, L.nseg, L.skeys, L.max_seg,
                 h->n_save.as<uint64_t>(), 0, st);
    }
    nfd_zero2(h->w_cnt.p, L.n_idx * 4, h->n_ctl.p, 24, st);  // match counts + counter block
    if (nf_lst_ready(h)) return fail(h, SH_E_OOM, "list values");
    nf_cols& cols = L.cols;
    if (h->has_lists && (cols.lst != h->n_lst.as<uint64_t>() || cols.lst_cap != (uint64_t)h->lst_cap)) {
        cols.lst = h->n_lst.as<uint64_t>();
        cols.lst_ctr = h->n_lst_ctr.as<unsigned long long>();
        cols.lst_cap = (uint64_t)h->lst_cap;
        nf_put_cols(h, cols);
    }
    if (h->sm_on) {
        if (nf_sev_ready(h, L.n, false)) return fail(h, SH_E_OOM, "scheduler history");
        if (cols.sev != h->n_sev.as<uint64_t>() || cols.sev_cap != (uint64_t)h->sev_cap) {
            // the buffer moved: refresh the column image
            const nf_cols keep = cols;
            cols = nf_store_cols(h);
            if (L.sorted_cols) {
                for (size_t a = 0; a < h->stream_types[0].size(); a++)
                    if (a >= 32 || ((h->T->attr_used[0] >> a) & 1u)) cols.col[0][a] = keep.col[0][a];
            }
            nf_put_cols(h, cols);
        }
    }
    nfd_emit em = nf_emit(h);
    // the rise-and-fall sequence engine: fresh single-query runs of that shape
    h->seq3_last = L.s3_shape ? 1 : 0;
    if (L.s3_shape) {
        if (nfd_seq3(h->d_T.as<nf_table>(), h->d_ncols.as<nf_cols>(), &L.E, L.n, L.seg_list, L.nseg, L.skeys,
                     L.nkeys, L.max_seg, &em, st, L.s3_col, h->s3_compact ? 1 : 0, h->s3_agg ? 1 : 0, h->s3_rw))
            return fail(h, SH_E_HIP, "k_seq3 launch failed");
    } else if (nfd_run(h->d_T.as<nf_table>(), h->d_ncols.as<nf_cols>(), h->n_kstate.as<uint64_t>(), &L.E, L.n,
                       L.seg_list, L.nseg, L.skeys, L.nkeys, L.max_seg, h->tick, h->clock, &em, st))
        return fail(h, SH_E_HIP, "k_nfa_run launch failed");
    hipEventRecord(h->ev[2], st);
    L.early = false;
    // early jobs are opt-in (SH_HIST_EARLY=1): on the 3,000-call A/B they measured no
    // faster than queueing the job at settle (profiles/r4_c4_hist_ab.txt)
    static const bool early_off = !(getenv("SH_HIST_EARLY") && getenv("SH_HIST_EARLY")[0] == '1');
    if (L.defer && L.attempt == 0 && h->sm_on && !h->coord_on && h->sev_cap >= kHistSpec && !early_off) {
        // its history job is queued now: the replay thread applies the records as
        // soon as they land, while the caller prepares the next call
        if (h->pin_ctl2.ensure(16 * 32)) return fail(h, SH_E_OOM, "pinned staging");
        if ((size_t)(h->hist_used + kHistSpec) * 16 > h->pin_hist.bytes) {
            const int frc = nf_sev_flush(h);
            if (frc) return frc;
            if (h->pin_hist.ensure((size_t)kHistSpec * 16 * 4)) return fail(h, SH_E_OOM, "pinned staging");
        }
        uint8_t* slot = h->pin_ctl2.as<uint8_t>((size_t)h->hw_ev_next * 32);  // (the job's event index)
        hipMemcpyAsync(slot, h->n_ctl.p, 24, hipMemcpyDeviceToHost, st);
        hipMemcpyAsync(h->pin_hist.as<uint8_t>((size_t)h->hist_used * 16), h->n_sev.p, (size_t)kHistSpec * 16,
                       hipMemcpyDeviceToHost, st);
        const int qrc = hw_submit(h, h->hist_used, -1, true, slot);
        if (qrc) return qrc;
        h->hist_used += kHistSpec;
        h->hist_spec = false;
        L.early = true;
        L.ctl = slot;
    } else {
        nf_ctl_read(h);
    }
    L.attempt++;
    return SH_OK;
}

// wait for a launched attempt; on success its history and rows, else restore the
// touched keys (or the fresh state), grow what overflowed, and launch again
int nf_complete(sh_handle* h, NfLaunch& L, int64_t* n_rows) {
    hipStream_t st = h->stream;
    L.on = false;
    for (;;) {
        if (nf_sync(h, st) != hipSuccess) return fail(h, SH_E_HIP, "device error in k_nfa_run");
        const uint8_t* ctl = L.early ? L.ctl : nf_ctl(h);
        const unsigned err = *(const unsigned*)(ctl + 8);
        if (!err) {
            h->tick++;
            const int64_t nrec = *(const int64_t*)ctl;
            if (L.early) {
                // its job is queued; more records than came back: the thread skips
                // them, so they are applied here, in order, once it is idle
                const int64_t ns = *(const int64_t*)(ctl + 16);
                h->hp_n[9] += ns;
                if (ns > kHistSpec) {
                    int frc = nf_sev_flush(h);
                    if (frc) return frc;
                    if (h->pin_hist.ensure((size_t)ns * 16)) return fail(h, SH_E_OOM, "pinned staging");
                    hipMemcpyAsync(h->pin_hist.p, h->n_sev.p, (size_t)ns * 16, hipMemcpyDeviceToHost, st);
                    const int qrc = hw_submit(h, 0, ns, true);
                    if (qrc) return qrc;
                    h->hist_used = ns;
                }
            } else {
                int src = nf_sev_apply(h, true);
                if (src) return src;
            }
            int64_t rows = 0;
            int rc = nf_place(h, L.n_idx, &rows, L.d_seq, L.d_vals, L.cap, h->tick - 1, nrec);
            if (n_rows) *n_rows = rows;
            hipEventElapsedTime(&h->times.segment_ms, h->ev[0], h->ev[1]);
            hipEventElapsedTime(&h->times.advance_ms, h->ev[1], h->ev[2]);
            if (rows >= 0) {
                hipEventRecord(h->ev[3], st);
                nf_sync(h, st);
                hipEventElapsedTime(&h->times.emit_ms, h->ev[2], h->ev[3]);
                hipEventElapsedTime(&h->times.total_ms, h->ev[0], h->ev[3]);
            } else {  // deferred rows: the placement is still on the stream
                h->times.emit_ms = 0.0f;
                hipEventElapsedTime(&h->times.total_ms, h->ev[0], h->ev[2]);
            }
            h->times.advance_launches = L.attempt;
            return rc;
        }
        if (err & NF_E_KEY) return fail(h, SH_E_INVALID_ARG, "partition key id >= n_keys");
        if (err & NF_E_UNSUP)
            return fail(h, SH_E_UNSUPPORTED, "CountPreStateProcessor.startStateReset recursion (reference overflows)");
        if (L.attempt >= 64) return fail(h, SH_E_STATE_OVERFLOW, "replay limit");
        const size_t kw = (size_t)h->T->key_words;
        if (!L.fresh)
            nfd_save(h->n_kstate.as<uint64_t>(), (int64_t)kw, L.seg_list, L.nseg, L.skeys, L.max_seg,
                     h->n_save.as<uint64_t>(), 1, st);
        if (err & NF_E_EMIT) {
            if (nf_ensure_recs(h, h->rec_cap * 4)) return fail(h, SH_E_OOM, "emission buffer");
        }
        if (err & NF_E_SEV) {
            nf_sync(h, st);
            if (h->n_sev.ensure_fresh((size_t)h->sev_cap * 4 * 16)) return fail(h, SH_E_OOM, "scheduler history");
            h->sev_cap *= 4;
        }
        if ((err & NF_E_LST) && nf_lst_grow(h)) return fail(h, SH_E_OOM, "list values");
        if (err & ~(unsigned)(NF_E_EMIT | NF_E_SEV | NF_E_LST)) {
            int rc = nf_grow(h, err);
            if (rc) return rc;
        }
        if (L.fresh) {
            hipMemsetAsync(h->n_kstate.p, 0, (size_t)L.nkeys * h->T->key_words * 8, st);
            if (!h->T->partitioned) {
                h->started = false;
                int rc = nf_start(h);
                if (rc) return rc;
            }
        }
        int lrc = nf_launch(h, L);
        if (lrc) return lrc;
    }
}

// complete a streaming push's launch left pending (see nf_process); before every
// other use of the handle's device state
int nf_settle(sh_handle* h) {
    if (!h->pend.on) return SH_OK;
    return nf_complete(h, h->pend, nullptr);
}

// earliest queued notify time over every scheduler and key (INT64_MAX: none;
// key-sharded: over every rank)
static int nf_next_due_local(sh_handle* h, int64_t* out) {
    *out = INT64_MAX;
    {
        int src = nf_settle(h);
        if (src) return src;
    }
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
            if (nf_sync(h, st) != hipSuccess) return fail(h, SH_E_HIP, "k_nfa_due");
            const int64_t nc = (int64_t)*h->pin_rd.as<unsigned long long>(PR_NC);
            if (nc == 0) continue;
            nfd_cand_tmin(h->n_cand.as<nfd_cand>(), nc, h->n_tmin.as<unsigned long long>(), st);
            hipMemcpyAsync(h->pin_rd.as<void>(PR_TMIN), h->n_tmin.p, 8, hipMemcpyDeviceToHost, st);
            if (nf_sync(h, st) != hipSuccess) return fail(h, SH_E_HIP, "k_cand_tmin");
            *out = std::min(*out, (int64_t)*h->pin_rd.as<unsigned long long>(PR_TMIN));
        }
    }
    return SH_OK;
}

int nf_next_due(sh_handle* h, int64_t* out) {
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
int nf_timers(sh_handle* h, int64_t now, bool wall) {
    HpScope hp_(h, 1);
    hipStream_t st = h->stream;
    bool first_pass = true;
    int n_absent = 0;  // a key's armed flag may be cleared only when it has one scheduler
    for (int q = 0; q < h->T->n_queries; q++)
        for (int p = 0; p < h->T->q[q].n_proc; p++) n_absent += nf_has_sched(h->T->q[q].proc[p]);
    // the due pass of scheduler (q, p): the candidate count and the first candidates
    // into pinned memory, no sync (list: the armed-key list form; first: the pass
    // that also folds the keys armed since the last one into the next list)
    auto due_launch = [&](int q, int p, bool list, bool first) -> int {
        const int32_t nkeys = h->n_nkeys;
        if (h->n_cand.ensure_fresh((size_t)nkeys * sizeof(nfd_cand))) return fail(h, SH_E_OOM, "candidates");
        if (h->pin_cand.ensure((size_t)kCandSpec * sizeof(nfd_cand))) return fail(h, SH_E_OOM, "pinned staging");
        const bool host_stamps = h->sm_on && !h->coord_on;
        const uint64_t* rank = h->sm_on && !host_stamps ? h->n_rank[q * NF_MAX_PROC + p].as<uint64_t>() : nullptr;
        if (!(list && first)) hipMemsetAsync(h->n_ctr.p, 0, 8, st);
        if (list) {
            unsigned long long* ln = h->n_klist_n.as<unsigned long long>();
            const int c = h->klist_cur;
            if (first) {
                nfd_zero2(h->n_ctr.p, 8, ln + (c ^ 1), 8, st);  // candidates + the next list's count
                nfd_due_list(h->d_T.as<nf_table>(), q, p, h->n_kstate.as<uint64_t>(), h->n_klist[c].as<int32_t>(),
                             ln + c, h->n_arm_log.as<int32_t>(), h->n_arm_ctr.as<unsigned long long>(), now,
                             h->n_cand.as<nfd_cand>(), h->n_ctr.as<unsigned long long>(), nkeys, armed_flags(h),
                             n_absent == 1 ? 1 : 0, rank, h->n_klist[c ^ 1].as<int32_t>(), ln + (c ^ 1),
                             (int64_t)nkeys, st);
                hipMemsetAsync(h->n_arm_ctr.p, 0, 8, st);
                h->klist_cur ^= 1;
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
        // the first candidates come back with the count (most passes need no second copy)
        hipMemcpyAsync(h->pin_cand.p, h->n_cand.p, (size_t)std::min<int64_t>(nkeys, kCandSpec) * sizeof(nfd_cand),
                       hipMemcpyDeviceToHost, st);
        return SH_OK;
    };
    // (queueing the first due pass behind a pending event launch saved a sync per call
    // but made the candidates' stamps wait longer for the scheduler-map replay: 1,486-1,511
    // vs 1,377-1,379 ms per 3,000 C4 calls, profiles/r5_c4_spec_due_ab.txt; removed)
    {
        int src = nf_settle(h);
        if (src) return src;
    }
    if (!h->T->has_absent) return SH_OK;
    if (h->n_nkeys == 0 && !h->coord_on) return SH_OK;
    if (pin_rd_ready(h)) return fail(h, SH_E_OOM, "pinned staging");
    nf_put_cols(h, nf_store_cols(h));
    for (int q = 0; q < h->T->n_queries; q++) {
        // Scheduler creation order (the TimestampGenerator's listener order)
        for (int si = 0; si < h->T->q[q].n_sched; si++) {
            const int p = h->T->q[q].sched_seq[si];
            // single process: the due pass runs while the replay thread applies the
            // last launches' history; the candidates' stamps (the scheduler map's
            // order) come from the models once it is done (host_stamps). Key-sharded:
            // the ranks are current on the device (applied at each exchange)
            const bool host_stamps = h->sm_on && !h->coord_on;
            if (!host_stamps) {
                const int frc = nf_sev_flush(h);
                if (frc) return frc;
            }
            const int32_t nkeys = h->n_nkeys;
            unsigned long long nc = 0;
            if (nkeys > 0) {
                // due keys: the armed-key list (+ the keys armed since the last pass on
                // the first scheduler's pass, which also rebuilds the list)
                {
                    const bool list_pass = armed_flags(h) && h->n_arm_log.p;
                    const int rc = due_launch(q, p, list_pass, list_pass && first_pass);
                    if (rc) return rc;
                    if (list_pass) first_pass = false;
                    if (nf_sync(h, st) != hipSuccess) return fail(h, SH_E_HIP, "k_nfa_due");
                }
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
                if (host_stamps) {
                    const int rrc = nf_rank_sync(h);
                    if (rrc) return rrc;
                    nfd_cand_restamp(h->n_cand.as<nfd_cand>(), (int64_t)nc, h->n_rank[q * NF_MAX_PROC + p].as<uint64_t>(),
                                     st);
                }
                if (h->n_tmin.ensure_fresh(8)) return fail(h, SH_E_OOM, "timer tie-break");
                nfd_cand_tmin(h->n_cand.as<nfd_cand>(), (int64_t)nc, h->n_tmin.as<unsigned long long>(), st);
                hipMemcpyAsync(h->pin_rd.as<void>(PR_TMIN), h->n_tmin.p, 8, hipMemcpyDeviceToHost, st);
                if (nf_sync(h, st) != hipSuccess) return fail(h, SH_E_HIP, "k_cand_tmin");
                const int64_t tmin = (int64_t)*h->pin_rd.as<unsigned long long>(PR_TMIN);
                const int64_t range = now - tmin + 1;
                if (tmin >= 0 && range > 0 && range <= kTieBreakSlots) {
                    if (h->n_slot_s.ensure_fresh((size_t)range * 8) || h->n_slot_k.ensure_fresh((size_t)range * 4) ||
                        h->pin_out.ensure((size_t)range * 4))
                        return fail(h, SH_E_OOM, "timer tie-break");
                    nfd_cand_select(h->n_cand.as<nfd_cand>(), (int64_t)nc, tmin, range,
                                    h->n_slot_s.as<unsigned long long>(), h->n_slot_k.as<int32_t>(), st);
                    hipMemcpyAsync(h->pin_out.p, h->n_slot_k.p, (size_t)range * 4, hipMemcpyDeviceToHost, st);
                    if (nf_sync(h, st) != hipSuccess) return fail(h, SH_E_HIP, "k_cand_select");
                    const int32_t* sk = h->pin_out.as<int32_t>();
                    for (int64_t r = 0; r < range; r++)
                        if (sk[r] >= 0) sel.push_back(sk[r]);
                    picked = true;
                }
            }
            if (!picked) {
                std::vector<nfd_cand> cs(nc);
                if ((int64_t)nc <= kCandSpec)
                    memcpy(cs.data(), h->pin_cand.p, nc * sizeof(nfd_cand));
                else
                    hipMemcpy(cs.data(), h->n_cand.p, nc * sizeof(nfd_cand), hipMemcpyDeviceToHost);
                if (host_stamps) {
                    const int frc = nf_sev_flush(h);
                    if (frc) return frc;
                    const ShJMap& M = h->sm.maps[q * NF_MAX_PROC + p];
                    for (auto& c : cs) c.stamp = M.present(c.key) ? M.rank(c.key) : ~0ull;
                }
                int64_t tlo = INT64_MAX, thi = INT64_MIN;
                for (const auto& c : cs) {
                    tlo = std::min(tlo, c.t);
                    thi = std::max(thi, c.t);
                }
                const int64_t range = cs.empty() ? 0 : thi - tlo + 1;
                static const bool slots_off = getenv("SH_HOST_SLOTS") && getenv("SH_HOST_SLOTS")[0] == '0';
                if (!slots_off && !wall && range > 0 && range <= std::max<int64_t>(4 * (int64_t)nc, 65536)) {
                    // one slot per due millisecond: the least (stamp) candidate of each
                    // (TreeMultimap with a zero comparator keeps the first per time)
                    auto& sl = h->pick_slots;
                    sl.assign((size_t)range, nfd_cand{0, ~0ull, -1, 0});
                    for (const auto& c : cs) {
                        nfd_cand& o = sl[(size_t)(c.t - tlo)];
                        if (o.key < 0 || c.stamp < o.stamp) o = c;
                    }
                    for (const auto& o : sl)
                        if (o.key >= 0) sel.push_back(o.key);
                } else {
                    std::sort(cs.begin(), cs.end(), [](const nfd_cand& a, const nfd_cand& b) {
                        if (a.t != b.t) return a.t < b.t;
                        return a.stamp < b.stamp;
                    });
                    for (size_t i = 0; i < cs.size(); i++)
                        if (wall || i == 0 || cs[i].t != cs[i - 1].t) sel.push_back(cs[i].key);
                }
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
                nfd_zero2(h->w_cnt.p, (int64_t)n_idx * 4, h->n_ctl.p, 24, st);  // match counts + counter block
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
                if (nf_sync(h, st) != hipSuccess) return fail(h, SH_E_HIP, "device error in k_nfa_timer");
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
                    nf_sync(h, st);
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

int nf_start(sh_handle* h) {
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
    if (nf_sync(h, h->stream) != hipSuccess) return fail(h, SH_E_HIP, "k_nfa_start");
    h->tick++;
    return err ? fail(h, SH_E_STATE_OVERFLOW, "start state overflow") : SH_OK;
}

// InputHandler.send(Event[]) on the general engine: playback clock + due timers
// first (InputHandler.java:85-96), then the batch. index (key-sharded): the
// positions of this rank's events in the whole call of call_n events, whose last
// timestamp is call_last; the rank takes every step of the call even when it owns
// none of its events (the coordinator's exchanges are collectives).
int nf_push(sh_handle* h, const sh_batch* b, int64_t r0, const uint32_t* index, int64_t call_n,
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
    const int64_t n = b->n;
    hipStream_t st = h->stream;
    if (index && n == 0) {
        if (h->app.playback) {
            const int64_t last = index ? call_last : b->ts[b->n - 1];
            if (last >= h->clock) {
                h->clock = last;
                int rc = nf_timers(h, last);
                if (rc) return rc;
            }
        }
        // none of the call's events is ours: the launch still ticks and its
        // (empty) scheduler history joins the others'
        if (h->sm_on && nf_sev_ready(h, 0)) return fail(h, SH_E_OOM, "scheduler history");
        h->tick++;
        int rc = nf_sev_apply(h);
        h->seq_next += call_n;
        h->seq_staged0 = h->seq_next;
        return rc;
    }
    // the events are staged first (host copies and one upload), so this work overlaps
    // the last call's launch, which the timer pass below settles
    // staged in pinned memory (pin_in; the column copies of this call are complete);
    // the staging buffers alternate per call: the last call's launch may still read its own
    PinBuf& ps = h->pst ? h->pin_stage2 : h->pin_stage;
    DevBuf& ds = h->pst ? h->w_pstage2 : h->w_pstage;
    const size_t o_ts = 0, o_rows = (size_t)n * 8, o_keys = o_rows + (size_t)n * 4, o_sv = o_keys + (size_t)n * 4;
    if ((size_t)(o_sv + n) > ps.bytes || (size_t)(o_sv + n) > ds.bytes) {
        int src = nf_settle(h);  // (a reallocation waits for the device)
        if (src) return src;
    }
    if (ps.ensure(o_sv + (size_t)n)) return fail(h, SH_E_OOM, "pinned staging");
    uint8_t* sv = ps.as<uint8_t>(o_sv);
    uint32_t* rows = ps.as<uint32_t>(o_rows);
    int32_t* keys = ps.as<int32_t>(o_keys);
    memset(sv, (uint8_t)b->stream, (size_t)n);
    memcpy(ps.as<int64_t>(o_ts), b->ts, (size_t)n * 8);
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
    if (ds.ensure_fresh(o_sv + (size_t)n)) return fail(h, SH_E_OOM, "staging");
    hipMemcpyAsync(ds.p, ps.p, o_sv + (size_t)n, hipMemcpyHostToDevice, st);
    shd_batch B;
    B.ts = ds.as<int64_t>();
    B.stream = ds.as<uint8_t>() + o_sv;
    B.row = (const uint32_t*)(ds.as<uint8_t>() + o_rows);
    B.keys = h->partitioned ? (const int32_t*)(ds.as<uint8_t>() + o_keys) : nullptr;
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
    if (h->app.playback) {
        const int64_t last = index ? call_last : b->ts[b->n - 1];
        if (last >= h->clock) {
            h->clock = last;
            int rc = nf_timers(h, last);
            if (rc) return rc;
        }
    }
    {
        int src = nf_settle(h);  // the last call's launch completes (its work overlapped this staging)
        if (src) return src;
    }
    int rc = nf_process(h, B, nk, nf_store_cols(h), nullptr, nullptr, 0, &nrows, false, 0, nullptr, gidx, call_n);
    if (h->pend.on) h->pst ^= 1;
    h->seq_next += index ? call_n : n;
    h->seq_staged0 = h->seq_next;
    return rc;
}
