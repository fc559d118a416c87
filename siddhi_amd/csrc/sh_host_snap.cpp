// sh_host_snap.cpp -- sh_snapshot / sh_restore: the handle's processing state
// (State.snapshot / restore of the pattern processors) as one versioned image.
#include "sh_host_int.h"

// ---- snapshot / restore (State.snapshot / restore of the pattern processors,
// StreamPreStateProcessor.java:450-469, driven by SnapshotService.java:90-187,
// 333-430): one opaque, versioned image of everything the matcher carries between
// calls -- partial matches and their events (the column stores they index), the
// schedulers (queues, armed-key lists, HashMap-order models), per-key aggregates,
// the playback clock, sequence counters and undelivered output.

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

// the per-key records as the image's per-field arrays (the image layout predates them)
template <class T, class F>
static std::vector<T> jmap_field(const ShJMap& M, F get) {
    std::vector<T> v(M.nd.size());
    for (size_t i = 0; i < v.size(); i++) v[i] = get(M.nd[i]);
    return v;
}

void put_jmap(SnapW& w, const ShJMap& M) {
    using N = ShJMap::Node;
    w.vec(jmap_field<int32_t>(M, [](const N& x) { return x.h; }));
    w.vec(jmap_field<int32_t>(M, [](const N& x) { return x.nx; }));
    w.vec(jmap_field<int32_t>(M, [](const N& x) { return x.pv; }));
    w.vec(jmap_field<int32_t>(M, [](const N& x) { return x.pa; }));
    w.vec(jmap_field<int32_t>(M, [](const N& x) { return x.lf; }));
    w.vec(jmap_field<int32_t>(M, [](const N& x) { return x.rt; }));
    w.vec(jmap_field<uint8_t>(M, [](const N& x) { return x.fl; }));
    w.vec(jmap_field<uint64_t>(M, [](const N& x) { return x.code; }));
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
    std::vector<int32_t> h, nx, pv, pa, lf, rt;
    std::vector<uint8_t> fl;
    std::vector<uint64_t> code;
    r.vec(h);
    r.vec(nx);
    r.vec(pv);
    r.vec(pa);
    r.vec(lf);
    r.vec(rt);
    r.vec(fl);
    r.vec(code);
    M.nd.assign(h.size(), ShJMap::Node{0, 0, -1, -1, -1, -1, -1, 0});
    for (size_t i = 0; i < h.size(); i++) {
        ShJMap::Node& x = M.nd[i];
        x.h = h[i];
        x.nx = i < nx.size() ? nx[i] : -1;
        x.pv = i < pv.size() ? pv[i] : -1;
        x.pa = i < pa.size() ? pa[i] : -1;
        x.lf = i < lf.size() ? lf[i] : -1;
        x.rt = i < rt.size() ? rt[i] : -1;
        x.fl = i < fl.size() ? fl[i] : 0;
        x.code = i < code.size() ? code[i] : 0;
    }
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
        // settle the pending launch first (it queues its scheduler history), then
        // wait for the history thread: the image reads the models and ranks
        int frc = h->mode == 2 ? SH_OK : flush(h);
        if (!frc) frc = nf_sev_flush(h);
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
