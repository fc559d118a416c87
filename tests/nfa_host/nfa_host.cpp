// nfa_host.cpp — TEST INFRASTRUCTURE: the general engine's per-key logic
// (siddhi_amd/csrc/sh_nfa.h, the code k_nfa runs on the GPU) compiled for the
// CPU, driven exactly like sh_host.cpp drives k_nfa: each flush is segmented by
// key (stable), one NfLane walks each key segment, emissions are ordered by
// their (run index, ordinal) tag, playback timers run the same selection rule.
// tests/ use it to diff the kernel logic against the oracle without a GPU. The
// product (libsiddhi_hip.so) never runs this code on the host.
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "../../siddhi_amd/csrc/sh_jmap.h"
#include "../../siddhi_amd/csrc/sh_nfa.h"
#include "../../siddhi_amd/csrc/sh_nfa_lower.h"
#include "../../include/siddhi_hip.h"

namespace {

struct HostSink {
    std::vector<uint64_t> recs;
    int words = 0;
    uint64_t* slot(int w) {
        words = w;
        recs.resize(recs.size() + w);
        return recs.data() + recs.size() - w;
    }
};

struct Ev {
    int64_t ts;
    uint32_t row;
    uint64_t seq;
    int stream;
    uint32_t local;
    uint32_t batch;
};
struct SegEvents {
    const std::vector<Ev>* v;
    int64_t ts(int64_t k) const { return (*v)[k].ts; }
    uint32_t row(int64_t k) const { return (*v)[k].row; }
    uint64_t seq(int64_t k) const { return (*v)[k].seq; }
    int stream(int64_t k) const { return (*v)[k].stream; }
    uint32_t local(int64_t k) const { return (*v)[k].local; }
    uint32_t batch(int64_t k) const { return (*v)[k].batch; }
    bool joins(int64_t e, int64_t k) const { return local(e) == local(e - 1) + 1 && batch(e) == batch(k); }
};

struct OutRow {
    int32_t query;
    uint64_t seq;
    int64_t ts;
    std::vector<int64_t> v;
    std::vector<uint8_t> nul;
};

}  // namespace

struct nfh {
    nf_table T;
    std::string err;
    // column stores
    std::vector<std::vector<std::vector<uint8_t>>> cols, nuls;
    std::vector<std::vector<bool>> has_nul;
    std::vector<int64_t> rows;
    std::vector<uint64_t> kstate;
    int32_t nkeys = 0;
    int64_t clock = 0;
    uint64_t tick = 1;
    bool started = false;
    std::vector<OutRow> out;
    int caps[6] = {16, 32, 64, 32, 8, 4};
    // scheduler-map order models (as sh_host.cpp keeps them)
    bool sm_on = false;
    ShSchedModels sm;
    std::vector<uint64_t> sev;
    unsigned long long sev_n = 0;
    uint64_t next_seq = 0;  // sequence number of the next input event
    // key-sharded streaming (sh_coordinator, as sh_host.cpp drives it)
    bool coord_on = false;
    sh_coordinator coord{};
    std::vector<uint64_t> order;  // per output row: launch << 32 | position in the launch
    // List values: this launch's buffer (nf_cols.lst) and the lists handed out
    bool has_lists = false;
    std::vector<uint64_t> lst;
    unsigned long long lst_n = 0;
    std::vector<std::vector<int64_t>> listV;
    std::vector<std::vector<uint8_t>> listN;
};

static int width(int t) {
    switch (t) {
        case SH_T_LONG:
        case SH_T_DOUBLE: return 8;
        case SH_T_BOOL: return 1;
        default: return 4;
    }
}

static nf_cols host_cols(nfh* h) {
    nf_cols c;
    memset(&c, 0, sizeof(c));
    for (int s = 0; s < h->T.n_streams; s++)
        for (int a = 0; a < h->T.stream_nattr[s]; a++) {
            c.col[s][a] = h->cols[s][a].data();
            c.nul[s][a] = h->has_nul[s][a] ? h->nuls[s][a].data() : nullptr;
        }
    if (h->sm_on) {
        if (h->sev.size() < (1u << 20)) h->sev.resize(1u << 20);
        h->sev_n = 0;
        c.sev = h->sev.data();
        c.sev_ctr = &h->sev_n;
        c.sev_cap = h->sev.size() / 2;
    }
    if (h->has_lists) {
        if (h->lst.size() < 4096) h->lst.resize(4096);
        h->lst_n = 0;
        c.lst = h->lst.data();
        c.lst_ctr = &h->lst_n;
        c.lst_cap = h->lst.size();
    }
    return c;
}

// a launch's getState history -> the order models (key-sharded: every rank's)
static int apply_history(nfh* h) {
    if (!h->sm_on) return 0;
    const uint64_t* recs = h->sev.data();
    int64_t n = (int64_t)h->sev_n;
    if (h->coord_on) {
        const uint64_t* all = nullptr;
        int64_t n_all = 0;
        if (h->coord.history(h->coord.user, recs, n, &all, &n_all)) {
            h->err = "coordinator: history exchange failed";
            return -1;
        }
        recs = all;
        n = n_all;
    }
    h->sev_n = 0;
    if (n == 0) return 0;
    if (!h->sm.apply(recs, (size_t)n)) {
        h->err = "scheduler map beyond the rank encoding";
        return -4;
    }
    for (int s : h->sm.used) {
        h->sm.maps[s].dirty.clear();
        h->sm.maps[s].rerank_all = false;
    }
    return 0;
}

static void ensure_keys(nfh* h, int32_t n) {
    if (n <= h->nkeys) return;
    h->kstate.resize((size_t)n * h->T.key_words, 0);
    h->nkeys = n;
}

// grow every capacity named by the error bits; re-lay every key block
static bool grow(nfh* h, uint32_t err) {
    if (err & NF_E_LST) {
        h->lst.resize(h->lst.size() * 4);
        err &= ~(uint32_t)NF_E_LST;
        if (!err) return true;
    }
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
        return false;
    nf_table old = h->T;
    nf_set_caps(&h->T, c[0], c[1], c[2], c[3], c[4], c[5]);
    std::vector<uint64_t> ns((size_t)h->nkeys * h->T.key_words, 0);
    for (int32_t k = 0; k < h->nkeys; k++) {
        const uint64_t* src = h->kstate.data() + (size_t)k * old.key_words;
        uint64_t* dst = ns.data() + (size_t)k * h->T.key_words;
        dst[0] = src[0];
        for (int q = 0; q < h->T.n_queries; q++) {
            const nf_query& A = old.q[q];
            const nf_query& B = h->T.q[q];
            const uint64_t* s = src + A.q_off;
            uint64_t* d = dst + B.q_off;
            for (int w = 0; w < NF_QH_WORDS; w++) d[w] = s[w];
            for (int w = 0; w < A.n_proc * NF_PS_WORDS; w++) d[B.lay.off_pstate + w] = s[A.lay.off_pstate + w];
            for (int p = 0; p < A.n_proc; p++)
                for (int wh = 0; wh < 2; wh++) {
                    const uint32_t* sl = (const uint32_t*)(s + A.lay.off_lists) + ((int64_t)p * 2 + wh) * A.lay.list_cap;
                    uint32_t* dl = (uint32_t*)(d + B.lay.off_lists) + ((int64_t)p * 2 + wh) * B.lay.list_cap;
                    for (int i = 0; i < A.lay.list_cap; i++) dl[i] = sl[i];
                }
            for (int w = 0; w < nf_agg_words(A); w++) d[B.lay.off_agg + w] = s[A.lay.off_agg + w];
            for (int w = 0; w < 3; w++) d[B.lay.off_hold + w] = s[A.lay.off_hold + w];
            for (int w = 0; w < A.lay.hold_cap; w++) d[B.lay.off_hold + 3 + w] = s[A.lay.off_hold + 3 + w];
            for (int p = 0; p < A.n_proc; p++) {
                const uint64_t* sq = s + A.lay.off_sched + (int64_t)p * (2 + A.lay.sched_cap);
                uint64_t* dq = d + B.lay.off_sched + (int64_t)p * (2 + B.lay.sched_cap);
                const uint32_t head = (uint32_t)sq[0], n = (uint32_t)(sq[0] >> 32);
                dq[0] = (uint64_t)n << 32;  // re-based ring
                dq[1] = sq[1];
                for (uint32_t i = 0; i < n; i++) dq[2 + i] = sq[2 + (head + i) % A.lay.sched_cap];
            }
            for (int64_t w = 0; w < (int64_t)A.lay.se_cap * A.lay.se_words; w++) d[B.lay.off_se + w] = s[A.lay.off_se + w];
            for (int64_t w = 0; w < (int64_t)A.lay.node_cap * 2; w++) d[B.lay.off_node + w] = s[A.lay.off_node + w];
        }
    }
    h->kstate.swap(ns);
    memcpy(h->caps, c, sizeof(c));
    return true;
}

static void take_records(nfh* h, HostSink& sink, int32_t nq, uint64_t launch) {
    // records are appended per lane; order them by (tag index, ordinal)
    struct R {
        uint64_t tag;
        size_t off;
        int words;
    };
    std::vector<R> rs;
    size_t off = 0;
    while (off < sink.recs.size()) {
        const uint64_t* r = sink.recs.data() + off;
        const int q = (int)(r[2] >> 32);
        const int w = NF_REC_HDR + h->T.q[q].n_out;
        rs.push_back({r[0], off, w});
        off += w;
    }
    std::stable_sort(rs.begin(), rs.end(), [](const R& a, const R& b) {
        const uint32_t ia = (uint32_t)a.tag, ib = (uint32_t)b.tag;
        if (ia != ib) return ia < ib;
        return (a.tag >> 32) < (b.tag >> 32);
    });
    (void)nq;
    for (auto& x : rs) {
        const uint64_t* r = sink.recs.data() + x.off;
        OutRow o;
        o.query = (int32_t)(r[2] >> 32);
        o.ts = (int64_t)r[1];
        o.seq = r[3];
        const nf_query& Q = h->T.q[o.query];
        const int n = Q.n_out;
        for (int c = 0; c < n; c++) {
            int64_t v = (int64_t)r[NF_REC_HDR + c];
            if (Q.out_pc[c] == NF_PC_LIST) {
                // this launch's List buffer -> a list handed out with the row
                const uint64_t* L = h->lst.data() + v;
                const uint64_t len = L[0];
                std::vector<int64_t> lv(len);
                std::vector<uint8_t> ln(len);
                for (uint64_t i = 0; i < len; i++) {
                    lv[i] = (int64_t)L[1 + i];
                    ln[i] = (uint8_t)((L[1 + len + i / 64] >> (i % 64)) & 1);
                }
                v = (int64_t)h->listV.size();
                h->listV.push_back(std::move(lv));
                h->listN.push_back(std::move(ln));
            }
            o.v.push_back(v);
            o.nul.push_back((uint8_t)((r[2] >> c) & 1));
        }
        h->out.push_back(std::move(o));
        if (h->coord_on) h->order.push_back((launch << 32) | (uint32_t)x.tag);
    }
}

static NfLane<HostSink> make_lane(nfh* h, const nf_cols* C, HostSink* sink, int32_t key) {
    NfLane<HostSink> L;
    memset(&L, 0, sizeof(L));
    L.T = &h->T;
    L.C = C;
    L.kb = h->kstate.data() + (size_t)key * h->T.key_words;
    L.sink = sink;
    L.partitioned = h->T.partitioned;
    L.clock = h->clock;
    L.key = key;
    return L;
}

// Scheduler.onTimeChange for every scheduler (absent pre-state), in creation order.
// wall: the EventCaller form (outside playback) -- every due key fires, no
// collapse of equal due times
static int timers(nfh* h, int64_t now, bool wall = false) {
    if (!h->T.has_absent) return 0;
    for (int q = 0; q < h->T.n_queries; q++) {
        const nf_query& Q = h->T.q[q];
        for (int si = 0; si < Q.n_sched; si++) {
            const int p = Q.sched_seq[si];
            // due keys: head <= now; one key per distinct due time (TreeMultimap
            // with a zero comparator), the earliest-registered wins
            struct Cand {
                int64_t t;
                uint64_t stamp;
                int32_t key;
            };
            std::vector<Cand> cs;
            {
                nf_cols C = host_cols(h);
                for (int32_t k = 0; k < h->nkeys; k++) {
                    NfLane<HostSink> L = make_lane(h, &C, nullptr, k);
                    L.Q = &Q;
                    L.qb = L.kb + Q.q_off;
                    int64_t t;
                    if (!(L.sched(p)[1] >> 63) && h->T.partitioned) continue;
                    // rank: the key's position in the scheduler map's iteration order
                    const bool stamp_order = getenv("SH_NFAH_STAMP_ORDER") != nullptr;  // test control
                    const uint64_t rank = (h->sm_on && !stamp_order) ? h->sm.maps[q * NF_MAX_PROC + p].rank(k)
                                                                     : (L.sched(p)[1] & ~(1ull << 63));
                    if (L.sched_head(p, &t) && t <= now) cs.push_back({t, rank, k});
                }
            }
            // the fired keys with their positions in the firing order
            std::vector<std::pair<uint32_t, int32_t>> fire;
            if (h->coord_on) {
                std::vector<sh_due_cand> dc(cs.size());
                for (size_t i = 0; i < cs.size(); i++) dc[i] = {cs[i].t, cs[i].stamp, cs[i].key, 0};
                std::vector<int64_t> pos(cs.size(), -1);
                int64_t n_fire = 0;
                if (h->coord.select(h->coord.user, wall ? 1 : 0, dc.data(), (int64_t)dc.size(), pos.data(), &n_fire)) {
                    h->err = "coordinator: select failed";
                    return -1;
                }
                if (n_fire == 0) continue;
                for (size_t i = 0; i < cs.size(); i++)
                    if (pos[i] >= 0) fire.emplace_back((uint32_t)pos[i], cs[i].key);
                std::sort(fire.begin(), fire.end());
            } else {
                if (cs.empty()) continue;
                std::sort(cs.begin(), cs.end(), [](const Cand& a, const Cand& b) {
                    if (a.t != b.t) return a.t < b.t;
                    return a.stamp < b.stamp;
                });
                uint32_t rank = 0;
                for (size_t i = 0; i < cs.size(); i++) {
                    if (i && cs[i].t == cs[i - 1].t && !wall) continue;
                    fire.emplace_back(rank++, cs[i].key);
                }
            }
            // sendTimerEvents per fired key (state growth: restore, grow, replay)
            HostSink sink;
            for (int attempt = 0;; attempt++) {
                if (attempt >= 40) {
                    h->err = "state overflow in timers";
                    return -5;
                }
                std::vector<uint64_t> backup = h->kstate;
                nf_cols C = host_cols(h);
                sink = HostSink();
                uint32_t err = 0;
                for (auto& f : fire) {
                    NfLane<HostSink> L = make_lane(h, &C, &sink, f.second);
                    L.Q = &Q;
                    L.qb = L.kb + Q.q_off;
                    L.qi = q;
                    L.tag_index = f.first;
                    L.cur_seq = h->next_seq;
                    L.stamp = (h->tick << 32) | L.tag_index;
                    L.send_timer_events(p, now);
                    err |= L.err;
                }
                if (!err) break;
                h->kstate.swap(backup);
                if ((err & (NF_E_UNSUP | NF_E_EMIT | NF_E_KEY)) || !grow(h, err)) {
                    h->err = "state overflow / unsupported in timers";
                    return -5;
                }
            }
            h->tick++;
            take_records(h, sink, h->T.n_queries, h->tick - 1);
            const int rc = apply_history(h);
            if (rc) return rc;
        }
    }
    return 0;
}

extern "C" {

nfh* nfh_create(const sh_app_desc* d, char* err, int errlen) {
    nfh* h = new nfh();
    std::string e;
    if (nf_lower(d, &h->T, &e)) {
        if (err && errlen > 0) snprintf(err, errlen, "%s", e.c_str());
        delete h;
        return nullptr;
    }
    h->cols.resize(d->n_streams);
    h->nuls.resize(d->n_streams);
    h->has_nul.resize(d->n_streams);
    h->rows.assign(d->n_streams, 0);
    for (int s = 0; s < d->n_streams; s++) {
        h->cols[s].resize(d->streams[s].n_attrs);
        h->nuls[s].resize(d->streams[s].n_attrs);
        h->has_nul[s].assign(d->streams[s].n_attrs, false);
    }
    nf_set_caps(&h->T, h->caps[0], h->caps[1], h->caps[2], h->caps[3], h->caps[4], h->caps[5]);
    for (int q = 0; q < h->T.n_queries; q++)
        for (int o = 0; o < h->T.q[q].n_out; o++)
            if (h->T.q[q].out_pc[o] == NF_PC_LIST) h->has_lists = true;
    if (h->T.partitioned && h->T.has_absent) {
        std::vector<int> ids;
        for (int q = 0; q < h->T.n_queries; q++)
            for (int p = 0; p < h->T.q[q].n_proc; p++)
                if (nf_has_sched(h->T.q[q].proc[p])) ids.push_back(q * NF_MAX_PROC + p);
        h->sm_on = true;
        h->sm.init(ids, NF_MAX_QUERIES * NF_MAX_PROC);
    }
    return h;
}

int nfh_set_partition_keys(nfh* h, int32_t first, int32_t n, const uint16_t* utf16, const int64_t* offsets) {
    h->sm.set_keys(first, n, utf16, offsets);
    return 0;
}

int nfh_start(nfh* h) {
    if (h->started) return 0;
    h->started = true;
    if (h->T.partitioned) return 0;
    ensure_keys(h, 1);
    nf_cols C = host_cols(h);
    HostSink sink;
    NfLane<HostSink> L = make_lane(h, &C, &sink, 0);
    L.kb[0] |= 1ull;
    for (int q = 0; q < h->T.n_queries; q++) {
        L.Q = &h->T.q[q];
        L.qb = L.kb + L.Q->q_off;
        L.qi = q;
        L.stamp = h->tick << 32;
        L.init_partition();
    }
    h->tick++;
    return L.err ? -5 : 0;
}

// earliest queued notify time over every scheduler and key
static int64_t next_due(nfh* h) {
    int64_t tmin = INT64_MAX;
    if (!h->T.has_absent) return tmin;
    nf_cols C = host_cols(h);
    for (int q = 0; q < h->T.n_queries; q++) {
        const nf_query& Q = h->T.q[q];
        for (int si = 0; si < Q.n_sched; si++) {
            const int p = Q.sched_seq[si];
            for (int32_t k = 0; k < h->nkeys; k++) {
                NfLane<HostSink> L = make_lane(h, &C, nullptr, k);
                L.Q = &Q;
                L.qb = L.kb + Q.q_off;
                int64_t t;
                if (!(L.sched(p)[1] >> 63) && h->T.partitioned) continue;
                if (L.sched_head(p, &t)) tmin = std::min(tmin, t);
            }
        }
    }
    return tmin;
}

static int64_t next_due_all(nfh* h) {
    int64_t t = next_due(h), g = t;
    if (h->coord_on && h->coord.min_time(h->coord.user, t, &g)) return INT64_MIN;
    return g;
}

int nfh_advance_time(nfh* h, int64_t now) {
    if (now < h->clock) return 0;
    if (!h->T.playback) {
        // wall clock: step through every queued notify time
        for (;;) {
            const int64_t t = next_due_all(h);
            if (t == INT64_MIN) return -1;
            if (t > now) break;
            h->clock = std::max(h->clock, t);
            const int rc = timers(h, h->clock, true);
            if (rc) return rc;
        }
        h->clock = now;
        return 0;
    }
    h->clock = now;
    return timers(h, now);
}

// index (key-sharded): positions of this rank's events in the whole call of
// call_n events whose last timestamp is call_last (the rank takes every step)
static int send_impl(nfh* h, const sh_batch* b, uint64_t first_seq, const uint32_t* index, int64_t call_n,
                     int64_t call_last) {
    if (b->n <= 0 && !index) return 0;
    const int s = b->stream;
    const int64_t r0 = h->rows[s];
    for (int a = 0; a < h->T.stream_nattr[s]; a++) {
        const int w = width(h->T.attr_type[s][a]);
        auto& col = h->cols[s][a];
        col.resize((size_t)(r0 + b->n) * w);
        memcpy(col.data() + r0 * w, b->cols[a], (size_t)b->n * w);
        const uint8_t* nm = b->nulls ? b->nulls[a] : nullptr;
        auto& nc = h->nuls[s][a];
        nc.resize((size_t)(r0 + b->n), 0);
        if (nm) {
            memcpy(nc.data() + r0, nm, b->n);
            h->has_nul[s][a] = true;
        }
    }
    h->rows[s] += b->n;
    // InputHandler.send in playback: clock -> last timestamp, due timers first
    h->next_seq = first_seq;
    if (h->T.playback) {
        int rc = nfh_advance_time(h, index ? call_last : b->ts[b->n - 1]);
        if (rc) return rc;
    }
    h->next_seq = first_seq + (uint64_t)(index ? call_n : b->n);
    // stable segment by key (null keys dropped)
    std::vector<Ev> evs;
    int32_t maxk = 0;
    for (int64_t i = 0; i < b->n; i++) {
        int32_t k = h->T.partitioned ? (b->keys ? b->keys[i] : 0) : 0;
        if (k < 0) continue;
        maxk = std::max(maxk, k + 1);
    }
    ensure_keys(h, std::max(maxk, 1));
    std::vector<std::vector<Ev>> byKey(std::max(maxk, 1));
    for (int64_t i = 0; i < b->n; i++) {
        int32_t k = h->T.partitioned ? (b->keys ? b->keys[i] : 0) : 0;
        if (k < 0) continue;
        const uint32_t at = index ? index[i] : (uint32_t)i;  // position in the call
        byKey[k].push_back({b->ts[i], (uint32_t)(r0 + i), first_seq + at, s, at, 0});
    }
    for (int attempt = 0; attempt < 40; attempt++) {
        std::vector<uint64_t> backup = h->kstate;
        nf_cols C = host_cols(h);
        HostSink sink;
        uint32_t err = 0;
        for (size_t k = 0; k < byKey.size() && !err; k++) {
            if (byKey[k].empty()) continue;
            NfLane<HostSink> L = make_lane(h, &C, &sink, (int32_t)k);
            SegEvents E{&byKey[k]};
            nf_process_segment(L, E, 0, (int64_t)byKey[k].size(), h->tick, nullptr);
            err |= L.err;
        }
        if (!err) {
            h->tick++;
            take_records(h, sink, h->T.n_queries, h->tick - 1);
            return apply_history(h);
        }
        h->kstate.swap(backup);
        if ((err & (NF_E_UNSUP | NF_E_EMIT | NF_E_KEY)) || !grow(h, err)) {
            h->err = (err & NF_E_UNSUP) ? "unsupported reference behaviour" : "state overflow";
            return -5;
        }
    }
    return -5;
}

int nfh_send(nfh* h, const sh_batch* b, uint64_t first_seq) { return send_impl(h, b, first_seq, nullptr, 0, 0); }

int nfh_send_part(nfh* h, const sh_batch* b, uint64_t first_seq, const uint32_t* index, int64_t call_n,
                  int64_t call_last) {
    static const uint32_t none = 0;
    if (!h->coord_on || call_n <= 0) return -1;
    return send_impl(h, b, first_seq, index ? index : &none, call_n, call_last);
}

int nfh_set_coordinator(nfh* h, const sh_coordinator* c) {
    if (!c || !c->history || !c->select || !c->min_time || !h->T.partitioned || h->started) return -1;
    h->coord = *c;
    h->coord_on = true;
    return 0;
}

int64_t nfh_list_get(nfh* h, int64_t list, int64_t cap, int64_t* values, uint8_t* nulls) {
    if (list < 0 || list >= (int64_t)h->listV.size()) return -1;
    const auto& v = h->listV[list];
    for (int64_t i = 0; i < (int64_t)v.size() && i < cap; i++) {
        if (values) values[i] = v[i];
        if (nulls) nulls[i] = h->listN[list][i];
    }
    return (int64_t)v.size();
}

int nfh_out_order(nfh* h, int64_t start, int64_t count, uint64_t* order) {
    if (!h->coord_on || start < 0 || start + count > (int64_t)h->order.size()) return -1;
    memcpy(order, h->order.data() + start, (size_t)count * 8);
    return 0;
}

int64_t nfh_out_count(nfh* h) { return (int64_t)h->out.size(); }

int nfh_out_read(nfh* h, int64_t start, int64_t count, int32_t* query, uint64_t* seq, int64_t* ts, int64_t* values,
                 uint8_t* nulls, int32_t n_out) {
    if (start < 0 || start + count > (int64_t)h->out.size()) return -1;
    for (int64_t i = 0; i < count; i++) {
        const OutRow& r = h->out[start + i];
        if (query) query[i] = r.query;
        if (seq) seq[i] = r.seq;
        if (ts) ts[i] = r.ts;
        for (int c = 0; c < n_out; c++) {
            const bool has = c < (int)r.v.size();
            if (values) values[i * n_out + c] = has ? r.v[c] : 0;
            if (nulls) nulls[i * n_out + c] = has ? r.nul[c] : 1;
        }
    }
    return 0;
}

const char* nfh_last_error(nfh* h) { return h->err.c_str(); }

void nfh_destroy(nfh* h) { delete h; }

}  // extern "C"
