// sh_host_fast.cpp -- drivers of the fast batch engines behind sh_run_device:
// the rule engine (sh_rules.hip), the tile-local bucketed window engine and the
// sequence bucket-carry engine (sh_bucket.hip + shb_match), the aggregate post-pass
// (sh_agg.hip), and the key-segment helpers they share.
#include "sh_host_int.h"

int bits_for(uint64_t v) {
    int b = 0;
    while (b < 64 && (v >> b)) b++;
    return b;
}

shd_segment_ws seg_ws(sh_handle* h, int64_t n) {
    shd_segment_ws ws;
    ws.keys_a = h->w_keys_a.as<uint32_t>();
    ws.keys_b = h->w_keys_b.as<uint32_t>();
    ws.idx_a = h->w_idx_a.as<uint32_t>();
    ws.idx_b = h->w_idx_b.as<uint32_t>();
    ws.hist = h->w_hist.as<uint32_t>();
    ws.scan_tmp = h->w_scan.as<uint32_t>();
    ws.seg_off = h->w_seg.as<uint32_t>();
    ws.cap = n;
    return ws;
}

// ts and every column of stream 0 moved into key-segment order by the segment
// A 4-byte column that is the key array itself (the partition attribute, passed
// as the same device buffer) is not carried: its key-segment order is the
// sorted key array (*alias = that attribute, -1 if none). Null-key events
// (sorted to the sentinel bucket) are never read.
int carry_setup(sh_handle* h, const sh_device_run* run, shd_payload* carry, void** mid, int* alias,
                       bool used_only, bool with_ts) {
    const int64_t n = run->n;
    const int na = (int)h->stream_types[0].size();
    memset(carry, 0, sizeof(*carry));
    *alias = -1;
    int c = 0;
    if (with_ts) {
        if (h->v_sts.ensure_fresh(n * 8) || h->v_mid_ts.ensure_fresh(n * 8)) return SH_E_OOM;
        carry->src[c] = run->d_ts;
        carry->dst[c] = h->v_sts.p;
        carry->width[c] = 8;
        mid[c++] = h->v_mid_ts.p;
    }
    for (int a = 0; a < na; a++) {
        const int w = type_width(h->stream_types[0][a]);
        if (used_only && h->T && a < 32 && !((h->T->attr_used[0] >> a) & 1u)) continue;  // no expression reads it
        if (*alias < 0 && w == 4 && run->d_cols[a] == (const void*)run->d_keys && !getenv("SH_NO_KEY_ALIAS")) {
            *alias = a;
            continue;
        }
        if (h->v_scol[a].ensure_fresh(n * w) || h->v_mid[a].ensure_fresh(n * w)) return SH_E_OOM;
        carry->src[c] = run->d_cols[a];
        carry->dst[c] = h->v_scol[a].p;
        carry->width[c] = (uint8_t)w;
        mid[c++] = h->v_mid[a].p;
    }
    carry->n = c;
    return SH_OK;
}

// log2 of the arrival tile (0: untiled) for a partitioned window run: tiles of
// 2^19 events when the stream spans several and the directory stays small
// (SH_TILE_SHIFT overrides, for tests)
int tile_shift_for(int64_t n, int32_t nkeys) {
    int shift = 19;
    if (const char* e = getenv("SH_TILE_SHIFT")) shift = atoi(e);
    if (shift < 12 || shift > 24) return 0;
    const int64_t ntile = (n + ((int64_t)1 << shift) - 1) >> shift;
    if (ntile < 2 || ntile * ((int64_t)nkeys + 1) > ((int64_t)1 << 26)) return 0;
    return shift;
}

// batch-compiled rule sets (sh_rules.hip) over HBM-resident columns

// the records' output order -- (run, query, consuming event), stable over the
// records' (opening event, rule) order; by_p: the records are in any order, so
// the first sort stage restores that order -- and the placed rows
static int rules_order_place(sh_handle* h, sh_device_run* run, int64_t m, const uint32_t* rec_p, const uint32_t* rec_q,
                             const uint32_t* rec_r, const uint32_t* perm, const int64_t* sts, const shd_cols* dC,
                             const uint32_t* sts32, int64_t tlo, bool sorted, bool by_p) {
    hipStream_t st = h->stream;
    const int64_t n = run->n;
    const shr_table* dT = h->rd_tab.as<shr_table>();
    const int64_t mt = (m + 4095) / 4096;
    const size_t sw = std::max(shd_scan_tmp_words(256 * mt), (size_t)16);
    if (h->r_keys.ensure_fresh((size_t)m * 12) || h->r_g.ensure_fresh((size_t)m * 8) ||
        h->r_sk.ensure_fresh((size_t)m * 8) || h->r_sv.ensure_fresh((size_t)m * 8) ||
        h->r_hist.ensure_fresh((size_t)256 * mt * 4 + 64) || h->r_scan.ensure_fresh(sw * 4 + 64))
        return fail(h, SH_E_OOM, "match records");
    // PartitionStreamReceiver runs inside each send() call
    const int64_t batch = run->batch_events > 0 ? run->batch_events : 0;
    const uint32_t* flags = nullptr;
    const uint32_t* rid = nullptr;
    const uint32_t* rfirst = nullptr;
    // the runs of the consuming events only, walked back from each record's event
    // (SH_RULES_RUNSCAN=1: flags, scan and first index over every event)
    const bool walk_runs = sorted && !getenv("SH_RULES_RUNSCAN");
    // order key (run, query, consuming event), least significant first; the
    // records are in (opening event, rule) order, which the stable sort keeps
    // among equal keys (creation order of the partials a consumer takes)
    const int64_t runlen = batch > 0 ? std::min(batch, n) : n;
    const int qbits = bits_for((uint64_t)(runlen - 1));
    const int rbits = bits_for((uint64_t)(h->r_rules.size() - 1));
    const int nbits = bits_for((uint64_t)(n - 1));
    const bool packed = qbits + rbits <= 32;
    uint32_t* k0 = h->r_keys.as<uint32_t>();
    uint32_t* k1 = k0 + m;
    uint32_t* k2 = k1 + m;
    bool scan_runs = sorted && !walk_runs;
    if (walk_runs) {
        int32_t* long_run = h->v_flag.as<int32_t>() + 1;
        int32_t lr = 0;
        hipMemsetAsync(long_run, 0, 4, st);
        if (shr_keys(rec_q, rec_r, m, perm, nullptr, nullptr, nullptr, batch, qbits, packed ? 1 : 0, k0, k1, k2,
                     st, run->d_keys, run->d_run, long_run))
            return fail(h, SH_E_HIP, "rule key launch failed");
        hipMemcpyAsync(&lr, long_run, 4, hipMemcpyDeviceToHost, st);
        if (hipStreamSynchronize(st) != hipSuccess) return fail(h, SH_E_HIP, "device error in the rule keys");
        scan_runs = lr != 0;
    }
    if (scan_runs) {
        if (h->r_run.ensure_fresh((size_t)n * 12)) return fail(h, SH_E_OOM, "run ids");
        uint32_t* f = h->r_run.as<uint32_t>();
        if (shr_run_ids(run->d_keys, run->d_run, n, batch, f, f + n, f + 2 * n, h->w_scan.as<uint32_t>(), st))
            return fail(h, SH_E_HIP, "run id launch failed");
        flags = f;
        rid = f + n;
        rfirst = f + 2 * n;
    }
    if ((scan_runs || !walk_runs) &&
        shr_keys(rec_q, rec_r, m, perm, flags, rid, rfirst, batch, qbits, packed ? 1 : 0, k0, k1, k2, st))
        return fail(h, SH_E_HIP, "rule key launch failed");
    const uint32_t* stage_key[4];
    int stage_bits[4];
    int ns = 0;
    // by_p (records in any order): no stage by opening event -- four radix passes --
    // but the last stage's runs of equal keys put in rec_p order afterwards
    // (shr_order_ties; profiles/r6_c5_ties_ab.txt: advance -0.11 ms)
    const bool ties = by_p;
    if (packed) {
        stage_key[ns] = k0;
        stage_bits[ns++] = qbits + rbits;
    } else {
        stage_key[ns] = k0;
        stage_bits[ns++] = qbits;
        stage_key[ns] = k1;
        stage_bits[ns++] = rbits;
    }
    stage_key[ns] = packed ? k1 : k2;
    stage_bits[ns++] = nbits;
    const uint32_t* order = nullptr;
    uint32_t* gk = h->r_g.as<uint32_t>();
    uint32_t* gv = gk + m;
    uint32_t* kb[2] = {h->r_sk.as<uint32_t>(), h->r_sk.as<uint32_t>() + m};
    uint32_t* vb[2] = {h->r_sv.as<uint32_t>(), h->r_sv.as<uint32_t>() + m};
    for (int s = 0; s < ns; s++) {
        if (stage_bits[s] == 0) continue;
        const uint32_t* ko = nullptr;
        const uint32_t* vo = nullptr;
        if (shr_gather(stage_key[s], order, m, gk, gv, st) ||
            shd_sort_pairs(gk, gv, m, stage_bits[s], kb, vb, h->r_hist.as<uint32_t>(), h->r_scan.as<uint32_t>(),
                           st, &ko, &vo))
            return fail(h, SH_E_HIP, "rule sort launch failed");
        order = vo;
    }
    if (ties && !order) {  // (every stage empty: the identity order, in a buffer of ours)
        if (shr_gather(k0, nullptr, m, h->r_g.as<uint32_t>(), h->r_g.as<uint32_t>() + m, st))
            return fail(h, SH_E_HIP, "rule order launch failed");
        order = h->r_g.as<uint32_t>() + m;
    }
    if (ties &&
        shr_order_ties(const_cast<uint32_t*>(order), m, k0, k1, packed ? nullptr : k2, rec_p, st))
        return fail(h, SH_E_HIP, "rule order launch failed");
    hipEventRecord(h->ev[2], st);
    if (h->r_aggp) {
        if (!run->d_out_query) {
            if (h->a_q.ensure((size_t)m * 4)) return fail(h, SH_E_OOM, "aggregate query ids");
            run->d_out_query = h->a_q.as<int32_t>();
        }
        if (!run->d_out_seq) {
            if (h->a_seq.ensure((size_t)m * 8)) return fail(h, SH_E_OOM, "aggregate sequence numbers");
            run->d_out_seq = h->a_seq.as<uint64_t>();
        }
    }
    if (shr_place(dT, order, m, rec_p, rec_q, rec_r, perm, sts, dC, 0, std::max(1, h->n_out), run->d_out_seq,
                  run->d_out_query, nullptr, run->d_out_values, st, sts32, tlo))
        return fail(h, SH_E_HIP, "rule placement launch failed");
    return SH_OK;
}

// the end of a rule run: kernel times, the aggregate post-pass
static int rules_finish(sh_handle* h, sh_device_run* run, int64_t m, int32_t nkeys) {
    hipStream_t st = h->stream;
    hipEventRecord(h->ev[3], st);
    if (hipStreamSynchronize(st) != hipSuccess) return fail(h, SH_E_HIP, "device error in the rule engine");
    hipEventElapsedTime(&h->times.segment_ms, h->ev[0], h->ev[1]);
    hipEventElapsedTime(&h->times.advance_ms, h->ev[1], h->ev[2]);
    hipEventElapsedTime(&h->times.emit_ms, h->ev[2], h->ev[3]);
    hipEventElapsedTime(&h->times.total_ms, h->ev[0], h->ev[3]);
    h->times.advance_launches = 1;
    if (h->r_aggp && m > 0) {
        const int arc = agg_post(h, run, nkeys, run->d_out_query, (int)h->r_rules.size(), h->r_agg, h->r_argt,
                                 std::max(1, h->n_out));
        if (arc < 0) return arc;
        if (arc == 1) return 1;  // not exact in parallel: the caller runs the general engine
    }
    return SH_OK;
}

// partitioned rule sets whose start filters open few partials: no key segment
// (sh_rules.hip, "sparse partials"); 1 = not taken (decreasing timestamps, keys
// out of range, more partials than max(65536, n / 8) or than 64 per key): the
// caller runs the key-segment path.
// Phases: segment = the partials and their lists, advance = the consuming events
// and the records' order, emit = placement.
static int run_rules_sparse(sh_handle* h, sh_device_run* run, int32_t nkeys) {
    h->rs_last = 0;
    if (const char* e = getenv("SH_RULES_SPARSE"))
        if (e[0] == '0') return 1;
    hipStream_t st = h->stream;
    const int64_t n = run->n;
    if (n <= 1 || n >= (int64_t)0xFFFFFFFFll || !run->d_keys) return 1;
    if (h->r_rules.size() >= ((size_t)1 << 20)) return 1;  // (k_sparse_open's pairs hold 20-bit rule ids)
    const int64_t cap = std::max<int64_t>(65536, n / 8);
    const size_t nk1 = (size_t)nkeys + 1;
    if (h->rs_pr.ensure_fresh((size_t)cap * 16) || h->rs_key.ensure_fresh(nk1 * 12) ||
        h->rs_list.ensure_fresh((size_t)cap * 20) || h->rs_ctl.ensure_fresh(64) || ensure_ws(h, (int64_t)nk1))
        return fail(h, SH_E_OOM, "rule workspace");
    uint32_t* pr = h->rs_pr.as<uint32_t>();
    uint32_t* key_cnt = h->rs_key.as<uint32_t>();
    uint32_t* key_off = key_cnt + nk1;
    uint32_t* key_fill = key_off + nk1;
    unsigned long long* ctl = h->rs_ctl.as<unsigned long long>();  // [0] partials, [1] records, [2] flag
    shd_cols sc;
    memset(&sc, 0, sizeof(sc));
    const int na = (int)h->stream_types[0].size();
    for (int a = 0; a < na; a++) sc.col[0][a] = run->d_cols[a];
    hipEventRecord(h->ev[0], st);
    hipMemcpyAsync(h->d_cols_desc.p, &sc, sizeof(sc), hipMemcpyHostToDevice, st);
    const shd_cols* dC = h->d_cols_desc.as<shd_cols>();
    const shr_table* dT = h->rd_tab.as<shr_table>();
    hipMemsetAsync(key_cnt, 0, nk1 * 4, st);
    hipMemsetAsync(key_fill, 0, nk1 * 4, st);
    hipMemsetAsync(ctl, 0, 24, st);
    // the attributes the rules' terms read most on the opening event's row (f1) and on
    // the consumer's row (f2): loaded once per event by the sparse kernels
    int32_t pre_open[2] = {-1, -1}, pre_take[2] = {-1, -1};
    {
        int cnt0[32] = {0}, cnt1[32] = {0};
        for (const shr_rule& R : h->r_rules) {
            for (int t = 0; t < R.nt[0]; t++) {
                const shp_term& T = R.t[0][t];
                if (T.lslot == 0 && T.lattr >= 0 && T.lattr < 32) cnt0[T.lattr]++;
                if (T.rkind != 1 && T.rslot == 0 && T.rattr >= 0 && T.rattr < 32) cnt0[T.rattr]++;
            }
            for (int t = 0; t < R.nt[1]; t++) {
                const shp_term& T = R.t[1][t];
                if (T.lslot == 1 && T.lattr >= 0 && T.lattr < 32) cnt1[T.lattr]++;
                if (T.rkind != 1 && T.rslot == 1 && T.rattr >= 0 && T.rattr < 32) cnt1[T.rattr]++;
            }
        }
        auto top2 = [](const int* c, int32_t* out) {
            for (int k = 0; k < 2; k++) {
                int best = -1;
                for (int a = 0; a < 32; a++)
                    if (c[a] > 0 && a != out[0] && (best < 0 || c[a] > c[best])) best = a;
                out[k] = best;
            }
        };
        top2(cnt0, pre_open);
        top2(cnt1, pre_take);
    }
    if (shr_sparse_open(dT, run->d_ts, run->d_keys, n, nkeys, dC, h->r_img.bytes ? h->rd_img.as<uint8_t>() : nullptr,
                        &h->r_img, pr, pr + cap, pr + 2 * cap, key_cnt, ctl, cap, (int32_t*)(ctl + 2), pre_open,
                        st))
        return fail(h, SH_E_HIP, "sparse partial launch failed");
    unsigned long long rd[5] = {0, 0, 0, 0, 0};
    hipMemcpyAsync(rd, ctl, 24, hipMemcpyDeviceToHost, st);
    hipMemcpyAsync(rd + 3, run->d_ts, 8, hipMemcpyDeviceToHost, st);
    hipMemcpyAsync(rd + 4, run->d_ts + (n - 1), 8, hipMemcpyDeviceToHost, st);
    if (hipStreamSynchronize(st) != hipSuccess) return fail(h, SH_E_HIP, "device error in the sparse partials");
    const int64_t np = (int64_t)rd[0];
    // a key's events each test all of its key's partials: dense partials per key take
    // the key-segment path (whose walk stops at each partial's window)
    if (rd[2] || np > cap || np > (int64_t)64 * nkeys) return 1;
    if (shd_exclusive_scan(key_cnt, key_off, (int64_t)nk1, h->w_scan.as<uint32_t>(), st))
        return fail(h, SH_E_HIP, "scan");
    hipEventRecord(h->ev[1], st);
    uint32_t* l_p = h->rs_list.as<uint32_t>();
    uint32_t* l_r = l_p + cap;
    uint32_t* l_q = l_r + cap;
    int64_t* l_te = (int64_t*)(l_q + cap);
    const int64_t rcap = std::max<int64_t>(np, 1);
    if (h->r_rec.ensure_fresh((size_t)rcap * 12)) return fail(h, SH_E_OOM, "match records");
    // the live-partial bitmap (shr_live): the run's time span in <= SH_SPARSE_SLICES
    // (default 256) power-of-two slices, one bit per key and slice (SH_SPARSE_LIVE=0: off)
    shr_live LV;
    memset(&LV, 0, sizeof(LV));
    {
        static const bool live_off = getenv("SH_SPARSE_LIVE") && getenv("SH_SPARSE_LIVE")[0] == '0';
        static const int max_sl = getenv("SH_SPARSE_SLICES") ? std::max(1, atoi(getenv("SH_SPARSE_SLICES"))) : 256;
        const int64_t tmin = (int64_t)rd[3], span = (int64_t)rd[4] - tmin + 1;
        if (!live_off && span > 0) {
            int shift = 0;
            while (shift < 62 && ((span - 1) >> shift) + 1 > max_sl) shift++;
            LV.tmin = tmin;
            LV.shift = shift;
            LV.nslices = (int32_t)(((span - 1) >> shift) + 1);
            LV.wps = (nkeys + 31) / 32;
            const size_t bytes = (size_t)LV.nslices * LV.wps * 4;
            if (h->rs_live.ensure(bytes)) return fail(h, SH_E_OOM, "live bitmap");
            LV.bits = h->rs_live.as<uint32_t>();
            hipMemsetAsync(LV.bits, 0, bytes, st);
        }
    }
    uint32_t* rec_p = h->r_rec.as<uint32_t>();
    uint32_t* rec_q = rec_p + rcap;
    uint32_t* rec_r = rec_q + rcap;
    if (np > 0 &&
        shr_sparse_match(dT, run->d_ts, run->d_keys, n, dC, h->r_img.bytes ? h->rd_img.as<uint8_t>() : nullptr,
                         &h->r_img, pr, pr + cap, pr + 2 * cap, key_fill, ctl, np, key_off,
                         l_p, l_r, l_te, l_q, rec_p, rec_q, rec_r, ctl + 1, rcap, nkeys, &LV, pre_take, st))
        return fail(h, SH_E_HIP, "sparse match launch failed");
    hipMemcpyAsync(rd, ctl, 16, hipMemcpyDeviceToHost, st);
    if (hipStreamSynchronize(st) != hipSuccess) return fail(h, SH_E_HIP, "device error in the sparse match");
    const int64_t m = (int64_t)rd[1];
    h->rs_last = 1;
    run->out_count = m;
    if (m > run->out_capacity) return fail(h, SH_E_MORE, "output capacity too small");
    if (m > 0) {
        // the records' arrays hold rcap entries each: compact them for the order stages
        if (m < rcap) {
            hipMemcpyAsync(rec_p + m, rec_q, (size_t)m * 4, hipMemcpyDeviceToDevice, st);
            hipMemcpyAsync(rec_p + 2 * m, rec_r, (size_t)m * 4, hipMemcpyDeviceToDevice, st);
        }
        int prc = rules_order_place(h, run, m, rec_p, rec_p + m, rec_p + 2 * m, nullptr, run->d_ts, dC, nullptr, 0,
                                    true, true);
        if (prc) return prc;
    } else {
        hipEventRecord(h->ev[2], st);
    }
    return rules_finish(h, run, m, nkeys);
}

int run_rules(sh_handle* h, sh_device_run* run) {
    hipStream_t st = h->stream;
    const int64_t n = run->n;
    const int na = (int)h->stream_types[0].size();
    if (na > 7) return fail(h, SH_E_UNSUPPORTED, "rule engine: at most 7 attributes per stream");
    const bool sorted = h->r_partitioned;
    const int32_t nkeys = sorted ? std::max(1, run->n_keys) : 1;
    if (ensure_ws(h, n) || h->v_flag.ensure_fresh(64)) return fail(h, SH_E_OOM, "workspace");
    h->times = sh_kernel_times{};
    if (sorted) {
        const int src = run_rules_sparse(h, run, nkeys);
        if (src != 1) return src;
    }
    shd_batch B;
    memset(&B, 0, sizeof(B));
    B.ts = run->d_ts;
    B.keys = sorted ? run->d_keys : nullptr;
    B.n = n;
    shd_payload carry;
    void* mid[8] = {nullptr};
    int alias = -1;
    hipEventRecord(h->ev[0], st);
    // SH_RULES_TS32=1: timestamps travel through the segment as 32-bit offsets from
    // the run's first time when its range fits (4 bytes fewer per event and pass).
    // Off by default: on C5 the three passes gained 0.35 ms, the range and
    // conversion passes cost 0.66 ms (profiles/r3_c5_ts32_ab.txt)
    int64_t tlo = 0, thi = 0;
    bool ts32 = false;
    if (sorted && getenv("SH_RULES_TS32") && getenv("SH_RULES_TS32")[0] == '1') {
        if (h->r_tsr.ensure_fresh(64)) return fail(h, SH_E_OOM, "rule workspace");
        if (shr_ts_range(run->d_ts, n, &tlo, &thi, h->r_tsr.p, st)) return fail(h, SH_E_HIP, "timestamp range");
        ts32 = thi >= tlo && (uint64_t)(thi - tlo) <= 0xFFFFFFFFull;
    }
    if (sorted && carry_setup(h, run, &carry, mid, &alias, false, !ts32)) return fail(h, SH_E_OOM, "rule workspace");
    if (ts32) {
        if (h->v_ts32.ensure_fresh((size_t)n * 4) || h->v_sts32.ensure_fresh((size_t)n * 4) ||
            h->v_mid_ts32.ensure_fresh((size_t)n * 4))
            return fail(h, SH_E_OOM, "rule workspace");
        if (shr_ts_to32(run->d_ts, n, tlo, h->v_ts32.as<uint32_t>(), st)) return fail(h, SH_E_HIP, "timestamps");
        carry.src[carry.n] = h->v_ts32.p;
        carry.dst[carry.n] = h->v_sts32.p;
        carry.width[carry.n] = 4;
        mid[carry.n] = h->v_mid_ts32.p;
        carry.n++;
    }
    const uint32_t* sts32 = ts32 ? h->v_sts32.as<uint32_t>() : nullptr;
    shd_segment_ws ws = seg_ws(h, n);
    const uint32_t* perm = nullptr;
    const uint32_t* skeys = nullptr;
    if (shd_segment_payload(&B, nkeys, &ws, st, &perm, &skeys, sorted ? &carry : nullptr, mid, 0, 0))
        return fail(h, SH_E_HIP, "segment launch failed");
    hipEventRecord(h->ev[1], st);
    const int64_t* sts = ts32 ? nullptr : (sorted ? h->v_sts.as<int64_t>() : run->d_ts);
    shd_cols sc;
    memset(&sc, 0, sizeof(sc));
    for (int a = 0; a < na; a++) sc.col[0][a] = sorted ? (const void*)h->v_scol[a].p : run->d_cols[a];
    if (alias >= 0) sc.col[0][alias] = skeys;
    hipMemcpyAsync(h->d_cols_desc.p, &sc, sizeof(sc), hipMemcpyHostToDevice, st);
    const shd_cols* dC = h->d_cols_desc.as<shd_cols>();
    const shr_table* dT = h->rd_tab.as<shr_table>();
    const uint32_t sentinel = sorted ? (uint32_t)nkeys : 0xFFFFFFFFu;
    uint32_t* cnt = h->w_cnt.as<uint32_t>();
    uint32_t* off = h->w_off.as<uint32_t>();
    hipMemsetAsync(h->v_flag.p, 0, 4, st);
    if (shr_count(dT, sts, skeys, n, sentinel, dC, cnt, h->v_flag.as<int32_t>(), st,
                  h->r_img.bytes ? h->rd_img.as<uint8_t>() : nullptr, &h->r_img, sts32, tlo) ||
        shd_exclusive_scan(cnt, off, n, h->w_scan.as<uint32_t>(), st))
        return fail(h, SH_E_HIP, "rule scan launch failed");
    uint32_t lo = 0, lc = 0;
    int32_t flag = 0;
    hipMemcpyAsync(&lo, off + (n - 1), 4, hipMemcpyDeviceToHost, st);
    hipMemcpyAsync(&lc, cnt + (n - 1), 4, hipMemcpyDeviceToHost, st);
    hipMemcpyAsync(&flag, h->v_flag.p, 4, hipMemcpyDeviceToHost, st);
    if (hipStreamSynchronize(st) != hipSuccess) return fail(h, SH_E_HIP, "device error in the rule scan");
    if (flag) return fail(h, SH_E_UNSUPPORTED, "rule engine: timestamps decrease inside a key");
    const int64_t m = (int64_t)lo + lc;
    run->out_count = m;
    if (m > run->out_capacity) return fail(h, SH_E_MORE, "output capacity too small");
    if (m > 0) {
        if (h->r_rec.ensure_fresh((size_t)m * 12)) return fail(h, SH_E_OOM, "match records");
        uint32_t* rec_p = h->r_rec.as<uint32_t>();
        uint32_t* rec_q = rec_p + m;
        uint32_t* rec_r = rec_q + m;
        if (shr_write(dT, sts, skeys, n, sentinel, dC, cnt, off, rec_p, rec_q, rec_r, st,
                      h->r_img.bytes ? h->rd_img.as<uint8_t>() : nullptr, &h->r_img, sts32, tlo))
            return fail(h, SH_E_HIP, "rule write launch failed");
        int prc = rules_order_place(h, run, m, rec_p, rec_q, rec_r, perm, sts, dC, sts32, tlo, sorted, false);
        if (prc) return prc;
    } else {
        hipEventRecord(h->ev[2], st);
    }
    return rules_finish(h, run, m, nkeys);
}

// bucketed window engine (sh_bucket.hip): partitioned window programs with a
// consumer-side form and a null-free projection; 0 ok, 1 = not applicable or a
// premise failed on the device (the caller runs the general window path),
// SH_E_MORE = output capacity too small (out_count = matches), <0 error
int run_bucket(sh_handle* h, sh_device_run* run, int32_t nkeys, bool force_carry) {
    static const bool off = getenv("SH_DISABLE_BUCKET") != nullptr;
    h->bk_last = 0;
    const shp_program& P = h->prog;
    const int64_t n = run->n;
    if (off || !h->partitioned || nkeys < 1024 || !P.out_fast || n < SHB_TILE) return 1;
    const int kb = std::max(0, bits_for((uint64_t)(nkeys - 1)) - 8);
    if (kb > 8) return 1;
    // select list: e2-side values (and e1's partition attribute, equal to e2's
    // for these types) from the consumer row; other e1-side values ride the match stream
    shb_out O;
    memset(&O, 0, sizeof(O));
    O.n_out = P.n_out;
    int ms[SHB_MAX_MS], n_ms = 0;
    const int part_attr = h->part_attr0;
    for (int o = 0; o < P.n_out; o++) {
        const int a = P.out_attr[o], t = P.attr_type[0][a];
        O.type[o] = t;
        const bool fold = a == part_attr && (t == SH_T_STRING || t == SH_T_INT || t == SH_T_LONG || t == SH_T_BOOL);
        if (P.out_slot[o] == 1 || fold) {
            O.kind[o] = 1;
            O.src[o] = run->d_cols[a];
            continue;
        }
        int m = 0;
        while (m < n_ms && ms[m] != a) m++;
        if (m == n_ms) {
            if (n_ms == SHB_MAX_MS) return 1;
            ms[n_ms++] = a;
        }
        O.kind[o] = 0;
        O.src[o] = (const void*)(intptr_t)m;  // resolved below
    }
    if (h->bk_state == 0) {
        const int lrc = shj_bucket_load(&P, ms, n_ms, &h->bk, &h->bk_err);
        h->bk_state = lrc == 0 ? 1 : (lrc == -1 ? -2 : -1);  // -2: no consumer-side form (not applicable)
    }
    if (h->bk_state != 1) return 1;
    hipStream_t st = h->stream;
    shb_plan B;
    memset(&B, 0, sizeof(B));
    if (n >= ((int64_t)1 << 32) - SHB_TILE) return 1;  // event indices are 32-bit on this engine
    B.n = n;
    B.nt = (int32_t)((n + SHB_TILE - 1) / SHB_TILE);
    B.kb = kb;
    // tiles per matcher chunk: 15/16 of the pass's consumer limit in events of a
    // bucket at uniform keys (32 per tile; 60 tiles at 2,048), so a chunk and its
    // halo fit the LDS span; denser buckets split (C2: 60 tiles 1.90 ms, 56 1.97-1.99,
    // 52 2.07, 64 2.50 in one call, profiles/r6_c2_ct_ab.txt)
    static const int ct_env = getenv("SH_BK_CT") ? atoi(getenv("SH_BK_CT")) : 0;
    B.ct = ct_env > 0 ? std::min(ct_env, SHB_CT_MAX) : std::min(shj_bucket_chunk() * 15 / 512, SHB_CT_MAX);
    B.n_chunks = (B.nt + B.ct - 1) / B.ct;
    const int64_t slots = (int64_t)B.nt * SHB_TILE;  // the tiles' bucket order
    if (ensure_ws(h, std::max<int64_t>(n, (int64_t)B.nt + 1)) || h->bk_w0.ensure_fresh(slots * 4) ||
        h->bk_sp.ensure_fresh(n * 2) || h->bk_toff.ensure_fresh((int64_t)B.nt * SHB_TOFF * 2) ||
        h->bk_cnt.ensure_fresh(slots) || h->bk_mstart.ensure_fresh((int64_t)B.nt * SHB_NB * 4) ||
        h->bk_tpre.ensure_fresh((int64_t)B.nt * 8) || h->bk_tfirst.ensure_fresh((int64_t)B.nt * 8) ||
        h->bk_hstart.ensure_fresh((int64_t)B.nt * 4) || h->bk_ttot.ensure_fresh(((int64_t)B.nt + 1) * 4) ||
        h->bk_flag.ensure_fresh(64) || h->bk_rd.ensure(64))
        return fail(h, SH_E_OOM, "bucket workspace");
    B.n_staged = h->bk.n_staged;
    for (int k = 0; k < B.n_staged; k++) {
        const int a = h->bk.staged_attr[k];
        const int w = type_width(P.attr_type[0][a]);
        if (h->bk_st[k].ensure_fresh(slots * w)) return fail(h, SH_E_OOM, "bucket workspace");
        B.st_src[k] = run->d_cols[a];
        B.st_dst[k] = h->bk_st[k].p;
        B.st_width[k] = w;
    }
    // match stream: one region of SHB_SPAN values per matcher workgroup (its first
    // pass), then a shared tail for further passes; every partial is consumed at
    // most once, so n values suffice for the tail
    B.n_ms = n_ms;
    const int64_t ms_vals = (int64_t)SHB_NB * B.n_chunks * SHB_SPAN + n;
    for (int m = 0; m < n_ms; m++) {
        const int w = type_width(P.attr_type[0][ms[m]]);
        if (h->bk_ms[m].ensure_fresh(ms_vals * w)) return fail(h, SH_E_OOM, "match stream");
        B.ms[m] = h->bk_ms[m].p;
        B.ms_width[m] = w;
    }
    int ms_of[SHB_MAX_OUT];
    for (int o = 0; o < O.n_out; o++) {
        ms_of[o] = O.kind[o] == 0 ? (int)(intptr_t)O.src[o] : -1;
        if (O.kind[o] == 0) O.src[o] = B.ms[ms_of[o]];
    }
    // aggregators carried per key in arrival order (k_bk_aggc: the reference's own
    // additions, no exactness proof): e1-side arguments from one 4-byte match-stream
    // column, e2-side ones from up to two staged columns (one of them 4-byte), count()
    // without one; anything else takes the post-pass (sh_agg.hip)
    shb_aggc AG;
    memset(&AG, 0, sizeof(AG));
    AG.e1_col = AG.e2_col[0] = AG.e2_col[1] = -1;
    // k_bk_aggp first (the additions as a segmented prefix, exact in 64-bit fixed point,
    // refused on the device by a value that is not); k_bk_aggc (every key of a bucket
    // walked in one workgroup: C2's 40 keys per bucket leave most lanes idle -- 28 ms
    // against the post-pass's 8.7) when the post-pass refuses too, or SH_BK_AGGC=1
    const bool aggc_env = getenv("SH_BK_AGGC") != nullptr;
    const bool aggp_off = getenv("SH_BK_AGGP") && getenv("SH_BK_AGGP")[0] == '0';
    const bool par = !force_carry && !aggc_env && !aggp_off && !h->aggp_refused && run->n < ((int64_t)1 << 31);
    bool carry = P.agg_post && !getenv("SH_BK_AGG_POST") && (force_carry || aggc_env || par);
    AG.parallel = par ? 1 : 0;
    // (the running values go by match-stream position; by output row, through a per-slot
    // row map, measured 8.39 vs 7.65 ms/step in round 5: removed)
    int agg_of[SHB_MAX_OUT];
    for (int o = 0; o < P.n_out; o++) agg_of[o] = -1;
    for (int o = 0; o < P.n_out && carry; o++) {
        const int ak = P.out_agg[o];
        if (ak == SH_AGG_NONE) continue;
        if (AG.n == SHB_MAX_AGG || (ak != SH_AGG_SUM && ak != SH_AGG_AVG && ak != SH_AGG_COUNT)) {
            carry = false;
            break;
        }
        const int i = AG.n++;
        AG.kind[i] = ak;
        agg_of[o] = i;
        if (ak == SH_AGG_COUNT) {
            AG.side[i] = 3;
            continue;
        }
        const int a = P.out_attr[o], t = P.attr_type[0][a];
        if (t != SH_T_INT && t != SH_T_FLOAT && t != SH_T_LONG && t != SH_T_DOUBLE) {
            carry = false;
            break;
        }
        const int w = type_width(t);
        if (P.out_slot[o] == 0 && ms_of[o] >= 0 && w == 4 && (AG.e1_col < 0 || AG.e1_col == ms_of[o])) {
            AG.e1_col = ms_of[o];
            AG.e1_type = t;
            AG.side[i] = 0;
        } else if (P.out_slot[o] == 1) {
            // the consumer's column at its slot: staged by the partition (the matcher's
            // own staged columns first, then the carry's)
            int k = 0;
            while (k < B.n_staged && (B.st_src[k] != run->d_cols[a])) k++;
            if (k == B.n_staged) {
                if (B.n_staged == SHB_MAX_STAGED || h->bk_st[k].ensure_fresh(slots * w))
                    return B.n_staged == SHB_MAX_STAGED ? 1 : fail(h, SH_E_OOM, "bucket workspace");
                B.st_src[k] = run->d_cols[a];
                B.st_dst[k] = h->bk_st[k].p;
                B.st_width[k] = w;
                B.n_staged++;
            }
            int c = (AG.e2_col[0] == k) ? 0 : (AG.e2_col[1] == k ? 1 : -1);
            if (c < 0) {
                if (AG.e2_col[0] < 0) c = 0;
                else if (AG.e2_col[1] < 0 && w == 4) c = 1;
                else if (AG.e2_col[1] < 0 && type_width(AG.e2_type[0]) == 4) {
                    // keep the 8-byte column in slot 0
                    AG.e2_col[1] = AG.e2_col[0];
                    AG.e2_type[1] = AG.e2_type[0];
                    for (int j = 0; j < i; j++)
                        if (AG.side[j] == 1) AG.side[j] = 2;
                    c = 0;
                } else {
                    carry = false;
                    break;
                }
                AG.e2_col[c] = k;
                AG.e2_type[c] = t;
            }
            AG.side[i] = 1 + c;
        } else {
            carry = false;
        }
    }
    if (carry) {
        for (int i = 0; i < AG.n; i++) {
            if (h->bk_agg[i].ensure_fresh(ms_vals * 8)) return fail(h, SH_E_OOM, "aggregate columns");
            AG.out[i] = h->bk_agg[i].p;
        }
        for (int o = 0; o < O.n_out; o++)
            if (agg_of[o] >= 0) {
                O.kind[o] = 0;
                O.src[o] = AG.out[agg_of[o]];
                O.type[o] = P.out_type[o];
            }
    }
    if (h->aggp_only && !(carry && AG.parallel)) return 1;
    h->bk_agg_carried = false;
    shb_cols OC;
    memset(&OC, 0, sizeof(OC));
    if (!P.agg_post || carry) {
        int32_t wd[SHB_MAX_OUT];
        for (int o = 0; o < O.n_out; o++) wd[o] = type_width(O.type[o]);
        direct_layout(h, run, wd, O.n_out, &OC);
    }
    B.ts = run->d_ts;
    B.keys = run->d_keys;
    B.w0 = h->bk_w0.as<uint32_t>();
    B.sp = h->bk_sp.as<uint16_t>();
    B.toff = h->bk_toff.as<uint16_t>();
    B.tstride = (B.nt + 63) & ~63;
    if (h->bk_tofft.ensure_fresh((int64_t)(SHB_NB + 1) * B.tstride * 2)) return fail(h, SH_E_OOM, "bucket workspace");
    B.tofft = h->bk_tofft.as<uint16_t>();
    B.cnt = h->bk_cnt.as<uint8_t>();
    B.mstart = h->bk_mstart.as<uint32_t>();
    B.tpre = h->bk_tpre.as<int64_t>();
    B.tfirst = h->bk_tfirst.as<int64_t>();
    B.hstart = h->bk_hstart.as<int32_t>();
    B.within = std::max<int64_t>(0, P.within_ms);
    B.ttot = h->bk_ttot.as<uint32_t>();
    B.flag = h->bk_flag.as<int32_t>();
    B.ms_ctr = h->bk_flag.as<uint32_t>() + 4;
    static const bool prof = getenv("SH_BK_PROFILE") != nullptr;
    if (prof) {
        if (h->bk_prof.ensure_fresh(128)) return fail(h, SH_E_OOM, "profile");
        hipMemsetAsync(h->bk_prof.p, 0, 128, h->stream);
        B.prof = h->bk_prof.as<unsigned long long>();
    }
    // packed timestamps: ts - tbase in 32 - kb bits, centred on the first event
    hipMemcpyAsync(h->bk_rd.p, run->d_ts, 8, hipMemcpyDeviceToHost, st);
    if (hipStreamSynchronize(st) != hipSuccess) return fail(h, SH_E_HIP, "bucket: timestamp read");
    B.tbase = *h->bk_rd.as<int64_t>() - ((int64_t)1 << (31 - kb));
    hipEventRecord(h->ev[0], st);
    hipMemsetAsync(B.flag, 0, 32, st);  // flag word + match-stream allocator
    hipMemsetAsync(B.ttot, 0, ((int64_t)B.nt + 1) * 4, st);
    if (shb_partition(run->d_keys, run->d_ts, nkeys, &B, st)) return fail(h, SH_E_HIP, "bucket partition launch failed");
    hipEventRecord(h->ev[1], st);
    void* args[] = {&B};
    if (hipModuleLaunchKernel((hipFunction_t)h->bk.match, (unsigned)(SHB_NB * B.n_chunks), 1, 1, 512, 1, 1, 0, st, args,
                              nullptr) != hipSuccess)
        return fail(h, SH_E_HIP, "shb_match launch failed");
    if (carry && shb_agg_carry(&B, &AG, st)) return fail(h, SH_E_HIP, "aggregate carry launch failed");
    if (shb_finish(&B, h->w_scan.as<uint32_t>(), st)) return fail(h, SH_E_HIP, "bucket scan launch failed");
    hipEventRecord(h->ev[2], st);
    if (shb_emit(&B, &O, &OC, 0, run->d_out_seq, run->d_out_values, run->out_capacity, st))
        return fail(h, SH_E_HIP, "bucket emit launch failed");
    hipEventRecord(h->ev[3], st);
    hipMemcpyAsync(h->bk_rd.as<void>(0), B.flag, 4, hipMemcpyDeviceToHost, st);
    hipMemcpyAsync(h->bk_rd.as<void>(8), B.ttot + B.nt, 4, hipMemcpyDeviceToHost, st);
    if (hipStreamSynchronize(st) != hipSuccess) return fail(h, SH_E_HIP, "device error in bucket engine");
    const int32_t flag = *h->bk_rd.as<int32_t>(0);
    const int64_t total = *h->bk_rd.as<uint32_t>(8);
    if (B.prof) {
        unsigned long long pr[16];
        hipMemcpy(pr, B.prof, 128, hipMemcpyDeviceToHost);
        fprintf(stderr, "[shb_match clock ticks, sum over workgroups] table %llu load %llu rank %llu walk %llu "
                        "scan+psum %llu emit %llu\n",
                pr[5], pr[0], pr[1], pr[2], pr[3], pr[4]);
        if (carry && AG.parallel)
            fprintf(stderr, "[k_bk_aggp clock ticks, sum over workgroups] table+load %llu sort %llu rows %llu "
                            "scans %llu\n",
                    pr[8], pr[9], pr[10], pr[11]);
        else if (carry)
            fprintf(stderr, "[k_bk_aggc clock ticks, sum over workgroups] table %llu load+prefix %llu e1 %llu "
                            "sort %llu walk %llu\n",
                    pr[8], pr[9], pr[10], pr[11], pr[12]);
    }
    if (flag & SHB_F_KEY) return fail(h, SH_E_INVALID_ARG, "partition key id >= n_keys");
    if (flag == SHB_F_AGG && carry && AG.parallel) {
        // a value the fixed point cannot hold exactly (or a chunk too dense): the
        // batch again without the carry, the post-pass (or k_bk_aggc) adding instead
        // The refusal sticks to the handle: data that fails the fixed-point test once
        // (a price such as 12.34) fails it in every batch, and each refused attempt costs
        // a whole bucketed pipeline
        h->aggp_refused = true;
        if (h->aggp_only) return 1;  // (the caller's raw rows first)
        return run_bucket(h, run, nkeys, force_carry);
    }
    if (flag) return 1;
    run->out_count = total;
    if (total > run->out_capacity) return fail(h, SH_E_MORE, "output capacity too small");
    if (run->d_out_query && total > 0) hipMemsetAsync(run->d_out_query, 0, total * 4, st);
    hipEventElapsedTime(&h->times.segment_ms, h->ev[0], h->ev[1]);
    hipEventElapsedTime(&h->times.advance_ms, h->ev[1], h->ev[2]);
    hipEventElapsedTime(&h->times.emit_ms, h->ev[2], h->ev[3]);
    hipEventElapsedTime(&h->times.total_ms, h->ev[0], h->ev[3]);
    h->times.advance_launches = 1;
    h->bk_last = 1;
    h->bk_agg_carried = carry;
    if (carry) h->agg_last = AG.parallel ? 5 : 4;
    return hipStreamSynchronize(st) == hipSuccess ? SH_OK : fail(h, SH_E_HIP, "bucket engine");
}

// the rise-and-fall sequence on the bucket-carry engine (sh_bucket.hip k_s3b):
// the tile-local bucket partition, one workgroup per bucket carrying its keys'
// state across the stream, the ordered rows by k_bk_emit. 0 ok, 1 = not
// applicable or refused on the device (the caller runs k_seq3s), <0 error
int run_s3b(sh_handle* h, sh_device_run* run, int32_t nkeys) {
    const bool off = getenv("SH_DISABLE_S3B") != nullptr || getenv("SH_NO_SEQ3") != nullptr;  // (per call: tests A/B it)
    h->s3b_last = 0;
    if (off || !h->partitioned || h->T->n_queries != 1 || !h->T->q[0].s3 || nkeys < 1024 || run->n < SHB_TILE)
        return 1;
    const nf_query& Q = h->T->q[0];
    const int kb = std::max(0, bits_for((uint64_t)(nkeys - 1)) - 8);
    if (kb > 12 || Q.contains_agg) return 1;
    // every operand and select value: one 4-byte attribute A (no null masks on this path)
    const int A = Q.s3_a2, ty = Q.s3_t2;
    if (!(ty == SH_T_FLOAT || ty == SH_T_INT) || A < 0 || A >= (int)h->stream_types[0].size() ||
        type_width(h->stream_types[0][A]) != 4 || Q.s3_a3 != A || Q.s3_e1a != A || Q.s3_la != A || Q.s3_t3 != ty ||
        Q.s3_e1t != ty || Q.s3_lt != ty)
        return 1;
    shb_out O;
    memset(&O, 0, sizeof(O));
    O.n_out = Q.n_out;
    shb_s3 S;
    memset(&S, 0, sizeof(S));
    S.type = ty;
    S.warm = 1;  // (the next chunk's gather overlaps the walk: 3.42 vs 3.52 ms, profiles/r4_c3_s3b_warm_ab.txt)
    S.op2 = Q.s3_op2;
    S.dom2 = Q.s3_dom2;
    S.op3 = Q.s3_op3;
    S.dom3 = Q.s3_dom3;
    for (int o = 0; o < Q.n_out; o++) {
        if (Q.s3_out_attr[o] != A || Q.s3_out_type[o] != ty) return 1;
        O.type[o] = ty;
        const int sl = Q.s3_out_slot[o];
        if (sl == 2) {
            O.kind[o] = 1;
            O.src[o] = run->d_cols[A];
            continue;
        }
        int m = 0;
        while (m < S.n_ms && S.ms_slot[m] != sl) m++;
        if (m == S.n_ms) S.ms_slot[S.n_ms++] = sl;
        O.kind[o] = 0;
        O.src[o] = (const void*)(intptr_t)m;  // resolved below
    }
    hipStream_t st = h->stream;
    shb_plan B;
    memset(&B, 0, sizeof(B));
    B.n = run->n;
    B.nt = (int32_t)((run->n + SHB_TILE - 1) / SHB_TILE);
    B.kb = kb;
    B.no_ts = 1;
    const int64_t slots = (int64_t)B.nt * SHB_TILE;
    if (ensure_ws(h, (int64_t)B.nt + 1) || h->bk_w0.ensure_fresh(slots * 4) || h->bk_sp.ensure_fresh(run->n * 2) ||
        h->bk_toff.ensure_fresh((int64_t)B.nt * SHB_TOFF * 2) || h->bk_cnt.ensure_fresh(slots) ||
        h->bk_mstart.ensure_fresh((int64_t)B.nt * SHB_NB * 4) || h->bk_tpre.ensure_fresh((int64_t)B.nt * 8) ||
        h->bk_tfirst.ensure_fresh((int64_t)B.nt * 8) || h->bk_hstart.ensure_fresh((int64_t)B.nt * 4) ||
        h->bk_ttot.ensure_fresh(((int64_t)B.nt + 1) * 4) || h->bk_flag.ensure_fresh(64) || h->bk_rd.ensure(64) ||
        h->bk_st[0].ensure_fresh(slots * 4))
        return fail(h, SH_E_OOM, "sequence workspace");
    B.n_staged = 1;
    B.st_src[0] = run->d_cols[A];
    B.st_dst[0] = h->bk_st[0].p;
    B.st_width[0] = 4;
    // match stream: at most one match per event, in its segment's slots
    B.n_ms = S.n_ms;
    for (int m = 0; m < S.n_ms; m++) {
        if (h->bk_ms[m].ensure_fresh(slots * 4)) return fail(h, SH_E_OOM, "match stream");
        B.ms[m] = h->bk_ms[m].p;
        B.ms_width[m] = 4;
    }
    for (int o = 0; o < O.n_out; o++)
        if (O.kind[o] == 0) O.src[o] = B.ms[(int)(intptr_t)O.src[o]];
    shb_cols OC;
    memset(&OC, 0, sizeof(OC));
    {
        int32_t wd[SHB_MAX_OUT];
        for (int o = 0; o < O.n_out; o++) wd[o] = 4;
        direct_layout(h, run, wd, O.n_out, &OC);
    }
    B.ts = run->d_ts;
    B.keys = run->d_keys;
    B.w0 = h->bk_w0.as<uint32_t>();
    B.sp = h->bk_sp.as<uint16_t>();
    B.toff = h->bk_toff.as<uint16_t>();
    B.tstride = (B.nt + 63) & ~63;
    if (h->bk_tofft.ensure_fresh((int64_t)(SHB_NB + 1) * B.tstride * 2)) return fail(h, SH_E_OOM, "bucket workspace");
    B.tofft = h->bk_tofft.as<uint16_t>();
    B.cnt = h->bk_cnt.as<uint8_t>();
    B.mstart = h->bk_mstart.as<uint32_t>();
    B.tpre = h->bk_tpre.as<int64_t>();
    B.tfirst = h->bk_tfirst.as<int64_t>();
    B.hstart = h->bk_hstart.as<int32_t>();
    B.ttot = h->bk_ttot.as<uint32_t>();
    B.flag = h->bk_flag.as<int32_t>();
    B.ms_ctr = h->bk_flag.as<uint32_t>() + 4;
    static const bool prof = getenv("SH_BK_PROFILE") != nullptr;
    if (prof) {
        if (h->bk_prof.ensure_fresh(128)) return fail(h, SH_E_OOM, "profile");
        hipMemsetAsync(h->bk_prof.p, 0, 128, st);
        B.prof = h->bk_prof.as<unsigned long long>();
    }
    hipEventRecord(h->ev[0], st);
    hipMemsetAsync(B.flag, 0, 32, st);
    hipMemsetAsync(B.ttot, 0, ((int64_t)B.nt + 1) * 4, st);
    if (shb_partition(run->d_keys, run->d_ts, nkeys, &B, st)) return fail(h, SH_E_HIP, "sequence partition failed");
    hipEventRecord(h->ev[1], st);
    if (shb_s3_carry(&B, &S, st)) return fail(h, SH_E_HIP, "sequence carry launch failed");
    if (shb_finish(&B, h->w_scan.as<uint32_t>(), st)) return fail(h, SH_E_HIP, "sequence scan failed");
    hipEventRecord(h->ev[2], st);
    if (shb_emit(&B, &O, &OC, 0, run->d_out_seq, run->d_out_values, run->out_capacity, st))
        return fail(h, SH_E_HIP, "sequence emit failed");
    hipEventRecord(h->ev[3], st);
    hipMemcpyAsync(h->bk_rd.as<void>(0), B.flag, 4, hipMemcpyDeviceToHost, st);
    hipMemcpyAsync(h->bk_rd.as<void>(8), B.ttot + B.nt, 4, hipMemcpyDeviceToHost, st);
    if (hipStreamSynchronize(st) != hipSuccess) return fail(h, SH_E_HIP, "device error in the sequence engine");
    const int32_t flag = *h->bk_rd.as<int32_t>(0);
    const int64_t total = *h->bk_rd.as<uint32_t>(8);
    if (B.prof) {
        unsigned long long pr[16];
        hipMemcpy(pr, B.prof, 128, hipMemcpyDeviceToHost);
        fprintf(stderr, "[k_s3b clock ticks, sum over workgroups] tables+load %llu sort %llu carry %llu out %llu\n",
                pr[0], pr[1], pr[2], pr[3]);
    }
    if (flag & SHB_F_KEY) return fail(h, SH_E_INVALID_ARG, "partition key id >= n_keys");
    if (flag) return 1;
    run->out_count = total;
    if (total > run->out_capacity) return fail(h, SH_E_MORE, "output capacity too small");
    if (run->d_out_query && total > 0) hipMemsetAsync(run->d_out_query, 0, total * 4, st);
    hipEventElapsedTime(&h->times.segment_ms, h->ev[0], h->ev[1]);
    hipEventElapsedTime(&h->times.advance_ms, h->ev[1], h->ev[2]);
    hipEventElapsedTime(&h->times.emit_ms, h->ev[2], h->ev[3]);
    hipEventElapsedTime(&h->times.total_ms, h->ev[0], h->ev[3]);
    h->times.advance_launches = 1;
    h->s3b_last = 1;
    return hipStreamSynchronize(st) == hipSuccess ? SH_OK : fail(h, SH_E_HIP, "sequence engine");
}

// typed output columns requested: engines that write raw rows write them into a
// workspace that sh_run_device narrows afterwards (the bucketed engine writes
// the columns itself)
int rows_for_cols(sh_handle* h, sh_device_run* run) {
    if (h->out_mode == SHB_OUT_RAW || h->cols_rows) return SH_OK;
    const size_t cap = (size_t)std::max<int64_t>(1, run->out_capacity);
    if (h->w_colrows.ensure(cap * std::max(1, h->n_out) * 8)) return fail(h, SH_E_OOM, "typed-column row workspace");
    run->d_out_values = h->w_colrows.as<int64_t>();
    if (h->out_mode == SHB_OUT_PACKED) {
        if (h->w_packseq.ensure(cap * 8)) return fail(h, SH_E_OOM, "packed-row workspace");
        run->d_out_seq = h->w_packseq.as<uint64_t>();
    }
    h->cols_rows = true;
    return SH_OK;
}

void direct_layout(sh_handle* h, sh_device_run* run, const int32_t* widths, int n_out, shb_cols* OC) {
    memset(OC, 0, sizeof(*OC));
    if (h->out_mode == SHB_OUT_RAW || h->cols_rows) return;
    OC->use = h->out_mode;
    for (int o = 0; o < n_out && o < SHB_MAX_OUT; o++) {
        OC->colw[o] = h->out_mode == SHB_OUT_PACKED ? h->pk_w[o] : widths[o];
        if (h->out_mode == SHB_OUT_COLS) OC->cols[o] = run->d_out_cols[o];
        else OC->woff[o] = h->pk_woff[o];
    }
    if (h->out_mode == SHB_OUT_PACKED) {
        OC->rw = h->pk_rw;
        OC->rows = run->d_out_values;
    }
}

// the running aggregates of the fast engines' ordered rows (sh_agg.hip): SH_OK,
// 1 = the double additions would round (the caller reruns sequentially), < 0 error
int agg_post(sh_handle* h, sh_device_run* run, int32_t nkeys, const int32_t* d_query, int n_query,
                    const int32_t* agg_kind, const int32_t* arg_type, int n_out) {
    const int64_t m = run->out_count;
    if (m <= 0) return SH_OK;
    sha_desc D;
    memset(&D, 0, sizeof(D));
    for (int o = 0; o < n_out && D.n_cols < SHA_MAX_COLS; o++)
        if (agg_kind[o] != SH_AGG_NONE) {
            D.c[D.n_cols].col = o;
            D.c[D.n_cols].kind = agg_kind[o];
            D.c[D.n_cols].arg_type = arg_type[o];
            D.n_cols++;
        }
    if (D.n_cols == 0) return SH_OK;
    if (h->a_scratch.ensure((size_t)sha_scratch_bytes(m, D.n_cols))) return fail(h, SH_E_OOM, "aggregate scratch");
    hipEventRecord(h->ev[4], h->stream);
    const int rc = sha_running(run->d_out_seq, run->d_out_values, n_out, m, d_query, n_query,
                               h->partitioned ? run->d_keys : nullptr, h->partitioned ? nkeys : 1, 0, &D,
                               h->a_scratch.p, h->stream);
    if (rc < 0) return fail(h, SH_E_HIP, "aggregate post-pass failed");
    hipEventRecord(h->ev[5], h->stream);
    hipEventSynchronize(h->ev[5]);
    float ms = 0.f;
    hipEventElapsedTime(&ms, h->ev[4], h->ev[5]);
    h->times.emit_ms += ms;
    h->times.total_ms += ms;
    h->agg_last = rc == 0 ? 1 : 2;
    return rc;
}
