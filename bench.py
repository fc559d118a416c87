#!/usr/bin/env python3
"""Benchmark: input events/sec for the partitioned pattern query (config C2).

Workload (BASELINE.json configs[1]):
  partition with (symbol of StockStream) begin
    from every e1=StockStream[price>20] -> e2=StockStream[symbol==e1.symbol and price>e1.price]
    within 1 sec select e1.symbol as symbol, e1.price as p1, e2.price as p2, e2.volume as v2
    insert into Out; end;
  100M synthetic ticks, 10,000 symbols, R = 100 ev/ms, resident in HBM.

A step = one full pass of the matcher over the 100M events from fresh per-key
state (radix segment -> per-key NFA advance -> ordered match placement), with
the ordered match stream written to HBM.

Multi-GPU (torchrun; C2, C3, C5): one process per GPU. The headline at N > 1 is
the north-star design, strong scaling over ONE stream: every rank ingests an
arrival-contiguous slice (cut at send() call boundaries); a step routes the
slice's events to the ranks owning their keys (mix32(key) % world, one RCCL
all-to-all of packed records), runs the matcher on the owned events, sends every
match row back to the rank holding its trigger event (a second all-to-all) and
k-way merges the runs by trigger sequence (C5: by the trigger's
PartitionStreamReceiver run, whose rows stay query-major) (siddhi_amd/shard.py,
include/siddhi_shard.h). value = the stream's events / the max-over-ranks step
time; the roofline is per GPU (all ranks' algorithmic matcher bytes / world /
the slowest rank's matcher kernel time). The same run then times the weak form
(every GPU its own partition of the key space: its own stream over its own
keys, no data-path collective) and prints it beside the headline as
`weak_value` / `weak`. --strong / --weak run one form only. C1 (no partition)
runs replicas; C4 runs its streaming path per rank (main_c4).
"""
import argparse
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--events", type=int, default=100_000_000)
    ap.add_argument("--keys", type=int, default=10_000)
    ap.add_argument("--rate", type=int, default=100)
    ap.add_argument("--cpu-sample", type=int, default=2_000_000,
                    help="events of the same workload timed on the CPU oracle (0 = skip)")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="CPU baseline threads for partitioned configs without timers (events split by key; "
                         "0 = 1 thread, except C5: min(16, nproc))")
    ap.add_argument("--no-verify", action="store_true")
    ap.add_argument("--agg", action="store_true",
                    help="c2 / c3: SURVEY.md 8d select variant (ii), the projection + sum / avg aggregators")
    ap.add_argument("--columns", action="store_true",
                    help="c2: typed output columns (d_out_cols); same as --layout columns")
    ap.add_argument("--layout", choices=["packed", "raw", "columns"], default=None,
                    help="c2 output layout: packed (default: SH_OUT_PACKED rows, trigger_seq + natural-width "
                         "values, 32 B per match), raw (trigger_seq + 8-byte words, 40 B), columns (d_out_cols)")
    ap.add_argument("--config", choices=["c1", "c2", "c3", "c4", "c5"], default="c2",
                    help="c2 (default, BASELINE.json configs[1]); c1 / c3 / c4 / c5 measure the other configs")
    ap.add_argument("--c4-calls", type=int, default=0, help="c4: send only the first N calls (profiling; 0 = all)")
    ap.add_argument("--c4-every", action="store_true", help="c4: the `every (e1=Login and e2=Txn) -> ...` variant")
    ap.add_argument("--rules", type=int, default=1000, help="c5: rule count")
    ap.add_argument("--strong", action="store_true",
                    help="N > 1: only the ONE-stream form over all ranks (c2 / c3 / c5: key-routed RCCL all-to-all "
                         "+ row return + k-way merge; c4: key-sharded streaming with gloo coordination). Default "
                         "for c2 / c3 / c5: that form as the headline, then the weak form beside it (weak_value)")
    ap.add_argument("--weak", action="store_true",
                    help="N > 1: only the weak form (every GPU matches its own partition of the key space: its own "
                         "stream over its own keys, no data-path collective; rank 0's stream is the canonical one)")
    args = ap.parse_args()
    args.seed_offset = 0  # (rank r of a weak-scaling run: its own partition's stream)
    if args.config == "c1":
        # BASELINE.json configs[0]: 10M ticks, 100 symbols, R = 1 ev/ms, no partition
        if args.events == 100_000_000:
            args.events = 10_000_000
        if args.keys == 10_000:
            args.keys = 100
        if args.rate == 100:
            args.rate = 1
        if args.cpu_sample == 2_000_000:
            args.cpu_sample = 300_000
    if args.config == "c5" and args.keys == 10_000:
        args.keys = 1_000_000
    if args.config == "c3" and args.keys == 10_000:
        args.keys = 1_000_000
        if args.rate == 100:
            args.rate = 1000
    if args.config == "c4" and args.keys == 10_000:
        args.keys = 10_000_000
    return args


def log(msg):
    """progress on stderr (long phases must keep writing, or the run looks hung)"""
    print(f"[bench] {msg}", file=sys.stderr, flush=True)


def workload(args):
    """Synthetic stream, compiled app, columns, bytes and checks of one config
    (one stream: at N > 1 the ranks split it by key, or replicate it for C1)."""
    from siddhi_amd import compiler, synth
    n, K = args.events, args.keys
    so = args.seed_offset
    if args.config == "c5":
        ts, card, amount, merchant = synth.txn_stream(n, K, args.rate, seed=synth.SEED + 5 + so)
        rules = synth.c5_rules(args.rules)
        text = synth.c5_query(rules)
        strings = compiler.StringDict()
        compiled = compiler.compile_app(text, strings)

        def expected():
            sys.path.insert(0, os.path.join(HERE, "tests"))
            from c5_check import c5_expected
            eseq, erule, evals = c5_expected(ts, card, amount, merchant, rules)
            return eseq, evals, erule

        def cpu(s, idx=None):
            sys.path.insert(0, os.path.join(HERE, "tests"))
            from oracle_engine import run_columns_oracle
            ix = np.arange(s) if idx is None else idx
            run_columns_oracle(compiled, ts[ix], [card[ix], amount[ix], merchant[ix]], card[ix], batch=4096)

        return dict(
            ts=ts, keys=card, cols=[card, amount, merchant], compiled=compiled, expected=expected, cpu=cpu,
            with_query=True, runs=True,
            b_event=20, b_match=20, cpu_sample=min(args.cpu_sample, 1_000_000), cpu_split=True,
            desc=f"C5: {args.rules} fraud rules `every e1=Txn[amount > A and merchant == M] -> "
                 f"e2=Txn[card == e1.card and amount > e1.amount * F] within W sec`, one partition (card of Txn)",
            key_name="cards_per_gpu", bytes_note="event: ts 8 + card 4 + amount 4 + merchant 4 = 20 B; "
            "match: seq 8 + query 4 + card 4 + amount 4 = 20 B")
    if args.config == "c1":
        ts, keys, price, vol = synth.stock_stream(n, K, args.rate, config_index=1, seed=synth.SEED + 1 + so)
        compiled = compiler.compile_app(synth.C1_QUERY)

        def expected():
            sys.path.insert(0, os.path.join(HERE, "tests"))
            from c2_check import c2_expected
            return c2_expected(ts, keys, price, vol) + (None,)

        def cpu(s):
            sys.path.insert(0, os.path.join(HERE, "tests"))
            from oracle_engine import run_columns_oracle
            run_columns_oracle(compiled, ts[:s], [keys[:s], price[:s], vol[:s]], None, batch=4096)

        return dict(ts=ts, keys=keys, cols=[keys, price, vol], compiled=compiled, expected=expected, cpu=cpu,
                    run_keys=np.zeros(n, np.int32), n_keys=1, b_event=24, b_match=28, cpu_sample=args.cpu_sample,
                    desc="C1: every e1[price>20] -> e2[symbol==e1.symbol and price>e1.price] within 1 sec, "
                         "no partition (BASELINE.json configs[0])", key_name="symbols_per_gpu",
                    bytes_note="event: ts 8 + symbol 4 + price 4 + volume 8 = 24 B; "
                               "match: seq 8 + symbol 4 + p1 4 + p2 4 + v2 8 = 28 B")
    ts, keys, price, vol = synth.stock_stream(n, K, args.rate, config_index=3 if args.config == "c3" else 2,
                                              seed=synth.SEED + (3 if args.config == "c3" else 2) + so)
    if args.config == "c3":
        compiled = compiler.compile_app(synth.C3_AGG_QUERY if args.agg else synth.C3_QUERY)

        def expected():
            sys.path.insert(0, os.path.join(HERE, "tests"))
            from c3_check import c3_expected
            eseq, ev = c3_expected(ts, keys, price)
            if args.agg:
                ev = with_aggregates(keys[eseq], ev, [("sum", ev[:, 2]), ("avg", ev[:, 1])])
            return eseq, ev, None

        def cpu(s, idx=None):
            sys.path.insert(0, os.path.join(HERE, "tests"))
            from oracle_engine import run_stock_oracle
            ix = np.arange(s) if idx is None else idx
            run_stock_oracle(compiled, ts[ix], keys[ix], price[ix], vol[ix], batch=4096)

        return dict(ts=ts, keys=keys, cols=[keys, price, vol], compiled=compiled, expected=expected, cpu=cpu,
                    b_event=16, b_match=20 + (16 if args.agg else 0), cpu_sample=args.cpu_sample, cpu_split=True,
                    desc="C3: every e1=S, e2=S[price>e1.price]+, e3=S[price<e2[last].price], "
                         "partition with (symbol of S)" + AGG_NOTE[args.agg], key_name="keys_per_gpu",
                    bytes_note="event: ts 8 + symbol 4 + price 4 = 16 B; match: seq 8 + 3 x price 4 = 20 B"
                               + (" + sum 8 + avg 8 = 36 B" if args.agg else ""))
    compiled = compiler.compile_app(synth.C2_AGG_QUERY if args.agg else synth.C2_QUERY)

    def expected():
        sys.path.insert(0, os.path.join(HERE, "tests"))
        from c2_check import c2_expected
        eseq, ev = c2_expected(ts, keys, price, vol)
        if args.agg:
            ev = with_aggregates(keys[eseq], ev, [("sum", ev[:, 2]), ("avg", ev[:, 1])])
        return eseq, ev, None

    def cpu(s, idx=None):
        sys.path.insert(0, os.path.join(HERE, "tests"))
        from oracle_engine import run_stock_oracle
        ix = np.arange(s) if idx is None else idx
        run_stock_oracle(compiled, ts[ix], keys[ix], price[ix], vol[ix], batch=4096)

    return dict(ts=ts, keys=keys, cols=[keys, price, vol], compiled=compiled, expected=expected, cpu=cpu,
                b_event=24, b_match=28 + (16 if args.agg else 0), cpu_sample=args.cpu_sample, cpu_split=True,
                desc="C2: every e1[price>20] -> e2[symbol==e1.symbol and price>e1.price] within 1 sec, "
                     "partition with (symbol of StockStream)" + AGG_NOTE[args.agg], key_name="symbols_per_gpu",
                bytes_note="event: ts 8 + symbol 4 + price 4 + volume 8 = 24 B; "
                           "match: seq 8 + symbol 4 + p1 4 + p2 4 + v2 8 = 28 B"
                           + (" + sum 8 + avg 8 = 44 B" if args.agg else ""))


AGG_NOTE = {False: "", True: "; select variant (ii): + sum / avg running per partition key"}


def with_aggregates(group, ev, aggs):
    """the restatement's rows + the running aggregates (tests/agg_check.py): each
    (kind, raw float column) adds one double-valued column"""
    sys.path.insert(0, os.path.join(HERE, "tests"))
    from agg_check import raw_bits, running
    g = group.astype(np.int64)
    extra = [raw_bits(running(g, col.astype(np.uint32).view(np.float32).astype(np.float64), kind))
             for kind, col in aggs]
    return np.concatenate([ev] + [e.reshape(-1, 1) for e in extra], 1)


import numpy as np  # noqa: E402


def main_c4(args, torch, dist, world, rank, dev):
    """C4 (BASELINE.json configs[3]): `(e1=Login and e2=Txn) -> not Logout for 5 sec`
    (or the `every (...)` variant, --c4-every) partitioned by user, playback time,
    on the SURVEY 8d workload: --events (100M) over Login 20% / Txn 60% / Logout 20%,
    --keys (10M) users, R = --rate (100) ev/ms, send(Event[]) calls of 4,096 events
    per stream (synth.c4_spec_stream). Absent states need the playback scheduler,
    so this config runs through the streaming C-ABI (sh_push_batch per call,
    sh_advance_time, sh_drain): host buffers cross PCIe inside the timed region.
    At N > 1 the users are key-sharded (siddhi_amd/shard_stream.py): every rank sees
    every call and pushes its users' events (sh_push_batch_part); the one state per
    due time Scheduler.onTimeChange fires and the state map's HashMap order are
    agreed over gloo (candidate gather + history exchange). A step = one fresh
    engine start + the whole stream + the drain of every match."""
    sys.path.insert(0, os.path.join(HERE, "tests"))
    from c4_cases import register_users
    from siddhi_amd import compiler, synth
    from siddhi_amd._native import HipEngine
    log(f"generating c4 workload: {args.events} events, {args.keys} users, R = {args.rate} ev/ms")
    strong = world > 1 and args.strong
    # weak scaling (default at N > 1): rank r streams its own partition of the users
    # (its own stream, seed offset; rank 0's is the canonical one), no coordination
    blocks = synth.c4_spec_stream(args.events, args.keys, rate_per_ms=args.rate, batch=BATCH,
                                  seed=synth.SEED + 40 + (0 if strong else args.seed_offset))
    if args.c4_calls:
        blocks = blocks[:args.c4_calls]
    n = sum(len(b[1]) for b in blocks)
    text = synth.C4_EVERY_QUERY if args.c4_every else synth.C4_QUERY
    c = compiler.compile_app(text)
    end = synth.c4_end_time(blocks)
    group = dist.new_group(backend="gloo") if world > 1 else None

    # phase clocks of the streaming path (sh_host_nfa.cpp HpScope; a few clock reads
    # per call): host work vs time blocked on the device and copies
    os.environ["SH_HOST_PROF"] = "1"

    def step():
        base = HipEngine(c)
        eng = base
        comm = None
        if strong:
            from siddhi_amd.shard_stream import ShardedStreamEngine, TorchGroupComm
            comm = TorchGroupComm(group)
            eng = ShardedStreamEngine(base, comm)
        register_users(eng, blocks)
        t = time.perf_counter()
        eng.start()
        t_log = time.monotonic()
        for i, (st, ts, cols, keys) in enumerate(blocks):
            if time.monotonic() - t_log > 20:
                t_log = time.monotonic()
                log(f"{i}/{len(blocks)} send calls")
            eng.send(st, ts, cols, [None] * len(cols), keys, 0)
        eng.advance_time(end)
        out = eng.drain()
        dt = time.perf_counter() - t
        if strong:
            eng.check()
        last["prof"] = base.host_profile()
        last["comm"] = (comm.seconds, comm.calls) if comm is not None else None
        base.close()
        last["out"] = out
        last["dt"] = dt
        return len(out["seq"]), dt

    last = {}

    for i in range(args.warmup):
        log(f"warmup {i}")
        step()
    if world > 1:
        dist.barrier()
    tot, m = 0.0, 0
    for i in range(args.steps):
        m, dt = step()
        tot += dt
        log(f"step {i}: {dt * 1000:.0f} ms, {m} matches")
    dt_t = torch.tensor([tot, float(m)], dtype=torch.float64)
    if world > 1:
        dist.all_reduce(dt_t[:1], op=dist.ReduceOp.MAX, group=group)
        dist.all_reduce(dt_t[1:], op=dist.ReduceOp.SUM, group=group)
    tot, m = float(dt_t[0].item()), int(dt_t[1].item())
    # strong: the one stream over all ranks; weak: every rank's own stream
    value = (n if strong else n * world) * args.steps / tot
    # the ordered output vs the oracle's digest on the same stream (tests/golden/
    # c4_digest.json, tests/golden/make_c4_digest.py), when it holds this workload
    verified = None
    if (world == 1 or not strong) and not args.c4_calls:
        try:
            from c4_cases import c4_digest
            key = ("every" if args.c4_every else "default") + f"_{args.events}_{args.keys}"
            want = json.load(open(os.path.join(HERE, "tests", "golden", "c4_digest.json"))).get(key)
            if want is not None:
                verified = c4_digest(last["out"]) == {"rows": want["rows"], "sha256": want["sha256"]}
        except (OSError, ValueError):
            verified = None
    # algorithmic bytes: Login / Logout 12 B, Txn 16 B, + 1 B stream
    # tag per event; per alert seq 8 + user 4 + ip 4 + amount 4 = 20 B
    n_txn = sum(len(b[1]) for b in blocks if b[0] == 1)
    b_alg = 13 * n + 4 * n_txn + 20 * m
    achieved = b_alg / (tot / args.steps)
    cpu = None
    if rank == 0 and args.cpu_sample > 0:
        from oracle_engine import OracleEngine
        from c4_cases import run_c4
        acc, sub = 0, []
        want = max(1_000_000, min(args.cpu_sample, 2_000_000))
        for b in blocks:
            if acc >= want:
                break
            sub.append(b)
            acc += len(b[1])
        log(f"CPU baseline on {acc} events")
        t1 = time.perf_counter()
        run_c4(OracleEngine(c), sub)
        cdt = time.perf_counter() - t1
        cpu = {"value": acc / cdt, "unit": "events/s", "cores": 1, "kind": "port",
               "sample": f"first {acc} events ({len(sub)} send(Event[]) calls) of the same C4 stream, C++ "
                         f"restatement of siddhi-core's processors (oracle/), 1 thread"}
    # the last step's split (rank 0): wall = host work + time blocked in stream syncs
    # (kernels and copies the host waits for) + coordination (N > 1: all_gathers)
    hp = last.get("prof") or {}
    wall_ms = last.get("dt", 0.0) * 1000.0
    wait_ms = hp.get("sync_wait", (0.0, 0))[0]
    comm_ms = last["comm"][0] * 1000.0 if last.get("comm") else 0.0
    split = {"wall_ms": wall_ms, "blocked_on_device_ms": wait_ms, "syncs": hp.get("sync_wait", (0.0, 0))[1],
             "coordination_ms": comm_ms, "coordination_calls": last["comm"][1] if last.get("comm") else 0,
             "host_ms": wall_ms - wait_ms - comm_ms,
             "phases_ms": {k: round(v[0], 1) for k, v in hp.items() if k not in ("hist_records", "sync_wait")},
             "calls": len(blocks)}
    if rank == 0:
        print(json.dumps({
            "metric": "input events/sec (node) for partitioned pattern query; achieved HBM GB/s %",
            "value": value, "unit": "events/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "split_last_step": split,
            "ms_per_step": tot * 1000.0 / args.steps, "higher_is_better": True,
            "scaling": "strong" if strong else "weak",
            "vs_baseline": None, "dtype": "f32+i64", "data": "synthetic", "nproc": os.cpu_count(),
            "ingest": {"path": "host buffers of every send(Event[]) call cross PCIe inside the timed step"},
            "config": {"workload": ("C4: " + ("every " if args.c4_every else "") + "(e1=Login and e2=Txn) -> not "
                                    "Logout for 5 sec, partition with (user of Login, user of Txn, user of "
                                    "Logout), @app:playback; Login 20% / Txn 60% / Logout 20%, calls of 4,096 "
                                    "per stream"),
                       "events_total": n if strong else n * world, "events_per_gpu": n if not strong else None,
                       "users": args.keys, "rate_ev_per_ms": args.rate,
                       "send_calls": len(blocks), "matches_total": int(m),
                       "path": "streaming C-ABI from host buffers (PCIe-inclusive)",
                       "parallelism": (f"key-sharded x{world}: events routed per call by user, due-timer "
                                       "candidates and scheduler-map history exchanged per time step (gloo)")
                       if strong else (f"dp{world}: every GPU its own partition of the users (own stream), "
                                       "no data-path collective" if world > 1 else "one GPU")},
            "roofline": {"bound": "hbm", "achieved": achieved / 1e9, "peak": 8000.0, "unit": "GB/s",
                         "frac": achieved / 8.0e12, "traffic": None,
                         "kernel": "whole streaming step (wall clock, PCIe and per-call launches included): "
                                   "algorithmic bytes / step time",
                         "algorithmic_bytes": b_alg},
            "cpu_baseline": cpu,
            "verified_vs_restatement": verified,
            "verified_against": "digest of the oracle's ordered output on this stream (tests/golden/c4_digest.json)",
            "parity": "tests/test_gpu_c4.py (whole streams vs the oracle up to 1M users; the 10M-user stream vs "
                      "the oracle's digest), tests/test_gpu_shard_stream.py (2 / 4 key-sharded virtual ranks)"}))
    if world > 1:
        dist.destroy_process_group()


def check_rows(W, oseq, ovals, oq, sel_range=None):
    """the device's ordered rows == the vectorised restatement's (optionally only
    the rows whose trigger events lie in [lo, hi): one rank's slice)"""
    eseq, evals, eq = W["expected"]()
    if sel_range is not None:
        sel = (eseq >= sel_range[0]) & (eseq < sel_range[1])
        eseq, evals = eseq[sel], evals[sel]
        eq = eq[sel] if eq is not None else None
    ok = len(oseq) == len(eseq) and np.array_equal(oseq, eseq) and np.array_equal(ovals[:, :evals.shape[1]], evals)
    if eq is not None:
        ok = ok and oq is not None and np.array_equal(oq, eq)
    return bool(ok)


def engine_tag():
    """identifies the device pipeline a PMC profile was taken on (bumped when a
    pipeline's kernels change what they move)"""
    return "r6"


def cpu_baseline(args, W, n):
    """the oracle (C++ restatement of siddhi-core's processors) on a bounded sample
    of the same stream, on this host's cores"""
    if args.cpu_sample <= 0:
        return None
    s = min(W["cpu_sample"], n)
    threads = args.cpu_threads or (min(16, os.cpu_count() or 1) if args.config == "c5" else 1)
    if not W.get("cpu_split"):
        threads = 1
    log(f"CPU baseline on {s} events, {threads} thread(s)")
    from concurrent.futures import ThreadPoolExecutor, wait
    t1 = time.perf_counter()
    # partitions are independent (no timers): with several threads the sample's
    # events split by key, each thread with its own oracle instance (ctypes releases
    # the GIL inside the restatement); the main thread logs while they run
    part = W["keys"][:s] % threads if threads > 1 else None
    jobs = [None] if threads == 1 else [np.flatnonzero(part == t) for t in range(threads)]
    with ThreadPoolExecutor(threads) as ex:
        futs = [ex.submit((lambda: W["cpu"](s)) if ix is None else (lambda ix=ix: W["cpu"](s, ix))) for ix in jobs]
        while wait(futs, timeout=30).not_done:
            log(f"CPU baseline: {time.perf_counter() - t1:.0f} s")
        for f in futs:
            f.result()
    cdt = time.perf_counter() - t1
    return {"value": s / cdt, "unit": "events/s", "cores": threads, "kind": "port",
            "sample": f"first {s} events of the same {args.config.upper()} stream, send(Event[]) batches of "
                      f"4096, C++ restatement of siddhi-core's processors (oracle/), {threads} thread(s)"
                      + (" over key-disjoint sub-streams" if threads > 1 else "")}


BATCH = 4096  # events per send(Event[]) call


def main_sharded(args, torch, dist, world, rank, dev):
    """C2 / C3 / C5 over `world` GPUs: one stream, key-sharded step (module docstring)."""
    from siddhi_amd import shard
    from siddhi_amd.device_run import DeviceRunner
    log(f"rank {rank}: generating the {args.config} stream, slice {rank}/{world}")
    W = workload(args)
    n = len(W["ts"])
    K = W.get("n_keys", args.keys)
    b = shard.slice_bounds(n, world, align=BATCH)
    lo, hi = b[rank], b[rank + 1]
    d_ts = torch.from_numpy(W["ts"][lo:hi].copy()).to(dev)
    d_cols = [torch.from_numpy(c[lo:hi].copy()).to(dev) for c in W["cols"]]
    d_run = None
    if W.get("runs"):
        # PartitionStreamReceiver runs of the whole stream (a property of its
        # send() calls), computed at ingest
        d_run = torch.from_numpy(shard.stream_run_ids(W["keys"], BATCH)[lo:hi].copy()).to(dev)
    runner = DeviceRunner(W["compiled"], device=str(dev))
    stream = torch.cuda.current_stream(dev)
    wq = bool(W.get("with_query"))
    kt_acc = {"ms": 0.0}

    def matcher(t, k, c, nk, run=None):
        r = runner.run(t, k, c, nk, stream=stream, with_query=wq, run_ids=run)
        kt = runner.kernel_times()
        kt_acc["ms"] += kt["total_ms"]
        kt_acc["last"] = kt
        if not wq:
            return r
        m, s_, v, q = r
        return m, s_, torch.cat([v, q[:m].to(torch.int64).view(-1, 1)], 1)

    comm = shard.BounceComm(world) if os.environ.get("SH_BENCH_SHARE_GPU") else None
    step = shard.KeyShardedStep(world, rank, shard.HipShardOps(str(dev)), matcher,
                                n_out=runner.n_out + (1 if wq else 0), comm=comm)
    rdev = "cpu" if comm is not None else dev  # device of the timing / count reductions

    def one():
        return step.run(d_ts, d_cols[0], d_cols, lo, K, key_attr=0, run_ids=d_run, batch=BATCH)

    log("warmup")
    for _ in range(args.warmup):
        one()
    torch.cuda.synchronize(dev)
    dist.barrier()
    torch.cuda.synchronize(dev)
    kt_acc["ms"] = 0.0
    t0 = time.perf_counter()
    for _ in range(args.steps):
        seq, vals = one()
    torch.cuda.synchronize(dev)
    dist.barrier()
    torch.cuda.synchronize(dev)
    dt = time.perf_counter() - t0
    dt_t = torch.tensor([dt], dtype=torch.float64, device=rdev)
    dist.all_reduce(dt_t, op=dist.ReduceOp.MAX)
    dt = float(dt_t.item())
    # per rank: matches triggered by its slice, matches made here, events received,
    # matcher kernel time per step
    mine = torch.tensor([[float(seq.numel()), float(step.last["matches_here"]), float(sum(step.last["received"])),
                          kt_acc["ms"] / args.steps]], dtype=torch.float64, device=rdev)
    allr = [torch.zeros_like(mine) for _ in range(world)]
    dist.all_gather(allr, mine)
    allr = torch.cat(allr).cpu().numpy()
    m = int(allr[:, 0].sum())
    # roofline per GPU: the algorithmic bytes of every rank's matcher (events it
    # received + matches it made) over the slowest rank's matcher kernel time
    b_alg = W["b_event"] * allr[:, 2] + W["b_match"] * allr[:, 1]
    kmax = float(allr[:, 3].max())
    achieved = float(b_alg.sum()) / world / (kmax / 1000.0)
    peak = 8.0e12
    verified = None
    if not args.no_verify and rank == 0:
        log("verifying rank 0's ordered rows against the vectorised restatement")
        v = vals.cpu().numpy()
        oq = v[:, -1].astype(np.int32) if wq else None
        verified = check_rows(W, seq.cpu().numpy(), v[:, :-1] if wq else v, oq, (lo, hi))
    cpu = cpu_baseline(args, W, n) if rank == 0 and args.cpu_sample else None
    # the same phase names as the one-GPU line (shard.KeyShardedStep.PHASES): the step's phases on
    # rank 0's launch stream, the matcher's own split inside unpack_match
    phases = dict(step.phase_ms() or {})
    last = kt_acc.get("last") or {}
    phases.update({"segment": last.get("segment_ms"), "advance": last.get("advance_ms"),
                   "emit": last.get("emit_ms")})
    line = None
    if rank == 0:
        line = {
            "metric": "input events/sec (node) for partitioned pattern query; achieved HBM GB/s %",
            "value": n * args.steps / dt, "unit": "events/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": dt * 1000.0 / args.steps, "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": "f32+i64", "data": "synthetic",
            "nproc": os.cpu_count(),
            "config": {"workload": W["desc"] + "; one stream split by key", "events_total": n,
                       W["key_name"].replace("_per_gpu", ""): args.keys, "rate_ev_per_ms": args.rate,
                       "matches_total": m,
                       "parallelism": f"key-sharded x{world}: RCCL all-to-all route + return, k-way merge",
                       "rank0_slice": [lo, hi], "rank0_step": step.last, "bytes": W["bytes_note"]},
            "phase_ms": phases,
            "phase_ms_scope": "rank 0, last timed step",
            "roofline": {"bound": "hbm", "achieved": achieved / 1e9, "peak": peak / 1e9, "unit": "GB/s",
                         "frac": achieved / peak, "traffic": None,
                         "kernel": "matcher step per GPU (every matcher kernel; HIP events on the launch stream): "
                                   "algorithmic bytes of all ranks / world / slowest rank's matcher time",
                         "kernels_ms_per_step_max": kmax, "algorithmic_bytes_per_rank": b_alg.tolist()},
            "cpu_baseline": cpu,
            "verified_vs_restatement": verified}
    runner.close()
    del step, d_ts, d_cols, d_run
    torch.cuda.synchronize(dev)
    torch.cuda.empty_cache()
    return line


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if os.environ.get("SH_BENCH_SHARE_GPU"):
        # rehearsal of the N-rank path on a one-GPU box: every rank on device 0
        local = 0
    share = bool(os.environ.get("SH_BENCH_SHARE_GPU"))
    if world > 1:
        torch.cuda.set_device(local)
        # rehearsal on one GPU: gloo through host memory (RCCL refuses duplicate devices)
        dist.init_process_group("gloo" if share else "nccl")
    dev = torch.device(f"cuda:{local}")
    if args.config == "c4":
        if world > 1 and not args.strong:
            args.seed_offset = 7919 * rank  # each rank its own partition of the users
        return main_c4(args, torch, dist, world, rank, dev)
    if args.config in ("c2", "c3", "c5") and world > 1 and not args.weak:
        # the north-star form first: one stream, key-routed over RCCL, rows merged back
        strong = main_sharded(args, torch, dist, world, rank, dev)
        if args.strong:
            if rank == 0:
                print(json.dumps(strong))
            dist.destroy_process_group()
            return
        # then the weak form in the same run (its stream is rank 0's verified one at N = 1)
        args.seed_offset = 7919 * rank
        args.no_verify, args.cpu_sample = True, 0
        weak = run_partitions(args, torch, dist, world, rank, dev)
        if rank == 0:
            strong["weak_value"] = weak["value"]
            strong["weak"] = {k: weak[k] for k in ("value", "ms_per_step", "scaling", "roofline", "config",
                                                   "phase_ms", "engine")}
            print(json.dumps(strong))
        dist.destroy_process_group()
        return
    if world > 1:
        # every rank matches its own partition of the key space (its own stream over
        # its own keys; rank 0's is the canonical one, verified)
        args.seed_offset = 7919 * rank
    line = run_partitions(args, torch, dist, world, rank, dev)
    if rank == 0:
        print(json.dumps(line))
    if world > 1:
        dist.destroy_process_group()


def run_partitions(args, torch, dist, world, rank, dev):
    """The one-GPU step, or at N > 1 the weak form: every rank its own partition of
    the key space, ranks meeting only in the timing barrier and the max reduction.
    Returns rank 0's line (None elsewhere)."""
    from siddhi_amd.device_run import DeviceRunner

    n, K = args.events, args.keys
    log(f"generating {args.config} workload: {n} events, {K} keys")
    W = workload(args)
    runner = DeviceRunner(W["compiled"], device=str(dev))
    # host -> device ingest of the input columns (outside the timed region:
    # the timed step starts from HBM-resident events)
    torch.cuda.synchronize(dev)
    t_in = time.perf_counter()
    t_ts = torch.from_numpy(W["ts"]).to(dev)
    cols = [torch.from_numpy(c).to(dev) for c in W["cols"]]
    t_k = torch.from_numpy(W["run_keys"]).to(dev) if "run_keys" in W else cols[0]
    torch.cuda.synchronize(dev)
    ingest_s = time.perf_counter() - t_in
    ingest_bytes = W["ts"].nbytes + sum(c.nbytes for c in W["cols"])
    K = W.get("n_keys", K)
    stream = torch.cuda.current_stream(dev)
    with_q = bool(W.get("with_query"))

    # c2's output layout: packed rows (SH_OUT_PACKED: seq 8 + symbol 4 + p1 4 + p2 4
    # + pad 4 + v2 8 = 32 B per match, two 16-byte stores) by default; raw rows
    # (seq 8 apart + four 8-byte words, 40 B) or typed columns (28 B in five
    # arrays: more store instructions, measured slower) on request
    # (--agg too: the bucketed engine's aggregate carry hands the running values to
    # the emitter, which packs them like any 8-byte column: + total 8 + a1 8 = 48 B)
    layout = (args.layout or ("columns" if args.columns else "packed")
              if args.config == "c2" else "raw")
    use_cols = layout == "columns"
    use_packed = layout == "packed"

    def step():
        if use_packed:
            r = runner.run(t_ts, t_k, cols, K, stream=stream, with_query=with_q, packed=True)
            r = (r[0], None, r[1]) + ((r[2],) if with_q else ())
        else:
            r = runner.run(t_ts, t_k, cols, K, stream=stream, with_query=with_q, columns=use_cols)
        return r if with_q else r + (None,)

    log("warmup")
    for _ in range(args.warmup):
        m, _, _, _ = step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    seg = adv = emt = 0.0
    t0 = time.perf_counter()
    for _ in range(args.steps):
        m, oseq, ovals, oq = step()
        kt = runner.kernel_times()
        seg += kt["segment_ms"]
        adv += kt["advance_ms"]
        emt += kt["emit_ms"]
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    dt = time.perf_counter() - t0
    # (max over ranks; a one-GPU rehearsal's gloo group reduces host tensors)
    dt_t = torch.tensor([dt], dtype=torch.float64, device="cpu" if os.environ.get("SH_BENCH_SHARE_GPU") else dev)
    if world > 1:
        dist.all_reduce(dt_t, op=dist.ReduceOp.MAX)
    dt = float(dt_t.item())
    ms_step = dt * 1000.0 / args.steps
    events_total = n * world
    value = events_total * args.steps / dt

    # algorithmic bytes: event columns the query reads + the
    # emitted records (see W["bytes_note"])
    b_alg = W["b_event"] * n + W["b_match"] * m
    adv_ms = adv / args.steps
    seg_ms = seg / args.steps
    emt_ms = emt / args.steps
    peak = 8.0e12
    # the roofline is priced on the whole matcher step (every kernel of one
    # pass: segment + match + ordered placement, HIP events on the launch
    # stream); the match kernel alone is reported beside it
    step_kernels_ms = seg_ms + adv_ms + emt_ms
    achieved = b_alg / (step_kernels_ms / 1000.0)
    match_only = b_alg / (adv_ms / 1000.0)

    verified = None
    if not args.no_verify and rank == 0:
        log("verifying the full output against the vectorised restatement")
        if use_packed:
            import numpy as np
            from siddhi_amd.device_run import packed_to_raw
            offs, rb = runner.packed_layout()
            oseq_np, ovals_np = packed_to_raw(ovals.cpu().numpy(), runner.out_types, offs, rb)
            oseq_np = oseq_np.view(np.int64)
        elif use_cols:
            from siddhi_amd.device_run import columns_to_raw
            ovals_np = columns_to_raw([c.cpu().numpy() for c in ovals], runner.out_types)
            oseq_np = oseq.cpu().numpy()
        else:
            ovals_np = ovals.cpu().numpy()
            oseq_np = oseq.cpu().numpy()
        verified = check_rows(W, oseq_np, ovals_np, oq.cpu().numpy() if oq is not None else None)

    # HBM bytes per step from the committed rocprofv3 PMC passes of this exact
    # workload and variant (scripts/pmc_traffic.py): config, events, keys, --agg,
    # --columns and the engine build must all match, else null
    traffic, traffic_src = None, None
    variant = args.config + ("_agg" if args.agg else "") + {"packed": "", "raw": "_raw", "columns": "_cols"}[layout]
    if args.config != "c2":
        variant = args.config + ("_agg" if args.agg else "")
    prof = os.path.join(HERE, "profiles", f"pmc_{variant}.json")
    if os.path.exists(prof):
        try:
            pj = json.load(open(prof))
            if (pj.get("events") == n and pj.get("keys") == K and bool(pj.get("agg")) == bool(args.agg)
                    and pj.get("layout", "raw") == layout and pj.get("engine") == engine_tag()):
                traffic = pj.get("hbm_bytes_per_step")
                traffic_src = os.path.relpath(prof, HERE)
        except Exception:
            traffic = None

    cpu = cpu_baseline(args, W, n) if rank == 0 and args.cpu_sample else None

    line = None
    if rank == 0:
        line = {
            "metric": "input events/sec (node) for partitioned pattern query; achieved HBM GB/s %",
            "value": value, "unit": "events/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": ms_step, "higher_is_better": True,
            # N > 1 here: every GPU its own key partition (main_sharded: --strong)
            "scaling": "weak",  # per-GPU work fixed as N grows (its own key partition)
            "vs_baseline": None, "dtype": "f32+i64", "data": "synthetic",
            "nproc": os.cpu_count(),
            "ingest": {"bytes": ingest_bytes, "ms": ingest_s * 1000.0, "GBps": ingest_bytes / ingest_s / 1e9,
                       "path": "pageable host numpy -> HBM (torch .to), before the timed steps"},
            "config": {"workload": W["desc"], "events_per_gpu": n, W["key_name"]: args.keys,
                       "rate_ev_per_ms": args.rate,
                       "output": {"packed": f"packed rows (SH_OUT_PACKED, {48 if args.agg else 32} B per match)",
                                  "columns": "typed columns (d_out_cols)",
                                  "raw": "raw 8-byte rows (d_out_values) + trigger_seq"}[layout],
                       "matches_per_gpu": int(m),
                       "parallelism": (f"dp{world}: every GPU matches its own partition of the key space (own "
                                       "stream, own keys), no data-path collective; rank 0's stream verified")
                       if world > 1 else "one GPU",
                       "bytes": W["bytes_note"]},
            "roofline": {"bound": "hbm", "achieved": achieved / 1e9, "peak": peak / 1e9, "unit": "GB/s",
                         "frac": achieved / peak, "traffic": traffic, "traffic_source": traffic_src,
                         "kernel": "matcher step (every kernel of one pass, HIP events on the launch stream)",
                         "kernels_ms_per_step": step_kernels_ms, "algorithmic_bytes": b_alg,
                         "match_kernel_only_GBps": match_only / 1e9},
            # the sharded step's phase names (main_sharded), so that a SCALE line reads
            # against this one: at N = 1 the whole step is the matcher
            "phase_ms": {"route_pack": 0.0, "exchange_out": 0.0, "unpack_match": step_kernels_ms,
                         "exchange_back": 0.0, "merge": 0.0, "segment": seg_ms, "advance": adv_ms,
                         "emit": emt_ms},
            "phase_ms_scope": "mean over the timed steps",
            # which device engine ran (DeviceRunner status: bucketed 1, sequence carry
            # seq3 2 / key-segment seq3 1, aggregates carried 4 / post-pass 1 / in lanes 3,
            # rule sets: sparse partials 1 / key-segment scan 0)
            "engine": {"bucket": runner.bucket_status(), "seq3": runner.seq3_status(),
                       "agg": runner.agg_status(), "rules_sparse": runner.rules_status()},
            "cpu_baseline": cpu,
            "verified_vs_restatement": verified,
        }
    runner.close()
    return line


if __name__ == "__main__":
    main()
