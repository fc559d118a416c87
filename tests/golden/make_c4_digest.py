#!/usr/bin/env python3
"""Generates tests/golden/c4_digest.json: the CPU oracle (oracle/refcpu.cpp, the
C++ restatement of siddhi-core's processors, pinned by the reference's own test
fixtures in tests/test_oracle_golden.py) run once over the full SURVEY.md 8d C4
stream -- 100M events, 10M users, Login 20% / Txn 60% / Logout 20%, R = 100
ev/ms, send(Event[]) calls of 4,096 per stream (synth.c4_spec_stream, its fixed
seed) -- and the digest of its ordered output (tests/c4_cases.c4_digest: row
count and SHA-256 over trigger sequence, query, timestamp, values, nulls).
tests/test_gpu_c4.py holds the device to this digest: the scheduler's HashMap
(PartitionStateHolder / Scheduler.onTimeChange order) only resizes through the
tables of a 10M-key run at that size. Runtime ~10 min on one core.

The smaller streams of tests/test_gpu_c4.py are digested the same way
(--kind stream: synth.c4_stream(users, seconds); --kind spec --events 3000000
--users 1000000 [--every]), so the GPU suite compares against them instead of
running the oracle on the GPU box.

usage: python tests/golden/make_c4_digest.py [--kind spec|stream] [--events N --users U
       --seconds S --every]"""
import argparse
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--events", type=int, default=100_000_000)
    ap.add_argument("--users", type=int, default=10_000_000)
    ap.add_argument("--every", action="store_true")
    ap.add_argument("--kind", choices=["spec", "stream"], default="spec")
    ap.add_argument("--seconds", type=int, default=60)
    ap.add_argument("--out", default=os.path.join(HERE, "c4_digest.json"))
    a = ap.parse_args()
    from c4_cases import c4_digest, run_c4
    from oracle_engine import OracleEngine
    from siddhi_amd import compiler, synth
    t0 = time.time()
    if a.kind == "spec":
        blocks = synth.c4_spec_stream(a.events, a.users, rate_per_ms=100, batch=4096)
    else:
        blocks = synth.c4_stream(a.users, seconds=a.seconds)
    print(f"stream: {len(blocks)} calls in {time.time() - t0:.0f} s", flush=True)
    c = compiler.compile_app(synth.C4_EVERY_QUERY if a.every else synth.C4_QUERY)
    t1 = time.time()
    out = run_c4(OracleEngine(c), blocks, progress=lambda m: print(m, flush=True))
    d = c4_digest(out)
    if a.kind == "spec":
        d.update({"events": a.events, "users": a.users, "rate_ev_per_ms": 100, "batch": 4096,
                  "generator": "tests/golden/make_c4_digest.py (synth.c4_spec_stream, oracle/refcpu.cpp)"})
        key = ("every" if a.every else "default") + f"_{a.events}_{a.users}"
    else:
        d.update({"users": a.users, "seconds": a.seconds,
                  "generator": "tests/golden/make_c4_digest.py --kind stream (synth.c4_stream, oracle/refcpu.cpp)"})
        key = ("every" if a.every else "default") + f"_stream_{a.users}_{a.seconds}"
    d.update({"query": "every" if a.every else "default", "oracle_seconds": round(time.time() - t1, 1)})
    res = json.load(open(a.out)) if os.path.exists(a.out) else {}
    res[key] = d
    json.dump(res, open(a.out, "w"), indent=1, sort_keys=True)
    print(json.dumps(d), flush=True)


if __name__ == "__main__":
    main()
