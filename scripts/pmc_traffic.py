#!/usr/bin/env python3
"""HBM traffic per bench step from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE).

usage: pmc_traffic.py <fetch_dir> <write_dir> <steps> <events> <keys> <out.json> [config]
                      [--calib <cal_fetch_dir> <cal_write_dir> <bytes_per_kernel>]
                      [--agg] [--layout packed|raw|columns] [--engine TAG]

steps = every matcher pass the profiled bench ran (its --warmup + --steps). The
output records the variant (config, --agg, --layout, bench.engine_tag()) so
bench.py attaches it only to a line of that exact workload.

FETCH_SIZE / WRITE_SIZE are in KB (rocprofv3 derived counters). MI355X_MICROARCH.md
(HBM section) calibrates FETCH_SIZE at 1/2 of the bytes only for 16-B-per-lane
streaming reads and leaves other widths uncalibrated. With --calib the factors are
measured on this machine from known-byte streams in the widths the matcher kernels
use (scripts/pmc_calib.py: 4 and 8 B per lane, 2 GiB each, past the Infinity Cache):
factor = bytes / counter bytes, read4 for reads, write4 for writes (the dominant
widths); without it the guide's x2 read correction is used. Both counters count
memory-side (fabric) requests, so Infinity-Cache hits are included: this is L2-miss
traffic, an upper bound on HBM bytes.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def load(d, counter):
    per = defaultdict(float)
    calls = defaultdict(set)
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    for f in files:
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") != counter:
                continue
            name = r.get("Kernel_Name", "?").split("(")[0]
            per[name] += float(r["Counter_Value"])
            calls[name].add(r.get("Dispatch_Id"))
    return per, {k: len(v) for k, v in calls.items()}, files


def calib(fdir, wdir, nbytes):
    f, _, _ = load(fdir, "FETCH_SIZE")
    w, _, _ = load(wdir, "WRITE_SIZE")
    fac = {}
    for k, v in f.items():
        if "k_cal_read" in k and v > 0:
            fac["read8" if "unsigned long" in k or "ImE" in k else "read4"] = nbytes / (v * 1024.0)
    for k, v in w.items():
        if "k_cal_write" in k and v > 0:
            fac["write8" if "unsigned long" in k or "ImE" in k else "write4"] = nbytes / (v * 1024.0)
    return fac


def main():
    args = sys.argv[1:]
    cal = None
    if "--calib" in args:
        i = args.index("--calib")
        cal = calib(args[i + 1], args[i + 2], float(args[i + 3]))
        args = args[:i] + args[i + 4:]
    agg = "--agg" in args
    layout = "raw"
    if "--layout" in args:
        i = args.index("--layout")
        layout = args[i + 1]
        args = args[:i] + args[i + 2:]
    engine = None
    if "--engine" in args:
        i = args.index("--engine")
        engine = args[i + 1]
        args = args[:i] + args[i + 2:]
    args = [a for a in args if a != "--agg"]
    fdir, wdir, steps, events, keys, out = args[:6]
    config = args[6] if len(args) > 6 else "c2"
    steps = int(steps)
    rfac = cal.get("read4", 2.0) if cal else 2.0
    wfac = cal.get("write4", 1.0) if cal else 1.0
    fetch, fcalls, ff = load(fdir, "FETCH_SIZE")
    write, _, wf = load(wdir, "WRITE_SIZE")
    if not ff or not wf:
        print("no counter files found", ff, wf)
        sys.exit(1)
    kernels = {}
    tot = 0.0
    for k in sorted(set(fetch) | set(write)):
        if k.startswith("__amd_rocclr"):
            continue  # memsets / copies outside the matcher
        rb = rfac * fetch.get(k, 0.0) * 1024.0 / steps
        wb = wfac * write.get(k, 0.0) * 1024.0 / steps
        kernels[k] = {"read_bytes": rb, "write_bytes": wb, "calls_per_step": fcalls.get(k, 0) / steps}
        tot += rb + wb
    res = {"config": config, "events": int(events), "keys": int(keys), "steps": steps, "agg": agg, "layout": layout,
           "engine": engine,
           "hbm_bytes_per_step": tot, "kernels": kernels,
           "calibration": cal, "read_factor": rfac, "write_factor": wfac,
           "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate runs; counters scaled by "
                     + ("factors measured on known 4/8-B-per-lane streams (scripts/pmc_calib.py)" if cal else
                        "the guide's x2 read correction (MI355X_MICROARCH.md HBM section)")
                     + "; L2-miss bytes incl. Infinity-Cache hits"}
    json.dump(res, open(out, "w"), indent=1)
    for k, v in sorted(kernels.items(), key=lambda kv: -(kv[1]["read_bytes"] + kv[1]["write_bytes"])):
        print(f"{k[:40]:40s} R {v['read_bytes']/1e9:7.3f} GB  W {v['write_bytes']/1e9:7.3f} GB")
    print(f"total {tot/1e9:.3f} GB per step")


if __name__ == "__main__":
    main()
