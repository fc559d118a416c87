#!/usr/bin/env python3
"""Predicted 1/2/4/8-GPU curves from one-GPU measurements (DESIGN.md "Multi-GPU").

Inputs (committed):
  profiles/r5_scale/<cfg>_n<N>_bench.json  one-GPU bench lines at the per-rank size of an
      N-GPU run: events/N, keys/N, rate/N (scripts/scale_predict.sh), kernel split in phase_ms
  profiles/r4_rehearse_c2_2ranks_gloo.json  rank 0's route + pack, unpack + match and merge
      times of the key-sharded step at 2 ranks (host-side rates of those kernels)

Weak scaling (bench.py's default at N > 1: every GPU its own key partition, no data-path
collective): the per-GPU step is the one-GPU step, so value(N) = N x events / t(1) before
host-side jitter. Strong scaling (--strong: one stream split by key): per rank
  t(N) = route_pack + exchange_out + unpack + match(N) + exchange_back + merge
with route / unpack / merge priced at the rehearsal's per-event and per-row rates, match(N)
the measured per-rank-size kernel time, and each all-to-all as the bytes one rank sends to
ONE peer (every pair of MI355X GPUs in a node has its own xGMI link) over LINK_GBPS.
usage: python scripts/scale_model.py [LINK_GBPS]"""
import json
import os
import sys

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
LINK = float(sys.argv[1]) if len(sys.argv) > 1 else 100.0  # GB/s per peer link (xGMI ~153 nominal)


def line(path):
    txt = open(os.path.join(HERE, path)).read().strip().splitlines()
    return json.loads([t for t in txt if t.startswith("{")][-1])


reh = line("profiles/r4_rehearse_c2_2ranks_gloo.json")
ph = reh["phase_ms_rank0_last_step"]
st = reh["config"]["rank0_step"]
recv, rows_home = sum(st["received"]), st["rows_home"]
match2 = reh["roofline"]["kernels_ms_per_step_max"]
route_per_ev = ph["route_pack"] / sum(st["sent"])               # ms per event sent
unpack_per_ev = (ph["unpack_match"] - match2) / recv            # ms per event received
merge_per_row = ph["merge"] / rows_home                         # ms per row merged

CFG = {  # events, record bytes out, row bytes back (raw rows: seq 8 + 8 per value)
    "c2": (100_000_000, 24, 8 + 4 * 8),
    "c3": (100_000_000, 24, 8 + 3 * 8),
    "c5": (100_000_000, 24, 8 + 8 + 2 * 8),
}

print(f"| config | N | per-rank match (measured, ms) | weak: events/s (N x one GPU) | strong: route+pack | exch. out | unpack | "
      f"exch. back | merge | strong: step ms | strong: events/s |")
print("|---|---|---|---|---|---|---|---|---|---|---|")
for cfg, (n, rec_b, row_b) in CFG.items():
    t1 = None
    for N in (1, 2, 4, 8):
        d = line(f"profiles/r5_scale/{cfg}_n{N}_bench.json")
        match = d["phase_ms"]["unpack_match"]
        m = d["config"]["matches_per_gpu"]  # rows of the per-rank slice
        if N == 1:
            t1 = d["ms_per_step"]
            print(f"| {cfg.upper()} | 1 | {match:.2f} | {n / t1 * 1e3 / 1e9:.1f} G | -- | -- | -- | -- | -- | "
                  f"{t1:.2f} | {n / t1 * 1e3 / 1e9:.1f} G |")
            continue
        ev = n / N
        route = route_per_ev * ev
        xout = (n / N / N) * rec_b / (LINK * 1e9) * 1e3
        unpack = unpack_per_ev * ev
        xback = (m / N) * row_b / (LINK * 1e9) * 1e3  # rows of one rank's keys going to one peer: m/N of m*N ... per pair
        merge = merge_per_row * m
        tot = route + xout + unpack + match + xback + merge
        print(f"| {cfg.upper()} | {N} | {match:.2f} | {N * n / t1 * 1e3 / 1e9:.1f} G | {route:.2f} | {xout:.2f} | "
              f"{unpack:.2f} | {xback:.2f} | {merge:.2f} | {tot:.2f} | {n / tot * 1e3 / 1e9:.1f} G |")
print(f"\nrates from the 2-rank rehearsal: route+pack {route_per_ev * 1e6:.3f} ns/event, unpack "
      f"{unpack_per_ev * 1e6:.3f} ns/event, merge {merge_per_row * 1e6:.3f} ns/row; link {LINK:.0f} GB/s per peer")
