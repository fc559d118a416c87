"""Probe: the C5 rule engine on one rank's share of the 100M stream (cards owned
by rank 0 of 2, arrival order), without any exchange -- does the per-key
timestamp check trip, and at which sizes?"""
import sys
import os
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from siddhi_amd import compiler, shard, synth  # noqa: E402
from siddhi_amd.device_run import DeviceRunner  # noqa: E402

n_all = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
K = 1_000_000
ts, card, amount, merchant = synth.txn_stream(n_all, K, 100, seed=synth.SEED + 5)
rules = synth.c5_rules(1000)
ca = compiler.compile_app(synth.c5_query(rules))
own = shard.shard_of(card, 2) == 0
idx = np.flatnonzero(own)
print("owned", len(idx), "of", n_all, flush=True)
# host check: per key non-decreasing timestamps in arrival order
o = np.lexsort((np.arange(len(idx)), card[idx]))
k2, t2 = card[idx][o], ts[idx][o]
bad = np.flatnonzero((k2[1:] == k2[:-1]) & (t2[1:] < t2[:-1]))
print("host: decreasing pairs", len(bad), flush=True)
dev = torch.device("cuda:0")
for n in [len(idx), len(idx) // 2, 20_000_000, 5_000_000]:
    sel = idx[:n]
    r = DeviceRunner(ca)
    tk = torch.from_numpy(card[sel].copy()).to(dev)
    t0 = time.time()
    try:
        m = r.run(torch.from_numpy(ts[sel].copy()).to(dev), tk,
                  [tk, torch.from_numpy(amount[sel].copy()).to(dev), torch.from_numpy(merchant[sel].copy()).to(dev)], K,
                  with_query=True)[0]
        print(n, "ok", m, f"{time.time() - t0:.2f}s", flush=True)
    except Exception as e:  # noqa: BLE001
        print(n, "FAILED", e, flush=True)
    r.close()
# the full stream (N = 1 path) for comparison
r = DeviceRunner(ca)
tk = torch.from_numpy(card).to(dev)
try:
    m = r.run(torch.from_numpy(ts).to(dev), tk, [tk, torch.from_numpy(amount).to(dev),
                                                torch.from_numpy(merchant).to(dev)], K, with_query=True)[0]
    print("full", n_all, "ok", m, flush=True)
except Exception as e:  # noqa: BLE001
    print("full FAILED", e, flush=True)
