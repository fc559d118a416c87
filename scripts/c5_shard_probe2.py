"""Probe: the sharded C5 step at full size with 2 virtual ranks on one GPU (threads);
when a rank's matcher fails, check its received events on the host (per-key
timestamps in arrival order, run ids, sequence numbers)."""
import os
import sys
import threading

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from siddhi_amd import compiler, shard, synth  # noqa: E402
from siddhi_amd.device_run import DeviceRunner  # noqa: E402
from test_gpu_shard import _ThreadComm, _ops  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
K = 1_000_000
world = 2
ts, card, amount, merchant = synth.txn_stream(n, K, 100, seed=synth.SEED + 5)
ca = compiler.compile_app(synth.c5_query(synth.c5_rules(1000)))
b = shard.slice_bounds(n, world, align=4096)
rid = shard.stream_run_ids(card, 4096)
comm = _ThreadComm(world)
errs = []


def check_inputs(r, t, kk, run):
    t, kk = t.cpu().numpy(), kk.cpu().numpy()
    o = np.lexsort((np.arange(len(kk)), kk))
    bad = np.flatnonzero((kk[o][1:] == kk[o][:-1]) & (t[o][1:] < t[o][:-1]))
    print(f"rank {r}: received {len(t)}, ts non-decreasing overall: {bool(np.all(np.diff(t) >= 0))}, "
          f"per-key decreases: {len(bad)}", flush=True)
    if len(bad):
        i = o[bad[0]]
        print(f"  first: key {kk[o][bad[0]]} positions {o[bad[0]]} / {o[bad[0] + 1]} ts {t[o][bad[0]]} -> "
              f"{t[o][bad[0] + 1]}", flush=True)
    if run is not None:
        rr = run.cpu().numpy().view(np.uint32)
        print(f"  run ids non-decreasing: {bool(np.all(np.diff(rr.astype(np.int64)) >= 0))}", flush=True)
    _ = i if len(bad) else None


def rank_main(r):
    try:
        runner = DeviceRunner(ca)

        def matcher(t, kk, cc, nk, run=None):
            try:
                res = runner.run(t, kk, cc, nk, with_query=True, run_ids=run)
            except Exception as e:  # noqa: BLE001
                print(f"rank {r}: matcher failed: {e}", flush=True)
                check_inputs(r, t, kk, run)
                raise
            m, s_, v, q = res
            print(f"rank {r}: ok, {m} matches", flush=True)
            return m, s_, torch.cat([v, q[:m].to(torch.int64).view(-1, 1)], 1)

        step = shard.KeyShardedStep(world, r, _ops(), matcher, n_out=runner.n_out + 1, comm=comm.view(r))
        lo, hi = b[r], b[r + 1]
        dev = [torch.from_numpy(a[lo:hi].copy()).cuda() for a in [ts, card, amount, merchant]]
        d_run = torch.from_numpy(rid[lo:hi].copy()).cuda()
        step.run(dev[0], dev[1], dev[1:], lo, K, key_attr=0, run_ids=d_run)
        torch.cuda.synchronize()
        runner.close()
    except BaseException as e:  # noqa: BLE001
        errs.append(e)
        comm.bar.abort()


th = [threading.Thread(target=rank_main, args=(r,)) for r in range(world)]
for t in th:
    t.start()
for t in th:
    t.join(timeout=600)
print("errors:", errs)
