"""One C2-shaped run on the GPU on the stack matcher (SH_STACK=1) with its diagnostics (SH_STK_DEBUG)."""
import os
import sys
import time

os.environ.setdefault("SH_STK_DEBUG", "1")
os.environ.setdefault("SH_STACK", "1")
ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)
import numpy as np
import torch

from c2_check import c2_expected
from siddhi_amd import compiler, synth
from siddhi_amd.device_run import DeviceRunner, packed_to_raw

n = int(sys.argv[1]) if len(sys.argv) > 1 else 400_000
nk = int(sys.argv[2]) if len(sys.argv) > 2 else 2000
ts, k, p, v = synth.stock_stream(n, nk, 100)
runner = DeviceRunner(compiler.compile_app(synth.C2_QUERY))
dev = torch.device("cuda:0")
tcols = [torch.from_numpy(c).to(dev) for c in (k, p, v)]
offs, rb = runner.packed_layout()
for it in range(3):
    t0 = time.perf_counter()
    m, rows = runner.run(torch.from_numpy(ts).to(dev), tcols[0], tcols, nk, packed=True)
    torch.cuda.synchronize()
    print("run", it, "m", m, "status", runner.bucket_status(), "refused", hex(runner.stack_refused()),
          "times", runner.kernel_times(), "wall ms", (time.perf_counter() - t0) * 1e3, flush=True)
oseq, ovals = packed_to_raw(rows.cpu().numpy(), runner.out_types, offs, rb)
eseq, evals = c2_expected(ts, k, p, v)
print("expected", len(eseq), "seq equal", len(oseq) == len(eseq) and np.array_equal(oseq.astype(np.int64), eseq),
      "vals equal", len(oseq) == len(eseq) and np.array_equal(ovals, evals))
if len(oseq) == len(eseq):
    bad = np.flatnonzero((oseq.astype(np.int64) != eseq) | (ovals != evals).any(1))
    print("first bad rows", bad[:10])
oc = np.bincount(oseq.astype(np.int64), minlength=n)
ec = np.bincount(eseq, minlength=n)
bad = np.flatnonzero(oc != ec)
print("events with wrong counts", len(bad), "first", bad[:8].tolist())
for j in bad[:3]:
    key = k[j]
    idx = np.flatnonzero(k[:j + 1] == key)[-14:]
    print(f"event {j} key {key} got {oc[j]} expected {ec[j]}")
    for i in idx:
        print(f"   i {i} ts {ts[i] - ts[0]} price {p[i]:.2f} got {oc[i]} exp {ec[i]}")
    sel = np.flatnonzero(oseq == j)
    print("   got rows p1:", [np.array([r], np.uint32).view(np.float32)[0] for r in ovals[sel, 1]])
    sel = np.flatnonzero(eseq == j)
    print("   exp rows p1:", [np.array([r], np.uint32).view(np.float32)[0] for r in evals[sel, 1]])
