"""C3 on the general engine: device run vs the oracle (small), timing at scale."""
import sys, time
sys.path.insert(0, '.'); sys.path.insert(0, 'tests')
import numpy as np, torch
from siddhi_amd import compiler, synth
from siddhi_amd.device_run import DeviceRunner
from oracle_engine import run_stock_oracle

def run(n, K, rate, check):
    ts, k, p, v = synth.stock_stream(n, K, rate, config_index=3)
    ca = compiler.compile_app(synth.C3_QUERY)
    r = DeviceRunner(ca)
    dev = torch.device('cuda:0')
    tts, tk, tp, tv = [torch.from_numpy(x).to(dev) for x in (ts, k, p, v)]
    for it in range(3):
        torch.cuda.synchronize(); t0 = time.perf_counter()
        m, oseq, ovals = r.run(tts, tk, [tk, tp, tv], K, out_capacity=n)
        torch.cuda.synchronize(); dt = time.perf_counter() - t0
        print(f"n={n} K={K} matches={m} {dt*1e3:.1f} ms {n/dt/1e9:.3f} Gev/s kt={r.kernel_times()}", flush=True)
    if check:
        seq, ots, vals, _ = run_stock_oracle(ca, ts, k, p, v, batch=4096)
        ok = m == len(seq) and np.array_equal(oseq.cpu().numpy(), seq.astype(np.int64)) and np.array_equal(ovals.cpu().numpy(), vals)
        print("parity vs oracle:", ok, m, len(seq), flush=True)
        assert ok
    r.close()

run(200_000, 2_000, 1000, True)
run(2_000_000, 100_000, 1000, True)
run(100_000_000, 1_000_000, 1000, False)
