"""tests/agg_check.py (per-key running sums in match order) pinned to the oracle on
the C2 aggregate query, so it can check the device at full size."""
import numpy as np


def test_running_aggregates_equal_the_oracle():
    from agg_check import raw_bits, running
    from c2_check import c2_expected
    from oracle_engine import run_stock_oracle
    from siddhi_amd import compiler, synth
    from test_gpu_agg import C2_AGG
    ts, k, p, v = synth.stock_stream(150_000, 500, 100)
    seq, _, vals, _ = run_stock_oracle(compiler.compile_app(C2_AGG), ts, k, p, v)
    eseq, ev = c2_expected(ts, k, p, v)
    assert np.array_equal(seq.astype(np.int64), eseq) and len(eseq) > 0
    grp = k[eseq].astype(np.int64)
    p2 = ev[:, 2].astype(np.uint32).view(np.float32).astype(np.float64)
    p1 = ev[:, 1].astype(np.uint32).view(np.float32).astype(np.float64)
    assert np.array_equal(vals[:, 0], ev[:, 0])
    assert np.array_equal(vals[:, 1], raw_bits(running(grp, p2, "sum")))
    assert np.array_equal(vals[:, 2], raw_bits(running(grp, p1, "avg")))
    assert np.array_equal(vals[:, 3], running(grp, None, "count"))
    assert np.array_equal(vals[:, 4], running(grp, ev[:, 3], "sum"))
