"""GPU parity of the bucketed window engine (sh_bucket.hip + shb_match) through
the C-ABI (sh_run_device) against the CPU oracle: partitioned
`every e1=S[f1] -> e2=S[f2] within W` with >= 1,024 keys. Bit-exact rows:
trigger sequence numbers and raw select values. The engine's device premises
(packed timestamp range, non-decreasing timestamps per key, halo coverage,
<= 255 partials per consumer) send the run back to the general window path;
those cases must stay exact too."""
import os
import random

import numpy as np
import pytest

from c2_check import c2_expected
from oracle_engine import run_columns_oracle, run_stock_oracle
from window_cases import window_case
from siddhi_amd import compiler, synth

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _device():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _run(app, strings, ts, cols, keys, nk, columns=False, batch_events=4096):
    """columns: typed output columns (d_out_cols), "packed": SH_OUT_PACKED rows;
    both returned as raw rows for comparison"""
    return _run_inner(app, strings, ts, cols, keys, nk, columns, batch_events)


def _run_inner(app, strings, ts, cols, keys, nk, columns, batch_events):
    import torch
    from siddhi_amd.device_run import DeviceRunner, columns_to_raw, packed_to_raw
    runner = DeviceRunner(compiler.compile_app(app, strings))
    dev = torch.device("cuda:0")
    tcols = [torch.from_numpy(c).to(dev) for c in cols]
    if columns == "packed":
        offs, rb = runner.packed_layout()
        m, rows = runner.run(torch.from_numpy(ts).to(dev), torch.from_numpy(keys).to(dev), tcols, nk,
                             packed=True, batch_events=batch_events)
        torch.cuda.synchronize()
        status, err = runner.bucket_status(), runner.last_error()
        oseq, ovals = packed_to_raw(rows.cpu().numpy(), runner.out_types, offs, rb)
        runner.close()
        return (m, oseq.astype(np.int64), ovals), status, err
    m, oseq, ovals = runner.run(torch.from_numpy(ts).to(dev), torch.from_numpy(keys).to(dev), tcols, nk,
                                columns=columns, batch_events=batch_events)
    torch.cuda.synchronize()
    status = runner.bucket_status()
    err = runner.last_error()
    if columns:
        assert [c.dtype for c in ovals] == [{0: torch.int32, 1: torch.int32, 2: torch.int64, 3: torch.float32,
                                             4: torch.float64, 5: torch.uint8}[t] for t in runner.out_types]
        res = (m, oseq.cpu().numpy(), columns_to_raw([c.cpu().numpy() for c in ovals], runner.out_types))
    else:
        res = (m, oseq.cpu().numpy(), ovals.cpu().numpy())
    runner.close()
    return res, status, err


def test_c2_bucket_vs_oracle():
    n, nk = 400_000, 2_000
    ts, k, p, v = synth.stock_stream(n, nk, 100)
    ca = compiler.compile_app(synth.C2_QUERY)
    seq, _, vals, _ = run_stock_oracle(ca, ts, k, p, v)
    (m, oseq, ovals), status, err = _run(synth.C2_QUERY, None, ts, [k, p, v], k, nk)
    assert status == 1, err
    assert m == len(seq) > 0
    assert np.array_equal(oseq, seq.astype(np.int64))
    assert np.array_equal(ovals, vals)


@pytest.mark.parametrize("n,nk,bucketed,columns", [
    (10_000_000, 10_000, 1, False), (100_000_000, 10_000, 1, "packed"), (100_000_000, 10_000, 1, True),
    (3_000_000, 60_000, 1, False), (3_000_000, 60_000, 1, True), (3_000_000, 60_000, 1, "packed")])
def test_c2_bucket_full_size_vs_restatement(n, nk, bucketed, columns):
    """60k symbols at 100 ev/ms: a key's previous event is often more than a
    window back, so many walks leave their key's run in the span; the halo covers
    the window in time and the check against the latest timestamp before the
    span (tpre) proves those walks complete, so the run stays bucketed.
    `columns`: typed output columns or packed rows (the bucketed engine writes them
    itself; "packed" at 100M is the bench's layout)"""
    ts, k, p, v = synth.stock_stream(n, nk, 100)
    (m, oseq, ovals), status, err = _run(synth.C2_QUERY, None, ts, [k, p, v], k, nk, columns)
    assert status == bucketed, err
    eseq, evals = c2_expected(ts, k, p, v)
    assert m == len(eseq) > 0
    assert np.array_equal(oseq, eseq)
    assert np.array_equal(ovals, evals)


def _random_stream(seed, n, nk, ts_steps=(0, 0, 1, 2, 3), skew=False):
    rng = np.random.default_rng(seed)
    if skew:  # a few hot keys and a long tail (sparse keys exercise the halo)
        keys = np.minimum(rng.zipf(1.3, n) - 1, nk - 1).astype(np.int32)
    else:
        keys = rng.integers(0, nk, n).astype(np.int32)
    ts = (1_700_000_000_000 + np.cumsum(rng.choice(ts_steps, n))).astype(np.int64)
    price = (rng.integers(0, 40, n) + rng.choice([0.0, 0.5, 0.25], n)).astype(np.float32)
    vol = rng.integers(0, 6, n).astype(np.int64)
    x = rng.integers(-3, 25, n).astype(np.int32)
    return keys, ts, price, vol, x


@pytest.mark.parametrize("seed", range(16))
def test_random_window_queries_bucket_vs_oracle(seed):
    rng = random.Random(9100 + seed)
    app, partitioned = window_case(rng)
    if not partitioned:
        defs = app[:app.index(";") + 2]
        app = defs + "partition with (sym of S) begin " + app[len(defs):] + " end;"
    nk = rng.choice([1024, 3000, 20000])
    n = rng.choice([40_000, 120_000, 300_000])
    keys, ts, price, vol, x = _random_stream(seed, n, nk, skew=seed % 4 == 3)
    strings = compiler.StringDict()
    for i in range(nk):
        strings.id(f"K{i}")
    ca = compiler.compile_app(app, strings)
    seq, _, vals, nulls = run_columns_oracle(ca, ts, [keys, price, vol, x], keys)
    layout = [False, "packed", True][seed % 3]  # raw rows, packed rows, typed columns
    (m, oseq, ovals), status, err = _run(app, strings, ts, [keys, price, vol, x], keys, nk, layout)
    assert status >= 0, err  # 1 bucketed, 0 another engine (not applicable / premise failed)
    assert m == len(seq), app
    assert np.array_equal(oseq, seq.astype(np.int64)), app
    nn = ~nulls.astype(bool)
    assert np.array_equal(ovals[nn], vals[nn]), app


def test_decreasing_timestamps_fall_back_exactly():
    """timestamps going back inside a key: the device flags it and the run is
    redone on the general window path (StreamPreStateProcessor's expiry is then
    not a forward scan)"""
    n, nk = 120_000, 2048
    keys, ts, price, vol, x = _random_stream(5, n, nk)
    ts[::97] -= 5
    app = ("define stream S (sym string, price float, volume long, x int); partition with (sym of S) begin "
           "from every e1=S[price > 5.0f] -> e2=S[price > e1.price] within 40 milliseconds "
           "select e1.sym as a, e1.price as b, e2.price as c, e2.volume as d insert into Out; end;")
    strings = compiler.StringDict()
    for i in range(nk):
        strings.id(f"K{i}")
    ca = compiler.compile_app(app, strings)
    seq, _, vals, _ = run_columns_oracle(ca, ts, [keys, price, vol, x], keys)
    (m, oseq, ovals), status, err = _run(app, strings, ts, [keys, price, vol, x], keys, nk, "packed")
    assert status == 0, "the bucketed engine must not accept decreasing timestamps"
    assert m == len(seq) and np.array_equal(oseq, seq.astype(np.int64)) and np.array_equal(ovals, vals)


def test_long_window_counts_exact():
    """a wide window with few distinct prices: consumers take many partials each"""
    n, nk = 200_000, 1024
    rng = np.random.default_rng(11)
    keys = rng.integers(0, nk, n).astype(np.int32)
    ts = (1_700_000_000_000 + np.arange(n) // 50).astype(np.int64)
    price = rng.choice([1.0, 2.0, 3.0], n).astype(np.float32)
    vol = rng.integers(0, 6, n).astype(np.int64)
    x = rng.integers(-3, 25, n).astype(np.int32)
    app = ("define stream S (sym string, price float, volume long, x int); partition with (sym of S) begin "
           "from every e1=S[price < 3.0f] -> e2=S[price > e1.price] within 1 sec "
           "select e1.sym as a, e1.x as b, e2.price as c, e2.volume as d, e1.price as e insert into Out; end;")
    strings = compiler.StringDict()
    for i in range(nk):
        strings.id(f"K{i}")
    ca = compiler.compile_app(app, strings)
    seq, _, vals, _ = run_columns_oracle(ca, ts, [keys, price, vol, x], keys)
    (m, oseq, ovals), status, err = _run(app, strings, ts, [keys, price, vol, x], keys, nk)
    assert status >= 0, err
    assert m == len(seq) > 0 and np.array_equal(oseq, seq.astype(np.int64)) and np.array_equal(ovals, vals)


@pytest.mark.parametrize("query,layout", [("c3", "packed"), ("c3", True), ("c1", "packed"), ("c2agg", "packed")])
def test_layouts_on_other_engines(query, layout):
    """packed rows / typed columns from the engines that write raw rows into the
    workspace for a conversion (rise-and-fall sequence, the unpartitioned window
    path, the aggregate post-pass): identical to the raw rows of the same run"""
    app = {"c3": synth.C3_QUERY, "c1": synth.C1_QUERY, "c2agg": synth.C2_AGG_QUERY}[query]
    n, nk = 300_000, 2_000
    ts, k, p, v = synth.stock_stream(n, nk, 100)
    (m0, seq0, vals0), _, err0 = _run(app, None, ts, [k, p, v], k, nk)
    (m1, seq1, vals1), _, err1 = _run(app, None, ts, [k, p, v], k, nk, layout)
    assert m0 == m1 > 0, (err0, err1)
    assert np.array_equal(seq0, seq1)
    assert np.array_equal(vals0, vals1)
