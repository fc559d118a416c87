"""GPU parity of the bucketed engine's stack matcher (sh_stack.hip k_bk_stk)
through the C-ABI (sh_run_device) against the CPU oracle (oracle/refcpu.cpp, a
restatement of StreamPreStateProcessor.java:325-403) and, at full size, the
vectorised C2 restatement. Shapes: partitioned `every e1=S[f1] -> e2=S[x.a op
e1.a] within W` with every comparison operator, float and int attributes, ties
and NaN, 4 to 64 local keys per bucket, stacks deeper than the 16-entry LDS ring
(the HBM spill, and the host's retry with a deeper spill), bursts of one
millisecond, and skewed keys (one key's segment longer than a wave). Opening
filters on other attributes take the sort-and-walk matcher (status 1). Bit-exact
rows: trigger sequence numbers and raw select values.
DeviceRunner.bucket_status(): 2 = the stack matcher ran, 1 = the sort-and-walk one.
The stack matcher is opt-in (SH_STACK=1, the `engine="stack"` runs here): on C2 it
is slower than the sort-and-walk matcher (DESIGN.md "stack matcher")."""
import random

import numpy as np
import pytest

from c2_check import c2_expected
from oracle_engine import run_columns_oracle
from siddhi_amd import compiler, synth
from test_gpu_bucket import _run

pytestmark = pytest.mark.gpu

DEFS = "define stream S (sym string, price float, volume long, x int); "


@pytest.fixture(scope="module", autouse=True)
def _device():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _strings(nk):
    strings = compiler.StringDict()
    for i in range(nk):
        strings.id(f"K{i}")
    return strings


def _app(f1, f2, w, sel):
    q = (f"@info(name = 'query1') from every e1=S[{f1}] -> e2=S[{f2}] within {w} milliseconds "
         f"select {sel} insert into Out;")
    return DEFS + f"partition with (sym of S) begin {q} end;"


def _oracle_check(app, nk, ts, keys, price, vol, x, layout=False, expect=2):
    strings = _strings(nk)
    ca = compiler.compile_app(app, strings)
    seq, _, vals, nulls = run_columns_oracle(ca, ts, [keys, price, vol, x], keys)
    (m, oseq, ovals), status, err = _run(app, strings, ts, [keys, price, vol, x], keys, nk, layout, engine="stack")
    assert status in (expect if isinstance(expect, tuple) else (expect,)), (app, status, err)
    assert m == len(seq), app
    assert np.array_equal(oseq, seq.astype(np.int64)), app
    nn = ~nulls.astype(bool)
    assert np.array_equal(ovals[nn], vals[nn]), app
    return m


def _stream(seed, n, nk, rate_ms=50, prices=None, nan=0.0):
    rng = np.random.default_rng(seed)
    keys = rng.integers(0, nk, n).astype(np.int32)
    ts = (1_700_000_000_000 + np.arange(n, dtype=np.int64) // rate_ms).astype(np.int64)
    if prices is None:
        price = (rng.integers(0, 40, n) + rng.choice([0.0, 0.5, 0.25], n)).astype(np.float32)
    else:
        price = rng.choice(prices, n).astype(np.float32)
    if nan:
        price[rng.random(n) < nan] = np.float32("nan")
    vol = rng.integers(0, 6, n).astype(np.int64)
    x = rng.integers(-3, 25, n).astype(np.int32)
    return ts, keys, price, vol, x


@pytest.mark.parametrize("nk,n", [(2_000, 400_000), (4_000, 2_000_000), (9_000, 2_000_000), (16_000, 2_000_000)])
def test_c2_groups_vs_restatement(nk, n):
    """C2's query at 8 / 16 / 36 / 63 local keys per bucket (kb = 3, 4, 6, 6)"""
    ts, k, p, v = synth.stock_stream(n, nk, 100)
    (m, oseq, ovals), status, err = _run(synth.C2_QUERY, None, ts, [k, p, v], k, nk, "packed", engine="stack")
    assert status == 2, err
    eseq, evals = c2_expected(ts, k, p, v)
    assert m == len(eseq) > 0
    assert np.array_equal(oseq, eseq)
    assert np.array_equal(ovals, evals)


@pytest.mark.parametrize("seed", range(12))
def test_random_ordering_queries_vs_oracle(seed):
    """every operator on a float or an int attribute, opening filters on other
    attributes, windows from 0 ms, ties (few distinct values) and NaN prices"""
    rng = random.Random(7300 + seed)
    attr = rng.choice(["price", "x"])
    op = rng.choice([">", ">=", "<", "<="])
    f1t = rng.choice(["price > {c}f", "x < {c}", "volume >= {c}L", "price > 10.0 and x != {c}", "x % 3 == 1",
                      "price * 2.0f > {c}f", "{a} <= {c}", "{a} != {c}"])
    f1 = f1t.format(c=rng.randint(0, 20), a=attr)
    f2 = f"{attr} {op} e1.{attr}"
    extra = rng.random() < 0.3
    if extra:
        f2 += f" and e1.volume >= {rng.randint(0, 4)}L"  # a term on e1 alone joins the opening filter
    # the stack matcher's opening filter: terms on the ordering attribute and constants
    stack = not extra and (f1t.startswith("{a}") or (f1t == "price > {c}f" and attr == "price")
                           or (f1t == "x < {c}" and attr == "x"))
    w = rng.choice([0, 1, 5, 40, 1000])
    sel = ["e1.sym as a", f"e1.{attr} as b", "e2.price as c", "e2.volume as d", "e2.x as e"]
    rng.shuffle(sel)
    sel = sel[:rng.randint(2, 5)]
    app = _app(f1, f2, w, ", ".join(sel))
    nk = rng.choice([1024, 3000, 7000])
    n = rng.choice([120_000, 300_000])
    prices = [1.0, 2.0, 2.5, 3.0] if seed % 3 == 0 else None
    ts, keys, price, vol, x = _stream(seed, n, nk, rate_ms=rng.choice([1, 20, 100]), prices=prices,
                                      nan=0.01 if seed % 4 == 1 else 0.0)
    layout = [False, "packed", True][seed % 3]
    _oracle_check(app, nk, ts, keys, price, vol, x, layout, expect=2 if stack else (0, 1))


def test_deep_stacks_spill_exact():
    """long falling runs per key (stacks deeper than the 16-entry LDS ring) with
    occasional jumps that pop through the ring into the spilled entries"""
    n, nk = 400_000, 1500
    rng = np.random.default_rng(3)
    keys = rng.integers(0, nk, n).astype(np.int32)
    ts = (1_700_000_000_000 + np.arange(n, dtype=np.int64) // 100).astype(np.int64)
    step = np.where(rng.random(n) < 0.04, rng.uniform(1.0, 30.0, n), -rng.uniform(0.0, 0.3, n))
    price = np.zeros(n, np.float32)
    cur = np.full(nk, 50.0)
    for i in range(n):  # a per-key walk, mostly down
        cur[keys[i]] = max(1.0, cur[keys[i]] + step[i])
        price[i] = round(cur[keys[i]], 2)
    vol = rng.integers(0, 6, n).astype(np.int64)
    x = rng.integers(-3, 25, n).astype(np.int32)
    app = _app("price > 0.0f", "price > e1.price", 400, "e1.sym as a, e1.price as b, e2.price as c, e2.volume as d")
    m = _oracle_check(app, nk, ts, keys, price, vol, x, "packed", expect=2)
    assert m > 0


def test_bursts_longer_halo_exact():
    """one burst of 100k events in a single millisecond of an otherwise sparse
    stream: runs sized for the mean rate replay the burst's tiles as their halo,
    and the keys' stacks outgrow the spill sized for the mean rate (the host
    retries with a deeper one)"""
    n, nk = 600_000, 3000
    rng = np.random.default_rng(5)
    keys = rng.integers(0, nk, n).astype(np.int32)
    steps = np.ones(n, np.int64)
    steps[250_000:350_000] = 0
    ts = (1_700_000_000_000 + np.cumsum(steps)).astype(np.int64)
    price = (rng.integers(0, 30, n) + 0.5).astype(np.float32)
    vol = rng.integers(0, 6, n).astype(np.int64)
    x = rng.integers(-3, 25, n).astype(np.int32)
    app = _app("price > 3.0f", "price > e1.price", 1000, "e1.sym as a, e1.price as b, e2.price as c, e2.x as e")
    _oracle_check(app, nk, ts, keys, price, vol, x, expect=2)


def test_window_edge_exact():
    """partials exactly W apart are still pending (ts_q - ts_i > W expires)"""
    n, nk = 200_000, 1024
    rng = np.random.default_rng(8)
    keys = rng.integers(0, nk, n).astype(np.int32)
    ts = (1_700_000_000_000 + (np.arange(n, dtype=np.int64) // 64) * 5).astype(np.int64)
    price = rng.choice([1.0, 2.0, 3.0, 4.0], n).astype(np.float32)
    vol = rng.integers(0, 6, n).astype(np.int64)
    x = rng.integers(-3, 25, n).astype(np.int32)
    for w in (0, 5, 10):
        app = _app("price < 4.0f", "price > e1.price", w, "e1.sym as a, e1.price as b, e2.price as c")
        _oracle_check(app, nk, ts, keys, price, vol, x)


def test_skewed_keys_exact():
    """a few hot keys: one key's segment of a tile is longer than a wave (the
    matcher's rounds serialise its events)"""
    n, nk = 300_000, 4096
    rng = np.random.default_rng(9)
    keys = np.minimum(rng.zipf(1.3, n) - 1, nk - 1).astype(np.int32)
    ts = (1_700_000_000_000 + np.arange(n, dtype=np.int64) // 20).astype(np.int64)
    price = (rng.integers(0, 40, n) + 0.25).astype(np.float32)
    vol = rng.integers(0, 6, n).astype(np.int64)
    x = rng.integers(-3, 25, n).astype(np.int32)
    app = _app("price > 5.0f", "price > e1.price", 40, "e1.sym as a, e1.price as b, e2.price as c")
    _oracle_check(app, nk, ts, keys, price, vol, x, expect=2)
