"""C3 (BASELINE.json configs[2]) through sh_run_device on its device forms:
the bucket-carry engine (sh_bucket.hip, seq3 status 2: k_s3b, one workgroup per key
bucket, the default), the
rise-and-fall key-segment engine (k_seq3s / k_seq3, sh_nfa.hip, status 1;
SH_DISABLE_S3B=1) and the general engine (SH_NO_SEQ3=1, status 0): bit-exact
against the oracle at 300k events (with price ties), against the vectorised
restatement tests/c3_check.py (pinned to the oracle in tests/test_c3_checker.py)
at the full 100M events / 1M keys, and the shape's near relatives."""
import os

import numpy as np
import pytest

from c3_check import c3_expected
from oracle_engine import run_columns_oracle, run_stock_oracle
from siddhi_amd import compiler, synth

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _device():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _gpu(text, ts, cols, keys, nk):
    import torch
    from siddhi_amd.device_run import DeviceRunner
    runner = DeviceRunner(compiler.compile_app(text))
    dev = torch.device("cuda:0")
    m, oseq, ovals = runner.run(torch.from_numpy(ts).to(dev), torch.from_numpy(keys).to(dev),
                                [torch.from_numpy(c).to(dev) for c in cols], nk)
    torch.cuda.synchronize()
    r = (oseq.cpu().numpy(), ovals.cpu().numpy(), runner.seq3_status())
    runner.close()
    return r


ENGINE = {"s3b": 2, "seq3": 1, "general": 0}


def _engine(engine, monkeypatch):
    if engine == "general":
        monkeypatch.setenv("SH_NO_SEQ3", "1")
    elif engine == "seq3":
        monkeypatch.setenv("SH_DISABLE_S3B", "1")
    return ENGINE[engine]


@pytest.mark.parametrize("ties,engine", [(False, "s3b"), (True, "s3b"),
                                         (False, "seq3"), (True, "seq3"), (False, "general")])
def test_c3_vs_oracle(ties, engine, monkeypatch):
    want = _engine(engine, monkeypatch)
    n, nk = 300_000, 5_000
    ts, k, p, v = synth.stock_stream(n, nk, 1000, config_index=3)
    if ties:
        p = np.random.default_rng(3).integers(0, 5, n).astype(np.float32)
    seq, _, vals, _ = run_stock_oracle(compiler.compile_app(synth.C3_QUERY), ts, k, p, v)
    gseq, gvals, st = _gpu(synth.C3_QUERY, ts, [k, p, v], k, nk)
    assert st == want
    assert len(gseq) == len(seq) > 0
    assert np.array_equal(gseq, seq.astype(np.int64)) and np.array_equal(gvals, vals)


@pytest.mark.parametrize("engine", ["s3b", "seq3"])
def test_c3_full_size_vs_restatement(engine, monkeypatch):
    want = _engine(engine, monkeypatch)
    n, nk = 100_000_000, 1_000_000
    ts, k, p, v = synth.stock_stream(n, nk, 1000, config_index=3)
    gseq, gvals, st = _gpu(synth.C3_QUERY, ts, [k, p, v], k, nk)
    assert st == want
    eseq, evals = c3_expected(ts, k, p)
    assert len(gseq) == len(eseq) > 0
    assert np.array_equal(gseq, eseq) and np.array_equal(gvals, evals)


def test_mixed_attribute_shape_vs_oracle():
    """other attributes / operators / select columns of the same shape"""
    text = ("define stream S (symbol string, price float, volume long); partition with (symbol of S) begin "
            "from every e1=S, e2=S[volume >= e1.volume]+, e3=S[e2[last].price > price] "
            "select e3.volume as v3, e1.symbol as s, e2[last].volume as lv, e1.price as p1 insert into Out; end;")
    n, nk = 200_000, 3_000
    ts, k, p, v = synth.stock_stream(n, nk, 100, config_index=3)
    v = np.random.default_rng(9).integers(0, 4, n).astype(np.int64)
    seq, _, vals, _ = run_columns_oracle(compiler.compile_app(text), ts, [k, p, v], k)
    gseq, gvals, st = _gpu(text, ts, [k, p, v], k, nk)
    assert st == 1
    assert len(gseq) == len(seq) > 0
    assert np.array_equal(gseq, seq.astype(np.int64)) and np.array_equal(gvals, vals)


@pytest.mark.parametrize("engine", ["s3b", "seq3", "general"])
def test_c3_18bit_keys_vs_restatement(engine, monkeypatch):
    """200k keys (18 bits): 10 local key bits per bucket on the carry engine (two
    6-bit sort passes per chunk); three 8-bit radix passes on the key-segment ones"""
    want = _engine(engine, monkeypatch)
    n, nk = 4_000_000, 200_000
    ts, k, p, v = synth.stock_stream(n, nk, 1000, config_index=3)
    gseq, gvals, st = _gpu(synth.C3_QUERY, ts, [k, p, v], k, nk)
    assert st == want
    eseq, evals = c3_expected(ts, k, p)
    assert len(gseq) == len(eseq) > 0
    assert np.array_equal(gseq, eseq) and np.array_equal(gvals, evals)


@pytest.mark.parametrize("engine", ["s3b", "seq3"])
@pytest.mark.parametrize("variant", ["null_keys", "all_null", "hot_key", "generic_records", "unstaged",
                                     "few_keys"])
def test_c3_seq3_edge_cases_vs_oracle(variant, engine, monkeypatch):
    """edges: null-key events (no bucket on the carry engine; the run after the
    last segment on k_seq3s), no keyed event at all, one hot key (30% of the events:
    one tile per carry chunk; many rounds of one lane on k_seq3s), 64 local keys
    (kb = 6: one sort pass); and k_seq3s's A/B forms (generic records, the one-lane-
    per-key k_seq3)"""
    if engine == "s3b" and variant in ("generic_records", "unstaged"):
        pytest.skip("k_seq3s forms")
    want = _engine(engine, monkeypatch)
    n, nk = 200_000, 2_000
    if variant == "few_keys":
        nk = 16_384
    ts, k, p, v = synth.stock_stream(n, nk, 1000, config_index=3)
    k = k.copy()
    rng = np.random.default_rng(11)
    if variant == "null_keys":
        k[rng.random(n) < 0.1] = -1
    elif variant == "all_null":
        k[:] = -1
    elif variant == "hot_key":
        k[rng.random(n) < 0.3] = 7
    elif variant == "generic_records":
        monkeypatch.setenv("SH_S3_COMPACT", "0")
    else:
        monkeypatch.setenv("SH_S3_STAGED", "0")
    seq, _, vals, _ = run_columns_oracle(compiler.compile_app(synth.C3_QUERY), ts, [k, p, v], k)
    gseq, gvals, st = _gpu(synth.C3_QUERY, ts, [k, p, v], k, nk)
    assert st == want
    assert len(gseq) == len(seq)
    assert (len(seq) == 0) == (variant == "all_null")
    assert np.array_equal(gseq, seq.astype(np.int64)) and np.array_equal(gvals, vals)
