"""Select-clause aggregators on the fast engines. The bucketed engine (C2 shape)
carries every key's running sum / avg / count across its buckets: by default as a
segmented prefix in 64-bit fixed point, exact by construction (k_bk_aggp,
agg_status 5), and in arrival order (k_bk_aggc, agg_status 4: the reference's own
sequence of additions) when that and the post-pass refuse or SH_BK_AGGC=1; the
window engine (C1), the rise-and-fall key-segment engine (C3) and the rule set
(C5) write the aggregators' arguments and the sh_agg.hip post-pass forms the
running values per (query, partition key) in match order after proving the
double additions exact (agg_status 1; SH_BK_AGG_POST=1 sends the bucketed engine
there too). Bit-exact against the oracle (QuerySelector + Sum/Avg aggregators
restated), and at full size against the vectorised restatement
(tests/agg_check.py). A stream whose additions round takes the sequential
engines from the post-pass (agg_status 2) and still matches the oracle."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

C2_AGG = ("define stream StockStream (symbol string, price float, volume long); "
          "partition with (symbol of StockStream) begin @info(name = 'query1') "
          "from every e1=StockStream[price>20] -> e2=StockStream[symbol==e1.symbol and price>e1.price] "
          "within 1 sec select e1.symbol as symbol, sum(e2.price) as total, avg(e1.price) as a1, "
          "count() as n, sum(e2.volume) as vol insert into Out; end;")
C1_AGG = C2_AGG.replace("partition with (symbol of StockStream) begin ", "").replace(" end;", "")
C3_AGG = ("define stream S (symbol string, price float, volume long); "
          "partition with (symbol of S) begin @info(name = 'query1') "
          "from every e1=S, e2=S[price>e1.price]+, e3=S[price<e2[last].price] "
          "select e1.price as p1, sum(e3.price) as s3, avg(e2[last].price) as apeak, count() as n "
          "insert into Out; end;")


@pytest.fixture(scope="module", autouse=True)
def _device():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _run(text, ts, k, cols, nkeys, with_query=False, packed=False):
    import torch
    from siddhi_amd import compiler
    from siddhi_amd.device_run import DeviceRunner, packed_to_raw
    r = DeviceRunner(compiler.compile_app(text))
    dev = torch.device("cuda:0")
    tk = torch.from_numpy(k).to(dev)
    res = r.run(torch.from_numpy(ts).to(dev), tk, [torch.from_numpy(c).to(dev) for c in cols], nkeys,
                with_query=with_query, packed=packed)
    torch.cuda.synchronize()
    if packed:
        offs, rb = r.packed_layout()
        oseq, ovals = packed_to_raw(res[1].cpu().numpy(), r.out_types, offs, rb)
        out = [res[0], oseq.view(np.int64), ovals]
    else:
        out = [res[0]] + [x.cpu().numpy() for x in res[1:]]
    st = dict(agg=r.agg_status(), bucket=r.bucket_status(), seq3=r.seq3_status())
    r.close()
    return out, st


def _oracle(text, ts, cols, keys):
    from oracle_engine import OracleEngine
    from siddhi_amd import compiler
    eng = OracleEngine(compiler.compile_app(text))
    eng.start()
    for b0 in range(0, len(ts), 4096):
        b1 = min(len(ts), b0 + 4096)
        eng.send(0, ts[b0:b1], [np.ascontiguousarray(c[b0:b1]) for c in cols], [None] * len(cols),
                 None if keys is None else np.ascontiguousarray(keys[b0:b1]), b0)
    out = eng.drain()
    eng.close()
    return out


@pytest.mark.parametrize("carry", ["aggp", "post", "aggc", "aggp-packed", "aggc-packed"])
@pytest.mark.parametrize("n,K", [(400_000, 2_000), (300_000, 20_000)])
def test_c2_aggregates_bucketed_vs_oracle(n, K, carry, monkeypatch):
    """default: the parallel fixed-point carry (k_bk_aggp, status 5); SH_BK_AGGP=0: the
    post-pass (status 1); SH_BK_AGGC=1: the sequential per-key carry (status 4); the
    carries into SH_OUT_PACKED rows too"""
    from siddhi_amd import synth
    packed = carry.endswith("-packed")
    carry = carry.replace("-packed", "")
    if carry == "aggc":
        monkeypatch.setenv("SH_BK_AGGC", "1")
    if carry == "post":
        monkeypatch.setenv("SH_BK_AGGP", "0")
    ts, k, p, v = synth.stock_stream(n, K, 100)
    (m, seq, vals), st = _run(C2_AGG, ts, k, [k, p, v], K, packed=packed)
    ref = _oracle(C2_AGG, ts, [k, p, v], k)
    assert st["bucket"] == 1 and st["agg"] == {"aggp": 5, "post": 1, "aggc": 4}[carry], st
    assert m == len(ref["seq"]) > 0
    assert np.array_equal(seq, ref["seq"].astype(np.int64))
    assert np.array_equal(vals, ref["values"])


def test_c1_aggregates_unpartitioned_window_vs_oracle():
    from siddhi_amd import synth
    ts, k, p, v = synth.stock_stream(100_000, 100, 1, config_index=1)
    (m, seq, vals), st = _run(C1_AGG, ts, np.zeros(len(ts), np.int32), [k, p, v], 1)
    ref = _oracle(C1_AGG, ts, [k, p, v], None)
    assert st["agg"] == 1, st
    assert m == len(ref["seq"]) > 0
    assert np.array_equal(seq, ref["seq"].astype(np.int64))
    assert np.array_equal(vals, ref["values"])


@pytest.mark.parametrize("post", [False, True])
def test_c3_aggregates_seq3_vs_oracle(post, monkeypatch):
    """sum / avg in the rise-and-fall kernel's lanes (agg status 3), or as the
    post-pass over the rows (SH_S3_AGG_POST, status 1)"""
    from siddhi_amd import synth
    if post:
        monkeypatch.setenv("SH_S3_AGG_POST", "1")
    ts, k, p, v = synth.stock_stream(300_000, 3_000, 1000, config_index=3)
    (m, seq, vals), st = _run(C3_AGG, ts, k, [k, p, v], 3_000)
    ref = _oracle(C3_AGG, ts, [k, p, v], k)
    assert st["seq3"] == 1 and st["agg"] == (1 if post else 3), st
    assert m == len(ref["seq"]) > 0
    assert np.array_equal(seq, ref["seq"].astype(np.int64))
    assert np.array_equal(vals, ref["values"])


def test_c5_aggregates_rule_set_vs_oracle():
    from siddhi_amd import synth
    rules = synth.c5_rules(100)
    text = synth.c5_query(rules).replace("e2.amount as amount", "sum(e2.amount) as total, avg(e1.amount) as a1")
    ts, card, amount, merchant = synth.txn_stream(200_000, 5_000, 100)
    (m, seq, vals, q), st = _run(text, ts, card, [card, amount, merchant], 5_000, with_query=True)
    ref = _oracle(text, ts, [card, amount, merchant], card)
    assert st["agg"] == 1, st
    assert m == len(ref["seq"]) > 0
    assert np.array_equal(seq, ref["seq"].astype(np.int64))
    assert np.array_equal(q, ref["query"])
    assert np.array_equal(vals, ref["values"])


@pytest.mark.parametrize("post", [False, True])
def test_rounding_additions_stay_exact(post, monkeypatch):
    """prices spanning 2^-60 .. 2^60: the double additions round. The parallel carry
    (k_bk_aggp) and the post-pass refuse, and the sequential carry adds in the
    reference's sequence instead (agg_status 4);
    with SH_BK_AGG_POST=1 the sequential engine's sums are returned (agg_status 2);
    both == the oracle's"""
    from siddhi_amd import synth
    if post:
        monkeypatch.setenv("SH_BK_AGG_POST", "1")
    ts, k, p, v = synth.stock_stream(200_000, 2_000, 100)
    p = p.copy()
    p[::7] *= np.float32(2.0 ** 60)
    p[3::11] *= np.float32(2.0 ** -60)
    (m, seq, vals), st = _run(C2_AGG, ts, k, [k, p, v], 2_000)
    ref = _oracle(C2_AGG, ts, [k, p, v], k)
    assert st["agg"] == (2 if post else 4), st
    assert m == len(ref["seq"]) > 0
    assert np.array_equal(seq, ref["seq"].astype(np.int64))
    assert np.array_equal(vals, ref["values"])


def test_c2_aggregates_full_size_vs_restatement():
    """BASELINE size (100M ticks, 10k symbols): the running sums of every key over
    the whole match stream equal per-key left-to-right double additions"""
    from agg_check import raw_bits, running
    from c2_check import c2_expected
    from siddhi_amd import synth
    ts, k, p, v = synth.stock_stream(100_000_000, 10_000, 100)
    (m, seq, vals), st = _run(C2_AGG, ts, k, [k, p, v], 10_000)
    assert st["bucket"] == 1 and st["agg"] == 5, st
    eseq, ev = c2_expected(ts, k, p, v)
    assert np.array_equal(seq, eseq)
    grp = k[eseq].astype(np.int64)
    p2 = ev[:, 2].astype(np.uint32).view(np.float32).astype(np.float64)
    p1 = ev[:, 1].astype(np.uint32).view(np.float32).astype(np.float64)
    assert np.array_equal(vals[:, 0], ev[:, 0])
    assert np.array_equal(vals[:, 1], raw_bits(running(grp, p2, "sum")))
    assert np.array_equal(vals[:, 2], raw_bits(running(grp, p1, "avg")))
    assert np.array_equal(vals[:, 3], running(grp, None, "count"))
    assert np.array_equal(vals[:, 4], running(grp, ev[:, 3], "sum"))


def test_aggp_refusal_sticks_to_the_handle():
    """double prices that are not whole units of 2^-24 (12.34): k_bk_aggp refuses the
    first batch, the refusal is kept, and both runs on the handle come out
    of the post-pass (agg_status 1) exactly as the oracle adds them, in packed rows"""
    import torch
    from siddhi_amd import compiler, synth
    from siddhi_amd.device_run import DeviceRunner, packed_to_raw
    text = C2_AGG.replace("price float", "price double")
    n, K = 200_000, 2_048
    ts, k, p, v = synth.stock_stream(n, K, 100)
    pd = np.round(p.astype(np.float64) + 0.003, 2)  # two decimals as doubles: 12.34 etc.
    ref = _oracle(text, ts, [k, pd, v], k)
    r = DeviceRunner(compiler.compile_app(text))
    dev = torch.device("cuda:0")
    tk = torch.from_numpy(k).to(dev)
    cols = [tk, torch.from_numpy(pd).to(dev), torch.from_numpy(v).to(dev)]
    offs, rb = r.packed_layout()
    for _ in range(2):
        m, rows = r.run(torch.from_numpy(ts).to(dev), tk, cols, K, packed=True)
        torch.cuda.synchronize()
        oseq, ovals = packed_to_raw(rows.cpu().numpy(), r.out_types, offs, rb)
        assert r.bucket_status() == 1 and r.agg_status() in (1, 2), (r.bucket_status(), r.agg_status())
        assert m == len(ref["seq"]) > 0
        assert np.array_equal(oseq.view(np.int64), ref["seq"].astype(np.int64))
        assert np.array_equal(ovals, ref["values"])
    r.close()
