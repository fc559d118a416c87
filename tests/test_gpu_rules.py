"""GPU parity of the batch-compiled rule engine (sh_rules.hip, config C5) through
sh_run_device, bit-exact against the CPU oracle: same rows, same order (same-key
run, query, consuming event, opening event), same query ids and values. At C5
size the device output is checked against the vectorised restatement
(tests/c5_check.py, itself checked against the oracle on CPU)."""
import numpy as np
import pytest

from c5_check import c5_expected
from rules_cases import CASES, card_strings, case_data, oracle_run
from siddhi_amd import compiler, synth

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _device():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _device_run(text, n_cards, ts, card, amount, merchant, batch, partitioned=True, status=None):
    import torch
    from siddhi_amd.device_run import DeviceRunner
    runner = DeviceRunner(compiler.compile_app(text, card_strings(n_cards)))
    dev = torch.device("cuda:0")
    cols = [torch.from_numpy(c).to(dev) for c in (card, amount, merchant)]
    m, seq, vals, q = runner.run(torch.from_numpy(ts).to(dev), cols[0], cols, n_cards if partitioned else 1,
                                 batch_events=batch, with_query=True)
    torch.cuda.synchronize()
    res = (seq.cpu().numpy(), vals.cpu().numpy(), q.cpu().numpy())
    if status is not None:
        status.append(runner.rules_status())
    runner.close()
    return res


@pytest.mark.parametrize("engine", ["sparse", "segment", "general"])
@pytest.mark.parametrize("ci", range(len(CASES)))
def test_rule_sets_vs_oracle(ci, engine, monkeypatch):
    """sparse: the partials found in arrival order (partitioned sets; small runs
    always fit its buffers), segment: the key-segment scan (SH_RULES_SPARSE=0),
    general: the general NFA engine"""
    case = CASES[ci]
    n, cards, nr, rate, batch, merchants, partitioned, free, seed = case
    if engine == "general":
        if nr > 16:
            pytest.skip("the general engine's query table holds 16 queries")
        monkeypatch.setenv("SH_DISABLE_RULES", "1")
    if engine == "segment":
        monkeypatch.setenv("SH_RULES_SPARSE", "0")
    text, rules, (ts, card, amount, merchant) = case_data(case)
    ref = oracle_run(text, cards, ts, card, amount, merchant, batch, partitioned)
    st = []
    seq, vals, q = _device_run(text, cards, ts, card, amount, merchant, batch, partitioned, status=st)
    if engine == "segment" or (engine == "sparse" and not partitioned):
        assert st == [0]
    assert len(seq) == len(ref["seq"]) > 0
    assert np.array_equal(seq, ref["seq"].astype(np.int64))
    assert np.array_equal(q, ref["query"])
    assert np.array_equal(vals[:, :2], ref["values"][:, :2])


# selective start filters (the C5 distributions at small size): the sparse path
SPARSE_CASES = [
    # n, cards, rules, rate, batch, merchants, free, seed, amount range, factor range of the rules
    (60_000, 300, 100, 2, 4096, 50, (), 31, (100.0, 400.0), (1.05, 1.8)),
    (40_000, 2000, 40, 50, 997, 8, (0, 3), 32, (150.0, 600.0), (1.05, 1.8)),  # free rules (no merchant conjunct)
    (30_000, 20, 30, 5, 64, 6, (), 33, (400.0, 1500.0), (0.3, 1.0)),          # 20 cards: long same-card runs
]


@pytest.mark.parametrize("ci", range(len(SPARSE_CASES)))
def test_sparse_partials_vs_oracle(ci):
    n, cards, nr, rate, batch, merchants, free, seed, amt, fac = SPARSE_CASES[ci]
    ts, card, amount, merchant = synth.txn_stream(n, cards, rate, n_merchants=merchants, seed=seed)
    rules = synth.c5_rules(nr, seed=seed, amount=amt, merchants=merchants, factor=fac, within=(1, 40))
    text = synth.c5_query(rules, unit="milliseconds", free=free)
    ref = oracle_run(text, cards, ts, card, amount, merchant, batch, True)
    st = []
    seq, vals, q = _device_run(text, cards, ts, card, amount, merchant, batch, True, status=st)
    assert st == [1]
    assert len(seq) == len(ref["seq"]) > 0
    assert np.array_equal(seq, ref["seq"].astype(np.int64))
    assert np.array_equal(q, ref["query"])
    assert np.array_equal(vals[:, :2], ref["values"][:, :2])


def test_sparse_hot_card_vs_oracle():
    """a skewed stream: half the transactions on one card and rules whose f2 factor
    (2-4) lets partials pile up until a large amount takes many of one rule at once
    (up to 17 per (event, rule) on this stream, 739 such runs), so that card's
    partial list is long -- k_sparse_take's per-wave pair queue and k_rules_ties'
    long runs (shell sort) against the oracle"""
    n, cards, nr, seed = 24_000, 400, 12, 35
    ts, card, amount, merchant = synth.txn_stream(n, cards, 4, n_merchants=4, seed=seed)
    card = card.copy()
    card[::2] = 0
    rules = synth.c5_rules(nr, seed=seed, amount=(60.0, 400.0), merchants=4, factor=(2.0, 4.0), within=(100, 400))
    text = synth.c5_query(rules, unit="milliseconds")
    ref = oracle_run(text, cards, ts, card, amount, merchant, 4096, True)
    st = []
    seq, vals, q = _device_run(text, cards, ts, card, amount, merchant, 4096, True, status=st)
    assert st == [1]
    assert len(seq) == len(ref["seq"]) > 0
    assert np.array_equal(seq, ref["seq"].astype(np.int64))
    assert np.array_equal(q, ref["query"])
    assert np.array_equal(vals[:, :2], ref["values"][:, :2])


@pytest.mark.parametrize("n,cards,sparse", [(20_000_000, 200_000, "1"), (20_000_000, 200_000, "0"),
                                            (100_000_000, 1_000_000, "1")], ids=["20M", "20M-segment", "100M"])
def test_c5_large_vs_vectorised_restatement(n, cards, sparse, monkeypatch):
    """1,000 rules (BASELINE distributions): 20M card transactions over 200k cards
    (sparse-partial and key-segment paths), and the full SURVEY 8d size, 100M
    transactions over 1M cards."""
    monkeypatch.setenv("SH_RULES_SPARSE", sparse)
    ts, card, amount, merchant = synth.txn_stream(n, cards, 100)
    rules = synth.c5_rules()
    text = synth.c5_query(rules)
    st = []
    seq, vals, q = _device_run(text, cards, ts, card, amount, merchant, 4096, status=st)
    assert st == [int(sparse)]
    eseq, erule, evals = c5_expected(ts, card, amount, merchant, rules)
    assert len(seq) == len(eseq) > 0
    assert np.array_equal(seq, eseq)
    assert np.array_equal(q, erule)
    assert np.array_equal(vals[:, :2], evals)


def test_sparse_falls_back_on_decreasing_timestamps():
    """a run whose timestamps decrease somewhere (but not inside a key) leaves the
    sparse path; the key-segment scan gives the oracle's rows"""
    case = CASES[0]
    n, cards, nr, rate, batch, merchants, partitioned, free, seed = case
    text, rules, (ts, card, amount, merchant) = case_data(case)
    # swap two adjacent events of different cards whose times differ
    i = next(k for k in range(1, n) if card[k] != card[k - 1] and ts[k] > ts[k - 1])
    for a in (ts, card, amount, merchant):
        a[[i - 1, i]] = a[[i, i - 1]]
    ref = oracle_run(text, cards, ts, card, amount, merchant, batch, partitioned)
    st = []
    seq, vals, q = _device_run(text, cards, ts, card, amount, merchant, batch, partitioned, status=st)
    assert st == [0]
    assert np.array_equal(seq, ref["seq"].astype(np.int64))
    assert np.array_equal(q, ref["query"])
    assert np.array_equal(vals[:, :2], ref["values"][:, :2])
