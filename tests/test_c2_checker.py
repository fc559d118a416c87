"""The vectorised C2 restatement (tests/c2_check.py) agrees with the oracle."""
import numpy as np
import pytest

from c2_check import c2_expected
from oracle_engine import run_stock_oracle
from siddhi_amd import compiler, synth


@pytest.mark.parametrize("n,keys,rate", [(60000, 1000, 100), (20000, 50, 5), (30000, 3, 1)])
def test_c2_vectorised_matches_oracle(n, keys, rate):
    ts, k, p, v = synth.stock_stream(n, keys, rate)
    ca = compiler.compile_app(synth.C2_QUERY)
    seq, ots, vals, nulls = run_stock_oracle(ca, ts, k, p, v)
    eseq, evals = c2_expected(ts, k, p, v)
    assert len(seq) == len(eseq) > 0
    assert np.array_equal(seq.astype(np.int64), eseq)
    assert np.array_equal(vals, evals)
    assert not nulls.any()
    assert np.array_equal(ots, ts[eseq])


@pytest.mark.parametrize("n,keys,rate", [(20000, 100, 1), (8000, 7, 3)])
def test_c1_unpartitioned_oracle_equals_c2_restatement(n, keys, rate):
    """C1 (BASELINE.json configs[0]: the same pattern without `partition with`):
    the unpartitioned pending list holds every symbol's partials, but
    `symbol == e1.symbol` confines each consumer to its own symbol's partials in
    arrival order, so the ordered output equals the per-symbol restatement"""
    from oracle_engine import run_columns_oracle
    ts, k, p, v = synth.stock_stream(n, keys, rate, config_index=1)
    ca = compiler.compile_app(synth.C1_QUERY)
    seq, ots, vals, nulls = run_columns_oracle(ca, ts, [k, p, v], None)
    eseq, evals = c2_expected(ts, k, p, v)
    assert len(seq) == len(eseq) > 0
    assert np.array_equal(seq.astype(np.int64), eseq)
    assert np.array_equal(vals, evals)
