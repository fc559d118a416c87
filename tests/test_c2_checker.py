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
