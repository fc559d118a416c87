"""The vectorised C3 restatement (tests/c3_check.py) agrees with the oracle,
including price ties and a key with a single event."""
import numpy as np
import pytest

from c3_check import c3_expected
from oracle_engine import run_stock_oracle
from siddhi_amd import compiler, synth


@pytest.mark.parametrize("n,keys,rate,ties", [(40000, 3, 10, False), (40000, 50, 10, True), (60000, 2000, 100, False),
                                              (20000, 400, 1000, True)])
def test_c3_vectorised_matches_oracle(n, keys, rate, ties):
    ts, k, p, v = synth.stock_stream(n, keys, rate, config_index=3)
    if ties:
        p = (np.random.default_rng(n).integers(0, 6, n)).astype(np.float32)
    seq, ots, vals, nulls = run_stock_oracle(compiler.compile_app(synth.C3_QUERY), ts, k, p, v)
    eseq, evals = c3_expected(ts, k, p)
    assert len(seq) == len(eseq) > 0
    assert np.array_equal(seq.astype(np.int64), eseq)
    assert np.array_equal(vals, evals)
    assert np.array_equal(ots, ts[eseq])
