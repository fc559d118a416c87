"""The vectorised C5 restatement (tests/c5_check.py) agrees with the oracle, and the
C-ABI lowers C5-shaped rule sets (no GPU needed)."""
import ctypes as C

import numpy as np
import pytest

from c5_check import c5_expected
from rules_cases import CASES, card_strings, case_data, oracle_run
from siddhi_amd import abi, build, compiler, synth


@pytest.mark.parametrize("ci", [i for i, c in enumerate(CASES) if c[6]])
def test_c5_vectorised_matches_oracle(ci):
    case = CASES[ci]
    n, cards, nr, rate, batch, merchants, partitioned, free, seed = case
    text, rules, (ts, card, amount, merchant) = case_data(case)
    out = oracle_run(text, cards, ts, card, amount, merchant, batch)
    eseq, erule, evals = c5_expected(ts, card, amount, merchant, rules, within_ms=1, batch=batch, free=free)
    assert len(out["seq"]) == len(eseq) > 0
    assert np.array_equal(out["seq"].astype(np.int64), eseq)
    assert np.array_equal(out["query"], erule)
    assert np.array_equal(out["values"][:, :2], evals)


@pytest.fixture(scope="module")
def lib():
    return abi.bind_product(C.CDLL(build.build()))


@pytest.mark.parametrize("n_rules", [2, 40, 1000])
def test_rule_sets_lower(lib, n_rules):
    text = synth.c5_query(synth.c5_rules(n_rules), free=(1,) if n_rules > 1 else ())
    ca = compiler.compile_app(text, card_strings(4))
    d = ca.descriptor()
    h = C.c_void_p()
    rc = lib.sh_compile(C.byref(d), C.byref(h))
    assert rc == abi.SH_OK, lib.sh_last_error(h)
    lib.sh_destroy(h)
