"""GPU parity of the general NFA engine (k_nfa_run / k_nfa_timer, sh_nfa.hip)
through the C-ABI: randomized pattern / sequence apps with Count, Logical and
Absent states, `every`, `within`, partitions and multi-query partitions against
the oracle, bit-exact (same events, same order, same values). A second pass
starts every capacity at 2 so that arena / list / queue growth with replay runs."""
import os
import random

import pytest

from nfa_cases import nfa_case, run_case, same_rows
from oracle_engine import OracleEngine

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _device():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def hip_factory(compiled):
    from siddhi_amd._native import HipEngine, HipError
    try:
        return HipEngine(compiled)
    except HipError as e:
        if e.code == -4:
            raise _Unlowered(str(e))
        raise


class _Unlowered(Exception):
    pass


def _check(seed):
    rng = random.Random(seed)
    app, actions = nfa_case(rng)
    try:
        ref = run_case(OracleEngine, app, actions)
    except Exception as e:
        pytest.skip(str(e)[:100])
    try:
        got = run_case(hip_factory, app, actions)
    except _Unlowered as e:
        pytest.skip(f"not lowered: {e}")
    assert same_rows(got, ref), app


@pytest.mark.parametrize("seed", range(150))
def test_random_apps_on_gpu_vs_oracle(seed):
    _check(seed)


@pytest.mark.parametrize("seed", range(150, 190))
def test_random_apps_on_gpu_with_growth(seed, monkeypatch):
    monkeypatch.setenv("SH_NFA_CAPS", "2,2,2,2,2")
    _check(seed)
