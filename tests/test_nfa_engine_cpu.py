"""The general engine's per-key kernel logic (siddhi_amd/csrc/sh_nfa.h, run on the
GPU by k_nfa) compiled for the CPU (tests/nfa_host) and diffed against the oracle:
every golden fixture of the reference's test suite and randomized apps with
count / logical / absent states, sequences, `every`, `within`, partitions and
multi-query partitions. Bit-exact: same events, same order, same values."""
import random

import pytest

from fixture_runner import Unsupported, check_fixture, load_fixtures, run_fixture
from nfa_cases import nfa_case, run_case, same_rows
from nfa_host_engine import NfaHostEngine, NfaUnsupported
from oracle_engine import OracleEngine
from test_oracle_golden import KNOWN_GAPS

FIXTURES = load_fixtures()


@pytest.mark.parametrize("fx", FIXTURES, ids=[f["id"] for f in FIXTURES])
def test_fixture_kernel_logic_vs_oracle(fx):
    try:
        ref = run_fixture(fx, OracleEngine)
    except Unsupported as e:
        pytest.skip(f"outside the hot-path subset: {e}")
    except RuntimeError as e:
        pytest.skip(f"oracle: {e}")
    try:
        got = run_fixture(fx, NfaHostEngine)
    except NfaUnsupported as e:
        pytest.skip(f"not lowered: {e}")
    assert [(e.timestamp, e.data) for e in got] == [(e.timestamp, e.data) for e in ref]
    if fx["id"] not in KNOWN_GAPS:
        assert not check_fixture(fx, got)


@pytest.mark.parametrize("seed", range(150))
def test_random_apps_kernel_logic_vs_oracle(seed):
    rng = random.Random(seed)
    app, actions = nfa_case(rng)
    try:
        ref = run_case(OracleEngine, app, actions)
    except Exception as e:  # generator produced something outside the subset
        pytest.skip(str(e)[:100])
    try:
        got = run_case(NfaHostEngine, app, actions)
    except NfaUnsupported as e:
        pytest.skip(f"not lowered: {e}")
    assert same_rows(got, ref), app
