"""`having` on pattern / sequence queries (the part of device
selection beyond pass-through that the reference's pattern tests use).

QuerySelector runs the having condition on each selected event after its output
attributes are populated (QuerySelector.java:161-205 drops the events that fail;
processInBatchNoGroupBy :271-313 keeps the last event that passes, with aggregators);
a bare name in the condition is first an output attribute (HAVING_STATE,
ExpressionParser.java:1308-1318). Pinned by CountPatternTestCase.testQuery14 and
testQuery26 (tests/golden/fixtures.json, run by test_oracle_golden /
test_nfa_engine_cpu / test_gpu_parity); here randomized apps hold the general engine's
kernel logic (compiled for the CPU) and the device to the oracle."""
import random

import pytest

from fixture_runner import Unsupported
from nfa_cases import nfa_case, run_case, same_rows
from nfa_host_engine import NfaHostEngine, NfaUnsupported
from oracle_engine import OracleEngine
from siddhi_amd import SiddhiAppCreationException, compiler

HAVING = ["c0 is null", "not (c0 is null)", "c1 != 'K0'", "s > 20.0", "n > 1", "c0 > 3 or c1 == 'K1'",
          "not (n > 2)", "s is null", "instanceOfLong(c2)", "instanceOfFloat(c2) or n == 1"]


def having_case(seed):
    rng = random.Random(9000 + seed)
    app, actions = nfa_case(rng)
    if " select " not in app:
        return None
    h = rng.choice(HAVING)
    # every generated select list starts with c0, c1, c2 and may add s / n (aggregators)
    if ("s" in h.split() or "s " in h) and " as s" not in app:
        h = "c0 is null"
    if ("n" in h.split()) and " as n" not in app:
        h = "not (c0 is null)"
    app = app.replace(" insert into Out;", f" having {h} insert into Out;")
    return app, actions


def _apps(n):
    out = []
    for seed in range(n):
        c = having_case(seed)
        if c is not None:
            out.append((seed, c))
    return out


def test_parse_and_lower_having():
    app = ("define stream S (sym string, price float); "
           "from every e1=S -> e2=S[price > e1.price] select e1.price as p1, e2.price as p2 "
           "having p2 > p1 * 2.0f and e1.sym == 'A' insert into Out;")
    c = compiler.compile_app(app)
    q = c.queries[0]
    assert q.having >= 0
    ops = [x["op"] for x in q.exprs]
    assert 20 in ops  # output-attribute variables (HAVING_STATE)
    d = c.descriptor()
    assert d.queries[0].having == q.having
    # group by + having lowers too (tests/test_group_by.py)
    assert compiler.compile_app(app.replace("having", "group by e1.sym having")).descriptor().queries[0].n_group == 1


@pytest.mark.parametrize("seed,case", _apps(120), ids=lambda x: str(x) if isinstance(x, int) else "")
def test_having_kernel_logic_vs_oracle(seed, case):
    app, actions = case
    try:
        ref = run_case(OracleEngine, app, actions)
    except (SiddhiAppCreationException, Unsupported, RuntimeError) as e:
        pytest.skip(f"outside the subset: {e}")
    try:
        got = run_case(NfaHostEngine, app, actions)
    except NfaUnsupported as e:
        pytest.skip(f"not lowered: {e}")
    assert same_rows(got, ref), app


@pytest.mark.gpu
@pytest.mark.parametrize("seed,case", _apps(60), ids=lambda x: str(x) if isinstance(x, int) else "")
def test_having_gpu_vs_oracle(seed, case):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from siddhi_amd._native import HipEngine, HipError

    def hip(c):
        try:
            return HipEngine(c)
        except HipError as e:
            if e.code == -4:
                raise Unsupported(str(e))
            raise

    app, actions = case
    try:
        ref = run_case(OracleEngine, app, actions)
        got = run_case(hip, app, actions)
    except (SiddhiAppCreationException, Unsupported, RuntimeError) as e:
        pytest.skip(f"outside the subset: {e}")
    assert same_rows(got, ref), app
