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
import re

import pytest

from fixture_runner import Unsupported
from nfa_cases import nfa_case, run_case, same_rows
from nfa_host_engine import NfaHostEngine, NfaUnsupported
from oracle_engine import OracleEngine
from siddhi_amd import SiddhiAppCreationException, compiler

_ATTR_T = {"price": "f", "x": "i", "sym": "s", "volume": "i"}


def _outputs(select):
    """output attribute -> 'f' / 'i' / 's' (float-like, int-like, string) of a
    generated select list (c0.., s = sum(...) double, n = count() long)"""
    outs = {}
    for expr, name in re.findall(r"([^,]+?) as (\w+)", select):
        expr = expr.strip()
        if name == "s":
            outs[name] = "f"
        elif name == "n":
            outs[name] = "i"
        else:
            a = expr.rsplit(".", 1)[-1]
            outs[name] = _ATTR_T.get(a, "i")
    return outs


def _cond(rng, outs):
    c = rng.choice(sorted(outs))
    t = outs[c]
    forms = [f"{c} is null", f"not ({c} is null)", f"instanceOfLong({c})", f"instanceOfFloat({c})"]
    forms += {"f": [f"{c} > 20.0", f"{c} < 15.5", f"not ({c} >= 12.0)"],
              "i": [f"{c} > 3", f"{c} != 2", f"not ({c} > 1)"],
              "s": [f"{c} != 'K0'", f"{c} == 'K1'"]}[t]
    return rng.choice(forms)


def having_case(seed):
    """a random app of tests/nfa_cases.py with a `having` over the outputs its
    first query's select list defines, each compared with a constant of its type"""
    rng = random.Random(9000 + seed)
    app, actions = nfa_case(rng)
    m = re.search(r" select (.*?) insert into Out;", app)
    if m is None:
        return None
    outs = _outputs(m.group(1))
    if not outs:
        return None
    h = _cond(rng, outs)
    if rng.random() < 0.4:
        h = f"{h} {rng.choice(['and', 'or'])} {_cond(rng, outs)}"
    app = app.replace(" insert into Out;", f" having {h} insert into Out;", 1)
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
