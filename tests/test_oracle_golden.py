"""Pin the CPU oracle against the reference's own known-answer tests.

Each fixture in tests/golden/fixtures.json was transcribed (by
tests/golden/extract_fixtures.py) from a TestNG @Test of the reference; its
`source` field names the file:line. The oracle must reproduce the asserted
event count and every asserted data row.
"""
import pytest

from fixture_runner import Unsupported, check_fixture, load_fixtures, run_fixture
from oracle_engine import OracleEngine

FIXTURES = load_fixtures()

# Known oracle gaps (tracked in DESIGN.md "parity status"):
#  - AbsentLogicalPreStateProcessor (`A and not B for T` …) is not restated yet
#  - wall-clock `every not X for T` timer re-arming is modelled in event time; the
#    reference's ScheduledExecutorService timing differs for these tests
KNOWN_GAPS = {
    "AbsentPatternTestCase.testQueryAbsent6",
    "EveryAbsentPatternTestCase.testQueryAbsent1",
    "EveryAbsentPatternTestCase.testQueryAbsent7",
    "EveryAbsentPatternTestCase.testQueryAbsent13",
    "EveryAbsentPatternTestCase.testQueryAbsent14",
    "EveryAbsentPatternTestCase.testQueryAbsent22",
    "AbsentWithEveryPatternTestCase.testQuery8",
}


@pytest.mark.parametrize("fx", FIXTURES, ids=[f["id"] for f in FIXTURES])
def test_oracle_matches_reference_fixture(fx):
    if fx["id"] in KNOWN_GAPS:
        pytest.xfail("known oracle gap (absent timers in wall-clock mode)")
    try:
        got = run_fixture(fx, OracleEngine)
    except Unsupported as e:
        pytest.skip(f"outside the hot-path subset: {e}")
    except RuntimeError as e:
        if "not restated yet" in str(e):
            pytest.xfail(str(e))
        raise
    errs = check_fixture(fx, got)
    assert not errs, f"{fx['source']}: {errs}"
