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

KNOWN_GAPS = set()


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
