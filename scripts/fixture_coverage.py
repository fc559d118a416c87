#!/usr/bin/env python3
"""Per-fixture coverage table of the reference's transcribed tests
(tests/golden/fixtures.json): oracle result, device-engine lowering (the general
engine's kernel logic, tests/nfa_host) and, when not lowered, the reason the
library gives (sh_compile -> SH_E_UNSUPPORTED). Writes profiles/fixture_coverage.txt."""
import collections
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "tests"))
sys.path.insert(0, os.path.join(HERE, ".."))
from fixture_runner import Unsupported, check_fixture, load_fixtures, run_fixture  # noqa: E402
from nfa_host_engine import NfaHostEngine, NfaUnsupported  # noqa: E402
from oracle_engine import OracleEngine  # noqa: E402

rows, why = [], collections.defaultdict(list)
for fx in load_fixtures():
    try:
        ref = run_fixture(fx, OracleEngine)
        o = "pass" if not check_fixture(fx, ref) else "FAIL"
    except Unsupported as e:
        rows.append((fx["id"], "outside subset", "-", str(e)))
        why["outside the hot-path subset: " + str(e)].append(fx["id"])
        continue
    try:
        run_fixture(fx, NfaHostEngine)
        d = "lowered"
        r = ""
    except NfaUnsupported as e:
        d = "not lowered"
        r = str(e)
        why["device: " + r].append(fx["id"])
    rows.append((fx["id"], o, d, r))
out = os.path.join(HERE, "..", "profiles", "fixture_coverage.txt")
with open(out, "w") as f:
    n = len(rows)
    f.write(f"{n} fixtures; oracle pass {sum(r[1] == 'pass' for r in rows)}; "
            f"device lowered {sum(r[2] == 'lowered' for r in rows)}\n\n")
    for reason, ids in sorted(why.items(), key=lambda kv: -len(kv[1])):
        f.write(f"[{len(ids)}] {reason}\n")
        for i in ids:
            f.write(f"    {i}\n")
print(open(out).read()[:3000])
