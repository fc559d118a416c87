"""C4 on the CPU: the general engine's kernel logic (tests/nfa_host) against the
oracle on a small login-session stream, and the generator's invariants."""
import numpy as np

from c4_cases import run_c4, same_output
from nfa_host_engine import NfaHostEngine
from oracle_engine import OracleEngine
from siddhi_amd import compiler, synth


def test_c4_stream_shape():
    blocks = synth.c4_stream(3000, seconds=5)
    last = None
    for st, ts, cols, keys in blocks:
        assert st in (0, 1, 2) and len(ts) == len(keys) > 0
        assert np.all(ts == ts[0])
        assert last is None or ts[0] > last
        last = ts[0]
    n = sum(len(b[1]) for b in blocks)
    assert 2 * 3000 <= n <= 3 * 3000


def test_c4_kernel_logic_vs_oracle():
    c = compiler.compile_app(synth.C4_QUERY)
    blocks = synth.c4_stream(1000, seconds=5)
    ref = run_c4(OracleEngine(c), blocks)
    got = run_c4(NfaHostEngine(c), blocks)
    assert len(ref["seq"]) > 100
    assert same_output(got, ref)
