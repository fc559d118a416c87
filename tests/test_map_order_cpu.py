"""The playback scheduler's one-state-per-due-time pick follows java.util.HashMap
iteration order over the partition keys' toString() (Scheduler.java:75-87,
PartitionStateHolder.java:36). Checked on the CPU:
  * the product's order model (siddhi_amd/csrc/sh_jmap.h) against the oracle's
    restatement of OpenJDK 8 HashMap (oracle/jhashmap.h) on random
    computeIfAbsent / remove sequences, including fully colliding String keys
    that treeify bins (tests/jmap_check);
  * the general engine's kernel logic driven like sh_host.cpp drives it
    (tests/nfa_host, ranks from the model) against the oracle on C4 streams where
    >= 1,000 users share due milliseconds, with plain and colliding user names.
Parity unpinned by reference fixtures: no siddhi-core test asserts a
cross-key tie."""
import os
import subprocess

import pytest

from c4_cases import CollidingNames, run_c4, same_output, ties
from nfa_host_engine import NfaHostEngine
from oracle_engine import OracleEngine
from siddhi_amd import compiler, javastr, synth

HERE = os.path.dirname(os.path.abspath(__file__))


def test_order_model_matches_hashmap_restatement():
    d = os.path.join(HERE, "jmap_check")
    subprocess.run(["make", "-s", "-C", d], check=True)
    r = subprocess.run([os.path.join(d, "jmap_check"), "30"], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr


def test_java_string_hash_known_values():
    assert javastr.java_string_hash("") == 0
    assert javastr.java_string_hash("Aa") == javastr.java_string_hash("BB") == 2112
    assert javastr.java_string_hash("hello") == 99162322
    assert javastr.java_string_hash("polygenelubricants") == -2147483648


@pytest.mark.parametrize("users,seconds", [(5_000, 5), (2_000, 10)])
def test_c4_ties_follow_map_order(users, seconds):
    c = compiler.compile_app(synth.C4_QUERY)
    blocks = synth.c4_stream(users, seconds=seconds)
    assert ties(blocks) > 100
    ref = run_c4(OracleEngine(c), blocks)
    got = run_c4(NfaHostEngine(c), blocks)
    assert len(ref["seq"]) > 1000
    assert same_output(got, ref)


def test_c4_colliding_names_follow_map_order():
    n = 2000
    c = compiler.compile_app(synth.C4_QUERY)
    blocks = synth.c4_stream(n, seconds=10)
    ref = run_c4(CollidingNames(OracleEngine(c), n), blocks)
    got = run_c4(CollidingNames(NfaHostEngine(c), n), blocks)
    assert len(ref["seq"]) > 500
    assert same_output(got, ref)


def test_registration_order_is_not_map_order():
    """sanity: insertion (registration) order and HashMap order disagree on this
    stream, so the tests above are sensitive to the tie rule"""
    import ctypes as C  # noqa: F401
    c = compiler.compile_app(synth.C4_QUERY)
    blocks = synth.c4_stream(5_000, seconds=5)
    ref = run_c4(OracleEngine(c), blocks)
    os.environ["SH_NFAH_STAMP_ORDER"] = "1"
    try:
        got = run_c4(NfaHostEngine(c), blocks)
    finally:
        del os.environ["SH_NFAH_STAMP_ORDER"]
    assert not same_output(got, ref)
