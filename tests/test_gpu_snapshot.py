"""Snapshot / restore of the device matcher state: sh_snapshot /
sh_restore through SiddhiAppRuntime.snapshot / restore / persist / restoreLastRevision.

Pinned by the reference's own persistence test of a pattern
(managment/PersistenceTestCase.java:146-231, persistenceTest2: a count pattern
persisted mid-match, the app restarted and restored, one output row asserted), and by
construction elsewhere: a stream cut anywhere, snapshotted, and continued on a fresh
runtime restored from the image must produce exactly the rows of the uninterrupted
run (general engine with absent timers and the HashMap-order scheduler models, the
chain / window engines, C4 whole streams)."""
import random
import struct

import numpy as np
import pytest

from c4_cases import run_c4, same_output
from fixture_runner import Unsupported
from nfa_cases import nfa_case, same_rows
from window_cases import window_case
from siddhi_amd import InMemoryPersistenceStore, SiddhiAppCreationException, SiddhiManager, synth
from siddhi_amd import compiler

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _device():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def hip(compiled):
    from siddhi_amd._native import HipEngine, HipError
    try:
        return HipEngine(compiled)
    except HipError as e:
        if e.code == -4:
            raise Unsupported(str(e))
        raise


PERSIST_APP = ("@app:name('Test') "
               "define stream Stream1 (symbol string, price float, volume int); "
               "define stream Stream2 (symbol string, price float, volume int); "
               "@info(name = 'query1') "
               "from e1=Stream1[price>20] <2:5> -> e2=Stream2[price>20] "
               "select e1[0].price as price1_0, e1[1].price as price1_1, e1[2].price as price1_2, "
               "   e1[3].price as price1_3, e2.price as price2 "
               "insert into OutputStream ;")


def _f32(x):
    return struct.unpack("<f", struct.pack("<f", x))[0]


def test_reference_persistence_test2_pattern_count():
    """PersistenceTestCase.java:146-231: three Stream1 events, persist, restart,
    restoreLastRevision, then Stream2 / Stream1 / Stream2 -> exactly one row
    [25.6f, 47.6f, null, null, 45.7f]."""
    store = InMemoryPersistenceStore()
    mgr = SiddhiManager(engine_factory=hip)
    mgr.setPersistenceStore(store)
    got = []

    def cb(ts, ins, rem):
        got.extend(e.data for e in (ins or []))

    rt = mgr.createSiddhiAppRuntime(PERSIST_APP)
    rt.addCallback("query1", cb)
    s1 = rt.getInputHandler("Stream1")
    rt.start()
    s1.send(["WSO2", 25.6, 100])
    rt.sleep(100)
    s1.send(["GOOG", 47.6, 100])
    rt.sleep(100)
    s1.send(["GOOG", 13.7, 100])
    rt.sleep(100)
    assert got == []
    rt.sleep(500)
    rt.persist()
    rt.sleep(500)
    rt.shutdown()

    rt = mgr.createSiddhiAppRuntime(PERSIST_APP)
    rt.addCallback("query1", cb)
    s1 = rt.getInputHandler("Stream1")
    s2 = rt.getInputHandler("Stream2")
    rt.start()
    assert rt.restoreLastRevision() is not None
    s2.send(["IBM", 45.7, 100])
    rt.sleep(500)
    s1.send(["GOOG", 47.8, 100])
    rt.sleep(500)
    s2.send(["IBM", 55.7, 100])
    rt.sleep(500)
    rt.shutdown()
    assert got == [[_f32(25.6), _f32(47.6), None, None, _f32(45.7)]]


def _run_split(app, actions, cut, factory=hip):
    """actions[:cut] on one runtime, snapshot, actions[cut:] on a fresh restored one"""
    got = []

    def attach(rt):
        for name in ("query1", "query2", "query3"):
            try:
                rt.addCallback(name, (lambda nm: lambda ts, i, r: got.extend((nm, e.timestamp, e.data)
                                                                              for e in (i or [])))(name))
            except Exception:
                pass

    def play(rt, acts):
        hs = {}
        for a in acts:
            if a[0] == "send":
                h = hs.setdefault(a[1], rt.getInputHandler(a[1]))
                h.send_batch([t for t, _ in a[2]], [d for _, d in a[2]])
            else:
                rt.advance_time(a[1])

    mgr = SiddhiManager(engine_factory=factory)
    rt = mgr.createSiddhiAppRuntime(app)
    attach(rt)
    rt.start()
    play(rt, actions[:cut])
    image = rt.snapshot()
    rt.shutdown()
    rt = mgr.createSiddhiAppRuntime(app)
    attach(rt)
    rt.start()
    rt.restore(image)
    play(rt, actions[cut:])
    rt.shutdown()
    return got


def _full(app, actions):
    return _run_split(app, actions, len(actions))


@pytest.mark.parametrize("seed", range(40))
def test_random_apps_continue_exactly_after_restore(seed):
    rng = random.Random(4000 + seed)
    app, actions = nfa_case(rng)
    try:
        ref = _full(app, actions)
    except (Unsupported, SiddhiAppCreationException):
        pytest.skip("invalid app or a shape not lowered to the device")
    for cut in sorted({1, len(actions) // 3, len(actions) // 2, (2 * len(actions)) // 3}):
        got = _run_split(app, actions, cut)
        assert same_rows(got, ref), (app, cut)


@pytest.mark.parametrize("seed", range(16))
def test_rate_limited_apps_continue_exactly_after_restore(seed):
    """the output rate limiter's per-partition counter (FirstPer / LastPerEventOutputRateLimiter
    RateLimiterState.snapshot) travels in the key blocks of the image"""
    import re
    rng = random.Random(4600 + seed)
    app, actions = nfa_case(rng)
    app = re.sub(r" insert into Out;", lambda m: f" output {rng.choice(['first', 'last'])} every "
                 f"{rng.choice([2, 3, 4])} events insert into Out;", app)
    try:
        ref = _full(app, actions)
    except (Unsupported, SiddhiAppCreationException):
        pytest.skip("invalid app or a shape not lowered to the device")
    for cut in sorted({1, len(actions) // 3, len(actions) // 2, (2 * len(actions)) // 3}):
        got = _run_split(app, actions, cut)
        assert same_rows(got, ref), (app, cut)


@pytest.mark.parametrize("seed", range(8))
def test_window_apps_continue_exactly_after_restore(seed):
    """streaming chain / window engine (mode 0): partial lists in the key blocks"""
    rng = random.Random(8100 + seed)
    app, _ = window_case(rng)
    syms = ["A", "B", "C"]
    t, actions = 1000, []
    for _ in range(60):
        b = []
        for _ in range(rng.randint(1, 9)):
            t += rng.choice([0, 1, 2, 7])
            b.append((t, [rng.choice(syms), float(rng.randint(0, 30)), rng.randint(0, 9), rng.randint(-3, 20)]))
        actions.append(("send", "S", b))
    ref = _full(app, actions)
    got = _run_split(app, actions, 25)
    assert same_rows(got, ref), app


@pytest.mark.parametrize("drain_first", [True, False])
def test_c4_stream_continues_exactly_after_restore(drain_first):
    """playback absence timers + HashMap-order scheduler models, 20k users; the
    snapshot taken straight after a send() (no drain: the pending launch, its
    scheduler history and its undelivered rows go into the image) or after a drain"""
    from siddhi_amd._native import HipEngine
    blocks = synth.c4_stream(20_000, seconds=20, seed=synth.SEED + 44)
    c = compiler.compile_app(synth.C4_QUERY)
    ref = run_c4(HipEngine(c), blocks)

    class Split:
        """engine that is snapshotted and replaced by a restored one after `cut` sends"""

        def __init__(self, cut):
            self.eng, self.cut, self.n = HipEngine(c), cut, 0
            self.rows = []

        def send(self, *a):
            self.eng.send(*a)
            self.n += 1
            if self.n == self.cut:
                if drain_first:
                    self.rows.append(self.eng.drain())
                image = self.eng.snapshot()
                self.eng.close()
                self.eng = HipEngine(c)
                self.eng.start()
                self.eng.restore(image)

        def drain(self):
            d = self.eng.drain()
            from siddhi_amd.abi import concat_drains
            return concat_drains(self.rows + [d])

        def __getattr__(self, name):
            return getattr(self.eng, name)

    sp = Split(len(blocks) // 2)
    got = run_c4(sp, blocks)
    assert len(ref["seq"]) > 0
    assert same_output(got, ref)


def test_restore_refuses_another_app_and_used_handles():
    from siddhi_amd._native import HipEngine, HipError
    a = compiler.compile_app(synth.C4_QUERY)
    b = compiler.compile_app(synth.C2_QUERY)
    ea = HipEngine(a)
    ea.start()
    image = ea.snapshot()
    eb = HipEngine(b)
    eb.start()
    with pytest.raises(HipError):
        eb.restore(image)
    ea2 = HipEngine(a)
    ea2.start()
    with pytest.raises(HipError):
        ea2.restore(image[: len(image) // 2])
    # a failed restore leaves the handle as it was: the good image still restores
    ea2.restore(image)
    ea3 = HipEngine(a)
    ea3.start()
    ea3.restore(image)
    for e in (ea, eb, ea2, ea3):
        e.close()


def test_failed_restore_leaves_the_handle_usable():
    """a damaged image is refused after part of it was applied; the handle keeps
    working from its own state (the C4 stream then matches the oracle's)"""
    from c4_cases import register_users, run_c4, same_output
    from siddhi_amd._native import HipEngine, HipError
    from oracle_engine import OracleEngine
    c = compiler.compile_app(synth.C4_QUERY)
    blocks = synth.c4_stream(3_000, seconds=20, seed=11)
    src = HipEngine(c)
    register_users(src, blocks)
    src.start()
    seq = 0
    for st, ts, cols, keys in blocks[: len(blocks) // 2]:
        src.send(st, ts, cols, [None] * len(cols), keys, seq)
        seq += len(ts)
    image = src.snapshot()
    src.close()
    eng = HipEngine(c)
    with pytest.raises(HipError) as ei:
        eng.restore(image[: len(image) - 16])  # parsed almost to the end before it fails
    assert "could not be reset" not in str(ei.value), str(ei.value)
    got = run_c4(eng, blocks)
    ref = run_c4(OracleEngine(c), blocks)
    eng.close()
    assert len(ref["seq"]) > 0 and same_output(got, ref)
