"""Key-sharded C4 on the GPU: 2 and 4 virtual ranks (threads of one process, one
handle each, sharing the card) run the product engine (libsiddhi_hip.so,
sh_push_batch_part / sh_set_coordinator / sh_drain_ordered) with the product's
coordinator (siddhi_amd/shard_stream.py); the merged output must equal the
single-process oracle's row for row (Scheduler.onTimeChange's cross-key pick,
core/util/Scheduler.java:74-99, decided over all ranks)."""
import threading

import pytest

from c4_cases import CollidingNames, register_users, run_c4, same_output, ties
from oracle_engine import OracleEngine

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _device():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _sharded(c, blocks, world, names=None):
    from siddhi_amd import synth
    from siddhi_amd._native import HipEngine
    from siddhi_amd.shard_stream import ShardedStreamEngine, ThreadComm, merge_ordered
    comm = ThreadComm(world)
    outs, errs, owned = [None] * world, [], [0] * world

    def body(r):
        try:
            base = HipEngine(c)
            eng = ShardedStreamEngine(CollidingNames(base, names) if names else base, comm.view(r))
            register_users(eng, blocks)
            eng.start()
            for st, ts, cols, keys in blocks:
                eng.send(st, ts, cols, [None] * len(cols), keys)
            eng.advance_time(synth.c4_end_time(blocks))
            eng.check()
            outs[r] = eng.drain()
            owned[r] = eng.owned
            base.close()
        except Exception as e:  # noqa: BLE001
            errs.append(e)
            comm.bar.abort()

    th = [threading.Thread(target=body, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=900)
    assert not errs, errs
    assert all(o > 0 for o in owned)
    return merge_ordered(outs)


@pytest.mark.parametrize("world", [2, 4])
def test_c4_key_sharded_virtual_ranks_vs_oracle(world):
    from siddhi_amd import compiler, synth
    c = compiler.compile_app(synth.C4_QUERY)
    blocks = synth.c4_stream(5_000, seconds=5)
    assert ties(blocks) > 100
    ref = run_c4(OracleEngine(c), blocks)
    got = _sharded(c, blocks, world)
    assert len(ref["seq"]) > 1000
    assert same_output(got, ref)


def test_c4_key_sharded_colliding_names():
    from siddhi_amd import compiler, synth
    n = 2000
    c = compiler.compile_app(synth.C4_QUERY)
    blocks = synth.c4_stream(n, seconds=10)
    ref = run_c4(CollidingNames(OracleEngine(c), n), blocks)
    got = _sharded(c, blocks, 2, names=n)
    assert len(ref["seq"]) > 500
    assert same_output(got, ref)


@pytest.mark.parametrize("query", ["C4_QUERY", "C4_EVERY_QUERY"])
def test_c4_spec_mix_key_sharded(query):
    """the SURVEY 8d mix (Login 20% / Txn 60% / Logout 20%, send() calls of 4,096
    per stream), both select variants, 2 ranks"""
    from siddhi_amd import compiler, synth
    c = compiler.compile_app(getattr(synth, query))
    blocks = synth.c4_spec_stream(300_000, 20_000, rate_per_ms=5, seed=3)
    ref = run_c4(OracleEngine(c), blocks)
    got = _sharded(c, blocks, 2)
    assert len(ref["seq"]) > 1000
    assert same_output(got, ref)


@pytest.mark.parametrize("query", ["C4_QUERY", "C4_EVERY_QUERY"])
def test_c4_spec_mix_single_gpu(query):
    """the spec mix on one handle (the N = 1 bench path) at 1M users"""
    from siddhi_amd import compiler, synth
    from siddhi_amd._native import HipEngine
    c = compiler.compile_app(getattr(synth, query))
    blocks = synth.c4_spec_stream(2_000_000, 1_000_000, seed=4)
    ref = run_c4(OracleEngine(c), blocks)
    eng = HipEngine(c)
    got = run_c4(eng, blocks)
    eng.close()
    assert len(ref["seq"]) > 1000
    assert same_output(got, ref)
