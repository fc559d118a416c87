"""Key-sharded streaming (siddhi_amd/shard_stream.py) on CPU: C4's absence timers
couple keys only through Scheduler.onTimeChange's one-state-per-due-time pick and
the state map's HashMap order (core/util/Scheduler.java:74-99,
PartitionStateHolder.java:36,131-162). Each rank runs the general engine's kernel
logic built for the CPU (tests/nfa_host, the code k_nfa runs on the GPU) on its
own keys, with the product's coordinator (candidate gather + history exchange)
and the product's merge; the merged output must equal the single-process
oracle's, row for row. Virtual ranks share one process (threads, ThreadComm);
the gloo test runs real processes (TorchGroupComm)."""
import os
import sys
import threading

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from c4_cases import CollidingNames, register_users, same_output, ties

HERE = os.path.dirname(os.path.abspath(__file__))


def _oracle(c, blocks, names=None):
    from c4_cases import run_c4
    from oracle_engine import OracleEngine
    eng = OracleEngine(c)
    return run_c4(CollidingNames(eng, names) if names else eng, blocks)


def _run_rank(eng, blocks, end_time):
    register_users(eng, blocks)
    eng.start()
    for st, ts, cols, keys in blocks:
        eng.send(st, ts, cols, [None] * len(cols), keys)
    eng.advance_time(end_time)
    eng.check()
    return eng.drain()


def _threads(c, blocks, world, names=None):
    """world virtual ranks in threads; returns the merged output and per-rank info"""
    from nfa_host_engine import NfaHostEngine
    from siddhi_amd import synth
    from siddhi_amd.shard_stream import ShardedStreamEngine, ThreadComm, merge_ordered
    comm = ThreadComm(world)
    outs, errs, info = [None] * world, [], [None] * world

    def body(r):
        try:
            base = NfaHostEngine(c)
            eng = ShardedStreamEngine(CollidingNames(base, names) if names else base, comm.view(r))
            outs[r] = _run_rank(eng, blocks, synth.c4_end_time(blocks))
            info[r] = (eng.owned, eng.sent, eng.coord.exchanges)
        except Exception as e:  # noqa: BLE001
            errs.append(e)
            comm.bar.abort()

    th = [threading.Thread(target=body, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=600)
    assert not errs, errs
    return merge_ordered(outs), info


def test_pick_one_state_per_due_time():
    from siddhi_amd.shard_stream import _CAND, pick
    a = np.zeros(3, _CAND)
    a["t"], a["order"], a["key"] = [5, 7, 5], [30, 1, 10], [1, 2, 3]
    b = np.zeros(2, _CAND)
    b["t"], b["order"], b["key"] = [5, 6], [20, 9], [4, 5]
    pos, n = pick([a, b], wall=False)
    # due 5: order 10 (rank 0, key 3) wins; due 6: key 5; due 7: key 2
    assert n == 3
    assert pos[0].tolist() == [-1, 2, 0] and pos[1].tolist() == [-1, 1]
    pos, n = pick([a, b], wall=True)
    assert n == 5
    assert pos[0].tolist() == [2, 4, 0] and pos[1].tolist() == [1, 3]
    pos, n = pick([np.zeros(0, _CAND), np.zeros(0, _CAND)], wall=False)
    assert n == 0


@pytest.mark.parametrize("world", [2, 3])
def test_c4_virtual_ranks_equal_single_process(world):
    from siddhi_amd import compiler, synth
    c = compiler.compile_app(synth.C4_QUERY)
    blocks = synth.c4_stream(3000, seconds=5)
    assert ties(blocks) > 100  # shared due milliseconds: the cross-rank pick matters
    ref = _oracle(c, blocks)
    got, info = _threads(c, blocks, world)
    assert len(ref["seq"]) > 1000
    assert all(o > 0 for o, _, _ in info) and sum(o for o, _, _ in info) == info[0][1]
    assert same_output(got, ref)


def test_c4_virtual_ranks_colliding_names():
    """names sharing one String.hashCode per length: the ranks' models must agree
    on treeified bins (compareTo order) as well"""
    from siddhi_amd import compiler, synth
    n = 1500
    c = compiler.compile_app(synth.C4_QUERY)
    blocks = synth.c4_stream(n, seconds=8)
    ref = _oracle(c, blocks, names=n)
    got, _ = _threads(c, blocks, 2, names=n)
    assert len(ref["seq"]) > 300
    assert same_output(got, ref)


def test_c4_every_variant_virtual_ranks():
    """`every (e1=Login and e2=Txn) -> not Logout for 5 sec`: several alerts per key"""
    from siddhi_amd import compiler, synth
    c = compiler.compile_app(synth.C4_EVERY_QUERY)
    blocks = synth.c4_spec_stream(40_000, 2_000, rate_per_ms=2, batch=512, seed=11)
    ref = _oracle(c, blocks)
    got, _ = _threads(c, blocks, 2)
    assert len(ref["seq"]) > 1000
    assert same_output(got, ref)


def _gloo_worker(rank, world, port, result_q):
    sys.path.insert(0, HERE)
    sys.path.insert(0, os.path.dirname(HERE))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from nfa_host_engine import NfaHostEngine
    from siddhi_amd import compiler, synth
    from siddhi_amd.shard_stream import ShardedStreamEngine, TorchGroupComm
    c = compiler.compile_app(synth.C4_QUERY)
    blocks = synth.c4_stream(3000, seconds=5)
    eng = ShardedStreamEngine(NfaHostEngine(c), TorchGroupComm())
    out = _run_rank(eng, blocks, synth.c4_end_time(blocks))
    parts = [None] * world
    dist.all_gather_object(parts, (out, eng.owned))
    if rank == 0:
        result_q.put(parts)
    dist.barrier()
    dist.destroy_process_group()


def test_c4_gloo_world2_equals_single_process():
    from siddhi_amd import compiler, synth
    from siddhi_amd.shard_stream import merge_ordered
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + (os.getpid() + 17) % 1000
    procs = [ctx.Process(target=_gloo_worker, args=(r, 2, port, q)) for r in range(2)]
    for pr in procs:
        pr.start()
    parts = q.get(timeout=600)
    for pr in procs:
        pr.join(timeout=120)
        assert pr.exitcode == 0
    assert all(p[1] > 0 for p in parts)
    got = merge_ordered([p[0] for p in parts])
    c = compiler.compile_app(synth.C4_QUERY)
    ref = _oracle(c, synth.c4_stream(3000, seconds=5))
    assert len(ref["seq"]) > 1000
    assert same_output(got, ref)


class _RecEngine:
    """records what ShardedStreamEngine pushes (no device)"""

    def __init__(self):
        self.parts = []

    def set_coordinator(self, coord):
        pass

    def send_part(self, stream, ts, cols, nulls, keys, index, call_n, call_last):
        self.parts.append((len(ts), None if keys is None else keys.copy(), index.copy(), call_n))


def test_keyless_stream_goes_to_the_null_key_rank_only():
    """a stream without a partition key (null keys) is pushed by the rank that
    owns null keys, as owner() routes keys < 0 -- never by every rank"""
    from siddhi_amd.shard_stream import ShardedStreamEngine, ThreadComm
    comm = ThreadComm(3)
    engs = [_RecEngine() for _ in range(3)]
    shards = [ShardedStreamEngine(e, comm.view(r), null_key_rank=1) for r, e in enumerate(engs)]
    ts = np.arange(10, dtype=np.int64)
    for s in shards:
        s.send(0, ts, [np.arange(10, dtype=np.int32)], [None], None)
    assert [e.parts[0][0] for e in engs] == [0, 10, 0]
    assert all(e.parts[0][3] == 10 for e in engs)  # every rank still takes the call's steps
    keys = np.array([-1, 3, -1, 7, 5], np.int32)
    for s in shards:
        s.send(0, ts[:5], [keys], [None], keys)
    pushed = sorted(int(i) for e in engs for i in e.parts[1][2])
    assert pushed == list(range(5))
    assert set(engs[1].parts[1][2]) >= {0, 2}


def test_thread_comm_failure_breaks_the_group():
    """one rank's failing coordinator callback aborts the barrier: the other
    ranks' all_gather fails promptly instead of waiting forever"""
    import threading
    from siddhi_amd.shard_stream import Coordinator, ThreadComm
    comm = ThreadComm(3)
    c0 = Coordinator(comm.view(0))
    errors = []

    def peer(r):
        try:
            comm.view(r).all_gather(np.zeros(1, np.int64))
        except threading.BrokenBarrierError as e:
            errors.append(e)

    th = [threading.Thread(target=peer, args=(r,)) for r in (1, 2)]
    for t in th:
        t.start()
    assert c0._fail(RuntimeError("rank 0 failed")) == 1
    for t in th:
        t.join(timeout=10)
    assert not any(t.is_alive() for t in th)
    assert len(errors) == 2 and isinstance(c0.error, RuntimeError)
