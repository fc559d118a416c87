"""N>1 path on CPU: key-hash sharding over a gloo process group (world size 2)
reproduces the single-process ordered match stream exactly."""
import os
import sys

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))


def _worker(rank, world, port, result_q):
    sys.path.insert(0, HERE)
    sys.path.insert(0, os.path.dirname(HERE))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle_engine import run_stock_oracle
    from siddhi_amd import compiler, shard, synth
    ts, k, p, v = synth.stock_stream(40_000, 300, 20)
    idx = shard.split(k, world)[rank]
    ca = compiler.compile_app(synth.C2_QUERY)
    # this rank's events keep their global sequence numbers
    seq, ots, vals, _ = run_stock_oracle(ca, ts[idx], k[idx], p[idx], v[idx])
    gseq = idx[seq.astype(np.int64)]
    parts = [None] * world
    dist.all_gather_object(parts, (gseq, ots, vals))
    if rank == 0:
        result_q.put(shard.merge(parts))
    dist.barrier()
    dist.destroy_process_group()


def test_key_sharded_world2_equals_single_process():
    from oracle_engine import run_stock_oracle
    from siddhi_amd import compiler, synth
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + os.getpid() % 1000
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for pr in procs:
        pr.start()
    merged = q.get(timeout=300)
    for pr in procs:
        pr.join(timeout=120)
        assert pr.exitcode == 0
    ts, k, p, v = synth.stock_stream(40_000, 300, 20)
    seq, ots, vals, _ = run_stock_oracle(compiler.compile_app(synth.C2_QUERY), ts, k, p, v)
    mseq, mts, mvals = merged
    assert len(mseq) == len(seq) > 0
    assert np.array_equal(mseq, seq.astype(np.int64))
    assert np.array_equal(mts, ots)
    assert np.array_equal(mvals, vals)
