"""N>1 path on CPU over gloo (world size 2): the product's sharded step
(siddhi_amd.shard.KeyShardedStep: route -> all-to-all shuffle -> per-rank match
-> return all-to-all -> k-way merge by trigger sequence) reproduces the
single-process ordered match stream exactly.

The device kernels of the step (include/siddhi_shard.h) need a GPU; here the
same orchestration runs with numpy stand-ins of those kernels (CpuShardOps,
test infrastructure, checked against the kernels' contract on the GPU in
tests/test_gpu_shard.py) and the CPU oracle as each rank's matcher."""
import os
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))


class CpuShardOps:
    """numpy restatement of the shs_* kernels' contract (test infrastructure)"""

    def route(self, keys, world):
        from siddhi_amd import shard
        own = shard.shard_of(keys.numpy(), world)
        order = np.argsort(own, kind="stable")
        pos = np.empty(len(own), np.int64)
        pos[order] = np.arange(len(own))
        counts = np.bincount(own, minlength=world)
        return torch.from_numpy(pos), [int(c) for c in counts]

    def pack(self, pos, cols, seq0):
        n = cols[0].numel()
        words = []
        for c in cols:
            a = c.numpy()
            if a.dtype.itemsize == 8:
                w = a.view(np.uint32).reshape(n, 2)
            else:
                w = a.view(np.uint32).reshape(n, 1)
            words.append(w)
        seq = (np.arange(n, dtype=np.uint64) + np.uint64(seq0)).view(np.uint32).reshape(n, 2)
        rows = np.concatenate(words + [seq], axis=1)
        out = np.empty_like(rows)
        out[pos.numpy()] = rows
        return torch.from_numpy(out.view(np.int32).reshape(-1).copy()), rows.shape[1]

    def unpack(self, rec, n, like):
        stride = sum(2 if c.element_size() == 8 else 1 for c in like) + 2
        rows = rec.numpy().view(np.uint32).reshape(n, stride)
        cols, w = [], 0
        for c in like:
            k = 2 if c.element_size() == 8 else 1
            cols.append(torch.from_numpy(rows[:, w:w + k].copy().view(c.numpy().dtype).reshape(n)))
            w += k
        seq = torch.from_numpy(rows[:, w:w + 2].copy().view(np.int64).reshape(n))
        return cols, seq

    def rows_home(self, oseq, m, seq_base, gseq, src_off, world):
        local = oseq.numpy()[:m] - seq_base
        b = np.searchsorted(local, np.asarray(src_off), side="left")
        oseq.numpy()[:m] = gseq.numpy()[local]
        return [int(b[r + 1] - b[r]) for r in range(world)]

    def merge(self, seq, vals, n_out, run_off):
        s = seq.numpy()
        order = np.argsort(s, kind="stable")
        v = vals.numpy().reshape(-1, n_out) if n_out else np.zeros((len(s), 0), np.int64)
        return torch.from_numpy(s[order].copy()), torch.from_numpy(v[order].copy())


def _oracle_matcher(compiled):
    sys.path.insert(0, HERE)
    from oracle_engine import run_stock_oracle

    def match(ts, keys, cols, n_keys):
        seq, _, vals, _ = run_stock_oracle(compiled, ts.numpy(), keys.numpy(), cols[0].numpy(), cols[1].numpy())
        return len(seq), torch.from_numpy(seq.astype(np.int64)), torch.from_numpy(vals)
    return match


def _stream():
    from siddhi_amd import synth
    return synth.stock_stream(60_000, 300, 20)


def _worker(rank, world, port, result_q):
    sys.path.insert(0, HERE)
    sys.path.insert(0, os.path.dirname(HERE))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from siddhi_amd import compiler, shard, synth
    ts, k, p, v = _stream()
    b = shard.slice_bounds(len(ts), world)
    lo, hi = b[rank], b[rank + 1]
    ca = compiler.compile_app(synth.C2_QUERY)
    step = shard.KeyShardedStep(world, rank, CpuShardOps(), _oracle_matcher(ca), n_out=4)
    seq, vals = step.run(torch.from_numpy(ts[lo:hi].copy()), torch.from_numpy(k[lo:hi].copy()),
                         [torch.from_numpy(p[lo:hi].copy()), torch.from_numpy(v[lo:hi].copy())], lo, 300)
    parts = [None] * world
    dist.all_gather_object(parts, (seq.numpy(), vals.numpy(), step.last))
    if rank == 0:
        result_q.put(parts)
    dist.barrier()
    dist.destroy_process_group()


def test_sharded_step_world2_equals_single_process():
    from oracle_engine import run_stock_oracle
    from siddhi_amd import compiler, synth
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + os.getpid() % 1000
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for pr in procs:
        pr.start()
    parts = q.get(timeout=300)
    for pr in procs:
        pr.join(timeout=120)
        assert pr.exitcode == 0
    ts, k, p, v = _stream()
    seq, _, vals, _ = run_stock_oracle(compiler.compile_app(synth.C2_QUERY), ts, k, p, v)
    mseq = np.concatenate([x[0] for x in parts])
    mvals = np.concatenate([x[1] for x in parts])
    # both ranks shuffled events both ways and matched
    assert all(min(x[2]["sent"]) > 0 and x[2]["matches_here"] > 0 for x in parts)
    assert len(mseq) == len(seq) > 0
    assert np.array_equal(mseq, seq.astype(np.int64))
    assert np.array_equal(mvals, vals)


@pytest.mark.parametrize("world", [1, 3])
def test_cpu_ops_route_pack_roundtrip(world):
    """the stand-in ops keep the kernels' contract: owner-major stable routing,
    exact record round trip, merge by sequence"""
    from siddhi_amd import shard
    rng = np.random.default_rng(world)
    n = 5000
    keys = rng.integers(0, 777, n).astype(np.int32)
    ts = np.arange(n, dtype=np.int64) * 3
    f = rng.random(n).astype(np.float32)
    ops = CpuShardOps()
    pos, counts = ops.route(torch.from_numpy(keys), world)
    own = shard.shard_of(keys, world)
    assert counts == [int((own == r).sum()) for r in range(world)]
    rec, stride = ops.pack(pos, [torch.from_numpy(ts), torch.from_numpy(keys), torch.from_numpy(f)], 1000)
    cols, seq = ops.unpack(rec, n, [torch.from_numpy(ts), torch.from_numpy(keys), torch.from_numpy(f)])
    order = np.argsort(own, kind="stable")
    assert np.array_equal(cols[0].numpy(), ts[order]) and np.array_equal(cols[1].numpy(), keys[order])
    assert np.array_equal(cols[2].numpy(), f[order]) and np.array_equal(seq.numpy(), 1000 + order)
