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

    # the compact record contract (shs_pack_compact / shs_unpack_compact): column 0
    # as a 32-bit offset from the slice's timestamp base, the sequence number as a
    # 32-bit index into the source slice
    compact = True

    def pack_compact(self, pos, cols, tbase):
        n = cols[0].numel()
        words = [(cols[0].numpy().astype(np.int64) - tbase).astype(np.uint32).reshape(n, 1)]
        for c in cols[1:]:
            a = c.numpy()
            words.append(a.view(np.uint32).reshape(n, 2 if a.dtype.itemsize == 8 else 1))
        idx = np.arange(n, dtype=np.uint32).reshape(n, 1)
        rows = np.concatenate(words + [idx], axis=1)
        out = np.empty_like(rows)
        out[pos.numpy()] = rows
        return torch.from_numpy(out.view(np.int32).reshape(-1).copy()), rows.shape[1]

    def unpack_compact(self, rec, like, src_off, src_tbase, src_seq0):
        n = src_off[-1]
        stride = 1 + sum(2 if c.element_size() == 8 else 1 for c in like[1:]) + 1
        rows = rec.numpy().view(np.uint32).reshape(n, stride)
        src = np.searchsorted(np.asarray(src_off[1:]), np.arange(n), side="right")
        cols = [torch.from_numpy((rows[:, 0].astype(np.int64) + np.asarray(src_tbase, np.int64)[src]))]
        w = 1
        for c in like[1:]:
            k = 2 if c.element_size() == 8 else 1
            cols.append(torch.from_numpy(rows[:, w:w + k].copy().view(c.numpy().dtype).reshape(n)))
            w += k
        seq = np.asarray(src_seq0, np.int64)[src] + rows[:, w].astype(np.int64)
        return cols, torch.from_numpy(seq)

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


def _oracle_matcher(compiled, with_query=False):
    """the CPU oracle on the received events: send() calls cut at the run ids when
    given (each PartitionStreamReceiver run of the whole stream its own call, which
    keeps the reference's (run, query, event) order), else calls of 4096"""
    sys.path.insert(0, HERE)
    from oracle_engine import OracleEngine

    def match(ts, keys, cols, n_keys, run=None):
        ts, keys = ts.numpy(), keys.numpy()
        cols = [c.numpy() for c in cols]
        n = len(ts)
        if run is not None:
            r = run.numpy()
            cuts = np.concatenate([[0], np.flatnonzero(r[1:] != r[:-1]) + 1, [n]])
        else:
            cuts = np.concatenate([np.arange(0, n, 4096), [n]])
        eng = OracleEngine(compiled)
        eng.start()
        for a, b in zip(cuts[:-1], cuts[1:]):
            if b > a:
                eng.send(0, ts[a:b], [np.ascontiguousarray(c[a:b]) for c in cols], [None] * len(cols),
                         np.ascontiguousarray(keys[a:b]), int(a))
        out = eng.drain()
        eng.close()
        vals = out["values"]
        if with_query:
            vals = np.concatenate([vals, out["query"].astype(np.int64)[:, None]], 1)
        return len(out["seq"]), torch.from_numpy(out["seq"].astype(np.int64)), torch.from_numpy(vals)
    return match


C5_TEST_RULES = 40


def _case(config):
    """(compiled, ts, keys, cols, n_keys, n_out, with_query, run ids?) of a small stream"""
    from siddhi_amd import compiler, synth
    if config == "c5":
        ts, card, amount, merchant = synth.txn_stream(60_000, 300, 20, n_merchants=20)
        rules = synth.c5_rules(C5_TEST_RULES, merchants=20, within=(1, 3), amount=(20.0, 200.0))
        ca = compiler.compile_app(synth.c5_query(rules))
        return ca, ts, card, [card, amount, merchant], 300, 2, True, True
    ts, k, p, v = synth.stock_stream(60_000, 300, 20)
    ca = compiler.compile_app(synth.C3_QUERY if config == "c3" else synth.C2_QUERY)
    return ca, ts, k, [k, p, v], 300, 3 if config == "c3" else 4, False, False


def _worker(rank, world, port, config, result_q):
    sys.path.insert(0, HERE)
    sys.path.insert(0, os.path.dirname(HERE))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from siddhi_amd import shard
    ca, ts, k, cols, K, n_out, wq, runs = _case(config)
    b = shard.slice_bounds(len(ts), world, align=4096)
    lo, hi = b[rank], b[rank + 1]
    rid = shard.stream_run_ids(k, 4096) if runs else None
    step = shard.KeyShardedStep(world, rank, CpuShardOps(), _oracle_matcher(ca, wq), n_out=n_out + (1 if wq else 0))
    t = lambda a: torch.from_numpy(a[lo:hi].copy())  # noqa: E731
    seq, vals = step.run(t(ts), t(k), [t(c) for c in cols], lo, K, key_attr=0,
                         run_ids=t(rid) if rid is not None else None)
    parts = [None] * world
    dist.all_gather_object(parts, (seq.numpy(), vals.numpy(), step.last))
    if rank == 0:
        result_q.put(parts)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("config", ["c2", "c3", "c5"])
def test_sharded_step_world2_equals_single_process(config):
    """C2, C3 and C5 (1 stream, world 2): the ranks' outputs concatenated equal the
    single-process oracle's ordered match stream (C5 with its query column; its
    rows leave each run query-major, so the step carries the run ids)."""
    from oracle_engine import OracleEngine
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + (os.getpid() + hash(config)) % 1000
    procs = [ctx.Process(target=_worker, args=(r, 2, port, config, q)) for r in range(2)]
    for pr in procs:
        pr.start()
    parts = q.get(timeout=300)
    for pr in procs:
        pr.join(timeout=120)
        assert pr.exitcode == 0
    ca, ts, k, cols, K, n_out, wq, runs = _case(config)
    eng = OracleEngine(ca)
    eng.start()
    for b0 in range(0, len(ts), 4096):
        b1 = min(len(ts), b0 + 4096)
        eng.send(0, ts[b0:b1], [np.ascontiguousarray(c[b0:b1]) for c in cols], [None] * len(cols),
                 np.ascontiguousarray(k[b0:b1]), b0)
    ref = eng.drain()
    eng.close()
    want = ref["values"]
    if wq:
        want = np.concatenate([want, ref["query"].astype(np.int64)[:, None]], 1)
    mseq = np.concatenate([x[0] for x in parts])
    mvals = np.concatenate([x[1] for x in parts])
    # both ranks shuffled events both ways and matched, in compact records
    assert all(min(x[2]["sent"]) > 0 and x[2]["matches_here"] > 0 for x in parts)
    assert all(x[2]["compact"] for x in parts)
    if config == "c2":  # ts offset 4 + symbol 4 + price 4 + volume 8 + slice index 4
        assert all(x[2]["record_bytes"] == 24 for x in parts)
    assert len(mseq) == len(ref["seq"]) > 0
    assert np.array_equal(mseq, ref["seq"].astype(np.int64))
    assert np.array_equal(mvals, want)
    if config == "c5":
        # the stream has same-card runs longer than one event, and the order inside
        # them is not the trigger order (what the run-keyed merge must keep)
        assert not np.all(np.diff(ref["seq"].astype(np.int64)) >= 0)


def test_stream_run_ids():
    from siddhi_amd import shard
    k = np.array([5, 5, 7, 7, 7, 5, 5, 5, 9], np.int32)
    assert shard.stream_run_ids(k, 4).tolist() == [0, 0, 2, 2, 4, 5, 5, 5, 8]
    assert shard.stream_run_ids(k, 0).tolist() == [0, 0, 2, 2, 2, 5, 5, 5, 8]
    assert shard.slice_bounds(10_000, 3, align=4096) == [0, 4096, 8192, 10_000]


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


def test_cpu_ops_compact_roundtrip():
    """compact records: timestamps rebuilt from each source's base, sequence
    numbers from each source's first one"""
    rng = np.random.default_rng(5)
    ops = CpuShardOps()
    parts = []
    for src, (n, tb, s0) in enumerate([(700, 1_700_000_000_000, 0), (500, 1_700_000_900_000, 700)]):
        keys = rng.integers(0, 99, n).astype(np.int32)
        ts = tb + np.sort(rng.integers(0, 1 << 31, n)).astype(np.int64)
        v = rng.integers(-5, 5, n).astype(np.int64)
        pos = torch.from_numpy(np.arange(n))
        rec, stride = ops.pack_compact(pos, [torch.from_numpy(ts), torch.from_numpy(keys), torch.from_numpy(v)],
                                       int(ts.min()))
        assert stride == 5  # 1 + 1 + 2 + 1 words
        parts.append((rec, ts, keys, v, int(ts.min()), s0))
    rec = torch.cat([p[0] for p in parts])
    like = [torch.zeros(1, dtype=torch.int64), torch.zeros(1, dtype=torch.int32), torch.zeros(1, dtype=torch.int64)]
    cols, seq = ops.unpack_compact(rec, like, [0, 700, 1200], [p[4] for p in parts], [p[5] for p in parts])
    assert np.array_equal(cols[0].numpy(), np.concatenate([p[1] for p in parts]))
    assert np.array_equal(cols[1].numpy(), np.concatenate([p[2] for p in parts]))
    assert np.array_equal(cols[2].numpy(), np.concatenate([p[3] for p in parts]))
    assert np.array_equal(seq.numpy(), np.arange(1200))
