"""GPU checks of the key-sharded multi-GPU path (include/siddhi_shard.h,
siddhi_amd/shard.py):
  * the shs_* kernels against their numpy contract (tests/test_sharding.py
    CpuShardOps): owner-major stable routing, record round trip, return route,
    k-way merge by trigger sequence;
  * the whole sharded step with 2 and 4 virtual ranks on one GPU (threads, the
    all-to-all exchanges done in host memory), each rank running the product
    matcher (sh_run_device) on the events of its keys: the ranks' outputs
    concatenated equal the single-stream result of the vectorised restatement,
    bit for bit. Real multi-GPU runs use the same step with RCCL (bench.py)."""
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _device():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _ops():
    from siddhi_amd.shard import HipShardOps
    return HipShardOps("cuda:0")


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_route_pack_unpack_match_contract(world):
    import torch
    from test_sharding import CpuShardOps
    rng = np.random.default_rng(40 + world)
    n = 300_001
    keys = rng.integers(0, 10_000, n).astype(np.int32)
    ts = np.cumsum(rng.integers(0, 3, n)).astype(np.int64)
    f = rng.random(n).astype(np.float32)
    v = rng.integers(-5, 5, n).astype(np.int64)
    host = [torch.from_numpy(a) for a in (ts, keys, f, v)]
    dev = [t.cuda() for t in host]
    hip, cpu = _ops(), CpuShardOps()
    pos_d, cnt_d = hip.route(dev[1], world)
    pos_c, cnt_c = cpu.route(host[1], world)
    assert cnt_d == cnt_c
    assert np.array_equal(pos_d[:n].cpu().numpy().astype(np.int64), pos_c.numpy())
    rec_d, stride_d = hip.pack(pos_d, dev, 77)
    rec_c, stride_c = cpu.pack(pos_c, host, 77)
    assert stride_d == stride_c == 8
    assert np.array_equal(rec_d.cpu().numpy(), rec_c.numpy())
    cols, seq = hip.unpack(rec_d, n, dev)
    order = np.argsort(pos_c.numpy())
    for c, a in zip(cols, (ts, keys, f, v)):
        assert np.array_equal(c.cpu().numpy(), a[order])
    assert np.array_equal(seq.cpu().numpy(), 77 + order)


def test_compact_pack_unpack_match_contract():
    """shs_pack_compact / shs_unpack_compact against the numpy contract: two
    sources with their own timestamp bases and first sequence numbers"""
    import torch
    from test_sharding import CpuShardOps
    rng = np.random.default_rng(71)
    hip, cpu = _ops(), CpuShardOps()
    recs_d, recs_c, want, s0s, tbs = [], [], [], [], []
    s0 = 0
    for n, tb in ((200_003, 1_700_000_000_000), (150_001, 1_700_003_000_000)):
        keys = rng.integers(0, 10_000, n).astype(np.int32)
        ts = tb + np.cumsum(rng.integers(0, 3, n)).astype(np.int64)
        f = rng.random(n).astype(np.float32)
        v = rng.integers(-5, 5, n).astype(np.int64)
        host = [torch.from_numpy(a) for a in (ts, keys, f, v)]
        pos_c, _ = cpu.route(host[1], 3)
        pos_d = pos_c.to(torch.int32).cuda()
        rd, sd = hip.pack_compact(pos_d, [t.cuda() for t in host], int(ts.min()))
        rc, sc = cpu.pack_compact(pos_c, host, int(ts.min()))
        assert sd == sc == 6  # ts 1 + key 1 + price 1 + volume 2 + index 1 words (24 B)
        assert np.array_equal(rd.cpu().numpy(), rc.numpy())
        order = np.argsort(pos_c.numpy())
        recs_d.append(rd)
        want.append((ts[order], keys[order], f[order], v[order], s0 + order))
        s0s.append(s0)
        tbs.append(int(ts.min()))
        s0 += n
    like = [torch.zeros(1, dtype=t, device="cuda:0") for t in (torch.int64, torch.int32, torch.float32, torch.int64)]
    off = [0, 200_003, 350_004, 350_004]
    cols, seq = hip.unpack_compact(torch.cat(recs_d), like, off, tbs + [0], s0s + [0])
    for i, c in enumerate(cols):
        assert np.array_equal(c.cpu().numpy(), np.concatenate([w[i] for w in want]))
    assert np.array_equal(seq.cpu().numpy(), np.concatenate([w[4] for w in want]))


def test_rows_home_and_merge():
    import torch
    rng = np.random.default_rng(5)
    # 3 owners' runs of ascending, disjoint sequence numbers
    allseq = rng.permutation(np.arange(50_000, dtype=np.int64))[:30_000]
    runs = [np.sort(allseq[i::3]) for i in range(3)]
    off = [0]
    for r in runs:
        off.append(off[-1] + len(r))
    seq = torch.from_numpy(np.concatenate(runs)).cuda()
    vals = torch.from_numpy(np.stack([np.concatenate(runs) * 3, -np.concatenate(runs)], 1).reshape(-1)).cuda()
    so, vo = _ops().merge(seq, vals, 2, off)
    want = np.sort(allseq)
    assert np.array_equal(so.cpu().numpy(), want)
    assert np.array_equal(vo.cpu().numpy(), np.stack([want * 3, -want], 1))
    # return route: local row indices -> global sequence numbers, per-source counts
    gseq = torch.from_numpy(np.arange(1000, dtype=np.int64) * 7 + 3).cuda()
    local = np.sort(rng.choice(1000, 400, replace=False)).astype(np.int64)
    oseq = torch.from_numpy(local.copy()).cuda()
    src_off = [0, 100, 450, 1000]
    counts = _ops().rows_home(oseq, len(local), 0, gseq, src_off, 3)
    assert counts == [int(((local >= src_off[r]) & (local < src_off[r + 1])).sum()) for r in range(3)]
    assert np.array_equal(oseq.cpu().numpy(), local * 7 + 3)


class _ThreadComm:
    """host-memory all-to-all between threads (test infrastructure)"""

    def __init__(self, world):
        self.world = world
        self.bar = threading.Barrier(world)
        self.box = {}

    def view(self, rank):
        comm = self

        class V:
            def meta(self, vals, device):
                comm.box[("meta", rank)] = list(vals)
                comm.bar.wait()
                got = [list(comm.box[("meta", s)]) for s in range(comm.world)]
                comm.bar.wait()
                return got

            def counts(self, counts, device):
                for d in range(comm.world):
                    comm.box[(rank, d)] = counts[d]
                comm.bar.wait()
                got = [comm.box[(s, rank)] for s in range(comm.world)]
                comm.bar.wait()
                return got

            def exchange(self, send, send_counts, recv_counts, per):
                import torch
                torch.cuda.synchronize()
                o = 0
                for d in range(comm.world):
                    k = send_counts[d] * per
                    comm.box[(rank, d)] = send[o:o + k].clone()
                    o += k
                torch.cuda.synchronize()
                comm.bar.wait()
                got = torch.cat([comm.box[(s, rank)] for s in range(comm.world)])
                comm.bar.wait()
                return got
        return V()


def _shard_case(config):
    """(compiled, ts, keys, cols, n_keys, expected(), with_query, runs) per config"""
    from siddhi_amd import compiler, synth
    if config == "c5":
        from c5_check import c5_expected
        ts, card, amount, merchant = synth.txn_stream(2_000_000, 20_000, 100)
        rules = synth.c5_rules(200)
        return (compiler.compile_app(synth.c5_query(rules)), ts, card, [card, amount, merchant], 20_000,
                lambda: (lambda r: (r[0], r[2], r[1]))(c5_expected(ts, card, amount, merchant, rules)), True, True)
    ts, k, p, v = synth.stock_stream(2_000_000, 100_000 if config == "c3" else 10_000,
                                     1000 if config == "c3" else 100)
    if config == "c3":
        from c3_check import c3_expected
        return (compiler.compile_app(synth.C3_QUERY), ts, k, [k, p, v], 100_000,
                lambda: c3_expected(ts, k, p) + (None,), False, False)
    from c2_check import c2_expected
    return (compiler.compile_app(synth.C2_QUERY), ts, k, [k, p, v], 10_000,
            lambda: c2_expected(ts, k, p, v) + (None,), False, False)


@pytest.mark.parametrize("config", ["c2", "c3", "c5"])
@pytest.mark.parametrize("world", [2, 4])
def test_sharded_step_virtual_ranks_equal_single_stream(world, config):
    import torch
    from siddhi_amd import shard
    from siddhi_amd.device_run import DeviceRunner
    ca, ts, k, cols, K, expected, wq, runs = _shard_case(config)
    n = len(ts)
    b = shard.slice_bounds(n, world, align=4096)
    rid = shard.stream_run_ids(k, 4096) if runs else None
    comm = _ThreadComm(world)
    out = [None] * world
    errs = []

    def rank_main(r):
        try:
            runner = DeviceRunner(ca)

            def matcher(t, kk, cc, nk, run=None):
                res = runner.run(t, kk, cc, nk, with_query=wq, run_ids=run)
                if not wq:
                    return res
                m, s_, v, q = res
                return m, s_, torch.cat([v, q[:m].to(torch.int64).view(-1, 1)], 1)

            step = shard.KeyShardedStep(world, r, _ops(), matcher, n_out=runner.n_out + (1 if wq else 0),
                                        comm=comm.view(r))
            lo, hi = b[r], b[r + 1]
            dev = [torch.from_numpy(a[lo:hi].copy()).cuda() for a in [ts] + cols]
            d_run = torch.from_numpy(rid[lo:hi].copy()).cuda() if rid is not None else None
            seq, vals = step.run(dev[0], dev[1], dev[1:], lo, K, key_attr=0, run_ids=d_run)
            torch.cuda.synchronize()
            out[r] = (seq.cpu().numpy(), vals.cpu().numpy(), step.last)
            runner.close()
        except BaseException as e:  # noqa: BLE001
            errs.append(e)
            comm.bar.abort()

    th = [threading.Thread(target=rank_main, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    assert not errs, errs
    eseq, evals, eq = expected()
    mseq = np.concatenate([o[0] for o in out])
    mvals = np.concatenate([o[1] for o in out])
    assert all(o[2]["matches_here"] > 0 for o in out)
    assert all(o[2]["compact"] for o in out)
    assert len(mseq) == len(eseq) > 0
    assert np.array_equal(mseq, eseq)
    if wq:
        assert np.array_equal(mvals[:, -1], eq)
        mvals = mvals[:, :-1]
    assert np.array_equal(mvals[:, :evals.shape[1]], evals)
