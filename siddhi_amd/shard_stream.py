"""Key-sharded streaming for apps with scheduler (absent) states, e.g. C4:
`(e1=Login and e2=Txn) -> not Logout for 5 sec` partitioned by user, @app:playback.

One process (rank) per GPU, each with a handle compiled from the same app. Every
rank sees every InputHandler.send(Event[]) call and pushes only the events of
the partition keys it owns (owner = mix32(key id) % world, shard.shard_of), with
their positions in the call (sh_push_batch_part): PartitionStreamReceiver.receive
(core/partition/PartitionStreamReceiver.java:176-272) routes per key, and the
call's playback clock step (InputHandler.java:85-96) and trigger sequence numbers
stay the whole call's. Keys never interact except through
Scheduler.onTimeChange (core/util/Scheduler.java:74-99):

  1. per distinct due time ONE state fires -- the first in the iteration order
     of the scheduler's state map over ALL keys (a TreeMultimap with a zero value
     comparator). The handle hands this rank's due candidates (due time, position
     in the map's order, key) to Coordinator.select, which gathers every rank's,
     keeps the earliest position per due time and returns each candidate's
     position in the global firing order;
  2. the map's order (PartitionStateHolder's HashMap<String, ...>,
     util/snapshot/state/PartitionStateHolder.java:36,131-162) depends on every
     getState / returnAllStates of every key: after each launch the handle hands
     its history records to Coordinator.history, which returns every rank's
     records of that launch, so each rank's HashMap model (sh_jmap.h) replays
     the one map's history. Launch ticks advance in lockstep on every rank (a
     rank owning none of a call's events still takes the call's steps), so the
     records' processing stamps are comparable across ranks.

Output: each row carries its position in the global processing order (launch <<
32 | position inside the launch, sh_drain_ordered); the ranks' rows merged by it
(merge_ordered) are the single-process output. The exchanges are small host
arrays (candidates: 24 B per due state; history: 16 B per getState), so they go
over a host transport: gloo (TorchGroupComm) between processes, or a barrier
(ThreadComm) between virtual ranks that share one GPU in one process.
"""
from __future__ import annotations

import ctypes as C
import threading

import numpy as np

from . import abi
from .shard import shard_of


class TorchGroupComm:
    """all_gather of 1-D int64 arrays over torch.distributed (gloo: host memory)"""

    def __init__(self, group=None):
        import torch.distributed as dist
        self.dist, self.group = dist, group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.seconds = 0.0   # wall time inside all_gather (the coordination cost)
        self.calls = 0

    def all_gather(self, arr):
        import time
        t0 = time.perf_counter()
        try:
            return self._all_gather(arr)
        finally:
            self.seconds += time.perf_counter() - t0
            self.calls += 1

    def _all_gather(self, arr):
        import torch
        arr = np.ascontiguousarray(arr, dtype=np.int64)
        n = torch.tensor([arr.size], dtype=torch.int64)
        ns = [torch.zeros(1, dtype=torch.int64) for _ in range(self.world)]
        self.dist.all_gather(ns, n, group=self.group)
        ns = [int(x.item()) for x in ns]
        m = max(ns)
        if m == 0:
            return [np.zeros(0, np.int64) for _ in ns]
        buf = torch.zeros(m, dtype=torch.int64)
        buf[:arr.size] = torch.from_numpy(arr)
        out = [torch.zeros(m, dtype=torch.int64) for _ in range(self.world)]
        self.dist.all_gather(out, buf, group=self.group)
        return [o[:k].numpy().copy() for o, k in zip(out, ns)]


class ThreadComm:
    """virtual ranks as threads of one process (each with its own handle): a
    barrier-synchronised all_gather; comm.view(r) is rank r's end"""

    def __init__(self, world):
        self.world = world
        self.slots = [None] * world
        self.bar = threading.Barrier(world)

    def view(self, rank):
        return _ThreadView(self, rank)

    def abort(self):
        """a failed rank breaks the barrier: every other rank's pending or next
        all_gather raises BrokenBarrierError (its call fails) instead of waiting"""
        self.bar.abort()


class _ThreadView:
    def __init__(self, comm, rank):
        self.c, self.rank, self.world = comm, rank, comm.world

    def all_gather(self, arr):
        c = self.c
        c.slots[self.rank] = np.ascontiguousarray(arr, dtype=np.int64).copy()
        c.bar.wait()
        out = [s.copy() for s in c.slots]
        c.bar.wait()  # every rank has read before the slots are reused
        return out

    def abort(self):
        self.c.abort()


_CAND = np.dtype([("t", np.int64), ("order", np.uint64), ("key", np.int32), ("pad", np.int32)])


def pick(parts, wall):
    """Scheduler.onTimeChange's pick over every rank's candidates (lists of _CAND
    arrays, rank order): the firing order is by (due time, map order); playback
    keeps the first state per distinct due time, wall clock every state. Returns,
    per rank, each candidate's position in the firing order (-1: not fired), and
    the number fired."""
    sizes = [len(p) for p in parts]
    if sum(sizes) == 0:
        return [np.zeros(0, np.int64) for _ in parts], 0
    allc = np.concatenate(parts)
    o = np.lexsort((allc["order"], allc["t"]))
    keep = np.ones(len(o), bool)
    if not wall:
        ts = allc["t"][o]
        keep[1:] = ts[1:] != ts[:-1]
    pos = np.full(len(allc), -1, np.int64)
    pos[o[keep]] = np.arange(int(keep.sum()), dtype=np.int64)
    out, a = [], 0
    for n in sizes:
        out.append(pos[a:a + n])
        a += n
    return out, int(keep.sum())


class Coordinator:
    """The sh_coordinator callbacks of one rank over `comm` (all_gather of int64
    arrays). Exceptions inside a callback are kept and reported as a failed call;
    the comm is aborted too (ThreadComm: the barrier breaks, so the other ranks'
    calls fail instead of waiting; gloo: the peers' collectives fail at the
    process group's timeout, `init_process_group(timeout=...)`)."""

    def _fail(self, e):
        self.error = e
        abort = getattr(self.comm, "abort", None)
        if abort is not None:
            abort()
        return 1

    def __init__(self, comm):
        self.comm = comm
        self.error = None
        self._hist = np.zeros(0, np.uint64)  # the merged history handed out last
        self._hist_p = C.POINTER(C.c_uint64)()
        self._fns = (abi.HISTORY_FN(self._history), abi.SELECT_FN(self._select), abi.MIN_TIME_FN(self._min_time))
        self._struct = abi.sh_coordinator(None, *self._fns)
        self.exchanges = 0

    def struct(self):
        return self._struct

    def _history(self, user, local, n_local, all_pp, n_all_p):
        try:
            loc = np.ctypeslib.as_array(local, (2 * n_local,)).view(np.int64).copy() if n_local else \
                np.zeros(0, np.int64)
            parts = self.comm.all_gather(loc)
            self._hist = np.ascontiguousarray(np.concatenate(parts).view(np.uint64))
            self._hist_p = self._hist.ctypes.data_as(C.POINTER(C.c_uint64))
            all_pp[0] = self._hist_p
            n_all_p[0] = len(self._hist) // 2
            self.exchanges += 1
            return 0
        except Exception as e:  # noqa: BLE001 (reported to the handle as a failure)
            return self._fail(e)

    def _select(self, user, wall, cand, n_local, pos_p, n_fire_p):
        try:
            loc = np.zeros(n_local, _CAND)
            if n_local:
                loc[:] = np.ctypeslib.as_array(C.cast(cand, C.POINTER(C.c_uint8)),
                                               (n_local * _CAND.itemsize,)).view(_CAND)
            parts = self.comm.all_gather(loc.view(np.int64))
            parts = [p.view(_CAND) for p in parts]
            pos, n_fire = pick(parts, bool(wall))
            mine = pos[self.comm.rank]
            for i in range(n_local):
                pos_p[i] = int(mine[i])
            n_fire_p[0] = n_fire
            self.exchanges += 1
            return 0
        except Exception as e:  # noqa: BLE001
            return self._fail(e)

    def _min_time(self, user, local, out_p):
        try:
            parts = self.comm.all_gather(np.array([local], np.int64))
            out_p[0] = int(min(int(p[0]) for p in parts))
            return 0
        except Exception as e:  # noqa: BLE001
            return self._fail(e)


class ShardedStreamEngine:
    """One rank of a key-sharded streaming app: the engine protocol
    (start / send / advance_time / drain / close) over an engine with
    set_coordinator / send_part / drain(ordered=True) (the product HipEngine, or
    the CPU build of its kernel logic in tests). send() takes the WHOLE call and
    pushes this rank's share."""

    def __init__(self, engine, comm, null_key_rank=0):
        self.eng = engine
        self.comm = comm
        self.rank, self.world = comm.rank, comm.world
        self.coord = Coordinator(comm)
        self.null_key_rank = null_key_rank
        engine.set_coordinator(self.coord)
        self.sent = 0      # events of the whole stream so far
        self.owned = 0     # of which this rank pushed
        self.calls = 0

    def owner(self, keys):
        o = shard_of(np.maximum(keys, 0), self.world)
        return np.where(keys < 0, self.null_key_rank, o)

    def set_partition_keys(self, *a, **k):
        # every rank models the one state map: it needs every key's text
        self.eng.set_partition_keys(*a, **k)

    def start(self):
        self.eng.start()

    def send(self, stream, ts, cols, nulls, keys, first_seq=None):
        n = len(ts)
        if n == 0:
            return
        if keys is not None:
            idx = np.flatnonzero(self.owner(keys) == self.rank)
        else:  # a stream without a key: null-key events, owned like keys < 0
            idx = np.arange(n) if self.rank == self.null_key_rank else np.zeros(0, np.int64)
        self.eng.send_part(stream, ts[idx], [c[idx] for c in cols],
                           [None if m is None else m[idx] for m in nulls],
                           None if keys is None else keys[idx], idx.astype(np.uint32), n, int(ts[-1]))
        self.sent += n
        self.owned += len(idx)
        self.calls += 1

    def advance_time(self, now):
        self.eng.advance_time(now)

    def drain(self):
        return self.eng.drain(ordered=True)

    def close(self):
        self.eng.close()

    def check(self):
        if self.coord.error is not None:
            raise RuntimeError(f"coordinator failed: {self.coord.error!r}")


def merge_ordered(outs):
    """the ranks' drained rows (dicts with 'order') merged into the single-process
    order: a stable sort by the processing-order tag (rows sharing a tag come
    from one key, hence one rank, already in order)"""
    from .abi import concat_drains
    cat = concat_drains(list(outs))
    o = np.argsort(cat["order"], kind="stable")
    res = {k: v[o] for k, v in cat.items() if k != "lists"}
    pos = np.empty(len(o), np.int64)
    pos[o] = np.arange(len(o))
    res["lists"] = {(int(pos[r]), c): v for (r, c), v in cat["lists"].items()}
    return res
