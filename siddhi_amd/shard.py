"""Key-sharded multi-GPU path (one process per GPU, torch.distributed over RCCL).

Partitions never interact in the reference: every partition key has its own
state (core/partition/PartitionRuntimeImpl.java:346-364, PartitionStateHolder),
so ONE arrival-ordered stream is split across the ranks by key: rank r owns the
keys with mix32(key id) % world == r. Every rank ingests an arrival-contiguous
slice of the stream (global sequence numbers seq0 .. seq0 + n). A step:

  1. route   owner rank of every event of the slice; stable owner-major
             positions (shs_route) and packed records (shs_pack: the event
             columns + the global sequence number, 32 B per C2 event)
  2. shuffle one all-to-all of the records (RCCL), split sizes exchanged first
  3. match   the owner unpacks (shs_unpack; received runs are laid out by
             source rank, so arrival order holds) and runs its own matcher on
             the events of its keys (sh_run_device)
  4. return  each match row goes back to the rank whose slice holds its trigger
             event (shs_rows_home: the rows are already grouped by source
             rank), one all-to-all of (seq, values)
  5. merge   k-way merge of the owners' ordered runs by trigger sequence
             (shs_merge): rank r ends with the reference's output order for its
             slice, so the ranks' outputs concatenated are the single-process
             output.

Step 3 is the only compute; 2 and 4 are the only collectives (no collective
inside the matcher). Scaling is strong: the stream is fixed, the ranks split it.
The device kernels live in libsiddhi_hip.so (include/siddhi_shard.h); tests can
drive the same orchestration with other ops / matchers on CPU over gloo.
"""
from __future__ import annotations

import ctypes as C

import numpy as np


def mix32(x):
    """splitmix-style 32-bit finaliser (vectorised; = shs_owner's hash)."""
    x = np.asarray(x, dtype=np.uint64) & np.uint64(0xFFFFFFFF)
    x = (x ^ (x >> np.uint64(16))) * np.uint64(0x85EBCA6B) & np.uint64(0xFFFFFFFF)
    x = (x ^ (x >> np.uint64(13))) * np.uint64(0xC2B2AE35) & np.uint64(0xFFFFFFFF)
    return (x ^ (x >> np.uint64(16))).astype(np.uint32)


def shard_of(keys, world):
    return (mix32(keys) % np.uint32(world)).astype(np.int32)


def split(keys, world):
    """Index arrays (arrival order preserved) of the events each rank owns."""
    s = shard_of(keys, world)
    return [np.nonzero(s == r)[0] for r in range(world)]


def slice_bounds(n_total, world, align=1):
    """arrival-contiguous ingest slices: rank r holds [b[r], b[r+1]); align: cut
    only at multiples of it (the send() call size, so no call spans two slices)"""
    units = (n_total + align - 1) // align
    return [min(n_total, (units * r // world) * align) for r in range(world + 1)]


def stream_run_ids(keys, batch):
    """PartitionStreamReceiver runs of an arrival-ordered stream sent as
    send(Event[]) calls of `batch` events (core/partition/PartitionStreamReceiver.java:176-216:
    a run is the consecutive same-key events of one call): per event, the arrival
    index of its run's first event (uint32, non-decreasing). A key shard of the
    stream keeps these ids, so its matcher sees the runs the whole stream had
    (sh_device_run.d_run)."""
    keys = np.asarray(keys)
    n = len(keys)
    start = np.ones(n, bool)
    if n > 1:
        start[1:] = keys[1:] != keys[:-1]
    if batch > 0:
        start[::batch] = True
    idx = np.where(start, np.arange(n, dtype=np.int64), 0)
    return np.maximum.accumulate(idx).astype(np.uint32).view(np.int32)


def _width(t):
    return t.element_size()


class HipShardOps:
    """The device kernels of include/siddhi_shard.h on torch-allocated HBM."""

    def __init__(self, device):
        import torch
        from ._native import lib
        self.torch = torch
        self.device = torch.device(device)
        self.lib = lib()
        L = self.lib
        L.shs_route_scratch_bytes.argtypes = [C.c_int64, C.c_int32]
        L.shs_route_scratch_bytes.restype = C.c_int64
        L.shs_route.argtypes = [C.c_void_p, C.c_int64, C.c_int32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
        L.shs_route.restype = C.c_int
        L.shs_record_words.argtypes = [C.c_int32, C.c_void_p]
        L.shs_record_words.restype = C.c_int32
        L.shs_pack.argtypes = [C.c_void_p, C.c_int64, C.c_int32, C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p,
                               C.c_void_p]
        L.shs_pack.restype = C.c_int
        L.shs_unpack.argtypes = [C.c_void_p, C.c_int64, C.c_int32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
        L.shs_unpack.restype = C.c_int
        L.shs_record_words_compact.argtypes = [C.c_int32, C.c_void_p]
        L.shs_record_words_compact.restype = C.c_int32
        L.shs_pack_compact.argtypes = [C.c_void_p, C.c_int64, C.c_int32, C.c_void_p, C.c_void_p, C.c_void_p,
                                       C.c_void_p, C.c_void_p]
        L.shs_pack_compact.restype = C.c_int
        L.shs_unpack_compact.argtypes = [C.c_void_p, C.c_int32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int32,
                                         C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
        L.shs_unpack_compact.restype = C.c_int
        L.shs_rows_home.argtypes = [C.c_void_p, C.c_int64, C.c_uint64, C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p,
                                    C.c_void_p]
        L.shs_rows_home.restype = C.c_int
        L.shs_merge.argtypes = [C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p, C.c_int32, C.c_void_p, C.c_void_p,
                                C.c_void_p]
        L.shs_merge.restype = C.c_int
        self._scratch = None

    def _stream(self):
        return self.torch.cuda.current_stream(self.device).cuda_stream

    @staticmethod
    def _check(rc, what):
        if rc != 0:
            raise RuntimeError(f"{what} failed with status {rc}")

    def route(self, keys, world):
        torch = self.torch
        n = keys.numel()
        need = int(self.lib.shs_route_scratch_bytes(n, world))
        if self._scratch is None or self._scratch.numel() < need:
            self._scratch = torch.empty(need, dtype=torch.uint8, device=self.device)
        pos = torch.empty(max(n, 1), dtype=torch.int32, device=self.device)
        counts = (C.c_int64 * world)()
        self._check(self.lib.shs_route(keys.data_ptr(), n, world, pos.data_ptr(), self._scratch.data_ptr(),
                                       counts, self._stream()), "shs_route")
        return pos, [int(c) for c in counts]

    def record_words(self, widths):
        w = (C.c_int32 * len(widths))(*widths)
        return int(self.lib.shs_record_words(len(widths), w))

    def pack(self, pos, cols, seq0):
        torch = self.torch
        n = cols[0].numel()
        widths = [_width(c) for c in cols]
        stride = self.record_words(widths)
        rec = torch.empty(max(n * stride, 1), dtype=torch.int32, device=self.device)
        cp = (C.c_void_p * len(cols))(*[c.data_ptr() for c in cols])
        wp = (C.c_int32 * len(cols))(*widths)
        self._check(self.lib.shs_pack(pos.data_ptr(), n, len(cols), cp, wp, seq0, rec.data_ptr(), self._stream()),
                    "shs_pack")
        return rec[: n * stride], stride

    def unpack(self, rec, n, like):
        torch = self.torch
        cols = [torch.empty(n, dtype=c.dtype, device=self.device) for c in like]
        seq = torch.empty(n, dtype=torch.int64, device=self.device)
        cp = (C.c_void_p * len(cols))(*[c.data_ptr() for c in cols])
        wp = (C.c_int32 * len(cols))(*[_width(c) for c in cols])
        self._check(self.lib.shs_unpack(rec.data_ptr(), n, len(cols), cp, wp, seq.data_ptr(), self._stream()),
                    "shs_unpack")
        return cols, seq

    # compact records: column 0 (timestamps) as a 32-bit offset from the slice's
    # base, the sequence number as a 32-bit index into the source slice
    compact = True

    def pack_compact(self, pos, cols, tbase):
        torch = self.torch
        n = cols[0].numel()
        widths = [SHS_W_OFF] + [_width(c) for c in cols[1:]]
        w = (C.c_int32 * len(widths))(*widths)
        stride = int(self.lib.shs_record_words_compact(len(widths), w))
        rec = torch.empty(max(n * stride, 1), dtype=torch.int32, device=self.device)
        cp = (C.c_void_p * len(cols))(*[c.data_ptr() for c in cols])
        base = (C.c_int64 * len(cols))(*([tbase] + [0] * (len(cols) - 1)))
        self._check(self.lib.shs_pack_compact(pos.data_ptr(), n, len(cols), cp, w, base, rec.data_ptr(),
                                              self._stream()), "shs_pack_compact")
        return rec[: n * stride], stride

    def unpack_compact(self, rec, like, src_off, src_tbase, src_seq0):
        torch = self.torch
        n = src_off[-1]
        world = len(src_off) - 1
        cols = [torch.empty(max(n, 1), dtype=c.dtype, device=self.device)[:n] for c in like]
        seq = torch.empty(max(n, 1), dtype=torch.int64, device=self.device)[:n]
        widths = [SHS_W_OFF] + [_width(c) for c in like[1:]]
        nc = len(like)
        cp = (C.c_void_p * nc)(*[c.data_ptr() for c in cols])
        w = (C.c_int32 * nc)(*widths)
        offs = (C.c_int64 * (world + 1))(*src_off)
        base = (C.c_int64 * (world * nc))(*[src_tbase[r] if c == 0 else 0 for r in range(world) for c in range(nc)])
        s0 = (C.c_uint64 * world)(*src_seq0)
        self._check(self.lib.shs_unpack_compact(rec.data_ptr(), nc, cp, w, offs, world, base, s0, seq.data_ptr(),
                                                self._stream()), "shs_unpack_compact")
        return cols, seq

    def rows_home(self, oseq, m, seq_base, gseq, src_off, world):
        offs = (C.c_int64 * (world + 1))(*src_off)
        counts = (C.c_int64 * world)()
        self._check(self.lib.shs_rows_home(oseq.data_ptr(), m, seq_base, gseq.data_ptr(), offs, world, counts,
                                           self._stream()), "shs_rows_home")
        return [int(c) for c in counts]

    def merge(self, seq, vals, n_out, run_off):
        torch = self.torch
        m = run_off[-1]
        seq_out = torch.empty(max(m, 1), dtype=torch.int64, device=self.device)
        vals_out = torch.empty(max(m * n_out, 1), dtype=torch.int64, device=self.device)
        offs = (C.c_int64 * len(run_off))(*run_off)
        self._check(self.lib.shs_merge(seq.data_ptr(), vals.data_ptr(), n_out, offs, len(run_off) - 1,
                                       seq_out.data_ptr(), vals_out.data_ptr(), self._stream()), "shs_merge")
        return seq_out[:m], vals_out[: m * n_out].view(m, n_out)


SHS_W_OFF = 5  # include/siddhi_shard.h: an 8-byte column carried as a 32-bit offset


class TorchComm:
    """the step's two exchanges over torch.distributed (RCCL "nccl" on GPUs, gloo
    on CPU): all_to_all_single with per-rank split sizes"""

    def __init__(self, world, group=None):
        import torch.distributed as dist
        self.dist, self.world, self.group = dist, world, group

    def meta(self, vals, device):
        """every rank's small int64 vector (all_gather): list per rank"""
        import torch
        mine = torch.tensor(vals, dtype=torch.int64, device=device)
        out = [torch.empty_like(mine) for _ in range(self.world)]
        self.dist.all_gather(out, mine, group=self.group)
        return [[int(x) for x in o.cpu().tolist()] for o in out]

    def counts(self, counts, device):
        import torch
        send = torch.tensor(counts, dtype=torch.int64, device=device)
        recv = torch.empty(self.world, dtype=torch.int64, device=device)
        self.dist.all_to_all_single(recv, send, group=self.group)
        return [int(x) for x in recv.cpu().tolist()]

    def exchange(self, send, send_counts, recv_counts, per):
        import torch
        n = sum(recv_counts) * per
        recv = torch.empty(max(n, 1), dtype=send.dtype, device=send.device)[:n]
        self.dist.all_to_all_single(recv, send, output_split_sizes=[c * per for c in recv_counts],
                                    input_split_sizes=[c * per for c in send_counts], group=self.group)
        return recv


class BounceComm(TorchComm):
    """rehearsal of the exchanges over gloo through host memory (several ranks on one
    GPU, where RCCL refuses duplicate devices); same split semantics as TorchComm"""

    def counts(self, counts, device):
        return super().counts(counts, "cpu")

    def meta(self, vals, device):
        return super().meta(vals, "cpu")

    def exchange(self, send, send_counts, recv_counts, per):
        return super().exchange(send.cpu(), send_counts, recv_counts, per).to(send.device)


class KeyShardedStep:
    """One sharded pass on this rank (see the module docstring).

    matcher(ts, keys, cols, n_keys) -> (m, local_seq[m] ascending (event index
    into the received events), values[m, n_out]) runs on the received events.
    comm: the two all-to-all exchanges (TorchComm by default).
    """

    def __init__(self, world, rank, ops, matcher, n_out, comm=None):
        self.world, self.rank = world, rank
        self.ops, self.matcher, self.n_out = ops, matcher, n_out
        self.comm = comm if comm is not None else TorchComm(world)
        self.last = {}

    def run(self, ts, keys, cols, seq0, n_keys, key_attr=None, run_ids=None, batch=None):
        """ts / keys / cols: this rank's ingest slice (arrival order), seq0 its
        first global sequence number; key_attr: index of the attribute column
        that holds the partition key ids (then `keys` travels once); run_ids
        (optional, stream_run_ids of the slice): travel with the events and reach
        the matcher as `run=` (apps whose output order depends on the
        PartitionStreamReceiver runs, e.g. several queries in one partition).
        Returns (seq[m], values[m, n_out]) of the rows triggered by the slice's
        events, in the reference's order. batch: events per send() call; with
        run_ids the slice must start at a call boundary (a run never spans two
        ranks' slices), which is checked when batch is given."""
        if run_ids is not None and batch:
            assert seq0 % batch == 0, "run ids need ingest slices cut at send() call boundaries"
        dev = ts.device
        world = self.world
        ev = self._events(dev)
        self._mark(ev, 0)
        # compact records when every rank's slice fits 32-bit timestamp offsets:
        # every rank's first sequence number and timestamp base travel once
        compact = False
        if getattr(self.ops, "compact", False) and hasattr(self.comm, "meta") and ts.numel() > 0:
            import torch
            lo_hi = torch.stack([ts.min(), ts.max()]).cpu().tolist()
            meta = self.comm.meta([seq0, lo_hi[0], int(lo_hi[1] - lo_hi[0] < (1 << 32) - 1)], dev)
            compact = all(m[2] for m in meta)
        elif getattr(self.ops, "compact", False) and hasattr(self.comm, "meta"):
            meta = self.comm.meta([seq0, 0, 1], dev)
            compact = all(m[2] for m in meta)
        # 1. route + pack (columns: ts, [keys,] then the attribute columns[, run ids])
        pos, send_counts = self.ops.route(keys, world)
        allc = [ts] + ([] if key_attr is not None else [keys]) + list(cols) + ([run_ids] if run_ids is not None else [])
        if compact:
            rec, stride = self.ops.pack_compact(pos, allc, meta[self.rank][1])
        else:
            rec, stride = self.ops.pack(pos, allc, seq0)
        self._mark(ev, 1)
        # 2. shuffle
        recv_counts = self.comm.counts(send_counts, dev)
        rrec = self.comm.exchange(rec, send_counts, recv_counts, stride)
        n_recv = sum(recv_counts)
        self._mark(ev, 2)
        if compact:
            off = [0]
            for c in recv_counts:
                off.append(off[-1] + c)
            ucols, gseq = self.ops.unpack_compact(rrec, allc, off, [m[1] for m in meta], [m[0] for m in meta])
        else:
            ucols, gseq = self.ops.unpack(rrec, n_recv, allc)
        r_run = None
        if run_ids is not None:
            r_run, ucols = ucols[-1], ucols[:-1]
        if key_attr is not None:
            r_ts, r_cols = ucols[0], ucols[1:]
            r_keys = r_cols[key_attr]
        else:
            r_ts, r_keys, r_cols = ucols[0], ucols[1], ucols[2:]
        # 3. match on the owned keys' events
        if r_run is None:
            m, oseq, ovals = self.matcher(r_ts, r_keys, r_cols, n_keys)
        else:
            m, oseq, ovals = self.matcher(r_ts, r_keys, r_cols, n_keys, run=r_run)
        self._mark(ev, 3)
        # 4. rows back to the ranks holding their trigger events
        src_off = [0]
        for c in recv_counts:
            src_off.append(src_off[-1] + c)
        oseq = oseq[:m].contiguous()
        ovals = ovals[:m].contiguous().view(-1)
        # merge key: the trigger sequence, or with run ids the trigger's run (rows of
        # one run stay in the matcher's order, e.g. query-major inside the run, and
        # a run lives on one owner; its rows are grouped by source rank as long as
        # the ingest slices cut the stream at send() call boundaries)
        # (run ids are uint32 carried in int32 lanes: zero-extended, so slices past
        # 2^31 events keep their order)
        mkey = (r_run[oseq].to(oseq.dtype) & 0xFFFFFFFF) if r_run is not None else None
        row_counts = self.ops.rows_home(oseq, m, 0, gseq, src_off, world)
        back_counts = self.comm.counts(row_counts, dev)
        n_val = self.n_out
        if mkey is not None:
            import torch
            ovals = torch.cat([oseq.view(m, 1), ovals.view(m, self.n_out)], 1).contiguous().view(-1)
            oseq, n_val = mkey.contiguous(), self.n_out + 1
        hseq = self.comm.exchange(oseq, row_counts, back_counts, 1)
        hvals = self.comm.exchange(ovals, row_counts, back_counts, n_val)
        self._mark(ev, 4)
        # 5. k-way merge of the owners' runs by trigger sequence (or run)
        run_off = [0]
        for c in back_counts:
            run_off.append(run_off[-1] + c)
        seq, vals = self.ops.merge(hseq, hvals, n_val, run_off)
        if mkey is not None:
            seq, vals = vals[:, 0].contiguous(), vals[:, 1:].contiguous()
        self._mark(ev, 5)
        self.last = dict(sent=send_counts, received=recv_counts, matches_here=m, rows_home=run_off[-1],
                         record_bytes=4 * stride, compact=compact)
        self._ev = ev
        return seq, vals

    PHASES = ("route_pack", "exchange_out", "unpack_match", "exchange_back", "merge")

    def _events(self, dev):
        """timing marks on the launch stream (device GPUs only)"""
        if getattr(dev, "type", "cpu") != "cuda":
            return None
        import torch
        return [torch.cuda.Event(enable_timing=True) for _ in range(6)]

    @staticmethod
    def _mark(ev, i):
        if ev is not None:
            ev[i].record()

    def phase_ms(self):
        """the last step's phases in ms (route + pack, exchange out, unpack +
        match, row return, merge), from events on the launch stream"""
        ev = getattr(self, "_ev", None)
        if ev is None:
            return None
        ev[5].synchronize()
        return {k: ev[i].elapsed_time(ev[i + 1]) for i, k in enumerate(self.PHASES)}
