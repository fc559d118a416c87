"""Device-resident bulk path (sh_run_device) driven with torch-allocated HBM
buffers. torch is plumbing here (allocation, streams); the matcher runs in
libsiddhi_hip.so."""
from __future__ import annotations

import ctypes as C

import numpy as np
import torch

from . import abi
from . import compiler as cp
from ._native import CompiledHandle, check, lib


_TORCH = {cp.LONG: torch.int64, cp.DOUBLE: torch.float64, cp.INT: torch.int32, cp.STRING: torch.int32,
          cp.FLOAT: torch.float32, cp.BOOL: torch.uint8}


def columns_to_raw(cols, types):
    """typed output columns (numpy) -> the raw 8-byte row values of d_out_values
    (sh_vm.h load_attr: float bits zero-extended, int / string id sign-extended)"""
    out = np.empty((len(cols[0]) if cols else 0, len(cols)), dtype=np.int64)
    for o, (c, t) in enumerate(zip(cols, types)):
        if t == cp.FLOAT:
            out[:, o] = c.view(np.uint32).astype(np.int64)
        elif t == cp.DOUBLE:
            out[:, o] = c.view(np.int64)
        else:
            out[:, o] = c.astype(np.int64)
    return out


def packed_to_raw(rows, types, offsets, row_bytes):
    """SH_OUT_PACKED rows (numpy uint8, m x row_bytes) -> (trigger_seq, the raw
    8-byte row values of d_out_values)"""
    rows = np.ascontiguousarray(rows).reshape(-1, row_bytes)
    seq = rows[:, 0:8].copy().view(np.uint64).reshape(-1)
    cols = []
    for t, off in zip(types, offsets):
        w = {cp.LONG: 8, cp.DOUBLE: 8, cp.BOOL: 4}.get(t, 4)
        c = rows[:, off:off + w].copy()
        if t == cp.LONG:
            cols.append(c.view(np.int64).reshape(-1))
        elif t == cp.DOUBLE:
            cols.append(c.view(np.float64).reshape(-1))
        elif t == cp.FLOAT:
            cols.append(c.view(np.float32).reshape(-1))
        elif t == cp.BOOL:
            cols.append(c.view(np.uint32).reshape(-1).astype(np.uint8))
        else:
            cols.append(c.view(np.int32).reshape(-1))
    return seq, columns_to_raw(cols, types)


class DeviceRunner:
    def __init__(self, compiled, device="cuda:0"):
        self.compiled = compiled
        self.device = torch.device(device)
        self.handle = CompiledHandle(compiled)
        self.n_out = max([1] + [len(q.outs) for q in compiled.queries])
        self.out_types = list(compiled.queries[0].out_types) if compiled.queries else []
        self._out_cap = 0
        self._col_cap = 0

    def packed_layout(self):
        """(byte offset of each select value, row bytes) of the SH_OUT_PACKED rows"""
        offs = (C.c_int32 * 16)()
        n, rb = C.c_int32(), C.c_int32()
        check(self.handle.h, lib().sh_packed_row_layout(self.handle.h, offs, 16, C.byref(n), C.byref(rb)))
        return [offs[i] for i in range(n.value)], rb.value

    def run(self, ts, keys, cols, n_keys, out_capacity=None, stream=None, batch_events=4096, with_query=False,
            columns=False, run_ids=None, packed=False):
        """ts/keys/cols: device tensors (int64 / int32 / stream attribute order);
        the events arrive as send(Event[]) calls of `batch_events`.
        run_ids (optional int32/uint32 device tensor): the PartitionStreamReceiver
        run of every event (sh_device_run.d_run), for a key shard of a stream.
        Returns (n_matches, out_seq[n], out_values[n, n_out]) as device tensors,
        plus out_query[n] (emitting query index) when `with_query`. With
        `columns`, out_values is a list of typed columns (sh_device_run.d_out_cols:
        natural width per select attribute) instead of the raw 8-byte rows. With
        `packed`, the SH_OUT_PACKED rows: (n_matches, rows[n, row_bytes] uint8)
        (plus out_query), decoded by packed_to_raw with packed_layout()."""
        n = ts.numel()
        cap = out_capacity or n
        if packed:
            _, rb = self.packed_layout()
        for attempt in range(2):
            if packed:
                if getattr(self, "_row_cap", 0) < cap or getattr(self, "_row_bytes", 0) != rb:
                    self.out_rows = torch.empty(cap * rb, dtype=torch.uint8, device=self.device)
                    self._row_cap, self._row_bytes = cap, rb
                if not hasattr(self, "out_q") or self.out_q.numel() < cap:
                    self.out_q = torch.empty(cap, dtype=torch.int32, device=self.device)
                r = abi.sh_device_run()
                r.version = abi.SH_DEVICE_RUN_V2
                r.out_layout = abi.SH_OUT_PACKED
                r.d_run = run_ids.data_ptr() if run_ids is not None else None
                r.n = n
                r.d_ts = ts.data_ptr()
                r.d_keys = keys.data_ptr()
                r.n_keys = int(n_keys)
                r.batch_events = int(batch_events)
                r.d_cols = (C.c_void_p * len(cols))(*[c.data_ptr() for c in cols])
                r.out_capacity = self._row_cap
                r.d_out_seq = None
                r.d_out_values = self.out_rows.data_ptr()
                r.stream = stream.cuda_stream if stream is not None else torch.cuda.current_stream(self.device).cuda_stream
                r.d_out_query = self.out_q.data_ptr() if with_query else None
                rc = lib().sh_run_device_v2(self.handle.h, C.byref(r))
                if rc == abi.SH_E_MORE and attempt == 0 and int(r.out_count) > self._row_cap:
                    cap = int(r.out_count)
                    continue
                check(self.handle.h, rc)
                m = int(r.out_count)
                res = (m, self.out_rows[: m * rb].view(m, rb))
                return res + (self.out_q[:m],) if with_query else res
            if self._out_cap < cap:
                self.out_seq = torch.empty(cap, dtype=torch.int64, device=self.device)
                self.out_vals = (torch.empty(0, dtype=torch.int64, device=self.device) if columns else
                                 torch.empty(cap * self.n_out, dtype=torch.int64, device=self.device))
                self.out_q = torch.empty(cap, dtype=torch.int32, device=self.device)
                self._out_cap = cap
            if columns and (self._col_cap < self._out_cap or not hasattr(self, "out_cols")):
                self.out_cols = [torch.empty(self._out_cap, dtype=_TORCH[t], device=self.device)
                                 for t in self.out_types]
                self._col_cap = self._out_cap
            if not columns and self.out_vals.numel() < self._out_cap * self.n_out:
                self.out_vals = torch.empty(self._out_cap * self.n_out, dtype=torch.int64, device=self.device)
            cp = (C.c_void_p * len(cols))(*[c.data_ptr() for c in cols])
            r = abi.sh_device_run()
            r.version = abi.SH_DEVICE_RUN_V2
            r.d_run = run_ids.data_ptr() if run_ids is not None else None
            r.n = n
            r.d_ts = ts.data_ptr()
            r.d_keys = keys.data_ptr()
            r.n_keys = int(n_keys)
            r.batch_events = int(batch_events)
            r.d_cols = cp
            r.out_capacity = self._out_cap
            r.d_out_seq = self.out_seq.data_ptr()
            r.d_out_values = None if columns else self.out_vals.data_ptr()
            if columns:
                ocp = (C.c_void_p * len(self.out_cols))(*[c.data_ptr() for c in self.out_cols])
                r.d_out_cols = ocp
            r.stream = stream.cuda_stream if stream is not None else torch.cuda.current_stream(self.device).cuda_stream
            r.d_out_query = self.out_q.data_ptr() if with_query else None
            rc = lib().sh_run_device_v2(self.handle.h, C.byref(r))
            if rc == abi.SH_E_MORE and attempt == 0 and int(r.out_count) > self._out_cap:
                # more matches than events: grow the output to the reported count and rerun
                cap = int(r.out_count)
                continue
            check(self.handle.h, rc)
            break
        m = int(r.out_count)
        if columns:
            res = (m, self.out_seq[:m], [c[:m] for c in self.out_cols])
            return res + (self.out_q[:m],) if with_query else res
        res = (m, self.out_seq[:m], self.out_vals[: m * self.n_out].view(m, self.n_out))
        return res + (self.out_q[:m],) if with_query else res

    def kernel_times(self):
        t = abi.sh_kernel_times()
        lib().sh_last_kernel_times(self.handle.h, C.byref(t))
        return dict(segment_ms=t.segment_ms, advance_ms=t.advance_ms, emit_ms=t.emit_ms, total_ms=t.total_ms)

    def jit_status(self):
        """1: hipRTC-specialised window kernels ran, -1: ahead-of-time kernels, 0: not tried."""
        return lib().shx_jit_status(self.handle.h)

    def bucket_status(self):
        """1: the last run took the bucketed window engine (sh_bucket.hip +
        shb_match), 0: another engine."""
        return lib().shx_bucket_status(self.handle.h)

    def seq3_status(self):
        """1: the last run took the rise-and-fall sequence engine (k_seq3)."""
        return lib().shx_seq3_status(self.handle.h)

    def rules_status(self):
        """1: the last rule-set run took the sparse-partial path (no key segment),
        0: the key-segment path (or not a rule set)."""
        return lib().shx_rules_status(self.handle.h)

    def agg_status(self):
        """aggregators of the last run: 1 post-pass over a fast engine's rows
        (sh_agg.hip), 2 not exact in parallel (a sequential engine ran), 0 none."""
        return lib().shx_agg_status(self.handle.h)

    def last_error(self):
        return lib().sh_last_error(self.handle.h).decode()

    def close(self):
        self.handle.close()
