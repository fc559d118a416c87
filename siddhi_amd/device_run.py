"""Device-resident bulk path (sh_run_device) driven with torch-allocated HBM
buffers. torch is plumbing here (allocation, streams); the matcher runs in
libsiddhi_hip.so."""
from __future__ import annotations

import ctypes as C

import torch

from . import abi
from ._native import CompiledHandle, check, lib


class DeviceRunner:
    def __init__(self, compiled, device="cuda:0"):
        self.compiled = compiled
        self.device = torch.device(device)
        self.handle = CompiledHandle(compiled)
        self.n_out = max([1] + [len(q.outs) for q in compiled.queries])
        self._out_cap = 0

    def run(self, ts, keys, cols, n_keys, out_capacity=None, stream=None, batch_events=4096, with_query=False):
        """ts/keys/cols: device tensors (int64 / int32 / stream attribute order);
        the events arrive as send(Event[]) calls of `batch_events`.
        Returns (n_matches, out_seq[n], out_values[n, n_out]) as device tensors,
        plus out_query[n] (emitting query index) when `with_query`."""
        n = ts.numel()
        cap = out_capacity or n
        for attempt in range(2):
            if self._out_cap < cap:
                self.out_seq = torch.empty(cap, dtype=torch.int64, device=self.device)
                self.out_vals = torch.empty(cap * self.n_out, dtype=torch.int64, device=self.device)
                self.out_q = torch.empty(cap, dtype=torch.int32, device=self.device)
                self._out_cap = cap
            cp = (C.c_void_p * len(cols))(*[c.data_ptr() for c in cols])
            r = abi.sh_device_run()
            r.n = n
            r.d_ts = ts.data_ptr()
            r.d_keys = keys.data_ptr()
            r.n_keys = int(n_keys)
            r.batch_events = int(batch_events)
            r.d_cols = cp
            r.out_capacity = self._out_cap
            r.d_out_seq = self.out_seq.data_ptr()
            r.d_out_values = self.out_vals.data_ptr()
            r.stream = stream.cuda_stream if stream is not None else torch.cuda.current_stream(self.device).cuda_stream
            r.d_out_query = self.out_q.data_ptr() if with_query else None
            rc = lib().sh_run_device(self.handle.h, C.byref(r))
            if rc == abi.SH_E_MORE and attempt == 0 and int(r.out_count) > self._out_cap:
                # more matches than events: grow the output to the reported count and rerun
                cap = int(r.out_count)
                continue
            check(self.handle.h, rc)
            break
        m = int(r.out_count)
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
        """1: the last run took the bucketed window engine (sh_bucket.hip)."""
        return lib().shx_bucket_status(self.handle.h)

    def seq3_status(self):
        """1: the last run took the rise-and-fall sequence engine (k_seq3)."""
        return lib().shx_seq3_status(self.handle.h)

    def last_error(self):
        return lib().sh_last_error(self.handle.h).decode()

    def close(self):
        self.handle.close()
