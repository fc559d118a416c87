"""Engine adapter over the CPU ORACLE (oracle/librefcpu.so) — test infrastructure.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this,
as the checker. It speaks the same engine protocol as siddhi_amd._native.HipEngine.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

from siddhi_amd import abi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
ORACLE_SO = os.path.join(ORACLE_DIR, "librefcpu.so")
_lib = None


def build_oracle():
    subprocess.run(["make", "-s", "-C", ORACLE_DIR], check=True)


def load_oracle():
    global _lib
    if _lib is None:
        if not os.path.exists(ORACLE_SO):
            build_oracle()
        _lib = abi.bind_oracle(C.CDLL(ORACLE_SO))
    return _lib


def make_batch(stream, tsa, cols, nulls, keys):
    """sh_batch over host numpy arrays (arrays must outlive the call)."""
    n = len(tsa)
    cp = (C.c_void_p * max(1, len(cols)))(*[c.ctypes.data for c in cols])
    npp = (C.c_void_p * max(1, len(cols)))(*[(m.ctypes.data if m is not None else None) for m in nulls])
    b = abi.sh_batch()
    b.stream = stream
    b.on_device = 0
    b.n = n
    b.ts = tsa.ctypes.data
    b.keys = keys.ctypes.data if keys is not None else None
    b.cols = cp
    b.nulls = npp if any(m is not None for m in nulls) else None
    return b, (cp, npp)


class OracleEngine:
    def __init__(self, compiled):
        self.lib = load_oracle()
        self.compiled = compiled
        self.desc = compiled.descriptor()
        err = C.create_string_buffer(512)
        self.h = self.lib.ref_create(C.byref(self.desc), err, 512)
        if not self.h:
            raise RuntimeError("oracle: " + err.value.decode())
        self.n_out = max([len(q.outs) for q in compiled.queries] + [1])
        self.read = 0

    def start(self):
        self.lib.ref_start(self.h)

    def send(self, stream, tsa, cols, nulls, keys, first_seq):
        tsa = np.ascontiguousarray(tsa, dtype=np.int64)
        b, keep = make_batch(stream, tsa, cols, nulls, keys)
        rc = self.lib.ref_send(self.h, C.byref(b), first_seq)
        if rc != 0:
            raise RuntimeError(f"ref_send -> {rc}")

    def set_partition_keys(self, first, strings=None, utf16=None, offsets=None):
        from siddhi_amd.javastr import pack_utf16
        if utf16 is None:
            utf16, offsets = pack_utf16(strings)
        n = len(offsets) - 1
        rc = self.lib.ref_set_partition_keys(self.h, int(first), int(n), utf16.ctypes.data, offsets.ctypes.data)
        if rc != 0:
            raise RuntimeError(f"ref_set_partition_keys -> {rc}")

    def advance_time(self, now):
        self.lib.ref_advance_time(self.h, int(now))

    def drain(self):
        total = self.lib.ref_out_count(self.h)
        n = total - self.read
        q = np.zeros(n, np.int32)
        seq = np.zeros(n, np.uint64)
        ts = np.zeros(n, np.int64)
        vals = np.zeros((n, self.n_out), np.int64)
        nls = np.zeros((n, self.n_out), np.uint8)
        grp = np.zeros(n, np.int32)
        if n:
            self.lib.ref_out_read(self.h, self.read, n, q.ctypes.data, seq.ctypes.data, ts.ctypes.data,
                                  vals.ctypes.data, nls.ctypes.data, self.n_out, grp.ctypes.data)
        self.read = total
        out = dict(query=q, seq=seq, ts=ts, values=vals, nulls=nls, group=grp)
        return abi.resolve_lists(out, abi.object_columns(self.compiled), abi.list_getter(self.lib.ref_list_get, self.h))

    def close(self):
        if self.h:
            self.lib.ref_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def run_stock_oracle(compiled, ts, keys, price, vol, batch=4096, partitioned=True):
    """Drive the oracle with send(Event[]) calls of `batch` events over the
    StockStream columns; returns (seq, ts, values[n, n_out], nulls) of all matches."""
    eng = OracleEngine(compiled)
    eng.start()
    n = len(ts)
    sym = keys.astype(np.int32)
    for b0 in range(0, n, batch):
        b1 = min(n, b0 + batch)
        cols = [np.ascontiguousarray(sym[b0:b1]), np.ascontiguousarray(price[b0:b1]),
                np.ascontiguousarray(vol[b0:b1])]
        eng.send(0, np.ascontiguousarray(ts[b0:b1]), cols, [None, None, None],
                 np.ascontiguousarray(sym[b0:b1]) if partitioned else None, b0)
    out = eng.drain()
    eng.close()
    return out["seq"], out["ts"], out["values"], out["nulls"]


def run_columns_oracle(compiled, ts, cols, keys, batch=4096):
    """Single-stream app: drive the oracle with send(Event[]) batches over the
    given arrival-order columns; returns (seq, ts, values, nulls)."""
    eng = OracleEngine(compiled)
    eng.start()
    n = len(ts)
    for b0 in range(0, n, batch):
        b1 = min(n, b0 + batch)
        eng.send(0, np.ascontiguousarray(ts[b0:b1]), [np.ascontiguousarray(c[b0:b1]) for c in cols],
                 [None] * len(cols), np.ascontiguousarray(keys[b0:b1]) if keys is not None else None, b0)
    out = eng.drain()
    eng.close()
    return out["seq"], out["ts"], out["values"], out["nulls"]
