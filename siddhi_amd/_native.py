"""Product engine: ctypes binding of the in-tree libsiddhi_hip.so (C-ABI).

Fails loudly: importing this module raises ImportError when the extension is
missing, and every processing call raises when the HIP runtime reports no
device (the matcher has no CPU fallback).
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

from . import abi

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libsiddhi_hip.so")

if not os.path.exists(LIB_PATH):
    raise ImportError(f"libsiddhi_hip.so is not built ({LIB_PATH}); run `python -m siddhi_amd.build` "
                      "or __graft_entry__.build()")

_lib = abi.bind_product(C.CDLL(LIB_PATH))


def lib():
    return _lib


class HipError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"{abi.STATUS_NAMES.get(code, code)}: {msg}")
        self.code = code


def check(h, rc):
    if rc not in (abi.SH_OK, abi.SH_E_MORE):
        msg = _lib.sh_last_error(h).decode() if h else ""
        raise HipError(rc, msg)
    return rc


class CompiledHandle:
    """RAII wrapper of sh_handle*."""

    def __init__(self, compiled):
        self.compiled = compiled
        self.desc = compiled.descriptor()
        h = C.c_void_p()
        rc = _lib.sh_compile(C.byref(self.desc), C.byref(h))
        self.h = h
        if rc != abi.SH_OK:
            msg = _lib.sh_last_error(h).decode() if h.value else ""
            if h.value:
                _lib.sh_destroy(h)
                self.h = None
            raise HipError(rc, msg)

    def close(self):
        if self.h:
            _lib.sh_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class HipEngine:
    """Engine protocol (start/send/advance_time/drain/close) over libsiddhi_hip.so."""

    def __init__(self, compiled):
        self.handle = CompiledHandle(compiled)
        self.h = self.handle.h
        self.n_out = max([len(q.outs) for q in compiled.queries] + [1])
        self.obj_cols = abi.object_columns(compiled)

    def start(self):
        check(self.h, _lib.sh_start(self.h))

    def send(self, stream, tsa, cols, nulls, keys, first_seq):
        tsa = np.ascontiguousarray(tsa, dtype=np.int64)
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
        check(self.h, _lib.sh_push_batch(self.h, C.byref(b)))

    def set_coordinator(self, coord):
        """make this handle one rank of a key-sharded group (shard_stream.Coordinator)"""
        self._coord = coord  # the callbacks must outlive the handle's use of them
        check(self.h, _lib.sh_set_coordinator(self.h, C.byref(coord.struct())))

    def send_part(self, stream, tsa, cols, nulls, keys, index, call_n, call_last):
        """this rank's events of one send() call: index = their positions in the
        call (uint32, ascending), call_n its size, call_last its last timestamp"""
        tsa = np.ascontiguousarray(tsa, dtype=np.int64)
        index = np.ascontiguousarray(index, dtype=np.uint32)
        cols = [np.ascontiguousarray(c) for c in cols]
        cp = (C.c_void_p * max(1, len(cols)))(*[c.ctypes.data for c in cols])
        npp = (C.c_void_p * max(1, len(cols)))(*[(m.ctypes.data if m is not None else None) for m in nulls])
        b = abi.sh_batch()
        b.stream = stream
        b.on_device = 0
        b.n = len(tsa)
        b.ts = tsa.ctypes.data if len(tsa) else None
        ka = np.ascontiguousarray(keys, dtype=np.int32) if keys is not None else None
        b.keys = ka.ctypes.data if ka is not None and len(tsa) else None
        b.cols = cp
        b.nulls = npp if any(m is not None for m in nulls) else None
        check(self.h, _lib.sh_push_batch_part(self.h, C.byref(b), index.ctypes.data if len(index) else None,
                                              int(call_n), int(call_last)))

    def set_partition_keys(self, first, strings=None, utf16=None, offsets=None):
        """attr.toString() of key ids first.. (a list of str, or packed UTF-16 + offsets)"""
        from .javastr import pack_utf16
        if utf16 is None:
            utf16, offsets = pack_utf16(strings)
        n = len(offsets) - 1
        check(self.h, _lib.sh_set_partition_keys(self.h, int(first), int(n), utf16.ctypes.data, offsets.ctypes.data))

    def advance_time(self, now):
        check(self.h, _lib.sh_advance_time(self.h, int(now)))

    HOST_PHASES = ("push", "timers", "process", "history", "place", "drain", "hist_copy", "hist_apply",
                   "hist_rank", "hist_records", "sync_wait", "pull")

    def host_profile(self):
        """SH_HOST_PROF phase clocks of this handle: {phase: (ms, count)} (zeros
        unless SH_HOST_PROF was set when the calls ran)"""
        k = len(self.HOST_PHASES)
        ms = (C.c_double * k)()
        cnt = (C.c_int64 * k)()
        _lib.shx_host_profile(self.h, ms, cnt, k)
        return {name: (float(ms[i]), int(cnt[i])) for i, name in enumerate(self.HOST_PHASES)}

    def snapshot(self) -> bytes:
        """the matcher state image (sh_snapshot)"""
        size = C.c_int64(0)
        rc = _lib.sh_snapshot(self.h, None, 0, C.byref(size))
        if rc != abi.SH_E_MORE:
            check(self.h, rc)
        buf = C.create_string_buffer(max(1, size.value))
        check(self.h, _lib.sh_snapshot(self.h, buf, size.value, C.byref(size)))
        return buf.raw[: size.value]

    def restore(self, image: bytes):
        """load an image taken from an engine of the same app (sh_restore)"""
        check(self.h, _lib.sh_restore(self.h, image, len(image)))

    def drain(self, ordered=False):
        """ordered: also each row's position in the global processing order
        (key-sharded handles; sh_drain_ordered)"""
        n = _lib.sh_pending(self.h)
        if n < 0:
            check(self.h, int(n))
        q = np.zeros(n, np.int32)
        seq = np.zeros(n, np.uint64)
        ts = np.zeros(n, np.int64)
        vals = np.zeros((n, self.n_out), np.int64)
        nls = np.zeros((n, self.n_out), np.uint8)
        order = np.zeros(n, np.uint64)
        if n:
            mb = abi.sh_match_buf()
            mb.capacity = n
            mb.query = q.ctypes.data_as(C.POINTER(C.c_int32))
            mb.trigger_seq = seq.ctypes.data_as(C.POINTER(C.c_uint64))
            mb.ts = ts.ctypes.data_as(C.POINTER(C.c_int64))
            mb.values = vals.ctypes.data_as(C.POINTER(C.c_int64))
            mb.nulls = nls.ctypes.data_as(C.POINTER(C.c_uint8))
            mb.n_out = self.n_out
            if ordered:
                check(self.h, _lib.sh_drain_ordered(self.h, C.byref(mb), order.ctypes.data))
            else:
                check(self.h, _lib.sh_drain(self.h, C.byref(mb)))
        # one callback chunk per (send, query): the device path keeps arrival
        # order; chunking of callbacks is cosmetic
        grp = np.zeros(n, np.int32)
        out = dict(query=q, seq=seq, ts=ts, values=vals, nulls=nls, group=grp)
        if ordered:
            out["order"] = order
        # List values (multi-value selects) are read before the next drain
        return abi.resolve_lists(out, self.obj_cols, abi.list_getter(_lib.sh_list_get, self.h))

    def close(self):
        self.handle.close()
