"""Engine adapter over tests/nfa_host/libnfahost.so — TEST INFRASTRUCTURE.

libnfahost.so is the general engine's per-key kernel logic (siddhi_amd/csrc/sh_nfa.h,
the code k_nfa runs on the GPU) compiled for the CPU. The CPU test suite drives it
with the reference's fixtures and randomized apps and diffs it against the oracle,
so the kernel logic is checked without a GPU. The product never uses it.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

from siddhi_amd import abi
from oracle_engine import make_batch

HERE = os.path.dirname(os.path.abspath(__file__))
DIR = os.path.join(HERE, "nfa_host")
SO = os.path.join(DIR, "libnfahost.so")
_lib = None


def load():
    global _lib
    if _lib is None:
        subprocess.run(["make", "-s", "-C", DIR], check=True)
        lib = C.CDLL(SO)
        lib.nfh_create.argtypes = [C.POINTER(abi.sh_app_desc), C.c_char_p, C.c_int]
        lib.nfh_create.restype = C.c_void_p
        lib.nfh_start.argtypes = [C.c_void_p]
        lib.nfh_start.restype = C.c_int
        lib.nfh_send.argtypes = [C.c_void_p, C.POINTER(abi.sh_batch), C.c_uint64]
        lib.nfh_send.restype = C.c_int
        lib.nfh_advance_time.argtypes = [C.c_void_p, C.c_int64]
        lib.nfh_advance_time.restype = C.c_int
        lib.nfh_out_count.argtypes = [C.c_void_p]
        lib.nfh_out_count.restype = C.c_int64
        lib.nfh_out_read.argtypes = [C.c_void_p, C.c_int64, C.c_int64, C.c_void_p, C.c_void_p,
                                     C.c_void_p, C.c_void_p, C.c_void_p, C.c_int32]
        lib.nfh_out_read.restype = C.c_int
        lib.nfh_last_error.argtypes = [C.c_void_p]
        lib.nfh_last_error.restype = C.c_char_p
        lib.nfh_set_partition_keys.argtypes = [C.c_void_p, C.c_int32, C.c_int32, C.c_void_p, C.c_void_p]
        lib.nfh_set_partition_keys.restype = C.c_int
        lib.nfh_send_part.argtypes = [C.c_void_p, C.POINTER(abi.sh_batch), C.c_uint64, C.c_void_p, C.c_int64,
                                      C.c_int64]
        lib.nfh_send_part.restype = C.c_int
        lib.nfh_set_coordinator.argtypes = [C.c_void_p, C.POINTER(abi.sh_coordinator)]
        lib.nfh_set_coordinator.restype = C.c_int
        lib.nfh_list_get.argtypes = [C.c_void_p, C.c_int64, C.c_int64, C.c_void_p, C.c_void_p]
        lib.nfh_list_get.restype = C.c_int64
        lib.nfh_out_order.argtypes = [C.c_void_p, C.c_int64, C.c_int64, C.c_void_p]
        lib.nfh_out_order.restype = C.c_int
        lib.nfh_destroy.argtypes = [C.c_void_p]
        lib.nfh_destroy.restype = None
        _lib = lib
    return _lib


class NfaUnsupported(Exception):
    pass


class NfaHostEngine:
    def __init__(self, compiled):
        self.lib = load()
        self.compiled = compiled
        self.desc = compiled.descriptor()
        err = C.create_string_buffer(512)
        self.h = self.lib.nfh_create(C.byref(self.desc), err, 512)
        if not self.h:
            raise NfaUnsupported(err.value.decode())
        self.n_out = max([len(q.outs) for q in compiled.queries] + [1])
        self.read = 0
        self.seq = 0  # next input sequence number (send_part)

    def start(self):
        self._check(self.lib.nfh_start(self.h))

    def _check(self, rc):
        if rc != 0:
            raise RuntimeError(f"nfa_host rc={rc}: {self.lib.nfh_last_error(self.h).decode()}")

    def send(self, stream, tsa, cols, nulls, keys, first_seq):
        tsa = np.ascontiguousarray(tsa, dtype=np.int64)
        b, keep = make_batch(stream, tsa, cols, nulls, keys)
        self._check(self.lib.nfh_send(self.h, C.byref(b), first_seq))

    def set_coordinator(self, coord):
        self._coord = coord
        self._check(self.lib.nfh_set_coordinator(self.h, C.byref(coord.struct())))

    def send_part(self, stream, tsa, cols, nulls, keys, index, call_n, call_last, first_seq=None):
        tsa = np.ascontiguousarray(tsa, dtype=np.int64)
        index = np.ascontiguousarray(index, dtype=np.uint32)
        cs = [np.ascontiguousarray(c) for c in cols]
        ka = None if keys is None else np.ascontiguousarray(keys, dtype=np.int32)
        b, keep = make_batch(stream, tsa, cs, nulls, ka)
        self._check(self.lib.nfh_send_part(self.h, C.byref(b), self.seq if first_seq is None else first_seq,
                                           index.ctypes.data if len(index) else None, int(call_n), int(call_last)))
        self.seq += int(call_n)

    def set_partition_keys(self, first, strings=None, utf16=None, offsets=None):
        from siddhi_amd.javastr import pack_utf16
        if utf16 is None:
            utf16, offsets = pack_utf16(strings)
        self.lib.nfh_set_partition_keys(self.h, int(first), int(len(offsets) - 1), utf16.ctypes.data,
                                        offsets.ctypes.data)

    def advance_time(self, now):
        self._check(self.lib.nfh_advance_time(self.h, int(now)))

    def drain(self, ordered=False):
        total = self.lib.nfh_out_count(self.h)
        n = total - self.read
        q = np.zeros(n, np.int32)
        seq = np.zeros(n, np.uint64)
        ts = np.zeros(n, np.int64)
        vals = np.zeros((n, self.n_out), np.int64)
        nls = np.zeros((n, self.n_out), np.uint8)
        if n:
            self.lib.nfh_out_read(self.h, self.read, n, q.ctypes.data, seq.ctypes.data, ts.ctypes.data,
                                  vals.ctypes.data, nls.ctypes.data, self.n_out)
        out = dict(query=q, seq=seq, ts=ts, values=vals, nulls=nls, group=np.zeros(n, np.int32))
        if ordered:
            order = np.zeros(n, np.uint64)
            if n:
                self._check(self.lib.nfh_out_order(self.h, self.read, n, order.ctypes.data))
            out["order"] = order
        self.read = total
        return abi.resolve_lists(out, abi.object_columns(self.compiled), abi.list_getter(self.lib.nfh_list_get, self.h))

    def close(self):
        if self.h:
            self.lib.nfh_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
