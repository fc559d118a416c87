#!/usr/bin/env python3
"""Known-byte streams for FETCH_SIZE / WRITE_SIZE calibration (run under
rocprofv3 --pmc FETCH_SIZE, then --pmc WRITE_SIZE): 2 GiB per kernel (past the
256 MiB Infinity Cache), 4 and 8 bytes per lane like the matcher kernels.
The factor per width = bytes / counter; scripts/pmc_traffic.py applies it."""
import ctypes as C
import sys

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from siddhi_amd._native import lib  # noqa: E402

L = lib()
L.shx_pmc_calibrate.argtypes = [C.c_int, C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p]
L.shx_pmc_calibrate.restype = C.c_int
nbytes = 2 << 30
buf = torch.ones(nbytes // 8, dtype=torch.int64, device="cuda:0")
sink = torch.zeros(4, dtype=torch.int64, device="cuda:0")
st = torch.cuda.current_stream().cuda_stream
for kind in range(4):
    assert L.shx_pmc_calibrate(kind, buf.data_ptr(), nbytes, sink.data_ptr(), st) == 0
torch.cuda.synchronize()
print(f"calibration: 4 kernels x {nbytes} bytes (read4, read8, write4, write8)")
