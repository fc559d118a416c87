"""C-ABI checks that need no GPU: the library loads, exports every symbol
include/siddhi_hip.h declares, lowers supported apps and refuses the rest."""
import ctypes as C
import os
import re
import subprocess

import pytest

from siddhi_amd import abi, build, compiler, synth

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def lib():
    path = build.build()
    return abi.bind_product(C.CDLL(path))


def test_shard_header_symbols_are_exported(lib):
    """include/siddhi_shard.h (key-sharded multi-GPU path) is implemented by the
    same library"""
    hdr = open(os.path.join(ROOT, "include", "siddhi_shard.h")).read()
    declared = set(re.findall(r"\b(shs_[a-z_]+)\s*\(", hdr))
    assert len(declared) >= 8
    out = subprocess.run(["nm", "-D", "--defined-only", build.OUT], capture_output=True, text=True).stdout
    assert declared <= set(re.findall(r" T (shs_[a-z_]+)", out))


def test_shard_owner_matches_python_hash(lib):
    import ctypes
    import numpy as np
    from siddhi_amd import shard
    lib.shs_owner.argtypes = [ctypes.c_int32, ctypes.c_int32]
    lib.shs_owner.restype = ctypes.c_int32
    keys = np.arange(0, 50_000, 7, dtype=np.int32)
    for world in (1, 2, 3, 8):
        assert [lib.shs_owner(int(k), world) for k in keys] == list(shard.shard_of(keys, world))


def test_header_declares_exactly_the_exported_symbols(lib):
    hdr = open(os.path.join(ROOT, "include", "siddhi_hip.h")).read()
    declared = set(re.findall(r"\b(sh_[a-z0-9_]+)\s*\(", hdr))
    assert declared == set(abi.EXPORTED)
    out = subprocess.run(["nm", "-D", "--defined-only", build.OUT], capture_output=True, text=True).stdout
    exported = set(re.findall(r" T (sh_[a-z0-9_]+)", out))
    assert declared <= exported


def test_device_run_struct_keeps_the_v1_layout():
    """sh_device_run: the V1 struct (round 2 callers) is the first 96 bytes with
    d_out_cols at 88; the V2 fields follow it (sh_run_device reads the prefix only,
    sh_run_device_v2 the whole struct)"""
    R = abi.sh_device_run
    assert R.d_out_query.offset == 80 and R.d_out_cols.offset == 88
    assert R.version.offset == 96 and R.d_run.offset == 104 and C.sizeof(R) == 112
    hdr = open(os.path.join(ROOT, "include", "siddhi_hip.h")).read()
    assert "#define SH_DEVICE_RUN_V1_BYTES 96" in hdr


def _compile(lib, text):
    ca = compiler.compile_app(text)
    d = ca.descriptor()
    h = C.c_void_p()
    rc = lib.sh_compile(C.byref(d), C.byref(h))
    return rc, h, ca


def test_c2_query_lowers(lib):
    rc, h, _ = _compile(lib, synth.C2_QUERY)
    assert rc == abi.SH_OK, lib.sh_last_error(h)
    lib.sh_destroy(h)


def test_packed_row_layout(lib):
    """SH_OUT_PACKED: trigger_seq 8 B, then symbol (string id) 4, p1 4, p2 4, a pad to
    align v2 (long) 8: one 32-byte row for the C2 select"""
    rc, h, _ = _compile(lib, synth.C2_QUERY)
    assert rc == abi.SH_OK, lib.sh_last_error(h)
    offs = (C.c_int32 * 16)()
    n, rb = C.c_int32(), C.c_int32()
    assert lib.sh_packed_row_layout(h, offs, 16, C.byref(n), C.byref(rb)) == abi.SH_OK
    assert (n.value, rb.value, list(offs[:4])) == (4, 32, [8, 12, 16, 24])
    assert abi.sh_device_run.out_layout.offset == 100
    lib.sh_destroy(h)


def test_packed_rows_decode():
    """packed_to_raw reads what the layout says (host-side decoder, no device)"""
    import numpy as np
    from siddhi_amd.device_run import packed_to_raw
    rows = np.zeros((2, 32), np.uint8)
    rows[:, 0:8] = np.array([7, 9], np.uint64).view(np.uint8).reshape(2, 8)
    rows[:, 8:12] = np.array([3, -1], np.int32).view(np.uint8).reshape(2, 4)
    rows[:, 12:16] = np.array([1.5, 2.5], np.float32).view(np.uint8).reshape(2, 4)
    rows[:, 16:20] = np.array([0.25, -4.0], np.float32).view(np.uint8).reshape(2, 4)
    rows[:, 24:32] = np.array([2**40, -5], np.int64).view(np.uint8).reshape(2, 8)
    seq, raw = packed_to_raw(rows, [compiler.STRING, compiler.FLOAT, compiler.FLOAT, compiler.LONG], [8, 12, 16, 24], 32)
    assert seq.tolist() == [7, 9]
    assert raw[:, 0].tolist() == [3, -1] and raw[:, 3].tolist() == [2**40, -5]
    assert raw[0, 1] == np.array([1.5], np.float32).view(np.uint32)[0]


@pytest.mark.parametrize("text", [
    # C3 (sequence + Kleene count) and a logical pattern: the general engine
    "define stream S (a int); from every e1=S, e2=S[a>e1.a]+, e3=S select e1.a as a insert into O;",
    "define stream S (a int); define stream T (a int); from e1=S and e2=T -> e3=S select e3.a as a insert into O;",
    # C4: logical + absent, playback, partitioned
    "@app:playback define stream L (u string, ip int); define stream T (u string, amt float); "
    "define stream O (u string); partition with (u of L, u of T, u of O) begin "
    "from (e1=L and e2=T) -> not O for 5 sec select e1.u as u, e2.amt as a insert into A; end;",
    "define stream S (a int); define stream T (a int); from e1=S and not T for 1 sec select e1.a as a insert into O;",
    "define stream S (a int); define stream T (a int); from every (not S for 1 sec or not T for 2 sec) -> e3=S "
    "select e3.a as a insert into O;",
])
def test_general_engine_lowers(lib, text):
    """includes AbsentLogicalPreStateProcessor (`A and not B for T`)"""
    rc, h, _ = _compile(lib, text)
    assert rc == abi.SH_OK, lib.sh_last_error(h)
    lib.sh_destroy(h)


@pytest.mark.parametrize("text", [
    # a final min-0 count inside a partition hands isEventReturned across keys
    "define stream S (k int, a int); partition with (k of S) begin "
    "from every e1=S -> e2=S[a > e1.a]<0:2> select e1.a as a insert into O; end;",
])
def test_unlowered_shapes_are_refused(lib, text):
    rc, h, _ = _compile(lib, text)
    assert rc == abi.SH_E_UNSUPPORTED
    assert lib.sh_last_error(h)
    lib.sh_destroy(h)


def test_no_cpu_fallback_without_device(lib):
    if lib.sh_device_count() > 0:
        pytest.skip("a GPU is present")
    rc, h, _ = _compile(lib, synth.C2_QUERY)
    assert rc == abi.SH_OK
    import numpy as np
    ts = np.zeros(1, np.int64)
    cols = [np.zeros(1, np.int32), np.zeros(1, np.float32), np.zeros(1, np.int64)]
    cp = (C.c_void_p * 3)(*[c.ctypes.data for c in cols])
    keys = np.zeros(1, np.int32)
    b = abi.sh_batch(stream=0, on_device=0, n=1, ts=ts.ctypes.data, keys=keys.ctypes.data, cols=cp, nulls=None)
    assert lib.sh_push_batch(h, C.byref(b)) == abi.SH_E_NO_DEVICE
    lib.sh_destroy(h)


def test_version_string(lib):
    assert b"gfx950" in lib.sh_version()


def test_round3_layout_caller_is_refused(lib):
    """a binding built against the 0.1 header put version (2) at offset 88, where
    d_out_cols now sits: sh_run_device refuses the struct instead of treating the
    integer as a column-pointer array (checked before any device work)"""
    rc, h, _ = _compile(lib, synth.C2_QUERY)
    assert rc == abi.SH_OK
    run = abi.sh_device_run()
    run.n = 1
    C.memmove(C.addressof(run) + 88, C.byref(C.c_int64(2)), 8)  # version = 2, pad = 0 at offset 88
    assert lib.sh_run_device(h, C.byref(run)) == abi.SH_E_INVALID_ARG
    assert b"0.1" in lib.sh_last_error(h)
    lib.sh_destroy(h)
    assert b"layout 2" in lib.sh_version()
