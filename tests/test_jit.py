"""hipRTC code generation of the window kernels (sh_jit.cpp), checked on the CPU:
the specialised source is generated and compiles for gfx950 for the C2 query and
for the random window-engine queries the GPU parity tests run."""
import ctypes as C
import random

import pytest

from siddhi_amd import abi, build, compiler, synth
from window_cases import window_case


@pytest.fixture(scope="module")
def lib():
    return abi.bind_product(C.CDLL(build.build()))


def _handle(lib, text, strings=None):
    d = compiler.compile_app(text, strings).descriptor()
    h = C.c_void_p()
    assert lib.sh_compile(C.byref(d), C.byref(h)) == abi.SH_OK, lib.sh_last_error(h)
    return h


def _source(lib, h):
    n = lib.shx_jit_source(h, None, 0)
    assert n > 0
    buf = C.create_string_buffer(n + 1)
    lib.shx_jit_source(h, buf, n + 1)
    return buf.value.decode()


def test_c2_specialised_source(lib):
    h = _handle(lib, synth.C2_QUERY)
    src = _source(lib, h)
    # partition-key tautology `symbol == e1.symbol` folded: only price staged
    assert "s_c1[SHJ_SPAN]" in src and "s_c0[" not in src
    assert "vm_cmp(7, 2," in src  # price > ... compared in the float domain
    assert lib.shx_jit_compile(h) == abi.SH_OK, lib.sh_last_error(h)
    lib.sh_destroy(h)


def test_non_window_shape_has_no_source(lib):
    h = _handle(lib, "define stream S (a int); from e1=S[a > 1] -> e2=S[a > e1.a] -> e3=S[a > e2.a] "
                     "select e1.a as x insert into Out;")
    assert lib.shx_jit_source(h, None, 0) == -1
    assert lib.shx_jit_compile(h) == abi.SH_E_UNSUPPORTED
    lib.sh_destroy(h)


@pytest.mark.parametrize("seed", range(24))
def test_random_window_queries_compile(lib, seed):
    app, _ = window_case(random.Random(7000 + seed))
    strings = compiler.StringDict()
    h = _handle(lib, app, strings)
    assert lib.shx_jit_compile(h) == abi.SH_OK, (app, lib.sh_last_error(h))
    lib.sh_destroy(h)


def test_c2_bucket_matcher_compiles(lib):
    """shb_match (bucketed window engine) for C2: only price is staged and the
    match stream carries e1.price (e1.symbol is the partition key, taken from e2)"""
    h = _handle(lib, synth.C2_QUERY)
    buf = C.create_string_buffer(1 << 20)
    rc = lib.shx_bucket_compile(h, buf, 1 << 20)
    src = buf.value.decode()
    assert rc == abi.SH_OK, (lib.sh_last_error(h), src[-3000:])
    assert "s_a1[SHB_SPANJ]" in src and "s_a0[" not in src and "s_a2[" not in src
    assert "P.ms[0])[dst] = s_a1[o]" in src
    lib.sh_destroy(h)


@pytest.mark.parametrize("seed", range(12))
def test_random_window_queries_bucket_compile(lib, seed):
    app, _ = window_case(random.Random(7000 + seed))
    strings = compiler.StringDict()
    h = _handle(lib, app, strings)
    rc = lib.shx_bucket_compile(h, None, 0)
    assert rc in (abi.SH_OK, abi.SH_E_UNSUPPORTED), (app, lib.sh_last_error(h))
    lib.sh_destroy(h)


def test_c3_has_the_rise_and_fall_sequence_shape(lib):
    """C3 lowers to the k_seq3 engine; near misses (a filter on e1, `within`,
    e2[last] read from a different position) stay on the general engine"""
    h = _handle(lib, synth.C3_QUERY)
    assert lib.shx_seq3_shape(h) == 1
    lib.sh_destroy(h)
    base = ("define stream S (symbol string, price float, volume long); partition with (symbol of S) begin "
            "from every e1=S{e1f}, e2=S[price>e1.price]+, e3=S[price<e2[last].price]{w} "
            "select e1.price as p1, e2[last].price as peak, e3.price as p3 insert into Out; end;")
    for e1f, w, want in [("", "", 1), ("[price > 1.0f]", "", 0), ("", " within 1 sec", 0)]:
        h = _handle(lib, base.format(e1f=e1f, w=w))
        assert lib.shx_seq3_shape(h) == want, (e1f, w)
        lib.sh_destroy(h)
    mixed = ("define stream S (symbol string, price float, volume long); partition with (symbol of S) begin "
             "from every e1=S, e2=S[volume >= e1.volume]+, e3=S[e2[last].price > price] "
             "select e3.volume as v3, e1.symbol as s, e2[last].volume as lv insert into Out; end;")
    h = _handle(lib, mixed)
    assert lib.shx_seq3_shape(h) == 1
    lib.sh_destroy(h)
