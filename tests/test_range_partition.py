"""Range partitions (`partition with (cond as 'label' or ... of S)`), SURVEY.md 8(f) row 4.

The reference evaluates every RangePartitionExecutor of the stream per event, in
declaration order, and sends the event to the partition of each range that holds
(core/partition/executor/RangePartitionExecutor.java:38-43,
core/partition/PartitionStreamReceiver.java:176-272); an event no range accepts is
dropped. The host mirror expands the batch accordingly and keys it by the labels.

Parity: no reference test runs a pattern inside a range partition (the range tests in
query/partition/PartitionTestCase1.java:1037-1226 use windows and sum), so these
results are checked by construction: a range partition over disjoint ranges must
equal a value partition over a column holding the label, and overlapping ranges must
equal the value partition over the explicitly expanded stream. The GPU test then
holds the HIP engine to the oracle on the same range-partitioned apps.
"""
import random

import pytest

from fixture_runner import Unsupported
from oracle_engine import OracleEngine
from siddhi_amd import SiddhiManager, compiler
from siddhi_amd.hostexpr import RangeEvaluator

RANGE_APP = """
define stream S (symbol string, price float, volume long);
partition with (price >= 100 as 'large' or price < 100 and price >= 50 as 'medium' or price < 50 as 'small' of S)
begin
  @info(name = 'q')
  from every e1=S[volume > 10] -> e2=S[price > e1.price] within 40 milliseconds
  select e1.symbol as s1, e1.price as p1, e2.symbol as s2, e2.price as p2
  insert into Out;
end;
"""

VALUE_APP = """
define stream S (symbol string, price float, volume long, band string);
partition with (band of S)
begin
  @info(name = 'q')
  from every e1=S[volume > 10] -> e2=S[price > e1.price] within 40 milliseconds
  select e1.symbol as s1, e1.price as p1, e2.symbol as s2, e2.price as p2
  insert into Out;
end;
"""

OVERLAP_APP = """
define stream S (symbol string, price float, volume long);
partition with (price >= 40 as 'hi' or price < 120 as 'lo' or volume == 7 as 'seven' of S)
begin
  @info(name = 'q')
  from every e1=S -> e2=S[price > e1.price]
  select e1.price as p1, e2.price as p2, e2.volume as v2
  insert into Out;
end;
"""


def _stream(seed, n=400):
    rng = random.Random(seed)
    rows, ts, t = [], [], 1000
    for _ in range(n):
        t += rng.randint(0, 9)
        rows.append([rng.choice(["IBM", "WSO2", "ORCL"]), float(rng.choice([20, 45, 55, 75, 99, 100, 101, 150, 30.5])),
                     rng.randint(1, 20)])
        ts.append(t)
    return ts, rows


def _band(price):
    return "large" if price >= 100 else ("medium" if price >= 50 else "small")


def run_app(app, ts, rows, factory, batch=7):
    mgr = SiddhiManager(engine_factory=factory)
    rt = mgr.createSiddhiAppRuntime(app)
    got = []
    rt.addCallback("Out", lambda evs: got.extend((e.timestamp, tuple(e.data)) for e in evs))
    rt.start()
    h = rt.getInputHandler("S")
    for b in range(0, len(rows), batch):
        h.send_batch(ts[b:b + batch], rows[b:b + batch])
    rt.shutdown()
    return got


def test_parse_range_partition():
    app = compiler.parse(RANGE_APP)
    spec = app.partitions[0]["S"]
    assert isinstance(spec, compiler.RangeSpec)
    assert [lb for _, lb in spec.ranges] == ["large", "medium", "small"]
    # the second range is one `and` condition (the `or` separates ranges)
    assert isinstance(spec.ranges[1][0], compiler.EBin) and spec.ranges[1][0].op == "and"
    c = compiler.compile_app(RANGE_APP)
    d = c.descriptor()
    assert d.partition_streams[0] == 1 and d.partition_attr[0] == -1


def test_parse_errors():
    with pytest.raises(compiler.SiddhiParserException):
        compiler.parse("define stream S (a int); partition with (a > 1 as large of S) begin "
                       "from every e1=S -> e2=S select e1.a as a insert into O; end;")
    with pytest.raises(Exception):
        compiler.compile_app("define stream S (a int); partition with (b > 1 as 'x' of S) begin "
                             "from every e1=S -> e2=S select e1.a as a insert into O; end;")


def test_host_condition_semantics():
    sd = compiler.StreamDef("S", [("f", compiler.FLOAT), ("i", compiler.INT), ("l", compiler.LONG)])
    ev = RangeEvaluator(sd, "S")

    def cond(text, row):
        p = compiler.Parser(text)
        return ev.cond(p.expr(), row)

    # FloatInt compare promotes the int to float (16777217 -> 16777216.0f)
    assert cond("f >= 16777217", [16777216.0, 0, 0])
    assert not cond("f > 16777217", [16777216.0, 0, 0])
    # a compare with null is false, not(null compare) is true, `is null`
    assert not cond("f > 1", [None, 0, 0]) and cond("not (f > 1)", [None, 0, 0])
    assert cond("f is null", [None, 0, 0])
    # integer division by zero is null (so the compare is false); int wraps
    assert not cond("i / 0 == 0", [1.0, 5, 0])
    assert cond("i * 2 < 0", [1.0, 2 ** 30, 0])
    assert cond("-7 / 2 == -3 and -7 % 2 == -1", [1.0, 0, 0])
    assert cond("l + 1 > i", [0.0, 5, 5])


@pytest.mark.parametrize("seed", range(6))
def test_disjoint_ranges_equal_value_partition(seed):
    ts, rows = _stream(seed)
    got_r = run_app(RANGE_APP, ts, rows, OracleEngine)
    got_v = run_app(VALUE_APP, ts, [r + [_band(r[1])] for r in rows], OracleEngine)
    assert got_r == got_v and len(got_r) > 0


@pytest.mark.parametrize("seed", range(4))
def test_overlapping_ranges_equal_expanded_stream(seed):
    ts, rows = _stream(100 + seed, 300)
    got_r = run_app(OVERLAP_APP, ts, rows, OracleEngine, batch=len(rows))
    ets, erows = [], []
    for t, r in zip(ts, rows):
        for lb, ok in (("hi", r[1] >= 40), ("lo", r[1] < 120), ("seven", r[2] == 7)):
            if ok:
                ets.append(t)
                erows.append(r + [lb])
    value = OVERLAP_APP.replace("volume long);", "volume long, band string);").replace(
        "price >= 40 as 'hi' or price < 120 as 'lo' or volume == 7 as 'seven' of S", "band of S")
    got_v = run_app(value, ets, erows, OracleEngine, batch=len(erows))
    assert got_r == got_v and len(got_r) > 0


def test_event_in_no_range_is_dropped():
    app = RANGE_APP.replace("or price < 50 as 'small' ", "")
    ts, rows = _stream(7)
    got = run_app(app, ts, rows, OracleEngine)
    assert got and all(p1 >= 50 and p2 >= 50 for _, (_, p1, _, p2) in got)


@pytest.mark.gpu
@pytest.mark.parametrize("app", [RANGE_APP, OVERLAP_APP])
@pytest.mark.parametrize("seed", range(3))
def test_range_partition_gpu_vs_oracle(app, seed):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from siddhi_amd._native import HipEngine, HipError

    def hip(c):
        try:
            return HipEngine(c)
        except HipError as e:
            if e.code == -4:
                raise Unsupported(str(e))
            raise

    ts, rows = _stream(200 + seed, 600)
    assert run_app(app, ts, rows, hip) == run_app(app, ts, rows, OracleEngine)


def test_range_stream_read_outside_the_partition_is_refused():
    """a query outside a range partition reads the original stream, one inside it
    the expanded one: such apps stay on the Java runtime"""
    from siddhi_amd.runtime import SiddhiAppCreationException
    app = RANGE_APP.replace("end;", "end;\n@info(name = 'g') from every e1=S -> e2=S[price > e1.price] "
                                    "select e1.price as p1, e2.price as p2 insert into G;")
    with pytest.raises(SiddhiAppCreationException):
        SiddhiManager(engine_factory=OracleEngine).createSiddhiAppRuntime(app)


ABSENT_RANGE_APP = """
@app:playback
define stream S (symbol string, price float, volume long);
partition with (price >= 100 as 'large' of S)
begin
  @info(name = 'q')
  from e1=S[price >= 100] -> not S[price > e1.price] for 1 sec
  select e1.price as p
  insert into Out;
end;
"""


def _absent_range(factory):
    steps = []
    for second in ([[1500, 2500], [["A", 120.0, 1], ["A", 10.0, 1]]],   # the last event is in no range
                   [[2500], [["A", 10.0, 1]]]):                        # no event is in a range
        mgr = SiddhiManager(engine_factory=factory)
        rt = mgr.createSiddhiAppRuntime(ABSENT_RANGE_APP)
        got = []
        rt.addCallback("Out", lambda evs: got.extend((e.timestamp, tuple(e.data)) for e in evs))
        rt.start()
        h = rt.getInputHandler("S")
        h.send_batch([1000], [["A", 150.0, 1]])
        # the clock moves to the batch's last event (2500) before the batch
        # (InputHandler.java:85-96), so the timer due at 2000 fires first
        h.send_batch(*second)
        steps.append(list(got))
        rt.shutdown()
    return steps


def test_playback_clock_moves_on_events_no_range_keeps():
    assert _absent_range(OracleEngine) == [[(2000, (150.0,))], [(2000, (150.0,))]]


@pytest.mark.gpu
def test_playback_clock_no_range_gpu_vs_oracle():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from siddhi_amd._native import HipEngine
    assert _absent_range(HipEngine) == _absent_range(OracleEngine)


def test_labels_and_string_literals_are_verbatim():
    """STRING_LITERAL has no escapes (SiddhiQL.g4:854-860): non-ASCII labels and
    backslashes reach the partition key text unchanged (its String.hashCode
    orders the scheduler's map)"""
    app = compiler.parse("define stream S (s string, p float); partition with (p >= 1 as 'größer' or "
                         "p < 1 as \"a\\tb\" of S) begin from every e1=S -> e2=S[s == 'x\\y'] "
                         "select e1.p as p insert into O; end;")
    assert [lb for _, lb in app.partitions[0]["S"].ranges] == ["größer", "a\\tb"]
    got = run_app(app_text := RANGE_APP.replace("'large'", "'größer'"), *_stream(3), OracleEngine)
    assert got == run_app(RANGE_APP, *_stream(3), OracleEngine) and app_text
