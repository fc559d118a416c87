"""SiddhiQL subset compiler: app text -> query-api-like tree -> sh_app_desc.

This mirrors, for the pattern/sequence hot path only, what the reference does in
  modules/siddhi-query-compiler/src/main/antlr4/io/siddhi/query/compiler/SiddhiQL.g4:180-330
  modules/siddhi-query-compiler/.../internal/SiddhiQLBaseVisitorImpl.java:760-1400 (tree shape)
  modules/siddhi-core/.../util/parser/StateInputStreamParser.java:148-408      (slot order)
  modules/siddhi-core/.../util/parser/ExpressionParser.java:225-1439          (typed executors,
                                                                               variable positions)
  modules/siddhi-core/.../util/parser/SelectorParser.java:215                 (select default index 0)

Supported: `define stream`, `@app:playback`, `@info(name=...)`, `partition with
(attr of Stream | cond as 'label' or ... of Stream, ...) begin ... end`, pattern (`->`) and sequence (`,`) queries with
`every`, `within`, filters, logical `and`/`or`, `not X for T`, counts `<m:n>` `+` `*` `?`,
`e[i]` / `e[last]` / `e[last-k]` references, `select ... [as ...]` with
sum/avg/count/max/min, `insert [current events] into`.
Anything else raises SiddhiParserException / UnsupportedQuery.
"""
from __future__ import annotations

import ctypes
import re
import struct
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

from . import abi

# Attribute.Type
STRING, INT, LONG, FLOAT, DOUBLE, BOOL, OBJECT = range(7)
TYPE_NAMES = {"string": STRING, "int": INT, "long": LONG, "float": FLOAT,
              "double": DOUBLE, "bool": BOOL, "object": OBJECT}
TYPE_STR = {v: k.upper() for k, v in TYPE_NAMES.items()}

CURRENT = -1   # SiddhiConstants.CURRENT
LAST = -2      # SiddhiConstants.LAST
UNKNOWN_STATE = -1
HAVING_STATE = -2  # SiddhiConstants.HAVING_STATE


class SiddhiParserException(Exception):
    pass


class SiddhiAppValidationException(Exception):
    pass


class UnsupportedQuery(Exception):
    pass


# ----------------------------------------------------------------- lexer
_TOKEN_RE = re.compile(r"""
    (?P<ws>\s+|--[^\n]*|/\*.*?\*/)
  | (?P<str>"{3}.*?"{3}|'[^'"\x00-\x1f]*'|"[^"\x00-\x1f]*")
  | (?P<num>(?:\d+\.\d*|\.\d+|\d+)(?:[eE][-+]?\d+)?[lLfFdD]?)
  | (?P<id>[A-Za-z_][A-Za-z0-9_]*)
  | (?P<op>->|==|!=|>=|<=|[-+*/%<>=(),;\[\].@:#!?{}])
""", re.VERBOSE | re.DOTALL)


def _str_text(lit: str) -> str:
    """STRING_LITERAL text (SiddhiQL.g4:854-860): the characters between the quotes,
    verbatim -- the grammar has no escape sequences"""
    return lit[3:-3] if lit.startswith('"""') else lit[1:-1]


@dataclass
class Tok:
    kind: str
    text: str
    pos: int


def tokenize(s: str) -> List[Tok]:
    out = []
    i = 0
    while i < len(s):
        m = _TOKEN_RE.match(s, i)
        if not m:
            raise SiddhiParserException(f"unexpected character {s[i]!r} at {i}")
        kind = m.lastgroup
        if kind != "ws":
            out.append(Tok(kind, m.group(kind), i))
        i = m.end()
    out.append(Tok("eof", "", len(s)))
    return out


# ----------------------------------------------------------------- AST
@dataclass
class StreamDef:
    name: str
    attrs: List[Tuple[str, int]]

    def index(self, attr):
        for i, (n, _) in enumerate(self.attrs):
            if n == attr:
                return i
        return -1


@dataclass
class EConst:
    type: int
    value: object
    is_null: bool = False


@dataclass
class EVar:
    stream: Optional[str]        # reference id / stream id or None
    name: str
    index: Optional[int] = None  # e[k]: k; e[last]: -2; e[last-k]: -2-k


@dataclass
class EStreamRef:                # `e1 is null` / `e1[0] is null`
    stream: str
    index: Optional[int] = None


@dataclass
class EBin:
    op: str
    l: object
    r: object


@dataclass
class ENot:
    x: object


@dataclass
class EIsNull:
    x: object


@dataclass
class EFunc:
    name: str
    args: list


@dataclass
class SStream:                   # StreamStateElement / AbsentStreamStateElement
    ref: Optional[str]
    stream: str
    filter: object = None
    absent: bool = False
    waiting_ms: int = -1


@dataclass
class SNext:
    a: object
    b: object


@dataclass
class SEvery:
    x: object


@dataclass
class SLogical:
    kind: str                    # 'and' / 'or'
    a: object
    b: object


@dataclass
class SCount:
    x: SStream
    min: int
    max: int


@dataclass
class OutAttr:
    expr: object
    name: str


@dataclass
class Query:
    name: Optional[str]
    state_type: int              # 0 pattern 1 sequence
    root: object
    within_ms: int
    select: List[OutAttr]
    select_star: bool
    output: str
    partition: int = -1
    having: object = None        # Selector.having (QuerySelector havingConditionExecutor)
    order_by: list = field(default_factory=list)   # [(EVar, desc)] (Selector.orderByList)
    group_by: list = field(default_factory=list)   # [EVar] (Selector.groupByList)
    limit: object = None         # Selector.limit / offset expressions (constants)
    offset: object = None
    rate: Optional[Tuple[int, int]] = None   # (enum sh_rate, N): `output first|last every N events`


@dataclass
class RangeSpec:
    """range partition of one stream: (condition, label) in declaration order
    (core/partition/executor/RangePartitionExecutor.java; PartitionParser builds one
    executor per range, evaluated in this order)"""
    ranges: List[Tuple[object, str]]


@dataclass
class App:
    name: Optional[str]
    playback: bool
    streams: Dict[str, StreamDef]
    stream_order: List[str]
    queries: List[Query]
    partitions: List[Dict[str, object]]   # per partition: stream -> attribute name | RangeSpec
    output_streams: List[str] = field(default_factory=list)


# ----------------------------------------------------------------- parser
_TIME_UNITS = {
    "millisec": 1, "millisecond": 1, "milliseconds": 1, "millis": 1, "ms": 1,
    "sec": 1000, "second": 1000, "seconds": 1000,
    "min": 60000, "minute": 60000, "minutes": 60000,
    "hour": 3600000, "hours": 3600000,
    "day": 86400000, "days": 86400000,
    "week": 604800000, "weeks": 604800000,
    "month": 2630000000, "months": 2630000000,
    "year": 31556900000, "years": 31556900000,
}


class Parser:
    def __init__(self, text: str):
        self.t = tokenize(text)
        self.i = 0

    # -- token helpers
    def peek(self, k=0) -> Tok:
        return self.t[min(self.i + k, len(self.t) - 1)]

    def kw(self, word, k=0) -> bool:
        tk = self.peek(k)
        return tk.kind == "id" and tk.text.lower() == word

    def op(self, s, k=0) -> bool:
        tk = self.peek(k)
        return tk.kind == "op" and tk.text == s

    def next(self) -> Tok:
        tk = self.t[self.i]
        self.i += 1
        return tk

    def expect_op(self, s):
        if not self.op(s):
            self.err(f"expected '{s}'")
        return self.next()

    def expect_kw(self, w):
        if not self.kw(w):
            self.err(f"expected '{w}'")
        return self.next()

    def ident(self) -> str:
        tk = self.peek()
        if tk.kind != "id":
            self.err("expected identifier")
        self.i += 1
        return tk.text

    def err(self, msg):
        tk = self.peek()
        raise SiddhiParserException(f"{msg} at offset {tk.pos} near {tk.text!r}")

    # -- app
    def parse_app(self) -> App:
        app = App(None, False, {}, [], [], [])
        pending_ann = []
        while self.peek().kind != "eof":
            if self.op(";"):
                self.next()
                continue
            if self.op("@"):
                ann = self.annotation()
                if ann[0] == "app:playback":
                    app.playback = True
                elif ann[0] == "app:name":
                    app.name = ann[1].get(None)
                elif not ann[0].startswith("app:"):
                    pending_ann.append(ann)
                continue
            if self.kw("define"):
                self.next()
                if not self.kw("stream"):
                    raise UnsupportedQuery("only `define stream` is supported")
                self.next()
                name = self.source_name()
                self.expect_op("(")
                attrs = []
                while True:
                    an = self.ident()
                    ty = self.ident().lower()
                    if ty not in TYPE_NAMES:
                        self.err("bad attribute type")
                    attrs.append((an, TYPE_NAMES[ty]))
                    if self.op(","):
                        self.next()
                        continue
                    break
                self.expect_op(")")
                app.streams[name] = StreamDef(name, attrs)
                app.stream_order.append(name)
                pending_ann = []
                continue
            if self.kw("from"):
                q = self.query(pending_ann)
                pending_ann = []
                app.queries.append(q)
                continue
            if self.kw("partition"):
                self.partition(app)
                pending_ann = []
                continue
            self.err("unexpected token")
        return app

    def source_name(self) -> str:
        if self.op("#") or self.op("!"):
            raise UnsupportedQuery("inner/fault streams are out of scope")
        return self.ident()

    def annotation(self):
        self.expect_op("@")
        name = self.ident()
        if self.op(":"):
            self.next()
            name = name + ":" + self.ident()
        name = name.lower()
        elems = {}
        if self.op("("):
            self.next()
            depth = 1
            while depth:
                if self.op("("):
                    depth += 1
                    self.next()
                elif self.op(")"):
                    depth -= 1
                    self.next()
                elif self.peek().kind == "id" and self.op("=", 1):
                    k = self.next().text.lower()
                    self.next()
                    v = self.next().text
                    elems[k] = v.strip("'\"")
                elif self.peek().kind == "str":
                    elems[None] = self.next().text.strip("'\"")
                else:
                    self.next()
        return name, elems

    def partition(self, app: App):
        self.expect_kw("partition")
        self.expect_kw("with")
        self.expect_op("(")
        spec = {}
        while True:
            # partition_with_stream (SiddhiQL.g4): `attr of S` (value partition) or
            # `cond as 'label' (or cond as 'label')* of S` (range partition)
            e = self.expr()
            if self.kw("as"):
                ranges = []
                while True:
                    self.expect_kw("as")
                    tk = self.peek()
                    if tk.kind != "str":
                        self.err("expected a range label string")
                    self.next()
                    ranges.append((e, _str_text(tk.text)))
                    if self.kw("or"):
                        self.next()
                        e = self.expr()
                        continue
                    break
                self.expect_kw("of")
                spec[self.ident()] = RangeSpec(ranges)
            else:
                if not isinstance(e, EVar) or e.stream is not None or e.index is not None:
                    self.err("expected `attribute of Stream` or `condition as 'label' of Stream`")
                self.expect_kw("of")
                spec[self.ident()] = e.name
            if self.op(","):
                self.next()
                continue
            break
        self.expect_op(")")
        self.expect_kw("begin")
        pidx = len(app.partitions)
        app.partitions.append(spec)
        ann = []
        while not self.kw("end"):
            if self.op(";"):
                self.next()
                continue
            if self.op("@"):
                ann.append(self.annotation())
                continue
            if self.kw("from"):
                q = self.query(ann)
                ann = []
                q.partition = pidx
                app.queries.append(q)
                continue
            self.err("expected query inside partition")
        self.next()

    def query(self, anns) -> Query:
        name = None
        for a, el in anns:
            if a == "info":
                name = el.get("name")
        self.expect_kw("from")
        # decide pattern vs sequence: scan to 'select' at depth 0 for '->' vs ','
        st = self.detect_state_type()
        if st is None:
            raise UnsupportedQuery("only pattern/sequence queries are on the hot path")
        root = self.chain(st)
        within = -1
        if self.kw("within"):
            self.next()
            within = self.time_value()
        sel, star, having = [], False, None
        order, limit, offset, group = [], None, None, []
        if self.kw("select"):
            self.next()
            if self.op("*"):
                self.next()
                star = True
            else:
                while True:
                    e = self.expr()
                    if self.kw("as"):
                        self.next()
                        nm = self.ident()
                    elif isinstance(e, EVar):
                        nm = e.name
                    else:
                        self.err("output attribute needs `as`")
                    sel.append(OutAttr(e, nm))
                    if self.op(","):
                        self.next()
                        continue
                    break
            if self.kw("group"):
                # group_by: GROUP BY attribute_reference (, attribute_reference)* (SiddhiQL.g4)
                self.next()
                self.expect_kw("by")
                while True:
                    v = self.primary()
                    if not isinstance(v, EVar):
                        self.err("group by takes attribute references")
                    group.append(v)
                    if self.op(","):
                        self.next()
                        continue
                    break
            if self.kw("having"):
                self.next()
                having = self.expr()
            if self.kw("order"):
                # order_by: ORDER BY attribute_reference (ASC|DESC)? (, ...)* (SiddhiQL.g4:375-385)
                self.next()
                self.expect_kw("by")
                while True:
                    v = self.primary()
                    if not isinstance(v, EVar):
                        self.err("order by takes attribute references")
                    desc = False
                    if self.kw("asc") or self.kw("desc"):
                        desc = self.next().text.lower() == "desc"
                    order.append((v, desc))
                    if self.op(","):
                        self.next()
                        continue
                    break
            if self.kw("limit"):
                self.next()
                limit = self.expr()
            if self.kw("offset"):
                self.next()
                offset = self.expr()
        else:
            star = True
        rate = None
        if self.kw("output"):
            # output_rate: OUTPUT (ALL|LAST|FIRST)? EVERY (INT EVENTS | time) | OUTPUT SNAPSHOT EVERY time
            # (SiddhiQL.g4 output_rate); the device runs `output first every N events`
            self.next()
            kind = None
            for w in ("all", "last", "first", "snapshot"):
                if self.kw(w):
                    kind = self.next().text.lower()
                    break
            self.expect_kw("every")
            tk = self.peek()
            if kind == "first" and tk.kind == "num" and self.peek(1).kind == "id" and \
                    self.peek(1).text.lower() in _TIME_UNITS:
                # FirstPerTimeOutputRateLimiter against the timestamp generator's clock
                # (playback apps only: checked when the query is lowered)
                ms = self.time_value()
                if ms >= 1 << 31:
                    raise UnsupportedQuery("output first every T: T >= 2^31 ms")
                rate = (4, ms)
            elif kind == "snapshot" or tk.kind != "num" or not self.peek(1).text.lower() == "events":
                # LastPerTime / AllPerTime schedule from System.currentTimeMillis() when a
                # partition is created (AllPerTimeOutputRateLimiter.java:97-108), even in
                # playback, and the snapshot limiters run on such a timer: no replayable answer
                raise UnsupportedQuery("output rate limiting: `output [first|last|all] every N events` and "
                                       "`output first every T` (@app:playback) run on the device")
            else:
                n = int(self.next().text)
                self.next()  # events
                if n < 1:
                    raise UnsupportedQuery(f"output {kind} every 0 events")
                # OutputParser.constructOutputRateLimiter: no keyword is ALL
                rate = ({"first": 1, "last": 2}.get(kind, 3), n)
        self.expect_kw("insert")
        if self.kw("current"):
            self.next()
            self.expect_kw("events")
        elif self.kw("all") or self.kw("expired"):
            raise UnsupportedQuery("only current events output is supported")
        elif self.kw("events"):
            self.next()
        self.expect_kw("into")
        if self.op("#"):
            raise UnsupportedQuery("inner-stream outputs (#Stream) are out of scope")
        out = self.ident()
        return Query(name, st, root, within, sel, star, out, having=having, order_by=order, group_by=group,
                     limit=limit, offset=offset, rate=rate)

    def detect_state_type(self):
        depth = 0
        j = self.i
        saw_arrow = saw_comma = False
        while j < len(self.t):
            tk = self.t[j]
            if tk.kind == "op" and tk.text in "([":
                depth += 1
            elif tk.kind == "op" and tk.text in ")]":
                depth -= 1
            elif tk.kind == "op" and tk.text == "->":
                saw_arrow = True
            elif tk.kind == "op" and tk.text == "," and depth == 0:
                saw_comma = True
            elif tk.kind == "id" and tk.text.lower() in ("select", "insert", "within") and depth == 0:
                break
            elif tk.kind == "op" and tk.text == ";":
                break
            j += 1
        if saw_arrow:
            return 0
        if saw_comma:
            return 1
        # single-state pattern: `from e1=A[...] select` is a standard stream (not hot path)
        # unless it uses every / not / and / or / counts
        k = self.i
        while k < j:
            tk = self.t[k]
            if tk.kind == "id" and tk.text.lower() in ("every", "not", "and", "or"):
                return 0
            k += 1
        return None

    def time_value(self) -> int:
        total = 0
        got = False
        while self.peek().kind == "num" and self.peek(1).kind == "id" and \
                self.peek(1).text.lower() in _TIME_UNITS:
            n = int(self.next().text)
            u = self.next().text.lower()
            total += n * _TIME_UNITS[u]
            got = True
        if not got:
            self.err("expected time value")
        return total

    # -- state chains (every_pattern_source_chain / sequence_source_chain)
    def chain(self, st):
        sep = "->" if st == 0 else ","
        left = self.chain_term(st)
        while self.op(sep):
            self.next()
            right = self.chain_term(st)
            left = SNext(left, right)
        return left

    def chain_term(self, st):
        if self.kw("every"):
            self.next()
            if self.op("("):
                self.next()
                inner = self.chain(st)
                self.expect_op(")")
                return SEvery(inner)
            return SEvery(self.source(st))
        if self.op("("):
            self.next()
            inner = self.chain(st)
            self.expect_op(")")
            return inner
        return self.source(st)

    def source(self, st):
        # pattern_source: logical | collection | standard | logical absent | absent
        left = self.stateful(st)
        if self.kw("and") or self.kw("or"):
            kind = self.next().text.lower()
            right = self.stateful(st)
            if isinstance(left, SCount) or isinstance(right, SCount):
                self.err("counts cannot be logical operands")
            if right.absent and not left.absent:
                # a present/absent mix puts the absent element first
                # (SiddhiQLBaseVisitorImpl.visitLogical_absent_stateful_source:
                # State.logicalNotAnd(absent, present) / logicalOr(absent, present))
                left, right = right, left
            return SLogical(kind, left, right)
        return left

    def stateful(self, st):
        if self.kw("not"):
            self.next()
            ss = self.basic_source(None)
            ss.absent = True
            if self.kw("for"):
                self.next()
                ss.waiting_ms = self.time_value()
            else:
                # `A and not B` without `for`: AbsentStreamStateElement without waiting time
                ss.waiting_ms = -1
            return ss
        ref = None
        if self.peek().kind == "id" and self.op("=", 1):
            ref = self.next().text
            self.next()
        ss = self.basic_source(ref)
        if self.op("<"):
            self.next()
            mn, mx = -1, -1
            if self.op(":"):
                self.next()
                mx = int(self.next().text)
            else:
                a = int(self.next().text)
                if self.op(":"):
                    self.next()
                    mn = a
                    if self.peek().kind == "num":
                        mx = int(self.next().text)
                else:
                    mn = mx = a
            self.expect_op(">")
            return SCount(ss, mn, mx)
        if st == 1 and (self.op("+") or self.op("*") or self.op("?")):
            o = self.next().text
            return SCount(ss, *{"+": (1, -1), "*": (0, -1), "?": (0, 1)}[o])
        return ss

    def basic_source(self, ref):
        stream = self.source_name()
        flt = None
        while self.op("["):
            self.next()
            e = self.expr()
            self.expect_op("]")
            flt = e if flt is None else EBin("and", flt, e)
        if self.op("#"):
            raise UnsupportedQuery("stream functions/windows inside states are out of scope")
        return SStream(ref, stream, flt)

    # -- expressions (math_operation precedence, SiddhiQL.g4:460-474)
    def expr(self):
        return self.or_expr()

    def or_expr(self):
        l = self.and_expr()
        while self.kw("or"):
            self.next()
            l = EBin("or", l, self.and_expr())
        return l

    def and_expr(self):
        l = self.eq_expr()
        while self.kw("and"):
            self.next()
            l = EBin("and", l, self.eq_expr())
        return l

    def eq_expr(self):
        l = self.cmp_expr()
        while self.op("==") or self.op("!="):
            o = self.next().text
            l = EBin(o, l, self.cmp_expr())
        return l

    def cmp_expr(self):
        l = self.add_expr()
        while self.op(">=") or self.op("<=") or self.op(">") or self.op("<"):
            o = self.next().text
            l = EBin(o, l, self.add_expr())
        return l

    def add_expr(self):
        l = self.mul_expr()
        while self.op("+") or self.op("-"):
            o = self.next().text
            l = EBin(o, l, self.mul_expr())
        return l

    def mul_expr(self):
        l = self.unary()
        while self.op("*") or self.op("/") or self.op("%"):
            o = self.next().text
            l = EBin(o, l, self.unary())
        return l

    def unary(self):
        if self.kw("not"):
            self.next()
            return ENot(self.unary())
        if self.op("-") and self.peek(1).kind == "num":
            self.next()
            c = self.number(self.next().text)
            c.value = -c.value
            return self.postfix(c)
        return self.postfix(self.primary())

    def postfix(self, e):
        if self.kw("is") and self.kw("null", 1):
            self.next()
            self.next()
            if isinstance(e, EVar) and e.stream is None and e.index is None and getattr(e, "_bare", False):
                return EIsNull(e)
            return EIsNull(e)
        return e

    def number(self, txt) -> EConst:
        low = txt.lower()
        if low.endswith("l"):
            return EConst(LONG, int(txt[:-1]))
        if low.endswith("f"):
            return EConst(FLOAT, float(txt[:-1]))
        if low.endswith("d"):
            return EConst(DOUBLE, float(txt[:-1]))
        if "." in txt or "e" in low:
            return EConst(DOUBLE, float(txt))
        return EConst(INT, int(txt))

    def primary(self):
        tk = self.peek()
        if self.op("("):
            self.next()
            e = self.expr()
            self.expect_op(")")
            return e
        if tk.kind == "num":
            self.next()
            return self.number(tk.text)
        if tk.kind == "str":
            self.next()
            return EConst(STRING, _str_text(tk.text))
        if tk.kind == "id":
            low = tk.text.lower()
            if low in ("true", "false"):
                self.next()
                return EConst(BOOL, low == "true")
            if low == "null":
                self.next()
                return EConst(OBJECT, None, True)
            name = self.next().text
            if self.op("("):  # function
                self.next()
                args = []
                if not self.op(")"):
                    if self.op("*"):
                        self.next()
                    else:
                        while True:
                            args.append(self.expr())
                            if self.op(","):
                                self.next()
                                continue
                            break
                self.expect_op(")")
                return EFunc(name, args)
            if self.op(":") and self.peek(1).kind == "id" and self.op("(", 2):
                raise UnsupportedQuery(f"namespaced function {name}:... is out of scope")
            index = None
            if self.op("["):
                self.next()
                if self.kw("last"):
                    self.next()
                    index = LAST
                    if self.op("-"):
                        self.next()
                        index = LAST - int(self.next().text)
                else:
                    index = int(self.next().text)
                self.expect_op("]")
            if self.op("."):
                self.next()
                attr = self.ident()
                return EVar(name, attr, index)
            if index is not None:
                return EStreamRef(name, index)
            v = EVar(None, name, None)
            v._bare = True
            return v
        self.err("expected expression")


def parse(text: str) -> App:
    return Parser(text).parse_app()


# ----------------------------------------------------------------- lowering
class Lowerer:
    """Assigns state slots in StateInputStreamParser parse order and resolves
    expression types / variable positions like ExpressionParser."""

    def __init__(self, app: App, strings: "StringDict"):
        self.multi_ok = False   # expr(): a multi-value variable is allowed here
        self.last_multi = False
        self.app = app
        self.strings = strings
        self.stream_ids = {n: i for i, n in enumerate(app.stream_order)}

    def lower_query(self, q: Query):
        self.elems: List[dict] = []
        self.exprs: List[dict] = []
        self.slots: List[Tuple[StreamDef, Optional[str], bool]] = []  # (def, ref, multiValue)
        self.q = q
        # slot assignment (parse order): Next: current, next; Logical: element2 then element1
        self.pending_filters = []
        root = self.elem(q.root, False)
        for (eidx, flt, slot) in self.pending_filters:
            self.elems[eidx]["filter"] = self.expr(flt, slot, CURRENT)
        outs = []
        if q.select_star:
            # SelectorParser.java:180-205: every attribute of every state's stream, in
            # slot order, each as a bare variable; a name two streams share is a
            # DuplicateAttributeException
            sel, seen = [], set()
            for sd, _, _ in self.slots:
                for name, _ in sd.attrs:
                    if name in seen:
                        raise SiddhiAppValidationException(
                            f"Duplicate attribute exist in streams: '{name}' (select *)")
                    seen.add(name)
                    sel.append(OutAttr(EVar(None, name), name))
            q.select, q.select_star = sel, False
        for oa in q.select:
            outs.append(self.out_attr(oa))
        self.having = -1
        # HAVING_STATE (ExpressionParser.java:1308-1318): a bare name is first an
        # output attribute of the selected event, else a state-event attribute
        self.out_alias = {oa.name: (o, outs[o]["type"]) for o, oa in enumerate(q.select)}
        if q.having is not None:
            self.having = self.expr(q.having, HAVING_STATE, 0)
            self._want_bool(self.having)
        # OrderByEventComparator parses each attribute at HAVING_STATE (SelectorParser.java:110-114)
        # GroupByKeyGenerator (SelectorParser.java:102-108): UNKNOWN_STATE, default index 0
        self.group = []
        if len(q.group_by) > abi.SH_MAX_GROUP:
            raise UnsupportedQuery(f"group by: at most {abi.SH_MAX_GROUP} attributes")
        for v in q.group_by:
            self.group.append(self.expr(v, UNKNOWN_STATE, 0))
        if q.group_by and q.rate and q.rate[0] in (1, 2, 4):
            # OutputParser picks the GroupBy first / last limiters (one counter per group)
            raise UnsupportedQuery("group by with `output first|last every ...` (per-group limiters)")
        if q.rate and q.rate[0] == 4 and not self.app.playback:
            # TimestampGeneratorImpl.currentTime is System.currentTimeMillis() outside playback
            raise UnsupportedQuery("output first every T outside @app:playback reads the wall clock")
        self.order = []
        if len(q.order_by) > abi.SH_MAX_ORDER:
            raise UnsupportedQuery(f"order by: at most {abi.SH_MAX_ORDER} attributes")
        for v, desc in q.order_by:
            i = self.expr(v, HAVING_STATE, 0)
            if self.etype(i) in (STRING, OBJECT):
                raise UnsupportedQuery("order by a string attribute needs the text (host-side order)")
            self.order.append((i, desc))
        self.limit = self._count_const(q.limit, "limit")
        self.offset = self._count_const(q.offset, "offset")
        if any(o["agg"] != 0 for o in outs) and (self.offset > 0 or self.limit == 0):
            raise UnsupportedQuery("an aggregating selector with offset > 0 or limit 0 never emits")
        return root, outs

    @staticmethod
    def _count_const(e, what):
        """QuerySelector.setLimit / setOffset (:436-450): a constant, read as Number.longValue()."""
        if e is None:
            return -1
        if not isinstance(e, EConst) or e.type not in (INT, LONG, FLOAT, DOUBLE) or e.value is None:
            raise SiddhiAppValidationException(f"'{what}' must be a numeric constant")
        v = int(e.value)  # longValue(): truncation toward zero
        if v < 0:
            raise SiddhiAppValidationException(f"'{what}' cannot have negative value, but found '{v}'")
        return v

    def elem(self, s, multi):
        if isinstance(s, SStream):
            if s.stream not in self.app.streams:
                raise SiddhiAppValidationException(f"stream {s.stream} is not defined")
            slot = len(self.slots)
            self.slots.append((self.app.streams[s.stream], s.ref, multi))
            d = dict(kind=1 if s.absent else 0, child0=-1, child1=-1,
                     stream=self.stream_ids[s.stream], filter=-1, slot=slot,
                     min_count=-1, max_count=-1, waiting_ms=s.waiting_ms)
            self.elems.append(d)
            idx = len(self.elems) - 1
            if s.filter is not None:
                self.pending_filters.append((idx, s.filter, slot))
            return idx
        if isinstance(s, SNext):
            a = self.elem(s.a, multi)
            b = self.elem(s.b, multi)
            return self._push(kind=2, child0=a, child1=b)
        if isinstance(s, SEvery):
            a = self.elem(s.x, multi)
            return self._push(kind=3, child0=a, child1=-1)
        if isinstance(s, SLogical):
            b = self.elem(s.b, multi)   # element 2 parsed first (StateInputStreamParser.java:350-361)
            a = self.elem(s.a, multi)
            return self._push(kind=4 if s.kind == "and" else 5, child0=a, child1=b)
        if isinstance(s, SCount):
            a = self.elem(s.x, True)
            return self._push(kind=6, child0=a, child1=-1, min_count=s.min, max_count=s.max)
        raise UnsupportedQuery(f"state element {s!r}")

    def _push(self, **kw):
        d = dict(kind=0, child0=-1, child1=-1, stream=-1, filter=-1, slot=-1,
                 min_count=-1, max_count=-1, waiting_ms=-1)
        d.update(kw)
        self.elems.append(d)
        return len(self.elems) - 1

    # -- expressions
    def _e(self, **kw):
        d = dict(op=0, type=OBJECT, lhs=-1, rhs=-1, third=-1, ltype=OBJECT, rtype=OBJECT,
                 slot=-1, chain=0, attr=-1, is_null=0, cval=0)
        d.update(kw)
        self.exprs.append(d)
        return len(self.exprs) - 1

    def etype(self, i):
        return self.exprs[i]["type"]

    def const_bits(self, c: EConst):
        if c.is_null:
            return 0
        t = c.type
        if t == STRING:
            return self.strings.id(c.value)
        if t == BOOL:
            return 1 if c.value else 0
        if t == INT:
            v = int(c.value)
            return v
        if t == LONG:
            return int(c.value)
        if t == FLOAT:
            return struct.unpack("<I", struct.pack("<f", float(c.value)))[0]
        if t == DOUBLE:
            return struct.unpack("<q", struct.pack("<d", float(c.value)))[0]
        return 0

    def resolve_var(self, v: EVar, current: int, default_index: int):
        """ExpressionParser.parseVariable for a MetaStateEvent (ExpressionParser.java:1254-1439)."""
        if v.index is not None:
            chain = v.index + 1 if v.index <= LAST else v.index
        else:
            chain = default_index
        slot = -1
        typ = None
        multi = False
        if v.stream is None:
            if current == UNKNOWN_STATE:
                for i, (sd, ref, mv) in enumerate(self.slots):
                    ai = sd.index(v.name)
                    if ai >= 0:
                        if typ is None:
                            typ = sd.attrs[ai][1]
                            slot = i
                        else:
                            raise SiddhiAppValidationException(
                                f"attribute '{v.name}' is ambiguous across pattern states")
            else:
                sd = self.slots[current][0]
                ai = sd.index(v.name)
                if ai < 0:
                    raise SiddhiAppValidationException(f"no attribute '{v.name}' in {sd.name}")
                slot = current
                typ = sd.attrs[ai][1]
        else:
            for i, (sd, ref, mv) in enumerate(self.slots):
                if ref is None:
                    if sd.name == v.stream:
                        ai = sd.index(v.name)
                        if ai < 0:
                            raise SiddhiAppValidationException(f"no attribute '{v.name}' in {sd.name}")
                        slot, typ = i, sd.attrs[ai][1]
                        break
                elif ref == v.stream:
                    ai = sd.index(v.name)
                    if ai < 0:
                        raise SiddhiAppValidationException(f"no attribute '{v.name}' in {sd.name}")
                    slot, typ = i, sd.attrs[ai][1]
                    if current > -1 and self.slots[current][1] is not None and v.index is not None \
                            and v.index <= LAST:
                        if v.stream == self.slots[current][1]:
                            chain = v.index
                    elif current == UNKNOWN_STATE and v.index is None:
                        multi = mv
                    break
        if slot < 0:
            raise SiddhiAppValidationException(
                f"no matching stream reference for attribute '{v.name}'")
        self.last_multi = bool(multi)
        sd = self.slots[slot][0]
        return slot, chain, sd.index(v.name), typ

    def expr(self, e, current, default_index) -> int:
        if isinstance(e, EConst):
            t = e.type
            return self._e(op=0, type=t, is_null=1 if e.is_null else 0, cval=self.const_bits(e))
        if isinstance(e, EVar):
            if current == HAVING_STATE:
                if e.stream is None and e.index is None and e.name in self.out_alias:
                    o, t = self.out_alias[e.name]
                    return self._e(op=20, type=t, attr=o)
                current = UNKNOWN_STATE
            slot, chain, attr, typ = self.resolve_var(e, current, default_index)
            if self.last_multi:
                # MultiValueVariableFunctionExecutor: a List of the chain's values
                # (ExpressionParser.java:1385-1437); only a select output may hold it
                if not self.multi_ok:
                    raise UnsupportedQuery("multi-value (List) attribute inside an expression")
                return self._e(op=21, type=OBJECT, slot=slot, chain=chain, attr=attr, ltype=typ)
            return self._e(op=1, type=typ, slot=slot, chain=chain, attr=attr)
        if isinstance(e, EStreamRef):
            raise UnsupportedQuery("bare stream reference outside `is null`")
        if isinstance(e, EIsNull):
            x = e.x
            if isinstance(x, EStreamRef) or (isinstance(x, EVar) and getattr(x, "_bare", False)
                                            and self._is_ref(x.name)):
                name = x.stream if isinstance(x, EStreamRef) else x.name
                idx = x.index
                slot = self._ref_slot(name)
                chain = CURRENT if idx is None else (idx + 1 if idx <= LAST else idx)
                return self._e(op=17, type=BOOL, slot=slot, chain=chain)
            c = self.expr(x, current, default_index)
            return self._e(op=16, type=BOOL, lhs=c)
        if isinstance(e, ENot):
            c = self.expr(e.x, current, default_index)
            self._want_bool(c)
            return self._e(op=4, type=BOOL, lhs=c)
        if isinstance(e, EBin):
            if e.op in ("and", "or"):
                l = self.expr(e.l, current, default_index)
                r = self.expr(e.r, current, default_index)
                self._want_bool(l)
                self._want_bool(r)
                return self._e(op=2 if e.op == "and" else 3, type=BOOL, lhs=l, rhs=r)
            l = self.expr(e.l, current, default_index)
            r = self.expr(e.r, current, default_index)
            lt, rt = self.etype(l), self.etype(r)
            if e.op in ("==", "!=", ">", ">=", "<", "<="):
                op = {"==": 5, "!=": 6, ">": 7, ">=": 8, "<": 9, "<=": 10}[e.op]
                self._check_compare(e.op, lt, rt)
                return self._e(op=op, type=BOOL, lhs=l, rhs=r, ltype=lt, rtype=rt)
            op = {"+": 11, "-": 12, "*": 13, "/": 14, "%": 15}[e.op]
            rtp = self._arith_type(lt, rt)
            return self._e(op=op, type=rtp, lhs=l, rhs=r, ltype=lt, rtype=rt)
        if isinstance(e, EFunc):
            n = e.name.lower()
            if n == "ifthenelse" and len(e.args) == 3:
                c = self.expr(e.args[0], current, default_index)
                a = self.expr(e.args[1], current, default_index)
                b = self.expr(e.args[2], current, default_index)
                if self.etype(a) != self.etype(b):
                    raise SiddhiAppValidationException("ifThenElse branches must have one type")
                return self._e(op=18, type=self.etype(a), lhs=c, rhs=a, third=b)
            inst = {"instanceoffloat": FLOAT, "instanceofinteger": INT, "instanceoflong": LONG,
                    "instanceofdouble": DOUBLE, "instanceofstring": STRING, "instanceofboolean": BOOL}
            if n in inst and len(e.args) == 1:
                # function/InstanceOf*FunctionExecutor: `value instanceof T` -- with static
                # types, true iff the argument has type T and is not null
                a = self.expr(e.args[0], current, default_index)
                if self.etype(a) != inst[n]:
                    return self._e(op=0, type=BOOL, cval=0)
                return self._e(op=4, type=BOOL, lhs=self._e(op=16, type=BOOL, lhs=a))
            raise UnsupportedQuery(f"function {e.name}() is out of scope")
        raise UnsupportedQuery(f"expression {e!r}")

    def _is_ref(self, name):
        return any(ref == name for (_, ref, _) in self.slots)

    def _ref_slot(self, name):
        for i, (sd, ref, _) in enumerate(self.slots):
            if ref == name or (ref is None and sd.name == name):
                return i
        raise SiddhiAppValidationException(f"unknown stream reference {name}")

    def _want_bool(self, i):
        if self.etype(i) != BOOL:
            raise SiddhiAppValidationException("condition must be BOOL")

    @staticmethod
    def _check_compare(op, lt, rt):
        num = (INT, LONG, FLOAT, DOUBLE)
        if lt in num and rt in num:
            return
        if op in ("==", "!=") and lt == rt and lt in (STRING, BOOL):
            return
        if lt == OBJECT or rt == OBJECT:
            return
        raise SiddhiAppValidationException(f"cannot compare {TYPE_STR[lt]} {op} {TYPE_STR[rt]}")

    @staticmethod
    def _arith_type(lt, rt):
        order = {INT: 0, LONG: 1, FLOAT: 2, DOUBLE: 3}
        if lt not in order or rt not in order:
            raise SiddhiAppValidationException("arithmetic on non-numeric attribute")
        return lt if order[lt] >= order[rt] else rt

    def out_attr(self, oa: OutAttr):
        e = oa.expr
        if isinstance(e, EFunc) and e.name.lower() in ("sum", "avg", "count", "max", "min"):
            n = e.name.lower()
            if n == "count":
                return dict(expr=-1, agg=3, type=LONG)
            a = self.expr(e.args[0], UNKNOWN_STATE, 0)
            at = self.etype(a)
            if n == "sum":
                return dict(expr=a, agg=1, type=LONG if at in (INT, LONG) else DOUBLE)
            if n == "avg":
                return dict(expr=a, agg=2, type=DOUBLE)
            return dict(expr=a, agg=4 if n == "max" else 5, type=at)
        # a bare count-state attribute may select a List (MultiValueVariableFunctionExecutor)
        self.multi_ok = isinstance(e, EVar)
        try:
            x = self.expr(e, UNKNOWN_STATE, 0)
        finally:
            self.multi_ok = False
        return dict(expr=x, agg=0, type=self.etype(x))


class StringDict:
    """Host-side string dictionary (one per app runtime): string <-> int32 id."""

    def __init__(self):
        self._ids: Dict[str, int] = {}
        self._strs: List[str] = []

    def id(self, s) -> int:
        if s is None:
            return -1
        s = str(s)
        i = self._ids.get(s)
        if i is None:
            i = len(self._strs)
            self._ids[s] = i
            self._strs.append(s)
        return i

    def str(self, i: int) -> str:
        return self._strs[i]

    def __len__(self):
        return len(self._strs)


@dataclass
class CompiledQuery:
    query: Query
    elems: List[dict]
    exprs: List[dict]
    outs: List[dict]
    root: int
    n_slots: int
    slot_streams: List[str]
    out_names: List[str]
    out_types: List[int]
    output_stream: int
    having: int = -1
    order: list = field(default_factory=list)   # [(expr index, desc)]
    limit: int = -1
    offset: int = -1
    out_elem_types: List[int] = field(default_factory=list)  # OBJECT (List) outputs: element type, else -1
    group: List[int] = field(default_factory=list)           # group-by expression roots


@dataclass
class CompiledApp:
    app: App
    queries: List[CompiledQuery]
    strings: StringDict
    output_streams: List[str]
    _keep: list = field(default_factory=list)

    def descriptor(self) -> abi.sh_app_desc:
        """Build the C-ABI sh_app_desc (buffers kept alive on self)."""
        app = self.app
        keep = []
        streams = (abi.sh_stream_def * len(app.stream_order))()
        for i, name in enumerate(app.stream_order):
            sd = app.streams[name]
            types = (ctypes.c_int32 * len(sd.attrs))(*[t for _, t in sd.attrs])
            keep.append(types)
            streams[i].n_attrs = len(sd.attrs)
            streams[i].attr_types = types
        qs = (abi.sh_query_desc * len(self.queries))()
        for qi, cq in enumerate(self.queries):
            el = (abi.sh_state_elem * len(cq.elems))()
            for j, d in enumerate(cq.elems):
                for k, v in d.items():
                    setattr(el[j], k, v)
            ex = (abi.sh_expr * max(1, len(cq.exprs)))()
            for j, d in enumerate(cq.exprs):
                for k, v in d.items():
                    if k == "cval":
                        v = ctypes.c_int64(v & 0xFFFFFFFFFFFFFFFF).value
                    setattr(ex[j], k, v)
            ou = (abi.sh_output_attr * max(1, len(cq.outs)))()
            for j, d in enumerate(cq.outs):
                for k, v in d.items():
                    setattr(ou[j], k, v)
            keep += [el, ex, ou]
            q = qs[qi]
            q.state_type = cq.query.state_type
            q.root = cq.root
            q.n_elems = len(cq.elems)
            q.n_exprs = len(cq.exprs)
            q.n_outputs = len(cq.outs)
            q.n_slots = cq.n_slots
            q.partition = cq.query.partition
            q.output_stream = cq.output_stream
            q.within_ms = cq.query.within_ms
            q.having = cq.having
            q.n_order = len(cq.order)
            q.order_desc = 0
            for i, (ei, desc) in enumerate(cq.order):
                q.order_expr[i] = ei
                q.order_desc |= (1 << i) if desc else 0
            q.limit = cq.limit
            q.offset = cq.offset
            if cq.query.rate:
                q.rate_kind, q.rate_value = cq.query.rate
            q.n_group = len(cq.group)
            for i, ei in enumerate(cq.group):
                q.group_expr[i] = ei
            q.elems = el
            q.exprs = ex
            q.outputs = ou
        ns = len(app.stream_order)
        np_ = len(app.partitions)
        ps = (ctypes.c_uint8 * max(1, np_ * ns))()
        pa = (ctypes.c_int32 * max(1, np_ * ns))()
        for p, spec in enumerate(app.partitions):
            for s, name in enumerate(app.stream_order):
                ps[p * ns + s] = 1 if name in spec else 0
                # -1 for a range partition: the host computes the keys from the ranges
                pa[p * ns + s] = (app.streams[name].index(spec[name])
                                  if name in spec and isinstance(spec[name], str) else -1)
        keep += [streams, qs, ps, pa]
        d = abi.sh_app_desc()
        d.version = abi.SH_DESC_VERSION
        d.n_streams = ns
        d.n_queries = len(self.queries)
        d.n_partitions = np_
        d.playback = 1 if app.playback else 0
        d.streams = streams
        d.queries = qs
        d.partition_streams = ps
        d.partition_attr = pa
        self._keep = keep
        return d


def compile_app(text: str, strings: Optional[StringDict] = None) -> CompiledApp:
    app = parse(text)
    strings = strings or StringDict()
    low = Lowerer(app, strings)
    out_streams: List[str] = []
    cqs = []
    for q in app.queries:
        if q.partition >= 0:
            spec = app.partitions[q.partition]
            for sname in spec:
                if sname not in app.streams:
                    raise SiddhiAppValidationException(f"partition stream {sname} undefined")
                if isinstance(spec[sname], RangeSpec):
                    from .hostexpr import RangeEvaluator
                    ev = RangeEvaluator(app.streams[sname], sname)
                    probe = [None] * len(app.streams[sname].attrs)
                    for cond, _ in spec[sname].ranges:
                        ev.cond(cond, probe)  # validates attributes and types on an all-null row
                elif app.streams[sname].index(spec[sname]) < 0:
                    raise SiddhiAppValidationException(f"partition attribute {spec[sname]} undefined")
        root, outs = low.lower_query(q)
        if q.output not in out_streams:
            out_streams.append(q.output)
        cqs.append(CompiledQuery(
            query=q, elems=low.elems, exprs=low.exprs, outs=outs, root=root,
            n_slots=len(low.slots), slot_streams=[sd.name for sd, _, _ in low.slots],
            out_names=[o.name for o in q.select], out_types=[o["type"] for o in outs],
            output_stream=out_streams.index(q.output), having=low.having,
            order=low.order, limit=low.limit, offset=low.offset, group=low.group,
            out_elem_types=[low.exprs[o["expr"]]["ltype"] if o["expr"] >= 0 and o["agg"] == 0
                            and low.exprs[o["expr"]]["op"] == 21 else -1 for o in outs]))
    # a stream may be keyed by at most one partition (one key array per batch)
    owner = {}
    for p, spec in enumerate(app.partitions):
        for s in spec:
            if s in owner and owner[s] != p:
                raise UnsupportedQuery(f"stream {s} partitioned twice")
            owner[s] = p
    # a range partition hands each query inside it the expanded stream (one copy of
    # an event per range that holds, none when no range does), while a query outside
    # it reads the original stream (PartitionStreamReceiver feeds only the
    # partition's own junction): one batch cannot serve both, so such apps stay on
    # the Java runtime
    for cq in cqs:
        for sname in set(cq.slot_streams):
            p = owner.get(sname)
            if p is not None and isinstance(app.partitions[p][sname], RangeSpec) and cq.query.partition != p:
                raise UnsupportedQuery(f"stream {sname} is range-partitioned and also read outside the partition")
    app.output_streams = out_streams
    return CompiledApp(app, cqs, strings, out_streams)
