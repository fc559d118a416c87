#!/usr/bin/env python3
"""Generate golden fixtures (JSON data) from the reference's own known-answer tests.

Reads the reference's TestNG test classes AS TEXT (study, not execution) from
/root/reference and writes, per @Test method it can interpret, one fixture:
    app text (SiddhiQL input), the ordered send/sleep actions, the callback it
    listens on, and the asserted outputs (event count and asserted data rows).
No reference source is copied into the fixtures: only inputs and expected outputs.

Run here (the reference is not present on the GPU box):
    python tests/golden/extract_fixtures.py
Output: tests/golden/fixtures.json (committed).

Timing model (documented in DESIGN.md): non-playback tests stamp each send with a
virtual clock advanced by Thread.sleep(ms); playback tests use their explicit
timestamps. Asserted rows keep their guard (`case k:` / `inEventCount == k`) when
the test pins an index, else they are checked as "must appear".
"""
import json
import os
import re
import sys

REF = "/root/reference/modules/siddhi-core/src/test/java/io/siddhi/core/"
FILES = [
    "query/pattern/WithinPatternTestCase.java",
    "query/pattern/EveryPatternTestCase.java",
    "query/pattern/CountPatternTestCase.java",
    "query/pattern/LogicalPatternTestCase.java",
    "query/pattern/ComplexPatternTestCase.java",
    "query/sequence/SequenceTestCase.java",
    "query/partition/PatternPartitionTestCase.java",
    "query/partition/SequencePartitionTestCase.java",
    "query/pattern/absent/AbsentPatternTestCase.java",
    "query/pattern/absent/EveryAbsentPatternTestCase.java",
    "query/pattern/absent/AbsentWithEveryPatternTestCase.java",
    "query/sequence/absent/AbsentSequenceTestCase.java",
    "query/pattern/absent/LogicalAbsentPatternTestCase.java",
    "query/sequence/absent/LogicalAbsentSequenceTestCase.java",
    "query/sequence/absent/EveryAbsentSequenceTestCase.java",
    "query/sequence/absent/AbsentWithEverySequenceTestCase.java",
]

# `long now = System.currentTimeMillis();` in playback tests: any base works (the
# asserted outputs depend on differences only); a fixed one keeps fixtures stable
TIME_BASE = 1_700_000_000_000

TOKEN = re.compile(r'''
    (?P<ws>\s+|//[^\n]*|/\*.*?\*/)
  | (?P<str>"(?:[^"\\]|\\.)*")
  | (?P<chr>'(?:[^'\\]|\\.)')
  | (?P<num>-?(?:\d+\.\d*|\.\d+|\d+)(?:[eE][-+]?\d+)?[lLfFdD]?)
  | (?P<id>[A-Za-z_][A-Za-z0-9_.]*)
  | (?P<op>==|!=|>=|<=|\+\+|\+=|&&|\|\||->|[-+*/%<>=(),;\[\]{}:?!&|])
''', re.VERBOSE | re.DOTALL)


def tokens(src):
    out = []
    i = 0
    while i < len(src):
        m = TOKEN.match(src, i)
        if not m:
            i += 1
            continue
        k = m.lastgroup
        if k != "ws":
            out.append((k, m.group(k), i))
        i = m.end()
    return out


def jstr(lit):
    return bytes(lit[1:-1], "utf-8").decode("unicode_escape")


def line_of(src, pos):
    return src.count("\n", 0, pos) + 1


def value(tok):
    """Java literal -> tagged JSON value."""
    k, t, _ = tok
    if k == "str":
        return jstr(t)
    if k == "num":
        low = t.lower()
        if low.endswith("f"):
            return {"f": t[:-1]}
        if low.endswith("l"):
            return {"l": int(t[:-1])}
        if low.endswith("d"):
            return {"d": t[:-1]}
        if "." in t or "e" in low:
            return {"d": t}
        return int(t)
    if k == "id":
        if t == "null":
            return None
        if t in ("true", "false"):
            return t == "true"
    raise ValueError(f"unsupported literal {t}")


class Skip(Exception):
    pass


def parse_object_array(toks, i):
    """toks[i] == 'new' ... 'Object' '[' ']' '{' v, v '}' -> (values, next index)"""
    assert toks[i][1] == "new"
    if toks[i + 1][1] not in ("Object",):
        raise Skip("non Object[] literal")
    j = i + 2
    while toks[j][1] != "{":
        j += 1
    j += 1
    vals = []
    while toks[j][1] != "}":
        if toks[j][1] == ",":
            j += 1
            continue
        # unary minus before number token handled by regex; casts like (Object) skip
        if toks[j][1] == "(":
            raise Skip("expression inside Object[]")
        if toks[j][1] == "new":
            # a nested Object[] (the List value of a multi-value select, compared
            # through Arrays.deepToString)
            inner, j = parse_object_array(toks, j)
            vals.append(inner)
            continue
        if toks[j + 1][1] not in (",", "}"):
            raise Skip("expression inside Object[]")
        vals.append(value(toks[j]))
        j += 1
    return vals, j + 1


def method_bodies(src):
    for m in re.finditer(r"@Test[^\n]*\n\s*public void (\w+)\([^)]*\)[^{]*\{", src):
        start = m.end()
        depth = 1
        i = start
        while depth:
            c = src[i]
            if c == '"':
                i += 1
                while src[i] != '"':
                    if src[i] == "\\":
                        i += 1
                    i += 1
            elif c == "{":
                depth += 1
            elif c == "}":
                depth -= 1
            i += 1
        yield m.group(1), m.start(), src[start:i - 1], start


def extract(fname):
    src = open(os.path.join(REF, fname)).read()
    out = []
    for name, mpos, body, bstart in method_bodies(src):
        fx = {"id": f"{os.path.basename(fname)[:-5]}.{name}",
              "source": f"modules/siddhi-core/src/test/java/io/siddhi/core/{fname}:{line_of(src, mpos)}"}
        try:
            fx.update(interpret(body))
            out.append(fx)
        except Skip as e:
            fx["skipped"] = str(e)
            out.append(fx)
        except Exception as e:  # noqa
            fx["skipped"] = f"extractor: {type(e).__name__}: {e}"
            out.append(fx)
    return out


def interpret(body):
    toks = tokens(body)
    strs = {}
    handlers = {}
    actions = []
    app = None
    callbacks = []
    expect_count = None
    rows = []
    started = False
    shut = False
    i = 0
    n = len(toks)
    # guard tracking for assertArrayEquals: last `case K:` or `== K` seen in callback
    guard = None
    in_callback_depth = None
    depth = 0
    cb_kind = None
    if "siddhiAppRuntime.persist" in body or "restoreRevision" in body or ".persist()" in body:
        raise Skip("persistence test (next row, SURVEY 8f)")
    if "getInputHandler" not in body:
        raise Skip("no input handler")
    tv = {}  # long time variables of the test body (playback timestamps)
    while i < n:
        k, t, _ = toks[i]
        # long X = System.currentTimeMillis(); / long X = 123L;
        if k == "id" and t == "long" and toks[i + 1][0] == "id" and toks[i + 2][1] == "=":
            var = toks[i + 1][1]
            if toks[i + 3][1] == "System.currentTimeMillis":
                tv[var] = TIME_BASE
                i += 7
                continue
            j = i + 3
            expr = []
            while toks[j][1] != ";":
                expr.append(toks[j])
                j += 1
            tv[var] = int_expr(expr, tv)
            i = j + 1
            continue
        # X += e; X -= e; X = e; X++; ++X;
        if k == "id" and t in tv and toks[i + 1][1] in ("+=", "=", "-", "++"):
            op = toks[i + 1][1]
            if op == "++":
                tv[t] += 1
                i += 2
                continue
            if op == "-" and toks[i + 2][1] == "=":
                j = i + 3
                sign = -1
            elif op == "-":
                i += 1
                continue
            else:
                j = i + 2
                sign = 1
            expr = []
            while toks[j][1] != ";":
                expr.append(toks[j])
                j += 1
            v = int_expr(expr, tv)
            tv[t] = tv[t] + sign * v if op in ("+=", "-") else v
            i = j + 1
            continue
        if t == "++" and toks[i + 1][0] == "id" and toks[i + 1][1] in tv and toks[i + 2][1] == ";":
            tv[toks[i + 1][1]] += 1
            i += 3
            continue
        if t == "{":
            depth += 1
        elif t == "}":
            depth -= 1
            if in_callback_depth is not None and depth < in_callback_depth:
                in_callback_depth = None
        # String X = "..." + "..." + Y;   /  X = ...;  / X += ...;
        if k == "id" and t == "String" and toks[i + 1][0] == "id" and toks[i + 2][1] == "=":
            var = toks[i + 1][1]
            s, i = concat(toks, i + 3, strs)
            strs[var] = s
            continue
        if k == "id" and t in strs and toks[i + 1][1] in ("=", "+="):
            op = toks[i + 1][1]
            s, i = concat(toks, i + 2, strs)
            strs[t] = (strs[t] + s) if op == "+=" else s
            continue
        if t.endswith("createSiddhiAppRuntime") and toks[i + 1][1] == "(":
            s, j = concat(toks, i + 2, strs, stop=")")
            app = s
            i = j
            continue
        if t.endswith("addCallback") and toks[i + 1][1] == "(" and toks[i + 2][0] == "str":
            cbname = jstr(toks[i + 2][1])
            kind = None
            j = i + 3
            while j < n and toks[j][1] not in ("QueryCallback", "StreamCallback"):
                j += 1
            kind = "query" if toks[j][1] == "QueryCallback" else "stream"
            callbacks.append({"kind": kind, "name": cbname})
            in_callback_depth = depth + 1
            cb_kind = kind
            i += 3
            continue
        if t in ("TestUtil.addQueryCallback", "TestUtil.addStreamCallback") and toks[i + 1][1] == "(":
            j = i + 2
            while toks[j][0] != "str":
                j += 1
            callbacks.append({"kind": "query" if "Query" in t else "stream", "name": jstr(toks[j][1])})
            j += 1
            idx = 1
            while toks[j][1] != ")":
                if toks[j][1] == "new":
                    vals, j = parse_object_array(toks, j)
                    rows.append({"guard": idx, "row": vals, "first_of_callback": False})
                    idx += 1
                    continue
                j += 1
            i = j
            continue
        if t == "TestUtil.waitForInEvents" and toks[i + 2][0] == "num":
            actions.append(["wait_in_events", int(toks[i + 2][1].rstrip("lL")), int(toks[i + 6][1])])
            i += 7
            continue
        if t == "SiddhiTestHelper.waitForEvents" and toks[i + 2][0] == "num" and toks[i + 4][0] == "num":
            actions.append(["wait_for_events", int(toks[i + 2][1].rstrip("lL")), int(toks[i + 4][1]),
                            int(toks[i + 8][1].rstrip("lL")) if toks[i + 8][0] == "num" else 60000])
            i += 5
            continue
        if k == "id" and t == "InputHandler" and toks[i + 1][0] == "id":
            var = toks[i + 1][1]
            j = i + 2
            while toks[j][0] != "str":
                j += 1
            handlers[var] = jstr(toks[j][1])
            i = j + 1
            continue
        if k == "id" and t.endswith(".start") and "Runtime" in t or t == "siddhiAppRuntime.start":
            started = True
        if k == "id" and "." in t and t.split(".")[0] in handlers and t.endswith(".send"):
            h = t.split(".")[0]
            j = i + 2
            ts = None
            if toks[j][0] == "num" and toks[j + 1][1] == ",":
                ts = int(value(toks[j])["l"]) if isinstance(value(toks[j]), dict) else int(value(toks[j]))
                j += 2
            elif toks[j][1] != "new":
                # a timestamp expression over the time variables: ++now, now++, now + 100
                depth0 = 0
                expr = []
                while not (toks[j][1] == "," and depth0 == 0):
                    if toks[j][1] == "(":
                        depth0 += 1
                    elif toks[j][1] == ")":
                        depth0 -= 1
                    expr.append(toks[j])
                    j += 1
                ts = ts_expr(expr, tv)
                j += 1
            if toks[j][1] != "new":
                raise Skip("send of non-literal event")
            if toks[j + 1][1] == "Event":
                raise Skip("send(Event[])")
            vals, j = parse_object_array(toks, j)
            if not shut:
                actions.append(["send", handlers[h], ts, vals])
            i = j
            continue
        if k == "id" and t.endswith(".shutdown") and started and in_callback_depth is None:
            # the runtime is gone: later sleeps and sends reach nothing (count
            # assertions after this point are still read)
            shut = True
        if t == "Thread.sleep" and toks[i + 2][0] == "num":
            if not shut:
                actions.append(["sleep", int(toks[i + 2][1].rstrip("lL"))])
            i += 3
            continue
        if in_callback_depth is not None:
            if t == "case" and toks[i + 1][0] == "num":
                guard = int(toks[i + 1][1])
            if t == "==" and toks[i + 1][0] == "num" and toks[i - 1][1] in ("inEventCount", ")", "count"):
                guard = int(toks[i + 1][1])
            if t.endswith("assertEquals") and toks[i + 1][1] == "(":
                # assertEquals(event.getData(k), literal) / assertEquals(literal, event.getData(k))
                fld = field_assert(toks, i + 2)
                if fld is not None:
                    idx, val, j = fld
                    if rows and rows[-1].get("fields") is not None and rows[-1]["guard"] == guard:
                        rows[-1]["fields"][str(idx)] = val
                    else:
                        rows.append({"guard": guard, "fields": {str(idx): val}, "row": None,
                                     "first_of_callback": False})
                    i = j
                    continue
            if t.endswith("assertEquals") and toks[i + 1][1] == "(" and toks[i + 2][1] == "Arrays.deepToString" \
                    and toks[i + 4][1] == "new":
                # assertEquals(Arrays.deepToString(new Object[]{new Object[]{..}, ..}),
                #              Arrays.deepToString(event.getData()))
                vals, j = parse_object_array(toks, i + 4)
                rows.append({"guard": guard, "row": vals, "first_of_callback": False})
                i = j
                continue
            if t.endswith("assertArrayEquals") and toks[i + 1][1] == "(":
                vals, j = parse_object_array(toks, i + 2)
                # which event: inEvents[0] / events[0] / event
                rest = " ".join(x[1] for x in toks[j:j + 6])
                first_only = "[ 0 ]" in rest or "[0]" in rest
                rows.append({"guard": guard, "row": vals, "first_of_callback": first_only})
                i = j
                continue
        else:
            if t.endswith("assertEquals") and toks[i + 1][1] == "(":
                # assertEquals("Number of success events", N, inEventCount[.get()])
                j = i + 2
                if toks[j][0] == "str":
                    msg = jstr(toks[j][1]).lower()
                    j += 2
                else:
                    msg = ""
                if toks[j][0] == "id" and toks[j + 1][1] == "," and toks[j + 2][0] == "num" and \
                        toks[j + 3][1] == ")" and toks[j][1].startswith(("inEventCount", "count", "eventCount")):
                    # assertEquals(inEventCount, N)
                    if toks[j][1].startswith("inEventCount") or expect_count is None:
                        expect_count = int(toks[j + 2][1])
                    i = j + 3
                    continue
                if toks[j][0] == "num" and toks[j + 1][1] == ",":
                    var = toks[j + 2][1]
                    if ("success" in msg or msg == "" or "in event" in msg) and (
                            var.startswith("inEventCount") or var == "callback.getInEventCount"):
                        expect_count = int(toks[j][1])
                    elif ("number of events" in msg or msg == "") and var.startswith(("count", "eventCount")):
                        if expect_count is None:
                            expect_count = int(toks[j][1])
                i = j
                continue
        i += 1
    if app is None:
        raise Skip("no app string")
    if not callbacks:
        raise Skip("no callback")
    if len(callbacks) > 1:
        raise Skip("multiple callbacks")
    if expect_count is None:
        raise Skip("no asserted event count")
    return {"app": app, "actions": actions, "callback": callbacks[0],
            "expect_count": expect_count, "expect_rows": rows}


def int_expr(expr, tv):
    """integer arithmetic over numbers and time variables (no side effects)"""
    parts = []
    for k, t, _ in expr:
        if k == "num":
            parts.append(t.rstrip("lL"))
        elif k == "id" and t in tv:
            parts.append(str(tv[t]))
        elif t in ("+", "-", "*", "/", "(", ")"):
            parts.append("//" if t == "/" else t)
        elif k == "id" and t in ("long", "int"):
            continue
        else:
            raise Skip(f"timestamp expression near {t}")
    return int(eval("".join(parts), {"__builtins__": {}}, {}))


def ts_expr(expr, tv):
    """send(ts, ...) first argument: ++X, X++, X, or an arithmetic expression"""
    ts = [t for _, t, _ in expr]
    if len(ts) == 2 and ts[0] == "++" and ts[1] in tv:
        tv[ts[1]] += 1
        return tv[ts[1]]
    if len(ts) == 2 and ts[1] == "++" and ts[0] in tv:
        v = tv[ts[0]]
        tv[ts[0]] += 1
        return v
    return int_expr(expr, tv)


def field_assert(toks, j):
    """(index, literal value, next index) of assertEquals(e.getData(k), v) in either order, else None"""
    def getdata(at):
        if toks[at][0] == "id" and toks[at][1].endswith(".getData") and toks[at + 1][1] == "(" and \
                toks[at + 2][0] == "num" and toks[at + 3][1] == ")":
            return int(toks[at + 2][1]), at + 4
        return None
    g = getdata(j)
    if g is not None and toks[g[1]][1] == ",":
        try:
            v = value(toks[g[1] + 1])
        except ValueError:
            return None
        if toks[g[1] + 2][1] != ")":
            return None
        return g[0], v, g[1] + 3
    if toks[j + 1][1] == ",":
        g = getdata(j + 2)
        if g is not None and toks[g[1]][1] == ")":
            try:
                v = value(toks[j])
            except ValueError:
                return None
            return g[0], v, g[1] + 1
    return None


def concat(toks, i, strs, stop=";"):
    parts = []
    while toks[i][1] != stop:
        k, t, _ = toks[i]
        if k == "str":
            parts.append(jstr(t))
        elif k == "id" and t in strs:
            parts.append(strs[t])
        elif t in ("+", "(", ")"):
            pass
        else:
            raise Skip(f"non-literal string expression near {t}")
        i += 1
    return "".join(parts), i + 1


def main():
    all_fx = []
    for f in FILES:
        all_fx.extend(extract(f))
    here = os.path.dirname(os.path.abspath(__file__))
    with open(os.path.join(here, "fixtures.json"), "w") as fh:
        json.dump(all_fx, fh, indent=1)
    ok = [x for x in all_fx if "skipped" not in x]
    print(f"{len(all_fx)} tests scanned, {len(ok)} fixtures, {len(all_fx) - len(ok)} skipped", file=sys.stderr)


if __name__ == "__main__":
    main()
