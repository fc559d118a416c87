"""Host evaluation of range-partition conditions with the reference's executor
semantics (the partition key is computed on the host, like a value partition's
attr.toString(): RangePartitionExecutor.execute returns the range's label when its
ConditionExpressionExecutor is true, core/partition/executor/RangePartitionExecutor.java:38-43).

Typing follows ExpressionParser (core/util/parser/ExpressionParser.java): numeric
operands are promoted int < long < float < double; compares return false when an
operand is null (CompareConditionExpressionExecutor.java:38-42); and/or treat null as
false; not(null) is true (NotConditionExpressionExecutor.java:43-50); integer and
floating `/` and `%` by zero give null (math/divide/*, math/mod/*); int/long
arithmetic wraps like the JVM; float arithmetic rounds to binary32.
"""
from __future__ import annotations

import numpy as np

from . import compiler as cp

_NUM_RANK = {cp.INT: 0, cp.LONG: 1, cp.FLOAT: 2, cp.DOUBLE: 3}


def _wrap(v: int, t: int) -> int:
    bits = 32 if t == cp.INT else 64
    v &= (1 << bits) - 1
    return v - (1 << bits) if v >> (bits - 1) else v


def _as(t: int, v):
    """Number.xxxValue() of a promoted operand"""
    if t == cp.FLOAT:
        return float(np.float32(v))
    if t == cp.DOUBLE:
        return float(v)
    return _wrap(int(v), t)


def _promote(a: int, b: int) -> int:
    return a if _NUM_RANK[a] >= _NUM_RANK[b] else b


def _arith(op: str, t: int, x, y):
    if t in (cp.INT, cp.LONG):
        if op == "+":
            return _wrap(x + y, t)
        if op == "-":
            return _wrap(x - y, t)
        if op == "*":
            return _wrap(x * y, t)
        if y == 0:
            return None
        q = abs(x) // abs(y)  # Java truncates toward zero
        q = q if (x >= 0) == (y >= 0) else -q
        return _wrap(q, t) if op == "/" else _wrap(x - q * y, t)
    if op in ("/", "%") and y == 0.0:
        return None
    if op == "+":
        r = x + y
    elif op == "-":
        r = x - y
    elif op == "*":
        r = x * y
    elif op == "/":
        r = x / y
    else:
        r = float(np.fmod(x, y))
    return float(np.float32(r)) if t == cp.FLOAT else r


class RangeEvaluator:
    """Evaluates one stream's range conditions over a row (list of values in the
    stream's attribute order, None for null)."""

    def __init__(self, sd: cp.StreamDef, stream_name: str):
        self.sd = sd
        self.name = stream_name

    def value(self, e, row):
        """-> (type, value or None)"""
        if isinstance(e, cp.EConst):
            return e.type, (None if e.is_null else e.value)
        if isinstance(e, cp.EVar):
            if e.stream not in (None, self.name) or e.index is not None:
                raise cp.UnsupportedQuery("range partition conditions read the partitioned stream's attributes")
            ai = self.sd.index(e.name)
            if ai < 0:
                raise cp.SiddhiAppValidationException(f"attribute {e.name} undefined in {self.name}")
            t = self.sd.attrs[ai][1]
            v = row[ai] if ai < len(row) else None
            if v is not None and t == cp.FLOAT:
                v = float(np.float32(v))
            return t, v
        if isinstance(e, cp.ENot):
            return cp.BOOL, not self.cond(e.x, row)
        if isinstance(e, cp.EIsNull):
            return cp.BOOL, self.value(e.x, row)[1] is None
        if isinstance(e, cp.EBin):
            if e.op in ("and", "or"):
                a = self.cond(e.l, row)
                if e.op == "and":
                    return cp.BOOL, a and self.cond(e.r, row)
                return cp.BOOL, a or self.cond(e.r, row)
            lt, lv = self.value(e.l, row)
            rt, rv = self.value(e.r, row)
            if e.op in ("==", "!=", ">", ">=", "<", "<="):
                return cp.BOOL, self._compare(e.op, lt, lv, rt, rv)
            if lt not in _NUM_RANK or rt not in _NUM_RANK:
                raise cp.UnsupportedQuery(f"arithmetic on {cp.TYPE_STR[lt]} and {cp.TYPE_STR[rt]}")
            t = _promote(lt, rt)
            if lv is None or rv is None:
                return t, None
            return t, _arith(e.op, t, _as(t, lv), _as(t, rv))
        raise cp.UnsupportedQuery(f"range partition condition {type(e).__name__} is out of scope")

    def _compare(self, op, lt, lv, rt, rv) -> bool:
        if lv is None or rv is None:
            return False
        if lt in _NUM_RANK and rt in _NUM_RANK:
            t = _promote(lt, rt)
            x, y = _as(t, lv), _as(t, rv)
        elif lt == rt and lt in (cp.STRING, cp.BOOL):
            if op not in ("==", "!="):
                raise cp.UnsupportedQuery(f"{op} on {cp.TYPE_STR[lt]}")
            x, y = lv, rv
        else:
            raise cp.UnsupportedQuery(f"compare of {cp.TYPE_STR[lt]} and {cp.TYPE_STR[rt]}")
        return {"==": x == y, "!=": x != y, ">": x > y, ">=": x >= y, "<": x < y, "<=": x <= y}[op]

    def cond(self, e, row) -> bool:
        t, v = self.value(e, row)
        if t != cp.BOOL:
            raise cp.SiddhiAppValidationException("range partition condition is not a bool expression")
        return bool(v) if v is not None else False
