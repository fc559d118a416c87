"""Vectorised restatement of the select-clause aggregators over an ordered match
stream, for full-size checks of the fast engines' aggregate post-pass.

QuerySelector.processInBatchNoGroupBy (QuerySelector.java:271-313) with one state
event per chunk emits every match with the running aggregate of its partition
key (and query): sum of float / double and avg add `(double) x` one match at a
time (SumAttributeAggregatorExecutor.java:167-185, AvgAttributeAggregatorExecutor.java:
145-155, avg = value / count), sum of int / long adds in long, count() counts.
numpy's add.accumulate is a left-to-right loop of IEEE double additions, so a
per-key cumsum in match order is the reference's arithmetic."""
import numpy as np


def running(group, x, kind):
    """group: per row the (query, key) segment; x: per row the addend (float64,
    or int64 for long sums); kind: 'sum' | 'avg' | 'count'. Returns the running
    values (float64, or int64 for count and long sums) in row order."""
    n = len(group)
    order = np.argsort(group, kind="stable")
    g = group[order]
    starts = np.flatnonzero(np.r_[True, g[1:] != g[:-1]]) if n else np.zeros(0, np.int64)
    ends = np.r_[starts[1:], n] if n else np.zeros(0, np.int64)
    out = np.empty(n, np.int64 if (kind == "count" or x.dtype == np.int64) else np.float64)
    xs = x[order] if x is not None else None
    for a, b in zip(starts, ends):
        if kind == "count":
            r = np.arange(1, b - a + 1, dtype=np.int64)
        elif kind == "avg":
            r = np.add.accumulate(xs[a:b]) / np.arange(1, b - a + 1, dtype=np.float64)
        else:
            r = np.add.accumulate(xs[a:b])
        out[order[a:b]] = r
    return out


def raw_bits(v):
    """raw 8-byte row value of a running aggregate (double bits / long)"""
    return v.view(np.int64) if v.dtype == np.float64 else v.astype(np.int64)
