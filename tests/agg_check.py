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
    values (float64, or int64 for count and long sums) in row order. The groups
    are laid out as the rows of a padded 2-D array and accumulated along its
    columns: each group is still a left-to-right chain of additions."""
    n = len(group)
    out_t = np.int64 if (kind == "count" or (x is not None and x.dtype == np.int64)) else np.float64
    if n == 0:
        return np.zeros(0, out_t)
    order = np.argsort(group, kind="stable")
    g = group[order]
    starts = np.flatnonzero(np.r_[True, g[1:] != g[:-1]])
    lens = np.diff(np.r_[starts, n])
    gi = np.repeat(np.arange(len(starts)), lens)            # group index per sorted row
    col = np.arange(n) - np.repeat(starts, lens)             # position inside its group
    ordinal = (col + 1).astype(np.int64)
    out = np.empty(n, out_t)
    if kind == "count":
        out[order] = ordinal
        return out
    grid = np.zeros((len(starts), int(lens.max())), x.dtype)
    grid[gi, col] = x[order]
    acc = np.add.accumulate(grid, axis=1)[gi, col]
    out[order] = acc / ordinal.astype(np.float64) if kind == "avg" else acc
    return out


def raw_bits(v):
    """raw 8-byte row value of a running aggregate (double bits / long)"""
    return v.view(np.int64) if v.dtype == np.float64 else v.astype(np.int64)
