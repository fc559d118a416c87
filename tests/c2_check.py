"""Independent vectorised restatement of config C2's matches, for full-size checks.

For `every e1=S[price>20] -> e2=S[symbol==e1.symbol and price>e1.price] within W`
partitioned by symbol, with non-decreasing timestamps, the reference's
processors (StreamPreStateProcessor.expireEvents/processAndReturn, PATTERN,
every on the start state, one-event delay of new partials) reduce to:
  each event i with price_i > 20 opens one partial; it is matched by the first
  later event j of the same key with price_j > price_i, provided
  ts_j - ts_i <= W (expiry is checked before matching at every event and the
  pending list is in creation order, so break-early expiry removes exactly the
  over-age partials); output rows are ordered by (j, i).
Used by tests/ at sizes the object-graph oracle cannot finish in seconds.
"""
import numpy as np


def c2_expected(ts, keys, price, vol, within=1000, thr=20):
    n = len(ts)
    order = np.argsort(keys, kind="stable")
    sk = keys[order]
    st = ts[order]
    sp = price[order]
    cand = np.nonzero(sp > np.float32(thr))[0]
    mi = []
    mj = []
    idx = cand
    d = 1
    while idx.size:
        j = idx + d
        ok = j < n
        idx, j = idx[ok], j[ok]
        ok = sk[j] == sk[idx]
        idx, j = idx[ok], j[ok]
        ok = (st[j] - st[idx]) <= within
        idx, j = idx[ok], j[ok]
        hit = sp[j] > sp[idx]
        mi.append(idx[hit])
        mj.append(j[hit])
        idx = idx[~hit]
        d += 1
    mi = np.concatenate(mi) if mi else np.zeros(0, np.int64)
    mj = np.concatenate(mj) if mj else np.zeros(0, np.int64)
    oi = order[mi]
    oj = order[mj]
    srt = np.lexsort((oi, oj))
    oi, oj = oi[srt], oj[srt]
    seq = oj.astype(np.int64)
    vals = np.empty((len(oi), 4), np.int64)
    vals[:, 0] = keys[oi].astype(np.int64)
    vals[:, 1] = price[oi].view(np.uint32).astype(np.int64)
    vals[:, 2] = price[oj].view(np.uint32).astype(np.int64)
    vals[:, 3] = vol[oj]
    return seq, vals
