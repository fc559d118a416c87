"""Independent vectorised restatement of config C5 (batch-compiled fraud rules),
for full-size checks.

Rule r is query r of one `partition with (card of Txn)`:
  every e1=Txn[amount > A_r and merchant == M_r]
     -> e2=Txn[card == e1.card and amount > e1.amount * F_r] within W_r
Per rule the window reduction of c2_check.py holds (non-decreasing timestamps):
the partial opened at event i is consumed by the first later event j of the card
with f2(i, j), provided ts_j - ts_i <= W_r. Rules meet only in the output order:
PartitionStreamReceiver.receive(Event[]) (core/partition/PartitionStreamReceiver.java:176-216)
hands each run of consecutive same-card events of a send() call to every query in
order and a Multi receiver emits after the whole run
(core/query/input/MultiProcessStreamReceiver.java:95-122), so rows sort by
(run, rule, j, i). Float compares and the double product follow the executors
(float -> double promotion against a double literal). Used by tests/ at sizes the
object-graph oracle cannot finish in seconds; itself checked against the oracle
(tests/test_c5_checker.py).
"""
import numpy as np


def c5_expected(ts, card, amount, merchant, rules, within_ms=1000, batch=4096, free=()):
    """Returns (seq, rule, values[n, 2]) of every match in output order."""
    n = len(ts)
    order = np.argsort(card, kind="stable")
    sk = card[order]
    st = ts[order]
    sa = amount[order].astype(np.float64)
    sm = merchant[order]
    by_m = np.argsort(sm, kind="stable")
    m_sorted = sm[by_m]
    free = set(free)
    P, Q, R = [], [], []
    for r, (a, m, f, w) in enumerate(rules):
        if r in free:
            cand = np.nonzero(sa > a)[0]
        else:
            lo, hi = np.searchsorted(m_sorted, [m, m + 1])
            cand = np.sort(by_m[lo:hi])
            cand = cand[sa[cand] > a]
        wms = w * within_ms
        idx = cand
        d = 1
        while idx.size:
            j = idx + d
            ok = j < n
            idx, j = idx[ok], j[ok]
            ok = sk[j] == sk[idx]
            idx, j = idx[ok], j[ok]
            ok = (st[j] - st[idx]) <= wms
            idx, j = idx[ok], j[ok]
            hit = sa[j] > sa[idx] * f
            P.append(idx[hit])
            Q.append(j[hit])
            R.append(np.full(int(hit.sum()), r, np.int64))
            idx = idx[~hit]
            d += 1
    if not P:
        return np.zeros(0, np.int64), np.zeros(0, np.int32), np.zeros((0, 2), np.int64)
    p = order[np.concatenate(P)]
    q = order[np.concatenate(Q)]
    rr = np.concatenate(R)
    # runs of consecutive same-card events inside each send() call
    start = np.ones(n, bool)
    start[1:] = card[1:] != card[:-1]
    start[::batch] = True
    run = np.cumsum(start) - 1
    srt = np.lexsort((p, q, rr, run[q]))
    p, q, rr = p[srt], q[srt], rr[srt]
    vals = np.empty((len(p), 2), np.int64)
    vals[:, 0] = card[p].astype(np.int64)
    vals[:, 1] = amount[q].view(np.uint32).astype(np.int64)
    return q.astype(np.int64), rr.astype(np.int32), vals
