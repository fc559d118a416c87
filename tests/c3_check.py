"""Vectorised restatement of C3 (BASELINE.json configs[2]):

  partition with (symbol of S) begin
    from every e1=S, e2=S[price>e1.price]+, e3=S[price<e2[last].price]
    select e1.price as p1, e2[last].price as peak, e3.price as p3 insert into Out; end;

SEQUENCE semantics per key reduce to one partial (e1, last e2) — see
sh_nfa_lower.cpp detect_seq3 for the processor argument: at each event x,
hit = (a last e2 exists) and x < last -> emit (e1, last, x) and restart at x;
else if x > e1 -> last = x; else restart at x. All keys advance together
(numpy over keys, one step per position inside the key). Checked against the
oracle on CPU in tests/test_c3_checker.py (test infrastructure)."""
import numpy as np


def c3_expected(ts, keys, price):
    n = len(price)
    order = np.argsort(keys, kind="stable")
    sk = keys[order]
    starts = np.flatnonzero(np.r_[True, sk[1:] != sk[:-1]])
    lens = np.diff(np.r_[starts, n])
    nk = len(starts)
    p = price.astype(np.float32)
    e1 = np.zeros(nk, np.float32)
    last = np.zeros(nk, np.float32)
    has_p = np.zeros(nk, bool)
    has_last = np.zeros(nk, bool)
    out_idx, out_e1, out_last, out_x = [], [], [], []
    maxlen = int(lens.max()) if nk else 0
    for j in range(maxlen):
        live = lens > j
        kk = np.flatnonzero(live)
        idx = order[starts[kk] + j]
        x = p[idx]
        hit = has_last[kk] & (x < last[kk])
        if hit.any():
            out_idx.append(idx[hit])
            out_e1.append(e1[kk][hit])
            out_last.append(last[kk][hit])
            out_x.append(x[hit])
        ext = ~hit & has_p[kk] & (x > e1[kk])
        ke, kr = kk[ext], kk[~ext]
        has_last[ke] = True
        last[ke] = x[ext]
        has_last[kr] = False
        e1[kr] = x[~ext]
        has_p[kk] = True
    if not out_idx:
        return np.zeros(0, np.int64), np.zeros((0, 3), np.int64)
    idx = np.concatenate(out_idx)
    o = np.argsort(idx, kind="stable")
    vals = np.stack([np.concatenate(out_e1)[o].view(np.uint32), np.concatenate(out_last)[o].view(np.uint32),
                     np.concatenate(out_x)[o].view(np.uint32)], 1).astype(np.int64)
    return idx[o].astype(np.int64), vals
