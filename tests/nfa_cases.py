"""Randomized apps for the general NFA engine: pattern / sequence queries with
Stream, Count (<m:n> + * ?), Logical (and / or) and Absent (`not X for T`)
states, `every`, `within`, partitions and multi-query partitions, driven by
random send() batches and playback time advances. Shared by the CPU suite
(tests/nfa_host vs the oracle) and the GPU suite (libsiddhi_hip.so vs the oracle).
"""
from __future__ import annotations

import random

DEFS = ("define stream S1 (sym string, price float, volume long, x int); "
        "define stream S2 (sym string, price float, volume long, x int); "
        "define stream S3 (sym string, price float, volume long, x int); ")


def _filter(rng, k, aliases):
    opts = ["price > {c}f", "x < {c}", "price >= 10.5", "not (x == {c})", "volume % 3 != 1", "x > 2"]
    refs = [a for a in aliases if a[0] < k]
    if refs:
        a, cnt = rng.choice(refs)[1:]
        # a count state's attribute always indexed: without an index it is a List
        # (MultiValueVariableFunctionExecutor), which no filter expression takes
        idx = rng.choice(["[0]", "[last]"]) if cnt else ""
        opts += [f"price > {a}{idx}.price", f"x < {a}{idx}.x + {{c}}", f"price * 2 > {a}{idx}.price + x",
                 f"{a}{idx}.price - price < {{c}}.0", f"volume >= {a}{idx}.volume"]
    return rng.choice(opts).format(c=rng.randint(1, 20))


def nfa_query(rng, streams, qname, allow_absent, partitioned=False):
    """partitioned: the last state is never a count with min 0 (the device leaves
    that shape -- CountPostStateProcessor.isEventReturned, one field shared by every
    key -- to the reference runtime)"""
    seq = rng.random() < 0.4
    sep = ", " if seq else " -> "
    n = rng.randint(2, 4)
    parts = []
    aliases = []   # (state index, alias, is_count)
    used = set()
    alias_no = 0
    k = 0
    for i in range(n):
        kind = rng.choices(["stream", "count", "logical", "absent"],
                           [5, 2.5, 1.5, 1.5 if allow_absent else 0])[0]
        if kind == "absent" and (i == 0 and rng.random() < 0.5):
            kind = "stream"
        s = rng.choice(streams)
        used.add(s)
        if kind == "absent":
            f = _filter(rng, k, [])
            parts.append(f"not {s}[{f}] for {rng.choice([5, 20, 50])} milliseconds")
            k += 1
            continue
        if kind == "logical":
            s2 = rng.choice(streams)
            used.add(s2)
            a1, a2 = f"e{alias_no}", f"e{alias_no + 1}"
            alias_no += 2
            f1 = _filter(rng, k, aliases)
            f2 = _filter(rng, k, aliases)
            op = rng.choice(["and", "or"])
            parts.append(f"{a1}={s}[{f1}] {op} {a2}={s2}[{f2}]")
            aliases += [(k, a1, False), (k, a2, False)]
            k += 2
            continue
        a = f"e{alias_no}"
        alias_no += 1
        f = _filter(rng, k + 1 if kind == "count" else k, aliases + ([(k, a, True)] if kind == "count" else []))
        src = f"{a}={s}[{f}]"
        if kind == "count":
            min0 = ["<0:2>"] + (["*", "?"] * 2 if seq else [])
            counts = ["<1:3>", "<2:4>", "<2>", "<1:>"] + (["+"] * 2 if seq else [])
            if not (partitioned and i == n - 1):
                counts += min0
            src += rng.choice(counts)
        parts.append(src)
        aliases.append((k, a, kind == "count"))
        k += 1
    if rng.random() < 0.65 and not parts[0].startswith("not"):
        parts[0] = "every " + parts[0]
    within = rng.choice([None, None, 3, 8, 20, 60])
    body = sep.join(parts) + (f" within {within} milliseconds" if within else "")
    sel = []
    for (_, a, cnt) in aliases[:3]:
        idx = rng.choice(["[0]", "[1]", "[last]"]) if cnt else ""
        sel.append(f"{a}{idx}.{rng.choice(['price', 'x', 'sym', 'volume'])} as c{len(sel)}")
    if not sel:
        sel = ["1 as c0"]
    if rng.random() < 0.25 and aliases:
        sel.append(f"sum({aliases[-1][1]}{'[last]' if aliases[-1][2] else ''}.price) as s")
    if rng.random() < 0.15 and aliases:
        sel.append(f"count() as n")
    q = f"@info(name = '{qname}') from {body} select {', '.join(sel)} insert into Out;"
    return q, used


def nfa_case(rng, multi_query=None):
    """Returns (app text, actions); actions are ("send", stream, [(ts, row)]) or
    ("advance", ts)."""
    streams = rng.choice([["S1"], ["S1", "S2"], ["S1", "S2", "S3"]])
    playback = rng.random() < 0.5
    nq = multi_query if multi_query else (rng.choice([1, 1, 1, 2, 3]))
    partitioned = rng.random() < 0.6 or nq > 1
    qs, used = [], set()
    for i in range(nq):
        q, u = nfa_query(rng, streams, f"query{i + 1}", allow_absent=playback, partitioned=partitioned)
        qs.append(q)
        used |= u
    body = " ".join(qs)
    if partitioned:
        app = DEFS + "partition with (" + ", ".join(f"sym of {s}" for s in sorted(used)) + ") begin " + \
            body + " end;"
    else:
        app = DEFS + body
    if playback:
        app = "@app:playback " + app
    syms = [f"K{i}" for i in range(rng.choice([1, 2, 4]))]
    t = 1000
    actions = []
    n_ev = rng.randint(30, 300)
    i = 0
    while i < n_ev:
        if playback and rng.random() < 0.08:
            t += rng.choice([10, 30, 80])
            actions.append(("advance", t))
            continue
        s = rng.choice(sorted(used))
        b = []
        for _ in range(rng.randint(1, 12)):
            t += rng.choice([0, 1, 1, 2, 5, 12])
            b.append((t, [rng.choice(syms), float(rng.randint(0, 40)) + rng.choice([0.0, 0.5, 0.25]),
                          rng.randint(0, 9), rng.randint(-3, 25)]))
            i += 1
        actions.append(("send", s, b))
    return app, actions


def run_case(factory, app, actions):
    """Returns [(query, ts, data)] of every output event, in callback order."""
    from siddhi_amd import SiddhiManager
    mgr = SiddhiManager(engine_factory=factory)
    rt = mgr.createSiddhiAppRuntime(app)
    got = []
    for name in ("query1", "query2", "query3"):
        try:
            rt.addCallback(name, (lambda nm: lambda ts, i, r: got.extend((nm, e.timestamp, e.data)
                                                                          for e in (i or [])))(name))
        except Exception:
            pass
    rt.start()
    hs = {}
    try:
        for a in actions:
            if a[0] == "send":
                h = hs.setdefault(a[1], rt.getInputHandler(a[1]))
                h.send_batch([t for t, _ in a[2]], [d for _, d in a[2]])
            else:
                rt.advance_time(a[1])
    finally:
        rt.shutdown()
    return got


def same_rows(got, ref):
    if len(got) != len(ref):
        return False
    for g, r in zip(got, ref):
        if g[0] != r[0] or g[1] != r[1] or len(g[2]) != len(r[2]):
            return False
        for a, b in zip(g[2], r[2]):
            if not ((a == b) or (a != a and b != b)):
                return False
    return True
