"""C4 (logical + absent, partitioned by user) drivers shared by the CPU and GPU
tests and bench.py: feed synth.c4_stream's send(Event[]) batches to any engine
of the start/send/advance_time/drain protocol."""
import numpy as np

from siddhi_amd import javastr, synth


def register_users(engine, blocks):
    """attr.toString() of every user id: synth.c4_user_strings (the scheduler's
    HashMap<String, ...> order depends on their String.hashCode)"""
    n = max((int(k.max()) + 1 for _, _, _, k in blocks if len(k)), default=0)
    if n and hasattr(engine, "set_partition_keys"):
        chars, offs = synth.c4_user_strings(n)
        engine.set_partition_keys(0, utf16=chars, offsets=offs)


def run_c4(engine, blocks, keep=None, progress=None):
    """Sends every block (optionally only the rows whose user is in `keep`, a
    bool mask over user ids), advances playback time past the last timer and
    drains. Returns the engine's drain dict."""
    import time
    register_users(engine, blocks)
    engine.start()
    seq = 0
    t_log = time.monotonic()
    for i, (st, ts, cols, keys) in enumerate(blocks):
        if progress is not None and time.monotonic() - t_log > 20:
            t_log = time.monotonic()
            progress(f"{i}/{len(blocks)} send calls")
        if keep is not None:
            m = keep[keys]
            if not m.any():
                continue
            ts, cols, keys = ts[m], [c[m] for c in cols], keys[m]
        engine.send(st, ts, cols, [None] * len(cols), keys, seq)
        seq += len(ts)
    engine.advance_time(synth.c4_end_time(blocks))
    return engine.drain()


def same_output(a, b):
    """same rows in the same order: trigger sequence, emitting query, output
    timestamp, raw values and null flags"""
    return (len(a["seq"]) == len(b["seq"]) and np.array_equal(a["seq"], b["seq"])
            and np.array_equal(a["query"], b["query"]) and np.array_equal(a["ts"], b["ts"])
            and np.array_equal(a["values"], b["values"]) and np.array_equal(a["nulls"], b["nulls"]))


def ties(blocks):
    """due milliseconds shared by more than one user (fired one per call)"""
    due = {}
    for st, ts, cols, keys in blocks:
        if st == 1:
            for t in np.unique(ts):
                due[int(t)] = due.get(int(t), 0) + int((ts == t).sum())
    return sum(1 for v in due.values() if v > 1)


class CollidingNames:
    """engine wrapper registering user names built from "Aa"/"BB" blocks, which
    all share one String.hashCode per length: bins overflow into trees"""

    def __init__(self, eng, n):
        self.eng = eng
        names = []
        for u in range(n):
            bits = format(u, "014b")
            names.append("".join("Aa" if b == "0" else "BB" for b in bits[-9:]) + str(u // 512))
        self.utf16, self.offs = javastr.pack_utf16(names)

    def set_partition_keys(self, first, strings=None, utf16=None, offsets=None):
        self.eng.set_partition_keys(0, utf16=self.utf16, offsets=self.offs)

    def __getattr__(self, name):
        return getattr(self.eng, name)


def c4_digest(out):
    """count and SHA-256 of a drained output's rows in order: per row the trigger
    sequence (int64), query (int32), output timestamp (int64), raw values (int64)
    and null flags (the fields same_output compares)"""
    import hashlib
    m = len(out["seq"])
    h = hashlib.sha256()
    h.update(np.ascontiguousarray(np.asarray(out["seq"], np.int64)).tobytes())
    h.update(np.ascontiguousarray(np.asarray(out["query"], np.int32)).tobytes())
    h.update(np.ascontiguousarray(np.asarray(out["ts"], np.int64)).tobytes())
    h.update(np.ascontiguousarray(np.asarray(out["values"], np.int64)).tobytes())
    h.update(np.ascontiguousarray(np.asarray(out["nulls"]).astype(np.uint8)).tobytes())
    return {"rows": int(m), "sha256": h.hexdigest()}
