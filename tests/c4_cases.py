"""C4 (logical + absent, partitioned by user) drivers shared by the CPU and GPU
tests and bench.py: feed synth.c4_stream's send(Event[]) batches to any engine
of the start/send/advance_time/drain protocol."""
import numpy as np

from siddhi_amd import synth


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
