"""C5-shaped rule sets (batch-compiled `every e1 -> e2 within` queries over one
stream) and an oracle driver; shared by the CPU checker test and the GPU parity
tests."""
import numpy as np

from oracle_engine import OracleEngine
from siddhi_amd import compiler, synth


def card_strings(n_cards):
    """Card dictionary ids 0..n-1 (the partition key ids of the same values)."""
    s = compiler.StringDict()
    for i in range(n_cards):
        s.id(f"C{i}")
    return s


def oracle_run(text, n_cards, ts, card, amount, merchant, batch, partitioned=True):
    """send(Event[]) calls of `batch` events; returns the oracle's drained rows."""
    eng = OracleEngine(compiler.compile_app(text, card_strings(n_cards)))
    eng.start()
    for b0 in range(0, len(ts), batch):
        b1 = min(len(ts), b0 + batch)
        cols = [card[b0:b1].copy(), amount[b0:b1].copy(), merchant[b0:b1].copy()]
        eng.send(0, ts[b0:b1].copy(), cols, [None] * 3, card[b0:b1].copy() if partitioned else None, b0)
    out = eng.drain()
    eng.close()
    return out


# (events, cards, rules, rate ev/ms, batch, merchants, partitioned, free rules, seed)
CASES = [
    (20000, 50, 40, 2, 4096, 10, True, (0, 5), 11),
    (15000, 3, 12, 5, 64, 6, True, (), 12),          # long same-card runs
    (20000, 500, 100, 1, 4096, 10, True, (1,), 13),
    (12000, 1, 8, 3, 100, 4, True, (), 14),          # one card: whole send() calls are runs
    (8000, 30, 20, 2, 4096, 8, False, (2,), 15),     # unpartitioned: each send() call is one run
    (30000, 2000, 300, 1, 4096, 40, True, (), 16),
    (20000, 200, 64, 4, 997, 12, True, (3, 7, 9), 17),
    (10000, 10, 2, 1, 4096, 5, True, (), 18),
    (10000, 1, 6, 2, 4096, 4, True, (), 19),         # one card, 4096-event runs (beyond the keys kernel's walk)
]


def case_data(case):
    n, cards, nr, rate, batch, merchants, partitioned, free, seed = case
    ts, card, amount, merchant = synth.txn_stream(n, cards, rate, n_merchants=merchants, seed=seed)
    rules = synth.c5_rules(nr, seed=seed, amount=(10.0, 150.0), merchants=merchants, factor=(0.6, 1.6),
                           within=(1, 40))
    text = synth.c5_query(rules, unit="milliseconds", partitioned=partitioned, free=free)
    return text, rules, (ts, card, amount, merchant)


def same(a, b):
    return np.array_equal(np.asarray(a), np.asarray(b))
