"""Key sharding across GPUs (one process per GPU).

Partitions never interact in the reference (per-key state, PartitionSyncStateHolder),
so a partitioned app shards by key with no data-path collective: rank =
mix32(key id) % world. Each rank runs its own matcher handle; the per-rank ordered
match streams are merged by trigger sequence number.
"""
import numpy as np


def mix32(x):
    """splitmix-style 32-bit finaliser (vectorised)."""
    x = np.asarray(x, dtype=np.uint64) & np.uint64(0xFFFFFFFF)
    x = (x ^ (x >> np.uint64(16))) * np.uint64(0x85EBCA6B) & np.uint64(0xFFFFFFFF)
    x = (x ^ (x >> np.uint64(13))) * np.uint64(0xC2B2AE35) & np.uint64(0xFFFFFFFF)
    return (x ^ (x >> np.uint64(16))).astype(np.uint32)


def shard_of(keys, world):
    return (mix32(keys) % np.uint32(world)).astype(np.int32)


def split(keys, world):
    """Index arrays (arrival order preserved) of the events each rank owns."""
    s = shard_of(keys, world)
    return [np.nonzero(s == r)[0] for r in range(world)]


def merge(parts):
    """k-way merge of per-rank ordered outputs: list of (seq, *columns) tuples of
    arrays, each ordered by seq. Rows sharing a seq come from one rank and keep
    their order (stable sort)."""
    seqs = np.concatenate([p[0] for p in parts])
    order = np.argsort(seqs, kind="stable")
    return tuple(np.concatenate([p[i] for p in parts])[order] for i in range(len(parts[0])))
