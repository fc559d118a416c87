"""Host-side mirror of siddhi-core's public API for the pattern/sequence path.

Same names, argument meaning and error behaviour as
  core/SiddhiManager.java:93                       createSiddhiAppRuntime
  core/SiddhiAppRuntime.java:115-144               getInputHandler / addCallback / start / shutdown
  core/stream/input/InputHandler.java:65-96        send(Object[]) / send(long, Object[]) / send(Event[])
  core/stream/output/StreamCallback.java           receive(Event[])
  core/query/output/callback/QueryCallback.java    receive(timestamp, inEvents, removeEvents)
  core/event/Event.java                            Event(timestamp, data, isExpired)

The matcher itself runs behind the C-ABI (libsiddhi_hip.so) through an engine
object; the default engine is the HIP one (siddhi_amd._native.HipEngine), which
fails loudly when the extension is missing.

Time: `send(Object[])` stamps events with the runtime clock. Outside
@app:playback the reference uses System.currentTimeMillis(); this mirror keeps a
virtual clock advanced by `SiddhiAppRuntime.sleep(ms)` so that tests written with
Thread.sleep are deterministic ("time").
"""
from __future__ import annotations

import json
import struct
from typing import Callable, Dict, List, Optional

import numpy as np

from . import compiler as cp
from . import javastr
from .hostexpr import RangeEvaluator
from .compiler import (BOOL, DOUBLE, FLOAT, INT, LONG, OBJECT, STRING, CompiledApp,
                       SiddhiAppValidationException, SiddhiParserException, UnsupportedQuery)

__all__ = ["SiddhiManager", "SiddhiAppRuntime", "InputHandler", "StreamCallback", "QueryCallback",
           "Event", "SiddhiAppCreationException", "SiddhiAppRuntimeException", "InMemoryPersistenceStore",
           "NoPersistenceStoreException"]


class SiddhiAppCreationException(Exception):
    pass


class SiddhiAppRuntimeException(Exception):
    pass


class Event:
    """core/event/Event.java"""

    __slots__ = ("timestamp", "data", "is_expired")

    def __init__(self, timestamp: int = -1, data=None, is_expired: bool = False):
        self.timestamp = timestamp
        self.data = list(data) if data is not None else []
        self.is_expired = is_expired

    def getTimestamp(self):
        return self.timestamp

    def getData(self, i=None):
        return self.data if i is None else self.data[i]

    def isExpired(self):
        return self.is_expired

    def __repr__(self):
        return f"Event{{timestamp={self.timestamp}, data={self.data}, isExpired={self.is_expired}}}"


class StreamCallback:
    """core/stream/output/StreamCallback.java — override receive(events)."""

    def receive(self, events: List[Event]):  # pragma: no cover - user hook
        raise NotImplementedError


class QueryCallback:
    """core/query/output/callback/QueryCallback.java — override receive(ts, in, remove)."""

    def receive(self, timestamp: int, in_events: Optional[List[Event]],
                remove_events: Optional[List[Event]]):  # pragma: no cover - user hook
        raise NotImplementedError


class _FnStreamCallback(StreamCallback):
    def __init__(self, fn):
        self.fn = fn

    def receive(self, events):
        self.fn(events)


class _FnQueryCallback(QueryCallback):
    def __init__(self, fn):
        self.fn = fn

    def receive(self, timestamp, in_events, remove_events):
        self.fn(timestamp, in_events, remove_events)


# ---------------------------------------------------------------- value packing
_NP = {STRING: np.int32, INT: np.int32, LONG: np.int64, FLOAT: np.float32,
       DOUBLE: np.float64, BOOL: np.uint8, OBJECT: np.int64}


def _to_float32(x) -> float:
    return struct.unpack("<f", struct.pack("<f", float(x)))[0]


def decode_value(bits: int, typ: int, strings: cp.StringDict):
    """raw 8-byte value -> Python value (Java boxing of the output attribute)."""
    if typ == STRING:
        return strings.str(int(np.int32(np.int64(bits))))
    if typ == INT:
        return int(np.int32(np.int64(bits)))
    if typ == LONG:
        return int(bits)
    if typ == FLOAT:
        return struct.unpack("<f", struct.pack("<I", int(bits) & 0xFFFFFFFF))[0]
    if typ == DOUBLE:
        return struct.unpack("<d", struct.pack("<q", int(bits)))[0]
    if typ == BOOL:
        return bool(bits)
    return int(bits)


class KeyDict:
    """Partition keys: ValuePartitionExecutor.execute = attr.toString()
    (core/partition/executor/ValuePartitionExecutor.java:34-40). Two values share a
    partition iff their Java toString() is equal; ids are dense in first-seen order
    and `text[id]` is that toString() (handed to the library: the scheduler's
    HashMap<String, ...> order depends on it)."""

    def __init__(self):
        self.ids: Dict[str, int] = {}
        self.text: List[str] = []
        self.registered = 0  # ids [0, registered) already handed to the engine

    @staticmethod
    def java_text(value, typ) -> str:
        if typ == FLOAT:
            return javastr.java_float_to_string(value)
        if typ == DOUBLE:
            return javastr.java_double_to_string(value)
        if typ == BOOL:
            return "true" if value else "false"
        if typ in (INT, LONG):
            return str(int(value))
        return str(value)

    def key(self, value, typ) -> int:
        if value is None:
            return -1
        t = self.java_text(value, typ)
        i = self.ids.get(t)
        if i is None:
            i = len(self.text)
            self.ids[t] = i
            self.text.append(t)
        return i

    def flush_new(self, engine):
        """register ids added since the last call with the engine"""
        if self.registered < len(self.text) and hasattr(engine, "set_partition_keys"):
            engine.set_partition_keys(self.registered, self.text[self.registered:])
        self.registered = len(self.text)


# ---------------------------------------------------------------- runtime
class InputHandler:
    """core/stream/input/InputHandler.java"""

    def __init__(self, rt: "SiddhiAppRuntime", stream: str):
        self.rt = rt
        self.stream = stream
        self.stream_id = rt._stream_index[stream]

    def getStreamId(self):
        return self.stream

    def send(self, *args):
        """send(Object[] data) | send(long timestamp, Object[] data) | send(Event) | send(Event[])"""
        if len(args) == 2:
            ts, data = args
            self.rt._send(self.stream_id, [int(ts)], [list(data)])
            return
        (x,) = args
        if isinstance(x, Event):
            self.rt._send(self.stream_id, [x.timestamp], [x.data])
        elif isinstance(x, (list, tuple)) and x and isinstance(x[0], Event):
            self.rt._send(self.stream_id, [e.timestamp for e in x], [e.data for e in x])
        else:
            self.rt._send(self.stream_id, [None], [list(x)])

    def send_batch(self, timestamps, rows):
        """One send(Event[]) call from parallel lists of timestamps and data rows."""
        self.rt._send(self.stream_id, list(timestamps), [list(r) for r in rows])


class SiddhiAppRuntime:
    """core/SiddhiAppRuntime.java (pattern/sequence apps)."""

    def __init__(self, compiled: CompiledApp, engine_factory: Callable):
        self.compiled = compiled
        self.app = compiled.app
        self.strings = compiled.strings
        self.keys = KeyDict()
        self._stream_index = {n: i for i, n in enumerate(self.app.stream_order)}
        self._stream_cbs: Dict[str, List[StreamCallback]] = {}
        self._query_cbs: Dict[int, List[QueryCallback]] = {}
        self._query_by_name = {q.query.name: i for i, q in enumerate(compiled.queries)
                               if q.query.name}
        self._engine = engine_factory(compiled)
        self._manager_store = None  # () -> the SiddhiManager's PersistenceStore
        self._revision = 0
        self._started = False
        self._seq = 0
        self._range_ev: Dict[str, RangeEvaluator] = {}
        self._labels = None
        self.clock = 0 if self.app.playback else 1_000_000_000_000
        self.name = self.app.name

    # -- API
    def getName(self):
        return self.name

    def getInputHandler(self, stream: str) -> InputHandler:
        if stream not in self._stream_index:
            raise SiddhiAppRuntimeException(f"stream {stream} is not defined")
        return InputHandler(self, stream)

    def addCallback(self, name: str, cb):
        if name in self._query_by_name:
            if callable(cb) and not isinstance(cb, QueryCallback):
                cb = _FnQueryCallback(cb)
            self._query_cbs.setdefault(self._query_by_name[name], []).append(cb)
            return
        if callable(cb) and not isinstance(cb, StreamCallback):
            cb = _FnStreamCallback(cb)
        self._stream_cbs.setdefault(name, []).append(cb)

    def start(self):
        if not self._started:
            if not self.app.playback:
                # wall-clock apps: the scheduler's "now" at start (partitionCreated)
                self._engine.advance_time(self.clock)
            self._engine.start()
            self._started = True

    def shutdown(self):
        if self._engine is not None:
            self._engine.close()
            self._engine = None

    # -- persistence (core/SiddhiAppRuntimeImpl.java snapshot / restore / persist /
    # restoreLastRevision; core/util/snapshot/SnapshotService.java)
    _SNAP_MAGIC = b"SHAP1\0"

    def snapshot(self) -> bytes:
        """byte[] snapshot(): the matcher image (sh_snapshot) plus the host state the
        device ids refer to (string and partition-key dictionaries, clock, sequence)."""
        if self._engine is None or not hasattr(self._engine, "snapshot"):
            raise SiddhiAppRuntimeException("snapshot: the engine keeps no restorable state")
        image = self._engine.snapshot()
        host = json.dumps({"strings": list(self.strings._strs), "keys": list(self.keys.text),
                           "clock": int(self.clock), "seq": int(self._seq)}).encode()
        return self._SNAP_MAGIC + struct.pack("<Q", len(host)) + host + image

    def restore(self, snapshot: bytes):
        """restore(byte[]): into a started runtime of the same app that has not
        received events (the reference restores into a fresh runtime after start)"""
        m = self._SNAP_MAGIC
        if not snapshot.startswith(m):
            raise SiddhiAppRuntimeException("restore: not a snapshot of this engine")
        (n,) = struct.unpack_from("<Q", snapshot, len(m))
        host = json.loads(snapshot[len(m) + 8: len(m) + 8 + n].decode())
        image = snapshot[len(m) + 8 + n:]
        strs = host["strings"]
        if strs[: len(self.strings)] != self.strings._strs:
            raise SiddhiAppRuntimeException("restore: the snapshot was taken from another app")
        for v in strs[len(self.strings):]:
            self.strings.id(v)
        if self.keys.text and self.keys.text != host["keys"][: len(self.keys.text)]:
            raise SiddhiAppRuntimeException("restore: the runtime has seen other partition keys")
        for t in host["keys"][len(self.keys.text):]:
            self.keys.ids[t] = len(self.keys.text)
            self.keys.text.append(t)
        self.keys.registered = len(self.keys.text)  # the image carries the engine's key strings
        self._engine.restore(image)
        self.clock = max(self.clock, host["clock"])
        self._seq = max(self._seq, host["seq"])
        self._deliver()

    def persist(self):
        """persist(): snapshot into the manager's persistence store; returns the revision"""
        store = self._manager_store() if self._manager_store else None
        if store is None:
            raise NoPersistenceStoreException("no persistence store assigned")
        self._revision += 1
        rev = f"{self._revision}_{self.name or 'SiddhiApp'}"
        store.save(self.name or "SiddhiApp", rev, self.snapshot())
        return rev

    def restoreRevision(self, revision: str):
        store = self._manager_store() if self._manager_store else None
        if store is None:
            raise NoPersistenceStoreException("no persistence store assigned")
        data = store.load(self.name or "SiddhiApp", revision)
        if data is None:
            raise SiddhiAppRuntimeException(f"no revision {revision}")
        self.restore(data)

    def restoreLastRevision(self):
        store = self._manager_store() if self._manager_store else None
        if store is None:
            raise NoPersistenceStoreException("no persistence store assigned")
        rev = store.getLastRevision(self.name or "SiddhiApp")
        if rev is not None:
            self.restoreRevision(rev)
        return rev

    def sleep(self, ms: int):
        """Thread.sleep stand-in: advances the virtual clock (and fires due timers)."""
        self.clock += int(ms)
        if not self.app.playback and self._engine is not None:
            self._engine.advance_time(self.clock)
            self._deliver()

    def advance_time(self, now: int):
        self.clock = max(self.clock, int(now))
        self._engine.advance_time(self.clock)
        self._deliver()

    # -- internals
    def _pack(self, stream_id: int, ts: List[Optional[int]], rows: List[list]):
        sd = self.app.streams[self.app.stream_order[stream_id]]
        n = len(rows)
        tsa = np.empty(n, dtype=np.int64)
        for i, t in enumerate(ts):
            tsa[i] = self.clock if t is None else t
        cols, nulls = [], []
        for ai, (aname, typ) in enumerate(sd.attrs):
            col = np.zeros(n, dtype=_NP[typ])
            nm = None
            for i, r in enumerate(rows):
                v = r[ai] if ai < len(r) else None
                if v is None:
                    if nm is None:
                        nm = np.zeros(n, dtype=np.uint8)
                    nm[i] = 1
                    continue
                if typ == STRING:
                    col[i] = self.strings.id(v)
                elif typ == BOOL:
                    col[i] = 1 if v else 0
                else:
                    col[i] = v
            cols.append(col)
            nulls.append(nm)
        keys = None
        for p, spec in enumerate(self.app.partitions):
            sname = self.app.stream_order[stream_id]
            if sname in spec and isinstance(spec[sname], cp.RangeSpec):
                # the range labels are the partition keys (RangePartitionExecutor.execute)
                keys = np.array([self.keys.key(lb, STRING) for lb in self._labels], dtype=np.int32)
            elif sname in spec:
                ai = sd.index(spec[sname])
                typ = sd.attrs[ai][1]
                keys = np.array([self.keys.key(r[ai], typ) for r in rows], dtype=np.int32)
        return tsa, cols, nulls, keys

    def _range_expand(self, stream_id: int, ts, rows):
        """Range partitions (PartitionStreamReceiver.receive, core/partition/
        PartitionStreamReceiver.java:176-272): every range executor is evaluated per
        event in declaration order and the event goes to the partition of each range
        whose condition holds (none: dropped); consecutive same-key events form one
        chunk. Returns the expanded (ts, rows, labels)."""
        sname = self.app.stream_order[stream_id]
        for spec in self.app.partitions:
            rs = spec.get(sname)
            if isinstance(rs, cp.RangeSpec):
                ev = self._range_ev.get(sname)
                if ev is None:
                    ev = self._range_ev[sname] = RangeEvaluator(self.app.streams[sname], sname)
                ots, orows, labels = [], [], []
                for t, r in zip(ts, rows):
                    for cond, label in rs.ranges:
                        if ev.cond(cond, r):
                            ots.append(t)
                            orows.append(r)
                            labels.append(label)
                return ots, orows, labels
        return ts, rows, None

    def _send(self, stream_id: int, ts, rows):
        if not self._started:
            raise SiddhiAppRuntimeException("SiddhiAppRuntime not started")
        last_in = None
        if rows and self.app.playback:
            last_in = self.clock if ts[-1] is None else int(ts[-1])
        ts, rows, labels = self._range_expand(stream_id, ts, rows)
        self._labels = labels
        if last_in is not None and labels is not None:
            # InputHandler.send moves the playback clock to the batch's last event
            # before any partition routing (InputHandler.java:85-96), even when no
            # range keeps that event: one time change to it here; the engine's own
            # advance to an earlier kept timestamp then notifies nobody
            # (TimestampGeneratorImpl.setCurrentTimestamp: only ts >= current)
            kept = None if not rows else (self.clock if ts[-1] is None else int(ts[-1]))
            if (kept is None or kept < last_in) and last_in >= self.clock:
                self.advance_time(last_in)
        if not rows:
            return
        tsa, cols, nulls, keys = self._pack(stream_id, ts, rows)
        self.keys.flush_new(self._engine)
        if self.app.playback:
            self.clock = max(self.clock, int(tsa[-1]))
        first = self._seq
        self._seq += len(rows)
        self._engine.send(stream_id, tsa, cols, nulls, keys, first)
        self._deliver()

    def _deliver(self):
        res = self._engine.drain()
        if res is None or len(res["query"]) == 0:
            return
        qs, tss, vals, nls, groups = res["query"], res["ts"], res["values"], res["nulls"], res["group"]
        # group consecutive rows by callback chunk (sendToCallBacks call)
        i = 0
        n = len(qs)
        while i < n:
            j = i + 1
            while j < n and groups[j] == groups[i] and qs[j] == qs[i]:
                j += 1
            q = int(qs[i])
            cq = self.compiled.queries[q]
            evs = []
            lists = res.get("lists") or {}
            for k in range(i, j):
                data = []
                for c in range(len(cq.out_types)):
                    if nls[k, c]:
                        data.append(None)
                    elif cq.out_types[c] == OBJECT and (k, c) in lists:
                        # a List (MultiValueVariableFunctionExecutor) of the element type
                        lv, ln = lists[(k, c)]
                        et = cq.out_elem_types[c]
                        data.append([None if ln[x] else decode_value(int(lv[x]), et, self.strings)
                                     for x in range(len(lv))])
                    else:
                        data.append(decode_value(int(vals[k, c]), cq.out_types[c], self.strings))
                evs.append(Event(int(tss[k]), data))
            for cb in self._query_cbs.get(q, []):
                cb.receive(evs[-1].timestamp, evs, None)
            for cb in self._stream_cbs.get(cq.query.output, []):
                cb.receive(evs)
            i = j


class NoPersistenceStoreException(Exception):
    pass


class InMemoryPersistenceStore:
    """core/util/persistence/InMemoryPersistenceStore.java: revisions per app, in order"""

    def __init__(self):
        self._revs: Dict[str, List[tuple]] = {}

    def save(self, app: str, revision: str, snapshot: bytes):
        self._revs.setdefault(app, []).append((revision, bytes(snapshot)))

    def load(self, app: str, revision: str):
        for r, b in self._revs.get(app, []):
            if r == revision:
                return b
        return None

    def getLastRevision(self, app: str):
        revs = self._revs.get(app)
        return revs[-1][0] if revs else None

    def clearAllRevisions(self, app: str):
        self._revs.pop(app, None)


class SiddhiManager:
    """core/SiddhiManager.java"""

    def __init__(self, engine_factory: Optional[Callable] = None):
        if engine_factory is None:
            from ._native import HipEngine  # raises ImportError when the extension is absent
            engine_factory = HipEngine
        self._engine_factory = engine_factory
        self._runtimes = []
        self._store = None

    def setPersistenceStore(self, store):
        self._store = store

    def createSiddhiAppRuntime(self, app: str) -> SiddhiAppRuntime:
        try:
            compiled = cp.compile_app(app)
        except (SiddhiParserException, SiddhiAppValidationException, UnsupportedQuery) as e:
            raise SiddhiAppCreationException(str(e)) from e
        rt = SiddhiAppRuntime(compiled, self._engine_factory)
        rt._manager_store = lambda: self._store
        self._runtimes.append(rt)
        return rt

    def shutdown(self):
        for rt in self._runtimes:
            rt.shutdown()
        self._runtimes = []
