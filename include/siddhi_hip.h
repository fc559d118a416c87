/*
 * siddhi_hip.h — C-ABI of libsiddhi_hip.so, the MI355X (gfx950) batch NFA
 * matcher that replaces siddhi-core's pattern/sequence runtime
 * (io.siddhi.core.query.input.stream.state) behind the unchanged
 * SiddhiManager / SiddhiAppRuntime / InputHandler / StreamCallback API.
 *
 * Each entry point names the reference interface it replaces. The Java host
 * (JNI shim) or the Python mirror (siddhi_amd/) calls these;
 * no torch types cross this boundary.
 *
 * Threading: calls on one handle are serialised by the caller (the reference
 * serialises a query under patternSyncObject, MultiProcessStreamReceiver.java:158).
 * Independent handles may run concurrently, each on its own HIP stream.
 * Results come back through sh_drain; the library never calls back, except
 * through the coordinator a key-sharded handle is given (sh_set_coordinator).
 */
#ifndef SIDDHI_HIP_H
#define SIDDHI_HIP_H

#include <stddef.h>
#include <stdint.h>
#include "sh_query.h"

#ifdef __cplusplus
extern "C" {
#endif

/* status codes (the JNI shim maps them to SiddhiAppCreationException /
   SiddhiAppRuntimeException; SH_E_UNSUPPORTED at compile time means the host
   keeps the stock Java runtime for that app) */
#define SH_OK 0
#define SH_E_INVALID_ARG (-1)
#define SH_E_OOM (-2)
#define SH_E_HIP (-3)
#define SH_E_UNSUPPORTED (-4)
#define SH_E_STATE_OVERFLOW (-5)
#define SH_E_MORE (-6)
#define SH_E_NO_DEVICE (-7)

typedef struct sh_handle sh_handle;

/* One InputHandler.send(Event[]) call, packed as SoA (columns in the stream
   definition's attribute order, each in its natural width: INT/STRING-id ->
   int32, LONG -> int64, FLOAT -> float, DOUBLE -> double, BOOL -> uint8). */
typedef struct sh_batch {
    int32_t stream;              /* app stream index                                */
    int32_t on_device;           /* 1: every pointer below is a device (HBM) pointer */
    int64_t n;                   /* events in this send() call                      */
    const int64_t* ts;           /* event timestamps (ms)                           */
    const int32_t* keys;         /* partition key ids (attr.toString() dictionary), -1 = null key; NULL if unpartitioned */
    const void* const* cols;     /* n_attrs column pointers                         */
    const uint8_t* const* nulls; /* per column null mask (1 = null) or NULL          */
} sh_batch;

/* Match output: the ordered stream StreamCallback.receive(Event[]) would see.
   Caller-provided buffers with a capacity; SH_E_MORE if more remain. */
typedef struct sh_match_buf {
    int64_t capacity;            /* rows the buffers below can hold                 */
    int64_t count;               /* out: rows written                               */
    int32_t* query;              /* out: query index that emitted the row           */
    uint64_t* trigger_seq;       /* out: global input sequence number of the event being processed */
    int64_t* ts;                 /* out: output Event timestamp (StateEvent ts)      */
    int64_t* values;             /* out: count x n_out raw 8-byte values (row-major) */
    uint8_t* nulls;              /* out: count x n_out null flags                    */
    int32_t n_out;               /* columns per row = max outputs over the app's queries */
    int32_t pad;
} sh_match_buf;

/* Replaces SiddhiAppParser/QueryParser -> StateInputStreamParser.parseInputStream
   (core/util/parser/StateInputStreamParser.java:76-146): lowers every query's
   state-element tree to the device NFA table. */
int sh_compile(const sh_app_desc* app, sh_handle** out);

/* Replaces SiddhiAppRuntime.start -> StateStreamRuntime.initPartition for
   unpartitioned queries (core/query/input/stream/state/StateStreamRuntime.java:90-97,
   AbsentStreamPreStateProcessor.partitionCreated :303-314): arms start states and
   absent-state timers at the current clock. Call once, before the first batch. */
int sh_start(sh_handle* h);

/* Replaces InputHandler.send(Event[]) -> StreamJunction.sendEvent ->
   [PartitionStreamReceiver.receive] -> Pattern/Sequence*ProcessStreamReceiver.receive
   (core/stream/input/InputHandler.java:85-96, core/partition/PartitionStreamReceiver.java:176-216,
   core/query/input/MultiProcessStreamReceiver.java:155-183).
   Streaming handles (general engine) launch a push's device work and return
   before it completes: an error the device raises for that batch (state or replay
   capacity, a key id out of range) is returned by the NEXT call into the handle --
   sh_push_batch, sh_drain, sh_pending, sh_advance_time, sh_snapshot or
   sh_run_device -- and the handle keeps the state from before the failed batch. */
int sh_push_batch(sh_handle* h, const sh_batch* batch);

/* Registers attr.toString() of partition key ids [first_key, first_key + n) as
   UTF-16 (offsets[0..n] index into utf16): the ids the host put in sh_batch.keys
   (ValuePartitionExecutor.execute, core/partition/executor/ValuePartitionExecutor.java:34-40).
   Their String.hashCode / compareTo fix the iteration order of the playback
   scheduler's state map (PartitionStateHolder.states, a HashMap<String, ...>,
   util/snapshot/state/PartitionStateHolder.java:36), which decides the one
   state per due time Scheduler.onTimeChange fires (util/Scheduler.java:75-87).
   Call before the ids first appear in a batch; an unregistered id is taken to
   be its decimal digits. */
int sh_set_partition_keys(sh_handle* h, int32_t first_key, int32_t n, const uint16_t* utf16, const int64_t* offsets);

/* Replaces the playback clock advance TimestampGeneratorImpl.setCurrentTimestamp
   -> Scheduler.onTimeChange (core/util/timestamp/TimestampGeneratorImpl.java:105-121,
   core/util/Scheduler.java:74-99). */
int sh_advance_time(sh_handle* h, int64_t now_ms);

/* Replaces OutputRateLimiter.sendToCallBacks -> StreamCallback.receive
   (core/query/output/ratelimit/OutputRateLimiter.java:63-106): ordered matches. */
int sh_drain(sh_handle* h, sh_match_buf* out);

/* A List value -- the select of a count state's attribute without an index,
   MultiValueVariableFunctionExecutor (core/executor/MultiValueVariableFunctionExecutor.java:39-70):
   an SH_T_OBJECT output column holds a list handle. Copies up to cap elements
   (raw 8-byte values of the attribute's type, null flags) and returns the list's
   length (SH_E_INVALID_ARG: no such list). A row's handles stay valid until the
   next sh_drain call. */
int64_t sh_list_get(sh_handle* h, int64_t list, int64_t cap, int64_t* values, uint8_t* nulls);

/* Number of rows sh_drain would return right now (forces pending device work). */
int64_t sh_pending(sh_handle* h);

/* Replaces SiddhiAppRuntime.shutdown for the matcher's state. */
void sh_destroy(sh_handle* h);

const char* sh_last_error(sh_handle* h);

/* ---- device-resident bulk path (bench / throughput) ----------------------
   Matches on `n` events already resident in HBM for a single-stream app,
   starting from fresh per-key state, writing the ordered match stream to
   device buffers. Times only device work; the caller owns all buffers. */
typedef struct sh_device_run {
    int64_t n;                   /* events                                         */
    const int64_t* d_ts;
    const int32_t* d_keys;       /* partition key ids (dense 0..n_keys-1)           */
    int32_t n_keys;
    int32_t batch_events;        /* events per send(Event[]) call (0: one call)     */
    const void* const* d_cols;   /* device column pointers, stream attribute order  */
    int64_t out_capacity;        /* rows the output buffers hold                    */
    uint64_t* d_out_seq;         /* out: trigger_seq per match (ordered)            */
    int64_t* d_out_values;       /* out: out_capacity x n_out raw values            */
    int64_t out_count;           /* out: matches produced                           */
    void* stream;                /* hipStream_t to run on (NULL = default)          */
    int32_t* d_out_query;        /* out (optional): query index per match (ordered) */
    /* out (optional): the select values as typed columns, one device pointer per
       output attribute in its natural width (long/double 8 B, int/float/string id
       4 B, bool 1 B), ordered like d_out_seq. When set, d_out_values may be NULL
       and is not written; the row-major raw layout stays the default. */
    void* const* d_out_cols;
    /* ---- end of the V1 struct (96 bytes): sh_run_device reads only the fields
       above. The fields below are read by sh_run_device_v2 alone, which requires
       version == SH_DEVICE_RUN_V2. */
    int32_t version;
    /* SH_OUT_RAW (0): d_out_seq + d_out_values as above (or d_out_cols).
       SH_OUT_PACKED (1): d_out_values holds out_capacity packed rows instead, one
       per match: the trigger_seq (8 B), then each select value at its natural
       width (as d_out_cols; bool in a 4-byte slot) aligned to that width, the row
       padded to a multiple of 16 B -- sh_packed_row_layout gives the offsets.
       d_out_seq is not written; d_out_cols must be NULL. */
    int32_t out_layout;
    /* optional: the PartitionStreamReceiver run of every event (one run = the
       consecutive same-key events of one send() call,
       core/partition/PartitionStreamReceiver.java:176-216), as a non-decreasing
       id; equal ids that are adjacent here form one run. Lets a caller hand over
       a subsequence of a stream (one key shard) with the runs the whole stream
       had. NULL: runs follow from d_keys and batch_events. */
    const uint32_t* d_run;
} sh_device_run;
#define SH_DEVICE_RUN_V2 2
#define SH_DEVICE_RUN_V1_BYTES 96
#define SH_OUT_RAW 0
#define SH_OUT_PACKED 1

/* reads the V1 prefix of *run (SH_DEVICE_RUN_V1_BYTES) and writes out_count.
   Layout 2 (sh_version() "... layout 2"): the 0.1 header of round 3 had version /
   pad at offset 88 and d_out_cols at 96; a caller still built against it leaves a
   small integer in d_out_cols and gets SH_E_INVALID_ARG instead of a write
   through it -- rebuild the binding against this header. */
int sh_run_device(sh_handle* h, sh_device_run* run);
/* the whole struct; SH_E_INVALID_ARG unless run->version == SH_DEVICE_RUN_V2 */
int sh_run_device_v2(sh_handle* h, sh_device_run* run);

/* The SH_OUT_PACKED row of this app: byte offset of each select value
   (offsets[0 .. *n_out - 1]; cap entries at most) and the row size. The same
   Event the reference hands StreamCallback.receive (core/stream/output/
   StreamCallback.java:44-60: timestamp-ordered data[] of the select), as one
   fixed-size record. SH_E_UNSUPPORTED: queries select different types at one
   position. */
int sh_packed_row_layout(sh_handle* h, int32_t* offsets, int32_t cap, int32_t* n_out, int32_t* row_bytes);

/* kernel timing of the last sh_run_device call (HIP events on run->stream) */
typedef struct sh_kernel_times {
    float segment_ms;            /* radix segment by (key, seq)                    */
    float advance_ms;            /* per-key NFA state advance                       */
    float emit_ms;               /* match compaction / ordered placement            */
    float total_ms;
    int64_t advance_launches;
} sh_kernel_times;
int sh_last_kernel_times(sh_handle* h, sh_kernel_times* t);

/* Snapshot of the matcher state -- replaces the State.snapshot() maps of the
   pattern processors collected by SiddhiAppRuntime.snapshot() / persist()
   (core/util/snapshot/SnapshotService.java:90-187; state/StreamPreStateProcessor.java:
   450-469): every partial match with the events it holds, scheduler queues and
   their HashMap-order models, per-key aggregates, the playback clock, sequence
   counters and undelivered output, as one opaque versioned image. Pending send()s
   are processed first. buf == NULL or cap < size: *size is set and SH_E_MORE
   returned. */
int sh_snapshot(sh_handle* h, void* buf, int64_t cap, int64_t* size);
/* Restore an image into a handle compiled from the same app that has not
   processed events yet (SiddhiAppRuntime.restore(byte[]) / restoreLastRevision,
   SnapshotService.java:333-430). SH_E_INVALID_ARG: another app's image or a
   damaged one. */
int sh_restore(sh_handle* h, const void* buf, int64_t size);

/* ---- key-sharded streaming: apps with scheduler (absent) states on several GPUs
   One process per GPU, each with a handle compiled from the same app. Every rank
   sees every InputHandler.send(Event[]) call and pushes only the events of the
   partition keys it owns (PartitionStreamReceiver.receive routes per key,
   core/partition/PartitionStreamReceiver.java:176-272), keeping the call's
   playback clock step (InputHandler.java:85-96) and global sequence numbers.
   Keys couple only through Scheduler.onTimeChange (core/util/Scheduler.java:74-99):
   (1) one state per distinct due time fires -- the first in the scheduler's state
       map iteration order over ALL keys (TreeMultimap with a zero value comparator);
   (2) that order is PartitionStateHolder's HashMap<String, ...>
       (util/snapshot/state/PartitionStateHolder.java:36,131-162), shaped by every
       rank's getState / returnAllStates history.
   The handle reaches the other ranks through three callbacks, invoked at the same
   points of the call sequence on every rank (collectives; any transport). */
typedef struct sh_due_cand {
    int64_t t;                   /* head notify time (the TreeMultimap key)          */
    uint64_t order;              /* the key's position in the state map's iteration order */
    int32_t key;                 /* partition key id                                 */
    int32_t pad;
} sh_due_cand;
typedef struct sh_coordinator {
    void* user;
    /* one launch's scheduler-map history: this rank's records in (2 words each:
       processing stamp, key | scheduler << 32 | kind << 48), every rank's records
       of the launch out (*all stays valid until the next callback) */
    int (*history)(void* user, const uint64_t* local, int64_t n_local, const uint64_t** all, int64_t* n_all);
    /* the pick: this rank's due candidates in; out: pos[i] = position of candidate
       i in the firing order over all ranks (-1: not fired) and *n_fire = states
       fired over all ranks. Playback (wall == 0): the earliest `order` per distinct
       t, fired in t order; wall clock (wall == 1): every candidate, by (t, order). */
    int (*select)(void* user, int32_t wall, const sh_due_cand* local, int64_t n_local, int64_t* pos, int64_t* n_fire);
    /* the minimum over the ranks of a time (wall-clock stepping through notify times) */
    int (*min_time)(void* user, int64_t local, int64_t* global);
} sh_coordinator;
/* Turns the handle into one rank of a key-sharded group (before sh_start). */
int sh_set_coordinator(sh_handle* h, const sh_coordinator* c);
/* One send(Event[]) call of `call_n` events of which this rank owns `batch->n`
   (may be 0): index[i] is event i's position in the call (ascending), call_last_ts
   the call's last timestamp (the playback clock step). Trigger sequence numbers
   and processing order are the whole call's. */
int sh_push_batch_part(sh_handle* h, const sh_batch* batch, const uint32_t* index, int64_t call_n,
                       int64_t call_last_ts);
/* sh_drain plus, per row, its position in the global processing order
   (launch << 32 | position inside the launch): the ranks' drained rows merged by
   it (a stable sort) are the single-process output. */
int sh_drain_ordered(sh_handle* h, sh_match_buf* out, uint64_t* order);

/* library / device info */
const char* sh_version(void);
int sh_device_count(void);

#ifdef __cplusplus
}
#endif
#endif /* SIDDHI_HIP_H */
