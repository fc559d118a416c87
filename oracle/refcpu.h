/*
 * refcpu.h — C API of the CPU ORACLE (test infrastructure, NOT the product).
 *
 * librefcpu.so is a line-by-line C++ restatement of siddhi-core's
 * pattern/sequence engine (io.siddhi.core.query.input.stream.state and the
 * receivers, partition routing, selector and state holders it runs under).
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load it — as the checker, never as the thing measured or shipped.
 *
 * Parity pinning: the restatement is pinned against the reference's own
 * known-answer tests, transcribed as fixtures under tests/golden/ (the
 * reference is Java and cannot run in this image: no JDK, no jars).
 */
#ifndef REFCPU_H
#define REFCPU_H

#include <stdint.h>
#include "../include/siddhi_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ref_app ref_app;

/* build the processor graph of every query (StateInputStreamParser.parse) */
ref_app* ref_create(const sh_app_desc* app, char* err, int errlen);
/* SiddhiAppRuntime.start(): init non-partitioned state runtimes */
void ref_start(ref_app* a);
/* one InputHandler.send(Event[]) call; events get sequence numbers first_seq.. */
int ref_send(ref_app* a, const sh_batch* b, uint64_t first_seq);
/* attr.toString() of partition key ids [first, first+n) as UTF-16 (n+1
   offsets into utf16): hashCode / compareTo of the keys fix the iteration
   order of the scheduler's HashMap (jhashmap.h) */
int ref_set_partition_keys(ref_app* a, int32_t first, int32_t n, const uint16_t* utf16, const int64_t* offsets);
/* playback clock / timer advance (Scheduler.onTimeChange) */
int ref_advance_time(ref_app* a, int64_t now);
/* emitted output rows so far (ordered as StreamCallback would see them) */
int64_t ref_out_count(ref_app* a);
int ref_out_read(ref_app* a, int64_t start, int64_t count, int32_t* query, uint64_t* seq,
                 int64_t* ts, int64_t* values, uint8_t* nulls, int32_t n_out, int32_t* cb_group);
void ref_out_clear(ref_app* a);
/* a List output value (SH_OP_MULTI_VAR): copies up to cap elements, returns the length (-1: no such list) */
int64_t ref_list_get(ref_app* a, int64_t list, int64_t cap, int64_t* values, uint8_t* nulls);
void ref_destroy(ref_app* a);
const char* ref_last_error(ref_app* a);

#ifdef __cplusplus
}
#endif
#endif
