/*
 * siddhi_shard.h — the key-sharded multi-GPU path of libsiddhi_hip.so.
 *
 * One process per GPU. Partitions never interact in the reference
 * (PartitionRuntimeImpl gives every partition key its own state,
 * core/partition/PartitionRuntimeImpl.java:346-364, PartitionStateHolder), so one
 * arrival-ordered stream is split by partition key across the ranks: rank r
 * owns the keys with mix32(key) % world == r. Every rank ingests an arrival-
 * contiguous slice of the stream; these entry points route the slice's events
 * to their owners (records exchanged with one RCCL all-to-all by the caller),
 * unpack them on the owner, and merge the owners' ordered match streams back
 * into one trigger-sequence order on the slice's rank.
 *
 * There is no reference interface for this: the reference runs one JVM
 * process per app. The matcher calls on each rank are the sh_* entry points of
 * siddhi_hip.h. All pointers named d_* are device pointers; `stream` is a
 * hipStream_t. Return: SH_OK or a negative SH_E_* status.
 */
#ifndef SIDDHI_SHARD_H
#define SIDDHI_SHARD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SHS_MAX_COLS 8
#define SHS_MAX_WORLD 256

/* owner rank of a partition key id (splitmix-style 32-bit finaliser) */
int32_t shs_owner(int32_t key, int32_t world);

/* scratch bytes shs_route needs for n events */
int64_t shs_route_scratch_bytes(int64_t n, int32_t world);

/* d_pos[i] = position of event i in the owner-major send buffer (stable:
   arrival order inside each owner's run); h_counts[r] = events for rank r */
int shs_route(const int32_t* d_keys, int64_t n, int32_t world, uint32_t* d_pos, void* d_scratch,
              int64_t* h_counts, void* stream);

/* words (4 bytes) per packed record: the columns (width 1 and 4 -> 1 word,
   8 -> 2) followed by the 8-byte global sequence number */
int32_t shs_record_words(int32_t n_cols, const int32_t* widths);

/* rec[d_pos[i]] = cols[0..n_cols)[i] ++ (seq0 + i) */
int shs_pack(const uint32_t* d_pos, int64_t n, int32_t n_cols, const void* const* d_cols, const int32_t* widths,
             uint64_t seq0, uint32_t* d_rec, void* stream);

/* the inverse on the owner: columns and global sequence numbers back out of
   n received records */
int shs_unpack(const uint32_t* d_rec, int64_t n, int32_t n_cols, void* const* d_cols, const int32_t* widths,
               uint64_t* d_seq, void* stream);

/* Compact records (C2: 24 bytes instead of 32): a column of width code
   SHS_W_OFF is an 8-byte column (timestamps) carried as a 32-bit offset from
   h_base[c] (the caller checks the slice's range fits), and the sequence number
   is carried as the 32-bit index into the source slice. */
#define SHS_W_OFF 5
int32_t shs_record_words_compact(int32_t n_cols, const int32_t* widths);
/* rec[d_pos[i]] = cols (SHS_W_OFF: v - h_base[c]) ++ (uint32)i */
int shs_pack_compact(const uint32_t* d_pos, int64_t n, int32_t n_cols, const void* const* d_cols,
                     const int32_t* widths, const int64_t* h_base, uint32_t* d_rec, void* stream);
/* the inverse over the records received from each source rank r (records
   [h_src_off[r], h_src_off[r+1])): SHS_W_OFF columns + h_src_base[r * n_cols + c],
   sequence numbers h_src_seq0[r] + index */
int shs_unpack_compact(const uint32_t* d_rec, int32_t n_cols, void* const* d_cols, const int32_t* widths,
                       const int64_t* h_src_off, int32_t world, const int64_t* h_src_base, const uint64_t* h_src_seq0,
                       uint64_t* d_seq, void* stream);

/* owner side of the return route: d_oseq (m matcher rows, values seq_base +
   local event index, ascending) -> global sequence numbers d_gseq[local]; and
   h_counts[r] = rows whose event came from rank r (received events are laid
   out by source rank: h_src_off[0..world] local offsets) */
int shs_rows_home(uint64_t* d_oseq, int64_t m, uint64_t seq_base, const uint64_t* d_gseq,
                  const int64_t* h_src_off, int32_t world, int64_t* h_counts, void* stream);

/* k-way merge by trigger sequence of n_runs ascending runs [h_off[r],
   h_off[r+1]) of (seq, n_out values): out position = own index in the run +
   rows of the other runs with a smaller sequence number. Sequence numbers of
   different runs are distinct (an event belongs to one key, so to one rank). */
int shs_merge(const uint64_t* d_seq, const int64_t* d_vals, int32_t n_out, const int64_t* h_off, int32_t n_runs,
              uint64_t* d_seq_out, int64_t* d_vals_out, void* stream);

#ifdef __cplusplus
}
#endif
#endif
