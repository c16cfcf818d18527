/*
 * cask_scan.h — C ABI of the MI355X-native Cask log-record scan (libcask_scan.so).
 *
 * Drop-in boundary for the replay/compaction hot path of andresilva/cask v0.7.1. The reference
 * is a Rust crate whose `log`/`data` modules are private (src/lib.rs:46,49), so it has no FFI of
 * its own; the seams these entry points replace are cited per function. A Rust binding
 * (`extern "C"` block + safe wrapper) is shown in INTEGRATION.md.
 *
 * Conventions: plain pointers and sizes only; the caller owns every buffer it passes in; the
 * library never frees caller memory. Return 0 (CASK_OK) on success, a negative cask_status on
 * failure. No C++ exception crosses this boundary.
 */
#ifndef CASK_SCAN_H
#define CASK_SCAN_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CASK_SCAN_ABI_VERSION 1

/* Status codes. The first five map onto the reference's Error enum (src/errors.rs:12-25). */
typedef enum cask_status {
  CASK_OK = 0,
  CASK_E_CHECKSUM = -1,        /* Error::InvalidChecksum { expected, found } (errors.rs:22) */
  CASK_E_EOF = -2,             /* Error::Io(UnexpectedEof) from read_exact (data.rs:163,172,181) */
  CASK_E_IO = -3,              /* Error::Io(other) (errors.rs:14) */
  CASK_E_INVALID_PATH = -4,    /* Error::InvalidPath (errors.rs:24; log.rs:46-56) */
  CASK_E_INVALID_FILE_ID = -5, /* Error::InvalidFileId (errors.rs:16; log.rs:200-202) */
  CASK_E_INVALID_ARG = -10,    /* bad argument to this ABI */
  CASK_E_DEVICE = -11,         /* HIP runtime / device failure */
  CASK_E_CAPACITY = -12,       /* caller's row buffer too small; needed count is reported */
  CASK_E_NOMEM = -13,
  CASK_E_LOCKED = -14          /* cask.lock held by another process (log.rs:58-59) */
} cask_status;

/* Per-row status (what Entries::next yields for the record at `pos`, log.rs:403-429). */
enum { CASK_ROW_OK = 0, CASK_ROW_CHECKSUM = 1, CASK_ROW_EOF = 2 };

/* Record format constants (data.rs:11-14). */
#define CASK_ENTRY_STATIC_SIZE 18u
#define CASK_ENTRY_TOMBSTONE 0xFFFFFFFFu

/* ------------------------------------------------------------------------------------------ */
/* Device scan context                                                                         */
/* ------------------------------------------------------------------------------------------ */
typedef struct cask_ctx cask_ctx;

/* One context per GPU: owns a HIP stream, chunk scratch and pinned staging. Contexts are
 * independent and may be used from different threads; one context is not re-entrant. */
cask_ctx* cask_ctx_create(int device, int* status);
void cask_ctx_destroy(cask_ctx* ctx);
/* Use a caller stream (hipStream_t passed as void*) instead of the context's own; NULL resets.
 * The context's own stream is non-blocking: it does not wait for work queued on other streams,
 * so device inputs still being produced elsewhere must be complete (or produced on the stream
 * set here) before a call reads them. (A walk-mode scan also runs one kernel on a second stream
 * the context owns, ordered after the work queued on this stream and joined back into it before
 * the call returns: work queued on this stream afterwards sees the call complete.) */
int cask_ctx_set_stream(cask_ctx* ctx, void* hip_stream);
void* cask_ctx_stream(cask_ctx* ctx);
/* Make the context's stream wait, on the device and without blocking the host, for the work queued
 * so far on another stream (hipStream_t as void*; NULL = the null stream) — how a caller hands over
 * inputs another library is still producing. */
int cask_ctx_wait_stream(cask_ctx* ctx, void* hip_stream);
int cask_ctx_device(const cask_ctx* ctx);
/* Device scratch the context holds now, in bytes (its buffers only grow; cask_ctx_destroy frees
 * them): chunk table, slot rows, call blocks, repair state, host-scan staging. */
uint64_t cask_ctx_scratch_bytes(const cask_ctx* ctx);

/* Human-readable cause of the last CASK_E_DEVICE returned on this context ("" if none). */
const char* cask_ctx_last_error(const cask_ctx* ctx);
/* Chunk size in bytes used by the scan kernels (the unit of speculation and staging). */
uint32_t cask_scan_chunk_bytes(void);

/* A data file to scan: `{:010}.cask.data` contents (log.rs:473-476), no header/footer. */
#define CASK_VIEW_DEVICE 1u /* data points to device memory (else host memory) */
typedef struct cask_file_view {
  uint32_t file_id;
  uint32_t flags;
  const uint8_t* data;
  uint64_t len;
} cask_file_view;

/* Rows in (file, pos) order, struct-of-arrays. One row per record the reference iterator
 * yields: Ok records, InvalidChecksum records (iteration continues past them, log.rs:467-471)
 * and at most one trailing UnexpectedEof record per file (iteration ends there).
 * The key of row i lives at data[pos[i] + 18 .. + ksz[i]] of its file (not copied). */
typedef struct cask_rows {
  uint64_t capacity; /* in: slots in every array */
  uint64_t count;    /* out: rows produced (also set on CASK_E_CAPACITY = rows needed) */
  uint64_t* pos;     /* entry_pos (log.rs:413) */
  uint64_t* seq;     /* Entry.sequence (data.rs:167) */
  uint32_t* vsz;     /* raw value_size field; 0xFFFFFFFF = tombstone (data.rs:169,174) */
  uint16_t* ksz;     /* key_size (data.rs:168) */
  uint8_t* status;   /* CASK_ROW_* */
} cask_rows;

/* First failing record in (call file order, pos) order — what Cask::open's `?` returns
 * (cask.rs:360,365). kind = 0 when every record verified. */
typedef struct cask_scan_error {
  int32_t kind;      /* 0, CASK_ROW_CHECKSUM or CASK_ROW_EOF */
  uint32_t file_id;
  uint64_t pos;
  uint32_t expected; /* stored checksum (InvalidChecksum.expected) */
  uint32_t found;    /* computed XXH32 (InvalidChecksum.found) */
  uint64_t row;      /* index of that row in the output */
} cask_scan_error;

/* Upper bound on rows for a set of files (every record is >= 18 bytes). */
uint64_t cask_rows_bound(const cask_file_view* files, uint32_t nfiles);

/* Device-resident scan: replaces `Log::entries`/`Entries::next` + `Entry::from_read`
 * (log.rs:108-119, 403-429; data.rs:161-206) and the per-record work of
 * `Log::recreate_hints`/`RecreateHints::next` (log.rs:137-148, 454-465) for many files at once.
 * files[i].data must be device pointers (CASK_VIEW_DEVICE); rows arrays must be device memory.
 * file_row_offset (host, nfiles+1 entries, may be NULL) receives each file's first row index.
 * Returns CASK_OK even when records fail verification: those are reported per row and in
 * *err (first failure). Synchronous: returns after the results are complete. */
int cask_scan_device(cask_ctx* ctx, const cask_file_view* files, uint32_t nfiles,
                     cask_rows* rows, uint64_t* file_row_offset, cask_scan_error* err);

/* Same, for host-resident files and host row arrays: stages H2D, scans, copies rows D2H. */
int cask_scan_host(cask_ctx* ctx, const cask_file_view* files, uint32_t nfiles,
                   cask_rows* rows, uint64_t* file_row_offset, cask_scan_error* err);

/* Timing of the last cask_scan_* call on the context's stream (HIP events, milliseconds):
 * [0] whole device pipeline, [1] chunk-scan kernel, [2] long-record + summary kernels,
 * [3] validation kernels, [4] repair (0 when speculation held), [5] compaction. */
int cask_last_timings(const cask_ctx* ctx, float* ms6);
/* The same six, then, in walk mode, [6] the run searches (k_walk_search) and [7] the header chase
 * (k_walk_chase); [1] is then the hashing kernel alone (cask_last_walk() == 1), or the hashing
 * kernel and k_scan_chunks together when one call ran both modes (cask_last_walk() == 2). */
int cask_last_timings8(const cask_ctx* ctx, float* ms8);
/* Counters of the last call: [0] chunks, [1] long records, [2] chunks from each file's first
 * invalid one on (0: speculation held), [3] local exact re-scans, [4] 1 if the serial boundary
 * walk ran. */
int cask_last_counters(const cask_ctx* ctx, uint64_t* c5);
/* 1 if the last cask_scan_device / cask_scan_host call took the two-kernel dense path (k_scan_chunks
 * + k_finish: every speculated chunk start held), 0 if it went through the repair path. */
int cask_last_dense(const cask_ctx* ctx);
/* The last call's scan mode: 1 walk mode (record headers chased from HBM, every record hashed from
 * HBM: picked where the records sampled at 8 points of each file average >= 1 KiB), 0 chunk mode
 * (k_scan_chunks), 2 both in one call (each run of chunks in the mode of its file region). */
int cask_last_walk(const cask_ctx* ctx);
/* The last call's k_scan_chunks geometry: 0 for the wide 4,080-B halo, 3 for the short 1,008-B halo
 * (picked when the sampled chunk-mode records are short), -1 when only the walk mode ran. */
int cask_last_geometry(const cask_ctx* ctx);

/* ------------------------------------------------------------------------------------------ */
/* Batched record encoder (Entry::write_bytes, data.rs:90-121) — the bulk write path and the   */
/* synthetic workload generator. Record r is written at out[off[r]]:                            */
/*   [xxh32 | seq[r] | ksz[r] | vsz_raw[r] | key | value], key/value bytes generated from        */
/*   key_id[r] and (value_seed, r) by the generator documented in DESIGN.md §Synthetic data.    */
/* All arrays are device memory.                                                               */
/* ------------------------------------------------------------------------------------------ */
int cask_encode_synthetic_device(cask_ctx* ctx, uint64_t nrec, const uint64_t* off,
                                 const uint64_t* seq, const uint16_t* ksz,
                                 const uint32_t* vsz_raw, const uint64_t* key_id,
                                 uint64_t value_seed, uint8_t* out);

/* Encode caller-supplied keys/values (device memory): key r = keys[key_off[r] .. +ksz[r]],
 * value r = vals[val_off[r] .. +vsz] (ignored for tombstones). */
int cask_encode_device(cask_ctx* ctx, uint64_t nrec, const uint64_t* off, const uint64_t* seq,
                       const uint16_t* ksz, const uint32_t* vsz_raw, const uint8_t* keys,
                       const uint64_t* key_off, const uint8_t* vals, const uint64_t* val_off,
                       uint8_t* out);

/* Bulk load through one LogWriter that is then dropped (LogWriter::write rollover, log.rs:282-306;
 * EntryWriter / HintWriter, log.rs:317-395): entries r = 0..n-1 in write order (host memory; key r =
 * keys[key_off[r] .. +ksz[r]], value r = vals[val_off[r] .. +vsz_raw[r]], vsz_raw = CASK_ENTRY_TOMBSTONE
 * for a deletion) are encoded and checksummed on `device` (Entry::write_bytes, data.rs:90-121) and
 * written to data files first_file_id, first_file_id + 1, ... in `dir`, each with its hint file
 * (hints + XXH32 trailer) when write_hints. Replaces the per-entry Log::append_entry /
 * LogWriter::write loop (log.rs:168-183, 282-306) for a batch. Returns the number of files
 * written (their ids in file_ids[0..min(count, cap))) or a negative status. */
int64_t cask_log_write(const char* dir, uint32_t first_file_id, uint64_t max_file_size, int write_hints, int device,
                       uint64_t n, const uint64_t* seq, const uint16_t* ksz, const uint32_t* vsz_raw,
                       const uint8_t* keys, const uint64_t* key_off, const uint8_t* vals, const uint64_t* val_off,
                       uint32_t* file_ids, uint64_t cap);

/* Log::read_entry + Entry::from_read at caller positions (log.rs:150-166, data.rs:161-206), on the
 * device — what compaction does for each live record (cask.rs:505-508), without re-scanning whole
 * files. Record r is read at byte pos[r] of source src[r] (srcs[src[r]]: device pointer to src_len
 * bytes). Host arrays out: len[r] = 18 + ksz + vsz_eff (0 when the record runs past its source:
 * UnexpectedEof), status[r] (CASK_ROW_*), expected[r] (stored checksum), found[r] (computed XXH32). */
int cask_read_entries_device(cask_ctx* ctx, const uint8_t* const* srcs, const uint64_t* src_len, uint32_t nsrc,
                             const uint32_t* src, const uint64_t* pos, uint64_t n, uint64_t* len, uint8_t* status,
                             uint32_t* expected, uint32_t* found);

/* XXH32 seed 0 on the host (util.rs:37-41) — convenience for bindings. */
uint32_t cask_xxh32(const uint8_t* data, uint64_t len);

/* ------------------------------------------------------------------------------------------ */
/* Engine: the Cask::open replay (cask.rs:335-382) with the device scan underneath.            */
/* ------------------------------------------------------------------------------------------ */
typedef struct cask_db cask_db;

/* CaskOptions (cask.rs:194-237); only the fields the replay/compaction path reads. */
typedef struct cask_options {
  int32_t create;               /* default 1 (cask.rs:223) */
  int32_t write_hints;          /* recreate missing/corrupt hint files (log.rs:137-148); 1 */
  uint64_t max_file_size;       /* default 2 GiB (cask.rs:225) */
  int32_t device;               /* GPU ordinal for the scan */
  int32_t reserved;
} cask_options;

void cask_options_default(cask_options* o);

/* Open error detail (mirrors Error::InvalidChecksum / Io(UnexpectedEof) plus location). */
typedef struct cask_open_error {
  int32_t status;    /* cask_status */
  uint32_t file_id;
  uint64_t pos;
  uint32_t expected;
  uint32_t found;
} cask_open_error;

/* CaskOptions::open / Cask::open (cask.rs:328-330, 335-382). On failure returns NULL and fills
 * *err; hint files already recreated stay on disk, as in the reference. */
cask_db* cask_db_open(const char* path, const cask_options* opts, cask_open_error* err);
void cask_db_close(cask_db* db);

/* IndexEntry (cask.rs:20-26). */
typedef struct cask_index_entry {
  uint32_t file_id;
  uint32_t pad;
  uint64_t entry_pos;
  uint64_t entry_size;
  uint64_t sequence;
} cask_index_entry;

uint64_t cask_db_len(const cask_db* db);
/* Index::get (cask.rs:41-43). Returns 1 if present, 0 if absent. */
int cask_db_get_entry(const cask_db* db, const uint8_t* key, uint64_t ksz, cask_index_entry* out);
/* All live keys sorted bytewise: keys concatenated into key_bytes (capacity key_cap), with
 * key_off/key_len/entries of nkeys slots. Returns total key bytes, or negative on error. */
int64_t cask_db_export(const cask_db* db, uint8_t* key_bytes, uint64_t key_cap,
                       uint64_t* key_off, uint64_t* key_len, cask_index_entry* entries,
                       uint64_t nkeys);
/* Stats (stats.rs:6-67) sorted by file id. Returns the number of rows (may exceed cap). */
uint64_t cask_db_stats(const cask_db* db, uint32_t* file_id, uint64_t* entries,
                       uint64_t* dead_entries, uint64_t* dead_bytes, uint64_t cap);
/* current_sequence = max sequence seen + 1 (cask.rs:379). */
uint64_t cask_db_current_sequence(const cask_db* db);
/* Data file ids in ascending order (Log::files, log.rs:104-106). Returns count (may exceed cap). */
uint64_t cask_db_files(const cask_db* db, uint32_t* ids, uint64_t cap);
/* Timing of the replay phases (ms): [0] discover+read, [1] device scan, [2] hint write,
 * [3] keydir fold, [4] total. */
int cask_db_open_timings(const cask_db* db, double* ms5);

/* ------------------------------------------------------------------------------------------ */
/* Compaction merge (Cask::compact / compact_files / compact_files_aux, cask.rs:451-642).      */
/* ------------------------------------------------------------------------------------------ */
/* The CaskOptions compaction thresholds (cask.rs:229-234). */
typedef struct cask_compact_options {
  double fragmentation_trigger;    /* 0.6 */
  uint64_t dead_bytes_trigger;     /* 512 MiB */
  double fragmentation_threshold;  /* 0.4 */
  uint64_t dead_bytes_threshold;   /* 128 MiB */
  uint64_t small_file_threshold;   /* 10 MiB */
} cask_compact_options;

void cask_compact_options_default(cask_compact_options* o);

typedef struct cask_compact_result {
  uint32_t n_compacted;   /* files compacted (those with a valid hint file) */
  uint32_t n_new;         /* files created by live records (the reference's new_files) */
  uint32_t n_tomb_only;   /* files created by the tombstone tail alone (not in new_files,
                             cask.rs:518-520: on disk, not indexed, found at the next open) */
  uint32_t pad;
  uint64_t live_records;
  uint64_t tombstones;
  uint64_t bytes_in;      /* data bytes of the compacted files with live records (read from) */
  uint64_t bytes_out;     /* bytes written to new data files */
  double ms[5];           /* [0] hints + liveness, [1] live records copied from the mapped
                             sources + to the device + device verify, [2] placement,
                             [3] file writes (the wait for the writer thread and its last
                             batch), [4] keydir update + file swap */
  double ms_total;
} cask_compact_result;

/* Cask::compact_files(files) (cask.rs:525-560 over compact_files_aux 451-523): files are taken
 * as a set in ascending order; ids that are not data files of this db are ignored. Live records
 * (index sequence == hint sequence) are verified (Log::read_entry, log.rs:150-166) and rewritten
 * byte for byte through the LogWriter rollover; tombstones of keys absent from the index follow,
 * one per key with its highest sequence, in the order the keys were first seen (the reference
 * iterates a HashMap: its order is unspecified). On an error nothing is written and the
 * reference's error is returned (the reference may have written part of the output by then). */
int cask_db_compact_files(cask_db* db, const uint32_t* files, uint64_t nfiles, cask_compact_result* res,
                          cask_open_error* err);

/* Cask::compact (cask.rs:563-642): selects files by fragmentation, dead bytes and size, and
 * compacts them if a trigger fired. Returns the number of files compacted (0: not triggered) or
 * a negative status. */
int64_t cask_db_compact(cask_db* db, const cask_compact_options* opts, cask_compact_result* res,
                        cask_open_error* err);

/* The hint-file fast path's parse on the device (Log::hints -> Hints::next -> Hint::from_read,
 * log.rs:121-135, 437-447; data.rs:258-276): `files` are hint-file bodies in device memory, each
 * without its 4-byte XXH32 trailer (the caller checks it: is_valid_hint_file, log.rs:512-539).
 * Rows as cask_scan_device's, per hint record in order: pos = the record's offset in its body,
 * seq, ksz, vsz (raw: 0xFFFFFFFF for a tombstone), status Ok, or EOF for a record the body cuts
 * short (the first failure goes to *err: Io(UnexpectedEof), expected = found = 0). The entry
 * position and key are at pos + 14 and pos + 22 of the body. */
int cask_parse_hints_device(cask_ctx* ctx, const cask_file_view* files, uint32_t nfiles, cask_rows* rows,
                            uint64_t* file_row_offset, cask_scan_error* err);

/* Hint-file bodies on the device (RecreateHints::next + HintWriter::write, log.rs:382-386,
 * 454-465; Hint::write_bytes, data.rs:242-256): for every Ok row of a cask_scan_device call (same
 * files, rows and file_row_offset), in order, [sequence u64][key_size u16][value_size u32,
 * 0xFFFFFFFF for a tombstone][entry_pos u64][key], file after file into `out` (device memory,
 * `cap` bytes). file_hint_offset (host, nfiles + 1) receives where each file's body starts; the
 * caller appends the XXH32 trailer of each body (HintWriter::drop, log.rs:389-395). Returns
 * CASK_E_CAPACITY, with file_hint_offset filled in, when cap < file_hint_offset[nfiles]
 * (out may be NULL to ask for the size). */
int cask_hints_device(cask_ctx* ctx, const cask_file_view* files, uint32_t nfiles, const cask_rows* rows,
                      const uint64_t* file_row_offset, uint8_t* out, uint64_t cap, uint64_t* file_hint_offset);

/* ------------------------------------------------------------------------------------------ */
/* Multi-GPU replay. Data files shard in contiguous file-id ranges; each shard's   */
/* rows become a keydir block on its GPU; rank 0 folds the blocks in rank order. The block format */
/* is cask_amd/csrc/keydir_format.h: per key only the records that can decide the final keydir    */
/* (the suffix-strict maxima of the key's sequences within the shard), each tombstone whose stale */
/* count depends on the shards before it (with its threshold), per-file put counts, key bytes.    */
/* Keydir and Stats come out exactly as the single-process Cask::open (cask.rs:346-382, 60-90).   */
/* ------------------------------------------------------------------------------------------ */
/* A shard's keydir block from its device rows (cask_scan_device on `files`, every row Ok;
 * file_row_offset as that call returned it). *block points to device memory owned by the context,
 * valid until its next call; *bytes is its size. */
int cask_shard_keydir(cask_ctx* ctx, const cask_file_view* files, uint32_t nfiles, const cask_rows* rows,
                      const uint64_t* file_row_offset, const void** block, uint64_t* bytes);

/* The same block from hint-file bodies (the hint fast path of the replay, log.rs:121-135): `files`
 * and `rows` as cask_parse_hints_device took and returned them, every row Ok; the rows' pos is
 * rewritten to the entry positions the hints hold. */
int cask_shard_keydir_hints(cask_ctx* ctx, const cask_file_view* files, uint32_t nfiles, cask_rows* rows,
                            const uint64_t* file_row_offset, const void** block, uint64_t* bytes);

/* Copy `bytes` between any two memories (device or host) on the context's stream, synchronously:
 * e.g. a keydir block out of the context's buffer. */
int cask_copy(cask_ctx* ctx, void* dst, const void* src, uint64_t bytes);

/* Rank 0's fold: a keydir handle with no files, the blocks merged in rank order (host memory),
 * then finished (Stats). The result is a cask_db: cask_db_export / _stats / _current_sequence /
 * _len / _files / _get_entry read it; cask_db_close frees it. */
cask_db* cask_keydir_new(void);
int cask_keydir_merge(cask_db* db, const uint8_t* block, uint64_t bytes);
/* blocks[0..n) merged in order in one pass: the same keydir, terms and sequence as n calls of
 * cask_keydir_merge, with the tables sized once for all of them. */
int cask_keydir_merge_many(cask_db* db, const uint8_t* const* blocks, const uint64_t* bytes, uint32_t n);
int cask_keydir_finish(cask_db* db);

/* Key-hash partition, for a keyspace too large to gather on one host: a block splits
 * into nparts blocks of the same format (keydir_format.h), part o holding, in block order, the
 * records of the keys whose owner is o (cask_keydir_owner) with their keys, and the per-file stats
 * table (its counts in part 0 only). Owner o merges the parts it is sent in rank order
 * (cask_keydir_merge into a cask_keydir_new handle), reports its per-file terms
 * (cask_keydir_terms: 56-B KeydirTerm records), and every owner finishes with the terms of all
 * owners (cask_keydir_finish_terms): each then holds its own keys and the Stats, file list and
 * sequence of the whole replay — together exactly what cask_keydir_finish gives after one fold of
 * every block. */
uint32_t cask_keydir_owner(const uint8_t* key, uint64_t ksz, uint32_t nparts);
/* On the device (block in device memory, e.g. from cask_shard_keydir): *parts points to device
 * memory owned by the context, valid until its next partition; part_off (host, nparts + 1). */
int cask_keydir_partition(cask_ctx* ctx, const void* block, uint64_t bytes, uint32_t nparts, const void** parts,
                          uint64_t* part_off);
/* On the host, byte for byte the same parts: CASK_E_CAPACITY (part_off filled in) when cap <
 * part_off[nparts]; out may be NULL to ask for the size. */
int cask_keydir_partition_host(const uint8_t* block, uint64_t bytes, uint32_t nparts, uint8_t* out, uint64_t cap,
                               uint64_t* part_off);
/* Bytes of this owner's terms (written to out when cap allows), or a negative status. */
int64_t cask_keydir_terms(const cask_db* db, uint8_t* out, uint64_t cap);
int cask_keydir_finish_terms(cask_db* db, const uint8_t* terms, uint64_t bytes);

/* RCCL over xGMI (no torch needed; librccl is loaded on first use, CASK_E_DEVICE without it): a
 * communicator per rank from a unique id that one rank makes and the caller distributes (any side
 * channel: MPI, a file, a TCP socket). Every rank of the communicator makes the same calls; a failure
 * on any rank is agreed on (ncclAllReduce(min) of the ranks' statuses) before data moves, so every
 * rank returns the same status rather than waiting on a peer that stopped.
 *  - cask_keydir_gather_rccl: the rooted gather. Every rank passes its block (device memory, from
 *    cask_shard_keydir); the sizes and maximum sequences go round by ncclAllGather (*max_seq, on
 *    every rank, may be NULL), the blocks to `root` by grouped ncclSend/ncclRecv (one message per
 *    rank, each over its own xGMI link). On `root`, `db` (cask_keydir_new) gets the blocks merged in
 *    rank order — rank order must be replay order (contiguous file-id ranges) — and the caller then
 *    calls cask_keydir_finish. *gathered: the bytes the root received (its own block's size
 *    elsewhere). Replaces rank 0's side of the replay loop (cask.rs:346-382) for a sharded open.
 *  - cask_keydir_exchange_rccl: the key-hash all-to-all. Every rank's block is partitioned on its
 *    device into one part per rank, part o goes to rank o (grouped ncclSend/ncclRecv), each rank
 *    merges the parts it owns in rank order into its `db` (cask_keydir_new) and, after an
 *    ncclAllGather of the owners' terms, finishes it (cask_keydir_finish_terms). No rank holds more
 *    than its share of the keys. *sent / *received: this rank's bytes out to and in from the others
 *    (its own part included in *received). */
#define CASK_RCCL_ID_BYTES 128
int cask_rccl_unique_id(uint8_t* id /* CASK_RCCL_ID_BYTES */);
int cask_rccl_comm_init(const uint8_t* id, int nranks, int rank, int device, void** comm);
int cask_rccl_comm_destroy(void* comm);
int cask_keydir_gather_rccl(cask_ctx* ctx, void* comm, const void* block, uint64_t bytes, int root, cask_db* db,
                            uint64_t* gathered, uint64_t* max_seq);
int cask_keydir_exchange_rccl(cask_ctx* ctx, void* comm, const void* block, uint64_t bytes, cask_db* db,
                              uint64_t* sent, uint64_t* received);

/* Test hook (effective only with CASK_TEST_HOOKS=1 in the environment; CASK_E_INVALID_ARG
 * otherwise): force failures on one context — bit 1 the gather root's receive buffer cannot be
 * allocated, 2 cask_keydir_partition runs out of device memory, 4 the exchange cannot read its
 * per-file terms, 8 the next entry point called with it throws std::bad_alloc inside the library
 * (which must come back as CASK_E_NOMEM), 16 the fold of the received blocks fails. Lets a
 * multi-rank test make one rank fail at a chosen point. */
int cask_debug_inject(cask_ctx* ctx, uint32_t bits);

/* Cask::open over several GPUs of this process (replaces cask.rs:346-382 like cask_db_open): the
 * data files are split into contiguous ranges, one per entry of `devices` (a device may appear more
 * than once: its shards run one after another); within a range, files with a valid hint file are
 * replayed from it (the body parsed on the device, cask_parse_hints_device), the others scanned
 * (and given their hint files when opts->write_hints); each stretch of files of one kind becomes a
 * keydir block on its device, and the blocks are folded on the host in order. The ranges run in
 * parallel, but on a failure the hint files on disk are the reference's: those of the files up to
 * the failing one (it included, with its Ok records), none after it (cask.rs:357-368). */
cask_db* cask_db_open_multi(const char* path, const cask_options* opts, const int* devices, int ndevices,
                            cask_open_error* err);

#ifdef __cplusplus
}
#endif
#endif /* CASK_SCAN_H */
