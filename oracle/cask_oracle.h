/*
 * cask_oracle.h — CPU restatement of Cask's replay hot path. TEST INFRASTRUCTURE ONLY.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this
 * library, and only as the checker / the timed CPU baseline. The product path
 * (cask_amd/, include/cask_scan.h) never links or calls it.
 *
 * Reference: andresilva/cask v0.7.1 (Rust). Each function cites the reference lines it
 * restates. The Rust crate cannot be built here (no rustc/cargo), so there is no
 * oracle/_ref build; the XXH32 arithmetic lives in the absent crate `twox-hash`
 * ("1.1.0", caret: Cargo.toml:18) and is restated from the published XXH32 spec, pinned
 * against libxxhash 0.8.2 (python-xxhash 3.8.1) by tests/test_oracle.py.
 */
#ifndef CASK_ORACLE_H
#define CASK_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- XXH32 (util.rs:10-41 -> twox-hash XxHash32::with_seed(0)) ---- */
typedef struct {
  uint64_t total_len;
  uint32_t v[4];
  uint8_t mem[16];
  uint32_t memsize;
  uint32_t seed;
} orc_xxh32_state;

void orc_xxh32_reset(orc_xxh32_state* s, uint32_t seed);
void orc_xxh32_update(orc_xxh32_state* s, const uint8_t* p, size_t len);
uint32_t orc_xxh32_digest(const orc_xxh32_state* s);
uint32_t orc_xxh32(const uint8_t* p, size_t len, uint32_t seed);

/* ---- record codec (data.rs) ---- */
#define ORC_ENTRY_STATIC_SIZE 18u        /* data.rs:11 */
#define ORC_ENTRY_TOMBSTONE 0xFFFFFFFFu  /* data.rs:12 */

/* Entry::write_bytes (data.rs:90-121). Returns bytes written to out (18+ksz+vsz_eff). */
size_t orc_entry_encode(uint64_t seq, const uint8_t* key, uint16_t ksz, const uint8_t* value,
                        uint32_t vsz, int deleted, uint8_t* out);

/* Row = what Entries::next yields per record (log.rs:403-429) in the scan's SoA form. */
enum { ORC_ROW_OK = 0, ORC_ROW_CHECKSUM = 1, ORC_ROW_EOF = 2 };
typedef struct {
  uint64_t pos;      /* entry_pos (log.rs:413) */
  uint64_t seq;      /* Entry.sequence */
  uint32_t vsz_raw;  /* value_size header field; 0xFFFFFFFF = tombstone */
  uint16_t ksz;
  uint8_t status;    /* ORC_ROW_* */
  uint8_t pad;
  uint32_t expected; /* stored checksum (InvalidChecksum.expected) */
  uint32_t found;    /* computed XXH32 (InvalidChecksum.found) */
} orc_row;

/* Entries over an in-memory data file: Entry::from_read per record (data.rs:161-206),
 * position advances by the bytes consumed (log.rs:415-417); iteration keeps going after a
 * checksum error (the RecreateHints::drop drain, log.rs:467-471) and ends after an EOF.
 * Returns the number of rows (>= 0), or -1 if cap is too small. */
int64_t orc_scan_buffer(const uint8_t* buf, uint64_t len, orc_row* rows, uint64_t cap);

/* Hint bytes for one OK row (Hint::write_bytes, data.rs:242-256). Returns bytes (22+ksz). */
size_t orc_hint_encode(uint64_t seq, uint16_t ksz, uint32_t vsz_raw, uint64_t pos,
                       const uint8_t* key, uint8_t* out);

/* ---- keydir fold (cask.rs:60-90) + stats (stats.rs:23-48) ---- */
typedef struct orc_index orc_index;
orc_index* orc_index_new(void);
void orc_index_free(orc_index* ix);
/* Index::update for one Hint of file file_id. vsz_raw is the hint value_size field. */
void orc_index_update(orc_index* ix, const uint8_t* key, uint16_t ksz, uint32_t file_id,
                      uint64_t pos, uint32_t vsz_raw, uint64_t seq);
uint64_t orc_index_len(const orc_index* ix);
/* Export live entries sorted by key bytes (memcmp order, shorter first on tie).
 * keys_out receives concatenated keys; each array has orc_index_len() slots. */
void orc_index_export(const orc_index* ix, uint8_t* keys_out, uint64_t* key_off,
                      uint16_t* key_len, uint32_t* file_id, uint64_t* pos, uint64_t* size,
                      uint64_t* seq);
/* Stats rows sorted by file_id; returns the number of stats rows (<= cap). */
uint64_t orc_index_stats(const orc_index* ix, uint32_t* file_id, uint64_t* entries,
                         uint64_t* dead_entries, uint64_t* dead_bytes, uint64_t cap);

/* ---- replay drivers: Cask::open (cask.rs:335-382) for data files with no hint file ---- */
typedef struct {
  uint64_t records;      /* rows folded */
  uint64_t bytes;        /* data-file bytes consumed */
  uint64_t max_seq;      /* sequence = max(sequence, hint.sequence) (cask.rs:350-352) */
  int32_t err_kind;      /* 0 none, ORC_ROW_CHECKSUM, ORC_ROW_EOF, -1 io */
  uint32_t err_file_id;
  uint64_t err_pos;
  uint32_t err_expected, err_found;
  uint64_t live_keys;
} orc_replay_result;

/* Reference-faithful replay of one data file: unbuffered read(2) of header/key/value per
 * record (data.rs:162-183), streaming XXH32 in 3 updates (data.rs:185-191), 5 write(2) per
 * hint into hint_path (data.rs:242-256, log.rs:382-386) plus the trailer (log.rs:389-395),
 * and Index::update with a key copy (cask.rs:60-90). Single thread (cask.rs:348). */
int orc_replay_file_faithful(const char* data_path, const char* hint_path, uint32_t file_id,
                             orc_index* ix, orc_replay_result* res);

/* Fast restatement (mmap'd buffer, tight loop): scan + fold, no hint file. Context only. */
int orc_replay_buffer_fast(const uint8_t* buf, uint64_t len, uint32_t file_id, orc_index* ix,
                           orc_replay_result* res);

/* Index::get (cask.rs:41-43): 1 and the entry if the key is live, else 0. */
int orc_index_get(const orc_index* ix, const uint8_t* key, uint16_t ksz, uint32_t* file_id, uint64_t* pos,
                  uint64_t* size, uint64_t* seq);

/* ---- compaction merge: Cask::compact_files_aux (cask.rs:451-523) ---- */
typedef struct {
  uint32_t n_compacted;  /* files with a valid hint file (compacted_files) */
  uint32_t n_new;        /* files started by live records (new_files, cask.rs:510-512) */
  uint32_t n_tomb_only;  /* files started by the tombstone tail (not in new_files, cask.rs:518-520) */
  uint32_t file_id_seq;  /* the id sequence after the call (Sequence, util.rs:55-65) */
  uint64_t n_out;        /* files written, in creation order (out_ids) */
  uint64_t live_records, tombstones, bytes_out;
  int32_t err_kind;      /* 0, ORC_ROW_CHECKSUM, ORC_ROW_EOF (read_entry / a hint cut short), -1 io */
  uint32_t err_file_id;
  uint64_t err_pos;
  uint32_t err_expected, err_found;
} orc_compact_result;

/* compact_files_aux over `files` in the given order, reading data/hint files from src_dir and
 * writing the new data/hint files (ids file_id_seq+1, ...) into dst_dir: per file with a valid hint
 * file, every hint decides liveness against `ix` (index sequence == hint sequence, cask.rs:500) or
 * records a tombstone of an absent key (highest sequence per key, cask.rs:487-499); the live
 * entries are read back (Log::read_entry, log.rs:150-166: EOF / checksum errors end the call) and
 * written through the LogWriter rollover (log.rs:282-306); the tombstones follow, in first-seen
 * order (the reference's HashMap order is unspecified). out_ids/out_live (cap entries) receive the
 * created files in order and whether a live record started each. Returns 0, or -1 with res->err_*.
 * Nothing is removed from src_dir and `ix` is not updated. Test infrastructure only. */
int orc_compact_files(const char* src_dir, const char* dst_dir, const orc_index* ix, const uint32_t* files,
                      uint64_t nfiles, uint32_t file_id_seq, uint64_t max_file_size, uint32_t* out_ids,
                      uint8_t* out_live, uint64_t cap, orc_compact_result* res);

/* The same with liveness from any keydir: seq_of(ix, key, ksz, &seq) returns 1 and the key's
 * sequence if the key is live (Index::get, cask.rs:41-43), else 0. */
typedef int (*orc_seq_fn)(const void* ix, const uint8_t* key, uint16_t ksz, uint64_t* seq);
int orc_compact_files_fn(const char* src_dir, const char* dst_dir, orc_seq_fn seq_of, const void* ix,
                         const uint32_t* files, uint64_t nfiles, uint32_t file_id_seq, uint64_t max_file_size,
                         uint32_t* out_ids, uint8_t* out_live, uint64_t cap, orc_compact_result* res);

/* RecreateHints over one in-memory data file (log.rs:137-148, 449-471): the hint body (no trailer)
 * into out; its length, or -1 if cap is too small. */
int64_t orc_hint_body(const uint8_t* buf, uint64_t len, uint8_t* out, uint64_t cap);

/* ---- Cask::open replay of many in-memory data files on host threads (cask_oracle_par.c) ---- */
typedef struct {
  uint64_t records;    /* rows folded */
  uint64_t live;       /* keys in the keydir */
  uint64_t max_seq;
  uint64_t digest;     /* sum (mod 2^64) of orc_entry_digest over the keydir: order-independent */
  uint64_t stats_rows; /* per-file Stats rows (may exceed the caller's cap) */
  int32_t err_kind;    /* the first failure in replay order (0 none): open() stops there */
  uint32_t err_file_id;
  uint64_t err_pos;
  uint32_t err_expected, err_found;
} orc_parallel_result;

/* One keydir entry's digest: splitmix64-chained over ksz, the key in 8-byte little-endian words
 * (zero-padded), file_id, entry_pos, entry_size, sequence. orc_index_digest sums it over the live
 * entries of an index. */
uint64_t orc_entry_digest(const uint8_t* key, uint16_t ksz, uint32_t file_id, uint64_t pos, uint64_t size,
                          uint64_t seq);
uint64_t orc_index_digest(const orc_index* ix);

/* The scan + Index::update fold of files bufs[0..nfiles) in that (replay) order, exactly as
 * Cask::open without hint files (cask.rs:346-382, 60-90): files scanned on nthreads threads, the
 * fold split by key over nthreads partitions. Stats rows (unsorted) go to st_* (st_cap entries). */
int orc_replay_parallel(const uint8_t* const* bufs, const uint64_t* lens, const uint32_t* file_ids, uint32_t nfiles,
                        uint32_t nthreads, orc_parallel_result* res, uint32_t* st_fid, uint64_t* st_e, uint64_t* st_d,
                        uint64_t* st_b, uint64_t st_cap);
/* The same, keeping the partitioned keydir for lookups (orc_pindex_seq, an orc_seq_fn) — e.g. the
 * liveness of orc_compact_files_fn. */
typedef struct orc_pindex orc_pindex;
orc_pindex* orc_pindex_build(const uint8_t* const* bufs, const uint64_t* lens, const uint32_t* file_ids,
                             uint32_t nfiles, uint32_t nthreads, orc_parallel_result* res, uint32_t* st_fid,
                             uint64_t* st_e, uint64_t* st_d, uint64_t* st_b, uint64_t st_cap);
int orc_pindex_seq(const void* pindex, const uint8_t* key, uint16_t ksz, uint64_t* seq);
void orc_pindex_free(orc_pindex* p);

#ifdef __cplusplus
}
#endif
#endif
