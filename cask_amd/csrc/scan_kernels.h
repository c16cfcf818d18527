// Shared between the HIP kernels (scan_kernels.hip) and the host runtime (scan_runtime.cpp).
#pragma once
#include <stdint.h>

namespace cask_dev {

// A chunk is the unit one workgroup stages into LDS and speculates a record boundary for; the
// geometry (chunk bytes, halo bytes, threads) is a template of k_scan_chunks chosen per call.
constexpr int kDefaultGeometry = 0;           // index into the k_scan_chunks instantiations
constexpr uint64_t kNone = ~0ull;             // "no record starts in this chunk" / no error
constexpr uint64_t kTerm = ~0ull;             // chain ended by an UnexpectedEof record

enum : uint8_t { kRowOk = 0, kRowChecksum = 1, kRowEof = 2 };

// Slot row (16 B) written by the chunk scan at slots[chunk * slot_cap + r]:
//   w0,w1 = seq (u64), w2 = vsz raw, w3 = ksz | offset-in-chunk << 16 | checksum-bad << 31.
// Status is implied: EOF if the record runs past the file end, else bad bit ? CHECKSUM : OK.
constexpr uint32_t kSlotBad = 0x80000000u;

// count[c] flag: the chunk is regular — its n rows are records of one length rl, all verified Ok
// and inside the window, with key size, value size and sequence step of one from its first row
// (row r = pos0 + r*rl, seq0 + r, vsz0, ksz0). Only that row is stored, in desc[c] (slot-row
// format); k_compact expands the rest.
// Set only when the dense output is requested (ScanArgs.regular_ok); the segmented output keeps
// every row.
constexpr uint32_t kCountRegular = 0x80000000u;
constexpr uint32_t kCountMask = 0x7FFFFFFFu;

struct FileDesc {
  const uint8_t* data;   // device pointer to the file's bytes
  uint64_t len;
  uint64_t first_chunk;  // global chunk index of this file's chunk 0
  uint64_t nchunks;      // ceil(len / chunk)
  uint64_t first_tile;   // first validation tile (kTile chunks) of this file
  uint64_t pad;
};

constexpr uint32_t kTileChunks = 1024;  // chunks per validation tile (k_pipeline.hip kTile)

// Per-call counters and flags, at the head of the call block (zeroed by one memset per call and
// read back by the host in one copy, with the per-file arrays that follow it: see CallLayout).
struct Counters {
  unsigned long long nlong;      // records longer than the LDS window
  unsigned long long walk_steps; // repair walk iterations
  unsigned long long total_rows; // k_finish: rows of the call
  unsigned int run_next;         // k_scan_chunks: next run of chunks to hand out
  unsigned int tile_next;        // k_finish: next tile of chunks to hand out
  unsigned int any_invalid;      // k_finish: some chunk's speculated start is wrong (repair path)
  unsigned int long_pending;     // k_finish: some chunk has rows for k_long
  unsigned int lq_cnt[22];       // long-record queue: entries per length class 2^10 .. 2^31+
  unsigned int walk_next[8];     // k_walk_runs: next run of each walk group to hand out (kWalkGroups)
  unsigned int search_next[8];   // k_walk_search: the same, for the searches
  unsigned int hash_next;        // k_walk_hash: next run to hand out (after the first by index)
  unsigned int slot_overflow;    // k_walk_chase: a chunk had more records than the slot rows sized
};

// Layout of the call block: Counters, then row_off[nfiles + 1] (each file's first dense row,
// written by k_finish at the file's first chunk), then err_inv[nfiles] (~ the file's first failing
// dense row, by atomicMax: 0 = none).
struct CallLayout {
  static constexpr uint64_t kHead = 256;  // bytes reserved for Counters
  static uint64_t bytes(uint32_t nfiles) { return kHead + 8ull * (nfiles + 1) + 8ull * nfiles; }
};
static_assert(sizeof(Counters) <= CallLayout::kHead, "Counters outgrew the call block head");

// Long-record queue (k_long_enqueue -> k_long_hash): slot indices of the records hashed from HBM,
// one region per length class b (record length in [2^b, 2^(b+1)), b = 10..31, the last open-ended),
// so that the lanes of a wave hash records of similar length. Region b holds at most
// (chunk >> b) + 1 records per chunk: records do not overlap, and those of a chunk start within it.
constexpr uint32_t kLqMinLog = 10, kLqClasses = 22;
constexpr uint32_t kMinBigRec = 1u << kLqMinLog;  // ScanArgs::big is never below this
__host__ __device__ __forceinline__ uint64_t lq_region_cap(uint64_t chunks, uint32_t chunk, uint32_t b) {
  return chunks * ((uint64_t)(chunk >> b) + 1);
}
__host__ __device__ __forceinline__ uint64_t lq_region_base(uint64_t chunks, uint32_t chunk, uint32_t b) {
  uint64_t o = 0;
  for (uint32_t j = kLqMinLog; j < b; ++j) o += lq_region_cap(chunks, chunk, j);
  return o;
}

struct ScanArgs {
  const FileDesc* files;
  uint32_t nfiles;
  uint32_t exact;              // 1: spec[] holds exact chunk starts (repair pass), no search
  uint64_t total_chunks;
  uint32_t chunk;              // chunk bytes of the geometry in use
  uint32_t slot_cap;           // row slots per chunk (chunk / 18 + 2)
  // per-chunk
  uint64_t* spec;              // start used by the chunk (kNone if none)
  uint64_t* exit;              // first chain position >= chunk end, or kTerm
  uint32_t* count;             // rows in the chunk
  uint64_t* base;              // exclusive row prefix of the chunk within its file
  uint64_t* tin;               // validate: chain position entering the chunk
  uint32_t* slots;             // 4 words per slot row
  // validation tiles
  uint64_t total_tiles;
  uint64_t* tile_max;          // per tile: max exit
  uint64_t* tile_sum;          // per tile: row count
  uint64_t* tile_pmax;         // per tile: exclusive max within the file
  uint64_t* tile_psum;         // per tile: exclusive row prefix within the file
  // per-file
  uint64_t* file_total;        // rows per file
  unsigned long long* file_err;  // min slot index with a failing row
  uint64_t* first_bad;         // first chunk whose speculated start is wrong (kNone: none)
  // global
  Counters* ctr;
  uint32_t* long_r;            // per chunk: row of its record longer than the window, or !0
  uint32_t* desc;              // per chunk, 4 words: the first row of a regular chunk (kCountRegular)
  // dense rows (compaction output, device)
  uint64_t* pos;
  uint64_t* seq;
  uint32_t* vsz;
  uint16_t* ksz;
  uint8_t* status;
  uint64_t row_cap;
  unsigned long long* stamps;  // diagnostic builds only (-DCASK_STAMPS): per-phase cycle sums, then
                               // k_run_hash's per-wave start/end real times ([16 + 2 w], [17 + 2 w])
  uint32_t run;                // k_scan_chunks: consecutive chunks a workgroup walks with a carry
  uint32_t run_small;          // k_scan_chunks: chunks per run from run_tail on
  uint64_t run_tail;           // k_scan_chunks: first chunk of the short runs (a multiple of run;
                               // >= total_chunks: none)
  uint32_t regular_ok;         // 1: a regular chunk may keep only its first slot row (kCountRegular)
  uint32_t respec;             // 1: validation rewrites an invalid chunk's start from T[c] (local repair)
  uint32_t big;                // records longer than this are hashed by k_long from HBM, not in LDS
  uint32_t win;                // bytes staged per chunk (chunk + halo): the LDS window
  // sparse repair: chunk errors that outlive a pass, and the chunks a repair pass re-scans
  uint32_t* cerr;              // per chunk: first failing row (!0: none), written by every scan of it
  uint8_t* redo;               // per chunk: 1 if the last validation found its start wrong
  const uint64_t* runs;        // repair pass: [first, end) chunk stretches to re-scan (null: all)
  uint64_t nruns_list;         // stretches in runs[]
  uint8_t* long_done;          // per chunk: 1 once k_long_enqueue has queued its long records
                               // (every scan of the chunk clears it)
  uint64_t* lq;                // long-record queue: slot indices by length class (lq_region_base)
  // dense path (k_finish): rows go straight from the chunk table to the caller's arrays
  uint32_t dense;              // 1: k_finish validated every chunk; k_long also fixes dense rows
  uint32_t epoch;              // tag of this call's lookback granules (1..255)
  uint64_t* tstate;            // k_finish lookback: 8 granules per tile
  uint64_t* gbase;             // per chunk: its first dense row (k_finish)
  uint64_t* row_off;           // call block: per file first dense row
  unsigned long long* err_inv; // call block: per file ~first failing dense row (0: none)
  uint32_t vec_ok;             // dense arrays aligned for the 4-row vector stores of k_finish
  uint32_t hint;               // 1: the files are hint-file bodies (cask_parse_hints_device), not data files
  uint32_t call_zero_words;    // k_finish: words of call_zero to clear
  uint32_t fin_static;         // k_finish: tile = blockIdx.x (the grid fits the GPU at once)
  uint64_t* call_zero;         // k_finish: the call block the next call uses (null: none)
  uint32_t walk_pre;           // 1: k_walk_search left each run's speculative start in tin[first chunk]
  uint32_t grp;                // walk mode: the group of runs a launch covers (its claim counters)
  // walk mode, one group of runs per launch (0 = to the end): runs [run_lo, run_hi) for
  // k_walk_search / k_walk_runs, chunks [t_lo, t_hi) for k_long_enqueue, and per
  // length class the queue entries [lq_lo, lq_hi) for k_long_hash (null: from 0 / to lq_cnt)
  uint64_t run_lo, run_hi;
  uint64_t t_lo, t_hi;
  const uint32_t* lq_lo;
  const uint32_t* lq_hi;
  // walk mode, split path (k_walk_chase -> k_run_hash): per chunk, the address of its first byte and
  // the end of its file's last 16-B granule (2 x u64), written by the chase
  uint64_t* cdesc;
  // a call whose runs are split between the modes (per region of each file: k_probe_regions): the
  // walk-mode runs, by index (k_walk_search, k_walk_chase, k_run_hash; null: every run); the
  // chunk-mode runs go to k_scan_chunks as a.runs stretches
  const uint64_t* wruns;
  uint64_t nwruns;
  // k_walk_search: candidates of at most this many bytes are verified by their checksum, longer
  // ones are listed for the hop back (kSearchShort; CASK_SEARCH_SHORT tuning knob)
  uint32_t search_short;
  uint32_t pad_ss;
  // walk mode, k_run_hash's tail: the last hash_ntail runs are handed out in kTailSplit pieces,
  // each piece twice — its records of at least kTailLong bytes right after the other runs, its
  // shorter ones last — so that the kernel ends on short records; tbits: per piece kTailBitWords
  // words, bit i = its record i is long (written by k_walk_chase). hash_ntail 0: one pass.
  uint64_t hash_ntail;
  uint32_t* tbits;
};

// Default ScanArgs::big: records longer than 2 KiB are hashed by k_long_hash, many lanes at once,
// instead of by one quad of the chunk's workgroup while the rest of it waits (configs[2]: 32 GiB of
// Zipf-length records, 841 -> 1,005 GiB/s with per-lane hashing, 1,337 with quads; fixed
// 290-B records never reach it).
constexpr uint32_t kBigRec = 2048u;

// Whether the chunk scan hashes the record [p, p + rl) of a chunk whose window ends at wend out of
// LDS (the same rule in k_scan_chunks and k_long): it fits the window and is at most `big` long.
__host__ __device__ __forceinline__ bool lds_hashed(uint64_t p, uint64_t rl, uint64_t wend, uint32_t big) {
  return p + rl <= wend && rl <= big;
}

constexpr uint32_t kDefaultRun = 16, kMaxRun = 64;
// Walk mode (k_walk.hip): chunks per run, and the mean record length (bytes, sampled at the heads
// of the files by k_probe) from which a call takes it.
// Slot rows per chunk of a pure walk-mode call (records average >= kWalkMean bytes: 32 per 32-KiB
// chunk on average; configs[2], mean 5,114 B: at most 60 in 11 M chunks). A chunk with more sets
// Counters::slot_overflow and the call is redone with the full count (chunk / 18 + 2).
constexpr uint32_t kWalkSlotCap = 128;
constexpr uint32_t kWalkRun = 32, kWalkMean = 1024;  // (configs[2]: 32-chunk runs 2 % faster than 64)
#ifndef CASK_TAIL_SPLIT_N  // (A/B variant)
#define CASK_TAIL_SPLIT_N 2
#endif
constexpr uint32_t kTailSplit = CASK_TAIL_SPLIT_N;  // pieces per tail run (k_run_hash)
#ifndef CASK_TAIL_LONG
#define CASK_TAIL_LONG 24576
#endif
constexpr uint32_t kTailLong = CASK_TAIL_LONG;  // a tail piece's records at least this long go first
constexpr uint32_t kTailMaxRecs = kWalkRun / kTailSplit * kWalkSlotCap;  // records a piece can hold
constexpr uint32_t kTailBitWords = kTailMaxRecs / 32;
// k_run_hash loads a piece's bit words one per lane and lists its records in LDS: a variant with
// more words than lanes would leave records unhashed, so it must not compile
static_assert(kTailBitWords <= 64, "a tail piece's long-record bits are loaded one word per lane");
static_assert(4 * 2 * kTailMaxRecs * 2 <= 32768, "k_run_hash's tail lists outgrew their LDS budget");
// Chunk mode: the short-halo geometry (kGeoShortHalo, a 1,008-B halo) when the records at the file
// heads average at most kShortHaloMean bytes and none is longer than kShortHaloMax; else the wide
// halo (kDefaultGeometry, 4,080 B). Speed only: a record that crosses the window goes to k_long.
constexpr int kGeoShortHalo = 3;
constexpr uint32_t kShortHaloMean = 512, kShortHaloMax = 1008;
constexpr uint32_t kHintRun = 2;  // hint bodies: 22 + ksz-byte records, ~1,700 per 64 KiB run
// Walk mode on data files runs in groups of runs: group g's long records are hashed on a second
// stream while group g + 1 is walked (the walk is bound by latency, the long hash by HBM).
constexpr uint32_t kWalkGroups = 8, kWalkGroupsDefault = 4;
// Walk mode on data files: ScanArgs::big. The walker hashes records up to this long out of its
// 1-KiB LDS window (its usable bytes); longer ones go to k_long_hash. (Length class 10 of the
// long-record queue holds them: at most (chunk >> 10) + 1 records longer than this start per chunk.)
constexpr uint32_t kWalkHashMax = 1008;
static_assert(sizeof(((Counters*)nullptr)->walk_next) == 4 * kWalkGroups, "a claim counter per walk group");

// Per-call summary written by k_summary, copied to the host in one transfer.
struct SummaryHead {
  uint64_t total_rows;
  uint64_t nlong;
  uint64_t any_invalid;
  uint64_t invalid_chunks;
  uint64_t walk_steps;
  uint64_t pad[3];
};
// followed by row_off[nfiles+1], then per file: first_bad, bad_T, err_row, err_slot

// Host-callable launchers (defined in scan_kernels.hip).
void launch_read_entries(const uint64_t* pos, const uint32_t* src, uint64_t n, const uint8_t* const* srcs,
                         const uint64_t* slen, uint64_t* len, uint8_t* st, uint32_t* expct, uint32_t* found, void* stream);
uint32_t geometry_chunk(int geo);
uint32_t geometry_halo(int geo);
void launch_scan_chunks(const ScanArgs& a, int geo, void* stream);
int device_cus();  // compute units of the current device (cached per device)
void launch_long(const ScanArgs& a, void* stream, bool enqueue = true);  // k_long_enqueue + k_long_hash
void launch_long_enqueue(const ScanArgs& a, void* stream);
void launch_long_hash(const ScanArgs& a, void* stream);
void launch_validate(const ScanArgs& a, void* stream);
void launch_summary(const ScanArgs& a, uint64_t* summary, void* stream);
void launch_compact(const ScanArgs& a, const uint64_t* summary, void* stream);
constexpr uint32_t kFinTile = 256;  // chunks per k_finish tile (one per thread)
constexpr uint32_t kFinGroup = 32;  // k_finish tiles per group of the two-level prefix
void launch_finish(const ScanArgs& a, void* stream);
void launch_err_dense(const ScanArgs& a, uint32_t fi, uint64_t row, uint32_t* out, void* stream);
// k_keydir.hip: a shard's keydir block (keydir_format.h) from its dense rows
void* kd_scratch_create();
void kd_scratch_destroy(void* s);
int kd_build(void* scratch, const FileDesc* files_host, const uint32_t* file_ids_host, uint32_t nfiles,
             const uint64_t* row_off_host, const uint64_t* pos, const uint64_t* seq, const uint32_t* vsz,
             const uint16_t* ksz, uint64_t n, void* stream, void** out, uint64_t* bytes,
             const uint64_t* key_at = nullptr);
int kd_partition(void* scratch, const void* block, uint64_t bytes, uint32_t nparts, void* stream, void** out,
                 uint64_t* part_off);
int hint_entries(void* scratch, const FileDesc* files_host, uint32_t nfiles, const uint64_t* row_off_host,
                 uint64_t n, uint64_t* pos, uint64_t* key_at, void* stream);
int hint_pack(void* scratch, const FileDesc* files_host, uint32_t nfiles, const uint64_t* row_off_host,
              const uint64_t* pos, const uint64_t* seq, const uint32_t* vsz, const uint16_t* ksz, const uint8_t* status,
              uint64_t n, uint8_t* out, uint64_t cap, uint64_t* file_start, void* stream);
void launch_walk(const ScanArgs& a, const uint64_t* summary, void* stream);
void launch_walk_runs(const ScanArgs& a, void* stream);  // k_walk.hip: hint bodies (cask_parse_hints_device)
// (cus: the compute units the launch's stream may use, for its persistent grid; 0 = all of them)
void launch_walk_search(const ScanArgs& a, void* stream, int cus = 0);  // k_walk.hip: each walk run's speculative start
// k_walk_hash.hip: k_walk_chase (a lane per run of a.run chunks chases the record
// headers: slot rows, chunk table, cdesc), then k_run_hash (a wave per claimed run, a quad per record:
// every record hashed from HBM, whole 128-B lines per load instruction)
void launch_walk_chase(const ScanArgs& a, void* stream);
void launch_run_hash(const ScanArgs& a, void* stream, int cus = 0);
uint64_t run_hash_waves();  // k_run_hash's persistent grid, in waves
// after k_finish ran beside k_run_hash: the checksum statuses of the chunks with a failing row
void launch_hash_fix(const ScanArgs& a, void* stream);
// the slot rows of a walk-mode call re-strided from a.slot_cap to cap_dst rows per chunk (the
// repair path's exact chunk scans may write a chunk's full count)
void launch_restride(const ScanArgs& a, uint32_t* dst, uint32_t cap_dst, void* stream);
// k_walk.hip: record lengths at kProbeRegions points of every file, 3 u64 per point (k_probe_regions)
constexpr uint32_t kProbeRegions = 8;
constexpr uint32_t kStampWaves = 8192;  // diagnostic builds: waves with start/end stamps
constexpr uint32_t kStampRuns = 65536;  // diagnostic builds: searches with start/end/windows stamps
constexpr uint64_t kStampDry = 16 + 2ull * kStampWaves + 4ull * kStampRuns;  // k_run_hash: per wave, runs ran dry
constexpr uint64_t kStampWords = kStampDry + kStampWaves;
void launch_probe_regions(const FileDesc* files, uint32_t nfiles, unsigned long long* out, void* stream);
void launch_err_detail(const ScanArgs& a, uint32_t fi, uint64_t slot, uint32_t* out, void* stream);
void launch_encode_synth(uint64_t nrec, const uint64_t* off, const uint64_t* seq,
                         const uint16_t* ksz, const uint32_t* vsz_raw, const uint64_t* key_id,
                         uint64_t value_seed, uint8_t* out, void* stream);
void launch_encode(uint64_t nrec, const uint64_t* off, const uint64_t* seq, const uint16_t* ksz,
                   const uint32_t* vsz_raw, const uint8_t* keys, const uint64_t* key_off,
                   const uint8_t* vals, const uint64_t* val_off, uint8_t* out, void* stream);
void launch_encode_checksum(uint64_t nrec, const uint64_t* off, const uint16_t* ksz,
                            const uint32_t* vsz_raw, uint8_t* out, void* stream);

}  // namespace cask_dev
