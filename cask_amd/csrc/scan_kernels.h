// Shared between the HIP kernels (scan_kernels.hip) and the host runtime (scan_runtime.cpp).
#pragma once
#include <stdint.h>

namespace cask_dev {

// Chunking: the unit a workgroup stages into LDS and speculates a record boundary for.
constexpr uint32_t kWG = 256;                 // threads per workgroup (4 waves of 64)
constexpr uint32_t kChunk = 32768;            // bytes of file owned by one workgroup
constexpr uint32_t kHalo = 4096;              // extra bytes staged so boundary records hash in LDS
constexpr uint32_t kWin = kChunk + kHalo;     // staged window
constexpr uint32_t kMaxStarts = kChunk / 18 + 2;  // every record is >= 18 bytes (data.rs:11)
constexpr uint64_t kNone = ~0ull;             // "no record starts in this chunk"
constexpr uint64_t kTerm = ~0ull;             // chain ended by an UnexpectedEof record

enum : uint8_t { kRowOk = 0, kRowChecksum = 1, kRowEof = 2, kRowPendingLong = 3 };

struct FileDesc {
  const uint8_t* data;   // device pointer to the file's bytes
  uint64_t len;
  uint64_t first_chunk;  // global chunk index of this file's chunk 0
  uint64_t nchunks;      // ceil(len / kChunk)
};

struct Counters {
  unsigned long long ticket;   // chunk tickets handed out (in-order grab => deadlock-free look-back)
  unsigned long long nlong;    // records longer than the LDS window
  unsigned int overflow;       // row capacity exceeded
  unsigned int timeout;        // a bounded spin gave up (never expected)
  unsigned long long walk_steps;
};

struct ScanArgs {
  const FileDesc* files;
  uint32_t nfiles;
  uint32_t exact;              // 1: spec[] holds exact chunk starts (repair pass), no search
  uint64_t total_chunks;
  // per-chunk scratch
  unsigned long long* lb;      // decoupled look-back words: flag(2) | value(62)
  uint64_t* spec;              // start used by the chunk (kNone if none)
  uint64_t* exit;              // first chain position >= chunk end, or kTerm
  uint64_t* base;              // exclusive row prefix
  uint32_t* count;             // rows emitted by the chunk
  uint64_t* tin;               // validate: chain position entering the chunk
  // global
  Counters* ctr;
  uint64_t* long_row;          // row index of each long record
  uint32_t* long_file;         // file index of each long record
  uint64_t long_cap;
  unsigned long long* file_err_row;  // per file: min row index with a failing status
  // rows (device)
  uint64_t* pos;
  uint64_t* seq;
  uint32_t* vsz;
  uint16_t* ksz;
  uint8_t* status;
  uint64_t row_cap;
};

// Per-call summary written by k_summary, copied to the host in one transfer.
struct SummaryHead {
  uint64_t total_rows;
  uint64_t nlong;
  uint64_t overflow;
  uint64_t timeout;
  uint64_t any_invalid;
  uint64_t invalid_chunks;
  uint64_t walk_steps;
  uint64_t pad;
};
// followed by, per file f: row_off[f] (nfiles+1 entries), first_bad[f], bad_T[f], err_row[f]

// Host-callable launchers (defined in scan_kernels.hip).
void launch_scan_chunks(const ScanArgs& a, void* stream);
void launch_long(const ScanArgs& a, void* stream);
void launch_validate(const ScanArgs& a, uint64_t* first_bad, void* stream);
void launch_summary(const ScanArgs& a, const uint64_t* first_bad, uint64_t* summary, void* stream);
void launch_walk(const ScanArgs& a, const uint64_t* summary, void* stream);
void launch_err_detail(const ScanArgs& a, uint32_t fi, uint64_t row, uint32_t* out2, void* stream);
void launch_encode_synth(uint64_t nrec, const uint64_t* off, const uint64_t* seq,
                         const uint16_t* ksz, const uint32_t* vsz_raw, const uint64_t* key_id,
                         uint64_t value_seed, uint8_t* out, void* stream);
void launch_encode(uint64_t nrec, const uint64_t* off, const uint64_t* seq, const uint16_t* ksz,
                   const uint32_t* vsz_raw, const uint8_t* keys, const uint64_t* key_off,
                   const uint8_t* vals, const uint64_t* val_off, uint8_t* out, void* stream);
void launch_encode_checksum(uint64_t nrec, const uint64_t* off, const uint16_t* ksz,
                            const uint32_t* vsz_raw, uint8_t* out, void* stream);

}  // namespace cask_dev
