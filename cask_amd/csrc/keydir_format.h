// The keydir block of one shard: what a rank of the multi-GPU replay sends to rank 0 (SURVEY.md
// §8e). Built on the device by cask_shard_keydir (k_keydir.hip), folded on the host by
// cask_keydir_merge (engine.cpp). Little-endian, 8-byte aligned:
//   ShardHeader | ShardRec[nrec] | ShardFileStat[nfiles] | key bytes of the records, in record order
// Records of one key appear in the shard's replay order (file id, pos).
//
// Key-hash partition (the huge-keyspace case): a block splits into nparts blocks of
// the same format, part o holding, in block order, the records whose key's owner is o (every record
// of a key goes to one part, so each part folds exactly as the whole block would for those keys),
// their keys, and the per-file stats table — its counts in part 0 only (they are per-shard sums),
// zeroed in the others so that every owner still learns every file. Owner o folds the parts it gets
// from the ranks in rank order and reports its KeydirTerm per file; the terms of all owners summed
// give Stats (stats.rs) exactly as one fold of the whole blocks.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace cask_kd {

constexpr uint32_t kMagic = 0x52444B43u;  // "CKDR"
constexpr uint32_t kVersion = 1;

struct ShardHeader {      // 64 B
  uint32_t magic, version;
  uint64_t nrec;          // records
  uint64_t key_bytes;     // bytes of the key blob
  uint32_t nfiles;        // ShardFileStat entries
  uint32_t pad;
  uint64_t max_seq_p1;    // max sequence over every record of the shard, + 1 (0: no record)
  uint64_t rows_in;       // rows the shard's scan produced
  uint64_t bytes;         // total bytes of the block
  uint64_t pad2;
};

// kind: what the fold on rank 0 does with the record
enum : uint8_t {
  kKept = 0,  // a suffix-strict maximum of its key in the shard: Index::update's keydir effect
  kCond = 1,  // a tombstone whose stale count depends on the keydir entering the shard: it counts
              // (entries, dead, dead_bytes) += (1, 1, 18 + ksz) in its file iff the key's entry at
              // that point has sequence + 1 > seq (seq holds the threshold T + 1; a vacant key is 0)
  kRaw = 2,   // every record of a 64-bit key-hash collision: folded one by one (Index::update)
};

struct ShardRec {         // 32 B
  uint64_t pos;           // entry_pos
  uint64_t seq;           // sequence (kCond: the threshold + 1)
  uint32_t file_id;
  uint32_t vsz;           // raw value_size (0xFFFFFFFF: tombstone)
  uint16_t ksz;
  uint8_t kind;
  uint8_t pad0;
  uint32_t pad1;
};

struct ShardFileStat {    // 40 B: the shard's order-free stats terms per data file
  uint32_t file_id, pad;
  uint64_t puts;          // records that are not tombstones (each adds one entry)
  uint64_t put_bytes;     // their entry sizes
  uint64_t stale;         // tombstones stale whatever the keydir entering the shard
  uint64_t stale_bytes;   // their entry sizes (18 + ksz)
};

// An owner's share of the per-file Stats terms after folding its parts (cask_keydir_terms).
struct KeydirTerm {       // 56 B
  uint32_t file_id, pad;
  uint64_t puts, put_bytes;      // from part 0's stats table
  uint64_t stale, stale_bytes;   // stale tombstones (part 0's order-free ones + this owner's kCond)
  uint64_t live, live_bytes;     // this owner's keys whose final entry is in the file
};

static_assert(sizeof(ShardHeader) == 64 && sizeof(ShardRec) == 32 && sizeof(ShardFileStat) == 40 &&
                  sizeof(KeydirTerm) == 56, "layout");

// The 64-bit key hash of the blocks (k_keydir.hip groups a shard's rows by it) and the owner of a key
// among nparts (its high 32 bits scaled to [0, nparts)): the same function on the device and the host.
__host__ __device__ inline uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
__host__ __device__ inline uint64_t key_hash(const uint8_t* k, uint32_t n) {
  uint64_t h = 0x9E3779B97F4A7C15ull ^ ((uint64_t)n * 0xD6E8FEB86659FD93ull);
  uint32_t i = 0;
  for (; i + 8 <= n; i += 8) {
    uint64_t w;
    __builtin_memcpy(&w, k + i, 8);
    h = mix64(h ^ w);
  }
  uint64_t t = 0;
  for (uint32_t j = 0; i + j < n; ++j) t |= (uint64_t)k[i + j] << (8 * j);
  return mix64(h ^ t ^ 0xA0761D6478BD642Full);
}
__host__ __device__ inline uint32_t key_owner(uint64_t h, uint32_t nparts) {
  return (uint32_t)(((h >> 32) * (uint64_t)nparts) >> 32);
}
constexpr uint32_t kMaxParts = 4096;

// The size of part o's block (8-B aligned) from its record count and key bytes.
__host__ __device__ inline uint64_t part_bytes(uint64_t nrec, uint64_t key_bytes, uint32_t nfiles) {
  return (sizeof(ShardHeader) + sizeof(ShardRec) * nrec + sizeof(ShardFileStat) * (uint64_t)nfiles + key_bytes + 7) &
         ~7ull;
}

}  // namespace cask_kd
