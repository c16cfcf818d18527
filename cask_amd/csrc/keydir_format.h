// The keydir block of one shard: what a rank of the multi-GPU replay sends to rank 0 (SURVEY.md
// §8e). Built on the device by cask_shard_keydir (k_keydir.hip), folded on the host by
// cask_keydir_merge (engine.cpp). Little-endian, 8-byte aligned:
//   ShardHeader | ShardRec[nrec] | ShardFileStat[nfiles] | key bytes of the records, in record order
// Records of one key appear in the shard's replay order (file id, pos).
#pragma once
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

static_assert(sizeof(ShardHeader) == 64 && sizeof(ShardRec) == 32 && sizeof(ShardFileStat) == 40, "layout");

}  // namespace cask_kd
