/*
 * cask_oracle.c — CPU restatement of Cask's replay hot path. TEST INFRASTRUCTURE ONLY
 * (see cask_oracle.h for who may call it). Not linked into the product.
 */
#define _GNU_SOURCE
#include "cask_oracle.h"

#include <errno.h>
#include <stdio.h>
#include <fcntl.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

/* ------------------------------------------------------------------------------------ */
/* XXH32: published algorithm (the arithmetic of twox-hash XxHash32, util.rs:10-41).      */
/* Streaming form mirrors Hasher::write + finish (util.rs:18-23): buffering of partial    */
/* stripes makes any split of the input give the one-shot digest (data.rs:102-108 vs :83). */
/* ------------------------------------------------------------------------------------ */
#define P1 2654435761u
#define P2 2246822519u
#define P3 3266489917u
#define P4 668265263u
#define P5 374761393u

static inline uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
static inline uint32_t rd32(const uint8_t* p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
static inline uint64_t rd64(const uint8_t* p) {
  return (uint64_t)rd32(p) | ((uint64_t)rd32(p + 4) << 32);
}
static inline uint16_t rd16(const uint8_t* p) { return (uint16_t)(p[0] | (p[1] << 8)); }
static inline void wr32(uint8_t* p, uint32_t v) {
  p[0] = (uint8_t)v; p[1] = (uint8_t)(v >> 8); p[2] = (uint8_t)(v >> 16); p[3] = (uint8_t)(v >> 24);
}
static inline void wr64(uint8_t* p, uint64_t v) { wr32(p, (uint32_t)v); wr32(p + 4, (uint32_t)(v >> 32)); }
static inline void wr16(uint8_t* p, uint16_t v) { p[0] = (uint8_t)v; p[1] = (uint8_t)(v >> 8); }

static inline uint32_t xround(uint32_t acc, uint32_t w) { return rotl32(acc + w * P2, 13) * P1; }

void orc_xxh32_reset(orc_xxh32_state* s, uint32_t seed) {
  memset(s, 0, sizeof(*s));
  s->seed = seed;
  s->v[0] = seed + P1 + P2;
  s->v[1] = seed + P2;
  s->v[2] = seed;
  s->v[3] = seed - P1;
}

void orc_xxh32_update(orc_xxh32_state* s, const uint8_t* p, size_t len) {
  s->total_len += len;
  if (s->memsize + len < 16) {
    memcpy(s->mem + s->memsize, p, len);
    s->memsize += (uint32_t)len;
    return;
  }
  if (s->memsize) {
    size_t fill = 16 - s->memsize;
    memcpy(s->mem + s->memsize, p, fill);
    s->v[0] = xround(s->v[0], rd32(s->mem));
    s->v[1] = xround(s->v[1], rd32(s->mem + 4));
    s->v[2] = xround(s->v[2], rd32(s->mem + 8));
    s->v[3] = xround(s->v[3], rd32(s->mem + 12));
    p += fill;
    len -= fill;
    s->memsize = 0;
  }
  while (len >= 16) {
    s->v[0] = xround(s->v[0], rd32(p));
    s->v[1] = xround(s->v[1], rd32(p + 4));
    s->v[2] = xround(s->v[2], rd32(p + 8));
    s->v[3] = xround(s->v[3], rd32(p + 12));
    p += 16;
    len -= 16;
  }
  if (len) {
    memcpy(s->mem, p, len);
    s->memsize = (uint32_t)len;
  }
}

uint32_t orc_xxh32_digest(const orc_xxh32_state* s) {
  uint32_t h;
  if (s->total_len >= 16)
    h = rotl32(s->v[0], 1) + rotl32(s->v[1], 7) + rotl32(s->v[2], 12) + rotl32(s->v[3], 18);
  else
    h = s->seed + P5;
  h += (uint32_t)s->total_len;
  const uint8_t* p = s->mem;
  uint32_t n = s->memsize;
  while (n >= 4) {
    h = rotl32(h + rd32(p) * P3, 17) * P4;
    p += 4;
    n -= 4;
  }
  while (n) {
    h = rotl32(h + (*p) * P5, 11) * P1;
    ++p;
    --n;
  }
  h ^= h >> 15;
  h *= P2;
  h ^= h >> 13;
  h *= P3;
  h ^= h >> 16;
  return h;
}

uint32_t orc_xxh32(const uint8_t* p, size_t len, uint32_t seed) {
  orc_xxh32_state s;
  orc_xxh32_reset(&s, seed);
  orc_xxh32_update(&s, p, len);
  return orc_xxh32_digest(&s);
}

/* ------------------------------------------------------------------------------------ */
/* Record codec                                                                           */
/* ------------------------------------------------------------------------------------ */

/* Entry::write_bytes (data.rs:90-121): header tail seq|ksz|vsz-or-tombstone at [4,18),
 * checksum = XXH32 streamed over header tail, key, value (data.rs:102-108), then key and
 * (unless deleted) value. */
size_t orc_entry_encode(uint64_t seq, const uint8_t* key, uint16_t ksz, const uint8_t* value,
                        uint32_t vsz, int deleted, uint8_t* out) {
  wr64(out + 4, seq);
  wr16(out + 12, ksz);
  wr32(out + 14, deleted ? ORC_ENTRY_TOMBSTONE : vsz);
  orc_xxh32_state s;
  orc_xxh32_reset(&s, 0);
  orc_xxh32_update(&s, out + 4, 14);
  orc_xxh32_update(&s, key, ksz);
  if (!deleted) orc_xxh32_update(&s, value, vsz);  /* a deleted Entry has an empty value */
  wr32(out, orc_xxh32_digest(&s));
  if (ksz) memcpy(out + 18, key, ksz);
  if (!deleted && vsz) memcpy(out + 18 + ksz, value, vsz);
  return 18 + (size_t)ksz + (deleted ? 0 : vsz);
}

/* Entries::next over a Take<File> of the whole file (log.rs:108-119, 403-429) with
 * Entry::from_read per record (data.rs:161-206):
 *   header read_exact(18) -> key read_exact(ksz) -> value read_exact(vsz) unless tombstone;
 *   any short read is Io(UnexpectedEof) and consumes the rest of the limit (iteration ends);
 *   otherwise all 18+ksz+vsz_eff bytes are consumed and XXH32 decides Ok vs InvalidChecksum.
 * Rows after a checksum error keep coming, as RecreateHints::drop drains them (log.rs:467-471). */
int64_t orc_scan_buffer(const uint8_t* buf, uint64_t len, orc_row* rows, uint64_t cap) {
  uint64_t pos = 0;
  int64_t n = 0;
  while (pos < len) {  /* Entries::next: limit == 0 -> None (log.rs:408-410) */
    if ((uint64_t)n >= cap) return -1;
    orc_row* r = &rows[n++];
    memset(r, 0, sizeof(*r));
    r->pos = pos;
    uint64_t rem = len - pos;
    if (rem < 18) {  /* data.rs:163 read_exact(header) */
      r->status = ORC_ROW_EOF;
      return n;
    }
    const uint8_t* h = buf + pos;
    r->expected = rd32(h);
    r->seq = rd64(h + 4);
    r->ksz = rd16(h + 12);
    r->vsz_raw = rd32(h + 14);
    uint64_t vsz_eff = (r->vsz_raw == ORC_ENTRY_TOMBSTONE) ? 0 : r->vsz_raw;
    uint64_t rec = 18 + (uint64_t)r->ksz + vsz_eff;
    if (rem < 18 + (uint64_t)r->ksz || rem < rec) { /* data.rs:172 / :181 */
      r->status = ORC_ROW_EOF;
      return n;
    }
    r->found = orc_xxh32(h + 4, rec - 4, 0); /* data.rs:185-191 (stream == one-shot) */
    r->status = (r->found == r->expected) ? ORC_ROW_OK : ORC_ROW_CHECKSUM; /* data.rs:193-198 */
    pos += rec;  /* log.rs:415-417; entry.size() == read (log.rs:421) */
  }
  return n;
}

/* Hint::write_bytes (data.rs:242-256). */
size_t orc_hint_encode(uint64_t seq, uint16_t ksz, uint32_t vsz_raw, uint64_t pos,
                       const uint8_t* key, uint8_t* out) {
  wr64(out, seq);
  wr16(out + 8, ksz);
  wr32(out + 10, vsz_raw == ORC_ENTRY_TOMBSTONE ? ORC_ENTRY_TOMBSTONE : vsz_raw);
  wr64(out + 14, pos);
  if (ksz) memcpy(out + 22, key, ksz);
  return 22 + (size_t)ksz;
}

/* ------------------------------------------------------------------------------------ */
/* Keydir: HashMap<Vec<u8>, IndexEntry> (cask.rs:28-31) + Stats (stats.rs:14-16)          */
/* ------------------------------------------------------------------------------------ */
typedef struct {
  uint8_t* key;  /* owned copy: hint.key.to_vec() (cask.rs:68) */
  uint64_t hash;
  uint64_t pos, size, seq;
  uint32_t file_id;
  uint16_t ksz;
  uint8_t used;  /* 0 empty, 1 live, 2 tombstone slot (removed) */
} orc_slot;

typedef struct {
  uint32_t file_id;
  uint64_t entries, dead_entries, dead_bytes;
  uint8_t used;
} orc_stat;

struct orc_index {
  orc_slot* slots;
  uint64_t cap, live, used_slots;
  orc_stat* stats;
  uint64_t stats_cap, stats_n;
};

static uint64_t key_hash(const uint8_t* k, uint16_t n) {
  uint64_t h = 1469598103934665603ull;
  for (uint16_t i = 0; i < n; ++i) {
    h ^= k[i];
    h *= 1099511628211ull;
  }
  return h ^ (h >> 29);
}

orc_index* orc_index_new(void) {
  orc_index* ix = (orc_index*)calloc(1, sizeof(orc_index));
  ix->cap = 1024;
  ix->slots = (orc_slot*)calloc(ix->cap, sizeof(orc_slot));
  ix->stats_cap = 64;
  ix->stats = (orc_stat*)calloc(ix->stats_cap, sizeof(orc_stat));
  return ix;
}

void orc_index_free(orc_index* ix) {
  if (!ix) return;
  for (uint64_t i = 0; i < ix->cap; ++i)
    if (ix->slots[i].used == 1) free(ix->slots[i].key);
  free(ix->slots);
  free(ix->stats);
  free(ix);
}

static orc_stat* stat_find(orc_index* ix, uint32_t file_id, int create) {
  uint64_t m = ix->stats_cap - 1;
  uint64_t i = (file_id * 2654435761u) & m;
  for (;;) {
    orc_stat* s = &ix->stats[i];
    if (!s->used) {
      if (!create) return NULL;
      if ((ix->stats_n + 1) * 2 > ix->stats_cap) {
        orc_stat* old = ix->stats;
        uint64_t oc = ix->stats_cap;
        ix->stats_cap *= 2;
        ix->stats = (orc_stat*)calloc(ix->stats_cap, sizeof(orc_stat));
        ix->stats_n = 0;
        for (uint64_t j = 0; j < oc; ++j)
          if (old[j].used) {
            orc_stat* d = stat_find(ix, old[j].file_id, 1);
            *d = old[j];
          }
        free(old);
        return stat_find(ix, file_id, 1);
      }
      s->used = 1;
      s->file_id = file_id;
      ix->stats_n++;
      return s;
    }
    if (s->file_id == file_id) return s;
    i = (i + 1) & m;
  }
}

/* Stats::add_entry (stats.rs:23-36) */
static void stats_add(orc_index* ix, uint32_t file_id) {
  orc_stat* s = stat_find(ix, file_id, 0);
  if (s) {
    s->entries += 1;
  } else {
    s = stat_find(ix, file_id, 1);
    s->entries = 1;
    s->dead_entries = 0;
    s->dead_bytes = 0;
  }
}

/* Stats::remove_entry (stats.rs:38-48): a missing row only warns. */
static void stats_remove(orc_index* ix, uint32_t file_id, uint64_t size) {
  orc_stat* s = stat_find(ix, file_id, 0);
  if (s) {
    s->dead_entries += 1;
    s->dead_bytes += size;
  }
}

static void index_grow(orc_index* ix) {
  orc_slot* old = ix->slots;
  uint64_t oc = ix->cap;
  ix->cap *= 2;
  ix->slots = (orc_slot*)calloc(ix->cap, sizeof(orc_slot));
  ix->used_slots = 0;
  uint64_t m = ix->cap - 1;
  for (uint64_t i = 0; i < oc; ++i) {
    if (old[i].used != 1) continue;
    uint64_t j = old[i].hash & m;
    while (ix->slots[j].used) j = (j + 1) & m;
    ix->slots[j] = old[i];
    ix->used_slots++;
  }
  free(old);
}

/* Index::update (cask.rs:60-90). */
void orc_index_update(orc_index* ix, const uint8_t* key, uint16_t ksz, uint32_t file_id,
                      uint64_t pos, uint32_t vsz_raw, uint64_t seq) {
  int deleted = (vsz_raw == ORC_ENTRY_TOMBSTONE);
  /* Hint.value_size is 0 for a tombstone (data.rs:222/232, :272); entry_size :238-240 */
  uint64_t size = 18 + (uint64_t)ksz + (deleted ? 0 : vsz_raw);
  if ((ix->used_slots + 1) * 4 > ix->cap * 3) index_grow(ix);
  uint64_t h = key_hash(key, ksz);
  uint64_t m = ix->cap - 1;
  uint64_t i = h & m;
  int64_t tomb = -1;
  for (;;) {
    orc_slot* s = &ix->slots[i];
    if (s->used == 0) break;
    if (s->used == 2) {
      if (tomb < 0) tomb = (int64_t)i;
    } else if (s->hash == h && s->ksz == ksz && memcmp(s->key, key, ksz) == 0) {
      /* HashMapEntry::Occupied (cask.rs:69-82) */
      if (s->seq <= seq) {
        stats_remove(ix, s->file_id, s->size);
        if (deleted) {
          free(s->key);
          s->key = NULL;
          s->used = 2;
          ix->live--;
        } else {
          stats_add(ix, file_id);
          s->file_id = file_id;
          s->pos = pos;
          s->size = size;
          s->seq = seq;
        }
      } else {
        stats_add(ix, file_id);
        stats_remove(ix, file_id, size);
      }
      return;
    }
    i = (i + 1) & m;
  }
  /* HashMapEntry::Vacant (cask.rs:83-88) */
  if (deleted) return;
  stats_add(ix, file_id);
  orc_slot* s = (tomb >= 0) ? &ix->slots[tomb] : &ix->slots[i];
  if (tomb < 0) ix->used_slots++;
  s->key = (uint8_t*)malloc(ksz ? ksz : 1);
  if (ksz) memcpy(s->key, key, ksz);
  s->ksz = ksz;
  s->hash = h;
  s->file_id = file_id;
  s->pos = pos;
  s->size = size;
  s->seq = seq;
  s->used = 1;
  ix->live++;
}

uint64_t orc_index_len(const orc_index* ix) { return ix->live; }

static int cmp_key(const uint8_t* a, uint16_t an, const uint8_t* b, uint16_t bn) {
  uint16_t n = an < bn ? an : bn;
  int c = n ? memcmp(a, b, n) : 0;
  if (c) return c;
  return (int)an - (int)bn;
}

static const orc_index* g_sort_ix;
static int cmp_slot_idx(const void* x, const void* y) {
  const orc_slot* a = &g_sort_ix->slots[*(const uint64_t*)x];
  const orc_slot* b = &g_sort_ix->slots[*(const uint64_t*)y];
  return cmp_key(a->key, a->ksz, b->key, b->ksz);
}

void orc_index_export(const orc_index* ix, uint8_t* keys_out, uint64_t* key_off,
                      uint16_t* key_len, uint32_t* file_id, uint64_t* pos, uint64_t* size,
                      uint64_t* seq) {
  uint64_t* idx = (uint64_t*)malloc((ix->live + 1) * sizeof(uint64_t));
  uint64_t n = 0;
  for (uint64_t i = 0; i < ix->cap; ++i)
    if (ix->slots[i].used == 1) idx[n++] = i;
  g_sort_ix = ix;
  qsort(idx, n, sizeof(uint64_t), cmp_slot_idx);
  uint64_t off = 0;
  for (uint64_t j = 0; j < n; ++j) {
    const orc_slot* s = &ix->slots[idx[j]];
    if (keys_out) memcpy(keys_out + off, s->key, s->ksz);
    if (key_off) key_off[j] = off;
    if (key_len) key_len[j] = s->ksz;
    if (file_id) file_id[j] = s->file_id;
    if (pos) pos[j] = s->pos;
    if (size) size[j] = s->size;
    if (seq) seq[j] = s->seq;
    off += s->ksz;
  }
  free(idx);
}

static int cmp_stat(const void* x, const void* y) {
  uint32_t a = ((const orc_stat*)x)->file_id, b = ((const orc_stat*)y)->file_id;
  return a < b ? -1 : a > b;
}

uint64_t orc_index_stats(const orc_index* ix, uint32_t* file_id, uint64_t* entries,
                         uint64_t* dead_entries, uint64_t* dead_bytes, uint64_t cap) {
  orc_stat* tmp = (orc_stat*)malloc((ix->stats_n + 1) * sizeof(orc_stat));
  uint64_t n = 0;
  for (uint64_t i = 0; i < ix->stats_cap; ++i)
    if (ix->stats[i].used) tmp[n++] = ix->stats[i];
  qsort(tmp, n, sizeof(orc_stat), cmp_stat);
  uint64_t m = n < cap ? n : cap;
  for (uint64_t j = 0; j < m; ++j) {
    file_id[j] = tmp[j].file_id;
    entries[j] = tmp[j].entries;
    dead_entries[j] = tmp[j].dead_entries;
    dead_bytes[j] = tmp[j].dead_bytes;
  }
  free(tmp);
  return n;
}

/* ------------------------------------------------------------------------------------ */
/* Replay drivers                                                                         */
/* ------------------------------------------------------------------------------------ */

/* std::io::Read::read_exact over an unbuffered File: read(2) until filled or EOF. */
static int read_exact_fd(int fd, uint8_t* p, uint64_t n, uint64_t* limit) {
  /* Take<File> caps reads at the file size measured at open (log.rs:112-115). */
  uint64_t want = n;
  int short_read = 0;
  if (want > *limit) {
    want = *limit;
    short_read = 1;
  }
  uint64_t got = 0;
  while (got < want) {
    ssize_t r = read(fd, p + got, (size_t)(want - got));
    if (r < 0) {
      if (errno == EINTR) continue;
      return -1;
    }
    if (r == 0) {
      short_read = 1;
      break;
    }
    got += (uint64_t)r;
  }
  *limit -= got;
  return short_read ? 1 : 0;
}

static int write_all_fd(int fd, const uint8_t* p, size_t n) {
  while (n) {
    ssize_t w = write(fd, p, n);
    if (w < 0) {
      if (errno == EINTR) continue;
      return -1;
    }
    p += w;
    n -= (size_t)w;
  }
  return 0;
}

int orc_replay_file_faithful(const char* data_path, const char* hint_path, uint32_t file_id,
                             orc_index* ix, orc_replay_result* res) {
  memset(res, 0, sizeof(*res));
  int fd = open(data_path, O_RDONLY);
  if (fd < 0) return -1;
  off_t fsz = lseek(fd, 0, SEEK_END);
  lseek(fd, 0, SEEK_SET);
  uint64_t limit = (uint64_t)fsz;
  /* HintWriter::new: create + truncate (log.rs:373-380, util.rs:45-49) */
  int hfd = hint_path ? open(hint_path, O_WRONLY | O_CREAT | O_TRUNC, 0644) : -1;
  orc_xxh32_state hint_hasher;
  orc_xxh32_reset(&hint_hasher, 0);
  uint64_t pos = 0;
  int draining = 0;  /* after the first InvalidChecksum: RecreateHints::drop's drain */
  while (limit > 0) {
    uint64_t before = limit;
    /* Entry::from_read (data.rs:161-206): three Vec allocations per record */
    uint8_t* header = (uint8_t*)calloc(18, 1);
    int eof = read_exact_fd(fd, header, 18, &limit);
    uint8_t* key = NULL;
    uint8_t* value = NULL;
    uint16_t ksz = 0;
    uint32_t vsz_raw = 0;
    int deleted = 0;
    if (eof == 0) {
      ksz = rd16(header + 12);
      vsz_raw = rd32(header + 14);
      key = (uint8_t*)calloc(ksz ? ksz : 1, 1);
      eof = read_exact_fd(fd, key, ksz, &limit);
      deleted = (vsz_raw == ORC_ENTRY_TOMBSTONE);
      if (eof == 0 && !deleted) {
        value = (uint8_t*)calloc(vsz_raw ? vsz_raw : 1, 1);
        eof = read_exact_fd(fd, value, vsz_raw, &limit);
      }
    }
    if (eof != 0) {
      if (!res->err_kind) {
        res->err_kind = eof < 0 ? -1 : ORC_ROW_EOF;
        res->err_file_id = file_id;
        res->err_pos = pos;
      }
      free(header); free(key); free(value);
      break;  /* the Take limit is exhausted: Entries::next yields None next */
    }
    orc_xxh32_state hs;
    orc_xxh32_reset(&hs, 0);
    orc_xxh32_update(&hs, header + 4, 14);
    orc_xxh32_update(&hs, key, ksz);
    if (!deleted) orc_xxh32_update(&hs, value, vsz_raw);
    uint32_t hash = orc_xxh32_digest(&hs);
    uint32_t stored = rd32(header);
    uint64_t read_bytes = before - limit;
    res->bytes += read_bytes;
    if (hash != stored) {
      /* InvalidChecksum aborts open() at the `?` (cask.rs:365): no more folding. RecreateHints::drop
       * (log.rs:466-470) then drains the iterator: later Ok records still get their hints. */
      if (!res->err_kind) {
        res->err_kind = ORC_ROW_CHECKSUM;
        res->err_file_id = file_id;
        res->err_pos = pos;
        res->err_expected = stored;
        res->err_found = hash;
      }
      draining = 1;
    } else {
      uint64_t seq = rd64(header + 4);
      /* HintWriter::write: Hint::write_bytes into the file (5 write(2)) and the hasher. */
      if (hfd >= 0) {
        uint8_t b8[8], b2[2], b4[4];
        wr64(b8, seq);
        write_all_fd(hfd, b8, 8);
        orc_xxh32_update(&hint_hasher, b8, 8);
        wr16(b2, ksz);
        write_all_fd(hfd, b2, 2);
        orc_xxh32_update(&hint_hasher, b2, 2);
        wr32(b4, deleted ? ORC_ENTRY_TOMBSTONE : vsz_raw);
        write_all_fd(hfd, b4, 4);
        orc_xxh32_update(&hint_hasher, b4, 4);
        wr64(b8, pos);
        write_all_fd(hfd, b8, 8);
        orc_xxh32_update(&hint_hasher, b8, 8);
        write_all_fd(hfd, key, ksz);
        orc_xxh32_update(&hint_hasher, key, ksz);
      }
      /* Cask::open closure (cask.rs:349-355), until the first error */
      if (!draining) {
        if (seq > res->max_seq) res->max_seq = seq;
        orc_index_update(ix, key, ksz, file_id, pos, deleted ? ORC_ENTRY_TOMBSTONE : vsz_raw, seq);
        res->records++;
      }
    }
    pos += read_bytes;
    free(header); free(key); free(value);
  }
  if (hfd >= 0) {
    uint8_t b4[4];
    wr32(b4, orc_xxh32_digest(&hint_hasher));  /* HintWriter::drop (log.rs:389-395) */
    write_all_fd(hfd, b4, 4);
    close(hfd);
  }
  close(fd);
  res->live_keys = orc_index_len(ix);
  return 0;
}

int orc_replay_buffer_fast(const uint8_t* buf, uint64_t len, uint32_t file_id, orc_index* ix,
                           orc_replay_result* res) {
  memset(res, 0, sizeof(*res));
  uint64_t pos = 0;
  while (pos < len) {
    uint64_t rem = len - pos;
    if (rem < 18) {
      res->err_kind = ORC_ROW_EOF; res->err_file_id = file_id; res->err_pos = pos;
      break;
    }
    const uint8_t* h = buf + pos;
    uint16_t ksz = rd16(h + 12);
    uint32_t vsz_raw = rd32(h + 14);
    uint64_t rec = 18 + (uint64_t)ksz + (vsz_raw == ORC_ENTRY_TOMBSTONE ? 0 : vsz_raw);
    if (rem < rec) {
      res->err_kind = ORC_ROW_EOF; res->err_file_id = file_id; res->err_pos = pos;
      break;
    }
    uint32_t hash = orc_xxh32(h + 4, rec - 4, 0);
    if (hash != rd32(h)) {
      res->err_kind = ORC_ROW_CHECKSUM; res->err_file_id = file_id; res->err_pos = pos;
      res->err_expected = rd32(h); res->err_found = hash;
      break;
    }
    uint64_t seq = rd64(h + 4);
    if (seq > res->max_seq) res->max_seq = seq;
    orc_index_update(ix, h + 18, ksz, file_id, pos, vsz_raw, seq);
    res->records++;
    res->bytes += rec;
    pos += rec;
  }
  res->live_keys = orc_index_len(ix);
  return 0;
}

/* ------------------------------------------------------------------------------------ */
/* Index lookup (Index::get, cask.rs:41-43)                                               */
/* ------------------------------------------------------------------------------------ */
int orc_index_get(const orc_index* ix, const uint8_t* key, uint16_t ksz, uint32_t* file_id, uint64_t* pos,
                  uint64_t* size, uint64_t* seq) {
  uint64_t h = key_hash(key, ksz);
  uint64_t m = ix->cap - 1;
  for (uint64_t i = h & m;; i = (i + 1) & m) {
    const orc_slot* s = &ix->slots[i];
    if (s->used == 0) return 0;
    if (s->used == 1 && s->hash == h && s->ksz == ksz && (ksz == 0 || memcmp(s->key, key, ksz) == 0)) {
      if (file_id) *file_id = s->file_id;
      if (pos) *pos = s->pos;
      if (size) *size = s->size;
      if (seq) *seq = s->seq;
      return 1;
    }
  }
}

/* ------------------------------------------------------------------------------------ */
/* Compaction merge: Cask::compact_files_aux (cask.rs:451-523), fast restatement          */
/* ------------------------------------------------------------------------------------ */
static int read_whole(const char* path, uint8_t** out, uint64_t* len) {
  int fd = open(path, O_RDONLY);
  if (fd < 0) return -1;
  off_t n = lseek(fd, 0, SEEK_END);
  lseek(fd, 0, SEEK_SET);
  uint8_t* b = (uint8_t*)malloc(n > 0 ? (size_t)n : 1);
  uint64_t got = 0;
  while (got < (uint64_t)n) {
    ssize_t r = read(fd, b + got, (size_t)((uint64_t)n - got));
    if (r < 0 && errno == EINTR) continue;
    if (r <= 0) break;
    got += (uint64_t)r;
  }
  close(fd);
  *out = b;
  *len = got;
  return 0;
}

static void file_name(char* out, size_t cap, const char* dir, uint32_t id, const char* ext) {
  /* get_data_file_path / hint path: "{:010}.cask.data" (log.rs:473-481) */
  snprintf(out, cap, "%s/%010u.cask.%s", dir, id, ext);
}

/* LogWriter (log.rs:245-306) + EntryWriter (:317-358) + HintWriter (:360-395), buffered in memory
 * and flushed when the writer moves on (the files are the same bytes the reference writes). */
typedef struct {
  const char* dir;
  uint64_t max_file_size;
  uint32_t seq;       /* Sequence (util.rs:55-65): the last id handed out */
  int open;
  uint32_t fid;
  uint8_t* data;
  uint64_t dlen, dcap;
  uint8_t* hint;
  uint64_t hlen, hcap;
  int io_err;
} orc_writer;

static void grow_buf(uint8_t** b, uint64_t* cap, uint64_t need) {
  if (need <= *cap) return;
  uint64_t c = *cap ? *cap : 1 << 16;
  while (c < need) c *= 2;
  *b = (uint8_t*)realloc(*b, c);
  *cap = c;
}

static int write_file(const char* path, const uint8_t* p, uint64_t n, const uint8_t* tail, size_t tn) {
  int fd = open(path, O_WRONLY | O_CREAT | O_TRUNC, 0644);
  if (fd < 0) return -1;
  int rc = write_all_fd(fd, p, (size_t)n);
  if (rc == 0 && tn) rc = write_all_fd(fd, tail, tn);
  close(fd);
  return rc;
}

static void writer_flush(orc_writer* w) {
  if (!w->open) return;
  char path[4096];
  file_name(path, sizeof path, w->dir, w->fid, "data");
  if (write_file(path, w->data, w->dlen, NULL, 0)) w->io_err = 1;
  uint8_t tr[4];
  wr32(tr, orc_xxh32(w->hint, w->hlen, 0)); /* HintWriter::drop: the trailer (log.rs:389-395) */
  file_name(path, sizeof path, w->dir, w->fid, "hint");
  if (write_file(path, w->hint, w->hlen, tr, 4)) w->io_err = 1;
  w->open = 0;
  w->dlen = w->hlen = 0;
}

/* LogWriter::write: a new file when there is none or data_file_pos + entry.size() > max_file_size
 * (log.rs:282-306); returns 1 if this entry started a file (LogWrite::NewFile). */
static int writer_write(orc_writer* w, uint64_t seq, const uint8_t* key, uint16_t ksz, const uint8_t* value,
                        uint32_t vsz, int deleted) {
  uint64_t size = 18 + (uint64_t)ksz + (deleted ? 0 : vsz); /* Entry::size (data.rs:63-65) */
  int nf = 0;
  if (!w->open || w->dlen + size > w->max_file_size) {
    writer_flush(w);
    w->fid = ++w->seq; /* Sequence::increment (util.rs:62-64) */
    w->open = 1;
    nf = 1;
  }
  uint64_t pos = w->dlen;
  grow_buf(&w->data, &w->dcap, w->dlen + size);
  orc_entry_encode(seq, key, ksz, value, vsz, deleted, w->data + w->dlen); /* Entry::write_bytes */
  w->dlen += size;
  grow_buf(&w->hint, &w->hcap, w->hlen + 22 + ksz);
  /* Hint::new(entry, entry_pos) + Hint::write_bytes (data.rs:218-226, 242-256) */
  w->hlen += orc_hint_encode(seq, ksz, deleted ? ORC_ENTRY_TOMBSTONE : vsz, pos, key, w->hint + w->hlen);
  return nf;
}

/* deletes: HashMap<Vec<u8>, u64> (cask.rs:471, 487-499), kept in first-seen order (the reference
 * iterates its RandomState HashMap: the order of its tombstone writes is unspecified) */
typedef struct {
  uint8_t* key;
  uint64_t hash, seq;
  uint16_t ksz;
  uint8_t used;
} del_slot;
typedef struct {
  del_slot* slots;
  uint64_t cap, n;
  uint64_t* order; /* slot indices in first-seen order */
  uint64_t ocap;
} del_map;

static void del_put(del_map* d, const uint8_t* key, uint16_t ksz, uint64_t seq) {
  if ((d->n + 1) * 2 > d->cap) {
    del_slot* old = d->slots;
    uint64_t oc = d->cap;
    d->cap = oc ? oc * 2 : 1024;
    d->slots = (del_slot*)calloc(d->cap, sizeof(del_slot));
    for (uint64_t k = 0; k < d->n; ++k) { /* re-insert in first-seen order, indices rebuilt */
      del_slot s = old[d->order[k]];
      uint64_t j = s.hash & (d->cap - 1);
      while (d->slots[j].used) j = (j + 1) & (d->cap - 1);
      d->slots[j] = s;
      d->order[k] = j;
    }
    free(old);
  }
  uint64_t h = key_hash(key, ksz);
  uint64_t m = d->cap - 1;
  uint64_t i = h & m;
  for (;; i = (i + 1) & m) {
    del_slot* s = &d->slots[i];
    if (!s->used) break;
    if (s->hash == h && s->ksz == ksz && (ksz == 0 || memcmp(s->key, key, ksz) == 0)) {
      if (s->seq < seq) s->seq = seq; /* Occupied: keep the higher sequence (cask.rs:490-494) */
      return;
    }
  }
  del_slot* s = &d->slots[i];
  s->used = 1;
  s->hash = h;
  s->ksz = ksz;
  s->seq = seq;
  s->key = (uint8_t*)malloc(ksz ? ksz : 1);
  if (ksz) memcpy(s->key, key, ksz);
  if (d->n == d->ocap) {
    d->ocap = d->ocap ? d->ocap * 2 : 1024;
    d->order = (uint64_t*)realloc(d->order, d->ocap * sizeof(uint64_t));
  }
  d->order[d->n++] = i;
}

static void set_cerr(orc_compact_result* r, int kind, uint32_t fid, uint64_t pos, uint32_t e, uint32_t f) {
  r->err_kind = kind;
  r->err_file_id = fid;
  r->err_pos = pos;
  r->err_expected = e;
  r->err_found = f;
}

static int index_seq_of(const void* ix, const uint8_t* key, uint16_t ksz, uint64_t* seq) {
  return orc_index_get((const orc_index*)ix, key, ksz, NULL, NULL, NULL, seq);
}

int orc_compact_files(const char* src_dir, const char* dst_dir, const orc_index* ix, const uint32_t* files,
                      uint64_t nfiles, uint32_t file_id_seq, uint64_t max_file_size, uint32_t* out_ids,
                      uint8_t* out_live, uint64_t cap, orc_compact_result* res) {
  return orc_compact_files_fn(src_dir, dst_dir, index_seq_of, ix, files, nfiles, file_id_seq, max_file_size, out_ids,
                              out_live, cap, res);
}

int orc_compact_files_fn(const char* src_dir, const char* dst_dir, orc_seq_fn seq_of, const void* ix,
                         const uint32_t* files, uint64_t nfiles, uint32_t file_id_seq, uint64_t max_file_size,
                         uint32_t* out_ids, uint8_t* out_live, uint64_t cap, orc_compact_result* res) {
  memset(res, 0, sizeof(*res));
  orc_writer w;
  memset(&w, 0, sizeof w);
  w.dir = dst_dir;
  w.max_file_size = max_file_size;
  w.seq = file_id_seq;
  del_map dels;
  memset(&dels, 0, sizeof dels);
  uint64_t nout = 0;
  int rc = 0;
  char path[4096];
  for (uint64_t fi = 0; fi < nfiles && !rc; ++fi) {
    const uint32_t fid = files[fi];
    /* Log::hints (log.rs:121-135): a missing or invalid hint file skips the file (cask.rs:456-468) */
    file_name(path, sizeof path, src_dir, fid, "hint");
    uint8_t* hb = NULL;
    uint64_t hn = 0;
    if (read_whole(path, &hb, &hn) != 0) continue;
    if (hn < 4 || orc_xxh32(hb, hn - 4, 0) != rd32(hb + hn - 4)) { /* is_valid_hint_file (log.rs:512-539) */
      free(hb);
      continue;
    }
    const uint64_t body = hn - 4;
    /* the data file, for Log::read_entry (log.rs:150-166) of its live entries */
    file_name(path, sizeof path, src_dir, fid, "data");
    uint8_t* db = NULL;
    uint64_t dn = 0;
    if (read_whole(path, &db, &dn) != 0) {
      free(hb);
      set_cerr(res, -1, fid, 0, 0, 0);
      rc = -1;
      break;
    }
    /* pass 1 (cask.rs:481-503): liveness of every hint, tombstones of absent keys */
    uint64_t* ins = NULL;
    uint64_t nins = 0, icap = 0;
    for (uint64_t p = 0; p < body;) {
      /* Hint::from_read (data.rs:258-276): seq u64 | ksz u16 | vsz u32 | pos u64 | key */
      if (body - p < 22) {
        set_cerr(res, ORC_ROW_EOF, fid, p, 0, 0);
        rc = -1;
        break;
      }
      const uint8_t* h = hb + p;
      const uint64_t seq = rd64(h);
      const uint16_t ksz = rd16(h + 8);
      const uint32_t vsz = rd32(h + 10);
      if (body - p - 22 < ksz) {
        set_cerr(res, ORC_ROW_EOF, fid, p, 0, 0);
        rc = -1;
        break;
      }
      const uint8_t* key = h + 22;
      uint64_t iseq = 0;
      const int present = seq_of(ix, key, ksz, &iseq);
      if (vsz == ORC_ENTRY_TOMBSTONE) {
        if (!present) del_put(&dels, key, ksz, seq);
      } else if (present && iseq == seq) { /* live iff the index holds this sequence (cask.rs:500) */
        if (nins == icap) {
          icap = icap ? icap * 2 : 1024;
          ins = (uint64_t*)realloc(ins, icap * sizeof(uint64_t));
        }
        ins[nins++] = p;
      }
      p += 22 + (uint64_t)ksz;
    }
    /* pass 2 (cask.rs:505-513): read_entry + LogWriter::write of each live entry, in hint order */
    for (uint64_t k = 0; k < nins && !rc; ++k) {
      const uint8_t* h = hb + ins[k];
      const uint64_t pos = rd64(h + 14);
      /* Entry::from_read at pos (data.rs:161-206) */
      if (pos > dn || dn - pos < 18) {
        set_cerr(res, ORC_ROW_EOF, fid, pos, 0, 0);
        rc = -1;
        break;
      }
      const uint8_t* e = db + pos;
      const uint16_t ksz = rd16(e + 12);
      const uint32_t vraw = rd32(e + 14);
      const int del = vraw == ORC_ENTRY_TOMBSTONE;
      const uint64_t rl = 18 + (uint64_t)ksz + (del ? 0 : vraw);
      if (dn - pos < rl) {
        set_cerr(res, ORC_ROW_EOF, fid, pos, 0, 0);
        rc = -1;
        break;
      }
      const uint32_t found = orc_xxh32(e + 4, rl - 4, 0);
      if (found != rd32(e)) {
        set_cerr(res, ORC_ROW_CHECKSUM, fid, pos, rd32(e), found);
        rc = -1;
        break;
      }
      const int nf = writer_write(&w, rd64(e + 4), e + 18, ksz, e + 18 + ksz, del ? 0 : vraw, del);
      if (nf) { /* LogWrite::NewFile -> new_files (cask.rs:510-512) */
        if (nout < cap) {
          out_ids[nout] = w.fid;
          out_live[nout] = 1;
        }
        ++nout;
        res->n_new++;
      }
      res->live_records++;
      res->bytes_out += rl;
    }
    free(ins);
    free(db);
    free(hb);
    if (!rc) res->n_compacted++;
  }
  /* the tombstone tail (cask.rs:518-520): files it starts are not in new_files */
  for (uint64_t k = 0; k < dels.n && !rc; ++k) {
    const del_slot* s = &dels.slots[dels.order[k]];
    if (writer_write(&w, s->seq, s->key, s->ksz, NULL, 0, 1)) {
      if (nout < cap) {
        out_ids[nout] = w.fid;
        out_live[nout] = 0;
      }
      ++nout;
      res->n_tomb_only++;
    }
    res->tombstones++;
    res->bytes_out += 18 + (uint64_t)s->ksz;
  }
  writer_flush(&w); /* the writers' Drop (log.rs:360-395) */
  if (w.io_err && !rc) {
    set_cerr(res, -1, 0, 0, 0, 0);
    rc = -1;
  }
  for (uint64_t i = 0; i < dels.cap; ++i)
    if (dels.slots && dels.slots[i].used) free(dels.slots[i].key);
  free(dels.slots);
  free(dels.order);
  free(w.data);
  free(w.hint);
  res->n_out = nout;
  res->file_id_seq = w.seq;
  return rc;
}

uint64_t orc_index_digest(const orc_index* ix) {
  uint64_t d = 0;
  for (uint64_t i = 0; i < ix->cap; ++i) {
    const orc_slot* s = &ix->slots[i];
    if (s->used == 1) d += orc_entry_digest(s->key, s->ksz, s->file_id, s->pos, s->size, s->seq);
  }
  return d;
}

/* RecreateHints over a data file in memory (log.rs:137-148, 449-471; Hint::write_bytes, data.rs:242-256):
 * one hint per Ok record in order, records after a checksum failure included (the drain of
 * RecreateHints::drop), none after an EOF. Returns the body length (the trailer is not written), or
 * -1 when cap is too small. */
int64_t orc_hint_body(const uint8_t* buf, uint64_t len, uint8_t* out, uint64_t cap) {
  uint64_t pos = 0, n = 0;
  while (pos < len) {
    if (len - pos < 18) break;
    const uint8_t* h = buf + pos;
    const uint16_t ksz = rd16(h + 12);
    const uint32_t vsz = rd32(h + 14);
    const uint64_t rl = 18 + (uint64_t)ksz + (vsz == ORC_ENTRY_TOMBSTONE ? 0 : vsz);
    if (len - pos < rl) break;
    if (orc_xxh32(h + 4, rl - 4, 0) == rd32(h)) {
      if (n + 22 + ksz > cap) return -1;
      n += orc_hint_encode(rd64(h + 4), ksz, vsz, pos, h + 18, out + n);
    }
    pos += rl;
  }
  return (int64_t)n;
}
