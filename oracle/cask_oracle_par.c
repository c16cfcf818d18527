/*
 * cask_oracle_par.c — Cask::open over many in-memory data files on host threads, for the large
 * BASELINE configs. TEST INFRASTRUCTURE ONLY (see cask_oracle.h).
 *
 * Index::update touches one key's entry and per-file counters (cask.rs:60-90, stats.rs:23-48), and
 * a Stats::remove_entry always follows an add of the same file in the same key's history (the
 * occupant's own add, or the add just before a stale record's remove), so the fold splits exactly
 * by key: each partition of the key space folds its keys in replay order (file, pos) into its own
 * index (orc_index_update, the restatement of cask.rs:60-90), and the per-file counters of the
 * partitions add up. The scan is Entries::next + Entry::from_read (log.rs:403-429,
 * data.rs:161-206) in two passes: each file's chain of record lengths from the headers (files on
 * threads), then every record's checksum with the records split over the threads by byte range (so
 * a sample of a few large files still uses every thread); a file's first failure is its first
 * failing checksum before the chain's cut-short record, else that record, and the first failure in
 * replay order ends the replay (cask.rs:360,365).
 */
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#include "cask_oracle.h"

static inline uint16_t rd16(const uint8_t* p) { return (uint16_t)(p[0] | (p[1] << 8)); }
static inline uint32_t rd32(const uint8_t* p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
static inline uint64_t rd64(const uint8_t* p) { return (uint64_t)rd32(p) | ((uint64_t)rd32(p + 4) << 32); }

static uint64_t mix64(uint64_t x) {
  x ^= x >> 30;
  x *= 0xBF58476D1CE4E5B9ull;
  x ^= x >> 27;
  x *= 0x94D049BB133111EBull;
  x ^= x >> 31;
  return x;
}

uint64_t orc_entry_digest(const uint8_t* key, uint16_t ksz, uint32_t file_id, uint64_t pos, uint64_t size,
                          uint64_t seq) {
  uint64_t h = mix64(0x9E3779B97F4A7C15ull ^ ksz);
  for (uint32_t i = 0; i < ksz; i += 8) {
    uint64_t w = 0;
    for (uint32_t k = 0; k < 8 && i + k < ksz; ++k) w |= (uint64_t)key[i + k] << (8 * k);
    h = mix64(h ^ w);
  }
  h = mix64(h ^ file_id);
  h = mix64(h ^ pos);
  h = mix64(h ^ size);
  return mix64(h ^ seq);
}

static uint64_t part_hash(const uint8_t* k, uint16_t n) { /* FNV-1a: which partition folds the key */
  uint64_t h = 1469598103934665603ull;
  for (uint16_t i = 0; i < n; ++i) {
    h ^= k[i];
    h *= 1099511628211ull;
  }
  return mix64(h);
}

typedef struct {
  uint64_t pos, seq;
  uint32_t vsz;
  uint16_t ksz;
  uint8_t part;
  uint8_t pad;
} prow;

typedef struct {
  const uint8_t* const* bufs;
  const uint64_t* lens;
  const uint32_t* fids;
  uint32_t nfiles, nparts, nthreads;
  uint64_t** offs;  /* per file: the record chain's offsets, up to its first cut-short record */
  prow** rows;      /* per file: its Ok rows before its first failure */
  uint64_t* nrows;
  uint64_t* fbad;   /* per file: the index of its first record whose checksum fails (UINT64_MAX none) */
  uint64_t* fbyte;  /* prefix of the file lengths: the byte ranges the verify threads split */
  int32_t* ferr;    /* per file: the first failure's kind (0 none), pos, expected, found */
  uint64_t* fpos;
  uint32_t *fexp, *ffound;
  uint32_t stop;    /* files folded: through the first failing one */
  orc_index** ix;   /* per partition */
  uint64_t* pmax;   /* per partition: max sequence */
  uint64_t* pdig;   /* per partition: digest */
  uint32_t next;    /* work counter of the chain walk */
  pthread_mutex_t mu;
} pjob;

static uint32_t take(pjob* j) {
  pthread_mutex_lock(&j->mu);
  const uint32_t v = j->next++;
  pthread_mutex_unlock(&j->mu);
  return v;
}

/* 1. Entries::next per file (log.rs:403-429): the chain of record lengths from the headers alone,
 * to the first record cut short by the file's end (Io(UnexpectedEof), data.rs:163,172,181: a
 * record's reads fail before its checksum is computed). Files on threads. */
static void* walk_worker(void* arg) {
  pjob* j = (pjob*)arg;
  for (uint32_t f; (f = take(j)) < j->nfiles;) {
    const uint8_t* b = j->bufs[f];
    const uint64_t len = j->lens[f];
    uint64_t* o = (uint64_t*)malloc((len / 18 + 1) * sizeof(uint64_t));
    uint64_t n = 0, pos = 0;
    while (pos < len) {
      if (len - pos < 18) { /* header cut short */
        j->ferr[f] = ORC_ROW_EOF;
        j->fpos[f] = pos;
        break;
      }
      const uint8_t* h = b + pos;
      const uint32_t vsz = rd32(h + 14);
      const uint64_t rl = 18 + (uint64_t)rd16(h + 12) + (vsz == ORC_ENTRY_TOMBSTONE ? 0 : vsz);
      if (len - pos < rl) { /* key or value cut short */
        j->ferr[f] = ORC_ROW_EOF;
        j->fpos[f] = pos;
        break;
      }
      o[n++] = pos;
      pos += rl;
    }
    j->offs[f] = o;
    j->nrows[f] = n;
    j->rows[f] = (prow*)malloc((n + 1) * sizeof(prow));
  }
  return NULL;
}

typedef struct {
  pjob* j;
  uint32_t t;
} pverify;

/* 2. Entry::from_read's checksum (data.rs:185-198) of every walked record, the records split over
 * threads by byte range (a record belongs to the thread whose range holds its first byte); each
 * file's first failing index is kept (an atomic minimum). */
static void* verify_worker(void* arg) {
  const pverify* a = (const pverify*)arg;
  pjob* j = a->j;
  const uint64_t total = j->fbyte[j->nfiles];
  const uint64_t b0 = (uint64_t)(((unsigned __int128)total * a->t) / j->nthreads);
  const uint64_t b1 = (uint64_t)(((unsigned __int128)total * (a->t + 1)) / j->nthreads);
  for (uint32_t f = 0; f < j->nfiles; ++f) {
    const uint64_t fs = j->fbyte[f], fe = j->fbyte[f + 1];
    if (fe <= b0 || fs >= b1 || !j->nrows[f]) continue;
    const uint64_t* o = j->offs[f];
    const uint64_t n = j->nrows[f];
    const uint64_t s = b0 > fs ? b0 - fs : 0, e = b1 - fs; /* offsets in [s, e) of this file */
    uint64_t i = 0, hi = n; /* the first record at or after s */
    while (i < hi) {
      const uint64_t m = (i + hi) / 2;
      if (o[m] < s) i = m + 1; else hi = m;
    }
    const uint8_t* b = j->bufs[f];
    prow* r = j->rows[f];
    for (; i < n && o[i] < e; ++i) {
      const uint8_t* h = b + o[i];
      const uint16_t ksz = rd16(h + 12);
      const uint32_t vsz = rd32(h + 14);
      const uint64_t rl = 18 + (uint64_t)ksz + (vsz == ORC_ENTRY_TOMBSTONE ? 0 : vsz);
      if (orc_xxh32(h + 4, rl - 4, 0) != rd32(h)) {
        uint64_t cur = __atomic_load_n(&j->fbad[f], __ATOMIC_RELAXED);
        while (i < cur && !__atomic_compare_exchange_n(&j->fbad[f], &cur, i, 0, __ATOMIC_RELAXED, __ATOMIC_RELAXED)) {
        }
        continue;
      }
      prow* x = &r[i];
      x->pos = o[i];
      x->seq = rd64(h + 4);
      x->vsz = vsz;
      x->ksz = ksz;
      x->part = (uint8_t)(part_hash(h + 18, ksz) % j->nparts);
    }
  }
  return NULL;
}

typedef struct {
  pjob* j;
  uint32_t p;
} pfold;

static void* fold_worker(void* arg) {
  const pfold* a = (const pfold*)arg;
  pjob* j = a->j;
  orc_index* ix = j->ix[a->p];
  uint64_t mx = 0;
  for (uint32_t f = 0; f < j->stop; ++f) { /* the Cask::open closure (cask.rs:349-355), in replay order */
    const prow* r = j->rows[f];
    const uint8_t* b = j->bufs[f];
    for (uint64_t i = 0; i < j->nrows[f]; ++i) {
      if (r[i].part != a->p) continue;
      if (r[i].seq > mx) mx = r[i].seq;
      orc_index_update(ix, b + r[i].pos + 18, r[i].ksz, j->fids[f], r[i].pos, r[i].vsz, r[i].seq);
    }
  }
  j->pmax[a->p] = mx;
  j->pdig[a->p] = orc_index_digest(ix);
  return NULL;
}

struct orc_pindex {
  orc_index** ix;
  uint32_t nparts;
};

int orc_pindex_seq(const void* pindex, const uint8_t* key, uint16_t ksz, uint64_t* seq) {
  const orc_pindex* p = (const orc_pindex*)pindex;
  return orc_index_get(p->ix[part_hash(key, ksz) % p->nparts], key, ksz, NULL, NULL, NULL, seq);
}

void orc_pindex_free(orc_pindex* p) {
  if (!p) return;
  for (uint32_t i = 0; i < p->nparts; ++i) orc_index_free(p->ix[i]);
  free(p->ix);
  free(p);
}

int orc_replay_parallel(const uint8_t* const* bufs, const uint64_t* lens, const uint32_t* file_ids, uint32_t nfiles,
                        uint32_t nthreads, orc_parallel_result* res, uint32_t* st_fid, uint64_t* st_e, uint64_t* st_d,
                        uint64_t* st_b, uint64_t st_cap) {
  orc_pindex_free(orc_pindex_build(bufs, lens, file_ids, nfiles, nthreads, res, st_fid, st_e, st_d, st_b, st_cap));
  return 0;
}

orc_pindex* orc_pindex_build(const uint8_t* const* bufs, const uint64_t* lens, const uint32_t* file_ids,
                             uint32_t nfiles, uint32_t nthreads, orc_parallel_result* res, uint32_t* st_fid,
                             uint64_t* st_e, uint64_t* st_d, uint64_t* st_b, uint64_t st_cap) {
  memset(res, 0, sizeof(*res));
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 64) nthreads = 64;
  pjob j;
  memset(&j, 0, sizeof j);
  j.bufs = bufs;
  j.lens = lens;
  j.fids = file_ids;
  j.nfiles = nfiles;
  j.nparts = nthreads;
  j.nthreads = nthreads;
  j.offs = (uint64_t**)calloc(nfiles + 1, sizeof(uint64_t*));
  j.rows = (prow**)calloc(nfiles + 1, sizeof(prow*));
  j.nrows = (uint64_t*)calloc(nfiles + 1, 8);
  j.fbad = (uint64_t*)malloc((nfiles + 1) * 8);
  j.fbyte = (uint64_t*)calloc(nfiles + 1, 8);
  j.ferr = (int32_t*)calloc(nfiles + 1, 4);
  j.fpos = (uint64_t*)calloc(nfiles + 1, 8);
  j.fexp = (uint32_t*)calloc(nfiles + 1, 4);
  j.ffound = (uint32_t*)calloc(nfiles + 1, 4);
  for (uint32_t f = 0; f < nfiles; ++f) {
    j.fbad[f] = UINT64_MAX;
    j.fbyte[f + 1] = j.fbyte[f] + lens[f];
  }
  pthread_mutex_init(&j.mu, NULL);
  pthread_t th[64];
  for (uint32_t t = 0; t < nthreads; ++t) pthread_create(&th[t], NULL, walk_worker, &j);
  for (uint32_t t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
  pverify va[64];
  for (uint32_t t = 0; t < nthreads; ++t) {
    va[t].j = &j;
    va[t].t = t;
    pthread_create(&th[t], NULL, verify_worker, &va[t]);
  }
  for (uint32_t t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
  /* each file's first failure: a checksum failure before the walk's cut-short record, else that */
  for (uint32_t f = 0; f < nfiles; ++f) {
    if (j.fbad[f] == UINT64_MAX) continue;
    const uint8_t* h = bufs[f] + j.offs[f][j.fbad[f]];
    const uint64_t rl = 18 + (uint64_t)rd16(h + 12) + (rd32(h + 14) == ORC_ENTRY_TOMBSTONE ? 0 : rd32(h + 14));
    j.ferr[f] = ORC_ROW_CHECKSUM;
    j.fpos[f] = j.offs[f][j.fbad[f]];
    j.fexp[f] = rd32(h);
    j.ffound[f] = orc_xxh32(h + 4, rl - 4, 0);
    j.nrows[f] = j.fbad[f];
  }
  j.stop = nfiles;
  for (uint32_t f = 0; f < nfiles; ++f)
    if (j.ferr[f]) {
      res->err_kind = j.ferr[f];
      res->err_file_id = file_ids[f];
      res->err_pos = j.fpos[f];
      res->err_expected = j.fexp[f];
      res->err_found = j.ffound[f];
      j.stop = f + 1;
      break;
    }
  for (uint32_t f = 0; f < j.stop; ++f) res->records += j.nrows[f];
  j.ix = (orc_index**)calloc(j.nparts, sizeof(orc_index*));
  j.pmax = (uint64_t*)calloc(j.nparts, 8);
  j.pdig = (uint64_t*)calloc(j.nparts, 8);
  pfold pa[64];
  for (uint32_t p = 0; p < j.nparts; ++p) {
    j.ix[p] = orc_index_new();
    pa[p].j = &j;
    pa[p].p = p;
    pthread_create(&th[p], NULL, fold_worker, &pa[p]);
  }
  for (uint32_t p = 0; p < j.nparts; ++p) pthread_join(th[p], NULL);
  /* per-file counters: the partitions' rows added up (a file has a row if any partition has one) */
  uint64_t ns = 0;
  uint32_t* fid_tmp = (uint32_t*)malloc(sizeof(uint32_t) * 65536);
  uint64_t* e_tmp = (uint64_t*)malloc(8 * 65536 * 3);
  for (uint32_t p = 0; p < j.nparts; ++p) {
    const orc_index* ix = j.ix[p];
    res->live += orc_index_len(ix);
    res->digest += j.pdig[p];
    if (j.pmax[p] > res->max_seq) res->max_seq = j.pmax[p];
    uint32_t* sf = fid_tmp;
    uint64_t *se = e_tmp, *sd = e_tmp + 65536, *sb = e_tmp + 2 * 65536;
    const uint64_t n = orc_index_stats(ix, sf, se, sd, sb, 65536);
    for (uint64_t i = 0; i < n && i < 65536; ++i) {
      uint64_t k = 0;
      while (k < ns && k < st_cap && st_fid[k] != sf[i]) ++k;
      if (k == ns) {
        if (ns < st_cap) {
          st_fid[ns] = sf[i];
          st_e[ns] = st_d[ns] = st_b[ns] = 0;
        }
        ++ns;
      }
      if (k < st_cap) {
        st_e[k] += se[i];
        st_d[k] += sd[i];
        st_b[k] += sb[i];
      }
    }
  }
  free(fid_tmp);
  free(e_tmp);
  res->stats_rows = ns;
  orc_pindex* out = (orc_pindex*)malloc(sizeof(orc_pindex));
  out->ix = j.ix;
  out->nparts = j.nparts;
  for (uint32_t f = 0; f < nfiles; ++f) {
    free(j.rows[f]);
    free(j.offs[f]);
  }
  free(j.offs);
  free(j.fbad);
  free(j.fbyte);
  free(j.pmax);
  free(j.pdig);
  free(j.rows);
  free(j.nrows);
  free(j.ferr);
  free(j.fpos);
  free(j.fexp);
  free(j.ffound);
  pthread_mutex_destroy(&j.mu);
  return out;
}
