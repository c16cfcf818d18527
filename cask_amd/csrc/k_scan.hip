// k_scan_chunks — the hot kernel of the Cask data-file scan (gfx950 / CDNA4).
//
// The reference walks each data file record by record on one CPU thread:
//   Entries::next (log.rs:403-429) -> Entry::from_read (data.rs:161-206)
// reading the 18-byte header `xxh32 u32 | seq u64 | ksz u16 | vsz u32` (LE), the key, the value
// (absent for a tombstone, vsz == 0xFFFFFFFF) and checking XXH32(header[4..] ‖ key ‖ value).
//
// Here every file is cut into fixed-size chunks and a persistent grid streams through them, in
// runs of consecutive chunks claimed from a counter. Per chunk, one workgroup:
//   1. has the chunk (+ halo) staged into LDS by its loader waves: the 16-B loads for the next
//      chunk are issued into registers before this one is processed;
//   2. takes the chunk's first record boundary from the previous chunk of the run (the carry) or,
//      for a run's first chunk, finds it speculatively: the lowest offset whose header gives a
//      record that fits and whose XXH32 matches its stored checksum;
//   3. stride pass: one record per lane at the first record's length, header checked, XXH32 out of
//      LDS (aligned dwords only); the rows go to an LDS row buffer that the store wave flushes
//      during the next chunk — or, for a regular chunk, only its first row is kept (kCountRegular);
//   4. slow path when the stride breaks: walk the chain, hash one record per quad of lanes.
// No workgroup ever waits on another: boundary speculation is checked afterwards (k_val_*) and
// rows are ordered by a later pass (k_compact), both in k_pipeline.hip.
#include "device_util.h"

#include <stdlib.h>
#include "knobs.h"

namespace cask_dev {

template <uint32_t CH, uint32_t HALO, uint32_t NT, uint32_t PER_CU, bool NT_LOADS = false>
struct Geo {
  static constexpr uint32_t kCh = CH, kHaloB = HALO, kNT = NT, kWinB = CH + HALO, kPerCU = PER_CU;
  // staging loads with the nontemporal policy (the bytes are read once): measured faster only
  // together with the short halo (GeoS), see DESIGN.md
  static constexpr bool kNtLoads = NT_LOADS;
  static constexpr uint32_t kWavesPerSimd = PER_CU * NT / 256;  // 4 SIMDs of 64-lane waves per CU
  static constexpr uint32_t kMaxStartsG = CH / 18 + 2;  // every record is >= 18 bytes
  static constexpr uint32_t kRowBuf = kMaxStartsG / 16;   // slot rows per LDS row buffer (2 in starts' space)
  static constexpr uint32_t kWinWords = (kWinB + 64) / 4;
  // With 4+ waves, the last wave loads nothing: it issues the workgroup's stores (slot rows, chunk
  // table, run claims), so no wave that stages the window ever waits for a store to complete.
  static constexpr bool kStoreWave = NT >= 256;
  static constexpr uint32_t kLoadT = kStoreWave ? NT - 64 : NT;  // threads that stage the window
  static constexpr uint32_t kMetaT = kStoreWave ? NT - 64 : 0;   // the thread that issues the stores
  static constexpr uint32_t kNL = ((kWinB + 16) / 16 + kLoadT - 1) / kLoadT;  // 16-B loads per loader
};

// Records no longer than this are "short": the boundary search verifies them first.
constexpr uint32_t kShortMax = 1024;
// Offsets each thread tests per step of the boundary search (1: measured no slower than 4).
constexpr uint32_t kSearchPer = 1;

#define BAR() __syncthreads()

template <class G>
struct __attribute__((aligned(16))) ScanLdsT {
  uint32_t win[G::kWinWords];        // staged bytes (16-B aligned base + <= 15 B shift + slop)
  union {
    uint16_t starts[G::kMaxStartsG];  // slow path: record starts relative to the chunk start
    u32x4 rows[2][G::kRowBuf];        // stride pass: the first kRowBuf slot rows of the chunk (parity
                                      // buffer), flushed as 16-B stores while the next chunk runs
  };
  uint32_t found, n;  // search result; slow path: rows of the chunk
  uint32_t claimed;   // the run this workgroup takes after its current one
  uint32_t ffail;     // stride pass: first row whose header breaks the stride
  uint32_t ldefer;    // slow path: first row left to k_long (longer than ScanArgs::big)
  uint32_t irreg;     // stride pass: some row breaks the regular-chunk pattern (kCountRegular)
  uint32_t cerr_s;    // stride pass: lowest failing row (rows past the stride break included)
  uint32_t cerr_w;    // slow path: lowest failing row
  uint64_t exitv, lastp, lastrl;  // slow path: walk results (wave 0 -> workgroup)
};

struct ChunkPos {
  const uint8_t* data;
  uint64_t len, c0, c1, wend;
  uintptr_t a0;
  uint32_t fi, shift, n16;
};

// The window of the chunk at byte c0 of file fi.
template <class G>
__device__ __forceinline__ ChunkPos chunk_at(const uint8_t* data, uint64_t len, uint32_t fi, uint64_t c0) {
  ChunkPos c;
  c.fi = fi;
  c.data = data;
  c.len = len;
  c.c0 = c0;
  c.c1 = (c.c0 + G::kCh < c.len) ? c.c0 + G::kCh : c.len;
  c.wend = (c.c0 + G::kWinB < c.len) ? c.c0 + G::kWinB : c.len;
  const uintptr_t gstart = (uintptr_t)(c.data + c.c0);
  c.a0 = gstart & ~(uintptr_t)15;
  c.shift = (uint32_t)(gstart - c.a0);
  const uintptr_t aend = ((uintptr_t)(c.data + c.wend) + 15) & ~(uintptr_t)15;
  c.n16 = (uint32_t)((aend - c.a0) >> 4);
  return c;
}

template <class G>
__device__ __forceinline__ ChunkPos locate(const FileDesc* files, uint32_t nfiles, uint64_t t) {
  const uint32_t fi = find_file(files, nfiles, t);
  DCHECK(fi < nfiles, "fi %u t %llu", fi, (unsigned long long)t);
  const FileDesc fd = files[fi];
  DCHECK(t >= fd.first_chunk && t < fd.first_chunk + fd.nchunks, "fi %u t %llu first %llu n %llu", fi,
         (unsigned long long)t, (unsigned long long)fd.first_chunk, (unsigned long long)fd.nchunks);
  return chunk_at<G>(fd.data, fd.len, fi, (t - fd.first_chunk) * (uint64_t)G::kCh);
}

// Chunk tn, the successor of cur's chunk t: the next chunk of the same file needs no table lookup
// (the binary search is a chain of dependent scalar loads).
template <class G>
__device__ __forceinline__ ChunkPos next_chunk(const FileDesc* files, uint32_t nfiles, const ChunkPos& cur,
                                               uint64_t t, uint64_t tn) {
  if (tn == t + 1 && cur.c0 + G::kCh < cur.len) return chunk_at<G>(cur.data, cur.len, cur.fi, cur.c0 + G::kCh);
  return locate<G>(files, nfiles, tn);
}

// Issue every 16-B load of a window (clamped index: no branch around a load, so all of them are
// in flight at once); the data lands in LDS later, in stage_store.
// Global (address space 1) view of the staged bytes. Without it the loads compile to flat_load,
// which also count on lgkmcnt and retire out of order with LDS reads: a counted LDS wait in the
// walk could then be satisfied by a prefetch load instead of its own read.
typedef __attribute__((address_space(1))) const u32x4 gu32x4;

template <class G>
__device__ __forceinline__ void stage_issue(u32x4 (&v)[G::kNL], const ChunkPos& c,
                                            unsigned long long* dbg = nullptr, uint64_t t = 0) {
  const gu32x4* src = (const gu32x4*)c.a0;
  DCHECK(c.n16 >= 1 && c.n16 <= G::kNL * G::kLoadT && c.n16 * 16 <= G::kWinWords * 4 &&
             c.a0 >= ((uintptr_t)c.data & ~(uintptr_t)15) && c.a0 + 16ull * c.n16 <= (((uintptr_t)c.data + c.len + 15) & ~(uintptr_t)15),
         "n16 %u a0 %llx data %llx len %llu c0 %llu", c.n16, (unsigned long long)c.a0,
         (unsigned long long)(uintptr_t)c.data, (unsigned long long)c.len, (unsigned long long)c.c0);
  if (G::kStoreWave && threadIdx.x >= G::kLoadT) return;
  if (c.n16 == G::kNL * G::kLoadT) {  // the whole window is inside the file: no clamping
#pragma unroll
    for (uint32_t j = 0; j < G::kNL; ++j) {
      if constexpr (G::kNtLoads) v[j] = __builtin_nontemporal_load(&src[threadIdx.x + j * G::kLoadT]);
      else v[j] = src[threadIdx.x + j * G::kLoadT];
    }
    return;
  }
#pragma unroll
  for (uint32_t j = 0; j < G::kNL; ++j) {
    const uint32_t i = threadIdx.x + j * G::kLoadT;
    // (the same policy on both paths: the compiler merges them, and a merged load keeps no policy)
    if constexpr (G::kNtLoads) v[j] = __builtin_nontemporal_load(&src[i < c.n16 ? i : c.n16 - 1]);
    else v[j] = src[i < c.n16 ? i : c.n16 - 1];
  }
}

template <class G>
__device__ __forceinline__ void stage_store(ScanLdsT<G>& L, const u32x4 (&v)[G::kNL], const ChunkPos& c) {
  u32x4* dst = (u32x4*)L.win;
  if (G::kStoreWave && threadIdx.x >= G::kLoadT) return;
  if (c.n16 == G::kNL * G::kLoadT) {
#pragma unroll
    for (uint32_t j = 0; j < G::kNL; ++j) dst[threadIdx.x + j * G::kLoadT] = v[j];
    return;
  }
#pragma unroll
  for (uint32_t j = 0; j < G::kNL; ++j) {
    const uint32_t i = threadIdx.x + j * G::kLoadT;
    // lanes past the window loaded the last 16-B unit again (stage_issue clamps): storing that same
    // value to it keeps every v[j] consumed on every path, so the compiler's memory-counter waits
    // for these loads all happen here and none is left over for the next prefetch to wait on
    dst[i < c.n16 ? i : c.n16 - 1] = v[j];
  }
}

// The slot row of the record at chunk offset `off` (row r of chunk t), built by a quad of lanes
// (lane a = 0..3 of the quad): header fields, and the checksum verified out of LDS by the quad
// unless the record runs past the window (then k_long does it). Lane a writes dword a of the
// 16-B row, so a wave's rows go out as contiguous 256-B stores. All four lanes return whether
// the row is a failure (InvalidChecksum, or the UnexpectedEof row).
template <class G>
__device__ __forceinline__ bool quad_row(const uint32_t* W, const ChunkPos& c, uint32_t* slots, uint32_t r,
                                         uint32_t off, uint32_t a, uint32_t big, Diag& dg) {
#ifdef CASK_STAMPS
  const uint64_t st_h0_ = __builtin_amdgcn_s_memtime();
#endif
  const uint64_t p = c.c0 + off;
  uint32_t w0 = 0, w1 = 0, w2 = 0, w3 = off << 16;
  bool fail = false;
  if (p + 18 > c.len) {
    fail = true;  // EOF row: seq/ksz/vsz stay 0
  } else {
    const uint32_t x = off + c.shift;
    const Hdr h = lds_hdr(W, x);
    w0 = (uint32_t)h.seq;
    w1 = (uint32_t)(h.seq >> 32);
    w2 = h.vsz;
    w3 |= h.ksz;
    const uint64_t rl = 18ull + h.ksz + ((h.vsz == 0xFFFFFFFFu) ? 0ull : (uint64_t)h.vsz);
    if (p + rl > c.len) {
      fail = true;  // EOF row (data.rs:172,181)
    } else if (lds_hashed(p, rl, c.wend, big)) {
      if (quad_xxh32(W, x + 4, (uint32_t)rl - 4, a) != h.stored) {  // data.rs:193-198
        w3 |= kSlotBad;
        fail = true;
      }
    }  // else: left to k_long (hashed from HBM)
  }
  const uint32_t word = a == 0 ? w0 : a == 1 ? w1 : a == 2 ? w2 : w3;
#ifdef CASK_STAMPS
  const uint64_t st_h1_ = __builtin_amdgcn_s_memtime();
  dg.st[8] += st_h1_ - st_h0_;  // phase 8: header + hash of one record
#endif
  slots[4ull * r + a] = word;
#ifdef CASK_STAMPS
  dg.st[9] += __builtin_amdgcn_s_memtime() - st_h1_;  // phase 9: issuing the slot store
#endif
  return fail;
}

// ceil(a / b) for 0 < b < a <= 2^16 (wave-uniform): a float quotient, corrected to the exact one.
__device__ __forceinline__ uint32_t ceil_div_small(uint32_t a, uint32_t b) {
  uint32_t c = (uint32_t)__builtin_ceilf((float)a / (float)b);
  if (c * b < a) ++c;
  if ((c - 1) * b >= a) --c;
  return c;
}

// A chunk's entries in the chunk table (wave-uniform): written by the store wave for a whole run
// of chunks at once (consecutive entries: a few full-line stores instead of five scattered ones
// per chunk), or straight away where there is no store wave.
struct Meta {
  uint64_t spec, exit;
  uint32_t count, long_r;
  uint32_t cerr;  // first failing row (!0: none): ScanArgs::cerr
  u32x4 desc;  // first row of a regular chunk
};

// Slot rows [0, n) of a chunk from LDS row buffer `par` to its slots, one 16-B store per row.
template <class G>
__device__ __forceinline__ void flush_rows(ScanLdsT<G>& L, uint32_t par, uint32_t* slots, uint32_t n) {
  u32x4* srow = (u32x4*)slots;
  if (G::kStoreWave && threadIdx.x < G::kLoadT) return;  // the store wave's job
  const uint32_t first = G::kStoreWave ? threadIdx.x - G::kLoadT : threadIdx.x;
  const uint32_t step = G::kStoreWave ? 64u : G::kNT;
  for (uint32_t r = first; r < n; r += step) srow[r] = L.rows[par][r];
}

template <class G, bool EXACT>
__device__ __forceinline__ void process_chunk(ScanLdsT<G>& L, const ScanArgs& a, uint64_t t, const ChunkPos& c,
                                              uint64_t s_exact, uint64_t& carry, bool& known, bool& strided, uint32_t par,
                                              uint32_t& pf_n, uint32_t*& pf_slots, Meta& m, Diag& dg) {
  constexpr uint32_t NT = G::kNT;
  constexpr uint32_t NQ = NT / 4;  // quads: one record per quad of lanes
  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, quad = tid >> 2, qa = tid & 3;
  const uint32_t* W = L.win;
  const uint64_t len = c.len, c0 = c.c0, c1 = c.c1, wend = c.wend;
  const uint32_t shift = c.shift;
  STAMP_INIT

  // 2. the chunk's first record boundary
  uint64_t s;
  if (c0 == 0) {
    s = 0;  // a file's first record starts at 0 (log.rs:116)
  } else if (known) {
    // the previous chunk of this range ended its chain at `carry` (>= c0): no search needed. In
    // the exact pass too: the run's first start is exact, so the carry is, and a stretch of
    // chunks whose stale starts came from the speculative pass is settled in this one pass.
    s = (carry == kTerm || carry >= c1) ? kNone : carry;
  } else if (EXACT) {
    s = s_exact;
  } else {
    const uint32_t span = (uint32_t)(c1 - c0);
    // pass A: short records starting in the first kShortMax bytes; pass B: everything, in order.
    // Control flow depends on L.found only as read between the two barriers of a step: any other
    // read could see a faster wave's atomicMin of the next step, and the waves' barrier counts
    // would part ways.
    bool found = false;
    for (uint32_t pass = 0; pass < 2 && !found; ++pass) {
      const uint32_t lim = pass == 0 ? (span < kShortMax ? span : kShortMax) : span;
      // kSearchPer offsets per thread per step (1: measured no slower than 4 on either workload)
      for (uint32_t kb = 0; kb < lim; kb += kSearchPer * NT) {
        uint64_t rl[kSearchPer];
#pragma unroll
        for (uint32_t j = 0; j < kSearchPer; ++j) {  // all header reads first
          const uint32_t k = kb + tid + j * NT;
          rl[j] = (k < lim && c0 + k + 18 <= len) ? lds_reclen(W, k + shift) : ~0ull;
        }
#pragma unroll
        for (uint32_t j = 0; j < kSearchPer; ++j) {
          const uint32_t k = kb + tid + j * NT;
          const uint64_t p = c0 + k;
          if (rl[j] != ~0ull && p + rl[j] <= wend && (pass == 1 || rl[j] <= kShortMax)) {
            const uint32_t x = k + shift;
            const Hdr h = lds_hdr(W, x);
            if (lds_xxh32(W, x + 4, (uint32_t)rl[j] - 4) == h.stored) atomicMin(&L.found, k);
          }
        }
        BAR();
        const bool done = L.found != 0xFFFFFFFFu;
        BAR();
        if (done) {
          found = true;
          break;
        }
      }
    }
    s = found ? c0 + L.found : kNone;  // no atomicMin after the last step's barriers
    s = uni64(s);
  }
  STAMP(0)

  // 3. The chunk's records. Stride pass: assume every record from s on has the first record's
  // length rl0 and let thread i take the record at s + i*rl0 — check its header, verify it,
  // write its row. The first i whose header breaks the stride (L.ffail) ends the run of true
  // records; rows past it are discarded. A file of equal-length records never leaves this pass.
  uint32_t* slots = a.slots + ((uint64_t)t * a.slot_cap) * 4;
  uint32_t n = 0, cerr = 0xFFFFFFFFu;  // cerr: the chunk's first failing row
  uint64_t exitv = 0, lastp = 0, lastrl = 0;
  bool rl0_big = false;  // the stride rows' records are longer than a.big (k_long hashes them)
  uint32_t k = 0;  // rows settled by the stride pass
  bool slow = false, regular = false;
  if (s != kNone) {
    // Chunk-relative 32-bit offsets: every stride record starts below c1 <= c0 + CH.
    const uint32_t srel = (uint32_t)(s - c0), span = (uint32_t)(c1 - s);
    const uint64_t lrel64 = len - c0;
    const uint32_t lrel = lrel64 < 0xFFFFFFFFull ? (uint32_t)lrel64 : 0xFFFFFFFFu;
    uint64_t rl0 = 0;
    uint32_t cnt = 0;
    if (s + 18 <= len) {
      rl0 = uni64(lds_reclen(W, srel + shift));  // wave-uniform: scalar loop counts in the hash
      if (s + rl0 <= len) cnt = rl0 >= span ? 1u : ceil_div_small(span, (uint32_t)rl0);
    }
    // Records 1..3 at the stride (uniform reads, one LDS round trip): if one breaks it, the chunk's
    // records vary in length and the slow path takes them all — otherwise the stride pass would
    // hash cnt strided stretches of bytes that are not records.
    // Skipped after a chunk the stride pass settled whole (uniform logs: the next chunk almost
    // always is too, and the pass itself finds a break).
    if (cnt > 1 && !strided) {
      bool brk = false;
#pragma unroll
      for (uint32_t j = 1; j <= 3; ++j) {
        const uint64_t q = s + j * rl0;
        if (j < cnt && q + 18 <= len) brk |= lds_reclen(W, (uint32_t)(q - c0) + shift) != rl0;
      }
      if (brk) cnt = 0;
    }
    rl0_big = rl0 > a.big;
    const uint32_t r32 = cnt > 1 ? (uint32_t)rl0 : 0u;  // stride; rl0 < span <= CH when cnt > 1
    // One record per lane, its four XXH32 accumulators interleaved.
    const uint32_t hl = (uint32_t)rl0 - 4;
    auto stride_ok = [&](uint32_t i, uint32_t o, const Hdr& h) -> bool {
      if (!i) return true;  // cnt > 0: the first record fits the file
      const uint64_t rl = 18ull + h.ksz + ((h.vsz == 0xFFFFFFFFu) ? 0ull : (uint64_t)h.vsz);
      return o + 18 <= lrel && rl == rl0 && o + r32 <= lrel;  // o + r32 < 2 * CH: no wrap
    };
#ifdef CASK_STAMPS
    const uint64_t st_h0_ = __builtin_amdgcn_s_memtime();
#endif
    // the first record's header, for the regular-chunk test (one LDS broadcast)
    const Hdr hf = cnt ? lds_hdr(W, srel + shift) : Hdr{};
    bool irreg = false;
    for (uint32_t i = tid; i < cnt; i += NT) {
      const uint32_t o = srel + i * r32;
      const Hdr h = lds_hdr(W, o + shift);  // inside the window: o < CH
      const bool ok = stride_ok(i, o, h);
      const bool hs = ok && lds_hashed(c0 + o, rl0, wend, a.big);  // else k_long
      const uint32_t g = hs ? lane_xxh32(W, o + shift + 4, hl) : h.stored;
      if (!ok) {
        atomicMin(&L.ffail, i);
      } else {
        const bool bad = hs && g != h.stored;  // data.rs:193-198
        u32x4 row;
        row.x = (uint32_t)h.seq;
        row.y = (uint32_t)(h.seq >> 32);
        row.z = h.vsz;
        row.w = h.ksz | (o << 16) | (bad ? kSlotBad : 0u);
        if (i < G::kRowBuf) L.rows[par][i] = row;
        else ((u32x4*)slots)[i] = row;
        if (bad) atomicMin(&L.cerr_s, i);
        irreg |= bad || !hs || h.ksz != hf.ksz || h.vsz != hf.vsz || h.seq != hf.seq + i;
      }
    }
    if (__ballot(irreg) && lane == 0) atomicOr(&L.irreg, 1u);
#ifdef CASK_STAMPS
    dg.st[8] += __builtin_amdgcn_s_memtime() - st_h0_;  // phase 8: the stride pass's rows
#endif
    BAR();
    k = L.ffail < cnt ? L.ffail : cnt;
    pf_n = k < G::kRowBuf ? k : G::kRowBuf;  // buffered rows of the settled records [0, k)
    pf_slots = slots;
    regular = a.regular_ok && k == cnt && cnt && !L.irreg;
    if (regular) {  // the first row describes them all (kCountRegular): it goes to desc[t]
      pf_n = 0;
      m.desc.x = (uint32_t)hf.seq;
      m.desc.y = (uint32_t)(hf.seq >> 32);
      m.desc.z = hf.vsz;
      m.desc.w = hf.ksz | (srel << 16);
    }
    // the lowest failing row counts only if it lies before the stride break (then it is the first)
    cerr = L.cerr_s < k ? L.cerr_s : 0xFFFFFFFFu;
    if (k == cnt && cnt) {
      n = cnt;
      lastp = s + (uint64_t)(cnt - 1) * rl0;
      lastrl = rl0;
      exitv = lastp + rl0;  // >= c1
    } else {
      slow = true;  // the stride broke at row k (or the first record is cut short)
    }
  }
  STAMP(1)

  // 4. Slow path: walk the chain from the first record the stride pass did not settle (wave 0;
  // each step tests up to 256 equal-stride successors with one LDS round trip), then verify
  // those records, one per thread.
  if (slow) {
    // starts[] overlays both row buffers: flush this chunk's buffered rows now (the previous chunk's
    // were read before this chunk's barrier... and its flush loop runs before process_chunk)
    flush_rows<G>(L, par, pf_slots, pf_n);
    pf_n = 0;
    BAR();
    if (wave == 0) {
      uint32_t nn = k, ld = 0xFFFFFFFFu;  // ld: first walked row longer than a.big
      uint64_t ex = 0, lp = 0, lr = 0;
      uint64_t p = s + (k ? (uint64_t)k * lds_reclen(W, (uint32_t)(s - c0) + shift) : 0ull);
      for (;;) {
        if (p >= c1) {
          ex = p;
          break;
        }
        if (p + 18 > len) {  // header cut short: Io(UnexpectedEof) (data.rs:163)
          if (lane == 0) L.starts[nn] = (uint16_t)(p - c0);
          ++nn;
          ex = kTerm;
          break;
        }
        const uint64_t rl = lds_reclen(W, (uint32_t)(p - c0) + shift);
        if (p + rl > len) {  // key/value cut short (data.rs:172,181)
          if (lane == 0) L.starts[nn] = (uint16_t)(p - c0);
          ++nn;
          ex = kTerm;
          break;
        }
        if (rl > a.big && ld == 0xFFFFFFFFu) ld = nn;
        const uint64_t span = c1 - p;
        const uint32_t M = span > 192ull * rl ? 4u : span > 128ull * rl ? 3u : span > 64ull * rl ? 2u : 1u;
        bool vj[4];
#pragma unroll
        for (uint32_t jj = 0; jj < 4; ++jj) {  // all reads first: they do not wait on each other
          const uint64_t i = (uint64_t)lane + 64u * jj;
          const uint64_t q = p + i * rl;
          bool v = jj < M;
          if (v && i) {
            v = (q < c1) && (q + 18 <= len);
            if (v) v = (lds_reclen(W, (uint32_t)(q - c0) + shift) == rl) && (q + rl <= len);
          }
          vj[jj] = v;
        }
        uint32_t kk = 0;
        bool open = true;
#pragma unroll
        for (uint32_t jj = 0; jj < 4; ++jj) {
          const unsigned long long okm = __ballot(vj[jj]);
          if (open) {
            const uint32_t kj = (~okm) ? (uint32_t)__builtin_ctzll(~okm) : 64u;
            if (lane < kj) L.starts[nn + kk + lane] = (uint16_t)(p + ((uint64_t)lane + 64u * jj) * rl - c0);
            kk += kj;
            open = kj == 64u;
          }
        }
        nn += kk;
        lp = p + (uint64_t)(kk - 1) * rl;
        lr = rl;
        p += (uint64_t)kk * rl;
      }
      if (lane == 0) {
        L.n = nn;
        L.ldefer = ld;
        L.exitv = ex;
        L.lastp = lp;
        L.lastrl = lr;
      }
    }
    BAR();
    n = L.n;
    exitv = L.exitv;
    lastp = L.lastp;
    lastrl = L.lastrl;
    for (uint32_t r = k + quad; r < n; r += NQ) {
      if (quad_row<G>(W, c, slots, r, L.starts[r], qa, a.big, dg) && qa == 0) atomicMin(&L.cerr_w, r);
    }
    BAR();  // every slow-path row's verdict is in L.cerr_w
    cerr = cerr < L.cerr_w ? cerr : L.cerr_w;
  }
  DCHECK(n <= a.slot_cap && t < a.total_chunks, "n %u t %llu", n, (unsigned long long)t);
  m.spec = s;
  m.exit = (s == kNone) ? 0 : exitv;
  m.count = n | (regular ? kCountRegular : 0u);
  m.cerr = cerr;
  // a record that does not fit the window is hashed from HBM by k_long (only the last can)
  // k_long hashes, from row long_r on, the rows lds_hashed() rejects: from 0 when the stride rows
  // are longer than a.big; else the slow path's first such row; else the last row when it runs
  // past the window
  m.long_r = (s == kNone || !n) ? 0xFFFFFFFFu
             : (k && rl0_big) ? 0u
             : (L.ldefer != 0xFFFFFFFFu) ? L.ldefer
             : (exitv != kTerm && lastp + lastrl > wend) ? n - 1 : 0xFFFFFFFFu;
  if (!G::kStoreWave && tid == G::kMetaT) {
    a.spec[t] = m.spec;  // the exact pass too: the start it used (the carry may replace spec[t])
    a.exit[t] = m.exit;
    a.count[t] = m.count;
    a.long_r[t] = m.long_r;
    a.cerr[t] = m.cerr;
    a.long_done[t] = 0;
    if (regular) ((u32x4*)a.desc)[t] = m.desc;
  }
  // the next chunk of the run starts where this chain left off
  if (s != kNone) {
    carry = exitv;
    known = true;
  }  // else: a known chain skips this chunk and stays known; an unknown one stays unknown
  strided = s != kNone && !slow;
  STAMP(2)
}

// Persistent grid, kPerCU workgroups per CU; each workgroup walks a contiguous range of chunks in
// order. Only a range's first chunk searches for its first record boundary: every later chunk
// starts where the previous one's chain left off (the carry), so the search — a third of the
// cycles of a speculated chunk — runs once per range. Placement only affects speed: any
// assignment of chunks to workgroups is correct, and the validation pass checks every start.
// EXACT (the repair re-scan) reads each run's first start from spec[] (later chunks of the run take
// the carry) and writes back the start it used; the speculative kernel
// issues no global load besides the staging loads, so the compiler's counted waits never make the
// processing of one chunk wait for the prefetch of the next.
// `files` is the same table as a.files, passed as a restrict-qualified argument: the kernel never
// writes it, so its (wave-uniform) loads go through the scalar cache.
template <class G, bool EXACT>
__global__ __launch_bounds__(G::kNT, G::kWavesPerSimd) void k_scan_chunks(ScanArgs a, const FileDesc* __restrict__ files_r) {
  __shared__ ScanLdsT<G> L;
  const FileDesc* __restrict__ files = files_r;
  // Runs of a.run consecutive chunks are handed out in order by a counter (one atomic per run, a
  // run ahead), so workgroups that run slower take fewer runs and all finish together; each run is
  // walked in order with a carry.
  // A repair pass re-scans only the stretches listed in a.runs (each one walked like a run).
  // The last stretch of chunks (from a.run_tail) goes out in shorter runs of a.run_small, so that
  // the workgroups run out of work closer together (a run of 16 chunks is ~90 us of one workgroup).
  const uint64_t R = a.run, Rs = a.run_small;
  const uint64_t nbig = a.run_tail / R;  // a.run_tail: a multiple of R (>= total_chunks: no tail)
  const uint64_t nruns = a.runs ? a.nruns_list
                         : a.run_tail < a.total_chunks ? nbig + (a.total_chunks - a.run_tail + Rs - 1) / Rs
                                                       : (a.total_chunks + R - 1) / R;
  auto run_at = [&](uint64_t r, uint64_t& first, uint64_t& end) {
    if (a.runs) {
      first = a.runs[2 * r];
      end = a.runs[2 * r + 1];
    } else {
      const bool big = r < nbig;
      first = big ? r * R : a.run_tail + (r - nbig) * Rs;
      end = first + (big ? R : Rs);
      end = end < a.total_chunks ? end : a.total_chunks;
    }
  };
  uint32_t my_claim = 0;  // thread kMetaT: the run claimed for after the current one
  bool publish = false;   // thread kMetaT: my_claim still to be published in L.claimed
  // The first two runs of every workgroup are fixed by its index (a grid's worth of claims on one
  // counter at once queue for tens of microseconds); later ones come from the counter.
  if (threadIdx.x == G::kMetaT) {
    L.found = blockIdx.x;
    L.claimed = blockIdx.x + gridDim.x;
  }
  BAR();
  const uint64_t r0 = L.found;
  if (r0 >= nruns) return;
  uint64_t t, run_end;
  run_at(r0, t, run_end);
  uint64_t run_first = t;  // first chunk of the current run (its chunk-table entries go out together)
  BAR();  // L.found is reset by thread 0 below
#ifdef CASK_STAMPS
  const uint64_t rt0_ = __builtin_amdgcn_s_memrealtime();  // 100 MHz: calibrates s_memtime, shows imbalance
#endif
  Diag dg{};
  uint32_t par = 0;          // row buffer of the current chunk
  uint32_t pf_n = 0;         // rows of the previous chunk waiting in row buffer par ^ 1
  uint32_t* pf_slots = a.slots;
  uint64_t carry = 0;  // chain position entering chunk t, when known
  bool known = false;  // only the first chunk of the range (and chunks after a failed search) search
  bool strided = false;  // the previous chunk's records were all settled by the stride pass
  ChunkPos cur = locate<G>(files, a.nfiles, t);
  u32x4 v[G::kNL];
  stage_issue<G>(v, cur, a.stamps, t);
  for (;;) {
#ifdef CASK_STAMPS
    const uint64_t st_top_ = __builtin_amdgcn_s_memtime();
    if (dg.st[7] == 0) dg.st[7] = st_top_;  // first stamp: total = last - first
#endif
    if (threadIdx.x == 0) {  // every reader of the last chunk's values is past the end barrier
      L.found = 0xFFFFFFFFu;
      L.ffail = 0xFFFFFFFFu;
      L.irreg = 0u;
      L.ldefer = 0xFFFFFFFFu;
      L.cerr_s = 0xFFFFFFFFu;
      L.cerr_w = 0xFFFFFFFFu;
    }
    if (threadIdx.x == G::kMetaT && publish) {
      L.claimed = my_claim;
      publish = false;
    }
    stage_store<G>(L, v, cur);
    BAR();
#ifdef CASK_STAMPS
    dg.st[3] += __builtin_amdgcn_s_memtime() - st_top_;  // phase 3: window wait + LDS store
    dg.st[4] += 1;
#endif
    // exact (repair) pass: the chunk's known start, loaded before the prefetch is issued so that
    // waiting for it never waits for the prefetch
    const uint64_t s_exact = EXACT ? a.spec[t] : 0;
    uint64_t tn = t + 1, next_end = run_end;
    if (tn >= run_end) {  // next run of this workgroup: the one claimed a run ago
      const uint64_t rn = L.claimed;
      if (rn < nruns) {
        run_at(rn, tn, next_end);
      } else {
        tn = a.total_chunks;
        next_end = tn;
      }
      if (threadIdx.x == G::kMetaT && rn < nruns) {
        my_claim = 2u * gridDim.x + atomicAdd(&a.ctr->run_next, 1u);  // published at the next chunk's top
        publish = true;
      }
    }
    const bool more = tn < a.total_chunks;
#ifdef CASK_STAMPS
    const uint64_t st_pf_ = __builtin_amdgcn_s_memtime();
#endif
    // the previous chunk's buffered rows go out ahead of the prefetch: no vector-memory instruction
    // is issued while the chunk is processed, and none waits behind the prefetch's loads
    flush_rows<G>(L, par ^ 1, pf_slots, pf_n);
    pf_n = 0;
    ChunkPos nxt = cur;
    if (more) {
      nxt = next_chunk<G>(files, a.nfiles, cur, t, tn);
      stage_issue<G>(v, nxt, a.stamps, tn);  // prefetch the next window
    }
#ifdef CASK_STAMPS
    dg.st[5] += __builtin_amdgcn_s_memtime() - st_pf_;  // phase 5: issuing the prefetch
#endif
    Meta m;
    m.desc = u32x4{0u, 0u, 0u, 0u};
    process_chunk<G, EXACT>(L, a, t, cur, s_exact, carry, known, strided, par, pf_n, pf_slots, m, dg);
    if (G::kStoreWave && threadIdx.x >= G::kLoadT) {
      // store wave: lane (t - run_first) keeps chunk t's entries in the staging registers this wave
      // never loads into; the run's entries go out when the run ends
      const uint32_t li = (uint32_t)(t - run_first), sl = threadIdx.x & 63;
      if (sl == li) {
        v[0] = u32x4{(uint32_t)m.spec, (uint32_t)(m.spec >> 32), (uint32_t)m.exit, (uint32_t)(m.exit >> 32)};
        v[1] = u32x4{m.count, m.long_r, m.cerr, 0u};
        v[2] = m.desc;
      }
      const bool run_ends = tn != t + 1 || !more || li == 63;  // (a run is at most 64 chunks)
      if (run_ends) {  // run ends (or a wave's worth of entries)
        if (sl <= li) {
          const uint64_t g = run_first + sl;
          a.spec[g] = (uint64_t)v[0].x | ((uint64_t)v[0].y << 32);
          a.exit[g] = (uint64_t)v[0].z | ((uint64_t)v[0].w << 32);
          a.count[g] = v[1].x;
          a.long_r[g] = v[1].y;
          a.cerr[g] = v[1].z;
          a.long_done[g] = 0;  // its long records (if any) are queued again by k_long_enqueue
          if (v[1].x & kCountRegular) ((u32x4*)a.desc)[g] = v[2];
        }
        run_first = tn;
      }
    }
#ifdef CASK_STAMPS
    const uint64_t st_end_ = __builtin_amdgcn_s_memtime();
#endif
    known = known && tn == t + 1;  // a new run searches
    BAR();
#ifdef CASK_STAMPS
    dg.st[6] += __builtin_amdgcn_s_memtime() - st_end_;  // phase 6: end-of-chunk barrier
#endif
    par ^= 1;
    if (!more) break;
    t = tn;
    run_end = next_end;
    cur = nxt;
  }
  flush_rows<G>(L, par ^ 1, pf_slots, pf_n);  // the last chunk's rows (visible: the loop ended on a barrier)
#ifdef CASK_STAMPS
  dg.st[7] = __builtin_amdgcn_s_memtime() - dg.st[7];
  if (a.stamps && threadIdx.x == 0) {
    const uint64_t rt = __builtin_amdgcn_s_memrealtime() - rt0_;
    atomicAdd(&a.stamps[11], (unsigned long long)rt);
    atomicMax(&a.stamps[12], (unsigned long long)rt);
    atomicAdd(&a.stamps[13], 1ull);
  }
  if (a.stamps && threadIdx.x == 0) atomicAdd(&a.stamps[7], (unsigned long long)dg.st[7]);
  if (a.stamps && threadIdx.x == 0)
    for (int i = 0; i < 10; ++i)
      if (i != 7) atomicAdd(&a.stamps[i], (unsigned long long)dg.st[i]);
#endif
}

// Geometry 0 (wide halo): a record of up to ~4 KiB that starts in the chunk is still hashed out of
// LDS. Geometry 3 (short halo, nontemporal staging): 11 instead of 12 loads per loader thread (3 %
// of halo instead of 12.5 %), picked when the records at the file heads are short (kShortHaloMean);
// a longer record that crosses the window's end goes to k_long like any other (correct either way).
using GeoA = Geo<32768, 4080, 256, 4>;
using GeoB = Geo<16384, 2032, 128, 8>;
using GeoC = Geo<8192, 1008, 64, 16>;
using GeoS = Geo<32768, 1008, 256, 4, true>;

static inline hipStream_t S(void* s) { return (hipStream_t)s; }

uint32_t geometry_chunk(int geo) {
  return geo == 1 ? GeoB::kCh : geo == 2 ? GeoC::kCh : geo == 3 ? GeoS::kCh : GeoA::kCh;
}
uint32_t geometry_halo(int geo) {
  return geo == 1 ? GeoB::kHaloB : geo == 2 ? GeoC::kHaloB : geo == 3 ? GeoS::kHaloB : GeoA::kHaloB;
}

template <class G>
static void launch_geo(const ScanArgs& a, void* stream) {
  const int cus = device_cus();
  // CASK_WG_PER_CU (diagnostic): fewer resident workgroups per CU than the LDS allows
  static const uint32_t per_cu = cask_knobs::tune("CASK_WG_PER_CU") ? (uint32_t)atoi(cask_knobs::tune("CASK_WG_PER_CU")) : G::kPerCU;
  uint64_t grid = (uint64_t)cus * per_cu;
  grid = (grid + 7) & ~7ull;
  const uint64_t need = (a.total_chunks + 7) & ~7ull;  // never more workgroups than chunks
  if (need < grid) grid = need;
  // CASK_LDS_PAD (diagnostic): extra dynamic LDS per workgroup, to lower workgroups per CU
  static const uint32_t pad = cask_knobs::tune("CASK_LDS_PAD") ? (uint32_t)atoi(cask_knobs::tune("CASK_LDS_PAD")) : 0u;
  // a.ctr->run_next is zero: every launch follows a fresh call block or the repair path's reset
  if (a.exact)
    hipLaunchKernelGGL((k_scan_chunks<G, true>), dim3((uint32_t)grid), dim3(G::kNT), pad, S(stream), a, a.files);
  else
    hipLaunchKernelGGL((k_scan_chunks<G, false>), dim3((uint32_t)grid), dim3(G::kNT), pad, S(stream), a, a.files);
}

void launch_scan_chunks(const ScanArgs& a, int geo, void* stream) {
  if (!a.total_chunks) return;
  if (geo == 1)
    launch_geo<GeoB>(a, stream);
  else if (geo == 2)
    launch_geo<GeoC>(a, stream);
  else if (geo == 3)
    launch_geo<GeoS>(a, stream);
  else
    launch_geo<GeoA>(a, stream);
}

}  // namespace cask_dev
