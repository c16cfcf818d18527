// The header chase of walk mode (Entries::next, log.rs:403-429): a lane follows a run's record
// chain header to header and writes the slot rows and chunk table. Shared by k_walk_chase
// (k_walk_hash.hip) and k_walk_find (k_walk.hip, the search and chase in one kernel).
#pragma once
#include "device_util.h"

namespace cask_dev {
namespace {

typedef __attribute__((address_space(1))) uint32_t g_u32;
typedef __attribute__((address_space(1))) uint64_t g_u64;
typedef __attribute__((address_space(1))) u32x4 g_u32x4;

constexpr uint32_t kNoChunk = 0xFFFFFFFFu;

// The piece of a run inside one file: chunks [t0, t0 + nch) of the file at `data`.
struct WSeg {
  const uint8_t* data;
  uint64_t len;
  int64_t sl;      // the highest file offset a 16-B load may start at: such a load stays within the
                   // 16-B granules that hold the file's bytes (sl < 0 for a file inside one granule)
  uint64_t b0, b1; // the segment's file bytes
  uint64_t t0;     // global index of its first chunk
  uint32_t nch;
};

// One chunk's table entries. A chunk with more records than its slot rows (a.slot_cap: small in a
// walk-mode call) keeps slot_cap of them and flags the call, which the host then redoes with full
// slot rows: every later kernel reads rows r < count only, so nothing reads past the slots.
__device__ __forceinline__ void put_chunk(const ScanArgs& a, uint64_t t, uint64_t spec, uint64_t ex, uint32_t count,
                                          uint32_t cerr) {
  if (count > a.slot_cap) {
    a.ctr->slot_overflow = 1u;
    count = a.slot_cap;
  }
  ((g_u64*)a.spec)[t] = spec;
  ((g_u64*)a.exit)[t] = ex;
  ((g_u32*)a.count)[t] = count;
  ((g_u32*)a.long_r)[t] = 0xFFFFFFFFu;  // every record is hashed here: nothing left for k_long
  ((g_u32*)a.cerr)[t] = cerr;
}

// A quad's walk state (every field the same in the quad's four lanes).
struct Walk {
  WSeg S;
  uint64_t run_end;  // the run's end chunk (global)
  // chunk state of the segment
  uint32_t cj, cn, ccerr;
  uint64_t cspec;
};

// The chain enters the record at `pos`: close the chunks it leaves, open its chunk; returns the
// record's row within its chunk (and the chunk in *j).
__device__ __forceinline__ uint32_t open_record(const ScanArgs& a, Walk& W, uint64_t pos, uint32_t csh, bool writer,
                                                uint32_t* jout) {
  const uint32_t j = (uint32_t)((pos - W.S.b0) >> csh);
  if (j != W.cj) {
    if (W.cj != kNoChunk && writer) put_chunk(a, W.S.t0 + W.cj, W.cspec, pos, W.cn, W.ccerr);
    for (uint32_t k = W.cj == kNoChunk ? 0u : W.cj + 1; k < j; ++k)
      if (writer) put_chunk(a, W.S.t0 + k, kNone, 0ull, 0u, 0xFFFFFFFFu);
    W.cj = j;
    W.cn = 0;
    W.ccerr = 0xFFFFFFFFu;
    W.cspec = pos;
  }
  *jout = j;
  return W.cn++;
}

// The segment ends: the chain leaves it at `ex` (kTerm after an EOF row).
__device__ __forceinline__ void close_segment(const ScanArgs& a, Walk& W, uint64_t ex, bool writer) {
  uint32_t k0 = 0;
  if (W.cj != kNoChunk) {
    if (writer) put_chunk(a, W.S.t0 + W.cj, W.cspec, ex, W.cn, W.ccerr);
    k0 = W.cj + 1;
  }
  for (uint32_t k = k0; k < W.S.nch; ++k)
    if (writer) put_chunk(a, W.S.t0 + k, kNone, 0ull, 0u, 0xFFFFFFFFu);
  W.cj = kNoChunk;
}

// The segment of chunks [t, min(file end, W.run_end)) of the file holding chunk t.
__device__ __forceinline__ void seg_setup(const ScanArgs& a, const FileDesc* files, Walk& W, uint64_t t) {
  const uint32_t fi = find_file(files, a.nfiles, t);
  const FileDesc fd = files[fi];
  const uint64_t fend = fd.first_chunk + fd.nchunks;
  const uint64_t se = fend < W.run_end ? fend : W.run_end;
  W.S.data = fd.data;
  W.S.len = fd.len;
  const uintptr_t end16 = ((uintptr_t)(fd.data + fd.len) + 15) & ~(uintptr_t)15;
  W.S.sl = (int64_t)(end16 - (uintptr_t)fd.data) - 16;
  W.S.b0 = (t - fd.first_chunk) * (uint64_t)a.chunk;
  const uint64_t e = (se - fd.first_chunk) * (uint64_t)a.chunk;
  W.S.b1 = e < fd.len ? e : fd.len;
  W.S.t0 = t;
  W.S.nch = (uint32_t)(se - t);
  W.cj = kNoChunk;
}

// ---------------------------------------------------------------------------------------------
// The chase (k_walk_chase; k_walk_find): one lane per run of a.run chunks walks the record chain
// from the run's speculative start (walk_search_sw) reading only each record's 18-B header
// (Entries::next, log.rs:403-429: each record starts where the previous one ends), and writes what
// k_walk_runs would: slot rows (without the checksum verdict: k_run_hash adds it), the chunk table
// (spec, exit, count, cerr, long_r = none) and, per chunk, the address of its first byte and of its
// file's end (cdesc). A record cut short by the end of its file is its UnexpectedEof row (data.rs:163,
// 172, 181) and ends the chain.
// ---------------------------------------------------------------------------------------------
// Chunks [tb, te) of one run (te <= the run's end): the chain enters the range's first segment at
// p_in (ignored when the segment starts a file: the chain starts there at 0); returns the position
// it leaves the range at (kTerm once an EOF row ended it, kNone if it never had a start). Chasing a
// run as [t0, tm) and then [tm, t1) from the first range's exit writes exactly what one range
// [t0, t1) writes: the chain is one walk either way.
//
// A run among the last a.hash_ntail (k_run_hash's tail runs) also marks, per piece of it
// (kTailSplit per run), which of the piece's records are at least kTailLong bytes long: bit i of
// the piece's kTailBitWords words in a.tbits, record i counted from the piece's first chunk.
struct TailBits {
  bool on = false;
  uint64_t r0 = 0, unit0 = 0;  // the run's first chunk, its first piece
  uint64_t qr = 1;             // chunks per piece
  uint64_t q = ~0ull;          // the piece being marked
  uint32_t i = 0, word = 0;    // its next record, the bits of its current word
  __device__ __forceinline__ void flush(const ScanArgs& a) {
    if (q != ~0ull && (i & 31) && i <= kTailMaxRecs) a.tbits[(unit0 + q) * kTailBitWords + ((i - 1) >> 5)] = word;
  }
  __device__ __forceinline__ void record(const ScanArgs& a, uint64_t t, bool longr) {
    const uint64_t qq = (t - r0) / qr;
    if (qq != q) {
      flush(a);
      q = qq;
      i = 0;
      word = 0;
    }
    word |= (longr ? 1u : 0u) << (i & 31);
    ++i;
    if (!(i & 31)) {
      if (i <= kTailMaxRecs) a.tbits[(unit0 + q) * kTailBitWords + ((i - 1) >> 5)] = word;
      word = 0;
    }
  }
};

__device__ uint64_t chase_range(const ScanArgs& a, const FileDesc* __restrict__ files, uint64_t tb, uint64_t te,
                                uint64_t p_in) {
  const uint32_t csh = (uint32_t)__builtin_ctz(a.chunk);
  g_u32* slots = (g_u32*)a.slots;
  g_u64* cd = (g_u64*)a.cdesc;
  TailBits tbt;
  {
    const uint64_t R = a.run, nruns = (a.total_chunks + R - 1) / R, k = tb / R;
    if (a.hash_ntail && k >= nruns - a.hash_ntail) {
      tbt.on = true;
      tbt.r0 = k * R;
      tbt.qr = (R + kTailSplit - 1) / kTailSplit;
      tbt.unit0 = (k - (nruns - a.hash_ntail)) * kTailSplit;
    }
  }
  Walk W;
  W.cn = 0;
  W.ccerr = 0xFFFFFFFFu;
  W.cspec = 0;
  W.run_end = te;
  uint64_t p = p_in;
  bool term = false;
  for (uint64_t t = tb; t < te;) {
    seg_setup(a, files, W, t);
    t = W.S.t0 + W.S.nch;
    const uint64_t fend = (uint64_t)(uintptr_t)(W.S.data + W.S.len);
    for (uint32_t c = 0; c < W.S.nch; ++c) {
      cd[2 * (W.S.t0 + c)] = (uint64_t)(uintptr_t)(W.S.data + W.S.b0 + ((uint64_t)c << csh));
      cd[2 * (W.S.t0 + c) + 1] = fend;
    }
    // the range's first segment starts at p_in; a later one starts a file (b0 == 0)
    if (W.S.b0 == 0) p = 0ull;
    else if (W.S.t0 != tb) p = kNone;  // (unreachable: a later segment starts a file)
    term = false;
    // The next record's header is loaded before this record's stores go out: a wait for a load
    // also waits for every store issued before it (one vmcnt counts both), so loading after the
    // stores would cost each hop a store round trip as well. Headers past the file's end are not
    // read (an address inside the file is loaded instead).
    const bool has = p != kNone && p < W.S.b1;
    // one 16-B load per hop, of header bytes 2..17 (seq, key size, value size; the checksum's first
    // two bytes are not needed)
    const uint64_t p0 = has && p + 18 <= W.S.len ? p + 2 : 0ull;
    u32x4 h = gld16g((const g_u8*)(W.S.data + p0));
    asm volatile("" ::"v"(h.x), "v"(h.y), "v"(h.z), "v"(h.w));
    while (p != kNone && p < W.S.b1) {
      uint32_t j = 0;
      if (p + 18 > W.S.len) {  // header cut short: Io(UnexpectedEof) (data.rs:163)
        const uint32_t r = open_record(a, W, p, csh, true, &j);
        if (tbt.on) tbt.record(a, W.S.t0 + j, false);
        const uint32_t off = (uint32_t)(p - W.S.b0 - ((uint64_t)j << csh));
        if (r < a.slot_cap) *(g_u32x4*)(slots + ((W.S.t0 + j) * (uint64_t)a.slot_cap + r) * 4) = u32x4{0u, 0u, 0u, off << 16};
        if (r < W.ccerr) W.ccerr = r;
        term = true;
        break;
      }
      const uint32_t ksz = h.z >> 16, vsz = h.w;
      const u32x4 row = u32x4{fun(h.x, h.y, 2), fun(h.y, h.z, 2), vsz, ksz};
      const uint64_t rl = 18ull + ksz + (vsz == 0xFFFFFFFFu ? 0ull : (uint64_t)vsz);
      const uint64_t pn = p + rl;
      const uint64_t pl = pn + 18 <= W.S.len ? pn + 2 : 0ull;  // (pn < p: rl wrapped, impossible)
      h = gld16g((const g_u8*)(W.S.data + pl));
      const uint32_t r = open_record(a, W, p, csh, true, &j);
      if (tbt.on) tbt.record(a, W.S.t0 + j, rl >= kTailLong);
      const uint32_t off = (uint32_t)(p - W.S.b0 - ((uint64_t)j << csh));
      if (r < a.slot_cap)
        *(g_u32x4*)(slots + ((W.S.t0 + j) * (uint64_t)a.slot_cap + r) * 4) = u32x4{row.x, row.y, row.z, row.w | (off << 16)};
      if (pn > W.S.len) {  // key or value cut short (data.rs:172,181)
        if (r < W.ccerr) W.ccerr = r;
        term = true;
        break;
      }
      p = pn;
    }
    close_segment(a, W, term ? kTerm : p, true);
    if (term) p = kTerm;
  }
  if (tbt.on) tbt.flush(a);
  return p;
}

// The chunk range of walk run i (an index into a.wruns, or the run itself): [t0, t1).
__device__ __forceinline__ void walk_run_chunks(const ScanArgs& a, uint64_t i, uint64_t* t0, uint64_t* t1) {
  const uint64_t R = a.run;
  const uint64_t k = a.wruns ? a.wruns[i] : i;
  *t0 = k * R;
  *t1 = k * R + R < a.total_chunks ? k * R + R : a.total_chunks;
}

}  // namespace
}  // namespace cask_dev
