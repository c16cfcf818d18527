// Walk mode, gfx950 (the scan of logs of long records): every log byte read once, by the quad of
// lanes that hashes its record.
//
//   k_walk_search (k_walk.hip)  each run of a.run chunks gets a speculative first record start
//   k_walk_chase                one lane per run follows the record chain header to header
//                               (Entries::next, log.rs:403-429) and writes slot rows + chunk table
//   k_run_hash                  Entry::from_read's checksum (data.rs:185-198) of every record the
//                               chase found, a quad of lanes per record, straight from HBM
//   k_finish (k_pipeline.hip)   validates the speculated starts (spec[c] == T[c]) and writes rows
//
// Why a quad per record: XXH32's four stripe accumulators are the only parallelism inside a record
// (one lane each); a log of long records needs thousands of records in flight at once to keep HBM
// busy. Why split the chase from the hash: the chase is a chain of dependent 18-B loads (latency
// bound, ~0.5 ms for configs[2]) and the hash a stream (HBM bound); in one kernel (a quad per run
// chasing and hashing, round 3's first walk) each quad's stream stalled on its own header chain.
//
// Output: the chunk table and slot rows of k_scan_chunks (spec, exit, count, cerr, long_r = none,
// slot rows with the checksum verdict), so k_finish and the repair path run unchanged.
#include "device_util.h"

#include <stdlib.h>
#include "knobs.h"

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

// The 16 bytes of v from byte s on (s in 0..15), zero-filled past the end.
__device__ __forceinline__ u32x4 shr_bytes(const u32x4& v, uint32_t s) {
  const uint32_t k = s >> 2, b = s & 3;
  const uint32_t w0 = k == 0 ? v.x : k == 1 ? v.y : k == 2 ? v.z : v.w;
  const uint32_t w1 = k == 0 ? v.y : k == 1 ? v.z : k == 2 ? v.w : 0u;
  const uint32_t w2 = k == 0 ? v.z : k == 1 ? v.w : 0u;
  const uint32_t w3 = k == 0 ? v.w : 0u;
  return u32x4{fun(w0, w1, b), fun(w1, w2, b), fun(w2, w3, b), fun(w3, 0u, b)};
}

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

}  // namespace

// ---------------------------------------------------------------------------------------------
// Split path, pass 1 — k_walk_chase: one lane per run of a.run chunks walks the record chain from
// the run's speculative start (k_walk_search) reading only each record's 18-B header
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

// A run among the last a.hash_ntail (k_run_hash's tail runs) also marks, per piece of it
// (kTailSplit per run), which of the piece's records are at least kTailLong bytes long: bit i of the
// piece's kTailBitWords words in a.tbits, record i counted from the piece's first chunk.
struct TailBits {
  bool on = false;
  uint64_t r0 = 0, unit0 = 0;  // the run's first chunk, its first piece
  uint64_t qr = 1;             // chunks per piece
  uint64_t q = ~0ull;          // the piece being marked
  uint64_t qe = 0;             // the first chunk after it (the chain only moves forward)
  uint32_t i = 0, word = 0;    // its next record, the bits of its current word
  __device__ __forceinline__ void flush(const ScanArgs& a) {
    if (q != ~0ull && (i & 31) && i <= kTailMaxRecs) a.tbits[(unit0 + q) * kTailBitWords + ((i - 1) >> 5)] = word;
  }
  __device__ __forceinline__ void record(const ScanArgs& a, uint64_t t, bool longr) {
    if (t >= qe) {  // (a division per piece, not per record)
      flush(a);
      q = (uint32_t)(t - r0) / (uint32_t)qr;
      qe = r0 + (q + 1) * qr;
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

__global__ __launch_bounds__(256) void k_walk_chase(ScanArgs a, const FileDesc* __restrict__ files) {
  const uint64_t R = a.run;
  const uint64_t nruns = a.wruns ? a.nwruns : (a.total_chunks + R - 1) / R;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < nruns; i += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t t0, t1;
    walk_run_chunks(a, i, &t0, &t1);
    (void)chase_range(a, files, t0, t1, a.walk_pre ? a.tin[t0] : kNone);
  }
}

// ---------------------------------------------------------------------------------------------
// Split path, pass 2 — k_run_hash: Entry::from_read's checksum (data.rs:185-198) of every record the
// chase found. A wave claims runs and hands their records, in order, to its 16 quads: a quad hashes
// its record straight from HBM, and takes the next record of the wave's stream as it starts one (its
// slot row and chunk address are loaded one iteration ahead). A failed record gets the bad bit in its
// slot row and lowers its chunk's first failing row (cerr), which k_finish reads. The wave's stream
// runs on from one claimed run to the next (the next run's row counts are loaded one iteration
// before they are needed), so no quad waits for a run's last record.
//
// Loads: whole 128-B lines per instruction, nontemporal. The quads are pairs across the two halves
// of the wave (quad j of lanes 0..31 with quad j of lanes 32..63). A round of a record is its lines
// [La + 1 KiB i, La + 1 KiB (i + 1)) (La: the line of the body's first byte), so no line is read by
// two rounds of one record. Instruction 2m loads line m of the lower quad's round, 2m + 1 line m of
// the upper quad's, the lower half of the wave a line's first 64 B and the upper half its second:
// every instruction reads whole lines — nontemporal loads then fetch each line once (a quad's 64 B
// per instruction fetched a line twice under that policy, and rounds starting mid-line fetched the
// line at each round boundary twice under the default one: 1.11x the log bytes) — and one
// v_permlane32_swap per dword hands each half its own line. A body dword is funneled out of two line
// dwords at the body's byte offset (v_alignbyte; the lower one from the previous lane by DPP, lane
// 0's carried from the previous block), quad_transpose_dpp gives lane q its dword position's words,
// and the words outside the record's full stripes are masked; lane q keeps the stripe accumulator of
// its dword position ((q - cM - 1) mod 4).
//
// The pipeline: iteration i issues round i (2 x 8 line loads, the record's last partial stripe, the
// stored checksum of a record's first round) and then mixes round i - 1. Every quad issues every
// one of those loads (past a round's last line a quad reads that line again; a quad with nothing to
// load reads one safe line), and the two rounds live in two register sets used in turn (the loop
// body twice, no copies), so the compiler's counted waits wait for round i - 1 only and round i
// stays in flight while it is mixed. The loads whose results the next iteration's bookkeeping needs
// (slot rows, chunk addresses, the next run's counts) are issued before the round's.
// ---------------------------------------------------------------------------------------------
// v_permlane32_swap: lanes 32..63 of a trade places with lanes 0..31 of b — afterwards a holds the
// lower halves of both, b the upper halves
__device__ __forceinline__ void swap32(uint32_t& a, uint32_t& b) {
  const auto r = __builtin_amdgcn_permlane32_swap(a, b, false, false);
  a = r[0];
  b = r[1];
}
__device__ __forceinline__ void swap32(u32x4& a, u32x4& b) {
  const auto x = __builtin_amdgcn_permlane32_swap(a.x, b.x, false, false);
  const auto y = __builtin_amdgcn_permlane32_swap(a.y, b.y, false, false);
  const auto z = __builtin_amdgcn_permlane32_swap(a.z, b.z, false, false);
  const auto w = __builtin_amdgcn_permlane32_swap(a.w, b.w, false, false);
  a = u32x4{x[0], y[0], z[0], w[0]};
  b = u32x4{x[1], y[1], z[1], w[1]};
}
__device__ __forceinline__ u32x4 gld16nt(uint64_t p) {
  typedef __attribute__((address_space(1))) const u32x4 gcu32x4;
  return __builtin_nontemporal_load((gcu32x4*)(uintptr_t)p);
}

__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void k_run_hash(ScanArgs a) {
  constexpr uint32_t D = 8;    // lines of a record per round
  constexpr uint32_t RW = 256; // dwords per round
  constexpr uint32_t RT = kMaxRun + 1;
  __shared__ uint32_t s_pf[4][2][RT];
  __shared__ uint64_t s_cd[4][2][2 * kMaxRun];
  __shared__ uint32_t s_fq[4][64][12];  // per wave: records whose checksums are to be finished
  __shared__ uint16_t s_tl[4][2][kTailMaxRecs];  // per wave, two units: a tail piece's pass's records
  const uint32_t lane = threadIdx.x & 63, q = lane & 3, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), h = lane >> 5;
  const bool qlead = q == 0;
  const uint64_t R = a.run;
  const uint64_t nruns = a.wruns ? a.nwruns : (a.total_chunks + R - 1) / R;
  g_u32* slots = (g_u32*)a.slots;
  const g_u64* cd = (const g_u64*)a.cdesc;
  uint32_t* pfA = s_pf[wv][0];
  uint32_t* pfB = s_pf[wv][1];
  uint64_t* cdA = s_cd[wv][0];
  uint64_t* cdB = s_cd[wv][1];
  uint16_t* tlA = s_tl[wv][0];  // a tail piece's pass: its records in that pass
  uint16_t* tlB = s_tl[wv][1];
  bool flA = false, flB = false;  // the unit's records are handed out through its list
  const unsigned long long qmask = 0x1111111111111111ull;
  const uint64_t safe = (uint64_t)(uintptr_t)a.cdesc;  // (a 128-B aligned allocation: its first line)

  // The wave's record stream (uniform): two runs, A (records are handed out from it, at cursor
  // cur) and B (the next one, once loaded: fullB), each as its first chunk, chunk count and row
  // count. B is refilled from the claim counter as soon as it is free. (Plain variables, not arrays
  // indexed by the slot: those go to scratch memory, whose loads wait for every load.) Units of
  // work: the runs in order, except that the tail runs (a.hash_ntail: two grids' worth; else one) are
  // handed out in kTailSplit pieces, each twice with a.hash_ntail (long records, then short ones), so
  // that the waves run dry close together (A/B in DESIGN §4 and profiles/r05_hash_lines_ab.txt).
  uint64_t rtA = 0, rtB = 0;
  uint32_t rnA = 0, rnB = 0, rchA = 0, rchB = 0;
  bool fullB = false;
  uint32_t cur = 0;
  bool runs_left = true;
  auto run_start = [&](uint64_t k) __attribute__((always_inline)) { return (a.wruns ? a.wruns[k] : k) * R; };
  constexpr uint64_t TS = kTailSplit;
  // With a.hash_ntail (walk mode over data files): the last hash_ntail runs' pieces are each handed
  // out twice, through a list of their records: the records of at least kTailLong bytes right after
  // the other runs (units [nhead, nhead + NT)), the shorter ones last — so that no long record is
  // still being hashed when the units run out
  const bool split = a.hash_ntail != 0;
  const uint64_t tcap = (uint64_t)gridDim.x * 4;
  const uint64_t ntail = split ? a.hash_ntail : nruns < tcap ? nruns : tcap;
  const uint64_t nhead = nruns - ntail, NT = TS * ntail, nunits = nhead + (split ? 2 * NT : NT);
  auto load_run = [&](bool intoA, uint64_t u) __attribute__((always_inline)) -> bool {
    if (u >= nunits) return false;
    // pass: 0 a whole head run or (no split) a tail piece, 1 a tail piece's long records, 2 its others
    const bool tl = u >= nhead;
    const uint64_t piece = tl ? (u - nhead) % NT : 0ull;
    const uint32_t pass = split && tl ? (u - nhead < NT ? 1u : 2u) : 0u;
    const uint64_t k = tl ? nhead + piece / TS : u;
    const uint64_t tr = run_start(k);
    const uint64_t nk = a.total_chunks - tr < R ? a.total_chunks - tr : R;
    const uint64_t qr = (R + TS - 1) / TS, c0 = tl ? (piece % TS) * qr : 0ull;
    const uint64_t c1 = tl ? (c0 + qr < nk ? c0 + qr : nk) : nk;
    const uint64_t t0 = tr + c0;
    const uint32_t nch = (uint32_t)(c1 > c0 ? c1 - c0 : 0ull);
    uint32_t inc = lane < nch ? (((const g_u32*)a.count)[t0 + lane] & kCountMask) : 0u;
    // (the piece's long-record bits, loaded with the counts: one round trip)
    const uint32_t bits = pass && lane < kTailBitWords ? ((const g_u32*)a.tbits)[piece * kTailBitWords + lane] : 0u;
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t u = __shfl_up(inc, o, 64);
      if ((int)lane >= o) inc += u;
    }
    uint32_t* pf = intoA ? pfA : pfB;
    if (lane < nch) pf[lane + 1] = inc;
    if (lane == 0) pf[0] = 0;
    uint64_t* cdt = intoA ? cdA : cdB;
    if (lane < nch) {
      cdt[2 * lane] = cd[2 * (t0 + lane)];
      cdt[2 * lane + 1] = cd[2 * (t0 + lane) + 1];
    }
    uint32_t n = __builtin_amdgcn_readfirstlane((uint32_t)__shfl((int)inc, 63, 64));
    if (pass) {  // the pass's records, in order, into the unit's list
      const uint32_t nb = 32 * lane;
      const uint32_t valid = lane >= kTailBitWords || nb >= n ? 0u : n - nb >= 32 ? ~0u : (1u << (n - nb)) - 1u;
      uint32_t w = (pass == 1 ? bits : ~bits) & valid;
      const uint32_t c = (uint32_t)__builtin_popcount(w);
      uint32_t pre = c;
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t t = __shfl_up(pre, o, 64);
        if ((int)lane >= o) pre += t;
      }
      uint16_t* lst = intoA ? tlA : tlB;
      uint32_t at = pre - c;
      while (w) {
        const uint32_t b = (uint32_t)__builtin_ctz(w);
        w &= w - 1;
        lst[at++] = (uint16_t)(nb + b);
      }
      n = __builtin_amdgcn_readfirstlane((uint32_t)__shfl((int)pre, 63, 64));
    }
    if (intoA) {
      rtA = t0;
      rchA = nch;
      rnA = n;
      flA = pass != 0;
    } else {
      rtB = t0;
      rchB = nch;
      rnB = n;
      flB = pass != 0;
    }
    return true;
  };
  runs_left = load_run(true, blockIdx.x * 4ull + wv);

  // a quad's current record (cv) and the round of it in hand: round cri of its cnrd rounds, rfin if
  // it is the last (the record's tail bytes in T), head if it is the first (its stored checksum in
  // x). The body (data.rs:185-198: everything after the stored checksum) starts at cb, chl bytes;
  // line dword t (t = 0 at cb & ~127) funneled at byte csb is body dword t - cM - 1 (cM: the dword of
  // cb in its line); ctl: the last dword a full stripe uses. tclamp: the tail's 16 bytes were loaded
  // from the file's last granule instead (shifted by ctsh).
  bool cv = false, rfin = false, head = false, tclamp = false;
  uint64_t cb = 0, cend = 0, ct_t = 0;
  uint32_t chl = 0, cM = 0, csb = 0, ctl = 0, cnrd = 0, cri = 0, ctsh = 0;
  uint32_t v = 0, carry = 0, mrot = 1, cstored = 0, ct_r = 0, cw3 = 0;
  uint32_t ns = 0;
  uint64_t nt = 0;
  uint32_t nr = 0;
  u32x4 nrow = u32x4{0u, 0u, 0u, 0u};
  uint64_t ncb = 0, nce = 0;
  uint64_t carow = safe;
  u32x4 XA[2 * D], XB[2 * D], TA = u32x4{0u, 0u, 0u, 0u}, TB = u32x4{0u, 0u, 0u, 0u};
  uint32_t sA = 0, sB = 0;
#pragma unroll
  for (uint32_t d = 0; d < 2 * D; ++d) XA[d] = XB[d] = u32x4{0u, 0u, 0u, 0u};
  // the queued checksums (s_fq): lane i finishes record i (merged accumulators + length, tail bytes,
  // their count, the stored checksum, where its slot row is) and marks a mismatch
  uint32_t fq_n = 0;  // (uniform)
  auto fq_flush = [&]() __attribute__((always_inline)) {
    if (lane < fq_n) {
      const uint32_t* e = s_fq[wv][lane];
      uint32_t hh = e[0];
      const u32x4 tw = u32x4{e[1], e[2], e[3], e[4]};
      const uint32_t tb = e[5], n4 = tb >> 2, n1 = tb & 3;
      hh = n4 > 0 ? tail4(hh, tw.x) : hh;
      hh = n4 > 1 ? tail4(hh, tw.y) : hh;
      hh = n4 > 2 ? tail4(hh, tw.z) : hh;
      const uint32_t lw = n4 == 0 ? tw.x : n4 == 1 ? tw.y : n4 == 2 ? tw.z : tw.w;
      hh = n1 > 0 ? tail1(hh, lw & 0xFFu) : hh;
      hh = n1 > 1 ? tail1(hh, (lw >> 8) & 0xFFu) : hh;
      hh = n1 > 2 ? tail1(hh, (lw >> 16) & 0xFFu) : hh;
      hh = avalanche(hh);
      if (hh != e[6]) {  // InvalidChecksum{expected: stored, found: hh} (data.rs:193-198)
        const uint64_t t = (uint64_t)e[8] | ((uint64_t)e[9] << 32);
        const uint32_t r = e[7];
        slots[(t * (uint64_t)a.slot_cap + r) * 4 + 3] = e[10] | kSlotBad;
        atomicMin(&a.cerr[t], r);
      }
    }
  };
#ifdef CASK_STAMPS
  const uint64_t wid = blockIdx.x * 4ull + wv;
  if (a.stamps && lane == 0 && wid < kStampWaves) a.stamps[16 + 2 * wid] = __builtin_amdgcn_s_memrealtime();
#endif
  auto step = [&](u32x4 (&Xm)[2 * D], u32x4& Tm, uint32_t& xm, u32x4 (&Xi)[2 * D], u32x4& Ti, uint32_t& xi) __attribute__((always_inline)) -> bool {
    if (ns == 1) ns = 2;
    // the next unit is claimed once the current one has at most 16 records left to hand out (the
    // stream still never waits: B is loaded an iteration before it is needed), so that a wave holds
    // one unit's worth of records, not two, when the units run out (A/B: 0.5 % faster than claiming
    // as soon as B is free)
    if (runs_left && !fullB && rnA - cur <= 16) {
      const uint32_t old = atomicAdd(&a.ctr->hash_next, lane == 0 ? 1u : 0u);
      const bool got = load_run(false, (uint64_t)gridDim.x * 4ull + __builtin_amdgcn_readfirstlane(old));
      runs_left = got;
      fullB = got;
#ifdef CASK_STAMPS
      if (!got && a.stamps && lane == 0 && wid < kStampWaves) a.stamps[kStampDry + wid] = __builtin_amdgcn_s_memrealtime();
#endif
    }
    // ---- plan this quad's next round: the rest of its record, or the next record from its slot row
    // and its chunk's address (branch-free: every lane computes both and selects, so the counted
    // waits see one path)
    const bool cont = cv && !rfin;
    const bool promote = !cont && ns == 2;
    const uint32_t w3n = nrow.w, vszn = nrow.z;
    const uint64_t bn = ncb + ((w3n >> 16) & 0x7FFFu);
    const uint64_t en = nce;
    const uint64_t rln = 18ull + (w3n & 0xFFFFu) + (vszn == 0xFFFFFFFFu ? 0ull : (uint64_t)vszn);
    const bool round2 = cont || (promote && bn + rln <= en);
    const uint64_t b2 = cont ? cb : bn + 4, end2 = cont ? cend : en;
    const uint32_t hl2 = cont ? chl : (uint32_t)(rln - 4);
    const uint64_t la2 = b2 & ~127ull;
    const uint32_t M2 = cont ? cM : (uint32_t)((b2 - la2) >> 2), sb2 = cont ? csb : (uint32_t)(b2 & 3);
    const uint32_t ns2 = hl2 >> 4;  // full stripes
    const uint32_t tl2 = cont ? ctl : M2 + 4 * ns2;
    const uint32_t nrd2 = cont ? cnrd : (ns2 ? (tl2 >> 8) + 1 : 1u);
    const uint32_t ri2 = cont ? cri + 1 : 0u;
    const uint32_t nl2 = round2 && ns2 ? (((tl2 - RW * ri2) >> 5) + 1 < D ? ((tl2 - RW * ri2) >> 5) + 1 : D) : 0u;
    const bool fin2 = round2 && ri2 + 1 == nrd2;
    const uint64_t pt = nt;
    const uint32_t pr = nr, pw3 = w3n;
    ns = promote ? 0u : ns;
    // ---- the stream's next records to the quads that have none (in lane order; branch-free for
    // the lanes: every lane loads a slot row every iteration, the safe line when it takes none)
    const bool want = ns == 0;
    const unsigned long long wm = __ballot(qlead && want) & qmask;
    const uint32_t nw = (uint32_t)__builtin_popcountll(wm);
    const uint32_t l0 = lane & ~3u;
    const uint32_t myrank = (uint32_t)__builtin_popcountll(wm & (l0 ? (~0ull >> (64 - l0)) : 0ull));
    const uint32_t rem = rnA - cur;
    const bool up = myrank >= rem;
    const uint32_t idx = up ? myrank - rem : cur + myrank;
    const bool claimed = want && (up ? (fullB && idx < rnB) : true);
    const uint32_t* pf = up ? pfB : pfA;
    // the unit's idx-th record to hand out: itself, or its list's entry (a tail piece's pass)
    const uint16_t* tlc = up ? tlB : tlA;
    const uint32_t rec = (up ? flB : flA) ? (uint32_t)tlc[idx < kTailMaxRecs ? idx : 0u] : idx;
    uint32_t lo = 0, hi = up ? rchB : rchA;
#pragma unroll
    for (int it = 0; it < 6; ++it) {
      const uint32_t mid = (lo + hi) >> 1;
      const bool go = hi - lo > 1;
      const bool le = go && pf[mid] <= rec;
      lo = le ? mid : lo;
      hi = go && !le ? mid : hi;
    }
    const uint64_t ntc = (up ? rtB : rtA) + lo;
    const uint32_t nrc = rec - pf[lo];
    nt = claimed ? ntc : nt;
    nr = claimed ? nrc : nr;
    const uint64_t* cdt = up ? cdB : cdA;
    const uint64_t cbc = cdt[2 * lo], cec = cdt[2 * lo + 1];
    ncb = claimed ? cbc : ncb;
    nce = claimed ? cec : nce;
    carow = claimed ? (uint64_t)(uintptr_t)(slots + (ntc * (uint64_t)a.slot_cap + nrc) * 4) : promote ? safe : carow;
    uint64_t arow = carow;
    if (nw) {
      const uint32_t avail = rem + (fullB ? rnB : 0u);
      const uint32_t used = nw < avail ? nw : avail;
      if (used >= rem && fullB) {
        rtA = rtB;
        rnA = rnB;
        rchA = rchB;
        uint32_t* t = pfA;
        pfA = pfB;
        pfB = t;
        uint64_t* tc = cdA;
        cdA = cdB;
        cdB = tc;
        uint16_t* tt = tlA;
        tlA = tlB;
        tlB = tt;
        flA = flB;
        fullB = false;
        cur = used - rem;
      } else {
        cur += used;
      }
    }
    ns = claimed ? 1u : ns;
    // ---- issue the round: the record's tail (its last hl % 16 bytes, into T) and stored checksum
    // (first round) as plain loads, first, then the octet's 2 x D line loads (a line past the
    // round's last is that last line again: the same line, merged with its first request; a quad
    // with no lines reads the safe line)
    const uint64_t end16 = (end2 + 15) & ~15ull;
    const bool tail2 = round2 && fin2 && (hl2 & 15) != 0;
    const uint64_t tp = b2 + 16ull * ns2;
    const bool tclamp2 = tail2 && tp + 16 > end16;
    uint64_t ta = tail2 ? (tclamp2 ? end16 - 16 : tp) : safe;
    uint64_t sa = round2 && !cont ? b2 - 4 : safe;
    const uint64_t rb = la2 + 1024ull * ri2;
    // the pair's two rounds: quad j of the lower half (lanes 0..31) with quad j of the upper half;
    // a quad with no lines reads the safe line (as one line)
    const uint64_t rbq = nl2 ? rb : safe;
    const uint32_t nlq = nl2 ? nl2 - 1 : 0u;  // its last line
    uint32_t a0 = (uint32_t)rbq, a1 = a0, c0 = (uint32_t)(rbq >> 32), c1 = c0, n0 = nlq, n1 = nlq;
    swap32(a0, a1);  // a0: the lower quad's, a1: the upper quad's
    swap32(c0, c1);
    swap32(n0, n1);
    // this lane's 16 B of each line: the lower half of the wave reads a line's first 64 B, the upper
    // half its second (lanes j and j + 32 have the same q)
    const uint64_t lof = 64ull * h + 16ull * q;
    const uint64_t rb0 = (((uint64_t)c0 << 32) | a0) + lof, rb1 = (((uint64_t)c1 << 32) | a1) + lof;
    const uint32_t e0 = 128 * n0, e1 = 128 * n1;  // the last line's offset
    uint64_t ya[2 * D];
#pragma unroll
    for (uint32_t m = 0; m < D; ++m) {
      ya[2 * m] = rb0 + (uint64_t)(128 * m < e0 ? 128 * m : e0);
      ya[2 * m + 1] = rb1 + (uint64_t)(128 * m < e1 ? 128 * m : e1);
    }
    asm volatile("" : "+v"(arow), "+v"(sa), "+v"(ta));
#pragma unroll
    for (uint32_t d = 0; d < 2 * D; ++d) asm volatile("" : "+v"(ya[d]));
    {  // (the 8 bytes used: the dead half of a 16-B destination is a register the compiler reuses,
       // and writing it would wait for this load)
      const uint64_t zw = *(const g_u64*)(uintptr_t)(arow + 8);
      nrow = u32x4{0u, 0u, (uint32_t)zw, (uint32_t)(zw >> 32)};
    }
    Ti = gld16g((const g_u8*)(uintptr_t)ta);
    xi = gld4g((const g_u8*)(uintptr_t)sa);
#pragma unroll
    for (uint32_t d = 0; d < 2 * D; ++d) Xi[d] = gld16nt(ya[d]);
    // the round in hand is used from here on: nothing that reads it (the pair selects included) nor
    // the wait for it is scheduled above the loads
    asm volatile("" : "+v"(xm)::"memory");
#pragma unroll
    for (uint32_t d = 0; d < 2 * D; ++d) asm volatile("" : "+v"(Xm[d]));
    // ---- mix the round in hand (every lane: the swizzles need both quads of a pair). The elements
    // the record's full stripes use: dword t = 256 cri + 16 d + 4 k + q of its lines (lane q, block
    // d, word k after the transpose) for t in [cM + 1, ctl], i.e. e = 4 d + k in [e_lo, e_lo + span]
    // (e_lo <= 8: only the first elements of a first round can precede the first stripe)
    {
      const int32_t A = (int32_t)(cM + 1 - q) - (int32_t)(RW * cri), B = (int32_t)(ctl - q) - (int32_t)(RW * cri);
      int32_t e_lo = A <= 0 ? 0 : (A + 3) >> 2;
      int32_t e_hi = !cv || B < 0 ? -1 : (B >> 2 < 63 ? B >> 2 : 63);
      const bool none = e_hi < e_lo;  // (no element: both tests fail)
      e_lo = none ? 64 : e_lo;
      e_hi = none ? -1 : e_hi;
      const uint32_t span = (uint32_t)(e_hi - e_lo);
      const bool hi1 = e_hi & 1, hi2 = e_hi & 2;  // (e_hi % 4 = 3: that block is whole)
#pragma unroll
      for (uint32_t m = 0; m < D; ++m) {
        const u32x4 xa = Xm[2 * m], xb = Xm[2 * m + 1];
        // line m of the lower quad's round (its first 64 B in the lower half of the wave, its second
        // in the upper half) and of the upper quad's: after the swap each half holds its line
        u32x4 blk[2] = {xa, xb};
        swap32(blk[0], blk[1]);
#pragma unroll
        for (uint32_t e = 0; e < 2; ++e) {
          const uint32_t d = 2 * m + e;
          const u32x4 gg = blk[e];
          const uint32_t dv = (uint32_t)__builtin_amdgcn_mov_dpp((int)gg.w, 0x93, 0xF, 0xF, false);  // [3,0,1,2]
          const uint32_t p0 = q == 0 ? carry : dv;
          carry = dv;
          u32x4 x = u32x4{fun(p0, gg.x, csb), fun(gg.x, gg.y, csb), fun(gg.y, gg.z, csb), fun(gg.z, gg.w, csb)};
          quad_transpose_dpp(x);
          if (d < 2) {  // (a first round's first stripe can start in these: each word masked)
#pragma unroll
            for (uint32_t k = 0; k < 4; ++k) {
              const uint32_t el = 4 * d + k;
              const bool ok = (uint32_t)((int32_t)el - e_lo) <= span;
              uint32_t w = xround(v, x[k]);
              asm volatile("" : "+v"(w));
              v = ok ? w : v;
            }
          } else {  // the whole block, or its first e_hi % 4 + 1 words (the record's last full stripe's
                    // block), or none of it
            uint32_t w1 = xround(v, x.x), w2 = xround(w1, x.y), w3 = xround(w2, x.z), w4 = xround(w3, x.w);
            asm volatile("" : "+v"(w1), "+v"(w2), "+v"(w3), "+v"(w4));
            const uint32_t part = hi2 ? w3 : hi1 ? w2 : w1;
            const int32_t e0 = (int32_t)(4 * d);
            v = e0 + 3 <= e_hi ? w4 : e0 <= e_hi ? part : v;
          }
        }
      }
    }
    if (cv && head) cstored = xm;
    // ---- a record that ends with this round: its stripe accumulators merged in the quad, the rest of
    // its checksum (data.rs:185-198: length, tail bytes, avalanche, the compare) queued per wave and
    // finished up to 64 at once, a record per lane (a few of the 16 quads finish a record in an
    // iteration, and per quad every lane of the wave would run those steps every iteration)
    const bool fin_now = cv && rfin;
    const unsigned long long fm = __ballot(fin_now && qlead) & qmask;
    if (fm) {
      uint32_t m = rotl_var(v, mrot);
      m += quad_xor1(m);
      m += quad_xor2(m);
      u32x4 tw = Tm;
      if (__any(fin_now && tclamp)) tw = shr_bytes(Tm, tclamp ? ctsh : 0u);  // (rare: the file ends in the tail's 16 B)
      if (fin_now && qlead) {
        uint32_t* e = s_fq[wv][fq_n + (uint32_t)__builtin_popcountll(fm & (lane ? (~0ull >> (64 - lane)) : 0ull))];
        e[0] = (chl >= 16 ? m : P5) + chl;
        e[1] = tw.x;
        e[2] = tw.y;
        e[3] = tw.z;
        e[4] = tw.w;
        e[5] = chl & 15;
        e[6] = cstored;
        e[7] = ct_r;
        e[8] = (uint32_t)ct_t;
        e[9] = (uint32_t)(ct_t >> 32);
        e[10] = cw3;
      }
      fq_n += (uint32_t)__builtin_popcountll(fm);
      if (fq_n > 64 - 16) {
        fq_flush();
        fq_n = 0;
      }
    }
    // ---- state for the next iteration
    if (cont) {
      cri = ri2;
      rfin = fin2;
      tclamp = tclamp2;
      ctsh = (uint32_t)(tp - (end16 - 16));
      head = false;
    } else {
      cv = promote && round2;
      cb = b2;
      cend = end2;
      chl = hl2;
      cM = M2;
      csb = sb2;
      ctl = tl2;
      cnrd = nrd2;
      cri = 0;
      rfin = fin2;
      tclamp = tclamp2;
      ctsh = (uint32_t)(tp - (end16 - 16));
      head = true;
      // lane q holds the words of stripe accumulator j = w mod 4 = (q - cM - 1) mod 4
      const uint32_t j = (q - M2 - 1) & 3;
      v = j == 0 ? P1 + P2 : j == 1 ? P2 : j == 2 ? 0u : 0u - P1;
      mrot = j == 0 ? 1u : j == 1 ? 7u : j == 2 ? 12u : 18u;
      ct_t = pt;
      ct_r = pr;
      cw3 = pw3;
    }
    const bool stream_left = rnA != cur || (fullB && rnB != 0) || runs_left;
    return __builtin_amdgcn_readfirstlane((int)(stream_left || __any(cv || ns != 0))) != 0;
  };
  for (;;) {
    (void)step(XA, TA, sA, XB, TB, sB);
    if (!step(XB, TB, sB, XA, TA, sA)) break;
  }
  if (fq_n) fq_flush();
#ifdef CASK_STAMPS
  if (a.stamps && lane == 0 && wid < kStampWaves) a.stamps[17 + 2 * wid] = __builtin_amdgcn_s_memrealtime();
#endif
}

// ---------------------------------------------------------------------------------------------
// Walk mode with k_finish running beside k_run_hash (it needs only the chase's output, so it runs
// in the slots the hash's last waves leave): the checksum verdicts k_finish may have read before
// the hash wrote them. Every chunk with a failing row has cerr set (the chase's EOF rows, the
// hash's atomicMin for every checksum failure), so only those chunks are walked again: a row whose
// slot has the bad bit and is not an EOF row gets kRowChecksum (k_finish's rule), and the file's
// first failing row takes the chunk's final cerr. Usually no chunk is flagged: one thread per chunk
// reads cerr and exits.
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_hash_fix(ScanArgs a) {
  const uint64_t c = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (c >= a.total_chunks) return;
  const uint32_t ce = a.cerr[c];
  if (ce == 0xFFFFFFFFu) return;
  const uint32_t fi = find_file(a.files, a.nfiles, c);
  const FileDesc fd = a.files[fi];
  const uint64_t base = a.gbase[c], c0 = (c - fd.first_chunk) * (uint64_t)a.chunk;
  const uint32_t n = a.count[c] & kCountMask;
  for (uint32_t r = 0; r < n; ++r) {
    const u32x4 w = *(const u32x4*)(a.slots + (c * (uint64_t)a.slot_cap + r) * 4);
    const uint32_t ksz = w.w & 0xFFFFu;
    const uint64_t p = c0 + ((w.w >> 16) & 0x7FFFu);
    const uint64_t end = p + 18ull + ksz + (w.z == 0xFFFFFFFFu ? 0ull : (uint64_t)w.z);
    const bool eof = p + 18 > fd.len || end > fd.len;
    if (!eof && (w.w & kSlotBad) && base + r < a.row_cap) a.status[base + r] = kRowChecksum;
  }
  atomicMax(&a.err_inv[fi], ~(unsigned long long)(base + ce));
}

// A walk-mode call that needs the repair path: its slot rows (kWalkSlotCap per chunk, every chunk's
// count within them: no slot_overflow) moved to the full stride, one thread per slot row.
__global__ __launch_bounds__(256) void k_restride(const uint32_t* __restrict__ src, uint32_t* __restrict__ dst,
                                                  const uint32_t* __restrict__ count, uint64_t nchunks,
                                                  uint32_t cap_src, uint32_t cap_dst) {
  const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  const uint64_t c = i / cap_src;
  const uint32_t r = (uint32_t)(i - c * cap_src);
  if (c >= nchunks || r >= (count[c] & kCountMask)) return;
  *(u32x4*)(dst + (c * cap_dst + r) * 4) = *(const u32x4*)(src + (c * cap_src + r) * 4);
}

void launch_restride(const ScanArgs& a, uint32_t* dst, uint32_t cap_dst, void* stream) {
  const uint64_t n = a.total_chunks * (uint64_t)a.slot_cap;
  if (!n) return;
  hipLaunchKernelGGL(k_restride, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, a.slots, dst,
                     a.count, a.total_chunks, a.slot_cap, cap_dst);
}

void launch_hash_fix(const ScanArgs& a, void* stream) {
  if (!a.total_chunks) return;
  hipLaunchKernelGGL(k_hash_fix, dim3((uint32_t)((a.total_chunks + 255) / 256)), dim3(256), 0, (hipStream_t)stream, a);
}

void launch_walk_chase(const ScanArgs& a, void* stream) {
  if (!a.total_chunks) return;
  const uint64_t nruns = a.wruns ? a.nwruns : (a.total_chunks + a.run - 1) / a.run;
  if (!nruns) return;
  // CASK_CHASE_WG (tuning knob): threads per workgroup (a lane per run). One-wave workgroups spread
  // the chase over every CU (configs[2]: 128 four-wave groups left half of the CUs idle; with
  // one-wave groups the chase takes 0.35 instead of 0.46 ms)
  static const uint32_t wg = cask_knobs::tune("CASK_CHASE_WG") ? (uint32_t)atoi(cask_knobs::tune("CASK_CHASE_WG")) : 64u;
  const uint32_t tpb = wg == 64 || wg == 128 ? wg : 256u;
  const uint32_t grid = (uint32_t)((nruns + tpb - 1) / tpb);
  hipLaunchKernelGGL(k_walk_chase, dim3(grid), dim3(tpb), 0, (hipStream_t)stream, a, a.files);
}

// A persistent grid of exactly the resident workgroups: a workgroup beyond them would start only as
// the first ones finish, holding its first run (claimed by block index) until the end.
uint64_t run_hash_waves() {
  static int per_cu = 0;
  if (!per_cu) {
    int nb = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_run_hash, 256, 0) == hipSuccess && nb > 0) per_cu = 4 * nb;
    if (per_cu <= 0) per_cu = 8;
  }
  return (uint64_t)device_cus() * (uint64_t)per_cu;
}

void launch_run_hash(const ScanArgs& a, void* stream, int cus) {
  if (!a.total_chunks) return;
  const uint64_t nruns = a.wruns ? a.nwruns : (a.total_chunks + a.run - 1) / a.run;
  if (!nruns) return;
  uint64_t waves = run_hash_waves();
  if (cus > 0) waves = waves / (uint64_t)device_cus() * (uint64_t)cus;
  if (const char* e = cask_knobs::tune("CASK_HASH_WAVES_PER_CU")) waves = (uint64_t)device_cus() * (uint64_t)atoi(e);
  if (waves > nruns) waves = nruns;
  hipLaunchKernelGGL(k_run_hash, dim3((uint32_t)((waves + 3) / 4)), dim3(256), 0, (hipStream_t)stream, a);
}

}  // namespace cask_dev
