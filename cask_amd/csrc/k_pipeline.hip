// The kernels around k_scan_chunks: long records, validation of the speculated boundaries with
// per-file row prefixes, the summary the host reads back, dense compaction, and the exact repair
// walk. All are small next to the scan; none needs inter-workgroup hand-offs.
#include "device_util.h"

namespace cask_dev {

// ------------------------------------------------------------------------------------------
// K_long: the records the chunk scan did not hash out of LDS — those that run past the window, or
// are longer than ScanArgs::big — hashed straight from HBM (the same rule picks them:
// lds_hashed()). EOF rows have already failed.
//  * k_long_enqueue, one lane per chunk not yet queued since its last scan (long_done): rows
//    long_r[t] .. count-1 go to the queue region of their length class;
//  * k_long_hash, one lane per queued record, longest class first: the lanes of a wave hash
//    records of similar length, so a wave's lifetime is not set by one 64-KiB record among 1-KiB
//    ones. Each lane keeps 128 B of its record in flight while it mixes the previous 128 B.
// Chunks are queued whatever their file's validity: a repair pass re-scans only flagged chunks,
// and re-scanning one clears long_done, so every chunk's long records are hashed once per scan.
// ------------------------------------------------------------------------------------------
// A long record failed its checksum: mark its slot row and chunk (the repair/compaction path reads
// those), and when k_finish has already written the dense rows, its dense row and the file's first
// failing row too.
__device__ __forceinline__ void long_failed(const ScanArgs& a, uint64_t slot, uint64_t t, uint32_t r, uint32_t fi,
                                            uint32_t w3) {
  a.slots[slot * 4 + 3] = w3 | kSlotBad;
  atomicMin(&a.cerr[t], r);  // outlives the pass: validation rebuilds file_err from cerr
  atomicMin(&a.file_err[fi], (unsigned long long)slot);
  if (a.dense) {
    const uint64_t d = a.gbase[t] + r;
    if (d < a.row_cap) a.status[d] = kRowChecksum;
    atomicMax(&a.err_inv[fi], ~(unsigned long long)d);
  }
}

__device__ __forceinline__ void long_verify(const ScanArgs& a, uint64_t slot, uint32_t& nl) {
  const uint64_t t = slot / a.slot_cap;
  const uint32_t r = (uint32_t)(slot % a.slot_cap);
  const uint32_t fi = find_file(a.files, a.nfiles, t);
  const FileDesc fd = a.files[fi];
  const uint64_t c0 = (t - fd.first_chunk) * (uint64_t)a.chunk;
  uint32_t* w = a.slots + slot * 4;
  const uint32_t w3 = w[3], vsz = w[2];
  const uint64_t p = c0 + ((w3 >> 16) & 0x7FFFu);
  const uint64_t rl = 18ull + (w3 & 0xFFFFu) + ((vsz == 0xFFFFFFFFu) ? 0ull : (uint64_t)vsz);
  ++nl;
  const uint32_t stored = gld4(fd.data + p);
  if (gbl_xxh32(fd.data + p + 4, rl - 4) != stored) long_failed(a, slot, t, r, fi, w3);  // data.rs:193-198
}

// The rows of chunk t that k_long hashes, with their length class (f(slot, class) per row).
template <class F>
__device__ __forceinline__ void long_rows(const ScanArgs& a, uint64_t t, F f) {
  const uint32_t r0 = a.long_r[t];
  const uint32_t n = a.count[t] & kCountMask;
  const uint32_t fi = find_file(a.files, a.nfiles, t);
  const FileDesc fd = a.files[fi];
  const uint64_t c0 = (t - fd.first_chunk) * (uint64_t)a.chunk;
  const uint64_t wend = c0 + a.win < fd.len ? c0 + a.win : fd.len;
  for (uint32_t r = r0; r < n; ++r) {
    const uint64_t slot = t * a.slot_cap + r;
    const uint32_t* w = a.slots + slot * 4;
    const uint32_t w3 = w[3], vsz = w[2];
    const uint64_t p = c0 + ((w3 >> 16) & 0x7FFFu);
    const uint64_t rl = 18ull + (w3 & 0xFFFFu) + ((vsz == 0xFFFFFFFFu) ? 0ull : (uint64_t)vsz);
    if (p + rl > fd.len || lds_hashed(p, rl, wend, a.big)) continue;  // EOF row, or done in LDS
    uint32_t b = 63u - (uint32_t)__builtin_clzll(rl);
    b = b < kLqMinLog ? kLqMinLog : b > 31u ? 31u : b;
    f(slot, b - kLqMinLog);
  }
}

// Each block queues the long records of 256 consecutive chunks at a time (8 MiB of log with the
// default geometry) as one contiguous piece per length class, so a wave of k_long_hash reads a
// few neighbouring stretches of HBM rather than 64 pages spread over every file.
__global__ __launch_bounds__(256) void k_long_enqueue(ScanArgs a) {
  __shared__ uint32_t cnt1[kLqClasses], cnt2[kLqClasses];
  __shared__ uint64_t gb[kLqClasses];
  uint32_t nl = 0;
  const uint64_t t_hi = a.t_hi ? a.t_hi : a.total_chunks;
  for (uint64_t base = a.t_lo + blockIdx.x * 256ull; base < t_hi; base += (uint64_t)gridDim.x * 256ull) {
    if (threadIdx.x < kLqClasses) cnt1[threadIdx.x] = cnt2[threadIdx.x] = 0;
    __syncthreads();
    const uint64_t t = base + threadIdx.x;
    const bool act = t < t_hi && a.long_r[t] != 0xFFFFFFFFu && !a.long_done[t];
    if (act) long_rows(a, t, [&](uint64_t, uint32_t c) { atomicAdd(&cnt1[c], 1u); });
    __syncthreads();
    if (threadIdx.x < kLqClasses && cnt1[threadIdx.x])
      gb[threadIdx.x] = atomicAdd(&a.ctr->lq_cnt[threadIdx.x], cnt1[threadIdx.x]);
    __syncthreads();
    if (act) {
      a.long_done[t] = 1;
      long_rows(a, t, [&](uint64_t slot, uint32_t c) {
        const uint64_t k = gb[c] + atomicAdd(&cnt2[c], 1u);
        const uint32_t b = c + kLqMinLog;
        if (k < lq_region_cap(a.total_chunks, a.chunk, b)) {
          a.lq[lq_region_base(a.total_chunks, a.chunk, b) + k] = slot;
        } else {
          long_verify(a, slot, nl);  // cannot happen (region bound); hashed here rather than lost
        }
      });
    }
    __syncthreads();  // cnt1/cnt2/gb are reused by the next stretch
  }
  for (int o = 32; o; o >>= 1) nl += __shfl_xor(nl, o, 64);  // one counter update per wave
  if ((threadIdx.x & 63) == 0 && nl) atomicAdd(&a.ctr->nlong, (unsigned long long)nl);
}

// long_verify by a quad of lanes (the same slot in all four, all four active): quad_gbl_xxh32.
__device__ __forceinline__ void long_verify_quad(const ScanArgs& a, uint64_t slot, uint32_t q, uint32_t& nl) {
  const uint64_t t = slot / a.slot_cap;
  const uint32_t r = (uint32_t)(slot % a.slot_cap);
  const uint32_t fi = find_file(a.files, a.nfiles, t);
  const FileDesc fd = a.files[fi];
  const uint64_t c0 = (t - fd.first_chunk) * (uint64_t)a.chunk;
  uint32_t* w = a.slots + slot * 4;
  const uint32_t w3 = w[3], vsz = w[2];
  const uint64_t p = c0 + ((w3 >> 16) & 0x7FFFu);
  const uint64_t rl = 18ull + (w3 & 0xFFFFu) + ((vsz == 0xFFFFFFFFu) ? 0ull : (uint64_t)vsz);
  const uint32_t stored = gld4(fd.data + p);
  const uint32_t got = quad_gbl_xxh32(fd.data + p + 4, rl - 4, q);
  if (q == 0) {
    ++nl;
    if (got != stored) long_failed(a, slot, t, r, fi, w3);  // data.rs:193-198
  }
}

// One quad of lanes per queued record, longest length class first.
__global__ __launch_bounds__(256) void k_long_hash(ScanArgs a) {
  __shared__ uint64_t cnt[kLqClasses], base[kLqClasses];
  if (threadIdx.x < kLqClasses) {
    const uint32_t b = kLqMinLog + threadIdx.x;
    const uint64_t cap = lq_region_cap(a.total_chunks, a.chunk, b);
    uint64_t hi = a.lq_hi ? a.lq_hi[threadIdx.x] : a.ctr->lq_cnt[threadIdx.x];
    uint64_t lo = a.lq_lo ? a.lq_lo[threadIdx.x] : 0u;
    hi = hi < cap ? hi : cap;
    lo = lo < hi ? lo : hi;
    cnt[threadIdx.x] = hi - lo;
    base[threadIdx.x] = lq_region_base(a.total_chunks, a.chunk, b) + lo;
  }
  __syncthreads();
  uint64_t total = 0;
  for (uint32_t j = 0; j < kLqClasses; ++j) total += cnt[j];
  uint32_t nl = 0;
  const uint32_t q = threadIdx.x & 3;
  const uint64_t nq = (uint64_t)gridDim.x * (blockDim.x >> 2);
  for (uint64_t i = blockIdx.x * (uint64_t)(blockDim.x >> 2) + (threadIdx.x >> 2); i < total; i += nq) {
    uint64_t k = i;
    uint32_t j = kLqClasses - 1;  // longest class first
    while (k >= cnt[j]) k -= cnt[j--];
    long_verify_quad(a, a.lq[base[j] + k], q, nl);
  }
  for (int o = 32; o; o >>= 1) nl += __shfl_xor(nl, o, 64);
  if ((threadIdx.x & 63) == 0 && nl) atomicAdd(&a.ctr->nlong, (unsigned long long)nl);
}

// ------------------------------------------------------------------------------------------
// Validation, as a three-launch segmented scan over tiles of kTile chunks (a tile never spans
// two files):
//  * T[c] = max over earlier chunks' exits (0 for chunks that found no start) is the true chain
//    position entering chunk c as long as every earlier chunk of the file is valid; chunk c is
//    valid iff its speculated start equals T[c] (or it found none and T[c] is past its end);
//  * base[c] = exclusive sum of the earlier chunks' row counts within the file.
// ------------------------------------------------------------------------------------------
constexpr uint32_t kTile = kTileChunks;  // chunks per tile (256 threads x 4)

__device__ __forceinline__ uint32_t tile_file(const ScanArgs& a, uint64_t T) {
  uint32_t lo = 0, hi = a.nfiles;
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (a.files[mid].first_tile <= T) lo = mid; else hi = mid;
  }
  return lo;
}

__device__ __forceinline__ uint64_t chunk_exit(const ScanArgs& a, uint64_t g) {
  return a.spec[g] == kNone ? 0ull : a.exit[g];
}

// Block-wide (256 threads) exclusive max-scan and sum-scan of one value pair per thread, plus the
// block totals.
__device__ __forceinline__ void block_excl_scan2(unsigned long long mx, unsigned long long sm,
                                                 unsigned long long& ex_mx, unsigned long long& ex_sm,
                                                 unsigned long long& tot_mx, unsigned long long& tot_sm) {
  __shared__ unsigned long long smx[4], ssm[4];
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int o = 1; o < 64; o <<= 1) {
    const unsigned long long u = __shfl_up(mx, o, 64), us = __shfl_up(sm, o, 64);
    if ((int)lane >= o) {
      mx = mx > u ? mx : u;
      sm += us;
    }
  }
  const unsigned long long pm = __shfl_up(mx, 1, 64), ps = __shfl_up(sm, 1, 64);
  if (lane == 63) {
    smx[wave] = mx;
    ssm[wave] = sm;
  }
  __syncthreads();
  unsigned long long wm = 0, ws = 0;
  for (uint32_t k = 0; k < wave; ++k) {
    wm = wm > smx[k] ? wm : smx[k];
    ws += ssm[k];
  }
  ex_mx = wm;
  ex_sm = ws;
  if (lane > 0) {
    ex_mx = ex_mx > pm ? ex_mx : pm;
    ex_sm += ps;
  }
  tot_mx = 0;
  tot_sm = 0;
  for (uint32_t k = 0; k < 4; ++k) {
    tot_mx = tot_mx > smx[k] ? tot_mx : smx[k];
    tot_sm += ssm[k];
  }
  __syncthreads();
}

__global__ __launch_bounds__(256) void k_val_reduce(ScanArgs a) {
  const uint64_t T = blockIdx.x;
  const uint32_t f = tile_file(a, T);
  const FileDesc fd = a.files[f];
  const uint64_t c_lo = (T - fd.first_tile) * kTile;
  unsigned long long mx = 0, sm = 0;
  for (uint32_t j = 0; j < 4; ++j) {
    const uint64_t c = c_lo + threadIdx.x * 4 + j;
    if (c < fd.nchunks) {
      const uint64_t g = fd.first_chunk + c;
      const unsigned long long e = chunk_exit(a, g);
      mx = mx > e ? mx : e;
      sm += a.count[g] & kCountMask;
    }
  }
  unsigned long long em, es, tm, ts;
  block_excl_scan2(mx, sm, em, es, tm, ts);
  if (threadIdx.x == 0) {
    a.tile_max[T] = tm;
    a.tile_sum[T] = ts;
  }
}

__global__ __launch_bounds__(256) void k_val_files(ScanArgs a) {
  const uint32_t f = blockIdx.x;
  const FileDesc fd = a.files[f];
  const uint64_t nt = (fd.nchunks + kTile - 1) / kTile;
  unsigned long long cmx = 0, csm = 0;
  for (uint64_t b = 0; b < nt; b += 256) {
    const uint64_t i = b + threadIdx.x;
    unsigned long long mx = 0, sm = 0;
    if (i < nt) {
      mx = a.tile_max[fd.first_tile + i];
      sm = a.tile_sum[fd.first_tile + i];
    }
    unsigned long long em, es, tm, ts;
    block_excl_scan2(mx, sm, em, es, tm, ts);
    if (i < nt) {
      a.tile_pmax[fd.first_tile + i] = cmx > em ? cmx : em;
      a.tile_psum[fd.first_tile + i] = csm + es;
    }
    cmx = cmx > tm ? cmx : tm;
    csm += ts;
  }
  if (threadIdx.x == 0) a.file_total[f] = csm;
}

__global__ __launch_bounds__(256) void k_val_apply(ScanArgs a) {
  const uint64_t T = blockIdx.x;
  const uint32_t f = tile_file(a, T);
  const FileDesc fd = a.files[f];
  const uint64_t c_lo = (T - fd.first_tile) * kTile;
  unsigned long long e[4], cn[4];
  unsigned long long mx = 0, sm = 0;
  for (uint32_t j = 0; j < 4; ++j) {
    const uint64_t c = c_lo + threadIdx.x * 4 + j;
    e[j] = 0;
    cn[j] = 0;
    if (c < fd.nchunks) {
      const uint64_t g = fd.first_chunk + c;
      e[j] = chunk_exit(a, g);
      cn[j] = a.count[g] & kCountMask;
    }
    mx = mx > e[j] ? mx : e[j];
    sm += cn[j];
  }
  unsigned long long em, es, tm, ts;
  block_excl_scan2(mx, sm, em, es, tm, ts);
  const unsigned long long pmax = a.tile_pmax[T];
  unsigned long long run_max = pmax > em ? pmax : em;
  unsigned long long run_sum = a.tile_psum[T] + es;
  for (uint32_t j = 0; j < 4; ++j) {
    const uint64_t c = c_lo + threadIdx.x * 4 + j;
    if (c < fd.nchunks) {
      const uint64_t g = fd.first_chunk + c;
      a.tin[g] = run_max;
      a.base[g] = run_sum;
      const uint64_t c0 = c * (uint64_t)a.chunk;
      const uint64_t c1 = (c0 + a.chunk < fd.len) ? c0 + a.chunk : fd.len;
      const uint64_t sp = a.spec[g];
      bool ok;
      if (c == 0) ok = true;
      else if (sp != kNone) ok = (sp == run_max);
      else ok = (run_max >= c1);
      a.redo[g] = ok ? 0 : 1;  // a repair pass re-scans the chunks flagged here
      const uint32_t ce = a.cerr[g];
      if (ce != 0xFFFFFFFFu) atomicMin(&a.file_err[f], (unsigned long long)(g * a.slot_cap + ce));
      if (!ok) {
        atomicMin((unsigned long long*)&a.first_bad[f], (unsigned long long)c);
        // local repair: T[c] is the chain's true entry into chunk c whenever every earlier chunk
        // is valid, so the next exact pass starts chunk c there (or skips it: T[c] past its
        // end). A T[c] behind the chunk comes from a stale earlier exit: keep the old start.
        if (a.respec) {
          if (run_max >= c1) a.spec[g] = kNone;
          else if (run_max >= c0) a.spec[g] = run_max;
        }
      }
    }
    run_max = run_max > e[j] ? run_max : e[j];
    run_sum += cn[j];
  }
}

// Summary: row offsets per file, first failing row per file, flags -> one buffer for the host.
__global__ void k_summary(ScanArgs a, uint64_t* out) {
  SummaryHead* h = (SummaryHead*)out;
  uint64_t* row_off = out + sizeof(SummaryHead) / 8;
  uint64_t* fbad = row_off + a.nfiles + 1;
  uint64_t* badT = fbad + a.nfiles;
  uint64_t* err = badT + a.nfiles;
  uint64_t* err_slot = err + a.nfiles;
  __shared__ uint64_t total;
  if (threadIdx.x == 0) {
    uint64_t acc = 0;
    for (uint32_t f = 0; f < a.nfiles; ++f) {
      row_off[f] = acc;
      acc += a.file_total[f];
    }
    row_off[a.nfiles] = acc;
    total = acc;
  }
  __syncthreads();
  for (uint32_t f = threadIdx.x; f < a.nfiles; f += blockDim.x) {
    const FileDesc fd = a.files[f];
    const uint64_t b = a.first_bad[f];
    fbad[f] = b;
    badT[f] = (b != kNone) ? a.tin[fd.first_chunk + b] : 0;
    const unsigned long long s = a.file_err[f];
    err_slot[f] = s;
    if (s == kNone) {
      err[f] = kNone;
    } else {
      const uint64_t t = s / a.slot_cap, r = s % a.slot_cap;
      err[f] = row_off[f] + a.base[t] + r;
    }
  }
  if (threadIdx.x == 0) {
    h->total_rows = total;
    h->nlong = a.ctr->nlong;
    uint64_t any = 0, cnt = 0;
    for (uint32_t f = 0; f < a.nfiles; ++f)
      if (a.first_bad[f] != kNone) {
        any = 1;
        cnt += a.files[f].nchunks - a.first_bad[f];
      }
    h->any_invalid = any;
    h->invalid_chunks = cnt;
    h->walk_steps = a.ctr->walk_steps;
  }
}

// ------------------------------------------------------------------------------------------
// K_finish (dense path): one launch after k_scan_chunks that validates every speculated chunk
// start, numbers the rows and writes them dense, in (file, pos) order, into the caller's arrays.
// It replaces the three validation launches, the summary and k_compact of the repair path.
//
// Chunks are taken in tiles of kFinTile (one per thread), tiles in order from a counter. A tile's
// chunks give (rows, exit) pairs; the exclusive prefix over all earlier chunks — row count
// (global: files are consecutive chunk ranges, so the dense row index is a global prefix) and the
// maximum exit within the current file, T[c], the chain position entering chunk c as long as
// every earlier chunk of the file is valid — comes from a decoupled look-back over the earlier
// tiles' published aggregates (north_star's prefix scan). Chunk c is valid iff its start equals
// T[c] (or it found none and T[c] is past its end); any invalid chunk sends the call to the
// repair path, which rewrites every row (k_compact). Rows are then expanded from the chunk table:
// a regular chunk from its first row, the others from their slot rows; each thread writes four
// consecutive rows with 16-B (pos, seq, vsz), 8-B (ksz) and 4-B (status) stores.
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_finish(ScanArgs a) {
  constexpr uint32_t TC = kFinTile;
  __shared__ uint32_t s_tile;
  __shared__ SegAgg s_wave[4];
  __shared__ uint32_t s_base[TC + 1];      // row base of each chunk of the tile, relative to the tile
  __shared__ u32x4 s_desc[TC];            // regular chunk: first row; else slot row of the chunk
  __shared__ uint64_t s_c0[TC], s_len[TC];
  __shared__ uint32_t s_reg[TC];          // regular flag
  __shared__ uint32_t s_long;             // the tile has a record for k_long_hash
  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // tiles by index when the whole grid is resident at once (a grid's worth of claims on one
  // counter queue for microseconds), else claimed in order from the counter
  if (tid == 0) {
    s_tile = a.fin_static ? blockIdx.x : atomicAdd(&a.ctr->tile_next, 1u);
    s_long = 0u;
  }
  __syncthreads();
  const uint64_t tile = __builtin_amdgcn_readfirstlane(s_tile);
  if (tile == 0 && a.call_zero)  // the other call block, for the next call (no copy before it)
    for (uint32_t i = tid; i < a.call_zero_words; i += TC) a.call_zero[i] = 0;
  const uint64_t c = tile * TC + tid;
  const bool act = c < a.total_chunks;
  // the chunk's table entries, all loaded at once (the descriptor too: only regular chunks use it)
  uint32_t n = 0, cw = 0, fi = 0, cerr = 0xFFFFFFFFu, lr = 0xFFFFFFFFu;
  uint64_t e = 0, spec = kNone, c0 = 0, c1 = 0, len = 0;
  u32x4 dsc = u32x4{0u, 0u, 0u, 0u};
  bool head = false;
  // the file of the wave's first chunk (uniform: scalar loads), then each lane's own (a wave's
  // chunks rarely cross a file boundary)
  fi = find_file(a.files, a.nfiles, (uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(tile * TC + wave * 64)));
  if (act) {
    cw = a.count[c];
    n = cw & kCountMask;
    spec = a.spec[c];
    const uint64_t ex = a.exit[c];
    cerr = a.cerr[c];
    lr = a.long_r[c];
    dsc = ((const u32x4*)a.desc)[c];
    e = spec == kNone ? 0ull : ex;
    while (fi + 1 < a.nfiles && a.files[fi + 1].first_chunk <= c) ++fi;
    const FileDesc fd = a.files[fi];
    c0 = (c - fd.first_chunk) * (uint64_t)a.chunk;
    c1 = (c0 + a.chunk < fd.len) ? c0 + a.chunk : fd.len;
    len = fd.len;
    head = c0 == 0;
  }
  // in-tile inclusive scan of (rows, segmented max exit), by wave then across the 4 waves
  SegAgg v{n, e, act ? fi : 0xFFFFFFFFu, head ? 1u : 0u};
  SegAgg inc = v;
  for (int o = 1; o < 64; o <<= 1) {
    SegAgg u;
    u.rows = __shfl_up(inc.rows, o, 64);
    u.mx = __shfl_up(inc.mx, o, 64);
    u.fl = __shfl_up(inc.fl, o, 64);
    u.hs = __shfl_up(inc.hs, o, 64);
    if ((int)lane >= o) inc = seg_combine(u, inc);
  }
  if (lane == 63) s_wave[wave] = inc;
  __syncthreads();
  SegAgg wpre{0, 0, 0xFFFFFFFFu, 0};
  for (uint32_t k = 0; k < wave; ++k) wpre = seg_combine(wpre, s_wave[k]);
  inc = seg_combine(wpre, inc);
  SegAgg total = seg_combine(seg_combine(seg_combine(s_wave[0], s_wave[1]), s_wave[2]), s_wave[3]);
  // Publish the tile's aggregate, then the prefix of the earlier tiles in two levels (every tile
  // starts at about the same time, so a chained look-back would wait for its predecessors' own
  // look-backs): the tiles of this tile's group of kFinGroup, then the groups before it, whose
  // aggregates the last tile of each group publishes. Two round trips, whatever the tile's index.
  const uint64_t ntiles = (a.total_chunks + TC - 1) / TC, grp = tile / kFinGroup;
  uint64_t* st2 = a.tstate + 8ull * (ntiles + 1);  // group aggregates
  if (tid == 0) agg_put(a.tstate + 8ull * tile, a.epoch, total);
  SegAgg P1{0, 0, 0xFFFFFFFFu, 0}, P2{0, 0, 0xFFFFFFFFu, 0};
  // (tile is the same in every thread: the barriers inside are uniform)
  bool got = block_prefix(a.tstate, a.epoch, grp * kFinGroup, tile, P1);
  if (got && tid == 0 && (tile % kFinGroup == kFinGroup - 1 || tile + 1 == ntiles))
    agg_put(st2 + 8ull * grp, a.epoch, seg_combine(P1, total));
  got = got && block_prefix(st2, a.epoch, 0, grp, P2);
  if (!got && tid == 0) atomicOr(&a.ctr->any_invalid, 1u);  // gave up waiting: the repair path redoes the call
  const SegAgg P = seg_combine(P2, P1);
  const SegAgg full = seg_combine(P, inc);  // inclusive prefix through this chunk
  const uint64_t base = full.rows - n;      // this chunk's first dense row
  // T[c]: max exit of the earlier chunks of this file. The lane before holds the tile's inclusive
  // prefix through c - 1 (lane 0: the earlier waves' total).
  SegAgg prev;
  prev.rows = __shfl_up(inc.rows, 1, 64);
  prev.mx = __shfl_up(inc.mx, 1, 64);
  prev.fl = __shfl_up(inc.fl, 1, 64);
  prev.hs = __shfl_up(inc.hs, 1, 64);
  if (lane == 0) prev = wpre;
  const SegAgg pf = seg_combine(P, prev);
  if (act) {
    const uint64_t T = (pf.fl == fi) ? pf.mx : 0ull;
    const bool ok = head || (spec != kNone ? spec == T : T >= c1);
    if (!ok) atomicOr(&a.ctr->any_invalid, 1u);
    a.gbase[c] = base;
    if (head) a.row_off[fi] = base;
    if (cerr != 0xFFFFFFFFu) atomicMax(&a.err_inv[fi], ~(unsigned long long)(base + cerr));
    if (c + 1 == a.total_chunks) a.ctr->total_rows = base + n;
  }
  // one store per tile that has long records (configs[2]: nearly every tile; an atomic per wave on
  // one word serialised thousands of updates in L2)
  if (__ballot(act && lr != 0xFFFFFFFFu) && lane == 0) s_long = 1u;
  // rows of the tile: [tile_lo, tile_lo + tile_rows)
  const uint64_t tile_lo = P.rows, tile_rows = total.rows;
  s_base[tid] = (uint32_t)(base - tile_lo);
  if (tid == TC - 1) s_base[TC] = (uint32_t)tile_rows;
  s_reg[tid] = act && (cw & kCountRegular);
  s_c0[tid] = c0;
  s_len[tid] = len;
  if (act && (cw & kCountRegular)) s_desc[tid] = dsc;
  __syncthreads();
  if (tid == 0 && s_long) a.ctr->long_pending = 1u;  // every writer stores the same value
  if (!tile_rows) return;
  const uint32_t nch = (uint32_t)((a.total_chunks - tile * TC) < TC ? (a.total_chunks - tile * TC) : TC);
  const float per_row = (float)nch / (float)tile_rows;
  const uint64_t hb = a.hint ? 22ull : 18ull;  // header bytes (a hint: data.rs:242-256)
  // row d of the tile (tile_lo <= d < tile_lo + tile_rows); j: its chunk, advanced from the last one
  auto row_at = [&](uint64_t d, uint32_t& j, uint64_t& P, uint64_t& S, uint32_t& V, uint32_t& K, uint32_t& T) {
    const uint32_t rel = (uint32_t)(d - tile_lo);
    while (j + 1 < nch && s_base[j + 1] <= rel) ++j;  // (skips chunks with no rows)
    const uint32_t r = rel - s_base[j];
    const uint64_t cc0 = s_c0[j];
    if (s_reg[j]) {
      const u32x4 w = s_desc[j];
      const uint32_t ksz = w.w & 0xFFFFu;
      const uint64_t rl = 18ull + ksz + ((w.z == 0xFFFFFFFFu) ? 0ull : (uint64_t)w.z);
      P = cc0 + ((w.w >> 16) & 0x7FFFu) + (uint64_t)r * rl;
      S = (((uint64_t)w.y << 32) | w.x) + r;
      V = w.z;
      K = ksz;
      T = kRowOk;
    } else {
      const u32x4 w = *(const u32x4*)(a.slots + ((tile * TC + j) * (uint64_t)a.slot_cap + r) * 4);
      const uint32_t ksz = w.w & 0xFFFFu;
      const uint64_t p = cc0 + ((w.w >> 16) & 0x7FFFu);
      const uint64_t end = p + hb + ksz + ((a.hint || w.z == 0xFFFFFFFFu) ? 0ull : (uint64_t)w.z);
      const uint64_t fl = s_len[j];
      P = p;
      S = ((uint64_t)w.y << 32) | w.x;
      V = w.z;
      K = ksz;
      T = (p + hb > fl || end > fl) ? kRowEof : (w.w & kSlotBad) ? kRowChecksum : kRowOk;
    }
  };
  // Blocks of 256 rows (aligned to the row index), one per wave at a time; in each half of a block
  // lane l writes rows 2l and 2l + 1, so every store instruction covers one contiguous stretch of its
  // array (1 KiB of pos or seq, 512 B of vsz, 256 B of ksz, 128 B of status): whole lines from
  // every instruction, not halves of them completed by the next one.
  const uint64_t lo = tile_lo, hi = tile_lo + tile_rows;
  for (uint64_t blk = (lo >> 8) + wave; blk < ((hi + 255) >> 8); blk += TC / 64) {
#pragma unroll
    for (uint32_t h = 0; h < 2; ++h) {
      const uint64_t d0 = (blk << 8) + 128u * h + 2u * lane;
      const bool in0 = d0 >= lo && d0 < hi, in1 = d0 + 1 >= lo && d0 + 1 < hi;
      if (!in0 && !in1) continue;
      const uint64_t dfirst = in0 ? d0 : d0 + 1;
      // the last chunk j with s_base[j] <= the first row: guessed from the tile's mean rows per
      // chunk, then stepped (one or two LDS reads for tiles of similar chunks)
      const uint32_t rel0 = (uint32_t)(dfirst - lo);
      uint32_t j = (uint32_t)((float)rel0 * per_row);  // (only a guess: corrected below)
      j = j < nch ? j : nch - 1;
      while (j > 0 && s_base[j] > rel0) --j;
      uint64_t P0 = 0, S0 = 0, P1 = 0, S1 = 0;
      uint32_t V0 = 0, K0 = 0, T0 = 0, V1 = 0, K1 = 0, T1 = 0;
      if (in0) row_at(d0, j, P0, S0, V0, K0, T0);
      if (in1) row_at(d0 + 1, j, P1, S1, V1, K1, T1);
      if (a.vec_ok && in0 && in1 && d0 + 1 < a.row_cap) {
        typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));
        typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
        // pos and seq (16 of the 23 bytes) bypass the caches (nontemporal): no dirty lines left in
        // the Infinity Cache for the next call's scan to write back; the narrow arrays keep the
        // default policy (nontemporal stores of 2-8 B per lane ran slower)
        __builtin_nontemporal_store(u64x2{P0, P1}, (u64x2*)(a.pos + d0));
        __builtin_nontemporal_store(u64x2{S0, S1}, (u64x2*)(a.seq + d0));
        *(u32x2*)(a.vsz + d0) = u32x2{V0, V1};
        *(uint32_t*)(a.ksz + d0) = (K0 & 0xFFFFu) | (K1 << 16);
        *(uint16_t*)(a.status + d0) = (uint16_t)(T0 | (T1 << 8));
      } else {
        if (in0 && d0 < a.row_cap) {
          a.pos[d0] = P0;
          a.seq[d0] = S0;
          a.vsz[d0] = V0;
          a.ksz[d0] = (uint16_t)K0;
          a.status[d0] = (uint8_t)T0;
        }
        if (in1 && d0 + 1 < a.row_cap) {
          a.pos[d0 + 1] = P1;
          a.seq[d0 + 1] = S1;
          a.vsz[d0 + 1] = V1;
          a.ksz[d0 + 1] = (uint16_t)K1;
          a.status[d0 + 1] = (uint8_t)T1;
        }
      }
    }
  }
}

// Error detail of the first failing dense row `row` of file fi (error path only): out[0] stored
// checksum, out[1] computed XXH32, out[2] row status, out[3..4] pos.
__global__ void k_err_dense(ScanArgs a, uint32_t fi, uint64_t row, uint32_t* out) {
  if (threadIdx.x || blockIdx.x) return;
  const FileDesc fd = a.files[fi];
  const uint64_t p = a.pos[row];
  out[0] = 0;
  out[1] = 0;
  out[2] = a.status[row];
  out[3] = (uint32_t)p;
  out[4] = (uint32_t)(p >> 32);
  if (p + 18 > fd.len) return;
  const uint8_t* hp = fd.data + p;
  const uint64_t rl = g_reclen(hp);
  out[0] = gld4(hp);
  if (p + rl > fd.len) return;
  out[1] = gbl_xxh32(hp + 4, rl - 4);
}

// K_compact: slot rows -> dense SoA rows in (file, pos) order. One wave per chunk.
__global__ __launch_bounds__(256) void k_compact(ScanArgs a, const uint64_t* summary) {
  const uint64_t* row_off = summary + sizeof(SummaryHead) / 8;
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t nw = (uint64_t)gridDim.x * (blockDim.x >> 6);
  for (uint64_t t = blockIdx.x * (uint64_t)(blockDim.x >> 6) + (threadIdx.x >> 6); t < a.total_chunks; t += nw) {
    const uint32_t fi = find_file(a.files, a.nfiles, t);
    if (a.first_bad[fi] != kNone) continue;  // invalid: the repair pass re-scans this file
    const FileDesc fd = a.files[fi];
    const uint64_t c0 = (t - fd.first_chunk) * (uint64_t)a.chunk;
    const uint32_t cw = a.count[t], n = cw & kCountMask;
    const uint64_t dst0 = row_off[fi] + a.base[t];
    const u32x4* src = (const u32x4*)(a.slots + (uint64_t)t * a.slot_cap * 4);
    if (cw & kCountRegular) {  // rows from the first: equal lengths, consecutive sequences, all Ok
      const u32x4 w = ((const u32x4*)a.desc)[t];
      const uint64_t p0 = c0 + ((w.w >> 16) & 0x7FFFu);
      const uint32_t ksz = w.w & 0xFFFFu;
      const uint64_t rl = 18ull + ksz + ((w.z == 0xFFFFFFFFu) ? 0ull : (uint64_t)w.z);
      const uint64_t seq0 = (uint64_t)w.x | ((uint64_t)w.y << 32);
      for (uint32_t r = lane; r < n; r += 64) {
        const uint64_t d = dst0 + r;
        if (d < a.row_cap) {
          a.pos[d] = p0 + r * rl;
          a.seq[d] = seq0 + r;
          a.vsz[d] = w.z;
          a.ksz[d] = (uint16_t)ksz;
          a.status[d] = kRowOk;
        }
      }
      continue;
    }
    for (uint32_t r = lane; r < n; r += 64) {
      const u32x4 w = src[r];
      const uint64_t p = c0 + ((w.w >> 16) & 0x7FFFu);
      const uint32_t ksz = w.w & 0xFFFFu;
      const uint64_t hb = a.hint ? 22ull : 18ull;
      const uint64_t end = p + hb + ksz + ((a.hint || w.z == 0xFFFFFFFFu) ? 0ull : (uint64_t)w.z);
      const uint8_t st = (p + hb > fd.len || end > fd.len) ? kRowEof : (w.w & kSlotBad) ? kRowChecksum : kRowOk;
      const uint64_t d = dst0 + r;
      if (d < a.row_cap) {
        a.pos[d] = p;
        a.seq[d] = (uint64_t)w.x | ((uint64_t)w.y << 32);
        a.vsz[d] = w.z;
        a.ksz[d] = (uint16_t)ksz;
        a.status[d] = st;
      }
    }
  }
}

// ------------------------------------------------------------------------------------------
// K_walk (repair): exact boundary chain from the first invalid chunk of a file, one wave per
// file. Rewrites spec[] for that chunk onward; the re-scan then runs with exact=1.
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(64) void k_walk(ScanArgs a, const uint64_t* summary) {
  const uint32_t f = blockIdx.x, lane = threadIdx.x;
  const uint64_t* row_off = summary + sizeof(SummaryHead) / 8;
  const uint64_t* fbad = row_off + a.nfiles + 1;
  const uint64_t* badT = fbad + a.nfiles;
  const uint64_t cb = fbad[f];
  if (cb == kNone) return;
  const FileDesc fd = a.files[f];
  const uint64_t len = fd.len;
  const uint64_t CHK = a.chunk;
  uint64_t* spec = a.spec + fd.first_chunk;
  uint64_t cur = cb;  // next chunk whose start is not yet written
  uint64_t p = badT[f];
  uint64_t steps = 0;
  while (p < len) {
    ++steps;
    const uint8_t* hp = fd.data + p;
    bool eof = (p + 18 > len);
    const uint64_t rl = eof ? 0 : g_reclen(hp);
    if (!eof && p + rl > len) eof = true;
    if (eof) {  // the chain ends with this record (an UnexpectedEof row)
      const uint64_t ci = p / CHK;
      for (uint64_t g = cur + lane; g < ci; g += 64) spec[g] = kNone;
      if (lane == 0 && ci >= cur) spec[ci] = p;
      cur = ci + 1 > cur ? ci + 1 : cur;
      break;
    }
    const uint64_t q = p + (uint64_t)lane * rl;
    bool v = true;
    if (lane) {
      v = (q + 18 <= len);
      if (v) v = (g_reclen(fd.data + q) == rl) && (q + rl <= len);
    }
    const unsigned long long okm = __ballot(v);
    const uint32_t k = (~okm) ? (uint32_t)__builtin_ctzll(~okm) : 64u;
    if (lane < k) {
      const uint64_t ci = q / CHK;
      const uint64_t prevc = (lane == 0) ? (cur == 0 ? ~0ull : cur - 1) : (q - rl) / CHK;
      if (lane == 0 ? (ci >= cur) : (ci != prevc)) {
        spec[ci] = q;
        const uint64_t gs = (lane == 0) ? cur : prevc + 1;
        for (uint64_t g = gs; g < ci; ++g) spec[g] = kNone;
      }
    }
    const uint64_t lastq = p + (uint64_t)(k - 1) * rl;
    const uint64_t lc = lastq / CHK;
    cur = lc + 1 > cur ? lc + 1 : cur;
    p += (uint64_t)k * rl;
  }
  for (uint64_t g = cur + lane; g < fd.nchunks; g += 64) spec[g] = kNone;
  if (lane == 0) atomicAdd(&a.ctr->walk_steps, (unsigned long long)steps);
}

// Error detail of one failing slot row (error path only):
// out[0] stored checksum, out[1] computed XXH32, out[2] row status, out[3..4] pos.
__global__ void k_err_detail(ScanArgs a, uint32_t fi, uint64_t slot, uint32_t* out) {
  if (threadIdx.x || blockIdx.x) return;
  const FileDesc fd = a.files[fi];
  const uint32_t* w = a.slots + slot * 4;
  const uint64_t t = slot / a.slot_cap;
  const uint64_t p = (t - fd.first_chunk) * (uint64_t)a.chunk + ((w[3] >> 16) & 0x7FFFu);
  out[0] = 0;
  out[1] = 0;
  out[2] = kRowEof;
  out[3] = (uint32_t)p;
  out[4] = (uint32_t)(p >> 32);
  if (p + 18 > fd.len) return;
  const uint8_t* hp = fd.data + p;
  const uint64_t rl = g_reclen(hp);
  out[0] = gld4(hp);
  if (p + rl > fd.len) return;
  out[1] = gbl_xxh32(hp + 4, rl - 4);
  out[2] = (w[3] & kSlotBad) ? kRowChecksum : kRowOk;
}

// ------------------------------------------------------------------------------------------
static inline hipStream_t S(void* s) { return (hipStream_t)s; }

int device_cus() {
  static int cached[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (!cached[dev]) {
    int cus = 256;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    cached[dev] = cus > 0 ? cus : 256;
  }
  return cached[dev];
}

void launch_long_enqueue(const ScanArgs& a, void* stream) {
  const uint64_t t_hi = a.t_hi ? a.t_hi : a.total_chunks;
  if (t_hi <= a.t_lo) return;
  uint64_t blocks = (t_hi - a.t_lo + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(k_long_enqueue, dim3((uint32_t)blocks), dim3(256), 0, S(stream), a);
}
void launch_long_hash(const ScanArgs& a, void* stream) {
  if (!a.total_chunks) return;
  const int cus = device_cus();
  hipLaunchKernelGGL(k_long_hash, dim3((uint32_t)cus * 8u), dim3(256), 0, S(stream), a);
}
void launch_long(const ScanArgs& a, void* stream, bool enqueue) {
  if (!a.total_chunks) return;
  if (enqueue) launch_long_enqueue(a, stream);
  launch_long_hash(a, stream);
}
void launch_validate(const ScanArgs& a, void* stream) {
  if (!a.nfiles) return;
  // k_val_files runs even with no tiles at all (every file empty): it writes the file totals
  if (a.total_tiles) hipLaunchKernelGGL(k_val_reduce, dim3((uint32_t)a.total_tiles), dim3(256), 0, S(stream), a);
  hipLaunchKernelGGL(k_val_files, dim3(a.nfiles), dim3(256), 0, S(stream), a);
  if (a.total_tiles) hipLaunchKernelGGL(k_val_apply, dim3((uint32_t)a.total_tiles), dim3(256), 0, S(stream), a);
}
void launch_summary(const ScanArgs& a, uint64_t* summary, void* stream) {
  hipLaunchKernelGGL(k_summary, dim3(1), dim3(256), 0, S(stream), a, summary);
}
// K_read_entries (compaction, cask.rs:505-508 -> Log::read_entry, log.rs:150-166 ->
// Entry::from_read, data.rs:161-206): the live records only, verified where the hints say they
// are — not a re-scan of their files. One quad of lanes per record (quad_gbl_xxh32).
__global__ __launch_bounds__(256) void k_read_entries(const uint64_t* __restrict__ pos, const uint32_t* __restrict__ src,
                                                      uint64_t n, const uint8_t* const* __restrict__ srcs,
                                                      const uint64_t* __restrict__ slen, uint64_t* len_out, uint8_t* st_out,
                                                      uint32_t* exp_out, uint32_t* found_out) {
  const uint32_t q = threadIdx.x & 3;
  const uint64_t nq = (uint64_t)gridDim.x * (blockDim.x >> 2);
  for (uint64_t r = blockIdx.x * (uint64_t)(blockDim.x >> 2) + (threadIdx.x >> 2); r < n; r += nq) {
    const uint64_t p = pos[r];
    const uint32_t s = src[r];
    const uint64_t L = slen[s];
    const uint8_t* d = srcs[s];
    uint64_t rl = 0;
    uint8_t st = kRowEof;
    uint32_t stored = 0, got = 0;
    if (p + 18 <= L) {  // read_exact(header) (data.rs:163)
      stored = gld4(d + p);
      rl = g_reclen(d + p);
      if (p + rl <= L) {  // read_exact(key), read_exact(value) (data.rs:172,181)
        got = quad_gbl_xxh32(d + p + 4, rl - 4, q);
        st = got == stored ? kRowOk : kRowChecksum;  // data.rs:193-198
      } else {
        rl = 0;
      }
    }
    if (q == 0) {
      len_out[r] = rl;
      st_out[r] = st;
      exp_out[r] = stored;
      found_out[r] = got;
    }
  }
}

void launch_read_entries(const uint64_t* pos, const uint32_t* src, uint64_t n, const uint8_t* const* srcs,
                         const uint64_t* slen, uint64_t* len, uint8_t* st, uint32_t* expct, uint32_t* found, void* stream) {
  if (!n) return;
  uint64_t g = (n + 63) / 64;
  if (g > 16384) g = 16384;
  hipLaunchKernelGGL(k_read_entries, dim3((uint32_t)g), dim3(256), 0, S(stream), pos, src, n, srcs, slen, len, st, expct, found);
}

void launch_compact(const ScanArgs& a, const uint64_t* summary, void* stream) {
  if (!a.total_chunks) return;
  // one wave per chunk where possible: each chunk's rows wait on a chain of dependent table loads
  // (file, count, base, descriptor), so the launch needs many chunks in flight
  uint64_t g = (a.total_chunks + 3) / 4;
  if (g > 65536) g = 65536;
  hipLaunchKernelGGL(k_compact, dim3((uint32_t)g), dim3(256), 0, S(stream), a, summary);
}
void launch_finish(const ScanArgs& a, void* stream) {
  if (!a.total_chunks) return;
  const uint64_t tiles = (a.total_chunks + kFinTile - 1) / kFinTile;
  ScanArgs af = a;
  af.fin_static = tiles <= 4ull * (uint64_t)device_cus() ? 1u : 0u;  // 4 of its workgroups fit a CU
  hipLaunchKernelGGL(k_finish, dim3((uint32_t)tiles), dim3(kFinTile), 0, S(stream), af);
}
void launch_err_dense(const ScanArgs& a, uint32_t fi, uint64_t row, uint32_t* out, void* stream) {
  hipLaunchKernelGGL(k_err_dense, dim3(1), dim3(64), 0, S(stream), a, fi, row, out);
}
void launch_walk(const ScanArgs& a, const uint64_t* summary, void* stream) {
  if (!a.nfiles) return;
  hipLaunchKernelGGL(k_walk, dim3(a.nfiles), dim3(64), 0, S(stream), a, summary);
}
void launch_err_detail(const ScanArgs& a, uint32_t fi, uint64_t slot, uint32_t* out, void* stream) {
  hipLaunchKernelGGL(k_err_detail, dim3(1), dim3(64), 0, S(stream), a, fi, slot, out);
}

}  // namespace cask_dev
