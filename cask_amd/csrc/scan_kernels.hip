// HIP kernels (gfx950 / CDNA4) for the Cask data-file scan.
//
// The reference walks each data file record by record on one CPU thread:
//   Entries::next (log.rs:403-429) -> Entry::from_read (data.rs:161-206)
// reading an 18-byte header `xxh32 u32 | seq u64 | ksz u16 | vsz u32` (LE), the key, the value
// (absent for a tombstone, vsz == 0xFFFFFFFF) and checking XXH32(header[4..] ‖ key ‖ value).
//
// Here a file is cut into 32 KiB chunks, one workgroup per chunk (k_scan_chunks):
//   1. stage the chunk (+4 KiB halo) into LDS with coalesced 16-B loads;
//   2. find the chunk's first record boundary speculatively: the lowest offset whose header
//      gives a record that fits the window AND whose XXH32 matches its stored checksum;
//   3. walk the boundary chain inside LDS (a wave tests 64 equal-stride successors at once);
//   4. publish the row count with a decoupled look-back, so rows land in file order;
//   5. hash one record per lane out of LDS and write SoA rows.
// A record too long for the window is hashed from HBM by k_long. k_validate then checks every
// speculated boundary against its predecessor's chain exit (a segmented max-scan); a mismatch
// (adversarial or corrupt data) sends the file through an exact header walk (k_walk) and a
// re-scan with known boundaries, so the result is exact by construction.
#include <hip/hip_runtime.h>

#include "scan_kernels.h"
#include "xxh32.h"

namespace cask_dev {

using namespace cask_xxh;

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

#define RLX_AGENT __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT

// ------------------------------------------------------------------------------------------
// LDS byte-stream helpers. The window is staged 16-B aligned; records start at arbitrary byte
// offsets, so every unaligned 32-bit word is assembled from two aligned dword reads with
// v_alignbyte_b32 (a byte funnel shift).
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t funnel(uint32_t hi, uint32_t lo, uint32_t sh) {
  return __builtin_amdgcn_alignbyte(hi, lo, sh);
}

// Record length fields at LDS byte index x: returns 18 + ksz + vsz_eff (data.rs:63-65).
__device__ __forceinline__ uint64_t lds_reclen(const uint32_t* w, uint32_t x) {
  uint32_t q = (x + 12) >> 2, sh = (x + 12) & 3;
  uint32_t d0 = w[q], d1 = w[q + 1], d2 = w[q + 2];
  uint32_t b3 = funnel(d1, d0, sh);  // bytes x+12..x+15: ksz | vsz.lo16
  uint32_t b4 = funnel(d2, d1, sh);  // bytes x+16..x+19: vsz.hi16 | ...
  uint32_t ksz = b3 & 0xFFFFu;
  uint32_t vsz = (b3 >> 16) | (b4 << 16);
  uint64_t veff = (vsz == 0xFFFFFFFFu) ? 0ull : (uint64_t)vsz;
  return 18ull + ksz + veff;
}

struct Hdr {
  uint32_t stored;
  uint64_t seq;
  uint32_t ksz;
  uint32_t vsz;
};

__device__ __forceinline__ Hdr lds_hdr(const uint32_t* w, uint32_t x) {
  uint32_t q = x >> 2, sh = x & 3;
  uint32_t d0 = w[q], d1 = w[q + 1], d2 = w[q + 2], d3 = w[q + 3], d4 = w[q + 4], d5 = w[q + 5];
  Hdr h;
  h.stored = funnel(d1, d0, sh);
  uint32_t s0 = funnel(d2, d1, sh), s1 = funnel(d3, d2, sh);
  h.seq = (uint64_t)s0 | ((uint64_t)s1 << 32);
  uint32_t b3 = funnel(d4, d3, sh), b4 = funnel(d5, d4, sh);
  h.ksz = b3 & 0xFFFFu;
  h.vsz = (b3 >> 16) | (b4 << 16);
  return h;
}

// XXH32 (seed 0) of LDS bytes [xs, xs + len).
__device__ __forceinline__ uint32_t lds_xxh32(const uint32_t* w, uint32_t xs, uint32_t len) {
  uint32_t sh = xs & 3;
  uint32_t wi = xs >> 2;
  uint32_t prev = w[wi];
  uint32_t h;
  uint32_t nstr = len >> 4;
  if (nstr) {
    Acc a = acc_init(0);
    for (uint32_t s = 0; s < nstr; ++s) {
      uint32_t d1 = w[wi + 1], d2 = w[wi + 2], d3 = w[wi + 3], d4 = w[wi + 4];
      acc_stripe(a, funnel(d1, prev, sh), funnel(d2, d1, sh), funnel(d3, d2, sh), funnel(d4, d3, sh));
      prev = d4;
      wi += 4;
    }
    h = acc_merge(a);
  } else {
    h = P5;
  }
  h += len;
  uint32_t rem = len & 15;
  while (rem >= 4) {
    uint32_t d1 = w[wi + 1];
    h = tail4(h, funnel(d1, prev, sh));
    prev = d1;
    ++wi;
    rem -= 4;
  }
  const uint8_t* b = (const uint8_t*)w;
  uint32_t xb = (wi << 2) + sh;
  while (rem) {
    h = tail1(h, b[xb]);
    ++xb;
    --rem;
  }
  return avalanche(h);
}

// XXH32 of global bytes [p, p+len) by one lane: unaligned 16-B loads (gfx950 runs in
// unaligned-access mode; the compiler emits global_load_dwordx4 for these memcpys).
__device__ __forceinline__ u32x4 gld16(const uint8_t* p) {
  u32x4 v;
  __builtin_memcpy(&v, p, 16);
  return v;
}
__device__ __forceinline__ uint32_t gld4(const uint8_t* p) {
  uint32_t v;
  __builtin_memcpy(&v, p, 4);
  return v;
}

__device__ uint32_t gbl_xxh32(const uint8_t* p, uint64_t len) {
  const uint8_t* end = p + len;
  uint32_t h;
  if (len >= 16) {
    Acc a = acc_init(0);
    uint64_t nstr = len >> 4;
    for (uint64_t s = 0; s < nstr; ++s) {
      u32x4 v = gld16(p);
      acc_stripe(a, v.x, v.y, v.z, v.w);
      p += 16;
    }
    h = acc_merge(a);
  } else {
    h = P5;
  }
  h += (uint32_t)len;
  while (p + 4 <= end) {
    h = tail4(h, gld4(p));
    p += 4;
  }
  while (p < end) {
    h = tail1(h, *p);
    ++p;
  }
  return avalanche(h);
}

__device__ __forceinline__ uint64_t g_reclen(const uint8_t* hdr) {
  uint32_t b3 = gld4(hdr + 12);
  uint32_t b4 = (uint32_t)hdr[16] | ((uint32_t)hdr[17] << 8);
  uint32_t ksz = b3 & 0xFFFFu;
  uint32_t vsz = (b3 >> 16) | (b4 << 16);
  return 18ull + ksz + ((vsz == 0xFFFFFFFFu) ? 0ull : (uint64_t)vsz);
}

__device__ __forceinline__ uint32_t find_file(const FileDesc* files, uint32_t nfiles, uint64_t t) {
  // last file with first_chunk <= t (empty files share first_chunk with their successor)
  uint32_t lo = 0, hi = nfiles;  // answer in [lo, hi)
  while (hi - lo > 1) {
    uint32_t mid = (lo + hi) >> 1;
    if (files[mid].first_chunk <= t) lo = mid; else hi = mid;
  }
  return lo;
}

// ------------------------------------------------------------------------------------------
// Decoupled look-back (one wave). Words: flag in bits 63..62 (1 aggregate, 2 inclusive),
// value in bits 61..0. Each word is one 8-B agent-scope atomic store, so the value IS the flag
// (no fence needed); polls are relaxed agent-scope loads with s_sleep and a spin bound.
// ------------------------------------------------------------------------------------------
constexpr unsigned long long kFlagAgg = 1ull << 62, kFlagInc = 2ull << 62, kValMask = (1ull << 62) - 1;

__device__ __forceinline__ unsigned long long wave_sum64(unsigned long long v) {
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ unsigned long long lookback_exclusive(unsigned long long* lb, uint64_t t, uint32_t lane,
                                                 Counters* ctr) {
  unsigned long long excl = 0;
  int64_t j = (int64_t)t - 1;
  while (j >= 0) {
    int64_t idx = j - (int64_t)lane;
    unsigned long long w = kFlagInc;  // lanes past chunk 0 act as an inclusive zero
    if (idx >= 0) {
      uint32_t spins = 0;
      for (;;) {
        w = __hip_atomic_load(&lb[idx], RLX_AGENT);
        if (w >> 62) break;
        if (++spins > (1u << 24)) {
          atomicOr(&ctr->timeout, 1u);
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
    }
    bool inc = (w >> 62) == 2;
    unsigned long long mask = __ballot(inc);
    if (mask) {
      uint32_t first = __builtin_ctzll(mask);
      unsigned long long v = (lane <= first) ? (w & kValMask) : 0ull;
      excl += wave_sum64(v);
      break;
    }
    excl += wave_sum64(w & kValMask);
    j -= 64;
  }
  return excl;
}

// ------------------------------------------------------------------------------------------
// K1: chunk scan
// ------------------------------------------------------------------------------------------
struct __attribute__((aligned(16))) ScanLds {
  uint32_t win[(kWin + 64) / 4];   // staged bytes (16-B aligned base + up to 15 B shift + slop)
  uint16_t starts[kMaxStarts];     // record starts, relative to the chunk start
  uint64_t t, base, spec, exitv;
  uint32_t fi, n, found;
};

__global__ __launch_bounds__(kWG) void k_scan_chunks(ScanArgs a) {
  __shared__ ScanLds L;
  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;

  if (tid == 0) {
    uint64_t t = atomicAdd(&a.ctr->ticket, 1ull);  // in-order grab: predecessors are resident
    L.t = t;
    L.fi = find_file(a.files, a.nfiles, t);
    L.found = 0xFFFFFFFFu;
  }
  __syncthreads();
  const uint64_t t = L.t;
  const uint32_t fi = L.fi;
  const FileDesc fd = a.files[fi];
  const uint64_t len = fd.len;
  const uint64_t c0 = (t - fd.first_chunk) * (uint64_t)kChunk;
  const uint64_t c1 = (c0 + kChunk < len) ? c0 + kChunk : len;
  const uint64_t wend = (c0 + kWin < len) ? c0 + kWin : len;

  // 1. stage [c0, wend) into LDS: aligned 16-B granules, coalesced across the workgroup.
  const uintptr_t gstart = (uintptr_t)(fd.data + c0);
  const uintptr_t a0 = gstart & ~(uintptr_t)15;
  const uint32_t shift = (uint32_t)(gstart - a0);
  const uintptr_t aend = ((uintptr_t)(fd.data + wend) + 15) & ~(uintptr_t)15;
  const uint32_t n16 = (uint32_t)((aend - a0) >> 4);
  {
    const u32x4* src = (const u32x4*)a0;
    u32x4* dst = (u32x4*)L.win;
    for (uint32_t i = tid; i < n16; i += kWG) dst[i] = src[i];
  }
  __syncthreads();
  const uint32_t* W = L.win;

  // 2. the chunk's first record boundary
  uint64_t s;
  if (a.exact) {
    s = a.spec[t];
  } else if (c0 == 0) {
    s = 0;  // a file's first record starts at 0 (log.rs:116)
  } else {
    const uint32_t span = (uint32_t)(c1 - c0);
    for (uint32_t kb = 0; kb < span; kb += kWG) {
      uint32_t k = kb + tid;
      if (k < span) {
        uint64_t p = c0 + k;
        if (p + 18 <= len) {
          uint32_t x = k + shift;
          uint64_t rl = lds_reclen(W, x);
          uint64_t end = p + rl;
          if (end <= wend) {  // record fits the window: verify its checksum here
            Hdr h = lds_hdr(W, x);
            if (lds_xxh32(W, x + 4, (uint32_t)rl - 4) == h.stored) atomicMin(&L.found, k);
          }
        }
      }
      __syncthreads();
      bool done = L.found != 0xFFFFFFFFu;
      __syncthreads();
      if (done) break;
    }
    s = (L.found != 0xFFFFFFFFu) ? c0 + L.found : kNone;
  }

  // 3. walk the chain inside the window (wave 0). Each step tests 64 equal-stride successors.
  if (wave == 0) {
    uint32_t n = 0;
    uint64_t exitv = 0;
    if (s != kNone) {
      uint64_t p = s;
      for (;;) {
        if (p >= c1) { exitv = p; break; }
        if (p + 18 > len) {  // header cut short: Io(UnexpectedEof) (data.rs:163)
          if (lane == 0) L.starts[n] = (uint16_t)(p - c0);
          ++n;
          exitv = kTerm;
          break;
        }
        const uint64_t rl = lds_reclen(W, (uint32_t)(p - c0) + shift);
        if (p + rl > len) {  // key/value cut short (data.rs:172,181)
          if (lane == 0) L.starts[n] = (uint16_t)(p - c0);
          ++n;
          exitv = kTerm;
          break;
        }
        const uint64_t q = p + (uint64_t)lane * rl;
        bool v = true;
        if (lane) {
          v = (q < c1) && (q + 18 <= len);
          if (v) {
            uint64_t rq = lds_reclen(W, (uint32_t)(q - c0) + shift);
            v = (rq == rl) && (q + rl <= len);
          }
        }
        unsigned long long okm = __ballot(v);
        uint32_t k = (~okm) ? (uint32_t)__builtin_ctzll(~okm) : 64u;
        if (lane < k) L.starts[n + lane] = (uint16_t)(q - c0);
        n += k;
        p += (uint64_t)k * rl;
      }
    }
    // 4. publish this chunk's row count, look back for the exclusive prefix.
    unsigned long long base;
    if (t == 0) {
      base = 0;
      if (lane == 0) __hip_atomic_store(&a.lb[0], kFlagInc | (unsigned long long)n, RLX_AGENT);
    } else {
      if (lane == 0) __hip_atomic_store(&a.lb[t], kFlagAgg | (unsigned long long)n, RLX_AGENT);
      base = lookback_exclusive(a.lb, t, lane, a.ctr);
      if (lane == 0) __hip_atomic_store(&a.lb[t], kFlagInc | (base + n), RLX_AGENT);
    }
    if (lane == 0) {
      L.n = n;
      L.base = base;
      L.spec = s;
      L.exitv = (s == kNone) ? 0 : exitv;
    }
  }
  __syncthreads();

  const uint32_t n = L.n;
  const uint64_t base = L.base;
  if (tid == 0) {
    if (!a.exact) a.spec[t] = s;
    a.exit[t] = L.exitv;
    a.base[t] = base;
    a.count[t] = n;
  }
  const bool fits = base + n <= a.row_cap;
  if (!fits) {
    if (tid == 0) atomicOr(&a.ctr->overflow, 1u);
    return;
  }

  // 5. one record per lane: verify and emit rows.
  for (uint32_t r = tid; r < n; r += kWG) {
    const uint64_t p = c0 + L.starts[r];
    const uint32_t x = L.starts[r] + shift;
    uint64_t seq = 0;
    uint32_t ksz = 0, vsz = 0;
    uint8_t st;
    if (p + 18 > len) {
      st = kRowEof;
    } else {
      Hdr h = lds_hdr(W, x);
      seq = h.seq;
      ksz = h.ksz;
      vsz = h.vsz;
      uint64_t rl = 18ull + ksz + ((vsz == 0xFFFFFFFFu) ? 0ull : (uint64_t)vsz);
      uint64_t end = p + rl;
      if (end > len) {
        st = kRowEof;
      } else if (end <= wend) {
        st = (lds_xxh32(W, x + 4, (uint32_t)rl - 4) == h.stored) ? kRowOk : kRowChecksum;
      } else {
        st = kRowPendingLong;
        unsigned long long li = atomicAdd(&a.ctr->nlong, 1ull);
        if (li < a.long_cap) {
          a.long_row[li] = base + r;
          a.long_file[li] = fi;
        }
      }
    }
    const uint64_t row = base + r;
    a.pos[row] = p;
    a.seq[row] = seq;
    a.ksz[row] = (uint16_t)ksz;
    a.vsz[row] = vsz;
    a.status[row] = st;
    if (st == kRowChecksum || st == kRowEof) atomicMin(&a.file_err_row[fi], (unsigned long long)row);
  }
}

// ------------------------------------------------------------------------------------------
// K_long: records longer than the LDS window, one lane each, straight from HBM.
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_long(ScanArgs a) {
  const uint64_t n = a.ctr->nlong < a.long_cap ? a.ctr->nlong : a.long_cap;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t row = a.long_row[i];
    const uint32_t fi = a.long_file[i];
    const uint8_t* base = a.files[fi].data;
    const uint64_t p = a.pos[row];
    const uint32_t vsz = a.vsz[row];
    const uint64_t rl = 18ull + a.ksz[row] + ((vsz == 0xFFFFFFFFu) ? 0ull : (uint64_t)vsz);
    const uint32_t stored = gld4(base + p);
    const uint32_t h = gbl_xxh32(base + p + 4, rl - 4);
    const uint8_t st = (h == stored) ? kRowOk : kRowChecksum;
    a.status[row] = st;
    if (st != kRowOk) atomicMin(&a.file_err_row[fi], (unsigned long long)row);
  }
}

// ------------------------------------------------------------------------------------------
// K_validate: one workgroup per file. T[c] = max over earlier chunks' exits (0 for chunks that
// found no start) is the true chain position entering chunk c as long as every earlier chunk is
// valid; chunk c is valid iff its speculated start equals T[c] (or it found none and T[c] is
// already past its end).
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_validate(ScanArgs a, uint64_t* first_bad) {
  __shared__ unsigned long long wmax[4];
  __shared__ unsigned long long bad;
  const uint32_t f = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const FileDesc fd = a.files[f];
  if (tid == 0) bad = kNone;
  __syncthreads();
  unsigned long long carry = 0;
  for (uint64_t tb = 0; tb < fd.nchunks; tb += 256) {
    const uint64_t c = tb + tid;
    const bool in = c < fd.nchunks;
    const uint64_t g = fd.first_chunk + c;
    uint64_t sp = kNone, ex = 0;
    if (in) {
      sp = a.spec[g];
      ex = (sp == kNone) ? 0 : a.exit[g];
    }
    // inclusive max-scan of ex across the workgroup
    unsigned long long v = ex;
    for (int o = 1; o < 64; o <<= 1) {
      unsigned long long u = __shfl_up(v, o, 64);
      if ((int)lane >= o) v = v > u ? v : u;
    }
    if (lane == 63) wmax[wave] = v;
    __syncthreads();
    unsigned long long pre = carry;
    for (uint32_t k = 0; k < wave; ++k) pre = pre > wmax[k] ? pre : wmax[k];
    unsigned long long excl_lane = __shfl_up(v, 1, 64);
    unsigned long long T = pre;
    if (lane > 0) T = T > excl_lane ? T : excl_lane;
    if (in) {
      a.tin[g] = T;
      const uint64_t c0 = c * (uint64_t)kChunk;
      const uint64_t c1 = (c0 + kChunk < fd.len) ? c0 + kChunk : fd.len;
      bool ok;
      if (c == 0) ok = true;
      else if (sp != kNone) ok = (sp == T);
      else ok = (T >= c1);
      if (!ok) atomicMin(&bad, (unsigned long long)c);
    }
    unsigned long long tile = wmax[0];
    for (uint32_t k = 1; k < 4; ++k) tile = tile > wmax[k] ? tile : wmax[k];
    carry = carry > tile ? carry : tile;
    __syncthreads();
  }
  if (tid == 0) first_bad[f] = bad;
}

// Summary: row offsets per file, totals, flags -> one buffer the host copies back.
__global__ void k_summary(ScanArgs a, const uint64_t* first_bad, uint64_t* out) {
  SummaryHead* h = (SummaryHead*)out;
  uint64_t* row_off = out + sizeof(SummaryHead) / 8;
  uint64_t* fbad = row_off + a.nfiles + 1;
  uint64_t* badT = fbad + a.nfiles;
  uint64_t* err = badT + a.nfiles;
  const uint64_t total = a.total_chunks ? a.base[a.total_chunks - 1] + a.count[a.total_chunks - 1] : 0;
  for (uint32_t f = threadIdx.x; f <= a.nfiles; f += blockDim.x) {
    if (f == a.nfiles) {
      row_off[f] = total;
      continue;
    }
    const FileDesc fd = a.files[f];
    row_off[f] = (fd.first_chunk < a.total_chunks) ? a.base[fd.first_chunk] : total;
    const uint64_t b = first_bad ? first_bad[f] : kNone;
    fbad[f] = b;
    badT[f] = (b != kNone) ? a.tin[fd.first_chunk + b] : 0;
    err[f] = a.file_err_row[f];
  }
  if (threadIdx.x == 0) {
    h->total_rows = total;
    h->nlong = a.ctr->nlong;
    h->overflow = a.ctr->overflow;
    h->timeout = a.ctr->timeout;
    uint64_t any = 0, cnt = 0;
    if (first_bad)
      for (uint32_t f = 0; f < a.nfiles; ++f)
        if (first_bad[f] != kNone) { any = 1; cnt += a.files[f].nchunks - first_bad[f]; }
    h->any_invalid = any;
    h->invalid_chunks = cnt;
    h->walk_steps = a.ctr->walk_steps;
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
  uint64_t* spec = a.spec + fd.first_chunk;
  uint64_t cur = cb;  // next chunk whose start is not yet written
  uint64_t p = badT[f];
  uint64_t steps = 0;
  while (p < len) {
    ++steps;
    const uint8_t* hp = fd.data + p;
    bool eof = (p + 18 > len);
    uint64_t rl = eof ? 0 : g_reclen(hp);
    if (!eof && p + rl > len) eof = true;
    if (eof) {  // the chain ends with this record (an UnexpectedEof row)
      const uint64_t ci = p / kChunk;
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
    unsigned long long okm = __ballot(v);
    const uint32_t k = (~okm) ? (uint32_t)__builtin_ctzll(~okm) : 64u;
    if (lane < k) {
      const uint64_t ci = q / kChunk;
      const uint64_t prevc = (lane == 0) ? (cur == 0 ? ~0ull : cur - 1) : (q - rl) / kChunk;
      if (lane == 0 ? (ci >= cur) : (ci != prevc)) {
        spec[ci] = q;
        const uint64_t gs = (lane == 0) ? cur : prevc + 1;
        for (uint64_t g = gs; g < ci; ++g) spec[g] = kNone;
      }
    }
    const uint64_t lastq = p + (uint64_t)(k - 1) * rl;
    const uint64_t lc = lastq / kChunk;
    cur = lc + 1 > cur ? lc + 1 : cur;
    p += (uint64_t)k * rl;
  }
  for (uint64_t g = cur + lane; g < fd.nchunks; g += 64) spec[g] = kNone;
  if (lane == 0) atomicAdd(&a.ctr->walk_steps, (unsigned long long)steps);
}

// Expected/found checksum of one failing row (error path only).
__global__ void k_err_detail(ScanArgs a, uint32_t fi, uint64_t row, uint32_t* out2) {
  if (threadIdx.x || blockIdx.x) return;
  const FileDesc fd = a.files[fi];
  const uint64_t p = a.pos[row];
  out2[0] = 0;
  out2[1] = 0;
  if (p + 18 > fd.len) return;
  const uint8_t* hp = fd.data + p;
  const uint64_t rl = g_reclen(hp);
  out2[0] = gld4(hp);
  if (p + rl > fd.len) return;
  out2[1] = gbl_xxh32(hp + 4, rl - 4);
}

// ------------------------------------------------------------------------------------------
// Encoder (Entry::write_bytes, data.rs:90-121): pass 1 writes header tail + key + value bytes,
// pass 2 hashes [off+4, off+len) and stores the checksum at off.
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ uint64_t splitmix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__device__ __forceinline__ void put_hdr_tail(uint8_t* o, uint64_t seq, uint16_t ksz, uint32_t vsz) {
  for (int i = 0; i < 8; ++i) o[4 + i] = (uint8_t)(seq >> (8 * i));
  o[12] = (uint8_t)ksz;
  o[13] = (uint8_t)(ksz >> 8);
  for (int i = 0; i < 4; ++i) o[14 + i] = (uint8_t)(vsz >> (8 * i));
}

__global__ __launch_bounds__(256) void k_encode_synth(uint64_t nrec, const uint64_t* off,
                                                      const uint64_t* seq, const uint16_t* ksz,
                                                      const uint32_t* vsz_raw, const uint64_t* key_id,
                                                      uint64_t value_seed, uint8_t* out) {
  for (uint64_t r = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; r < nrec;
       r += (uint64_t)gridDim.x * blockDim.x) {
    uint8_t* o = out + off[r];
    const uint16_t k = ksz[r];
    const uint32_t v = vsz_raw[r];
    put_hdr_tail(o, seq[r], k, v);
    const uint64_t kid = key_id[r];
    for (uint32_t j = 0; j < k; j += 8) {
      uint64_t wv = splitmix64((kid << 16) | (j >> 3));
      for (uint32_t b = 0; b < 8 && j + b < k; ++b) o[18 + j + b] = (uint8_t)(wv >> (8 * b));
    }
    if (v != 0xFFFFFFFFu) {
      const uint64_t rs = splitmix64(value_seed + r);
      uint8_t* vo = o + 18 + k;
      for (uint32_t j = 0; j < v; j += 8) {
        uint64_t wv = splitmix64(rs + (j >> 3));
        for (uint32_t b = 0; b < 8 && j + b < v; ++b) vo[j + b] = (uint8_t)(wv >> (8 * b));
      }
    }
  }
}

__global__ __launch_bounds__(256) void k_encode(uint64_t nrec, const uint64_t* off, const uint64_t* seq,
                                                const uint16_t* ksz, const uint32_t* vsz_raw,
                                                const uint8_t* keys, const uint64_t* key_off,
                                                const uint8_t* vals, const uint64_t* val_off,
                                                uint8_t* out) {
  for (uint64_t r = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; r < nrec;
       r += (uint64_t)gridDim.x * blockDim.x) {
    uint8_t* o = out + off[r];
    const uint16_t k = ksz[r];
    const uint32_t v = vsz_raw[r];
    put_hdr_tail(o, seq[r], k, v);
    const uint8_t* ks = keys + key_off[r];
    for (uint32_t j = 0; j < k; ++j) o[18 + j] = ks[j];
    if (v != 0xFFFFFFFFu) {
      const uint8_t* vs = vals + val_off[r];
      for (uint32_t j = 0; j < v; ++j) o[18 + k + j] = vs[j];
    }
  }
}

__global__ __launch_bounds__(256) void k_encode_checksum(uint64_t nrec, const uint64_t* off,
                                                         const uint16_t* ksz, const uint32_t* vsz_raw,
                                                         uint8_t* out) {
  for (uint64_t r = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; r < nrec;
       r += (uint64_t)gridDim.x * blockDim.x) {
    uint8_t* o = out + off[r];
    const uint32_t v = vsz_raw[r];
    const uint64_t rl = 18ull + ksz[r] + ((v == 0xFFFFFFFFu) ? 0ull : (uint64_t)v);
    const uint32_t h = gbl_xxh32(o + 4, rl - 4);
    o[0] = (uint8_t)h;
    o[1] = (uint8_t)(h >> 8);
    o[2] = (uint8_t)(h >> 16);
    o[3] = (uint8_t)(h >> 24);
  }
}

// ------------------------------------------------------------------------------------------
// launchers
// ------------------------------------------------------------------------------------------
static inline hipStream_t S(void* s) { return (hipStream_t)s; }

void launch_scan_chunks(const ScanArgs& a, void* stream) {
  if (!a.total_chunks) return;
  hipLaunchKernelGGL(k_scan_chunks, dim3((uint32_t)a.total_chunks), dim3(kWG), 0, S(stream), a);
}
void launch_long(const ScanArgs& a, void* stream) {
  if (!a.total_chunks) return;
  hipLaunchKernelGGL(k_long, dim3(1024), dim3(256), 0, S(stream), a);
}
void launch_validate(const ScanArgs& a, uint64_t* first_bad, void* stream) {
  if (!a.nfiles) return;
  hipLaunchKernelGGL(k_validate, dim3(a.nfiles), dim3(256), 0, S(stream), a, first_bad);
}
void launch_summary(const ScanArgs& a, const uint64_t* first_bad, uint64_t* summary, void* stream) {
  hipLaunchKernelGGL(k_summary, dim3(1), dim3(256), 0, S(stream), a, first_bad, summary);
}
void launch_walk(const ScanArgs& a, const uint64_t* summary, void* stream) {
  if (!a.nfiles) return;
  hipLaunchKernelGGL(k_walk, dim3(a.nfiles), dim3(64), 0, S(stream), a, summary);
}
void launch_err_detail(const ScanArgs& a, uint32_t fi, uint64_t row, uint32_t* out2, void* stream) {
  hipLaunchKernelGGL(k_err_detail, dim3(1), dim3(64), 0, S(stream), a, fi, row, out2);
}
static inline uint32_t grid_for(uint64_t n) {
  uint64_t g = (n + 255) / 256;
  if (g > 65536) g = 65536;
  return g ? (uint32_t)g : 1u;
}
void launch_encode_synth(uint64_t nrec, const uint64_t* off, const uint64_t* seq, const uint16_t* ksz,
                         const uint32_t* vsz_raw, const uint64_t* key_id, uint64_t value_seed,
                         uint8_t* out, void* stream) {
  if (!nrec) return;
  hipLaunchKernelGGL(k_encode_synth, dim3(grid_for(nrec)), dim3(256), 0, S(stream), nrec, off, seq, ksz,
                     vsz_raw, key_id, value_seed, out);
}
void launch_encode(uint64_t nrec, const uint64_t* off, const uint64_t* seq, const uint16_t* ksz,
                   const uint32_t* vsz_raw, const uint8_t* keys, const uint64_t* key_off,
                   const uint8_t* vals, const uint64_t* val_off, uint8_t* out, void* stream) {
  if (!nrec) return;
  hipLaunchKernelGGL(k_encode, dim3(grid_for(nrec)), dim3(256), 0, S(stream), nrec, off, seq, ksz, vsz_raw,
                     keys, key_off, vals, val_off, out);
}
void launch_encode_checksum(uint64_t nrec, const uint64_t* off, const uint16_t* ksz, const uint32_t* vsz_raw,
                            uint8_t* out, void* stream) {
  if (!nrec) return;
  hipLaunchKernelGGL(k_encode_checksum, dim3(grid_for(nrec)), dim3(256), 0, S(stream), nrec, off, ksz,
                     vsz_raw, out);
}

}  // namespace cask_dev
