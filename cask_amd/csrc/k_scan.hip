// k_scan_chunks — the hot kernel of the Cask data-file scan (gfx950 / CDNA4).
//
// The reference walks each data file record by record on one CPU thread:
//   Entries::next (log.rs:403-429) -> Entry::from_read (data.rs:161-206)
// reading the 18-byte header `xxh32 u32 | seq u64 | ksz u16 | vsz u32` (LE), the key, the value
// (absent for a tombstone, vsz == 0xFFFFFFFF) and checking XXH32(header[4..] ‖ key ‖ value).
//
// Here every file is cut into fixed-size chunks and a persistent grid streams through them.
// Per chunk, one workgroup:
//   1. has the chunk (+ halo) staged into LDS: the 16-B loads for chunk i+1 are issued into
//      registers before chunk i is processed, so HBM latency hides behind the work;
//   2. finds the chunk's first record boundary speculatively: the lowest offset whose header gives
//      a record that fits the window and whose XXH32 matches its stored checksum (short records
//      first, so long false candidates are rarely hashed);
//   3. walks the boundary chain inside LDS (a wave tests 64 equal-stride successors per step);
//   4. hashes one record per lane out of LDS and writes one 16-B slot row per record into the
//      chunk's own slot range.
// No workgroup ever waits on another: boundary speculation is checked afterwards (k_validate)
// and rows are ordered by a later pass (k_compact), both in k_pipeline.hip.
#include "device_util.h"

#include <stdlib.h>

namespace cask_dev {

template <uint32_t CH, uint32_t HALO, uint32_t NT, uint32_t PER_CU>
struct Geo {
  static constexpr uint32_t kCh = CH, kHaloB = HALO, kNT = NT, kWinB = CH + HALO, kPerCU = PER_CU;
  static constexpr uint32_t kMaxStartsG = CH / 18 + 2;  // every record is >= 18 bytes
  static constexpr uint32_t kWinWords = (kWinB + 64) / 4;
  static constexpr uint32_t kNL = ((kWinB + 32) / 16 + NT - 1) / NT;  // 16-B loads per thread
};

// Records no longer than this are "short": the boundary search verifies them first.
constexpr uint32_t kShortMax = 1024;

// Diagnostic (-DCASK_BAR_CHECK): every thread counts the barriers it passed; after the walk
// barrier each wave compares its count with wave 0's and records a mismatch in stamps[8..].
#ifdef CASK_BAR_CHECK
#define BAR()        \
  {                  \
    __syncthreads(); \
    ++dg.nb;         \
  }
#else
#define BAR() __syncthreads()
#endif

template <class G>
struct __attribute__((aligned(16))) ScanLdsT {
  uint32_t win[G::kWinWords];        // staged bytes (16-B aligned base + <= 15 B shift + slop)
  uint16_t starts[G::kMaxStartsG];   // record starts relative to the chunk start
  uint32_t found, n;
#ifdef CASK_BAR_CHECK
  uint32_t nb0;
#endif
};

struct ChunkPos {
  const uint8_t* data;
  uint64_t len, c0, c1, wend;
  uintptr_t a0;
  uint32_t fi, shift, n16;
};

template <class G>
__device__ __forceinline__ ChunkPos locate(const FileDesc* files, uint32_t nfiles, uint64_t t) {
  ChunkPos c;
  c.fi = find_file(files, nfiles, t);
  DCHECK(c.fi < nfiles, "fi %u t %llu", c.fi, (unsigned long long)t);
  const FileDesc fd = files[c.fi];
  DCHECK(t >= fd.first_chunk && t < fd.first_chunk + fd.nchunks, "fi %u t %llu first %llu n %llu", c.fi,
         (unsigned long long)t, (unsigned long long)fd.first_chunk, (unsigned long long)fd.nchunks);
  c.data = fd.data;
  c.len = fd.len;
  c.c0 = (t - fd.first_chunk) * (uint64_t)G::kCh;
  c.c1 = (c.c0 + G::kCh < c.len) ? c.c0 + G::kCh : c.len;
  c.wend = (c.c0 + G::kWinB < c.len) ? c.c0 + G::kWinB : c.len;
  const uintptr_t gstart = (uintptr_t)(c.data + c.c0);
  c.a0 = gstart & ~(uintptr_t)15;
  c.shift = (uint32_t)(gstart - c.a0);
  const uintptr_t aend = ((uintptr_t)(c.data + c.wend) + 15) & ~(uintptr_t)15;
  c.n16 = (uint32_t)((aend - c.a0) >> 4);
  return c;
}

// Issue every 16-B load of a window (clamped index: no branch around a load, so all of them are
// in flight at once); the data lands in LDS later, in stage_store.
// Global (address space 1) view of the staged bytes. Without it the loads compile to flat_load,
// which also count on lgkmcnt and retire out of order with LDS reads: a counted LDS wait in the
// walk could then be satisfied by a prefetch load instead of its own read.
typedef __attribute__((address_space(1))) const u32x4 gu32x4;

// Diagnostic (-DCASK_ADDR_GUARD, stamps builds): an address outside [lo, hi) is recorded in
// stamps[8..15] and replaced by lo instead of being accessed.
#ifdef CASK_ADDR_GUARD
#define ADDR_GUARD(stamps, ptr, lo, hi, tag, t)                                                      \
  if ((uintptr_t)(ptr) < (uintptr_t)(lo) || (uintptr_t)(ptr) >= (uintptr_t)(hi)) {                  \
    if ((stamps) && atomicCAS(&(stamps)[8], 0ull, (unsigned long long)(tag)) == 0ull) {            \
      (stamps)[9] = (uintptr_t)(ptr); (stamps)[10] = (uintptr_t)(lo); (stamps)[11] = (uintptr_t)(hi); \
      (stamps)[12] = (t); (stamps)[13] = blockIdx.x | ((uint64_t)threadIdx.x << 32);                \
    }                                                                                                \
    (ptr) = (decltype(ptr))(lo);                                                                     \
  }
#else
#define ADDR_GUARD(stamps, ptr, lo, hi, tag, t)
#endif

template <class G>
__device__ __forceinline__ void stage_issue(u32x4 (&v)[G::kNL], const ChunkPos& c,
                                            unsigned long long* dbg = nullptr, uint64_t t = 0) {
  const gu32x4* src = (const gu32x4*)c.a0;
  DCHECK(c.n16 >= 1 && c.n16 <= G::kNL * G::kNT && c.n16 * 16 <= G::kWinWords * 4 &&
             c.a0 >= ((uintptr_t)c.data & ~(uintptr_t)15) && c.a0 + 16ull * c.n16 <= (((uintptr_t)c.data + c.len + 15) & ~(uintptr_t)15),
         "n16 %u a0 %llx data %llx len %llu c0 %llu", c.n16, (unsigned long long)c.a0,
         (unsigned long long)(uintptr_t)c.data, (unsigned long long)c.len, (unsigned long long)c.c0);
#pragma unroll
  for (uint32_t j = 0; j < G::kNL; ++j) {
    const uint32_t i = threadIdx.x + j * G::kNT;
    const gu32x4* ptr = src + (i < c.n16 ? i : c.n16 - 1);
    ADDR_GUARD(dbg, ptr, (uintptr_t)c.data & ~(uintptr_t)15, (uintptr_t)c.data + c.len + 16, 1, t)
    v[j] = *ptr;
  }
}

template <class G>
__device__ __forceinline__ void stage_store(ScanLdsT<G>& L, const u32x4 (&v)[G::kNL], const ChunkPos& c) {
  u32x4* dst = (u32x4*)L.win;
#pragma unroll
  for (uint32_t j = 0; j < G::kNL; ++j) {
    const uint32_t i = threadIdx.x + j * G::kNT;
    if (i < c.n16) dst[i] = v[j];
  }
}

template <class G, bool EXACT>
__device__ __forceinline__ void process_chunk(ScanLdsT<G>& L, const ScanArgs& a, uint64_t t, const ChunkPos& c,
                                              uint64_t s_exact, Diag& dg) {
  constexpr uint32_t NT = G::kNT;
  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const uint32_t* W = L.win;
  const uint64_t len = c.len, c0 = c.c0, c1 = c.c1, wend = c.wend;
  const uint32_t shift = c.shift;
  STAMP_INIT

  // 2. the chunk's first record boundary
  uint64_t s;
  if (EXACT) {
    s = s_exact;
  } else if (c0 == 0) {
    s = 0;  // a file's first record starts at 0 (log.rs:116)
  } else {
    const uint32_t span = (uint32_t)(c1 - c0);
    // pass A: short records starting in the first kShortMax bytes; pass B: everything, in order.
    // Control flow depends on L.found only as read between the two barriers of a step: any other
    // read could see a faster wave's atomicMin of the next step, and the waves' barrier counts
    // would part ways.
    bool found = false;
    for (uint32_t pass = 0; pass < 2 && !found; ++pass) {
      const uint32_t lim = pass == 0 ? (span < kShortMax ? span : kShortMax) : span;
      for (uint32_t kb = 0; kb < lim; kb += NT) {
        const uint32_t k = kb + tid;
        if (k < lim) {
          const uint64_t p = c0 + k;
          if (p + 18 <= len) {
            const uint32_t x = k + shift;
            const uint64_t rl = lds_reclen(W, x);
            if (p + rl <= wend && (pass == 1 || rl <= kShortMax)) {
              const Hdr h = lds_hdr(W, x);
              if (lds_xxh32(W, x + 4, (uint32_t)rl - 4) == h.stored) atomicMin(&L.found, k);
            }
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
  }
  STAMP(0)

  // 3. walk the chain inside the window (wave 0). Each step tests 64 equal-stride successors.
  if (wave == 0) {
    uint32_t n = 0;
    uint64_t exitv = 0;
    uint64_t lastp = 0, lastrl = 0;  // last record of the chunk: the only one that can be long
    if (s != kNone) {
      uint64_t p = s;
      for (;;) {
        if (p >= c1) {
          exitv = p;
          break;
        }
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
          if (v) v = (lds_reclen(W, (uint32_t)(q - c0) + shift) == rl) && (q + rl <= len);
        }
        const unsigned long long okm = __ballot(v);
        const uint32_t k = (~okm) ? (uint32_t)__builtin_ctzll(~okm) : 64u;
        if (lane < k) L.starts[n + lane] = (uint16_t)(q - c0);
        n += k;
        lastp = p + (uint64_t)(k - 1) * rl;
        lastrl = rl;
        p += (uint64_t)k * rl;
      }
    }
    if (lane == 0) {
#ifdef CASK_BAR_CHECK
      L.nb0 = dg.nb;
#endif
      L.n = n;
      {
        uint64_t* sp = a.spec + t;
        ADDR_GUARD(a.stamps, sp, a.spec, a.spec + a.total_chunks, 2, t)
        (void)sp;
      }
      if (!EXACT) a.spec[t] = s;
      a.exit[t] = (s == kNone) ? 0 : exitv;
      a.count[t] = n;
      // a record that does not fit the window is hashed from HBM by k_long
      a.long_r[t] = (exitv != kTerm && n && lastp + lastrl > wend) ? n - 1 : 0xFFFFFFFFu;
    }
  }
  BAR();
  STAMP(1)
  const uint32_t n = L.n;
#ifdef CASK_BAR_CHECK
  if (L.nb0 + 1 != dg.nb && a.stamps && atomicCAS(&a.stamps[8], 0ull, 7ull) == 0ull) {
    a.stamps[9] = L.nb0;
    a.stamps[10] = dg.nb;
    a.stamps[11] = n;
    a.stamps[12] = t;
    a.stamps[13] = blockIdx.x | ((uint64_t)threadIdx.x << 32);
  }
#endif
  DCHECK(n <= a.slot_cap && t < a.total_chunks, "n %u t %llu", n, (unsigned long long)t);

  // 4. verify one record per lane out of LDS and write its slot row.
  uint32_t* slots = a.slots + ((uint64_t)t * a.slot_cap) * 4;
  for (uint32_t r = tid; r < n; r += NT) {
    const uint32_t off = L.starts[r];
    const uint64_t p = c0 + off;
    uint32_t w0 = 0, w1 = 0, w2 = 0, w3 = off << 16;
    bool fail = false;
    if (p + 18 > len) {
      fail = true;  // EOF row: seq/ksz/vsz stay 0
    } else {
      const uint32_t x = off + shift;
      const Hdr h = lds_hdr(W, x);
      w0 = (uint32_t)h.seq;
      w1 = (uint32_t)(h.seq >> 32);
      w2 = h.vsz;
      w3 |= h.ksz;
      const uint64_t rl = 18ull + h.ksz + ((h.vsz == 0xFFFFFFFFu) ? 0ull : (uint64_t)h.vsz);
      if (p + rl > len) {
        fail = true;  // EOF row
      } else if (p + rl <= wend) {
        if (lds_xxh32(W, x + 4, (uint32_t)rl - 4) != h.stored) {
          w3 |= kSlotBad;
          fail = true;
        }
      }  // else: longer than the window, left to k_long (a.long_r[t] == r)
    }
    u32x4 row;
    row.x = w0;
    row.y = w1;
    row.z = w2;
    row.w = w3;
    uint32_t* sl = slots + 4ull * r;
    ADDR_GUARD(a.stamps, sl, a.slots, a.slots + 4ull * a.slot_cap * a.total_chunks, 3, t)
    *(u32x4*)sl = row;
    if (fail) atomicMin(&a.file_err[c.fi], (unsigned long long)((uint64_t)t * a.slot_cap + r));
  }
  STAMP(2)
}

// Persistent grid, kPerCU workgroups per CU. Workgroup b works on XCD (b mod 8) under round-robin
// placement; each XCD gets one contiguous eighth of the chunks and its workgroups stride through
// it, so neighbouring chunks (which share halo bytes) are staged by the same XCD at about the same
// time. Placement only affects speed: any assignment of chunks to workgroups is correct.
// EXACT (the repair re-scan) reads each chunk's known start from spec[]; the speculative kernel
// issues no global load besides the staging loads, so the compiler's counted waits never make the
// processing of one chunk wait for the prefetch of the next.
// `files` is the same table as a.files, passed as a restrict-qualified argument: the kernel never
// writes it, so its (wave-uniform) loads go through the scalar cache.
template <class G, bool EXACT>
__global__ __launch_bounds__(G::kNT) void k_scan_chunks(ScanArgs a, const FileDesc* __restrict__ files_r) {
  __shared__ ScanLdsT<G> L;
#ifdef CASK_VEC_FILES
  const FileDesc* files = a.files;
#else
  const FileDesc* __restrict__ files = files_r;
#endif
  const uint32_t x = blockIdx.x & 7, nx = gridDim.x >> 3;
  const uint64_t per = (a.total_chunks + 7) >> 3;
  uint64_t t = x * per + (blockIdx.x >> 3);
  const uint64_t tend = (x + 1) * per < a.total_chunks ? (x + 1) * per : a.total_chunks;
  if (t >= tend) return;
  if (threadIdx.x == 0) L.found = 0xFFFFFFFFu;
  Diag dg{};
  ChunkPos cur = locate<G>(files, a.nfiles, t);
  u32x4 v[G::kNL];
  stage_issue<G>(v, cur, a.stamps, t);
  for (;;) {
#ifdef CASK_STAMPS
    const uint64_t st_top_ = __builtin_amdgcn_s_memtime();
#endif
    stage_store<G>(L, v, cur);
    BAR();
#ifdef CASK_STAMPS
    dg.st[3] += __builtin_amdgcn_s_memtime() - st_top_;  // phase 3: window wait + LDS store
    dg.st[4] += 1;
#endif
#ifdef CASK_VERIFY_LDS
    if (a.stamps) {  // diagnostic: the staged window must equal HBM
      const volatile gu32x4* src = (const volatile gu32x4*)cur.a0;
      for (uint32_t i = threadIdx.x; i < cur.n16; i += G::kNT) {
        const u32x4 g = src[i];
        const u32x4 l = ((const u32x4*)L.win)[i];
        if ((g.x != l.x || g.y != l.y || g.z != l.z || g.w != l.w) &&
            atomicCAS(&a.stamps[8], 0ull, 9ull) == 0ull) {
          a.stamps[9] = i;
          a.stamps[10] = ((uint64_t)g.x << 32) | l.x;
          a.stamps[11] = cur.n16;
          a.stamps[12] = t;
          a.stamps[13] = blockIdx.x | ((uint64_t)threadIdx.x << 32);
        }
      }
      BAR();
    }
#endif
    // exact (repair) pass: the chunk's known start, loaded before the prefetch is issued so that
    // waiting for it never waits for the prefetch
    const uint64_t s_exact = EXACT ? a.spec[t] : 0;
    const uint64_t tn = t + nx;
    const bool more = tn < tend;
    if (more) stage_issue<G>(v, locate<G>(files, a.nfiles, tn), a.stamps, tn);  // prefetch the next window
    process_chunk<G, EXACT>(L, a, t, cur, s_exact, dg);
    if (threadIdx.x == 0) L.found = 0xFFFFFFFFu;
    BAR();
    if (!more) break;
    t = tn;
    cur = locate<G>(files, a.nfiles, t);
  }
#ifdef CASK_STAMPS
  if (a.stamps && threadIdx.x == 0)
    for (int i = 0; i < 5; ++i) atomicAdd(&a.stamps[i], (unsigned long long)dg.st[i]);
#endif
}

using GeoA = Geo<32768, 4096, 256, 4>;
using GeoB = Geo<16384, 1536, 128, 8>;
using GeoC = Geo<8192, 1024, 64, 16>;

static inline hipStream_t S(void* s) { return (hipStream_t)s; }

uint32_t geometry_chunk(int geo) { return geo == 1 ? GeoB::kCh : geo == 2 ? GeoC::kCh : GeoA::kCh; }

template <class G>
static void launch_geo(const ScanArgs& a, void* stream) {
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  uint64_t grid = (uint64_t)cus * G::kPerCU;
  grid = (grid + 7) & ~7ull;
  const uint64_t need = (a.total_chunks + 7) & ~7ull;  // never more workgroups than chunks
  if (need < grid) grid = need;
  // CASK_LDS_PAD (diagnostic): extra dynamic LDS per workgroup, to lower workgroups per CU
  static const uint32_t pad = getenv("CASK_LDS_PAD") ? (uint32_t)atoi(getenv("CASK_LDS_PAD")) : 0u;
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
  else
    launch_geo<GeoA>(a, stream);
}

}  // namespace cask_dev
