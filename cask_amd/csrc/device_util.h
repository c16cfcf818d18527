// Device helpers shared by the scan kernels (gfx950): LDS byte-stream reads, XXH32 over LDS and
// over HBM, record-length decoding, file lookup, diagnostic stamps.
#pragma once
#include <hip/hip_runtime.h>

#include "scan_kernels.h"
#include "xxh32.h"

namespace cask_dev {

using namespace cask_xxh;

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// Per-thread diagnostic state of k_scan_chunks (unused, and compiled away, in the shipped library).
struct Diag {
  uint32_t nb;      // -DCASK_BAR_CHECK: barriers passed
  uint64_t st[5];   // -DCASK_STAMPS: s_memtime cycles per phase, summed over the workgroup's chunks
};

// Diagnostic build (-DCASK_STAMPS): every thread sums the s_memtime cycles of each phase of
// k_scan_chunks in registers; thread 0 adds its sums into a.stamps[] once, at the end.
#ifdef CASK_STAMPS
#define STAMP_INIT uint64_t st_prev_ = __builtin_amdgcn_s_memtime();
#define STAMP(i)                                             \
  {                                                          \
    const uint64_t st_now_ = __builtin_amdgcn_s_memtime();   \
    dg.st[i] += st_now_ - st_prev_;                          \
    st_prev_ = st_now_;                                      \
  }
#else
#define STAMP_INIT
#define STAMP(i)
#endif

// Diagnostic build (-DCASK_CHECKS): bounds checks that print the offending values and trap.
#ifdef CASK_CHECKS
#define DCHECK(cond, fmt, ...)                                                         \
  if (!(cond)) {                                                                       \
    printf("CHECK %s:%d " #cond " " fmt "\n", __FILE__, __LINE__, ##__VA_ARGS__);      \
    __builtin_trap();                                                                  \
  }
#else
#define DCHECK(cond, fmt, ...)
#endif

// The window is staged 16-B aligned; records start at arbitrary byte offsets, so every unaligned
// 32-bit word is assembled from two aligned dword reads with v_alignbyte_b32 (a funnel shift).
__device__ __forceinline__ uint32_t funnel(uint32_t hi, uint32_t lo, uint32_t sh) {
  return __builtin_amdgcn_alignbyte(hi, lo, sh);
}

// Record length at LDS byte index x: 18 + ksz + vsz_eff (data.rs:63-65; tombstone vsz = !0).
__device__ __forceinline__ uint64_t lds_reclen(const uint32_t* w, uint32_t x) {
  const uint32_t q = (x + 12) >> 2, sh = (x + 12) & 3;
  const uint32_t d0 = w[q], d1 = w[q + 1], d2 = w[q + 2];
  const uint32_t b3 = funnel(d1, d0, sh);  // bytes x+12..x+15: ksz | vsz.lo16
  const uint32_t b4 = funnel(d2, d1, sh);  // bytes x+16..x+19: vsz.hi16 | ...
  const uint32_t ksz = b3 & 0xFFFFu;
  const uint32_t vsz = (b3 >> 16) | (b4 << 16);
  return 18ull + ksz + ((vsz == 0xFFFFFFFFu) ? 0ull : (uint64_t)vsz);
}

// The 18-byte header `xxh32 u32 | seq u64 | ksz u16 | vsz u32`, little-endian (data.rs:161-169).
struct Hdr {
  uint32_t stored;
  uint64_t seq;
  uint32_t ksz;
  uint32_t vsz;
};

__device__ __forceinline__ Hdr lds_hdr(const uint32_t* w, uint32_t x) {
  const uint32_t q = x >> 2, sh = x & 3;
  const uint32_t d0 = w[q], d1 = w[q + 1], d2 = w[q + 2], d3 = w[q + 3], d4 = w[q + 4], d5 = w[q + 5];
  Hdr h;
  h.stored = funnel(d1, d0, sh);
  const uint32_t s0 = funnel(d2, d1, sh), s1 = funnel(d3, d2, sh);
  h.seq = (uint64_t)s0 | ((uint64_t)s1 << 32);
  const uint32_t b3 = funnel(d4, d3, sh), b4 = funnel(d5, d4, sh);
  h.ksz = b3 & 0xFFFFu;
  h.vsz = (b3 >> 16) | (b4 << 16);
  return h;
}

// XXH32 (seed 0) of LDS bytes [xs, xs + len): aligned dword reads + funnel, 16-B stripes.
__device__ __forceinline__ uint32_t lds_xxh32(const uint32_t* w, uint32_t xs, uint32_t len) {
  const uint32_t sh = xs & 3;
  uint32_t wi = xs >> 2;
  uint32_t prev = w[wi];
  uint32_t h;
  const uint32_t nstr = len >> 4;
  if (nstr) {
    Acc a = acc_init(0);
    for (uint32_t s = 0; s < nstr; ++s) {
      const uint32_t d1 = w[wi + 1], d2 = w[wi + 2], d3 = w[wi + 3], d4 = w[wi + 4];
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
    const uint32_t d1 = w[wi + 1];
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

// Unaligned global loads: gfx950 runs in unaligned-access mode, so these memcpys become
// global_load_dwordx4 / global_load_dword at any byte address.
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

// XXH32 of global bytes [p, p+len) by one lane (long records, repair, error detail).
__device__ __forceinline__ uint32_t gbl_xxh32(const uint8_t* p, uint64_t len) {
  const uint8_t* end = p + len;
  uint32_t h;
  if (len >= 16) {
    Acc a = acc_init(0);
    const uint64_t nstr = len >> 4;
    for (uint64_t s = 0; s < nstr; ++s) {
      const u32x4 v = gld16(p);
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
  const uint32_t b3 = gld4(hdr + 12);
  const uint32_t b4 = (uint32_t)hdr[16] | ((uint32_t)hdr[17] << 8);
  const uint32_t ksz = b3 & 0xFFFFu;
  const uint32_t vsz = (b3 >> 16) | (b4 << 16);
  return 18ull + ksz + ((vsz == 0xFFFFFFFFu) ? 0ull : (uint64_t)vsz);
}

// Last file with first_chunk <= t (empty files share first_chunk with their successor). Call it
// with wave-uniform t from every lane: the loads then go through the scalar cache.
__device__ __forceinline__ uint32_t find_file(const FileDesc* files, uint32_t nfiles, uint64_t t) {
  uint32_t lo = 0, hi = nfiles;  // answer in [lo, hi)
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (files[mid].first_chunk <= t) lo = mid; else hi = mid;
  }
  return lo;
}

}  // namespace cask_dev
