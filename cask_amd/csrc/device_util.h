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
  uint64_t st[10];  // -DCASK_STAMPS: s_memtime cycles per phase, summed over the workgroup's chunks
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

// The window is staged 16-B aligned; records start at arbitrary byte offsets. gfx950 serves
// unaligned LDS reads (unaligned-ds-access): a memcpy from a byte address compiles to one
// ds_read_b32/b64/b128 at that address, so no funnel shifts are needed to assemble words.
__device__ __forceinline__ uint32_t lds_u32(const uint32_t* w, uint32_t x) {
  uint32_t v;
  __builtin_memcpy(&v, (const uint8_t*)w + x, 4);
  return v;
}
__device__ __forceinline__ uint64_t lds_u64(const uint32_t* w, uint32_t x) {
  uint64_t v;
  __builtin_memcpy(&v, (const uint8_t*)w + x, 8);
  return v;
}
__device__ __forceinline__ u32x4 lds_u128(const uint32_t* w, uint32_t x) {
  u32x4 v;
  __builtin_memcpy(&v, (const uint8_t*)w + x, 16);
  return v;
}

// Record length at LDS byte index x: 18 + ksz + vsz_eff (data.rs:63-65; tombstone vsz = !0).
__device__ __forceinline__ uint64_t lds_reclen(const uint32_t* w, uint32_t x) {
  const uint64_t b = lds_u64(w, x + 12);  // ksz u16 | vsz u32 | 2 bytes of what follows
  const uint32_t ksz = (uint32_t)b & 0xFFFFu;
  const uint32_t vsz = (uint32_t)(b >> 16);
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
  const u32x4 d = lds_u128(w, x);          // bytes x .. x+15
  const uint32_t e = lds_u32(w, x + 14);   // bytes x+14 .. x+17: vsz
  Hdr h;
  h.stored = d.x;
  h.seq = (uint64_t)d.y | ((uint64_t)d.z << 32);
  h.ksz = d.w & 0xFFFFu;
  h.vsz = e;
  return h;
}

// XXH32 (seed 0) of LDS bytes [xs, xs + len), 16-B stripes read with unaligned ds_read_b128.
// Two stripes are mixed per step while the next two are in flight: under load an LDS read takes
// longer than one stripe's multiplies.
template <bool FAKE = false>  // FAKE (diagnostic): stripes from registers, not LDS; wrong hash
__device__ __forceinline__ uint32_t lds_xxh32(const uint32_t* w, uint32_t xs, uint32_t len) {
  uint32_t h;
  const uint32_t nstr = len >> 4;
  uint32_t x = xs;
  if (nstr) {
    Acc a = acc_init(0);
    auto ld = [&](uint32_t y) -> u32x4 {
      if (!FAKE) return lds_u128(w, y);
      u32x4 v;
      v.x = y;
      v.y = y ^ 0x5bd1e995u;
      v.z = y * 3u;
      v.w = y + 0x27d4eb2fu;
      return v;
    };
    u32x4 d0 = ld(x), d1 = ld(x + 16);  // reads past the record stay in LDS
    uint32_t s = 0;
    for (; s + 2 <= nstr; s += 2) {
      const u32x4 e0 = ld(x + 32), e1 = ld(x + 48);  // next pair in flight
      __builtin_amdgcn_sched_barrier(0);  // keep them issued ahead of this pair's multiplies
      acc_stripe(a, d0.x, d0.y, d0.z, d0.w);
      acc_stripe(a, d1.x, d1.y, d1.z, d1.w);
      d0 = e0;
      d1 = e1;
      x += 32;
    }
    if (s < nstr) {
      acc_stripe(a, d0.x, d0.y, d0.z, d0.w);
      x += 16;
    }
    h = acc_merge(a);
  } else {
    h = P5;
  }
  h += len;
  uint32_t rem = len & 15;
  while (rem >= 4) {
    h = tail4(h, lds_u32(w, x));
    x += 4;
    rem -= 4;
  }
  const uint8_t* b = (const uint8_t*)w;
  while (rem) {
    h = tail1(h, b[x]);
    ++x;
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
