// XXH32 (seed 0) building blocks shared by the device kernels and the host runtime.
//
// Cask checksums every record with XXH32, seed 0, via the `twox-hash` crate
// (reference: src/util.rs:8,14,37-41; Cargo.toml:18 `twox-hash = "1.1.0"`).
// The arithmetic below is the published XXH32 algorithm: 4 lane accumulators over
// 16-byte stripes, length fold-in, 4-byte then 1-byte tail, avalanche.
//
// Everything is wrapping u32 arithmetic; the rotate maps to v_alignbit_b32 on gfx950
// and the prime multiplies to v_mul_lo_u32.
#pragma once
#include <stdint.h>

#if defined(__HIP__)
#include <hip/hip_runtime.h>
#define XXH_FN __host__ __device__ __forceinline__
#else
#define XXH_FN static inline
#endif

namespace cask_xxh {

constexpr uint32_t P1 = 2654435761u;
constexpr uint32_t P2 = 2246822519u;
constexpr uint32_t P3 = 3266489917u;
constexpr uint32_t P4 = 668265263u;
constexpr uint32_t P5 = 374761393u;

XXH_FN uint32_t rotl(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }

XXH_FN uint32_t xround(uint32_t acc, uint32_t w) {
  acc += w * P2;
  acc = rotl(acc, 13);
  return acc * P1;
}

// Accumulator state for the >=16-byte branch.
struct Acc {
  uint32_t v1, v2, v3, v4;
};

XXH_FN Acc acc_init(uint32_t seed) {
  Acc a;
  a.v1 = seed + P1 + P2;
  a.v2 = seed + P2;
  a.v3 = seed;
  a.v4 = seed - P1;
  return a;
}

XXH_FN void acc_stripe(Acc& a, uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3) {
  a.v1 = xround(a.v1, w0);
  a.v2 = xround(a.v2, w1);
  a.v3 = xround(a.v3, w2);
  a.v4 = xround(a.v4, w3);
}

XXH_FN uint32_t acc_merge(const Acc& a) {
  return rotl(a.v1, 1) + rotl(a.v2, 7) + rotl(a.v3, 12) + rotl(a.v4, 18);
}

XXH_FN uint32_t tail4(uint32_t h, uint32_t w) { return rotl(h + w * P3, 17) * P4; }
XXH_FN uint32_t tail1(uint32_t h, uint32_t b) { return rotl(h + b * P5, 11) * P1; }

XXH_FN uint32_t avalanche(uint32_t h) {
  h ^= h >> 15;
  h *= P2;
  h ^= h >> 13;
  h *= P3;
  h ^= h >> 16;
  return h;
}

XXH_FN uint32_t load_le32(const uint8_t* p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

// One-shot XXH32 over a contiguous byte range (host + device; byte loads, used by
// the slow/long-record paths and by the host runtime).
XXH_FN uint32_t xxh32(const uint8_t* p, uint64_t len, uint32_t seed) {
  const uint8_t* end = p + len;
  uint32_t h;
  if (len >= 16) {
    Acc a = acc_init(seed);
    const uint8_t* limit = end - 16;
    do {
      acc_stripe(a, load_le32(p), load_le32(p + 4), load_le32(p + 8), load_le32(p + 12));
      p += 16;
    } while (p <= limit);
    h = acc_merge(a);
  } else {
    h = seed + P5;
  }
  h += (uint32_t)len;  // XXH32 folds the length in mod 2^32
  while (p + 4 <= end) {
    h = tail4(h, load_le32(p));
    p += 4;
  }
  while (p < end) {
    h = tail1(h, *p);
    ++p;
  }
  return avalanche(h);
}

}  // namespace cask_xxh
