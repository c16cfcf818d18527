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

// The window is staged 16-B aligned; records start at arbitrary byte offsets. On gfx950 an LDS
// read whose address is not a multiple of its width is served one lane per clock (measured in
// tools/ubench_lds.hip: ~27 ns per wave-instruction per CU against 2 ns aligned, for b32, b64 and
// b128 alike), so every read here is of naturally aligned dwords and the bytes at an arbitrary
// offset are funnelled out of two neighbours with v_alignbyte_b32.
__device__ __forceinline__ uint32_t fun(uint32_t lo, uint32_t hi, uint32_t sh) {
  return __builtin_amdgcn_alignbyte(hi, lo, sh);  // bytes sh..sh+3 of hi:lo (sh in 0..3)
}
__device__ __forceinline__ uint32_t lds_u32(const uint32_t* w, uint32_t x) {
  const uint32_t i = x >> 2;
  return fun(w[i], w[i + 1], x & 3);  // ds_read2_b32: two aligned dwords
}

// The 18-byte header `xxh32 u32 | seq u64 | ksz u16 | vsz u32`, little-endian (data.rs:161-169),
// from the 6 aligned dwords that cover bytes x .. x+17.
struct Hdr {
  uint32_t stored;
  uint64_t seq;
  uint32_t ksz;
  uint32_t vsz;
};

__device__ __forceinline__ Hdr lds_hdr(const uint32_t* w, uint32_t x) {
  const uint32_t i = x >> 2, sh = x & 3;
  const uint32_t d0 = w[i], d1 = w[i + 1], d2 = w[i + 2], d3 = w[i + 3], d4 = w[i + 4], d5 = w[i + 5];
  const uint32_t w3 = fun(d3, d4, sh), w4 = fun(d4, d5, sh);
  Hdr h;
  h.stored = fun(d0, d1, sh);
  h.seq = (uint64_t)fun(d1, d2, sh) | ((uint64_t)fun(d2, d3, sh) << 32);
  h.ksz = w3 & 0xFFFFu;
  h.vsz = (w3 >> 16) | (w4 << 16);
  return h;
}

// Record length at LDS byte index x: 18 + ksz + vsz_eff (data.rs:63-65; tombstone vsz = !0),
// from bytes x+12 .. x+17.
__device__ __forceinline__ uint64_t lds_reclen(const uint32_t* w, uint32_t x) {
  const uint32_t i = (x + 12) >> 2, sh = x & 3;
  const uint32_t d0 = w[i], d1 = w[i + 1], d2 = w[i + 2];
  const uint32_t w3 = fun(d0, d1, sh), w4 = fun(d1, d2, sh);
  const uint32_t ksz = w3 & 0xFFFFu;
  const uint32_t vsz = (w3 >> 16) | (w4 << 16);
  return 18ull + ksz + ((vsz == 0xFFFFFFFFu) ? 0ull : (uint64_t)vsz);
}

// XXH32 tail of `rem` (< 16) bytes at LDS byte x onto h, and the avalanche. The at most five
// aligned dwords covering the bytes are read at once; the serial steps then run on registers.
__device__ __forceinline__ uint32_t lds_tail_fin(const uint32_t* w, uint32_t x, uint32_t rem, uint32_t h) {
  const uint32_t i = x >> 2, sh = x & 3;
  const uint32_t e0 = w[i], e1 = w[i + 1], e2 = w[i + 2], e3 = w[i + 3], e4 = w[i + 4];
  const uint32_t t0 = fun(e0, e1, sh), t1 = fun(e1, e2, sh), t2 = fun(e2, e3, sh), t3 = fun(e3, e4, sh);
  const uint32_t nw = rem >> 2;
  if (nw > 0) h = tail4(h, t0);
  if (nw > 1) h = tail4(h, t1);
  if (nw > 2) h = tail4(h, t2);
  const uint32_t lw = nw == 0 ? t0 : nw == 1 ? t1 : nw == 2 ? t2 : t3;
  const uint32_t nb = rem & 3;
  if (nb > 0) h = tail1(h, lw & 0xFFu);
  if (nb > 1) h = tail1(h, (lw >> 8) & 0xFFu);
  if (nb > 2) h = tail1(h, (lw >> 16) & 0xFFu);
  return avalanche(h);
}

// XXH32 (seed 0) of LDS bytes [xs, xs + len) by one lane (the boundary search's candidates).
__device__ __forceinline__ uint32_t lds_xxh32(const uint32_t* w, uint32_t xs, uint32_t len) {
  uint32_t h;
  const uint32_t nstr = len >> 4, sh = xs & 3;
  uint32_t i = xs >> 2;
  if (nstr) {
    Acc a = acc_init(0);
    uint32_t d0 = w[i];
    for (uint32_t s = 0; s < nstr; ++s) {
      const uint32_t d1 = w[i + 1], d2 = w[i + 2], d3 = w[i + 3], d4 = w[i + 4];
      acc_stripe(a, fun(d0, d1, sh), fun(d1, d2, sh), fun(d2, d3, sh), fun(d3, d4, sh));
      d0 = d4;
      i += 4;
    }
    h = acc_merge(a);
  } else {
    h = P5;
  }
  return lds_tail_fin(w, xs + (nstr << 4), len & 15, h + len);
}

// XXH32 (seed 0) of LDS bytes [xs, xs + len) by one lane with its four stripe accumulators
// interleaved (the stride pass: one record per lane). Two stripes' aligned dwords are read per step.
__device__ __forceinline__ uint32_t lane_xxh32(const uint32_t* w, uint32_t xs, uint32_t len) {
  uint32_t h;
  const uint32_t nstr = len >> 4, sh = xs & 3;
  uint32_t i = xs >> 2;
  if (nstr) {
    Acc a = acc_init(0);
    uint32_t d0 = w[i];
    uint32_t s = 0;
    for (; s + 2 <= nstr; s += 2) {
      const uint32_t d1 = w[i + 1], d2 = w[i + 2], d3 = w[i + 3], d4 = w[i + 4];
      const uint32_t e1 = w[i + 5], e2 = w[i + 6], e3 = w[i + 7], e4 = w[i + 8];
      acc_stripe(a, fun(d0, d1, sh), fun(d1, d2, sh), fun(d2, d3, sh), fun(d3, d4, sh));
      acc_stripe(a, fun(d4, e1, sh), fun(e1, e2, sh), fun(e2, e3, sh), fun(e3, e4, sh));
      d0 = e4;
      i += 8;
    }
    if (s < nstr) {
      const uint32_t d1 = w[i + 1], d2 = w[i + 2], d3 = w[i + 3], d4 = w[i + 4];
      acc_stripe(a, fun(d0, d1, sh), fun(d1, d2, sh), fun(d2, d3, sh), fun(d3, d4, sh));
    }
    h = acc_merge(a);
  } else {
    h = P5;
  }
  return lds_tail_fin(w, xs + (nstr << 4), len & 15, h + len);
}

// Quad-lane DPP moves (quad_perm): lane a of each group of 4 receives lane perm[a]'s value.
__device__ __forceinline__ uint32_t quad_xor1(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);  // [1,0,3,2]
}
__device__ __forceinline__ uint32_t quad_xor2(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, false);  // [2,3,0,1]
}
__device__ __forceinline__ uint32_t rotl_var(uint32_t x, uint32_t r) {
  return __builtin_amdgcn_alignbit(x, x, 32u - r);  // r in [1, 31]
}

// XXH32 (seed 0) of LDS bytes [xs, xs + len) computed by a quad of lanes, lane a = 0..3 of the
// quad keeping stripe accumulator v_{a+1} (XXH32's four accumulators are independent until the
// merge). Every lane of the quad returns the hash. The four lanes must be active together and
// call with the same xs/len. Lane a reads the two aligned dwords around its word of each stripe,
// four stripes ahead.
__device__ __forceinline__ uint32_t quad_xxh32(const uint32_t* w, uint32_t xs, uint32_t len, uint32_t a) {
  uint32_t h;
  const uint32_t nstr = len >> 4;
  if (nstr) {
    uint32_t v = a == 0 ? P1 + P2 : a == 1 ? P2 : a == 2 ? 0u : 0u - P1;
    const uint32_t sh = xs & 3;
    uint32_t i = (xs >> 2) + a;  // lane a: dwords i, i+1 of every stripe (aligned ds_read2_b32)
    uint32_t s = 0;
    if (nstr >= 8) {  // double-buffered: the next block's 8 reads are in flight while this one mixes
      uint32_t A[8];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        A[2 * k] = w[i + 4 * k];
        A[2 * k + 1] = w[i + 4 * k + 1];
      }
      for (; s + 8 <= nstr; s += 4) {
        uint32_t An[8];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          An[2 * k] = w[i + 16 + 4 * k];
          An[2 * k + 1] = w[i + 16 + 4 * k + 1];
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) v = xround(v, fun(A[2 * k], A[2 * k + 1], sh));
#pragma unroll
        for (int k = 0; k < 8; ++k) A[k] = An[k];
        i += 16;
      }
    }
    for (; s + 4 <= nstr; s += 4) {  // 8 reads in flight, then 4 rounds
      const uint32_t a0 = w[i], b0 = w[i + 1], a1 = w[i + 4], b1 = w[i + 5];
      const uint32_t a2 = w[i + 8], b2 = w[i + 9], a3 = w[i + 12], b3 = w[i + 13];
      v = xround(v, fun(a0, b0, sh));
      v = xround(v, fun(a1, b1, sh));
      v = xround(v, fun(a2, b2, sh));
      v = xround(v, fun(a3, b3, sh));
      i += 16;
    }
    for (; s < nstr; ++s) {
      v = xround(v, fun(w[i], w[i + 1], sh));
      i += 4;
    }
    uint32_t m = rotl_var(v, a == 0 ? 1u : a == 1 ? 7u : a == 2 ? 12u : 18u);
    m += quad_xor1(m);
    m += quad_xor2(m);
    h = m;
  } else {
    h = P5;
  }
  return lds_tail_fin(w, xs + (nstr << 4), len & 15, h + len);
}

// A value every lane holds equally (read from the same LDS word), moved to scalar registers so
// that the loops and branches it controls compile to scalar control flow.
__device__ __forceinline__ uint64_t uni64(uint64_t v) {
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v), hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  return ((uint64_t)hi << 32) | lo;
}

// Unaligned global loads: gfx950 runs in unaligned-access mode, so these memcpys become
// global_load_dwordx4 / global_load_dword at any byte address. Through a global-address-space
// pointer: from a generic one they compile to flat loads, and every wait on a flat load is a
// wait for all of them (vmcnt(0) lgkmcnt(0)) — a loop that issued the next block's loads before
// mixing this one's then waited for both, and the double buffering bought nothing.
typedef __attribute__((address_space(1))) const uint8_t g_u8;
__device__ __forceinline__ u32x4 gld16(const uint8_t* p) {
  u32x4 v;
  __builtin_memcpy(&v, (g_u8*)p, 16);
  return v;
}
__device__ __forceinline__ uint32_t gld4(const uint8_t* p) {
  uint32_t v;
  __builtin_memcpy(&v, (g_u8*)p, 4);
  return v;
}
__device__ __forceinline__ u32x4 gld16g(const g_u8* p) {
  u32x4 v;
  __builtin_memcpy(&v, p, 16);
  return v;
}
__device__ __forceinline__ uint32_t gld4g(const g_u8* p) {
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
    uint64_t s = 0;
    if (nstr >= 8) {  // double-buffered: the next 128 B are in flight while these 128 B mix
      u32x4 A[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) A[k] = gld16(p + 16 * k);
      for (; s + 16 <= nstr; s += 8) {
        u32x4 B[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) B[k] = gld16(p + 128 + 16 * k);
#pragma unroll
        for (int k = 0; k < 8; ++k) acc_stripe(a, A[k].x, A[k].y, A[k].z, A[k].w);
#pragma unroll
        for (int k = 0; k < 8; ++k) A[k] = B[k];
        p += 128;
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) acc_stripe(a, A[k].x, A[k].y, A[k].z, A[k].w);
      p += 128;
      s += 8;
    }
    for (; s < nstr; ++s) {
      const u32x4 v = gld16(p);
      acc_stripe(a, v.x, v.y, v.z, v.w);
      p += 16;
    }
    h = acc_merge(a);
  } else {
    h = P5;
  }
  h += (uint32_t)len;
  // the last < 16 bytes: loaded at once (no load waits on another), then folded in order
  const uint32_t nt = (uint32_t)(end - p);
  uint32_t t4[3] = {0u, 0u, 0u};
  uint8_t t1[3] = {0, 0, 0};
  const uint32_t n4 = nt >> 2, n1 = nt & 3;
#pragma unroll
  for (uint32_t k = 0; k < 3; ++k)
    if (k < n4) t4[k] = gld4(p + 4 * k);
#pragma unroll
  for (uint32_t k = 0; k < 3; ++k)
    if (k < n1) t1[k] = p[4 * n4 + k];
#pragma unroll
  for (uint32_t k = 0; k < 3; ++k)
    if (k < n4) h = tail4(h, t4[k]);
#pragma unroll
  for (uint32_t k = 0; k < 3; ++k)
    if (k < n1) h = tail1(h, t1[k]);
  return avalanche(h);
}

// 4x4 transpose across a quad: lane q enters with stripe q of a 4-stripe block (words 0..3) and
// leaves with word q of stripes 0..3, in order (two butterfly stages of quad DPP moves).
__device__ __forceinline__ void quad_transpose(u32x4& v, uint32_t q) {
  const bool b1 = q & 2, b0 = q & 1;
  uint32_t r0 = quad_xor2(b1 ? v.x : v.z), r1 = quad_xor2(b1 ? v.y : v.w);  // swap off-diagonal 2x2 blocks
  if (b1) { v.x = r0; v.y = r1; } else { v.z = r0; v.w = r1; }
  r0 = quad_xor1(b0 ? v.x : v.y);  // transpose within the 2x2 blocks
  r1 = quad_xor1(b0 ? v.z : v.w);
  if (b0) { v.x = r0; v.z = r1; } else { v.y = r0; v.w = r1; }
}
// The same transpose, each stage as four v_cndmask_b32_dpp (word = the lane's bit set ? its own word :
// the partner's, the DPP operand): 8 vector instructions instead of 16 (k_run_hash). The two
// s_mov to vcc before each stage are the two wait states a DPP read of a VGPR the previous vector
// instruction wrote needs (no s_nop).
__device__ __forceinline__ void quad_transpose_dpp(u32x4& v) {
  uint32_t x1, y1, z1, w1, x2, y2, z2, w2;
  // stage 1, partner q ^ 2 (vcc: lanes with q & 2): off-diagonal 2x2 blocks swapped
  asm volatile(
      "s_mov_b32 vcc_lo, 0xcccccccc\n"
      "s_mov_b32 vcc_hi, 0xcccccccc\n"
      "v_cndmask_b32_dpp %2, %4, %6, vcc quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n"
      "v_cndmask_b32_dpp %3, %5, %7, vcc quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n"
      "s_not_b64 vcc, vcc\n"
      "v_cndmask_b32_dpp %0, %6, %4, vcc quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n"
      "v_cndmask_b32_dpp %1, %7, %5, vcc quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n"
      : "=&v"(x1), "=&v"(y1), "=&v"(z1), "=&v"(w1)
      : "v"(v.x), "v"(v.y), "v"(v.z), "v"(v.w)
      : "vcc");
  // stage 2, partner q ^ 1 (vcc: lanes with q & 1): the 2x2 blocks transposed
  asm volatile(
      "s_mov_b32 vcc_lo, 0xaaaaaaaa\n"
      "s_mov_b32 vcc_hi, 0xaaaaaaaa\n"
      "v_cndmask_b32_dpp %1, %4, %5, vcc quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"
      "v_cndmask_b32_dpp %3, %6, %7, vcc quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"
      "s_not_b64 vcc, vcc\n"
      "v_cndmask_b32_dpp %0, %5, %4, vcc quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"
      "v_cndmask_b32_dpp %2, %7, %6, vcc quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"
      : "=&v"(x2), "=&v"(y2), "=&v"(z2), "=&v"(w2)
      : "v"(x1), "v"(y1), "v"(z1), "v"(w1)
      : "vcc");
  v = u32x4{x2, y2, z2, w2};
}

// XXH32 (seed 0) of global bytes [p, p+len) by a quad of lanes (q = lane & 3), lane q keeping stripe
// accumulator v_{q+1}. Lane q loads stripe q of each 64-B block (one 16-B load: the quad reads 64
// contiguous bytes per instruction), quad_transpose hands every lane its word of the block's four
// stripes. The four lanes must be active together and call with the same p/len; all four return
// the hash. Rounds of D blocks: the next round's loads are in flight while this one mixes, two
// register sets in turn (no copies), and the loads of a round share one address register
// (immediate offsets), the last partial round loaded under a predicate rather than at clamped
// addresses. k_long_hash is VALU-bound as much as HBM-bound (XXH32's two quarter-rate multiplies
// per word; 64 % VALU-busy before these address and copy savings), and a dword per lane per stripe
// instead of the transpose ran it at half speed (4x the load instructions).
// D: blocks per round (64 B each).
template <uint32_t D = 8>
__device__ __forceinline__ uint32_t quad_gbl_xxh32(const uint8_t* p, uint64_t len, uint32_t q) {
  const uint64_t nstr = len >> 4;
  uint32_t h;
  if (nstr) {
    uint32_t v = q == 0 ? P1 + P2 : q == 1 ? P2 : q == 2 ? 0u : 0u - P1;
    const uint64_t nblk = nstr >> 2;
    const g_u8* lp = (const g_u8*)p + 16 * q;  // stripe q of block b: lp + 64 b
    auto mix = [&](u32x4 X) {
      quad_transpose(X, q);
      v = xround(v, X.x);
      v = xround(v, X.y);
      v = xround(v, X.z);
      v = xround(v, X.w);
    };
    uint64_t k = 0;  // blocks mixed
    if (nblk >= D) {
      u32x4 A[D], B[D];
#pragma unroll
      for (uint32_t d = 0; d < D; ++d) A[d] = gld16g(lp + 64 * d);
      for (;;) {  // A holds blocks [k, k + D)
        if (k + 2 * D > nblk) {
#pragma unroll
          for (uint32_t d = 0; d < D; ++d) mix(A[d]);
          k += D;
          break;
        }
        const g_u8* bp = lp + 64 * (k + D);
#pragma unroll
        for (uint32_t d = 0; d < D; ++d) B[d] = gld16g(bp + 64 * d);
#pragma unroll
        for (uint32_t d = 0; d < D; ++d) mix(A[d]);
        k += D;  // B holds blocks [k, k + D)
        if (k + 2 * D > nblk) {
#pragma unroll
          for (uint32_t d = 0; d < D; ++d) mix(B[d]);
          k += D;
          break;
        }
        const g_u8* ap = lp + 64 * (k + D);
#pragma unroll
        for (uint32_t d = 0; d < D; ++d) A[d] = gld16g(ap + 64 * d);
#pragma unroll
        for (uint32_t d = 0; d < D; ++d) mix(B[d]);
        k += D;
      }
    }
    {  // the last nblk - k < D blocks, loaded together
      const uint32_t tb = (uint32_t)(nblk - k);
      const g_u8* tp = lp + 64 * k;
      u32x4 T[D];
#pragma unroll
      for (uint32_t d = 0; d < D; ++d)
        if (d < tb) T[d] = gld16g(tp + 64 * d);
#pragma unroll
      for (uint32_t d = 0; d < D; ++d)
        if (d < tb) mix(T[d]);
    }
    const uint32_t rem = (uint32_t)(nstr & 3);
    if (rem) {  // the last 1-3 stripes: lanes q < rem load one each
      u32x4 R = gld16(p + 64 * nblk + 16 * (q < rem ? q : 0));
      quad_transpose(R, q);
      v = xround(v, R.x);
      if (rem > 1) v = xround(v, R.y);
      if (rem > 2) v = xround(v, R.z);
    }
    uint32_t m = rotl_var(v, q == 0 ? 1u : q == 1 ? 7u : q == 2 ? 12u : 18u);
    m += quad_xor1(m);
    m += quad_xor2(m);
    h = m;
  } else {
    h = P5;
  }
  h += (uint32_t)len;
  const uint8_t* t = p + 16 * nstr;
  const uint32_t nt = (uint32_t)(len & 15), n4 = nt >> 2, n1 = nt & 3;
  uint32_t t4[3] = {0u, 0u, 0u};
  uint8_t t1[3] = {0, 0, 0};
#pragma unroll
  for (uint32_t k = 0; k < 3; ++k)
    if (k < n4) t4[k] = gld4(t + 4 * k);
#pragma unroll
  for (uint32_t k = 0; k < 3; ++k)
    if (k < n1) t1[k] = t[4 * n4 + k];
#pragma unroll
  for (uint32_t k = 0; k < 3; ++k)
    if (k < n4) h = tail4(h, t4[k]);
#pragma unroll
  for (uint32_t k = 0; k < 3; ++k)
    if (k < n1) h = tail1(h, t1[k]);
  return avalanche(h);
}

__device__ __forceinline__ uint64_t g_reclen(const uint8_t* hdr) {
  const uint32_t b3 = gld4(hdr + 12);
  const uint32_t b4 = (uint32_t)hdr[16] | ((uint32_t)hdr[17] << 8);
  const uint32_t ksz = b3 & 0xFFFFu;
  const uint32_t vsz = (b3 >> 16) | (b4 << 16);
  return 18ull + ksz + ((vsz == 0xFFFFFFFFu) ? 0ull : (uint64_t)vsz);
}

// ------------------------------------------------------------------------------------------
// Single-pass prefix over elements handed out in order (k_finish's tiles): the dense row numbering
// and the chunk-start validation are a prefix over every earlier chunk of (row count, max chain
// exit within the file).
// ------------------------------------------------------------------------------------------
struct SegAgg {  // prefix aggregate: rows, and the max exit within the last file seen
  uint64_t rows, mx;
  uint32_t fl;     // file of the last chunk (0xFFFFFFFF: empty)
  uint32_t hs;     // the aggregate contains file fl's first chunk (T restarts there)
};

// a, then b. An aggregate of no chunks (fl = 0xFFFFFFFF: a tile's lanes past the last chunk, the
// prefix of tile 0) is the identity on either side.
__device__ __forceinline__ SegAgg seg_combine(const SegAgg& a, const SegAgg& b) {
  SegAgg r;
  if (b.fl == 0xFFFFFFFFu) {
    r = a;
    r.rows += b.rows;
    return r;
  }
  if (a.fl == 0xFFFFFFFFu) {
    r = b;
    r.rows += a.rows;
    return r;
  }
  r.rows = a.rows + b.rows;
  r.fl = b.fl;
  if (b.hs || a.fl != b.fl) {
    r.mx = b.mx;
    r.hs = b.hs;
  } else {
    r.mx = a.mx > b.mx ? a.mx : b.mx;
    r.hs = a.hs;
  }
  return r;
}

// Look-back granules: 8-B words written once per call by one relaxed agent-scope atomic store and
// polled the same way (untorn, no ordering needed), each tagged with the call's epoch in its top
// byte so that no memset is needed between calls. Per tile: aggregate (rows, mx, fl|hs) at 0..2,
// inclusive prefix at 3..5.
constexpr uint64_t kPay = (1ull << 56) - 1;
__device__ __forceinline__ void gran_put(uint64_t* p, uint32_t epoch, uint64_t v) {
  __hip_atomic_store(p, ((uint64_t)epoch << 56) | (v & kPay), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ bool gran_get(const uint64_t* p, uint32_t epoch, uint64_t& v) {
  const uint64_t g = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  v = g & kPay;
  return (uint32_t)(g >> 56) == epoch;
}
__device__ __forceinline__ void agg_put(uint64_t* p, uint32_t epoch, const SegAgg& x) {
  gran_put(p, epoch, x.rows);
  gran_put(p + 1, epoch, x.mx > kPay ? kPay : x.mx);  // kTerm (the chain ended) -> kPay
  gran_put(p + 2, epoch, ((uint64_t)x.hs << 32) | x.fl);
}
__device__ __forceinline__ bool agg_get(const uint64_t* p, uint32_t epoch, SegAgg& x) {
  uint64_t a, b, c;
  const int ok = (int)gran_get(p, epoch, a) & (int)gran_get(p + 1, epoch, b) & (int)gran_get(p + 2, epoch, c);
  x.rows = a;
  x.mx = b == kPay ? kTerm : b;
  x.fl = (uint32_t)c;
  x.hs = (uint32_t)(c >> 32) & 1u;
  return ok != 0;
}

__device__ __forceinline__ SegAgg seg_shfl_down(const SegAgg& v, uint32_t o) {
  SegAgg u;
  u.rows = __shfl_down(v.rows, o, 64);
  u.mx = __shfl_down(v.mx, o, 64);
  u.fl = __shfl_down(v.fl, o, 64);
  u.hs = __shfl_down(v.hs, o, 64);
  return u;
}

// Ordered combination of the aggregates of elements [lo, hi) (state: 8 granules per element,
// aggregate at 0..2) by a whole 256-thread workgroup, 256 elements per round trip; every thread
// calls it and gets the result. An element that has not published yet is polled (elements are
// handed out in order, so it is being worked on); gives up (returns false) after about a quarter of
// a second of polling, so that a protocol fault ends in the repair path, not in a hung kernel.
__device__ bool block_prefix(const uint64_t* state, uint32_t epoch, uint64_t lo, uint64_t hi, SegAgg& out) {
  __shared__ uint32_t s_miss;
  __shared__ SegAgg s_w[4];
  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const SegAgg id{0, 0, 0xFFFFFFFFu, 0};
  SegAgg acc = id;
  uint32_t polls = 0;
  for (uint64_t r = lo; r < hi;) {
    const uint64_t j = r + tid;
    SegAgg v = id;
    bool have = true;
    if (j < hi) have = agg_get(state + 8ull * j, epoch, v);
    if (tid == 0) s_miss = 0;
    __syncthreads();
    if (!have) s_miss = 1;
    __syncthreads();
    const bool miss = s_miss != 0;
    __syncthreads();  // (s_miss is reset by the next round)
    if (miss) {
      if (++polls > (1u << 20)) return false;
      __builtin_amdgcn_s_sleep(2);
      continue;
    }
    // lane l + o holds newer elements than lane l
    for (uint32_t o = 1; o < 64; o <<= 1) {
      const SegAgg u = seg_shfl_down(v, o);
      if (lane + o < 64) v = seg_combine(v, u);
    }
    if (lane == 0) s_w[wave] = v;
    __syncthreads();
    acc = seg_combine(acc, seg_combine(seg_combine(seg_combine(s_w[0], s_w[1]), s_w[2]), s_w[3]));
    __syncthreads();
    r += 256;
  }
  out = acc;
  return true;
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
