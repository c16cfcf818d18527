// Design microbenchmark (not part of the product): HBM read rate of the k_run_hash access pattern —
// every quad of lanes streams its own contiguous segment (a "record") in rounds of D 64-B blocks
// (one 16-B load per lane per block), the next round's loads in flight while the current one is
// mixed — by segment size, waves per CU, depth, with XXH32 mixing (quad_transpose + 4 rounds per
// block) or a plain XOR, and with the quads of a wave on adjacent or on scattered segments.
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/ubench_quads.hip -o tools/ubench_quads
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../cask_amd/csrc/device_util.h"

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

using namespace cask_dev;

// nseg segments of S bytes at base + perm(seg) * S + 4 (the body of a record: 4 B past its start);
// quad k of the grid takes segments k, k + Q, k + 2Q, ... (Q = quads in the grid).
template <uint32_t D, bool HASH, uint32_t OFF = 4>
__global__ __launch_bounds__(256) void k_quads(const uint8_t* __restrict__ base, uint64_t nseg, uint32_t S,
                                               uint32_t scatter, uint32_t* __restrict__ sink, uint32_t idle = 0,
                                               uint32_t extra = 0) {
  const uint32_t lane = threadIdx.x & 63, q = lane & 3;
  const uint64_t Q = (uint64_t)gridDim.x * 64, qid = (uint64_t)blockIdx.x * 64 + (threadIdx.x >> 2);
  const bool idleq = ((threadIdx.x >> 2) & 3) < idle;  // this quad reads the safe line only
  uint32_t v = q == 0 ? P1 + P2 : q == 1 ? P2 : q == 2 ? 0u : 0u - P1;
  const uint32_t nblk = (S - 64) / 64;  // full blocks of a segment's body
  for (uint64_t k = qid; k < nseg; k += Q) {
    const uint64_t seg = scatter ? (k * 0x9E3779B97F4A7C15ull) % nseg : k;  // (nseg odd: a permutation)
    const g_u8* lp = idleq ? (const g_u8*)(base + 16 * q) - 64 * 0 : (const g_u8*)(base + seg * S + OFF + 16 * q);
    const int64_t step = idleq ? 0 : 64;
    u32x4 A[D], B[D];
#pragma unroll
    for (uint32_t d = 0; d < D; ++d) A[d] = gld16g(lp + step * d);
    uint32_t b = D;
    for (;;) {
      const bool more = b + D <= nblk;
      if (more) {
#pragma unroll
        for (uint32_t d = 0; d < D; ++d) B[d] = gld16g(lp + step * (int64_t)(b + d));
        for (uint32_t e = 0; e < extra; ++e) B[0].x ^= gld4g(lp + 4 * e);
      }
#pragma unroll
      for (uint32_t d = 0; d < D; ++d) {
        u32x4 x = A[d];
        if (HASH) {
          quad_transpose(x, q);
          v = xround(xround(xround(xround(v, x.x), x.y), x.z), x.w);
        } else {
          v ^= x.x ^ x.y ^ x.z ^ x.w;
        }
      }
      if (!more) break;
#pragma unroll
      for (uint32_t d = 0; d < D; ++d) A[d] = B[d];
      b += D;
    }
  }
  if (v == 0x12345678u) sink[0] = v;
}

// The same segments, one lane per segment (all four XXH32 accumulators in the lane, no transpose):
// lane k of the grid takes segments k, k + N, ... (N = lanes in the grid), D 16-B loads per round.
template <uint32_t D, bool HASH>
__global__ __launch_bounds__(256) void k_lanes(const uint8_t* __restrict__ base, uint64_t nseg, uint32_t S,
                                               uint32_t scatter, uint32_t* __restrict__ sink) {
  const uint64_t N = (uint64_t)gridDim.x * 256, lid = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  uint32_t v0 = P1 + P2, v1 = P2, v2 = 0u, v3 = 0u - P1;
  const uint32_t nstr = (S - 64) / 16;  // full stripes read of a segment's body
  for (uint64_t k = lid; k < nseg; k += N) {
    const uint64_t seg = scatter ? (k * 0x9E3779B97F4A7C15ull) % nseg : k;
    const g_u8* lp = (const g_u8*)(base + seg * S + 4);
    u32x4 A[D], B[D];
#pragma unroll
    for (uint32_t d = 0; d < D; ++d) A[d] = gld16g(lp + 16 * d);
    uint32_t b = D;
    for (;;) {
      const bool more = b + D <= nstr;
      if (more) {
#pragma unroll
        for (uint32_t d = 0; d < D; ++d) B[d] = gld16g(lp + 16 * (b + d));
      }
#pragma unroll
      for (uint32_t d = 0; d < D; ++d) {
        const u32x4 x = A[d];
        if (HASH) {
          v0 = xround(v0, x.x);
          v1 = xround(v1, x.y);
          v2 = xround(v2, x.z);
          v3 = xround(v3, x.w);
        } else {
          v0 ^= x.x ^ x.y ^ x.z ^ x.w;
        }
      }
      if (!more) break;
#pragma unroll
      for (uint32_t d = 0; d < D; ++d) A[d] = B[d];
      b += D;
    }
  }
  if ((v0 ^ v1 ^ v2 ^ v3) == 0x12345678u) sink[0] = v0;
}


// Round 5: pairs of quads (octets) so that every load instruction covers whole 128-B lines. Octet o
// takes segments 2o (A, hashed by its low quad) and 2o + 1 (B, its high quad), 128-B aligned; per
// round D lines of each: instruction 2m loads line m of A (low quad its first 64 B, high quad its
// second), instruction 2m + 1 line m of B (low quad its second 64 B, high quad its first), so each
// quad has one of its blocks and the other comes from the partner lane (lane ^ 4, ds_swizzle).
// NT: nontemporal loads (whole lines per instruction: nothing of a line is left to fetch again).
template <uint32_t D, bool NT>
__global__ __launch_bounds__(256) void k_octets(const uint8_t* __restrict__ base, uint64_t nseg, uint32_t S,
                                                uint32_t scatter, uint32_t* __restrict__ sink) {
  const uint32_t lane = threadIdx.x & 63, q = lane & 3, h = (lane >> 2) & 1;
  const uint64_t O = (uint64_t)gridDim.x * 32, oid = (uint64_t)blockIdx.x * 32 + (threadIdx.x >> 3);
  uint32_t v = q == 0 ? P1 + P2 : q == 1 ? P2 : q == 2 ? 0u : 0u - P1;
  const uint32_t nline = S / 128;
  const uint64_t npair = nseg / 2;
  for (uint64_t k = oid; k < npair; k += O) {
    const uint64_t pr = scatter ? (k * 0x9E3779B97F4A7C15ull) % npair : k;
    const uint8_t* pa = base + (2 * pr) * (uint64_t)S + 64 * h + 16 * q;        // A: low quad first half
    const uint8_t* pb = base + (2 * pr + 1) * (uint64_t)S + 64 * (1 - h) + 16 * q;  // B: low quad second half
    u32x4 A[2 * D], B[2 * D];
    auto ld = [&](const uint8_t* p) __attribute__((always_inline)) -> u32x4 {
      return NT ? __builtin_nontemporal_load((const u32x4*)p) : *(const u32x4*)p;
    };
#pragma unroll
    for (uint32_t m = 0; m < D; ++m) {
      A[2 * m] = ld(pa + 128 * m);
      A[2 * m + 1] = ld(pb + 128 * m);
    }
    uint32_t l = D;
    for (;;) {
      const bool more = l + D <= nline;
      if (more) {
#pragma unroll
        for (uint32_t m = 0; m < D; ++m) {
          B[2 * m] = ld(pa + 128 * (l + m));
          B[2 * m + 1] = ld(pb + 128 * (l + m));
        }
      }
#pragma unroll
      for (uint32_t m = 0; m < D; ++m) {
        // low quad (A): own A[2m] first, then the high quad's A[2m]; high quad (B): own A[2m+1]
        // (B's first half), then the low quad's A[2m+1]
        const u32x4 xa = A[2 * m], xb = A[2 * m + 1];
        u32x4 f, g;
        f.x = h ? xb.x : xa.x; f.y = h ? xb.y : xa.y; f.z = h ? xb.z : xa.z; f.w = h ? xb.w : xa.w;
        g.x = h ? xa.x : xb.x; g.y = h ? xa.y : xb.y; g.z = h ? xa.z : xb.z; g.w = h ? xa.w : xb.w;
        u32x4 sdn;
        sdn.x = (uint32_t)__builtin_amdgcn_ds_swizzle((int)g.x, 0x101F);  // lane ^ 4 (bitmask mode: and 0x1F, xor 4)
        sdn.y = (uint32_t)__builtin_amdgcn_ds_swizzle((int)g.y, 0x101F);
        sdn.z = (uint32_t)__builtin_amdgcn_ds_swizzle((int)g.z, 0x101F);
        sdn.w = (uint32_t)__builtin_amdgcn_ds_swizzle((int)g.w, 0x101F);
        quad_transpose(f, q);
        v = xround(xround(xround(xround(v, f.x), f.y), f.z), f.w);
        quad_transpose(sdn, q);
        v = xround(xround(xround(xround(v, sdn.x), sdn.y), sdn.z), sdn.w);
      }
      if (!more) break;
#pragma unroll
      for (uint32_t d = 0; d < 2 * D; ++d) A[d] = B[d];
      l += D;
    }
  }
  if (v == 0x12345678u) sink[0] = v;
}

template <uint32_t D, bool NT>
static float run_octets(const uint8_t* buf, uint64_t bytes, uint32_t S, uint32_t waves_per_cu, uint32_t scatter, int cus,
                        uint32_t* sink) {
  uint64_t nseg = bytes / S;
  uint64_t npair = nseg / 2;
  if (!(npair & 1)) --npair;
  nseg = 2 * npair;
  const uint32_t grid = (uint32_t)(cus * waves_per_cu / 4);
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  hipLaunchKernelGGL((k_octets<D, NT>), dim3(grid), dim3(256), 0, 0, buf, nseg, S, scatter, sink);
  CK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int it = 0; it < 3; ++it) {
    CK(hipEventRecord(a));
    hipLaunchKernelGGL((k_octets<D, NT>), dim3(grid), dim3(256), 0, 0, buf, nseg, S, scatter, sink);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    best = ms < best ? ms : best;
  }
  const uint64_t nline = S / 128, rdl = nline >= D ? nline / D * D : D;
  const double rd = (double)nseg * (double)(rdl * 128);
  printf("octets D=%2u %s S=%6u waves/CU=%2u %s: %.3f ms %.0f GB/s read (%.3f GB per launch)\n", D, NT ? "nt   " : "plain",
         S, waves_per_cu, scatter ? "scattered" : "adjacent ", best, rd / best / 1e6, rd / 1e9);
  fflush(stdout);
  return best;
}


// The same with unaligned record bodies (byte `off` of the segment's first line, 0..127, varying by
// segment): whole lines are loaded, each body dword is funneled out of two line dwords (v_alignbyte,
// the lower one from the previous lane by DPP), lanes take the accumulator role of their dword
// position, and MASK 1 masks every word against the body's bounds (the line-aligned variant's cost),
// MASK 0 none (a lower bound on the VALU).
template <uint32_t D, bool NT, uint32_t MASK>
__global__ __launch_bounds__(256) void k_octets_al(const uint8_t* __restrict__ base, uint64_t nseg, uint32_t S,
                                                   uint32_t scatter, uint32_t* __restrict__ sink) {
  const uint32_t lane = threadIdx.x & 63, q = lane & 3, h = (lane >> 2) & 1;
  const uint64_t O = (uint64_t)gridDim.x * 32, oid = (uint64_t)blockIdx.x * 32 + (threadIdx.x >> 3);
  uint32_t acc = 0;
  const uint32_t nline = S / 128;
  const uint64_t npair = nseg / 2;
  for (uint64_t k = oid; k < npair; k += O) {
    const uint64_t pr = scatter ? (k * 0x9E3779B97F4A7C15ull) % npair : k;
    const uint64_t mine = 2 * pr + h;
    const uint32_t off = (uint32_t)((mine * 0x2545F491ull) >> 7) & 127u;  // body start in the first line
    const uint32_t sb = off & 3, cM = off >> 2;
    const uint32_t j = (q - cM - 1) & 3;
    uint32_t v = j == 0 ? P1 + P2 : j == 1 ? P2 : j == 2 ? 0u : 0u - P1;
    const int32_t lo = (int32_t)cM + 1, hi = (int32_t)(nline * 32) - 8;  // body dwords (line dword index)
    uint32_t carry = 0;
    const uint8_t* pa = base + (2 * pr) * (uint64_t)S + 64 * h + 16 * q;
    const uint8_t* pb = base + (2 * pr + 1) * (uint64_t)S + 64 * (1 - h) + 16 * q;
    u32x4 A[2 * D], B[2 * D];
    auto ld = [&](const uint8_t* p) __attribute__((always_inline)) -> u32x4 {
      return NT ? __builtin_nontemporal_load((const u32x4*)p) : *(const u32x4*)p;
    };
#pragma unroll
    for (uint32_t m = 0; m < D; ++m) {
      A[2 * m] = ld(pa + 128 * m);
      A[2 * m + 1] = ld(pb + 128 * m);
    }
    uint32_t l = D;
    for (;;) {
      const bool more = l + D <= nline;
      if (more) {
#pragma unroll
        for (uint32_t m = 0; m < D; ++m) {
          B[2 * m] = ld(pa + 128 * (l + m));
          B[2 * m + 1] = ld(pb + 128 * (l + m));
        }
      }
      const int32_t r0 = (int32_t)((l - D) * 32);  // line dword index of the round's first dword
#pragma unroll
      for (uint32_t m = 0; m < D; ++m) {
        const u32x4 xa = A[2 * m], xb = A[2 * m + 1];
        u32x4 blk[2], g;
        blk[0].x = h ? xb.x : xa.x; blk[0].y = h ? xb.y : xa.y; blk[0].z = h ? xb.z : xa.z; blk[0].w = h ? xb.w : xa.w;
        g.x = h ? xa.x : xb.x; g.y = h ? xa.y : xb.y; g.z = h ? xa.z : xb.z; g.w = h ? xa.w : xb.w;
        blk[1].x = (uint32_t)__builtin_amdgcn_ds_swizzle((int)g.x, 0x101F);
        blk[1].y = (uint32_t)__builtin_amdgcn_ds_swizzle((int)g.y, 0x101F);
        blk[1].z = (uint32_t)__builtin_amdgcn_ds_swizzle((int)g.z, 0x101F);
        blk[1].w = (uint32_t)__builtin_amdgcn_ds_swizzle((int)g.w, 0x101F);
#pragma unroll
        for (uint32_t e = 0; e < 2; ++e) {
          const u32x4 gg = blk[e];
          const uint32_t dv = (uint32_t)__builtin_amdgcn_mov_dpp((int)gg.w, 0x93, 0xF, 0xF, false);  // [3,0,1,2]
          const uint32_t p0 = q == 0 ? carry : dv;
          carry = dv;
          u32x4 x = u32x4{fun(p0, gg.x, sb), fun(gg.x, gg.y, sb), fun(gg.y, gg.z, sb), fun(gg.z, gg.w, sb)};
          quad_transpose(x, q);
#pragma unroll
          for (uint32_t kk = 0; kk < 4; ++kk) {
            uint32_t w = xround(v, x[kk]);
            if (MASK) {
              const int32_t t = r0 + 32 * (int32_t)m + 16 * (int32_t)e + 4 * (int32_t)kk + (int32_t)q;
              asm volatile("" : "+v"(w));
              v = (t >= lo && t <= hi) ? w : v;
            } else {
              v = w;
            }
          }
        }
      }
      if (!more) break;
#pragma unroll
      for (uint32_t d = 0; d < 2 * D; ++d) A[d] = B[d];
      l += D;
    }
    acc ^= v;
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

template <uint32_t D, bool NT, uint32_t MASK>
static float run_octets_al(const uint8_t* buf, uint64_t bytes, uint32_t S, uint32_t waves_per_cu, uint32_t scatter,
                           int cus, uint32_t* sink) {
  uint64_t nseg = bytes / S;
  uint64_t npair = nseg / 2;
  if (!(npair & 1)) --npair;
  nseg = 2 * npair;
  const uint32_t grid = (uint32_t)(cus * waves_per_cu / 4);
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  hipLaunchKernelGGL((k_octets_al<D, NT, MASK>), dim3(grid), dim3(256), 0, 0, buf, nseg, S, scatter, sink);
  CK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int it = 0; it < 3; ++it) {
    CK(hipEventRecord(a));
    hipLaunchKernelGGL((k_octets_al<D, NT, MASK>), dim3(grid), dim3(256), 0, 0, buf, nseg, S, scatter, sink);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    best = ms < best ? ms : best;
  }
  const uint64_t nline = S / 128, rdl = nline >= D ? nline / D * D : D;
  const double rd = (double)nseg * (double)(rdl * 128);
  printf("octets_al D=%2u %s mask=%u S=%6u waves/CU=%2u %s: %.3f ms %.0f GB/s read (%.3f GB per launch)\n", D,
         NT ? "nt   " : "plain", MASK, S, waves_per_cu, scatter ? "scattered" : "adjacent ", best, rd / best / 1e6,
         rd / 1e9);
  fflush(stdout);
  return best;
}

template <uint32_t D, bool HASH>
static float run_lanes(const uint8_t* buf, uint64_t bytes, uint32_t S, uint32_t waves_per_cu, uint32_t scatter, int cus,
                       uint32_t* sink) {
  uint64_t nseg = bytes / S;
  if (!(nseg & 1)) --nseg;
  const uint32_t grid = (uint32_t)(cus * waves_per_cu / 4);
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  hipLaunchKernelGGL((k_lanes<D, HASH>), dim3(grid), dim3(256), 0, 0, buf, nseg, S, scatter, sink);
  CK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int it = 0; it < 3; ++it) {
    CK(hipEventRecord(a));
    hipLaunchKernelGGL((k_lanes<D, HASH>), dim3(grid), dim3(256), 0, 0, buf, nseg, S, scatter, sink);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    best = ms < best ? ms : best;
  }
  const uint64_t nstr = (S - 64) / 16, rds = nstr >= D ? nstr / D * D : D;
  const double rd = (double)nseg * (double)(rds * 16);
  printf("lanes D=%2u %s S=%6u waves/CU=%2u %s: %.3f ms %.0f GB/s\n", D, HASH ? "hash" : "xor ", S, waves_per_cu,
         scatter ? "scattered" : "adjacent ", best, rd / best / 1e6);
  fflush(stdout);
  return best;
}

template <uint32_t D, bool HASH, uint32_t OFF = 4>
static float run(const uint8_t* buf, uint64_t bytes, uint32_t S, uint32_t waves_per_cu, uint32_t scatter, int cus,
                 uint32_t* sink, uint32_t idle = 0, uint32_t extra = 0) {
  uint64_t nseg = bytes / S;
  if (!(nseg & 1)) --nseg;
  const uint32_t grid = (uint32_t)(cus * waves_per_cu / 4);
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  hipLaunchKernelGGL((k_quads<D, HASH, OFF>), dim3(grid), dim3(256), 0, 0, buf, nseg, S, scatter, sink, idle, extra);
  CK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int it = 0; it < 3; ++it) {
    CK(hipEventRecord(a));
    hipLaunchKernelGGL((k_quads<D, HASH, OFF>), dim3(grid), dim3(256), 0, 0, buf, nseg, S, scatter, sink, idle, extra);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    best = ms < best ? ms : best;
  }
  // bytes read: the rounds of D blocks that fit a segment's nblk full blocks (D * floor(nblk / D)),
  // by the non-idle quads (round 3: counting all nblk blocks overstated short segments by up to 2x)
  const uint64_t nblk = (S - 64) / 64, rdb = nblk >= D ? nblk / D * D : D;
  const double rd = (double)nseg * (double)(rdb * 64) * (4 - idle) / 4.0;
  printf("D=%2u %s S=%6u off=%u waves/CU=%2u %s idle=%u/4 extra=%u: %.3f ms %.0f GB/s read (%.3f GB per launch)\n", D,
         HASH ? "hash" : "xor ", S, OFF, waves_per_cu, scatter ? "scattered" : "adjacent ", idle, extra, best,
         rd / best / 1e6, rd / 1e9);
  fflush(stdout);
  return best;
}

int main(int argc, char** argv) {
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const uint64_t bytes = 16ull << 30;
  uint8_t* buf;
  CK(hipMalloc(&buf, bytes + 4096));
  CK(hipMemset(buf, 0x5A, bytes + 4096));
  uint32_t* sink;
  CK(hipMalloc(&sink, 64));
  const bool sweep = argc > 1 && argv[1][0] == 's';  // depth / occupancy / mixing sweep (round 3)
  if (argc > 1 && argv[1][0] == 'o') {  // round 4: record bodies at +4 (rounds share a line) vs 128-B aligned rounds
    for (uint32_t S : {8192u, 65536u}) {
      run<16, true, 4>(buf, bytes, S, 8, 1, cus, sink);
      run<16, true, 0>(buf, bytes, S, 8, 1, cus, sink);
      run<16, true, 64>(buf, bytes, S, 8, 1, cus, sink);
    }
    return 0;
  }  // depth / occupancy / mixing sweep (round 3)
  if (argc > 1 && argv[1][0] == 'w') {  // round 5: whole-line octets (plain / nontemporal) vs aligned quads
    for (uint32_t S : {4096u, 8192u, 65536u}) {
      run<16, true, 0>(buf, bytes, S, 8, 1, cus, sink);
      run_octets<8, false>(buf, bytes, S, 8, 1, cus, sink);
      run_octets<8, true>(buf, bytes, S, 8, 1, cus, sink);
      run_octets_al<8, true, 0>(buf, bytes, S, 8, 1, cus, sink);
      run_octets_al<8, true, 1>(buf, bytes, S, 8, 1, cus, sink);
      run_octets_al<8, false, 1>(buf, bytes, S, 8, 1, cus, sink);
    }
    return 0;
  }
  if (argc > 1 && argv[1][0] == 'a') {  // adjacent (a wave's quads on consecutive segments) vs scattered
    for (uint32_t S : {2048u, 4096u, 8192u, 16384u, 65536u})
      for (uint32_t sc : {0u, 1u}) run<16, true>(buf, bytes, S, 8, sc, cus, sink);
    return 0;
  }
  for (uint32_t S : {8192u, 65536u}) {
    if (sweep) {
      run<16, true>(buf, bytes, S, 8, 1, cus, sink);
      run<16, false>(buf, bytes, S, 8, 1, cus, sink);
      run<16, false>(buf, bytes, S, 12, 1, cus, sink);
      run<8, true>(buf, bytes, S, 8, 1, cus, sink);
      run<8, true>(buf, bytes, S, 16, 1, cus, sink);
      run<8, false>(buf, bytes, S, 16, 1, cus, sink);
      run<32, false>(buf, bytes, S, 4, 1, cus, sink);
      run<32, false>(buf, bytes, S, 8, 1, cus, sink);
      run_lanes<16, true>(buf, bytes, S, 8, 1, cus, sink);
      continue;
    }
    run<16, true>(buf, bytes, S, 8, 1, cus, sink, 0, 0);
    run<16, true>(buf, bytes, S, 8, 1, cus, sink, 1, 0);
    run<16, true>(buf, bytes, S, 8, 1, cus, sink, 2, 0);
    run<16, true>(buf, bytes, S, 8, 1, cus, sink, 0, 2);
    run<16, true>(buf, bytes, S, 8, 1, cus, sink, 0, 4);
  }
  return 0;
}
