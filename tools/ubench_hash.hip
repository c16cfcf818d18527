// Microbenchmark of the record-hash layouts of k_scan_chunks on gfx950 (not part of the product).
// A workgroup stages one 32 KiB window of 290-B records (the configs[1] shape) into LDS and hashes
// all its records ITERS times with one layout; cycles per pass and mismatches are reported, at 1 and
// 4 workgroups per CU.
//   quad_pair : 4 lanes per record (one XXH32 accumulator each), two records per quad (shipped)
//   quad_one  : 4 lanes per record, one record per quad at a time
//   lane_ilp4 : 1 lane per record, its 4 accumulators interleaved
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../cask_amd/csrc/device_util.h"

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

using namespace cask_dev;

constexpr uint32_t RL = 290, NREC = 113, WIN = NREC * RL + 64;

__device__ __forceinline__ uint32_t lane_ilp4(const uint32_t* w, uint32_t xs, uint32_t len) {
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

typedef __attribute__((address_space(1))) const u32x4 gu32x4;

// V 3 / 4: quad_pair while 9 16-B loads per thread (a 36 KiB window, the prefetch of k_scan_chunks)
// are in flight from `big`: into registers (3) or straight into a second LDS buffer by LDS-DMA (4).
template <int V>
__global__ __launch_bounds__(256) void k(const uint8_t* buf, uint32_t iters, uint32_t* bad, unsigned long long* cyc,
                                         const uint8_t* big, uint64_t big_n16) {
  __shared__ __attribute__((aligned(16))) uint32_t W[(WIN + 64) / 4 + (V == 4 ? 9 * 1024 : 0)];
  const uint32_t base = (blockIdx.x & 15) * 4 * RL;  // vary which records, keep 16-B aligned staging
  for (uint32_t i = threadIdx.x; i < (WIN + 15) / 16; i += 256)
    ((u32x4*)W)[i] = ((const u32x4*)(buf + base))[i];
  __syncthreads();
  const uint32_t tid = threadIdx.x, quad = tid >> 2, qa = tid & 3;
  uint32_t nbad = 0;
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  uint64_t gpos = ((uint64_t)blockIdx.x * 9 * 256) % (big_n16 - 9 * 256 * 2);
  u32x4 pf[9];
  for (uint32_t it = 0; it < iters; ++it) {
    if (V == 3) {
      const gu32x4* src = (const gu32x4*)big + gpos;
#pragma unroll
      for (int j = 0; j < 9; ++j) pf[j] = src[threadIdx.x + j * 256];
    }
    if (V == 4) {
      const uint8_t* src = big + gpos * 16;
#pragma unroll
      for (int j = 0; j < 9; ++j)
        __builtin_amdgcn_global_load_lds((const void*)(src + (threadIdx.x + j * 256) * 16),
                                         (__attribute__((address_space(3))) void*)(W + (WIN + 64) / 4 + j * 1024 + (threadIdx.x & ~63u) * 4), 16, 0, 0);
    }
    gpos += 9 * 256 * 1024 / 16;
    if (gpos + 9 * 256 >= big_n16) gpos = (gpos * 7) % (big_n16 - 9 * 256 * 2);
    if (V == 0 || V >= 3) {  // quad_pair
      for (uint32_t i0 = quad; i0 < NREC; i0 += 128) {
        const uint32_t i1 = i0 + 64 < NREC ? i0 + 64 : i0;
        const Hdr h0 = lds_hdr(W, i0 * RL), h1 = lds_hdr(W, i1 * RL);
        uint32_t g0, g1;
        quad_xxh32_pair(W, i0 * RL + 4, i1 * RL + 4, RL - 4, qa, g0, g1);
        nbad += (g0 != h0.stored) + (g1 != h1.stored);
      }
    } else if (V == 1) {
      for (uint32_t i = quad; i < NREC; i += 64) {
        const Hdr h = lds_hdr(W, i * RL);
        nbad += quad_xxh32(W, i * RL + 4, RL - 4, qa) != h.stored;
      }
    } else {
      for (uint32_t i = tid; i < NREC; i += 256) {
        const Hdr h = lds_hdr(W, i * RL);
        nbad += lane_ilp4(W, i * RL + 4, RL - 4) != h.stored;
      }
    }
    if (V == 3) {
      uint32_t x = 0;
#pragma unroll
      for (int j = 0; j < 9; ++j) x ^= pf[j].x ^ pf[j].w;
      nbad += x == 0x12345u;
    }
    if (V == 4) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (nbad) atomicAdd(bad, nbad);
  if (tid == 0) atomicAdd(cyc, (unsigned long long)(t1 - t0));
}

static uint32_t host_xxh(const uint8_t* p, uint32_t n) { return cask_xxh::xxh32(p, n, 0); }

int main() {
  std::vector<uint8_t> h(64 * RL * 16 + WIN + 256);
  uint64_t s = 0xC0FFEE;
  for (auto& b : h) { s = s * 6364136223846793005ull + 1442695040888963407ull; b = (uint8_t)(s >> 56); }
  for (uint32_t r = 0; r * RL + RL <= h.size(); ++r) {
    uint8_t* p = h.data() + (size_t)r * RL;
    uint64_t seq = r + 1; memcpy(p + 4, &seq, 8);
    uint16_t ksz = 16; memcpy(p + 12, &ksz, 2);
    uint32_t vsz = RL - 34; memcpy(p + 14, &vsz, 4);
    uint32_t x = host_xxh(p + 4, RL - 4); memcpy(p, &x, 4);
  }
  uint8_t* d; CK(hipMalloc(&d, h.size())); CK(hipMemcpy(d, h.data(), h.size(), hipMemcpyHostToDevice));
  uint32_t* bad; unsigned long long* cyc;
  CK(hipMalloc(&bad, 4)); CK(hipMalloc(&cyc, 8));
  const uint32_t iters = 200;
  const char* names[5] = {"quad_pair", "quad_one", "lane_ilp4", "pair+loads", "pair+glds"};
  const uint64_t big_bytes = 2ull << 30;
  uint8_t* big; CK(hipMalloc(&big, big_bytes)); CK(hipMemset(big, 1, big_bytes));
  for (int v = 0; v < 5; ++v) {
    for (uint32_t per_cu : {1u, 4u}) {
      const uint32_t grid = 256 * per_cu;
      for (int rep = 0; rep < 2; ++rep) {
        CK(hipMemset(bad, 0, 4)); CK(hipMemset(cyc, 0, 8));
        hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
        CK(hipEventRecord(a));
        const uint64_t bn = big_bytes / 16;
        if (v == 0) hipLaunchKernelGGL(k<0>, dim3(grid), dim3(256), 0, 0, d, iters, bad, cyc, big, bn);
        if (v == 1) hipLaunchKernelGGL(k<1>, dim3(grid), dim3(256), 0, 0, d, iters, bad, cyc, big, bn);
        if (v == 2) hipLaunchKernelGGL(k<2>, dim3(grid), dim3(256), 0, 0, d, iters, bad, cyc, big, bn);
        if (v == 3) hipLaunchKernelGGL(k<3>, dim3(grid), dim3(256), 0, 0, d, iters, bad, cyc, big, bn);
        if (v == 4) hipLaunchKernelGGL(k<4>, dim3(grid), dim3(256), 0, 0, d, iters, bad, cyc, big, bn);
        CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
        float ms; CK(hipEventElapsedTime(&ms, a, b));
        uint32_t hb; unsigned long long hc;
        CK(hipMemcpy(&hb, bad, 4, hipMemcpyDeviceToHost)); CK(hipMemcpy(&hc, cyc, 8, hipMemcpyDeviceToHost));
        if (rep == 1)
          printf("%-10s %u WG/CU: %.3f ms, %.0f cycles per pass per WG (113 x 290 B), chip %.0f GB/s-equivalent, bad=%u\n",
                 names[v], per_cu, ms, (double)hc / grid / iters, (double)grid * iters * NREC * RL / ms / 1e6, hb);
      }
    }
  }
  return 0;
}
