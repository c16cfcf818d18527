// Design microbenchmarks for the Cask scan kernels on gfx950 (not part of the product).
// Answers: (1) read-stream ceiling, (2) XXH32 VALU ceiling, (3) lane-per-record hashing
// straight from HBM with unaligned 16-B loads vs aligned loads + alignbyte, (4) via LDS.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include <chrono>
#include "../cask_amd/csrc/xxh32.h"

using namespace cask_xxh;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__global__ void stream_read(const u32x4* __restrict__ p, size_t n, uint32_t* out) {
  uint32_t acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    u32x4 v = p[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) out[0] = acc;
}

// VALU ceiling: hash `stripes` synthetic stripes per lane.
__global__ void hash_regs(uint32_t stripes, uint32_t* out) {
  uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  Acc a = acc_init(0);
  uint32_t w0 = t, w1 = t * 3, w2 = t * 5, w3 = t * 7;
  for (uint32_t s = 0; s < stripes; ++s) {
    acc_stripe(a, w0, w1, w2, w3);
    w0 += 1; w1 += 1; w2 += 1; w3 += 1;
  }
  uint32_t h = avalanche(acc_merge(a));
  if (h == 0x12345678u) out[0] = h;
}

__device__ __forceinline__ u32x4 ld16_unaligned(const uint8_t* p) {
  u32x4 v;
  __builtin_memcpy(&v, p, 16);
  return v;
}
__device__ __forceinline__ uint32_t ld4_unaligned(const uint8_t* p) {
  uint32_t v;
  __builtin_memcpy(&v, p, 4);
  return v;
}

// Records of fixed length L packed from offset 0; hash bytes [4, L) of each, compare to stored.
__global__ void hash_global_unaligned(const uint8_t* __restrict__ buf, uint32_t L, uint32_t nrec, uint32_t* out_bad) {
  uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= nrec) return;
  const uint8_t* p = buf + (size_t)r * L;
  uint32_t stored = ld4_unaligned(p);
  const uint8_t* q = p + 4;
  uint32_t len = L - 4;
  const uint8_t* end = q + len;
  Acc a = acc_init(0);
  uint32_t nstr = len >> 4;
  for (uint32_t s = 0; s < nstr; ++s) {
    u32x4 v = ld16_unaligned(q);
    acc_stripe(a, v.x, v.y, v.z, v.w);
    q += 16;
  }
  uint32_t h = (len >= 16 ? acc_merge(a) : P5) + len;
  while (q + 4 <= end) { h = tail4(h, ld4_unaligned(q)); q += 4; }
  while (q < end) { h = tail1(h, *q); ++q; }
  h = avalanche(h);
  if (h != stored) atomicAdd(out_bad, 1u);
}

// Aligned dword loads + alignbyte funnel.
__global__ void hash_global_alignbyte(const uint8_t* __restrict__ buf, uint32_t L, uint32_t nrec, uint32_t* out_bad) {
  uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= nrec) return;
  size_t p = (size_t)r * L;
  const uint32_t* w = (const uint32_t*)buf;
  size_t q = p + 4;
  uint32_t sh = (uint32_t)(q & 3);
  size_t wi = q >> 2;
  uint32_t stored;
  {
    size_t pi = p >> 2; uint32_t ps = p & 3;
    stored = __builtin_amdgcn_alignbyte(w[pi + 1], w[pi], ps);
  }
  uint32_t len = L - 4;
  Acc a = acc_init(0);
  uint32_t nstr = len >> 4;
  uint32_t prev = w[wi];
  for (uint32_t s = 0; s < nstr; ++s) {
    uint32_t d1 = w[wi + 1], d2 = w[wi + 2], d3 = w[wi + 3], d4 = w[wi + 4];
    acc_stripe(a, __builtin_amdgcn_alignbyte(d1, prev, sh), __builtin_amdgcn_alignbyte(d2, d1, sh),
               __builtin_amdgcn_alignbyte(d3, d2, sh), __builtin_amdgcn_alignbyte(d4, d3, sh));
    prev = d4;
    wi += 4;
  }
  uint32_t h = (len >= 16 ? acc_merge(a) : P5) + len;
  uint32_t rem = len & 15;
  while (rem >= 4) { uint32_t d1 = w[wi + 1]; h = tail4(h, __builtin_amdgcn_alignbyte(d1, prev, sh)); prev = d1; wi++; rem -= 4; }
  size_t qb = (wi << 2) + sh;
  while (rem) { h = tail1(h, buf[qb]); ++qb; --rem; }
  h = avalanche(h);
  if (h != stored) atomicAdd(out_bad, 1u);
}

// LDS staged: block owns CH bytes window (record-aligned for this ubench: CH multiple of L).
template <int CH>
__global__ __launch_bounds__(256) void hash_lds(const uint8_t* __restrict__ buf, uint32_t L, size_t total, uint32_t* out_bad) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[CH + 16];
  size_t c0 = (size_t)blockIdx.x * CH;
  if (c0 >= total) return;
  uint32_t n = (uint32_t)((total - c0) < CH ? (total - c0) : CH);
  const u32x4* src = (const u32x4*)(buf + c0);
  u32x4* dst = (u32x4*)lds;
  for (uint32_t i = threadIdx.x; i < (n + 15) / 16; i += 256) dst[i] = src[i];
  __syncthreads();
  uint32_t nrec = n / L;
  const uint32_t* w = (const uint32_t*)lds;
  for (uint32_t r = threadIdx.x; r < nrec; r += 256) {
    uint32_t p = r * L;
    uint32_t q = p + 4;
    uint32_t sh = q & 3;
    uint32_t wi = q >> 2;
    uint32_t stored = __builtin_amdgcn_alignbyte(w[(p >> 2) + 1], w[p >> 2], p & 3);
    uint32_t len = L - 4;
    Acc a = acc_init(0);
    uint32_t nstr = len >> 4;
    uint32_t prev = w[wi];
    for (uint32_t s = 0; s < nstr; ++s) {
      uint32_t d1 = w[wi + 1], d2 = w[wi + 2], d3 = w[wi + 3], d4 = w[wi + 4];
      acc_stripe(a, __builtin_amdgcn_alignbyte(d1, prev, sh), __builtin_amdgcn_alignbyte(d2, d1, sh),
                 __builtin_amdgcn_alignbyte(d3, d2, sh), __builtin_amdgcn_alignbyte(d4, d3, sh));
      prev = d4;
      wi += 4;
    }
    uint32_t h = (len >= 16 ? acc_merge(a) : P5) + len;
    uint32_t rem = len & 15;
    while (rem >= 4) { uint32_t d1 = w[wi + 1]; h = tail4(h, __builtin_amdgcn_alignbyte(d1, prev, sh)); prev = d1; wi++; rem -= 4; }
    uint32_t qb = (wi << 2) + sh;
    while (rem) { h = tail1(h, lds[qb]); ++qb; --rem; }
    h = avalanche(h);
    if (h != stored) atomicAdd(out_bad, 1u);
  }
}

static void make_records(std::vector<uint8_t>& host, uint32_t L, uint32_t nrec) {
  host.assign((size_t)L * nrec + 64, 0);
  uint64_t s = 0xC0FFEE;
  for (size_t i = 0; i < host.size(); ++i) {
    s = s * 6364136223846793005ull + 1442695040888963407ull;
    host[i] = (uint8_t)(s >> 56);
  }
  for (uint32_t r = 0; r < nrec; ++r) {
    uint8_t* p = host.data() + (size_t)r * L;
    uint64_t seq = r + 1; memcpy(p + 4, &seq, 8);
    uint16_t ksz = 16; memcpy(p + 12, &ksz, 2);
    uint32_t vsz = L - 34; memcpy(p + 16 - 2, &vsz, 4);
    uint32_t h = xxh32(p + 4, L - 4, 0);
    memcpy(p, &h, 4);
  }
}

template <typename F>
static float time_ms(F f, int iters) {
  hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  f();
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a));
  for (int i = 0; i < iters; ++i) f();
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms; CK(hipEventElapsedTime(&ms, a, b));
  return ms / iters;
}

int main() {
  uint32_t* d_out; CK(hipMalloc(&d_out, 64)); CK(hipMemset(d_out, 0, 64));
  // 1. stream read, 4 GiB
  {
    size_t bytes = 4ull << 30;
    void* d; CK(hipMalloc(&d, bytes)); CK(hipMemset(d, 1, bytes));
    size_t n = bytes / 16;
    for (int grid : {1024, 2048, 4096, 8192}) {
      float ms = time_ms([&] { stream_read<<<grid, 256>>>((const u32x4*)d, n, d_out); }, 10);
      printf("stream_read grid=%d: %.3f ms  %.1f GB/s\n", grid, ms, bytes / ms / 1e6);
    }
    CK(hipFree(d));
  }
  // 2. hash ceiling
  {
    uint32_t stripes = 4096; int grid = 8192;
    float ms = time_ms([&] { hash_regs<<<grid, 256>>>(stripes, d_out); }, 5);
    double bytes = (double)grid * 256 * stripes * 16;
    printf("hash_regs: %.3f ms  %.1f GB/s equivalent\n", ms, bytes / ms / 1e6);
  }
  // 3/4. record hashing, 290 B and 82 B
  for (uint32_t L : {290u, 82u}) {
    uint32_t nrec = (uint32_t)((2ull << 30) / L);
    std::vector<uint8_t> host;
    make_records(host, L, nrec);
    uint8_t* d; CK(hipMalloc(&d, host.size() + 256));
    CK(hipMemcpy(d, host.data(), host.size(), hipMemcpyHostToDevice));
    size_t total = (size_t)L * nrec;
    int grid = (nrec + 255) / 256;
    CK(hipMemset(d_out, 0, 64));
    float ms = time_ms([&] { hash_global_unaligned<<<grid, 256>>>(d, L, nrec, d_out); }, 5);
    uint32_t bad; CK(hipMemcpy(&bad, d_out, 4, hipMemcpyDeviceToHost));
    printf("L=%u hash_global_unaligned: %.3f ms %.1f GB/s bad=%u (of %u x6)\n", L, ms, total / ms / 1e6, bad, nrec);
    CK(hipMemset(d_out, 0, 64));
    ms = time_ms([&] { hash_global_alignbyte<<<grid, 256>>>(d, L, nrec, d_out); }, 5);
    CK(hipMemcpy(&bad, d_out, 4, hipMemcpyDeviceToHost));
    printf("L=%u hash_global_alignbyte: %.3f ms %.1f GB/s bad=%u\n", L, ms, total / ms / 1e6, bad);
    // LDS: CH multiple of L
    {
      constexpr int CH = 32768;
      uint32_t ch = (CH / L) * L;
      // use a per-L chunk: recompute by launching with exact record-aligned chunks (emulate via L-multiple)
      (void)ch;
    }
    CK(hipMemset(d_out, 0, 64));
    if (L == 290) {
      constexpr int CH = 290 * 112;  // 32480
      int g2 = (int)((total + CH - 1) / CH);
      ms = time_ms([&] { hash_lds<CH><<<g2, 256>>>(d, L, total, d_out); }, 5);
    } else {
      constexpr int CH = 82 * 400;  // 32800
      int g2 = (int)((total + CH - 1) / CH);
      ms = time_ms([&] { hash_lds<CH><<<g2, 256>>>(d, L, total, d_out); }, 5);
    }
    CK(hipMemcpy(&bad, d_out, 4, hipMemcpyDeviceToHost));
    printf("L=%u hash_lds: %.3f ms %.1f GB/s bad=%u\n", L, ms, total / ms / 1e6, bad);
    CK(hipFree(d));
  }
  return 0;
}
