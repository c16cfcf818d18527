// Microbenchmark: the dense-row store pattern of k_finish (5 SoA arrays: pos u64, seq u64, vsz u32,
// ksz u16, status u8) at configs[1] size (29.6 M rows), trivial values, three thread layouts.
//   hipcc -O3 --offload-arch=gfx950 tools/ubench_store.hip -o tools/ubench_store && tools/ubench_store
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void k4(uint64_t* pos, uint64_t* seq, uint32_t* vsz, uint16_t* ksz, uint8_t* st, uint64_t n) {
  for (uint64_t g = blockIdx.x * 256ull + threadIdx.x; g * 4 < n; g += (uint64_t)gridDim.x * 256) {
    const uint64_t d = g * 4;
    *(u64x2*)(pos + d) = u64x2{d, d + 1};
    *(u64x2*)(pos + d + 2) = u64x2{d + 2, d + 3};
    *(u64x2*)(seq + d) = u64x2{d, d + 1};
    *(u64x2*)(seq + d + 2) = u64x2{d + 2, d + 3};
    *(u32x4*)(vsz + d) = u32x4{256u, 256u, 256u, 256u};
    *(uint64_t*)(ksz + d) = 0x0010001000100010ull;
    *(uint32_t*)(st + d) = 0;
  }
}
__global__ __launch_bounds__(256) void k8(uint64_t* pos, uint64_t* seq, uint32_t* vsz, uint16_t* ksz, uint8_t* st, uint64_t n) {
  for (uint64_t g = blockIdx.x * 256ull + threadIdx.x; g * 8 < n; g += (uint64_t)gridDim.x * 256) {
    const uint64_t d = g * 8;
#pragma unroll
    for (int k = 0; k < 4; ++k) *(u64x2*)(pos + d + 2 * k) = u64x2{d + 2 * k, d + 2 * k + 1};
#pragma unroll
    for (int k = 0; k < 4; ++k) *(u64x2*)(seq + d + 2 * k) = u64x2{d + 2 * k, d + 2 * k + 1};
    *(u32x4*)(vsz + d) = u32x4{256u, 256u, 256u, 256u};
    *(u32x4*)(vsz + d + 4) = u32x4{256u, 256u, 256u, 256u};
    *(u32x4*)(ksz + d) = u32x4{0x00100010u, 0x00100010u, 0x00100010u, 0x00100010u};
    *(uint64_t*)(st + d) = 0;
  }
}
__global__ __launch_bounds__(256) void k1(uint64_t* pos, uint64_t* seq, uint32_t* vsz, uint16_t* ksz, uint8_t* st, uint64_t n) {
  for (uint64_t d = blockIdx.x * 256ull + threadIdx.x; d < n; d += (uint64_t)gridDim.x * 256) {
    pos[d] = d;
    seq[d] = d;
    vsz[d] = 256;
    ksz[d] = 16;
    st[d] = 0;
  }
}

int main() {
  const uint64_t n = 29620464;
  uint64_t *pos, *seq;
  uint32_t* vsz;
  uint16_t* ksz;
  uint8_t* st;
  hipMalloc(&pos, n * 8 + 64);
  hipMalloc(&seq, n * 8 + 64);
  hipMalloc(&vsz, n * 4 + 64);
  hipMalloc(&ksz, n * 2 + 64);
  hipMalloc(&st, n + 64);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const char* names[3] = {"4 rows/thread", "8 rows/thread", "1 row/lane"};
  for (int rep = 0; rep < 3; ++rep)
    for (int v = 0; v < 3; ++v)
      for (int grid : {1024, 2048, 8192}) {
        float best = 1e9f;
        for (int it = 0; it < 10; ++it) {
          hipEventRecord(e0);
          if (v == 0) hipLaunchKernelGGL(k4, dim3(grid), dim3(256), 0, 0, pos, seq, vsz, ksz, st, n);
          else if (v == 1) hipLaunchKernelGGL(k8, dim3(grid), dim3(256), 0, 0, pos, seq, vsz, ksz, st, n);
          else hipLaunchKernelGGL(k1, dim3(grid), dim3(256), 0, 0, pos, seq, vsz, ksz, st, n);
          hipEventRecord(e1);
          hipEventSynchronize(e1);
          float ms;
          hipEventElapsedTime(&ms, e0, e1);
          if (ms < best) best = ms;
        }
        if (rep == 2) printf("%-14s grid %5d: %.1f us  %.2f TB/s\n", names[v], grid, best * 1e3, n * 23.0 / (best * 1e-3) / 1e12);
      }
  return 0;
}
