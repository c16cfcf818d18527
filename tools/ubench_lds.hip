// LDS read microbenchmark for the scan's access shapes on gfx950 (not part of the product):
// cycles per wave-instruction of aligned vs unaligned ds_read_b32/b64/b128 at the strides the
// record hashing uses (lanes of a quad on consecutive dwords, quads 290 B apart).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

template <int W>
__device__ __forceinline__ uint32_t rd(const uint8_t* lds, uint32_t x) {
  if (W == 4) { uint32_t v; __builtin_memcpy(&v, lds + x, 4); return v; }
  if (W == 8) { u32x2 v; __builtin_memcpy(&v, lds + x, 8); return v.x ^ v.y; }
  u32x4 v; __builtin_memcpy(&v, lds + x, 16); return v.x ^ v.y ^ v.z ^ v.w;
}

// mode 0: lane-per-record (lane stride `rs`), mode 1: quad-per-record (quad stride rs, lane a at +4a)
template <int W, int MODE>
__global__ __launch_bounds__(256) void k(uint32_t mis, uint32_t rs, uint32_t iters, uint32_t* out, unsigned long long* cyc) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[65536];
  for (uint32_t i = threadIdx.x; i < 65536 / 4; i += 256) ((uint32_t*)lds)[i] = i * 2654435761u;
  __syncthreads();
  const uint32_t l = threadIdx.x;
  uint32_t base = MODE == 0 ? (l & 63) * rs : (((l & 63) >> 2) * rs + 4 * (l & 3));
  base = (base + mis) & 16383;
  uint32_t acc = 0;
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (uint32_t it = 0; it < iters; ++it) {
    const uint32_t x = (base + it * 16) & 32767;
    acc += rd<W>(lds, x);
    acc += rd<W>(lds, x + 16);
    acc += rd<W>(lds, x + 32);
    acc += rd<W>(lds, x + 48);
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (acc == 0x12345u) out[0] = acc;
  if (threadIdx.x == 0) atomicAdd(cyc, (unsigned long long)(t1 - t0));
}

template <int W, int MODE>
static void run(const char* name, uint32_t mis, uint32_t rs) {
  uint32_t* out; unsigned long long* cyc;
  CK(hipMalloc(&out, 64)); CK(hipMalloc(&cyc, 8)); CK(hipMemset(cyc, 0, 8));
  const uint32_t iters = 4096, grid = 256 * 2;
  hipLaunchKernelGGL((k<W, MODE>), dim3(grid), dim3(256), 0, 0, mis, rs, iters, out, cyc);
  CK(hipDeviceSynchronize());
  CK(hipMemset(cyc, 0, 8));
  hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  CK(hipEventRecord(a));
  hipLaunchKernelGGL((k<W, MODE>), dim3(grid), dim3(256), 0, 0, mis, rs, iters, out, cyc);
  CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
  float ms; CK(hipEventElapsedTime(&ms, a, b));
  unsigned long long c; CK(hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost));
  const double insts = (double)grid * 4 * iters * 4;  // wave-instructions
  const double bytes = insts * 64 * W;
  printf("%-34s mis=%u rs=%3u: %.3f ms  %.1f TB/s LDS  %.2f ns/wave-inst/CU  memtime/wg-iter %.1f\n", name, mis, rs, ms,
         bytes / ms / 1e9, ms * 1e6 / (insts / 256), (double)c / grid / iters);
  CK(hipFree(out)); CK(hipFree(cyc));
}

int main() {
  for (uint32_t mis : {0u, 1u, 2u}) {
    run<4, 1>("quad b32", mis, 290);
    run<4, 1>("quad b32 rs=288", mis, 288);
    run<8, 1>("quad b64", mis, 290);
    run<16, 0>("lane b128", mis, 290);
    run<16, 0>("lane b128 rs=288", mis, 288);
    run<4, 0>("lane b32", mis, 290);
  }
  return 0;
}
