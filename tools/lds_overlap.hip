// Diagnostic: do co-resident workgroups ever see each other's LDS? Each workgroup tags its whole
// static LDS block with its id, then re-reads it many times; any foreign value is counted.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

template <int WORDS, int NT>
__global__ __launch_bounds__(NT) void k_tag(unsigned long long* bad, unsigned long long* first, int iters) {
  __shared__ unsigned buf[WORDS];
  const unsigned tag = blockIdx.x * 65536u;
  for (int i = threadIdx.x; i < WORDS; i += NT) buf[i] = tag + (i & 0xFFFF);
  __syncthreads();
  for (int it = 0; it < iters; ++it) {
    for (int i = threadIdx.x; i < WORDS; i += NT) {
      const unsigned v = buf[i];
      if (v != tag + (i & 0xFFFF)) {
        atomicAdd(bad, 1ull);
        atomicCAS(first, 0ull, ((unsigned long long)blockIdx.x << 40) | ((unsigned long long)i << 20) | (v >> 16));
      }
    }
    __builtin_amdgcn_s_sleep(2);
  }
}

template <int WORDS, int NT>
static void run(const char* name, int grid, int iters) {
  unsigned long long *d, h[2];
  hipMalloc(&d, 16);
  hipMemset(d, 0, 16);
  hipLaunchKernelGGL((k_tag<WORDS, NT>), dim3(grid), dim3(NT), 0, 0, d, d + 1, iters);
  hipError_t e = hipDeviceSynchronize();
  hipMemcpy(h, d, 16, hipMemcpyDeviceToHost);
  printf("%s: words %d (%d B) threads %d grid %d -> %s, bad %llu first blk %llu idx %llu\n", name, WORDS, WORDS * 4,
         NT, grid, hipGetErrorString(e), h[0], h[1] >> 40, (h[1] >> 20) & 0xFFFFF);
  hipFree(d);
}

int main() {
  run<10148, 256>("geoA-like", 4096, 200);
  run<4956, 128>("geoB-like", 8192, 200);
  run<2552, 64>("geoC-like", 16384, 200);
  run<16384, 256>("64KB", 2048, 200);
  return 0;
}
