// Diagnostic: issue rate of the integer ops XXH32 uses on gfx950 (v_mul_lo_u32,
// v_mad_u64_u32, v_alignbit_b32, v_add_u32), 8 independent chains per lane, enough waves to
// fill every SIMD. Prints cycles per wave-instruction (s_memtime, one SIMD's view).
#include <hip/hip_runtime.h>
#include <stdio.h>

#define CHAINS 8
template <int OP>
__global__ __launch_bounds__(256) void k_op(uint32_t iters, uint32_t* out, unsigned long long* cyc) {
  uint32_t v[CHAINS];
  for (int c = 0; c < CHAINS; ++c) v[c] = threadIdx.x * (c + 3) + blockIdx.x;
  const uint32_t k = out[1] | 0x9E3779B1u;  // opaque constant
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (uint32_t i = 0; i < iters; ++i) {
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) {
      if (OP == 0) v[c] = v[c] * k;                                        // v_mul_lo_u32
      if (OP == 1) v[c] = (uint32_t)((uint64_t)v[c] * k + v[(c + 1) % CHAINS]);  // v_mad_u64_u32
      if (OP == 2) v[c] = __builtin_amdgcn_alignbit(v[c], v[c], 19);       // v_alignbit_b32
      if (OP == 3) v[c] = v[c] + k;                                        // v_add_u32
      if (OP == 4) v[c] = __builtin_amdgcn_alignbit(v[c] + v[(c+1)%CHAINS] * 0x85EBCA77u, v[c] + v[(c+1)%CHAINS] * 0x85EBCA77u, 19) * 0x9E3779B1u;  // xround
    }
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  uint32_t s = 0;
  for (int c = 0; c < CHAINS; ++c) s ^= v[c];
  if (s == 0x12345678u) out[0] = s;
  if (threadIdx.x == 0 && blockIdx.x == 0) cyc[0] = t1 - t0;
}

template <int OP>
static void run(const char* name, int per_iter_instr) {
  uint32_t* out;
  unsigned long long* cyc;
  (void)hipMalloc(&out, 64);
  (void)hipMalloc(&cyc, 8);
  (void)hipMemset(out, 0, 64);
  const uint32_t iters = 4096;
  const int grid = 256 * 8;  // 8 WGs x 4 waves per CU = 8 waves per SIMD
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  hipLaunchKernelGGL(k_op<OP>, dim3(grid), dim3(256), 0, 0, iters, out, cyc);
  (void)hipEventRecord(a);
  hipLaunchKernelGGL(k_op<OP>, dim3(grid), dim3(256), 0, 0, iters, out, cyc);
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, a, b);
  unsigned long long c = 0;
  (void)hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
  const double winstr = (double)grid * 4 * iters * CHAINS * per_iter_instr;  // wave-instructions
  const double per_simd = winstr / (256.0 * 4);
  printf("%-14s %8.3f ms  %6.2f ns per wave-instr per SIMD; wave0 cycles/iter %.1f\n", name, ms,
         ms * 1e6 / per_simd, (double)c / iters);
}

int main() {
  run<0>("v_mul_lo_u32", 1);
  run<1>("v_mad_u64_u32", 1);
  run<2>("v_alignbit", 1);
  run<3>("v_add_u32", 1);
  run<4>("xround", 4);
  return 0;
}
