// The measured read-only stream ceiling of the GPU over the bench's own resident files (SURVEY.md
// §8d: "also report a measured read-only stream ceiling"): every byte of the buffers read once per
// pass, XOR-folded, nothing written but one word per workgroup. A measurement utility for bench.py,
// built as its own library (libcask_stream.so), not part of the scan library.
//
//   int cask_stream_read(const void* const* bufs, const uint64_t* lens, uint32_t n, uint32_t passes,
//                        int nontemporal, int device, double* gbps, double* ms_per_pass)
//
// One launch per pass over all the buffers (at most kMax): the 32-KiB tiles of every buffer in
// order, a tile per workgroup turn (256 lanes x 8 loads of 16 B in flight), tiles dealt round-robin to
// a grid of 8 workgroups per CU. Lengths are rounded down to 16 B (the tail is not read). Returns 0,
// or the HIP error code.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
constexpr uint32_t kMax = 64, kLoads = 8, kTile = 256 * kLoads;  // tile in 16-B granules (32 KiB)

struct Bufs {
  const u32x4* p[kMax];
  uint64_t first_tile[kMax + 1];  // prefix of the buffers' tile counts
  uint64_t n16[kMax];
  uint32_t n;
};

template <bool NT>
__global__ __launch_bounds__(256) void k_stream_read(Bufs b, uint32_t* sink) {
  const uint64_t ntiles = b.first_tile[b.n];
  u32x4 acc = u32x4{0u, 0u, 0u, 0u};
  uint32_t f = 0;
  for (uint64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    while (t >= b.first_tile[f + 1]) ++f;  // (tiles only move forward)
    const u32x4* p = b.p[f];
    const uint64_t g0 = (t - b.first_tile[f]) * kTile + threadIdx.x, n16 = b.n16[f];
    u32x4 v[kLoads];
#pragma unroll
    for (uint32_t k = 0; k < kLoads; ++k) {
      const uint64_t g = g0 + 256ull * k;
      const u32x4* a = p + (g < n16 ? g : n16 - 1);
      v[k] = NT ? __builtin_nontemporal_load(a) : *a;
    }
#pragma unroll
    for (uint32_t k = 0; k < kLoads; ++k) acc ^= v[k];
  }
  const uint32_t x = acc.x ^ acc.y ^ acc.z ^ acc.w;
  if (x == 0x9E3779B9u) sink[blockIdx.x] = x;  // (keeps the loads; almost never stores)
}
}  // namespace

extern "C" int cask_stream_read(const void* const* bufs, const uint64_t* lens, uint32_t n, uint32_t passes, int nontemporal,
                                int device, double* gbps, double* ms_per_pass) {
  if (!bufs || !lens || !n || n > kMax || !passes) return (int)hipErrorInvalidValue;
  hipError_t e = hipSetDevice(device);
  if (e != hipSuccess) return (int)e;
  Bufs b{};
  b.n = n;
  uint64_t bytes = 0;
  for (uint32_t i = 0; i < n; ++i) {
    b.p[i] = (const u32x4*)bufs[i];
    b.n16[i] = lens[i] / 16;
    b.first_tile[i + 1] = b.first_tile[i] + (b.n16[i] + kTile - 1) / kTile;
    bytes += b.n16[i] * 16;
  }
  int cus = 0;
  if ((e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device)) != hipSuccess) return (int)e;
  const uint32_t grid = 8u * (uint32_t)(cus > 0 ? cus : 256);
  uint32_t* sink = nullptr;
  hipStream_t s = nullptr;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  float ms = 0.f;
  auto launch = [&]() {
    if (nontemporal)
      k_stream_read<true><<<grid, 256, 0, s>>>(b, sink);
    else
      k_stream_read<false><<<grid, 256, 0, s>>>(b, sink);
    return hipGetLastError();
  };
  if ((e = hipMalloc(&sink, 4ull * grid)) != hipSuccess) return (int)e;
  if ((e = hipStreamCreateWithFlags(&s, hipStreamNonBlocking)) == hipSuccess &&
      (e = hipEventCreate(&e0)) == hipSuccess && (e = hipEventCreate(&e1)) == hipSuccess &&
      (e = launch()) == hipSuccess &&  // (warm-up pass)
      (e = hipEventRecord(e0, s)) == hipSuccess) {
    for (uint32_t i = 0; i < passes && e == hipSuccess; ++i) e = launch();
    if (e == hipSuccess) e = hipEventRecord(e1, s);
    if (e == hipSuccess) e = hipEventSynchronize(e1);
    if (e == hipSuccess) e = hipEventElapsedTime(&ms, e0, e1);
  }
  if (s) (void)hipStreamSynchronize(s);
  if (e1) (void)hipEventDestroy(e1);
  if (e0) (void)hipEventDestroy(e0);
  if (s) (void)hipStreamDestroy(s);
  (void)hipFree(sink);
  if (e != hipSuccess) return (int)e;
  const double per = (double)ms / passes;
  if (ms_per_pass) *ms_per_pass = per;
  if (gbps) *gbps = per > 0 ? (double)bytes / (per * 1e-3) / 1e9 : 0.0;
  return 0;
}
