// Batched record encoder (Entry::write_bytes, data.rs:90-121): the bulk write path and the
// generator of the synthetic benchmark workloads. Pass 1 writes header tail + key + value bytes
// (one lane per record), pass 2 hashes [off+4, off+len) and stores the XXH32 at off.
#include "device_util.h"

namespace cask_dev {

__device__ __forceinline__ uint64_t splitmix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__device__ __forceinline__ void put_hdr_tail(uint8_t* o, uint64_t seq, uint16_t ksz, uint32_t vsz) {
  for (int i = 0; i < 8; ++i) o[4 + i] = (uint8_t)(seq >> (8 * i));
  o[12] = (uint8_t)ksz;
  o[13] = (uint8_t)(ksz >> 8);
  for (int i = 0; i < 4; ++i) o[14 + i] = (uint8_t)(vsz >> (8 * i));
}

__global__ __launch_bounds__(256) void k_encode_synth(uint64_t nrec, const uint64_t* off,
                                                      const uint64_t* seq, const uint16_t* ksz,
                                                      const uint32_t* vsz_raw, const uint64_t* key_id,
                                                      uint64_t value_seed, uint8_t* out) {
  for (uint64_t r = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; r < nrec;
       r += (uint64_t)gridDim.x * blockDim.x) {
    uint8_t* o = out + off[r];
    const uint16_t k = ksz[r];
    const uint32_t v = vsz_raw[r];
    put_hdr_tail(o, seq[r], k, v);
    const uint64_t kid = key_id[r];
    for (uint32_t j = 0; j < k; j += 8) {
      uint64_t wv = splitmix64((kid << 16) | (j >> 3));
      for (uint32_t b = 0; b < 8 && j + b < k; ++b) o[18 + j + b] = (uint8_t)(wv >> (8 * b));
    }
    if (v != 0xFFFFFFFFu) {
      const uint64_t rs = splitmix64(value_seed + r);
      uint8_t* vo = o + 18 + k;
      for (uint32_t j = 0; j < v; j += 8) {
        uint64_t wv = splitmix64(rs + (j >> 3));
        for (uint32_t b = 0; b < 8 && j + b < v; ++b) vo[j + b] = (uint8_t)(wv >> (8 * b));
      }
    }
  }
}

__global__ __launch_bounds__(256) void k_encode(uint64_t nrec, const uint64_t* off, const uint64_t* seq,
                                                const uint16_t* ksz, const uint32_t* vsz_raw,
                                                const uint8_t* keys, const uint64_t* key_off,
                                                const uint8_t* vals, const uint64_t* val_off,
                                                uint8_t* out) {
  for (uint64_t r = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; r < nrec;
       r += (uint64_t)gridDim.x * blockDim.x) {
    uint8_t* o = out + off[r];
    const uint16_t k = ksz[r];
    const uint32_t v = vsz_raw[r];
    put_hdr_tail(o, seq[r], k, v);
    const uint8_t* ks = keys + key_off[r];
    for (uint32_t j = 0; j < k; ++j) o[18 + j] = ks[j];
    if (v != 0xFFFFFFFFu) {
      const uint8_t* vs = vals + val_off[r];
      for (uint32_t j = 0; j < v; ++j) o[18 + k + j] = vs[j];
    }
  }
}

__global__ __launch_bounds__(256) void k_encode_checksum(uint64_t nrec, const uint64_t* off,
                                                         const uint16_t* ksz, const uint32_t* vsz_raw,
                                                         uint8_t* out) {
  for (uint64_t r = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; r < nrec;
       r += (uint64_t)gridDim.x * blockDim.x) {
    uint8_t* o = out + off[r];
    const uint32_t v = vsz_raw[r];
    const uint64_t rl = 18ull + ksz[r] + ((v == 0xFFFFFFFFu) ? 0ull : (uint64_t)v);
    const uint32_t h = gbl_xxh32(o + 4, rl - 4);
    o[0] = (uint8_t)h;
    o[1] = (uint8_t)(h >> 8);
    o[2] = (uint8_t)(h >> 16);
    o[3] = (uint8_t)(h >> 24);
  }
}

static inline hipStream_t S(void* s) { return (hipStream_t)s; }
static inline uint32_t grid_for(uint64_t n) {
  uint64_t g = (n + 255) / 256;
  if (g > 65536) g = 65536;
  return g ? (uint32_t)g : 1u;
}
void launch_encode_synth(uint64_t nrec, const uint64_t* off, const uint64_t* seq, const uint16_t* ksz,
                         const uint32_t* vsz_raw, const uint64_t* key_id, uint64_t value_seed,
                         uint8_t* out, void* stream) {
  if (!nrec) return;
  hipLaunchKernelGGL(k_encode_synth, dim3(grid_for(nrec)), dim3(256), 0, S(stream), nrec, off, seq, ksz,
                     vsz_raw, key_id, value_seed, out);
}
void launch_encode(uint64_t nrec, const uint64_t* off, const uint64_t* seq, const uint16_t* ksz,
                   const uint32_t* vsz_raw, const uint8_t* keys, const uint64_t* key_off,
                   const uint8_t* vals, const uint64_t* val_off, uint8_t* out, void* stream) {
  if (!nrec) return;
  hipLaunchKernelGGL(k_encode, dim3(grid_for(nrec)), dim3(256), 0, S(stream), nrec, off, seq, ksz, vsz_raw,
                     keys, key_off, vals, val_off, out);
}
void launch_encode_checksum(uint64_t nrec, const uint64_t* off, const uint16_t* ksz, const uint32_t* vsz_raw,
                            uint8_t* out, void* stream) {
  if (!nrec) return;
  hipLaunchKernelGGL(k_encode_checksum, dim3(grid_for(nrec)), dim3(256), 0, S(stream), nrec, off, ksz,
                     vsz_raw, out);
}

}  // namespace cask_dev
