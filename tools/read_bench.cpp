// Design microbenchmark (not part of the product): how fast can open() move data files from the
// page cache (/dev/shm) to the device? Compares, over NF files of 1 GiB:
//   dma   H2D from pinned buffers only (no file reads): the copy engines' ceiling
//   pread T threads pread into pinned 32-MiB buffers, no copy to the device
//   ring  pread + H2D, two pinned buffers per thread (engine.cpp's read_to_device)
//   reg   mmap each file, hipHostRegister it in pieces, H2D straight from the page cache (no CPU copy)
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/read_bench.cpp -o tools/read_bench
//   tools/read_bench [dir] [nfiles] [threads]
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#define CK(x)                                                                     \
  do {                                                                            \
    hipError_t e = (x);                                                           \
    if (e != hipSuccess) {                                                        \
      printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__);             \
      exit(1);                                                                    \
    }                                                                             \
  } while (0)

static double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static const size_t kFile = 1ull << 30, kPiece = 32ull << 20;

template <class F>
static void par(unsigned nt, F f) {
  std::vector<std::thread> th;
  for (unsigned t = 0; t < nt; ++t) th.emplace_back(f, t);
  for (auto& x : th) x.join();
}

int main(int argc, char** argv) {
  const std::string dir = argc > 1 ? argv[1] : "/dev/shm";
  const unsigned nf = argc > 2 ? (unsigned)atoi(argv[2]) : 16;
  const unsigned nt = argc > 3 ? (unsigned)atoi(argv[3]) : 16;
  std::vector<std::string> paths;
  {  // files of pseudo-random bytes
    std::vector<uint64_t> buf(kPiece / 8);
    for (unsigned f = 0; f < nf; ++f) {
      paths.push_back(dir + "/cask_readbench_" + std::to_string(f));
      const int fd = open(paths.back().c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0644);
      uint64_t x = 0x9E3779B97F4A7C15ull * (f + 1);
      for (size_t o = 0; o < kFile; o += kPiece) {
        for (auto& w : buf) {
          x += 0x9E3779B97F4A7C15ull;
          w = x ^ (x >> 29);
        }
        if (write(fd, buf.data(), kPiece) != (ssize_t)kPiece) { printf("write failed\n"); return 1; }
      }
      close(fd);
    }
  }
  const double gib = (double)nf * kFile / (1ull << 30);
  uint8_t* dev;
  CK(hipMalloc(&dev, nf * kFile));
  std::vector<void*> pin(2 * nt);
  for (auto& p : pin) CK(hipHostMalloc(&p, kPiece, hipHostMallocDefault));
  std::vector<hipStream_t> rs(nt);
  for (auto& s : rs) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  std::vector<hipEvent_t> ev(2 * nt);
  for (size_t i = 0; i < ev.size(); ++i) CK(hipEventCreateWithFlags(&ev[i], hipEventDisableTiming));
  const size_t npieces = nf * (kFile / kPiece);
  for (int rep = 0; rep < 2; ++rep) {
    double t0 = now();
    par(nt, [&](unsigned t) {  // dma
      CK(hipSetDevice(0));
      unsigned k = 0;
      for (size_t j = t; j < npieces; j += nt, k ^= 1)
        CK(hipMemcpyAsync(dev + j * kPiece, pin[2 * t + k], kPiece, hipMemcpyHostToDevice, rs[t]));
      CK(hipStreamSynchronize(rs[t]));
    });
    printf("rep %d dma   %6.2f GiB/s\n", rep, gib / (now() - t0));
    t0 = now();
    par(nt, [&](unsigned t) {  // pread only
      std::vector<int> fds(nf, -1);
      unsigned k = 0;
      for (size_t j = t; j < npieces; j += nt, k ^= 1) {
        const size_t f = j / (kFile / kPiece), off = (j % (kFile / kPiece)) * kPiece;
        if (fds[f] < 0) fds[f] = open(paths[f].c_str(), O_RDONLY);
        if (pread(fds[f], pin[2 * t + k], kPiece, (off_t)off) != (ssize_t)kPiece) printf("short read\n");
      }
      for (int fd : fds) if (fd >= 0) close(fd);
    });
    printf("rep %d pread %6.2f GiB/s\n", rep, gib / (now() - t0));
    t0 = now();
    par(nt, [&](unsigned t) {  // ring
      CK(hipSetDevice(0));
      std::vector<int> fds(nf, -1);
      unsigned k = 0;
      for (size_t j = t; j < npieces; j += nt, k ^= 1) {
        const size_t f = j / (kFile / kPiece), off = (j % (kFile / kPiece)) * kPiece;
        if (fds[f] < 0) fds[f] = open(paths[f].c_str(), O_RDONLY);
        CK(hipEventSynchronize(ev[2 * t + k]));
        if (pread(fds[f], pin[2 * t + k], kPiece, (off_t)off) != (ssize_t)kPiece) printf("short read\n");
        CK(hipMemcpyAsync(dev + j * kPiece, pin[2 * t + k], kPiece, hipMemcpyHostToDevice, rs[t]));
        CK(hipEventRecord(ev[2 * t + k], rs[t]));
      }
      CK(hipStreamSynchronize(rs[t]));
      for (int fd : fds) if (fd >= 0) close(fd);
    });
    printf("rep %d ring  %6.2f GiB/s\n", rep, gib / (now() - t0));
    t0 = now();
    double treg = 0;
    std::atomic<int> bad{0};
    par(nt, [&](unsigned t) {  // reg: map, register, copy, unregister
      CK(hipSetDevice(0));
      double tr = 0;
      for (size_t f = t; f < nf; f += nt) {
        const int fd = open(paths[f].c_str(), O_RDONLY);
        void* m = mmap(nullptr, kFile, PROT_READ, MAP_SHARED | MAP_POPULATE, fd, 0);
        close(fd);
        if (m == MAP_FAILED) { bad = 1; continue; }
        const double a = now();
        hipError_t e = hipHostRegister(m, kFile, hipHostRegisterReadOnly);
        tr += now() - a;
        if (e != hipSuccess) {
          if (!bad.exchange(1)) printf("hipHostRegister: %s\n", hipGetErrorString(e));
          munmap(m, kFile);
          continue;
        }
        void* dp = nullptr;
        CK(hipHostGetDevicePointer(&dp, m, 0));
        CK(hipMemcpyAsync(dev + f * kFile, m, kFile, hipMemcpyHostToDevice, rs[t]));
        CK(hipStreamSynchronize(rs[t]));
        CK(hipHostUnregister(m));
        munmap(m, kFile);
      }
      if (t == 0) treg = tr;
    });
    printf("rep %d reg   %6.2f GiB/s%s (thread 0 register time %.3f s)\n", rep, gib / (now() - t0),
           bad ? " (FAILED)" : "", treg);
    fflush(stdout);
  }
  {  // check the last copy (reg, or ring if reg failed) against the files
    std::vector<uint8_t> h(kPiece), d(kPiece);
    int fd = open(paths[nf - 1].c_str(), O_RDONLY);
    if (pread(fd, h.data(), kPiece, (off_t)(kFile - kPiece)) != (ssize_t)kPiece) printf("short read\n");
    close(fd);
    CK(hipMemcpy(d.data(), dev + (nf - 1) * kFile + kFile - kPiece, kPiece, hipMemcpyDeviceToHost));
    printf("device copy %s\n", memcmp(h.data(), d.data(), kPiece) ? "DIFFERS" : "matches");
  }
  for (auto& p : paths) unlink(p.c_str());
  return 0;
}
