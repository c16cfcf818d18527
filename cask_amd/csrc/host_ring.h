// Host-side helpers shared by the engine (engine.cpp) and the runtime (scan_runtime.cpp): the host
// thread count, a fork/join over threads, and a ring of pinned staging buffers that moves pageable
// host memory to and from the device on several threads at once (a copy between pageable memory
// and the device goes through the driver's own staging at ~10-25 GB/s).
#pragma once
#include <hip/hip_runtime.h>
#include <sched.h>
#include <sys/mman.h>

#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <thread>
#include <vector>
#include "knobs.h"

namespace cask_host {

// The CPUs this process may run on (sched_getaffinity, so cgroup/affinity limits count), at most
// 16. CASK_HOST_THREADS (test and tuning knob) sets the count, e.g. to force the threaded paths on a
// one-CPU machine.
inline unsigned host_threads() {
  if (const char* e = cask_knobs::hook("CASK_HOST_THREADS")) {
    const int v = atoi(e);
    if (v > 0) return (unsigned)std::min(v, 64);
  }
  unsigned k = 0;
  cpu_set_t set;
  CPU_ZERO(&set);
  if (sched_getaffinity(0, sizeof(set), &set) == 0) k = (unsigned)CPU_COUNT(&set);
  if (!k) k = std::thread::hardware_concurrency();
  return std::max(1u, std::min(k, 16u));
}

// fn(t) for t in [0, nt): t = 1.. on threads of their own, t = 0 on the caller. A thread that cannot
// be created (std::system_error) has its share run on the calling thread, so the result does not
// depend on how many threads actually ran. An exception thrown by any share (std::bad_alloc under
// memory pressure) is caught on its thread and the first one is rethrown here once every thread
// has been joined: it reaches the entry point's own handler (engine.cpp: abi_status / abi_db) instead of
// std::terminate, and no thread is left running over the caller's state.
template <class F>
void parallel_for(unsigned nt, F fn) {
  if (!nt) nt = 1;
  // (everything that allocates happens before the first thread starts: an exception from here on
  // would unwind past running threads)
  std::vector<std::exception_ptr> ex(nt);
  std::vector<char> spawned(nt, 0);
  std::vector<std::thread> th;
  th.reserve(nt);
  auto run = [&](unsigned t) {
    try {
      fn(t);
    } catch (...) {
      ex[t] = std::current_exception();
    }
  };
  for (unsigned t = 1; t < nt; ++t) {
    try {
      th.emplace_back(run, t);
      spawned[t] = 1;
    } catch (...) {
    }
  }
  run(0u);
  for (unsigned t = 1; t < nt; ++t)
    if (!spawned[t]) run(t);
  for (auto& x : th) x.join();
  for (auto& e : ex)
    if (e) std::rethrow_exception(e);
}

// Page-locked host memory the device can DMA to and from: an anonymous mapping populated when it is
// made (huge pages where the kernel has them) and then registered. hipHostMalloc's memory is
// mapped into the process lazily instead: the first host write to each 4-KiB page faults, which
// cost the first open() of a process ~1 s per GiB of staging (tools/read_bench.cpp).
inline void* pinned_alloc(size_t n) {
  void* p = mmap(nullptr, n, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
  if (p == MAP_FAILED) return nullptr;
  (void)madvise(p, n, MADV_HUGEPAGE);
  memset(p, 0, n);  // (populated now, on huge pages if any: MAP_POPULATE would fault in 4-KiB pages first)
  if (hipHostRegister(p, n, hipHostRegisterDefault) != hipSuccess) {
    munmap(p, n);
    return nullptr;
  }
  return p;
}
inline void pinned_free(void* p, size_t n) {
  (void)hipHostUnregister(p);
  munmap(p, n);
}

// kThreads x 2 pinned buffers of kBytes, a stream per thread, an event per buffer. Thread t takes
// every nt-th piece and alternates between its two buffers, so the DMA of one piece overlaps the
// host copy of the next (host -> device) or of the previous one (device -> host).
struct PinnedRing {
  static constexpr int kThreads = 16, kSlots = 2;
  static constexpr size_t kBytes = 32ull << 20;
  int device = -1;
  int nthr = kThreads;  // threads (and slot pairs) this ring was made with
  void* pin[kThreads][kSlots] = {};
  hipStream_t rs[kThreads] = {};
  hipEvent_t ev[kThreads][kSlots] = {};

  struct Piece {  // at most kBytes
    uint8_t* host;
    uint8_t* dev;
    uint64_t n;
  };
  static void split(uint8_t* host, uint8_t* dev, uint64_t n, std::vector<Piece>& out) {
    for (uint64_t o = 0; o < n; o += kBytes) out.push_back(Piece{host + o, dev + o, std::min<uint64_t>(kBytes, n - o)});
  }

  PinnedRing() = default;
  PinnedRing(const PinnedRing&) = delete;
  PinnedRing& operator=(const PinnedRing&) = delete;
  ~PinnedRing() { release(); }

  // Allocates what is missing (on `dev`) for `threads` threads; false on failure (what was made stays
  // for release()).
  bool init(int dev, int threads = kThreads) {
    device = dev;
    nthr = std::max(1, std::min(threads, kThreads));
    if (hipSetDevice(dev) != hipSuccess) return false;
    for (int t = 0; t < nthr; ++t) {
      if (!rs[t] && hipStreamCreateWithFlags(&rs[t], hipStreamNonBlocking) != hipSuccess) return false;
      for (int k = 0; k < kSlots; ++k) {
        if (!pin[t][k] && !(pin[t][k] = pinned_alloc(kBytes))) return false;
        if (!ev[t][k] && hipEventCreateWithFlags(&ev[t][k], hipEventDisableTiming) != hipSuccess) return false;
      }
    }
    return true;
  }
  void release() {
    if (device >= 0) (void)hipSetDevice(device);
    for (int t = 0; t < kThreads; ++t) {
      if (rs[t]) (void)hipStreamSynchronize(rs[t]);
      for (int k = 0; k < kSlots; ++k) {
        if (pin[t][k]) pinned_free(pin[t][k], kBytes);
        if (ev[t][k]) (void)hipEventDestroy(ev[t][k]);
        pin[t][k] = nullptr;
        ev[t][k] = nullptr;
      }
      if (rs[t]) (void)hipStreamDestroy(rs[t]);
      rs[t] = nullptr;
    }
  }

  // host (pageable) -> device. Returns false on a device error. The caller orders later device work
  // after it (every stream here is synchronised before returning).
  bool h2d(const std::vector<Piece>& ps) {
    const unsigned nt = threads_for(ps.size());
    std::vector<char> ok(nt, 1);
    parallel_for(nt, [&](unsigned t) {
      if (hipSetDevice(device) != hipSuccess) {
        ok[t] = 0;
        return;
      }
      unsigned k = 0;
      for (size_t j = t; j < ps.size(); j += nt, k ^= 1) {
        if (hipEventSynchronize(ev[t][k]) != hipSuccess) {  // the buffer's last DMA is done
          ok[t] = 0;
          break;
        }
        memcpy(pin[t][k], ps[j].host, ps[j].n);
        if (hipMemcpyAsync(ps[j].dev, pin[t][k], ps[j].n, hipMemcpyHostToDevice, rs[t]) != hipSuccess ||
            hipEventRecord(ev[t][k], rs[t]) != hipSuccess) {
          ok[t] = 0;
          break;
        }
      }
      if (hipStreamSynchronize(rs[t]) != hipSuccess) ok[t] = 0;
    });
    return std::all_of(ok.begin(), ok.end(), [](char c) { return c != 0; });
  }

  // device -> host (pageable). The device work that produced the bytes must be complete.
  bool d2h(const std::vector<Piece>& ps) {
    const unsigned nt = threads_for(ps.size());
    std::vector<char> ok(nt, 1);
    parallel_for(nt, [&](unsigned t) {
      if (hipSetDevice(device) != hipSuccess) {
        ok[t] = 0;
        return;
      }
      size_t prev = SIZE_MAX;
      unsigned k = 0, pk = 0;
      for (size_t j = t;; j += nt, k ^= 1) {
        bool have = j < ps.size();
        if (have && (hipMemcpyAsync(pin[t][k], ps[j].dev, ps[j].n, hipMemcpyDeviceToHost, rs[t]) != hipSuccess ||
                     hipEventRecord(ev[t][k], rs[t]) != hipSuccess)) {
          ok[t] = 0;
          have = false;
        }
        if (prev != SIZE_MAX) {  // the previous piece, out of the other buffer, while this one moves
          if (hipEventSynchronize(ev[t][pk]) != hipSuccess) {
            ok[t] = 0;
            break;
          }
          memcpy(ps[prev].host, pin[t][pk], ps[prev].n);
        }
        if (!have) break;
        prev = j;
        pk = k;
      }
      if (hipStreamSynchronize(rs[t]) != hipSuccess) ok[t] = 0;
    });
    return std::all_of(ok.begin(), ok.end(), [](char c) { return c != 0; });
  }

 private:
  unsigned threads_for(size_t pieces) const {
    return std::max(1u, std::min<unsigned>((unsigned)nthr, std::min<unsigned>(host_threads(), (unsigned)pieces)));
  }
};

}  // namespace cask_host
