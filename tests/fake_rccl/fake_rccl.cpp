// Test double of librccl (never shipped; loaded only under CASK_TEST_HOOKS=1 through CASK_RCCL_LIB):
// the RCCL entry points rccl_gather.cpp uses, for ranks that are threads of one process sharing
// one GPU. It lets tests/test_rccl_ranks_gpu.py drive the multi-rank control flow of
// cask_keydir_gather_rccl / cask_keydir_exchange_rccl — the status agreements, the early-error
// paths, a rank that fails between collectives — without a second GPU.
//
// Semantics follow NCCL's: a communicator per rank from one unique id (init blocks until every rank
// has joined); AllGather / AllReduce are collective (every rank must call them, in the same order);
// Send / Recv pair up per (source, destination) in issue order, and inside GroupStart / GroupEnd they
// run together at GroupEnd. Data moves with hipMemcpy between the ranks' device buffers after each
// caller's stream is synchronized (the caller's preceding async copies are then complete).
//
// A rank that never reaches a collective its peers wait in is the bug these tests look for: every
// wait gives up after CASK_FAKE_RCCL_TIMEOUT seconds (default 20) with ncclSystemError, so the
// test sees a status instead of hanging.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

namespace {

std::chrono::milliseconds wait_limit() {
  const char* e = getenv("CASK_FAKE_RCCL_TIMEOUT");
  return std::chrono::milliseconds((long long)((e ? atof(e) : 20.0) * 1000));
}

struct Msg {  // one posted send
  const void* buf;
  size_t bytes;
  bool done = false;
};

struct World {
  int nranks = 0;
  int joined = 0;
  int destroyed = 0;
  std::mutex mu;
  std::condition_variable cv;
  // collective rendezvous: a generation counter and per-rank slots
  uint64_t gen = 0;
  int arrived = 0;
  std::vector<const void*> slot;
  std::vector<std::vector<uint8_t>> hslot;
  bool broken = false;  // a rank timed out: every later wait fails at once
  // point-to-point: FIFO of sends per (src, dst)
  std::map<std::pair<int, int>, std::deque<std::shared_ptr<Msg>>> box;
};

std::mutex g_mu;
std::map<std::string, std::shared_ptr<World>> g_worlds;
std::atomic<uint64_t> g_ids{1};

struct FakeComm {
  std::shared_ptr<World> w;
  int rank;
};

// All ranks meet (called with the world's lock held): true once every rank has arrived, false when
// a rank timed out waiting here or anywhere else in this world.
bool barrier(World& W, std::unique_lock<std::mutex>& lk) {
  if (W.broken) return false;
  const uint64_t g = W.gen;
  if (++W.arrived == W.nranks) {
    W.arrived = 0;
    ++W.gen;
    W.cv.notify_all();
    return true;
  }
  if (!W.cv.wait_for(lk, wait_limit(), [&] { return W.gen != g || W.broken; }) || W.broken) {
    W.broken = true;
    W.cv.notify_all();
    return false;
  }
  return true;
}

size_t type_size(ncclDataType_t t) {
  switch (t) {
    case ncclInt8:
    case ncclUint8:
      return 1;
    case ncclInt32:
    case ncclUint32:
      return 4;
    case ncclInt64:
    case ncclUint64:
      return 8;
    default:
      return 0;
  }
}

template <class T>
void reduce_into(T* acc, const T* v, size_t n, ncclRedOp_t op) {
  for (size_t i = 0; i < n; ++i) {
    if (op == ncclMin) acc[i] = std::min(acc[i], v[i]);
    else if (op == ncclMax) acc[i] = std::max(acc[i], v[i]);
    else acc[i] = (T)(acc[i] + v[i]);
  }
}

// Thread-local group state: ops queued between GroupStart and GroupEnd.
struct P2p {
  bool send;
  void* buf;
  size_t bytes;
  int peer;
  FakeComm* comm;
  hipStream_t stream;
};
thread_local int t_depth = 0;
thread_local std::vector<P2p> t_ops;

ncclResult_t run_p2p(std::vector<P2p>& ops) {
  for (auto& o : ops)
    if (hipStreamSynchronize(o.stream) != hipSuccess) return ncclUnhandledCudaError;
  // post every send, then serve every receive in order, then wait for this rank's sends to be taken
  std::vector<std::pair<World*, std::shared_ptr<Msg>>> mine;
  for (auto& o : ops) {
    if (!o.send) continue;
    World& W = *o.comm->w;
    std::lock_guard<std::mutex> lk(W.mu);
    auto m = std::make_shared<Msg>();
    m->buf = o.buf;
    m->bytes = o.bytes;
    W.box[{o.comm->rank, o.peer}].push_back(m);
    mine.push_back({&W, m});
    W.cv.notify_all();
  }
  for (auto& o : ops) {
    if (o.send) continue;
    World& W = *o.comm->w;
    std::unique_lock<std::mutex> lk(W.mu);
    auto& q = W.box[{o.peer, o.comm->rank}];
    if (!W.cv.wait_for(lk, wait_limit(), [&] { return !q.empty() || W.broken; }) || W.broken) {
      W.broken = true;
      W.cv.notify_all();
      return ncclSystemError;
    }
    auto m = q.front();
    q.pop_front();
    if (m->bytes != o.bytes) {
      W.broken = true;
      W.cv.notify_all();
      return ncclInvalidUsage;
    }
    lk.unlock();
    const bool ok = !o.bytes || hipMemcpy(o.buf, m->buf, o.bytes, hipMemcpyDeviceToDevice) == hipSuccess;
    lk.lock();
    m->done = true;
    W.cv.notify_all();
    if (!ok) return ncclUnhandledCudaError;
  }
  for (auto& pm : mine) {
    World& W = *pm.first;
    const std::shared_ptr<Msg>& m = pm.second;
    std::unique_lock<std::mutex> lk(W.mu);
    if (!W.cv.wait_for(lk, wait_limit(), [&] { return m->done || W.broken; }) || !m->done) {
      W.broken = true;
      W.cv.notify_all();
      return ncclSystemError;
    }
  }
  return ncclSuccess;
}

}  // namespace

extern "C" {

ncclResult_t ncclGetUniqueId(ncclUniqueId* id) {
  memset(id, 0, sizeof(*id));
  const std::string s = "fake-rccl-" + std::to_string(g_ids.fetch_add(1)) + "-" +
                        std::to_string((unsigned long long)std::chrono::steady_clock::now().time_since_epoch().count());
  memcpy(id->internal, s.data(), std::min(s.size(), sizeof(id->internal) - 1));
  return ncclSuccess;
}

ncclResult_t ncclCommInitRank(ncclComm_t* comm, int nranks, ncclUniqueId id, int rank) {
  if (!comm || nranks < 1 || rank < 0 || rank >= nranks) return ncclInvalidArgument;
  const std::string key(id.internal, strnlen(id.internal, sizeof(id.internal)));
  std::shared_ptr<World> w;
  {
    std::lock_guard<std::mutex> g(g_mu);
    auto& slot = g_worlds[key];
    if (!slot) {
      slot = std::make_shared<World>();
      slot->nranks = nranks;
      slot->slot.assign(nranks, nullptr);
      slot->hslot.assign(nranks, {});
    }
    w = slot;
  }
  if (w->nranks != nranks) return ncclInvalidUsage;
  std::unique_lock<std::mutex> lk(w->mu);
  ++w->joined;
  w->cv.notify_all();
  if (!w->cv.wait_for(lk, wait_limit(), [&] { return w->joined == w->nranks; })) return ncclSystemError;
  *comm = (ncclComm_t) new FakeComm{w, rank};
  return ncclSuccess;
}

ncclResult_t ncclCommDestroy(ncclComm_t comm) {
  FakeComm* c = (FakeComm*)comm;
  if (!c) return ncclInvalidArgument;
  {
    std::lock_guard<std::mutex> lk(c->w->mu);
    ++c->w->destroyed;
  }
  delete c;
  return ncclSuccess;
}

ncclResult_t ncclCommCount(const ncclComm_t comm, int* count) {
  *count = ((FakeComm*)comm)->w->nranks;
  return ncclSuccess;
}

ncclResult_t ncclCommUserRank(const ncclComm_t comm, int* rank) {
  *rank = ((FakeComm*)comm)->rank;
  return ncclSuccess;
}

ncclResult_t ncclAllGather(const void* send, void* recv, size_t count, ncclDataType_t dt, ncclComm_t comm,
                           hipStream_t stream) {
  FakeComm* c = (FakeComm*)comm;
  World& W = *c->w;
  const size_t b = count * type_size(dt);
  if (hipStreamSynchronize(stream) != hipSuccess) return ncclUnhandledCudaError;
  std::unique_lock<std::mutex> lk(W.mu);
  W.slot[c->rank] = send;
  if (!barrier(W, lk)) return ncclSystemError;
  std::vector<const void*> src = W.slot;
  lk.unlock();
  bool ok = true;
  for (int r = 0; r < W.nranks; ++r)
    ok = ok && (!b || hipMemcpy((uint8_t*)recv + r * b, src[r], b, hipMemcpyDeviceToDevice) == hipSuccess);
  lk.lock();
  if (!barrier(W, lk)) return ncclSystemError;  // every rank has read every send buffer
  return ok ? ncclSuccess : ncclUnhandledCudaError;
}

ncclResult_t ncclAllReduce(const void* send, void* recv, size_t count, ncclDataType_t dt, ncclRedOp_t op,
                           ncclComm_t comm, hipStream_t stream) {
  FakeComm* c = (FakeComm*)comm;
  World& W = *c->w;
  const size_t b = count * type_size(dt);
  if (!b && count) return ncclInvalidArgument;
  if (hipStreamSynchronize(stream) != hipSuccess) return ncclUnhandledCudaError;
  std::vector<uint8_t> mine(b);
  if (b && hipMemcpy(mine.data(), send, b, hipMemcpyDeviceToHost) != hipSuccess) return ncclUnhandledCudaError;
  std::unique_lock<std::mutex> lk(W.mu);
  W.hslot[c->rank] = std::move(mine);
  if (!barrier(W, lk)) return ncclSystemError;
  std::vector<uint8_t> acc = W.hslot[0];
  for (int r = 1; r < W.nranks; ++r) {
    const uint8_t* v = W.hslot[r].data();
    switch (dt) {
      case ncclInt32: reduce_into((int32_t*)acc.data(), (const int32_t*)v, count, op); break;
      case ncclUint32: reduce_into((uint32_t*)acc.data(), (const uint32_t*)v, count, op); break;
      case ncclInt64: reduce_into((int64_t*)acc.data(), (const int64_t*)v, count, op); break;
      case ncclUint64: reduce_into((uint64_t*)acc.data(), (const uint64_t*)v, count, op); break;
      default: reduce_into((uint8_t*)acc.data(), v, b, op); break;
    }
  }
  if (!barrier(W, lk)) return ncclSystemError;  // every rank has read every contribution
  lk.unlock();
  return !b || hipMemcpy(recv, acc.data(), b, hipMemcpyHostToDevice) == hipSuccess ? ncclSuccess : ncclUnhandledCudaError;
}

ncclResult_t ncclGroupStart() {
  ++t_depth;
  return ncclSuccess;
}

ncclResult_t ncclGroupEnd() {
  if (t_depth <= 0) return ncclInvalidUsage;
  if (--t_depth) return ncclSuccess;
  std::vector<P2p> ops;
  ops.swap(t_ops);
  return run_p2p(ops);
}

ncclResult_t ncclSend(const void* buf, size_t count, ncclDataType_t dt, int peer, ncclComm_t comm, hipStream_t stream) {
  P2p o{true, const_cast<void*>(buf), count * type_size(dt), peer, (FakeComm*)comm, stream};
  if (t_depth) {
    t_ops.push_back(o);
    return ncclSuccess;
  }
  std::vector<P2p> one{o};
  return run_p2p(one);
}

ncclResult_t ncclRecv(void* buf, size_t count, ncclDataType_t dt, int peer, ncclComm_t comm, hipStream_t stream) {
  P2p o{false, buf, count * type_size(dt), peer, (FakeComm*)comm, stream};
  if (t_depth) {
    t_ops.push_back(o);
    return ncclSuccess;
  }
  std::vector<P2p> one{o};
  return run_p2p(one);
}

}  // extern "C"
