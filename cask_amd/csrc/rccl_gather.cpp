// RCCL over xGMI for the multi-GPU replay, behind the C ABI so that a host in any
// language (the reference's Rust Cask::open, cask.rs:346-382) can move the shards' keydir blocks
// without torch. A communicator from a unique id the caller distributes, then either
//  * cask_keydir_gather_rccl: one rooted gather of variable-size device blocks — sizes by
//    ncclAllGather, the blocks by grouped ncclSend/ncclRecv (RCCL has no gatherv; one message per
//    rank, each on its own xGMI link into the root) — folded on the root in rank order
//    (cask_keydir_merge: rank order is replay order, the shards being contiguous file-id ranges); or
//  * cask_keydir_exchange_rccl: the key-hash all-to-all for a keyspace too large for one host
//    (cfg5's ~45 GB of blocks): every block split by key owner on its device
//    (cask_keydir_partition), part o to rank o by grouped send/recv, each rank folding the parts it
//    owns in rank order, then Stats from every owner's per-file terms (one more all-gather).
// RCCL is loaded on first use (dlopen): the library itself needs no librccl to load, and a host
// without it gets CASK_E_DEVICE from these calls only. (Under CASK_TEST_HOOKS=1, CASK_RCCL_LIB names
// another library with RCCL's entry points: tests/fake_rccl, ranks as threads of one process.)
//
// Every rank issues the same sequence of collectives whatever it passes (a bad argument, a NULL
// max_seq, an empty block) and whatever fails on it between two collectives (an allocation, the
// partition, the fold): each such status is carried to the next agreement — an ncclAllReduce(min)
// of the ranks' statuses — before any data moves, so all ranks return the same status and none is
// left waiting in a send, receive or all-gather that a peer will never issue. Nothing allocates
// between an agreement and the collective it guards: the small all-gathers use device scratch made
// with the communicator, the large buffers are allocated before the agreement that covers them.
// Only a collective that itself fails (a broken communicator) returns without agreeing.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstring>
#include <map>
#include <mutex>
#include <new>
#include <string>
#include <type_traits>
#include <vector>

#include "../../include/cask_scan.h"
#include "abi_guard.h"
#include "keydir_format.h"
#include "knobs.h"

static_assert(CASK_RCCL_ID_BYTES == NCCL_UNIQUE_ID_BYTES, "unique id size");

namespace {

// The RCCL entry points this file uses, resolved from a library at first use.
struct Rccl {
  decltype(&ncclGetUniqueId) GetUniqueId = nullptr;
  decltype(&ncclCommInitRank) CommInitRank = nullptr;
  decltype(&ncclCommDestroy) CommDestroy = nullptr;
  decltype(&ncclCommCount) CommCount = nullptr;
  decltype(&ncclCommUserRank) CommUserRank = nullptr;
  decltype(&ncclAllGather) AllGather = nullptr;
  decltype(&ncclAllReduce) AllReduce = nullptr;
  decltype(&ncclSend) Send = nullptr;
  decltype(&ncclRecv) Recv = nullptr;
  decltype(&ncclGroupStart) GroupStart = nullptr;
  decltype(&ncclGroupEnd) GroupEnd = nullptr;
  bool ok = false;
};

const Rccl* load_rccl(const char* path) {
  Rccl* r = new (std::nothrow) Rccl();
  if (!r) return nullptr;
  void* h = path ? dlopen(path, RTLD_NOW | RTLD_LOCAL) : dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
  if (!h && !path) h = dlopen("librccl.so", RTLD_NOW | RTLD_LOCAL);
  if (!h) return r;
  bool all = true;
  auto sym = [&](auto& f, const char* name) {
    f = reinterpret_cast<std::remove_reference_t<decltype(f)>>(dlsym(h, name));
    all = all && f != nullptr;
  };
  sym(r->GetUniqueId, "ncclGetUniqueId");
  sym(r->CommInitRank, "ncclCommInitRank");
  sym(r->CommDestroy, "ncclCommDestroy");
  sym(r->CommCount, "ncclCommCount");
  sym(r->CommUserRank, "ncclCommUserRank");
  sym(r->AllGather, "ncclAllGather");
  sym(r->AllReduce, "ncclAllReduce");
  sym(r->Send, "ncclSend");
  sym(r->Recv, "ncclRecv");
  sym(r->GroupStart, "ncclGroupStart");
  sym(r->GroupEnd, "ncclGroupEnd");
  r->ok = all;
  return r;
}

// librccl, or the test hook's library; each loaded once and kept for the process.
const Rccl* rccl() {
  static std::mutex mu;
  static std::map<std::string, const Rccl*> loaded;
  const char* alt = cask_knobs::hook("CASK_RCCL_LIB");
  const std::string key = alt ? alt : "";
  std::lock_guard<std::mutex> g(mu);
  auto it = loaded.find(key);
  const Rccl* r = it != loaded.end() ? it->second : (loaded[key] = load_rccl(alt));
  return r && r->ok ? r : nullptr;
}

// What cask_rccl_comm_init hands out: the communicator, the library that made it, and device scratch
// for the small collectives (statuses, sizes) so that they never allocate between two agreements.
struct Comm {
  const Rccl* R = nullptr;
  ncclComm_t c = nullptr;
  int nranks = 0, rank = 0, device = 0;
  void* scratch = nullptr;
  uint64_t cap = 0;  // bytes of scratch
};

uint64_t scratch_bytes(int nranks) {  // the N x N size matrix, in and out, and the status words
  const uint64_t n = (uint64_t)nranks;
  return 8 * (n * n + 2 * n + 8) + 256;
}

struct DevMem {  // device memory of one call
  void* p = nullptr;
  ~DevMem() {
    if (p) (void)hipFree(p);
  }
};

// Every rank's `n` u64 values, in rank order, on every rank (ncclAllGather through device memory:
// the communicator's scratch, or `big` when the values do not fit it). A rank that has failed takes
// part all the same: with `mine` NULL it sends zeros, with `all` empty it keeps nothing. False when
// a collective or copy fails: the communicator is then unusable and the caller returns
// CASK_E_DEVICE.
bool allgather_u64(const Comm& K, hipStream_t st, const uint64_t* mine, uint64_t n, std::vector<uint64_t>& all,
                   void* big = nullptr) {
  const uint64_t need = 8ull * n * (K.nranks + 1);
  uint64_t* dm = (uint64_t*)(need <= K.cap ? K.scratch : big);
  if (!dm) return false;
  if (!n) return true;
  const bool in = mine ? hipMemcpyAsync(dm + n * K.nranks, mine, 8ull * n, hipMemcpyHostToDevice, st) == hipSuccess
                       : hipMemsetAsync(dm + n * K.nranks, 0, 8ull * n, st) == hipSuccess;
  return in && K.R->AllGather(dm + n * K.nranks, dm, n, ncclUint64, K.c, st) == ncclSuccess &&
         (all.size() < n * K.nranks ||
          hipMemcpyAsync(all.data(), dm, 8ull * n * K.nranks, hipMemcpyDeviceToHost, st) == hipSuccess) &&
         hipStreamSynchronize(st) == hipSuccess;
}

// The status every rank returns: the lowest (most severe) of the ranks' own statuses (0 = ok), by
// ncclAllReduce(min) in the communicator's scratch. A rank that fails between two collectives still
// calls this, so no peer is left waiting in a collective it will never match.
int agree(const Comm& K, hipStream_t st, int mine) {
  int32_t* dm = (int32_t*)K.scratch;
  int32_t v = mine, out = 0;
  if (hipMemcpyAsync(dm, &v, 4, hipMemcpyHostToDevice, st) != hipSuccess ||
      K.R->AllReduce(dm, dm + 1, 1, ncclInt32, ncclMin, K.c, st) != ncclSuccess ||
      hipMemcpyAsync(&out, dm + 1, 4, hipMemcpyDeviceToHost, st) != hipSuccess || hipStreamSynchronize(st) != hipSuccess)
    return CASK_E_DEVICE;
  return out;
}

// A host vector sized without throwing: false (and the vector empty) when the memory is not there.
template <class T>
bool host_alloc(std::vector<T>& v, uint64_t n) {
  try {
    v.assign(n, T{});
    return true;
  } catch (const std::bad_alloc&) {
    v.clear();
    return false;
  }
}

}  // namespace

extern "C" int cask_rccl_unique_id(uint8_t* id) {
  return cask_abi::guard([&]() -> int {
    if (!id) return CASK_E_INVALID_ARG;
    const Rccl* R = rccl();
    if (!R) return CASK_E_DEVICE;
    ncclUniqueId u;
    if (R->GetUniqueId(&u) != ncclSuccess) return CASK_E_DEVICE;
    memcpy(id, &u, sizeof(u));
    return CASK_OK;
  });
}

extern "C" int cask_rccl_comm_init(const uint8_t* id, int nranks, int rank, int device, void** comm) {
  return cask_abi::guard([&]() -> int {
    if (!id || !comm || nranks < 1 || rank < 0 || rank >= nranks) return CASK_E_INVALID_ARG;
    const Rccl* R = rccl();
    if (!R) return CASK_E_DEVICE;
    if (hipSetDevice(device) != hipSuccess) return CASK_E_DEVICE;
    Comm* K = new (std::nothrow) Comm();
    if (!K) return CASK_E_NOMEM;
    K->R = R;
    K->nranks = nranks;
    K->rank = rank;
    K->device = device;
    K->cap = scratch_bytes(nranks);
    // (the scratch first: a rank that cannot make it fails before joining, and the others' init
    // fails on the missing peer, as RCCL's own would)
    if (hipMalloc(&K->scratch, K->cap) != hipSuccess) {
      delete K;
      return CASK_E_NOMEM;
    }
    ncclUniqueId u;
    memcpy(&u, id, sizeof(u));
    if (R->CommInitRank(&K->c, nranks, u, rank) != ncclSuccess) {
      (void)hipFree(K->scratch);
      delete K;
      return CASK_E_DEVICE;
    }
    *comm = K;
    return CASK_OK;
  });
}

extern "C" int cask_rccl_comm_destroy(void* comm) {
  return cask_abi::guard([&]() -> int {
    if (!comm) return CASK_E_INVALID_ARG;
    Comm* K = (Comm*)comm;
    const int st = K->R->CommDestroy(K->c) == ncclSuccess ? CASK_OK : CASK_E_DEVICE;
    (void)hipSetDevice(K->device);
    (void)hipFree(K->scratch);
    delete K;
    return st;
  });
}

static int gather_impl(cask_ctx* ctx, Comm& K, const void* block, uint64_t bytes, int root, cask_db* db,
                       uint64_t* gathered, uint64_t* max_seq) {
  using namespace cask_kd;
  const int nranks = K.nranks, rank = K.rank;
  if (hipSetDevice(cask_ctx_device(ctx)) != hipSuccess) return CASK_E_DEVICE;
  hipStream_t st = (hipStream_t)cask_ctx_stream(ctx);
  // argument errors on any rank are agreed on below, like any other failure (a bad root: this rank
  // goes through the all-gather with root 0 in its place, then every rank stops at the agreement)
  int status = (bytes && !block) ? CASK_E_INVALID_ARG : CASK_OK;
  std::vector<uint64_t> all, off;
  if (!host_alloc(all, 3ull * nranks) || !host_alloc(off, (uint64_t)nranks + 1)) status = CASK_E_NOMEM;
  const uint64_t root_given = (uint64_t)(int64_t)root;  // (compared across the ranks below)
  if (root < 0 || root >= nranks) {
    status = CASK_E_INVALID_ARG;
    root = 0;
  }
  if (rank == root && !db) status = CASK_E_INVALID_ARG;
  // this rank's block header (its max sequence) from the device
  ShardHeader hd{};
  const bool has_hd = status == CASK_OK && bytes >= sizeof(hd);
  if (has_hd && (hipMemcpyAsync(&hd, block, sizeof(hd), hipMemcpyDeviceToHost, st) != hipSuccess ||
                 hipStreamSynchronize(st) != hipSuccess))
    status = CASK_E_DEVICE;
  // every rank's block size, max sequence + 1 and root (ncclAllGather of three u64 per rank): the
  // global maximum sequence is the largest of them on every rank, with no collective of its own; ranks
  // that name different roots would each post the root's receives, and the grouped send/recv would
  // never match — every rank sees the disagreement here and stops at the agreement instead
  const uint64_t mine[3] = {status == CASK_OK ? bytes : 0, has_hd ? hd.max_seq_p1 : 0, root_given};
  if (!allgather_u64(K, st, mine, 3, all)) return CASK_E_DEVICE;
  if (status == CASK_OK && !all.empty())
    for (int r = 0; r < nranks; ++r)
      if (all[3ull * r + 2] != root_given) status = CASK_E_INVALID_ARG;
  if (status == CASK_OK) {
    uint64_t mx = 0;
    for (int r = 0; r < nranks; ++r) mx = std::max(mx, all[3ull * r + 1]);
    if (max_seq) *max_seq = mx ? mx - 1 : 0;
    for (int r = 0; r < nranks; ++r) off[r + 1] = off[r] + ((all[3ull * r] + 255) & ~255ull);
    if (gathered) *gathered = rank == root ? off[nranks] : bytes;
  }
  // the root's receive and host buffers, then the agreed status: every rank goes on, or every one stops
  DevMem buf;
  std::vector<uint8_t> host;
  if (status == CASK_OK && rank == root &&
      (cask_abi::take_inject(ctx, cask_abi::kInjRootAlloc) || (off[nranks] && hipMalloc(&buf.p, off[nranks]) != hipSuccess) ||
       !host_alloc(host, off[nranks] ? off[nranks] : 1)))
    status = CASK_E_NOMEM;
  if ((status = agree(K, st, status)) != CASK_OK) return status;
  // the blocks to the root: one grouped send per rank, nranks - 1 receives on the root
  if (K.R->GroupStart() != ncclSuccess) return CASK_E_DEVICE;
  bool sent = true;
  if (rank == root) {
    for (int r = 0; r < nranks; ++r) {
      if (!all[3ull * r]) continue;
      uint8_t* dst = (uint8_t*)buf.p + off[r];
      if (r == root)
        sent = sent && hipMemcpyAsync(dst, block, bytes, hipMemcpyDeviceToDevice, st) == hipSuccess;
      else
        sent = sent && K.R->Recv(dst, all[3ull * r], ncclUint8, r, K.c, st) == ncclSuccess;
    }
  } else if (bytes) {
    sent = K.R->Send(block, bytes, ncclUint8, root, K.c, st) == ncclSuccess;
  }
  if (K.R->GroupEnd() != ncclSuccess || !sent || hipStreamSynchronize(st) != hipSuccess) return CASK_E_DEVICE;
  // the root's fold, in rank order (= replay order); its outcome is every rank's status
  int fst = CASK_OK;
  if (rank == root) {
    if (off[nranks] && hipMemcpy(host.data(), buf.p, off[nranks], hipMemcpyDeviceToHost) != hipSuccess) fst = CASK_E_DEVICE;
    if (fst == CASK_OK && cask_abi::take_inject(ctx, cask_abi::kInjFold)) fst = CASK_E_NOMEM;
    if (fst == CASK_OK) {  // (one pass over the ranks' blocks, in rank order)
      std::vector<const uint8_t*> bp;
      std::vector<uint64_t> bl;
      for (int r = 0; r < nranks; ++r)
        if (all[3ull * r]) {
          bp.push_back(host.data() + off[r]);
          bl.push_back(all[3ull * r]);
        }
      fst = cask_keydir_merge_many(db, bp.data(), bl.data(), (uint32_t)bp.size());
    }
  }
  return agree(K, st, fst);
}

extern "C" int cask_keydir_gather_rccl(cask_ctx* ctx, void* comm, const void* block, uint64_t bytes, int root,
                                       cask_db* db, uint64_t* gathered, uint64_t* max_seq) {
  return cask_abi::guard([&]() -> int {
    if (!ctx || !comm) return CASK_E_INVALID_ARG;  // (no communicator to agree over)
    return gather_impl(ctx, *(Comm*)comm, block, bytes, root, db, gathered, max_seq);
  });
}

static int exchange_impl(cask_ctx* ctx, Comm& K, const void* block, uint64_t bytes, cask_db* db, uint64_t* sent_bytes,
                         uint64_t* recv_bytes) {
  using namespace cask_kd;
  const int nranks = K.nranks, rank = K.rank;
  const uint64_t N = (uint64_t)nranks;
  if (hipSetDevice(cask_ctx_device(ctx)) != hipSuccess) return CASK_E_DEVICE;
  hipStream_t st = (hipStream_t)cask_ctx_stream(ctx);
  int status = (!db || (bytes && !block) || N > kMaxParts) ? CASK_E_INVALID_ARG : CASK_OK;
  std::vector<uint64_t> poff, mine, all, roff, counts;
  if (!host_alloc(poff, N + 1) || !host_alloc(mine, N) || !host_alloc(all, N * N) || !host_alloc(roff, N + 1) ||
      !host_alloc(counts, N))
    status = CASK_E_NOMEM;
  // 1. this rank's block split by key owner, on its device
  const void* parts = nullptr;
  if (status == CASK_OK && bytes) status = cask_keydir_partition(ctx, block, bytes, (uint32_t)nranks, &parts, poff.data());
  // 2. the nranks x nranks matrix of part sizes (row r: what rank r sends to each owner)
  for (int o = 0; o < nranks && status == CASK_OK; ++o) mine[o] = poff[o + 1] - poff[o];
  if (!allgather_u64(K, st, status == CASK_OK ? mine.data() : nullptr, N, all)) return CASK_E_DEVICE;
  for (int r = 0; r < nranks && status == CASK_OK; ++r) roff[r + 1] = roff[r] + ((all[(uint64_t)r * N + rank] + 255) & ~255ull);
  DevMem buf;
  std::vector<uint8_t> host;
  if (status == CASK_OK && roff[nranks] && (hipMalloc(&buf.p, roff[nranks]) != hipSuccess || !host_alloc(host, roff[nranks])))
    status = CASK_E_NOMEM;
  if ((status = agree(K, st, status)) != CASK_OK) return status;
  // 3. the all-to-all: part o to rank o, one grouped send/recv per pair
  if (K.R->GroupStart() != ncclSuccess) return CASK_E_DEVICE;
  bool moved = true;
  for (int r = 0; r < nranks; ++r) {
    const uint64_t in = all[(uint64_t)r * N + rank], out = all[(uint64_t)rank * N + r];
    if (r == rank) {
      if (in) moved = moved && hipMemcpyAsync((uint8_t*)buf.p + roff[r], (const uint8_t*)parts + poff[r], in,
                                              hipMemcpyDeviceToDevice, st) == hipSuccess;
      continue;
    }
    if (out) moved = moved && K.R->Send((const uint8_t*)parts + poff[r], out, ncclUint8, r, K.c, st) == ncclSuccess;
    if (in) moved = moved && K.R->Recv((uint8_t*)buf.p + roff[r], in, ncclUint8, r, K.c, st) == ncclSuccess;
  }
  if (K.R->GroupEnd() != ncclSuccess || !moved || hipStreamSynchronize(st) != hipSuccess) return CASK_E_DEVICE;
  uint64_t sent = 0, got = 0;
  for (int r = 0; r < nranks; ++r) {
    if (r != rank) sent += all[(uint64_t)rank * N + r];
    got += all[(uint64_t)r * N + rank];
  }
  if (sent_bytes) *sent_bytes = sent;
  if (recv_bytes) *recv_bytes = got;
  // 4. this owner's fold of its parts, in rank order (= replay order)
  int fst = CASK_OK;
  if (roff[nranks] && hipMemcpy(host.data(), buf.p, roff[nranks], hipMemcpyDeviceToHost) != hipSuccess) fst = CASK_E_DEVICE;
  if (fst == CASK_OK && cask_abi::take_inject(ctx, cask_abi::kInjFold)) fst = CASK_E_NOMEM;
  if (fst == CASK_OK) {  // (one pass over the parts, in rank order)
    std::vector<const uint8_t*> bp;
    std::vector<uint64_t> bl;
    for (int r = 0; r < nranks; ++r) {
      const uint64_t in = all[(uint64_t)r * N + rank];
      if (in) {
        bp.push_back(host.data() + roff[r]);
        bl.push_back(in);
      }
    }
    fst = cask_keydir_merge_many(db, bp.data(), bl.data(), (uint32_t)bp.size());
  }
  // 5. Stats: every owner's per-file terms to every rank (counts, then the padded tables), summed
  int64_t tb = fst == CASK_OK ? cask_keydir_terms(db, nullptr, 0) : 0;
  if (tb < 0) {
    fst = (int)tb;
    tb = 0;
  }
  if ((fst = agree(K, st, fst)) != CASK_OK) return fst;
  const uint64_t nt = (uint64_t)tb / sizeof(KeydirTerm);
  if (!allgather_u64(K, st, &nt, 1, counts)) return CASK_E_DEVICE;
  uint64_t mt = 0;
  for (uint64_t x : counts) mt = std::max(mt, x);
  const uint64_t w = mt * sizeof(KeydirTerm) / 8;  // u64 per rank's padded table
  std::vector<uint64_t> tab, tall;
  DevMem big;  // the all-gather's device buffer when the tables do not fit the scratch
  int tst = host_alloc(tab, std::max<uint64_t>(w, 1)) && host_alloc(tall, std::max<uint64_t>(w * N, 1)) ? CASK_OK : CASK_E_NOMEM;
  if (tst == CASK_OK && 8ull * w * (N + 1) > K.cap && hipMalloc(&big.p, 8ull * w * (N + 1)) != hipSuccess) tst = CASK_E_NOMEM;
  if (tst == CASK_OK && cask_abi::take_inject(ctx, cask_abi::kInjTerms)) tst = CASK_E_INVALID_ARG;
  if (tst == CASK_OK && tb && cask_keydir_terms(db, (uint8_t*)tab.data(), (uint64_t)tb) != tb) tst = CASK_E_INVALID_ARG;
  if ((tst = agree(K, st, tst)) != CASK_OK) return tst;
  if (w && !allgather_u64(K, st, tab.data(), w, tall, big.p)) return CASK_E_DEVICE;
  int ft = CASK_OK;
  try {
    std::vector<uint8_t> terms;
    for (int r = 0; r < nranks; ++r) {
      const uint8_t* p = (const uint8_t*)(tall.data() + (uint64_t)r * w);
      terms.insert(terms.end(), p, p + counts[r] * sizeof(KeydirTerm));
    }
    ft = cask_keydir_finish_terms(db, terms.data(), terms.size());
  } catch (const std::bad_alloc&) {
    ft = CASK_E_NOMEM;
  }
  return agree(K, st, ft);
}

extern "C" int cask_keydir_exchange_rccl(cask_ctx* ctx, void* comm, const void* block, uint64_t bytes, cask_db* db,
                                         uint64_t* sent_bytes, uint64_t* recv_bytes) {
  return cask_abi::guard([&]() -> int {
    if (!ctx || !comm) return CASK_E_INVALID_ARG;  // (no communicator to agree over)
    return exchange_impl(ctx, *(Comm*)comm, block, bytes, db, sent_bytes, recv_bytes);
  });
}
