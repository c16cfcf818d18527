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
// without it gets CASK_E_DEVICE from these calls only.
//
// Every rank issues the same sequence of collectives whatever it passes (a NULL max_seq, an empty
// block), and a failure on any rank between two collectives (a root that cannot allocate the
// gathered size) is agreed on by an ncclAllReduce(min) of a status flag before the data moves: all
// ranks then return the same error instead of some blocking in ncclSend forever.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstring>
#include <mutex>
#include <type_traits>
#include <new>
#include <vector>

#include "../../include/cask_scan.h"
#include "keydir_format.h"

static_assert(CASK_RCCL_ID_BYTES == NCCL_UNIQUE_ID_BYTES, "unique id size");

namespace {

// The RCCL entry points this file uses, resolved from librccl at first use.
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

const Rccl* rccl() {
  static Rccl r;
  static std::once_flag once;
  std::call_once(once, [] {
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_LOCAL);
    if (!h) return;
    bool all = true;
    auto sym = [&](auto& f, const char* name) {
      f = reinterpret_cast<std::remove_reference_t<decltype(f)>>(dlsym(h, name));
      all = all && f != nullptr;
    };
    sym(r.GetUniqueId, "ncclGetUniqueId");
    sym(r.CommInitRank, "ncclCommInitRank");
    sym(r.CommDestroy, "ncclCommDestroy");
    sym(r.CommCount, "ncclCommCount");
    sym(r.CommUserRank, "ncclCommUserRank");
    sym(r.AllGather, "ncclAllGather");
    sym(r.AllReduce, "ncclAllReduce");
    sym(r.Send, "ncclSend");
    sym(r.Recv, "ncclRecv");
    sym(r.GroupStart, "ncclGroupStart");
    sym(r.GroupEnd, "ncclGroupEnd");
    r.ok = all;
  });
  return r.ok ? &r : nullptr;
}

struct DevMem {  // device memory of one call
  void* p = nullptr;
  ~DevMem() {
    if (p) (void)hipFree(p);
  }
};

// Every rank's `n` u64 values, in rank order, on every rank (ncclAllGather through device memory).
bool allgather_u64(const Rccl& R, ncclComm_t c, hipStream_t st, int nranks, const uint64_t* mine, uint64_t n,
                   std::vector<uint64_t>& all) {
  DevMem m;
  if (hipMalloc(&m.p, 8ull * n * (nranks + 1)) != hipSuccess) return false;
  uint64_t* dm = (uint64_t*)m.p;
  all.assign(n * nranks, 0);
  return hipMemcpyAsync(dm + n * nranks, mine, 8ull * n, hipMemcpyHostToDevice, st) == hipSuccess &&
         R.AllGather(dm + n * nranks, dm, n, ncclUint64, c, st) == ncclSuccess &&
         hipMemcpyAsync(all.data(), dm, 8ull * n * nranks, hipMemcpyDeviceToHost, st) == hipSuccess &&
         hipStreamSynchronize(st) == hipSuccess;
}

// The status every rank returns: the lowest (most severe) of the ranks' own statuses (0 = ok), by
// ncclAllReduce(min). A rank that fails between two collectives still calls this, so no peer is left
// waiting in a send or receive it will never match.
int agree(const Rccl& R, ncclComm_t c, hipStream_t st, int mine) {
  DevMem m;
  if (hipMalloc(&m.p, 16) != hipSuccess) return CASK_E_NOMEM;  // (16 B: peers would wait here)
  int32_t* dm = (int32_t*)m.p;
  int32_t v = mine, out = 0;
  if (hipMemcpyAsync(dm, &v, 4, hipMemcpyHostToDevice, st) != hipSuccess ||
      R.AllReduce(dm, dm + 1, 1, ncclInt32, ncclMin, c, st) != ncclSuccess ||
      hipMemcpyAsync(&out, dm + 1, 4, hipMemcpyDeviceToHost, st) != hipSuccess || hipStreamSynchronize(st) != hipSuccess)
    return CASK_E_DEVICE;
  return out;
}

int comm_shape(const Rccl& R, ncclComm_t c, int* nranks, int* rank) {
  return R.CommCount(c, nranks) == ncclSuccess && R.CommUserRank(c, rank) == ncclSuccess ? CASK_OK : CASK_E_DEVICE;
}

}  // namespace

extern "C" int cask_rccl_unique_id(uint8_t* id) {
  if (!id) return CASK_E_INVALID_ARG;
  const Rccl* R = rccl();
  if (!R) return CASK_E_DEVICE;
  ncclUniqueId u;
  if (R->GetUniqueId(&u) != ncclSuccess) return CASK_E_DEVICE;
  memcpy(id, &u, sizeof(u));
  return CASK_OK;
}

extern "C" int cask_rccl_comm_init(const uint8_t* id, int nranks, int rank, int device, void** comm) {
  if (!id || !comm || nranks < 1 || rank < 0 || rank >= nranks) return CASK_E_INVALID_ARG;
  const Rccl* R = rccl();
  if (!R) return CASK_E_DEVICE;
  if (hipSetDevice(device) != hipSuccess) return CASK_E_DEVICE;
  ncclUniqueId u;
  memcpy(&u, id, sizeof(u));
  ncclComm_t c = nullptr;
  if (R->CommInitRank(&c, nranks, u, rank) != ncclSuccess) return CASK_E_DEVICE;
  *comm = c;
  return CASK_OK;
}

extern "C" int cask_rccl_comm_destroy(void* comm) {
  if (!comm) return CASK_E_INVALID_ARG;
  const Rccl* R = rccl();
  if (!R) return CASK_E_DEVICE;
  return R->CommDestroy((ncclComm_t)comm) == ncclSuccess ? CASK_OK : CASK_E_DEVICE;
}

extern "C" int cask_keydir_gather_rccl(cask_ctx* ctx, void* comm, const void* block, uint64_t bytes, int root,
                                       cask_db* db, uint64_t* gathered, uint64_t* max_seq) {
  using namespace cask_kd;
  if (!ctx || !comm || (bytes && !block)) return CASK_E_INVALID_ARG;
  const Rccl* Rp = rccl();
  if (!Rp) return CASK_E_DEVICE;
  const Rccl& R = *Rp;
  ncclComm_t c = (ncclComm_t)comm;
  int nranks = 0, rank = 0;
  if (comm_shape(R, c, &nranks, &rank) != CASK_OK) return CASK_E_DEVICE;
  // (argument errors that differ between ranks are agreed on below, like any other failure)
  if (root < 0 || root >= nranks) return CASK_E_INVALID_ARG;
  if (hipSetDevice(cask_ctx_device(ctx)) != hipSuccess) return CASK_E_DEVICE;
  hipStream_t st = (hipStream_t)cask_ctx_stream(ctx);
  // this rank's block header (its max sequence) from the device
  ShardHeader hd{};
  int status = rank == root && !db ? CASK_E_INVALID_ARG : CASK_OK;
  if (bytes >= sizeof(hd) &&
      (hipMemcpyAsync(&hd, block, sizeof(hd), hipMemcpyDeviceToHost, st) != hipSuccess ||
       hipStreamSynchronize(st) != hipSuccess))
    status = CASK_E_DEVICE;
  // every rank's block size and max sequence + 1 (ncclAllGather of two u64 per rank): the global
  // maximum sequence is the largest of them on every rank, with no collective of its own
  const uint64_t mine[2] = {status == CASK_OK ? bytes : 0, bytes >= sizeof(hd) ? hd.max_seq_p1 : 0};
  std::vector<uint64_t> all;
  if (!allgather_u64(R, c, st, nranks, mine, 2, all)) return CASK_E_DEVICE;
  uint64_t mx = 0;
  for (int r = 0; r < nranks; ++r) mx = std::max(mx, all[2ull * r + 1]);
  if (max_seq) *max_seq = mx ? mx - 1 : 0;
  std::vector<uint64_t> off(nranks + 1, 0);
  for (int r = 0; r < nranks; ++r) off[r + 1] = off[r] + ((all[2ull * r] + 255) & ~255ull);
  if (gathered) *gathered = rank == root ? off[nranks] : bytes;
  // the root's receive buffer, then the agreed status: every rank goes on, or every rank stops
  DevMem buf;
  if (status == CASK_OK && rank == root && off[nranks] && hipMalloc(&buf.p, off[nranks]) != hipSuccess)
    status = CASK_E_NOMEM;
  if ((status = agree(R, c, st, status)) != CASK_OK) return status;
  // the blocks to the root: one grouped send per rank, nranks - 1 receives on the root
  if (R.GroupStart() != ncclSuccess) return CASK_E_DEVICE;
  bool sent = true;
  if (rank == root) {
    for (int r = 0; r < nranks; ++r) {
      if (!all[2ull * r]) continue;
      uint8_t* dst = (uint8_t*)buf.p + off[r];
      if (r == root)
        sent = sent && hipMemcpyAsync(dst, block, bytes, hipMemcpyDeviceToDevice, st) == hipSuccess;
      else
        sent = sent && R.Recv(dst, all[2ull * r], ncclUint8, r, c, st) == ncclSuccess;
    }
  } else if (bytes) {
    sent = R.Send(block, bytes, ncclUint8, root, c, st) == ncclSuccess;
  }
  if (R.GroupEnd() != ncclSuccess || !sent || hipStreamSynchronize(st) != hipSuccess) return CASK_E_DEVICE;
  if (rank != root) return CASK_OK;
  // the root's fold, in rank order (= replay order)
  std::vector<uint8_t> host;
  try {
    host.resize(off[nranks] ? off[nranks] : 1);
  } catch (const std::bad_alloc&) {
    return CASK_E_NOMEM;
  }
  if (off[nranks] && hipMemcpy(host.data(), buf.p, off[nranks], hipMemcpyDeviceToHost) != hipSuccess)
    return CASK_E_DEVICE;
  for (int r = 0; r < nranks; ++r) {
    if (!all[2ull * r]) continue;
    const int rc = cask_keydir_merge(db, host.data() + off[r], all[2ull * r]);
    if (rc != CASK_OK) return rc;
  }
  return CASK_OK;
}

extern "C" int cask_keydir_exchange_rccl(cask_ctx* ctx, void* comm, const void* block, uint64_t bytes, cask_db* db,
                                         uint64_t* sent_bytes, uint64_t* recv_bytes) {
  using namespace cask_kd;
  if (!ctx || !comm || !db || (bytes && !block)) return CASK_E_INVALID_ARG;
  const Rccl* Rp = rccl();
  if (!Rp) return CASK_E_DEVICE;
  const Rccl& R = *Rp;
  ncclComm_t c = (ncclComm_t)comm;
  int nranks = 0, rank = 0;
  if (comm_shape(R, c, &nranks, &rank) != CASK_OK) return CASK_E_DEVICE;
  if ((uint32_t)nranks > kMaxParts) return CASK_E_INVALID_ARG;
  if (hipSetDevice(cask_ctx_device(ctx)) != hipSuccess) return CASK_E_DEVICE;
  hipStream_t st = (hipStream_t)cask_ctx_stream(ctx);
  // 1. this rank's block split by key owner, on its device
  std::vector<uint64_t> poff(nranks + 1, 0);
  const void* parts = nullptr;
  int status = bytes ? cask_keydir_partition(ctx, block, bytes, (uint32_t)nranks, &parts, poff.data()) : CASK_OK;
  // 2. the nranks x nranks matrix of part sizes (row r: what rank r sends to each owner)
  std::vector<uint64_t> mine(nranks, 0), all;
  for (int o = 0; o < nranks && status == CASK_OK; ++o) mine[o] = poff[o + 1] - poff[o];
  if (!allgather_u64(R, c, st, nranks, mine.data(), (uint64_t)nranks, all)) return CASK_E_DEVICE;
  std::vector<uint64_t> roff(nranks + 1, 0);  // what this rank receives from each rank, in rank order
  for (int r = 0; r < nranks; ++r) roff[r + 1] = roff[r] + ((all[(uint64_t)r * nranks + rank] + 255) & ~255ull);
  DevMem buf;
  if (status == CASK_OK && roff[nranks] && hipMalloc(&buf.p, roff[nranks]) != hipSuccess) status = CASK_E_NOMEM;
  if ((status = agree(R, c, st, status)) != CASK_OK) return status;
  // 3. the all-to-all: part o to rank o, one grouped send/recv per pair
  if (R.GroupStart() != ncclSuccess) return CASK_E_DEVICE;
  bool moved = true;
  for (int r = 0; r < nranks; ++r) {
    const uint64_t in = all[(uint64_t)r * nranks + rank], out = all[(uint64_t)rank * nranks + r];
    if (r == rank) {
      if (in) moved = moved && hipMemcpyAsync((uint8_t*)buf.p + roff[r], (const uint8_t*)parts + poff[r], in,
                                              hipMemcpyDeviceToDevice, st) == hipSuccess;
      continue;
    }
    if (out) moved = moved && R.Send((const uint8_t*)parts + poff[r], out, ncclUint8, r, c, st) == ncclSuccess;
    if (in) moved = moved && R.Recv((uint8_t*)buf.p + roff[r], in, ncclUint8, r, c, st) == ncclSuccess;
  }
  if (R.GroupEnd() != ncclSuccess || !moved || hipStreamSynchronize(st) != hipSuccess) return CASK_E_DEVICE;
  uint64_t sent = 0, got = 0;
  for (int r = 0; r < nranks; ++r) {
    if (r != rank) sent += all[(uint64_t)rank * nranks + r];
    got += all[(uint64_t)r * nranks + rank];
  }
  if (sent_bytes) *sent_bytes = sent;
  if (recv_bytes) *recv_bytes = got;
  // 4. this owner's fold of its parts, in rank order (= replay order)
  std::vector<uint8_t> host;
  int fst = CASK_OK;
  try {
    host.resize(roff[nranks] ? roff[nranks] : 1);
  } catch (const std::bad_alloc&) {
    fst = CASK_E_NOMEM;
  }
  if (fst == CASK_OK && roff[nranks] && hipMemcpy(host.data(), buf.p, roff[nranks], hipMemcpyDeviceToHost) != hipSuccess)
    fst = CASK_E_DEVICE;
  for (int r = 0; r < nranks && fst == CASK_OK; ++r) {
    const uint64_t in = all[(uint64_t)r * nranks + rank];
    if (in) fst = cask_keydir_merge(db, host.data() + roff[r], in);
  }
  // 5. Stats: every owner's per-file terms to every rank (sizes, then the padded tables), summed
  int64_t tb = fst == CASK_OK ? cask_keydir_terms(db, nullptr, 0) : 0;
  if (tb < 0) {
    fst = (int)tb;
    tb = 0;
  }
  if ((fst = agree(R, c, st, fst)) != CASK_OK) return fst;
  const uint64_t nt = (uint64_t)tb / sizeof(KeydirTerm);
  std::vector<uint64_t> counts;
  if (!allgather_u64(R, c, st, nranks, &nt, 1, counts)) return CASK_E_DEVICE;
  uint64_t mt = 0;
  for (uint64_t x : counts) mt = std::max(mt, x);
  const uint64_t w = mt * sizeof(KeydirTerm) / 8;  // u64 per rank's padded table
  std::vector<uint64_t> tab(std::max<uint64_t>(w, 1), 0), tall;
  if (tb && cask_keydir_terms(db, (uint8_t*)tab.data(), (uint64_t)tb) != tb) return CASK_E_INVALID_ARG;
  if (w && !allgather_u64(R, c, st, nranks, tab.data(), w, tall)) return CASK_E_DEVICE;
  std::vector<uint8_t> terms;
  for (int r = 0; r < nranks; ++r) {
    const uint8_t* p = (const uint8_t*)(tall.data() + (uint64_t)r * w);
    terms.insert(terms.end(), p, p + counts[r] * sizeof(KeydirTerm));
  }
  return cask_keydir_finish_terms(db, terms.data(), terms.size());
}
