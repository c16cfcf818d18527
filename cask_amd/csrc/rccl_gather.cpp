// RCCL over xGMI for the multi-GPU replay, behind the C ABI so that a host in any
// language (the reference's Rust Cask::open, cask.rs:346-382) can gather the shards' keydir blocks
// without torch: a communicator from a unique id the caller distributes, then one rooted gather of
// variable-size device blocks — the block sizes by ncclAllGather, the blocks by grouped
// ncclSend/ncclRecv (RCCL has no gatherv; one message per rank, each on its own xGMI link into the
// root) — and the maximum sequence by ncclAllReduce. The root folds the blocks in rank order
// (cask_keydir_merge: rank order is replay order, the shards being contiguous file-id ranges).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstring>
#include <new>
#include <vector>

#include "../../include/cask_scan.h"
#include "keydir_format.h"

static_assert(CASK_RCCL_ID_BYTES == NCCL_UNIQUE_ID_BYTES, "unique id size");

extern "C" int cask_rccl_unique_id(uint8_t* id) {
  if (!id) return CASK_E_INVALID_ARG;
  ncclUniqueId u;
  if (ncclGetUniqueId(&u) != ncclSuccess) return CASK_E_DEVICE;
  memcpy(id, &u, sizeof(u));
  return CASK_OK;
}

extern "C" int cask_rccl_comm_init(const uint8_t* id, int nranks, int rank, int device, void** comm) {
  if (!id || !comm || nranks < 1 || rank < 0 || rank >= nranks) return CASK_E_INVALID_ARG;
  if (hipSetDevice(device) != hipSuccess) return CASK_E_DEVICE;
  ncclUniqueId u;
  memcpy(&u, id, sizeof(u));
  ncclComm_t c = nullptr;
  if (ncclCommInitRank(&c, nranks, u, rank) != ncclSuccess) return CASK_E_DEVICE;
  *comm = c;
  return CASK_OK;
}

extern "C" int cask_rccl_comm_destroy(void* comm) {
  if (!comm) return CASK_E_INVALID_ARG;
  return ncclCommDestroy((ncclComm_t)comm) == ncclSuccess ? CASK_OK : CASK_E_DEVICE;
}

namespace {

struct DevMem {  // device memory of one call
  void* p = nullptr;
  ~DevMem() {
    if (p) (void)hipFree(p);
  }
};

}  // namespace

extern "C" int cask_keydir_gather_rccl(cask_ctx* ctx, void* comm, const void* block, uint64_t bytes, int root,
                                       cask_db* db, uint64_t* gathered, uint64_t* max_seq) {
  using namespace cask_kd;
  if (!ctx || !comm || (bytes && !block)) return CASK_E_INVALID_ARG;
  ncclComm_t c = (ncclComm_t)comm;
  int nranks = 0, rank = 0;
  if (ncclCommCount(c, &nranks) != ncclSuccess || ncclCommUserRank(c, &rank) != ncclSuccess) return CASK_E_DEVICE;
  if (root < 0 || root >= nranks || (rank == root && !db)) return CASK_E_INVALID_ARG;
  if (hipSetDevice(cask_ctx_device(ctx)) != hipSuccess) return CASK_E_DEVICE;
  hipStream_t st = (hipStream_t)cask_ctx_stream(ctx);
  // this rank's block header (its max sequence) from the device
  ShardHeader hd{};
  if (bytes >= sizeof(hd) &&
      (hipMemcpyAsync(&hd, block, sizeof(hd), hipMemcpyDeviceToHost, st) != hipSuccess ||
       hipStreamSynchronize(st) != hipSuccess))
    return CASK_E_DEVICE;
  // every rank's block size and max sequence + 1: ncclAllGather of two u64 per rank
  DevMem meta;
  if (hipMalloc(&meta.p, 16ull * (nranks + 1)) != hipSuccess) return CASK_E_DEVICE;
  uint64_t mine[2] = {bytes, bytes >= sizeof(hd) ? hd.max_seq_p1 : 0};
  uint64_t* dm = (uint64_t*)meta.p;
  std::vector<uint64_t> all(2ull * nranks);
  if (hipMemcpyAsync(dm + 2ull * nranks, mine, 16, hipMemcpyHostToDevice, st) != hipSuccess ||
      ncclAllGather(dm + 2ull * nranks, dm, 2, ncclUint64, c, st) != ncclSuccess ||
      hipMemcpyAsync(all.data(), dm, 16ull * nranks, hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipStreamSynchronize(st) != hipSuccess)
    return CASK_E_DEVICE;
  // the global maximum sequence (+ 1) by ncclAllReduce(max), on every rank
  if (max_seq) {
    uint64_t mx = 0;
    if (hipMemcpyAsync(dm, &mine[1], 8, hipMemcpyHostToDevice, st) != hipSuccess ||
        ncclAllReduce(dm, dm + 1, 1, ncclUint64, ncclMax, c, st) != ncclSuccess ||
        hipMemcpyAsync(&mx, dm + 1, 8, hipMemcpyDeviceToHost, st) != hipSuccess || hipStreamSynchronize(st) != hipSuccess)
      return CASK_E_DEVICE;
    *max_seq = mx ? mx - 1 : 0;
  }
  std::vector<uint64_t> off(nranks + 1, 0);
  for (int r = 0; r < nranks; ++r) off[r + 1] = off[r] + ((all[2ull * r] + 255) & ~255ull);
  if (gathered) *gathered = rank == root ? off[nranks] : bytes;
  // the blocks to the root: one grouped send per rank, nranks - 1 receives on the root
  DevMem buf;
  if (rank == root && off[nranks] && hipMalloc(&buf.p, off[nranks]) != hipSuccess) return CASK_E_NOMEM;
  if (ncclGroupStart() != ncclSuccess) return CASK_E_DEVICE;
  bool ok = true;
  if (rank == root) {
    for (int r = 0; r < nranks; ++r) {
      if (!all[2ull * r]) continue;
      uint8_t* dst = (uint8_t*)buf.p + off[r];
      if (r == root)
        ok = ok && hipMemcpyAsync(dst, block, bytes, hipMemcpyDeviceToDevice, st) == hipSuccess;
      else
        ok = ok && ncclRecv(dst, all[2ull * r], ncclUint8, r, c, st) == ncclSuccess;
    }
  } else if (bytes) {
    ok = ncclSend(block, bytes, ncclUint8, root, c, st) == ncclSuccess;
  }
  if (ncclGroupEnd() != ncclSuccess || !ok || hipStreamSynchronize(st) != hipSuccess) return CASK_E_DEVICE;
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
