// Host runtime behind include/cask_scan.h: device contexts, scratch management, the scan
// pipeline (speculative chunk scan -> long records -> validate -> [repair] -> summary) and the
// batched encoder. Compiled with hipcc into libcask_scan.so.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <new>
#include <vector>

#include "../../include/cask_scan.h"
#include "abi_guard.h"
#include "host_ring.h"
#include "keydir_format.h"
#include "scan_kernels.h"
#include "xxh32.h"
#include "knobs.h"

using namespace cask_dev;

namespace {

// Device scratch that only grows. Owned by a context; freed by its destructor (cask_ctx_destroy),
// so no buffer outlives its context.
struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
  DevBuf() = default;
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  ~DevBuf() { release(); }
  // Returns false on allocation failure; `fresh` (optional) is set when the buffer was reallocated.
  bool ensure(size_t bytes, bool* fresh = nullptr) {
    if (fresh) *fresh = false;
    if (bytes <= cap) return true;
    release();
    size_t want = bytes + bytes / 4 + 256;
    if (hipMalloc(&p, want) != hipSuccess) {
      p = nullptr;
      return false;
    }
    cap = want;
    if (fresh) *fresh = true;
    return true;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
  template <typename T>
  T* as() const { return (T*)p; }
  void swap(DevBuf& o) {
    std::swap(p, o.p);
    std::swap(cap, o.cap);
  }
};

struct HostPinned {
  void* p = nullptr;
  size_t cap = 0;
  HostPinned() = default;
  HostPinned(const HostPinned&) = delete;
  HostPinned& operator=(const HostPinned&) = delete;
  ~HostPinned() { release(); }
  bool ensure(size_t bytes) {
    if (bytes <= cap) return true;
    release();
    size_t want = bytes + bytes / 4 + 256;
    if (hipHostMalloc(&p, want, hipHostMallocDefault) != hipSuccess) {
      p = nullptr;
      return false;
    }
    cap = want;
    return true;
  }
  void release() {
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
  }
};

inline uint64_t align_up(uint64_t x, uint64_t a) { return (x + a - 1) / a * a; }

}  // namespace

struct cask_ctx {
  int device = 0;
  hipStream_t own = nullptr;
  hipStream_t side = nullptr;  // walk mode: k_finish beside k_run_hash
  hipStream_t masked[2] = {};  // diagnostic builds: streams held to some of the CUs (CASK_HASH_CUS, CASK_PRE_CUS)
  hipStream_t stream = nullptr;
  // Members are destroyed in reverse order: every buffer is freed before the context goes.
  DevBuf chunk;      // spec | exit | base | tin (u64 x4) | count (u32) | tiles | long_r | desc | gbase
  DevBuf slots;      // 16-B slot rows, slot_cap per chunk
  DevBuf slots_alt;  // walk mode's repair path: the slot rows re-strided to the full count
  DevBuf filebuf;    // FileDesc[] | call block (CallLayout) | file_err[] | first_bad[] | file_total[] | summary
  DevBuf err2;       // error detail words
  DevBuf gather;     // cask_read_entries_device: positions, sources and outputs of one batch
  DevBuf stamps;     // diagnostic builds (-DCASK_STAMPS) only
  DevBuf repair;     // runs (u64 x 2 per chunk) | cerr (u32) | redo (u8) | long_done (u8)
  DevBuf lq;         // long-record queue (slot indices by length class)
  DevBuf tstate;     // k_finish look-back granules (8 per tile), tagged with `epoch`
  DevBuf keyat;      // cask_shard_keydir_hints: per row, its key's offset in its hint body
  DevBuf cdesc;      // walk mode, split path: per chunk its address and its file's end (2 x u64)
  DevBuf tbits;      // walk mode: the tail pieces' long-record bits (kTailBitWords per piece)
  DevBuf probe;      // k_probe_regions: 3 u64 per region of each file
  DevBuf mruns;      // mixed call: walk-mode run indices | chunk-mode [first, end) stretches
  uint32_t epoch = 0;
  uint32_t inject = 0;  // test hooks: cask_debug_inject (abi_guard.h)
  bool full_slots_next = false;  // the next call (a redo) sizes its slot rows in full
  uint64_t* dbg_spec = nullptr;
  uint64_t* dbg_exit = nullptr;
  uint64_t* dbg_tin = nullptr;
  uint32_t* dbg_count = nullptr;
  uint64_t dbg_n = 0;
  HostPinned hfiles;
  HostPinned hsum;
  HostPinned hcall;
  // host-scan staging
  DevBuf stage_data;
  DevBuf stage_rows;
  std::unique_ptr<cask_host::PinnedRing> ring;  // cask_scan_host: pinned staging, made on first use
  int geo = -1;      // k_scan_chunks geometry: -1 picks one per call (CASK_SCAN_GEOMETRY forces one)
  hipEvent_t ev[8] = {};
  hipEvent_t evw = nullptr;  // cask_ctx_wait_stream
  hipEvent_t evf = nullptr;  // walk mode: k_finish done on the side stream
  void* kd = nullptr;        // cask_shard_keydir scratch (k_keydir.hip)
  float last_ms[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  uint64_t last_counters[5] = {0, 0, 0, 0, 0};
  int last_dense = 0;  // the last call's rows came from k_finish (every speculated start held)
  int last_walk = 0;   // the last call's mode: 0 chunk, 1 walk, 2 mixed
  int last_geo = -1;   // the last call's k_scan_chunks geometry (-1: walk mode)
  // The file table and two call blocks stay on the device between calls: a call whose file table is
  // the last one's, and whose call block k_finish zeroed during the last call, needs no copy to the
  // device before its first kernel.
  std::vector<FileDesc> fd_last;
  const void* fb_last = nullptr;
  size_t callb_last = 0;
  int cb_cur = 0;               // the call block the last call used
  bool cb_zero[2] = {false, false};
  uint64_t probe_sig = 0;  // files of the last k_probe_regions, and its answer
  bool probe_walk = false;   // every region of every file reads fastest in walk mode
  bool probe_mixed = false;  // some regions in walk mode, some in chunk mode
  bool probe_short = false;  // chunk mode: the short-halo geometry (kGeoShortHalo)
  std::vector<uint8_t> probe_region;     // per file and region (kProbeRegions): 1 = walk mode
  std::vector<unsigned long long> probe_host;
  uint64_t mixed_key = 0;                // the run lists in mruns: for this probe and run length
  uint64_t mixed_nw = 0, mixed_nc = 0;   // walk-mode runs, chunk-mode runs
  std::vector<uint64_t> mruns_host;
  std::mutex mu;
  char last_error[256] = {0};
  ~cask_ctx() {
    (void)hipSetDevice(device);
    if (stream) (void)hipStreamSynchronize(stream);
    if (side) (void)hipStreamSynchronize(side);
    for (auto& e : ev)
      if (e) (void)hipEventDestroy(e);
    if (evw) (void)hipEventDestroy(evw);
    if (kd) kd_scratch_destroy(kd);
    if (own) (void)hipStreamDestroy(own);
    if (side) (void)hipStreamDestroy(side);
    for (hipStream_t m : masked)
      if (m) (void)hipStreamDestroy(m);
    if (evf) (void)hipEventDestroy(evf);
  }
};

static int set_dev(const cask_ctx* c) {
  return hipSetDevice(c->device) == hipSuccess ? CASK_OK : CASK_E_DEVICE;
}

bool cask_abi::take_inject(cask_ctx* c, uint32_t bit) {
  if (!c || !(c->inject & bit)) return false;
  c->inject &= ~bit;
  return true;
}

// Test hook: force failures on this context (abi_guard.h); CASK_E_INVALID_ARG outside the tests.
extern "C" int cask_debug_inject(cask_ctx* c, uint32_t bits) {
  if (!c || !cask_knobs::test_hooks()) return CASK_E_INVALID_ARG;
  c->inject = bits;
  return CASK_OK;
}

extern "C" {

cask_ctx* cask_ctx_create(int device, int* status) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n) {
    if (status) *status = CASK_E_DEVICE;
    return nullptr;
  }
  cask_ctx* c = new (std::nothrow) cask_ctx();
  if (!c) {
    if (status) *status = CASK_E_NOMEM;
    return nullptr;
  }
  c->device = device;
  if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&c->own, hipStreamNonBlocking) != hipSuccess) {
    delete c;
    if (status) *status = CASK_E_DEVICE;
    return nullptr;
  }
  c->stream = c->own;
  c->geo = -1;
  if (const char* g = cask_knobs::tune("CASK_SCAN_GEOMETRY")) c->geo = atoi(g);
  for (auto& e : c->ev) (void)hipEventCreate(&e);
  (void)hipEventCreateWithFlags(&c->evw, hipEventDisableTiming);
  (void)hipEventCreateWithFlags(&c->evf, hipEventDisableTiming);
  (void)hipStreamCreateWithFlags(&c->side, hipStreamNonBlocking);
  if (!c->err2.ensure(64)) {
    cask_ctx_destroy(c);
    if (status) *status = CASK_E_NOMEM;
    return nullptr;
  }
  if (status) *status = CASK_OK;
  return c;
}

void cask_ctx_destroy(cask_ctx* c) {
  delete c;  // ~cask_ctx waits for the stream, then every DevBuf/HostPinned frees its memory
}

int cask_ctx_set_stream(cask_ctx* c, void* s) {
  return cask_abi::guard([&]() -> int {
    if (!c) return CASK_E_INVALID_ARG;
    c->stream = s ? (hipStream_t)s : c->own;
    return CASK_OK;
  });
}

int cask_ctx_wait_stream(cask_ctx* c, void* other) {
  return cask_abi::guard([&]() -> int {
    if (!c) return CASK_E_INVALID_ARG;
    if ((hipStream_t)other == c->stream) return CASK_OK;
    std::lock_guard<std::mutex> g(c->mu);
    if (set_dev(c)) return CASK_E_DEVICE;
    if (hipEventRecord(c->evw, (hipStream_t)other) != hipSuccess ||
        hipStreamWaitEvent(c->stream, c->evw, 0) != hipSuccess)
      return CASK_E_DEVICE;
    return CASK_OK;
  });
}

void* cask_ctx_stream(cask_ctx* c) { return c ? (void*)c->stream : nullptr; }
int cask_ctx_device(const cask_ctx* c) { return c ? c->device : -1; }
const char* cask_ctx_last_error(const cask_ctx* c) { return c ? c->last_error : ""; }
uint32_t cask_scan_chunk_bytes(void) { return geometry_chunk(kDefaultGeometry); }

uint64_t cask_rows_bound(const cask_file_view* files, uint32_t nfiles) {
  uint64_t b = 0;
  for (uint32_t i = 0; i < nfiles; ++i) b += files[i].len / CASK_ENTRY_STATIC_SIZE + 1;
  return b;
}

uint32_t cask_xxh32(const uint8_t* data, uint64_t len) { return cask_xxh::xxh32(data, len, 0); }

int cask_last_timings(const cask_ctx* c, float* ms6) {
  return cask_abi::guard([&]() -> int {
    if (!c || !ms6) return CASK_E_INVALID_ARG;
    memcpy(ms6, c->last_ms, 6 * sizeof(float));
    return CASK_OK;
  });
}

int cask_last_timings8(const cask_ctx* c, float* ms8) {
  return cask_abi::guard([&]() -> int {
    if (!c || !ms8) return CASK_E_INVALID_ARG;
    memcpy(ms8, c->last_ms, 8 * sizeof(float));
    return CASK_OK;
  });
}

int cask_last_dense(const cask_ctx* c) { return c ? c->last_dense : 0; }

uint64_t cask_ctx_scratch_bytes(const cask_ctx* c) {
  if (!c) return 0;
  const DevBuf* bufs[] = {&c->chunk, &c->slots, &c->filebuf, &c->err2, &c->gather, &c->stamps, &c->repair, &c->lq,
                          &c->tstate, &c->keyat, &c->cdesc, &c->tbits, &c->probe, &c->mruns, &c->stage_data, &c->stage_rows};
  uint64_t t = 0;
  for (const DevBuf* b : bufs) t += b->cap;
  return t;
}

int cask_last_walk(const cask_ctx* c) { return c ? c->last_walk : 0; }

int cask_last_geometry(const cask_ctx* c) { return c ? c->last_geo : -1; }

int cask_last_counters(const cask_ctx* c, uint64_t* c5) {
  return cask_abi::guard([&]() -> int {
    if (!c || !c5) return CASK_E_INVALID_ARG;
    memcpy(c5, c->last_counters, sizeof(c->last_counters));
    return CASK_OK;
  });
}

}  // extern "C"

// Core pipeline on device-resident files: dense SoA rows in the caller's arrays.
//
// Dense path (the common case): k_scan_chunks, then k_finish validates every speculated chunk
// start and writes the dense rows; one copy of the call block tells the host whether every start
// held and whether records longer than the window wait for k_long. Two kernels when the log has
// no long records. If some start was wrong the repair path takes over (validate, exact re-scans,
// k_compact).
static int scan_device_impl(cask_ctx* c, const cask_file_view* files, uint32_t nfiles, cask_rows* rows,
                            uint64_t* file_row_offset, cask_scan_error* err, bool hint = false) {
  if (nfiles && !files) return CASK_E_INVALID_ARG;
  if (rows && rows->capacity && (!rows->pos || !rows->seq || !rows->vsz || !rows->ksz || !rows->status))
    return CASK_E_INVALID_ARG;
  for (uint32_t i = 0; i < nfiles; ++i)
    if (files[i].len && !files[i].data) return CASK_E_INVALID_ARG;
  if (set_dev(c)) return CASK_E_DEVICE;
  hipStream_t st = c->stream;

  // file table (every geometry picked automatically has the default's chunk size)
  int geo = c->geo >= 0 ? c->geo : kDefaultGeometry;
  const uint32_t chunk = geometry_chunk(geo);
  // slot rows per chunk, rounded to 8 rows: every chunk's rows start on a 128-B line, so the
  // scan's 1-KiB row stores cover whole lines and need no fill from HBM. The full count holds every
  // record a chunk can start (18-B records); a walk-mode call uses kWalkSlotCap (below).
  const uint32_t slot_full = ((chunk / 18 + 2) + 7) & ~7u;
  uint64_t total_chunks = 0, total_tiles = 0;
  const size_t head_words = sizeof(SummaryHead) / 8;
  const size_t sum_words = head_words + (nfiles + 1) + 4ull * nfiles;
  const size_t call_bytes = CallLayout::bytes(nfiles);
  // the file table and the zeroed call block go to the device in one copy: [FileDesc | call block]
  const size_t fd_bytes = align_up(sizeof(FileDesc) * (nfiles + 1), 256);
  if (!c->hfiles.ensure(fd_bytes + call_bytes) || !c->hsum.ensure(sum_words * 8) || !c->hcall.ensure(call_bytes))
    return CASK_E_NOMEM;
  memset((uint8_t*)c->hfiles.p + fd_bytes, 0, call_bytes);
  FileDesc* fd = (FileDesc*)c->hfiles.p;
  for (uint32_t i = 0; i < nfiles; ++i) {
    fd[i].data = files[i].data;
    fd[i].len = files[i].len;
    fd[i].first_chunk = total_chunks;
    fd[i].nchunks = (files[i].len + chunk - 1) / chunk;
    fd[i].first_tile = total_tiles;
    fd[i].pad = 0;
    total_chunks += fd[i].nchunks;
    total_tiles += (fd[i].nchunks + kTileChunks - 1) / kTileChunks;
  }
  const uint64_t fin_tiles = (total_chunks + kFinTile - 1) / kFinTile;
  // device scratch
  const size_t pf_bytes = align_up(8ull * (nfiles + 1), 256);
  const size_t sum_bytes = align_up(sum_words * 8, 256);
  const size_t callb = align_up(call_bytes, 256);
  const uint64_t C = total_chunks + 1;
  bool fb_fresh = false;  // (a new allocation may reuse the old address: never resident)
  if (!c->filebuf.ensure(fd_bytes + 2 * callb + 3 * pf_bytes + sum_bytes, &fb_fresh)) return CASK_E_NOMEM;
  if (!c->chunk.ensure(C * (4 * 8 + 4 + 4 + 16 + 8) + (total_tiles + 1) * 4 * 8 + 1024)) return CASK_E_NOMEM;
  const size_t runs_bytes = align_up(16ull * (total_chunks + 1), 256), cerr_bytes = align_up(4ull * (total_chunks + 1), 256),
               redo_bytes = align_up(total_chunks + 1, 256);
  if (!c->repair.ensure(runs_bytes + cerr_bytes + 2 * redo_bytes)) return CASK_E_NOMEM;
  if (!c->lq.ensure(8 * (lq_region_base(total_chunks, chunk, 32) + 1))) return CASK_E_NOMEM;
  bool fresh = false;  // k_finish look-back granules, 8 per tile
  // (then the group aggregates of the two-level prefix)
  if (!c->tstate.ensure(64ull * (fin_tiles + 1) + 64ull * (fin_tiles / kFinGroup + 2), &fresh)) return CASK_E_NOMEM;

  uint8_t* fbase = c->filebuf.as<uint8_t>();
  FileDesc* d_files = (FileDesc*)fbase;
  // call block: the other one than last time if that one is known zero and the file table is the
  // same (then nothing is copied to the device before the first kernel), else block 0 with a copy
  const bool fd_same = !fb_fresh && c->fb_last == fbase && c->callb_last == callb && c->fd_last.size() == nfiles &&
                       (nfiles == 0 || !memcmp(c->fd_last.data(), fd, sizeof(FileDesc) * nfiles));
  const bool resident = fd_same && c->cb_zero[c->cb_cur ^ 1];
  const int cbi = resident ? (c->cb_cur ^ 1) : 0;
  c->cb_zero[0] = c->cb_zero[1] = false;  // (set again only when this call completes on the dense path)
  c->fd_last.assign(fd, fd + nfiles);
  c->fb_last = fbase;
  c->callb_last = callb;
  c->cb_cur = cbi;
  uint8_t* callp = fbase + fd_bytes + cbi * callb;
  unsigned long long* d_ferr = (unsigned long long*)(fbase + fd_bytes + 2 * callb);
  uint64_t* d_fbad = (uint64_t*)(fbase + fd_bytes + 2 * callb + pf_bytes);
  uint64_t* d_ftot = (uint64_t*)(fbase + fd_bytes + 2 * callb + 2 * pf_bytes);
  uint64_t* d_sum = (uint64_t*)(fbase + fd_bytes + 2 * callb + 3 * pf_bytes);

  uint64_t* cb = c->chunk.as<uint64_t>();
  ScanArgs a{};
  a.files = d_files;
  a.nfiles = nfiles;
  a.exact = 0;
  a.total_chunks = total_chunks;
  a.chunk = chunk;
  a.spec = cb;
  a.exit = cb + C;
  a.base = cb + 2 * C;
  a.tin = cb + 3 * C;
  a.count = (uint32_t*)(cb + 4 * C);
  {
    uint64_t* tb = cb + 4 * C + (C + 1) / 2 + 1;
    const uint64_t TT = total_tiles + 1;
    a.long_r = (uint32_t*)(tb + 4 * TT);
    uint64_t doff = (uint64_t)(tb - cb) + 4 * TT + (C + 1) / 2 + 2;  // after long_r, 16-B aligned
    doff = (doff + 1) & ~1ull;
    a.desc = (uint32_t*)(cb + doff);
    a.gbase = cb + doff + 2 * C;  // after desc (16 B per chunk)
    a.total_tiles = total_tiles;
    a.tile_max = tb;
    a.tile_sum = tb + TT;
    a.tile_pmax = tb + 2 * TT;
    a.tile_psum = tb + 3 * TT;
  }
  a.file_total = d_ftot;
  a.file_err = d_ferr;
  a.first_bad = d_fbad;
  a.ctr = (Counters*)callp;
  a.row_off = (uint64_t*)(callp + CallLayout::kHead);
  a.err_inv = (unsigned long long*)(a.row_off + nfiles + 1);
  uint8_t* rb = c->repair.as<uint8_t>();
  uint64_t* d_runs = (uint64_t*)rb;
  a.cerr = (uint32_t*)(rb + runs_bytes);
  a.redo = rb + runs_bytes + cerr_bytes;
  a.long_done = rb + runs_bytes + cerr_bytes + redo_bytes;
  a.lq = c->lq.as<uint64_t>();
  a.runs = nullptr;
  a.nruns_list = 0;
  a.tstate = c->tstate.as<uint64_t>();
  a.call_zero = (uint64_t*)(fbase + fd_bytes + (cbi ^ 1) * callb);  // k_finish clears the other block
  a.call_zero_words = (uint32_t)(callb / 8);
  if (rows) {
    a.pos = rows->pos;
    a.seq = rows->seq;
    a.vsz = rows->vsz;
    a.ksz = rows->ksz;
    a.status = rows->status;
    a.row_cap = rows->capacity;
    a.vec_ok = ((uintptr_t)rows->pos % 16 == 0 && (uintptr_t)rows->seq % 16 == 0 && (uintptr_t)rows->vsz % 16 == 0 &&
                (uintptr_t)rows->ksz % 8 == 0 && (uintptr_t)rows->status % 4 == 0) ? 1u : 0u;
  }
  a.stamps = nullptr;
  a.hint = hint ? 1u : 0u;
  {  // CASK_RUN_CHUNKS (tuning knob): chunks per workgroup run; one boundary search per run.
    // Default: about 8 runs per resident workgroup, at least kDefaultRun and at most kMaxRun chunks —
    // longer runs search less often, which is what variable-length logs pay for (a search that lands
    // inside a record longer than the window scans the whole chunk); the balance at the end comes
    // from the quarter-length tail runs below (configs[1]: 32-chunk runs, 1.2 % faster than 16).
    static const uint32_t run = cask_knobs::tune("CASK_RUN_CHUNKS") ? (uint32_t)atoi(cask_knobs::tune("CASK_RUN_CHUNKS")) : 0u;
    if (run) {
      a.run = run;
    } else {
      const int cus = device_cus();
      const uint64_t per_wg = total_chunks / ((uint64_t)cus * 4u * 8u);
      a.run = (uint32_t)std::min<uint64_t>(kMaxRun, std::max<uint64_t>(kDefaultRun, per_wg));
    }
    // The last grid's worth of runs in runs of a quarter of the length (CASK_RUN_TAIL=0: tuning
    // knob, no short runs): the workgroups then run dry within a short run of each other.
    static const bool tail_on = !(cask_knobs::tune("CASK_RUN_TAIL") && atoi(cask_knobs::tune("CASK_RUN_TAIL")) == 0);
    const uint64_t grid_runs = (uint64_t)device_cus() * 4u;  // resident k_scan_chunks workgroups
    // CASK_RUN_SMALL / CASK_RUN_TAIL_X (tuning knobs): the short runs' length; the tail's length in
    // resident workgroups x run, in quarters
    static const uint32_t rs_env = cask_knobs::tune("CASK_RUN_SMALL") ? (uint32_t)atoi(cask_knobs::tune("CASK_RUN_SMALL")) : 0u;
    static const uint64_t tx = cask_knobs::tune("CASK_RUN_TAIL_X") ? (uint64_t)atoi(cask_knobs::tune("CASK_RUN_TAIL_X")) : 4u;
    a.run_small = rs_env ? std::min(rs_env, a.run) : std::max<uint32_t>(2u, a.run / 4);
    a.run_tail = ~0ull;
    const uint64_t tail = grid_runs * a.run * tx / 4;
    if (tail_on && total_chunks >= 4 * tail) a.run_tail = (total_chunks - tail) / a.run * a.run;
  }
  // regular chunks keep only their first slot row (k_finish and k_compact expand them)
  a.regular_ok = 1u;
  a.respec = 1u;
  // CASK_BIG_REC (tuning knob): records longer than this go to k_long even when they fit the window
  static const uint32_t big_env = cask_knobs::tune("CASK_BIG_REC") ? (uint32_t)atoi(cask_knobs::tune("CASK_BIG_REC")) : kBigRec;
  a.big = big_env;
  if (a.big < kMinBigRec) a.big = kMinBigRec;  // the long-record queue's smallest length class
  a.win = chunk + geometry_halo(geo);
  // CASK_SEARCH_SHORT (tuning knob): k_walk_search verifies candidates up to this long by checksum
  static const uint32_t ss_env = cask_knobs::tune("CASK_SEARCH_SHORT") ? (uint32_t)atoi(cask_knobs::tune("CASK_SEARCH_SHORT")) : 2048u;
  a.search_short = ss_env < 64 ? 64 : ss_env > 2048 ? 2048 : ss_env;
  // the dense path: CASK_DENSE=0 (tuning knob) sends every call through the repair path's k_compact
  static const bool dense_on = !(cask_knobs::tune("CASK_DENSE") && atoi(cask_knobs::tune("CASK_DENSE")) == 0);
  const bool dense = rows != nullptr && dense_on && total_chunks > 0;
  a.dense = 0;  // k_long fixes dense rows only once they are validated

  // look-back granules carry the call's epoch: no memset between calls, one when the tag wraps
  if (fresh || c->epoch >= 255) {
    if (hipMemsetAsync(a.tstate, 0, c->tstate.cap, st) != hipSuccess) return CASK_E_DEVICE;
    c->epoch = 0;
  }
  a.epoch = ++c->epoch;
#ifdef CASK_STAMPS
  if (c->stamps.ensure(8ull * kStampWords)) a.stamps = c->stamps.as<unsigned long long>();
#endif

  bool ok = true;
  auto H = [&](hipError_t e, const char* what = "hip call") {
    if (e != hipSuccess && ok) {
      ok = false;
      snprintf(c->last_error, sizeof(c->last_error), "%s: %s", what, hipGetErrorString(e));
    }
  };
  // CASK_SYNC_EACH=1 (diagnostic): synchronise after every launch so a fault names its kernel
  static const bool sync_each = cask_knobs::tune("CASK_SYNC_EACH") != nullptr;
  auto L = [&](const char* what) {
    H(hipGetLastError(), what);
    if (sync_each) {  // (names the kernel a hang or fault is in, on stderr)
      fprintf(stderr, "cask: %s ...", what);
      H(hipDeviceSynchronize(), what);  // (the walk groups' side streams too)
      fprintf(stderr, " done\n");
    }
  };
  const Counters* hc = (const Counters*)c->hcall.p;
  const uint64_t* h_rowoff = (const uint64_t*)((const uint8_t*)c->hcall.p + CallLayout::kHead);
  const unsigned long long* h_errinv = (const unsigned long long*)(h_rowoff + nfiles + 1);
  auto read_call = [&]() {
    H(hipMemcpyAsync(c->hcall.p, callp, call_bytes, hipMemcpyDeviceToHost, st), "call block D2H");
    H(hipStreamSynchronize(st), "stream sync");
  };

  c->last_error[0] = 0;
  (void)hipGetLastError();  // drop any stale error another library left on this thread
  if (!resident) H(hipMemcpyAsync(d_files, fd, fd_bytes + call_bytes, hipMemcpyHostToDevice, st), "file table H2D");
  // The scan mode, per region of each file (speed only: both modes read any file correctly). Walk
  // mode (k_walk_search -> k_walk_chase -> k_run_hash: the record chain followed header to header,
  // every record hashed from HBM) where the records average kWalkMean bytes or more; chunk mode
  // (k_scan_chunks: every chunk staged through LDS, its records found by search and hashed there)
  // elsewhere. k_probe_regions samples kProbeRegions points of every file once per set of files
  // (the answer is cached on the context). A call whose regions differ runs both, on their own runs.
  // CASK_SCAN_MODE=walk|chunk (test and tuning knob) forces a mode for the whole call.
  // The chunk scan's halo comes from the same probe: CASK_SCAN_MODE=wide|narrow forces the chunk
  // mode with the wide (4,080-B) or the short (1,008-B) halo.
  bool walk = false, mixed = false;
  int halo_pick = 0;  // 1: wide, 2: short (forced); 0: from the probe
  if (hint) {
    walk = true;  // hint bodies are always walked (k_walk_runs' hint mode)
  } else {
    const char* mode = cask_knobs::hook("CASK_SCAN_MODE");
    if (mode && !strcmp(mode, "walk")) {
      walk = true;
    } else if (mode && !strcmp(mode, "chunk")) {
      walk = false;
    } else if (mode && !strcmp(mode, "wide")) {
      halo_pick = 1;
    } else if (mode && !strcmp(mode, "narrow")) {
      halo_pick = 2;
    }
    if (!mode && total_chunks) {
      uint64_t sig = 0x9E3779B97F4A7C15ull ^ nfiles;
      for (uint32_t i = 0; i < nfiles; ++i) {
        sig = (sig ^ (uint64_t)(uintptr_t)files[i].data) * 0xBF58476D1CE4E5B9ull;
        sig = (sig ^ files[i].len) * 0x94D049BB133111EBull;
        sig ^= sig >> 31;
      }
      if (sig != c->probe_sig) {
        const uint64_t np = (uint64_t)nfiles * kProbeRegions;
        if (!c->probe.ensure(24 * np)) return CASK_E_NOMEM;
        c->probe_host.assign(3 * np, 0ull);
        launch_probe_regions(d_files, nfiles, c->probe.as<unsigned long long>(), st);
        L("k_probe_regions");
        H(hipMemcpyAsync(c->probe_host.data(), c->probe.p, 24 * np, hipMemcpyDeviceToHost, st), "probe D2H");
        H(hipStreamSynchronize(st), "probe sync");
        if (!ok) return CASK_E_DEVICE;
        c->probe_region.assign(np, 0);
        uint64_t nw = 0, nreg = 0, cb = 0, cr = 0, cm = 0;
        for (uint64_t i = 0; i < np; ++i) {
          const unsigned long long b = c->probe_host[3 * i], r = c->probe_host[3 * i + 1], m = c->probe_host[3 * i + 2];
          if (!b) continue;  // an empty file
          ++nreg;
          // no record start in the probe window (a longer record covers the point), or long records
          const bool w = r == 0 || b >= (unsigned long long)kWalkMean * r;
          c->probe_region[i] = w ? 1 : 0;
          if (w) {
            ++nw;
          } else {
            cb += b;
            cr += r;
            cm = m > cm ? m : cm;
          }
        }
        c->probe_sig = sig;
        c->probe_walk = nreg && nw == nreg;
        c->probe_mixed = nw && nw < nreg;
        c->probe_short = cr && cb <= kShortHaloMean * cr && cm <= kShortHaloMax;
        c->mixed_key = 0;
      }
      walk = c->probe_walk;
      mixed = c->probe_mixed;
      halo_pick = c->probe_short ? 2 : 1;
    }
  }
  if (mixed) {
    // Each run of kWalkRun chunks in the mode of the region its first chunk lies in: the walk-mode
    // runs by index, the chunk-mode runs as [first, end) stretches for k_scan_chunks (a.runs). Built
    // and copied to the device once per set of files.
    const char* wr = cask_knobs::tune("CASK_WALK_RUN");
    a.run = wr ? (uint32_t)std::min<int>(std::max(1, atoi(wr)), (int)kMaxRun) : kWalkRun;
    a.run_tail = ~0ull;
    const uint64_t R = a.run, nr = (total_chunks + R - 1) / R;
    const uint64_t key = (c->probe_sig ^ (R << 1) ^ (total_chunks << 20)) | 1ull;
    if (c->mixed_key != key) {
      c->mruns_host.assign(3 * nr, 0ull);
      uint64_t* wl = c->mruns_host.data();
      uint64_t* cl = wl + nr;
      uint64_t nw = 0, nc = 0;
      uint32_t fi = 0;
      for (uint64_t r = 0; r < nr; ++r) {
        const uint64_t t = r * R;
        while (fi + 1 < nfiles && (fd[fi].nchunks == 0 || t >= fd[fi].first_chunk + fd[fi].nchunks)) ++fi;
        const uint64_t reg = fd[fi].nchunks ? (t - fd[fi].first_chunk) * kProbeRegions / fd[fi].nchunks : 0;
        if (c->probe_region[(uint64_t)fi * kProbeRegions + std::min<uint64_t>(reg, kProbeRegions - 1)]) {
          wl[nw++] = r;
        } else {
          cl[2 * nc] = t;
          cl[2 * nc + 1] = std::min<uint64_t>(t + R, total_chunks);
          ++nc;
        }
      }
      if (nw && nc) {
        memmove(wl + nw, cl, 16 * nc);
        if (!c->mruns.ensure(8 * (nw + 2 * nc))) return CASK_E_NOMEM;
        H(hipMemcpyAsync(c->mruns.p, wl, 8 * (nw + 2 * nc), hipMemcpyHostToDevice, st), "run lists H2D");
        H(hipStreamSynchronize(st), "run lists sync");
        if (!ok) return CASK_E_DEVICE;
      }
      c->mixed_nw = nw;
      c->mixed_nc = nc;
      c->mixed_key = key;
    }
    if (!c->mixed_nw || !c->mixed_nc) {  // (every run's first chunk fell in one mode)
      mixed = false;
      walk = c->mixed_nw != 0;
    }
  }
  if (c->geo < 0 && (!walk || mixed) && halo_pick == 2) {
    geo = kGeoShortHalo;  // same chunk size: only the window (and the kernel) change
    a.win = chunk + geometry_halo(geo);
  }
  c->last_geo = walk && !mixed ? -1 : geo;
  if (walk && !hint && !mixed) a.big = kWalkHashMax;  // the walker hashes what fits its window, k_long the rest
  if (walk && !mixed) {  // CASK_WALK_RUN (tuning knob): chunks per walk run, at most kMaxRun
    const char* wr = cask_knobs::tune("CASK_WALK_RUN");
    a.run = wr ? (uint32_t)std::min<int>(std::max(1, atoi(wr)), (int)kMaxRun) : hint ? kHintRun : kWalkRun;
    a.run_tail = ~0ull;  // (the chunk scan's short tail runs were sized for its own run length)
  }
  c->last_walk = mixed ? 2 : walk ? 1 : 0;
  // Slot rows: kWalkSlotCap per chunk in a walk-mode call over data files with dense rows (the
  // chase is their only writer; 2 KiB per 32-KiB chunk instead of 29 KiB), else the full count. The
  // small size is redone at full size when a chunk overflows it (Counters::slot_overflow) or the
  // call needs the repair path, whose exact chunk scans may write up to the full count.
  const bool small_slots = walk && !mixed && !hint && dense && !c->full_slots_next;
  c->full_slots_next = false;
  a.slot_cap = small_slots ? kWalkSlotCap : slot_full;
  if (!c->slots.ensure((total_chunks * (uint64_t)a.slot_cap + 1) * 16)) return CASK_E_NOMEM;
  a.slots = c->slots.as<uint32_t>();
  H(hipEventRecord(c->ev[1], st));
  // walk mode on data files: the runs in G groups; per group the walk (which hashes the records
  // that fit its window) and the long records' queueing on the call's stream, then their hashing
  // on a side stream, overlapping the next group's walk (the walk waits on header loads, the long
  // hash on HBM bandwidth). Long records hashed before k_finish mark their rows like any failed
  // check (slot bad bit, cerr), so k_finish sees them.
  bool long_pre = false;
  bool fused = false;
  bool fin_done = false;  // k_finish already launched (beside the hash)
  if (mixed) {  // the walk-mode runs (split path), then the chunk-mode runs, then k_finish for all
    fused = true;
    ScanArgs aw = a;
    aw.wruns = c->mruns.as<uint64_t>();
    aw.nwruns = c->mixed_nw;
    launch_walk_search(aw, st);
    L("k_walk_search");
    H(hipEventRecord(c->ev[6], st));
    aw.walk_pre = 1;
    if (!c->cdesc.ensure(16ull * (total_chunks + 1))) return CASK_E_NOMEM;
    aw.cdesc = c->cdesc.as<uint64_t>();
    launch_walk_chase(aw, st);
    L("k_walk_chase");
    H(hipEventRecord(c->ev[7], st));
    launch_run_hash(aw, st);
    L("k_run_hash");
    ScanArgs ac = a;
    ac.runs = c->mruns.as<uint64_t>() + c->mixed_nw;
    ac.nruns_list = c->mixed_nc;
    launch_scan_chunks(ac, geo, st);
    L("k_scan_chunks");
    // (the chunk-mode runs' long records go to k_long after k_finish, as in a chunk-mode call)
    if (!ok) return CASK_E_DEVICE;
  } else if (walk && !hint) {
    fused = true;
    const uint64_t nruns = (total_chunks + a.run - 1) / a.run;
    ScanArgs as = a;
    as.run_lo = 0;
    as.run_hi = nruns;
    if (!c->cdesc.ensure(16ull * (total_chunks + 1))) return CASK_E_NOMEM;
    // CASK_PRE_CUS / CASK_HASH_CUS (tuning knobs, diagnostics): the search + chase, or the hash, on a
    // stream held to that many CUs (hipExtStreamCreateWithCUMask, the excluded ones spread evenly),
    // each grid sized for them — what reserving CUs for an overlapped pre-hash would cost each side
    static const int pre_cus = cask_knobs::tune("CASK_PRE_CUS") ? atoi(cask_knobs::tune("CASK_PRE_CUS")) : 0;
    static const int hash_cus = cask_knobs::tune("CASK_HASH_CUS") ? atoi(cask_knobs::tune("CASK_HASH_CUS")) : 0;
    auto masked = [&](int k, int ncu) -> hipStream_t {
      const int all = device_cus();
      if (ncu <= 0 || ncu >= all) return st;
      if (!c->masked[k]) {
        std::vector<uint32_t> m((all + 31) / 32, 0u);
        for (int i = 0, kept = 0; i < all; ++i)
          if ((int64_t)(i + 1) * ncu / all > kept) {  // ncu of the all bits, spread evenly
            m[i / 32] |= 1u << (i % 32);
            ++kept;
          }
        if (hipExtStreamCreateWithCUMask(&c->masked[k], (uint32_t)m.size(), m.data()) != hipSuccess) c->masked[k] = nullptr;
      }
      return c->masked[k] ? c->masked[k] : st;
    };
    hipStream_t ps = masked(0, pre_cus), hs = masked(1, hash_cus);
    if (ps != st) {
      H(hipEventRecord(c->evw, st));
      H(hipStreamWaitEvent(ps, c->evw, 0));
    }
    launch_walk_search(as, ps, ps != st ? pre_cus : 0);
    L("k_walk_search");
    H(hipEventRecord(c->ev[6], ps));
    a.walk_pre = 1;
    a.cdesc = c->cdesc.as<uint64_t>();
    // The hash's tail: the last runs, in pieces whose long records are hashed before
    // their short ones (k_run_hash). Only with small slot rows (a piece's records fit its list).
    // CASK_TAIL_SPLIT=0 (tuning knob) turns it off.
    static const bool tail_on = !(cask_knobs::tune("CASK_TAIL_SPLIT") && atoi(cask_knobs::tune("CASK_TAIL_SPLIT")) == 0);
    const uint64_t qr = (a.run + kTailSplit - 1) / kTailSplit;
    a.hash_ntail = 0;
    if (tail_on && small_slots && qr * a.slot_cap <= kTailMaxRecs) {
      // the last two grids' worth of runs (configs[2], A/B: one grid's worth 0.8 % slower, four 0.5 %,
      // half 1.7 %); CASK_TAIL_PCT (tuning knob): the tail runs as a percentage of the hash's grid
      static const uint64_t tail_pct = cask_knobs::tune("CASK_TAIL_PCT") ? (uint64_t)atoi(cask_knobs::tune("CASK_TAIL_PCT")) : 200u;
      a.hash_ntail = std::min<uint64_t>(nruns, std::max<uint64_t>(1, run_hash_waves() * tail_pct / 100));
      if (!c->tbits.ensure(4ull * kTailBitWords * kTailSplit * a.hash_ntail + 256)) return CASK_E_NOMEM;
      a.tbits = c->tbits.as<uint32_t>();
    }
    launch_walk_chase(a, ps);
    L("k_walk_chase");
    H(hipEventRecord(c->ev[7], ps));
    if (ps != st) H(hipStreamWaitEvent(st, c->ev[7], 0));
    if (hs != st) {
      H(hipStreamWaitEvent(hs, c->ev[7], 0));
      launch_run_hash(a, hs, hash_cus);
      H(hipEventRecord(c->evw, hs));
      H(hipStreamWaitEvent(st, c->evw, 0));
    } else {
      launch_run_hash(a, st);
    }
    L("k_run_hash");
    // k_finish needs only the chase's output (the chunk table, the slot rows, the speculated
    // starts): on a side stream it runs in the slots the hash's last waves leave, and k_hash_fix
    // then adds the checksum statuses it may have missed. CASK_FIN_OVERLAP=0 (tuning knob): after.
    static const bool fin_overlap = !(cask_knobs::tune("CASK_FIN_OVERLAP") && atoi(cask_knobs::tune("CASK_FIN_OVERLAP")) == 0);
    if (dense && fin_overlap && c->side && c->evf) {
      H(hipEventRecord(c->ev[2], st));  // (the hash's end, for the timings)
      H(hipStreamWaitEvent(c->side, c->ev[7], 0));
      launch_finish(a, c->side);
      L("k_finish (beside the hash)");
      H(hipEventRecord(c->evf, c->side));
      H(hipStreamWaitEvent(st, c->evf, 0));
      launch_hash_fix(a, st);
      L("k_hash_fix");
      fin_done = true;
    }
    a.walk_pre = 0;
    long_pre = true;
    if (!ok) return CASK_E_DEVICE;
  } else if (walk) {  // hint bodies: the walk searches its own starts (cheaply: hint records are small)
    launch_walk_runs(a, st);
    L("k_walk_runs");
  } else {
    launch_scan_chunks(a, geo, st);
    L("k_scan_chunks");
  }
  if (!fin_done) H(hipEventRecord(c->ev[2], st));
  // (walk mode has hashed its long records already. Queueing them from the walk itself instead of
  // k_long_enqueue measured 1 ms slower: the queue counters' atomics.)
  const bool long_now = long_pre;
  if (dense) {
    if (!fin_done) {
      launch_finish(a, st);
      L("k_finish");
    }
    H(hipEventRecord(c->ev[3], st));
    read_call();
    if (!ok) return CASK_E_DEVICE;
  }

  if (small_slots && hc->slot_overflow) {  // a chunk's rows were cut at kWalkSlotCap: redo in full
    c->full_slots_next = true;
    return scan_device_impl(c, files, nfiles, rows, file_row_offset, err, hint);
  }
  if (small_slots && hc->any_invalid) {
    // the repair path's exact chunk scans may write a chunk's full count: the rows found so far
    // move to the full stride (every chunk's count is within kWalkSlotCap), and only the chunks
    // validation flagged are scanned again
    if (!c->slots_alt.ensure((total_chunks * (uint64_t)slot_full + 1) * 16)) return CASK_E_NOMEM;
    launch_restride(a, c->slots_alt.as<uint32_t>(), slot_full, st);
    L("k_restride");
    c->slots.swap(c->slots_alt);
    a.slots = c->slots.as<uint32_t>();
    a.slot_cap = slot_full;
  }
  c->last_dense = 0;
  if (dense && !hc->any_invalid) {
    // every speculated start held: the rows are final but for the long records' checksums
    a.dense = 1;
    c->last_dense = 1;
    // (no long records left: the call block read above already waited for everything; no
    // further event or round trip)
    const bool more = !long_now && hc->long_pending;
    if (more) {
      launch_long(a, st);
      L("k_long");
      H(hipEventRecord(c->ev[4], st));
      read_call();
    }
    if (!ok) return CASK_E_DEVICE;
    float t_all = 0, t_k1 = 0, t_fin = 0, t_long = 0, t_search = 0;
    (void)hipEventElapsedTime(&t_all, c->ev[1], more ? c->ev[4] : c->ev[3]);
    float t_chase = 0;
    if (fused) {  // [1] is k_run_hash alone, [6] the run searches, [7] the chase
      (void)hipEventElapsedTime(&t_search, c->ev[1], c->ev[6]);
      (void)hipEventElapsedTime(&t_chase, c->ev[6], c->ev[7]);
      (void)hipEventElapsedTime(&t_k1, c->ev[7], c->ev[2]);
    } else {
      (void)hipEventElapsedTime(&t_k1, c->ev[1], c->ev[2]);
    }
    (void)hipEventElapsedTime(&t_fin, c->ev[2], c->ev[3]);
    if (more) (void)hipEventElapsedTime(&t_long, c->ev[3], c->ev[4]);
    c->last_ms[0] = t_all;
    c->last_ms[1] = t_k1;
    c->last_ms[2] = t_long;
    c->last_ms[3] = t_fin;
    c->last_ms[4] = 0.f;
    c->last_ms[5] = 0.f;
    c->last_ms[6] = t_search;
    c->last_ms[7] = t_chase;
    c->last_counters[0] = total_chunks;
    c->last_counters[1] = hc->nlong;
    c->last_counters[2] = c->last_counters[3] = c->last_counters[4] = 0;
    const uint64_t total = hc->total_rows;
    if (file_row_offset) {  // empty files have no chunk: they start where the next file does
      file_row_offset[nfiles] = total;
      for (uint32_t f = nfiles; f-- > 0;)
        file_row_offset[f] = fd[f].nchunks ? h_rowoff[f] : file_row_offset[f + 1];
    }
    rows->count = total;
    c->cb_zero[cbi ^ 1] = true;  // k_finish has run (and cleared the other call block)
    if (total > rows->capacity) return CASK_E_CAPACITY;
    if (err) {
      memset(err, 0, sizeof(*err));
      for (uint32_t f = 0; f < nfiles; ++f) {
        if (!h_errinv[f]) continue;
        const uint64_t d = ~(uint64_t)h_errinv[f];
        uint32_t e5[6] = {0, 0, 0, 0, 0, 0};
        launch_err_dense(a, f, d, c->err2.as<uint32_t>(), st);
        H(hipMemcpyAsync(e5, c->err2.p, 24, hipMemcpyDeviceToHost, st));
        H(hipStreamSynchronize(st));
        if (!ok) return CASK_E_DEVICE;
        err->kind = (int32_t)e5[2];
        err->file_id = files[f].file_id;
        err->pos = (uint64_t)e5[3] | ((uint64_t)e5[4] << 32);
        err->row = d;
        err->expected = hint ? 0 : e5[0];  // a hint has no checksum of its own
        err->found = e5[2] == CASK_ROW_CHECKSUM ? e5[1] : 0;
        break;
      }
    }
    return CASK_OK;
  }

  // ---- repair path ------------------------------------------------------------------------------
  auto reset = [&]() {
    H(hipMemsetAsync(a.ctr, 0, sizeof(Counters), st), "memset counters");
    H(hipMemsetAsync(d_ferr, 0xFF, 8ull * (nfiles + 1), st), "memset file_err");
    H(hipMemsetAsync(d_fbad, 0xFF, 8ull * (nfiles + 1), st), "memset first_bad");
    if (a.stamps) H(hipMemsetAsync(a.stamps, 0, 8ull * kStampWords, st));
  };
  uint64_t nlong_total = 0;  // records hashed by k_long over all passes (each pass queues only chunks it scanned)
  // validation, long records and summary after a scan of the chunks (events 2..4 when timed)
  auto post = [&](bool timed) {
    launch_validate(a, st);
    L("k_val");
    if (timed) H(hipEventRecord(c->ev[3], st));
    launch_long(a, st);
    L("k_long");
    launch_summary(a, d_sum, st);
    L("k_summary");
    if (timed) H(hipEventRecord(c->ev[4], st));
    H(hipMemcpyAsync(c->hsum.p, d_sum, sum_words * 8, hipMemcpyDeviceToHost, st), "summary D2H");
    H(hipStreamSynchronize(st), "stream sync");
    if (ok) nlong_total += ((const SummaryHead*)c->hsum.p)->nlong;
  };
  auto pass = [&]() {
    reset();
    if (hint) {  // hint bodies: the walker from the exact starts (a.runs) or from each file's start
      launch_walk_runs(a, st);
      L("k_walk_runs");
    } else {
      launch_scan_chunks(a, geo, st);
      L("k_scan_chunks");
    }
    post(false);
  };
  // (long records hashed before k_finish keep their marks: a re-scanned chunk is queued again)
  // the first scan has run (its counters are in the call block): keep its run counter's effects,
  // clear the per-file error state the validation builds
  H(hipMemsetAsync(d_ferr, 0xFF, 8ull * (nfiles + 1), st), "memset file_err");
  H(hipMemsetAsync(d_fbad, 0xFF, 8ull * (nfiles + 1), st), "memset first_bad");
  H(hipMemsetAsync(a.ctr, 0, sizeof(Counters), st), "memset counters");
  post(true);
  if (!ok) return CASK_E_DEVICE;

  uint64_t* hs = (uint64_t*)c->hsum.p;
  SummaryHead* head = (SummaryHead*)hs;
  float repair_ms = 0.f;
  uint64_t invalid_chunks = 0;
#ifdef CASK_STAMPS
  if (cask_knobs::hook("CASK_NO_REPAIR")) {  // diagnostic: keep the speculative pass for inspection
    c->dbg_spec = a.spec;
    c->dbg_exit = a.exit;
    c->dbg_count = a.count;
    c->dbg_tin = a.tin;
    c->dbg_n = total_chunks;
    float t_k1 = 0;
    (void)hipEventElapsedTime(&t_k1, c->ev[1], c->ev[2]);
    memset(c->last_ms, 0, sizeof(c->last_ms));
    c->last_ms[1] = t_k1;
    return head->any_invalid ? 1 : 0;
  }
#endif
  uint64_t local_passes = 0, walked = 0;
  std::vector<uint8_t> redo;
  std::vector<uint64_t> runs;
  H(hipEventRecord(c->ev[5], st));
  if (head->any_invalid) {
    // Repair. First, local: validation has already moved every invalid chunk's start to T[c]
    // (a.respec), which is exact for the first invalid chunk of each stretch, so exact re-scans
    // (exact=1, no search) settle isolated misses — e.g. a record longer than the window whose
    // start the search cannot verify — in one or two passes. If that does not converge, the
    // exact boundary walk from each file's first invalid chunk, then one more exact re-scan.
    // Chunks before the first invalid one keep their (validated) speculative starts.
    // A local pass re-scans only the chunks validation flagged (redo), as maximal stretches of
    // consecutive flagged chunks walked with a carry; files that were valid keep their chunk
    // table, rows and per-chunk errors (cerr), and k_long queues only chunks scanned since it last ran.
    a.exact = 1;
    static const bool sparse = cask_knobs::tune("CASK_FULL_REPAIR") == nullptr;  // diagnostic: re-scan everything
    const int max_local = cask_knobs::hook("CASK_LOCAL_REPAIRS") ? atoi(cask_knobs::hook("CASK_LOCAL_REPAIRS")) : 3;
    if (sparse) redo.resize(total_chunks);
    for (int it = 0; it < max_local && head->any_invalid; ++it) {
      if (sparse) {
        H(hipMemcpyAsync(redo.data(), a.redo, total_chunks, hipMemcpyDeviceToHost, st), "redo D2H");
        H(hipStreamSynchronize(st), "redo sync");
        if (!ok) return CASK_E_DEVICE;
        runs.clear();
        for (uint64_t g = 0; g < total_chunks;) {
          if (!redo[g]) {  // skip unflagged chunks 8 at a time
            uint64_t w;
            if (!(g & 7) && g + 8 <= total_chunks && (memcpy(&w, &redo[g], 8), w == 0)) g += 8;
            else ++g;
            continue;
          }
          const uint64_t g0 = g;
          while (g < total_chunks && redo[g]) ++g;
          runs.push_back(g0);
          runs.push_back(g);
          invalid_chunks += g - g0;
        }
        H(hipMemcpyAsync(d_runs, runs.data(), runs.size() * 8, hipMemcpyHostToDevice, st), "runs H2D");
        a.runs = d_runs;
        a.nruns_list = runs.size() / 2;
      } else {
        invalid_chunks += head->invalid_chunks;
      }
      pass();
      if (!ok) return CASK_E_DEVICE;
      ++local_passes;
    }
    if (head->any_invalid && hint) {  // every file walked whole from its first record
      walked = 1;
      invalid_chunks += total_chunks;
      runs.clear();
      for (uint32_t f = 0; f < nfiles; ++f)
        if (fd[f].nchunks) {
          runs.push_back(fd[f].first_chunk);
          runs.push_back(fd[f].first_chunk + fd[f].nchunks);
        }
      H(hipMemcpyAsync(d_runs, runs.data(), runs.size() * 8, hipMemcpyHostToDevice, st), "runs H2D");
      a.runs = d_runs;
      a.nruns_list = runs.size() / 2;
      pass();
      if (!ok) return CASK_E_DEVICE;
    } else if (head->any_invalid) {
      walked = 1;
      invalid_chunks += total_chunks;
      a.runs = nullptr;  // the walk rewrites every start from each file's first bad chunk: re-scan all
      a.nruns_list = 0;
      launch_walk(a, d_sum, st);
      L("k_walk");
      pass();
      if (!ok) return CASK_E_DEVICE;
    }
    if (head->any_invalid) {  // the exact pass must validate
      snprintf(c->last_error, sizeof(c->last_error), "exact re-scan did not validate");
      return CASK_E_DEVICE;
    }
  }
  H(hipEventRecord(c->ev[6], st));
  if (rows) {
    launch_compact(a, d_sum, st);
    L("k_compact");
  }
  H(hipEventRecord(c->ev[7], st));
  H(hipStreamSynchronize(st), "stream sync");
  if (!ok) return CASK_E_DEVICE;
  float t_all = 0, t_k1 = 0, t_long = 0, t_val = 0, t_cmp = 0;
  (void)hipEventElapsedTime(&t_k1, c->ev[1], c->ev[2]);
  (void)hipEventElapsedTime(&t_val, c->ev[2], c->ev[3]);  // with k_finish's time on a dense attempt
  (void)hipEventElapsedTime(&t_long, c->ev[3], c->ev[4]);  // with the summary (a few us)
  (void)hipEventElapsedTime(&repair_ms, c->ev[5], c->ev[6]);
  (void)hipEventElapsedTime(&t_cmp, c->ev[6], c->ev[7]);
  (void)hipEventElapsedTime(&t_all, c->ev[1], c->ev[7]);
  c->last_ms[0] = t_all;
  c->last_ms[1] = t_k1;
  c->last_ms[2] = t_long;
  c->last_ms[3] = t_val;
  c->last_ms[4] = repair_ms;
  c->last_ms[5] = t_cmp;
  c->last_ms[6] = 0.f;
  c->last_ms[7] = 0.f;
  c->last_counters[0] = total_chunks;
  c->last_counters[1] = nlong_total;
  c->last_counters[2] = invalid_chunks;
  c->last_counters[3] = local_passes;
  c->last_counters[4] = walked;

  const uint64_t* row_off = hs + head_words;
  const uint64_t* ferr_row = row_off + nfiles + 1 + 2ull * nfiles;
  const uint64_t* ferr_slot = ferr_row + nfiles;
  if (file_row_offset) memcpy(file_row_offset, row_off, 8ull * (nfiles + 1));
  if (rows) {
    rows->count = head->total_rows;
    if (head->total_rows > rows->capacity) return CASK_E_CAPACITY;
  }

  if (err) {
    memset(err, 0, sizeof(*err));
    for (uint32_t f = 0; f < nfiles; ++f) {
      if (ferr_slot[f] == kNone) continue;
      uint32_t e5[6] = {0, 0, 0, 0, 0, 0};
      launch_err_detail(a, f, ferr_slot[f], c->err2.as<uint32_t>(), st);
      H(hipMemcpyAsync(e5, c->err2.p, 24, hipMemcpyDeviceToHost, st));
      H(hipStreamSynchronize(st));
      if (!ok) return CASK_E_DEVICE;
      err->kind = (int32_t)e5[2];
      err->file_id = files[f].file_id;
      err->pos = (uint64_t)e5[3] | ((uint64_t)e5[4] << 32);
      err->row = ferr_row[f];
      err->expected = hint ? 0 : e5[0];
      err->found = e5[2] == CASK_ROW_CHECKSUM ? e5[1] : 0;
      break;
    }
  }
  return CASK_OK;
}

extern "C" int cask_parse_hints_device(cask_ctx* c, const cask_file_view* files, uint32_t nfiles, cask_rows* rows,
                                       uint64_t* file_row_offset, cask_scan_error* err) {
  return cask_abi::guard([&]() -> int {
    cask_abi::maybe_throw(c);
    if (!c || !rows) return CASK_E_INVALID_ARG;
    for (uint32_t i = 0; i < nfiles; ++i)
      if (files && !(files[i].flags & CASK_VIEW_DEVICE)) return CASK_E_INVALID_ARG;
    std::lock_guard<std::mutex> g(c->mu);
    return scan_device_impl(c, files, nfiles, rows, file_row_offset, err, true);
  });
}

extern "C" int cask_scan_device(cask_ctx* c, const cask_file_view* files, uint32_t nfiles, cask_rows* rows,
                                uint64_t* file_row_offset, cask_scan_error* err) {
  return cask_abi::guard([&]() -> int {
    cask_abi::maybe_throw(c);
    if (!c || !rows) return CASK_E_INVALID_ARG;
    for (uint32_t i = 0; i < nfiles; ++i)
      if (files && !(files[i].flags & CASK_VIEW_DEVICE)) return CASK_E_INVALID_ARG;
    std::lock_guard<std::mutex> g(c->mu);
    return scan_device_impl(c, files, nfiles, rows, file_row_offset, err);
  });
}

extern "C" int cask_scan_host(cask_ctx* c, const cask_file_view* files, uint32_t nfiles, cask_rows* rows,
                              uint64_t* file_row_offset, cask_scan_error* err) {
  return cask_abi::guard([&]() -> int {
    cask_abi::maybe_throw(c);
    if (!c || !rows || (nfiles && !files)) return CASK_E_INVALID_ARG;
    std::lock_guard<std::mutex> g(c->mu);
    if (set_dev(c)) return CASK_E_DEVICE;
    hipStream_t st = c->stream;
    // stage every file at a 256-B aligned offset of one device buffer
    std::vector<uint64_t> off(nfiles + 1, 0);
    uint64_t total = 0;
    for (uint32_t i = 0; i < nfiles; ++i) {
      off[i] = total;
      total = align_up(total + files[i].len, 256);
    }
    const uint64_t bound = cask_rows_bound(files, nfiles);
    const uint64_t rcap = std::min<uint64_t>(bound, rows->capacity ? rows->capacity : bound);
    if (!c->stage_data.ensure(total + 256)) return CASK_E_NOMEM;
    if (!c->stage_rows.ensure(rcap * 23 + 5 * 256)) return CASK_E_NOMEM;
    std::vector<cask_file_view> dv(nfiles);
    uint8_t* d = c->stage_data.as<uint8_t>();
    // Large inputs go through the pinned ring on host threads (CASK_STAGE_MIN: the smallest staged
    // input, default 64 MiB; 0 stages everything — the tests' knob)
    const char* mv = cask_knobs::hook("CASK_STAGE_MIN");
    const bool staged = total && total >= (mv ? strtoull(mv, nullptr, 10) : (64ull << 20));
    if (staged) {
      if (!c->ring) c->ring.reset(new (std::nothrow) cask_host::PinnedRing());
      if (!c->ring || !c->ring->init(c->device)) return CASK_E_NOMEM;
      if (hipStreamSynchronize(st) != hipSuccess) return CASK_E_DEVICE;  // stage_data is free
    }
    std::vector<cask_host::PinnedRing::Piece> ps;
    for (uint32_t i = 0; i < nfiles; ++i) {
      dv[i] = files[i];
      dv[i].flags = CASK_VIEW_DEVICE;
      dv[i].data = d + off[i];
      if (staged) {
        cask_host::PinnedRing::split((uint8_t*)files[i].data, d + off[i], files[i].len, ps);
      } else if (files[i].len && hipMemcpyAsync(d + off[i], files[i].data, files[i].len, hipMemcpyHostToDevice, st) != hipSuccess) {
        return CASK_E_DEVICE;
      }
    }
    if (staged && !c->ring->h2d(ps)) return CASK_E_DEVICE;
    (void)set_dev(c);  // (the calling thread's device, for the launches below)
    uint8_t* rb = c->stage_rows.as<uint8_t>();
    cask_rows dr{};
    dr.capacity = rcap;
    dr.pos = (uint64_t*)rb;
    dr.seq = (uint64_t*)(rb + align_up(rcap * 8, 256));
    dr.vsz = (uint32_t*)(rb + 2 * align_up(rcap * 8, 256));
    dr.ksz = (uint16_t*)(rb + 2 * align_up(rcap * 8, 256) + align_up(rcap * 4, 256));
    dr.status = (uint8_t*)(rb + 2 * align_up(rcap * 8, 256) + align_up(rcap * 4, 256) + align_up(rcap * 2, 256));
    int rc = scan_device_impl(c, dv.data(), nfiles, &dr, file_row_offset, err);
    rows->count = dr.count;
    if (rc != CASK_OK) return rc;
    if (dr.count > rows->capacity) return CASK_E_CAPACITY;
    const uint64_t n = dr.count;
    bool ok = true;
    auto H = [&](hipError_t e) { ok = ok && (e == hipSuccess); };
    if (n && staged) {  // the five row arrays through the ring too
      H(hipStreamSynchronize(st));
      std::vector<cask_host::PinnedRing::Piece> rp;
      cask_host::PinnedRing::split((uint8_t*)rows->pos, (uint8_t*)dr.pos, n * 8, rp);
      cask_host::PinnedRing::split((uint8_t*)rows->seq, (uint8_t*)dr.seq, n * 8, rp);
      cask_host::PinnedRing::split((uint8_t*)rows->vsz, (uint8_t*)dr.vsz, n * 4, rp);
      cask_host::PinnedRing::split((uint8_t*)rows->ksz, (uint8_t*)dr.ksz, n * 2, rp);
      cask_host::PinnedRing::split(rows->status, dr.status, n, rp);
      if (ok && !c->ring->d2h(rp)) ok = false;
      return ok ? CASK_OK : CASK_E_DEVICE;
    }
    if (n) {
      H(hipMemcpyAsync(rows->pos, dr.pos, n * 8, hipMemcpyDeviceToHost, st));
      H(hipMemcpyAsync(rows->seq, dr.seq, n * 8, hipMemcpyDeviceToHost, st));
      H(hipMemcpyAsync(rows->vsz, dr.vsz, n * 4, hipMemcpyDeviceToHost, st));
      H(hipMemcpyAsync(rows->ksz, dr.ksz, n * 2, hipMemcpyDeviceToHost, st));
      H(hipMemcpyAsync(rows->status, dr.status, n, hipMemcpyDeviceToHost, st));
    }
    H(hipStreamSynchronize(st));
    return ok ? CASK_OK : CASK_E_DEVICE;
  });
}

extern "C" int cask_copy(cask_ctx* c, void* dst, const void* src, uint64_t bytes) {
  return cask_abi::guard([&]() -> int {
    if (!c || (bytes && (!dst || !src))) return CASK_E_INVALID_ARG;
    std::lock_guard<std::mutex> g(c->mu);
    if (set_dev(c)) return CASK_E_DEVICE;
    if (bytes && (hipMemcpyAsync(dst, src, bytes, hipMemcpyDefault, c->stream) != hipSuccess ||
                  hipStreamSynchronize(c->stream) != hipSuccess))
      return CASK_E_DEVICE;
    return CASK_OK;
  });
}

extern "C" int cask_hints_device(cask_ctx* c, const cask_file_view* files, uint32_t nfiles, const cask_rows* rows,
                                 const uint64_t* file_row_offset, uint8_t* out, uint64_t cap, uint64_t* file_hint_offset) {
  return cask_abi::guard([&]() -> int {
    cask_abi::maybe_throw(c);
    if (!c || !rows || !file_hint_offset || (nfiles && (!files || !file_row_offset))) return CASK_E_INVALID_ARG;
    if (rows->count && (!rows->pos || !rows->seq || !rows->vsz || !rows->ksz || !rows->status)) return CASK_E_INVALID_ARG;
    for (uint32_t i = 0; i < nfiles; ++i)
      if (!(files[i].flags & CASK_VIEW_DEVICE) || (files[i].len && !files[i].data)) return CASK_E_INVALID_ARG;
    if (file_row_offset[nfiles] != rows->count) return CASK_E_INVALID_ARG;
    std::lock_guard<std::mutex> g(c->mu);
    if (set_dev(c)) return CASK_E_DEVICE;
    if (!c->kd && !(c->kd = kd_scratch_create())) return CASK_E_NOMEM;
    std::vector<FileDesc> fd(nfiles + 1);
    for (uint32_t i = 0; i < nfiles; ++i) fd[i] = FileDesc{files[i].data, files[i].len, 0, 0, 0, 0};
    if (rows->count <= (uint64_t)INT32_MAX)
      return hint_pack(c->kd, fd.data(), nfiles, file_row_offset, rows->pos, rows->seq, rows->vsz, rows->ksz,
                       rows->status, rows->count, out, out ? cap : 0, file_hint_offset, c->stream);
    // more rows than one device scan takes (an int count): groups of whole files, bodies back to back
    uint64_t at = 0;  // bytes of the bodies so far
    int rc = CASK_OK;
    for (uint32_t f0 = 0; f0 < nfiles;) {
      const uint64_t r0 = file_row_offset[f0];
      uint32_t f1 = f0 + 1;
      while (f1 < nfiles && file_row_offset[f1 + 1] - r0 <= (uint64_t)INT32_MAX) ++f1;
      const uint64_t n = file_row_offset[f1] - r0;
      if (n > (uint64_t)INT32_MAX) return CASK_E_CAPACITY;  // one file of more than 2^31 records
      std::vector<uint64_t> ro(f1 - f0 + 1), fs(f1 - f0 + 1);
      for (uint32_t f = f0; f <= f1; ++f) ro[f - f0] = file_row_offset[f] - r0;
      const bool room = out && at <= cap;
      const int st = hint_pack(c->kd, fd.data() + f0, f1 - f0, ro.data(), rows->pos + r0, rows->seq + r0, rows->vsz + r0,
                               rows->ksz + r0, rows->status + r0, n, room ? out + at : nullptr, room ? cap - at : 0,
                               fs.data(), c->stream);
      if (st != CASK_OK && st != CASK_E_CAPACITY) return st;
      if (st == CASK_E_CAPACITY) rc = CASK_E_CAPACITY;
      for (uint32_t f = f0; f < f1; ++f) file_hint_offset[f] = at + fs[f - f0];
      at += fs[f1 - f0];
      f0 = f1;
    }
    file_hint_offset[nfiles] = at;
    if (out && at > cap) rc = CASK_E_CAPACITY;
    return rc;
  });
}

// The shard block of hint-file bodies (the hint fast path on the multi-GPU replay): rows as
// cask_parse_hints_device left them; their pos is rewritten to the entry positions.
extern "C" int cask_shard_keydir_hints(cask_ctx* c, const cask_file_view* files, uint32_t nfiles, cask_rows* rows,
                                       const uint64_t* file_row_offset, const void** block, uint64_t* bytes) {
  return cask_abi::guard([&]() -> int {
    cask_abi::maybe_throw(c);
    if (!c || !rows || !block || !bytes || (nfiles && (!files || !file_row_offset))) return CASK_E_INVALID_ARG;
    if (rows->count && (!rows->pos || !rows->seq || !rows->vsz || !rows->ksz)) return CASK_E_INVALID_ARG;
    for (uint32_t i = 0; i < nfiles; ++i)
      if (!(files[i].flags & CASK_VIEW_DEVICE) || (files[i].len && !files[i].data)) return CASK_E_INVALID_ARG;
    if (file_row_offset[nfiles] != rows->count) return CASK_E_INVALID_ARG;
    std::lock_guard<std::mutex> g(c->mu);
    if (set_dev(c)) return CASK_E_DEVICE;
    if (!c->kd && !(c->kd = kd_scratch_create())) return CASK_E_NOMEM;
    if (!c->keyat.ensure(8 * (rows->count + 1))) return CASK_E_NOMEM;
    std::vector<FileDesc> fd(nfiles + 1);
    std::vector<uint32_t> ids(nfiles + 1, 0);
    for (uint32_t i = 0; i < nfiles; ++i) {
      fd[i] = FileDesc{files[i].data, files[i].len, 0, 0, 0, 0};
      ids[i] = files[i].file_id;
    }
    uint64_t* key_at = c->keyat.as<uint64_t>();
    int rc = hint_entries(c->kd, fd.data(), nfiles, file_row_offset, rows->count, rows->pos, key_at, c->stream);
    void* out = nullptr;
    uint64_t nb = 0;
    if (!rc)
      rc = kd_build(c->kd, fd.data(), ids.data(), nfiles, file_row_offset, rows->pos, rows->seq, rows->vsz, rows->ksz,
                    rows->count, c->stream, &out, &nb, key_at);
    if (rc) {
      snprintf(c->last_error, sizeof(c->last_error), "cask_shard_keydir_hints: %s", rc == CASK_E_NOMEM ? "out of memory" : "device");
      return rc;
    }
    *block = out;
    *bytes = nb;
    return CASK_OK;
  });
}

extern "C" int cask_shard_keydir(cask_ctx* c, const cask_file_view* files, uint32_t nfiles, const cask_rows* rows,
                                 const uint64_t* file_row_offset, const void** block, uint64_t* bytes) {
  return cask_abi::guard([&]() -> int {
    cask_abi::maybe_throw(c);
    if (!c || !rows || !block || !bytes || (nfiles && (!files || !file_row_offset))) return CASK_E_INVALID_ARG;
    if (rows->count && (!rows->pos || !rows->seq || !rows->vsz || !rows->ksz)) return CASK_E_INVALID_ARG;
    for (uint32_t i = 0; i < nfiles; ++i)
      if (!(files[i].flags & CASK_VIEW_DEVICE) || (files[i].len && !files[i].data)) return CASK_E_INVALID_ARG;
    if (file_row_offset[nfiles] != rows->count) return CASK_E_INVALID_ARG;
    std::lock_guard<std::mutex> g(c->mu);
    if (set_dev(c)) return CASK_E_DEVICE;
    if (!c->kd && !(c->kd = kd_scratch_create())) return CASK_E_NOMEM;
    std::vector<FileDesc> fd(nfiles + 1);
    std::vector<uint32_t> ids(nfiles + 1, 0);
    for (uint32_t i = 0; i < nfiles; ++i) {
      fd[i] = FileDesc{files[i].data, files[i].len, 0, 0, 0, 0};
      ids[i] = files[i].file_id;
    }
    void* out = nullptr;
    uint64_t nb = 0;
    const int rc = kd_build(c->kd, fd.data(), ids.data(), nfiles, file_row_offset, rows->pos, rows->seq, rows->vsz,
                            rows->ksz, rows->count, c->stream, &out, &nb);
    if (rc) {
      snprintf(c->last_error, sizeof(c->last_error), "cask_shard_keydir: %s", rc == CASK_E_NOMEM ? "out of memory" : "device");
      return rc;
    }
    *block = out;
    *bytes = nb;
    return CASK_OK;
  });
}

extern "C" int cask_keydir_partition(cask_ctx* c, const void* block, uint64_t bytes, uint32_t nparts, const void** parts,
                                     uint64_t* part_off) {
  return cask_abi::guard([&]() -> int {
    cask_abi::maybe_throw(c);
    if (!c || !block || !parts || !part_off || nparts < 1 || nparts > cask_kd::kMaxParts) return CASK_E_INVALID_ARG;
    std::lock_guard<std::mutex> g(c->mu);
    if (set_dev(c)) return CASK_E_DEVICE;
    if (!c->kd && !(c->kd = kd_scratch_create())) return CASK_E_NOMEM;
    if (cask_abi::take_inject(c, cask_abi::kInjPartition)) return CASK_E_NOMEM;
    void* out = nullptr;
    const int rc = kd_partition(c->kd, block, bytes, nparts, c->stream, &out, part_off);
    if (rc) {
      snprintf(c->last_error, sizeof(c->last_error), "cask_keydir_partition: %s",
               rc == CASK_E_NOMEM ? "out of memory" : rc == CASK_E_INVALID_ARG ? "not a keydir block" : "device");
      return rc;
    }
    *parts = out;
    return CASK_OK;
  });
}

extern "C" int cask_encode_synthetic_device(cask_ctx* c, uint64_t nrec, const uint64_t* off, const uint64_t* seq,
                                            const uint16_t* ksz, const uint32_t* vsz_raw, const uint64_t* key_id,
                                            uint64_t value_seed, uint8_t* out) {
  return cask_abi::guard([&]() -> int {
    if (!c || (nrec && (!off || !seq || !ksz || !vsz_raw || !key_id || !out))) return CASK_E_INVALID_ARG;
    std::lock_guard<std::mutex> g(c->mu);
    if (set_dev(c)) return CASK_E_DEVICE;
    launch_encode_synth(nrec, off, seq, ksz, vsz_raw, key_id, value_seed, out, c->stream);
    launch_encode_checksum(nrec, off, ksz, vsz_raw, out, c->stream);
    if (hipStreamSynchronize(c->stream) != hipSuccess || hipGetLastError() != hipSuccess) return CASK_E_DEVICE;
    return CASK_OK;
  });
}

extern "C" int cask_encode_device(cask_ctx* c, uint64_t nrec, const uint64_t* off, const uint64_t* seq,
                                  const uint16_t* ksz, const uint32_t* vsz_raw, const uint8_t* keys,
                                  const uint64_t* key_off, const uint8_t* vals, const uint64_t* val_off,
                                  uint8_t* out) {
  return cask_abi::guard([&]() -> int {
    cask_abi::maybe_throw(c);
    if (!c || (nrec && (!off || !seq || !ksz || !vsz_raw || !keys || !key_off || !out))) return CASK_E_INVALID_ARG;
    std::lock_guard<std::mutex> g(c->mu);
    if (set_dev(c)) return CASK_E_DEVICE;
    launch_encode(nrec, off, seq, ksz, vsz_raw, keys, key_off, vals, val_off, out, c->stream);
    launch_encode_checksum(nrec, off, ksz, vsz_raw, out, c->stream);
    if (hipStreamSynchronize(c->stream) != hipSuccess || hipGetLastError() != hipSuccess) return CASK_E_DEVICE;
    return CASK_OK;
  });
}

extern "C" int cask_read_entries_device(cask_ctx* c, const uint8_t* const* srcs, const uint64_t* src_len, uint32_t nsrc,
                                        const uint32_t* src, const uint64_t* pos, uint64_t n, uint64_t* len,
                                        uint8_t* status, uint32_t* expected, uint32_t* found) {
  return cask_abi::guard([&]() -> int {
    cask_abi::maybe_throw(c);
    if (!c || (n && (!srcs || !src_len || !src || !pos || !len || !status || !expected || !found))) return CASK_E_INVALID_ARG;
    for (uint64_t r = 0; r < n; ++r)
      if (src[r] >= nsrc) return CASK_E_INVALID_ARG;
    std::lock_guard<std::mutex> g(c->mu);
    if (set_dev(c)) return CASK_E_DEVICE;
    if (!n) return CASK_OK;
    const size_t a8 = align_up(8 * n, 256), a4 = align_up(4 * n, 256), a1 = align_up(n, 256), as = align_up(8ull * nsrc, 256);
    if (!c->gather.ensure(4 * a8 + 3 * a4 + a1 + 2 * as)) return CASK_E_NOMEM;
    uint8_t* b = c->gather.as<uint8_t>();
    uint64_t* d_pos = (uint64_t*)b;
    uint64_t* d_len = (uint64_t*)(b + a8);
    uint32_t* d_src = (uint32_t*)(b + 2 * a8);
    uint32_t* d_exp = (uint32_t*)(b + 2 * a8 + a4);
    uint32_t* d_fnd = (uint32_t*)(b + 2 * a8 + 2 * a4);
    uint8_t* d_st = b + 2 * a8 + 3 * a4;
    const uint8_t** d_srcs = (const uint8_t**)(b + 2 * a8 + 3 * a4 + a1);
    uint64_t* d_slen = (uint64_t*)(b + 2 * a8 + 3 * a4 + a1 + as);
    hipStream_t st = c->stream;
    bool ok = true;
    auto H = [&](hipError_t e) { ok = ok && e == hipSuccess; };
    H(hipMemcpyAsync(d_pos, pos, 8 * n, hipMemcpyHostToDevice, st));
    H(hipMemcpyAsync(d_src, src, 4 * n, hipMemcpyHostToDevice, st));
    H(hipMemcpyAsync(d_srcs, srcs, 8ull * nsrc, hipMemcpyHostToDevice, st));
    H(hipMemcpyAsync(d_slen, src_len, 8ull * nsrc, hipMemcpyHostToDevice, st));
    launch_read_entries(d_pos, d_src, n, d_srcs, d_slen, d_len, d_st, d_exp, d_fnd, st);
    H(hipGetLastError());
    H(hipMemcpyAsync(len, d_len, 8 * n, hipMemcpyDeviceToHost, st));
    H(hipMemcpyAsync(status, d_st, n, hipMemcpyDeviceToHost, st));
    H(hipMemcpyAsync(expected, d_exp, 4 * n, hipMemcpyDeviceToHost, st));
    H(hipMemcpyAsync(found, d_fnd, 4 * n, hipMemcpyDeviceToHost, st));
    H(hipStreamSynchronize(st));
    return ok ? CASK_OK : CASK_E_DEVICE;
  });
}

#ifdef CASK_STAMPS
// Diagnostic build only: per-phase cycle sums of the last k_scan_chunks launch.
extern "C" int cask_debug_stamps(cask_ctx* c, uint64_t* out16) {
  if (!c || !c->stamps.p) return CASK_E_INVALID_ARG;
  if (hipMemcpy(out16, c->stamps.p, 16 * 8, hipMemcpyDeviceToHost) != hipSuccess) return CASK_E_DEVICE;
  return CASK_OK;
}
// Diagnostic build only: k_run_hash's per-wave start/end real times (2 per wave, kStampWaves waves).
extern "C" int cask_debug_wave_stamps(cask_ctx* c, uint64_t* out, uint64_t n) {
  if (!c || !c->stamps.p || n > 2ull * kStampWaves) return CASK_E_INVALID_ARG;
  if (hipMemcpy(out, (uint8_t*)c->stamps.p + 16 * 8, n * 8, hipMemcpyDeviceToHost) != hipSuccess) return CASK_E_DEVICE;
  return CASK_OK;
}
// Diagnostic build only: k_run_hash's per-wave time its runs ran out (kStampWaves words).
extern "C" int cask_debug_dry_stamps(cask_ctx* c, uint64_t* out, uint64_t n) {
  if (!c || !c->stamps.p || n > kStampWaves) return CASK_E_INVALID_ARG;
  if (hipMemcpy(out, (uint8_t*)c->stamps.p + kStampDry * 8, n * 8, hipMemcpyDeviceToHost) != hipSuccess)
    return CASK_E_DEVICE;
  return CASK_OK;
}
// Diagnostic build only: k_walk_search's per-search records (start, end real time, windows, wave).
extern "C" int cask_debug_search_stamps(cask_ctx* c, uint64_t* out, uint64_t n) {
  if (!c || !c->stamps.p || n > 4ull * kStampRuns) return CASK_E_INVALID_ARG;
  if (hipMemcpy(out, (uint8_t*)c->stamps.p + (16 + 2ull * kStampWaves) * 8, n * 8, hipMemcpyDeviceToHost) != hipSuccess)
    return CASK_E_DEVICE;
  return CASK_OK;
}
// Diagnostic build only: per-chunk spec / exit / tin / count of the last (unrepaired) pass.
extern "C" int cask_debug_chunks(cask_ctx* c, uint64_t* spec, uint64_t* exitv, uint64_t* tin, uint32_t* count, uint64_t n) {
  if (!c || !c->dbg_spec || n > c->dbg_n) return CASK_E_INVALID_ARG;
  const bool ok = hipMemcpy(spec, c->dbg_spec, n * 8, hipMemcpyDeviceToHost) == hipSuccess &&
                  hipMemcpy(exitv, c->dbg_exit, n * 8, hipMemcpyDeviceToHost) == hipSuccess &&
                  hipMemcpy(tin, c->dbg_tin, n * 8, hipMemcpyDeviceToHost) == hipSuccess &&
                  hipMemcpy(count, c->dbg_count, n * 4, hipMemcpyDeviceToHost) == hipSuccess;
  return ok ? CASK_OK : CASK_E_DEVICE;
}
#endif
