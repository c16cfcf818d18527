// Keydir rows of one shard for the multi-GPU replay (Cask::open, cask.rs:346-382 with
// Index::update, cask.rs:60-90, folded per key).
//
// A rank scans a contiguous range of data files. Its rows are grouped by key on the device: a
// 64-bit hash of the key bytes per row, a stable radix sort of (hash, row) and segments of equal
// hash. Per key (one thread walks a segment):
//  * keydir: only the suffix-strict maxima of the key's records in the shard — records with a
//    larger sequence than every later record of the key — can decide the keydir after the whole
//    replay, so only they are sent (kKept). With unique keys every row is one.
//  * stats (stats.rs): Index::update adds one entry per put and removes each put that is not the
//    key's final entry, so per file entries = puts and dead = puts - live (live from the final
//    keydir, on rank 0): the shard sends per-file put counts and bytes. What is left are stale
//    tombstones (an occupant with a larger sequence: add + remove of the tombstone itself). Whether a
//    tombstone is stale depends on the key's entry when it arrives, a function of the entry
//    entering the shard; composing the per-record maps (put a: S -> max(S, a); tombstone b:
//    S -> S > b ? S : vacant) gives, per tombstone, "stale always" (counted here) or "stale iff
//    the entering entry's sequence is > T" (kCond, resolved on rank 0 against its keydir).
//  * keys whose hash collides with another key's are sent whole (kRaw) and folded record by record.
// The result is exact, keydir and stats, whatever the distribution of keys over shards.
#include <hipcub/hipcub.hpp>

#include "device_util.h"
#include "keydir_format.h"
#include "knobs.h"

namespace cask_dev {

using namespace cask_kd;

struct KdArgs {
  const FileDesc* files;
  const uint32_t* file_ids;
  const uint64_t* row_off;  // nfiles + 1: first dense row of each file
  uint32_t nfiles;
  uint32_t pad;
  const uint64_t* pos;
  const uint64_t* seq;
  const uint32_t* vsz;
  const uint16_t* ksz;
  uint64_t n;
  uint64_t* h;        // key hash per row
  uint32_t* idx;      // row index
  uint32_t* fidx;     // file index per row
  uint64_t* hs;       // sorted hashes
  uint32_t* is;       // rows in sorted order
  uint8_t* head;      // sorted position starts a segment
  uint8_t* kind;      // per sorted position: bit 0 kKept, bit 1 kCond, bit 2 kRaw
  uint64_t* tval;     // per sorted position: kCond threshold + 1
  uint64_t* ecnt;     // per sorted position: records emitted
  uint64_t* ekey;     // ... and their key bytes
  uint64_t* eoff;     // exclusive sums
  uint64_t* koff;
  uint32_t* seg;      // segment starts
  // per sorted position i, row is[i]'s fields (k_kd_gather): what k_kd_segs and k_kd_write read,
  // in segment order instead of one scattered load per field per record
  uint64_t* sseq;
  uint32_t* svsz;
  uint32_t* sf;       // file index
  uint16_t* sksz;
  u32x4* skey;        // the key's first 16 bytes, zero-filled past its end
  // per row, in row order (k_kd_hash, written as it reads the rows): (seq lo, seq hi, vsz, file
  // index) and the key's first 16 bytes — two 16-B loads per row for k_kd_gather instead of five
  // scattered fields and a byte loop over the key
  u32x4* rfld;
  u32x4* rkey;
  uint32_t* nseg;
  uint64_t* fstat;    // per file: puts, put_bytes, stale, stale_bytes
  unsigned long long* tot;  // [0] max seq + 1, [1] records, [2] key bytes
  uint8_t* out;       // the block
  uint64_t rec_at, key_at;
  const uint64_t* key_at_row;  // per row: offset of its key in its file's bytes (null: pos + 18)
  uint64_t hmask;     // the key hash's bits that group rows (all but under CASK_KD_HASH_BITS)
};

// key_hash: keydir_format.h (shared with the host's partition and owner lookups)

__device__ __forceinline__ uint32_t row_file(const KdArgs& a, uint64_t d) {
  uint32_t lo = 0, hi = a.nfiles;  // last f with row_off[f] <= d
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (a.row_off[mid] <= d) lo = mid; else hi = mid;
  }
  return lo;
}

// A row's key: at pos + 18 of a data file, or at key_at[d] of its file's bytes (a hint body).
__device__ __forceinline__ const uint8_t* row_key(const KdArgs& a, uint64_t d, uint32_t f) {
  return a.files[f].data + (a.key_at_row ? a.key_at_row[d] : a.pos[d] + 18);
}

// Hash every row's key; per-file put counts and bytes, max sequence.
__global__ __launch_bounds__(256) void k_kd_hash(KdArgs a) {
  const uint32_t lane = threadIdx.x & 63;
  unsigned long long mx = 0;
  for (uint64_t d0 = blockIdx.x * 256ull; d0 < a.n; d0 += (uint64_t)gridDim.x * 256ull) {
    const uint64_t d = d0 + threadIdx.x;
    const bool in = d < a.n;
    uint32_t f = 0;
    unsigned long long put = 0, pb = 0;
    if (in) {
      f = row_file(a, d);
      const uint32_t k = a.ksz[d], v = a.vsz[d];
      const uint8_t* kp = row_key(a, d, f);
      // the key's first 16 bytes from the aligned dwords that hold them (a dword read past the key
      // stays inside the dword of its last byte), zero past its end; a key of at most 16 bytes is
      // hashed from them (key_hash's words), a longer one by key_hash itself
      uint32_t w[4] = {0u, 0u, 0u, 0u};
      const uint32_t m = k < 16u ? k : 16u;
      if (m) {
        const uint32_t sh = (uint32_t)((uintptr_t)kp & 3), nd = (sh + m + 3) >> 2;
        const uint32_t* q = (const uint32_t*)((uintptr_t)kp - sh);
        uint32_t x[5];
#pragma unroll
        for (uint32_t j = 0; j < 5; ++j) x[j] = j < nd ? q[j] : 0u;
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j) {
          const uint32_t b0 = 4 * j;  // key bytes b0..b0+3
          const uint32_t v4 = fun(x[j], x[j + 1], sh);
          w[j] = b0 >= m ? 0u : m - b0 >= 4 ? v4 : v4 & ((1u << (8 * (m - b0))) - 1u);
        }
      }
      uint64_t hk;
      if (k <= 16) {
        const uint64_t w0 = (uint64_t)w[0] | ((uint64_t)w[1] << 32), w1 = (uint64_t)w[2] | ((uint64_t)w[3] << 32);
        uint64_t hh = 0x9E3779B97F4A7C15ull ^ ((uint64_t)k * 0xD6E8FEB86659FD93ull), t = w0;
        if (k >= 8) {
          hh = mix64(hh ^ w0);
          t = w1;
          if (k >= 16) {
            hh = mix64(hh ^ w1);
            t = 0;
          }
        }
        hk = mix64(hh ^ t ^ 0xA0761D6478BD642Full);
      } else {
        hk = key_hash(kp, k);
      }
      a.h[d] = hk & a.hmask;
      a.idx[d] = (uint32_t)d;
      a.fidx[d] = f;
      const uint64_t sq = a.seq[d];
      a.rfld[d] = u32x4{(uint32_t)sq, (uint32_t)(sq >> 32), v, f};
      a.rkey[d] = u32x4{w[0], w[1], w[2], w[3]};
      const unsigned long long s1 = (unsigned long long)sq + 1;
      mx = mx > s1 ? mx : s1;
      if (v != 0xFFFFFFFFu) {
        put = 1;
        pb = 18ull + k + v;
      }
    }
    // per-file sums: one atomic per wave when the wave's rows are all of one file (rows are in file order)
    const uint32_t f0 = __shfl(f, 0, 64);
    if (__all(!in || f == f0)) {
      for (int o = 32; o; o >>= 1) {
        put += __shfl_xor(put, o, 64);
        pb += __shfl_xor(pb, o, 64);
      }
      if (lane == 0 && put) {
        atomicAdd((unsigned long long*)&a.fstat[4ull * f0], put);
        atomicAdd((unsigned long long*)&a.fstat[4ull * f0 + 1], pb);
      }
    } else if (put) {
      atomicAdd((unsigned long long*)&a.fstat[4ull * f], put);
      atomicAdd((unsigned long long*)&a.fstat[4ull * f + 1], pb);
    }
  }
  for (int o = 32; o; o >>= 1) {
    const unsigned long long y = __shfl_xor(mx, o, 64);
    mx = mx > y ? mx : y;
  }
  if (lane == 0 && mx) atomicMax(&a.tot[0], mx);
}

__global__ __launch_bounds__(256) void k_kd_heads(KdArgs a) {
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < a.n; i += (uint64_t)gridDim.x * 256ull)
    a.head[i] = (i == 0 || a.hs[i] != a.hs[i - 1]) ? 1 : 0;
}

// Every row's fields in sorted order (a thread per sorted position: independent scattered loads,
// many in flight), the key's first 16 bytes with them: two 16-B loads of k_kd_hash's packed rows.
__global__ __launch_bounds__(256) void k_kd_gather(KdArgs a) {
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < a.n; i += (uint64_t)gridDim.x * 256ull) {
    const uint64_t d = a.is[i];
    const u32x4 r = a.rfld[d];
    a.sseq[i] = (uint64_t)r.x | ((uint64_t)r.y << 32);
    a.svsz[i] = r.z;
    a.sf[i] = r.w;
    a.sksz[i] = a.ksz[d];
    a.skey[i] = a.rkey[d];
  }
}

// Sorted positions i0 and i1 hold the same key: sizes and first 16 bytes from the gathered arrays,
// the rest of a longer key from the files.
__device__ __forceinline__ bool same_key(const KdArgs& a, uint64_t i0, uint64_t i1) {
  const uint32_t k = a.sksz[i0];
  if (a.sksz[i1] != k) return false;
  const u32x4 x = a.skey[i0], y = a.skey[i1];
  if (x.x != y.x || x.y != y.y || x.z != y.z || x.w != y.w) return false;
  if (k <= 16) return true;
  const uint8_t* p = row_key(a, a.is[i0], a.sf[i0]);
  const uint8_t* q = row_key(a, a.is[i1], a.sf[i1]);
  for (uint32_t j = 16; j < k; ++j)
    if (p[j] != q[j]) return false;
  return true;
}

// One thread per segment (records of one key hash, in replay order): what each record emits.
__global__ __launch_bounds__(256) void k_kd_segs(KdArgs a) {
  const uint32_t ns = *a.nseg;
  for (uint64_t j = blockIdx.x * 256ull + threadIdx.x; j < ns; j += (uint64_t)gridDim.x * 256ull) {
    const uint64_t s = a.seg[j], e = (j + 1 < ns) ? a.seg[j + 1] : a.n;
    bool raw = false;
    for (uint64_t i = s + 1; i < e && !raw; ++i) raw = !same_key(a, s, i);
    if (raw) {  // a 64-bit collision between different keys: every record, folded one by one
      for (uint64_t i = s; i < e; ++i) {
        a.kind[i] = 4;
        a.ecnt[i] = 1;
        a.ekey[i] = a.sksz[i];
      }
      continue;
    }
    // keydir: suffix-strict maxima (sequence + 1 > every later record's)
    unsigned long long later = 0;
    for (uint64_t i = e; i-- > s;) {
      const unsigned long long q = (unsigned long long)a.sseq[i] + 1;
      a.kind[i] = q > later ? 1 : 0;
      later = later > q ? later : q;
    }
    // stats: the key's entry after the records so far, as a function of the entry x entering the
    // shard (sequence + 1, 0 = vacant): x > L ? max(x, A) : C
    unsigned long long L = 0, A = 0, C = 0;
    for (uint64_t i = s; i < e; ++i) {
      const unsigned long long q = (unsigned long long)a.sseq[i] + 1;
      uint8_t kd = a.kind[i];
      if (a.svsz[i] != 0xFFFFFFFFu) {
        A = A > q ? A : q;
        C = C > q ? C : q;
      } else {
        if (C > q) {  // stale whatever entered the shard
          const uint32_t f = a.sf[i];
          atomicAdd((unsigned long long*)&a.fstat[4ull * f + 2], 1ull);
          atomicAdd((unsigned long long*)&a.fstat[4ull * f + 3], 18ull + a.sksz[i]);
        } else {      // stale iff x > T
          kd |= 2;
          a.tval[i] = A > q ? L : (L > q ? L : q);
        }
        if (A > q) C = C > q ? C : 0;
        else {
          L = L > q ? L : q;
          C = 0;
        }
      }
      a.kind[i] = kd;
      const uint32_t m = (kd & 1) + ((kd >> 1) & 1);
      a.ecnt[i] = m;
      a.ekey[i] = (uint64_t)m * a.sksz[i];
    }
  }
}

__global__ void k_kd_totals(KdArgs a) {
  if (threadIdx.x || blockIdx.x || !a.n) return;
  a.tot[1] = a.eoff[a.n - 1] + a.ecnt[a.n - 1];
  a.tot[2] = a.koff[a.n - 1] + a.ekey[a.n - 1];
}

__device__ __forceinline__ void kd_emit(const KdArgs& a, uint64_t r, uint64_t ko, uint64_t i, uint64_t d, uint8_t kind,
                                        uint64_t seq) {
  ShardRec* rec = (ShardRec*)(a.out + a.rec_at) + r;
  const uint32_t f = a.sf[i];
  ShardRec x;
  x.pos = a.pos[d];
  x.seq = seq;
  x.file_id = a.file_ids[f];
  x.vsz = a.svsz[i];
  x.ksz = a.sksz[i];
  x.kind = kind;
  x.pad0 = 0;
  x.pad1 = 0;
  *rec = x;
  uint8_t* o = a.out + a.key_at + ko;
  if (x.ksz <= 16) {  // (the key's bytes are in its gathered prefix: no load from the files)
    const u32x4 w = a.skey[i];
    const uint32_t ww[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
    for (uint32_t j = 0; j < 16; ++j)  // (unrolled: ww stays in registers)
      if (j < x.ksz) o[j] = (uint8_t)(ww[j >> 2] >> (8 * (j & 3)));
    return;
  }
  const uint8_t* k = row_key(a, d, f);
  for (uint32_t j = 0; j < x.ksz; ++j) o[j] = k[j];
}

__global__ __launch_bounds__(256) void k_kd_write(KdArgs a) {
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < a.n; i += (uint64_t)gridDim.x * 256ull) {
    const uint8_t kd = a.kind[i];
    if (!kd) continue;
    const uint64_t d = a.is[i];
    uint64_t r = a.eoff[i], ko = a.koff[i];
    if (kd & 4) {
      kd_emit(a, r, ko, i, d, kRaw, a.sseq[i]);
      continue;
    }
    if (kd & 2) {  // the threshold first: rank 0 resolves it before it folds the shard's rows
      kd_emit(a, r, ko, i, d, kCond, a.tval[i]);
      ++r;
      ko += a.sksz[i];
    }
    if (kd & 1) kd_emit(a, r, ko, i, d, kKept, a.sseq[i]);
  }
}

// Header and per-file stats into the block.
__global__ void k_kd_header(KdArgs a, uint64_t rows_in, uint64_t fstat_at, uint64_t bytes) {
  if (blockIdx.x) return;
  if (threadIdx.x == 0) {
    ShardHeader hd{};
    hd.magic = kMagic;
    hd.version = kVersion;
    hd.nrec = a.n ? a.tot[1] : 0;
    hd.key_bytes = a.n ? a.tot[2] : 0;
    hd.nfiles = a.nfiles;
    hd.max_seq_p1 = a.tot[0];
    hd.rows_in = rows_in;
    hd.bytes = bytes;
    *(ShardHeader*)a.out = hd;
  }
  const uint64_t end = a.key_at + (a.n ? a.tot[2] : 0);  // zero the padding to the 8-B boundary
  if (threadIdx.x < bytes - end) a.out[end + threadIdx.x] = 0;
  for (uint32_t f = threadIdx.x; f < a.nfiles; f += blockDim.x) {
    ShardFileStat st{};
    st.file_id = a.file_ids[f];
    st.puts = a.fstat[4ull * f];
    st.put_bytes = a.fstat[4ull * f + 1];
    st.stale = a.fstat[4ull * f + 2];
    st.stale_bytes = a.fstat[4ull * f + 3];
    ((ShardFileStat*)(a.out + fstat_at))[f] = st;
  }
}

// ------------------------------------------------------------------------------------------
// Host side of the pipeline (called from scan_runtime.cpp with the context's scratch).
// ------------------------------------------------------------------------------------------
static inline hipStream_t S(void* s) { return (hipStream_t)s; }
static inline uint64_t al(uint64_t x) { return (x + 255) & ~255ull; }

struct KdScratch {
  void* p = nullptr;
  size_t cap = 0;
  void* out = nullptr;
  size_t out_cap = 0;
  void* part = nullptr;  // kd_partition's output (the block it splits may be `out`)
  size_t part_cap = 0;
  ~KdScratch() {
    if (p) (void)hipFree(p);
    if (out) (void)hipFree(out);
    if (part) (void)hipFree(part);
  }
  // The per-row scratch of a large build (~96 B per row: 23 GB for configs[3]'s 237 M rows) goes back
  // once the block is written; the block itself stays until the next call.
  void trim() {
    if (p && cap > (4ull << 30)) {
      (void)hipFree(p);
      p = nullptr;
      cap = 0;
    }
  }
  bool ensure_part(size_t b) {
    if (b <= part_cap) return true;
    if (part) (void)hipFree(part);
    part = nullptr;
    part_cap = 0;
    if (hipMalloc(&part, b + b / 8 + 256) != hipSuccess) return false;
    part_cap = b + b / 8 + 256;
    return true;
  }
  bool ensure(size_t b) {
    if (b <= cap) return true;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    if (hipMalloc(&p, b + b / 4 + 256) != hipSuccess) return false;
    cap = b + b / 4 + 256;
    return true;
  }
  bool ensure_out(size_t b) {
    if (b <= out_cap) return true;
    if (out) (void)hipFree(out);
    out = nullptr;
    out_cap = 0;
    if (hipMalloc(&out, b + b / 8 + 256) != hipSuccess) return false;
    out_cap = b + b / 8 + 256;
    return true;
  }
};

void* kd_scratch_create() { return new (std::nothrow) KdScratch(); }
void kd_scratch_destroy(void* s) { delete (KdScratch*)s; }

// Returns 0, or a negative cask_status; *out / *bytes: the block in device memory (owned by the
// scratch, valid until the next call).
int kd_build(void* scratch, const FileDesc* files_host, const uint32_t* file_ids_host, uint32_t nfiles,
             const uint64_t* row_off_host, const uint64_t* pos, const uint64_t* seq, const uint32_t* vsz,
             const uint16_t* ksz, uint64_t n, void* stream, void** out, uint64_t* bytes, const uint64_t* key_at) {
  KdScratch& S_ = *(KdScratch*)scratch;
  hipStream_t st = S(stream);
  // row indices are 32-bit per shard and every hipCUB call below takes an int count
  if (n > (uint64_t)INT32_MAX) return -12;  // CASK_E_CAPACITY: split the shard
  // temp storage sizes of the hipCUB calls
  size_t t_sort = 0, t_sel = 0, t_scan = 0;
  if (hipcub::DeviceRadixSort::SortPairs(nullptr, t_sort, (uint64_t*)nullptr, (uint64_t*)nullptr, (uint32_t*)nullptr,
                                          (uint32_t*)nullptr, (int)std::max<uint64_t>(n, 1), 0, 64, st) != hipSuccess ||
      hipcub::DeviceSelect::Flagged(nullptr, t_sel, hipcub::CountingInputIterator<uint32_t>(0), (uint8_t*)nullptr,
                                    (uint32_t*)nullptr, (uint32_t*)nullptr, (int)std::max<uint64_t>(n, 1), st) != hipSuccess ||
      hipcub::DeviceScan::ExclusiveSum(nullptr, t_scan, (uint64_t*)nullptr, (uint64_t*)nullptr,
                                       (int)std::max<uint64_t>(n, 1), st) != hipSuccess)
    return -11;
  const size_t tmp = std::max(t_sort, std::max(t_sel, t_scan));
  // layout of the scratch
  uint64_t o = 0;
  auto take = [&](uint64_t b) { const uint64_t r = o; o = al(o + b); return r; };
  const uint64_t n1 = n ? n : 1;
  const uint64_t o_fd = take(sizeof(FileDesc) * (nfiles + 1)), o_files = take(4ull * (nfiles + 1)), o_rowoff = take(8ull * (nfiles + 1)), o_h = take(8 * n1),
                 o_idx = take(4 * n1), o_fidx = take(4 * n1), o_hs = take(8 * n1), o_is = take(4 * n1),
                 o_head = take(n1), o_kind = take(n1), o_tval = take(8 * n1), o_ek = take(16 * n1),
                 o_ok = take(16 * n1), o_seg = take(4 * n1), o_sf = take(4 * n1), o_sksz = take(2 * n1),
                 o_skey = take(16 * n1),
                 o_nseg = take(8), o_fstat = take(32ull * (nfiles + 1)), o_tot = take(64), o_tmp = take(tmp);
  if (!S_.ensure(o)) return -13;
  uint8_t* b = (uint8_t*)S_.p;
  KdArgs a{};
  a.files = (const FileDesc*)(b + o_fd);
  a.file_ids = (const uint32_t*)(b + o_files);
  a.row_off = (const uint64_t*)(b + o_rowoff);
  a.nfiles = nfiles;
  a.pos = pos;
  a.seq = seq;
  a.vsz = vsz;
  a.ksz = ksz;
  a.n = n;
  a.key_at_row = key_at;
  // CASK_KD_HASH_BITS=b (test hook): rows grouped by b bits of their key hash, so that different
  // keys share segments and take the collision path (kRaw) — the fold of the block is the same
  {
    const char* hb = cask_knobs::hook("CASK_KD_HASH_BITS");
    const int bits = hb ? atoi(hb) : 64;
    a.hmask = bits >= 64 ? ~0ull : bits <= 0 ? 0ull : (1ull << bits) - 1;
  }
  a.h = (uint64_t*)(b + o_h);
  a.idx = (uint32_t*)(b + o_idx);
  a.fidx = (uint32_t*)(b + o_fidx);
  a.hs = (uint64_t*)(b + o_hs);
  a.is = (uint32_t*)(b + o_is);
  a.head = b + o_head;
  a.kind = b + o_kind;
  a.tval = (uint64_t*)(b + o_tval);
  // (ecnt/ekey and eoff/koff are written from k_kd_segs on; until k_kd_gather has run, the same
  // bytes hold k_kd_hash's packed rows: rfld and rkey)
  a.ecnt = (uint64_t*)(b + o_ek);
  a.ekey = (uint64_t*)(b + o_ek) + n1;
  a.eoff = (uint64_t*)(b + o_ok);
  a.koff = (uint64_t*)(b + o_ok) + n1;
  a.seg = (uint32_t*)(b + o_seg);
  a.sseq = (uint64_t*)(b + o_h);    // (the sort's inputs are dead once it has run)
  a.svsz = (uint32_t*)(b + o_idx);
  a.sf = (uint32_t*)(b + o_sf);
  a.sksz = (uint16_t*)(b + o_sksz);
  a.skey = (u32x4*)(b + o_skey);
  a.rfld = (u32x4*)(b + o_ek);
  a.rkey = (u32x4*)(b + o_ok);
  a.nseg = (uint32_t*)(b + o_nseg);
  a.fstat = (uint64_t*)(b + o_fstat);
  a.tot = (unsigned long long*)(b + o_tot);
  void* tmpp = b + o_tmp;
  bool ok = true;
  auto H = [&](hipError_t e) { ok = ok && e == hipSuccess; };
  H(hipMemcpyAsync((void*)a.files, files_host, sizeof(FileDesc) * nfiles, hipMemcpyHostToDevice, st));
  H(hipMemcpyAsync((void*)a.file_ids, file_ids_host, 4ull * nfiles, hipMemcpyHostToDevice, st));
  H(hipMemcpyAsync((void*)a.row_off, row_off_host, 8ull * (nfiles + 1), hipMemcpyHostToDevice, st));
  H(hipMemsetAsync(a.fstat, 0, 32ull * (nfiles + 1), st));
  H(hipMemsetAsync(a.tot, 0, 64, st));
  const int cus = device_cus();
  const uint32_t grid = (uint32_t)std::min<uint64_t>((n + 255) / 256, (uint64_t)cus * 16);
  if (n) {
    hipLaunchKernelGGL(k_kd_hash, dim3(grid), dim3(256), 0, st, a);
    size_t tb = tmp;
    H(hipcub::DeviceRadixSort::SortPairs(tmpp, tb, a.h, a.hs, a.idx, a.is, (int)n, 0, 64, st));
    hipLaunchKernelGGL(k_kd_heads, dim3(grid), dim3(256), 0, st, a);
    tb = tmp;
    H(hipcub::DeviceSelect::Flagged(tmpp, tb, hipcub::CountingInputIterator<uint32_t>(0), a.head, a.seg, a.nseg,
                                     (int)n, st));
    hipLaunchKernelGGL(k_kd_gather, dim3(grid), dim3(256), 0, st, a);
    hipLaunchKernelGGL(k_kd_segs, dim3(grid), dim3(256), 0, st, a);
    tb = tmp;
    H(hipcub::DeviceScan::ExclusiveSum(tmpp, tb, a.ecnt, a.eoff, (int)n, st));
    tb = tmp;
    H(hipcub::DeviceScan::ExclusiveSum(tmpp, tb, a.ekey, a.koff, (int)n, st));
    hipLaunchKernelGGL(k_kd_totals, dim3(1), dim3(64), 0, st, a);
  }
  unsigned long long tot[3] = {0, 0, 0};
  H(hipMemcpyAsync(tot, a.tot, sizeof(tot), hipMemcpyDeviceToHost, st));
  H(hipStreamSynchronize(st));
  H(hipGetLastError());
  if (!ok) return -11;
  const uint64_t nrec = n ? tot[1] : 0, kb = n ? tot[2] : 0;
  a.rec_at = sizeof(ShardHeader);
  const uint64_t fstat_at = a.rec_at + sizeof(ShardRec) * nrec;
  a.key_at = fstat_at + sizeof(ShardFileStat) * nfiles;
  const uint64_t total = (a.key_at + kb + 7) & ~7ull;
  if (!S_.ensure_out(total)) return -13;
  a.out = (uint8_t*)S_.out;
  if (n && nrec) hipLaunchKernelGGL(k_kd_write, dim3(grid), dim3(256), 0, st, a);
  hipLaunchKernelGGL(k_kd_header, dim3(1), dim3(256), 0, st, a, n, fstat_at, total);
  H(hipStreamSynchronize(st));
  H(hipGetLastError());
  S_.trim();
  if (!ok) return -11;
  *out = S_.out;
  *bytes = total;
  return 0;
}

// ------------------------------------------------------------------------------------------
// Key-hash partition of a keydir block (keydir_format.h): what each rank sends each owner in the
// all-to-all of the huge-keyspace replay. Owner per record from its key hash, a
// stable radix sort of (owner, record) — block order within each part — then the parts written
// whole: records and keys gathered, headers and stats tables. Byte for byte the host's
// cask_keydir_partition_host.
// ------------------------------------------------------------------------------------------
struct PtArgs {
  const ShardRec* rec;
  const uint8_t* keys;
  const ShardFileStat* fst;
  uint64_t n;
  uint32_t nparts, nfiles;
  uint64_t max_seq_p1, rows_in;
  uint64_t* kl;       // n + 1: key length (input order), then its exclusive sum ko
  uint64_t* ko;
  uint16_t* own;      // owner (input order)
  uint16_t* own_s;    // sorted
  uint32_t* idx;
  uint32_t* idx_s;
  uint64_t* kl2;      // n + 1: key length in sorted order, then its exclusive sum ko2
  uint64_t* ko2;
  uint64_t* start;    // nparts + 1: each part's first sorted position, then ko2 there (pkey)
  uint64_t* pkey;
  const uint64_t* poff;  // nparts + 1: each part's offset in out
  uint8_t* out;
};

__global__ __launch_bounds__(256) void k_pt_len(PtArgs a) {
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i <= a.n; i += (uint64_t)gridDim.x * 256ull)
    a.kl[i] = i < a.n ? a.rec[i].ksz : 0ull;
}

__global__ __launch_bounds__(256) void k_pt_own(PtArgs a) {
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < a.n; i += (uint64_t)gridDim.x * 256ull) {
    a.own[i] = (uint16_t)key_owner(key_hash(a.keys + a.ko[i], a.rec[i].ksz), a.nparts);
    a.idx[i] = (uint32_t)i;
  }
}

__global__ __launch_bounds__(256) void k_pt_len2(PtArgs a) {
  for (uint64_t j = blockIdx.x * 256ull + threadIdx.x; j <= a.n; j += (uint64_t)gridDim.x * 256ull)
    a.kl2[j] = j < a.n ? a.rec[a.idx_s[j]].ksz : 0ull;
}

__global__ __launch_bounds__(256) void k_pt_bounds(PtArgs a) {
  for (uint32_t o = blockIdx.x * 256u + threadIdx.x; o <= a.nparts; o += gridDim.x * 256u) {
    uint64_t lo = 0, hi = a.n;  // the first sorted position with owner >= o
    while (lo < hi) {
      const uint64_t mid = (lo + hi) >> 1;
      if (a.own_s[mid] < o) lo = mid + 1; else hi = mid;
    }
    a.start[o] = lo;
    a.pkey[o] = a.ko2[lo];
  }
}

__device__ __forceinline__ uint64_t pt_key_at(const PtArgs& a, uint32_t o) {
  return sizeof(ShardHeader) + sizeof(ShardRec) * (a.start[o + 1] - a.start[o]) + sizeof(ShardFileStat) * (uint64_t)a.nfiles;
}

__global__ __launch_bounds__(256) void k_pt_write(PtArgs a) {
  for (uint64_t j = blockIdx.x * 256ull + threadIdx.x; j < a.n; j += (uint64_t)gridDim.x * 256ull) {
    const uint32_t o = a.own_s[j];
    const uint64_t i = a.idx_s[j], r = j - a.start[o];
    uint8_t* base = a.out + a.poff[o];
    ((ShardRec*)(base + sizeof(ShardHeader)))[r] = a.rec[i];
    uint8_t* kd = base + pt_key_at(a, o) + (a.ko2[j] - a.pkey[o]);
    const uint8_t* ks = a.keys + a.ko[i];
    for (uint32_t b = 0, k = a.rec[i].ksz; b < k; ++b) kd[b] = ks[b];
  }
}

// Headers, stats tables (part 0: the block's; the others: its file ids with zero counts) and the
// zero padding of each part.
__global__ __launch_bounds__(256) void k_pt_head(PtArgs a) {
  const uint64_t tot = (uint64_t)(a.nparts) * (a.nfiles + 1);
  for (uint64_t x = blockIdx.x * 256ull + threadIdx.x; x < tot; x += (uint64_t)gridDim.x * 256ull) {
    const uint32_t o = (uint32_t)(x / (a.nfiles + 1)), f = (uint32_t)(x % (a.nfiles + 1));
    uint8_t* base = a.out + a.poff[o];
    const uint64_t nr = a.start[o + 1] - a.start[o], kb = a.pkey[o + 1] - a.pkey[o];
    if (f == a.nfiles) {
      ShardHeader hd{};
      hd.magic = kMagic;
      hd.version = kVersion;
      hd.nrec = nr;
      hd.key_bytes = kb;
      hd.nfiles = a.nfiles;
      hd.max_seq_p1 = a.max_seq_p1;
      hd.rows_in = o == 0 ? a.rows_in : 0ull;
      hd.bytes = a.poff[o + 1] - a.poff[o];
      *(ShardHeader*)base = hd;
      for (uint64_t e = pt_key_at(a, o) + kb; e < hd.bytes; ++e) base[e] = 0;
      continue;
    }
    ShardFileStat st = a.fst[f];
    if (o) st.puts = st.put_bytes = st.stale = st.stale_bytes = 0;
    st.pad = 0;
    ((ShardFileStat*)(base + sizeof(ShardHeader) + sizeof(ShardRec) * nr))[f] = st;
  }
}

// Returns 0 or a negative cask_status; *out: the parts (device memory owned by the scratch, valid
// until its next partition), part_off (host, nparts + 1): part o is out[part_off[o], part_off[o + 1]).
int kd_partition(void* scratch, const void* block, uint64_t bytes, uint32_t nparts, void* stream, void** out,
                 uint64_t* part_off) {
  KdScratch& S_ = *(KdScratch*)scratch;
  hipStream_t st = S(stream);
  if (!block || nparts < 1 || nparts > kMaxParts || bytes < sizeof(ShardHeader)) return -10;
  ShardHeader hd;
  if (hipMemcpyAsync(&hd, block, sizeof(hd), hipMemcpyDeviceToHost, st) != hipSuccess || hipStreamSynchronize(st) != hipSuccess)
    return -11;
  // the same checks as the fold (cask_keydir_merge): counts bounded by the block's size first
  if (hd.magic != kMagic || hd.version != kVersion || hd.bytes > bytes ||
      hd.nrec > (bytes - sizeof(ShardHeader)) / sizeof(ShardRec) ||
      (uint64_t)hd.nfiles > (bytes - sizeof(ShardHeader)) / sizeof(ShardFileStat))
    return -10;
  const uint64_t n = hd.nrec, fst_at = sizeof(ShardHeader) + sizeof(ShardRec) * n,
                 key_at = fst_at + sizeof(ShardFileStat) * (uint64_t)hd.nfiles;
  if (key_at + hd.key_bytes > hd.bytes) return -10;
  if (n > (uint64_t)INT32_MAX) return -12;  // (hipCUB's int counts)
  int bits = 1;
  while ((1u << bits) < nparts) ++bits;
  size_t t_sort = 0, t_scan = 0;
  if (hipcub::DeviceRadixSort::SortPairs(nullptr, t_sort, (uint16_t*)nullptr, (uint16_t*)nullptr, (uint32_t*)nullptr,
                                          (uint32_t*)nullptr, (int)std::max<uint64_t>(n, 1), 0, bits, st) != hipSuccess ||
      hipcub::DeviceScan::ExclusiveSum(nullptr, t_scan, (uint64_t*)nullptr, (uint64_t*)nullptr, (int)(n + 1), st) != hipSuccess)
    return -11;
  uint64_t o = 0;
  auto take = [&](uint64_t b) { const uint64_t r = o; o = al(o + b); return r; };
  const uint64_t n1 = n + 1;
  const uint64_t o_kl = take(8 * n1), o_ko = take(8 * n1), o_own = take(2 * n1), o_owns = take(2 * n1),
                 o_idx = take(4 * n1), o_idxs = take(4 * n1), o_kl2 = take(8 * n1), o_ko2 = take(8 * n1),
                 o_start = take(8ull * (nparts + 1)), o_pkey = take(8ull * (nparts + 1)), o_poff = take(8ull * (nparts + 1)),
                 o_tmp = take(std::max(t_sort, t_scan));
  if (!S_.ensure(o)) return -13;
  uint8_t* b = (uint8_t*)S_.p;
  PtArgs a{};
  a.rec = (const ShardRec*)((const uint8_t*)block + sizeof(ShardHeader));
  a.fst = (const ShardFileStat*)((const uint8_t*)block + fst_at);
  a.keys = (const uint8_t*)block + key_at;
  a.n = n;
  a.nparts = nparts;
  a.nfiles = hd.nfiles;
  a.max_seq_p1 = hd.max_seq_p1;
  a.rows_in = hd.rows_in;
  a.kl = (uint64_t*)(b + o_kl);
  a.ko = (uint64_t*)(b + o_ko);
  a.own = (uint16_t*)(b + o_own);
  a.own_s = (uint16_t*)(b + o_owns);
  a.idx = (uint32_t*)(b + o_idx);
  a.idx_s = (uint32_t*)(b + o_idxs);
  a.kl2 = (uint64_t*)(b + o_kl2);
  a.ko2 = (uint64_t*)(b + o_ko2);
  a.start = (uint64_t*)(b + o_start);
  a.pkey = (uint64_t*)(b + o_pkey);
  a.poff = (const uint64_t*)(b + o_poff);
  void* tmpp = b + o_tmp;
  bool ok = true;
  auto H = [&](hipError_t e) { ok = ok && e == hipSuccess; };
  const uint32_t grid = (uint32_t)std::min<uint64_t>((n + 256) / 256, (uint64_t)device_cus() * 16);
  hipLaunchKernelGGL(k_pt_len, dim3(grid), dim3(256), 0, st, a);
  size_t tb = std::max(t_sort, t_scan);
  H(hipcub::DeviceScan::ExclusiveSum(tmpp, tb, a.kl, a.ko, (int)(n + 1), st));
  uint64_t kt = 0;  // the keys the records claim must be the block's key bytes
  H(hipMemcpyAsync(&kt, a.ko + n, 8, hipMemcpyDeviceToHost, st));
  H(hipStreamSynchronize(st));
  if (!ok) return -11;
  if (kt != hd.key_bytes) return -10;
  if (n) {
    hipLaunchKernelGGL(k_pt_own, dim3(grid), dim3(256), 0, st, a);
    tb = std::max(t_sort, t_scan);
    H(hipcub::DeviceRadixSort::SortPairs(tmpp, tb, a.own, a.own_s, a.idx, a.idx_s, (int)n, 0, bits, st));
  }
  hipLaunchKernelGGL(k_pt_len2, dim3(grid), dim3(256), 0, st, a);
  tb = std::max(t_sort, t_scan);
  H(hipcub::DeviceScan::ExclusiveSum(tmpp, tb, a.kl2, a.ko2, (int)(n + 1), st));
  hipLaunchKernelGGL(k_pt_bounds, dim3((nparts + 256) / 256), dim3(256), 0, st, a);
  std::vector<uint64_t> hs(2ull * (nparts + 1));
  H(hipMemcpyAsync(hs.data(), a.start, 8ull * (nparts + 1), hipMemcpyDeviceToHost, st));
  H(hipMemcpyAsync(hs.data() + nparts + 1, a.pkey, 8ull * (nparts + 1), hipMemcpyDeviceToHost, st));
  H(hipStreamSynchronize(st));
  if (!ok) return -11;
  part_off[0] = 0;
  for (uint32_t p = 0; p < nparts; ++p)
    part_off[p + 1] = part_off[p] + part_bytes(hs[p + 1] - hs[p], hs[nparts + 1 + p + 1] - hs[nparts + 1 + p], hd.nfiles);
  if (!S_.ensure_part(part_off[nparts])) return -13;
  a.out = (uint8_t*)S_.part;
  H(hipMemcpyAsync((void*)a.poff, part_off, 8ull * (nparts + 1), hipMemcpyHostToDevice, st));
  if (n) hipLaunchKernelGGL(k_pt_write, dim3(grid), dim3(256), 0, st, a);
  const uint64_t th = (uint64_t)nparts * (hd.nfiles + 1);
  hipLaunchKernelGGL(k_pt_head, dim3((uint32_t)std::min<uint64_t>((th + 255) / 256, 4096)), dim3(256), 0, st, a);
  H(hipStreamSynchronize(st));
  H(hipGetLastError());
  S_.trim();
  if (!ok) return -11;
  *out = S_.part;
  return 0;
}

// ------------------------------------------------------------------------------------------
// Hint-file bodies on the device (RecreateHints::next + HintWriter::write, log.rs:382-386,
// 454-465; Hint::write_bytes, data.rs:242-256): for every Ok row, in order,
// [sequence u64][key_size u16][value_size u32 (0xFFFFFFFF: tombstone)][entry_pos u64][key],
// little-endian, one body per file laid out file after file. The host appends the XXH32 trailer
// (HintWriter::drop, log.rs:389-395) and writes the files.
// ------------------------------------------------------------------------------------------
struct HpArgs {
  const FileDesc* files;
  const uint64_t* row_off;
  uint32_t nfiles;
  const uint64_t* pos;
  const uint64_t* seq;
  const uint32_t* vsz;
  const uint16_t* ksz;
  const uint8_t* status;
  uint64_t n;
  uint64_t* sz;
  uint64_t* off;
  uint64_t* fstart;  // nfiles + 1
  uint8_t* out;
};

__global__ __launch_bounds__(256) void k_hint_sizes(HpArgs a) {
  for (uint64_t d = blockIdx.x * 256ull + threadIdx.x; d < a.n; d += (uint64_t)gridDim.x * 256ull)
    a.sz[d] = a.status[d] == kRowOk ? 22ull + a.ksz[d] : 0ull;
}

__global__ __launch_bounds__(256) void k_hint_write(HpArgs a) {
  for (uint64_t d = blockIdx.x * 256ull + threadIdx.x; d < a.n; d += (uint64_t)gridDim.x * 256ull) {
    if (a.status[d] != kRowOk) continue;
    uint32_t lo = 0, hi = a.nfiles;  // the row's file: last f with row_off[f] <= d
    while (hi - lo > 1) {
      const uint32_t mid = (lo + hi) >> 1;
      if (a.row_off[mid] <= d) lo = mid; else hi = mid;
    }
    uint8_t* o = a.out + a.off[d];
    const uint64_t s = a.seq[d], p = a.pos[d];
    const uint32_t k = a.ksz[d], v = a.vsz[d];
    for (int i = 0; i < 8; ++i) o[i] = (uint8_t)(s >> (8 * i));
    o[8] = (uint8_t)k;
    o[9] = (uint8_t)(k >> 8);
    for (int i = 0; i < 4; ++i) o[10 + i] = (uint8_t)(v >> (8 * i));
    for (int i = 0; i < 8; ++i) o[14 + i] = (uint8_t)(p >> (8 * i));
    const uint8_t* key = a.files[lo].data + p + 18;
    for (uint32_t i = 0; i < k; ++i) o[22 + i] = key[i];
  }
}

__global__ void k_hint_starts(HpArgs a) {
  for (uint32_t f = threadIdx.x; f <= a.nfiles; f += blockDim.x) {
    const uint64_t r = a.row_off[f];
    a.fstart[f] = r < a.n ? a.off[r] : (a.n ? a.off[a.n - 1] + a.sz[a.n - 1] : 0ull);
  }
}

// Rows of hint bodies (cask_parse_hints_device) into keydir rows: pos becomes the entry position
// the hint records (bytes 14..21 of the hint, Hint::write_bytes, data.rs:242-256) and key_at the
// key's offset in the body (22 bytes in).
__global__ __launch_bounds__(256) void k_hint_entries(const FileDesc* files, const uint64_t* row_off, uint32_t nfiles,
                                                      uint64_t n, uint64_t* pos, uint64_t* key_at) {
  for (uint64_t d = blockIdx.x * 256ull + threadIdx.x; d < n; d += (uint64_t)gridDim.x * 256ull) {
    uint32_t lo = 0, hi = nfiles;  // the row's file: last f with row_off[f] <= d
    while (hi - lo > 1) {
      const uint32_t mid = (lo + hi) >> 1;
      if (row_off[mid] <= d) lo = mid; else hi = mid;
    }
    const uint64_t off = pos[d];
    const uint8_t* h = files[lo].data + off;
    uint64_t ep = 0;
    for (int i = 0; i < 8; ++i) ep |= (uint64_t)h[14 + i] << (8 * i);
    pos[d] = ep;
    key_at[d] = off + 22;
  }
}

int hint_entries(void* scratch, const FileDesc* files_host, uint32_t nfiles, const uint64_t* row_off_host,
                 uint64_t n, uint64_t* pos, uint64_t* key_at, void* stream) {
  KdScratch& S_ = *(KdScratch*)scratch;
  hipStream_t st = S(stream);
  const uint64_t o_rowoff = al(sizeof(FileDesc) * (nfiles + 1));
  if (!S_.ensure(o_rowoff + 8ull * (nfiles + 1))) return -13;
  FileDesc* d_fd = (FileDesc*)S_.p;
  uint64_t* d_ro = (uint64_t*)((uint8_t*)S_.p + o_rowoff);
  bool ok = hipMemcpyAsync(d_fd, files_host, sizeof(FileDesc) * nfiles, hipMemcpyHostToDevice, st) == hipSuccess &&
            hipMemcpyAsync(d_ro, row_off_host, 8ull * (nfiles + 1), hipMemcpyHostToDevice, st) == hipSuccess;
  if (!ok) return -11;
  if (n) {
    const uint32_t grid = (uint32_t)std::min<uint64_t>((n + 255) / 256, (uint64_t)device_cus() * 16);
    hipLaunchKernelGGL(k_hint_entries, dim3(grid), dim3(256), 0, st, d_fd, d_ro, nfiles, n, pos, key_at);
  }
  return hipGetLastError() == hipSuccess ? 0 : -11;
}

// Returns 0 or a negative cask_status. file_start (host, nfiles + 1): each file's body in `out`.
int hint_pack(void* scratch, const FileDesc* files_host, uint32_t nfiles, const uint64_t* row_off_host,
              const uint64_t* pos, const uint64_t* seq, const uint32_t* vsz, const uint16_t* ksz, const uint8_t* status,
              uint64_t n, uint8_t* out, uint64_t cap, uint64_t* file_start, void* stream) {
  KdScratch& S_ = *(KdScratch*)scratch;
  hipStream_t st = S(stream);
  if (n > (uint64_t)INT32_MAX) return -12;  // CASK_E_CAPACITY: the scan takes an int count (callers batch files)
  size_t t_scan = 0;
  if (hipcub::DeviceScan::ExclusiveSum(nullptr, t_scan, (uint64_t*)nullptr, (uint64_t*)nullptr,
                                       (int)std::max<uint64_t>(n, 1), st) != hipSuccess)
    return -11;
  uint64_t o = 0;
  auto take = [&](uint64_t b) { const uint64_t r = o; o = al(o + b); return r; };
  const uint64_t n1 = n ? n : 1;
  const uint64_t o_fd = take(sizeof(FileDesc) * (nfiles + 1)), o_ro = take(8ull * (nfiles + 1)), o_sz = take(8 * n1),
                 o_off = take(8 * n1), o_fs = take(8ull * (nfiles + 1)), o_tmp = take(t_scan);
  if (!S_.ensure(o)) return -13;
  uint8_t* b = (uint8_t*)S_.p;
  HpArgs a{};
  a.files = (const FileDesc*)(b + o_fd);
  a.row_off = (const uint64_t*)(b + o_ro);
  a.nfiles = nfiles;
  a.pos = pos;
  a.seq = seq;
  a.vsz = vsz;
  a.ksz = ksz;
  a.status = status;
  a.n = n;
  a.sz = (uint64_t*)(b + o_sz);
  a.off = (uint64_t*)(b + o_off);
  a.fstart = (uint64_t*)(b + o_fs);
  a.out = out;
  bool ok = true;
  auto H = [&](hipError_t e) { ok = ok && e == hipSuccess; };
  H(hipMemcpyAsync((void*)a.files, files_host, sizeof(FileDesc) * nfiles, hipMemcpyHostToDevice, st));
  H(hipMemcpyAsync((void*)a.row_off, row_off_host, 8ull * (nfiles + 1), hipMemcpyHostToDevice, st));
  const uint32_t grid = (uint32_t)std::min<uint64_t>((n + 255) / 256 + 1, (uint64_t)device_cus() * 16);
  if (n) {
    hipLaunchKernelGGL(k_hint_sizes, dim3(grid), dim3(256), 0, st, a);
    size_t tb = t_scan;
    H(hipcub::DeviceScan::ExclusiveSum(b + o_tmp, tb, a.sz, a.off, (int)n, st));
  }
  hipLaunchKernelGGL(k_hint_starts, dim3(1), dim3(256), 0, st, a);
  H(hipMemcpyAsync(file_start, a.fstart, 8ull * (nfiles + 1), hipMemcpyDeviceToHost, st));
  H(hipStreamSynchronize(st));
  if (!ok) return -11;
  if (file_start[nfiles] > cap) return -12;  // CASK_E_CAPACITY: file_start[nfiles] bytes are needed
  if (n) hipLaunchKernelGGL(k_hint_write, dim3(grid), dim3(256), 0, st, a);
  H(hipStreamSynchronize(st));
  H(hipGetLastError());
  return ok ? 0 : -11;
}

}  // namespace cask_dev
