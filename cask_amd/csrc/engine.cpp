// Host engine above the C ABI: the Cask::open replay (cask.rs:335-382) with the data-file scan
// on the GPU. Mirrors Log::open (log.rs:36-85), find_data_files (log.rs:483-510), the hint-file
// fast path (log.rs:121-135, 432-447, 512-539; data.rs:258-276), hint recreation
// (log.rs:137-148, 367-395, 449-471), and the keydir fold Index::update + Stats
// (cask.rs:28-95; stats.rs:6-67). The scan itself is cask_scan_host (scan_runtime.cpp).
// Also the compaction merge (cask.rs:451-640): liveness against the keydir on the host, the
// live records verified by the device scan and copied into the new data files on the device.
#include <dirent.h>
#include <fcntl.h>
#include <sched.h>
#include <sys/file.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <deque>
#include <initializer_list>
#include <atomic>
#include <condition_variable>
#include <cerrno>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <memory>
#include <map>
#include <mutex>
#include <new>
#include <regex>
#include <thread>
#include <string>
#include <unordered_map>
#include <vector>

#include <hip/hip_runtime_api.h>

#include "abi_guard.h"
#include "../../include/cask_scan.h"
#include "host_ring.h"
#include "keydir_format.h"
#include "xxh32.h"
#include "knobs.h"

namespace {

inline uint16_t rd16(const uint8_t* p) { return (uint16_t)(p[0] | (p[1] << 8)); }
inline uint32_t rd32(const uint8_t* p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
inline uint64_t rd64(const uint8_t* p) { return (uint64_t)rd32(p) | ((uint64_t)rd32(p + 4) << 32); }
inline void wr16(uint8_t* p, uint16_t v) { p[0] = (uint8_t)v; p[1] = (uint8_t)(v >> 8); }
inline void wr32(uint8_t* p, uint32_t v) { for (int i = 0; i < 4; ++i) p[i] = (uint8_t)(v >> (8 * i)); }
inline void wr64(uint8_t* p, uint64_t v) { for (int i = 0; i < 8; ++i) p[i] = (uint8_t)(v >> (8 * i)); }

inline uint64_t hash_key(const uint8_t* k, uint32_t n) {
  uint64_t h = 0x9E3779B97F4A7C15ull ^ (n * 0xC2B2AE3D27D4EB4Full);
  uint32_t i = 0;
  for (; i + 8 <= n; i += 8) {
    uint64_t w;
    memcpy(&w, k + i, 8);
    h = (h ^ w) * 0xBF58476D1CE4E5B9ull;
    h ^= h >> 31;
  }
  uint64_t t = 0;
  for (uint32_t j = 0; i + j < n; ++j) t |= (uint64_t)k[i + j] << (8 * j);
  h = (h ^ t) * 0x94D049BB133111EBull;
  return h ^ (h >> 29);
}

struct StatsEntry {  // stats.rs:7-11
  uint64_t entries = 0, dead_entries = 0, dead_bytes = 0;
};
using StatsMap = std::unordered_map<uint32_t, StatsEntry>;

// Stats::add_entry / remove_entry (stats.rs:23-48) into `st`. A fold on threads keeps per-table
// deltas: then `base` is the map entering the fold, and a remove of a file absent from the delta
// still counts when that file has a row there (remove_entry only skips files with no row at all).
// The rows a fold touches are few (the files of the replay) and each is touched by most records: a
// 16-entry cache of row pointers by file id (unordered_map elements never move) keeps the map
// lookups off the per-record path.
class StatsDelta {
 public:
  StatsDelta(StatsMap& st, const StatsMap* base) : st_(st), base_(base) {}
  void add(uint32_t file_id) { get(file_id, true)->entries += 1; }
  void remove(uint32_t file_id, uint64_t size) {
    StatsEntry* e = get(file_id, false);
    if (!e) return;  // "Tried to reclaim non-existant entry": warn only
    e->dead_entries += 1;
    e->dead_bytes += size;
  }

 private:
  StatsEntry* get(uint32_t fid, bool create) {
    const unsigned c = fid & 15u;
    if (ce_[c] && cf_[c] == fid) return ce_[c];
    auto it = st_.find(fid);
    if (it == st_.end()) {
      if (!create && !(base_ && base_->count(fid))) return nullptr;
      it = st_.emplace(fid, StatsEntry{}).first;
    }
    cf_[c] = fid;
    ce_[c] = &it->second;
    return ce_[c];
  }
  StatsMap& st_;
  const StatsMap* base_;
  uint32_t cf_[16] = {};
  StatsEntry* ce_[16] = {};
};

// Allocator for large tables: 2-MiB-aligned and advised as transparent huge pages (a keydir fold
// hits random slots of tables of tens of MB; with 4-KiB pages nearly every access also misses the
// TLB). Small allocations take the ordinary heap; up to kMap the heap's huge-aligned blocks (which a
// later table of the process reuses without new page faults: the host fold's 16-MB tables), above it
// fresh anonymous pages, zero until first written, so a table of empty slots costs no fill pass
// (KeyDir::reserve; configs[3]'s merge tables of ~90 MB, which the heap would map afresh anyway).
template <class T>
struct HugeAlloc {
  using value_type = T;
  HugeAlloc() = default;
  template <class U>
  HugeAlloc(const HugeAlloc<U>&) {}
  static constexpr size_t kHuge = 2ull << 20, kMap = 32ull << 20;
  static size_t rounded(size_t b) { return (b + kHuge - 1) & ~(kHuge - 1); }
  T* allocate(size_t n) {
    const size_t b = n * sizeof(T);
    if (b < kHuge) {
      void* p = ::operator new(b, std::align_val_t(alignof(T) < 64 ? 64 : alignof(T)));
      return static_cast<T*>(p);
    }
    const size_t r = rounded(b);
    if (b < kMap) {
      void* p = std::aligned_alloc(kHuge, r);
      if (!p) throw std::bad_alloc();
      (void)madvise(p, r, MADV_HUGEPAGE);
      return static_cast<T*>(p);
    }
    // (over-map by one huge page and trim to a 2-MiB-aligned range)
    void* m = mmap(nullptr, r + kHuge, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    if (m == MAP_FAILED) throw std::bad_alloc();
    const uintptr_t a = ((uintptr_t)m + kHuge - 1) & ~(uintptr_t)(kHuge - 1);
    if (a > (uintptr_t)m) munmap(m, a - (uintptr_t)m);
    const uintptr_t e = (uintptr_t)m + r + kHuge;
    if (e > a + r) munmap((void*)(a + r), e - (a + r));
    (void)madvise((void*)a, r, MADV_HUGEPAGE);
    return reinterpret_cast<T*>(a);
  }
  static bool zeroed(size_t n) { return n * sizeof(T) >= kMap; }  // allocate(n) hands out zero bytes
  template <class U>
  void construct(U* p) noexcept {  // resize/size-constructor leave trivial elements uninitialized
    ::new (static_cast<void*>(p)) U;
  }
  template <class U, class... A>
  void construct(U* p, A&&... a) {
    ::new (static_cast<void*>(p)) U(std::forward<A>(a)...);
  }
  void deallocate(T* p, size_t n) {
    const size_t b = n * sizeof(T);
    if (b < kHuge) ::operator delete(p, std::align_val_t(alignof(T) < 64 ? 64 : alignof(T)));
    else if (b < kMap) std::free(p);
    else munmap(p, rounded(b));
  }
  template <class U>
  bool operator==(const HugeAlloc<U>&) const { return true; }
  template <class U>
  bool operator!=(const HugeAlloc<U>&) const { return false; }
};

// One table of HashMap<Vec<u8>, IndexEntry> (cask.rs:28-31). Open addressing over 64-B slots (one
// cache line each); a key of up to 16 bytes lives in its slot, a longer one in an append-only arena
// (the reference copies every key: hint.key.to_vec(), cask.rs:68). A fold touches one line per
// record for short keys: the slot holds hash, entry and key.
class KeyDir {
 public:
  static constexpr uint32_t kInline = 16;
  struct alignas(64) Slot {
    uint64_t hash;
    cask_index_entry e;
    uint32_t ksz;
    uint32_t state;  // 0 empty, 1 live, 2 deleted
    union {
      uint8_t kin[kInline];  // ksz <= kInline
      uint64_t key_off;      // else: the key's offset in the arena
    };
  };
  static_assert(sizeof(Slot) == 64, "a slot is one cache line");
  std::vector<Slot, HugeAlloc<Slot>> slots;
  std::vector<uint8_t> arena;
  uint64_t live = 0, used = 0;

  KeyDir() { slots.assign(256, Slot{}); }

  const uint8_t* key_of(const Slot& s) const { return s.ksz <= kInline ? s.kin : arena.data() + s.key_off; }
  // a key's home slot: the hash's bits below the table bits (Index::sub_of), scaled to the table —
  // any size, not only powers of two (a table sized to its keys: 4.5 instead of 8 GB of slots for
  // configs[3]'s 52 M keys, all of which are first-touch page faults in the merge)
  uint64_t home(uint64_t h) const { return (uint64_t)(((unsigned __int128)(h << 6) * slots.size()) >> 64); }
  void prefetch(uint64_t h) const { __builtin_prefetch(&slots[home(h)]); }
  // the arena bytes of a long key on the slot h lands on, once that slot is in cache (prefetch() a
  // few records before)
  void prefetch_key(uint64_t h) const {
    const Slot& s = slots[home(h)];
    if (s.state == 1 && s.hash == h && s.ksz > kInline) __builtin_prefetch(arena.data() + s.key_off);
  }

  bool key_eq(const Slot& s, const uint8_t* k, uint32_t n) const {
    if (n == kInline) {  // (the common fixed-size key: two word compares, no call)
      uint64_t a[2], b[2];
      memcpy(a, s.kin, 16);
      memcpy(b, k, 16);
      return a[0] == b[0] && a[1] == b[1];
    }
    return n == 0 || memcmp(key_of(s), k, n) == 0;
  }

  int64_t find(const uint8_t* k, uint32_t n, uint64_t h) const {
    const uint64_t c = slots.size();
    for (uint64_t i = home(h);; i = i + 1 == c ? 0 : i + 1) {
      const Slot& s = slots[i];
      if (s.state == 0) return -(int64_t)i - 1;
      if (s.state == 1 && s.hash == h && s.ksz == n && key_eq(s, k, n)) return (int64_t)i;
    }
  }

  // Room for n live keys without growing; a rebuild drops the slots of deleted keys.
  void reserve(uint64_t n) {
    // A table holds up to 3/4 of its slots; one that must grow is sized to 2/5 (a slot is a line:
    // each probe past the home slot is one more line, each slot a first-touch fault. configs[3]'s
    // 52 M-key merge: loads 0.39-0.6 within 15 % of each other, 0.39 the fastest,
    // profiles/r06h_merge_loadsweep.txt; its compaction's 42 M lookups: 0.70-0.74 s at 0.39 against
    // 0.86-0.87 at 0.6, profiles/r06k_compaction_ab.txt)
    const uint64_t m = std::max(n, live) + 1;
    const bool fits = slots.size() * 3 >= m * 4;
    if (fits && (used + 1) * 4 <= slots.size() * 3) return;
    constexpr uint64_t kG = HugeAlloc<Slot>::kHuge / sizeof(Slot);  // (whole huge pages when large)
    const uint64_t need = m * 5 / 2 + 1;
    const uint64_t cap = fits ? slots.size()  // (same size: the deleted slots dropped)
                         : need <= 256 ? 256 : need < kG ? (need + 63) & ~63ull : (need + kG - 1) / kG * kG;
    std::vector<Slot, HugeAlloc<Slot>> old;
    old.swap(slots);
    slots.resize(cap);  // (default-initialised: a huge allocation is zero already, see HugeAlloc)
    if (!HugeAlloc<Slot>::zeroed(cap)) memset((void*)slots.data(), 0, cap * sizeof(Slot));
    used = 0;
    for (const Slot& s : old) {
      if (s.state != 1) continue;
      uint64_t i = home(s.hash);
      while (slots[i].state) i = i + 1 == cap ? 0 : i + 1;
      slots[i] = s;
      ++used;
    }
  }

  // Index::update's effect on the keydir alone (cask.rs:60-90 without the Stats calls): the fold of
  // the sharded replay, whose stats come from per-file counts (cask_keydir_finish).
  void update_kd(const uint8_t* key, uint32_t ksz, uint32_t file_id, uint64_t pos, uint32_t vsz_raw, uint64_t seq,
                 uint64_t h) {
    const bool deleted = vsz_raw == CASK_ENTRY_TOMBSTONE;
    if ((used + 1) * 4 > slots.size() * 3) reserve(live + live / 2 + 1);
    const int64_t f = find(key, ksz, h);
    if (f >= 0) {
      Slot& s = slots[f];
      if (s.e.sequence <= seq) {
        if (deleted) {
          s.state = 2;
          --live;
        } else {
          s.e = cask_index_entry{file_id, 0, pos, 18ull + ksz + vsz_raw, seq};
        }
      }
      return;
    }
    if (deleted) return;
    insert_at((uint64_t)(-f - 1), key, ksz, h, cask_index_entry{file_id, 0, pos, 18ull + ksz + vsz_raw, seq});
  }

  // Index::update (cask.rs:60-90). vsz_raw is the hint's value_size field.
  void update(const uint8_t* key, uint32_t ksz, uint32_t file_id, uint64_t pos, uint32_t vsz_raw, uint64_t seq,
              uint64_t h, StatsDelta& sd) {
    const bool deleted = vsz_raw == CASK_ENTRY_TOMBSTONE;
    cask_index_entry ie{};
    ie.file_id = file_id;
    ie.entry_pos = pos;
    ie.entry_size = 18ull + ksz + (deleted ? 0ull : (uint64_t)vsz_raw);  // data.rs:238-240
    ie.sequence = seq;
    if ((used + 1) * 4 > slots.size() * 3) reserve(live + live / 2 + 1);
    int64_t f = find(key, ksz, h);
    if (f >= 0) {  // Occupied
      Slot& s = slots[f];
      if (s.e.sequence <= seq) {
        sd.remove(s.e.file_id, s.e.entry_size);
        if (deleted) {
          s.state = 2;
          --live;
        } else {
          sd.add(file_id);
          s.e = ie;
        }
      } else {
        sd.add(file_id);
        sd.remove(file_id, ie.entry_size);
      }
      return;
    }
    if (deleted) return;  // Vacant + tombstone: nothing
    sd.add(file_id);
    insert_at((uint64_t)(-f - 1), key, ksz, h, ie);
  }

 private:
  void insert_at(uint64_t i, const uint8_t* key, uint32_t ksz, uint64_t h, const cask_index_entry& e) {
    Slot& s = slots[i];
    s.hash = h;
    s.ksz = ksz;
    s.state = 1;
    s.e = e;
    if (ksz <= kInline) {
      if (ksz) memcpy(s.kin, key, ksz);
    } else {
      s.key_off = arena.size();
      arena.insert(arena.end(), key, key + ksz);
    }
    ++live;
    ++used;
  }
};

// The keydir (Index, cask.rs:28-95): kSub tables split by key hash, so a fold on threads writes each
// table from one thread with no merge pass afterwards; one Stats map.
class Index {
 public:
  static constexpr unsigned kSub = 64;
  KeyDir sub[kSub];
  StatsMap stats;

  static unsigned sub_of(uint64_t h) { return (unsigned)(h >> 58); }
  uint64_t live() const {
    uint64_t n = 0;
    for (const KeyDir& k : sub) n += k.live;
    return n;
  }
  const cask_index_entry* get(const uint8_t* k, uint32_t n) const {  // Index::get (cask.rs:41-43)
    return get_h(k, n, hash_key(k, n));
  }
  const cask_index_entry* get_h(const uint8_t* k, uint32_t n, uint64_t h) const {
    const KeyDir& t = sub[sub_of(h)];
    const int64_t f = t.find(k, n, h);
    return f >= 0 ? &t.slots[(uint64_t)f].e : nullptr;
  }
  void update(const uint8_t* key, uint32_t ksz, uint32_t file_id, uint64_t pos, uint32_t vsz_raw, uint64_t seq) {
    const uint64_t h = hash_key(key, ksz);
    StatsDelta sd(stats, nullptr);
    sub[sub_of(h)].update(key, ksz, file_id, pos, vsz_raw, seq, h, sd);
  }
  void update_kd(const uint8_t* key, uint32_t ksz, uint32_t file_id, uint64_t pos, uint32_t vsz_raw, uint64_t seq) {
    const uint64_t h = hash_key(key, ksz);
    sub[sub_of(h)].update_kd(key, ksz, file_id, pos, vsz_raw, seq, h);
  }
  void prefetch(uint64_t h) const { sub[sub_of(h)].prefetch(h); }
  void prefetch_key(uint64_t h) const { sub[sub_of(h)].prefetch_key(h); }
  template <class F>
  void for_each_live(F fn) const {
    for (const KeyDir& t : sub)
      for (const KeyDir::Slot& s : t.slots)
        if (s.state == 1) fn(t, s);
  }
};

bool is_dir(const std::string& p) {
  struct stat st;
  return stat(p.c_str(), &st) == 0 && S_ISDIR(st.st_mode);
}
bool exists(const std::string& p) {
  struct stat st;
  return stat(p.c_str(), &st) == 0;
}
bool is_file_follow(const std::string& p) {  // Path::is_file (follows symlinks)
  struct stat st;
  return stat(p.c_str(), &st) == 0 && S_ISREG(st.st_mode);
}

std::string data_path(const std::string& dir, uint32_t id) {  // log.rs:473-476
  char b[32];
  snprintf(b, sizeof(b), "%010u.cask.data", id);
  return dir + "/" + b;
}
std::string hint_path(const std::string& dir, uint32_t id) {  // log.rs:478-481
  char b[32];
  snprintf(b, sizeof(b), "%010u.cask.hint", id);
  return dir + "/" + b;
}

bool read_file(const std::string& p, std::vector<uint8_t>& out) {
  int fd = open(p.c_str(), O_RDONLY);
  if (fd < 0) return false;
  struct stat st;
  if (fstat(fd, &st) != 0) {
    close(fd);
    return false;
  }
  try {  // (std::bad_alloc for a file larger than the memory left: the fd is not leaked on the way out)
    out.resize((size_t)st.st_size);
  } catch (...) {
    close(fd);
    throw;
  }
  size_t got = 0;
  while (got < out.size()) {
    ssize_t r = read(fd, out.data() + got, out.size() - got);
    if (r < 0) {
      if (errno == EINTR) continue;
      close(fd);
      return false;
    }
    if (r == 0) break;
    got += (size_t)r;
  }
  out.resize(got);
  close(fd);
  return true;
}

bool write_file(const std::string& p, const std::vector<uint8_t>& body, uint32_t trailer) {
  int fd = open(p.c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0644);  // util.rs:45-49
  if (fd < 0) return false;
  std::vector<uint8_t> buf(body);
  uint8_t t[4];
  wr32(t, trailer);
  buf.insert(buf.end(), t, t + 4);
  size_t off = 0;
  while (off < buf.size()) {
    ssize_t w = write(fd, buf.data() + off, buf.size() - off);
    if (w < 0) {
      if (errno == EINTR) continue;
      close(fd);
      return false;
    }
    off += (size_t)w;
  }
  close(fd);
  return true;
}

bool write_raw(const std::string& p, const uint8_t* b, size_t n) {
  int fd = open(p.c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0644);
  if (fd < 0) return false;
  size_t off = 0;
  while (off < n) {
    ssize_t w = write(fd, b + off, n - off);
    if (w < 0) {
      if (errno == EINTR) continue;
      close(fd);
      return false;
    }
    off += (size_t)w;
  }
  close(fd);
  return true;
}

// find_data_files (log.rs:483-510): regex "(\d+).cask.data$" (unescaped '.', unanchored),
// regular files only (DirEntry::metadata does not follow symlinks), u32 parse, ascending.
// Files a compaction renamed away (`<id>.cask.data.gone`, `<id>.cask.hint.gone`: no longer
// matched by find_data_files) are unlinked by the db's reclaim thread; a process that ended before
// that thread ran leaves them behind. Log::open removes them once it holds the lock (no compaction
// of this database can be running then). Not in the reference, whose swap_files removes the
// compacted files itself (log.rs:198-217).
static void remove_gone_files(const std::string& dir) {
  DIR* d = opendir(dir.c_str());
  if (!d) return;
  std::vector<std::string> dead;
  auto ends = [](const std::string& n, const char* suf) {
    const size_t k = strlen(suf);
    return n.size() > k && n.compare(n.size() - k, k, suf) == 0;
  };
  while (struct dirent* e = readdir(d)) {
    const std::string name = e->d_name;
    if (ends(name, ".cask.data.gone") || ends(name, ".cask.hint.gone")) dead.push_back(dir + "/" + name);
  }
  closedir(d);
  for (const std::string& f : dead) (void)unlink(f.c_str());
}

bool find_data_files(const std::string& dir, std::vector<uint32_t>& out) {
  DIR* d = opendir(dir.c_str());
  if (!d) return false;
  static const std::regex re("(\\d+).cask.data$");
  while (struct dirent* e = readdir(d)) {
    std::string name = e->d_name;
    std::string full = dir + "/" + name;
    struct stat st;
    if (lstat(full.c_str(), &st) != 0 || !S_ISREG(st.st_mode)) continue;
    std::smatch m;
    if (!std::regex_search(name, m, re)) continue;
    const std::string digits = m[1].str();
    // str::parse::<u32>: overflow -> Err -> skipped
    uint64_t v = 0;
    bool okp = true;
    for (char ch : digits) {
      v = v * 10 + (uint64_t)(ch - '0');
      if (v > 0xFFFFFFFFull) {
        okp = false;
        break;
      }
    }
    if (okp) out.push_back((uint32_t)v);
  }
  closedir(d);
  std::sort(out.begin(), out.end());
  return true;
}

using cask_host::host_threads;
using cask_host::parallel_for;

// Per file: (live entries, their bytes) over the whole keydir, counted on threads by table (a dense
// array per thread for the usual small file ids; the Stats that a sharded replay completes from it,
// cask_keydir_finish, and an owner's terms).
std::unordered_map<uint32_t, std::pair<uint64_t, uint64_t>> live_by_file(const Index& ix) {
  using Acc = std::pair<uint64_t, uint64_t>;
  constexpr uint32_t kDense = 1u << 16;
  const unsigned nt = std::max(1u, std::min(host_threads(), Index::kSub));
  std::vector<std::vector<Acc>> dense(nt);
  std::vector<std::unordered_map<uint32_t, Acc>> sparse(nt);
  parallel_for(nt, [&](unsigned t) {
    std::vector<Acc>& d = dense[t];
    for (unsigned q = t; q < Index::kSub; q += nt)
      for (const KeyDir::Slot& sl : ix.sub[q].slots) {
        if (sl.state != 1) continue;
        const uint32_t f = sl.e.file_id;
        Acc* a;
        if (f < kDense) {
          if (f >= d.size()) d.resize(std::min<size_t>(kDense, std::max<size_t>(f + 1, 2 * d.size())));
          a = &d[f];
        } else {
          a = &sparse[t][f];
        }
        a->first += 1;
        a->second += sl.e.entry_size;
      }
  });
  std::unordered_map<uint32_t, Acc> out;
  for (unsigned t = 0; t < nt; ++t) {
    for (uint32_t f = 0; f < dense[t].size(); ++f)
      if (dense[t][f].first) {
        Acc& a = out[f];
        a.first += dense[t][f].first;
        a.second += dense[t][f].second;
      }
    for (const auto& kv : sparse[t]) {
      Acc& a = out[kv.first];
      a.first += kv.second.first;
      a.second += kv.second.second;
    }
  }
  return out;
}

double ms_since(std::chrono::steady_clock::time_point t0) {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

}  // namespace

// A hint file: body + XXH32 trailer (HintWriter::drop, log.rs:389-395), created/truncated
// (util.rs:45-49), two write(2)s and no copy of the body.
bool write_file_raw2(const std::string& p, const uint8_t* b, size_t n, uint32_t trailer) {
  int fd = open(p.c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0644);
  if (fd < 0) return false;
  uint8_t t[4];
  wr32(t, trailer);
  bool ok = true;
  for (int part = 0; part < 2 && ok; ++part) {
    const uint8_t* q = part ? t : b;
    size_t m = part ? 4 : n, off = 0;
    while (off < m) {
      ssize_t w = write(fd, q + off, m - off);
      if (w < 0) {
        if (errno == EINTR) continue;
        ok = false;
        break;
      }
      off += (size_t)w;
    }
  }
  close(fd);
  return ok;
}

// A host byte buffer that is not zero-filled (a std::vector<uint8_t> of the hint bodies would write
// every byte once more before the copy from the device overwrites it).
struct RawBytes {
  std::unique_ptr<uint8_t[]> p;
  uint64_t n = 0;
  bool resize(uint64_t b) {
    p.reset(b ? new (std::nothrow) uint8_t[b] : nullptr);
    n = p || !b ? b : 0;
    return p || !b;
  }
  uint8_t* data() { return p.get(); }
  const uint8_t* data() const { return p.get(); }
  uint64_t size() const { return n; }
  bool empty() const { return n == 0; }
};

// A host buffer of anonymous memory advised to huge pages (2 MiB faults instead of 4-KiB ones when a
// multi-GiB batch is first written), unmapped when dropped.
struct HostBuf {
  uint8_t* p = nullptr;
  size_t n = 0;
  HostBuf() = default;
  HostBuf(const HostBuf&) = delete;
  HostBuf& operator=(const HostBuf&) = delete;
  HostBuf(HostBuf&& o) noexcept : p(o.p), n(o.n) {
    o.p = nullptr;
    o.n = 0;
  }
  HostBuf& operator=(HostBuf&& o) noexcept {
    if (this != &o) {
      reset();
      p = o.p;
      n = o.n;
      o.p = nullptr;
      o.n = 0;
    }
    return *this;
  }
  ~HostBuf() { reset(); }
  void reset() {
    if (p) munmap(p, n);
    p = nullptr;
    n = 0;
  }
  bool alloc(size_t bytes) {
    reset();
    void* q = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    if (q == MAP_FAILED) return false;
    (void)madvise(q, bytes, MADV_HUGEPAGE);
    p = (uint8_t*)q;
    n = bytes;
    return true;
  }
  uint8_t* get() const { return p; }
};
// A whole file into a HostBuf (no zero fill before the read, huge pages); false on an I/O error.
bool read_file_buf(const std::string& p, HostBuf& out, uint64_t& len) {
  len = 0;
  const int fd = open(p.c_str(), O_RDONLY);
  if (fd < 0) return false;
  struct stat st;
  if (fstat(fd, &st) != 0) {
    close(fd);
    return false;
  }
  if (!out.alloc(std::max<size_t>((size_t)st.st_size, 1))) {
    close(fd);
    throw std::bad_alloc();  // (mapping refused: the entry point's handler reports CASK_E_NOMEM)
  }
  uint64_t got = 0;
  while (got < (uint64_t)st.st_size) {
    const ssize_t r = read(fd, out.get() + got, (size_t)st.st_size - got);
    if (r < 0) {
      if (errno == EINTR) continue;
      close(fd);
      return false;
    }
    if (r == 0) break;
    got += (uint64_t)r;
  }
  close(fd);
  len = got;
  return true;
}

// The scan side of Cask::open on one GPU, kept per device for the life of the process (a context,
// its buffers and a ring of pinned staging buffers are created once, not per open): data files
// read by host threads into pinned buffers and copied to the device as they arrive, the device
// scan, and the hint bodies built on the device (cask_hints_device) and copied back.
struct EngineDev {
  int device = 0;
  std::mutex mu;  // one open() at a time per device
  cask_ctx* ctx = nullptr;
  struct Buf {
    uint8_t* p = nullptr;
    size_t cap = 0;
    bool ensure(size_t b) {
      if (b <= cap) return true;
      if (p) (void)hipFree(p);
      p = nullptr;
      cap = 0;
      if (hipMalloc(&p, b + b / 8 + 4096) != hipSuccess) {
        p = nullptr;
        return false;
      }
      cap = b + b / 8 + 4096;
      return true;
    }
  } data, rows, hint;
  // pinned staging: reads of data files to the device, copies of results back to the host
  cask_host::PinnedRing ring;
  // open(): hint bodies back to the host while `ring` reads files in. Hint bodies are ~1/8 of the data
  // at most (22 + key bytes per record), so 4 threads' slots (256 MiB) are made, and only when the
  // first hint copy is large enough to be staged; if they cannot be made, cask_copy carries it.
  cask_host::PinnedRing ring_out;
  bool ring_out_tried = false, ring_out_ok = false;
  static constexpr int kOutThreads = 4;
  static constexpr int kReaders = cask_host::PinnedRing::kThreads;
  static constexpr size_t kSlotBytes = cask_host::PinnedRing::kBytes;
  cask_rows r{};

  // After a large open: the data, row and hint buffers go back to the device (they are sized for
  // the largest batch or stretch seen; kept only while small, for the next open or compaction).
  void trim() {
    constexpr size_t kKeep = 4ull << 30;
    (void)hipSetDevice(device);
    for (Buf* b : {&data, &rows, &hint})
      if (b->cap > kKeep) {
        (void)hipFree(b->p);
        b->p = nullptr;
        b->cap = 0;
      }
  }

  int prepare() {
    if (hipSetDevice(device) != hipSuccess) return CASK_E_DEVICE;
    if (!ctx) {
      int st = CASK_OK;
      ctx = cask_ctx_create(device, &st);
      if (!ctx) return st;
    }
    return ring.init(device) ? CASK_OK : CASK_E_NOMEM;
  }

  // Reader thread t takes every kReaders-th 32-MiB piece of the files, alternating between its two
  // pinned slots: pread into one while the other's copy to the device is in flight.
  int read_to_device(const std::vector<std::string>& paths, const std::vector<cask_file_view>& v, std::vector<char>& ok) {
    struct Piece {
      uint32_t f;
      uint64_t off, n;
    };
    std::vector<Piece> pieces;
    for (uint32_t f = 0; f < v.size(); ++f)
      for (uint64_t o = 0; o < v[f].len; o += kSlotBytes) pieces.push_back(Piece{f, o, std::min<uint64_t>(kSlotBytes, v[f].len - o)});
    // CASK_OPEN_READERS (tuning knob): reader threads, at most kReaders (default: the host threads)
    static const unsigned readers = cask_knobs::tune("CASK_OPEN_READERS") ? (unsigned)atoi(cask_knobs::tune("CASK_OPEN_READERS")) : 0u;
    const unsigned want = readers ? std::min<unsigned>(readers, (unsigned)kReaders) : (unsigned)kReaders;
    const unsigned nt = std::max(1u, std::min<unsigned>(want, std::min<unsigned>(host_threads(), (unsigned)pieces.size())));
    std::vector<int> status(nt, CASK_OK);
    parallel_for(nt, [&](unsigned t) {
      if (hipSetDevice(device) != hipSuccess) {
        status[t] = CASK_E_DEVICE;
        return;
      }
      std::vector<int> fds(v.size(), -1);
      unsigned k = 0;
      for (size_t j = t; j < pieces.size(); j += nt, k ^= 1) {
        const Piece& pc = pieces[j];
        if (!ok[pc.f]) continue;
        if (fds[pc.f] < 0 && (fds[pc.f] = open(paths[pc.f].c_str(), O_RDONLY)) < 0) {
          ok[pc.f] = 0;
          continue;
        }
        if (hipEventSynchronize(ring.ev[t][k]) != hipSuccess) {
          status[t] = CASK_E_DEVICE;
          break;
        }
        uint64_t got = 0;
        while (got < pc.n) {
          const ssize_t m = pread(fds[pc.f], (uint8_t*)ring.pin[t][k] + got, pc.n - got, (off_t)(pc.off + got));
          if (m < 0 && errno == EINTR) continue;
          if (m <= 0) break;
          got += (uint64_t)m;
        }
        if (got != pc.n) {  // the file shrank or could not be read
          ok[pc.f] = 0;
          continue;
        }
        if (hipMemcpyAsync((uint8_t*)v[pc.f].data + pc.off, ring.pin[t][k], pc.n, hipMemcpyHostToDevice, ring.rs[t]) != hipSuccess ||
            hipEventRecord(ring.ev[t][k], ring.rs[t]) != hipSuccess) {
          status[t] = CASK_E_DEVICE;
          break;
        }
      }
      for (int fd : fds)
        if (fd >= 0) close(fd);
      if (hipStreamSynchronize(ring.rs[t]) != hipSuccess) status[t] = CASK_E_DEVICE;
    });
    for (int s : status)
      if (s != CASK_OK) return s;
    return CASK_OK;
  }

  // Device -> pageable host copy staged through the pinned slots: threads take every nt-th 32-MiB
  // piece (CASK_STAGE_MIN=0 stages every copy: the tests run the small cases through it), the DMA of one piece into a slot overlapping the host copy of the previous piece out of
  // the other (a copy to pageable memory straight from the device runs at ~10 GB/s). Small copies
  // take cask_copy. The device work that produced `src` (on the context's stream) is waited for first.
  static bool staged(uint64_t n) {
    const char* mv = cask_knobs::hook("CASK_STAGE_MIN");  // test knob: smallest copy staged (default 64 MiB)
    return n && n >= (mv ? strtoull(mv, nullptr, 10) : (64ull << 20));
  }
  int to_host(uint8_t* dst, const uint8_t* src, uint64_t n, cask_host::PinnedRing* rg = nullptr) {
    if (!staged(n)) return cask_copy(ctx, dst, src, n);
    if (hipSetDevice(device) != hipSuccess || hipStreamSynchronize((hipStream_t)cask_ctx_stream(ctx)) != hipSuccess)
      return CASK_E_DEVICE;
    std::vector<cask_host::PinnedRing::Piece> ps;
    cask_host::PinnedRing::split(dst, (uint8_t*)src, n, ps);
    return (rg ? rg : &ring)->d2h(ps) ? CASK_OK : CASK_E_DEVICE;
  }

  // open() with the keydir built on the device: every batch's rows, appended in file order (the
  // block needs the rows of all the scanned files at once; the data files stay resident anyway)
  struct AllRows {
    uint8_t* p = nullptr;
    uint64_t cap = 0, n = 0;
    ~AllRows() {
      if (p) (void)hipFree(p);
    }
    static uint64_t a(uint64_t c, uint32_t w) { return (c * w + 255) & ~255ull; }
    cask_rows view() const {
      cask_rows r{};
      r.capacity = cap;
      r.count = n;
      r.pos = (uint64_t*)p;
      r.seq = (uint64_t*)(p + a(cap, 8));
      r.vsz = (uint32_t*)(p + 2 * a(cap, 8));
      r.ksz = (uint16_t*)(p + 2 * a(cap, 8) + a(cap, 4));
      r.status = p + 2 * a(cap, 8) + a(cap, 4) + a(cap, 2);
      return r;
    }
    // rows [0, m) of `src` after the n already here (the buffer grows by half again when short)
    int append(const cask_rows& src, uint64_t m, hipStream_t st) {
      if (n + m > cap) {
        const uint64_t nc = std::max<uint64_t>(n + m, cap + cap / 2);
        uint8_t* q = nullptr;
        if (hipMalloc(&q, 2 * a(nc, 8) + a(nc, 4) + a(nc, 2) + nc + 256) != hipSuccess) return CASK_E_NOMEM;
        AllRows grown;
        grown.p = q;
        grown.cap = nc;
        if (n) {
          const cask_rows o = view(), g = grown.view();
          if (hipMemcpyAsync(g.pos, o.pos, 8 * n, hipMemcpyDeviceToDevice, st) != hipSuccess ||
              hipMemcpyAsync(g.seq, o.seq, 8 * n, hipMemcpyDeviceToDevice, st) != hipSuccess ||
              hipMemcpyAsync(g.vsz, o.vsz, 4 * n, hipMemcpyDeviceToDevice, st) != hipSuccess ||
              hipMemcpyAsync(g.ksz, o.ksz, 2 * n, hipMemcpyDeviceToDevice, st) != hipSuccess ||
              hipMemcpyAsync(g.status, o.status, n, hipMemcpyDeviceToDevice, st) != hipSuccess ||
              hipStreamSynchronize(st) != hipSuccess)
            return CASK_E_DEVICE;
        }
        std::swap(p, grown.p);
        std::swap(cap, grown.cap);
      }
      const cask_rows d = view();
      if (m && (hipMemcpyAsync(d.pos + n, src.pos, 8 * m, hipMemcpyDeviceToDevice, st) != hipSuccess ||
                hipMemcpyAsync(d.seq + n, src.seq, 8 * m, hipMemcpyDeviceToDevice, st) != hipSuccess ||
                hipMemcpyAsync(d.vsz + n, src.vsz, 4 * m, hipMemcpyDeviceToDevice, st) != hipSuccess ||
                hipMemcpyAsync(d.ksz + n, src.ksz, 2 * m, hipMemcpyDeviceToDevice, st) != hipSuccess ||
                hipMemcpyAsync(d.status + n, src.status, m, hipMemcpyDeviceToDevice, st) != hipSuccess ||
                hipStreamSynchronize(st) != hipSuccess))
        return CASK_E_DEVICE;
      n += m;
      return CASK_OK;
    }
  };

  // Device rows sized from a guess (average record >= 48 B), once more at the exact count if short.
  int scan(const std::vector<cask_file_view>& v, std::vector<uint64_t>& row_off, cask_scan_error& se) {
    uint64_t total = 0;
    for (const auto& f : v) total += f.len;
    const uint64_t bound = cask_rows_bound(v.data(), (uint32_t)v.size());
    uint64_t cap = std::min<uint64_t>(bound, total / 48 + v.size() + 1024);
    for (int attempt = 0; attempt < 2; ++attempt) {
      const uint64_t a8 = (cap * 8 + 255) & ~255ull, a4 = (cap * 4 + 255) & ~255ull, a2 = (cap * 2 + 255) & ~255ull;
      if (!rows.ensure(2 * a8 + a4 + a2 + cap + 256)) return CASK_E_NOMEM;
      r = cask_rows{};
      r.capacity = cap;
      r.pos = (uint64_t*)rows.p;
      r.seq = (uint64_t*)(rows.p + a8);
      r.vsz = (uint32_t*)(rows.p + 2 * a8);
      r.ksz = (uint16_t*)(rows.p + 2 * a8 + a4);
      r.status = rows.p + 2 * a8 + a4 + a2;
      const int st = cask_scan_device(ctx, v.data(), (uint32_t)v.size(), &r, row_off.data(), &se);
      if (st != CASK_E_CAPACITY) return st;
      cap = r.count;
    }
    return CASK_E_DEVICE;
  }

  // The hint bodies of the scanned files v (rows of the last scan) into hbuf, file k's at
  // [fo[k], fo[k + 1]); copied back through ring_out (open() reads the next files through `ring`).
  int hints(const std::vector<cask_file_view>& v, const std::vector<uint64_t>& row_off, RawBytes& hbuf,
            std::vector<uint64_t>& fo) {
    fo.assign(v.size() + 1, 0);
    int st = cask_hints_device(ctx, v.data(), (uint32_t)v.size(), &r, row_off.data(), nullptr, 0, fo.data());
    if (st != CASK_E_CAPACITY && st != CASK_OK) return st;
    if (!hint.ensure(fo[v.size()] + 256)) return CASK_E_NOMEM;
    st = cask_hints_device(ctx, v.data(), (uint32_t)v.size(), &r, row_off.data(), hint.p, hint.cap, fo.data());
    if (st != CASK_OK) return st;
    if (!hbuf.resize(fo[v.size()])) return CASK_E_NOMEM;
    if (hbuf.empty()) return CASK_OK;
    if (staged(hbuf.size()) && !ring_out_tried) {
      ring_out_tried = true;
      ring_out_ok = ring_out.init(device, kOutThreads);
      if (!ring_out_ok) ring_out.release();
    }
    if (staged(hbuf.size()) && !ring_out_ok) return cask_copy(ctx, hbuf.data(), hint.p, hbuf.size());
    return to_host(hbuf.data(), hint.p, hbuf.size(), &ring_out) != CASK_OK ? CASK_E_DEVICE : CASK_OK;
  }
};

EngineDev* engine_dev(int device) {
  static std::mutex mu;
  static EngineDev* devs[64] = {};
  if (device < 0 || device >= 64) return nullptr;
  std::lock_guard<std::mutex> g(mu);
  if (!devs[device]) {
    devs[device] = new (std::nothrow) EngineDev();
    if (devs[device]) devs[device]->device = device;
  }
  return devs[device];
}

constexpr uint64_t kFoldPiece = 1ull << 19;  // records per fold source (pass 1's unit of work)

// A stretch of a hint body (Hint::write_bytes records, data.rs:242-256: seq u64, ksz u16, vsz u32,
// pos u64, key) holding `cnt` whole records, all of one file: what the replay folds, in order.
struct FoldSrc {
  const uint8_t* b;
  uint64_t n, cnt;
  uint32_t file_id;
};

// One record on its way to its keydir table: everything Index::update reads, key bytes included
// when short, so the table's fold streams its list and touches only its own slots.
struct FoldItem {
  uint64_t hash, seq, pos;
  uint32_t file_id, vsz_raw, ksz, pad;
  union {
    uint8_t kin[KeyDir::kInline];
    const uint8_t* kp;  // ksz > kInline: the key in its hint body
  };
  const uint8_t* key() const { return ksz <= KeyDir::kInline ? kin : kp; }
};

// Index::update over the hint records of `src` in order (the open replay, cask.rs:346-382;
// compact_files' re-index, cask.rs:528-536), on threads by key-hash table. Index::update's outcome
// for a key depends only on that key's records in order, and each table sees its keys' records in
// replay order. Pass 1 (threads by source) hashes every key and appends the record to its
// (source, table) list; pass 2 (threads by table) folds each table's lists in source order. Stats
// rows are per-file counters (order-free sums): each table keeps deltas, summed at the end; a remove
// counts when its file has a row in the delta or in the map entering the fold. The two differ from
// one serial fold only if a key's entry pointed at a file with no stats row, which cannot happen:
// every entry's file got its row when the entry was written, and compaction drops a file's row only
// after re-indexing all of its live entries elsewhere. Small replays fold on the calling thread.
// Pass 1's lists, kept across the batches of one open() so that later batches reuse their pages.
struct FoldScratch {
  std::vector<std::vector<FoldItem>> lists;
  std::vector<uint8_t> hll;
};

void parallel_fold(const std::vector<FoldSrc>& src, Index& out, FoldScratch* keep = nullptr) {
  uint64_t n = 0;
  for (const FoldSrc& f : src) n += f.cnt;
  const char* mv = cask_knobs::hook("CASK_PAR_FOLD_MIN");  // tuning/test knob: smallest replay folded in parallel
  const uint64_t min_par = mv ? strtoull(mv, nullptr, 10) : (1ull << 16);
  const unsigned nt = std::min(host_threads(), Index::kSub);
  if (n < min_par || nt == 1) {
    StatsDelta sd(out.stats, nullptr);
    for (const FoldSrc& f : src)
      for (uint64_t p = 0, j = 0; j < f.cnt; ++j) {
        const uint8_t* h = f.b + p;
        const uint16_t k = rd16(h + 8);
        const uint64_t hs = hash_key(h + 22, k);
        out.sub[Index::sub_of(hs)].update(h + 22, k, f.file_id, rd64(h + 14), rd32(h + 10), rd64(h), hs, sd);
        p += 22ull + k;
      }
    return;
  }
  constexpr unsigned S = Index::kSub;
  const size_t ns = src.size();
  // 1. per (source, table) lists, sources claimed by threads
  FoldScratch local;
  FoldScratch& fs = keep ? *keep : local;
  if (fs.lists.size() < ns * S) fs.lists.resize(ns * S);
  std::vector<std::vector<FoldItem>>& lists = fs.lists;
  // and per (source, table) a 256-register HyperLogLog sketch of the keys (hash bits below the
  // table's), so that each table is sized once for the keys it will hold: a table sized from the
  // record count instead (configs[3]: 5 records per key) costs pass 2 a third more in page faults
  // and cache misses, one sized too small a rehash per doubling.
  constexpr unsigned kReg = 256;
  std::vector<uint8_t>& hll = fs.hll;
  hll.assign(ns * S * kReg, 0);
  std::atomic<size_t> next{0};
  parallel_for(nt, [&](unsigned) {
    for (size_t k; (k = next.fetch_add(1)) < ns;) {
      const FoldSrc& f = src[k];
      std::vector<FoldItem>* L = &lists[k * S];
      for (unsigned q = 0; q < S; ++q) {
        L[q].clear();
        L[q].reserve(f.cnt / S + f.cnt / (4 * S) + 16);
      }
      for (uint64_t p = 0, j = 0; j < f.cnt; ++j) {
        const uint8_t* h = f.b + p;
        FoldItem it;
        it.ksz = rd16(h + 8);
        it.hash = hash_key(h + 22, it.ksz);
        it.seq = rd64(h);
        it.pos = rd64(h + 14);
        it.file_id = f.file_id;
        it.vsz_raw = rd32(h + 10);
        it.pad = 0;
        if (it.ksz <= KeyDir::kInline) {  // (16 bytes at once unless that would pass the body's end)
          if (p + 22 + KeyDir::kInline <= f.n) memcpy(it.kin, h + 22, KeyDir::kInline);
          else memcpy(it.kin, h + 22, it.ksz);
        } else {
          it.kp = h + 22;
        }
        const unsigned q = Index::sub_of(it.hash);
        L[q].push_back(it);
        uint8_t& reg = hll[(k * S + q) * kReg + ((it.hash >> 50) & (kReg - 1))];
        const uint8_t rank = (uint8_t)(__builtin_clzll((it.hash << 14) | (1ull << 13)) + 1);
        reg = rank > reg ? rank : reg;
        p += 22ull + it.ksz;
      }
    }
  });
  // 2. each table folds its lists in source order, stats into its own delta map
  std::vector<StatsMap> delta(S);
  parallel_for(nt, [&](unsigned t) {
    for (unsigned q = t; q < S; q += nt) {
      KeyDir& kd = out.sub[q];
      uint64_t cnt = 0;
      for (size_t k = 0; k < ns; ++k) cnt += lists[k * S + q].size();
      {  // the sketches of the table's lists merged: an estimate of its distinct keys (+-7 %)
        uint8_t m[kReg] = {};
        for (size_t k = 0; k < ns; ++k) {
          const uint8_t* r = &hll[(k * S + q) * kReg];
          for (unsigned j = 0; j < kReg; ++j) m[j] = r[j] > m[j] ? r[j] : m[j];
        }
        double z = 0;
        unsigned zeros = 0;
        for (unsigned j = 0; j < kReg; ++j) {
          z += std::ldexp(1.0, -(int)m[j]);
          zeros += m[j] == 0;
        }
        double est = 0.7213 / (1 + 1.079 / kReg) * kReg * kReg / z;
        if (est < 2.5 * kReg && zeros) est = kReg * std::log((double)kReg / zeros);
        const uint64_t want = std::min<uint64_t>(cnt, (uint64_t)(est * 1.15) + 64);
        // A fresh table is sized for its keys at once. A table holding keys grows when it fills
        // (update()): how many of the batch's keys it holds already is not known here, and sizing
        // for all of them as new rebuilt every table of compact_files' re-index, whose keys are all
        // in the keydir (0.36 -> 0.63-0.74 s on configs[3], profiles/r06k_compaction_ab.txt).
        if (!kd.live) kd.reserve(want);
      }
      StatsDelta sd(delta[q], &out.stats);
      for (size_t k = 0; k < ns; ++k) {
        const std::vector<FoldItem>& L = lists[k * S + q];
        const size_t m = L.size();
        for (size_t j = 0; j < m; ++j) {  // the slot of the record 8 ahead, a long key 4 ahead
          if (j + 16 < m) kd.prefetch(L[j + 16].hash);
          if (j + 4 < m) kd.prefetch_key(L[j + 4].hash);
          const FoldItem& r = L[j];
          kd.update(r.key(), r.ksz, r.file_id, r.pos, r.vsz_raw, r.seq, r.hash, sd);
        }
        if (!keep) std::vector<FoldItem>().swap(lists[k * S + q]);
      }
    }
  });
  // 3. stats deltas
  for (const StatsMap& d : delta)
    for (const auto& kv : d) {
      StatsEntry& e = out.stats[kv.first];
      e.entries += kv.second.entries;
      e.dead_entries += kv.second.dead_entries;
      e.dead_bytes += kv.second.dead_bytes;
    }
}

struct cask_db {
  std::string path;
  cask_options opts{};
  int lock_fd = -1;
  std::vector<uint32_t> files;
  Index index;
  uint64_t sequence = 0;
  uint32_t file_seq = 0;  // Log::file_id_seq: the last data file id at open (log.rs:63-69)
  double timings[5] = {0, 0, 0, 0, 0};
  // sharded replay (cask_keydir_merge): per-file order-free stats terms, summed over shards
  struct ShardTerms {
    uint64_t puts = 0, put_bytes = 0, stale = 0, stale_bytes = 0;
  };
  std::unordered_map<uint32_t, ShardTerms> terms;
  bool merging = false;
  uint32_t shards = 0;
  // the merge's scratch (key hashes, items), kept from block to block and given back after the
  // last one (cask_keydir_finish), off the calling thread
  HostBuf mhash, mitems;
  // Host buffers of GiBs given back on threads of the db's own (unmapping them takes a while and
  // nothing waits for it: a thread per discard, each owning what it unmaps), all joined at close;
  // here when no thread can be had.
  std::vector<std::thread> gone_th;
  void discard(std::initializer_list<HostBuf*> bs) {
    std::vector<HostBuf> g;
    for (HostBuf* b : bs)
      if (b->p) g.push_back(std::move(*b));
    if (g.empty()) return;
    try {
      gone_th.emplace_back([v = std::move(g)]() mutable { v.clear(); });
    } catch (...) {
    }  // (g, if not moved into a thread, is unmapped here)
  }
  // the bytes of files a compaction took out of the database, released on a thread of their own
  // (joined before the next compaction and at close)
  std::thread reclaim;
  void reclaim_join() {
    if (reclaim.joinable()) reclaim.join();
  }
  ~cask_db() {
    reclaim_join();
    for (std::thread& t : gone_th)
      if (t.joinable()) t.join();
    if (lock_fd >= 0) {
      flock(lock_fd, LOCK_UN);  // Drop for Log (log.rs:225-229)
      close(lock_fd);
    }
  }
};

extern "C" {

void cask_options_default(cask_options* o) {
  if (!o) return;
  memset(o, 0, sizeof(*o));
  o->create = 1;
  o->write_hints = 1;
  o->max_file_size = 2ull * 1024 * 1024 * 1024;  // cask.rs:225
  o->device = 0;
}

static void set_err(cask_open_error* err, int status, uint32_t fid = 0, uint64_t pos = 0, uint32_t e = 0,
                    uint32_t f = 0) {
  if (!err) return;
  err->status = status;
  err->file_id = fid;
  err->pos = pos;
  err->expected = e;
  err->found = f;
}

// No C++ exception crosses the C ABI (cask_scan.h): the entry points that allocate or start threads
// run their bodies under these guards — std::bad_alloc (host memory pressure: a huge hint file, a
// keydir at cfg5 scale) is CASK_E_NOMEM, anything else (std::system_error from a thread or a mutex)
// CASK_E_IO. parallel_for (host_ring.h) carries a worker's exception back to its caller, and the open
// pipeline's threads turn theirs into a batch status, so every exception ends up here.
extern "C++" {  // (templates; this part of the file is inside the extern "C" block)
template <class F>
static auto abi_status(F&& f) noexcept -> decltype(f()) {
  return cask_abi::guard(static_cast<F&&>(f));
}
template <class F>
static cask_db* abi_db(cask_open_error* err, F&& f) noexcept {
  try {
    return f();
  } catch (const std::bad_alloc&) {
    set_err(err, CASK_E_NOMEM);
  } catch (...) {
    set_err(err, CASK_E_IO);
  }
  return nullptr;
}
}  // extern "C++"

// Log::open (log.rs:36-85): path checks, the lock file, the data files in id order. Returns the
// handle (no keydir yet) or NULL with *err set.
static cask_db* open_log(const char* path_c, const cask_options* opts_in, cask_open_error* err) {
  set_err(err, CASK_OK);
  if (!path_c) {
    set_err(err, CASK_E_INVALID_ARG);
    return nullptr;
  }
  cask_options opts;
  if (opts_in) opts = *opts_in; else cask_options_default(&opts);
  std::string path = path_c;
  // Log::open path checks (log.rs:46-56)
  if (opts.create) {
    if (exists(path) && !is_dir(path)) {
      set_err(err, CASK_E_INVALID_PATH);
      return nullptr;
    }
    if (!exists(path) && mkdir(path.c_str(), 0755) != 0) {
      set_err(err, CASK_E_IO);
      return nullptr;
    }
  } else if (!exists(path) || !is_dir(path)) {
    set_err(err, CASK_E_INVALID_PATH);
    return nullptr;
  }
  cask_db* db = new (std::nothrow) cask_db();
  if (!db) {
    set_err(err, CASK_E_NOMEM);
    return nullptr;
  }
  db->path = path;
  db->opts = opts;
  // File::create("cask.lock") + try_lock_exclusive (log.rs:58-59)
  db->lock_fd = open((path + "/cask.lock").c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0644);
  if (db->lock_fd < 0) {
    delete db;
    set_err(err, CASK_E_IO);
    return nullptr;
  }
  if (flock(db->lock_fd, LOCK_EX | LOCK_NB) != 0) {
    close(db->lock_fd);
    db->lock_fd = -1;
    delete db;
    set_err(err, CASK_E_LOCKED);
    return nullptr;
  }
  remove_gone_files(path);
  if (!find_data_files(path, db->files)) {
    delete db;
    set_err(err, CASK_E_IO);
    return nullptr;
  }
  db->file_seq = db->files.empty() ? 0u : db->files.back();
  return db;
}

static cask_db* db_open_impl(const char* path_c, const cask_options* opts_in, cask_open_error* err);
cask_db* cask_db_open(const char* path_c, const cask_options* opts_in, cask_open_error* err) {
  return abi_db(err, [&] { return db_open_impl(path_c, opts_in, err); });
}

static cask_db* db_open_impl(const char* path_c, const cask_options* opts_in, cask_open_error* err) {
  auto t0 = std::chrono::steady_clock::now();
  std::unique_ptr<cask_db> own(open_log(path_c, opts_in, err));  // (deleted on every failure: the lock goes)
  cask_db* db = own.get();
  if (!db) return nullptr;
  const cask_options opts = db->opts;
  const std::string path = db->path;

  // Which files have a valid hint file (log.rs:121-135, 512-539)? The others are scanned.
  const size_t nf = db->files.size();
  std::vector<std::vector<uint8_t>> hints(nf);
  std::vector<char> use_hint(nf, 0), data_ok(nf, 1);
  std::vector<uint32_t> scan_idx;
  std::vector<uint64_t> flen(nf, 0);
  {  // hint files read and checked on threads
    const unsigned nt = std::max(1u, std::min<unsigned>(host_threads(), (unsigned)nf));
    parallel_for(nt, [&](unsigned t) {
      for (size_t i = t; i < nf; i += nt) {
        const std::string hp = hint_path(path, db->files[i]);
        if (is_file_follow(hp) && read_file(hp, hints[i]) && hints[i].size() >= 4) {
          const size_t n = hints[i].size();
          if (cask_xxh::xxh32(hints[i].data(), n - 4, 0) == rd32(hints[i].data() + n - 4)) {
            use_hint[i] = 1;
            continue;
          }
        }
        std::vector<uint8_t>().swap(hints[i]);
      }
    });
  }
  for (size_t i = 0; i < nf; ++i) {
    if (use_hint[i]) continue;
    struct stat stt;
    if (stat(data_path(path, db->files[i]).c_str(), &stt) != 0) data_ok[i] = 0;
    else flen[i] = (uint64_t)stt.st_size;
    scan_idx.push_back((uint32_t)i);
  }

  // The scanned files, in batches of consecutive files (an eighth of their bytes each, at least
  // 1 GiB): a reader thread reads batch b + 1 from disk straight to the device (host threads,
  // pinned buffers) while a device thread scans batch b and brings its hint bodies back (built on
  // the device, cask_hints_device), and this thread replays the batches before it in file order —
  // the fold and the hint files. The host never holds the data bytes, only the hint records it
  // writes and folds.
  std::vector<cask_file_view> views;
  std::vector<uint32_t> view_file;
  std::vector<int64_t> view_of(nf, -1);
  for (uint32_t i : scan_idx)
    if (data_ok[i]) {
      view_of[i] = (int64_t)views.size();
      views.push_back(cask_file_view{db->files[i], CASK_VIEW_DEVICE, nullptr, flen[i]});
      view_file.push_back(i);
    }
  std::vector<size_t> vcut{0};
  {
    uint64_t all = 0, acc = 0;
    for (const auto& v : views) all += v.len;
    // CASK_OPEN_BATCH (test and tuning knob): bytes per batch (1: every file a batch of its own)
    const uint64_t bb_env = cask_knobs::hook("CASK_OPEN_BATCH") ? strtoull(cask_knobs::hook("CASK_OPEN_BATCH"), nullptr, 10) : 0ull;
    const uint64_t bb = bb_env ? bb_env : std::max<uint64_t>(1ull << 30, all / 8);
    for (size_t v = 0; v < views.size(); ++v) {
      acc += views[v].len;
      if (acc >= bb && v + 1 < views.size()) {
        vcut.push_back(v + 1);
        acc = 0;
      }
    }
    vcut.push_back(views.size());
  }
  const size_t nbat = vcut.size() - 1;
  // Every file scanned (no valid hint file): the keydir is reduced on the device — each batch's rows
  // kept, and after the last batch one block of the whole replay (cask_shard_keydir: per key only the
  // records that can decide the final keydir; configs[3]: a fifth of the records) that this thread
  // merges (cask_keydir_merge + cask_keydir_finish, as the multi-GPU open folds its ranges' blocks)
  // instead of folding every hint record. A replay that also has hint files folds on the host
  // (CASK_OPEN_DEVFOLD=0, a test hook, forces the host fold).
  const char* dfh = cask_knobs::hook("CASK_OPEN_DEVFOLD");
  const bool dev_fold = !views.empty() && scan_idx.size() == nf && !(dfh && !strcmp(dfh, "0"));
  std::vector<uint64_t> roff_all(views.size() + 1, 0);  // (dev_fold) each view's first row
  EngineDev::AllRows all_rows;
  HostBuf dblock;               // (dev_fold) the block, on the host (huge pages: the copy faults 2-MiB pages)
  double t_blk = 0, t_blk_d2h = 0;  // (dev_fold) its build on the device, its copy to the host
  uint64_t dblock_n = 0;        // (dev_fold) its bytes
  int dblock_st = CASK_E_IO;    // (dev_fold) CASK_OK once the block is here
  bool dblock_done = false;
  struct Batch {
    RawBytes hb;                // hint bodies of the batch's files
    std::vector<uint64_t> fo;   // view k of the batch: hb[fo[k], fo[k + 1])
    cask_scan_error se{};
    int st = CASK_OK;
    bool read_done = false, ready = false;
  };
  std::vector<Batch> bat(nbat);
  std::mutex bm;
  std::condition_variable bcv;
  std::atomic<bool> stop{false};
  double t_read = 0, t_dev = 0;
  EngineDev* ed = nullptr;
  std::unique_lock<std::mutex> edlock;
  int dst = CASK_OK;
  if (!views.empty()) {
    ed = engine_dev(opts.device);
    if (!ed) {
      set_err(err, CASK_E_DEVICE);
      return nullptr;
    }
    edlock = std::unique_lock<std::mutex>(ed->mu);
    dst = ed->prepare();
    std::vector<uint64_t> doff(views.size() + 1, 0);
    for (size_t v = 0; v < views.size(); ++v) doff[v + 1] = doff[v] + ((views[v].len + 255) & ~255ull);
    if (dst == CASK_OK && !ed->data.ensure(doff.back() + 256)) dst = CASK_E_NOMEM;
    if (dst == CASK_OK)
      for (size_t v = 0; v < views.size(); ++v) views[v].data = ed->data.p + doff[v];
  }
  auto mark = [&](size_t b, int st, bool ready) {
    {
      std::lock_guard<std::mutex> g(bm);
      if (st != CASK_OK && bat[b].st == CASK_OK) bat[b].st = st;
      (ready ? bat[b].ready : bat[b].read_done) = true;
    }
    bcv.notify_all();
  };
  // (the two pipeline threads catch their own exceptions: a batch that throws gets a status, and
  // every batch is still marked, so nobody waits forever and the threads can be joined)
  auto reader = [&]() {
    const auto tr = std::chrono::steady_clock::now();
    for (size_t b = 0; b < nbat; ++b) {
      int st = dst;
      if (st == CASK_OK && !stop.load() && vcut[b + 1] > vcut[b]) {
        st = abi_status([&] {
          std::vector<std::string> paths;
          std::vector<cask_file_view> vb(views.begin() + (ptrdiff_t)vcut[b], views.begin() + (ptrdiff_t)vcut[b + 1]);
          for (size_t v = vcut[b]; v < vcut[b + 1]; ++v) paths.push_back(data_path(path, db->files[view_file[v]]));
          std::vector<char> ok(vb.size(), 1);
          const int rs = ed->read_to_device(paths, vb, ok);
          for (size_t k = 0; k < vb.size(); ++k)
            if (!ok[k]) {  // the file could not be read whole: Log::entries' Io error when its turn comes
              data_ok[view_file[vcut[b] + k]] = 0;
              views[vcut[b] + k].len = 0;
            }
          return rs;
        });
      }
      mark(b, st, false);
    }
    t_read = ms_since(tr);
  };
  auto device = [&]() {
    for (size_t b = 0; b < nbat; ++b) {
      {
        std::unique_lock<std::mutex> lk(bm);
        bcv.wait(lk, [&] { return bat[b].read_done; });
      }
      const auto td = std::chrono::steady_clock::now();
      int st = bat[b].st;
      if (st == CASK_OK && !stop.load() && vcut[b + 1] > vcut[b]) {
        st = abi_status([&] {
          std::vector<cask_file_view> vb(views.begin() + (ptrdiff_t)vcut[b], views.begin() + (ptrdiff_t)vcut[b + 1]);
          std::vector<uint64_t> ro(vb.size() + 1);
          int ds = ed->scan(vb, ro, bat[b].se);
          // the hint bodies: for the hint files, and for the host fold (with the keydir reduced on
          // the device and no hint files to write, none)
          if (ds == CASK_OK && dev_fold && !opts.write_hints) bat[b].fo.assign(vb.size() + 1, 0);
          else if (ds == CASK_OK) ds = ed->hints(vb, ro, bat[b].hb, bat[b].fo);
          if (ds == CASK_OK && dev_fold && !bat[b].se.kind) {  // the batch's rows, kept for the block
            for (size_t k = 0; k <= vb.size(); ++k) roff_all[vcut[b] + k] = all_rows.n + ro[k];
            ds = all_rows.append(ed->r, ro[vb.size()], (hipStream_t)cask_ctx_stream(ed->ctx));
          }
          return ds;
        });
      }
      t_dev += ms_since(td);
      mark(b, st, true);
    }
    // (dev_fold) every batch scanned clean: the replay's block, reduced on the device, to the host
    bool clean = dev_fold;
    for (size_t b = 0; b < nbat && clean; ++b) clean = bat[b].st == CASK_OK && !bat[b].se.kind && !stop.load();
    int bs = CASK_E_IO;
    if (clean) {
      const auto td = std::chrono::steady_clock::now();
      bs = abi_status([&] {
        const cask_rows r = all_rows.view();
        const void* blk = nullptr;
        uint64_t nb = 0;
        int st = cask_shard_keydir(ed->ctx, views.data(), (uint32_t)views.size(), &r, roff_all.data(), &blk, &nb);
        if (st != CASK_OK) return st;
        t_blk = ms_since(td);
        const auto tc = std::chrono::steady_clock::now();
        if (!dblock.alloc(std::max<uint64_t>(nb, 1))) return (int)CASK_E_NOMEM;
        dblock_n = nb;
        st = ed->to_host(dblock.get(), (const uint8_t*)blk, nb);
        t_blk_d2h = ms_since(tc);
        return st;
      });
      t_dev += ms_since(td);
    }
    {
      std::lock_guard<std::mutex> g(bm);
      dblock_st = bs;
      dblock_done = true;
    }
    bcv.notify_all();
  };
  std::thread th_read, th_dev;
  bool threaded = false;
  if (!views.empty()) {
    try {
      th_read = std::thread(reader);
      try {
        th_dev = std::thread(device);
        threaded = true;
      } catch (...) {
        stop = true;  // (the reader marks every batch and ends)
        th_read.join();
      }
    } catch (...) {
    }
    if (!threaded) {  // no threads to be had: the same steps, one after the other
      stop = false;
      for (auto& bt : bat) bt = Batch();
      reader();
      device();
    }
  } else {
    for (size_t b = 0; b < nbat; ++b) bat[b].read_done = bat[b].ready = true;
    dblock_done = true;
  }
  auto join_all = [&]() {
    stop = true;
    if (th_read.joinable()) th_read.join();
    if (th_dev.joinable()) th_dev.join();
  };
  // an exception in the replay below (std::bad_alloc in the fold) unwinds through here: the pipeline
  // threads are stopped and joined before anything they use goes away
  struct JoinOnExit {
    decltype(join_all)& f;
    ~JoinOnExit() { f(); }
  } join_on_exit{join_all};
  db->timings[0] = ms_since(t0);  // (until the replay starts; the reads' own span is added below)

  // Replay in ascending file order (cask.rs:348-369), batch after batch; the first Err aborts open().
  // Hint files of the scanned files up to that point are written on threads: each is its body +
  // XXH32 trailer (RecreateHints keeps draining after an error, so a failing file's hint file has
  // every Ok row).
  double t_fold = 0, t_hint = 0;
  int fail = CASK_OK;
  uint32_t fail_fid = 0;
  uint64_t fail_pos = 0;
  uint32_t fail_e = 0, fail_f = 0;
  // each file's hint body (a hint file's, or the one built for a scanned file), walked on threads:
  // its record count, highest sequence and first short read (Hints::next / Hint::from_read,
  // log.rs:437-447; data.rs:258-276)
  struct Body {
    const uint8_t* b = nullptr;
    uint64_t n = 0, cnt = 0, max_seq = 0, bad = UINT64_MAX;
    std::vector<uint64_t> cut;  // the offset of every kPiece-th record: the fold's sources
  };
  constexpr uint64_t kPiece = kFoldPiece;
  std::vector<Body> bodies(nf);
  const unsigned ntb = std::max(1u, std::min<unsigned>(host_threads(), (unsigned)std::max<size_t>(nf, 1)));
  size_t fi = 0;  // the next file to replay
  FoldScratch fscratch;
  for (size_t b = 0; b < nbat && fail == CASK_OK; ++b) {
    {
      std::unique_lock<std::mutex> lk(bm);
      bcv.wait(lk, [&] { return bat[b].ready; });
    }
    if (bat[b].st != CASK_OK) {
      fail = bat[b].st;
      break;
    }
    const size_t fe = b + 1 < nbat ? (size_t)view_file[vcut[b + 1] - 1] + 1 : nf;
    uint32_t err_file = UINT32_MAX;  // the batch's first failing record is in this file
    if (bat[b].se.kind)
      for (size_t v = vcut[b]; v < vcut[b + 1]; ++v)
        if (views[v].file_id == bat[b].se.file_id) err_file = view_file[v];
    auto tf = std::chrono::steady_clock::now();
    for (size_t i = fi; i < fe; ++i) {
      if (use_hint[i]) {
        bodies[i].b = hints[i].data();
        bodies[i].n = hints[i].size() - 4;  // Take(size - 4) (log.rs:129)
      } else if (data_ok[i] && view_of[i] >= 0) {
        const size_t k = (size_t)view_of[i] - vcut[b];
        bodies[i].b = bat[b].hb.data() + bat[b].fo[k];
        bodies[i].n = bat[b].fo[k + 1] - bat[b].fo[k];
      }
    }
    const unsigned nt = std::max(1u, std::min<unsigned>(ntb, (unsigned)std::max<size_t>(fe - fi, 1)));
    // (dev_fold: the bodies were built on the device from the scan's rows — whole records, and the
    // block carries the highest sequence — so only their hint files are written below)
    if (!dev_fold) parallel_for(nt, [&](unsigned t) {
      for (size_t i = fi + t; i < fe; i += nt) {
        Body& B = bodies[i];
        B.cut.clear();
        for (uint64_t p = 0; p < B.n;) {
          if (B.n - p < 22 || B.n - p - 22 < rd16(B.b + p + 8)) {
            B.bad = p;
            break;
          }
          if (!(B.cnt & (kPiece - 1))) B.cut.push_back(p);
          B.max_seq = std::max(B.max_seq, rd64(B.b + p));
          ++B.cnt;
          p += 22ull + rd16(B.b + p + 8);
        }
      }
    });
    size_t nrep = fi;  // files of the batch replayed: [fi, nrep)
    std::vector<uint32_t> to_write;
    for (size_t i = fi; i < fe && fail == CASK_OK; ++i) {
      const uint32_t fid = db->files[i];
      if (!use_hint[i]) {
        if (!data_ok[i]) {
          // HintWriter::new truncated the hint file before Log::entries failed; its Drop then wrote
          // the trailer of an empty body (log.rs:141-142, 389-395).
          if (opts.write_hints) write_file(hint_path(path, fid), {}, cask_xxh::xxh32(nullptr, 0, 0));
          fail = CASK_E_IO;
          fail_fid = fid;
          break;
        }
        if (opts.write_hints) to_write.push_back((uint32_t)i);
        if (err_file == i) {
          const cask_scan_error& se = bat[b].se;
          fail = se.kind == CASK_ROW_CHECKSUM ? CASK_E_CHECKSUM : CASK_E_EOF;
          fail_fid = fid;
          fail_pos = se.pos;
          fail_e = se.expected;
          fail_f = se.found;
          break;
        }
      }
      if (bodies[i].bad != UINT64_MAX) {
        fail = CASK_E_EOF;
        fail_fid = fid;
        fail_pos = bodies[i].bad;
        break;
      }
      if (bodies[i].cnt && bodies[i].max_seq > db->sequence) db->sequence = bodies[i].max_seq;
      nrep = i + 1;
    }
    // the batch's fold sources, in order: pieces of kPiece records of each replayed file's body
    std::vector<FoldSrc> srcs;
    if (fail == CASK_OK)
      for (size_t i = fi; i < nrep; ++i) {
        const Body& B = bodies[i];
        for (size_t c = 0; c < B.cut.size(); ++c) {
          const uint64_t e = c + 1 < B.cut.size() ? B.cut[c + 1] : B.n;
          const uint64_t k = c + 1 < B.cut.size() ? kPiece : B.cnt - c * kPiece;
          srcs.push_back(FoldSrc{B.b + B.cut[c], e - B.cut[c], k, db->files[i]});
        }
      }
    t_fold += ms_since(tf);
    auto th = std::chrono::steady_clock::now();
    {
      std::vector<char> wok(to_write.size(), 1);
      const unsigned nw = std::max(1u, std::min<unsigned>(host_threads(), (unsigned)to_write.size()));
      parallel_for(nw, [&](unsigned t) {
        for (size_t j = t; j < to_write.size(); j += nw) {
          const Body& B = bodies[to_write[j]];
          wok[j] = write_file_raw2(hint_path(path, db->files[to_write[j]]), B.b, B.n, cask_xxh::xxh32(B.b, B.n, 0));
        }
      });
      for (size_t j = 0; j < to_write.size() && fail == CASK_OK; ++j)
        if (!wok[j]) {
          fail = CASK_E_IO;
          fail_fid = db->files[to_write[j]];
        }
    }
    t_hint += ms_since(th);
    if (fail != CASK_OK) break;
    // Index::update + Stats over the batch's records (their keys stay in hints[] / the batch's
    // bodies until here)
    auto tf2 = std::chrono::steady_clock::now();
    if (!dev_fold) parallel_fold(srcs, db->index, &fscratch);
    t_fold += ms_since(tf2);
    RawBytes().p.swap(bat[b].hb.p);  // (the batch's bodies are no longer needed)
    for (size_t i = fi; i < fe; ++i)
      if (use_hint[i]) std::vector<uint8_t>().swap(hints[i]);
    fi = fe;
  }
  if (dev_fold && fail == CASK_OK) {  // the whole replay's block, merged in one fold
    auto tf3 = std::chrono::steady_clock::now();
    {
      std::unique_lock<std::mutex> lk(bm);
      bcv.wait(lk, [&] { return dblock_done; });
    }
    const double t_wait = ms_since(tf3);
    int st = dblock_st;
    double t_merge = 0;
    if (st == CASK_OK) {
      const auto tm = std::chrono::steady_clock::now();
      db->merging = true;
      st = cask_keydir_merge(db, dblock.get(), dblock_n);
      t_merge = ms_since(tm);
      if (st == CASK_OK) st = cask_keydir_finish(db);
    }
    if (cask_knobs::hook("CASK_OPEN_TRACE"))
      fprintf(stderr, "open (device-reduced keydir): block %.1f ms on the device, %.1f ms to the host (%llu B); "
                      "waited %.1f ms; merge %.1f ms, finish %.1f ms\n",
              t_blk, t_blk_d2h, (unsigned long long)dblock_n, t_wait, t_merge, ms_since(tf3) - t_wait - t_merge);
    db->discard({&dblock});
    if (st != CASK_OK) {
      fail = st;
      fail_fid = 0;
    }
    t_fold += ms_since(tf3);
  }
  join_all();
  if (ed) ed->trim();
  edlock = std::unique_lock<std::mutex>();
  db->timings[0] = t_read;
  db->timings[1] = t_dev;
  db->timings[2] = t_hint;
  db->timings[3] = t_fold;
  db->timings[4] = ms_since(t0);
  if (fail != CASK_OK) {
    set_err(err, fail, fail_fid, fail_pos, fail_e, fail_f);
    return nullptr;
  }
  return own.release();
}

void cask_compact_options_default(cask_compact_options* o) {  // cask.rs:229-234
  if (!o) return;
  o->fragmentation_trigger = 0.6;
  o->dead_bytes_trigger = 512ull * 1024 * 1024;
  o->fragmentation_threshold = 0.4;
  o->dead_bytes_threshold = 128ull * 1024 * 1024;
  o->small_file_threshold = 10ull * 1024 * 1024;
}

// Cask::compact_files_aux + compact_files (cask.rs:451-560). The hint pass and the liveness test
// run on the host against the keydir; the live records' checksums are verified by the device scan
// of their files (Log::read_entry -> Entry::from_read, log.rs:150-166) and their bytes are copied
// into the new data files by the device gather. LogWriter rollover (log.rs:282-306) and the
// EntryWriter/HintWriter output (log.rs:317-395) are restated on the host.
static int compact_files_impl(cask_db* db, const uint32_t* files_in, uint64_t nfiles, cask_compact_result* res,
                              cask_open_error* err);
int cask_db_compact_files(cask_db* db, const uint32_t* files_in, uint64_t nfiles, cask_compact_result* res,
                          cask_open_error* err) {
  const int st = abi_status([&] { return compact_files_impl(db, files_in, nfiles, res, err); });
  if (st != CASK_OK && err && err->status == CASK_OK) set_err(err, st);  // (an exception's status)
  return st;
}

static int compact_files_impl(cask_db* db, const uint32_t* files_in, uint64_t nfiles, cask_compact_result* res,
                              cask_open_error* err) {
  set_err(err, CASK_OK);
  if (!db || (nfiles && !files_in)) return CASK_E_INVALID_ARG;
  db->reclaim_join();  // (the previous compaction's files are gone before this one starts)
  cask_compact_result R{};
  auto t0 = std::chrono::steady_clock::now();
  const std::string& path = db->path;
  // BTreeSet<u32> order (cask.rs:574, 639-640); only files of this Log
  std::vector<uint32_t> files(files_in, files_in + nfiles);
  std::sort(files.begin(), files.end());
  files.erase(std::unique(files.begin(), files.end()), files.end());
  files.erase(std::remove_if(files.begin(), files.end(),
                             [&](uint32_t f) { return !std::binary_search(db->files.begin(), db->files.end(), f); }),
              files.end());

  // 1. hints of each file with a valid hint file (files without one are skipped: cask.rs:456-468).
  // Hints::next (log.rs:437-447) per file on threads: the record offsets (`hint?` aborts,
  // cask.rs:483, the first bad file in order wins), then the keydir lookups (read-only), the live
  // list and the tombstone tail in hint order.
  struct Ins {
    uint32_t src;  // index into `srcs`
    uint64_t pos;
  };
  struct HintFile {
    HostBuf hb;
    uint64_t hn = 0;  // the file's length
    bool ok = false;
    uint64_t bad = UINT64_MAX, base = 0, nlive = 0, ntomb = 0, ins0 = 0, tomb0 = 0;
    std::vector<uint64_t> offs;
    std::vector<uint8_t> kind;  // 1: live (cask.rs:500-502); 2: tombstone of an absent key (:487-499)
  };
  std::vector<uint32_t> compacted, srcs;  // srcs: compacted files with live records
  std::vector<Ins> ins;
  std::vector<uint8_t> del_key_bytes;     // the tombstone tail, in first-seen order
  std::vector<uint64_t> del_key_off, del_seq;
  std::thread reaper;  // frees the hint pass's buffers beside the batches
  struct JoinReaper {
    std::thread& t;
    ~JoinReaper() {
      if (t.joinable()) t.join();
    }
  } join_reaper{reaper};
  // (test hook CASK_COMPACT_TRACE: the hint pass's sub-phases to stderr)
  const bool tracing = cask_knobs::hook("CASK_COMPACT_TRACE") != nullptr;
  auto tp = std::chrono::steady_clock::now();
  auto trace = [&](const char* what) {
    if (!tracing) return;
    fprintf(stderr, "compact hint pass: %s %.1f ms\n", what, ms_since(tp));
    tp = std::chrono::steady_clock::now();
  };
  {
    const size_t nh = files.size();
    std::vector<HintFile> hf(nh);
    const unsigned ntf = std::max(1u, std::min<unsigned>(host_threads(), (unsigned)std::max<size_t>(nh, 1)));
    parallel_for(ntf, [&](unsigned t) {
      for (size_t i = t; i < nh; i += ntf) {
        HintFile& H = hf[i];
        const std::string hp = hint_path(path, files[i]);
        if (!is_file_follow(hp) || !read_file_buf(hp, H.hb, H.hn) || H.hn < 4 ||
            cask_xxh::xxh32(H.hb.get(), H.hn - 4, 0) != rd32(H.hb.get() + H.hn - 4)) {
          H.hb.reset();
          H.hn = 0;
          continue;
        }
        H.ok = true;
        const uint64_t body = H.hn - 4;
        for (uint64_t p = 0; p < body;) {
          if (body - p < 22 || body - p - 22 < rd16(H.hb.get() + p + 8)) {
            H.bad = p;
            break;
          }
          H.offs.push_back(p);
          p += 22ull + rd16(H.hb.get() + p + 8);
        }
      }
    });
    trace("read+parse");
    uint64_t nrec = 0;
    std::vector<size_t> used;  // indices into hf of the compacted files, in order
    for (size_t i = 0; i < nh; ++i) {
      if (!hf[i].ok) continue;
      if (hf[i].bad != UINT64_MAX) {
        set_err(err, CASK_E_EOF, files[i], hf[i].bad);
        return CASK_E_EOF;
      }
      hf[i].base = nrec;
      nrec += hf[i].offs.size();
      hf[i].kind.resize(hf[i].offs.size());
      used.push_back(i);
    }
    unsigned nt = host_threads();
    const char* mv = cask_knobs::hook("CASK_PAR_FOLD_MIN");  // the same knob as parallel_fold
    if (nrec < (mv ? strtoull(mv, nullptr, 10) : (1ull << 16))) nt = 1;
    // keydir lookups over all the records, split evenly over threads
    parallel_for(nt, [&](unsigned t) {
      const uint64_t lo = nrec * t / nt, hi = nrec * (t + 1) / nt;
      size_t u = 0;
      while (u + 1 < used.size() && hf[used[u + 1]].base <= lo) ++u;
      for (uint64_t g = lo; g < hi;) {
        HintFile& H = hf[used[u]];
        const uint64_t e = std::min<uint64_t>(hi, H.base + H.offs.size());
        // lookups in flight: slots prefetched D records ahead, keys D/2 (test hook
        // CASK_COMPACT_LOOKAHEAD: a power of two up to 64)
        static const uint64_t D = [] {
          const char* v = cask_knobs::hook("CASK_COMPACT_LOOKAHEAD");
          const uint64_t d = v ? strtoull(v, nullptr, 10) : 16;
          return d >= 2 && d <= 64 && !(d & (d - 1)) ? d : 16ull;
        }();
        uint64_t hr[64];
        auto hash_at = [&](uint64_t i) {
          const uint8_t* h = H.hb.get() + H.offs[i];
          return hash_key(h + 22, rd16(h + 8));
        };
        const uint64_t i0 = g - H.base, i1 = e - H.base;
        for (uint64_t i = i0; i < std::min(i1, i0 + D); ++i) {
          hr[i & (D - 1)] = hash_at(i);
          db->index.prefetch(hr[i & (D - 1)]);
        }
        for (uint64_t i = i0; i < i1; ++i) {
          if (i + D / 2 < i1) db->index.prefetch_key(hr[(i + D / 2) & (D - 1)]);
          const uint8_t* h = H.hb.get() + H.offs[i];
          const cask_index_entry* ie = db->index.get_h(h + 22, rd16(h + 8), hr[i & (D - 1)]);
          H.kind[i] = rd32(h + 10) == CASK_ENTRY_TOMBSTONE ? (ie ? 0 : 2) : (ie && ie->sequence == rd64(h)) ? 1 : 0;
          if (i + D < i1) {
            hr[i & (D - 1)] = hash_at(i + D);
            db->index.prefetch(hr[i & (D - 1)]);
          }
        }
        g = e;
        ++u;
      }
    });
    trace("lookups");
    const unsigned ntu = std::max(1u, std::min<unsigned>(nt, (unsigned)std::max<size_t>(used.size(), 1)));
    parallel_for(ntu, [&](unsigned t) {
      for (size_t j = t; j < used.size(); j += ntu) {
        HintFile& H = hf[used[j]];
        for (uint8_t k : H.kind) {
          H.nlive += k == 1;
          H.ntomb += k == 2;
        }
      }
    });
    uint64_t nins = 0, ntomb = 0;
    for (size_t u : used) {
      HintFile& H = hf[u];
      compacted.push_back(files[u]);
      H.ins0 = nins;
      H.tomb0 = ntomb;
      if (H.nlive) srcs.push_back(files[u]);
      nins += H.nlive;
      ntomb += H.ntomb;
    }
    // the live list (hint order) and the tombstones of absent keys (hint order), file by file
    struct Tomb {
      const uint8_t* key;
      uint64_t seq;
      uint64_t hash;
      uint32_t ksz;
      uint32_t first;  // 1: the key's first tombstone (its place in the tail)
    };
    ins.resize(nins);
    std::vector<Tomb> tombs(ntomb);
    parallel_for(ntu, [&](unsigned t) {
      for (size_t j = t; j < used.size(); j += ntu) {
        const HintFile& H = hf[used[j]];
        const uint32_t si = (uint32_t)(std::lower_bound(srcs.begin(), srcs.end(), files[used[j]]) - srcs.begin());
        uint64_t a = H.ins0, d = H.tomb0;
        for (uint64_t i = 0; i < H.kind.size(); ++i) {
          if (!H.kind[i]) continue;
          const uint8_t* h = H.hb.get() + H.offs[i];
          if (H.kind[i] == 1) {
            ins[a++] = Ins{si, rd64(h + 14)};
          } else {
            const uint16_t k = rd16(h + 8);
            tombs[d++] = Tomb{h + 22, rd64(h), hash_key(h + 22, k), k, 0};
          }
        }
      }
    });
    trace("lists");
    // the tail: each absent key once, at its first tombstone, with its highest sequence; keys
    // deduplicated by hash-split tables on threads
    constexpr unsigned S = Index::kSub;
    std::vector<std::vector<uint64_t>> tl(S);
    for (uint64_t i = 0; i < ntomb; ++i) tl[Index::sub_of(tombs[i].hash)].push_back(i);
    const unsigned ntt = ntomb < 4096 ? 1u : std::min(nt, S);
    parallel_for(ntt, [&](unsigned t) {
      for (unsigned q = t; q < S; q += ntt) {
        std::unordered_map<uint64_t, uint64_t> seen;  // hash -> the key's first tombstone
        std::vector<uint64_t> more;                     // first tombstones of keys whose hash was taken
        seen.reserve(tl[q].size());
        auto same = [&](const Tomb& A, const Tomb& B) {
          return A.hash == B.hash && A.ksz == B.ksz && (A.ksz == 0 || memcmp(A.key, B.key, A.ksz) == 0);
        };
        for (uint64_t i : tl[q]) {
          Tomb& T = tombs[i];
          auto ins_at = seen.emplace(T.hash, i);
          uint64_t f = UINT64_MAX;
          if (!ins_at.second) {
            if (same(tombs[ins_at.first->second], T)) f = ins_at.first->second;
            for (size_t m = 0; f == UINT64_MAX && m < more.size(); ++m)
              if (same(tombs[more[m]], T)) f = more[m];
            if (f == UINT64_MAX) more.push_back(i);
          }
          if (f == UINT64_MAX) {
            T.first = 1;
          } else if (tombs[f].seq < T.seq) {
            tombs[f].seq = T.seq;
          }
        }
      }
    });
    trace("tail-dedup");
    // the tail's keys and sequences in first-seen order: counted per slice of `tombs` on threads,
    // then each slice writes its part at its prefix
    {
      const unsigned nts = ntomb < 65536 ? 1u : nt;
      std::vector<uint64_t> cnt(nts + 1, 0), kb(nts + 1, 0);
      parallel_for(nts, [&](unsigned t) {
        for (uint64_t i = ntomb * t / nts, e = ntomb * (t + 1) / nts; i < e; ++i)
          if (tombs[i].first) {
            ++cnt[t + 1];
            kb[t + 1] += tombs[i].ksz;
          }
      });
      for (unsigned t = 0; t < nts; ++t) {
        cnt[t + 1] += cnt[t];
        kb[t + 1] += kb[t];
      }
      del_key_off.resize(cnt[nts] + 1);
      del_seq.resize(cnt[nts]);
      del_key_bytes.resize(kb[nts]);
      parallel_for(nts, [&](unsigned t) {
        uint64_t j = cnt[t], o = kb[t];
        for (uint64_t i = ntomb * t / nts, e = ntomb * (t + 1) / nts; i < e; ++i) {
          const Tomb& T = tombs[i];
          if (!T.first) continue;
          del_key_off[j] = o;
          del_seq[j++] = T.seq;
          if (T.ksz) memcpy(del_key_bytes.data() + o, T.key, T.ksz);
          o += T.ksz;
        }
      });
      del_key_off[cnt[nts]] = kb[nts];
    }
    trace("tail");
    // the hint files' buffers (GiB at configs[3] scale) are unmapped on a thread of their own while
    // the live records go through the device
    std::vector<HintFile>* dying = new std::vector<HintFile>(std::move(hf));
    try {
      reaper = std::thread([dying] { delete dying; });
    } catch (...) {  // (no thread: freed here)
      delete dying;
    }
  }
  trace("hint pass end");
  R.ms[0] = ms_since(t0);

  // 2-5. The live records, source file batch by batch (at most ~kBatch bytes of sources on the
  // device at once): the sources read straight to the device, each live record read and verified
  // where its hint says it is (Log::read_entry -> Entry::from_read, log.rs:150-166; the device
  // hashes only the live bytes), placed by the LogWriter rollover (log.rs:282-306), its bytes
  // gathered on the device in write order and appended to the new data files; then the tombstone
  // tail. On an error, the files this call created are removed and the reference's error returned.
  const size_t ns = srcs.size();
  const size_t nt = del_seq.size();
  struct OutFile {
    uint32_t fid;
    uint64_t len = 0;
    int fd = -1;
    std::vector<uint8_t> hints;
  };
  // (a deque: the writer thread below holds references into `outs` while placement appends to it,
  // and push_back on a deque never moves the elements already there)
  std::deque<OutFile> outs;
  std::vector<uint32_t> new_files, tomb_files;
  uint64_t cur = 0;
  auto place = [&](uint64_t size, bool live) -> size_t {  // LogWriter::write's rollover
    if (outs.empty() || cur + size > db->opts.max_file_size) {
      const uint32_t fid = ++db->file_seq;  // Sequence::increment (util.rs:62-64)
      (live ? new_files : tomb_files).push_back(fid);  // cask.rs:510-512, 518-520
      outs.push_back(OutFile{fid});
      cur = 0;
    }
    cur += size;
    return outs.size() - 1;
  };
  auto remove_outs = [&]() {
    for (OutFile& o : outs) {  // every file this call created, with any hint file already written
      if (o.fd >= 0) close(o.fd);
      o.fd = -1;
      (void)unlink(data_path(path, o.fid).c_str());
      (void)unlink(hint_path(path, o.fid).c_str());
    }
    db->file_seq -= (uint32_t)outs.size();
    outs.clear();
  };
  auto abort_with = [&](int st, uint32_t fid = 0, uint64_t pos = 0, uint32_t e = 0, uint32_t f = 0) {
    remove_outs();
    set_err(err, st, fid, pos, e, f);
    return st;
  };
  // an exception before the new files are complete (std::bad_alloc while gathering or placing)
  // removes them too, on its way to cask_db_compact_files' handler (the writer thread, declared
  // after this guard, is joined first)
  struct RemoveOnThrow {
    decltype(remove_outs)& f;
    bool armed = true;
    ~RemoveOnThrow() {
      if (armed && std::uncaught_exceptions()) f();
    }
  } remove_on_throw{remove_outs};
  // one record's bytes into its file, and its hint (Hint::new(entry, entry_pos), data.rs:218-226)
  auto append = [&](OutFile& o, const uint8_t* rec, uint64_t n) -> bool {
    if (o.fd < 0 && (o.fd = open(data_path(path, o.fid).c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0644)) < 0) return false;
    const uint16_t k = rd16(rec + 12);
    uint8_t h[22];
    wr64(h, rd64(rec + 4));
    wr16(h + 8, k);
    wr32(h + 10, rd32(rec + 14));
    wr64(h + 14, o.len);
    o.hints.insert(o.hints.end(), h, h + 22);
    o.hints.insert(o.hints.end(), rec + 18, rec + 18 + k);
    o.len += n;
    return true;
  };
  auto pwrite_all = [](int fd, const uint8_t* b, uint64_t n, uint64_t at) -> bool {
    while (n) {
      const ssize_t w = pwrite(fd, b, n, (off_t)at);
      if (w < 0 && errno == EINTR) continue;
      if (w <= 0) return false;
      b += w;
      at += (uint64_t)w;
      n -= (uint64_t)w;
    }
    return true;
  };
  // The live records' writes, one batch behind the device: a writer thread takes each batch's
  // gathered bytes (in write order) while this thread reads, verifies and gathers the next batch
  // on the device. Within a batch, the runs of records bound for one file (placement only moves
  // forward: one run per file per batch) get their hints appended on a thread each, and their bytes
  // written with pwrite in pieces of at most 64 MiB at their offsets in the file, all on threads.
  struct WBatch {
    std::vector<HostBuf> regions;       // per source file of the batch: its live records' bytes, in order
    std::vector<const uint8_t*> at;     // per record: its bytes (in a region)
    std::vector<uint64_t> len, foff;    // per record: length, offset in its output file
    std::vector<OutFile*> op;           // per record: its output file
    // outs[done, complete) take no record after this batch: the writer finishes them. (The writer
    // never indexes `outs`: placement appends to it meanwhile, which may rewrite the deque's block
    // map; the elements themselves never move, so pointers resolved at placement stay valid.)
    std::vector<OutFile*> fin;
    size_t complete = 0;
  };
  struct Writer {
    std::thread th;
    std::mutex m;
    std::condition_variable cv;
    std::unique_ptr<WBatch> pending;
    bool busy = false, quit = false;
    uint32_t fail_fid = 0;
    int status = CASK_OK;
    double ms = 0;
    void wait_idle() {
      std::unique_lock<std::mutex> lk(m);
      cv.wait(lk, [&] { return !busy && !pending; });
    }
    void stop() {
      if (!th.joinable()) return;
      {
        std::lock_guard<std::mutex> g(m);
        quit = true;
      }
      cv.notify_all();
      th.join();
    }
    ~Writer() { stop(); }
  } writer;
  auto write_batch = [&](WBatch& B) -> int {  // (on the writer thread)
    const uint64_t n = B.op.size();
    std::vector<std::pair<uint64_t, uint64_t>> runs;
    for (uint64_t k = 0; k < n;) {
      uint64_t e = k;
      while (e < n && B.op[e] == B.op[k]) ++e;
      runs.emplace_back(k, e);
      k = e;
    }
    for (const auto& r : runs) {  // (fds opened here, on one thread)
      OutFile& o = *B.op[r.first];
      if (o.fd < 0 && (o.fd = open(data_path(path, o.fid).c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0644)) < 0) {
        writer.fail_fid = o.fid;
        return CASK_E_IO;
      }
    }
    struct Piece {
      size_t run;
      const uint8_t* at;  // host bytes
      uint64_t n, foff;
    };
    std::vector<Piece> pieces;
    constexpr uint64_t kWPiece = 64ull << 20;
    for (size_t r = 0; r < runs.size(); ++r) {  // each run's records contiguous in memory (one source's region)
      for (uint64_t k = runs[r].first, e = runs[r].second; k < e;) {
        uint64_t j = k + 1;
        while (j < e && B.at[j] == B.at[j - 1] + B.len[j - 1]) ++j;
        const uint8_t* a = B.at[k];
        const uint64_t nb = (uint64_t)(B.at[j - 1] + B.len[j - 1] - a);
        for (uint64_t x = 0; x < nb; x += kWPiece) pieces.push_back(Piece{r, a + x, std::min(kWPiece, nb - x), B.foff[k] + x});
        k = j;
      }
    }
    std::vector<char> ok(runs.size(), 1);
    const size_t ntask = runs.size() + pieces.size();  // tasks [0, runs): hints; then the pieces
    const unsigned ntw = std::max(1u, std::min<unsigned>(host_threads(), (unsigned)ntask));
    parallel_for(ntw, [&](unsigned t) {
      for (size_t x = t; x < ntask; x += ntw) {
        if (x < runs.size()) {
          for (uint64_t j = runs[x].first; j < runs[x].second; ++j) append(*B.op[j], B.at[j], B.len[j]);
        } else {
          const Piece& pc = pieces[x - runs.size()];
          if (!pwrite_all(B.op[runs[pc.run].first]->fd, pc.at, pc.n, pc.foff)) ok[pc.run] = 0;
        }
      }
    });
    for (size_t r = 0; r < runs.size(); ++r)
      if (!ok[r]) {
        writer.fail_fid = B.op[runs[r].first]->fid;
        return CASK_E_IO;
      }
    return CASK_OK;
  };
  // an error while the writer may hold a batch: it finishes (or skips) that batch and stops before
  // the files are removed
  auto abort_w = [&](int st, uint32_t fid = 0, uint64_t pos = 0, uint32_t e = 0, uint32_t f = 0) {
    writer.stop();
    return abort_with(st, fid, pos, e, f);
  };
  // Output files [lo, hi) finished: hint file (HintWriter: body + XXH32 trailer) written and data
  // file closed, a file per thread (the first failure in file order is the error). The writer thread
  // finishes each output file once no later batch can add to it; this thread the rest at the end.
  size_t hints_done = 0;  // (the writer's; read here only once it has stopped)
  size_t fin_next = 0;    // (this thread's: the output files already handed to the writer to finish)
  auto finish_outputs = [&](const std::vector<OutFile*>& fo, uint32_t* fail) -> int {
    const size_t lo = 0, hi = fo.size();
    if (hi <= lo) return CASK_OK;
    std::vector<char> okh(hi - lo, 1);
    const unsigned nth = std::max(1u, std::min<unsigned>(host_threads(), (unsigned)(hi - lo)));
    parallel_for(nth, [&](unsigned t) {
      for (size_t i = lo + t; i < hi; i += nth) {
        OutFile& o = *fo[i];
        if (o.fd < 0 && (o.fd = open(data_path(path, o.fid).c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0644)) < 0) {
          okh[i - lo] = 0;
          continue;
        }
        close(o.fd);
        o.fd = -1;
        okh[i - lo] = write_file_raw2(hint_path(path, o.fid), o.hints.data(), o.hints.size(),
                                      cask_xxh::xxh32(o.hints.data(), o.hints.size(), 0));
      }
    });
    for (size_t i = lo; i < hi; ++i)
      if (!okh[i - lo]) {
        *fail = fo[i]->fid;
        return CASK_E_IO;
      }
    return CASK_OK;
  };
  auto start_writer = [&]() {
    writer.th = std::thread([&] {
      for (;;) {
        std::unique_ptr<WBatch> B;
        {
          std::unique_lock<std::mutex> lk(writer.m);
          writer.cv.wait(lk, [&] { return writer.quit || writer.pending; });
          if (!writer.pending) return;  // quit
          B = std::move(writer.pending);
          writer.busy = true;
        }
        const auto tw0 = std::chrono::steady_clock::now();
        int st = writer.status == CASK_OK ? abi_status([&] { return write_batch(*B); }) : writer.status;
        if (st == CASK_OK && B->complete > hints_done) {  // (output files no later batch adds to)
          st = abi_status([&] { return finish_outputs(B->fin, &writer.fail_fid); });
          if (st == CASK_OK) hints_done = B->complete;
        }
        const double dt = ms_since(tw0);
        B.reset();  // (the batch's host bytes go before the next one is taken)
        {
          std::lock_guard<std::mutex> g(writer.m);
          if (writer.status == CASK_OK) writer.status = st;
          writer.ms += dt;
          writer.busy = false;
        }
        writer.cv.notify_all();
      }
    });
  };
  double t_verify = 0, t_gather = 0, t_write = 0, tr_read = 0, tr_h2d = 0;
  std::vector<uint64_t> slen(ns, 0);
  for (size_t i = 0; i < ns; ++i) {
    struct stat stt;
    slen[i] = stat(data_path(path, srcs[i]).c_str(), &stt) == 0 ? (uint64_t)stt.st_size : 0;
  }
  // Per batch of source files (at most ~kBatch bytes of them): pass 1 on host threads, a source
  // file each — the file mapped, each live record's header read at its hint position and its bytes
  // copied, in write order, into the file's region of the batch (Log::read_entry's reads,
  // log.rs:150-166; only the live records' lines are touched, not the dead 80 % of configs[3]); a
  // record cut short by the file's end is its UnexpectedEof and ends that file's pass. Then the
  // regions' bytes go to the device through the pinned ring and the device verifies every copied
  // record (cask_read_entries_device: the header's length again, XXH32 against the stored
  // checksum, Entry::from_read, data.rs:161-206). The first failure in write order — an EOF from
  // pass 1 or a checksum from the device — is the reference's error. The batch's bytes are already
  // in write order on the host: placement, and the batch to the writer thread.
  if (!ins.empty()) {
    EngineDev* ed = engine_dev(db->opts.device);
    if (!ed) return abort_w(CASK_E_DEVICE);
    std::lock_guard<std::mutex> g(ed->mu);
    int st = ed->prepare();
    if (st != CASK_OK) return abort_w(st);
    // (test hook CASK_COMPACT_BATCH: source bytes per batch, so small databases run several batches)
    const char* bh = cask_knobs::hook("CASK_COMPACT_BATCH");
    const uint64_t kBatch = bh && strtoull(bh, nullptr, 10) ? strtoull(bh, nullptr, 10) : (16ull << 30);
    size_t k0 = 0;
    for (size_t b0 = 0; b0 < ns;) {
      auto tv = std::chrono::steady_clock::now();
      size_t b1 = b0 + 1;
      uint64_t bytes = slen[b0];
      while (b1 < ns && bytes + slen[b1] <= kBatch) bytes += slen[b1++];
      R.bytes_in += bytes;
      const size_t nf = b1 - b0;
      // the batch's records: ins[k0, k1), file f's from fk[f]
      std::vector<size_t> fk(nf + 1, k0);
      size_t k1 = k0;
      for (size_t f = 0; f < nf; ++f) {
        fk[f] = k1;
        while (k1 < ins.size() && ins[k1].src == b0 + f) ++k1;
      }
      fk[nf] = k1;
      const uint64_t n = k1 - k0;
      std::unique_ptr<WBatch> WB(new WBatch());
      WB->regions.resize(nf);
      WB->at.assign(n, nullptr);
      WB->len.assign(n, 0);
      std::vector<uint64_t> used(nf, 0);      // bytes copied into each region
      std::vector<uint64_t> eof(nf, UINT64_MAX);  // per file: its first record cut short (batch index)
      std::vector<char> io_ok(nf, 1);
      auto ts = std::chrono::steady_clock::now();
      const unsigned ntf = std::max(1u, std::min<unsigned>(host_threads(), (unsigned)nf));
      parallel_for(ntf, [&](unsigned t) {
        for (size_t f = t; f < nf; f += ntf) {
          if (fk[f] == fk[f + 1]) continue;
          const int fdsc = open(data_path(path, srcs[b0 + f]).c_str(), O_RDONLY);  // File::open: Io
          struct stat stt;
          if (fdsc < 0 || fstat(fdsc, &stt) != 0) {
            if (fdsc >= 0) close(fdsc);
            io_ok[f] = 0;
            continue;
          }
          const uint64_t flen = (uint64_t)stt.st_size;
          const uint8_t* m = nullptr;
          if (flen) {
            void* q = mmap(nullptr, flen, PROT_READ, MAP_PRIVATE, fdsc, 0);
            if (q == MAP_FAILED) {
              close(fdsc);
              io_ok[f] = 0;
              continue;
            }
            m = (const uint8_t*)q;
          }
          close(fdsc);
          HostBuf& rg = WB->regions[f];
          if (!rg.alloc(std::max<uint64_t>(flen, 1))) {
            if (m) munmap((void*)m, flen);
            throw std::bad_alloc();
          }
          uint64_t o = 0;
          for (size_t k = fk[f]; k < fk[f + 1]; ++k) {
            const uint64_t pos = ins[k].pos;
            if (pos > flen || flen - pos < 18) {  // header cut short (data.rs:163)
              eof[f] = k - k0;
              break;
            }
            const uint8_t* h = m + pos;
            const uint32_t vsz = rd32(h + 14);
            const uint64_t rl = 18ull + rd16(h + 12) + (vsz == CASK_ENTRY_TOMBSTONE ? 0ull : (uint64_t)vsz);
            if (flen - pos < rl) {  // key or value cut short (data.rs:172,181)
              eof[f] = k - k0;
              break;
            }
            memcpy(rg.get() + o, h, rl);
            WB->at[k - k0] = rg.get() + o;
            WB->len[k - k0] = rl;
            o += rl;
          }
          used[f] = o;
          if (m) munmap((void*)m, flen);
        }
      });
      tr_read += ms_since(ts);
      // the first file that could not be opened ends the batch there (its records come first in
      // write order after the earlier files')
      size_t nv = n;  // records verified: those before the batch's first failure from pass 1
      for (size_t f = 0; f < nf; ++f) {
        if (!io_ok[f] && fk[f] != fk[f + 1]) {
          nv = std::min<size_t>(nv, fk[f] - k0);
          break;
        }
        if (eof[f] != UINT64_MAX) {
          nv = std::min<size_t>(nv, eof[f]);
          break;
        }
      }
      // the copied bytes to the device, contiguous; the device verifies records [0, nv)
      uint64_t total = 0;
      std::vector<uint64_t> doff(nf, 0);
      for (size_t f = 0; f < nf; ++f) {
        doff[f] = total;
        total += used[f];
      }
      std::vector<uint64_t> pos(nv), len(nv);
      std::vector<uint32_t> src(nv, 0u), ex(nv), fd(nv);
      std::vector<uint8_t> stv(nv);
      if (nv) {
        if (!ed->data.ensure(total + 256)) return abort_w(CASK_E_NOMEM);
        ts = std::chrono::steady_clock::now();
        std::vector<cask_host::PinnedRing::Piece> ps;
        for (size_t f = 0; f < nf; ++f)
          if (used[f]) cask_host::PinnedRing::split(WB->regions[f].get(), ed->data.p + doff[f], used[f], ps);
        if (!ed->ring.h2d(ps)) return abort_w(CASK_E_DEVICE);
        tr_h2d += ms_since(ts);
        size_t f = 0;
        for (uint64_t k = 0; k < nv; ++k) {
          while (k0 + k >= fk[f + 1]) ++f;
          pos[k] = doff[f] + (uint64_t)(WB->at[k] - WB->regions[f].get());
        }
        const uint8_t* dsrc = ed->data.p;
        st = cask_read_entries_device(ed->ctx, &dsrc, &total, 1, src.data(), pos.data(), nv, len.data(), stv.data(),
                                      ex.data(), fd.data());
        if (st != CASK_OK) return abort_w(st);
      }
      for (uint64_t k = 0; k < nv; ++k)  // in write order: the first failure is the reference's
        if (stv[k] != CASK_ROW_OK || len[k] != WB->len[k])
          return stv[k] == CASK_ROW_CHECKSUM ? abort_w(CASK_E_CHECKSUM, srcs[ins[k0 + k].src], ins[k0 + k].pos, ex[k], fd[k])
                                             : abort_w(CASK_E_EOF, srcs[ins[k0 + k].src], ins[k0 + k].pos);
      if (nv < n) {  // pass 1's failure: File::open / read (Io) or a record cut short (UnexpectedEof)
        const uint32_t fid = srcs[ins[k0 + nv].src];
        const size_t f = ins[k0 + nv].src - b0;
        if (!io_ok[f]) return abort_w(CASK_E_IO, fid);
        return abort_w(CASK_E_EOF, fid, ins[k0 + nv].pos);
      }
      t_verify += ms_since(tv);
      // placement (LogWriter::write's rollover, log.rs:282-306), in write order
      auto tg = std::chrono::steady_clock::now();
      WB->op.resize(n);
      WB->foff.resize(n);
      for (uint64_t k = 0; k < n; ++k) {
        WB->op[k] = &outs[place(WB->len[k], true)];
        WB->foff[k] = cur - WB->len[k];  // (its offset in its file: placement just added it)
      }
      WB->complete = outs.empty() ? 0 : outs.size() - 1;  // (the last output file may take more)
      for (size_t i = fin_next; i < WB->complete; ++i) WB->fin.push_back(&outs[i]);
      fin_next = std::max(fin_next, WB->complete);
      t_gather += ms_since(tg);
      // hand the batch to the writer once it has taken the previous one
      auto tw = std::chrono::steady_clock::now();
      if (!writer.th.joinable()) start_writer();
      writer.wait_idle();
      if (writer.status != CASK_OK) return abort_w(writer.status, writer.fail_fid);
      {
        std::lock_guard<std::mutex> g(writer.m);
        writer.pending = std::move(WB);
      }
      writer.cv.notify_all();
      t_write += ms_since(tw);  // (the time this thread waited for the writer)
      k0 = k1;
      b0 = b1;
    }
  }
  // the last batch's writes (R.ms[3] counts what this thread waited for the writer, not the writer's
  // time beside the device work)
  auto twl = std::chrono::steady_clock::now();
  writer.wait_idle();
  writer.stop();
  t_write += ms_since(twl);
  if (writer.status != CASK_OK) return abort_with(writer.status, writer.fail_fid);
  R.ms[1] = t_verify;
  R.ms[2] = t_gather;
  if (tracing)
    fprintf(stderr, "compact batches: live records copied from the mapped sources %.1f ms, to the device %.1f ms (of verify), writer busy %.1f ms\n",
            tr_read, tr_h2d, writer.ms);
  // the tombstone tail: Entry::deleted(sequence, key).write_bytes (data.rs:90-121), in first-seen
  // order. The placement (the rollover) runs in order; the records, their checksums and their hints
  // are then laid out on threads, and each output file's run of them goes out in one pwrite.
  auto tw = std::chrono::steady_clock::now();
  if (nt) {
    std::vector<uint32_t> to(nt);
    std::vector<uint64_t> at(nt), hat(nt);  // offset in its file; offset in its file's hints
    std::vector<uint64_t> hl;               // per output: hint bytes as placed
    for (size_t j = 0; j < nt; ++j) {
      const uint64_t kn = del_key_off[j + 1] - del_key_off[j];
      const size_t o = place(18 + kn, false);
      to[j] = (uint32_t)o;
      at[j] = cur - (18 + kn);
      if (hl.size() <= o) hl.resize(o + 1, UINT64_MAX);
      if (hl[o] == UINT64_MAX) hl[o] = outs[o].hints.size();
      hat[j] = hl[o];
      hl[o] += 22 + kn;
    }
    struct TRun {
      size_t j0, j1;
      std::vector<uint8_t> bytes;
    };
    std::vector<TRun> runs;
    for (size_t j = 0; j < nt;) {
      size_t e = j + 1;
      while (e < nt && to[e] == to[j]) ++e;
      runs.push_back(TRun{j, e, {}});
      j = e;
    }
    std::vector<uint32_t> run_of(nt);
    for (size_t r = 0; r < runs.size(); ++r) {
      const TRun& R = runs[r];
      const uint64_t kl = del_key_off[R.j1] - del_key_off[R.j1 - 1];
      runs[r].bytes.resize(at[R.j1 - 1] + 18 + kl - at[R.j0]);
      OutFile& o = outs[to[R.j0]];
      o.hints.resize(hl[to[R.j0]]);
      o.len = at[R.j1 - 1] + 18 + kl;
      for (size_t j = R.j0; j < R.j1; ++j) run_of[j] = (uint32_t)r;
    }
    const unsigned ntt = nt < 65536 ? 1u : host_threads();
    parallel_for(ntt, [&](unsigned t) {
      for (size_t j = nt * t / ntt, e = nt * (t + 1) / ntt; j < e; ++j) {
        const TRun& R = runs[run_of[j]];
        const uint64_t ko = del_key_off[j], kn = del_key_off[j + 1] - ko;
        uint8_t* rec = (uint8_t*)R.bytes.data() + (at[j] - at[R.j0]);
        wr64(rec + 4, del_seq[j]);
        wr16(rec + 12, (uint16_t)kn);
        wr32(rec + 14, CASK_ENTRY_TOMBSTONE);
        if (kn) memcpy(rec + 18, del_key_bytes.data() + ko, kn);
        wr32(rec, cask_xxh::xxh32(rec + 4, 14 + kn, 0));
        uint8_t* h = outs[to[j]].hints.data() + hat[j];  // Hint::new(entry, entry_pos) (data.rs:218-226)
        wr64(h, del_seq[j]);
        wr16(h + 8, (uint16_t)kn);
        wr32(h + 10, CASK_ENTRY_TOMBSTONE);
        wr64(h + 14, at[j]);
        if (kn) memcpy(h + 22, del_key_bytes.data() + ko, kn);
      }
    });
    for (const TRun& R : runs) {
      OutFile& o = outs[to[R.j0]];
      if ((o.fd < 0 && (o.fd = open(data_path(path, o.fid).c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0644)) < 0) ||
          !pwrite_all(o.fd, R.bytes.data(), R.bytes.size(), at[R.j0]))
        return abort_with(CASK_E_IO, o.fid);
    }
  }
  // the output files the writer thread has not finished (the last live one, the tombstone tail's)
  {
    uint32_t ff = 0;
    std::vector<OutFile*> rest;
    for (size_t i = hints_done; i < outs.size(); ++i) rest.push_back(&outs[i]);
    if (finish_outputs(rest, &ff) != CASK_OK) return abort_with(CASK_E_IO, ff);
  }
  t_write += ms_since(tw);
  tp = tw;
  trace("(writes) tombstone tail + hint files");
  R.ms[3] = t_write;
  uint64_t bytes_out = 0;
  for (const OutFile& o : outs) bytes_out += o.len;

  // 6. compact_files (cask.rs:528-550): index the new files from their hints, drop the compacted
  // files' stats, swap the file sets
  remove_on_throw.armed = false;
  auto t4 = std::chrono::steady_clock::now();
  tp = t4;
  {
    std::vector<FoldSrc> srcs;
    for (uint32_t fid : new_files) {
      const OutFile& o = *std::find_if(outs.begin(), outs.end(), [&](const OutFile& x) { return x.fid == fid; });
      const std::vector<uint8_t>& hb = o.hints;
      uint64_t p0 = 0, k = 0;
      for (uint64_t p = 0; p < hb.size();) {
        if (k == kFoldPiece) {
          srcs.push_back(FoldSrc{hb.data() + p0, p - p0, k, fid});
          p0 = p;
          k = 0;
        }
        p += 22ull + rd16(hb.data() + p + 8);
        ++k;
      }
      if (k) srcs.push_back(FoldSrc{hb.data() + p0, hb.size() - p0, k, fid});
    }
    parallel_fold(srcs, db->index);
  }
  trace("(swap) re-index of the new files");
  for (uint32_t fid : compacted) db->index.stats.erase(fid);  // Stats::remove_files (stats.rs:50-54)
  {  // Log::swap_files (log.rs:198-217): the compacted files leave the database here, on threads (the
     // first failure in file order is the error, as the reference's loop would return it): each
     // data file and its hint file renamed out of the names find_data_files matches (log.rs:473-510:
     // `...cask.data.gone` does not end in `.cask.data`), then unlinked by a thread of the db's own
     // while this call returns (unlinking configs[3]'s 64 GiB in place took 1.4 s on /dev/shm)
    std::vector<char> gone(compacted.size(), 1);
    std::vector<std::string> dead(2 * compacted.size());
    const unsigned ntu = std::max(1u, std::min<unsigned>(host_threads(), (unsigned)compacted.size()));
    parallel_for(ntu, [&](unsigned t) {
      for (size_t j = t; j < compacted.size(); j += ntu) {
        const std::string dp = data_path(path, compacted[j]), hp = hint_path(path, compacted[j]);
        gone[j] = rename(dp.c_str(), (dp + ".gone").c_str()) == 0;
        if (!gone[j]) continue;
        dead[2 * j] = dp + ".gone";
        if (rename(hp.c_str(), (hp + ".gone").c_str()) == 0) dead[2 * j + 1] = hp + ".gone";
      }
    });
    try {
      db->reclaim = std::thread([dead = std::move(dead)] {
        for (const std::string& f : dead)
          if (!f.empty()) (void)unlink(f.c_str());
      });
    } catch (...) {  // (no thread: unlinked here)
      for (const std::string& f : dead)
        if (!f.empty()) (void)unlink(f.c_str());
    }
    for (size_t j = 0; j < compacted.size(); ++j) {
      db->files.erase(std::lower_bound(db->files.begin(), db->files.end(), compacted[j]));
      if (!gone[j]) {
        set_err(err, CASK_E_IO, compacted[j]);
        return CASK_E_IO;
      }
    }
  }
  db->files.insert(db->files.end(), new_files.begin(), new_files.end());
  std::sort(db->files.begin(), db->files.end());
  trace("(swap) stats + unlink");
  R.ms[4] = ms_since(t4);

  R.n_compacted = (uint32_t)compacted.size();
  R.n_new = (uint32_t)new_files.size();
  R.n_tomb_only = (uint32_t)tomb_files.size();
  R.live_records = ins.size();
  R.tombstones = nt;
  R.bytes_out = bytes_out;
  R.ms_total = ms_since(t0);
  if (res) *res = R;
  return CASK_OK;
}

// Cask::compact (cask.rs:563-642): pick the files by the stats and their sizes; compact them if
// a trigger fired. Returns the number of files compacted (0: no trigger), or a negative status.
static int64_t compact_impl(cask_db* db, const cask_compact_options* opts_in, cask_compact_result* res,
                            cask_open_error* err);
int64_t cask_db_compact(cask_db* db, const cask_compact_options* opts_in, cask_compact_result* res,
                        cask_open_error* err) {
  const int64_t st = abi_status([&] { return compact_impl(db, opts_in, res, err); });
  if (st < 0 && err && err->status == CASK_OK) set_err(err, (int)st);
  return st;
}

static int64_t compact_impl(cask_db* db, const cask_compact_options* opts_in, cask_compact_result* res,
                            cask_open_error* err) {
  set_err(err, CASK_OK);
  if (!db) return CASK_E_INVALID_ARG;
  cask_compact_options o;
  if (opts_in) o = *opts_in; else cask_compact_options_default(&o);
  std::vector<uint32_t> sel;
  bool triggered = false;
  std::vector<uint32_t> ids;
  for (const auto& kv : db->index.stats) ids.push_back(kv.first);
  std::sort(ids.begin(), ids.end());  // the reference iterates a HashMap; the selected set is order-free
  for (uint32_t fid : ids) {
    const StatsEntry& se = db->index.stats[fid];
    const double frag = (double)se.dead_entries / (double)se.entries;  // stats.rs:56-67
    const uint64_t dead = se.dead_bytes;
    auto has = [&](uint32_t f) { return std::find(sel.begin(), sel.end(), f) != sel.end(); };
    if (!triggered) {
      if (frag >= o.fragmentation_trigger) {
        triggered = true;
        sel.push_back(fid);
      } else if (dead >= o.dead_bytes_trigger && !has(fid)) {
        triggered = true;
        sel.push_back(fid);
      }
    }
    if (frag >= o.fragmentation_threshold && !has(fid)) {
      sel.push_back(fid);
    } else if (dead >= o.dead_bytes_threshold && !has(fid)) {
      sel.push_back(fid);
    }
    if (!has(fid)) {
      struct stat st;
      if (stat(data_path(db->path, fid).c_str(), &st) == 0 && (uint64_t)st.st_size <= o.small_file_threshold)
        sel.push_back(fid);
    }
  }
  if (res) *res = cask_compact_result{};
  if (!triggered) return 0;
  const int st = cask_db_compact_files(db, sel.data(), sel.size(), res, err);
  return st == CASK_OK ? (int64_t)sel.size() : (int64_t)st;
}

// ------------------------------------------------------------------------------------------
// Sharded replay: rank 0 folds the shards' keydir blocks (keydir_format.h) in
// rank order — the replay order, since shards are contiguous file-id ranges.
// ------------------------------------------------------------------------------------------
cask_db* cask_keydir_new(void) {
  cask_db* db = new (std::nothrow) cask_db();
  if (db) db->merging = true;
  return db;
}

static int keydir_merge_impl(cask_db* db, const uint8_t* const* blks, const uint64_t* bytes, uint32_t nb);

int cask_keydir_merge(cask_db* db, const uint8_t* blk, uint64_t bytes) {
  try {  // the block comes from a peer rank: no exception crosses the C ABI
    return keydir_merge_impl(db, &blk, &bytes, 1);
  } catch (const std::bad_alloc&) {
    return CASK_E_NOMEM;
  } catch (...) {
    return CASK_E_INVALID_ARG;
  }
}

int cask_keydir_merge_many(cask_db* db, const uint8_t* const* blocks, const uint64_t* bytes, uint32_t n) {
  try {
    if (n && (!blocks || !bytes)) return CASK_E_INVALID_ARG;
    return keydir_merge_impl(db, blocks, bytes, n);
  } catch (const std::bad_alloc&) {
    return CASK_E_NOMEM;
  } catch (...) {
    return CASK_E_INVALID_ARG;
  }
}

// Blocks [0, nb) merged in order, in one pass: each keydir table takes its records block after
// block (for each, the thresholds of its conditional tombstones against the table as the block
// finds it, then the updates), which is what merging the blocks one by one does — a key's outcome
// depends on that key's records alone, in order — with one hashing and scatter pass over all the
// blocks and a fresh table sized once for all of them (one by one, every later block grew the
// tables: 8 blocks of 2 M records merged in 0.78-1.44 s against 0.46-0.83 s for one block of 16 M,
// tools/merge_bench.py's blocks on this container's 8 threads).
static int keydir_merge_impl(cask_db* db, const uint8_t* const* blks, const uint64_t* bytes, uint32_t nb) {
  using namespace cask_kd;
  if (!db || !db->merging) return CASK_E_INVALID_ARG;
  struct Blk {
    ShardHeader hd;
    const ShardRec* rec;
    const uint8_t* keys;
    const ShardFileStat* fs;
    uint64_t n, r0;  // records, the first record's index over all blocks
  };
  std::vector<Blk> B(nb);
  uint64_t n = 0;
  for (uint32_t b = 0; b < nb; ++b) {  // every block checked before anything changes
    const uint8_t* blk = blks[b];
    if ((bytes[b] && !blk) || bytes[b] < sizeof(ShardHeader)) return CASK_E_INVALID_ARG;
    ShardHeader& hd = B[b].hd;
    memcpy(&hd, blk, sizeof(hd));
    // counts bounded by the block's size before any offset is derived from them (no wrap-around)
    if (hd.nrec > (bytes[b] - sizeof(ShardHeader)) / sizeof(ShardRec) ||
        (uint64_t)hd.nfiles > (bytes[b] - sizeof(ShardHeader)) / sizeof(ShardFileStat))
      return CASK_E_INVALID_ARG;
    const uint64_t rec_at = sizeof(ShardHeader), fst_at = rec_at + sizeof(ShardRec) * hd.nrec,
                   key_at = fst_at + sizeof(ShardFileStat) * (uint64_t)hd.nfiles;
    if (hd.magic != kMagic || hd.version != kVersion || hd.bytes > bytes[b] || key_at + hd.key_bytes > hd.bytes)
      return CASK_E_INVALID_ARG;
    B[b].rec = (const ShardRec*)(blk + rec_at);
    B[b].keys = blk + key_at;
    B[b].fs = (const ShardFileStat*)(blk + fst_at);
    B[b].n = hd.nrec;
    B[b].r0 = n;
    n += hd.nrec;
  }
  // The fold of a block depends on each key's records alone, in order: on threads by keydir table
  // (parallel_fold's split), each table taking its records in block order — first the thresholds
  // against the keydir entering the block, then the updates. Stale terms are per-file sums.
  // Pass 1, threads by piece of a block: each record with its key hash (and its key when short)
  // written to its place in one array of items in (table, block, piece, record) order, so that
  // pass 2 streams each table's items instead of reaching back into the blocks for every record.
  const char* mv = cask_knobs::hook("CASK_PAR_FOLD_MIN");
  const uint64_t min_par = mv ? strtoull(mv, nullptr, 10) : (1ull << 16);
  const unsigned nt = n < min_par ? 1u : std::min(host_threads(), Index::kSub);
  constexpr unsigned S = Index::kSub;
  const unsigned np = nt == 1 ? 1u : 4 * nt;  // pieces per block
  const size_t NP = (size_t)nb * np;          // pieces over all blocks: P = b * np + g
  auto piece = [&](size_t P, uint64_t* lo, uint64_t* hi) {
    const Blk& k = B[P / np];
    const uint64_t g = P % np;
    *lo = k.n * g / np;
    *hi = k.n * (g + 1) / np;
  };
  const auto tm0 = std::chrono::steady_clock::now();
  // every piece's first key offset in its block (the keys lie in record order), checked first
  std::vector<uint64_t> pko(NP + 1, 0);
  parallel_for(nt, [&](unsigned t) {
    for (size_t P = t; P < NP; P += nt) {
      uint64_t lo, hi, o = 0;
      piece(P, &lo, &hi);
      const ShardRec* rec = B[P / np].rec;
      for (uint64_t i = lo; i < hi; ++i) o += rec[i].ksz;
      pko[P + 1] = o;
    }
  });
  for (uint32_t b = 0; b < nb; ++b) {  // (exclusive prefix within each block)
    uint64_t o = 0;
    for (unsigned g = 0; g < np; ++g) {
      const uint64_t k = pko[(size_t)b * np + g + 1];
      pko[(size_t)b * np + g + 1] = 0;
      pko[(size_t)b * np + g] = o;
      o += k;
    }
    if (o > B[b].hd.key_bytes) return CASK_E_INVALID_ARG;
  }
  struct Item {
    uint64_t hash, seq, pos;
    uint32_t file_id, vsz;
    uint16_t ksz;
    uint8_t kind, pad0;
    uint32_t pad1;
    union {
      uint8_t kin[KeyDir::kInline];
      const uint8_t* kp;  // ksz > kInline: the key in its block
    };
    const uint8_t* key() const { return ksz <= KeyDir::kInline ? kin : kp; }
  };
  // (a) every record's key hash, and per (piece, table) how many; (b) the items scattered to their
  // places — written once, no list growing (a list per piece and table of freshly allocated small
  // vectors cost the pass its page faults: 0.39 s per 20 M records on 8 threads, tools/merge_bench.py)
  const auto tmA = std::chrono::steady_clock::now();
  // (scratch in db: the next call reuses its pages; cask_keydir_finish gives it back)
  auto scratch = [&](HostBuf& hb, uint64_t nbytes) -> uint8_t* {
    if (hb.n >= nbytes) return hb.get();
    db->discard({&hb});
    if (!hb.alloc(nbytes + nbytes / 2)) throw std::bad_alloc();  // (headroom for a larger next call:
    return hb.get();                                              // untouched pages cost nothing)
  };
  uint64_t* hs = (uint64_t*)scratch(db->mhash, std::max<uint64_t>(n, 1) * sizeof(uint64_t));
  std::vector<uint64_t> cnt(NP * S, 0);
  std::vector<uint64_t> nconds(NP, 0);
  parallel_for(nt, [&](unsigned t) {
    for (size_t P = t; P < NP; P += nt) {
      uint64_t lo, hi;
      piece(P, &lo, &hi);
      const Blk& k = B[P / np];
      uint64_t* c = &cnt[P * S];
      uint64_t ko = pko[P];
      uint64_t lc[S] = {}, nc = 0;  // (locals: no stores to lines other threads write)
      for (uint64_t i = lo; i < hi; ++i) {
        const uint64_t h = hash_key(k.keys + ko, k.rec[i].ksz);
        hs[k.r0 + i] = h;
        ++lc[Index::sub_of(h)];
        nc += k.rec[i].kind == kCond;
        ko += k.rec[i].ksz;
      }
      for (unsigned q = 0; q < S; ++q) c[q] = lc[q];
      nconds[P] = nc;
    }
  });
  std::vector<uint64_t> at(NP * S + 1, 0);  // (table q, piece P) starts at at[q * NP + P]
  for (size_t q = 0, k = 0; q < S; ++q)
    for (size_t P = 0; P < NP; ++P, ++k) at[k + 1] = at[k] + cnt[P * S + q];
  const auto tmB = std::chrono::steady_clock::now();
  Item* items = (Item*)scratch(db->mitems, std::max<uint64_t>(n, 1) * sizeof(Item));
  parallel_for(nt, [&](unsigned t) {
    for (size_t P = t; P < NP; P += nt) {
      uint64_t lo, hi;
      piece(P, &lo, &hi);
      const Blk& k = B[P / np];
      uint64_t w[S];
      for (unsigned q = 0; q < S; ++q) w[q] = at[q * NP + P];
      uint64_t ko = pko[P];
      for (uint64_t i = lo; i < hi; ++i) {
        const ShardRec& r = k.rec[i];
        const uint64_t h = hs[k.r0 + i];
        Item& it = items[w[Index::sub_of(h)]++];
        it.hash = h;
        it.seq = r.seq;
        it.pos = r.pos;
        it.file_id = r.file_id;
        it.vsz = r.vsz;
        it.ksz = r.ksz;
        it.kind = r.kind;
        it.pad0 = 0;
        it.pad1 = 0;
        if (r.ksz <= KeyDir::kInline) memcpy(it.kin, k.keys + ko, r.ksz);
        else it.kp = k.keys + ko;
        ko += r.ksz;
      }
    }
  });
  const bool tracing = cask_knobs::hook("CASK_OPEN_TRACE") != nullptr;
  const auto tm1 = std::chrono::steady_clock::now();
  if (tracing) fprintf(stderr, "keydir merge: %u blocks, %llu records, lists %.1f ms (pko %.1f, hash %.1f)\n", nb, (unsigned long long)n, ms_since(tm0), std::chrono::duration<double, std::milli>(tmA - tm0).count(), std::chrono::duration<double, std::milli>(tmB - tmA).count());
  std::vector<char> has_cond(nb, 0);  // the blocks with conditional tombstones
  for (size_t P = 0; P < NP; ++P)
    if (nconds[P]) has_cond[P / np] = 1;
  std::vector<std::unordered_map<uint32_t, cask_db::ShardTerms>> sterms(nt);
  parallel_for(nt, [&](unsigned t) {
    auto stale = [&](uint32_t fid, uint32_t ksz) {  // Stats add + remove of a stale tombstone
      cask_db::ShardTerms& x = sterms[t][fid];
      x.stale += 1;
      x.stale_bytes += 18ull + ksz;
    };
    for (unsigned q = t; q < S; q += nt) {
      KeyDir& kd = db->index.sub[q];
      // (a fresh table: room for every record's key — a block holds about one record per key; a
      // table holding keys grows when it fills, as in parallel_fold)
      if (!kd.live) kd.reserve(at[(q + 1) * NP] - at[q * NP]);
      for (uint32_t b = 0; b < nb; ++b) {
        const Item* Lq = items + at[q * NP + (size_t)b * np];
        const size_t m = at[q * NP + (size_t)(b + 1) * np] - at[q * NP + (size_t)b * np];  // block b's, in order
        // phase 0 (the thresholds) only for a block with conditional tombstones, against a table
        // that holds something (an empty one stales none of them)
        for (int phase = has_cond[b] && kd.live ? 0 : 1; phase < 2; ++phase) {
          for (size_t jj = 0; jj < m; ++jj) {
            if (jj + 16 < m) kd.prefetch(Lq[jj + 16].hash);
            if (jj + 4 < m) kd.prefetch_key(Lq[jj + 4].hash);
            const Item& r = Lq[jj];
            auto entry = [&]() -> const cask_index_entry* {
              const int64_t f = kd.find(r.key(), r.ksz, r.hash);
              return f >= 0 ? &kd.slots[(uint64_t)f].e : nullptr;
            };
            if (phase == 0) {  // 1. thresholds, against the keydir entering the block
              if (r.kind == kCond) {
                const cask_index_entry* e = entry();
                if ((e ? e->sequence + 1 : 0ull) > r.seq) stale(r.file_id, r.ksz);
              }
              continue;
            }
            // 2. the keydir: kept rows, and collided keys record by record, in the block's order
            if (r.kind == kCond) continue;
            if (r.kind == kRaw && r.vsz == CASK_ENTRY_TOMBSTONE) {
              const cask_index_entry* e = entry();
              if (e && e->sequence > r.seq) stale(r.file_id, r.ksz);
            }
            kd.update_kd(r.key(), r.ksz, r.file_id, r.pos, r.vsz, r.seq, r.hash);
          }
        }
      }
    }
  });
  if (tracing) fprintf(stderr, "keydir merge: tables %.1f ms\n", ms_since(tm1));
  for (const auto& m : sterms)
    for (const auto& kv : m) {
      cask_db::ShardTerms& x = db->terms[kv.first];
      x.stale += kv.second.stale;
      x.stale_bytes += kv.second.stale_bytes;
    }
  for (uint32_t b = 0; b < nb; ++b) {
    const ShardHeader& hd = B[b].hd;
    for (uint32_t f = 0; f < hd.nfiles; ++f) {
      const ShardFileStat& fs = B[b].fs[f];
      cask_db::ShardTerms& t = db->terms[fs.file_id];
      t.puts += fs.puts;
      t.put_bytes += fs.put_bytes;
      t.stale += fs.stale;
      t.stale_bytes += fs.stale_bytes;
      db->files.push_back(fs.file_id);
    }
    if (hd.max_seq_p1 && hd.max_seq_p1 - 1 > db->sequence) db->sequence = hd.max_seq_p1 - 1;
    ++db->shards;
  }
  return CASK_OK;
}

// Stats after the last shard: per file, entries = puts + stale tombstones, dead = puts that are not
// the key's final entry + stale tombstones (stats.rs:23-48 summed over Index::update's cases).
int cask_keydir_finish(cask_db* db) {
  return cask_abi::guard([&]() -> int {
    if (!db || !db->merging) return CASK_E_INVALID_ARG;
    const auto live = live_by_file(db->index);  // file -> (entries, bytes)
    db->index.stats.clear();
    for (const auto& kv : db->terms) {
      const cask_db::ShardTerms& t = kv.second;
      if (!t.puts && !t.stale) continue;  // no Stats::add_entry for this file
      const auto it = live.find(kv.first);
      const uint64_t le = it == live.end() ? 0 : it->second.first, lb = it == live.end() ? 0 : it->second.second;
      StatsEntry& e = db->index.stats[kv.first];
      e.entries = t.puts + t.stale;
      e.dead_entries = t.puts - le + t.stale;
      e.dead_bytes = t.put_bytes - lb + t.stale_bytes;
    }
    std::sort(db->files.begin(), db->files.end());
    db->files.erase(std::unique(db->files.begin(), db->files.end()), db->files.end());
    db->file_seq = db->files.empty() ? 0u : db->files.back();
    db->merging = false;
    db->discard({&db->mhash, &db->mitems});
    return CASK_OK;
  });
}

// ------------------------------------------------------------------------------------------
// Key-hash partition of the sharded replay (keydir_format.h, SURVEY.md §8e's huge-keyspace case):
// every rank splits its block by key owner, owner o folds the parts it receives in rank order (the
// fold above: each key's records arrive in replay order, all in one part), and the owners' per-file
// terms summed are the Stats of one fold of every block.
// ------------------------------------------------------------------------------------------
uint32_t cask_keydir_owner(const uint8_t* key, uint64_t ksz, uint32_t nparts) {
  if (nparts < 1 || ksz > 0xFFFFu || (ksz && !key)) return 0;
  return cask_kd::key_owner(cask_kd::key_hash(key, (uint32_t)ksz), nparts);
}

static int partition_host_impl(const uint8_t* blk, uint64_t bytes, uint32_t nparts, uint8_t* out, uint64_t cap,
                               uint64_t* part_off) {
  using namespace cask_kd;
  if (!blk || !part_off || nparts < 1 || nparts > kMaxParts || bytes < sizeof(ShardHeader)) return CASK_E_INVALID_ARG;
  ShardHeader hd;
  memcpy(&hd, blk, sizeof(hd));
  if (hd.magic != kMagic || hd.version != kVersion || hd.bytes > bytes ||
      hd.nrec > (bytes - sizeof(ShardHeader)) / sizeof(ShardRec) ||
      (uint64_t)hd.nfiles > (bytes - sizeof(ShardHeader)) / sizeof(ShardFileStat))
    return CASK_E_INVALID_ARG;
  const uint64_t n = hd.nrec, fst_at = sizeof(ShardHeader) + sizeof(ShardRec) * n,
                 key_at = fst_at + sizeof(ShardFileStat) * (uint64_t)hd.nfiles;
  if (key_at + hd.key_bytes > hd.bytes) return CASK_E_INVALID_ARG;
  const ShardRec* rec = (const ShardRec*)(blk + sizeof(ShardHeader));
  const uint8_t* keys = blk + key_at;
  std::vector<uint64_t> ko(n + 1, 0);
  for (uint64_t i = 0; i < n; ++i) ko[i + 1] = ko[i] + rec[i].ksz;
  if (ko[n] != hd.key_bytes) return CASK_E_INVALID_ARG;
  std::vector<uint32_t> own(n);
  std::vector<uint64_t> cnt(nparts, 0), kb(nparts, 0);
  for (uint64_t i = 0; i < n; ++i) {
    own[i] = key_owner(key_hash(keys + ko[i], rec[i].ksz), nparts);
    ++cnt[own[i]];
    kb[own[i]] += rec[i].ksz;
  }
  part_off[0] = 0;
  for (uint32_t o = 0; o < nparts; ++o) part_off[o + 1] = part_off[o] + part_bytes(cnt[o], kb[o], hd.nfiles);
  if (!out || cap < part_off[nparts]) return CASK_E_CAPACITY;
  memset(out, 0, part_off[nparts]);
  std::vector<uint64_t> r(nparts, 0), k(nparts, 0);
  const ShardFileStat* fst = (const ShardFileStat*)(blk + fst_at);
  for (uint32_t o = 0; o < nparts; ++o) {
    uint8_t* base = out + part_off[o];
    ShardHeader h{};
    h.magic = kMagic;
    h.version = kVersion;
    h.nrec = cnt[o];
    h.key_bytes = kb[o];
    h.nfiles = hd.nfiles;
    h.max_seq_p1 = hd.max_seq_p1;
    h.rows_in = o == 0 ? hd.rows_in : 0;
    h.bytes = part_off[o + 1] - part_off[o];
    memcpy(base, &h, sizeof(h));
    ShardFileStat* fo = (ShardFileStat*)(base + sizeof(ShardHeader) + sizeof(ShardRec) * cnt[o]);
    for (uint32_t f = 0; f < hd.nfiles; ++f) {
      ShardFileStat st = fst[f];
      if (o) st.puts = st.put_bytes = st.stale = st.stale_bytes = 0;
      st.pad = 0;
      memcpy(fo + f, &st, sizeof(st));
    }
  }
  for (uint64_t i = 0; i < n; ++i) {  // records and keys in block order within each part
    const uint32_t o = own[i];
    uint8_t* base = out + part_off[o];
    memcpy(base + sizeof(ShardHeader) + sizeof(ShardRec) * r[o]++, rec + i, sizeof(ShardRec));
    const uint64_t ka = sizeof(ShardHeader) + sizeof(ShardRec) * cnt[o] + sizeof(ShardFileStat) * (uint64_t)hd.nfiles;
    memcpy(base + ka + k[o], keys + ko[i], rec[i].ksz);
    k[o] += rec[i].ksz;
  }
  return CASK_OK;
}

int cask_keydir_partition_host(const uint8_t* block, uint64_t bytes, uint32_t nparts, uint8_t* out, uint64_t cap,
                               uint64_t* part_off) {
  return abi_status([&] { return partition_host_impl(block, bytes, nparts, out, cap, part_off); });
}

// This owner's terms: per file the part-0 sums and stale tombstones folded here, and its live keys.
static int64_t keydir_terms_impl(const cask_db* db, uint8_t* out, uint64_t cap) {
  using namespace cask_kd;
  if (!db || !db->merging) return CASK_E_INVALID_ARG;
  std::map<uint32_t, KeydirTerm> t;
  for (const auto& kv : db->terms) {
    KeydirTerm& x = t[kv.first];
    x.file_id = kv.first;
    x.puts += kv.second.puts;
    x.put_bytes += kv.second.put_bytes;
    x.stale += kv.second.stale;
    x.stale_bytes += kv.second.stale_bytes;
  }
  for (uint32_t f : db->files) t[f].file_id = f;  // (files with no terms still travel)
  for (const auto& kv : live_by_file(db->index)) {
    KeydirTerm& x = t[kv.first];
    x.file_id = kv.first;
    x.live += kv.second.first;
    x.live_bytes += kv.second.second;
  }
  const uint64_t need = sizeof(KeydirTerm) * t.size();
  if (out && cap >= need) {
    uint64_t o = 0;
    for (const auto& kv : t) {
      memcpy(out + o, &kv.second, sizeof(KeydirTerm));
      o += sizeof(KeydirTerm);
    }
  }
  return (int64_t)need;
}

int64_t cask_keydir_terms(const cask_db* db, uint8_t* out, uint64_t cap) {
  return abi_status([&] { return keydir_terms_impl(db, out, cap); });
}

// Stats from every owner's terms (this one's included), as cask_keydir_finish computes them from one
// whole fold: entries = puts + stale, dead = puts - live + stale, dead_bytes likewise.
static int keydir_finish_terms_impl(cask_db* db, const uint8_t* terms, uint64_t bytes) {
  using namespace cask_kd;
  if (!db || !db->merging || (bytes && !terms) || bytes % sizeof(KeydirTerm)) return CASK_E_INVALID_ARG;
  std::map<uint32_t, KeydirTerm> sum;
  for (uint64_t o = 0; o < bytes; o += sizeof(KeydirTerm)) {
    KeydirTerm t;
    memcpy(&t, terms + o, sizeof(t));
    KeydirTerm& x = sum[t.file_id];
    x.file_id = t.file_id;
    x.puts += t.puts;
    x.put_bytes += t.put_bytes;
    x.stale += t.stale;
    x.stale_bytes += t.stale_bytes;
    x.live += t.live;
    x.live_bytes += t.live_bytes;
  }
  for (const auto& kv : sum)
    if (kv.second.live > kv.second.puts || kv.second.live_bytes > kv.second.put_bytes) return CASK_E_INVALID_ARG;
  db->index.stats.clear();
  for (const auto& kv : sum) {
    const KeydirTerm& t = kv.second;
    db->files.push_back(kv.first);
    if (!t.puts && !t.stale) continue;  // no Stats::add_entry for this file
    StatsEntry& e = db->index.stats[kv.first];
    e.entries = t.puts + t.stale;
    e.dead_entries = t.puts - t.live + t.stale;
    e.dead_bytes = t.put_bytes - t.live_bytes + t.stale_bytes;
  }
  std::sort(db->files.begin(), db->files.end());
  db->files.erase(std::unique(db->files.begin(), db->files.end()), db->files.end());
  db->file_seq = db->files.empty() ? 0u : db->files.back();
  db->merging = false;
  return CASK_OK;
}

int cask_keydir_finish_terms(cask_db* db, const uint8_t* terms, uint64_t bytes) {
  return abi_status([&] { return keydir_finish_terms_impl(db, terms, bytes); });
}

// Cask::open over several GPUs of this process: contiguous file-id ranges, one per devices[] entry;
// each range is reduced to keydir blocks on its device (one host thread per distinct device, its
// ranges one after another), and the blocks are folded here in range order. Within a range, files
// with a valid hint file take the fast path (log.rs:121-135): their bodies are parsed on the device
// (cask_parse_hints_device) and reduced (cask_shard_keydir_hints); the others are scanned
// (cask_scan_device, cask_shard_keydir) and, with write_hints, get their hint files from the device
// (cask_hints_device). Each maximal stretch of files of one kind gives one block.
// The ranges run in parallel, but the reference's replay stops at the first Err (cask.rs:357-368)
// and never reaches a later file: so every hint file is first written under a temporary name
// (`.part`), and only once all ranges are done are the ones up to the first failure (in replay order)
// renamed into place — the failing range's own, which end at its failing file, included — and the
// later ranges' removed.
static cask_db* open_multi_impl(const char* path_c, const cask_options* opts_in, const int* devices, int ndev,
                                cask_open_error* err);
cask_db* cask_db_open_multi(const char* path_c, const cask_options* opts_in, const int* devices, int ndev,
                            cask_open_error* err) {
  return abi_db(err, [&] { return open_multi_impl(path_c, opts_in, devices, ndev, err); });
}

static std::string part_path(const std::string& hp) { return hp + ".part"; }

static cask_db* open_multi_impl(const char* path_c, const cask_options* opts_in, const int* devices, int ndev,
                                cask_open_error* err) {
  set_err(err, CASK_OK);
  if (!devices || ndev < 1) {
    set_err(err, CASK_E_INVALID_ARG);
    return nullptr;
  }
  auto t0 = std::chrono::steady_clock::now();
  std::unique_ptr<cask_db> own(open_log(path_c, opts_in, err));
  cask_db* db = own.get();
  if (!db) return nullptr;
  const std::string path = db->path;
  const size_t nf = db->files.size();
  // which files have a valid hint file (is_valid_hint_file, log.rs:512-539), on threads
  std::vector<std::vector<uint8_t>> hints(nf);
  std::vector<char> use_hint(nf, 0);
  {
    const unsigned nt = std::max(1u, std::min<unsigned>(host_threads(), (unsigned)std::max<size_t>(nf, 1)));
    parallel_for(nt, [&](unsigned t) {
      for (size_t i = t; i < nf; i += nt) {
        const std::string hp = hint_path(path, db->files[i]);
        if (is_file_follow(hp) && read_file(hp, hints[i]) && hints[i].size() >= 4 &&
            cask_xxh::xxh32(hints[i].data(), hints[i].size() - 4, 0) == rd32(hints[i].data() + hints[i].size() - 4))
          use_hint[i] = 1;
        else
          std::vector<uint8_t>().swap(hints[i]);
      }
    });
  }
  struct Shard {
    size_t lo = 0, hi = 0;
    std::vector<RawBytes> blocks;
    std::vector<uint32_t> parts;  // hint files written under their temporary names, in order
    cask_open_error e{};
    double ms_read = 0, ms_scan = 0;
  };
  std::vector<Shard> sh((size_t)ndev);
  for (int r = 0; r < ndev; ++r) {
    sh[r].lo = nf * (size_t)r / (size_t)ndev;
    sh[r].hi = nf * (size_t)(r + 1) / (size_t)ndev;
  }
  const bool write_hints = db->opts.write_hints != 0;
  // One stretch [lo, hi) of files of one kind on device `dev` through its EngineDev `ed` (locked by
  // the caller; its context, pinned rings and buffers), reduced to one keydir block; false on failure
  // (s.e set). Hint bodies: parsed on the device (cask_parse_hints_device). Data files: read straight
  // to the device by the pinned ring's reader threads (the stretch's bytes stay resident: the block
  // reads its keys there), scanned in batches of at most an eighth of the stretch (at least 1 GiB:
  // the scan's scratch stays bounded), each batch's hint bodies written under their temporary names
  // and its rows kept, then one block over every row of the stretch (as open() does).
  auto run_stretch = [&](Shard& s, int dev, EngineDev* ed, size_t lo, size_t hi, bool hint) -> bool {
    auto fail = [&](int st, uint32_t fid = 0, uint64_t pos = 0, uint32_t e = 0, uint32_t f = 0) {
      s.e = cask_open_error{st, fid, pos, e, f};
      return false;
    };
    cask_ctx* ctx = ed->ctx;
    hipStream_t cst = (hipStream_t)cask_ctx_stream(ctx);
    auto tr = std::chrono::steady_clock::now();
    const size_t n = hi - lo;
    std::vector<uint64_t> blen(n);
    std::vector<std::string> paths;
    uint64_t total = 0;
    for (size_t i = 0; i < n; ++i) {
      if (hint) {
        blen[i] = hints[lo + i].size() - 4;  // the body: Take(size - 4) (log.rs:129)
      } else {  // File::open + metadata (log.rs:190-196): a file that cannot be read is its Io error
        struct stat stt;
        paths.push_back(data_path(path, db->files[lo + i]));
        if (stat(paths.back().c_str(), &stt) != 0) return fail(CASK_E_IO, db->files[lo + i]);
        blen[i] = (uint64_t)stt.st_size;
      }
      total += (blen[i] + 255) & ~255ull;
    }
    uint8_t* dbuf = nullptr;
    struct Free {
      uint8_t*& a;
      ~Free() {
        if (a) (void)hipFree(a);
      }
    } release{dbuf};
    if (hipSetDevice(dev) != hipSuccess) return fail(CASK_E_DEVICE);
    if (hipMalloc(&dbuf, total + 256) != hipSuccess) return fail(CASK_E_NOMEM);
    std::vector<cask_file_view> views(n);
    uint64_t off = 0;
    for (size_t i = 0; i < n; ++i) {
      views[i] = cask_file_view{db->files[lo + i], CASK_VIEW_DEVICE, dbuf + off, blen[i]};
      off += (blen[i] + 255) & ~255ull;
    }
    std::vector<uint64_t> roff(n + 1, 0);
    EngineDev::AllRows all;
    auto ts = std::chrono::steady_clock::now();
    if (hint) {  // (the bodies are in host memory already)
      for (size_t i = 0; i < n; ++i)
        if (blen[i] && hipMemcpy((void*)views[i].data, hints[lo + i].data(), blen[i], hipMemcpyHostToDevice) != hipSuccess)
          return fail(CASK_E_DEVICE);
      s.ms_read += ms_since(tr);
      ts = std::chrono::steady_clock::now();
      // rows sized from the body bytes (hint records are at least 22 B)
      cask_rows rows{};
      const uint64_t cap = cask_rows_bound(views.data(), (uint32_t)n);
      if (!ed->rows.ensure(cap * 23 + 5 * 256)) return fail(CASK_E_NOMEM);
      const uint64_t a8 = (cap * 8 + 255) & ~255ull, a4 = (cap * 4 + 255) & ~255ull, a2 = (cap * 2 + 255) & ~255ull;
      rows.capacity = cap;
      rows.pos = (uint64_t*)ed->rows.p;
      rows.seq = (uint64_t*)(ed->rows.p + a8);
      rows.vsz = (uint32_t*)(ed->rows.p + 2 * a8);
      rows.ksz = (uint16_t*)(ed->rows.p + 2 * a8 + a4);
      rows.status = ed->rows.p + 2 * a8 + a4 + a2;
      cask_scan_error se{};
      int st = cask_parse_hints_device(ctx, views.data(), (uint32_t)n, &rows, roff.data(), &se);
      if (st != CASK_OK) return fail(st);
      if (se.kind)  // a hint record cut short: Cask::open's `?` (cask.rs:360,365)
        return fail(CASK_E_EOF, se.file_id, se.pos, se.expected, se.found);
      const void* blk = nullptr;
      uint64_t nb = 0;
      st = cask_shard_keydir_hints(ctx, views.data(), (uint32_t)n, &rows, roff.data(), &blk, &nb);
      if (st == CASK_OK) {
        s.blocks.emplace_back();
        st = s.blocks.back().resize(nb) ? ed->to_host(s.blocks.back().data(), (const uint8_t*)blk, nb) : CASK_E_NOMEM;
      }
      if (st != CASK_OK) return fail(st);
      s.ms_scan += ms_since(ts);
      return true;
    }
    // data files: batches of consecutive files
    const uint64_t bb = std::max<uint64_t>(1ull << 30, total / 8);
    for (size_t b0 = 0; b0 < n;) {
      size_t b1 = b0 + 1;
      uint64_t acc = blen[b0];
      while (b1 < n && acc + blen[b1] <= bb) acc += blen[b1++];
      const std::vector<cask_file_view> vb(views.begin() + (ptrdiff_t)b0, views.begin() + (ptrdiff_t)b1);
      const std::vector<std::string> pb(paths.begin() + (ptrdiff_t)b0, paths.begin() + (ptrdiff_t)b1);
      auto tb = std::chrono::steady_clock::now();
      std::vector<char> ok(vb.size(), 1);
      int st = ed->read_to_device(pb, vb, ok);
      if (st != CASK_OK) return fail(st);
      for (size_t k = 0; k < vb.size(); ++k)
        if (!ok[k]) return fail(CASK_E_IO, vb[k].file_id);
      s.ms_read += ms_since(tb);
      tb = std::chrono::steady_clock::now();
      std::vector<uint64_t> ro(vb.size() + 1);
      cask_scan_error se{};
      st = ed->scan(vb, ro, se);
      if (st != CASK_OK) return fail(st);
      if (write_hints) {  // RecreateHints (log.rs:137-148): every Ok row of each file, trailer
        RawBytes hb;
        std::vector<uint64_t> fo;
        st = ed->hints(vb, ro, hb, fo);
        if (st != CASK_OK) return fail(st);
        // files up to the first failing one (that one included: the drain on drop, log.rs:466-470)
        for (size_t k = 0; k < vb.size(); ++k) {
          s.parts.push_back(vb[k].file_id);
          if (!write_file_raw2(part_path(hint_path(path, vb[k].file_id)), hb.data() + fo[k], fo[k + 1] - fo[k],
                               cask_xxh::xxh32(hb.data() + fo[k], fo[k + 1] - fo[k], 0)))
            return fail(CASK_E_IO, vb[k].file_id);
          if (se.kind && se.file_id == vb[k].file_id) break;
        }
      }
      if (se.kind)  // the stretch's first failing record: Cask::open's `?` (cask.rs:360,365)
        return fail(se.kind == CASK_ROW_CHECKSUM ? CASK_E_CHECKSUM : CASK_E_EOF, se.file_id, se.pos, se.expected, se.found);
      for (size_t k = 0; k <= vb.size(); ++k) roff[b0 + k] = all.n + ro[k];
      st = all.append(ed->r, ro[vb.size()], cst);
      if (st != CASK_OK) return fail(st);
      s.ms_scan += ms_since(tb);
      b0 = b1;
    }
    ts = std::chrono::steady_clock::now();
    const cask_rows rows = all.view();
    const void* blk = nullptr;
    uint64_t nb = 0;
    int st = cask_shard_keydir(ctx, views.data(), (uint32_t)n, &rows, roff.data(), &blk, &nb);
    if (st == CASK_OK) {
      s.blocks.emplace_back();
      st = s.blocks.back().resize(nb) ? ed->to_host(s.blocks.back().data(), (const uint8_t*)blk, nb) : CASK_E_NOMEM;
    }
    if (st != CASK_OK) return fail(st);
    s.ms_scan += ms_since(ts);
    return true;
  };
  auto run_shard = [&](int r) {
    Shard& s = sh[r];
    if (s.lo == s.hi) return;
    EngineDev* ed = engine_dev(devices[r]);  // (its pinned ring, for the reads; one user at a time)
    if (!ed) {
      s.e = cask_open_error{CASK_E_DEVICE, 0, 0, 0, 0};
      return;
    }
    std::lock_guard<std::mutex> edg(ed->mu);
    const int st0 = ed->prepare();
    if (st0 != CASK_OK) {
      s.e = cask_open_error{st0, 0, 0, 0, 0};
      return;
    }
    for (size_t i = s.lo; i < s.hi;) {  // maximal stretches of one kind, in order
      size_t j = i + 1;
      while (j < s.hi && use_hint[j] == use_hint[i]) ++j;
      // (an exception in a stretch is its failure)
      const int st = abi_status([&] { return run_stretch(s, devices[r], ed, i, j, use_hint[i] != 0) ? CASK_OK : 1; });
      if (st != CASK_OK) {
        if (st != 1) s.e = cask_open_error{st, 0, 0, 0, 0};
        break;
      }
      i = j;
    }
    ed->trim();
  };
  // one thread per distinct device; a device's shards run in order on its thread
  std::vector<int> devs;
  for (int r = 0; r < ndev; ++r)
    if (std::find(devs.begin(), devs.end(), devices[r]) == devs.end()) devs.push_back(devices[r]);
  parallel_for((unsigned)devs.size(), [&](unsigned t) {
    for (int r = 0; r < ndev; ++r)
      if (devices[r] == devs[t]) run_shard(r);
  });
  int rf = ndev;  // the first range that failed, in replay order
  for (int r = 0; r < ndev && rf == ndev; ++r)
    if (sh[r].e.status != CASK_OK) rf = r;
  // hint files: into place up to the first failure, removed after it
  uint32_t ren_fail = 0;
  bool ren_ok = true;
  for (int r = 0; r < ndev; ++r)
    for (uint32_t fid : sh[r].parts) {
      const std::string hp = hint_path(path, fid);
      if (r <= rf) {
        if (ren_ok && rename(part_path(hp).c_str(), hp.c_str()) != 0) {
          ren_ok = false;
          ren_fail = fid;
        }
        if (!ren_ok) (void)unlink(part_path(hp).c_str());
      } else {
        (void)unlink(part_path(hp).c_str());
      }
    }
  if (rf < ndev) {
    if (err) *err = sh[rf].e;
    return nullptr;
  }
  if (!ren_ok) {
    set_err(err, CASK_E_IO, ren_fail);
    return nullptr;
  }
  double rd = 0, sc = 0;
  for (const Shard& s : sh) {
    rd = std::max(rd, s.ms_read);
    sc = std::max(sc, s.ms_scan);
  }
  std::vector<std::vector<uint8_t>>().swap(hints);
  auto tf = std::chrono::steady_clock::now();
  db->merging = true;
  {  // every range's blocks, in range order, in one pass
    std::vector<const uint8_t*> bp;
    std::vector<uint64_t> bl;
    for (int r = 0; r < ndev; ++r)
      for (const auto& b : sh[r].blocks) {
        bp.push_back(b.data());
        bl.push_back(b.size());
      }
    const int st = cask_keydir_merge_many(db, bp.data(), bl.data(), (uint32_t)bp.size());
    if (st != CASK_OK) {
      set_err(err, st);
      return nullptr;
    }
  }
  cask_keydir_finish(db);
  db->timings[0] = rd;
  db->timings[1] = sc;
  db->timings[2] = 0;
  db->timings[3] = ms_since(tf);
  db->timings[4] = ms_since(t0);
  return own.release();
}

// LogWriter::write (log.rs:282-306) for a batch of entries written through one writer that is then
// dropped — a bulk load. EntryWriter's bytes (Entry::write_bytes, data.rs:90-121) are encoded and
// checksummed on the device (cask_encode_device); HintWriter's records (Hint::write_bytes,
// data.rs:242-256) and its trailer on Drop (log.rs:367-395) are built per file on host threads.
// Rollover: a new file when there is no writer or pos + size > max_file_size (a record larger than
// the limit gets a file of its own). File ids are first_file_id, first_file_id + 1, ...
static int64_t log_write_impl(const char* dir_c, uint32_t first_file_id, uint64_t max_file_size, int write_hints,
                              int device, uint64_t n, const uint64_t* seq, const uint16_t* ksz, const uint32_t* vsz_raw,
                              const uint8_t* keys, const uint64_t* key_off, const uint8_t* vals, const uint64_t* val_off,
                              uint32_t* file_ids, uint64_t cap);
int64_t cask_log_write(const char* dir_c, uint32_t first_file_id, uint64_t max_file_size, int write_hints, int device,
                       uint64_t n, const uint64_t* seq, const uint16_t* ksz, const uint32_t* vsz_raw,
                       const uint8_t* keys, const uint64_t* key_off, const uint8_t* vals, const uint64_t* val_off,
                       uint32_t* file_ids, uint64_t cap) {
  return abi_status([&]() -> int64_t {
    return log_write_impl(dir_c, first_file_id, max_file_size, write_hints, device, n, seq, ksz, vsz_raw, keys,
                          key_off, vals, val_off, file_ids, cap);
  });
}

static int64_t log_write_impl(const char* dir_c, uint32_t first_file_id, uint64_t max_file_size, int write_hints,
                              int device, uint64_t n, const uint64_t* seq, const uint16_t* ksz, const uint32_t* vsz_raw,
                              const uint8_t* keys, const uint64_t* key_off, const uint8_t* vals, const uint64_t* val_off,
                              uint32_t* file_ids, uint64_t cap) {
  if (!dir_c || (n && (!seq || !ksz || !vsz_raw || !key_off || !val_off))) return CASK_E_INVALID_ARG;
  const std::string dir = dir_c;
  if (!n) return 0;  // the writer is created by the first write (log.rs:282-290)
  // 1. placement: file of each record and its position there; key/value extents to upload
  std::vector<uint64_t> goff(n), fpos(n);
  std::vector<uint64_t> fstart;  // first record of each file
  uint64_t total = 0, pos = 0, kend = 0, vend = 0;
  for (uint64_t r = 0; r < n; ++r) {
    const uint64_t ve = vsz_raw[r] == CASK_ENTRY_TOMBSTONE ? 0 : vsz_raw[r];
    const uint64_t size = 18ull + ksz[r] + ve;  // Entry::size (data.rs:63-65)
    if (fstart.empty() || pos + size > max_file_size) {
      fstart.push_back(r);
      pos = 0;
    }
    goff[r] = total;
    fpos[r] = pos;
    pos += size;
    total += size;
    kend = std::max(kend, key_off[r] + ksz[r]);
    vend = std::max(vend, ve ? val_off[r] + ve : 0);
  }
  if ((kend && !keys) || (vend && !vals)) return CASK_E_INVALID_ARG;
  const uint64_t nf = fstart.size();
  if ((uint64_t)first_file_id + nf - 1 > UINT32_MAX) return CASK_E_INVALID_ARG;
  fstart.push_back(n);
  // 2. the bytes, encoded on the device
  std::unique_ptr<uint8_t[]> host(new (std::nothrow) uint8_t[total]);
  if (!host) return CASK_E_NOMEM;
  {
    EngineDev* ed = engine_dev(device);
    if (!ed) return CASK_E_DEVICE;
    std::lock_guard<std::mutex> g(ed->mu);
    int st = ed->prepare();
    if (st != CASK_OK) return st;
    auto al = [](uint64_t b) { return (b + 255) & ~255ull; };
    const uint64_t a8 = al(8 * n), a4 = al(4 * n), a2 = al(2 * n);
    if (!ed->rows.ensure(4 * a8 + a4 + a2) || !ed->hint.ensure(al(kend) + al(vend) + 256) ||
        !ed->data.ensure(total + 256))
      return CASK_E_NOMEM;
    uint8_t* R = ed->rows.p;
    uint64_t* d_off = (uint64_t*)R;
    uint64_t* d_seq = (uint64_t*)(R + a8);
    uint64_t* d_koff = (uint64_t*)(R + 2 * a8);
    uint64_t* d_voff = (uint64_t*)(R + 3 * a8);
    uint32_t* d_vsz = (uint32_t*)(R + 4 * a8);
    uint16_t* d_ksz = (uint16_t*)(R + 4 * a8 + a4);
    uint8_t* d_keys = ed->hint.p;
    uint8_t* d_vals = ed->hint.p + al(kend);
    bool ok = hipSetDevice(device) == hipSuccess &&
              hipMemcpy(d_off, goff.data(), 8 * n, hipMemcpyHostToDevice) == hipSuccess &&
              hipMemcpy(d_seq, seq, 8 * n, hipMemcpyHostToDevice) == hipSuccess &&
              hipMemcpy(d_koff, key_off, 8 * n, hipMemcpyHostToDevice) == hipSuccess &&
              hipMemcpy(d_voff, val_off, 8 * n, hipMemcpyHostToDevice) == hipSuccess &&
              hipMemcpy(d_vsz, vsz_raw, 4 * n, hipMemcpyHostToDevice) == hipSuccess &&
              hipMemcpy(d_ksz, ksz, 2 * n, hipMemcpyHostToDevice) == hipSuccess &&
              (!kend || hipMemcpy(d_keys, keys, kend, hipMemcpyHostToDevice) == hipSuccess) &&
              (!vend || hipMemcpy(d_vals, vals, vend, hipMemcpyHostToDevice) == hipSuccess);
    if (!ok) return CASK_E_DEVICE;
    st = cask_encode_device(ed->ctx, n, d_off, d_seq, d_ksz, d_vsz, d_keys, d_koff, d_vals, d_voff, ed->data.p);
    if (st == CASK_OK) st = ed->to_host(host.get(), ed->data.p, total);
    if (st != CASK_OK) return st;
  }
  // 3. each file's data bytes and hint file, files on threads
  std::vector<char> fok(nf, 1);
  const unsigned nt = std::max(1u, std::min<unsigned>(host_threads(), (unsigned)nf));
  parallel_for(nt, [&](unsigned t) {
    for (uint64_t f = t; f < nf; f += nt) {
      const uint32_t fid = first_file_id + (uint32_t)f;
      const uint64_t r0 = fstart[f], r1 = fstart[f + 1];
      const uint64_t b0 = goff[r0], b1 = r1 < n ? goff[r1] : total;
      int fd = open(data_path(dir, fid).c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0644);
      bool ok = fd >= 0;
      for (uint64_t b = b0; ok && b < b1;) {
        const ssize_t w = write(fd, host.get() + b, b1 - b);
        if (w < 0 && errno == EINTR) continue;
        ok = w > 0;
        if (ok) b += (uint64_t)w;
      }
      if (fd >= 0) close(fd);
      if (ok && write_hints) {
        std::vector<uint8_t> hb;
        for (uint64_t r = r0; r < r1; ++r) {
          uint8_t h[22];
          wr64(h, seq[r]);
          wr16(h + 8, ksz[r]);
          wr32(h + 10, vsz_raw[r]);  // the hint's value_size: 0xFFFFFFFF for a tombstone (data.rs:246-250)
          wr64(h + 14, fpos[r]);
          hb.insert(hb.end(), h, h + 22);
          hb.insert(hb.end(), host.get() + goff[r] + 18, host.get() + goff[r] + 18 + ksz[r]);
        }
        ok = write_file_raw2(hint_path(dir, fid), hb.data(), hb.size(), cask_xxh::xxh32(hb.data(), hb.size(), 0));
      } else if (ok) {
        // no hints: a hint file left from an earlier file of this id would describe other bytes, and
        // the next open would trust it (log.rs:121-135); the reference's HintWriter::new always
        // truncates it (log.rs:373-380, util.rs:45-49)
        if (unlink(hint_path(dir, fid).c_str()) != 0 && errno != ENOENT) ok = false;
      }
      fok[f] = ok;
    }
  });
  for (uint64_t f = 0; f < nf; ++f)
    if (!fok[f]) return CASK_E_IO;
  for (uint64_t f = 0; f < nf && f < cap && file_ids; ++f) file_ids[f] = first_file_id + (uint32_t)f;
  return (int64_t)nf;
}

void cask_db_close(cask_db* db) { delete db; }

uint64_t cask_db_len(const cask_db* db) { return db ? db->index.live() : 0; }

int cask_db_get_entry(const cask_db* db, const uint8_t* key, uint64_t ksz, cask_index_entry* out) {
  // 1 (found) or 0 by contract: not under cask_abi::guard, whose negative statuses a caller testing
  // for 0 would take as "found"; the lookup allocates nothing, and anything thrown is "not found"
  try {
    if (!db || (ksz && !key) || ksz > 0xFFFF) return 0;
    const cask_index_entry* e = db->index.get(key, (uint32_t)ksz);
    if (!e) return 0;
    if (out) *out = *e;
    return 1;
  } catch (...) {
    return 0;
  }
}

int64_t cask_db_export(const cask_db* db, uint8_t* key_bytes, uint64_t key_cap, uint64_t* key_off,
                       uint64_t* key_len, cask_index_entry* entries, uint64_t nkeys) {
  return cask_abi::guard([&]() -> int64_t {
    if (!db) return CASK_E_INVALID_ARG;
    if (!key_bytes && !key_off && !key_len && !entries) {  // sizing call: no order needed
      uint64_t total = 0, n = 0;
      db->index.for_each_live([&](const KeyDir&, const KeyDir::Slot& s) {
        total += s.ksz;
        ++n;
      });
      return nkeys < n ? CASK_E_CAPACITY : (int64_t)total;
    }
    struct Ref {
      const uint8_t* key;
      uint32_t ksz;
      const cask_index_entry* e;
    };
    // Bytewise key order on host threads: refs bucketed by their first two bytes (a missing byte
    // sorts first: "" < "a" < "a\0"), each bucket sorted with the full comparison, then written out
    // in parallel pieces. (One std::sort of 237 M refs, configs[4]'s keydir, took minutes.)
    auto bucket_of = [](const uint8_t* k, uint32_t n) -> uint32_t {
      const uint32_t b0 = n >= 1 ? k[0] + 1u : 0u, b1 = n >= 2 ? k[1] + 1u : 0u;
      return b0 * 257u + b1;
    };
    constexpr uint32_t kB = 257u * 257u;
    const auto& sub = db->index.sub;
    const unsigned nt = std::min<unsigned>(host_threads(), (unsigned)Index::kSub);
    // pass 1: per-thread bucket counts over the thread's tables
    std::vector<std::vector<uint64_t>> cnt(nt, std::vector<uint64_t>(kB, 0));
    parallel_for(nt, [&](unsigned t) {
      for (size_t q = t; q < Index::kSub; q += nt)
        for (const KeyDir::Slot& sl : sub[q].slots)
          if (sl.state == 1) ++cnt[t][bucket_of(sub[q].key_of(sl), sl.ksz)];
    });
    std::vector<uint64_t> bstart(kB + 1, 0);
    for (uint32_t b = 0; b < kB; ++b) {
      uint64_t c = 0;
      for (unsigned t = 0; t < nt; ++t) c += cnt[t][b];
      bstart[b + 1] = bstart[b] + c;
    }
    const uint64_t n = bstart[kB];
    if (nkeys < n) return CASK_E_CAPACITY;
    // pass 2: scatter (thread t's refs of bucket b after threads 0..t-1's; the counts become each
    // thread's write positions first)
    for (uint32_t b = 0; b < kB; ++b) {
      uint64_t o = bstart[b];
      for (unsigned t = 0; t < nt; ++t) {
        const uint64_t c = cnt[t][b];
        cnt[t][b] = o;
        o += c;
      }
    }
    std::vector<Ref> idx(n);
    parallel_for(nt, [&](unsigned t) {
      std::vector<uint64_t>& at = cnt[t];
      for (size_t q = t; q < Index::kSub; q += nt)
        for (const KeyDir::Slot& sl : sub[q].slots)
          if (sl.state == 1) {
            const uint8_t* k = sub[q].key_of(sl);
            idx[at[bucket_of(k, sl.ksz)]++] = Ref{k, sl.ksz, &sl.e};
          }
    });
    // pass 3: buckets sorted on threads (claimed in order)
    std::atomic<uint32_t> next{0};
    parallel_for(host_threads(), [&](unsigned) {
      for (uint32_t b; (b = next.fetch_add(1)) < kB;)
        if (bstart[b + 1] - bstart[b] > 1)
          std::sort(idx.begin() + bstart[b], idx.begin() + bstart[b + 1], [](const Ref& A, const Ref& B) {
            const uint32_t m = std::min(A.ksz, B.ksz);
            const int c = m ? memcmp(A.key, B.key, m) : 0;
            if (c) return c < 0;
            return A.ksz < B.ksz;
          });
    });
    // pass 4: key offsets (prefix over pieces), then the arrays in parallel pieces
    const unsigned np = host_threads();
    std::vector<uint64_t> pbytes(np + 1, 0);
    parallel_for(np, [&](unsigned t) {
      uint64_t b = 0;
      for (uint64_t j = n * t / np; j < n * (t + 1) / np; ++j) b += idx[j].ksz;
      pbytes[t + 1] = b;
    });
    for (unsigned t = 0; t < np; ++t) pbytes[t + 1] += pbytes[t];
    const uint64_t total = pbytes[np];
    if (key_bytes && key_cap < total) return CASK_E_CAPACITY;
    parallel_for(np, [&](unsigned t) {
      uint64_t off = pbytes[t];
      for (uint64_t j = n * t / np; j < n * (t + 1) / np; ++j) {
        const Ref& r = idx[j];
        if (key_bytes && r.ksz) memcpy(key_bytes + off, r.key, r.ksz);
        if (key_off) key_off[j] = off;
        if (key_len) key_len[j] = r.ksz;
        if (entries) entries[j] = *r.e;
        off += r.ksz;
      }
    });
    return (int64_t)total;
  });
}

uint64_t cask_db_stats(const cask_db* db, uint32_t* file_id, uint64_t* entries, uint64_t* dead_entries,
                       uint64_t* dead_bytes, uint64_t cap) {
  if (!db) return 0;
  std::vector<std::pair<uint32_t, StatsEntry>> v(db->index.stats.begin(), db->index.stats.end());
  std::sort(v.begin(), v.end(), [](const auto& a, const auto& b) { return a.first < b.first; });
  for (uint64_t i = 0; i < v.size() && i < cap; ++i) {
    if (file_id) file_id[i] = v[i].first;
    if (entries) entries[i] = v[i].second.entries;
    if (dead_entries) dead_entries[i] = v[i].second.dead_entries;
    if (dead_bytes) dead_bytes[i] = v[i].second.dead_bytes;
  }
  return v.size();
}

uint64_t cask_db_current_sequence(const cask_db* db) { return db ? db->sequence + 1 : 0; }

uint64_t cask_db_files(const cask_db* db, uint32_t* ids, uint64_t cap) {
  if (!db) return 0;
  for (uint64_t i = 0; i < db->files.size() && i < cap; ++i) ids[i] = db->files[i];
  return db->files.size();
}

int cask_db_open_timings(const cask_db* db, double* ms5) {
  return cask_abi::guard([&]() -> int {
    if (!db || !ms5) return CASK_E_INVALID_ARG;
    memcpy(ms5, db->timings, sizeof(db->timings));
    return CASK_OK;
  });
}

}  // extern "C"
