// k_walk_runs — the speculative pass for logs of long records (walk mode), gfx950.
//
// k_scan_chunks stages every byte of a chunk to find and verify the records that start in it; on a
// log whose bytes are mostly in records longer than ScanArgs::big (configs[2]: Zipf value sizes up
// to 64 KiB, 96 % of the bytes in records > 2 KiB) those bytes are then read a second time by
// k_long_hash. Here a wave walks a run of chunks by chasing record headers (Entries::next,
// log.rs:403-429: each record starts where the previous one ends; a KiB staged in LDS per round
// trip), writing the rows and hashing the records that fit that KiB out of LDS; k_long_hash hashes
// the longer ones, so every byte is read about once.
//
// The output is the chunk table and slot rows of k_scan_chunks (spec, exit, count, long_r, cerr,
// long_done, slot rows; never a regular chunk), so k_finish, the validation/repair passes and
// k_long_hash run unchanged: a run's first start is speculative and k_finish checks it
// (spec[c] == T[c]) like any other.
//
// First start of a run (its first chunk's c0 != 0): the lowest offset >= c0 holding a record of at
// most ScanArgs::search_short bytes whose XXH32 matches (windows staged in LDS); then, going back, the
// lowest offset >= c0 whose header gives a record longer than that which ends exactly at the
// start found (repeated: a chain of long records before the first verified one).
#include "device_util.h"

#include <stdlib.h>

#include <algorithm>
#include "knobs.h"

namespace cask_dev {

constexpr uint32_t kWalkWin = 4096;                   // LDS window (16-B aligned)
constexpr uint32_t kWalkUse = kWalkWin - 16;          // bytes usable from any start in the window
constexpr uint32_t kStepB = kWalkUse - 18;            // candidate offsets per hop-back window
constexpr uint32_t kSearchPast = 1u << 20;            // pass A looks this far past the run's end
constexpr uint32_t kLongList = 256;  // pass A's long candidates kept for the hop back (64: no faster)
#ifdef CASK_STAMPS  // diagnostic build: per-wave s_memtime sums -> a.stamps[0..7] (tools/walk_stamps.py)
#define WST(v) const uint64_t v = __builtin_amdgcn_s_memtime();
#define WADD(i, v) wst[i] += __builtin_amdgcn_s_memtime() - (v);
#define WCNT(i) wst[i] += 1;
#else
#define WST(v)
#define WADD(i, v)
#define WCNT(i)
#endif

// LDS of a chasing wave (k_walk_runs): a 1-KiB window and the chunk state of its segment.
struct WalkLds {
  uint32_t win[1024 / 4 + 16];
  uint64_t spec[kMaxRun], exitv[kMaxRun];
  uint32_t cnt[kMaxRun], lr[kMaxRun], cerr[kMaxRun];
  // records of the window waiting for their checksum (walk_flush): LDS byte, length, chunk, row
  uint32_t hx[16], hrl[16], hj[16], hr[16];
  u32x4 hrow[16];
};

// A single-wave workgroup's claim of the next item of a work counter: every lane takes part in the
// atomic (adding 1 from lane 0, 0 from the rest) and lane 0's old value is read out. (No lane-0
// branch: with one, the compiler threads that branch into the claiming loop's back edge, the loop
// becomes a per-lane one, and the other lanes run on without lane 0 forever — k_walk_search hung
// that way, barriers or not, as a one-wave workgroup's barrier is only a wave barrier.)
__device__ __forceinline__ uint32_t wave_claim(unsigned int* ctr) {
  const uint32_t old = atomicAdd(ctr, threadIdx.x == 0 ? 1u : 0u);
  return __builtin_amdgcn_readfirstlane(old);
}

// Stage the window whose first usable byte is file byte wb: NL 16-B loads per lane (NL KiB), the
// file bytes [wb, min(wb + NL KiB - 16, len)) readable. Returns the LDS byte index of wb.
template <uint32_t NL>
__device__ __forceinline__ uint32_t walk_stage(uint32_t* W, const uint8_t* data, uint64_t len, uint64_t wb) {
  constexpr uint32_t use = NL * 1024 - 16;
  const uintptr_t g = (uintptr_t)(data + wb), a0 = g & ~(uintptr_t)15;
  const uint64_t we = (wb + use < len) ? wb + use : len;
  const uintptr_t aend = ((uintptr_t)(data + we) + 15) & ~(uintptr_t)15;
  const uint32_t n16 = (uint32_t)((aend - a0) >> 4);  // >= 1: wb < len
  typedef __attribute__((address_space(1))) const u32x4 gu32x4;
  const gu32x4* src = (const gu32x4*)a0;
  u32x4 v[NL];
#pragma unroll
  for (uint32_t k = 0; k < NL; ++k) {
    const uint32_t i = threadIdx.x + 64 * k;
    v[k] = src[i < n16 ? i : n16 - 1];
  }
  __syncthreads();  // every lane is done with the previous window
#pragma unroll
  for (uint32_t k = 0; k < NL; ++k) {
    const uint32_t i = threadIdx.x + 64 * k;
    ((u32x4*)W)[i < n16 ? i : n16 - 1] = v[k];
  }
  __syncthreads();
  return (uint32_t)(g - a0);
}
constexpr uint32_t kSearchNL = kWalkWin / 1024;  // the search's windows: 4 KiB
constexpr uint32_t kChaseNL = 1;                 // the chase's windows: 1 KiB
constexpr uint32_t kChaseUse = kChaseNL * 1024 - 16;
static_assert(kChaseUse == kWalkHashMax, "the walker hashes records that fit its window");

// The first record start >= b0 of the chain, speculatively (see the file comment); kNone if no
// verified short record is found before min(len, b1 + kSearchPast). A record's value_size field ends
// 17 bytes into its header, and a record that ends within the search horizon (or a tombstone) has a
// last value_size byte of 0x00 (0xFF) — only offsets whose byte +17 is 0x00 or 0xFF are decoded,
// found four at a time per aligned dword (SWAR zero-byte test), in 8-KiB windows. The short
// candidates of a window are hashed 16 at a time in offset order (lane l scans the window's dwords
// [32l, 32l + 32): lane order is offset order) until one verifies; long ones are listed for the hop
// back. The filter skips offsets whose record could neither be short nor end within the horizon,
// and offsets whose key_size is over 4,351 B (a run start after such a key is found later and
// k_finish's check sends the run to the repair: speed only).
#ifndef CASK_SW_NL  // (A/B variant: the window in KiB)
#define CASK_SW_NL 8
#endif
constexpr uint32_t kSwNL = CASK_SW_NL, kSwWin = kSwNL * 1024, kSwUse = kSwWin - 16, kSwStep = kSwUse - 18;
constexpr uint32_t kSwDw = 4 * kSwNL;  // dwords of candidate bytes per lane per window (64 x 32 x 4 >= kSwStep)
static_assert(64 * kSwDw * 4 >= kSwStep, "every candidate byte of a window is scanned");
#ifndef CASK_SW_PROBE  // (A/B variant: 0 = no chain probe)
#define CASK_SW_PROBE 16
#endif
constexpr uint32_t kProbeHops = CASK_SW_PROBE;  // phase 3: headers a long candidate's chain is followed for
struct SearchLdsSw {
  uint32_t wins[1][kSwWin / 4 + 16];
  uint32_t cand[16];
  uint32_t nl;
  uint32_t pad[3];
  // phase 3: a round's short records reached from long candidates (file offset, length, candidate)
  uint64_t pp[16];
  uint32_t prl[16], pcx[16];
  // long candidates as offsets from the run's first byte (x - b0 and x + rl - b0: both within the
  // run and kSearchPast past it, far below 2^32), 2 KiB instead of 4: more searching waves per CU
  uint32_t lx[kLongList], le[kLongList];
};

__device__ __forceinline__ uint64_t walk_search_sw(SearchLdsSw& L, const uint8_t* data, uint64_t len, uint64_t b0,
                                                   uint64_t b1, uint64_t* wst, uint32_t sshort) {
  const uint32_t lane = threadIdx.x, q = lane >> 2, qa = lane & 3;
  (void)wst;
  WST(ts0)
  const uint64_t lim = (b1 + kSearchPast < len) ? b1 + kSearchPast : len;
  uint64_t kA = kNone;
  if (lane == 0) L.nl = 0;
  bool over = false;
  uint32_t nl0 = 0;  // long candidates already followed by phase 3
  // (staging the next window into registers while this one is searched measured no faster: 207
  // VGPRs, 2 waves per SIMD instead of 3)
  for (uint64_t wb = b0; wb < lim && kA == kNone; wb += kSwStep) {
    WST(tw0)
    uint32_t* W = L.wins[0];
    const uint32_t x0 = walk_stage<kSwNL>(W, data, len, wb);  // (its barriers also publish L.nl)
    WADD(1, tw0)
    WCNT(5)
    WST(tw1)
    const uint64_t wend = (wb + kSwUse < len) ? wb + kSwUse : len;
    // offsets o in [0, ostop) of this window are candidates (their 18-B header is staged)
    const uint64_t oa = (lim - wb < kSwStep) ? lim - wb : kSwStep;
    const uint64_t ob = (len - wb >= 18) ? len - wb - 17 : 0;
    const uint32_t ostop = (uint32_t)(oa < ob ? oa : ob);
    // phase 1: candidate bytes (+17) of lane's dwords; short candidates into a bit mask (bit 4k+b
    // of sm[k>>4], k = the dword), long ones appended to the list. A candidate's key_size high byte
    // (+13, the same byte of the dword before) must be at most 0x10: keys over 4,351 B are left to
    // the repair (speed only), random bytes pass 1 time in 15.
    // lane l: the 16-B aligned dwords [d0, d0 + 32) (a lane-contiguous layout keeps lane order =
    // offset order), read as 8 ds_read_b128 in an order rotated by the lane — piece (j + l) % 8 at
    // read j — so that the 8 lanes of each LDS cycle hit 8 different bank quads (in plain order a
    // 128-B lane stride put every lane on 2 of them)
    const uint32_t d0 = (((x0 + 17) >> 2) & ~3u) + kSwDw * lane;
    constexpr uint32_t kP = kSwDw / 4, kG = kSwDw / 16;  // b128 pieces per lane; 64-bit masks of them
    uint64_t sm[kG];
#pragma unroll
    for (uint32_t g = 0; g < kG; ++g) sm[g] = 0ull;
    u32x4 wv[kP];
    const uint32_t dprev = W[d0 - 1];  // (x0 + 17 >= 17: d0 >= 4)
#pragma unroll
    for (uint32_t j = 0; j < kP; ++j) wv[j] = ((const u32x4*)W)[d0 / 4 + ((j + lane) & (kP - 1))];
#pragma unroll
    for (uint32_t j = 0; j < kP; ++j) {
      const uint32_t pc = (j + lane) & (kP - 1);  // the piece in wv[j]
#pragma unroll
      for (uint32_t e = 0; e < 4; ++e) {
        const uint32_t w = wv[j][e];
        const uint32_t wp = e ? wv[j][e - 1] : (pc ? wv[(j + kP - 1) & (kP - 1)][3] : dprev);
        const uint32_t kszhi_small = ~(((wp & 0x7F7F7F7Fu) + 0x6F6F6F6Fu) | wp) & 0x80808080u;  // byte < 0x11
        // bytes 0x00 or 0xFF: all eight bits equal, i.e. no bit differs from the one above it
        // (the shift's bit 7 comes from the next byte and is masked off); y <= 0x7F per byte, so
        // the add sets bit 7 exactly where y is not 0 and carries into no other byte
        const uint32_t y = (w ^ (w >> 1)) & 0x7F7F7F7Fu;
        uint32_t m = ~(y + 0x7F7F7F7Fu) & 0x80808080u & kszhi_small;
        const uint32_t k = 4 * pc + e;
        while (m) {
          const uint32_t b = (uint32_t)__builtin_ctz(m) >> 3;
          m &= m - 1;
          const int64_t o = (int64_t)(4 * (d0 + k) + b) - 17 - (int64_t)x0;
          if (o < 0 || o >= (int64_t)ostop) continue;
          const uint64_t rl = lds_reclen(W, x0 + (uint32_t)o);
          const uint64_t x = wb + (uint64_t)o;
          if (rl <= sshort) {
            if (x + rl <= len) sm[k >> 4] |= 1ull << (4 * (k & 15) + b);
          } else if (x + rl <= lim) {
            const uint32_t r = atomicAdd(&L.nl, 1u);
            if (r < kLongList) {
              L.lx[r] = (uint32_t)(x - b0);
              L.le[r] = (uint32_t)(x + rl - b0);
            } else {
              over = true;
            }
          }
        }
      }
    }
    WADD(2, tw1)
    WST(tw2)
    // phase 2: the short candidates in offset order, 16 per round (one per quad)
    for (;;) {
      WCNT(6)
      uint32_t mine = 0;
#pragma unroll
      for (uint32_t g = 0; g < kG; ++g) mine += (uint32_t)__builtin_popcountll(sm[g]);
      // exclusive prefix of the counts over lanes (lane order is offset order)
      uint32_t pre = mine;
      for (int s = 1; s < 64; s <<= 1) {
        const uint32_t u = __shfl_up(pre, s, 64);
        if ((int)lane >= s) pre += u;
      }
      const uint32_t total = __shfl(pre, 63, 64);
      pre -= mine;
      if (!total) break;
      // this lane's candidates with global rank < 16 go to cand[rank]
      uint32_t r = pre;
#pragma unroll
      for (uint32_t g = 0; g < kG; ++g) {
        while (sm[g] && r < 16) {
          const uint32_t bit = (uint32_t)__builtin_ctzll(sm[g]);
          sm[g] &= sm[g] - 1;
          const uint32_t k = 16 * g + (bit >> 2), b = bit & 3;
          L.cand[r++] = 4 * (d0 + k) + b - 17 - x0;
        }
      }
      __syncthreads();
      const uint32_t nc = total < 16 ? total : 16u;
      bool ok = false;
      if (q < nc) {
        const uint32_t ko = L.cand[q];
        const uint64_t xc = wb + ko;
        const uint64_t rlc = lds_reclen(W, x0 + ko);
        const uint32_t st = lds_u32(W, x0 + ko);
        const uint32_t h = (xc + rlc <= wend) ? quad_xxh32(W, x0 + ko + 4, (uint32_t)rlc - 4, qa)
                                               : quad_gbl_xxh32<2>(data + xc + 4, rlc - 4, qa);
        ok = qa == 0 && h == st;
      }
      const unsigned long long mo = __ballot(ok);
      if (mo) kA = wb + L.cand[__builtin_ctzll(mo) >> 2];  // quads are in offset order
      __syncthreads();
      if (mo) break;
    }
    WADD(3, tw2)
    // phase 3 (no short record of this window verified): each long candidate listed from this
    // window has its chain followed header to header (a lane each, one 16-B load per hop:
    // Entries::next, log.rs:403-429) to the first record of at most sshort bytes, within the horizon;
    // the lowest candidate whose chain reaches a record whose XXH32 matches is the start, as the
    // windows scanned one by one would find it — that record is the first short one after the
    // candidate, and the hop back below reaches the candidate from it. A stretch of 64-KiB records
    // then costs a few dependent loads instead of a window per 8 KiB. A false candidate (value bytes
    // that look like a header) lands on some true record start about once per mean record length
    // of its random "length", and its chain would then verify too: each hop must also raise the
    // sequence number by at most 2^32 (LogWriter appends records in sequence order: cask.rs:132-136,
    // log.rs:282-306), which random bytes pass about once in 2^32. A log whose sequence numbers do
    // not rise along a chain (a compaction's tombstone tail) is scanned window by window as before.
    // (Speed only: any start taken is checked by k_finish.)
    if (kProbeHops && kA == kNone) {
      __syncthreads();
      const uint32_t n1 = L.nl < kLongList ? L.nl : kLongList;
      uint64_t best = kNone;  // (uniform) the lowest verified candidate, as an offset from b0
      for (uint32_t c0 = nl0; c0 < n1; c0 += 64) {
        const uint32_t ci = c0 + lane;
        uint64_t tp = kNone;
        uint32_t trl = 0;
        if (ci < n1) {
          uint64_t p = b0 + L.le[ci];
          // the candidate's sequence number, from its header in this window
          uint64_t sq = lds_hdr(W, x0 + (uint32_t)(b0 + L.lx[ci] - wb)).seq;
          for (uint32_t hop = 0; hop < kProbeHops; ++hop) {
            if (p >= lim || p + 18 > len) break;
            const u32x4 hd = gld16g((const g_u8*)(data + p + 2));  // header bytes 2..17
            const uint32_t ksz = hd.z >> 16, vsz = hd.w;
            const uint64_t sn = (uint64_t)fun(hd.x, hd.y, 2) | ((uint64_t)fun(hd.y, hd.z, 2) << 32);
            if (ksz > 4351u || ((vsz >> 24) != 0u && vsz != 0xFFFFFFFFu)) break;  // (not a record)
            if (sn <= sq || sn - sq > (1ull << 32)) break;  // (sequence numbers rise along a log)
            sq = sn;
            const uint64_t rl = 18ull + ksz + (vsz == 0xFFFFFFFFu ? 0ull : (uint64_t)vsz);
            if (rl <= sshort) {
              if (p + rl <= len) {
                tp = p;
                trl = (uint32_t)rl;
              }
              break;
            }
            p += rl;
          }
        }
        // the reached records, 16 per round (a quad each), in candidate-list order
        const unsigned long long hm = __ballot(tp != kNone);
        const uint32_t nh = (uint32_t)__builtin_popcountll(hm);
        const uint32_t rank = (uint32_t)__builtin_popcountll(hm & (lane ? (~0ull >> (64 - lane)) : 0ull));
        for (uint32_t r0 = 0; r0 < nh; r0 += 16) {
          if (tp != kNone && rank >= r0 && rank < r0 + 16) {
            L.pp[rank - r0] = tp;
            L.prl[rank - r0] = trl;
            L.pcx[rank - r0] = L.lx[ci];
          }
          __syncthreads();
          const uint32_t nq = nh - r0 < 16 ? nh - r0 : 16u;
          uint64_t x = kNone;
          if (q < nq) {
            const uint64_t pq = L.pp[q];
            const uint32_t rq = L.prl[q];
            const uint32_t st = gld4g((const g_u8*)(data + pq));
            const uint32_t h = quad_gbl_xxh32<2>(data + pq + 4, rq - 4, qa);
            if (qa == 0 && h == st) x = L.pcx[q];
          }
          for (int s = 32; s; s >>= 1) {
            const uint64_t y = __shfl_xor(x, s, 64);
            x = y < x ? y : x;
          }
          best = x < best ? x : best;
          __syncthreads();
        }
      }
      nl0 = n1;
      if (best != kNone) kA = b0 + best;
    }
  }
  over = __any(over) || L.nl > kLongList;
  WST(th0)
  if (kA == kNone) return kNone;
  // hop back over long records ending exactly at the current target (lowest such offset)
  uint64_t target = kA;
  const uint32_t nlist = L.nl < kLongList ? L.nl : kLongList;
  for (int it = 0; it < 64; ++it) {
    uint64_t found = kNone;
    if (!over) {
      for (uint32_t i0 = 0; i0 < nlist; i0 += 64) {
        const uint32_t i = i0 + lane;
        uint64_t x = (i < nlist && b0 + L.lx[i] < target && b0 + L.le[i] == target) ? b0 + L.lx[i] : kNone;
        for (int s = 32; s; s >>= 1) {
          const uint64_t y = __shfl_xor(x, s, 64);
          x = y < x ? y : x;
        }
        found = x < found ? x : found;
      }
    } else {
      for (uint64_t wb = b0; wb < target && found == kNone; wb += kStepB) {
        const uint32_t x0 = walk_stage<kSearchNL>(L.wins[0], data, len, wb);
        for (uint32_t k0 = 0; k0 < kStepB; k0 += 64) {
          const uint64_t x = wb + k0 + lane;
          bool hit = false;
          if (k0 + lane < kStepB && x < target && x + 18 <= len) {
            const uint64_t rl = lds_reclen(L.wins[0], x0 + k0 + lane);
            hit = rl > sshort && x + rl == target;
          }
          const unsigned long long m = __ballot(hit);
          if (m) {
            found = wb + k0 + (uint64_t)__builtin_ctzll(m);
            break;
          }
        }
      }
    }
    if (found == kNone) break;
    target = found;
  }
  WADD(4, th0)
  WADD(0, ts0)
  WCNT(7)
  return target;
}

// Hint-file bodies (cask_parse_hints_device): records `seq u64 | ksz u16 | vsz u32 | entry_pos u64 |
// key` (Hint::write_bytes, data.rs:242-256), 22 + ksz bytes, no checksum of their own. A run's first
// start is the lowest offset >= b0 whose record, and the two after it, have entry positions that
// follow on from each other (each data record starts where the previous one ended: RecreateHints
// writes one hint per Ok record in order, log.rs:454-465) — or whose record ends the body exactly.
// The chain is then checked by k_finish like any speculated start.
__device__ __forceinline__ uint64_t hint_field64(const uint32_t* W, uint32_t x) {
  return (uint64_t)lds_u32(W, x) | ((uint64_t)lds_u32(W, x + 4) << 32);
}
__device__ __forceinline__ uint64_t hint_search(WalkLds& L, const uint8_t* data, uint64_t len, uint64_t b0, uint64_t b1) {
  const uint32_t lane = threadIdx.x;
  constexpr uint32_t step = kChaseUse - 22;  // (1-KiB windows: hint records are small)
  for (uint64_t wb = b0; wb < b1; wb += step) {
    const uint32_t x0 = walk_stage<kChaseNL>(L.win, data, len, wb);
    const uint64_t wend = (wb + kChaseUse < len) ? wb + kChaseUse : len;
    for (uint32_t k0 = 0; k0 < step; k0 += 64) {
      const uint64_t x = wb + k0 + lane;
      bool hit = false;
      if (k0 + lane < step && x < b1 && x + 22 <= wend) {
        uint64_t y = x, pos = 0;
        hit = true;
        for (int h = 0; h < 3; ++h) {  // x and the two records after it
          const uint32_t xi = x0 + (uint32_t)(y - wb);
          const uint32_t ksz = lds_u32(L.win, xi + 8) & 0xFFFFu, vsz = lds_u32(L.win, xi + 10);
          const uint64_t ep = hint_field64(L.win, xi + 14);
          if (h && ep != pos) {  // not where the previous record's entry ended
            hit = false;
            break;
          }
          pos = ep + 18 + ksz + (vsz == 0xFFFFFFFFu ? 0ull : (uint64_t)vsz);
          y += 22ull + ksz;
          if (y == len || h == 2) break;  // ends the body exactly, or three records chained
          if (y + 22 > wend) {            // past the body, or the next header is not staged
            hit = false;
            break;
          }
        }
      }
      const unsigned long long m = __ballot(hit);
      if (m) return wb + k0 + (uint64_t)__builtin_ctzll(m);
    }
  }
  return kNone;
}

// The window's records waiting for their checksum (lane 0 listed them: LDS byte, length, chunk,
// row): a quad per record hashes it out of the window (Entry::from_read's check, data.rs:193-198),
// then writes its slot row with the verdict; a failure lowers its chunk's first failing row.
// Runs before the window is restaged and before the segment's chunk state goes out.
__device__ __forceinline__ void walk_flush(WalkLds& L, const ScanArgs& a, uint64_t t0, uint32_t n) {
  const uint32_t lane = threadIdx.x, q = lane >> 2, qa = lane & 3;
  __syncthreads();  // the list is in LDS
  if (q < n) {      // whole quads
    const uint32_t x = L.hx[q], rl = L.hrl[q];
    const uint32_t h = quad_xxh32(L.win, x + 4, rl - 4, qa);
    if (qa == 0) {
      u32x4 row = L.hrow[q];
      const uint32_t j = L.hj[q], r = L.hr[q];
      if (h != lds_u32(L.win, x)) {
        row.w |= kSlotBad;
        atomicMin(&L.cerr[j], r);
      }
      *(u32x4*)(a.slots + ((t0 + j) * (uint64_t)a.slot_cap + r) * 4) = row;
    }
  }
  __syncthreads();  // before the list or the window is reused
}

// One stretch of a run inside one file: chunks [t0, t1) of file fd.
// s_in: the exact start of the segment's first chunk (repair passes: spec[t0]), or kSearch for a
// speculative one. Returns the chain position after the segment (kTerm after an EOF row).
// Data files: a record of at most ScanArgs::big bytes (kWalkHashMax: the window's usable bytes) is
// hashed out of the chase's window — when it runs past the window the window is restaged at its
// header first — 16 at a time or when the window moves on (walk_flush); longer ones are left to
// k_long_hash (long_r). Hint bodies have no checksums.
constexpr uint64_t kSearch = ~0ull - 1;
__device__ __forceinline__ uint64_t walk_segment(WalkLds& L, const ScanArgs& a, const FileDesc& fd, uint64_t t0, uint64_t t1,
                                 uint64_t s_in, uint64_t* wst) {
  const uint32_t lane = threadIdx.x;
  const uint32_t nch = (uint32_t)(t1 - t0);
  const uint64_t CH = a.chunk, len = fd.len;
  const uint32_t csh = (uint32_t)__builtin_ctz(a.chunk);
  const uint8_t* data = fd.data;
  const uint64_t b0 = (t0 - fd.first_chunk) * CH;
  const uint64_t b1 = ((t1 - fd.first_chunk) * CH < len) ? (t1 - fd.first_chunk) * CH : len;
  if (lane < nch) {
    L.spec[lane] = kNone;
    L.exitv[lane] = 0;
    L.cnt[lane] = 0;
    L.lr[lane] = 0xFFFFFFFFu;
    L.cerr[lane] = 0xFFFFFFFFu;
  }
  __syncthreads();
  WST(ts0)
  const bool hint = a.hint != 0;
  const uint32_t hdr = hint ? 22u : 18u;
  // (data files get their speculative starts from k_walk_search: here only hint bodies search)
  uint64_t p = uni64(b0 == 0 ? 0 : s_in != kSearch ? s_in : hint ? hint_search(L, data, len, b0, b1) : kNone);
  WADD(0, ts0)
  if (b0 && s_in == kSearch) { WCNT(6) }
  // the chase: uniform state of the chunk the chain is in
  uint32_t cj = 0xFFFFFFFFu, cn = 0;  // current chunk (segment index) and its rows so far
  uint64_t wb = 0, wv = 0;  // the chase's window: file bytes [wb, wv) at LDS byte x0
  uint32_t x0 = 0;
  uint32_t nh = 0;  // records listed for walk_flush
  auto stage = [&](uint64_t at) {  // the next KiB from `at`, after the listed records are hashed
    if (nh) walk_flush(L, a, t0, nh);
    nh = 0;
    WST(tw0)
    x0 = walk_stage<kChaseNL>(L.win, data, len, at);
    WADD(1, tw0)
    WCNT(4)
    wb = at;
    wv = (at + kChaseUse < len) ? at + kChaseUse : len;
  };
  while (p != kNone && p < b1) {
    const uint32_t j = (uint32_t)((p - b0) >> csh);  // chunk sizes are powers of two
    if (j != cj) {  // the chain enters chunk j: the previous chunk's rows and exit are final
      if (cj != 0xFFFFFFFFu && lane == 0) {
        L.cnt[cj] = cn;
        L.exitv[cj] = p;
      }
      cj = j;
      cn = 0;
      if (lane == 0) L.spec[j] = p;
    }
    WCNT(5)
    const uint32_t off = (uint32_t)(p - b0 - (uint64_t)j * CH);
    const uint32_t r = cn++;
    u32x4 row = u32x4{0u, 0u, 0u, off << 16};
    bool fail = false, eof = false;
    uint64_t rl = 0;
    if (p + hdr > len) {
      fail = eof = true;  // header cut short: Io(UnexpectedEof) (data.rs:163; a hint: data.rs:258-265)
    } else {
      if (p < wb || p + hdr > wv) stage(p);  // the header is not staged: one round trip brings the next KiB
      Hdr h;
      if (hint) {  // seq u64 | ksz u16 | vsz u32 | entry_pos u64
        const uint32_t xi = x0 + (uint32_t)(p - wb);
        h.stored = 0;
        h.seq = hint_field64(L.win, xi);
        h.ksz = lds_u32(L.win, xi + 8) & 0xFFFFu;
        h.vsz = lds_u32(L.win, xi + 10);
      } else {
        h = lds_hdr(L.win, x0 + (uint32_t)(p - wb));
      }
      // wave-uniform: into scalar registers
      h.seq = uni64(h.seq);
      h.ksz = __builtin_amdgcn_readfirstlane(h.ksz);
      h.vsz = __builtin_amdgcn_readfirstlane(h.vsz);
      row = u32x4{(uint32_t)h.seq, (uint32_t)(h.seq >> 32), h.vsz, h.ksz | (off << 16)};
      rl = hint ? 22ull + h.ksz : 18ull + h.ksz + ((h.vsz == 0xFFFFFFFFu) ? 0ull : (uint64_t)h.vsz);
      if (p + rl > len) fail = eof = true;  // key/value cut short (data.rs:172,181; a hint's key: :266-270)
    }
    // a data record of at most `big` bytes is hashed out of the window (restaged at its header if
    // it runs past the window's end: it then fits, as big <= kChaseUse)
    const bool inwin = !hint && !fail && rl <= a.big;
    if (inwin) {
      if (p + rl > wv) stage(p);
      if (lane == 0) {
        L.hx[nh] = x0 + (uint32_t)(p - wb);
        L.hrl[nh] = (uint32_t)rl;
        L.hj[nh] = j;
        L.hr[nh] = r;
        L.hrow[nh] = row;
      }
      if (++nh == 16) {
        walk_flush(L, a, t0, nh);
        nh = 0;
      }
    } else if (lane == 0) {  // the row goes out now: an EOF row fails here, a longer record is k_long's
      *(u32x4*)(a.slots + ((t0 + j) * (uint64_t)a.slot_cap + r) * 4) = row;
      if (fail) atomicMin(&L.cerr[j], r);
      else if (!hint) atomicMin(&L.lr[j], r);  // (rl > big: not lds_hashed, data.rs:193-198 in k_long_hash)
    }
    if (eof) {
      if (lane == 0) {
        L.cnt[j] = cn;
        L.exitv[j] = kTerm;
      }
      cj = 0xFFFFFFFFu;
      break;
    }
    p += rl;
  }
  if (nh) walk_flush(L, a, t0, nh);
  if (cj != 0xFFFFFFFFu && lane == 0) {
    L.cnt[cj] = cn;
    L.exitv[cj] = p;  // >= b1, the end of the segment's last chunk
  }
  __syncthreads();
  if (lane < nch) {
    const uint64_t t = t0 + lane;
    const uint64_t sp = L.spec[lane];
    a.spec[t] = sp;
    a.exit[t] = sp == kNone ? 0ull : L.exitv[lane];
    a.count[t] = L.cnt[lane];
    a.long_r[t] = L.lr[lane];
    a.cerr[t] = L.cerr[lane];
    a.long_done[t] = 0;
  }
  __syncthreads();
  return cj == 0xFFFFFFFFu && p != kNone && p < b1 ? kTerm : p;
}

// Persistent grid of single-wave workgroups; runs of a.run chunks claimed from ctr->run_next.
__global__ __launch_bounds__(64) void k_walk_runs(ScanArgs a, const FileDesc* __restrict__ files) {
  __shared__ WalkLds L;
  uint64_t wst[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  WST(tk0)
  const uint64_t R = a.run;
  // a repair pass walks the stretches in a.runs from their exact starts (spec[first]); otherwise
  // runs of R chunks, each from a speculative start
  const uint64_t nruns = a.runs ? a.nruns_list : a.run_hi ? a.run_hi : (a.total_chunks + R - 1) / R;
  // the first run of every wave is fixed by its index, later ones come from the counter
  for (uint64_t k = blockIdx.x;; k = gridDim.x + (a.runs ? wave_claim(&a.ctr->run_next) : wave_claim(&a.ctr->walk_next[a.grp]))) {
    const uint64_t r = a.runs ? k : a.run_lo + k;
    if (r >= nruns) break;
    uint64_t t = a.runs ? a.runs[2ull * r] : (uint64_t)r * R;
    const uint64_t tend = a.runs ? a.runs[2ull * r + 1] : ((t + R < a.total_chunks) ? t + R : a.total_chunks);
    uint64_t s = a.runs ? uni64(a.spec[t]) : a.walk_pre ? uni64(a.tin[t]) : kSearch;
    while (t < tend) {
      const uint32_t fi = find_file(files, a.nfiles, t);
      const FileDesc fd = files[fi];
      const uint64_t fend = fd.first_chunk + fd.nchunks;
      uint64_t se = fend < tend ? fend : tend;
      if (se - t > kMaxRun) se = t + kMaxRun;  // the chunk state of a segment lives in LDS
      const uint64_t ex = walk_segment(L, a, fd, t, se, s, wst);
      // the next piece of a stretch continues the chain; a new file starts at 0 (walk_segment)
      s = a.runs ? ex : kSearch;
      t = se;
    }
  }
#ifdef CASK_STAMPS
  WADD(3, tk0)
  if (a.stamps && threadIdx.x == 0)
    for (int i = 0; i < 8; ++i) atomicAdd(&a.stamps[i], (unsigned long long)wst[i]);
#endif
}

// Each walk run's speculative first start (walk_search), ahead of the chase: a run whose first chunk
// starts a file needs none, and only the first segment of a run can. Kept out of k_walk_runs: the
// search's registers would lower how many chasing waves fit on a CU.
// (At most 168 VGPRs, so that 3 searching waves fit a SIMD instead of 2 at the 193 the compiler
// takes unbounded — 12 bytes per lane of spill: search 0.54-0.59 -> 0.47-0.48 ms on configs[2];
// at 128 VGPRs, 4 per SIMD, the spills cost more than the waves bring: 0.56-0.58 ms.)
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(3))) void k_walk_search(ScanArgs a, const FileDesc* __restrict__ files) {
  __shared__ SearchLdsSw L;
  uint64_t wst[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  (void)wst;
  const uint64_t R = a.run;
  const uint64_t nruns = a.wruns ? a.nwruns : a.run_hi ? a.run_hi : (a.total_chunks + R - 1) / R;
  for (uint64_t k = blockIdx.x;; k = gridDim.x + wave_claim(&a.ctr->search_next[a.grp])) {
    const uint64_t r = a.wruns ? k : a.run_lo + k;
    if (r >= nruns) break;
    const uint64_t t = (a.wruns ? a.wruns[r] : r) * R;
    const uint32_t fi = find_file(files, a.nfiles, t);
    const FileDesc fd = files[fi];
    const uint64_t fend = fd.first_chunk + fd.nchunks;
    const uint64_t tend = (t + R < a.total_chunks) ? t + R : a.total_chunks;
    const uint64_t se = fend < tend ? fend : tend;
    const uint64_t b0 = (t - fd.first_chunk) * (uint64_t)a.chunk;
    const uint64_t b1 = ((se - fd.first_chunk) * (uint64_t)a.chunk < fd.len) ? (se - fd.first_chunk) * (uint64_t)a.chunk : fd.len;
#ifdef CASK_STAMPS
    const uint64_t rt0 = __builtin_amdgcn_s_memrealtime();
    const uint64_t win0 = wst[5];
#endif
    const uint64_t s0 = b0 == 0 ? 0 : walk_search_sw(L, fd.data, fd.len, b0, b1, wst, a.search_short);
    if (threadIdx.x == 0) a.tin[t] = s0;
#ifdef CASK_STAMPS
    if (a.stamps && threadIdx.x == 0 && r < kStampRuns) {  // per search: start, end, windows, wave
      unsigned long long* sr = a.stamps + 16 + 2ull * kStampWaves + 4 * r;
      sr[0] = rt0;
      sr[1] = __builtin_amdgcn_s_memrealtime();
      sr[2] = wst[5] - win0;
      sr[3] = blockIdx.x;
    }
#endif
  }
#ifdef CASK_STAMPS
  if (a.stamps && threadIdx.x == 0)
    for (int i = 0; i < 8; ++i) atomicAdd(&a.stamps[i], (unsigned long long)wst[i]);
#endif
}


// Record lengths at kProbeRegions points of every file (one wave per file and point), for the scan
// mode of each region (speed only: every mode reads every file correctly). Point 0 is the file's
// head, walked exactly; point s > 0 is s/kProbeRegions of the way in, where the first offset of a
// 4-KiB window from which four headers chain plausibly (key <= 4 KiB, value inside the file,
// each record inside the file) is taken as a record start. Up to 32 records are walked from it:
// out[3 * (f * kProbeRegions + s)] = {bytes, records, longest}. No start in the window (a record
// longer than it covers the point): {window, 0, window}.
__device__ __forceinline__ bool probe_chain(const uint8_t* d, uint64_t len, uint64_t p) {
#pragma unroll 1
  for (int j = 0; j < 4; ++j) {
    if (p == len) return j > 0;  // the file ends exactly at a record boundary
    if (p + 18 > len) return false;
    const uint32_t b3 = gld4(d + p + 12);
    const uint32_t ksz = b3 & 0xFFFFu;
    const uint32_t vsz = (b3 >> 16) | ((uint32_t)d[p + 16] << 16) | ((uint32_t)d[p + 17] << 24);
    if (ksz > 4096u) return false;
    const uint64_t rl = 18ull + ksz + (vsz == 0xFFFFFFFFu ? 0ull : (uint64_t)vsz);
    if (p + rl > len) return false;
    p += rl;
  }
  return true;
}

__global__ __launch_bounds__(64) void k_probe_regions(const FileDesc* __restrict__ files, uint32_t nfiles,
                                                      unsigned long long* __restrict__ out) {
  const uint32_t f = blockIdx.x / kProbeRegions, s = blockIdx.x % kProbeRegions, lane = threadIdx.x;
  if (f >= nfiles) return;
  const FileDesc fd = files[f];
  const uint64_t x = fd.len * s / kProbeRegions;
  constexpr uint32_t kWin = 4096;
  uint64_t p0 = kNone;
  if (s == 0) {
    p0 = 0;
  } else {
    for (uint32_t i = 0; i < kWin / 64 && p0 == kNone; ++i) {
      const uint64_t p = x + 64ull * i + lane;
      const bool ok = p < fd.len && probe_chain(fd.data, fd.len, p);
      const unsigned long long b = __ballot(ok);
      if (b) p0 = x + 64ull * i + (uint64_t)__builtin_ctzll(b);
    }
  }
  if (lane) return;
  uint64_t bytes = 0, recs = 0, mx = 0;
  if (p0 == kNone) {
    bytes = kWin;
    mx = kWin;
  } else {
    uint64_t p = p0;
    for (int k = 0; k < 32 && p + 18 <= fd.len; ++k) {
      const uint64_t rl = g_reclen(fd.data + p);
      if (p + rl > fd.len) break;
      bytes += rl;
      ++recs;
      mx = rl > mx ? rl : mx;
      p += rl;
    }
  }
  unsigned long long* o = out + 3ull * blockIdx.x;
  o[0] = bytes;
  o[1] = recs;
  o[2] = mx;
}

// Runs a launch covers: its group's, or the repair pass's list.
static uint64_t launch_runs(const ScanArgs& a) {
  if (a.runs) return a.nruns_list;
  if (a.wruns) return a.nwruns;
  const uint64_t hi = a.run_hi ? a.run_hi : (a.total_chunks + a.run - 1) / a.run;
  return hi > a.run_lo ? hi - a.run_lo : 0;
}

void launch_walk_runs(const ScanArgs& a, void* stream) {
  const uint64_t nruns = launch_runs(a);
  if (!a.total_chunks || !nruns) return;
  // CASK_WALK_WAVES (tuning knob): waves per CU of the persistent grid
  // (7 waves per SIMD fit: 66 VGPRs, 2.9 KB of LDS)
  static const uint32_t per_cu = cask_knobs::tune("CASK_WALK_WAVES") ? (uint32_t)atoi(cask_knobs::tune("CASK_WALK_WAVES")) : 28u;
  uint64_t grid = (uint64_t)device_cus() * per_cu;
  if (grid > nruns) grid = nruns;
  hipLaunchKernelGGL(k_walk_runs, dim3((uint32_t)grid), dim3(64), 0, (hipStream_t)stream, a, a.files);
}

void launch_walk_search(const ScanArgs& a, void* stream, int cus) {
  const uint64_t nruns = launch_runs(a);
  if (!a.total_chunks || !nruns) return;
  // A persistent grid of exactly the resident workgroups (LDS-bound: ~12 per CU): a workgroup
  // beyond them would start only as the first ones finish, holding its first run (by block index)
  // until the end of the kernel.
  static int per_cu = 0;
  if (!per_cu) {
    int nb = 0;
    if (cask_knobs::tune("CASK_SEARCH_WAVES")) per_cu = atoi(cask_knobs::tune("CASK_SEARCH_WAVES"));  // (tuning)
    else if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_walk_search, 64, 0) == hipSuccess && nb > 0) per_cu = nb;
    if (per_cu <= 0) per_cu = 12;
  }
  uint64_t grid = (uint64_t)(cus > 0 ? cus : device_cus()) * (uint64_t)per_cu;
  if (grid > nruns) grid = nruns;
  hipLaunchKernelGGL(k_walk_search, dim3((uint32_t)grid), dim3(64), 0, (hipStream_t)stream, a, a.files);
}


void launch_probe_regions(const FileDesc* files, uint32_t nfiles, unsigned long long* out, void* stream) {
  if (!nfiles) return;
  hipLaunchKernelGGL(k_probe_regions, dim3(nfiles * kProbeRegions), dim3(64), 0, (hipStream_t)stream, files, nfiles,
                     out);
}

}  // namespace cask_dev
