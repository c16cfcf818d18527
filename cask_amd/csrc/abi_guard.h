// No C++ exception crosses the C ABI (include/cask_scan.h): every entry point that allocates, locks a
// mutex or starts threads runs its body under cask_abi::guard — std::bad_alloc (host memory
// pressure: a huge hint file, a keydir at cfg5 scale, the row staging of a large host scan) becomes
// CASK_E_NOMEM, anything else (std::system_error from a thread or a mutex, std::length_error)
// CASK_E_IO. The reference's Error (errors.rs:12-25) has no variant for either; the status is the
// C ABI's own.
#pragma once
#include <cstdint>
#include <new>

#include "../../include/cask_scan.h"

namespace cask_abi {

template <class F>
inline auto guard(F&& f) noexcept -> decltype(f()) {
  try {
    return f();
  } catch (const std::bad_alloc&) {
    return CASK_E_NOMEM;
  } catch (...) {
    return CASK_E_IO;
  }
}

// Test hooks (cask_debug_inject, effective only under CASK_TEST_HOOKS=1): failures forced on one
// context, so that a multi-rank test can make exactly one rank fail at a chosen point. Each bit is
// taken (cleared) by the first place that checks it.
constexpr uint32_t kInjRootAlloc = 1;  // the gather root's receive buffer cannot be allocated
constexpr uint32_t kInjPartition = 2;  // cask_keydir_partition runs out of device memory
constexpr uint32_t kInjTerms = 4;      // the exchange's per-file terms table cannot be read
constexpr uint32_t kInjThrow = 8;      // the next guarded entry point throws std::bad_alloc
constexpr uint32_t kInjFold = 16;      // the fold of the received blocks fails (CASK_E_NOMEM)
bool take_inject(cask_ctx* c, uint32_t bit);
inline void maybe_throw(cask_ctx* c) {
  if (take_inject(c, kInjThrow)) throw std::bad_alloc();
}

}  // namespace cask_abi
