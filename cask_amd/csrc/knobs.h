// Environment knobs, of two kinds; a plain run of the product library reads neither:
//  * test hooks force the paths the tests cover — CASK_SCAN_MODE (walk|chunk|wide|narrow),
//    CASK_HOST_THREADS, CASK_OPEN_BATCH, CASK_OPEN_DEVFOLD, CASK_OPEN_TRACE, CASK_PAR_FOLD_MIN, CASK_STAGE_MIN, CASK_LOCAL_REPAIRS,
//    CASK_NO_REPAIR, CASK_KD_HASH_BITS — and are read only when CASK_TEST_HOOKS=1 is in the environment when the library
//    is first used (tests/conftest.py sets it; bench.py refuses to run with it);
//  * tuning knobs (the A/B studies recorded in DESIGN.md: run lengths, grid sizes, hash depth, ...)
//    exist only in diagnostic builds compiled with -DCASK_TUNING (`make -C cask_amd variant
//    VNAME=x VDEF=-DCASK_TUNING`, tools/ab.py), never in libcask_scan.so.
// Every result of the library depends on its arguments alone; these change only its speed, or
// which of several exact paths computes the same rows.
#pragma once
#include <cstdlib>
#include <cstring>

namespace cask_knobs {

inline bool test_hooks() {
  static const bool on = [] {
    const char* e = getenv("CASK_TEST_HOOKS");
    return e && strcmp(e, "1") == 0;
  }();
  return on;
}

// A test hook's value, or nullptr.
inline const char* hook(const char* name) { return test_hooks() ? getenv(name) : nullptr; }

// A tuning knob's value (diagnostic builds only), or nullptr.
#ifdef CASK_TUNING
inline const char* tune(const char* name) { return getenv(name); }
#else
inline const char* tune(const char*) { return nullptr; }
#endif

}  // namespace cask_knobs
