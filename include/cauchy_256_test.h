/* cauchy_256_test.h -- test-only hooks (not part of the drop-in API).  Exported by the checked
 * build only (liblonghair_amd_check.so, `make LH_DEBUG=1`, which defines LH_TEST_HOOKS); the
 * product library liblonghair_amd.so has none, so no caller can inject a failure into it.
 *
 * SURVEY 8(b) asks that no C++ exception crosses the C ABI: every int-returning entry point
 * of cauchy_256.h, cauchy_256_batch.h and cauchy_256_dispatch.h catches whatever the
 * implementation throws (std::bad_alloc, std::system_error, ...) and returns -3 with
 * cauchy_256_last_error() naming it.  This hook proves it: after it, the calling thread's
 * next such call throws inside that barrier (tests/test_abi.py). */
#ifndef CAUCHY_256_TEST_H
#define CAUCHY_256_TEST_H

#ifdef __cplusplus
extern "C" {
#endif

void cauchy_256_debug_throw_next(void);

#ifdef __cplusplus
}
#endif

#endif /* CAUCHY_256_TEST_H */
