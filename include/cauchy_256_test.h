/* cauchy_256_test.h -- test-only hooks of liblonghair_amd.so (not part of the drop-in API).
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
