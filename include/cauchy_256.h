/*
 * cauchy_256.h -- drop-in C ABI of the MI355X Cauchy Reed-Solomon codec (longhair_amd).
 *
 * Declares exactly the entry points a caller of catid/longhair's cauchy_256.h binds:
 *
 *   _cauchy_256_init / cauchy_256_init()  replaces reference cauchy_256.h:47-48
 *                                          (implementation cauchy_256.cpp:390-399)
 *   cauchy_256_encode                      replaces reference cauchy_256.h:78
 *                                          (implementation cauchy_256.cpp:1495-1594)
 *   cauchy_256_decode                      replaces reference cauchy_256.h:103
 *                                          (implementation cauchy_256.cpp:1249-1408)
 *   Block                                  same layout as reference cauchy_256.h:52-55
 *
 * Behaviour follows the reference implementation (not its header comments):
 *   - init returns 0 on success, -1 on a version mismatch.  Without a HIP device it still
 *     returns 0 under the AUTO (default) and HOST dispatch policies (cauchy_256_dispatch.h):
 *     the drop-in calls then run on the library's host SIMD engine; under the GPU policy
 *     init and the drop-in calls return -2.  No C++ exception crosses this ABI: an internal
 *     one returns -3 (cauchy_256_last_error() names it).
 *   - encode writes m * block_bytes bytes to recovery_blocks.  Recovery block 0 is the
 *     XOR of the k data blocks and is written before parameters are validated; with
 *     m > 1, k + m > 256 or block_bytes % 8 != 0 then returns -1.  k <= 1 copies data[0]
 *     into every recovery block.
 *   - decode recovers erased originals in place: the i-th recovery Block (array order)
 *     receives the i-th missing original row (ascending) and its row field is
 *     rewritten.  -1 when erasures are present and k + m > 256 or block_bytes % 8 != 0.
 *   - any HIP failure returns -3.  For m > 1, rows that index outside the code
 *     (row >= k + m) or duplicated rows return -1 instead of the reference's undefined
 *     behaviour; for m = 1 any rows are accepted, as by the reference's cauchy_decode_m1
 *     (cauchy_256.cpp:487-535: every row >= k is a recovery block, the last one in array
 *     order is the output).
 *
 * Buffers may be host memory (pageable or pinned) or HIP device memory.  Where a call runs
 * is the dispatch policy of cauchy_256_dispatch.h: by default (AUTO) a small all-host call
 * runs on the host SIMD engine and every other call on the GPU.  No GPU is needed under
 * AUTO or HOST: without one every drop-in call runs on the host engine (under GPU, init and
 * the drop-in calls return -2).  For batches of stripes
 * resident in device memory use
 * cauchy_256_batch.h, which avoids the per-call PCIe round trip.
 */
#ifndef LONGHAIR_AMD_CAUCHY_256_H
#define LONGHAIR_AMD_CAUCHY_256_H

#ifdef __cplusplus
extern "C" {
#endif

#define CAUCHY_256_VERSION 2

extern int _cauchy_256_init(int expected_version);
#define cauchy_256_init() _cauchy_256_init(CAUCHY_256_VERSION)

typedef struct _Block {
    unsigned char *data;
    unsigned char row;
} Block;

extern int cauchy_256_encode(int k, int m, const unsigned char *data_ptrs[],
                             void *recovery_blocks, int block_bytes);

extern int cauchy_256_decode(int k, int m, Block *blocks, int block_bytes);

#ifdef __cplusplus
}
#endif

#endif /* LONGHAIR_AMD_CAUCHY_256_H */
