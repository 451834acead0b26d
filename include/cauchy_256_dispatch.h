/*
 * cauchy_256_dispatch.h -- where the drop-in entry points of cauchy_256.h run.
 *
 * Not part of the reference API.  The reference codes one stripe per call on the host
 * CPU (cauchy_256.h:78, :103; README.md:111-182).  Staging such a call to the GPU costs
 * tens of microseconds of PCIe round trip for a stripe whose XOR work takes about two
 * microseconds of host SIMD.  The policy chooses:
 *
 *   CAUCHY_256_DISPATCH_GPU  (0)  every drop-in call runs on the GPU.
 *   CAUCHY_256_DISPATCH_AUTO (1, default)  a call whose blocks all live in host memory
 *        and whose XOR work (sub-block bytes times bit-matrix terms) is at most
 *        `host_max_work` bytes runs on the host SIMD engine (AVX-512BW / AVX2); larger
 *        calls, and calls with device pointers, run on the GPU.  An unchanged caller of
 *        the reference API therefore keeps host-CPU latency for small stripes.
 *   CAUCHY_256_DISPATCH_HOST (2)  every all-host-memory call runs on the host engine.
 *
 * Both engines return the same bytes and codes.  The library requires a HIP device under
 * every policy (cauchy_256_init returns -2 without one).  The initial policy comes from
 * the environment: LONGHAIR_AMD_DISPATCH=auto|gpu|host, LONGHAIR_AMD_HOST_MAX_WORK=bytes
 * (default 4 MiB).  The batched API (cauchy_256_batch.h) always runs on the GPU.
 */
#ifndef LONGHAIR_AMD_CAUCHY_256_DISPATCH_H
#define LONGHAIR_AMD_CAUCHY_256_DISPATCH_H

#ifdef __cplusplus
extern "C" {
#endif

#define CAUCHY_256_DISPATCH_GPU 0
#define CAUCHY_256_DISPATCH_AUTO 1
#define CAUCHY_256_DISPATCH_HOST 2

/* Sets the policy (and, if host_max_work >= 0, the AUTO work threshold in bytes).
 * Returns the previous policy, or -1 for an unknown policy.  Process-wide. */
int cauchy_256_set_dispatch(int policy, long long host_max_work);

/* The current policy. */
int cauchy_256_get_dispatch(void);

/* Instruction set the host engine uses on this CPU: "avx512bw", "avx2" or "scalar". */
const char *cauchy_256_host_isa(void);

#ifdef __cplusplus
}
#endif

#endif /* LONGHAIR_AMD_CAUCHY_256_DISPATCH_H */
