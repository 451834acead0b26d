/*
 * cauchy_256_batch.h -- batched, device-resident extension of the cauchy_256.h ABI.
 *
 * Not part of the reference API: the reference codes one stripe per call from host
 * memory (cauchy_256.h:78, :103).  These entry points code `stripes` independent
 * stripes that already live in HIP device memory, asynchronously on a caller stream,
 * with exactly the per-stripe results of cauchy_256_encode / cauchy_256_decode.
 *
 * Layout (all pointers are device pointers, strides in bytes):
 *   data block x of stripe s       d_data     + s * data_stride     + x * block_bytes
 *   recovery block r of stripe s   d_recovery + s * recovery_stride + r * block_bytes
 *   decode slot i of stripe s      d_blocks   + s * stripe_stride   + i * block_bytes
 *   row of decode slot i           d_rows[s * k + i]   (the Block.row of that slot)
 *
 * `stream` is a hipStream_t (NULL = the null stream).  Calls only enqueue work.
 * Return codes: 0 ok, -1 invalid parameters, -2 no device, -3 HIP error.
 * All work runs on the GPU; there is no CPU fallback.
 */
#ifndef LONGHAIR_AMD_CAUCHY_256_BATCH_H
#define LONGHAIR_AMD_CAUCHY_256_BATCH_H

#ifdef __cplusplus
extern "C" {
#endif

/* Encode every stripe: recovery = G * data (as cauchy_256_encode).  Parameter checks
 * follow the reference: recovery block 0 is written for every stripe, then -1 is
 * returned when m > 1 and (k + m > 256 or block_bytes % 8 != 0). */
int cauchy_256_encode_batch(int k, int m, int block_bytes, int stripes,
                            const void *d_data, long long data_stride,
                            void *d_recovery, long long recovery_stride, void *stream);

/* Decode every stripe in place (as cauchy_256_decode applied to the k slots of each
 * stripe in array order).  d_status, if not NULL, receives one signed byte per stripe:
 * 0 = ok, -1 = the stripe's rows are invalid (duplicate or >= k + m; m > 1 only: for
 * m == 1 every row is accepted, as by the reference's cauchy_decode_m1); such a stripe is
 * left untouched.  Returns -1 (nothing done) when m > 1 and k + m > 256 or
 * block_bytes % 8 != 0. */
int cauchy_256_decode_batch(int k, int m, int block_bytes, int stripes,
                            void *d_blocks, long long stripe_stride,
                            unsigned char *d_rows, signed char *d_status, void *stream);

/* Scattered blocks: the reference's per-block pointers (data_ptrs[], cauchy_256.h:78;
 * Block.data, cauchy_256.h:103) for a batch of stripes, e.g. packets left where a NIC put
 * them.  The pointer tables are device arrays of device pointers, one row per stripe:
 *   encode: d_data_ptrs[s * k + x] = data block x of stripe s,
 *           d_recovery_ptrs[s * m + r] = recovery block r of stripe s;
 *   decode: d_block_ptrs[s * k + i] = decode slot i of stripe s (Block.data), its row
 *           d_rows[s * k + i] (Block.row), rewritten as by cauchy_256_decode_batch.
 * Blocks may sit at any address (the register-network shapes read and write them in place;
 * others go through a workspace chunk).  Same results, return codes and asynchronous
 * semantics as cauchy_256_encode_batch / cauchy_256_decode_batch. */
int cauchy_256_encode_batch_ptrs(int k, int m, int block_bytes, int stripes,
                                 const void *const *d_data_ptrs, void *const *d_recovery_ptrs, void *stream);
int cauchy_256_decode_batch_ptrs(int k, int m, int block_bytes, int stripes,
                                 void *const *d_block_ptrs, unsigned char *d_rows, signed char *d_status,
                                 void *stream);
/* Optional: compile the pointer-table forms of the shape's specialised kernels now
 * (synchronous), so the first pointer-table calls already code the blocks in place instead
 * of gathering them while the modules compile in the background.  0 or -3. */
int cauchy_256_batch_prepare_ptrs(int k, int m, int block_bytes);

/* Host-memory batches: the same operations on stripes that live
 * in host memory, pipelined in chunks of `chunk_stripes` (0 = about 64 MiB for encode,
 * up to 256 MiB with at least 4 chunks for decode, the last chunks halving in size) over
 * three streams so the PCIe copies overlap the kernels (each chunk's host-to-device copy is
 * enqueued before the previous chunk's kernels).  Decode moves the rows and status once per
 * call.  Host buffers should be pinned (hipHostMalloc / hipHostRegister).
 * Synchronous: returns when the results are in host memory.  Decode writes back only the
 * slots decode can write (each stripe's recovery slots) and the rewritten rows: for k, m > 1
 * with pinned, 8-byte-aligned blocks a kernel stores exactly those blocks through the
 * buffer's device mapping; otherwise one copy per chunk covers their slot range. */
int cauchy_256_encode_host_batch(int k, int m, int block_bytes, int stripes,
                                 const void *h_data, long long data_stride,
                                 void *h_recovery, long long recovery_stride, int chunk_stripes);
int cauchy_256_decode_host_batch(int k, int m, int block_bytes, int stripes,
                                 void *h_blocks, long long stripe_stride,
                                 unsigned char *h_rows, signed char *h_status, int chunk_stripes);

/* Optional: compile the specialised kernels and reserve workspace for up to
 * `max_stripes` stripes of this shape ahead of time (e.g. before hipGraph capture or
 * a timed region).  Synchronous.  Returns 0 or an error code. */
int cauchy_256_batch_prepare(int k, int m, int block_bytes, int max_stripes);

/* As cauchy_256_batch_prepare, reserving the decode workspace of `stream` (workspaces are
 * per stream).  A batch call made while its stream is being captured into a graph never
 * allocates: if the stream's workspace (or the device's zero page or generator) would
 * have to grow, the call returns -3 without enqueuing anything.  Prepare the capture
 * stream first. */
int cauchy_256_batch_prepare_stream(int k, int m, int block_bytes, int max_stripes, void *stream);

/* Diagnostics: semicolon-separated names of the kernels the calling thread's last entry-point
 * call (drop-in or batch) enqueued, each once, in launch order (empty when it ran none,
 * e.g. on the host engine). */
const char *cauchy_256_last_launch(void);

/* Which kernel family serves this shape: 0 = generic coefficient-driven kernels,
 * 1 = run-time specialised (JIT) network, 2 (decode only) = specialised network with the
 * erasure plan computed inside the same kernel, 3 (encode only) = run-time specialised
 * 4-bit-windowed network for large m, 4 (decode only) = per-stripe planner + fused
 * windowed decode for large m (m <= 64).  `what` = 0 for encode, 1 for decode.
 * `what` = 2 (encode) / 5 (decode): 1 when the shape's register network stages its columns in
 * LDS by LDS-DMA, else 0.  `what` = 6 (encode) / 7 (decode): the dword lanes per sub-block of
 * the generic jump kernel on the current device (1: lh_apply_jump_kernel, 2:
 * lh_apply_jump2_kernel), 0 when the generic kernels below dword lanes serve the shape; -2
 * without a device.  `what` = 8: 1 when the (k, m) block-size family module (one module per
 * (k, m) for every 16-byte-multiple size up to 4 KiB with m <= 6) can serve the encode: batch
 * and drop-in encodes take it while no size-specialised module is loaded or cached.  `what` =
 * 9: the same for the decode's family (the fused decode: min(k, m) <= 4, k <= 64, at least
 * ceil(k / 8) 8-byte lanes per stripe). */
int cauchy_256_batch_path(int k, int m, int block_bytes, int what);

/* Compile the specialised kernels of a shape into the on-disk code-object cache
 * ($LONGHAIR_AMD_CACHE_DIR, else jit_cache/ beside the library).  Needs no GPU.  With
 * LONGHAIR_AMD_PRECOMPILE_FAMILY=1 also the (k, m) block-size family modules.
 * Returns 0 or -3. */
int cauchy_256_jit_precompile(int k, int m, int block_bytes);

/* Packet framing: the reference transmits every block with its
 * one-byte row (README.md:66-72).  A packet is [row][block_bytes bytes of the block],
 * block_bytes + 1 bytes long, at any alignment.
 *   frame:   the k data and m recovery blocks of stripe s become packets
 *            d_packets + s * packet_stride + i * (block_bytes + 1), rows i = 0 .. k + m - 1.
 *   unframe: the k packets received for stripe s (any order, any rows) at
 *            d_packets + s * packet_stride + i * (block_bytes + 1) become decode slot i of
 *            d_blocks and d_rows[s * k + i], ready for cauchy_256_decode_batch.
 * Asynchronous on `stream`; 0, -1 (invalid parameters), -2 or -3. */
int cauchy_256_frame_batch(int k, int m, int block_bytes, int stripes,
                           const void *d_data, long long data_stride,
                           const void *d_recovery, long long recovery_stride,
                           void *d_packets, long long packet_stride, void *stream);
int cauchy_256_unframe_batch(int k, int block_bytes, int stripes,
                             const void *d_packets, long long packet_stride,
                             void *d_blocks, long long stripe_stride, unsigned char *d_rows, void *stream);

/* Last error message of the calling thread (empty string if none). */
const char *cauchy_256_last_error(void);

#ifdef __cplusplus
}
#endif

#endif /* LONGHAIR_AMD_CAUCHY_256_BATCH_H */
