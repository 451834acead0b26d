// Micro-benchmark (not product code): the two ceilings the codec's rooflines are priced
// against on this MI355X.
//  1. HBM streaming read: 2.46 GB (the k29/m4 batch) read with dwordx4 lanes, U loads in
//     flight per lane per iteration, over several persistent grid sizes; plain and
//     non-temporal loads.  The best line is the measured read ceiling.
//  2. VALU issue rate of v_bitop3_b32 (the XOR3 every XOR network here is built from):
//     8 independent chains per lane, W waves per SIMD; reports wave-instructions per
//     second and cycles per wave-instruction per SIMD at the observed clock.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define CK(x) do{hipError_t e=(x); if(e!=hipSuccess){printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} }while(0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int U, bool NT>
__global__ void __launch_bounds__(256) stream_u(const u32x4 *__restrict__ in, u32x4 *__restrict__ out, size_t n) {
  const size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  u32x4 acc = {0, 0, 0, 0};
  size_t i = t;
  for (; i + (U - 1) * stride < n; i += U * stride) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = NT ? __builtin_nontemporal_load(in + i + u * stride) : in[i + u * stride];
#pragma unroll
    for (int u = 0; u < U; ++u) acc ^= v[u];
  }
  for (; i < n; i += stride) acc ^= in[i];
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) out[t] = acc;  // keeps the loads live
}

// ITER x 8 chains of v_bitop3_b32 (XOR3) per lane; operands rotate so nothing folds.
template <int ITER>
__global__ void __launch_bounds__(256) valu_bitop3(uint32_t *__restrict__ out, uint32_t seed) {
  uint32_t a[8], b = seed ^ threadIdx.x, c = seed * 2654435761u + blockIdx.x;
#pragma unroll
  for (int j = 0; j < 8; ++j) a[j] = seed + j * 977u + threadIdx.x;
  for (int it = 0; it < ITER; ++it) {
#pragma unroll
    for (int j = 0; j < 8; ++j) a[j] = __builtin_amdgcn_bitop3_b32(a[j], b, c, 0x96);
#pragma unroll
    for (int j = 0; j < 8; ++j) a[j] = __builtin_amdgcn_bitop3_b32(a[j], c, b ^ j, 0x96);
    asm volatile("" : "+v"(b), "+v"(c));
  }
  uint32_t r = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) r ^= a[j];
  if (r == 0xdeadbeefu) out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

int main() {
  const size_t in_bytes = (size_t)65536 * 29 * 1296;
  uint8_t *din, *dout;
  CK(hipMalloc(&din, in_bytes + 256));
  CK(hipMalloc(&dout, (size_t)64 << 20));
  CK(hipMemset(din, 0x5a, in_bytes + 256));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto timeit = [&](auto launch) {
    for (int i = 0; i < 3; ++i) launch();
    CK(hipDeviceSynchronize());
    const int reps = 10;
    CK(hipEventRecord(e0));
    for (int i = 0; i < reps; ++i) launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms / reps;
  };
  const size_t n16 = in_bytes / 16;
  printf("# HBM streaming read, %.3f GB per launch\n", in_bytes / 1e9);
#define STREAM(U, NT)                                                                                          \
  for (int grid : {1024, 2048, 4096, 8192}) {                                                               \
    const float ms = timeit([&] { stream_u<U, NT><<<grid, 256>>>((const u32x4 *)din, (u32x4 *)dout, n16); }); \
    printf("stream U=%d nt=%d grid=%-6d %8.3f ms %8.1f GB/s\n", U, (int)NT, grid, ms, in_bytes / (ms * 1e-3) / 1e9); \
  }
  STREAM(1, false) STREAM(4, false) STREAM(8, false) STREAM(4, true) STREAM(8, true)
  int cus = 0, clk_khz = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  CK(hipDeviceGetAttribute(&clk_khz, hipDeviceAttributeClockRate, 0));
  printf("# VALU v_bitop3_b32 issue rate (%d CUs, max clock %.0f MHz)\n", cus, clk_khz / 1e3);
  const int ITER = 4096;
  for (int wps : {1, 2, 4, 8}) {  // waves per SIMD: blocks of 4 waves, wps blocks per CU
    const int grid = cus * wps;
    const float ms = timeit([&] { valu_bitop3<ITER><<<grid, 256>>>((uint32_t *)dout, 7u); });
    const double winstr = (double)grid * 4 * ITER * 16;  // wave-level bitop3 instructions
    const double rate = winstr / (ms * 1e-3);
    const double cyc = (double)cus * 4 * (clk_khz * 1e3) / rate;  // SIMD cycles per wave-instr at max clock
    printf("valu waves/SIMD=%d %8.3f ms %10.1f G wave-instr/s  %.2f SIMD-cycles/instr at max clock\n", wps, ms,
           rate / 1e9, cyc);
  }
  CK(hipGetLastError());
  return 0;
}
