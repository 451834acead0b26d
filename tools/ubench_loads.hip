// Micro-benchmark: HBM read efficiency of the k=29/bytes=1296 stripe access
// pattern (8 sub-blocks of 162 B per block, 2-byte aligned) for several
// per-lane load widths, vs an aligned dwordx4 stream. Not product code.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#define CK(x) do{hipError_t e=(x); if(e!=hipSuccess){printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} }while(0)

typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__global__ void stream_read(const u32x4* __restrict__ in, u32x4* __restrict__ out, size_t n) {
  size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  size_t stride = (size_t)gridDim.x * blockDim.x;
  u32x4 acc = {0,0,0,0};
  for (size_t i = t; i < n; i += stride) acc ^= in[i];
  out[t] = acc;
}

// FETCH_SIZE calibration: the same aligned stream read with 4- and 8-byte lanes.
__global__ void stream_read4(const uint32_t* __restrict__ in, uint32_t* __restrict__ out, size_t n) {
  size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  size_t stride = (size_t)gridDim.x * blockDim.x;
  uint32_t acc = 0;
  for (size_t i = t; i < n; i += stride) acc ^= in[i];
  out[t] = acc;
}
__global__ void stream_read8(const u32x2* __restrict__ in, u32x2* __restrict__ out, size_t n) {
  size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  size_t stride = (size_t)gridDim.x * blockDim.x;
  u32x2 acc = {0, 0};
  for (size_t i = t; i < n; i += stride) acc ^= in[i];
  out[t] = acc;
}

template <int W> struct Word;
template <> struct Word<2> { typedef uint16_t T; };
template <> struct Word<4> { typedef uint32_t T; };
template <> struct Word<8> { typedef u32x2 T; };
template <> struct Word<16> { typedef u32x4 T; };

template <int W>
__global__ void stripe_pattern(const uint8_t* __restrict__ in, uint8_t* __restrict__ out,
                               int stripes, int k, int bytes) {
  typedef typename Word<W>::T T;
  const int sub = bytes / 8;
  const int nch = (sub + W - 1) / W;
  long g = blockIdx.x * (long)blockDim.x + threadIdx.x;
  int s = (int)(g / nch), c = (int)(g % nch);
  if (s >= stripes) return;
  const uint8_t* base = in + (size_t)s * k * bytes + c * W;
  T acc[8];
#pragma unroll
  for (int y = 0; y < 8; ++y) { T z; __builtin_memset(&z, 0, sizeof(T)); acc[y] = z; }
  for (int x = 0; x < k; ++x) {
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      T v; __builtin_memcpy(&v, base + x * bytes + b * sub, W);
      acc[b] ^= v;
    }
  }
  uint8_t* o = out + (size_t)s * bytes + c * W;
#pragma unroll
  for (int y = 0; y < 8; ++y) __builtin_memcpy(o + y * sub, &acc[y], W);
}

// Ideal traffic for k=29/m=4: every input byte read once with 16 B/lane coalesced
// loads, every output byte written once with 16 B/lane stores (outputs are XORs of
// disjoint column sets).  Lower bound on encode time for this read/write mix.
__global__ void ideal_stripe(const u32x4* __restrict__ in, u32x4* __restrict__ out, long nout, int k, int m, int cpb) {
  for (long o = blockIdx.x * (long)blockDim.x + threadIdx.x; o < nout; o += (long)gridDim.x * blockDim.x) {
    long s = o / (m * cpb); int rem = (int)(o % (m * cpb)); int r = rem / cpb, c = rem % cpb;
    u32x4 acc = {0,0,0,0};
    const u32x4* src = in + s * (long)k * cpb + c;
    for (int x = r; x < k; x += m) acc ^= __builtin_nontemporal_load(src + (long)x * cpb);
    __builtin_nontemporal_store(acc, out + o);
  }
}

int main() {
  const int k = 29, bytes = 1296, stripes = 65536;
  size_t in_bytes = (size_t)stripes * k * bytes, out_bytes = (size_t)stripes * bytes;
  uint8_t *din, *dout;
  size_t out_alloc = out_bytes + 256;
  for (int grid : {2048, 8192, 32768}) { size_t need = (size_t)grid * 256 * 16; if (need > out_alloc) out_alloc = need; }
  CK(hipMalloc(&din, in_bytes + 256)); CK(hipMalloc(&dout, out_alloc));
  printf("in %zu out_alloc %zu\n", in_bytes, out_alloc);
  CK(hipMemset(din, 0x5a, in_bytes + 256));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  auto timeit = [&](const char* name, double gb, auto launch) {
    for (int i = 0; i < 3; ++i) launch();
    CK(hipDeviceSynchronize());
    const int reps = 10;
    CK(hipEventRecord(e0));
    for (int i = 0; i < reps; ++i) launch();
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    printf("%-28s %8.3f ms  %8.1f GB/s (input)\n", name, ms / reps, gb / (ms / reps * 1e-3) / 1e9);
  };
  size_t n16 = in_bytes / 16;
  for (int grid : {2048, 8192, 32768}) {
    char nm[64]; snprintf(nm, 64, "stream dwordx4 grid=%d", grid);
    timeit(nm, (double)in_bytes, [&] { stream_read<<<grid, 256>>>((const u32x4*)din, (u32x4*)dout, n16); });
  }
  timeit("stream dword grid=2048", (double)in_bytes, [&] { stream_read4<<<2048, 256>>>((const uint32_t*)din, (uint32_t*)dout, in_bytes / 4); });
  timeit("stream dwordx2 grid=2048", (double)in_bytes, [&] { stream_read8<<<2048, 256>>>((const u32x2*)din, (u32x2*)dout, in_bytes / 8); });
#define PAT(W) { int nch = (bytes/8 + W - 1)/W; long thr = (long)stripes * nch; int grid = (int)((thr + 255)/256); \
    timeit("pattern W=" #W, (double)in_bytes, [&]{ stripe_pattern<W><<<grid,256>>>(din, dout, stripes, k, bytes); }); }
  PAT(2) PAT(4) PAT(8) PAT(16)
  { const int m = 4, cpb = bytes / 16; long nout = (long)stripes * m * cpb;
    uint8_t* dout2; CK(hipMalloc(&dout2, nout * 16));
    for (int grid : {2048, 4096, 8192, 16384}) { char nm[64]; snprintf(nm, 64, "ideal 29r/4w grid=%d", grid);
      timeit(nm, (double)in_bytes, [&] { ideal_stripe<<<grid, 256>>>((const u32x4*)din, (u32x4*)dout2, nout, k, m, cpb); }); }
    printf("  (ideal traffic per launch: %.3f GB read + %.3f GB written)\n", in_bytes / 1e9, nout * 16 / 1e9); }
  CK(hipGetLastError());
  return 0;
}
