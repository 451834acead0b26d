// Micro-benchmark (not product code): a calibrated HBM floor for the k29/m4/1296-B encode
// and decode (VERDICT r3 "Next round" item 1), in three steps:
//   copy  : the MI355X_MICROARCH.md float4 copy (6.29 TB/s there) -- reproduces the guide's
//           number on this box first, so the floors below are known to be tuned;
//   read  : a read-only stream, grid swept past 8192 and one-shot (one chunk set per thread);
//   mix   : the encode's bytes as a flat 29:4 read:write stream with the stores interleaved
//           (each wave reads 29 KiB and writes 4 KiB, then moves on), default / nt policies;
//   enc   : the encode's access pattern on the real [stripe][29][1296] layout with 8-byte
//           lanes (the kernel today) and 16-byte lanes (11 lanes per stripe, 5 stripes per
//           wave), light (8 accumulators) and heavy (m x 8 accumulators, the real network's
//           register footprint) compute;
//   lds   : the encode's columns fetched by coalesced LDS-DMA and read back per lane
//           (unaligned ds_read_b64, or dword reads + v_alignbyte).
// Usage: ubench_floor [group ...]   (default: all groups)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
constexpr int K = 29, M = 4, BYTES = 1296, SUB = 162;
constexpr long long STRIPES = 65536;
constexpr long long IN_BYTES = STRIPES * K * BYTES;   // 2.463 GB
constexpr long long OUT_BYTES = STRIPES * M * BYTES;  // 0.340 GB

template <bool NT>
__device__ __forceinline__ u32x4 ld4(const u32x4 *p) { return NT ? __builtin_nontemporal_load(p) : *p; }
template <bool NT>
__device__ __forceinline__ void st4(u32x4 *p, u32x4 v) {
  if (NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}

// ---------------------------------------------------------------- copy
// Grid-stride float4 copy, U independent chunks per thread per iteration.
template <int U, bool NTL, bool NTS>
__global__ void __launch_bounds__(256) copy_gs(const u32x4 *__restrict__ in, u32x4 *__restrict__ out, long long n) {
  const long long st = (long long)gridDim.x * blockDim.x;
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + (U - 1) * st < n; i += U * st) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = ld4<NTL>(in + i + u * st);
#pragma unroll
    for (int u = 0; u < U; ++u) st4<NTS>(out + i + u * st, v[u]);
  }
  for (; i < n; i += st) st4<NTS>(out + i, ld4<NTL>(in + i));
}
// One-shot: block b copies chunks [b*256*U, (b+1)*256*U), lane-contiguous per u.
template <int U, bool NTL, bool NTS>
__global__ void __launch_bounds__(256) copy_os(const u32x4 *__restrict__ in, u32x4 *__restrict__ out, long long n) {
  const long long base = (long long)blockIdx.x * 256 * U + threadIdx.x;
  u32x4 v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) v[u] = base + u * 256 < n ? ld4<NTL>(in + base + u * 256) : u32x4{0, 0, 0, 0};
#pragma unroll
  for (int u = 0; u < U; ++u)
    if (base + u * 256 < n) st4<NTS>(out + base + u * 256, v[u]);
}

// ---------------------------------------------------------------- read
template <int U, bool NT>
__global__ void __launch_bounds__(256) read_gs(const u32x4 *__restrict__ in, u32x4 *__restrict__ sink, long long n) {
  const long long st = (long long)gridDim.x * blockDim.x;
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  u32x4 acc = {0, 0, 0, 0};
  for (; i + (U - 1) * st < n; i += U * st) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = ld4<NT>(in + i + u * st);
#pragma unroll
    for (int u = 0; u < U; ++u) acc ^= v[u];
  }
  for (; i < n; i += st) acc ^= in[i];
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) sink[threadIdx.x] = acc;
}
template <int U, bool NT>
__global__ void __launch_bounds__(256) read_os(const u32x4 *__restrict__ in, u32x4 *__restrict__ sink, long long n) {
  const long long base = (long long)blockIdx.x * 256 * U + threadIdx.x;
  u32x4 acc = {0, 0, 0, 0};
#pragma unroll
  for (int u = 0; u < U; ++u)
    if (base + u * 256 < n) acc ^= ld4<NT>(in + base + u * 256);
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) sink[threadIdx.x] = acc;
}

// ---------------------------------------------------------------- mix (29:4 interleaved)
// Unit u: input chunks [u*29*64, (u+1)*29*64) (29 KiB), output [u*4*64, (u+1)*4*64) (4 KiB);
// one wave per unit, G loads issued before they are combined.  PERSIST: grid-stride over
// units with the launched waves, else one unit per wave.
template <int G, bool NTL, bool NTS>
__device__ __forceinline__ void mix_unit(const u32x4 *__restrict__ in, u32x4 *__restrict__ out, long long u, int lane) {
  const u32x4 *src = in + u * (K * 64) + lane;
  u32x4 acc[M];
#pragma unroll
  for (int r = 0; r < M; ++r) acc[r] = u32x4{0, 0, 0, 0};
#pragma unroll
  for (int x0 = 0; x0 < K; x0 += G) {
    u32x4 v[G];
#pragma unroll
    for (int g = 0; g < G; ++g)
      if (x0 + g < K) v[g] = ld4<NTL>(src + (x0 + g) * 64);
#pragma unroll
    for (int g = 0; g < G; ++g)
      if (x0 + g < K) acc[(x0 + g) % M] ^= v[g];
  }
  u32x4 *dst = out + u * (M * 64) + lane;
#pragma unroll
  for (int r = 0; r < M; ++r) st4<NTS>(dst + r * 64, acc[r]);
}
template <int G, bool NTL, bool NTS, bool PERSIST>
__global__ void __launch_bounds__(256) mix(const u32x4 *__restrict__ in, u32x4 *__restrict__ out, long long units) {
  const int lane = threadIdx.x & 63;
  const long long w0 = ((long long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (PERSIST) {
    const long long ws = (long long)gridDim.x * (blockDim.x >> 6);
    for (long long u = w0; u < units; u += ws) mix_unit<G, NTL, NTS>(in, out, u, lane);
  } else if (w0 < units) {
    mix_unit<G, NTL, NTS>(in, out, w0, lane);
  }
}

// ---------------------------------------------------------------- enc (stripe layout)
// W-byte lanes: nch = ceil(162 / W) lanes per stripe, spw = 64 / nch stripes per wave; the
// last chunk of a sub-block is shifted back to end at the sub-block's end.  Column x at
// soffset x * 1296, sub-block b in the voffset.  HEAVY: M x 8 accumulators (the real
// network's registers), acc[r][y] ^= d[(y + r) & 7]; else 8 accumulators.
template <int W>
struct wt;
template <>
struct wt<8> { typedef u32x2 T; };
template <>
struct wt<16> { typedef u32x4 T; };

template <int W, int AUX>
__device__ __forceinline__ typename wt<W>::T bload(__amdgpu_buffer_rsrc_t rs, int off, int soff) {
  if constexpr (W == 8) return __builtin_amdgcn_raw_buffer_load_b64(rs, off, soff, AUX);
  else return __builtin_amdgcn_raw_buffer_load_b128(rs, off, soff, AUX);
}
template <int W>
__device__ __forceinline__ void gstore_nt(uint8_t *p, typename wt<W>::T v) {
  __builtin_nontemporal_store(v, (typename wt<W>::T *)p);
}

template <int W, int PF, bool HEAVY, int LAUX, int LB>
__global__ void __launch_bounds__(256, LB) enc_pat(const uint8_t *__restrict__ in, uint8_t *__restrict__ out, int stripes) {
  typedef typename wt<W>::T T;
  constexpr int NCH = (SUB + W - 1) / W, SPW = 64 / NCH;
  constexpr int NA = HEAVY ? M : 1;
  const long long wave = ((long long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63, sl = lane / NCH, c = lane - sl * NCH;
  const long long s0 = (long long)__builtin_amdgcn_readfirstlane((int)wave) * SPW;
  const long long s = s0 + sl;
  if (sl >= SPW || s >= stripes) return;
  const int p = c == NCH - 1 ? SUB - W : c * W;
  const long long nst = stripes - s0 < SPW ? stripes - s0 : SPW;
  const long long stride = (long long)K * BYTES;
  __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *)(in + s0 * stride), 0, (int)(nst * stride), 0x00020000);
  const int lbase = (int)(sl * stride) + p;
  T acc[NA][8];
#pragma unroll
  for (int r = 0; r < NA; ++r)
#pragma unroll
    for (int y = 0; y < 8; ++y) acc[r][y] = T{};
  T ring[PF][8];
#pragma unroll
  for (int q = 0; q < PF; ++q)
#pragma unroll
    for (int b = 0; b < 8; ++b) ring[q][b] = bload<W, LAUX>(rs, lbase + b * SUB, q * BYTES);
#pragma unroll
  for (int x = 0; x < K; ++x) {
    T nxt[8];
    if (x + PF < K)
#pragma unroll
      for (int b = 0; b < 8; ++b) nxt[b] = bload<W, LAUX>(rs, lbase + b * SUB, (x + PF) * BYTES);
#pragma unroll
    for (int r = 0; r < NA; ++r)
#pragma unroll
      for (int y = 0; y < 8; ++y) acc[r][y] ^= ring[x % PF][(y + r + x) & 7];
#pragma unroll
    for (int r = 0; r < NA; ++r)
#pragma unroll
      for (int y = 0; y < 8; ++y) asm volatile("" : "+v"(acc[r][y]));
    if (x + PF < K)
#pragma unroll
      for (int b = 0; b < 8; ++b) ring[x % PF][b] = nxt[b];
  }
  uint8_t *o = out + s * (long long)(M * BYTES) + p;
#pragma unroll
  for (int r = 0; r < M; ++r)
#pragma unroll
    for (int y = 0; y < 8; ++y) gstore_nt<W>(o + r * BYTES + y * SUB, acc[HEAVY ? r : 0][y] ^ T{(uint32_t)r});
}

// ---------------------------------------------------------------- enc, aligned layout
// 8-byte lanes, 21 per stripe, 3 stripes per wave, lane c owns sub-block bytes [8c, 8c + 8).
// A fake layout with 168-byte sub-blocks: every load and store is 8-byte aligned, so the time
// against enc_pat is the pure cost of the real layout's 2-byte alignment.  (A DPP-realign
// variant of the real layout was removed in round 5: it wrote wrong bytes.)
template <int PF>
__global__ void __launch_bounds__(256) enc_al(const uint8_t *__restrict__ in, uint8_t *__restrict__ out, int stripes) {
  constexpr int NCH = 21, SPW = 3, SB = 168, BY = 8 * SB;
  const long long wave = ((long long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63, sl = min(lane / NCH, SPW - 1), c = lane - (lane / NCH) * NCH;
  const long long s0 = (long long)__builtin_amdgcn_readfirstlane((int)wave) * SPW;
  if (s0 >= stripes) return;
  const long long nst = stripes - s0 < SPW ? stripes - s0 : SPW;
  const long long stride = (long long)K * BY;
  __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *)(in + s0 * stride), 0, (int)(nst * stride), 0x00020000);
  const int lbase = (int)(sl * stride) + 8 * c;
  u32x2 acc[M][8];
#pragma unroll
  for (int r = 0; r < M; ++r)
#pragma unroll
    for (int y = 0; y < 8; ++y) acc[r][y] = u32x2{0, 0};
  u32x2 ring[PF][8];
  auto col = [&](int x, u32x2 (&d)[8]) {
#pragma unroll
    for (int b = 0; b < 8; ++b) d[b] = __builtin_amdgcn_raw_buffer_load_b64(rs, lbase + b * SB, x * BY, 2);
  };
#pragma unroll
  for (int q = 0; q < PF; ++q) col(q, ring[q]);
#pragma unroll
  for (int x = 0; x < K; ++x) {
    u32x2 nxt[8];
    if (x + PF < K) col(x + PF, nxt);
#pragma unroll
    for (int r = 0; r < M; ++r)
#pragma unroll
      for (int y = 0; y < 8; ++y) acc[r][y] ^= ring[x % PF][(y + r + x) & 7];
#pragma unroll
    for (int r = 0; r < M; ++r)
#pragma unroll
      for (int y = 0; y < 8; ++y) asm volatile("" : "+v"(acc[r][y]));
    if (x + PF < K)
#pragma unroll
      for (int b = 0; b < 8; ++b) ring[x % PF][b] = nxt[b];
  }
  if (lane >= SPW * NCH || s0 + sl >= stripes) return;
  uint8_t *o = out + (s0 + sl) * (long long)(M * 8 * SB);
#pragma unroll
  for (int r = 0; r < M; ++r)
#pragma unroll
    for (int y = 0; y < 8; ++y)
      __builtin_nontemporal_store(acc[r][y] ^ u32x2{(uint32_t)r, 0}, (u32x2 *)(o + r * 8 * SB + y * SB + 8 * c));
}

// ---------------------------------------------------------------- lds (DMA-staged columns)
// Per wave: 3 stripes, 21 lanes of 8 B per stripe (the kernel's mapping).  Column x of the
// wave's 3 stripes = 3 x 1296 B = 243 aligned 16-B chunks: 4 global_load_lds_dwordx4 per
// column into a per-wave ring of D slots (4 KiB each).  ALIGNED: each lane reads 3 aligned
// dwords per sub-block and realigns with v_alignbyte, else one 2-byte-aligned ds_read_b64.
template <int D, bool ALIGNED>
__global__ void __launch_bounds__(256) lds_pat(const uint8_t *__restrict__ in, uint8_t *__restrict__ out, int stripes) {
  constexpr int NCH = 21, SPW = 3;
  __shared__ __attribute__((aligned(16))) uint8_t ring[4][D][4096];
  const long long wave = ((long long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int w = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63, sl = lane / NCH, c = lane - sl * NCH;
  const long long s0 = (long long)__builtin_amdgcn_readfirstlane((int)wave) * SPW;
  if (s0 >= stripes) return;
  const int ns = (int)min((long long)SPW, stripes - s0);
  const int p = c == NCH - 1 ? SUB - 8 : c * 8;
  const long long stride = (long long)K * BYTES;
  const uint8_t *src[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int j = min(i * 64 + lane, SPW * 81 - 1);
    src[i] = in + (s0 + min(j / 81, ns - 1)) * stride + (j % 81) * 16;
  }
  auto issue = [&](int x, int slot) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
      __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void *)(src[i] + x * BYTES),
                                       (__attribute__((address_space(3))) void *)&ring[w][slot][i * 1024], 16, 0, 2);
  };
#pragma unroll
  for (int q = 0; q < D; ++q) issue(q, q);
  u32x2 acc[8];
#pragma unroll
  for (int b = 0; b < 8; ++b) acc[b] = u32x2{0, 0};
  const int lo = min(sl, SPW - 1) * BYTES + p;
#pragma unroll
  for (int x = 0; x < K; ++x) {
    const int left = min(D - 1, K - 1 - x);  // column groups issued after x (4 DMA each)
    // vmcnt(4 * left): bits [3:0] and [15:14]; expcnt and lgkmcnt left at their maxima.
    if (left >= 5) __builtin_amdgcn_s_waitcnt((20 & 15) | ((20 >> 4) << 14) | (7 << 4) | (15 << 8));
    else if (left == 4) __builtin_amdgcn_s_waitcnt((16 & 15) | ((16 >> 4) << 14) | (7 << 4) | (15 << 8));
    else if (left == 3) __builtin_amdgcn_s_waitcnt(12 | (7 << 4) | (15 << 8));
    else if (left == 2) __builtin_amdgcn_s_waitcnt(8 | (7 << 4) | (15 << 8));
    else if (left == 1) __builtin_amdgcn_s_waitcnt(4 | (7 << 4) | (15 << 8));
    else __builtin_amdgcn_s_waitcnt(0 | (7 << 4) | (15 << 8));
    asm volatile("" ::: "memory");  // no LDS read moves above the wait
    const uint8_t *t = &ring[w][x % D][0];
    u32x2 v[8];
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      const int o = lo + b * SUB;
      if (ALIGNED) {
        const uint32_t *q = (const uint32_t *)(t + (o & ~3));
        const uint32_t w0 = q[0], w1 = q[1], w2 = q[2];
        v[b] = u32x2{__builtin_amdgcn_alignbyte(w1, w0, o & 3), __builtin_amdgcn_alignbyte(w2, w1, o & 3)};
      } else {
        v[b] = *(const u32x2 *)(t + o);
      }
    }
#pragma unroll
    for (int b = 0; b < 8; ++b) acc[b] ^= v[b];
#pragma unroll
    for (int b = 0; b < 8; ++b) asm volatile("" : "+v"(acc[b]));
    if (x + D < K) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      issue(x + D, x % D);
    }
  }
  if (sl >= SPW || s0 + sl >= stripes) return;
  uint8_t *o = out + (s0 + sl) * (long long)(M * BYTES) + p;
#pragma unroll
  for (int r = 0; r < M; ++r)
#pragma unroll
    for (int b = 0; b < 8; ++b) __builtin_nontemporal_store(acc[b] ^ u32x2{(uint32_t)r, 0}, (u32x2 *)(o + r * BYTES + b * SUB));
}

// ---------------------------------------------------------------- driver
static hipEvent_t e0, e1;
template <class F>
static float timeit(F launch) {
  for (int i = 0; i < 3; ++i) launch();
  CK(hipGetLastError());
  CK(hipDeviceSynchronize());
  float best = 1e9f;
  for (int rep = 0; rep < 3; ++rep) {
    CK(hipEventRecord(e0));
    for (int i = 0; i < 10; ++i) launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    best = std::min(best, ms / 10);
  }
  return best;
}

static bool want(int argc, char **argv, const char *g) {
  if (argc < 2) return true;
  for (int i = 1; i < argc; ++i)
    if (!strcmp(argv[i], g)) return true;
  return false;
}

int main(int argc, char **argv) {
  uint8_t *din, *dout;
  CK(hipMalloc(&din, IN_BYTES + 4096));
  CK(hipMalloc(&dout, IN_BYTES + 4096));  // copy destination is as large as the source
  CK(hipMemset(din, 0x5a, IN_BYTES + 4096));
  CK(hipMemset(dout, 0, IN_BYTES + 4096));
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const u32x4 *in4 = (const u32x4 *)din;
  u32x4 *out4 = (u32x4 *)dout;
  printf("# ubench_floor: %d CUs; input %.3f GB, output %.3f GB (k29/m4/1296 x 65536)\n", cus, IN_BYTES / 1e9, OUT_BYTES / 1e9);

  if (want(argc, argv, "copy")) {
    // 1.2315 GB read + 1.2315 GB written (half the encode input, so both fit one buffer each).
    const long long n = IN_BYTES / 2 / 16, bytes = n * 16 * 2;
    printf("# copy: float4, %.3f GB moved per launch (read + write); GB/s = moved bytes / time\n", bytes / 1e9);
#define COPY_GS(U, NL, NS)                                                                                       \
    for (int g : {2048, 4096, 8192, 16384, 32768}) {                                                           \
      const float ms = timeit([&] { copy_gs<U, NL, NS><<<g, 256>>>(in4, out4, n); });                          \
      printf("copy gs U=%d ntl=%d nts=%d grid=%-6d %8.4f ms %8.1f GB/s\n", U, NL, NS, g, ms, bytes / (ms * 1e-3) / 1e9); \
    }
#define COPY_OS(U, NL, NS)                                                                                       \
    {                                                                                                          \
      const int g = (int)((n + 256LL * U - 1) / (256LL * U));                                                  \
      const float ms = timeit([&] { copy_os<U, NL, NS><<<g, 256>>>(in4, out4, n); });                          \
      printf("copy os U=%d ntl=%d nts=%d grid=%-6d %8.4f ms %8.1f GB/s\n", U, NL, NS, g, ms, bytes / (ms * 1e-3) / 1e9); \
    }
    COPY_GS(1, false, false) COPY_GS(2, false, false) COPY_GS(4, false, false)
    COPY_GS(1, true, true) COPY_GS(2, true, true) COPY_GS(4, true, true) COPY_GS(2, true, false) COPY_GS(2, false, true)
    COPY_OS(1, false, false) COPY_OS(2, false, false) COPY_OS(4, false, false) COPY_OS(8, false, false)
    COPY_OS(1, true, true) COPY_OS(2, true, true) COPY_OS(4, true, true) COPY_OS(8, true, true)
  }
  if (want(argc, argv, "read")) {
    const long long n = IN_BYTES / 16;
    printf("# read: %.3f GB per launch\n", IN_BYTES / 1e9);
#define READ_GS(U, NT)                                                                                             \
    for (int g : {4096, 8192, 16384, 32768, 65536}) {                                                            \
      const float ms = timeit([&] { read_gs<U, NT><<<g, 256>>>(in4, out4, n); });                                 \
      printf("read gs U=%d nt=%d grid=%-6d %8.4f ms %8.1f GB/s\n", U, NT, g, ms, IN_BYTES / (ms * 1e-3) / 1e9);   \
    }
#define READ_OS(U, NT)                                                                                             \
    {                                                                                                            \
      const int g = (int)((n + 256LL * U - 1) / (256LL * U));                                                    \
      const float ms = timeit([&] { read_os<U, NT><<<g, 256>>>(in4, out4, n); });                                 \
      printf("read os U=%d nt=%d grid=%-6d %8.4f ms %8.1f GB/s\n", U, NT, g, ms, IN_BYTES / (ms * 1e-3) / 1e9);   \
    }
    READ_GS(4, false) READ_GS(8, false) READ_GS(4, true) READ_GS(8, true)
    READ_OS(4, false) READ_OS(8, false) READ_OS(16, false) READ_OS(4, true) READ_OS(8, true) READ_OS(16, true)
  }
  if (want(argc, argv, "mix")) {
    const long long units = IN_BYTES / (K * 1024);  // 82944 units of 29 KiB in + 4 KiB out
    printf("# mix: %lld units x (29 KiB read + 4 KiB written) = %.3f + %.3f GB; GB/s of input (and of all traffic)\n",
           units, IN_BYTES / 1e9, OUT_BYTES / 1e9);
    auto rep = [&](const char *name, float ms) {
      printf("%-34s %8.4f ms %8.1f GB/s input %8.1f GB/s total\n", name, ms, IN_BYTES / (ms * 1e-3) / 1e9,
             (IN_BYTES + OUT_BYTES) / (ms * 1e-3) / 1e9);
    };
    const int g1 = (int)((units + 3) / 4);
#define MIX1(G, NL, NS)                                                                                    \
    { char nm[64]; snprintf(nm, 64, "mix one-shot G=%d ntl=%d nts=%d", G, NL, NS);                          \
      rep(nm, timeit([&] { mix<G, NL, NS, false><<<g1, 256>>>(in4, out4, units); })); }
#define MIXP(G, NL, NS, GR)                                                                                \
    { char nm[64]; snprintf(nm, 64, "mix persist g=%d G=%d ntl=%d nts=%d", GR, G, NL, NS);                  \
      rep(nm, timeit([&] { mix<G, NL, NS, true><<<GR, 256>>>(in4, out4, units); })); }
    MIX1(4, false, false) MIX1(8, false, false) MIX1(16, false, false) MIX1(29, false, false)
    MIX1(4, true, true) MIX1(8, true, true) MIX1(16, true, true) MIX1(29, true, true)
    MIX1(8, true, false) MIX1(8, false, true) MIX1(16, true, false) MIX1(16, false, true)
    MIXP(8, true, true, 1024) MIXP(8, true, true, 2048) MIXP(8, true, true, 4096)
    MIXP(16, true, true, 1024) MIXP(16, true, true, 2048) MIXP(16, false, false, 2048)
  }
  if (want(argc, argv, "enc")) {
    printf("# enc: access pattern on [65536][29][1296] -> [65536][4][1296]; GB/s of input\n");
    auto rep = [&](const char *name, float ms) {
      printf("%-34s %8.4f ms %8.1f GB/s input %8.1f GB/s total\n", name, ms, IN_BYTES / (ms * 1e-3) / 1e9,
             (IN_BYTES + OUT_BYTES) / (ms * 1e-3) / 1e9);
    };
#define ENC(W, PF, HEAVY, LAUX, LB)                                                                                    \
    {                                                                                                                \
      constexpr int nch = (SUB + W - 1) / W, spw = 64 / nch;                                                         \
      const int g = (int)((STRIPES + spw - 1) / spw + 3) / 4;                                                        \
      char nm[64]; snprintf(nm, 64, "enc W=%d PF=%d heavy=%d aux=%d lb=%d", W, PF, HEAVY, LAUX, LB);                  \
      rep(nm, timeit([&] { enc_pat<W, PF, HEAVY, LAUX, LB><<<g, 256>>>(din, dout, (int)STRIPES); }));                 \
    }
    ENC(8, 3, false, 2, 1) ENC(8, 3, true, 2, 1) ENC(8, 2, true, 2, 1) ENC(8, 3, false, 0, 1)
    ENC(16, 1, false, 2, 1) ENC(16, 2, false, 2, 1) ENC(16, 3, false, 2, 1) ENC(16, 2, false, 0, 1)
    ENC(16, 1, true, 2, 1) ENC(16, 2, true, 2, 1) ENC(16, 1, true, 2, 2) ENC(16, 1, true, 0, 2) ENC(16, 1, true, 2, 3)
    // the fake layout's stripes are larger (29 x 1344 B): as many as fit the same input bytes, time scaled to 65536
    {
      const int st1 = (int)(IN_BYTES / (K * 8 * 168));  // stripes of the fake layout in the same bytes
      const int g1 = (int)((st1 + 2) / 3 + 3) / 4;
      const float ms = timeit([&] { enc_al<3><<<g1, 256>>>(din, dout, st1); });
      printf("%-34s %8.4f ms %8.1f GB/s input (fake 168-B sub-blocks, %d stripes, scaled to 65536: %.4f ms)\n",
             "enc aligned-layout PF=3", ms, IN_BYTES / (ms * 1e-3) / 1e9, st1, ms * 65536.0 / st1);
    }
  }
  if (want(argc, argv, "lds")) {
    printf("# lds: columns by LDS-DMA (4 x dwordx4 per column per wave), per-wave ring of D slots\n");
    const int g = (int)((STRIPES + 2) / 3 + 3) / 4;
    auto rep = [&](const char *name, float ms) {
      printf("%-34s %8.4f ms %8.1f GB/s input %8.1f GB/s total\n", name, ms, IN_BYTES / (ms * 1e-3) / 1e9,
             (IN_BYTES + OUT_BYTES) / (ms * 1e-3) / 1e9);
    };
    rep("lds D=3 unaligned b64", timeit([&] { lds_pat<3, false><<<g, 256>>>(din, dout, (int)STRIPES); }));
    rep("lds D=3 aligned+alignbyte", timeit([&] { lds_pat<3, true><<<g, 256>>>(din, dout, (int)STRIPES); }));
    rep("lds D=4 aligned+alignbyte", timeit([&] { lds_pat<4, true><<<g, 256>>>(din, dout, (int)STRIPES); }));
    rep("lds D=6 aligned+alignbyte", timeit([&] { lds_pat<6, true><<<g, 256>>>(din, dout, (int)STRIPES); }));
  }
  CK(hipGetLastError());
  CK(hipDeviceSynchronize());
  return 0;
}
