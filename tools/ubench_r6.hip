// Micro-benchmark (not product code), round 6: how the k29/m4/1296-B encode's HBM rate depends
// on the geometry of its LDS-DMA column stream.
//
// Round 6 found that the hipcc builtin for global_load_lds makes the compiler wait vmcnt(0)
// before every LDS read of the ring (it cannot tell the slot being read from the slots being
// filled), so the product's 4-slot ring ran one column per wave at a time -- and issuing the
// DMAs from asm (the ring really 3 columns deep) made the encode SLOWER (0.533 against 0.501 ms).
// This bench separates the factors, with the DMAs issued from asm so the depth is what it says:
//   SPW    stripes per wave (21 lanes of 8 bytes per stripe, as the product)
//   CPS    columns per DMA step (a stripe's step is CPS x 1296 contiguous bytes)
//   AHEAD  steps in flight beyond the one being combined (0: issue the next step, then wait
//          for it -- the product's drained pattern)
//   WG     resident 256-thread workgroups per CU (LDS padding caps it)
// Combine: acc[r][y] ^= d[(y + r + x) & 7] ^ d[(y + r + x + 3) & 7] (about the product's VALU
// per column); stores: the product's per-lane 8-byte stores into the bench layout.
// Usage: ubench_r6 [group ...]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
constexpr int K = 29, M = 4, BYTES = 1296, SUB = 162, NCH = 21;
constexpr long long STRIPES = 65536;
constexpr long long STRIDE = (long long)K * BYTES;    // 37584
constexpr long long IN_BYTES = STRIPES * STRIDE;      // 2.463 GB
constexpr long long OUT_BYTES = STRIPES * M * BYTES;  // 0.340 GB
constexpr long long OUT_OFF = (long long)(K - M) * BYTES;  // bench layout: recovery in slots 25..28

__device__ __forceinline__ long long xcd_block() {
  const unsigned b = blockIdx.x, per = gridDim.x / 8;
  return b < per * 8 ? (long long)(b % 8) * per + b / 8 : (long long)b;
}
template <int S>
__device__ __forceinline__ u32x2 funnel(u32x2 a, u32x2 b) {
  if constexpr (S == 0) return a;
  else if constexpr (S == 4) return u32x2{a.y, b.x};
  else if constexpr (S < 4) return u32x2{__builtin_amdgcn_alignbyte(a.y, a.x, S), __builtin_amdgcn_alignbyte(b.x, a.y, S)};
  else return u32x2{__builtin_amdgcn_alignbyte(b.x, a.y, S - 4), __builtin_amdgcn_alignbyte(b.y, b.x, S - 4)};
}
template <int B>
__device__ __forceinline__ u32x2 slot_word(const uint8_t *col, int lo, int lo8) {
  constexpr int S = (2 * B) & 7;
  const u32x2 a = *(const u32x2 *)(col + lo + B * SUB - S);
  if constexpr (S == 0) return a;
  else return funnel<S>(a, *(const u32x2 *)(col + lo8 + B * SUB - S));
}
__device__ __forceinline__ uint32_t dpp_row_shr1(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, false);
}
template <int NT>
__device__ __forceinline__ void dma16(const void *src, const void *lds) {
  const unsigned m = __builtin_amdgcn_readfirstlane((unsigned)(unsigned long long)lds);
  if constexpr (NT)
    asm volatile("global_load_lds_dwordx4 %0, off nt" ::"v"(src), "{m0}"(m) : "memory");
  else
    asm volatile("global_load_lds_dwordx4 %0, off" ::"v"(src), "{m0}"(m) : "memory");
}
template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N <= 63, "vmcnt");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

template <int SPW, int CPS, int AHEAD, int NT>
struct Geo {
  static constexpr int D = AHEAD + 1;                       // ring slots
  static constexpr int CH = CPS * BYTES / 16;               // chunks per stripe per step
  static constexpr int NQ = (SPW * CH + 63) / 64;           // DMA instructions per step
  static constexpr int SLOT = NQ * 1024;
  static constexpr int NS = (K + CPS - 1) / CPS;            // steps
  static constexpr int RING = D * SLOT + 16;
};

template <int SPW, int CPS, int AHEAD, int NT, int X>
__device__ __forceinline__ void column(u32x2 (&acc)[M][8], const uint8_t *col, int lo, int lo8) {
  u32x2 d[8];
  d[0] = slot_word<0>(col, lo, lo8); d[1] = slot_word<1>(col, lo, lo8);
  d[2] = slot_word<2>(col, lo, lo8); d[3] = slot_word<3>(col, lo, lo8);
  d[4] = slot_word<4>(col, lo, lo8); d[5] = slot_word<5>(col, lo, lo8);
  d[6] = slot_word<6>(col, lo, lo8); d[7] = slot_word<7>(col, lo, lo8);
#pragma unroll
  for (int r = 0; r < M; ++r)
#pragma unroll
    for (int y = 0; y < 8; ++y) acc[r][y] ^= d[(y + r + X) & 7] ^ d[(y + r + X + 3) & 7];
#pragma unroll
  for (int r = 0; r < M; ++r)
#pragma unroll
    for (int y = 0; y < 8; ++y) asm volatile("" : "+v"(acc[r][y]));
}

template <int SPW, int CPS, int AHEAD, int NT, int T>
struct Steps {
  using G = Geo<SPW, CPS, AHEAD, NT>;
  __device__ __forceinline__ static void run(u32x2 (&acc)[M][8], uint8_t *ring, const uint8_t *const (&src)[G::NQ],
                                             int lo, int lo8) {
    if constexpr (T < G::NS) {
      constexpr int issued_after = (G::NS - 1 - T) < AHEAD ? (G::NS - 1 - T) : AHEAD;
      wait_vm<G::NQ * issued_after>();
      asm volatile("" ::: "memory");
      uint8_t *slot = ring + (T % G::D) * G::SLOT;
      Cols<T, 0>::go(acc, slot, lo, lo8);
      if constexpr (T + G::D < G::NS) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
        for (int q = 0; q < G::NQ; ++q) dma16<NT>(src[q] + (T + G::D) * CPS * BYTES, slot + q * 1024);
      }
      Steps<SPW, CPS, AHEAD, NT, T + 1>::run(acc, ring, src, lo, lo8);
    }
  }
  template <int TT, int CC>
  struct Cols {
    __device__ __forceinline__ static void go(u32x2 (&acc)[M][8], const uint8_t *slot, int lo, int lo8) {
      if constexpr (CC < CPS && TT * CPS + CC < K) {
        column<SPW, CPS, AHEAD, NT, TT * CPS + CC>(acc, slot + CC * BYTES, lo, lo8);
        Cols<TT, CC + 1>::go(acc, slot, lo, lo8);
      }
    }
  };
};

template <int SPW, int CPS, int AHEAD, int NT, int PADKB>
__global__ void __launch_bounds__(256) geo_enc(const uint8_t *__restrict__ in, uint8_t *__restrict__ out, int stripes) {
  using G = Geo<SPW, CPS, AHEAD, NT>;
  __shared__ __attribute__((aligned(16))) uint8_t rings[4][G::RING];
  __shared__ uint8_t pad[PADKB * 1024 + 4];
  if (stripes < 0) pad[threadIdx.x] = 1;  // (keeps the padding allocated)
  const long long wave = (xcd_block() * 256 + threadIdx.x) >> 6;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const long long s0 = (long long)__builtin_amdgcn_readfirstlane((int)wave) * SPW;
  if (s0 >= stripes) return;
  const int nst = (int)(stripes - s0 < SPW ? stripes - s0 : SPW);
  uint8_t *ring = rings[w];
  // stripe js's step image [stripe][CPS x BYTES]: chunk j = 64 q + lane (clamped)
  const uint8_t *src[G::NQ];
  const int stripe_img = CPS * BYTES;
#pragma unroll
  for (int q = 0; q < G::NQ; ++q) {
    const int j = std::min(64 * q + lane, nst * G::CH - 1);
    src[q] = in + (s0 + j / G::CH) * STRIDE + (j % G::CH) * 16;
  }
#pragma unroll
  for (int t = 0; t < G::D && t < G::NS; ++t)
#pragma unroll
    for (int q = 0; q < G::NQ; ++q) dma16<NT>(src[q] + t * CPS * BYTES, ring + t * G::SLOT + q * 1024);
  const int sl = lane / NCH, c = lane % NCH;
  const int lo = (sl < SPW ? sl : SPW - 1) * stripe_img + 8 * c;
  int lo8 = lo + 8;
  asm volatile("" : "+v"(lo8));
  u32x2 acc[M][8];
#pragma unroll
  for (int r = 0; r < M; ++r)
#pragma unroll
    for (int y = 0; y < 8; ++y) acc[r][y] = u32x2{0, 0};
  Steps<SPW, CPS, AHEAD, NT, 0>::run(acc, ring, src, lo, lo8);
  if (sl >= nst) return;
  const bool last = c == NCH - 1;
  uint8_t *o = out + (s0 + sl) * STRIDE + OUT_OFF + (last ? SUB - 8 : 8 * c);
#pragma unroll
  for (int r = 0; r < M; ++r)
#pragma unroll
    for (int y = 0; y < 8; ++y) {
      const u32x2 v = acc[r][y];
      const u32x2 pv = u32x2{dpp_row_shr1(v.x), dpp_row_shr1(v.y)};
      const u32x2 f = funnel<2>(pv, v);
      __builtin_nontemporal_store(last ? f : v, (u32x2 *)(o + r * BYTES + y * SUB));
    }
}


// ---------------------------------------------------------------- loader / consumers
// One loader wave per workgroup streams the LDS-DMA ring (D slots, each one column-step of the
// workgroup's NC x 3 stripes), NC consumer waves combine; one raw s_barrier per step: the loader
// waits for step t's DMAs (counted vmcnt), meets the consumers, then refills the slot they
// finished with step t - 1 (D - 1 steps in flight).
template <int NC, int D, int CPS>
struct LC {
  static constexpr int NST = 3 * NC;                 // stripes per workgroup
  static constexpr int CH = CPS * BYTES / 16;        // chunks per stripe per step
  static constexpr int NQ = (NST * CH + 63) / 64;    // DMA instructions per step
  static constexpr int SLOT = NQ * 1024;
  static constexpr int NS = (K + CPS - 1) / CPS;
};
template <int NC, int D, int CPS, int T>
struct LCSteps {
  using L = LC<NC, D, CPS>;
  __device__ __forceinline__ static void loader(uint8_t *ring, const uint8_t *const (&src)[L::NQ]) {
    if constexpr (T < L::NS) {
      constexpr int after = (L::NS - 1 - T) < (D - 1) ? (L::NS - 1 - T) : (D - 1);
      wait_vm<L::NQ * after>();
      __builtin_amdgcn_s_barrier();
      if constexpr (T + D - 1 < L::NS && T >= 1) {
        uint8_t *slot = ring + ((T + D - 1) % D) * L::SLOT;
#pragma unroll
        for (int q = 0; q < L::NQ; ++q) dma16<1>(src[q] + (T + D - 1) * CPS * BYTES, slot + q * 1024);
      }
      LCSteps<NC, D, CPS, T + 1>::loader(ring, src);
    }
  }
  __device__ __forceinline__ static void consumer(u32x2 (&acc)[M][8], const uint8_t *ring, int lo, int lo8) {
    if constexpr (T < L::NS) {
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      const uint8_t *slot = ring + (T % D) * L::SLOT;
      Cols<0>::go(acc, slot, lo, lo8);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      LCSteps<NC, D, CPS, T + 1>::consumer(acc, ring, lo, lo8);
    }
  }
  template <int CC>
  struct Cols {
    __device__ __forceinline__ static void go(u32x2 (&acc)[M][8], const uint8_t *slot, int lo, int lo8) {
      if constexpr (CC < CPS && T * CPS + CC < K) {
        column<3, CPS, 0, 1, T * CPS + CC>(acc, slot + CC * BYTES, lo, lo8);
        Cols<CC + 1>::go(acc, slot, lo, lo8);
      }
    }
  };
};
template <int NC, int D, int CPS, int PADKB>
__global__ void __launch_bounds__(64 * (NC + 1)) lc_enc(const uint8_t *__restrict__ in, uint8_t *__restrict__ out, int stripes) {
  using L = LC<NC, D, CPS>;
  __shared__ __attribute__((aligned(16))) uint8_t ring[D * L::SLOT + 16];
  __shared__ uint8_t pad[PADKB * 1024 + 4];
  if (stripes < 0) pad[threadIdx.x] = 1;
  const long long s0 = xcd_block() * L::NST;  // workgroup-uniform (grid covers whole groups)
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (w == 0) {
    const uint8_t *src[L::NQ];
#pragma unroll
    for (int q = 0; q < L::NQ; ++q) {
      const int j = std::min(64 * q + lane, L::NST * L::CH - 1);
      src[q] = in + (s0 + j / L::CH) * STRIDE + (j % L::CH) * 16;
    }
#pragma unroll
    for (int t = 0; t < D && t < L::NS; ++t)
#pragma unroll
      for (int q = 0; q < L::NQ; ++q) dma16<1>(src[q] + t * CPS * BYTES, ring + t * L::SLOT + q * 1024);
    LCSteps<NC, D, CPS, 0>::loader(ring, src);
    return;
  }
  const int sl = lane / NCH, c = lane % NCH;
  const int ls = 3 * (w - 1) + (sl < 3 ? sl : 2);  // stripe in the workgroup
  const int lo = ls * CPS * BYTES + 8 * c;
  int lo8 = lo + 8;
  asm volatile("" : "+v"(lo8));
  u32x2 acc[M][8];
#pragma unroll
  for (int r = 0; r < M; ++r)
#pragma unroll
    for (int y = 0; y < 8; ++y) acc[r][y] = u32x2{0, 0};
  LCSteps<NC, D, CPS, 0>::consumer(acc, ring, lo, lo8);
  if (sl >= 3) return;
  const bool last = c == NCH - 1;
  uint8_t *o = out + (s0 + ls) * STRIDE + OUT_OFF + (last ? SUB - 8 : 8 * c);
#pragma unroll
  for (int r = 0; r < M; ++r)
#pragma unroll
    for (int y = 0; y < 8; ++y) {
      const u32x2 v = acc[r][y];
      const u32x2 pv = u32x2{dpp_row_shr1(v.x), dpp_row_shr1(v.y)};
      const u32x2 f = funnel<2>(pv, v);
      __builtin_nontemporal_store(last ? f : v, (u32x2 *)(o + r * BYTES + y * SUB));
    }
}

static hipEvent_t e0, e1;
template <class F>
static float timeit(F launch) {
  for (int i = 0; i < 3; ++i) launch();
  CK(hipGetLastError());
  CK(hipDeviceSynchronize());
  float best = 1e9f;
  for (int rep = 0; rep < 5; ++rep) {
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
static std::vector<uint8_t> g_ref;
static uint8_t *g_out;

template <int SPW, int CPS, int AHEAD, int NT, int WG>
static void run_geo(const uint8_t *din, uint8_t *dout) {
  using G = Geo<SPW, CPS, AHEAD, NT>;
  constexpr int used = 4 * G::RING;
  constexpr int want_b = 160 * 1024 / WG;  // LDS per workgroup that leaves WG resident
  constexpr int PADKB = used >= want_b - 1024 ? 0 : (want_b - used) / 1024 - 1;
  const long long waves = (STRIPES + SPW - 1) / SPW;
  const int g = (int)((waves + 3) / 4);
  hipFuncAttributes fa;
  CK(hipFuncGetAttributes(&fa, reinterpret_cast<const void *>(geo_enc<SPW, CPS, AHEAD, NT, PADKB>)));
  int occ = 0;
  CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, geo_enc<SPW, CPS, AHEAD, NT, PADKB>, 256, 0));
  const float ms = timeit([&] { geo_enc<SPW, CPS, AHEAD, NT, PADKB><<<g, 256>>>(din, dout, (int)STRIPES); });
  // outputs must not depend on the geometry
  std::vector<uint8_t> got((size_t)(STRIPES * STRIDE));
  CK(hipMemcpy(got.data(), dout, got.size(), hipMemcpyDeviceToHost));
  long long bad = 0;
  if (g_ref.empty()) g_ref = got;
  else
    for (long long s = 0; s < STRIPES; ++s)
      bad += memcmp(got.data() + s * STRIDE + OUT_OFF, g_ref.data() + s * STRIDE + OUT_OFF, M * BYTES) != 0;
  printf("geo SPW=%d CPS=%d AHEAD=%d NT=%d WG=%d (occ %d, %d VGPR, %5.1f KB LDS) %8.4f ms %8.1f GB/s in  %s\n", SPW, CPS,
         AHEAD, NT, WG, occ, fa.numRegs, fa.sharedSizeBytes / 1024.0, ms, IN_BYTES / (ms * 1e-3) / 1e9,
         bad ? "OUTPUT DIFFERS" : "ok");
  fflush(stdout);
  CK(hipMemset(dout, 0, (size_t)(STRIPES * STRIDE) + 65536));
}


template <int NC, int D, int CPS, int WG>
static void run_lc(const uint8_t *din, uint8_t *dout) {
  using L = LC<NC, D, CPS>;
  constexpr int used = D * L::SLOT + 16;
  constexpr int want_b = 160 * 1024 / WG;
  constexpr int PADKB = used >= want_b - 1024 ? 0 : (want_b - used) / 1024 - 1;
  // whole workgroups only (65536 = 7281 x 9 + 7: the remainder is left out of both timing and check)
  const int g = (int)(STRIPES / L::NST);
  hipFuncAttributes fa;
  CK(hipFuncGetAttributes(&fa, reinterpret_cast<const void *>(lc_enc<NC, D, CPS, PADKB>)));
  int occ = 0;
  CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, lc_enc<NC, D, CPS, PADKB>, 64 * (NC + 1), 0));
  const float ms = timeit([&] { lc_enc<NC, D, CPS, PADKB><<<g, 64 * (NC + 1)>>>(din, dout, (int)STRIPES); });
  std::vector<uint8_t> got((size_t)(STRIPES * STRIDE));
  CK(hipMemcpy(got.data(), dout, got.size(), hipMemcpyDeviceToHost));
  long long bad = 0;
  for (long long s = 0; s < (long long)g * L::NST; ++s)
    bad += memcmp(got.data() + s * STRIDE + OUT_OFF, g_ref.data() + s * STRIDE + OUT_OFF, M * BYTES) != 0;
  const double in_b = (double)g * L::NST * STRIDE;
  printf("lc NC=%d D=%d CPS=%d WG=%d (occ %d, %d VGPR, %5.1f KB LDS) %8.4f ms %8.1f GB/s in (scaled to 65536: %.4f ms) %s\n",
         NC, D, CPS, WG, occ, fa.numRegs, fa.sharedSizeBytes / 1024.0, ms, in_b / (ms * 1e-3) / 1e9,
         ms * IN_BYTES / in_b, bad ? "OUTPUT DIFFERS" : "ok");
  fflush(stdout);
  CK(hipMemset(dout, 0, (size_t)(STRIPES * STRIDE) + 65536));
}

int main(int argc, char **argv) {
  uint8_t *din, *dout;
  CK(hipMalloc(&din, IN_BYTES + 65536));
  CK(hipMalloc(&dout, IN_BYTES + 65536));
  {
    std::vector<uint8_t> rnd(1 << 20);
    uint64_t z = 0x9E3779B97F4A7C15ull;
    for (size_t i = 0; i < rnd.size(); ++i) {
      z += 0x9E3779B97F4A7C15ull;
      uint64_t t = z;
      t = (t ^ (t >> 30)) * 0xBF58476D1CE4E5B9ull;
      t = (t ^ (t >> 27)) * 0x94D049BB133111EBull;
      rnd[i] = (uint8_t)(t >> 56);
    }
    for (long long i = 0; i < IN_BYTES + 65536; i += 1 << 20)
      CK(hipMemcpy(din + i, rnd.data(), std::min<long long>(1 << 20, IN_BYTES + 65536 - i), hipMemcpyHostToDevice));
  }
  CK(hipMemset(dout, 0, IN_BYTES + 65536));
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  printf("# ubench_r6: input %.3f GB, output %.3f GB (k29/m4/1296 x 65536)\n", IN_BYTES / 1e9, OUT_BYTES / 1e9);
  if (want(argc, argv, "base")) {  // the product's geometry: 3 stripes, 1 column per step
    run_geo<3, 1, 0, 1, 2>(din, dout);
    run_geo<3, 1, 1, 1, 2>(din, dout);
    run_geo<3, 1, 2, 1, 2>(din, dout);
    run_geo<3, 1, 3, 1, 2>(din, dout);
    run_geo<3, 1, 0, 0, 2>(din, dout);
  }
  if (want(argc, argv, "occ")) {  // waves per CU
    run_geo<3, 1, 0, 1, 1>(din, dout);
    run_geo<3, 1, 0, 1, 3>(din, dout);
    run_geo<3, 1, 0, 1, 4>(din, dout);
    run_geo<3, 1, 1, 1, 1>(din, dout);
    run_geo<3, 1, 1, 1, 3>(din, dout);
  }
  if (want(argc, argv, "cps")) {  // longer contiguous runs per stripe and step
    run_geo<3, 2, 0, 1, 2>(din, dout);
    run_geo<3, 2, 0, 1, 1>(din, dout);
    run_geo<3, 3, 0, 1, 1>(din, dout);
    run_geo<1, 3, 0, 1, 2>(din, dout);
    run_geo<1, 3, 0, 1, 4>(din, dout);
    run_geo<1, 3, 1, 1, 4>(din, dout);
    run_geo<2, 2, 0, 1, 2>(din, dout);
    run_geo<2, 2, 0, 1, 3>(din, dout);
  }
  if (want(argc, argv, "one")) {  // one stripe per wave
    run_geo<1, 1, 0, 1, 4>(din, dout);
    run_geo<1, 1, 1, 1, 4>(din, dout);
    run_geo<1, 1, 2, 1, 4>(din, dout);
    run_geo<1, 2, 0, 1, 4>(din, dout);
    run_geo<1, 2, 1, 1, 4>(din, dout);
    run_geo<1, 1, 0, 1, 6>(din, dout);
  }
  if (want(argc, argv, "wg1")) {  // one workgroup (4 waves) per CU, longer steps
    run_geo<3, 1, 0, 1, 2>(din, dout);
    run_geo<3, 3, 0, 1, 1>(din, dout);
    run_geo<3, 3, 1, 1, 1>(din, dout);
    run_geo<3, 4, 0, 1, 1>(din, dout);
    run_geo<3, 4, 1, 1, 1>(din, dout);
    run_geo<3, 5, 0, 1, 1>(din, dout);
    run_geo<3, 5, 1, 1, 1>(din, dout);
    run_geo<3, 6, 0, 1, 1>(din, dout);
    run_geo<3, 8, 0, 1, 1>(din, dout);
    run_geo<2, 3, 0, 1, 1>(din, dout);
    run_geo<2, 4, 1, 1, 1>(din, dout);
    run_geo<2, 6, 0, 1, 1>(din, dout);
    run_geo<1, 6, 0, 1, 1>(din, dout);
    run_geo<1, 6, 1, 1, 1>(din, dout);
    run_geo<1, 9, 0, 1, 1>(din, dout);
    run_geo<3, 4, 0, 0, 1>(din, dout);
  }
  if (want(argc, argv, "lc")) {  // loader / consumer waves
    run_geo<3, 1, 0, 1, 2>(din, dout);  // (reference output for the check)
    run_lc<3, 2, 1, 4>(din, dout);
    run_lc<3, 3, 1, 4>(din, dout);
    run_lc<3, 4, 1, 3>(din, dout);
    run_lc<3, 3, 1, 2>(din, dout);
    run_lc<3, 4, 1, 2>(din, dout);
    run_lc<7, 2, 1, 2>(din, dout);
    run_lc<7, 3, 1, 2>(din, dout);
    run_lc<7, 3, 1, 1>(din, dout);
    run_lc<3, 2, 2, 2>(din, dout);
    run_lc<3, 3, 2, 2>(din, dout);
    run_lc<7, 2, 2, 1>(din, dout);
    run_lc<3, 3, 1, 1>(din, dout);
  }
  return 0;
}
