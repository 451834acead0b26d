// Micro-benchmark (not product code): the k29/m4/1296-B decode ACCESS PATTERN as the fused
// decode kernel issues it -- slot map held in registers (no per-column memory lookup, which
// ubench_pattern.hip's pattern_buf has: its vmcnt wait on the slot byte also waits for the
// ring's earlier loads), 33 columns (25 shuffled originals, 4 erased = out-of-range buffer
// offsets, then the 4 recovery slots), trivial compute -- to split the remaining decode
// time into "in-place writes" and "the rest of the kernel".
//   inplace   : the 4 outputs overwrite the recovery slots (the reference's semantics)
//   separate  : the 4 outputs go to a compact [stripe][4][bytes] buffer
//   recfirst  : in place, the recovery slots read first (columns k..k+m-1 before the data)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <numeric>
#include <random>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
constexpr int K = 29, M = 4, BYTES = 1296, SUB = 162, NCH = 21, SPW = 3, NC = K + M, NW = (NC + 3) / 4;

template <int X>
__device__ __forceinline__ unsigned slot_of(const unsigned (&w)[NW]) { return (w[X / 4] >> (8 * (X % 4))) & 0xFFu; }

template <int X, int PF, int LAUX>
struct cols {
  __device__ __forceinline__ static void run(u32x2 (&acc)[8], u32x2 (&ring)[PF][8], const __amdgpu_buffer_rsrc_t &rs,
                                             int lbase, const unsigned (&w)[NW]) {
    if constexpr (X < NC) {
      u32x2 nxt[8];
      if constexpr (X + PF < NC) {
        const unsigned s = slot_of<X + PF>(w);
        const int off = s == 0xFFu ? (int)0x80000000 : lbase + (int)s * BYTES;
#pragma unroll
        for (int b = 0; b < 8; ++b) nxt[b] = __builtin_amdgcn_raw_buffer_load_b64(rs, off + b * SUB, 0, LAUX);
      }
#pragma unroll
      for (int b = 0; b < 8; ++b) acc[b] ^= ring[X % PF][b] + (uint32_t)(X + 1);
      if constexpr (X + PF < NC)
#pragma unroll
        for (int b = 0; b < 8; ++b) ring[X % PF][b] = nxt[b];
      cols<X + 1, PF, LAUX>::run(acc, ring, rs, lbase, w);
    }
  }
};

// MODE 0 in place, 1 separate output buffer; SAUX: cache policy of the in-place stores.
template <int PF, int LAUX, int MODE, int SAUX = 2>
__global__ void __launch_bounds__(256) dec_reg(uint8_t *__restrict__ in, uint8_t *__restrict__ out, long long in_stride,
                                                const uint8_t *__restrict__ colmap, const uint8_t *__restrict__ outs,
                                                int stripes) {
  const long long wave = ((long long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63, sl = lane / NCH, c = lane - sl * NCH;
  const long long s0 = __builtin_amdgcn_readfirstlane((int)wave) * (long long)SPW;
  const long long s = s0 + sl;
  if (sl >= SPW || s >= stripes) return;
  const int p = c == NCH - 1 ? SUB - 8 : c * 8;
  const long long nst = stripes - s0 < SPW ? stripes - s0 : SPW;
  __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(in + s0 * in_stride, 0, (int)(nst * in_stride), 0x00020000);
  const int lbase = (int)(sl * in_stride) + p;
  unsigned w[NW];
#pragma unroll
  for (int i = 0; i < NW; ++i) w[i] = ((const unsigned *)(colmap + s * 4 * NW))[i];
  const unsigned ow = *(const unsigned *)(outs + s * 4);
  u32x2 acc[8];
#pragma unroll
  for (int b = 0; b < 8; ++b) acc[b] = u32x2{0, 0};
  u32x2 ring[PF][8];
#pragma unroll
  for (int q = 0; q < PF; ++q) {
    const unsigned sq = (w[q / 4] >> (8 * (q % 4))) & 0xFFu;
    const int off = sq == 0xFFu ? (int)0x80000000 : lbase + (int)sq * BYTES;
#pragma unroll
    for (int b = 0; b < 8; ++b) ring[q][b] = __builtin_amdgcn_raw_buffer_load_b64(rs, off + b * SUB, 0, LAUX);
  }
  cols<0, PF, LAUX>::run(acc, ring, rs, lbase, w);
#pragma unroll
  for (int r = 0; r < M; ++r) {
    const int slot = (ow >> (8 * r)) & 0xFF;
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      const u32x2 v = acc[b] ^ u32x2{(uint32_t)r, 0};
      if (MODE == 0) __builtin_amdgcn_raw_buffer_store_b64(v, rs, lbase + slot * BYTES + b * SUB, 0, SAUX);
      else __builtin_nontemporal_store(v, (u32x2 *)(out + s * (long long)(M * BYTES) + r * BYTES + b * SUB + p));
    }
  }
}

int main() {
  const int stripes = 65536;
  const size_t in_bytes = (size_t)stripes * K * BYTES;
  uint8_t *din, *dout, *dcols, *douts;
  CK(hipMalloc(&din, in_bytes + 4096));
  CK(hipMalloc(&dout, (size_t)stripes * M * BYTES + 4096));
  CK(hipMalloc(&dcols, (size_t)stripes * 4 * NW));
  CK(hipMalloc(&douts, (size_t)stripes * 4));
  CK(hipMemset(din, 0x5a, in_bytes));
  std::mt19937 rng(7);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int grid = (stripes / SPW + 1 + 3) / 4;
  auto setup = [&](bool recfirst) {
    std::vector<uint8_t> cols((size_t)stripes * 4 * NW, 0xFF), outs((size_t)stripes * 4);
    for (int s = 0; s < stripes; ++s) {
      // slot layout as the bench: originals in a shuffled order, 4 of them erased and
      // their slots holding the recovery blocks.
      std::vector<int> perm(K);
      std::iota(perm.begin(), perm.end(), 0);
      std::shuffle(perm.begin(), perm.end(), rng);  // perm[slot] = original held there
      std::vector<int> rslots;
      for (int i = 0; i < M; ++i) rslots.push_back(K - M + i);
      uint8_t *cl = &cols[(size_t)s * 4 * NW];
      std::vector<int> where(K, 0xFF);
      for (int slot = 0; slot < K - M; ++slot) where[perm[slot]] = slot;
      int x = 0;
      if (recfirst) for (int r = 0; r < M; ++r) cl[x++] = (uint8_t)rslots[r];
      for (int o = 0; o < K; ++o) cl[x++] = (uint8_t)where[o];
      if (!recfirst) for (int r = 0; r < M; ++r) cl[x++] = (uint8_t)rslots[r];
      for (int r = 0; r < M; ++r) outs[s * 4 + r] = (uint8_t)rslots[r];
    }
    CK(hipMemcpy(dcols, cols.data(), cols.size(), hipMemcpyHostToDevice));
    CK(hipMemcpy(douts, outs.data(), outs.size(), hipMemcpyHostToDevice));
  };
  auto run = [&](const char *name, auto kern) {
    auto launch = [&] { kern<<<grid, 256>>>(din, dout, (long long)K * BYTES, dcols, douts, stripes); };
    for (int i = 0; i < 3; ++i) launch();
    CK(hipDeviceSynchronize());
    float best = 1e9;
    for (int rep = 0; rep < 3; ++rep) {
      CK(hipEventRecord(e0));
      for (int i = 0; i < 10; ++i) launch();
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      best = std::min(best, ms / 10);
    }
    printf("%-28s %7.4f ms  %7.1f GB/s input\n", name, best, in_bytes / (best * 1e-3) / 1e9);
  };
  for (int round = 0; round < 2; ++round) {
    setup(false);
    run("reg inplace def PF1", dec_reg<1, 0, 0>);
    run("reg inplace def PF2", dec_reg<2, 0, 0>);
    run("reg inplace def PF3", dec_reg<3, 0, 0>);
    run("reg inplace nt PF3", dec_reg<3, 2, 0>);
    run("reg separate def PF1", dec_reg<1, 0, 1>);
    run("reg separate def PF3", dec_reg<3, 0, 1>);
    run("reg separate nt PF3", dec_reg<3, 2, 1>);
    setup(true);
    run("reg recfirst inplace def PF1", dec_reg<1, 0, 0>);
    run("reg recfirst inplace def PF3", dec_reg<3, 0, 0>);
    run("reg recfirst inplace st-def PF1", dec_reg<1, 0, 0, 0>);
    run("reg recfirst inplace st-sc1 PF1", dec_reg<1, 0, 0, 16>);
    run("reg recfirst inplace ld-nt PF1", dec_reg<1, 2, 0>);
    setup(false);
    run("reg inplace st-def PF1", dec_reg<1, 0, 0, 0>);
  }
  CK(hipGetLastError());
  return 0;
}
