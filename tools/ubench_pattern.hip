// Micro-benchmark (not product code): the k29/m4/1296-B decode and encode ACCESS PATTERNS
// with trivial compute, to split the decode/encode time gap into access-pattern and
// instruction-side parts.  Lane mapping as the specialised kernels: 8-byte lanes, 21
// lanes per stripe, 3 stripes per wave, loads 2-byte aligned, non-temporal.
//   enc      : read blocks 0..28 of each stripe in order, write 4 blocks to a separate buffer
//   dec_id   : read 29 slots in identity order, write 4 slots in place
//   dec_perm : read 29 slots in a per-stripe random order (the bench's shuffled layout),
//              write 4 slots in place
//   dec_zero : as the decode kernel does: 25 permuted originals + 4 zero-page columns +
//              4 recovery slots (33 column loads), write 4 slots in place
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <numeric>
#include <random>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
constexpr int K = 29, M = 4, BYTES = 1296, SUB = 162, NCH = 21, SPW = 3;

template <int PF>
__global__ void __launch_bounds__(256) pattern(const uint8_t *__restrict__ in, uint8_t *__restrict__ out, long long in_stride,
                                               long long out_stride, const uint8_t *__restrict__ cols, int ncols,
                                               const uint8_t *__restrict__ outs, const uint8_t *__restrict__ zero,
                                               int stripes) {
  const long long wave = ((long long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63, sl = lane / NCH, c = lane - sl * NCH;
  const long long s = wave * SPW + sl;
  if (sl >= SPW || s >= stripes) return;
  const int p = c == NCH - 1 ? SUB - 8 : c * 8;
  const uint8_t *base = in + s * in_stride + p;
  const uint8_t *cl = cols + s * 40;  // per-stripe column list: slot index, 0xFF = zero page
  u32x2 acc[8];
#pragma unroll
  for (int b = 0; b < 8; ++b) acc[b] = u32x2{0, 0};
  u32x2 ring[PF][8];
  auto src = [&](int x) { const unsigned sl2 = cl[x]; return sl2 == 0xFF ? zero + p : base + (long long)sl2 * BYTES; };
#pragma unroll
  for (int q = 0; q < PF; ++q) {
    const uint8_t *a = src(q);
#pragma unroll
    for (int b = 0; b < 8; ++b) ring[q][b] = __builtin_nontemporal_load((const u32x2 *)(a + b * SUB));
  }
  for (int x = 0; x < ncols; x += PF) {
#pragma unroll
    for (int q = 0; q < PF; ++q) {
      if (x + q < ncols) {
#pragma unroll
        for (int b = 0; b < 8; ++b) acc[b] ^= ring[q][b];
        if (x + q + PF < ncols) {
          const uint8_t *a = src(x + q + PF);
#pragma unroll
          for (int b = 0; b < 8; ++b) ring[q][b] = __builtin_nontemporal_load((const u32x2 *)(a + b * SUB));
        }
      }
    }
  }
  uint8_t *o = out + s * out_stride + p;
#pragma unroll
  for (int r = 0; r < M; ++r)
#pragma unroll
    for (int b = 0; b < 8; ++b)
      __builtin_nontemporal_store(acc[b] ^ u32x2{(uint32_t)r, 0}, (u32x2 *)(o + (long long)outs[s * 4 + r] * BYTES + b * SUB));
}

// Buffer-load variant: the wave's three stripes are one buffer resource (wave-uniform
// base, num_records = their bytes); an erased column's offset is out of range, which the
// hardware answers with zeros and no memory request (OOB = 1) -- or it reads the zero page.
// LAUX / SAUX: cache-policy bits of the loads / stores (2 = nt, 0 = default, 1 = sc0, 17 = sc0 sc1).
template <int LAUX, int SAUX, bool OOB>
__global__ void __launch_bounds__(256) pattern_buf(uint8_t *__restrict__ in, long long in_stride,
                                                   const uint8_t *__restrict__ cols, int ncols,
                                                   const uint8_t *__restrict__ outs, const uint8_t *__restrict__ zero,
                                                   int stripes) {
  const long long wave = ((long long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63, sl = lane / NCH, c = lane - sl * NCH;
  const long long s0 = __builtin_amdgcn_readfirstlane((int)wave) * (long long)SPW;
  const long long s = s0 + sl;
  if (sl >= SPW || s >= stripes) return;
  const int p = c == NCH - 1 ? SUB - 8 : c * 8;
  __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(in + s0 * in_stride, 0, (int)(SPW * in_stride), 0x00020000);
  const int lbase = (int)(sl * in_stride) + p;
  const uint8_t *cl = cols + s * 40;
  u32x2 acc[8];
#pragma unroll
  for (int b = 0; b < 8; ++b) acc[b] = u32x2{0, 0};
  u32x2 ring[3][8];
  auto ld = [&](int x, u32x2 (&d)[8]) {
    const unsigned slot = cl[x];
    if (OOB || slot != 0xFF) {
      const int off = slot == 0xFF ? (int)0x80000000 : lbase + (int)slot * BYTES;
#pragma unroll
      for (int b = 0; b < 8; ++b) d[b] = __builtin_amdgcn_raw_buffer_load_b64(rs, off + b * SUB, 0, LAUX);
    } else {
#pragma unroll
      for (int b = 0; b < 8; ++b) d[b] = __builtin_nontemporal_load((const u32x2 *)(zero + p + b * SUB));
    }
  };
#pragma unroll
  for (int q = 0; q < 3; ++q) ld(q, ring[q]);
  for (int x = 0; x < ncols; x += 3) {
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      if (x + q < ncols) {
#pragma unroll
        for (int b = 0; b < 8; ++b) acc[b] ^= ring[q][b];
        if (x + q + 3 < ncols) ld(x + q + 3, ring[q]);
      }
    }
  }
#pragma unroll
  for (int r = 0; r < M; ++r)
#pragma unroll
    for (int b = 0; b < 8; ++b)
      __builtin_amdgcn_raw_buffer_store_b64(acc[b] ^ u32x2{(uint32_t)r, 0}, rs, lbase + (int)outs[s * 4 + r] * BYTES + b * SUB, 0, SAUX);
}

// Encode pattern with buffer loads: column x at soffset x * BYTES (wave-uniform SGPR),
// sub-block b in the immediate offset, one 32-bit lane offset; separate output buffer.
template <int LAUX>
__global__ void __launch_bounds__(256) pattern_enc_buf(const uint8_t *__restrict__ in, uint8_t *__restrict__ out,
                                                       long long in_stride, long long out_stride, int stripes) {
  const long long wave = ((long long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63, sl = lane / NCH, c = lane - sl * NCH;
  const long long s0 = __builtin_amdgcn_readfirstlane((int)wave) * (long long)SPW;
  const long long s = s0 + sl;
  if (sl >= SPW || s >= stripes) return;
  const int p = c == NCH - 1 ? SUB - 8 : c * 8;
  __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *)(in + s0 * in_stride), 0, (int)(SPW * in_stride), 0x00020000);
  const int lbase = (int)(sl * in_stride) + p;
  u32x2 acc[8];
#pragma unroll
  for (int b = 0; b < 8; ++b) acc[b] = u32x2{0, 0};
  u32x2 ring[3][8];
#pragma unroll
  for (int q = 0; q < 3; ++q)
#pragma unroll
    for (int b = 0; b < 8; ++b) ring[q][b] = __builtin_amdgcn_raw_buffer_load_b64(rs, lbase + b * SUB, q * BYTES, LAUX);
#pragma unroll
  for (int x = 0; x < K; ++x) {
#pragma unroll
    for (int b = 0; b < 8; ++b) acc[b] ^= ring[x % 3][b];
    if (x + 3 < K)
#pragma unroll
      for (int b = 0; b < 8; ++b) ring[x % 3][b] = __builtin_amdgcn_raw_buffer_load_b64(rs, lbase + b * SUB, (x + 3) * BYTES, LAUX);
  }
  uint8_t *o = out + s * out_stride + p;
#pragma unroll
  for (int r = 0; r < M; ++r)
#pragma unroll
    for (int b = 0; b < 8; ++b) __builtin_nontemporal_store(acc[b] ^ u32x2{(uint32_t)r, 0}, (u32x2 *)(o + r * BYTES + b * SUB));
}

// Encode pattern with the columns staged by LDS-DMA: per column, the wave's three
// stripe-columns (3 x 1296 contiguous bytes) arrive as 16-B chunks in consecutive lanes
// (global_load_lds_dwordx4, fully coalesced: 4 wave instructions instead of 8 scattered
// 8-B loads), D columns in flight in a per-wave LDS ring; each lane then reads its 8
// sub-block words from LDS (2-byte aligned ds_read_b64).
template <int D>
__global__ void __launch_bounds__(256) pattern_enc_dma(const uint8_t *__restrict__ in, uint8_t *__restrict__ out,
                                                       long long in_stride, long long out_stride, int stripes) {
  __shared__ __attribute__((aligned(16))) uint8_t ring[4][D][4096];
  const long long wave = ((long long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int w = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63, sl = lane / NCH, c = lane - sl * NCH;
  const long long s0 = __builtin_amdgcn_readfirstlane((int)wave) * (long long)SPW;
  if (s0 >= stripes) return;
  const int ns = (int)min((long long)SPW, stripes - s0);
  const int p = c == NCH - 1 ? SUB - 8 : c * 8;
  const uint8_t *src[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int j = min(i * 64 + lane, SPW * 81 - 1);
    src[i] = in + (s0 + min(j / 81, ns - 1)) * in_stride + (j % 81) * 16;
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
    const int left = min(D - 1, K - 1 - x);  // columns issued after x
    if (left == 2) __builtin_amdgcn_s_waitcnt((8 & 15) | ((8 >> 4) << 14) | (7 << 4) | (15 << 8));
    else if (left == 1) __builtin_amdgcn_s_waitcnt(4 | (7 << 4) | (15 << 8));
    else if (left == 3) __builtin_amdgcn_s_waitcnt(12 | (7 << 4) | (15 << 8));
    else __builtin_amdgcn_s_waitcnt(0 | (7 << 4) | (15 << 8));
    const uint8_t *t = &ring[w][x % D][lo];
    u32x2 v[8];
#pragma unroll
    for (int b = 0; b < 8; ++b) v[b] = *(const u32x2 *)(t + b * SUB);
#pragma unroll
    for (int b = 0; b < 8; ++b) acc[b] ^= v[b];
    if (x + D < K) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      issue(x + D, x % D);
    }
  }
  if (sl >= SPW || s0 + sl >= stripes) return;
  uint8_t *o = out + (s0 + sl) * out_stride + p;
#pragma unroll
  for (int r = 0; r < M; ++r)
#pragma unroll
    for (int b = 0; b < 8; ++b) __builtin_nontemporal_store(acc[b] ^ u32x2{(uint32_t)r, 0}, (u32x2 *)(o + r * BYTES + b * SUB));
}

// The floor for the encode's bytes: read the input and write the output as flat arrays,
// 16 B per lane, fully coalesced, grid-stride (no stripe structure at all).
template <int U>
__global__ void __launch_bounds__(256) pattern_stream(const uint8_t *__restrict__ in, uint8_t *__restrict__ out,
                                                      long long in_bytes, long long out_bytes) {
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  const long long n = in_bytes / 16, no = out_bytes / 16, tid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long nt = (long long)gridDim.x * blockDim.x;
  u32x4 acc = {0, 0, 0, 0};
  for (long long i = tid; i < n; i += U * nt) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = i + u * nt < n ? __builtin_nontemporal_load((const u32x4 *)in + i + u * nt) : u32x4{0, 0, 0, 0};
#pragma unroll
    for (int u = 0; u < U; ++u) acc ^= v[u];
  }
  for (long long i = tid; i < no; i += nt) __builtin_nontemporal_store(acc ^ u32x4{(uint32_t)i, 0, 0, 0}, (u32x4 *)out + i);
}

int main() {
  const int stripes = 65536;
  const size_t in_bytes = (size_t)stripes * K * BYTES;
  uint8_t *din, *dout, *dzero, *dcols, *douts;
  CK(hipMalloc(&din, in_bytes + 4096));
  CK(hipMalloc(&dout, (size_t)stripes * M * BYTES + 4096));
  CK(hipMalloc(&dzero, 64 * BYTES));
  CK(hipMalloc(&dcols, (size_t)stripes * 40));
  CK(hipMalloc(&douts, (size_t)stripes * 4));
  CK(hipMemset(din, 0x5a, in_bytes));
  CK(hipMemset(dzero, 0, 64 * BYTES));
  std::mt19937 rng(7);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int grid = (stripes / SPW + 1 + 3) / 4;
  struct Case { const char *name; int mode; };
  for (Case cs : {Case{"enc", 0}, Case{"dec_id", 1}, Case{"dec_perm", 2}, Case{"dec_zero", 3}}) {
    std::vector<uint8_t> cols((size_t)stripes * 40, 0), outs((size_t)stripes * 4);
    int ncols = K;
    for (int s = 0; s < stripes; ++s) {
      std::vector<int> perm(K);
      std::iota(perm.begin(), perm.end(), 0);
      if (cs.mode >= 2) std::shuffle(perm.begin(), perm.end(), rng);
      if (cs.mode == 3) {  // erase 4 originals: their columns read the zero page, recovery slots appended
        ncols = K + M;
        std::vector<int> erased(perm.begin() + K - M, perm.end());
        for (int x = 0; x < K; ++x) cols[s * 40 + x] = (std::find(erased.begin(), erased.end(), x) != erased.end()) ? 0xFF : (uint8_t)x;
        for (int r = 0; r < M; ++r) cols[s * 40 + K + r] = (uint8_t)(K - M + r);
      } else {
        for (int x = 0; x < K; ++x) cols[s * 40 + x] = (uint8_t)perm[x];
      }
      for (int r = 0; r < M; ++r) outs[s * 4 + r] = cs.mode == 0 ? (uint8_t)r : (uint8_t)(K - M + r);
    }
    CK(hipMemcpy(dcols, cols.data(), cols.size(), hipMemcpyHostToDevice));
    CK(hipMemcpy(douts, outs.data(), outs.size(), hipMemcpyHostToDevice));
    uint8_t *o = cs.mode == 0 ? dout : din;
    const long long os = cs.mode == 0 ? (long long)M * BYTES : (long long)K * BYTES;
    for (int pf : {1, 3}) {
      auto launch = [&] {
        if (pf == 1) pattern<1><<<grid, 256>>>(din, o, (long long)K * BYTES, os, dcols, ncols, douts, dzero, stripes);
        else pattern<3><<<grid, 256>>>(din, o, (long long)K * BYTES, os, dcols, ncols, douts, dzero, stripes);
      };
      for (int i = 0; i < 3; ++i) launch();
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0));
      for (int i = 0; i < 10; ++i) launch();
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      printf("%-9s PF=%d  %7.4f ms  %7.1f GB/s input\n", cs.name, pf, ms / 10, in_bytes / (ms / 10 * 1e-3) / 1e9);
    }
  }
  // buffer-load variants on the decode layout (33 columns, 4 erased -> zero page or OOB)
  {
    std::vector<uint8_t> cols((size_t)stripes * 40, 0), outs((size_t)stripes * 4);
    for (int s = 0; s < stripes; ++s) {
      std::vector<int> perm(K);
      std::iota(perm.begin(), perm.end(), 0);
      std::shuffle(perm.begin(), perm.end(), rng);
      std::vector<int> erased(perm.begin() + K - M, perm.end());
      for (int x = 0; x < K; ++x) cols[s * 40 + x] = (std::find(erased.begin(), erased.end(), x) != erased.end()) ? 0xFF : (uint8_t)x;
      for (int r = 0; r < M; ++r) cols[s * 40 + K + r] = (uint8_t)(K - M + r);
      for (int r = 0; r < M; ++r) outs[s * 4 + r] = (uint8_t)(K - M + r);
    }
    CK(hipMemcpy(dcols, cols.data(), cols.size(), hipMemcpyHostToDevice));
    CK(hipMemcpy(douts, outs.data(), outs.size(), hipMemcpyHostToDevice));
    auto run = [&](const char *name, auto kern) {
      auto launch = [&] { kern<<<grid, 256>>>(din, (long long)K * BYTES, dcols, K + M, douts, dzero, stripes); };
      for (int i = 0; i < 3; ++i) launch();
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0));
      for (int i = 0; i < 10; ++i) launch();
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      printf("%-22s %7.4f ms  %7.1f GB/s input\n", name, ms / 10, in_bytes / (ms / 10 * 1e-3) / 1e9);
    };
    auto run_enc = [&](const char *name, auto kern) {
      auto launch = [&] { kern<<<grid, 256>>>(din, dout, (long long)K * BYTES, (long long)M * BYTES, stripes); };
      for (int i = 0; i < 3; ++i) launch();
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0));
      for (int i = 0; i < 10; ++i) launch();
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      printf("%-22s %7.4f ms  %7.1f GB/s input\n", name, ms / 10, in_bytes / (ms / 10 * 1e-3) / 1e9);
    };
    run_enc("enc buf nt", pattern_enc_buf<2>);
    {  // the DMA variant must produce the buffer variant's bytes
      const size_t ob = (size_t)stripes * M * BYTES;
      std::vector<uint8_t> h(ob);
      for (size_t i = 0; i < in_bytes; i += 4096) CK(hipMemset(din + i, (int)((i * 2654435761u) >> 24), std::min<size_t>(4096, in_bytes - i)));
      pattern_enc_buf<2><<<grid, 256>>>(din, dout, (long long)K * BYTES, (long long)M * BYTES, stripes);
      CK(hipMemcpy(h.data(), dout, ob, hipMemcpyDeviceToHost));
      CK(hipMemset(dout, 0, ob));
      pattern_enc_dma<3><<<grid, 256>>>(din, dout, (long long)K * BYTES, (long long)M * BYTES, stripes);
      std::vector<uint8_t> h2(ob);
      CK(hipMemcpy(h2.data(), dout, ob, hipMemcpyDeviceToHost));
      printf("enc dma bytes %s\n", h == h2 ? "match" : "DIFFER");
    }
    run_enc("enc dma D=2", pattern_enc_dma<2>);
    run_enc("enc dma D=3", pattern_enc_dma<3>);
    run_enc("enc dma D=4", pattern_enc_dma<4>);
    for (int g : {2048, 8192, 32768})
      for (int u : {4, 8}) {
        const long long ob = (long long)stripes * M * BYTES;
        auto launch = [&] {
          if (u == 4) pattern_stream<4><<<g, 256>>>(din, dout, (long long)in_bytes, ob);
          else pattern_stream<8><<<g, 256>>>(din, dout, (long long)in_bytes, ob);
        };
        for (int i = 0; i < 3; ++i) launch();
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0));
        for (int i = 0; i < 10; ++i) launch();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        printf("flat stream r+w g=%-5d U=%d %7.4f ms  %7.1f GB/s input\n", g, u, ms / 10, in_bytes / (ms / 10 * 1e-3) / 1e9);
      }
    run_enc("enc buf def", pattern_enc_buf<0>);
    run("buf zero-page nt/nt", pattern_buf<2, 2, false>);
    run("buf oob nt/nt", pattern_buf<2, 2, true>);
    run("buf oob def/nt", pattern_buf<0, 2, true>);
    run("buf oob nt/def", pattern_buf<2, 0, true>);
    run("buf oob sc0sc1/nt", pattern_buf<17, 2, true>);
    run("buf oob nt/sc0sc1", pattern_buf<2, 17, true>);
    run("buf oob sc1nt/nt", pattern_buf<18, 2, true>);
    run("buf oob nt/sc1nt", pattern_buf<2, 18, true>);
  }
  CK(hipGetLastError());
  return 0;
}
