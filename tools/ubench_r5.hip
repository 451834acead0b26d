// Micro-benchmark (not product code), round 5: the k29/m4/1296-B encode's HBM floor and a
// new load pattern for it.
//   copy / read : calibration (the float4 copy and the read-only stream of round 4);
//   mix         : the encode's bytes as a flat 29:4 stream, by lane width (8 / 16 B), by
//                 contiguous segment per instruction (1024 .. 128 B), by block size, and with
//                 the stores of one unit issued between the loads of the next;
//   enc         : the product's access pattern (8-byte lanes, 3 stripes per wave, 8 loads of
//                 3 x 168-B pieces per column), heavy register footprint, bench output layout;
//   flat        : columns loaded as aligned 16-B chunks (4 dwordx4 per column per wave of 3
//                 stripes), light compute: the load pattern of the transposed kernels below;
//   ldst        : flat loads into a VGPR ring, ds_write_b128 into a per-wave LDS slot, every
//                 lane's 8 bytes of sub-block b read back as two naturally aligned ds_read_b64
//                 (misaligned DS accesses replay at 64 cycles, cdna_hip_programming.md G17)
//                 and funnelled with v_alignbyte; heavy compute; outputs as the product;
//   ldsd        : the same with the columns landed by LDS-DMA (global_load_lds_dwordx4) into a
//                 ring of D slots per wave.
// The transposed kernels' outputs are compared byte for byte with enc's.
// Usage: ubench_r5 [group ...]   (default: all groups)
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
constexpr long long STRIDE = (long long)K * BYTES;    // 37584
constexpr long long IN_BYTES = STRIPES * STRIDE;      // 2.463 GB
constexpr long long OUT_BYTES = STRIPES * M * BYTES;  // 0.340 GB
constexpr long long OUT_OFF = (long long)(K - M) * BYTES;  // bench layout: recovery in slots 25..28

template <bool NT, class T>
__device__ __forceinline__ T ldg(const T *p) { return NT ? __builtin_nontemporal_load(p) : *p; }
template <bool NT, class T>
__device__ __forceinline__ void stg(T *p, T v) {
  if (NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}
template <int W>
struct wt;
template <>
struct wt<8> { typedef u32x2 T; };
template <>
struct wt<16> { typedef u32x4 T; };

// Each XCD (own L2) walks one contiguous run of blocks (the product's LH_XCD mapping).
__device__ __forceinline__ long long xcd_block() {
  const unsigned b = blockIdx.x, per = gridDim.x / 8;
  return b < per * 8 ? (long long)(b % 8) * per + b / 8 : (long long)b;
}

// ---------------------------------------------------------------- calibration
__global__ void __launch_bounds__(256) copy_os(const u32x4 *__restrict__ in, u32x4 *__restrict__ out, long long n) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i < n) stg<true>(out + i, ldg<true>(in + i));
}
__global__ void __launch_bounds__(256) read_os(const u32x4 *__restrict__ in, u32x4 *__restrict__ sink, long long n) {
  const long long base = (long long)blockIdx.x * 256 * 8 + threadIdx.x;
  u32x4 acc = {0, 0, 0, 0};
#pragma unroll
  for (int u = 0; u < 8; ++u)
    if (base + u * 256 < n) acc ^= ldg<true>(in + base + u * 256);
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) sink[threadIdx.x] = acc;
}

// ---------------------------------------------------------------- mix
// Unit = 29 columns of SEG contiguous bytes in (29 * SEG B) and 4 x SEG out.  LB-byte lanes,
// SEG / LB lanes per unit, 64 * LB / SEG units per wave (so an instruction touches that many
// segments); all 29 loads in flight, then the 4 stores.
template <int LB, int SEG, int BS>
__global__ void __launch_bounds__(BS) mixv(const uint8_t *__restrict__ in, uint8_t *__restrict__ out, long long units) {
  typedef typename wt<LB>::T T;
  constexpr int LPS = SEG / LB, U = 64 / LPS;
  const long long wave = (xcd_block() * BS + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  const long long u = wave * U + lane / LPS;
  if (u >= units) return;
  const int off = (lane % LPS) * LB;
  const T *src = (const T *)(in + u * K * SEG + off);
  T v[K];
#pragma unroll
  for (int x = 0; x < K; ++x) v[x] = ldg<true>((const T *)((const uint8_t *)src + x * SEG));
  T acc[M] = {};
#pragma unroll
  for (int x = 0; x < K; ++x) acc[x % M] ^= v[x];
#pragma unroll
  for (int r = 0; r < M; ++r) stg<true>((T *)(out + u * M * SEG + off + r * SEG), acc[r]);
}
// Two units per wave (16-B lanes, 1-KiB segments): unit B's first H loads are issued before
// unit A's stores, so stores sit between loads.
template <int H>
__global__ void __launch_bounds__(256) mix2(const uint8_t *__restrict__ in, uint8_t *__restrict__ out, long long units) {
  const long long wave = (xcd_block() * 256 + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  const long long ua = wave * 2, ub = ua + 1;
  if (ub >= units) return;
  const u32x4 *sa = (const u32x4 *)(in + ua * K * 1024) + lane, *sb = (const u32x4 *)(in + ub * K * 1024) + lane;
  u32x4 v[K];
#pragma unroll
  for (int x = 0; x < K; ++x) v[x] = ldg<true>(sa + x * 64);
  u32x4 acc[M] = {};
#pragma unroll
  for (int x = 0; x < K; ++x) acc[x % M] ^= v[x];
  u32x4 w[K];
#pragma unroll
  for (int x = 0; x < H; ++x) w[x] = ldg<true>(sb + x * 64);
#pragma unroll
  for (int r = 0; r < M; ++r) stg<true>((u32x4 *)(out + ua * M * 1024) + lane + r * 64, acc[r]);
#pragma unroll
  for (int x = H; x < K; ++x) w[x] = ldg<true>(sb + x * 64);
  u32x4 acc2[M] = {};
#pragma unroll
  for (int x = 0; x < K; ++x) acc2[x % M] ^= w[x];
#pragma unroll
  for (int r = 0; r < M; ++r) stg<true>((u32x4 *)(out + ub * M * 1024) + lane + r * 64, acc2[r]);
}

// ---------------------------------------------------------------- enc (the product's pattern)
// 8-byte lanes, 21 per stripe, 3 stripes per wave; the last chunk of a sub-block shifted back
// to [154, 162).  acc[r][y] ^= d[(y + r + x) & 7] stands in for the network (the same function
// of the loaded bytes in every kernel below, so the outputs can be compared).
template <int PF>
__global__ void __launch_bounds__(256) enc_pat(const uint8_t *__restrict__ in, uint8_t *__restrict__ out, int stripes) {
  constexpr int NCH = 21, SPW = 3;
  const long long wave = (xcd_block() * 256 + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63, sl = lane / NCH, c = lane - sl * NCH;
  const long long s0 = (long long)__builtin_amdgcn_readfirstlane((int)wave) * SPW;
  const long long s = s0 + sl;
  if (sl >= SPW || s >= stripes) return;
  const int p = c == NCH - 1 ? SUB - 8 : c * 8;
  const long long nst = stripes - s0 < SPW ? stripes - s0 : SPW;
  __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *)(in + s0 * STRIDE), 0, (int)(nst * STRIDE), 0x00020000);
  const int lbase = (int)(sl * STRIDE) + p;
  u32x2 acc[M][8];
#pragma unroll
  for (int r = 0; r < M; ++r)
#pragma unroll
    for (int y = 0; y < 8; ++y) acc[r][y] = u32x2{0, 0};
  u32x2 ring[PF][8];
#pragma unroll
  for (int q = 0; q < PF; ++q)
#pragma unroll
    for (int b = 0; b < 8; ++b) ring[q][b] = __builtin_amdgcn_raw_buffer_load_b64(rs, lbase + b * SUB, q * BYTES, 2);
#pragma unroll
  for (int x = 0; x < K; ++x) {
    u32x2 nxt[8];
    if (x + PF < K)
#pragma unroll
      for (int b = 0; b < 8; ++b) nxt[b] = __builtin_amdgcn_raw_buffer_load_b64(rs, lbase + b * SUB, (x + PF) * BYTES, 2);
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
  uint8_t *o = out + s * STRIDE + OUT_OFF + p;
#pragma unroll
  for (int r = 0; r < M; ++r)
#pragma unroll
    for (int y = 0; y < 8; ++y) __builtin_nontemporal_store(acc[r][y] ^ u32x2{(uint32_t)r * 0x01010101u, (uint32_t)r * 0x01010101u}, (u32x2 *)(o + r * BYTES + y * SUB));
}

// ---------------------------------------------------------------- flat column loads
// Column x of the wave's 3 stripes = 243 aligned 16-B chunks, chunk j = 64 q + lane (q < 4):
// stripe j / 81, bytes (j % 81) * 16 of its block x.  One buffer resource over the 3 stripes,
// column offset in soffset.
struct flat_src {
  __amdgpu_buffer_rsrc_t rs;
  int voff[4];
  __device__ __forceinline__ void init(const uint8_t *in, long long s0, int nst, int lane) {
    rs = __builtin_amdgcn_make_buffer_rsrc((void *)(in + s0 * STRIDE), 0, (int)(nst * STRIDE), 0x00020000);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int j = 64 * q + lane, js = j / 81;
      voff[q] = (j < 243 && js < nst) ? (int)(js * STRIDE) + (j % 81) * 16 : (int)0x80000000;
    }
  }
  __device__ __forceinline__ void load(u32x4 (&v)[4], int x) const {
#pragma unroll
    for (int q = 0; q < 4; ++q) v[q] = __builtin_amdgcn_raw_buffer_load_b128(rs, voff[q], x * BYTES, 2);
  }
};

// STM 0: outputs as flat aligned 16-B chunks (16 dwordx4 stores per wave); STM 1: 32 8-byte
// stores per lane at the product's 2-byte-aligned positions.
template <int PF, int STM>
__global__ void __launch_bounds__(256) flat_pat(const uint8_t *__restrict__ in, uint8_t *__restrict__ out, int stripes) {
  const long long wave = (xcd_block() * 256 + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  const long long s0 = (long long)__builtin_amdgcn_readfirstlane((int)wave) * 3;
  if (s0 >= stripes) return;
  const int nst = (int)(stripes - s0 < 3 ? stripes - s0 : 3);
  flat_src S;
  S.init(in, s0, nst, lane);
  u32x4 ring[PF][4], acc[4] = {};
#pragma unroll
  for (int q = 0; q < PF; ++q) S.load(ring[q], q);
#pragma unroll
  for (int x = 0; x < K; ++x) {
    u32x4 nxt[4];
    if (x + PF < K) S.load(nxt, x + PF);
#pragma unroll
    for (int q = 0; q < 4; ++q) acc[q] ^= ring[x % PF][q];
#pragma unroll
    for (int q = 0; q < 4; ++q) asm volatile("" : "+v"(acc[q]));
    if (x + PF < K)
#pragma unroll
      for (int q = 0; q < 4; ++q) ring[x % PF][q] = nxt[q];
  }
  if (STM == 0) {
    // 3 x 324 output chunks of 16 B
    for (int j = lane; j < nst * 324; j += 64) {
      const int js = j / 324, jc = j % 324;
      stg<true>((u32x4 *)(out + (s0 + js) * STRIDE + OUT_OFF + jc * 16), acc[j & 3] ^ u32x4{(uint32_t)j, 0, 0, 0});
    }
  } else {
    const int sl = lane / 21, c = lane % 21;
    if (sl >= nst) return;
    const int p = c == 20 ? SUB - 8 : c * 8;
    uint8_t *o = out + (s0 + sl) * STRIDE + OUT_OFF + p;
#pragma unroll
    for (int r = 0; r < M; ++r)
#pragma unroll
      for (int y = 0; y < 8; ++y) {
        const u32x4 a = acc[(r + y) & 3];
        __builtin_nontemporal_store(u32x2{a.x ^ (uint32_t)r, a.y ^ (uint32_t)y}, (u32x2 *)(o + r * BYTES + y * SUB));
      }
  }
}

// ---------------------------------------------------------------- transposed through LDS
// Bytes [S, S + 8) of the 16 little-endian bytes (a, b); S a compile-time constant.
template <int S>
__device__ __forceinline__ u32x2 funnel(u32x2 a, u32x2 b) {
  if constexpr (S == 0) return a;
  else if constexpr (S == 4) return u32x2{a.y, b.x};
  else if constexpr (S < 4) return u32x2{__builtin_amdgcn_alignbyte(a.y, a.x, S), __builtin_amdgcn_alignbyte(b.x, a.y, S)};
  else return u32x2{__builtin_amdgcn_alignbyte(b.x, a.y, S - 4), __builtin_amdgcn_alignbyte(b.y, b.x, S - 4)};
}
// Lane (sl, c) of a 3-stripe slot image (stripe sl at sl * 1296, chunk j at 16 j): bytes
// [8c, 8c + 8) of sub-block B, from the two naturally aligned words around them.  c = 20 holds
// bytes 160..161 (the rest is the next sub-block's, never stored).
// SPLIT: the second word's address is opaque to the compiler (lo8 = lo + 8), so the pair stays
// two ds_read_b64 (2 LDS cycles each) instead of being merged into one ds_read2_b64 (8).
template <int B, bool SPLIT>
__device__ __forceinline__ u32x2 slot_word(const uint8_t *slot, int lo, int lo8) {
  constexpr int S = (2 * B) & 7;
  const u32x2 *p = (const u32x2 *)(slot + lo + B * SUB - S);
  if constexpr (S == 0) return p[0];
  else if constexpr (SPLIT) return funnel<S>(p[0], *(const u32x2 *)(slot + lo8 + B * SUB - S));
  else return funnel<S>(p[0], p[1]);
}
template <bool SPLIT>
__device__ __forceinline__ void slot_col(u32x2 (&d)[8], const uint8_t *slot, int lo, int lo8) {
  d[0] = slot_word<0, SPLIT>(slot, lo, lo8); d[1] = slot_word<1, SPLIT>(slot, lo, lo8);
  d[2] = slot_word<2, SPLIT>(slot, lo, lo8); d[3] = slot_word<3, SPLIT>(slot, lo, lo8);
  d[4] = slot_word<4, SPLIT>(slot, lo, lo8); d[5] = slot_word<5, SPLIT>(slot, lo, lo8);
  d[6] = slot_word<6, SPLIT>(slot, lo, lo8); d[7] = slot_word<7, SPLIT>(slot, lo, lo8);
}
__device__ __forceinline__ uint32_t dpp_row_shr1(uint32_t v) {  // lane i <- lane i - 1 within a row of 16
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, false);
}
// Outputs as the product stores them: lane c < 20 at [8c, 8c + 8) of every sub-row, lane 20
// at [154, 162): lane 19's bytes 154..159 (same DPP row for the lanes 19/20, 40/41, 61/62 of
// the three stripes) and its own 160..161.
__device__ __forceinline__ void store_rows(uint8_t *out, long long s, int c, u32x2 (&acc)[M][8]) {
  const bool last = c == 20;
  uint8_t *o = out + s * STRIDE + OUT_OFF + (last ? SUB - 8 : 8 * c);
#pragma unroll
  for (int r = 0; r < M; ++r)
#pragma unroll
    for (int y = 0; y < 8; ++y) {
      const u32x2 v = acc[r][y] ^ u32x2{(uint32_t)r * 0x01010101u, (uint32_t)r * 0x01010101u};
      const u32x2 pv = u32x2{dpp_row_shr1(v.x), dpp_row_shr1(v.y)};
      const u32x2 f = funnel<2>(pv, v);
      __builtin_nontemporal_store(last ? f : v, (u32x2 *)(o + r * BYTES + y * SUB));
    }
}

template <int PF, bool SPLIT>
__global__ void __launch_bounds__(256) lds_t(const uint8_t *__restrict__ in, uint8_t *__restrict__ out, int stripes) {
  __shared__ __attribute__((aligned(16))) uint8_t slots[4][4096];
  const long long wave = (xcd_block() * 256 + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  uint8_t *slot = slots[threadIdx.x >> 6];
  const long long s0 = (long long)__builtin_amdgcn_readfirstlane((int)wave) * 3;
  if (s0 >= stripes) return;
  const int nst = (int)(stripes - s0 < 3 ? stripes - s0 : 3);
  flat_src S;
  S.init(in, s0, nst, lane);
  const int sl = lane / 21, c = lane % 21;
  const int lo = (sl < 3 ? sl : 2) * BYTES + 8 * c;
  int lo8 = lo + 8;
  asm volatile("" : "+v"(lo8));
  u32x2 acc[M][8];
#pragma unroll
  for (int r = 0; r < M; ++r)
#pragma unroll
    for (int y = 0; y < 8; ++y) acc[r][y] = u32x2{0, 0};
  u32x4 ring[PF][4];
#pragma unroll
  for (int q = 0; q < PF; ++q) S.load(ring[q], q);
#pragma unroll
  for (int x = 0; x < K; ++x) {
    u32x4 nxt[4];
    if (x + PF < K) S.load(nxt, x + PF);
#pragma unroll
    for (int q = 0; q < 3; ++q) *(u32x4 *)(slot + 1024 * q + 16 * lane) = ring[x % PF][q];
    if (lane < 243 - 192) *(u32x4 *)(slot + 3072 + 16 * lane) = ring[x % PF][3];
    u32x2 d[8];
    slot_col<SPLIT>(d, slot, lo, lo8);
#pragma unroll
    for (int r = 0; r < M; ++r)
#pragma unroll
      for (int y = 0; y < 8; ++y) acc[r][y] ^= d[(y + r + x) & 7];
#pragma unroll
    for (int r = 0; r < M; ++r)
#pragma unroll
      for (int y = 0; y < 8; ++y) asm volatile("" : "+v"(acc[r][y]));
    if (x + PF < K)
#pragma unroll
      for (int q = 0; q < 4; ++q) ring[x % PF][q] = nxt[q];
  }
  if (sl >= nst) return;
  store_rows(out, s0 + sl, c, acc);
}

// LDS-DMA ring: D slots of 4 KiB per wave; column x lands in slot x % D by 4
// global_load_lds_dwordx4 (lane l of piece q writes 16 B at 1024 q + 16 l).
template <int D, bool SPLIT>
__global__ void __launch_bounds__(256) lds_d(const uint8_t *__restrict__ in, uint8_t *__restrict__ out, int stripes) {
  __shared__ __attribute__((aligned(16))) uint8_t ring[4][D][4096];
  const long long wave = (xcd_block() * 256 + threadIdx.x) >> 6;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const long long s0 = (long long)__builtin_amdgcn_readfirstlane((int)wave) * 3;
  if (s0 >= stripes) return;
  const int nst = (int)(stripes - s0 < 3 ? stripes - s0 : 3);
  const uint8_t *src[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int j = std::min(64 * q + lane, nst * 81 - 1);
    src[q] = in + (s0 + j / 81) * STRIDE + (j % 81) * 16;
  }
  auto issue = [&](int x, int sl) {
#pragma unroll
    for (int q = 0; q < 4; ++q)
      __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void *)(src[q] + x * BYTES),
                                       (__attribute__((address_space(3))) void *)&ring[w][sl][q * 1024], 16, 0, 2);
  };
#pragma unroll
  for (int q = 0; q < D; ++q) issue(q, q);
  const int sl = lane / 21, c = lane % 21;
  const int lo = (sl < 3 ? sl : 2) * BYTES + 8 * c;
  int lo8 = lo + 8;
  asm volatile("" : "+v"(lo8));
  u32x2 acc[M][8];
#pragma unroll
  for (int r = 0; r < M; ++r)
#pragma unroll
    for (int y = 0; y < 8; ++y) acc[r][y] = u32x2{0, 0};
#pragma unroll
  for (int x = 0; x < K; ++x) {
    const int left = std::min(D - 1, K - 1 - x);  // columns issued after x (4 DMA each)
    // vmcnt(4 * left): bits [3:0] and [15:14]; expcnt and lgkmcnt at their maxima.
    if (left >= 5) __builtin_amdgcn_s_waitcnt((20 & 15) | ((20 >> 4) << 14) | (7 << 4) | (15 << 8));
    else if (left == 4) __builtin_amdgcn_s_waitcnt((16 & 15) | ((16 >> 4) << 14) | (7 << 4) | (15 << 8));
    else if (left == 3) __builtin_amdgcn_s_waitcnt(12 | (7 << 4) | (15 << 8));
    else if (left == 2) __builtin_amdgcn_s_waitcnt(8 | (7 << 4) | (15 << 8));
    else if (left == 1) __builtin_amdgcn_s_waitcnt(4 | (7 << 4) | (15 << 8));
    else __builtin_amdgcn_s_waitcnt(0 | (7 << 4) | (15 << 8));
    asm volatile("" ::: "memory");  // no LDS read moves above the wait
    u32x2 d[8];
    slot_col<SPLIT>(d, ring[w][x % D], lo, lo8);
#pragma unroll
    for (int r = 0; r < M; ++r)
#pragma unroll
      for (int y = 0; y < 8; ++y) acc[r][y] ^= d[(y + r + x) & 7];
#pragma unroll
    for (int r = 0; r < M; ++r)
#pragma unroll
      for (int y = 0; y < 8; ++y) asm volatile("" : "+v"(acc[r][y]));
    if (x + D < K) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      issue(x + D, x % D);
    }
  }
  if (sl >= nst) return;
  store_rows(out, s0 + sl, c, acc);
}


// ---------------------------------------------------------------- wave lifetime
// mixL: each wave reads U consecutive 29-KiB units (one contiguous region of U x 29 KiB), G
// loads in flight (a sliding window), and writes U x 4 KiB: the mix's geometry with the
// lifetime of a wave that codes 3 stripes (U = 4 ~ 3 x 37.6 KB).
template <int U, int G>
__global__ void __launch_bounds__(256) mixL(const uint8_t *__restrict__ in, uint8_t *__restrict__ out, long long waves) {
  const long long wave = (xcd_block() * 256 + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (wave >= waves) return;
  const u32x4 *src = (const u32x4 *)(in + wave * U * K * 1024) + lane;
  u32x4 *dst = (u32x4 *)(out + wave * U * M * 1024) + lane;
  u32x4 ring[G], acc[M] = {};
#pragma unroll
  for (int g = 0; g < G; ++g) ring[g] = ldg<true>(src + g * 64);
#pragma unroll
  for (int i = 0; i < U * K; ++i) {
    const u32x4 v = ring[i % G];
    if (i + G < U * K) ring[i % G] = ldg<true>(src + (i + G) * 64);
    acc[i % M] ^= v;
    if (i % K == K - 1) {
#pragma unroll
      for (int r = 0; r < M; ++r) {
        stg<true>(dst + ((i / K) * M + r) * 64, acc[r]);
        acc[r] = u32x4{0, 0, 0, 0};
      }
    }
  }
}

// flat1: one stripe per wave, column x = 81 aligned 16-B chunks (2 dwordx4: 64 + 17 lanes),
// PF columns in flight, light compute, flat stores (5184 B = 324 chunks).
template <int PF>
__global__ void __launch_bounds__(256) flat1(const uint8_t *__restrict__ in, uint8_t *__restrict__ out, int stripes) {
  const long long wave = (xcd_block() * 256 + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (wave >= stripes) return;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *)(in + wave * STRIDE), 0, (int)STRIDE, 0x00020000);
  const int v0 = lane * 16, v1 = lane < 17 ? (64 + lane) * 16 : (int)0x80000000;
  u32x4 ring[PF][2], acc[2] = {};
#pragma unroll
  for (int q = 0; q < PF; ++q) {
    ring[q][0] = __builtin_amdgcn_raw_buffer_load_b128(rs, v0, q * BYTES, 2);
    ring[q][1] = __builtin_amdgcn_raw_buffer_load_b128(rs, v1, q * BYTES, 2);
  }
#pragma unroll
  for (int x = 0; x < K; ++x) {
    u32x4 n0 = {}, n1 = {};
    if (x + PF < K) {
      n0 = __builtin_amdgcn_raw_buffer_load_b128(rs, v0, (x + PF) * BYTES, 2);
      n1 = __builtin_amdgcn_raw_buffer_load_b128(rs, v1, (x + PF) * BYTES, 2);
    }
    acc[0] ^= ring[x % PF][0];
    acc[1] ^= ring[x % PF][1];
    asm volatile("" : "+v"(acc[0]), "+v"(acc[1]));
    if (x + PF < K) {
      ring[x % PF][0] = n0;
      ring[x % PF][1] = n1;
    }
  }
  for (int j = lane; j < 324; j += 64)
    stg<true>((u32x4 *)(out + wave * STRIDE + OUT_OFF + j * 16), acc[j & 1] ^ u32x4{(uint32_t)j, 0, 0, 0});
}


// ---------------------------------------------------------------- stream geometry
// geo: unit u = L bytes at in + u * US, read as ceil(L / 1024) 1-KiB chunks (16 B per lane,
// the last chunk partial); a wave owns S units and reads chunk j of each of them back to back
// (S streams), G chunk steps in flight; then writes OB bytes per unit at out + u * OS + OO.
template <int S, int G, int NC>
__global__ void __launch_bounds__(256) geo(const uint8_t *__restrict__ in, uint8_t *__restrict__ out, int units, int L,
                                           long long US, long long OS, long long OO, int OB) {
  const long long wave = (xcd_block() * 256 + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  const long long u0 = wave * S;
  if (u0 >= units) return;
  __amdgpu_buffer_rsrc_t rs[S];
#pragma unroll
  for (int s = 0; s < S; ++s)
    rs[s] = __builtin_amdgcn_make_buffer_rsrc((void *)(in + (u0 + s < units ? u0 + s : u0) * US), 0, L, 0x00020000);
  u32x4 ring[G][S], acc[4] = {};
  const int lo = lane * 16;
#pragma unroll
  for (int j = 0; j < G && j < NC; ++j)
#pragma unroll
    for (int s = 0; s < S; ++s) ring[j][s] = __builtin_amdgcn_raw_buffer_load_b128(rs[s], lo, j * 1024, 2);
#pragma unroll
  for (int j = 0; j < NC; ++j) {
#pragma unroll
    for (int s = 0; s < S; ++s) acc[(j + s) & 3] ^= ring[j % G][s];
#pragma unroll
    for (int q = 0; q < 4; ++q) asm volatile("" : "+v"(acc[q]));
    if (j + G < NC)
#pragma unroll
      for (int s = 0; s < S; ++s) ring[j % G][s] = __builtin_amdgcn_raw_buffer_load_b128(rs[s], lo, (j + G) * 1024, 2);
  }
#pragma unroll
  for (int s = 0; s < S; ++s) {
    if (u0 + s >= units) break;
    uint8_t *o = out + (u0 + s) * OS + OO;
    for (int c = lane; c * 16 < OB; c += 64) stg<true>((u32x4 *)(o + c * 16), acc[c & 3] ^ u32x4{(uint32_t)c, 0, 0, 0});
  }
}


// ---------------------------------------------------------------- one stripe per wave, dword lanes
// w4d: lane c < 41 owns bytes [4c, 4c + 4) of every sub-block of the wave's ONE stripe (the
// last lane [158, 162)); 8 buffer_load_dword per column (2-byte aligned for odd sub-blocks),
// PF columns in flight; 4 x 8 dword accumulators.  The wave streams one contiguous 37.6 KB
// region (the geometry of flat1 / mixL U=1) at the price of 41 of 64 lanes.
template <int PF>
__global__ void __launch_bounds__(256) w4d(const uint8_t *__restrict__ in, uint8_t *__restrict__ out, int stripes) {
  const long long wave = (xcd_block() * 256 + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (wave >= stripes) return;
  const bool act = lane < 41;
  const int p = lane >= 40 ? SUB - 4 : 4 * lane;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *)(in + wave * STRIDE), 0, (int)STRIDE, 0x00020000);
  const int lb = act ? p : (int)0x80000000;
  uint32_t acc[M][8];
#pragma unroll
  for (int r = 0; r < M; ++r)
#pragma unroll
    for (int y = 0; y < 8; ++y) acc[r][y] = 0;
  uint32_t ring[PF][8];
#pragma unroll
  for (int q = 0; q < PF; ++q)
#pragma unroll
    for (int b = 0; b < 8; ++b) ring[q][b] = __builtin_amdgcn_raw_buffer_load_b32(rs, lb + b * SUB, q * BYTES, 2);
#pragma unroll
  for (int x = 0; x < K; ++x) {
    uint32_t nxt[8];
    if (x + PF < K)
#pragma unroll
      for (int b = 0; b < 8; ++b) nxt[b] = __builtin_amdgcn_raw_buffer_load_b32(rs, lb + b * SUB, (x + PF) * BYTES, 2);
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
  if (!act) return;
  uint8_t *o = out + wave * STRIDE + OUT_OFF + p;
#pragma unroll
  for (int r = 0; r < M; ++r)
#pragma unroll
    for (int y = 0; y < 8; ++y)
      __builtin_nontemporal_store(acc[r][y] ^ ((uint32_t)r * 0x01010101u), (uint32_t *)(o + r * BYTES + y * SUB));
}


// geop: geo S=1 G=37 on the stripe layout with the stores' cache-policy bits AUX (gfx950
// buffer instructions: bit 0 sc0, bit 1 nt, bit 4 sc1) and the loads' LAUX.
template <int SAUX, int LAUX>
__global__ void __launch_bounds__(256) geop(const uint8_t *__restrict__ in, uint8_t *__restrict__ out, int units,
                                            long long OS, long long OO) {
  constexpr int NC = 37;
  const long long u = (xcd_block() * 256 + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (u >= units) return;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *)(in + u * STRIDE), 0, (int)STRIDE, 0x00020000);
  u32x4 ring[NC], acc[4] = {};
#pragma unroll
  for (int j = 0; j < NC; ++j) ring[j] = __builtin_amdgcn_raw_buffer_load_b128(rs, lane * 16, j * 1024, LAUX);
#pragma unroll
  for (int j = 0; j < NC; ++j) acc[j & 3] ^= ring[j];
  const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc((void *)(out + u * OS + OO), 0, M * BYTES, 0x00020000);
#pragma unroll
  for (int c = 0; c < 6; ++c)
    if (c * 64 + lane < M * BYTES / 16)
      __builtin_amdgcn_raw_buffer_store_b128(acc[c & 3] ^ u32x4{(uint32_t)c, 0, 0, 0}, ro, (c * 64 + lane) * 16, 0, SAUX);
}

// ---------------------------------------------------------------- driver
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
static void rep(const char *name, float ms) {
  printf("%-40s %8.4f ms %8.1f GB/s input %8.1f GB/s total\n", name, ms, IN_BYTES / (ms * 1e-3) / 1e9,
         (IN_BYTES + OUT_BYTES) / (ms * 1e-3) / 1e9);
  fflush(stdout);
}

int main(int argc, char **argv) {
  uint8_t *din, *dout;
  CK(hipMalloc(&din, 2 * IN_BYTES + 4096));   // 2x: the "scale" group codes twice the stripes
  CK(hipMalloc(&dout, 2 * IN_BYTES + 4096));
  {  // random-looking input (the clock depends on the data, MI355X_MICROARCH.md DVFS)
    std::vector<uint8_t> rnd(1 << 20);
    uint64_t z = 0x9E3779B97F4A7C15ull;
    for (size_t i = 0; i < rnd.size(); ++i) {
      z += 0x9E3779B97F4A7C15ull;
      uint64_t t = z;
      t = (t ^ (t >> 30)) * 0xBF58476D1CE4E5B9ull;
      t = (t ^ (t >> 27)) * 0x94D049BB133111EBull;
      rnd[i] = (uint8_t)(t >> 56);
    }
    for (long long i = 0; i < 2 * IN_BYTES; i += 1 << 20)
      CK(hipMemcpy(din + i, rnd.data(), std::min<long long>(1 << 20, 2 * IN_BYTES - i), hipMemcpyHostToDevice));
  }
  CK(hipMemset(dout, 0, 2 * IN_BYTES + 4096));
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  printf("# ubench_r5: %d CUs; input %.3f GB, output %.3f GB (k29/m4/1296 x 65536)\n", cus, IN_BYTES / 1e9, OUT_BYTES / 1e9);
  const int g3 = (int)((STRIPES + 2) / 3 + 3) / 4;  // one wave per 3 stripes, 4 waves per block

  if (want(argc, argv, "copy")) {
    const long long n = IN_BYTES / 2 / 16, bytes = n * 16 * 2;
    const float ms = timeit([&] { copy_os<<<(int)((n + 255) / 256), 256>>>((const u32x4 *)din, (u32x4 *)dout, n); });
    printf("%-40s %8.4f ms %8.1f GB/s moved (read + write)\n", "copy float4 one-shot nt", ms, bytes / (ms * 1e-3) / 1e9);
  }
  if (want(argc, argv, "read")) {
    const long long n = IN_BYTES / 16;
    const float ms = timeit([&] { read_os<<<(int)((n + 2047) / 2048), 256>>>((const u32x4 *)din, (u32x4 *)dout, n); });
    printf("%-40s %8.4f ms %8.1f GB/s read\n", "read dwordx4 one-shot nt U=8", ms, IN_BYTES / (ms * 1e-3) / 1e9);
  }
  if (want(argc, argv, "mix")) {
#define MIXV(LB, SEG, BS)                                                                                \
    {                                                                                                    \
      const long long units = IN_BYTES / (K * SEG);                                                      \
      constexpr int U = 64 / (SEG / LB);                                                                 \
      const long long waves = (units + U - 1) / U;                                                       \
      const int g = (int)((waves * 64 + BS - 1) / BS);                                                   \
      char nm[64]; snprintf(nm, 64, "mix LB=%d SEG=%d BS=%d", LB, SEG, BS);                               \
      rep(nm, timeit([&] { mixv<LB, SEG, BS><<<g, BS>>>(din, dout, units); }));                          \
    }
    MIXV(16, 1024, 256) MIXV(16, 1024, 512) MIXV(16, 1024, 128) MIXV(8, 512, 256) MIXV(16, 512, 256)
    MIXV(16, 256, 256) MIXV(8, 256, 256) MIXV(16, 128, 256) MIXV(8, 128, 256)
    {
      const long long units = IN_BYTES / (K * 1024);
      const int g = (int)((units / 2 + 3) / 4);
      rep("mix2 H=8 (stores between loads)", timeit([&] { mix2<8><<<g, 256>>>(din, dout, units); }));
      rep("mix2 H=16 (stores between loads)", timeit([&] { mix2<16><<<g, 256>>>(din, dout, units); }));
    }
  }
  if (want(argc, argv, "enc")) {
    rep("enc product pattern PF=3", timeit([&] { enc_pat<3><<<g3, 256>>>(din, dout, (int)STRIPES); }));
    rep("enc product pattern PF=2", timeit([&] { enc_pat<2><<<g3, 256>>>(din, dout, (int)STRIPES); }));
  }
  if (want(argc, argv, "flat")) {
    rep("flat PF=2 flat stores", timeit([&] { flat_pat<2, 0><<<g3, 256>>>(din, dout, (int)STRIPES); }));
    rep("flat PF=3 flat stores", timeit([&] { flat_pat<3, 0><<<g3, 256>>>(din, dout, (int)STRIPES); }));
    rep("flat PF=4 flat stores", timeit([&] { flat_pat<4, 0><<<g3, 256>>>(din, dout, (int)STRIPES); }));
    rep("flat PF=6 flat stores", timeit([&] { flat_pat<6, 0><<<g3, 256>>>(din, dout, (int)STRIPES); }));
    rep("flat PF=3 product stores", timeit([&] { flat_pat<3, 1><<<g3, 256>>>(din, dout, (int)STRIPES); }));
    rep("flat PF=4 product stores", timeit([&] { flat_pat<4, 1><<<g3, 256>>>(din, dout, (int)STRIPES); }));
  }
  if (want(argc, argv, "ldst") || want(argc, argv, "ldsd")) {
    const size_t ob = (size_t)(STRIPES * STRIDE);
    std::vector<uint8_t> ref(ob), got(ob);
    auto check = [&](const char *name) {
      CK(hipDeviceSynchronize());
      CK(hipMemcpy(got.data(), dout, ob, hipMemcpyDeviceToHost));
      size_t bad = 0;
      for (long long s = 0; s < STRIPES; ++s)
        for (long long i = 0; i < M * BYTES; ++i) bad += got[s * STRIDE + OUT_OFF + i] != ref[s * STRIDE + OUT_OFF + i];
      printf("check %-34s %zu of %lld output bytes differ from enc\n", name, bad, (long long)OUT_BYTES);
      fflush(stdout);
    };
    CK(hipMemset(dout, 0, ob));
    enc_pat<3><<<g3, 256>>>(din, dout, (int)STRIPES);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(ref.data(), dout, ob, hipMemcpyDeviceToHost));
    if (want(argc, argv, "ldst")) {
#define LDST(PF, SP)                                                                                      \
      {                                                                                                   \
        char nm[64]; snprintf(nm, 64, "ldst PF=%d split=%d", PF, SP);                                      \
        CK(hipMemset(dout, 0, ob));                                                                       \
        lds_t<PF, SP><<<g3, 256>>>(din, dout, (int)STRIPES);                                              \
        check(nm);                                                                                        \
        rep(nm, timeit([&] { lds_t<PF, SP><<<g3, 256>>>(din, dout, (int)STRIPES); }));                    \
      }
      LDST(2, false) LDST(3, false) LDST(4, false) LDST(2, true) LDST(3, true) LDST(4, true)
    }
    if (want(argc, argv, "ldsd")) {
#define LDSD(D, SP)                                                                                       \
      {                                                                                                   \
        char nm[64]; snprintf(nm, 64, "ldsd D=%d split=%d", D, SP);                                        \
        CK(hipMemset(dout, 0, ob));                                                                       \
        lds_d<D, SP><<<g3, 256>>>(din, dout, (int)STRIPES);                                               \
        check(nm);                                                                                        \
        rep(nm, timeit([&] { lds_d<D, SP><<<g3, 256>>>(din, dout, (int)STRIPES); }));                     \
      }
      LDSD(2, false) LDSD(3, false) LDSD(4, false) LDSD(3, true) LDSD(4, true)
    }
  }

  if (want(argc, argv, "life")) {
#define MIXL(U, G)                                                                                        \
    {                                                                                                     \
      const long long waves = IN_BYTES / (K * 1024 * U);                                                  \
      char nm[64]; snprintf(nm, 64, "mixL U=%d G=%d (%lld waves)", U, G, waves);                         \
      rep(nm, timeit([&] { mixL<U, G><<<(int)((waves + 3) / 4), 256>>>(din, dout, waves); }));            \
    }
    MIXL(1, 4) MIXL(1, 16) MIXL(1, 29) MIXL(2, 8) MIXL(4, 4) MIXL(4, 8) MIXL(4, 16) MIXL(8, 16)
  }
  if (want(argc, argv, "flat1")) {
    const int g1 = (int)((STRIPES + 3) / 4);
    rep("flat1 PF=4 (1 stripe per wave)", timeit([&] { flat1<4><<<g1, 256>>>(din, dout, (int)STRIPES); }));
    rep("flat1 PF=8 (1 stripe per wave)", timeit([&] { flat1<8><<<g1, 256>>>(din, dout, (int)STRIPES); }));
    rep("flat1 PF=16 (1 stripe per wave)", timeit([&] { flat1<16><<<g1, 256>>>(din, dout, (int)STRIPES); }));
    rep("flat1 PF=29 (1 stripe per wave)", timeit([&] { flat1<29><<<g1, 256>>>(din, dout, (int)STRIPES); }));
  }
  if (want(argc, argv, "scale")) {
    // the same kernels on twice the stripes: a fixed (ramp / tail) cost shows as time(2N) < 2 time(N)
    const int g6 = (int)((2 * STRIPES + 2) / 3 + 3) / 4;
    const float a = timeit([&] { flat_pat<4, 0><<<g3, 256>>>(din, dout, (int)STRIPES); });
    const float b = timeit([&] { flat_pat<4, 0><<<g6, 256>>>(din, dout, (int)(2 * STRIPES)); });
    printf("scale flat PF=4: N %.4f ms, 2N %.4f ms, 2N - N %.4f ms (fixed part %.4f ms)\n", a, b, b - a, 2 * a - b);
    const float c = timeit([&] { enc_pat<3><<<g3, 256>>>(din, dout, (int)STRIPES); });
    const float d = timeit([&] { enc_pat<3><<<g6, 256>>>(din, dout, (int)(2 * STRIPES)); });
    printf("scale enc PF=3: N %.4f ms, 2N %.4f ms, 2N - N %.4f ms (fixed part %.4f ms)\n", c, d, d - c, 2 * c - d);
    const long long u1 = IN_BYTES / (K * 512);
    const float e = timeit([&] { mixv<8, 512, 256><<<(int)((u1 + 3) / 4), 256>>>(din, dout, u1); });
    const float f = timeit([&] { mixv<8, 512, 256><<<(int)((2 * u1 + 3) / 4), 256>>>(din, dout, 2 * u1); });
    printf("scale mix LB=8: N %.4f ms, 2N %.4f ms, 2N - N %.4f ms (fixed part %.4f ms)\n", e, f, f - e, 2 * e - f);
    fflush(stdout);
  }

  if (want(argc, argv, "geo")) {
    auto run = [&](const char *nm, auto kern, int S, int L, long long US, long long OS, long long OO, int OB) {
      const int units = (int)STRIPES;
      const long long waves = (units + S - 1) / S;
      const float ms = timeit([&] { kern<<<(int)((waves + 3) / 4), 256>>>(din, dout, units, L, US, OS, OO, OB); });
      const double inb = (double)units * L, outb = (double)units * OB;
      printf("%-52s %8.4f ms %8.1f GB/s input (%.3f GB in)\n", nm, ms, inb / (ms * 1e-3) / 1e9, inb / 1e9);
      fflush(stdout);
    };
    const long long L29 = 29 * 1024, LS = STRIDE;  // 29 KiB units; 37584-B stripes
    run("geo S=1 G=29 L=29K US=29K out compact 4K", geo<1, 29, 29>, 1, L29, L29, 4096, 0, 4096);
    run("geo S=1 G=4  L=29K US=29K out compact 4K", geo<1, 4, 29>, 1, L29, L29, 4096, 0, 4096);
    run("geo S=1 G=37 L=stripe US=stripe out bench", geo<1, 37, 37>, 1, LS, LS, LS, OUT_OFF, M * BYTES);
    run("geo S=1 G=37 L=stripe US=stripe out compact", geo<1, 37, 37>, 1, LS, LS, M * BYTES, 0, M * BYTES);
    run("geo S=1 G=37 L=stripe US=37632(128B) out bench", geo<1, 37, 37>, 1, LS, 37632, 37632, OUT_OFF, M * BYTES);
    run("geo S=1 G=37 L=stripe US=37888(1K) out bench", geo<1, 37, 37>, 1, LS, 37888, 37888, OUT_OFF, M * BYTES);
    run("geo S=1 G=16 L=stripe US=stripe out bench", geo<1, 16, 37>, 1, LS, LS, LS, OUT_OFF, M * BYTES);
    run("geo S=1 G=8  L=stripe US=stripe out bench", geo<1, 8, 37>, 1, LS, LS, LS, OUT_OFF, M * BYTES);
    run("geo S=1 G=4  L=stripe US=stripe out bench", geo<1, 4, 37>, 1, LS, LS, LS, OUT_OFF, M * BYTES);
    run("geo S=3 G=4  L=stripe US=stripe out bench", geo<3, 4, 37>, 3, LS, LS, LS, OUT_OFF, M * BYTES);
    run("geo S=3 G=8  L=stripe US=stripe out bench", geo<3, 8, 37>, 3, LS, LS, LS, OUT_OFF, M * BYTES);
    run("geo S=2 G=8  L=stripe US=stripe out bench", geo<2, 8, 37>, 2, LS, LS, LS, OUT_OFF, M * BYTES);
    run("geo S=1 G=37 L=stripe US=stripe no output", geo<1, 37, 37>, 1, LS, LS, LS, 0, 0);
    run("geo S=1 G=4  L=stripe US=stripe no output", geo<1, 4, 37>, 1, LS, LS, LS, 0, 0);
    run("geo S=3 G=4  L=stripe US=stripe no output", geo<3, 4, 37>, 3, LS, LS, LS, 0, 0);
  }

  if (want(argc, argv, "w4")) {
    const size_t ob = (size_t)(STRIPES * STRIDE);
    std::vector<uint8_t> ref(ob), got(ob);
    CK(hipMemset(dout, 0, ob));
    enc_pat<3><<<g3, 256>>>(din, dout, (int)STRIPES);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(ref.data(), dout, ob, hipMemcpyDeviceToHost));
    auto check = [&](const char *name) {
      CK(hipDeviceSynchronize());
      CK(hipMemcpy(got.data(), dout, ob, hipMemcpyDeviceToHost));
      size_t bad = 0;
      for (long long s = 0; s < STRIPES; ++s)
        for (long long i = 0; i < M * BYTES; ++i) bad += got[s * STRIDE + OUT_OFF + i] != ref[s * STRIDE + OUT_OFF + i];
      printf("check %-34s %zu of %lld output bytes differ from enc\n", name, bad, (long long)OUT_BYTES);
      fflush(stdout);
    };
    const int g1 = (int)((STRIPES + 3) / 4);
#define W4(KER, P)                                                                                        \
    {                                                                                                     \
      char nm[64]; snprintf(nm, 64, #KER " %d (1 stripe per wave, dword lanes)", P);                        \
      CK(hipMemset(dout, 0, ob));                                                                         \
      KER<P><<<g1, 256>>>(din, dout, (int)STRIPES);                                                       \
      check(nm);                                                                                          \
      rep(nm, timeit([&] { KER<P><<<g1, 256>>>(din, dout, (int)STRIPES); }));                             \
    }
    W4(w4d, 3) W4(w4d, 6) W4(w4d, 10)
  }

  if (want(argc, argv, "pol")) {
    auto run = [&](const char *nm, auto kern, long long OS, long long OO) {
      const int units = (int)STRIPES;
      const float ms = timeit([&] { kern<<<(units + 3) / 4, 256>>>(din, dout, units, OS, OO); });
      printf("%-52s %8.4f ms %8.1f GB/s input\n", nm, ms, IN_BYTES / (ms * 1e-3) / 1e9);
      fflush(stdout);
    };
#define POL(S, L)                                                                                       \
    run("pol stores aux=" #S " loads aux=" #L " out bench", geop<S, L>, STRIDE, OUT_OFF);                \
    run("pol stores aux=" #S " loads aux=" #L " out compact", geop<S, L>, M * BYTES, 0);
    POL(2, 2) POL(0, 2) POL(1, 2) POL(3, 2) POL(16, 2) POL(17, 2) POL(18, 2) POL(19, 2) POL(2, 0) POL(0, 0)
  }
  CK(hipGetLastError());
  CK(hipDeviceSynchronize());
  return 0;
}
