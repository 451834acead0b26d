// jit_codec.hip -- run-time specialised encode/decode kernels (compiled by hiprtc).
//
// The host (jit.cpp) prepends a configuration header defining LH_K, LH_M, LH_BYTES,
// LH_SUB, LH_W, LH_NCH, LH_SPW and the constant expanded generator LH_BM[m][k][8] (row
// y of element G[r][x] is G[r][x] * 2^y, the bit-sliced form of cauchy_256.cpp:1553-1587),
// then compiles this file for gfx950.  Because every bit of the generator is a compile-
// time constant, the XOR network below unrolls into exactly the XORs the bit-matrix
// needs (the reference executes the same network one 162-byte memcpy-sized XOR at a time
// through gf256_add_mem); hipcc fuses chains into v_xor3 / v_bitop3.
//
// Mapping ("small sub-block" regime, nch = ceil(sub / W) <= 64 lanes per stripe):
//   a wave holds LH_SPW whole stripes; lane = (stripe in wave, column chunk c).  A lane
//   owns bytes [p, p + W) of every sub-block of its stripe (p = c * W, the last chunk
//   shifted back to sub - W so it never leaves the sub-block; the overlap is recomputed
//   identically by both lanes of the same wave).  Stripes never straddle waves, so the
//   in-place decode is race free: every load of a wave completes before its first store.
//
// This file is also compiled by hipcc at build time with the defaults below as a
// syntax check; the product only uses the hiprtc-compiled code objects.

#ifndef LH_K
#define LH_K 4
#define LH_M 2
#define LH_BYTES 64
#define LH_SUB 8
#define LH_W 8
#define LH_NCH 1
#define LH_SPW 64
#define LH_WPS 0
static constexpr unsigned char LH_BM[LH_M][LH_K][8] = {
    {{1, 2, 4, 8, 16, 32, 64, 128}, {1, 2, 4, 8, 16, 32, 64, 128},
     {1, 2, 4, 8, 16, 32, 64, 128}, {1, 2, 4, 8, 16, 32, 64, 128}},
    {{1, 2, 4, 8, 16, 32, 64, 128}, {2, 4, 8, 16, 32, 64, 128, 135},
     {3, 6, 12, 24, 48, 96, 192, 7}, {4, 8, 16, 32, 64, 128, 135, 137}}};
#define LH_G_INIT {{1, 1, 1, 1}, {1, 2, 3, 4}}
#include <hip/hip_runtime.h>
#endif

#define LH_NW ((LH_W + 3) / 4)


struct lh_word {
    unsigned int v[LH_NW];
};

#ifndef LH_NT
#define LH_NT 1  // non-temporal (streaming) loads and stores: +3% on k29/m4 (tools/tune.py)
#endif
typedef unsigned int lh_u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned int lh_u32x3 __attribute__((ext_vector_type(3)));
typedef unsigned int lh_u32x4 __attribute__((ext_vector_type(4)));

// W-byte loads/stores at the sub-block's natural (often 2-byte) alignment: gfx950
// serves unaligned global accesses in hardware.
__device__ __forceinline__ lh_word lh_load(const unsigned char *p) {
    lh_word w;
#if LH_NT && LH_W == 16
    const lh_u32x4 v = __builtin_nontemporal_load((const lh_u32x4 *)p);
    w.v[0] = v.x; w.v[1] = v.y; w.v[2] = v.z; w.v[3] = v.w;
#elif LH_NT && LH_W == 12
    const lh_u32x3 v = __builtin_nontemporal_load((const lh_u32x3 *)p);
    w.v[0] = v.x; w.v[1] = v.y; w.v[2] = v.z;
#elif LH_NT && LH_W == 8
    const lh_u32x2 v = __builtin_nontemporal_load((const lh_u32x2 *)p);
    w.v[0] = v.x; w.v[1] = v.y;
#elif LH_NT && LH_W == 4
    w.v[0] = __builtin_nontemporal_load((const unsigned int *)p);
#else
#pragma unroll
    for (int i = 0; i < LH_NW; ++i) w.v[i] = 0;
    __builtin_memcpy(&w.v[0], p, LH_W);
#endif
    return w;
}

#ifndef LH_NT_ST
#define LH_NT_ST LH_NT  // non-temporal stores (tools/tune.py knob, independent of the loads)
#endif
__device__ __forceinline__ void lh_store(unsigned char *p, const lh_word &w) {
#if LH_NT_ST && LH_W == 16
    lh_u32x4 v = {w.v[0], w.v[1], w.v[2], w.v[3]};
    __builtin_nontemporal_store(v, (lh_u32x4 *)p);
#elif LH_NT_ST && LH_W == 12
    lh_u32x3 v = {w.v[0], w.v[1], w.v[2]};
    __builtin_nontemporal_store(v, (lh_u32x3 *)p);
#elif LH_NT_ST && LH_W == 8
    lh_u32x2 v = {w.v[0], w.v[1]};
    __builtin_nontemporal_store(v, (lh_u32x2 *)p);
#elif LH_NT_ST && LH_W == 4
    __builtin_nontemporal_store(w.v[0], (unsigned int *)p);
#else
    __builtin_memcpy(p, &w.v[0], LH_W);
#endif
}

__device__ __forceinline__ void lh_xor(lh_word &a, const lh_word &b) {
#pragma unroll
    for (int i = 0; i < LH_NW; ++i) a.v[i] ^= b.v[i];
}

// gfx950 v_bitop3_b32: any 3-input boolean function in one VALU op.  The LUT index is
// (src0 << 2) | (src1 << 1) | src2: 0x96 = src0 ^ src1 ^ src2, 0x78 = src0 ^ (src1 & src2).
// hipcc does not fuse XOR chains on its own (it emits one v_xor_b32 per term).
__device__ __forceinline__ unsigned int lh_x3(unsigned int a, unsigned int b, unsigned int c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}
__device__ __forceinline__ unsigned int lh_xand(unsigned int a, unsigned int b, unsigned int c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x78);
}
__device__ __forceinline__ void lh_xor2(lh_word &a, const lh_word &b, const lh_word &c) {
#pragma unroll
    for (int i = 0; i < LH_NW; ++i) a.v[i] = lh_x3(a.v[i], b.v[i], c.v[i]);
}

// a ^= sum of d[b] over the set bits b of S, the terms taken two at a time (XOR3).
template <unsigned S, int B = 0, int P = -1>
struct lh_net {
    __device__ __forceinline__ static void run(lh_word &a, const lh_word (&d)[8]) {
        if constexpr (B == 8) {
            if constexpr (P >= 0) lh_xor(a, d[P]);
        } else if constexpr (((S >> B) & 1u) == 0) {
            lh_net<S, B + 1, P>::run(a, d);
        } else if constexpr (P < 0) {
            lh_net<S, B + 1, B>::run(a, d);
        } else {
            lh_xor2(a, d[P], d[B]);
            lh_net<S, B + 1, -1>::run(a, d);
        }
    }
};

// acc[r][y] ^= sum_x B(G[r][x]) d_x, one column x at a time, all constants.
template <int X, int I = 0>
struct lh_col_net {
    __device__ __forceinline__ static void run(lh_word (&acc)[LH_M][8], const lh_word (&d)[8]) {
        if constexpr (I < LH_M * 8) {
            lh_net<LH_BM[I / 8][X][I % 8]>::run(acc[I / 8][I % 8], d);
            lh_col_net<X, I + 1>::run(acc, d);
        }
    }
};
template <int X>
__device__ __forceinline__ void lh_column(lh_word (&acc)[LH_M][8], const lh_word (&d)[8]) {
    lh_col_net<X>::run(acc, d);
}

struct lh_lane {
    long long stripe;
    int p;
    bool active;
};

// Waves needed for a batch; kernels loop over them (grid-stride) so the host may launch
// either one wave per work item or a persistent grid.
__device__ __forceinline__ long long lh_total_waves(int stripes) {
#if LH_NCH <= 64
    return ((long long)stripes + LH_SPW - 1) / LH_SPW;
#else
    return (long long)stripes * LH_WPS;
#endif
}

__device__ __forceinline__ lh_lane lh_map_lane(int stripes, long long wave) {
    const int lane = threadIdx.x & 63;
    lh_lane l;
#if LH_NCH <= 64
    // LH_SPW whole stripes per wave.
    const int sl = lane / LH_NCH;
    const int c = lane - sl * LH_NCH;
    l.stripe = wave * LH_SPW + sl;
    l.active = (sl < LH_SPW) && (l.stripe < stripes);
#else
    // LH_WPS waves per stripe (the host only picks this when LH_SUB % LH_W == 0 for
    // decode, so no chunk overlaps another wave's bytes).
    const long long c0 = (wave % LH_WPS) * 64 + lane;
    const int c = (int)c0;
    l.stripe = wave / LH_WPS;
    l.active = (c0 < LH_NCH) && (l.stripe < stripes);
#endif
    l.p = (c == LH_NCH - 1) ? (LH_SUB - LH_W) : c * LH_W;
    return l;
}

// LH_XCD = 1: the dispatcher deals blocks round-robin over the 8 XCDs; renumber them so
// each XCD (own L2) walks one contiguous run of stripes.  k29/m4 encode 0.569 -> 0.556 ms,
// decode 0.625 -> 0.620 ms (profiles/r1c_tune_xcd2.txt, six interleaved rounds).
#ifndef LH_XCD
#define LH_XCD 1
#endif
__device__ __forceinline__ long long lh_block_id() {
#if LH_XCD
    const unsigned b = blockIdx.x, per = gridDim.x / 8;
    return b < per * 8 ? (long long)(b % 8) * per + b / 8 : (long long)b;
#else
    return blockIdx.x;
#endif
}

#define LH_WAVE_LOOP(stripes)                                                                   \
    const long long lh_nw = lh_total_waves(stripes);                                           \
    const long long lh_ws = (long long)gridDim.x * (blockDim.x >> 6);                          \
    for (long long lh_w = (lh_block_id() * blockDim.x + threadIdx.x) >> 6; lh_w < lh_nw;       \
         lh_w += lh_ws)

// Keeps the accumulators in registers between columns: stops the compiler from
// re-associating XORs across columns (which lengthens live ranges past the register file).
__device__ __forceinline__ void lh_opaque(lh_word (&acc)[LH_M][8]) {
#pragma unroll
    for (int r = 0; r < LH_M; ++r)
#pragma unroll
        for (int y = 0; y < 8; ++y)
#pragma unroll
            for (int i = 0; i < LH_NW; ++i) asm volatile("" : "+v"(acc[r][y].v[i]));
}

// Column loop, unrolled at compile time, with the next LH_PF columns' loads in flight
// while column X is combined.
#ifndef LH_PF
#define LH_PF 3  // columns in flight ahead of the one being combined
#endif
template <int X>
struct lh_unroll_encode {
    __device__ __forceinline__ static void run(lh_word (&acc)[LH_M][8], lh_word (&ring)[LH_PF][8],
                                               const unsigned char *base) {
        if (X + LH_PF < LH_K) {
            lh_word nxt[8];
#pragma unroll
            for (int b = 0; b < 8; ++b) nxt[b] = lh_load(base + (long long)(X + LH_PF) * LH_BYTES + b * LH_SUB);
            lh_column<X>(acc, ring[X % LH_PF]);
            lh_opaque(acc);
#pragma unroll
            for (int b = 0; b < 8; ++b) ring[X % LH_PF][b] = nxt[b];
        } else {
            lh_column<X>(acc, ring[X % LH_PF]);
            lh_opaque(acc);
        }
        lh_unroll_encode<X + 1>::run(acc, ring, base);
    }
};
template <>
struct lh_unroll_encode<LH_K> {
    __device__ __forceinline__ static void run(lh_word (&)[LH_M][8], lh_word (&)[LH_PF][8], const unsigned char *) {}
};

// LH_PAIR = 1: columns combined two at a time, so the odd terms left by one column's
// XOR3 pairing pair up with the next column's (row 0 of the generator is all ones: its
// eight single terms per column halve).  Needs LH_PF >= 2.
#ifndef LH_PAIR
#define LH_PAIR 0
#endif
template <unsigned S0, unsigned S1, int B = 0, int P = -1>
struct lh_net2 {
    __device__ __forceinline__ static void run(lh_word &a, const lh_word (&d0)[8], const lh_word (&d1)[8]) {
        constexpr unsigned S = S0 | (S1 << 8);
        if constexpr (B == 16) {
            if constexpr (P >= 0) lh_xor(a, P < 8 ? d0[P & 7] : d1[P & 7]);
        } else if constexpr (((S >> B) & 1u) == 0) {
            lh_net2<S0, S1, B + 1, P>::run(a, d0, d1);
        } else if constexpr (P < 0) {
            lh_net2<S0, S1, B + 1, B>::run(a, d0, d1);
        } else {
            lh_xor2(a, P < 8 ? d0[P & 7] : d1[P & 7], B < 8 ? d0[B & 7] : d1[B & 7]);
            lh_net2<S0, S1, B + 1, -1>::run(a, d0, d1);
        }
    }
};
template <int X, int I = 0>
struct lh_col_net2 {
    __device__ __forceinline__ static void run(lh_word (&acc)[LH_M][8], const lh_word (&d0)[8], const lh_word (&d1)[8]) {
        if constexpr (I < LH_M * 8) {
            lh_net2<LH_BM[I / 8][X][I % 8], LH_BM[I / 8][X + 1][I % 8]>::run(acc[I / 8][I % 8], d0, d1);
            lh_col_net2<X, I + 1>::run(acc, d0, d1);
        }
    }
};
template <int X>
struct lh_unroll_encode2 {
    __device__ __forceinline__ static void run(lh_word (&acc)[LH_M][8], lh_word (&ring)[LH_PF][8],
                                               const unsigned char *base) {
        if constexpr (X + 1 >= LH_K) {
            lh_unroll_encode<X>::run(acc, ring, base);  // odd column count: last one alone
        } else {
            lh_word n0[8], n1[8];
            if constexpr (X + LH_PF < LH_K) {
#pragma unroll
                for (int b = 0; b < 8; ++b) n0[b] = lh_load(base + (long long)(X + LH_PF) * LH_BYTES + b * LH_SUB);
            }
            if constexpr (X + 1 + LH_PF < LH_K) {
#pragma unroll
                for (int b = 0; b < 8; ++b) n1[b] = lh_load(base + (long long)(X + 1 + LH_PF) * LH_BYTES + b * LH_SUB);
            }
            lh_col_net2<X>::run(acc, ring[X % LH_PF], ring[(X + 1) % LH_PF]);
            lh_opaque(acc);
            if constexpr (X + LH_PF < LH_K) {
#pragma unroll
                for (int b = 0; b < 8; ++b) ring[X % LH_PF][b] = n0[b];
            }
            if constexpr (X + 1 + LH_PF < LH_K) {
#pragma unroll
                for (int b = 0; b < 8; ++b) ring[(X + 1) % LH_PF][b] = n1[b];
            }
            lh_unroll_encode2<X + 2>::run(acc, ring, base);
        }
    }
};
template <>
struct lh_unroll_encode2<LH_K> {
    __device__ __forceinline__ static void run(lh_word (&)[LH_M][8], lh_word (&)[LH_PF][8], const unsigned char *) {}
};

__device__ __forceinline__ void lh_encode_wave(long long wave, const unsigned char *__restrict__ in,
                                               long long in_stride, unsigned char *__restrict__ out,
                                               long long out_stride, int stripes) {
    const lh_lane l = lh_map_lane(stripes, wave);
    if (!l.active) return;
    lh_word acc[LH_M][8];
#pragma unroll
    for (int r = 0; r < LH_M; ++r)
#pragma unroll
        for (int y = 0; y < 8; ++y)
#pragma unroll
            for (int i = 0; i < LH_NW; ++i) acc[r][y].v[i] = 0;
    const unsigned char *base = in + l.stripe * in_stride + l.p;
    lh_word ring[LH_PF][8];
#pragma unroll
    for (int q = 0; q < LH_PF; ++q)
        if (q < LH_K)
#pragma unroll
            for (int b = 0; b < 8; ++b) ring[q][b] = lh_load(base + (long long)q * LH_BYTES + b * LH_SUB);
#if LH_PAIR && LH_PF >= 2
    lh_unroll_encode2<0>::run(acc, ring, base);
#else
    lh_unroll_encode<0>::run(acc, ring, base);
#endif
    unsigned char *o = out + l.stripe * out_stride + l.p;
#pragma unroll
    for (int r = 0; r < LH_M; ++r)
#pragma unroll
        for (int y = 0; y < 8; ++y) lh_store(o + (long long)r * LH_BYTES + y * LH_SUB, acc[r][y]);
}

#if 1
// recovery[s][r] = sum_x B(G[r][x]) data[s][x]   (cauchy_256_encode for m > 1, valid k, m)
#ifndef LH_ENC_LB
#define LH_ENC_LB 1  // min waves per SIMD the register allocator must allow (tools/tune.py)
#endif
extern "C" __global__ void __launch_bounds__(256, LH_ENC_LB)
lh_jit_encode(const unsigned char *__restrict__ in, long long in_stride,
              unsigned char *__restrict__ out, long long out_stride, int stripes) {
    LH_WAVE_LOOP(stripes) { lh_encode_wave(lh_w, in, in_stride, out, out_stride, stripes); }
}
#endif


// ------------------------------------------------------------------------ decode
// Plan record layout: kernels.hpp PlanView (e at [0], out_slot at [16], then src_slot[k],
// rec_slot[m], coef[e_max][m]).  e_max = min(k, m) for m > 1.
#define LH_EMAX (LH_K < LH_M ? LH_K : LH_M)
#define LH_P_OUT 16
#define LH_P_SRC (16 + LH_EMAX)
#define LH_P_REC (16 + LH_EMAX + LH_K)
#define LH_P_COEF (16 + LH_EMAX + LH_K + LH_M)

// Plan bytes are fetched as packed dwords (one load per 4 slots) and unpacked with
// constant shifts where used, so per-column slot indices cost no registers up front.
#define LH_NSRC ((LH_K + 3) / 4)
#define LH_NREC ((LH_M + 3) / 4)
#define LH_NCOEF ((LH_EMAX * LH_M + 3) / 4)
#define LH_NOUT ((LH_EMAX + 3) / 4)

__device__ __forceinline__ unsigned int lh_load32(const unsigned char *p) {
    unsigned int w;
    __builtin_memcpy(&w, p, 4);
    return w;
}

template <int N>
__device__ __forceinline__ void lh_load_packed(unsigned int (&w)[N], const unsigned char *p) {
#pragma unroll
    for (int j = 0; j < N; ++j) w[j] = lh_load32(p + 4 * j);
}

#define LH_BYTE(w, idx) (((w)[(idx) / 4] >> (8 * ((idx) % 4))) & 0xFFu)

__device__ __forceinline__ const unsigned char *lh_slot_ptr(unsigned int slot, const unsigned char *base,
                                                            const unsigned char *zero) {
    return (slot == 0xFFu) ? zero : base + (long long)slot * LH_BYTES;
}

// Phase A streams LH_K data columns (erased ones read the zero page) and then the LH_M
// recovery rows (absent ones read the zero page) through one prefetch ring, so the
// recovery loads are in flight while the last data columns combine.
#ifndef LH_COLS_PROBE
#define LH_COLS_PROBE 0  // timing probe only: phase A streams the k data columns, no recovery rows
#endif
#define LH_DCOLS (LH_COLS_PROBE ? LH_K : LH_K + LH_M)
#ifndef LH_PF_DEC
#define LH_PF_DEC 1  // decode prefetch depth (tools/tune.py, fused plan: 1 > 2 > 3)
#endif
#ifndef LH_REFILL
#define LH_REFILL 0  // decode ring: refill a slot right after its column is combined (no staging copy)
#endif
#ifndef LH_PREP_FIRST
#define LH_PREP_FIRST 0  // fused decode: solve the plan before (1) or while (0) the first columns load
#endif

template <int X>
__device__ __forceinline__ const unsigned char *lh_dcol_src(const unsigned int (&srcw)[LH_NSRC],
                                                            const unsigned int (&recw)[LH_NREC],
                                                            const unsigned char *base, const unsigned char *zero) {
    if (X < LH_K) return lh_slot_ptr(LH_BYTE(srcw, X < LH_K ? X : 0), base, zero);
    return lh_slot_ptr(LH_BYTE(recw, X >= LH_K ? X - LH_K : 0), base, zero);
}

// Column load of the decode ring.  LH_ZSKIP: lanes whose column is absent (erased
// original, missing recovery row) do not load the zero page, they zero their words under
// the exec mask, so no wave-instruction fetches from one hot 1.3-KB page.
#ifndef LH_NZ
#define LH_NZ 1  // zero pages the stripes spread over (the host allocates 64): one hot page
                 // concentrates every erased column's reads on a few L2 channels
#endif
#ifndef LH_ZSKIP
#define LH_ZSKIP 0  // measured equal (0.6255 vs 0.6212 ms, k29/m4): the zero page stays L2-resident
#endif
__device__ __forceinline__ void lh_load_col(lh_word (&d)[8], const unsigned char *src, const unsigned char *zero) {
#if LH_ZSKIP
    if (src != zero) {
#pragma unroll
        for (int b = 0; b < 8; ++b) d[b] = lh_load(src + b * LH_SUB);
    } else {
#pragma unroll
        for (int b = 0; b < 8; ++b)
#pragma unroll
            for (int i = 0; i < LH_NW; ++i) d[b].v[i] = 0;
    }
#else
#pragma unroll
    for (int b = 0; b < 8; ++b) d[b] = lh_load(src + b * LH_SUB);
#endif
}

template <int X>
__device__ __forceinline__ void lh_dcombine(lh_word (&acc)[LH_M][8], const lh_word (&d)[8]) {
    if (X < LH_K) {
        lh_column<(X < LH_K ? X : 0)>(acc, d);
    } else {
#pragma unroll
        for (int y = 0; y < 8; ++y) lh_xor(acc[X >= LH_K ? X - LH_K : 0][y], d[y]);
    }
}

template <int X>
struct lh_unroll_decode {
    __device__ __forceinline__ static void run(lh_word (&acc)[LH_M][8], lh_word (&ring)[LH_PF_DEC][8],
                                               const unsigned char *base, const unsigned char *zero,
                                               const unsigned int (&srcw)[LH_NSRC], const unsigned int (&recw)[LH_NREC]) {
        if (X + LH_PF_DEC < LH_DCOLS) {
#if LH_REFILL
            // Combine column X, then refill its ring slot with column X + PF: no staging
            // copy (16 VGPRs fewer), and the refill's address passes through an empty asm
            // after the accumulator pin, so the load cannot be hoisted above the combine.
            lh_dcombine<X>(acc, ring[X % LH_PF_DEC]);
            lh_opaque(acc);
            constexpr int XN = X + LH_PF_DEC < LH_DCOLS ? X + LH_PF_DEC : 0;
            // (an integer passes through the asm: a pointer would lose its global address
            // space and turn the loads into flat loads)
            unsigned int w = XN < LH_K ? srcw[(XN < LH_K ? XN : 0) / 4] : recw[(XN >= LH_K ? XN - LH_K : 0) / 4];
            asm volatile("" : "+v"(w));
            const unsigned int slot = (w >> (8 * ((XN < LH_K ? XN : XN - LH_K) % 4))) & 0xFFu;
            lh_load_col(ring[X % LH_PF_DEC], lh_slot_ptr(slot, base, zero), zero);
#else
            const unsigned char *src = lh_dcol_src<(X + LH_PF_DEC < LH_DCOLS ? X + LH_PF_DEC : 0)>(srcw, recw, base, zero);
            lh_word nxt[8];
            lh_load_col(nxt, src, zero);
            lh_dcombine<X>(acc, ring[X % LH_PF_DEC]);
            lh_opaque(acc);
#pragma unroll
            for (int b = 0; b < 8; ++b) ring[X % LH_PF_DEC][b] = nxt[b];
#endif
        } else {
            lh_dcombine<X>(acc, ring[X % LH_PF_DEC]);
            lh_opaque(acc);
        }
        lh_unroll_decode<X + 1>::run(acc, ring, base, zero, srcw, recw);
    }
};
template <>
struct lh_unroll_decode<LH_DCOLS> {
    __device__ __forceinline__ static void run(lh_word (&)[LH_M][8], lh_word (&)[LH_PF_DEC][8], const unsigned char *,
                                               const unsigned char *, const unsigned int (&)[LH_NSRC],
                                               const unsigned int (&)[LH_NREC]) {}
};

// Per-stripe decode plan in registers: e, packed src/rec slot maps, coef, out slots.
struct lh_plan_regs {
    int e;
    unsigned int srcw[LH_NSRC], recw[LH_NREC], coefw[LH_NCOEF], outw[LH_NOUT];
};

struct lh_no_prep {
    __device__ __forceinline__ void operator()(lh_plan_regs &) const {}
};

// In-place erasure decode.  Phase A: V_r = R_r + sum_{x present} B(G[r][x]) D_x for every
// recovery row r.  Phase B: D_{E_i} = sum_r B(coef[i][r]) V_r with the per-stripe inverse,
// by Horner over the coefficient bits: B(c) v = B(2)(...B(2)(c_7 v)...) + c_0 v.
// `prep` runs while the first columns are in flight (the fused kernel solves its plan there).
// Decode pieces.  Ring issue: the first LH_PF_DEC columns of a stripe group.
__device__ __forceinline__ void lh_dec_issue(lh_word (&ring)[LH_PF_DEC][8], const lh_plan_regs &pr,
                                             const unsigned char *base, const unsigned char *zero) {
#pragma unroll
    for (int q = 0; q < LH_PF_DEC; ++q) {
        const unsigned char *src = (q == 0) ? lh_dcol_src<0>(pr.srcw, pr.recw, base, zero)
                                 : (q == 1) ? lh_dcol_src<1>(pr.srcw, pr.recw, base, zero)
                                 : (q == 2) ? lh_dcol_src<2>(pr.srcw, pr.recw, base, zero)
                                            : lh_dcol_src<3>(pr.srcw, pr.recw, base, zero);
        lh_load_col(ring[q], src, zero);
    }
}

// Phase A: V_r = R_r + sum_{x present} B(G[r][x]) D_x for every recovery row r, streaming
// the ring (already issued) through all k + m columns.
__device__ __forceinline__ void lh_dec_phase_a(lh_word (&v)[LH_M][8], lh_word (&ring)[LH_PF_DEC][8],
                                               const lh_plan_regs &pr, const unsigned char *base,
                                               const unsigned char *zero) {
#pragma unroll
    for (int r = 0; r < LH_M; ++r)
#pragma unroll
        for (int y = 0; y < 8; ++y)
#pragma unroll
            for (int i = 0; i < LH_NW; ++i) v[r][y].v[i] = 0;
    lh_unroll_decode<0>::run(v, ring, base, zero, pr.srcw, pr.recw);
}

// Phase B: D_{E_i} = sum_r B(coef[i][r]) V_r with the per-stripe inverse, by Horner over
// the coefficient bits: B(c) v = B(2)(...B(2)(c_7 v)...) + c_0 v, one v_bitop3 masked XOR
// per (row, bit, sub-row); the recovered blocks go to the plan's output slots.
#ifndef LH_PB_PROBE
#define LH_PB_PROBE 0  // timing probe only (tools/tune.py): V_i stored as output i, no phase-B XORs
#endif
__device__ __forceinline__ void lh_dec_phase_b(const lh_word (&v)[LH_M][8], const lh_plan_regs &pr,
                                               unsigned char *base) {
    const int e = pr.e;
#if LH_PB_PROBE
#pragma unroll
    for (int i = 0; i < LH_EMAX; ++i)
        if (i < e)
#pragma unroll
            for (int y = 0; y < 8; ++y) lh_store(base + (long long)LH_BYTE(pr.outw, i) * LH_BYTES + y * LH_SUB, v[i][y]);
    return;
#endif
    const unsigned int(&coefw)[LH_NCOEF] = pr.coefw;
    const unsigned int(&outw)[LH_NOUT] = pr.outw;
#pragma unroll
    for (int i = 0; i < LH_EMAX; ++i) {
        if (i < e) {
            lh_word o[8];
#pragma unroll
            for (int y = 0; y < 8; ++y)
#pragma unroll
                for (int q = 0; q < LH_NW; ++q) o[y].v[q] = 0;
#pragma unroll
            for (int t = 7; t >= 0; --t) {
                if (t != 7) {  // o = B(2) o
                    lh_word t7;
#pragma unroll
                    for (int q = 0; q < LH_NW; ++q) t7.v[q] = lh_x3(o[0].v[q], o[1].v[q], o[2].v[q]) ^ o[7].v[q];
#pragma unroll
                    for (int y = 0; y < 7; ++y) o[y] = o[y + 1];
                    o[7] = t7;
                }
#pragma unroll
                for (int r = 0; r < LH_M; ++r) {
                    const int idx = i * LH_M + r;
                    // 0 or ~0: bit t of coef[i][r], sign-extended (one v_bfe_i32)
                    const unsigned int mask =
                        (unsigned int)((int)(coefw[idx / 4] << (31 - (8 * (idx % 4) + t))) >> 31);
#pragma unroll
                    for (int y = 0; y < 8; ++y)
#pragma unroll
                        for (int q = 0; q < LH_NW; ++q) o[y].v[q] = lh_xand(o[y].v[q], v[r][y].v[q], mask);
                }
#pragma unroll
                for (int y = 0; y < 8; ++y)
#pragma unroll
                    for (int q = 0; q < LH_NW; ++q) asm volatile("" : "+v"(o[y].v[q]));
            }
            unsigned char *dst = base + (long long)LH_BYTE(outw, i) * LH_BYTES;
#pragma unroll
            for (int y = 0; y < 8; ++y) lh_store(dst + y * LH_SUB, o[y]);
        }
    }
}

// In-place erasure decode of one stripe group: ring issue, `prep` (the fused kernel
// solves its plan there, while the first columns are in flight), phase A, phase B.
template <class PREP>
__device__ __forceinline__ void lh_decode_body(const lh_lane &l, unsigned char *__restrict__ blocks,
                                               long long stripe_stride, lh_plan_regs &pr,
                                               const unsigned char *__restrict__ zero_page, const PREP &prep) {
    unsigned char *base = blocks + l.stripe * stripe_stride + l.p;
    const unsigned char *zero = zero_page + (l.stripe % LH_NZ) * LH_BYTES + l.p;
    lh_word v[LH_M][8];
    {
#if LH_PREP_FIRST
        prep(pr);  // solve before the first loads: the ring is not live across the solve
#endif
        lh_word ring[LH_PF_DEC][8];
        lh_dec_issue(ring, pr, base, zero);
#if !LH_PREP_FIRST
        prep(pr);
#endif
        lh_dec_phase_a(v, ring, pr, base, zero);
    }
    lh_dec_phase_b(v, pr, base);
}

__device__ __forceinline__ void lh_decode_wave(long long wave, unsigned char *__restrict__ blocks,
                                               long long stripe_stride, const unsigned char *__restrict__ plan,
                                               long long plan_stride, const unsigned char *__restrict__ zero_page,
                                               int stripes) {
    const lh_lane l = lh_map_lane(stripes, wave);
    if (!l.active) return;
    const unsigned char *pl = plan + l.stripe * plan_stride;
    lh_plan_regs pr;
    pr.e = pl[0];
    if (pr.e == 0) return;
    lh_load_packed(pr.srcw, pl + LH_P_SRC);
    lh_load_packed(pr.recw, pl + LH_P_REC);
    lh_load_packed(pr.coefw, pl + LH_P_COEF);
    lh_load_packed(pr.outw, pl + LH_P_OUT);
    lh_decode_body(l, blocks, stripe_stride, pr, zero_page, lh_no_prep());
}

#if 1
extern "C" __global__ void __launch_bounds__(256)
lh_jit_decode(unsigned char *__restrict__ blocks, long long stripe_stride,
              const unsigned char *__restrict__ plan, long long plan_stride,
              const unsigned char *__restrict__ zero_page, int stripes) {
    LH_WAVE_LOOP(stripes) { lh_decode_wave(lh_w, blocks, stripe_stride, plan, plan_stride, zero_page, stripes); }
}
#endif

// ------------------------------------------------------------ fused decode planner
// LH_EMAX <= 4: the plan is computed inside the decode kernel, per lane (every lane of a
// stripe derives the same plan; the wave is SIMD, so redundancy costs no extra time).
// Slot maps are built in a per-wave LDS scratch; the e x e inverse runs in registers with
// GF(256) log/exp tables in LDS.  Semantics follow lh_plan_small_kernel (kernels.hip):
// reference sort_blocks (cauchy_256.cpp:538-570) and generate_bitmatrix's row
// assignment (:786); duplicate / out-of-range rows mark the stripe invalid, untouched.
#if LH_EMAX <= 4 && LH_NCH <= 64 && LH_K <= 64
#define LH_FUSED 1
static constexpr unsigned char LH_GRAW[LH_M][LH_K] = LH_G_INIT;
#define LH_P4(n) (((n) + 3) / 4 * 4)
#define LH_SR (2 * LH_P4(LH_K) + LH_P4(LH_M))  // per-stripe scratch: rows | src map | rec map
#define LH_NRW ((LH_K + LH_NCH - 1) / LH_NCH)    // Block.row bytes per lane
// Lanes of one stripe as a ballot mask (LH_NCH may be 64: a 64-bit shift by 64 is UB).
#define LH_STRIPE_LANES (LH_NCH >= 64 ? ~0ull : ((1ull << (LH_NCH & 63)) - 1))

// The lane's Block.row bytes (slots c, c + LH_NCH, ...), loaded ahead of the plan.
__device__ __forceinline__ void lh_fused_rows(const lh_lane &l, int c, const unsigned char *__restrict__ rows,
                                              unsigned int (&rowv)[LH_NRW]) {
    const unsigned char *grow = rows + l.stripe * LH_K;
#pragma unroll
    for (int t = 0; t < LH_NRW; ++t) {
        const int i = c + t * LH_NCH;
        rowv[t] = (l.active && i < LH_K) ? (unsigned int)grow[i] : 0u;
    }
}

__device__ __forceinline__ unsigned int lh_gmul(const unsigned char *gexp, const short *glog, unsigned int a,
                                                unsigned int b) {
    return (a && b) ? gexp[glog[a] + glog[b]] : 0u;
}

// Returns false when the stripe has nothing to do (no erasure or invalid rows).
// Part 2 of the fused plan (run while the first columns load): invert, pack, rewrite rows.
struct lh_fused_solve {
    unsigned int rs[LH_EMAX], rr[LH_EMAX], er[LH_EMAX];
    unsigned char *grow;
    const unsigned char *gexp;
    const short *glog;
    int c;
    __device__ __forceinline__ void operator()(lh_plan_regs &pr) const;
};

// Part 1: slot maps, validity and the erasure / recovery lists.  Returns false when the
// stripe has nothing to do (no erasure or invalid rows).
__device__ __forceinline__ bool lh_fused_plan(const lh_lane &l, int c, int sl, unsigned char *scr,
                                              const unsigned int (&rowv)[LH_NRW],
                                              unsigned char *__restrict__ rows, signed char *__restrict__ status,
                                              lh_fused_solve &sv, lh_plan_regs &pr) {
    unsigned char *lrows = scr;
    unsigned char *lsrc = scr + LH_P4(LH_K);
    unsigned char *lrec = lsrc + LH_P4(LH_K);
    unsigned char *grow = rows + l.stripe * LH_K;
    // Clear the maps (0xFF = absent), then every lane records the rows of its slots.
    for (int q = c; q < (LH_P4(LH_K) + LH_P4(LH_M)) / 4; q += LH_NCH) ((unsigned int *)lsrc)[q] = 0xFFFFFFFFu;
    bool bad = false;
#pragma unroll
    for (int t = 0; t < LH_NRW; ++t) {
        const int i = c + t * LH_NCH;
        if (i >= LH_K) continue;
        const unsigned int r = rowv[t];
        lrows[i] = (unsigned char)r;
        if (r < LH_K) lsrc[r] = (unsigned char)i;
        else if (r < LH_K + LH_M) lrec[r - LH_K] = (unsigned char)i;
        else bad = true;
    }
    for (int i = c; i < LH_K; i += LH_NCH) {  // a repeated row leaves another slot in the map
        const unsigned int r = lrows[i];
        if (r < LH_K + LH_M && (r < LH_K ? lsrc[r] : lrec[r - LH_K]) != i) bad = true;
    }
    const unsigned long long lanes_bad = __ballot(bad);
    const unsigned long long my = LH_STRIPE_LANES << (sl * LH_NCH);
    const bool invalid = (lanes_bad & my) != 0;
    // Recovery slots in array order and missing originals ascending, as per-stripe bit
    // masks gathered with wave ballots (slot/row i = c + t * LH_NCH), then unpacked by
    // lowest-set-bit extraction.
    unsigned long long rcvmask = 0, ermask = 0;
#pragma unroll
    for (int t = 0; t < (LH_K + LH_NCH - 1) / LH_NCH; ++t) {
        const int i = c + t * LH_NCH;
        const bool isrcv = (i < LH_K) && (lrows[i] >= LH_K);
        const bool iser = (i < LH_K) && (lsrc[i] == 0xFF);
        const unsigned long long lanes = LH_STRIPE_LANES;
        rcvmask |= ((__ballot(isrcv) >> (sl * LH_NCH)) & lanes) << (t * LH_NCH);
        ermask |= ((__ballot(iser) >> (sl * LH_NCH)) & lanes) << (t * LH_NCH);
    }
    const int nr = __builtin_popcountll(rcvmask);
    unsigned int rs[LH_EMAX], rr[LH_EMAX], er[LH_EMAX];
#pragma unroll
    for (int q = 0; q < LH_EMAX; ++q) {
        rs[q] = rcvmask ? (unsigned int)__builtin_ctzll(rcvmask) : 0u;
        er[q] = ermask ? (unsigned int)__builtin_ctzll(ermask) : 0u;
        rcvmask &= rcvmask - 1;
        ermask &= ermask - 1;
        rr[q] = (unsigned int)lrows[rs[q]] - LH_K;
    }
    if (invalid || nr > LH_EMAX) {
        if (c == 0 && status) status[l.stripe] = -1;
        return false;
    }
    if (c == 0 && status) status[l.stripe] = 0;
    pr.e = nr;
    if (nr == 0) return false;
#pragma unroll
    for (int q = 0; q < LH_EMAX; ++q) { sv.rs[q] = rs[q]; sv.rr[q] = rr[q]; sv.er[q] = er[q]; }
    sv.grow = grow;
    sv.c = c;
#pragma unroll
    for (int q = 0; q < LH_NSRC; ++q) pr.srcw[q] = ((const unsigned int *)lsrc)[q];
#pragma unroll
    for (int q = 0; q < LH_NREC; ++q) pr.recw[q] = ((const unsigned int *)lrec)[q];
    return true;
}

__device__ __forceinline__ void lh_fused_solve::operator()(lh_plan_regs &pr) const {
    const int nr = pr.e;
    // Gauss-Jordan on A = G[rr_i][er_j], identity-padded to LH_EMAX.
    unsigned int A[LH_EMAX][LH_EMAX], I[LH_EMAX][LH_EMAX];
#pragma unroll
    for (int i = 0; i < LH_EMAX; ++i)
#pragma unroll
        for (int j = 0; j < LH_EMAX; ++j) {
            A[i][j] = (i < nr && j < nr) ? LH_GRAW[rr[i]][er[j]] : (i == j ? 1u : 0u);
            I[i][j] = (i == j) ? 1u : 0u;
        }
#pragma unroll
    for (int cc = 0; cc < LH_EMAX; ++cc) {
        int p = cc;
#pragma unroll
        for (int r = LH_EMAX - 1; r >= cc; --r) if (A[r][cc]) p = r;
#pragma unroll
        for (int r = cc + 1; r < LH_EMAX; ++r)
            if (r == p)
#pragma unroll
                for (int j = 0; j < LH_EMAX; ++j) {
                    unsigned int t = A[cc][j]; A[cc][j] = A[r][j]; A[r][j] = t;
                    t = I[cc][j]; I[cc][j] = I[r][j]; I[r][j] = t;
                }
        const unsigned int inv = gexp[255 - glog[A[cc][cc]]];
#pragma unroll
        for (int j = 0; j < LH_EMAX; ++j) { A[cc][j] = lh_gmul(gexp, glog, A[cc][j], inv); I[cc][j] = lh_gmul(gexp, glog, I[cc][j], inv); }
#pragma unroll
        for (int r = 0; r < LH_EMAX; ++r) {
            if (r == cc) continue;
            const unsigned int f = A[r][cc];
#pragma unroll
            for (int j = 0; j < LH_EMAX; ++j) { A[r][j] ^= lh_gmul(gexp, glog, f, A[cc][j]); I[r][j] ^= lh_gmul(gexp, glog, f, I[cc][j]); }
        }
    }
    // Pack: coef[i][r] = Ainv[i][j] for the recovery row r = rr[j]; out slots; maps.
#pragma unroll
    for (int q = 0; q < LH_NCOEF; ++q) pr.coefw[q] = 0;
#pragma unroll
    for (int i = 0; i < LH_EMAX; ++i)
#pragma unroll
        for (int r = 0; r < LH_M; ++r) {
            unsigned int v = 0;
#pragma unroll
            for (int j = 0; j < LH_EMAX; ++j) if (j < nr && rr[j] == (unsigned int)r) v = I[i][j];
            const int idx = i * LH_M + r;
            pr.coefw[idx / 4] |= v << (8 * (idx % 4));
        }
#pragma unroll
    for (int q = 0; q < LH_NOUT; ++q) pr.outw[q] = 0;
#pragma unroll
    for (int i = 0; i < LH_EMAX; ++i) pr.outw[i / 4] |= rs[i] << (8 * (i % 4));
    // Recovery slot i takes missing row er[i] (reference generate_bitmatrix, :786).
    if (c == 0)
#pragma unroll
        for (int i = 0; i < LH_EMAX; ++i) if (i < nr) grow[rs[i]] = (unsigned char)er[i];
    // Materialise the packed plan here, so the solve's matrices die before phase A: left
    // alone, the compiler sinks the packing into phase B and keeps the e x e inverse and
    // the row lists live across all k + m columns (k29/m4: 218 -> 158 VGPRs, 2 -> 3
    // waves/SIMD).
#pragma unroll
    for (int q = 0; q < LH_NCOEF; ++q) asm volatile("" : "+v"(pr.coefw[q]));
#pragma unroll
    for (int q = 0; q < LH_NOUT; ++q) asm volatile("" : "+v"(pr.outw[q]));
}

#ifndef LH_ROWPF
#define LH_ROWPF 0  // fused decode: prefetch the next grid-stride group's rows (persistent grids)
#endif
#ifndef LH_DEC_LB
#define LH_DEC_LB 1  // min waves per SIMD the register allocator must allow (tools/tune.py)
#endif
extern "C" __global__ void __launch_bounds__(256, LH_DEC_LB)
lh_jit_decode_fused(unsigned char *__restrict__ blocks, long long stripe_stride, unsigned char *__restrict__ rows,
                    signed char *__restrict__ status, const unsigned char *__restrict__ zero_page,
                    const unsigned char *__restrict__ gf_exp, const short *__restrict__ gf_log, int stripes) {
    __shared__ unsigned char gexp[512];
    __shared__ short glog[256];
    __shared__ __attribute__((aligned(16))) unsigned char scratch[4][LH_SPW > 0 ? LH_SPW : 1][LH_SR];
    for (int i = threadIdx.x; i < 256; i += blockDim.x) {
        gexp[i] = gf_exp[i];
        gexp[i + 256] = gf_exp[i + 256];
        glog[i] = gf_log[i];
    }
    __syncthreads();
    const int wid = threadIdx.x >> 6;
#if LH_ROWPF
    // Grid-stride waves (the host caps the grid, LONGHAIR_AMD_GRID) with the next stripe
    // group's Block.row bytes loaded while the current group decodes, so a group's plan
    // starts without a global-memory round trip.
    {
        const int lane = threadIdx.x & 63;
        const int sl = lane / LH_NCH;
        const int c = lane - sl * LH_NCH;
        const long long nw = lh_total_waves(stripes);
        const long long ws = (long long)gridDim.x * (blockDim.x >> 6);
        long long w = (lh_block_id() * blockDim.x + threadIdx.x) >> 6;
        unsigned int rowv[LH_NRW];
        if (w < nw) lh_fused_rows(lh_map_lane(stripes, w), c, rows, rowv);
        for (; w < nw; w += ws) {
            const lh_lane l = lh_map_lane(stripes, w);
            unsigned int cur[LH_NRW];
#pragma unroll
            for (int t = 0; t < LH_NRW; ++t) cur[t] = rowv[t];
            if (w + ws < nw) lh_fused_rows(lh_map_lane(stripes, w + ws), c, rows, rowv);
            lh_plan_regs pr;
            lh_fused_solve sv;
            sv.gexp = gexp;
            sv.glog = glog;
            if (l.active && lh_fused_plan(l, c, sl, &scratch[wid][sl][0], cur, rows, status, sv, pr))
                lh_decode_body(l, blocks, stripe_stride, pr, zero_page, sv);
        }
    }
#else
    LH_WAVE_LOOP(stripes) {
        const lh_lane l = lh_map_lane(stripes, lh_w);
        const int lane = threadIdx.x & 63;
        const int sl = lane / LH_NCH;
        const int c = lane - sl * LH_NCH;
        lh_plan_regs pr;
        lh_fused_solve sv;
        sv.gexp = gexp;
        sv.glog = glog;
        unsigned int rowv[LH_NRW];
        lh_fused_rows(l, c, rows, rowv);
        if (l.active && lh_fused_plan(l, c, sl, &scratch[wid][sl][0], rowv, rows, status, sv, pr))
            lh_decode_body(l, blocks, stripe_stride, pr, zero_page, sv);
    }
#endif
}

// Persistent, software-pipelined variant (host launches at most one resident grid): while
// a wave runs phase B of its stripe group, the next group's plan is already derived (its
// Block.row bytes were loaded before phase A) and its first columns are in flight.
extern "C" __global__ void __launch_bounds__(256, LH_DEC_LB)
lh_jit_decode_pipe(unsigned char *__restrict__ blocks, long long stripe_stride, unsigned char *__restrict__ rows,
                   signed char *__restrict__ status, const unsigned char *__restrict__ zero_page,
                   const unsigned char *__restrict__ gf_exp, const short *__restrict__ gf_log, int stripes) {
    __shared__ unsigned char gexp[512];
    __shared__ short glog[256];
    __shared__ __attribute__((aligned(16))) unsigned char scratch[4][LH_SPW > 0 ? LH_SPW : 1][LH_SR];
    for (int i = threadIdx.x; i < 256; i += blockDim.x) {
        gexp[i] = gf_exp[i];
        gexp[i + 256] = gf_exp[i + 256];
        glog[i] = gf_log[i];
    }
    __syncthreads();
    const int wid = threadIdx.x >> 6;
    const int lane = threadIdx.x & 63;
    const int sl = lane / LH_NCH;
    const int c = lane - sl * LH_NCH;
    const long long nw = lh_total_waves(stripes);
    const long long wstride = (long long)gridDim.x * (blockDim.x >> 6);
    long long w = (long long)blockIdx.x * (blockDim.x >> 6) + wid;
    if (w >= nw) return;
    lh_lane l = lh_map_lane(stripes, w);
    unsigned int rowv[LH_NRW];
    lh_fused_rows(l, c, rows, rowv);
    lh_plan_regs pr;
    lh_fused_solve sv;
    sv.gexp = gexp;
    sv.glog = glog;
    bool go = l.active && lh_fused_plan(l, c, sl, &scratch[wid][sl][0], rowv, rows, status, sv, pr);
    lh_word ring[LH_PF_DEC][8];
    if (go) lh_dec_issue(ring, pr, blocks + l.stripe * stripe_stride + l.p, zero_page + l.p);
    for (;;) {
        const long long w2 = w + wstride;
        const bool more = w2 < nw;
        const lh_lane l2 = lh_map_lane(stripes, w2);
        unsigned int rowv2[LH_NRW];
        if (more) lh_fused_rows(l2, c, rows, rowv2);  // in flight during phase A
        unsigned char *base = blocks + l.stripe * stripe_stride + l.p;
        lh_word v[LH_M][8];
        if (go) {
            sv(pr);
            lh_dec_phase_a(v, ring, pr, base, zero_page + l.p);
        }
        lh_plan_regs pr2;
        lh_fused_solve sv2;
        sv2.gexp = gexp;
        sv2.glog = glog;
        bool go2 = false;
        if (more) {
            go2 = l2.active && lh_fused_plan(l2, c, sl, &scratch[wid][sl][0], rowv2, rows, status, sv2, pr2);
            if (go2) lh_dec_issue(ring, pr2, blocks + l2.stripe * stripe_stride + l2.p, zero_page + l2.p);
        }
        if (go) lh_dec_phase_b(v, pr, base);
        if (!more) break;
        w = w2;
        l = l2;
        pr = pr2;
        sv = sv2;
        go = go2;
    }
}
#endif  // LH_EMAX <= 4 && LH_NCH <= 64 && LH_K <= 64
