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
#ifndef LH_BUF
// Column loads through buffer resources (32-bit lane offsets, wave-uniform column offsets in
// SGPRs, out-of-range offsets read as zero): k29/m4 access pattern 0.5175 against 0.549 ms
// for 64-bit global addresses (profiles/r2_ubench_pattern.txt).
#define LH_BUF 1
#endif
#ifndef LH_PTR
#define LH_PTR 0
#endif
#if LH_PTR && LH_BUF
#error "LH_PTR: scattered blocks are addressed by 64-bit pointers (LH_BUF 0)"
#endif
#ifndef LH_NT_DEC
// Decode loads: default cache policy.  The decode writes its outputs in place, into lines
// it (or a neighbour stripe's wave) read; non-temporal loads of those lines cost ~6 % in
// the access-pattern microbenchmark (profiles/r2_ubench_pattern.txt: 0.623 vs 0.587 ms).
#define LH_NT_DEC 0
#endif

// Decode-side column loads (W-byte lanes as lh_load, cache policy LH_NT_DEC).
__device__ __forceinline__ lh_word lh_load_dec(const unsigned char *p) {
#if LH_NT_DEC
    return lh_load(p);
#else
    lh_word w;
#if LH_W == 16
    const lh_u32x4 v = *(const lh_u32x4 *)p;
    w.v[0] = v.x; w.v[1] = v.y; w.v[2] = v.z; w.v[3] = v.w;
#elif LH_W == 12
    const lh_u32x3 v = *(const lh_u32x3 *)p;
    w.v[0] = v.x; w.v[1] = v.y; w.v[2] = v.z;
#elif LH_W == 8
    const lh_u32x2 v = *(const lh_u32x2 *)p;
    w.v[0] = v.x; w.v[1] = v.y;
#elif LH_W == 4
    w.v[0] = *(const unsigned int *)p;
#else
#pragma unroll
    for (int i = 0; i < LH_NW; ++i) w.v[i] = 0;
    __builtin_memcpy(&w.v[0], p, LH_W);
#endif
    return w;
#endif
}
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

// W-byte lane load through a buffer resource: voffset `off` (per lane), soffset `soff`
// (wave-uniform, e.g. a column offset), cache policy `aux` (2 = non-temporal).
template <int AUX>
__device__ __forceinline__ lh_word lh_load_buf(const __amdgpu_buffer_rsrc_t &rs, int off, int soff = 0) {
    lh_word w;
#if LH_W == 16
    const lh_u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, off, soff, AUX);
    w.v[0] = v.x; w.v[1] = v.y; w.v[2] = v.z; w.v[3] = v.w;
#elif LH_W == 12
    const lh_u32x3 v = __builtin_amdgcn_raw_buffer_load_b96(rs, off, soff, AUX);
    w.v[0] = v.x; w.v[1] = v.y; w.v[2] = v.z;
#elif LH_W == 8
    const lh_u32x2 v = __builtin_amdgcn_raw_buffer_load_b64(rs, off, soff, AUX);
    w.v[0] = v.x; w.v[1] = v.y;
#elif LH_W == 4
    w.v[0] = __builtin_amdgcn_raw_buffer_load_b32(rs, off, soff, AUX);
#else  // 1- or 2-byte lanes (tiny sub-blocks)
    w.v[0] = LH_W == 2 ? (unsigned int)__builtin_amdgcn_raw_buffer_load_b16(rs, off, soff, AUX)
                       : (unsigned int)__builtin_amdgcn_raw_buffer_load_b8(rs, off, soff, AUX);
#endif
    return w;
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

// a ^= sum of d[b] over the set bits b of S, the terms taken two at a time (XOR3): bits
// (b0, b1), (b2, b3), ... in ascending order, an odd last one alone.  Written flat (the set
// bits' positions computed at compile time) rather than as a recursion over the 8 bits, and
// the column's 8 LH_M row words through a pack expansion rather than a recursion over them:
// the recursions' forced inlining made the front end emit ~4 500 IR lines per column (572 000
// for a k127/m3 encode, 147 s in hiprtc, mostly inliner and instcombine) for the same code.
struct lh_bits {
    int n, b[8];
};
__device__ constexpr lh_bits lh_bits_of(unsigned S) {
    lh_bits r{0, {0, 0, 0, 0, 0, 0, 0, 0}};
    for (int b = 0; b < 8; ++b)
        if ((S >> b) & 1u) r.b[r.n++] = b;
    return r;
}
template <unsigned S>
__device__ __forceinline__ void lh_net(lh_word &a, const lh_word (&d)[8]) {
    constexpr lh_bits t = lh_bits_of(S);
    if constexpr (t.n >= 2) lh_xor2(a, d[t.b[0]], d[t.b[1]]);
    if constexpr (t.n >= 4) lh_xor2(a, d[t.b[2]], d[t.b[3]]);
    if constexpr (t.n >= 6) lh_xor2(a, d[t.b[4]], d[t.b[5]]);
    if constexpr (t.n >= 8) lh_xor2(a, d[t.b[6]], d[t.b[7]]);
    if constexpr (t.n % 2 == 1) lh_xor(a, d[t.b[t.n - 1]]);
}

// acc[r][y] ^= sum_x B(G[r][x]) d_x, one column x at a time, all constants.
template <class T, T... I>
struct lh_iseq {};
template <int X, int... I>
__device__ __forceinline__ void lh_col_net(lh_word (&acc)[LH_M][8], const lh_word (&d)[8], lh_iseq<int, I...>) {
    (lh_net<LH_BM[I / 8][X][I % 8]>(acc[I / 8][I % 8], d), ...);
}
#ifndef LH_PROBE_LIGHT
#define LH_PROBE_LIGHT 0  // (probe, wrong bytes: one XOR per sub-row of row 0 instead of the network)
#endif
template <int X>
__device__ __forceinline__ void lh_column(lh_word (&acc)[LH_M][8], const lh_word (&d)[8]) {
#if LH_PROBE_LIGHT
#pragma unroll
    for (int y = 0; y < 8; ++y) lh_xor(acc[0][y], d[(y + X) & 7]);
#else
    lh_col_net<X>(acc, d, __make_integer_seq<lh_iseq, int, LH_M * 8>{});
#endif
}

struct lh_lane {
    long long stripe;
    int p;       // first byte of the lane's chunk in every sub-block
    bool last;   // last chunk of its stripe
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
    l.last = c == LH_NCH - 1;
    l.p = l.last ? (LH_SUB - LH_W) : c * LH_W;
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

// The wave's index in its workgroup, wave-uniform to the compiler (LH_UNIWID): the per-wave LDS
// rings indexed by it then have their addresses -- the LDS-DMAs' M0 -- in SGPRs.  With
// threadIdx.x >> 6 the compiler treats the index as per-lane, keeps every ring slot / chunk
// address in a VGPR (16 in the k29/m4 decode) and reads one back with v_readfirstlane before
// each DMA.
#ifndef LH_UNIWID
#define LH_UNIWID 1
#endif
template <int ROLE>  // (LH_UNIWID bit 0: the encode's rings, bit 1: the decode's)
__device__ __forceinline__ int lh_wid() {
    if constexpr ((LH_UNIWID >> ROLE) & 1) return __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    return (int)(threadIdx.x >> 6);
}

#define LH_WAVE_LOOP(stripes)                                                                   \
    const long long lh_nw = lh_total_waves(stripes);                                           \
    const long long lh_ws = (long long)gridDim.x * (blockDim.x >> 6);                          \
    for (long long lh_w = (lh_block_id() * blockDim.x + threadIdx.x) >> 6; lh_w < lh_nw;       \
         lh_w += lh_ws)

// Keeps the accumulators in registers between columns: stops the compiler from
// re-associating XORs across columns (which lengthens live ranges past the register file).
// One asm statement per 8 (NW <= 3) or 4 words: each volatile asm is a memory side effect
// to LLVM, and the IR sinking pass's cost grows with their number (jit.cpp LH_PIN).
#if LH_NW == 1
#define LH_OPS(w) "+v"((w).v[0])
#elif LH_NW == 2
#define LH_OPS(w) "+v"((w).v[0]), "+v"((w).v[1])
#elif LH_NW == 3
#define LH_OPS(w) "+v"((w).v[0]), "+v"((w).v[1]), "+v"((w).v[2])
#else
#define LH_OPS(w) "+v"((w).v[0]), "+v"((w).v[1]), "+v"((w).v[2]), "+v"((w).v[3])
#endif
// LH_PIN_WORDS (bit 0: decode phase A, bit 1: phase B, bit 2: everywhere): one asm
// statement per word instead of per row.  The per-row statements let the register allocator
// keep more copies live: the fused k29/m4 decode grew from 162 to 180 VGPRs (3 -> 2 waves
// per SIMD) when they replaced the per-word ones.  Per-word pins cost build time only for
// large column counts, so they are the default where the fused decode is compiled.
#ifndef LH_PIN_WORDS
#if (LH_K < LH_M ? LH_K : LH_M) <= 4 && LH_K <= 64
#define LH_PIN_WORDS 1
#else
#define LH_PIN_WORDS 0
#endif
#endif
__device__ __forceinline__ void lh_pin8w(lh_word (&a)[8]) {
#pragma unroll
    for (int y = 0; y < 8; ++y)
#pragma unroll
        for (int i = 0; i < LH_NW; ++i) asm volatile("" : "+v"(a[y].v[i]));
}
__device__ __forceinline__ void lh_pin8(lh_word (&a)[8]) {
#if LH_PIN_WORDS & 4
    lh_pin8w(a);
#elif LH_NW <= 3
    asm volatile("" : LH_OPS(a[0]), LH_OPS(a[1]), LH_OPS(a[2]), LH_OPS(a[3]), LH_OPS(a[4]), LH_OPS(a[5]),
                 LH_OPS(a[6]), LH_OPS(a[7]));
#else
    asm volatile("" : LH_OPS(a[0]), LH_OPS(a[1]), LH_OPS(a[2]), LH_OPS(a[3]));
    asm volatile("" : LH_OPS(a[4]), LH_OPS(a[5]), LH_OPS(a[6]), LH_OPS(a[7]));
#endif
}

__device__ __forceinline__ void lh_opaque(lh_word (&acc)[LH_M][8]) {
#pragma unroll
    for (int r = 0; r < LH_M; ++r) lh_pin8(acc[r]);
}
// Decode phase A's pins (LH_PIN_WORDS & 1: one statement per word).
__device__ __forceinline__ void lh_dopaque(lh_word (&acc)[LH_M][8]) {
#pragma unroll
    for (int r = 0; r < LH_M; ++r) {
#if LH_PIN_WORDS & 1
        lh_pin8w(acc[r]);
#else
        lh_pin8(acc[r]);
#endif
    }
}

#if LH_PTR
// Scattered blocks (cauchy_256_encode_batch_ptrs / cauchy_256_decode_batch_ptrs): the
// kernel's block argument is a device table of block pointers, one row of LH_K pointers per
// stripe (row stride `stride` bytes).  Each wave copies the rows of its stripes into LDS
// (its own 8 * LH_SPW * (LH_K + 1) bytes; the host keeps 4 waves' worth <= 33 KiB); every column
// address is then an LDS read, counted by lgkmcnt and so never waiting behind the block loads
// in flight (vmcnt), unlike a pointer fetched from memory per column.  The lanes of a stripe
// fill its row (they share the stripe's early exits, so a partial wave fills what it reads).
// An index the compiler cannot see through: the LDS read of a column's pointer stays next to
// that column's loads (each asm is ordered after the previous column's accumulator pins)
// instead of every column's pointer being read up front and held in registers (k29/m4 fused
// decode: 192 VGPRs, 2 waves/SIMD, with them hoisted).
__device__ __forceinline__ int lh_late(int i) {
    asm volatile("" : "+v"(i));
    return i;
}
// Entry LH_K of a row is `extra` (decode: the zero page, so an absent column is one more
// table index, not a 64-bit select: with the select the k29/m4 fused decode took 192 VGPRs
// instead of 157).
__device__ __forceinline__ const unsigned long long *lh_ptab(const lh_lane &l, const unsigned char *tab,
                                                            long long stride, const unsigned char *extra) {
    __shared__ unsigned long long lh_pt[4][LH_SPW * (LH_K + 1)];
    const int lane = threadIdx.x & 63;
#if LH_NCH <= 64
    const int sl = lane / LH_NCH, c = lane - sl * LH_NCH, step = LH_NCH;
#else
    const int sl = 0, c = lane, step = 64;
#endif
    unsigned long long *row = &lh_pt[threadIdx.x >> 6][sl * (LH_K + 1)];
    const unsigned long long *src = (const unsigned long long *)(tab + l.stripe * stride);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // the previous stripe group's reads
    __builtin_amdgcn_wave_barrier();
    for (int x = c; x < LH_K; x += step) row[x] = src[x];
    if (c == 0) row[LH_K] = (unsigned long long)extra;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    return row;
}
#endif

// Encode column source of a lane: with LH_BUF one buffer resource over the wave's stripes
// (column x at soffset x * LH_BYTES, a wave-uniform SGPR; sub-block b in the immediate
// offset; one 32-bit lane offset), else the lane's 64-bit chunk pointer.
struct lh_esrc {
#if LH_BUF
    __amdgpu_buffer_rsrc_t rs;
    int lbase;
    __device__ __forceinline__ lh_word load(int x, int b) const {
        return lh_load_buf<LH_NT ? 2 : 0>(rs, lbase + b * LH_SUB, x * LH_BYTES);
    }

    // The 8 sub-block words of column x.
    __device__ __forceinline__ void load8(lh_word (&d)[8], int x) const {
#pragma unroll
        for (int b = 0; b < 8; ++b) d[b] = load(x, b);
    }
#elif LH_PTR
    const unsigned long long *pt;  // LDS: the lane's stripe's LH_K block pointers
    int p;
    __device__ __forceinline__ lh_word load(int x, int b) const {
        return lh_load((const unsigned char *)pt[x] + p + b * LH_SUB);
    }
    __device__ __forceinline__ void load8(lh_word (&d)[8], int x) const {
        const unsigned char *q = (const unsigned char *)pt[lh_late(x)] + p;
#pragma unroll
        for (int b = 0; b < 8; ++b) d[b] = lh_load(q + b * LH_SUB);
    }
#else
    const unsigned char *base;
    __device__ __forceinline__ lh_word load(int x, int b) const {
        return lh_load(base + (long long)x * LH_BYTES + b * LH_SUB);
    }
    __device__ __forceinline__ void load8(lh_word (&d)[8], int x) const {
#pragma unroll
        for (int b = 0; b < 8; ++b) d[b] = load(x, b);
    }
#endif
};

// Column loop, unrolled at compile time, with the next LH_PF columns' loads in flight
// while column X is combined.
#ifndef LH_PF
#define LH_PF 3  // columns in flight ahead of the one being combined
#endif
template <int X>
struct lh_unroll_encode {
    __device__ __forceinline__ static void run(lh_word (&acc)[LH_M][8], lh_word (&ring)[LH_PF][8], const lh_esrc &S) {
        if (X + LH_PF < LH_K) {
            lh_word nxt[8];
            S.load8(nxt, X + LH_PF);
            lh_column<X>(acc, ring[X % LH_PF]);
            lh_opaque(acc);
#pragma unroll
            for (int b = 0; b < 8; ++b) ring[X % LH_PF][b] = nxt[b];
        } else {
            lh_column<X>(acc, ring[X % LH_PF]);
            lh_opaque(acc);
        }
        lh_unroll_encode<X + 1>::run(acc, ring, S);
    }
};
template <>
struct lh_unroll_encode<LH_K> {
    __device__ __forceinline__ static void run(lh_word (&)[LH_M][8], lh_word (&)[LH_PF][8], const lh_esrc &) {}
};

// ---------------------------------------------------------------- LDS-DMA column loads
// LH_LDS = 1 (jit.cpp, whole stripes per wave with 8-byte lanes and 16-byte-multiple blocks,
// e.g. k29/m4/1296): the column x of the wave's LH_SPW stripes is fetched as aligned 16-byte
// chunks -- LH_LQ global_load_lds_dwordx4 per column, chunk j = 64 q + lane of the image
// [stripe][bytes], per-lane source addresses -- into a per-wave LDS ring of LH_LD slots, and
// every lane reads its 8 bytes of sub-block b back as two naturally aligned ds_read_b64
// funnelled by v_alignbyte (sub-block b starts (b * sub) % 8 bytes past an 8-byte boundary in
// both memory and the image, a compile-time constant; a misaligned ds_read_b64 would replay at
// 64 cycles).  Versus 8 loads of 3 x 168-byte pieces per column, the wave issues LH_LQ = 4
// loads of whole 1-KiB runs: the k29/m4 access pattern 0.546 against 0.563-0.594 ms on two
// boxes (profiles/r5a/r5c_ubench_floor.txt, `ldsd`).  The last lane of a stripe reads its
// chunk unshifted (only LH_VLAST bytes are its own) and stores [sub - 8, sub) assembled with
// the previous lane's word (DPP row_shr:1; the host checks both lanes share a DPP row).
// That last lane's word pair may reach up to 16 bytes past its stripe's image (bytes that are
// never its own): when the image ends within 16 bytes of its slot's end, each ring carries 16
// bytes of padding (LH_LPAD), so the read stays in the wave's ring.
#ifndef LH_LDS
#define LH_LDS 0
#endif
#if LH_LDS
#if LH_W != 8 || LH_NCH > 64 || LH_BYTES % 16 != 0 || (LH_BUF == 0 && !LH_PTR)
#error "LH_LDS: 8-byte lanes, whole stripes per wave, 16-byte-multiple blocks, strided or pointer-table batches"
#endif
#ifndef LH_LD
#define LH_LD 4  // ring slots per wave (columns in flight + the one being read)
#endif
#ifndef LH_LDE
#define LH_LDE LH_LD  // the encode's ring (its module is compiled apart from the decode's)
#endif
#define LH_LQ ((LH_SPW * LH_BYTES + 1023) / 1024)  // DMA instructions per column
#define LH_VLAST (LH_SUB - 8 * (LH_NCH - 1))      // valid bytes of the last chunk of a sub-block
// (ring padding: only when the image ends within 16 bytes of its slot's end)
#define LH_LPAD ((LH_SPW * LH_BYTES + 16 > LH_LQ * 1024) ? 16 : 0)
typedef unsigned int lh_u32x2a __attribute__((ext_vector_type(2)));
// Bytes [S, S + 8) of the 16 little-endian bytes (a, b).
template <int S>
__device__ __forceinline__ lh_word lh_funnel(unsigned a0, unsigned a1, unsigned b0, unsigned b1) {
    lh_word w;
    if constexpr (S == 0) {
        w.v[0] = a0; w.v[1] = a1;
    } else if constexpr (S == 4) {
        w.v[0] = a1; w.v[1] = b0;
    } else if constexpr (S < 4) {
        w.v[0] = __builtin_amdgcn_alignbyte(a1, a0, S); w.v[1] = __builtin_amdgcn_alignbyte(b0, a1, S);
    } else if constexpr (S == 8) {
        w.v[0] = b0; w.v[1] = b1;
    } else {
        w.v[0] = __builtin_amdgcn_alignbyte(b0, a1, S - 4); w.v[1] = __builtin_amdgcn_alignbyte(b1, b0, S - 4);
    }
    return w;
}
// The lane's word of sub-block B from a ring slot: `lo` its chunk's offset in the image
// (stripe * bytes + 8 c), `lo8` = lo + 8 hidden from the compiler so the pair stays two
// ds_read_b64 (2 LDS cycles each) instead of one ds_read2_b64 (8).
template <int B>
__device__ __forceinline__ lh_word lh_slot_word(const unsigned char *slot, int lo, int lo8) {
    constexpr int S = (B * LH_SUB) % 8, O = B * LH_SUB - S;
    const lh_u32x2a a = *(const lh_u32x2a *)(slot + lo + O);
    if constexpr (S == 0) {
        lh_word w;
        w.v[0] = a.x; w.v[1] = a.y;
        return w;
    } else {
        const lh_u32x2a b = *(const lh_u32x2a *)(slot + lo8 + O);
        return lh_funnel<S>(a.x, a.y, b.x, b.y);
    }
}
template <int B = 0>
__device__ __forceinline__ void lh_slot_col(lh_word (&d)[8], const unsigned char *slot, int lo, int lo8) {
    if constexpr (B < 8) {
        d[B] = lh_slot_word<B>(slot, lo, lo8);
        lh_slot_col<B + 1>(d, slot, lo, lo8);
    }
}
__device__ __forceinline__ unsigned lh_row_shr1(unsigned v) {  // lane i <- lane i - 1 within a DPP row of 16
    return (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, false);
}
typedef unsigned int lh_u32x4a __attribute__((ext_vector_type(4)));
// An 8-byte word into LDS at an address A (mod 8) bytes past an 8-byte boundary, in naturally
// aligned pieces (a misaligned ds_write_b64 would replay like the reads).
template <int A>
__device__ __forceinline__ void lh_lds_put(unsigned char *p, const lh_word &w) {
    if constexpr (A == 0) {
        lh_u32x2a v;
        v.x = w.v[0]; v.y = w.v[1];
        *(lh_u32x2a *)p = v;
    } else if constexpr (A == 4) {
        ((unsigned *)p)[0] = w.v[0];
        ((unsigned *)p)[1] = w.v[1];
    } else {
        typedef unsigned short lh_u16a __attribute__((aligned(2)));
        *(lh_u16a *)(p + 0) = (unsigned short)w.v[0];
        *(lh_u16a *)(p + 2) = (unsigned short)(w.v[0] >> 16);
        *(lh_u16a *)(p + 4) = (unsigned short)w.v[1];
        *(lh_u16a *)(p + 6) = (unsigned short)(w.v[1] >> 16);
    }
}
// LH_LDS_FLAT_ST: the encode's recovery blocks leave through the ring (below) when the
// wave's output image fits it.
#ifndef LH_LDS_FLAT_ST
#define LH_LDS_FLAT_ST (LH_SPW * LH_M * LH_BYTES <= LH_LDE * LH_LQ * 1024)
#endif
// Block pointers in LDS: each wave writes its stripes' rows (LH_K data then LH_M recovery
// block addresses: from the pointer tables with LH_PTR, else computed from base and stride)
// into LDS; a DMA lane's source for column x is its chunk's row entry plus the chunk's offset,
// read before the column's wait, and the stores take their rows' entries.  For strided
// batches too: k29/m4 encode 0.532 -> 0.502 ms against per-lane 64-bit source pointers
// advanced by x * bytes (profiles/r7q_tune_k29m4_erows.txt; found because the pointer-table
// form ran faster, r7n_seq_probe_ptr.txt; padding the ring to the same LDS size: no change).
// One 16-byte-per-lane LDS-DMA (global_load_lds_dwordx4): `lds` the wave-uniform LDS address
// of lane 0's 16 bytes.
// Round 6 found that with the builtin, hipcc's waitcnt pass cannot tell a ring slot being read
// from the slots being filled (one __shared__ array) and puts s_waitcnt vmcnt(0) before every
// column's first LDS read: the "4-slot ring" of the one-column kernels ran one column per wave
// at a time.  Issued from inline asm (LH_ASM_DMA=1) the compiler sees no LDS write in flight
// and the kernels' own counted waits (lh_wait_vmcnt) order the landing, so the ring really
// runs 3 columns deep -- and measured SLOWER: encode 0.533 against 0.501 ms, decode 0.566
// against 0.554 (ring depth 2 / 3: 0.562 / 0.557; profiles/r9a_tune_k29m4_asm_dma.txt).  The
// HBM stream of this access pattern prefers fewer, longer runs in flight over deeper
// prefetch (tools/ubench_r6.hip), which the multi-column steps below turn into a design:
// they issue their DMAs from asm (lh_dma16_bufs) with one step in flight by construction.
// The builtin (with its drain) stays the default of the one-column kernels.
#ifndef LH_ASM_DMA
#define LH_ASM_DMA 0
#endif
template <int NT>
__device__ __forceinline__ void lh_dma16(const void *src, const void *lds) {
#if LH_ASM_DMA
    const unsigned m = __builtin_amdgcn_readfirstlane((unsigned)(unsigned long long)lds);
    if constexpr (NT)
        asm volatile("global_load_lds_dwordx4 %0, off nt" ::"v"(src), "{m0}"(m) : "memory");
    else
        asm volatile("global_load_lds_dwordx4 %0, off" ::"v"(src), "{m0}"(m) : "memory");
#else
    __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void *)src,
                                     (__attribute__((address_space(3))) void *)lds, 16, 0, NT ? 2 : 0);
#endif
}
#define LH_LPR (LH_K + LH_M)
struct lh_ldsrc {
    const unsigned long long *pt;  // LDS: the wave's pointer rows [stripe][LH_LPR]
    int pr[LH_LQ];                 // DMA chunk q: its stripe's row in pt
    int off[LH_LQ];                // ... its offset in the block
    unsigned char *ring;           // this wave's LH_LDE slots of LH_LQ KiB
    // The lanes' source addresses of column x.
    __device__ __forceinline__ void addrs(int x, const unsigned char *(&a)[LH_LQ]) const {
#pragma unroll
        for (int q = 0; q < LH_LQ; ++q) a[q] = (const unsigned char *)pt[pr[q] + x] + off[q];
    }
    __device__ __forceinline__ void issue(const unsigned char *const (&a)[LH_LQ], int slot) const {
#pragma unroll
        for (int q = 0; q < LH_LQ; ++q)
            lh_dma16<LH_NT>(a[q], ring + slot * (LH_LQ * 1024) + q * 1024);
    }
    __device__ __forceinline__ void issue(int x, int slot) const {
        const unsigned char *a[LH_LQ];
        addrs(x, a);
        issue(a, slot);
    }
};
// The same through a buffer resource (word 3 = 0x00020000 as lh_encode_wave's
// make_buffer_rsrc): lane offset `voff`, out-of-range offsets land zeros and fetch nothing.
typedef unsigned int lh_u32x4r __attribute__((ext_vector_type(4)));
__device__ __forceinline__ lh_u32x4r lh_rsrc(const void *base, unsigned bytes) {
    const unsigned long long b = (unsigned long long)base;
    lh_u32x4r r;
    r.x = __builtin_amdgcn_readfirstlane((unsigned)b);
    r.y = __builtin_amdgcn_readfirstlane((unsigned)(b >> 32) & 0xFFFFu);
    r.z = __builtin_amdgcn_readfirstlane(bytes);
    r.w = 0x00020000u;
    return r;
}
template <int NT>
__device__ __forceinline__ void lh_dma16_buf(const lh_u32x4r &rs, int voff, const void *lds) {
    const unsigned m = __builtin_amdgcn_readfirstlane((unsigned)(unsigned long long)lds);
    if constexpr (NT)
        asm volatile("buffer_load_dwordx4 %0, %1, 0 offen nt lds" ::"v"(voff), "s"(rs), "{m0}"(m) : "memory");
    else
        asm volatile("buffer_load_dwordx4 %0, %1, 0 offen lds" ::"v"(voff), "s"(rs), "{m0}"(m) : "memory");
}
// ... with a wave-uniform byte offset `soff` added (SGPR soffset).
#ifndef LH_CPS_POLI
#define LH_CPS_POLI 0  // cache policy of the multi-column-step DMAs: 0 nt, 1 sc1 nt, 2 sc0 nt, 3 sc0 sc1 nt
#endif
#if LH_CPS_POLI == 1
#define LH_CPS_POL "sc1 nt"
#elif LH_CPS_POLI == 2
#define LH_CPS_POL "sc0 nt"
#elif LH_CPS_POLI == 3
#define LH_CPS_POL "sc0 sc1 nt"
#else
#define LH_CPS_POL "nt"
#endif
template <int NT>
__device__ __forceinline__ void lh_dma16_bufs(const lh_u32x4r &rs, int voff, int soff, const void *lds) {
    const unsigned m = __builtin_amdgcn_readfirstlane((unsigned)(unsigned long long)lds);
    if constexpr (NT)
        asm volatile("buffer_load_dwordx4 %0, %1, %2 offen " LH_CPS_POL " lds" ::"v"(voff), "s"(rs), "s"(soff), "{m0}"(m)
                     : "memory");
    else
        asm volatile("buffer_load_dwordx4 %0, %1, %2 offen lds" ::"v"(voff), "s"(rs), "s"(soff), "{m0}"(m) : "memory");
}
// s_waitcnt vmcnt(N) (gfx9 encoding, expcnt / lgkmcnt left at their maxima); N a constant.
template <int N>
__device__ __forceinline__ void lh_wait_vmcnt() {
    __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}
template <int X>
struct lh_unroll_encode_lds {
    __device__ __forceinline__ static void run(lh_word (&acc)[LH_M][8], const lh_ldsrc &S, int lo, int lo8) {
        if constexpr (X < LH_K) {
            // this column's DMAs landed: all but those of the columns issued after it
            constexpr int ahead = (LH_LDE - 1) < (LH_K - 1 - X) ? (LH_LDE - 1) : (LH_K - 1 - X);
            const unsigned char *a[LH_LQ];
            if constexpr (X + LH_LDE < LH_K) S.addrs(X + LH_LDE, a);
            lh_wait_vmcnt<LH_LQ * ahead>();
            asm volatile("" ::: "memory");  // no LDS read moves above the wait
            lh_word d[8];
            lh_slot_col(d, S.ring + (X % LH_LDE) * (LH_LQ * 1024), lo, lo8);
            lh_column<X>(acc, d);
            lh_opaque(acc);
            if constexpr (X + LH_LDE < LH_K) {
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the slot's reads are done
                S.issue(a, X % LH_LDE);
            }
            lh_unroll_encode_lds<X + 1>::run(acc, S, lo, lo8);
        }
    }
};

// Sub-rows Y.. of one output row into the ring image (LH_LDS_FLAT_ST): the last lane's
// word funnelled as for a direct store and written at its own alignment.
template <int Y>
__device__ __forceinline__ void lh_img_row(unsigned char *row, const lh_word (&a)[8], bool last, bool on) {
    if constexpr (Y < 8) {
        lh_word w = a[Y];
        if constexpr (LH_VLAST != 8) {
            const lh_word f = lh_funnel<LH_VLAST>(lh_row_shr1(w.v[0]), lh_row_shr1(w.v[1]), w.v[0], w.v[1]);
            w.v[0] = last ? f.v[0] : w.v[0];
            w.v[1] = last ? f.v[1] : w.v[1];
        }
        if (on) {
            if (last) lh_lds_put<((Y + 1) * LH_SUB) % 8>(row + Y * LH_SUB, w);
            else lh_lds_put<(Y * LH_SUB) % 8>(row + Y * LH_SUB, w);
        }
        lh_img_row<Y + 1>(row, a, last, on);
    }
}

__device__ __forceinline__ void lh_encode_wave_lds(long long wave, const unsigned char *__restrict__ in,
                                                   long long in_stride, unsigned char *__restrict__ out,
                                                   long long out_stride, int stripes) {
    __shared__ __attribute__((aligned(16))) unsigned char lh_lring[4][LH_LDE * LH_LQ * 1024 + LH_LPAD];
    const int lane = threadIdx.x & 63;
    const int sl = lane / LH_NCH, c = lane - sl * LH_NCH;
    const long long s0 = (long long)__builtin_amdgcn_readfirstlane((int)wave) * LH_SPW;  // wave-uniform
    if (s0 >= stripes) return;  // wave-uniform
    const int nst = (int)((stripes - s0) < LH_SPW ? (stripes - s0) : LH_SPW);
    lh_ldsrc S;
    S.ring = lh_lring[lh_wid<0>()];
    // LH_PTR: in / out are the data and recovery pointer tables (rows of LH_K / LH_M pointers)
    __shared__ unsigned long long lh_lpt[4][LH_SPW * LH_LPR];
    unsigned long long *prow = lh_lpt[threadIdx.x >> 6];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // the previous stripe group's reads
    __builtin_amdgcn_wave_barrier();
    if (sl < nst) {
#if LH_PTR
        const unsigned long long *it = (const unsigned long long *)(in + (s0 + sl) * in_stride);
        const unsigned long long *ot = (const unsigned long long *)(out + (s0 + sl) * out_stride);
        for (int x = c; x < LH_LPR; x += LH_NCH) prow[sl * LH_LPR + x] = x < LH_K ? it[x] : ot[x - LH_K];
#else
        for (int x = c; x < LH_LPR; x += LH_NCH)
            prow[sl * LH_LPR + x] = x < LH_K ? (unsigned long long)(in + (s0 + sl) * in_stride + (long long)x * LH_BYTES)
                                             : (unsigned long long)(out + (s0 + sl) * out_stride + (long long)(x - LH_K) * LH_BYTES);
#endif
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    S.pt = prow;
#pragma unroll
    for (int q = 0; q < LH_LQ; ++q) {  // every lane moves chunks, whatever its own stripe
        int j = 64 * q + lane;
        if (j >= nst * (LH_BYTES / 16)) j = nst * (LH_BYTES / 16) - 1;  // (lands past the image)
        const int js = j / (LH_BYTES / 16);
        S.pr[q] = js * LH_LPR;
        S.off[q] = (j - js * (LH_BYTES / 16)) * 16;
    }
#pragma unroll
    for (int q = 0; q < LH_LDE; ++q)
        if (q < LH_K) S.issue(q, q);
    lh_word acc[LH_M][8];
#pragma unroll
    for (int r = 0; r < LH_M; ++r)
#pragma unroll
        for (int y = 0; y < 8; ++y)
#pragma unroll
            for (int i = 0; i < LH_NW; ++i) acc[r][y].v[i] = 0;
    const int lo = (sl < LH_SPW ? sl : LH_SPW - 1) * LH_BYTES + 8 * c;
    int lo8 = lo + 8;
    asm volatile("" : "+v"(lo8));
    lh_unroll_encode_lds<0>::run(acc, S, lo, lo8);
    const bool last = c == LH_NCH - 1;
#if LH_LDS_FLAT_ST
    // The wave's recovery blocks [stripe][row][bytes] assembled in its (now idle) ring, then
    // stored as aligned 16-byte chunks, chunk j = 64 q + lane: half the store instructions of
    // the per-lane 8-byte stores, each a contiguous 1 KiB run (profiles/r5c_ubench_floor.txt
    // `flat`: 0.532 against 0.544 ms).  A lane writes its word of sub-row y at offset
    // y * sub + 8 c of the row (the last lane its funnelled [sub - 8, sub)) in naturally
    // aligned pieces, the alignment a compile-time constant per sub-row and lane kind.
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // every ring read of the last column done
    {
        unsigned char *img = S.ring + (sl < LH_SPW ? sl : LH_SPW - 1) * (LH_M * LH_BYTES) + (last ? LH_SUB - 8 : 8 * c);
        // (the last lane's word starts at y * sub + sub - 8: its own alignment, a second case)
#pragma unroll
        for (int r = 0; r < LH_M; ++r) lh_img_row<0>(img + r * LH_BYTES, acc[r], last, sl < nst);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the image is complete (one wave: in order)
    {
        constexpr int per = LH_M * LH_BYTES / 16;  // chunks per stripe
        const int n = nst * per;
#pragma unroll
        for (int q = 0; q < (LH_SPW * per + 63) / 64; ++q) {
            const int j = 64 * q + lane;
            if (j < n) {
                const int js = j / per, t = j - js * per;
                const lh_u32x4a v = *(const lh_u32x4a *)(S.ring + js * (LH_M * LH_BYTES) + t * 16);
                const int r = t / (LH_BYTES / 16);
                unsigned char *dst = (unsigned char *)S.pt[js * LH_LPR + LH_K + r] + (t - r * (LH_BYTES / 16)) * 16;
#if LH_NT_ST
                __builtin_nontemporal_store(v, (lh_u32x4a *)dst);
#else
                *(lh_u32x4a *)dst = v;
#endif
            }
        }
    }
    return;
#endif
    if (sl >= nst) return;
    const int p = last ? LH_SUB - 8 : 8 * c;
#pragma unroll
    for (int r = 0; r < LH_M; ++r) {
        unsigned char *o = (unsigned char *)S.pt[sl * LH_LPR + LH_K + r] + p;
#pragma unroll
        for (int y = 0; y < 8; ++y) {
            lh_word w = acc[r][y];
            if constexpr (LH_VLAST != 8) {
                const lh_word f = lh_funnel<LH_VLAST>(lh_row_shr1(w.v[0]), lh_row_shr1(w.v[1]), w.v[0], w.v[1]);
                w.v[0] = last ? f.v[0] : w.v[0];
                w.v[1] = last ? f.v[1] : w.v[1];
            }
            lh_store(o + y * LH_SUB, w);
        }
    }
}

// ------------------------------------------------------------ multi-column steps
// LH_CPS > 1 (strided batches; jit.cpp): the wave fetches LH_CPS columns of its stripes per
// step -- per stripe LH_CPS x bytes contiguous, LH_SQ buffer_load_dwordx4 ... lds of 1 KiB
// runs into one slot [stripe][LH_CPS x bytes] -- then combines them, then issues the next step
// and waits for it (one step in flight, nothing while the wave combines).  With the host
// running one 4-wave workgroup per CU (LH_WGCU, dynamic LDS pads the rest), the chip keeps
// fewer, longer runs in flight: the k29/m4 access pattern 0.526-0.533 -> 0.504-0.509 ms at 5-6
// columns per step (tools/ubench_r6.hip, profiles/r9*_ubench_r6*.txt).  Each DMA lane's chunk
// is a fixed lane offset into the wave's stripes (voffset) plus the step's column offset
// (soffset): no address arithmetic per DMA.  Chunks past the stripes (a partial wave) or past
// column LH_K (the last step) get an out-of-range offset: zeros, no memory request.
#ifndef LH_CPS
#define LH_CPS 1
#endif
#ifndef LH_WPB
#define LH_WPB 4  // waves per workgroup of the LH_CPS encode (the host launches LH_WPB x 64 threads)
#endif
#if LH_LDS && LH_CPS > 1 && !LH_PTR
#define LH_CCH (LH_BYTES / 16)                              // 16-byte chunks per block
#define LH_SCH (LH_CPS * LH_CCH)                            // ... per stripe and step
#define LH_SQ ((LH_SPW * LH_SCH + 63) / 64)                 // DMA instructions per step
#define LH_NSTEP ((LH_K + LH_CPS - 1) / LH_CPS)
#define LH_LASTC (LH_K - (LH_NSTEP - 1) * LH_CPS)           // columns of the last step
#define LH_SSLOT (LH_SQ * 1024 + 16)                        // (+16: the last lane's second word)
static_assert(LH_SQ <= 63, "vmcnt");
static_assert(LH_NSTEP >= 2, "LH_CPS: at least two steps");
template <int T, int CC>
struct lh_cps_cols {
    __device__ __forceinline__ static void run(lh_word (&acc)[LH_M][8], const unsigned char *slot, int lo, int lo8) {
        if constexpr (CC < LH_CPS && T * LH_CPS + CC < LH_K) {
            lh_word d[8];
            lh_slot_col(d, slot + CC * LH_BYTES, lo, lo8);
            lh_column<T * LH_CPS + CC>(acc, d);
            lh_opaque(acc);
            lh_cps_cols<T, CC + 1>::run(acc, slot, lo, lo8);
        }
    }
};
#ifndef LH_CPS_AHEAD
#define LH_CPS_AHEAD 0  // 1: two slots, step T + 1 issued before step T is combined (tools/tune.py)
#endif
// Step T1's DMAs into `slot` (the last step's chunks past column LH_K out of range).
template <int T1>
__device__ __forceinline__ void lh_cps_issue(const lh_u32x4r &rs, const int (&voff)[LH_SQ], unsigned char *slot) {
    constexpr int x1 = T1 * LH_CPS;  // first column of the step
#pragma unroll
    for (int q = 0; q < LH_SQ; ++q) {
        int v = voff[q];
        if constexpr (T1 + 1 == LH_NSTEP && LH_LASTC < LH_CPS) {  // last step: columns < LH_K only
            const int r = (64 * q + (int)(threadIdx.x & 63)) % LH_SCH;
            v = r < LH_LASTC * LH_CCH ? v : (int)0x80000000;
        }
        lh_dma16_bufs<LH_NT>(rs, v, x1 * LH_BYTES, slot + q * 1024);
    }
}
template <int T>
struct lh_unroll_cps {
    __device__ __forceinline__ static void run(lh_word (&acc)[LH_M][8], const lh_u32x4r &rs, const int (&voff)[LH_SQ],
                                               unsigned char *slot, int lo, int lo8) {
        if constexpr (T < LH_NSTEP) {
#if LH_CPS_AHEAD
            unsigned char *cur = slot + (T & 1) * LH_SSLOT;
            if constexpr (T + 1 < LH_NSTEP) {
                lh_cps_issue<T + 1>(rs, voff, slot + ((T + 1) & 1) * LH_SSLOT);  // (its slot was read at T - 1)
                lh_wait_vmcnt<LH_SQ>();  // step T landed, T + 1 in flight
            } else {
                lh_wait_vmcnt<0>();
            }
            asm volatile("" ::: "memory");
            lh_cps_cols<T, 0>::run(acc, cur, lo, lo8);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the slot's reads are done
#else
            lh_wait_vmcnt<0>();  // this step's DMAs landed (the only ones in flight)
            asm volatile("" ::: "memory");
            lh_cps_cols<T, 0>::run(acc, slot, lo, lo8);
            if constexpr (T + 1 < LH_NSTEP) {
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the slot's reads are done
                lh_cps_issue<T + 1>(rs, voff, slot);
            }
#endif
            lh_unroll_cps<T + 1>::run(acc, rs, voff, slot, lo, lo8);
        }
    }
};
#ifndef LH_CPS_FLAT
#define LH_CPS_FLAT 0  // (per-lane stores: at one workgroup per CU the slot-image stores measured slower)
#endif
// Recovery rows per slot image (the slot holds LH_SQ KiB).
#define LH_CRP ((LH_SQ * 1024) / (LH_SPW * LH_BYTES) < LH_M ? (LH_SQ * 1024) / (LH_SPW * LH_BYTES) : LH_M)
#if LH_CRP >= 1
template <int R0>
struct lh_cps_flat {
    __device__ __forceinline__ static void run(const lh_word (&acc)[LH_M][8], unsigned char *slot,
                                               unsigned char *__restrict__ out, long long out_stride, long long s0,
                                               int nst, int sl, int c, bool last) {
        if constexpr (R0 < LH_M) {
            constexpr int nr = (LH_M - R0) < LH_CRP ? (LH_M - R0) : LH_CRP;
            unsigned char *img = slot + (sl < LH_SPW ? sl : LH_SPW - 1) * (nr * LH_BYTES) + (last ? LH_SUB - 8 : 8 * c);
#pragma unroll
            for (int r = 0; r < nr; ++r) lh_img_row<0>(img + r * LH_BYTES, acc[R0 + r], last, sl < nst);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the image is complete
            constexpr int per = nr * LH_BYTES / 16;  // chunks per stripe
            const int n = nst * per, lane = threadIdx.x & 63;
#pragma unroll
            for (int q = 0; q < (LH_SPW * per + 63) / 64; ++q) {
                const int j = 64 * q + lane;
                if (j < n) {
                    const int js = j / per, t = j - js * per;
                    const lh_u32x4a v = *(const lh_u32x4a *)(slot + j * 16);
                    unsigned char *dst = out + (s0 + js) * out_stride + R0 * LH_BYTES + t * 16;
#if LH_NT_ST
                    __builtin_nontemporal_store(v, (lh_u32x4a *)dst);
#else
                    *(lh_u32x4a *)dst = v;
#endif
                }
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the slot's reads are done
            lh_cps_flat<R0 + nr>::run(acc, slot, out, out_stride, s0, nst, sl, c, last);
        }
    }
};
#endif
__device__ __forceinline__ void lh_encode_wave_cps(long long wave, const unsigned char *__restrict__ in,
                                                   long long in_stride, unsigned char *__restrict__ out,
                                                   long long out_stride, int stripes) {
    __shared__ __attribute__((aligned(16))) unsigned char lh_cring[LH_WPB][(1 + LH_CPS_AHEAD) * LH_SSLOT];
    const int lane = threadIdx.x & 63;
    const int sl = lane / LH_NCH, c = lane - sl * LH_NCH;
    const long long s0 = (long long)__builtin_amdgcn_readfirstlane((int)wave) * LH_SPW;  // wave-uniform
    if (s0 >= stripes) return;  // wave-uniform
    const int nst = (int)((stripes - s0) < LH_SPW ? (stripes - s0) : LH_SPW);
    unsigned char *slot = lh_cring[lh_wid<0>()];
    const lh_u32x4r rs = lh_rsrc(in + s0 * in_stride, (unsigned)(nst * in_stride));
    int voff[LH_SQ];
#pragma unroll
    for (int q = 0; q < LH_SQ; ++q) {  // chunk j = 64 q + lane of the slot image [stripe][LH_CPS x bytes]
        const int j = 64 * q + lane, js = j / LH_SCH, r = j - js * LH_SCH;
        voff[q] = js < nst ? js * (int)in_stride + r * 16 : (int)0x80000000;
    }
    // step 0 (LH_NSTEP >= 2: LH_K >= 2 LH_CPS is required by the host)
#pragma unroll
    for (int q = 0; q < LH_SQ; ++q) lh_dma16_bufs<LH_NT>(rs, voff[q], 0, slot + q * 1024);
    lh_word acc[LH_M][8];
#pragma unroll
    for (int r = 0; r < LH_M; ++r)
#pragma unroll
        for (int y = 0; y < 8; ++y)
#pragma unroll
            for (int i = 0; i < LH_NW; ++i) acc[r][y].v[i] = 0;
    const int lo = (sl < LH_SPW ? sl : LH_SPW - 1) * (LH_CPS * LH_BYTES) + 8 * c;
    int lo8 = lo + 8;
    asm volatile("" : "+v"(lo8));
    lh_unroll_cps<0>::run(acc, rs, voff, slot, lo, lo8);
    const bool last = c == LH_NCH - 1;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // every slot read of the last step done
#if LH_CPS_FLAT && LH_CRP >= 1
    // The recovery blocks leave through the slot, LH_CRP rows at a time ([stripe][row][bytes]
    // images, 16-byte stores of contiguous runs; a stripe's rows are contiguous in memory).
    lh_cps_flat<0>::run(acc, slot, out, out_stride, s0, nst, sl, c, last);
#else
    if (sl >= nst) return;
    const int p = last ? LH_SUB - 8 : 8 * c;
    unsigned char *o = out + (s0 + sl) * out_stride + p;
#pragma unroll
    for (int r = 0; r < LH_M; ++r)
#pragma unroll
        for (int y = 0; y < 8; ++y) {
            lh_word w = acc[r][y];
            if constexpr (LH_VLAST != 8) {
                const lh_word f = lh_funnel<LH_VLAST>(lh_row_shr1(w.v[0]), lh_row_shr1(w.v[1]), w.v[0], w.v[1]);
                w.v[0] = last ? f.v[0] : w.v[0];
                w.v[1] = last ? f.v[1] : w.v[1];
            }
            lh_store(o + (long long)r * LH_BYTES + y * LH_SUB, w);
            // (stores kept in address order: a line two neighbouring sub-rows share then gets
            // both halves back to back; reordered by the scheduler, the non-temporal halves
            // left as partial-line writes, +14 MB per k29/m4 launch, profiles/r10x/r10y PMC)
            asm volatile("" ::: "memory");
        }
#endif
}
#endif  // LH_CPS

#endif

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
    lh_esrc S;
#if LH_BUF
#if LH_NCH <= 64
    const long long s0 = (long long)__builtin_amdgcn_readfirstlane((int)wave) * LH_SPW;  // wave-uniform
    const long long nst = (stripes - s0) < LH_SPW ? (stripes - s0) : LH_SPW;
#else
    const long long s0 = (long long)__builtin_amdgcn_readfirstlane((int)(wave / LH_WPS));
    const long long nst = 1;
#endif
    S.rs = __builtin_amdgcn_make_buffer_rsrc((void *)(in + s0 * in_stride), 0, (int)(nst * in_stride), 0x00020000);
    S.lbase = (int)((l.stripe - s0) * in_stride) + l.p;
#elif LH_PTR
    S.pt = lh_ptab(l, in, in_stride, nullptr);
    S.p = l.p;
#else
    S.base = in + l.stripe * in_stride + l.p;
#endif
    lh_word ring[LH_PF][8];
#pragma unroll
    for (int q = 0; q < LH_PF; ++q)
        if (q < LH_K) S.load8(ring[q], q);
    lh_unroll_encode<0>::run(acc, ring, S);
#if LH_PTR
    // out: the recovery blocks' pointer table, LH_M per stripe (row stride out_stride bytes)
    const unsigned long long *ot = (const unsigned long long *)(out + l.stripe * out_stride);
#pragma unroll
    for (int r = 0; r < LH_M; ++r) {
        unsigned char *o = (unsigned char *)ot[r] + l.p;
#pragma unroll
        for (int y = 0; y < 8; ++y) lh_store(o + y * LH_SUB, acc[r][y]);
    }
    return;
#endif
    unsigned char *o = out + l.stripe * out_stride + l.p;
#pragma unroll
    for (int r = 0; r < LH_M; ++r)
#pragma unroll
        for (int y = 0; y < 8; ++y) lh_store(o + (long long)r * LH_BYTES + y * LH_SUB, acc[r][y]);
}

// LH_ROLE (jit.cpp): 1 = the encode module, 2 = the decode module (LH_DEC_PLAIN: lh_jit_decode,
// else lh_jit_decode_fused); undefined (the build-time syntax check) = every kernel.
#ifndef LH_ROLE
#define LH_ROLE 0
#define LH_DEC_PLAIN 0
#endif
// ------------------------------------------------------------ block-size family (LH_FAMILY)
// One module per (k, m) serves every 16-byte-multiple block size whose sub-blocks fit 8-byte
// lanes with at most 64 lanes per stripe (bytes <= 4096): the multi-column-step encode above
// with the block size a kernel argument (the reference serves any size at full
// speed on its first call, cauchy_256.cpp:423-481).  Run-time per wave (all wave-uniform):
// sub = bytes / 8, lanes per stripe nch = ceil(sub / 8), stripes per wave spw = 64 / nch, DMA
// instructions per step sq = ceil(spw x LH_CPS x bytes / 1024) <= 4 LH_CPS (spw x bytes <=
// 4096).  A lane's LDS word of sub-block B sits (B x sub) mod 8 bytes past an 8-byte boundary:
// with even sub that is one of four patterns, so each column's LDS reads are one of four
// compile-time funnel forms picked by a wave-uniform branch on sub mod 8; the XOR network is
// shared.  The sub-block addresses (lane offset + B x sub, aligned) are 16 per-lane registers
// computed once; a column adds its offset in the slot.
#ifndef LH_FAMILY
#define LH_FAMILY 0
#endif
#if LH_FAMILY
#ifndef LH_FAM_SPLIT
#define LH_FAM_SPLIT 0
#endif
#if LH_FAM_SPLIT
#define LH_FAM_AD8 ad8[b]
#else
#define LH_FAM_AD8 (ad[b] + 8)
#endif
struct lh_fam {
    int bytes, sub, nch, spw, sch, sq, r8;
};
// The 8 sub-block words of one column, sub mod 8 = R (compile-time form): `ad[b]` is the lane's
// LDS address of sub-block b's first aligned word in this column, computed once per wave
// (sub-block b starts b x sub = b (sub - R) + b R bytes in: the first part a multiple of 8, the
// second a constant).  All reads are issued before any is used (the empty asm takes every
// word): left alone, the compiler placed each read next to its use with a wait of its own,
// which with one wave per SIMD exposed the LDS latency 16 times per column (k29/m4 encode
// 0.587 ms).
template <int R>
__device__ __forceinline__ void lh_fam_col(lh_word (&d)[8], const unsigned char *slot, const int (&ad)[8],
                                           const int (&ad8)[8]) {
    lh_u32x2a x[8], y[8];
#pragma unroll
    for (int b = 0; b < 8; ++b) {
        x[b] = *(const lh_u32x2a *)(slot + ad[b] + ((b * R) & ~7));
        if (((b * R) & 7) != 0) y[b] = *(const lh_u32x2a *)(slot + LH_FAM_AD8 + ((b * R) & ~7));
    }
#pragma unroll
    for (int b = 0; b < 8; ++b) {
        asm volatile("" : "+v"(x[b]));
        if (((b * R) & 7) != 0) asm volatile("" : "+v"(y[b]));
    }
#pragma unroll
    for (int b = 0; b < 8; ++b) {
        const int S = (b * R) & 7;  // (constant after unrolling)
        if (S == 0) {
            d[b].v[0] = x[b].x;
            d[b].v[1] = x[b].y;
        } else if (S == 2) {
            d[b] = lh_funnel<2>(x[b].x, x[b].y, y[b].x, y[b].y);
        } else if (S == 4) {
            d[b] = lh_funnel<4>(x[b].x, x[b].y, y[b].x, y[b].y);
        } else {
            d[b] = lh_funnel<6>(x[b].x, x[b].y, y[b].x, y[b].y);
        }
    }
}
#endif  // LH_FAMILY
#if LH_FAMILY && LH_ROLE != 2
#define LH_FSQ (4 * LH_CPS)  // DMA instructions per step, at most
template <int T, int CC, int R>
struct lh_fam_cols {
    __device__ __forceinline__ static void run(lh_word (&acc)[LH_M][8], const unsigned char *slot,
                                               const int (&ad)[LH_CPS][8], const int (&ad8)[LH_CPS][8]) {
        if constexpr (CC < LH_CPS && T * LH_CPS + CC < LH_K) {
            lh_word d[8];
            lh_fam_col<R>(d, slot, ad[CC], ad8[CC]);
            lh_column<T * LH_CPS + CC>(acc, d);
            lh_opaque(acc);
            lh_fam_cols<T, CC + 1, R>::run(acc, slot, ad, ad8);
        }
    }
};
template <int T, int R>
struct lh_unroll_fam {
    __device__ __forceinline__ static void run(lh_word (&acc)[LH_M][8], const lh_u32x4r &rs, const int (&voff)[LH_FSQ],
                                               const int (&voffl)[LH_FSQ], unsigned char *slot, const lh_fam &F,
                                               const int (&ad)[LH_CPS][8], const int (&ad8)[LH_CPS][8]) {
        if constexpr (T < LH_NSTEP) {
            lh_wait_vmcnt<0>();  // this step's DMAs landed (the only ones in flight)
            asm volatile("" ::: "memory");
            lh_fam_cols<T, 0, R>::run(acc, slot, ad, ad8);
            if constexpr (T + 1 < LH_NSTEP) {
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the slot's reads are done
                const int x1b = (T + 1) * LH_CPS * F.bytes;
#pragma unroll
                for (int q = 0; q < LH_FSQ; ++q) {
                    if (q < F.sq) {  // wave-uniform
                        // (the last step: the chunks of columns < LH_K only)
                        const int v = (T + 2 == LH_NSTEP && LH_LASTC < LH_CPS) ? voffl[q] : voff[q];
                        int off = q * 1024;  // (opaque: no SGPR held per chunk address for the whole kernel)
                        asm volatile("" : "+s"(off));
                        lh_dma16_bufs<LH_NT>(rs, v, x1b, slot + off);
                    }
                }
            }
            lh_unroll_fam<T + 1, R>::run(acc, rs, voff, voffl, slot, F, ad, ad8);
        }
    }
};
// The recovery blocks from the accumulators, per lane; the last lane of a stripe keeps the
// sub-block's last VL (= sub - 8 (nch - 1)) bytes, funnelled with its neighbour's word.
template <int VL>
__device__ __forceinline__ void lh_fam_store(const lh_word (&acc)[LH_M][8], unsigned char *o, const lh_fam &F, bool last) {
#pragma unroll
    for (int r = 0; r < LH_M; ++r)
#pragma unroll
        for (int y = 0; y < 8; ++y) {
            lh_word w = acc[r][y];
            if constexpr (VL != 8) {
                const lh_word f = lh_funnel<VL>(lh_row_shr1(w.v[0]), lh_row_shr1(w.v[1]), w.v[0], w.v[1]);
                w.v[0] = last ? f.v[0] : w.v[0];
                w.v[1] = last ? f.v[1] : w.v[1];
            }
            lh_store(o + (long long)r * F.bytes + y * F.sub, w);
            asm volatile("" ::: "memory");  // (in address order, as lh_encode_wave_cps's stores)
        }
}
// One wave's stripes; R = sub mod 8 (0, 2, 4 or 6), a compile-time form chosen once per launch,
// so every column's LDS reads are scheduled as in the size-specialised kernel.
template <int R>
__device__ __forceinline__ void lh_encode_wave_fam(long long wave, const lh_fam &F, const unsigned char *__restrict__ in,
                                                   long long in_stride, unsigned char *__restrict__ out,
                                                   long long out_stride, int stripes, unsigned char *slot) {
    const int lane = threadIdx.x & 63;
    const int sl = lane / F.nch, c = lane - sl * F.nch;
    const long long s0 = (long long)__builtin_amdgcn_readfirstlane((int)wave) * F.spw;  // wave-uniform
    if (s0 >= stripes) return;
    const int nst = (int)((stripes - s0) < F.spw ? (stripes - s0) : F.spw);
    const lh_u32x4r rs = lh_rsrc(in + s0 * in_stride, (unsigned)(nst * in_stride));
    int voff[LH_FSQ], voffl[LH_FSQ];  // (voffl: the last step's, chunks past column LH_K out of range)
    const float inv = 1.0f / (float)F.sch;  // (j < 2^12: the float quotient is off by at most one)
#pragma unroll
    for (int q = 0; q < LH_FSQ; ++q) {
        const int j = 64 * q + lane;
        int js = (int)((float)j * inv);
        js -= js * F.sch > j;
        js += (js + 1) * F.sch <= j;
        const int r = j - js * F.sch;
        voff[q] = js < nst ? js * (int)in_stride + r * 16 : (int)0x80000000;
        voffl[q] = r < LH_LASTC * (F.bytes >> 4) ? voff[q] : (int)0x80000000;
    }
#pragma unroll
    for (int q = 0; q < LH_FSQ; ++q)
        if (q < F.sq) {
            int off = q * 1024;
            asm volatile("" : "+s"(off));
            lh_dma16_bufs<LH_NT>(rs, voff[q], 0, slot + off);
        }
    lh_word acc[LH_M][8];
#pragma unroll
    for (int r = 0; r < LH_M; ++r)
#pragma unroll
        for (int y = 0; y < 8; ++y)
#pragma unroll
            for (int i = 0; i < LH_NW; ++i) acc[r][y].v[i] = 0;
    const int lo = (sl < F.spw ? sl : F.spw - 1) * (LH_CPS * F.bytes) + 8 * c;
    // column cc, sub-block b: lo + cc bytes + b (sub - R) (the constant part in the reads).
    // LH_FAM_SPLIT: the second word's address in registers of its own, hidden from the compiler
    // (two ds_read_b64, 2 LDS cycles each, instead of one ds_read2_b64, 8) -- measured slower
    // here (0.540 against 0.529 ms), unlike in the size-specialised kernels.
    int ad[LH_CPS][8], ad8[LH_CPS][8];
#pragma unroll
    for (int cc = 0; cc < LH_CPS; ++cc)
#pragma unroll
        for (int b = 0; b < 8; ++b) {
            ad[cc][b] = lo + cc * F.bytes + b * (F.sub - R);
            ad8[cc][b] = ad[cc][b] + 8;
#if LH_FAM_SPLIT
            asm volatile("" : "+v"(ad8[cc][b]));
#endif
        }
    lh_unroll_fam<0, R>::run(acc, rs, voff, voffl, slot, F, ad, ad8);
    if (sl >= nst) return;
    const bool last = c == F.nch - 1;
    unsigned char *o = out + (s0 + sl) * out_stride + (last ? F.sub - 8 : 8 * c);
    lh_fam_store<R == 0 ? 8 : R>(acc, o, F, last);  // (sub - 8 (nch - 1) = R, or 8 when R = 0)
}
template <int R>
__device__ __forceinline__ void lh_encode_fam(const lh_fam &F, const unsigned char *__restrict__ in, long long in_stride,
                                              unsigned char *__restrict__ out, long long out_stride, int stripes,
                                              unsigned char *slot) {
    const long long nw = ((long long)stripes + F.spw - 1) / F.spw;
    const long long ws = (long long)gridDim.x * (blockDim.x >> 6);
    for (long long w = (lh_block_id() * blockDim.x + threadIdx.x) >> 6; w < nw; w += ws)
        lh_encode_wave_fam<R>(w, F, in, in_stride, out, out_stride, stripes, slot);
}
extern "C" __global__ void __launch_bounds__(256, 1)
lh_jit_encode(const unsigned char *__restrict__ in, long long in_stride, unsigned char *__restrict__ out,
              long long out_stride, int stripes, int bytes) {
    lh_fam F;
    F.bytes = bytes;
    F.sub = bytes >> 3;
    F.nch = (F.sub + 7) >> 3;
    F.spw = 64 / F.nch;
    F.sch = LH_CPS * (bytes >> 4);
    F.sq = (F.spw * F.sch + 63) >> 6;
    F.r8 = F.sub & 7;
    __shared__ __attribute__((aligned(16))) unsigned char lh_fring[LH_WPB][LH_FSQ * 1024 + 16];
    // (the wave index made wave-uniform explicitly, so the DMAs' LDS addresses live in SGPRs:
    // as the decode's family, lh_jit_decode_fused below)
    unsigned char *slot = lh_fring[__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6))];
    switch (F.r8) {  // (launch-uniform; bytes % 16 == 0 makes sub even)
        case 0: lh_encode_fam<0>(F, in, in_stride, out, out_stride, stripes, slot); break;
        case 2: lh_encode_fam<2>(F, in, in_stride, out, out_stride, stripes, slot); break;
        case 4: lh_encode_fam<4>(F, in, in_stride, out, out_stride, stripes, slot); break;
        default: lh_encode_fam<6>(F, in, in_stride, out, out_stride, stripes, slot); break;
    }
}
#endif  // LH_FAMILY

#if LH_ROLE != 2 && !LH_FAMILY
// recovery[s][r] = sum_x B(G[r][x]) data[s][x]   (cauchy_256_encode for m > 1, valid k, m)
#ifndef LH_ENC_LB
#define LH_ENC_LB 1  // min waves per SIMD the register allocator must allow (tools/tune.py)
#endif
#ifndef LH_WPB
#define LH_WPB 4
#endif
extern "C" __global__ void __launch_bounds__(LH_WPB > 4 ? 64 * LH_WPB : 256, LH_ENC_LB)
lh_jit_encode(const unsigned char *__restrict__ in, long long in_stride,
              unsigned char *__restrict__ out, long long out_stride, int stripes) {
#if LH_LDS && LH_CPS > 1 && !LH_PTR
    LH_WAVE_LOOP(stripes) { lh_encode_wave_cps(lh_w, in, in_stride, out, out_stride, stripes); }
#elif LH_LDS
    LH_WAVE_LOOP(stripes) { lh_encode_wave_lds(lh_w, in, in_stride, out, out_stride, stripes); }
#else
    LH_WAVE_LOOP(stripes) { lh_encode_wave(lh_w, in, in_stride, out, out_stride, stripes); }
#endif
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

// Phase A streams the LH_M recovery rows (absent ones read as zeros) and the LH_K data
// columns (erased ones read as zeros) through one prefetch ring (order: LH_REC_FIRST).
#define LH_DCOLS (LH_K + LH_M)
#ifndef LH_PF_DEC
#define LH_PF_DEC 1  // decode prefetch depth (tools/tune.py, fused plan: 1 >= 2 > 3)
#endif
#ifndef LH_PREP_FIRST
#define LH_PREP_FIRST 0  // fused decode: solve the plan before (1) or while (0) the first columns load
#endif
#if LH_BUF
// Column source of a wave: one buffer resource over the wave's stripes (wave-uniform base,
// num_records = their bytes; the host keeps that below 2^31).  An absent column (erased
// original, missing recovery row) gets an out-of-range offset, which the hardware answers
// with zeros without a memory request -- no zero page and no extra L2 traffic -- and every
// column address is one 32-bit offset instead of a 64-bit pointer.
struct lh_dsrc {
    __amdgpu_buffer_rsrc_t rs;
    int lbase;  // this lane's offset: (stripe - first stripe of the wave) * stride + chunk
    __device__ __forceinline__ int col(unsigned int slot) const {
        return slot == 0xFFu ? (int)0x80000000 : lbase + (int)slot * LH_BYTES;
    }
};
// NT: non-temporal loads for this column.  LH_NT_DEC == 2: data columns non-temporal (read
// once, never written), recovery rows -- the slots the outputs overwrite -- default policy.
template <bool NT = (LH_NT_DEC == 1)>
__device__ __forceinline__ void lh_load_col(lh_word (&d)[8], const lh_dsrc &S, unsigned int slot) {
    const int off = S.col(slot);
#pragma unroll
    for (int b = 0; b < 8; ++b) d[b] = lh_load_buf<NT ? 2 : 0>(S.rs, off + b * LH_SUB);
}
#else
// Column source of a lane: its stripe's chunk pointer (LH_PTR: its stripe's block pointers
// in LDS and its chunk offset) and the zero page.
struct lh_dsrc {
#if LH_PTR
    const unsigned long long *pt;  // LDS: the stripe's block pointers, then the zero page
    int p;
    __device__ __forceinline__ const unsigned char *col(unsigned int slot) const {
        return (const unsigned char *)pt[lh_late(slot == 0xFFu ? LH_K : (int)slot)] + p;
    }
#else
    const unsigned char *base, *zero;
    __device__ __forceinline__ const unsigned char *col(unsigned int slot) const {
        return (slot == 0xFFu) ? zero : base + (long long)slot * LH_BYTES;
    }
#endif
};
#ifndef LH_ZSKIP
#define LH_ZSKIP 0  // lanes of absent columns skip the zero-page load (exec-masked)
#endif
__device__ __forceinline__ void lh_load_col(lh_word (&d)[8], const lh_dsrc &S, unsigned int slot) {
    const unsigned char *src = S.col(slot);
#if LH_ZSKIP
    if (slot != 0xFFu) {
#pragma unroll
        for (int b = 0; b < 8; ++b) d[b] = lh_load_dec(src + b * LH_SUB);
    } else {
#pragma unroll
        for (int b = 0; b < 8; ++b)
#pragma unroll
            for (int i = 0; i < LH_NW; ++i) d[b].v[i] = 0;
    }
#else
#pragma unroll
    for (int b = 0; b < 8; ++b) d[b] = lh_load_dec(src + b * LH_SUB);
#endif
}
#endif

// Column order of phase A.  LH_REC_FIRST = 1: the m recovery rows first, then the k data
// columns.  The outputs overwrite the recovery slots; read last, those lines are still in
// L2 when the stores arrive, and in-place stores into L2-resident clean lines measured
// slower than into lines long evicted (tools/ubench_decode.hip, k29/m4 access pattern:
// 0.613 ms recovery rows last, 0.586 ms first, 0.574 ms into a separate buffer).
#ifndef LH_REC_FIRST
#define LH_REC_FIRST 1
#endif
// Decode column X in stream order: data column x (the slot holding original x) or
// recovery row r.
template <int X, int RF = LH_REC_FIRST>
struct lh_dcol {
    static constexpr bool rec = RF ? (X < LH_M) : (X >= LH_K);
    static constexpr int idx = RF ? (X < LH_M ? X : X - LH_M) : (X < LH_K ? X : X - LH_K);
    static constexpr int x = rec ? 0 : (idx < LH_K ? idx : 0);
    static constexpr int r = rec ? (idx < LH_M ? idx : 0) : 0;
};
template <int X>
__device__ __forceinline__ unsigned int lh_dcol_slot(const unsigned int (&srcw)[LH_NSRC],
                                                     const unsigned int (&recw)[LH_NREC]) {
    if (lh_dcol<X>::rec) return LH_BYTE(recw, lh_dcol<X>::r);
    return LH_BYTE(srcw, lh_dcol<X>::x);
}

template <int X, int RF = LH_REC_FIRST>
__device__ __forceinline__ void lh_dcombine(lh_word (&acc)[LH_M][8], const lh_word (&d)[8]) {
    if constexpr (lh_dcol<X, RF>::rec) {
#pragma unroll
        for (int y = 0; y < 8; ++y) lh_xor(acc[lh_dcol<X, RF>::r][y], d[y]);
    } else {
        lh_column<lh_dcol<X, RF>::x>(acc, d);
    }
}

template <int X, int PF>
struct lh_unroll_decode {
    __device__ __forceinline__ static void run(lh_word (&acc)[LH_M][8], lh_word (&ring)[PF][8],
                                               const lh_dsrc &S, const unsigned int (&srcw)[LH_NSRC],
                                               const unsigned int (&recw)[LH_NREC]) {
        if constexpr (X >= LH_DCOLS) {
            return;
        } else {
            if (X + PF < LH_DCOLS) {
                lh_word nxt[8];
#if LH_BUF
                lh_load_col<LH_NT_DEC == 1 || (LH_NT_DEC == 2 && !lh_dcol<(X + PF < LH_DCOLS ? X + PF : 0)>::rec)>(
                    nxt, S, lh_dcol_slot<(X + PF < LH_DCOLS ? X + PF : 0)>(srcw, recw));
#else
                lh_load_col(nxt, S, lh_dcol_slot<(X + PF < LH_DCOLS ? X + PF : 0)>(srcw, recw));
#endif
                lh_dcombine<X>(acc, ring[X % PF]);
                lh_dopaque(acc);
#pragma unroll
                for (int b = 0; b < 8; ++b) ring[X % PF][b] = nxt[b];
            } else {
                lh_dcombine<X>(acc, ring[X % PF]);
                lh_dopaque(acc);
            }
            lh_unroll_decode<X + 1, PF>::run(acc, ring, S, srcw, recw);
        }
    }
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
// Decode pieces.  Ring issue: the first PF columns of a stripe group (PF <= 4).
template <int PF>
__device__ __forceinline__ void lh_dec_issue(lh_word (&ring)[PF][8], const lh_plan_regs &pr, const lh_dsrc &S) {
    static_assert(PF >= 1 && PF <= 4, "decode prefetch depth");
#pragma unroll
    for (int q = 0; q < PF; ++q) {
        const unsigned int slot = (q == 0) ? lh_dcol_slot<0>(pr.srcw, pr.recw)
                                : (q == 1) ? lh_dcol_slot<1>(pr.srcw, pr.recw)
                                : (q == 2) ? lh_dcol_slot<2>(pr.srcw, pr.recw)
                                           : lh_dcol_slot<3>(pr.srcw, pr.recw);
#if LH_BUF
        lh_load_col<LH_NT_DEC == 1 || (LH_NT_DEC == 2 && !LH_REC_FIRST)>(ring[q], S, slot);
#else
        lh_load_col(ring[q], S, slot);
#endif
    }
}

// Phase A: V_r = R_r + sum_{x present} B(G[r][x]) D_x for every recovery row r, streaming
// the ring (already issued) through all k + m columns.
template <int PF>
__device__ __forceinline__ void lh_dec_phase_a(lh_word (&v)[LH_M][8], lh_word (&ring)[PF][8],
                                               const lh_plan_regs &pr, const lh_dsrc &S) {
#pragma unroll
    for (int r = 0; r < LH_M; ++r)
#pragma unroll
        for (int y = 0; y < 8; ++y)
#pragma unroll
            for (int i = 0; i < LH_NW; ++i) v[r][y].v[i] = 0;
    lh_unroll_decode<0, PF>::run(v, ring, S, pr.srcw, pr.recw);
}

// Phase B: D_{E_i} = sum_r B(coef[i][r]) V_r with the per-stripe inverse, by Horner over
// the coefficient bits: B(c) v = B(2)(...B(2)(c_7 v)...) + c_0 v, one v_bitop3 masked XOR
// per (row, bit, sub-row); the recovered blocks go to the plan's output slots.
struct lh_dsrc;
__device__ __forceinline__ void lh_dec_phase_b(const lh_word (&v)[LH_M][8], const lh_plan_regs &pr,
                                               unsigned char *base, bool last, const lh_dsrc &S, int soff) {
    (void)last;
    (void)S;
    (void)soff;
    const int e = pr.e;
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
#if LH_PIN_WORDS & 2
                lh_pin8w(o);
#else
                lh_pin8(o);
#endif
            }
#if LH_PTR
            unsigned char *dst = (unsigned char *)S.pt[LH_BYTE(outw, i)] + soff;  // soff: the lane's store offset
#else
            unsigned char *dst = base + (long long)LH_BYTE(outw, i) * LH_BYTES;
#endif
#pragma unroll
            for (int y = 0; y < 8; ++y) lh_store(dst + y * LH_SUB, o[y]);
        }
    }
}

// Column source of lane `l` (stripe l.stripe, chunk l.p) of wave `wave`.
__device__ __forceinline__ lh_dsrc lh_make_dsrc(const lh_lane &l, long long wave, unsigned char *__restrict__ blocks,
                                               long long stripe_stride, const unsigned char *__restrict__ zero_page,
                                               int stripes) {
    lh_dsrc S;
#if LH_BUF
#if LH_NCH <= 64
    const long long s0 = (long long)__builtin_amdgcn_readfirstlane((int)wave) * LH_SPW;  // wave-uniform
    const long long nst = (stripes - s0) < LH_SPW ? (stripes - s0) : LH_SPW;
#else
    const long long s0 = (long long)__builtin_amdgcn_readfirstlane((int)(wave / LH_WPS));
    const long long nst = 1;
#endif
    S.rs = __builtin_amdgcn_make_buffer_rsrc(blocks + s0 * stripe_stride, 0, (int)(nst * stripe_stride), 0x00020000);
    S.lbase = (int)((l.stripe - s0) * stripe_stride) + l.p;
#elif LH_PTR
    S.pt = lh_ptab(l, blocks, stripe_stride, zero_page);
    S.p = l.p;
#else
    S.base = blocks + l.stripe * stripe_stride + l.p;
    S.zero = zero_page + l.p;
#endif
    return S;
}

// In-place erasure decode of one stripe group: ring issue, `prep` (the fused kernel
// solves its plan there, while the first columns are in flight), phase A, phase B.
template <int PF, class PREP>
__device__ __forceinline__ void lh_decode_body(const lh_lane &l, long long wave, unsigned char *__restrict__ blocks,
                                               long long stripe_stride, lh_plan_regs &pr,
                                               const unsigned char *__restrict__ zero_page, int stripes,
                                               const PREP &prep) {
    const lh_dsrc S = lh_make_dsrc(l, wave, blocks, stripe_stride, zero_page, stripes);
    lh_word v[LH_M][8];
    {
#if LH_PREP_FIRST
        prep(pr);  // solve before the first loads: the ring is not live across the solve
#endif
        lh_word ring[PF][8];
        lh_dec_issue<PF>(ring, pr, S);
#if !LH_PREP_FIRST
        prep(pr);
#endif
        lh_dec_phase_a<PF>(v, ring, pr, S);
    }
#if LH_BUF
    lh_dec_phase_b(v, pr, blocks + l.stripe * stripe_stride + l.p, l.last, S, S.lbase - l.p);
#elif LH_PTR
    lh_dec_phase_b(v, pr, nullptr, l.last, S, l.p);
#else
    lh_dec_phase_b(v, pr, blocks + l.stripe * stripe_stride + l.p, l.last, S, 0);
#endif
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
    lh_decode_body<LH_PF_DEC>(l, wave, blocks, stripe_stride, pr, zero_page, stripes, lh_no_prep());
}

#if LH_ROLE == 0 || (LH_ROLE == 2 && (LH_DEC_PLAIN || !(LH_EMAX <= 4 && LH_NCH <= 64 && LH_K <= 64)))
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
#ifndef LH_DWPB
#define LH_DWPB 4  // waves per workgroup of the fused decode (strided batches; jit.cpp dec_wpb)
#endif
static constexpr unsigned char LH_GRAW[LH_M][LH_K] = LH_G_INIT;
#define LH_P4(n) (((n) + 3) / 4 * 4)
#define LH_SR (2 * LH_P4(LH_K) + LH_P4(LH_M))  // per-stripe scratch: rows | src map | rec map
#define LH_NRW ((LH_K + LH_NCH - 1) / LH_NCH)    // Block.row bytes per lane
// Lanes of one stripe as a ballot mask (LH_NCH may be 64: a 64-bit shift by 64 is UB).
#define LH_STRIPE_LANES (LH_NCH >= 64 ? ~0ull : ((1ull << (LH_NCH & 63)) - 1))

// Stripe geometry of the fused plan: lanes per stripe (nch), Block.row bytes per lane
// (nrw = ceil(LH_K / nch), at most maxrw) and a stripe's lanes as a ballot mask.  Compile-time
// constants in the size-specialised modules (lh_gct), run-time values in the block-size family
// (lh_grt, below).
struct lh_gct {
    static constexpr int nch = LH_NCH, nrw = LH_NRW, maxrw = LH_NRW;
    static constexpr unsigned long long lanes = LH_STRIPE_LANES;
};

// The lane's Block.row bytes (slots c, c + nch, ...), loaded ahead of the plan.
template <class G>
__device__ __forceinline__ void lh_fused_rows(const G &g, const lh_lane &l, int c, const unsigned char *__restrict__ rows,
                                              unsigned int (&rowv)[G::maxrw]) {
    const unsigned char *grow = rows + l.stripe * LH_K;
#pragma unroll
    for (int t = 0; t < G::maxrw; ++t) {
        const int i = c + t * g.nch;
        rowv[t] = (l.active && t < g.nrw && i < LH_K) ? (unsigned int)grow[i] : 0u;
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
    const unsigned char *gmat;  // LDS copy of LH_GRAW: a lookup from the code object's constant
                                // memory is a global load whose wait (vmcnt) would also drain
                                // the first columns' DMAs issued just before the solve
    int c;
    __device__ __forceinline__ void operator()(lh_plan_regs &pr) const;
};

// Part 1: slot maps, validity and the erasure / recovery lists.  Returns false when the
// stripe has nothing to do (no erasure or invalid rows).
template <class G>
__device__ __forceinline__ bool lh_fused_plan(const G &g, const lh_lane &l, int c, int sl, unsigned char *scr,
                                              const unsigned int (&rowv)[G::maxrw],
                                              unsigned char *__restrict__ rows, signed char *__restrict__ status,
                                              lh_fused_solve &sv, lh_plan_regs &pr) {
    unsigned char *lrows = scr;
    unsigned char *lsrc = scr + LH_P4(LH_K);
    unsigned char *lrec = lsrc + LH_P4(LH_K);
    unsigned char *grow = rows + l.stripe * LH_K;
    // Clear the maps (0xFF = absent), then every lane records the rows of its slots.
    for (int q = c; q < (LH_P4(LH_K) + LH_P4(LH_M)) / 4; q += g.nch) ((unsigned int *)lsrc)[q] = 0xFFFFFFFFu;
    bool bad = false;
#pragma unroll
    for (int t = 0; t < G::maxrw; ++t) {
        const int i = c + t * g.nch;
        if (t >= g.nrw || i >= LH_K) continue;
        const unsigned int r = rowv[t];
        lrows[i] = (unsigned char)r;
        if (r < LH_K) lsrc[r] = (unsigned char)i;
        else if (r < LH_K + LH_M) lrec[r - LH_K] = (unsigned char)i;
        else bad = true;
    }
    for (int i = c; i < LH_K; i += g.nch) {  // a repeated row leaves another slot in the map
        const unsigned int r = lrows[i];
        if (r < LH_K + LH_M && (r < LH_K ? lsrc[r] : lrec[r - LH_K]) != i) bad = true;
    }
    const unsigned long long lanes_bad = __ballot(bad);
    const unsigned long long my = g.lanes << (sl * g.nch);
    const bool invalid = (lanes_bad & my) != 0;
    // Recovery slots in array order and missing originals ascending, as per-stripe bit
    // masks gathered with wave ballots (slot/row i = c + t * nch), then unpacked by
    // lowest-set-bit extraction.
    unsigned long long rcvmask = 0, ermask = 0;
#pragma unroll
    for (int t = 0; t < G::maxrw; ++t) {
        if (t >= g.nrw) break;  // (uniform; never taken in the size-specialised modules)
        const int i = c + t * g.nch;
        const bool isrcv = (i < LH_K) && (lrows[i] >= LH_K);
        const bool iser = (i < LH_K) && (lsrc[i] == 0xFF);
        rcvmask |= ((__ballot(isrcv) >> (sl * g.nch)) & g.lanes) << (t * g.nch);
        ermask |= ((__ballot(iser) >> (sl * g.nch)) & g.lanes) << (t * g.nch);
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
#ifndef LH_PROBE_NOMETA
#define LH_PROBE_NOMETA 0  // (probe, wrong rows / status: neither written -- their share of the HBM writes)
#endif
    if (c == 0 && status && !LH_PROBE_NOMETA) status[l.stripe] = 0;
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

#ifndef LH_SOLVE_GJ
#define LH_SOLVE_GJ 0  // fused planner: Gauss-Jordan instead of the adjugate inverse (A/B knob)
#endif

// Permutations of n <= 3 elements, for the cofactor expansion below.
template <int n> struct lh_perms;
template <> struct lh_perms<0> { static constexpr int cnt = 1; static constexpr int p[1][1] = {{0}}; };
template <> struct lh_perms<1> { static constexpr int cnt = 1; static constexpr int p[1][1] = {{0}}; };
template <> struct lh_perms<2> { static constexpr int cnt = 2; static constexpr int p[2][2] = {{0, 1}, {1, 0}}; };
template <> struct lh_perms<3> {
    static constexpr int cnt = 6;
    static constexpr int p[6][3] = {{0, 1, 2}, {0, 2, 1}, {1, 0, 2}, {1, 2, 0}, {2, 0, 1}, {2, 1, 0}};
};

// A^-1 = adj(A) / det(A) for the N x N GF(256) matrix A (N = LH_EMAX <= 4; characteristic
// 2, so no signs).  Every cofactor is a sum of products of N - 1 elements, each product one
// exp lookup of a sum of logs, so the inverse costs a handful of dependent LDS round trips
// (logs of A; all cofactor terms; logs of the cofactors and det; the quotients) where
// Gauss-Jordan needs one chain of lookups per elimination step.  gexp has 1024 entries
// (exp of any sum of up to four logs without a modulo).
template <int N>
__device__ __forceinline__ void lh_inv_adj(const unsigned int (&A)[N][N], unsigned int (&Ainv)[N][N],
                                           const unsigned char *gexp, const short *glog) {
    int L[N][N];
#pragma unroll
    for (int i = 0; i < N; ++i)
#pragma unroll
        for (int j = 0; j < N; ++j) L[i][j] = glog[A[i][j]];
    constexpr int M = N - 1;
    unsigned int C[N][N];  // cofactors
#pragma unroll
    for (int i = 0; i < N; ++i) {
        // One cofactor row at a time: the logs pass through an empty asm that also takes
        // the previous row's cofactors, so at most N * (N-1)! lookups are in flight (all 96
        // at once held ~25 more VGPRs than the rest of the kernel needs).
        if (i > 0) {
#pragma unroll
            for (int j = 0; j < N; ++j) asm volatile("" : "+v"(C[i - 1][j]));
#pragma unroll
            for (int r = 0; r < N; ++r)
#pragma unroll
                for (int c = 0; c < N; ++c) asm volatile("" : "+v"(L[r][c]));
        }
#pragma unroll
        for (int j = 0; j < N; ++j) {
            unsigned int c = 0;
#pragma unroll
            for (int q = 0; q < lh_perms<M>::cnt; ++q) {
                int sum = 0;
                bool zero = false;
#pragma unroll
                for (int t = 0; t < M; ++t) {
                    const int r = t < i ? t : t + 1;
                    const int cc0 = lh_perms<M>::p[q][t];
                    const int cc = cc0 < j ? cc0 : cc0 + 1;
                    sum += L[r][cc];
                    zero = zero || A[r][cc] == 0u;
                }
                c ^= zero ? 0u : (unsigned int)gexp[sum];
            }
            C[i][j] = c;
        }
    }
    int LC[N][N];
#pragma unroll
    for (int i = 0; i < N; ++i)
#pragma unroll
        for (int j = 0; j < N; ++j) LC[i][j] = glog[C[i][j]];
    unsigned int det = 0;
#pragma unroll
    for (int j = 0; j < N; ++j) det ^= (A[0][j] && C[0][j]) ? (unsigned int)gexp[L[0][j] + LC[0][j]] : 0u;
    const int ninv = 255 - glog[det];  // det != 0: A is a square sub-matrix of an MDS code
#pragma unroll
    for (int i = 0; i < N; ++i)
#pragma unroll
        for (int j = 0; j < N; ++j) Ainv[i][j] = C[j][i] ? (unsigned int)gexp[LC[j][i] + ninv] : 0u;
}

__device__ __forceinline__ void lh_fused_solve::operator()(lh_plan_regs &pr) const {
    const int nr = pr.e;
    // A = G[rr_i][er_j], identity-padded to LH_EMAX; I = A^-1.
    unsigned int A[LH_EMAX][LH_EMAX], I[LH_EMAX][LH_EMAX];
#pragma unroll
    for (int i = 0; i < LH_EMAX; ++i)
#pragma unroll
        for (int j = 0; j < LH_EMAX; ++j)
            A[i][j] = (i < nr && j < nr) ? gmat[rr[i] * LH_K + er[j]] : (i == j ? 1u : 0u);
#if LH_SOLVE_GJ  // Gauss-Jordan (round 1): one dependent chain of table lookups per step
#pragma unroll
    for (int i = 0; i < LH_EMAX; ++i)
#pragma unroll
        for (int j = 0; j < LH_EMAX; ++j) I[i][j] = (i == j) ? 1u : 0u;
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
#else
    lh_inv_adj<LH_EMAX>(A, I, gexp, glog);
#endif
#pragma unroll
    for (int i = 0; i < LH_EMAX; ++i)
#pragma unroll
        for (int j = 0; j < LH_EMAX; ++j) asm volatile("" : "+v"(I[i][j]));  // inverse complete here
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
        for (int i = 0; i < LH_EMAX; ++i) if (i < nr && !LH_PROBE_NOMETA) grow[rs[i]] = (unsigned char)er[i];
    // Materialise the packed plan here, so the solve's matrices die before phase A: left
    // alone, the compiler sinks the packing into phase B and keeps the e x e inverse and
    // the row lists live across all k + m columns (k29/m4: 218 -> 158 VGPRs, 2 -> 3
    // waves/SIMD).
#pragma unroll
    for (int q = 0; q < LH_NCOEF; ++q) asm volatile("" : "+v"(pr.coefw[q]));
#pragma unroll
    for (int q = 0; q < LH_NOUT; ++q) asm volatile("" : "+v"(pr.outw[q]));
}

#if LH_LDS
// The fused decode with its columns staged like the encode's (LH_LDS = 1): the wave's
// LH_SPW stripes of column X (stream order, lh_dcol) arrive as LH_LQ buffer_load_dwordx4
// ... lds per column into the wave's ring, chunk j = 64 q + lane of the image
// [stripe][bytes].  A DMA lane takes its stripe's slot for X from the plan's slot maps in
// the wave's LDS scratch (lh_fused_plan); an absent column (erased original, missing
// recovery row) or a stripe with nothing to do gets an out-of-range offset: zeros into the
// ring, no memory request.  Compute lanes read their words as the encode's do and store
// the recovered blocks as it stores recovery blocks (the last lane of a stripe funnels the
// previous lane's word).  Pointer-table batches (LH_PTR): the wave's stripes' rows of block
// pointers (slot order, the zero page at LH_K) copied into LDS, each DMA lane's address its
// chunk's slot pointer from there, absent columns read from the zero page (L2-resident) --
// flat global_load_lds, no buffer range to clip against.
// Column order and cache policy of this form (profiles/r5i_tune_k29m4_lds_dec.txt, k29/m4:
// 0.611 ms register ring; 0.588 staged, recovery rows first, default policy; 0.577 recovery
// rows last with non-temporal loads -- the slots the outputs overwrite are then no longer
// L2-resident when the stores arrive, the pattern DESIGN.md 5.2 measured for the stores).
#ifndef LH_LDS_REC_FIRST
#define LH_LDS_REC_FIRST 0
#endif
#ifndef LH_LDS_NT_DEC
#define LH_LDS_NT_DEC 1
#endif
#define LH_SR_SRC LH_P4(LH_K)        // scratch offsets of the src / rec slot maps
#define LH_SR_REC (2 * LH_P4(LH_K))
template <int X>
struct lh_dmoff {  // scratch offset of column X's slot byte
    using D = lh_dcol<X, LH_LDS_REC_FIRST>;
    static constexpr int v = D::rec ? LH_SR_REC + D::r : LH_SR_SRC + D::x;
};
#ifndef LH_DOPQ
#define LH_DOPQ 0  // the DMAs' LDS offsets opaque where used (no SGPR held per slot / chunk address)
#endif
struct lh_dldsrc {
#if LH_PTR
    const unsigned long long *pt;  // LDS: the wave's pointer rows [stripe][LH_K + 1]
    int prow[LH_LQ];               // DMA chunk q: its stripe's row in pt
    int joff[LH_LQ];               // ... its offset in the block
#elif LH_ASM_DMA
    lh_u32x4r rs;
    int joff[LH_LQ];  // DMA chunk q: byte offset in the wave's stripes (block 0)
#else
    __amdgpu_buffer_rsrc_t rs;
    int joff[LH_LQ];  // DMA chunk q: byte offset in the wave's stripes (block 0)
#endif
    int jsc[LH_LQ];   // ... its stripe's scratch offset, or -1: nothing to do there
    const unsigned char *scr;  // the wave's scratch (LDS)
    unsigned char *ring;
    template <int X>
    __device__ __forceinline__ void slots(unsigned (&sv)[LH_LQ]) const {
#pragma unroll
        for (int q = 0; q < LH_LQ; ++q) {  // (unconditional read: no branch per chunk)
            const unsigned b = scr[(jsc[q] & 0x7FFFFFFF) + lh_dmoff<X>::v];
            sv[q] = jsc[q] < 0 ? 0xFFu : b;
        }
    }
    __device__ __forceinline__ void issue(const unsigned (&sv)[LH_LQ], int slot) const {
#pragma unroll
        for (int q = 0; q < LH_LQ; ++q)
#if LH_PTR
            lh_dma16<LH_LDS_NT_DEC>((const unsigned char *)pt[prow[q] + (sv[q] == 0xFFu ? LH_K : (int)sv[q])] + joff[q],
                                    ring + slot * (LH_LQ * 1024) + q * 1024);
#elif LH_ASM_DMA
            lh_dma16_buf<LH_LDS_NT_DEC>(rs, sv[q] == 0xFFu ? (int)0x80000000 : joff[q] + (int)sv[q] * LH_BYTES,
                                        ring + slot * (LH_LQ * 1024) + q * 1024);
#else
        {
            int off = slot * (LH_LQ * 1024) + q * 1024;
            if (LH_DOPQ) asm volatile("" : "+s"(off));  // (opaque: see lh_fdsrc::issue)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(
                rs, (__attribute__((address_space(3))) void *)(ring + off), 16,
                sv[q] == 0xFFu ? (int)0x80000000 : joff[q] + (int)sv[q] * LH_BYTES, 0, 0, LH_LDS_NT_DEC ? 2 : 0);
        }
#endif
    }
};
// LH_LDG: the ring refilled LH_LDG slots at a time (after every LH_LDG-th column) instead of
// one slot per column: k29/m4 decode 0.577 -> 0.559 ms (profiles/r7a_tune_k29m4_ldg.txt; 2
// and 3 alike, the encode unchanged).  The refill's slot maps are read before the wait of the
// column that ends its group (0.561 -> 0.558 ms against reading them at the issue,
// r7w_tune_k29m4_dec_slot_prefetch.txt).
#ifndef LH_LDG
#define LH_LDG (LH_LD > 2 ? 2 : 1)
#endif
#if LH_LDG < 1 || LH_LDG >= LH_LD
#error "LH_LDG: 1 <= LH_LDG < LH_LD"
#endif
// Columns C .. C + N - 1 (those that exist): their slot maps read into sv[0 .. N - 1] (before
// the wait of the column that ends the group), then their DMAs issued into their slots.
template <int C, int N>
__device__ __forceinline__ void lh_dslots(const lh_dldsrc &S, unsigned (&sv)[LH_LDG][LH_LQ]) {
    if constexpr (N > 0 && C < LH_DCOLS) {
        S.slots<C>(sv[LH_LDG - N]);
        lh_dslots<C + 1, N - 1>(S, sv);
    }
}
template <int C, int N>
__device__ __forceinline__ void lh_dissue(const lh_dldsrc &S, const unsigned (&sv)[LH_LDG][LH_LQ]) {
    if constexpr (N > 0 && C < LH_DCOLS) {
        S.issue(sv[LH_LDG - N], C % LH_LD);
        lh_dissue<C + 1, N - 1>(S, sv);
    }
}
template <int X>
struct lh_unroll_decode_lds {
    __device__ __forceinline__ static void run(lh_word (&v)[LH_M][8], const lh_dldsrc &S, int lo, int lo8) {
        if constexpr (X < LH_DCOLS) {
            constexpr int issued = (LH_LD + LH_LDG * (X / LH_LDG)) < LH_DCOLS ? (LH_LD + LH_LDG * (X / LH_LDG)) : LH_DCOLS;
            constexpr int ahead = issued - 1 - X;
            unsigned sv[LH_LQ];
            if constexpr (LH_LDG == 1 && X + LH_LD < LH_DCOLS) S.slots<(X + LH_LD < LH_DCOLS ? X + LH_LD : 0)>(sv);
            constexpr bool refill = LH_LDG > 1 && (X + 1) % LH_LDG == 0 && LH_LD + X + 1 - LH_LDG < LH_DCOLS;
            unsigned svg[LH_LDG][LH_LQ];
            if constexpr (refill) lh_dslots<LH_LD + X + 1 - LH_LDG, LH_LDG>(S, svg);
            lh_wait_vmcnt<LH_LQ * ahead>();
            asm volatile("" ::: "memory");  // no LDS read moves above the wait
            lh_word d[8];
            lh_slot_col(d, S.ring + (X % LH_LD) * (LH_LQ * 1024), lo, lo8);
            lh_dcombine<X, LH_LDS_REC_FIRST>(v, d);
            lh_dopaque(v);
            if constexpr (LH_LDG == 1 && X + LH_LD < LH_DCOLS) {
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the slot's reads are done
                S.issue(sv, X % LH_LD);
            } else if constexpr (refill) {
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the slots' reads are done
                lh_dissue<LH_LD + X + 1 - LH_LDG, LH_LDG>(S, svg);
            }
            lh_unroll_decode_lds<X + 1>::run(v, S, lo, lo8);
        }
    }
};
template <int X = 0>
__device__ __forceinline__ void lh_decode_lds_prologue(const lh_dldsrc &S) {
    if constexpr (X < LH_LD && X < LH_DCOLS) {
        unsigned sv[LH_LQ];
        S.slots<X>(sv);
        S.issue(sv, X);
        lh_decode_lds_prologue<X + 1>(S);
    }
}
// Phase B and the stores of a stripe's recovered blocks: block i = sum_r coef[i][r] V_r, stored
// at the slot `dst(out slot i)` returns (the lane's chunk of it); the last lane of a stripe
// funnels the previous lane's word (its chunk's last LH_VLAST bytes are its own).
#ifndef LH_PROBE_NOPB
#define LH_PROBE_NOPB 0
#endif
#ifndef LH_DEC_ST_PEND
#define LH_DEC_ST_PEND 0  // (1: measured no change in write bytes, decode 0.5548 -> 0.5598 ms; profiles/r10w_*)
#endif
// (VL: the last lane's own bytes, sub: the sub-block size -- LH_VLAST, LH_SUB except in the
// block-size family)
template <int VL, class DST>
__device__ __forceinline__ void lh_fused_out_g(const lh_word (&v)[LH_M][8], const lh_plan_regs &pr, bool last, int sub,
                                               DST dst) {
    const int e = pr.e;
#if LH_DEC_ST_PEND
    lh_word pend;  // the last block's last sub-row, stored with the next block
    unsigned char *pd = nullptr;
#pragma unroll
    for (int q = 0; q < LH_NW; ++q) pend.v[q] = 0;
#endif
#pragma unroll
    for (int i = 0; i < LH_EMAX; ++i) {
        if (i < e) {  // stripe-uniform: the funnel's source lane is active too
            lh_word o[8];
#pragma unroll
            for (int y = 0; y < 8; ++y)
#pragma unroll
                for (int q = 0; q < LH_NW; ++q) o[y].v[q] = 0;
#if LH_PROBE_NOPB  // (probe, wrong bytes: no phase B, V_(i mod m) stored as block i -- what phase B costs)
#pragma unroll
            for (int y = 0; y < 8; ++y) o[y] = v[i % LH_M][y];
#else
#pragma unroll
            for (int t = 7; t >= 0; --t) {
                if (t != 7) {
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
                    const unsigned int mask =
                        (unsigned int)((int)(pr.coefw[idx / 4] << (31 - (8 * (idx % 4) + t))) >> 31);
#pragma unroll
                    for (int y = 0; y < 8; ++y)
#pragma unroll
                        for (int q = 0; q < LH_NW; ++q) o[y].v[q] = lh_xand(o[y].v[q], v[r][y].v[q], mask);
                }
#if LH_PIN_WORDS & 2
                lh_pin8w(o);
#else
                lh_pin8(o);
#endif
            }
#endif
            unsigned char *d = dst((int)LH_BYTE(pr.outw, i));
#if LH_DEC_ST_PEND
            // the previous block's last sub-row right before this block's first: when the two
            // blocks are neighbours (the recovery slots usually are), the line they share gets
            // both parts back to back instead of a block's phase B apart (non-temporal stores
            // leave the earlier part as a partial-line write)
            if (i > 0) {
                lh_store(pd + 7 * sub, pend);
                asm volatile("" ::: "memory");
            }
#endif
#pragma unroll
            for (int y = 0; y < 8; ++y) {
                lh_word w = o[y];
                if constexpr (VL != 8) {
                    const lh_word f = lh_funnel<VL>(lh_row_shr1(w.v[0]), lh_row_shr1(w.v[1]), w.v[0], w.v[1]);
                    w.v[0] = last ? f.v[0] : w.v[0];
                    w.v[1] = last ? f.v[1] : w.v[1];
                }
#if LH_DEC_ST_PEND
                if (y == 7) {
                    pend = w;
                    pd = d;
                    continue;
                }
#endif
                lh_store(d + y * sub, w);
                asm volatile("" ::: "memory");
            }
        }
    }
#if LH_DEC_ST_PEND
    if (e > 0) lh_store(pd + 7 * sub, pend);
#endif
}
template <class DST>
__device__ __forceinline__ void lh_fused_out(const lh_word (&v)[LH_M][8], const lh_plan_regs &pr, bool last, DST dst) {
    lh_fused_out_g<LH_VLAST>(v, pr, last, LH_SUB, dst);
}
// One wave's stripe group; `work`: this lane's stripe has a plan (lh_fused_plan true).
// Every lane of the wave runs this (the DMAs need them all); only working lanes solve and store.
__device__ __forceinline__ void lh_fused_wave_lds(const lh_lane &l, long long wave, int c, int sl, bool work,
                                                  const unsigned char *scr, unsigned char *__restrict__ blocks,
                                                  long long stripe_stride, int stripes, const lh_fused_solve &sv,
                                                  lh_plan_regs &pr, const unsigned char *zero_page) {
    __shared__ __attribute__((aligned(16))) unsigned char lh_dring[LH_DWPB][LH_LD * LH_LQ * 1024 + LH_LPAD];
    const int lane = threadIdx.x & 63;
    const long long s0 = (long long)__builtin_amdgcn_readfirstlane((int)wave) * LH_SPW;  // wave-uniform
    if (s0 >= stripes) return;  // wave-uniform
    const int nst = (int)((stripes - s0) < LH_SPW ? (stripes - s0) : LH_SPW);
    const unsigned long long wm = __ballot(work);
    if (wm == 0) return;  // wave-uniform
    lh_dldsrc S;
#if LH_PTR
    // blocks: the pointer table (rows of LH_K block pointers, stride stripe_stride bytes)
    __shared__ unsigned long long lh_dpt[LH_DWPB][LH_SPW * (LH_K + 1)];
    unsigned long long *prow = lh_dpt[threadIdx.x >> 6];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // the previous stripe group's reads
    __builtin_amdgcn_wave_barrier();
    if (sl < nst) {
        const unsigned long long *t = (const unsigned long long *)(blocks + (s0 + sl) * stripe_stride);
        for (int x = c; x <= LH_K; x += LH_NCH)
            prow[sl * (LH_K + 1) + x] = x < LH_K ? t[x] : (unsigned long long)zero_page;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    S.pt = prow;
#else
    (void)zero_page;
#if LH_ASM_DMA
    S.rs = lh_rsrc(blocks + s0 * stripe_stride, (unsigned)(nst * stripe_stride));
#else
    S.rs = __builtin_amdgcn_make_buffer_rsrc(blocks + s0 * stripe_stride, 0, (int)(nst * stripe_stride), 0x00020000);
#endif
#endif
    S.scr = scr;
    S.ring = lh_dring[lh_wid<1>()];
#pragma unroll
    for (int q = 0; q < LH_LQ; ++q) {
        int j = 64 * q + lane;
        if (j >= nst * (LH_BYTES / 16)) j = nst * (LH_BYTES / 16) - 1;  // (lands past the image)
        const int js = j / (LH_BYTES / 16);
#if LH_PTR
        S.prow[q] = js * (LH_K + 1);
        S.joff[q] = (j - js * (LH_BYTES / 16)) * 16;
#else
        S.joff[q] = js * (int)stripe_stride + (j - js * (LH_BYTES / 16)) * 16;
#endif
        S.jsc[q] = js * LH_SR | (((wm >> (js * LH_NCH)) & 1ull) ? 0 : (int)0x80000000);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the previous group's ring reads are done
    lh_decode_lds_prologue(S);
    if (work) sv(pr);  // the solve, while the first columns land
    lh_word v[LH_M][8];
#pragma unroll
    for (int r = 0; r < LH_M; ++r)
#pragma unroll
        for (int y = 0; y < 8; ++y)
#pragma unroll
            for (int i = 0; i < LH_NW; ++i) v[r][y].v[i] = 0;
    const int lo = (sl < LH_SPW ? sl : LH_SPW - 1) * LH_BYTES + 8 * c;
    int lo8 = lo + 8;
    asm volatile("" : "+v"(lo8));
    lh_unroll_decode_lds<0>::run(v, S, lo, lo8);
    if (!work) return;
    // Phase B as lh_dec_phase_b; the stores as the LDS encode's.  (Storing the recovered
    // blocks through the ring as the encode does measured slower in place:
    // profiles/r5l_tune_k29m4_flat_dec.txt, 0.604 against 0.574 ms.)
#if LH_PTR
    lh_fused_out(v, pr, l.last, [&](int slot) {
        return (unsigned char *)S.pt[sl * (LH_K + 1) + slot] + (l.last ? LH_SUB - 8 : 8 * c);
    });
#else
    unsigned char *base = blocks + l.stripe * stripe_stride + (l.last ? LH_SUB - 8 : 8 * c);
    lh_fused_out(v, pr, l.last, [&](int slot) { return base + (long long)slot * LH_BYTES; });
#endif
}
#endif  // LH_LDS

// ------------------------------------------------------------ memory-order decode (LH_DMO)
// The fused decode above reads a stripe's slots in row order (its networks are compiled per
// row), so in a shuffled stripe each slot is a lone 1 296-byte run and the 64-byte sector two
// neighbouring slots share is fetched once per slot: k29/m4 HBM traffic 1.075x the algorithmic
// bytes (profiles/r9g_pmc_k29m4_decode_variants.txt).  LH_DMO = 1 reads the slots in memory
// order instead, LH_CPS slots of every stripe per step (one contiguous run per stripe, as the
// multi-column encode), and runs each slot's network by its row, known only at run time: the
// wave takes the rows present at that slot one at a time (a stripe's lanes hold one row; the
// wave's stripes usually hold different ones), each through a binary tree of wave-uniform
// branches down to the row's compile-time network, executed by the lanes holding that row.
// The networks cost up to LH_SPW times their VALU work of the row-order form -- affordable, the
// decode's VALU runs below 10 % of its time -- for the encode's memory stream.  Strided batches
// (LH_PTR keeps the row-order form); plan, solve, phase B and stores as above.
#ifndef LH_DMO
#define LH_DMO 0
#endif
#if LH_DMO && !(LH_LDS && LH_CPS > 1 && !LH_PTR && defined(LH_FUSED))
#undef LH_DMO
#define LH_DMO 0
#endif
#if LH_DMO
#ifndef LH_DMO_AHEAD
#define LH_DMO_AHEAD 1  // two step slots: step T + 1 lands while step T is combined
#endif
// Row r's contribution (wave-uniform r < LH_DCOLS): original column r's network, or recovery
// row r - LH_K XORed into V_(r - LH_K).  The dispatch is a sequence of one-sided uniform tests,
// first on r / 8, then on r, each test against r passed through an empty asm so the compiler
// cannot chain them into a switch: a branch tree (an if / else nest or a lowered switch) is
// structurised with flow blocks whose paths carry the accumulators past the leaves, and each
// such path cost up to 64 register copies; a one-sided test updates them in place.
#ifndef LH_DMO_PROBE
#define LH_DMO_PROBE 0  // (probes, wrong bytes: 1 no dispatch, one XOR per slot; 2 the dispatch with one-XOR leaves)
#endif
template <int X>
__device__ __forceinline__ void lh_rowleaf(lh_word (&v)[LH_M][8], const lh_word (&d)[8]) {
    if constexpr (LH_DMO_PROBE == 2) {
#pragma unroll
        for (int y = 0; y < 8; ++y) lh_xor(v[X % LH_M][y], d[(y + X) & 7]);
    } else if constexpr (X < LH_K) {
        lh_column<X>(v, d);
    } else {
#pragma unroll
        for (int y = 0; y < 8; ++y) lh_xor(v[X - LH_K][y], d[y]);
    }
    asm volatile("; row %0" ::"i"(X));  // (a leaf of its own: no merging of leaves by the compiler)
}
template <int X, int END>
struct lh_rowgrp {
    __device__ __forceinline__ static void run(unsigned r, lh_word (&v)[LH_M][8], const lh_word (&d)[8]) {
        if constexpr (X < END) {
            asm volatile("" : "+s"(r));
            if (r == (unsigned)X) lh_rowleaf<X>(v, d);
            lh_rowgrp<X + 1, END>::run(r, v, d);
        }
    }
};
template <int G>
struct lh_rowdisp {
    __device__ __forceinline__ static void run(unsigned r, lh_word (&v)[LH_M][8], const lh_word (&d)[8]) {
        if constexpr (8 * G < LH_DCOLS) {
            unsigned g = r >> 3;
            asm volatile("" : "+s"(g));
            if (g == (unsigned)G) lh_rowgrp<8 * G, (8 * G + 8 < LH_DCOLS ? 8 * G + 8 : LH_DCOLS)>::run(r, v, d);
            lh_rowdisp<G + 1>::run(r, v, d);
        }
    }
};
// The lane's 8 words of one slot in the ring (`col` its run-time address): every read issued
// before any is used (a wait per read, placed by the compiler next to each use, exposes the
// LDS latency 8 times per slot with one wave per SIMD; as lh_fam_col).
template <int B>
__device__ __forceinline__ void lh_dmo_rd(lh_u32x2a (&x)[8], lh_u32x2a (&y)[8], const unsigned char *col, int lo, int lo8) {
    if constexpr (B < 8) {
        constexpr int S = (B * LH_SUB) % 8, O = B * LH_SUB - S;
        x[B] = *(const lh_u32x2a *)(col + lo + O);
        if constexpr (S != 0) y[B] = *(const lh_u32x2a *)(col + lo8 + O);
        lh_dmo_rd<B + 1>(x, y, col, lo, lo8);
    }
}
template <int B>
__device__ __forceinline__ void lh_dmo_fn(lh_word (&d)[8], const lh_u32x2a (&x)[8], const lh_u32x2a (&y)[8]) {
    if constexpr (B < 8) {
        constexpr int S = (B * LH_SUB) % 8;
        if constexpr (S == 0) {
            d[B].v[0] = x[B].x;
            d[B].v[1] = x[B].y;
        } else {
            d[B] = lh_funnel<S>(x[B].x, x[B].y, y[B].x, y[B].y);
        }
        lh_dmo_fn<B + 1>(d, x, y);
    }
}
__device__ __forceinline__ void lh_dmo_col(lh_word (&d)[8], const unsigned char *col, int lo, int lo8) {
    lh_u32x2a x[8], y[8];
    lh_dmo_rd<0>(x, y, col, lo, lo8);
#pragma unroll
    for (int b = 0; b < 8; ++b) {
        asm volatile("" : "+v"(x[b]));
        if ((b * LH_SUB) % 8 != 0) asm volatile("" : "+v"(y[b]));
    }
    lh_dmo_fn<0>(d, x, y);
}
// Step t's DMAs (slots t LH_CPS .. of every working stripe) into `ring`; in the last step the
// chunks past slot LH_K are out of range.
__device__ __forceinline__ void lh_dmo_issue(const lh_u32x4r &rs, const int (&voff)[LH_SQ], int t, unsigned char *ring) {
    const int lane = threadIdx.x & 63;
    const bool lastep = t + 1 == LH_NSTEP;
#pragma unroll
    for (int q = 0; q < LH_SQ; ++q) {
        int v = voff[q];
        if (LH_LASTC < LH_CPS && lastep) v = ((64 * q + lane) % LH_SCH) < LH_LASTC * LH_CCH ? v : (int)0x80000000;
        lh_dma16_bufs<LH_LDS_NT_DEC>(rs, v, t * (LH_CPS * LH_BYTES), ring + q * 1024);
    }
}
__device__ __forceinline__ void lh_fused_wave_dmo(const lh_lane &l, long long wave, int c, int sl, bool work,
                                                  const unsigned char *scr, unsigned char *__restrict__ blocks,
                                                  long long stripe_stride, int stripes, const lh_fused_solve &sv,
                                                  lh_plan_regs &pr) {
    __shared__ __attribute__((aligned(16))) unsigned char lh_mring[LH_DWPB][(1 + LH_DMO_AHEAD) * LH_SSLOT];
    const int lane = threadIdx.x & 63;
    const long long s0 = (long long)__builtin_amdgcn_readfirstlane((int)wave) * LH_SPW;  // wave-uniform
    if (s0 >= stripes) return;  // wave-uniform
    const int nst = (int)((stripes - s0) < LH_SPW ? (stripes - s0) : LH_SPW);
    const unsigned long long wm = __ballot(work);
    if (wm == 0) return;  // wave-uniform
    unsigned char *ring = lh_mring[lh_wid<1>()];
    const lh_u32x4r rs = lh_rsrc(blocks + s0 * stripe_stride, (unsigned)(nst * stripe_stride));
    int voff[LH_SQ];  // chunk j = 64 q + lane of the step image [stripe][LH_CPS x bytes]
#pragma unroll
    for (int q = 0; q < LH_SQ; ++q) {
        const int j = 64 * q + lane, js = j / LH_SCH, r = j - js * LH_SCH;
        const bool on = js < nst && ((wm >> (js * LH_NCH)) & 1ull);  // (a stripe with nothing to do: no reads)
        voff[q] = on ? js * (int)stripe_stride + r * 16 : (int)0x80000000;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the previous group's ring reads are done
    lh_dmo_issue(rs, voff, 0, ring);
    if (work) sv(pr);  // the solve, while the first step lands
    lh_word v[LH_M][8];
#pragma unroll
    for (int r = 0; r < LH_M; ++r)
#pragma unroll
        for (int y = 0; y < 8; ++y)
#pragma unroll
            for (int i = 0; i < LH_NW; ++i) v[r][y].v[i] = 0;
    const int sc = sl < LH_SPW ? sl : LH_SPW - 1;
    const int lo = sc * (LH_CPS * LH_BYTES) + 8 * c;
    int lo8 = lo + 8;
    asm volatile("" : "+v"(lo8));
    const unsigned char *lrows = scr + sc * LH_SR;  // the lane's stripe's slot rows (lh_fused_plan)
#pragma unroll 1
    for (int t = 0; t < LH_NSTEP; ++t) {
#if LH_DMO_AHEAD
        unsigned char *cur = ring + (t & 1) * LH_SSLOT;
        if (t + 1 < LH_NSTEP) {
            lh_dmo_issue(rs, voff, t + 1, ring + ((t + 1) & 1) * LH_SSLOT);  // (its slot's reads ended at t - 1)
            lh_wait_vmcnt<LH_SQ>();  // step t landed, t + 1 in flight
        } else {
            lh_wait_vmcnt<0>();
        }
#else
        unsigned char *cur = ring;
        lh_wait_vmcnt<0>();  // this step's DMAs landed (the only ones in flight)
#endif
        asm volatile("" ::: "memory");  // no LDS read moves above the wait
        const int ncol = t + 1 < LH_NSTEP ? LH_CPS : LH_LASTC;
#pragma unroll 1
        for (int cc = 0; cc < ncol; ++cc) {
            lh_word d[8];
            lh_dmo_col(d, cur + cc * LH_BYTES, lo, lo8);
            const unsigned row = work ? (unsigned)lrows[t * LH_CPS + cc] : 0xFFu;
            unsigned long long rem = wm;
            if (LH_DMO_PROBE == 1) {
#pragma unroll
                for (int y = 0; y < 8; ++y) lh_xor(v[0][y], d[y]);
                rem = 0;
            }
            while (rem) {  // wave-uniform: one pass per distinct row among the working lanes
                const unsigned r = (unsigned)__builtin_amdgcn_readlane((int)row, (int)__builtin_ctzll(rem));
                // (the test through an opaque difference: from `row == r` the compiler would
                // substitute the lane's row for r under the branch, making the tree per-lane)
                unsigned diff = row ^ r;
                asm volatile("" : "+v"(diff));
                const bool mine = diff == 0u;
                rem &= ~__ballot(mine);
                if (mine) lh_rowdisp<0>::run(r, v, d);
            }
            lh_dopaque(v);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the slot's reads are done
#if !LH_DMO_AHEAD
        if (t + 1 < LH_NSTEP) lh_dmo_issue(rs, voff, t + 1, ring);
#endif
    }
    if (!work) return;
    unsigned char *base = blocks + l.stripe * stripe_stride + (l.last ? LH_SUB - 8 : 8 * c);
    lh_fused_out(v, pr, l.last, [&](int slot) { return base + (long long)slot * LH_BYTES; });
}
#endif  // LH_DMO

#ifndef LH_DEC_LB
#define LH_DEC_LB 1  // min waves per SIMD the register allocator must allow (tools/tune.py)
#endif
template <int PF>
__device__ __forceinline__ void lh_fused_body(unsigned char *__restrict__ blocks, long long stripe_stride,
                                              unsigned char *__restrict__ rows, signed char *__restrict__ status,
                                              const unsigned char *__restrict__ zero_page,
                                              const unsigned char *__restrict__ gf_exp,
                                              const short *__restrict__ gf_log, int stripes) {
    __shared__ unsigned char gexp[1024];  // exp(i mod 255) for i < 1024 (lh_inv_adj)
    __shared__ short glog[256];
    __shared__ unsigned char gmat[LH_M * LH_K];
    __shared__ __attribute__((aligned(16))) unsigned char scratch[LH_DWPB][LH_SPW > 0 ? LH_SPW : 1][LH_SR];
    for (int i = threadIdx.x; i < 256; i += blockDim.x) {
#pragma unroll
        for (int q = 0; q < 4; ++q) gexp[i + 256 * q] = gf_exp[(i + 256 * q) % 255];
        glog[i] = gf_log[i];
    }
    for (int i = threadIdx.x; i < LH_M * LH_K; i += blockDim.x) gmat[i] = LH_GRAW[i / LH_K][i % LH_K];
    __syncthreads();
    const int wid = threadIdx.x >> 6;
    LH_WAVE_LOOP(stripes) {
        const lh_lane l = lh_map_lane(stripes, lh_w);
        const int lane = threadIdx.x & 63;
        const int sl = lane / LH_NCH;
        const int c = lane - sl * LH_NCH;
        lh_plan_regs pr;
        lh_fused_solve sv;
        sv.gexp = gexp;
        sv.glog = glog;
        sv.gmat = gmat;
        unsigned int rowv[lh_gct::maxrw];
        lh_fused_rows(lh_gct(), l, c, rows, rowv);
#if LH_DMO
        const bool work = l.active && lh_fused_plan(lh_gct(), l, c, sl, &scratch[wid][sl][0], rowv, rows, status, sv, pr);
        lh_fused_wave_dmo(l, lh_w, c, sl, work, &scratch[wid][0][0], blocks, stripe_stride, stripes, sv, pr);
#elif LH_LDS
        const bool work = l.active && lh_fused_plan(lh_gct(), l, c, sl, &scratch[wid][sl][0], rowv, rows, status, sv, pr);
        lh_fused_wave_lds(l, lh_w, c, sl, work, &scratch[wid][0][0], blocks, stripe_stride, stripes, sv, pr, zero_page);
#else
        if (l.active && lh_fused_plan(lh_gct(), l, c, sl, &scratch[wid][sl][0], rowv, rows, status, sv, pr))
            lh_decode_body<PF>(l, lh_w, blocks, stripe_stride, pr, zero_page, stripes, sv);
#endif
    }
}

#if (LH_ROLE == 0 || (LH_ROLE == 2 && !LH_DEC_PLAIN)) && !LH_FAMILY
extern "C" __global__ void __launch_bounds__(64 * LH_DWPB, LH_DEC_LB)
lh_jit_decode_fused(unsigned char *__restrict__ blocks, long long stripe_stride, unsigned char *__restrict__ rows,
                    signed char *__restrict__ status, const unsigned char *__restrict__ zero_page,
                    const unsigned char *__restrict__ gf_exp, const short *__restrict__ gf_log, int stripes) {
    lh_fused_body<LH_PF_DEC>(blocks, stripe_stride, rows, status, zero_page, gf_exp, gf_log, stripes);
}
#endif

// ------------------------------------------------------------ decode block-size family
// The fused, LDS-staged decode of lh_fused_wave_lds with the block size a kernel argument (one
// module per (k, m) for every 16-byte-multiple size with 8-byte lanes, at most 64 lanes and at
// least ceil(k / 8) lanes per stripe; jit.cpp jit_family_ok): the wave's geometry (lanes and
// stripes per wave, DMA instructions per column) is run-time and wave-uniform; every column
// issues 4 DMA instructions (one column of 4 KiB at most), those past the wave's stripes with an
// out-of-range offset (no memory request), so the waits count a constant; the LDS reads take
// the per-lane sub-block addresses computed once per wave with the alignment form R = sub mod 8
// fixed per launch (lh_fam_col, as the encode's family).
#if LH_FAMILY && LH_ROLE == 2 && LH_LDS && !LH_PTR
#define LH_FNRW 8                                   // Block.row bytes per lane, at most
#define LH_FSPW (64 / ((LH_K + LH_FNRW - 1) / LH_FNRW))  // stripes per wave, at most
#define LH_FRS (4 * 1024 + 16)                      // ring slot: 4 KiB (+16: the last lane's second word)
struct lh_grt {
    int nch, nrw;
    unsigned long long lanes;
    static constexpr int maxrw = LH_FNRW;
};
struct lh_dfam {
    int bytes, sub, nch, spw, cch;
};
struct lh_fdsrc {
    __amdgpu_buffer_rsrc_t rs;
    int joff[4], jsc[4];  // DMA chunk q: byte offset in the wave's stripes (block 0); its stripe's scratch offset or < 0
    int bytes;
    const unsigned char *scr;
    unsigned char *ring;
    template <int X>
    __device__ __forceinline__ void slots(unsigned (&sv)[4]) const {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const unsigned b = scr[(jsc[q] & 0x7FFFFFFF) + lh_dmoff<X>::v];
            sv[q] = jsc[q] < 0 ? 0xFFu : b;
        }
    }
    __device__ __forceinline__ void issue(const unsigned (&sv)[4], int slot) const {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            // (the LDS offset made opaque where it is used: left alone, the compiler keeps all 16
            // slot / chunk addresses in SGPRs for the whole kernel and spills others for them)
            int off = slot * LH_FRS + q * 1024;
            asm volatile("" : "+s"(off));
            __builtin_amdgcn_raw_ptr_buffer_load_lds(
                rs, (__attribute__((address_space(3))) void *)(ring + off), 16,
                sv[q] == 0xFFu ? (int)0x80000000 : joff[q] + (int)sv[q] * bytes, 0, 0, LH_LDS_NT_DEC ? 2 : 0);
        }
    }
};
template <int C, int N>
__device__ __forceinline__ void lh_fdslots(const lh_fdsrc &S, unsigned (&sv)[LH_LDG][4]) {
    if constexpr (N > 0 && C < LH_DCOLS) {
        S.slots<C>(sv[LH_LDG - N]);
        lh_fdslots<C + 1, N - 1>(S, sv);
    }
}
template <int C, int N>
__device__ __forceinline__ void lh_fdissue(const lh_fdsrc &S, const unsigned (&sv)[LH_LDG][4]) {
    if constexpr (N > 0 && C < LH_DCOLS) {
        S.issue(sv[LH_LDG - N], C % LH_LD);
        lh_fdissue<C + 1, N - 1>(S, sv);
    }
}
#ifndef LH_DFAM_PIN
#define LH_DFAM_PIN 0  // 1: a column's 16 LDS reads all issued before any is used (lh_fam_col)
#endif
// A column's words, each read next to its use (the compiler's schedule).
template <int R>
__device__ __forceinline__ void lh_dfam_col(lh_word (&d)[8], const unsigned char *slot, const int (&ad)[8]) {
#pragma unroll
    for (int b = 0; b < 8; ++b) {
        const int S = (b * R) & 7;  // (constant after unrolling)
        const lh_u32x2a x = *(const lh_u32x2a *)(slot + ad[b] + ((b * R) & ~7));
        if (S == 0) {
            d[b].v[0] = x.x;
            d[b].v[1] = x.y;
        } else {
            const lh_u32x2a y = *(const lh_u32x2a *)(slot + ad[b] + 8 + ((b * R) & ~7));
            if (S == 2) d[b] = lh_funnel<2>(x.x, x.y, y.x, y.y);
            else if (S == 4) d[b] = lh_funnel<4>(x.x, x.y, y.x, y.y);
            else d[b] = lh_funnel<6>(x.x, x.y, y.x, y.y);
        }
    }
}
// Phase A over the k + m columns, as lh_unroll_decode_lds (refills of LH_LDG slots).
template <int X, int R>
struct lh_unroll_dfam {
    __device__ __forceinline__ static void run(lh_word (&v)[LH_M][8], const lh_fdsrc &S, const int (&ad)[8], const int (&ad8)[8]) {
        if constexpr (X < LH_DCOLS) {
            constexpr int issued = (LH_LD + LH_LDG * (X / LH_LDG)) < LH_DCOLS ? (LH_LD + LH_LDG * (X / LH_LDG)) : LH_DCOLS;
            constexpr int ahead = issued - 1 - X;
            unsigned sv[4];
            if constexpr (LH_LDG == 1 && X + LH_LD < LH_DCOLS) S.slots<(X + LH_LD < LH_DCOLS ? X + LH_LD : 0)>(sv);
            constexpr bool refill = LH_LDG > 1 && (X + 1) % LH_LDG == 0 && LH_LD + X + 1 - LH_LDG < LH_DCOLS;
            unsigned svg[LH_LDG][4];
            if constexpr (refill) lh_fdslots<LH_LD + X + 1 - LH_LDG, LH_LDG>(S, svg);
            lh_wait_vmcnt<4 * ahead>();
            asm volatile("" ::: "memory");  // no LDS read moves above the wait
            lh_word d[8];
#if LH_DFAM_PIN
            lh_fam_col<R>(d, S.ring + (X % LH_LD) * LH_FRS, ad, ad8);
#else
            lh_dfam_col<R>(d, S.ring + (X % LH_LD) * LH_FRS, ad);
#endif
            lh_dcombine<X, LH_LDS_REC_FIRST>(v, d);
            lh_dopaque(v);
            if constexpr (LH_LDG == 1 && X + LH_LD < LH_DCOLS) {
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the slot's reads are done
                S.issue(sv, X % LH_LD);
            } else if constexpr (refill) {
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the slots' reads are done
                lh_fdissue<LH_LD + X + 1 - LH_LDG, LH_LDG>(S, svg);
            }
            lh_unroll_dfam<X + 1, R>::run(v, S, ad, ad8);
        }
    }
};
template <int X = 0>
__device__ __forceinline__ void lh_dfam_prologue(const lh_fdsrc &S) {
    if constexpr (X < LH_LD && X < LH_DCOLS) {
        unsigned sv[4];
        S.slots<X>(sv);
        S.issue(sv, X);
        lh_dfam_prologue<X + 1>(S);
    }
}
template <int R>
__device__ __forceinline__ void lh_fused_wave_fam(const lh_dfam &F, const lh_lane &l, long long wave, int c, int sl, bool work,
                                                  const unsigned char *scr, unsigned char *__restrict__ blocks,
                                                  long long stripe_stride, int stripes, const lh_fused_solve &sv,
                                                  lh_plan_regs &pr, unsigned char *ring) {
    const int lane = threadIdx.x & 63;
    const long long s0 = (long long)__builtin_amdgcn_readfirstlane((int)wave) * F.spw;  // wave-uniform
    if (s0 >= stripes) return;  // wave-uniform
    const int nst = (int)((stripes - s0) < F.spw ? (stripes - s0) : F.spw);
    const unsigned long long wm = __ballot(work);
    if (wm == 0) return;  // wave-uniform
    lh_fdsrc S;
    S.rs = __builtin_amdgcn_make_buffer_rsrc(blocks + s0 * stripe_stride, 0, (int)(nst * stripe_stride), 0x00020000);
    S.bytes = F.bytes;
    S.scr = scr;
    S.ring = ring;
#pragma unroll
    for (int q = 0; q < 4; ++q) {  // chunk j = 64 q + lane of the image [stripe][bytes]
        const int j = 64 * q + lane;
        const int js = j / F.cch;
        const bool on = js < nst && ((wm >> (js * F.nch)) & 1ull);
        S.joff[q] = js * (int)stripe_stride + (j - js * F.cch) * 16;
        S.jsc[q] = on ? js * LH_SR : (int)0x80000000;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the previous group's ring reads are done
    lh_dfam_prologue(S);
    if (work) sv(pr);  // the solve, while the first columns land
    lh_word v[LH_M][8];
#pragma unroll
    for (int r = 0; r < LH_M; ++r)
#pragma unroll
        for (int y = 0; y < 8; ++y)
#pragma unroll
            for (int i = 0; i < LH_NW; ++i) v[r][y].v[i] = 0;
    const int lo = (sl < F.spw ? sl : F.spw - 1) * F.bytes + 8 * c;
    int ad[8], ad8[8];
#pragma unroll
    for (int b = 0; b < 8; ++b) {
        ad[b] = lo + b * (F.sub - R);
        ad8[b] = ad[b] + 8;
#if LH_FAM_SPLIT
        asm volatile("" : "+v"(ad8[b]));
#endif
    }
    lh_unroll_dfam<0, R>::run(v, S, ad, ad8);
    if (!work) return;
    unsigned char *base = blocks + l.stripe * stripe_stride + (l.last ? F.sub - 8 : 8 * c);
    lh_fused_out_g<R == 0 ? 8 : R>(v, pr, l.last, F.sub, [&](int slot) { return base + (long long)slot * F.bytes; });
}
template <int R>
__device__ __forceinline__ void lh_dfam_body(const lh_dfam &F, const lh_grt &g, unsigned char *__restrict__ blocks,
                                             long long stripe_stride, unsigned char *__restrict__ rows,
                                             signed char *__restrict__ status, const unsigned char *gexp, const short *glog,
                                             const unsigned char *gmat, unsigned char (*scratch)[LH_FSPW][LH_SR],
                                             unsigned char *ring, int stripes) {
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int sl = lane / F.nch, c = lane - sl * F.nch;
    const long long nw = ((long long)stripes + F.spw - 1) / F.spw;
    const long long ws = (long long)gridDim.x * (blockDim.x >> 6);
    for (long long w = (lh_block_id() * blockDim.x + threadIdx.x) >> 6; w < nw; w += ws) {
        lh_lane l;
        l.stripe = w * F.spw + sl;
        l.active = sl < F.spw && l.stripe < stripes;
        l.last = c == F.nch - 1;
        l.p = 0;  // (unused here)
        lh_plan_regs pr;
        lh_fused_solve sv;
        sv.gexp = gexp;
        sv.glog = glog;
        sv.gmat = gmat;
        unsigned int rowv[LH_FNRW];
        lh_fused_rows(g, l, c, rows, rowv);
        const bool work = l.active && lh_fused_plan(g, l, c, sl, &scratch[wid][sl][0], rowv, rows, status, sv, pr);
        lh_fused_wave_fam<R>(F, l, w, c, sl, work, &scratch[wid][0][0], blocks, stripe_stride, stripes, sv, pr, ring);
    }
}
extern "C" __global__ void __launch_bounds__(256, LH_DEC_LB)
lh_jit_decode_fused(unsigned char *__restrict__ blocks, long long stripe_stride, unsigned char *__restrict__ rows,
                    signed char *__restrict__ status, const unsigned char *__restrict__ zero_page,
                    const unsigned char *__restrict__ gf_exp, const short *__restrict__ gf_log, int stripes, int bytes) {
    (void)zero_page;
    __shared__ unsigned char gexp[1024];  // exp(i mod 255) for i < 1024 (lh_inv_adj)
    __shared__ short glog[256];
    __shared__ unsigned char gmat[LH_M * LH_K];
    __shared__ __attribute__((aligned(16))) unsigned char scratch[4][LH_FSPW][LH_SR];
    __shared__ __attribute__((aligned(16))) unsigned char lh_fdring[4][LH_LD * LH_FRS];
    for (int i = threadIdx.x; i < 256; i += blockDim.x) {
#pragma unroll
        for (int q = 0; q < 4; ++q) gexp[i + 256 * q] = gf_exp[(i + 256 * q) % 255];
        glog[i] = gf_log[i];
    }
    for (int i = threadIdx.x; i < LH_M * LH_K; i += blockDim.x) gmat[i] = LH_GRAW[i / LH_K][i % LH_K];
    __syncthreads();
    lh_dfam F;
    F.bytes = bytes;
    F.sub = bytes >> 3;
    F.nch = (F.sub + 7) >> 3;
    F.spw = 64 / F.nch;
    F.cch = bytes >> 4;
    lh_grt g;
    g.nch = F.nch;
    g.nrw = (LH_K + F.nch - 1) / F.nch;
    g.lanes = F.nch >= 64 ? ~0ull : ((1ull << F.nch) - 1);
    // (the wave index made wave-uniform explicitly: the ring's LDS addresses, the DMAs' M0, then
    // live in SGPRs, not in 16 VGPRs read back with readfirstlane before every DMA)
    unsigned char *ring = lh_fdring[__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6))];
    switch (F.sub & 7) {  // (launch-uniform; bytes % 16 == 0 makes sub even)
        case 0: lh_dfam_body<0>(F, g, blocks, stripe_stride, rows, status, gexp, glog, gmat, scratch, ring, stripes); break;
        case 2: lh_dfam_body<2>(F, g, blocks, stripe_stride, rows, status, gexp, glog, gmat, scratch, ring, stripes); break;
        case 4: lh_dfam_body<4>(F, g, blocks, stripe_stride, rows, status, gexp, glog, gmat, scratch, ring, stripes); break;
        default: lh_dfam_body<6>(F, g, blocks, stripe_stride, rows, status, gexp, glog, gmat, scratch, ring, stripes); break;
    }
}
#endif  // LH_FAMILY && LH_ROLE == 2

#endif  // LH_EMAX <= 4 && LH_NCH <= 64 && LH_K <= 64
