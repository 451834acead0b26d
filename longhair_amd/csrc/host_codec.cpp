// host_codec.cpp -- the host SIMD engine of the drop-in dispatch policy (SURVEY.md §8f,
// rank 2): one stripe per call from host memory, the reference's call shape
// (cauchy_256.h:78, :103; README.md:111-182).  A single small stripe is latency-bound:
// staging it over PCIe to the GPU costs ~30-66 us per call where the bit-sliced XOR work
// itself is ~2 us of AVX-512 (profiles/r2_bench_k29m4.json, dropin_per_call).  The
// dispatch policy (codec.cpp, cauchy_256_dispatch.h) sends such calls here by default
// (AUTO: all-host calls with at most LONGHAIR_AMD_HOST_MAX_WORK bytes of XOR work) or when
// the caller selects HOST; the library still requires a GPU.
//
// Both operations are one bit-sliced coefficient apply (same algebra as the GPU kernels):
//   out[i] sub-row y  ^=  in[j] sub-block b   for every bit b of C[i][j] * 2^y,
// encode with C = the generator rows 1..m-1 (row 0 is the plain XOR, as the reference
// writes it first: cauchy_256.cpp:1511-1516); decode in two applies, V = R + G_p D_p and
// D_E = A^-1 V, A = G[recovery rows][erased rows] (cauchy_256.cpp:707-790 solve the same
// system bit by bit; the solution is unique, so the bytes are equal).
// The apply walks the sub-block in 64-byte (AVX-512BW) or 32-byte (AVX2) chunks, every
// output sub-row of a chunk accumulated in a register from L1-resident input chunks,
// input terms paired through a 3-input XOR (vpternlogq 0x96).
#include <immintrin.h>

#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <string>
#include <map>
#include <mutex>
#include <vector>

#include "../../include/cauchy_256.h"
#include "field.hpp"
#include "host_codec.hpp"

namespace lh {
namespace host {

namespace {

// Term lists of a coefficient matrix: for output sub-row o = 8 i + y, the input
// sub-blocks t = 8 j + b whose bit is set in C[i][j] * 2^y.
struct Terms {
    int nout = 0, nin = 0;
    std::vector<uint32_t> begin;  // nout * 8 + 1 offsets into idx
    std::vector<uint16_t> idx;
};

// BM[c][y] = bit-row y of element c (c * 2^y): the input sub-blocks of output sub-row y.
struct BitRows {
    uint8_t r[256][8];
    BitRows() {
        for (int c = 0; c < 256; ++c) {
            const uint64_t bm = bitmatrix((uint8_t)c);
            for (int y = 0; y < 8; ++y) r[c][y] = (uint8_t)(bm >> (8 * y));
        }
    }
};
const BitRows &bitrows() {
    static const BitRows t;
    return t;
}

void build_terms(const uint8_t *C, int nout, int nin, Terms *T) {
    const BitRows &BR = bitrows();
    T->nout = nout;
    T->nin = nin;
    T->begin.resize((size_t)nout * 8 + 1);
    T->idx.resize((size_t)nout * nin * 64);  // upper bound: every bit set
    uint16_t *out = T->idx.data();
    uint32_t n = 0;
    for (int i = 0; i < nout; ++i) {
        const uint8_t *row = C + (size_t)i * nin;
        for (int y = 0; y < 8; ++y) {
            T->begin[(size_t)i * 8 + y] = n;
            for (int j = 0; j < nin; ++j)
                for (unsigned s = BR.r[row[j]][y]; s; s &= s - 1) out[n++] = (uint16_t)(8 * j + __builtin_ctz(s));
        }
    }
    T->begin[(size_t)nout * 8] = n;
    T->idx.resize(n);
}

// One output sub-row of an apply: dst = (init ? init : 0) ^ XOR of src[idx[0..n)].  No
// output may alias an input of the same apply (decode phase A writes a scratch V, phase B
// reads it), so chunks are written straight back.
struct OutRow {
    const uint16_t *idx;
    uint32_t n;
    uint8_t *dst;
    const uint8_t *init;
};

void apply_scalar(const OutRow *rows, int nrows, const uint8_t *const *src, int sub, int p0) {
    for (int o = 0; o < nrows; ++o) {
        const OutRow &R = rows[o];
        for (int p = p0; p < sub; ++p) {
            uint8_t acc = R.init ? R.init[p] : 0;
            for (uint32_t t = 0; t < R.n; ++t) acc ^= src[R.idx[t]][p];
            R.dst[p] = acc;
        }
    }
}

__attribute__((target("avx512f,avx512bw"))) void apply_avx512(const OutRow *rows, int nrows,
                                                                 const uint8_t *const *src, int sub) {
    for (int p = 0; p < sub; p += 64) {
        const int w = std::min(64, sub - p);
        const __mmask64 mk = w == 64 ? ~0ull : ((1ull << w) - 1);
        for (int o = 0; o < nrows; ++o) {
            const OutRow &R = rows[o];
            __m512i acc = R.init ? _mm512_maskz_loadu_epi8(mk, R.init + p) : _mm512_setzero_si512();
            uint32_t t = 0;
            if (w == 64) {
                for (; t + 1 < R.n; t += 2)
                    acc = _mm512_ternarylogic_epi64(acc, _mm512_loadu_si512((const void *)(src[R.idx[t]] + p)),
                                                    _mm512_loadu_si512((const void *)(src[R.idx[t + 1]] + p)), 0x96);
                if (t < R.n) acc = _mm512_xor_si512(acc, _mm512_loadu_si512((const void *)(src[R.idx[t]] + p)));
                _mm512_storeu_si512((void *)(R.dst + p), acc);
            } else {
                for (; t + 1 < R.n; t += 2)
                    acc = _mm512_ternarylogic_epi64(acc, _mm512_maskz_loadu_epi8(mk, src[R.idx[t]] + p),
                                                    _mm512_maskz_loadu_epi8(mk, src[R.idx[t + 1]] + p), 0x96);
                if (t < R.n) acc = _mm512_xor_si512(acc, _mm512_maskz_loadu_epi8(mk, src[R.idx[t]] + p));
                _mm512_mask_storeu_epi8(R.dst + p, mk, acc);
            }
        }
    }
}

__attribute__((target("avx2"))) void apply_avx2(const OutRow *rows, int nrows, const uint8_t *const *src, int sub) {
    const int full = sub & ~31;
    for (int p = 0; p < full; p += 32) {
        for (int o = 0; o < nrows; ++o) {
            const OutRow &R = rows[o];
            __m256i a0 = R.init ? _mm256_loadu_si256((const __m256i *)(R.init + p)) : _mm256_setzero_si256();
            __m256i a1 = _mm256_setzero_si256();
            uint32_t t = 0;
            for (; t + 1 < R.n; t += 2) {
                a0 = _mm256_xor_si256(a0, _mm256_loadu_si256((const __m256i *)(src[R.idx[t]] + p)));
                a1 = _mm256_xor_si256(a1, _mm256_loadu_si256((const __m256i *)(src[R.idx[t + 1]] + p)));
            }
            if (t < R.n) a0 = _mm256_xor_si256(a0, _mm256_loadu_si256((const __m256i *)(src[R.idx[t]] + p)));
            _mm256_storeu_si256((__m256i *)(R.dst + p), _mm256_xor_si256(a0, a1));
        }
    }
    if (full < sub) apply_scalar(rows, nrows, src, sub, full);
}

enum Isa { kScalar = 0, kAvx2 = 1, kAvx512 = 2 };

Isa detect() {
    static const Isa hw = [] {
        __builtin_cpu_init();
        if (__builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512bw")) return kAvx512;
        if (__builtin_cpu_supports("avx2")) return kAvx2;
        return kScalar;
    }();
    // LONGHAIR_AMD_HOST_ISA=avx2|scalar caps the level (the tests run every variant).
    const char *cap = std::getenv("LONGHAIR_AMD_HOST_ISA");
    if (!cap) return hw;
    const Isa lim = std::strcmp(cap, "scalar") == 0 ? kScalar : std::strcmp(cap, "avx2") == 0 ? kAvx2 : kAvx512;
    return hw < lim ? hw : lim;
}

void apply(const OutRow *rows, int nrows, const uint8_t *const *src, int sub) {
    switch (detect()) {
        case kAvx512: apply_avx512(rows, nrows, src, sub); break;
        case kAvx2: apply_avx2(rows, nrows, src, sub); break;
        default: apply_scalar(rows, nrows, src, sub, 0); break;
    }
}

// The 8 output rows of matrix row r of term list T, written to dst + y * sub.
void term_rows(const Terms &T, int r, uint8_t *dst, int sub, const uint8_t *init, int init_sub, OutRow *out) {
    for (int y = 0; y < 8; ++y) {
        const uint32_t b = T.begin[(size_t)8 * r + y], e = T.begin[(size_t)8 * r + y + 1];
        out[y] = OutRow{T.idx.data() + b, e - b, dst + (size_t)y * sub, init ? init + (size_t)y * init_sub : nullptr};
    }
}

// out = XOR of n blocks of `bytes` bytes (out may alias in[0]: every chunk is read
// before it is written).
__attribute__((target("avx512f,avx512bw"))) void xor_avx512(uint8_t *out, const uint8_t *const *in, int n,
                                                               int bytes) {
    for (int p = 0; p < bytes; p += 64) {
        const int w = std::min(64, bytes - p);
        const __mmask64 mk = w == 64 ? ~0ull : ((1ull << w) - 1);
        __m512i acc = _mm512_maskz_loadu_epi8(mk, in[0] + p);
        int j = 1;
        for (; j + 1 < n; j += 2)
            acc = _mm512_ternarylogic_epi64(acc, _mm512_maskz_loadu_epi8(mk, in[j] + p),
                                            _mm512_maskz_loadu_epi8(mk, in[j + 1] + p), 0x96);
        if (j < n) acc = _mm512_xor_si512(acc, _mm512_maskz_loadu_epi8(mk, in[j] + p));
        _mm512_mask_storeu_epi8(out + p, mk, acc);
    }
}

__attribute__((target("avx2"))) void xor_avx2(uint8_t *out, const uint8_t *const *in, int n, int bytes) {
    int p = 0;
    for (; p + 32 <= bytes; p += 32) {
        __m256i acc = _mm256_loadu_si256((const __m256i *)(in[0] + p));
        for (int j = 1; j < n; ++j) acc = _mm256_xor_si256(acc, _mm256_loadu_si256((const __m256i *)(in[j] + p)));
        _mm256_storeu_si256((__m256i *)(out + p), acc);
    }
    for (; p < bytes; ++p) {
        uint8_t acc = in[0][p];
        for (int j = 1; j < n; ++j) acc ^= in[j][p];
        out[p] = acc;
    }
}

void xor_blocks(uint8_t *out, const uint8_t *const *in, int n, int bytes) {
    switch (detect()) {
        case kAvx512: xor_avx512(out, in, n, bytes); break;
        case kAvx2: xor_avx2(out, in, n, bytes); break;
        default:
            for (int p = 0; p < bytes; ++p) {
                uint8_t acc = in[0][p];
                for (int j = 1; j < n; ++j) acc ^= in[j][p];
                out[p] = acc;
            }
    }
}

// Per (k, m): the generator and its full term list (rows 0..m-1), built once.
struct ShapeCache {
    std::mutex mu;
    struct Entry {
        std::vector<uint8_t> G;
        Terms T;
    };
    std::map<std::pair<int, int>, Entry> shapes;  // entries are never erased
};

const ShapeCache::Entry &shape(int k, int m) {
    static ShapeCache c;
    std::lock_guard<std::mutex> g(c.mu);
    auto it = c.shapes.find({k, m});
    if (it == c.shapes.end()) {
        ShapeCache::Entry e;
        e.G = generator_matrix(k, m);
        build_terms(e.G.data(), m, k, &e.T);
        it = c.shapes.emplace(std::make_pair(k, m), std::move(e)).first;
    }
    return it->second;  // the reference stays valid unlocked
}

}  // namespace

const char *isa_name() {
    switch (detect()) {
        case kAvx512: return "avx512bw";
        case kAvx2: return "avx2";
        default: return "scalar";
    }
}

// cauchy_256_encode semantics (cauchy_256.cpp:1495-1594); the caller validated k, m >= 1.
int encode(int k, int m, const uint8_t *const *data, uint8_t *rec, int bytes) {
    if (k <= 1) {  // :1501-1509
        for (int r = 0; r < m; ++r) std::memcpy(rec + (size_t)r * bytes, data[0], (size_t)bytes);
        return 0;
    }
    xor_blocks(rec, data, k, bytes);  // row 0 first, whatever the parameters (:1511-1516)
    if (m == 1) return 0;
    if (k + m > 256 || bytes % 8 != 0) return -1;
    const int sub = bytes / 8;
    const ShapeCache::Entry &S = shape(k, m);
    // Per-thread scratch, not stack arrays: callers' threads may have small stacks.
    thread_local std::vector<const uint8_t *> srcv;
    thread_local std::vector<OutRow> rowv;
    srcv.resize((size_t)8 * k);
    rowv.resize((size_t)8 * (m - 1));
    const uint8_t **src = srcv.data();
    for (int x = 0; x < k; ++x)
        for (int b = 0; b < 8; ++b) src[8 * x + b] = data[x] + (size_t)b * sub;
    OutRow *rows = rowv.data();
    for (int r = 1; r < m; ++r) term_rows(S.T, r, rec + (size_t)r * bytes, sub, nullptr, 0, rows + 8 * (r - 1));
    apply(rows, 8 * (m - 1), src, sub);
    return 0;
}

// cauchy_256_decode semantics for valid parameters with at least one recovery block and
// m > 1 (the caller handles k <= 1, m == 1, no erasure and the parameter checks).
// Returns -1 (blocks untouched) for duplicate or out-of-range rows.  Same two phases as
// the GPU kernels: V_j = R_j + sum_{x present} B(G[r_j][x]) D_x for each recovery block j
// (the cached generator terms; erased columns read a zero block), then
// D_{E_i} = sum_j B(A^-1[i][j]) V_j with A = G[rows of the recovery blocks][erased rows].
int decode(int k, int m, Block *blocks, int bytes) {
    const Field &F = Field::get();
    int slot_of_row[256];
    for (int r = 0; r < k + m; ++r) slot_of_row[r] = -1;
    int rcv[256], e = 0;  // slots of the recovery blocks, array order
    for (int i = 0; i < k; ++i) {
        const int r = blocks[i].row;
        if (r >= k + m || slot_of_row[r] >= 0) return -1;
        slot_of_row[r] = i;
        if (r >= k) rcv[e++] = i;
    }
    int erased[256], ne = 0;  // missing original rows, ascending (sort_blocks, :538-570)
    for (int x = 0; x < k && ne < e; ++x)
        if (slot_of_row[x] < 0) erased[ne++] = x;
    const ShapeCache::Entry &S = shape(k, m);
    const uint8_t *G = S.G.data();
    // A[j][i] = G[row of recovery j - k][erased i]; Gauss-Jordan for A^-1.
    thread_local std::vector<uint8_t> AI;
    AI.assign((size_t)2 * e * e, 0);
    uint8_t *A = AI.data(), *I = A + (size_t)e * e;
    for (int j = 0; j < e; ++j) {
        I[(size_t)j * e + j] = 1;
        for (int i = 0; i < e; ++i) A[(size_t)j * e + i] = G[(size_t)(blocks[rcv[j]].row - k) * k + erased[i]];
    }
    for (int c = 0; c < e; ++c) {
        int p = c;
        while (p < e && !A[(size_t)p * e + c]) ++p;
        if (p == e) return -1;  // singular: cannot happen for a Cauchy-derived matrix
        if (p != c)
            for (int q = 0; q < e; ++q) {
                std::swap(A[(size_t)p * e + q], A[(size_t)c * e + q]);
                std::swap(I[(size_t)p * e + q], I[(size_t)c * e + q]);
            }
        const uint8_t inv = F.inv[A[(size_t)c * e + c]];
        for (int q = 0; q < e; ++q) {
            A[(size_t)c * e + q] = F.mul(A[(size_t)c * e + q], inv);
            I[(size_t)c * e + q] = F.mul(I[(size_t)c * e + q], inv);
        }
        for (int r = 0; r < e; ++r) {
            const uint8_t f = A[(size_t)r * e + c];
            if (r == c || !f) continue;
            for (int q = 0; q < e; ++q) {
                A[(size_t)r * e + q] ^= F.mul(f, A[(size_t)c * e + q]);
                I[(size_t)r * e + q] ^= F.mul(f, I[(size_t)c * e + q]);
            }
        }
    }
    const int sub = bytes / 8;
    // Phase A into a scratch V (e blocks); erased columns read a zero block.
    thread_local std::vector<uint8_t> zero, V;
    if (zero.size() < (size_t)bytes) zero.assign((size_t)bytes, 0);
    if (V.size() < (size_t)e * bytes) V.resize((size_t)e * bytes);
    thread_local std::vector<const uint8_t *> srcv;
    srcv.resize((size_t)8 * k);
    const uint8_t **src = srcv.data();
    for (int x = 0; x < k; ++x) {
        const uint8_t *d = slot_of_row[x] >= 0 ? blocks[slot_of_row[x]].data : zero.data();
        for (int b = 0; b < 8; ++b) src[8 * x + b] = d + (size_t)b * sub;
    }
    thread_local std::vector<OutRow> rows;
    rows.resize((size_t)8 * e);
    for (int j = 0; j < e; ++j)
        term_rows(S.T, blocks[rcv[j]].row - k, V.data() + (size_t)j * bytes, sub, blocks[rcv[j]].data, sub,
                  rows.data() + 8 * j);
    apply(rows.data(), 8 * e, src, sub);
    // Phase B: recovery slot i (array order) receives erased row i.
    thread_local Terms TB;
    build_terms(I, e, e, &TB);
    for (int j = 0; j < e; ++j)  // phase A's inputs are consumed: src now names V's sub-blocks
        for (int b = 0; b < 8; ++b) src[8 * j + b] = V.data() + (size_t)j * bytes + (size_t)b * sub;
    for (int i = 0; i < e; ++i) term_rows(TB, i, blocks[rcv[i]].data, sub, nullptr, 0, rows.data() + 8 * i);
    apply(rows.data(), 8 * e, src, sub);
    for (int i = 0; i < e; ++i) blocks[rcv[i]].row = (unsigned char)erased[i];
    return 0;
}

// cauchy_decode_m1 (cauchy_256.cpp:487-535), including its no-erasure quirk: with no
// recovery block present, blocks[0] is the output.
void decode_m1(int k, Block *blocks, int bytes) {
    Block *out = blocks;
    bool seen[256] = {};
    for (int i = 0; i < k; ++i) {
        if (blocks[i].row >= k) out = &blocks[i];
        else seen[blocks[i].row] = true;
    }
    for (int x = 0; x < k; ++x)
        if (!seen[x]) {
            out->row = (unsigned char)x;
            break;
        }
    std::vector<const uint8_t *> in;
    in.push_back(out->data);
    for (int i = 0; i < k; ++i)
        if (&blocks[i] != out) in.push_back(blocks[i].data);
    xor_blocks(out->data, in.data(), (int)in.size(), bytes);
}

}  // namespace host
}  // namespace lh
