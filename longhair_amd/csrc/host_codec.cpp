// host_codec.cpp -- the host SIMD engine of the drop-in dispatch policy (SURVEY.md §8f,
// rank 2): one stripe per call from host memory, the reference's call shape
// (cauchy_256.h:78, :103; README.md:111-182).  A single small stripe is latency-bound:
// staging it over PCIe to the GPU costs ~30-66 us per call where the bit-sliced XOR work
// itself is ~2 us of AVX-512 (profiles/r2_bench_k29m4.json, dropin_per_call).  The
// policy (codec.cpp) sends such calls here only when the caller selects it
// (cauchy_256_set_dispatch / LONGHAIR_AMD_DISPATCH); the library still requires a GPU.
//
// Both operations are one bit-sliced coefficient apply (same algebra as the GPU kernels):
//   out[i] sub-row y  ^=  in[j] sub-block b   for every bit b of C[i][j] * 2^y,
// encode with C = the generator rows 1..m-1 (row 0 is the plain XOR, as the reference
// writes it first: cauchy_256.cpp:1511-1516), decode with C = [A^-1 G_present | A^-1]
// over the k received blocks, A = G[recovery rows][erased rows] (cauchy_256.cpp:707-790
// solve the same system bit by bit; the solution is unique, so the bytes are equal).
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

void build_terms(const uint8_t *C, int nout, int nin, Terms *T) {
    T->nout = nout;
    T->nin = nin;
    T->begin.assign((size_t)nout * 8 + 1, 0);
    T->idx.clear();
    T->idx.reserve((size_t)nout * nin * 32);
    std::vector<uint64_t> bm((size_t)nin);
    for (int i = 0; i < nout; ++i) {
        for (int j = 0; j < nin; ++j) bm[j] = bitmatrix(C[(size_t)i * nin + j]);
        for (int y = 0; y < 8; ++y) {
            T->begin[(size_t)i * 8 + y] = (uint32_t)T->idx.size();
            for (int j = 0; j < nin; ++j) {
                const unsigned s = (unsigned)((bm[j] >> (8 * y)) & 0xFF);
                for (unsigned b = 0; b < 8; ++b)
                    if (s & (1u << b)) T->idx.push_back((uint16_t)(8 * j + b));
            }
        }
    }
    T->begin[(size_t)nout * 8] = (uint32_t)T->idx.size();
}

// Scalar tail / fallback: bytes [p0, sub) of every output sub-row, through a staging row
// so in-place outputs never feed later terms.
void apply_scalar(const Terms &T, const uint8_t *const *src, uint8_t *const *dst, int sub, int p0, uint8_t *tmp) {
    const int nrow = T.nout * 8;
    for (int p = p0; p < sub; p += 64) {
        const int n = std::min(64, sub - p);
        for (int o = 0; o < nrow; ++o) {
            uint8_t acc[64];
            std::memset(acc, 0, (size_t)n);
            for (uint32_t t = T.begin[o]; t < T.begin[o + 1]; ++t) {
                const uint8_t *s = src[T.idx[t]] + p;
                for (int q = 0; q < n; ++q) acc[q] ^= s[q];
            }
            std::memcpy(tmp + (size_t)o * 64, acc, (size_t)n);
        }
        for (int o = 0; o < nrow; ++o) std::memcpy(dst[o] + p, tmp + (size_t)o * 64, (size_t)n);
    }
}

__attribute__((target("avx512f,avx512bw"))) void apply_avx512(const Terms &T, const uint8_t *const *src,
                                                                 uint8_t *const *dst, int sub, uint8_t *tmp) {
    const int nrow = T.nout * 8;
    for (int p = 0; p < sub; p += 64) {
        const int n = std::min(64, sub - p);
        const __mmask64 mk = n == 64 ? ~0ull : ((1ull << n) - 1);
        for (int o = 0; o < nrow; ++o) {
            __m512i acc = _mm512_setzero_si512();
            uint32_t t = T.begin[o];
            const uint32_t e = T.begin[o + 1];
            for (; t + 1 < e; t += 2)
                acc = _mm512_ternarylogic_epi64(acc, _mm512_maskz_loadu_epi8(mk, src[T.idx[t]] + p),
                                                _mm512_maskz_loadu_epi8(mk, src[T.idx[t + 1]] + p), 0x96);
            if (t < e) acc = _mm512_xor_si512(acc, _mm512_maskz_loadu_epi8(mk, src[T.idx[t]] + p));
            _mm512_store_si512((void *)(tmp + (size_t)o * 64), acc);
        }
        // Outputs are written after every input of this chunk was read (in-place decode).
        for (int o = 0; o < nrow; ++o)
            _mm512_mask_storeu_epi8(dst[o] + p, mk, _mm512_load_si512((const void *)(tmp + (size_t)o * 64)));
    }
}

__attribute__((target("avx2"))) void apply_avx2(const Terms &T, const uint8_t *const *src, uint8_t *const *dst,
                                                 int sub, uint8_t *tmp) {
    const int nrow = T.nout * 8;
    const int full = sub & ~31;
    for (int p = 0; p < full; p += 32) {
        for (int o = 0; o < nrow; ++o) {
            __m256i a0 = _mm256_setzero_si256(), a1 = _mm256_setzero_si256();
            uint32_t t = T.begin[o];
            const uint32_t e = T.begin[o + 1];
            for (; t + 1 < e; t += 2) {
                a0 = _mm256_xor_si256(a0, _mm256_loadu_si256((const __m256i *)(src[T.idx[t]] + p)));
                a1 = _mm256_xor_si256(a1, _mm256_loadu_si256((const __m256i *)(src[T.idx[t + 1]] + p)));
            }
            if (t < e) a0 = _mm256_xor_si256(a0, _mm256_loadu_si256((const __m256i *)(src[T.idx[t]] + p)));
            _mm256_storeu_si256((__m256i *)(tmp + (size_t)o * 32), _mm256_xor_si256(a0, a1));
        }
        for (int o = 0; o < nrow; ++o)
            _mm256_storeu_si256((__m256i *)(dst[o] + p), _mm256_loadu_si256((const __m256i *)(tmp + (size_t)o * 32)));
    }
    if (full < sub) apply_scalar(T, src, dst, sub, full, tmp);
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

// src: nin * 8 sub-block pointers, dst: nout * 8 sub-row pointers.
void apply(const Terms &T, const uint8_t *const *src, uint8_t *const *dst, int sub) {
    thread_local std::vector<uint8_t> tmp_store;
    const size_t need = (size_t)T.nout * 8 * 64 + 64;
    if (tmp_store.size() < need) tmp_store.resize(need);
    uint8_t *tmp = (uint8_t *)(((uintptr_t)tmp_store.data() + 63) & ~(uintptr_t)63);
    switch (detect()) {
        case kAvx512: apply_avx512(T, src, dst, sub, tmp); break;
        case kAvx2: apply_avx2(T, src, dst, sub, tmp); break;
        default: apply_scalar(T, src, dst, sub, 0, tmp); break;
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

struct EncodeCache {
    std::mutex mu;
    std::map<std::pair<int, int>, Terms> terms;  // (k, m) -> rows 1..m-1 of the generator
};

EncodeCache &encode_cache() {
    static EncodeCache c;
    return c;
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
    const Terms *T = nullptr;
    {
        EncodeCache &c = encode_cache();
        std::lock_guard<std::mutex> g(c.mu);
        auto it = c.terms.find({k, m});
        if (it == c.terms.end()) {
            const std::vector<uint8_t> G = generator_matrix(k, m);
            Terms t;
            build_terms(G.data() + k, m - 1, k, &t);
            it = c.terms.emplace(std::make_pair(k, m), std::move(t)).first;
        }
        T = &it->second;  // entries are never erased: the reference stays valid unlocked
    }
    std::vector<const uint8_t *> src((size_t)k * 8);
    for (int x = 0; x < k; ++x)
        for (int b = 0; b < 8; ++b) src[(size_t)8 * x + b] = data[x] + (size_t)b * sub;
    std::vector<uint8_t *> dst((size_t)(m - 1) * 8);
    for (int r = 1; r < m; ++r)
        for (int y = 0; y < 8; ++y) dst[(size_t)8 * (r - 1) + y] = rec + (size_t)r * bytes + (size_t)y * sub;
    apply(*T, src.data(), dst.data(), sub);
    return 0;
}

// cauchy_256_decode semantics for valid parameters with at least one recovery block and
// m > 1 (the caller handles k <= 1, m == 1, no erasure and the parameter checks).
// Returns -1 (blocks untouched) for duplicate or out-of-range rows.
int decode(int k, int m, Block *blocks, int bytes) {
    const Field &F = Field::get();
    int slot_of_row[256];
    for (int r = 0; r < k + m; ++r) slot_of_row[r] = -1;
    std::vector<int> present, rcv;  // slots of originals / recovery blocks, array order
    for (int i = 0; i < k; ++i) {
        const int r = blocks[i].row;
        if (r >= k + m || slot_of_row[r] >= 0) return -1;
        slot_of_row[r] = i;
        (r < k ? present : rcv).push_back(i);
    }
    const int e = (int)rcv.size();
    std::vector<int> erased;  // missing original rows, ascending (sort_blocks, :538-570)
    for (int x = 0; x < k && (int)erased.size() < e; ++x)
        if (slot_of_row[x] < 0) erased.push_back(x);
    const std::vector<uint8_t> G = generator_matrix(k, m);
    // A[j][i] = G[row of recovery j - k][erased i]; Gauss-Jordan for A^-1.
    std::vector<uint8_t> A((size_t)e * e), I((size_t)e * e, 0);
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
    // D_E = A^-1 (R - G_p D_p): coefficients over the k received blocks in array order.
    // Inputs: present originals (coefficient -(A^-1 G[rcv rows][x]) = A^-1 G, char 2) and
    // recovery blocks (coefficient A^-1).
    const int sub = bytes / 8;
    std::vector<uint8_t> C((size_t)e * k, 0);
    for (int i = 0; i < e; ++i) {
        for (int jj = 0; jj < e; ++jj) C[(size_t)i * k + rcv[jj]] = I[(size_t)i * e + jj];
        for (int s : present) {
            const int x = blocks[s].row;
            uint8_t acc = 0;
            for (int jj = 0; jj < e; ++jj)
                acc ^= F.mul(I[(size_t)i * e + jj], G[(size_t)(blocks[rcv[jj]].row - k) * k + x]);
            C[(size_t)i * k + s] = acc;
        }
    }
    Terms T;
    build_terms(C.data(), e, k, &T);
    std::vector<const uint8_t *> src((size_t)k * 8);
    for (int s = 0; s < k; ++s)
        for (int b = 0; b < 8; ++b) src[(size_t)8 * s + b] = blocks[s].data + (size_t)b * sub;
    std::vector<uint8_t *> dst((size_t)e * 8);
    for (int i = 0; i < e; ++i)  // recovery slot i (array order) receives erased row i
        for (int y = 0; y < 8; ++y) dst[(size_t)8 * i + y] = blocks[rcv[i]].data + (size_t)y * sub;
    apply(T, src.data(), dst.data(), sub);
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
