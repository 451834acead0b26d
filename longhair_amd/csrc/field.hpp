// field.hpp -- GF(256) arithmetic (polynomial 0x187) and the Cauchy generator rows.
//
// Host-side half of the codec: the field tables are regenerated from the polynomial
// (the reference hard-codes them, cauchy_256.cpp:273-344) and the generator rows come
// from the reference's constants, embedded from data/cauchy_tables_256.bin.
#pragma once

#include <cstdint>
#include <vector>

namespace lh {

struct Field {
    uint8_t exp[512];
    int16_t log[256];
    uint8_t inv[256];

    Field();
    static const Field &get();

    uint8_t mul(uint8_t a, uint8_t b) const {
        return (a && b) ? exp[log[a] + log[b]] : 0;
    }
    // Reference GFC256Divide semantics: x / 0 == 0 (cauchy_256.cpp:359-387).
    uint8_t div(uint8_t a, uint8_t b) const {
        return (a && b) ? exp[log[a] + 255 - log[b]] : 0;
    }
    static uint8_t xtime(uint8_t v) { return (uint8_t)((v << 1) ^ ((v & 0x80) ? 0x87 : 0)); }
};

// Full m x k generator over GF(256): row 0 is all ones (recovery block 0 = XOR of the
// data, cauchy_256.cpp:1511-1516), rows 1..m-1 are the reference's Cauchy rows
// (cauchy_matrix, cauchy_256.cpp:423-481).  Preconditions: k >= 1, m >= 1, k + m <= 256.
std::vector<uint8_t> generator_matrix(int k, int m);
bool cauchy_points(int k, int m, std::vector<uint8_t> &xs, std::vector<uint8_t> &ys);

// Expanded 8x8 GF(2) bit-matrix of element e, one byte per bit-row: row y = e * 2^y.
// Bit b of row y set <=> data sub-block b contributes to output sub-block y.
inline uint64_t bitmatrix(uint8_t e) {
    uint64_t r = 0;
    for (int y = 0; y < 8; ++y, e = Field::xtime(e)) r |= (uint64_t)e << (8 * y);
    return r;
}

// Raw constants blob (tables_blob.cpp) and its expected size.
extern "C" const unsigned char lh_cauchy_tables_blob[];
extern "C" const unsigned char lh_cauchy_tables_blob_end[];
constexpr int kTablesBlobSize = 34902;

}  // namespace lh
