// host_codec.hpp -- host SIMD engine of the drop-in dispatch policy (host_codec.cpp).
#pragma once

#include <cstdint>

#include "../../include/cauchy_256.h"

namespace lh {
namespace host {

// cauchy_256_encode semantics for one stripe in host memory (k, m >= 1).
int encode(int k, int m, const uint8_t *const *data, uint8_t *rec, int bytes);
// cauchy_256_decode for m > 1, valid k + m and bytes, at least one recovery block:
// 0, or -1 (untouched) for duplicate / out-of-range rows.
int decode(int k, int m, Block *blocks, int bytes);
// cauchy_decode_m1 semantics (m == 1, k > 1).
void decode_m1(int k, Block *blocks, int bytes);
// "avx512bw", "avx2" or "scalar": the instruction set the engine dispatched to.
const char *isa_name();

}  // namespace host
}  // namespace lh
