// kernels.hip -- ahead-of-time compiled CDNA4 (gfx950) kernels of the codec.
//
//   lh_plan_kernel          decode planner: per stripe, classify the k slots (reference
//                           sort_blocks, cauchy_256.cpp:538-570), invert the e x e
//                           GF(256) sub-matrix of the erased columns (replaces the GF(2)
//                           Gaussian elimination of :1018-1080 / :1229-1247; same unique
//                           solution) and emit the per-slot coefficients.
//   lh_apply_generic_kernel out_i = sum_j B(W[i][j]) * in_j for any per-stripe GF(256)
//                           coefficient matrix W, in the bit-sliced representation of the
//                           reference (bit-row y of element e is e * 2^y, bit b selects
//                           sub-block b: cauchy_256.cpp:1553-1587).  Used for shapes the
//                           run-time specialised kernels (jit_codec.hip) do not cover.
//   lh_xor_reduce_kernel    out = XOR of n inputs for any block size (m == 1 encode
//                           :1511-1522, k <= 1 copies :1501-1509, m == 1 decode :487-535).
//   lh_scatter_kernel       moves recovered blocks from the workspace into their slots.
//
// Lanes own W-byte columns of a stripe's sub-blocks: a lane loads the same byte range of
// all 8 sub-blocks of a block and produces the same range of all 8 output sub-blocks, so
// every output byte depends only on input bytes at the same sub-block offset.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kernels.hpp"

namespace {

template <int W>
struct Word {
    static constexpr int N = (W + 3) / 4;
    uint32_t v[N];
};

template <int W>
__device__ __forceinline__ Word<W> wload(const uint8_t *p) {
    Word<W> w;
#pragma unroll
    for (int i = 0; i < Word<W>::N; ++i) w.v[i] = 0;
    __builtin_memcpy(&w.v[0], p, W);  // unaligned global loads are legal on gfx950
    return w;
}

template <int W>
__device__ __forceinline__ void wstore(uint8_t *p, const Word<W> &w) {
    __builtin_memcpy(p, &w.v[0], W);
}

template <int W>
__device__ __forceinline__ void wzero(Word<W> &w) {
#pragma unroll
    for (int i = 0; i < Word<W>::N; ++i) w.v[i] = 0;
}

// acc ^= x & mask (one v_bitop3_b32 per dword on gfx950)
template <int W>
__device__ __forceinline__ void wxor_masked(Word<W> &acc, const Word<W> &x, uint32_t mask) {
#pragma unroll
    for (int i = 0; i < Word<W>::N; ++i) acc.v[i] ^= x.v[i] & mask;
}

template <int W>
__device__ __forceinline__ void wxor(Word<W> &acc, const Word<W> &x) {
#pragma unroll
    for (int i = 0; i < Word<W>::N; ++i) acc.v[i] ^= x.v[i];
}

// Bit-sliced multiply by 2: (B(2) v)_y = v_{y+1} for y < 7, v_0^v_1^v_2^v_7 for y = 7,
// because 2 * 2^7 reduces to 0x87 under the field polynomial 0x187.
template <int W>
__device__ __forceinline__ void mul2(const Word<W> (&in)[8], Word<W> (&out)[8]) {
#pragma unroll
    for (int y = 0; y < 7; ++y) out[y] = in[y + 1];
#pragma unroll
    for (int i = 0; i < Word<W>::N; ++i) out[7].v[i] = in[0].v[i] ^ in[1].v[i] ^ in[2].v[i] ^ in[7].v[i];
}

}  // namespace

// ------------------------------------------------------------------ generic apply
// Grid: x covers (stripe, column chunk) lanes; y covers output tiles of LH_TILE_OUT rows.
template <int W>
__global__ void __launch_bounds__(256) lh_apply_generic_kernel(lh::ApplyArgs a) {
    constexpr int TO = lh::kGenericTileOut;
    const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    const long long s = t / a.nch;
    if (s >= a.stripes) return;
    const int c = (int)(t - s * a.nch);
    // Last chunk of a sub-block re-reads the final W bytes (overlapping its neighbour
    // with identical results) instead of running past the sub-block.
    const int p = (c == a.nch - 1) ? (a.sub - W) : c * W;
    const int i0 = blockIdx.y * TO;
    int nout = a.n_out;
    if (a.nout_per_stripe) nout = a.nout_per_stripe[s * a.nout_stride];
    if (i0 >= nout) return;
    const int ni = min(TO, nout - i0);

    const uint8_t *in = a.in + s * a.in_stride + p;
    const uint8_t *coef = a.coef + s * a.coef_stride + (long long)i0 * a.n_in;

    Word<W> acc[TO][8];
#pragma unroll
    for (int i = 0; i < TO; ++i)
#pragma unroll
        for (int y = 0; y < 8; ++y) wzero(acc[i][y]);

    for (int j = 0; j < a.n_in; ++j) {
        Word<W> lad[8][8];  // lad[t] = B(2^t) * d
#pragma unroll
        for (int b = 0; b < 8; ++b) lad[0][b] = wload<W>(in + (long long)j * a.bytes + b * a.sub);
#pragma unroll
        for (int q = 1; q < 8; ++q) mul2<W>(lad[q - 1], lad[q]);
#pragma unroll
        for (int i = 0; i < TO; ++i) {
            if (i < ni) {
                const uint32_t e = coef[i * a.n_in + j];
#pragma unroll
                for (int q = 0; q < 8; ++q) {
                    const uint32_t mask = 0u - ((e >> q) & 1u);
#pragma unroll
                    for (int y = 0; y < 8; ++y) wxor_masked(acc[i][y], lad[q][y], mask);
                }
            }
        }
    }
    uint8_t *out = a.out + s * a.out_stride + (long long)i0 * a.bytes + p;
#pragma unroll
    for (int i = 0; i < TO; ++i)
        if (i < ni)
#pragma unroll
            for (int y = 0; y < 8; ++y) wstore(out + (long long)i * a.bytes + y * a.sub, acc[i][y]);
}

// --------------------------------------------------------------------- XOR reduce
// out[s][r] = XOR_j in[s][slot_j] for r < n_rep.  16-byte lanes plus a byte-wise tail, no
// overlapping chunks, so it may run in place (decode m == 1: the output slot is one of
// the inputs; every lane reads all its inputs before writing).
__global__ void __launch_bounds__(256) lh_xor_reduce_kernel(lh::XorArgs a) {
    const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    const long long s = t / a.nch;
    if (s >= a.stripes) return;
    const int c = (int)(t - s * a.nch);
    const uint8_t *in = a.in + s * a.in_stride;
    uint8_t *out;
    if (a.plan) {
        const lh::PlanView pv(a.plan + s * a.plan_stride, a.k, a.m, a.e_max);
        if (pv.e() == 0) return;
        out = a.out + s * a.out_stride + (long long)pv.out_slot(0) * a.bytes;
    } else {
        out = a.out + s * a.out_stride;
    }
    const int full = a.bytes / 16;
    if (c < full) {
        uint4 acc = make_uint4(0, 0, 0, 0);
        for (int j = 0; j < a.n_in; ++j) {
            uint4 v;
            __builtin_memcpy(&v, in + (long long)j * a.bytes + c * 16, 16);
            acc.x ^= v.x; acc.y ^= v.y; acc.z ^= v.z; acc.w ^= v.w;
        }
        for (int r = 0; r < a.n_rep; ++r) __builtin_memcpy(out + (long long)r * a.bytes + c * 16, &acc, 16);
    } else {
        const int b0 = full * 16;
        for (int q = b0; q < a.bytes; ++q) {
            uint8_t acc = 0;
            for (int j = 0; j < a.n_in; ++j) acc ^= in[(long long)j * a.bytes + q];
            for (int r = 0; r < a.n_rep; ++r) out[(long long)r * a.bytes + q] = acc;
        }
    }
}

// ------------------------------------------------------------------------ scatter
// blocks[s][out_slot[i]] = work[s][i] for i < e_s, 16 bytes per lane (bytes % 8 == 0).
__global__ void __launch_bounds__(256) lh_scatter_kernel(lh::ScatterArgs a) {
    const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    const int per_block = (a.bytes + 15) / 16;
    const long long per_stripe = (long long)per_block * a.e_max;
    const long long s = t / per_stripe;
    if (s >= a.stripes) return;
    const int rem = (int)(t - s * per_stripe);
    const int i = rem / per_block, c = rem % per_block;
    const lh::PlanView pv(a.plan + s * a.plan_stride, a.k, a.m, a.e_max);
    if (i >= pv.e()) return;
    const uint8_t *src = a.work + s * a.work_stride + (long long)i * a.bytes;
    uint8_t *dst = a.blocks + s * a.blocks_stride + (long long)pv.out_slot(i) * a.bytes;
    const int off = c * 16, n = min(16, a.bytes - off);
    if (n == 16) {
        uint4 v;
        __builtin_memcpy(&v, src + off, 16);
        __builtin_memcpy(dst + off, &v, 16);
    } else {
        for (int q = 0; q < n; ++q) dst[off + q] = src[off + q];
    }
}

// -------------------------------------------------------------------- decode plan
// One 64-lane wave per stripe.  LDS: GF tables + the e x 2e augmented matrix.
__global__ void __launch_bounds__(64) lh_plan_kernel(lh::PlanArgs a) {
    const int s = blockIdx.x;
    const int lane = threadIdx.x;
    const int k = a.k, m = a.m, e_max = a.e_max;
    __shared__ uint8_t gexp[512];
    __shared__ int16_t glog[256];
    __shared__ uint8_t rows[256];
    __shared__ uint8_t rcv_slot[256], rcv_row[256], erasure[256], orig_slot_of[256];
    __shared__ int sh_e, sh_status;
    extern __shared__ uint8_t aug[];  // e_max x (2 * e_max)

    for (int i = lane; i < 256; i += 64) {
        gexp[i] = a.gf_exp[i];
        gexp[i + 256] = a.gf_exp[i + 256];
        glog[i] = a.gf_log[i];
    }
    uint8_t *rws = a.rows + (long long)s * k;
    for (int i = lane; i < k; i += 64) rows[i] = rws[i];
    __syncthreads();

    auto gmul = [&](uint8_t x, uint8_t y) -> uint8_t {
        return (x && y) ? gexp[glog[x] + glog[y]] : (uint8_t)0;
    };

    uint8_t *rec = a.plan + (long long)s * a.plan_stride;
    lh::PlanView pv(rec, k, m, e_max);

    if (lane == 0) {
        // Classification in array order (reference sort_blocks).  Rows outside the code
        // or repeated make the stripe invalid (undefined behaviour in the reference).
        uint8_t seen[256];
        for (int i = 0; i < 256; ++i) seen[i] = 0;
        int status = 0, n_rcv = 0;
        for (int i = 0; i < 256; ++i) orig_slot_of[i] = 0xFF;
        for (int i = 0; i < k; ++i) {
            const int r = rows[i];
            if (r >= k + m || seen[r]) status = -1;
            else seen[r] = 1;
            if (r < k) orig_slot_of[r] = (uint8_t)i;
            else if (n_rcv < 256) { rcv_slot[n_rcv] = (uint8_t)i; rcv_row[n_rcv] = (uint8_t)(r - k); ++n_rcv; }
        }
        int e = 0;
        if (status == 0) {
            if (k <= 1) {
                rows[0] = 0;  // cauchy_256.cpp:1252-1256
            } else if (m == 1) {
                // cauchy_decode_m1 (:487-535): the recovery block (or blocks[0] when none is
                // present) becomes the XOR of all k blocks and takes the first missing row.
                int out = 0;
                for (int i = 0; i < k; ++i) if (rows[i] >= k) out = i;
                int miss = -1;
                for (int i = 0; i < k; ++i) if (!seen[i]) { miss = i; break; }
                if (miss >= 0) rows[out] = (uint8_t)miss;
                rcv_slot[0] = (uint8_t)out;
                e = 1;
            } else {
                for (int i = 0, j = 0; i < 256 && j < n_rcv; ++i)
                    if (!seen[i]) erasure[j++] = (uint8_t)i;
                e = n_rcv;
            }
        }
        sh_e = e;
        sh_status = status;
    }
    __syncthreads();
    const int e = sh_e;
    if (lane == 0) {
        rec[0] = (uint8_t)e;
        rec[1] = (uint8_t)(int8_t)sh_status;
        if (a.status) a.status[s] = (int8_t)sh_status;
    }
    if (sh_status != 0) {
        if (lane == 0) rec[0] = 0;
        return;
    }
    if (m == 1 || k <= 1) {
        if (lane == 0 && e) pv.set_out_slot(0, rcv_slot[0]);
        for (int i = lane; i < k; i += 64) rws[i] = rows[i];
        return;
    }
    if (e == 0) return;

    // Augmented [A | I] with A[i][j] = G[r_i][E_j] (r_i = recovery row of the i-th
    // recovery slot, E_j = j-th missing original).
    const int w2 = 2 * e;
    for (int q = lane; q < e * w2; q += 64) {
        const int i = q / w2, j = q % w2;
        uint8_t v;
        if (j < e) v = a.G[rcv_row[i] * k + erasure[j]];
        else v = (j - e == i) ? 1 : 0;
        aug[i * w2 + j] = v;
    }
    __syncthreads();
    // Gauss-Jordan over GF(256).
    for (int col = 0; col < e; ++col) {
        __shared__ int piv;
        if (lane == 0) {
            int p = -1;
            for (int r = col; r < e; ++r) if (aug[r * w2 + col]) { p = r; break; }
            piv = p;
        }
        __syncthreads();
        const int p = piv;
        if (p < 0) {  // singular: cannot happen for distinct valid rows (Cauchy MDS)
            if (lane == 0) { rec[0] = 0; rec[1] = 0xFF; if (a.status) a.status[s] = -1; }
            return;
        }
        if (p != col) {
            for (int j = lane; j < w2; j += 64) {
                const uint8_t t0 = aug[col * w2 + j];
                aug[col * w2 + j] = aug[p * w2 + j];
                aug[p * w2 + j] = t0;
            }
        }
        __syncthreads();
        const uint8_t pinv = gexp[255 - glog[aug[col * w2 + col]]];
        __syncthreads();
        for (int j = lane; j < w2; j += 64) aug[col * w2 + j] = gmul(aug[col * w2 + j], pinv);
        __syncthreads();
        for (int q = lane; q < e * w2; q += 64) {
            const int r = q / w2, j = q % w2;
            if (r == col) continue;
            const uint8_t f = aug[r * w2 + col];
            if (j == col) continue;  // column `col` cleared below, after every row used f
            aug[r * w2 + j] ^= gmul(f, aug[col * w2 + j]);
        }
        __syncthreads();
        for (int r = lane; r < e; r += 64) if (r != col) aug[r * w2 + col] = 0;
        __syncthreads();
    }
    // Ainv[i][j] = aug[i][e + j].  Emit: out slots, src/rec slot maps, coef (e x m over
    // recovery rows) and W (e x k over slots).
    for (int i = lane; i < e; i += 64) pv.set_out_slot(i, rcv_slot[i]);
    for (int x = lane; x < k; x += 64) pv.set_src_slot(x, orig_slot_of[x]);
    for (int r = lane; r < m; r += 64) pv.set_rec_slot(r, 0xFF);
    __syncthreads();
    for (int j = lane; j < e; j += 64) pv.set_rec_slot(rcv_row[j], rcv_slot[j]);
    for (int q = lane; q < e * m; q += 64) pv.set_coef(q / m, q % m, 0);
    __syncthreads();
    for (int q = lane; q < e * e; q += 64) {
        const int i = q / e, j = q % e;
        pv.set_coef(i, rcv_row[j], aug[i * w2 + e + j]);
    }
    for (int q = lane; a.want_w && q < e * k; q += 64) {
        const int i = q / k, slot = q % k;
        const int r = rows[slot];
        uint8_t v = 0;
        if (r >= k) {
            for (int j = 0; j < e; ++j) if (rcv_slot[j] == slot) v = aug[i * w2 + e + j];
        } else {
            for (int j = 0; j < e; ++j) v ^= gmul(aug[i * w2 + e + j], a.G[rcv_row[j] * k + r]);
        }
        pv.set_w(i, slot, v);
    }
    __syncthreads();
    // Recovery slot i takes erased row E_i (reference generate_bitmatrix, :786).
    for (int i = lane; i < e; i += 64) rows[rcv_slot[i]] = erasure[i];
    __syncthreads();
    for (int i = lane; i < k; i += 64) rws[i] = rows[i];
}

// ------------------------------------------------------- decode plan, small e_max
// One thread per stripe for e_max <= EM (m <= 8 or k <= 8): the e x e inverse lives in
// registers (padded to EM x EM with an identity block so every loop bound is a compile-
// time constant), GF(256) log/exp tables in LDS.  Same record as lh_plan_kernel.
template <int EM>
__global__ void __launch_bounds__(256) lh_plan_small_kernel(lh::PlanArgs a) {
    __shared__ uint8_t gexp[512];
    __shared__ int16_t glog[256];
    for (int i = threadIdx.x; i < 256; i += blockDim.x) {
        gexp[i] = a.gf_exp[i];
        gexp[i + 256] = a.gf_exp[i + 256];
        glog[i] = a.gf_log[i];
    }
    __syncthreads();
    const long long s = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= a.stripes) return;
    const int k = a.k, m = a.m, e_max = a.e_max;
    auto gmul = [&](uint32_t x, uint32_t y) -> uint32_t {
        return (x && y) ? gexp[glog[x] + glog[y]] : 0u;
    };
    uint8_t *rws = a.rows + s * k;
    uint8_t *rec = a.plan + s * a.plan_stride;
    lh::PlanView pv(rec, k, m, e_max);

    // Classify slots (reference sort_blocks): seen-bitmap over rows, recovery slots in
    // array order; rows outside the code or repeated invalidate the stripe.
    uint32_t seen[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    int n_rcv = 0, status = 0;
    uint32_t rslot[EM], rrow[EM];
#pragma unroll
    for (int i = 0; i < EM; ++i) rslot[i] = rrow[i] = 0;
    for (int x = 0; x < k; ++x) pv.set_src_slot(x, 0xFF);
    for (int i = 0; i < k; ++i) {
        const uint32_t r = rws[i];
        const uint32_t bit = 1u << (r & 31);
        uint32_t w = 0;
#pragma unroll
        for (int q = 0; q < 8; ++q) if ((int)(r >> 5) == q) w = seen[q];
        if (r >= (uint32_t)(k + m) || (w & bit)) status = -1;
#pragma unroll
        for (int q = 0; q < 8; ++q) if ((int)(r >> 5) == q) seen[q] |= bit;
        if (r < (uint32_t)k) {
            pv.set_src_slot(r, (uint8_t)i);
        } else {
#pragma unroll
            for (int q = 0; q < EM; ++q) if (q == n_rcv) { rslot[q] = i; rrow[q] = r - k; }
            ++n_rcv;
        }
    }
    if (n_rcv > e_max) status = -1;
    if (a.status) a.status[s] = (int8_t)status;
    rec[1] = (uint8_t)(int8_t)status;
    if (status != 0 || n_rcv == 0) {
        rec[0] = 0;
        return;
    }
    const int e = n_rcv;
    rec[0] = (uint8_t)e;
    // Missing originals, ascending.
    uint32_t er[EM];
#pragma unroll
    for (int i = 0; i < EM; ++i) er[i] = 0;
    for (int x = 0, j = 0; x < k && j < e; ++x) {
        if (!((seen[x >> 5] >> (x & 31)) & 1u)) {
#pragma unroll
            for (int q = 0; q < EM; ++q) if (q == j) er[q] = x;
            ++j;
        }
    }
    // [A | I], A[i][j] = G[r_i][E_j], identity padding beyond e.
    uint32_t A[EM][EM], I[EM][EM];
#pragma unroll
    for (int i = 0; i < EM; ++i)
#pragma unroll
        for (int j = 0; j < EM; ++j) {
            uint32_t v;
            if (i < e && j < e) v = a.G[rrow[i] * k + er[j]];
            else v = (i == j) ? 1u : 0u;
            A[i][j] = v;
            I[i][j] = (i == j) ? 1u : 0u;
        }
#pragma unroll
    for (int c = 0; c < EM; ++c) {
        // Pivot: first row p >= c with A[p][c] != 0; swap into row c.
        int p = -1;
#pragma unroll
        for (int r = EM - 1; r >= c; --r) if (A[r][c]) p = r;
        if (p < 0) { status = -1; break; }
#pragma unroll
        for (int r = c + 1; r < EM; ++r) {
            if (r == p) {
#pragma unroll
                for (int j = 0; j < EM; ++j) {
                    uint32_t t = A[c][j]; A[c][j] = A[r][j]; A[r][j] = t;
                    t = I[c][j]; I[c][j] = I[r][j]; I[r][j] = t;
                }
            }
        }
        const uint32_t inv = gexp[255 - glog[A[c][c]]];
#pragma unroll
        for (int j = 0; j < EM; ++j) { A[c][j] = gmul(A[c][j], inv); I[c][j] = gmul(I[c][j], inv); }
#pragma unroll
        for (int r = 0; r < EM; ++r) {
            if (r == c) continue;
            const uint32_t f = A[r][c];
            if (f) {
#pragma unroll
                for (int j = 0; j < EM; ++j) { A[r][j] ^= gmul(f, A[c][j]); I[r][j] ^= gmul(f, I[c][j]); }
            }
        }
    }
    if (status != 0) {
        rec[0] = 0;
        rec[1] = 0xFF;
        if (a.status) a.status[s] = -1;
        return;
    }
    // Emit out slots, recovery slot map and coef[i][r] (A^-1 over recovery rows).
    for (int r = 0; r < m; ++r) pv.set_rec_slot(r, 0xFF);
    for (int q = 0; q < e_max * m; ++q) pv.set_coef(q / m, q % m, 0);
#pragma unroll
    for (int i = 0; i < EM; ++i) {
        if (i < e) {
            pv.set_out_slot(i, (uint8_t)rslot[i]);
            pv.set_rec_slot(rrow[i], (uint8_t)rslot[i]);
#pragma unroll
            for (int j = 0; j < EM; ++j) if (j < e) pv.set_coef(i, rrow[j], (uint8_t)I[i][j]);
        }
    }
    if (a.want_w) {
        for (int slot = 0; slot < k; ++slot) {
            const uint32_t r = rws[slot];
#pragma unroll
            for (int i = 0; i < EM; ++i) {
                if (i >= e) continue;
                uint32_t v = 0;
#pragma unroll
                for (int j = 0; j < EM; ++j) {
                    if (j >= e) continue;
                    if (r >= (uint32_t)k) { if (rslot[j] == (uint32_t)slot) v = I[i][j]; }
                    else v ^= gmul(I[i][j], a.G[rrow[j] * k + r]);
                }
                pv.set_w(i, slot, (uint8_t)v);
            }
        }
    }
    // Recovery slot i takes missing row E_i (reference generate_bitmatrix, :786).
#pragma unroll
    for (int i = 0; i < EM; ++i) if (i < e) rws[rslot[i]] = (uint8_t)er[i];
}

// ------------------------------------------------------- wide decode, phase B
// Large-m decode, second half: D_{E_i} = sum_r B(coef[i][r]) V_r, where V (m rows per
// stripe, written by the windowed phase-A kernel lh_jit_elim_win) already holds
// R_r + sum_{x present} B(G[r][x]) D_x.  One workgroup per (stripe, 256-byte column
// chunk); wave g owns outputs [8g, 8g + 8).  Coefficients are uniform per workgroup, so
// every coefficient bit is a scalar branch: only set bits cost XORs (8 per set bit and
// output).  V_r is expanded once per row into its B(2^t) ladder.
__global__ void __launch_bounds__(512) lh_apply_wide_kernel(lh::WideArgs a) {
    constexpr int W = 4, RO = 8;
    const int g = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int cps = a.sub / (64 * W);
    const long long s = blockIdx.x / cps;
    if (s >= a.stripes) return;
    const int p = (int)(blockIdx.x % cps) * 64 * W + lane * W;
    const lh::PlanView pv(a.plan + s * a.plan_stride, a.k, a.m, a.e_max);
    const int e = pv.e();
    const int i0 = g * RO;
    if (i0 >= e) return;
    const uint8_t *coef = pv.coef_ptr();
    const uint8_t *v = a.ws + s * a.ws_stride + p;
    uint32_t acc[RO][8];
#pragma unroll
    for (int i = 0; i < RO; ++i)
#pragma unroll
        for (int y = 0; y < 8; ++y) acc[i][y] = 0;
    for (int r = 0; r < a.m; ++r) {
        // Skip rows no output of this wave uses (absent recovery rows).
        uint32_t any = 0;
#pragma unroll
        for (int i = 0; i < RO; ++i) any |= (i0 + i < e) ? coef[(i0 + i) * a.m + r] : 0u;
        any = __builtin_amdgcn_readfirstlane(any);
        if (!any) continue;
        uint32_t lad[8][8];
#pragma unroll
        for (int b = 0; b < 8; ++b) __builtin_memcpy(&lad[0][b], v + (long long)r * a.bytes + b * a.sub, 4);
#pragma unroll
        for (int t = 1; t < 8; ++t) {
#pragma unroll
            for (int y = 0; y < 7; ++y) lad[t][y] = lad[t - 1][y + 1];
            lad[t][7] = lad[t - 1][0] ^ lad[t - 1][1] ^ lad[t - 1][2] ^ lad[t - 1][7];
        }
#pragma unroll
        for (int i = 0; i < RO; ++i) {
            const uint32_t c = __builtin_amdgcn_readfirstlane((i0 + i < e) ? coef[(i0 + i) * a.m + r] : 0u);
#pragma unroll
            for (int t = 0; t < 8; ++t)
                if ((c >> t) & 1u)
#pragma unroll
                    for (int y = 0; y < 8; ++y) acc[i][y] ^= lad[t][y];
        }
    }
#pragma unroll
    for (int i = 0; i < RO; ++i) {
        if (i0 + i < e) {
            uint8_t *dst = a.blocks + s * a.blocks_stride + (long long)pv.out_slot(i0 + i) * a.bytes + p;
#pragma unroll
            for (int y = 0; y < 8; ++y) __builtin_memcpy(dst + y * a.sub, &acc[i][y], 4);
        }
    }
}

// ------------------------------------------------------------------ host launchers
namespace lh {

hipError_t launch_apply_generic(const ApplyArgs &a, int W, hipStream_t st) {
    const long long lanes = (long long)a.stripes * a.nch;
    dim3 grid((unsigned)((lanes + 255) / 256), (unsigned)((a.n_out + kGenericTileOut - 1) / kGenericTileOut));
    switch (W) {
        case 1: hipLaunchKernelGGL(lh_apply_generic_kernel<1>, grid, dim3(256), 0, st, a); break;
        case 2: hipLaunchKernelGGL(lh_apply_generic_kernel<2>, grid, dim3(256), 0, st, a); break;
        case 4: hipLaunchKernelGGL(lh_apply_generic_kernel<4>, grid, dim3(256), 0, st, a); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_xor_reduce(const XorArgs &a, hipStream_t st) {
    const long long lanes = (long long)a.stripes * a.nch;
    hipLaunchKernelGGL(lh_xor_reduce_kernel, dim3((unsigned)((lanes + 255) / 256)), dim3(256), 0, st, a);
    return hipGetLastError();
}

hipError_t launch_scatter(const ScatterArgs &a, hipStream_t st) {
    const long long lanes = (long long)a.stripes * a.e_max * ((a.bytes + 15) / 16);
    hipLaunchKernelGGL(lh_scatter_kernel, dim3((unsigned)((lanes + 255) / 256)), dim3(256), 0, st, a);
    return hipGetLastError();
}

hipError_t launch_apply_wide(const WideArgs &a, hipStream_t st) {
    const long long blocks = (long long)a.stripes * (a.sub / 256);
    const int waves = (a.e_max + 7) / 8;
    hipLaunchKernelGGL(lh_apply_wide_kernel, dim3((unsigned)blocks), dim3(64 * waves), 0, st, a);
    return hipGetLastError();
}

hipError_t launch_plan(const PlanArgs &a, hipStream_t st) {
    if (a.k > 1 && a.m > 1 && a.e_max <= 8) {
        const unsigned blocks = (unsigned)((a.stripes + 255) / 256);
        if (a.e_max <= 4) hipLaunchKernelGGL(lh_plan_small_kernel<4>, dim3(blocks), dim3(256), 0, st, a);
        else hipLaunchKernelGGL(lh_plan_small_kernel<8>, dim3(blocks), dim3(256), 0, st, a);
        return hipGetLastError();
    }
    const size_t lds = (size_t)a.e_max * 2 * a.e_max;
    hipLaunchKernelGGL(lh_plan_kernel, dim3((unsigned)a.stripes), dim3(64), lds, st, a);
    return hipGetLastError();
}

}  // namespace lh
