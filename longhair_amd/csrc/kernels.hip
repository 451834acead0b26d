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
//   lh_inverse_gt_kernel    large-m decode phase B (after the windowed phase A left V_r in
//                           the recovery slots): D_E = A^-1 V by a computed jump into 256
//                           fixed multiply-by-c bodies (back-substitution :1083-1247, same
//                           solution).
//   lh_writeback_kernel     pinned-host decode pipeline: recovered blocks straight into
//                           the caller's pinned buffer.
//   lh_ptr_copy_kernel      pointer-table batches on the paths without a pointer form:
//                           scattered blocks into a contiguous chunk and back.
//
// Lanes own W-byte columns of a stripe's sub-blocks: a lane loads the same byte range of
// all 8 sub-blocks of a block and produces the same range of all 8 output sub-blocks, so
// every output byte depends only on input bytes at the same sub-block offset.
#include <hip/hip_runtime.h>

#include <type_traits>
#include <stdint.h>

#include <cstdlib>
#include <map>
#include <mutex>

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
// The next input column's words are loaded before the current one is combined (one column
// in flight per lane while the 64 masked XORs per output of this one issue).  When every lane
// of a wave codes the same stripe (the encode's coefficients are the same for all stripes;
// the decode's are per stripe, uniform when a stripe spans whole waves) the coefficient is a
// scalar load and its bit masks are scalar work.
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
    const bool uni = a.coef_stride == 0 ||
                     __all(s == (((long long)__builtin_amdgcn_readfirstlane((int)(s >> 32)) << 32) |
                                 (unsigned)__builtin_amdgcn_readfirstlane((int)s)));

    Word<W> acc[TO][8];
#pragma unroll
    for (int i = 0; i < TO; ++i)
#pragma unroll
        for (int y = 0; y < 8; ++y) wzero(acc[i][y]);

    auto run = [&](auto uniform) {
        constexpr bool U = decltype(uniform)::value;
        Word<W> cur[8];
#pragma unroll
        for (int b = 0; b < 8; ++b) cur[b] = wload<W>(in + b * a.sub);
        for (int j = 0; j < a.n_in; ++j) {
            Word<W> nxt[8];
            const int jn = j + 1 < a.n_in ? j + 1 : j;  // (the last column reloads itself)
#pragma unroll
            for (int b = 0; b < 8; ++b) nxt[b] = wload<W>(in + (long long)jn * a.bytes + b * a.sub);
            Word<W> lad[8][8];  // lad[t] = B(2^t) * d
#pragma unroll
            for (int b = 0; b < 8; ++b) lad[0][b] = cur[b];
#pragma unroll
            for (int q = 1; q < 8; ++q) mul2<W>(lad[q - 1], lad[q]);
#pragma unroll
            for (int i = 0; i < TO; ++i) {
                if (i < ni) {
                    uint32_t e = coef[i * a.n_in + j];
                    if (U) e = (uint32_t)__builtin_amdgcn_readfirstlane((int)e);
#pragma unroll
                    for (int q = 0; q < 8; ++q) {
                        const uint32_t mask = 0u - ((e >> q) & 1u);
#pragma unroll
                        for (int y = 0; y < 8; ++y) wxor_masked(acc[i][y], lad[q][y], mask);
                    }
                }
            }
#pragma unroll
            for (int b = 0; b < 8; ++b) cur[b] = nxt[b];
        }
    };
    if (uni) run(std::true_type{});
    else run(std::false_type{});
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
// One workgroup per stripe (1 or 4 waves), every step lane-parallel.
//  * Classification (reference sort_blocks, cauchy_256.cpp:538-570): a row -> slot map in
//    LDS; recovery slots (array order) and missing originals (ascending) are compacted
//    with wave ballots and prefix popcounts.
//  * e x e GF(256) inverse by Gauss-Jordan without row swaps: lane i owns rows i and
//    i + 64 of [A | I], stored column-major in LDS so a wave's same-column accesses hit
//    consecutive bytes; the pivot of column c is the lowest unused row with a non-zero
//    entry (one ballot).  [A | I] reduces to [P | M] with row p_c of the permutation P
//    holding the 1 of column c, so A^-1[c][:] = M[p_c][:].
//  * Closed form instead, whenever the generator is a Cauchy matrix (every m >= 7, so every
//    e > 8 this kernel sees): A[i][j] = x_j / (x_j + y_i) with x_j = X'[E_j], y_i =
//    Y'[r_i] (field.cpp cauchy_points), and over GF(2^8)
//        A^-1[j][i] = P_j Q_i / ((x_j + y_i) C_j D_i x_j),
//    P_j = prod_k (x_j + y_k), Q_i = prod_k (x_k + y_i), C_j = prod_{k!=j} (x_j + x_k),
//    D_i = prod_{k!=i} (y_i + y_k): O(e^2) table lookups in the log domain instead of the
//    O(e^3) elimination (the inverse is unique, so the bytes are the same).
// LDS: GF tables, maps, and 2 e_max x RC bytes (RC = 64 or 128 rows).
__global__ void __launch_bounds__(256) lh_plan_kernel(lh::PlanArgs a) {
    const int s = blockIdx.x;
    const int tid = threadIdx.x, nth = blockDim.x;
    const int lane = tid & 63, wv = tid >> 6, NW = nth >> 6;
    const int k = a.k, m = a.m, e_max = a.e_max;
    const int RC = e_max > 64 ? 128 : 64;  // row capacity of the augmented matrix
    __shared__ uint8_t gexp[512];
    __shared__ int16_t glog[256];
    __shared__ uint8_t rows[256];
    __shared__ uint8_t slot_of[256];  // row -> slot, 0xFF absent
    __shared__ uint8_t rcv_slot[256], rcv_row[256], erasure[256];
    __shared__ uint8_t piv_row[128];  // p_c per column
    __shared__ int16_t plog[256];     // normalised pivot row in log form, -1 = zero
    extern __shared__ uint8_t aug[];  // element (i, j) at aug[j * RC + i], j < 2 e_max

    for (int i = tid; i < 256; i += nth) {
        gexp[i] = a.gf_exp[i];
        gexp[i + 256] = a.gf_exp[i + 256];
        glog[i] = a.gf_log[i];
        slot_of[i] = 0xFF;
    }
    uint8_t *rws = a.rows + (long long)s * k;
    for (int i = tid; i < k; i += nth) rows[i] = rws[i];
    __syncthreads();

    uint8_t *rec = a.plan + (long long)s * a.plan_stride;
    lh::PlanView pv(rec, k, m, e_max);

    // Row -> slot map.  A row outside the code or a repeated row invalidates the stripe
    // (undefined behaviour in the reference).
    bool bad = false;
    for (int i = lane; i < k; i += 64) {
        const int r = rows[i];
        if (r >= k + m) bad = true;
        else slot_of[r] = (uint8_t)i;
    }
    __syncthreads();
    for (int i = lane; i < k; i += 64) {
        const int r = rows[i];
        if (r < k + m && slot_of[r] != i) bad = true;
    }
    // m == 1 follows cauchy_decode_m1 (:487-535), which accepts any rows: every row >= k is
    // a recovery block (the last one in array order is the output), repeats are harmless.
    const int status = (__ballot(bad) && m > 1) ? -1 : 0;
    const unsigned long long below = (1ull << lane) - 1;
    int n_rcv = 0, n_miss = 0;
    for (int i0 = 0; i0 < k; i0 += 64) {
        const int i = i0 + lane;
        const bool isrcv = i < k && rows[i] >= k;
        const bool miss = i < k && slot_of[i] == 0xFF;
        const unsigned long long br = __ballot(isrcv), bm = __ballot(miss);
        if (isrcv) {
            const int q = n_rcv + __builtin_popcountll(br & below);
            rcv_slot[q] = (uint8_t)i;
            rcv_row[q] = (uint8_t)(rows[i] - k);
        }
        if (miss) erasure[n_miss + __builtin_popcountll(bm & below)] = (uint8_t)i;
        n_rcv += __builtin_popcountll(br);
        n_miss += __builtin_popcountll(bm);
    }
    __syncthreads();
    const int e = (status != 0 || k <= 1) ? 0 : (m == 1 ? 1 : n_rcv);
    if (tid == 0) {
        rec[0] = (uint8_t)e;
        rec[1] = (uint8_t)(int8_t)status;
        if (a.status) a.status[s] = (int8_t)status;
    }
    if (status != 0) return;
    if (k <= 1) {  // cauchy_256.cpp:1252-1256
        if (tid == 0 && k == 1) rws[0] = 0;
        return;
    }
    if (m == 1) {
        // cauchy_decode_m1 (:487-535): the last recovery slot (or slot 0 when none is
        // present) becomes the XOR of all k blocks and takes the first missing row.
        if (tid == 0) {
            const int out = n_rcv ? rcv_slot[n_rcv - 1] : 0;
            pv.set_out_slot(0, (uint8_t)out);
            if (n_miss) rws[out] = erasure[0];
        }
        return;
    }
    if (e == 0) return;

    if (a.points) {
        __shared__ uint8_t cx[128], cy[128];  // x_j, y_i
        __shared__ int16_t al[128], be[128];  // log(P_j / (C_j x_j)), log(Q_i / D_i), in [0, 255)
        for (int t = tid; t < e; t += nth) {
            cx[t] = a.points[erasure[t]];
            cy[t] = a.points[k + rcv_row[t]];
        }
        __syncthreads();
        for (int t = tid; t < e; t += nth) {
            const int x = cx[t], y = cy[t];
            int pc = -glog[x], qd = 0;
            for (int u = 0; u < e; ++u) {
                const int xu = cx[u], yu = cy[u];
                pc += glog[x ^ yu];
                qd += glog[xu ^ y];
                if (u != t) {
                    pc -= glog[x ^ xu];
                    qd -= glog[y ^ yu];
                }
            }
            al[t] = (int16_t)((pc % 255 + 255) % 255);
            be[t] = (int16_t)((qd % 255 + 255) % 255);
        }
        __syncthreads();
        // A^-1[i][j] lands where the elimination would leave it: aug[e + j][p_i], p_i = i.
        for (int q = tid; q < e * e; q += nth) {
            const int i = q / e, j = q - i * e;
            int v = al[i] + be[j] - glog[cx[i] ^ cy[j]];
            v += v < 0 ? 255 : 0;
            aug[(e + j) * RC + i] = gexp[v];
        }
        for (int i = tid; i < e; i += nth) piv_row[i] = (uint8_t)i;
        __syncthreads();
    } else {
    // [A | I]: A[i][j] = G[r_i][E_j] (r_i = recovery row of the i-th recovery slot,
    // E_j = j-th missing original).
    const int w2 = 2 * e;
    for (int h = 0; h < RC / 64; ++h) {
        const int i = lane + 64 * h;
        if (i >= e) continue;
        const uint8_t *grow = a.G + rcv_row[i] * k;
        for (int j0 = 8 * wv; j0 < e; j0 += 8 * NW) {  // 8 independent gathers in flight, no branches
            uint8_t v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = grow[erasure[min(j0 + u, e - 1)]];
#pragma unroll
            for (int u = 0; u < 8; ++u) aug[min(j0 + u, e - 1) * RC + i] = v[u];  // clamped: same value
        }
        for (int j = wv; j < e; j += NW) aug[(e + j) * RC + i] = (uint8_t)(j == i);
    }
    __syncthreads();
    bool used0 = false, used1 = false;  // rows lane and lane + 64 are pivots already
    const int r1 = lane + 64;
    for (int c = 0; c < e; ++c) {
        const bool c0 = lane < e && !used0 && aug[c * RC + lane] != 0;
        const bool c1 = RC > 64 && r1 < e && !used1 && aug[c * RC + r1] != 0;
        const unsigned long long b0 = __ballot(c0), b1 = __ballot(c1);
        if (!b0 && !b1) {  // singular: impossible for distinct valid rows (Cauchy MDS)
            if (tid == 0) { rec[0] = 0; rec[1] = 0xFF; if (a.status) a.status[s] = -1; }
            return;
        }
        const int p = b0 ? __builtin_ctzll(b0) : 64 + __builtin_ctzll(b1);
        if (p == lane) used0 = true;
        if (p == r1) used1 = true;
        const int linv = 255 - glog[aug[c * RC + p]];
        // Factors of this thread's rows, read before any wave touches column c.
        const uint32_t f0 = (lane < e && lane != p) ? aug[c * RC + lane] : 0u;
        const uint32_t f1 = (RC > 64 && r1 < e && r1 != p) ? aug[c * RC + r1] : 0u;
        __syncthreads();
        // Normalise the pivot row (its columns < c are zero: earlier pivots cleared them).
        for (int j = c + tid; j < w2; j += nth) {
            const uint32_t v = aug[j * RC + p];
            const uint32_t nv = v ? gexp[glog[v] + linv] : 0u;
            aug[j * RC + p] = (uint8_t)nv;
            plog[j] = nv ? glog[nv] : (int16_t)-1;
        }
        if (tid == 0) piv_row[c] = (uint8_t)p;
        __syncthreads();
        // Clear column c from every other row; the waves split the columns.
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int i = lane + 64 * h;
            const uint32_t f = h ? f1 : f0;
            if (!f) continue;
            const int lf = glog[f];
            // 8 independent updates per step and no branches, so the LDS latencies overlap
            // (indices past the row are clamped to its last column: same value rewritten).
            for (int j0 = c + 8 * wv; j0 < w2; j0 += 8 * NW) {
                int pl[8];
                uint32_t av[8], gv[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    const int j = min(j0 + u, w2 - 1);
                    pl[u] = plog[j];
                    av[u] = aug[j * RC + i];
                }
#pragma unroll
                for (int u = 0; u < 8; ++u) gv[u] = gexp[lf + max(pl[u], 0)];
#pragma unroll
                for (int u = 0; u < 8; ++u)
                    aug[min(j0 + u, w2 - 1) * RC + i] = (uint8_t)(av[u] ^ (pl[u] >= 0 ? gv[u] : 0u));
            }
        }
        __syncthreads();
    }
    }
    // A^-1[c][j] = aug[e + j][p_c].  Emit: out slots, src/rec slot maps, coef (e x m over
    // recovery rows) and W (e x k over slots).
    for (int i = tid; i < e; i += nth) pv.set_out_slot(i, rcv_slot[i]);
    for (int x = tid; x < k; x += nth) pv.set_src_slot(x, slot_of[x]);
    for (int r = tid; r < m; r += nth) pv.set_rec_slot(r, slot_of[k + r]);
    for (int q = tid; q < e * m; q += nth) pv.set_coef(q / m, q % m, 0);
    __syncthreads();
    for (int q = tid; q < e * e; q += nth) {
        const int i = q / e, j = q % e;
        pv.set_coef(i, rcv_row[j], aug[(e + j) * RC + piv_row[i]]);
    }
    for (int q = tid; a.want_w && q < e * k; q += nth) {
        const int i = q / k, slot = q % k;
        const int r = rows[slot];
        uint32_t v = 0;
        if (r >= k) {
            for (int j = 0; j < e; ++j) if (rcv_slot[j] == slot) v = aug[(e + j) * RC + piv_row[i]];
        } else {
            for (int j = 0; j < e; ++j) {
                const uint32_t x = aug[(e + j) * RC + piv_row[i]], y = a.G[rcv_row[j] * k + r];
                if (x && y) v ^= gexp[glog[x] + glog[y]];
            }
        }
        pv.set_w(i, slot, (uint8_t)v);
    }
    // Recovery slot i takes erased row E_i (reference generate_bitmatrix, :786).
    for (int i = tid; i < e; i += nth) rws[rcv_slot[i]] = erasure[i];
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

// -------------------------------------------------------------------- framing
// One thread per 4 bytes of a block; the packet payload sits one byte after the row, so
// one side of every copy is unaligned (gfx950 serves unaligned dword accesses).
typedef uint32_t lh_u32_unaligned __attribute__((aligned(1)));
__global__ void __launch_bounds__(256) lh_frame_kernel(lh::FrameArgs a) {
    const int words = (a.bytes + 3) / 4;
    const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    const long long per_stripe = (long long)a.npk * words;
    const long long s = t / per_stripe;
    if (s >= a.stripes) return;
    const int rem = (int)(t - s * per_stripe);
    const int i = rem / words, w = rem - i * words;
    uint8_t *pk = a.packets + s * a.packet_stride + (long long)i * (a.bytes + 1);
    const uint8_t *src;
    uint8_t *dst;
    if (a.unframe) {
        src = pk + 1;
        dst = a.blocks + s * a.blocks_stride + (long long)i * a.bytes;
        if (w == 0) a.rows[s * a.k + i] = pk[0];
    } else {
        src = i < a.k ? a.data + s * a.data_stride + (long long)i * a.bytes
                      : a.rec + s * a.rec_stride + (long long)(i - a.k) * a.bytes;
        dst = pk + 1;
        if (w == 0) pk[0] = (uint8_t)i;
    }
    const int off = 4 * w, n = min(4, a.bytes - off);
    if (n == 4) {
        *(lh_u32_unaligned *)(dst + off) = *(const lh_u32_unaligned *)(src + off);
    } else {
        for (int q = 0; q < n; ++q) dst[off + q] = src[off + q];
    }
}

// ------------------------------------------------------------------ large-m decode, phase B
// After the windowed phase-A kernel (jit.cpp, split modules) has replaced every present
// recovery block R_r by V_r = R_r + sum_{x present} B(G[r][x]) D_x in place:
// D_{E_i} = sum_r B(coef[i][r]) V_r (the reference's back-substitution,
// cauchy_256.cpp:1083-1247; same unique solution).  One workgroup per (stripe, 256-byte
// chunk of every sub-block), ceil(e_max / 8) waves, at most 8 outputs per wave.  The chunk's
// V rows are staged in LDS by LDS-DMA in double-buffered 8-row tiles (2 KiB per row); per
// used row a wave builds the 16-entry XOR tables of V_r's sub-blocks 0..3 (tl) and 4..7 (th)
// in registers, and a multiply by c is, for every output sub-row y, one XOR3 of two table
// entries whose indices are the nibbles of c * 2^y: compile-time constants of 256 fixed-size
// bodies (8 v_bitop3_b32 + a return, 68 bytes; inv_jump.inc, tools/gen_inv_jump.py) that the
// wave enters with c wave-uniform.  Round 3 measured seven forms of this phase (DESIGN.md
// §5.3); two remain: the bodies once per code object (lh_inverse_gt_kernel, the default) and
// the same bodies inside the asm statement (its fallback, lh_inverse_dma_body).
#include "inv_jump.inc"

// The in-asm table: the 8 outputs of a wave keep their accumulators in pinned registers
// v[40 + 8i .. 40 + 8i + 7]; one asm statement per row builds the 8 jump targets from the
// packed coefficient bytes (masked to 8 bits in the asm), enters the table once per output
// with GPR indexing on (SRC0 and DST relative to index 8i) and returns through s[94:95].
__device__ __forceinline__ void lh_mul_jump_idx8(unsigned c0, unsigned c1, uint32_t (&a)[8][8],
                                                 const uint32_t (&tl)[16], const uint32_t (&th)[16]) {
    asm volatile(LH_INV_JUMPI8_ASM : LH_INV_JUMPI8_OUTS(a) : [c0] "s"(c0), [c1] "s"(c1), LH_INV_JUMPI_INS(tl, th)
                 : "s88", "s89", "s90", "s91", "s92", "s93", "s94", "s95", "s96", "s97", "scc");
}

// Common to both forms: the plan view, the used recovery rows, the LDS-DMA staging of the
// chunk's V rows (2 global_load_lds_dwordx4 per row, 16 B per lane: lane l moves bytes
// (l % 16) * 16 of sub-block 4 h + l / 16, so each instruction fills 1 KiB of the row's
// [sub-block][256 B] image in lane order) and the tile loop: the DMA of tile t + 1 is issued
// right after the barrier that publishes tile t and lands while tile t is computed (one
// counted wait + a raw barrier per tile, no __syncthreads, whose fence would drain it).
struct lh_pb_ctx {
    const lh::InverseArgs &a;
    int nw, g, lane, e, m, sub;
    lh::PlanView pv;
    uint32_t rslot;
    unsigned long long used;
    uint8_t *sbase;        // the stripe's first block (strided batches)
    uint8_t *const *ptab;  // pointer-table batches: the stripe's k slot pointers, else NULL
    int c0, nch;           // this workgroup's 2 KiB chunks: c0 .. c0 + nch - 1 of every block
    // pointer-table batches: lane r holds the block pointer of recovery row r (vp) and of
    // output r (op), fetched once, so a DMA or a store never waits for a pointer load
    unsigned long long vp, op;
    int dof0, dof1;
    __device__ __forceinline__ lh_pb_ctx(const lh::InverseArgs &a_, const uint8_t *pl, long long stripe, int c0_,
                                         int nch_)
        : a(a_), pv(pl, a_.k, a_.m, a_.e_max) {
        nw = (int)(blockDim.x >> 6);
        g = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
        lane = (int)(threadIdx.x & 63);
        e = pl[0];
        m = a.m;
        sub = a.bytes >> 3;
        rslot = lane < m ? (uint32_t)pv.rec_slot(lane) : 0xFFu;
        used = __ballot(rslot != 0xFFu);
        c0 = c0_;
        nch = nch_;
        ptab = a.ptrs ? a.ptrs + stripe * a.k : nullptr;
        sbase = ptab ? nullptr : a.blocks + stripe * a.stride;  // wave-uniform
        vp = op = 0;
        if (ptab) {
            if (rslot != 0xFFu) vp = (unsigned long long)ptab[rslot];
            if (lane < e) op = (unsigned long long)ptab[pv.out_slot(lane)];
        }
        dof0 = (lane >> 4) * sub + (lane & 15) * 16;
        dof1 = dof0 + 4 * sub;
    }
    // Lane r's pointer of a per-lane table, wave-uniform.
    __device__ __forceinline__ static uint8_t *lane_ptr(unsigned long long t, int r) {
        const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)t, r);
        const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(t >> 32), r);
        return (uint8_t *)(((unsigned long long)hi << 32) | lo);
    }
    // DMA of the tile starting at `rest` of chunk `ch` into `buf`: this wave moves tile
    // positions g, g + nw, ...
    __device__ __forceinline__ void issue(int ch, unsigned long long rest, uint32_t *buf) const {
        for (int q = 0; q < g && rest; ++q) rest &= rest - 1;
        for (int j = g; rest && j < 8; j += nw) {
            const int r = __builtin_ctzll(rest);
            const uint8_t *src = ptab ? lane_ptr(vp, r) + ch * 256
                                      : sbase + (long long)(uint32_t)__builtin_amdgcn_readlane((int)rslot, r) * a.bytes +
                                            ch * 256;
            uint8_t *dst = (uint8_t *)buf + j * 2048;
            __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void *)(src + dof0),
                                             (__attribute__((address_space(3))) void *)dst, 16, 0, 0);
            __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void *)(src + dof1),
                                             (__attribute__((address_space(3))) void *)(dst + 1024), 16, 0, 0);
            for (int q = 0; q < nw && rest; ++q) rest &= rest - 1;
        }
    }
    __device__ __forceinline__ static unsigned long long skip_tile(unsigned long long rest) {
        for (int j = 0; rest && j < 8; ++j) rest &= rest - 1;
        return rest;
    }
    // s_waitcnt vmcnt(0) (this wave's DMAs landed), then lgkmcnt(0) (its LDS reads done), then
    // the raw barrier (gfx9 encodings; expcnt / the other counter left at their maxima).
    __device__ __forceinline__ static void publish() {
        __builtin_amdgcn_s_waitcnt((7 << 4) | (15 << 8));
        __builtin_amdgcn_s_waitcnt(0xF | (7 << 4) | (3 << 14));
        __builtin_amdgcn_s_barrier();
    }
    // The tile loop over the workgroup's chunks: compute(rest, buf) multiplies the rows of the
    // tile starting at `rest`; done(ch) runs after the last tile of chunk ch (the outputs).
    // The pipeline runs across chunks: the DMA of a chunk's first tile is issued while the
    // previous chunk's last tile is computed.  Before done(ch) every wave has waited for its
    // DMAs of chunk ch and passed a barrier after them, so all of the chunk's V rows have been
    // read and its recovery slots may be overwritten; the DMA in flight reads the next chunk's
    // bytes, which no store of chunk ch touches.
    template <class F, class D>
    __device__ __forceinline__ void tiles(uint32_t *lvA, uint32_t *lvB, F &&compute, D &&done) const {
        int ch = c0;
        unsigned long long todo = used;
        issue(ch, todo, lvA);
        bool inA = true;
        while (true) {  // workgroup-uniform
            publish();  // tile in its buffer; every wave is done with the other one
            unsigned long long next = skip_tile(todo);
            int nch_ = ch;
            if (!next && ch + 1 < c0 + nch) {
                nch_ = ch + 1;
                next = used;
            }
            if (next) issue(nch_, next, inA ? lvB : lvA);
            compute(todo, inA ? lvA : lvB);
            if (nch_ != ch || !next) done(ch);
            if (!next) break;
            todo = next;
            ch = nch_;
            inA = !inA;
        }
    }
    // Row j of a tile: the 16-entry tables of V_r's sub-blocks 0..3 and 4..7.
    __device__ __forceinline__ void tables(const uint32_t *buf, int j, uint32_t (&tl)[16], uint32_t (&th)[16]) const {
        uint32_t v[8];
#pragma unroll
        for (int y = 0; y < 8; ++y) v[y] = buf[(j * 8 + y) * 64 + lane];
        tl[0] = th[0] = 0;
#pragma unroll
        for (int q = 1; q < 16; ++q) {
            const int low = __builtin_ctz(q), pre = q & (q - 1);
            tl[q] = pre ? (tl[pre] ^ v[low]) : v[low];
            th[q] = pre ? (th[pre] ^ v[4 + low]) : v[4 + low];
        }
    }
    __device__ __forceinline__ void store(int ch, int out, const uint32_t (&acc)[8]) const {
        uint8_t *dst = (ptab ? lane_ptr(op, out) : sbase + (long long)pv.out_slot(out) * a.bytes) + ch * 256 + lane * 4;
#pragma unroll
        for (int y = 0; y < 8; ++y) __builtin_nontemporal_store(acc[y], (uint32_t *)(dst + (long long)y * sub));
    }
};

// The workgroup's stripe and chunks: a.chunks_per_wg consecutive 2 KiB chunks of one stripe,
// the stripes taken in a.order (largest e first) when given.
struct lh_pb_span {
    long long stripe;
    int c0, nch;
    __device__ __forceinline__ explicit lh_pb_span(const lh::InverseArgs &a) {
        const int cps = a.bytes >> 11, cpw = a.chunks_per_wg > 0 ? a.chunks_per_wg : 1;
        const int wps = (cps + cpw - 1) / cpw;  // workgroups per stripe
        stripe = blockIdx.x / wps;
        if (a.order && stripe < a.stripes) stripe = a.order[stripe];
        c0 = (int)(blockIdx.x % wps) * cpw;
        nch = cps - c0 < cpw ? cps - c0 : cpw;
    }
};

// Fallback form: outputs g, g + nw, ... (at most 8) per wave, the in-asm table.
__device__ __forceinline__ void lh_inverse_dma_body(const lh::InverseArgs &a, uint32_t *__restrict__ lvA,
                                                    uint32_t *__restrict__ lvB) {
    const lh_pb_span sp(a);
    if (sp.stripe >= a.stripes) return;  // workgroup-uniform
    const uint8_t *pl = a.plan + sp.stripe * a.plan_stride;
    if (pl[0] == 0) return;  // workgroup-uniform
    const lh_pb_ctx C(a, pl, sp.stripe, sp.c0, sp.nch);
    const int nout = C.g < C.e ? (C.e - C.g + C.nw - 1) / C.nw : 0;
    uint32_t cpk0 = 0, cpk1 = 0;  // lane r: this wave's coefficients for recovery row r
    if (C.rslot != 0xFFu) {
        const uint8_t *cf = C.pv.coef_ptr();
#pragma unroll
        for (int i = 0; i < 8; ++i)
            if (i < nout) {
                const uint32_t c = (uint32_t)cf[(C.g + i * C.nw) * C.m + C.lane] << (8 * (i & 3));
                if (i < 4) cpk0 |= c;
                else cpk1 |= c;
            }
    }
    uint32_t acc[8][8];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int y = 0; y < 8; ++y) acc[i][y] = 0;
    C.tiles(lvA, lvB, [&](unsigned long long rest, const uint32_t *buf) {
        for (int j = 0; rest && j < 8; ++j, rest &= rest - 1) {
            if (nout == 0) continue;
            const int r = __builtin_ctzll(rest);
            uint32_t tl[16], th[16];
            C.tables(buf, j, tl, th);
            // unused outputs (i >= nout) have coefficient 0: body 0 leaves them unchanged
            lh_mul_jump_idx8((uint32_t)__builtin_amdgcn_readlane((int)cpk0, r),
                             (uint32_t)__builtin_amdgcn_readlane((int)cpk1, r), acc, tl, th);
        }
    }, [&](int ch) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            if (i < nout) C.store(ch, C.g + i * C.nw, acc[i]);
#pragma unroll
            for (int y = 0; y < 8; ++y) acc[i][y] = 0;
        }
    });
}

// ---- the default: the 256 bodies once per code object, in the never-launched kernel below
// under the hidden symbol lh_inv_gtab, every register they touch fixed
// (tools/gen_inv_jump.py render_global_table).  A wave holds, per output slot i, the absolute
// low address of the body for row r's coefficient in lane r of t[i] (computed once), so per
// (output, row) only v_readlane + s_set_gpr_idx_idx + s_swappc_b64 + the body's s_setpc_b64
// issue on the scalar unit (3 SALU, against 7 for the in-asm table).
//
// Register and mode state: each LH_INV_JUMPG<n>_ASM statement saves M0,
// turns GPR indexing on before the first call, moves the index between calls, and turns it
// off and restores M0 after the last return, in straight-line code; each body is 8 VALU and
// s_setpc_b64 s[94:95], which the s_swappc_b64 that entered it has just written and nothing
// in the body writes.  So every call returns to the statement, and control leaves the
// statement only through its end, with indexing off and M0 restored.  A wave with no
// outputs (nout == 0) never executes the statement.
__global__ void lh_inv_gtab_holder() { asm volatile(LH_INV_GTAB_TEXT); }

#ifndef LH_GT_CHECK
// Debug build (make -C longhair_amd/csrc LH_DEBUG=1): every jump target is checked to be a
// body of the table before the call, and GPR indexing off after it; a failed check skips
// the call and poisons the wave's outputs, so the parity tests fail loudly.
#define LH_GT_CHECK 0
#endif

template <int N>
__device__ __forceinline__ bool lh_mul_jump_g(uint32_t (&acc)[8][8], const uint32_t (&tl)[16],
                                              const uint32_t (&th)[16], const uint32_t (&t)[8], int r,
                                              uint32_t tlo, uint32_t hi) {
#if LH_GT_CHECK
#pragma unroll
    for (int i = 0; i < N; ++i) {
        const uint32_t d = (uint32_t)__builtin_amdgcn_readlane((int)t[i], r) - tlo;
        if (d >= 256u * 68u || d % 68u != 0u) return false;  // wave-uniform
    }
#else
    (void)tlo;
#endif
#define LH_GT_CASE(n)                                                                                       \
    if constexpr (N == n)                                                                                   \
        asm volatile(LH_INV_JUMPG##n##_ASM : LH_INV_JUMPG##n##_OUTS(acc) : LH_INV_JUMPG_INS(tl, th, t),      \
                     [r] "s"(r), [hi] "s"(hi) : "s92", "s93", "s94", "s95", "s97", "scc");
    LH_GT_CASE(1) LH_GT_CASE(2) LH_GT_CASE(3) LH_GT_CASE(4) LH_GT_CASE(5) LH_GT_CASE(6) LH_GT_CASE(7)
    LH_GT_CASE(8)
#undef LH_GT_CASE
#if LH_GT_CHECK
    // MODE.GPR_IDX_EN (bit 27 of HW_REG_MODE on gfx9): must be off again after the statement.
    if (__builtin_amdgcn_s_getreg(1 | (27 << 6) | (0 << 11)) != 0) return false;
#endif
    return true;
}

// Outputs: pack ? wave g recovers outputs 8g .. 8g + 7 (fewer waves build the row tables) :
// g, g + nw, ... as the fallback.  The row loop is instantiated per output count (1..8,
// wave-uniform) so no slot jumps for an unused output.
__device__ __forceinline__ void lh_inverse_gt_body(const lh::InverseArgs &a, uint32_t *__restrict__ lvA,
                                                   uint32_t *__restrict__ lvB, uint32_t tlo, uint32_t thi) {
    const lh_pb_span sp(a);
    if (sp.stripe >= a.stripes) return;  // workgroup-uniform
    const uint8_t *pl = a.plan + sp.stripe * a.plan_stride;
    if (pl[0] == 0) return;  // workgroup-uniform
    const lh_pb_ctx C(a, pl, sp.stripe, sp.c0, sp.nch);
    const bool pack = a.pack != 0;
    int nout = pack ? C.e - 8 * C.g : (C.g < C.e ? (C.e - C.g + C.nw - 1) / C.nw : 0);
    nout = nout < 0 ? 0 : (nout > 8 ? 8 : nout);
    auto out_of = [&](int i) { return pack ? 8 * C.g + i : C.g + i * C.nw; };
    uint32_t t[8];  // lane r: body address of output slot i for recovery row r
    {
        const uint8_t *cf = C.pv.coef_ptr();
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const uint32_t c = (C.rslot != 0xFFu && i < nout) ? cf[out_of(i) * C.m + C.lane] : 0u;
            t[i] = tlo + c * 68u;
        }
    }
    auto run = [&](auto no) {
        constexpr int N = decltype(no)::value;
        uint32_t acc[8][8];
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
            for (int y = 0; y < 8; ++y) acc[i][y] = 0;
        bool ok = true;
        C.tiles(lvA, lvB, [&](unsigned long long rest, const uint32_t *buf) {
            if constexpr (N > 0) {
                for (int j = 0; rest && j < 8; ++j, rest &= rest - 1) {
                    uint32_t tl[16], th[16];
                    C.tables(buf, j, tl, th);
                    if (ok) ok = lh_mul_jump_g<N>(acc, tl, th, t, __builtin_ctzll(rest), tlo, thi);
                }
            }
        }, [&](int ch) {
#pragma unroll
            for (int i = 0; i < N; ++i) {
                if (!ok)
#pragma unroll
                    for (int y = 0; y < 8; ++y) acc[i][y] = 0xDEADBEEFu;
                C.store(ch, out_of(i), acc[i]);
#pragma unroll
                for (int y = 0; y < 8; ++y) acc[i][y] = 0;
            }
        });
    };
    switch (nout) {  // wave-uniform
        case 0: run(std::integral_constant<int, 0>{}); break;
        case 1: run(std::integral_constant<int, 1>{}); break;
        case 2: run(std::integral_constant<int, 2>{}); break;
        case 3: run(std::integral_constant<int, 3>{}); break;
        case 4: run(std::integral_constant<int, 4>{}); break;
        case 5: run(std::integral_constant<int, 5>{}); break;
        case 6: run(std::integral_constant<int, 6>{}); break;
        case 7: run(std::integral_constant<int, 7>{}); break;
        default: run(std::integral_constant<int, 8>{}); break;
    }
}

// The table's address comes from a PC-relative relocation.  A table that would straddle a
// 4 GiB boundary (the body addresses' high word differs; never seen) or a.jump_fallback
// (tests) takes the in-asm table instead.
__global__ void __launch_bounds__(1024) lh_inverse_gt_kernel(lh::InverseArgs a) {
    __shared__ __attribute__((aligned(16))) uint32_t lvA[8 * 8 * 64];
    __shared__ __attribute__((aligned(16))) uint32_t lvB[8 * 8 * 64];
    uint32_t tlo, thi;
    asm volatile(
        "s_getpc_b64 s[92:93]\n"
        "s_add_u32 s92, s92, lh_inv_gtab@rel32@lo+4\n"
        "s_addc_u32 s93, s93, lh_inv_gtab@rel32@hi+12\n"
        "s_mov_b32 %0, s92\n"
        "s_mov_b32 %1, s93\n"
        : "=s"(tlo), "=s"(thi)
        :
        : "s92", "s93", "scc");
    if (a.jump_fallback || tlo > 0xFFFFFFFFu - 256u * 68u) {
        lh_inverse_dma_body(a, lvA, lvB);
        return;
    }
    lh_inverse_gt_body(a, lvA, lvB, tlo, thi);
}

// Phase B's launch order: a stripe's phase-B work grows with e^2 (e outputs, each a sum over
// e rows), so with random erasures (k200/m56: e uniform in [1, 56]) a few heavy stripes set
// the kernel's tail.  One workgroup counting-sorts the stripes by e, largest first, and
// lh_pb_span maps workgroup b to stripe order[b / wps].
__global__ void __launch_bounds__(1024) lh_order_kernel(const uint8_t *__restrict__ plan, long long plan_stride,
                                                        int stripes, int *__restrict__ order) {
    __shared__ int cnt[256];
    for (int i = threadIdx.x; i < 256; i += blockDim.x) cnt[i] = 0;
    __syncthreads();
    for (int s = threadIdx.x; s < stripes; s += blockDim.x) atomicAdd(&cnt[plan[(long long)s * plan_stride]], 1);
    __syncthreads();
    if (threadIdx.x == 0) {  // start of each e's run, descending e
        int run = 0;
        for (int e = 255; e >= 0; --e) {
            const int c = cnt[e];
            cnt[e] = run;
            run += c;
        }
    }
    __syncthreads();
    for (int s = threadIdx.x; s < stripes; s += blockDim.x)
        order[atomicAdd(&cnt[plan[(long long)s * plan_stride]], 1)] = s;
}

// ------------------------------------------------------------ generic apply, jump table
// lh_apply_jump_kernel (kernels.hpp JumpApplyArgs): every shape without a specialised module,
// and every shape while its module compiles in the background.  Per input column a lane
// builds the 16-entry XOR tables of its dword of sub-blocks 0..3 (tl) and 4..7 (th) -- the
// win_encode idea of cauchy_256.cpp:1414-1493 with the tables in registers -- and a multiply
// by a runtime coefficient c is a jump into body c of the phase-B table (lh_inv_gtab: one XOR3
// per output sub-row, the nibble indices of c * 2^y compile-time constants of the body), the
// body address of output i for column j held in lane j of t[i].  Column loads are unaligned
// dword loads (a sub-block starts 2-byte aligned at 1296-byte blocks); the next column is in
// flight while the current one is combined.
namespace {
typedef uint32_t lh_u32u __attribute__((aligned(1)));

struct lh_ja_lane {
    long long stripe;   // (clamped to a valid stripe for the loads of an inactive lane)
    int p;              // the lane's byte offset in every sub-block
    bool active;
};

// (an inactive lane -- past the last stripe, or past the chunk's sub-block bytes -- loads
// nothing: exec-masked, no memory request)
__device__ __forceinline__ void lh_ja_load(uint32_t (&d)[8], const uint8_t *col, int sub, bool active) {
#pragma unroll
    for (int b = 0; b < 8; ++b) d[b] = 0;
    if (active) {
#pragma unroll
        for (int b = 0; b < 8; ++b) d[b] = *(const lh_u32u *)(col + (long long)b * sub);
    }
}

// Input column j of the lane's stripe at its chunk offset, through the pointer table when
// the batch has one; the output slot / row `o` likewise.
// (PTR: a separate kernel instantiation, so the strided form keeps its register budget)
template <bool PTR>
__device__ __forceinline__ const uint8_t *lh_ja_col(const lh::JumpApplyArgs &a, const lh_ja_lane &l, int j) {
    if constexpr (PTR) return a.in_ptrs[l.stripe * a.in_n + j] + l.p;
    return a.in + l.stripe * a.in_stride + (long long)j * a.bytes + l.p;
}
template <bool PTR>
__device__ __forceinline__ uint8_t *lh_ja_out(const lh::JumpApplyArgs &a, const lh_ja_lane &l, int o) {
    if constexpr (PTR) return a.out_ptrs[l.stripe * a.out_n + o] + l.p;
    return a.out + l.stripe * a.out_stride + (long long)o * a.bytes + l.p;
}

__device__ __forceinline__ void lh_ja_tables(const uint32_t (&d)[8], uint32_t (&tl)[16], uint32_t (&th)[16]) {
    tl[0] = th[0] = 0;
#pragma unroll
    for (int q = 1; q < 16; ++q) {
        const int low = __builtin_ctz(q), pre = q & (q - 1);
        tl[q] = pre ? (tl[pre] ^ d[low]) : d[low];
        th[q] = pre ? (th[pre] ^ d[4 + low]) : d[4 + low];
    }
}

// One round: outputs i0 .. i0 + N - 1 of this wave over every input column.  GT: the table
// once per code object (lh_mul_jump_g); else the in-asm table (lh_mul_jump_idx8, a table
// straddling a 4 GiB boundary; coefficient 0 = body 0 leaves unused outputs unchanged).
template <int N, bool GT, bool PTR = false>
__device__ __forceinline__ void lh_ja_round(const lh::JumpApplyArgs &a, const lh_ja_lane &l, const uint8_t *coef,
                                            int i0, uint32_t (&acc)[8][8], uint32_t tlo, uint32_t thi) {
    const int lane = threadIdx.x & 63;
    for (int jq = 0; jq * 64 < a.n_in; ++jq) {  // 64 columns per block of body addresses
        const int jc = jq * 64 + lane;
        uint32_t t[8], cpk0 = 0, cpk1 = 0;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const uint32_t c = (i < N && jc < a.n_in) ? coef[(long long)(i0 + i) * a.n_in + jc] : 0u;
            t[i] = tlo + c * 68u;
            if (i < 4) cpk0 |= c << (8 * i);
            else cpk1 |= c << (8 * (i - 4));
        }
        const int nj = a.n_in - jq * 64 < 64 ? a.n_in - jq * 64 : 64;
        uint32_t cur[8];
        lh_ja_load(cur, lh_ja_col<PTR>(a, l, jq * 64), a.sub, l.active);
        for (int jl = 0; jl < nj; ++jl) {  // wave-uniform
            const int jn = jq * 64 + jl + 1 < a.n_in ? jq * 64 + jl + 1 : jq * 64 + jl;  // (the last reloads itself)
            uint32_t nxt[8];
            lh_ja_load(nxt, lh_ja_col<PTR>(a, l, jn), a.sub, l.active);
            uint32_t tl[16], th[16];
            lh_ja_tables(cur, tl, th);
            if constexpr (GT) {
                (void)lh_mul_jump_g<N>(acc, tl, th, t, jl, tlo, thi);
            } else {
                lh_mul_jump_idx8((uint32_t)__builtin_amdgcn_readlane((int)cpk0, jl),
                                 (uint32_t)__builtin_amdgcn_readlane((int)cpk1, jl), acc, tl, th);
            }
#pragma unroll
            for (int b = 0; b < 8; ++b) cur[b] = nxt[b];
        }
    }
}

template <bool GT, bool PTR>
__device__ __forceinline__ void lh_apply_jump_body(const lh::JumpApplyArgs &a, uint32_t tlo, uint32_t thi) {
    const int lane = threadIdx.x & 63;
    const int g = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)), ng = (int)(blockDim.x >> 6);
    lh_ja_lane l;
    int c;
    if (a.per_stripe) {
        l.stripe = blockIdx.x / a.wps;
        if (l.stripe >= a.stripes) return;  // workgroup-uniform
        if (a.order) l.stripe = a.order[l.stripe];
        c = (int)(blockIdx.x % a.wps) * 64 + lane;
        l.active = c < a.nch;
        c = l.active ? c : a.nch - 1;
    } else {
        const long long t = (long long)blockIdx.x * 64 + lane;
        l.stripe = t / a.nch;
        c = (int)(t - l.stripe * a.nch);
        l.active = l.stripe < a.stripes;
        if (!l.active) l.stripe = a.stripes - 1;
    }
    // The last chunk of a sub-block re-reads its final 4 bytes (overlapping its neighbour
    // with identical results) instead of running past the sub-block.
    l.p = c == a.nch - 1 ? a.sub - 4 : 4 * c;
    const uint8_t *pl = a.plan ? a.plan + l.stripe * a.plan_stride : nullptr;
    const int n_out = pl ? pl[0] : a.n_out;  // per_stripe: workgroup-uniform
    if (pl && n_out == 0) return;           // workgroup-uniform: nothing erased
    const uint8_t *coef = a.coef + l.stripe * a.coef_stride;
    const int rounds = (a.n_out + 8 * ng - 1) / (8 * ng);  // the same for every wave (barriers)
    for (int q = 0; q < rounds; ++q) {
        const int i0 = 8 * (q * ng + g);
        int nout = n_out - i0;
        nout = nout < 0 ? 0 : (nout > 8 ? 8 : nout);  // wave-uniform
        // In place (a single round): a wave past its stripe's e neither reads nor writes, and
        // an ended wave no longer counts at the workgroup barrier, so it leaves now and frees
        // its slot (random e: k200/m56 keeps ~half of each workgroup's waves).
        if (pl && nout == 0) return;
        uint32_t acc[8][8];
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
            for (int y = 0; y < 8; ++y) acc[i][y] = 0;
        switch (nout) {  // wave-uniform
            case 0: break;
            case 1: lh_ja_round<1, GT, PTR>(a, l, coef, i0, acc, tlo, thi); break;
            case 2: lh_ja_round<2, GT, PTR>(a, l, coef, i0, acc, tlo, thi); break;
            case 3: lh_ja_round<3, GT, PTR>(a, l, coef, i0, acc, tlo, thi); break;
            case 4: lh_ja_round<4, GT, PTR>(a, l, coef, i0, acc, tlo, thi); break;
            case 5: lh_ja_round<5, GT, PTR>(a, l, coef, i0, acc, tlo, thi); break;
            case 6: lh_ja_round<6, GT, PTR>(a, l, coef, i0, acc, tlo, thi); break;
            case 7: lh_ja_round<7, GT, PTR>(a, l, coef, i0, acc, tlo, thi); break;
            default: lh_ja_round<8, GT, PTR>(a, l, coef, i0, acc, tlo, thi); break;
        }
        // In place (decode): every wave of the workgroup has read every slot of this chunk
        // before any output overwrites one (the host runs a single round there).
        if (pl && ng > 1) __syncthreads();
        if (l.active) {
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                if (i < nout) {
                    uint8_t *dst = lh_ja_out<PTR>(a, l, pl ? (int)pl[16 + i0 + i] : i0 + i);
#pragma unroll
                    for (int y = 0; y < 8; ++y) *(lh_u32u *)(dst + (long long)y * a.sub) = acc[i][y];
                }
            }
        }
    }
}
}  // namespace

template <bool PTR>
__global__ void __launch_bounds__(1024) lh_apply_jump_kernel(lh::JumpApplyArgs a) {
    uint32_t tlo, thi;
    asm volatile(
        "s_getpc_b64 s[92:93]\n"
        "s_add_u32 s92, s92, lh_inv_gtab@rel32@lo+4\n"
        "s_addc_u32 s93, s93, lh_inv_gtab@rel32@hi+12\n"
        "s_mov_b32 %0, s92\n"
        "s_mov_b32 %1, s93\n"
        : "=s"(tlo), "=s"(thi)
        :
        : "s92", "s93", "scc");
    if (a.jump_fallback || tlo > 0xFFFFFFFFu - 256u * 68u) {  // the table straddles a 4 GiB boundary
        lh_apply_jump_body<false, PTR>(a, tlo, thi);              // (never seen), or the tests' switch
        return;
    }
    lh_apply_jump_body<true, PTR>(a, tlo, thi);
}

// ---- two-dword form (a.dw == 2): a lane owns 8 bytes of every sub-block and a jump enters
// lh_inv_gtab2, whose body c adds B(c) V to 16 accumulator words (tools/gen_inv_jump.py
// render_global_table2) -- half the jumps per byte, at twice the table registers (60) and 4
// outputs per wave.  ~150 VGPRs: at most 12 waves per workgroup (3 per SIMD).
__global__ void lh_inv_gtab2_holder() { asm volatile(LH_INV_GTAB2_TEXT); }

template <int N>
__device__ __forceinline__ bool lh_mul_jump_g2(uint32_t (&acc)[4][16], const uint32_t (&tl)[16][2],
                                               const uint32_t (&th)[16][2], const uint32_t (&t)[4], int r,
                                               uint32_t tlo, uint32_t hi) {
#if LH_GT_CHECK
#pragma unroll
    for (int i = 0; i < N; ++i) {
        const uint32_t d = (uint32_t)__builtin_amdgcn_readlane((int)t[i], r) - tlo;
        if (d >= 256u * 132u || d % 132u != 0u) return false;  // wave-uniform
    }
#else
    (void)tlo;
#endif
#define LH_GT2_CASE(n)                                                                                       \
    if constexpr (N == n)                                                                                    \
        asm volatile(LH_INV_JUMPG2_##n##_ASM : LH_INV_JUMPG2_##n##_OUTS(acc) : LH_INV_JUMPG2_INS(tl, th, t),  \
                     [r] "s"(r), [hi] "s"(hi) : "s92", "s93", "s94", "s95", "s97", "scc");
    LH_GT2_CASE(1) LH_GT2_CASE(2) LH_GT2_CASE(3) LH_GT2_CASE(4)
#undef LH_GT2_CASE
#if LH_GT_CHECK
    if (__builtin_amdgcn_s_getreg(1 | (27 << 6) | (0 << 11)) != 0) return false;
#endif
    return true;
}

namespace {
typedef unsigned long long lh_u64u __attribute__((aligned(1)));

__device__ __forceinline__ void lh_ja_load2(uint32_t (&d)[8][2], const uint8_t *col, int sub, bool active) {
#pragma unroll
    for (int b = 0; b < 8; ++b) d[b][0] = d[b][1] = 0;
    if (active) {
#pragma unroll
        for (int b = 0; b < 8; ++b) {
            const unsigned long long v = *(const lh_u64u *)(col + (long long)b * sub);
            d[b][0] = (uint32_t)v;
            d[b][1] = (uint32_t)(v >> 32);
        }
    }
}

__device__ __forceinline__ void lh_ja_tables2(const uint32_t (&d)[8][2], uint32_t (&tl)[16][2],
                                              uint32_t (&th)[16][2]) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        tl[0][h] = th[0][h] = 0;
#pragma unroll
        for (int q = 1; q < 16; ++q) {
            const int low = __builtin_ctz(q), pre = q & (q - 1);
            tl[q][h] = pre ? (tl[pre][h] ^ d[low][h]) : d[low][h];
            th[q][h] = pre ? (th[pre][h] ^ d[4 + low][h]) : d[4 + low][h];
        }
    }
}

template <int N, bool PTR>
__device__ __forceinline__ bool lh_ja_round2(const lh::JumpApplyArgs &a, const lh_ja_lane &l, const uint8_t *coef,
                                             int i0, uint32_t (&acc)[4][16], uint32_t tlo, uint32_t thi) {
    const int lane = threadIdx.x & 63;
    bool ok = true;
    for (int jq = 0; jq * 64 < a.n_in; ++jq) {
        const int jc = jq * 64 + lane;
        uint32_t t[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const uint32_t c = (i < N && jc < a.n_in) ? coef[(long long)(i0 + i) * a.n_in + jc] : 0u;
            t[i] = tlo + c * 132u;
        }
        const int nj = a.n_in - jq * 64 < 64 ? a.n_in - jq * 64 : 64;
        uint32_t cur[8][2];
        lh_ja_load2(cur, lh_ja_col<PTR>(a, l, jq * 64), a.sub, l.active);
        for (int jl = 0; jl < nj; ++jl) {  // wave-uniform
            const int jn = jq * 64 + jl + 1 < a.n_in ? jq * 64 + jl + 1 : jq * 64 + jl;
            uint32_t nxt[8][2];
            lh_ja_load2(nxt, lh_ja_col<PTR>(a, l, jn), a.sub, l.active);
            uint32_t tl[16][2], th[16][2];
            lh_ja_tables2(cur, tl, th);
            if (ok) ok = lh_mul_jump_g2<N>(acc, tl, th, t, jl, tlo, thi);
#pragma unroll
            for (int b = 0; b < 8; ++b) cur[b][0] = nxt[b][0], cur[b][1] = nxt[b][1];
        }
    }
    return ok;
}

// gt: the table's address is usable.  The host launches this kernel only after
// probe_jump_tables found lh_inv_gtab2 within one 4 GiB page; a failed check here (or in the
// debug build's target check) poisons the outputs, so the parity tests fail loudly.
template <bool PTR>
__device__ __forceinline__ void lh_apply_jump2_body(const lh::JumpApplyArgs &a, bool gt, uint32_t tlo,
                                                    uint32_t thi) {
    const int lane = threadIdx.x & 63;
    const int g = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)), ng = (int)(blockDim.x >> 6);
    lh_ja_lane l;
    int c;
    if (a.per_stripe) {
        l.stripe = blockIdx.x / a.wps;
        if (l.stripe >= a.stripes) return;  // workgroup-uniform
        if (a.order) l.stripe = a.order[l.stripe];
        c = (int)(blockIdx.x % a.wps) * 64 + lane;
        l.active = c < a.nch;
        c = l.active ? c : a.nch - 1;
    } else {
        const long long t = (long long)blockIdx.x * 64 + lane;
        l.stripe = t / a.nch;
        c = (int)(t - l.stripe * a.nch);
        l.active = l.stripe < a.stripes;
        if (!l.active) l.stripe = a.stripes - 1;
    }
    l.p = c == a.nch - 1 ? a.sub - 8 : 8 * c;  // (the last chunk overlaps its neighbour)
    const uint8_t *pl = a.plan ? a.plan + l.stripe * a.plan_stride : nullptr;
    const int n_out = pl ? pl[0] : a.n_out;
    if (pl && n_out == 0) return;  // workgroup-uniform
    const uint8_t *coef = a.coef + l.stripe * a.coef_stride;
    const int rounds = (a.n_out + 4 * ng - 1) / (4 * ng);
    for (int q = 0; q < rounds; ++q) {
        const int i0 = 4 * (q * ng + g);
        int nout = n_out - i0;
        nout = nout < 0 ? 0 : (nout > 4 ? 4 : nout);  // wave-uniform
        if (pl && nout == 0) return;  // (as lh_apply_jump_body)
        uint32_t acc[4][16];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int y = 0; y < 16; ++y) acc[i][y] = 0;
        bool ok = gt;
        if (gt) {
            switch (nout) {  // wave-uniform
                case 0: break;
                case 1: ok = lh_ja_round2<1, PTR>(a, l, coef, i0, acc, tlo, thi); break;
                case 2: ok = lh_ja_round2<2, PTR>(a, l, coef, i0, acc, tlo, thi); break;
                case 3: ok = lh_ja_round2<3, PTR>(a, l, coef, i0, acc, tlo, thi); break;
                default: ok = lh_ja_round2<4, PTR>(a, l, coef, i0, acc, tlo, thi); break;
            }
        }
        if (pl && ng > 1) __syncthreads();  // in place: every slot read before any is written
        if (l.active) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                if (i < nout) {
                    uint8_t *dst = lh_ja_out<PTR>(a, l, pl ? (int)pl[16 + i0 + i] : i0 + i);
#pragma unroll
                    for (int y = 0; y < 8; ++y) {
                        const unsigned long long v = ok ? ((unsigned long long)acc[i][2 * y + 1] << 32) | acc[i][2 * y]
                                                        : 0xDEADBEEFDEADBEEFull;
                        *(lh_u64u *)(dst + (long long)y * a.sub) = v;
                    }
                }
            }
        }
    }
}
}  // namespace

template <bool PTR>
__global__ void __launch_bounds__(768) lh_apply_jump2_kernel(lh::JumpApplyArgs a) {
    uint32_t tlo, thi;
    asm volatile(
        "s_getpc_b64 s[92:93]\n"
        "s_add_u32 s92, s92, lh_inv_gtab2@rel32@lo+4\n"
        "s_addc_u32 s93, s93, lh_inv_gtab2@rel32@hi+12\n"
        "s_mov_b32 %0, s92\n"
        "s_mov_b32 %1, s93\n"
        : "=s"(tlo), "=s"(thi)
        :
        : "s92", "s93", "scc");
    lh_apply_jump2_body<PTR>(a, tlo <= 0xFFFFFFFFu - 256u * 132u, tlo, thi);
}

// The low words of the two jump tables' addresses (out[0]: lh_inv_gtab, out[1]: lh_inv_gtab2),
// read once per device: a table whose bodies straddle a 4 GiB boundary is not entered.
__global__ void lh_jump_probe_kernel(uint32_t *out) {
    uint32_t t1, t2;
    asm volatile(
        "s_getpc_b64 s[92:93]\n"
        "s_add_u32 s92, s92, lh_inv_gtab@rel32@lo+4\n"
        "s_mov_b32 %0, s92\n"
        "s_getpc_b64 s[92:93]\n"
        "s_add_u32 s92, s92, lh_inv_gtab2@rel32@lo+4\n"
        "s_mov_b32 %1, s92\n"
        : "=s"(t1), "=s"(t2)
        :
        : "s92", "s93", "scc");
    if (threadIdx.x == 0) {
        out[0] = t1;
        out[1] = t2;
    }
}

// ---------------------------------------------------------- pointer-table gather / scatter
// One wave per (stripe, block): 16 B per lane when both addresses and the block size allow,
// else 8 B, else single bytes (the caller's blocks may sit at any alignment).  Wave-uniform
// choice: every lane of the wave copies the same block.
__global__ void __launch_bounds__(256) lh_ptr_copy_kernel(lh::PtrCopyArgs a) {
    const long long item = ((long long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int lane = threadIdx.x & 63;
    if (item >= (long long)a.stripes * a.ncopy) return;
    const long long s = item / a.ncopy;
    const int j = (int)(item - s * a.ncopy);
    const long long t = s * a.n + j;  // table entry
    if (a.scatter) {  // wave-uniform tests: the wave copies one block
        if (a.status && a.status[s] != 0) return;
        if (a.sel && a.m1) {
            int out = 0;
            for (int i = 0; i < a.n; ++i)
                if (a.sel[s * a.n + i] >= a.sel_min) out = i;
            if (j != out) return;
        } else if (a.sel && a.sel[t] < a.sel_min) {
            return;
        }
    }
    uint8_t *blk = a.ptrs[t];
    uint8_t *lin = a.chunk + s * a.stride + (long long)j * a.bytes;
    const uint8_t *src = a.scatter ? lin : blk;
    uint8_t *dst = a.scatter ? blk : lin;
    const uintptr_t al = (uintptr_t)src | (uintptr_t)dst | (uintptr_t)a.bytes;
    if ((al & 15) == 0) {
        for (int o = lane * 16; o < a.bytes; o += 64 * 16) {
            uint4 v;
            __builtin_memcpy(&v, src + o, 16);
            __builtin_memcpy(dst + o, &v, 16);
        }
    } else if ((al & 7) == 0) {
        for (int o = lane * 8; o < a.bytes; o += 64 * 8) {
            uint2 v;
            __builtin_memcpy(&v, src + o, 8);
            __builtin_memcpy(dst + o, &v, 8);
        }
    } else {
        for (int o = lane; o < a.bytes; o += 64) dst[o] = src[o];
    }
}

// ------------------------------------------------------------------ pinned-host write-back
// One workgroup per stripe: the slots whose row was a recovery row before the decode are
// the slots decode may have written (its outputs; an invalid stripe is untouched, so the
// copy is the host's own bytes).  16 B per lane when the block size allows, else 8 B
// (bytes % 8 == 0 for m > 1).  Vector stores over PCIe into the mapped host buffer.
// Grid: x = stripe, y = segment of the block (large blocks are split over gridDim.y
// workgroups, so a chunk of a few large stripes -- the pipeline's last, k200/m56: 2 stripes --
// still has enough workgroups writing over the link: one per stripe took 0.31 ms for 7 MB).
__global__ void __launch_bounds__(256) lh_writeback_kernel(lh::WritebackArgs a) {
    const long long s = blockIdx.x;
    if (s >= a.stripes) return;
    const uint8_t *rows = a.rows_orig + s * a.k;
    const uint8_t *src = a.blocks + s * a.stride;
    uint8_t *dst = a.host + s * a.host_stride;
    const bool wide = ((a.bytes | a.host_stride | (long long)(uintptr_t)a.host) & 15) == 0;
    const int unit = wide ? 16 : 8, n = a.bytes / unit;  // lanes' units per block
    const int per = (n + (int)gridDim.y - 1) / (int)gridDim.y;
    const int q0 = (int)blockIdx.y * per, q1 = q0 + per < n ? q0 + per : n;
    for (int j = 0; j < a.k; ++j) {
        if (rows[j] < a.k) continue;  // workgroup-uniform
        const long long off = (long long)j * a.bytes;
        if (wide) {
            for (int q = q0 + (int)threadIdx.x; q < q1; q += blockDim.x)
                ((uint4 *)(dst + off))[q] = ((const uint4 *)(src + off))[q];
        } else {
            for (int q = q0 + (int)threadIdx.x; q < q1; q += blockDim.x)
                ((uint2 *)(dst + off))[q] = ((const uint2 *)(src + off))[q];
        }
    }
}

// ------------------------------------------------------------------ host launchers
namespace lh {

// Writes `order` (the stripes by their plan's e, largest first: lh_order_kernel) when there is
// a scratch, more than one stripe and more than one wave of outputs (e_max > 8: below that a
// stripe's work varies too little to pay for the sort); false: launch in stripe order.
#ifndef LH_PB_ORDER
#define LH_PB_ORDER 1  // (0: an A/B build of the launch order, make HIP_EXTRA=-DLH_PB_ORDER=0)
#endif
static bool order_stripes(int *order, const uint8_t *plan, long long plan_stride, int stripes, int e_max,
                          hipStream_t st) {
    if (!LH_PB_ORDER || !order || !plan || stripes < 2 || e_max <= 8) return false;
    hipLaunchKernelGGL(lh_order_kernel, dim3(1), dim3(1024), 0, st, plan, plan_stride, stripes, order);
    note_launch("lh_order_kernel");
    return true;
}

hipError_t launch_apply_generic(const ApplyArgs &a, int W, hipStream_t st) {
    const long long lanes = (long long)a.stripes * a.nch;
    dim3 grid((unsigned)((lanes + 255) / 256), (unsigned)((a.n_out + kGenericTileOut - 1) / kGenericTileOut));
    switch (W) {
        case 1: hipLaunchKernelGGL(lh_apply_generic_kernel<1>, grid, dim3(256), 0, st, a); break;
        case 2: hipLaunchKernelGGL(lh_apply_generic_kernel<2>, grid, dim3(256), 0, st, a); break;
        case 4: hipLaunchKernelGGL(lh_apply_generic_kernel<4>, grid, dim3(256), 0, st, a); break;
        default: return hipErrorInvalidValue;
    }
    note_launch("lh_apply_generic_kernel");
    return hipGetLastError();
}

hipError_t launch_apply_jump(const JumpApplyArgs &a, hipStream_t st) {
    // sub >= 4 (dword lanes); at most 16 waves of 8 outputs per workgroup; in place a single
    // round (e_max <= 128 always holds: e_max = min(k, m) and k + m <= 256).
    if (a.sub < 4 || a.n_out < 1 || a.n_in < 1 || a.nch < 1) return hipErrorInvalidValue;
    if (a.dw == 2) {  // 4 outputs per wave, at most 12 waves, the rounds balanced over them
        const int groups = (a.n_out + 3) / 4, rounds = (groups + 11) / 12, ng = (groups + rounds - 1) / rounds;
        if (a.sub < 8 || (a.plan && rounds > 1)) return hipErrorInvalidValue;
        const long long wgs = a.per_stripe ? (long long)a.stripes * a.wps : ((long long)a.stripes * a.nch + 63) / 64;
        if (wgs <= 0) return hipSuccess;
        if (wgs > 0x7FFFFFFF) return hipErrorInvalidValue;
        JumpApplyArgs g = a;
        if (!order_stripes(g.order, a.plan, a.plan_stride, a.per_stripe ? a.stripes : 0, a.n_out, st)) g.order = nullptr;
        if (a.in_ptrs)
            hipLaunchKernelGGL(lh_apply_jump2_kernel<true>, dim3((unsigned)wgs), dim3(64u * (unsigned)ng), 0, st, g);
        else
            hipLaunchKernelGGL(lh_apply_jump2_kernel<false>, dim3((unsigned)wgs), dim3(64u * (unsigned)ng), 0, st, g);
        note_launch(a.in_ptrs ? "lh_apply_jump2_kernel(pointer table)" : "lh_apply_jump2_kernel");
        return hipGetLastError();
    }
    if (a.dw != 1) return hipErrorInvalidValue;
    // Flat (encode) launches: a power-of-two number of waves per workgroup, further rounds for
    // the remaining outputs, so whole workgroups fill a CU's 16 wave slots (124 VGPRs: 4 per
    // SIMD); 7 waves left 2 slots idle.  k200/m56 generic encode 1.20-1.23 -> 1.10-1.11 ms
    // (profiles/r5v_generic_pow2.txt).  In place: one round, every output's wave present.
    int ng = (a.n_out + 7) / 8 < 16 ? (a.n_out + 7) / 8 : 16;
    if (!a.plan)
        while (ng & (ng - 1)) ng &= ng - 1;
    if (a.plan && a.n_out > 8 * ng) return hipErrorInvalidValue;
    const long long wgs = a.per_stripe ? (long long)a.stripes * a.wps : ((long long)a.stripes * a.nch + 63) / 64;
    if (wgs <= 0) return hipSuccess;
    if (wgs > 0x7FFFFFFF) return hipErrorInvalidValue;
    JumpApplyArgs g = a;
    if (!order_stripes(g.order, a.plan, a.plan_stride, a.per_stripe ? a.stripes : 0, a.n_out, st)) g.order = nullptr;
    const char *fb = std::getenv("LONGHAIR_AMD_INV_FALLBACK");  // (tests: the in-asm table)
    g.jump_fallback = fb && std::atoi(fb) ? 1 : 0;
    if (a.in_ptrs)
        hipLaunchKernelGGL(lh_apply_jump_kernel<true>, dim3((unsigned)wgs), dim3(64u * (unsigned)ng), 0, st, g);
    else
        hipLaunchKernelGGL(lh_apply_jump_kernel<false>, dim3((unsigned)wgs), dim3(64u * (unsigned)ng), 0, st, g);
    note_launch(g.jump_fallback ? (a.in_ptrs ? "lh_apply_jump_kernel(pointer table, fallback)" : "lh_apply_jump_kernel(fallback)")
                                : (a.in_ptrs ? "lh_apply_jump_kernel(pointer table)" : "lh_apply_jump_kernel"));
    return hipGetLastError();
}

bool jump_table2_usable(int device) {
    static std::mutex mu;
    static std::map<int, bool> known;
    std::lock_guard<std::mutex> g(mu);
    auto it = known.find(device);
    if (it != known.end()) return it->second;
    bool ok = false;
    uint32_t *d_out = nullptr, h[2] = {0, 0};
    if (hipMalloc(&d_out, 8) == hipSuccess) {
        hipLaunchKernelGGL(lh_jump_probe_kernel, dim3(1), dim3(64), 0, nullptr, d_out);
        ok = hipGetLastError() == hipSuccess && hipMemcpy(h, d_out, 8, hipMemcpyDeviceToHost) == hipSuccess &&
             h[1] <= 0xFFFFFFFFu - 256u * 132u;
        (void)hipFree(d_out);
    }
    known[device] = ok;
    return ok;
}

hipError_t launch_inverse(const InverseArgs &a, hipStream_t st) {
    // sub-blocks in 256-byte chunks (the windowed configurations: sub % 256 == 0)
    if (a.bytes % 2048 != 0 || a.e_max < 1 || a.e_max > 64 || a.m > 64) return hipErrorInvalidValue;
    const long long blocks = (long long)a.stripes * (a.bytes / 2048);
    if (blocks <= 0) return hipSuccess;
    if (blocks > 0x7FFFFFFF) return hipErrorInvalidValue;
    // lh_inverse_gt_kernel: 8 outputs per wave, packed (wave g: outputs 8g .. 8g + 7) for
    // e_max <= 32 and spread (g, g + nw, ...) above (profiles/r3m_phase_b_gtab.txt: k128/m32
    // decode 3.56 -> 3.51 ms packed, k200/m56 0.583 -> 0.567 spread).
    // LONGHAIR_AMD_INV_FALLBACK=1: the in-asm table inside the same kernel (tests).
    InverseArgs g = a;
    const char *fb = std::getenv("LONGHAIR_AMD_INV_FALLBACK");
    g.pack = a.e_max <= 32 ? 1 : 0;
    g.jump_fallback = fb && std::atoi(fb) ? 1 : 0;
    // Two consecutive 2 KiB chunks of a stripe per workgroup, the tile pipeline carried across
    // them, so the pipeline's start (plan, jump targets, first tile's DMA) is paid once per
    // pair (profiles/r4k_tune_*_inv_chunks.txt: k200/m56 decode 0.665 -> 0.617 ms with 2, 0.635
    // with 4; k128/m32 3.634 ms with 1, 2 or 4).
#ifndef LH_PB_CPW
#define LH_PB_CPW 2  // (an A/B build may set another, make HIP_EXTRA=-DLH_PB_CPW=n)
#endif
    const int cps = a.bytes / 2048;
    const int cpw = cps < LH_PB_CPW ? cps : LH_PB_CPW;
    g.chunks_per_wg = cpw;
    const long long wgs = (long long)a.stripes * ((cps + cpw - 1) / cpw);
    if (!order_stripes(g.order, a.plan, a.plan_stride, a.stripes, a.e_max, st)) g.order = nullptr;
    // Spread outputs (e_max > 32) over a power-of-two number of waves, so whole workgroups
    // fill a CU's wave slots (k200/m56: 8 waves instead of 7, decode 0.594 / 0.583 -> 0.570 /
    // 0.579 ms, profiles/r5w_phase_b_pow2.txt).
    int nw = (a.e_max + 7) / 8;
    if (!g.pack)
        while (nw & (nw - 1)) nw += nw & -nw;  // round up
    hipLaunchKernelGGL(lh_inverse_gt_kernel, dim3((unsigned)wgs), dim3(64u * (unsigned)nw), 0, st, g);
    note_launch(g.jump_fallback ? "lh_inverse_gt_kernel(fallback)" : "lh_inverse_gt_kernel");
    return hipGetLastError();
}

hipError_t launch_writeback(const WritebackArgs &a, hipStream_t st) {
    if (a.stripes <= 0) return hipSuccess;
    // 8-byte lanes need 8-byte aligned blocks on the host side (16-byte lanes when aligned)
    if (((a.bytes | a.host_stride | (long long)(uintptr_t)a.host) & 7) != 0 || a.k < 1 || a.k > 255)
        return hipErrorInvalidValue;
    // One segment per 4 KiB of block (256 lanes x 16 B), at most 16, and only while the
    // chunk has fewer than 1 024 stripes.
    int seg = a.stripes >= 1024 ? 1 : a.bytes / 4096;
    seg = seg < 1 ? 1 : (seg > 16 ? 16 : seg);
    hipLaunchKernelGGL(lh_writeback_kernel, dim3((unsigned)a.stripes, (unsigned)seg), dim3(256), 0, st, a);
    note_launch("lh_writeback_kernel");
    return hipGetLastError();
}

hipError_t launch_xor_reduce(const XorArgs &a, hipStream_t st) {
    const long long lanes = (long long)a.stripes * a.nch;
    hipLaunchKernelGGL(lh_xor_reduce_kernel, dim3((unsigned)((lanes + 255) / 256)), dim3(256), 0, st, a);
    note_launch("lh_xor_reduce_kernel");
    return hipGetLastError();
}

hipError_t launch_scatter(const ScatterArgs &a, hipStream_t st) {
    const long long lanes = (long long)a.stripes * a.e_max * ((a.bytes + 15) / 16);
    hipLaunchKernelGGL(lh_scatter_kernel, dim3((unsigned)((lanes + 255) / 256)), dim3(256), 0, st, a);
    note_launch("lh_scatter_kernel");
    return hipGetLastError();
}

hipError_t launch_ptr_copy(const PtrCopyArgs &a, hipStream_t st) {
    const long long waves = (long long)a.stripes * a.ncopy;
    if (waves <= 0) return hipSuccess;
    if ((waves + 3) / 4 > 0x7FFFFFFF) return hipErrorInvalidValue;
    hipLaunchKernelGGL(lh_ptr_copy_kernel, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, st, a);
    note_launch(a.scatter ? "lh_ptr_copy_kernel(scatter)" : "lh_ptr_copy_kernel(gather)");
    return hipGetLastError();
}

hipError_t launch_frame(const FrameArgs &a, hipStream_t st) {
    const long long threads = (long long)a.stripes * a.npk * ((a.bytes + 3) / 4);
    if (threads <= 0) return hipSuccess;
    hipLaunchKernelGGL(lh_frame_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, st, a);
    note_launch("lh_frame_kernel");
    return hipGetLastError();
}

hipError_t launch_plan(const PlanArgs &a, hipStream_t st) {
    if (a.k > 1 && a.m > 1 && a.e_max <= 8) {
        const unsigned blocks = (unsigned)((a.stripes + 255) / 256);
        if (a.e_max <= 4) hipLaunchKernelGGL(lh_plan_small_kernel<4>, dim3(blocks), dim3(256), 0, st, a);
        else hipLaunchKernelGGL(lh_plan_small_kernel<8>, dim3(blocks), dim3(256), 0, st, a);
        note_launch(a.e_max <= 4 ? "lh_plan_small_kernel<4>" : "lh_plan_small_kernel<8>");
        return hipGetLastError();
    }
    // Few stripes (latency-bound: one workgroup per stripe cannot fill the chip): four
    // waves per stripe split the elimination's columns; many stripes: one wave each.
    const size_t lds = (size_t)2 * a.e_max * (a.e_max > 64 ? 128 : 64);
    unsigned threads = (a.stripes <= 4096 && a.e_max > 8) ? 256u : 64u;
    hipLaunchKernelGGL(lh_plan_kernel, dim3((unsigned)a.stripes), dim3(threads), lds, st, a);
    note_launch(a.points ? "lh_plan_kernel(closed form)" : "lh_plan_kernel");
    return hipGetLastError();
}

}  // namespace lh
