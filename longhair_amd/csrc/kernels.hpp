// kernels.hpp -- argument blocks and launchers shared by the host code and kernels.hip.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace lh {

constexpr int kGenericTileOut = 4;  // outputs per lane in lh_apply_generic_kernel

// Per-stripe decode plan record (written by lh_plan_kernel):
//   [0] e (erasures to recover)   [1] status (int8)   [2..15] reserved
//   [16]                     out_slot[e_max]   slot receiving the i-th recovered original
//   [16+e_max]               src_slot[k]       slot of original x, 0xFF if erased
//   [16+e_max+k]             rec_slot[m]       slot of recovery row r, 0xFF if absent
//   [16+e_max+k+m]           coef[e_max][m]    A^-1 over recovery rows (0 = unused row)
//   [16+e_max+k+m+e_max*m]   w[e_max][k]       per-slot coefficients of the recovered
//                                              originals (single-pass form)
struct PlanView {
    uint8_t *p;
    int k, m, e_max;
    __host__ __device__ PlanView(uint8_t *p_, int k_, int m_, int e_max_) : p(p_), k(k_), m(m_), e_max(e_max_) {}
    __host__ __device__ PlanView(const uint8_t *p_, int k_, int m_, int e_max_)
        : p(const_cast<uint8_t *>(p_)), k(k_), m(m_), e_max(e_max_) {}
    __host__ __device__ static long long bytes(int k, int m, int e_max) {
        long long n = 16 + e_max + k + m + (long long)e_max * m + (long long)e_max * k;
        return (n + 15) / 16 * 16;
    }
    __host__ __device__ int e() const { return p[0]; }
    __host__ __device__ int out_slot(int i) const { return p[16 + i]; }
    __host__ __device__ void set_out_slot(int i, uint8_t v) { p[16 + i] = v; }
    __host__ __device__ int src_slot(int x) const { return p[16 + e_max + x]; }
    __host__ __device__ void set_src_slot(int x, uint8_t v) { p[16 + e_max + x] = v; }
    __host__ __device__ int rec_slot(int r) const { return p[16 + e_max + k + r]; }
    __host__ __device__ void set_rec_slot(int r, uint8_t v) { p[16 + e_max + k + r] = v; }
    __host__ __device__ uint8_t *coef_ptr() const { return p + 16 + e_max + k + m; }
    __host__ __device__ void set_coef(int i, int r, uint8_t v) { coef_ptr()[i * m + r] = v; }
    __host__ __device__ uint8_t *w_ptr() const { return p + 16 + e_max + k + m + e_max * m; }
    __host__ __device__ void set_w(int i, int slot, uint8_t v) { w_ptr()[i * k + slot] = v; }
    __host__ __device__ static long long w_offset(int k, int m, int e_max) {
        return 16 + e_max + k + m + (long long)e_max * m;
    }
};

struct ApplyArgs {
    const uint8_t *in;            // stripe s, input j: in + s*in_stride + j*bytes
    long long in_stride;
    uint8_t *out;                 // stripe s, output i: out + s*out_stride + i*bytes
    long long out_stride;
    const uint8_t *coef;          // coef[s*coef_stride + i*n_in + j]  (stride 0: shared)
    long long coef_stride;
    const uint8_t *nout_per_stripe;  // optional: valid outputs of stripe s at [s*nout_stride]
    long long nout_stride;
    int n_in, n_out, bytes, sub, stripes, nch;
};

// Generic apply through the phase-B jump table (lh_apply_jump_kernel): out_i = sum_j
// B(W[i][j]) in_j for any coefficient matrix, at the nibble-table cost (22 XORs per input
// column and lane, then one XOR3 per output sub-row) instead of lh_apply_generic_kernel's 64
// masked XORs per output and column.  Dword lanes (sub >= 4), up to 8 outputs per wave and
// ceil(n_out / 8) waves per workgroup (at most 16; more outputs take further rounds).
//  per_stripe = 0 (encode: one coefficient matrix for every stripe): lanes run flat over
//    (stripe, dword chunk), so small blocks fill whole waves;
//  per_stripe = 1 (decode: the plan's per-stripe W over the k slots): a workgroup codes one
//    stripe's 64-lane chunk; the outputs go in place to the plan's output slots (count e =
//    plan[0]) after a workgroup barrier, so no wave still reads a slot another overwrites.
struct JumpApplyArgs {
    const uint8_t *in;            // stripe s, input j: in + s*in_stride + j*bytes
    long long in_stride;
    uint8_t *out;                 // per_stripe 0: stripe s, output i at out + s*out_stride + i*bytes
    long long out_stride;
    const uint8_t *coef;          // W[i][j] at coef + s*coef_stride + i*n_in + j (stride 0: shared)
    long long coef_stride;
    const uint8_t *plan;          // per_stripe 1: e and the output slots (PlanView), in place
    long long plan_stride;
    int n_in, n_out, bytes, sub, nch, stripes;
    int per_stripe, wps;          // wps: workgroups per stripe (per_stripe 1) = ceil(nch / 64)
    uint8_t *const *in_ptrs;      // pointer tables (cauchy_256_*_batch_ptrs), else NULL: input j of
    uint8_t *const *out_ptrs;     // stripe s at in_ptrs[s*in_n + j], output i (or, per_stripe 1, the
    int in_n, out_n;              // plan's slot i) at out_ptrs[s*out_n + i] (in, out, strides unused)
    int *order;                   // per_stripe 1: scratch of `stripes` ints, the stripes by e, largest
                                  // first (written by launch_apply_jump), or NULL: stripe order
    int dw;                       // bytes per lane per sub-block / 4: 1 (nch = ceil(sub / 4)) or
                                  // 2 (nch = ceil(sub / 8), the two-dword table, sub >= 8)
    int jump_fallback;            // dw 1: the in-asm table (set by launch_apply_jump from
                                  // LONGHAIR_AMD_INV_FALLBACK, tests), as a straddling table would
};

struct XorArgs {
    const uint8_t *in;            // stripe s, input j: in + s*in_stride + j*bytes
    long long in_stride;
    uint8_t *out;                 // stripe s: out + s*out_stride (+ out_slot*bytes with plan)
    long long out_stride;
    const uint8_t *plan;          // optional (decode m == 1): output slot from the plan
    long long plan_stride;
    int k, m, e_max;
    int n_in, n_rep, bytes, stripes, nch;
};

struct ScatterArgs {
    const uint8_t *work;
    long long work_stride;
    uint8_t *blocks;
    long long blocks_stride;
    const uint8_t *plan;
    long long plan_stride;
    int k, m, e_max, bytes, stripes;
};

struct PlanArgs {
    uint8_t *rows;                // stripes x k, rewritten
    int8_t *status;               // optional, stripes
    uint8_t *plan;
    long long plan_stride;
    const uint8_t *G;             // m x k generator (row 0 = ones)
    const uint8_t *points;        // Cauchy points X'[k], Y'[m] of G, or null (no closed form)
    const uint8_t *gf_exp;        // 512
    const int16_t *gf_log;        // 256
    int k, m, e_max, stripes;
    int want_w;                   // emit the single-pass coefficients (generic path)
};

struct FrameArgs {
    const uint8_t *data;          // frame: data blocks (stripe stride data_stride)
    long long data_stride;
    const uint8_t *rec;           // frame: recovery blocks
    long long rec_stride;
    uint8_t *packets;             // [stripe][packet i][row byte + block]
    long long packet_stride;
    uint8_t *blocks;              // unframe: decode slots
    long long blocks_stride;
    uint8_t *rows;                // unframe: Block.row bytes, stripes x k
    int k, m, bytes, stripes, npk, unframe;
};

// Phase B of the large-m decode (after the windowed phase-A kernel replaced every present
// recovery block R_r by V_r in place): D_{E_i} = sum_r B(coef[i][r]) V_r into out_slot(i).
struct InverseArgs {
    uint8_t *blocks;              // stripe s, slot j: blocks + s*stride + j*bytes
    long long stride;
    const uint8_t *plan;          // PlanView records
    long long plan_stride;
    int k, m, e_max, bytes, stripes;
    int pack;                     // lh_inverse_gt_kernel: 8 consecutive outputs per wave
    int jump_fallback;            // lh_inverse_gt_kernel: take the in-asm table (tests)
    int chunks_per_wg;            // lh_inverse_gt_kernel: consecutive 2 KiB chunks per workgroup (>= 1)
    uint8_t *const *ptrs;         // pointer-table batches: slot j of stripe s at ptrs[s*k + j]
                                  // (blocks and stride unused), else NULL
    int *order;                   // scratch of `stripes` ints: the stripes by e, largest first
                                  // (written by launch_inverse; NULL: launch order = stripe order)
};

hipError_t launch_inverse(const InverseArgs &a, hipStream_t st);

// Pinned-host decode pipeline: write every slot that held a recovery block before the
// decode (rows_orig >= k: the only slots decode writes) straight into the caller's pinned
// host buffer (device-mapped pointer), so only the recovered blocks cross PCIe back.
struct WritebackArgs {
    const uint8_t *blocks;        // device chunk: stripe s, slot j at blocks + s*stride + j*bytes
    long long stride;
    uint8_t *host;                // device-mapped pinned host buffer of the chunk
    long long host_stride;
    const uint8_t *rows_orig;     // the chunk's Block.row bytes before the decode, stripes x k
    int k, bytes, stripes;
};

// Pointer-table batches (cauchy_256_*_batch_ptrs) on the paths without a pointer form:
// block j of stripe s lives at ptrs[s * n + j].  gather: into a contiguous chunk (stripe s,
// block j at chunk + s * stride + j * bytes); scatter: back from it, only the blocks the
// decode may have changed when sel is set (sel = the chunk's rows before the decode):
// the slots with sel[s * n + j] >= sel_min (k, m > 1: the slots that held recovery rows), or
// with m1 the one output slot of cauchy_decode_m1 (the last slot with a row >= k, else slot 0,
// cauchy_256.cpp:487-535); and never a stripe whose status (when given) is non-zero (invalid
// rows: the decode left it untouched).  Only the first ncopy blocks of each stripe are copied.
struct PtrCopyArgs {
    uint8_t *const *ptrs;         // [stripe][n]
    uint8_t *chunk;
    long long stride;
    const uint8_t *sel;           // [stripe][n] or NULL
    const int8_t *status;         // [stripe] or NULL (scatter)
    int sel_min, m1;
    int n, ncopy, bytes, stripes, scatter;
};

// Launch trace (codec.cpp): every launch site records the kernel it enqueued, so the
// calling thread can ask which kernels its last batch call ran (cauchy_256_last_launch).
void note_launch(const char *kernel);

hipError_t launch_writeback(const WritebackArgs &a, hipStream_t st);
hipError_t launch_apply_generic(const ApplyArgs &a, int W, hipStream_t st);
hipError_t launch_apply_jump(const JumpApplyArgs &a, hipStream_t st);
// lh_inv_gtab2 lies within one 4 GiB page on `device` (probed once; dw 2 only then)
bool jump_table2_usable(int device);
hipError_t launch_frame(const FrameArgs &a, hipStream_t st);
hipError_t launch_xor_reduce(const XorArgs &a, hipStream_t st);
hipError_t launch_scatter(const ScatterArgs &a, hipStream_t st);
hipError_t launch_plan(const PlanArgs &a, hipStream_t st);
hipError_t launch_ptr_copy(const PtrCopyArgs &a, hipStream_t st);

}  // namespace lh
