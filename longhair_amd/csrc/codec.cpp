// codec.cpp -- the C ABI: drop-in cauchy_256.h entry points and the batched
// device-resident extension (cauchy_256_batch.h).
//
// Host code only validates parameters, looks up plans/kernels and enqueues work; every
// byte of encode/decode output is produced by GPU kernels (kernels.hip, jit_codec.hip).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <thread>
#include <string>
#include <vector>

#include "../../include/cauchy_256.h"
#include "../../include/cauchy_256_batch.h"
#include "field.hpp"
#include "jit.hpp"
#include "host_codec.hpp"
#include "kernels.hpp"

namespace lh {

enum { kOk = 0, kInvalid = -1, kNoDevice = -2, kHipError = -3 };

thread_local std::string g_last_error;
thread_local std::string g_last_launch;  // kernels enqueued by this thread's last call

static int fail(int code, const std::string &msg) {
    g_last_error = msg;
    return code;
}

// The C ABI's exception barrier (LH_TRY / LH_CATCH below): called inside a catch block.
static int internal_error() noexcept {
    const char *what = "unknown exception";
    try {
        throw;
    } catch (const std::bad_alloc &) {
        what = "out of host memory";
    } catch (const std::exception &e) {
        what = e.what();
    } catch (...) {
    }
    try {
        g_last_error = std::string("longhair_amd: internal error: ") + what;
    } catch (...) {
    }
    return kHipError;
}

// Test-only (cauchy_256_debug_throw_next, include/cauchy_256_test.h; built into the checked
// library only, LH_TEST_HOOKS): the calling thread's next guarded entry point throws inside
// its guard.
#ifdef LH_TEST_HOOKS
thread_local int g_throw_next = 0;
static void test_hook() {
    if (g_throw_next) {
        g_throw_next = 0;
        throw std::runtime_error("exception injected by cauchy_256_debug_throw_next");
    }
}
#else
static inline void test_hook() {}
#endif

void note_launch(const char *kernel) {
    const std::string k(kernel);
    // each kernel once, in order of first launch (the host-batch pipeline repeats them per chunk)
    size_t pos = 0;
    while ((pos = g_last_launch.find(k, pos)) != std::string::npos) {
        const size_t end = pos + k.size();
        if ((pos == 0 || g_last_launch[pos - 1] == ';') && (end == g_last_launch.size() || g_last_launch[end] == ';'))
            return;
        pos = end;
    }
    if (!g_last_launch.empty()) g_last_launch += ';';
    g_last_launch += k;
}

// Starts a new launch trace for one entry-point call.
struct LaunchTrace {
    LaunchTrace() { g_last_launch.clear(); }
};

#define LH_HIP(expr)                                                                       \
    do {                                                                                   \
        hipError_t e_ = (expr);                                                            \
        if (e_ != hipSuccess)                                                              \
            return fail(kHipError, std::string(#expr) + ": " + hipGetErrorString(e_));     \
    } while (0)

// Grow-only device buffer.  Growing never synchronises the device:
//  - reserve(n): for buffers whose every earlier use the caller has already waited for
//    (drop-in staging, host-batch pipelines: both end in a stream synchronisation);
//  - reserve(n, st): for buffers used on one stream only (per-stream workspaces): the old
//    allocation is released and the new one allocated in that stream's order
//    (hipFreeAsync / hipMallocAsync), so later kernels on `st` see the new buffer and
//    earlier ones finish with the old.
struct DevBuf {
    uint8_t *ptr = nullptr;
    size_t size = 0;
    bool stream_ordered = false;
    hipError_t reserve(size_t n) {
        if (n <= size) return hipSuccess;
        release(nullptr);
        hipError_t e = hipMalloc(&ptr, n);
        if (e == hipSuccess) size = n;
        else ptr = nullptr;
        return e;
    }
    hipError_t reserve(size_t n, hipStream_t st) {
        if (n <= size) return hipSuccess;
        release(st);
        hipError_t e = hipMallocAsync((void **)&ptr, n, st);
        if (e == hipSuccess) {
            size = n;
            stream_ordered = true;
        } else {
            ptr = nullptr;
        }
        return e;
    }
    void release(hipStream_t st) {
        if (ptr) {
            if (stream_ordered) (void)hipFreeAsync(ptr, st);
            else (void)hipFree(ptr);
        }
        ptr = nullptr;
        size = 0;
        stream_ordered = false;
    }
};

struct HostPinned {
    uint8_t *ptr = nullptr;
    size_t size = 0;
    unsigned flags = hipHostMallocDefault;  // hipHostMallocCoherent: read and written by kernels
    hipError_t reserve(size_t n) {
        if (n <= size) return hipSuccess;
        if (ptr) (void)hipHostFree(ptr);
        ptr = nullptr;
        size = 0;
        hipError_t e = hipHostMalloc(&ptr, n, flags);
        if (e == hipSuccess) size = n;
        return e;
    }
};

// Per-stream scratch (decode plans and the generic path's output workspace).
struct Workspace {
    DevBuf plan, work;
    DevBuf gather;  // pointer-table batches without a pointer form: the contiguous chunk
};

// Per-device state.
struct Device {
    int id = 0;
    int cus = 0;                         // compute units
    bool jump2 = false;                  // lh_apply_jump2_kernel may run (jump_table2_usable)
    std::mutex mu;                       // guards maps below and the drop-in staging
    uint8_t *gf_exp = nullptr;           // 512 B
    int16_t *gf_log = nullptr;           // 256 x int16
    // (k, m) -> m x k generator on device, followed by the Cauchy points X'[k], Y'[m]
    // when the generator has that form (second: points present).
    std::map<std::pair<int, int>, std::pair<uint8_t *, bool>> generators;
    DevBuf zero;                         // zero page (>= block bytes)
    std::vector<uint8_t *> retired;      // outgrown zero pages (never freed: see zero_page)
    std::map<hipStream_t, Workspace> ws;
    JitCache jit;
    // Drop-in (single stripe) calls on the GPU: kDropinSlots independent staging slots, each
    // with its own stream and buffers, so concurrent callers (the reference's calls are
    // re-entrant) run side by side instead of one at a time per device.
    struct DropinSlot {
        std::mutex mu;
        hipStream_t stream = nullptr;  // created on first use
        DevBuf stage;
        HostPinned host_stage;
        // all-device drop-in calls: the pointer table, rows and status, read and written by
        // the kernels straight from host memory (coherent: never cached on the device, so a
        // later call's table is never read stale), no copies
        HostPinned ptab{nullptr, 0, hipHostMallocCoherent | hipHostMallocMapped};
    };
    static constexpr int kDropinSlots = 4;  // GPU_MAX_HW_QUEUES is 4 by default
    DropinSlot dropin[kDropinSlots];
    // host-batch pipeline: per ring slot a stream, device buffers and an event
    std::mutex pipe_mu;
    hipStream_t pipe_stream[3] = {nullptr, nullptr, nullptr};
    hipEvent_t pipe_meta_ev = nullptr;  // decode: the call's rows are on the device
    DevBuf pipe_blocks[3], pipe_out[3];
    DevBuf pipe_rows, pipe_rows0, pipe_status;  // decode: the whole call's rows / status
    HostPinned pipe_meta;  // decode: the call's Block.row bytes and status, pinned
};

static std::mutex g_devices_mu;
static std::map<int, std::unique_ptr<Device>> g_devices;

static int current_device(Device **out) {
    int id = 0;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0)
        return fail(kNoDevice, "longhair_amd: no HIP device available (the codec has no CPU path)");
    LH_HIP(hipGetDevice(&id));
    std::lock_guard<std::mutex> g(g_devices_mu);
    auto &slot = g_devices[id];
    if (!slot) {
        std::unique_ptr<Device> d(new Device());
        d->id = id;
        const Field &F = Field::get();
        LH_HIP(hipMalloc(&d->gf_exp, 512));
        LH_HIP(hipMalloc(&d->gf_log, 256 * sizeof(int16_t)));
        LH_HIP(hipMemcpy(d->gf_exp, F.exp, 512, hipMemcpyHostToDevice));
        LH_HIP(hipMemcpy(d->gf_log, F.log, 256 * sizeof(int16_t), hipMemcpyHostToDevice));
        LH_HIP(hipDeviceGetAttribute(&d->cus, hipDeviceAttributeMultiprocessorCount, id));
        d->jump2 = jump_table2_usable(id);
        slot = std::move(d);
    }
    *out = slot.get();
    return kOk;
}

// True when `st` is being captured into a graph: memory must not be allocated then (a
// stream-ordered allocation would become graph-owned memory that later non-graph launches
// still point at, and the old buffer would be freed inside the graph).
static bool capturing(hipStream_t st) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(st, &cs) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return cs != hipStreamCaptureStatusNone;
}

static int capture_growth_error(const char *what) {
    return fail(kHipError, std::string("longhair_amd: the ") + what +
                               " must grow while the stream is being captured; reserve it before capture with "
                               "cauchy_256_batch_prepare_stream(k, m, bytes, max_stripes, stream) or an "
                               "uncaptured call of the same size on that stream");
}

static int device_generator(Device *d, int k, int m, const uint8_t **out, const uint8_t **points = nullptr,
                            hipStream_t st = nullptr) {
    std::lock_guard<std::mutex> g(d->mu);
    auto it = d->generators.find({k, m});
    if (it == d->generators.end()) {
        if (capturing(st)) return capture_growth_error("generator matrix");
        std::vector<uint8_t> G = generator_matrix(k, m);
        std::vector<uint8_t> xs, ys;
        const bool pts = cauchy_points(k, m, xs, ys);
        if (pts) {
            G.insert(G.end(), xs.begin(), xs.end());
            G.insert(G.end(), ys.begin(), ys.end());
        }
        uint8_t *p = nullptr;
        LH_HIP(hipMalloc(&p, G.size()));
        LH_HIP(hipMemcpy(p, G.data(), G.size(), hipMemcpyHostToDevice));
        it = d->generators.emplace(std::make_pair(k, m), std::make_pair(p, pts)).first;
    }
    *out = it->second.first;
    if (points) *points = it->second.second ? it->second.first + (size_t)k * m : nullptr;
    return kOk;
}

// Zero page (>= block bytes), shared by every stream.  A larger one replaces it without a
// device synchronisation: the old page stays allocated (kernels in flight on other streams
// may still read it) and the new page is cleared on the null stream, which this thread
// waits for before publishing the pointer (non-blocking streams are not stalled).
static int zero_page(Device *d, size_t bytes, const uint8_t **out, hipStream_t st = nullptr) {
    std::lock_guard<std::mutex> g(d->mu);
    if (d->zero.size < bytes) {
        if (capturing(st)) return capture_growth_error("zero page");
        uint8_t *p = nullptr;
        LH_HIP(hipMalloc(&p, bytes));
        LH_HIP(hipMemsetAsync(p, 0, bytes, nullptr));
        LH_HIP(hipStreamSynchronize(nullptr));
        if (d->zero.ptr) d->retired.push_back(d->zero.ptr);
        d->zero.ptr = p;
        d->zero.size = bytes;
    }
    *out = d->zero.ptr;
    return kOk;
}

static int workspace(Device *d, hipStream_t st, size_t plan_bytes, size_t work_bytes, Workspace **out) {
    std::lock_guard<std::mutex> g(d->mu);
    Workspace &w = d->ws[st];
    if ((plan_bytes > w.plan.size || work_bytes > w.work.size) && capturing(st))
        return capture_growth_error("per-stream decode workspace");
    LH_HIP(w.plan.reserve(plan_bytes, st));
    if (work_bytes) LH_HIP(w.work.reserve(work_bytes, st));
    *out = &w;
    return kOk;
}

// Grid for a specialised kernel: one 4-wave block per 4 waves of work.
static long long jit_blocks(const JitConfig &cfg, int stripes) {
    const long long waves = cfg.spw ? (stripes + cfg.spw - 1) / cfg.spw : (long long)stripes * cfg.wps;
    long long blocks = (waves + 3) / 4;
    return blocks;
}
// The encode's grid: one block per cfg.enc_wpb waves of work.
static long long jit_encode_blocks(const JitConfig &cfg, int stripes) {
    const long long waves = cfg.spw ? (stripes + cfg.spw - 1) / cfg.spw : (long long)stripes * cfg.wps;
    return (waves + cfg.enc_wpb - 1) / cfg.enc_wpb;
}
static int generic_word(int sub) {
    if (sub >= 4) return 4;
    if (sub >= 2) return 2;
    return 1;
}

// Specialised kernels of a configuration.  A module loaded or in the on-disk cache
// (jit_cache/, tools/precompile.py) is used at once.  Otherwise batch calls (allow_compile)
// start hiprtc on a background thread and take the generic kernels until the module is
// ready (batch_jit_mode: LONGHAIR_AMD_JIT_SYNC=1 compiles in the call instead,
// LONGHAIR_AMD_JIT_COMPILE=0 never compiles); drop-in calls never compile.  Returns nullptr
// with *hard set when a compilation made for this call (LONGHAIR_AMD_JIT_SYNC=1) failed;
// a failed background compilation leaves the shape on the generic kernels.
static const JitKernels *jit_lookup(Device *d, const JitConfig &cfg, bool allow_compile, std::string *err,
                                    bool *hard) {
    const JitMode mode = allow_compile ? batch_jit_mode() : JitMode::kCached;
    bool failed = false;
    const JitKernels *jk = d->jit.get(cfg, err, mode, &failed);
    *hard = !jk && failed && mode == JitMode::kBlocking;
    return jk;
}

// ------------------------------------------------------------------------ encode
// The jump-table apply's lane width (a.sub, a.n_out, a.per_stripe set): two-dword lanes
// (lh_apply_jump2_kernel: a jump covers 8 bytes per lane) only where a one-dword wave would be
// half empty -- at most 4 outputs -- and the lanes stay full: a flat (encode) launch with
// sub >= 8, an in-place decode with sub >= 512.  With more outputs the one-dword form wins
// (its wave carries 8 outputs per jump target fetch; profiles/r5f_jump_dw.txt: k128/m32
// encode 5.31 ms one-dword, 8.27 two-dword; k29/m4 encode 0.700 / 0.665).  In place, the last
// lane of a sub-block (shifted back over its neighbour when the width does not divide sub)
// must share its neighbour's workgroup, whose barrier orders every read of a slot before its
// overwrite.
static void jump_layout(const Device *d, JumpApplyArgs &a, bool in_place) {
    auto lone_tail = [&](int w) {
        const int nch = (a.sub + w - 1) / w;
        return a.sub % w != 0 && nch > 1 && (nch - 1) % 64 == 0;
    };
    bool two = a.n_out <= 4 && a.sub >= 8 && (!in_place || (a.sub >= 512 && !lone_tail(8)));
    const char *fb = std::getenv("LONGHAIR_AMD_INV_FALLBACK");  // (tests: the in-asm table)
    if (fb && std::atoi(fb)) two = false;
    a.dw = two && d->jump2 ? 2 : 1;
    a.nch = (a.sub + 4 * a.dw - 1) / (4 * a.dw);
    a.wps = (a.nch + 63) / 64;
}

static int xor_rows(int k, int n_rep, int bytes, int stripes, const uint8_t *in, long long in_stride,
                    uint8_t *out, long long out_stride, hipStream_t st) {
    XorArgs a{};
    a.in = in;
    a.in_stride = in_stride;
    a.out = out;
    a.out_stride = out_stride;
    a.plan = nullptr;
    a.n_in = k;
    a.n_rep = n_rep;
    a.bytes = bytes;
    a.stripes = stripes;
    a.nch = bytes / 16 + ((bytes % 16) ? 1 : 0);
    LH_HIP(launch_xor_reduce(a, st));
    return kOk;
}

static int encode_batch(int k, int m, int bytes, int stripes, const uint8_t *d_data, long long data_stride,
                        uint8_t *d_rec, long long rec_stride, hipStream_t st, bool allow_compile) {
    if (k < 1 || m < 1 || bytes <= 0 || stripes < 0 || k > 256 || m > 256)
        return fail(kInvalid, "invalid k, m, block_bytes or stripes");
    if (stripes == 0) return kOk;
    if (data_stride < (long long)k * bytes || rec_stride < (long long)m * bytes)
        return fail(kInvalid, "stripe strides smaller than the stripe");
    Device *d = nullptr;
    if (int rc = current_device(&d)) return rc;

    if (k == 1) return xor_rows(1, m, bytes, stripes, d_data, data_stride, d_rec, rec_stride, st);
    if (m == 1 || k + m > 256 || bytes % 8 != 0) {
        // Recovery block 0 first, as the reference (cauchy_256.cpp:1511-1527).
        if (int rc = xor_rows(k, 1, bytes, stripes, d_data, data_stride, d_rec, rec_stride, st)) return rc;
        return m == 1 ? kOk : fail(kInvalid, "k + m > 256 or block_bytes % 8 != 0");
    }

    JitConfig cfg;
    // (the specialised encode reads a wave's stripes through one buffer resource, whose
    // 32-bit range must cover them: jit_codec.hip lh_encode_wave)
    if (jit_config_for(k, m, bytes, false, &cfg) && data_stride * (cfg.spw ? cfg.spw : 1) < (1ll << 31)) {
        std::string err;
        bool hard = false;
        const JitKernels *jk = jit_lookup(d, cfg, allow_compile, &err, &hard);
        // No size-specialised module yet (compiling in the background, or a drop-in call, which
        // never compiles): the (k, m) block-size family's module, if loaded or cached (a batch
        // call queues its compilation too).
        JitConfig fcfg;
        if (!jk && !hard && !cfg.family && jit_family_config_for(k, m, bytes, &fcfg) &&
            data_stride * fcfg.spw < (1ll << 31)) {
            std::string ferr;
            bool fhard = false;
            if (const JitKernels *fk = jit_lookup(d, fcfg, allow_compile, &ferr, &fhard)) {
                jk = fk;
                cfg = fcfg;
            }
        }
        if (jk) {
            long long blocks = jit_encode_blocks(cfg, stripes);
            int bb = bytes;
            if (cfg.family) {  // (the family kernel takes the block size; spw follows from it)
                const long long spw = 64 / ((bytes / 8 + 7) / 8);
                blocks = ((stripes + spw - 1) / spw + cfg.enc_wpb - 1) / cfg.enc_wpb;
            }
            if (blocks > 0x7FFFFFFF) return fail(kInvalid, "batch too large");
            long long in_stride = data_stride, out_stride = rec_stride;
            int n = stripes;
            void *args[] = {(void *)&d_data, &in_stride, (void *)&d_rec, &out_stride, &n, &bb};
            LH_HIP(hipModuleLaunchKernel(jk->encode, (unsigned)blocks, 1, 1, 64u * (unsigned)cfg.enc_wpb,
                                         1, 1, jk->dyn_lds, st, args, nullptr));
            note_launch(cfg.family ? "lh_jit_encode(family)" : "lh_jit_encode");
            return kOk;
        }
        if (hard) return fail(kHipError, err);
    }
    if (jit_win_config_for(k, m, bytes, &cfg)) {
        std::string err;
        bool hard = false;
        const JitKernels *jk = jit_lookup(d, cfg, allow_compile, &err, &hard);
        if (jk && jk->encode_win) {
            const long long blocks = (long long)stripes * (cfg.sub / (64 * cfg.W));
            if (blocks > 0x7FFFFFFF) return fail(kInvalid, "batch too large");
            const unsigned threads = 64u * (unsigned)((m + cfg.rows_per_wave - 1) / cfg.rows_per_wave);
            long long in_stride = data_stride, out_stride = rec_stride;
            int n = stripes;
            int bb = bytes;  // (windowed modules take the block size as an argument)
            void *args[] = {(void *)&d_data, &in_stride, (void *)&d_rec, &out_stride, &n, &bb};
            LH_HIP(hipModuleLaunchKernel(jk->encode_win, (unsigned)blocks, 1, 1, threads, 1, 1, 0, st, args, nullptr));
            note_launch("lh_jit_encode_win");
            return kOk;
        }
        if (hard) return fail(kHipError, err);
    }
    const uint8_t *G = nullptr;
    if (int rc = device_generator(d, k, m, &G, nullptr, st)) return rc;
    if (bytes / 8 >= 4) {  // the jump-table apply (dword lanes)
        JumpApplyArgs a{};
        a.in = d_data;
        a.in_stride = data_stride;
        a.out = d_rec;
        a.out_stride = rec_stride;
        a.coef = G;
        a.coef_stride = 0;
        a.n_in = k;
        a.n_out = m;
        a.bytes = bytes;
        a.sub = bytes / 8;
        a.stripes = stripes;
        a.per_stripe = 0;
        jump_layout(d, a, false);
        LH_HIP(launch_apply_jump(a, st));
        return kOk;
    }
    ApplyArgs a{};
    a.in = d_data;
    a.in_stride = data_stride;
    a.out = d_rec;
    a.out_stride = rec_stride;
    a.coef = G;
    a.coef_stride = 0;
    a.n_in = k;
    a.n_out = m;
    a.bytes = bytes;
    a.sub = bytes / 8;
    a.stripes = stripes;
    const int W = generic_word(a.sub);
    a.nch = (a.sub + W - 1) / W;
    LH_HIP(launch_apply_generic(a, W, st));
    return kOk;
}

// ------------------------------------------------------------------------ decode
// The per-stripe erasure planner (lh_plan_kernel / lh_plan_small_kernel) into the stream's
// plan workspace (reserved with `work_bytes` of generic-path workspace beside it).
// LONGHAIR_AMD_PLAN_GJ (knob): Gauss-Jordan even where the closed form applies.
// The plan workspace holds the stripes' plans, then (16-byte aligned) one int per stripe:
// phase B's launch order (InverseArgs::order).
static size_t plan_order_offset(int stripes, long long plan_stride) {
    return ((size_t)stripes * (size_t)plan_stride + 15) & ~(size_t)15;
}

static int run_planner(Device *d, hipStream_t st, int k, int m, int e_max, int stripes, uint8_t *d_rows,
                       int8_t *d_status, size_t work_bytes, bool want_w, Workspace **out) {
    const long long plan_stride = PlanView::bytes(k, m, e_max);
    Workspace *w = nullptr;
    if (int rc = workspace(d, st, plan_order_offset(stripes, plan_stride) + (size_t)stripes * sizeof(int), work_bytes, &w))
        return rc;
    const uint8_t *G = nullptr, *points = nullptr;
    if (int rc = device_generator(d, k, m, &G, &points, st)) return rc;
    PlanArgs pa{};
    pa.rows = d_rows;
    pa.status = d_status;
    pa.plan = w->plan.ptr;
    pa.plan_stride = plan_stride;
    pa.G = G;
    pa.points = std::getenv("LONGHAIR_AMD_PLAN_GJ") ? nullptr : points;
    pa.gf_exp = d->gf_exp;
    pa.gf_log = d->gf_log;
    pa.k = k;
    pa.m = m;
    pa.e_max = e_max;
    pa.stripes = stripes;
    pa.want_w = want_w ? 1 : 0;
    LH_HIP(launch_plan(pa, st));
    *out = w;
    return kOk;
}

static int decode_batch(int k, int m, int bytes, int stripes, uint8_t *d_blocks, long long stride,
                        uint8_t *d_rows, int8_t *d_status, hipStream_t st, bool allow_compile) {
    if (k < 1 || m < 1 || bytes <= 0 || stripes < 0 || k > 256 || m > 256)
        return fail(kInvalid, "invalid k, m, block_bytes or stripes");
    if (stripes == 0) return kOk;
    if (stride < (long long)k * bytes) return fail(kInvalid, "stripe stride smaller than the stripe");
    if (m > 1 && k > 1 && (k + m > 256 || bytes % 8 != 0))
        return fail(kInvalid, "k + m > 256 or block_bytes % 8 != 0");
    Device *d = nullptr;
    if (int rc = current_device(&d)) return rc;

    const int e_max = (m == 1 || k <= 1) ? 1 : (k < m ? k : m);
    const long long plan_stride = PlanView::bytes(k, m, e_max);
    JitConfig cfg;
    // The specialised decode reads a wave's stripes through one buffer resource, whose
    // 32-bit range must cover them (jit_codec.hip lh_make_dsrc).
    const bool jit_ok = (k > 1 && m > 1) && jit_config_for(k, m, bytes, true, &cfg) &&
                        stride * (cfg.spw ? cfg.spw : 1) < (1ll << 31);
    const JitKernels *jk = nullptr;
    std::string err;
    if (jit_ok) {
        bool hard = false;
        jk = jit_lookup(d, cfg, allow_compile, &err, &hard);
        if (hard) return fail(kHipError, err);
    }
    // No size-specialised module yet (compiling in the background, or a drop-in call, which
    // never compiles): the (k, m) block-size family's fused decode, if loaded or cached (a batch
    // call queues its compilation too), as encode_batch does.
    JitConfig fcfg;
    if (!jk && k > 1 && m > 1 && !cfg.family && jit_family_config_for(k, m, bytes, &fcfg, true) &&
        stride * fcfg.spw < (1ll << 31)) {
        std::string ferr;
        bool fhard = false;
        if (const JitKernels *fk = jit_lookup(d, fcfg, allow_compile, &ferr, &fhard)) {
            if (fk->decode_fused) {
                jk = fk;
                cfg = fcfg;
            }
        }
    }
    const bool generic = (k > 1 && m > 1) && !jk;
    if (jk && jk->decode_fused && std::getenv("LONGHAIR_AMD_NO_FUSED_PLAN") == nullptr) {
        // Plan computed inside the decode kernel: one launch, no plan workspace.
        const uint8_t *zero = nullptr;
        if (int rc = zero_page(d, (size_t)bytes, &zero, st)) return rc;
        hipFunction_t fn = jk->decode_fused;
        long long s1 = stride;
        const uint8_t *gexp = d->gf_exp;
        const int16_t *glog = d->gf_log;
        // (Stripes past the last whole round of resident waves on a prefetch-depth-3 copy of
        // this kernel measured slower, 0.627 vs 0.610 ms at k29/m4 x 65 536: the partial round
        // costs < 1 %, the second launch more; profiles/r3w_decode_tail.txt.)
        int n = stripes, bb = bytes;  // (bb: the family kernel's block-size argument; cfg.spw follows it)
        void *args[] = {(void *)&d_blocks, &s1, (void *)&d_rows, (void *)&d_status, (void *)&zero,
                        (void *)&gexp, (void *)&glog, &n, &bb};
        const long long waves = cfg.spw ? (stripes + cfg.spw - 1) / cfg.spw : (long long)stripes * cfg.wps;
        const int wpb = cfg.family ? 4 : cfg.dec_wpb;  // (LH_DWPB; the family kernel runs 4-wave workgroups)
        LH_HIP(hipModuleLaunchKernel(fn, (unsigned)((waves + wpb - 1) / wpb), 1, 1, 64u * (unsigned)wpb, 1, 1,
                                     jk->dyn_lds, st, args, nullptr));
        note_launch(cfg.family ? "lh_jit_decode_fused(family)" : "lh_jit_decode_fused");
        return kOk;
    }
    // Large m (<= 64), sub % (64 W) == 0, after the planner: the windowed phase-A kernel
    // lh_jit_decode_wide (V_r in place of R_r), then lh_inverse_gt_kernel (phase B).
    JitConfig wcfg;
    const JitKernels *wk = nullptr;
    if (generic && jit_win_config_for(k, m, bytes, &wcfg, true)) {
        bool hard = false;
        wk = jit_lookup(d, wcfg, allow_compile, &err, &hard);
        if (hard) return fail(kHipError, err);
        if (wk && !wk->decode_wide) wk = nullptr;
    }
    // The generic decode: the jump-table apply in place (dword lanes), unless the last dword
    // lane of a sub-block -- shifted back over its neighbour's bytes when sub % 4 != 0 -- would
    // sit alone in a workgroup of its own (sub = 256 t + 1..3): then the old apply into a
    // workspace and a scatter.
    const int sub = bytes / 8, jnch = (sub + 3) / 4;
    const bool jump = generic && !wk && sub >= 4 && !(sub % 4 != 0 && jnch > 1 && (jnch - 1) % 64 == 0);
    const size_t work_bytes = (generic && !wk && !jump) ? (size_t)stripes * e_max * bytes : 0;
    Workspace *w = nullptr;
    if (int rc = run_planner(d, st, k, m, e_max, stripes, d_rows, d_status, work_bytes, generic && !wk, &w)) return rc;
    if (k <= 1) return kOk;

    if (m == 1) {
        XorArgs a{};
        a.in = d_blocks;
        a.in_stride = stride;
        a.out = d_blocks;
        a.out_stride = stride;
        a.plan = w->plan.ptr;
        a.plan_stride = plan_stride;
        a.k = k;
        a.m = m;
        a.e_max = e_max;
        a.n_in = k;
        a.n_rep = 1;
        a.bytes = bytes;
        a.stripes = stripes;
        a.nch = bytes / 16 + ((bytes % 16) ? 1 : 0);
        LH_HIP(launch_xor_reduce(a, st));
        return kOk;
    }
    if (jk) {
        const uint8_t *zero = nullptr;
        if (int rc = zero_page(d, (size_t)bytes, &zero, st)) return rc;
        const long long blocks = jit_blocks(cfg, stripes);
        long long s1 = stride, s2 = plan_stride;
        const uint8_t *plan = w->plan.ptr;
        int n = stripes;
        void *args[] = {(void *)&d_blocks, &s1, (void *)&plan, &s2, (void *)&zero, &n};
        LH_HIP(hipModuleLaunchKernel(jk->decode, (unsigned)blocks, 1, 1, 256, 1, 1, 0, st, args, nullptr));
        note_launch("lh_jit_decode");
        return kOk;
    }
    if (wk) {
        const uint8_t *zero = nullptr;
        if (int rc = zero_page(d, (size_t)bytes, &zero, st)) return rc;
        const long long cps = wcfg.sub / (64 * wcfg.W);
        if ((long long)stripes * cps > 0x7FFFFFFF) return fail(kInvalid, "batch too large");
        const unsigned threads = 64u * (unsigned)((m + wcfg.rows_per_wave - 1) / wcfg.rows_per_wave);
        // Phase A then phase B over the whole batch.  (Round 3 also ran them per chunk of
        // stripes, so a chunk's V could be read back from the Infinity Cache, optionally with
        // phase B on a side stream: slower at every chunk size, profiles/r3c_wide_chunk.txt;
        // removed in round 5.)
        {
            long long s1 = stride, s2 = plan_stride;
            const uint8_t *plan = w->plan.ptr;
            int nn = stripes;
            int bb = bytes;  // (windowed modules take the block size as an argument)
            void *args[] = {(void *)&d_blocks, &s1, (void *)&plan, &s2, (void *)&zero, &nn, &bb};
            LH_HIP(hipModuleLaunchKernel(wk->decode_wide, (unsigned)(stripes * cps), 1, 1, threads, 1, 1, 0, st, args,
                                         nullptr));
            note_launch("lh_jit_decode_wide");
            InverseArgs ia{};  // phase A left V_r in the recovery slots: phase B
            ia.blocks = d_blocks;
            ia.stride = stride;
            ia.plan = plan;
            ia.plan_stride = plan_stride;
            ia.k = k;
            ia.m = m;
            ia.e_max = e_max;
            ia.bytes = bytes;
            ia.stripes = stripes;
            ia.order = (int *)(w->plan.ptr + plan_order_offset(stripes, plan_stride));
            LH_HIP(launch_inverse(ia, st));
        }
        return kOk;
    }
    if (jump) {
        JumpApplyArgs a{};
        a.in = d_blocks;
        a.in_stride = stride;
        a.out = d_blocks;
        a.out_stride = stride;
        a.coef = w->plan.ptr + PlanView::w_offset(k, m, e_max);
        a.coef_stride = plan_stride;
        a.plan = w->plan.ptr;
        a.plan_stride = plan_stride;
        a.n_in = k;
        a.n_out = e_max;
        a.bytes = bytes;
        a.sub = sub;
        a.stripes = stripes;
        a.per_stripe = 1;
        a.order = (int *)(w->plan.ptr + plan_order_offset(stripes, plan_stride));  // by e, largest first
        jump_layout(d, a, true);
        LH_HIP(launch_apply_jump(a, st));
        return kOk;
    }
    // Generic, tiny blocks: recovered originals into the workspace, then into their slots.
    ApplyArgs a{};
    a.in = d_blocks;
    a.in_stride = stride;
    a.out = w->work.ptr;
    a.out_stride = (long long)e_max * bytes;
    a.coef = w->plan.ptr + PlanView::w_offset(k, m, e_max);
    a.coef_stride = plan_stride;
    a.nout_per_stripe = w->plan.ptr;
    a.nout_stride = plan_stride;
    a.n_in = k;
    a.n_out = e_max;
    a.bytes = bytes;
    a.sub = bytes / 8;
    a.stripes = stripes;
    const int W = generic_word(a.sub);
    a.nch = (a.sub + W - 1) / W;
    LH_HIP(launch_apply_generic(a, W, st));
    ScatterArgs sa{};
    sa.work = w->work.ptr;
    sa.work_stride = (long long)e_max * bytes;
    sa.blocks = d_blocks;
    sa.blocks_stride = stride;
    sa.plan = w->plan.ptr;
    sa.plan_stride = plan_stride;
    sa.k = k;
    sa.m = m;
    sa.e_max = e_max;
    sa.bytes = bytes;
    sa.stripes = stripes;
    LH_HIP(launch_scatter(sa, st));
    return kOk;
}

// ------------------------------------------------------------ pointer-table batches
// The reference's per-block pointers (cauchy_256.h:78 data_ptrs[], :103 Block *) for a batch
// of stripes, with the pointer tables in device memory: row s of a table holds stripe s's
// block pointers.  Shapes with a register network (jit.cpp jit_ptr_config_for: the k29/m4
// family) read and write the blocks where they lie (jit_codec.hip LH_PTR: a wave's table rows
// staged in LDS).  Every other shape gathers each chunk of stripes into the stream's
// workspace (lh_ptr_copy_kernel), runs the strided batch path on it and scatters the outputs
// back: one extra read and write of the inputs, bit-identical results.
static constexpr long long kPtrChunkBytes = 256ll << 20;

static int gather_chunk(Device *d, hipStream_t st, long long per_stripe, int stripes, uint8_t **buf, int *chunk) {
    long long cap = kPtrChunkBytes;
    if (const char *e = std::getenv("LONGHAIR_AMD_PTR_CHUNK_BYTES")) cap = std::max(1ll, std::atoll(e));  // (tests)
    const long long c = std::max(1ll, std::min((long long)stripes, cap / std::max(1ll, per_stripe)));
    std::lock_guard<std::mutex> g(d->mu);
    Workspace &w = d->ws[st];
    if ((size_t)(c * per_stripe) > w.gather.size && capturing(st))
        return capture_growth_error("per-stream gather chunk");
    LH_HIP(w.gather.reserve((size_t)(c * per_stripe), st));
    *buf = w.gather.ptr;
    *chunk = (int)c;
    return kOk;
}

static int ptr_copy(uint8_t *const *ptrs, int n, int ncopy, uint8_t *chunk, long long stride, int bytes, int stripes,
                    bool scatter, const uint8_t *sel, int sel_min, hipStream_t st, const int8_t *status = nullptr,
                    bool m1 = false) {
    PtrCopyArgs a{};
    a.ptrs = ptrs;
    a.chunk = chunk;
    a.stride = stride;
    a.sel = sel;
    a.sel_min = sel_min;
    a.status = status;
    a.m1 = m1 ? 1 : 0;
    a.n = n;
    a.ncopy = ncopy;
    a.bytes = bytes;
    a.stripes = stripes;
    a.scatter = scatter ? 1 : 0;
    LH_HIP(launch_ptr_copy(a, st));
    return kOk;
}

static int encode_batch_ptrs(int k, int m, int bytes, int stripes, uint8_t *const *data_ptrs, uint8_t *const *rec_ptrs,
                             hipStream_t st, bool allow_compile = true) {
    if (k < 1 || m < 1 || bytes <= 0 || stripes < 0 || k > 256 || m > 256)
        return fail(kInvalid, "invalid k, m, block_bytes or stripes");
    if (stripes == 0) return kOk;
    if (!data_ptrs || !rec_ptrs) return fail(kInvalid, "null pointer table");
    Device *d = nullptr;
    if (int rc = current_device(&d)) return rc;
    JitConfig cfg;
    if (jit_ptr_config_for(k, m, bytes, false, &cfg)) {
        std::string err;
        bool hard = false;
        const JitKernels *jk = jit_lookup(d, cfg, allow_compile, &err, &hard);
        if (jk) {
            const long long blocks = jit_blocks(cfg, stripes);
            if (blocks > 0x7FFFFFFF) return fail(kInvalid, "batch too large");
            long long in_stride = (long long)k * 8, out_stride = (long long)m * 8;
            int n = stripes;
            void *args[] = {(void *)&data_ptrs, &in_stride, (void *)&rec_ptrs, &out_stride, &n};
            LH_HIP(hipModuleLaunchKernel(jk->encode, (unsigned)blocks, 1, 1, 256, 1, 1, 0, st, args, nullptr));
            note_launch("lh_jit_encode(pointer table)");
            return kOk;
        }
        if (hard) return fail(kHipError, err);
    }
    if (jit_win_ptr_config_for(k, m, bytes, &cfg)) {
        std::string err;
        bool hard = false;
        const JitKernels *jk = jit_lookup(d, cfg, allow_compile, &err, &hard);
        if (jk && jk->encode_win) {
            const long long blocks = (long long)stripes * (cfg.sub / (64 * cfg.W));
            if (blocks > 0x7FFFFFFF) return fail(kInvalid, "batch too large");
            const unsigned threads = 64u * (unsigned)((m + cfg.rows_per_wave - 1) / cfg.rows_per_wave);
            long long in_stride = (long long)k * 8, out_stride = (long long)m * 8;
            int n = stripes;
            int bb = bytes;  // (windowed modules take the block size as an argument)
            void *args[] = {(void *)&data_ptrs, &in_stride, (void *)&rec_ptrs, &out_stride, &n, &bb};
            LH_HIP(hipModuleLaunchKernel(jk->encode_win, (unsigned)blocks, 1, 1, threads, 1, 1, 0, st, args, nullptr));
            note_launch("lh_jit_encode_win(pointer table)");
            return kOk;
        }
        if (hard) return fail(kHipError, err);
    }
    // Generic shapes (no specialised module, or one still compiling): the jump-table apply
    // reads the data blocks and writes the recovery blocks through the tables themselves.
    if (k > 1 && m > 1 && k + m <= 256 && bytes % 8 == 0 && bytes / 8 >= 4) {
        const uint8_t *G = nullptr;
        if (int rc = device_generator(d, k, m, &G, nullptr, st)) return rc;
        JumpApplyArgs a{};
        a.in_ptrs = data_ptrs;
        a.in_n = k;
        a.out_ptrs = rec_ptrs;
        a.out_n = m;
        a.coef = G;
        a.coef_stride = 0;
        a.n_in = k;
        a.n_out = m;
        a.bytes = bytes;
        a.sub = bytes / 8;
        a.stripes = stripes;
        a.per_stripe = 0;
        jump_layout(d, a, false);
        LH_HIP(launch_apply_jump(a, st));
        return kOk;
    }
    // Gather / strided encode / scatter, per chunk (m = 1, k = 1, sub < 4).  An invalid shape
    // (m > 1 with k + m > 256 or bytes % 8 != 0) still gets recovery block 0 first, as the
    // reference.
    const bool invalid = m > 1 && k > 1 && (k + m > 256 || bytes % 8 != 0);
    const long long per = (long long)(k + m) * bytes;
    uint8_t *buf = nullptr;
    int chunk = 0;
    if (int rc = gather_chunk(d, st, per, stripes, &buf, &chunk)) return rc;
    for (int s0 = 0; s0 < stripes; s0 += chunk) {
        const int n = std::min(chunk, stripes - s0);
        uint8_t *dat = buf, *rec = buf + (long long)n * k * bytes;
        if (int rc = ptr_copy(data_ptrs + (long long)s0 * k, k, k, dat, (long long)k * bytes, bytes, n, false, nullptr,
                              0, st))
            return rc;
        const int rc = encode_batch(k, m, bytes, n, dat, (long long)k * bytes, rec, (long long)m * bytes, st, allow_compile);
        if (rc != kOk && !(rc == kInvalid && invalid)) return rc;
        if (int rc = ptr_copy(rec_ptrs + (long long)s0 * m, m, invalid ? 1 : m, rec, (long long)m * bytes, bytes, n,
                              true, nullptr, 0, st))
            return rc;
    }
    return invalid ? fail(kInvalid, "k + m > 256 or block_bytes % 8 != 0") : kOk;
}

static int decode_batch_ptrs(int k, int m, int bytes, int stripes, uint8_t *const *block_ptrs, uint8_t *d_rows,
                             int8_t *d_status, hipStream_t st, bool allow_compile = true) {
    if (k < 1 || m < 1 || bytes <= 0 || stripes < 0 || k > 256 || m > 256)
        return fail(kInvalid, "invalid k, m, block_bytes or stripes");
    if (stripes == 0) return kOk;
    if (m > 1 && k > 1 && (k + m > 256 || bytes % 8 != 0))
        return fail(kInvalid, "k + m > 256 or block_bytes % 8 != 0");
    if (!block_ptrs || !d_rows) return fail(kInvalid, "null pointer table or rows");
    Device *d = nullptr;
    if (int rc = current_device(&d)) return rc;
    JitConfig cfg;
    if (k > 1 && m > 1 && jit_ptr_config_for(k, m, bytes, true, &cfg)) {
        std::string err;
        bool hard = false;
        const JitKernels *jk = jit_lookup(d, cfg, allow_compile, &err, &hard);
        if (hard) return fail(kHipError, err);
        if (jk) {
            if (jit_blocks(cfg, stripes) > 0x7FFFFFFF) return fail(kInvalid, "batch too large");
            const uint8_t *zero = nullptr;
            if (int rc = zero_page(d, (size_t)bytes, &zero, st)) return rc;
            long long s1 = (long long)k * 8;
            int n = stripes;
            if (jk->decode_fused && std::getenv("LONGHAIR_AMD_NO_FUSED_PLAN") == nullptr) {
                const uint8_t *gexp = d->gf_exp;
                const int16_t *glog = d->gf_log;
                void *args[] = {(void *)&block_ptrs, &s1, (void *)&d_rows, (void *)&d_status, (void *)&zero,
                                (void *)&gexp, (void *)&glog, &n};
                LH_HIP(hipModuleLaunchKernel(jk->decode_fused, (unsigned)jit_blocks(cfg, stripes), 1, 1, 256, 1, 1, 0,
                                             st, args, nullptr));
                note_launch("lh_jit_decode_fused(pointer table)");
                return kOk;
            }
            const int e_max = k < m ? k : m;
            const long long plan_stride = PlanView::bytes(k, m, e_max);
            Workspace *w = nullptr;
            if (int rc = run_planner(d, st, k, m, e_max, stripes, d_rows, d_status, 0, false, &w)) return rc;
            long long s2 = plan_stride;
            const uint8_t *plan = w->plan.ptr;
            void *args[] = {(void *)&block_ptrs, &s1, (void *)&plan, &s2, (void *)&zero, &n};
            LH_HIP(hipModuleLaunchKernel(jk->decode, (unsigned)jit_blocks(cfg, stripes), 1, 1, 256, 1, 1, 0, st, args,
                                         nullptr));
            note_launch("lh_jit_decode(pointer table)");
            return kOk;
        }
    }
    // Large m: the planner, the windowed phase A reading the slots through the table (V_r
    // back in place of R_r) and phase B through the same table.
    if (k > 1 && m > 1 && !jit_config_for(k, m, bytes, true, &cfg) && jit_win_ptr_config_for(k, m, bytes, &cfg, true)) {
        std::string err;
        bool hard = false;
        const JitKernels *wk = jit_lookup(d, cfg, allow_compile, &err, &hard);
        if (hard) return fail(kHipError, err);
        if (wk && wk->decode_wide) {
            const int e_max = k < m ? k : m;
            const long long plan_stride = PlanView::bytes(k, m, e_max);
            const long long cps = cfg.sub / (64 * cfg.W);
            if ((long long)stripes * cps > 0x7FFFFFFF) return fail(kInvalid, "batch too large");
            Workspace *w = nullptr;
            const uint8_t *zero = nullptr;
            if (int rc = zero_page(d, (size_t)bytes, &zero, st)) return rc;
            if (int rc = run_planner(d, st, k, m, e_max, stripes, d_rows, d_status, 0, false, &w)) return rc;
            const unsigned threads = 64u * (unsigned)((m + cfg.rows_per_wave - 1) / cfg.rows_per_wave);
            long long s1 = (long long)k * 8, s2 = plan_stride;
            const uint8_t *plan = w->plan.ptr;
            int n = stripes;
            int bb = bytes;  // (windowed modules take the block size as an argument)
            void *args[] = {(void *)&block_ptrs, &s1, (void *)&plan, &s2, (void *)&zero, &n, &bb};
            LH_HIP(hipModuleLaunchKernel(wk->decode_wide, (unsigned)(stripes * cps), 1, 1, threads, 1, 1, 0, st, args,
                                         nullptr));
            note_launch("lh_jit_decode_wide(pointer table)");
            InverseArgs ia{};
            ia.ptrs = block_ptrs;
            ia.plan = plan;
            ia.plan_stride = plan_stride;
            ia.k = k;
            ia.m = m;
            ia.e_max = e_max;
            ia.bytes = bytes;
            ia.stripes = stripes;
            ia.order = (int *)(w->plan.ptr + plan_order_offset(stripes, plan_stride));
            LH_HIP(launch_inverse(ia, st));
            return kOk;
        }
    }
    // Generic shapes: the planner, then the jump-table apply in place through the table (the
    // strided decode's rules: dword lanes from sub = 4, and the overlapping last lane of a
    // sub-block must share its neighbour's workgroup).
    if (k > 1 && m > 1) {
        const int sub = bytes / 8, jnch = (sub + 3) / 4;
        if (sub >= 4 && !(sub % 4 != 0 && jnch > 1 && (jnch - 1) % 64 == 0)) {
            const int e_max = k < m ? k : m;
            const long long plan_stride = PlanView::bytes(k, m, e_max);
            Workspace *w = nullptr;
            if (int rc = run_planner(d, st, k, m, e_max, stripes, d_rows, d_status, 0, true, &w)) return rc;
            JumpApplyArgs a{};
            a.in_ptrs = block_ptrs;
            a.out_ptrs = block_ptrs;
            a.in_n = k;
            a.out_n = k;
            a.coef = w->plan.ptr + PlanView::w_offset(k, m, e_max);
            a.coef_stride = plan_stride;
            a.plan = w->plan.ptr;
            a.plan_stride = plan_stride;
            a.n_in = k;
            a.n_out = e_max;
            a.bytes = bytes;
            a.sub = sub;
            a.stripes = stripes;
            a.per_stripe = 1;
            a.order = (int *)(w->plan.ptr + plan_order_offset(stripes, plan_stride));
            jump_layout(d, a, true);
            LH_HIP(launch_apply_jump(a, st));
            return kOk;
        }
    }
    // Gather / strided decode / scatter, per chunk (m = 1, k = 1, tiny or lone-tail blocks).
    // Only the slots the decode may have
    // changed go back, judged by the rows before the call (a copy of the chunk's rows rides
    // at the end of the chunk): for k, m > 1 the slots that held recovery rows (row >= k) of
    // the stripes it decoded (status 0); for m = 1 the one output slot of cauchy_decode_m1
    // (which may hold an original row, cauchy_256.cpp:487-535); k = 1: the single slot.
    const long long per = (long long)k * bytes + k;
    uint8_t *buf = nullptr;
    int chunk = 0;
    if (int rc = gather_chunk(d, st, per, stripes, &buf, &chunk)) return rc;
    const bool by_row = k > 1;
    for (int s0 = 0; s0 < stripes; s0 += chunk) {
        const int n = std::min(chunk, stripes - s0);
        uint8_t *blk = buf, *rows0 = buf + (long long)n * k * bytes;
        uint8_t *const *tab = block_ptrs + (long long)s0 * k;
        if (int rc = ptr_copy(tab, k, k, blk, (long long)k * bytes, bytes, n, false, nullptr, 0, st)) return rc;
        if (by_row) LH_HIP(hipMemcpyAsync(rows0, d_rows + (long long)s0 * k, (size_t)n * k, hipMemcpyDefault, st));
        if (int rc = decode_batch(k, m, bytes, n, blk, (long long)k * bytes, d_rows + (long long)s0 * k,
                                  d_status ? d_status + s0 : nullptr, st, allow_compile))
            return rc;
        if (int rc = ptr_copy(tab, k, k, blk, (long long)k * bytes, bytes, n, true, by_row ? rows0 : nullptr, k, st,
                              d_status ? d_status + s0 : nullptr, m == 1))
            return rc;
    }
    return kOk;
}

// -------------------------------------------------------------- drop-in helpers
// Where a drop-in block lives: host memory (pageable or pinned), memory the current device's
// kernels may address directly (its own allocations; managed memory), or another device's
// memory, which kernels here must not touch (no peer mapping is assumed) -- such blocks
// travel by hipMemcpyDefault, which the runtime routes as a peer copy.
enum PtrKind { kHostPtr, kLocalPtr, kRemotePtr };
static PtrKind pointer_kind(const void *p, int device) {
    hipPointerAttribute_t attr;
    if (hipPointerGetAttributes(&attr, p) != hipSuccess) {
        (void)hipGetLastError();
        return kHostPtr;
    }
    if (attr.type == hipMemoryTypeManaged) return kLocalPtr;
    if (attr.type != hipMemoryTypeDevice) return kHostPtr;
    return attr.device == device ? kLocalPtr : kRemotePtr;
}

// ----------------------------------------------------------- host-batch pipeline
// Stripes that start and end in host memory (packet buffers, files): chunks of stripes
// rotate over three streams, so chunk c + 1's host-to-device copy overlaps chunk c's
// kernels and chunk c - 1's device-to-host copy.  Host buffers should be pinned
// (hipHostMalloc / hipHostRegister) for the copies to be asynchronous.
static int pipe_streams(Device *d) {
    for (auto &s : d->pipe_stream)
        if (!s) LH_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    return kOk;
}

// On every exit from a host-batch call (errors included), wait for the three pipe
// streams: earlier chunks' asynchronous copies into or out of the caller's (pinned)
// buffers must not outlive the call.
struct PipeDrain {
    Device *d;
    ~PipeDrain() {
        for (auto s : d->pipe_stream)
            if (s) (void)hipStreamSynchronize(s);
    }
};

// Stripes per pipeline chunk: ~64 MiB for the encode; the decode's three kernels need
// larger launches to fill the GPU, so up to 256 MiB while keeping >= 4 chunks in flight
// (tools/pcie_bench.py PCIE_CHUNK sweep, shuffled slots: k200/m56 decode 39.1 GB/s at 5
// stripes per chunk, 43.3 at 10, 45.4 at 16; k29/m4 46.7 at 2048, 48.4 at 8192).
static int auto_chunk(long long stripe_bytes, int stripes, int chunk, bool decode = false) {
    if (chunk > 0) return chunk < stripes ? chunk : stripes;
    const long long sb = stripe_bytes > 0 ? stripe_bytes : 1;
    long long c = (64ll << 20) / sb;
    if (decode) {
        const long long big = (256ll << 20) / sb, quarter = ((long long)stripes + 3) / 4;
        c = std::max(c, std::min(big, quarter));
    }
    if (c < 1) c = 1;
    return (int)(c < stripes ? c : stripes);
}

// Chunk sizes of one pipelined call.  The last chunk's kernels and copy back run with the
// host-to-device link idle, so with automatic sizing the final stretch is cut into halving
// chunks (down to 1/8 of the regular size): the tail shrinks from one regular chunk's
// write-back (k29/m4 decode: ~0.7 ms of ~47) to a small one's, at the cost of a few more
// chunks.  An explicit chunk size is used as given.
static std::vector<int> chunk_list(int stripes, int chunk, bool tail) {
    std::vector<int> v;
    const int minc = std::max(1, chunk / 8);
    for (int rem = stripes; rem > 0;) {
        int n = rem < chunk ? rem : chunk;
        if (tail && rem <= 2 * chunk && rem > minc) n = std::max((rem + 1) / 2, minc);
        if (n > rem) n = rem;
        v.push_back(n);
        rem -= n;
    }
    return v;
}

static int host_encode_batch(int k, int m, int bytes, int stripes, const uint8_t *h_data, long long data_stride,
                             uint8_t *h_rec, long long rec_stride, int chunk) {
    if (k < 1 || m < 1 || bytes <= 0 || stripes < 0) return fail(kInvalid, "invalid k, m, block_bytes or stripes");
    if (data_stride < (long long)k * bytes || rec_stride < (long long)m * bytes)
        return fail(kInvalid, "stripe strides smaller than the stripe");
    if (stripes == 0) return kOk;
    Device *d = nullptr;
    if (int rc = current_device(&d)) return rc;
    std::lock_guard<std::mutex> g(d->pipe_mu);
    if (int rc = pipe_streams(d)) return rc;
    PipeDrain drain{d};
    const long long in_sz = (long long)k * bytes, out_sz = (long long)m * bytes;
    const bool tail = chunk <= 0;
    chunk = auto_chunk(in_sz + out_sz, stripes, chunk);
    const std::vector<int> sizes = chunk_list(stripes, chunk, tail);
    for (int i = 0; i < 3; ++i) {
        LH_HIP(d->pipe_blocks[i].reserve((size_t)chunk * in_sz));
        LH_HIP(d->pipe_out[i].reserve((size_t)chunk * out_sz));
    }
    int rc_all = kOk;
    const int nc = (int)sizes.size();
    std::vector<long long> first(nc);
    for (int c = 0, s0 = 0; c < nc; s0 += sizes[c], ++c) first[c] = s0;
    auto h2d = [&](int c) {
        return hipMemcpy2DAsync(d->pipe_blocks[c % 3].ptr, in_sz, h_data + first[c] * data_stride, data_stride, in_sz,
                                sizes[c], hipMemcpyHostToDevice, d->pipe_stream[c % 3]);
    };
    LH_HIP(h2d(0));
    for (int c = 0; c < nc; ++c) {
        const long long s0 = first[c];
        const int n = sizes[c];
        const int i = c % 3;
        hipStream_t st = d->pipe_stream[i];
        // The next chunk's host-to-device copy is enqueued before this chunk's kernel and
        // copy back (see host_decode_batch).
        if (c + 1 < nc) LH_HIP(h2d(c + 1));
        const int rc = encode_batch(k, m, bytes, n, d->pipe_blocks[i].ptr, in_sz, d->pipe_out[i].ptr, out_sz, st, true);
        if (rc != kOk && rc != kInvalid) return rc;
        if (rc == kInvalid) rc_all = kInvalid;
        const long long copy = rc == kOk ? out_sz : (long long)bytes;  // only block 0 on invalid params
        LH_HIP(hipMemcpy2DAsync(h_rec + (long long)s0 * rec_stride, rec_stride, d->pipe_out[i].ptr, out_sz, copy, n,
                                hipMemcpyDeviceToHost, st));
    }
    for (auto s : d->pipe_stream) LH_HIP(hipStreamSynchronize(s));
    return rc_all == kOk ? kOk : fail(kInvalid, "k + m > 256 or block_bytes % 8 != 0");
}

static int host_decode_batch(int k, int m, int bytes, int stripes, uint8_t *h_blocks, long long stride,
                             uint8_t *h_rows, int8_t *h_status, int chunk) {
    if (k < 1 || m < 1 || bytes <= 0 || stripes < 0) return fail(kInvalid, "invalid k, m, block_bytes or stripes");
    if (stride < (long long)k * bytes) return fail(kInvalid, "stripe stride smaller than the stripe");
    if (stripes == 0) return kOk;
    Device *d = nullptr;
    if (int rc = current_device(&d)) return rc;
    std::lock_guard<std::mutex> g(d->pipe_mu);
    if (int rc = pipe_streams(d)) return rc;
    PipeDrain drain{d};
    const long long sz = (long long)k * bytes;
    const bool tail = chunk <= 0;
    chunk = auto_chunk(sz, stripes, chunk, true);
    const std::vector<int> sizes = chunk_list(stripes, chunk, tail);
    // Only the slots decode can write travel back: the recovery slots (for m == 1 the
    // last one, or slot 0 when there is none: cauchy_decode_m1's quirk).  For k, m > 1 a
    // kernel writes exactly those blocks into the caller's pinned buffer through its
    // device mapping (lh_writeback_kernel); otherwise -- or when the buffer has no device
    // mapping, or LONGHAIR_AMD_PIPE_WRITEBACK=range -- one 2-D copy per chunk covers the
    // range [lo, hi] of such slots over the chunk's stripes (per-slot copies of small
    // blocks would be dominated by per-call overhead), which with recovery blocks spread
    // over the slots is most of the stripe.
    uint8_t *h_dev = nullptr;
    bool kernel_wb = k > 1 && m > 1;
    if (const char *e = std::getenv("LONGHAIR_AMD_PIPE_WRITEBACK")) kernel_wb = kernel_wb && std::string(e) != "range";
    if (((uintptr_t)h_blocks | (uintptr_t)stride | (uintptr_t)bytes) & 7) kernel_wb = false;  // 8-byte lanes
    if (kernel_wb && hipHostGetDevicePointer((void **)&h_dev, h_blocks, 0) != hipSuccess) {
        (void)hipGetLastError();
        kernel_wb = false;
    }
    for (int i = 0; i < 3; ++i) LH_HIP(d->pipe_blocks[i].reserve((size_t)chunk * sz));
    // The Block.row bytes and the status travel once per call, not per chunk: one copy in
    // (plus the device-side copy of the original rows the write-back kernel reads) before
    // the first chunk, one copy out after the last.  Per chunk, 3-4 small copies beside the
    // stripe data cost ~90 us each in the pipeline (profiles/r3l_pcie_chunk_sweep.json:
    // k29/m4 decode 48.0 GB/s at 1 024 stripes per chunk, 52.1 at 7 140) and kept the
    // chunks large, so the last chunk's kernels and write-back ran with the link idle.
    // Through pinned staging: a copy from pageable memory (numpy arrays, the status vector
    // callers typically allocate) is synchronous (profiles/r3_pcie_timeline.txt).
    const size_t nrows = (size_t)stripes * k;
    LH_HIP(d->pipe_rows.reserve(nrows));
    if (kernel_wb) LH_HIP(d->pipe_rows0.reserve(nrows));
    LH_HIP(d->pipe_status.reserve((size_t)stripes));
    LH_HIP(d->pipe_meta.reserve(nrows + (size_t)stripes));
    if (!d->pipe_meta_ev) LH_HIP(hipEventCreateWithFlags(&d->pipe_meta_ev, hipEventDisableTiming));
    uint8_t *prows = d->pipe_meta.ptr;
    int8_t *pstatus = (int8_t *)(prows + nrows);
    std::memcpy(prows, h_rows, nrows);
    {
        hipStream_t st0 = d->pipe_stream[0];
        LH_HIP(hipMemcpyAsync(d->pipe_rows.ptr, prows, nrows, hipMemcpyHostToDevice, st0));
        if (kernel_wb) LH_HIP(hipMemcpyAsync(d->pipe_rows0.ptr, d->pipe_rows.ptr, nrows, hipMemcpyDeviceToDevice, st0));
        LH_HIP(hipEventRecord(d->pipe_meta_ev, st0));
        for (int i = 1; i < 3; ++i) LH_HIP(hipStreamWaitEvent(d->pipe_stream[i], d->pipe_meta_ev, 0));
    }
    // Enqueue order: the host-to-device copy of chunk c + 1 before the kernels of chunk c.
    // Streams beyond the device's hardware queues (GPU_MAX_HW_QUEUES, 4 by default) share
    // one in FIFO order; enqueued after chunk c's write-back, chunk c + 1's copy on a stream
    // sharing chunk c's queue waited for that write-back with the link idle (~0.75 ms, once
    // every three chunks: rocprofv3 copy trace of tools/pcie_bench.py, session R).
    const int nc = (int)sizes.size();
    std::vector<long long> first(nc);
    for (int c = 0, s0 = 0; c < nc; s0 += sizes[c], ++c) first[c] = s0;
    auto h2d = [&](int c) {
        return hipMemcpy2DAsync(d->pipe_blocks[c % 3].ptr, sz, h_blocks + first[c] * stride, stride, sz, sizes[c],
                                hipMemcpyHostToDevice, d->pipe_stream[c % 3]);
    };
    LH_HIP(h2d(0));
    for (int c = 0; c < nc; ++c) {
        const long long s0 = first[c];
        const int n = sizes[c];
        const int i = c % 3;
        hipStream_t st = d->pipe_stream[i];
        if (c + 1 < nc) LH_HIP(h2d(c + 1));
        int lo = k, hi = -1;  // slot range [lo, hi] decode may write in this chunk
        if (k > 1 && !kernel_wb) {
            for (long long s = s0; s < s0 + n; ++s) {
                const uint8_t *r = h_rows + (long long)s * k;
                int first = -1, last = -1;  // first / last recovery slot of the stripe
                for (int x = 0; x < k; ++x) {
                    if (r[x] < k) continue;
                    if (first < 0) first = x;
                    last = x;
                }
                if (m == 1) first = last = (last < 0 ? 0 : last);  // the single output slot
                if (first < 0) continue;
                lo = first < lo ? first : lo;
                hi = last > hi ? last : hi;
            }
        }
        const int rc = decode_batch(k, m, bytes, n, d->pipe_blocks[i].ptr, sz, d->pipe_rows.ptr + (long long)s0 * k,
                                    (int8_t *)d->pipe_status.ptr + s0, st, true);
        if (rc != kOk) return rc;
        if (kernel_wb) {
            WritebackArgs wa{};
            wa.blocks = d->pipe_blocks[i].ptr;
            wa.stride = sz;
            wa.host = h_dev + (long long)s0 * stride;
            wa.host_stride = stride;
            wa.rows_orig = d->pipe_rows0.ptr + (long long)s0 * k;
            wa.k = k;
            wa.bytes = bytes;
            wa.stripes = n;
            LH_HIP(launch_writeback(wa, st));
        } else if (hi >= lo) {
            const long long off = (long long)lo * bytes, w = (long long)(hi - lo + 1) * bytes;
            LH_HIP(hipMemcpy2DAsync(h_blocks + (long long)s0 * stride + off, stride, d->pipe_blocks[i].ptr + off, sz, w,
                                    n, hipMemcpyDeviceToHost, st));
        }
    }
    for (auto s : d->pipe_stream) LH_HIP(hipStreamSynchronize(s));
    LH_HIP(hipMemcpy(prows, d->pipe_rows.ptr, nrows, hipMemcpyDeviceToHost));
    LH_HIP(hipMemcpy(pstatus, d->pipe_status.ptr, (size_t)stripes, hipMemcpyDeviceToHost));
    std::memcpy(h_rows, prows, nrows);
    if (h_status) std::memcpy(h_status, pstatus, (size_t)stripes);
    return kOk;
}

// ------------------------------------------------------------ drop-in dispatch
// Where a drop-in call (one stripe, the reference's call shape) runs.  kAuto (default):
// calls whose blocks all live in host memory and whose XOR work is at most
// g_host_max_work bytes run on the host SIMD engine (host_codec.cpp), the rest on the
// device -- a one-stripe call from host memory cannot amortise a PCIe round trip (k29/m4:
// ~35 us staged through the GPU against ~7 us on the host engine and ~9 us for the
// reference).  kGpu: always on the device.  kHost: every all-host-memory call on the host
// engine.  Device (or mixed) pointers always go to the device.  The library needs a GPU
// under every policy.
enum { kDispatchGpu = 0, kDispatchAuto = 1, kDispatchHost = 2 };

static int env_dispatch() {
    const char *e = std::getenv("LONGHAIR_AMD_DISPATCH");
    if (!e) return kDispatchAuto;
    const std::string v(e);
    return v == "gpu" ? kDispatchGpu : v == "host" ? kDispatchHost : kDispatchAuto;
}
static std::atomic<int> g_dispatch{env_dispatch()};
static std::atomic<long long> g_host_max_work{[] {
    const char *e = std::getenv("LONGHAIR_AMD_HOST_MAX_WORK");
    return e ? std::atoll(e) : (4ll << 20);
}()};

// Estimated XOR work of one call in bytes (terms x sub-block bytes), from the average
// density of a bit-matrix (32 of 64 bits): encode = rows 1..m-1 plus the row-0 XOR;
// decode = phase A over the k columns for e rows plus the e x e phase B.
static long long host_work(int k, int m, int e, int bytes, bool decode) {
    const long long sub = bytes / 8;
    if (!decode) return (32ll * k * (m - 1) + k) * sub;
    return 32ll * e * (k + e) * sub;
}

static bool want_host(long long work) {
    const int pol = g_dispatch.load(std::memory_order_relaxed);
    return pol == kDispatchHost || (pol == kDispatchAuto && work <= g_host_max_work.load(std::memory_order_relaxed));
}

// 1 if every pointer is host memory, 0 if every one is memory of `device` itself (the
// pointer-table form reads and writes it in place), -1 otherwise (mixed, or any block on
// another device: per-block hipMemcpyDefault staging).
static int classify(const void *const *ptrs, int n, const void *extra, int device) {
    int host = 0, local = 0;
    const int tot = n + (extra ? 1 : 0);
    for (int i = 0; i < tot; ++i) {
        const PtrKind kd = pointer_kind(i < n ? ptrs[i] : extra, device);
        host += kd == kHostPtr;
        local += kd == kLocalPtr;
    }
    return host == tot ? 1 : local == tot ? 0 : -1;
}

// Drop-in calls in a process without a HIP device (cauchy_256.cpp:390-399 initialises on any
// CPU): under the AUTO and HOST policies every call runs on the host SIMD engine; under GPU
// the call fails with -2.  Batch calls always need a device.
static bool host_only(int rc) {
    return rc == kNoDevice && g_dispatch.load(std::memory_order_relaxed) != kDispatchGpu;
}

// A free drop-in slot (the first whose lock is free), else the slot this thread hashes to,
// waited for.  Its stream is created on first use.
static int dropin_slot(Device *d, std::unique_lock<std::mutex> *lk, Device::DropinSlot **out) {
    Device::DropinSlot *s = nullptr;
    for (int i = 0; i < Device::kDropinSlots && !s; ++i) {
        std::unique_lock<std::mutex> l(d->dropin[i].mu, std::try_to_lock);
        if (l.owns_lock()) {
            *lk = std::move(l);
            s = &d->dropin[i];
        }
    }
    if (!s) {
        s = &d->dropin[std::hash<std::thread::id>{}(std::this_thread::get_id()) % Device::kDropinSlots];
        *lk = std::unique_lock<std::mutex>(s->mu);
    }
    if (!s->stream) LH_HIP(hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking));
    *out = s;
    return kOk;
}

static int dropin_encode(int k, int m, const unsigned char *data_ptrs[], void *recovery, int bytes) {
    if (k < 1 || m < 1 || bytes <= 0 || k > 256 || m > 256) return fail(kInvalid, "invalid k, m or block_bytes");
    Device *d = nullptr;
    const int drc = current_device(&d);
    if (drc && !host_only(drc)) return drc;
    const int where = drc ? 1 : classify((const void *const *)data_ptrs, k, recovery, d->id);
    if (drc || (where == 1 && want_host(k > 1 && m > 1 && k + m <= 256 && bytes % 8 == 0 ? host_work(k, m, 0, bytes, false) : 0))) {
        const int rc = host::encode(k, m, (const uint8_t *const *)data_ptrs, (uint8_t *)recovery, bytes);
        return rc == 0 ? kOk : fail(kInvalid, "k + m > 256 or block_bytes % 8 != 0");
    }
    std::unique_lock<std::mutex> g;
    Device::DropinSlot *sl = nullptr;
    if (int rc = dropin_slot(d, &g, &sl)) return rc;
    const size_t in_n = (size_t)k * bytes, out_n = (size_t)m * bytes;
    const size_t need = std::max(in_n + out_n, (size_t)(k + m) * 8);  // (the pointer table, all-device calls)
    LH_HIP(sl->stage.reserve(need));
    LH_HIP(sl->host_stage.reserve(need));
    hipStream_t st = sl->stream;
    if (where == 0) {
        // Every block in device memory: the pointer-table form reads them where they lie and
        // writes the recovery blocks in place -- one host-to-device copy of k + m pointers
        // instead of k + 1 block copies.
        LH_HIP(sl->ptab.reserve((size_t)(256 + 256) * 8 + 512));
        uint64_t *ht = (uint64_t *)sl->ptab.ptr;
        for (int x = 0; x < k; ++x) ht[x] = (uint64_t)(uintptr_t)data_ptrs[x];
        for (int r = 0; r < m; ++r) ht[k + r] = (uint64_t)(uintptr_t)((uint8_t *)recovery + (size_t)r * bytes);
        uint8_t *const *dt = (uint8_t *const *)sl->ptab.ptr;
        const int rc = encode_batch_ptrs(k, m, bytes, 1, dt, dt + k, st, false);
        LH_HIP(hipStreamSynchronize(st));
        return rc;
    }
    uint8_t *din = sl->stage.ptr, *dout = sl->stage.ptr + in_n;
    if (where == 1) {  // gather into pinned staging, one host-to-device copy
        for (int x = 0; x < k; ++x) std::memcpy(sl->host_stage.ptr + (size_t)x * bytes, data_ptrs[x], bytes);
        LH_HIP(hipMemcpyAsync(din, sl->host_stage.ptr, in_n, hipMemcpyHostToDevice, st));
    } else {  // device or mixed pointers: the runtime resolves each copy's direction
        for (int x = 0; x < k; ++x) LH_HIP(hipMemcpyAsync(din + (size_t)x * bytes, data_ptrs[x], bytes, hipMemcpyDefault, st));
    }
    const int rc = encode_batch(k, m, bytes, 1, din, (long long)in_n, dout, (long long)out_n, st, false);
    if (rc != kOk && rc != kInvalid) {
        (void)hipStreamSynchronize(st);
        return rc;
    }
    // On kInvalid only recovery block 0 was produced (reference behaviour).
    const size_t n = (rc == kOk) ? out_n : (size_t)bytes;
    if (where == 1) {
        LH_HIP(hipMemcpyAsync(sl->host_stage.ptr + in_n, dout, n, hipMemcpyDeviceToHost, st));
        LH_HIP(hipStreamSynchronize(st));
        std::memcpy(recovery, sl->host_stage.ptr + in_n, n);
    } else {
        LH_HIP(hipMemcpyAsync(recovery, dout, n, hipMemcpyDefault, st));
        LH_HIP(hipStreamSynchronize(st));
    }
    return rc;
}

static int dropin_decode(int k, int m, Block *blocks, int bytes) {
    if (k <= 1) {  // cauchy_256.cpp:1252-1256: the only block is the data
        if (k == 1) blocks[0].row = 0;
        return k == 1 ? kOk : fail(kInvalid, "k < 1");
    }
    if (m < 1 || bytes <= 0 || k > 256 || m > 256) return fail(kInvalid, "invalid m or block_bytes");
    int n_rcv = 0;
    for (int i = 0; i < k; ++i) n_rcv += blocks[i].row >= k;
    if (m > 1) {
        if (n_rcv == 0) return kOk;  // nothing erased (:1282-1284)
        if (k + m > 256 || bytes % 8 != 0) return fail(kInvalid, "k + m > 256 or block_bytes % 8 != 0");
    }
    Device *d = nullptr;
    const int drc = current_device(&d);
    if (drc && !host_only(drc)) return drc;
    const void *ptrs[256];
    for (int i = 0; i < k; ++i) ptrs[i] = blocks[i].data;
    const int where = drc ? 1 : classify(ptrs, k, nullptr, d->id);
    if (drc || (where == 1 && want_host(m == 1 ? (long long)k * bytes : host_work(k, m, n_rcv, bytes, true)))) {
        if (m == 1) {
            host::decode_m1(k, blocks, bytes);
            return kOk;
        }
        return host::decode(k, m, blocks, bytes) == 0 ? kOk : fail(kInvalid, "invalid or duplicated block rows");
    }
    std::unique_lock<std::mutex> g;
    Device::DropinSlot *sl = nullptr;
    if (int rc = dropin_slot(d, &g, &sl)) return rc;
    // Device and host staging share one layout: [k blocks][256 rows][16 status], so each
    // direction is a single copy for host pointers.
    const size_t in_n = (size_t)k * bytes, tot = in_n + 256 + 16;
    const size_t need = std::max(tot, (size_t)k * 8 + 256 + 16);  // (the pointer table, all-device calls)
    LH_HIP(sl->stage.reserve(need));
    LH_HIP(sl->host_stage.reserve(need));
    hipStream_t st = sl->stream;
    uint8_t *hs = sl->host_stage.ptr, *ds = sl->stage.ptr;
    if (where == 0) {
        // Every block in device memory: the pointer-table form decodes them in place -- one
        // copy of [k pointers][rows] in, one of [rows][status] out.
        LH_HIP(sl->ptab.reserve((size_t)(256 + 256) * 8 + 512));
        uint64_t *ht = (uint64_t *)sl->ptab.ptr;
        for (int i = 0; i < k; ++i) ht[i] = (uint64_t)(uintptr_t)blocks[i].data;
        uint8_t *hr = sl->ptab.ptr + (size_t)256 * 8;  // rows, then status at +256
        for (int i = 0; i < k; ++i) hr[i] = blocks[i].row;
        hr[256] = 0;
        const int rc = decode_batch_ptrs(k, m, bytes, 1, (uint8_t *const *)ht, hr, (int8_t *)(hr + 256), st, false);
        if (rc != kOk) {
            (void)hipStreamSynchronize(st);
            return rc;
        }
        LH_HIP(hipStreamSynchronize(st));
        if ((int8_t)hr[256] != 0) return fail(kInvalid, "invalid or duplicated block rows");
        for (int i = 0; i < k; ++i) blocks[i].row = hr[i];
        return kOk;
    }
    uint8_t *hrows = hs + in_n, *drows = ds + in_n;
    for (int i = 0; i < k; ++i) hrows[i] = blocks[i].row;
    if (where == 1) {
        for (int i = 0; i < k; ++i) std::memcpy(hs + (size_t)i * bytes, blocks[i].data, bytes);
        LH_HIP(hipMemcpyAsync(ds, hs, in_n + k, hipMemcpyHostToDevice, st));
    } else {
        for (int i = 0; i < k; ++i)
            LH_HIP(hipMemcpyAsync(ds + (size_t)i * bytes, blocks[i].data, bytes, hipMemcpyDefault, st));
        LH_HIP(hipMemcpyAsync(drows, hrows, k, hipMemcpyHostToDevice, st));
    }
    int rc = decode_batch(k, m, bytes, 1, ds, (long long)in_n, drows, (int8_t *)(drows + 256), st, false);
    if (rc != kOk) {
        (void)hipStreamSynchronize(st);
        return rc;
    }
    // Slots whose bytes can change: recovery slots (m > 1); for m == 1 the recovery slot
    // or, when none is present, slot 0 (cauchy_decode_m1's quirk).
    int changed[256], nch = 0;
    if (m == 1) {
        int out = 0;
        for (int i = 0; i < k; ++i) if (blocks[i].row >= k) out = i;
        changed[nch++] = out;
    } else {
        for (int i = 0; i < k; ++i) if (blocks[i].row >= k) changed[nch++] = i;
    }
    if (where == 1) {  // one copy back: blocks, rows, status
        LH_HIP(hipMemcpyAsync(hs, ds, tot, hipMemcpyDeviceToHost, st));
        LH_HIP(hipStreamSynchronize(st));
    } else {
        LH_HIP(hipMemcpyAsync(hrows, drows, 256 + 16, hipMemcpyDeviceToHost, st));
        LH_HIP(hipStreamSynchronize(st));
    }
    if ((int8_t)hrows[256] != 0) return fail(kInvalid, "invalid or duplicated block rows");
    if (where == 1) {
        for (int j = 0; j < nch; ++j) std::memcpy(blocks[changed[j]].data, hs + (size_t)changed[j] * bytes, bytes);
    } else {
        for (int j = 0; j < nch; ++j)
            LH_HIP(hipMemcpyAsync(blocks[changed[j]].data, ds + (size_t)changed[j] * bytes, bytes, hipMemcpyDefault, st));
        LH_HIP(hipStreamSynchronize(st));
    }
    for (int i = 0; i < k; ++i) blocks[i].row = hrows[i];
    return kOk;
}

}  // namespace lh

// =============================================================================== C ABI

#define LH_API __attribute__((visibility("default")))

// No C++ exception crosses the C ABI: every int-returning entry point runs
// inside LH_TRY / LH_CATCH, which turns any exception (std::bad_alloc from a vector or string,
// std::system_error from a background-compile thread, a runtime_error) into -3 with
// cauchy_256_last_error() naming it.
#define LH_TRY try { lh::test_hook();
#define LH_CATCH } catch (...) { return lh::internal_error(); }

extern "C" {

LH_API int _cauchy_256_init(int expected_version) {
    LH_TRY
        if (expected_version != CAUCHY_256_VERSION) return -1;  // cauchy_256.cpp:392-394
        (void)lh::Field::get();
        lh::Device *d = nullptr;
        const int rc = lh::current_device(&d);
        // No HIP device: the drop-in calls still work on the host engine unless the policy is
        // GPU (lh::host_only); cauchy_256_last_error() says which.
        if (lh::host_only(rc)) {
            lh::g_last_error = "longhair_amd: no HIP device; drop-in calls run on the host engine, batch calls return -2";
            return 0;
        }
        return rc;
    LH_CATCH
}

LH_API int cauchy_256_encode(int k, int m, const unsigned char *data_ptrs[], void *recovery_blocks, int block_bytes) {
    LH_TRY
        lh::LaunchTrace trace;
        return lh::dropin_encode(k, m, data_ptrs, recovery_blocks, block_bytes);
    LH_CATCH
}

LH_API int cauchy_256_decode(int k, int m, Block *blocks, int block_bytes) {
    LH_TRY
        lh::LaunchTrace trace;
        return lh::dropin_decode(k, m, blocks, block_bytes);
    LH_CATCH
}

LH_API int cauchy_256_encode_batch(int k, int m, int block_bytes, int stripes, const void *d_data, long long data_stride,
                            void *d_recovery, long long recovery_stride, void *stream) {
    LH_TRY
        lh::LaunchTrace trace;
        return lh::encode_batch(k, m, block_bytes, stripes, (const uint8_t *)d_data, data_stride, (uint8_t *)d_recovery,
                                recovery_stride, (hipStream_t)stream, true);
    LH_CATCH
}

LH_API int cauchy_256_decode_batch(int k, int m, int block_bytes, int stripes, void *d_blocks, long long stripe_stride,
                            unsigned char *d_rows, signed char *d_status, void *stream) {
    LH_TRY
        lh::LaunchTrace trace;
        return lh::decode_batch(k, m, block_bytes, stripes, (uint8_t *)d_blocks, stripe_stride, d_rows,
                                (int8_t *)d_status, (hipStream_t)stream, true);
    LH_CATCH
}

LH_API int cauchy_256_encode_batch_ptrs(int k, int m, int block_bytes, int stripes, const void *const *d_data_ptrs,
                                        void *const *d_recovery_ptrs, void *stream) {
    LH_TRY
        lh::LaunchTrace trace;
        return lh::encode_batch_ptrs(k, m, block_bytes, stripes, (uint8_t *const *)d_data_ptrs,
                                     (uint8_t *const *)d_recovery_ptrs, (hipStream_t)stream);
    LH_CATCH
}

LH_API int cauchy_256_decode_batch_ptrs(int k, int m, int block_bytes, int stripes, void *const *d_block_ptrs,
                                        unsigned char *d_rows, signed char *d_status, void *stream) {
    LH_TRY
        lh::LaunchTrace trace;
        return lh::decode_batch_ptrs(k, m, block_bytes, stripes, (uint8_t *const *)d_block_ptrs, d_rows,
                                     (int8_t *)d_status, (hipStream_t)stream);
    LH_CATCH
}

LH_API int cauchy_256_encode_host_batch(int k, int m, int block_bytes, int stripes, const void *h_data,
                                        long long data_stride, void *h_recovery, long long recovery_stride,
                                        int chunk_stripes) {
    LH_TRY
        lh::LaunchTrace trace;
        return lh::host_encode_batch(k, m, block_bytes, stripes, (const uint8_t *)h_data, data_stride,
                                     (uint8_t *)h_recovery, recovery_stride, chunk_stripes);
    LH_CATCH
}

LH_API int cauchy_256_decode_host_batch(int k, int m, int block_bytes, int stripes, void *h_blocks,
                                        long long stripe_stride, unsigned char *h_rows, signed char *h_status,
                                        int chunk_stripes) {
    LH_TRY
        lh::LaunchTrace trace;
        return lh::host_decode_batch(k, m, block_bytes, stripes, (uint8_t *)h_blocks, stripe_stride, h_rows,
                                     (int8_t *)h_status, chunk_stripes);
    LH_CATCH
}

LH_API int cauchy_256_batch_prepare_stream(int k, int m, int block_bytes, int max_stripes, void *stream) {
    LH_TRY
        lh::Device *d = nullptr;
        if (int rc = lh::current_device(&d)) return rc;
        std::string err;
        for (int dec = 0; dec < 2; ++dec) {
            lh::JitConfig cfg;
            if (lh::jit_config_for(k, m, block_bytes, dec == 1, &cfg) && !d->jit.get(cfg, &err))
                return lh::fail(lh::kHipError, err);
        }
        {
            lh::JitConfig cfg;
            if (!lh::jit_config_for(k, m, block_bytes, false, &cfg) && lh::jit_win_config_for(k, m, block_bytes, &cfg) &&
                !d->jit.get(cfg, &err))
                return lh::fail(lh::kHipError, err);
            if (!lh::jit_config_for(k, m, block_bytes, true, &cfg) && lh::jit_win_config_for(k, m, block_bytes, &cfg, true) &&
                !d->jit.get(cfg, &err))
                return lh::fail(lh::kHipError, err);
        }
        if (max_stripes > 0 && k > 1 && m > 1) {
            const int e_max = k < m ? k : m;
            lh::JitConfig cfg;
            const bool generic = !lh::jit_config_for(k, m, block_bytes, true, &cfg);
            lh::Workspace *w = nullptr;
            hipStream_t st = (hipStream_t)stream;
            if (int rc = lh::workspace(d, st,
                                       lh::plan_order_offset(max_stripes, lh::PlanView::bytes(k, m, e_max)) +
                                           (size_t)max_stripes * sizeof(int),
                                       generic ? (size_t)max_stripes * e_max * block_bytes : 0, &w))
                return rc;
            const uint8_t *G = nullptr, *z = nullptr;
            if (int rc = lh::zero_page(d, (size_t)block_bytes, &z, st)) return rc;
            if (int rc = lh::device_generator(d, k, m, &G, nullptr, st)) return rc;
        }
        return 0;
    LH_CATCH
}

LH_API int cauchy_256_batch_prepare_ptrs(int k, int m, int block_bytes) {
    LH_TRY
        lh::Device *d = nullptr;
        if (int rc = lh::current_device(&d)) return rc;
        std::string err;
        for (int dec = 0; dec < 2; ++dec) {
            lh::JitConfig cfg;
            const bool reg = lh::jit_config_for(k, m, block_bytes, dec == 1, &cfg);
            if (reg ? lh::jit_ptr_config_for(k, m, block_bytes, dec == 1, &cfg)
                    : lh::jit_win_ptr_config_for(k, m, block_bytes, &cfg, dec == 1))
                if (!d->jit.get(cfg, &err)) return lh::fail(lh::kHipError, err);
        }
        return 0;
    LH_CATCH
}

LH_API int cauchy_256_batch_prepare(int k, int m, int block_bytes, int max_stripes) {
    LH_TRY
        return cauchy_256_batch_prepare_stream(k, m, block_bytes, max_stripes, nullptr);
    LH_CATCH
}

LH_API const char *cauchy_256_last_launch(void) { return lh::g_last_launch.c_str(); }

// Compile the specialised code objects of a shape into the on-disk cache without a GPU
// (build-time warm-up for shapes whose compilation takes long).  0 ok, -3 on failure.
// LONGHAIR_AMD_PRECOMPILE_PART=enc|dec restricts it to the encode or decode modules, so
// a build can compile the two large-m modules of a shape in parallel processes.
LH_API int cauchy_256_jit_precompile(int k, int m, int block_bytes) {
    LH_TRY
        std::string err;
        std::vector<char> code;
        lh::JitConfig cfg;
        const char *part = std::getenv("LONGHAIR_AMD_PRECOMPILE_PART");
        for (int dec = 0; dec < 2; ++dec) {
            if (part && std::string(part) != (dec ? "dec" : "enc")) continue;
            if (lh::jit_config_for(k, m, block_bytes, dec == 1, &cfg)) {
                if (!lh::compile_code_object(cfg, &code, &err)) return lh::fail(lh::kHipError, err);
                // the (k, m) block-size family modules too (one per (k, m) and role, shared by every
                // block size), with LONGHAIR_AMD_PRECOMPILE_FAMILY=1
                const char *fam = std::getenv("LONGHAIR_AMD_PRECOMPILE_FAMILY");
                if (!cfg.family && fam && std::string(fam) == "1" &&
                    lh::jit_family_config_for(k, m, block_bytes, &cfg, dec == 1) &&
                    !lh::compile_code_object(cfg, &code, &err))
                    return lh::fail(lh::kHipError, err);
                // the pointer-table form (cauchy_256_*_batch_ptrs) as well, with LONGHAIR_AMD_PRECOMPILE_PTR=1
                const char *ptr = std::getenv("LONGHAIR_AMD_PRECOMPILE_PTR");
                if (ptr && std::string(ptr) == "1" && lh::jit_ptr_config_for(k, m, block_bytes, dec == 1, &cfg) &&
                    !lh::compile_code_object(cfg, &code, &err))
                    return lh::fail(lh::kHipError, err);
            } else if (lh::jit_win_config_for(k, m, block_bytes, &cfg, dec == 1)) {
                if (!lh::compile_code_object(cfg, &code, &err)) return lh::fail(lh::kHipError, err);
                const char *ptr = std::getenv("LONGHAIR_AMD_PRECOMPILE_PTR");
                if (ptr && std::string(ptr) == "1" && lh::jit_win_ptr_config_for(k, m, block_bytes, &cfg, dec == 1) &&
                    !lh::compile_code_object(cfg, &code, &err))
                    return lh::fail(lh::kHipError, err);
            }
        }
        return 0;
    LH_CATCH
}

LH_API int cauchy_256_batch_path(int k, int m, int block_bytes, int what) {
    LH_TRY
        lh::JitConfig cfg;
        if (what == 2 || what == 5)  // 1: the register network stages its columns by LDS-DMA (LH_LDS)
            return lh::jit_config_for(k, m, block_bytes, what == 5, &cfg) && cfg.lds ? 1 : 0;
        if (what == 8 || what == 9)  // 1: a block-size family module can serve the encode / decode (LH_FAMILY)
            return lh::jit_family_ok(k, m, block_bytes, what == 9) ? 1 : 0;
        if (what == 6 || what == 7) {  // the generic jump kernel's lane width (jump_layout)
            if (block_bytes <= 0 || block_bytes % 8 || block_bytes / 8 < 4) return 0;
            lh::Device *d = nullptr;
            if (int rc = lh::current_device(&d)) return rc;
            lh::JumpApplyArgs a{};
            a.sub = block_bytes / 8;
            a.n_out = what == 6 ? m : (k < m ? k : m);
            lh::jump_layout(d, a, what == 7);
            return a.dw;
        }
        if (!lh::jit_config_for(k, m, block_bytes, what == 1, &cfg)) {
            if (what == 0) return lh::jit_win_config_for(k, m, block_bytes, &cfg) ? 3 : 0;
            return lh::jit_win_config_for(k, m, block_bytes, &cfg, true) ? 4 : 0;
        }
        // Decode: 2 when the plan is computed inside the specialised kernel (jit_codec.hip,
        // LH_FUSED: e_max <= 4, one stripe per <= 64 lanes, k <= 64).
        const int e_max = k < m ? k : m;
        if (what == 1 && e_max <= 4 && cfg.nch <= 64 && k <= 64 && std::getenv("LONGHAIR_AMD_NO_FUSED_PLAN") == nullptr)
            return 2;
        return 1;
    LH_CATCH
}

LH_API int cauchy_256_frame_batch(int k, int m, int block_bytes, int stripes, const void *d_data,
                                  long long data_stride, const void *d_recovery, long long recovery_stride,
                                  void *d_packets, long long packet_stride, void *stream) {
    LH_TRY
        if (k < 1 || m < 0 || k + m > 256 || block_bytes <= 0 || stripes < 0 ||
            data_stride < (long long)k * block_bytes || (m > 0 && recovery_stride < (long long)m * block_bytes) ||
            packet_stride < (long long)(k + m) * (block_bytes + 1))
            return lh::fail(lh::kInvalid, "invalid framing parameters");
        lh::Device *d = nullptr;
        if (int rc = lh::current_device(&d)) return rc;
        lh::FrameArgs a{};
        a.data = (const uint8_t *)d_data;
        a.data_stride = data_stride;
        a.rec = (const uint8_t *)d_recovery;
        a.rec_stride = recovery_stride;
        a.packets = (uint8_t *)d_packets;
        a.packet_stride = packet_stride;
        a.k = k;
        a.m = m;
        a.bytes = block_bytes;
        a.stripes = stripes;
        a.npk = k + m;
        a.unframe = 0;
        if (hipError_t e = lh::launch_frame(a, (hipStream_t)stream))
            return lh::fail(lh::kHipError, std::string("frame: ") + hipGetErrorString(e));
        return 0;
    LH_CATCH
}

LH_API int cauchy_256_unframe_batch(int k, int block_bytes, int stripes, const void *d_packets,
                                    long long packet_stride, void *d_blocks, long long stripe_stride,
                                    unsigned char *d_rows, void *stream) {
    LH_TRY
        if (k < 1 || k > 256 || block_bytes <= 0 || stripes < 0 || packet_stride < (long long)k * (block_bytes + 1) ||
            stripe_stride < (long long)k * block_bytes)
            return lh::fail(lh::kInvalid, "invalid framing parameters");
        lh::Device *d = nullptr;
        if (int rc = lh::current_device(&d)) return rc;
        lh::FrameArgs a{};
        a.packets = (uint8_t *)d_packets;
        a.packet_stride = packet_stride;
        a.blocks = (uint8_t *)d_blocks;
        a.blocks_stride = stripe_stride;
        a.rows = d_rows;
        a.k = k;
        a.bytes = block_bytes;
        a.stripes = stripes;
        a.npk = k;
        a.unframe = 1;
        if (hipError_t e = lh::launch_frame(a, (hipStream_t)stream))
            return lh::fail(lh::kHipError, std::string("unframe: ") + hipGetErrorString(e));
        return 0;
    LH_CATCH
}

LH_API const char *cauchy_256_last_error(void) { return lh::g_last_error.c_str(); }

LH_API int cauchy_256_set_dispatch(int policy, long long host_max_work) {
    LH_TRY
        if (policy < lh::kDispatchGpu || policy > lh::kDispatchHost) return lh::fail(lh::kInvalid, "unknown dispatch policy");
        if (host_max_work >= 0) lh::g_host_max_work.store(host_max_work);
        return lh::g_dispatch.exchange(policy);
    LH_CATCH
}

LH_API int cauchy_256_get_dispatch(void) {
    LH_TRY
        return lh::g_dispatch.load();
    LH_CATCH
}

LH_API const char *cauchy_256_host_isa(void) { return lh::host::isa_name(); }

// Test-only (include/cauchy_256_test.h; the checked library only, LH_TEST_HOOKS): the
// calling thread's next guarded entry point throws inside its exception barrier, which must
// turn it into -3.  The product library does not export it.
#ifdef LH_TEST_HOOKS
LH_API void cauchy_256_debug_throw_next(void) { lh::g_throw_next = 1; }
#endif

}  // extern "C"
