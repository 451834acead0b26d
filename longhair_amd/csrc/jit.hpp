// jit.hpp -- run-time specialisation of the XOR network per (k, m, bytes).
#pragma once

#include <hip/hip_runtime.h>

#include <condition_variable>
#include <cstdint>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <tuple>
#include <vector>

namespace lh {

struct JitConfig {
    int k, m, bytes, sub;
    int W;     // bytes per lane per sub-block
    int nch;   // lanes per stripe = ceil(sub / W)
    int spw;   // stripes per wave (nch <= 64) or 0
    int wps;   // waves per stripe (nch > 64) or 0
    std::string defines;  // extra -D style tuning knobs (LONGHAIR_AMD_JIT_DEFINES)
    int win = 0;          // 1: windowed encode module, 2: windowed decode phase-A module
    int rows_per_wave = 8;
    int win_pf = 3;       // windowed modules: columns in flight ahead of the one combined
    int win_lds = 1;      // windowed modules: column tiles staged in LDS by LDS-DMA (the only form since round 5)
    int win_split = 1;    // windowed decode: phase A writes V in place, lh_inverse_gt_kernel does phase B
                          // (0: the fused kernel, phase B from an LDS tile of V)
    int ptr = 0;          // register networks: blocks addressed through a pointer table (LH_PTR,
                          // cauchy_256_*_batch_ptrs)
    int lds = 0;          // register networks: columns staged by LDS-DMA (LH_LDS, jit_codec.hip)
    int role = 0;         // register networks: 1 = the encode module (lh_jit_encode only),
                          // 2 = the decode module: lh_jit_decode_fused, or lh_jit_decode when
                          // the fused plan does not apply or is switched off (plain = 1)
    int plain = 0;
    int wgcu = 0;         // register networks: resident workgroups per CU of the module's kernel,
                          // forced by dynamic LDS (0: natural)
    int cps = 1;          // LDS encode of strided batches: columns per DMA step (LH_CPS)
    int family = 0;       // the block-size family module (LH_FAMILY: one module per (k, m)
                          // serves every qualifying block size, which the kernel takes as an argument)
    int enc_wpb = 4;      // encode: waves per workgroup (LH_WPB, multi-column-step encode only)
    int dec_wpb = 4;      // fused decode of strided batches: waves per workgroup (LH_DWPB)
    int lanes_per_launch_unit() const { return 64; }
};

struct JitKernels {
    hipModule_t module = nullptr;
    hipFunction_t encode = nullptr;
    hipFunction_t decode = nullptr;
    hipFunction_t decode_fused = nullptr;  // plan computed in-kernel (e_max <= 4)
    hipFunction_t encode_win = nullptr;    // windowed large-m encode (win modules)
    hipFunction_t decode_wide = nullptr;   // fused windowed decode (win == 2 modules, m <= 64)
    unsigned dyn_lds = 0;                  // dynamic LDS bytes per launch of the module's kernel (cfg.wgcu)
    JitConfig cfg{};
};

// Chooses the specialised configuration for a shape, or returns false when the shape
// is served by the generic kernel (too many recovery rows for the register budget, or
// a network too large for the instruction cache).
bool jit_config_for(int k, int m, int bytes, bool decode, JitConfig *cfg);

// The pointer-table form of a register-network configuration (cauchy_256_*_batch_ptrs):
// false when the shape has none (no register network, or a wave's stripes hold more block
// pointers than its LDS share: spw * k > 1024).
bool jit_ptr_config_for(int k, int m, int bytes, bool decode, JitConfig *cfg);

// Windowed large-m encode configuration (m too large for the register-resident network).
bool jit_win_config_for(int k, int m, int bytes, JitConfig *cfg, bool decode = false);
// Its pointer-table form (LDS-staged columns, split decode).
bool jit_win_ptr_config_for(int k, int m, int bytes, JitConfig *cfg, bool decode = false);

// Number of ones in the expanded generator (= XORs of the straight-line network).
long long generator_ones(int k, int m);

// Whether the encode's block-size family module (one per (k, m), the block size a kernel
// argument; jit_codec.hip LH_FAMILY) can serve (k, m, bytes).
// decode: the fused, LDS-staged decode's family (e_max <= 4, k <= 64, at least ceil(k / 8)
// lanes per stripe).
bool jit_family_ok(int k, int m, int bytes, bool decode = false);
// The family module's configuration for (k, m, bytes), when jit_family_ok.  Batch and drop-in
// encodes take it when the size-specialised module is neither loaded nor cached: one cached
// module per (k, m) serves every qualifying block size at near-specialised speed (k29/m4
// encode 0.528 against 0.489 ms) instead of the generic kernels (0.665 ms).
bool jit_family_config_for(int k, int m, int bytes, JitConfig *cfg, bool decode = false);

// How a lookup may obtain a module that is neither loaded nor in the on-disk cache.
enum class JitMode {
    kCached,    // not at all: nullptr, *err = "not cached" (drop-in calls)
    kAsync,     // start hiprtc on a background thread and return nullptr at once; the
                // caller serves the call with the generic kernels, a later lookup loads
                // the module once it is compiled (batch calls, the default)
    kBlocking,  // compile now (or wait for the compile in flight) and load it
                // (cauchy_256_batch_prepare*, LONGHAIR_AMD_JIT_SYNC=1)
};

class JitCache {
public:
    // Kernels of the configuration, obtained as `mode` allows.  nullptr with *err filled
    // when there is no module (yet); *failed (optional) is set when a compilation of this
    // configuration failed.  No lock is held while hiprtc runs: lookups of other shapes
    // (and of this one, in kAsync / kCached mode) proceed meanwhile.
    const JitKernels *get(const JitConfig &cfg, std::string *err, JitMode mode, bool *failed = nullptr);
    const JitKernels *get(const JitConfig &cfg, std::string *err) { return get(cfg, err, JitMode::kBlocking); }
    // Only returns an already loaded entry.
    const JitKernels *peek(const JitConfig &cfg);

private:
    using Key = std::tuple<int, int, int, int, std::string, int>;
    // A compilation in flight (or finished, not yet loaded); shared with its worker thread,
    // which touches nothing else of the cache.
    struct Pending {
        std::mutex mu;
        std::condition_variable cv;
        bool done = false, ok = false;
        std::vector<char> code;
        std::string err;
    };
    static Key key_of(const JitConfig &cfg);
    const JitKernels *load_locked(const Key &key, const JitConfig &cfg, std::vector<char> &code, std::string *err);
    std::mutex mu_;
    std::map<Key, JitKernels> cache_;
    std::map<Key, bool> not_cached_;                  // kCached lookups that found no module
    std::map<Key, std::shared_ptr<Pending>> pending_;  // compilations in flight / not yet loaded
    std::map<Key, std::string> failed_;               // compilations that failed (not retried)
};

std::string jit_source_for(const JitConfig &cfg);

// Compile (or fetch from the on-disk cache) the code object of a configuration.  Needs
// no GPU, so build steps can pre-populate the cache.
// fresh: ignore (and delete) a cached object.
// compile = false: only read the on-disk cache (false, *err = "not cached", if absent).
bool compile_code_object(const JitConfig &cfg, std::vector<char> *code, std::string *err, bool fresh = false,
                         bool compile = true);

// True unless LONGHAIR_AMD_JIT_COMPILE=0: batch calls may run hiprtc for a shape whose
// specialised module is not cached (drop-in calls never do).
bool jit_compile_allowed();

// How batch calls obtain a missing module: kAsync by default, kBlocking with
// LONGHAIR_AMD_JIT_SYNC=1, kCached with LONGHAIR_AMD_JIT_COMPILE=0.
JitMode batch_jit_mode();

// Waits for every background compilation to finish (also run at process exit).
void jit_join_background();

}  // namespace lh
