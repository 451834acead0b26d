// jit.hpp -- run-time specialisation of the XOR network per (k, m, bytes).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <map>
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
    int win_lds = 1;      // windowed modules: stage column tiles in LDS by LDS-DMA (0: per-wave loads)
    int win_split = 1;    // windowed decode: phase A writes V in place, lh_inverse_kernel does phase B
                          // (0: the fused kernel, phase B from an LDS tile of V)
    int lanes_per_launch_unit() const { return 64; }
};

struct JitKernels {
    hipModule_t module = nullptr;
    hipFunction_t encode = nullptr;
    hipFunction_t decode = nullptr;
    hipFunction_t decode_fused = nullptr;  // plan computed in-kernel (e_max <= 4)
    hipFunction_t encode_win = nullptr;    // windowed large-m encode (win modules)
    hipFunction_t decode_wide = nullptr;   // fused windowed decode (win == 2 modules, m <= 64)
    JitConfig cfg{};
};

// Chooses the specialised configuration for a shape, or returns false when the shape
// is served by the generic kernel (too many recovery rows for the register budget, or
// a network too large for the instruction cache).
bool jit_config_for(int k, int m, int bytes, bool decode, JitConfig *cfg);

// Windowed large-m encode configuration (m too large for the register-resident network).
bool jit_win_config_for(int k, int m, int bytes, JitConfig *cfg, bool decode = false);

// Number of ones in the expanded generator (= XORs of the straight-line network).
long long generator_ones(int k, int m);

class JitCache {
public:
    // Returns compiled kernels for the configuration (compiling on first use).  On
    // failure returns nullptr and fills *err.  compile = false: only a module already in
    // memory or in the on-disk cache (nullptr, *err = "not cached", when there is none).
    const JitKernels *get(const JitConfig &cfg, std::string *err, bool compile = true);
    // Only returns an already compiled entry (no compilation).
    const JitKernels *peek(const JitConfig &cfg);

private:
    using Key = std::tuple<int, int, int, int, std::string, int>;
    std::mutex mu_;
    std::map<Key, JitKernels> cache_;
    std::map<Key, bool> not_cached_;  // lookups without compilation that found no module
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

}  // namespace lh
