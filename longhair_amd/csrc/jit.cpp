// jit.cpp -- hiprtc specialisation of jit_codec.hip per (k, m, bytes).
#include "jit.hpp"

#include <hip/hiprtc.h>

#include <cstdio>
#include <cstdlib>
#include <sstream>

#include "field.hpp"

extern "C" const char lh_jit_source[];

namespace lh {

namespace {
constexpr long long kMaxNetworkOnes = 24000;  // keeps the unrolled network in the I-cache
constexpr int kMaxAccDwords = 96;              // accumulator registers per lane
}  // namespace

long long generator_ones(int k, int m) {
    const std::vector<uint8_t> g = generator_matrix(k, m);
    long long ones = 0;
    for (uint8_t e : g) ones += __builtin_popcountll(bitmatrix(e));
    return ones;
}

bool jit_config_for(int k, int m, int bytes, bool decode, JitConfig *cfg) {
    if (const char *env = std::getenv("LONGHAIR_AMD_PATH")) {
        if (std::string(env) == "generic") return false;
    }
    if (k < 2 || m < 2 || k + m > 256 || bytes % 8 != 0 || bytes <= 0) return false;
    const int sub = bytes / 8;
    const int emax = k < m ? k : m;
    if (decode && (long long)emax * m > 64) return false;
    // Pick W (bytes per lane per sub-block): accumulators must fit the register budget;
    // among those prefer the best-packed waves, sub-dword words count at their fill.
    const int rows = decode ? m + 1 : m;  // decode also holds the Horner output
    int best_w = 0, best_nch = 0, spw = 0, wps = 0;
    double best_score = -1.0;
    for (int W : {16, 8, 4, 2, 1}) {
        if (W > sub || rows * 8 * ((W + 3) / 4) > kMaxAccDwords) continue;
        const int nch = (sub + W - 1) / W;
        double util;
        if (nch <= 64) {
            util = (double)((64 / nch) * nch) / 64.0;
        } else {
            if (decode && sub % W != 0) continue;  // a tail overlap would cross waves
            util = (double)nch / (double)(((nch + 63) / 64) * 64);
        }
        const double score = util * (W >= 4 ? 1.0 : W / 4.0);
        if (score > best_score + 0.02) {
            best_score = score;
            best_w = W;
            best_nch = nch;
        }
    }
    if (const char *fw = std::getenv("LONGHAIR_AMD_JIT_W")) {  // tuning override
        const int W = std::atoi(fw);
        if ((W == 1 || W == 2 || W == 4 || W == 8 || W == 16) && W <= sub &&
            rows * 8 * ((W + 3) / 4) <= 2 * kMaxAccDwords) {
            const int nch = (sub + W - 1) / W;
            if (!(nch > 64 && decode && sub % W != 0)) { best_w = W; best_nch = nch; }
        }
    }
    if (!best_w) return false;
    const int W = best_w, nch2 = best_nch;
    if (nch2 <= 64) spw = 64 / nch2;
    else wps = (nch2 + 63) / 64;
    if (generator_ones(k, m) > kMaxNetworkOnes) return false;
    cfg->k = k;
    cfg->m = m;
    cfg->bytes = bytes;
    cfg->sub = sub;
    cfg->W = W;
    cfg->nch = nch2;
    cfg->spw = spw;
    cfg->wps = wps;
    cfg->defines.clear();
    if (const char *d = std::getenv("LONGHAIR_AMD_JIT_DEFINES")) cfg->defines = d;
    return true;
}

std::string jit_source_for(const JitConfig &c) {
    std::ostringstream os;
    // Tuning knobs "NAME=VALUE" separated by spaces or commas.
    {
        std::string tok;
        for (char ch : c.defines + " ") {
            if (ch == ' ' || ch == ',') {
                const size_t eq = tok.find('=');
                if (!tok.empty()) os << "#define " << (eq == std::string::npos ? tok : tok.substr(0, eq) + " " + tok.substr(eq + 1)) << "\n";
                tok.clear();
            } else {
                tok += ch;
            }
        }
    }
    os << "#define LH_K " << c.k << "\n#define LH_M " << c.m << "\n#define LH_BYTES " << c.bytes
       << "\n#define LH_SUB " << c.sub << "\n#define LH_W " << c.W << "\n#define LH_NCH " << c.nch
       << "\n#define LH_SPW " << (c.spw ? c.spw : 1) << "\n#define LH_WPS " << (c.wps ? c.wps : 1) << "\n";
    const std::vector<uint8_t> g = generator_matrix(c.k, c.m);
    os << "static constexpr unsigned char LH_BM[" << c.m << "][" << c.k << "][8] = {";
    for (int r = 0; r < c.m; ++r) {
        os << "{";
        for (int x = 0; x < c.k; ++x) {
            const uint64_t bm = bitmatrix(g[(size_t)r * c.k + x]);
            os << "{";
            for (int y = 0; y < 8; ++y) os << (unsigned)((bm >> (8 * y)) & 0xFF) << (y < 7 ? "," : "");
            os << "}" << (x + 1 < c.k ? "," : "");
        }
        os << "}" << (r + 1 < c.m ? "," : "");
    }
    os << "};\n";
    os << "#define LH_G_INIT {";
    for (int r = 0; r < c.m; ++r) {
        os << "{";
        for (int x = 0; x < c.k; ++x) os << (unsigned)g[(size_t)r * c.k + x] << (x + 1 < c.k ? "," : "");
        os << "}" << (r + 1 < c.m ? "," : "");
    }
    os << "}\n";
    os << lh_jit_source;
    return os.str();
}

const JitKernels *JitCache::peek(const JitConfig &cfg) {
    std::lock_guard<std::mutex> g(mu_);
    auto it = cache_.find(Key(cfg.k, cfg.m, cfg.bytes, cfg.W, cfg.defines));
    return it == cache_.end() ? nullptr : &it->second;
}

const JitKernels *JitCache::get(const JitConfig &cfg, std::string *err) {
    std::lock_guard<std::mutex> g(mu_);
    const Key key(cfg.k, cfg.m, cfg.bytes, cfg.W, cfg.defines);
    auto it = cache_.find(key);
    if (it != cache_.end()) return &it->second;

    const std::string src = jit_source_for(cfg);
    hiprtcProgram prog;
    if (hiprtcCreateProgram(&prog, src.c_str(), "lh_jit_codec.hip", 0, nullptr, nullptr) != HIPRTC_SUCCESS) {
        *err = "hiprtcCreateProgram failed";
        return nullptr;
    }
    const char *opts[] = {"--offload-arch=gfx950", "-O3", "-std=c++17"};
    const hiprtcResult rc = hiprtcCompileProgram(prog, 3, opts);
    if (rc != HIPRTC_SUCCESS) {
        size_t n = 0;
        hiprtcGetProgramLogSize(prog, &n);
        std::string log(n + 1, '\0');
        hiprtcGetProgramLog(prog, &log[0]);
        *err = "hiprtc compile failed: " + log;
        hiprtcDestroyProgram(&prog);
        return nullptr;
    }
    size_t code_size = 0;
    hiprtcGetCodeSize(prog, &code_size);
    std::vector<char> code(code_size);
    hiprtcGetCode(prog, code.data());
    hiprtcDestroyProgram(&prog);

    JitKernels kern;
    kern.cfg = cfg;
    if (hipModuleLoadData(&kern.module, code.data()) != hipSuccess ||
        hipModuleGetFunction(&kern.encode, kern.module, "lh_jit_encode") != hipSuccess ||
        hipModuleGetFunction(&kern.decode, kern.module, "lh_jit_decode") != hipSuccess) {
        *err = "hipModuleLoadData/GetFunction failed for the specialised kernels";
        return nullptr;
    }
    if (hipModuleGetFunction(&kern.encode_dma, kern.module, "lh_jit_encode_dma") != hipSuccess) {
        (void)hipGetLastError();
        kern.encode_dma = nullptr;
    }
    if (hipModuleGetFunction(&kern.decode_fused, kern.module, "lh_jit_decode_fused") != hipSuccess) {
        (void)hipGetLastError();
        kern.decode_fused = nullptr;
    }
    auto res = cache_.emplace(key, kern);
    return &res.first->second;
}

}  // namespace lh
