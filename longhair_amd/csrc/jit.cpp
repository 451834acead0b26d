// jit.cpp -- hiprtc specialisation of jit_codec.hip per (k, m, bytes).
#include "jit.hpp"

#include <hip/hiprtc.h>
#include <dlfcn.h>
#include <sys/stat.h>
#include <unistd.h>
#include <utime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <functional>
#include <sstream>
#include <thread>

#include "field.hpp"

extern "C" const char lh_jit_source[];
extern "C" const char lh_inv_jump_source[];  // inv_jump.inc (blobs.cpp)

namespace lh {

namespace {
constexpr long long kMaxNetworkOnes = 24000;  // keeps the unrolled network in the I-cache
constexpr int kMaxAccDwords = 96;              // accumulator registers per lane
constexpr int kMaxJitColumns = 128;            // data columns of a register-resident network
}  // namespace

long long generator_ones(int k, int m) {
    const std::vector<uint8_t> g = generator_matrix(k, m);
    long long ones = 0;
    for (uint8_t e : g) ones += __builtin_popcountll(bitmatrix(e));
    return ones;
}

// The encode's block-size family serves (k, m, bytes) when: 16-byte-multiple blocks, 8-byte
// lanes with at most 64 per stripe (bytes <= 4096), the 8 x m accumulator words of 8-byte
// lanes within the register budget (m <= 6), at least two steps of columns (k >= 4), and, when
// the last lane of a stripe holds a partial word, every stripe's last lane in the same DPP row
// of 16 as its neighbour (its stores funnel that lane's word).
// The decode's family (jit_codec.hip, decode block-size family): the fused plan's shapes
// (e_max = min(k, m) <= 4, k <= 64) with at most 8 Block.row bytes per lane (nch >= ceil(k / 8)).
bool jit_family_ok(int k, int m, int bytes, bool decode) {
    if (decode ? (k < 2 || std::min(k, m) > 4 || k > 64) : k < 4) return false;
    if (m < 2 || k + m > 256 || k > kMaxJitColumns || bytes <= 0 || bytes % 16 != 0) return false;
    if (m * 8 * 2 > kMaxAccDwords) return false;
    const int sub = bytes / 8, nch = (sub + 7) / 8;
    if (nch > 64 || (decode && nch < (k + 7) / 8)) return false;
    const int spw = 64 / nch;
    if (sub - 8 * (nch - 1) != 8)
        for (int s = 0; s < spw; ++s)
            if ((s * nch + nch - 1) % 16 == 0) return false;
    return generator_ones(k, m) <= kMaxNetworkOnes;
}

static bool config_impl(int k, int m, int bytes, bool decode, JitConfig *cfg, bool allow_family);

bool jit_config_for(int k, int m, int bytes, bool decode, JitConfig *cfg) {
    return config_impl(k, m, bytes, decode, cfg, true);
}

static bool config_impl(int k, int m, int bytes, bool decode, JitConfig *cfg, bool allow_family) {
    if (const char *env = std::getenv("LONGHAIR_AMD_PATH")) {
        if (std::string(env) == "generic") return false;
    }
    if (k < 2 || m < 2 || k + m > 256 || bytes % 8 != 0 || bytes <= 0) return false;
    // k > 128 with few rows: the generic kernel.  Its straight-line network of > 128
    // columns took hiprtc ~7 minutes per module (k250/m3) for a shape outside the
    // benchmarked configurations.
    if (k > kMaxJitColumns) return false;
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
    // LDS-DMA column staging (jit_codec.hip LH_LDS): 8-byte lanes, whole stripes per wave,
    // 16-byte-multiple blocks (a DMA chunk never spans two blocks) and, when the last chunk
    // of a sub-block is partial, every stripe's last lane in the same 16-lane DPP row as its
    // neighbour (its stores funnel that lane's word through row_shr:1).
    cfg->lds = 0;
    if (W == 8 && nch2 <= 64 && bytes % 16 == 0) {
        bool dpp_ok = true;
        if (sub - 8 * (nch2 - 1) != 8)
            for (int s = 0; s < spw; ++s) dpp_ok = dpp_ok && (s * nch2 + nch2 - 1) % 16 != 0;
        cfg->lds = dpp_ok ? 1 : 0;
        // The encode's LDS also holds its stripes' block-pointer rows (spw x (k + m) x 8 bytes
        // per wave): keep ring plus rows within two workgroups per CU.
        const long long lq = ((long long)spw * bytes + 1023) / 1024;
        if (!decode && 4 * (4 * lq * 1024 + 16) + 4ll * spw * (k + m) * 8 > 80 * 1024) cfg->lds = 0;
    }
    // One role per module: an encode module holds lh_jit_encode only, a decode module the one
    // decode kernel its calls launch (the fused plan for e_max <= 4, one stripe per <= 64
    // lanes, k <= 64, unless LONGHAIR_AMD_NO_FUSED_PLAN).  A module with all three compiled
    // three copies of the network (six when encode and decode pick different lane widths,
    // as m = 3 does), of which a call uses one.
    cfg->role = decode ? 2 : 1;
    cfg->plain = decode && !(emax <= 4 && nch2 <= 64 && k <= 64 && std::getenv("LONGHAIR_AMD_NO_FUSED_PLAN") == nullptr);
    cfg->defines.clear();
    if (const char *d = std::getenv("LONGHAIR_AMD_JIT_DEFINES")) cfg->defines = d;
    // The LDS encode of strided batches fetches LH_CPS = 5 columns per DMA step (one step in
    // flight) and runs one 4-wave workgroup per CU (dynamic LDS pads the rest): k29/m4 encode
    // 0.502-0.509 -> 0.489-0.491 ms against the one-column ring at two workgroups per CU
    // (profiles/r9e_tune_k29m4_cps.txt; 3 columns 0.496, 4: 0.501, 6: 0.498, 7: 0.513; two
    // workgroups per CU 0.534; jit_codec.hip LH_CPS).  At least two steps (k >= 4).
    // Tuning overrides in LONGHAIR_AMD_JIT_DEFINES: LH_CPS=, LH_WGCU=, LH_WPB=.
    auto knob = [&](const char *name, int dflt) {
        const size_t at = cfg->defines.find(name);
        return at == std::string::npos ? dflt : std::atoi(cfg->defines.c_str() + at + std::strlen(name));
    };
    // The fused decode's memory-order form (jit_codec.hip LH_DMO) streams slots in the same
    // multi-slot steps.
    const bool dmo = decode && cfg->lds && !cfg->plain && knob("LH_DMO=", 0) == 1;
    cfg->cps = 1;
    if ((!decode || dmo) && cfg->lds) cfg->cps = std::max(1, std::min(5, k / 2));
    cfg->cps = knob("LH_CPS=", cfg->cps);
    if (cfg->cps > 1 && !((!decode || dmo) && cfg->lds && k >= 2 * cfg->cps)) cfg->cps = 1;
    cfg->wgcu = knob("LH_WGCU=", cfg->cps > 1 ? 1 : 0);
    const int wpb = knob("LH_WPB=", 4);
    cfg->enc_wpb = (cfg->cps > 1 && wpb >= 1 && wpb <= 8) ? wpb : 4;
    const int dwpb = knob("LH_DWPB=", 4);
    cfg->dec_wpb = (decode && !cfg->plain && dwpb >= 1 && dwpb <= 8) ? dwpb : 4;
    // Block-size family (jit_codec.hip LH_FAMILY): the multi-column-step encode with the block
    // size a kernel argument, keyed by (k, m) alone.
    cfg->family = 0;
    // (LH_FAMILY=1, tests: the family module even where a size-specialised one would serve)
    if (allow_family && knob("LH_FAMILY=", 0) && jit_family_config_for(k, m, bytes, cfg, decode)) return true;
    return true;
}

bool jit_family_config_for(int k, int m, int bytes, JitConfig *cfg, bool decode) {
    if (const char *env = std::getenv("LONGHAIR_AMD_PATH")) {
        if (std::string(env) == "generic") return false;
    }
    if (!jit_family_ok(k, m, bytes, decode)) return false;
    if (decode && std::getenv("LONGHAIR_AMD_NO_FUSED_PLAN") != nullptr) return false;
    JitConfig c;
    c.k = k;
    c.m = m;
    c.bytes = bytes;
    c.sub = bytes / 8;
    c.W = 8;
    c.nch = (c.sub + 7) / 8;
    c.spw = 64 / c.nch;
    c.wps = 0;
    c.lds = 1;
    c.role = decode ? 2 : 1;
    c.plain = 0;
    c.family = 1;
    if (const char *d = std::getenv("LONGHAIR_AMD_JIT_DEFINES")) c.defines = d;
    auto knob = [&](const char *name, int dflt) {
        const size_t at = c.defines.find(name);
        return at == std::string::npos ? dflt : std::atoi(c.defines.c_str() + at + std::strlen(name));
    };
    c.cps = std::max(2, std::min(5, k / 2));
    // (tuning knobs that switch off what the family kernel is made of leave it out)
    if (knob("LH_LDS=", 1) == 0 || knob("LH_CPS=", c.cps) < 2 || knob("LH_WPB=", 4) != 4) return false;
    c.wgcu = knob("LH_WGCU=", decode ? 0 : 1);  // (the decode: two workgroups per CU, as its size-specialised form)
    c.enc_wpb = 4;
    *cfg = c;
    return true;
}

bool jit_ptr_config_for(int k, int m, int bytes, bool decode, JitConfig *cfg) {
    if (!config_impl(k, m, bytes, decode, cfg, false)) return false;
    // (the multi-column steps read a stripe's columns as one contiguous run: strided batches only)
    cfg->cps = 1;
    cfg->enc_wpb = 4;
    if (cfg->defines.find("LH_WGCU=") == std::string::npos) cfg->wgcu = 0;
    if ((long long)(cfg->spw ? cfg->spw : 1) * k > 1024) return false;  // LDS: 4 waves x 8 B x spw x (k + 1) <= 35 KiB
    cfg->ptr = 1;
    // LDS staging as for strided batches (the encode's pointer rows already counted by
    // jit_config_for); the fused decode's rows (its plan scratch shares the budget) at most
    // 4 KiB.
    const long long spw = cfg->spw ? cfg->spw : 1;
    if (decode && 4 * spw * (k + 1) * 8 > 4096) cfg->lds = 0;
    return true;
}

bool jit_win_ptr_config_for(int k, int m, int bytes, JitConfig *cfg, bool decode) {
    if (!jit_win_config_for(k, m, bytes, cfg, decode)) return false;
    cfg->ptr = 1;
    return true;
}

bool jit_win_config_for(int k, int m, int bytes, JitConfig *cfg, bool decode) {
    if (const char *env = std::getenv("LONGHAIR_AMD_PATH")) {
        if (std::string(env) == "generic") return false;
    }
    if (k < 2 || m < 2 || k + m > 256 || bytes % 8 != 0 || bytes <= 0) return false;
    const int sub = bytes / 8, W = 4;
    if (sub % (64 * W) != 0) return false;
    cfg->k = k;
    cfg->m = m;
    cfg->bytes = bytes;
    cfg->sub = sub;
    cfg->W = W;
    cfg->nch = sub / W;
    cfg->spw = 0;
    cfg->wps = (cfg->nch + 63) / 64;
    cfg->win = decode ? 2 : 1;
    // Decode: phase A writes V_r in place of R_r and lh_inverse_gt_kernel (kernels.hip) does
    // phase B.  (Round 4 built two fused forms, V kept in the registers of the wave that
    // computed it: both slower, k128/m32 5.55 / 4.03 ms against 3.44 ms, and removed in round 5;
    // DESIGN.md 5.3.)
    cfg->win_split = decode ? 1 : 0;
    // Rows per wave: 16 (half the redundant column loads and nibble tables of 8: k128/m32
    // encode 4.21 -> 3.00 ms; split decode phase A: k128/m32 decode 4.24 -> 4.14 ms,
    // k200/m56 0.87 -> 0.79; 11 or 12 measured slower, profiles/r4i_tune_*_rows.txt).
    // At most 16 rows per wave, spread evenly over the ceil(m / 16) waves: the waves meet
    // at a barrier every column, so the fullest one sets the pace (k200/m56: 14-row groups
    // instead of 16 + 16 + 16 + 8, encode 0.414 -> 0.396 ms, decode 0.810 -> 0.788 ms).
    {
        const int cap = 16, ng = (m + cap - 1) / cap;
        cfg->rows_per_wave = (m + ng - 1) / ng;
    }
    cfg->win_pf = 3;
    // Column tiles staged once per workgroup by LDS-DMA (round 3: per-wave global loads and a
    // private LDS ring per wave measured slower, profiles/r3t_win_private_ring.txt).
    cfg->win_lds = 1;
    if ((m + cfg->rows_per_wave - 1) / cfg->rows_per_wave > 16) return false;  // <= 1024 threads
    if (decode && m > 64) return false;  // the plan's used-row mask is one 64-lane ballot
    cfg->defines.clear();
    if (const char *d = std::getenv("LONGHAIR_AMD_JIT_DEFINES")) cfg->defines = d;
    return true;
}

// Straight-line source of the 4-bit-windowed network for row group `g` (win modules):
// per data column, the nibble-table entries the group's rows need are built once from
// their lowest-bit predecessor, then every output sub-row XORs at most two entries.
// Encode modules store the rows to the recovery blocks; decode modules (c.win == 2)
// read the columns through the stripe's slot map and leave V in the LDS tile `lv`.
static void emit_win_group(std::ostream &os, const JitConfig &c, const std::vector<uint8_t> &G, int g) {
    const int R = c.rows_per_wave, k = c.k, m = c.m, PF = c.win_pf;
    const int r0 = g * R, r1 = std::min(m, r0 + R);
    const bool elim = c.win == 2;  // decode phase A: slot-mapped columns + recovery rows
    // LDS staging (c.win_lds): the workgroup's 8 x 256-byte column tile is fetched once by
    // LDS-DMA (global_load_lds_dwordx4, 16 B per lane; waves 0 and 1 each move one 1-KiB
    // half, or wave 0 both when the group has one wave) into a ring of D = PF + 1 tiles,
    // PF columns ahead; per column every wave waits for its own DMA (counted vmcnt), meets
    // the others at s_barrier, issues the DMA of column x + PF into the tile of column
    // x - 1 (read by every wave before the barrier) and reads its 8 dwords from LDS.  Each
    // column crosses HBM once per workgroup, at 16 B per lane, instead of once per wave at
    // 4 B per lane (a 4-byte-lane stream reads at 4.1 TB/s against 6.3 for 16-byte lanes).
    const int NG = (m + R - 1) / R, D = PF + 1;
    const int ndma = NG == 1 ? 2 : (g < 2 ? 1 : 0);  // DMA instructions per column, this wave
    // c.ptr (pointer-table batches; LDS staging and the split decode only): the stripe's
    // block pointers ride in VGPR lanes (ptl: k slots / columns, otl: m recovery blocks) and
    // lh_pp reads one as a wave-uniform pointer; coff = the workgroup's byte offset in every
    // block, loff = the lane's.
    // (Decode: cpl instead, lane i of cpl[i / 64] = the block pointer of stream column i --
    // original i < k or recovery row i - k -- through the stripe's slot map, the zero page
    // for an absent one: resolved once per workgroup, so a column's base is two v_readlane
    // with constant lane selects.)
    if (c.ptr)
        os << "__device__ __forceinline__ void lh_wg" << g << "("
           << (elim ? "const unsigned long long (&cpl)[LH_NQ], const unsigned int (&slv)[LH_NQ], "
                      "const unsigned char *__restrict__ pl"
                    : "const unsigned long long (&ptl)[LH_NP], const unsigned long long (&otl)[LH_NPO]")
           << ", const int coff, const int loff, const int lh_bytes, const int lh_sub) {\n";
    else
    os << "__device__ __forceinline__ void lh_wg" << g << "(" << (elim ? "" : "const ") << "unsigned char *__restrict__ base, "
       << (elim ? "const unsigned int (&slv)[LH_NQ], const unsigned char *__restrict__ pl"
                : "unsigned char *__restrict__ o")
       << ", const unsigned char *__restrict__ sb, const unsigned char *__restrict__ zb, const int lh_bytes,"
          " const int lh_sub) {\n";
    {  // (Starting the accumulators at R_r, loaded before the column loop, measured equal:
       // k128/m32 decode 4.12 / 4.11 ms, k200/m56 0.83 / 0.81 ms.)
        for (int r = r0; r < r1; ++r)
            for (int y = 0; y < 8; ++y) os << "  unsigned int a" << (r - r0) << "_" << y << " = 0;\n";
    }
    // (Skipping the XORs of a recovery row the stripe did not receive, a wave-uniform branch
    // per row and column, measured slower: k200/m56 random-e decode 0.629 against 0.591 ms,
    // profiles/r5o_bench_k200m56.json / r5o_rs0_bench_k200m56.json.)
    auto dcol = [&](int x) {  // uniform base of column x for the DMA (stripe + chunk, or zero page)
        std::ostringstream e;
        if (c.ptr && elim) e << "(lh_pp(cpl, " << x << ") + coff)";
        else if (c.ptr) e << "(lh_pp(ptl, " << x << ") + coff)";
        else if (elim) e << "lh_slot(slv, " << x << ", sb, zb, lh_bytes)";
        else e << "(sb + (long long)" << x << " * lh_bytes)";
        return e.str();
    };
    auto dma = [&](int x, const char *ind) {
        for (int h = 0; h < 2; ++h) {
            if (!(NG == 1 || g == h)) continue;
            os << ind << "lh_dma(" << dcol(x) << " + dof" << h << ", tile" << x % D << " + " << h * 1024 << ");\n";
        }
    };
    os << "  const int lane = threadIdx.x & 63;\n";
    for (int h = 0; h < 2; ++h)
        if (NG == 1 || g == h)
            os << "  const unsigned int dof" << h << " = ((" << 64 * h << " + lane) >> 4) * (unsigned)lh_sub"
               << " + ((lane & 15) << 4);\n";
    for (int q = 0; q < PF && q < k; ++q) dma(q, "  ");
    for (int x = 0; x < k; ++x) {
        os << "  {\n";
        {
            const int ahead = std::min(PF - 1, k - 1 - x);  // this wave's DMAs issued after column x
            if (ndma) os << "    lh_wait_vm(" << ndma * ahead << ");\n";
            os << "    __builtin_amdgcn_s_barrier();\n";
            if (x + PF < k) dma(x + PF, "    ");
        }
        // Decode: an erased original contributes nothing -- skip its tables and XORs (a
        // wave-uniform branch; the column's DMA / ring slot bookkeeping above still runs).
        if (elim)
            os << "    if (__builtin_amdgcn_readlane((int)slv[" << x / 64 << "], " << x % 64 << ") != 0xFF) {\n";
        for (int b = 0; b < 8; ++b)
            os << "    const unsigned int d0_" << b << " = ((const unsigned int *)(tile" << x % D << " + " << b * 256
               << "))[lane];\n";
        // Which nibble-table entries (lo: sub-blocks 0..3, hi: 4..7) this group needs.
        bool need[2][16] = {};
        for (int r = r0; r < r1; ++r) {
            const uint64_t bm = bitmatrix(G[(size_t)r * k + x]);
            for (int y = 0; y < 8; ++y) {
                const int s = (int)((bm >> (8 * y)) & 0xFF);
                need[0][s & 15] = need[1][s >> 4] = true;
            }
        }
        for (int h = 0; h < 2; ++h) {
            // close under "drop the lowest bit" so every entry has its predecessor
            for (int n = 15; n >= 1; --n)
                if (need[h][n]) need[h][n & (n - 1)] = true;
            for (int n = 1; n < 16; ++n) {
                if (!need[h][n]) continue;
                const int low = __builtin_ctz(n), pre = n & (n - 1);
                os << "    const unsigned int t" << h << "_" << n << " = ";
                if (pre) os << "t" << h << "_" << pre << " ^ ";
                os << "d0_" << (4 * h + low) << ";\n";
            }
        }
        for (int r = r0; r < r1; ++r) {
            const uint64_t bm = bitmatrix(G[(size_t)r * k + x]);
            for (int y = 0; y < 8; ++y) {
                const int s = (int)((bm >> (8 * y)) & 0xFF), lo = s & 15, hi = s >> 4;
                if (!lo && !hi) continue;
                const std::string a = "a" + std::to_string(r - r0) + "_" + std::to_string(y);
                if (lo && hi)  // XOR3 in one v_bitop3_b32 (hipcc does not fuse XOR chains)
                    os << "    " << a << " = __builtin_amdgcn_bitop3_b32(" << a << ", t0_" << lo << ", t1_" << hi
                       << ", 0x96);\n";
                else
                    os << "    " << a << " ^= " << (lo ? "t0_" + std::to_string(lo) : "t1_" + std::to_string(hi)) << ";\n";
            }
        }
        os << "    LH_PIN" << (r1 - r0) << ";\n";
        if (elim) os << "    }\n";
        os << "  }\n";
    }
    if (elim) {  // V_r = R_r + sum_x ...: read R_r, store V_r over it (absent rows: nothing)
        for (int r = r0; r < r1; ++r) {
            os << "  {\n    const unsigned int s = (unsigned int)__builtin_amdgcn_readlane((int)slv[" << (k + r) / 64
               << "], " << (k + r) % 64 << ");\n    if (s != 0xFFu) {\n";
            if (c.ptr)
                os << "      unsigned char *rp = lh_pp(cpl, " << k + r << ") + loff;\n";
            else
                os << "      unsigned char *rp = base + (long long)s * lh_bytes;\n";
            for (int y = 0; y < 8; ++y)
                os << "      const unsigned int r" << y << " = lh_ld_r(rp + " << y << " * lh_sub);\n";
            for (int y = 0; y < 8; ++y)
                os << "      lh_st(rp + " << y << " * lh_sub, a" << (r - r0) << "_" << y << " ^ r" << y << ");\n";
            os << "    }\n  }\n";
        }
    } else if (c.ptr) {
        for (int r = r0; r < r1; ++r) {
            os << "  {\n    unsigned char *op = lh_pp(otl, " << r << ") + loff;\n";
            for (int y = 0; y < 8; ++y)
                os << "    lh_st(op + " << y << " * lh_sub, a" << (r - r0) << "_" << y << ");\n";
            os << "  }\n";
        }
    } else {
        for (int r = r0; r < r1; ++r)
            for (int y = 0; y < 8; ++y)
                os << "  lh_st(o + (long long)" << r << " * lh_bytes + " << y << " * lh_sub, a" << (r - r0) << "_" << y << ");\n";
    }
    os << "}\n";
}

// Large-m decode modules (m <= 64, one workgroup per (stripe, 64 * W-byte column chunk)):
// phase A (V_r = R_r + sum_{x present} B(G[r][x]) D_x, windowed network above, slot maps
// from the stripe's plan held in VGPR lanes and read with v_readlane).
// V_r is written back in place of R_r; phase B is lh_inverse_gt_kernel (kernels.hip).
static void emit_wide_decode(std::ostream &os, const JitConfig &c, const std::vector<uint8_t> &G) {
    const int R = c.rows_per_wave, NG = (c.m + R - 1) / R;
    const int e_max = std::min(c.k, c.m), km = c.k + c.m;
    os << "#define LH_NQ " << (km + 63) / 64 << "\n"
       << "__device__ __forceinline__ const unsigned char *lh_slot(const unsigned int (&slv)[LH_NQ], const int i,\n"
       << "    const unsigned char *base, const unsigned char *zero, const int bytes) {\n"
       << "  const unsigned int s = (unsigned int)__builtin_amdgcn_readlane((int)slv[i / 64], i % 64);\n"
       << "  return s == 0xFFu ? zero : base + (long long)s * bytes;\n}\n";
    for (int g = 0; g < NG; ++g) emit_win_group(os, c, G, g);
    if (c.ptr) {
        // blocks: the pointer table, k slot pointers per stripe (row stride `stride` bytes)
        os << "extern \"C\" __global__ void __launch_bounds__(" << 64 * NG << ")\n"
           << "lh_jit_decode_wide(unsigned char *__restrict__ blocks, long long stride,\n"
           << "                   const unsigned char *__restrict__ plan, long long plan_stride,\n"
           << "                   const unsigned char *__restrict__ zero_page, int stripes, int bytes) {\n"
           << "  const int g = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);\n"
           << "  const int lh_sub = bytes >> 3, lh_cps = lh_sub / " << 64 * c.W << ";  // (the block size: an argument)\n"
           << "  const int lane = threadIdx.x & 63;\n"
           << "  const long long stripe = blockIdx.x / lh_cps;\n"
           << "  if (stripe >= stripes) return;\n"
           << "  const unsigned char *pl = plan + stripe * plan_stride;\n"
           << "  if (pl[0] == 0) return;  // workgroup-uniform\n"
           << "  unsigned int slv[LH_NQ];\n"
           << "#pragma unroll\n  for (int q = 0; q < LH_NQ; ++q) {\n"
           << "    const int i = q * 64 + lane;\n"
           << "    slv[q] = i < " << km << " ? (unsigned int)pl[" << 16 + e_max << " + i] : 0xFFu;\n"
           << "  }\n"
           << "  const unsigned long long *tab = (const unsigned long long *)(blocks + stripe * stride);\n"
           << "  unsigned long long cpl[LH_NQ];\n"
           << "#pragma unroll\n  for (int q = 0; q < LH_NQ; ++q)\n"
           << "    cpl[q] = slv[q] == 0xFFu ? (unsigned long long)zero_page : tab[slv[q]];\n"
           << "  const int coff = (int)(blockIdx.x % lh_cps) * " << 64 * c.W << ";\n";
        for (int g = 0; g < NG; ++g)
            os << "  " << (g ? "else " : "") << "if (g == " << g << ") lh_wg" << g << "(cpl, slv, pl, coff, coff + lane * "
               << c.W << ", bytes, lh_sub);\n";
        os << "}\n";
        return;
    }
    os << "extern \"C\" __global__ void __launch_bounds__(" << 64 * NG << ")\n"
       << "lh_jit_decode_wide(unsigned char *__restrict__ blocks, long long stride,\n"
       << "                   const unsigned char *__restrict__ plan, long long plan_stride,\n"
       << "                   const unsigned char *__restrict__ zero_page, int stripes, int bytes) {\n";
    os << "  const int g = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);\n"
       << "  const int lh_sub = bytes >> 3, lh_cps = lh_sub / " << 64 * c.W << ";  // (the block size: an argument)\n"
       << "  const int lane = threadIdx.x & 63;\n"
       << "  const long long stripe = blockIdx.x / lh_cps;\n"
       << "  if (stripe >= stripes) return;\n"
       << "  const unsigned char *pl = plan + stripe * plan_stride;\n"
       << "  if (pl[0] == 0) return;  // workgroup-uniform\n"
       << "  unsigned int slv[LH_NQ];\n"
       << "#pragma unroll\n  for (int q = 0; q < LH_NQ; ++q) {\n"
       << "    const int i = q * 64 + lane;\n"
       << "    slv[q] = i < " << km << " ? (unsigned int)pl[" << 16 + e_max << " + i] : 0xFFu;\n"
       << "  }\n"
       << "  const int chunk = (int)(blockIdx.x % lh_cps) * " << 64 * c.W << ";\n"
       << "  unsigned char *b = blocks + stripe * stride + chunk + lane * " << c.W << ";\n";
    os << "  const unsigned char *sb = blocks + stripe * stride + chunk;\n"
       << "  const unsigned char *zb = zero_page + chunk;\n";
    const std::string dargs = "(b, slv, pl, sb, zb, bytes, lh_sub)";
    for (int g = 0; g < NG; ++g) os << "  " << (g ? "else " : "") << "if (g == " << g << ") lh_wg" << g << dargs << ";\n";
    os << "}\n";
}

static std::string win_source_for(const JitConfig &c) {
    std::ostringstream os;
    const std::vector<uint8_t> G = generator_matrix(c.k, c.m);
    const int R = c.rows_per_wave, NG = (c.m + R - 1) / R;
    os << "// longhair_amd windowed " << (c.win == 2 ? "decode" : "encode") << ", k=" << c.k << " m=" << c.m
       << " (block size: a kernel argument; one module serves every size with sub % " << 64 * c.W << " == 0)\n"
       << "#ifndef LH_NT\n#define LH_NT 1\n#endif\n"
       << "__device__ __forceinline__ unsigned int lh_ld(const unsigned char *p) {\n"
       << "#if LH_NT\n  return __builtin_nontemporal_load((const unsigned int *)p);\n#else\n"
       << "  unsigned int w; __builtin_memcpy(&w, p, 4); return w;\n#endif\n}\n"
       << "// R_r, read just before V_r is stored over it (split decode): cache policy LH_NT_R\n"
       << "#ifndef LH_NT_R\n#define LH_NT_R LH_NT\n#endif\n"
       << "__device__ __forceinline__ unsigned int lh_ld_r(const unsigned char *p) {\n"
       << "#if LH_NT_R\n  return __builtin_nontemporal_load((const unsigned int *)p);\n#else\n"
       << "  unsigned int w; __builtin_memcpy(&w, p, 4); return w;\n#endif\n}\n"
       << "__device__ __forceinline__ void lh_st(unsigned char *p, unsigned int v) {\n"
       << "#if LH_NT\n  __builtin_nontemporal_store(v, (unsigned int *)p);\n#else\n"
       << "  __builtin_memcpy(p, &v, 4);\n#endif\n}\n"
       << "__device__ __forceinline__ void lh_dma(const unsigned char *src, unsigned char *lds) {  // 16 B per lane\n"
       << "  __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void *)src,\n"
       << "                                   (__attribute__((address_space(3))) void *)lds, 16, 0, LH_NT ? 2 : 0);\n}\n"
       << "// s_waitcnt vmcnt(N) with expcnt / lgkmcnt untouched (gfx9 encoding)\n"
       << "#define lh_wait_vm(N) __builtin_amdgcn_s_waitcnt(((N) & 15) | (((N) >> 4) << 14) | (7 << 4) | (15 << 8))\n";
    if (c.ptr)
        os << "#define LH_NP " << (c.k + 63) / 64 << "\n#define LH_NPO " << (c.m + 63) / 64 << "\n"
           << "// entry i of a pointer table held in VGPR lanes (lane i % 64 of t[i / 64]), wave-uniform\n"
           << "template <int N>\n"
           << "__device__ __forceinline__ unsigned char *lh_pp(const unsigned long long (&t)[N], const int i) {\n"
           << "  unsigned lo = 0, hi = 0;\n"
           << "#pragma unroll\n  for (int q = 0; q < N; ++q)\n"
           << "    if ((i >> 6) == q) {\n"
           << "      lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)t[q], i & 63);\n"
           << "      hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(t[q] >> 32), i & 63);\n"
           << "    }\n"
           << "  return (unsigned char *)(((unsigned long long)hi << 32) | lo);\n}\n"
           << "template <int N>\n"
           << "__device__ __forceinline__ void lh_ptab_lanes(unsigned long long (&t)[N], const unsigned long long *row, int n) {\n"
           << "  const int lane = threadIdx.x & 63;\n"
           << "#pragma unroll\n  for (int q = 0; q < N; ++q) t[q] = q * 64 + lane < n ? row[q * 64 + lane] : 0ull;\n}\n";
    // One __shared__ object per LDS ring slot: the compiler's LDS-DMA wait tracking tells
    // distinct objects apart, so reading tile x % D does not wait for the DMA into another.
    for (int q = 0; q <= c.win_pf; ++q)
        os << "__shared__ __attribute__((aligned(16))) unsigned char tile" << q << "[2048];\n";
    // LH_PINn: keep the accumulators in registers between columns (no re-association).
    // One asm statement per row (8 operands): every volatile asm is a memory side effect
    // to LLVM, and the IR sinking pass's cost grows with their number times the loads of
    // the block -- one statement per accumulator made hiprtc spend 387 of the 451 s of the
    // k200/m56 encode module in "Code sinking" (grouped: 85 s, 221 -> 217 VGPRs).
    for (int n = 1; n <= R; ++n) {
        os << "#define LH_PIN" << n << " do {";
        for (int r = 0; r < n; ++r) {
            os << " asm volatile(\"\" :";
            for (int y = 0; y < 8; ++y) os << (y ? ", " : " ") << "\"+v\"(a" << r << "_" << y << ")";
            os << ");";
        }
        os << " } while (0)\n";
    }
    if (c.win == 2) {
        emit_wide_decode(os, c, G);
        return os.str();
    }
    for (int g = 0; g < NG; ++g) emit_win_group(os, c, G, g);
    if (c.ptr) {
        // in / out: the pointer tables (k data, m recovery block pointers per stripe)
        os << "extern \"C\" __global__ void __launch_bounds__(" << 64 * NG << ")\n"
           << "lh_jit_encode_win(const unsigned char *__restrict__ in, long long in_stride,\n"
           << "                  unsigned char *__restrict__ out, long long out_stride, int stripes, int bytes) {\n"
           << "  const int g = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);\n"
           << "  const int lh_sub = bytes >> 3, lh_cps = lh_sub / " << 64 * c.W << ";  // (the block size: an argument)\n"
           << "  const long long stripe = blockIdx.x / lh_cps;\n"
           << "  if (stripe >= stripes) return;\n"
           << "  unsigned long long ptl[LH_NP], otl[LH_NPO];\n"
           << "  lh_ptab_lanes(ptl, (const unsigned long long *)(in + stripe * in_stride), " << c.k << ");\n"
           << "  lh_ptab_lanes(otl, (const unsigned long long *)(out + stripe * out_stride), " << c.m << ");\n"
           << "  const int coff = (int)(blockIdx.x % lh_cps) * " << 64 * c.W << ";\n";
        for (int g = 0; g < NG; ++g)
            os << "  " << (g ? "else " : "") << "if (g == " << g << ") lh_wg" << g << "(ptl, otl, coff, coff + (int)(threadIdx.x & 63) * "
               << c.W << ", bytes, lh_sub);\n";
        os << "}\n";
        return os.str();
    }
    os << "extern \"C\" __global__ void __launch_bounds__(" << 64 * NG << ")\n"
       << "lh_jit_encode_win(const unsigned char *__restrict__ in, long long in_stride,\n"
       << "                  unsigned char *__restrict__ out, long long out_stride, int stripes, int bytes) {\n"
       << "  const int g = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);\n"
       << "  const int lh_sub = bytes >> 3, lh_cps = lh_sub / " << 64 * c.W << ";  // (the block size: an argument)\n"
       << "  const long long stripe = blockIdx.x / lh_cps;\n"
       << "  if (stripe >= stripes) return;\n"
       << "  const int p = (int)(blockIdx.x % lh_cps) * " << 64 * c.W << " + (int)(threadIdx.x & 63) * "
       << c.W << ";\n"
       << "  const unsigned char *b = in + stripe * in_stride + p;\n"
       << "  unsigned char *o = out + stripe * out_stride + p;\n";
    os << "  const unsigned char *sb = in + stripe * in_stride + (int)(blockIdx.x % lh_cps) * " << 64 * c.W
       << ";\n";
    const char *eargs = "(b, o, sb, nullptr, bytes, lh_sub)";
    for (int g = 0; g < NG; ++g) os << "  " << (g ? "else " : "") << "if (g == " << g << ") lh_wg" << g << eargs << ";\n";
    os << "}\n";
    return os.str();
}

std::string jit_source_for(const JitConfig &c) {
    std::ostringstream os;
    if (c.win) {
        std::string tok;
        for (char ch : c.defines + " ") {  // tuning knobs as for the regular modules
            if (ch == ' ' || ch == ',') {
                const size_t eq = tok.find('=');
                if (!tok.empty()) os << "#define " << (eq == std::string::npos ? tok : tok.substr(0, eq) + " " + tok.substr(eq + 1)) << "\n";
                tok.clear();
            } else {
                tok += ch;
            }
        }
        os << win_source_for(c);
        return os.str();
    }
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
    if (c.family) {  // (block-size family: the size macros are placeholders the family kernel ignores)
        os << "#define LH_FAMILY 1\n#define LH_K " << c.k << "\n#define LH_M " << c.m
           << "\n#define LH_BYTES 1024\n#define LH_SUB 128\n#define LH_W 8\n#define LH_NCH 16\n#define LH_SPW 4"
              "\n#define LH_WPS 1\n#ifndef LH_LDS\n#define LH_LDS 1\n#endif\n#ifndef LH_CPS\n#define LH_CPS "
           << c.cps << "\n#endif\n#define LH_ROLE " << c.role << "\n#define LH_DEC_PLAIN 0\n";
    } else {
    os << "#define LH_K " << c.k << "\n#define LH_M " << c.m << "\n#define LH_BYTES " << c.bytes
       << "\n#define LH_SUB " << c.sub << "\n#define LH_W " << c.W << "\n#define LH_NCH " << c.nch
       << "\n#define LH_SPW " << (c.spw ? c.spw : 1) << "\n#define LH_WPS " << (c.wps ? c.wps : 1) << "\n";
    if (c.ptr) os << "#define LH_PTR 1\n#define LH_BUF 0\n";
    if (c.lds) os << "#ifndef LH_LDS\n#define LH_LDS 1\n#endif\n";  // (a LONGHAIR_AMD_JIT_DEFINES value wins)
    if (c.cps > 1 && !c.ptr) os << "#ifndef LH_CPS\n#define LH_CPS " << c.cps << "\n#endif\n";
    if (c.role) os << "#define LH_ROLE " << c.role << "\n#define LH_DEC_PLAIN " << c.plain << "\n";
    }
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

JitCache::Key JitCache::key_of(const JitConfig &cfg) {
    // (windowed modules take the block size as an argument: one per (k, m, W, ...))
    return Key(cfg.k, cfg.m, (cfg.win || cfg.family) ? 0 : cfg.bytes, cfg.W, cfg.defines + (cfg.family ? "|family" : ""),
               cfg.lds * 1000000000 + cfg.ptr * 100000000 + (cfg.role + 3 * cfg.plain) * 10000000 +
                   cfg.win_split * 1000000 + cfg.win * 100000 + cfg.win_lds * 10000 +
                   cfg.rows_per_wave * 100 + cfg.win_pf);
}

const JitKernels *JitCache::peek(const JitConfig &cfg) {
    std::lock_guard<std::mutex> g(mu_);
    auto it = cache_.find(key_of(cfg));
    return it == cache_.end() ? nullptr : &it->second;
}

// ------------------------------------------------------------ code-object cache
// Compiled code objects are kept on disk, keyed by a hash of the generated source and
// the compile options, so a shape is compiled once per machine (the large-m windowed
// modules take about a minute).  Directory: $LONGHAIR_AMD_CACHE_DIR, else jit_cache/
// next to liblonghair_amd.so (it travels with the repository), else ~/.cache/longhair_amd.
// GVN's memory-dependence analysis and load PRE find nothing to do in the straight-line
// networks (every column is loaded once; the accumulator pins are memory side effects that
// make the analysis expensive): off, the generated code is byte-identical (checked on the
// k29/m4, k64/m5 and k128/m32 modules) and the large register networks compile ~30 % faster
// (k64/m5/4096: 113 -> 81 s).
static const char *kOpts[] = {"--offload-arch=gfx950", "-O3", "-std=c++17", "-mllvm", "-enable-gvn-memdep=false",
                              "-mllvm", "-enable-load-pre=false"};

static uint64_t fnv1a(const std::string &s, uint64_t h = 1469598103934665603ull) {
    for (unsigned char ch : s) h = (h ^ ch) * 1099511628211ull;
    return h;
}

static std::string cache_dir() {
    if (const char *d = std::getenv("LONGHAIR_AMD_CACHE_DIR")) return d;
    Dl_info info;
    if (dladdr((void *)&fnv1a, &info) && info.dli_fname) {
        std::string p = info.dli_fname;
        const size_t slash = p.rfind('/');
        if (slash != std::string::npos) {
            std::string d = p.substr(0, slash) + "/jit_cache";
            mkdir(d.c_str(), 0755);
            if (access(d.c_str(), W_OK) == 0) return d;
        }
    }
    if (const char *home = std::getenv("HOME")) {
        std::string d = std::string(home) + "/.cache";
        mkdir(d.c_str(), 0755);
        d += "/longhair_amd";
        mkdir(d.c_str(), 0755);
        return d;
    }
    return "";
}

static std::string cache_path(const std::string &src) {
    // Key: generated source, compile options and the hiprtc / HIP runtime versions, so a
    // cache made by another ROCm is never loaded.
    std::string key = src;
    for (const char *o : kOpts) key += std::string("\n") + o;
    // (HIP_VERSION is the build's headers; hipRuntimeGetVersion would need a device, and
    // the cache is filled on a machine without one.)
    // hiprtcVersion once per process: hiprtc serialises its API calls, so asking while a
    // background compilation runs would wait for it (a cached-module lookup blocked ~1.4 s).
    static const std::string ver = [] {
        int major = 0, minor = 0;
        (void)hiprtcVersion(&major, &minor);
        return std::to_string(major) + "." + std::to_string(minor);
    }();
    key += "\nhiprtc " + ver + " hip " + std::to_string(HIP_VERSION);
    char name[64];
    snprintf(name, sizeof(name), "/lh_%016llx.co", (unsigned long long)fnv1a(key));
    const std::string d = cache_dir();
    return d.empty() ? "" : d + name;
}

bool jit_compile_allowed() {
    const char *e = std::getenv("LONGHAIR_AMD_JIT_COMPILE");
    return !(e && std::string(e) == "0");
}

JitMode batch_jit_mode() {
    if (!jit_compile_allowed()) return JitMode::kCached;
    const char *s = std::getenv("LONGHAIR_AMD_JIT_SYNC");
    return (s && std::string(s) == "1") ? JitMode::kBlocking : JitMode::kAsync;
}

// Background compilations run on ONE long-lived worker thread fed by a queue (round 5,
// a thread per compilation stayed mapped until process exit, so a process meeting
// many shapes grew without bound).  The worker is started by the first background request.
// Exit: before that first request is queued, the posting thread compiles a
// trivial program, so hiprtc's lazily constructed state (and its exit-time teardown) exists
// before the drain handler is registered with atexit(); handlers and static destructors run
// in reverse order, so at exit the drain runs first: it drops the queued requests and joins
// the worker (waiting for the compilation in flight) while hiprtc is still intact.  The
// worker is never detached.
namespace {
void warm_hiprtc() {
    hiprtcProgram p;
    if (hiprtcCreateProgram(&p, "extern \"C\" __global__ void lh_warm() {}", "lh_warm.hip", 0, nullptr, nullptr) !=
        HIPRTC_SUCCESS)
        return;
    const char *opts[] = {"--offload-arch=gfx950", "-O0"};
    (void)hiprtcCompileProgram(p, 2, opts);
    hiprtcDestroyProgram(&p);
}
struct CompileWorker {
    std::mutex mu;
    std::condition_variable cv, idle_cv;
    std::deque<std::function<void()>> q;
    std::thread th;
    bool busy = false, stop = false, drain_registered = false;
    void post(std::function<void()> f) {
        std::unique_lock<std::mutex> g(mu);
        if (stop) return;  // exiting: the request stays pending, its shape on the generic kernels
        if (!drain_registered) {
            drain_registered = true;
            g.unlock();
            warm_hiprtc();
            std::atexit(drain_at_exit);
            g.lock();
            if (stop) return;
        }
        q.push_back(std::move(f));
        if (!th.joinable()) th = std::thread([this] { run(); });
        cv.notify_one();
    }
    void run() {
        for (;;) {
            std::function<void()> f;
            {
                std::unique_lock<std::mutex> l(mu);
                cv.wait(l, [&] { return stop || !q.empty(); });
                if (q.empty()) return;  // stop requested and nothing left
                f = std::move(q.front());
                q.pop_front();
                busy = true;
            }
            f();
            {
                std::lock_guard<std::mutex> g(mu);
                busy = false;
            }
            idle_cv.notify_all();
        }
    }
    // Wait until every queued request has run (jit_join_background).
    void wait_idle() {
        std::unique_lock<std::mutex> l(mu);
        idle_cv.wait(l, [&] { return q.empty() && !busy; });
    }
    // Drop queued requests, let the one in flight finish, end the worker.
    void shutdown() {
        {
            std::lock_guard<std::mutex> g(mu);
            stop = true;
            q.clear();
        }
        cv.notify_all();
        if (th.joinable() && th.get_id() != std::this_thread::get_id()) th.join();
    }
    static void drain_at_exit();
    ~CompileWorker() { shutdown(); }  // (the drain handler has normally joined it already)
};
CompileWorker &compile_worker() {
    static CompileWorker w;
    return w;
}
void CompileWorker::drain_at_exit() { compile_worker().shutdown(); }
}  // namespace

void jit_join_background() { compile_worker().wait_idle(); }

bool compile_code_object(const JitConfig &cfg, std::vector<char> *code, std::string *err, bool fresh, bool compile) {
    const std::string src = jit_source_for(cfg);
    const std::string path = cache_path(src);
    if (fresh && !path.empty()) unlink(path.c_str());  // a cached object the loader rejected
    if (!path.empty()) {
        if (FILE *f = fopen(path.c_str(), "rb")) {
            fseek(f, 0, SEEK_END);
            const long n = ftell(f);
            fseek(f, 0, SEEK_SET);
            code->resize(n > 0 ? (size_t)n : 0);
            const bool ok = n > 0 && fread(code->data(), 1, (size_t)n, f) == (size_t)n;
            fclose(f);
            if (ok) {
                (void)utime(path.c_str(), nullptr);  // mark as used (tools/precompile.py --prune)
                return true;
            }
        }
    }
    if (!compile) {
        *err = "not cached";
        return false;
    }
    if (const char *dump = std::getenv("LONGHAIR_AMD_JIT_DUMP")) {  // (diagnostics: the generated source)
        const size_t slash = path.rfind('/');
        const std::string name = std::string(dump) + "/" + (slash == std::string::npos ? path : path.substr(slash + 1)) + ".hip";
        if (FILE *f = fopen(name.c_str(), "wb")) {
            fwrite(src.data(), 1, src.size(), f);
            fclose(f);
        }
    }
    hiprtcProgram prog;
    if (hiprtcCreateProgram(&prog, src.c_str(), "lh_jit_codec.hip", 0, nullptr, nullptr) != HIPRTC_SUCCESS) {
        *err = "hiprtcCreateProgram failed";
        return false;
    }
    const hiprtcResult rc = hiprtcCompileProgram(prog, (int)(sizeof(kOpts) / sizeof(kOpts[0])), kOpts);
    if (rc != HIPRTC_SUCCESS) {
        size_t n = 0;
        hiprtcGetProgramLogSize(prog, &n);
        std::string log(n + 1, '\0');
        hiprtcGetProgramLog(prog, &log[0]);
        *err = "hiprtc compile failed: " + log;
        hiprtcDestroyProgram(&prog);
        return false;
    }
    size_t code_size = 0;
    hiprtcGetCodeSize(prog, &code_size);
    code->resize(code_size);
    hiprtcGetCode(prog, code->data());
    hiprtcDestroyProgram(&prog);
    if (!path.empty()) {  // write-then-rename so concurrent processes never read a torn file
        const std::string tmp = path + ".tmp." + std::to_string((long long)getpid());
        if (FILE *f = fopen(tmp.c_str(), "wb")) {
            const bool ok = fwrite(code->data(), 1, code->size(), f) == code->size();
            fclose(f);
            if (ok) rename(tmp.c_str(), path.c_str());
            else unlink(tmp.c_str());
        }
    }
    return true;
}

// Loads a code object into the current device's context and records its kernels (mu_ held).
const JitKernels *JitCache::load_locked(const Key &key, const JitConfig &cfg, std::vector<char> &code,
                                        std::string *err) {
    JitKernels kern;
    kern.cfg = cfg;
    if (hipModuleLoadData(&kern.module, code.data()) != hipSuccess) {
        // A damaged or foreign cached object: drop it and compile once more (synchronously).
        (void)hipGetLastError();
        if (!compile_code_object(cfg, &code, err, true, true)) return nullptr;
        if (hipModuleLoadData(&kern.module, code.data()) != hipSuccess) {
            *err = "hipModuleLoadData failed for the specialised kernels";
            return nullptr;
        }
    }
    auto fn = [&](const char *name) -> hipFunction_t {
        hipFunction_t f = nullptr;
        if (hipModuleGetFunction(&f, kern.module, name) != hipSuccess) {
            (void)hipGetLastError();
            return nullptr;
        }
        return f;
    };
    kern.encode = fn("lh_jit_encode");
    kern.decode = fn("lh_jit_decode");
    kern.decode_fused = fn("lh_jit_decode_fused");
    kern.encode_win = fn("lh_jit_encode_win");
    kern.decode_wide = fn("lh_jit_decode_wide");
    if (hipFunction_t f = kern.encode ? kern.encode : kern.decode_fused ? kern.decode_fused : kern.decode;
        f && cfg.wgcu > 0 && !cfg.win) {
        int st = 0;
        if (hipFuncGetAttribute(&st, HIP_FUNC_ATTRIBUTE_SHARED_SIZE_BYTES, f) != hipSuccess) {
            (void)hipGetLastError();
            st = 0;
        }
        const int per = 160 * 1024 / cfg.wgcu;  // gfx950: 160 KiB of LDS per CU
        kern.dyn_lds = st > 0 && per - 1024 > st ? (unsigned)(per - 1024 - st + 16) : 0u;
        if (kern.dyn_lds && st + (int)kern.dyn_lds > 160 * 1024) kern.dyn_lds = 0;
    }
    // (one role per register-network module: the encode, or one of the two decodes)
    if (!kern.encode && !kern.decode && !kern.decode_fused && !kern.encode_win && !kern.decode_wide) {
        *err = "specialised module has no kernel";
        return nullptr;
    }
    not_cached_.erase(key);
    auto res = cache_.emplace(key, kern);
    return &res.first->second;
}

const JitKernels *JitCache::get(const JitConfig &cfg, std::string *err, JitMode mode, bool *failed) {
    const Key key = key_of(cfg);
    std::shared_ptr<Pending> p;
    bool compile_here = false;  // kBlocking and no compilation in flight: run hiprtc on this thread
    {
        std::lock_guard<std::mutex> g(mu_);
        auto it = cache_.find(key);
        if (it != cache_.end()) return &it->second;
        auto f = failed_.find(key);
        if (f != failed_.end()) {
            *err = f->second;
            if (failed) *failed = true;
            return nullptr;
        }
        auto pi = pending_.find(key);
        if (pi != pending_.end()) {
            p = pi->second;
            bool done;
            {
                std::lock_guard<std::mutex> pg(p->mu);
                done = p->done;
            }
            if (done) {  // compiled in the background: load it here (this thread's device)
                pending_.erase(pi);
                if (!p->ok) {
                    failed_[key] = *err = p->err;
                    if (failed) *failed = true;
                    return nullptr;
                }
                return load_locked(key, cfg, p->code, err);
            }
            if (mode != JitMode::kBlocking) {
                *err = "specialised module compiling in the background";
                return nullptr;
            }
        } else {
            // Not compiled in this process: the on-disk cache (fast: a file read), unless an
            // earlier cached-only lookup already found nothing there.
            if (!(mode == JitMode::kCached && not_cached_.count(key))) {
                std::vector<char> code;
                std::string e2;
                if (compile_code_object(cfg, &code, &e2, false, false)) return load_locked(key, cfg, code, err);
            }
            if (mode == JitMode::kCached) {
                not_cached_[key] = true;
                *err = "not cached";
                return nullptr;
            }
            p = std::make_shared<Pending>();
            pending_[key] = p;
            if (mode == JitMode::kAsync) {
                // hiprtc only (no device calls) on the worker; the module is loaded by the
                // first lookup after it finishes.
                compile_worker().post([p, cfg] {
                    std::vector<char> code;
                    std::string e;
                    const bool ok = compile_code_object(cfg, &code, &e, false, true);
                    std::lock_guard<std::mutex> pg(p->mu);
                    p->ok = ok;
                    p->code.swap(code);
                    p->err = e;
                    p->done = true;
                    p->cv.notify_all();
                });
                *err = "specialised module compiling in the background";
                return nullptr;
            }
            compile_here = true;
        }
    }
    // kBlocking: compile here without mu_ (other shapes' lookups proceed), or wait for the
    // compilation in flight.
    if (compile_here) {
        std::vector<char> code;
        std::string e;
        const bool ok = compile_code_object(cfg, &code, &e, false, true);
        std::lock_guard<std::mutex> pg(p->mu);
        p->ok = ok;
        p->code.swap(code);
        p->err = e;
        p->done = true;
        p->cv.notify_all();
    } else {
        std::unique_lock<std::mutex> pg(p->mu);
        p->cv.wait(pg, [&] { return p->done; });
    }
    std::lock_guard<std::mutex> g(mu_);
    auto it = cache_.find(key);
    if (it != cache_.end()) return &it->second;  // another waiter loaded it
    auto fi = failed_.find(key);
    if (fi != failed_.end()) {
        *err = fi->second;
        if (failed) *failed = true;
        return nullptr;
    }
    auto pi = pending_.find(key);
    if (pi != pending_.end() && pi->second == p) pending_.erase(pi);
    if (!p->ok) {
        failed_[key] = *err = p->err;
        if (failed) *failed = true;
        return nullptr;
    }
    std::vector<char> code = p->code;  // other waiters hold p too
    return load_locked(key, cfg, code, err);
}

}  // namespace lh
