// host_engine_check.cpp -- TEST INFRASTRUCTURE: the host SIMD engine of the drop-in
// dispatch policy (longhair_amd/csrc/host_codec.cpp) against the C oracle
// (oracle/liblh_oracle.so, dlopened as the checker) on random stripes: encode bytes and
// codes, then decode with random erasures, random recovery rows and shuffled slots
// (rows and bytes).  Built by tests/test_host_engine.py, also under ASan + UBSan.
// Usage: host_engine_check ORACLE_SO TABLES_BIN   (LONGHAIR_AMD_HOST_ISA picks the level)
#include <dlfcn.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "field.hpp"
#include "host_codec.hpp"

typedef int (*enc_t)(int, int, const unsigned char *const *, unsigned char *, int);
typedef int (*dec_t)(int, int, Block *, int);
typedef int (*init_t)(const unsigned char *, size_t);

int main(int argc, char **argv) {
    if (argc < 3) return 2;
    void *h = dlopen(argv[1], RTLD_NOW);
    if (!h) return 2;
    std::vector<unsigned char> blob(34902);
    FILE *f = fopen(argv[2], "rb");
    if (!f || fread(blob.data(), 1, blob.size(), f) != blob.size()) return 2;
    fclose(f);
    if (((init_t)dlsym(h, "lho_init"))(blob.data(), blob.size()) != 0) return 2;
    const enc_t oenc = (enc_t)dlsym(h, "lho_encode");
    const dec_t odec = (dec_t)dlsym(h, "lho_decode");
    srand(12345);
    int bad = 0, n = 0;
    // The decode planner's closed-form inverse (kernels.hip lh_plan_kernel): every m >= 7
    // generator must expose its Cauchy points, and A^-1[j][i] = P_j Q_i / ((x_j + y_i) C_j
    // D_i x_j) must invert random e x e submatrices (checked here by A * A^-1 = I).
    {
        const lh::Field &F = lh::Field::get();
        for (int m = 7; m <= 128; m += 11)
            for (int k : {1, 2, 9, 64, 256 - m}) {
                std::vector<uint8_t> xs, ys;
                ++n;
                if (!lh::cauchy_points(k, m, xs, ys)) {
                    printf("no Cauchy points k=%d m=%d\n", k, m);
                    ++bad;
                    continue;
                }
                const std::vector<uint8_t> G = lh::generator_matrix(k, m);
                const int e = 1 + rand() % std::min(k, m);
                std::vector<int> E, R;
                for (int x = 0; x < k && (int)E.size() < e; ++x) if (rand() % 3 == 0 || k - x == e - (int)E.size()) E.push_back(x);
                for (int r = 0; r < m && (int)R.size() < e; ++r) if (rand() % 3 == 0 || m - r == e - (int)R.size()) R.push_back(r);
                std::vector<uint8_t> inv((size_t)e * e);
                for (int j = 0; j < e; ++j)
                    for (int i = 0; i < e; ++i) {
                        const uint8_t x = xs[E[j]], y = ys[R[i]];
                        int lg = -F.log[x] - F.log[x ^ y];
                        for (int u = 0; u < e; ++u) {
                            lg += F.log[x ^ ys[R[u]]] + F.log[xs[E[u]] ^ y];
                            if (u != j) lg -= F.log[x ^ xs[E[u]]];
                            if (u != i) lg -= F.log[y ^ ys[R[u]]];
                        }
                        inv[(size_t)j * e + i] = F.exp[(lg % 255 + 255) % 255];
                    }
                for (int i = 0; i < e; ++i)
                    for (int c = 0; c < e; ++c) {
                        uint8_t acc = 0;
                        for (int j = 0; j < e; ++j) acc ^= F.mul(G[(size_t)R[i] * k + E[j]], inv[(size_t)j * e + c]);
                        if (acc != (i == c)) {
                            printf("closed-form inverse wrong k=%d m=%d e=%d\n", k, m, e);
                            ++bad;
                            i = c = e;
                        }
                    }
            }
    }
    const int shapes[][3] = {{29, 4, 1296}, {29, 1, 1296}, {2, 2, 8},     {17, 6, 520},   {128, 32, 8192},
                             {10, 6, 24},   {250, 6, 16},  {1, 3, 16},    {29, 4, 1304},  {64, 4, 4096},
                             {5, 3, 8},     {200, 56, 2048}, {29, 3, 12}, {200, 57, 16},  {3, 2, 520}};
    for (const auto &sh : shapes) {
        const int k = sh[0], m = sh[1], B = sh[2];
        for (int c = 0; c < 4; ++c) {
            std::vector<unsigned char> d((size_t)k * B);
            for (auto &x : d) x = (unsigned char)rand();
            std::vector<const unsigned char *> p(k);
            for (int x = 0; x < k; ++x) p[x] = d.data() + (size_t)x * B;
            std::vector<unsigned char> r1((size_t)m * B), r2((size_t)m * B);
            const int a = lh::host::encode(k, m, p.data(), r1.data(), B), b = oenc(k, m, p.data(), r2.data(), B);
            ++n;
            if (a != b || (a == 0 ? r1 != r2 : !std::equal(r1.begin(), r1.begin() + B, r2.begin()))) {
                printf("encode mismatch k=%d m=%d bytes=%d rc %d/%d\n", k, m, B, a, b);
                ++bad;
                continue;
            }
            if (k < 2 || a != 0) continue;
            const int e = m == 1 ? 1 : 1 + rand() % std::min(k, m);
            std::vector<int> er(k, 0), rr(m, 0), rows;
            for (int cnt = 0; cnt < e;) { const int x = rand() % k; if (!er[x]) { er[x] = 1; ++cnt; } }
            for (int cnt = 0; cnt < e;) { const int j = rand() % m; if (!rr[j]) { rr[j] = 1; ++cnt; } }
            std::vector<std::vector<unsigned char>> s1;
            for (int x = 0; x < k; ++x)
                if (!er[x]) { s1.emplace_back(d.begin() + (size_t)x * B, d.begin() + (size_t)(x + 1) * B); rows.push_back(x); }
            for (int j = 0; j < m; ++j)
                if (rr[j]) { s1.emplace_back(r2.begin() + (size_t)j * B, r2.begin() + (size_t)(j + 1) * B); rows.push_back(k + j); }
            for (int i = k - 1; i > 0; --i) {
                const int j = rand() % (i + 1);
                std::swap(s1[i], s1[j]);
                std::swap(rows[i], rows[j]);
            }
            std::vector<std::vector<unsigned char>> s2 = s1;
            std::vector<Block> b1(k), b2(k);
            for (int i = 0; i < k; ++i) {
                b1[i].data = s1[i].data(); b1[i].row = (unsigned char)rows[i];
                b2[i].data = s2[i].data(); b2[i].row = (unsigned char)rows[i];
            }
            int x1 = 0;
            if (m == 1) lh::host::decode_m1(k, b1.data(), B);
            else x1 = lh::host::decode(k, m, b1.data(), B);
            const int x2 = odec(k, m, b2.data(), B);
            bool ok = x1 == x2;
            for (int i = 0; i < k; ++i) ok = ok && b1[i].row == b2[i].row && s1[i] == s2[i];
            ++n;
            if (!ok) {
                printf("decode mismatch k=%d m=%d bytes=%d e=%d\n", k, m, B, e);
                ++bad;
            }
        }
    }
    printf("%d checks, %d mismatches (isa %s)\n", n, bad, lh::host::isa_name());
    return bad != 0;
}
