// field.cpp -- see field.hpp.
#include "field.hpp"

#include <cstring>
#include <stdexcept>

namespace lh {

Field::Field() {
    uint8_t v = 1;
    for (int i = 0; i < 255; ++i) {
        exp[i] = exp[i + 255] = v;
        log[v] = (int16_t)i;
        v = xtime(v);
    }
    exp[510] = exp[511] = 0;
    log[0] = 0;
    inv[0] = 0;
    for (int i = 1; i < 256; ++i) inv[i] = exp[255 - log[i]];
}

const Field &Field::get() {
    static const Field f;
    return f;
}

// Blob layout written by tools/extract_tables.py:
//   M2 (254) | M3 (506) | M4 (756) | M5 (1004) | M6 (1250) | Y (256) | X (30876)
std::vector<uint8_t> generator_matrix(int k, int m) {
    if (lh_cauchy_tables_blob_end - lh_cauchy_tables_blob != kTablesBlobSize)
        throw std::runtime_error("longhair_amd: Cauchy constants blob has the wrong size");
    static const int offs[7] = {0, 0, 0, 254, 760, 1516, 2520};
    const unsigned char *Y = lh_cauchy_tables_blob + 3770;
    const unsigned char *Xall = lh_cauchy_tables_blob + 4026;
    const Field &F = Field::get();

    std::vector<uint8_t> g((size_t)k * m);
    for (int x = 0; x < k; ++x) g[x] = 1;
    if (m <= 1) return g;
    if (m <= 6) {
        // Improved rows stored with stride 256 - m (cauchy_256.cpp:428-444).
        const unsigned char *t = lh_cauchy_tables_blob + offs[m];
        const int stride = 256 - m;
        for (int r = 1; r < m; ++r)
            for (int x = 0; x < k; ++x) g[(size_t)r * k + x] = t[(r - 1) * stride + x];
        return g;
    }
    // m >= 7: element(r, x) = X_x / (X_x + Y_{r-1}), X_0 = 1 (cauchy_256.cpp:453-478).
    const int n = m - 7;
    const unsigned char *X = Xall + n * 249 - n * (n + 1) / 2;
    for (int r = 1; r < m; ++r) {
        const uint8_t G = Y[r - 1];
        g[(size_t)r * k] = F.inv[1 ^ G];
        for (int x = 1; x < k; ++x) {
            const uint8_t B = X[x - 1];
            g[(size_t)r * k + x] = F.div(B, (uint8_t)(B ^ G));
        }
    }
    return g;
}

// Cauchy points of the m >= 7 generators: element(r, x) = X_x / (X_x + Y'_r) with
// X_0 = 1, Y'_0 = 0 (the all-ones row) and Y'_r = Y_{r-1}.  The decode planner inverts
// e x e submatrices of this form in closed form.  Checked against the generator itself;
// false (no closed form) for m < 7, whose rows are tabulated (cauchy_256.cpp:428-444).
bool cauchy_points(int k, int m, std::vector<uint8_t> &xs, std::vector<uint8_t> &ys) {
    if (m < 7 || k < 1) return false;
    const unsigned char *Y = lh_cauchy_tables_blob + 3770;
    const unsigned char *Xall = lh_cauchy_tables_blob + 4026;
    const int n = m - 7;
    const unsigned char *X = Xall + n * 249 - n * (n + 1) / 2;
    xs.assign((size_t)k, 1);
    ys.assign((size_t)m, 0);
    for (int x = 1; x < k; ++x) xs[x] = X[x - 1];
    for (int r = 1; r < m; ++r) ys[r] = Y[r - 1];
    const Field &F = Field::get();
    const std::vector<uint8_t> g = generator_matrix(k, m);
    for (int r = 0; r < m; ++r)
        for (int x = 0; x < k; ++x) {
            const uint8_t d = (uint8_t)(xs[x] ^ ys[r]);
            if (!xs[x] || !d || g[(size_t)r * k + x] != F.div(xs[x], d)) return false;
        }
    return true;
}

}  // namespace lh
