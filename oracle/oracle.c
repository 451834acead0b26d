/*
 * oracle.c -- TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * Plain-C restatement of catid/longhair's Cauchy Reed-Solomon codec.  Every function
 * cites the reference lines it restates (paths relative to the reference root).  It
 * favours obviousness over speed: every sub-block XOR is a byte loop.
 */
#include "oracle.h"

#include <stdlib.h>
#include <string.h>

/* ---------------------------------------------------------------- GF(256), 0x187 */
/* cauchy_256.cpp:273-413 hard-codes LOG/EXP/INV tables for the polynomial 0x187 and
 * derives MUL/DIV tables from them.  Here they are regenerated from the polynomial:
 * 2 is a generator, xtime(v) = (v << 1) ^ (v & 0x80 ? 0x87 : 0). */
static unsigned char g_exp[512];
static int g_log[256];
static unsigned char g_inv[256];

/* Constants blob layout (tools/extract_tables.py). */
static unsigned char g_tab[34902];
static const unsigned char *g_m[7]; /* g_m[2..6] */
static const unsigned char *g_y, *g_x;
static int g_ready;

static unsigned char xtime(unsigned char v) {
    return (unsigned char)((v << 1) ^ ((v & 0x80) ? 0x87 : 0));
}

unsigned char lho_mul(unsigned char a, unsigned char b) {
    if (!a || !b) return 0;
    return g_exp[g_log[a] + g_log[b]];
}

unsigned char lho_inv(unsigned char a) { return g_inv[a]; }

/* GFC256Divide semantics (cauchy_256.cpp:349-388, 410-413): x/0 == 0. */
unsigned char lho_div(unsigned char a, unsigned char b) {
    if (!a || !b) return 0;
    return g_exp[g_log[a] + 255 - g_log[b]];
}

int lho_init(const unsigned char *blob, size_t len) {
    static const int sizes[7] = {254, 506, 756, 1004, 1250, 256, 30876};
    size_t off = 0;
    unsigned char v = 1;
    int i;
    if (len != sizeof(g_tab)) return -1;
    memcpy(g_tab, blob, len);
    for (i = 0; i < 5; ++i) {
        g_m[i + 2] = g_tab + off;
        off += (size_t)sizes[i];
    }
    g_y = g_tab + off;
    off += 256;
    g_x = g_tab + off;
    for (i = 0; i < 255; ++i) {
        g_exp[i] = g_exp[i + 255] = v;
        g_log[v] = i;
        v = xtime(v);
    }
    g_exp[510] = g_exp[511] = 0;
    g_log[0] = 0;
    g_inv[0] = 0;
    for (i = 1; i < 256; ++i) g_inv[i] = g_exp[255 - g_log[i]];
    g_ready = 1;
    return 0;
}

/* ------------------------------------------------------------- generator rows */
/* cauchy_256.cpp:423-481.  m = 2..6 use the improved tables with stride 256 - m;
 * m >= 7 rebuild rows from X/Y: element(y, x) = X_x / (X_x ^ Y_{y-1}) with X_0 = 1. */
static const unsigned char *generator(int k, int m, int *stride, unsigned char **heap) {
    int y, x, n;
    const unsigned char *X;
    unsigned char *mat;
    *heap = NULL;
    if (m >= 2 && m <= 6) {
        *stride = 256 - m;
        return g_m[m];
    }
    mat = (unsigned char *)malloc((size_t)k * (size_t)(m - 1));
    n = m - 7;
    X = g_x + n * 249 - n * (n + 1) / 2;
    for (y = 1; y < m; ++y) {
        unsigned char G = g_y[y - 1];
        mat[(y - 1) * k] = g_inv[1 ^ G];
        for (x = 1; x < k; ++x) {
            unsigned char B = X[x - 1];
            mat[(y - 1) * k + x] = lho_div(B, (unsigned char)(B ^ G));
        }
    }
    *stride = k;
    *heap = mat;
    return mat;
}

void lho_cauchy_rows(int k, int m, unsigned char *out) {
    int stride, r, x;
    unsigned char *heap;
    const unsigned char *g = generator(k, m, &stride, &heap);
    for (r = 0; r < m - 1; ++r)
        for (x = 0; x < k; ++x) out[r * k + x] = g[r * stride + x];
    free(heap);
}

static void xor_into(unsigned char *dst, const unsigned char *src, int n) {
    int i;
    for (i = 0; i < n; ++i) dst[i] ^= src[i];
}

/* ------------------------------------------------------------------- encoder */
/* cauchy_256.cpp:1495-1594 (the m > 4 windowed path, :1414-1493, yields the same
 * bytes; it is restated here by the plain bit loop of :1553-1587). */
int lho_encode(int k, int m, const unsigned char *const *data, unsigned char *rec, int bytes) {
    int x, r, y, b, stride, sub;
    unsigned char *heap;
    const unsigned char *g;
    if (k <= 1) { /* :1501-1509 */
        for (r = 0; r < m; ++r) memcpy(rec + (size_t)r * bytes, data[0], (size_t)bytes);
        return 0;
    }
    /* Row 0 = XOR of all data blocks, written before any validation (:1511-1516). */
    memcpy(rec, data[0], (size_t)bytes);
    for (x = 1; x < k; ++x) xor_into(rec, data[x], bytes);
    if (m == 1) return 0; /* :1519-1522 */
    if (k + m > 256 || (bytes % 8) != 0) return -1; /* :1525-1527 */
    g = generator(k, m, &stride, &heap);
    sub = bytes / 8;
    memset(rec + bytes, 0, (size_t)bytes * (size_t)(m - 1));
    for (r = 1; r < m; ++r) {
        unsigned char *out = rec + (size_t)r * bytes;
        for (x = 0; x < k; ++x) {
            unsigned char s = g[(r - 1) * stride + x];
            /* Bit-row y of element s is s * 2^y; bit b selects data sub-block b. */
            for (y = 0; y < 8; ++y, s = xtime(s))
                for (b = 0; b < 8; ++b)
                    if (s & (1u << b)) xor_into(out + y * sub, data[x] + b * sub, sub);
        }
    }
    free(heap);
    return 0;
}

/* ------------------------------------------------------------------- decoder */
/* cauchy_256.cpp:487-535: m == 1.  The (single) recovery block takes the missing row
 * and becomes the XOR of all other blocks.  With no recovery block present the
 * reference leaves `erased` at blocks[0] and XORs the others into it; kept as-is. */
static void decode_m1(int k, lho_block *blocks, int bytes) {
    unsigned char present[256];
    lho_block *erased = blocks;
    int i;
    memset(present, 0, sizeof(present));
    for (i = 0; i < k; ++i) {
        if (blocks[i].row >= k) erased = &blocks[i];
        else present[blocks[i].row] = 1;
    }
    for (i = 0; i < k; ++i)
        if (!present[i]) { erased->row = (unsigned char)i; break; }
    for (i = 0; i < k; ++i)
        if (&blocks[i] != erased) xor_into(erased->data, blocks[i].data, bytes);
}

int lho_decode(int k, int m, lho_block *blocks, int bytes) {
    lho_block *orig[256], *rcv[256];
    unsigned char seen[256], erasures[256];
    int n_orig = 0, n_rcv = 0, i, j, sub, stride, bitrows, words, pivot;
    unsigned char *heap;
    const unsigned char *g;
    uint64_t *bm;

    if (k <= 1) { blocks[0].row = 0; return 0; } /* :1251-1256 */
    if (m == 1) { decode_m1(k, blocks, bytes); return 0; } /* :1259-1262 */

    /* sort_blocks, :538-570: array order split; erasures = first n_rcv missing rows,
     * ascending. */
    memset(seen, 0, sizeof(seen));
    for (i = 0; i < k; ++i) {
        if (blocks[i].row < k) { orig[n_orig++] = &blocks[i]; seen[blocks[i].row] = 1; }
        else rcv[n_rcv++] = &blocks[i];
    }
    for (i = 0, j = 0; i < 256 && j < n_rcv; ++i)
        if (!seen[i]) erasures[j++] = (unsigned char)i;

    if (n_rcv <= 0) return 0; /* :1282-1284 */
    if (k + m > 256 || (bytes % 8) != 0) return -1; /* :1287-1289 */

    g = generator(k, m, &stride, &heap);
    sub = bytes / 8;

    /* eliminate_original, :650-705: R_j ^= B(G[r_j][x]) D_x for each surviving x.
     * Recovery row k (matrix row -1) is the all-ones row: identity elements. */
    for (i = 0; i < n_rcv; ++i) {
        int mrow = rcv[i]->row - (k + 1);
        for (j = 0; j < n_orig; ++j) {
            int x = orig[j]->row, y, b;
            unsigned char s = (mrow < 0) ? 1 : g[mrow * stride + x];
            for (y = 0; y < 8; ++y, s = xtime(s))
                for (b = 0; b < 8; ++b)
                    if (s & (1u << b))
                        xor_into(rcv[i]->data + y * sub, orig[j]->data + b * sub, sub);
        }
    }

    /* generate_bitmatrix, :707-790: bit-row 8i+y, bit-column 8j+b is bit b of
     * A[i][j] * 2^y with A[i][j] = G[r_i][erasures[j]]; recovery i takes row erasures[i]. */
    bitrows = 8 * n_rcv;
    words = (bitrows + 63) / 64;
    bm = (uint64_t *)calloc((size_t)bitrows * (size_t)words, sizeof(uint64_t));
    for (i = 0; i < n_rcv; ++i) {
        int rrow = rcv[i]->row - k;
        for (j = 0; j < n_rcv; ++j) {
            unsigned char s = (rrow == 0) ? 1 : g[(rrow - 1) * stride + erasures[j]];
            int y;
            for (y = 0; y < 8; ++y, s = xtime(s)) {
                int col = 8 * j;
                bm[(8 * i + y) * words + col / 64] |= (uint64_t)s << (col % 64);
            }
        }
        rcv[i]->row = erasures[i];
    }

    /* gaussian_elimination, :1018-1080: forward elimination to upper-triangular form,
     * each bit-row operation mirrored on the recovery sub-blocks (bit-row r lives in
     * recovery block r/8, sub-block r%8). */
    for (pivot = 0; pivot < bitrows - 1; ++pivot) {
        int w = pivot / 64, opt;
        uint64_t mask = (uint64_t)1 << (pivot % 64);
        for (opt = pivot; opt < bitrows; ++opt) {
            if (bm[opt * words + w] & mask) {
                unsigned char *src = rcv[pivot / 8]->data + (pivot % 8) * sub;
                int other;
                if (opt != pivot) {
                    unsigned char *od = rcv[opt / 8]->data + (opt % 8) * sub;
                    int t;
                    for (t = 0; t < sub; ++t) { unsigned char c = src[t]; src[t] = od[t]; od[t] = c; }
                    for (t = w; t < words; ++t) {
                        uint64_t c = bm[pivot * words + t];
                        bm[pivot * words + t] = bm[opt * words + t];
                        bm[opt * words + t] = c;
                    }
                }
                for (other = opt + 1; other < bitrows; ++other) {
                    if (bm[other * words + w] & mask) {
                        int t;
                        for (t = w; t < words; ++t) bm[other * words + t] ^= bm[pivot * words + t];
                        xor_into(rcv[other / 8]->data + (other % 8) * sub, src, sub);
                    }
                }
                break;
            }
        }
    }
    /* back_substitution, :1229-1247. */
    for (pivot = bitrows - 1; pivot > 0; --pivot) {
        const unsigned char *src = rcv[pivot / 8]->data + (pivot % 8) * sub;
        uint64_t mask = (uint64_t)1 << (pivot % 64);
        int other;
        for (other = pivot - 1; other >= 0; --other)
            if (bm[other * words + pivot / 64] & mask)
                xor_into(rcv[other / 8]->data + (other % 8) * sub, src, sub);
    }
    free(bm);
    free(heap);
    return 0;
}
