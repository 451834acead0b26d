/*
 * c_caller.c -- TEST PROGRAM: a plain C caller of the drop-in boundary, compiled against
 * include/cauchy_256.h (+ cauchy_256_dispatch.h) and linked with -llonghair_amd, exactly as
 * a user of the reference would build.
 *
 * stdin: one case per line, "k m block_bytes seed".  For each case: data = the fixture
 * byte spec (tests/lhutil.py fill: little-endian splitmix64 words of seed * 2^32 + i),
 * cauchy_256_encode, then the return code (int32 LE) and the m * block_bytes recovery
 * bytes are appended to OUT_FILE (the test compares them with the reference's goldens and
 * the oracle).  When encode succeeds and k > 1, a decode round trip in the style of the
 * reference's order_test (tests/cauchy_256_tests.cpp:122-205, restated here): min(k, m)
 * random originals are removed from the Block array (later entries shift down) and a
 * recovery block is appended in their place; decode must return 0 and every Block must
 * then hold the original of its row.  Exit status 0 = every round trip restored its data.
 *
 * Usage: c_caller default|gpu|auto|host OUT_FILE < cases
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "cauchy_256.h"
#include "cauchy_256_dispatch.h"

static uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

static void fill(uint32_t seed, unsigned char *out, size_t n) {
    size_t i;
    for (i = 0; i < n; i += 8) {
        uint64_t w = splitmix64(((uint64_t)seed << 32) + i / 8);
        size_t j;
        for (j = 0; j < 8 && i + j < n; ++j) out[i + j] = (unsigned char)(w >> (8 * j));
    }
}

int main(int argc, char **argv) {
    int k, m, bytes, failures = 0, cases = 0;
    unsigned seed;
    uint64_t prng = 0x243F6A8885A308D3ull;
    FILE *out;
    if (argc < 3) {
        fprintf(stderr, "usage: %s default|gpu|auto|host OUT_FILE < cases\n", argv[0]);
        return 2;
    }
    if (cauchy_256_init() != 0) {
        fprintf(stderr, "cauchy_256_init failed\n");
        return 2;
    }
    /* "default": an unchanged reference caller, whatever policy the library starts with */
    if (strcmp(argv[1], "default") != 0)
        cauchy_256_set_dispatch(strcmp(argv[1], "host") == 0   ? CAUCHY_256_DISPATCH_HOST
                                : strcmp(argv[1], "auto") == 0 ? CAUCHY_256_DISPATCH_AUTO
                                                               : CAUCHY_256_DISPATCH_GPU,
                                -1);
    out = fopen(argv[2], "wb");
    if (!out) return 2;
    while (scanf("%d %d %d %u", &k, &m, &bytes, &seed) == 4) {
        unsigned char *data = (unsigned char *)malloc((size_t)k * bytes);
        unsigned char *rec = (unsigned char *)calloc((size_t)m * bytes + 1, 1);
        const unsigned char *data_ptrs[256];
        Block blocks[256];
        int32_t rc;
        int x;
        fill(seed, data, (size_t)k * bytes);
        for (x = 0; x < k; ++x) data_ptrs[x] = data + (size_t)x * bytes;
        rc = cauchy_256_encode(k, m, data_ptrs, rec, bytes);
        fwrite(&rc, sizeof(rc), 1, out);
        fwrite(rec, 1, (size_t)m * bytes, out);
        ++cases;
        if (rc == 0 && k > 1) {
            int rem = k, ii, e = k < m ? k : m;
            for (x = 0; x < k; ++x) {
                blocks[x].data = (unsigned char *)data_ptrs[x];
                blocks[x].row = (unsigned char)x;
            }
            /* decode writes the recovered originals into the recovery buffers (the
             * surviving originals are only read), so `data` stays the reference copy. */
            for (ii = 0; ii < e; ++ii) {
                int jj, kk;
                prng = splitmix64(prng);
                jj = (int)(prng % (uint64_t)rem);
                --rem;
                for (kk = jj; kk < rem; ++kk) blocks[kk] = blocks[kk + 1];
                blocks[rem].data = rec + (size_t)ii * bytes;
                blocks[rem].row = (unsigned char)(k + ii);
            }
            if (cauchy_256_decode(k, m, blocks, bytes) != 0) {
                fprintf(stderr, "decode failed k=%d m=%d bytes=%d\n", k, m, bytes);
                ++failures;
            } else {
                for (x = 0; x < k; ++x)
                    if (blocks[x].row >= k || memcmp(blocks[x].data, data_ptrs[blocks[x].row], (size_t)bytes) != 0) {
                        fprintf(stderr, "round trip mismatch k=%d m=%d bytes=%d slot %d row %d\n", k, m, bytes, x,
                                blocks[x].row);
                        ++failures;
                        break;
                    }
            }
        }
        free(data);
        free(rec);
    }
    fclose(out);
    printf("%d cases, %d round-trip failures (policy %s, host isa %s)\n", cases, failures, argv[1],
           cauchy_256_host_isa());
    return failures ? 1 : 0;
}
