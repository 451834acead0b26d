/*
 * oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C, single-threaded restatement of the reference codec's algorithm
 * (catid/longhair, cauchy_256.cpp).  It is the checker for the HIP product path:
 * only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.
 * The product library (longhair_amd/liblonghair_amd.so) never links or calls it.
 *
 * Parity pinning: golden fixtures in tests/golden/ were produced by the reference
 * itself (oracle/_ref/liblonghair_ref.so, compiled from /root/reference sources by
 * oracle/Makefile); tests check this restatement against those fixtures.
 */
#ifndef LH_ORACLE_H
#define LH_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Same layout as the reference Block (cauchy_256.h:52-55). */
typedef struct lho_block {
    unsigned char *data;
    unsigned char row;
} lho_block;

/* Load the Cauchy constants blob (34902 bytes, see tools/extract_tables.py) and build
 * the GF(256)/0x187 tables from the polynomial.  Returns 0 on success, -1 otherwise. */
int lho_init(const unsigned char *tables_blob, size_t len);

/* cauchy_256_encode restated (cauchy_256.cpp:1495-1594). */
int lho_encode(int k, int m, const unsigned char *const *data, unsigned char *recovery, int bytes);

/* cauchy_256_decode restated (cauchy_256.cpp:1249-1408), using the non-windowed
 * elimination + GF(2) Gaussian elimination + back substitution. */
int lho_decode(int k, int m, lho_block *blocks, int bytes);

/* Generator rows 1..m-1 for (k, m), written compactly as (m-1) x k bytes
 * (cauchy_256.cpp:423-481).  Precondition: m > 1, k + m <= 256. */
void lho_cauchy_rows(int k, int m, unsigned char *out);

/* GF(256) helpers with polynomial 0x187. */
unsigned char lho_mul(unsigned char a, unsigned char b);
unsigned char lho_div(unsigned char a, unsigned char b);
unsigned char lho_inv(unsigned char a);

#ifdef __cplusplus
}
#endif

#endif
