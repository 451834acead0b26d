/*
 * cpu_bench.c -- TEST/BENCH INFRASTRUCTURE ONLY: times a CPU codec with the reference
 * ABI (the reference itself from oracle/_ref, or the oracle restatement) over a batch of
 * stripes, split across pthreads.  Used by bench.py's cpu_baseline leg.
 *
 * One "step" per stripe = cauchy_256_encode of the k data blocks, then
 * cauchy_256_decode of k-e surviving originals + e recovery blocks (decoded in place), as
 * the reference test does per (k, m, e) (tests/cauchy_256_tests.cpp:265-324).  The
 * erasure count e and the recovery rows may differ per stripe (lhb_run_pattern: the same
 * erasure patterns as the GPU workload the baseline is reported beside).
 */
#define _POSIX_C_SOURCE 199309L
#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "oracle.h"

typedef int (*enc_fn)(int, int, const unsigned char **, void *, int);
typedef int (*dec_fn)(int, int, lho_block *, int);

typedef struct {
    enc_fn enc;
    dec_fn dec;
    int k, m, bytes, e, s0, s1, passes;
    const unsigned char *data;    /* [stripes][k][bytes] */
    const unsigned char *erased;  /* [stripes][e] erased original rows */
    const unsigned char *e_of;    /* optional [stripes]: erasures of stripe s (<= e) */
    const unsigned char *rec_row; /* optional [stripes][e]: recovery row indices (else 0..e-1) */
    int ok;
} job_t;

static void *worker(void *arg) {
    job_t *j = (job_t *)arg;
    const int k = j->k, m = j->m, bytes = j->bytes, e_max = j->e;
    unsigned char *rec = (unsigned char *)malloc((size_t)m * bytes);
    const unsigned char **ptrs = (const unsigned char **)malloc(sizeof(void *) * (size_t)k);
    lho_block *blocks = (lho_block *)malloc(sizeof(lho_block) * (size_t)k);
    unsigned char is_erased[256];
    int p, s, x, i;
    j->ok = 1;
    for (p = 0; p < j->passes; ++p) {
        for (s = j->s0; s < j->s1; ++s) {
            const unsigned char *d = j->data + (size_t)s * k * bytes;
            for (x = 0; x < k; ++x) ptrs[x] = d + (size_t)x * bytes;
            if (j->enc(k, m, ptrs, rec, bytes) != 0) j->ok = 0;
            const int e = j->e_of ? j->e_of[s] : e_max;
            memset(is_erased, 0, sizeof(is_erased));
            for (i = 0; i < e; ++i) is_erased[j->erased[(size_t)s * e_max + i]] = 1;
            for (x = 0, i = 0; x < k; ++x)
                if (!is_erased[x]) { blocks[i].data = (unsigned char *)ptrs[x]; blocks[i].row = (unsigned char)x; ++i; }
            for (x = 0; x < e; ++x, ++i) {
                const int r = j->rec_row ? j->rec_row[(size_t)s * e_max + x] : x;
                blocks[i].data = rec + (size_t)r * bytes;
                blocks[i].row = (unsigned char)(k + r);
            }
            if (j->dec(k, m, blocks, bytes) != 0) j->ok = 0;
            if (p == 0)
                for (i = 0; i < k; ++i)
                    if (memcmp(blocks[i].data, d + (size_t)blocks[i].row * bytes, (size_t)bytes) != 0) j->ok = 0;
        }
    }
    free(rec);
    free(ptrs);
    free(blocks);
    return NULL;
}

/* Returns wall seconds; *ok = 1 if every call succeeded and decoded data matched;
 * *cpu_seconds = CPU time the process consumed over the timed region (all threads,
 * CLOCK_PROCESS_CPUTIME_ID), so a thread count above the cores actually granted shows. */
double lhb_run_pattern(void *enc, void *dec, int k, int m, int bytes, int stripes, const unsigned char *data,
                       const unsigned char *erased, const unsigned char *e_of, const unsigned char *rec_row,
                       int e, int threads, int passes, int *ok, double *cpu_seconds) {
    pthread_t tid[1024];
    job_t jobs[1024];
    struct timespec t0, t1, c0, c1;
    int t;
    if (threads < 1) threads = 1;
    if (threads > 1024) threads = 1024;
    for (t = 0; t < threads; ++t) {
        jobs[t].enc = (enc_fn)enc;
        jobs[t].dec = (dec_fn)dec;
        jobs[t].k = k; jobs[t].m = m; jobs[t].bytes = bytes; jobs[t].e = e;
        jobs[t].s0 = (int)((long long)stripes * t / threads);
        jobs[t].s1 = (int)((long long)stripes * (t + 1) / threads);
        jobs[t].passes = passes;
        jobs[t].data = data;
        jobs[t].erased = erased;
        jobs[t].e_of = e_of;
        jobs[t].rec_row = rec_row;
    }
    clock_gettime(CLOCK_PROCESS_CPUTIME_ID, &c0);
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (t = 0; t < threads; ++t) pthread_create(&tid[t], NULL, worker, &jobs[t]);
    for (t = 0; t < threads; ++t) pthread_join(tid[t], NULL);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    clock_gettime(CLOCK_PROCESS_CPUTIME_ID, &c1);
    if (cpu_seconds) *cpu_seconds = (double)(c1.tv_sec - c0.tv_sec) + 1e-9 * (double)(c1.tv_nsec - c0.tv_nsec);
    *ok = 1;
    for (t = 0; t < threads; ++t) *ok &= jobs[t].ok;
    return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}

/* Every stripe with e erasures, recovery rows 0 .. e-1. */
double lhb_run(void *enc, void *dec, int k, int m, int bytes, int stripes, const unsigned char *data,
               const unsigned char *erased, int e, int threads, int passes, int *ok, double *cpu_seconds) {
    return lhb_run_pattern(enc, dec, k, m, bytes, stripes, data, erased, NULL, NULL, e, threads, passes, ok,
                           cpu_seconds);
}
