/*
 * fmath_libm_check.c — include/bre_fmath.h against the host libm (test infrastructure).
 *
 * The reference calls std::exp / std::log / std::sin / std::cos on floats, i.e. libm's expf, logf,
 * sinf and cosf (spectrum.h:222-224, homogeneous.cpp:47,74, grid.cpp:76,104, sampling.cpp:127,
 * geometry.h SphericalDirection via medium.cpp:194-213).  This program evaluates bre_expf, bre_logf
 * and bre_sincosf (and that the pair equals bre_sinf / bre_cosf) and the libm functions on every
 * STRIDE-th float bit pattern (stride 1: all 2^32) in THREADS threads and counts the results that
 * differ in any bit (two NaNs count as equal).
 *
 *   fmath_libm_check STRIDE THREADS    -> one line per function, exit status 1 if any differ
 *
 * Build: gcc -O2 -ffp-contract=off -fno-builtin -pthread -I include tests/fmath_libm_check.c -lm
 */
#include <math.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>

#include "bre_fmath.h"

typedef struct {
    uint64_t begin, end, stride;
    uint64_t tested, bad[4];
    uint32_t first_bad[4];
} Job;

static int same(float a, float b) { return bre_f2u(a) == bre_f2u(b) || (a != a && b != b); }

static void *run(void *arg) {
    Job *j = (Job *)arg;
    for (uint64_t u = j->begin; u < j->end; u += j->stride) {
        const float x = bre_u2f((uint32_t)u);
        float s, c;
        bre_sincosf(x, &s, &c);
        const float mine[4] = {bre_expf(x), bre_logf(x), s, c};
        const float ref[4] = {expf(x), logf(x), sinf(x), cosf(x)};
        for (int k = 0; k < 4; ++k)
            if (!same(mine[k], ref[k]) && j->bad[k]++ == 0) j->first_bad[k] = (uint32_t)u;
        /* the one-reduction pair equals the two functions (the photon pass calls the pair) */
        if ((!same(s, bre_sinf(x)) || !same(c, bre_cosf(x))) && j->bad[2]++ == 0) j->first_bad[2] = (uint32_t)u;
        ++j->tested;
    }
    return NULL;
}

int main(int argc, char **argv) {
    const uint64_t stride = argc > 1 ? strtoull(argv[1], NULL, 0) : 1;
    int threads = argc > 2 ? atoi(argv[2]) : 8;
    if (stride == 0 || threads < 1 || threads > 256) return 2;
    const uint64_t total = 1ull << 32, span = (total / stride + threads - 1) / threads * stride;
    Job jobs[256];
    pthread_t th[256];
    for (int t = 0; t < threads; ++t) {
        Job *j = &jobs[t];
        j->begin = (uint64_t)t * span;
        j->end = j->begin + span < total ? j->begin + span : total;
        j->stride = stride;
        j->tested = 0;
        for (int k = 0; k < 4; ++k) j->bad[k] = 0, j->first_bad[k] = 0;
        pthread_create(&th[t], NULL, run, j);
    }
    uint64_t tested = 0, bad[4] = {0, 0, 0, 0};
    uint32_t first[4] = {0, 0, 0, 0};
    for (int t = 0; t < threads; ++t) {
        pthread_join(th[t], NULL);
        tested += jobs[t].tested;
        for (int k = 0; k < 4; ++k) {
            if (jobs[t].bad[k] && !bad[k]) first[k] = jobs[t].first_bad[k];
            bad[k] += jobs[t].bad[k];
        }
    }
    const char *name[4] = {"expf", "logf", "sinf", "cosf"};
    int rc = 0;
    for (int k = 0; k < 4; ++k) {
        printf("%s: %llu of %llu inputs differ from libm", name[k], (unsigned long long)bad[k],
               (unsigned long long)tested);
        if (bad[k]) printf(" (first 0x%08x)", first[k]), rc = 1;
        printf("\n");
    }
    return rc;
}
