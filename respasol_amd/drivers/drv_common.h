/*
 * drv_common.h — helpers shared by the reference-CLI drivers (test_spmv,
 * test_ilu0, test_spmv_cpu): matrix acquisition (a .mtx path through the
 * reference-compatible loader, or "surrogate:NAME[@scale]" for the seeded
 * stand-ins), flag parsing for the options appended after the reference's
 * positional arguments, and wall-clock timing.
 */
#ifndef RSP_DRV_COMMON_H
#define RSP_DRV_COMMON_H

#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "rsp_host.h"

static inline double drv_wtime(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

/* "--key=value" lookup over argv[first..argc). Returns NULL if absent; for a
 * bare "--key" returns "". */
static inline const char *drv_flag(int argc, char **argv, int first, const char *key) {
    size_t kl = strlen(key);
    for (int i = first; i < argc; i++) {
        const char *a = argv[i];
        if (strncmp(a, "--", 2) != 0) continue;
        if (strncmp(a + 2, key, kl) != 0) continue;
        if (a[2 + kl] == '=') return a + 3 + kl;
        if (a[2 + kl] == '\0') return "";
    }
    return NULL;
}

/* Acquire the matrix named by `spec`: a Matrix-Market path (reference loader
 * semantics, loadMatrixMarket.cpp:47-253, with outputBase/transpose) or
 * "surrogate:NAME[@scale]" (base 0 only). Returns 1 on success like the
 * reference loader; exits(-1) on a missing file like the reference. */
static inline int drv_load(const char *spec, CSR *A, int base, int full_symmetric) {
    if (strncmp(spec, "surrogate:", 10) == 0) {
        char name[256];
        double scale = 1.0;
        snprintf(name, sizeof(name), "%s", spec + 10);
        char *at = strchr(name, '@');
        if (at) {
            *at = '\0';
            scale = atof(at + 1);
        }
        if (rsp_surrogate_csr(name, scale, 0, A) != 0) {
            fprintf(stderr, "Error: unknown surrogate %s\n", name);
            return 0;
        }
        if (base != 0) {
            for (int i = 0; i <= A->m; i++) A->rowptr[i] += base;
            for (int k = 0; k < A->nnz; k++) A->colidx[k] += base;
        }
        return 1;
    }
    int st = rsp_mm_load(spec, A, base, 0, full_symmetric ? RSP_MM_FULL_SYMMETRIC : 0);
    if (st == RSP_MM_OPEN_FAILED) exit(-1);
    return st == RSP_MM_OK;
}

#endif
