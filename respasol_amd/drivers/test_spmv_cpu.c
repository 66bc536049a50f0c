/*
 * test_spmv_cpu.c — CPU SpMV driver with the CLI and CSV schema of
 * ReSpaSol's test_spmv.c (the CPU reference path).
 *
 *   OMP_NUM_THREADS=T test_spmv_cpu <A.mtx | surrogate:NAME[@scale]> <out.csv> [--reps=N]
 *
 * Appends one CSV row `threads,name,t64,t32,err,<%c date>,` (test_spmv.c:49-62,
 * 173,183,208,218-220): threads = $OMP_NUM_THREADS, name = the first word run
 * followed by ".mtx" in the path (the regex `(\w+)\.mtx`, :57-62, so
 * matrix-new_3 -> new_3), t64/t32 = seconds of one cold fp64 / fp32 SpMV each
 * (:165-183; --reps=N reports the mean of N warm calls instead), err = mean
 * |y64 - y32| over m (:200-208). x = dlarnv(1, {0,0,0,1}) (:74-76); the fp32
 * copies are (float) round-to-nearest with the reference's positive-overflow
 * message (:109-145).
 * The SpMV is the OpenMP CSR kernel of librsp_host (MKL is not part of this
 * build). Deliberate differences, all documented in DESIGN.md: the product is
 * the correct base-0 A*x (the reference hands 1-based arrays to MKL as
 * base 0, :54-55,91-92, and computes a shifted product — SURVEY §0.4); the
 * error sum is a proper reduction (the reference's `error +=` races, :202-205);
 * an unset OMP_NUM_THREADS writes an empty field (the reference streams a
 * NULL char*, which fails the stream and drops the whole row, :51).
 */
#include <float.h>
#include <math.h>
#include <omp.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "drv_common.h"
#include "rsp_host.h"

static int is_word(char c) {
    return (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || (c >= '0' && c <= '9') || c == '_';
}

/* leftmost match of (\w+)\.mtx -> group 1 */
static void matrix_name(const char *path, char *out, size_t cap) {
    out[0] = '\0';
    size_t n = strlen(path);
    for (size_t a = 0; a < n; a++) {
        if (!is_word(path[a])) continue;
        size_t e = a;
        while (e < n && is_word(path[e])) e++;
        if (strncmp(path + e, ".mtx", 4) == 0) {
            size_t len = e - a < cap - 1 ? e - a : cap - 1;
            memcpy(out, path + a, len);
            out[len] = '\0';
            return;
        }
        a = e; /* later starts inside this run cannot match either */
    }
}

int main(int argc, char **argv) {
    if (argc < 3) {
        fprintf(stderr,
                "-- Usage examples --\n"
                "  %s inline_1.mtx type: run with inline_1 matrix in matrix market "
                "format\n",
                argv[0]);
        return -1;
    }
    const char *reps_s = drv_flag(argc, argv, 3, "reps");
    int reps = reps_s && *reps_s ? atoi(reps_s) : 0;

    FILE *fout = fopen(argv[2], "a");
    if (!fout) {
        fprintf(stderr, "Failed to open %s\n", argv[2]);
        return 1;
    }
    const char *thr = getenv("OMP_NUM_THREADS");
    fprintf(fout, "%s,", thr ? thr : "");

    CSR A;
    if (!drv_load(argv[1], &A, 0, 0)) {
        fprintf(stderr, "Error: failed to load %s\n", argv[1]);
        fclose(fout);
        return 1;
    }
    char name[256];
    if (strncmp(argv[1], "surrogate:", 10) == 0) {
        snprintf(name, sizeof(name), "%s", argv[1] + 10);
        char *at = strchr(name, '@');
        if (at) *at = '\0';
    } else {
        matrix_name(argv[1], name, sizeof(name));
    }
    fprintf(fout, "%s,", name);

    const int m = A.m;
    const int nnz = A.rowptr[m];
    double *x = (double *)malloc(sizeof(double) * (size_t)(A.n > m ? A.n : m));
    double *y = (double *)malloc(sizeof(double) * (size_t)(m ? m : 1));
    int seed[4] = {0, 0, 0, 1};
    rsp_dlarnv(1, seed, A.n > m ? A.n : m, x);

    const double RMAX = (double)FLT_MAX; /* LAPACKE_slamch('O') */
    float *x32 = (float *)malloc(sizeof(float) * (size_t)(A.n > m ? A.n : m));
    float *y32 = (float *)malloc(sizeof(float) * (size_t)(m ? m : 1));
    float *v32 = (float *)malloc(sizeof(float) * (size_t)(nnz ? nnz : 1));
    int overflow = 0;
    for (int k = 0; k < nnz; k++) {
        if (A.values[k] > RMAX) overflow = 1;
        v32[k] = (float)A.values[k];
    }
    if (overflow) printf("Conversion of A overflow\n");
    overflow = 0;
    for (int k = 0; k < (A.n > m ? A.n : m); k++) {
        if (x[k] > RMAX) overflow = 1;
        x32[k] = (float)x[k];
    }
    if (overflow) printf("Conversion of X overflow\n");

    double t, t64, t32;
    if (reps > 0) {
        rsp_host_spmv_f64(m, A.rowptr, A.colidx, A.values, x, y); /* warm */
        t = omp_get_wtime();
        for (int r = 0; r < reps; r++) rsp_host_spmv_f64(m, A.rowptr, A.colidx, A.values, x, y);
        t64 = (omp_get_wtime() - t) / reps;
        rsp_host_spmv_f32(m, A.rowptr, A.colidx, v32, x32, y32);
        t = omp_get_wtime();
        for (int r = 0; r < reps; r++) rsp_host_spmv_f32(m, A.rowptr, A.colidx, v32, x32, y32);
        t32 = (omp_get_wtime() - t) / reps;
    } else {
        t = omp_get_wtime();
        rsp_host_spmv_f64(m, A.rowptr, A.colidx, A.values, x, y);
        t64 = omp_get_wtime() - t;
        t = omp_get_wtime();
        rsp_host_spmv_f32(m, A.rowptr, A.colidx, v32, x32, y32);
        t32 = omp_get_wtime() - t;
    }
    fprintf(fout, "%g,", t64);
    fprintf(fout, "%g,", t32);

    double error = 0.0;
#pragma omp parallel for reduction(+ : error)
    for (int i = 0; i < m; i++) error += fabs(y[i] - (double)y32[i]);
    fprintf(fout, "%g,", m ? error / m : 0.0);

    time_t now = time(NULL);
    char date[128];
    strftime(date, sizeof(date), "%c", localtime(&now));
    fprintf(fout, "%s,\n", date);
    fclose(fout);

    free(x);
    free(y);
    free(x32);
    free(y32);
    free(v32);
    rsp_csr_free(&A);
    return 0;
}
