// ref_dump.cpp — TEST INFRASTRUCTURE ONLY. A tiny driver of our own that is
// linked against the reference's UNMODIFIED loader sources
// (/root/reference/ReadMatrixMarket/{mm_io,loadMatrixMarket}.cpp, compiled
// where they lie by oracle/Makefile; output in oracle/_ref/, git-ignored).
// It writes the CSR (or COO) the reference loader produces in a flat binary
// form so tests/ can compare the product loader byte for byte.
//
//   ref_dump <file.mtx> <outputBase> <transpose> <out.bin> [coo]
//
// Layout (little-endian int32 unless noted):
//   csr: ok, isSymmetric, m, n, nnz, stored, rowptr[m+1], colidx[stored], f64 values[stored]
//   coo: ok, isSymmetric, m, n, nnz, Rowidx[nnz], Colidx[nnz], f64 values[nnz]
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "loadMatrixMarket.h"

static void put(FILE *f, const void *p, size_t sz, size_t n) {
    if (n) fwrite(p, sz, n, f);
}

int main(int argc, char **argv) {
    if (argc < 5) {
        fprintf(stderr, "usage: %s file.mtx base transpose out.bin [coo]\n", argv[0]);
        return 2;
    }
    const int base = atoi(argv[2]), tr = atoi(argv[3]);
    const bool coo = argc > 5 && strcmp(argv[5], "coo") == 0;
    FILE *f = fopen(argv[4], "wb");
    if (!f) return 2;
    if (coo) {
        COO A;
        memset(&A, 0, sizeof(A));
        int ok = loadCooMatrix(argv[1], &A, base, tr);
        int hdr[5] = {ok, A.isSymmetric, A.m, A.n, ok ? A.nnz : 0};
        put(f, hdr, sizeof(int), 5);
        if (ok) {
            put(f, A.Rowidx, sizeof(int), (size_t)A.nnz);
            put(f, A.Colidx, sizeof(int), (size_t)A.nnz);
            put(f, A.values, sizeof(double), (size_t)A.nnz);
        }
    } else {
        CSR A;
        memset(&A, 0, sizeof(A));
        int ok = loadMatrixMarket(argv[1], &A, base, tr);
        int stored = ok ? A.rowptr[A.m] - base : 0;
        int hdr[6] = {ok, A.isSymmetric, A.m, A.n, ok ? A.nnz : 0, stored};
        put(f, hdr, sizeof(int), 6);
        if (ok) {
            put(f, A.rowptr, sizeof(int), (size_t)A.m + 1);
            put(f, A.colidx, sizeof(int), (size_t)stored);
            put(f, A.values, sizeof(double), (size_t)stored);
        }
    }
    fclose(f);
    return 0;
}
