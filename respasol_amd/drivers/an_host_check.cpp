// an_host_check.cpp — sanitizer driver for the ILU analysis' host half
// (never shipped): builds the plan of a surrogate twice (the second time with
// the U plan too) through rsp_an::plan_host — the worker pool, the concurrent
// L / L^T / factor plans, the factor pieces' shared position table and the
// block cache all run — and checks the two digests agree. Built by
// `make -C respasol_amd/csrc tsan` (ThreadSanitizer) and `asan-an`
// (Address + UndefinedBehaviorSanitizer); tests/test_sanitize.py runs both.
//     an_host_check <surrogate> [scale]
#include "ilu_analysis.h"
#include "rsp_host.h"
#include <stdio.h>
#include <stdlib.h>
#include <vector>
int main(int argc, char **argv) {
    const char *name = argc > 1 ? argv[1] : "dc1";
    const double scale = argc > 2 ? atof(argv[2]) : 0.02;
    int m = 0;
    if (rsp_surrogate_rows(name, scale, &m) != 0) return 2;
    std::vector<int> len((size_t)m), rp((size_t)m + 1, 0);
    if (rsp_surrogate_rowlens(name, scale, 0, 0, m, len.data()) != 0) return 2;
    for (int i = 0; i < m; i++) rp[(size_t)i + 1] = rp[(size_t)i] + len[(size_t)i];
    std::vector<int> ci((size_t)rp[(size_t)m]);
    std::vector<double> v((size_t)rp[(size_t)m]);
    if (rsp_surrogate_fill(name, scale, 0, 0, m, rp.data(), ci.data(), v.data()) != 0) return 2;
    unsigned long long d0 = 0;
    for (int rep = 0; rep < 2; rep++) {
        rsp_an::IluHostPlan hp;
        rsp_an::Phases ph;
        ph.start();
        if (rsp_an::plan_host(m, rp.data(), ci.data(), 1LL << 26, rep == 1, hp, ph) != RSP_STATUS_SUCCESS) return 3;
        const unsigned long long d = rsp_an::digest(hp);
        if (rep == 0) d0 = d; else if (d != d0) { fprintf(stderr, "digest differs\n"); return 4; }
    }
    printf("%s n=%d digest %016llx\n", name, m, d0);
    return 0;
}
