/*
 * dlarnv.c — LAPACK DLARNV/DLARUV restated (the `x` generator of the CPU
 * driver: LAPACKE_dlarnv(1, {0,0,0,1}, m, x), test_spmv.c:75-76).
 *
 * DLARUV is a multiplicative congruential generator modulo 2^48 with
 * multiplier a = 33952834046453 (first row of its MM table: 494, 322, 2508,
 * 2549 in 12-bit limbs). A batch of k numbers returns seed*a^i / 2^48 for
 * i = 1..k and leaves seed*a^k as the new seed, and DLARNV calls it in
 * consecutive batches, so the stream is simply x_k = seed*a^k mod 2^48 / 2^48.
 * The nested 12-bit evaluation in DLARUV is exact in double precision (48
 * significant bits), so the value equals the integer divided by 2^48 exactly
 * and can never round to 1.0 (DLARUV's retry branch is dead for doubles).
 * SURVEY §0.7 pins x[0..2] = 0.12062469795087694, 0.6438459108216854,
 * 0.06234171577016312 against MKL's LAPACKE_dlarnv.
 */
#include <math.h>
#include <stdint.h>
#include <xmmintrin.h>

#include "rsp_host.h"

#define LCG_A 33952834046453ULL
#define MASK48 ((1ULL << 48) - 1)

int rsp_dlarnv(int idist, int *iseed, int64_t n, double *x) {
    if (idist < 1 || idist > 3 || n < 0 || !iseed) return -1;
    uint64_t s = ((uint64_t)(iseed[0] & 4095) << 36) | ((uint64_t)(iseed[1] & 4095) << 24) |
                 ((uint64_t)(iseed[2] & 4095) << 12) | (uint64_t)(iseed[3] & 4095);
    const double r48 = 1.0 / 281474976710656.0; /* 2^-48 */
    if (idist == 3) {
        /* Box-Muller on consecutive pairs (DLARNV, IDIST = 3). */
        for (int64_t i = 0; i < n; i++) {
            s = (s * LCG_A) & MASK48;
            double u1 = (double)s * r48;
            s = (s * LCG_A) & MASK48;
            double u2 = (double)s * r48;
            x[i] = sqrt(-2.0 * log(u1)) * cos(6.2831853071795864769252867663 * u2);
        }
    } else {
        for (int64_t i = 0; i < n; i++) {
            s = (s * LCG_A) & MASK48;
            double u = (double)s * r48;
            x[i] = (idist == 1) ? u : 2.0 * u - 1.0;
        }
    }
    iseed[0] = (int)((s >> 36) & 4095);
    iseed[1] = (int)((s >> 24) & 4095);
    iseed[2] = (int)((s >> 12) & 4095);
    iseed[3] = (int)(s & 4095);
    return 0;
}

/* test_pardiso.c:19-24 (`set_ftz`): MXCSR |= 0x8040 (FTZ bit 15, DAZ bit 6). */
void rsp_set_cpu_ftz(int enable) {
    unsigned csr = _mm_getcsr();
    if (enable)
        csr |= 0x8040u;
    else
        csr &= ~0x8040u;
    _mm_setcsr(csr);
}
