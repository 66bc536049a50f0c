// lds_chain.hip — microbenchmark (diagnostics only, never shipped): cycles per
// iteration of a one-wave dependent LDS chain shaped like a narrow level of
// the thin triangular solve (trsv_thin_pf): G y loads from LDS -> G dependent
// fp64 fmas -> one y store, with or without the independent prefetch loads a
// level issues for the next levels, and where they are issued.
//   hipcc --offload-arch=gfx950 -O3 -o lds_chain lds_chain.hip && ./lds_chain
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int NY = 4096, NIT = 20000;

template <int MODE, int G>
__global__ __launch_bounds__(64) void chain(const int *idx, double *out, long long *cyc) {
    __shared__ double y[NY];
    __shared__ double4 val[1024];
    __shared__ int4 rec[1024];
    const int lane = threadIdx.x;
    for (int i = lane; i < NY; i += 64) y[i] = 1.0 + i * 1e-9;
    for (int i = lane; i < 1024; i += 64) {
        val[i] = make_double4(1e-3, 2e-3, 3e-3, 4e-3);
        rec[i] = make_int4(idx[i] & (NY - 1), idx[i + 1] & (NY - 1), idx[i + 2] & (NY - 1), idx[i + 3] & 1023);
    }
    __syncthreads();
    int4 r = rec[lane];
    double4 v = val[lane];
    int k = lane;
    __builtin_amdgcn_s_waitcnt(0xc07f);
    long long t0 = clock64();
    double s = 0.0;
    for (int it = 0; it < NIT; ++it) {
        int4 rn = r;
        double4 vn = v;
        if (MODE >= 1) {  // prefetch before the y loads (as the solve does)
            rn = rec[(r.w + it) & 1023];
            vn = val[(r.w + 3 * it) & 1023];
        }
        double a0 = y[r.x], a1 = y[r.y], a2 = y[r.z], a3 = y[(r.x + 7) & (NY - 1)];
        if (MODE == 2) {  // prefetch after the y loads
            rn = rec[(r.w + it) & 1023];
            vn = val[(r.w + 3 * it) & 1023];
        }
        s = v.x * 0.5;
        s = __builtin_fma(-v.x, a0, s);
        if (G >= 2) s = __builtin_fma(-v.y, a1, s);
        if (G >= 3) s = __builtin_fma(-v.z, a2, s);
        if (G >= 4) s = __builtin_fma(-v.w, a3, s);
        y[(k + it * 13) & (NY - 1)] = s;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
        r = rn;
        v = vn;
        if (MODE == 0) r.x = (r.x + 1) & (NY - 1);
    }
    long long t1 = clock64();
    if (lane == 0) cyc[0] = t1 - t0;
    out[lane] = s;
}

template <int MODE, int G>
static void run(const int *d_idx, double *d_out, long long *d_cyc, const char *name) {
    chain<MODE, G><<<1, 64>>>(d_idx, d_out, d_cyc);
    long long c = 0;
    hipMemcpy(&c, d_cyc, sizeof(c), hipMemcpyDeviceToHost);
    printf("%-34s G=%d  %7.1f cycles / iteration\n", name, G, (double)c / NIT);
}

int main() {
    int h[1030];
    unsigned s = 12345;
    for (int i = 0; i < 1030; ++i) h[i] = (int)((s = s * 1103515245u + 12345u) >> 8);
    int *d_idx; double *d_out; long long *d_cyc;
    hipMalloc(&d_idx, sizeof(h)); hipMalloc(&d_out, 64 * sizeof(double)); hipMalloc(&d_cyc, 8);
    hipMemcpy(d_idx, h, sizeof(h), hipMemcpyHostToDevice);
    for (int rep = 0; rep < 2; ++rep) {
        run<0, 1>(d_idx, d_out, d_cyc, "chain only");
        run<0, 4>(d_idx, d_out, d_cyc, "chain only");
        run<1, 4>(d_idx, d_out, d_cyc, "prefetch before y loads");
        run<2, 4>(d_idx, d_out, d_cyc, "prefetch after y loads");
        run<1, 2>(d_idx, d_out, d_cyc, "prefetch before y loads");
    }
    return 0;
}
