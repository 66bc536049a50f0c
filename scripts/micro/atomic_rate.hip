// Micro-benchmark (diagnostics only): throughput of same-address agent-scope
// fetch_add on MI355X, one lane per workgroup, K atomics each.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void hammer(unsigned long long *c, int k, int spread) {
    if (threadIdx.x != 0) return;
    unsigned long long *p = c + (spread ? (blockIdx.x % 8) * 32 : 0);
    unsigned long long s = 0;
    for (int i = 0; i < k; ++i) s += __hip_atomic_fetch_add(p, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (s == 12345) c[1000] = s;
}
int main() {
    unsigned long long *c;
    hipMalloc(&c, 8192 * 8);
    hipMemset(c, 0, 8192 * 8);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int spread = 0; spread < 2; ++spread)
        for (int g : {256, 1024})
            for (int k : {1, 8, 64}) {
                hammer<<<g, 64>>>(c, k, spread);
                hipEventRecord(a);
                for (int r = 0; r < 5; ++r) hammer<<<g, 64>>>(c, k, spread);
                hipEventRecord(b);
                hipEventSynchronize(b);
                float ms;
                hipEventElapsedTime(&ms, a, b);
                printf("spread %d grid %5d k %3d: %8.1f us per launch, %7.2f ns per atomic\n", spread, g, k, ms * 1000 / 5,
                       ms * 1e6 / 5 / (double(g) * k));
            }
    return 0;
}
