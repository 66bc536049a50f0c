// testkit.hip — test-only kernels, never called by the product: a bounded
// occupant that holds whole CUs for a given wall time, so the co-residency
// tests (tests/test_gpu_ilu0.py) can run the ILU flow launches beside a
// kernel that keeps some of their workgroups from being scheduled.
// Built into librsp_testkit.so (its own library: librsp.so exports only the
// include/rsp.h interface).
#include <hip/hip_runtime.h>

namespace {

// One 1024-thread workgroup per CU (its dynamic LDS is the CU's whole LDS),
// spinning on the 100 MHz wall clock until `ticks`
// have passed: every wave reaches the end, whatever else runs.
__global__ __launch_bounds__(1024) void occupy(unsigned long long ticks) {
    extern __shared__ int pad[];
    if (threadIdx.x == 0) {
        pad[0] = 0;
        const unsigned long long t0 = wall_clock64();
        while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(32);
    }
    __syncthreads();
}

}  // namespace

// blocks workgroups (one per CU, up to the CU count) on `stream` for `usec`
// microseconds (at most 10 s), each workgroup holding ALL of its CU's LDS (so
// no workgroup that uses LDS shares the CU with it); returns the hipError_t
extern "C" int rsp_testkit_occupy(void *stream, int blocks, long long usec) {
    if (blocks < 1 || usec < 0 || usec > 10000000) return (int)hipErrorInvalidValue;
    int dev = 0, lds = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e == hipSuccess) e = hipDeviceGetAttribute(&lds, hipDeviceAttributeMaxSharedMemoryPerMultiprocessor, dev);
    if (e == hipSuccess)
        e = hipFuncSetAttribute((const void *)occupy, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    if (e != hipSuccess) return (int)e;
    hipLaunchKernelGGL(occupy, dim3(blocks), dim3(1024), (size_t)lds, (hipStream_t)stream,
                       (unsigned long long)usec * 100ull);
    return (int)hipGetLastError();
}
