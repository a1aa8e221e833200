// Throughput microbenchmark: 8 independent fp64 FMA chains per lane, 1..16 waves per CU (one
// workgroup), reporting cycles per wave-instruction per SIMD.  Diagnostic.
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int N = 256;

template <typename T>
__global__ void k(unsigned long long* out, T seed) {
    T a0 = seed, a1 = seed + 1, a2 = seed + 2, a3 = seed + 3, a4 = seed + 4, a5 = seed + 5, a6 = seed + 6, a7 = seed + 7;
    const T m = (T)0.999, c = (T)1e-3;
    __syncthreads();
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int j = 0; j < N; j++) {
        a0 = a0 * m + c; a1 = a1 * m + c; a2 = a2 * m + c; a3 = a3 * m + c;
        a4 = a4 * m + c; a5 = a5 * m + c; a6 = a6 * m + c; a7 = a7 * m + c;
        asm volatile("" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));
    }
    __syncthreads();
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) out[0] = t1 - t0;
    if (threadIdx.x == 1) out[1] = (unsigned long long)(a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7);
}

int main() {
    unsigned long long* d;
    (void)hipMalloc(&d, 16);
    unsigned long long h[2];
    for (int waves : {1, 2, 4, 8, 16}) {
        for (int rep = 0; rep < 2; rep++) {
            hipLaunchKernelGGL(k<double>, dim3(1), dim3(64 * waves), 0, 0, d, 0.5);
            (void)hipMemcpy(h, d, 16, hipMemcpyDeviceToHost);
        }
        const double per_simd = (waves + 3) / 4;
        printf("fp64 fma  waves=%2d: %6.2f cycles per wave-instr per SIMD (%.2f per instr of one wave)\n", waves,
               (double)h[0] / (N * 8.0 * per_simd), (double)h[0] / (N * 8.0));
        for (int rep = 0; rep < 2; rep++) {
            hipLaunchKernelGGL(k<float>, dim3(1), dim3(64 * waves), 0, 0, d, 0.5f);
            (void)hipMemcpy(h, d, 16, hipMemcpyDeviceToHost);
        }
        printf("fp32 fma  waves=%2d: %6.2f cycles per wave-instr per SIMD\n", waves, (double)h[0] / (N * 8.0 * per_simd));
    }
    return 0;
}
