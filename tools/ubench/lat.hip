// Latency microbenchmark (one wave64): dependent chains of fp64 ops on gfx950, timed with
// s_memtime.  Diagnostic for the latency-bound PoseOptimization kernel.
#include <hip/hip_runtime.h>
#include <cstdio>

#define T0(t) asm volatile("s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t))
#define PIN(x) asm volatile("" : "+v"(x))
#define USE(x) do { unsigned u_; asm volatile("v_mov_b32 %0, %1" : "=v"(u_) : "v"((unsigned)__double_as_longlong(x))); } while (0)

constexpr int N = 64;

__global__ void k(unsigned long long* out, double seed) {
    double x = seed;
    unsigned long long a, b;
    int i = 0;
#define BENCH(expr)                          \
    PIN(x); T0(a); PIN(x);                   \
    for (int j = 0; j < N; j++) { expr; }    \
    USE(x); T0(b);                           \
    if (threadIdx.x == 0) out[i] = b - a;    \
    i++;
    BENCH(x = x * 1.0000001)                       // 0 mul
    BENCH(x = x + 1e-9)                            // 1 add
    BENCH(x = fma(x, 0.9999999, 1e-9))             // 2 fma
    BENCH(x = 1.0 / x)                             // 3 div (IEEE)
    BENCH(x = sqrt(x) + 0.5)                       // 4 sqrt (IEEE)
    BENCH(x = __builtin_amdgcn_rcp(x))             // 5 v_rcp_f64
    BENCH(x = sin(x) + 0.5)                        // 6 sin
    BENCH(x = (double)(float)x * 1.0000001)        // 7 cvt round trip + mul
    { float f = (float)x;
      PIN(f); T0(a); PIN(f);
      for (int j = 0; j < N; j++) f = f * 1.0000001f;
      { unsigned u_; asm volatile("v_mov_b32 %0, %1" : "=v"(u_) : "v"(__float_as_uint(f))); }
      T0(b); if (threadIdx.x == 0) out[i] = b - a; i++; x += f; }  // 8 fp32 mul
    // 9: LDS write -> barrier -> read round trip (single wave)
    __shared__ double sh[64];
    PIN(x); T0(a); PIN(x);
    for (int j = 0; j < N; j++) { sh[threadIdx.x] = x; __syncthreads(); x = sh[(threadIdx.x + 1) & 63] + 1e-9; }
    USE(x); T0(b); if (threadIdx.x == 0) out[i] = b - a; i++;
    // 10: ds_bpermute (shfl) chain
    PIN(x); T0(a); PIN(x);
    for (int j = 0; j < N; j++) x = __shfl_xor(x, 1, 64) + 1e-9;
    USE(x); T0(b); if (threadIdx.x == 0) out[i] = b - a; i++;
    // 11: readlane chain
    PIN(x); T0(a); PIN(x);
    for (int j = 0; j < N; j++) {
        const unsigned long long u = (unsigned long long)__double_as_longlong(x);
        const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)u, 3);
        const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(u >> 32), 3);
        x = __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo)) + 1e-9;
    }
    USE(x); T0(b); if (threadIdx.x == 0) out[i] = b - a; i++;
    if (threadIdx.x == 0) out[31] = (unsigned long long)__double_as_longlong(x);
}

// 8 waves: barrier-only loop (cost of a workgroup barrier with all waves present)
__global__ void kbar(unsigned long long* out) {
    unsigned long long a, b;
    __shared__ int s[512];
    int v = threadIdx.x;
    T0(a);
    for (int j = 0; j < N; j++) { s[threadIdx.x] = v; __syncthreads(); v = s[(threadIdx.x + 64) & 511] + 1; }
    T0(b);
    if (threadIdx.x == 0) { out[0] = b - a; out[1] = v; }
}

int main() {
    unsigned long long* d;
    hipMalloc(&d, 32 * 8);
    unsigned long long h[32];
    const char* names[] = {"mul_f64", "add_f64", "fma_f64", "div_f64 (IEEE)", "sqrt_f64 (IEEE)", "rcp_f64",
                           "sin_f64", "cvt f64->f32->f64 + mul", "mul_f32", "LDS st+barrier+ld (1 wave)",
                           "shfl_xor f64 (bpermute)", "readlane x2 + add"};
    for (int rep = 0; rep < 3; rep++) {
        hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, 0.75);
        hipMemcpy(h, d, 32 * 8, hipMemcpyDeviceToHost);
    }
    for (int i = 0; i < 12; i++) printf("%-28s %7.1f cycles/op\n", names[i], (double)h[i] / N);
    for (int rep = 0; rep < 3; rep++) {
        hipLaunchKernelGGL(kbar, dim3(1), dim3(512), 0, 0, d);
        hipMemcpy(h, d, 16, hipMemcpyDeviceToHost);
    }
    printf("%-28s %7.1f cycles/iter\n", "barrier 8 waves + LDS", (double)h[0] / N);
    return 0;
}
