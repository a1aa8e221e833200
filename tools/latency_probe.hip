// Primitive latencies on gfx950 for the latency-bound fp64 kernels (LocalBA solve, pose
// optimisation): dependent fp64 FMA, v_rcp_f64 (+ Newton), IEEE fp64 divide, LDS write->read
// round trip inside one wave, __syncthreads at 512 threads, one 6x6 LDL^T in one lane.
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -I include -I orb_slam2_with_comment_amd/csrc \
//        tools/latency_probe.hip -o tools/latency_probe
#include <hip/hip_runtime.h>

#include <cstdio>

__device__ unsigned long long g_out[64];
__device__ double g_sink[64];

__device__ inline unsigned long long now() { return __builtin_amdgcn_s_memtime(); }

__device__ inline double rcp_newton(double d) {
    double r = __builtin_amdgcn_rcp(d);
    double e = fma(-d, r, 1.0);
    return fma(r, e, r);
}

__global__ __launch_bounds__(512) void k_probe(double seed, int reps) {
    __shared__ double lds[1024];
    const int tid = threadIdx.x;
    double x = seed + tid * 1e-9;
    unsigned long long t0, t1;
    // 1. dependent fp64 FMA chain
    t0 = now();
    for (int i = 0; i < reps; i++) x = fma(x, 0.999999, 1e-7);
    t1 = now();
    if (tid == 0) g_out[0] = (t1 - t0) / reps;
    // 2. v_rcp_f64 dependent chain
    t0 = now();
    for (int i = 0; i < reps; i++) x = __builtin_amdgcn_rcp(x) + 1e-12;
    t1 = now();
    if (tid == 0) g_out[1] = (t1 - t0) / reps;
    // 3. rcp + one Newton step
    t0 = now();
    for (int i = 0; i < reps; i++) x = rcp_newton(x) + 1e-12;
    t1 = now();
    if (tid == 0) g_out[2] = (t1 - t0) / reps;
    // 4. IEEE divide
    t0 = now();
    for (int i = 0; i < reps; i++) x = 1.0 / x + 1e-12;
    t1 = now();
    if (tid == 0) g_out[3] = (t1 - t0) / reps;
    // 5. LDS write -> read round trip in one wave (dependent)
    if (tid < 64) {
        t0 = now();
        for (int i = 0; i < reps; i++) {
            lds[tid] = x;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            x = lds[(tid + 1) & 63] * 1.0000001;
        }
        t1 = now();
        if (tid == 0) g_out[4] = (t1 - t0) / reps;
    }
    __syncthreads();
    // 6. __syncthreads at 512 threads (with an LDS write before each)
    t0 = now();
    for (int i = 0; i < reps; i++) {
        lds[tid] = x;
        __syncthreads();
        x += lds[(tid + 64) & 511] * 1e-9;
    }
    t1 = now();
    if (tid == 0) g_out[5] = (t1 - t0) / reps;
    // 7. 6x6 LDL^T in one lane (dependent across repetitions)
    double F[36];
    for (int q = 0; q < 36; q++) F[q] = (q % 7 == 0) ? 10.0 + x * 1e-9 : 0.1 * ((q * 7) % 11);
    t0 = now();
    for (int i = 0; i < reps; i++) {
#pragma unroll
        for (int j = 0; j < 6; j++) {
            const double inv = rcp_newton(F[j * 7]);
#pragma unroll
            for (int c = j + 1; c < 6; c++) {
                const double u = F[j * 6 + c] * inv;
#pragma unroll
                for (int r = j + 1; r <= c; r++) F[r * 6 + c] -= F[j * 6 + r] * u;
            }
#pragma unroll
            for (int c = j + 1; c < 6; c++) F[j * 6 + c] *= inv;
        }
#pragma unroll
        for (int q = 0; q < 36; q++) F[q] = (q % 7 == 0) ? F[q] + 10.0 : F[q] * 0.5;
    }
    t1 = now();
    if (tid == 0) g_out[6] = (t1 - t0) / reps;
    double s = x;
    for (int q = 0; q < 36; q++) s += F[q];
    g_sink[tid & 63] = s;
}

int main() {
    hipLaunchKernelGGL(k_probe, dim3(1), dim3(512), 0, 0, 1.5, 200);
    hipDeviceSynchronize();
    hipLaunchKernelGGL(k_probe, dim3(1), dim3(512), 0, 0, 1.5, 200);
    unsigned long long o[64];
    hipMemcpyFromSymbol(o, HIP_SYMBOL(g_out), sizeof(o));
    const char* names[] = {"fp64 fma (dependent)", "v_rcp_f64 (dependent)", "rcp + 1 Newton", "IEEE 1/x",
                           "LDS write->read, one wave", "__syncthreads (512 thr)", "6x6 LDL^T one lane"};
    for (int i = 0; i < 7; i++) printf("%-28s %6llu cycles\n", names[i], o[i]);
    return 0;
}
