// Latency / throughput of the fp64 ops the MFMA solve's factorisation chains: v_fma_f64,
// v_fmac_f64_dpp row_newbcast (fused broadcast FMA), v_mov_b64_dpp + v_fma_f64, v_rcp_f64.
// One wave; s_memtime cycles per op.  Build: hipcc -O3 --offload-arch=gfx950 tools/ubench/dpp64.hip -o tools/ubench/dpp64
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>

__global__ void k(double* out, unsigned long long* cyc, double seed) {
    double a0 = seed + threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6,
           a7 = a0 + 7, m = 1e-9 * seed;
    unsigned long long t0, t1;
    const int R = 256;
    // 1: dependent v_fma_f64 chain
    t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < R; i++) asm volatile("v_fma_f64 %0, %0, %1, %0" : "+v"(a0) : "v"(m));
    t1 = __builtin_amdgcn_s_memtime();
    cyc[0] = t1 - t0;
    // 2: 8 independent v_fma_f64
    t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < R / 8; i++)
        asm volatile(
            "v_fma_f64 %0, %0, %8, %0\n v_fma_f64 %1, %1, %8, %1\n v_fma_f64 %2, %2, %8, %2\n v_fma_f64 %3, %3, %8, %3\n"
            "v_fma_f64 %4, %4, %8, %4\n v_fma_f64 %5, %5, %8, %5\n v_fma_f64 %6, %6, %8, %6\n v_fma_f64 %7, %7, %8, %7"
            : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(m));
    t1 = __builtin_amdgcn_s_memtime();
    cyc[1] = t1 - t0;
    // 3: dependent v_fmac_f64_dpp row_newbcast chain
    asm volatile("s_nop 4");
    t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < R; i++)
        asm volatile("v_fmac_f64_dpp %0, %1, %2 row_newbcast:3 row_mask:0xf bank_mask:0xf" : "+v"(a0) : "v"(a1), "v"(m));
    t1 = __builtin_amdgcn_s_memtime();
    cyc[2] = t1 - t0;
    // 4: 8 independent v_fmac_f64_dpp
    asm volatile("s_nop 4");
    t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < R / 8; i++)
        asm volatile(
            "v_fmac_f64_dpp %0, %8, %9 row_newbcast:3 row_mask:0xf bank_mask:0xf\n"
            "v_fmac_f64_dpp %1, %8, %9 row_newbcast:4 row_mask:0xf bank_mask:0xf\n"
            "v_fmac_f64_dpp %2, %8, %9 row_newbcast:5 row_mask:0xf bank_mask:0xf\n"
            "v_fmac_f64_dpp %3, %8, %9 row_newbcast:6 row_mask:0xf bank_mask:0xf\n"
            "v_fmac_f64_dpp %4, %8, %9 row_newbcast:7 row_mask:0xf bank_mask:0xf\n"
            "v_fmac_f64_dpp %5, %8, %9 row_newbcast:8 row_mask:0xf bank_mask:0xf\n"
            "v_fmac_f64_dpp %6, %8, %9 row_newbcast:9 row_mask:0xf bank_mask:0xf\n"
            "v_fmac_f64_dpp %7, %8, %9 row_newbcast:10 row_mask:0xf bank_mask:0xf"
            : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(a6), "v"(m));
    t1 = __builtin_amdgcn_s_memtime();
    cyc[3] = t1 - t0;
    // 5: 8 independent v_mov_b64_dpp
    double b0, b1, b2, b3, b4, b5, b6, b7;
    t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < R / 8; i++)
        asm volatile(
            "v_mov_b64_dpp %0, %8 row_newbcast:3 row_mask:0xf bank_mask:0xf\n"
            "v_mov_b64_dpp %1, %8 row_newbcast:4 row_mask:0xf bank_mask:0xf\n"
            "v_mov_b64_dpp %2, %8 row_newbcast:5 row_mask:0xf bank_mask:0xf\n"
            "v_mov_b64_dpp %3, %8 row_newbcast:6 row_mask:0xf bank_mask:0xf\n"
            "v_mov_b64_dpp %4, %8 row_newbcast:7 row_mask:0xf bank_mask:0xf\n"
            "v_mov_b64_dpp %5, %8 row_newbcast:8 row_mask:0xf bank_mask:0xf\n"
            "v_mov_b64_dpp %6, %8 row_newbcast:9 row_mask:0xf bank_mask:0xf\n"
            "v_mov_b64_dpp %7, %8 row_newbcast:10 row_mask:0xf bank_mask:0xf"
            : "=v"(b0), "=v"(b1), "=v"(b2), "=v"(b3), "=v"(b4), "=v"(b5), "=v"(b6), "=v"(b7) : "v"(a5));
    t1 = __builtin_amdgcn_s_memtime();
    cyc[4] = t1 - t0;
    // 6: dependent v_rcp_f64 chain
    double r = a2;
    t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < R; i++) asm volatile("v_rcp_f64 %0, %0" : "+v"(r));
    t1 = __builtin_amdgcn_s_memtime();
    cyc[5] = t1 - t0;
    // 7: dependent v_mul_f64 chain
    t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < R; i++) asm volatile("v_mul_f64 %0, %0, %1" : "+v"(a3) : "v"(m));
    t1 = __builtin_amdgcn_s_memtime();
    cyc[6] = t1 - t0;
    // 8: dependent v_mov_b64_dpp chain
    double c = a4;
    t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < R; i++) asm volatile("s_nop 1\n v_mov_b64_dpp %0, %0 row_newbcast:2 row_mask:0xf bank_mask:0xf" : "+v"(c));
    t1 = __builtin_amdgcn_s_memtime();
    cyc[7] = t1 - t0;
    // 9: dependent v_mfma_f64_16x16x4f64 chain (accumulator), 10: 4 independent accumulators
    typedef __attribute__((ext_vector_type(4))) double d4;
    d4 z0 = {0, 0, 0, 0}, z1 = z0, z2 = z0, z3 = z0;
    t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < R; i++) z0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a5, a6, z0, 0, 0, 0);
    asm volatile("s_nop 7\n s_nop 7\n s_nop 7" ::: "memory");
    double zz = z0[0] + z0[3];
    t1 = __builtin_amdgcn_s_memtime();
    cyc[8] = t1 - t0;
    t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < R / 4; i++) {
        z1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a5, a6, z1, 0, 0, 0);
        z2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a5, a7, z2, 0, 0, 0);
        z3 = __builtin_amdgcn_mfma_f64_16x16x4f64(a6, a7, z3, 0, 0, 0);
        z0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a7, a5, z0, 0, 0, 0);
    }
    zz += z0[1] + z1[2] + z2[0] + z3[3];
    t1 = __builtin_amdgcn_s_memtime();
    cyc[9] = t1 - t0;
    // 11: rcp accuracy: max relative error of v_rcp_f64 over this lane's 256 values
    double worst = 0;
    for (int i = 0; i < 256; i++) {
        const double x = (1.0 + 0.0037 * (threadIdx.x * 256 + i)) * (i & 1 ? 1e-3 : 7.0);
        const double rc = __builtin_amdgcn_rcp(x);
        const double e = fabs(rc * x - 1.0);
        worst = e > worst ? e : worst;
    }
    out[64 + threadIdx.x] = worst;
    out[threadIdx.x] = zz + a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + r + c + b0 + b1 + b2 + b3 + b4 + b5 + b6 + b7;
}

int main() {
    double* o;
    unsigned long long* c;
    hipMalloc(&o, 128 * 8);
    hipMalloc(&c, 16 * 8);
    for (int rep = 0; rep < 3; rep++) hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, o, c, 1.0);
    hipDeviceSynchronize();
    unsigned long long h[16];
    hipMemcpy(h, c, sizeof(h), hipMemcpyDeviceToHost);
    const char* names[] = {"fma_f64 dependent", "fma_f64 8 independent", "fmac_f64_dpp dependent",
                           "fmac_f64_dpp 8 independent", "mov_b64_dpp 8 independent", "rcp_f64 dependent",
                           "mul_f64 dependent", "mov_b64_dpp dependent (+s_nop 1)"};
    for (int i = 0; i < 8; i++) printf("%-34s %6.2f cycles/op\n", names[i], h[i] / 256.0);
    printf("%-34s %6.2f cycles/op\n", "mfma_f64_16x16x4 dependent", h[8] / 256.0);
    printf("%-34s %6.2f cycles/op\n", "mfma_f64_16x16x4 4 independent", h[9] / 256.0);
    double w[128];
    hipMemcpy(w, o, sizeof(w), hipMemcpyDeviceToHost);
    double m = 0;
    for (int i = 64; i < 128; i++) m = w[i] > m ? w[i] : m;
    printf("v_rcp_f64 max |rcp(x) x - 1| = %.3e (2^%.1f)\n", m, m > 0 ? log2(m) : -999.0);
    return 0;
}
