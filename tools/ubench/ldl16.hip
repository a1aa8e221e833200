// Cycles of the MFMA solve's 16 x 16 panel factorisation (ldl16 in csrc/lba.hip) on one wave,
// against its two halves: the bulk DPP FMAs alone (throughput floor) and the per-step dependent
// chain alone (pivot broadcast, reciprocal + Newton step, multiplier, select: latency floor).
// Build: hipcc -O3 -std=c++17 -ffp-contract=off --offload-arch=gfx950 -Wno-unused-value \
//        -I include -I orb_slam2_with_comment_amd/csrc tools/ubench/ldl16.hip -o tools/ubench/ldl16
#include "lba.hip"

#include <cstdio>

using namespace orbmi;

template <int J>
__device__ inline void bulk_only(double (&A)[16], double (&Eg)[4], double nl) {
    if constexpr (J < 15) {
        constexpr int NB = (14 - J) + (J / 4 + 1);
        asm volatile("s_nop 1");
        fmac_self<J>(A[J + 1], nl);
        ldl_bulk<J, 0, NB>(A, Eg, nl);
        bulk_only<J + 1>(A, Eg, nl);
    }
}

template <int J>
__device__ inline void chain_only(double (&A)[16], double (&inv)[16], int r, double nl) {
    if constexpr (J < 15) {
        const double msk = select_asm(-1.0, __builtin_amdgcn_ballot_w64(r > J + 1));
        asm volatile("s_nop 1");
        fmac_self<J>(A[J + 1], nl);
        const double am = mul_asm(A[J + 1], msk);
        asm volatile("s_nop 1");
        const double d = bcast16_asm<J + 1>(A[J + 1]);
        const double r0 = rcp_asm(d);
        const double e1 = newton_err_asm(d, r0);
        const double a0 = mul_asm(am, r0);
        const double nl_next = fma_asm(a0, e1, a0);
        inv[J + 1] = fma_asm(r0, e1, r0);
        chain_only<J + 1>(A, inv, r, nl_next);
    }
}

template <int V>
__global__ __launch_bounds__(256) void k(const double* Ain, double* out, unsigned long long* cyc, int iters) {
    const int lane = threadIdx.x & 63, n = lane & 15;
    double A0[16];
    for (int c = 0; c < 16; c++) A0[c] = Ain[n * 16 + c];
    double acc = 0.0;
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; it++) {
        double A[16], E[4], inv[16];
#pragma unroll
        for (int c = 0; c < 16; c++) {
            A[c] = A0[c];
            inv[c] = 0.0;
        }
#pragma unroll
        for (int c = 0; c < 4; c++) E[c] = (lane >> 4) + 4 * c == n ? 1.0 : 0.0;
        if constexpr (V == 0) ldl16(A, E, inv, n);
        if constexpr (V == 1) bulk_only<0>(A, E, 1e-3 * (1 + n));
        if constexpr (V == 2) chain_only<0>(A, inv, n, -0.5);
        double s = 0.0;
#pragma unroll
        for (int c = 0; c < 16; c++) s += A[c] + inv[c] + E[c & 3];
        acc += s;
        A0[it & 15] += 1e-300 * acc;  // a dependency: no iteration is hoisted
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = acc;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

int main() {
    double A[256];
    for (int i = 0; i < 16; i++)
        for (int j = 0; j < 16; j++) A[i * 16 + j] = (i == j ? 20.0 : 0.0) + 1.0 / (1 + i + j);
    double *dA, *dout;
    unsigned long long* dc;
    hipMalloc(&dA, sizeof(A));
    hipMalloc(&dout, 256 * sizeof(double));
    hipMalloc(&dc, 8);
    hipMemcpy(dA, A, sizeof(A), hipMemcpyHostToDevice);
    const int iters = 64;
    const char* names[3] = {"ldl16 (chain interleaved with the bulk FMAs)", "bulk DPP FMAs only", "dependent chain only"};
    for (int waves : {1, 4}) {
        for (int v = 0; v < 3; v++) {
            unsigned long long c = 0;
            for (int rep = 0; rep < 3; rep++) {
                if (v == 0) hipLaunchKernelGGL(k<0>, dim3(1), dim3(64 * waves), 0, 0, dA, dout, dc, iters);
                if (v == 1) hipLaunchKernelGGL(k<1>, dim3(1), dim3(64 * waves), 0, 0, dA, dout, dc, iters);
                if (v == 2) hipLaunchKernelGGL(k<2>, dim3(1), dim3(64 * waves), 0, 0, dA, dout, dc, iters);
                hipDeviceSynchronize();
                hipMemcpy(&c, dc, 8, hipMemcpyDeviceToHost);
            }
            printf("%d wave(s): %-48s %8.0f cycles per 16x16 factorisation\n", waves, names[v], (double)c / iters);
        }
    }
    return 0;
}
