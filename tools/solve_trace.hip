// Phase timing of k_ba_solve (LocalBA reduced-system LDL^T) on a random SPD 6K x 6K system.
// Build: hipcc -O3 -std=c++17 -ffp-contract=off --offload-arch=gfx950 -DORBMI_SOLVE_TRACE \
//        -I include -I orb_slam2_with_comment_amd/csrc tools/solve_trace.hip -o /tmp/solve_trace
#include "lba.hip"

#include <cstdio>
#include <random>

int main(int argc, char** argv) {
    using namespace orbmi;
    const int np = argc > 1 ? atoi(argv[1]) : 20, N = 6 * np;
    std::mt19937 rng(1);
    std::uniform_real_distribution<double> U(-1, 1);
    std::vector<double> M(N * N), A(N * N, 0.0), b(N), packedS(kBaPacked, 0.0);
    for (auto& v : M) v = U(rng);
    for (int i = 0; i < N; i++)
        for (int j = 0; j < N; j++) {
            double s = 0;
            for (int k = 0; k < N; k++) s += M[i * N + k] * M[j * N + k];
            A[i * N + j] = s + (i == j ? N : 0);
        }
    for (auto& v : b) v = U(rng);
    for (int r = 0; r < N; r++)
        for (int c = r; c < N; c++) packedS[r * N - r * (r - 1) / 2 + (c - r)] = A[r * N + c];
    double *dS, *dbs, *dxp;
    int* dist;
    hipMalloc(&dS, kBaPacked * 8); hipMalloc(&dbs, kBaMaxN * 8); hipMalloc(&dxp, kBaMaxN * 8); hipMalloc(&dist, 16);
    hipMemcpy(dS, packedS.data(), kBaPacked * 8, hipMemcpyHostToDevice);
    hipMemcpy(dbs, b.data(), N * 8, hipMemcpyHostToDevice);
    BaDev a{};
    a.S = dS; a.bs = dbs; a.xp = dxp; a.istat = dist;
    // no keyframes: the trial-pose tail only writes the scale
    double *dT, *dTt, *dbp, *dscal;
    hipMalloc(&dT, 64); hipMalloc(&dTt, 64); hipMalloc(&dbp, kBaMaxN * 8); hipMalloc(&dscal, 64);
    hipMemset(dbp, 0, kBaMaxN * 8);
    a.nkf = 0; a.bp = dbp; a.scal = dscal;
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    auto launch = [&] {
        if (np <= kBaSolveTpt2MaxPoses) hipLaunchKernelGGL(k_ba_solve<2>, dim3(1), dim3(kBaSolveThreads), 0, 0, a, np, 1.0, dT, dTt);
        else hipLaunchKernelGGL(k_ba_solve<1>, dim3(1), dim3(kBaSolveThreads), 0, 0, a, np, 1.0, dT, dTt);
    };
    for (int it = 0; it < 3; it++) launch();
    hipEventRecord(e0);
    const int reps = 20;
    for (int it = 0; it < reps; it++) launch();
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    unsigned long long tr[256];
    hipMemcpyFromSymbol(tr, HIP_SYMBOL(g_solve_trace), sizeof(tr));
    std::vector<double> x(N);
    hipMemcpy(x.data(), dxp, N * 8, hipMemcpyDeviceToHost);
    double res = 0;
    for (int i = 0; i < N; i++) {
        double s = 0;
        for (int j = 0; j < N; j++) s += A[i * N + j] * x[j];
        res = std::max(res, std::fabs(s - b[i]));
    }
    printf("np=%d N=%d  avg kernel %.2f us  residual %.3e\n", np, N, ms * 1e3 / reps, res);
    auto us = [&](int i, int j) { return (double)(tr[j] - tr[i]) * 0.01; };
    printf("load %.2f us\n", us(255, 0));
    double diag = 0, panel = 0, trail = 0;
    for (int k = 0; k < np; k++) {
        const int prev = k == 0 ? 0 : 3 + 3 * (k - 1);
        const double d0 = us(prev, 1 + 3 * k), d1 = us(1 + 3 * k, 2 + 3 * k), d2 = us(2 + 3 * k, 3 + 3 * k);
        if (k < 3 || k == np - 1) printf("step %2d: diag %.2f  panel %.2f  trailing %.2f\n", k, d0, d1, d2);
        diag += d0; panel += d1; trail += d2;
    }
    unsigned long long clk[2];
    hipMemcpyFromSymbol(clk, HIP_SYMBOL(g_solve_clk), sizeof(clk));
    printf("shader clock during the kernel: %.0f MHz\n", (double)(clk[1] - clk[0]) / us(255, 201));
    printf("sum diag %.2f  panel %.2f  trailing %.2f  write-back %.2f  bwd %.2f  total %.2f\n", diag, panel, trail,
           us(3 + 3 * (np - 1), 200), us(202, 201), us(255, 201));
    return 0;
}
