// Phase timing of k_ba_solve (LocalBA reduced-system LDL^T) on a random SPD 6K x 6K system.
// Build: hipcc -O3 -std=c++17 -ffp-contract=off --offload-arch=gfx950 -DORBMI_SOLVE_TRACE -Wno-unused-value \
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
    // no keyframes: the trial-pose tail only writes the scale; lambda = 1 in scal[3]
    double *dT, *dTt, *dbp, *dscal;
    hipMalloc(&dT, 64); hipMalloc(&dTt, 64); hipMalloc(&dbp, kBaMaxN * 8); hipMalloc(&dscal, 64);
    hipMemset(dbp, 0, kBaMaxN * 8);
    const double hscal[8] = {0, 0, 0, 1.0, 0, 0, 0, 0};
    hipMemcpy(dscal, hscal, sizeof(hscal), hipMemcpyHostToDevice);
    BaCtl hctl{};
    hctl.np = np;
    BaCtl* dctl;
    hipMalloc(&dctl, sizeof(BaCtl));
    hipMemcpy(dctl, &hctl, sizeof(BaCtl), hipMemcpyHostToDevice);
    a.nkf = 0; a.bp = dbp; a.scal = dscal; a.ctl = dctl; a.Tb[0] = dT; a.Tb[1] = dTt;
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    auto launch = [&] {
        if (np <= kBaSolveRowsMaxPoses && getenv("PIPE"))
            hipLaunchKernelGGL(k_ba_solve_pipe, dim3(1), dim3(kBaSolvePipeThreads), 0, 0, a);
        else if (np <= kBaSolveRowsMaxPoses && !getenv("TPT1") && !getenv("OLD"))
            hipLaunchKernelGGL(k_ba_solve_rows, dim3(1), dim3(kBaSolveRowsThreads), 0, 0, a);
        else if (np <= 21 && !getenv("TPT1"))  // the previous tile layout, TPT 2
            hipLaunchKernelGGL(k_ba_solve<2>, dim3(1), dim3(kBaSolveThreads), 0, 0, a);
        else hipLaunchKernelGGL(k_ba_solve<1>, dim3(1), dim3(kBaSolveThreads), 0, 0, a);
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
    // cycles (s_memtime) between stamps.  k_ba_solve<TPT>, per step k: panel(k, k+1) done,
    // (k+1, k+1) updated, (k+1, k+1) factored, end of step (thread 0 after the barrier).
    // k_ba_solve_rows: (k+1, k+1) updated, factored, pivot row k+1 done, end of step.
    auto cy = [&](int i, int j) { return (long long)(tr[j] - tr[i]); };
    printf("load+prologue %lld cycles\n", cy(250, 251));
    const bool rows = np <= kBaSolveRowsMaxPoses && !getenv("TPT1") && !getenv("OLD");
    long long sp = 0, su = 0, sf = 0, sb = 0;
    for (int k = 0; k + 1 < np; k++) {
        const int prev = k == 0 ? 251 : 4 * (k - 1) + 3;
        if (rows) {  // stamps 4k (diagonal k+1 updated), 4k+2 (pivot row k+1 done), 4k+3
            const long long p = cy(prev, 4 * k), f = cy(4 * k, 4 * k + 2), e = cy(4 * k + 2, 4 * k + 3);
            if (k < 3 || k == np - 2) printf("step %2d: start->updated %lld  pivot row %lld  ->end %lld\n", k, p, f, e);
            sp += p; sf += f; sb += e;
            continue;
        }
        const long long p = cy(prev, 4 * k), u = cy(4 * k, 4 * k + 1), f = cy(4 * k + 1, 4 * k + 2),
                        e = cy(4 * k + 2, 4 * k + 3);
        if (k < 3 || k == np - 2) printf("step %2d: start->panel %lld  panel->updated %lld  factor %lld  ->end %lld\n", k, p, u, f, e);
        sp += p; su += u; sf += f; sb += e;
    }
    printf("sums: %lld  %lld  %lld  %lld\n", sp, su, sf, sb);
    printf("factor loop %lld  back substitution %lld  tail %lld  total %lld cycles\n", cy(251, 4 * (np - 1) + 3),
           cy(4 * (np - 1) + 3, 252), cy(252, 253), cy(250, 253));
    return 0;
}
