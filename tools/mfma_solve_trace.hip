// Phase timing of k_ba_solve_mfma<T> (LocalBA reduced-system blocked LDL^T on MFMA) on a random
// SPD 6K x 6K system, against the VALU pivot-wave solve on the same system.
// Build: hipcc -O3 -std=c++17 -ffp-contract=off --offload-arch=gfx950 -DORBMI_SOLVE_TRACE -Wno-unused-value \
//        -I include -I orb_slam2_with_comment_amd/csrc tools/mfma_solve_trace.hip -o tools/ubench/mfma_solve_trace
#include "lba.hip"

#include <cstdio>
#include <random>

int main(int argc, char** argv) {
    using namespace orbmi;
    const int np = argc > 1 ? atoi(argv[1]) : 20, N = 6 * np, T = (N + 15) / 16;
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
    const bool pipe = getenv("PIPE") != nullptr;
    if (pipe) {
        hipMemcpy(dS, packedS.data(), kBaPacked * 8, hipMemcpyHostToDevice);
    } else {  // k_ba_schur's tile layout (both triangles of the diagonal tiles, right-hand side column)
        std::vector<double> tiles(kBaPacked, 0.0);
        for (int r = 0; r < N; r++) {
            for (int c = r; c < N; c++) {
                tiles[mfma_tile_pos(T, r, c)] = A[r * N + c];
                if ((r >> 4) == (c >> 4)) tiles[mfma_tile_pos(T, c, r)] = A[r * N + c];
            }
            tiles[mfma_tile_pos(T, r, 16 * T)] = b[r];
        }
        for (int r = N; r < 16 * T; r++) tiles[mfma_tile_pos(T, r, r)] = 1.0;  // identity padding
        hipMemcpy(dS, tiles.data(), kBaPacked * 8, hipMemcpyHostToDevice);
    }
    hipMemcpy(dbs, b.data(), N * 8, hipMemcpyHostToDevice);
    BaDev a{};
    a.S = dS; a.bs = dbs; a.xp = dxp; a.istat = dist;
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
        if (pipe) { hipLaunchKernelGGL(k_ba_solve_pipe, dim3(1), dim3(kBaSolvePipeThreads), 0, 0, a); return; }
        switch (T) {
            case 1: hipLaunchKernelGGL(k_ba_solve_mfma<1>, dim3(1), dim3(kBaMfmaThreads), 0, 0, a); break;
            case 2: hipLaunchKernelGGL(k_ba_solve_mfma<2>, dim3(1), dim3(kBaMfmaThreads), 0, 0, a); break;
            case 3: hipLaunchKernelGGL(k_ba_solve_mfma<3>, dim3(1), dim3(kBaMfmaThreads), 0, 0, a); break;
            case 4: hipLaunchKernelGGL(k_ba_solve_mfma<4>, dim3(1), dim3(kBaMfmaThreads), 0, 0, a); break;
            case 5: hipLaunchKernelGGL(k_ba_solve_mfma<5>, dim3(1), dim3(kBaMfmaThreads), 0, 0, a); break;
            case 6: hipLaunchKernelGGL(k_ba_solve_mfma<6>, dim3(1), dim3(kBaMfmaThreads), 0, 0, a); break;
            case 7: hipLaunchKernelGGL(k_ba_solve_mfma<7>, dim3(1), dim3(kBaMfmaThreads), 0, 0, a); break;
            default: hipLaunchKernelGGL(k_ba_solve_mfma<8>, dim3(1), dim3(kBaMfmaThreads), 0, 0, a); break;
        }
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
    printf("%s np=%d N=%d T=%d  avg kernel %.2f us  residual %.3e\n", pipe ? "pipe" : "mfma", np, N, T, ms * 1e3 / reps, res);
    if (pipe) return 0;
    auto cy = [&](int i, int j) { return (long long)(tr[j] - tr[i]); };
    // factor wave: 8p (A_pp final, factor starts), 8p+1 (E_p published); tile wave 0: 8p+2 (E_p
    // seen), 8p+3 (its row panel done), 8p+4 (every row panel done), 8p+5 (its updates done)
    printf("load issue %lld cycles\n", cy(250, 251));
    long long sf = 0, sw = 0;
    for (int p = 0; p < T; p++) {
        const long long f = cy(8 * p, 8 * p + 1), handoff = cy(8 * p + 1, 8 * p + 2), row = cy(8 * p + 2, 8 * p + 3);
        long long rs = 0, up = 0, next = 0;
        if (p + 1 < T) { rs = cy(8 * p + 3, 8 * p + 4); up = cy(8 * p + 4, 8 * p + 5); next = cy(8 * p + 1, 8 * (p + 1)); }
        printf("panel %d: factor %lld  E->tiles %lld  row %lld  row sync %lld  update(w0) %lld  | E_p -> A_p+1 final %lld\n",
               p, f, handoff, row, rs, up, next);
        sf += f;
        sw += next;
    }
    printf("factor sum %lld, waiting for the next diagonal tile %lld\n", sf, sw);
    printf("start->first factor %lld  panels %lld  back substitution %lld  tail %lld  total %lld cycles\n", cy(250, 0),
           cy(0, 252), cy(252, 254), cy(254, 253), cy(250, 253));
    return 0;
}
