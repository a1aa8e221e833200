// A/B of LocalBA's Schur pair products H_schur(a, b) -= sum_p B_ap D_p^-1 B_bp^T
// (block_solver.hpp:381-432; k_ba_schur) on gfx950, config-3 shape: 20 free poses, 3000 points,
// each point seen by a window of 3-8 consecutive poses (~16.6k edges, ~54k observation pairs over
// the 210 pose-pair blocks).
//   valu   the k_ba_schur scheme: 512-thread block per pose pair, thread per observation pair, D^-1
//          and B_a D^-1 per pair, 36 accumulators, DPP / permlane reduce-scatter + LDS
//   mfma1  256-thread block per pose pair: each wave forms B_a D^-1 and B_b for 64 observation
//          pairs at a time (lane = pair) into LDS, then v_mfma_f64_16x16x4f64 accumulates them as
//          K = 3 x pairs (rows / cols 0-5 of the 16x16 tile used); cross-wave sum of 36 values
//   mfma2  the same with two pose pairs per 16x16 tile (rows / cols 0-5 and 8-13; the cross
//          blocks are discarded), so each MFMA serves two blocks
// Results checked against a host fp64 sum; time per launch from hipEvents over repetitions.
// Build: hipcc -O3 --offload-arch=gfx950 mfma_schur.hip -o mfma_schur ; run: ./mfma_schur
// PMC:   rocprofv3 --pmc SQ_INSTS_VALU_MFMA_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES -- ./mfma_schur
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <random>
#include <vector>

#include "../../orb_slam2_with_comment_amd/csrc/wave_ops.h"

using namespace orbmi;
typedef double double4_t __attribute__((ext_vector_type(4)));

__device__ inline void dinv3(const double* H, double lam, double Di[9]) {
    double D[3][3];
    for (int r = 0; r < 3; r++)
        for (int c = 0; c < 3; c++) D[r][c] = H[3 * r + c] + (r == c ? lam : 0.0);
    const double c00 = D[1][1] * D[2][2] - D[1][2] * D[2][1];
    const double c10 = D[1][2] * D[2][0] - D[1][0] * D[2][2];
    const double c20 = D[1][0] * D[2][1] - D[1][1] * D[2][0];
    const double id = 1.0 / (D[0][0] * c00 + D[0][1] * c10 + D[0][2] * c20);
    Di[0] = c00 * id; Di[3] = c10 * id; Di[6] = c20 * id;
    Di[1] = (D[0][2] * D[2][1] - D[0][1] * D[2][2]) * id;
    Di[4] = (D[0][0] * D[2][2] - D[0][2] * D[2][0]) * id;
    Di[7] = (D[0][1] * D[2][0] - D[0][0] * D[2][1]) * id;
    Di[2] = (D[0][1] * D[1][2] - D[0][2] * D[1][1]) * id;
    Di[5] = (D[0][2] * D[1][0] - D[0][0] * D[1][2]) * id;
    Di[8] = (D[0][0] * D[1][1] - D[0][1] * D[1][0]) * id;
}

// ---- valu: the k_ba_schur scheme
constexpr int kVThreads = 512, kVWaves = 8;
__global__ __launch_bounds__(kVThreads) void k_valu(const int* __restrict__ start, const int2* __restrict__ pairs,
                                                    const int* __restrict__ ppt, const double* __restrict__ Hpl,
                                                    const double* __restrict__ Hll, double lam, double* __restrict__ out) {
    __shared__ double red[kVWaves][36];
    const int b = blockIdx.x, lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    double acc[36];
#pragma unroll
    for (int q = 0; q < 36; q++) acc[q] = 0;
    for (int j = start[b] + threadIdx.x; j < start[b + 1]; j += blockDim.x) {
        const int2 pr = pairs[j];
        double Di[9];
        dinv3(Hll + 9 * ppt[j], lam, Di);
        const double* B1 = Hpl + 18 * (long long)pr.x;
        const double* B2 = Hpl + 18 * (long long)pr.y;
        double BD[18], b2[18];
#pragma unroll
        for (int r = 0; r < 6; r++)
#pragma unroll
            for (int c = 0; c < 3; c++) BD[r * 3 + c] = B1[r * 3] * Di[c] + B1[r * 3 + 1] * Di[3 + c] + B1[r * 3 + 2] * Di[6 + c];
#pragma unroll
        for (int q = 0; q < 18; q++) b2[q] = B2[q];
#pragma unroll
        for (int r = 0; r < 6; r++)
#pragma unroll
            for (int c = 0; c < 6; c++)
                acc[r * 6 + c] += BD[r * 3] * b2[c * 3] + BD[r * 3 + 1] * b2[c * 3 + 1] + BD[r * 3 + 2] * b2[c * 3 + 2];
    }
    double v[32];
#pragma unroll
    for (int q = 0; q < 32; q++) v[q] = acc[q];
    const double s = wave_reduce_scatter32(v);
    if (!(lane & 1)) red[wid][lane >> 1] = s;
#pragma unroll
    for (int q = 32; q < 36; q++) {
        const double x = wave_sum(acc[q]);
        if (lane == 0) red[wid][q] = x;
    }
    __syncthreads();
    if (threadIdx.x < 36) {
        double t = 0;
        for (int w = 0; w < kVWaves; w++) t += red[w][threadIdx.x];
        out[36 * b + threadIdx.x] = t;
    }
}

// ---- mfma: PAIRS pose-pair blocks per 16x16 tile
constexpr int kMThreads = 256, kMWaves = 4;
template <int PAIRS>
__global__ __launch_bounds__(kMThreads) void k_mfma(const int* __restrict__ start, const int2* __restrict__ pairs,
                                                    const int* __restrict__ ppt, const double* __restrict__ Hpl,
                                                    const double* __restrict__ Hll, double lam, int nblk,
                                                    double* __restrict__ out) {
    // per wave: the A operand (B_a D^-1, 18 per pair) and the B operand (B_b, 18 per pair) of 64
    // pairs of each of the PAIRS blocks, [pair][row][comp]
    __shared__ double opA[kMWaves][PAIRS][64 * 18], opB[kMWaves][PAIRS][64 * 18];
    __shared__ double red[kMWaves][PAIRS][36];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    int b0[PAIRS], n[PAIRS], nmax = 0;
#pragma unroll
    for (int t = 0; t < PAIRS; t++) {
        const int b = blockIdx.x * PAIRS + t;
        b0[t] = b < nblk ? start[b] : 0;
        n[t] = b < nblk ? start[b + 1] - b0[t] : 0;
        nmax = max(nmax, n[t]);
    }
    double4_t acc = {0, 0, 0, 0};
    const int row = lane & 15, kk = lane >> 4;
    for (int base = wid * 64; base < nmax; base += kMWaves * 64) {
        // phase 1: lane = observation pair base + lane of each block
#pragma unroll
        for (int t = 0; t < PAIRS; t++) {
            const int j = base + lane;
            double* A = &opA[wid][t][lane * 18];
            double* B = &opB[wid][t][lane * 18];
            if (j < n[t]) {
                const int2 pr = pairs[b0[t] + j];
                double Di[9];
                dinv3(Hll + 9 * ppt[b0[t] + j], lam, Di);
                const double* B1 = Hpl + 18 * (long long)pr.x;
                const double* B2 = Hpl + 18 * (long long)pr.y;
#pragma unroll
                for (int r = 0; r < 6; r++)
#pragma unroll
                    for (int c = 0; c < 3; c++)
                        A[r * 3 + c] = B1[r * 3] * Di[c] + B1[r * 3 + 1] * Di[3 + c] + B1[r * 3 + 2] * Di[6 + c];
#pragma unroll
                for (int q = 0; q < 18; q++) B[q] = B2[q];
            } else {
#pragma unroll
                for (int q = 0; q < 18; q++) { A[q] = 0; B[q] = 0; }
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        // phase 2: K = 3 x 64 components in 48 MFMAs; lane (row | kk << 4) supplies
        // A[row][k] and B[k][col = row] of K position k = 4 s + kk = 3 pair + comp
        const int np = min(64, nmax - base);
        const int nk = 3 * np;
        for (int s = 0; s < nk; s += 4) {
            const int k = s + kk, p = k / 3, c = k - 3 * p;
            double a = 0, bb = 0;
            if (k < nk) {
                if (PAIRS == 1) {
                    if (row < 6) { a = opA[wid][0][p * 18 + row * 3 + c]; bb = opB[wid][0][p * 18 + row * 3 + c]; }
                } else {
                    const int t = row >> 3, r = row & 7;
                    if (r < 6) { a = opA[wid][t][p * 18 + r * 3 + c]; bb = opB[wid][t][p * 18 + r * 3 + c]; }
                }
            }
            acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, bb, acc, 0, 0, 0);
        }
        __builtin_amdgcn_wave_barrier();
    }
    // C layout: lane l, reg g -> C[row (l >> 4) + 4 g][col l & 15]
#pragma unroll
    for (int g = 0; g < 4; g++) {
        const int r = (lane >> 4) + 4 * g, c = lane & 15;
        if (PAIRS == 1) {
            if (r < 6 && c < 6) red[wid][0][r * 6 + c] = acc[g];
        } else {
            if ((r >> 3) == (c >> 3) && (r & 7) < 6 && (c & 7) < 6) red[wid][r >> 3][(r & 7) * 6 + (c & 7)] = acc[g];
        }
    }
    __syncthreads();
    if (threadIdx.x < 36 * PAIRS) {
        const int t = threadIdx.x / 36, q = threadIdx.x % 36;
        const int b = blockIdx.x * PAIRS + t;
        double sum = 0;
        for (int w = 0; w < kMWaves; w++) sum += red[w][t][q];
        if (b < nblk) out[36 * b + q] = sum;
    }
}

int main() {
    const int K = 20, M = 3000, reps = 300;
    std::mt19937 rng(42);
    std::uniform_real_distribution<double> U(-1, 1);
    std::vector<int> ps(M), pk(M);
    std::vector<std::vector<int>> edge_of(M, std::vector<int>(K, -1));
    int E = 0;
    for (int p = 0; p < M; p++) {
        pk[p] = 3 + rng() % 6;
        ps[p] = rng() % (K - pk[p] + 1);
        for (int a = ps[p]; a < ps[p] + pk[p]; a++) edge_of[p][a] = E++;
    }
    std::vector<double> Hpl((size_t)E * 18), Hll((size_t)M * 9);
    for (auto& v : Hpl) v = U(rng);
    for (int p = 0; p < M; p++) {
        double A[9];
        for (auto& v : A) v = U(rng);
        for (int r = 0; r < 3; r++)
            for (int c = 0; c < 3; c++) {
                double s = r == c ? 3.0 : 0.0;
                for (int t = 0; t < 3; t++) s += A[3 * r + t] * A[3 * c + t];
                Hll[9 * p + 3 * r + c] = s;
            }
    }
    const double lam = 1e-3;
    std::vector<int> start(1, 0);
    std::vector<int2> pairs;
    std::vector<int> ppt;
    for (int a = 0; a < K; a++)
        for (int b = a; b < K; b++) {
            for (int p = 0; p < M; p++)
                if (edge_of[p][a] >= 0 && edge_of[p][b] >= 0) {
                    pairs.push_back(make_int2(edge_of[p][a], edge_of[p][b]));
                    ppt.push_back(p);
                }
            start.push_back((int)pairs.size());
        }
    const int nblk = (int)start.size() - 1;
    // host reference
    std::vector<double> ref((size_t)36 * nblk, 0.0);
    for (int b = 0; b < nblk; b++)
        for (int j = start[b]; j < start[b + 1]; j++) {
            const double* H = &Hll[9 * ppt[j]];
            double D[9];
            for (int q = 0; q < 9; q++) D[q] = H[q] + ((q % 4) == 0 ? lam : 0.0);
            const double det = D[0] * (D[4] * D[8] - D[5] * D[7]) - D[1] * (D[3] * D[8] - D[5] * D[6]) +
                               D[2] * (D[3] * D[7] - D[4] * D[6]);
            double Di[9] = {(D[4] * D[8] - D[5] * D[7]) / det, (D[2] * D[7] - D[1] * D[8]) / det,
                            (D[1] * D[5] - D[2] * D[4]) / det, (D[5] * D[6] - D[3] * D[8]) / det,
                            (D[0] * D[8] - D[2] * D[6]) / det, (D[2] * D[3] - D[0] * D[5]) / det,
                            (D[3] * D[7] - D[4] * D[6]) / det, (D[1] * D[6] - D[0] * D[7]) / det,
                            (D[0] * D[4] - D[1] * D[3]) / det};
            const double* B1 = &Hpl[18 * (size_t)pairs[j].x];
            const double* B2 = &Hpl[18 * (size_t)pairs[j].y];
            for (int r = 0; r < 6; r++)
                for (int c = 0; c < 6; c++) {
                    double s = 0;
                    for (int t = 0; t < 3; t++)
                        for (int u = 0; u < 3; u++) s += B1[r * 3 + t] * Di[t * 3 + u] * B2[c * 3 + u];
                    ref[36 * b + r * 6 + c] += s;
                }
        }
    printf("config-3 shape: %d poses, %d points, %d edges, %d pose-pair blocks, %zu observation pairs\n", K, M, E,
           nblk, pairs.size());
    int *d_start, *d_ppt;
    int2* d_pairs;
    double *d_Hpl, *d_Hll, *d_out;
    (void)hipMalloc(&d_start, start.size() * 4);
    (void)hipMalloc(&d_ppt, ppt.size() * 4);
    (void)hipMalloc(&d_pairs, pairs.size() * 8);
    (void)hipMalloc(&d_Hpl, Hpl.size() * 8);
    (void)hipMalloc(&d_Hll, Hll.size() * 8);
    (void)hipMalloc(&d_out, ref.size() * 8);
    (void)hipMemcpy(d_start, start.data(), start.size() * 4, hipMemcpyHostToDevice);
    (void)hipMemcpy(d_ppt, ppt.data(), ppt.size() * 4, hipMemcpyHostToDevice);
    (void)hipMemcpy(d_pairs, pairs.data(), pairs.size() * 8, hipMemcpyHostToDevice);
    (void)hipMemcpy(d_Hpl, Hpl.data(), Hpl.size() * 8, hipMemcpyHostToDevice);
    (void)hipMemcpy(d_Hll, Hll.data(), Hll.size() * 8, hipMemcpyHostToDevice);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const char* names[3] = {"valu (k_ba_schur scheme)", "mfma f64 16x16x4, 1 block/tile", "mfma f64 16x16x4, 2 blocks/tile"};
    for (int v = 0; v < 3; v++) {
        auto launch = [&]() {
            if (v == 0)
                hipLaunchKernelGGL(k_valu, dim3(nblk), dim3(kVThreads), 0, 0, d_start, d_pairs, d_ppt, d_Hpl, d_Hll, lam, d_out);
            else if (v == 1)
                hipLaunchKernelGGL(k_mfma<1>, dim3(nblk), dim3(kMThreads), 0, 0, d_start, d_pairs, d_ppt, d_Hpl, d_Hll, lam,
                                   nblk, d_out);
            else
                hipLaunchKernelGGL(k_mfma<2>, dim3((nblk + 1) / 2), dim3(kMThreads), 0, 0, d_start, d_pairs, d_ppt, d_Hpl,
                                   d_Hll, lam, nblk, d_out);
        };
        (void)hipMemset(d_out, 0, ref.size() * 8);
        for (int i = 0; i < 20; i++) launch();
        (void)hipDeviceSynchronize();
        std::vector<float> ms;
        for (int i = 0; i < reps; i++) {  // one launch per event pair: the per-launch duration
            (void)hipEventRecord(e0, 0);
            launch();
            (void)hipEventRecord(e1, 0);
            (void)hipEventSynchronize(e1);
            float t;
            (void)hipEventElapsedTime(&t, e0, e1);
            ms.push_back(t);
        }
        std::sort(ms.begin(), ms.end());
        std::vector<double> out(ref.size());
        (void)hipMemcpy(out.data(), d_out, out.size() * 8, hipMemcpyDeviceToHost);
        double err = 0, mx = 0;
        for (size_t q = 0; q < out.size(); q++) { err = std::max(err, std::fabs(out[q] - ref[q])); mx = std::max(mx, std::fabs(ref[q])); }
        printf("%-34s median %7.2f us (min %7.2f), max abs err %.2e (|S| max %.2e)\n", names[v], ms[ms.size() / 2] * 1e3,
               ms[0] * 1e3, err, mx);
    }
    return 0;
}
