// A/B of the J^T W J reduction of PoseOptimization / LocalBA on gfx950: fp64 VALU accumulation +
// DPP/permlane reduce-scatter (what k_pose_opt and the LocalBA kernels do) against
// v_mfma_f64_16x16x4f64 on the same data.  One 512-thread workgroup (the pose kernel's shape):
// E edges with R rows each (2 mono / 3 stereo); row = sqrt(w) [J (6) | e] -> the 7x7 Gram matrix
// (28 upper values: the 21 of H, the 6 of b and chi2), reduced to wave 0.  Cycle counts from
// s_memtime inside the kernel (median of repetitions); results compared with a host fp64 sum.
// Build: hipcc -O3 --offload-arch=gfx950 mfma_jtj.hip -o mfma_jtj ; run: ./mfma_jtj
// PMC:   rocprofv3 --pmc SQ_INSTS_VALU_MFMA_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES -- ./mfma_jtj
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <vector>

#include "../../orb_slam2_with_comment_amd/csrc/wave_ops.h"

using namespace orbmi;
constexpr int kThreads = 512, kWaves = kThreads / 64, kCols = 7;
typedef double double4_t __attribute__((ext_vector_type(4)));

// VALU: thread t owns rows t, t + 512, ...; 28 accumulators; reduce-scatter + LDS cross-wave
__global__ __launch_bounds__(kThreads) void k_valu(const double* __restrict__ rows, int nrows, double* out,
                                                   unsigned long long* cyc) {
    __shared__ double red[kWaves][32];
    __shared__ double tot[32];
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    double acc[28];
#pragma unroll
    for (int q = 0; q < 28; q++) acc[q] = 0;
    for (int r = threadIdx.x; r < nrows; r += kThreads) {
        double v[kCols];
#pragma unroll
        for (int c = 0; c < kCols; c++) v[c] = rows[r * 8 + c];
        int q = 0;
#pragma unroll
        for (int i = 0; i < kCols; i++)
#pragma unroll
            for (int j = i; j < kCols; j++, q++) acc[q] += v[i] * v[j];
    }
    double v32[32];
#pragma unroll
    for (int q = 0; q < 28; q++) v32[q] = acc[q];
    v32[28] = v32[29] = v32[30] = v32[31] = 0;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const double s = wave_reduce_scatter32(v32);
    if (!(lane & 1)) red[wid][lane >> 1] = s;
    __syncthreads();
    if (wid == 0 && lane < 28) {
        double t = 0;
        for (int w = 0; w < kWaves; w++) t += red[w][lane];
        tot[lane] = t;
    }
    __syncthreads();
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x < 28) out[threadIdx.x] = tot[threadIdx.x];
    if (threadIdx.x == 0) *cyc = t1 - t0;
}

// MFMA: the rows are this kernel's operand in the 16x16x4 f64 layout (A = B = X^T with X the
// rows x 16 matrix, lane l holds X[k = l >> 4][i = l & 15]); each wave accumulates its chunks of
// 4 rows into one 16x16 tile, then the 28 needed entries are summed across the waves
__global__ __launch_bounds__(kThreads) void k_mfma(const double* __restrict__ rows, int nrows, double* out,
                                                   unsigned long long* cyc) {
    __shared__ double red[kWaves][32];
    __shared__ double tot[32];
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int k = lane >> 4, i = lane & 15;
    // four independent accumulators, so consecutive MFMAs do not wait on each other's results
    double4_t a0 = {0, 0, 0, 0}, a1 = a0, a2 = a0, a3 = a0;
    int r0 = 4 * wid;
    for (; r0 + 12 * kWaves < nrows; r0 += 16 * kWaves) {
        const int r = r0 + k;
        const double x0 = i < kCols ? rows[r * 8 + i] : 0.0;
        const double x1 = i < kCols ? rows[(r + 4 * kWaves) * 8 + i] : 0.0;
        const double x2 = i < kCols ? rows[(r + 8 * kWaves) * 8 + i] : 0.0;
        const double x3 = (i < kCols && r + 12 * kWaves < nrows) ? rows[(r + 12 * kWaves) * 8 + i] : 0.0;
        a0 = __builtin_amdgcn_mfma_f64_16x16x4f64(x0, x0, a0, 0, 0, 0);
        a1 = __builtin_amdgcn_mfma_f64_16x16x4f64(x1, x1, a1, 0, 0, 0);
        a2 = __builtin_amdgcn_mfma_f64_16x16x4f64(x2, x2, a2, 0, 0, 0);
        a3 = __builtin_amdgcn_mfma_f64_16x16x4f64(x3, x3, a3, 0, 0, 0);
    }
    for (; r0 < nrows; r0 += 4 * kWaves) {
        const int r = r0 + k;
        const double x = (r < nrows && i < kCols) ? rows[r * 8 + i] : 0.0;
        a0 = __builtin_amdgcn_mfma_f64_16x16x4f64(x, x, a0, 0, 0, 0);
    }
    const double4_t acc = (a0 + a1) + (a2 + a3);
    // C layout (f64 16x16x4): lane l, reg g -> C[row (l >> 4) + 4 g][col l & 15]
#pragma unroll
    for (int g = 0; g < 4; g++) {
        const int row = (lane >> 4) + 4 * g, col = lane & 15;
        if (row < kCols && col < kCols && col >= row) {
            const int q = row * kCols - row * (row - 1) / 2 + (col - row);
            red[wid][q] = acc[g];
        }
    }
    __syncthreads();
    if (wid == 0 && lane < 28) {
        double t = 0;
        for (int w = 0; w < kWaves; w++) t += red[w][lane];
        tot[lane] = t;
    }
    __syncthreads();
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x < 28) out[threadIdx.x] = tot[threadIdx.x];
    if (threadIdx.x == 0) *cyc = t1 - t0;
}

int main() {
    const int reps = 200;
    for (int E : {420, 680, 2000}) {
        const int nrows = E * 3;  // stereo edges: 3 rows
        std::vector<double> h(nrows * 8, 0.0);
        unsigned s = 12345;
        for (auto& v : h) { s = s * 1664525u + 1013904223u; v = ((s >> 8) & 0xFFFF) / 65536.0 - 0.5; }
        for (int r = 0; r < nrows; r++) h[r * 8 + 7] = 0;
        std::vector<double> ref(28, 0.0);
        for (int r = 0; r < nrows; r++) {
            int q = 0;
            for (int a = 0; a < kCols; a++)
                for (int b = a; b < kCols; b++, q++) ref[q] += h[r * 8 + a] * h[r * 8 + b];
        }
        double *d_rows, *d_out;
        unsigned long long* d_cyc;
        (void)hipMalloc(&d_rows, h.size() * 8);
        (void)hipMalloc(&d_out, 28 * 8);
        (void)hipMalloc(&d_cyc, 8);
        (void)hipMemcpy(d_rows, h.data(), h.size() * 8, hipMemcpyHostToDevice);
        for (int variant = 0; variant < 2; variant++) {
            std::vector<unsigned long long> cyc;
            std::vector<double> out(28);
            for (int it = 0; it < reps; it++) {
                if (variant == 0) hipLaunchKernelGGL(k_valu, dim3(1), dim3(kThreads), 0, 0, d_rows, nrows, d_out, d_cyc);
                else hipLaunchKernelGGL(k_mfma, dim3(1), dim3(kThreads), 0, 0, d_rows, nrows, d_out, d_cyc);
                unsigned long long c;
                (void)hipMemcpy(&c, d_cyc, 8, hipMemcpyDeviceToHost);
                cyc.push_back(c);
            }
            (void)hipMemcpy(out.data(), d_out, 28 * 8, hipMemcpyDeviceToHost);
            double err = 0;
            for (int q = 0; q < 28; q++) err = std::max(err, std::fabs(out[q] - ref[q]) / (std::fabs(ref[q]) + 1e-12));
            std::sort(cyc.begin(), cyc.end());
            printf("E=%4d rows=%4d %s: median %6llu cycles (min %6llu), max rel err %.1e\n", E, nrows,
                   variant ? "MFMA f64 16x16x4" : "VALU + DPP     ", cyc[cyc.size() / 2], cyc[0], err);
        }
        (void)hipFree(d_rows);
        (void)hipFree(d_out);
        (void)hipFree(d_cyc);
    }
    return 0;
}
