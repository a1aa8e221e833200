// Optimizer::PoseOptimization (src/Optimizer.cc:257-481) on MI355X, fp64, one workgroup per
// frame.  A frame's pose is a single 6-dof vertex with unary edges, so the linear system is one
// 6x6 block (BlockSolver_6_3 + LinearSolverDense): the per-edge work (error, Huber weight,
// Jacobian, J^T W J) is spread over the workgroup and reduced in a fixed order; the 6x6 solve,
// the SE3 exponential and the Levenberg decisions are computed redundantly by every thread from
// the same reduced values, so the LM state never needs a broadcast.
//   EdgeSE3ProjectXYZOnlyPose / EdgeStereoSE3ProjectXYZOnlyPose  types_six_dof_expmap.h:142-205,
//                                                              .cpp:266-364 (float invz, stereo)
//   BaseUnaryEdge::constructQuadraticForm                      core/base_unary_edge.hpp:43-75
//   OptimizationAlgorithmLevenberg::solve                      levenberg.cpp:61-189
// The edge errors of the last computeActiveErrors stay in LDS: the outlier classification after
// each optimize(10) reads them as g2o does (stale after a rejected trial).  Parity: 1e-4 on the
// pose, identical outlier flags and inlier count (tests/test_pose_gpu.py).
#include <cfloat>
#include <cmath>
#include <new>

#include "extractor.h"
#include "se3_device.h"

#pragma clang fp contract(fast)  // fp64 with a 1e-4 parity tolerance (as lba.hip)

namespace orbmi {

constexpr int kPoseThreads = 256;
constexpr int kPoseMaxObs = 4096;

struct PoseCam { double fx, fy, cx, cy, bf; };

// obs - cam_project(T Xw) (EdgeSE3ProjectXYZOnlyPose::computeError / the stereo variant)
__device__ inline void pose_error(const double* T, const PoseCam& c, const orbmi_pose_obs& o, double e[3]) {
    const double X[3] = {o.Xw[0], o.Xw[1], o.Xw[2]};
    double p[3];
    se3_map(T, X, p);
    if (o.ur < 0) {
        const double px = p[0] / p[2], py = p[1] / p[2];
        e[0] = (double)o.u - (px * c.fx + c.cx);
        e[1] = (double)o.v - (py * c.fy + c.cy);
        e[2] = 0;
    } else {
        const float invz = (float)(1.0f / p[2]);  // types_six_dof_expmap.cpp:309
        const double r0 = p[0] * invz * c.fx + c.cx;
        const double r1 = p[1] * invz * c.fy + c.cy;
        const double r2 = r0 - c.bf * invz;
        e[0] = (double)o.u - r0;
        e[1] = (double)o.v - r1;
        e[2] = (double)o.ur - r2;
    }
}

__device__ inline double pose_chi2(const orbmi_pose_obs& o, const double e[3]) {
    const double info = (double)o.inv_sigma2;
    return e[0] * (info * e[0]) + e[1] * (info * e[1]) + (o.ur < 0 ? 0.0 : e[2] * (info * e[2]));
}

// Huber delta of the edge (src/Optimizer.cc:290-291, float sqrt)
__device__ inline double pose_delta(const orbmi_pose_obs& o) {
    return o.ur < 0 ? (double)sqrtf(5.991f) : (double)sqrtf(7.815f);
}

// fixed-order workgroup sum of NV doubles: lane 0 of each wave publishes, every thread adds the
// wave partials in wave order (uniform result, no broadcast step)
template <int NV>
__device__ inline void pose_reduce(double (&v)[NV], double (*red)[NV]) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
    for (int q = 0; q < NV; q++) {
        double x = v[q];
        for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
        if (lane == 0) red[wid][q] = x;
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < NV; q++) {
        double s = 0;
        for (int w = 0; w < kPoseThreads / 64; w++) s += red[w][q];
        v[q] = s;
    }
    __syncthreads();
}

__device__ inline int pose_reduce_int(int v, int* redi) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if (lane == 0) redi[wid] = v;
    __syncthreads();
    int s = 0;
    for (int w = 0; w < kPoseThreads / 64; w++) s += redi[w];
    __syncthreads();
    return s;
}

// LDL^T solve of the damped 6x6 system (LinearSolverDense); false on a non-positive pivot
__device__ inline bool pose_solve6(const double H[21], const double b[6], double lam, double x[6]) {
    double A[6][6];
    {
        int q = 0;
#pragma unroll
        for (int r = 0; r < 6; r++)
#pragma unroll
            for (int c = r; c < 6; c++, q++) { A[r][c] = H[q]; A[c][r] = H[q]; }
    }
#pragma unroll
    for (int j = 0; j < 6; j++) A[j][j] += lam;
    bool ok = true;
#pragma unroll
    for (int j = 0; j < 6; j++) {
        double d = A[j][j];
#pragma unroll
        for (int k = 0; k < j; k++) d -= A[j][k] * A[j][k] * A[k][k];
        ok &= (fabs(d) > 0) && isfinite(d);
        A[j][j] = d;
#pragma unroll
        for (int i = j + 1; i < 6; i++) {
            double s = A[i][j];
#pragma unroll
            for (int k = 0; k < j; k++) s -= A[i][k] * A[j][k] * A[k][k];
            A[i][j] = s / d;
        }
    }
    double y[6];
#pragma unroll
    for (int i = 0; i < 6; i++) {
        double s = b[i];
#pragma unroll
        for (int k = 0; k < i; k++) s -= A[i][k] * y[k];
        y[i] = s;
    }
#pragma unroll
    for (int i = 0; i < 6; i++) y[i] /= A[i][i];
#pragma unroll
    for (int i = 5; i >= 0; i--) {
        double s = y[i];
#pragma unroll
        for (int k = i + 1; k < 6; k++) s -= A[k][i] * x[k];
        x[i] = s;
    }
    return ok;
}

__global__ __launch_bounds__(kPoseThreads) void k_pose_opt(orbmi_pose_frame* __restrict__ frames,
                                                           const orbmi_pose_obs* __restrict__ obs,
                                                           uint8_t* __restrict__ outlier_out) {
    __shared__ double err[kPoseMaxObs][3];
    __shared__ uint8_t outl[kPoseMaxObs];  // mvbOutlier; the edge's level is the same flag
    __shared__ double red[kPoseThreads / 64][28];
    __shared__ int redi[kPoseThreads / 64];
    const int tid = threadIdx.x;
    orbmi_pose_frame& F = frames[blockIdx.x];
    const int n = F.n_obs;
    const orbmi_pose_obs* O = obs + F.obs_begin;
    uint8_t* out_flags = outlier_out + F.obs_begin;
    if (n > kPoseMaxObs) {  // sized for kPoseMaxObs edges per frame (the host path checks first)
        if (tid == 0) { F.inliers = -1; F.iterations = 0; }
        return;
    }
    for (int k = tid; k < n; k += kPoseThreads) outl[k] = 0;
    if (n < 3) {  // src/Optimizer.cc:378-379: no optimisation, pose untouched
        for (int k = tid; k < n; k += kPoseThreads) out_flags[k] = 0;
        if (tid == 0) { F.inliers = 0; F.iterations = 0; }
        return;
    }
    const PoseCam cam{F.fx, F.fy, F.cx, F.cy, F.bf};
    double T0[8];  // Converter::toSE3Quat(pFrame->mTcw)
    {
        double R[3][3];
        for (int r = 0; r < 3; r++)
            for (int c = 0; c < 3; c++) R[r][c] = F.tcw[4 * r + c];
        Q q = q_from_matrix(R);
        q_normalize(q);
        T0[0] = q.x; T0[1] = q.y; T0[2] = q.z; T0[3] = q.w;
        T0[4] = F.tcw[3]; T0[5] = F.tcw[7]; T0[6] = F.tcw[11]; T0[7] = 0;
    }
    double T[8];
    int nBad = 0, iters = 0;
    __syncthreads();
    for (int it = 0; it < 4; it++) {
        const bool robust = it < 3;  // setRobustKernel(0) after the third round (:463-464)
#pragma unroll
        for (int q = 0; q < 8; q++) T[q] = T0[q];
        int nact = 0;
        for (int k = tid; k < n; k += kPoseThreads) nact += !outl[k];
        nact = pose_reduce_int(nact, redi);
        // ---- optimize(10) on the level-0 edges
        double lambda = 0, ni = 2;
        int nbadIt = 0;
        for (int i = 0; i < 10 && nact > 0; i++) {
            // computeActiveErrors + activeRobustChi2 + buildSystem at T, one pass
            double acc[28];
#pragma unroll
            for (int q = 0; q < 28; q++) acc[q] = 0;
            for (int k = tid; k < n; k += kPoseThreads) {
                if (outl[k]) continue;
                const orbmi_pose_obs o = O[k];
                double e[3];
                pose_error(T, cam, o, e);
                err[k][0] = e[0]; err[k][1] = e[1]; err[k][2] = e[2];
                const double c2 = pose_chi2(o, e), info = (double)o.inv_sigma2;
                double rho0 = c2, rho1 = 1.0;
                if (robust) {
                    const double d = pose_delta(o), dsqr = d * d;
                    if (c2 > dsqr) { const double sq = sqrt(c2); rho0 = 2 * sq * d - dsqr; rho1 = d / sq; }
                }
                acc[27] += rho0;
                // linearizeOplus (types_six_dof_expmap.cpp:266-290, :332-364)
                const double X[3] = {o.Xw[0], o.Xw[1], o.Xw[2]};
                double p[3];
                se3_map(T, X, p);
                const double x = p[0], y = p[1], invz = 1.0 / p[2], invz_2 = invz * invz;
                double J[3][6];
                J[0][0] = x * y * invz_2 * cam.fx; J[0][1] = -(1 + (x * x * invz_2)) * cam.fx; J[0][2] = y * invz * cam.fx;
                J[0][3] = -invz * cam.fx; J[0][4] = 0; J[0][5] = x * invz_2 * cam.fx;
                J[1][0] = (1 + y * y * invz_2) * cam.fy; J[1][1] = -x * y * invz_2 * cam.fy; J[1][2] = -x * invz * cam.fy;
                J[1][3] = 0; J[1][4] = -invz * cam.fy; J[1][5] = y * invz_2 * cam.fy;
                const bool st = !(o.ur < 0);
                J[2][0] = st ? J[0][0] - cam.bf * y * invz_2 : 0.0;
                J[2][1] = st ? J[0][1] + cam.bf * x * invz_2 : 0.0;
                J[2][2] = st ? J[0][2] : 0.0;
                J[2][3] = st ? J[0][3] : 0.0;
                J[2][4] = 0;
                J[2][5] = st ? J[0][5] - cam.bf * invz_2 : 0.0;
                const double w = rho1 * info;  // robustInformation
                const double om[3] = {info * e[0], info * e[1], st ? info * e[2] : 0.0};
                int q = 0;
#pragma unroll
                for (int r = 0; r < 6; r++)
#pragma unroll
                    for (int c = r; c < 6; c++, q++) acc[q] += J[0][r] * w * J[0][c] + J[1][r] * w * J[1][c] + J[2][r] * w * J[2][c];
#pragma unroll
                for (int r = 0; r < 6; r++) acc[21 + r] -= rho1 * (J[0][r] * om[0] + J[1][r] * om[1] + J[2][r] * om[2]);
            }
            pose_reduce<28>(acc, red);
            const double* H = acc;        // upper 6x6, row by row
            const double* bvec = acc + 21;
            double currentChi = acc[27];
            const double iniChi = currentChi;
            if (i == 0) {  // computeLambdaInit, tau = 1e-5
                const int dq[6] = {0, 6, 11, 15, 18, 20};
                double m = 0;
#pragma unroll
                for (int j = 0; j < 6; j++) m = fmax(m, fabs(H[dq[j]]));
                lambda = 1e-5 * m;
                ni = 2;
                nbadIt = 0;
            }
            double rho = 0;
            int qmax = 0;
            do {
                double xv[6];
                const bool ok2 = pose_solve6(H, bvec, lambda, xv);
                double Tt[8];
                if (ok2) se3_oplus(xv, T, Tt);
                else {
#pragma unroll
                    for (int q = 0; q < 8; q++) Tt[q] = T[q];
#pragma unroll
                    for (int q = 0; q < 6; q++) xv[q] = 0;
                }
                double tc[1] = {0};
                for (int k = tid; k < n; k += kPoseThreads) {
                    if (outl[k]) continue;
                    const orbmi_pose_obs o = O[k];
                    double e[3];
                    pose_error(Tt, cam, o, e);
                    err[k][0] = e[0]; err[k][1] = e[1]; err[k][2] = e[2];
                    const double c2 = pose_chi2(o, e);
                    double rho0 = c2;
                    if (robust) {
                        const double d = pose_delta(o), dsqr = d * d;
                        if (c2 > dsqr) rho0 = 2 * sqrt(c2) * d - dsqr;
                    }
                    tc[0] += rho0;
                }
                pose_reduce<1>(tc, reinterpret_cast<double(*)[1]>(&red[0][0]));
                const double tempChi = ok2 ? tc[0] : DBL_MAX;
                double scale = 0;
#pragma unroll
                for (int j = 0; j < 6; j++) scale += xv[j] * (lambda * xv[j] + bvec[j]);
                rho = (currentChi - tempChi) / (scale + 1e-3);
                if (rho > 0 && isfinite(tempChi)) {
                    double alpha = 1. - pow(2 * rho - 1, 3);
                    alpha = fmin(alpha, 2. / 3.);
                    lambda *= fmax(1. / 3., alpha);
                    ni = 2;
                    currentChi = tempChi;
#pragma unroll
                    for (int q = 0; q < 8; q++) T[q] = Tt[q];
                } else {
                    lambda *= ni;
                    ni *= 2;
                }
                qmax++;
            } while (rho < 0 && qmax < 10);
            iters++;
            if (qmax == 10 || rho == 0) break;
            if ((iniChi - currentChi) * 1e3 < iniChi) nbadIt++;
            else nbadIt = 0;
            if (nbadIt >= 3) break;
        }
        // ---- outlier classification (:418-466): stale errors of the inliers, fresh ones of the
        // outliers, chi2 compared in float
        int bad = 0;
        for (int k = tid; k < n; k += kPoseThreads) {
            const orbmi_pose_obs o = O[k];
            double e[3] = {err[k][0], err[k][1], err[k][2]};
            if (outl[k]) {
                pose_error(T, cam, o, e);
                err[k][0] = e[0]; err[k][1] = e[1]; err[k][2] = e[2];
            }
            const float c2 = (float)pose_chi2(o, e);
            const bool out = c2 > (o.ur < 0 ? 5.991f : 7.815f);
            outl[k] = out;
            bad += out;
        }
        nBad = pose_reduce_int(bad, redi);
        if (n < 10) break;  // optimizer.edges().size() < 10
    }
    for (int k = tid; k < n; k += kPoseThreads) out_flags[k] = outl[k];
    if (tid == 0) {  // Converter::toCvMat(SE3quat_recov)
        double R[3][3];
        q_to_matrix(load_q(T), R);
        for (int r = 0; r < 3; r++) {
            for (int c = 0; c < 3; c++) F.tcw[4 * r + c] = (float)R[r][c];
            F.tcw[4 * r + 3] = (float)T[4 + r];
        }
        F.tcw[12] = 0; F.tcw[13] = 0; F.tcw[14] = 0; F.tcw[15] = 1;
        F.inliers = n - nBad;
        F.iterations = iters;
    }
}

}  // namespace orbmi

// ---------------------------------------------------------------- host
struct orbmi_pose {
    int device = 0;
    hipStream_t stream = nullptr;
    uint8_t* d_buf = nullptr;  // staging of host frames / obs / flags
    size_t cap = 0;
};

namespace {

bool is_device_ptr(const void* p) {
    if (!p) return false;
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return a.type == hipMemoryTypeDevice;
}

}  // namespace

extern "C" {

int orbmi_pose_create(int device, orbmi_pose** out) {
    if (!out) return ORBMI_E_ARG;
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return ORBMI_E_HIP;
    orbmi_pose* h = new (std::nothrow) orbmi_pose();
    if (!h) return ORBMI_E_ARG;
    h->device = device;
    if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess) {
        orbmi_pose_destroy(h);
        return ORBMI_E_HIP;
    }
    *out = h;
    return ORBMI_OK;
}

void orbmi_pose_destroy(orbmi_pose* h) {
    if (!h) return;
    (void)hipSetDevice(h->device);
    if (h->stream) (void)hipStreamSynchronize(h->stream);
    if (h->d_buf) (void)hipFree(h->d_buf);
    if (h->stream) (void)hipStreamDestroy(h->stream);
    delete h;
}

int orbmi_pose_synchronize(orbmi_pose* h) {
    if (!h) return ORBMI_E_ARG;
    ORBMI_HIP(hipStreamSynchronize(h->stream));
    return ORBMI_OK;
}

int orbmi_pose_optimization(orbmi_pose* h, orbmi_pose_frame* frames, int nframes, const orbmi_pose_obs* obs,
                            int nobs, uint8_t* outlier) {
    using namespace orbmi;
    if (!h || nframes < 0 || nobs < 0 || (nframes && !frames) || (nobs && (!obs || !outlier))) return ORBMI_E_ARG;
    if (nframes == 0) return ORBMI_OK;
    ORBMI_HIP(hipSetDevice(h->device));
    const bool dev = is_device_ptr(frames);
    if (dev != is_device_ptr(obs) && nobs) return ORBMI_E_ARG;
    if (nobs && dev != is_device_ptr(outlier)) return ORBMI_E_ARG;
    if (dev) {
        hipLaunchKernelGGL(k_pose_opt, dim3(nframes), dim3(kPoseThreads), 0, h->stream, frames, obs, outlier);
        ORBMI_HIP(hipGetLastError());
        return ORBMI_OK;
    }
    for (int f = 0; f < nframes; f++) {  // host frames: the ranges are checked here
        const orbmi_pose_frame& F = frames[f];
        if (F.n_obs < 0 || F.obs_begin < 0 || F.obs_begin + F.n_obs > nobs) return ORBMI_E_ARG;
        if (F.n_obs > kPoseMaxObs) return ORBMI_E_UNSUPPORTED;
    }
    const size_t fb = sizeof(orbmi_pose_frame) * nframes, ob = sizeof(orbmi_pose_obs) * nobs;
    const size_t need = ((fb + 255) & ~(size_t)255) + ((ob + 255) & ~(size_t)255) + nobs + 256;
    if (need > h->cap) {
        if (h->d_buf) (void)hipFree(h->d_buf);
        h->d_buf = nullptr;
        h->cap = 0;
        ORBMI_HIP(hipMalloc((void**)&h->d_buf, need));
        h->cap = need;
    }
    orbmi_pose_frame* dF = (orbmi_pose_frame*)h->d_buf;
    orbmi_pose_obs* dO = (orbmi_pose_obs*)(h->d_buf + ((fb + 255) & ~(size_t)255));
    uint8_t* dFl = h->d_buf + ((fb + 255) & ~(size_t)255) + ((ob + 255) & ~(size_t)255);
    ORBMI_HIP(hipMemcpyAsync(dF, frames, fb, hipMemcpyHostToDevice, h->stream));
    if (nobs) ORBMI_HIP(hipMemcpyAsync(dO, obs, ob, hipMemcpyHostToDevice, h->stream));
    hipLaunchKernelGGL(k_pose_opt, dim3(nframes), dim3(kPoseThreads), 0, h->stream, dF, dO, dFl);
    ORBMI_HIP(hipGetLastError());
    ORBMI_HIP(hipMemcpyAsync(frames, dF, fb, hipMemcpyDeviceToHost, h->stream));
    if (nobs) ORBMI_HIP(hipMemcpyAsync(outlier, dFl, nobs, hipMemcpyDeviceToHost, h->stream));
    ORBMI_HIP(hipStreamSynchronize(h->stream));
    return ORBMI_OK;
}

}  // extern "C"
