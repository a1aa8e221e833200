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
#include <algorithm>
#include <cfloat>
#include <cstring>
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
                                                           uint8_t* __restrict__ outlier_out, int by_index) {
    __shared__ double err[kPoseMaxObs][3];
    __shared__ uint8_t outl[kPoseMaxObs];  // mvbOutlier; the edge's level is the same flag
    __shared__ double red[kPoseThreads / 64][28];
    __shared__ int redi[kPoseThreads / 64];
    const int tid = threadIdx.x;
    orbmi_pose_frame& F = frames[blockIdx.x];
    const int n = F.n_obs;
    const orbmi_pose_obs* O = obs + F.obs_begin;
    // mvbOutlier per observation (orbmi_pose_optimization) or per keypoint (by_index: obs.index)
    auto put_flag = [&](int k, uint8_t v) {
        if (by_index) outlier_out[O[k].index] = v;
        else outlier_out[F.obs_begin + k] = v;
    };
    if (n > kPoseMaxObs) {  // sized for kPoseMaxObs edges per frame (the host path checks first)
        if (tid == 0) { F.inliers = -1; F.iterations = 0; }
        return;
    }
    for (int k = tid; k < n; k += kPoseThreads) outl[k] = 0;
    if (n < 3) {  // src/Optimizer.cc:378-379: no optimisation, pose untouched
        for (int k = tid; k < n; k += kPoseThreads) put_flag(k, 0);
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
    for (int k = tid; k < n; k += kPoseThreads) put_flag(k, outl[k]);
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

// Edge assembly of PoseOptimization (src/Optimizer.cc:296-375): one edge per keypoint holding a
// map point, compacted in keypoint order (workgroup scan), plus the frame record.  The map
// point of keypoint i is mps[match_mp[i]] if match_mp[i] >= 0, else lfp[match_lf[i]] if
// match_lf[i] >= 0 (orbmi_frame_mappoints); out-of-range indices read as NULL.
struct PoseGatherArgs {
    int n;                  // keypoint capacity
    const int* n_dev;       // device count (optional)
    const orbmi_keypoint* keys;
    const float* u_right;   // NULL = monocular
    const float* tcw_dev;   // initial pose on the device, else tcw
    float tcw[16];
    float fx, fy, cx, cy, bf;
    float inv_sigma2[kMaxLevels];
    int nlevels;
    const int* match_lf;
    const orbmi_lastframe_point* lfp;
    int n_lf;
    const int* match_mp;
    const orbmi_mappoint* mps;
    int n_mp;
    orbmi_pose_frame* rec;
    orbmi_pose_obs* obs;
    uint8_t* outlier;       // per keypoint, zeroed here
};

constexpr int kGatherThreads = 1024;

__global__ __launch_bounds__(kGatherThreads) void k_pose_gather(PoseGatherArgs a) {
    __shared__ int wsum[kGatherThreads / 64];
    __shared__ int base;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int n = a.n_dev ? min(*a.n_dev, a.n) : a.n;
    if (tid == 0) base = 0;
    for (int c0 = 0; c0 < n; c0 += kGatherThreads) {
        const int i = c0 + tid;
        const float* X = nullptr;
        if (i < n) {
            const int jm = a.match_mp ? a.match_mp[i] : -1;
            const int jl = a.match_lf ? a.match_lf[i] : -1;
            if (jm >= 0 && jm < a.n_mp) X = a.mps[jm].pos;
            else if (jl >= 0 && jl < a.n_lf) X = a.lfp[jl].pos;
            a.outlier[i] = 0;
        }
        const unsigned long long m = __ballot(X != nullptr);
        const int before = __popcll(m & ((1ull << lane) - 1));
        if (lane == 0) wsum[wid] = __popcll(m);
        __syncthreads();
        int off = base;
        for (int w = 0; w < wid; w++) off += wsum[w];
        if (X) {
            const orbmi_keypoint kp = a.keys[i];
            orbmi_pose_obs o;
            o.Xw[0] = X[0]; o.Xw[1] = X[1]; o.Xw[2] = X[2];
            o.u = kp.x;
            o.v = kp.y;
            o.ur = a.u_right ? a.u_right[i] : -1.0f;
            const int oct = min(max(kp.octave, 0), a.nlevels - 1);
            o.inv_sigma2 = a.inv_sigma2[oct];
            o.index = i;
            a.obs[off + before] = o;
        }
        __syncthreads();
        if (tid == 0) {
            int t = 0;
            for (int w = 0; w < kGatherThreads / 64; w++) t += wsum[w];
            base += t;
        }
        __syncthreads();
    }
    if (tid < 16) a.rec->tcw[tid] = a.tcw_dev ? a.tcw_dev[tid] : a.tcw[tid];
    if (tid == 0) {
        orbmi_pose_frame& R = *a.rec;
        R.fx = a.fx; R.fy = a.fy; R.cx = a.cx; R.cy = a.cy; R.bf = a.bf;
        R.obs_begin = 0;
        R.n_obs = base;
        R.inliers = 0;
        R.iterations = 0;
    }
}

}  // namespace orbmi

// ---------------------------------------------------------------- host
struct orbmi_pose {
    int device = 0;
    hipStream_t stream = nullptr;
    bool own_stream = true;
    uint8_t* d_buf = nullptr;  // staging of host frames / obs / flags
    size_t cap = 0;
    // orbmi_pose_optimization_frame: edge buffer + staging of host inputs (reset per call)
    orbmi_pose_obs* d_obs = nullptr;
    size_t cap_obs = 0;
    uint8_t* d_stage = nullptr;
    size_t cap_stage = 0, used_stage = 0;
};

hipStream_t orbmi_extractor_stream_(orbmi_extractor* ex);  // capi_extract.cpp

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
    if (h->d_obs) (void)hipFree(h->d_obs);
    if (h->d_stage) (void)hipFree(h->d_stage);
    if (h->stream && h->own_stream) (void)hipStreamDestroy(h->stream);
    delete h;
}

int orbmi_pose_share_stream(orbmi_pose* h, orbmi_extractor* ex) {
    if (!h || !ex) return ORBMI_E_ARG;
    hipStream_t s = orbmi_extractor_stream_(ex);
    if (!s) return ORBMI_E_STATE;
    ORBMI_HIP(hipSetDevice(h->device));
    ORBMI_HIP(hipStreamSynchronize(h->stream));
    if (h->own_stream) ORBMI_HIP(hipStreamDestroy(h->stream));
    h->stream = s;
    h->own_stream = false;
    return ORBMI_OK;
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
        hipLaunchKernelGGL(k_pose_opt, dim3(nframes), dim3(kPoseThreads), 0, h->stream, frames, obs, outlier, 0);
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
    hipLaunchKernelGGL(k_pose_opt, dim3(nframes), dim3(kPoseThreads), 0, h->stream, dF, dO, dFl, 0);
    ORBMI_HIP(hipGetLastError());
    ORBMI_HIP(hipMemcpyAsync(frames, dF, fb, hipMemcpyDeviceToHost, h->stream));
    if (nobs) ORBMI_HIP(hipMemcpyAsync(outlier, dFl, nobs, hipMemcpyDeviceToHost, h->stream));
    ORBMI_HIP(hipStreamSynchronize(h->stream));
    return ORBMI_OK;
}

int orbmi_pose_optimization_frame(orbmi_pose* h, const orbmi_frame_view* F, const float* inv_level_sigma2,
                                  const orbmi_frame_mappoints* mp, orbmi_pose_frame* rec, uint8_t* outlier) {
    using namespace orbmi;
    if (!h || !F || !inv_level_sigma2 || !mp || !rec || !outlier || F->n < 0 || !F->tcw) return ORBMI_E_ARG;
    if (F->nlevels < 1 || F->nlevels > kMaxLevels || (F->n > 0 && !F->keys_un)) return ORBMI_E_ARG;
    if ((mp->match_lf && (!mp->lf_points || mp->n_lf_points < 0)) || (mp->match_mp && (!mp->mps || mp->n_mps < 0)))
        return ORBMI_E_ARG;
    if (F->n_device && !is_device_ptr(F->n_device)) return ORBMI_E_ARG;
    ORBMI_HIP(hipSetDevice(h->device));
    const bool async = is_device_ptr(rec) && is_device_ptr(outlier);
    const size_t n = (size_t)std::max(F->n, 1);
    if (n > h->cap_obs) {
        if (h->d_obs) { ORBMI_HIP(hipStreamSynchronize(h->stream)); (void)hipFree(h->d_obs); }
        h->d_obs = nullptr;
        h->cap_obs = 0;
        ORBMI_HIP(hipMalloc((void**)&h->d_obs, n * sizeof(orbmi_pose_obs)));
        h->cap_obs = n;
    }
    // staging of host inputs / outputs: one block, sized for this call
    auto host_bytes = [&](const void* p, size_t b) { return (p && !is_device_ptr(p)) ? ((b + 255) & ~(size_t)255) : 0; };
    const size_t need = host_bytes(F->keys_un, n * sizeof(orbmi_keypoint)) + host_bytes(F->u_right, n * 4) +
                        host_bytes(mp->match_lf, n * 4) + host_bytes(mp->match_mp, n * 4) +
                        (mp->match_lf ? host_bytes(mp->lf_points, mp->n_lf_points * sizeof(orbmi_lastframe_point)) : 0) +
                        (mp->match_mp ? host_bytes(mp->mps, mp->n_mps * sizeof(orbmi_mappoint)) : 0) +
                        host_bytes(rec, sizeof(orbmi_pose_frame)) + host_bytes(outlier, n) + 512;
    if (h->used_stage) ORBMI_HIP(hipStreamSynchronize(h->stream));  // an earlier call may still read it
    h->used_stage = 0;
    if (need > h->cap_stage) {
        if (h->d_stage) (void)hipFree(h->d_stage);
        h->d_stage = nullptr;
        h->cap_stage = 0;
        ORBMI_HIP(hipMalloc((void**)&h->d_stage, need));
        h->cap_stage = need;
    }
    int rc = ORBMI_OK;
    auto dev_in = [&](const void* p, size_t b) -> const void* {
        if (!p || is_device_ptr(p) || b == 0) return p;
        uint8_t* d = h->d_stage + h->used_stage;
        h->used_stage += (b + 255) & ~(size_t)255;
        if (hipMemcpyAsync(d, p, b, hipMemcpyHostToDevice, h->stream) != hipSuccess) rc = ORBMI_E_HIP;
        return d;
    };
    auto dev_out = [&](void* p, size_t b) -> void* {
        if (is_device_ptr(p)) return p;
        uint8_t* d = h->d_stage + h->used_stage;
        h->used_stage += (b + 255) & ~(size_t)255;
        return d;
    };
    PoseGatherArgs a{};
    a.n = F->n;
    a.n_dev = F->n_device;
    a.keys = (const orbmi_keypoint*)dev_in(F->keys_un, n * sizeof(orbmi_keypoint));
    a.u_right = (const float*)dev_in(F->u_right, n * 4);
    if (is_device_ptr(F->tcw)) a.tcw_dev = F->tcw;
    else memcpy(a.tcw, F->tcw, sizeof(a.tcw));
    a.fx = F->fx; a.fy = F->fy; a.cx = F->cx; a.cy = F->cy; a.bf = F->bf;
    for (int l = 0; l < F->nlevels; l++) a.inv_sigma2[l] = inv_level_sigma2[l];
    a.nlevels = F->nlevels;
    a.match_lf = (const int*)dev_in(mp->match_lf, n * 4);
    a.lfp = mp->match_lf ? (const orbmi_lastframe_point*)dev_in(mp->lf_points, mp->n_lf_points * sizeof(orbmi_lastframe_point))
                         : nullptr;
    a.n_lf = mp->match_lf ? mp->n_lf_points : 0;
    a.match_mp = (const int*)dev_in(mp->match_mp, n * 4);
    a.mps = mp->match_mp ? (const orbmi_mappoint*)dev_in(mp->mps, mp->n_mps * sizeof(orbmi_mappoint)) : nullptr;
    a.n_mp = mp->match_mp ? mp->n_mps : 0;
    a.rec = (orbmi_pose_frame*)dev_out(rec, sizeof(orbmi_pose_frame));
    a.obs = h->d_obs;
    a.outlier = (uint8_t*)dev_out(outlier, n);
    if (rc) return rc;
    hipLaunchKernelGGL(k_pose_gather, dim3(1), dim3(kGatherThreads), 0, h->stream, a);
    ORBMI_HIP(hipGetLastError());
    hipLaunchKernelGGL(k_pose_opt, dim3(1), dim3(kPoseThreads), 0, h->stream, a.rec, (const orbmi_pose_obs*)h->d_obs,
                       a.outlier, 1);
    ORBMI_HIP(hipGetLastError());
    if (async) return ORBMI_OK;
    if (!is_device_ptr(rec))
        ORBMI_HIP(hipMemcpyAsync(rec, a.rec, sizeof(orbmi_pose_frame), hipMemcpyDeviceToHost, h->stream));
    if (!is_device_ptr(outlier))
        ORBMI_HIP(hipMemcpyAsync(outlier, a.outlier, (size_t)std::max(F->n, 0), hipMemcpyDeviceToHost, h->stream));
    ORBMI_HIP(hipStreamSynchronize(h->stream));
    h->used_stage = 0;
    if (rec->inliers < 0) return ORBMI_E_UNSUPPORTED;  // more than kPoseMaxObs edges
    return ORBMI_OK;
}

}  // extern "C"
