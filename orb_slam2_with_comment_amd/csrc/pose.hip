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
// The edges live in LDS for the whole kernel; the chi2 of each edge's last computeActiveErrors
// stays there too: the outlier classification after each optimize(10) reads it as g2o does
// (stale after a rejected trial).  Reductions are wave reduce-scatters on DPP / permlane swaps
// plus one LDS slot per wave, in a fixed order.  Parity: 1e-4 on the pose, outlier flags and
// inlier count equal up to chi2-on-threshold flips (tests/test_pose_gpu.py).
#include <algorithm>
#include <cfloat>
#include <cstring>
#include <cmath>
#include <new>
#include <utility>
#include <vector>

#include "extractor.h"
#include "se3_device.h"
#include "track_update.h"
#include "wave_ops.h"

#pragma clang fp contract(fast)  // fp64 with a 1e-4 parity tolerance (as lba.hip)

namespace orbmi {

#ifndef ORBMI_POSE_THREADS
#define ORBMI_POSE_THREADS 512
#endif
constexpr int kPoseThreads = ORBMI_POSE_THREADS;  // 8 waves, 2 per SIMD: the per-edge passes hide fp64 latency
constexpr int kPoseWaves = kPoseThreads / 64;
// buildSystem runs on one wave per SIMD: its pass is VALU-issue-bound, so two waves per SIMD
// take as long for the same edges, and each extra wave pays ~250 instructions of reduce-scatter
#ifndef ORBMI_POSE_FULL_WAVES
#define ORBMI_POSE_FULL_WAVES 4
#endif
constexpr int kPoseFullWaves = ORBMI_POSE_FULL_WAVES;
constexpr int kPoseFullThreads = kPoseFullWaves * 64;
static_assert(kPoseFullWaves >= 1 && kPoseFullWaves <= kPoseWaves, "buildSystem waves");
constexpr int kPoseTraceWaves = 8;  // trace layout (orbmi_debug_pose_trace), whatever kPoseWaves
#ifndef ORBMI_POSE_MAX_OBS
#define ORBMI_POSE_MAX_OBS 4096
#endif
constexpr int kPoseMaxObs = ORBMI_POSE_MAX_OBS;
constexpr int kPoseTraceSeqs = 64;  // passes recorded by orbmi_debug_pose_trace
constexpr int kPoseTraceWords = 16 + kPoseTraceSeqs * kPoseTraceWaves * 8;

struct PoseCam { double fx, fy, cx, cy, bf; };

// Huber delta of the edge (src/Optimizer.cc:290-291, float sqrt)
__device__ inline double pose_delta(const orbmi_pose_obs& o) {
    return o.ur < 0 ? (double)sqrtf(5.991f) : (double)sqrtf(7.815f);
}

// camera-frame point and obs - cam_project(T Xw) (EdgeSE3ProjectXYZOnlyPose::computeError /
// the stereo variant); invz = 1 / p.z (the stereo projection rounds it to float,
// types_six_dof_expmap.cpp:309)
__device__ inline void pose_error(const double* T, const PoseCam& c, const orbmi_pose_obs& o, double p[3],
                                  double& invz, double e[3]) {
    const double X[3] = {o.Xw[0], o.Xw[1], o.Xw[2]};
    se3_map(T, X, p);
    invz = fast_rcp(p[2]);
    if (o.ur < 0) {
        e[0] = (double)o.u - (p[0] * invz * c.fx + c.cx);
        e[1] = (double)o.v - (p[1] * invz * c.fy + c.cy);
        e[2] = 0;
    } else {
        const float fz = (float)invz;
        const double r0 = p[0] * fz * c.fx + c.cx;
        const double r1 = p[1] * fz * c.fy + c.cy;
        e[0] = (double)o.u - r0;
        e[1] = (double)o.v - r1;
        e[2] = (double)o.ur - (r0 - c.bf * fz);
    }
}

// The pass's pose as a rotation matrix and translation, formed once per pass and held in SGPRs
// (the pose is the same for every lane: readfirstlane), so each edge's camera-frame point is
// 9 FMAs (p = R X + t) instead of the quaternion rotation's ~24 operations
struct PoseRt { double r[9], t[3]; };
__device__ inline double uniform_d(double v) {
    const unsigned long long x = __double_as_longlong(v);
    const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)x), hi = __builtin_amdgcn_readfirstlane((unsigned)(x >> 32));
    return __longlong_as_double(((unsigned long long)hi << 32) | lo);
}
__device__ inline PoseRt pose_rt(const double* T) {
    double R[3][3];
    q_to_matrix(load_q(T), R);
    PoseRt P;
#pragma unroll
    for (int k = 0; k < 9; k++) P.r[k] = R[k / 3][k % 3];
#pragma unroll
    for (int k = 0; k < 3; k++) P.t[k] = T[4 + k];
    return P;
}
__device__ inline void pose_error_rt(const PoseRt& P, const PoseCam& c, const orbmi_pose_obs& o, double p[3],
                                     double& invz, double e[3]) {
    const double X[3] = {o.Xw[0], o.Xw[1], o.Xw[2]};
#pragma unroll
    for (int r = 0; r < 3; r++) p[r] = fma(P.r[3 * r], X[0], fma(P.r[3 * r + 1], X[1], fma(P.r[3 * r + 2], X[2], P.t[r])));
    invz = fast_rcp(p[2]);
    if (o.ur < 0) {
        e[0] = (double)o.u - (p[0] * invz * c.fx + c.cx);
        e[1] = (double)o.v - (p[1] * invz * c.fy + c.cy);
        e[2] = 0;
    } else {
        const float fz = (float)invz;
        const double r0 = p[0] * fz * c.fx + c.cx;
        const double r1 = p[1] * fz * c.fy + c.cy;
        e[0] = (double)o.u - r0;
        e[1] = (double)o.v - r1;
        e[2] = (double)o.ur - (r0 - c.bf * fz);
    }
}

__device__ inline double pose_chi2(const orbmi_pose_obs& o, const double e[3]) {
    const double info = (double)o.inv_sigma2;
    return e[0] * (info * e[0]) + e[1] * (info * e[1]) + (o.ur < 0 ? 0.0 : e[2] * (info * e[2]));
}

// fixed-order workgroup sum of the 28 normal-equation terms into wave 0: each of the first
// kPoseFullWaves waves (the ones that ran buildSystem) reduce-scatters its lanes' terms (DPP /
// permlane swaps) and writes one LDS slot per (wave, value); after the barrier wave 0's lane q
// sums value q over those waves in wave order, stores it in stot[q] and every lane of wave 0
// reads the 28 totals back (broadcast LDS reads).  The other waves' acc is left unspecified;
// stot keeps the system for a later re-solve.
__device__ inline void pose_reduce28_w0(double (&acc)[28], double (*red)[32], double* stot) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    if (wid < kPoseFullWaves) {
        double v[32];
#pragma unroll
        for (int q = 0; q < 28; q++) v[q] = acc[q];
        v[28] = v[29] = v[30] = v[31] = 0;
        const double s = wave_reduce_scatter32(v);
        if (!(lane & 1)) red[wid][lane >> 1] = s;
    }
    __syncthreads();
    if (wid == 0) {
        double t = 0;
#pragma unroll
        for (int w = 0; w < kPoseFullWaves; w++) t += red[w][lane & 31];
        if (lane < 28) stot[lane] = t;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
        for (int q = 0; q < 28; q++) acc[q] = stot[q];
    }
}

__device__ inline double pose_reduce1(double v, double* red1) {
    v = wave_sum(v);
    if ((threadIdx.x & 63) == 0) red1[threadIdx.x >> 6] = v;
    __syncthreads();
    double t = 0;
#pragma unroll
    for (int w = 0; w < kPoseWaves; w++) t += red1[w];
    return t;
}

// LDL^T solve of the damped 6x6 system (LinearSolverDense); false on a non-positive pivot.
// LD[i][k] = L[i][k] * D[k] is kept so every inner product is a chain of FMAs.
__device__ inline bool pose_solve6(const double H[21], const double b[6], double lam, double x[6]) {
    double A[6][6], LD[6][6];
    {
        int q = 0;
#pragma unroll
        for (int r = 0; r < 6; r++)
#pragma unroll
            for (int c = r; c < 6; c++, q++) A[c][r] = H[q];  // lower triangle
    }
#pragma unroll
    for (int j = 0; j < 6; j++) A[j][j] += lam;
    bool ok = true;
    double inv[6];
#pragma unroll
    for (int j = 0; j < 6; j++) {
        double d = A[j][j];
#pragma unroll
        for (int k = 0; k < j; k++) d -= A[j][k] * LD[j][k];
        ok &= (fabs(d) > 0) && isfinite(d);
        A[j][j] = d;
        inv[j] = fast_rcp(d);
#pragma unroll
        for (int i = j + 1; i < 6; i++) {
            double s = A[i][j];
#pragma unroll
            for (int k = 0; k < j; k++) s -= A[i][k] * LD[j][k];
            LD[i][j] = s;          // L[i][j] * D[j]
            A[i][j] = s * inv[j];  // L[i][j]
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
    for (int i = 0; i < 6; i++) y[i] *= inv[i];
#pragma unroll
    for (int i = 5; i >= 0; i--) {
        double s = y[i];
#pragma unroll
        for (int k = i + 1; k < 6; k++) s -= A[k][i] * x[k];
        x[i] = s;
    }
    return ok;
}

// linearizeOplus + constructQuadraticForm of one edge at its camera-frame point p (1/z = invz),
// error e and weight wsel = rho' * information
__device__ inline void pose_quadratic(const PoseCam& cam, bool stereo, const double p[3], double invz, const double e[3],
                                      double wsel, double (&acc)[28]) {
    // linearizeOplus (types_six_dof_expmap.cpp:266-290, :332-364) in normalised coordinates
    // X = x / z, Y = y / z; J[0][4] = J[1][3] = J[2][4] = 0 and the third row is zero for
    // monocular edges: those products are skipped.  Every term is one FMA into its
    // accumulator (the contraction order differs from g2o's by rounding only).
    const double iz = invz, X = p[0] * iz, Y = p[1] * iz;
    const double Xfx = X * cam.fx, Yfy = Y * cam.fy;
    const double a0 = Xfx * Y, a1 = -(cam.fx + X * Xfx), a2 = Y * cam.fx, a3 = -iz * cam.fx, a5 = Xfx * iz;
    const double b0 = cam.fy + Y * Yfy, b1 = -X * Yfy, b2 = -X * cam.fy, b4 = -iz * cam.fy, b5 = Yfy * iz;
    const double w = wsel;  // robustInformation
    const double wa0 = w * a0, wa1 = w * a1, wa2 = w * a2, wa3 = w * a3, wa5 = w * a5;
    const double wb0 = w * b0, wb1 = w * b1, wb2 = w * b2, wb4 = w * b4, wb5 = w * b5;
    const double ea = w * e[0], eb = w * e[1];
    // upper triangle, row-major: (0,0..5) (1,1..5) (2,2..5) (3,3..5) (4,4..5) (5,5)
    acc[0] += a0 * wa0;  acc[0] += b0 * wb0;  acc[1] += a0 * wa1;  acc[1] += b0 * wb1;
    acc[2] += a0 * wa2;  acc[2] += b0 * wb2;  acc[3] += a0 * wa3;  acc[4] += b0 * wb4;
    acc[5] += a0 * wa5;  acc[5] += b0 * wb5;
    acc[6] += a1 * wa1;  acc[6] += b1 * wb1;  acc[7] += a1 * wa2;  acc[7] += b1 * wb2;
    acc[8] += a1 * wa3;  acc[9] += b1 * wb4;  acc[10] += a1 * wa5; acc[10] += b1 * wb5;
    acc[11] += a2 * wa2; acc[11] += b2 * wb2; acc[12] += a2 * wa3; acc[13] += b2 * wb4;
    acc[14] += a2 * wa5; acc[14] += b2 * wb5;
    acc[15] += a3 * wa3; acc[17] += a3 * wa5;  // acc[16] = H(3,4) = 0
    acc[18] += b4 * wb4; acc[19] += b4 * wb5;
    acc[20] += a5 * wa5; acc[20] += b5 * wb5;
    acc[21] -= a0 * ea;  acc[21] -= b0 * eb;  acc[22] -= a1 * ea;  acc[22] -= b1 * eb;
    acc[23] -= a2 * ea;  acc[23] -= b2 * eb;  acc[24] -= a3 * ea;  acc[25] -= b4 * eb;
    acc[26] -= a5 * ea;  acc[26] -= b5 * eb;
    {  // stereo: third row, J[2] = J[0] + bf / z^2 * (-y, x, 0, 0, 0, -1); weight 0 for a
       // monocular edge (branch-free: a wave with both kinds runs both paths anyway)
        const double bfz = cam.bf * iz, wm = stereo ? w : 0.0;
        const double c0 = a0 - bfz * Y, c1 = a1 + bfz * X, c2_ = a2, c3 = a3, c5 = a5 - bfz * iz;
        const double wc0 = wm * c0, wc1 = wm * c1, wc2 = wm * c2_, wc3 = wm * c3, wc5 = wm * c5;
        const double ec = wm * e[2];
        acc[0] += c0 * wc0;  acc[1] += c0 * wc1;  acc[2] += c0 * wc2;  acc[3] += c0 * wc3;  acc[5] += c0 * wc5;
        acc[6] += c1 * wc1;  acc[7] += c1 * wc2;  acc[8] += c1 * wc3;  acc[10] += c1 * wc5;
        acc[11] += c2_ * wc2; acc[12] += c2_ * wc3; acc[14] += c2_ * wc5;
        acc[15] += c3 * wc3; acc[17] += c3 * wc5;
        acc[20] += c5 * wc5;
        acc[21] -= c0 * ec;  acc[22] -= c1 * ec;  acc[23] -= c2_ * ec; acc[24] -= c3 * ec;  acc[26] -= c5 * ec;
    }
}

// computeActiveErrors + activeRobustChi2 + buildSystem at T for this thread's level-0 edges
// (threads < kPoseFullThreads):
// acc[0..20] = upper 6x6 of J^T W J, acc[21..26] = b, acc[27] = robust chi2; schi = (float) chi2
// of each edge (the stale errors the outlier test reads).
__device__ inline void pose_pass(const double* T, const PoseCam& cam, const orbmi_pose_obs* sobs, const uint8_t* outl,
                                 float* schi, int n, bool robust, double (&acc)[28]) {
#pragma unroll
    for (int q = 0; q < 28; q++) acc[q] = 0;
    const int k0 = threadIdx.x < kPoseFullThreads ? (int)threadIdx.x : n;  // the other waves: no edges
    const PoseRt P = pose_rt(T);
    for (int k = k0; k < n; k += kPoseFullThreads) {
        if (outl[k]) continue;
        const orbmi_pose_obs o = sobs[k];
        double p[3], invz, e[3];
        pose_error_rt(P, cam, o, p, invz, e);
        const double c2 = pose_chi2(o, e), info = (double)o.inv_sigma2;
        schi[k] = (float)c2;
        double rho0 = c2, rho1 = 1.0;
        if (robust) {
            const double d = pose_delta(o), dsqr = d * d;
            if (c2 > dsqr) { const double r = fast_rsqrt(c2), sq = c2 * r; rho0 = 2 * sq * d - dsqr; rho1 = d * r; }
        }
        acc[27] += rho0;
        pose_quadratic(cam, !(o.ur < 0), p, invz, e, rho1 * info, acc);
    }
}

// A trial of the Levenberg chain: the pose oplus(x) * T, scale = x^T (lambda x + b) and whether
// the damped solve succeeded (else T itself, x = 0: tempChi is then DBL_MAX).
constexpr int kPoseCands = 16;
struct PoseCand { double T[8]; double scale; double ok; };

// Wave 0, lane-parallel: lane j < kPoseCands solves (H + lambda_j I) x = b for the damping of the
// trial after j rejections (lambda *= ni; ni *= 2 per rejection, levenberg.cpp:143-146 -- the
// same multiplications in the same order) and publishes the trial pose in cand[j].
__device__ inline void pose_candidates(const double (&hb)[28], double lambda, double ni, const double* T,
                                       PoseCand* cand) {
    const int lane = threadIdx.x & 63;
    double l = lambda, nn = ni;
#pragma unroll
    for (int m = 0; m < kPoseCands - 1; m++)
        if (m < lane) { l *= nn; nn *= 2; }
    double xv[6], Tt[8];
    const bool ok = pose_solve6(hb, hb + 21, l, xv);
    if (ok) se3_oplus(xv, T, Tt);
    else {
#pragma unroll
        for (int q = 0; q < 8; q++) Tt[q] = T[q];
#pragma unroll
        for (int q = 0; q < 6; q++) xv[q] = 0;
    }
    double scale = 0;
#pragma unroll
    for (int j = 0; j < 6; j++) scale += xv[j] * (l * xv[j] + hb[21 + j]);
    if (lane < kPoseCands) {
#pragma unroll
        for (int q = 0; q < 8; q++) cand[lane].T[q] = Tt[q];
        cand[lane].scale = scale;
        cand[lane].ok = ok ? 1.0 : 0.0;
    }
}

// computeActiveErrors + activeRobustChi2 only (a trial's evaluation): this thread's robust chi2
// sum; schi as pose_pass.  The Jacobians are formed only if the trial is accepted.
__device__ inline double pose_chi_pass(const double* T, const PoseCam& cam, const orbmi_pose_obs* sobs,
                                       const uint8_t* outl, float* schi, int n, bool robust) {
    double chi = 0;
    const PoseRt P = pose_rt(T);
    for (int k = threadIdx.x; k < n; k += kPoseThreads) {
        if (outl[k]) continue;
        const orbmi_pose_obs o = sobs[k];
        double p[3], invz, e[3];
        pose_error_rt(P, cam, o, p, invz, e);
        const double c2 = pose_chi2(o, e);
        schi[k] = (float)c2;
        double rho0 = c2;
        if (robust) {
            const double d = pose_delta(o), dsqr = d * d;
            if (c2 > dsqr) rho0 = 2 * (c2 * fast_rsqrt(c2)) * d - dsqr;
        }
        chi += rho0;
    }
    return chi;
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
    // orbmi_pose_optimization_frame_track: Tracking's pass over mvpMapPoints (track_update.h)
    // as the kernel's tail, on the keypoints' final outlier flags; upd_counts == NULL: none
    int* upd_counts;
    int upd_stage;
    uint8_t* upd_occ;
    int* upd_match_lf;      // match_lf / match_mp, which the update rewrites
    int* upd_match_mp;
};


// One workgroup per frame.  The Levenberg trial pass is fused with the next iteration's
// buildSystem: g2o's next iteration starts with computeActiveErrors + buildSystem at the state
// the accepted trial left (levenberg.cpp:67-85), so the trial pass accumulates J^T W J and b at
// the trial pose too, and an accepted trial hands them on (a rejected one keeps H, b: g2o
// re-solves the same system with a larger lambda).  One edge pass + one reduction per trial.
// TR = event trace (orbmi_debug_pose_trace): lane 0 of every wave stamps s_memtime per edge
// pass (seq) into trace[16 + (seq * kPoseTraceWaves + wave) * 8 + e]: e = 0 pass start, 1 pass end,
// 2 chi2 barrier (B1) passed, 3 Levenberg decision taken, 4 (accepted trial) system reduced,
// 5 (wave 0) trial chain published, 6 candidates barrier (B3) passed, 7 (accepted trial) full
// pass done; trace[0] = total cycles,
// [1] = total s_memrealtime ticks, [2] = passes of thread 0's wave.
// GATHER = the edge assembly (PoseGatherArgs g) runs in the prologue, straight into LDS: the
// frame record is g.rec, edges are compacted in keypoint order by a workgroup scan, mvbOutlier
// is written per keypoint (by_index) and zeroed for keypoints without a map point.
template <bool TR, bool GATHER>
__global__ __launch_bounds__(kPoseThreads) void k_pose_opt(orbmi_pose_frame* __restrict__ frames,
                                                           const orbmi_pose_obs* __restrict__ obs,
                                                           uint8_t* __restrict__ outlier_out, int by_index,
                                                           unsigned long long* __restrict__ trace,
                                                           PoseGatherArgs g) {
    __shared__ orbmi_pose_obs sobs[kPoseMaxObs];
    __shared__ float schi[kPoseMaxObs];    // (float) chi2 of the last computeActiveErrors
    __shared__ uint8_t outl[kPoseMaxObs];  // mvbOutlier; the edge's level is the same flag
    __shared__ uint8_t eflag[GATHER ? kPoseMaxObs : 1];  // gather: 1 = point from match_mp, 2 = Observations() > 0
    __shared__ double red[2][kPoseWaves][32];
    __shared__ double red1[2][kPoseWaves];
    __shared__ PoseCand scand[kPoseCands];  // wave 0's trial chain
    __shared__ double stot[32];              // wave 0's reduced system (H upper, b, chi2)
    __shared__ double chiw[2][kPoseWaves];   // per-wave chi2 of a trial pass
    int cb = 0;                              // chiw buffer
    unsigned long long tstart = 0, rstart = 0;
    if (TR && threadIdx.x == 0) { tstart = __builtin_amdgcn_s_memtime(); rstart = __builtin_amdgcn_s_memrealtime(); }
    int seq = 0;  // passes run by this wave (trace builds)
    auto evp = [&]() -> unsigned long long* {
        return (TR && seq < kPoseTraceSeqs) ? trace + 16 + (seq * kPoseTraceWaves + (threadIdx.x >> 6)) * 8 : nullptr;
    };
#define EV(e)                                                                                    \
    if (TR && (threadIdx.x & 63) == 0 && seq < kPoseTraceSeqs) evp()[e] = __builtin_amdgcn_s_memtime();
    const int tid = threadIdx.x;
    orbmi_pose_frame& F = GATHER ? *g.rec : frames[blockIdx.x];
    int n, nkp = 0;
    const orbmi_pose_obs* O = nullptr;
    float tcw0[12];
    PoseCam cam;
    if (GATHER) {  // Optimizer::PoseOptimization's edge loop (src/Optimizer.cc:296-375)
        __shared__ int gscan[kPoseWaves + 1];
        nkp = g.n_dev ? min(*g.n_dev, g.n) : g.n;
        // each thread owns a contiguous run of keypoints: count, one block scan, then write in
        // keypoint order (2 barriers whatever the keypoint count)
        const int per = (nkp + kPoseThreads - 1) / kPoseThreads;
        const int i0 = min(tid * per, nkp), i1 = min(i0 + per, nkp);
        // the point of keypoint i: mps[match_mp[i]] if in range, else lfp[match_lf[i]] if in
        // range (out-of-range indices read as NULL); its flags give Observations() > 0
        struct PointRef { const float* X; uint8_t ef; };
        auto point_ref = [&](int i, int jm, int jl) -> PointRef {
            if (jm >= 0 && jm < g.n_mp) return {g.mps[jm].pos, (uint8_t)(1 | ((g.mps[jm].flags & ORBMI_MP_HAS_OBS) ? 2 : 0))};
            if (jl >= 0 && jl < g.n_lf) return {g.lfp[jl].pos, (uint8_t)((g.lfp[jl].flags & ORBMI_MP_HAS_OBS) ? 2 : 0)};
            return {nullptr, 0};
        };
        auto put_edge = [&](int off, int i, const float* X, const orbmi_keypoint& kp, float ur, uint8_t ef) {
            orbmi_pose_obs o;
            o.Xw[0] = X[0]; o.Xw[1] = X[1]; o.Xw[2] = X[2];
            o.u = kp.x;
            o.v = kp.y;
            o.ur = ur;
            const int oct = min(max(kp.octave, 0), g.nlevels - 1);
            o.inv_sigma2 = g.inv_sigma2[oct];
            o.index = i;
            sobs[off] = o;
            outl[off] = 0;
            eflag[off] = ef;
        };
        int total;
        constexpr int kGP = 8;  // keypoints per thread gathered with their loads in flight together
        if (per <= kGP) {
            // round trip 1: the match indices; round trip 2: the points, their flags and the
            // keypoints (indices clamped into range: straight-line loads, a dependent chain per
            // batch instead of per keypoint)
            int jm[kGP], jl[kGP];
#pragma unroll
            for (int u = 0; u < kGP; u++) {
                const int i = min(i0 + u, max(nkp - 1, 0));
                jm[u] = (u < per && g.match_mp) ? g.match_mp[i] : -1;
                jl[u] = (u < per && g.match_lf) ? g.match_lf[i] : -1;
            }
            PointRef P[kGP];
            float Xv[kGP][3], ur[kGP];
            orbmi_keypoint kp[kGP];
            int cnt = 0;
#pragma unroll
            for (int u = 0; u < kGP; u++) {
                const int i = i0 + u;
                P[u] = i < i1 ? point_ref(i, jm[u], jl[u]) : PointRef{nullptr, 0};
                cnt += P[u].X != nullptr;
                if (P[u].X) {
                    Xv[u][0] = P[u].X[0]; Xv[u][1] = P[u].X[1]; Xv[u][2] = P[u].X[2];
                    kp[u] = g.keys[i];
                    ur[u] = g.u_right ? g.u_right[i] : -1.0f;
                }
            }
            int off = block_excl_scan(cnt, gscan, &total);
#pragma unroll
            for (int u = 0; u < kGP; u++) {
                const int i = i0 + u;
                if (i >= i1) continue;
                g.outlier[i] = 0;
                if (!P[u].X) continue;
                if (off < kPoseMaxObs) put_edge(off, i, Xv[u], kp[u], ur[u], P[u].ef);
                off++;
            }
        } else {  // more keypoints than kGP per thread: one at a time
            auto ref_of = [&](int i) {
                return point_ref(i, g.match_mp ? g.match_mp[i] : -1, g.match_lf ? g.match_lf[i] : -1);
            };
            int cnt = 0;
            for (int i = i0; i < i1; i++) cnt += ref_of(i).X != nullptr;
            int off = block_excl_scan(cnt, gscan, &total);
            for (int i = i0; i < i1; i++) {
                const PointRef r = ref_of(i);
                g.outlier[i] = 0;
                if (!r.X) continue;
                if (off < kPoseMaxObs) put_edge(off, i, r.X, g.keys[i], g.u_right ? g.u_right[i] : -1.0f, r.ef);
                off++;
            }
        }
        n = total;
        for (int q = 0; q < 12; q++) tcw0[q] = g.tcw_dev ? g.tcw_dev[q] : g.tcw[q];
        cam = PoseCam{g.fx, g.fy, g.cx, g.cy, g.bf};
        if (tid < 16) F.tcw[tid] = tid < 12 ? tcw0[tid] : (tid == 15 ? 1.f : 0.f);
        if (tid == 0) {
            F.fx = g.fx; F.fy = g.fy; F.cx = g.cx; F.cy = g.cy; F.bf = g.bf;
            F.obs_begin = 0;
            F.n_obs = n;
        }
    } else {
        n = F.n_obs;
        O = obs + F.obs_begin;
        for (int q = 0; q < 12; q++) tcw0[q] = F.tcw[q];
        cam = PoseCam{F.fx, F.fy, F.cx, F.cy, F.bf};
    }
    // mvbOutlier per observation (orbmi_pose_optimization) or per keypoint (by_index: obs.index)
    auto put_flag = [&](int k, uint8_t v) {
        if (by_index) outlier_out[GATHER ? sobs[k].index : O[k].index] = v;
        else outlier_out[F.obs_begin + k] = v;
    };
    // sized for kPoseMaxObs edges per frame (the host path checks first); fewer than 3: no
    // optimisation, pose untouched (src/Optimizer.cc:378-379; the gather zeroed every flag)
    const bool run = n >= 3 && n <= kPoseMaxObs;
    if (!run) {
        if (!GATHER && n <= kPoseMaxObs)
            for (int k = tid; k < n; k += kPoseThreads) put_flag(k, 0);
        if (tid == 0) { F.inliers = n > kPoseMaxObs ? -1 : 0; F.iterations = 0; }
    }
    if (run) {
        if (!GATHER)
            for (int k = tid; k < n; k += kPoseThreads) { sobs[k] = O[k]; outl[k] = 0; }
        double T0[8];  // Converter::toSE3Quat(pFrame->mTcw)
        {
            double R[3][3];
            for (int r = 0; r < 3; r++)
                for (int c = 0; c < 3; c++) R[r][c] = tcw0[4 * r + c];
            Q q = q_from_matrix(R);
            q_normalize(q);
            T0[0] = q.x; T0[1] = q.y; T0[2] = q.z; T0[3] = q.w;
            T0[4] = tcw0[3]; T0[5] = tcw0[7]; T0[6] = tcw0[11]; T0[7] = 0;
        }
        double T[8];
        int nBad = 0, iters = 0, rb = 0;  // rb: alternating reduction buffer
        const int wid = tid >> 6;
        __syncthreads();
        for (int it = 0; it < 4; it++) {
            const bool robust = it < 3;  // setRobustKernel(0) after the third round (:463-464)
#pragma unroll
            for (int q = 0; q < 8; q++) T[q] = T0[q];
            double nact = 0;
            for (int k = tid; k < n; k += kPoseThreads) nact += !outl[k];
            nact = pose_reduce1(nact, red1[rb]);
            rb ^= 1;
            if (nact > 0) {
                // ---- optimize(10) on the level-0 edges.  Every wave runs the edge passes and the
                // Levenberg decisions (replicated: the same instructions on the same LDS values, so
                // every wave takes the same branch).  Wave 0 holds the reduced system and publishes,
                // in scand, the trial poses of the whole rejected-trial chain that follows it (lane j
                // solves for the lambda after j rejections): a rejected trial needs only the chi2
                // sum of its pass, and only an accepted trial pays for the 28-value reduction and a
                // fresh solve.
                double acc[28];
                double lambda = 0, ni = 2;  // meaningful in wave 0 only
                double currentChi = 0, iniChi = 0;
                int cj = 0, qmax = 0, nbadIt = 0, i = 0;
                bool first = true;  // the pass at T: computeActiveErrors + buildSystem of iteration 0
                for (;;) {
                    bool accept = true, regen = false;
                    if (!first) {
                        // trial cj of the chain: the pose of oplus(x(lambda_cj)), evaluated by all waves
                        double Tt[8];
#pragma unroll
                        for (int q = 0; q < 8; q++) Tt[q] = scand[cj].T[q];
                        const bool ok2 = scand[cj].ok != 0;
                        const double scale = scand[cj].scale;
                        seq++;
                        EV(0);
                        {
                            const double c = wave_sum(pose_chi_pass(Tt, cam, sobs, outl, schi, n, robust));
                            EV(1);
                            if ((tid & 63) == 0) chiw[cb][wid] = c;
                        }
                        __syncthreads();  // B1: the trial's chi2 partials
                        EV(2);
                        double tempChi = 0;
#pragma unroll
                        for (int w = 0; w < kPoseWaves; w++) tempChi += chiw[cb][w];
                        cb ^= 1;
                        if (!ok2) tempChi = DBL_MAX;
                        const double rho = (currentChi - tempChi) * fast_rcp(scale + 1e-3);
                        accept = rho > 0 && isfinite(tempChi);
                        if (accept) {
                            const double t = 2 * rho - 1;
                            double alpha = 1. - t * t * t;
                            alpha = fmin(alpha, 2. / 3.);
                            lambda *= fmax(1. / 3., alpha);
                            ni = 2;
                            currentChi = tempChi;
#pragma unroll
                            for (int q = 0; q < 8; q++) T[q] = Tt[q];
                        } else {
                            lambda *= ni;
                            ni *= 2;
                            cj++;
                        }
                        qmax++;
                        bool done = false;
                        if (!(rho < 0 && qmax < 10)) {  // the do-while of iteration i ends
                            iters++;
                            if (qmax == 10 || rho == 0) done = true;
                            else {
                                if ((iniChi - currentChi) * 1e3 < iniChi) nbadIt++;
                                else nbadIt = 0;
                                if (nbadIt >= 3 || ++i >= 10) done = true;
                                iniChi = currentChi;
                                qmax = 0;
                            }
                        }
                        EV(3);
                        if (done) break;
                        regen = !accept && cj == kPoseCands;  // chain exhausted: continue it
                    }
                    if (accept || regen) {
                        if (accept) {  // buildSystem at the (new) estimate: the first iteration's, or
                                       // the next iteration's after an accepted trial
                            pose_pass(T, cam, sobs, outl, schi, n, robust, acc);
                            EV(7);
                            pose_reduce28_w0(acc, red[rb], stot);  // B2 inside
                            rb ^= 1;
                        } else {
                            __syncthreads();  // every wave has read scand
                            if (wid == 0) {
#pragma unroll
                                for (int q = 0; q < 28; q++) acc[q] = stot[q];
                            }
                        }
                        EV(4);
                        if (wid == 0) {
                            if (first)  // computeLambdaInit, tau = 1e-5
                                lambda = 1e-5 * fmax(fmax(fmax(fabs(acc[0]), fabs(acc[6])), fmax(fabs(acc[11]), fabs(acc[15]))),
                                                     fmax(fabs(acc[18]), fabs(acc[20])));
                            pose_candidates(acc, lambda, ni, T, scand);
                            EV(5);
                        }
                        cj = 0;
                        __syncthreads();  // B3: the trial chain published
                        EV(6);
                        if (first) {
                            currentChi = iniChi = stot[27];
                            first = false;
                        }
                    }
                }
            }
            // ---- outlier classification (:418-466): stale errors of the inliers, fresh ones of the
            // outliers, chi2 compared in float
            double bad = 0;
            for (int k = tid; k < n; k += kPoseThreads) {
                const orbmi_pose_obs o = sobs[k];
                float c2 = schi[k];
                if (outl[k]) {
                    double p[3], invz, e[3];
                    pose_error(T, cam, o, p, invz, e);
                    c2 = (float)pose_chi2(o, e);
                    schi[k] = c2;
                }
                const bool out = c2 > (o.ur < 0 ? 5.991f : 7.815f);
                outl[k] = out;
                bad += out;
            }
            nBad = (int)pose_reduce1(bad, red1[rb]);
            rb ^= 1;
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
        if (TR && tid == 0) {
            trace[0] = __builtin_amdgcn_s_memtime() - tstart;
            trace[1] = __builtin_amdgcn_s_memrealtime() - rstart;
            trace[2] = seq;
        }
    }  // run
    if (GATHER && g.upd_counts) {  // Tracking's pass over mvpMapPoints (track_update.h) on the final flags
        __shared__ int ucnt[2];
        if (n <= kPoseMaxObs) {
            // from the edges in LDS: keypoint, final mvbOutlier, which match array holds the point
            // and its Observations() > 0 (eflag), so no global load; keypoints without a point
            // only get occupied_out = 0 (zeroed first, then the edges' values)
            if (tid < 2) ucnt[tid] = 0;
            if (g.upd_occ)
                for (int i = tid; i < nkp; i += kPoseThreads) g.upd_occ[i] = 0;
            __syncthreads();
            const bool stereo = g.u_right != nullptr;
            int c0 = 0, c1 = 0;
            for (int k = tid; k < n; k += kPoseThreads) {
                const int i = sobs[k].index;
                const uint8_t ef = eflag[k];
                const bool out = outl[k] != 0, obs = (ef & 2) != 0;
                int* slot = (ef & 1) ? &g.upd_match_mp[i] : &g.upd_match_lf[i];
                if (g.upd_stage == 0) {  // src/Tracking.cc:1042-1055
                    if (out) { *slot = -1; c0++; }
                    else if (obs) { c1++; if (g.upd_occ) g.upd_occ[i] = 1; }
                } else {                 // :1087-1101
                    if (!out) c0 += obs;
                    else { c1++; if (stereo) *slot = -1; }
                }
            }
            if (c0) atomicAdd(&ucnt[0], c0);
            if (c1) atomicAdd(&ucnt[1], c1);
            __syncthreads();
            if (tid < 2) g.upd_counts[tid] = ucnt[tid];
        } else {  // (more edges than LDS holds: the keypoint form)
            __syncthreads();
            track_update_body(nkp, g.u_right != nullptr, g.upd_stage, g.outlier, g.upd_match_lf, g.lfp, g.n_lf,
                              g.upd_match_mp, g.mps, g.n_mp, g.upd_occ, g.upd_counts, ucnt);
        }
    }
#undef EV
}


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
    // orbmi_pose_set_profiling: HIP event pairs around every stride-th k_pose_opt launch
    int prof_stride = 0;
    long long prof_seq = 0;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> events;
    size_t used_events = 0;
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

// event pair for the next profiled launch (grown on demand, reused after each read)
std::pair<hipEvent_t, hipEvent_t>* next_events(orbmi_pose* h) {
    if (h->used_events == h->events.size()) {
        hipEvent_t a, b;
        if (hipEventCreate(&a) != hipSuccess) return nullptr;
        if (hipEventCreate(&b) != hipSuccess) { (void)hipEventDestroy(a); return nullptr; }
        h->events.emplace_back(a, b);
    }
    return &h->events[h->used_events++];
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
    if (hipSetDevice(device) != hipSuccess || orbmi::stream_create(&h->stream, "POSE") != hipSuccess) {
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
    for (auto& e : h->events) { (void)hipEventDestroy(e.first); (void)hipEventDestroy(e.second); }
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

int orbmi_pose_share_matcher_stream(orbmi_pose* h, orbmi_matcher* m) {
    if (!h || !m) return ORBMI_E_ARG;
    void* sv = nullptr;
    if (orbmi_matcher_get_stream(m, &sv) != ORBMI_OK || !sv) return ORBMI_E_STATE;
    ORBMI_HIP(hipSetDevice(h->device));
    ORBMI_HIP(hipStreamSynchronize(h->stream));
    if (h->own_stream) ORBMI_HIP(hipStreamDestroy(h->stream));
    h->stream = (hipStream_t)sv;
    h->own_stream = false;
    return ORBMI_OK;
}

int orbmi_pose_set_profiling(orbmi_pose* h, int on) {
    if (!h) return ORBMI_E_ARG;
    h->prof_stride = on > 0 ? on : 0;
    h->prof_seq = 0;
    return ORBMI_OK;
}

int orbmi_pose_read_profile(orbmi_pose* h, double* ms, long long* launches) {
    if (!h || !ms || !launches) return ORBMI_E_ARG;
    ORBMI_HIP(hipSetDevice(h->device));
    ORBMI_HIP(hipStreamSynchronize(h->stream));
    double t = 0;
    for (size_t i = 0; i < h->used_events; i++) {
        float e = 0;
        ORBMI_HIP(hipEventElapsedTime(&e, h->events[i].first, h->events[i].second));
        t += e;
    }
    *ms = t;
    *launches = (long long)h->used_events;
    h->used_events = 0;
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
        hipLaunchKernelGGL((k_pose_opt<false, false>), dim3(nframes), dim3(kPoseThreads), 0, h->stream, frames, obs, outlier, 0,
                           nullptr, PoseGatherArgs{});
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
    hipLaunchKernelGGL((k_pose_opt<false, false>), dim3(nframes), dim3(kPoseThreads), 0, h->stream, dF, dO, dFl, 0, nullptr,
                       PoseGatherArgs{});
    ORBMI_HIP(hipGetLastError());
    ORBMI_HIP(hipMemcpyAsync(frames, dF, fb, hipMemcpyDeviceToHost, h->stream));
    if (nobs) ORBMI_HIP(hipMemcpyAsync(outlier, dFl, nobs, hipMemcpyDeviceToHost, h->stream));
    ORBMI_HIP(hipStreamSynchronize(h->stream));
    return ORBMI_OK;
}

}  // extern "C"

namespace {

// Tracking's update pass fused into the launch (orbmi_pose_optimization_frame_track)
struct TrackUpd { int stage; uint8_t* occ; int* counts; };

int pose_frame(orbmi_pose* h, const orbmi_frame_view* F, const float* inv_level_sigma2, const orbmi_frame_mappoints* mp,
               orbmi_pose_frame* rec, uint8_t* outlier, const TrackUpd* upd) {
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
    if (upd) {  // device arrays only (checked by the caller): the update rewrites them in place
        a.upd_counts = upd->counts;
        a.upd_stage = upd->stage;
        a.upd_occ = upd->occ;
        a.upd_match_lf = const_cast<int*>(a.match_lf);
        a.upd_match_mp = const_cast<int*>(a.match_mp);
    }
    if (rc) return rc;
    auto* ev = (h->prof_stride > 0 && h->prof_seq++ % h->prof_stride == 0) ? next_events(h) : nullptr;
    if (ev) ORBMI_HIP(hipEventRecord(ev->first, h->stream));
    // edge assembly fused into the optimiser's prologue (k_pose_gather is the standalone form)
    hipLaunchKernelGGL((k_pose_opt<false, true>), dim3(1), dim3(kPoseThreads), 0, h->stream, a.rec,
                       (const orbmi_pose_obs*)nullptr, a.outlier, 1, nullptr, a);
    ORBMI_HIP(hipGetLastError());
    if (ev) ORBMI_HIP(hipEventRecord(ev->second, h->stream));
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

}  // namespace

extern "C" {

int orbmi_pose_optimization_frame(orbmi_pose* h, const orbmi_frame_view* F, const float* inv_level_sigma2,
                                  const orbmi_frame_mappoints* mp, orbmi_pose_frame* rec, uint8_t* outlier) {
    return pose_frame(h, F, inv_level_sigma2, mp, rec, outlier, nullptr);
}

int orbmi_pose_optimization_frame_track(orbmi_pose* h, const orbmi_frame_view* F, const float* inv_level_sigma2,
                                        const orbmi_frame_mappoints* mp, orbmi_pose_frame* rec, uint8_t* outlier,
                                        int stage, uint8_t* occupied_out, int* counts) {
    if (!h || !mp || !counts || (stage != 0 && stage != 1)) return ORBMI_E_ARG;
    // one asynchronous launch: every array it reads or writes lives on the device
    auto dev = [](const void* p) { return !p || is_device_ptr(p); };
    if (!is_device_ptr(rec) || !is_device_ptr(outlier) || !is_device_ptr(counts) || !dev(occupied_out) ||
        !dev(mp->match_lf) || !dev(mp->match_mp) || (mp->match_lf && !dev(mp->lf_points)) ||
        (mp->match_mp && !dev(mp->mps)))
        return ORBMI_E_ARG;
    const TrackUpd u{stage, occupied_out, counts};
    return pose_frame(h, F, inv_level_sigma2, mp, rec, outlier, &u);
}

// debug: one traced launch of the pose kernel on device arrays (include/orbmi_debug.h)
int orbmi_debug_pose_trace(orbmi_pose* h, orbmi_pose_frame* frames, const orbmi_pose_obs* obs, uint8_t* outlier,
                           unsigned long long* trace) {
    using namespace orbmi;
    if (!h || !frames || !obs || !outlier || !trace) return ORBMI_E_ARG;
    ORBMI_HIP(hipSetDevice(h->device));
    unsigned long long* d_tr = nullptr;
    ORBMI_HIP(hipMalloc((void**)&d_tr, kPoseTraceWords * sizeof(unsigned long long)));
    hipError_t e = hipMemsetAsync(d_tr, 0, kPoseTraceWords * sizeof(unsigned long long), h->stream);
    if (e == hipSuccess) {
        hipLaunchKernelGGL((k_pose_opt<true, false>), dim3(1), dim3(kPoseThreads), 0, h->stream, frames, obs, outlier, 0, d_tr,
                           PoseGatherArgs{});
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipMemcpyAsync(trace, d_tr, kPoseTraceWords * sizeof(unsigned long long), hipMemcpyDeviceToHost, h->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
    (void)hipFree(d_tr);
    return e == hipSuccess ? ORBMI_OK : ORBMI_E_HIP;
}

}  // extern "C"
