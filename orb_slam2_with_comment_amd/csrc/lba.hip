// Optimizer::LocalBundleAdjustment (src/Optimizer.cc:483-808) on MI355X, fp64.
//
// One persistent workgroup (1024 threads) runs the whole g2o schedule -- optimize(5), outlier
// levels, optimize(10), erase list -- with every Levenberg trial on the device and no host
// round trip (g2o/core/optimization_algorithm_levenberg.cpp:61-164):
//   errors        thread per edge   EdgeSE3ProjectXYZ / EdgeStereoSE3ProjectXYZ::computeError
//   linearise     thread per point  Hll, bl, Hpl blocks (constructQuadraticForm, Huber weights)
//                 wave per pose     Hpp, bp (wave reduction over the pose's observations)
//   Schur         thread per point  D^-1, b_schur -= B D^-1 b_l, H_schur -= B_i D^-1 B_j^T
//                                   accumulated with ds_add_f64 into a packed upper-triangular
//                                   reduced camera system held in LDS
//   solve         block             dense LDL^T of the 6K x 6K system in LDS (K <= 30 poses)
//   update        thread per point/pose  x_l = D^-1 (b_l - B^T x_p); SE3 exp/oplus
// The g2o semantics kept: lambda init tau = 1e-5, rho test with computeScale + 1e-3, the
// ORB-SLAM "3 bad iterations" stop, stale edge errors after a rejected trial, push/pop of
// the estimates, Huber kernels removed for the second pass.  Parity with the oracle: 1e-4.
#include <algorithm>
#include <cfloat>
#include <new>
#include <vector>

#include "extractor.h"

namespace orbmi {

constexpr int kBaThreads = 1024;
constexpr int kBaMaxPoses = 30;                        // 6*30 = 180 unknowns
constexpr int kBaMaxN = 6 * kBaMaxPoses;
constexpr int kBaPacked = kBaMaxN * (kBaMaxN + 1) / 2;  // 16290 doubles = 127 KiB

struct BaArgs {
    int nkf, npt, nedge;
    // inputs
    const orbmi_ba_keyframe* kfs;
    const orbmi_ba_point* pts;
    const orbmi_ba_edge* edges;
    const int* kf_order;       // keyframe indices sorted by id (vertex order)
    const int* pt_start;       // edges of point p: [pt_start[p], pt_start[p+1])  (edges grouped by point)
    const int* kf_start;       // CSR by keyframe over edge indices
    const int* kf_edges;
    const volatile int* stop;  // host-mapped abort flag or nullptr
    // state
    double* T;                 // nkf x 8 : qx qy qz qw tx ty tz -
    double* Tt;                // trial
    double* X;                 // npt x 4
    double* Xt;
    double* err;               // nedge x 3 (stale semantics)
    unsigned char* eflag;      // bit0 level-1, bit1 no robust kernel, bit2 active
    int* pose_idx;             // nkf
    int* pose_kf;              // kBaMaxPoses
    double* Hpl;               // nedge x 18 (pose rows x point cols)
    double* Hll;               // npt x 9
    double* bl;                // npt x 3
    double* Dinv;              // npt x 9
    double* Hpp;               // kBaMaxPoses x 36
    double* bp;                // kBaMaxPoses x 6
    double* xp;                // kBaMaxN
    double* xl;                // npt x 3
    // outputs
    float* out_tcw;
    float* out_pos;
    unsigned char* out_erase;
    int* out_stats;            // [0..1] iterations, [2] aborted, [3] error
    double* out_chi2;          // [0..1]
};

// ---------------------------------------------------------------- SE3Quat helpers (fp64)
struct Q { double x, y, z, w; };

__device__ inline void q_normalize(Q& q) {
    if (q.w < 0) { q.x = -q.x; q.y = -q.y; q.z = -q.z; q.w = -q.w; }
    const double n = sqrt(q.x * q.x + q.y * q.y + q.z * q.z + q.w * q.w);
    q.x /= n; q.y /= n; q.z /= n; q.w /= n;
}

__device__ inline Q q_from_matrix(const double m[3][3]) {
    Q q;
    const double tr = m[0][0] + m[1][1] + m[2][2];
    if (tr > 0) {
        double t = sqrt(tr + 1.0);
        q.w = 0.5 * t;
        t = 0.5 / t;
        q.x = (m[2][1] - m[1][2]) * t;
        q.y = (m[0][2] - m[2][0]) * t;
        q.z = (m[1][0] - m[0][1]) * t;
    } else {
        int i = 0;
        if (m[1][1] > m[0][0]) i = 1;
        if (m[2][2] > m[i][i]) i = 2;
        const int j = (i + 1) % 3, k = (j + 1) % 3;
        double t = sqrt(m[i][i] - m[j][j] - m[k][k] + 1.0);
        double v[3];
        v[i] = 0.5 * t;
        t = 0.5 / t;
        q.w = (m[k][j] - m[j][k]) * t;
        v[j] = (m[j][i] + m[i][j]) * t;
        v[k] = (m[k][i] + m[i][k]) * t;
        q.x = v[0]; q.y = v[1]; q.z = v[2];
    }
    return q;
}

__device__ inline void q_to_matrix(const Q& q, double R[3][3]) {
    const double tx = 2 * q.x, ty = 2 * q.y, tz = 2 * q.z;
    const double twx = tx * q.w, twy = ty * q.w, twz = tz * q.w;
    const double txx = tx * q.x, txy = ty * q.x, txz = tz * q.x;
    const double tyy = ty * q.y, tyz = tz * q.y, tzz = tz * q.z;
    R[0][0] = 1 - (tyy + tzz); R[0][1] = txy - twz; R[0][2] = txz + twy;
    R[1][0] = txy + twz; R[1][1] = 1 - (txx + tzz); R[1][2] = tyz - twx;
    R[2][0] = txz - twy; R[2][1] = tyz + twx; R[2][2] = 1 - (txx + tyy);
}

__device__ inline void q_rotate(const Q& q, const double v[3], double o[3]) {
    double uv[3] = {q.y * v[2] - q.z * v[1], q.z * v[0] - q.x * v[2], q.x * v[1] - q.y * v[0]};
    uv[0] += uv[0]; uv[1] += uv[1]; uv[2] += uv[2];
    o[0] = v[0] + q.w * uv[0] + (q.y * uv[2] - q.z * uv[1]);
    o[1] = v[1] + q.w * uv[1] + (q.z * uv[0] - q.x * uv[2]);
    o[2] = v[2] + q.w * uv[2] + (q.x * uv[1] - q.y * uv[0]);
}

__device__ inline Q load_q(const double* T) { return Q{T[0], T[1], T[2], T[3]}; }

__device__ inline void se3_map(const double* T, const double* p, double o[3]) {
    const Q q = load_q(T);
    q_rotate(q, p, o);
    o[0] += T[4]; o[1] += T[5]; o[2] += T[6];
}

// T <- exp(u) * T   (VertexSE3Expmap::oplusImpl, SE3Quat::exp / operator*)
__device__ inline void se3_oplus(const double* u, const double* Tin, double* Tout) {
    const double w0 = u[0], w1 = u[1], w2 = u[2];
    const double theta = sqrt(w0 * w0 + w1 * w1 + w2 * w2);
    const double O[3][3] = {{0, -w2, w1}, {w2, 0, -w0}, {-w1, w0, 0}};
    double O2[3][3], R[3][3], V[3][3];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) O2[i][j] = O[i][0] * O[0][j] + O[i][1] * O[1][j] + O[i][2] * O[2][j];
    if (theta < 0.00001) {
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++) { R[i][j] = (i == j) + O[i][j] + O2[i][j]; V[i][j] = R[i][j]; }
    } else {
        const double a = sin(theta) / theta, b = (1 - cos(theta)) / (theta * theta);
        const double c = (theta - sin(theta)) / pow(theta, 3);
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++) {
                R[i][j] = (i == j) + a * O[i][j] + b * O2[i][j];
                V[i][j] = (i == j) + b * O[i][j] + c * O2[i][j];
            }
    }
    Q qe = q_from_matrix(R);
    double te[3];
    for (int i = 0; i < 3; i++) te[i] = V[i][0] * u[3] + V[i][1] * u[4] + V[i][2] * u[5];
    q_normalize(qe);
    const Q qb = load_q(Tin);
    const double tb[3] = {Tin[4], Tin[5], Tin[6]};
    double rt[3];
    q_rotate(qe, tb, rt);
    Q r{qe.w * qb.x + qe.x * qb.w + qe.y * qb.z - qe.z * qb.y, qe.w * qb.y + qe.y * qb.w + qe.z * qb.x - qe.x * qb.z,
        qe.w * qb.z + qe.z * qb.w + qe.x * qb.y - qe.y * qb.x, qe.w * qb.w - qe.x * qb.x - qe.y * qb.y - qe.z * qb.z};
    q_normalize(r);
    Tout[0] = r.x; Tout[1] = r.y; Tout[2] = r.z; Tout[3] = r.w;
    Tout[4] = te[0] + rt[0]; Tout[5] = te[1] + rt[1]; Tout[6] = te[2] + rt[2];
}

// ---------------------------------------------------------------- edges
__device__ inline bool edge_stereo(const orbmi_ba_edge& e) { return !(e.ur < 0); }

__device__ inline void edge_error(const BaArgs& a, int i, const double* T, const double* X, double* err) {
    const orbmi_ba_edge e = a.edges[i];
    const orbmi_ba_keyframe& kf = a.kfs[e.kf];
    double p[3];
    se3_map(T + 8 * e.kf, X + 4 * e.point, p);
    if (!edge_stereo(e)) {
        const double px = p[0] / p[2], py = p[1] / p[2];
        err[0] = (double)e.u - (px * (double)kf.fx + (double)kf.cx);
        err[1] = (double)e.v - (py * (double)kf.fy + (double)kf.cy);
        err[2] = 0;
    } else {
        const float invz = (float)(1.0f / p[2]);  // float invz (types_six_dof_expmap.cpp:151)
        const double r0 = p[0] * invz * (double)kf.fx + (double)kf.cx;
        const double r1 = p[1] * invz * (double)kf.fy + (double)kf.cy;
        const double r2 = r0 - (double)(kf.bf * invz);
        err[0] = (double)e.u - r0;
        err[1] = (double)e.v - r1;
        err[2] = (double)e.ur - r2;
    }
}

__device__ inline double edge_chi2(const BaArgs& a, int i) {
    const double* r = a.err + 3 * i;
    const double info = (double)a.edges[i].inv_sigma2;
    return r[0] * (info * r[0]) + r[1] * (info * r[1]) + (edge_stereo(a.edges[i]) ? r[2] * (info * r[2]) : 0.0);
}

__device__ inline double huber_delta(const orbmi_ba_edge& e) {
    // const float thHuberMono = sqrt(5.991), thHuberStereo = sqrt(7.815) (src/Optimizer.cc:599-600)
    const float th = edge_stereo(e) ? (float)sqrt(7.815) : (float)sqrt(5.991);
    return (double)th;
}

// robustified chi2 and weight rho' (RobustKernelHuber::robustify)
__device__ inline void edge_robust(const BaArgs& a, int i, double c, double* rho0, double* rho1) {
    if (a.eflag[i] & 2) { *rho0 = c; *rho1 = 1.0; return; }
    const double d = huber_delta(a.edges[i]), dsqr = d * d;
    if (c <= dsqr) { *rho0 = c; *rho1 = 1.0; }
    else { const double s = sqrt(c); *rho0 = 2 * s * d - dsqr; *rho1 = d / s; }
}

// Jacobians (types_six_dof_expmap.cpp:103-134, :188-234)
__device__ inline void edge_jacobians(const BaArgs& a, int i, const double* T, const double* X, double Jl[3][3],
                                      double Jp[3][6]) {
    const orbmi_ba_edge e = a.edges[i];
    const orbmi_ba_keyframe& kf = a.kfs[e.kf];
    const double* Tk = T + 8 * e.kf;
    double p[3], R[3][3];
    se3_map(Tk, X + 4 * e.point, p);
    q_to_matrix(load_q(Tk), R);
    const double x = p[0], y = p[1], z = p[2], z2 = z * z;
    const double fx = kf.fx, fy = kf.fy, bf = kf.bf;
    if (!edge_stereo(e)) {
        const double t02 = -x / z * fx, t12 = -y / z * fy;
        for (int c = 0; c < 3; c++) {
            Jl[0][c] = -1. / z * (fx * R[0][c] + 0 * R[1][c] + t02 * R[2][c]);
            Jl[1][c] = -1. / z * (0 * R[0][c] + fy * R[1][c] + t12 * R[2][c]);
            Jl[2][c] = 0;
        }
    } else {
        for (int c = 0; c < 3; c++) {
            Jl[0][c] = -fx * R[0][c] / z + fx * x * R[2][c] / z2;
            Jl[1][c] = -fy * R[1][c] / z + fy * y * R[2][c] / z2;
            Jl[2][c] = Jl[0][c] - bf * R[2][c] / z2;
        }
    }
    Jp[0][0] = x * y / z2 * fx; Jp[0][1] = -(1 + (x * x / z2)) * fx; Jp[0][2] = y / z * fx;
    Jp[0][3] = -1. / z * fx; Jp[0][4] = 0; Jp[0][5] = x / z2 * fx;
    Jp[1][0] = (1 + y * y / z2) * fy; Jp[1][1] = -x * y / z2 * fy; Jp[1][2] = -x / z * fy;
    Jp[1][3] = 0; Jp[1][4] = -1. / z * fy; Jp[1][5] = y / z2 * fy;
    if (edge_stereo(e)) {
        Jp[2][0] = Jp[0][0] - bf * y / z2; Jp[2][1] = Jp[0][1] + bf * x / z2; Jp[2][2] = Jp[0][2];
        Jp[2][3] = Jp[0][3]; Jp[2][4] = 0; Jp[2][5] = Jp[0][5] - bf / z2;
    } else {
        for (int c = 0; c < 6; c++) Jp[2][c] = 0;
    }
}

// weight W = rho' * info and omega_r = -info * e * rho' (constructQuadraticForm)
__device__ inline void edge_weights(const BaArgs& a, int i, double* w, double om[3]) {
    const double info = (double)a.edges[i].inv_sigma2;
    double r0, r1;
    edge_robust(a, i, edge_chi2(a, i), &r0, &r1);
    *w = (a.eflag[i] & 2) ? info : r1 * info;
    const double s = (a.eflag[i] & 2) ? 1.0 : r1;
    const double* e = a.err + 3 * i;
    for (int k = 0; k < 3; k++) om[k] = -(info * e[k]) * s;
}

// ---------------------------------------------------------------- block helpers
constexpr int kBaMaxKf = 1024;

struct BaShared {
    double H[kBaPacked];       // packed upper-triangular reduced camera system
    double bs[kBaMaxN];
    int kfact[kBaMaxKf];       // keyframe has an active edge
    double red[kBaThreads / 64];
    double dstate[8];          // lambda, ni, currentChi, tempChi, scale, rho, iniChi
    int istate[16];
};

__device__ inline double block_sum(double v, BaShared& S) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) S.red[threadIdx.x >> 6] = v;
    __syncthreads();
    double t = 0;
    for (int w = 0; w < kBaThreads / 64; w++) t += S.red[w];
    __syncthreads();
    return t;
}

__device__ inline double block_max(double v, BaShared& S) {
    for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, 64));
    __syncthreads();
    if ((threadIdx.x & 63) == 0) S.red[threadIdx.x >> 6] = v;
    __syncthreads();
    double t = 0;
    for (int w = 0; w < kBaThreads / 64; w++) t = fmax(t, S.red[w]);
    __syncthreads();
    return t;
}

__device__ inline int packed(int r, int c, int N) { return r * N - r * (r - 1) / 2 + (c - r); }  // r <= c

__device__ inline bool stop_requested(const BaArgs& a) {
    return a.stop && __hip_atomic_load((int*)a.stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0;
}

// ---------------------------------------------------------------- the optimiser
struct Lba {
    const BaArgs& a;
    BaShared& S;
    int np = 0, N = 0, nl = 0;

    __device__ Lba(const BaArgs& aa, BaShared& ss) : a(aa), S(ss) {}

    // SparseOptimizer::initializeOptimization(level 0) + buildIndexMapping
    __device__ void initialize() {
        const int tid = threadIdx.x;
        for (int k = tid; k < a.nkf; k += kBaThreads) S.kfact[k] = 0;
        if (tid == 0) S.istate[3] = 0;
        __syncthreads();
        for (int i = tid; i < a.nedge; i += kBaThreads) {
            unsigned char f = a.eflag[i] & 3;
            if (!(f & 1)) { f |= 4; S.kfact[a.edges[i].kf] = 1; }  // active at level 0
            a.eflag[i] = f;
        }
        __syncthreads();
        int nlp = 0;
        for (int p = tid; p < a.npt; p += kBaThreads) nlp += point_active(p);
        if (nlp) atomicAdd(&S.istate[3], nlp);
        if (tid == 0) {
            int n = 0;
            for (int oi = 0; oi < a.nkf; oi++) {
                const int k = a.kf_order[oi];
                a.pose_idx[k] = -1;
                if (a.kfs[k].fixed || !S.kfact[k]) continue;
                if (n < kBaMaxPoses) a.pose_kf[n] = k;
                a.pose_idx[k] = n < kBaMaxPoses ? n : -1;
                n++;
            }
            S.istate[0] = n;
            if (n > kBaMaxPoses) S.istate[1] = 1;  // unsupported size
        }
        __syncthreads();
        np = min(S.istate[0], kBaMaxPoses);
        N = 6 * np;
        nl = S.istate[3];
    }

    __device__ bool point_active(int p) const {
        for (int i = a.pt_start[p]; i < a.pt_start[p + 1]; i++)
            if (a.eflag[i] & 4) return true;
        return false;
    }

    // computeActiveErrors on (T, X) + activeRobustChi2
    __device__ double errors(const double* T, const double* X) {
        double s = 0;
        for (int i = threadIdx.x; i < a.nedge; i += kBaThreads) {
            if (!(a.eflag[i] & 4)) continue;
            edge_error(a, i, T, X, a.err + 3 * i);
            double r0, r1;
            edge_robust(a, i, edge_chi2(a, i), &r0, &r1);
            s += r0;
        }
        return block_sum(s, S);
    }

    __device__ double robust_chi2() {
        double s = 0;
        for (int i = threadIdx.x; i < a.nedge; i += kBaThreads) {
            if (!(a.eflag[i] & 4)) continue;
            double r0, r1;
            edge_robust(a, i, edge_chi2(a, i), &r0, &r1);
            s += r0;
        }
        return block_sum(s, S);
    }

    // BlockSolver::buildSystem
    __device__ void build_system() {
        const int tid = threadIdx.x;
        for (int p = tid; p < a.npt; p += kBaThreads) {
            double H[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0}, b[3] = {0, 0, 0};
            for (int i = a.pt_start[p]; i < a.pt_start[p + 1]; i++) {
                if (!(a.eflag[i] & 4)) continue;
                double Jl[3][3], Jp[3][6], w, om[3];
                edge_jacobians(a, i, a.T, a.X, Jl, Jp);
                edge_weights(a, i, &w, om);
                for (int r = 0; r < 3; r++) {
                    b[r] += Jl[0][r] * om[0] + Jl[1][r] * om[1] + Jl[2][r] * om[2];
                    for (int c = 0; c < 3; c++) H[r * 3 + c] += Jl[0][r] * w * Jl[0][c] + Jl[1][r] * w * Jl[1][c] + Jl[2][r] * w * Jl[2][c];
                }
                if (a.pose_idx[a.edges[i].kf] >= 0) {
                    double* B = a.Hpl + 18 * (long long)i;
                    for (int r = 0; r < 6; r++)
                        for (int c = 0; c < 3; c++) B[r * 3 + c] = Jp[0][r] * w * Jl[0][c] + Jp[1][r] * w * Jl[1][c] + Jp[2][r] * w * Jl[2][c];
                }
            }
            for (int k = 0; k < 9; k++) a.Hll[9 * p + k] = H[k];
            for (int k = 0; k < 3; k++) a.bl[3 * p + k] = b[k];
        }
        // poses: one wave each, lanes stride over the pose's observations
        const int wid = tid >> 6, lane = tid & 63;
        for (int pi = wid; pi < np; pi += kBaThreads / 64) {
            const int k = a.pose_kf[pi];
            double H[21], b[6];
            for (int q = 0; q < 21; q++) H[q] = 0;
            for (int q = 0; q < 6; q++) b[q] = 0;
            for (int j = a.kf_start[k] + lane; j < a.kf_start[k + 1]; j += 64) {
                const int i = a.kf_edges[j];
                if (!(a.eflag[i] & 4)) continue;
                double Jl[3][3], Jp[3][6], w, om[3];
                edge_jacobians(a, i, a.T, a.X, Jl, Jp);
                edge_weights(a, i, &w, om);
                int q = 0;
                for (int r = 0; r < 6; r++) {
                    b[r] += Jp[0][r] * om[0] + Jp[1][r] * om[1] + Jp[2][r] * om[2];
                    for (int c = r; c < 6; c++, q++) H[q] += Jp[0][r] * w * Jp[0][c] + Jp[1][r] * w * Jp[1][c] + Jp[2][r] * w * Jp[2][c];
                }
            }
            for (int q = 0; q < 21; q++)
                for (int o = 32; o > 0; o >>= 1) H[q] += __shfl_xor(H[q], o, 64);
            for (int q = 0; q < 6; q++)
                for (int o = 32; o > 0; o >>= 1) b[q] += __shfl_xor(b[q], o, 64);
            if (lane == 0) {
                int q = 0;
                for (int r = 0; r < 6; r++)
                    for (int c = r; c < 6; c++, q++) { a.Hpp[36 * pi + r * 6 + c] = H[q]; a.Hpp[36 * pi + c * 6 + r] = H[q]; }
                for (int r = 0; r < 6; r++) a.bp[6 * pi + r] = b[r];
            }
        }
        __syncthreads();
    }

    __device__ double lambda_init() {
        double m = 0;
        for (int q = threadIdx.x; q < np * 6; q += kBaThreads) m = fmax(m, fabs(a.Hpp[36 * (q / 6) + (q % 6) * 7]));
        for (int p = threadIdx.x; p < a.npt; p += kBaThreads)
            if (point_active(p))
                for (int j = 0; j < 3; j++) m = fmax(m, fabs(a.Hll[9 * p + 4 * j]));
        return 1e-5 * block_max(m, S);
    }

    // BlockSolver::setLambda + solve (Schur complement, reduced system, back substitution)
    __device__ bool solve(double lam) {
        const int tid = threadIdx.x;
        const int NP = N * (N + 1) / 2;
        for (int q = tid; q < NP; q += kBaThreads) S.H[q] = 0;
        __syncthreads();
        for (int q = tid; q < np * 36; q += kBaThreads) {
            const int pi = q / 36, r = (q % 36) / 6, c = q % 6;
            if (c < r) continue;
            S.H[packed(6 * pi + r, 6 * pi + c, N)] = a.Hpp[q] + (r == c ? lam : 0.0);
        }
        for (int q = tid; q < N; q += kBaThreads) S.bs[q] = a.bp[q];
        __syncthreads();
        for (int p = tid; p < a.npt; p += kBaThreads) {
            if (!point_active(p)) continue;
            double D[3][3];
            for (int r = 0; r < 3; r++)
                for (int c = 0; c < 3; c++) D[r][c] = a.Hll[9 * p + 3 * r + c] + (r == c ? lam : 0.0);
            const double c00 = D[1][1] * D[2][2] - D[1][2] * D[2][1];
            const double c10 = D[1][2] * D[2][0] - D[1][0] * D[2][2];
            const double c20 = D[1][0] * D[2][1] - D[1][1] * D[2][0];
            const double det = D[0][0] * c00 + D[0][1] * c10 + D[0][2] * c20;
            double Di[9];
            Di[0] = c00 / det; Di[3] = c10 / det; Di[6] = c20 / det;
            Di[1] = (D[0][2] * D[2][1] - D[0][1] * D[2][2]) / det;
            Di[4] = (D[0][0] * D[2][2] - D[0][2] * D[2][0]) / det;
            Di[7] = (D[0][1] * D[2][0] - D[0][0] * D[2][1]) / det;
            Di[2] = (D[0][1] * D[1][2] - D[0][2] * D[1][1]) / det;
            Di[5] = (D[0][2] * D[1][0] - D[0][0] * D[1][2]) / det;
            Di[8] = (D[0][0] * D[1][1] - D[0][1] * D[1][0]) / det;
            for (int k = 0; k < 9; k++) a.Dinv[9 * p + k] = Di[k];
            const double* blp = a.bl + 3 * p;
            double db[3];
            for (int r = 0; r < 3; r++) db[r] = Di[r * 3] * blp[0] + Di[r * 3 + 1] * blp[1] + Di[r * 3 + 2] * blp[2];
            for (int e1 = a.pt_start[p]; e1 < a.pt_start[p + 1]; e1++) {
                if (!(a.eflag[e1] & 4)) continue;
                const int i1 = a.pose_idx[a.edges[e1].kf];
                if (i1 < 0) continue;
                const double* B1 = a.Hpl + 18 * (long long)e1;
                double BD[6][3];
                for (int r = 0; r < 6; r++) {
                    for (int c = 0; c < 3; c++) BD[r][c] = B1[r * 3] * Di[c] + B1[r * 3 + 1] * Di[3 + c] + B1[r * 3 + 2] * Di[6 + c];
                    atomicAdd(&S.bs[6 * i1 + r], -(B1[r * 3] * db[0] + B1[r * 3 + 1] * db[1] + B1[r * 3 + 2] * db[2]));
                }
                for (int e2 = a.pt_start[p]; e2 < a.pt_start[p + 1]; e2++) {
                    if (!(a.eflag[e2] & 4)) continue;
                    const int i2 = a.pose_idx[a.edges[e2].kf];
                    if (i2 < i1) continue;
                    const double* B2 = a.Hpl + 18 * (long long)e2;
                    for (int r = 0; r < 6; r++)
                        for (int c = (i1 == i2 ? r : 0); c < 6; c++)
                            atomicAdd(&S.H[packed(6 * i1 + r, 6 * i2 + c, N)],
                                      -(BD[r][0] * B2[c * 3] + BD[r][1] * B2[c * 3 + 1] + BD[r][2] * B2[c * 3 + 2]));
                }
            }
        }
        __syncthreads();
        // LDL^T = U^T D U on the packed upper triangle (right-looking)
        bool ok = true;
        for (int j = 0; j < N; j++) {
            const double d = S.H[packed(j, j, N)];
            if (!(fabs(d) > 0) || !isfinite(d)) { ok = false; break; }
            // trailing update: wave per row, lanes across the row's upper part
            for (int rr = j + 1 + (tid >> 6); rr < N; rr += kBaThreads / 64) {
                const double ujr = S.H[packed(j, rr, N)];
                for (int cc = rr + (tid & 63); cc < N; cc += 64)
                    S.H[packed(rr, cc, N)] -= ujr * S.H[packed(j, cc, N)] / d;
            }
            __syncthreads();
            for (int c = j + 1 + tid; c < N; c += kBaThreads) S.H[packed(j, c, N)] /= d;
            __syncthreads();
        }
        if (!ok) return false;
        // U^T z = b ; y = z / D ; U x = y
        for (int k = 0; k < N; k++) {
            const double zk = S.bs[k];
            for (int jj = k + 1 + tid; jj < N; jj += kBaThreads) S.bs[jj] -= S.H[packed(k, jj, N)] * zk;
            __syncthreads();
        }
        for (int k = tid; k < N; k += kBaThreads) S.bs[k] /= S.H[packed(k, k, N)];
        __syncthreads();
        for (int k = N - 1; k >= 0; k--) {
            const double xk = S.bs[k];
            for (int jj = tid; jj < k; jj += kBaThreads) S.bs[jj] -= S.H[packed(jj, k, N)] * xk;
            __syncthreads();
        }
        for (int k = tid; k < N; k += kBaThreads) a.xp[k] = S.bs[k];
        __syncthreads();
        // landmarks: x_l = D^-1 (b_l - Hpl^T x_p)
        for (int p = tid; p < a.npt; p += kBaThreads) {
            double cl[3] = {a.bl[3 * p], a.bl[3 * p + 1], a.bl[3 * p + 2]};
            const bool act = point_active(p);
            if (act) {
                for (int e1 = a.pt_start[p]; e1 < a.pt_start[p + 1]; e1++) {
                    if (!(a.eflag[e1] & 4)) continue;
                    const int i1 = a.pose_idx[a.edges[e1].kf];
                    if (i1 < 0) continue;
                    const double* B = a.Hpl + 18 * (long long)e1;
                    for (int c = 0; c < 3; c++)
                        for (int r = 0; r < 6; r++) cl[c] -= B[r * 3 + c] * a.xp[6 * i1 + r];
                }
            }
            const double* Di = a.Dinv + 9 * p;
            for (int r = 0; r < 3; r++)
                a.xl[3 * p + r] = act ? Di[r * 3] * cl[0] + Di[r * 3 + 1] * cl[1] + Di[r * 3 + 2] * cl[2] : 0.0;
        }
        __syncthreads();
        return true;
    }

    // SparseOptimizer::update into the trial buffers; returns computeScale()
    __device__ double update(double lam) {
        const int tid = threadIdx.x;
        double s = 0;
        for (int p = tid; p < a.npt; p += kBaThreads) {
            for (int r = 0; r < 3; r++) {
                const double x = a.xl[3 * p + r];
                a.Xt[4 * p + r] = a.X[4 * p + r] + x;
                s += x * (lam * x + a.bl[3 * p + r]);
            }
        }
        for (int k = tid; k < a.nkf; k += kBaThreads) {
            const int pi = a.pose_idx[k];
            if (pi >= 0) se3_oplus(a.xp + 6 * pi, a.T + 8 * k, a.Tt + 8 * k);
            else for (int q = 0; q < 8; q++) a.Tt[8 * k + q] = a.T[8 * k + q];
        }
        for (int q = tid; q < N; q += kBaThreads) s += a.xp[q] * (lam * a.xp[q] + a.bp[q]);
        return block_sum(s, S);
    }

    __device__ void accept() {
        for (int p = threadIdx.x; p < a.npt; p += kBaThreads)
            for (int r = 0; r < 3; r++) a.X[4 * p + r] = a.Xt[4 * p + r];
        for (int q = threadIdx.x; q < 8 * a.nkf; q += kBaThreads) a.T[q] = a.Tt[q];
        __syncthreads();
    }

    // OptimizationAlgorithmLevenberg::solve ; returns 0 = OK, 1 = Terminate
    __device__ int lm_iteration(int iteration) {
        double currentChi = errors(a.T, a.X);
        const double iniChi = currentChi;
        build_system();
        if (iteration == 0) {
            const double l0 = lambda_init();
            if (threadIdx.x == 0) { S.dstate[0] = l0; S.dstate[1] = 2; S.istate[2] = 0; }
            __syncthreads();
        }
        double rho = 0;
        int qmax = 0;
        do {
            const double lam = S.dstate[0];
            const bool ok2 = solve(lam);
            double scale;
            if (ok2) scale = update(lam);
            else {
                for (int q = threadIdx.x; q < 8 * a.nkf; q += kBaThreads) a.Tt[q] = a.T[q];
                for (int q = threadIdx.x; q < 4 * a.npt; q += kBaThreads) a.Xt[q] = a.X[q];
                __syncthreads();
                scale = 0;
            }
            double tempChi = errors(a.Tt, a.Xt);
            if (!ok2) tempChi = DBL_MAX;
            rho = (currentChi - tempChi) / (scale + 1e-3);
            const bool good = rho > 0 && isfinite(tempChi);
            if (good) {
                double alpha = 1. - pow((2 * rho - 1), 3);
                alpha = fmin(alpha, 2. / 3.);
                const double sf = fmax(1. / 3., alpha);
                currentChi = tempChi;
                __syncthreads();
                if (threadIdx.x == 0) { S.dstate[0] = lam * sf; S.dstate[1] = 2; }
                accept();
            } else {
                __syncthreads();
                if (threadIdx.x == 0) { S.dstate[0] = lam * S.dstate[1]; S.dstate[1] *= 2; }
                __syncthreads();
            }
            qmax++;
        } while (rho < 0 && qmax < 10 && !stop_requested(a));
        if (qmax == 10 || rho == 0) return 1;
        int nBad = S.istate[2];
        if ((iniChi - currentChi) * 1e3 < iniChi) nBad++;
        else nBad = 0;
        __syncthreads();
        if (threadIdx.x == 0) S.istate[2] = nBad;
        __syncthreads();
        return nBad >= 3 ? 1 : 0;
    }

    __device__ int optimize(int iterations) {
        if (np + nl == 0) return -1;  // SparseOptimizer::optimize with an empty index mapping
        int it = 0;
        for (int i = 0; i < iterations && !stop_requested(a); i++) {
            const int r = lm_iteration(i);
            ++it;
            if (r != 0) break;
        }
        return it;
    }
};

__global__ __launch_bounds__(kBaThreads) void k_local_ba(BaArgs a) {
    __shared__ BaShared S;
    const int tid = threadIdx.x;
    if (tid < 16) S.istate[tid] = 0;
    // vertices: SE3Quat from float Tcw (Converter::toSE3Quat), points to double
    for (int k = tid; k < a.nkf; k += kBaThreads) {
        const float* t = a.kfs[k].tcw;
        double R[3][3];
        for (int r = 0; r < 3; r++)
            for (int c = 0; c < 3; c++) R[r][c] = t[4 * r + c];
        Q q = q_from_matrix(R);
        q_normalize(q);
        double* T = a.T + 8 * k;
        T[0] = q.x; T[1] = q.y; T[2] = q.z; T[3] = q.w; T[4] = t[3]; T[5] = t[7]; T[6] = t[11]; T[7] = 0;
    }
    for (int p = tid; p < a.npt; p += kBaThreads) {
        for (int r = 0; r < 3; r++) a.X[4 * p + r] = a.pts[p].pos[r];
        a.X[4 * p + 3] = 0;
    }
    for (int i = tid; i < a.nedge; i += kBaThreads) {
        a.eflag[i] = 0;
        a.out_erase[i] = 0;
        a.err[3 * i] = a.err[3 * i + 1] = a.err[3 * i + 2] = 0;
    }
    __syncthreads();
    Lba L(a, S);
    L.initialize();
    if (S.istate[1]) { if (tid == 0) a.out_stats[3] = ORBMI_E_UNSUPPORTED; return; }
    int it0 = L.optimize(5);
    const double chi0 = L.robust_chi2();
    const bool more = !stop_requested(a);
    int it1 = 0;
    double chi1 = 0;
    if (more) {
        // outlier levels, kernels off (src/Optimizer.cc:701-732), stale errors
        for (int i = tid; i < a.nedge; i += kBaThreads) {
            const orbmi_ba_edge e = a.edges[i];
            if (a.pts[e.point].bad) continue;
            double p[3];
            se3_map(a.T + 8 * e.kf, a.X + 4 * e.point, p);
            const double th = edge_stereo(e) ? 7.815 : 5.991;
            unsigned char f = a.eflag[i] & 3;
            if (edge_chi2(a, i) > th || !(p[2] > 0.0)) f |= 1;
            f |= 2;
            a.eflag[i] = f;
        }
        __syncthreads();
        L.initialize();
        if (S.istate[1]) { if (tid == 0) a.out_stats[3] = ORBMI_E_UNSUPPORTED; return; }
        it1 = L.optimize(10);
        chi1 = L.robust_chi2();
    }
    // vToErase (src/Optimizer.cc:741-773)
    for (int i = tid; i < a.nedge; i += kBaThreads) {
        const orbmi_ba_edge e = a.edges[i];
        if (a.pts[e.point].bad) continue;
        double p[3];
        se3_map(a.T + 8 * e.kf, a.X + 4 * e.point, p);
        const double th = edge_stereo(e) ? 7.815 : 5.991;
        a.out_erase[i] = (edge_chi2(a, i) > th || !(p[2] > 0.0)) ? 1 : 0;
    }
    // write back (Converter::toCvMat)
    for (int k = tid; k < a.nkf; k += kBaThreads) {
        const double* T = a.T + 8 * k;
        double R[3][3];
        q_to_matrix(load_q(T), R);
        float* o = a.out_tcw + 16 * k;
        for (int r = 0; r < 3; r++) {
            for (int c = 0; c < 3; c++) o[4 * r + c] = (float)R[r][c];
            o[4 * r + 3] = (float)T[4 + r];
        }
        o[12] = 0; o[13] = 0; o[14] = 0; o[15] = 1;
    }
    for (int p = tid; p < a.npt; p += kBaThreads)
        for (int r = 0; r < 3; r++) a.out_pos[3 * p + r] = (float)a.X[4 * p + r];
    if (tid == 0) {
        a.out_stats[0] = it0;
        a.out_stats[1] = it1;
        a.out_chi2[0] = chi0;
        a.out_chi2[1] = chi1;
    }
}

// ---------------------------------------------------------------- host
struct BaHandle {
    int device = 0;
    hipStream_t stream = nullptr;
    uint8_t* d_buf = nullptr;
    size_t cap = 0;
    int* h_stop = nullptr;  // pinned, device-mapped
    int* d_stop = nullptr;
};

}  // namespace orbmi

struct orbmi_ba {
    orbmi::BaHandle h;
};

extern "C" {

int orbmi_ba_create(int device, orbmi_ba** out) {
    if (!out) return ORBMI_E_ARG;
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return ORBMI_E_HIP;
    orbmi_ba* b = new (std::nothrow) orbmi_ba();
    if (!b) return ORBMI_E_ARG;
    b->h.device = device;
    if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&b->h.stream, hipStreamNonBlocking) != hipSuccess ||
        hipHostMalloc((void**)&b->h.h_stop, sizeof(int), hipHostMallocMapped) != hipSuccess ||
        hipHostGetDevicePointer((void**)&b->h.d_stop, b->h.h_stop, 0) != hipSuccess) {
        delete b;
        return ORBMI_E_HIP;
    }
    *b->h.h_stop = 0;
    *out = b;
    return ORBMI_OK;
}

void orbmi_ba_destroy(orbmi_ba* b) {
    if (!b) return;
    (void)hipSetDevice(b->h.device);
    if (b->h.d_buf) (void)hipFree(b->h.d_buf);
    if (b->h.h_stop) (void)hipHostFree(b->h.h_stop);
    if (b->h.stream) (void)hipStreamDestroy(b->h.stream);
    delete b;
}

int orbmi_local_bundle_adjustment(orbmi_ba* b, const orbmi_ba_problem* P, orbmi_ba_result* R,
                                  const volatile int* stop) {
    using namespace orbmi;
    if (!b || !P || !R || P->nkf < 0 || P->npt < 0 || P->nedge < 0) return ORBMI_E_ARG;
    if ((P->nkf && (!P->kfs || !R->tcw)) || (P->npt && (!P->pts || !R->pos)) || (P->nedge && (!P->edges || !R->erase)))
        return ORBMI_E_ARG;
    BaHandle& h = b->h;
    ORBMI_HIP(hipSetDevice(h.device));
    R->aborted = 0;
    R->iterations[0] = R->iterations[1] = 0;
    R->chi2[0] = R->chi2[1] = 0;
    for (int i = 0; i < P->nedge; i++) R->erase[i] = 0;
    if (stop && *stop) {  // src/Optimizer.cc:685-687
        R->aborted = 1;
        return ORBMI_OK;
    }
    const int nkf = P->nkf, npt = P->npt, ne = P->nedge;
    if (nkf > kBaMaxKf) return ORBMI_E_UNSUPPORTED;
    // host-side graph indexing: edges grouped by point (the reference inserts them point by
    // point), CSR by keyframe, keyframes ordered by id (SparseOptimizer vertex order)
    for (int i = 0; i < ne; i++) {
        const orbmi_ba_edge& e = P->edges[i];
        if (e.point < 0 || e.point >= npt || e.kf < 0 || e.kf >= nkf) return ORBMI_E_ARG;
        if (i && e.point < P->edges[i - 1].point) return ORBMI_E_ARG;
    }
    std::vector<int> pt_start(npt + 1, 0), kf_start(nkf + 1, 0), kf_edges(std::max(ne, 1)), order(std::max(nkf, 1));
    for (int i = 0; i < ne; i++) { pt_start[P->edges[i].point + 1]++; kf_start[P->edges[i].kf + 1]++; }
    for (int p = 0; p < npt; p++) pt_start[p + 1] += pt_start[p];
    for (int k = 0; k < nkf; k++) kf_start[k + 1] += kf_start[k];
    {
        std::vector<int> fill(kf_start.begin(), kf_start.end() - 1);
        for (int i = 0; i < ne; i++) kf_edges[fill[P->edges[i].kf]++] = i;
    }
    for (int k = 0; k < nkf; k++) order[k] = k;
    std::stable_sort(order.begin(), order.begin() + nkf, [&](int x, int y) { return P->kfs[x].id < P->kfs[y].id; });
    // one device arena
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    size_t off = 0;
    auto take = [&](size_t bytes) { size_t o = off; off += al(bytes); return o; };
    const size_t o_kfs = take(sizeof(orbmi_ba_keyframe) * nkf), o_pts = take(sizeof(orbmi_ba_point) * npt),
                 o_edges = take(sizeof(orbmi_ba_edge) * ne), o_order = take(4 * nkf), o_pts_start = take(4 * (npt + 1)),
                 o_kfs_start = take(4 * (nkf + 1)), o_kf_edges = take(4 * std::max(ne, 1)), o_T = take(64 * nkf),
                 o_Tt = take(64 * nkf), o_X = take(32 * npt), o_Xt = take(32 * npt), o_err = take(24 * ne),
                 o_eflag = take(ne), o_pidx = take(4 * nkf), o_pkf = take(4 * kBaMaxPoses), o_Hpl = take(144 * (size_t)ne),
                 o_Hll = take(72 * npt), o_bl = take(24 * npt), o_Dinv = take(72 * npt), o_Hpp = take(288 * kBaMaxPoses),
                 o_bp = take(48 * kBaMaxPoses), o_xp = take(8 * kBaMaxN), o_xl = take(24 * npt),
                 o_otcw = take(64 * nkf), o_opos = take(12 * npt), o_oerase = take(std::max(ne, 1)), o_stats = take(16),
                 o_chi2 = take(16);
    if (off > h.cap) {
        if (h.d_buf) (void)hipFree(h.d_buf);
        h.d_buf = nullptr;
        h.cap = 0;
        ORBMI_HIP(hipMalloc((void**)&h.d_buf, off));
        h.cap = off;
    }
    uint8_t* B = h.d_buf;
    hipStream_t s = h.stream;
    ORBMI_HIP(hipMemcpyAsync(B + o_kfs, P->kfs, sizeof(orbmi_ba_keyframe) * nkf, hipMemcpyHostToDevice, s));
    ORBMI_HIP(hipMemcpyAsync(B + o_pts, P->pts, sizeof(orbmi_ba_point) * npt, hipMemcpyHostToDevice, s));
    ORBMI_HIP(hipMemcpyAsync(B + o_edges, P->edges, sizeof(orbmi_ba_edge) * ne, hipMemcpyHostToDevice, s));
    ORBMI_HIP(hipMemcpyAsync(B + o_order, order.data(), 4 * nkf, hipMemcpyHostToDevice, s));
    ORBMI_HIP(hipMemcpyAsync(B + o_pts_start, pt_start.data(), 4 * (npt + 1), hipMemcpyHostToDevice, s));
    ORBMI_HIP(hipMemcpyAsync(B + o_kfs_start, kf_start.data(), 4 * (nkf + 1), hipMemcpyHostToDevice, s));
    ORBMI_HIP(hipMemcpyAsync(B + o_kf_edges, kf_edges.data(), 4 * std::max(ne, 1), hipMemcpyHostToDevice, s));
    ORBMI_HIP(hipMemsetAsync(B + o_stats, 0, 16, s));
    BaArgs a;
    a.nkf = nkf; a.npt = npt; a.nedge = ne;
    a.kfs = (const orbmi_ba_keyframe*)(B + o_kfs);
    a.pts = (const orbmi_ba_point*)(B + o_pts);
    a.edges = (const orbmi_ba_edge*)(B + o_edges);
    a.kf_order = (const int*)(B + o_order);
    a.pt_start = (const int*)(B + o_pts_start);
    a.kf_start = (const int*)(B + o_kfs_start);
    a.kf_edges = (const int*)(B + o_kf_edges);
    *h.h_stop = 0;
    a.stop = stop ? (const volatile int*)h.d_stop : nullptr;
    a.T = (double*)(B + o_T); a.Tt = (double*)(B + o_Tt);
    a.X = (double*)(B + o_X); a.Xt = (double*)(B + o_Xt);
    a.err = (double*)(B + o_err); a.eflag = B + o_eflag;
    a.pose_idx = (int*)(B + o_pidx); a.pose_kf = (int*)(B + o_pkf);
    a.Hpl = (double*)(B + o_Hpl); a.Hll = (double*)(B + o_Hll); a.bl = (double*)(B + o_bl);
    a.Dinv = (double*)(B + o_Dinv); a.Hpp = (double*)(B + o_Hpp); a.bp = (double*)(B + o_bp);
    a.xp = (double*)(B + o_xp); a.xl = (double*)(B + o_xl);
    a.out_tcw = (float*)(B + o_otcw); a.out_pos = (float*)(B + o_opos); a.out_erase = B + o_oerase;
    a.out_stats = (int*)(B + o_stats); a.out_chi2 = (double*)(B + o_chi2);
    hipLaunchKernelGGL(k_local_ba, dim3(1), dim3(kBaThreads), 0, s, a);
    ORBMI_HIP(hipGetLastError());
    // mirror the caller's abort flag (mbAbortBA) into device-visible memory while it runs
    while (true) {
        const hipError_t q = hipStreamQuery(s);
        if (q == hipSuccess) break;
        if (q != hipErrorNotReady) ORBMI_HIP(q);
        if (stop && *stop) __atomic_store_n(h.h_stop, 1, __ATOMIC_RELAXED);
    }
    int stats[4];
    ORBMI_HIP(hipMemcpy(stats, a.out_stats, 16, hipMemcpyDeviceToHost));
    if (stats[3]) return stats[3];
    ORBMI_HIP(hipMemcpy(R->chi2, a.out_chi2, 16, hipMemcpyDeviceToHost));
    if (nkf) ORBMI_HIP(hipMemcpy(R->tcw, a.out_tcw, 64 * nkf, hipMemcpyDeviceToHost));
    if (npt) ORBMI_HIP(hipMemcpy(R->pos, a.out_pos, 12 * npt, hipMemcpyDeviceToHost));
    if (ne) ORBMI_HIP(hipMemcpy(R->erase, a.out_erase, ne, hipMemcpyDeviceToHost));
    R->iterations[0] = stats[0];
    R->iterations[1] = stats[1];
    return ORBMI_OK;
}

}  // extern "C"
