// fp64 SE3Quat helpers shared by the LocalBundleAdjustment and PoseOptimization kernels
// (g2o types/se3quat.h, Eigen Quaternion): storage of a pose = 8 doubles (qx, qy, qz, qw, tx, ty,
// tz, -), the layout of VertexSE3Expmap's estimate in the kernels.
#pragma once
#include <hip/hip_runtime.h>

namespace orbmi {

// ---------------------------------------------------------------- SE3Quat helpers (fp64)
struct Q { double x, y, z, w; };

__device__ inline void q_normalize(Q& q) {
    if (q.w < 0) { q.x = -q.x; q.y = -q.y; q.z = -q.z; q.w = -q.w; }
    const double n = sqrt(q.x * q.x + q.y * q.y + q.z * q.z + q.w * q.w);
    q.x /= n; q.y /= n; q.z /= n; q.w /= n;
}

// Eigen::Quaternion(const Matrix3&): the largest-diagonal branch spelled out per pivot so that
// every index is static (no scratch memory)
template <int I>
__device__ inline Q q_from_matrix_pivot(const double m[3][3]) {
    constexpr int J = (I + 1) % 3, K = (J + 1) % 3;
    double t = sqrt(m[I][I] - m[J][J] - m[K][K] + 1.0);
    double v[3];
    v[I] = 0.5 * t;
    t = 0.5 / t;
    Q q;
    q.w = (m[K][J] - m[J][K]) * t;
    v[J] = (m[J][I] + m[I][J]) * t;
    v[K] = (m[K][I] + m[I][K]) * t;
    q.x = v[0]; q.y = v[1]; q.z = v[2];
    return q;
}

__device__ inline Q q_from_matrix(const double m[3][3]) {
    const double tr = m[0][0] + m[1][1] + m[2][2];
    if (tr > 0) {
        Q q;
        double t = sqrt(tr + 1.0);
        q.w = 0.5 * t;
        t = 0.5 / t;
        q.x = (m[2][1] - m[1][2]) * t;
        q.y = (m[0][2] - m[2][0]) * t;
        q.z = (m[1][0] - m[0][1]) * t;
        return q;
    }
    int i = 0;
    if (m[1][1] > m[0][0]) i = 1;
    if (m[2][2] > (i == 0 ? m[0][0] : m[1][1])) i = 2;
    return i == 0 ? q_from_matrix_pivot<0>(m) : i == 1 ? q_from_matrix_pivot<1>(m) : q_from_matrix_pivot<2>(m);
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
        const double c = (theta - sin(theta)) / (theta * theta * theta);
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

}  // namespace orbmi
