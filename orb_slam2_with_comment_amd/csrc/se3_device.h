// fp64 SE3Quat helpers shared by the LocalBundleAdjustment and PoseOptimization kernels
// (g2o types/se3quat.h, Eigen Quaternion): storage of a pose = 8 doubles (qx, qy, qz, qw, tx, ty,
// tz, -), the layout of VertexSE3Expmap's estimate in the kernels.
#pragma once
#include <hip/hip_runtime.h>

namespace orbmi {

// ---------------------------------------------------------------- fp64 latency helpers
// 1/x and 1/sqrt(x) from v_rcp_f64 / v_rsq_f64 with Newton steps: within an ulp or two of the
// IEEE quotient / root at a third of their dependent latency (gfx950: div 76, sqrt 111, rcp 17
// cycles; tools/ubench/lat.hip).  Used where the parity tolerance is 1e-4 (poses, BA).
__device__ inline double fast_rcp(double x) {
    double y = __builtin_amdgcn_rcp(x);
    double e = fma(-x, y, 1.0);
    y = fma(y, e, y);
    e = fma(-x, y, 1.0);
    return fma(y, e, y);
}

__device__ inline double fast_rsqrt(double x) {
    double y = __builtin_amdgcn_rsq(x);
    const double hx = 0.5 * x;
    double e = fma(-hx * y, y, 0.5);
    y = fma(y, e, y);
    e = fma(-hx * y, y, 0.5);
    return fma(y, e, y);
}

// ---------------------------------------------------------------- SE3Quat helpers (fp64)
// The helpers below contract multiply-adds (fp contract fast): the optimisers that use them
// carry a 1e-4 parity tolerance.
struct Q { double x, y, z, w; };

__device__ inline void q_normalize(Q& q) {
#pragma clang fp contract(fast)
    if (q.w < 0) { q.x = -q.x; q.y = -q.y; q.z = -q.z; q.w = -q.w; }
    const double inv = fast_rsqrt(q.x * q.x + q.y * q.y + q.z * q.z + q.w * q.w);
    q.x *= inv; q.y *= inv; q.z *= inv; q.w *= inv;
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
#pragma clang fp contract(fast)
    const double tx = 2 * q.x, ty = 2 * q.y, tz = 2 * q.z;
    const double twx = tx * q.w, twy = ty * q.w, twz = tz * q.w;
    const double txx = tx * q.x, txy = ty * q.x, txz = tz * q.x;
    const double tyy = ty * q.y, tyz = tz * q.y, tzz = tz * q.z;
    R[0][0] = 1 - (tyy + tzz); R[0][1] = txy - twz; R[0][2] = txz + twy;
    R[1][0] = txy + twz; R[1][1] = 1 - (txx + tzz); R[1][2] = tyz - twx;
    R[2][0] = txz - twy; R[2][1] = tyz + twx; R[2][2] = 1 - (txx + tyy);
}

__device__ inline void q_rotate(const Q& q, const double v[3], double o[3]) {
#pragma clang fp contract(fast)
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

// sin and cos of a small angle (|x| <= 0.1): Taylor to x^11 / x^12, below 1e-22 truncation
__device__ inline void sincos_small(double x, double& s, double& c) {
    const double x2 = x * x;
    s = x * (1.0 + x2 * (-1.0 / 6 + x2 * (1.0 / 120 + x2 * (-1.0 / 5040 + x2 * (1.0 / 362880 + x2 * (-1.0 / 39916800))))));
    c = 1.0 + x2 * (-0.5 + x2 * (1.0 / 24 + x2 * (-1.0 / 720 + x2 * (1.0 / 40320 + x2 * (-1.0 / 3628800 + x2 * (1.0 / 479001600))))));
}

// T <- exp(u) * T   (VertexSE3Expmap::oplusImpl, SE3Quat::exp / operator*; se3quat.h:223-257).
// For theta >= 1e-5 the exponential is formed in quaternion form: Quaterniond(R) of
// R = I + sin(t)/t Omega + (1-cos t)/t^2 Omega^2 is (sin(t/2)/t * omega, cos(t/2)) exactly, and
// V * upsilon = upsilon + b omega x upsilon + c omega x (omega x upsilon) with
// b = (1-cos t)/t^2 = 2 sin^2(t/2)/t^2, c = (t - sin t)/t^3; equal to the matrix form up to
// rounding.  Below 1e-5 the reference's non-orthonormal R = I + Omega + Omega^2 (V = R) is kept.
__device__ inline void se3_oplus(const double* u, const double* Tin, double* Tout) {
#pragma clang fp contract(fast)
    const double w0 = u[0], w1 = u[1], w2 = u[2];
    const double n2 = w0 * w0 + w1 * w1 + w2 * w2;
    Q qe;
    double te[3];
    if (n2 < 1e-10) {  // theta < 0.00001
        // R = I + Omega + Omega^2 (Omega^2 = w w^T - |w|^2 I, symmetric: R_kj - R_jk = 2 w_i
        // exactly), trace 3 - 2 |w|^2 > 0: Eigen's Quaternion(R) takes its trace branch,
        // q = ((R_kj - R_jk) / (2 t), ..., t / 2) with t = sqrt(trace + 1)
        const double R00 = 1 - (w1 * w1 + w2 * w2), R11 = 1 - (w0 * w0 + w2 * w2), R22 = 1 - (w0 * w0 + w1 * w1);
        const double R01 = w0 * w1 - w2, R02 = w0 * w2 + w1, R10 = w0 * w1 + w2;
        const double R12 = w1 * w2 - w0, R20 = w0 * w2 - w1, R21 = w1 * w2 + w0;
        const double x = R00 + R11 + R22 + 1.0, r = fast_rsqrt(x), hs = 0.5 * r;
        qe = Q{(R21 - R12) * hs, (R02 - R20) * hs, (R10 - R01) * hs, 0.5 * (x * r)};
        te[0] = R00 * u[3] + R01 * u[4] + R02 * u[5];
        te[1] = R10 * u[3] + R11 * u[4] + R12 * u[5];
        te[2] = R20 * u[3] + R21 * u[4] + R22 * u[5];
    } else {
        const double it = fast_rsqrt(n2), theta = n2 * it, it2 = it * it;
        double sh, ch;  // sin, cos of theta / 2
        const double h = 0.5 * theta;
        if (h <= 0.1) sincos_small(h, sh, ch);
        else sincos(h, &sh, &ch);
        const double k = sh * it;
        qe = Q{k * w0, k * w1, k * w2, ch};
        const double st = 2 * sh * ch;                  // sin(theta)
        const double b = 2 * sh * sh * it2;             // (1 - cos theta) / theta^2
        const double c = (theta - st) * (it2 * it);     // (theta - sin theta) / theta^3
        const double v0 = u[3], v1 = u[4], v2 = u[5];
        const double a0 = w1 * v2 - w2 * v1, a1 = w2 * v0 - w0 * v2, a2 = w0 * v1 - w1 * v0;  // omega x v
        const double c0 = w1 * a2 - w2 * a1, c1 = w2 * a0 - w0 * a2, c2 = w0 * a1 - w1 * a0;  // omega x a
        te[0] = v0 + b * a0 + c * c0;
        te[1] = v1 + b * a1 + c * c1;
        te[2] = v2 + b * a2 + c * c2;
    }
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
