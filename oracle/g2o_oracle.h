// ORACLE — test infrastructure only (see orb_oracle.h).
// g2o SE3Quat / Eigen quaternion helpers and a dense LDL^T shared by the LocalBundleAdjustment
// and PoseOptimization restatements (g2o types/se3quat.h, Eigen Quaternion / LDLT).
#pragma once
#include <cmath>
#include <cstring>
#include <vector>

namespace g2o_oracle {

struct Quat { double x, y, z, w; };
struct SE3 { Quat r; double t[3]; };

inline void normalize_rotation(Quat& q) {  // SE3Quat::normalizeRotation
    if (q.w < 0) { q.x = -q.x; q.y = -q.y; q.z = -q.z; q.w = -q.w; }
    const double n = std::sqrt(q.x * q.x + q.y * q.y + q.z * q.z + q.w * q.w);
    q.x /= n; q.y /= n; q.z /= n; q.w /= n;
}

inline Quat quat_from_matrix(const double m[3][3]) {  // Eigen::Quaternion(const Matrix3&)
    Quat q;
    const double tr = m[0][0] + m[1][1] + m[2][2];
    if (tr > 0) {
        double t = std::sqrt(tr + 1.0);
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
        double t = std::sqrt(m[i][i] - m[j][j] - m[k][k] + 1.0);
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

inline void quat_to_matrix(const Quat& q, double R[3][3]) {  // Eigen toRotationMatrix
    const double tx = 2 * q.x, ty = 2 * q.y, tz = 2 * q.z;
    const double twx = tx * q.w, twy = ty * q.w, twz = tz * q.w;
    const double txx = tx * q.x, txy = ty * q.x, txz = tz * q.x;
    const double tyy = ty * q.y, tyz = tz * q.y, tzz = tz * q.z;
    R[0][0] = 1 - (tyy + tzz); R[0][1] = txy - twz; R[0][2] = txz + twy;
    R[1][0] = txy + twz; R[1][1] = 1 - (txx + tzz); R[1][2] = tyz - twx;
    R[2][0] = txz - twy; R[2][1] = tyz + twx; R[2][2] = 1 - (txx + tyy);
}

inline Quat quat_mul(const Quat& a, const Quat& b) {
    return Quat{a.w * b.x + a.x * b.w + a.y * b.z - a.z * b.y, a.w * b.y + a.y * b.w + a.z * b.x - a.x * b.z,
                a.w * b.z + a.z * b.w + a.x * b.y - a.y * b.x, a.w * b.w - a.x * b.x - a.y * b.y - a.z * b.z};
}

inline void quat_rotate(const Quat& q, const double v[3], double o[3]) {  // Eigen _transformVector
    double uv[3] = {q.y * v[2] - q.z * v[1], q.z * v[0] - q.x * v[2], q.x * v[1] - q.y * v[0]};
    for (double& c : uv) c += c;
    const double cx = q.y * uv[2] - q.z * uv[1], cy = q.z * uv[0] - q.x * uv[2], cz = q.x * uv[1] - q.y * uv[0];
    o[0] = v[0] + q.w * uv[0] + cx;
    o[1] = v[1] + q.w * uv[1] + cy;
    o[2] = v[2] + q.w * uv[2] + cz;
}

inline void se3_map(const SE3& T, const double p[3], double o[3]) {
    quat_rotate(T.r, p, o);
    for (int i = 0; i < 3; i++) o[i] += T.t[i];
}

inline SE3 se3_from_tcw(const float* T) {  // Converter::toSE3Quat -> SE3Quat(R, t)
    double R[3][3];
    for (int r = 0; r < 3; r++)
        for (int c = 0; c < 3; c++) R[r][c] = T[4 * r + c];
    SE3 s;
    s.r = quat_from_matrix(R);
    s.t[0] = T[3]; s.t[1] = T[7]; s.t[2] = T[11];
    normalize_rotation(s.r);
    return s;
}

inline void se3_to_tcw(const SE3& s, float* T) {  // to_homogeneous_matrix -> float cv::Mat
    double R[3][3];
    quat_to_matrix(s.r, R);
    for (int r = 0; r < 3; r++) {
        for (int c = 0; c < 3; c++) T[4 * r + c] = (float)R[r][c];
        T[4 * r + 3] = (float)s.t[r];
    }
    T[12] = 0; T[13] = 0; T[14] = 0; T[15] = 1;
}

inline SE3 se3_exp(const double* u) {  // SE3Quat::exp
    const double w[3] = {u[0], u[1], u[2]}, up[3] = {u[3], u[4], u[5]};
    const double theta = std::sqrt(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]);
    const double O[3][3] = {{0, -w[2], w[1]}, {w[2], 0, -w[0]}, {-w[1], w[0], 0}};
    double O2[3][3];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) O2[i][j] = O[i][0] * O[0][j] + O[i][1] * O[1][j] + O[i][2] * O[2][j];
    double R[3][3], V[3][3];
    if (theta < 0.00001) {
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++) R[i][j] = (i == j) + O[i][j] + O2[i][j];
        memcpy(V, R, sizeof(R));
    } else {
        const double a = std::sin(theta) / theta, b = (1 - std::cos(theta)) / (theta * theta);
        const double c = (theta - std::sin(theta)) / std::pow(theta, 3);
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++) {
                R[i][j] = (i == j) + a * O[i][j] + b * O2[i][j];
                V[i][j] = (i == j) + b * O[i][j] + c * O2[i][j];
            }
    }
    SE3 s;
    s.r = quat_from_matrix(R);
    for (int i = 0; i < 3; i++) s.t[i] = V[i][0] * up[0] + V[i][1] * up[1] + V[i][2] * up[2];
    normalize_rotation(s.r);
    return s;
}

inline SE3 se3_mul(const SE3& a, const SE3& b) {  // SE3Quat::operator*
    SE3 r = a;
    double rt[3];
    quat_rotate(a.r, b.t, rt);
    for (int i = 0; i < 3; i++) r.t[i] += rt[i];
    r.r = quat_mul(a.r, b.r);
    normalize_rotation(r.r);
    return r;
}

// LDL^T of a dense symmetric positive definite matrix (n x n, row-major), solve in place.
inline bool ldlt_solve(std::vector<double>& A, int n, std::vector<double>& b) {
    for (int j = 0; j < n; j++) {
        double d = A[j * n + j];
        for (int k = 0; k < j; k++) d -= A[j * n + k] * A[j * n + k] * A[k * n + k];
        if (!(std::fabs(d) > 0) || !std::isfinite(d)) return false;
        A[j * n + j] = d;
        for (int i = j + 1; i < n; i++) {
            double s = A[i * n + j];
            for (int k = 0; k < j; k++) s -= A[i * n + k] * A[j * n + k] * A[k * n + k];
            A[i * n + j] = s / d;
        }
    }
    for (int i = 0; i < n; i++)
        for (int k = 0; k < i; k++) b[i] -= A[i * n + k] * b[k];
    for (int i = 0; i < n; i++) b[i] /= A[i * n + i];
    for (int i = n - 1; i >= 0; i--)
        for (int k = i + 1; k < n; k++) b[i] -= A[k * n + i] * b[k];
    return true;
}

}  // namespace g2o_oracle
