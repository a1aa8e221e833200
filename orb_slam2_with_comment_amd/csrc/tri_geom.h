// CreateNewMapPoints' per-match geometry (src/LocalMapping.cc:385-575), one source for the host
// (orbmi_triangulate_matches, mapping.cpp) and the device (k_triangulate, matcher.hip): the
// library builds with -ffp-contract=off, so both compile every expression below to the same
// correctly rounded float / double operations and make the same decisions bit for bit.
//
// Float semantics: cv::Mat CV_32F products and dot products accumulate in double and round to
// float (the build's convention for the reference's small float matrix algebra, as system.py's
// _mul); cv::SVD of the 4x4 linear-triangulation system is restated as the eigenvector of A^T A
// for its smallest eigenvalue (cyclic Jacobi in double), x3D = v[0:3] / v[3] in float -- the
// same null vector up to rounding, and the sign of v cancels in the division.
#pragma once
#include <cmath>

#include "../../include/orbmi.h"

#if defined(__HIP__) || defined(__HIPCC__)
#define ORBMI_HD __host__ __device__
#else
#define ORBMI_HD
#endif

namespace orbmi {
namespace tri {

constexpr int kLevels = 16;

// C = A(ra x ca) * B(ca x cb), float in/out, double accumulation, row-major
ORBMI_HD inline void matmul(const float* A, const float* B, float* C, int ra, int ca, int cb) {
    for (int r = 0; r < ra; r++)
        for (int c = 0; c < cb; c++) {
            double s = 0;
            for (int k = 0; k < ca; k++) s += (double)A[r * ca + k] * (double)B[k * cb + c];
            C[r * cb + c] = (float)s;
        }
}

ORBMI_HD inline void transpose3(const float* A, float* T) {
    for (int r = 0; r < 3; r++)
        for (int c = 0; c < 3; c++) T[3 * c + r] = A[3 * r + c];
}

ORBMI_HD inline void rot(const float* tcw, float* R) {
    for (int r = 0; r < 3; r++)
        for (int c = 0; c < 3; c++) R[3 * r + c] = tcw[4 * r + c];
}

ORBMI_HD inline double dot3(const float* a, const float* b) {
    return (double)a[0] * b[0] + (double)a[1] * b[1] + (double)a[2] * b[2];
}

// KeyFrame::GetCameraCenter: Ow = -Rcw^T tcw
ORBMI_HD inline void center(const float* tcw, float* ow) {
    float R[9], Rt[9], t[3] = {tcw[3], tcw[7], tcw[11]}, o[3];
    rot(tcw, R);
    transpose3(R, Rt);
    matmul(Rt, t, o, 3, 3, 1);
    for (int r = 0; r < 3; r++) ow[r] = -o[r];
}

// null vector of the 4x4 float system A (smallest eigenvalue of A^T A, cyclic Jacobi, double)
ORBMI_HD inline void null_vector4(const float* A, double v[4]) {
    double M[4][4], V[4][4];
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++) {
            double s = 0;
            for (int k = 0; k < 4; k++) s += (double)A[4 * k + i] * (double)A[4 * k + j];
            M[i][j] = s;
            V[i][j] = i == j ? 1.0 : 0.0;
        }
    double diag2 = 0;
    for (int p = 0; p < 4; p++) diag2 += M[p][p] * M[p][p];
    for (int sweep = 0; sweep < 30; sweep++) {
        double off = 0;
#pragma unroll
        for (int p = 0; p < 4; p++)
#pragma unroll
            for (int q = p + 1; q < 4; q++) off += M[p][q] * M[p][q];
        // converged to working precision: the off-diagonal mass is below (1e-17)^2 of the
        // diagonal's, so further rotations only move rounding (sweeping on to an exact zero
        // took ~4x the rotations)
        if (off <= 1e-34 * diag2) break;
        // p, q, k unrolled: every index static, so the matrices stay in registers on the device
        // (a rolled loop put them in scratch memory); the same operations in the same order
#pragma unroll
        for (int p = 0; p < 4; p++)
#pragma unroll
            for (int q = p + 1; q < 4; q++) {
                if (M[p][q] == 0) continue;
                const double theta = (M[q][q] - M[p][p]) / (2 * M[p][q]);
                const double t = (theta >= 0 ? 1.0 : -1.0) / (std::fabs(theta) + std::sqrt(theta * theta + 1));
                const double c = 1 / std::sqrt(t * t + 1), s = t * c;
#pragma unroll
                for (int k = 0; k < 4; k++) {  // M <- J^T M J
                    const double mkp = M[k][p], mkq = M[k][q];
                    M[k][p] = c * mkp - s * mkq;
                    M[k][q] = s * mkp + c * mkq;
                }
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    const double mpk = M[p][k], mqk = M[q][k];
                    M[p][k] = c * mpk - s * mqk;
                    M[q][k] = s * mpk + c * mqk;
                }
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    const double vkp = V[k][p], vkq = V[k][q];
                    V[k][p] = c * vkp - s * vkq;
                    V[k][q] = s * vkp + c * vkq;
                }
            }
    }
    int m = 0;
    double mm = M[0][0];
#pragma unroll
    for (int i = 1; i < 4; i++)
        if (M[i][i] < mm) { m = i; mm = M[i][i]; }
#pragma unroll
    for (int k = 0; k < 4; k++) {
        double x = V[k][0];
#pragma unroll
        for (int i = 1; i < 4; i++)
            if (m == i) x = V[k][i];
        v[k] = x;
    }
}

// One keyframe of a triangulation pair: pose (rows 0-2 of Tcw) and what derives from it, the
// intrinsics and the level tables by value; the keypoint arrays by pointer (host or device,
// whichever side runs)
struct Side {
    float tcw[12];
    float Rcw[9], Rwc[9], Ow[3], t[3];
    float fx, fy, cx, cy, bf, mb, invfx, invfy;
    float sigma2[kLevels], scale[kLevels];
    const orbmi_keypoint* keys;
    const float* ur;
    const float* depth;
    const float* cos_stereo;  // cos(2 atan2(mb / 2, depth)) per keypoint (device side only)
};

// host: the Side of an orbmi_tri_keyframe with nlev level entries (at most kLevels)
inline void make_side(const orbmi_tri_keyframe& K, int nlev, Side* S) {
    for (int k = 0; k < 12; k++) S->tcw[k] = K.tcw[k];
    rot(K.tcw, S->Rcw);
    transpose3(S->Rcw, S->Rwc);
    center(K.tcw, S->Ow);
    S->t[0] = K.tcw[3]; S->t[1] = K.tcw[7]; S->t[2] = K.tcw[11];
    S->fx = K.fx; S->fy = K.fy; S->cx = K.cx; S->cy = K.cy; S->bf = K.bf; S->mb = K.mb;
    S->invfx = 1.f / K.fx;
    S->invfy = 1.f / K.fy;
    for (int l = 0; l < kLevels; l++) {
        S->sigma2[l] = l < nlev ? K.level_sigma2[l] : 0.f;
        S->scale[l] = l < nlev ? K.scale_factors[l] : 0.f;
    }
    S->keys = K.keys_un;
    S->ur = K.u_right;
    S->depth = K.depth;
    S->cos_stereo = nullptr;
}

// CreateNewMapPoints' stereo parallax of one keypoint (:409-412), as float
inline float stereo_parallax_cos(float mb, float depth) { return std::cos(2 * std::atan2(mb / 2, depth)); }

// Frame / KeyFrame::UnprojectStereo (src/KeyFrame.cc, Frame.cc:701-715): `Rwc*x3Dc + Ow` is one
// cv::gemm(Rwc, x3Dc, 1, Ow, 1) MatExpr, so Ow is added before the single rounding to float
ORBMI_HD inline void unproject(const Side& K, int i, float* x3d) {
    const float z = K.depth[i];
    const float xc[3] = {(K.keys[i].x - K.cx) * z * K.invfx, (K.keys[i].y - K.cy) * z * K.invfy, z};
    for (int r = 0; r < 3; r++) x3d[r] = (float)(dot3(K.Rwc + 3 * r, xc) + (double)K.Ow[r]);
}

// the tests of one match (i1 of K1, i2 of K2); cps1 / cps2 = stereo_parallax_cos of each side's
// keypoint (read only when that keypoint is stereo).  true with x = the new point's position.
ORBMI_HD inline bool triangulate_one(const Side& K1, const Side& K2, int i1, int i2, float cps1, float cps2,
                                     float x[3]) {
    const float ratioFactor = 1.5f * K1.scale[1];  // 1.5f * mfScaleFactor
    const orbmi_keypoint kp1 = K1.keys[i1], kp2 = K2.keys[i2];
    const float kp1_ur = K1.ur[i1], kp2_ur = K2.ur[i2];
    const bool bStereo1 = kp1_ur >= 0, bStereo2 = kp2_ur >= 0;
    // parallax between the rays (:401-423)
    const float xn1[3] = {(kp1.x - K1.cx) * K1.invfx, (kp1.y - K1.cy) * K1.invfy, 1.f};
    const float xn2[3] = {(kp2.x - K2.cx) * K2.invfx, (kp2.y - K2.cy) * K2.invfy, 1.f};
    float ray1[3], ray2[3];
    matmul(K1.Rwc, xn1, ray1, 3, 3, 1);
    matmul(K2.Rwc, xn2, ray2, 3, 3, 1);
    const float cosParallaxRays =
        (float)(dot3(ray1, ray2) / (std::sqrt(dot3(ray1, ray1)) * std::sqrt(dot3(ray2, ray2))));
    float cosParallaxStereo = cosParallaxRays + 1;
    float cosParallaxStereo1 = cosParallaxStereo, cosParallaxStereo2 = cosParallaxStereo;
    if (bStereo1) cosParallaxStereo1 = cps1;
    else if (bStereo2) cosParallaxStereo2 = cps2;
    cosParallaxStereo = std::fmin(cosParallaxStereo1, cosParallaxStereo2);
    if (cosParallaxRays < cosParallaxStereo && cosParallaxRays > 0 &&
        (bStereo1 || bStereo2 || cosParallaxRays < 0.9998)) {
        // linear triangulation (:431-457)
        float A[16];
        for (int c = 0; c < 4; c++) {
            A[c] = xn1[0] * K1.tcw[8 + c] - K1.tcw[c];
            A[4 + c] = xn1[1] * K1.tcw[8 + c] - K1.tcw[4 + c];
            A[8 + c] = xn2[0] * K2.tcw[8 + c] - K2.tcw[c];
            A[12 + c] = xn2[1] * K2.tcw[8 + c] - K2.tcw[4 + c];
        }
        double v[4];
        null_vector4(A, v);
        const float v3 = (float)v[3];
        if (v3 == 0) return false;
        for (int r = 0; r < 3; r++) x[r] = (float)v[r] / v3;
    } else if (bStereo1 && cosParallaxStereo1 < cosParallaxStereo2) {
        unproject(K1, i1, x);
    } else if (bStereo2 && cosParallaxStereo2 < cosParallaxStereo1) {
        unproject(K2, i2, x);
    } else {
        return false;  // no stereo and very low parallax
    }
    // in front of both cameras (:474-482); cv::Mat::dot returns double, so `dot + tcw` is a
    // double sum rounded to float once
    const float z1 = (float)(dot3(K1.Rcw + 6, x) + (double)K1.t[2]);
    if (z1 <= 0) return false;
    const float z2 = (float)(dot3(K2.Rcw + 6, x) + (double)K2.t[2]);
    if (z2 <= 0) return false;
    // reprojection error in the first keyframe (:484-510)
    const float sigmaSquare1 = K1.sigma2[kp1.octave];
    const float x1 = (float)(dot3(K1.Rcw, x) + (double)K1.t[0]);
    const float y1 = (float)(dot3(K1.Rcw + 3, x) + (double)K1.t[1]);
    const float invz1 = (float)(1.0 / z1);
    if (!bStereo1) {
        const float u1 = K1.fx * x1 * invz1 + K1.cx, v1 = K1.fy * y1 * invz1 + K1.cy;
        const float ex = u1 - kp1.x, ey = v1 - kp1.y;
        if ((ex * ex + ey * ey) > 5.991 * sigmaSquare1) return false;
    } else {
        const float u1 = K1.fx * x1 * invz1 + K1.cx;
        const float u1_r = u1 - K1.bf * invz1;
        const float v1 = K1.fy * y1 * invz1 + K1.cy;
        const float ex = u1 - kp1.x, ey = v1 - kp1.y, er = u1_r - kp1_ur;
        if ((ex * ex + ey * ey + er * er) > 7.8 * sigmaSquare1) return false;
    }
    // ... and in the second (:512-537); the right coordinate uses the first keyframe's mbf
    const float sigmaSquare2 = K2.sigma2[kp2.octave];
    const float x2 = (float)(dot3(K2.Rcw, x) + (double)K2.t[0]);
    const float y2 = (float)(dot3(K2.Rcw + 3, x) + (double)K2.t[1]);
    const float invz2 = (float)(1.0 / z2);
    if (!bStereo2) {
        const float u2 = K2.fx * x2 * invz2 + K2.cx, v2 = K2.fy * y2 * invz2 + K2.cy;
        const float ex = u2 - kp2.x, ey = v2 - kp2.y;
        if ((ex * ex + ey * ey) > 5.991 * sigmaSquare2) return false;
    } else {
        const float u2 = K2.fx * x2 * invz2 + K2.cx;
        const float u2_r = u2 - K1.bf * invz2;
        const float v2 = K2.fy * y2 * invz2 + K2.cy;
        const float ex = u2 - kp2.x, ey = v2 - kp2.y, er = u2_r - kp2_ur;
        if ((ex * ex + ey * ey + er * er) > 7.8 * sigmaSquare2) return false;
    }
    // scale consistency (:539-557; the reference's text lost the `continue;` of upstream
    // ORB-SLAM2 and would not compile, DESIGN.md §8: the upstream rule is kept)
    const float n1[3] = {x[0] - K1.Ow[0], x[1] - K1.Ow[1], x[2] - K1.Ow[2]};
    const float n2[3] = {x[0] - K2.Ow[0], x[1] - K2.Ow[1], x[2] - K2.Ow[2]};
    const float dist1 = (float)std::sqrt(dot3(n1, n1)), dist2 = (float)std::sqrt(dot3(n2, n2));
    if (dist1 == 0 || dist2 == 0) return false;
    const float ratioDist = dist2 / dist1;
    const float ratioOctave = K1.scale[kp1.octave] / K2.scale[kp2.octave];
    if (ratioDist * ratioFactor < ratioOctave || ratioDist > ratioOctave * ratioFactor) return false;
    return true;
}

}  // namespace tri
}  // namespace orbmi
