// LocalMapping's host geometry around the GPU searches (src/LocalMapping.cc:290-577, :676-693):
// the fundamental matrix of a keyframe pair and the triangulation + acceptance tests of
// CreateNewMapPoints for the pairs SearchForTriangulation returned.  Host code (a few hundred
// matches per keyframe pair); both stereo SLAM host loops (system.py and the native slam.cpp)
// call these, so the two make the same decisions.
//
// Float semantics: cv::Mat CV_32F products and dot products accumulate in double and round to
// float (the build's convention for the reference's small float matrix algebra, as system.py's
// _mul); cv::SVD of the 4x4 linear-triangulation system is restated as the eigenvector of A^T A
// for its smallest eigenvalue (cyclic Jacobi in double), x3D = v[0:3] / v[3] in float -- the
// same null vector up to rounding, and the sign of v cancels in the division.
#include <cmath>
#include <cstring>

#include "../../include/orbmi.h"

namespace {

// C = A(ra x ca) * B(ca x cb), float in/out, double accumulation, row-major
void matmul(const float* A, const float* B, float* C, int ra, int ca, int cb) {
    for (int r = 0; r < ra; r++)
        for (int c = 0; c < cb; c++) {
            double s = 0;
            for (int k = 0; k < ca; k++) s += (double)A[r * ca + k] * (double)B[k * cb + c];
            C[r * cb + c] = (float)s;
        }
}

void transpose3(const float* A, float* T) {
    for (int r = 0; r < 3; r++)
        for (int c = 0; c < 3; c++) T[3 * c + r] = A[3 * r + c];
}

void rot(const float* tcw, float* R) {
    for (int r = 0; r < 3; r++)
        for (int c = 0; c < 3; c++) R[3 * r + c] = tcw[4 * r + c];
}

double dot3(const float* a, const float* b) { return (double)a[0] * b[0] + (double)a[1] * b[1] + (double)a[2] * b[2]; }

// KeyFrame::GetCameraCenter: Ow = -Rcw^T tcw
void center(const float* tcw, float* ow) {
    float R[9], Rt[9], t[3] = {tcw[3], tcw[7], tcw[11]}, o[3];
    rot(tcw, R);
    transpose3(R, Rt);
    matmul(Rt, t, o, 3, 3, 1);
    for (int r = 0; r < 3; r++) ow[r] = -o[r];
}

// null vector of the 4x4 float system A (smallest eigenvalue of A^T A, cyclic Jacobi, double)
void null_vector4(const float* A, double v[4]) {
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
        for (int p = 0; p < 4; p++)
            for (int q = p + 1; q < 4; q++) off += M[p][q] * M[p][q];
        // converged to working precision: the off-diagonal mass is below (1e-17)^2 of the
        // diagonal's, so further rotations only move rounding (sweeping on to an exact zero
        // took ~4x the rotations)
        if (off <= 1e-34 * diag2) break;
        for (int p = 0; p < 4; p++)
            for (int q = p + 1; q < 4; q++) {
                if (M[p][q] == 0) continue;
                const double theta = (M[q][q] - M[p][p]) / (2 * M[p][q]);
                const double t = (theta >= 0 ? 1.0 : -1.0) / (std::fabs(theta) + std::sqrt(theta * theta + 1));
                const double c = 1 / std::sqrt(t * t + 1), s = t * c;
                for (int k = 0; k < 4; k++) {  // M <- J^T M J
                    const double mkp = M[k][p], mkq = M[k][q];
                    M[k][p] = c * mkp - s * mkq;
                    M[k][q] = s * mkp + c * mkq;
                }
                for (int k = 0; k < 4; k++) {
                    const double mpk = M[p][k], mqk = M[q][k];
                    M[p][k] = c * mpk - s * mqk;
                    M[q][k] = s * mpk + c * mqk;
                }
                for (int k = 0; k < 4; k++) {
                    const double vkp = V[k][p], vkq = V[k][q];
                    V[k][p] = c * vkp - s * vkq;
                    V[k][q] = s * vkp + c * vkq;
                }
            }
    }
    int m = 0;
    for (int i = 1; i < 4; i++)
        if (M[i][i] < M[m][m]) m = i;
    for (int k = 0; k < 4; k++) v[k] = V[k][m];
}

// Frame / KeyFrame::UnprojectStereo (src/KeyFrame.cc, Frame.cc:701-715): `Rwc*x3Dc + Ow` is one
// cv::gemm(Rwc, x3Dc, 1, Ow, 1) MatExpr, so Ow is added before the single rounding to float
void unproject(const orbmi_tri_keyframe& K, int i, float* x3d) {
    const float z = K.depth[i];
    const float invfx = 1.f / K.fx, invfy = 1.f / K.fy;
    const float xc[3] = {(K.keys_un[i].x - K.cx) * z * invfx, (K.keys_un[i].y - K.cy) * z * invfy, z};
    float R[9], Rt[9], ow[3];
    rot(K.tcw, R);
    transpose3(R, Rt);
    center(K.tcw, ow);
    for (int r = 0; r < 3; r++) x3d[r] = (float)(dot3(Rt + 3 * r, xc) + (double)ow[r]);
}

}  // namespace

extern "C" {

int orbmi_compute_f12(const orbmi_tri_keyframe* kf1, const orbmi_tri_keyframe* kf2, float* F12) {
    if (!kf1 || !kf2 || !F12 || !kf1->tcw || !kf2->tcw) return ORBMI_E_ARG;
    float R1[9], R2[9], R2t[9], R12[9], t1[3] = {kf1->tcw[3], kf1->tcw[7], kf1->tcw[11]};
    float t2[3] = {kf2->tcw[3], kf2->tcw[7], kf2->tcw[11]};
    rot(kf1->tcw, R1);
    rot(kf2->tcw, R2);
    transpose3(R2, R2t);
    matmul(R1, R2t, R12, 3, 3, 3);                    // R12 = R1w R2w^T
    float m[3], t12[3];
    matmul(R12, t2, m, 3, 3, 1);                      // -R1w R2w^T t2w + t1w
    for (int r = 0; r < 3; r++) t12[r] = -m[r] + t1[r];
    const float tx[9] = {0, -t12[2], t12[1], t12[2], 0, -t12[0], -t12[1], t12[0], 0};  // SkewSymmetricMatrix
    // K^-1 of K = [fx 0 cx; 0 fy cy; 0 0 1]
    const float K1it[9] = {1.f / kf1->fx, 0, 0, 0, 1.f / kf1->fy, 0, -kf1->cx / kf1->fx, -kf1->cy / kf1->fy, 1};
    const float K2i[9] = {1.f / kf2->fx, 0, -kf2->cx / kf2->fx, 0, 1.f / kf2->fy, -kf2->cy / kf2->fy, 0, 0, 1};
    float a[9], b[9];
    matmul(K1it, tx, a, 3, 3, 3);                     // K1^-T t12x R12 K2^-1, left to right
    matmul(a, R12, b, 3, 3, 3);
    matmul(b, K2i, F12, 3, 3, 3);
    return ORBMI_OK;
}

int orbmi_triangulate_matches(const orbmi_tri_keyframe* kf1, const orbmi_tri_keyframe* kf2, const int32_t* idx1,
                              const int32_t* idx2, int n, float* x3d, uint8_t* ok) {
    if (!kf1 || !kf2 || n < 0 || (n > 0 && (!idx1 || !idx2 || !x3d || !ok))) return ORBMI_E_ARG;
    const orbmi_tri_keyframe &K1 = *kf1, &K2 = *kf2;
    float Rcw1[9], Rwc1[9], Rcw2[9], Rwc2[9], Ow1[3], Ow2[3];
    rot(K1.tcw, Rcw1);
    transpose3(Rcw1, Rwc1);
    rot(K2.tcw, Rcw2);
    transpose3(Rcw2, Rwc2);
    center(K1.tcw, Ow1);
    center(K2.tcw, Ow2);
    const float tcw1[3] = {K1.tcw[3], K1.tcw[7], K1.tcw[11]}, tcw2[3] = {K2.tcw[3], K2.tcw[7], K2.tcw[11]};
    const float invfx1 = 1.f / K1.fx, invfy1 = 1.f / K1.fy, invfx2 = 1.f / K2.fx, invfy2 = 1.f / K2.fy;
    const float ratioFactor = 1.5f * K1.scale_factors[1];  // 1.5f * mfScaleFactor
    for (int k = 0; k < n; k++) {
        ok[k] = 0;
        const int i1 = idx1[k], i2 = idx2[k];
        const orbmi_keypoint &kp1 = K1.keys_un[i1], &kp2 = K2.keys_un[i2];
        const float kp1_ur = K1.u_right[i1], kp2_ur = K2.u_right[i2];
        const bool bStereo1 = kp1_ur >= 0, bStereo2 = kp2_ur >= 0;
        // parallax between the rays (:401-423)
        const float xn1[3] = {(kp1.x - K1.cx) * invfx1, (kp1.y - K1.cy) * invfy1, 1.f};
        const float xn2[3] = {(kp2.x - K2.cx) * invfx2, (kp2.y - K2.cy) * invfy2, 1.f};
        float ray1[3], ray2[3];
        matmul(Rwc1, xn1, ray1, 3, 3, 1);
        matmul(Rwc2, xn2, ray2, 3, 3, 1);
        const float cosParallaxRays =
            (float)(dot3(ray1, ray2) / (std::sqrt(dot3(ray1, ray1)) * std::sqrt(dot3(ray2, ray2))));
        float cosParallaxStereo = cosParallaxRays + 1;
        float cosParallaxStereo1 = cosParallaxStereo, cosParallaxStereo2 = cosParallaxStereo;
        if (bStereo1) cosParallaxStereo1 = std::cos(2 * std::atan2(K1.mb / 2, K1.depth[i1]));
        else if (bStereo2) cosParallaxStereo2 = std::cos(2 * std::atan2(K2.mb / 2, K2.depth[i2]));
        cosParallaxStereo = std::fmin(cosParallaxStereo1, cosParallaxStereo2);
        float x[3];
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
            if (v3 == 0) continue;
            for (int r = 0; r < 3; r++) x[r] = (float)v[r] / v3;
        } else if (bStereo1 && cosParallaxStereo1 < cosParallaxStereo2) {
            unproject(K1, i1, x);
        } else if (bStereo2 && cosParallaxStereo2 < cosParallaxStereo1) {
            unproject(K2, i2, x);
        } else {
            continue;  // no stereo and very low parallax
        }
        // in front of both cameras (:474-482); cv::Mat::dot returns double, so `dot + tcw` is a
        // double sum rounded to float once
        const float z1 = (float)(dot3(Rcw1 + 6, x) + (double)tcw1[2]);
        if (z1 <= 0) continue;
        const float z2 = (float)(dot3(Rcw2 + 6, x) + (double)tcw2[2]);
        if (z2 <= 0) continue;
        // reprojection error in the first keyframe (:484-510)
        const float sigmaSquare1 = K1.level_sigma2[kp1.octave];
        const float x1 = (float)(dot3(Rcw1, x) + (double)tcw1[0]);
        const float y1 = (float)(dot3(Rcw1 + 3, x) + (double)tcw1[1]);
        const float invz1 = (float)(1.0 / z1);
        if (!bStereo1) {
            const float u1 = K1.fx * x1 * invz1 + K1.cx, v1 = K1.fy * y1 * invz1 + K1.cy;
            const float ex = u1 - kp1.x, ey = v1 - kp1.y;
            if ((ex * ex + ey * ey) > 5.991 * sigmaSquare1) continue;
        } else {
            const float u1 = K1.fx * x1 * invz1 + K1.cx;
            const float u1_r = u1 - K1.bf * invz1;
            const float v1 = K1.fy * y1 * invz1 + K1.cy;
            const float ex = u1 - kp1.x, ey = v1 - kp1.y, er = u1_r - kp1_ur;
            if ((ex * ex + ey * ey + er * er) > 7.8 * sigmaSquare1) continue;
        }
        // ... and in the second (:512-537); the right coordinate uses the first keyframe's mbf
        const float sigmaSquare2 = K2.level_sigma2[kp2.octave];
        const float x2 = (float)(dot3(Rcw2, x) + (double)tcw2[0]);
        const float y2 = (float)(dot3(Rcw2 + 3, x) + (double)tcw2[1]);
        const float invz2 = (float)(1.0 / z2);
        if (!bStereo2) {
            const float u2 = K2.fx * x2 * invz2 + K2.cx, v2 = K2.fy * y2 * invz2 + K2.cy;
            const float ex = u2 - kp2.x, ey = v2 - kp2.y;
            if ((ex * ex + ey * ey) > 5.991 * sigmaSquare2) continue;
        } else {
            const float u2 = K2.fx * x2 * invz2 + K2.cx;
            const float u2_r = u2 - K1.bf * invz2;
            const float v2 = K2.fy * y2 * invz2 + K2.cy;
            const float ex = u2 - kp2.x, ey = v2 - kp2.y, er = u2_r - kp2_ur;
            if ((ex * ex + ey * ey + er * er) > 7.8 * sigmaSquare2) continue;
        }
        // scale consistency (:539-557; the reference's text lost the `continue;` of upstream
        // ORB-SLAM2 and would not compile, DESIGN.md §8: the upstream rule is kept)
        const float n1[3] = {x[0] - Ow1[0], x[1] - Ow1[1], x[2] - Ow1[2]};
        const float n2[3] = {x[0] - Ow2[0], x[1] - Ow2[1], x[2] - Ow2[2]};
        const float dist1 = (float)std::sqrt(dot3(n1, n1)), dist2 = (float)std::sqrt(dot3(n2, n2));
        if (dist1 == 0 || dist2 == 0) continue;
        const float ratioDist = dist2 / dist1;
        const float ratioOctave = K1.scale_factors[kp1.octave] / K2.scale_factors[kp2.octave];
        if (ratioDist * ratioFactor < ratioOctave || ratioDist > ratioOctave * ratioFactor) continue;
        std::memcpy(x3d + 3 * k, x, sizeof(x));
        ok[k] = 1;
    }
    return ORBMI_OK;
}

}  // extern "C"
