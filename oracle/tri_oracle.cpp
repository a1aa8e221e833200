// ORACLE -- test infrastructure only (see orb_oracle.h).  An independent CPU restatement of
// LocalMapping::CreateNewMapPoints' per-match geometry (src/LocalMapping.cc:385-575), written
// from the reference text without the product's tri_geom.h, to check k_triangulate_par's
// decisions and new points (tests/test_triangulation_oracle.py, test_create_points_gpu.py).
//
// Differences from the product restatement are deliberate, so that agreement means something:
//  * cv::SVD::compute(A, w, u, vt) of the 4x4 system is restated as a one-sided (Hestenes) Jacobi
//    SVD of A in double -- the algorithm family OpenCV's JacobiSVD belongs to -- and x3D is the
//    right singular vector of the smallest singular value (vt.row(3)); the product takes the
//    eigenvector of A^T A instead.  The two agree to rounding, not bit for bit.
//  * every decision also reports its margin: the relative distance of the deciding quantity from
//    its threshold, so a test can tell a rounding-level disagreement from a real one.
// Shared conventions (pinned): cv::Mat CV_32F products and dot products
// accumulate in double and round to float; `Rcw.row(k).dot(x) + t` is a double sum rounded once;
// cos / atan2 on float arguments are the float overloads; mvKeys == mvKeysUn (rectified input,
// zero distortion), so UnprojectStereo's keypoint is the undistorted one.
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstring>

#include "orb_oracle.h"

namespace {

struct Kf {
    float R[3][3], t[3], Rwc[3][3], Ow[3];
    const orc_tri_keyframe* k;
};

void kf_setup(const orc_tri_keyframe* k, Kf* K) {  // KeyFrame::SetPose (src/KeyFrame.cc:72-86)
    K->k = k;
    for (int r = 0; r < 3; r++) {
        for (int c = 0; c < 3; c++) K->R[r][c] = k->tcw[4 * r + c];
        K->t[r] = k->tcw[4 * r + 3];
    }
    for (int r = 0; r < 3; r++)
        for (int c = 0; c < 3; c++) K->Rwc[r][c] = K->R[c][r];
    for (int r = 0; r < 3; r++) {  // Ow = -Rwc * tcw (one float gemm)
        double s = 0;
        for (int c = 0; c < 3; c++) s += (double)K->Rwc[r][c] * K->t[c];
        K->Ow[r] = -(float)s;
    }
}

float mat3vec(const float M[3][3], int r, const float v[3]) {  // row r of a float Mat product
    double s = 0;
    for (int c = 0; c < 3; c++) s += (double)M[r][c] * v[c];
    return (float)s;
}

float row_dot_plus(const float M[3][3], int r, const float x[3], float t) {  // Rcw.row(r).dot(x) + t
    double s = 0;
    for (int c = 0; c < 3; c++) s += (double)M[r][c] * x[c];
    return (float)(s + (double)t);
}

double rel_margin(double v, double th) {  // |v - th| relative to the larger magnitude
    const double d = std::fabs(v - th), m = std::max(std::fabs(v), std::fabs(th));
    return m > 0 ? d / m : d;
}

// right singular vector of the smallest singular value of the 4x4 A (one-sided Jacobi:
// orthogonalise the columns of U = A V by plane rotations until every pair is orthogonal)
void svd_null_vector(const float A[4][4], double v[4]) {
    double U[4][4], V[4][4];
    for (int r = 0; r < 4; r++)
        for (int c = 0; c < 4; c++) {
            U[r][c] = A[r][c];
            V[r][c] = r == c;
        }
    for (int sweep = 0; sweep < 60; sweep++) {
        bool rotated = false;
        for (int i = 0; i < 3; i++)
            for (int j = i + 1; j < 4; j++) {
                double a = 0, b = 0, g = 0;
                for (int r = 0; r < 4; r++) {
                    a += U[r][i] * U[r][i];
                    b += U[r][j] * U[r][j];
                    g += U[r][i] * U[r][j];
                }
                if (g == 0 || std::fabs(g) <= DBL_EPSILON * std::sqrt(a * b)) continue;
                rotated = true;
                const double zeta = (b - a) / (2 * g);
                const double t = (zeta >= 0 ? 1.0 : -1.0) / (std::fabs(zeta) + std::sqrt(1 + zeta * zeta));
                const double c = 1 / std::sqrt(1 + t * t), s = c * t;
                for (int r = 0; r < 4; r++) {
                    const double ui = U[r][i], uj = U[r][j];
                    U[r][i] = c * ui - s * uj;
                    U[r][j] = s * ui + c * uj;
                    const double vi = V[r][i], vj = V[r][j];
                    V[r][i] = c * vi - s * vj;
                    V[r][j] = s * vi + c * vj;
                }
            }
        if (!rotated) break;
    }
    int m = 0;
    double best = DBL_MAX;
    for (int c = 0; c < 4; c++) {
        double n2 = 0;
        for (int r = 0; r < 4; r++) n2 += U[r][c] * U[r][c];
        if (n2 < best) { best = n2; m = c; }
    }
    for (int r = 0; r < 4; r++) v[r] = V[r][m];
}

}  // namespace

extern "C" int orc_triangulate_matches(const orc_tri_keyframe* kf1, const orc_tri_keyframe* kf2, const int32_t* idx1,
                                       const int32_t* idx2, int n, float* x3d, uint8_t* ok, float* margin) {
    if (!kf1 || !kf2 || n < 0 || (n && (!idx1 || !idx2 || !x3d || !ok))) return -1;
    Kf K1, K2;
    kf_setup(kf1, &K1);
    kf_setup(kf2, &K2);
    const float invfx1 = 1.0f / kf1->fx, invfy1 = 1.0f / kf1->fy, invfx2 = 1.0f / kf2->fx, invfy2 = 1.0f / kf2->fy;
    const float ratioFactor = 1.5f * kf1->scale_factors[1];  // 1.5f * mfScaleFactor (:322)
    for (int m = 0; m < n; m++) {
        ok[m] = 0;
        x3d[3 * m] = x3d[3 * m + 1] = x3d[3 * m + 2] = 0;
        double mg = DBL_MAX;  // smallest relative margin of the decisions taken
        auto note = [&](double v, double th) { mg = std::min(mg, rel_margin(v, th)); };
        auto done = [&](bool accepted) {
            ok[m] = accepted;
            if (margin) margin[m] = (float)std::min(mg, (double)FLT_MAX);
        };
        const int i1 = idx1[m], i2 = idx2[m];
        const orc_keypoint& kp1 = kf1->keys_un[i1];
        const orc_keypoint& kp2 = kf2->keys_un[i2];
        const float kp1_ur = kf1->u_right[i1], kp2_ur = kf2->u_right[i2];
        const bool bStereo1 = kp1_ur >= 0, bStereo2 = kp2_ur >= 0;
        // :401-423 parallax of the two viewing rays
        const float xn1[3] = {(kp1.x - kf1->cx) * invfx1, (kp1.y - kf1->cy) * invfy1, 1.0f};
        const float xn2[3] = {(kp2.x - kf2->cx) * invfx2, (kp2.y - kf2->cy) * invfy2, 1.0f};
        float ray1[3], ray2[3];
        for (int r = 0; r < 3; r++) {
            ray1[r] = mat3vec(K1.Rwc, r, xn1);
            ray2[r] = mat3vec(K2.Rwc, r, xn2);
        }
        double d12 = 0, n1 = 0, n2 = 0;
        for (int r = 0; r < 3; r++) {
            d12 += (double)ray1[r] * ray2[r];
            n1 += (double)ray1[r] * ray1[r];
            n2 += (double)ray2[r] * ray2[r];
        }
        const float cosParallaxRays = (float)(d12 / (std::sqrt(n1) * std::sqrt(n2)));
        float cosParallaxStereo = cosParallaxRays + 1;
        float cosParallaxStereo1 = cosParallaxStereo, cosParallaxStereo2 = cosParallaxStereo;
        if (bStereo1)
            cosParallaxStereo1 = std::cos(2 * std::atan2(kf1->mb / 2, kf1->depth[i1]));
        else if (bStereo2)
            cosParallaxStereo2 = std::cos(2 * std::atan2(kf2->mb / 2, kf2->depth[i2]));
        cosParallaxStereo = std::min(cosParallaxStereo1, cosParallaxStereo2);
        float x[3];
        note(cosParallaxRays, cosParallaxStereo);
        note(cosParallaxRays, 0.0);
        if (!bStereo1 && !bStereo2) note(cosParallaxRays, 0.9998);
        if (cosParallaxRays < cosParallaxStereo && cosParallaxRays > 0 &&
            (bStereo1 || bStereo2 || cosParallaxRays < 0.9998)) {
            // :431-457 linear triangulation: rows x * T.row(2) - T.row(0|1) of both keyframes
            float A[4][4];
            for (int c = 0; c < 4; c++) {
                A[0][c] = xn1[0] * kf1->tcw[8 + c] - kf1->tcw[c];
                A[1][c] = xn1[1] * kf1->tcw[8 + c] - kf1->tcw[4 + c];
                A[2][c] = xn2[0] * kf2->tcw[8 + c] - kf2->tcw[c];
                A[3][c] = xn2[1] * kf2->tcw[8 + c] - kf2->tcw[4 + c];
            }
            double v[4];
            svd_null_vector(A, v);
            const float w = (float)v[3];
            if (w == 0) { done(false); continue; }
            for (int r = 0; r < 3; r++) x[r] = (float)v[r] / w;
        } else if (bStereo1 && cosParallaxStereo1 < cosParallaxStereo2) {
            note(cosParallaxStereo1, cosParallaxStereo2);
            const float z = kf1->depth[i1];  // KeyFrame::UnprojectStereo (src/KeyFrame.cc:629-645)
            const float xc[3] = {(kp1.x - kf1->cx) * z * invfx1, (kp1.y - kf1->cy) * z * invfy1, z};
            for (int r = 0; r < 3; r++) x[r] = row_dot_plus(K1.Rwc, r, xc, K1.Ow[r]);
        } else if (bStereo2 && cosParallaxStereo2 < cosParallaxStereo1) {
            note(cosParallaxStereo1, cosParallaxStereo2);
            const float z = kf2->depth[i2];
            const float xc[3] = {(kp2.x - kf2->cx) * z * invfx2, (kp2.y - kf2->cy) * z * invfy2, z};
            for (int r = 0; r < 3; r++) x[r] = row_dot_plus(K2.Rwc, r, xc, K2.Ow[r]);
        } else {
            done(false);
            continue;
        }
        // :474-482 in front of both cameras
        const float z1 = row_dot_plus(K1.R, 2, x, K1.t[2]);
        note(z1, 0.0);
        if (z1 <= 0) { done(false); continue; }
        const float z2 = row_dot_plus(K2.R, 2, x, K2.t[2]);
        note(z2, 0.0);
        if (z2 <= 0) { done(false); continue; }
        // :484-537 reprojection error in each keyframe (stereo: the right coordinate with the
        // current keyframe's mbf in both, as the reference writes it)
        auto reproj = [&](const Kf& K, const orc_keypoint& kp, float ur, bool stereo, float z) {
            const orc_tri_keyframe* k = K.k;
            const float s2 = k->level_sigma2[kp.octave];
            const float xx = row_dot_plus(K.R, 0, x, K.t[0]);
            const float yy = row_dot_plus(K.R, 1, x, K.t[1]);
            const float invz = 1.0 / z;
            const float u = k->fx * xx * invz + k->cx;
            const float vv = k->fy * yy * invz + k->cy;
            const float ex = u - kp.x, ey = vv - kp.y;
            if (!stereo) {
                const float e2 = ex * ex + ey * ey;
                note(e2, 5.991 * s2);
                return e2 > 5.991 * s2;
            }
            const float ur_p = u - kf1->bf * invz;
            const float er = ur_p - ur;
            const float e2 = ex * ex + ey * ey + er * er;
            note(e2, 7.8 * s2);
            return e2 > 7.8 * s2;
        };
        if (reproj(K1, kp1, kp1_ur, bStereo1, z1)) { done(false); continue; }
        if (reproj(K2, kp2, kp2_ur, bStereo2, z2)) { done(false); continue; }
        // :539-557 scale consistency (upstream ORB-SLAM2's rule: reject outside the factor)
        double s1 = 0, s2 = 0;
        for (int r = 0; r < 3; r++) {
            const float a = x[r] - K1.Ow[r], b = x[r] - K2.Ow[r];
            s1 += (double)a * a;
            s2 += (double)b * b;
        }
        const float dist1 = (float)std::sqrt(s1), dist2 = (float)std::sqrt(s2);
        if (dist1 == 0 || dist2 == 0) { done(false); continue; }
        const float ratioDist = dist2 / dist1;
        const float ratioOctave = kf1->scale_factors[kp1.octave] / kf2->scale_factors[kp2.octave];
        note(ratioDist * ratioFactor, ratioOctave);
        note(ratioDist, ratioOctave * ratioFactor);
        if (ratioDist * ratioFactor < ratioOctave || ratioDist > ratioOctave * ratioFactor) { done(false); continue; }
        for (int r = 0; r < 3; r++) x3d[3 * m + r] = x[r];
        done(true);
    }
    return 0;
}
