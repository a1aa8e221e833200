// LocalMapping's host geometry around the GPU searches (src/LocalMapping.cc:290-577, :676-693):
// the fundamental matrix of a keyframe pair and the triangulation + acceptance tests of
// CreateNewMapPoints for the pairs SearchForTriangulation returned.  The per-match tests are
// tri_geom.h's, shared with the device's k_triangulate (orbmi_create_new_map_points).
#include <algorithm>
#include <cmath>
#include <cstring>

#include "../../include/orbmi.h"
#include "tri_geom.h"

using namespace orbmi::tri;

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
    // the level tables the matches index (and mfScaleFactor = scale_factors[1])
    int nlev = 2;
    for (int k = 0; k < n; k++)
        nlev = std::max(nlev, 1 + std::max<int>(kf1->keys_un[idx1[k]].octave, kf2->keys_un[idx2[k]].octave));
    if (nlev > kLevels) return ORBMI_E_ARG;
    Side K1, K2;
    make_side(*kf1, nlev, &K1);
    make_side(*kf2, nlev, &K2);
    for (int k = 0; k < n; k++) {
        const int i1 = idx1[k], i2 = idx2[k];
        const float cps1 = kf1->u_right[i1] >= 0 ? stereo_parallax_cos(K1.mb, kf1->depth[i1]) : 0.f;
        const float cps2 = kf2->u_right[i2] >= 0 ? stereo_parallax_cos(K2.mb, kf2->depth[i2]) : 0.f;
        float x[3];
        ok[k] = triangulate_one(K1, K2, i1, i2, cps1, cps2, x) ? 1 : 0;
        if (ok[k]) std::memcpy(x3d + 3 * k, x, sizeof(x));
    }
    return ORBMI_OK;
}

int orbmi_stereo_parallax_cos(float mb, const float* depth, int n, float* out) {
    if (n < 0 || (n > 0 && (!depth || !out))) return ORBMI_E_ARG;
    for (int i = 0; i < n; i++) out[i] = stereo_parallax_cos(mb, depth[i]);
    return ORBMI_OK;
}

}  // extern "C"
