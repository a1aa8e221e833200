// ORACLE — test infrastructure only (see orb_oracle.h).
// ORBmatcher::SearchByProjection (x2), SearchByBoW, Frame::isInFrustum / GetFeaturesInArea /
// AssignFeaturesToGrid and MapPoint::PredictScale restated sequentially, literally in the
// reference's loop order.  Boundary structs come from include/orbmi.h (data layout only).
//
// Pinned float semantics (P10): 3x3*3x1 + t products are float, left to right
// ((r0*x + r1*y) + r2*z) + t (cv::gemm small-matrix path); -R^T t likewise; cv::norm and
// Mat::dot accumulate in double; PredictScale uses (float)log((double)ratio).
#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

#include "../include/orbmi.h"

namespace {

const int kGridCols = 64, kGridRows = 48;  // FRAME_GRID_COLS / ROWS  include/Frame.h:34-35
const int TH_HIGH = 100, TH_LOW = 50, HISTO_LENGTH = 30;  // src/ORBmatcher.cc:37-39

struct Grid {
    std::vector<int> cell[kGridCols][kGridRows];
};

// Frame::AssignFeaturesToGrid / PosInGrid  src/Frame.cc:232-247, :412-422
void build_grid(const orbmi_frame_view& F, Grid& g) {
    for (int i = 0; i < F.n; i++) {
        const orbmi_keypoint& kp = F.keys_un[i];
        const int px = (int)roundf((kp.x - F.min_x) * F.grid_w_inv);
        const int py = (int)roundf((kp.y - F.min_y) * F.grid_h_inv);
        if (px < 0 || px >= kGridCols || py < 0 || py >= kGridRows) continue;
        g.cell[px][py].push_back(i);
    }
}

// Frame::GetFeaturesInArea  src/Frame.cc:353-410
void features_in_area(const orbmi_frame_view& F, const Grid& g, float x, float y, float r, int minLevel,
                      int maxLevel, std::vector<int>& out) {
    out.clear();
    const int nMinCellX = std::max(0, (int)floorf((x - F.min_x - r) * F.grid_w_inv));
    if (nMinCellX >= kGridCols) return;
    const int nMaxCellX = std::min(kGridCols - 1, (int)ceilf((x - F.min_x + r) * F.grid_w_inv));
    if (nMaxCellX < 0) return;
    const int nMinCellY = std::max(0, (int)floorf((y - F.min_y - r) * F.grid_h_inv));
    if (nMinCellY >= kGridRows) return;
    const int nMaxCellY = std::min(kGridRows - 1, (int)ceilf((y - F.min_y + r) * F.grid_h_inv));
    if (nMaxCellY < 0) return;
    const bool bCheckLevels = (minLevel > 0) || (maxLevel >= 0);
    for (int ix = nMinCellX; ix <= nMaxCellX; ix++)
        for (int iy = nMinCellY; iy <= nMaxCellY; iy++)
            for (int idx : g.cell[ix][iy]) {
                const orbmi_keypoint& kp = F.keys_un[idx];
                if (bCheckLevels) {
                    if (kp.octave < minLevel) continue;
                    if (maxLevel >= 0 && kp.octave > maxLevel) continue;
                }
                const float distx = kp.x - x, disty = kp.y - y;
                if (fabsf(distx) < r && fabsf(disty) < r) out.push_back(idx);
            }
}

int hamming(const uint8_t* a, const uint8_t* b) {
    int d = 0;
    for (int i = 0; i < 32; i++) d += __builtin_popcount((unsigned)(a[i] ^ b[i]));
    return d;
}

// R*p + t with R = T[0..2][0..2], t = T[0..2][3] (row-major 4x4 float)
void transform(const float* T, const float* p, float* o) {
    for (int r = 0; r < 3; r++) o[r] = ((T[4 * r] * p[0] + T[4 * r + 1] * p[1]) + T[4 * r + 2] * p[2]) + T[4 * r + 3];
}

// -R^T t
void camera_center(const float* T, float* o) {
    for (int c = 0; c < 3; c++) o[c] = -((T[c] * T[3] + T[4 + c] * T[7]) + T[8 + c] * T[11]);
}

float radius_by_viewing_cos(float viewCos) { return viewCos > 0.998 ? 2.5f : 4.0f; }

// ORBmatcher::ComputeThreeMaxima  src/ORBmatcher.cc:1854-1895
void three_maxima(const std::vector<int>* histo, int L, int& ind1, int& ind2, int& ind3) {
    int max1 = 0, max2 = 0, max3 = 0;
    for (int i = 0; i < L; i++) {
        const int s = (int)histo[i].size();
        if (s > max1) { max3 = max2; max2 = max1; max1 = s; ind3 = ind2; ind2 = ind1; ind1 = i; }
        else if (s > max2) { max3 = max2; max2 = s; ind3 = ind2; ind2 = i; }
        else if (s > max3) { max3 = s; ind3 = i; }
    }
    if (max2 < 0.1f * (float)max1) { ind2 = -1; ind3 = -1; }
    else if (max3 < 0.1f * (float)max1) { ind3 = -1; }
}

int rot_bin(float a0, float a1) {
    const float factor = 1.0f / HISTO_LENGTH;
    float rot = a0 - a1;
    if (rot < 0.0) rot += 360.0f;
    int bin = (int)roundf(rot * factor);
    if (bin == HISTO_LENGTH) bin = 0;
    return bin;
}

}  // namespace

extern "C" {

// Frame::isInFrustum + MapPoint::PredictScale, skipping BAD / SEEN points like SearchLocalPoints.
int orc_is_in_frustum(const orbmi_frame_view* F, const orbmi_mappoint* mps, int n, float viewingCosLimit,
                      orbmi_mappoint_track* tr) {
    float Ow[3];
    camera_center(F->tcw, Ow);
    for (int i = 0; i < n; i++) {
        const orbmi_mappoint& mp = mps[i];
        orbmi_mappoint_track& t = tr[i];
        memset(&t, 0, sizeof(t));
        if (mp.flags & (ORBMI_MP_BAD | ORBMI_MP_SEEN)) continue;
        float Pc[3];
        transform(F->tcw, mp.pos, Pc);
        if (Pc[2] < 0.0f) continue;
        const float invz = 1.0f / Pc[2];
        const float u = F->fx * Pc[0] * invz + F->cx;
        const float v = F->fy * Pc[1] * invz + F->cy;
        if (u < F->min_x || u > F->max_x) continue;
        if (v < F->min_y || v > F->max_y) continue;
        const float maxDistance = 1.2f * mp.max_distance;
        const float minDistance = 0.8f * mp.min_distance;
        const float PO[3] = {mp.pos[0] - Ow[0], mp.pos[1] - Ow[1], mp.pos[2] - Ow[2]};
        const float dist = (float)sqrt((double)PO[0] * PO[0] + (double)PO[1] * PO[1] + (double)PO[2] * PO[2]);
        if (dist < minDistance || dist > maxDistance) continue;
        const double dot = (double)PO[0] * mp.normal[0] + (double)PO[1] * mp.normal[1] + (double)PO[2] * mp.normal[2];
        const float viewCos = (float)(dot / (double)dist);
        if (viewCos < viewingCosLimit) continue;
        const float ratio = mp.max_distance / dist;
        int nScale = (int)ceilf((float)log((double)ratio) / F->log_scale_factor);
        if (nScale < 0) nScale = 0;
        else if (nScale >= F->nlevels) nScale = F->nlevels - 1;
        t.in_view = 1;
        t.proj_x = u;
        t.proj_xr = u - F->bf * invz;
        t.proj_y = v;
        t.level = nScale;
        t.view_cos = viewCos;
    }
    return 0;
}

// ORBmatcher::SearchByProjection(Frame&, const vector<MapPoint*>&, th)  src/ORBmatcher.cc:59-155
int orc_search_by_projection_local(const orbmi_frame_view* F, const uint8_t* occupied0, const orbmi_mappoint* mps,
                                   const orbmi_mappoint_track* tr, int n_mp, float th, float nnratio,
                                   int32_t* match_mp, int* nmatches_out) {
    Grid g;
    build_grid(*F, g);
    std::vector<uint8_t> occupied(occupied0, occupied0 + F->n);
    for (int i = 0; i < F->n; i++) match_mp[i] = -1;
    const bool bFactor = th != 1.0;
    int nmatches = 0;
    std::vector<int> idx;
    for (int iMP = 0; iMP < n_mp; iMP++) {
        const orbmi_mappoint_track& t = tr[iMP];
        if (!t.in_view) continue;
        if (mps[iMP].flags & ORBMI_MP_BAD) continue;
        const int nPredictedLevel = t.level;
        float r = radius_by_viewing_cos(t.view_cos);
        if (bFactor) r *= th;
        const float rs = r * F->scale_factors[nPredictedLevel];
        features_in_area(*F, g, t.proj_x, t.proj_y, rs, nPredictedLevel - 1, nPredictedLevel, idx);
        if (idx.empty()) continue;
        int bestDist = 256, bestLevel = -1, bestDist2 = 256, bestLevel2 = -1, bestIdx = -1;
        for (int id : idx) {
            if (occupied[id]) continue;
            if (F->u_right && F->u_right[id] > 0) {
                const float er = fabsf(t.proj_xr - F->u_right[id]);
                if (er > r * F->scale_factors[nPredictedLevel]) continue;
            }
            const int dist = hamming(mps[iMP].desc, F->desc + 32 * id);
            if (dist < bestDist) {
                bestDist2 = bestDist; bestDist = dist;
                bestLevel2 = bestLevel; bestLevel = F->keys_un[id].octave;
                bestIdx = id;
            } else if (dist < bestDist2) {
                bestLevel2 = F->keys_un[id].octave;
                bestDist2 = dist;
            }
        }
        if (bestDist <= TH_HIGH) {
            if (bestLevel == bestLevel2 && bestDist > nnratio * bestDist2) continue;
            match_mp[bestIdx] = iMP;
            occupied[bestIdx] = (mps[iMP].flags & ORBMI_MP_HAS_OBS) ? 1 : 0;
            nmatches++;
        }
    }
    *nmatches_out = nmatches;
    return 0;
}

// ORBmatcher::SearchByProjection(Frame& CF, const Frame& LF, th, bMono)  src/ORBmatcher.cc:1540-1695
int orc_search_by_projection_last_frame(const orbmi_frame_view* CF, const uint8_t* occupied0,
                                        const orbmi_frame_view* LF, const orbmi_lastframe_point* lfp, float th,
                                        int mono, int check_ori, int32_t* match_lf, int* nmatches_out) {
    Grid g;
    build_grid(*CF, g);
    std::vector<uint8_t> occupied(occupied0, occupied0 + CF->n);
    for (int i = 0; i < CF->n; i++) match_lf[i] = -1;
    std::vector<int> rotHist[HISTO_LENGTH];
    const float* Tc = CF->tcw;
    const float* Tl = LF->tcw;
    float twc[3];
    camera_center(Tc, twc);
    float tlc[3];
    transform(Tl, twc, tlc);
    const bool bForward = tlc[2] > CF->mb && !mono;
    const bool bBackward = -tlc[2] > CF->mb && !mono;
    int nmatches = 0;
    std::vector<int> idx;
    for (int i = 0; i < LF->n; i++) {
        const orbmi_lastframe_point& p = lfp[i];
        if (!(p.flags & ORBMI_LF_HAS_MP) || (p.flags & ORBMI_LF_OUTLIER)) continue;
        float x3Dc[3];
        transform(Tc, p.pos, x3Dc);
        const float xc = x3Dc[0], yc = x3Dc[1];
        const float invzc = (float)(1.0 / (double)x3Dc[2]);
        if (invzc < 0) continue;
        const float u = CF->fx * xc * invzc + CF->cx;
        const float v = CF->fy * yc * invzc + CF->cy;
        if (u < CF->min_x || u > CF->max_x) continue;
        if (v < CF->min_y || v > CF->max_y) continue;
        const int nLastOctave = LF->keys_un[i].octave;
        const float radius = th * CF->scale_factors[nLastOctave];
        if (bForward) features_in_area(*CF, g, u, v, radius, nLastOctave, -1, idx);
        else if (bBackward) features_in_area(*CF, g, u, v, radius, 0, nLastOctave, idx);
        else features_in_area(*CF, g, u, v, radius, nLastOctave - 1, nLastOctave + 1, idx);
        if (idx.empty()) continue;
        int bestDist = 256, bestIdx2 = -1;
        for (int i2 : idx) {
            if (occupied[i2]) continue;
            if (CF->u_right && CF->u_right[i2] > 0) {
                const float ur = u - CF->bf * invzc;
                const float er = fabsf(ur - CF->u_right[i2]);
                if (er > radius) continue;
            }
            const int dist = hamming(p.desc, CF->desc + 32 * i2);
            if (dist < bestDist) { bestDist = dist; bestIdx2 = i2; }
        }
        if (bestDist <= TH_HIGH) {
            match_lf[bestIdx2] = i;
            occupied[bestIdx2] = (p.flags & ORBMI_MP_HAS_OBS) ? 1 : 0;
            nmatches++;
            if (check_ori) rotHist[rot_bin(LF->keys_un[i].angle, CF->keys_un[bestIdx2].angle)].push_back(bestIdx2);
        }
    }
    if (check_ori) {
        int ind1 = -1, ind2 = -1, ind3 = -1;
        three_maxima(rotHist, HISTO_LENGTH, ind1, ind2, ind3);
        for (int b = 0; b < HISTO_LENGTH; b++) {
            if (b == ind1 || b == ind2 || b == ind3) continue;
            for (int k : rotHist[b]) { match_lf[k] = -2; nmatches--; }  // mvpMapPoints[k] = NULL
        }
    }
    *nmatches_out = nmatches;
    return 0;
}

// ORBmatcher::SearchByBoW(KeyFrame*, Frame&, vector<MapPoint*>&)  src/ORBmatcher.cc:211-344
int orc_search_by_bow(const orbmi_frame_view* KF, const uint8_t* kf_mp_ok, const orbmi_feature_vector* kfv,
                      const orbmi_frame_view* F, const orbmi_feature_vector* fv, float nnratio, int check_ori,
                      int32_t* match_kf, int* nmatches_out) {
    for (int i = 0; i < F->n; i++) match_kf[i] = -1;
    std::vector<int> rotHist[HISTO_LENGTH];
    int nmatches = 0;
    int a = 0, b = 0;
    while (a < kfv->nnodes && b < fv->nnodes) {
        if (kfv->node_id[a] == fv->node_id[b]) {
            for (int ia = kfv->off[a]; ia < kfv->off[a + 1]; ia++) {
                const int realIdxKF = kfv->feat[ia];
                if (!kf_mp_ok[realIdxKF]) continue;
                const uint8_t* dKF = KF->desc + 32 * realIdxKF;
                int bestDist1 = 256, bestIdxF = -1, bestDist2 = 256;
                for (int ib = fv->off[b]; ib < fv->off[b + 1]; ib++) {
                    const int realIdxF = fv->feat[ib];
                    if (match_kf[realIdxF] >= 0) continue;
                    const int dist = hamming(dKF, F->desc + 32 * realIdxF);
                    if (dist < bestDist1) { bestDist2 = bestDist1; bestDist1 = dist; bestIdxF = realIdxF; }
                    else if (dist < bestDist2) { bestDist2 = dist; }
                }
                if (bestDist1 <= TH_LOW) {
                    if ((float)bestDist1 < nnratio * (float)bestDist2) {
                        match_kf[bestIdxF] = realIdxKF;
                        if (check_ori) rotHist[rot_bin(KF->keys_un[realIdxKF].angle, F->keys_un[bestIdxF].angle)].push_back(bestIdxF);
                        nmatches++;
                    }
                }
            }
            a++;
            b++;
        } else if (kfv->node_id[a] < fv->node_id[b]) {
            // KFit = vFeatVecKF.lower_bound(Fit->first)
            while (a < kfv->nnodes && kfv->node_id[a] < fv->node_id[b]) a++;
        } else {
            while (b < fv->nnodes && fv->node_id[b] < kfv->node_id[a]) b++;
        }
    }
    if (check_ori) {
        int ind1 = -1, ind2 = -1, ind3 = -1;
        three_maxima(rotHist, HISTO_LENGTH, ind1, ind2, ind3);
        for (int bb = 0; bb < HISTO_LENGTH; bb++) {
            if (bb == ind1 || bb == ind2 || bb == ind3) continue;
            for (int k : rotHist[bb]) { match_kf[k] = -1; nmatches--; }
        }
    }
    *nmatches_out = nmatches;
    return 0;
}

}  // extern "C"

// MapPoint::ComputeDistinctiveDescriptors  src/MapPoint.cc:247-316 (literal: float distance
// matrix, std::sort of each row, vDists[0.5*(N-1)], strict < over the rows)
extern "C" int orc_compute_distinctive_descriptors(const uint8_t* obs_desc, const int32_t* obs_off, int np,
                                                   int32_t* best, uint8_t* desc_out) {
    for (int p = 0; p < np; p++) {
        const int b = obs_off[p];
        const size_t N = (size_t)(obs_off[p + 1] - b);
        if (N == 0) { best[p] = -1; continue; }
        std::vector<float> Distances(N * N);
        for (size_t i = 0; i < N; i++) {
            Distances[i * N + i] = 0;
            for (size_t j = i + 1; j < N; j++) {
                int distij = 0;
                for (int q = 0; q < 32; q++)
                    distij += __builtin_popcount((unsigned)(obs_desc[32 * (b + i) + q] ^ obs_desc[32 * (b + j) + q]));
                Distances[i * N + j] = (float)distij;
                Distances[j * N + i] = (float)distij;
            }
        }
        int BestMedian = 0x7FFFFFFF, BestIdx = 0;
        for (size_t i = 0; i < N; i++) {
            std::vector<int> vDists(Distances.begin() + i * N, Distances.begin() + (i + 1) * N);
            std::sort(vDists.begin(), vDists.end());
            const int median = vDists[(size_t)(0.5 * (N - 1))];
            if (median < BestMedian) {
                BestMedian = median;
                BestIdx = (int)i;
            }
        }
        best[p] = BestIdx;
        memcpy(desc_out + 32 * (size_t)p, obs_desc + 32 * (size_t)(b + BestIdx), 32);
    }
    return 0;
}

// ORBmatcher::SearchForTriangulation  src/ORBmatcher.cc:783-975 with CheckDistEpipolarLine
// (:173-196) and ComputeThreeMaxima.  Literal: FeatureVector merge-join, no exclusion of already
// matched KF2 keypoints (vbMatched2 is never set in the reference), the last candidate of equal
// distance that passes the epipolar test wins.  The epipole uses the camera centre
// Ow1 = -R1w^T t1w and C2 = R2w Ow1 + t2w with the P10 float order.
extern "C" int orc_search_for_triangulation(const orbmi_frame_view* KF1, const uint8_t* has_mp1,
                                            const orbmi_feature_vector* fv1, const orbmi_frame_view* KF2,
                                            const uint8_t* has_mp2, const orbmi_feature_vector* fv2,
                                            const float* F12, int only_stereo, int check_ori, int32_t* match12,
                                            int* nmatches_out) {
    const float* T1 = KF1->tcw;
    const float* T2 = KF2->tcw;
    float Ow[3];
    for (int i = 0; i < 3; i++) Ow[i] = -(((T1[0 * 4 + i] * T1[3]) + T1[1 * 4 + i] * T1[7]) + T1[2 * 4 + i] * T1[11]);
    float C2[3];
    for (int i = 0; i < 3; i++) C2[i] = (((T2[i * 4 + 0] * Ow[0]) + T2[i * 4 + 1] * Ow[1]) + T2[i * 4 + 2] * Ow[2]) + T2[i * 4 + 3];
    const float invz = 1.0f / C2[2];
    const float ex = KF2->fx * C2[0] * invz + KF2->cx;
    const float ey = KF2->fy * C2[1] * invz + KF2->cy;
    std::vector<float> sigma2(KF2->nlevels);
    for (int l = 0; l < KF2->nlevels; l++) sigma2[l] = KF2->scale_factors[l] * KF2->scale_factors[l];
    int nmatches = 0;
    for (int i = 0; i < KF1->n; i++) match12[i] = -1;
    std::vector<int> rotHist[HISTO_LENGTH];
    auto check_epi = [&](const orbmi_keypoint& kp1, const orbmi_keypoint& kp2) {
        const float a = kp1.x * F12[0 * 3 + 0] + kp1.y * F12[1 * 3 + 0] + F12[2 * 3 + 0];
        const float b = kp1.x * F12[0 * 3 + 1] + kp1.y * F12[1 * 3 + 1] + F12[2 * 3 + 1];
        const float c = kp1.x * F12[0 * 3 + 2] + kp1.y * F12[1 * 3 + 2] + F12[2 * 3 + 2];
        const float num = a * kp2.x + b * kp2.y + c;
        const float den = a * a + b * b;
        if (den == 0) return false;
        const float dsqr = num * num / den;
        return dsqr < 3.84 * sigma2[kp2.octave];
    };
    int a = 0, b = 0;
    while (a < fv1->nnodes && b < fv2->nnodes) {
        if (fv1->node_id[a] == fv2->node_id[b]) {
            for (int i1 = fv1->off[a]; i1 < fv1->off[a + 1]; i1++) {
                const int idx1 = fv1->feat[i1];
                if (has_mp1[idx1]) continue;
                const bool bStereo1 = KF1->u_right[idx1] >= 0;
                if (only_stereo && !bStereo1) continue;
                const orbmi_keypoint& kp1 = KF1->keys_un[idx1];
                const uint8_t* d1 = KF1->desc + 32 * (size_t)idx1;
                int bestDist = TH_LOW, bestIdx2 = -1;
                for (int i2 = fv2->off[b]; i2 < fv2->off[b + 1]; i2++) {
                    const int idx2 = fv2->feat[i2];
                    if (has_mp2[idx2]) continue;
                    const bool bStereo2 = KF2->u_right[idx2] >= 0;
                    if (only_stereo && !bStereo2) continue;
                    int dist = 0;
                    for (int q = 0; q < 32; q++) dist += __builtin_popcount((unsigned)(d1[q] ^ KF2->desc[32 * (size_t)idx2 + q]));
                    if (dist > TH_LOW || dist > bestDist) continue;
                    const orbmi_keypoint& kp2 = KF2->keys_un[idx2];
                    if (!bStereo1 && !bStereo2) {
                        const float distex = ex - kp2.x;
                        const float distey = ey - kp2.y;
                        if (distex * distex + distey * distey < 100 * KF2->scale_factors[kp2.octave]) continue;
                    }
                    if (check_epi(kp1, kp2)) {
                        bestIdx2 = idx2;
                        bestDist = dist;
                    }
                }
                if (bestIdx2 >= 0) {
                    match12[idx1] = bestIdx2;
                    nmatches++;
                    if (check_ori) rotHist[rot_bin(kp1.angle, KF2->keys_un[bestIdx2].angle)].push_back(idx1);
                }
            }
            a++;
            b++;
        } else if (fv1->node_id[a] < fv2->node_id[b]) {
            while (a < fv1->nnodes && fv1->node_id[a] < fv2->node_id[b]) a++;
        } else {
            while (b < fv2->nnodes && fv2->node_id[b] < fv1->node_id[a]) b++;
        }
    }
    if (check_ori) {
        int ind1 = -1, ind2 = -1, ind3 = -1;
        three_maxima(rotHist, HISTO_LENGTH, ind1, ind2, ind3);
        for (int i = 0; i < HISTO_LENGTH; i++) {
            if (i == ind1 || i == ind2 || i == ind3) continue;
            for (int idx1 : rotHist[i]) { match12[idx1] = -1; nmatches--; }
        }
    }
    *nmatches_out = nmatches;
    return 0;
}

// ORBmatcher::Fuse(KeyFrame*, const vector<MapPoint*>&, th)  src/ORBmatcher.cc:977-1127, the
// search part in list order (the map updates are the caller's replay, include/orbmi.h).
extern "C" int orc_fuse_search(const orbmi_frame_view* KF, const orbmi_mappoint* mps, const uint8_t* in_kf, int n_mp,
                               float th, int32_t* best_idx, int32_t* best_dist, int* ncand) {
    Grid g;
    build_grid(*KF, g);
    float Ow[3];
    camera_center(KF->tcw, Ow);
    std::vector<int> idxs;
    int n = 0;
    for (int i = 0; i < n_mp; i++) {
        best_idx[i] = -1;
        best_dist[i] = 256;
        const orbmi_mappoint& mp = mps[i];
        if ((mp.flags & ORBMI_MP_BAD) || (in_kf && in_kf[i])) continue;
        float p3Dc[3];
        transform(KF->tcw, mp.pos, p3Dc);
        if (p3Dc[2] < 0.0f) continue;
        const float invz = 1 / p3Dc[2];
        const float x = p3Dc[0] * invz;
        const float y = p3Dc[1] * invz;
        const float u = KF->fx * x + KF->cx;
        const float v = KF->fy * y + KF->cy;
        if (!(u >= KF->min_x && u < KF->max_x && v >= KF->min_y && v < KF->max_y)) continue;  // IsInImage
        const float ur = u - KF->bf * invz;
        const float maxDistance = 1.2f * mp.max_distance;
        const float minDistance = 0.8f * mp.min_distance;
        const float PO[3] = {mp.pos[0] - Ow[0], mp.pos[1] - Ow[1], mp.pos[2] - Ow[2]};
        const float dist3D = (float)sqrt((double)PO[0] * PO[0] + (double)PO[1] * PO[1] + (double)PO[2] * PO[2]);
        if (dist3D < minDistance || dist3D > maxDistance) continue;
        const double dot = (double)PO[0] * mp.normal[0] + (double)PO[1] * mp.normal[1] + (double)PO[2] * mp.normal[2];
        if (dot < 0.5 * dist3D) continue;
        const float ratio = mp.max_distance / dist3D;
        int nPredictedLevel = (int)ceilf((float)log((double)ratio) / KF->log_scale_factor);
        if (nPredictedLevel < 0) nPredictedLevel = 0;
        else if (nPredictedLevel >= KF->nlevels) nPredictedLevel = KF->nlevels - 1;
        const float radius = th * KF->scale_factors[nPredictedLevel];
        features_in_area(*KF, g, u, v, radius, -1, -1, idxs);
        if (idxs.empty()) continue;
        int bestDist = 256, bestIdx = -1;
        for (int idx : idxs) {
            const orbmi_keypoint& kp = KF->keys_un[idx];
            const int kpLevel = kp.octave;
            if (kpLevel < nPredictedLevel - 1 || kpLevel > nPredictedLevel) continue;
            const float sigma2 = KF->scale_factors[kpLevel] * KF->scale_factors[kpLevel];
            const float inv = 1.0f / sigma2;  // mvInvLevelSigma2
            if (KF->u_right && KF->u_right[idx] >= 0) {
                const float ex = u - kp.x, ey = v - kp.y, er = ur - KF->u_right[idx];
                const float e2 = ex * ex + ey * ey + er * er;
                if (e2 * inv > 7.8) continue;
            } else {
                const float ex = u - kp.x, ey = v - kp.y;
                const float e2 = ex * ex + ey * ey;
                if (e2 * inv > 5.99) continue;
            }
            const int dist = hamming(mp.desc, KF->desc + 32 * idx);
            if (dist < bestDist) {
                bestDist = dist;
                bestIdx = idx;
            }
        }
        best_dist[i] = bestDist;
        if (bestDist <= TH_LOW) {
            best_idx[i] = bestIdx;
            n++;
        }
    }
    *ncand = n;
    return 0;
}
