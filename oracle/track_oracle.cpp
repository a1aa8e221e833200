// ORACLE — test infrastructure only (see orb_oracle.h).
// Tracking::TrackWithMotionModel + Tracking::TrackLocalMap (src/Tracking.cc:997-1104) for a
// stereo frame, restated sequentially over the oracle's matchers (orb_match_oracle.cpp) and
// PoseOptimization (pose_oracle.cpp):
//   SearchByProjection(CF, LF, th) [retry at 2*th when < 20 matches]     :1014-1026
//   PoseOptimization edge assembly (src/Optimizer.cc:296-375) + optimisation
//   discard outliers / nmatchesMap                                       :1036-1058
//   SearchLocalPoints (isInFrustum 0.5 + SearchByProjection th, 0.8)     :1362-1402
//   PoseOptimization, mnMatchesInliers, stereo outliers -> NULL          :1083-1104
// UpdateLastFrame / UpdateLocalMap (map management, out of scope) are the caller's inputs:
// the last frame's points and the local map arrive as flat arrays (include/orbmi.h).
#include <cstring>
#include <limits>
#include <vector>

#include "../include/orbmi.h"

extern "C" {
int orc_is_in_frustum(const orbmi_frame_view* F, const orbmi_mappoint* mps, int n, float viewingCosLimit,
                      orbmi_mappoint_track* tr);
int orc_search_by_projection_local(const orbmi_frame_view* F, const uint8_t* occupied0, const orbmi_mappoint* mps,
                                   const orbmi_mappoint_track* tr, int n, float th, float nnratio, int* out,
                                   int* nmatches);
int orc_search_by_projection_last_frame(const orbmi_frame_view* CF, const uint8_t* occupied0,
                                        const orbmi_frame_view* LF, const orbmi_lastframe_point* lfp, float th,
                                        int mono, int check_ori, int* out, int* nmatches);
int orc_pose_optimization(orbmi_pose_frame* f, const orbmi_pose_obs* obs, uint8_t* outlier);
void orc_pose_set_diag(float* chi2_rounds, double* stop_margin);
}

namespace {

// Frame::mvpMapPoints[i] as the match arrays describe it (orbmi_frame_mappoints)
const float* point_of(const orbmi_frame_mappoints& mp, int i, bool* has_obs) {
    if (mp.match_mp && mp.match_mp[i] >= 0 && mp.match_mp[i] < mp.n_mps) {
        const orbmi_mappoint& p = mp.mps[mp.match_mp[i]];
        *has_obs = (p.flags & ORBMI_MP_HAS_OBS) != 0;
        return p.pos;
    }
    if (mp.match_lf && mp.match_lf[i] >= 0 && mp.match_lf[i] < mp.n_lf_points) {
        const orbmi_lastframe_point& p = mp.lf_points[mp.match_lf[i]];
        *has_obs = (p.flags & ORBMI_MP_HAS_OBS) != 0;
        return p.pos;
    }
    return nullptr;
}

int* slot_of(const orbmi_frame_mappoints& mp, int i) {
    if (mp.match_mp && mp.match_mp[i] >= 0 && mp.match_mp[i] < mp.n_mps) return &mp.match_mp[i];
    if (mp.match_lf && mp.match_lf[i] >= 0 && mp.match_lf[i] < mp.n_lf_points) return &mp.match_lf[i];
    return nullptr;
}

}  // namespace

// Parity diagnostics (orc_pose_set_frame_diag): pose_oracle.cpp's per-round classification
// chi2, scattered to keypoint indices (4 x n_kp, NaN for keypoints without an edge).
thread_local float* g_frame_diag_chi2 = nullptr;
thread_local int g_frame_diag_n = 0;
thread_local double* g_frame_diag_stop = nullptr;

extern "C" {

void orc_pose_set_frame_diag(float* chi2_kp_rounds, int n_kp, double* stop_margin) {
    g_frame_diag_chi2 = chi2_kp_rounds;
    g_frame_diag_n = n_kp;
    g_frame_diag_stop = stop_margin;
}

// Optimizer::PoseOptimization(Frame*) (src/Optimizer.cc:257-481): edges in keypoint order
// (:296-375), then the 4-round optimisation of pose_oracle.cpp.  outlier: F->n entries.
int orc_pose_optimization_frame(const orbmi_frame_view* F, const float* inv_level_sigma2,
                                const orbmi_frame_mappoints* mp, orbmi_pose_frame* rec, uint8_t* outlier) {
    std::vector<orbmi_pose_obs> obs;
    for (int i = 0; i < F->n; i++) {
        outlier[i] = 0;
        bool has_obs;
        const float* X = point_of(*mp, i, &has_obs);
        if (!X) continue;
        const orbmi_keypoint& kp = F->keys_un[i];
        orbmi_pose_obs o;
        o.Xw[0] = X[0]; o.Xw[1] = X[1]; o.Xw[2] = X[2];
        o.u = kp.x;
        o.v = kp.y;
        o.ur = F->u_right ? F->u_right[i] : -1.0f;
        o.inv_sigma2 = inv_level_sigma2[kp.octave];
        o.index = i;
        obs.push_back(o);
    }
    memcpy(rec->tcw, F->tcw, sizeof(rec->tcw));
    rec->fx = F->fx; rec->fy = F->fy; rec->cx = F->cx; rec->cy = F->cy; rec->bf = F->bf;
    rec->obs_begin = 0;
    rec->n_obs = (int)obs.size();
    std::vector<uint8_t> fl(obs.size() + 1);
    std::vector<float> diag;
    if (g_frame_diag_chi2) {
        diag.assign(4 * obs.size() + 1, std::numeric_limits<float>::quiet_NaN());
        for (int k = 0; k < 4 * g_frame_diag_n; k++) g_frame_diag_chi2[k] = std::numeric_limits<float>::quiet_NaN();
        orc_pose_set_diag(diag.data(), g_frame_diag_stop);
    }
    orc_pose_optimization(rec, obs.data(), fl.data());
    if (g_frame_diag_chi2) {
        orc_pose_set_diag(nullptr, nullptr);
        const size_t no = obs.size();
        for (int r = 0; r < 4; r++)
            for (size_t k = 0; k < no; k++) g_frame_diag_chi2[r * g_frame_diag_n + obs[k].index] = diag[r * no + k];
    }
    for (size_t k = 0; k < obs.size(); k++) outlier[obs[k].index] = fl[k];
    return rec->inliers;
}

// Tracking's pass over mvpMapPoints after PoseOptimization (orbmi_track_update_matches).
int orc_track_update_matches(const orbmi_frame_view* F, int stage, const uint8_t* outlier,
                             const orbmi_frame_mappoints* mp, uint8_t* occupied_out, int* counts) {
    counts[0] = counts[1] = 0;
    for (int i = 0; i < F->n; i++) {
        bool obs = false;
        int* slot = slot_of(*mp, i);
        if (slot) point_of(*mp, i, &obs);
        bool occ = false;
        if (slot) {
            if (stage == 0) {  // :1042-1055
                if (outlier[i]) { *slot = -1; counts[0]++; }
                else if (obs) { counts[1]++; occ = true; }
            } else {           // :1087-1101
                if (!outlier[i]) counts[0] += obs;
                else { counts[1]++; if (F->u_right) *slot = -1; }
            }
        }
        if (occupied_out) occupied_out[i] = occ;
    }
    return 0;
}

// TrackWithMotionModel + TrackLocalMap of one stereo frame.  CF->tcw = mVelocity * LastTcw on
// entry.  Outputs: match_lf / match_mp (CF->n; final mvpMapPoints), outlier (CF->n; final
// mvbOutlier), tcw_mm = pose after the motion-model PoseOptimization, tcw = final pose,
// stats = {search matches, nmatchesMap, mnMatchesInliers, nToMatch}.  Returns 1 when both
// stages succeed (nmatchesMap >= 10, mnMatchesInliers >= 30), 0 when tracking is lost (the
// outputs then hold the state where it stopped).
int orc_track_frame(const orbmi_frame_view* CF, const orbmi_frame_view* LF, const orbmi_lastframe_point* lfp,
                    const orbmi_mappoint* mps, int n_mp, const float* inv_level_sigma2, float th, int* match_lf,
                    int* match_mp, uint8_t* outlier, float* tcw_mm, float* tcw, int* stats) {
    const int n = CF->n;
    std::vector<uint8_t> occ(n + 1, 0);
    for (int i = 0; i < n; i++) { match_mp[i] = -1; outlier[i] = 0; }
    memcpy(tcw_mm, CF->tcw, 16 * sizeof(float));
    memcpy(tcw, CF->tcw, 16 * sizeof(float));
    stats[0] = stats[1] = stats[2] = stats[3] = 0;
    int nm = 0;
    orc_search_by_projection_last_frame(CF, occ.data(), LF, lfp, th, 0, 1, match_lf, &nm);
    if (nm < 20) orc_search_by_projection_last_frame(CF, occ.data(), LF, lfp, 2 * th, 0, 1, match_lf, &nm);
    stats[0] = nm;
    if (nm < 20) return 0;
    orbmi_frame_mappoints mp{match_lf, lfp, LF->n, nullptr, mps, n_mp};
    orbmi_pose_frame rec;
    orc_pose_optimization_frame(CF, inv_level_sigma2, &mp, &rec, outlier);
    memcpy(tcw_mm, rec.tcw, sizeof(rec.tcw));
    int cnt[2];
    orc_track_update_matches(CF, 0, outlier, &mp, occ.data(), cnt);
    stats[1] = cnt[1];
    if (cnt[1] < 10) return 0;
    // TrackLocalMap at the optimised pose
    orbmi_frame_view F2 = *CF;
    F2.tcw = rec.tcw;
    std::vector<orbmi_mappoint_track> tr(n_mp + 1);
    orc_is_in_frustum(&F2, mps, n_mp, 0.5f, tr.data());
    for (int k = 0; k < n_mp; k++) stats[3] += tr[k].in_view;
    int nl = 0;
    if (stats[3] > 0) orc_search_by_projection_local(&F2, occ.data(), mps, tr.data(), n_mp, 1.0f, 0.8f, match_mp, &nl);
    mp.match_mp = match_mp;
    orbmi_pose_frame rec2;
    orc_pose_optimization_frame(&F2, inv_level_sigma2, &mp, &rec2, outlier);
    memcpy(tcw, rec2.tcw, sizeof(rec2.tcw));
    orc_track_update_matches(&F2, 1, outlier, &mp, nullptr, cnt);
    stats[2] = cnt[0];
    return cnt[0] >= 30 ? 1 : 0;
}

}  // extern "C"
