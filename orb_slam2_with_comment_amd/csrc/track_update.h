// Tracking's pass over mvpMapPoints after a PoseOptimization, as a workgroup routine: the body
// of k_track_update (orbmi_track_update_matches) and the tail of k_pose_opt when the two run
// as one launch (orbmi_pose_optimization_frame_track).
//   stage 0 = TrackWithMotionModel "Discard outliers" (src/Tracking.cc:1036-1058)
//   stage 1 = TrackLocalMap statistics (src/Tracking.cc:1085-1104)
// Keypoint i's point is the local map point when match_mp[i] >= 0, else the last-frame point
// when match_lf[i] >= 0 (out-of-range indices read as NULL).
#pragma once
#include "orbmi_common.h"

namespace orbmi {

// Every thread of the workgroup calls it (two barriers inside); cnt = two ints of LDS.
__device__ inline void track_update_body(int n, bool stereo, int stage, const uint8_t* __restrict__ outlier,
                                         int* __restrict__ match_lf, const orbmi_lastframe_point* __restrict__ lfp,
                                         int n_lf, int* __restrict__ match_mp,
                                         const orbmi_mappoint* __restrict__ mps, int n_mp,
                                         uint8_t* __restrict__ occ_out, int* __restrict__ counts, int* cnt) {
    if (threadIdx.x < 2) cnt[threadIdx.x] = 0;
    __syncthreads();
    int c0 = 0, c1 = 0;
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        int* slot = nullptr;
        bool obs = false;
        if (match_mp && match_mp[i] >= 0 && match_mp[i] < n_mp) {
            slot = &match_mp[i];
            obs = (mps[*slot].flags & ORBMI_MP_HAS_OBS) != 0;
        } else if (match_lf && match_lf[i] >= 0 && match_lf[i] < n_lf) {
            slot = &match_lf[i];
            obs = (lfp[*slot].flags & ORBMI_MP_HAS_OBS) != 0;
        }
        bool occ = false;
        if (slot) {
            const bool out = outlier[i] != 0;
            if (stage == 0) {          // :1042-1055
                if (out) { *slot = -1; c0++; }
                else if (obs) { c1++; occ = true; }
            } else {                   // :1087-1101
                if (!out) c0 += obs;
                else { c1++; if (stereo) *slot = -1; }
            }
        }
        if (occ_out) occ_out[i] = occ;
    }
    if (c0) atomicAdd(&cnt[0], c0);
    if (c1) atomicAdd(&cnt[1], c1);
    __syncthreads();
    if (threadIdx.x < 2) counts[threadIdx.x] = cnt[threadIdx.x];
}

}  // namespace orbmi
