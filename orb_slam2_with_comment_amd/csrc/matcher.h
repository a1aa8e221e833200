// Host-side state of the device matchers (matcher.hip, capi_match.cpp).
#pragma once
#include <vector>

#include "extractor.h"

namespace orbmi {

// Frame view resolved to device pointers; pose and scale tables travel by value.
struct DevFrame {
    int n;                 // capacity when n_dev is set
    const int* n_dev;      // device-resident count (optional)
    const orbmi_keypoint* keys;
    const float* u_right;
    const uint8_t* desc;
    float tcw[16];         // host pose (by value) ...
    const float* tcw_dev;  // ... or a device pose read when the kernel runs
    float fx, fy, cx, cy, bf, mb;
    float min_x, max_x, min_y, max_y, grid_w_inv, grid_h_inv;
    int nlevels;
    float scale[kMaxLevels];
    float log_scale_factor;
};

__device__ inline int frame_n(const DevFrame& F) { return F.n_dev ? min(*F.n_dev, F.n) : F.n; }

// Rows 0-2 of Tcw (12 floats, constant indices: registers).
struct Pose34 { float m[12]; };
__device__ inline Pose34 frame_pose(const DevFrame& F) {
    Pose34 T;
    if (F.tcw_dev) {
#pragma unroll
        for (int k = 0; k < 12; k++) T.m[k] = F.tcw_dev[k];
    } else {
#pragma unroll
        for (int k = 0; k < 12; k++) T.m[k] = F.tcw[k];
    }
    return T;
}

struct DevFV {
    int nnodes;
    const uint32_t* node_id;
    const int32_t* off;
    const int32_t* feat;
};

struct Mat3f { float m[9]; };  // row-major 3x3 (by value)

// One (KF1, KF2) pair of SearchForTriangulation, read by the kernels from device memory so that
// one launch serves all of a keyframe's neighbours (grid row = pair)
struct TriPair {
    DevFrame KF2;
    const uint8_t* has_mp2;
    DevFV fv2;
    Mat3f F12;
    int* match;     // KF1.n entries
    int* bin_of;    // KF1.n entries (rotation bins)
    int* hist;      // HISTO_LENGTH
    int* nmatches;  // one int (may be null)
};

// One keyframe of a batched Fuse search (grid row = keyframe): its frame, grid and outputs
struct FuseKF {
    DevFrame F;
    const int* cs;          // cell_start (kGridCells + 1)
    const int* cl;          // cell_list
    const uint8_t* in_kf;   // IsInKeyFrame per candidate (may be null)
    int* best_idx;          // n candidates
    int* best_dist;
    int* ncand;             // one int
};

struct Matcher {
    static constexpr int kCandCap = 96;  // candidates kept per query; overflow re-enumerates
    int device = 0;
    hipStream_t stream = nullptr;
    bool own_stream = true;
    // grid
    int* d_cell_start = nullptr; size_t cap_cell_start = 0;
    int* d_cell_list = nullptr; size_t cap_cell_list = 0;
    int* d_kp_cell = nullptr; size_t cap_kp_cell = 0;
    // grids of several keyframes (batched Fuse)
    int* d_mcell_start = nullptr; size_t cap_mcell_start = 0;
    int* d_mcell_list = nullptr; size_t cap_mcell_list = 0;
    int* d_mkp_cell = nullptr; size_t cap_mkp_cell = 0;
    // grid pinned to one frame by orbmi_matcher_assign_features_to_grid (device keypoints only):
    // searches on that frame skip the rebuild until the pin is released or another frame's grid
    // is built
    bool grid_pinned = false;
    const orbmi_keypoint* pin_keys = nullptr;
    const int* pin_ndev = nullptr;
    int pin_n = 0;
    float pin_geom[6] = {};
    // the grid the searches read: the one built above, or a slot grid pinned by
    // orbmi_matcher_pin_grid_slot
    const int* cur_cs = nullptr;
    const int* cur_cl = nullptr;
    // slot grids (orbmi_matcher_build_grid_slot): built on another stream (the extraction's)
    // ahead of the searches; each remembers the frame it was built for
    static constexpr int kGridSlots = 4;
    struct GridSlot {
        int* cs = nullptr;
        int* cl = nullptr;
        int* kc = nullptr;
        size_t cap = 0;
        bool built = false;
        const orbmi_keypoint* keys = nullptr;
        const int* ndev = nullptr;
        int n = 0;
        float geom[6] = {};
    } gslot[kGridSlots];
    // candidates / greedy
    unsigned long long* d_cand = nullptr; size_t cap_cand = 0;
    int* d_ncand = nullptr; size_t cap_ncand = 0;
    unsigned long long* d_top = nullptr; size_t cap_top = 0;
    int* d_res = nullptr; size_t cap_res = 0;
    int* d_bin_of = nullptr; size_t cap_bin_of = 0;
    int* d_hist = nullptr; size_t cap_hist = 0;
    int* d_scalars = nullptr; size_t cap_scalars = 0;   // small per-call outputs
    orbmi_mappoint_track* d_track = nullptr; size_t cap_track = 0;  // fused frustum output
    // staging arena for host inputs/outputs, in kArenaGens generations: each call stages into
    // the next generation, and waits only when that generation's last use (an event recorded
    // when the call after it began) has not finished -- so back-to-back asynchronous calls with
    // host inputs do not serialise on the host
    // Every block has a pinned host mirror of the same size: host inputs are copied into the
    // mirror and DMA'd from there, host outputs DMA'd into it and copied out after the call's
    // wait (pageable hipMemcpyAsync goes through the runtime's own staging, one blocking chunked
    // copy per array).  The mirror is reused with its block, under the same generation events.
    static constexpr int kArenaGens = 4;
    struct Block { uint8_t* p; size_t size, used; uint8_t* h; };
    struct Gen { std::vector<Block> blocks; hipEvent_t ev = nullptr; bool pending = false; };
    Gen gens[kArenaGens];
    int gen = 0;
    struct Pend { void* user; const uint8_t* mirror; size_t bytes; };
    std::vector<Pend> pend;  // device-to-host copies landing in mirrors, copied out by d2h_flush
    void* stage(size_t bytes);
    uint8_t* mirror(const void* d);  // host mirror of a staged device address, else nullptr
    hipError_t h2d(void* d, const void* src, size_t bytes);    // stream-ordered upload
    hipError_t d2h(void* user, const void* d, size_t bytes);   // stream-ordered read-back
    // Consecutive uploads into adjacent staging allocations go to the device as one copy: h2d
    // fills the mirror and extends the pending range; ls() (the stream for any enqueue: launch,
    // copy, wait) sends it first.  Each copy on the stream is a blit dispatch of several
    // microseconds, and a call stages 2-6 inputs.
    struct PendUp { uint8_t* d = nullptr; uint8_t* h = nullptr; size_t n = 0; } up;
    hipError_t up_err = hipSuccess;
    hipError_t flush_up();
    hipStream_t ls() {
        if (up.n) (void)flush_up();
        return stream;
    }
    void d2h_flush();                                          // after the stream's wait
    void arena_reset();
    void release();
};

int pin_grid(Matcher& m, const DevFrame& F);
int build_grid_slot(Matcher& m, const DevFrame& F, int k, hipStream_t s);
int pin_grid_slot(Matcher& m, const DevFrame& F, int k);
int launch_frustum(Matcher& m, const DevFrame& F, const orbmi_mappoint* mps, int n, float cosl,
                   orbmi_mappoint_track* tr, int* n_in_view);
int launch_local_search(Matcher& m, const DevFrame& F, const uint8_t* occ0, const orbmi_mappoint* mps,
                        const orbmi_mappoint_track* tr, int n, float th, float nnratio, int* out, int* nmatches);
int launch_lastframe_search(Matcher& m, const DevFrame& CF, const uint8_t* occ0, const DevFrame& LF,
                            const orbmi_lastframe_point* lfp, float th, int mono, int check_ori, int* out,
                            int* nmatches, const int* gate = nullptr, int gate_min = 0);
int launch_track_update(Matcher& m, const DevFrame& F, int stage, const uint8_t* outlier, int* match_lf,
                        const orbmi_lastframe_point* lfp, int n_lf, int* match_mp, const orbmi_mappoint* mps,
                        int n_mp, uint8_t* occ_out, int* counts);
int launch_bow(Matcher& m, const DevFrame& KF, const uint8_t* kf_ok, const DevFV& kfv, const DevFrame& F,
               const DevFV& fv, float nnratio, int check_ori, int* match, int* nmatches);
int launch_triangulation(Matcher& m, const DevFrame& KF1, const uint8_t* has_mp1, const DevFV& fv1, int npairs,
                         TriPair* pairs_host, TriPair* pairs_dev, int only_stereo, int check_ori, int* match);
namespace tri { struct Side; }
int tri_pairs_prepare(Matcher& m, const DevFrame& KF1, int npairs, TriPair* pairs_host, int* match);
// pairs_host == nullptr: the pair table is already prepared (tri_pairs_prepare) and uploaded
int launch_create_points(Matcher& m, const DevFrame& KF1, const uint8_t* has1, const DevFV& fv1, int npairs,
                         TriPair* pairs_host, TriPair* pairs_dev, const tri::Side& S1, const tri::Side* S2_dev,
                         int* match, uint8_t* ok, float* x3d);
int launch_fuse(Matcher& m, const DevFrame& F, const orbmi_mappoint* mps, const uint8_t* in_kf, int n, float th,
                int* best_idx, int* best_dist, int* ncand);
int launch_fuse_multi(Matcher& m, int nkf, FuseKF* kfs_host, FuseKF* kfs_dev, const orbmi_mappoint* mps, int n,
                      float th, int* best_idx, int* best_dist, int* ncand);
int launch_patch_desc(Matcher& m, orbmi_mappoint* mps, const int* desc_from, const uint8_t* desc, int n);
int greedy_stats(unsigned long long out[5], int reset);
int greedy_cycles(unsigned long long out[7], int reset);
int launch_distinctive(Matcher& m, const uint8_t* desc, const int* off, int np, int* best, uint8_t* out);
int launch_xmatch(Matcher& m, const uint8_t* qd, int nq_cap, const int* nq_dev, const uint8_t* td, int nseg,
                  int seg_cap, const int* seg_counts, int skip_seg, int th, float ratio, int* match, int* nmatches);

}  // namespace orbmi
