// Native stereo SLAM host loop: System::TrackStereo, the stereo Tracking state machine and a
// synchronous LocalMapping around the MI355X operators of this library (include/orbmi.h).
//
//   System::TrackStereo        -> orbmi_slam_track_stereo         src/System.cc:110-159
//   Tracking::Track (stereo)   -> Slam::track                     src/Tracking.cc:287-581
//   StereoInitialization       -> Slam::stereo_initialization     src/Tracking.cc:584-636
//   TrackReferenceKeyFrame     -> Slam::track_reference_kf        src/Tracking.cc:871-917
//   TrackWithMotionModel       -> Slam::track_motion_model        src/Tracking.cc:997-1063
//   TrackLocalMap, UpdateLocalKeyFrames / Points, SearchLocalPoints src/Tracking.cc:1075-1104, 1345-1580
//   NeedNewKeyFrame / CreateNewKeyFrame                           src/Tracking.cc:1140-1330
//   LocalMapping::Run: ProcessNewKeyFrame, MapPointCulling, CreateNewMapPoints,
//     SearchInNeighbors (ORBmatcher::Fuse + replay), LocalBundleAdjustment, KeyFrameCulling
//                                                                 src/LocalMapping.cc:47-841
//   KeyFrame::UpdateConnections, MapPoint bookkeeping             src/KeyFrame.cc, src/MapPoint.cc
//   Optimizer::LocalBundleAdjustment's graph assembly             src/Optimizer.cc:486-683
//   System::SaveTrajectoryKITTI / TUM / SaveKeyFrameTrajectoryTUM src/System.cc:334-486
//
// The same host logic as orb_slam2_with_comment_amd/system.py (which the tests also drive with
// the CPU oracle behind it); this native form is what --mode system measures.  Pose algebra in
// float32 with double accumulation (cv::Mat CV_32F products, src/Converter.cc); the
// deterministic replacements of the reference's pointer-ordered containers are the Python
// module's: keyframe-id order for std::map<KeyFrame*, ...>, covisibility ties to the higher id.
// Compiled with -ffp-contract=off: one rounding per float operation, as numpy does.
#include <algorithm>
#include <array>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <deque>
#include <mutex>
#include <thread>
#include <type_traits>
#include <cstdio>
#include <cstring>
#include <map>
#include <new>
#include <set>
#include <stdexcept>
#include <utility>
#include <vector>

#include <hip/hip_runtime_api.h>

#include "../../include/orbmi.h"
#include "../../include/orbmi_debug.h"
#include "tri_geom.h"

namespace {

using M4 = std::array<float, 16>;

M4 eye4() {
    M4 m{};
    m[0] = m[5] = m[10] = m[15] = 1.f;
    return m;
}

// float32(float64(a) @ float64(b)), 4x4 row-major
M4 mul(const M4& a, const M4& b) {
    M4 o;
    for (int r = 0; r < 4; r++)
        for (int c = 0; c < 4; c++) {
            double s = 0;
            for (int k = 0; k < 4; k++) s += (double)a[4 * r + k] * (double)b[4 * k + c];
            o[4 * r + c] = (float)s;
        }
    return o;
}

// Frame::UpdatePoseMatrices: Rwc = Rcw^T, Ow = -Rwc tcw; Twc as a 4x4
M4 pose_inverse(const M4& T) {
    M4 o = eye4();
    for (int r = 0; r < 3; r++)
        for (int c = 0; c < 3; c++) o[4 * r + c] = T[4 * c + r];
    for (int r = 0; r < 3; r++) {
        double s = 0;
        for (int k = 0; k < 3; k++) s += (double)o[4 * r + k] * (double)T[4 * k + 3];
        o[4 * r + 3] = -(float)s;
    }
    return o;
}

void camera_center(const M4& T, float ow[3]) {
    const M4 i = pose_inverse(T);
    ow[0] = i[3]; ow[1] = i[7]; ow[2] = i[11];
}

// Converter::toQuaternion (src/Converter.cc:137-149): Eigen::Quaterniond(Matrix3d) -> x y z w
void quaternion_xyzw(const float R[9], float q_out[4]) {
    double m[3][3], q[4] = {0, 0, 0, 0};
    for (int r = 0; r < 3; r++)
        for (int c = 0; c < 3; c++) m[r][c] = R[3 * r + c];
    double t = m[0][0] + m[1][1] + m[2][2];
    if (t > 0) {
        t = std::sqrt(t + 1.0);
        q[3] = 0.5 * t;
        t = 0.5 / t;
        q[0] = (m[2][1] - m[1][2]) * t;
        q[1] = (m[0][2] - m[2][0]) * t;
        q[2] = (m[1][0] - m[0][1]) * t;
    } else {
        int i = m[1][1] > m[0][0] ? 1 : 0;
        if (m[2][2] > m[i][i]) i = 2;
        const int j = (i + 1) % 3, k = (i + 2) % 3;
        t = std::sqrt(m[i][i] - m[j][j] - m[k][k] + 1.0);
        q[i] = 0.5 * t;
        t = 0.5 / t;
        q[3] = (m[k][j] - m[j][k]) * t;
        q[j] = (m[j][i] + m[i][j]) * t;
        q[k] = (m[k][i] + m[i][k]) * t;
    }
    for (int k = 0; k < 4; k++) q_out[k] = (float)q[k];
}

// DBoW2::FeatureVector as CSR (orbmi_feature_vector)
struct FeatVec {
    bool valid = false;
    int words = 0;  // the BowVector's word count (kept for the per-keyframe state record)
    std::vector<uint32_t> node;
    std::vector<int32_t> off, feat;
    orbmi_feature_vector view() const {
        return orbmi_feature_vector{(int)node.size(), node.data(), off.data(), feat.data()};
    }
};

struct KeyFrame {
    int id = 0, frame_id = 0;
    double ts = 0;
    M4 tcw{};
    std::vector<orbmi_keypoint> keys;
    std::vector<uint8_t> desc;
    std::vector<float> ur, depth;
    std::vector<int> mps;        // map point id per keypoint, -1 = NULL
    FeatVec fv;
    std::vector<int> covisible;  // mvpOrderedConnectedKeyFrames
    std::map<int, int> conn;     // mConnectedKeyFrameWeights (keyframe id order)
    int parent = -1;
    std::vector<int> children;   // mspChildrens (iterated in id order)
    bool first_connection = true;
    bool bad = false;
    int fuse_target_for_kf = -1;  // mnFuseTargetForKF
    M4 tcp{};                    // mTcp, set when the keyframe turns bad
    // device copies of keys / desc / u_right (one block): the searches read the keyframe in place
    uint8_t* d_block = nullptr;
    const orbmi_keypoint* d_keys = nullptr;
    const uint8_t* d_desc = nullptr;
    const float* d_ur = nullptr;
    const float* d_depth = nullptr;
    const float* d_cos = nullptr;  // orbmi_stereo_parallax_cos per keypoint (CreateNewMapPoints)
};

// MapPoint::mObservations (keyframe id -> keypoint index, keyframe-id order) as a sorted flat
// vector: a map point has a handful of observations, and the tracking thread walks them for every
// matched point each frame (UpdateLocalKeyFrames), which node-based std::map made pointer chases
struct ObsMap {
    using Entry = std::pair<int, int>;
    std::vector<Entry> v;
    using iterator = std::vector<Entry>::iterator;
    using const_iterator = std::vector<Entry>::const_iterator;
    iterator begin() { return v.begin(); }
    iterator end() { return v.end(); }
    const_iterator begin() const { return v.begin(); }
    const_iterator end() const { return v.end(); }
    size_t size() const { return v.size(); }
    bool empty() const { return v.empty(); }
    void clear() { v.clear(); }
    iterator lower(int k) {
        return std::lower_bound(v.begin(), v.end(), k, [](const Entry& e, int x) { return e.first < x; });
    }
    const_iterator lower(int k) const {
        return std::lower_bound(v.begin(), v.end(), k, [](const Entry& e, int x) { return e.first < x; });
    }
    iterator find(int k) {
        auto it = lower(k);
        return it != v.end() && it->first == k ? it : v.end();
    }
    const_iterator find(int k) const {
        auto it = lower(k);
        return it != v.end() && it->first == k ? it : v.end();
    }
    size_t count(int k) const { return find(k) != v.end() ? 1 : 0; }
    int& operator[](int k) {
        auto it = lower(k);
        if (it == v.end() || it->first != k) it = v.insert(it, Entry{k, 0});
        return it->second;
    }
    const int& at(int k) const {
        auto it = find(k);
        if (it == v.end()) throw std::out_of_range("ObsMap::at");
        return it->second;
    }
    iterator erase(iterator it) { return v.erase(it); }
};

struct MapPoint {
    int id = 0;
    float pos[3] = {0, 0, 0};
    int ref_kf = -1;
    uint8_t desc[32] = {};
    float normal[3] = {0, 0, 0};
    float max_distance = 0, min_distance = 0;
    ObsMap obs;                  // keyframe id -> keypoint index (keyframe id order)
    int nobs = 0;
    bool bad = false;
    int first_kf_id = 0;         // mnFirstKFid
    int visible = 1, found = 1;  // mnVisible, mnFound
    int replaced = -1;           // mpReplaced
    int fuse_candidate_for_kf = -1;
};
// The mapping thread's device calls read keyframes' FeatureVectors through host pointers with the
// map lock released, while Tracking may append to `kfs`: a reallocation must move the elements
// (their heap arrays stay put), never copy and free them.
static_assert(std::is_nothrow_move_constructible<KeyFrame>::value, "kfs growth would copy keyframes");
static_assert(std::is_nothrow_move_constructible<FeatVec>::value, "FeatVec growth would copy");

struct TrackedFrame {
    int id = 0;
    double ts = 0;
    std::vector<orbmi_keypoint> keys;
    std::vector<uint8_t> desc;
    std::vector<float> ur, depth;
    bool has_tcw = false;
    M4 tcw{};
    std::vector<int> mps;        // mvpMapPoints (map point ids, -1)
    std::vector<uint8_t> outlier;
    int ref_kf = -1;
    FeatVec fv;
    int dslot = -1;              // device slot holding keys / desc / u_right (orbmi_slam::Dev)
    int n() const { return (int)keys.size(); }
};

enum { NO_IMAGES_YET = 0, NOT_INITIALIZED = 1, OK = 2, LOST = 3 };

// wall time per phase of orbmi_slam_track_stereo (orbmi_slam_get_phase_ms; names in orbmi_debug.h)
enum Phase { PH_FRAME, PH_LOCK, PH_LF_SEARCH, PH_LF_POSE, PH_LOCAL_UPDATE, PH_LOCAL_RECORDS, PH_FRUSTUM,
             PH_LOCAL_SEARCH, PH_LOCAL_POSE, PH_KEYFRAME, PH_TOTAL,
             // LocalMapping::Run per keyframe (either thread): ProcessNewKeyFrame, MapPointCulling,
             // CreateNewMapPoints, SearchInNeighbors, LocalBundleAdjustment, KeyFrameCulling, all
             PH_LM_PROCESS, PH_LM_CULL, PH_LM_CREATE, PH_LM_FUSE, PH_LM_BA, PH_LM_KFCULL, PH_LM_TOTAL,
             // inside them: the device calls of CreateNewMapPoints, of the Fuse searches, and of
             // ComputeDistinctiveDescriptors (each with its staging and read-back)
             PH_LM_CREATE_CALL, PH_LM_FUSE_CALL, PH_LM_DISTINCTIVE_CALL,
             // the mapping thread's host work, finer: waits to re-take the map lock after a device
             // call; SearchInNeighbors' set-up (targets, records), its per-target check of changed
             // records, its Fuse replays; UpdateNormalAndDepth loops; UpdateConnections; the
             // observation rows of ComputeDistinctiveDescriptors; LocalBA's graph assembly, its
             // device call, its write-back
             PH_LM_LOCK, PH_LM_SIN_PREP, PH_LM_SIN_REDO, PH_LM_SIN_REPLAY, PH_LM_NORMALS, PH_LM_CONNECTIONS,
             PH_LM_OBSROWS, PH_LM_BA_GATHER, PH_LM_BA_CALL, PH_LM_BA_WRITEBACK, PH_COUNT };
struct PhaseTimer {
    double* acc;
    std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
    explicit PhaseTimer(double* a) : acc(a) {}
    ~PhaseTimer() { *acc += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count(); }
};

#define SLAM_CHECK(call)              \
    do {                              \
        const int rc_ = (call);       \
        if (rc_ != ORBMI_OK) return rc_; \
    } while (0)

// this thread's hold on its system's map_mtx when the GPU calls may release it (the mapping
// thread, and the tracking thread with the mapping thread running); null otherwise
thread_local std::unique_lock<std::mutex>* held_lock = nullptr;
thread_local bool on_mapping_thread = false;

}  // namespace

struct orbmi_slam {
    orbmi_slam_settings s{};
    int device = 0;
    orbmi_extractor* left = nullptr;
    orbmi_extractor* right = nullptr;
    orbmi_matcher* matcher = nullptr;
    orbmi_pose* pose = nullptr;
    orbmi_ba* ba = nullptr;
    orbmi_vocabulary* voc = nullptr;
    std::vector<float> scale_factors, inv_level_sigma2;
    float log_scale_factor = 0;

    int state = NO_IMAGES_YET;
    std::vector<KeyFrame> kfs;   // index = keyframe id
    std::vector<MapPoint> mps;   // index = map point id
    int frame_count = 0;
    TrackedFrame last_frame;
    bool have_last = false;
    bool has_velocity = false;
    M4 velocity{};
    int ref_kf = -1;
    int last_kf_frame_id = 0, last_reloc_frame_id = 0;
    std::vector<int> local_kfs, local_mps;
    int matches_inliers = 0;
    // mnLastFrameSeen == current frame, as a generation stamp per map point (O(1) insert / test /
    // clear instead of a std::set over thousands of points per frame)
    struct SeenSet {
        std::vector<int> mark;
        int gen = 1;
        void clear() { gen++; }
        void insert(int m) {
            if (m >= (int)mark.size()) mark.resize(std::max<size_t>(2 * mark.size(), m + 1), 0);
            mark[m] = gen;
        }
        bool count(int m) const { return m < (int)mark.size() && mark[m] == gen; }
    } seen;
    SeenSet local_mark;           // UpdateLocalPoints' mnTrackReferenceForFrame
    SeenSet local_kf_mark;        // UpdateLocalKeyFrames' mnTrackReferenceForFrame
    // LocalBundleAdjustment's mnBALocalForKF / mnBAFixedForKF and its points' marks (the mapping
    // thread's; generation stamps instead of std::set)
    SeenSet ba_local_mark, ba_fixed_mark, ba_mp_mark;
    // the points whose Fuse search record a replay may have changed (fuse_targets' check)
    SeenSet fuse_touched;
    std::vector<int> kf_counter;  // UpdateLocalKeyFrames' keyframe counter (indexed by id)
    // mlRelativeFramePoses, mlpReferences, mlFrameTimes, mlbLost
    std::vector<M4> rel_poses;
    std::vector<int> references;
    std::vector<double> frame_times;
    std::vector<uint8_t> lost;
    std::vector<orbmi_slam_frame_stats> stats;
    int ba_calls = 0;
    // LocalMapping::Run outcomes (orbmi_slam_get_local_mapping_counts): jobs, SearchInNeighbors
    // and LocalBA skipped because a keyframe was queued (src/LocalMapping.cc:79-90), LocalBAs that
    // saw mbAbortBA while optimising / before starting
    int lm_jobs = 0, sin_skipped = 0, ba_skipped = 0, ba_interrupted = 0, ba_aborted = 0;
    int resets = 0;  // Tracking::Reset calls (lost with <= 5 keyframes in the map)
    std::vector<float> level_sigma2;  // mvLevelSigma2
    std::vector<int> recent_mps;      // mlpRecentAddedMapPoints
    // extraction scratch
    std::vector<orbmi_keypoint> kbuf;
    std::vector<uint8_t> dbuf;
    // Device-resident frames: the image pair goes up once, both images are extracted as one
    // batch with the stereo match behind them on the extractor's stream, and the outputs stay
    // in one of three slots (current frame, last frame, the next frame's extraction running
    // ahead), so the searches and the pose optimisations read the frames in place instead of
    // staging them per call; the host gets its copy of the left outputs with one read-back.
    static constexpr int kSlots = 3;
    struct Dev {
        uint8_t* img = nullptr;  // 2 x rows x cols
        size_t img_bytes = 0;
        uint8_t* h_img = nullptr;  // pinned staging of the pair
        int cap = 0;               // keypoints per item
        orbmi_keypoint* kps[kSlots] = {};
        uint8_t* desc[kSlots] = {};
        int* cnt[kSlots] = {};
        float* ur[kSlots] = {};
        float* dep[kSlots] = {};
        // A slot is chosen per extraction (free_slot): never the current frame's nor the last
        // frame's, which tracking reads on its stream while the next pair is extracted
        // the extraction enqueued ahead (orbmi_slam_track_stereo_ahead) and not yet collected
        struct Ahead { bool on = false; int slot = -1, rows = 0, cols = 0; size_t step = 0; const uint8_t *L = nullptr, *R = nullptr; } ahead;
        // pinned host mirror of a slot's left outputs
        orbmi_keypoint* h_kps = nullptr;
        uint8_t* h_desc = nullptr;
        int* h_cnt = nullptr;
        float* h_ur = nullptr;
        float* h_dep = nullptr;
    } dev;
    hipStream_t xstream = nullptr;  // the left extractor's stream
    // The next pair's Frame-constructor work (image staging, the extraction and stereo launches,
    // the read-back copies: frame_enqueue) runs on a helper thread while the tracking thread
    // tracks the current frame; track_stereo joins it before returning, so the caller's next
    // images are never read after the call.  ORBMI_SLAM_INLINE_FRAME=1: on the tracking thread.
    struct FrameWorker {
        std::thread th;
        std::mutex mtx;
        std::condition_variable cv;
        bool job = false, busy = false, quit = false;
        int rc = ORBMI_OK;
        const uint8_t *L = nullptr, *R = nullptr;
        int rows = 0, cols = 0;
        size_t step = 0;
        int slot = -1;
    } fw;
    const bool inline_frame = getenv("ORBMI_SLAM_INLINE_FRAME") != nullptr;
    void frame_worker_run() {
        (void)hipSetDevice(device);  // the current device is per thread
        std::unique_lock<std::mutex> g(fw.mtx);
        for (;;) {
            fw.cv.wait(g, [this] { return fw.job || fw.quit; });
            if (fw.quit) return;
            fw.job = false;
            g.unlock();
            const int rc = frame_enqueue(fw.L, fw.R, fw.rows, fw.cols, fw.step, fw.slot);
            g.lock();
            fw.rc = rc;
            fw.busy = false;
            fw.cv.notify_all();
        }
    }
    void frame_post(const uint8_t* L, const uint8_t* R, int rows, int cols, size_t step, int slot) {
        std::lock_guard<std::mutex> g(fw.mtx);
        if (!fw.th.joinable()) fw.th = std::thread([this] { frame_worker_run(); });
        fw.L = L; fw.R = R; fw.rows = rows; fw.cols = cols; fw.step = step; fw.slot = slot;
        fw.job = true;
        fw.busy = true;
        fw.rc = ORBMI_OK;
        fw.cv.notify_all();
    }
    int frame_join() {  // the posted enqueue finished; its status
        std::unique_lock<std::mutex> g(fw.mtx);
        fw.cv.wait(g, [this] { return !fw.busy; });
        const int rc = fw.rc;
        fw.rc = ORBMI_OK;
        return rc;
    }
    void frame_worker_stop() {
        if (!fw.th.joinable()) return;
        (void)frame_join();
        {
            std::lock_guard<std::mutex> g(fw.mtx);
            fw.quit = true;
            fw.cv.notify_all();
        }
        fw.th.join();
    }
    // Device-resident tracking stages: TrackWithMotionModel (SearchByProjection(CF, LF) with the
    // retry gated on the device count, PoseOptimization on the device-held matches) and
    // TrackLocalMap (SearchLocalPoints, PoseOptimization over both match arrays) are each enqueued
    // on the tracking stream (the matcher's, shared with PoseOptimization) behind one upload of
    // the records the host builds, and read back with one synchronisation.  Host arrays are
    // pinned, so the copies are plain DMA.
    struct TrackBuf {
        size_t cap_kp = 0, cap_lf = 0, cap_rec = 0;
        // One device arena and its pinned host mirror, laid out so that each tracking stage moves
        // its inputs in one upload and its results in one read-back (every copy is a queue
        // packet of several microseconds on the stream):
        //   rec | mlf | occ | lfp | n | pose | out | m | tr
        // TrackWithMotionModel uploads occ .. n (n zeroed: the first search's gate) and reads
        // n .. m; TrackLocalMap uploads rec .. lfp and reads n .. tr.
        uint8_t* d_arena = nullptr;
        uint8_t* h_arena = nullptr;
        size_t arena_bytes = 0;
        // device
        orbmi_lastframe_point* d_lfp = nullptr;  // TWMM: the last frame's points / TLM: the current frame's
        orbmi_mappoint* d_rec = nullptr;         // TLM: the local map points
        orbmi_mappoint_track* d_tr = nullptr;
        int32_t* d_m = nullptr;                  // matches (TWMM: to LF keypoints; TLM: to local map points)
        int32_t* d_mlf = nullptr;                // TLM: keypoint -> its own point record (or -1)
        uint8_t* d_occ = nullptr;
        uint8_t* d_out = nullptr;                // mvbOutlier
        int* d_n = nullptr;                      // match count
        orbmi_pose_frame* d_pose = nullptr;
        // pinned host
        orbmi_lastframe_point* h_lfp = nullptr;
        orbmi_mappoint* h_rec = nullptr;
        orbmi_mappoint_track* h_tr = nullptr;
        int32_t* h_m = nullptr;
        int32_t* h_mlf = nullptr;
        uint8_t* h_occ = nullptr;
        uint8_t* h_out = nullptr;
        int* h_n = nullptr;
        orbmi_pose_frame* h_pose = nullptr;
    } tb;
    hipStream_t tstream = nullptr;  // the tracking stream (the matcher's)

    int track_buffers(size_t nkp, size_t nlf, size_t nrec) {
        nkp = std::max<size_t>(nkp, 1);
        nlf = std::max<size_t>(nlf, 1);
        nrec = std::max<size_t>(nrec, 1);
        TrackBuf& t = tb;
        if (nkp <= t.cap_kp && nlf <= t.cap_lf && nrec <= t.cap_rec && t.d_arena) return ORBMI_OK;
        if (nkp > t.cap_kp) t.cap_kp = nkp + nkp / 4;
        if (nlf > t.cap_lf) t.cap_lf = nlf + nlf / 4;
        if (nrec > t.cap_rec) t.cap_rec = nrec + nrec / 4;
        auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
        size_t off = 0;
        auto take = [&](size_t bytes) { const size_t o = off; off += al(bytes); return o; };
        const size_t o_rec = take(t.cap_rec * sizeof(orbmi_mappoint)), o_mlf = take(t.cap_kp * 4), o_occ = take(t.cap_kp);
        const size_t o_lfp = off;  // (no padding between lfp and n: TWMM's upload ends right after n)
        off += t.cap_lf * sizeof(orbmi_lastframe_point);
        off = (off + 15) & ~(size_t)15;
        const size_t o_n = take(2 * sizeof(int)), o_pose = take(sizeof(orbmi_pose_frame)), o_out = take(t.cap_kp),
                     o_m = take(t.cap_kp * 4), o_tr = take(t.cap_rec * sizeof(orbmi_mappoint_track));
        if (off > t.arena_bytes) {
            if (t.d_arena) (void)hipFree(t.d_arena);
            if (t.h_arena) (void)hipHostFree(t.h_arena);
            t.d_arena = t.h_arena = nullptr;
            t.arena_bytes = 0;
            if (hipMalloc((void**)&t.d_arena, off) != hipSuccess) return ORBMI_E_HIP;
            if (hipHostMalloc((void**)&t.h_arena, off, hipHostMallocDefault) != hipSuccess) return ORBMI_E_HIP;
            t.arena_bytes = off;
        }
        auto at = [&](uint8_t* base, size_t o) { return (void*)(base + o); };
        for (int side = 0; side < 2; side++) {
            uint8_t* B = side ? t.h_arena : t.d_arena;
            auto& rec = side ? t.h_rec : t.d_rec;
            auto& mlf = side ? t.h_mlf : t.d_mlf;
            auto& occ = side ? t.h_occ : t.d_occ;
            auto& lfp = side ? t.h_lfp : t.d_lfp;
            auto& n = side ? t.h_n : t.d_n;
            auto& pose = side ? t.h_pose : t.d_pose;
            auto& out = side ? t.h_out : t.d_out;
            auto& m = side ? t.h_m : t.d_m;
            auto& tr = side ? t.h_tr : t.d_tr;
            rec = (orbmi_mappoint*)at(B, o_rec);
            mlf = (int32_t*)at(B, o_mlf);
            occ = (uint8_t*)at(B, o_occ);
            lfp = (orbmi_lastframe_point*)at(B, o_lfp);
            n = (int*)at(B, o_n);
            pose = (orbmi_pose_frame*)at(B, o_pose);
            out = (uint8_t*)at(B, o_out);
            m = (int32_t*)at(B, o_m);
            tr = (orbmi_mappoint_track*)at(B, o_tr);
        }
        return ORBMI_OK;
    }
    void free_track_buffers() {
        TrackBuf& t = tb;
        if (t.d_arena) (void)hipFree(t.d_arena);
        if (t.h_arena) (void)hipHostFree(t.h_arena);
        tb = TrackBuf{};
    }
    // one contiguous copy of the arena's host bytes [from, to) up, or device bytes down
    int up_range(const void* from, const void* to) {
        const size_t o = (const uint8_t*)from - tb.h_arena, n = (const uint8_t*)to - (const uint8_t*)from;
        return hipMemcpyAsync(tb.d_arena + o, from, n, hipMemcpyHostToDevice, tstream) == hipSuccess ? ORBMI_OK : ORBMI_E_HIP;
    }
    int down_range(void* from, const void* to) {
        const size_t o = (uint8_t*)from - tb.h_arena, n = (const uint8_t*)to - (uint8_t*)from;
        return hipMemcpyAsync(from, tb.d_arena + o, n, hipMemcpyDeviceToHost, tstream) == hipSuccess ? ORBMI_OK : ORBMI_E_HIP;
    }
    double phase_ms[PH_COUNT] = {};
    long phase_frames = 0;

    // ---- LocalMapping on its own thread (settings.async_local_mapping, src/LocalMapping.cc:47-128)
    // The map and the handles both threads call (matcher, vocabulary) are guarded by map_mtx:
    // Tracking holds it for Track() (the Frame constructor's extraction runs outside it), the
    // mapping thread for a keyframe's LocalMapping::Run except the LocalBundleAdjustment's GPU
    // solve, which -- as the reference's mMutexMapUpdate does (src/Optimizer.cc:776) -- locks
    // only for the graph assembly and the write-back, so tracking proceeds while it runs.
    std::mutex map_mtx;
    // mMutexMapUpdate (include/Map.h:66): Tracking holds it for the whole Track(), including the
    // windows in which it releases map_mtx for its GPU work; LocalBundleAdjustment's write-back of
    // poses and positions takes it first (src/Optimizer.cc:776), so no frame is tracked half
    // against the map before a LocalBA and half against the map after it.  Lock order: update_mtx,
    // then map_mtx.
    std::mutex update_mtx;
    std::mutex q_mtx;
    std::condition_variable q_cv, idle_cv;
    std::deque<int> lm_queue;   // mlNewKeyFrames
    bool lm_busy = false;       // !mbAcceptKeyFrames
    bool lm_quit = false;
    int lm_rc = ORBMI_OK;       // the first error of the mapping thread
    // mbAbortBA: written by the tracking thread (InterruptBA, InsertKeyFrame) and the mapping
    // thread, read by the mapping thread and by LocalBA's stop-flag mirror (orbmi_local_bundle_
    // adjustment reads it with an atomic load): every access is an atomic operation on this word
    int abort_ba = 0;
    // ORBMI_SLAM_NO_INTERRUPT=1 (experiment, tools/concur_breakdown.py): Tracking never raises
    // mbAbortBA, so every LocalBA the mapping thread starts runs to its end
    const bool no_interrupt = getenv("ORBMI_SLAM_NO_INTERRUPT") != nullptr;
    void set_abort_ba(int v) {
        if (v && no_interrupt) return;
        __atomic_store_n(&abort_ba, v, __ATOMIC_RELEASE);
    }
    std::thread lm_thread;
    bool async_lm() const { return s.async_local_mapping != 0; }
    // the schedule (orbmi_slam_get_schedule): every acquisition of map_mtx with the mapping thread
    // running, logged by the thread that took it (so map_mtx guards the log too)
    std::vector<orbmi_slam_event> sched;
    // the schedule, the LocalBA log and the per-keyframe state log are kept only when recording
    // is on (orbmi_slam_set_recording, before the first frame): a replay / test hook, not part of
    // the production path
    bool recording = false;
    void log_section(int label, int arg) {
        if (recording && async_lm()) sched.push_back(orbmi_slam_event{on_mapping_thread ? 1 : 0, label, arg});
        if (lock_profile && on_mapping_thread) { hold_label = label; hold_t0 = std::chrono::steady_clock::now(); }
    }
    // ORBMI_SLAM_LOCK_PROFILE=1 (development aid): how long the mapping thread holds the map lock
    // after each kind of acquisition (by schedule label), printed to stderr at destroy
    const bool lock_profile = getenv("ORBMI_SLAM_LOCK_PROFILE") != nullptr;
    int hold_label = -1;
    std::chrono::steady_clock::time_point hold_t0;
    std::map<int, std::pair<double, double>> hold_ms;  // label -> (sum, max) ms (mapping thread only)
    std::map<int, long> hold_n;
    void hold_end() {  // the mapping thread releases the map lock
        if (!lock_profile || !on_mapping_thread || hold_label < 0) return;
        const double d = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - hold_t0).count();
        auto& e = hold_ms[hold_label];
        e.first += d;
        e.second = std::max(e.second, d);
        hold_n[hold_label]++;
        hold_label = -1;
    }
    void hold_report() const {
        if (!lock_profile) return;
        for (const auto& kv : hold_ms)
            fprintf(stderr, "map-lock hold after label %d: n %ld  total %.3f ms  mean %.4f ms  max %.4f ms\n", kv.first,
                    hold_n.at(kv.first), kv.second.first, kv.second.first / std::max(1L, hold_n.at(kv.first)),
                    kv.second.second);
    }
    std::vector<orbmi_slam_ba_record> ba_log;  // orbmi_slam_get_local_ba_log (under map_mtx)
    // orbmi_slam_get_keyframe_state_log (under map_mtx): the map as LocalMapping left it after each
    // stage of a keyframe's job, so a replay names the first keyframe and stage whose map differs
    std::vector<orbmi_slam_kf_state> kf_state;
    static uint32_t fnv_mix(uint32_t h, uint32_t v) { return (h ^ v) * 16777619u; }
    static constexpr uint32_t kFnv0 = 2166136261u;
    uint32_t slot_hash(int k) const {  // the keyframe's map-point slots (ids, -1 empty)
        uint32_t h = kFnv0;
        for (int m : kfs[k].mps) h = fnv_mix(h, (uint32_t)m);
        return h;
    }
    void log_state(int k, int stage, int a, uint32_t b, uint32_t c) {
        if (!recording) return;
        const int at = async_lm() ? (int)sched.size() - 1 : -1;
        kf_state.push_back(orbmi_slam_kf_state{k, stage, at, a, (int32_t)b, (int32_t)c});
    }
    int fuse_ops = 0;  // map updates made by Fuse replays (Replace that moved observations, AddMapPoint)

    // ---- Frame views (include/Frame.h members the matchers read) --------------------------
    orbmi_frame_view view(const std::vector<orbmi_keypoint>& keys, const std::vector<uint8_t>& desc,
                          const std::vector<float>& ur, const float* tcw) const {
        orbmi_frame_view v{};
        v.n = (int)keys.size();
        v.keys_un = keys.data();
        v.u_right = ur.data();
        v.desc = desc.data();
        v.tcw = tcw;
        v.fx = s.fx; v.fy = s.fy; v.cx = s.cx; v.cy = s.cy; v.bf = s.bf;
        v.mb = s.bf / s.fx;
        v.min_x = 0.f; v.max_x = (float)s.width; v.min_y = 0.f; v.max_y = (float)s.height;  // no distortion
        v.grid_w_inv = 64.f / (float)s.width;
        v.grid_h_inv = 48.f / (float)s.height;
        v.nlevels = (int)scale_factors.size();
        v.scale_factors = scale_factors.data();
        v.log_scale_factor = log_scale_factor;
        v.n_device = nullptr;
        return v;
    }
    orbmi_frame_view view(const TrackedFrame& f, const float* tcw) const {
        orbmi_frame_view v = view(f.keys, f.desc, f.ur, tcw);
        if (f.dslot >= 0) {  // the frame's arrays in HBM (left item of its slot)
            v.keys_un = dev.kps[f.dslot];
            v.desc = dev.desc[f.dslot];
            v.u_right = dev.ur[f.dslot];
        }
        return v;
    }

    // Frame::Frame (stereo, src/Frame.cc:58-100): ORBextractor on both images (one batch on the
    // left handle) and ComputeStereoMatches into the next device slot, enqueued on the extractor's
    // stream with the read-back of the left outputs into pinned memory (frame_collect waits)
    // the first device slot that is neither a nor b (kSlots = 3 leaves at least one)
    static int free_slot(int a, int b) {
        for (int k = 0; k < kSlots; k++)
            if (k != a && k != b) return k;
        return -1;
    }
    int frame_enqueue(const uint8_t* L, const uint8_t* R, int rows, int cols, size_t step, int k) {
        if (k < 0 || k >= kSlots) return ORBMI_E_ARG;
        const size_t img = (size_t)rows * cols;
        if (2 * img > dev.img_bytes) {
            if (dev.img) (void)hipFree(dev.img);
            if (dev.h_img) (void)hipHostFree(dev.h_img);
            dev.img = nullptr;
            dev.h_img = nullptr;
            if (hipMalloc((void**)&dev.img, 2 * img) != hipSuccess) return ORBMI_E_HIP;
            if (hipHostMalloc((void**)&dev.h_img, 2 * img, hipHostMallocDefault) != hipSuccess) return ORBMI_E_HIP;
            dev.img_bytes = 2 * img;
        }
        if (!dev.kps[0]) {
            const int cap = s.n_features + 16 * s.n_levels + 64;
            dev.cap = cap;
            for (int k = 0; k < kSlots; k++) {
                if (hipMalloc((void**)&dev.kps[k], 2 * (size_t)cap * sizeof(orbmi_keypoint)) != hipSuccess ||
                    hipMalloc((void**)&dev.desc[k], 2 * (size_t)cap * 32) != hipSuccess ||
                    hipMalloc((void**)&dev.cnt[k], 2 * sizeof(int)) != hipSuccess ||
                    hipMalloc((void**)&dev.ur[k], 2 * (size_t)cap * sizeof(float)) != hipSuccess ||
                    hipMalloc((void**)&dev.dep[k], 2 * (size_t)cap * sizeof(float)) != hipSuccess)
                    return ORBMI_E_HIP;
            }
            if (hipHostMalloc((void**)&dev.h_kps, (size_t)cap * sizeof(orbmi_keypoint), hipHostMallocDefault) != hipSuccess ||
                hipHostMalloc((void**)&dev.h_desc, (size_t)cap * 32, hipHostMallocDefault) != hipSuccess ||
                hipHostMalloc((void**)&dev.h_cnt, 2 * sizeof(int), hipHostMallocDefault) != hipSuccess ||
                hipHostMalloc((void**)&dev.h_ur, (size_t)cap * sizeof(float), hipHostMallocDefault) != hipSuccess ||
                hipHostMalloc((void**)&dev.h_dep, (size_t)cap * sizeof(float), hipHostMallocDefault) != hipSuccess)
                return ORBMI_E_HIP;
        }
        for (int r = 0; r < rows; r++) {
            std::memcpy(dev.h_img + (size_t)r * cols, L + (size_t)r * step, cols);
            std::memcpy(dev.h_img + img + (size_t)r * cols, R + (size_t)r * step, cols);
        }
        if (hipMemcpyAsync(dev.img, dev.h_img, 2 * img, hipMemcpyHostToDevice, xstream) != hipSuccess) return ORBMI_E_HIP;
        const int cap = dev.cap;
        SLAM_CHECK(orbmi_extract_batch_device(left, dev.img, 2, rows, cols, cols, img, dev.kps[k], dev.desc[k], dev.cnt[k],
                                              cap));
        SLAM_CHECK(orbmi_compute_stereo_matches_batch_device(left, s.bf, s.fx, dev.ur[k], dev.dep[k]));
        if (hipMemcpyAsync(dev.h_cnt, dev.cnt[k], 2 * sizeof(int), hipMemcpyDeviceToHost, xstream) != hipSuccess ||
            hipMemcpyAsync(dev.h_kps, dev.kps[k], (size_t)cap * sizeof(orbmi_keypoint), hipMemcpyDeviceToHost, xstream) !=
                hipSuccess ||
            hipMemcpyAsync(dev.h_desc, dev.desc[k], (size_t)cap * 32, hipMemcpyDeviceToHost, xstream) != hipSuccess ||
            hipMemcpyAsync(dev.h_ur, dev.ur[k], (size_t)cap * sizeof(float), hipMemcpyDeviceToHost, xstream) != hipSuccess ||
            hipMemcpyAsync(dev.h_dep, dev.dep[k], (size_t)cap * sizeof(float), hipMemcpyDeviceToHost, xstream) != hipSuccess)
            return ORBMI_E_HIP;
        return ORBMI_OK;
    }

    // the enqueued extraction's host copies into cf (waits for the extractor's stream)
    int frame_collect(TrackedFrame& cf, int slot) {
        if (hipStreamSynchronize(xstream) != hipSuccess) return ORBMI_E_HIP;
        const int n = std::min(dev.h_cnt[0], dev.cap);
        cf.keys.assign(dev.h_kps, dev.h_kps + n);
        cf.desc.assign(dev.h_desc, dev.h_desc + (size_t)n * 32);
        cf.ur.assign(dev.h_ur, dev.h_ur + n);
        cf.depth.assign(dev.h_dep, dev.h_dep + n);
        cf.dslot = slot;
        // new keypoints behind a slot's pointers: a grid pinned on an older frame there is stale.
        // Frame::AssignFeaturesToGrid (src/Frame.cc:98) then runs once for the frame, on the
        // tracking stream: its searches (the last-frame search, the retry, SearchLocalPoints)
        // reuse that grid instead of building one each
        SLAM_CHECK(orbmi_matcher_release_grid(matcher));
        const orbmi_frame_view v = view(cf, nullptr);
        return orbmi_matcher_assign_features_to_grid(matcher, &v);
    }

    int frame_stereo(TrackedFrame& cf, const uint8_t* L, const uint8_t* R, int rows, int cols, size_t step) {
        // a pair enqueued ahead and not asked for (a plain call after an ahead one): it shares the
        // pinned read-back buffers, so it is drained and dropped first
        if (dev.ahead.on) {
            dev.ahead.on = false;
            if (hipStreamSynchronize(xstream) != hipSuccess) return ORBMI_E_HIP;
        }
        // the last frame's slot is read by this frame's tracking: extract into another one
        const int slot = free_slot(last_frame.dslot, -1);
        SLAM_CHECK(frame_enqueue(L, R, rows, cols, step, slot));
        return frame_collect(cf, slot);
    }

    // orbmi_slam_track_stereo_ahead: the Frame constructor of this pair from the extraction
    // enqueued by the previous call when it was for the same pair (same buffers and geometry),
    // else now; then the next pair's extraction is enqueued to run while this frame is tracked.
    // Extraction depends on the images only, so the frame is the one the plain call builds.
    int frame_stereo_ahead(TrackedFrame& cf, const uint8_t* L, const uint8_t* R, int rows, int cols, size_t step,
                           const uint8_t* nL, const uint8_t* nR) {
        Dev::Ahead& a = dev.ahead;
        if (a.on && a.L == L && a.R == R && a.rows == rows && a.cols == cols && a.step == step) {
            a.on = false;
            SLAM_CHECK(frame_collect(cf, a.slot));
        } else {
            if (a.on && hipStreamSynchronize(xstream) != hipSuccess) return ORBMI_E_HIP;  // a pair not asked for
            a.on = false;
            SLAM_CHECK(frame_stereo(cf, L, R, rows, cols, step));
        }
        if (nL && nR) {
            // tracking this frame reads cf's slot and the last frame's while the next pair is
            // extracted; the next call then tracks a.slot against cf's
            a.slot = free_slot(cf.dslot, last_frame.dslot);
            if (inline_frame) SLAM_CHECK(frame_enqueue(nL, nR, rows, cols, step, a.slot));
            else frame_post(nL, nR, rows, cols, step, a.slot);  // joined before the call returns
            a.on = true;
            a.L = nL;
            a.R = nR;
            a.rows = rows;
            a.cols = cols;
            a.step = step;
        }
        return ORBMI_OK;
    }

    // forget the pair enqueued ahead (its extraction drained first)
    void drop_ahead() {
        if (dev.ahead.on && xstream) (void)hipStreamSynchronize(xstream);
        dev.ahead.on = false;
        dev.ahead.slot = -1;
    }

    void free_dev() {
        frame_worker_stop();
        free_bow_async();
        if (dev.ahead.on && xstream) (void)hipStreamSynchronize(xstream);
        for (int k = 0; k < kSlots; k++) {
            (void)hipFree(dev.kps[k]);
            (void)hipFree(dev.desc[k]);
            (void)hipFree(dev.cnt[k]);
            (void)hipFree(dev.ur[k]);
            (void)hipFree(dev.dep[k]);
        }
        (void)hipFree(dev.img);
        (void)hipHostFree(dev.h_img);
        (void)hipHostFree(dev.h_kps);
        (void)hipHostFree(dev.h_desc);
        (void)hipHostFree(dev.h_cnt);
        (void)hipHostFree(dev.h_ur);
        (void)hipHostFree(dev.h_dep);
        dev = Dev{};
    }

    // ---- backend operators ------------------------------------------------------------------
    int extract(orbmi_extractor* ex, const uint8_t* img, int rows, int cols, size_t step, std::vector<orbmi_keypoint>& k,
                std::vector<uint8_t>& d) {
        int cap = s.n_features + 16 * s.n_levels + 64, n = 0;
        for (;;) {
            kbuf.resize(cap);
            dbuf.resize((size_t)cap * 32);
            const int rc = orbmi_extract(ex, img, rows, cols, step, kbuf.data(), dbuf.data(), cap, &n);
            // grow only when the call asked for more room than it had: an E_CAP that does not
            // come from this capacity (the extractor's own output capacity) is an error
            if (rc == ORBMI_E_CAP && n > cap) { cap = n; continue; }
            SLAM_CHECK(rc);
            break;
        }
        k.assign(kbuf.begin(), kbuf.begin() + n);
        d.assign(dbuf.begin(), dbuf.begin() + (size_t)n * 32);
        return ORBMI_OK;
    }

    int compute_bow(const std::vector<uint8_t>& desc, FeatVec& fv) {
        if (!voc) return ORBMI_E_STATE;  // TrackReferenceKeyFrame needs the vocabulary
        const int n = (int)(desc.size() / 32), cap = std::max(n, 1);
        std::vector<uint32_t> word(cap), node(cap);
        std::vector<double> value(cap);
        std::vector<int32_t> off(cap + 1), feat(cap);
        int counts[2] = {0, 0};
        SLAM_CHECK(orbmi_transform(voc, desc.data(), n, nullptr, 4, word.data(), value.data(), node.data(), off.data(),
                                   feat.data(), counts));
        const int nn = counts[1];
        fv.words = counts[0];
        fv.node.assign(node.begin(), node.begin() + nn);
        fv.off.assign(off.begin(), off.begin() + nn + 1);
        fv.feat.assign(feat.begin(), feat.begin() + off[nn]);
        fv.valid = true;
        return ORBMI_OK;
    }

    // KeyFrame::ComputeBoW for the mapping thread from the keyframe's HBM descriptors, in two
    // halves so that ProcessNewKeyFrame's ComputeDistinctiveDescriptors call runs while the
    // transform does: bow_begin enqueues the transform (device outputs) and the read-back of the
    // FeatureVector into pinned memory on the vocabulary's stream; bow_end waits and parses.
    struct BowAsync {
        uint8_t* d = nullptr;   // value f64[cap] | word u32[cap] | node u32[cap] | off i32[cap+1] | feat i32[cap] | counts i32[2]
        uint8_t* h = nullptr;   // pinned mirror of node .. counts
        int cap = 0, n = 0;
        hipStream_t stream = nullptr;
        bool pending = false;
    } bowa;
    size_t bow_tail_bytes(int cap) const { return (size_t)(3 * cap + 3) * 4; }
    int bow_begin(const uint8_t* d_desc, int n) {
        BowAsync& b = bowa;
        if (n > b.cap) {
            if (b.d) (void)hipFree(b.d);
            if (b.h) (void)hipHostFree(b.h);
            b.d = b.h = nullptr;
            b.cap = 0;
            const int cap = std::max(n, 2048);
            if (hipMalloc((void**)&b.d, (size_t)cap * 12 + bow_tail_bytes(cap)) != hipSuccess) return ORBMI_E_HIP;
            if (hipHostMalloc((void**)&b.h, bow_tail_bytes(cap), hipHostMallocDefault) != hipSuccess) return ORBMI_E_HIP;
            b.cap = cap;
        }
        void* vs = nullptr;
        SLAM_CHECK(orbmi_vocabulary_get_stream(voc, &vs));
        b.stream = (hipStream_t)vs;
        b.n = n;
        const int cap = b.cap;
        double* value = (double*)b.d;
        uint32_t* word = (uint32_t*)(b.d + (size_t)cap * 8);
        uint8_t* tail = b.d + (size_t)cap * 12;
        uint32_t* node = (uint32_t*)tail;
        int32_t* off = (int32_t*)(node + cap);
        int32_t* feat = off + cap + 1;
        int* counts = (int*)(feat + cap);
        SLAM_CHECK(orbmi_transform(voc, d_desc, n, nullptr, 4, word, value, node, off, feat, counts));
        if (hipMemcpyAsync(b.h, tail, bow_tail_bytes(cap), hipMemcpyDeviceToHost, b.stream) != hipSuccess)
            return ORBMI_E_HIP;
        b.pending = true;
        return ORBMI_OK;
    }
    int bow_end(FeatVec& fv) {
        BowAsync& b = bowa;
        if (!b.pending) return ORBMI_E_STATE;
        b.pending = false;
        if (hipStreamSynchronize(b.stream) != hipSuccess) return ORBMI_E_HIP;
        const int cap = b.cap;
        const uint32_t* node = (const uint32_t*)b.h;
        const int32_t* off = (const int32_t*)(node + cap);
        const int32_t* feat = off + cap + 1;
        const int* counts = (const int*)(feat + cap);
        const int nn = counts[1];
        if (nn < 0 || nn > b.n || off[nn] > b.n) return ORBMI_E_STATE;
        fv.words = counts[0];
        fv.node.assign(node, node + nn);
        fv.off.assign(off, off + nn + 1);
        fv.feat.assign(feat, feat + off[nn]);
        fv.valid = true;
        return ORBMI_OK;
    }
    void free_bow_async() {
        if (bowa.pending && bowa.stream) (void)hipStreamSynchronize(bowa.stream);
        if (bowa.d) (void)hipFree(bowa.d);
        if (bowa.h) (void)hipHostFree(bowa.h);
        bowa = BowAsync{};
    }

    // Optimizer::PoseOptimization over keypoint i -> lfp[match[i]] (match[i] >= 0)
    int pose_optimization(const TrackedFrame& cf, const std::vector<int32_t>& match,
                          const std::vector<orbmi_lastframe_point>& lfp, M4& tcw_out, std::vector<uint8_t>& out) {
        orbmi_frame_view v = view(cf, cf.tcw.data());
        orbmi_frame_mappoints fm{};
        fm.match_lf = const_cast<int32_t*>(match.data());
        fm.lf_points = lfp.data();
        fm.n_lf_points = (int)lfp.size();
        orbmi_pose_frame rec{};
        out.assign(std::max(cf.n(), 1), 0);
        SLAM_CHECK(unlocked(ORBMI_SCHED_T_POSE, cf.id, [&] {
            return orbmi_pose_optimization_frame(pose, &v, inv_level_sigma2.data(), &fm, &rec, out.data());
        }));
        std::memcpy(tcw_out.data(), rec.tcw, sizeof(rec.tcw));
        out.resize(cf.n());
        return ORBMI_OK;
    }

    // ---- map model ----------------------------------------------------------------------------
    void kf_ow(int k, float ow[3]) const { camera_center(kfs[k].tcw, ow); }

    int tracked_map_points(const KeyFrame& kf, int min_obs) const {  // KeyFrame::TrackedMapPoints
        int n = 0;
        for (int m : kf.mps)
            if (m >= 0 && !mps[m].bad && (min_obs <= 0 || mps[m].nobs >= min_obs)) n++;
        return n;
    }

    void sort_covisible(KeyFrame& kf) {  // heaviest first, ties to the higher id
        std::vector<std::pair<int, int>> p;
        for (auto& c : kf.conn) p.push_back({c.second, c.first});
        std::sort(p.begin(), p.end(), [](const std::pair<int, int>& a, const std::pair<int, int>& b) {
            return a.first != b.first ? a.first > b.first : a.second > b.second;
        });
        kf.covisible.clear();
        for (auto& x : p) kf.covisible.push_back(x.second);
    }

    void add_connection(int k, int other, int w) {  // KeyFrame::AddConnection + UpdateBestCovisibles
        kfs[k].conn[other] = w;
        sort_covisible(kfs[k]);
    }

    void normals(const std::vector<int>& pts) {  // UpdateNormalAndDepth of each (timed)
        PhaseTimer pt(&phase_ms[PH_LM_NORMALS]);
        for (int m : pts) update_normal_and_depth(m);
    }
    void connections(int k) {
        PhaseTimer pt(&phase_ms[PH_LM_CONNECTIONS]);
        update_connections(k);
    }
    void update_connections(int k) {  // KeyFrame::UpdateConnections (src/KeyFrame.cc:285-371)
        std::map<int, int> counter;
        for (int m : kfs[k].mps) {
            if (m < 0 || mps[m].bad) continue;
            for (auto& o : mps[m].obs)
                if (o.first != k) counter[o.first]++;
        }
        if (counter.empty()) return;
        const int th = 15;
        int nmax = 0, kfmax = -1;
        std::vector<std::pair<int, int>> pairs;  // (w, id)
        for (auto& c : counter) {
            const int w = c.second;
            if (w > nmax) { nmax = w; kfmax = c.first; }
            if (w >= th) {
                pairs.push_back({w, c.first});
                add_connection(c.first, k, w);
            }
        }
        if (pairs.empty()) {
            pairs.push_back({nmax, kfmax});
            add_connection(kfmax, k, nmax);
        }
        std::sort(pairs.begin(), pairs.end(), [](const std::pair<int, int>& a, const std::pair<int, int>& b) {
            return a.first != b.first ? a.first > b.first : a.second > b.second;
        });
        KeyFrame& kf = kfs[k];
        kf.conn = counter;
        kf.covisible.clear();
        for (auto& p : pairs) kf.covisible.push_back(p.second);
        if (kf.first_connection && kf.id != 0) {
            kf.parent = kf.covisible[0];
            kfs[kf.parent].children.push_back(k);
            kf.first_connection = false;
        }
    }

    void add_observation(int m, int k, int idx) {  // MapPoint::AddObservation
        MapPoint& mp = mps[m];
        if (mp.obs.count(k)) return;
        mp.obs[k] = idx;
        mp.nobs += kfs[k].ur[idx] >= 0 ? 2 : 1;
    }

    void set_bad(int m) {  // MapPoint::SetBadFlag
        MapPoint& mp = mps[m];
        mp.bad = true;
        for (auto& o : mp.obs)
            if (kfs[o.first].mps[o.second] == m) kfs[o.first].mps[o.second] = -1;
        mp.obs.clear();
    }

    void erase_observation(int m, int k) {  // MapPoint::EraseObservation
        MapPoint& mp = mps[m];
        auto it = mp.obs.find(k);
        if (it == mp.obs.end()) return;
        const int idx = it->second;
        mp.obs.erase(it);
        mp.nobs -= kfs[k].ur[idx] >= 0 ? 2 : 1;
        if (mp.ref_kf == k && !mp.obs.empty()) mp.ref_kf = mp.obs.begin()->first;  // lowest id
        if (mp.nobs <= 2) set_bad(m);
    }

    // MapPoint::UpdateNormalAndDepth (src/MapPoint.cc:339-390), float32 arithmetic as
    // system.update_normals_and_depths (observing keyframes in id order)
    void update_normal_and_depth(int m) {
        MapPoint& mp = mps[m];
        if (mp.bad || mp.obs.empty()) return;
        float normal[3] = {0, 0, 0};
        for (auto& o : mp.obs) {
            float ow[3];
            kf_ow(o.first, ow);
            const float v[3] = {mp.pos[0] - ow[0], mp.pos[1] - ow[1], mp.pos[2] - ow[2]};
            const double n2 = ((double)v[0] * v[0] + (double)v[1] * v[1]) + (double)v[2] * v[2];
            const double inv = 1.0 / std::sqrt(n2);
            for (int r = 0; r < 3; r++) normal[r] = normal[r] + (float)((double)v[r] * inv);
        }
        const double ic = 1.0 / (double)mp.obs.size();
        for (int r = 0; r < 3; r++) mp.normal[r] = (float)((double)normal[r] * ic);
        float ow[3];
        kf_ow(mp.ref_kf, ow);
        const float pc[3] = {mp.pos[0] - ow[0], mp.pos[1] - ow[1], mp.pos[2] - ow[2]};
        const float dist = (float)std::sqrt(((double)pc[0] * pc[0] + (double)pc[1] * pc[1]) + (double)pc[2] * pc[2]);
        const KeyFrame& rk = kfs[mp.ref_kf];
        const int level = rk.keys[mp.obs.at(mp.ref_kf)].octave;
        mp.max_distance = dist * scale_factors[level];
        mp.min_distance = mp.max_distance / scale_factors[scale_factors.size() - 1];
    }

    // MapPoint::ComputeDistinctiveDescriptors for a batch of points (src/MapPoint.cc:247-316)
    // the observation descriptors of the points (CSR, mObservations order, bad keyframes left out)
    void obs_rows(const std::vector<int>& pts, std::vector<uint8_t>& rows, std::vector<int32_t>& off) const {
        rows.clear();
        off.assign(1, 0);
        for (int m : pts) {
            for (auto& o : mps[m].obs)
                if (!kfs[o.first].bad) rows.insert(rows.end(), &kfs[o.first].desc[32 * o.second], &kfs[o.first].desc[32 * o.second] + 32);
            off.push_back((int32_t)(rows.size() / 32));
        }
    }

    int distinctive(const std::vector<int>& pts) {
        std::vector<uint8_t> rows;
        std::vector<int32_t> off;
        {
            PhaseTimer pt(&phase_ms[PH_LM_OBSROWS]);
            obs_rows(pts, rows, off);
        }
        if (rows.empty()) return ORBMI_OK;
        const int np = (int)pts.size();
        std::vector<int32_t> best(std::max(np, 1));
        std::vector<uint8_t> out((size_t)std::max(np, 1) * 32);
        orbmi_matcher* mt = lmm();
        SLAM_CHECK(unlocked(ORBMI_SCHED_L_DISTINCTIVE, -1, [&] {
            PhaseTimer pt(&phase_ms[PH_LM_DISTINCTIVE_CALL]);
            return orbmi_compute_distinctive_descriptors(mt, rows.data(), off.data(), np, best.data(), out.data());
        }));
        for (int j = 0; j < np; j++)
            if (off[j + 1] > off[j]) std::memcpy(mps[pts[j]].desc, &out[32 * j], 32);
        return ORBMI_OK;
    }

    // ---- keyframes and map points -------------------------------------------------------------
    int new_keyframe(const TrackedFrame& cf) {
        KeyFrame kf;
        kf.id = (int)kfs.size();
        kf.frame_id = cf.id;
        kf.ts = cf.ts;
        kf.tcw = cf.tcw;
        kf.keys = cf.keys;
        kf.desc = cf.desc;
        kf.ur = cf.ur;
        kf.depth = cf.depth;
        kf.mps = cf.mps;
        kf.fv = cf.fv;
        // the keyframe's arrays in HBM, copied once (from the frame's device slot when it has one)
        const size_t n = kf.keys.size(), bk = n * sizeof(orbmi_keypoint), bd = n * 32, bu = n * sizeof(float);
        std::vector<float> dc(2 * n);  // depth, then the stereo parallax table
        const float mb = s.bf / s.fx;
        for (size_t i = 0; i < n; i++) {
            dc[i] = kf.depth[i];
            dc[n + i] = kf.ur[i] >= 0 ? orbmi::tri::stereo_parallax_cos(mb, kf.depth[i]) : 0.f;
        }
        if (n > 0 && hipMalloc((void**)&kf.d_block, bk + bd + 3 * bu) == hipSuccess) {
            const bool dslot = cf.dslot >= 0;
            const hipMemcpyKind kind = dslot ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice;
            const void* sk = dslot ? (const void*)dev.kps[cf.dslot] : (const void*)kf.keys.data();
            const void* sd = dslot ? (const void*)dev.desc[cf.dslot] : (const void*)kf.desc.data();
            const void* su = dslot ? (const void*)dev.ur[cf.dslot] : (const void*)kf.ur.data();
            // four copies in stream order on the tracking stream (idle here: the frame's stages
            // were read back), one wait -- instead of four blocking copies
            const hipStream_t cs = tstream;
            if (hipMemcpyAsync(kf.d_block, sk, bk, kind, cs) == hipSuccess &&
                hipMemcpyAsync(kf.d_block + bk, sd, bd, kind, cs) == hipSuccess &&
                hipMemcpyAsync(kf.d_block + bk + bd, su, bu, kind, cs) == hipSuccess &&
                hipMemcpyAsync(kf.d_block + bk + bd + bu, dc.data(), 2 * bu, hipMemcpyHostToDevice, cs) == hipSuccess &&
                hipStreamSynchronize(cs) == hipSuccess) {
                kf.d_keys = (const orbmi_keypoint*)kf.d_block;
                kf.d_desc = kf.d_block + bk;
                kf.d_ur = (const float*)(kf.d_block + bk + bd);
                kf.d_depth = (const float*)(kf.d_block + bk + bd + bu);
                kf.d_cos = (const float*)(kf.d_block + bk + bd + 2 * bu);
            }
        }
        kfs.push_back(std::move(kf));
        return (int)kfs.size() - 1;
    }

    // KeyFrame view for the searches: its HBM copy when there is one; tcw points at `tcw_copy`
    // (the caller's copy: the keyframe's own pose may move while the map lock is released)
    orbmi_frame_view kf_view(const KeyFrame& kf, const float* tcw) const {
        orbmi_frame_view v = view(kf.keys, kf.desc, kf.ur, tcw);
        if (kf.d_keys) {
            v.keys_un = kf.d_keys;
            v.desc = kf.d_desc;
            v.u_right = kf.d_ur;
        }
        return v;
    }

    // LocalMapping's GPU calls: on the mapping thread they use its own matcher and run with the
    // map lock released (their inputs are the caller's copies or the keyframes' HBM copies)
    orbmi_matcher* lm_matcher = nullptr;
    orbmi_matcher* lmm() const { return on_mapping_thread ? lm_matcher : matcher; }
    // `label`, `arg`: where the thread resumes, for the schedule (ORBMI_SCHED_*)
    template <class F>
    int unlocked(int label, int arg, F f) {
        if (!held_lock) return f();
        hold_end();
        held_lock->unlock();
        const int rc = f();
        if (on_mapping_thread) {
            PhaseTimer pt(&phase_ms[PH_LM_LOCK]);
            held_lock->lock();
        } else {
            PhaseTimer pt(&phase_ms[PH_LOCK]);
            held_lock->lock();
        }
        log_section(label, arg);
        return rc;
    }

    // Frame::UnprojectStereo (src/Frame.cc:701-715) + new MapPoint + AddObservation + AddMapPoint
    // + UpdateNormalAndDepth (src/Tracking.cc:602-616, :1308-1320)
    void create_points(int k, TrackedFrame& cf, const std::vector<int>& idx) {
        if (idx.empty()) return;
        const float invfx = 1.f / s.fx, invfy = 1.f / s.fy;
        const M4 twc = pose_inverse(cf.tcw);
        std::vector<int> made;
        for (int i : idx) {
            const float z = cf.depth[i];
            const float x = (cf.keys[i].x - s.cx) * z * invfx;
            const float y = (cf.keys[i].y - s.cy) * z * invfy;
            MapPoint mp;
            mp.id = (int)mps.size();
            for (int r = 0; r < 3; r++) {
                const double a = (double)twc[4 * r] * (double)x + (double)twc[4 * r + 1] * (double)y +
                                 (double)twc[4 * r + 2] * (double)z;
                mp.pos[r] = (float)(a + (double)twc[4 * r + 3]);  // one gemm(Rwc, x3Dc, 1, Ow, 1)
            }
            mp.ref_kf = k;
            mp.first_kf_id = k;
            std::memcpy(mp.desc, &cf.desc[32 * i], 32);  // ComputeDistinctiveDescriptors of one observation
            mps.push_back(mp);
            add_observation(mp.id, k, i);
            kfs[k].mps[i] = mp.id;
            cf.mps[i] = mp.id;
            made.push_back(mp.id);
        }
        for (int m : made) update_normal_and_depth(m);
    }

    int stereo_initialization(TrackedFrame& cf) {  // src/Tracking.cc:584-636
        if (cf.n() <= 500) return ORBMI_OK;
        cf.tcw = eye4();
        cf.has_tcw = true;
        const int k = new_keyframe(cf);
        std::vector<int> idx;
        for (int i = 0; i < cf.n(); i++)
            if (cf.depth[i] > 0) idx.push_back(i);
        create_points(k, cf, idx);
        SLAM_CHECK(insert_keyframe(k));
        last_kf_frame_id = cf.id;
        local_kfs = {k};
        local_mps.clear();
        for (auto& m : mps)
            if (!m.bad) local_mps.push_back(m.id);
        ref_kf = k;
        cf.ref_kf = k;
        state = OK;
        return ORBMI_OK;
    }

    bool need_new_keyframe(const TrackedFrame& cf, orbmi_slam_frame_stats& st) {  // src/Tracking.cc:1140-1249
        const int nkfs = keyframes_in_map();
        if (cf.id < last_reloc_frame_id + s.max_frames && nkfs > s.max_frames) return false;
        const int min_obs = nkfs <= 2 ? 2 : 3;
        const int n_ref = tracked_map_points(kfs[ref_kf], min_obs);
        int n_tracked_close = 0, n_non_tracked_close = 0;
        for (int i = 0; i < cf.n(); i++) {
            if (!(cf.depth[i] > 0 && cf.depth[i] < s.th_depth)) continue;
            if (cf.mps[i] >= 0 && !cf.outlier[i]) n_tracked_close++;
            else n_non_tracked_close++;
        }
        const bool need_close = n_tracked_close < 100 && n_non_tracked_close > 70;
        const float th_ref = nkfs < 2 ? 0.4f : 0.75f;
        bool idle = true;  // LocalMapping::AcceptKeyFrames (always, when it runs synchronously)
        size_t queued = 0;
        if (async_lm()) {
            std::lock_guard<std::mutex> g(q_mtx);
            idle = !lm_busy;
            queued = lm_queue.size();
        }
        const bool c1a = cf.id >= last_kf_frame_id + s.max_frames;
        const bool c1b = cf.id >= last_kf_frame_id + s.min_frames && idle;
        const bool c1c = matches_inliers < n_ref * 0.25 || need_close;
        const bool c2 = ((float)matches_inliers < (float)n_ref * th_ref || need_close) && matches_inliers > 15;
        st.need_kf = (c1a || c1b || c1c) && c2;
        if (!st.need_kf) return false;
        if (idle) return true;
        set_abort_ba(1);    // mpLocalMapper->InterruptBA()
        return queued < 3;  // stereo: KeyframesInQueue() < 3
    }

    int create_new_keyframe(TrackedFrame& cf) {  // src/Tracking.cc:1251-1330
        const int k = new_keyframe(cf);
        ref_kf = k;
        cf.ref_kf = k;
        std::vector<std::pair<float, int>> order;
        for (int i = 0; i < cf.n(); i++)
            if (cf.depth[i] > 0) order.push_back({cf.depth[i], i});
        std::sort(order.begin(), order.end());
        std::vector<int> fresh;
        int npts = 0;
        for (auto& zi : order) {
            const int i = zi.second;
            const int m = cf.mps[i];
            const bool create = m < 0 || mps[m].nobs < 1;
            if (create && m >= 0) {
                cf.mps[i] = -1;
                kfs[k].mps[i] = -1;
            }
            if (create) fresh.push_back(i);
            npts++;
            if (zi.first > s.th_depth && npts > 100) break;
        }
        create_points(k, cf, fresh);
        SLAM_CHECK(insert_keyframe(k));
        last_kf_frame_id = cf.id;
        return ORBMI_OK;
    }

    // LocalMapping::InsertKeyFrame: run it now (synchronous mode) or queue it for the thread
    int insert_keyframe(int k) {
        if (!async_lm()) return local_mapping(k);
        {
            std::lock_guard<std::mutex> g(q_mtx);
            if (lm_rc) return lm_rc;
            lm_queue.push_back(k);
            set_abort_ba(1);  // a new keyframe interrupts the running BA (src/LocalMapping.cc:134)
        }
        q_cv.notify_one();
        return ORBMI_OK;
    }

    bool new_keyframes_queued() {  // LocalMapping::CheckNewKeyFrames
        if (!async_lm()) return false;
        std::lock_guard<std::mutex> g(q_mtx);
        return !lm_queue.empty();
    }

    // the mapping thread: one keyframe at a time, holding map_mtx except inside its GPU calls.
    // The keyframe is taken from the queue and AcceptKeyFrames changes only under map_mtx (as
    // Tracking reads them), so the order of the map_mtx acquisitions (the schedule) decides every
    // interaction of the two threads.
    void lm_run() {
        on_mapping_thread = true;
        for (;;) {
            {
                std::unique_lock<std::mutex> g(q_mtx);
                q_cv.wait(g, [&] { return lm_quit || !lm_queue.empty(); });
                if (lm_queue.empty()) return;  // quit with nothing left
            }
            int rc = ORBMI_OK;
            {
                std::unique_lock<std::mutex> m(map_mtx);
                log_section(ORBMI_SCHED_L_JOB, -1);
                int k = -1;
                {
                    std::lock_guard<std::mutex> g(q_mtx);
                    if (!lm_queue.empty()) {  // (a reset may have dropped it meanwhile)
                        k = lm_queue.front();
                        lm_queue.pop_front();
                        lm_busy = true;  // SetAcceptKeyFrames(false)
                    }
                }
                if (recording) sched.back().arg = k;
                if (k >= 0) {
                    held_lock = &m;
                    rc = local_mapping(k);
                    held_lock = nullptr;
                }
                hold_end();
                std::lock_guard<std::mutex> g(q_mtx);
                lm_busy = false;  // SetAcceptKeyFrames(true), still under map_mtx
                if (rc && !lm_rc) lm_rc = rc;
            }
            idle_cv.notify_all();
        }
    }

    int wait_local_mapping() {  // until the queue is empty and the thread idle
        if (!async_lm()) return ORBMI_OK;
        std::unique_lock<std::mutex> g(q_mtx);
        idle_cv.wait(g, [&] { return lm_queue.empty() && !lm_busy; });
        return lm_rc;
    }

    // ---- LocalMapping (synchronous) -------------------------------------------------------------
    // LocalMapping::Run for one keyframe (src/LocalMapping.cc:47-128), no other keyframe queued and
    // no stop request: ProcessNewKeyFrame, MapPointCulling, CreateNewMapPoints,
    // SearchInNeighbors, LocalBundleAdjustment (more than 2 keyframes), KeyFrameCulling
    int local_mapping(int k) {
        PhaseTimer all(&phase_ms[PH_LM_TOTAL]);
        auto* pt = new PhaseTimer(&phase_ms[PH_LM_PROCESS]);
        auto next = [&](Phase p) {
            delete pt;
            pt = new PhaseTimer(&phase_ms[p]);
        };
        const int rc = local_mapping_steps(k, next);
        delete pt;
        return rc;
    }

    template <class Next>
    int local_mapping_steps(int k, Next&& next) {
        // ProcessNewKeyFrame (src/LocalMapping.cc:152-211): ComputeBoW, the observations of the
        // keyframe's points, UpdateNormalAndDepth, ComputeDistinctiveDescriptors, UpdateConnections.
        // The transform reads only the keyframe's descriptors, so it runs in the same window with
        // the map lock released as the descriptors of the updated points: one release, and the
        // two device calls overlap (the keyframe's descriptors are copied first when it has no
        // HBM copy: Tracking may grow kfs meanwhile).
        const bool need_bow = voc && !kfs[k].fv.valid;
        std::vector<int> updated;
        for (int i = 0; i < (int)kfs[k].mps.size(); i++) {
            const int m = kfs[k].mps[i];
            if (m < 0 || mps[m].bad) continue;
            if (!mps[m].obs.count(k)) {
                add_observation(m, k, i);
                updated.push_back(m);
            } else {
                recent_mps.push_back(m);  // the new stereo points the Tracking inserted
            }
        }
        normals(updated);
        std::vector<uint8_t> rows;
        std::vector<int32_t> off;
        {
            PhaseTimer pt(&phase_ms[PH_LM_OBSROWS]);
            obs_rows(updated, rows, off);
        }
        if (need_bow || !rows.empty()) {
            const int np = (int)updated.size();
            std::vector<int32_t> best(std::max(np, 1));
            std::vector<uint8_t> out((size_t)std::max(np, 1) * 32);
            const uint8_t* d_desc = kfs[k].d_desc;
            const int nk = (int)kfs[k].keys.size();
            const std::vector<uint8_t> desc = need_bow && !d_desc ? kfs[k].desc : std::vector<uint8_t>();
            FeatVec fv;
            orbmi_matcher* mt = lmm();
            SLAM_CHECK(unlocked(need_bow ? ORBMI_SCHED_L_BOW : ORBMI_SCHED_L_DISTINCTIVE, need_bow ? k : -1, [&] {
                int rc = ORBMI_OK;
                const bool async_bow = need_bow && d_desc && nk > 0;
                if (async_bow) rc = bow_begin(d_desc, nk);
                else if (need_bow) rc = compute_bow(desc, fv);
                if (!rc && !rows.empty()) {
                    PhaseTimer pt(&phase_ms[PH_LM_DISTINCTIVE_CALL]);
                    rc = orbmi_compute_distinctive_descriptors(mt, rows.data(), off.data(), np, best.data(), out.data());
                }
                if (async_bow) {
                    const int rc2 = bow_end(fv);
                    if (!rc) rc = rc2;
                }
                return rc;
            }));
            if (need_bow && !kfs[k].fv.valid) kfs[k].fv = std::move(fv);  // (Tracking may have computed it: the same)
            if (!rows.empty())
                for (int j = 0; j < np; j++)
                    if (off[j + 1] > off[j]) std::memcpy(mps[updated[j]].desc, &out[32 * j], 32);
        }
        connections(k);
        if (recording) {  // ProcessNewKeyFrame's outcome: BowVector words, FeatureVector, slots
            const FeatVec& fv = kfs[k].fv;
            uint32_t h = kFnv0;
            for (uint32_t v : fv.node) h = fnv_mix(h, v);
            for (int32_t v : fv.off) h = fnv_mix(h, (uint32_t)v);
            for (int32_t v : fv.feat) h = fnv_mix(h, (uint32_t)v);
            log_state(k, ORBMI_KF_STATE_PROCESS, fv.valid ? fv.words : -1, h, slot_hash(k));
        }
        next(PH_LM_CULL);
        map_point_culling(k);
        // SearchInNeighbors' last ComputeDistinctiveDescriptors (all the keyframe's points) rides in
        // LocalBA's device window when LocalBA runs (one map-lock release fewer per keyframe)
        std::vector<int> owed2;
        if (s.local_mapping) {
            next(PH_LM_CREATE);
            const size_t nmp0 = mps.size();
            std::vector<int> owed;
            SLAM_CHECK(create_new_map_points(k, owed));
            log_state(k, ORBMI_KF_STATE_CREATE, (int)(mps.size() - nmp0), (uint32_t)mps.size(), slot_hash(k));
            next(PH_LM_FUSE);
            if (new_keyframes_queued()) {
                sin_skipped++;
                SLAM_CHECK(distinctive(owed));
            } else {
                fuse_ops = 0;
                SLAM_CHECK(search_in_neighbors(k, owed, owed2));
                int filled = 0;
                for (int m : kfs[k].mps) filled += m >= 0;
                log_state(k, ORBMI_KF_STATE_FUSE, fuse_ops, (uint32_t)filled, slot_hash(k));
            }
        }
        set_abort_ba(0);
        lm_jobs++;
        if (new_keyframes_queued()) {
            ba_skipped++;
            SLAM_CHECK(distinctive(owed2));
        } else {
            next(PH_LM_BA);
            if (s.local_ba && keyframes_in_map() > 2) SLAM_CHECK(local_bundle_adjustment(k, owed2));
            else SLAM_CHECK(distinctive(owed2));
            next(PH_LM_KFCULL);
            if (s.local_mapping) keyframe_culling(k);
        }
        return ORBMI_OK;
    }

    void map_point_culling(int k) {  // src/LocalMapping.cc:219-263, stereo: nThObs = 3
        std::vector<int> keep;
        for (int m : recent_mps) {
            MapPoint& mp = mps[m];
            if (mp.bad) continue;
            if ((float)mp.found / (float)mp.visible < 0.25f) set_bad(m);  // GetFoundRatio
            else if (k - mp.first_kf_id >= 2 && mp.nobs <= 3) set_bad(m);
            else if (k - mp.first_kf_id >= 3) continue;
            else keep.push_back(m);
        }
        recent_mps = keep;
    }

    orbmi_tri_keyframe tri_view(const KeyFrame& kf) const {
        return orbmi_tri_keyframe{kf.tcw.data(), kf.keys.data(), kf.ur.data(), kf.depth.data(), s.fx, s.fy, s.cx,
                                  s.cy, s.bf, s.bf / s.fx, level_sigma2.data(), scale_factors.data()};
    }

    // src/LocalMapping.cc:290-577, stereo: the 10 best covisible keyframes.  The neighbours that
    // pass the baseline test go to the device in one orbmi_create_new_map_points call (searches and
    // triangulation pair by pair, the keypoints earlier pairs claimed excluded on the device), run
    // on the keyframes' HBM copies with the map lock released; the new points are then made here in
    // the reference's order.
    // `owed`: the new points, whose ComputeDistinctiveDescriptors the caller does (with
    // SearchInNeighbors' first device call when that runs: one round trip fewer)
    int create_new_map_points(int k, std::vector<int>& owed) {
        owed.clear();
        float ow1[3];
        kf_ow(k, ow1);
        const float mb = s.bf / s.fx;
        const std::vector<int> neigh(kfs[k].covisible.begin(),
                                     kfs[k].covisible.begin() + std::min<size_t>(10, kfs[k].covisible.size()));
        if (!kfs[k].fv.valid || !kfs[k].d_keys) return create_new_map_points_host(k);
        std::vector<int> pk, pos;  // the neighbours searched, and their index in `neigh`
        std::vector<M4> tcw2;
        std::vector<float> F12;
        std::vector<std::vector<uint8_t>> has2;
        const M4 tcw1 = kfs[k].tcw;
        for (size_t i = 0; i < neigh.size(); i++) {
            const int k2 = neigh[i];
            float ow2[3];
            kf_ow(k2, ow2);
            const float d[3] = {ow2[0] - ow1[0], ow2[1] - ow1[1], ow2[2] - ow1[2]};
            const float baseline = (float)std::sqrt(((double)d[0] * d[0] + (double)d[1] * d[1]) + (double)d[2] * d[2]);
            if (baseline < mb) continue;
            if (!kfs[k2].fv.valid) continue;
            if (!kfs[k2].d_keys) return create_new_map_points_host(k);
            float F[9];
            const orbmi_tri_keyframe v1 = tri_view(kfs[k]), v2 = tri_view(kfs[k2]);
            SLAM_CHECK(orbmi_compute_f12(&v1, &v2, F));
            pk.push_back(k2);
            pos.push_back((int)i);
            tcw2.push_back(kfs[k2].tcw);
            F12.insert(F12.end(), F, F + 9);
            has2.emplace_back(std::max<size_t>(kfs[k2].mps.size(), 1), 0);
            for (size_t q = 0; q < kfs[k2].mps.size(); q++) has2.back()[q] = kfs[k2].mps[q] >= 0;
        }
        const int np = (int)pk.size();
        if (np == 0) return ORBMI_OK;
        const size_t n1 = kfs[k].keys.size();
        std::vector<uint8_t> has1(std::max<size_t>(n1, 1), 0);
        for (size_t i = 0; i < n1; i++) has1[i] = kfs[k].mps[i] >= 0;
        // views on copies of the poses and on HBM arrays: valid while the lock is released
        auto tri_dev = [&](const KeyFrame& kf, const M4& tcw) {
            orbmi_tri_keyframe t = tri_view(kf);
            t.tcw = tcw.data();
            t.keys_un = kf.d_keys;
            t.u_right = kf.d_ur;
            t.depth = kf.d_depth;
            return t;
        };
        const orbmi_frame_view f1 = kf_view(kfs[k], tcw1.data());
        const orbmi_tri_keyframe t1 = tri_dev(kfs[k], tcw1);
        const orbmi_feature_vector fv1 = kfs[k].fv.view();
        const float* cos1 = kfs[k].d_cos;
        std::vector<orbmi_frame_view> f2(np);
        std::vector<orbmi_tri_keyframe> t2(np);
        std::vector<orbmi_feature_vector> fv2(np);
        std::vector<const float*> cos2(np);
        std::vector<const uint8_t*> mp2(np);
        for (int j = 0; j < np; j++) {
            const KeyFrame& K2 = kfs[pk[j]];
            f2[j] = kf_view(K2, tcw2[j].data());
            t2[j] = tri_dev(K2, tcw2[j]);
            fv2[j] = K2.fv.view();
            cos2[j] = K2.d_cos;
            mp2[j] = has2[j].data();
        }
        std::vector<int32_t> m12(std::max<size_t>(n1 * np, 1));
        std::vector<uint8_t> ok(std::max<size_t>(n1 * np, 1));
        std::vector<float> x3d(std::max<size_t>(3 * n1 * np, 1));
        orbmi_matcher* mt = lmm();
        SLAM_CHECK(unlocked(ORBMI_SCHED_L_CREATE, k, [&] {
            PhaseTimer pt(&phase_ms[PH_LM_CREATE_CALL]);
            return orbmi_create_new_map_points(mt, &f1, &t1, cos1, has1.data(), &fv1, np, f2.data(), t2.data(),
                                               cos2.data(), mp2.data(), fv2.data(), F12.data(), m12.data(), ok.data(),
                                               x3d.data());
        }));
        std::vector<int> fresh;
        for (int j = 0; j < np; j++) {
            if (pos[j] > 0 && new_keyframes_queued()) break;  // src/LocalMapping.cc:331
            const int k2 = pk[j];
            for (size_t i = 0; i < n1; i++) {
                const size_t r = (size_t)j * n1 + i;
                if (!ok[r]) continue;
                const int i2 = m12[r];
                MapPoint mp;
                mp.id = (int)mps.size();
                std::memcpy(mp.pos, &x3d[3 * r], 3 * sizeof(float));
                mp.ref_kf = k;
                mp.first_kf_id = k;
                mps.push_back(mp);
                add_observation(mp.id, k, (int)i);
                add_observation(mp.id, k2, i2);
                kfs[k].mps[i] = mp.id;
                kfs[k2].mps[i2] = mp.id;
                recent_mps.push_back(mp.id);
                fresh.push_back(mp.id);
            }
        }
        // ComputeDistinctiveDescriptors per point, so one batch for all pairs gives the
        // reference's per-pair results; UpdateNormalAndDepth does not read the descriptor
        normals(fresh);
        owed = std::move(fresh);
        return ORBMI_OK;
    }

    // the same loop with a search call per pair and the host geometry (keyframes without HBM copies)
    int create_new_map_points_host(int k) {
        float ow1[3];
        kf_ow(k, ow1);
        const float mb = s.bf / s.fx;
        std::vector<uint8_t> has1(std::max<size_t>(kfs[k].mps.size(), 1), 0);
        for (size_t i = 0; i < kfs[k].mps.size(); i++) has1[i] = kfs[k].mps[i] >= 0;
        const std::vector<int> neigh(kfs[k].covisible.begin(),
                                     kfs[k].covisible.begin() + std::min<size_t>(10, kfs[k].covisible.size()));
        const size_t n1 = kfs[k].keys.size();
        for (size_t i = 0; i < neigh.size(); i++) {
            if (i > 0 && new_keyframes_queued()) return ORBMI_OK;  // src/LocalMapping.cc:331
            const int k2 = neigh[i];
            float ow2[3];
            kf_ow(k2, ow2);
            const float d[3] = {ow2[0] - ow1[0], ow2[1] - ow1[1], ow2[2] - ow1[2]};
            const float baseline = (float)std::sqrt(((double)d[0] * d[0] + (double)d[1] * d[1]) + (double)d[2] * d[2]);
            if (baseline < mb) continue;
            float F12[9];
            {
                const orbmi_tri_keyframe v1 = tri_view(kfs[k]), v2 = tri_view(kfs[k2]);
                SLAM_CHECK(orbmi_compute_f12(&v1, &v2, F12));
            }
            if (!kfs[k].fv.valid || !kfs[k2].fv.valid) continue;
            std::vector<uint8_t> has2(std::max<size_t>(kfs[k2].mps.size(), 1), 0);
            for (size_t i = 0; i < kfs[k2].mps.size(); i++) has2[i] = kfs[k2].mps[i] >= 0;
            const M4 tcw1 = kfs[k].tcw, tcw2 = kfs[k2].tcw;
            const orbmi_frame_view f1 = kf_view(kfs[k], tcw1.data()), f2 = kf_view(kfs[k2], tcw2.data());
            const orbmi_feature_vector fv1 = kfs[k].fv.view(), fv2 = kfs[k2].fv.view();
            std::vector<int32_t> m12(std::max<size_t>(n1, 1));
            int nm = 0;
            orbmi_matcher* mt = lmm();
            SLAM_CHECK(unlocked(ORBMI_SCHED_L_CREATE_PAIR, (int)i, [&] {
                return orbmi_search_for_triangulation(mt, &f1, has1.data(), &fv1, &f2, has2.data(), &fv2, F12, 0, 0,
                                                      m12.data(), &nm);
            }));
            std::vector<int32_t> idx1, idx2;
            for (size_t i = 0; i < n1; i++)
                if (m12[i] >= 0) { idx1.push_back((int32_t)i); idx2.push_back(m12[i]); }
            if (idx1.empty()) continue;
            std::vector<float> x3d(3 * idx1.size());
            std::vector<uint8_t> ok(idx1.size());
            {
                const orbmi_tri_keyframe v1 = tri_view(kfs[k]), v2 = tri_view(kfs[k2]);
                SLAM_CHECK(orbmi_triangulate_matches(&v1, &v2, idx1.data(), idx2.data(), (int)idx1.size(), x3d.data(),
                                                     ok.data()));
            }
            std::vector<int> fresh;
            for (size_t q = 0; q < idx1.size(); q++) {
                if (!ok[q]) continue;
                const int i1 = idx1[q], i2 = idx2[q];
                MapPoint mp;
                mp.id = (int)mps.size();
                std::memcpy(mp.pos, &x3d[3 * q], 3 * sizeof(float));
                mp.ref_kf = k;
                mp.first_kf_id = k;
                mps.push_back(mp);
                add_observation(mp.id, k, i1);
                add_observation(mp.id, k2, i2);
                kfs[k].mps[i1] = mp.id;
                kfs[k2].mps[i2] = mp.id;
                has1[i1] = 1;
                recent_mps.push_back(mp.id);
                fresh.push_back(mp.id);
            }
            SLAM_CHECK(distinctive(fresh));
            for (int m : fresh) update_normal_and_depth(m);
        }
        return ORBMI_OK;
    }

    // MapPoint::Replace (src/MapPoint.cc:172-215): `other` takes over m's observations; m turns bad.
    // Returns true when other gained them (its descriptor is recomputed before the next search).
    bool replace(int m, int other) {
        if (m == other) return false;
        const ObsMap obs = mps[m].obs;
        mps[m].obs.clear();
        mps[m].bad = true;
        mps[m].replaced = other;
        for (auto& o : obs) {
            if (!mps[other].obs.count(o.first)) {
                kfs[o.first].mps[o.second] = other;  // KeyFrame::ReplaceMapPointMatch
                add_observation(other, o.first, o.second);
            } else {
                kfs[o.first].mps[o.second] = -1;     // KeyFrame::EraseMapPointMatch
            }
        }
        mps[other].found += mps[m].found;
        mps[other].visible += mps[m].visible;
        return true;
    }

    // the search record of a map point (orbmi_mappoint)
    orbmi_mappoint fuse_record(int m) const {
        const MapPoint& mp = mps[m];
        orbmi_mappoint r;
        std::memset(&r, 0, sizeof(r));
        std::memcpy(r.pos, mp.pos, sizeof(r.pos));
        std::memcpy(r.normal, mp.normal, sizeof(r.normal));
        r.max_distance = mp.max_distance;
        r.min_distance = mp.min_distance;
        r.flags = (mp.bad ? ORBMI_MP_BAD : 0u) | (mp.nobs > 0 ? ORBMI_MP_HAS_OBS : 0u);
        std::memcpy(r.desc, mp.desc, 32);
        return r;
    }

    // the search of Fuse(k, pts) on the GPU (map lock released on the mapping thread)
    int fuse_search(int k, const std::vector<int>& pts, std::vector<int32_t>& best) {
        std::vector<orbmi_mappoint> rec(pts.size());
        std::vector<uint8_t> in_kf(pts.size());
        for (size_t j = 0; j < pts.size(); j++) {
            rec[j] = fuse_record(pts[j]);
            in_kf[j] = mps[pts[j]].obs.count(k) ? 1 : 0;
        }
        const M4 tcw = kfs[k].tcw;
        const orbmi_frame_view v = kf_view(kfs[k], tcw.data());
        best.assign(pts.size(), -1);
        std::vector<int32_t> dist(pts.size());
        int nc = 0;
        orbmi_matcher* mt = lmm();
        return unlocked(ORBMI_SCHED_L_FUSE, k, [&] {
            PhaseTimer pt(&phase_ms[PH_LM_FUSE_CALL]);
            return orbmi_fuse_search(mt, &v, rec.data(), in_kf.data(), (int)pts.size(), 3.f, best.data(), dist.data(), &nc);
        });
    }

    // the map updates of Fuse(k, pts) (src/ORBmatcher.cc:1096-1124) in list order
    void fuse_replay(int k, const std::vector<int>& pts, const int32_t* best, std::set<int>& dirty) {
        for (size_t j = 0; j < pts.size(); j++) {
            const int m = pts[j], b = best[j];
            if (mps[m].bad || mps[m].obs.count(k) || b < 0) continue;
            const int in = kfs[k].mps[b];
            if (in >= 0) {
                if (!mps[in].bad) {
                    fuse_touched.insert(m);
                    fuse_touched.insert(in);
                    if (mps[in].nobs > mps[m].nobs) {
                        if (replace(m, in)) { dirty.insert(in); fuse_ops++; }
                    } else if (replace(in, m)) {
                        dirty.insert(m);
                        fuse_ops++;
                    }
                }
            } else {
                fuse_touched.insert(m);
                add_observation(m, k, b);
                kfs[k].mps[b] = m;
                fuse_ops++;
            }
        }
    }

    // ORBmatcher::Fuse(pKF, vpMapPoints, 3.0) (src/ORBmatcher.cc:977-1127): the search for every
    // point on the GPU, then the map updates in list order.  `dirty`: the survivors of Replace
    // whose ComputeDistinctiveDescriptors (MapPoint::Replace, src/MapPoint.cc:212) is still due.
    // The owed descriptors and the search go to the device as one orbmi_fuse_search_refresh call
    // (one round trip): the search reads each due point's record with its new descriptor.
    int fuse(int k, const std::vector<int>& list, std::set<int>& dirty) {
        std::vector<int> due;
        for (int m : dirty)
            if (!mps[m].bad) due.push_back(m);
        dirty.clear();
        std::vector<int> pts;
        for (int m : list)
            if (m >= 0) pts.push_back(m);
        if (pts.empty()) return distinctive(due);
        std::vector<uint8_t> rows;
        std::vector<int32_t> off;
        {
            PhaseTimer pt(&phase_ms[PH_LM_OBSROWS]);
            obs_rows(due, rows, off);
        }
        if (rows.empty()) {  // no descriptor changes: the plain search
            std::vector<int32_t> best;
            SLAM_CHECK(fuse_search(k, pts, best));
            fuse_replay(k, pts, best.data(), dirty);
            return ORBMI_OK;
        }
        const int nd = (int)due.size(), np = (int)pts.size();
        std::vector<orbmi_mappoint> rec(np);
        std::vector<uint8_t> in_kf(np);
        std::vector<int32_t> from(np, -1);
        for (int j = 0; j < np; j++) {
            rec[j] = fuse_record(pts[j]);
            in_kf[j] = mps[pts[j]].obs.count(k) ? 1 : 0;
            auto it = std::lower_bound(due.begin(), due.end(), pts[j]);  // (due ascending: a std::set's order)
            if (it != due.end() && *it == pts[j]) {
                const int d = (int)(it - due.begin());
                if (off[d + 1] > off[d]) from[j] = d;
            }
        }
        std::vector<int32_t> dbest(nd), best(np, -1), bd(np);
        std::vector<uint8_t> dout((size_t)nd * 32);
        for (int d = 0; d < nd; d++) std::memcpy(&dout[32 * d], mps[due[d]].desc, 32);
        const M4 tcw = kfs[k].tcw;
        const orbmi_frame_view v = kf_view(kfs[k], tcw.data());
        orbmi_matcher* mt = lmm();
        SLAM_CHECK(unlocked(ORBMI_SCHED_L_FUSE, k, [&] {
            PhaseTimer pt(&phase_ms[PH_LM_FUSE_CALL]);
            return orbmi_fuse_search_refresh(mt, rows.data(), off.data(), nd, dbest.data(), dout.data(), 1, &v,
                                             rec.data(), from.data(), in_kf.data(), np, 3.f, best.data(), bd.data());
        }));
        for (int d = 0; d < nd; d++)
            if (off[d + 1] > off[d]) std::memcpy(mps[due[d]].desc, &dout[32 * d], 32);
        fuse_replay(k, pts, best.data(), dirty);
        return ORBMI_OK;
    }

    // Fuse(target, the keyframe's points) for every target in order (src/LocalMapping.cc:620-628).
    // The searches of all targets run in one orbmi_fuse_search_batch on the records as they are
    // before the first target; a point's search depends only on its own record, its IsInKeyFrame
    // and the target, so a target's batch result is the reference's wherever neither changed in
    // the earlier targets' replays -- the points where one did (a Replace survivor's descriptor or
    // observations) are searched again before that target's replay.  ComputeDistinctiveDescriptors
    // of a survivor is done before the first read of its record (a survivor gains no observation
    // from AddObservation before then: only listed points do, and a listed dirty point is
    // recomputed before the target that could add one).
    // `owed`: points whose descriptors CreateNewMapPoints left to compute -- computed in the same
    // device call as the batched searches, which read them.
    int fuse_targets(const std::vector<int>& targets, const std::vector<int>& list, std::set<int>& dirty,
                     const std::vector<int>& owed) {
        std::vector<int> pts;
        for (int m : list)
            if (m >= 0) pts.push_back(m);
        const int nt = (int)targets.size(), np = (int)pts.size();
        if (nt == 0 || np == 0) return distinctive(owed);
        auto* prep = new PhaseTimer(&phase_ms[PH_LM_SIN_PREP]);
        fuse_touched.clear();
        std::vector<orbmi_mappoint> rec0(np);
        for (int j = 0; j < np; j++) rec0[j] = fuse_record(pts[j]);
        std::vector<uint8_t> in0((size_t)nt * np);
        std::vector<M4> tcw(nt);
        std::vector<orbmi_frame_view> views(nt);
        for (int t = 0; t < nt; t++) {
            for (int j = 0; j < np; j++) in0[(size_t)t * np + j] = mps[pts[j]].obs.count(targets[t]) ? 1 : 0;
            tcw[t] = kfs[targets[t]].tcw;
            views[t] = kf_view(kfs[targets[t]], tcw[t].data());
        }
        std::vector<int32_t> best((size_t)nt * np), dist((size_t)nt * np);
        orbmi_matcher* mt = lmm();
        // the owed descriptors (ascending ids, as created) and the records that take them
        std::vector<int> due;
        for (int m : owed)
            if (!mps[m].bad) due.push_back(m);
        std::vector<uint8_t> orows;
        std::vector<int32_t> ooff, ofrom;
        obs_rows(due, orows, ooff);
        const int nd = (int)due.size();
        std::vector<uint8_t> odesc;
        if (!orows.empty()) {
            ofrom.assign(np, -1);
            for (int j = 0; j < np; j++) {
                auto it = std::lower_bound(due.begin(), due.end(), pts[j]);
                if (it != due.end() && *it == pts[j]) {
                    const int d = (int)(it - due.begin());
                    if (ooff[d + 1] > ooff[d]) ofrom[j] = d;
                }
            }
            odesc.resize((size_t)nd * 32);
            for (int d = 0; d < nd; d++) std::memcpy(&odesc[32 * d], mps[due[d]].desc, 32);
        }
        delete prep;
        SLAM_CHECK(unlocked(ORBMI_SCHED_L_FUSE_BATCH, -1, [&] {
            PhaseTimer pt(&phase_ms[PH_LM_FUSE_CALL]);
            if (orows.empty())
                return orbmi_fuse_search_batch(mt, nt, views.data(), rec0.data(), in0.data(), np, 3.f, best.data(),
                                               dist.data(), nullptr);
            std::vector<int32_t> dbest(nd);
            return orbmi_fuse_search_refresh(mt, orows.data(), ooff.data(), nd, dbest.data(), odesc.data(), nt,
                                             views.data(), rec0.data(), ofrom.data(), in0.data(), np, 3.f, best.data(),
                                             dist.data());
        }));
        if (!orows.empty()) {
            for (int d = 0; d < nd; d++)
                if (ooff[d + 1] > ooff[d]) std::memcpy(mps[due[d]].desc, &odesc[32 * d], 32);
            for (int j = 0; j < np; j++)
                if (ofrom[j] >= 0) std::memcpy(rec0[j].desc, &odesc[32 * ofrom[j]], 32);
        }
        std::map<int, int> listed;  // point -> its (first) position in pts
        for (int j = np - 1; j >= 0; j--) listed[pts[j]] = j;
        for (int t = 0; t < nt; t++) {
            const int kt = targets[t];
            std::vector<int> due;
            for (auto it = dirty.begin(); it != dirty.end();) {
                if (listed.count(*it)) {
                    if (!mps[*it].bad) due.push_back(*it);
                    it = dirty.erase(it);
                } else {
                    ++it;
                }
            }
            if (!due.empty()) {
                // one device call: the due descriptors, and the searches of the listed records that
                // take them against this and every later target (their batch rows are stale)
                std::vector<uint8_t> rows;
                std::vector<int32_t> off;
                obs_rows(due, rows, off);
                const int nd = (int)due.size();
                std::vector<int> rj;  // positions in pts of the listed occurrences of due points
                std::vector<int32_t> from;
                for (int d = 0; d < nd; d++)
                    for (int j = 0; j < np; j++)
                        if (pts[j] == due[d]) {
                            rj.push_back(j);
                            from.push_back(off[d + 1] > off[d] ? d : -1);
                        }
                const int nr = (int)rj.size(), ntr = nt - t;
                std::vector<orbmi_mappoint> rrec(std::max(nr, 1));
                std::vector<uint8_t> rin(std::max((size_t)nr * ntr, (size_t)1));
                std::vector<orbmi_frame_view> rv(views.begin() + t, views.end());
                for (int q = 0; q < nr; q++) {
                    rrec[q] = fuse_record(pts[rj[q]]);
                    for (int u = 0; u < ntr; u++) rin[(size_t)u * nr + q] = mps[pts[rj[q]]].obs.count(targets[t + u]) ? 1 : 0;
                }
                std::vector<int32_t> dbest(nd), bi((size_t)std::max(nr * ntr, 1)), bd((size_t)std::max(nr * ntr, 1));
                std::vector<uint8_t> dout((size_t)nd * 32);
                for (int d = 0; d < nd; d++) std::memcpy(&dout[32 * d], mps[due[d]].desc, 32);
                orbmi_matcher* mt2 = lmm();
                SLAM_CHECK(unlocked(ORBMI_SCHED_L_FUSE_REFRESH, t, [&] {
                    PhaseTimer pt(&phase_ms[PH_LM_FUSE_CALL]);
                    return orbmi_fuse_search_refresh(mt2, rows.empty() ? nullptr : rows.data(), off.data(), nd,
                                                     dbest.data(), dout.data(), ntr, rv.data(), rrec.data(),
                                                     from.data(), rin.data(), nr, 3.f, bi.data(), bd.data());
                }));
                for (int d = 0; d < nd; d++)
                    if (off[d + 1] > off[d]) std::memcpy(mps[due[d]].desc, &dout[32 * d], 32);
                for (int q = 0; q < nr; q++) {
                    rec0[rj[q]] = fuse_record(pts[rj[q]]);
                    for (int u = 0; u < ntr; u++) best[(size_t)(t + u) * np + rj[q]] = bi[(size_t)u * nr + q];
                }
            }
            int32_t* row = best.data() + (size_t)t * np;
            std::vector<int> redo_pts, redo_j;
            auto* rt = new PhaseTimer(&phase_ms[PH_LM_SIN_REDO]);
            // A record can change here only through an earlier target's replay (Replace, a new
            // observation: fuse_touched) -- Tracking creates points but changes no existing
            // point's position, normal, distances, flags or descriptor, and the refreshed
            // descriptors are in rec0 -- so only touched points are compared.  With recording on
            // (the parity tests) every point is compared too and a difference fails the call.
            for (int j = 0; j < np; j++) {
                const int m = pts[j];
                // the replay skips bad points and points already in the target (observations are
                // only gained here, so a point in the target now was in it or is skipped anyway)
                if (!recording && !fuse_touched.count(m)) continue;
                if (mps[m].bad || mps[m].obs.count(kt)) continue;
                const orbmi_mappoint r = fuse_record(m);
                if (std::memcmp(&r, &rec0[j], sizeof(r)) != 0) {
                    if (!fuse_touched.count(m)) {
                        delete rt;
                        fprintf(stderr, "orbmi_slam: Fuse record of point %d changed untouched\n", m);
                        return ORBMI_E_STATE;
                    }
                    redo_pts.push_back(m);
                    redo_j.push_back(j);
                }
            }
            delete rt;
            if (!redo_pts.empty()) {
                std::vector<int32_t> b2;
                SLAM_CHECK(fuse_search(kt, redo_pts, b2));
                for (size_t q = 0; q < redo_j.size(); q++) row[redo_j[q]] = b2[q];
            }
            PhaseTimer rp(&phase_ms[PH_LM_SIN_REPLAY]);
            fuse_replay(kt, pts, row, dirty);
        }
        return ORBMI_OK;
    }

    // owed2 <- the keyframe's points, whose ComputeDistinctiveDescriptors (:656-667) the caller does
    // -- in LocalBA's device window when that runs next.  UpdateNormalAndDepth and UpdateConnections
    // do not read descriptors and are done here.
    int search_in_neighbors(int k, const std::vector<int>& owed, std::vector<int>& owed2) {  // src/LocalMapping.cc:589-674, stereo: nn = 10
        std::vector<int> targets;
        const std::vector<int> neigh(kfs[k].covisible.begin(),
                                     kfs[k].covisible.begin() + std::min<size_t>(10, kfs[k].covisible.size()));
        for (int k1 : neigh) {
            if (kfs[k1].bad || kfs[k1].fuse_target_for_kf == k) continue;
            targets.push_back(k1);
            kfs[k1].fuse_target_for_kf = k;
            const std::vector<int> second(kfs[k1].covisible.begin(),
                                          kfs[k1].covisible.begin() + std::min<size_t>(5, kfs[k1].covisible.size()));
            for (int k2 : second) {
                if (kfs[k2].bad || kfs[k2].fuse_target_for_kf == k || k2 == k) continue;
                targets.push_back(k2);
            }
        }
        std::set<int> dirty;
        const std::vector<int> matches = kfs[k].mps;
        SLAM_CHECK(fuse_targets(targets, matches, dirty, owed));
        std::vector<int> cands;
        for (int t : targets)
            for (int m : kfs[t].mps) {
                if (m < 0 || mps[m].bad || mps[m].fuse_candidate_for_kf == k) continue;
                mps[m].fuse_candidate_for_kf = k;
                cands.push_back(m);
            }
        SLAM_CHECK(fuse(k, cands, dirty));
        dirty.clear();
        std::vector<int> upd;
        std::set<int> seen_pt;
        for (int m : kfs[k].mps)
            if (m >= 0 && !mps[m].bad && seen_pt.insert(m).second) upd.push_back(m);
        normals(upd);
        connections(k);
        owed2 = std::move(upd);
        return ORBMI_OK;
    }

    // ---- KeyFrameCulling (src/LocalMapping.cc:775-841) and KeyFrame::SetBadFlag -------------------
    void erase_connection(int k, int other) {  // KeyFrame::EraseConnection + UpdateBestCovisibles
        if (kfs[k].conn.erase(other)) sort_covisible(kfs[k]);
    }

    int get_weight(int k, int other) const {
        auto it = kfs[k].conn.find(other);
        return it == kfs[k].conn.end() ? 0 : it->second;
    }

    void change_parent(int k, int p) {
        kfs[k].parent = p;
        auto& ch = kfs[p].children;
        if (std::find(ch.begin(), ch.end(), k) == ch.end()) ch.push_back(k);
    }

    void set_bad_keyframe(int k) {  // KeyFrame::SetBadFlag (src/KeyFrame.cc:467-559)
        if (kfs[k].id == 0) return;
        const std::map<int, int> conn = kfs[k].conn;
        for (auto& c : conn) erase_connection(c.first, k);
        for (int m : std::vector<int>(kfs[k].mps))
            if (m >= 0) erase_observation(m, k);
        kfs[k].conn.clear();
        kfs[k].covisible.clear();
        std::set<int> candidates{kfs[k].parent};
        std::vector<int> children = kfs[k].children;
        std::sort(children.begin(), children.end());
        while (!children.empty()) {
            bool cont = false;
            int best = -1, pc = -1, pp = -1;
            for (int c : children) {
                if (kfs[c].bad) continue;
                for (int cv : kfs[c].covisible)
                    for (int cand : candidates)
                        if (cv == cand) {
                            const int w = get_weight(c, cv);
                            if (w > best) { pc = c; pp = cv; best = w; cont = true; }
                        }
            }
            if (!cont) break;
            change_parent(pc, pp);
            candidates.insert(pc);
            children.erase(std::find(children.begin(), children.end(), pc));
            auto& own = kfs[k].children;
            own.erase(std::find(own.begin(), own.end(), pc));
        }
        const int parent = kfs[k].parent;
        for (int c : children) change_parent(c, parent);
        kfs[k].children.clear();
        auto& pch = kfs[parent].children;
        auto it = std::find(pch.begin(), pch.end(), k);
        if (it != pch.end()) pch.erase(it);
        kfs[k].tcp = mul(kfs[k].tcw, pose_inverse(kfs[parent].tcw));
        kfs[k].bad = true;
    }

    void keyframe_culling(int k) {
        const std::vector<int> local = kfs[k].covisible;
        for (int kk : local) {
            const KeyFrame& kf = kfs[kk];
            if (kf.id == 0) continue;
            int n_mps = 0, n_red = 0;
            for (size_t i = 0; i < kf.mps.size(); i++) {
                const int m = kf.mps[i];
                if (m < 0 || mps[m].bad) continue;
                if (kf.depth[i] > s.th_depth || kf.depth[i] < 0) continue;
                n_mps++;
                if (mps[m].nobs > 3) {
                    const int level = kf.keys[i].octave;
                    int n = 0;
                    for (auto& o : mps[m].obs) {
                        if (o.first == kk) continue;
                        if (kfs[o.first].keys[o.second].octave <= level + 1 && ++n >= 3) break;
                    }
                    if (n >= 3) n_red++;
                }
            }
            if (n_red > 0.9 * n_mps) set_bad_keyframe(kk);
        }
    }

    // Optimizer::LocalBundleAdjustment: the graph as src/Optimizer.cc:486-683 assembles it
    // (system/optimizer.gather_local_ba), the optimisation on the GPU, the write-back (:776-805)
    // `owed`: points whose ComputeDistinctiveDescriptors runs in the same device window as the
    // optimisation (the descriptors written back with the poses)
    int local_bundle_adjustment(int k, const std::vector<int>& owed) {
        auto* gt = new PhaseTimer(&phase_ms[PH_LM_BA_GATHER]);
        std::vector<int> lkf{k};
        SeenSet& local_set = ba_local_mark;
        local_set.clear();
        local_set.insert(k);
        for (int c : kfs[k].covisible) {
            local_set.insert(c);
            if (!kfs[c].bad) lkf.push_back(c);
        }
        std::vector<int> lmp;
        SeenSet& seen_mp = ba_mp_mark;
        seen_mp.clear();
        for (int kk : lkf)
            for (int m : kfs[kk].mps)
                if (m >= 0 && !mps[m].bad && !seen_mp.count(m)) {
                    seen_mp.insert(m);
                    lmp.push_back(m);
                }
        std::vector<int> fixed;
        SeenSet& fixed_set = ba_fixed_mark;
        fixed_set.clear();
        for (int m : lmp)
            for (auto& o : mps[m].obs)
                if (!local_set.count(o.first) && !fixed_set.count(o.first)) {
                    fixed_set.insert(o.first);
                    if (!kfs[o.first].bad) fixed.push_back(o.first);
                }
        std::vector<int> all = lkf;
        all.insert(all.end(), fixed.begin(), fixed.end());
        std::vector<int> kidx(kfs.size(), -1);  // keyframe id -> its vertex
        for (int i = 0; i < (int)all.size(); i++) kidx[all[i]] = i;
        std::vector<orbmi_ba_keyframe> K(all.size());
        for (int i = 0; i < (int)all.size(); i++) {
            const KeyFrame& kf = kfs[all[i]];
            std::memcpy(K[i].tcw, kf.tcw.data(), sizeof(K[i].tcw));
            K[i].id = (uint32_t)kf.id;
            K[i].fixed = (i >= (int)lkf.size() || kf.id == 0) ? 1 : 0;
            K[i].fx = s.fx; K[i].fy = s.fy; K[i].cx = s.cx; K[i].cy = s.cy; K[i].bf = s.bf;
        }
        std::vector<orbmi_ba_point> P(lmp.size());
        for (int j = 0; j < (int)lmp.size(); j++) {
            const MapPoint& mp = mps[lmp[j]];
            std::memcpy(P[j].pos, mp.pos, sizeof(P[j].pos));
            P[j].id = (uint32_t)mp.id;
            P[j].bad = mp.bad ? 1 : 0;
        }
        std::vector<orbmi_ba_edge> E;
        std::vector<std::pair<int, int>> e_ref;  // (map point id, keyframe id) per edge
        for (int j = 0; j < (int)lmp.size(); j++)
            for (auto& o : mps[lmp[j]].obs) {
                const int vi = kidx[o.first];
                if (kfs[o.first].bad || vi < 0) continue;
                const KeyFrame& kf = kfs[o.first];
                const orbmi_keypoint& kp = kf.keys[o.second];
                E.push_back(orbmi_ba_edge{j, vi, kp.x, kp.y, kf.ur[o.second], inv_level_sigma2[kp.octave]});
                e_ref.push_back({lmp[j], o.first});
            }
        delete gt;
        if (E.empty()) return distinctive(owed);
        std::vector<uint8_t> orows;
        std::vector<int32_t> ooff;
        {
            PhaseTimer pt(&phase_ms[PH_LM_OBSROWS]);
            obs_rows(owed, orows, ooff);
        }
        const int nod = (int)owed.size();
        std::vector<int32_t> obest(std::max(nod, 1));
        std::vector<uint8_t> oout((size_t)std::max(nod, 1) * 32);
        auto owed_call = [&]() -> int {
            if (orows.empty()) return ORBMI_OK;
            PhaseTimer pt(&phase_ms[PH_LM_DISTINCTIVE_CALL]);
            return orbmi_compute_distinctive_descriptors(lmm(), orows.data(), ooff.data(), nod, obest.data(), oout.data());
        };
        orbmi_ba_problem prob{(int)K.size(), (int)P.size(), (int)E.size(), K.data(), P.data(), E.data()};
        std::vector<float> tcw(K.size() * 16), pos(P.size() * 3 + 3);
        std::vector<uint8_t> erase(E.size());
        orbmi_ba_result res{};
        res.tcw = tcw.data();
        res.pos = pos.data();
        res.erase = erase.data();
        int rc;
        std::unique_lock<std::mutex> update_guard;  // held to the end of the write-back
        if (held_lock && on_mapping_thread) {  // tracking runs while the GPU solves
            hold_end();
            held_lock->unlock();
            rc = owed_call();
            if (!rc) {
                PhaseTimer ct(&phase_ms[PH_LM_BA_CALL]);
                rc = orbmi_local_bundle_adjustment(ba, &prob, &res, &abort_ba);
            }
            PhaseTimer lt(&phase_ms[PH_LM_LOCK]);
            update_guard = std::unique_lock<std::mutex>(update_mtx);  // (lock order: update, map)
            held_lock->lock();
            log_section(ORBMI_SCHED_L_BA, k);
        } else {
            rc = owed_call();
            PhaseTimer ct(&phase_ms[PH_LM_BA_CALL]);
            if (!rc) rc = orbmi_local_bundle_adjustment(ba, &prob, &res, nullptr);
        }
        SLAM_CHECK(rc);
        for (int j = 0; j < nod; j++)  // the owed descriptors (under the map lock again)
            if (ooff[j + 1] > ooff[j]) std::memcpy(mps[owed[j]].desc, &oout[32 * j], 32);
        PhaseTimer wb(&phase_ms[PH_LM_BA_WRITEBACK]);
        ba_calls++;
        if (res.aborted) ba_aborted++;
        else if (res.stop_check >= 0) ba_interrupted++;
        {
            int erased = 0;
            for (uint8_t x : erase) erased += x != 0;
            if (recording)
                ba_log.push_back(orbmi_slam_ba_record{k, res.stop_check, res.aborted, res.checks,
                                                  {res.iterations[0], res.iterations[1]}, (int)E.size(), erased});
        }
        if (res.aborted) return ORBMI_OK;  // src/Optimizer.cc:685-687: no write-back
        for (size_t e = 0; e < E.size(); e++) {
            if (!erase[e]) continue;
            const int m = e_ref[e].first, kk = e_ref[e].second;
            auto it = mps[m].obs.find(kk);
            if (it != mps[m].obs.end() && kfs[kk].mps[it->second] == m) kfs[kk].mps[it->second] = -1;  // EraseMapPointMatch
            erase_observation(m, kk);
        }
        int n_local = 1;
        for (int c : kfs[k].covisible)
            if (!kfs[c].bad) n_local++;
        for (int i = 0; i < n_local; i++) std::memcpy(kfs[all[i]].tcw.data(), &tcw[16 * i], 16 * sizeof(float));
        for (int j = 0; j < (int)lmp.size(); j++) std::memcpy(mps[lmp[j]].pos, &pos[3 * j], 3 * sizeof(float));
        for (int m : lmp) update_normal_and_depth(m);
        return ORBMI_OK;
    }

    // ---- tracking stages ----------------------------------------------------------------------
    std::vector<orbmi_mappoint> mp_records(const std::vector<int>& pts) const {
        std::vector<orbmi_mappoint> rec(pts.size());
        mp_records_into(pts, rec.data());
        return rec;
    }
    void mp_records_into(const std::vector<int>& pts, orbmi_mappoint* rec) const {
        for (size_t j = 0; j < pts.size(); j++) {
            const MapPoint& mp = mps[pts[j]];
            orbmi_mappoint& r = rec[j];
            std::memcpy(r.pos, mp.pos, sizeof(r.pos));
            std::memcpy(r.normal, mp.normal, sizeof(r.normal));
            r.max_distance = mp.max_distance;
            r.min_distance = mp.min_distance;
            r.flags = (mp.bad ? ORBMI_MP_BAD : 0u) | (seen.count(mp.id) ? ORBMI_MP_SEEN : 0u) |
                      (mp.nobs > 0 ? ORBMI_MP_HAS_OBS : 0u);
            std::memcpy(r.desc, mp.desc, 32);
        }
    }

    std::vector<orbmi_lastframe_point> lf_records(const std::vector<int>& lf_mps, const std::vector<uint8_t>* outlier) const {
        std::vector<orbmi_lastframe_point> rec(std::max<size_t>(lf_mps.size(), 1));
        lf_records_into(lf_mps, outlier, rec.data());
        rec.resize(lf_mps.size());
        return rec;
    }
    void lf_records_into(const std::vector<int>& lf_mps, const std::vector<uint8_t>* outlier,
                         orbmi_lastframe_point* rec) const {
        std::memset(rec, 0, std::max<size_t>(lf_mps.size(), 1) * sizeof(orbmi_lastframe_point));
        for (size_t i = 0; i < lf_mps.size(); i++) {
            const int m = lf_mps[i];
            if (m < 0) continue;
            std::memcpy(rec[i].pos, mps[m].pos, sizeof(rec[i].pos));
            std::memcpy(rec[i].desc, mps[m].desc, 32);
            rec[i].flags = ORBMI_LF_HAS_MP | (mps[m].nobs > 0 ? ORBMI_MP_HAS_OBS : 0u) |
                           (outlier && (*outlier)[i] ? ORBMI_LF_OUTLIER : 0u);
        }
    }

    int discard_outliers(TrackedFrame& cf, const std::vector<uint8_t>& outlier) {  // -> nmatchesMap
        int nmap = 0;
        for (int i = 0; i < cf.n(); i++) {
            const int m = cf.mps[i];
            if (m < 0) continue;
            if (outlier[i]) {
                cf.mps[i] = -1;
                cf.outlier[i] = 0;
                seen.insert(m);  // pMP->mnLastFrameSeen = mCurrentFrame.mnId
            } else if (mps[m].nobs > 0) {
                nmap++;
            }
        }
        return nmap;
    }

    int track_reference_kf(TrackedFrame& cf, orbmi_slam_frame_stats& st, bool& ok) {  // src/Tracking.cc:871-917
        ok = false;
        SLAM_CHECK(compute_bow(cf.desc, cf.fv));
        KeyFrame& kf = kfs[ref_kf];
        if (!kf.fv.valid) SLAM_CHECK(compute_bow(kf.desc, kf.fv));
        std::vector<uint8_t> ok_mp(std::max<size_t>(kf.mps.size(), 1), 0);
        for (size_t j = 0; j < kf.mps.size(); j++) ok_mp[j] = kf.mps[j] >= 0 && !mps[kf.mps[j]].bad;
        const M4 kf_tcw = kf.tcw;
        const orbmi_frame_view vk = kf_view(kf, kf_tcw.data());
        const M4 I = eye4();
        const orbmi_frame_view vf = view(cf, I.data());
        const orbmi_feature_vector fk = kf.fv.view(), ff = cf.fv.view();
        const std::vector<int> kf_mps = kf.mps;  // the keyframe's matches when the search ran
        std::vector<int32_t> m(std::max(cf.n(), 1));
        int n = 0;
        SLAM_CHECK(unlocked(ORBMI_SCHED_T_BOW, cf.id, [&] {
            return orbmi_search_by_bow(matcher, &vk, ok_mp.data(), &fk, &vf, &ff, 0.7f, 1, m.data(), &n);
        }));
        st.bow_matches = n;
        st.track = 2;
        if (n < 15) return ORBMI_OK;
        for (int i = 0; i < cf.n(); i++) cf.mps[i] = m[i] >= 0 ? kf_mps[m[i]] : -1;
        cf.tcw = last_frame.tcw;
        cf.has_tcw = true;
        const std::vector<orbmi_lastframe_point> lfp = lf_records(kf_mps, nullptr);
        m.resize(cf.n());
        M4 tcw;
        std::vector<uint8_t> out;
        SLAM_CHECK(pose_optimization(cf, m, lfp, tcw, out));
        cf.tcw = tcw;
        cf.outlier = out;
        seen.clear();
        const int nmap = discard_outliers(cf, out);
        st.nmatches_map = nmap;
        ok = nmap >= 10;
        return ORBMI_OK;
    }

    int track_motion_model_staged(TrackedFrame& cf, orbmi_slam_frame_stats& st, bool& ok) {  // src/Tracking.cc:997-1063
        ok = false;
        TrackedFrame& lf = last_frame;
        lf.tcw = mul(rel_poses.back(), kfs[lf.ref_kf].tcw);  // UpdateLastFrame (pose only, SLAM mode)
        cf.tcw = mul(velocity, lf.tcw);
        cf.has_tcw = true;
        const std::vector<orbmi_lastframe_point> lfp = lf_records(lf.mps, &lf.outlier);
        std::vector<uint8_t> occ(std::max(cf.n(), 1), 0);
        const orbmi_frame_view vc = view(cf, cf.tcw.data()), vl = view(lf, lf.tcw.data());
        std::vector<int32_t> m(std::max(cf.n(), 1));
        int n = 0;
        const float th = 7.f;  // stereo (src/Tracking.cc:1011-1014)
        {
            PhaseTimer pt(&phase_ms[PH_LF_SEARCH]);
            SLAM_CHECK(unlocked(ORBMI_SCHED_T_LF, cf.id, [&] {
                int rc = orbmi_search_by_projection_last_frame(matcher, &vc, occ.data(), &vl, lfp.data(), th, 0, 1,
                                                               m.data(), &n);
                if (!rc && n < 20)
                    rc = orbmi_search_by_projection_last_frame(matcher, &vc, occ.data(), &vl, lfp.data(), 2 * th, 0, 1,
                                                               m.data(), &n);
                return rc;
            }));
        }
        st.track = 1;
        st.lf_matches = n;
        if (n < 20) return ORBMI_OK;
        for (int i = 0; i < cf.n(); i++) cf.mps[i] = m[i] >= 0 ? lf.mps[m[i]] : -1;
        m.resize(cf.n());
        M4 tcw;
        std::vector<uint8_t> out;
        {
            PhaseTimer pt(&phase_ms[PH_LF_POSE]);
            SLAM_CHECK(pose_optimization(cf, m, lfp, tcw, out));
        }
        cf.tcw = tcw;
        cf.outlier = out;
        seen.clear();
        const int nmap = discard_outliers(cf, out);
        st.nmatches_map = nmap;
        ok = nmap >= 10;
        return ORBMI_OK;
    }

    void update_local_keyframes(TrackedFrame& cf) {  // src/Tracking.cc:1452-1580
        // keyframe counter in keyframe-id order (the std::map<KeyFrame*, int> of the reference,
        // id-ordered here): counts per id, touched ids sorted
        if (kf_counter.size() < kfs.size()) kf_counter.resize(kfs.size(), 0);
        std::vector<int> touched;
        for (int i = 0; i < cf.n(); i++) {
            const int m = cf.mps[i];
            if (m < 0) continue;
            if (mps[m].bad) { cf.mps[i] = -1; continue; }
            for (auto& o : mps[m].obs)
                if (kf_counter[o.first]++ == 0) touched.push_back(o.first);
        }
        if (touched.empty()) return;
        std::sort(touched.begin(), touched.end());
        int best = 0, kfmax = -1;
        std::vector<int> local;
        local_kf_mark.clear();  // mnTrackReferenceForFrame of the keyframes (generation stamps)
        SeenSet& mark = local_kf_mark;
        for (int id : touched) {
            const int cnt = kf_counter[id];
            kf_counter[id] = 0;
            if (kfs[id].bad) continue;
            if (cnt > best) { best = cnt; kfmax = id; }
            local.push_back(id);
            mark.insert(id);
        }
        size_t i = 0;
        std::vector<int> ch;
        while (i < local.size()) {
            if (local.size() > 80) break;
            const int k = local[i++];
            const std::vector<int>& cov = kfs[k].covisible;
            const size_t ncov = std::min<size_t>(10, cov.size());
            for (size_t c = 0; c < ncov; c++) {  // the first 10 (the list may grow below: by index)
                const int nb = kfs[k].covisible[c];
                if (!kfs[nb].bad && !mark.count(nb)) { local.push_back(nb); mark.insert(nb); break; }
            }
            ch.assign(kfs[k].children.begin(), kfs[k].children.end());
            std::sort(ch.begin(), ch.end());
            for (int c : ch)
                if (!kfs[c].bad && !mark.count(c)) { local.push_back(c); mark.insert(c); break; }
            const int p = kfs[k].parent;
            if (p >= 0 && !mark.count(p)) {
                local.push_back(p);
                mark.insert(p);
                break;
            }
        }
        local_kfs = local;
        if (kfmax >= 0) {
            ref_kf = kfmax;
            cf.ref_kf = kfmax;
        }
    }

    void update_local_points() {  // src/Tracking.cc:1421-1450
        std::vector<int> out;
        local_mark.clear();
        for (int k : local_kfs)
            for (int m : kfs[k].mps)
                if (m >= 0 && !local_mark.count(m) && !mps[m].bad) {
                    out.push_back(m);
                    local_mark.insert(m);
                }
        local_mps.swap(out);
    }

    int track_local_map_staged(TrackedFrame& cf, orbmi_slam_frame_stats& st, bool& ok) {  // src/Tracking.cc:1075-1104
        ok = false;
        {
            PhaseTimer pt(&phase_ms[PH_LOCAL_UPDATE]);
            update_local_keyframes(cf);
            update_local_points();
        }
        std::vector<uint8_t> occ(std::max(cf.n(), 1), 0);
        for (int i = 0; i < cf.n(); i++) {  // SearchLocalPoints' first loop
            const int m = cf.mps[i];
            if (m < 0) continue;
            if (mps[m].bad) cf.mps[i] = -1;
            else {
                mps[m].visible++;  // IncreaseVisible
                seen.insert(m);
                occ[i] = mps[m].nobs > 0 ? 1 : 0;
            }
        }
        PhaseTimer* ptr = new PhaseTimer(&phase_ms[PH_LOCAL_RECORDS]);
        const std::vector<orbmi_mappoint> rec = mp_records(local_mps);
        delete ptr;
        const orbmi_frame_view vc = view(cf, cf.tcw.data());
        std::vector<int32_t> m_mp(std::max(cf.n(), 1), -1);
        int nl = 0;
        // isInFrustum(0.5) -> IncreaseVisible, then SearchByProjection(F, points, th = 1), 0.8: one
        // fused call (with no point in view the search finds nothing, as the reference's skipped one)
        std::vector<orbmi_mappoint_track> tr(std::max<size_t>(rec.size(), 1));
        {
            PhaseTimer pt(&phase_ms[PH_LOCAL_SEARCH]);
            SLAM_CHECK(unlocked(ORBMI_SCHED_T_LOCAL, cf.id, [&] {
                return orbmi_search_local_points_track(matcher, &vc, occ.data(), rec.data(), (int)rec.size(), 1.f,
                                                       m_mp.data(), &nl, nullptr, tr.data());
            }));
        }
        for (size_t j = 0; j < rec.size(); j++)
            if (tr[j].in_view) mps[local_mps[j]].visible++;
        st.local_map_points = (int)local_mps.size();
        st.local_matches = nl;
        std::vector<int> cur = cf.mps;
        for (int i = 0; i < cf.n(); i++)
            if (m_mp[i] >= 0) cur[i] = local_mps[m_mp[i]];
        const std::vector<orbmi_lastframe_point> lfp = lf_records(cur, nullptr);
        std::vector<int32_t> m_lf(cf.n(), -1);
        for (int i = 0; i < cf.n(); i++)
            if (cur[i] >= 0) m_lf[i] = i;
        M4 tcw;
        std::vector<uint8_t> out;
        {
            PhaseTimer pt(&phase_ms[PH_LOCAL_POSE]);
            SLAM_CHECK(pose_optimization(cf, m_lf, lfp, tcw, out));
        }
        cf.tcw = tcw;
        cf.mps = cur;
        cf.outlier = out;
        int inliers = 0;
        for (int i = 0; i < cf.n(); i++) {  // (:1087-1101)
            const int m = cf.mps[i];
            if (m < 0) continue;
            if (!cf.outlier[i]) {
                mps[m].found++;  // IncreaseFound
                if (mps[m].nobs > 0) inliers++;
            } else if (cf.ur[i] >= 0) {
                cf.mps[i] = -1;  // stereo outliers are dropped
            }
        }
        matches_inliers = inliers;
        st.inliers = inliers;
        ok = inliers >= 30;
        return ORBMI_OK;
    }

    // the per-call staged path (ORBMI_SLAM_STAGED=1): every operator call stages its host inputs
    // and synchronises; the default enqueues a stage's operators behind one upload
    const bool staged_track = getenv("ORBMI_SLAM_STAGED") != nullptr;
    int track_motion_model(TrackedFrame& cf, orbmi_slam_frame_stats& st, bool& ok) {
        return staged_track ? track_motion_model_staged(cf, st, ok) : track_motion_model_dev(cf, st, ok);
    }
    int track_local_map(TrackedFrame& cf, orbmi_slam_frame_stats& st, bool& ok) {
        return staged_track ? track_local_map_staged(cf, st, ok) : track_local_map_dev(cf, st, ok);
    }

    // Tracking::TrackWithMotionModel (src/Tracking.cc:997-1063), device-resident: the last frame's
    // point records go up once; SearchByProjection(CF, LF, 7) and the retry at 14 when fewer than
    // 20 matched (the count stays on the device), PoseOptimization on those matches, then one
    // read-back.  The pose optimisation is enqueued even when the search will have found fewer
    // than 20 matches; the host then ignores it, as the reference never runs it.
    int track_motion_model_dev(TrackedFrame& cf, orbmi_slam_frame_stats& st, bool& ok) {
        ok = false;
        TrackedFrame& lf = last_frame;
        lf.tcw = mul(rel_poses.back(), kfs[lf.ref_kf].tcw);  // UpdateLastFrame (pose only, SLAM mode)
        cf.tcw = mul(velocity, lf.tcw);
        cf.has_tcw = true;
        const int nc = cf.n(), nl = lf.n();
        SLAM_CHECK(track_buffers(nc, nl, 0));
        TrackBuf& t = tb;
        lf_records_into(lf.mps, &lf.outlier, t.h_lfp);
        std::memset(t.h_occ, 0, (size_t)std::max(nc, 1));
        *t.h_n = 0;
        SLAM_CHECK(up_range(t.h_occ, t.h_n + 1));  // occ, the last frame's points, n = 0
        const orbmi_frame_view vc = view(cf, cf.tcw.data()), vl = view(lf, lf.tcw.data());
        const float th = 7.f;  // stereo (src/Tracking.cc:1011-1014)
        orbmi_frame_mappoints fm{};
        fm.match_lf = t.d_m;
        fm.lf_points = t.d_lfp;
        fm.n_lf_points = nl;
        {
            PhaseTimer pt(&phase_ms[PH_LF_SEARCH]);
            SLAM_CHECK(unlocked(ORBMI_SCHED_T_LF, cf.id, [&] {
                int rc = orbmi_search_by_projection_last_frame_if(matcher, &vc, t.d_occ, &vl, t.d_lfp, th, 0, 1, t.d_m,
                                                                  t.d_n, 1);
                if (!rc) rc = orbmi_search_by_projection_last_frame_if(matcher, &vc, t.d_occ, &vl, t.d_lfp, 2 * th, 0, 1,
                                                                       t.d_m, t.d_n, 20);
                if (!rc) rc = orbmi_pose_optimization_frame(pose, &vc, inv_level_sigma2.data(), &fm, t.d_pose, t.d_out);
                if (!rc) rc = down_range(t.h_n, t.h_m + nc);  // n, pose, outliers, matches
                if (!rc && hipStreamSynchronize(tstream) != hipSuccess) rc = ORBMI_E_HIP;
                return rc;
            }));
        }
        const int n = *t.h_n;
        st.track = 1;
        st.lf_matches = n;
        if (n < 20) return ORBMI_OK;
        for (int i = 0; i < nc; i++) cf.mps[i] = t.h_m[i] >= 0 ? lf.mps[t.h_m[i]] : -1;
        std::memcpy(cf.tcw.data(), t.h_pose->tcw, sizeof(t.h_pose->tcw));
        cf.outlier.assign(t.h_out, t.h_out + nc);
        seen.clear();
        const int nmap = discard_outliers(cf, cf.outlier);
        st.nmatches_map = nmap;
        ok = nmap >= 10;
        return ORBMI_OK;
    }

    // Tracking::TrackLocalMap (src/Tracking.cc:1075-1104), device-resident: UpdateLocalMap on the
    // host, then the local map points' records, the occupancy and the frame's own point records
    // go up once; SearchLocalPoints (isInFrustum + SearchByProjection(F, MPs, 1)) and
    // PoseOptimization over the frame's points and the new matches (keypoint i's edge uses the
    // local map point when it matched one, else its own point), then one read-back.
    int track_local_map_dev(TrackedFrame& cf, orbmi_slam_frame_stats& st, bool& ok) {
        ok = false;
        {
            PhaseTimer pt(&phase_ms[PH_LOCAL_UPDATE]);
            update_local_keyframes(cf);
            update_local_points();
        }
        const int nc = cf.n(), nr = (int)local_mps.size();
        SLAM_CHECK(track_buffers(nc, nc, nr));
        TrackBuf& t = tb;
        for (int i = 0; i < nc; i++) {  // SearchLocalPoints' first loop
            const int m = cf.mps[i];
            t.h_occ[i] = 0;
            if (m < 0) continue;
            if (mps[m].bad) cf.mps[i] = -1;
            else {
                mps[m].visible++;  // IncreaseVisible
                seen.insert(m);
                t.h_occ[i] = mps[m].nobs > 0 ? 1 : 0;
            }
        }
        {
            PhaseTimer pr(&phase_ms[PH_LOCAL_RECORDS]);
            mp_records_into(local_mps, t.h_rec);
            lf_records_into(cf.mps, nullptr, t.h_lfp);
            for (int i = 0; i < nc; i++) t.h_mlf[i] = cf.mps[i] >= 0 ? i : -1;
        }
        SLAM_CHECK(up_range(t.h_rec, t.h_lfp + nc));  // local map records, own-point index, occ, own records
        const orbmi_frame_view vc = view(cf, cf.tcw.data());
        orbmi_frame_mappoints fm{};
        fm.match_lf = t.d_mlf;
        fm.lf_points = t.d_lfp;
        fm.n_lf_points = nc;
        fm.match_mp = t.d_m;
        fm.mps = t.d_rec;
        fm.n_mps = nr;
        {
            PhaseTimer pt(&phase_ms[PH_LOCAL_SEARCH]);
            SLAM_CHECK(unlocked(ORBMI_SCHED_T_LOCAL, cf.id, [&] {
                int rc = orbmi_search_local_points_track(matcher, &vc, t.d_occ, t.d_rec, nr, 1.f, t.d_m, nullptr, nullptr,
                                                         t.d_tr);
                if (!rc) rc = orbmi_pose_optimization_frame(pose, &vc, inv_level_sigma2.data(), &fm, t.d_pose, t.d_out);
                if (!rc) rc = down_range(t.h_n, t.h_tr + nr);  // pose, outliers, matches, frustum records
                if (!rc && hipStreamSynchronize(tstream) != hipSuccess) rc = ORBMI_E_HIP;
                return rc;
            }));
        }
        int nl = 0;
        for (int j = 0; j < nr; j++)
            if (t.h_tr[j].in_view) mps[local_mps[j]].visible++;
        std::vector<int> cur = cf.mps;
        for (int i = 0; i < nc; i++)
            if (t.h_m[i] >= 0) { cur[i] = local_mps[t.h_m[i]]; nl++; }
        st.local_map_points = nr;
        st.local_matches = nl;
        std::memcpy(cf.tcw.data(), t.h_pose->tcw, sizeof(t.h_pose->tcw));
        cf.mps = cur;
        cf.outlier.assign(t.h_out, t.h_out + nc);
        int inliers = 0;
        for (int i = 0; i < nc; i++) {  // (:1087-1101)
            const int m = cf.mps[i];
            if (m < 0) continue;
            if (!cf.outlier[i]) {
                mps[m].found++;  // IncreaseFound
                if (mps[m].nobs > 0) inliers++;
            } else if (cf.ur[i] >= 0) {
                cf.mps[i] = -1;  // stereo outliers are dropped
            }
        }
        matches_inliers = inliers;
        st.inliers = inliers;
        ok = inliers >= 30;
        return ORBMI_OK;
    }

    // ---- Tracking::Track (stereo, SLAM mode) ------------------------------------------------------
    int track(TrackedFrame& cf) {
        if (state == NO_IMAGES_YET) state = NOT_INITIALIZED;
        orbmi_slam_frame_stats st;
        std::memset(&st, 0xff, sizeof(st));  // -1 = not run
        st.frame = cf.id;
        st.n = cf.n();
        if (state == NOT_INITIALIZED) {
            SLAM_CHECK(stereo_initialization(cf));
            st.init = state == OK;
            if (state != OK) {
                st.state = state;
                st.keyframes = (int)kfs.size();
                st.mappoints = count_mappoints();
                stats.push_back(st);
                return ORBMI_OK;
            }
        } else {
            bool ok = false;
            if (state == OK) {
                for (int& m : last_frame.mps)  // Tracking::CheckReplacedInLastFrame
                    if (m >= 0 && mps[m].replaced >= 0) m = mps[m].replaced;
                if (!has_velocity || cf.id < last_reloc_frame_id + 2) SLAM_CHECK(track_reference_kf(cf, st, ok));
                else {
                    SLAM_CHECK(track_motion_model(cf, st, ok));
                    if (!ok) SLAM_CHECK(track_reference_kf(cf, st, ok));
                }
            }  // else: Relocalization is out of scope
            cf.ref_kf = ref_kf;
            if (ok) SLAM_CHECK(track_local_map(cf, st, ok));
            state = ok ? OK : LOST;
            if (ok) {
                if (last_frame.has_tcw) {
                    velocity = mul(cf.tcw, pose_inverse(last_frame.tcw));
                    has_velocity = true;
                } else {
                    has_velocity = false;
                }
                for (int i = 0; i < cf.n(); i++) {  // clean VO matches (:504-513)
                    const int m = cf.mps[i];
                    if (m >= 0 && mps[m].nobs < 1) {
                        cf.outlier[i] = 0;
                        cf.mps[i] = -1;
                    }
                }
                if (need_new_keyframe(cf, st)) {
                    PhaseTimer pt(&phase_ms[PH_KEYFRAME]);
                    SLAM_CHECK(create_new_keyframe(cf));
                }
                for (int i = 0; i < cf.n(); i++)  // (:535-539)
                    if (cf.mps[i] >= 0 && cf.outlier[i]) cf.mps[i] = -1;
            }
            // Reset if the camera gets lost soon after initialisation (src/Tracking.cc:540-551):
            // the map is cleared and the next frame initialises again; this frame is not recorded.
            // With the mapping thread running, System::Reset only raises mbReset and
            // Tracking::Reset runs at the start of the next TrackStereo (src/System.cc:139-146),
            // outside mMutexMapUpdate: a LocalBA that finishes meanwhile needs that lock for its
            // write-back, so waiting for the mapping thread here, inside Track(), would deadlock.
            if (state == LOST && keyframes_in_map() <= 5) {
                if (async_lm()) {
                    request_reset();
                } else {
                    SLAM_CHECK(reset());
                }
                resets++;
                st.reset = 1;
                st.state = state;
                st.keyframes = 0;
                st.mappoints = 0;
                stats.push_back(st);
                return ORBMI_OK;
            }
            if (cf.ref_kf < 0) cf.ref_kf = ref_kf;
        }
        last_frame = cf;
        have_last = true;
        if (cf.has_tcw) {
            rel_poses.push_back(mul(cf.tcw, pose_inverse(kfs[cf.ref_kf].tcw)));
            references.push_back(ref_kf);
            frame_times.push_back(cf.ts);
            lost.push_back(state == LOST);
        } else if (!rel_poses.empty()) {
            rel_poses.push_back(rel_poses.back());
            references.push_back(references.back());
            frame_times.push_back(frame_times.back());
            lost.push_back(state == LOST);
        }
        st.state = state;
        st.keyframes = (int)kfs.size();
        st.mappoints = count_mappoints();
        stats.push_back(st);
        return ORBMI_OK;
    }

    // System::Reset with the mapping thread running: LocalMapping::RequestReset drops the queued
    // keyframes (its ResetIfRequested, src/LocalMapping.cc:700-716; the keyframe in hand is
    // finished first) and the rest of Tracking::Reset waits for the next TrackStereo
    bool reset_pending = false;
    void request_reset() {
        std::lock_guard<std::mutex> g(q_mtx);
        lm_queue.clear();
        reset_pending = true;
    }

    // the deferred Tracking::Reset at the start of orbmi_slam_track_stereo (no lock held): the
    // mapping thread finishes the keyframe in hand -- a LocalBA included, whose write-back takes
    // update_mtx, free now -- then the map is cleared under both locks
    int deferred_reset() {
        {
            std::unique_lock<std::mutex> g(q_mtx);
            idle_cv.wait(g, [&] { return lm_queue.empty() && !lm_busy; });
            reset_pending = false;
        }
        std::lock_guard<std::mutex> u(update_mtx);
        std::lock_guard<std::mutex> m(map_mtx);
        log_section(ORBMI_SCHED_T_RESET, -1);
        return reset();
    }

    // Tracking::Reset (src/Tracking.cc:1780-1826): the map, the tracking state, the frame /
    // keyframe ids and the trajectory lists start over (the mapping thread is idle: synchronous
    // mode, or deferred_reset)
    int reset() {
        for (auto& kf : kfs)
            if (kf.d_block) (void)hipFree(kf.d_block);
        kfs.clear();
        mps.clear();
        recent_mps.clear();
        local_kfs.clear();
        local_mps.clear();
        kf_counter.assign(kf_counter.size(), 0);
        last_frame = TrackedFrame();
        have_last = false;
        has_velocity = false;
        ref_kf = -1;
        last_kf_frame_id = 0;
        last_reloc_frame_id = 0;
        matches_inliers = 0;
        frame_count = 0;  // Frame::nNextId = 0 (KeyFrame ids restart with the emptied map)
        state = NO_IMAGES_YET;
        rel_poses.clear();
        references.clear();
        frame_times.clear();
        lost.clear();
        return ORBMI_OK;
    }

    int keyframes_in_map() const {  // Map::KeyFramesInMap
        int n = 0;
        for (auto& k : kfs) n += !k.bad;
        return n;
    }

    int count_mappoints() const {
        int n = 0;
        for (auto& m : mps) n += !m.bad;
        return n;
    }

    // the poses SaveTrajectory* write: Tcw = Tcr * Trw * Two per recorded frame
    std::vector<M4> frame_poses() const {
        std::vector<M4> out;
        if (kfs.empty()) return out;
        const M4 Two = pose_inverse(kfs[0].tcw);  // the first keyframe (lowest id)
        for (size_t f = 0; f < rel_poses.size(); f++) {
            M4 Trw = eye4();
            int k = references[f];
            while (kfs[k].bad) {  // a culled reference keyframe: through its parent (Tcp)
                Trw = mul(Trw, kfs[k].tcp);
                k = kfs[k].parent;
            }
            Trw = mul(mul(Trw, kfs[k].tcw), Two);
            out.push_back(mul(rel_poses[f], Trw));
        }
        return out;
    }
};

// CUs LocalMapping's stream leaves to Tracking (ORBMI_LM_RESERVE_CUS overrides)
constexpr int kLmReserveCus = 0;

extern "C" {

int orbmi_slam_create(const orbmi_slam_settings* s, int device, orbmi_vocabulary* vocabulary, orbmi_slam** out) {
    if (!s || !out || s->width <= 0 || s->height <= 0 || s->n_levels < 1 || s->n_levels > 16 || s->fx == 0.f)
        return ORBMI_E_ARG;
    *out = nullptr;
    orbmi_slam* h = new (std::nothrow) orbmi_slam();
    if (!h) return ORBMI_E_ARG;
    h->s = *s;
    h->device = device;
    h->voc = vocabulary;
    int rc = orbmi_extractor_create(device, s->n_features, s->scale_factor, s->n_levels, s->ini_th_fast, s->min_th_fast,
                                    &h->left);
    if (!rc) rc = orbmi_extractor_create(device, s->n_features, s->scale_factor, s->n_levels, s->ini_th_fast,
                                         s->min_th_fast, &h->right);
    if (!rc) {
        void* xs = nullptr;
        rc = orbmi_extractor_get_stream(h->left, &xs);
        h->xstream = (hipStream_t)xs;
    }
    if (!rc) rc = orbmi_matcher_create(device, &h->matcher);
    if (!rc && s->async_local_mapping) rc = orbmi_matcher_create(device, &h->lm_matcher);
    if (!rc && h->lm_matcher) {  // LocalMapping's stream kept off a few CUs (orbmi_matcher_reserve_cus)
        const char* v = getenv("ORBMI_LM_RESERVE_CUS");
        const int n = v ? atoi(v) : kLmReserveCus;
        if (n > 0) rc = orbmi_matcher_reserve_cus(h->lm_matcher, n);
    }
    if (!rc) rc = orbmi_pose_create(device, &h->pose);
    if (!rc) rc = orbmi_ba_create(device, &h->ba);
    // each thread's operators in order on one stream (Tracking: searches + PoseOptimization;
    // LocalMapping: searches + LocalBA), so the streams stay within the hardware queues
    if (!rc) rc = orbmi_pose_share_matcher_stream(h->pose, h->matcher);
    if (!rc) {
        void* ts = nullptr;
        rc = orbmi_matcher_get_stream(h->matcher, &ts);
        h->tstream = (hipStream_t)ts;
    }
    if (!rc) {
        void* st = nullptr;
        rc = orbmi_matcher_get_stream(h->lm_matcher ? h->lm_matcher : h->matcher, &st);
        if (!rc) rc = orbmi_ba_set_stream(h->ba, st);
    }
    if (!rc) {
        h->scale_factors.resize(s->n_levels);
        h->inv_level_sigma2.resize(s->n_levels);
        rc = orbmi_extractor_get_scale_factors(h->left, h->scale_factors.data());
        if (!rc) rc = orbmi_extractor_get_inverse_scale_sigma_squares(h->left, h->inv_level_sigma2.data());
        h->log_scale_factor = s->n_levels > 1 ? (float)std::log((double)h->scale_factors[1]) : 0.f;  // mfLogScaleFactor
        h->level_sigma2.resize(s->n_levels);
        for (int l = 0; l < s->n_levels; l++) h->level_sigma2[l] = h->scale_factors[l] * h->scale_factors[l];
    }
    if (rc) {
        orbmi_slam_destroy(h);
        return rc;
    }
    if (h->async_lm()) h->lm_thread = std::thread([h] { h->lm_run(); });
    *out = h;
    return ORBMI_OK;
}

int orbmi_slam_wait_local_mapping(orbmi_slam* h) {
    if (!h) return ORBMI_E_ARG;
    return h->wait_local_mapping();
}

void orbmi_slam_destroy(orbmi_slam* h) {
    if (!h) return;
    if (h->lm_thread.joinable()) {  // RequestFinish: the queued keyframes are processed first
        {
            std::lock_guard<std::mutex> g(h->q_mtx);
            h->lm_quit = true;
        }
        h->q_cv.notify_all();
        h->lm_thread.join();
    }
    if (h->xstream) (void)hipStreamSynchronize(h->xstream);
    if (h->tstream) (void)hipStreamSynchronize(h->tstream);
    h->hold_report();
    h->free_dev();
    h->free_track_buffers();
    orbmi_ba_destroy(h->ba);
    orbmi_pose_destroy(h->pose);
    orbmi_matcher_destroy(h->matcher);
    if (h->lm_matcher) orbmi_matcher_destroy(h->lm_matcher);
    for (auto& kf : h->kfs)
        if (kf.d_block) (void)hipFree(kf.d_block);
    orbmi_extractor_destroy(h->right);
    orbmi_extractor_destroy(h->left);
    delete h;
}

// Tracking::Track on a constructed frame, under the map locks
static int track_frame(orbmi_slam* h, TrackedFrame& cf, float* tcw_out, int* has_pose) {
    PhaseTimer* lock_t = new PhaseTimer(&h->phase_ms[PH_LOCK]);
    std::unique_lock<std::mutex> update_guard(h->update_mtx, std::defer_lock);
    if (h->async_lm()) update_guard.lock();
    std::unique_lock<std::mutex> map_guard(h->map_mtx);
    delete lock_t;
    h->log_section(ORBMI_SCHED_T_FRAME, cf.id);
    // with the mapping thread running, Tracking's GPU calls release the map lock (their inputs
    // are this thread's copies); the reference's Tracking and LocalMapping likewise interleave
    struct Hold {
        explicit Hold(std::unique_lock<std::mutex>* l) { held_lock = l; }
        ~Hold() { held_lock = nullptr; }
    } hold(h->async_lm() ? &map_guard : nullptr);
    {
        std::lock_guard<std::mutex> g(h->q_mtx);
        if (h->lm_rc) return h->lm_rc;
    }
    const int n = cf.n();
    cf.mps.assign(n, -1);
    cf.outlier.assign(n, 0);
    h->frame_count++;
    SLAM_CHECK(h->track(cf));
    const TrackedFrame& lf = h->last_frame;
    if (has_pose) *has_pose = lf.has_tcw ? 1 : 0;
    if (tcw_out && lf.has_tcw) std::memcpy(tcw_out, lf.tcw.data(), 16 * sizeof(float));
    return ORBMI_OK;
}

static int track_stereo(orbmi_slam* h, const uint8_t* left, const uint8_t* right, int rows, int cols, size_t step,
                        double timestamp, const uint8_t* next_left, const uint8_t* next_right, bool ahead, float* tcw_out,
                        int* has_pose) {
    if (!h || !left || !right || rows <= 0 || cols <= 0 || step < (size_t)cols) return ORBMI_E_ARG;
    if (h->reset_pending) SLAM_CHECK(h->deferred_reset());  // (src/System.cc:139-146)
    TrackedFrame cf;
    cf.id = h->frame_count;
    cf.ts = timestamp;
    // Frame::Frame (stereo, src/Frame.cc:58-100): ORBextractor on both images, ComputeStereoMatches
    // (touches no map state: outside the map lock)
    PhaseTimer total(&h->phase_ms[PH_TOTAL]);
    h->phase_frames++;
    {
        PhaseTimer pt(&h->phase_ms[PH_FRAME]);
        int rc = ahead ? h->frame_stereo_ahead(cf, left, right, rows, cols, step, next_left, next_right)
                       : h->frame_stereo(cf, left, right, rows, cols, step);
        if (rc) {
            if (h->frame_join() != ORBMI_OK) h->drop_ahead();
            return rc;
        }
    }
    const int rc = track_frame(h, cf, tcw_out, has_pose);
    // the next pair's enqueue (frame_post) has finished before the call returns: the caller's
    // images are not read afterwards.  A failed enqueue leaves its slot and the pinned read-back
    // buffers partly written: the pair is dropped, so the next call extracts it again
    const int jrc = h->frame_join();
    if (jrc != ORBMI_OK) h->drop_ahead();
    return rc ? rc : jrc;
}

int orbmi_slam_track_stereo(orbmi_slam* h, const uint8_t* left, const uint8_t* right, int rows, int cols, size_t step,
                            double timestamp, float* tcw_out, int* has_pose) {
    return track_stereo(h, left, right, rows, cols, step, timestamp, nullptr, nullptr, false, tcw_out, has_pose);
}

int orbmi_slam_track_stereo_ahead(orbmi_slam* h, const uint8_t* left, const uint8_t* right, int rows, int cols,
                                  size_t step, double timestamp, const uint8_t* next_left, const uint8_t* next_right,
                                  float* tcw_out, int* has_pose) {
    return track_stereo(h, left, right, rows, cols, step, timestamp, next_left, next_right, true, tcw_out, has_pose);
}

int orbmi_slam_get_schedule(orbmi_slam* h, orbmi_slam_event* out, int capacity, int* n) {
    if (!h || !n) return ORBMI_E_ARG;
    std::lock_guard<std::mutex> map_guard(h->map_mtx);
    *n = (int)h->sched.size();
    if (capacity < *n) return ORBMI_E_CAP;
    if (*n) std::memcpy(out, h->sched.data(), sizeof(orbmi_slam_event) * (size_t)*n);
    return ORBMI_OK;
}

int orbmi_slam_get_local_mapping_counts(orbmi_slam* h, int* out, int n) {
    if (!h || !out || n < 0) return ORBMI_E_ARG;
    std::lock_guard<std::mutex> map_guard(h->map_mtx);
    const int v[5] = {h->lm_jobs, h->sin_skipped, h->ba_skipped, h->ba_interrupted, h->ba_aborted};
    for (int i = 0; i < n && i < 5; i++) out[i] = v[i];
    return ORBMI_OK;
}

int orbmi_slam_set_recording(orbmi_slam* h, int on) {
    if (!h) return ORBMI_E_ARG;
    std::lock_guard<std::mutex> map_guard(h->map_mtx);
    h->recording = on != 0;
    return ORBMI_OK;
}

int orbmi_slam_get_keyframe_state_log(orbmi_slam* h, orbmi_slam_kf_state* out, int capacity, int* n) {
    if (!h || !n) return ORBMI_E_ARG;
    std::lock_guard<std::mutex> map_guard(h->map_mtx);
    *n = (int)h->kf_state.size();
    if (capacity < *n) return ORBMI_E_CAP;
    if (*n) std::memcpy(out, h->kf_state.data(), sizeof(orbmi_slam_kf_state) * (size_t)*n);
    return ORBMI_OK;
}

int orbmi_slam_get_local_ba_log(orbmi_slam* h, orbmi_slam_ba_record* out, int capacity, int* n) {
    if (!h || !n) return ORBMI_E_ARG;
    std::lock_guard<std::mutex> map_guard(h->map_mtx);
    *n = (int)h->ba_log.size();
    if (capacity < *n) return ORBMI_E_CAP;
    if (*n) std::memcpy(out, h->ba_log.data(), sizeof(orbmi_slam_ba_record) * (size_t)*n);
    return ORBMI_OK;
}

int orbmi_slam_get_stats(orbmi_slam* h, int frame, orbmi_slam_frame_stats* out) {
    if (!h || !out || frame < 0 || frame >= (int)h->stats.size()) return ORBMI_E_ARG;
    std::lock_guard<std::mutex> map_guard(h->map_mtx);
    *out = h->stats[frame];
    return ORBMI_OK;
}

int orbmi_slam_get_counts(orbmi_slam* h, int* frames, int* keyframes, int* mappoints, int* local_ba_calls) {
    if (!h) return ORBMI_E_ARG;
    std::lock_guard<std::mutex> map_guard(h->map_mtx);
    if (frames) *frames = h->frame_count;
    if (keyframes) *keyframes = (int)h->kfs.size();
    if (mappoints) *mappoints = h->count_mappoints();
    if (local_ba_calls) *local_ba_calls = h->ba_calls;
    return ORBMI_OK;
}

int orbmi_slam_get_trajectory(orbmi_slam* h, float* tcw, double* timestamps, uint8_t* lost, int capacity, int* n) {
    if (!h || !n) return ORBMI_E_ARG;
    std::lock_guard<std::mutex> map_guard(h->map_mtx);
    const std::vector<M4> P = h->frame_poses();
    *n = (int)P.size();
    if (capacity < *n) return ORBMI_E_CAP;
    for (int f = 0; f < *n; f++) {
        if (tcw) std::memcpy(tcw + 16 * f, P[f].data(), 16 * sizeof(float));
        if (timestamps) timestamps[f] = h->frame_times[f];
        if (lost) lost[f] = h->lost[f];
    }
    return ORBMI_OK;
}

int orbmi_slam_save_trajectory_kitti(orbmi_slam* h, const char* path) {  // src/System.cc:433-486
    if (!h || !path) return ORBMI_E_ARG;
    std::lock_guard<std::mutex> map_guard(h->map_mtx);
    FILE* f = std::fopen(path, "w");
    if (!f) return ORBMI_E_ARG;
    for (const M4& T : h->frame_poses()) {
        const M4 W = pose_inverse(T);  // Rwc = Rcw^T, twc = -Rwc tcw
        std::fprintf(f, "%.9f %.9f %.9f %.9f %.9f %.9f %.9f %.9f %.9f %.9f %.9f %.9f\n", W[0], W[1], W[2], W[3], W[4],
                     W[5], W[6], W[7], W[8], W[9], W[10], W[11]);
    }
    std::fclose(f);
    return ORBMI_OK;
}

int orbmi_slam_save_trajectory_tum(orbmi_slam* h, const char* path) {  // src/System.cc:334-389
    if (!h || !path) return ORBMI_E_ARG;
    std::lock_guard<std::mutex> map_guard(h->map_mtx);
    FILE* f = std::fopen(path, "w");
    if (!f) return ORBMI_E_ARG;
    const std::vector<M4> P = h->frame_poses();
    for (size_t i = 0; i < P.size(); i++) {
        if (h->lost[i]) continue;
        const M4 W = pose_inverse(P[i]);
        const float R[9] = {W[0], W[1], W[2], W[4], W[5], W[6], W[8], W[9], W[10]};
        float q[4];
        quaternion_xyzw(R, q);
        std::fprintf(f, "%.6f %.9f %.9f %.9f %.9f %.9f %.9f %.9f\n", h->frame_times[i], W[3], W[7], W[11], q[0], q[1],
                     q[2], q[3]);
    }
    std::fclose(f);
    return ORBMI_OK;
}

int orbmi_slam_save_keyframe_trajectory_tum(orbmi_slam* h, const char* path) {  // src/System.cc:392-431
    if (!h || !path) return ORBMI_E_ARG;
    std::lock_guard<std::mutex> map_guard(h->map_mtx);
    FILE* f = std::fopen(path, "w");
    if (!f) return ORBMI_E_ARG;
    for (const KeyFrame& kf : h->kfs) {
        if (kf.bad) continue;
        const M4 W = pose_inverse(kf.tcw);
        const float R[9] = {W[0], W[1], W[2], W[4], W[5], W[6], W[8], W[9], W[10]};
        float q[4];
        quaternion_xyzw(R, q);
        std::fprintf(f, "%.6f %.7f %.7f %.7f %.7f %.7f %.7f %.7f\n", kf.ts, W[3], W[7], W[11], q[0], q[1], q[2], q[3]);
    }
    std::fclose(f);
    return ORBMI_OK;
}

int orbmi_slam_get_phase_ms(orbmi_slam* h, double* ms, int n, long* frames) {
    if (!h || !ms || n < 0) return ORBMI_E_ARG;
    for (int i = 0; i < n && i < PH_COUNT; i++) ms[i] = h->phase_ms[i];
    if (frames) *frames = h->phase_frames;
    return ORBMI_OK;
}

}  // extern "C"
