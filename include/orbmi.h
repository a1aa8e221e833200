/*
 * orbmi — MI355X-native ORB front-end + local BA for ORB-SLAM2 (C ABI).
 *
 * Drop-in boundary for the hot path of AHzZ123/orb_slam2_with_comment.
 * Plain pointers and sizes only; every entry point cites the reference interface it replaces.
 * Host buffers are owned by the caller (capacity based); each handle owns its device
 * buffers, one HIP stream and the device-resident pyramid of its last extraction.
 * Distinct handles may be used concurrently from different host threads (the reference runs
 * the left and right ORBextractor on two std::threads, src/Frame.cc:78-81); one handle is not
 * re-entrant.  All functions return ORBMI_OK (0) or a negative orbmi_status.
 */
#ifndef ORBMI_H
#define ORBMI_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum orbmi_status {
    ORBMI_OK = 0,
    ORBMI_E_ARG = -1,         /* bad argument (null pointer, bad size)            */
    ORBMI_E_HIP = -2,         /* HIP runtime / kernel launch failure              */
    ORBMI_E_CAP = -3,         /* caller capacity too small; *n_out = needed count */
    ORBMI_E_UNSUPPORTED = -4, /* geometry outside what the kernels are sized for  */
    ORBMI_E_STATE = -5        /* call order violated (e.g. stereo before extract) */
} orbmi_status;

/* Field order of cv::KeyPoint (pt.x, pt.y, size, angle, response, octave, class_id). */
typedef struct orbmi_keypoint {
    float x, y, size, angle, response;
    int32_t octave, class_id;
} orbmi_keypoint;

typedef struct orbmi_extractor orbmi_extractor;

/* ---- ORBextractor ------------------------------------------------------------------ */

/* ORBextractor::ORBextractor(int nfeatures, float scaleFactor, int nlevels, int iniThFAST,
 * int minThFAST)  include/ORBextractor.h:58-59, src/ORBextractor.cc:410-470.
 * `device` is the HIP device ordinal the handle's buffers and stream live on. */
int orbmi_extractor_create(int device, int nfeatures, float scale_factor, int nlevels,
                           int ini_th_fast, int min_th_fast, orbmi_extractor** out);
void orbmi_extractor_destroy(orbmi_extractor* h);

/* ORBextractor::operator()(image, mask, keypoints, descriptors)
 * include/ORBextractor.h:64-66, src/ORBextractor.cc:1043-1105.  `image` is host u8 gray,
 * rows x cols with row pitch `step` bytes.  Writes n keypoints (level-major, coordinates at
 * level 0) and n x 32 descriptor bytes.  rows == 0 or cols == 0 -> *n_out = 0 (reference
 * returns on an empty image).  capacity < n -> ORBMI_E_CAP with *n_out = n. */
int orbmi_extract(orbmi_extractor* h, const uint8_t* image, int rows, int cols, size_t step,
                  orbmi_keypoint* kps, uint8_t* desc, int capacity, int* n_out);

/* Batched, device-resident form (config 5 / throughput mode).  Image b is at
 * d_images + b*image_stride (device memory).  Outputs stay on the device: keypoint i of
 * image b at d_kps[b*capacity + i], its descriptor at d_desc + (b*capacity + i)*32, count at
 * d_counts[b] (counts above `capacity` mean truncated output).  Asynchronous: enqueued on
 * the handle's stream; call orbmi_extractor_synchronize() before reading. */
int orbmi_extract_batch_device(orbmi_extractor* h, const uint8_t* d_images, int batch, int rows,
                               int cols, size_t step, size_t image_stride, orbmi_keypoint* d_kps,
                               uint8_t* d_desc, int* d_counts, int capacity);
/* The same with the images in host memory (the reference's operator() takes a host cv::Mat;
 * src/Tracking.cc:168-205 builds the Frame from it): image b at images + b*image_stride, rows
 * contiguous (pitch = cols).  The bytes go to HBM by a copy kernel on the handle's stream that
 * reads pinned memory (hipHostMalloc / hipHostRegister) in place -- asynchronous, the host does
 * not wait; the caller keeps the images unchanged until the stream has passed the call
 * (orbmi_extractor_synchronize, or an event on orbmi_extractor_get_stream).  Pageable memory is
 * first copied into one of two pinned staging buffers of the handle (the host may then wait for
 * the copy kernel two calls back). */
int orbmi_extract_batch_host(orbmi_extractor* h, const uint8_t* images, int batch, int rows, int cols,
                             size_t image_stride, orbmi_keypoint* d_kps, uint8_t* d_desc, int* d_counts, int capacity);
int orbmi_extractor_synchronize(orbmi_extractor* h);
/* The handle's HIP stream (hipStream_t), for callers that order their own work after it. */
int orbmi_extractor_get_stream(orbmi_extractor* h, void** stream);

/* Getters  include/ORBextractor.h:68-90. `out` holds nlevels floats. */
int orbmi_extractor_get_levels(const orbmi_extractor* h);
float orbmi_extractor_get_scale_factor(const orbmi_extractor* h);
int orbmi_extractor_get_scale_factors(const orbmi_extractor* h, float* out);
int orbmi_extractor_get_inverse_scale_factors(const orbmi_extractor* h, float* out);
int orbmi_extractor_get_scale_sigma_squares(const orbmi_extractor* h, float* out);
int orbmi_extractor_get_inverse_scale_sigma_squares(const orbmi_extractor* h, float* out);
int orbmi_extractor_get_features_per_level(const orbmi_extractor* h, int* out);

/* ORBextractor::mvImagePyramid[level] (public, read by Frame::ComputeStereoMatches,
 * src/Frame.cc:508,598,610) of batch item `item` of the last extraction.  padded = 0 copies
 * the W_l x H_l interior, padded = 1 the (W_l+38) x (H_l+38) buffer with its 19-px
 * reflect-101 border.  out_step = destination row pitch; *w, *h receive the copied size. */
int orbmi_extractor_get_pyramid_level(orbmi_extractor* h, int item, int level, int padded,
                                      uint8_t* out, size_t out_step, int* w, int* hgt);

/* ---- Frame::ComputeStereoMatches ----------------------------------------------------- */

/* Frame::ComputeStereoMatches()  src/Frame.cc:501-675 on the device-resident keypoints,
 * descriptors and pyramids of the last extraction of (left, item_left) and
 * (right, item_right); both handles must be on the same device.  bf = Camera.bf, fx =
 * Camera.fx (mb = bf/fx).  Writes mvuRight / mvDepth (-1 = no match) for
 * the n_left left keypoints, in left keypoint order. */
int orbmi_compute_stereo_matches(orbmi_extractor* left, int item_left, orbmi_extractor* right,
                                 int item_right, float bf, float fx, float* u_right,
                                 float* depth, int n_left);

/* Device-resident form: d_u_right / d_depth hold capacity floats per item of the last
 * batch (item-major, same layout as orbmi_extract_batch_device outputs).  Stereo pairs are
 * (left item 2p, right item 2p+1) of ONE handle for p < batch/2.  Asynchronous. */
int orbmi_compute_stereo_matches_batch_device(orbmi_extractor* h, float bf, float fx,
                                              float* d_u_right, float* d_depth);

/* ---- ORBmatcher ----------------------------------------------------------------------- */

/* Read-only view of the Frame members the matchers use (include/Frame.h).  Pointers may be
 * host or device memory of the matcher's device (detected per call).  keys_un = mvKeysUn,
 * u_right = mvuRight (NULL for monocular), desc = mDescriptors (n x 32), tcw = mTcw (4x4
 * row-major float, needed by the projection searches and isInFrustum).  A device tcw is read by
 * the kernels when they run (stream order), so it may be the output of an enqueued
 * orbmi_pose_optimization_frame (orbmi_pose_frame.tcw). */
typedef struct orbmi_frame_view {
    int n;
    const orbmi_keypoint* keys_un;
    const float* u_right;
    const uint8_t* desc;
    const float* tcw;
    float fx, fy, cx, cy;          /* Frame::fx, fy, cx, cy                         */
    float bf, mb;                  /* mbf, mb                                       */
    float min_x, max_x, min_y, max_y;      /* mnMinX, mnMaxX, mnMinY, mnMaxY        */
    float grid_w_inv, grid_h_inv;  /* mfGridElementWidthInv, mfGridElementHeightInv */
    int nlevels;
    const float* scale_factors;    /* mvScaleFactors (host or device, nlevels)      */
    float log_scale_factor;        /* mfLogScaleFactor                              */
    const int* n_device;           /* optional device count (e.g. the extractor's count
                                      output): the frame then has min(*n_device, n) keypoints
                                      and n is the capacity of keys_un/u_right/desc      */
} orbmi_frame_view;

/* MapPoint state read by Frame::isInFrustum (src/Frame.cc:274-342). flags: */
#define ORBMI_MP_BAD 1u            /* isBad()                                       */
#define ORBMI_MP_SEEN 2u           /* mnLastFrameSeen == current frame (already matched) */
#define ORBMI_MP_HAS_OBS 4u        /* Observations() > 0                            */
typedef struct orbmi_mappoint {
    float pos[3];                  /* GetWorldPos()                                 */
    float normal[3];               /* GetNormal()                                   */
    float max_distance;            /* mfMaxDistance (invariance = 1.2 x)            */
    float min_distance;            /* mfMinDistance (invariance = 0.8 x)            */
    uint32_t flags;
    uint8_t desc[32];              /* GetDescriptor()                               */
} orbmi_mappoint;

/* Output of isInFrustum: mbTrackInView, mTrackProjX/XR/Y, mnTrackScaleLevel, mTrackViewCos. */
typedef struct orbmi_mappoint_track {
    int32_t in_view;
    float proj_x, proj_xr, proj_y;
    int32_t level;
    float view_cos;
} orbmi_mappoint_track;

typedef struct orbmi_matcher orbmi_matcher;

/* ORBmatcher(float nnratio, bool checkOri) is stateless in the reference (include/ORBmatcher.h:
 * 40); the handle holds a device, a stream and scratch buffers. */
int orbmi_matcher_create(int device, orbmi_matcher** out);
void orbmi_matcher_destroy(orbmi_matcher* m);
/* Run the matcher on `ex`'s stream (the frame's keypoints/descriptors come from that
 * extraction): calls are then ordered behind it without host synchronisation, and a call whose
 * outputs are all device pointers with nmatches == NULL returns without waiting. */
int orbmi_matcher_share_stream(orbmi_matcher* m, orbmi_extractor* ex);
/* The handle's HIP stream (hipStream_t): its own, or the extractor's after share_stream. */
int orbmi_matcher_get_stream(orbmi_matcher* m, void** stream);
/* Keep the handle's own stream off `n` compute units (hipExtStreamCreateWithCUMask; the last n
 * bits of the device's CU mask cleared), so that work on other streams -- Tracking's one-
 * workgroup searches and PoseOptimization -- always finds free CUs beside a LocalMapping chain
 * (LocalBA, Fuse) that fills the device.  Call before the stream is shared or queried; n = 0
 * restores an unmasked stream.  ORBMI_E_STATE on a shared stream. */
int orbmi_matcher_reserve_cus(orbmi_matcher* m, int n);
/* Frame::AssignFeaturesToGrid (src/Frame.cc:232-247), run once per Frame as the Frame
 * constructor does (src/Frame.cc:98): builds the keypoint grid of F (device-resident keypoints
 * only, else ORBMI_E_ARG) on the handle's stream and pins it, so the searches on the same frame
 * (same keys / n / n_device / image bounds) skip their rebuild.  The pin ends with
 * orbmi_matcher_release_grid or when a search on another frame builds its grid; the caller
 * re-pins whenever the keypoints behind the pointers change (a new frame in the same buffers). */
int orbmi_matcher_assign_features_to_grid(orbmi_matcher* m, const orbmi_frame_view* F);
int orbmi_matcher_release_grid(orbmi_matcher* m);
/* The same grid built ahead, on another stream: Frame::AssignFeaturesToGrid of F (device arrays
 * only) into the handle's slot grid `slot` (0..3) on `stream` (hipStream_t; NULL = the handle's),
 * e.g. the extraction stream right after the Frame's keypoints, so the build leaves the tracking
 * chain.  The caller orders the searches that read the slot behind `stream` (an event), and the
 * next build of the slot behind those searches.  orbmi_matcher_pin_grid_slot then makes the
 * searches on F read that grid, pinned as above; ORBMI_E_STATE if the slot was built for another
 * frame (keys / n / n_device / image bounds). */
int orbmi_matcher_build_grid_slot(orbmi_matcher* m, const orbmi_frame_view* F, int slot, void* stream);
int orbmi_matcher_pin_grid_slot(orbmi_matcher* m, const orbmi_frame_view* F, int slot);

/* Frame::isInFrustum(pMP, viewingCosLimit) for n_mp points (src/Frame.cc:274-342) with
 * MapPoint::PredictScale (src/MapPoint.cc:421-436).  Points flagged BAD or SEEN are skipped
 * (in_view = 0) as in Tracking::SearchLocalPoints (src/Tracking.cc:1375-1379).  track: n_mp. */
int orbmi_is_in_frustum(orbmi_matcher* m, const orbmi_frame_view* F, const orbmi_mappoint* mps, int n_mp,
                        float viewing_cos_limit, orbmi_mappoint_track* track);

/* ORBmatcher::SearchByProjection(Frame& F, const vector<MapPoint*>& vpMapPoints, float th)
 * (src/ORBmatcher.cc:59-155), greedy in point order.  occupied[i] = F.mvpMapPoints[i] &&
 * Observations() > 0 on entry.  match_mp[i] (n entries) = index of the point newly assigned
 * to keypoint i, -1 otherwise.  Returns the count in *nmatches. */
int orbmi_search_by_projection_local(orbmi_matcher* m, const orbmi_frame_view* F, const uint8_t* occupied,
                                     const orbmi_mappoint* mps, const orbmi_mappoint_track* track, int n_mp,
                                     float th, float nnratio, int32_t* match_mp, int* nmatches);

/* Tracking::SearchLocalPoints (src/Tracking.cc:1345-1403) fused: isInFrustum(0.5) on every
 * point, then SearchByProjection(F, points, th) with nnratio 0.8.  *n_to_match = nToMatch. */
int orbmi_search_local_points(orbmi_matcher* m, const orbmi_frame_view* F, const uint8_t* occupied,
                              const orbmi_mappoint* mps, int n_mp, float th, int32_t* match_mp,
                              int* nmatches, int* n_to_match);
/* The same, also returning every point's isInFrustum outputs (mbTrackInView etc., n_mp entries;
 * host or device): the caller's IncreaseVisible for the points in view needs no second call. */
int orbmi_search_local_points_track(orbmi_matcher* m, const orbmi_frame_view* F, const uint8_t* occupied,
                                    const orbmi_mappoint* mps, int n_mp, float th, int32_t* match_mp,
                                    int* nmatches, int* n_to_match, orbmi_mappoint_track* track_out);

/* Last-frame map point view for SearchByProjection(CF, LF): one entry per LF keypoint. */
#define ORBMI_LF_HAS_MP 1u         /* LastFrame.mvpMapPoints[i] != NULL             */
#define ORBMI_LF_OUTLIER 2u        /* LastFrame.mvbOutlier[i]                       */
typedef struct orbmi_lastframe_point {
    float pos[3];                  /* pMP->GetWorldPos()                            */
    uint32_t flags;                /* ORBMI_LF_* | ORBMI_MP_HAS_OBS                 */
    uint8_t desc[32];              /* pMP->GetDescriptor()                          */
} orbmi_lastframe_point;

/* ORBmatcher::SearchByProjection(Frame& CF, const Frame& LF, float th, bool bMono)
 * (src/ORBmatcher.cc:1540-1695) incl. the rotation-consistency histogram when check_ori.
 * LF provides keys_un (octave = mvKeys[i].octave, angle = mvKeysUn[i].angle) and tcw.
 * match_lf[i] (CF.n entries) = LF keypoint index newly assigned to CF keypoint i, else -1. */
int orbmi_search_by_projection_last_frame(orbmi_matcher* m, const orbmi_frame_view* CF, const uint8_t* occupied,
                                          const orbmi_frame_view* LF, const orbmi_lastframe_point* lf_points,
                                          float th, int mono, int check_ori, int32_t* match_lf, int* nmatches);

/* DBoW2::FeatureVector as CSR: node ids ascending, feature indices of node k at
 * feat[off[k] .. off[k+1]) in insertion order (Thirdparty/DBoW2/DBoW2/FeatureVector.h:21-22). */
typedef struct orbmi_feature_vector {
    int nnodes;
    const uint32_t* node_id;
    const int32_t* off;            /* nnodes + 1 */
    const int32_t* feat;
} orbmi_feature_vector;

/* ORBmatcher::SearchByBoW(KeyFrame* pKF, Frame& F, vector<MapPoint*>& matches)
 * (src/ORBmatcher.cc:211-344).  kf_mp_ok[j] = pKF->GetMapPointMatches()[j] && !isBad().
 * KF keys_un supply angles (mvKeysUn), F keys_un supply angles of F.mvKeys.  match_kf[i]
 * (F.n entries) = KF keypoint index whose map point is assigned to F keypoint i, else -1. */
int orbmi_search_by_bow(orbmi_matcher* m, const orbmi_frame_view* KF, const uint8_t* kf_mp_ok,
                        const orbmi_feature_vector* kf_fv, const orbmi_frame_view* F,
                        const orbmi_feature_vector* f_fv, float nnratio, int check_ori, int32_t* match_kf,
                        int* nmatches);

/* ORBmatcher::SearchForTriangulation(KeyFrame* pKF1, KeyFrame* pKF2, cv::Mat F12,
 * vector<pair<size_t,size_t>>& vMatchedPairs, bool bOnlyStereo) (src/ORBmatcher.cc:783-975)
 * with CheckDistEpipolarLine (:173-196): KF1 / KF2 views need keys_un, u_right, desc, tcw, the
 * intrinsics and scale factors (mvLevelSigma2 = scale^2); has_mp[i] = pKF->GetMapPoint(i) !=
 * NULL; fv = the keyframes' mFeatVec; F12 = LocalMapping::ComputeF12 (3x3 row-major float, host
 * or device).  match12[i1] (KF1.n entries) = the KF2 keypoint paired with KF1 keypoint i1, else
 * -1 (vMatchedPairs = the pairs in i1 order); *nmatches = the return value.  The reference
 * never marks KF2 keypoints as used (vbMatched2 stays false), so one KF2 keypoint may pair with
 * several KF1 keypoints, as here. */
int orbmi_search_for_triangulation(orbmi_matcher* m, const orbmi_frame_view* KF1, const uint8_t* has_mp1,
                                   const orbmi_feature_vector* fv1, const orbmi_frame_view* KF2, const uint8_t* has_mp2,
                                   const orbmi_feature_vector* fv2, const float* F12, int only_stereo, int check_ori,
                                   int32_t* match12, int* nmatches);

/* SearchForTriangulation of one keyframe against npairs neighbours in one launch, as
 * LocalMapping::CreateNewMapPoints calls it in its loop over the best covisible keyframes
 * (src/LocalMapping.cc:326-384): pair j is (KF1, KF2[j]) with has_mp2[j], fv2[j] and
 * F12[9 j .. 9 j + 8]; its matches go to match12[j * KF1.n .. (j + 1) * KF1.n) and, when nmatches
 * is not NULL, its count to nmatches[j] (host, synchronises).  Per pair identical to
 * orbmi_search_for_triangulation; asynchronous when match12 is device memory and nmatches NULL. */
int orbmi_search_for_triangulation_batch(orbmi_matcher* m, const orbmi_frame_view* KF1, const uint8_t* has_mp1,
                                         const orbmi_feature_vector* fv1, int npairs, const orbmi_frame_view* KF2,
                                         const uint8_t* const* has_mp2, const orbmi_feature_vector* fv2,
                                         const float* F12, int only_stereo, int check_ori, int32_t* match12,
                                         int* nmatches);

/* ORBmatcher::Fuse(KeyFrame* pKF, const vector<MapPoint*>& vpMapPoints, float th)
 * (src/ORBmatcher.cc:977-1127), its search: for each of the n_mp candidate map points (in
 * vpMapPoints order; NULL entries left out by the caller, isBad() as ORBMI_MP_BAD, in_kf[i] =
 * IsInKeyFrame(pKF), in_kf may be NULL) the keyframe keypoint it fuses with: best_idx[i] (-1
 * when the point is skipped or its best distance exceeds TH_LOW = 50) and best_dist[i] (256
 * without a candidate).  The KF view needs keys_un, u_right (NULL = monocular), desc, tcw, the
 * intrinsics, bounds (mnMinX.., IsInImage) and scale factors.  The map updates stay with the
 * caller, replayed in list order as the reference does them: skip points that became bad or
 * joined pKF meanwhile; pMPinKF = pKF->GetMapPoint(best_idx[i]): if present and not bad,
 * Replace toward the point with more observations, otherwise AddObservation + AddMapPoint;
 * count nFused.  *ncandidates = the points with best_idx >= 0 (= nFused when
 * the replay skips none). */
int orbmi_fuse_search(orbmi_matcher* m, const orbmi_frame_view* KF, const orbmi_mappoint* mps, const uint8_t* in_kf,
                      int n_mp, float th, int32_t* best_idx, int32_t* best_dist, int* ncandidates);

/* The search of Fuse(pKFi, vpMapPointMatches) for every target keyframe of SearchInNeighbors
 * (src/LocalMapping.cc:631-641) in one launch: the same n_mp candidates against each of the nkf
 * keyframes kfs[k]; keyframe k's results at best_idx / best_dist[k * n_mp ..) (in_kf, when not
 * NULL, likewise nkf x n_mp) and its candidate count at ncandidates[k] (host, synchronises; may
 * be NULL).  Per keyframe identical to orbmi_fuse_search. */
int orbmi_fuse_search_batch(orbmi_matcher* m, int nkf, const orbmi_frame_view* kfs, const orbmi_mappoint* mps,
                            const uint8_t* in_kf, int n_mp, float th, int32_t* best_idx, int32_t* best_dist,
                            int* ncandidates);

/* SearchInNeighbors between two Fuse targets (src/LocalMapping.cc:620-628): the
 * ComputeDistinctiveDescriptors that MapPoint::Replace owes its survivors (src/MapPoint.cc:212),
 * then the Fuse searches of the records whose descriptor that changed -- one synchronisation.
 * orbmi_compute_distinctive_descriptors of nd points (obs_desc, obs_off, best, desc_out as
 * there; nd may be 0), then orbmi_fuse_search_batch of n_mp records against nkf keyframes
 * (kfs, in_kf, th, best_idx, best_dist as there), record i searched with descriptor
 * desc_out[desc_from[i]] when desc_from (may be NULL) has desc_from[i] >= 0.  `mps` is read,
 * not written. */
int orbmi_fuse_search_refresh(orbmi_matcher* m, const uint8_t* obs_desc, const int32_t* obs_off, int nd, int32_t* best,
                              uint8_t* desc_out, int nkf, const orbmi_frame_view* kfs, const orbmi_mappoint* mps,
                              const int32_t* desc_from, const uint8_t* in_kf, int n_mp, float th, int32_t* best_idx,
                              int32_t* best_dist);

/* MapPoint::ComputeDistinctiveDescriptors (src/MapPoint.cc:247-316) for np map points: the
 * observation descriptors of point p are rows obs_off[p] .. obs_off[p + 1] - 1 of obs_desc
 * (x 32 B), in mObservations order with bad keyframes left out by the caller (the reference
 * iterates a map keyed by KeyFrame*; the build orders by keyframe id).
 * best[p] = the row (within the point) of least median Hamming distance to the point's other
 * descriptors (sorted row incl. the self-distance, element 0.5 (N - 1)), first row on ties; -1
 * without observations.  desc_out[p] (32 B) = that descriptor (mDescriptor); left unchanged for
 * points without observations.  Arrays host or device; asynchronous when best and desc_out are
 * device memory. */
int orbmi_compute_distinctive_descriptors(orbmi_matcher* m, const uint8_t* obs_desc, const int32_t* obs_off, int np,
                                          int32_t* best, uint8_t* desc_out);

/* ---- DBoW2 vocabulary: Frame::ComputeBoW / KeyFrame::ComputeBoW ---- */

/* DBoW2::TemplatedVocabulary<FORB::TDescriptor, FORB> (Thirdparty/DBoW2/DBoW2/
 * TemplatedVocabulary.h) as flat arrays, nodes in id order (node 0 = root, as
 * loadFromTextFile builds them, :1338-1424): 32-B descriptor, children as CSR in insertion
 * order, word id (-1 for inner nodes) and weight (idf for TF_IDF) per node.  scoring and
 * weighting are DBoW2::ScoringType / WeightingType (BowVector.h:36-53). */
typedef struct orbmi_vocabulary_desc {
    int k, L;                      /* m_k, m_L                                               */
    int scoring, weighting;        /* L1_NORM .. DOT_PRODUCT; TF_IDF, TF, IDF, BINARY         */
    int nnodes;
    const uint8_t* desc;           /* nnodes x 32                                            */
    const int32_t* child_off;      /* nnodes + 1                                             */
    const int32_t* children;       /* child_off[nnodes] node ids                             */
    const int32_t* word_id;        /* nnodes                                                 */
    const double* weight;          /* nnodes                                                 */
} orbmi_vocabulary_desc;

typedef struct orbmi_vocabulary orbmi_vocabulary;
/* Upload a vocabulary (host arrays) to `device`; the handle owns a stream. */
int orbmi_vocabulary_create(int device, const orbmi_vocabulary_desc* d, orbmi_vocabulary** out);
void orbmi_vocabulary_destroy(orbmi_vocabulary* v);
int orbmi_vocabulary_synchronize(orbmi_vocabulary* v);
/* Run the handle on `ex`'s stream (like orbmi_matcher_share_stream): a keyframe's ComputeBoW then
 * follows its extraction on the extraction stream, beside the LocalBA on the mapper's stream. */
int orbmi_vocabulary_share_stream(orbmi_vocabulary* v, orbmi_extractor* ex);
/* Run the handle on a caller's HIP stream (hipStream_t, e.g. orbmi_matcher_get_stream's), or on
 * a new stream of its own when `stream` is NULL.  The stream must outlive its use here.  Every
 * stream a process creates beyond the device's hardware queues (GPU_MAX_HW_QUEUES) shares a
 * queue with another and serialises behind its work: an in-order chain of operators (the
 * LocalMapping thread's) belongs on one stream. */
int orbmi_vocabulary_set_stream(orbmi_vocabulary* v, void* stream);
/* The handle's HIP stream (hipStream_t): its own, or the extractor's after share_stream. */
int orbmi_vocabulary_get_stream(orbmi_vocabulary* v, void** stream);

/* TemplatedVocabulary::transform(features, BowVector& v, FeatureVector& fv, levelsup)
 * (TemplatedVocabulary.h:1126-1194, per feature :1217-1259) as Frame::ComputeBoW calls it
 * (levelsup = 4, src/Frame.cc:425-432): each of the n descriptors (n x 32 u8) descends the tree
 * (FORB::distance, first child wins ties); features whose word weight is 0 are skipped.
 * Outputs (capacity n each; fv_off n + 1): the BowVector as word ids ascending + values
 * (addWeight for TF / TF_IDF, addIfNotExist for IDF / BINARY, 1/size for TF without
 * normalisation, then normalize(L1 | L2) when the scoring asks for it, BowVector.cpp:34-86),
 * the FeatureVector as CSR (orbmi_feature_vector: node ids at level L - levelsup ascending,
 * feature indices ascending), counts[0] = words, counts[1] = nodes.  n_device (optional)
 * overrides n with a device-resident count <= n.  Arrays host or device; asynchronous on the
 * handle's stream when every output (counts included) is device memory.  n <= 8192.  Calls on
 * one handle from several threads are serialised (the reference's transform is const). */
int orbmi_transform(orbmi_vocabulary* v, const uint8_t* desc, int n, const int* n_device, int levelsup,
                    uint32_t* bow_word, double* bow_value, uint32_t* fv_node, int32_t* fv_off, int32_t* fv_feat,
                    int* counts);

/* Cross-stream matching of config 4 (build-defined; no reference counterpart, SURVEY.md §8(d)
 * "Config 4"): brute-force Hamming nearest neighbour of each of the nq query descriptors over
 * the nseg gathered train segments (segment s = rows [s*seg_capacity, s*seg_capacity +
 * seg_counts[s]) of train_desc; segment skip_seg is ignored, -1 = none).  Accepted when
 * best <= th and best < ratio * second best (second = 256 when absent); equal distances
 * resolve to the lowest row.  match[q] = global train row or -1.  nq_device as in
 * orbmi_frame_view.  Inputs host or device; asynchronous when all outputs are device memory and
 * nmatches == NULL. */
int orbmi_match_descriptors_segments(orbmi_matcher* m, const uint8_t* q_desc, int nq, const int* nq_device,
                                     const uint8_t* train_desc, int nseg, int seg_capacity,
                                     const int* seg_counts, int skip_seg, int th, float ratio,
                                     int32_t* match, int* nmatches);

/* ---- Optimizer::LocalBundleAdjustment ------------------------------------------------ */

/* The local-BA graph exactly as src/Optimizer.cc:483-683 builds it: local keyframes
 * (optimised unless id == 0), fixed observer keyframes, local map points (marginalised), one
 * edge per (point, keyframe) observation in the reference's insertion order (points in
 * lLocalMapPoints order, observations in map order).  Poses cross as float Tcw (cv::Mat
 * CV_32F), converted to double inside (src/Converter.cc:37-47). */
typedef struct orbmi_ba_keyframe {
    float tcw[16];                 /* KeyFrame::GetPose(), row-major 4x4                */
    uint32_t id;                   /* KeyFrame::mnId (vertex id)                         */
    int32_t fixed;                 /* fixed camera or mnId == 0                          */
    float fx, fy, cx, cy, bf;      /* KeyFrame::fx, fy, cx, cy, mbf                     */
} orbmi_ba_keyframe;

typedef struct orbmi_ba_point {
    float pos[3];                  /* MapPoint::GetWorldPos()                            */
    uint32_t id;                   /* MapPoint::mnId (vertex id = id + maxKFid + 1)       */
    int32_t bad;                   /* isBad() when the outlier loops run (:705, :747)     */
} orbmi_ba_point;

typedef struct orbmi_ba_edge {
    int32_t point, kf;             /* indices into the point / keyframe arrays           */
    float u, v;                    /* mvKeysUn[idx].pt                                   */
    float ur;                      /* mvuRight[idx]; < 0 -> EdgeSE3ProjectXYZ (mono)     */
    float inv_sigma2;              /* mvInvLevelSigma2[octave]                            */
} orbmi_ba_edge;

typedef struct orbmi_ba_problem {
    int nkf, npt, nedge;
    const orbmi_ba_keyframe* kfs;
    const orbmi_ba_point* pts;
    const orbmi_ba_edge* edges;
} orbmi_ba_problem;

typedef struct orbmi_ba_result {
    float* tcw;                    /* nkf x 16: optimised poses (fixed ones unchanged)    */
    float* pos;                    /* npt x 3                                            */
    uint8_t* erase;                /* nedge: 1 -> (KF, MP) pair goes to vToErase (:741-773) */
    int iterations[2];             /* optimize(5) / optimize(10) iterations run          */
    double chi2[2];                /* final activeRobustChi2 of both optimisations       */
    int aborted;                   /* stop flag seen before the first optimisation: no write-back */
    int stop_check;                /* index of the first pbStopFlag check that found the flag
                                    * raised (-1: none); numbering: orbmi_ba_set_stop_at_check */
    int checks;                    /* pbStopFlag checks made by the call                 */
} orbmi_ba_result;

typedef struct orbmi_ba orbmi_ba;
int orbmi_ba_create(int device, orbmi_ba** out);
void orbmi_ba_destroy(orbmi_ba* h);
/* Run the handle on a caller's HIP stream, or its own new one when `stream` is NULL (as
 * orbmi_vocabulary_set_stream). */
int orbmi_ba_set_stream(orbmi_ba* b, void* stream);
/* Deterministic pbStopFlag (test and schedule-replay hook; no counterpart in the reference):
 * in every later call on the handle the flag reads raised from its k-th check on (k < 0: off),
 * whatever `stop` holds.  The checks are the reads of pbStopFlag in the order the reference
 * evaluates them, numbered from 0:
 *   #0  src/Optimizer.cc:685 (raised: return before optimising, `aborted`, no write-back);
 *   SparseOptimizer::optimize's loop condition before each iteration while i < iterations
 *       (Thirdparty/g2o/g2o/core/sparse_optimizer.cpp:376; none when the graph has no vertex);
 *   the LM inner loop's condition after a rejected trial while qmax < 10
 *       (optimization_algorithm_levenberg.cpp:149, evaluated only when rho < 0);
 *   src/Optimizer.cc:689 (bDoMore) after optimize(5); then optimize(10)'s, as optimize(5)'s.
 * A flag raised by another thread is first seen at one of these checks, so a call with
 * k = result.stop_check of a concurrent run repeats that run exactly. */
int orbmi_ba_set_stop_at_check(orbmi_ba* b, int k);
/* Host hook (no counterpart in the reference): in every later call on the handle, fn(arg) runs
 * on the calling thread once the LocalBA's work has been enqueued and before the call waits for
 * it, so a caller can enqueue independent work of its own (e.g. the next keyframe's
 * ComputeBoW on another stream) beside the solve.  fn must not call back into this handle.
 * fn = NULL removes it. */
int orbmi_ba_set_enqueued_hook(orbmi_ba* b, void (*fn)(void*), void* arg);

/* Optimizer::LocalBundleAdjustment(pKF, pbStopFlag, pMap) (include/Optimizer.h:62,
 * src/Optimizer.cc:483-808) on the assembled graph: LM (g2o OptimizationAlgorithmLevenberg,
 * BlockSolver_6_3 Schur complement, Huber sqrt(5.991)/sqrt(7.815)) 5 iterations, outlier
 * levels, 10 iterations without kernels, erase list.  All arithmetic fp64 on the GPU.
 * `stop` (may be NULL) is read like pbStopFlag / mbAbortBA, at the checks listed under
 * orbmi_ba_set_stop_at_check.  Edges must come grouped by point with at most one per (point,
 * keyframe), as a map point's observations give them; otherwise ORBMI_E_ARG. */
int orbmi_local_bundle_adjustment(orbmi_ba* h, const orbmi_ba_problem* problem, orbmi_ba_result* result,
                                  const volatile int* stop);

/* ---- Optimizer::PoseOptimization ---------------------------------------------------- */

/* One unary edge: a keypoint i of the Frame with a MapPoint (mvpMapPoints[i] != NULL),
 * src/Optimizer.cc:296-375.  `index` is the caller's keypoint index (mvbOutlier slot). */
typedef struct orbmi_pose_obs {
    float Xw[3];                   /* MapPoint::GetWorldPos()                             */
    float u, v;                    /* mvKeysUn[i].pt                                      */
    float ur;                      /* mvuRight[i]; < 0 -> EdgeSE3ProjectXYZOnlyPose (mono)  */
    float inv_sigma2;              /* mvInvLevelSigma2[mvKeysUn[i].octave]                 */
    int32_t index;                 /* keypoint index i (returned untouched)               */
} orbmi_pose_obs;

/* One frame: its observations are obs[obs_begin, obs_begin + n_obs). */
typedef struct orbmi_pose_frame {
    float tcw[16];                 /* in: Frame::mTcw (row-major); out: optimised pose;
                                      unchanged when fewer than 3 observations (:378-379)  */
    float fx, fy, cx, cy, bf;      /* Frame::fx, fy, cx, cy, mbf                           */
    int32_t obs_begin, n_obs;
    int32_t inliers;               /* out: nInitialCorrespondences - nBad, the return value;
                                      -1 when n_obs exceeds the kernel's 4096 (device path) */
    int32_t iterations;            /* out: LM iterations run over the 4 rounds (diagnostic) */
} orbmi_pose_frame;

typedef struct orbmi_pose orbmi_pose;
int orbmi_pose_create(int device, orbmi_pose** out);
void orbmi_pose_destroy(orbmi_pose* h);

/* Optimizer::PoseOptimization(Frame*) (include/Optimizer.h:58, src/Optimizer.cc:257-481) on
 * `nframes` independent frames in one launch (one workgroup per frame): 4 rounds of
 * optimize(10) (g2o Levenberg, BlockSolver_6_3 + LinearSolverDense, Huber sqrt(5.991) /
 * sqrt(7.815) for the first 3 rounds) from the frame's initial pose, outliers re-classified
 * after each round (chi2 > 5.991 / 7.815, level 1).  outlier[k] receives mvbOutlier for obs k.
 * fp64 on the GPU.  `frames`, `obs` and `outlier` may be host or device pointers; device
 * pointers leave the work enqueued on the handle's stream (orbmi_pose_synchronize). */
int orbmi_pose_optimization(orbmi_pose* h, orbmi_pose_frame* frames, int nframes, const orbmi_pose_obs* obs,
                            int nobs, uint8_t* outlier);
int orbmi_pose_synchronize(orbmi_pose* h);
/* Run the handle on `ex`'s stream (like orbmi_matcher_share_stream): a tracked frame's
 * extraction, searches and pose optimisations are then ordered without host round trips. */
int orbmi_pose_share_stream(orbmi_pose* h, orbmi_extractor* ex);
/* Run the handle on the matcher's stream instead: the tracking stages (searches, pose
 * optimisations) then form one stream that can run beside the next frame's extraction. */
int orbmi_pose_share_matcher_stream(orbmi_pose* h, orbmi_matcher* m);
/* Bracket PoseOptimization kernels launched by orbmi_pose_optimization_frame[_track] with HIP
 * events on the handle's stream: every launch for on == 1, every on-th launch for on > 1 (each
 * timed event is a queue packet of a few microseconds on the stream: sampling keeps the
 * measurement from slowing what it measures), none for on <= 0; orbmi_pose_read_profile
 * synchronises and returns the summed device time (ms) and the number of timed launches since
 * the last read. */
int orbmi_pose_set_profiling(orbmi_pose* h, int on);
int orbmi_pose_read_profile(orbmi_pose* h, double* ms, long long* launches);

/* Frame::mvpMapPoints of the frame being tracked, as the matchers left it: keypoint i holds
 * local map point mps[match_mp[i]] when match_mp && match_mp[i] >= 0, otherwise last-frame
 * point lf_points[match_lf[i]] when match_lf && match_lf[i] >= 0, otherwise NULL.  The match
 * arrays are the outputs of orbmi_search_local_points / orbmi_search_by_projection_last_frame
 * (CF.n entries; -1 and -2 both mean NULL). */
typedef struct orbmi_frame_mappoints {
    int32_t* match_lf;
    const orbmi_lastframe_point* lf_points;
    int n_lf_points;               /* entries of lf_points (last frame's N)                */
    int32_t* match_mp;
    const orbmi_mappoint* mps;
    int n_mps;                     /* entries of mps                                       */
} orbmi_frame_mappoints;

/* Optimizer::PoseOptimization(Frame* pFrame) (include/Optimizer.h:58, src/Optimizer.cc:257-481)
 * with its edge assembly (:296-375): one unary edge per keypoint holding a map point, in
 * keypoint order, stereo when mvuRight[i] >= 0, information mvInvLevelSigma2[octave].  The
 * initial pose is F->tcw (host or device).  rec receives the optimised tcw, fx..bf, n_obs =
 * nInitialCorrespondences, inliers (the return value) and iterations; outlier[i] = mvbOutlier[i]
 * (F->n entries; 0 for keypoints without a map point).  inv_level_sigma2: host, F->nlevels
 * floats.  Every array may be host or device memory; with rec and outlier in device memory the
 * call is asynchronous on the handle's stream (F->n_device is then honoured). */
int orbmi_pose_optimization_frame(orbmi_pose* h, const orbmi_frame_view* F, const float* inv_level_sigma2,
                                  const orbmi_frame_mappoints* mp, orbmi_pose_frame* rec, uint8_t* outlier);

/* ---- Tracking (TrackWithMotionModel / TrackLocalMap bookkeeping) -------------------- */

/* The wider-window retry of Tracking::TrackWithMotionModel (src/Tracking.cc:1018-1023) with
 * the count kept on the device: when *nmatches_dev < min_matches, SearchByProjection(CF, LF,
 * th) runs as orbmi_search_by_projection_last_frame (match_lf rewritten, *nmatches_dev = its
 * count); otherwise nothing changes.  nmatches_dev must be device memory; asynchronous. */
int orbmi_search_by_projection_last_frame_if(orbmi_matcher* m, const orbmi_frame_view* CF,
                                             const uint8_t* occupied, const orbmi_frame_view* LF,
                                             const orbmi_lastframe_point* lf_points, float th, int mono,
                                             int check_ori, int32_t* match_lf, int* nmatches_dev,
                                             int min_matches);

/* Tracking's pass over mvpMapPoints after a PoseOptimization, on the device:
 * stage 0 = TrackWithMotionModel "Discard outliers" (src/Tracking.cc:1036-1058): outlier map
 *   points become NULL (their match entry -1); counts[0] = outliers removed (the reference's
 *   nmatches -= counts[0]), counts[1] = nmatchesMap (inliers whose point has Observations() > 0);
 *   occupied_out[i] = 1 when keypoint i keeps a point with observations (the `occupied` input of
 *   the local-map search).
 * stage 1 = TrackLocalMap statistics (src/Tracking.cc:1085-1104): counts[0] = mnMatchesInliers
 *   (non-outliers with Observations() > 0), counts[1] = outliers; with stereo (F->u_right set)
 *   outliers become NULL.  occupied_out may be NULL.
 * counts: 2 ints, host or device (device -> asynchronous). */
int orbmi_track_update_matches(orbmi_matcher* m, const orbmi_frame_view* F, int stage, const uint8_t* outlier,
                               const orbmi_frame_mappoints* mp, uint8_t* occupied_out, int* counts);

/* orbmi_pose_optimization_frame followed by orbmi_track_update_matches(stage) on its outlier
 * flags, in one launch on the pose handle's stream (Tracking::TrackWithMotionModel's
 * PoseOptimization + "Discard outliers", src/Tracking.cc:1033-1058, with stage 0; TrackLocalMap's
 * PoseOptimization + statistics, :1079-1104, with stage 1): the same results as the two calls.
 * Every array (rec, outlier, counts, occupied_out, the match arrays and point records of mp)
 * must be device memory: the call is asynchronous; ORBMI_E_ARG otherwise. */
int orbmi_pose_optimization_frame_track(orbmi_pose* h, const orbmi_frame_view* F, const float* inv_level_sigma2,
                                        const orbmi_frame_mappoints* mp, orbmi_pose_frame* rec, uint8_t* outlier,
                                        int stage, uint8_t* occupied_out, int* counts);

/* ---- LocalMapping host geometry (CreateNewMapPoints around SearchForTriangulation) ----- */

/* The KeyFrame members CreateNewMapPoints reads (host arrays): pose, mvKeysUn, mvuRight,
 * mvDepth, intrinsics, mbf, mb, mvLevelSigma2 and mvScaleFactors (nlevels entries). */
typedef struct orbmi_tri_keyframe {
    const float* tcw;              /* 4x4 row-major Tcw                                     */
    const orbmi_keypoint* keys_un;
    const float* u_right;
    const float* depth;
    float fx, fy, cx, cy, bf, mb;
    const float* level_sigma2;
    const float* scale_factors;
} orbmi_tri_keyframe;

/* LocalMapping::ComputeF12 (src/LocalMapping.cc:676-693): F12 = K1^-T [t12]x R12 K2^-1 (3x3
 * row-major float), the epipolar constraint SearchForTriangulation takes. */
int orbmi_compute_f12(const orbmi_tri_keyframe* kf1, const orbmi_tri_keyframe* kf2, float* F12);

/* CreateNewMapPoints' per-match geometry (src/LocalMapping.cc:385-575) for the n matched
 * keypoint pairs (idx1[k] of kf1, idx2[k] of kf2): ray parallax, linear triangulation or stereo
 * back-projection, positive depth in both cameras, reprojection error (5.991 / 7.8 sigma^2) and
 * scale consistency.  ok[k] = 1 with x3d[3k..3k+2] the new point's world position, else 0. */
int orbmi_triangulate_matches(const orbmi_tri_keyframe* kf1, const orbmi_tri_keyframe* kf2, const int32_t* idx1,
                              const int32_t* idx2, int n, float* x3d, uint8_t* ok);

/* cos(2 atan2(mb / 2, depth[i])) as float for n keypoints: CreateNewMapPoints' stereo parallax
 * of a stereo keypoint (src/LocalMapping.cc:409-412), a per-keyframe table for
 * orbmi_create_new_map_points. */
int orbmi_stereo_parallax_cos(float mb, const float* depth, int n, float* out);

/* LocalMapping::CreateNewMapPoints' searches and geometry (src/LocalMapping.cc:290-577) for one
 * keyframe and npairs neighbours (in the order the reference visits them, the baseline test
 * already applied), all on the device with one synchronisation: pair j's SearchForTriangulation
 * (as orbmi_search_for_triangulation with bOnlyStereo = false and the matcher's
 * mbCheckOrientation = false, ORBmatcher matcher(0.6, false) at :306) sees KF1's map points as
 * the pairs before it left them -- a KF1 keypoint whose match an earlier pair's triangulation
 * accepted counts as having a map point, exactly as in the reference's loop -- and the pair's
 * matches are then tested as orbmi_triangulate_matches does.
 * kf1 / kf2[j]: frame views (keys_un, u_right, desc host or device; tcw host); tri1 / tri2[j]:
 * the geometry, of which tcw, depth (host or device, n entries), the intrinsics, level_sigma2
 * and scale_factors (host, nlevels of the frame view) are read; cos1 / cos2[j]: the keyframe's
 * orbmi_stereo_parallax_cos table (host or device), or NULL to compute it here from a host depth.
 * has_mp1 / has_mp2[j]: the keyframes' map points on entry (not modified).
 * Outputs (host or device), row j * kf1->n + i for pair j and KF1 keypoint i: match12 = the
 * KF2 keypoint SearchForTriangulation paired with i, or -1; ok = 1 when the geometry accepted a
 * new map point; x3d[3 * row ..] = its world position (unspecified where ok = 0). */
int orbmi_create_new_map_points(orbmi_matcher* m, const orbmi_frame_view* kf1, const orbmi_tri_keyframe* tri1,
                                const float* cos1, const uint8_t* has_mp1, const orbmi_feature_vector* fv1,
                                int npairs, const orbmi_frame_view* kf2, const orbmi_tri_keyframe* tri2,
                                const float* const* cos2, const uint8_t* const* has_mp2,
                                const orbmi_feature_vector* fv2, const float* F12, int32_t* match12, uint8_t* ok,
                                float* x3d);

/* ---- System::TrackStereo: the native stereo SLAM host loop ---------------------------- */

/* The Tracking constructor's view of a settings file (src/Tracking.cc:53-143) for a rectified
 * stereo rig: Camera.fx/fy/cx/cy, Camera.bf, mThDepth = bf * ThDepth / fx, mMinFrames = 0,
 * mMaxFrames = fps, the image size and the ORBextractor parameters. */
typedef struct orbmi_slam_settings {
    float fx, fy, cx, cy, bf;
    float th_depth;
    int min_frames, max_frames;
    int width, height;
    int n_features;
    float scale_factor;
    int n_levels, ini_th_fast, min_th_fast;
    int local_ba;                  /* 1: LocalMapping runs LocalBundleAdjustment (:89-90)      */
    int local_mapping;             /* 1: and CreateNewMapPoints, SearchInNeighbors, KeyFrameCulling */
    int async_local_mapping;       /* 1: LocalMapping on its own thread, concurrent with Tracking as
                                      in the reference (keyframe decisions then depend on timing);
                                      0: synchronous after each keyframe (deterministic) */
} orbmi_slam_settings;

/* Per tracked frame: Tracking's counters (-1 = the stage did not run). track: 0 none, 1
 * TrackWithMotionModel, 2 TrackReferenceKeyFrame (the last one tried). */
typedef struct orbmi_slam_frame_stats {
    int frame, n, state, init, track;
    int lf_matches, bow_matches, nmatches_map, local_map_points, local_matches, inliers;
    int need_kf, keyframes, mappoints;
    int reset; /* 1: the frame was lost with <= 5 keyframes in the map and the system reset
                * (src/Tracking.cc:540-551); the map and the trajectory lists start over */
} orbmi_slam_frame_stats;

typedef struct orbmi_slam orbmi_slam;

/* System(strSettingsFile, STEREO) + Tracking + a synchronous LocalMapping
 * (src/System.cc:36-107, src/Tracking.cc:53-143, src/LocalMapping.cc:47-128) on `device`: the
 * map (keyframes, map points, covisibility, spanning tree) is kept natively, every per-keypoint
 * operator is the MI355X one of this library.  vocabulary (may be NULL: TrackReferenceKeyFrame
 * then fails with ORBMI_E_STATE) is borrowed and must outlive the handle. */
int orbmi_slam_create(const orbmi_slam_settings* s, int device, orbmi_vocabulary* vocabulary, orbmi_slam** out);
/* System::Shutdown's wait for LocalMapping (src/System.cc:300-314): returns when no keyframe is
 * queued or being processed (immediately in synchronous mode); the mapping thread's first error. */
int orbmi_slam_wait_local_mapping(orbmi_slam* h);
void orbmi_slam_destroy(orbmi_slam* h);

/* System::TrackStereo(imLeft, imRight, timestamp) (src/System.cc:110-159): host u8 gray images
 * (rows x cols, row pitch step).  tcw_out (16 floats, may be NULL) receives mCurrentFrame.mTcw;
 * *has_pose = 0 while not initialised / lost (empty Tcw). */
int orbmi_slam_track_stereo(orbmi_slam* h, const uint8_t* left, const uint8_t* right, int rows, int cols, size_t step,
                            double timestamp, float* tcw_out, int* has_pose);

/* orbmi_slam_track_stereo for drivers that have the next pair at hand (a stereo_kitti loop over
 * image files): as the plain call, and then the next pair's Frame constructor (upload, ORB
 * extraction of both images, ComputeStereoMatches) is enqueued to run on the GPU while this frame
 * is tracked.  The next call must pass that pair as left/right -- the same buffers, unmodified,
 * same geometry -- to use it (any other pair is extracted as usual); next_left / next_right NULL:
 * nothing ahead.  The extraction depends on the images only, so every result is the plain call's.
 * The next pair is copied and enqueued by a helper thread of the handle while this frame is
 * tracked, and that work has finished when the call returns: next_left / next_right are not
 * read after it (ORBMI_SLAM_INLINE_FRAME=1: on the calling thread, before tracking). */
int orbmi_slam_track_stereo_ahead(orbmi_slam* h, const uint8_t* left, const uint8_t* right, int rows, int cols,
                                  size_t step, double timestamp, const uint8_t* next_left,
                                  const uint8_t* next_right, float* tcw_out, int* has_pose);

/* The counters of the `frame`-th TrackStereo call (0-based; the record stays across a reset,
 * while frame ids restart); ORBMI_E_ARG past the last call. */
int orbmi_slam_get_stats(orbmi_slam* h, int frame, orbmi_slam_frame_stats* out);
/* frames since the last reset (Frame::nNextId), keyframes, non-bad map points, LocalBundleAdjustment calls */
int orbmi_slam_get_counts(orbmi_slam* h, int* frames, int* keyframes, int* mappoints, int* local_ba_calls);
/* The poses SaveTrajectoryKITTI / TUM write (src/System.cc:334-486): per recorded frame Tcw =
 * Tcr * Trw * Two (16 floats), its timestamp and mlbLost.  capacity < n -> ORBMI_E_CAP, *n set. */
int orbmi_slam_get_trajectory(orbmi_slam* h, float* tcw, double* timestamps, uint8_t* lost, int capacity, int* n);
/* System::SaveTrajectoryKITTI / SaveTrajectoryTUM / SaveKeyFrameTrajectoryTUM. */
int orbmi_slam_save_trajectory_kitti(orbmi_slam* h, const char* path);
int orbmi_slam_save_trajectory_tum(orbmi_slam* h, const char* path);
int orbmi_slam_save_keyframe_trajectory_tum(orbmi_slam* h, const char* path);

/* ---- per-stage timing (HIP events on the handle's stream) ---------------------------- */

/* Kernel stages of one handle; each is a single kernel launch (resize: one per level). */
typedef enum orbmi_stage {
    ORBMI_STAGE_PYR_LEVEL0 = 0,
    ORBMI_STAGE_PYR_RESIZE = 1,
    ORBMI_STAGE_FAST = 2,
    ORBMI_STAGE_OCTREE = 3,
    ORBMI_STAGE_DESCRIBE = 4,
    ORBMI_STAGE_STEREO_ROWS = 5,
    ORBMI_STAGE_STEREO_MATCH = 6,
    ORBMI_STAGE_STEREO_FILTER = 7,
    ORBMI_STAGE_BLUR = 8,          /* GaussianBlur 7x7 of every level (ORBextractor.cc:1085-1086) */
    ORBMI_NUM_STAGES = 16
} orbmi_stage;

/* Bracket every launch of the stages in `stage_mask` (bit s = stage s) with HIP events. */
int orbmi_set_profiling(orbmi_extractor* h, unsigned stage_mask);
/* Synchronise, then add the elapsed device time (ms) and launch count of every bracketed
 * launch since the last call into ms[s], launches[s] (ORBMI_NUM_STAGES entries each). */
int orbmi_read_profile(orbmi_extractor* h, double* ms, long long* launches);

#ifdef __cplusplus
}
#endif
#endif /* ORBMI_H */
