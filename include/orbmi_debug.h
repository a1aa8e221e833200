/*
 * orbmi debug hooks — stage-level views used by the parity tests (tests/) to localise a
 * mismatch inside ORBextractor::operator().  Not part of the reference interface.
 */
#ifndef ORBMI_DEBUG_H
#define ORBMI_DEBUG_H
#include "orbmi.h"

#ifdef __cplusplus
extern "C" {
#endif

/* FAST candidates of `level` of batch item `item` of the last extraction, before
 * DistributeOctTree, in the reference's vToDistributeKeys order (src/ORBextractor.cc:778-829):
 * xyr = {x, y, score} int triples with x, y relative to minBorder (16, 16). */
int orbmi_debug_fast_candidates(orbmi_extractor* h, int item, int level, int* xyr, int cap, int* n_out);

/* Keypoints kept by DistributeOctTree for `level` (level coordinates, list order):
 * xyr = {x, y, score} triples. */
int orbmi_debug_octree_level(orbmi_extractor* h, int item, int level, int* xyr, int cap, int* n_out);

/* One PoseOptimization launch (orbmi_pose_optimization semantics, device arrays, one frame)
 * with an event trace in shader-clock cycles (s_memtime), trace = 16 + 64 * 8 * 8 words:
 * [0] total cycles, [1] total s_memrealtime ticks (100 MHz), [2] edge passes of wave 0; per
 * edge pass s < 64 and wave w, trace[16 + (s * 8 + w) * 8 + e] stamps e = 0 pass start, 1 pass
 * end, 2 chi2 barrier passed, 3 Levenberg decision taken, 4 (accepted trial) system reduced,
 * 5 (wave 0) trial chain published, 6 candidates barrier passed; unset stamps are 0. */
int orbmi_debug_pose_trace(orbmi_pose* h, orbmi_pose_frame* frames, const orbmi_pose_obs* obs, uint8_t* outlier,
                           unsigned long long* trace);

/* k_greedy (the order-dependent exclusion of SearchByProjection) since the last reset, summed
 * over every matcher of the process: out = {calls, rounds, largest round count, slow-path query
 * evaluations, calls that fell back to the sequential replay}; synchronises the device.  The
 * kernels collect these (and orbmi_debug_greedy_cycles) only after the first call of either. */
int orbmi_debug_greedy_stats(unsigned long long* out, int reset);

/* k_greedy's s_memtime cycles summed over calls since the last reset: out[0] prologue (queries'
 * prefixes and the keypoints' octave / occupancy loaded), [1] the rounds to the fixpoint,
 * [2] the outputs (rotation histogram, last assignment per keypoint); [3..5] thread 0's split of
 * the rounds (claims + barrier, evaluation, convergence flag + barrier); [6] reserved (0).
 * out: 7 entries. */
int orbmi_debug_greedy_cycles(unsigned long long* out, int reset);

/* The k_ba_schur launch of a LocalBA with nf free keyframes (host computation, no GPU): for
 * each of its *n_out = nf(nf+1)/2 + 2 nf + 1 blocks b, table[4b..4b+3] = {kind, x, y, z}:
 * kind 0 pose-pair block (x, y = the pair's keyframe ranks ra <= rb, z = its row-major pair
 * index); kind 1 keyframe
 * block (x = rank, y = half); kind 2 the MFMA padding block (x = y = z = -1).  cap = entries of
 * 4 ints; ORBMI_E_CAP with *n_out when short.  For the CPU test of the block table (every id a
 * permutation, every index a block reads in range). */
int orbmi_debug_ba_schur_blocks(int nf, int* table, int cap, int* n_out);

/* The schedule of a run with the concurrent LocalMapping (orbmi_slam_settings.async_local_mapping):
 * one event per acquisition of the map lock, in acquisition order.  Tracking and LocalMapping
 * touch shared state (the map, the keyframe queue, AcceptKeyFrames) only while they hold it, and
 * their GPU calls run on copies with it released, so this order -- with each LocalBA's first
 * raised pbStopFlag read (orbmi_slam_get_local_ba_log) -- determines the run: replayed through
 * the same host logic (system.StereoSLAM.replay_schedule, tests/test_native_slam_gpu.py) it gives
 * the same decisions and trajectory.  An event's label is where the thread resumes: */
#define ORBMI_SCHED_T_FRAME 1          /* Track() of frame `arg` begins                          */
#define ORBMI_SCHED_T_BOW 2            /* after TrackReferenceKeyFrame's SearchByBoW            */
#define ORBMI_SCHED_T_POSE 3           /* after a PoseOptimization call (TrackReferenceKeyFrame) */
#define ORBMI_SCHED_T_LF 4             /* after TrackWithMotionModel's searches + PoseOptimization */
#define ORBMI_SCHED_T_LOCAL 5          /* after TrackLocalMap's SearchLocalPoints + PoseOptimization */
#define ORBMI_SCHED_T_RESET 6          /* the deferred Tracking::Reset                           */
#define ORBMI_SCHED_L_JOB 16           /* the mapping thread takes the next queued keyframe (`arg`, -1 none) */
#define ORBMI_SCHED_L_DISTINCTIVE 17   /* after a ComputeDistinctiveDescriptors call             */
#define ORBMI_SCHED_L_CREATE 18        /* after CreateNewMapPoints' searches + triangulation     */
#define ORBMI_SCHED_L_CREATE_PAIR 19   /* after one pair's search (keyframes without HBM copies)  */
#define ORBMI_SCHED_L_FUSE_BATCH 20    /* after SearchInNeighbors' batched Fuse searches         */
#define ORBMI_SCHED_L_FUSE_REFRESH 21  /* after the refresh before target `arg`'s replay         */
#define ORBMI_SCHED_L_FUSE 22          /* after one Fuse search                                  */
#define ORBMI_SCHED_L_BA 23            /* after LocalBundleAdjustment's optimisation (keyframe `arg`) */
#define ORBMI_SCHED_L_BOW 24           /* after ProcessNewKeyFrame's ComputeBoW (keyframe `arg`)   */
typedef struct orbmi_slam_event {
    int32_t thread;                /* 0 Tracking, 1 LocalMapping                             */
    int32_t label, arg;
} orbmi_slam_event;
/* capacity < n -> ORBMI_E_CAP with *n set.  Empty in synchronous mode. */
int orbmi_slam_get_schedule(orbmi_slam* h, orbmi_slam_event* out, int capacity, int* n);

/* Per LocalBundleAdjustment call (either mode), in call order. */
typedef struct orbmi_slam_ba_record {
    int32_t keyframe;              /* the LocalMapping keyframe                              */
    int32_t stop_check, aborted, checks;  /* orbmi_ba_result's                               */
    int32_t iterations[2];
    int32_t edges, erased;
} orbmi_slam_ba_record;
int orbmi_slam_get_local_ba_log(orbmi_slam* h, orbmi_slam_ba_record* out, int capacity, int* n);

/* LocalMapping::Run outcomes since creation (either mode): out[0] jobs (keyframes processed),
 * [1] SearchInNeighbors skipped and [2] LocalBundleAdjustment skipped because another keyframe
 * was queued (CheckNewKeyFrames, src/LocalMapping.cc:79-90), [3] LocalBAs interrupted by
 * mbAbortBA while optimising, [4] LocalBAs that saw it raised before starting. */
int orbmi_slam_get_local_mapping_counts(orbmi_slam* h, int* out, int n);

/* Recording of the schedule, the LocalBA log and the per-keyframe state log: off by default (they
 * are replay / test hooks and grow with the run).  Turn it on before the first frame. */
int orbmi_slam_set_recording(orbmi_slam* h, int on);

/* Per-keyframe state of the map after each stage of the keyframe's LocalMapping job, in the
 * mapping thread's order (either mode; recording on).  A replay of the schedule computes the same
 * record at the same point and names the first keyframe and stage where the maps part
 * (system.StereoSLAM.replay_schedule), instead of a lock label many events later.  Hashes are
 * FNV-1a style over 32-bit words: h = (h ^ w) * 16777619, h0 = 2166136261. */
#define ORBMI_KF_STATE_PROCESS 0  /* after ProcessNewKeyFrame: a = BowVector words (-1 without a
                                     FeatureVector), b = hash of the FeatureVector (node ids, CSR
                                     offsets, feature indices), c = hash of the keyframe's slots */
#define ORBMI_KF_STATE_CREATE 1   /* after CreateNewMapPoints: a = new points, b = map points ever
                                     created, c = slot hash                                     */
#define ORBMI_KF_STATE_FUSE 2     /* after SearchInNeighbors (when it ran): a = Fuse map updates
                                     (Replace calls + AddMapPoint), b = filled slots, c = slot hash */
typedef struct orbmi_slam_kf_state {
    int32_t keyframe, stage;
    int32_t sched_index;           /* the schedule event of the section it was taken in (-1 sync) */
    int32_t a, b, c;
} orbmi_slam_kf_state;
int orbmi_slam_get_keyframe_state_log(orbmi_slam* h, orbmi_slam_kf_state* out, int capacity, int* n);

/* Wall time (ms) accumulated per phase of orbmi_slam_track_stereo since creation, and the frame
 * count: ms[0] Frame constructor (image upload, L+R extraction, stereo, read-back), [1] waiting
 * for the map lock (concurrent LocalMapping), [2] SearchByProjection(CF, LF) incl. the retry,
 * [3] its PoseOptimization, [4] UpdateLocalKeyFrames + UpdateLocalPoints, [5] the local map
 * points' records, [6] unused (isInFrustum runs inside [7]), [7] SearchByProjection(F, local
 * points), [8] its PoseOptimization, [9] CreateNewKeyFrame (+ LocalMapping when synchronous),
 * [10] total; then LocalMapping::Run on whichever thread runs it: [11] ProcessNewKeyFrame,
 * [12] MapPointCulling, [13] CreateNewMapPoints, [14] SearchInNeighbors, [15]
 * LocalBundleAdjustment, [16] KeyFrameCulling, [17] all of LocalMapping::Run; within those,
 * [18] the orbmi_create_new_map_points calls, [19] the Fuse search calls, [20] the
 * ComputeDistinctiveDescriptors calls; [21] the mapping thread's waits to re-take the map lock
 * after a device call, [22] SearchInNeighbors' set-up (targets, records, IsInKeyFrame masks),
 * [23] its per-target check of changed records, [24] its Fuse replays, [25] UpdateNormalAndDepth
 * loops, [26] UpdateConnections, [27] the observation rows of ComputeDistinctiveDescriptors,
 * [28] LocalBA's graph assembly, [29] its device call, [30] its write-back. */
int orbmi_slam_get_phase_ms(orbmi_slam* h, double* ms, int n, long* frames);

#ifdef __cplusplus
}
#endif
#endif
