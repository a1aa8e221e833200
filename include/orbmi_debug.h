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
 * [2] the outputs (rotation histogram, last assignment per keypoint); [3..6] reserved (0).
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
 * ComputeDistinctiveDescriptors calls. */
int orbmi_slam_get_phase_ms(orbmi_slam* h, double* ms, int n, long* frames);

#ifdef __cplusplus
}
#endif
#endif
