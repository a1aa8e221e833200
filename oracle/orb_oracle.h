/*
 * ORACLE — test infrastructure only.  CPU restatement of the reference ORB front-end
 * (AHzZ123/orb_slam2_with_comment, /root/reference).  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load this library; the product path
 * (orb_slam2_with_comment_amd/csrc, liborbmi.so) never links or calls it.
 *
 * Parity status: PARTIALLY PINNED.  The reference cannot be built in this container
 * (needs OpenCV/Eigen/Pangolin, none installed; src/Tracking.cc:380 is a syntax error)
 * and ships no tests or golden vectors, so the only reference-derived anchors are the
 * known-answer values checked by tests/test_known_answers.py (umax, bit_pattern_31_
 * checksum, mnFeaturesPerLevel, pyramid sizes, thresholds, Gaussian taps).  Everything
 * the reference delegates to OpenCV/glibc is pinned below (DESIGN.md "Pinned semantics").
 *
 * Pinned semantics:
 *  P1 FAST        OpenCV 3.2 FAST_t<16> scalar: 9-arc of 16, cornerScore<16>, strict 3x3 NMS
 *                 with score 0 outside the ROI's [3,size-3) window, row-major emission.
 *  P2 resize      OpenCV 3.2 INTER_LINEAR 8U, x86-64 SSE2 build, no IPP: 11-bit coefficients,
 *                 exact integer horizontal pass; vertical pass emulates VResizeLinearVec_32s8u
 *                 ((b0*(r0>>4))>>16 + (b1*(r1>>4))>>16 + 2)>>2 for x < Xv(width) and the scalar
 *                 (b0*r0 + b1*r1 + 2^21)>>22 tail beyond it.
 *  P3 GaussianBlur 7x7 sigma 2, REFLECT_101, OpenCV 3.2 non-IPP separable filter: integer taps
 *                 {18,34,49,55,49,34,18} (sum 257), exact integer row pass; column pass emulates
 *                 SymmColumnVec_32s8u (float taps/65536, round-half-even) for x < 4*floor(W/4),
 *                 scalar (sum + 2^15)>>16 beyond it.
 *  P4 fastAtan2   OpenCV polynomial (degrees), float arithmetic.
 *  P5 cvRound     round-half-even; std::round (Frame.cc, ORBmatcher.cc) half-away-from-zero.
 *  P6 cos/sin     (float)cos((double)theta), (float)sin((double)theta) (not glibc cosf/sinf).
 *  P7 no FMA contraction anywhere (-ffp-contract=off).
 *  P8 octree tie  equal-size nodes in DistributeOctTree's refinement sort are ordered by creation
 *                 sequence (later-created compares greater) instead of heap address
 *                 (src/ORBextractor.cc:684).
 *  P9 stereo      Frame::mb is read before it is assigned in the stereo constructor
 *                 (src/Frame.cc:531 vs :109); the oracle uses mb = bf/fx.  An empty stereo
 *                 match set (UB at src/Frame.cc:662) means "no median filtering".
 */
#ifndef ORB_ORACLE_H
#define ORB_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Same field order as cv::KeyPoint (pt.x, pt.y, size, angle, response, octave, class_id). */
typedef struct orc_keypoint {
    float x, y, size, angle, response;
    int octave, class_id;
} orc_keypoint;

typedef struct orc_params {
    int nfeatures;
    float scale_factor;
    int nlevels;
    int ini_th_fast;
    int min_th_fast;
} orc_params;

/* Tables of ORBextractor::ORBextractor (src/ORBextractor.cc:410-470). */
int orc_tables(const orc_params* p, float* scale, float* inv_scale, float* sigma2,
               float* inv_sigma2, int* features_per_level, int* umax16);

/* Level sizes of ComputePyramid (src/ORBextractor.cc:1111-1112). */
int orc_level_sizes(const orc_params* p, int rows, int cols, int* widths, int* heights);

/* Padded (+19 px reflect-101 border) pyramid, levels packed back to back, each level a
 * (H_l+38) x (W_l+38) plane with stride W_l+38.  Returns the byte count written. */
long orc_pyramid(const orc_params* p, const uint8_t* img, int rows, int cols, int step,
                 uint8_t* out, long cap);

/* FAST candidates of one level before the octree (ComputeKeyPointsOctTree :778-829).
 * xyr = {x,y,score} triples in minBorder-relative coordinates, original order. */
int orc_fast_level(const orc_params* p, const uint8_t* img, int rows, int cols, int step,
                   int level, int* xyr, int cap, int* n_out);

/* Keypoints kept by DistributeOctTree for one level (level coordinates, list order). */
int orc_octree_level(const orc_params* p, const uint8_t* img, int rows, int cols, int step,
                     int level, int* xyr, int cap, int* n_out);

/* GaussianBlur of one unpadded level (P3), W_l x H_l output, stride W_l. */
int orc_blur_level(const orc_params* p, const uint8_t* img, int rows, int cols, int step,
                   int level, uint8_t* out);

/* ORBextractor::operator() (src/ORBextractor.cc:1043-1105).  Keypoints level-major,
 * coordinates scaled to level 0; desc = n x 32 bytes.  Returns 0, or -3 if cap < n
 * (n_out then holds the required count). */
int orc_extract(const orc_params* p, const uint8_t* img, int rows, int cols, int step,
                orc_keypoint* kps, uint8_t* desc, int cap, int* n_out);

/* Frame::ComputeStereoMatches (src/Frame.cc:501-675) for given left/right keypoints and
 * descriptors; the pyramids are rebuilt from the two images.  uRight/depth: N floats. */
int orc_stereo(const orc_params* p, const uint8_t* imL, const uint8_t* imR, int rows, int cols,
               int step, float bf, float fx, const orc_keypoint* kpsL, const uint8_t* descL, int N,
               const orc_keypoint* kpsR, const uint8_t* descR, int Nr, float* uRight, float* depth);

float orc_fast_atan2(float y, float x);
int orc_descriptor_distance(const uint8_t* a, const uint8_t* b);

/* The KeyFrame members CreateNewMapPoints reads (src/LocalMapping.cc:385-575): Tcw (4x4
 * row-major), mvKeysUn, mvuRight, mvDepth, fx/fy/cx/cy, mbf, mb, mvLevelSigma2, mvScaleFactors. */
typedef struct orc_tri_keyframe {
    const float* tcw;
    const orc_keypoint* keys_un;
    const float* u_right;
    const float* depth;
    float fx, fy, cx, cy, bf, mb;
    const float* level_sigma2;
    const float* scale_factors;
} orc_tri_keyframe;

/* CreateNewMapPoints' geometry for n matches (idx1[k] of kf1, idx2[k] of kf2), tri_oracle.cpp:
 * ok[k], x3d[3k..3k+2], and margin[k] (may be NULL) = the smallest relative distance of a
 * deciding quantity from its threshold on the path taken. */
int orc_triangulate_matches(const orc_tri_keyframe* kf1, const orc_tri_keyframe* kf2, const int32_t* idx1,
                            const int32_t* idx2, int n, float* x3d, uint8_t* ok, float* margin);

#ifdef __cplusplus
}
#endif
#endif
