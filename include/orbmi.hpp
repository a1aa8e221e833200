// orbmi.hpp — C++ host layer over include/orbmi.h, keeping the reference's class names and call
// shapes (include/ORBextractor.h:45-111, include/ORBmatcher.h:37-102, include/Optimizer.h:62) so a
// Tracking / LocalMapping port reads like the original.  Header-only; link liborbmi.so.
//
// Differences from the reference surface, all at the type level: images are (pointer, rows, cols,
// step) instead of cv::InputArray, keypoints are orbmi::KeyPoint (cv::KeyPoint field order, so
// a std::vector<cv::KeyPoint> can be reinterpreted), descriptors are N x 32 bytes, frames and
// map points cross as the flat views of orbmi.h.  INTEGRATION.md shows the cv::Mat adapter.
// Every call throws orbmi::Error on a non-OK status: there is no CPU fallback.
#ifndef ORBMI_HPP
#define ORBMI_HPP

#include <cstdint>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "orbmi.h"

namespace orbmi {

class Error : public std::runtime_error {
public:
    Error(int status, const char* what) : std::runtime_error(std::string(what) + " failed: status " + std::to_string(status)),
                                          status_(status) {}
    int status() const { return status_; }

private:
    int status_;
};

inline void check(int rc, const char* what) {
    if (rc != ORBMI_OK) throw Error(rc, what);
}

using KeyPoint = orbmi_keypoint;
static_assert(sizeof(KeyPoint) == 28, "cv::KeyPoint layout");

// ORB_SLAM2::ORBextractor (include/ORBextractor.h:45-111)
class ORBextractor {
public:
    ORBextractor(int nfeatures, float scaleFactor, int nlevels, int iniThFAST, int minThFAST, int device = 0)
        : nfeatures_(nfeatures) {
        check(orbmi_extractor_create(device, nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST, &h_),
              "orbmi_extractor_create");
    }
    ~ORBextractor() { orbmi_extractor_destroy(h_); }
    ORBextractor(const ORBextractor&) = delete;
    ORBextractor& operator=(const ORBextractor&) = delete;
    ORBextractor(ORBextractor&& o) noexcept : h_(std::exchange(o.h_, nullptr)), nfeatures_(o.nfeatures_) {}

    // ORBextractor::operator()(image, mask, keypoints, descriptors) (src/ORBextractor.cc:1043-1105):
    // u8 gray image, rows x cols, row pitch `step`.  Empty image -> no keypoints; no keypoints ->
    // empty descriptors (descriptors.release()).
    void operator()(const uint8_t* image, int rows, int cols, size_t step, std::vector<KeyPoint>& keypoints,
                    std::vector<uint8_t>& descriptors) {
        keypoints.clear();
        descriptors.clear();
        if (rows == 0 || cols == 0 || !image) return;
        int cap = nfeatures_ + 16 * GetLevels() + 64, n = 0;
        for (;;) {
            keypoints.resize(cap);
            descriptors.resize((size_t)cap * 32);
            const int rc = orbmi_extract(h_, image, rows, cols, step, keypoints.data(), descriptors.data(), cap, &n);
            if (rc == ORBMI_E_CAP) { cap = n; continue; }
            check(rc, "orbmi_extract");
            break;
        }
        keypoints.resize(n);
        descriptors.resize((size_t)n * 32);
    }

    int GetLevels() const { return orbmi_extractor_get_levels(h_); }
    float GetScaleFactor() const { return orbmi_extractor_get_scale_factor(h_); }
    std::vector<float> GetScaleFactors() const { return levels(orbmi_extractor_get_scale_factors); }
    std::vector<float> GetInverseScaleFactors() const { return levels(orbmi_extractor_get_inverse_scale_factors); }
    std::vector<float> GetScaleSigmaSquares() const { return levels(orbmi_extractor_get_scale_sigma_squares); }
    std::vector<float> GetInverseScaleSigmaSquares() const {
        return levels(orbmi_extractor_get_inverse_scale_sigma_squares);
    }

    // mvImagePyramid[level] of the last extraction (read by Frame::ComputeStereoMatches)
    std::vector<uint8_t> ImagePyramid(int level, int rows_max, int cols_max, int* width, int* height,
                                      bool padded = false, int item = 0) const {
        const int cw = cols_max + 64, ch = rows_max + 64;
        std::vector<uint8_t> out((size_t)cw * ch);
        check(orbmi_extractor_get_pyramid_level(h_, item, level, padded, out.data(), cw, width, height),
              "orbmi_extractor_get_pyramid_level");
        std::vector<uint8_t> tight((size_t)*width * *height);
        for (int y = 0; y < *height; y++)
            for (int x = 0; x < *width; x++) tight[(size_t)y * *width + x] = out[(size_t)y * cw + x];
        return tight;
    }

    orbmi_extractor* handle() const { return h_; }

private:
    template <class F>
    std::vector<float> levels(F fn) const {
        std::vector<float> v(GetLevels());
        check(fn(h_, v.data()), "orbmi_extractor_get_*");
        return v;
    }
    orbmi_extractor* h_ = nullptr;
    int nfeatures_;
};

// Frame::ComputeStereoMatches (src/Frame.cc:501-675) on the last extractions of left / right
inline void ComputeStereoMatches(ORBextractor& left, ORBextractor& right, float bf, float fx, int nLeft,
                                 std::vector<float>& mvuRight, std::vector<float>& mvDepth) {
    mvuRight.assign(nLeft, -1.0f);
    mvDepth.assign(nLeft, -1.0f);
    if (nLeft == 0) return;
    check(orbmi_compute_stereo_matches(left.handle(), 0, right.handle(), 0, bf, fx, mvuRight.data(), mvDepth.data(),
                                       nLeft),
          "orbmi_compute_stereo_matches");
}

// ORB_SLAM2::ORBmatcher (include/ORBmatcher.h:37-102).  Results are the reference's side
// effects as index arrays (see orbmi.h for the codes).
class ORBmatcher {
public:
    static const int TH_HIGH = 100, TH_LOW = 50, HISTO_LENGTH = 30;  // src/ORBmatcher.cc:37-39

    explicit ORBmatcher(float nnratio = 0.6f, bool checkOri = true, int device = 0)
        : mfNNratio(nnratio), mbCheckOrientation(checkOri) {
        check(orbmi_matcher_create(device, &h_), "orbmi_matcher_create");
    }
    ~ORBmatcher() { orbmi_matcher_destroy(h_); }
    ORBmatcher(const ORBmatcher&) = delete;
    ORBmatcher& operator=(const ORBmatcher&) = delete;

    // ORBmatcher::DescriptorDistance (src/ORBmatcher.cc:1901-1917): popcount of a ^ b
    static int DescriptorDistance(const uint8_t* a, const uint8_t* b) {
        int d = 0;
        for (int i = 0; i < 32; i += 8) {
            uint64_t x, y;
            __builtin_memcpy(&x, a + i, 8);
            __builtin_memcpy(&y, b + i, 8);
            d += __builtin_popcountll(x ^ y);
        }
        return d;
    }

    // Frame::isInFrustum over all points (src/Frame.cc:274-342)
    void IsInFrustum(const orbmi_frame_view& F, const std::vector<orbmi_mappoint>& mps, float viewingCosLimit,
                     std::vector<orbmi_mappoint_track>& track) {
        track.resize(mps.size());
        check(orbmi_is_in_frustum(h_, &F, mps.data(), (int)mps.size(), viewingCosLimit, track.data()),
              "orbmi_is_in_frustum");
    }

    // SearchByProjection(Frame&, const vector<MapPoint*>&, th) (src/ORBmatcher.cc:59-155)
    int SearchByProjection(const orbmi_frame_view& F, const std::vector<uint8_t>& occupied,
                           const std::vector<orbmi_mappoint>& mps, const std::vector<orbmi_mappoint_track>& track,
                           float th, std::vector<int32_t>& match) {
        match.assign(F.n, -1);
        int n = 0;
        check(orbmi_search_by_projection_local(h_, &F, occupied.data(), mps.data(), track.data(), (int)mps.size(), th,
                                               mfNNratio, match.data(), &n),
              "orbmi_search_by_projection_local");
        return n;
    }

    // Tracking::SearchLocalPoints (src/Tracking.cc:1345-1403): isInFrustum(0.5) + nnratio 0.8
    int SearchLocalPoints(const orbmi_frame_view& F, const std::vector<uint8_t>& occupied,
                          const std::vector<orbmi_mappoint>& mps, float th, std::vector<int32_t>& match,
                          int* nToMatch = nullptr) {
        match.assign(F.n, -1);
        int n = 0;
        check(orbmi_search_local_points(h_, &F, occupied.data(), mps.data(), (int)mps.size(), th, match.data(), &n,
                                        nToMatch),
              "orbmi_search_local_points");
        return n;
    }

    // SearchByProjection(Frame& CF, const Frame& LF, th, bMono) (src/ORBmatcher.cc:1540-1695)
    int SearchByProjection(const orbmi_frame_view& CF, const std::vector<uint8_t>& occupied, const orbmi_frame_view& LF,
                           const std::vector<orbmi_lastframe_point>& lfPoints, float th, bool bMono,
                           std::vector<int32_t>& match) {
        match.assign(CF.n, -1);
        int n = 0;
        check(orbmi_search_by_projection_last_frame(h_, &CF, occupied.data(), &LF, lfPoints.data(), th, bMono,
                                                    mbCheckOrientation, match.data(), &n),
              "orbmi_search_by_projection_last_frame");
        return n;
    }

    // SearchByBoW(KeyFrame*, Frame&, vector<MapPoint*>&) (src/ORBmatcher.cc:211-344)
    int SearchByBoW(const orbmi_frame_view& KF, const std::vector<uint8_t>& kfMapPointOk,
                    const orbmi_feature_vector& kfFeat, const orbmi_frame_view& F, const orbmi_feature_vector& fFeat,
                    std::vector<int32_t>& match) {
        match.assign(F.n, -1);
        int n = 0;
        check(orbmi_search_by_bow(h_, &KF, kfMapPointOk.data(), &kfFeat, &F, &fFeat, mfNNratio, mbCheckOrientation,
                                  match.data(), &n),
              "orbmi_search_by_bow");
        return n;
    }

    // SearchForTriangulation(KeyFrame*, KeyFrame*, cv::Mat F12, vector<pair<size_t,size_t>>&,
    // bool bOnlyStereo) (src/ORBmatcher.cc:783-975): the matched pairs in i1 order
    int SearchForTriangulation(const orbmi_frame_view& KF1, const std::vector<uint8_t>& hasMapPoint1,
                               const orbmi_feature_vector& fv1, const orbmi_frame_view& KF2,
                               const std::vector<uint8_t>& hasMapPoint2, const orbmi_feature_vector& fv2,
                               const float F12[9], std::vector<std::pair<size_t, size_t>>& vMatchedPairs,
                               bool bOnlyStereo) {
        std::vector<int32_t> m12(KF1.n > 0 ? KF1.n : 1, -1);
        int n = 0;
        check(orbmi_search_for_triangulation(h_, &KF1, hasMapPoint1.data(), &fv1, &KF2, hasMapPoint2.data(), &fv2, F12,
                                             bOnlyStereo, mbCheckOrientation, m12.data(), &n),
              "orbmi_search_for_triangulation");
        vMatchedPairs.clear();
        vMatchedPairs.reserve(n);
        for (int i = 0; i < KF1.n; i++)
            if (m12[i] >= 0) vMatchedPairs.emplace_back((size_t)i, (size_t)m12[i]);
        return n;
    }

    // The search of Fuse(KeyFrame*, const vector<MapPoint*>&, th) (src/ORBmatcher.cc:977-1127):
    // bestIdx[i] (-1 = no fusion), bestDist[i]; the caller replays the map updates in list order
    int FuseSearch(const orbmi_frame_view& KF, const std::vector<orbmi_mappoint>& mps,
                   const std::vector<uint8_t>& inKeyFrame, float th, std::vector<int32_t>& bestIdx,
                   std::vector<int32_t>& bestDist) {
        bestIdx.assign(mps.size(), -1);
        bestDist.assign(mps.size(), 256);
        int n = 0;
        check(orbmi_fuse_search(h_, &KF, mps.data(), inKeyFrame.empty() ? nullptr : inKeyFrame.data(), (int)mps.size(),
                                th, bestIdx.data(), bestDist.data(), &n),
              "orbmi_fuse_search");
        return n;
    }

    // MapPoint::ComputeDistinctiveDescriptors (src/MapPoint.cc:247-316) for a batch of points
    void ComputeDistinctiveDescriptors(const std::vector<uint8_t>& obsDesc, const std::vector<int32_t>& obsOff,
                                       std::vector<int32_t>& best, std::vector<uint8_t>& descOut) {
        const int np = obsOff.empty() ? 0 : (int)obsOff.size() - 1;
        best.assign(np > 0 ? np : 1, -1);
        descOut.resize((size_t)(np > 0 ? np : 1) * 32);
        check(orbmi_compute_distinctive_descriptors(h_, obsDesc.data(), obsOff.data(), np, best.data(), descOut.data()),
              "orbmi_compute_distinctive_descriptors");
    }

    orbmi_matcher* handle() const { return h_; }

private:
    orbmi_matcher* h_ = nullptr;
    float mfNNratio;
    bool mbCheckOrientation;
};

// ORB_SLAM2::ORBVocabulary = DBoW2::TemplatedVocabulary<FORB::TDescriptor, FORB>
// (include/ORBVocabulary.h) on the device; transform() = TemplatedVocabulary::transform(
// features, BowVector&, FeatureVector&, levelsup), as Frame/KeyFrame::ComputeBoW call it.
class ORBVocabulary {
public:
    ORBVocabulary(const orbmi_vocabulary_desc& d, int device = 0) {
        check(orbmi_vocabulary_create(device, &d, &h_), "orbmi_vocabulary_create");
    }
    ~ORBVocabulary() { orbmi_vocabulary_destroy(h_); }
    ORBVocabulary(const ORBVocabulary&) = delete;
    ORBVocabulary& operator=(const ORBVocabulary&) = delete;

    struct BowVector { std::vector<uint32_t> word; std::vector<double> value; };
    struct FeatureVector {
        std::vector<uint32_t> node;
        std::vector<int32_t> off, feat;
        orbmi_feature_vector view() const {
            return orbmi_feature_vector{(int)node.size(), node.data(), off.data(), feat.data()};
        }
    };

    void transform(const uint8_t* desc, int n, BowVector& v, FeatureVector& fv, int levelsup) {
        const size_t cap = n > 0 ? (size_t)n : 1;
        v.word.resize(cap); v.value.resize(cap);
        fv.node.resize(cap); fv.off.resize(cap + 1); fv.feat.resize(cap);
        int counts[2] = {0, 0};
        check(orbmi_transform(h_, desc, n, nullptr, levelsup, v.word.data(), v.value.data(), fv.node.data(),
                              fv.off.data(), fv.feat.data(), counts),
              "orbmi_transform");
        v.word.resize(counts[0]); v.value.resize(counts[0]);
        fv.node.resize(counts[1]); fv.off.resize(counts[1] + 1); fv.feat.resize(fv.off.back());
    }

private:
    orbmi_vocabulary* h_ = nullptr;
};

// Optimizer::LocalBundleAdjustment (include/Optimizer.h:62) on the assembled local graph
// (src/Optimizer.cc:486-683 gathering; orbmi.h documents the arrays).  The handle keeps the
// device arena between calls; pbStopFlag is LocalMapping's mbAbortBA as an int flag.
class LocalBundleAdjuster {
public:
    struct Result {
        std::vector<float> tcw;       // nkf x 16
        std::vector<float> pos;       // npt x 3
        std::vector<uint8_t> erase;   // nedge
        int iterations[2] = {0, 0};
        double chi2[2] = {0, 0};
        bool aborted = false;
        int stop_check = -1;          // the first pbStopFlag check that found it raised (-1: none)
    };

    explicit LocalBundleAdjuster(int device = 0) { check(orbmi_ba_create(device, &h_), "orbmi_ba_create"); }
    ~LocalBundleAdjuster() { orbmi_ba_destroy(h_); }
    LocalBundleAdjuster(const LocalBundleAdjuster&) = delete;
    LocalBundleAdjuster& operator=(const LocalBundleAdjuster&) = delete;

    Result operator()(const std::vector<orbmi_ba_keyframe>& kfs, const std::vector<orbmi_ba_point>& pts,
                      const std::vector<orbmi_ba_edge>& edges, const volatile int* pbStopFlag = nullptr) {
        Result r;
        r.tcw.assign(kfs.size() * 16, 0.0f);
        r.pos.assign(pts.size() * 3, 0.0f);
        r.erase.assign(edges.size(), 0);
        orbmi_ba_problem p{(int)kfs.size(), (int)pts.size(), (int)edges.size(), kfs.data(), pts.data(), edges.data()};
        orbmi_ba_result out{r.tcw.data(), r.pos.data(), r.erase.data(), {0, 0}, {0, 0}, 0, -1, 0};
        check(orbmi_local_bundle_adjustment(h_, &p, &out, pbStopFlag), "orbmi_local_bundle_adjustment");
        r.iterations[0] = out.iterations[0];
        r.iterations[1] = out.iterations[1];
        r.chi2[0] = out.chi2[0];
        r.chi2[1] = out.chi2[1];
        r.aborted = out.aborted != 0;
        r.stop_check = out.stop_check;
        return r;
    }

    // the deterministic pbStopFlag of orbmi_ba_set_stop_at_check (k < 0: off)
    void SetStopAtCheck(int k) { check(orbmi_ba_set_stop_at_check(h_, k), "orbmi_ba_set_stop_at_check"); }

private:
    orbmi_ba* h_ = nullptr;
};

}  // namespace orbmi

#endif  // ORBMI_HPP
