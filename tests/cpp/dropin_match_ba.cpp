// C++ drop-in check of the matcher and LocalBA layers (include/orbmi.hpp): the call shapes
// Tracking and LocalMapping make, on inputs the Python test writes as raw arrays into a
// directory.  Usage: dropin_match_ba DIR  (reads DIR/in_*.bin, writes DIR/out_*.bin)
//
//   ORBmatcher(0.8).IsInFrustum + SearchByProjection(F, local map points, th = 1)   (Tracking::SearchLocalPoints)
//   ORBmatcher(0.8).SearchLocalPoints                                               (the fused call)
//   ORBmatcher(0.9, true).SearchByProjection(CF, LF, th = 7, bMono = false)         (TrackWithMotionModel)
//   ORBmatcher(0.7, true).SearchByBoW(KF, F)                                        (TrackReferenceKeyFrame)
//   LocalBundleAdjuster: no stop flag; pbStopFlag raised before the call; SetStopAtCheck(k)
//
// tests/test_cpp_dropin.py compares every output with the oracle.
#include <cstdio>
#include <cstring>
#include <fstream>
#include <iostream>
#include <string>
#include <vector>

#include "orbmi.hpp"

static std::string g_dir;

template <class T>
static std::vector<T> load(const char* name) {
    std::ifstream f(g_dir + "/in_" + name + ".bin", std::ios::binary | std::ios::ate);
    if (!f) throw std::runtime_error(std::string("missing input ") + name);
    const std::streamsize bytes = f.tellg();
    if (bytes % (std::streamsize)sizeof(T)) throw std::runtime_error(std::string("ragged input ") + name);
    std::vector<T> v((size_t)bytes / sizeof(T));
    f.seekg(0);
    if (bytes && !f.read(reinterpret_cast<char*>(v.data()), bytes)) throw std::runtime_error("short read");
    return v;
}

template <class T>
static void save(const char* name, const std::vector<T>& v) {
    std::ofstream f(g_dir + "/out_" + name + ".bin", std::ios::binary);
    f.write(reinterpret_cast<const char*>(v.data()), (std::streamsize)(v.size() * sizeof(T)));
}

// include/Frame.h members as the matchers read them; the derived floats (grid scale, mb,
// log scale factor) come from the writer so both sides use the same values
struct FrameData {
    std::vector<orbmi::KeyPoint> keys;
    std::vector<uint8_t> desc;
    std::vector<float> ur, tcw;
    orbmi_frame_view view(const std::vector<float>& cam, const std::vector<float>& sf) const {
        orbmi_frame_view v{};
        v.n = (int)keys.size();
        v.keys_un = keys.data();
        v.u_right = ur.data();
        v.desc = desc.data();
        v.tcw = tcw.data();
        v.fx = cam[0]; v.fy = cam[1]; v.cx = cam[2]; v.cy = cam[3]; v.bf = cam[4]; v.mb = cam[5];
        v.min_x = 0.f; v.max_x = cam[6]; v.min_y = 0.f; v.max_y = cam[7];
        v.grid_w_inv = cam[8]; v.grid_h_inv = cam[9];
        v.nlevels = (int)sf.size();
        v.scale_factors = sf.data();
        v.log_scale_factor = cam[10];
        v.n_device = nullptr;
        return v;
    }
};

static FrameData frame(const std::string& p) {
    FrameData f;
    f.keys = load<orbmi::KeyPoint>((p + "_keys").c_str());
    f.desc = load<uint8_t>((p + "_desc").c_str());
    f.ur = load<float>((p + "_ur").c_str());
    f.tcw = load<float>((p + "_tcw").c_str());
    return f;
}

struct FeatureVectorData {
    std::vector<uint32_t> node;
    std::vector<int32_t> off, feat;
    orbmi_feature_vector view() const { return orbmi_feature_vector{(int)node.size(), node.data(), off.data(), feat.data()}; }
};

static FeatureVectorData featvec(const std::string& p) {
    FeatureVectorData v;
    v.node = load<uint32_t>((p + "_node").c_str());
    v.off = load<int32_t>((p + "_off").c_str());
    v.feat = load<int32_t>((p + "_feat").c_str());
    return v;
}

int main(int argc, char** argv) {
    if (argc != 2) {
        std::cerr << "usage: dropin_match_ba DIR\n";
        return 2;
    }
    g_dir = argv[1];
    try {
        const auto cam = load<float>("cam");
        const auto sf = load<float>("scale_factors");
        // ---- Tracking::SearchLocalPoints: isInFrustum(0.5), then SearchByProjection(F, points, 1)
        {
            const FrameData F = frame("local");
            const orbmi_frame_view v = F.view(cam, sf);
            const auto mps = load<orbmi_mappoint>("local_mps");
            const auto occ = load<uint8_t>("local_occ");
            orbmi::ORBmatcher matcher(0.8f, true);
            std::vector<orbmi_mappoint_track> track;
            matcher.IsInFrustum(v, mps, 0.5f, track);
            std::vector<int32_t> m;
            const int n = matcher.SearchByProjection(v, occ, mps, track, 1.0f, m);
            save("local_track", track);
            save("local_match", m);
            std::vector<int32_t> m2;
            int to_match = 0;
            const int n2 = matcher.SearchLocalPoints(v, occ, mps, 1.0f, m2, &to_match);
            save("local_fused_match", m2);
            save("local_counts", std::vector<int32_t>{n, n2, to_match});
        }
        // ---- TrackWithMotionModel: SearchByProjection(CF, LF, 7, false), ORBmatcher(0.9, true)
        {
            const FrameData CF = frame("cf"), LF = frame("lf");
            const auto lfp = load<orbmi_lastframe_point>("lf_points");
            const auto occ = load<uint8_t>("lf_occ");
            orbmi::ORBmatcher matcher(0.9f, true);
            std::vector<int32_t> m;
            const int n = matcher.SearchByProjection(CF.view(cam, sf), occ, LF.view(cam, sf), lfp, 7.0f, false, m);
            save("lf_match", m);
            save("lf_counts", std::vector<int32_t>{n});
        }
        // ---- TrackReferenceKeyFrame: SearchByBoW(KF, F), ORBmatcher(0.7, true)
        {
            const FrameData KF = frame("bkf"), F = frame("bf");
            const auto ok = load<uint8_t>("bkf_ok");
            const FeatureVectorData fk = featvec("bkf_fv"), ff = featvec("bf_fv");
            orbmi::ORBmatcher matcher(0.7f, true);
            std::vector<int32_t> m;
            const int n = matcher.SearchByBoW(KF.view(cam, sf), ok, fk.view(), F.view(cam, sf), ff.view(), m);
            save("bow_match", m);
            save("bow_counts", std::vector<int32_t>{n});
        }
        // ---- Optimizer::LocalBundleAdjustment(pKF, pbStopFlag, pMap)
        {
            const auto kfs = load<orbmi_ba_keyframe>("ba_kfs");
            const auto pts = load<orbmi_ba_point>("ba_pts");
            const auto edges = load<orbmi_ba_edge>("ba_edges");
            const auto stop_at = load<int32_t>("ba_stop_at");
            orbmi::LocalBundleAdjuster ba;
            auto put = [&](const char* tag, const orbmi::LocalBundleAdjuster::Result& r) {
                save((std::string("ba_") + tag + "_tcw").c_str(), r.tcw);
                save((std::string("ba_") + tag + "_pos").c_str(), r.pos);
                save((std::string("ba_") + tag + "_erase").c_str(), r.erase);
                save((std::string("ba_") + tag + "_info").c_str(),
                     std::vector<int32_t>{r.iterations[0], r.iterations[1], r.aborted ? 1 : 0, r.stop_check});
            };
            put("free", ba(kfs, pts, edges));                   // no pbStopFlag
            volatile int raised = 1;                             // mbAbortBA already set
            put("raised", ba(kfs, pts, edges, &raised));
            volatile int clear = 0;                              // mbAbortBA raised at check k
            ba.SetStopAtCheck(stop_at.at(0));
            put("hook", ba(kfs, pts, edges, &clear));
            ba.SetStopAtCheck(-1);
        }
        std::cout << "dropin_match_ba ok\n";
    } catch (const std::exception& e) {
        std::cerr << "error: " << e.what() << "\n";
        return 1;
    }
    return 0;
}
