// ORACLE — test infrastructure only (see orb_oracle.h).
// Frame::ComputeStereoMatches (src/Frame.cc:501-675) restated without OpenCV.
#include <algorithm>
#include <climits>
#include <cmath>
#include <cstring>
#include <utility>
#include <vector>

#include "orb_oracle.h"

namespace orc {
// from orb_extract_oracle.cpp
long pyramid_levels(const orc_params& p, const uint8_t* img, int rows, int cols, int step,
                    std::vector<std::vector<uint8_t>>& bufs, std::vector<int>& W, std::vector<int>& H);
void scale_tables(const orc_params& p, std::vector<float>& scale, std::vector<float>& inv);
}  // namespace orc

namespace {

struct LevelView {
    const uint8_t* interior;
    int w, h, stride;
    int at(int x, int y) const { return interior[(long)y * stride + x]; }
};

int hamming(const uint8_t* a, const uint8_t* b) {
    int d = 0;
    for (int i = 0; i < 32; i++) d += __builtin_popcount((unsigned)(a[i] ^ b[i]));
    return d;
}

}  // namespace

extern "C" int orc_stereo(const orc_params* p, const uint8_t* imL, const uint8_t* imR, int rows, int cols,
                          int step, float bf, float fx, const orc_keypoint* kpsL, const uint8_t* descL, int N,
                          const orc_keypoint* kpsR, const uint8_t* descR, int Nr, float* uRight, float* depth) {
    std::vector<std::vector<uint8_t>> pl, pr;
    std::vector<int> W, H;
    orc::pyramid_levels(*p, imL, rows, cols, step, pl, W, H);
    orc::pyramid_levels(*p, imR, rows, cols, step, pr, W, H);
    std::vector<float> scale, inv;
    orc::scale_tables(*p, scale, inv);
    auto view = [&](std::vector<std::vector<uint8_t>>& b, int l) {
        const int pw = W[l] + 38;
        return LevelView{b[l].data() + 19 * pw + 19, W[l], H[l], pw};
    };

    for (int i = 0; i < N; i++) { uRight[i] = -1.0f; depth[i] = -1.0f; }
    const int thOrbDist = (100 + 50) / 2;  // (TH_HIGH + TH_LOW) / 2
    const int nRows = H[0];
    std::vector<std::vector<size_t>> rowIdx(nRows);
    for (int iR = 0; iR < Nr; iR++) {
        const orc_keypoint& kp = kpsR[iR];
        const float r = 2.0f * scale[kp.octave];
        const int maxr = (int)ceilf(kp.y + r), minr = (int)floorf(kp.y - r);
        for (int yi = minr; yi <= maxr; yi++) rowIdx.at(yi).push_back(iR);
    }
    // P9: mb = bf/fx at this point (the reference reads Frame::mb before assigning it)
    const float mb = bf / fx;
    const float minZ = mb, minD = 0, maxD = bf / minZ;
    std::vector<std::pair<int, int>> vDistIdx;
    for (int iL = 0; iL < N; iL++) {
        const orc_keypoint& kpL = kpsL[iL];
        const int levelL = kpL.octave;
        const float vL = kpL.y, uL = kpL.x;
        const std::vector<size_t>& cands = rowIdx.at((size_t)vL);
        if (cands.empty()) continue;
        const float minU = uL - maxD, maxU = uL - minD;
        if (maxU < 0) continue;
        int bestDist = 100;
        size_t bestIdxR = 0;
        for (size_t iR : cands) {
            const orc_keypoint& kpR = kpsR[iR];
            if (kpR.octave < levelL - 1 || kpR.octave > levelL + 1) continue;
            const float uR = kpR.x;
            if (uR >= minU && uR <= maxU) {
                const int dist = hamming(descL + 32 * iL, descR + 32 * iR);
                if (dist < bestDist) { bestDist = dist; bestIdxR = iR; }
            }
        }
        if (bestDist >= thOrbDist) continue;
        const float uR0 = kpsR[bestIdxR].x;
        const float sf = inv[kpL.octave];
        const float scaleduL = roundf(kpL.x * sf);
        const float scaledvL = roundf(kpL.y * sf);
        const float scaleduR0 = roundf(uR0 * sf);
        const int w = 5, L = 5;
        const LevelView IL = view(pl, kpL.octave), IR = view(pr, kpL.octave);
        const int yl0 = (int)scaledvL - w, xl0 = (int)scaleduL - w;
        const float cL = (float)IL.at(xl0 + w, yl0 + w);
        int bestD = INT_MAX;
        int bestincR = 0;
        float vDists[2 * L + 1];
        const float iniu = scaleduR0 + L - w;
        const float endu = scaleduR0 + L + w + 1;
        if (iniu < 0 || endu >= IR.w) continue;
        for (int incR = -L; incR <= L; incR++) {
            const int xr0 = (int)scaleduR0 + incR - w;
            const float cR = (float)IR.at(xr0 + w, yl0 + w);
            float dist = 0;  // cv::norm(IL - cL, IR - cR, NORM_L1): exact integer sum
            double acc = 0;
            for (int r = 0; r < 2 * w + 1; r++)
                for (int c = 0; c < 2 * w + 1; c++)
                    acc += fabs((double)((float)IL.at(xl0 + c, yl0 + r) - cL) - (double)((float)IR.at(xr0 + c, yl0 + r) - cR));
            dist = (float)acc;
            if (dist < bestD) { bestD = (int)dist; bestincR = incR; }
            vDists[L + incR] = dist;
        }
        if (bestincR == -L || bestincR == L) continue;
        const float dist1 = vDists[L + bestincR - 1];
        const float dist2 = vDists[L + bestincR];
        const float dist3 = vDists[L + bestincR + 1];
        const float deltaR = (dist1 - dist3) / (2.0f * (dist1 + dist3 - 2.0f * dist2));
        if (deltaR < -1 || deltaR > 1) continue;
        float bestuR = scale[kpL.octave] * ((float)scaleduR0 + (float)bestincR + deltaR);
        float disparity = uL - bestuR;
        if (disparity >= minD && disparity < maxD) {
            if (disparity <= 0) {
                disparity = 0.01f;
                bestuR = (float)((double)uL - 0.01);
            }
            depth[iL] = bf / disparity;
            uRight[iL] = bestuR;
            vDistIdx.push_back(std::make_pair(bestD, iL));
        }
    }
    if (vDistIdx.empty()) return 0;  // P9: reference UB -> no filtering
    std::sort(vDistIdx.begin(), vDistIdx.end());
    const float median = (float)vDistIdx[vDistIdx.size() / 2].first;
    const float thDist = 1.5f * 1.4f * median;
    for (int i = (int)vDistIdx.size() - 1; i >= 0; i--) {
        if (vDistIdx[i].first < thDist) break;
        uRight[vDistIdx[i].second] = -1;
        depth[vDistIdx[i].second] = -1;
    }
    return 0;
}
