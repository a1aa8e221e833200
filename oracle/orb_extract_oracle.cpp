// ORACLE — test infrastructure only (see orb_oracle.h for the pinned semantics P1-P9).
// CPU restatement of ORBextractor (src/ORBextractor.cc) without OpenCV.
#include "orb_oracle.h"
#include "../include/orbmi_pattern.h"

#include <cmath>
#include <cstring>
#include <list>
#include <algorithm>
#include <vector>

namespace orc {

static const int kPatch = 31;      // PATCH_SIZE      src/ORBextractor.cc:72
static const int kHalfPatch = 15;  // HALF_PATCH_SIZE src/ORBextractor.cc:73
static const int kEdge = 19;       // EDGE_THRESHOLD  src/ORBextractor.cc:74

// P5: cvRound = round-half-even (cvtss2si / cvtsd2si under the default MXCSR).
static inline int cv_round(float v) { return (int)lrintf(v); }
static inline int cv_round(double v) { return (int)lrint(v); }
static inline int cv_floor(float v) { int i = (int)v; return i - (i > v); }
static inline int cv_ceil(float v) { int i = (int)v; return i + (i < v); }
static inline uint8_t sat_u8(int v) { return (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v)); }
static inline short sat_s16(int v) { return (short)(v < -32768 ? -32768 : (v > 32767 ? 32767 : v)); }

// OpenCV borderInterpolate(BORDER_REFLECT_101).
static inline int reflect101(int p, int len) {
    if ((unsigned)p < (unsigned)len) return p;
    if (len == 1) return 0;
    do {
        if (p < 0) p = -p;
        else p = 2 * len - 2 - p;
    } while ((unsigned)p >= (unsigned)len);
    return p;
}

struct Plane {  // u8 plane view
    const uint8_t* p; int w, h, stride;
    uint8_t at(int x, int y) const { return p[(long)y * stride + x]; }
};

struct Tables {
    std::vector<float> scale, inv_scale, sigma2, inv_sigma2;
    std::vector<int> nfeat, umax;
};

// ORBextractor::ORBextractor  src/ORBextractor.cc:410-470
static Tables make_tables(const orc_params& p) {
    Tables t;
    const int L = p.nlevels;
    t.scale.resize(L); t.sigma2.resize(L); t.inv_scale.resize(L); t.inv_sigma2.resize(L);
    t.scale[0] = 1.0f; t.sigma2[0] = 1.0f;
    const double sf = (double)p.scale_factor;  // member `double scaleFactor` (include/ORBextractor.h:99)
    for (int i = 1; i < L; i++) {
        t.scale[i] = (float)((double)t.scale[i - 1] * sf);
        t.sigma2[i] = t.scale[i] * t.scale[i];
    }
    for (int i = 0; i < L; i++) {
        t.inv_scale[i] = 1.0f / t.scale[i];
        t.inv_sigma2[i] = 1.0f / t.sigma2[i];
    }
    t.nfeat.resize(L);
    const float factor = (float)(1.0f / sf);
    float ndes = (float)p.nfeatures * (1 - factor) /
                 (1 - (float)pow((double)factor, (double)L));
    int sum = 0;
    for (int l = 0; l < L - 1; l++) {
        t.nfeat[l] = cv_round(ndes);
        sum += t.nfeat[l];
        ndes *= factor;
    }
    t.nfeat[L - 1] = std::max(p.nfeatures - sum, 0);

    t.umax.resize(kHalfPatch + 1);
    const int vmax = cv_floor(kHalfPatch * sqrtf(2.f) / 2 + 1);
    const int vmin = cv_ceil(kHalfPatch * sqrtf(2.f) / 2);
    const double hp2 = kHalfPatch * kHalfPatch;
    for (int v = 0; v <= vmax; ++v) t.umax[v] = cv_round(sqrt(hp2 - v * v));
    for (int v = kHalfPatch, v0 = 0; v >= vmin; --v) {
        while (t.umax[v0] == t.umax[v0 + 1]) ++v0;
        t.umax[v] = v0;
        ++v0;
    }
    return t;
}

// ---------------------------------------------------------------- pyramid (P2)
// Padded level: (W+38) x (H+38), interior origin at (19,19).
struct Level {
    int w, h, pw, ph;
    std::vector<uint8_t> buf;  // pw*ph
    uint8_t* interior() { return buf.data() + kEdge * pw + kEdge; }
    const uint8_t* interior() const { return buf.data() + kEdge * pw + kEdge; }
    Plane plane() const { return Plane{interior(), w, h, pw}; }
};

// First column handled by the scalar tail of VResizeLinearVec_32s8u.
static int resize_simd_end(int width) {
    int x = 0;
    while (x <= width - 16) x += 16;
    while (x < width - 4) x += 4;
    return x;
}

// cv::resize(src, dst, Size(dw,dh), 0, 0, INTER_LINEAR) for 8U, one channel.
static void resize_linear(const Plane& s, uint8_t* dst, int dstride, int dw, int dh) {
    const int sw = s.w, sh = s.h;
    const double inv_sx = (double)dw / sw, inv_sy = (double)dh / sh;
    const double scale_x = 1. / inv_sx, scale_y = 1. / inv_sy;
    std::vector<int> xofs(dw);
    std::vector<short> ia(2 * dw);
    int xmax = dw;
    for (int dx = 0; dx < dw; dx++) {
        float fx = (float)((dx + 0.5) * scale_x - 0.5);
        int sx = cv_floor(fx);
        fx -= sx;
        if (sx < 0) { fx = 0; sx = 0; }
        if (sx + 1 >= sw) {
            xmax = std::min(xmax, dx);
            if (sx >= sw - 1) { fx = 0; sx = sw - 1; }
        }
        xofs[dx] = sx;
        ia[2 * dx] = sat_s16(cv_round((1.f - fx) * 2048));
        ia[2 * dx + 1] = sat_s16(cv_round(fx * 2048));
    }
    std::vector<int> r0(dw), r1(dw);
    auto hrow = [&](int sy, std::vector<int>& out) {
        const uint8_t* S = s.p + (long)sy * s.stride;
        for (int dx = 0; dx < dw; dx++) {
            const int sx = xofs[dx];
            out[dx] = dx < xmax ? S[sx] * ia[2 * dx] + S[sx + 1] * ia[2 * dx + 1]
                                : S[sx] * 2048;
        }
    };
    const int xv = resize_simd_end(dw);
    for (int dy = 0; dy < dh; dy++) {
        float fy = (float)((dy + 0.5) * scale_y - 0.5);
        int sy = cv_floor(fy);
        fy -= sy;
        const int b0 = sat_s16(cv_round((1.f - fy) * 2048));
        const int b1 = sat_s16(cv_round(fy * 2048));
        const int y0 = std::min(std::max(sy, 0), sh - 1);
        const int y1 = std::min(std::max(sy + 1, 0), sh - 1);
        hrow(y0, r0);
        hrow(y1, r1);
        uint8_t* D = dst + (long)dy * dstride;
        for (int dx = 0; dx < dw; dx++) {
            int v;
            if (dx < xv) {  // SSE2: srai 4, mulhi_epi16, adds, +2, srai 2, packus
                v = (((r0[dx] >> 4) * b0) >> 16) + (((r1[dx] >> 4) * b1) >> 16);
                v = (v + 2) >> 2;
            } else {
                v = (r0[dx] * b0 + r1[dx] * b1 + (1 << 21)) >> 22;
            }
            D[dx] = sat_u8(v);
        }
    }
}

static void fill_border(Level& L) {
    for (int y = 0; y < L.ph; y++)
        for (int x = 0; x < L.pw; x++) {
            const int ix = x - kEdge, iy = y - kEdge;
            if ((unsigned)ix < (unsigned)L.w && (unsigned)iy < (unsigned)L.h) continue;
            L.buf[(long)y * L.pw + x] =
                L.buf[(long)(reflect101(iy, L.h) + kEdge) * L.pw + reflect101(ix, L.w) + kEdge];
        }
}

static void level_sizes(const orc_params& p, const Tables& t, int rows, int cols,
                        std::vector<int>& W, std::vector<int>& H) {
    W.resize(p.nlevels); H.resize(p.nlevels);
    for (int l = 0; l < p.nlevels; l++) {
        W[l] = cv_round((float)cols * t.inv_scale[l]);
        H[l] = cv_round((float)rows * t.inv_scale[l]);
    }
}

// ORBextractor::ComputePyramid  src/ORBextractor.cc:1107-1132
static std::vector<Level> compute_pyramid(const orc_params& p, const Tables& t, const Plane& img) {
    std::vector<int> W, H;
    level_sizes(p, t, img.h, img.w, W, H);
    std::vector<Level> pyr(p.nlevels);
    for (int l = 0; l < p.nlevels; l++) {
        Level& L = pyr[l];
        L.w = W[l]; L.h = H[l]; L.pw = W[l] + 2 * kEdge; L.ph = H[l] + 2 * kEdge;
        L.buf.assign((size_t)L.pw * L.ph, 0);
        if (l == 0) {
            for (int y = 0; y < L.h; y++)
                memcpy(L.interior() + (long)y * L.pw, img.p + (long)y * img.stride, L.w);
        } else {
            resize_linear(pyr[l - 1].plane(), L.interior(), L.pw, L.w, L.h);
        }
        fill_border(L);  // copyMakeBorder REFLECT_101 (+ISOLATED for l>0: same on a ROI-only view)
    }
    return pyr;
}

// ---------------------------------------------------------------- FAST (P1)
// OpenCV offsets16 (circle of radius 3, clockwise from 12 o'clock in image coords).
static const int kCircle[16][2] = {{0, 3}, {1, 3}, {2, 2}, {3, 1}, {3, 0}, {3, -1}, {2, -2},
                                   {1, -3}, {0, -3}, {-1, -3}, {-2, -2}, {-3, -1}, {-3, 0},
                                   {-3, 1}, {-2, 2}, {-1, 3}};

static int corner_score16(const Plane& im, int x, int y, int threshold) {
    const int v = im.at(x, y);
    int d[25];
    for (int k = 0; k < 25; k++)
        d[k] = v - im.at(x + kCircle[k & 15][0], y + kCircle[k & 15][1]);
    int a0 = threshold;
    for (int k = 0; k < 16; k += 2) {
        int a = std::min(d[k + 1], d[k + 2]);
        a = std::min(a, d[k + 3]);
        if (a <= a0) continue;
        a = std::min(a, d[k + 4]);
        a = std::min(a, d[k + 5]);
        a = std::min(a, d[k + 6]);
        a = std::min(a, d[k + 7]);
        a = std::min(a, d[k + 8]);
        a0 = std::max(a0, std::min(a, d[k]));
        a0 = std::max(a0, std::min(a, d[k + 9]));
    }
    int b0 = -a0;
    for (int k = 0; k < 16; k += 2) {
        int b = std::max(d[k + 1], d[k + 2]);
        b = std::max(b, d[k + 3]);
        b = std::max(b, d[k + 4]);
        b = std::max(b, d[k + 5]);
        if (b >= b0) continue;
        b = std::max(b, d[k + 6]);
        b = std::max(b, d[k + 7]);
        b = std::max(b, d[k + 8]);
        b0 = std::min(b0, std::max(b, d[k]));
        b0 = std::min(b0, std::max(b, d[k + 9]));
    }
    return -b0 - 1;
}

static bool is_corner16(const Plane& im, int x, int y, int threshold) {
    const int v = im.at(x, y);
    int bright = 0, dark = 0;
    for (int k = 0; k < 16; k++) {
        const int q = im.at(x + kCircle[k][0], y + kCircle[k][1]);
        if (q > v + threshold) bright |= 1 << k;
        if (q < v - threshold) dark |= 1 << k;
    }
    for (int m : {bright, dark}) {
        int run = 0;
        for (int k = 0; k < 25; k++) {  // the 25-long wrapped scan of FAST_t
            if (m >> (k & 15) & 1) { if (++run > 8) return true; }
            else run = 0;
        }
    }
    return false;
}

struct Cand { int x, y, score; };

// cv::FAST(roi, kps, threshold, nonmax=true) on a w x h view; emits (col,row,score) in
// FAST_t's row-major order.
static void fast_roi(const Plane& roi, int threshold, std::vector<Cand>& out) {
    out.clear();
    threshold = std::min(std::max(threshold, 0), 255);
    const int w = roi.w, h = roi.h;
    if (w < 7 || h < 7) return;
    std::vector<uint8_t> score((size_t)w * h, 0);
    for (int y = 3; y < h - 3; y++)
        for (int x = 3; x < w - 3; x++)
            if (is_corner16(roi, x, y, threshold))
                score[(size_t)y * w + x] = (uint8_t)corner_score16(roi, x, y, threshold);
    for (int y = 3; y < h - 3; y++)
        for (int x = 3; x < w - 3; x++) {
            const int s = score[(size_t)y * w + x];
            if (!s) continue;
            bool keep = true;
            for (int dy = -1; dy <= 1 && keep; dy++)
                for (int dx = -1; dx <= 1; dx++) {
                    if (!dx && !dy) continue;
                    if (!(s > score[(size_t)(y + dy) * w + x + dx])) { keep = false; break; }
                }
            if (keep) out.push_back({x, y, s});
        }
}

// Candidate keypoints of ComputeKeyPointsOctTree's cell loop (src/ORBextractor.cc:778-829),
// in minBorder-relative coordinates.
static void fast_level(const orc_params& p, const Level& L, std::vector<Cand>& keys) {
    keys.clear();
    const float W = 30;
    const int minBX = kEdge - 3, minBY = minBX;
    const int maxBX = L.w - kEdge + 3, maxBY = L.h - kEdge + 3;
    const float width = (float)(maxBX - minBX), height = (float)(maxBY - minBY);
    const int nCols = (int)(width / W), nRows = (int)(height / W);
    const int wCell = (int)ceilf(width / nCols), hCell = (int)ceilf(height / nRows);
    const Plane lv = L.plane();
    std::vector<Cand> cell;
    for (int i = 0; i < nRows; i++) {
        const float iniY = (float)(minBY + i * hCell);
        float maxY = iniY + hCell + 6;
        if (iniY >= maxBY - 3) continue;
        if (maxY > maxBY) maxY = (float)maxBY;
        for (int j = 0; j < nCols; j++) {
            const float iniX = (float)(minBX + j * wCell);
            float maxX = iniX + wCell + 6;
            if (iniX >= maxBX - 6) continue;
            if (maxX > maxBX) maxX = (float)maxBX;
            const int x0 = (int)iniX, y0 = (int)iniY;
            Plane roi{lv.p + (long)y0 * lv.stride + x0, (int)maxX - x0, (int)maxY - y0, lv.stride};
            fast_roi(roi, p.ini_th_fast, cell);
            if (cell.empty()) fast_roi(roi, p.min_th_fast, cell);
            for (const Cand& c : cell) keys.push_back({c.x + j * wCell, c.y + i * hCell, c.score});
        }
    }
}

// ---------------------------------------------------------------- octree (P8)
struct Node {
    std::vector<int> keys;            // indices into the candidate vector, original order
    int ulx, uly, urx, ury, blx, bly, brx, bry;  // UL, UR, BL, BR corners
    std::list<Node>::iterator lit;
    bool no_more = false;
    long seq = 0;                     // creation sequence (P8 tie rule)
};

// ExtractorNode::DivideNode  src/ORBextractor.cc:481-537
static void divide(const Node& n, const std::vector<Cand>& C, Node& n1, Node& n2, Node& n3, Node& n4) {
    const int halfX = (int)ceilf((float)(n.urx - n.ulx) / 2);
    const int halfY = (int)ceilf((float)(n.bry - n.uly) / 2);
    n1.ulx = n.ulx; n1.uly = n.uly;
    n1.urx = n.ulx + halfX; n1.ury = n.uly;
    n1.blx = n.ulx; n1.bly = n.uly + halfY;
    n1.brx = n.ulx + halfX; n1.bry = n.uly + halfY;
    n2.ulx = n1.urx; n2.uly = n1.ury; n2.urx = n.urx; n2.ury = n.ury;
    n2.blx = n1.brx; n2.bly = n1.bry; n2.brx = n.urx; n2.bry = n.uly + halfY;
    n3.ulx = n1.blx; n3.uly = n1.bly; n3.urx = n1.brx; n3.ury = n1.bry;
    n3.blx = n.blx; n3.bly = n.bly; n3.brx = n1.brx; n3.bry = n.bly;
    n4.ulx = n3.urx; n4.uly = n3.ury; n4.urx = n2.brx; n4.ury = n2.bry;
    n4.blx = n3.brx; n4.bly = n3.bry; n4.brx = n.brx; n4.bry = n.bry;
    for (int k : n.keys) {
        const Cand& c = C[k];
        if (c.x < n1.urx) (c.y < n1.bry ? n1 : n3).keys.push_back(k);
        else (c.y < n1.bry ? n2 : n4).keys.push_back(k);
    }
    n1.no_more = n1.keys.size() == 1; n2.no_more = n2.keys.size() == 1;
    n3.no_more = n3.keys.size() == 1; n4.no_more = n4.keys.size() == 1;
}

// ORBextractor::DistributeOctTree  src/ORBextractor.cc:539-763.  Returns indices of the kept
// candidates in final list order.
static std::vector<int> distribute_octree(const std::vector<Cand>& C, int minX, int maxX,
                                          int minY, int maxY, int N) {
    const int nIni = (int)roundf((float)(maxX - minX) / (maxY - minY));
    const float hX = (float)(maxX - minX) / nIni;
    std::list<Node> nodes;
    long seq = 0;
    std::vector<Node*> ini(nIni);
    for (int i = 0; i < nIni; i++) {
        Node ni;
        ni.ulx = (int)(hX * (float)i); ni.uly = 0;
        ni.urx = (int)(hX * (float)(i + 1)); ni.ury = 0;
        ni.blx = ni.ulx; ni.bly = maxY - minY;
        ni.brx = ni.urx; ni.bry = maxY - minY;
        ni.seq = seq++;
        nodes.push_back(ni);
        ini[i] = &nodes.back();
    }
    for (size_t k = 0; k < C.size(); k++) {
        const size_t idx = (size_t)((float)C[k].x / hX);
        ini.at(idx)->keys.push_back((int)k);
    }
    for (auto it = nodes.begin(); it != nodes.end();) {
        if (it->keys.size() == 1) { it->no_more = true; ++it; }
        else if (it->keys.empty()) it = nodes.erase(it);
        else ++it;
    }

    typedef std::pair<int, Node*> SizeNode;
    // P8: sort key (size, creation sequence) instead of (size, heap address).
    auto cmp = [](const SizeNode& a, const SizeNode& b) {
        if (a.first != b.first) return a.first < b.first;
        return a.second->seq < b.second->seq;
    };
    auto push_children = [&](Node* kids, std::vector<SizeNode>* expand, int* nexp) {
        for (int q = 0; q < 4; q++) {
            if (kids[q].keys.empty()) continue;
            kids[q].seq = seq++;
            nodes.push_front(kids[q]);
            if (kids[q].keys.size() > 1) {
                if (nexp) (*nexp)++;
                expand->push_back(SizeNode((int)kids[q].keys.size(), &nodes.front()));
                nodes.front().lit = nodes.begin();
            }
        }
    };

    bool finish = false;
    std::vector<SizeNode> expand;
    while (!finish) {
        int prevSize = (int)nodes.size();
        int nToExpand = 0;
        expand.clear();
        for (auto it = nodes.begin(); it != nodes.end();) {
            if (it->no_more) { ++it; continue; }
            Node kids[4];
            divide(*it, C, kids[0], kids[1], kids[2], kids[3]);
            push_children(kids, &expand, &nToExpand);
            it = nodes.erase(it);
        }
        if ((int)nodes.size() >= N || (int)nodes.size() == prevSize) {
            finish = true;
        } else if ((int)nodes.size() + nToExpand * 3 > N) {
            while (!finish) {
                prevSize = (int)nodes.size();
                std::vector<SizeNode> prev = expand;
                expand.clear();
                std::sort(prev.begin(), prev.end(), cmp);
                for (int j = (int)prev.size() - 1; j >= 0; j--) {
                    Node kids[4];
                    divide(*prev[j].second, C, kids[0], kids[1], kids[2], kids[3]);
                    push_children(kids, &expand, nullptr);
                    nodes.erase(prev[j].second->lit);
                    if ((int)nodes.size() >= N) break;
                }
                if ((int)nodes.size() >= N || (int)nodes.size() == prevSize) finish = true;
            }
        }
    }
    std::vector<int> out;
    out.reserve(nodes.size());
    for (const Node& n : nodes) {
        int best = n.keys[0];
        for (size_t k = 1; k < n.keys.size(); k++)
            if (C[n.keys[k]].score > C[best].score) best = n.keys[k];
        out.push_back(best);
    }
    return out;
}

// ---------------------------------------------------------------- orientation (P4)
static const float kAtanP1 = 0.9997878412794807f * (float)(180 / M_PI);
static const float kAtanP3 = -0.3258083974640975f * (float)(180 / M_PI);
static const float kAtanP5 = 0.1555786518463281f * (float)(180 / M_PI);
static const float kAtanP7 = -0.04432655554792128f * (float)(180 / M_PI);

float fast_atan2(float y, float x) {
    const float ax = fabsf(x), ay = fabsf(y);
    float a, c, c2;
    if (ax >= ay) {
        c = ay / (ax + (float)2.220446049250313e-16);
        c2 = c * c;
        a = (((kAtanP7 * c2 + kAtanP5) * c2 + kAtanP3) * c2 + kAtanP1) * c;
    } else {
        c = ax / (ay + (float)2.220446049250313e-16);
        c2 = c * c;
        a = 90.f - (((kAtanP7 * c2 + kAtanP5) * c2 + kAtanP3) * c2 + kAtanP1) * c;
    }
    if (x < 0) a = 180.f - a;
    if (y < 0) a = 360.f - a;
    return a;
}

// IC_Angle  src/ORBextractor.cc:77-104
static float ic_angle(const Plane& im, int cx, int cy, const std::vector<int>& umax) {
    int m01 = 0, m10 = 0;
    for (int u = -kHalfPatch; u <= kHalfPatch; ++u) m10 += u * im.at(cx + u, cy);
    for (int v = 1; v <= kHalfPatch; ++v) {
        int vsum = 0;
        const int d = umax[v];
        for (int u = -d; u <= d; ++u) {
            const int vp = im.at(cx + u, cy + v), vm = im.at(cx + u, cy - v);
            vsum += vp - vm;
            m10 += u * (vp + vm);
        }
        m01 += v * vsum;
    }
    return fast_atan2((float)m01, (float)m10);
}

// ---------------------------------------------------------------- blur (P3)
static const int kGauss[7] = {18, 34, 49, 55, 49, 34, 18};

static void gaussian_blur(const Plane& s, std::vector<uint8_t>& out) {
    const int w = s.w, h = s.h;
    std::vector<int> rows((size_t)w * h);
    for (int y = 0; y < h; y++)
        for (int x = 0; x < w; x++) {
            int acc = 0;
            for (int k = -3; k <= 3; k++) acc += kGauss[k + 3] * s.at(reflect101(x + k, w), y);
            rows[(size_t)y * w + x] = acc;
        }
    float fk[4];
    for (int k = 0; k < 4; k++) fk[k] = (float)kGauss[3 + k] * (1.f / 65536.f);
    const int xv = (w / 4) * 4;  // SymmColumnVec_32s8u handles 16- then 4-wide blocks
    out.assign((size_t)w * h, 0);
    for (int y = 0; y < h; y++)
        for (int x = 0; x < w; x++) {
            const int c = rows[(size_t)y * w + x];
            int pr[4];
            for (int k = 1; k <= 3; k++)
                pr[k] = rows[(size_t)reflect101(y - k, h) * w + x] + rows[(size_t)reflect101(y + k, h) * w + x];
            int v;
            if (x < xv) {
                float sacc = (float)c * fk[0] + 0.0f;
                for (int k = 1; k <= 3; k++) sacc = sacc + (float)pr[k] * fk[k];
                v = (int)lrintf(sacc);
            } else {
                int iacc = c * kGauss[3];
                for (int k = 1; k <= 3; k++) iacc += pr[k] * kGauss[3 + k];
                v = (iacc + (1 << 15)) >> 16;
            }
            out[(size_t)y * w + x] = sat_u8(v);
        }
}

// ---------------------------------------------------------------- descriptor (P6)
static const float kFactorPI = (float)(M_PI / 180.f);

// computeOrbDescriptor  src/ORBextractor.cc:108-147
static void orb_descriptor(const Plane& im, float x, float y, float angle, uint8_t* desc) {
    const float ang = angle * kFactorPI;
    const float a = (float)cos((double)ang), b = (float)sin((double)ang);
    const int cx = cv_round(x), cy = cv_round(y);
    for (int i = 0; i < 32; i++) {
        int val = 0;
        for (int bit = 0; bit < 8; bit++) {
            const signed char* q = ORBMI_PATTERN[8 * i + bit];
            const float px0 = q[0], py0 = q[1], px1 = q[2], py1 = q[3];
            const int t0 = im.at(cx + cv_round(px0 * a - py0 * b), cy + cv_round(px0 * b + py0 * a));
            const int t1 = im.at(cx + cv_round(px1 * a - py1 * b), cy + cv_round(px1 * b + py1 * a));
            val |= (t0 < t1) << bit;
        }
        desc[i] = (uint8_t)val;
    }
}

struct Extracted {
    std::vector<orc_keypoint> kps;
    std::vector<uint8_t> desc;
};

// ORBextractor::operator()  src/ORBextractor.cc:1043-1105
static void extract(const orc_params& p, const Plane& img, Extracted& ex) {
    ex.kps.clear(); ex.desc.clear();
    if (img.w <= 0 || img.h <= 0) return;
    const Tables t = make_tables(p);
    std::vector<Level> pyr = compute_pyramid(p, t, img);
    std::vector<Cand> C;
    for (int l = 0; l < p.nlevels; l++) {
        const Level& L = pyr[l];
        fast_level(p, L, C);
        const int minB = kEdge - 3;
        std::vector<int> kept = distribute_octree(C, minB, L.w - kEdge + 3, minB, L.h - kEdge + 3, t.nfeat[l]);
        if (kept.empty()) continue;
        const int size = (int)(kPatch * t.scale[l]);
        std::vector<uint8_t> blurred;
        gaussian_blur(L.plane(), blurred);
        const Plane bp{blurred.data(), L.w, L.h, L.w};
        for (int k : kept) {
            orc_keypoint kp;
            const int lx = C[k].x + minB, ly = C[k].y + minB;
            kp.x = (float)lx; kp.y = (float)ly;
            kp.size = (float)size;
            kp.angle = ic_angle(L.plane(), lx, ly, t.umax);
            kp.response = (float)C[k].score;
            kp.octave = l;
            kp.class_id = -1;
            uint8_t d[32];
            orb_descriptor(bp, kp.x, kp.y, kp.angle, d);
            if (l != 0) { kp.x *= t.scale[l]; kp.y *= t.scale[l]; }
            ex.kps.push_back(kp);
            ex.desc.insert(ex.desc.end(), d, d + 32);
        }
    }
}

// Exposed to the stereo / matcher restatements.
long pyramid_levels(const orc_params& p, const uint8_t* img, int rows, int cols, int step,
                    std::vector<std::vector<uint8_t>>& bufs, std::vector<int>& W, std::vector<int>& H) {
    const Tables t = make_tables(p);
    std::vector<Level> pyr = compute_pyramid(p, t, Plane{img, cols, rows, step});
    bufs.clear(); W.clear(); H.clear();
    long total = 0;
    for (Level& L : pyr) {
        W.push_back(L.w); H.push_back(L.h);
        total += (long)L.buf.size();
        bufs.push_back(std::move(L.buf));
    }
    return total;
}

void scale_tables(const orc_params& p, std::vector<float>& scale, std::vector<float>& inv) {
    const Tables t = make_tables(p);
    scale = t.scale;
    inv = t.inv_scale;
}

}  // namespace orc

using namespace orc;

extern "C" {

int orc_tables(const orc_params* p, float* scale, float* inv_scale, float* sigma2,
               float* inv_sigma2, int* fpl, int* umax16) {
    const Tables t = make_tables(*p);
    for (int l = 0; l < p->nlevels; l++) {
        if (scale) scale[l] = t.scale[l];
        if (inv_scale) inv_scale[l] = t.inv_scale[l];
        if (sigma2) sigma2[l] = t.sigma2[l];
        if (inv_sigma2) inv_sigma2[l] = t.inv_sigma2[l];
        if (fpl) fpl[l] = t.nfeat[l];
    }
    if (umax16) for (int v = 0; v <= kHalfPatch; v++) umax16[v] = t.umax[v];
    return 0;
}

int orc_level_sizes(const orc_params* p, int rows, int cols, int* widths, int* heights) {
    const Tables t = make_tables(*p);
    std::vector<int> W, H;
    level_sizes(*p, t, rows, cols, W, H);
    for (int l = 0; l < p->nlevels; l++) { widths[l] = W[l]; heights[l] = H[l]; }
    return 0;
}

long orc_pyramid(const orc_params* p, const uint8_t* img, int rows, int cols, int step,
                 uint8_t* out, long cap) {
    const Tables t = make_tables(*p);
    std::vector<Level> pyr = compute_pyramid(*p, t, Plane{img, cols, rows, step});
    long off = 0;
    for (const Level& L : pyr) {
        if (off + (long)L.buf.size() > cap) return -3;
        memcpy(out + off, L.buf.data(), L.buf.size());
        off += (long)L.buf.size();
    }
    return off;
}

int orc_fast_level(const orc_params* p, const uint8_t* img, int rows, int cols, int step,
                   int level, int* xyr, int cap, int* n_out) {
    const Tables t = make_tables(*p);
    std::vector<Level> pyr = compute_pyramid(*p, t, Plane{img, cols, rows, step});
    std::vector<Cand> C;
    fast_level(*p, pyr[level], C);
    *n_out = (int)C.size();
    if ((int)C.size() > cap) return -3;
    for (size_t k = 0; k < C.size(); k++) {
        xyr[3 * k] = C[k].x; xyr[3 * k + 1] = C[k].y; xyr[3 * k + 2] = C[k].score;
    }
    return 0;
}

int orc_octree_level(const orc_params* p, const uint8_t* img, int rows, int cols, int step,
                     int level, int* xyr, int cap, int* n_out) {
    const Tables t = make_tables(*p);
    std::vector<Level> pyr = compute_pyramid(*p, t, Plane{img, cols, rows, step});
    std::vector<Cand> C;
    const Level& L = pyr[level];
    fast_level(*p, L, C);
    const int minB = kEdge - 3;
    std::vector<int> kept = distribute_octree(C, minB, L.w - kEdge + 3, minB, L.h - kEdge + 3, t.nfeat[level]);
    *n_out = (int)kept.size();
    if ((int)kept.size() > cap) return -3;
    for (size_t i = 0; i < kept.size(); i++) {
        xyr[3 * i] = C[kept[i]].x + minB; xyr[3 * i + 1] = C[kept[i]].y + minB; xyr[3 * i + 2] = C[kept[i]].score;
    }
    return 0;
}

int orc_blur_level(const orc_params* p, const uint8_t* img, int rows, int cols, int step,
                   int level, uint8_t* out) {
    const Tables t = make_tables(*p);
    std::vector<Level> pyr = compute_pyramid(*p, t, Plane{img, cols, rows, step});
    std::vector<uint8_t> b;
    gaussian_blur(pyr[level].plane(), b);
    memcpy(out, b.data(), b.size());
    return 0;
}

int orc_extract(const orc_params* p, const uint8_t* img, int rows, int cols, int step,
                orc_keypoint* kps, uint8_t* desc, int cap, int* n_out) {
    Extracted ex;
    extract(*p, Plane{img, cols, rows, step}, ex);
    *n_out = (int)ex.kps.size();
    if ((int)ex.kps.size() > cap) return -3;
    if (!ex.kps.empty()) {
        memcpy(kps, ex.kps.data(), ex.kps.size() * sizeof(orc_keypoint));
        memcpy(desc, ex.desc.data(), ex.desc.size());
    }
    return 0;
}

float orc_fast_atan2(float y, float x) { return fast_atan2(y, x); }

// ORBmatcher::DescriptorDistance  src/ORBmatcher.cc:1901-1917 (popcount of a^b, 256 bits)
int orc_descriptor_distance(const uint8_t* a, const uint8_t* b) {
    int d = 0;
    for (int i = 0; i < 32; i++) d += __builtin_popcount((unsigned)(a[i] ^ b[i]));
    return d;
}

}  // extern "C"
