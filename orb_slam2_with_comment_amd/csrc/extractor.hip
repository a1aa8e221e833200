// MI355X (gfx950) ORB extractor: ORBextractor::operator() (src/ORBextractor.cc:1043-1105)
// as five kernel stages over a batch of images resident in HBM:
//   k_pyramid                     ComputePyramid            (:1107-1132)    one WG per tile, all levels
//   k_fast                        cell FAST + NMS + fallback (:778-829)      one WG per cell
//   k_octree                      DistributeOctTree          (:539-763)      one WG per level
//   k_describe                    IC_Angle + GaussianBlur + computeOrbDescriptor (:77-147,
//                                 :1076-1104)                               one wave per keypoint
// Results are bit-exact with the pinned CPU restatement (oracle/, DESIGN.md "Pinned semantics").
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>

#include "../../include/orbmi_pattern.h"
#include "extractor.h"
#include "fast_score.h"
#include "trig_f64.h"

namespace orbmi {

__constant__ signed char c_pattern[256][4];
__constant__ signed char c_circle[768][2];  // (u, v) of the 749 IC_Angle patch pixels
__constant__ int c_ncircle;

// ------------------------------------------------------------------------------ pyramid
// ComputePyramid (src/ORBextractor.cc:1107-1132) in one launch: level 0 = copyMakeBorder(image,
// 19, BORDER_REFLECT_101); level l = resize(level l-1, INTER_LINEAR) + copyMakeBorder
// (REFLECT_101|ISOLATED).  One workgroup per (image, tile of the level grid): for every level the
// tile owns a rectangle (written to HBM, with the border pixels that mirror it) and computes a
// `need` rectangle into LDS = its own rectangle plus the rows / columns the next level's need
// rectangle reads (host-built, PyrTile), so the levels chain inside the workgroup with one
// barrier per level and no HBM round trip.  Halo pixels are computed by every tile that needs
// them, with the same formula.
__device__ inline void pyr_store(uint8_t* lvl, int W, int H, int stride, int x, int y, uint8_t v) {
    // interior (x, y) and every border pixel mirroring it (one reflection: W, H > kEdge)
    int xs[3], ys[3], nx = 0, ny = 0;
    xs[nx++] = x;
    if (x >= 1 && x <= kEdge) xs[nx++] = -x;
    if (x >= W - 1 - kEdge && x <= W - 2) xs[nx++] = 2 * W - 2 - x;
    ys[ny++] = y;
    if (y >= 1 && y <= kEdge) ys[ny++] = -y;
    if (y >= H - 1 - kEdge && y <= H - 2) ys[ny++] = 2 * H - 2 - y;
    for (int j = 0; j < ny; j++)
        for (int i = 0; i < nx; i++) lvl[(long long)(ys[j] + kEdge) * stride + xs[i] + kEdge] = v;
}

// cv::resize INTER_LINEAR 8U of one pixel from its four taps (pinned P2: the SSE2 vertical pass
// for x < resize_xv, the scalar tail after it).
__device__ inline int pyr_resize_px(int p00, int p01, int p10, int p11, const XTab& x, const YTab& y, bool vec) {
    const int h0 = p00 * x.a0 + p01 * x.a1;
    const int h1 = p10 * x.a0 + p11 * x.a1;
    int v;
    if (vec)  // VResizeLinearVec_32s8u lanes
        v = ((((h0 >> 4) * y.b0) >> 16) + (((h1 >> 4) * y.b1) >> 16) + 2) >> 2;
    else
        v = (h0 * y.b0 + h1 * y.b1 + (1 << 21)) >> 22;
    return v < 0 ? 0 : (v > 255 ? 255 : v);
}

constexpr int kPyrThreads = 1024;  // 64 columns x 16 rows per step
constexpr int kPyrRows = kPyrThreads / 64;
constexpr int kPyrTiledMaxBatch = 8;  // larger batches build the pyramid level by level
constexpr int kPyrLevelWords = 10; // per level in a tile's parameter block (PyrBlob, host)

// global -> LDS copy of n elements with kInFlight loads issued before the first store
template <int kInFlight, class T, class F>
__device__ inline void pyr_stage(T* dst, int n, F&& load) {
    for (int i0 = 0; i0 < n; i0 += kInFlight * kPyrThreads) {
        T v[kInFlight];
#pragma unroll
        for (int k = 0; k < kInFlight; k++) {
            const int i = i0 + k * kPyrThreads + (int)threadIdx.x;
            v[k] = i < n ? load(i) : T(0);
        }
#pragma unroll
        for (int k = 0; k < kInFlight; k++) {
            const int i = i0 + k * kPyrThreads + (int)threadIdx.x;
            if (i < n) dst[i] = v[k];
        }
    }
}

// The tile's level-0 need rectangle is its own rectangle grown by (hx, hy) (host: the largest
// halo of any tile), so it follows from blockIdx alone and the image loads go out together with
// the tile's parameter block (rectangles, level geometry, the resize taps of its need
// rectangles): one HBM round trip before all levels run out of LDS.
// It also clears the image's per-level candidate counters (k_fast allocates from them).
__global__ __launch_bounds__(kPyrThreads) void k_pyramid(const uint8_t* __restrict__ img, size_t step,
                                                         size_t img_stride, uint8_t* __restrict__ pyr, long long pimg,
                                                         const uint32_t* __restrict__ blobs, int blob_words,
                                                         int nlevels, int KX, int KY, int W0, int H0, int hx, int hy,
                                                         int* __restrict__ level_count, int lds0, int lds_half) {
    extern __shared__ uint32_t pw[];  // parameter block | level-0 rectangle | two need rectangles
    uint32_t* B = pw;
    uint8_t* L0 = reinterpret_cast<uint8_t*>(pw + blob_words);
    uint8_t* H2 = L0 + lds0;
    const int t = blockIdx.x, b = blockIdx.z, tid = threadIdx.x;
    const int tx = tid & 63, ty = tid >> 6;
    if (t == 0 && tid < nlevels * kFastRegions) level_count[b * nlevels * kFastRegions + tid] = 0;
    const uint8_t* im = img + b * img_stride;
    uint8_t* P = pyr + b * pimg;
    const int cx = t % KX, cy = t / KX;
    const int ox0 = W0 * cx / KX, ox1 = W0 * (cx + 1) / KX, oy0 = H0 * cy / KY, oy1 = H0 * (cy + 1) / KY;
    const int nx0 = max(ox0 - hx, 0), nx1 = min(ox1 + hx, W0), ny0 = max(oy0 - hy, 0), ny1 = min(oy1 + hy, H0);
    const int w0 = nx1 - nx0, a0 = w0 * (ny1 - ny0);
    const uint32_t* bl = blobs + (size_t)t * blob_words;
    pyr_stage<4>(B, blob_words, [&](int i) { return bl[i]; });
    pyr_stage<24>(L0, a0, [&](int i) {
        const int r = i / w0;
        return im[(size_t)(ny0 + r) * step + nx0 + (i - r * w0)];
    });
    __syncthreads();
    auto lo16 = [](uint32_t w) { return (int)(short)(w & 0xFFFF); };
    auto hi16 = [](uint32_t w) { return (int)(short)(w >> 16); };
    {   // level 0: the own rectangle with its border mirrors
        const uint32_t* G = B;
        const int W = lo16(G[4]), H = hi16(G[4]), stride = (int)G[5];
        uint8_t* lvl = P + G[6];
        for (int y = oy0 + ty; y < oy1; y += kPyrRows)
            for (int x = ox0 + tx; x < ox1; x += 64) pyr_store(lvl, W, H, stride, x, y, L0[(y - ny0) * w0 + x - nx0]);
    }
    int snx0 = nx0, sny0 = ny0, sw = w0;  // the source need rectangle of the next level
    for (int l = 1; l < nlevels; l++) {
        const uint32_t* G = B + l * kPyrLevelWords;
        const int o_x0 = lo16(G[0]), o_x1 = hi16(G[0]), o_y0 = lo16(G[1]), o_y1 = hi16(G[1]);
        const int n_x0 = lo16(G[2]), n_x1 = hi16(G[2]), n_y0 = lo16(G[3]), n_y1 = hi16(G[3]);
        const int W = lo16(G[4]), H = hi16(G[4]), stride = (int)G[5], rxv = (int)G[7];
        uint8_t* lvl = P + G[6];
        const uint32_t* XT = B + G[8];  // 2 words per column of the need rectangle
        const uint32_t* YT = B + G[9];  // 2 words per row
        const uint8_t* src = l == 1 ? L0 : H2 + ((l - 1) & 1) * lds_half;
        uint8_t* dst = H2 + (l & 1) * lds_half;
        const int nw = n_x1 - n_x0;
        const bool keep = l + 1 < nlevels;
        for (int y = n_y0 + ty; y < n_y1; y += kPyrRows) {
            const uint32_t y0w = YT[2 * (y - n_y0)], y1w = YT[2 * (y - n_y0) + 1];
            const YTab yy{(short)lo16(y0w), (short)hi16(y0w), (short)lo16(y1w), (short)hi16(y1w)};
            const uint8_t* r0 = src + (yy.y0 - sny0) * sw - snx0;
            const uint8_t* r1 = src + (yy.y1 - sny0) * sw - snx0;
            for (int x = n_x0 + tx; x < n_x1; x += 64) {
                const uint32_t x0w = XT[2 * (x - n_x0)], x1w = XT[2 * (x - n_x0) + 1];
                const XTab xx{(short)lo16(x0w), (short)hi16(x0w), (short)lo16(x1w), (short)hi16(x1w)};
                const uint8_t v = (uint8_t)pyr_resize_px(r0[xx.sx0], r0[xx.sx1], r1[xx.sx0], r1[xx.sx1], xx, yy, x < rxv);
                if (keep) dst[(y - n_y0) * nw + (x - n_x0)] = v;
                if (x >= o_x0 && x < o_x1 && y >= o_y0 && y < o_y1) pyr_store(lvl, W, H, stride, x, y, v);
            }
        }
        snx0 = n_x0;
        sny0 = n_y0;
        sw = nw;
        __syncthreads();
    }
}

// Large batches: one launch per level (the tiles' halo recomputation costs more than the
// launches once the batch fills the chip).  A 256-thread workgroup makes kPyrBRows padded rows of
// one level: the source rows they read are staged in LDS with aligned 16-B (level 0: 4-B) loads,
// then every thread forms 8 consecutive output bytes from LDS byte reads and stores them as one
// 8-B word (byte stores only at the row's end).  Global byte loads would bind on the texture
// addresser (one 64-lane address batch per byte).
#ifndef ORBMI_PYR_ROWS
#define ORBMI_PYR_ROWS 4
#endif
constexpr int kPyrBRows = ORBMI_PYR_ROWS;  // padded rows per workgroup (A/B builds: -DORBMI_PYR_ROWS)
constexpr int kPyrBThreads = 256;

// Level 0: copyMakeBorder(image, 19, BORDER_REFLECT_101) (src/ORBextractor.cc:1128-1129); it
// also clears the per-level candidate counters.  LDS: kPyrBRows image rows of `lrow` bytes.
__global__ __launch_bounds__(kPyrBThreads) void k_pyr_level0(const uint8_t* __restrict__ img, size_t step,
                                                             size_t img_stride, uint8_t* __restrict__ pyr, long long pimg,
                                                             LevelGeom g, int* __restrict__ level_count, int nlevels,
                                                             int lrow) {
    extern __shared__ uint32_t srow4[];
    const int b = blockIdx.z, yp0 = blockIdx.x * kPyrBRows, tid = threadIdx.x;
    if (blockIdx.x == 0 && tid < nlevels * kFastRegions) level_count[b * nlevels * kFastRegions + tid] = 0;
    const int PW = g.W + 2 * kEdge, nrow = min(kPyrBRows, g.ph - yp0);
    const int nd = (g.W + 3 + 3) / 4;  // dwords covering a row from its aligned start
    int o[kPyrBRows];
#pragma unroll
    for (int r = 0; r < kPyrBRows; r++) {
        const uint8_t* row = img + b * img_stride + (size_t)reflect101(min(yp0 + r, g.ph - 1) - kEdge, g.H) * step;
        o[r] = (int)((uintptr_t)row & 3);
    }
    for (int i = tid; i < nrow * nd; i += kPyrBThreads) {
        const int r = i / nd, d = i - r * nd;
        const uint8_t* row = img + b * img_stride + (size_t)reflect101(yp0 + r - kEdge, g.H) * step;
        srow4[r * (lrow / 4) + d] = reinterpret_cast<const uint32_t*>(row - ((uintptr_t)row & 3))[d];
    }
    __syncthreads();
    const uint8_t* sb = reinterpret_cast<const uint8_t*>(srow4);
    const int nch = (PW + 7) / 8;
    for (int t = tid; t < nrow * nch; t += kPyrBThreads) {
        const int r = t / nch, xp = 8 * (t - r * nch);
        const uint8_t* src = sb + r * lrow + o[r];
        uint8_t* dst = pyr + b * pimg + g.off + (long long)(yp0 + r) * g.stride + xp;
        uint32_t w[2] = {0u, 0u};
#pragma unroll
        for (int i = 0; i < 8; i++) w[i >> 2] |= (uint32_t)src[reflect101(min(xp + i, PW - 1) - kEdge, g.W)] << (8 * (i & 3));
        if (xp + 8 <= PW) *reinterpret_cast<uint2*>(dst) = make_uint2(w[0], w[1]);
        else
            for (int i = 0; i < PW - xp; i++) dst[i] = (uint8_t)(w[i >> 2] >> (8 * (i & 3)));
    }
}

// Level l: resize(level l-1, INTER_LINEAR) then copyMakeBorder(REFLECT_101|ISOLATED)
// (src/ORBextractor.cc:1118-1124).  Border pixels recompute the interior pixel they mirror.
// LDS: the two source rows of each output row (whole padded rows of level l-1, `lrow` bytes),
// then the level's horizontal taps (d.W entries): read per output byte, they are 8x the bytes
// written, and from global memory every 8-B lane load of a wave touched its own cache line.
__global__ __launch_bounds__(kPyrBThreads) void k_pyr_resize(uint8_t* __restrict__ pyr, long long pimg, LevelGeom s,
                                                             LevelGeom d, const XTab* __restrict__ xtg,
                                                             const YTab* __restrict__ yt, int lrow) {
    extern __shared__ uint4 srow16[];
    const int b = blockIdx.z, yp0 = blockIdx.x * kPyrBRows, tid = threadIdx.x;
    const int PW = d.W + 2 * kEdge, nrow = min(kPyrBRows, d.ph - yp0);
    const uint8_t* S = pyr + b * pimg + s.off;
    const int n16 = s.stride / 16;
    XTab* xt = reinterpret_cast<XTab*>(srow16 + 2 * kPyrBRows * (lrow / 16));
    for (int i = tid; i < d.W; i += kPyrBThreads) xt[i] = xtg[i];
    for (int i = tid; i < 2 * nrow * n16; i += kPyrBThreads) {
        const int rr = i / n16, c = i - rr * n16;  // rr = 2 * output row + tap
        const YTab y = yt[reflect101(yp0 + (rr >> 1) - kEdge, d.H)];
        const int sy = (rr & 1) ? y.y1 : y.y0;
        srow16[rr * (lrow / 16) + c] = reinterpret_cast<const uint4*>(S + (long long)(kEdge + sy) * s.stride)[c];
    }
    __syncthreads();
    const uint8_t* sb = reinterpret_cast<const uint8_t*>(srow16) + kEdge;
    const int nch = (PW + 7) / 8;
    for (int t = tid; t < nrow * nch; t += kPyrBThreads) {
        const int r = t / nch, xp = 8 * (t - r * nch);
        const YTab y = yt[reflect101(yp0 + r - kEdge, d.H)];
        const uint8_t* r0 = sb + (2 * r) * lrow;
        const uint8_t* r1 = r0 + lrow;
        uint8_t* dst = pyr + b * pimg + d.off + (long long)(yp0 + r) * d.stride + xp;
        uint32_t w[2] = {0u, 0u};
#pragma unroll
        for (int i = 0; i < 8; i++) {
            const int ix = reflect101(min(xp + i, PW - 1) - kEdge, d.W);
            const XTab x = xt[ix];
            w[i >> 2] |= (uint32_t)pyr_resize_px(r0[x.sx0], r0[x.sx1], r1[x.sx0], r1[x.sx1], x, y, ix < d.resize_xv)
                         << (8 * (i & 3));
        }
        if (xp + 8 <= PW) *reinterpret_cast<uint2*>(dst) = make_uint2(w[0], w[1]);
        else
            for (int i = 0; i < PW - xp; i++) dst[i] = (uint8_t)(w[i >> 2] >> (8 * (i & 3)));
    }
}

// Workgroup i of a 1-D grid runs on XCD i % 8.  With >= 8 images, xcd_image_map numbers the
// `per` workgroups of image b so that they share XCD b % 8 (unit w of image b: i = 8 (w + per
// (b / 8)) + b % 8): an XCD's L2 then serves the few images its workgroups walk together, not
// slices of every image.  Fewer images are interleaved over all XCDs (i = w nimg + b).
__host__ inline int xcd_image_grid(int per, int nimg) { return nimg >= 8 ? 8 * per * ((nimg + 7) / 8) : per * nimg; }
__device__ inline bool xcd_image_map(int nimg, int& unit, int& img) {
    const int i = blockIdx.x;
    if (nimg >= 8) {
        const int per = (int)gridDim.x / (8 * ((nimg + 7) / 8)), q = i >> 3;
        unit = q % per;
        img = 8 * (q / per) + (i & 7);
        return img < nimg;
    }
    unit = i / nimg;
    img = i - unit * nimg;
    return true;
}

// ------------------------------------------------------------------------------ FAST
constexpr int kTile = 64;               // max cell ROI edge (wCell+6, hCell+6): list entries are y << 6 | x
constexpr int kFastCells = 2;           // waves (cells) per workgroup
// A wave's LDS (dynamic, sized by the host for the level geometry's largest cell ROI maxW x maxH:
// ~37 x 37 for the 30-px cells of every level, so a CU holds ~3x the waves of a 64 x 64 sizing):
//   tile    maxH rows of tsd dwords (the ROI row from its aligned start: tsd = (maxW + 6) / 4)
//   scores  maxH rows of sp bytes (sp = maxW rounded up to 16)
//   list    (maxW - 6)(maxH - 6) u16 entries
struct FastLds { int tsd, sp, list, wave_bytes; };
__host__ __device__ inline FastLds fast_lds_layout(int maxW, int maxH) {
    FastLds f;
    f.tsd = (maxW + 6) / 4;
    f.sp = (maxW + 15) & ~15;
    f.list = (maxW - 6) * (maxH - 6);
    f.wave_bytes = ((4 * f.tsd * maxH + 15) & ~15) + ((maxH * f.sp + 15) & ~15) + ((2 * f.list + 15) & ~15);
    return f;
}

// LDS writes of this wave visible to its own later reads (wave-private LDS regions)
__device__ inline void wave_sync_lds_ex() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// The 16 pixels of OpenCV's offsets16 (radius-3 Bresenham circle, (dx, dy)) around (x, y).
__device__ inline void fast_circle(const uint8_t* t, int pitch, int x, int y, int p[16]) {
    const int o[16][2] = {{0, 3}, {1, 3}, {2, 2}, {3, 1}, {3, 0}, {3, -1}, {2, -2}, {1, -3},
                          {0, -3}, {-1, -3}, {-2, -2}, {-3, -1}, {-3, 0}, {-3, 1}, {-2, 2}, {-1, 3}};
    const uint8_t* c = t + y * pitch + x;
#pragma unroll
    for (int k = 0; k < 16; k++) p[k] = c[o[k][1] * pitch + o[k][0]];
}

// FAST_t's segment test: 9 contiguous circle pixels (the 25-long wrapped scan) all brighter
// than v + th or all darker than v - th.
__device__ inline bool fast_segment(int v, const int p[16], int th) {
    unsigned bright = 0, dark = 0;
#pragma unroll
    for (int k = 0; k < 16; k++) {
        bright |= (unsigned)(p[k] > v + th) << k;
        dark |= (unsigned)(p[k] < v - th) << k;
    }
    auto arc9 = [](unsigned m) {
        unsigned m2 = m | (m << 16), r = m2;
#pragma unroll
        for (int s = 1; s <= 8; s++) r &= m2 >> s;
        return (r & 0xFFFFu) != 0;
    };
    return arc9(bright) || arc9(dark);
}

// cornerScore<16> (OpenCV fast_score.cpp), d[k] = v - p[k mod 16], k < 25, stored as uchar.
// For a pixel that passes the segment test at th the value does not depend on th, and the
// pixel passes at any t >= th exactly when the value is >= t (checked exhaustively against the
// scalar restatement over 7.5e7 patches): one score per pixel serves both thresholds.
__device__ inline int fast_corner_score(int v, const int p[16], int th) {
    int d[25];
#pragma unroll
    for (int k = 0; k < 25; k++) d[k] = v - p[k & 15];
    int a0 = th;
#pragma unroll
    for (int k = 0; k < 16; k += 2) {
        int a = min(d[k + 1], d[k + 2]);
        a = min(a, d[k + 3]);
        if (a <= a0) continue;
        a = min(a, d[k + 4]);
        a = min(a, d[k + 5]);
        a = min(a, d[k + 6]);
        a = min(a, d[k + 7]);
        a = min(a, d[k + 8]);
        a0 = max(a0, min(a, d[k]));
        a0 = max(a0, min(a, d[k + 9]));
    }
    int b0 = -a0;
#pragma unroll
    for (int k = 0; k < 16; k += 2) {
        int bb = max(d[k + 1], d[k + 2]);
        bb = max(bb, d[k + 3]);
        bb = max(bb, d[k + 4]);
        bb = max(bb, d[k + 5]);
        if (bb >= b0) continue;
        bb = max(bb, d[k + 6]);
        bb = max(bb, d[k + 7]);
        bb = max(bb, d[k + 8]);
        b0 = min(b0, max(bb, d[k]));
        b0 = min(b0, max(bb, d[k + 9]));
    }
    return (-b0 - 1) & 0xFF;
}

__device__ inline int lanes_below(unsigned long long m) {
    return (int)__builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
}

// One wave per (image, cell), kFastCells cells per workgroup, so every step syncs at wave level
// only.  The cell ROI (<= 64 x 64) is staged in the wave's LDS as aligned dwords (its first byte
// at a per-cell offset 0..3).  FAST with nonmax at ini_th, then at min_th when that finds
// nothing (src/ORBextractor.cc:804-817), as four compaction stages over a row-major pixel list
// (u16 y << 6 | x, ballot-compacted in place, so the order is FAST_t's emission order):
//   A  every scored pixel: two cyclically adjacent compass pixels (0, 4, 8, 12) both brighter or
//      both darker at t = min(ini_th, min_th) -- necessary for a 9-arc (any 9 consecutive of 16
//      hold two adjacent multiples of 4);
//   B  the survivors: the full segment test at t;
//   C  the corners: cornerScore into the cell's score map (with > 64 corners, first only those at
//      ini_th, found by a second segment test; the others if the cell falls back to min_th);
//   D  strict 3x3 NMS of the corners at ini_th (score >= ini_th; neighbours below it count 0),
//      compacted in place; when none survives, the same at min_th.
// The survivors go to one of the level's kFastRegions dense candidate regions (cell k of the
// level: region k % R) at an offset taken with one atomic per cell, as {x | y << 12 | score << 24
// (x, y relative to minBorder, :820-825), cell << 10 | rank}: the tag orders them as the
// reference's cell loop does, so their position does not matter.
__global__ __launch_bounds__(64 * kFastCells) void k_fast(const uint8_t* __restrict__ pyr, long long pimg,
                                                          const LevelGeom* __restrict__ levels,
                                                          const CellGeom* __restrict__ cells, int ncells,
                                                          uint2* __restrict__ cand, int keys_cap,
                                                          int* __restrict__ level_count, int nlevels, int ini_th,
                                                          int min_th, int maxW, int maxH) {
    extern __shared__ uint4 fast_lds[];
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const FastLds F = fast_lds_layout(maxW, maxH);
    const int c = blockIdx.x * kFastCells + wid, b = blockIdx.y;
    if (c >= ncells) return;
    const CellGeom cg = cells[c];
    if (cg.w == 0) return;
    const long long a = b * pimg + cg.roi_off;
    const int o = (int)(a & 3);  // stride is a multiple of 64: the same offset on every row
    const unsigned* src = reinterpret_cast<const unsigned*>(pyr + (a - o));
    const int w = cg.w, h = cg.h, nd = (w + o + 3) >> 2, s4 = cg.stride >> 2;
    uint8_t* wl = reinterpret_cast<uint8_t*>(fast_lds) + wid * F.wave_bytes;
    unsigned* t4 = reinterpret_cast<unsigned*>(wl);
    uint4* scores4 = reinterpret_cast<uint4*>(wl + ((4 * F.tsd * maxH + 15) & ~15));
    unsigned short* L = reinterpret_cast<unsigned short*>(reinterpret_cast<uint8_t*>(scores4) + ((maxH * F.sp + 15) & ~15));
    const int TS = 4 * F.tsd, SP = F.sp;
    {
        constexpr int kLd = 8;  // loads in flight per lane (a 37 x 37 ROI: 370 dwords, one round)
        for (int i0 = 0; i0 < nd * h; i0 += 64 * kLd) {
            unsigned v[kLd];
#pragma unroll
            for (int k = 0; k < kLd; k++) {
                const int i = i0 + lane + 64 * k, r = i / nd, d = i - r * nd;
                v[k] = r < h ? src[(long long)r * s4 + d] : 0u;
            }
#pragma unroll
            for (int k = 0; k < kLd; k++) {
                const int i = i0 + lane + 64 * k, r = i / nd, d = i - r * nd;
                if (r < h) t4[r * F.tsd + d] = v[k];
            }
        }
    }
    for (int k = lane; k < (maxH * SP) / 16; k += 64) scores4[k] = make_uint4(0u, 0u, 0u, 0u);
    uint8_t* sc = reinterpret_cast<uint8_t*>(scores4);  // sc[y * SP + x]
    wave_sync_lds_ex();
    const uint8_t* tb = reinterpret_cast<const uint8_t*>(t4) + o;  // tb[y * TS + x]
    const int dw = w - 6, dh = h - 6, npix = dw > 0 && dh > 0 ? dw * dh : 0;
    const int ti = min(max(ini_th, 0), 255), tm = min(max(min_th, 0), 255), tl = min(ti, tm);
    // A: compass pre-test over the ROI's scored pixels, row-major
    int n = 0;
    if (npix > 0) {
        int y = lane / dw, x = lane - y * dw;
        const int q = 64 / dw, r = 64 - q * dw;
        for (int p0 = 0; p0 < npix; p0 += 64) {
            bool pass = false;
            const int X = x + 3, Y = y + 3;
            if (p0 + lane < npix) {
                const uint8_t* cp = tb + Y * TS + X;
                const int v = cp[0], hi = v + tl, lo = v - tl;
                const int pa = cp[3 * TS], pb = cp[3], pc = cp[-3 * TS], pd = cp[-3];
                const bool ba = pa > hi, bb = pb > hi, bc = pc > hi, bd = pd > hi;
                const bool da = pa < lo, db = pb < lo, dc = pc < lo, dd = pd < lo;
                pass = (ba & bb) | (bb & bc) | (bc & bd) | (bd & ba) | (da & db) | (db & dc) | (dc & dd) | (dd & da);
            }
            const unsigned long long m = __ballot(pass);
            if (pass) L[n + lanes_below(m)] = (unsigned short)(Y << 6 | X);
            n += __popcll(m);
            x += r;
            y += q;
            if (x >= dw) { x -= dw; y++; }
        }
    }
    wave_sync_lds_ex();
    // B: full segment test, compacted in place (a lane writes at or below the entry it read)
    int nc = 0;
    for (int i0 = 0; i0 < n; i0 += 64) {
        const int i = i0 + lane;
        bool pass = false;
        unsigned short e = 0;
        if (i < n) {
            e = L[i];
            const int X = e & 63, Y = e >> 6;
            int p[16];
            fast_circle(tb, TS, X, Y, p);
            pass = fast_segment(tb[Y * TS + X], p, tl);
        }
        const unsigned long long m = __ballot(pass);
        if (pass) L[nc + lanes_below(m)] = e;
        nc += __popcll(m);
    }
    wave_sync_lds_ex();
    // B': with more corners than one pass of the wave scores (nc > 64) and ini_th > min_th, the
    // corners at ini_th among them (segment test again, listed after them, L2 = L + nc, when the
    // list has room for both): a corner passes at t exactly
    // when its score is >= t, so the NMS at ini_th needs the scores of those only (the others
    // count 0 as neighbours); the rest are scored only if the cell falls back to min_th.  With
    // nc <= 64 the scoring pass costs the wave the same for any subset.
    const bool split = ti > tl && nc > 64 && 2 * nc <= F.list;
    unsigned short* L2 = L + nc;
    unsigned short* LH = L;
    int nh = nc;
    if (split) {
        LH = L2;
        nh = 0;
        for (int i0 = 0; i0 < nc; i0 += 64) {
            const int i = i0 + lane;
            bool pass = false;
            unsigned short e = 0;
            if (i < nc) {
                e = L[i];
                const int X = e & 63, Y = e >> 6;
                int p[16];
                fast_circle(tb, TS, X, Y, p);
                pass = fast_segment(tb[Y * TS + X], p, ti);
            }
            const unsigned long long m = __ballot(pass);
            if (pass) L2[nh + lanes_below(m)] = e;
            nh += __popcll(m);
        }
        wave_sync_lds_ex();
    }
    // C: scores of the corners (of LH)
    auto score = [&](const unsigned short* Ls, int ns) {
        for (int i = lane; i < ns; i += 64) {
            const unsigned short e = Ls[i];
            const int X = e & 63, Y = e >> 6;
            int p[16];
            fast_circle(tb, TS, X, Y, p);
            sc[Y * SP + X] = (uint8_t)fast_corner_score(tb[Y * TS + X], p, tl);
        }
        wave_sync_lds_ex();
    };
    // D: strict NMS at threshold t over Ls, survivors compacted in place
    auto nms = [&](unsigned short* Ls, int ns, int t) {
        int kept = 0;
        for (int i0 = 0; i0 < ns; i0 += 64) {
            const int i = i0 + lane;
            bool keep = false;
            unsigned short e = 0;
            if (i < ns) {
                e = Ls[i];
                const uint8_t* q = sc + (e >> 6) * SP + (e & 63);
                const int s = q[0];
                if (s >= t && s != 0) {
                    auto nb = [&](int off) {
                        const int u = q[off];
                        return u >= t ? u : 0;
                    };
                    keep = s > nb(-SP - 1) && s > nb(-SP) && s > nb(-SP + 1) && s > nb(-1) && s > nb(1) &&
                           s > nb(SP - 1) && s > nb(SP) && s > nb(SP + 1);
                }
            }
            const unsigned long long m = __ballot(keep);
            if (keep) Ls[kept + lanes_below(m)] = e;
            kept += __popcll(m);
        }
        return kept;
    };
    score(LH, nh);
    int total = nms(LH, nh, ti);  // at ini_th, then at min_th if nothing survived
    const unsigned short* LO = LH;
    if (total == 0 && tm != ti) {
        if (split) score(L, nc);
        total = nms(L, nc, tm);
        LO = L;
    }
    if (total == 0) return;
    wave_sync_lds_ex();
    int base = 0;
    if (lane == 0)
        base = atomicAdd(&level_count[(b * nlevels + cg.level) * kFastRegions + cg.lcell % kFastRegions], total);
    base = __shfl(base, 0);
    uint2* dst = cand + (long long)b * keys_cap + cg.slot_base + base;
    const unsigned tag = (unsigned)cg.lcell << 10;
    for (int i = lane; i < total; i += 64) {
        const unsigned short e = LO[i];
        const int X = e & 63, Y = e >> 6;
        dst[i] = make_uint2((uint32_t)(X + cg.sx) | ((uint32_t)(Y + cg.sy) << 12) | ((uint32_t)sc[Y * SP + X] << 24),
                            tag | (unsigned)i);
    }
}

// k_fast2: k_fast with fewer VALU instructions per cell (k_fast issues ≈2,900 per cell and is
// VALU-issue-bound).  The ROI tile and the score map have a compile-time pitch TS, so every
// circle / compass / NMS neighbour read is one ds_read_u8 with an immediate offset from the
// pixel's address, and the list holds tile offsets (y TS + x) rather than packed coordinates;
// each circle comparison enters the lane's 16-bit mask with one compare and one add-with-carry;
// the arc test is doubling on the mask (runs of 2, 4, 8, 9).  The compass pre-test combines its
// eight compares as lane masks.  Measured alternatives (profiles/r04/fast_seg_ab.txt): the arc
// test bit-sliced across the wave on the scalar unit (79 SALU ops per polarity for 64 pixels)
// cut the VALU count by 40 % but made the kernel slower, 0.327 vs 0.307 ms per 64 frames: the
// scalar unit issues at the same per-SIMD rate as the vector unit.  Outputs and their order are
// k_fast's.  Round 6 (kStrength, the default; ORBMI_FAST=split keeps the stages above for A/B):
// stages B and C are one pass of fast_arc_strength (fast_score.h: packed 16-bit min/max, S > t is
// the segment test at t and S - 1 the score), run first at ini_th on the compass survivors at
// ini_th and at min_th only for a cell with no survivor; the window bases are kept out of the
// reads' address folding (lds_window), and NMS reads its eight neighbours unconditionally.
// Config 5: FAST 0.289 -> 0.164 ms per 64 frames (profiles/r06/fastab.txt).
// m * 2 + (a > b): the compare's lane mask is the add's carry-in (two VALU ops per bit; the
// compiler's own form is compare, select, shift-or)
__device__ inline unsigned shift_in_gt(unsigned m, int a, int b) {
    unsigned r;
    asm("v_cmp_gt_i32_e32 vcc, %1, %2\n\tv_addc_co_u32_e32 %0, vcc, %3, %3, vcc" : "=v"(r) : "v"(a), "v"(b), "v"(m) : "vcc");
    return r;
}

// FAST's arc test on one lane's 16-bit circle mask (bit k = circle pixel k): runs of 2, 4, 8, 9
// by doubling on m | m << 16 (a cyclic run starting at s < 16 is bits s .. s + 8).
__device__ inline bool fast_arc9_word(unsigned m) {
    unsigned x = m | (m << 16);
    x &= x >> 1;
    x &= x >> 2;
    x &= x >> 4;
    x &= x >> 1;
    return (x & 0xFFFFu) != 0;
}

// The segment test of every lane's pixel: cm = the pixel at (X - 3, Y - 3) of the tile (pitch
// TS), so all 17 reads take non-negative immediate offsets.  The caller masks inactive lanes.
template <int TS>
__device__ inline bool fast_segment_lane(const uint8_t* cm, int th) {
    constexpr int o[16] = {6 * TS + 3, 6 * TS + 4, 5 * TS + 5, 4 * TS + 6, 3 * TS + 6, 2 * TS + 6, TS + 5, 4,
                           3, 2, TS + 1, 2 * TS, 3 * TS, 4 * TS, 5 * TS + 1, 6 * TS + 2};
    int p[16];
#pragma unroll
    for (int k = 0; k < 16; k++) p[k] = cm[o[k]];
    const int v = cm[3 * TS + 3], hi = v + th, lo = v - th;
    unsigned mb = 0, md = 0;
#pragma unroll
    for (int k = 15; k >= 0; k--) {
        mb = shift_in_gt(mb, p[k], hi);
        md = shift_in_gt(md, lo, p[k]);
    }
    return fast_arc9_word(mb) || fast_arc9_word(md);
}

// fast_arc_strength (fast_score.h) of every lane's pixel, cm as for fast_segment_lane
template <int TS>
__device__ inline int fast_strength_lane(const uint8_t* cm, int th) {
    constexpr int o[16] = {6 * TS + 3, 6 * TS + 4, 5 * TS + 5, 4 * TS + 6, 3 * TS + 6, 2 * TS + 6, TS + 5, 4,
                           3, 2, TS + 1, 2 * TS, 3 * TS, 4 * TS, 5 * TS + 1, 6 * TS + 2};
    int p[16];
#pragma unroll
    for (int k = 0; k < 16; k++) p[k] = cm[o[k]];
    return fast_arc_strength(cm[3 * TS + 3], p, th);
}

// e - back as an offset the compiler cannot fold into the reads that follow: they then take the
// window's offsets as non-negative ds_read immediates (folded, the negative ones cost a VALU add
// each)
__device__ inline int lds_window(int e, int back) {
    int b = e - back;
    asm volatile("" : "+v"(b));
    return b;
}

constexpr int fast2_tile_bytes(int TS, int maxH) { return (TS * maxH + 15) & ~15; }
__host__ __device__ inline int fast2_wave_bytes(int TS, int maxW, int maxH) {
    return 2 * fast2_tile_bytes(TS, maxH) + ((2 * (maxW - 6) * (maxH - 6) + 15) & ~15);
}

template <int TS, bool kStrength>
__global__ __launch_bounds__(64 * kFastCells) void k_fast2(const uint8_t* __restrict__ pyr, long long pimg,
                                                           const CellGeom* __restrict__ cells, int c0, int ncells,
                                                           uint2* __restrict__ cand, int keys_cap,
                                                           int* __restrict__ level_count, int nlevels, int ini_th,
                                                           int min_th, int maxW, int maxH, int nimg) {
    extern __shared__ uint4 fast_lds[];
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    int unit, b;
    if (!xcd_image_map(nimg, unit, b)) return;
    const int c = c0 + unit * kFastCells + wid;  // cells [c0, ncells)
    if (c >= ncells) return;
    const CellGeom cg = cells[c];
    if (cg.w == 0) return;
    const long long a = b * pimg + cg.roi_off;
    const int o = (int)(a & 3);  // stride is a multiple of 64: the same offset on every row
    const unsigned* src = reinterpret_cast<const unsigned*>(pyr + (a - o));
    const int w = cg.w, h = cg.h, nd = (w + o + 3) >> 2, s4 = cg.stride >> 2;
    const int tbytes = fast2_tile_bytes(TS, maxH), lcap = (maxW - 6) * (maxH - 6);
    uint8_t* wl = reinterpret_cast<uint8_t*>(fast_lds) + wid * fast2_wave_bytes(TS, maxW, maxH);
    unsigned* t4 = reinterpret_cast<unsigned*>(wl);
    uint8_t* sc = wl + tbytes;  // scores, sc[y * TS + x]
    unsigned short* L = reinterpret_cast<unsigned short*>(wl + 2 * tbytes);
    {   // lane = (row phase r0, dword d) of the tile, R rows per round: one division per lane
        const int R = 64 / nd, r0 = lane / nd, d = lane - r0 * nd;
        if (r0 < R) {
            constexpr int kLd = 8;
            for (int rb = r0; rb < h; rb += kLd * R) {
                unsigned v[kLd];
#pragma unroll
                for (int k = 0; k < kLd; k++) {
                    const int r = rb + k * R;
                    v[k] = r < h ? src[(long long)r * s4 + d] : 0u;
                }
#pragma unroll
                for (int k = 0; k < kLd; k++) {
                    const int r = rb + k * R;
                    if (r < h) t4[r * (TS / 4) + d] = v[k];
                }
            }
        }
    }
    for (int k = lane; k < tbytes / 16; k += 64) reinterpret_cast<uint4*>(sc)[k] = make_uint4(0u, 0u, 0u, 0u);
    wave_sync_lds_ex();
    const uint8_t* tb = reinterpret_cast<const uint8_t*>(t4) + o;  // tb[y * TS + x]
    const int dw = w - 6, dh = h - 6, npix = dw > 0 && dh > 0 ? dw * dh : 0;
    const int ti = min(max(ini_th, 0), 255), tm = min(max(min_th, 0), 255), tl = min(ti, tm);
    // A: compass pre-test at t over the ROI's scored pixels, row-major, into L
    auto compass = [&](int t) {
        int n = 0;
        if (npix > 0) {
            int y = lane / dw, x = lane - y * dw;
            const int q = 64 / dw, r = 64 - q * dw;
            for (int p0 = 0; p0 < npix; p0 += 64) {
                // lanes past the last pixel read the ROI's last row (masked off below)
                const int e0 = __umul24(min(y, dh - 1), TS) + x + 3;  // the pixel at (X, Y - 3)
                const uint8_t* cp = tb + e0;
                const int pc = cp[0], pd = cp[3 * TS - 3], v = cp[3 * TS], pb = cp[3 * TS + 3], pa = cp[6 * TS];
                const int hi = v + t, lo = v - t;
                const bool ba = pa > hi, bb = pb > hi, bc = pc > hi, bd = pd > hi;
                const bool da = pa < lo, db = pb < lo, dc = pc < lo, dd = pd < lo;
                const bool pass = (((ba | bc) & (bb | bd)) | ((da | dc) & (db | dd))) && p0 + lane < npix;
                const unsigned long long m = __ballot(pass);
                if (pass) L[n + lanes_below(m)] = (unsigned short)(e0 + 3 * TS);
                n += __popcll(m);
                x += r;
                y += q;
                if (x >= dw) { x -= dw; y++; }
            }
        }
        wave_sync_lds_ex();
        return n;
    };
    auto nms = [&](unsigned short* Ls, int ns, int t) {
        int kept = 0;
        for (int i0 = 0; i0 < ns; i0 += 64) {
            const int i = i0 + lane;
            bool keep = false;
            unsigned short e = 0;
            if (i < ns) {
                e = Ls[i];
                const uint8_t* q = sc + lds_window(e, TS + 1);  // the 3x3 window's top-left
                const int s = q[TS + 1];
                const int u[8] = {q[0], q[1], q[2], q[TS], q[TS + 2], q[2 * TS], q[2 * TS + 1], q[2 * TS + 2]};
                keep = s >= t && s != 0;  // a neighbour below t counts 0
#pragma unroll
                for (int k = 0; k < 8; k++) keep &= u[k] < t || s > u[k];
            }
            const unsigned long long m = __ballot(keep);
            if (keep) Ls[kept + lanes_below(m)] = e;
            kept += __popcll(m);
        }
        return kept;
    };
    int total = 0;
    const unsigned short* LO = L;
    if constexpr (kStrength) {
        // B + C at once: S = fast_arc_strength at t; a corner at t' >= t exactly when S > t', its
        // score S - 1 whatever t (fast_score.h), so the pass both finds and scores the corners and
        // NMS reads the map at either threshold (scores below it count 0 there)
        auto strength = [&](int n, int t) {
            int nc = 0;
            for (int i0 = 0; i0 < n; i0 += 64) {
                const int i = i0 + lane;
                const unsigned short e = L[min(i, n - 1)];
                const int S = fast_strength_lane<TS>(tb + lds_window(e, 3 * TS + 3), t);
                const bool pass = S > t && i < n;
                const unsigned long long m = __ballot(pass);
                if (pass) {
                    L[nc + lanes_below(m)] = e;
                    sc[e] = (uint8_t)(S - 1);
                }
                nc += __popcll(m);
            }
            wave_sync_lds_ex();
            return nc;
        };
        // FAST at ini_th first, from its own compass survivors (a corner at ini_th, and so every
        // neighbour NMS at ini_th counts, passes the compass at ini_th): about half the candidates
        // of the compass at min_th.  Only a cell without a survivor runs the min_th pass (the
        // scores it rewrites are the same values).  With min_th >= ini_th one pass at ini_th
        // holds the corners of both.
        const bool two = tm < ti;
        int nc = strength(compass(two ? ti : tl), two ? ti : tl);
        total = nms(L, nc, ti);
        if (total == 0 && tm != ti) {
            if (two) nc = strength(compass(tm), tm);
            total = nms(L, nc, tm);
        }
    } else {
        const int n = compass(tl);
        // B: full segment test at tl, compacted in place (a lane writes at or below the entry it read)
        auto segment_pass = [&](const unsigned short* Ls, int ns, unsigned short* Ld, int th) {
            int kept = 0;
            for (int i0 = 0; i0 < ns; i0 += 64) {
                const int i = i0 + lane;
                const unsigned short e = Ls[min(i, ns - 1)];  // the last lanes repeat an entry, masked off
                const bool pass = fast_segment_lane<TS>(tb + lds_window(e, 3 * TS + 3), th) && i < ns;
                const unsigned long long m = __ballot(pass);
                if (pass) Ld[kept + lanes_below(m)] = e;
                kept += __popcll(m);
            }
            wave_sync_lds_ex();
            return kept;
        };
        const int nc = segment_pass(L, n, L, tl);
        // B': the corners at ini_th among them, listed after them (see k_fast)
        const bool split = ti > tl && nc > 64 && 2 * nc <= lcap;
        unsigned short* LH = L;
        int nh = nc;
        if (split) {
            LH = L + nc;
            nh = segment_pass(L, nc, LH, ti);
        }
        // C: cornerScore of the corners
        auto score = [&](const unsigned short* Ls, int ns) {
            for (int i = lane; i < ns; i += 64) {
                const unsigned short e = Ls[i];
                int p[16];
                fast_circle(tb + e, TS, 0, 0, p);
                sc[e] = (uint8_t)fast_corner_score(tb[e], p, tl);
            }
            wave_sync_lds_ex();
        };
        score(LH, nh);
        total = nms(LH, nh, ti);
        LO = LH;
        if (total == 0 && tm != ti) {
            if (split) score(L, nc);
            total = nms(L, nc, tm);
            LO = L;
        }
    }
    if (total == 0) return;
    wave_sync_lds_ex();
    int base = 0;
    if (lane == 0)
        base = atomicAdd(&level_count[(b * nlevels + cg.level) * kFastRegions + cg.lcell % kFastRegions], total);
    base = __shfl(base, 0);
    uint2* dst = cand + (long long)b * keys_cap + cg.slot_base + base;
    const unsigned tag = (unsigned)cg.lcell << 10;
    for (int i = lane; i < total; i += 64) {
        const unsigned short e = LO[i];
        const int Y = e / TS, X = e - Y * TS;
        dst[i] = make_uint2((uint32_t)(X + cg.sx) | ((uint32_t)(Y + cg.sy) << 12) | ((uint32_t)sc[e] << 24),
                            tag | (unsigned)i);
    }
}

// ------------------------------------------------------------------------------ octree
// DistributeOctTree (src/ORBextractor.cc:539-763) as data-parallel passes inside one
// workgroup per (image, level).  The std::list of nodes is kept as arrays in list order:
// a pass that divides D nodes pushes their non-empty children to the list front in visit
// order, so the new list is [children in reverse push order] ++ [undivided nodes in order]
// -- two prefix scans.  Keys never move: each key carries the index of its node, remapped
// after every pass through the parent's (node, quadrant) -> child table.
constexpr int kOctThreads = 1024;
constexpr int kOctRegKeys = 12;  // candidates per thread held in registers (12,288 per level; 13 spills)
#ifdef ORBMI_OCT_TRACE  // tools/octree_trace.hip: s_memtime stamps of workgroup g_oct_trace_block
__device__ unsigned long long g_oct_trace[256];
__device__ int g_oct_trace_block;
#define OCT_STAMP(i, v)                                                                                   \
    do {                                                                                                  \
        if (threadIdx.x == 0 && (int)blockIdx.x == g_oct_trace_block && blockIdx.y == 0) g_oct_trace[i] = (v); \
    } while (0)
#define OCT_SUB(it, j) do { if ((it) < 15) OCT_STAMP(100 + 10 * (it) + (j), __builtin_amdgcn_s_memtime()); } while (0)
#else
#define OCT_STAMP(i, v) do {} while (0)
#define OCT_SUB(it, j) do {} while (0)
#endif

struct OctShared {
    int cnt[2][kOctNodeCap];
    int ccnt[kOctNodeCap][4];            // child key counts; reused as best-key words
    short remap[kOctNodeCap][4];         // (old node, quadrant) -> new index
    unsigned long long skey[kOctNodeCap];
    int tmp[kOctNodeCap];
    int newpos[kOctNodeCap];
    unsigned char dflag[kOctNodeCap];
    int scratch[kOctThreads / 64 + 2];
    int misc[8];
    int rpre[kFastRegions + 1];          // candidate regions: prefix of counts, first slots
    int rbase[kFastRegions];
    unsigned tagl[kOctThreads * kOctRegKeys];  // order tags of the register-resident keys
};

// Quadrant decisions of one axis down the quadtree's fixed geometry: bit d is the decision at
// depth d (coordinate >= the box's mid, mid = lo + ceil((hi - lo) / 2)).  A child's extent on an
// axis depends only on the parent's extent on that axis and the decision
// (ExtractorNode::DivideNode, src/ORBextractor.cc:481-537), so each axis descends alone and a
// key's quadrant in its node at depth d is ((px >> d) & 1) | ((py >> d) & 1) << 1.  Coordinates
// are < 4096, so two keys are separated within 13 divisions; 16 are kept.
__device__ inline unsigned oct_axis(int v, int lo, int hi) {
    unsigned bits = 0;
#pragma unroll
    for (int d = 0; d < 16; d++) {
        const int mid = lo + ((hi - lo + 1) >> 1);
        const bool up = v >= mid;
        bits |= (unsigned)up << d;
        lo = up ? mid : lo;
        hi = up ? hi : mid;
    }
    return bits;
}

// Root node of a key (src/ORBextractor.cc:573-579) and its path bits (x low half, y high half).
__device__ inline int oct_root(uint32_t key, const LevelGeom& g) {
    return min((int)((float)(key & 0xFFF) / g.hX), g.nIni - 1);
}
__device__ inline unsigned oct_path(uint32_t key, const LevelGeom& g) {
    const int n = oct_root(key, g);
    const int x0 = (int)(g.hX * (float)n), x1 = (int)(g.hX * (float)(n + 1));
    return oct_axis((int)(key & 0xFFF), x0, x1) | oct_axis((int)((key >> 12) & 0xFFF), 0, g.height) << 16;
}
__device__ inline int oct_quad(unsigned path, int depth) {
    return (int)(((path >> depth) & 1u) | (((path >> (16 + depth)) & 1u) << 1));
}

// Exclusive scan of n <= kOctNodeCap ints in place (2 per thread); returns the total.
__device__ inline int block_scan_array(int* a, int n, int* scratch) {
    const int i0 = 2 * threadIdx.x, i1 = i0 + 1;
    const int v0 = i0 < n ? a[i0] : 0, v1 = i1 < n ? a[i1] : 0;
    int total;
    const int e = block_excl_scan(v0 + v1, scratch, &total);
    if (i0 < n) a[i0] = e;
    if (i1 < n) a[i1] = e + v0;
    __syncthreads();
    return total;
}

__device__ inline void bitonic_sort(unsigned long long* k, int n) {  // n power of two
    for (int size = 2; size <= n; size <<= 1)
        for (int j = size >> 1; j > 0; j >>= 1) {
            for (int i = threadIdx.x; i < n; i += blockDim.x) {
                const int ixj = i ^ j;
                if (ixj > i) {
                    const bool asc = (i & size) == 0;
                    const unsigned long long a = k[i], c = k[ixj];
                    if ((a > c) == asc) { k[i] = c; k[ixj] = a; }
                }
            }
            __syncthreads();
        }
}

// Bitonic sort of n <= blockDim.x keys, one per thread (v), ascending by thread index: stages
// with a partner in the same wave exchange through lane shuffles, the others through LDS (lds,
// >= blockDim.x entries) with block barriers; every thread of the block takes part.
__device__ inline unsigned long long bitonic_sort_block(unsigned long long v, int n, unsigned long long* lds) {
    const int i = threadIdx.x;
    for (int size = 2; size <= n; size <<= 1)
        for (int j = size >> 1; j > 0; j >>= 1) {
            unsigned long long other;
            if (j >= 64) {
                lds[i] = v;
                __syncthreads();
                other = lds[i ^ j];
                __syncthreads();
            } else {
                other = __shfl_xor(v, j, 64);
            }
            const bool lower = (i & j) == 0, asc = (i & size) == 0;
            v = (lower == asc) ? (v < other ? v : other) : (v < other ? other : v);
        }
    return v;
}

__device__ __forceinline__ void octree_body(OctShared& S, int level, int b, const LevelGeom* __restrict__ levels,
                                            int nlevels, const uint2* __restrict__ cand,
                                            const int* __restrict__ level_count, const int* __restrict__ regbase,
                                            uint32_t* __restrict__ node_of, int keys_cap,
                                                         uint2* __restrict__ oct_out, int out_cap,
                                                         int* __restrict__ oct_count) {
    const int tid = threadIdx.x;
    const LevelGeom g = levels[level];
    const uint2* CK = cand + (long long)b * keys_cap;                 // {key, order tag}, regions
    uint32_t* NO = node_of + (long long)b * keys_cap + g.key_base;     // node | depth << 16

    OCT_STAMP(0, __builtin_amdgcn_s_memtime());
    // ---- the level's candidates (k_fast's dense array, in cell-completion order): thread t
    // holds keys t R .. t R + R - 1 in registers (R = kOctRegKeys; a cell's keys are contiguous,
    // so a thread's increments mostly hit one counter); keys from kOctThreads R on stay in CK
    // with their node in NO.  Nothing below depends on the keys' order except through the tags.
    // key k lives in region j with rpre[j] <= k < rpre[j + 1], at rbase[j] + k - rpre[j]
    if (tid < 64) {
        const int cnt = tid < kFastRegions ? level_count[(b * nlevels + level) * kFastRegions + tid] : 0;
        const int incl = wave_incl_scan(cnt);
        if (tid < kFastRegions) {
            S.rpre[tid + 1] = incl;
            S.rbase[tid] = regbase[level * kFastRegions + tid];
        }
        if (tid == 0) S.rpre[0] = 0;
    }
    // per-axis path tables (x: its own root's extent, y: the level height), in the LDS of the
    // careful-mode sort keys, built while the counts above are in flight
    unsigned short* xpath = reinterpret_cast<unsigned short*>(S.skey);
    unsigned short* ypath = xpath + 4096;
    const int wx = min(g.width, 4095), hy = min(g.height, 4095);
    for (int v = tid; v <= wx + 1 + hy; v += blockDim.x) {
        if (v <= wx) {
            const int n = oct_root((uint32_t)v, g);
            xpath[v] = (unsigned short)oct_axis(v, (int)(g.hX * (float)n), (int)(g.hX * (float)(n + 1)));
        } else {
            const int y = v - wx - 1;
            ypath[y] = (unsigned short)oct_axis(y, 0, g.height);
        }
    }
    for (int i = tid; i < g.nIni; i += blockDim.x) S.cnt[0][i] = 0;  // root counts (init below)
    __syncthreads();
    const int nkeys = min(S.rpre[kFastRegions], g.key_cap);
    auto key_slot = [&](int k, int& j) {  // j: a region at or before k's (walks forward)
        while (j < kFastRegions - 1 && S.rpre[j + 1] <= k) j++;
        return S.rbase[j] + (k - S.rpre[j]);
    };
    int j0 = 0;  // region of the thread's first key: the largest j with rpre[j] <= k
    {
        const int k0 = tid * kOctRegKeys;
        int lo = 0, hi = kFastRegions - 1;
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (S.rpre[mid] <= k0) lo = mid;
            else hi = mid - 1;
        }
        j0 = lo;
    }
    uint32_t kreg[kOctRegKeys];
    int nreg[kOctRegKeys];
    {
        int j = j0;
#pragma unroll
        for (int r = 0; r < kOctRegKeys; r++) {
            const int k = tid * kOctRegKeys + r;
            uint2 kv = make_uint2(0u, 0u);
            if (k < nkeys) kv = CK[key_slot(k, j)];
            kreg[r] = kv.x;
            S.tagl[k] = kv.y;
            nreg[r] = 0;
        }
    }
    // f(k, key, node&) for every key, in increasing k per thread: the register-resident
    // ones, then the global spill
    auto for_keys = [&](auto&& f) {
#pragma unroll
        for (int r = 0; r < kOctRegKeys; r++) {
            const int k = tid * kOctRegKeys + r;
            if (k < nkeys) f(k, kreg[r], nreg[r]);
        }
        for (int k = tid + kOctThreads * kOctRegKeys; k < nkeys; k += kOctThreads) {
            int no = (int)NO[k], j = 0;
            f(k, CK[key_slot(k, j)].x, no);
            NO[k] = (uint32_t)no;
        }
    };

    // path bits of the register keys (tables built above)
    unsigned preg[kOctRegKeys];
    {
#pragma unroll
        for (int r = 0; r < kOctRegKeys; r++)
            preg[r] = xpath[min((int)(kreg[r] & 0xFFF), wx)] | (unsigned)ypath[min((int)((kreg[r] >> 12) & 0xFFF), hy)] << 16;
        __syncthreads();
    }
    OCT_STAMP(1, __builtin_amdgcn_s_memtime());
    OCT_STAMP(62, nkeys);
    // ---- initial nodes (:543-579): counts per root (zeroed before the first barrier)
    const int nIni = g.nIni;
    int cur = 0;
    {
        int run = -1, rc = 0;  // consecutive keys of a thread share a node: one atomic per run
        for_keys([&](int, uint32_t key, int& no) {
            const int n = oct_root(key, g);
            no = n;
            if (n != run) {
                if (rc) atomicAdd(&S.cnt[cur][run], rc);
                run = n;
                rc = 0;
            }
            rc++;
        });
        if (rc) atomicAdd(&S.cnt[cur][run], rc);
    }
    __syncthreads();
    // drop empty initial nodes (:581-593): a ballot scan in wave 0 (nIni <= 64), else block scans
    int L;
    if (nIni <= 64) {
        if (tid < 64) {
            const int c = tid < nIni ? S.cnt[cur][tid] : 0;
            const unsigned long long m = __ballot(c > 0);
            const int ni = c > 0 ? __popcll(m & ((1ull << tid) - 1)) : -1;
            if (tid < nIni) {
                S.remap[tid][0] = S.remap[tid][1] = S.remap[tid][2] = S.remap[tid][3] = (short)ni;
                if (ni >= 0) S.cnt[cur ^ 1][ni] = c;
            }
            if (tid == 0) S.misc[4] = __popcll(m);
        }
        __syncthreads();
        L = S.misc[4];
    } else {
        for (int i = tid; i < nIni; i += blockDim.x) S.tmp[i] = S.cnt[cur][i] > 0;
        __syncthreads();
        L = block_scan_array(S.tmp, nIni, S.scratch);
        for (int i = tid; i < nIni; i += blockDim.x) {
            const short ni = S.cnt[cur][i] > 0 ? (short)S.tmp[i] : (short)-1;
            S.remap[i][0] = S.remap[i][1] = S.remap[i][2] = S.remap[i][3] = ni;
            if (ni >= 0) S.cnt[cur ^ 1][ni] = S.cnt[cur][i];
        }
        __syncthreads();
    }
    cur ^= 1;

    const int N = g.nfeat;
    bool careful = false, finish = false;
    OCT_STAMP(2, __builtin_amdgcn_s_memtime());
    int iters = 0;
    for (int iter = 0; iter < 256 && !finish; iter++) {
        iters++;
        const int prv = cur ^ 1;
        for (int i = tid; i < L; i += blockDim.x) {
            S.ccnt[i][0] = S.ccnt[i][1] = S.ccnt[i][2] = S.ccnt[i][3] = 0;
        }
        if (tid == 0) {
            S.misc[2 + (iter & 1)] = 0;  // read at the end of pass iter - 2
            S.misc[0] = 0;               // careful mode: candidate count, size >= 64 flag
            S.misc[6] = 0;
        }
        __syncthreads();
        OCT_SUB(iter, 0);
        // keys: apply the previous pass's remap (an entry with bit 14 set means the node was
        // divided: the key moved one level down), then histogram the key's quadrant in its new
        // node.  Nodes with one key get counts too; only nodes with >= 2 keys read them.
        {
            int tgt[kOctRegKeys];
#pragma unroll
            for (int r = 0; r < kOctRegKeys; r++) tgt[r] = S.remap[nreg[r] & 0xFFFF][oct_quad(preg[r], nreg[r] >> 16)];
            OCT_SUB(iter, 6);
#pragma unroll
            for (int r = 0; r < kOctRegKeys; r++) {
                const bool v = tid * kOctRegKeys + r < nkeys;  // absent keys stay on node 0
                const int e = tgt[r], node = e & 0x3FFF, dep = (nreg[r] >> 16) + ((e >> 14) & 1);
                nreg[r] = v ? node | dep << 16 : 0;
                tgt[r] = v ? 4 * node + oct_quad(preg[r], dep) : -1;
            }
            int run = -1, rc = 0;
#pragma unroll
            for (int r = 0; r < kOctRegKeys; r++) {
                if (tgt[r] != run) {
                    if (rc && run >= 0) atomicAdd(&S.ccnt[0][0] + run, rc);
                    run = tgt[r];
                    rc = 0;
                }
                rc++;
            }
            if (rc && run >= 0) atomicAdd(&S.ccnt[0][0] + run, rc);
            OCT_SUB(iter, 7);
            // spilled keys
            for (int k = tid + kOctThreads * kOctRegKeys; k < nkeys; k += kOctThreads) {
                int j = 0;
                const unsigned path = oct_path(CK[key_slot(k, j)].x, g);
                const int no = (int)NO[k];
                const int e = S.remap[no & 0xFFFF][oct_quad(path, no >> 16)];
                const int node = e & 0x3FFF, dep = (no >> 16) + ((e >> 14) & 1);
                NO[k] = (uint32_t)(node | dep << 16);
                atomicAdd(&S.ccnt[node][oct_quad(path, dep)], 1);
            }
            OCT_SUB(iter, 8);
        }
        __syncthreads();
        OCT_SUB(iter, 1);
        // which nodes divide, and in which push order
        int ncand = 0, kdiv = 0;
        if (careful) {
            // vSizeAndPointerToNode sorted by (size, creation); divided largest first (:681-733).
            // Only the nodes with >= 2 keys can divide, and their sizes are small integers: a
            // counting sort gives every such node its rank directly -- the nodes with a larger
            // size, plus the earlier nodes of its own size (per chunk of 64 nodes from the ballots
            // of the size's six bit planes, then a prefix over the chunks).  A size of 64 or more
            // takes round 5's path: a bitonic sort of the whole list, wave 0 walking the result.
            static_assert(2 * kOctThreads >= kOctNodeCap, "two nodes per thread");
            int* Wh = S.tmp;      // [32 chunks][64 sizes]: counts, then their prefix over chunks
            int* Sgt = S.newpos;  // [64]: candidates of a larger size (newpos is written after the sort)
            // a size of 64 or more anywhere takes round 5's bitonic path (misc[0], misc[6] were
            // reset at the top of the pass)
            {
                bool big = false;
                for (int i = tid; i < 32 * 64; i += blockDim.x) {
                    Wh[i] = 0;
                    big |= i < L && S.cnt[cur][i] >= 64;
                }
                if (__ballot(big) && (tid & 63) == 0) S.misc[6] = 1;
            }
            __syncthreads();
            if (!S.misc[6]) {
                int val[2], rnk[2];
#pragma unroll
                for (int h = 0; h < 2; h++) {
                    const int i = tid + h * kOctThreads, q = i >> 6;
                    const int c = i < L ? S.cnt[cur][i] : 0;
                    const int v = c >= 2 ? c : -1;
                    // the chunk's lanes of the same size: the six bit planes of the size, combined
                    unsigned long long same = __ballot(v >= 0);
                    if (same && (tid & 63) == 0) atomicAdd(&S.misc[0], __popcll(same));
#pragma unroll
                    for (int bit = 0; bit < 6; bit++) {
                        const unsigned long long pl = __ballot((v >> bit) & 1);
                        same &= ((v >> bit) & 1) ? pl : ~pl;
                    }
                    const int rw = lanes_below(same);
                    if (v >= 0 && rw == 0) Wh[q * 64 + v] = __popcll(same);  // the size's first lane
                    val[h] = v;
                    rnk[h] = rw;
                }
                for (int i = tid; i < L; i += blockDim.x) S.dflag[i] = 0;
                __syncthreads();
                ncand = S.misc[0];
                if (tid < 64) {  // lane = size: prefix over the chunks, then the larger sizes' total
                    int run = 0;
                    for (int q0 = 0; q0 < 32; q0 += 8) {  // 8 loads in flight (the VGPR budget)
                        int t[8];
#pragma unroll
                        for (int q = 0; q < 8; q++) t[q] = Wh[(q0 + q) * 64 + tid];
#pragma unroll
                        for (int q = 0; q < 8; q++) {
                            Wh[(q0 + q) * 64 + tid] = run;
                            run += t[q];
                        }
                    }
                    const int rv = __shfl(run, 63 - tid);  // total of size 63 - lane
                    const int incl = wave_incl_scan(rv);
                    Sgt[63 - tid] = incl - rv;
                }
                __syncthreads();
#pragma unroll
                for (int h = 0; h < 2; h++) {
                    const int i = tid + h * kOctThreads, v = val[h];
                    if (v >= 0)
                        S.skey[Sgt[v] + Wh[(i >> 6) * 64 + v] + rnk[h]] =
                            ((unsigned long long)(0xFFFFFFFFu - (unsigned)S.cnt[cur][i]) << 32) | (unsigned)i;
                }
                __syncthreads();
                // kdiv = 1 + the first r whose division brings the list to N (L + sum_{r' <= r}
                // (m_r' - 1) >= N, m the node's non-empty children), then the divided nodes' push bases
                // (prefix of m in sorted order): one block scan of m - 1 over the sorted candidates,
                // two per thread (the prefix of m is that of m - 1 plus r); the first r to reach N is
                // the only one whose exclusive prefix is still short of it, so one thread writes kdiv
                {
                    auto m_of = [&](int n) {
                        return (S.ccnt[n][0] > 0) + (S.ccnt[n][1] > 0) + (S.ccnt[n][2] > 0) + (S.ccnt[n][3] > 0);
                    };
                    if (tid == 0) S.misc[5] = ncand;  // no r reaches N: every candidate divides
                    const int r0 = 2 * tid, r1 = r0 + 1;
                    const int n0 = r0 < ncand ? (int)(S.skey[r0] & 0xFFFFFFFFu) : 0;
                    const int n1 = r1 < ncand ? (int)(S.skey[r1] & 0xFFFFFFFFu) : 0;
                    const int d0 = r0 < ncand ? m_of(n0) - 1 : 0, d1 = r1 < ncand ? m_of(n1) - 1 : 0;
                    int tot;
                    const int e0 = block_excl_scan(d0 + d1, S.scratch, &tot);  // its barriers publish misc[5]
                    if (r0 < ncand && (r0 == 0 || L + e0 < N) && L + e0 + d0 >= N) S.misc[5] = r0 + 1;
                    if (r1 < ncand && L + e0 + d0 < N && L + e0 + d0 + d1 >= N) S.misc[5] = r1 + 1;
                    __syncthreads();
                    const int kd = S.misc[5];
                    if (r0 < kd) {
                        S.dflag[n0] = 1;
                        S.newpos[n0] = e0 + r0;
                    }
                    if (r1 < kd) {
                        S.dflag[n1] = 1;
                        S.newpos[n1] = e0 + d0 + r1;
                    }
                    kdiv = kd;
                }
            } else {
                int np2 = 2;
                while (np2 < L) np2 <<= 1;
                if (np2 <= kOctThreads) {
                    const bool c2 = tid < L && S.cnt[cur][tid] >= 2;
                    const unsigned long long key =
                        c2 ? ((unsigned long long)(0xFFFFFFFFu - (unsigned)S.cnt[cur][tid]) << 32) | (unsigned)tid : ~0ull;
                    const int nw = __popcll(__ballot(c2));
                    if ((tid & 63) == 0 && nw) atomicAdd(&S.misc[0], nw);
                    const unsigned long long sorted = bitonic_sort_block(key, np2, S.skey);
                    __syncthreads();
                    if (tid < np2) S.skey[tid] = sorted;
                    for (int i = tid; i < L; i += blockDim.x) S.dflag[i] = 0;
                    ncand = S.misc[0];
                    __syncthreads();
                } else {
                    for (int i = tid; i < np2; i += blockDim.x) {
                        unsigned long long key = ~0ull;
                        if (i < L && S.cnt[cur][i] >= 2)
                            key = ((unsigned long long)(0xFFFFFFFFu - (unsigned)S.cnt[cur][i]) << 32) | (unsigned)i;
                        S.skey[i] = key;
                    }
                    for (int i = tid; i < L; i += blockDim.x) {
                        if (S.cnt[cur][i] >= 2) atomicAdd(&S.misc[0], 1);
                        S.dflag[i] = 0;
                    }
                    bitonic_sort(S.skey, np2);
                    ncand = S.misc[0];
                }
                // wave 0 walks the sorted candidates in chunks of 64 with wave scans: kdiv = 1 + the
                // first r whose division brings the list to N (L + sum_{r' <= r} (m_r' - 1) >= N),
                // then the divided nodes' push bases (prefix of m in sorted order)
                if (tid < 64) {
                    auto m_of = [&](int n) {
                        return (S.ccnt[n][0] > 0) + (S.ccnt[n][1] > 0) + (S.ccnt[n][2] > 0) + (S.ccnt[n][3] > 0);
                    };
                    int run = 0, kd = ncand;
                    for (int r0 = 0; r0 < ncand; r0 += 64) {
                        const int r = r0 + tid;
                        const int m = r < ncand ? m_of((int)(S.skey[r] & 0xFFFFFFFFu)) : 1;
                        const int incl = wave_incl_scan(m - 1);
                        const unsigned long long hit = __ballot(r < ncand && L + run + incl >= N);
                        if (hit) {
                            kd = r0 + __ffsll((long long)hit);
                            break;
                        }
                        run += __builtin_amdgcn_readlane(incl, 63);
                    }
                    int push = 0;
                    for (int r0 = 0; r0 < kd; r0 += 64) {
                        const int r = r0 + tid;
                        const int n = r < kd ? (int)(S.skey[r] & 0xFFFFFFFFu) : 0;
                        const int m = r < kd ? m_of(n) : 0;
                        const int incl = wave_incl_scan(m);
                        if (r < kd) {
                            S.dflag[n] = 1;
                            S.newpos[n] = push + incl - m;
                        }
                        push += __builtin_amdgcn_readlane(incl, 63);
                    }
                    kdiv = kd;
                }
            }
            __syncthreads();
        }
        OCT_SUB(iter, 2);
        // one packed scan over the list, two nodes per thread: child pushes of the dividing nodes
        // (outside the careful mode their push base in list order) | survivors << 16; the
        // children with more than one key go to one atomic per wave
        const int i0 = 2 * tid, i1 = i0 + 1;
        int ne = 0;
        auto classify = [&](int i) -> int {
            if (i >= L) return 0;
            const bool d = careful ? S.dflag[i] != 0 : S.cnt[cur][i] >= 2;
            if (!careful) S.dflag[i] = d;
            if (!d) return 1 << 16;
            int m = 0;
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const int c = S.ccnt[i][q];
                m += c > 0;
                ne += c > 1;
            }
            return m;
        };
        const int v0 = classify(i0), v1 = classify(i1);
        ne = wave_sum_i32(ne);
        if ((tid & 63) == 0 && ne) atomicAdd(&S.misc[2 + (iter & 1)], ne);
        int total;
        const int e0 = block_excl_scan(v0 + v1, S.scratch, &total);
        const int P = total & 0xFFFF, nsurv = total >> 16;
        const int nToExpand = S.misc[2 + (iter & 1)];  // every atomic precedes the scan's barriers
        OCT_SUB(iter, 3);
        auto rewrite = [&](int i, int e) {
            if (i >= L) return;
            if (S.dflag[i]) {
                int p = careful ? S.newpos[i] : (e & 0xFFFF);
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    const int c = S.ccnt[i][q];
                    if (c > 0) {
                        const int ni = P - 1 - p++;
                        if (ni < kOctNodeCap) S.cnt[prv][ni] = c;  // bound proven in DESIGN.md; guard LDS anyway
                        S.remap[i][q] = (short)(min(ni, kOctNodeCap - 1) | 0x4000);
                    } else {
                        S.remap[i][q] = -1;
                    }
                }
            } else {
                const int ni = min(P + (e >> 16), kOctNodeCap - 1);
                S.cnt[prv][ni] = S.cnt[cur][i];
                S.remap[i][0] = S.remap[i][1] = S.remap[i][2] = S.remap[i][3] = (short)ni;
            }
        };
        rewrite(i0, e0);
        rewrite(i1, e0 + v0);
        __syncthreads();  // the next pass clears ccnt and reads cnt[prv] / remap
        OCT_SUB(iter, 4);
        const int newL = min(P + nsurv, kOctNodeCap);
        // the remap just written maps list `cur` to list `prv`; keys apply it next pass
        cur = prv;
        if (newL >= N || newL == L) finish = true;
        else if (!careful && newL + nToExpand * 3 > N) careful = true;
        L = newL;
        (void)ncand;
        (void)kdiv;
        if (iter < 50) OCT_STAMP(3 + iter, __builtin_amdgcn_s_memtime() | ((unsigned long long)careful << 63));
    }
    OCT_STAMP(61, iters);
    (void)iters;
    OCT_STAMP(60, L);

    // ---- keep the max-response key per node, first in original order on ties (:744-760):
    // one 64-bit max per node over score << 56 | (2^24 - 1 - tag) << 24 | (y << 12 | x)
    unsigned long long* best = reinterpret_cast<unsigned long long*>(&S.ccnt[0][0]);  // 2 per row
    for (int i = tid; i < L; i += blockDim.x) best[2 * i] = 0;
    __syncthreads();
    {
        int fn[kOctRegKeys];  // final node of each register key, all reads first
#pragma unroll
        for (int r = 0; r < kOctRegKeys; r++) {
            const bool v = tid * kOctRegKeys + r < nkeys;
            const int e = S.remap[nreg[r] & 0xFFFF][oct_quad(preg[r], nreg[r] >> 16)];
            fn[r] = v ? (e & 0x3FFF) : -1;
        }
        uint32_t treg[kOctRegKeys];  // order tags
#pragma unroll
        for (int r = 0; r < kOctRegKeys; r++) treg[r] = S.tagl[tid * kOctRegKeys + r];
#pragma unroll
        for (int r = 0; r < kOctRegKeys; r++) {
            const uint32_t key = kreg[r];
            if (fn[r] >= 0)
                atomicMax(&best[2 * fn[r]], ((unsigned long long)(key >> 24) << 56) |
                                                ((unsigned long long)(0xFFFFFFu - treg[r]) << 24) | (key & 0xFFFFFFu));
        }
        for (int k = tid + kOctThreads * kOctRegKeys; k < nkeys; k += kOctThreads) {
            int j = 0;
            const uint2 kv = CK[key_slot(k, j)];
            const uint32_t key = kv.x, tg = kv.y;
            const int no = (int)NO[k];
            const int n = S.remap[no & 0xFFFF][oct_quad(oct_path(key, g), no >> 16)] & 0x3FFF;
            atomicMax(&best[2 * n], ((unsigned long long)(key >> 24) << 56) |
                                        ((unsigned long long)(0xFFFFFFu - tg) << 24) | (key & 0xFFFFFFu));
        }
    }
    __syncthreads();
    const int minB = kEdge - 3;
    uint2* out = oct_out + (long long)b * out_cap + g.out_base;
    for (int i = tid; i < L && i < g.out_cap; i += blockDim.x) {
        const unsigned long long v = best[2 * i];
        const uint32_t key = (uint32_t)(v & 0xFFFFFFu);
        out[i] = make_uint2(((key & 0xFFF) + minB) | ((((key >> 12) & 0xFFF) + minB) << 16), (uint32_t)(v >> 56));
    }
    if (tid == 0) oct_count[b * nlevels + level] = min(L, g.out_cap);
    OCT_STAMP(59, __builtin_amdgcn_s_memtime());
}

// ------------------------------------------------------------------------------ blur
// GaussianBlur(7x7, sigma 2, REFLECT_101) of every level (src/ORBextractor.cc:1085-1086), pinned
// as P3: separable integer taps {18,34,49,55,49,34,18}, float column pass for x < blur_xv,
// integer tail.  The reflect-101 border of the padded pyramid supplies the taps outside the
// image.  One 128x32 output tile per workgroup: 16-B loads of the padded rows (interior column
// x0 - 3 sits at a 16-B boundary) staged in LDS, row sums in registers, 4x4 outputs per thread stored as dwords
// into the interior-only blurred layout.
constexpr int kBlurInH = kBlurTH + 6, kBlurChunks = (kBlurTW + 6 + 15) / 16;  // 38 rows x 9 x 16 B
constexpr int kBlurInS = 16 * kBlurChunks;                                     // 144
struct BlurShared {
    uint4 in4[kBlurInH * kBlurChunks];
};
// One tile on a 256-thread slice of the workgroup (tid = 0..255).  The slice's block-wide barrier
// is reached by every slice, also one without a tile (valid = false).  The input rows are staged
// in LDS; thread (column group cg, row group rg) then forms the integer row sums of its 4 columns
// for the 10 input rows its 4 output rows read (3 aligned dword reads per row) in registers and
// the column pass from them: no row-sum array round-trips LDS.
__device__ __forceinline__ void blur_tile(BlurShared& B, const uint8_t* __restrict__ pyr, uint8_t* __restrict__ blur,
                                          long long pimg, long long bimg, const LevelGeom* __restrict__ levels,
                                          int2 t, int b, int tid, bool valid) {
    uint4* in4 = B.in4;
    const LevelGeom g = levels[valid ? t.x : 0];
    const int x0 = t.y & 0xFFFF, y0 = t.y >> 16;
    const uint8_t* lvl = pyr + b * pimg + g.off + kEdge - 3 + x0;  // column x0 - 3 of padded row 0
    for (int i = tid; valid && i < kBlurInH * kBlurChunks; i += 256) {
        const int r = i / kBlurChunks, ch = i - r * kBlurChunks;
        const int yy = min(y0 - 3 + r, g.H + 2);  // rows past H + 2 feed only discarded outputs
        in4[i] = *reinterpret_cast<const uint4*>(lvl + (long long)(kEdge + yy) * g.stride + 16 * ch);
    }
    __syncthreads();
    if (!valid) return;
    const int cq = 4 * (tid & 31), rb = 4 * (tid >> 5);  // 4 columns x 4 output rows per thread
    if (y0 + rb >= g.H) return;
    const unsigned* in = reinterpret_cast<const unsigned*>(in4);
    // row pass: the 7 taps of column cq + c are bytes c .. c + 6 of (w0, w1, w2): two v_dot4
    // over byte-aligned dwords (v_alignbyte), weights (18, 34, 49, 55) and (49, 34, 18, 0)
    constexpr unsigned kW0 = 18u | 34u << 8 | 49u << 16 | 55u << 24, kW1 = 49u | 34u << 8 | 18u << 16;
    unsigned rs[10][4];  // row sums of input rows rb .. rb + 9 (output row rb + rr reads rb + rr .. + 6)
#pragma unroll
    for (int r = 0; r < 10; r++) {
        const unsigned* q = in + (rb + r) * (kBlurInS / 4) + cq / 4;  // bytes = input columns cq - 3 ..
        const unsigned w0 = q[0], w1 = q[1], w2 = q[2];
#pragma unroll
        for (int c = 0; c < 4; c++) {
            const unsigned a = c ? __builtin_amdgcn_alignbyte(w1, w0, c) : w0;
            const unsigned h = c ? __builtin_amdgcn_alignbyte(w2, w1, c) : w1;
            rs[r][c] = __builtin_amdgcn_udot4(h, kW1, __builtin_amdgcn_udot4(a, kW0, 0u, false), false);
        }
    }
    // column pass: S = 55 c3 + 49 p1 + 34 p2 + 18 p3 < 2^24 unless the result saturates, so the
    // reference's float path (SymmColumnVec_32s8u: S / 65536 in float, one rounding per operation,
    // then rint) is exact: round-half-even of S / 65536; the scalar tail rounds half up
    uint8_t* dst = blur + b * bimg + g.boff;
#pragma unroll
    for (int rr = 0; rr < 4; rr++) {
        const int y = y0 + rb + rr;
        if (y >= g.H) break;
        unsigned packedv = 0;
#pragma unroll
        for (int cc = 0; cc < 4; cc++) {
            const int x = x0 + cq + cc;
            const unsigned S = __umul24(rs[rr + 3][cc], 55u) + __umul24(rs[rr + 2][cc] + rs[rr + 4][cc], 49u) +
                               __umul24(rs[rr + 1][cc] + rs[rr + 5][cc], 34u) + __umul24(rs[rr][cc] + rs[rr + 6][cc], 18u);
            const unsigned up = x < g.blur_xv ? (S >> 16) & 1u : 1u;
            const unsigned v = min((S + 0x7FFFu + up) >> 16, 255u);
            packedv |= v << (8 * cc);
        }
        if (x0 + cq < g.bstride)
            *reinterpret_cast<unsigned*>(dst + (long long)y * g.bstride + x0 + cq) = packedv;
    }
}

// DistributeOctTree and GaussianBlur in one launch, on a 1-D grid: the first blocks run one
// (image, level) octree each and are dispatched first; the blocks after them blur four
// 128x32 tiles each on the CUs the octrees leave idle.  A level-0 octree is the launch's longest
// workgroup (its candidates are the most), so the blur hides behind it instead of following it.
// Both only read the pyramid; the blur slices reuse the octree's LDS.
static_assert(sizeof(OctShared) >= 4 * sizeof(BlurShared), "blur slices overlay the octree LDS");
constexpr int kFuseBlurMaxOctrees = 64;  // octree workgroups up to which the blur rides along
__global__ __launch_bounds__(kOctThreads) void k_octree(const LevelGeom* __restrict__ levels, int nlevels,
                                                         const uint2* __restrict__ cand,
                                                         const int* __restrict__ level_count,
                                                         const int* __restrict__ regbase,
                                                         uint32_t* __restrict__ node_of,
                                                         int keys_cap, uint2* __restrict__ oct_out, int out_cap,
                                                         int* __restrict__ oct_count, const uint8_t* __restrict__ pyr,
                                                         uint8_t* __restrict__ blur, long long pimg, long long bimg,
                                                         const int2* __restrict__ btiles, int nbtiles, int batch) {
    __shared__ OctShared S;
    // workgroup i goes to XCD i % 8, and workgroups are dispatched in index order.  A large batch
    // takes two rounds of one octree workgroup per CU, so the octrees are numbered longest first
    // (level-major from the top level down: alone, every level takes 47-52 us and the top one
    // 84 us at config 5), each level spread over all XCDs (image 8 s + i % 8 for slot s).
    const int b8 = (batch + 7) / 8, noct = nlevels * 8 * b8;
    if ((int)blockIdx.x < noct) {
        const int q = blockIdx.x >> 3, lv = nlevels - 1 - q / b8, img = 8 * (q % b8) + (blockIdx.x & 7);
#ifdef ORBMI_OCT_ONLY_LEVEL  // timing experiment (tools: A/B builds): run the octrees of one level only
        if ((ORBMI_OCT_ONLY_LEVEL >= 0) != (lv == (ORBMI_OCT_ONLY_LEVEL < 0 ? -1 - ORBMI_OCT_ONLY_LEVEL : ORBMI_OCT_ONLY_LEVEL)))
            return;
#endif
        if (img < batch)
            octree_body(S, lv, img, levels, nlevels, cand, level_count, regbase, node_of, keys_cap, oct_out, out_cap,
                        oct_count);
        return;
    }
    const int slice = threadIdx.x >> 8, ti = ((int)blockIdx.x - noct) * 4 + slice;  // over (image, tile)
    const bool valid = ti < nbtiles * batch;
    const int img = valid ? ti / nbtiles : 0, tile = valid ? ti - img * nbtiles : 0;
    BlurShared* B = reinterpret_cast<BlurShared*>(&S) + slice;
    blur_tile(*B, pyr, blur, pimg, bimg, levels, btiles[tile], img, threadIdx.x & 255, valid);
}

// GaussianBlur alone: one 128x32 tile per 256-thread workgroup.
__global__ __launch_bounds__(256) void k_blur(const uint8_t* __restrict__ pyr, uint8_t* __restrict__ blur,
                                              long long pimg, long long bimg, const LevelGeom* __restrict__ levels,
                                              const int2* __restrict__ tiles, int nimg) {
    __shared__ BlurShared B;
    int tile, b;
    if (!xcd_image_map(nimg, tile, b)) return;
    blur_tile(B, pyr, blur, pimg, bimg, levels, tiles[tile], b, threadIdx.x, true);
}

// ------------------------------------------------------------------------------ describe
constexpr int kBR = 18;                 // rotated rBRIEF samples lie within 18 px (pattern radius 18.4)
constexpr int kBW = 2 * kBR + 1;        // blurred window 37 x 37
constexpr int kBD = (kBW + 3 + 3) / 4;  // dwords per window row (any start alignment): 10
constexpr int kUR = 15;                 // IC_Angle patch radius (HALF_PATCH_SIZE)
constexpr int kUW = 2 * kUR + 1;        // unblurred window 31 x 31
constexpr int kUD = (kUW + 3 + 3) / 4;  // 9

__device__ inline float fast_atan2_deg(float y, float x) {
    // cv::fastAtan2 (OpenCV 3.x mathfuncs): polynomial in degrees
    const float p1 = 0.9997878412794807f * (float)(180 / M_PI);
    const float p3 = -0.3258083974640975f * (float)(180 / M_PI);
    const float p5 = 0.1555786518463281f * (float)(180 / M_PI);
    const float p7 = -0.04432655554792128f * (float)(180 / M_PI);
    const float ax = fabsf(x), ay = fabsf(y);
    float a, c, c2;
    if (ax >= ay) {
        c = ay / (ax + (float)2.220446049250313e-16);
        c2 = c * c;
        a = (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
    } else {
        c = ax / (ay + (float)2.220446049250313e-16);
        c2 = c * c;
        a = 90.f - (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
    }
    if (x < 0) a = 180.f - a;
    if (y < 0) a = 360.f - a;
    return a;
}

// One wave per keypoint: the 31x31 unblurred patch (IC_Angle) and the 37x37 blurred window
// (k_blur output) go to the wave's LDS as aligned dwords covering each window row (the row's
// first byte sits at a per-window offset 0..3), then 4 ballots give the 256 bits.
__global__ __launch_bounds__(256) void k_describe(const uint8_t* __restrict__ pyr, const uint8_t* __restrict__ blur,
                                                  long long pimg, long long bimg, const LevelGeom* __restrict__ levels,
                                                  int nlevels,
                                                  const uint2* __restrict__ oct_out, int oct_cap,
                                                  const int* __restrict__ oct_count,
                                                  orbmi_keypoint* __restrict__ kps,
                                                  uint8_t* __restrict__ desc, int* __restrict__ counts,
                                                  int capacity) {
    __shared__ unsigned winb[4][kBW * kBD];
    __shared__ unsigned winu[4][kUW * kUD];
    const int b = blockIdx.y, wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int j = blockIdx.x * 4 + wid;
    const int* lc = oct_count + b * nlevels;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        int t = 0;
        for (int l = 0; l < nlevels; l++) t += lc[l];
        counts[b] = t;
    }
    int level = -1;
    for (int l = 0; l < nlevels; l++)
        if (j >= levels[l].out_base && j < levels[l].out_base + levels[l].out_cap) level = l;
    // every wave owns its own LDS windows, so only wave-level ordering is needed below
    if (level < 0) return;
    const LevelGeom g = levels[level];
    const int idx = j - g.out_base;
    if (idx >= lc[level]) return;
    int off = 0;
    for (int l = 0; l < level; l++) off += lc[l];
    const uint2 o = oct_out[(long long)b * oct_cap + j];
    const int x = o.x & 0xFFFF, y = o.x >> 16;
    unsigned* wb = winb[wid];
    unsigned* wu = winu[wid];
    const long long base = b * pimg + g.off + (long long)(kEdge + y) * g.stride + kEdge + x;
    const long long sb = b * bimg + g.boff + (long long)(y - kBR) * g.bstride + x - kBR;  // byte address
    const long long su = base - (long long)kUR * g.stride - kUR;
    const int ob = (int)(sb & 3), ou = (int)(su & 3);  // first window byte inside the first dword
    {
        const unsigned* b4 = reinterpret_cast<const unsigned*>(blur + (sb - ob));
        const unsigned* u4 = reinterpret_cast<const unsigned*>(pyr + (su - ou));
        const int bs4 = g.bstride >> 2, us4 = g.stride >> 2;
        unsigned vb[(kBW * kBD + 63) / 64], vu[(kUW * kUD + 63) / 64];
#pragma unroll
        for (int k = 0; k < (kBW * kBD + 63) / 64; k++) {  // all loads first, then the LDS stores
            const int i = lane + 64 * k, r = i / kBD, c = i - r * kBD;
            vb[k] = i < kBW * kBD ? b4[(long long)r * bs4 + c] : 0u;
        }
#pragma unroll
        for (int k = 0; k < (kUW * kUD + 63) / 64; k++) {
            const int i = lane + 64 * k, r = i / kUD, c = i - r * kUD;
            vu[k] = i < kUW * kUD ? u4[(long long)r * us4 + c] : 0u;
        }
#pragma unroll
        for (int k = 0; k < (kBW * kBD + 63) / 64; k++)
            if (lane + 64 * k < kBW * kBD) wb[lane + 64 * k] = vb[k];
#pragma unroll
        for (int k = 0; k < (kUW * kUD + 63) / 64; k++)
            if (lane + 64 * k < kUW * kUD) wu[lane + 64 * k] = vu[k];
    }
    const uint8_t* wbb = reinterpret_cast<const uint8_t*>(wb) + ob;  // wbb[r * 4 kBD + c] = window (r, c)
    const uint8_t* wub = reinterpret_cast<const uint8_t*>(wu) + ou;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): window stores landed in LDS
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // IC_Angle on the unblurred level (src/ORBextractor.cc:77-104)
    int m01 = 0, m10 = 0;
    for (int i = lane; i < c_ncircle; i += 64) {
        const int u = c_circle[i][0], v = c_circle[i][1];
        const int val = wub[(kUR + v) * 4 * kUD + kUR + u];
        m10 += u * val;
        m01 += v * val;
    }
    m10 = wave_sum_i32(m10);
    m01 = wave_sum_i32(m01);
    const float angle = fast_atan2_deg((float)m01, (float)m10);
    // computeOrbDescriptor on the blurred level (src/ORBextractor.cc:108-147), pinned P6
    const float ang = angle * (float)(3.14159265358979323846 / 180.0);
    double sd, cd;  // (float)cos((double)ang), (float)sin((double)ang), checked exhaustively (trig_f64.h)
    orbmi_sincos_f64((double)ang, &sd, &cd);
    const float ca = (float)cd, sa = (float)sd;
    unsigned long long masks[4];
#pragma unroll
    for (int kk = 0; kk < 4; kk++) {
        const int t = kk * 64 + lane;
        const float px0 = c_pattern[t][0], py0 = c_pattern[t][1];
        const float px1 = c_pattern[t][2], py1 = c_pattern[t][3];
        const int c0 = cv_round_f(px0 * ca - py0 * sa), r0 = cv_round_f(px0 * sa + py0 * ca);
        const int c1 = cv_round_f(px1 * ca - py1 * sa), r1 = cv_round_f(px1 * sa + py1 * ca);
        const int v0 = wbb[(kBR + r0) * 4 * kBD + kBR + c0];
        const int v1 = wbb[(kBR + r1) * 4 * kBD + kBR + c1];
        masks[kk] = __ballot(v0 < v1);
    }
    if (off + idx < capacity) {
        const long long oi = (long long)b * capacity + off + idx;
        if (lane < 4) reinterpret_cast<unsigned long long*>(desc + oi * 32)[lane] = masks[lane == 0 ? 0 : lane == 1 ? 1 : lane == 2 ? 2 : 3];
        if (lane == 0) {
            orbmi_keypoint kp;
            kp.x = level == 0 ? (float)x : (float)x * g.scale;
            kp.y = level == 0 ? (float)y : (float)y * g.scale;
            kp.size = g.size;
            kp.angle = angle;
            kp.response = (float)o.y;
            kp.octave = level;
            kp.class_id = -1;
            kps[oi] = kp;
        }
    }
}

// Four keypoints per wave, one DPP row (16 lanes) each: the per-keypoint scalar work -- the
// moment sums' reduction, fastAtan2, the fp64 sincos, the output record -- runs once for four
// keypoints, and the lane-parallel parts keep their instruction count per keypoint:
//   * IC_Angle (:77-104) straight from the unblurred level: the 749 patch pixels as <= 213
//     aligned dwords (c_ictab[ou], per 4-B phase ou of the patch's first byte), each dword
//     weighted by three v_dot4_u32_u8: (u + 16), (v + 16) and 1 on the circle's bytes, 0 off it,
//     so m_10 = S_u - 16 S_1 and m_01 = S_v - 16 S_1 (integers: exact);
//   * the blurred 37 x 37 window staged in LDS with 8-B loads (rows of kBP bytes);
//   * rBRIEF (:108-147, pinned P6): lane l takes the pairs 16 l + k, k = 15 .. 0; the rotation
//     in packed fp32 (the same products and sums, rounded as the reference's float expression),
//     cvRound by adding 1.5 * 2^23 (round-half-even to an integer in the low mantissa bits, which
//     index LDS directly), and the bits shifted into one 16-bit word per lane: lane l holds bytes
//     2l, 2l+1 of its keypoint's descriptor.
// A workgroup takes kDescKpWG consecutive slots per step and strides over the image's slots.
constexpr int kDescGroups = 4;                        // keypoints per wave
constexpr int kDescWaves = 4;                         // waves per workgroup
constexpr int kDescKpWG = kDescGroups * kDescWaves;  // slots per workgroup step
constexpr int kDescTargetWG = 1536;                   // workgroups per launch (3 per CU, 2 rounds)
#ifndef ORBMI_DESC_BP
#define ORBMI_DESC_BP 48
#endif
constexpr int kBP = ORBMI_DESC_BP;                    // LDS pitch: 37 bytes from any 8-B phase need 44
constexpr int kBQ = kBP / 8;                          // 8-B loads per window row
constexpr int kIcItems = 224;                         // IC dwords per phase (<= 213 used): 14 per lane
struct DescLevel { long long off, boff; int stride, bstride, out_base; float scale, size; };
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
__constant__ float4 c_pattern_f[256];     // (x0, x1, y0, y1) of pair t = 16 l + k at 16 k + l
__constant__ uint4 c_ictab[4][kIcItems];  // {u + 16 weights, circle mask, window row, 4 * dword}

__device__ inline unsigned row16_sum(unsigned v) {  // sum over the lane's DPP row, in every lane
    using namespace wave_detail;
    v += (unsigned)dpp<0xB1>((int)v);
    v += (unsigned)dpp<0x4E>((int)v);
    v += (unsigned)dpp<0x141>((int)v);
    return v + (unsigned)dpp<0x128>((int)v);
}

__global__ __launch_bounds__(64 * kDescWaves) void k_describe4(const uint8_t* __restrict__ pyr,
                                                               const uint8_t* __restrict__ blur, long long pimg,
                                                               long long bimg, const LevelGeom* __restrict__ levels,
                                                               int nlevels, const uint2* __restrict__ oct_out,
                                                               int oct_cap, const int* __restrict__ oct_count,
                                                               orbmi_keypoint* __restrict__ kps,
                                                               uint8_t* __restrict__ desc, int* __restrict__ counts,
                                                               int capacity, int out_cap, int nimg) {
    __shared__ float4 spat[256];
    __shared__ uint4 sic[4][kIcItems];
    __shared__ DescLevel slv[kMaxLevels];
    __shared__ int spre[kMaxLevels], scnt[kMaxLevels];
    __shared__ __attribute__((aligned(16))) uint8_t swin[kDescKpWG][kBW * kBP];
    // the gx workgroups of an image share an XCD (xcd_image_map)
    int w, b;
    if (!xcd_image_map(nimg, w, b)) return;
    const int gx = (int)gridDim.x / (nimg >= 8 ? 8 * ((nimg + 7) / 8) : nimg);
    const int tid = threadIdx.x, wid = tid >> 6, lane = tid & 63, grp = lane >> 4, l = lane & 15;
    spat[tid] = c_pattern_f[tid];
    for (int i = tid; i < 4 * kIcItems; i += 64 * kDescWaves) (&sic[0][0])[i] = (&c_ictab[0][0])[i];
    const int* lc = oct_count + b * nlevels;
    if (tid < nlevels) {
        const LevelGeom& g = levels[tid];
        slv[tid] = DescLevel{g.off, g.boff, g.stride, g.bstride, g.out_base, g.scale, g.size};
        int pre = 0;
        for (int q = 0; q < tid; q++) pre += lc[q];
        spre[tid] = pre;
        scnt[tid] = lc[tid];
        if (w == 0 && tid == nlevels - 1) counts[b] = pre + lc[tid];
    }
    __syncthreads();
    uint8_t* W = swin[wid * kDescGroups + grp];
    const int nchunks = (out_cap + kDescKpWG - 1) / kDescKpWG;
    for (int ch = w; ch < nchunks; ch += gx) {
        const int j = ch * kDescKpWG + wid * kDescGroups + grp;
        int level = -1;
        for (int q = 0; q < nlevels; q++)
            if (j >= levels[q].out_base && j < levels[q].out_base + levels[q].out_cap) level = q;
        const int lv = level < 0 ? 0 : level;
        const DescLevel G = slv[lv];
        const int idx = j - G.out_base;
        const bool valid = level >= 0 && idx < scnt[lv];
        if (__ballot(valid) == 0) continue;  // wave-uniform
        int x = 0, y = 0;
        unsigned resp = 0;
        if (valid) {
            const uint2 o = oct_out[(long long)b * oct_cap + j];
            x = o.x & 0xFFFF;
            y = o.x >> 16;
            resp = o.y;
        }
        // the blurred window, rows of kBP bytes from its 8-B aligned start: lanes 0..11 of the
        // group load 8-B column q = l % 6 of rows 2k + l / 6 (byte offsets inside the image's planes)
        const uint8_t* bimgp = blur + (long long)b * bimg;
        const uint8_t* pimgp = pyr + (long long)b * pimg;
        const unsigned sb = (unsigned)G.boff + (unsigned)((y - kBR) * G.bstride + x - kBR);
        const int ob = (int)(sb & 7);
        if (valid && l < 2 * kBQ) {
            const int par = l >= kBQ ? 1 : 0, q = l - par * kBQ;
            const unsigned go = sb - ob + 8 * q + par * G.bstride;
            uint8_t* wd = W + 8 * q + kBP * par;
            constexpr int kPairs = (kBW + 1) / 2;
            uint2 v[kPairs];
#pragma unroll
            for (int k = 0; k < kPairs; k++)
                v[k] = (2 * k + par < kBW) ? *reinterpret_cast<const uint2*>(bimgp + go + 2 * k * G.bstride)
                                           : make_uint2(0u, 0u);
#pragma unroll
            for (int k = 0; k < kPairs; k++)
                if (2 * k + par < kBW) *reinterpret_cast<uint2*>(wd + 2 * kBP * k) = v[k];
        }
        // IC_Angle: the patch's dwords from the padded level, weighted by c_ictab[ou]
        unsigned s_u = 0, s_v = 0, s_1 = 0;
        if (valid) {
            const unsigned su = (unsigned)G.off + (unsigned)((kEdge + y - kUR) * G.stride + kEdge + x - kUR);
            const int ou = (int)(su & 3);
            const unsigned sua = su - ou;
            unsigned val[kIcItems / 16];
            uint4 it[kIcItems / 16];
#pragma unroll
            for (int k = 0; k < kIcItems / 16; k++) {
                it[k] = sic[ou][l + 16 * k];
                val[k] = *reinterpret_cast<const unsigned*>(pimgp + (sua + __umul24(it[k].z, G.stride) + it[k].w));
            }
#pragma unroll
            for (int k = 0; k < kIcItems / 16; k++) {
                s_u = __builtin_amdgcn_udot4(val[k], it[k].x, s_u, false);
                s_1 = __builtin_amdgcn_udot4(val[k], it[k].y, s_1, false);
                // (v + 16) on the circle bytes: a packed 16-bit multiply (__umul24 would drop the top byte)
                const u16x2 wv = __builtin_bit_cast(u16x2, it[k].y) * (unsigned short)(it[k].z + 1);
                s_v = __builtin_amdgcn_udot4(val[k], __builtin_bit_cast(unsigned, wv), s_v, false);
            }
        }
        s_u = row16_sum(s_u);
        s_v = row16_sum(s_v);
        s_1 = row16_sum(s_1);
        const int m10 = (int)s_u - 16 * (int)s_1, m01 = (int)s_v - 16 * (int)s_1;
        const float angle = fast_atan2_deg((float)m01, (float)m10);
        const float ang = angle * (float)(3.14159265358979323846 / 180.0);
        double sd, cd;
        orbmi_sincos_f64((double)ang, &sd, &cd);
        const float ca = valid ? (float)cd : 1.f, sa = valid ? (float)sd : 0.f;
        // the window stores of this wave visible to its reads
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_s_waitcnt(0xc07f);
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        // rBRIEF: window (kBR + r, kBR + c) at W[ob + (kBR + r) kBP + kBR + c]; with r, c as the low
        // bits of (value + 1.5 * 2^23) the constant part folds into kadd (uint32 wrap-around)
        const float kMagic = 12582912.0f;
        const unsigned kadd = (unsigned)(ob + kBR * kBP + kBR) - 0x400000u * (unsigned)kBP - 0x4B400000u;
        unsigned word = 0;
#pragma unroll
        for (int k = 15; k >= 0; k--) {
            const float4 P = spat[16 * k + l];  // pair 16 l + k (k-major: one iteration reads 256 contiguous bytes)
            const f32x2 px = {P.x, P.y}, py = {P.z, P.w};
            const f32x2 cx = (px * ca - py * sa) + kMagic;
            const f32x2 ry = (px * sa + py * ca) + kMagic;
            const unsigned i0 = __umul24(__float_as_uint(ry.x), (unsigned)kBP) + __float_as_uint(cx.x) + kadd;
            const unsigned i1 = __umul24(__float_as_uint(ry.y), (unsigned)kBP) + __float_as_uint(cx.y) + kadd;
            word = 2 * word + (W[i0] < W[i1] ? 1u : 0u);
        }
        if (valid && spre[lv] + idx < capacity) {
            const long long oi = (long long)b * capacity + spre[lv] + idx;
            reinterpret_cast<unsigned short*>(desc + oi * 32)[l] = (unsigned short)word;
            if (l == 0) {
                orbmi_keypoint kp;
                kp.x = level == 0 ? (float)x : (float)x * G.scale;
                kp.y = level == 0 ? (float)y : (float)y * G.scale;
                kp.size = G.size;
                kp.angle = angle;
                kp.response = (float)resp;
                kp.octave = level;
                kp.class_id = -1;
                kps[oi] = kp;
            }
        }
    }
}

// ------------------------------------------------------------------------------ host
static int cv_round_host(float v) { return (int)lrintf(v); }

int Extractor::init(int dev, int nf, float sf, int nl, int ini, int mn) {
    if (nf < 0 || nl < 1 || nl > kMaxLevels || !(sf > 1.0f)) return ORBMI_E_ARG;
    device = dev; nfeatures = nf; scale_factor = sf; nlevels = nl; ini_th = ini; min_th = mn;
    ORBMI_HIP(hipSetDevice(device));
    ORBMI_HIP(orbmi::stream_create(&stream, "EXTRACTOR"));
    // ORBextractor::ORBextractor  src/ORBextractor.cc:410-470 (same float/double steps)
    scale.assign(nl, 1.f); sigma2.assign(nl, 1.f); inv_scale.resize(nl); inv_sigma2.resize(nl);
    const double sfd = (double)sf;
    for (int i = 1; i < nl; i++) {
        scale[i] = (float)((double)scale[i - 1] * sfd);
        sigma2[i] = scale[i] * scale[i];
    }
    for (int i = 0; i < nl; i++) { inv_scale[i] = 1.0f / scale[i]; inv_sigma2[i] = 1.0f / sigma2[i]; }
    nfeat.resize(nl);
    const float factor = (float)(1.0f / sfd);
    float ndes = (float)nf * (1 - factor) / (1 - (float)pow((double)factor, (double)nl));
    int sum = 0;
    for (int l = 0; l < nl - 1; l++) { nfeat[l] = cv_round_host(ndes); sum += nfeat[l]; ndes *= factor; }
    nfeat[nl - 1] = std::max(nf - sum, 0);
    umax.assign(kHalfPatch + 1, 0);
    const int vmax = cv_floor_f(kHalfPatch * sqrtf(2.f) / 2 + 1);
    const int vmin = (int)ceilf(kHalfPatch * sqrtf(2.f) / 2);
    const double hp2 = kHalfPatch * kHalfPatch;
    for (int v = 0; v <= vmax; ++v) umax[v] = (int)lrint(sqrt(hp2 - v * v));
    for (int v = kHalfPatch, v0 = 0; v >= vmin; --v) {
        while (umax[v0] == umax[v0 + 1]) ++v0;
        umax[v] = v0;
        ++v0;
    }
    // constant tables: pattern and the IC_Angle circle
    signed char circ[768][2];
    int nc = 0;
    for (int v = -kHalfPatch; v <= kHalfPatch; v++) {
        const int d = umax[v < 0 ? -v : v];
        for (int u = -d; u <= d; u++) { circ[nc][0] = (signed char)u; circ[nc][1] = (signed char)v; nc++; }
    }
    ORBMI_HIP(hipMemcpyToSymbol(HIP_SYMBOL(c_pattern), ORBMI_PATTERN, sizeof(ORBMI_PATTERN)));
    ORBMI_HIP(hipMemcpyToSymbol(HIP_SYMBOL(c_circle), circ, sizeof(circ)));
    ORBMI_HIP(hipMemcpyToSymbol(HIP_SYMBOL(c_ncircle), &nc, sizeof(int)));
    {   // k_describe4's tables: the pattern as (x0, x1, y0, y1) floats, and per 4-B phase ou of
        // the IC patch's first byte the dwords covering each circle row with their byte weights
        float4 pf[256];
        for (int t = 0; t < 256; t++)  // pair t = 16 l + k at 16 k + l
            pf[16 * (t & 15) + (t >> 4)] =
                make_float4(ORBMI_PATTERN[t][0], ORBMI_PATTERN[t][2], ORBMI_PATTERN[t][1], ORBMI_PATTERN[t][3]);
        ORBMI_HIP(hipMemcpyToSymbol(HIP_SYMBOL(c_pattern_f), pf, sizeof(pf)));
        static uint4 ic[4][kIcItems];
        memset(ic, 0, sizeof(ic));
        for (int ou = 0; ou < 4; ou++) {
            int n = 0;
            for (int v = -kHalfPatch; v <= kHalfPatch; v++) {
                const int d = umax[v < 0 ? -v : v], r = v + kHalfPatch;
                for (int dd = (ou + kHalfPatch - d) / 4; dd <= (ou + kHalfPatch + d) / 4; dd++) {
                    if (n >= kIcItems) return ORBMI_E_ARG;
                    unsigned wa = 0, wm = 0;
                    for (int p = 0; p < 4; p++) {
                        const int u = 4 * dd + p - ou - kHalfPatch;
                        if (u >= -d && u <= d) { wa |= (unsigned)(u + 16) << (8 * p); wm |= 1u << (8 * p); }
                    }
                    ic[ou][n++] = make_uint4(wa, wm, (unsigned)r, (unsigned)(4 * dd));
                }
            }
        }
        ORBMI_HIP(hipMemcpyToSymbol(HIP_SYMBOL(c_ictab), ic, sizeof(ic)));
        const char* e = getenv("ORBMI_DESC");
        describe_wave = e && !strcmp(e, "wave");
        e = getenv("ORBMI_FAST");
        fast_v1 = e && !strcmp(e, "v1");
        fast_split = e && !strcmp(e, "split");
        e = getenv("ORBMI_FAST_EARLY");
        fast_early = e && !strcmp(e, "1");
        e = getenv("ORBMI_BLUR");
        blur_mode = !e ? -1 : !strcmp(e, "side") ? 0 : !strcmp(e, "fused") ? 1 : !strcmp(e, "serial") ? 2
                  : !strcmp(e, "afterfast") ? 3 : !strcmp(e, "perlevel") ? 4 : -1;
    }
    std::vector<float> tab(scale);
    tab.insert(tab.end(), inv_scale.begin(), inv_scale.end());
    ORBMI_HIP(hipMalloc((void**)&d_scale_tab, tab.size() * sizeof(float)));
    ORBMI_HIP(hipMemcpy(d_scale_tab, tab.data(), tab.size() * sizeof(float), hipMemcpyHostToDevice));
    return ORBMI_OK;
}

static int resize_simd_end(int width) {
    int x = 0;
    while (x <= width - 16) x += 16;
    while (x < width - 4) x += 4;
    return x;
}

template <class T>
static int dev_alloc(T** p, size_t n) {
    if (*p) { (void)hipFree(*p); *p = nullptr; }
    if (n == 0) n = 1;
    ORBMI_HIP(hipMalloc((void**)p, n * sizeof(T)));
    return ORBMI_OK;
}

int Extractor::set_geometry(int r, int c) {
    if (r == rows && c == cols && !levels.empty()) return ORBMI_OK;
    ORBMI_HIP(hipSetDevice(device));
    levels.assign(nlevels, LevelGeom{});
    cells.clear();
    std::vector<XTab> xt;
    std::vector<YTab> yt;
    long long off = 0, boff = 0;
    int slot = 0, key = 0, outb = 0;
    regbase.assign((size_t)nlevels * kFastRegions, 0);
    for (int l = 0; l < nlevels; l++) {
        LevelGeom& g = levels[l];
        g.W = cv_round_host((float)c * inv_scale[l]);
        g.H = cv_round_host((float)r * inv_scale[l]);
        const int minB = kEdge - 3, maxBX = g.W - kEdge + 3, maxBY = g.H - kEdge + 3;
        if (maxBX - minB < 30 || maxBY - minB < 30) return ORBMI_E_UNSUPPORTED;
        g.stride = (g.W + 2 * kEdge + 63) & ~63;
        g.ph = g.H + 2 * kEdge;
        g.off = off;
        off += (long long)g.stride * g.ph;
        g.bstride = (g.W + 127) & ~127;
        g.boff = boff;
        boff += (long long)g.bstride * g.H;
        g.scale = scale[l];
        g.size = (float)(int)(kPatch * scale[l]);
        g.blur_xv = (g.W / 4) * 4;
        g.resize_xv = resize_simd_end(g.W);
        g.nfeat = nfeat[l];
        // cells (src/ORBextractor.cc:778-829)
        const float width = (float)(maxBX - minB), height = (float)(maxBY - minB);
        const int nCols = (int)(width / 30.f), nRows = (int)(height / 30.f);
        const int wCell = (int)ceilf(width / nCols), hCell = (int)ceilf(height / nRows);
        if (wCell + 6 > kTile || hCell + 6 > kTile) return ORBMI_E_UNSUPPORTED;  // list entries y << 6 | x
        const int cap = ((wCell + 1) / 2) * ((hCell + 1) / 2);
        g.cell_begin = (int)cells.size();
        g.key_base = key;
        for (int i = 0; i < nRows; i++) {
            const float iniY = (float)(minB + i * hCell);
            float maxY = iniY + hCell + 6;
            const bool skipY = iniY >= maxBY - 3;
            if (maxY > maxBY) maxY = (float)maxBY;
            for (int j = 0; j < nCols; j++) {
                const float iniX = (float)(minB + j * wCell);
                float maxX = iniX + wCell + 6;
                CellGeom cg{};
                cg.level = l;
                if (!skipY && !(iniX >= maxBX - 6)) {
                    if (maxX > maxBX) maxX = (float)maxBX;
                    cg.x0 = (short)(int)iniX; cg.y0 = (short)(int)iniY;
                    cg.w = (short)((int)maxX - (int)iniX); cg.h = (short)((int)maxY - (int)iniY);
                    cg.sx = (short)(j * wCell); cg.sy = (short)(i * hCell);
                    slot += cap;
                    key += cap;
                }
                cg.roi_off = g.off + (long long)(kEdge + cg.y0) * g.stride + kEdge + cg.x0;
                cg.stride = g.stride;
                cg.lcell = (int)cells.size() - g.cell_begin;
                cells.push_back(cg);
            }
        }
        g.cell_end = (int)cells.size();
        g.key_cap = key - g.key_base;
        {   // candidate regions: region j holds the cells k % R == j of the level, sized for their caps
            int rcap[kFastRegions] = {0}, base = g.key_base;
            for (int k = 0; k < g.cell_end - g.cell_begin; k++)
                if (cells[g.cell_begin + k].w) rcap[k % kFastRegions] += cap;
            for (int j = 0; j < kFastRegions; j++) {
                regbase[l * kFastRegions + j] = base;
                base += rcap[j];
            }
            for (int k = 0; k < g.cell_end - g.cell_begin; k++)
                cells[g.cell_begin + k].slot_base = regbase[l * kFastRegions + k % kFastRegions];
        }
        // order tags: cell index within the level (14 bits) << 10 | rank in the cell (< 1024)
        if (g.key_cap > (1 << 20) || g.cell_end - g.cell_begin >= (1 << 14) || cap >= 1024) return ORBMI_E_UNSUPPORTED;
        g.width = maxBX - minB;
        g.height = maxBY - minB;
        g.nIni = (int)roundf((float)g.width / (float)g.height);
        if (g.nIni < 1) return ORBMI_E_UNSUPPORTED;  // reference indexes an empty vector here
        g.hX = (float)g.width / g.nIni;
        g.out_cap = std::max(g.nfeat + 3, 4 * g.nIni) + 1;
        if (g.out_cap > kOctNodeCap || 4 * g.nIni > kOctNodeCap) return ORBMI_E_UNSUPPORTED;
        g.out_base = outb;
        outb += g.out_cap;
        // resize tables (level >= 1): cv::resize INTER_LINEAR 8U coefficients
        if (l > 0) {
            const LevelGeom& s = levels[l - 1];
            g.xtab_off = (int)xt.size();
            g.ytab_off = (int)yt.size();
            const double scale_x = 1. / ((double)g.W / s.W), scale_y = 1. / ((double)g.H / s.H);
            int xmax = g.W;
            std::vector<int> sxs(g.W);
            std::vector<float> fxs(g.W);
            for (int dx = 0; dx < g.W; dx++) {
                float fx = (float)((dx + 0.5) * scale_x - 0.5);
                int sx = cv_floor_f(fx);
                fx -= sx;
                if (sx < 0) { fx = 0; sx = 0; }
                if (sx + 1 >= s.W) { xmax = std::min(xmax, dx); if (sx >= s.W - 1) { fx = 0; sx = s.W - 1; } }
                sxs[dx] = sx; fxs[dx] = fx;
            }
            for (int dx = 0; dx < g.W; dx++) {
                XTab e;
                const int a0 = std::min(std::max(cv_round_host((1.f - fxs[dx]) * 2048), -32768), 32767);
                const int a1 = std::min(std::max(cv_round_host(fxs[dx] * 2048), -32768), 32767);
                e.sx0 = (short)sxs[dx];
                if (dx < xmax) { e.sx1 = (short)(sxs[dx] + 1); e.a0 = (short)a0; e.a1 = (short)a1; }
                else { e.sx1 = (short)sxs[dx]; e.a0 = 2048; e.a1 = 0; }
                xt.push_back(e);
            }
            for (int dy = 0; dy < g.H; dy++) {
                float fy = (float)((dy + 0.5) * scale_y - 0.5);
                int sy = cv_floor_f(fy);
                fy -= sy;
                YTab e;
                e.b0 = (short)std::min(std::max(cv_round_host((1.f - fy) * 2048), -32768), 32767);
                e.b1 = (short)std::min(std::max(cv_round_host(fy * 2048), -32768), 32767);
                e.y0 = (short)std::min(std::max(sy, 0), s.H - 1);
                e.y1 = (short)std::min(std::max(sy + 1, 0), s.H - 1);
                yt.push_back(e);
            }
        }
    }
    // pyramid tiles: own rectangles split every level KX x KY ways; need rectangles from the top
    // level down (need_{l-1} = own_{l-1} U the taps of need_l); level 0's need rectangle is the
    // own one grown by the largest halo (hx, hy) of any tile.  The grid grows until a tile's LDS
    // (parameter block, level-0 rectangle, two need rectangles) fits in 48 KB.  Each tile's
    // parameter block: kPyrLevelWords words per level (own, need, W | H << 16, stride, offset,
    // resize_xv, word offsets of the x / y taps), then the taps of its need rectangles.
    {
        int KX = 16, KY = 8;
        for (;;) {
            std::vector<PyrTile> tl((size_t)KX * KY * nlevels);
            int maxarea = 0, hx = 0, hy = 0, words = 0;
            for (int ty = 0; ty < KY; ty++)
                for (int tx = 0; tx < KX; tx++) {
                    PyrTile* T = &tl[((size_t)ty * KX + tx) * nlevels];
                    for (int l = 0; l < nlevels; l++) {
                        const LevelGeom& g = levels[l];
                        T[l].own = PyrRect{(short)(g.W * tx / KX), (short)(g.W * (tx + 1) / KX), (short)(g.H * ty / KY),
                                           (short)(g.H * (ty + 1) / KY)};
                    }
                    T[nlevels - 1].need = T[nlevels - 1].own;
                    for (int l = nlevels - 1; l >= 1; l--) {
                        const LevelGeom& g = levels[l];
                        PyrRect n = T[l].need, o = T[l - 1].own, r = o;
                        if (n.x1 > n.x0 && n.y1 > n.y0) {
                            const XTab* X = xt.data() + g.xtab_off;
                            const YTab* Y = yt.data() + g.ytab_off;
                            r.x0 = std::min<short>(o.x0, X[n.x0].sx0);
                            r.x1 = std::max<short>(o.x1, (short)(X[n.x1 - 1].sx1 + 1));
                            r.y0 = std::min<short>(o.y0, Y[n.y0].y0);
                            r.y1 = std::max<short>(o.y1, (short)(Y[n.y1 - 1].y1 + 1));
                        }
                        T[l - 1].need = r;
                    }
                    int w = kPyrLevelWords * nlevels;
                    for (int l = 1; l < nlevels; l++) {
                        const PyrRect& n = T[l].need;
                        maxarea = std::max(maxarea, (n.x1 - n.x0) * (n.y1 - n.y0));
                        w += 2 * (n.x1 - n.x0) + 2 * (n.y1 - n.y0);
                    }
                    words = std::max(words, w);
                    hx = std::max(hx, std::max(T[0].own.x0 - T[0].need.x0, T[0].need.x1 - T[0].own.x1));
                    hy = std::max(hy, std::max(T[0].own.y0 - T[0].need.y0, T[0].need.y1 - T[0].own.y1));
                }
            int area0 = 0;
            for (int ty = 0; ty < KY; ty++)
                for (int tx = 0; tx < KX; tx++) {
                    const int x0 = std::max(levels[0].W * tx / KX - hx, 0), x1 = std::min(levels[0].W * (tx + 1) / KX + hx, levels[0].W);
                    const int y0 = std::max(levels[0].H * ty / KY - hy, 0), y1 = std::min(levels[0].H * (ty + 1) / KY + hy, levels[0].H);
                    area0 = std::max(area0, (x1 - x0) * (y1 - y0));
                }
            const int half = (maxarea + 15) & ~15, a0 = (area0 + 15) & ~15;
            const int lds = 4 * words + a0 + 2 * half;
            if (lds <= 48 * 1024 || KX * KY >= 4096) {
                if (lds > 64 * 1024) return ORBMI_E_UNSUPPORTED;
                pyr_blob.assign((size_t)KX * KY * words, 0u);
                for (int t = 0; t < KX * KY; t++) {
                    const PyrTile* T = &tl[(size_t)t * nlevels];
                    uint32_t* B = &pyr_blob[(size_t)t * words];
                    auto pk = [](int lo, int hi) { return (uint32_t)(uint16_t)lo | (uint32_t)(uint16_t)hi << 16; };
                    int at = kPyrLevelWords * nlevels;
                    for (int l = 0; l < nlevels; l++) {
                        const LevelGeom& g = levels[l];
                        uint32_t* G = B + l * kPyrLevelWords;
                        G[0] = pk(T[l].own.x0, T[l].own.x1);
                        G[1] = pk(T[l].own.y0, T[l].own.y1);
                        G[2] = pk(T[l].need.x0, T[l].need.x1);
                        G[3] = pk(T[l].need.y0, T[l].need.y1);
                        G[4] = pk(g.W, g.H);
                        G[5] = (uint32_t)g.stride;
                        G[6] = (uint32_t)g.off;
                        G[7] = (uint32_t)g.resize_xv;
                        if (l == 0) continue;
                        const XTab* X = xt.data() + g.xtab_off;
                        const YTab* Y = yt.data() + g.ytab_off;
                        G[8] = (uint32_t)at;
                        for (int x = T[l].need.x0; x < T[l].need.x1; x++) {
                            B[at++] = pk(X[x].sx0, X[x].sx1);
                            B[at++] = pk(X[x].a0, X[x].a1);
                        }
                        G[9] = (uint32_t)at;
                        for (int y = T[l].need.y0; y < T[l].need.y1; y++) {
                            B[at++] = pk(Y[y].y0, Y[y].y1);
                            B[at++] = pk(Y[y].b0, Y[y].b1);
                        }
                    }
                }
                pyr_kx = KX;
                pyr_ky = KY;
                pyr_hx = hx;
                pyr_hy = hy;
                pyr_blob_words = words;
                pyr_lds_half = half;
                pyr_lds0 = a0;
                break;
            }
            if (KX <= 2 * KY) KX *= 2;
            else KY *= 2;
        }
    }
    pimg = off;
    fast_maxw = 7; fast_maxh = 7;  // k_fast's LDS: the largest cell ROI of the geometry
    for (const CellGeom& cg : cells)
        if (cg.w) { fast_maxw = std::max(fast_maxw, (int)cg.w); fast_maxh = std::max(fast_maxh, (int)cg.h); }
    fast_wave_bytes = fast_lds_layout(fast_maxw, fast_maxh).wave_bytes;
    bimg = boff;
    btiles.clear();
    for (int l = 0; l < nlevels; l++)
        for (int y0 = 0; y0 < levels[l].H; y0 += kBlurTH)
            for (int x0 = 0; x0 < levels[l].W; x0 += kBlurTW) btiles.push_back(make_int2(l, x0 | (y0 << 16)));
    nbtiles = (int)btiles.size();
    btile_off.assign(nlevels + 1, 0);
    for (const int2& t : btiles) btile_off[t.x + 1]++;
    for (int l = 0; l < nlevels; l++) btile_off[l + 1] += btile_off[l];
    (void)slot;
    keys_cap = key;
    out_cap = outb;
    rows = r; cols = c;
    int rc;
    if ((rc = dev_alloc(&d_levels, levels.size()))) return rc;
    if ((rc = dev_alloc(&d_cells, cells.size()))) return rc;
    if ((rc = dev_alloc(&d_regbase, regbase.size()))) return rc;
    if ((rc = dev_alloc(&d_pyr_blob, pyr_blob.size()))) return rc;
    ORBMI_HIP(hipMemcpy(d_pyr_blob, pyr_blob.data(), pyr_blob.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
    ORBMI_HIP(hipMemcpy(d_regbase, regbase.data(), regbase.size() * sizeof(int), hipMemcpyHostToDevice));
    if ((rc = dev_alloc(&d_btiles, btiles.size()))) return rc;
    ORBMI_HIP(hipMemcpy(d_btiles, btiles.data(), btiles.size() * sizeof(int2), hipMemcpyHostToDevice));
    if ((rc = dev_alloc(&d_xtab, xt.size()))) return rc;
    if ((rc = dev_alloc(&d_ytab, yt.size()))) return rc;
    ORBMI_HIP(hipMemcpy(d_levels, levels.data(), levels.size() * sizeof(LevelGeom), hipMemcpyHostToDevice));
    ORBMI_HIP(hipMemcpy(d_cells, cells.data(), cells.size() * sizeof(CellGeom), hipMemcpyHostToDevice));
    if (!xt.empty()) ORBMI_HIP(hipMemcpy(d_xtab, xt.data(), xt.size() * sizeof(XTab), hipMemcpyHostToDevice));
    if (!yt.empty()) ORBMI_HIP(hipMemcpy(d_ytab, yt.data(), yt.size() * sizeof(YTab), hipMemcpyHostToDevice));
    bcap = 0;  // force re-reservation of per-image buffers
    return ORBMI_OK;
}

int Extractor::reserve(int batch, int capacity) {
    int rc;
    if (batch > bcap) {
        if ((rc = dev_alloc(&d_pyr, (size_t)batch * pimg))) return rc;
        if ((rc = dev_alloc(&d_blur, (size_t)batch * bimg))) return rc;
        if ((rc = dev_alloc(&d_level_count, (size_t)batch * nlevels * kFastRegions))) return rc;
        if ((rc = dev_alloc(&d_cand, (size_t)batch * keys_cap))) return rc;
        if ((rc = dev_alloc(&d_node_of, (size_t)batch * keys_cap))) return rc;
        if ((rc = dev_alloc(&d_oct, (size_t)batch * out_cap))) return rc;
        if ((rc = dev_alloc(&d_oct_count, (size_t)batch * nlevels))) return rc;
        if ((rc = dev_alloc(&d_counts, (size_t)batch))) return rc;
        bcap = batch;
        out_capacity = 0;  // internal outputs are sized per bcap: re-reserve below
    }
    if (capacity > out_capacity) {  // internal outputs (host API): bcap images x capacity
        if ((rc = dev_alloc(&d_kps, (size_t)bcap * capacity))) return rc;
        if ((rc = dev_alloc(&d_desc, (size_t)bcap * capacity * 32))) return rc;
        out_capacity = capacity;
    }
    return ORBMI_OK;
}

// The side stream and its events, created on first use: only the large batches that put the
// blur (or the early level-0 FAST) on a side stream need them, and an idle stream per extractor
// would otherwise count against the process's hardware queues (GPU_MAX_HW_QUEUES) for nothing.
int Extractor::ensure_side_stream() {
    if (bstream) return ORBMI_OK;
    ORBMI_HIP(orbmi::stream_create(&bstream, "EXTRACTOR"));
    ORBMI_HIP(hipEventCreateWithFlags(&ev_pyr, hipEventDisableTiming));
    ORBMI_HIP(hipEventCreateWithFlags(&ev_blur, hipEventDisableTiming));
    ORBMI_HIP(hipEventCreateWithFlags(&ev_l0, hipEventDisableTiming));
    ORBMI_HIP(hipEventCreateWithFlags(&ev_f0, hipEventDisableTiming));
    return ORBMI_OK;
}

int Extractor::run(const uint8_t* d_images, int batch, size_t step, size_t image_stride,
                   orbmi_keypoint* kps, uint8_t* desc, int* counts, int capacity) {
    ORBMI_HIP(hipSetDevice(device));
    const int ncells = (int)cells.size();
    // GaussianBlur needs only the pyramid.  Small batches (<= kFuseBlurMaxOctrees octrees): it rides
    // in the octree launch as extra workgroups on the CUs the octrees leave idle (a side stream's
    // event round trip costs more there: 7.8k vs 6.9k stereo frames/s).  Large batches: it runs on
    // a side stream (bstream) beside FAST and the octrees, and the describe waits for it (88.3k
    // vs 84.9k frames/s at config 5).  ORBMI_BLUR=side|fused|serial overrides.
    const int blur_mode = this->blur_mode >= 0 ? this->blur_mode : batch * nlevels <= kFuseBlurMaxOctrees ? 1 : 0;
    // ORBMI_FAST_EARLY=1: with the level-wise pyramid and the side stream, level 0's FAST runs on
    // the side stream as soon as level 0 is written, beside the resize chain of levels 1..7.  Off
    // by default: every kernel here is issue-bound, so the overlap only slowed the resize chain
    // (0.143 -> 0.222 ms) and config 5 stayed at 89k frames/s (profiles/r04/fast_early_ab.txt).
    const bool early = batch > kPyrTiledMaxBatch && blur_mode == 0 && !fast_v1 && fast_early &&
                       levels[0].cell_begin == 0 && nlevels > 1;
    if (blur_mode == 0 || blur_mode >= 3 || early) {
        const int rc = ensure_side_stream();
        if (rc) return rc;
    }
    const bool per_level = blur_mode == 4 && batch > kPyrTiledMaxBatch;
    if (per_level && (int)ev_lv.size() < nlevels) {
        for (int l = (int)ev_lv.size(); l < nlevels; l++) {
            hipEvent_t e = nullptr;
            ORBMI_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
            ev_lv.push_back(e);
        }
    }
    auto launch_fast = [&](int c0, int c1, hipStream_t s) {
        const dim3 grid((c1 - c0 + kFastCells - 1) / kFastCells, batch), block(64 * kFastCells);
        if (fast_v1)  // ORBMI_FAST=v1: per-lane bit assembly, runtime tile pitch (A/B)
            hipLaunchKernelGGL(k_fast, grid, block, kFastCells * fast_wave_bytes, s, d_pyr, pimg, d_levels, d_cells,
                               ncells, d_cand, keys_cap, d_level_count, nlevels, ini_th, min_th, fast_maxw, fast_maxh);
        else {
            const bool narrow = fast_maxw + 3 <= 48;
            const size_t lds = kFastCells * fast2_wave_bytes(narrow ? 48 : 80, fast_maxw, fast_maxh);
            auto* kf = fast_split ? (narrow ? k_fast2<48, false> : k_fast2<80, false>)
                                  : (narrow ? k_fast2<48, true> : k_fast2<80, true>);
            hipLaunchKernelGGL(kf, dim3(xcd_image_grid(grid.x, batch)), block, lds, s, d_pyr, pimg, d_cells, c0, c1, d_cand,
                               keys_cap, d_level_count, nlevels, ini_th, min_th, fast_maxw, fast_maxh, batch);
        }
    };
    if (batch > kPyrTiledMaxBatch) {
        for (int l = 0; l < nlevels; l++) {
            const LevelGeom& g = levels[l];
            dim3 grid((g.ph + kPyrBRows - 1) / kPyrBRows, 1, batch);
            hipEvent_t ev = prof_begin(l == 0 ? ORBMI_STAGE_PYR_LEVEL0 : ORBMI_STAGE_PYR_RESIZE);
            if (l == 0) {
                const int lrow = (g.W + 3 + 3 + 15) & ~15;  // an image row from its aligned start
                hipLaunchKernelGGL(k_pyr_level0, grid, dim3(kPyrBThreads), kPyrBRows * lrow, stream, d_images, step,
                                   image_stride, d_pyr, pimg, g, d_level_count, nlevels, lrow);
                if (early) {  // level 0's FAST beside the resize chain (it reads level 0 only)
                    ORBMI_HIP(hipEventRecord(ev_l0, stream));
                    ORBMI_HIP(hipStreamWaitEvent(bstream, ev_l0, 0));
                    hipEvent_t ef = prof_begin(ORBMI_STAGE_FAST, bstream);
                    launch_fast(levels[0].cell_begin, levels[0].cell_end, bstream);
                    prof_end(ORBMI_STAGE_FAST, ef, bstream);
                    ORBMI_HIP(hipEventRecord(ev_f0, bstream));
                }
            } else {
                const int lrow = levels[l - 1].stride;  // a padded source row (64-B multiple)
                hipLaunchKernelGGL(k_pyr_resize, grid, dim3(kPyrBThreads), 2 * kPyrBRows * lrow + 8 * g.W, stream, d_pyr, pimg,
                                   levels[l - 1], g, d_xtab + g.xtab_off, d_ytab + g.ytab_off, lrow);
            }
            prof_end(l == 0 ? ORBMI_STAGE_PYR_LEVEL0 : ORBMI_STAGE_PYR_RESIZE, ev);
            if (per_level) {  // ORBMI_BLUR=perlevel: level l's blur as soon as level l is written (A/B)
                const int n_l = btile_off[l + 1] - btile_off[l];
                ORBMI_HIP(hipEventRecord(ev_lv[l], stream));
                ORBMI_HIP(hipStreamWaitEvent(bstream, ev_lv[l], 0));
                if (n_l > 0)
                    hipLaunchKernelGGL(k_blur, dim3(xcd_image_grid(n_l, batch)), dim3(256), 0, bstream, d_pyr, d_blur, pimg,
                                       bimg, d_levels, d_btiles + btile_off[l], batch);
                if (l == nlevels - 1) ORBMI_HIP(hipEventRecord(ev_blur, bstream));
            }
        }
    } else {
        hipEvent_t ev = prof_begin(ORBMI_STAGE_PYR_LEVEL0);  // the whole pyramid
        hipLaunchKernelGGL(k_pyramid, dim3(pyr_kx * pyr_ky, 1, batch), dim3(kPyrThreads),
                           4 * pyr_blob_words + pyr_lds0 + 2 * pyr_lds_half, stream, d_images, step, image_stride, d_pyr,
                           pimg, d_pyr_blob, pyr_blob_words, nlevels, pyr_kx, pyr_ky, levels[0].W, levels[0].H, pyr_hx,
                           pyr_hy, d_level_count, pyr_lds0, pyr_lds_half);
        prof_end(ORBMI_STAGE_PYR_LEVEL0, ev);
    }
    auto side_blur = [&]() -> int {  // the blur on the side stream from this point of the stream
        ORBMI_HIP(hipEventRecord(ev_pyr, stream));
        ORBMI_HIP(hipStreamWaitEvent(bstream, ev_pyr, 0));
        hipEvent_t eb = prof_begin(ORBMI_STAGE_BLUR, bstream);
        hipLaunchKernelGGL(k_blur, dim3(xcd_image_grid(nbtiles, batch)), dim3(256), 0, bstream, d_pyr, d_blur, pimg, bimg,
                           d_levels, d_btiles, batch);
        prof_end(ORBMI_STAGE_BLUR, eb, bstream);
        ORBMI_HIP(hipEventRecord(ev_blur, bstream));
        return ORBMI_OK;
    };
    if (blur_mode == 0 || (blur_mode == 4 && !per_level)) {
        ORBMI_HIP(hipEventRecord(ev_pyr, stream));
        ORBMI_HIP(hipStreamWaitEvent(bstream, ev_pyr, 0));
        hipEvent_t eb = prof_begin(ORBMI_STAGE_BLUR, bstream);
        hipLaunchKernelGGL(k_blur, dim3(xcd_image_grid(nbtiles, batch)), dim3(256), 0, bstream, d_pyr, d_blur, pimg, bimg,
                           d_levels, d_btiles, batch);
        prof_end(ORBMI_STAGE_BLUR, eb, bstream);
        ORBMI_HIP(hipEventRecord(ev_blur, bstream));
    }
    hipEvent_t ev = prof_begin(ORBMI_STAGE_FAST);
    launch_fast(early ? levels[1].cell_begin : 0, ncells, stream);
    prof_end(ORBMI_STAGE_FAST, ev);
    if (blur_mode == 3) {  // ORBMI_BLUR=afterfast: beside the octrees only (A/B)
        const int rc = side_blur();
        if (rc) return rc;
    }
    if (early) ORBMI_HIP(hipStreamWaitEvent(stream, ev_f0, 0));
    ev = prof_begin(ORBMI_STAGE_OCTREE);
    const bool fused = blur_mode == 1;
    const int blur_blocks = fused ? (nbtiles * batch + 3) / 4 : 0;
    hipLaunchKernelGGL(k_octree, dim3(nlevels * 8 * ((batch + 7) / 8) + blur_blocks), dim3(kOctThreads), 0, stream,
                       d_levels, nlevels,
                       d_cand, d_level_count, d_regbase, d_node_of, keys_cap, d_oct, out_cap, d_oct_count, d_pyr, d_blur,
                       pimg, bimg, d_btiles, fused ? nbtiles : 0, batch);
    prof_end(ORBMI_STAGE_OCTREE, ev);
    if (blur_mode == 2) {
        ev = prof_begin(ORBMI_STAGE_BLUR);
        hipLaunchKernelGGL(k_blur, dim3(xcd_image_grid(nbtiles, batch)), dim3(256), 0, stream, d_pyr, d_blur, pimg, bimg,
                           d_levels, d_btiles, batch);
        prof_end(ORBMI_STAGE_BLUR, ev);
    }
    if (blur_mode == 0 || blur_mode >= 3) ORBMI_HIP(hipStreamWaitEvent(stream, ev_blur, 0));
    ev = prof_begin(ORBMI_STAGE_DESCRIBE);
    if (describe_wave)  // ORBMI_DESC=wave: one keypoint per wave (A/B)
        hipLaunchKernelGGL(k_describe, dim3((out_cap + 3) / 4, batch), dim3(256), 0, stream, d_pyr, d_blur, pimg, bimg,
                           d_levels, nlevels, d_oct, out_cap, d_oct_count, kps, desc, counts, capacity);
    else {
        const int nch = (out_cap + kDescKpWG - 1) / kDescKpWG;
        const int gx = std::max(1, std::min(nch, (kDescTargetWG + batch - 1) / batch));
        hipLaunchKernelGGL(k_describe4, dim3(xcd_image_grid(gx, batch)), dim3(64 * kDescWaves),
                           0, stream, d_pyr, d_blur,
                           pimg, bimg, d_levels, nlevels, d_oct, out_cap, d_oct_count, kps, desc, counts, capacity,
                           out_cap, batch);
    }
    prof_end(ORBMI_STAGE_DESCRIBE, ev);
    ORBMI_HIP(hipGetLastError());
    last_batch = batch;
    last_kps = kps; last_desc = desc; last_counts = counts; last_capacity = capacity;
    return ORBMI_OK;
}

hipEvent_t Extractor::prof_event() {
    hipEvent_t e = nullptr;
    if (!prof_pool.empty()) { e = prof_pool.back(); prof_pool.pop_back(); return e; }
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    return e;
}

hipEvent_t Extractor::prof_begin(int stage, hipStream_t s) {
    if (!(prof_mask >> stage & 1u)) return nullptr;
    hipEvent_t a = prof_event();
    if (a) (void)hipEventRecord(a, s ? s : stream);
    return a;
}

void Extractor::prof_end(int stage, hipEvent_t a, hipStream_t s) {
    if (!a) return;
    hipEvent_t b = prof_event();
    if (!b) return;
    (void)hipEventRecord(b, s ? s : stream);
    prof_pending.push_back(ProfPair{stage, a, b});
}

// ---- host images into HBM (orbmi_extract_batch_host) -------------------------------------------
// The image bytes are read straight from pinned host memory by a copy kernel on the handle's
// stream: the host never waits (hipMemcpyAsync from host memory measured as waiting for the
// stream's earlier work, which serialised the host with the extraction it had queued).  16-B
// loads, 4 in flight per lane before the stores (PCIe read latency); bytewise when unaligned.
__global__ __launch_bounds__(256) void k_copy_host(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                                   size_t n) {
    const size_t tid = (size_t)blockIdx.x * blockDim.x + threadIdx.x, nth = (size_t)gridDim.x * blockDim.x;
    if ((((uintptr_t)src | (uintptr_t)dst) & 15) == 0) {
        const uint4* s4 = (const uint4*)src;
        uint4* d4 = (uint4*)dst;
        const size_t n16 = n >> 4;
        size_t i = tid;
        for (; i + 3 * nth < n16; i += 4 * nth) {
            const uint4 a = s4[i], b = s4[i + nth],
                        c = s4[i + 2 * nth], d = s4[i + 3 * nth];
            d4[i] = a;
            d4[i + nth] = b;
            d4[i + 2 * nth] = c;
            d4[i + 3 * nth] = d;
        }
        for (; i < n16; i += nth) d4[i] = s4[i];
        for (size_t j = (n16 << 4) + tid; j < n; j += nth) dst[j] = src[j];
    } else {
        for (size_t j = tid; j < n; j += nth) dst[j] = src[j];
    }
}

int Extractor::upload_host(const uint8_t* h_images, size_t bytes, const uint8_t** d_out) {
    if (bytes > image_bytes) {
        if (d_image) (void)hipFree(d_image);
        d_image = nullptr;
        image_bytes = 0;
        ORBMI_HIP(hipMalloc((void**)&d_image, bytes));
        image_bytes = bytes;
    }
    hipPointerAttribute_t at;
    bool pinned = false;
    if (hipPointerGetAttributes(&at, h_images) == hipSuccess) pinned = at.type == hipMemoryTypeHost;
    else (void)hipGetLastError();
    const uint8_t* src = h_images;
    if (!pinned) {  // pageable: one host copy into a pinned staging buffer of the handle (two, alternating)
        const int k = stage_next;
        stage_next ^= 1;
        if (bytes > stage_bytes[k]) {
            if (stage_ev[k]) ORBMI_HIP(hipEventSynchronize(stage_ev[k]));
            if (h_stage[k]) (void)hipHostFree(h_stage[k]);
            h_stage[k] = nullptr;
            stage_bytes[k] = 0;
            ORBMI_HIP(hipHostMalloc((void**)&h_stage[k], bytes, hipHostMallocDefault));
            stage_bytes[k] = bytes;
        }
        if (!stage_ev[k]) ORBMI_HIP(hipEventCreateWithFlags(&stage_ev[k], hipEventDisableTiming));
        else ORBMI_HIP(hipEventSynchronize(stage_ev[k]));  // its last copy kernel has read it
        std::memcpy(h_stage[k], h_images, bytes);
        src = h_stage[k];
        const int blocks = (int)std::min<size_t>(1024, (bytes / 16 + 255) / 256 + 1);
        hipLaunchKernelGGL(k_copy_host, dim3(blocks), dim3(256), 0, stream, src, d_image, bytes);
        ORBMI_HIP(hipGetLastError());
        ORBMI_HIP(hipEventRecord(stage_ev[k], stream));
    } else {
        const int blocks = (int)std::min<size_t>(1024, (bytes / 16 + 255) / 256 + 1);
        hipLaunchKernelGGL(k_copy_host, dim3(blocks), dim3(256), 0, stream, src, d_image, bytes);
        ORBMI_HIP(hipGetLastError());
    }
    *d_out = d_image;
    return ORBMI_OK;
}

void Extractor::release() {
    for (int k = 0; k < 2; k++) {
        if (stage_ev[k]) { (void)hipEventSynchronize(stage_ev[k]); (void)hipEventDestroy(stage_ev[k]); }
        if (h_stage[k]) (void)hipHostFree(h_stage[k]);
        stage_ev[k] = nullptr;
        h_stage[k] = nullptr;
        stage_bytes[k] = 0;
    }
    for (auto& p : prof_pending) { (void)hipEventDestroy(p.a); (void)hipEventDestroy(p.b); }
    for (auto e : prof_pool) (void)hipEventDestroy(e);
    prof_pending.clear();
    prof_pool.clear();
    if (device >= 0) (void)hipSetDevice(device);
    void* ptrs[] = {d_levels, d_cells, d_regbase, d_pyr_blob, d_btiles, d_blur, d_xtab, d_ytab, d_pyr, d_level_count, d_cand, d_node_of,
                    d_oct, d_oct_count, d_kps, d_desc, d_counts, d_image, d_scale_tab, d_row_start,
                    d_row_list, d_sad, d_stereo_u, d_stereo_d};
    for (void* p : ptrs)
        if (p) (void)hipFree(p);
    if (stream) (void)hipStreamDestroy(stream);
    stream = nullptr;
    if (bstream) (void)hipStreamDestroy(bstream);
    bstream = nullptr;
    for (hipEvent_t e : ev_lv) (void)hipEventDestroy(e);
    ev_lv.clear();
    if (ev_pyr) (void)hipEventDestroy(ev_pyr);
    if (ev_blur) (void)hipEventDestroy(ev_blur);
    if (ev_l0) (void)hipEventDestroy(ev_l0);
    if (ev_f0) (void)hipEventDestroy(ev_f0);
    ev_pyr = ev_blur = ev_l0 = ev_f0 = nullptr;
}

}  // namespace orbmi
