// Host-side runtime of the device ORB extractor (shared by extractor.hip, stereo.hip, capi.cpp).
#pragma once
#include <vector>

#include "orbmi_common.h"

namespace orbmi {

// Per pyramid level constants, resident in device memory (one copy per handle geometry).
struct LevelGeom {
    int W, H;            // interior size  (ComputePyramid :1111-1112)
    int stride, ph;      // padded row pitch (>= W+38, 64-aligned) and padded height H+38
    long long off;       // byte offset of the padded level inside one image's pyramid
    int cell_begin, cell_end;   // FAST cell range (global cell index)
    int nfeat;           // mnFeaturesPerLevel[level]
    int out_base, out_cap;      // octree output slots (per image)
    int key_base, key_cap;      // candidate scratch (per image)
    int width, height;   // octree area maxBorderX-minBorderX, maxBorderY-minBorderY
    int nIni;            // DistributeOctTree initial node count
    float hX;            // (float)width / nIni
    float scale;         // mvScaleFactor[level]
    float size;          // (float)(int)(PATCH_SIZE * scale)
    int blur_xv;         // first column of the GaussianBlur scalar tail (4*floor(W/4))
    int resize_xv;       // first column of the resize vertical scalar tail
    int xtab_off, ytab_off;     // offsets into the resize coefficient tables (level >= 1)
    long long boff;      // byte offset of the blurred level (interior only) inside one image's blur
    int bstride;         // blurred row pitch (W rounded up to 128)
};

// One FAST cell of ComputeKeyPointsOctTree (src/ORBextractor.cc:789-829).
struct CellGeom {
    short x0, y0, w, h;  // ROI in interior coordinates; w == 0 -> skipped cell
    short sx, sy;        // j*wCell, i*hCell shift added to ROI coordinates
    int slot_base;       // base of the cell's candidate region (per image; cells of one level
                         // share kFastRegions regions, cell k of the level writes region k % R)
    int level;
    long long roi_off;   // byte offset of the ROI's first pixel in one image's pyramid (level plane,
                         // border, stride folded in: k_fast needs no LevelGeom load)
    int stride;          // the level's row stride
    int lcell;           // index of the cell within its level
};

struct XTab { short sx0, sx1, a0, a1; };  // horizontal resize: source taps and 11-bit weights
struct YTab { short y0, y1, b0, b1; };    // vertical resize
struct PyrRect { short x0, x1, y0, y1; };  // half-open interior rectangle of one level
struct PyrTile { PyrRect own, need; };     // k_pyramid tile of one level: written to HBM / computed in LDS

constexpr int kOctNodeCap = 2048;  // live quadtree nodes per level held in LDS
constexpr int kFastRegions = 16;   // candidate regions per level (spreads k_fast's allocation atomics)
constexpr int kBlurTW = 128, kBlurTH = 32;  // GaussianBlur output tile

// Grow-only device buffer.
template <class T>
inline int ensure_buf(T** p, size_t* cap, size_t n) {
    if (*p && *cap >= n) return ORBMI_OK;
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    *cap = 0;
    if (n == 0) n = 1;
    ORBMI_HIP(hipMalloc((void**)p, n * sizeof(T)));
    *cap = n;
    return ORBMI_OK;
}

struct Extractor {
    int device = 0;
    int nfeatures = 0, nlevels = 0, ini_th = 0, min_th = 0;
    float scale_factor = 0.f;
    std::vector<float> scale, inv_scale, sigma2, inv_sigma2;
    std::vector<int> nfeat, umax;

    // geometry for the current image size
    int rows = 0, cols = 0;
    std::vector<LevelGeom> levels;
    std::vector<CellGeom> cells;
    std::vector<int2> btiles;
    long long pimg = 0;      // bytes of one padded pyramid
    long long bimg = 0;      // bytes of one blurred pyramid
    int keys_cap = 0, out_cap = 0;
    bool describe_wave = false;  // ORBMI_DESC=wave: the one-keypoint-per-wave describe kernel
    bool fast_v1 = false;        // ORBMI_FAST=v1: the per-lane FAST kernel
    bool fast_split = false;     // ORBMI_FAST=split: k_fast2 with the segment tests and scores as separate stages
    int blur_mode = -1;          // GaussianBlur (ORBMI_BLUR): -1 by batch, 0 side stream, 1 in the octree launch, 2 after it,
                                 // 3 side stream after FAST, 4 side stream level by level behind the pyramid
    hipStream_t bstream = nullptr;  // the blur's side stream
    hipEvent_t ev_pyr = nullptr, ev_blur = nullptr, ev_l0 = nullptr, ev_f0 = nullptr;
    std::vector<hipEvent_t> ev_lv;   // ORBMI_BLUR=perlevel: level l of the pyramid written
    std::vector<int> btile_off;      // first blur tile of each level (btiles are level-major), and the end
    bool fast_early = false;     // ORBMI_FAST_EARLY=1: level 0's FAST on the side stream beside the resize chain

    // device buffers (capacity for `bcap` images)
    int bcap = 0;
    hipStream_t stream = nullptr;
    LevelGeom* d_levels = nullptr;
    CellGeom* d_cells = nullptr;
    XTab* d_xtab = nullptr;
    YTab* d_ytab = nullptr;
    uint8_t* d_pyr = nullptr;
    uint8_t* d_blur = nullptr;     // blurred levels: interior only, rows of bstride bytes
    int2* d_btiles = nullptr;      // blur tiles: {level, x0 | y0 << 16}
    int nbtiles = 0;
    int fast_maxw = 0, fast_maxh = 0, fast_wave_bytes = 0;  // largest cell ROI, k_fast's LDS per wave
    int* d_level_count = nullptr;   // [b][level][region] FAST candidates (k_fast allocates, k_pyr_level0 clears)
    int* d_regbase = nullptr;       // [level][region] first slot of each candidate region (per image)
    std::vector<uint32_t> pyr_blob; // k_pyramid parameter blocks, pyr_blob_words per tile
    uint32_t* d_pyr_blob = nullptr;
    int pyr_kx = 0, pyr_ky = 0, pyr_hx = 0, pyr_hy = 0, pyr_blob_words = 0, pyr_lds0 = 0, pyr_lds_half = 0;
    std::vector<int> regbase;
    uint2* d_cand = nullptr;        // [b][keys_cap] {x | y << 12 | score << 24, cell << 10 | rank}
    uint32_t* d_node_of = nullptr;  // octree node | depth << 16 of keys beyond the register-resident ones
    uint2* d_oct = nullptr;        // {x | y << 16 (level coords), score}
    int* d_oct_count = nullptr;    // [b][level]
    // last outputs (host API and stereo input)
    int out_capacity = 0;          // keypoints per image in d_kps / d_desc
    orbmi_keypoint* d_kps = nullptr;
    uint8_t* d_desc = nullptr;
    int* d_counts = nullptr;
    uint8_t* d_image = nullptr;    // staging for host images
    size_t image_bytes = 0;
    // pageable host images of orbmi_extract_batch_host: pinned staging, two alternating buffers,
    // each guarded by the event after the copy kernel that reads it
    uint8_t* h_stage[2] = {nullptr, nullptr};
    size_t stage_bytes[2] = {0, 0};
    hipEvent_t stage_ev[2] = {nullptr, nullptr};
    int stage_next = 0;
    int last_batch = 0;
    // last batch output location (may be caller buffers for the device API)
    orbmi_keypoint* last_kps = nullptr;
    uint8_t* last_desc = nullptr;
    int* last_counts = nullptr;
    int last_capacity = 0;
    // stereo scratch
    float* d_scale_tab = nullptr;  // [scale | inv_scale], 2*nlevels floats
    int* d_row_start = nullptr;
    int* d_row_list = nullptr;
    int* d_sad = nullptr;
    size_t row_cap = 0, row_list_cap = 0, sad_cap = 0, stereo_cap = 0;
    float* d_stereo_u = nullptr;
    float* d_stereo_d = nullptr;

    // per-stage HIP-event profiling (orbmi_set_profiling / orbmi_read_profile)
    unsigned prof_mask = 0;
    struct ProfPair { int stage; hipEvent_t a, b; };
    std::vector<ProfPair> prof_pending;
    std::vector<hipEvent_t> prof_pool;
    hipEvent_t prof_event();
    hipEvent_t prof_begin(int stage, hipStream_t s = nullptr);
    void prof_end(int stage, hipEvent_t a, hipStream_t s = nullptr);

    int init(int dev, int nf, float sf, int nl, int ini, int mn);
    int set_geometry(int rows, int cols);
    int reserve(int batch, int capacity);
    int ensure_side_stream();  // bstream + its events on first use (large batches only)
    // host images -> d_image by a copy kernel on `stream` (pinned memory read in place, pageable
    // memory staged first); *d_out = d_image
    int upload_host(const uint8_t* h_images, size_t bytes, const uint8_t** d_out);
    int run(const uint8_t* d_images, int batch, size_t step, size_t image_stride,
            orbmi_keypoint* kps, uint8_t* desc, int* counts, int capacity);
    void release();
};

}  // namespace orbmi
