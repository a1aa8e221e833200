// C ABI of the extractor and stereo stages (include/orbmi.h).
#include <algorithm>
#include <cstring>
#include <new>

#include "extractor.h"

using orbmi::Extractor;

struct orbmi_extractor {
    Extractor ex;
};

namespace orbmi {
int stereo_run(Extractor& L, int itemL, Extractor& R, int itemR, float bf, float fx, float* d_u,
               float* d_depth, int n_left_cap);
}

hipStream_t orbmi_extractor_stream_(orbmi_extractor* ex) { return ex ? ex->ex.stream : nullptr; }

extern "C" {

int orbmi_extractor_get_stream(orbmi_extractor* h, void** stream) {
    if (!h || !stream) return ORBMI_E_ARG;
    *stream = (void*)h->ex.stream;
    return ORBMI_OK;
}

int orbmi_extractor_create(int device, int nfeatures, float scale_factor, int nlevels,
                           int ini_th_fast, int min_th_fast, orbmi_extractor** out) {
    if (!out) return ORBMI_E_ARG;
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return ORBMI_E_HIP;
    orbmi_extractor* h = new (std::nothrow) orbmi_extractor();
    if (!h) return ORBMI_E_ARG;
    const int rc = h->ex.init(device, nfeatures, scale_factor, nlevels, ini_th_fast, min_th_fast);
    if (rc) { h->ex.release(); delete h; return rc; }
    *out = h;
    return ORBMI_OK;
}

void orbmi_extractor_destroy(orbmi_extractor* h) {
    if (!h) return;
    h->ex.release();
    delete h;
}

int orbmi_extract(orbmi_extractor* h, const uint8_t* image, int rows, int cols, size_t step,
                  orbmi_keypoint* kps, uint8_t* desc, int capacity, int* n_out) {
    if (!h || !n_out) return ORBMI_E_ARG;
    *n_out = 0;
    if (rows <= 0 || cols <= 0) return ORBMI_OK;  // src/ORBextractor.cc:1046-1047
    if (!image || step < (size_t)cols || capacity < 0 || (capacity > 0 && (!kps || !desc))) return ORBMI_E_ARG;
    Extractor& e = h->ex;
    ORBMI_HIP(hipSetDevice(e.device));  // buffers grown below belong to the handle's device
    int rc;
    if ((rc = e.set_geometry(rows, cols))) return rc;
    const int cap = std::max(capacity, e.nfeatures + 64);
    if ((rc = e.reserve(1, cap))) return rc;
    const size_t bytes = (size_t)rows * cols;
    if (bytes > e.image_bytes) {
        if (e.d_image) (void)hipFree(e.d_image);
        e.d_image = nullptr;
        ORBMI_HIP(hipMalloc((void**)&e.d_image, bytes));
        e.image_bytes = bytes;
    }
    // a contiguous image goes as one copy (a pitched copy from pageable memory runs row by row)
    if (step == (size_t)cols) ORBMI_HIP(hipMemcpyAsync(e.d_image, image, bytes, hipMemcpyHostToDevice, e.stream));
    else ORBMI_HIP(hipMemcpy2DAsync(e.d_image, cols, image, step, cols, rows, hipMemcpyHostToDevice, e.stream));
    if ((rc = e.run(e.d_image, 1, cols, bytes, e.d_kps, e.d_desc, e.d_counts, e.out_capacity))) return rc;
    int n = 0;
    ORBMI_HIP(hipMemcpyAsync(&n, e.d_counts, sizeof(int), hipMemcpyDeviceToHost, e.stream));
    ORBMI_HIP(hipStreamSynchronize(e.stream));
    *n_out = n;
    if (n > e.out_capacity) return ORBMI_E_CAP;  // cannot happen: capacity covers the octree bound
    if (n > capacity) return ORBMI_E_CAP;
    if (n > 0) {
        ORBMI_HIP(hipMemcpyAsync(kps, e.d_kps, (size_t)n * sizeof(orbmi_keypoint), hipMemcpyDeviceToHost, e.stream));
        ORBMI_HIP(hipMemcpyAsync(desc, e.d_desc, (size_t)n * 32, hipMemcpyDeviceToHost, e.stream));
        ORBMI_HIP(hipStreamSynchronize(e.stream));
    }
    return ORBMI_OK;
}

int orbmi_extract_batch_device(orbmi_extractor* h, const uint8_t* d_images, int batch, int rows,
                               int cols, size_t step, size_t image_stride, orbmi_keypoint* d_kps,
                               uint8_t* d_desc, int* d_counts, int capacity) {
    if (!h || !d_images || batch <= 0 || rows <= 0 || cols <= 0 || step < (size_t)cols || !d_kps || !d_desc ||
        !d_counts || capacity <= 0)
        return ORBMI_E_ARG;
    Extractor& e = h->ex;
    ORBMI_HIP(hipSetDevice(e.device));
    int rc;
    if ((rc = e.set_geometry(rows, cols))) return rc;
    if ((rc = e.reserve(batch, 0))) return rc;
    return e.run(d_images, batch, step, image_stride, d_kps, d_desc, d_counts, capacity);
}

int orbmi_extract_batch_host(orbmi_extractor* h, const uint8_t* images, int batch, int rows, int cols,
                             size_t image_stride, orbmi_keypoint* d_kps, uint8_t* d_desc, int* d_counts, int capacity) {
    if (!h || !images || batch <= 0 || rows <= 0 || cols <= 0 || image_stride < (size_t)rows * cols || !d_kps ||
        !d_desc || !d_counts || capacity <= 0)
        return ORBMI_E_ARG;
    Extractor& e = h->ex;
    ORBMI_HIP(hipSetDevice(e.device));
    int rc;
    if ((rc = e.set_geometry(rows, cols))) return rc;
    if ((rc = e.reserve(batch, 0))) return rc;
    const uint8_t* d = nullptr;
    if ((rc = e.upload_host(images, image_stride * (size_t)(batch - 1) + (size_t)rows * cols, &d))) return rc;
    return e.run(d, batch, cols, image_stride, d_kps, d_desc, d_counts, capacity);
}

int orbmi_extractor_synchronize(orbmi_extractor* h) {
    if (!h) return ORBMI_E_ARG;
    ORBMI_HIP(hipSetDevice(h->ex.device));
    ORBMI_HIP(hipStreamSynchronize(h->ex.stream));
    return ORBMI_OK;
}

int orbmi_extractor_get_levels(const orbmi_extractor* h) { return h ? h->ex.nlevels : ORBMI_E_ARG; }
float orbmi_extractor_get_scale_factor(const orbmi_extractor* h) { return h ? h->ex.scale_factor : 0.f; }

static int copy_levels(const orbmi_extractor* h, const std::vector<float>& v, float* out) {
    if (!h || !out) return ORBMI_E_ARG;
    std::copy(v.begin(), v.end(), out);
    return ORBMI_OK;
}
int orbmi_extractor_get_scale_factors(const orbmi_extractor* h, float* out) {
    return h ? copy_levels(h, h->ex.scale, out) : ORBMI_E_ARG;
}
int orbmi_extractor_get_inverse_scale_factors(const orbmi_extractor* h, float* out) {
    return h ? copy_levels(h, h->ex.inv_scale, out) : ORBMI_E_ARG;
}
int orbmi_extractor_get_scale_sigma_squares(const orbmi_extractor* h, float* out) {
    return h ? copy_levels(h, h->ex.sigma2, out) : ORBMI_E_ARG;
}
int orbmi_extractor_get_inverse_scale_sigma_squares(const orbmi_extractor* h, float* out) {
    return h ? copy_levels(h, h->ex.inv_sigma2, out) : ORBMI_E_ARG;
}
int orbmi_extractor_get_features_per_level(const orbmi_extractor* h, int* out) {
    if (!h || !out) return ORBMI_E_ARG;
    std::copy(h->ex.nfeat.begin(), h->ex.nfeat.end(), out);
    return ORBMI_OK;
}

int orbmi_extractor_get_pyramid_level(orbmi_extractor* h, int item, int level, int padded,
                                      uint8_t* out, size_t out_step, int* w, int* hgt) {
    if (!h || !out || !w || !hgt) return ORBMI_E_ARG;
    Extractor& e = h->ex;
    if (e.levels.empty() || item < 0 || item >= e.last_batch) return ORBMI_E_STATE;
    if (level < 0 || level >= e.nlevels) return ORBMI_E_ARG;
    const orbmi::LevelGeom& g = e.levels[level];
    const int cw = padded ? g.W + 2 * orbmi::kEdge : g.W, ch = padded ? g.ph : g.H;
    if (out_step < (size_t)cw) return ORBMI_E_ARG;
    const uint8_t* src = e.d_pyr + item * e.pimg + g.off;
    if (!padded) src += (long long)orbmi::kEdge * g.stride + orbmi::kEdge;
    ORBMI_HIP(hipSetDevice(e.device));
    ORBMI_HIP(hipMemcpy2DAsync(out, out_step, src, g.stride, cw, ch, hipMemcpyDeviceToHost, e.stream));
    ORBMI_HIP(hipStreamSynchronize(e.stream));
    *w = cw;
    *hgt = ch;
    return ORBMI_OK;
}

int orbmi_compute_stereo_matches(orbmi_extractor* left, int item_left, orbmi_extractor* right,
                                 int item_right, float bf, float fx, float* u_right, float* depth,
                                 int n_left) {
    if (!left || !right || (n_left > 0 && (!u_right || !depth))) return ORBMI_E_ARG;
    Extractor& L = left->ex;
    Extractor& R = right->ex;
    if (L.device != R.device) return ORBMI_E_ARG;
    if (L.levels.empty() || R.levels.empty() || item_left >= L.last_batch || item_right >= R.last_batch ||
        item_left < 0 || item_right < 0)
        return ORBMI_E_STATE;
    if (L.rows != R.rows || L.cols != R.cols || L.nlevels != R.nlevels) return ORBMI_E_ARG;
    ORBMI_HIP(hipSetDevice(L.device));
    const int cap = L.last_capacity;
    size_t ucap = L.stereo_cap;
    int rc0;
    if ((rc0 = orbmi::ensure_buf(&L.d_stereo_u, &ucap, (size_t)cap))) return rc0;
    if ((rc0 = orbmi::ensure_buf(&L.d_stereo_d, &L.stereo_cap, (size_t)cap))) return rc0;
    // the right handle's work must be visible to the left handle's stream
    if (&L != &R) ORBMI_HIP(hipStreamSynchronize(R.stream));
    int rc = orbmi::stereo_run(L, item_left, R, item_right, bf, fx, L.d_stereo_u, L.d_stereo_d, cap);
    if (rc) return rc;
    int n = 0;
    ORBMI_HIP(hipMemcpyAsync(&n, L.last_counts + item_left, sizeof(int), hipMemcpyDeviceToHost, L.stream));
    ORBMI_HIP(hipStreamSynchronize(L.stream));
    n = std::min(n, cap);
    if (n_left < n) return ORBMI_E_CAP;
    if (n > 0) {
        ORBMI_HIP(hipMemcpyAsync(u_right, L.d_stereo_u, (size_t)n * sizeof(float), hipMemcpyDeviceToHost, L.stream));
        ORBMI_HIP(hipMemcpyAsync(depth, L.d_stereo_d, (size_t)n * sizeof(float), hipMemcpyDeviceToHost, L.stream));
        ORBMI_HIP(hipStreamSynchronize(L.stream));
    }
    return ORBMI_OK;
}

int orbmi_compute_stereo_matches_batch_device(orbmi_extractor* h, float bf, float fx, float* d_u_right,
                                              float* d_depth) {
    if (!h || !d_u_right || !d_depth) return ORBMI_E_ARG;
    Extractor& e = h->ex;
    if (e.last_batch < 2) return ORBMI_E_STATE;
    for (int p = 0; p + 1 < e.last_batch; p += 2) {
        const long long o = (long long)p * e.last_capacity;
        int rc = orbmi::stereo_run(e, p, e, p + 1, bf, fx, d_u_right + o, d_depth + o, e.last_capacity);
        if (rc) return rc;
    }
    return ORBMI_OK;
}

}  // extern "C"

extern "C" int orbmi_set_profiling(orbmi_extractor* h, unsigned stage_mask) {
    if (!h) return ORBMI_E_ARG;
    h->ex.prof_mask = stage_mask;
    return ORBMI_OK;
}

extern "C" int orbmi_read_profile(orbmi_extractor* h, double* ms, long long* launches) {
    if (!h || !ms || !launches) return ORBMI_E_ARG;
    Extractor& e = h->ex;
    ORBMI_HIP(hipSetDevice(e.device));
    ORBMI_HIP(hipStreamSynchronize(e.stream));
    for (auto& p : e.prof_pending) {
        float t = 0.f;
        ORBMI_HIP(hipEventElapsedTime(&t, p.a, p.b));
        if (p.stage >= 0 && p.stage < ORBMI_NUM_STAGES) { ms[p.stage] += t; launches[p.stage] += 1; }
        e.prof_pool.push_back(p.a);
        e.prof_pool.push_back(p.b);
    }
    e.prof_pending.clear();
    return ORBMI_OK;
}

// ---- debug hooks (include/orbmi_debug.h) ---------------------------------------------
#include "../../include/orbmi_debug.h"

extern "C" int orbmi_debug_fast_candidates(orbmi_extractor* h, int item, int level, int* xyr, int cap,
                                           int* n_out) {
    if (!h || !n_out || (cap > 0 && !xyr)) return ORBMI_E_ARG;
    Extractor& e = h->ex;
    if (e.levels.empty() || item < 0 || item >= e.last_batch || level < 0 || level >= e.nlevels)
        return ORBMI_E_STATE;
    ORBMI_HIP(hipSetDevice(e.device));
    ORBMI_HIP(hipStreamSynchronize(e.stream));
    int rc_[orbmi::kFastRegions];
    ORBMI_HIP(hipMemcpy(rc_, e.d_level_count + ((size_t)item * e.nlevels + level) * orbmi::kFastRegions,
                        sizeof(rc_), hipMemcpyDeviceToHost));
    std::vector<uint2> cand;
    for (int j = 0; j < orbmi::kFastRegions; j++) {
        if (rc_[j] <= 0) continue;
        const size_t at = cand.size();
        cand.resize(at + rc_[j]);
        ORBMI_HIP(hipMemcpy(cand.data() + at, e.d_cand + (size_t)item * e.keys_cap + e.regbase[level * orbmi::kFastRegions + j],
                            rc_[j] * sizeof(uint2), hipMemcpyDeviceToHost));
    }
    const int count = (int)cand.size();
    // k_fast's dense array is in cell-completion order; the tags restore the cell loop's order
    std::sort(cand.begin(), cand.end(), [](const uint2& a, const uint2& b) { return a.y < b.y; });
    int n = 0;
    for (int k = 0; k < count; k++, n++)
        if (n < cap) {
            const uint32_t v = cand[k].x;
            xyr[3 * n] = v & 0xFFF;
            xyr[3 * n + 1] = (v >> 12) & 0xFFF;
            xyr[3 * n + 2] = v >> 24;
        }
    *n_out = n;
    return n > cap ? ORBMI_E_CAP : ORBMI_OK;
}

extern "C" int orbmi_debug_octree_level(orbmi_extractor* h, int item, int level, int* xyr, int cap, int* n_out) {
    if (!h || !n_out || (cap > 0 && !xyr)) return ORBMI_E_ARG;
    Extractor& e = h->ex;
    if (e.levels.empty() || item < 0 || item >= e.last_batch || level < 0 || level >= e.nlevels)
        return ORBMI_E_STATE;
    ORBMI_HIP(hipSetDevice(e.device));
    ORBMI_HIP(hipStreamSynchronize(e.stream));
    const orbmi::LevelGeom& g = e.levels[level];
    int n = 0;
    ORBMI_HIP(hipMemcpy(&n, e.d_oct_count + (size_t)item * e.nlevels + level, sizeof(int), hipMemcpyDeviceToHost));
    std::vector<uint2> v(std::max(n, 1));
    if (n > 0)
        ORBMI_HIP(hipMemcpy(v.data(), e.d_oct + (size_t)item * e.out_cap + g.out_base, n * sizeof(uint2),
                            hipMemcpyDeviceToHost));
    for (int i = 0; i < n && i < cap; i++) {
        xyr[3 * i] = v[i].x & 0xFFFF;
        xyr[3 * i + 1] = v[i].x >> 16;
        xyr[3 * i + 2] = (int)v[i].y;
    }
    *n_out = n;
    return n > cap ? ORBMI_E_CAP : ORBMI_OK;
}
