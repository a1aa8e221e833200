// C ABI of the matchers (include/orbmi.h, "ORBmatcher" section).  Inputs may live in host
// or device memory; host arrays are staged through a per-handle device arena.
#include <algorithm>
#include <cstring>
#include <new>

#include "matcher.h"
#include "tri_geom.h"

using orbmi::DevFrame;
using orbmi::DevFV;
using orbmi::Matcher;
using orbmi::FuseKF;
using orbmi::TriPair;

struct orbmi_matcher {
    Matcher m;
};

hipStream_t orbmi_extractor_stream_(orbmi_extractor* ex);  // capi_extract.cpp

namespace orbmi {

void* Matcher::stage(size_t bytes) {
    bytes = (bytes + 255) & ~(size_t)255;
    std::vector<Block>& arena = gens[gen].blocks;
    for (Block& b : arena)
        if (b.size - b.used >= bytes) { void* p = b.p + b.used; b.used += bytes; return p; }
    Block b{nullptr, std::max(bytes, (size_t)(4 << 20)), 0, nullptr};
    if (hipMalloc((void**)&b.p, b.size) != hipSuccess) return nullptr;
    if (hipHostMalloc((void**)&b.h, b.size, hipHostMallocDefault) != hipSuccess) {
        (void)hipFree(b.p);
        return nullptr;
    }
    b.used = bytes;
    arena.push_back(b);
    return b.p;
}

uint8_t* Matcher::mirror(const void* d) {
    const uint8_t* q = (const uint8_t*)d;
    for (Block& b : gens[gen].blocks)
        if (q >= b.p && q < b.p + b.size) return b.h + (q - b.p);
    return nullptr;
}

hipError_t Matcher::flush_up() {
    if (!up.n) return hipSuccess;
    const hipError_t e = hipMemcpyAsync(up.d, up.h, up.n, hipMemcpyHostToDevice, stream);
    up.n = 0;
    if (e != hipSuccess && up_err == hipSuccess) up_err = e;
    return e;
}

hipError_t Matcher::h2d(void* d, const void* src, size_t bytes) {
    if (!bytes) return hipSuccess;
    uint8_t* h = mirror(d);
    if (!h) return hipMemcpyAsync(d, src, bytes, hipMemcpyHostToDevice, ls());
    memcpy(h, src, bytes);
    // the allocation right after the pending range (stage() rounds to 256 B; the gap is the
    // previous allocation's padding): extend the range, else send it and start a new one
    const size_t end = (up.n + 255) & ~(size_t)255;
    if (up.n && (uint8_t*)d == up.d + end && h == up.h + end) {
        up.n = end + bytes;
        return hipSuccess;
    }
    const hipError_t e = flush_up();
    up = PendUp{(uint8_t*)d, h, bytes};
    return e;
}

hipError_t Matcher::d2h(void* user, const void* d, size_t bytes) {
    if (!bytes) return hipSuccess;
    uint8_t* h = mirror(d);
    if (!h) return hipMemcpyAsync(user, d, bytes, hipMemcpyDeviceToHost, ls());
    pend.push_back(Pend{user, h, bytes});
    return hipMemcpyAsync(h, d, bytes, hipMemcpyDeviceToHost, ls());
}

void Matcher::d2h_flush() {
    for (const Pend& p : pend) memcpy(p.user, p.mirror, p.bytes);
    pend.clear();
}

void Matcher::arena_reset() {
    (void)flush_up();  // (nothing is left pending by a finished call; kept for safety)
    up_err = hipSuccess;
    // the generation just used may still be read by the work enqueued so far: mark it with an
    // event, move on, and wait only for the generation about to be reused
    bool used = false;
    for (Block& b : gens[gen].blocks) used |= b.used > 0;
    if (used) {
        if (!gens[gen].ev && hipEventCreateWithFlags(&gens[gen].ev, hipEventDisableTiming) != hipSuccess) {
            gens[gen].ev = nullptr;
            (void)hipStreamSynchronize(stream);  // no event: fall back to a full wait
        } else if (gens[gen].ev) {
            (void)hipEventRecord(gens[gen].ev, stream);
            gens[gen].pending = true;
        }
        gen = (gen + 1) % kArenaGens;
    }
    Gen& g = gens[gen];
    if (g.pending) {
        (void)hipEventSynchronize(g.ev);
        g.pending = false;
    }
    for (Block& b : g.blocks) b.used = 0;
    pend.clear();
}

void Matcher::release() {
    (void)hipSetDevice(device);
    if (stream) (void)flush_up();
    if (own_stream && stream) (void)hipStreamSynchronize(stream);
    if (!own_stream && stream) (void)hipStreamSynchronize(stream);  // staged inputs may still be read
    void* ptrs[] = {d_cell_start, d_cell_list, d_kp_cell, d_mcell_start, d_mcell_list, d_mkp_cell, d_cand, d_ncand, d_top,
                    d_res, d_bin_of, d_hist, d_scalars, d_track};
    for (void* p : ptrs)
        if (p) (void)hipFree(p);
    for (GridSlot& g : gslot) {
        if (g.cs) (void)hipFree(g.cs);
        if (g.cl) (void)hipFree(g.cl);
        if (g.kc) (void)hipFree(g.kc);
        g = GridSlot{};
    }
    for (Gen& g : gens) {
        for (Block& b : g.blocks) {
            (void)hipFree(b.p);
            if (b.h) (void)hipHostFree(b.h);
        }
        g.blocks.clear();
        if (g.ev) (void)hipEventDestroy(g.ev);
        g.ev = nullptr;
        g.pending = false;
    }
    if (stream && own_stream) (void)hipStreamDestroy(stream);
    stream = nullptr;
}

}  // namespace orbmi

namespace {

bool on_device(const void* p) {
    if (!p) return false;
    hipPointerAttribute_t at;
    if (hipPointerGetAttributes(&at, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return at.type == hipMemoryTypeDevice || at.type == hipMemoryTypeManaged;
}

// Device view of an input array (copied into the arena when it is host memory).
template <class T>
const T* dev_in(Matcher& m, const T* p, size_t n, int* rc) {
    if (!p || n == 0) return p;
    if (on_device(p)) return p;
    T* d = (T*)m.stage(n * sizeof(T));
    if (!d || m.h2d(d, p, n * sizeof(T)) != hipSuccess) {
        *rc = ORBMI_E_HIP;
        return nullptr;
    }
    return d;
}

struct OutBuf {
    void* user = nullptr;
    void* dev = nullptr;
    size_t bytes = 0;
};

template <class T>
T* dev_out(Matcher& m, T* p, size_t n, std::vector<OutBuf>& outs) {
    if (on_device(p)) return p;
    T* d = (T*)m.stage(std::max(n, (size_t)1) * sizeof(T));
    outs.push_back(OutBuf{p, d, n * sizeof(T)});
    return d;
}

// Copy host-bound outputs back and synchronise; fully device-resident calls (every output a
// device pointer, counts not requested) return without waiting.
int finish(Matcher& m, std::vector<OutBuf>& outs, int* nmatches_dev, int* nmatches, int* extra_dev = nullptr,
           int* extra = nullptr) {
    bool wait = false;
    ORBMI_HIP(m.flush_up());
    if (m.up_err != hipSuccess) return ORBMI_E_HIP;
    for (OutBuf& o : outs)
        if (o.bytes) { ORBMI_HIP(m.d2h(o.user, o.dev, o.bytes)); wait = true; }
    int tmp[2] = {0, 0};
    if (nmatches && nmatches_dev) { ORBMI_HIP(hipMemcpyAsync(&tmp[0], nmatches_dev, sizeof(int), hipMemcpyDeviceToHost, m.ls())); wait = true; }
    if (extra && extra_dev) { ORBMI_HIP(hipMemcpyAsync(&tmp[1], extra_dev, sizeof(int), hipMemcpyDeviceToHost, m.ls())); wait = true; }
    if (wait) ORBMI_HIP(hipStreamSynchronize(m.ls()));
    m.d2h_flush();
    if (nmatches) *nmatches = tmp[0];
    if (extra) *extra = tmp[1];
    return ORBMI_OK;
}

int read_small(const float* p, int n, float* out) {
    if (on_device(p)) {
        ORBMI_HIP(hipMemcpy(out, p, n * sizeof(float), hipMemcpyDeviceToHost));
    } else {
        memcpy(out, p, n * sizeof(float));
    }
    return ORBMI_OK;
}

int make_frame(Matcher& m, const orbmi_frame_view* v, DevFrame* F, bool need_pose) {
    if (!v || v->n < 0 || (v->n > 0 && (!v->keys_un || !v->desc))) return ORBMI_E_ARG;
    if (v->nlevels < 1 || v->nlevels > orbmi::kMaxLevels || !v->scale_factors) return ORBMI_E_ARG;
    int rc = 0;
    memset(F, 0, sizeof(*F));
    F->n = v->n;
    F->n_dev = v->n_device;
    if (F->n_dev && !on_device(F->n_dev)) return ORBMI_E_ARG;
    F->keys = dev_in(m, v->keys_un, (size_t)v->n, &rc);
    F->u_right = dev_in(m, v->u_right, v->u_right ? (size_t)v->n : 0, &rc);
    F->desc = dev_in(m, v->desc, (size_t)v->n * 32, &rc);
    if (rc) return rc;
    if (need_pose) {
        if (!v->tcw) return ORBMI_E_ARG;
        if (on_device(v->tcw)) F->tcw_dev = v->tcw;  // read by the kernels in stream order
        else memcpy(F->tcw, v->tcw, sizeof(F->tcw));
    }
    if ((rc = read_small(v->scale_factors, v->nlevels, F->scale))) return rc;
    F->fx = v->fx; F->fy = v->fy; F->cx = v->cx; F->cy = v->cy; F->bf = v->bf; F->mb = v->mb;
    F->min_x = v->min_x; F->max_x = v->max_x; F->min_y = v->min_y; F->max_y = v->max_y;
    F->grid_w_inv = v->grid_w_inv; F->grid_h_inv = v->grid_h_inv;
    F->nlevels = v->nlevels;
    F->log_scale_factor = v->log_scale_factor;
    return ORBMI_OK;
}

int make_fv(Matcher& m, const orbmi_feature_vector* v, DevFV* d) {
    if (!v || v->nnodes < 0) return ORBMI_E_ARG;
    int rc = 0;
    d->nnodes = v->nnodes;
    if (v->nnodes == 0) { d->node_id = nullptr; d->off = nullptr; d->feat = nullptr; return ORBMI_OK; }
    // total features = off[nnodes], needed only to stage a host feature list (a device one is
    // used in place: no read-back)
    int total = 0;
    if (!on_device(v->feat)) {
        if (on_device(v->off)) ORBMI_HIP(hipMemcpy(&total, v->off + v->nnodes, sizeof(int), hipMemcpyDeviceToHost));
        else total = v->off[v->nnodes];
    }
    d->node_id = dev_in(m, v->node_id, (size_t)v->nnodes, &rc);
    d->off = dev_in(m, v->off, (size_t)v->nnodes + 1, &rc);
    d->feat = dev_in(m, v->feat, (size_t)total, &rc);
    return rc;
}

int scalars(Matcher& m) {
    int rc = orbmi::ensure_buf(&m.d_scalars, &m.cap_scalars, 4);
    if (rc) return rc;
    ORBMI_HIP(hipMemsetAsync(m.d_scalars, 0, 4 * sizeof(int), m.ls()));
    return ORBMI_OK;
}

}  // namespace

extern "C" {

int orbmi_matcher_create(int device, orbmi_matcher** out) {
    if (!out) return ORBMI_E_ARG;
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return ORBMI_E_HIP;
    orbmi_matcher* h = new (std::nothrow) orbmi_matcher();
    if (!h) return ORBMI_E_ARG;
    h->m.device = device;
    if (hipSetDevice(device) != hipSuccess || orbmi::stream_create(&h->m.stream, "MATCHER") != hipSuccess) {
        delete h;
        return ORBMI_E_HIP;
    }
    *out = h;
    return ORBMI_OK;
}

int orbmi_matcher_share_stream(orbmi_matcher* h, orbmi_extractor* ex) {
    if (!h || !ex) return ORBMI_E_ARG;
    Matcher& m = h->m;
    hipStream_t s = orbmi_extractor_stream_(ex);
    if (!s) return ORBMI_E_STATE;
    ORBMI_HIP(hipSetDevice(m.device));
    ORBMI_HIP(hipStreamSynchronize(m.stream));
    if (m.own_stream) ORBMI_HIP(hipStreamDestroy(m.stream));
    m.stream = s;
    m.own_stream = false;
    return ORBMI_OK;
}

int orbmi_matcher_reserve_cus(orbmi_matcher* h, int n) {
    if (!h || n < 0) return ORBMI_E_ARG;
    Matcher& m = h->m;
    if (!m.own_stream) return ORBMI_E_STATE;
    ORBMI_HIP(hipSetDevice(m.device));
    int ncu = 0;
    ORBMI_HIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, m.device));
    if (n >= ncu) return ORBMI_E_ARG;
    hipStream_t s = nullptr;
    if (n == 0) {
        ORBMI_HIP(orbmi::stream_create(&s, "MATCHER"));
    } else {
        std::vector<uint32_t> mask((size_t)(ncu + 31) / 32, 0u);
        for (int c = 0; c < ncu - n; c++) mask[c >> 5] |= 1u << (c & 31);
        ORBMI_HIP(hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data()));
    }
    (void)hipStreamSynchronize(m.stream);
    (void)hipStreamDestroy(m.stream);
    m.stream = s;
    return ORBMI_OK;
}

int orbmi_matcher_assign_features_to_grid(orbmi_matcher* h, const orbmi_frame_view* v) {
    if (!h || !v || (v->n > 0 && !on_device(v->keys_un))) return ORBMI_E_ARG;
    Matcher& m = h->m;
    ORBMI_HIP(hipSetDevice(m.device));
    m.arena_reset();
    DevFrame F;
    int rc;
    if ((rc = make_frame(m, v, &F, false))) return rc;
    if ((rc = orbmi::pin_grid(m, F))) return rc;
    ORBMI_HIP(hipGetLastError());
    return ORBMI_OK;
}

int orbmi_matcher_build_grid_slot(orbmi_matcher* h, const orbmi_frame_view* v, int slot, void* stream) {
    if (!h || !v || slot < 0 || slot >= orbmi::Matcher::kGridSlots || (v->n > 0 && !on_device(v->keys_un)) ||
        (v->n > 0 && !on_device(v->desc)) || (v->u_right && !on_device(v->u_right)))
        return ORBMI_E_ARG;
    Matcher& m = h->m;
    ORBMI_HIP(hipSetDevice(m.device));
    DevFrame F;
    int rc;
    if ((rc = make_frame(m, v, &F, false))) return rc;  // device arrays: nothing staged
    hipStream_t s = stream ? (hipStream_t)stream : m.ls();
    if ((rc = orbmi::build_grid_slot(m, F, slot, s))) return rc;
    ORBMI_HIP(hipGetLastError());
    return ORBMI_OK;
}

int orbmi_matcher_pin_grid_slot(orbmi_matcher* h, const orbmi_frame_view* v, int slot) {
    if (!h || !v || slot < 0 || slot >= orbmi::Matcher::kGridSlots || (v->n > 0 && !on_device(v->keys_un)))
        return ORBMI_E_ARG;
    Matcher& m = h->m;
    ORBMI_HIP(hipSetDevice(m.device));
    DevFrame F;
    int rc;
    if ((rc = make_frame(m, v, &F, false))) return rc;
    return orbmi::pin_grid_slot(m, F, slot);
}

int orbmi_matcher_release_grid(orbmi_matcher* h) {
    if (!h) return ORBMI_E_ARG;
    h->m.grid_pinned = false;
    return ORBMI_OK;
}

int orbmi_matcher_get_stream(orbmi_matcher* h, void** stream) {
    if (!h || !stream) return ORBMI_E_ARG;
    *stream = (void*)h->m.stream;
    return ORBMI_OK;
}

void orbmi_matcher_destroy(orbmi_matcher* h) {
    if (!h) return;
    h->m.release();
    delete h;
}

int orbmi_is_in_frustum(orbmi_matcher* h, const orbmi_frame_view* v, const orbmi_mappoint* mps, int n_mp,
                        float viewing_cos_limit, orbmi_mappoint_track* track) {
    if (!h || n_mp < 0 || (n_mp > 0 && (!mps || !track))) return ORBMI_E_ARG;
    Matcher& m = h->m;
    ORBMI_HIP(hipSetDevice(m.device));
    m.arena_reset();
    DevFrame F;
    int rc;
    if ((rc = make_frame(m, v, &F, true))) return rc;
    const orbmi_mappoint* d_mps = dev_in(m, mps, (size_t)n_mp, &rc);
    if (rc) return rc;
    std::vector<OutBuf> outs;
    orbmi_mappoint_track* d_tr = dev_out(m, track, (size_t)n_mp, outs);
    if ((rc = orbmi::launch_frustum(m, F, d_mps, n_mp, viewing_cos_limit, d_tr, nullptr))) return rc;
    ORBMI_HIP(hipGetLastError());
    return finish(m, outs, nullptr, nullptr);
}

int orbmi_search_by_projection_local(orbmi_matcher* h, const orbmi_frame_view* v, const uint8_t* occupied,
                                     const orbmi_mappoint* mps, const orbmi_mappoint_track* track, int n_mp,
                                     float th, float nnratio, int32_t* match_mp, int* nmatches) {
    if (!h || !occupied || !match_mp || n_mp < 0 || (n_mp > 0 && (!mps || !track))) return ORBMI_E_ARG;
    Matcher& m = h->m;
    ORBMI_HIP(hipSetDevice(m.device));
    m.arena_reset();
    DevFrame F;
    int rc;
    if ((rc = make_frame(m, v, &F, false))) return rc;
    const uint8_t* d_occ = dev_in(m, occupied, (size_t)std::max(F.n, 1), &rc);
    const orbmi_mappoint* d_mps = dev_in(m, mps, (size_t)n_mp, &rc);
    const orbmi_mappoint_track* d_tr = dev_in(m, track, (size_t)n_mp, &rc);
    if (rc) return rc;
    if ((rc = scalars(m))) return rc;
    std::vector<OutBuf> outs;
    int* d_out = dev_out(m, match_mp, (size_t)F.n, outs);
    if ((rc = orbmi::launch_local_search(m, F, d_occ, d_mps, d_tr, n_mp, th, nnratio, d_out, m.d_scalars))) return rc;
    ORBMI_HIP(hipGetLastError());
    return finish(m, outs, m.d_scalars, nmatches);
}

int orbmi_search_local_points(orbmi_matcher* h, const orbmi_frame_view* v, const uint8_t* occupied,
                              const orbmi_mappoint* mps, int n_mp, float th, int32_t* match_mp, int* nmatches,
                              int* n_to_match) {
    return orbmi_search_local_points_track(h, v, occupied, mps, n_mp, th, match_mp, nmatches, n_to_match, nullptr);
}

int orbmi_search_local_points_track(orbmi_matcher* h, const orbmi_frame_view* v, const uint8_t* occupied,
                                    const orbmi_mappoint* mps, int n_mp, float th, int32_t* match_mp, int* nmatches,
                                    int* n_to_match, orbmi_mappoint_track* track_out) {
    if (!h || !occupied || !match_mp || n_mp < 0 || (n_mp > 0 && !mps)) return ORBMI_E_ARG;
    Matcher& m = h->m;
    ORBMI_HIP(hipSetDevice(m.device));
    m.arena_reset();
    DevFrame F;
    int rc;
    if ((rc = make_frame(m, v, &F, true))) return rc;
    const uint8_t* d_occ = dev_in(m, occupied, (size_t)std::max(F.n, 1), &rc);
    const orbmi_mappoint* d_mps = dev_in(m, mps, (size_t)n_mp, &rc);
    if (rc) return rc;
    // k_greedy stores the match count (slot 0) unconditionally; only the nToMatch counter (slot 1,
    // atomics in k_frustum) needs zeroing, and only when the caller asks for it
    if ((rc = n_to_match ? scalars(m) : orbmi::ensure_buf(&m.d_scalars, &m.cap_scalars, 4))) return rc;
    std::vector<OutBuf> outs;
    orbmi_mappoint_track* d_tr = nullptr;
    if (track_out) {  // the isInFrustum outputs go to the caller (host: copied back with the matches)
        d_tr = dev_out(m, track_out, (size_t)std::max(n_mp, 1), outs);
    } else {
        if ((rc = orbmi::ensure_buf(&m.d_track, &m.cap_track, (size_t)std::max(n_mp, 1)))) return rc;
        d_tr = m.d_track;
    }
    int* d_out = dev_out(m, match_mp, (size_t)F.n, outs);
    // Tracking::SearchLocalPoints: isInFrustum(pMP, 0.5); ORBmatcher matcher(0.8)
    if ((rc = orbmi::launch_frustum(m, F, d_mps, n_mp, 0.5f, d_tr, n_to_match ? m.d_scalars + 1 : nullptr))) return rc;
    if ((rc = orbmi::launch_local_search(m, F, d_occ, d_mps, d_tr, n_mp, th, 0.8f, d_out, m.d_scalars))) return rc;
    ORBMI_HIP(hipGetLastError());
    int ntm = 0;  // read back (and waited for) only when the caller asks for it
    rc = finish(m, outs, m.d_scalars, nmatches, m.d_scalars + 1, n_to_match ? &ntm : nullptr);
    if (n_to_match) *n_to_match = ntm;
    return rc;
}

int orbmi_search_by_projection_last_frame(orbmi_matcher* h, const orbmi_frame_view* cf, const uint8_t* occupied,
                                          const orbmi_frame_view* lf, const orbmi_lastframe_point* lf_points,
                                          float th, int mono, int check_ori, int32_t* match_lf, int* nmatches) {
    if (!h || !occupied || !match_lf || !lf || (lf->n > 0 && !lf_points)) return ORBMI_E_ARG;
    Matcher& m = h->m;
    ORBMI_HIP(hipSetDevice(m.device));
    m.arena_reset();
    DevFrame CF, LF;
    int rc;
    if ((rc = make_frame(m, cf, &CF, true))) return rc;
    if ((rc = make_frame(m, lf, &LF, true))) return rc;
    const uint8_t* d_occ = dev_in(m, occupied, (size_t)std::max(CF.n, 1), &rc);
    const orbmi_lastframe_point* d_lfp = dev_in(m, lf_points, (size_t)LF.n, &rc);
    if (rc) return rc;
    if ((rc = scalars(m))) return rc;
    std::vector<OutBuf> outs;
    int* d_out = dev_out(m, match_lf, (size_t)CF.n, outs);
    if ((rc = orbmi::launch_lastframe_search(m, CF, d_occ, LF, d_lfp, th, mono, check_ori, d_out, m.d_scalars)))
        return rc;
    ORBMI_HIP(hipGetLastError());
    return finish(m, outs, m.d_scalars, nmatches);
}

int orbmi_search_by_projection_last_frame_if(orbmi_matcher* h, const orbmi_frame_view* cf, const uint8_t* occupied,
                                             const orbmi_frame_view* lf, const orbmi_lastframe_point* lf_points,
                                             float th, int mono, int check_ori, int32_t* match_lf, int* nmatches_dev,
                                             int min_matches) {
    if (!h || !occupied || !match_lf || !lf || (lf->n > 0 && !lf_points) || !on_device(nmatches_dev)) return ORBMI_E_ARG;
    Matcher& m = h->m;
    ORBMI_HIP(hipSetDevice(m.device));
    m.arena_reset();
    DevFrame CF, LF;
    int rc;
    if ((rc = make_frame(m, cf, &CF, true))) return rc;
    if ((rc = make_frame(m, lf, &LF, true))) return rc;
    const uint8_t* d_occ = dev_in(m, occupied, (size_t)std::max(CF.n, 1), &rc);
    const orbmi_lastframe_point* d_lfp = dev_in(m, lf_points, (size_t)LF.n, &rc);
    if (rc) return rc;
    std::vector<OutBuf> outs;
    int* d_out = dev_out(m, match_lf, (size_t)CF.n, outs);
    if ((rc = orbmi::launch_lastframe_search(m, CF, d_occ, LF, d_lfp, th, mono, check_ori, d_out, nmatches_dev,
                                             nmatches_dev, min_matches)))
        return rc;
    ORBMI_HIP(hipGetLastError());
    return finish(m, outs, nullptr, nullptr);
}

int orbmi_track_update_matches(orbmi_matcher* h, const orbmi_frame_view* f, int stage, const uint8_t* outlier,
                               const orbmi_frame_mappoints* mp, uint8_t* occupied_out, int* counts) {
    if (!h || !f || !outlier || !mp || !counts || (stage != 0 && stage != 1)) return ORBMI_E_ARG;
    if ((mp->match_lf && (!mp->lf_points || mp->n_lf_points < 0)) || (mp->match_mp && (!mp->mps || mp->n_mps < 0)))
        return ORBMI_E_ARG;
    Matcher& m = h->m;
    ORBMI_HIP(hipSetDevice(m.device));
    m.arena_reset();
    DevFrame F;
    int rc;
    if ((rc = make_frame(m, f, &F, false))) return rc;
    // the match arrays are updated in place: host arrays go through the arena and back
    std::vector<OutBuf> outs;
    const size_t n = (size_t)std::max(F.n, 1);
    int* d_lf = nullptr;
    int* d_mp = nullptr;
    if (mp->match_lf) {
        d_lf = const_cast<int*>(dev_in(m, (const int*)mp->match_lf, n, &rc));
        if (!on_device(mp->match_lf)) outs.push_back(OutBuf{mp->match_lf, d_lf, n * sizeof(int)});
    }
    if (mp->match_mp) {
        d_mp = const_cast<int*>(dev_in(m, (const int*)mp->match_mp, n, &rc));
        if (!on_device(mp->match_mp)) outs.push_back(OutBuf{mp->match_mp, d_mp, n * sizeof(int)});
    }
    const uint8_t* d_outl = dev_in(m, outlier, n, &rc);
    const orbmi_lastframe_point* d_lfp = mp->match_lf ? dev_in(m, mp->lf_points, (size_t)mp->n_lf_points, &rc) : nullptr;
    const orbmi_mappoint* d_mps = mp->match_mp ? dev_in(m, mp->mps, (size_t)mp->n_mps, &rc) : nullptr;
    if (rc) return rc;
    uint8_t* d_occ = occupied_out ? dev_out(m, occupied_out, n, outs) : nullptr;
    int* d_cnt = dev_out(m, counts, 2, outs);
    if ((rc = orbmi::launch_track_update(m, F, stage, d_outl, d_lf, d_lfp, mp->n_lf_points, d_mp, d_mps,
                                                mp->n_mps, d_occ, d_cnt))) return rc;
    ORBMI_HIP(hipGetLastError());
    return finish(m, outs, nullptr, nullptr);
}

int orbmi_search_by_bow(orbmi_matcher* h, const orbmi_frame_view* kf, const uint8_t* kf_mp_ok,
                        const orbmi_feature_vector* kf_fv, const orbmi_frame_view* f,
                        const orbmi_feature_vector* f_fv, float nnratio, int check_ori, int32_t* match_kf,
                        int* nmatches) {
    if (!h || !kf_mp_ok || !match_kf) return ORBMI_E_ARG;
    Matcher& m = h->m;
    ORBMI_HIP(hipSetDevice(m.device));
    m.arena_reset();
    DevFrame KF, F;
    DevFV kfv, fv;
    int rc;
    if ((rc = make_frame(m, kf, &KF, false))) return rc;
    if ((rc = make_frame(m, f, &F, false))) return rc;
    if ((rc = make_fv(m, kf_fv, &kfv))) return rc;
    if ((rc = make_fv(m, f_fv, &fv))) return rc;
    const uint8_t* d_ok = dev_in(m, kf_mp_ok, (size_t)std::max(KF.n, 1), &rc);
    if (rc) return rc;
    if ((rc = scalars(m))) return rc;
    std::vector<OutBuf> outs;
    int* d_out = dev_out(m, match_kf, (size_t)F.n, outs);
    if ((rc = orbmi::launch_bow(m, KF, d_ok, kfv, F, fv, nnratio, check_ori, d_out, m.d_scalars))) return rc;
    ORBMI_HIP(hipGetLastError());
    return finish(m, outs, m.d_scalars, nmatches);
}

int orbmi_match_descriptors_segments(orbmi_matcher* h, const uint8_t* q_desc, int nq, const int* nq_device,
                                     const uint8_t* train_desc, int nseg, int seg_capacity, const int* seg_counts,
                                     int skip_seg, int th, float ratio, int32_t* match, int* nmatches) {
    if (!h || nq < 0 || nseg < 0 || seg_capacity < 0 || (nq > 0 && (!q_desc || !match))) return ORBMI_E_ARG;
    if ((long long)nseg * seg_capacity > 0xFFFFFFFLL) return ORBMI_E_UNSUPPORTED;
    if (nseg * seg_capacity > 0 && (!train_desc || !seg_counts)) return ORBMI_E_ARG;
    if (nq_device && !on_device(nq_device)) return ORBMI_E_ARG;
    Matcher& m = h->m;
    ORBMI_HIP(hipSetDevice(m.device));
    m.arena_reset();
    int rc = 0;
    const uint8_t* d_q = dev_in(m, q_desc, (size_t)nq * 32, &rc);
    const uint8_t* d_t = dev_in(m, train_desc, (size_t)nseg * seg_capacity * 32, &rc);
    const int* d_cnt = dev_in(m, seg_counts, (size_t)nseg, &rc);
    if (rc) return rc;
    if ((rc = scalars(m))) return rc;
    std::vector<OutBuf> outs;
    int* d_out = dev_out(m, match, (size_t)nq, outs);
    if (nseg * seg_capacity == 0 && nq > 0) ORBMI_HIP(hipMemsetAsync(d_out, 0xFF, (size_t)nq * sizeof(int), m.ls()));
    else if ((rc = orbmi::launch_xmatch(m, d_q, nq, nq_device, d_t, nseg, seg_capacity, d_cnt, skip_seg, th, ratio,
                                        d_out, m.d_scalars)))
        return rc;
    ORBMI_HIP(hipGetLastError());
    return finish(m, outs, m.d_scalars, nmatches);
}

int orbmi_compute_distinctive_descriptors(orbmi_matcher* h, const uint8_t* obs_desc, const int32_t* obs_off, int np,
                                          int32_t* best, uint8_t* desc_out) {
    if (!h || np < 0 || (np > 0 && (!obs_off || !best || !desc_out))) return ORBMI_E_ARG;
    if (np == 0) return ORBMI_OK;
    Matcher& m = h->m;
    ORBMI_HIP(hipSetDevice(m.device));
    m.arena_reset();
    // the row count is needed only to stage host descriptors (a device array is used in place)
    int total = 0;
    const bool desc_dev = on_device(obs_desc);
    if (!desc_dev) {
        if (on_device(obs_off)) ORBMI_HIP(hipMemcpy(&total, obs_off + np, sizeof(int), hipMemcpyDeviceToHost));
        else total = obs_off[np];
        if (total < 0 || (total > 0 && !obs_desc)) return ORBMI_E_ARG;
    }
    int rc = 0;
    const uint8_t* d_desc = desc_dev ? obs_desc : dev_in(m, obs_desc, (size_t)total * 32, &rc);
    const int* d_off = dev_in(m, obs_off, (size_t)np + 1, &rc);
    if (rc) return rc;
    std::vector<OutBuf> outs;
    int* d_best = dev_out(m, best, (size_t)np, outs);
    uint8_t* d_out = dev_out(m, desc_out, (size_t)np * 32, outs);
    if (!on_device(desc_out)) ORBMI_HIP(m.h2d(d_out, desc_out, (size_t)np * 32));
    if ((rc = orbmi::launch_distinctive(m, d_desc, d_off, np, d_best, d_out))) return rc;
    return finish(m, outs, nullptr, nullptr);
}

int orbmi_search_for_triangulation(orbmi_matcher* h, const orbmi_frame_view* kf1, const uint8_t* has_mp1,
                                   const orbmi_feature_vector* fv1, const orbmi_frame_view* kf2, const uint8_t* has_mp2,
                                   const orbmi_feature_vector* fv2, const float* F12, int only_stereo, int check_ori,
                                   int32_t* match12, int* nmatches) {
    if (!kf2 || !has_mp2 || !fv2 || !F12) return ORBMI_E_ARG;
    const uint8_t* mp2[1] = {has_mp2};
    return orbmi_search_for_triangulation_batch(h, kf1, has_mp1, fv1, 1, kf2, mp2, fv2, F12, only_stereo, check_ori,
                                                match12, nmatches);
}

int orbmi_search_for_triangulation_batch(orbmi_matcher* h, const orbmi_frame_view* kf1, const uint8_t* has_mp1,
                                         const orbmi_feature_vector* fv1, int npairs, const orbmi_frame_view* kf2,
                                         const uint8_t* const* has_mp2, const orbmi_feature_vector* fv2,
                                         const float* F12, int only_stereo, int check_ori, int32_t* match12,
                                         int* nmatches) {
    if (!h || !has_mp1 || !fv1 || !kf1 || !kf1->u_right || npairs < 0 || (npairs > 0 && (!kf2 || !has_mp2 || !fv2 ||
                                                                                      !F12 || !match12)))
        return ORBMI_E_ARG;
    if (npairs == 0) return ORBMI_OK;
    Matcher& m = h->m;
    ORBMI_HIP(hipSetDevice(m.device));
    m.arena_reset();
    DevFrame K1;
    DevFV f1;
    int rc;
    if ((rc = make_frame(m, kf1, &K1, true))) return rc;
    if ((rc = make_fv(m, fv1, &f1))) return rc;
    const uint8_t* d_mp1 = dev_in(m, has_mp1, (size_t)std::max(K1.n, 1), &rc);
    if (rc) return rc;
    std::vector<TriPair> pairs(npairs);
    const bool F_dev = on_device(F12);
    std::vector<float> Fh((size_t)9 * npairs);
    if (F_dev) ORBMI_HIP(hipMemcpy(Fh.data(), F12, Fh.size() * sizeof(float), hipMemcpyDeviceToHost));
    else memcpy(Fh.data(), F12, Fh.size() * sizeof(float));
    int* d_counts = nullptr;
    if (nmatches) d_counts = (int*)m.stage((size_t)npairs * sizeof(int));
    for (int j = 0; j < npairs; j++) {
        TriPair& P = pairs[j];
        memset(&P, 0, sizeof(P));
        if (!kf2[j].u_right || !has_mp2[j]) return ORBMI_E_ARG;
        if ((rc = make_frame(m, &kf2[j], &P.KF2, true))) return rc;
        if ((rc = make_fv(m, &fv2[j], &P.fv2))) return rc;
        P.has_mp2 = dev_in(m, has_mp2[j], (size_t)std::max(P.KF2.n, 1), &rc);
        if (rc) return rc;
        for (int q = 0; q < 9; q++) P.F12.m[q] = Fh[9 * j + q];
        P.nmatches = d_counts ? d_counts + j : nullptr;
    }
    TriPair* d_pairs = (TriPair*)m.stage(sizeof(TriPair) * npairs);
    std::vector<OutBuf> outs;
    int* d_out = dev_out(m, match12, (size_t)K1.n * npairs, outs);
    if (!d_pairs || !d_out) return ORBMI_E_HIP;
    if ((rc = orbmi::launch_triangulation(m, K1, d_mp1, f1, npairs, pairs.data(), d_pairs, only_stereo, check_ori,
                                          d_out)))
        return rc;
    bool wait = false;
    ORBMI_HIP(m.flush_up());
    if (m.up_err != hipSuccess) return ORBMI_E_HIP;
    for (OutBuf& o : outs)
        if (o.bytes) { ORBMI_HIP(m.d2h(o.user, o.dev, o.bytes)); wait = true; }
    if (nmatches) {
        ORBMI_HIP(m.d2h(nmatches, d_counts, (size_t)npairs * sizeof(int)));
        wait = true;
    }
    if (wait) ORBMI_HIP(hipStreamSynchronize(m.ls()));
    m.d2h_flush();
    return ORBMI_OK;
}

int orbmi_create_new_map_points(orbmi_matcher* h, const orbmi_frame_view* kf1, const orbmi_tri_keyframe* tri1,
                                const float* cos1, const uint8_t* has_mp1, const orbmi_feature_vector* fv1,
                                int npairs, const orbmi_frame_view* kf2, const orbmi_tri_keyframe* tri2,
                                const float* const* cos2, const uint8_t* const* has_mp2,
                                const orbmi_feature_vector* fv2, const float* F12, int32_t* match12, uint8_t* ok,
                                float* x3d) {
    if (!h || !kf1 || !tri1 || !has_mp1 || !fv1 || !kf1->u_right || npairs < 0 ||
        (npairs > 0 && (!kf2 || !tri2 || !has_mp2 || !fv2 || !F12 || !match12 || !ok || !x3d)))
        return ORBMI_E_ARG;
    if (npairs == 0) return ORBMI_OK;
    Matcher& m = h->m;
    ORBMI_HIP(hipSetDevice(m.device));
    m.arena_reset();
    DevFrame K1;
    DevFV f1;
    int rc;
    if ((rc = make_frame(m, kf1, &K1, true))) return rc;
    if ((rc = make_fv(m, fv1, &f1))) return rc;
    const size_t n1 = (size_t)std::max(K1.n, 1);
    const uint8_t* has1 = dev_in(m, has_mp1, n1, &rc);
    if (rc) return rc;
    std::vector<std::vector<float>> cos_tmp;  // tables computed here, alive until the copies ran
    cos_tmp.reserve((size_t)npairs + 1);
    // the triangulation side of a keyframe: keys / u_right from its frame view (device), the rest
    // from its tri view
    auto side = [&](const orbmi_tri_keyframe* T, const orbmi_frame_view* v, const DevFrame& D, const float* cs,
                    orbmi::tri::Side* S) -> int {
        if (!T->tcw || !T->depth || !T->level_sigma2 || !T->scale_factors || on_device(T->level_sigma2) ||
            on_device(T->scale_factors) || v->nlevels > orbmi::tri::kLevels)
            return ORBMI_E_ARG;
        orbmi::tri::make_side(*T, v->nlevels, S);
        S->keys = D.keys;
        S->ur = D.u_right;
        int r = 0;
        S->depth = dev_in(m, T->depth, (size_t)D.n, &r);
        if (r) return r;
        if (!cs) {
            if (on_device(T->depth)) return ORBMI_E_ARG;
            cos_tmp.emplace_back((size_t)std::max(D.n, 1));
            if ((r = orbmi_stereo_parallax_cos(T->mb, T->depth, D.n, cos_tmp.back().data()))) return r;
            cs = cos_tmp.back().data();
        }
        S->cos_stereo = dev_in(m, cs, (size_t)D.n, &r);
        return r;
    };
    orbmi::tri::Side S1;
    if ((rc = side(tri1, kf1, K1, cos1, &S1))) return rc;
    std::vector<orbmi::tri::Side> S2(npairs);
    std::vector<TriPair> pairs(npairs);
    const bool F_dev = on_device(F12);
    std::vector<float> Fh((size_t)9 * npairs);
    if (F_dev) ORBMI_HIP(hipMemcpy(Fh.data(), F12, Fh.size() * sizeof(float), hipMemcpyDeviceToHost));
    else memcpy(Fh.data(), F12, Fh.size() * sizeof(float));
    for (int j = 0; j < npairs; j++) {
        TriPair& P = pairs[j];
        memset(&P, 0, sizeof(P));
        if (!kf2[j].u_right || !has_mp2[j]) return ORBMI_E_ARG;
        if ((rc = make_frame(m, &kf2[j], &P.KF2, true))) return rc;
        if ((rc = make_fv(m, &fv2[j], &P.fv2))) return rc;
        P.has_mp2 = dev_in(m, has_mp2[j], (size_t)std::max(P.KF2.n, 1), &rc);
        if (rc) return rc;
        for (int q = 0; q < 9; q++) P.F12.m[q] = Fh[9 * j + q];
        if ((rc = side(&tri2[j], &kf2[j], P.KF2, cos2 ? cos2[j] : nullptr, &S2[j]))) return rc;
    }
    std::vector<OutBuf> outs;
    int* d_match = dev_out(m, match12, (size_t)K1.n * npairs, outs);
    uint8_t* d_ok = dev_out(m, ok, (size_t)K1.n * npairs, outs);
    float* d_x3d = dev_out(m, x3d, (size_t)3 * K1.n * npairs, outs);
    if (!d_match || !d_ok || !d_x3d) return ORBMI_E_HIP;
    if ((rc = orbmi::tri_pairs_prepare(m, K1, npairs, pairs.data(), d_match))) return rc;
    // the pair table and the KF2 sides go up in one copy
    const size_t o_s2 = (sizeof(TriPair) * npairs + 255) & ~(size_t)255;
    const size_t tab_bytes = o_s2 + sizeof(orbmi::tri::Side) * npairs;
    std::vector<uint8_t> tab(tab_bytes);
    memcpy(tab.data(), pairs.data(), sizeof(TriPair) * npairs);
    memcpy(tab.data() + o_s2, S2.data(), sizeof(orbmi::tri::Side) * npairs);
    uint8_t* d_tab = (uint8_t*)m.stage(tab_bytes);
    if (!d_tab) return ORBMI_E_HIP;
    ORBMI_HIP(m.h2d(d_tab, tab.data(), tab_bytes));
    TriPair* d_pairs = (TriPair*)d_tab;
    const orbmi::tri::Side* d_S2 = (const orbmi::tri::Side*)(d_tab + o_s2);
    if ((rc = orbmi::launch_create_points(m, K1, has1, f1, npairs, nullptr, d_pairs, S1, d_S2, d_match, d_ok, d_x3d)))
        return rc;
    return finish(m, outs, nullptr, nullptr);
}

int orbmi_fuse_search(orbmi_matcher* h, const orbmi_frame_view* kf, const orbmi_mappoint* mps, const uint8_t* in_kf,
                      int n_mp, float th, int32_t* best_idx, int32_t* best_dist, int* ncandidates) {
    if (!h || !kf || n_mp < 0 || (n_mp > 0 && (!mps || !best_idx || !best_dist))) return ORBMI_E_ARG;
    Matcher& m = h->m;
    ORBMI_HIP(hipSetDevice(m.device));
    m.arena_reset();
    DevFrame F;
    int rc;
    if ((rc = make_frame(m, kf, &F, true))) return rc;
    const orbmi_mappoint* d_mps = dev_in(m, mps, (size_t)n_mp, &rc);
    const uint8_t* d_in = dev_in(m, in_kf, in_kf ? (size_t)std::max(n_mp, 1) : 0, &rc);
    if (rc) return rc;
    if (ncandidates && (rc = scalars(m))) return rc;  // the count only when asked for
    std::vector<OutBuf> outs;
    int* d_bi = dev_out(m, best_idx, (size_t)n_mp, outs);
    int* d_bd = dev_out(m, best_dist, (size_t)n_mp, outs);
    int* d_cnt = ncandidates ? m.d_scalars : nullptr;
    if ((rc = orbmi::launch_fuse(m, F, d_mps, d_in, n_mp, th, d_bi, d_bd, d_cnt))) return rc;
    return finish(m, outs, d_cnt, ncandidates);
}

int orbmi_fuse_search_batch(orbmi_matcher* h, int nkf, const orbmi_frame_view* kfs, const orbmi_mappoint* mps,
                            const uint8_t* in_kf, int n_mp, float th, int32_t* best_idx, int32_t* best_dist,
                            int* ncandidates) {
    if (!h || nkf < 0 || n_mp < 0 || (nkf > 0 && !kfs) || (nkf > 0 && n_mp > 0 && (!mps || !best_idx || !best_dist)))
        return ORBMI_E_ARG;
    if (nkf == 0) return ORBMI_OK;
    Matcher& m = h->m;
    ORBMI_HIP(hipSetDevice(m.device));
    m.arena_reset();
    int rc = 0;
    std::vector<FuseKF> K(nkf);
    const orbmi_mappoint* d_mps = dev_in(m, mps, (size_t)n_mp, &rc);
    const uint8_t* d_in = dev_in(m, in_kf, in_kf ? (size_t)std::max(n_mp, 1) * nkf : 0, &rc);
    if (rc) return rc;
    for (int k = 0; k < nkf; k++) {
        memset(&K[k], 0, sizeof(FuseKF));
        if ((rc = make_frame(m, &kfs[k], &K[k].F, true))) return rc;
        K[k].in_kf = d_in ? d_in + (size_t)k * n_mp : nullptr;
    }
    FuseKF* d_k = (FuseKF*)m.stage(sizeof(FuseKF) * nkf);
    int* d_cnt = (int*)m.stage(sizeof(int) * nkf);
    std::vector<OutBuf> outs;
    int* d_bi = dev_out(m, best_idx, (size_t)n_mp * nkf, outs);
    int* d_bd = dev_out(m, best_dist, (size_t)n_mp * nkf, outs);
    if (!d_k || !d_cnt) return ORBMI_E_HIP;
    if ((rc = orbmi::launch_fuse_multi(m, nkf, K.data(), d_k, d_mps, n_mp, th, d_bi, d_bd, d_cnt))) return rc;
    bool wait = false;
    ORBMI_HIP(m.flush_up());
    if (m.up_err != hipSuccess) return ORBMI_E_HIP;
    for (OutBuf& o : outs)
        if (o.bytes) { ORBMI_HIP(m.d2h(o.user, o.dev, o.bytes)); wait = true; }
    if (ncandidates) {
        ORBMI_HIP(m.d2h(ncandidates, d_cnt, sizeof(int) * nkf));
        wait = true;
    }
    if (wait) ORBMI_HIP(hipStreamSynchronize(m.ls()));
    m.d2h_flush();
    return ORBMI_OK;
}

int orbmi_fuse_search_refresh(orbmi_matcher* h, const uint8_t* obs_desc, const int32_t* obs_off, int nd, int32_t* best,
                              uint8_t* desc_out, int nkf, const orbmi_frame_view* kfs, const orbmi_mappoint* mps,
                              const int32_t* desc_from, const uint8_t* in_kf, int n_mp, float th, int32_t* best_idx,
                              int32_t* best_dist) {
    if (!h || nd < 0 || nkf < 0 || n_mp < 0 || (nd > 0 && (!obs_off || !best || !desc_out)) ||
        (nkf > 0 && !kfs) || (nkf > 0 && n_mp > 0 && (!mps || !best_idx || !best_dist)))
        return ORBMI_E_ARG;
    Matcher& m = h->m;
    ORBMI_HIP(hipSetDevice(m.device));
    m.arena_reset();
    int rc = 0;
    std::vector<OutBuf> outs;
    // ComputeDistinctiveDescriptors of the nd due points
    uint8_t* d_dout = nullptr;
    if (nd > 0) {
        int total = 0;
        if (on_device(obs_off)) ORBMI_HIP(hipMemcpy(&total, obs_off + nd, sizeof(int), hipMemcpyDeviceToHost));
        else total = obs_off[nd];
        if (total < 0 || (total > 0 && !obs_desc)) return ORBMI_E_ARG;
        const uint8_t* d_desc = dev_in(m, obs_desc, (size_t)total * 32, &rc);
        const int* d_off = dev_in(m, obs_off, (size_t)nd + 1, &rc);
        if (rc) return rc;
        int* d_best = dev_out(m, best, (size_t)nd, outs);
        d_dout = dev_out(m, desc_out, (size_t)nd * 32, outs);
        if (!on_device(desc_out))
            ORBMI_HIP(m.h2d(d_dout, desc_out, (size_t)nd * 32));
        if ((rc = orbmi::launch_distinctive(m, d_desc, d_off, nd, d_best, d_dout))) return rc;
    }
    // the Fuse searches on records patched with the new descriptors
    if (nkf > 0 && n_mp > 0) {
        orbmi_mappoint* d_mps = (orbmi_mappoint*)m.stage(sizeof(orbmi_mappoint) * n_mp);
        if (!d_mps) return ORBMI_E_HIP;
        if (on_device(mps))
            ORBMI_HIP(hipMemcpyAsync(d_mps, mps, sizeof(orbmi_mappoint) * n_mp, hipMemcpyDeviceToDevice, m.ls()));
        else
            ORBMI_HIP(m.h2d(d_mps, mps, sizeof(orbmi_mappoint) * n_mp));
        if (desc_from && nd > 0) {
            const int* d_from = dev_in(m, desc_from, (size_t)n_mp, &rc);
            if (rc) return rc;
            if ((rc = orbmi::launch_patch_desc(m, d_mps, d_from, d_dout, n_mp))) return rc;
        }
        const uint8_t* d_in = dev_in(m, in_kf, in_kf ? (size_t)n_mp * nkf : 0, &rc);
        if (rc) return rc;
        std::vector<FuseKF> K(nkf);
        for (int k = 0; k < nkf; k++) {
            memset(&K[k], 0, sizeof(FuseKF));
            if ((rc = make_frame(m, &kfs[k], &K[k].F, true))) return rc;
            K[k].in_kf = d_in ? d_in + (size_t)k * n_mp : nullptr;
        }
        FuseKF* d_k = (FuseKF*)m.stage(sizeof(FuseKF) * nkf);
        int* d_cnt = (int*)m.stage(sizeof(int) * nkf);
        int* d_bi = dev_out(m, best_idx, (size_t)n_mp * nkf, outs);
        int* d_bd = dev_out(m, best_dist, (size_t)n_mp * nkf, outs);
        if (!d_k || !d_cnt) return ORBMI_E_HIP;
        if ((rc = orbmi::launch_fuse_multi(m, nkf, K.data(), d_k, d_mps, n_mp, th, d_bi, d_bd, d_cnt))) return rc;
    }
    return finish(m, outs, nullptr, nullptr);
}

int orbmi_debug_greedy_stats(unsigned long long* out, int reset) {
    if (!out) return ORBMI_E_ARG;
    return orbmi::greedy_stats(out, reset);
}

int orbmi_debug_greedy_cycles(unsigned long long* out, int reset) {
    if (!out) return ORBMI_E_ARG;
    return orbmi::greedy_cycles(out, reset);
}

}  // extern "C"
