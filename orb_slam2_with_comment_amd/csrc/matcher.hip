// ORBmatcher on MI355X (src/ORBmatcher.cc):
//   k_grid_build        Frame::AssignFeaturesToGrid (src/Frame.cc:232-247)        one workgroup
//   k_frustum           Frame::isInFrustum + MapPoint::PredictScale               thread / point
//   k_candidates<G>     SearchByProjection(F, MPs) / (CF, LF): window + static filters + Hamming,
//                       G lanes per query (map point / LF keypoint), sorted top-8 prefix
//   k_greedy            exact greedy replay of the order-dependent exclusion           one workgroup
//   k_bow_*             SearchByBoW: node merge-join + per-node greedy (one wave / node)
//   k_xmatch_*          cross-stream brute-force matching of config 4 (build-defined)
//
// Candidate order.  GetFeaturesInArea visits cells ix-major, iy-minor, keypoints in index
// order inside a cell, so the reference's candidate order is the lexicographic order of
// (cell ix*48+iy, keypoint index).  Entries are packed as dist<<40 | cellorder<<20 | idx and
// "first minimum in visit order" becomes a plain u64 minimum, independent of how the grid
// lists were filled.  The second best (bestDist2/bestLevel2 of :124-137) is the minimum entry
// once the best entry is excluded.
//
// Greedy exclusion.  Query q may not take a keypoint already matched by an earlier query whose
// map point has observations (:108-110, :1627-1629).  k_greedy iterates r_q = f(q, occ0 U
// {r_p : p < q}) to a fixpoint inside one workgroup: after round k every query whose
// dependency chain is <= k is final, and a fixpoint equals the sequential result by
// induction on q.  A bounded round count falls back to the sequential replay.
#include <algorithm>

#include <cstring>

#include "matcher.h"
#include "track_update.h"
#include "tri_geom.h"
#include "wave_ops.h"

namespace orbmi {

constexpr int kGridCols = 64, kGridRows = 48, kGridCells = kGridCols * kGridRows;
constexpr int TH_HIGH = 100, TH_LOW = 50, HISTO_LENGTH = 30;


__device__ inline int popc_desc(const uint8_t* a, const uint8_t* b) {
    const uint4* x = reinterpret_cast<const uint4*>(a);
    const uint4* y = reinterpret_cast<const uint4*>(b);
    return popc256(x[0], x[1], y[0], y[1]);
}

// -------------------------------------------------------------------------- grid
__device__ inline void grid_build_block(const DevFrame& F, int* __restrict__ cell_start, int* __restrict__ cell_list,
                                        int* __restrict__ kp_cell) {
    __shared__ int cnt[kGridCells + 1];
    __shared__ int scratch[20];
    const int tid = threadIdx.x;
    for (int i = tid; i < kGridCells; i += blockDim.x) cnt[i] = 0;
    __syncthreads();
    const int n = frame_n(F);
    for (int i = tid; i < n; i += blockDim.x) {
        const orbmi_keypoint kp = F.keys[i];
        const int px = (int)roundf((kp.x - F.min_x) * F.grid_w_inv);
        const int py = (int)roundf((kp.y - F.min_y) * F.grid_h_inv);
        int c = -1;
        if (!(px < 0 || px >= kGridCols || py < 0 || py >= kGridRows)) { c = px * kGridRows + py; atomicAdd(&cnt[c], 1); }
        kp_cell[i] = c;
    }
    __syncthreads();
    int v[3], s = 0;
    for (int k = 0; k < 3; k++) { v[k] = cnt[tid * 3 + k]; s += v[k]; }  // 1024*3 == kGridCells
    int total;
    int e = block_excl_scan(s, scratch, &total);
    for (int k = 0; k < 3; k++) { cell_start[tid * 3 + k] = e; cnt[tid * 3 + k] = e; e += v[k]; }
    if (tid == 0) cell_start[kGridCells] = total;
    __syncthreads();
    for (int i = tid; i < n; i += blockDim.x) {
        const int c = kp_cell[i];
        if (c >= 0) cell_list[atomicAdd(&cnt[c], 1)] = i;
    }
}

__global__ __launch_bounds__(1024) void k_grid_build(DevFrame F, int* __restrict__ cell_start,
                                                     int* __restrict__ cell_list, int* __restrict__ kp_cell,
                                                     const int* gate, int gate_min) {
    if (gate && *gate >= gate_min) return;
    grid_build_block(F, cell_start, cell_list, kp_cell);
}

// the grids of several keyframes (one workgroup each; keyframe k's arrays at k * stride)
__global__ __launch_bounds__(1024) void k_grid_build_multi(const FuseKF* __restrict__ kfs, int* __restrict__ kp_cell,
                                                           int ncap) {
    const FuseKF& K = kfs[blockIdx.x];
    if (threadIdx.x == 0) *K.ncand = 0;  // k_fuse_multi counts into it behind this launch
    grid_build_block(K.F, const_cast<int*>(K.cs), const_cast<int*>(K.cl), kp_cell + (size_t)blockIdx.x * ncap);
}

// Frame::GetFeaturesInArea (src/Frame.cc:353-410): calls fn(idx) for every keypoint in the
// window passing the level filter, in arbitrary order.
template <int G = 1, class Fn>
__device__ inline void for_features_in_area(const DevFrame& F, const int* cell_start, const int* cell_list,
                                            float x, float y, float r, int minLevel, int maxLevel, int glane, Fn fn) {
    const int nMinCellX = max(0, (int)floorf((x - F.min_x - r) * F.grid_w_inv));
    if (nMinCellX >= kGridCols) return;
    const int nMaxCellX = min(kGridCols - 1, (int)ceilf((x - F.min_x + r) * F.grid_w_inv));
    if (nMaxCellX < 0) return;
    const int nMinCellY = max(0, (int)floorf((y - F.min_y - r) * F.grid_h_inv));
    if (nMinCellY >= kGridRows) return;
    const int nMaxCellY = min(kGridRows - 1, (int)ceilf((y - F.min_y + r) * F.grid_h_inv));
    if (nMaxCellY < 0) return;
    const bool bCheckLevels = (minLevel > 0) || (maxLevel >= 0);
    const int ny = nMaxCellY - nMinCellY + 1, ncell = (nMaxCellX - nMinCellX + 1) * ny;
    for (int ci = glane; ci < ncell; ci += G) {  // G = 1: ix-major, iy-minor (the visit order)
        const int c = (nMinCellX + ci / ny) * kGridRows + nMinCellY + ci % ny;
        for (int j = cell_start[c]; j < cell_start[c + 1]; j++) {
            const int idx = cell_list[j];
            const orbmi_keypoint kp = F.keys[idx];
            if (bCheckLevels) {
                if (kp.octave < minLevel) continue;
                if (maxLevel >= 0 && kp.octave > maxLevel) continue;
            }
            const float distx = kp.x - x, disty = kp.y - y;
            if (fabsf(distx) < r && fabsf(disty) < r) fn(idx, c);
        }
    }
}
template <class Fn>
__device__ inline void for_features_in_area(const DevFrame& F, const int* cell_start, const int* cell_list,
                                            float x, float y, float r, int minLevel, int maxLevel, Fn fn) {
    for_features_in_area<1>(F, cell_start, cell_list, x, y, r, minLevel, maxLevel, 0, fn);
}

__device__ inline unsigned long long cand_entry(int dist, int cell, int idx) {
    return ((unsigned long long)dist << 40) | ((unsigned long long)cell << 20) | (unsigned)idx;
}

// R*p + t, float, left to right (pinned P10: cv::gemm small-matrix path)
__device__ inline void transform(const float* T, const float* p, float* o) {
#pragma unroll
    for (int r = 0; r < 3; r++) o[r] = ((T[4 * r] * p[0] + T[4 * r + 1] * p[1]) + T[4 * r + 2] * p[2]) + T[4 * r + 3];
}
__device__ inline void camera_center(const float* T, float* o) {
#pragma unroll
    for (int c = 0; c < 3; c++) o[c] = -((T[c] * T[3] + T[4 + c] * T[7]) + T[8 + c] * T[11]);
}

// -------------------------------------------------------------------------- frustum
__global__ __launch_bounds__(256) void k_frustum(DevFrame F, const orbmi_mappoint* __restrict__ mps, int n,
                                                 float viewingCosLimit, orbmi_mappoint_track* __restrict__ tr,
                                                 int* __restrict__ n_in_view) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    orbmi_mappoint_track t = {0, 0.f, 0.f, 0.f, 0, 0.f};
    const orbmi_mappoint mp = mps[i];
    bool ok = !(mp.flags & (ORBMI_MP_BAD | ORBMI_MP_SEEN));
    float Pc[3], Ow[3], u = 0, v = 0, invz = 0, dist = 0, viewCos = 0;
    const Pose34 T = frame_pose(F);
    if (ok) {
        transform(T.m, mp.pos, Pc);
        ok = !(Pc[2] < 0.0f);
    }
    if (ok) {
        invz = 1.0f / Pc[2];
        u = F.fx * Pc[0] * invz + F.cx;
        v = F.fy * Pc[1] * invz + F.cy;
        ok = !(u < F.min_x || u > F.max_x) && !(v < F.min_y || v > F.max_y);
    }
    if (ok) {
        camera_center(T.m, Ow);
        const float maxDistance = 1.2f * mp.max_distance, minDistance = 0.8f * mp.min_distance;
        const float PO[3] = {mp.pos[0] - Ow[0], mp.pos[1] - Ow[1], mp.pos[2] - Ow[2]};
        dist = (float)sqrt((double)PO[0] * PO[0] + (double)PO[1] * PO[1] + (double)PO[2] * PO[2]);
        ok = !(dist < minDistance || dist > maxDistance);
        if (ok) {
            const double dot = (double)PO[0] * mp.normal[0] + (double)PO[1] * mp.normal[1] + (double)PO[2] * mp.normal[2];
            viewCos = (float)(dot / (double)dist);
            ok = !(viewCos < viewingCosLimit);
        }
    }
    if (ok) {
        const float ratio = mp.max_distance / dist;
        int nScale = (int)ceilf((float)log((double)ratio) / F.log_scale_factor);
        if (nScale < 0) nScale = 0;
        else if (nScale >= F.nlevels) nScale = F.nlevels - 1;
        t.in_view = 1;
        t.proj_x = u;
        t.proj_xr = u - F.bf * invz;
        t.proj_y = v;
        t.level = nScale;
        t.view_cos = viewCos;
        if (n_in_view) atomicAdd(n_in_view, 1);
    }
    tr[i] = t;
}

// -------------------------------------------------------------------------- candidates
// SearchByProjection(F, vpMapPoints, th): static part of the per-point search (:66-123).
__device__ inline bool local_query(const DevFrame& F, const orbmi_mappoint& mp, const orbmi_mappoint_track& t,
                                   float th, float* x, float* y, float* rs, int* level) {
    if (!t.in_view || (mp.flags & ORBMI_MP_BAD)) return false;
    float r = t.view_cos > 0.998 ? 2.5f : 4.0f;  // RadiusByViewingCos (:157-163)
    if (th != 1.0) r *= th;
    *level = t.level;
    *rs = r * F.scale[t.level];
    *x = t.proj_x;
    *y = t.proj_y;
    return true;
}

template <class Fn>
__device__ inline void local_candidates(const DevFrame& F, const int* cs, const int* cl, const orbmi_mappoint& mp,
                                        const orbmi_mappoint_track& t, float th, Fn emit) {
    float x, y, rs;
    int level;
    if (!local_query(F, mp, t, th, &x, &y, &rs, &level)) return;
    const uint8_t* md = mp.desc;
    for_features_in_area(F, cs, cl, x, y, rs, level - 1, level, [&](int idx, int cell) {
        if (F.u_right && F.u_right[idx] > 0) {
            const float er = fabsf(t.proj_xr - F.u_right[idx]);
            if (er > rs) return;
        }
        emit(cand_entry(popc_desc(md, F.desc + 32 * (long long)idx), cell, idx));
    });
}

// SearchByProjection(CF, LF, th, bMono): projection + static part (:1566-1637)
struct LfQuery {
    float u, v, radius, ur;
    int minL, maxL;
};

__device__ inline bool lf_query(const DevFrame& CF, const float* Tc, const DevFrame& LF, const orbmi_lastframe_point& p, int i,
                                float th, bool bForward, bool bBackward, LfQuery* q) {
    if (!(p.flags & ORBMI_LF_HAS_MP) || (p.flags & ORBMI_LF_OUTLIER)) return false;
    float x3Dc[3];
    transform(Tc, p.pos, x3Dc);
    const float xc = x3Dc[0], yc = x3Dc[1];
    const float invzc = (float)(1.0 / (double)x3Dc[2]);
    if (invzc < 0) return false;
    const float u = CF.fx * xc * invzc + CF.cx;
    const float v = CF.fy * yc * invzc + CF.cy;
    if (!(u >= CF.min_x && u <= CF.max_x)) return false;  // also rejects NaN (zc == 0)
    if (!(v >= CF.min_y && v <= CF.max_y)) return false;
    const int nLastOctave = LF.keys[i].octave;
    q->u = u;
    q->v = v;
    q->radius = th * CF.scale[nLastOctave];
    q->ur = u - CF.bf * invzc;
    if (bForward) { q->minL = nLastOctave; q->maxL = -1; }
    else if (bBackward) { q->minL = 0; q->maxL = nLastOctave; }
    else { q->minL = nLastOctave - 1; q->maxL = nLastOctave + 1; }
    return true;
}

template <class Fn>
__device__ inline void lf_candidates(const DevFrame& CF, const float* Tc, const DevFrame& LF, const int* cs, const int* cl,
                                     const orbmi_lastframe_point& p, int i, float th, bool fw, bool bw, Fn emit) {
    LfQuery q;
    if (!lf_query(CF, Tc, LF, p, i, th, fw, bw, &q)) return;
    for_features_in_area(CF, cs, cl, q.u, q.v, q.radius, q.minL, q.maxL, [&](int i2, int cell) {
        if (CF.u_right && CF.u_right[i2] > 0) {
            const float er = fabsf(q.ur - CF.u_right[i2]);
            if (er > q.radius) return;
        }
        emit(cand_entry(popc_desc(p.desc, CF.desc + 32 * (long long)i2), cell, i2));
    });
}

__device__ inline void motion_direction(const DevFrame& CF, const float* Tc, const DevFrame& LF, int mono, bool* fw,
                                        bool* bw) {
    float twc[3], tlc[3];
    const Pose34 Tl = frame_pose(LF);
    camera_center(Tc, twc);
    transform(Tl.m, twc, tlc);
    *fw = tlc[2] > CF.mb && !mono;
    *bw = -tlc[2] > CF.mb && !mono;
}

// -------------------------------------------------------------------------- group candidates
// G lanes per query: lanes take the window's grid cells (ix-major order does not matter: the
// entries carry their cell order), filter and score the cells' keypoints, append to an LDS
// list, then select the kTopK smallest entries in order.  The greedy pass usually finds its
// best and second best unclaimed entries in that prefix; the full list (or, past kCandCap,
// a re-enumeration) is the fallback.
constexpr int kTopK = 8;

struct CandArgs {
    int mode;  // 0 = local map (query = map point), 1 = last frame (query = LF keypoint)
    int nq;    // mode 0: number of map points; mode 1: LF capacity (count read on the device)
    DevFrame F, LF;
    const int* cs;
    const int* cl;
    const orbmi_mappoint* mps;
    const orbmi_mappoint_track* tr;
    const orbmi_lastframe_point* lfp;
    float th;
    int mono;
    unsigned long long* cand;
    int* ncand;
    unsigned long long* top;
    const int* gate;  // optional: the launch does nothing when *gate >= gate_min
    int gate_min;
};

struct Window {
    float x, y, r, ur;
    int minL, maxL;
    const uint8_t* desc;
};

__device__ inline bool make_window(const CandArgs& a, int q, const float* Tc, bool fw, bool bw, Window* w) {
    if (a.mode == 0) {
        const orbmi_mappoint& mp = a.mps[q];
        const orbmi_mappoint_track t = a.tr[q];
        int level;
        if (!local_query(a.F, mp, t, a.th, &w->x, &w->y, &w->r, &level)) return false;
        w->minL = level - 1;
        w->maxL = level;
        w->ur = t.proj_xr;
        w->desc = mp.desc;
        return true;
    }
    const orbmi_lastframe_point& p = a.lfp[q];
    LfQuery lq;
    if (!lf_query(a.F, Tc, a.LF, p, q, a.th, fw, bw, &lq)) return false;
    w->x = lq.u; w->y = lq.v; w->r = lq.radius; w->ur = lq.ur; w->minL = lq.minL; w->maxL = lq.maxL;
    w->desc = p.desc;
    return true;
}

template <int G>
__global__ __launch_bounds__(256) void k_candidates(CandArgs a) {
    constexpr int NG = 256 / G, cap = Matcher::kCandCap;
    __shared__ unsigned long long buf[NG][cap];
    __shared__ int cnt[NG];
    const int gl = threadIdx.x / G, lane = threadIdx.x % G;
    const int q = blockIdx.x * NG + gl;
    if (a.gate && *a.gate >= a.gate_min) return;  // orbmi_search_by_projection_last_frame_if
    const int nq = a.mode == 1 ? frame_n(a.LF) : a.nq;
    Pose34 Tc;
    bool fw = false, bw = false;
    if (a.mode == 1) {
        Tc = frame_pose(a.F);
        motion_direction(a.F, Tc.m, a.LF, a.mono, &fw, &bw);
    }
    Window w;
    const bool valid = q < nq && make_window(a, q, Tc.m, fw, bw, &w);
    if (lane == 0) cnt[gl] = 0;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    if (valid) {
        const DevFrame& F = a.F;
        const int nMinCellX = max(0, (int)floorf((w.x - F.min_x - w.r) * F.grid_w_inv));
        const int nMaxCellX = min(kGridCols - 1, (int)ceilf((w.x - F.min_x + w.r) * F.grid_w_inv));
        const int nMinCellY = max(0, (int)floorf((w.y - F.min_y - w.r) * F.grid_h_inv));
        const int nMaxCellY = min(kGridRows - 1, (int)ceilf((w.y - F.min_y + w.r) * F.grid_h_inv));
        if (nMinCellX < kGridCols && nMaxCellX >= 0 && nMinCellY < kGridRows && nMaxCellY >= 0) {
            const int ny = nMaxCellY - nMinCellY + 1, ncell = (nMaxCellX - nMinCellX + 1) * ny;
            const bool bCheckLevels = (w.minL > 0) || (w.maxL >= 0);
            const uint4* md = reinterpret_cast<const uint4*>(w.desc);
            const uint4 m0 = md[0], m1 = md[1];
            for (int ci = lane; ci < ncell; ci += G) {
                const int c = (nMinCellX + ci / ny) * kGridRows + nMinCellY + ci % ny;
                for (int j = a.cs[c]; j < a.cs[c + 1]; j++) {
                    const int idx = a.cl[j];
                    const orbmi_keypoint kp = F.keys[idx];
                    if (bCheckLevels) {
                        if (kp.octave < w.minL) continue;
                        if (w.maxL >= 0 && kp.octave > w.maxL) continue;
                    }
                    if (!(fabsf(kp.x - w.x) < w.r && fabsf(kp.y - w.y) < w.r)) continue;
                    if (F.u_right && F.u_right[idx] > 0 && fabsf(w.ur - F.u_right[idx]) > w.r) continue;
                    const uint4* fd = reinterpret_cast<const uint4*>(F.desc + 32 * (long long)idx);
                    const int pos = atomicAdd(&cnt[gl], 1);
                    if (pos < cap) buf[gl][pos] = cand_entry(popc256(m0, m1, fd[0], fd[1]), c, idx);
                }
            }
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int n = cnt[gl], nk = min(n, cap);
    // kTopK smallest entries, ascending (entries are distinct: one per keypoint)
    unsigned long long last = 0;
    for (int k = 0; k < kTopK; k++) {
        unsigned long long m = ~0ull;
        for (int p = lane; p < nk; p += G) {
            const unsigned long long e = buf[gl][p];
            if ((k == 0 || e > last) && e < m) m = e;
        }
        if constexpr (G == 16) {  // group = one DPP row: four DPP moves, no LDS permute round trips
            unsigned long long v;
            v = dpp_mov_u64<kDppXor1>(m); m = v < m ? v : m;
            v = dpp_mov_u64<kDppXor2>(m); m = v < m ? v : m;
            v = dpp_mov_u64<kDppHalfMirror>(m); m = v < m ? v : m;
            v = dpp_mov_u64<kDppRor8>(m); m = v < m ? v : m;
        } else {
#pragma unroll
            for (int o = G / 2; o > 0; o >>= 1) {
                const unsigned long long v = __shfl_xor(m, o, G);
                m = v < m ? v : m;
            }
        }
        if (valid && lane == 0) a.top[(long long)q * kTopK + k] = m;
        last = m;
    }
    if (valid && n > kTopK)
        for (int p = lane; p < nk; p += G) a.cand[(long long)q * cap + p] = buf[gl][p];
    if (q < nq && lane == 0) a.ncand[q] = valid ? n : 0;
}

// -------------------------------------------------------------------------- greedy
struct GreedyArgs {
    int mode;             // 0 = local map (best + ratio test), 1 = last frame (best + rotation)
    int nq;               // queries (map points / LF keypoints), processed in index order
    const unsigned long long* cand;
    const int* ncand;
    const unsigned long long* top;  // kTopK smallest entries per query, ascending
    int cap;
    const uint8_t* occ0;  // initial occupancy (F.mvpMapPoints[i] && Observations() > 0)
    DevFrame F;           // frame searched (CF)
    DevFrame LF;          // last frame (mode 1)
    const int* cs;
    const int* cl;
    const orbmi_mappoint* mps;              // mode 0
    const orbmi_mappoint_track* tr;         // mode 0
    const orbmi_lastframe_point* lfp;       // mode 1
    float th, nnratio;
    int mono, check_ori;
    int* res;             // per query: chosen keypoint or -1
    int* out;             // per keypoint result (see orbmi.h)
    int* nmatches;
    const int* gate;      // optional: nothing happens when *gate >= gate_min (may alias nmatches:
    int gate_min;         // read by every thread before the single write at the end)
};

constexpr int kGreedyMaxKp = 16384;
constexpr int kGreedyRounds = 48;

// Result of query q under occupancy test occ(idx) (sequential semantics of one iteration).
template <class Occ>
__device__ inline int greedy_eval(const GreedyArgs& a, int q, const float* Tc, bool fw, bool bw, Occ occ) {
    unsigned long long b1 = ~0ull, b2 = ~0ull;
    auto take = [&](unsigned long long e) {
        if (occ((int)(e & 0xFFFFF))) return;
        if (e < b1) { b2 = b1; b1 = e; }
        else if (e < b2) b2 = e;
    };
    const int nc = a.ncand[q];
    // sorted prefix first: the two smallest unclaimed entries are usually there
    const unsigned long long* t = a.top + (long long)q * kTopK;
    const int kk = nc <= a.cap ? min(nc, kTopK) : 0;  // past kCandCap the prefix is partial
    for (int k = 0; k < kk && b2 == ~0ull; k++) take(t[k]);
    if (b2 == ~0ull && nc > kTopK) {
        b1 = b2 = ~0ull;
        if (nc <= a.cap) {
            // the list in chunks of 16 loads in flight (one dependent load per entry made a
            // query's slow path, and the whole workgroup's round with it, ~100 load latencies)
            const unsigned long long* c = a.cand + (long long)q * a.cap;
            for (int k0 = 0; k0 < nc; k0 += 16) {
                unsigned long long e[16];
#pragma unroll
                for (int j = 0; j < 16; j++) e[j] = k0 + j < nc ? c[k0 + j] : ~0ull;
#pragma unroll
                for (int j = 0; j < 16; j++)
                    if (e[j] != ~0ull) take(e[j]);
            }
        } else if (a.mode == 0) {  // overflowed list: enumerate again
            local_candidates(a.F, a.cs, a.cl, a.mps[q], a.tr[q], a.th, take);
        } else {
            lf_candidates(a.F, Tc, a.LF, a.cs, a.cl, a.lfp[q], q, a.th, fw, bw, take);
        }
    }
    if (b1 == ~0ull) return -1;
    const int bestDist = (int)(b1 >> 40);
    const int bestIdx = (int)(b1 & 0xFFFFF);
    if (a.mode == 0) {
        if (bestDist > TH_HIGH) return -1;
        const int bestDist2 = b2 == ~0ull ? 256 : (int)(b2 >> 40);
        const int bestLevel = a.F.keys[bestIdx].octave;
        const int bestLevel2 = b2 == ~0ull ? -1 : a.F.keys[(int)(b2 & 0xFFFFF)].octave;
        if (bestLevel == bestLevel2 && bestDist > a.nnratio * bestDist2) return -1;
        return bestIdx;
    }
    return bestDist <= TH_HIGH ? bestIdx : -1;
}

__device__ inline bool query_has_obs(const GreedyArgs& a, int q) {
    return a.mode == 0 ? (a.mps[q].flags & ORBMI_MP_HAS_OBS) != 0 : (a.lfp[q].flags & ORBMI_MP_HAS_OBS) != 0;
}

__device__ inline int rot_bin(float a0, float a1) {
    const float factor = 1.0f / HISTO_LENGTH;
    float rot = a0 - a1;
    if (rot < 0.0) rot += 360.0f;
    int bin = (int)roundf(rot * factor);
    if (bin == HISTO_LENGTH) bin = 0;
    return bin;
}

// query verdict from the two smallest unclaimed entries (dist, idx); idx2 < 0 = none
__device__ inline int greedy_decide(const GreedyArgs& a, const uint8_t* oct, int d1, int i1, int d2, int i2) {
    if (i1 < 0) return -1;
    if (a.mode == 0) {
        if (d1 > TH_HIGH) return -1;
        const int bestDist2 = i2 < 0 ? 256 : d2;
        const int bestLevel2 = i2 < 0 ? -1 : oct[i2];
        if (oct[i1] == bestLevel2 && d1 > a.nnratio * bestDist2) return -1;
        return i1;
    }
    return d1 <= TH_HIGH ? i1 : -1;
}

#ifndef ORBMI_GREEDY_THREADS
#define ORBMI_GREEDY_THREADS 1024
#endif
constexpr int kGreedyThreads = ORBMI_GREEDY_THREADS, kGreedyQPer = 4096 / kGreedyThreads, kGreedyPre = 4;
constexpr int kGreedyQBits = 24;  // query index field of a claim
constexpr int kGreedyMaxQueries = 1 << kGreedyQBits;

// A prefix entry in a register: octave << 25 | dist << 16 | keypoint index (dist <= 256, index <
// kGreedyMaxKp, octave < kMaxLevels); kNoEntry = none
constexpr unsigned kNoEntry = ~0u;
__device__ inline int pe_idx(unsigned e) { return (int)(e & 0xFFFF); }
__device__ inline int pe_dist(unsigned e) { return (int)((e >> 16) & 0x1FF); }
__device__ inline int pe_oct(unsigned e) { return (int)(e >> 25); }

// greedy_decide on two prefix entries (the octaves travel with them: no LDS read)
__device__ inline int greedy_decide_pe(const GreedyArgs& a, unsigned e1, unsigned e2) {
    if (e1 == kNoEntry) return -1;
    const int d1 = pe_dist(e1);
    if (d1 > TH_HIGH) return -1;
    if (a.mode == 0 && e2 != kNoEntry && pe_oct(e1) == pe_oct(e2) && d1 > a.nnratio * pe_dist(e2)) return -1;
    return pe_idx(e1);
}

// k_greedy statistics (orbmi_debug_greedy_stats): calls, rounds summed, largest round count,
// slow-path query evaluations summed, calls that fell back to the sequential replay
__device__ unsigned long long g_greedy_stats[5];
__device__ int g_greedy_on;  // set by the first orbmi_debug_greedy_* call: statistics collected from then on
// development aid: s_memtime cycles of k_greedy's phases summed over calls (prologue, rounds,
// epilogue; thread 0's split of the rounds: claims + barrier, evaluation, flag + barrier), read by
// orbmi_debug_greedy_cycles
__device__ unsigned long long g_greedy_cycles[7];

// Each thread keeps its queries (q = tid + k * 1024) in registers: current result, candidate
// count and the first kGreedyPre sorted entries (pe_* packing, the keypoint's octave included);
// the initial occupancy lives in LDS.  A round then touches LDS only, except for queries whose
// prefix runs out of unclaimed entries (full list / re-enumeration).
// Claims carry the round: claim[i] = tag(r) | q with tag(r) = (64 - r) << 24 (an atomicMin keeps
// the current round's smallest query, and an older round's claim reads as free), 0 for a keypoint
// occupied on entry; so the array is set once, and a round is claims, a barrier, the evaluation,
// a barrier (the convergence flag alternates between two slots).  Query indices take the low 24
// bits (the launchers refuse nq >= 2^24), the round tag the 7 above them.
// The evaluation is branch-free selects over the prefix's claim words; the prologue is two
// dependent global round trips (gate, counts and poses; then every per-query and per-keypoint
// load at once); the epilogue aggregates the rotation histogram per wave and takes its three
// maxima with wave reductions.
__global__ __launch_bounds__(kGreedyThreads) void k_greedy(GreedyArgs a) {
    __shared__ int claim[kGreedyMaxKp];   // round-tagged min query index holding the keypoint;
                                          // afterwards the max query index assigned to it
    __shared__ uint8_t occ0[kGreedyMaxKp], oct[kGreedyMaxKp];  // occ0: afterwards "rejected"
    __shared__ int ovfres[kGreedyQPer * kGreedyThreads];       // overflowed queries' results
    __shared__ int hist[HISTO_LENGTH];
    __shared__ int flag[4];
    const unsigned long long c0 = __builtin_amdgcn_s_memtime();
    const int tid = threadIdx.x, lane = tid & 63;
    // round trip 1: the gate, the device-resident counts, the poses (mode 1).  The loads are
    // unconditional, through a.ncand (at least one entry, always allocated) where a pointer is
    // absent, so that they issue together (a branch per optional load serialises them).
    const int gv = *(a.gate ? a.gate : a.ncand);
    const int nFv = *(a.F.n_dev ? a.F.n_dev : a.ncand);
    const int nLv = *(a.mode == 1 && a.LF.n_dev ? a.LF.n_dev : a.ncand);
    bool fw = false, bw = false;
    Pose34 Tc;
    if (a.mode == 1) {
        Tc = frame_pose(a.F);
        motion_direction(a.F, Tc.m, a.LF, a.mono, &fw, &bw);
    }
    const bool ori = a.mode == 1 && a.check_ori;
    // the same round trip: the queries' counts, prefixes, observation flags (and LF angles), and
    // the keypoints' occupancy and octave, for every slot up to the arrays' capacities (the device
    // counts above are not known yet; indices clamped into range, slots past the counts unused)
    const int nCapF = a.F.n, nqCap = a.mode == 1 ? a.LF.n : a.nq;
    int res[kGreedyQPer], nc[kGreedyQPer];
    unsigned pre[kGreedyQPer][kGreedyPre];
    bool obs[kGreedyQPer];
    float angL[kGreedyQPer];
#pragma unroll
    for (int k = 0; k < kGreedyQPer; k++) {
        res[k] = -1; nc[k] = 0; obs[k] = false; angL[k] = 0.f;
#pragma unroll
        for (int j = 0; j < kGreedyPre; j++) pre[k][j] = 0;
    }
    // the first 4096 keypoints' occupancy and octave (the rest, if any, in a loop below)
    int o0[4], v0[4];
#pragma unroll
    for (int u = 0; u < 4; u++) {
        o0[u] = 0; v0[u] = 0;
        if (u * kGreedyThreads < nCapF) {  // uniform: slots past the capacity issue nothing
            const int ic = min(tid + u * kGreedyThreads, nCapF - 1);
            o0[u] = a.occ0[ic];
            v0[u] = a.F.keys[ic].octave;
        }
    }
    int ncv[kGreedyQPer];
    unsigned flv[kGreedyQPer];
    float alv[kGreedyQPer];
    unsigned long long ev[kGreedyQPer][kGreedyPre];
    unsigned sink = 0;
#pragma unroll
    for (int k = 0; k < kGreedyQPer; k++) {
        ncv[k] = 0; flv[k] = 0; alv[k] = 0.f;
#pragma unroll
        for (int j = 0; j < kGreedyPre; j++) ev[k][j] = 0;
        if (k * kGreedyThreads >= nqCap) continue;  // uniform: slots past the capacity issue nothing
        const int qc = min(tid + k * kGreedyThreads, nqCap - 1);
        ncv[k] = a.ncand[qc];
        flv[k] = a.mode == 0 ? a.mps[qc].flags : a.lfp[qc].flags;
        alv[k] = *(ori ? &a.LF.keys[qc].angle : (const float*)a.ncand);
        const unsigned long long* t = a.top + (long long)qc * kTopK;
#pragma unroll
        for (int j = 0; j < kGreedyPre; j++) ev[k][j] = t[j];
    }
    // every load above is issued before the gate's branch (one wait for all of them; a load the
    // compiler sank past the branch would make a second round trip)
#pragma unroll
    for (int k = 0; k < kGreedyQPer; k++) {
        sink ^= (unsigned)ncv[k] ^ flv[k] ^ __float_as_uint(alv[k]);
#pragma unroll
        for (int j = 0; j < kGreedyPre; j++) sink ^= (unsigned)ev[k][j];
    }
#pragma unroll
    for (int u = 0; u < 4; u++) sink ^= (unsigned)(o0[u] ^ v0[u]);
    asm volatile("" ::"v"(sink));
    if (a.gate && gv >= a.gate_min) return;  // uniform: every thread reads before any write
    const int n = a.F.n_dev ? min(nFv, a.F.n) : a.F.n;
    const int nq = a.mode == 1 ? (a.LF.n_dev ? min(nLv, a.LF.n) : a.LF.n) : a.nq;  // (a.nq stays unmodified)
    const bool regs = nq <= kGreedyThreads * kGreedyQPer;
    if (regs && nq > 0) {
#pragma unroll
        for (int k = 0; k < kGreedyQPer; k++) {
            if (tid + k * kGreedyThreads >= nq) continue;
            nc[k] = ncv[k];
            obs[k] = (flv[k] & ORBMI_MP_HAS_OBS) != 0;
            angL[k] = alv[k];
#pragma unroll
            for (int j = 0; j < kGreedyPre; j++)
                pre[k][j] = ((unsigned)(ev[k][j] >> 40) << 16) | (unsigned)(ev[k][j] & 0xFFFF);
        }
    }
    for (int base = 0; base < n; base += 4 * kGreedyThreads) {
        int o[4], v[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            o[u] = o0[u]; v[u] = v0[u];
            if (base > 0) {
                const int ic = min(base + tid + u * kGreedyThreads, n - 1);
                o[u] = a.occ0[ic];
                v[u] = a.F.keys[ic].octave;
            }
        }
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int i = base + tid + u * kGreedyThreads;
            if (i < n) { occ0[i] = (uint8_t)o[u]; oct[i] = (uint8_t)v[u]; claim[i] = o[u] ? 0 : 0x7FFFFFFF; }
        }
    }
    if (!regs)
        for (int q = tid; q < nq; q += blockDim.x) a.res[q] = -1;
    if (tid < 2) flag[tid] = 0;
    __syncthreads();
    // usable prefix: past kCandCap the list is partial; entries past it point at keypoint 0
    // (their claim words are read and ignored); mode 0 packs the octaves in
    int kk[kGreedyQPer];
#pragma unroll
    for (int k = 0; k < kGreedyQPer; k++) {
        kk[k] = nc[k] <= a.cap ? min(nc[k], kGreedyPre) : 0;
#pragma unroll
        for (int j = 0; j < kGreedyPre; j++) {
            if (j >= kk[k]) pre[k][j] = 0;
            else if (a.mode == 0) pre[k][j] |= (unsigned)oct[pe_idx(pre[k][j])] << 25;
        }
    }
    const unsigned long long c1 = __builtin_amdgcn_s_memtime();
    bool converged = false;
    int rounds = 0, nslow = 0;
    unsigned long long tcl = 0, tev = 0, tfl = 0;  // thread 0's split of the rounds (development aid)
    static_assert(kGreedyRounds < 48 + 1 && kGreedyMaxKp <= 65536, "round tags (7 bits) above 24-bit query indices");
    for (int round = 0; round < kGreedyRounds && !converged; round++) {
        rounds++;
        const unsigned long long r0 = __builtin_amdgcn_s_memtime();
        const int tag = (64 - round) << kGreedyQBits;
        // keypoint idx is taken for query q: occupied on entry, or claimed this round by an earlier query
        // (one compare: claims of older rounds carry larger tags, 0 = occupied on entry)
        auto taken = [&](int idx, int q) { return claim[idx] < (tag | q); };
        // (claims double-buffered by round parity, posted right after each evaluation, one barrier
        // per round: no gain, the waves then wait at that barrier for the slowest one's atomics --
        // profiles/r06/greedy_ab.txt)
        if (regs) {
#pragma unroll
            for (int k = 0; k < kGreedyQPer; k++)
                if (res[k] >= 0 && obs[k]) atomicMin(&claim[res[k]], tag | (tid + k * kGreedyThreads));
        } else {
            for (int q = tid; q < nq; q += blockDim.x) {
                const int r = a.res[q];
                if (r >= 0 && query_has_obs(a, q)) atomicMin(&claim[r], tag | q);
            }
        }
        __syncthreads();
        const unsigned long long r1 = __builtin_amdgcn_s_memtime();
        if (tid == 0) flag[(round + 1) & 1] = 0;  // the next round's slot (last read before this round's claims)
        int changed = 0;
        if (regs) {
            unsigned slow = 0, ovf = 0;
            int nr[kGreedyQPer];
#pragma unroll
            for (int k = 0; k < kGreedyQPer; k++) {
                const int q = tid + k * kGreedyThreads;
                nr[k] = res[k];
                // every query is evaluated in every round (a per-wave skip of unchanged queries
                // measured no gain: after round 0 the re-evaluations are spread over all waves)
                if (q >= nq) continue;
                // the prefix's claim words read at once (independent LDS reads, one latency)
                int cv[kGreedyPre];
#pragma unroll
                for (int j = 0; j < kGreedyPre; j++) cv[j] = claim[pe_idx(pre[k][j])];
                // the two smallest unclaimed prefix entries, by selects
                unsigned e1 = kNoEntry, e2 = kNoEntry;
#pragma unroll
                for (int j = 0; j < kGreedyPre; j++) {
                    // taken <=> cv < tag | q: 0 (occupied on entry) and this round's earlier
                    // claims are below it, later queries' and older rounds' claims (larger
                    // tags) and 0x7FFFFFFF (never claimed) are not
                    const bool fr = j < kk[k] && cv[j] >= (tag | q);
                    const bool to1 = fr && e1 == kNoEntry;
                    const bool to2 = fr && !to1 && e2 == kNoEntry;
                    e2 = to2 ? pre[k][j] : e2;
                    e1 = to1 ? pre[k][j] : e1;
                }
                // mode 1 decides on the best entry alone; mode 0 needs the second (ratio test)
                const bool open = (a.mode == 0 ? e2 : e1) == kNoEntry && nc[k] > kGreedyPre;
                if (!open) nr[k] = greedy_decide_pe(a, e1, e2);
                else if (nc[k] <= a.cap) slow |= 1u << k;
                else ovf |= 1u << k;
            }
            nslow += __builtin_popcount(slow | ovf);
            // queries whose prefix ran out: the whole wave evaluates each one together, every
            // lane loading entries of its candidate list (one global latency instead of a serial
            // scan), the two smallest unclaimed entries by wave minima (entries are distinct)
#pragma unroll
            for (int k = 0; k < kGreedyQPer; k++) {
                unsigned long long pending = __ballot((slow >> k) & 1);
                while (pending) {
                    const int src = __builtin_ctzll(pending);
                    pending &= pending - 1;
                    const int q = tid - lane + src + k * kGreedyThreads;
                    const int ncq = __builtin_amdgcn_readlane(nc[k], src);
                    const unsigned long long* c =
                        ncq <= kTopK ? a.top + (long long)q * kTopK : a.cand + (long long)q * a.cap;
                    unsigned long long b1 = ~0ull, b2 = ~0ull;
                    for (int p = lane; p < ncq; p += 64) {
                        const unsigned long long e = c[p];
                        if (taken((int)(e & 0xFFFFF), q)) continue;
                        if (e < b1) { b2 = b1; b1 = e; }
                        else if (e < b2) b2 = e;
                    }
                    const unsigned long long m1 = wave_min_u64_dpp(b1);
                    const unsigned long long m2 = wave_min_u64_dpp(b1 == m1 ? b2 : b1);
                    const int r = greedy_decide(a, oct, (int)(m1 >> 40), m1 == ~0ull ? -1 : (int)(m1 & 0xFFFFF),
                                                (int)(m2 >> 40), m2 == ~0ull ? -1 : (int)(m2 & 0xFFFFF));
                    if (lane == src) nr[k] = r;
                }
            }
            // overflowed lists (more than kCandCap candidates): the owning lane enumerates again
            if (ovf) {
#pragma unroll 1
                for (int k = 0; k < kGreedyQPer; k++) {
                    if (!((ovf >> k) & 1)) continue;
                    const int q = tid + k * kGreedyThreads;
                    ovfres[k * kGreedyThreads + tid] =
                        greedy_eval(a, q, Tc.m, fw, bw, [&](int idx) { return taken(idx, q); });
                }
            }
#pragma unroll
            for (int k = 0; k < kGreedyQPer; k++) {
                const int r = (ovf >> k) & 1 ? ovfres[k * kGreedyThreads + tid] : nr[k];
                if (r != res[k]) { res[k] = r; changed = 1; }
            }
        } else {
            for (int q = tid; q < nq; q += blockDim.x) {
                const int r = greedy_eval(a, q, Tc.m, fw, bw, [&](int idx) { return taken(idx, q); });
                if (r != a.res[q]) { a.res[q] = r; changed = 1; }
            }
        }
        const unsigned long long r2 = __builtin_amdgcn_s_memtime();
        if (__ballot(changed) && lane == 0) flag[round & 1] = 1;  // one LDS store per wave, no atomics
        __syncthreads();
        converged = flag[round & 1] == 0;
        const unsigned long long r3 = __builtin_amdgcn_s_memtime();
        tcl += r1 - r0; tev += r2 - r1; tfl += r3 - r2;
    }
    if (regs) {
#pragma unroll
        for (int k = 0; k < kGreedyQPer; k++) {
            const int q = tid + k * kGreedyThreads;
            if (q < nq) a.res[q] = res[k];
        }
        __threadfence_block();
        __syncthreads();
    }
    if (!converged) {  // sequential replay (exact), bounded-rounds fallback
        if (tid == 0) {
            for (int i = 0; i < n; i++) claim[i] = occ0[i];
            for (int q = 0; q < nq; q++) {
                const int r = greedy_eval(a, q, Tc.m, fw, bw, [&](int idx) { return claim[idx] != 0; });
                a.res[q] = r;
                if (r >= 0 && query_has_obs(a, q)) claim[r] = 1;
            }
        }
        __syncthreads();
        if (regs) {  // the sequential replay's results
#pragma unroll
            for (int k = 0; k < kGreedyQPer; k++) {
                const int q = tid + k * kGreedyThreads;
                if (q < nq) res[k] = a.res[q];
            }
        }
    }
    const unsigned long long c2 = __builtin_amdgcn_s_memtime();
    // outputs: last assignment per keypoint (claim[] reused); rotation consistency (mode 1),
    // rejected keypoints flagged in occ0[].  The matched keypoints' angles are loaded first and
    // travel while the tables are cleared.
    float angF[kGreedyQPer];
#pragma unroll
    for (int k = 0; k < kGreedyQPer; k++) {
        angF[k] = 0.f;
        if (regs && ori && tid + k * kGreedyThreads < nq && res[k] >= 0) angF[k] = a.F.keys[res[k]].angle;
    }
    int* last = claim;
    uint8_t* rejected = occ0;
    for (int i = tid; i < n; i += blockDim.x) { last[i] = -1; rejected[i] = 0; }
    if (tid < HISTO_LENGTH) hist[tid] = 0;
    if (tid == 0) flag[3] = 0;
    __syncthreads();
    int fbin[kGreedyQPer];
    int nmine = 0;
    if (regs) {
#pragma unroll
        for (int k = 0; k < kGreedyQPer; k++) {
            const int q = tid + k * kGreedyThreads;
            const bool m = q < nq && res[k] >= 0;
            fbin[k] = -1;
            if (m) {
                atomicMax(&last[res[k]], q);
                nmine++;
                if (ori) fbin[k] = rot_bin(angL[k], angF[k]);
            }
            // the wave's bins: one LDS atomic per distinct bin (most matches share one or two)
            unsigned long long act = __ballot(fbin[k] >= 0);
            while (act) {
                const int b = __builtin_amdgcn_readlane(fbin[k], __builtin_ctzll(act));
                const unsigned long long same = __ballot(fbin[k] == b);
                if (lane == __builtin_ctzll(act)) atomicAdd(&hist[b], (int)__builtin_popcountll(same));
                act &= ~same;
            }
        }
    } else {
        for (int q = tid; q < nq; q += blockDim.x) {
            const int r = a.res[q];
            if (r < 0) continue;
            atomicMax(&last[r], q);
            nmine++;
            if (ori) atomicAdd(&hist[rot_bin(a.LF.keys[q].angle, a.F.keys[r].angle)], 1);
        }
    }
    // match counts per thread, then one LDS atomic per wave (a shared counter hit by every
    // thread serialises the wave's 64 atomics)
    auto wave_count = [&](int c, int sign) {
        c = (int)wave_sum((double)c);
        if (lane == 0 && c) atomicAdd(&flag[3], sign * c);
    };
    wave_count(nmine, 1);
    __syncthreads();
    if (ori) {
        // ComputeThreeMaxima (:1854-1895): the three largest non-empty bins, a tie going to the
        // lower bin (the scan's strict comparisons), by three wave maxima of count << 8 | (255 - bin)
        const int s = lane < HISTO_LENGTH ? hist[lane] : 0;
        const unsigned key = s > 0 ? ((unsigned)s << 8) | (unsigned)(255 - lane) : 0u;
        const unsigned k1 = wave_max_u32_dpp(key);
        const unsigned k2 = wave_max_u32_dpp(key == k1 ? 0u : key);
        const unsigned k3 = wave_max_u32_dpp(key == k1 || key == k2 ? 0u : key);
        const int max1 = (int)(k1 >> 8), max2 = (int)(k2 >> 8), max3 = (int)(k3 >> 8);
        int ind1 = k1 ? 255 - (int)(k1 & 255) : -1, ind2 = k2 ? 255 - (int)(k2 & 255) : -1;
        int ind3 = k3 ? 255 - (int)(k3 & 255) : -1;
        if (max2 < 0.1f * (float)max1) { ind2 = -1; ind3 = -1; }
        else if (max3 < 0.1f * (float)max1) { ind3 = -1; }
        auto keep = [&](int bin) { return bin == ind1 || bin == ind2 || bin == ind3; };
        int nrej = 0;
        if (regs) {
#pragma unroll
            for (int k = 0; k < kGreedyQPer; k++)
                if (fbin[k] >= 0 && !keep(fbin[k])) { rejected[res[k]] = 1; nrej++; }
        } else {
            for (int q = tid; q < nq; q += blockDim.x) {
                const int r = a.res[q];
                if (r >= 0 && !keep(rot_bin(a.LF.keys[q].angle, a.F.keys[r].angle))) { rejected[r] = 1; nrej++; }
            }
        }
        wave_count(nrej, -1);
        __syncthreads();
    }
    for (int i = tid; i < n; i += blockDim.x) a.out[i] = rejected[i] ? -2 : last[i];
    if (tid == 0) *a.nmatches = flag[3];
    if (!g_greedy_on) return;  // statistics only once a probe asked for them
    if (nslow) atomicAdd(&g_greedy_stats[3], (unsigned long long)nslow);
    if (tid == 0) {
        const unsigned long long c3 = __builtin_amdgcn_s_memtime();
        atomicAdd(&g_greedy_cycles[0], c1 - c0);
        atomicAdd(&g_greedy_cycles[1], c2 - c1);
        atomicAdd(&g_greedy_cycles[2], c3 - c2);
        atomicAdd(&g_greedy_cycles[3], tcl);
        atomicAdd(&g_greedy_cycles[4], tev);
        atomicAdd(&g_greedy_cycles[5], tfl);
        atomicAdd(&g_greedy_stats[0], 1ull);
        atomicAdd(&g_greedy_stats[1], (unsigned long long)rounds);
        atomicMax(&g_greedy_stats[2], (unsigned long long)rounds);
        if (!converged) atomicAdd(&g_greedy_stats[4], 1ull);
    }
}

int greedy_cycles(unsigned long long out[7], int reset) {
    ORBMI_HIP(hipDeviceSynchronize());
    const int on = 1;
    ORBMI_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_greedy_on), &on, sizeof(on)));
    ORBMI_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_greedy_cycles), sizeof(unsigned long long) * 7));
    if (reset) {
        const unsigned long long z[7] = {0, 0, 0, 0, 0, 0, 0};
        ORBMI_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_greedy_cycles), z, sizeof(z)));
    }
    return ORBMI_OK;
}

int greedy_stats(unsigned long long out[5], int reset) {
    ORBMI_HIP(hipDeviceSynchronize());
    const int on = 1;
    ORBMI_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_greedy_on), &on, sizeof(on)));
    ORBMI_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_greedy_stats), sizeof(unsigned long long) * 5));
    if (reset) {
        const unsigned long long z[5] = {0, 0, 0, 0, 0};
        ORBMI_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_greedy_stats), z, sizeof(z)));
    }
    return ORBMI_OK;
}

// -------------------------------------------------------------------------- Tracking
// Tracking's pass over mvpMapPoints after a PoseOptimization (orbmi_track_update_matches;
// track_update.h, which k_pose_opt also runs as its tail for orbmi_pose_optimization_frame_track)
__global__ __launch_bounds__(1024) void k_track_update(DevFrame F, int stage, const uint8_t* __restrict__ outlier,
                                                       int* __restrict__ match_lf,
                                                       const orbmi_lastframe_point* __restrict__ lfp, int n_lf,
                                                       int* __restrict__ match_mp,
                                                       const orbmi_mappoint* __restrict__ mps, int n_mp,
                                                       uint8_t* __restrict__ occ_out, int* __restrict__ counts) {
    __shared__ int cnt[2];
    track_update_body(frame_n(F), F.u_right != nullptr, stage, outlier, match_lf, lfp, n_lf, match_mp, mps, n_mp,
                      occ_out, counts, cnt);
}

// -------------------------------------------------------------------------- SearchByBoW
// Each node of the KF feature vector finds its partner node in F (merge-join of two sorted
// id lists, :234-320); nodes are independent (a feature belongs to one node), the greedy
// exclusion (:265-266) is sequential inside the node: one wave per node.
__global__ __launch_bounds__(256) void k_bow_match(DevFrame KF, const uint8_t* __restrict__ kf_ok, DevFV kfv,
                                                   DevFrame F, DevFV fv, float nnratio, int check_ori,
                                                   int* __restrict__ match, int* __restrict__ bin_of,
                                                   int* __restrict__ hist) {
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int a = blockIdx.x * 4 + wid;
    if (a >= kfv.nnodes) return;
    const unsigned id = kfv.node_id[a];
    int lo = 0, hi = fv.nnodes;  // lower_bound
    while (lo < hi) { const int mid = (lo + hi) >> 1; if (fv.node_id[mid] < id) lo = mid + 1; else hi = mid; }
    if (lo >= fv.nnodes || fv.node_id[lo] != id) return;
    const int f0 = fv.off[lo], nf = fv.off[lo + 1] - f0;
    constexpr int kPer = 8;  // F features per lane kept in registers
    bool matched[kPer];
#pragma unroll
    for (int k = 0; k < kPer; k++) matched[k] = false;
    for (int ia = kfv.off[a]; ia < kfv.off[a + 1]; ia++) {
        const int realIdxKF = kfv.feat[ia];
        if (!kf_ok[realIdxKF]) continue;
        const uint8_t* dKF = KF.desc + 32 * (long long)realIdxKF;
        unsigned long long b1 = ~0ull, b2 = ~0ull;
        for (int base = 0; base < nf; base += 64 * kPer) {
#pragma unroll
            for (int k = 0; k < kPer; k++) {
                const int pos = base + k * 64 + lane;
                if (pos >= nf) continue;
                const int realIdxF = fv.feat[f0 + pos];
                const bool done = base == 0 ? matched[k] : match[realIdxF] >= 0;
                if (done) continue;
                const unsigned long long e = ((unsigned long long)popc_desc(dKF, F.desc + 32 * (long long)realIdxF) << 32) | (unsigned)pos;
                if (e < b1) { b2 = b1; b1 = e; } else if (e < b2) b2 = e;
            }
        }
        // wave-wide best / second best of the (dist, position) keys
        const unsigned long long m1 = wave_min_u64(b1);
        const unsigned long long c2 = b1 == m1 ? b2 : b1;
        const unsigned long long m2 = wave_min_u64(c2);
        const int bestDist1 = m1 == ~0ull ? 256 : (int)(m1 >> 32);
        const int bestDist2 = m2 == ~0ull ? 256 : (int)(m2 >> 32);
        if (bestDist1 <= TH_LOW && (float)bestDist1 < nnratio * (float)bestDist2) {
            const int pos = (int)(m1 & 0xFFFFFFFFu);
            const int realIdxF = fv.feat[f0 + pos];
            if (pos < 64 * kPer && lane == (pos & 63)) {
#pragma unroll
                for (int k = 0; k < kPer; k++)
                    if (k == (pos >> 6)) matched[k] = true;
            }
            if (lane == 0) {
                match[realIdxF] = realIdxKF;
                if (check_ori) {
                    const int bin = rot_bin(KF.keys[realIdxKF].angle, F.keys[realIdxF].angle);
                    bin_of[realIdxF] = bin;
                    atomicAdd(&hist[bin], 1);
                }
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
        }
    }
}

// rotation-histogram filter (ComputeThreeMaxima, src/ORBmatcher.cc:1854-1895) of one search's
// matches and their count, one workgroup
__device__ inline void finalize_block(int n, int check_ori, const int* __restrict__ hist,
                                      const int* __restrict__ bin_of, int* __restrict__ match,
                                      int* __restrict__ nmatches) {
    __shared__ int cnt;
    if (threadIdx.x == 0) cnt = 0;
    __syncthreads();
    int ind1 = -1, ind2 = -1, ind3 = -1;
    if (check_ori) {
        int max1 = 0, max2 = 0, max3 = 0;
        for (int i = 0; i < HISTO_LENGTH; i++) {
            const int s = hist[i];
            if (s > max1) { max3 = max2; max2 = max1; max1 = s; ind3 = ind2; ind2 = ind1; ind1 = i; }
            else if (s > max2) { max3 = max2; max2 = s; ind3 = ind2; ind2 = i; }
            else if (s > max3) { max3 = s; ind3 = i; }
        }
        if (max2 < 0.1f * (float)max1) { ind2 = -1; ind3 = -1; }
        else if (max3 < 0.1f * (float)max1) { ind3 = -1; }
    }
    int local = 0;
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        if (match[i] < 0) continue;
        if (check_ori) {
            const int b = bin_of[i];
            if (b != ind1 && b != ind2 && b != ind3) { match[i] = -1; continue; }
        }
        local++;
    }
    atomicAdd(&cnt, local);
    __syncthreads();
    if (threadIdx.x == 0 && nmatches) *nmatches = cnt;
}

__global__ __launch_bounds__(1024) void k_bow_finalize(DevFrame F, int check_ori, const int* __restrict__ hist,
                                                       const int* __restrict__ bin_of, int* __restrict__ match,
                                                       int* __restrict__ nmatches) {
    finalize_block(frame_n(F), check_ori, hist, bin_of, match, nmatches);
}


// -------------------------------------------------------------------------- cross-stream
// Config 4 (build-defined): every query descriptor against every valid train
// row of the gathered segments.  Workgroup = 64 queries x one train chunk staged in LDS; the
// four waves split the chunk and merge (best, second) through LDS.  Entries are dist<<32 | row
// so ties resolve to the lowest global row.
constexpr int kXQ = 64, kXChunk = 512;

__global__ __launch_bounds__(256) void k_xmatch_partial(const uint8_t* __restrict__ qd, int nq_cap,
                                                        const int* __restrict__ nq_dev,
                                                        const uint8_t* __restrict__ td, int nseg, int seg_cap,
                                                        const int* __restrict__ seg_counts, int skip_seg,
                                                        int chunk, unsigned long long* __restrict__ part) {
    __shared__ uint4 tile[kXChunk * 2];
    __shared__ unsigned long long red[4][kXQ][2];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int nq = nq_dev ? min(*nq_dev, nq_cap) : nq_cap;
    const int q = blockIdx.x * kXQ + lane;
    const int t0 = blockIdx.y * chunk, t1 = min(t0 + chunk, nseg * seg_cap);
    uint4 a0 = make_uint4(0, 0, 0, 0), a1 = a0;
    if (q < nq) {
        const uint4* p = reinterpret_cast<const uint4*>(qd + 32 * (long long)q);
        a0 = p[0]; a1 = p[1];
    }
    unsigned long long b1 = ~0ull, b2 = ~0ull;
    for (int base = t0; base < t1; base += kXChunk) {
        const int nt = min(kXChunk, t1 - base);
        __syncthreads();
        for (int k = threadIdx.x; k < nt * 2; k += blockDim.x)
            tile[k] = reinterpret_cast<const uint4*>(td + 32 * (long long)base)[k];
        __syncthreads();
        for (int k = w; k < nt; k += 4) {
            const int row = base + k, seg = row / seg_cap;
            if (seg == skip_seg || row - seg * seg_cap >= seg_counts[seg]) continue;
            const unsigned long long e = ((unsigned long long)popc256(a0, a1, tile[2 * k], tile[2 * k + 1]) << 32) |
                                         (unsigned)row;
            if (e < b1) { b2 = b1; b1 = e; } else if (e < b2) b2 = e;
        }
    }
    red[w][lane][0] = b1;
    red[w][lane][1] = b2;
    __syncthreads();
    if (w == 0 && q < nq) {
        for (int o = 1; o < 4; o++)
            for (int j = 0; j < 2; j++) {
                const unsigned long long e = red[o][lane][j];
                if (e < b1) { b2 = b1; b1 = e; } else if (e < b2) b2 = e;
            }
        part[((long long)blockIdx.y * nq_cap + q) * 2] = b1;
        part[((long long)blockIdx.y * nq_cap + q) * 2 + 1] = b2;
    }
}

__global__ __launch_bounds__(256) void k_xmatch_final(int nq_cap, const int* __restrict__ nq_dev, int nsplit,
                                                      const unsigned long long* __restrict__ part, int th,
                                                      float ratio, int* __restrict__ match,
                                                      int* __restrict__ nmatches) {
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    const int nq = nq_dev ? min(*nq_dev, nq_cap) : nq_cap;
    if (q >= nq) return;
    unsigned long long b1 = ~0ull, b2 = ~0ull;
    for (int s = 0; s < nsplit; s++)
        for (int j = 0; j < 2; j++) {
            const unsigned long long e = part[((long long)s * nq_cap + q) * 2 + j];
            if (e < b1) { b2 = b1; b1 = e; } else if (e < b2) b2 = e;
        }
    int r = -1;
    if (b1 != ~0ull) {
        const int d1 = (int)(b1 >> 32), d2 = b2 == ~0ull ? 256 : (int)(b2 >> 32);
        if (d1 <= th && (float)d1 < ratio * (float)d2) r = (int)(b1 & 0xFFFFFFFFu);
    }
    match[q] = r;
    if (r >= 0) atomicAdd(nmatches, 1);
}

int launch_xmatch(Matcher& m, const uint8_t* qd, int nq_cap, const int* nq_dev, const uint8_t* td, int nseg,
                  int seg_cap, const int* seg_counts, int skip_seg, int th, float ratio, int* match, int* nmatches) {
    if (nq_cap <= 0) return ORBMI_OK;
    const long long ntrain = (long long)nseg * seg_cap;
    // enough workgroups to cover the chip: 64-query blocks x train splits
    const int qblocks = (nq_cap + kXQ - 1) / kXQ;
    int nsplit = (int)std::max(1LL, std::min<long long>((ntrain + 255) / 256, (1024 + qblocks - 1) / qblocks));
    const int chunk = (int)((ntrain + nsplit - 1) / nsplit);
    nsplit = (int)std::max(1LL, (ntrain + chunk - 1) / chunk);
    int rc;
    if ((rc = ensure_buf(&m.d_cand, &m.cap_cand, (size_t)nsplit * nq_cap * 2))) return rc;
    hipLaunchKernelGGL(k_xmatch_partial, dim3(qblocks, nsplit), dim3(256), 0, m.ls(), qd, nq_cap, nq_dev, td, nseg,
                       seg_cap, seg_counts, skip_seg, chunk, m.d_cand);
    hipLaunchKernelGGL(k_xmatch_final, dim3((nq_cap + 255) / 256), dim3(256), 0, m.ls(), nq_cap, nq_dev, nsplit,
                       m.d_cand, th, ratio, match, nmatches);
    return ORBMI_OK;
}

// -------------------------------------------------------------------------- host launchers
static bool grid_is_pinned_for(const Matcher& m, const DevFrame& F) {
    const float g[6] = {F.min_x, F.max_x, F.min_y, F.max_y, F.grid_w_inv, F.grid_h_inv};
    return m.grid_pinned && m.pin_keys == F.keys && m.pin_ndev == F.n_dev && m.pin_n == F.n &&
           memcmp(m.pin_geom, g, sizeof(g)) == 0;
}

static int grid_for(Matcher& m, const DevFrame& F, const int* gate = nullptr, int gate_min = 0) {
    if (F.n > kGreedyMaxKp) return ORBMI_E_UNSUPPORTED;
    // Frame::AssignFeaturesToGrid runs once per Frame (src/Frame.cc:232-247): a pinned grid of
    // this frame is reused as it is
    if (grid_is_pinned_for(m, F)) return ORBMI_OK;
    m.grid_pinned = false;
    int rc;
    if ((rc = ensure_buf(&m.d_cell_start, &m.cap_cell_start, (size_t)kGridCells + 1))) return rc;
    if ((rc = ensure_buf(&m.d_cell_list, &m.cap_cell_list, (size_t)std::max(F.n, 1)))) return rc;
    if ((rc = ensure_buf(&m.d_kp_cell, &m.cap_kp_cell, (size_t)std::max(F.n, 1)))) return rc;
    hipLaunchKernelGGL(k_grid_build, dim3(1), dim3(1024), 0, m.ls(), F, m.d_cell_start, m.d_cell_list, m.d_kp_cell,
                       gate, gate_min);
    m.cur_cs = m.d_cell_start;
    m.cur_cl = m.d_cell_list;
    return ORBMI_OK;
}

static void pin_key(Matcher& m, const DevFrame& F) {
    m.grid_pinned = true;
    m.pin_keys = F.keys;
    m.pin_ndev = F.n_dev;
    m.pin_n = F.n;
    const float g[6] = {F.min_x, F.max_x, F.min_y, F.max_y, F.grid_w_inv, F.grid_h_inv};
    memcpy(m.pin_geom, g, sizeof(g));
}

int pin_grid(Matcher& m, const DevFrame& F) {
    m.grid_pinned = false;
    int rc;
    if ((rc = grid_for(m, F))) return rc;
    pin_key(m, F);
    return ORBMI_OK;
}

// Frame::AssignFeaturesToGrid into slot grid k on stream s (the caller orders the searches that
// read it behind s, and the next build of slot k behind those searches)
int build_grid_slot(Matcher& m, const DevFrame& F, int k, hipStream_t s) {
    if (F.n > kGreedyMaxKp) return ORBMI_E_UNSUPPORTED;
    Matcher::GridSlot& g = m.gslot[k];
    const size_t need = (size_t)std::max(F.n, 1);
    if (!g.cs) ORBMI_HIP(hipMalloc((void**)&g.cs, ((size_t)kGridCells + 1) * sizeof(int)));
    if (need > g.cap) {
        if (g.cl) (void)hipFree(g.cl);
        if (g.kc) (void)hipFree(g.kc);
        g.cl = g.kc = nullptr;
        g.cap = 0;
        ORBMI_HIP(hipMalloc((void**)&g.cl, need * sizeof(int)));
        ORBMI_HIP(hipMalloc((void**)&g.kc, need * sizeof(int)));
        g.cap = need;
    }
    hipLaunchKernelGGL(k_grid_build, dim3(1), dim3(1024), 0, s, F, g.cs, g.cl, g.kc, (const int*)nullptr, 0);
    g.built = true;
    g.keys = F.keys;
    g.ndev = F.n_dev;
    g.n = F.n;
    const float geom[6] = {F.min_x, F.max_x, F.min_y, F.max_y, F.grid_w_inv, F.grid_h_inv};
    memcpy(g.geom, geom, sizeof(geom));
    return ORBMI_OK;
}

// the searches on frame F read slot grid k from now on (it must have been built for F)
int pin_grid_slot(Matcher& m, const DevFrame& F, int k) {
    const Matcher::GridSlot& g = m.gslot[k];
    const float geom[6] = {F.min_x, F.max_x, F.min_y, F.max_y, F.grid_w_inv, F.grid_h_inv};
    if (!g.built || g.keys != F.keys || g.ndev != F.n_dev || g.n != F.n || memcmp(g.geom, geom, sizeof(geom)) != 0)
        return ORBMI_E_STATE;
    pin_key(m, F);
    m.cur_cs = g.cs;
    m.cur_cl = g.cl;
    return ORBMI_OK;
}

int launch_frustum(Matcher& m, const DevFrame& F, const orbmi_mappoint* mps, int n, float cosl,
                   orbmi_mappoint_track* tr, int* n_in_view) {
    if (n <= 0) return ORBMI_OK;
    hipLaunchKernelGGL(k_frustum, dim3((n + 255) / 256), dim3(256), 0, m.ls(), F, mps, n, cosl, tr, n_in_view);
    return ORBMI_OK;
}

int launch_local_search(Matcher& m, const DevFrame& F, const uint8_t* occ0, const orbmi_mappoint* mps,
                        const orbmi_mappoint_track* tr, int n, float th, float nnratio, int* out, int* nmatches) {
    if (n >= kGreedyMaxQueries) return ORBMI_E_UNSUPPORTED;  // k_greedy's claim field
    int rc;
    if ((rc = grid_for(m, F))) return rc;
    const int cap = Matcher::kCandCap;
    if ((rc = ensure_buf(&m.d_cand, &m.cap_cand, (size_t)std::max(n, 1) * cap))) return rc;
    if ((rc = ensure_buf(&m.d_ncand, &m.cap_ncand, (size_t)std::max(n, 1)))) return rc;
    if ((rc = ensure_buf(&m.d_res, &m.cap_res, (size_t)std::max(n, 1)))) return rc;
    if ((rc = ensure_buf(&m.d_top, &m.cap_top, (size_t)std::max(n, 1) * kTopK))) return rc;
    if (n > 0) {
        CandArgs ca{};
        ca.mode = 0; ca.nq = n; ca.F = F; ca.cs = m.cur_cs; ca.cl = m.cur_cl; ca.mps = mps; ca.tr = tr;
        ca.th = th; ca.cand = m.d_cand; ca.ncand = m.d_ncand; ca.top = m.d_top;
        hipLaunchKernelGGL(k_candidates<16>, dim3((n + 15) / 16), dim3(256), 0, m.ls(), ca);
    }
    GreedyArgs a{};
    a.mode = 0; a.nq = n; a.cand = m.d_cand; a.ncand = m.d_ncand; a.top = m.d_top; a.cap = cap; a.occ0 = occ0; a.F = F;
    a.cs = m.cur_cs; a.cl = m.cur_cl; a.mps = mps; a.tr = tr; a.th = th; a.nnratio = nnratio;
    a.res = m.d_res; a.out = out; a.nmatches = nmatches;
    hipLaunchKernelGGL(k_greedy, dim3(1), dim3(kGreedyThreads), 0, m.ls(), a);
    return ORBMI_OK;
}

int launch_lastframe_search(Matcher& m, const DevFrame& CF, const uint8_t* occ0, const DevFrame& LF,
                            const orbmi_lastframe_point* lfp, float th, int mono, int check_ori, int* out,
                            int* nmatches, const int* gate, int gate_min) {
    int rc;
    if ((rc = grid_for(m, CF, gate, gate_min))) return rc;
    const int n = LF.n, cap = Matcher::kCandCap;
    if (n >= kGreedyMaxQueries) return ORBMI_E_UNSUPPORTED;  // k_greedy's claim field
    if ((rc = ensure_buf(&m.d_cand, &m.cap_cand, (size_t)std::max(n, 1) * cap))) return rc;
    if ((rc = ensure_buf(&m.d_ncand, &m.cap_ncand, (size_t)std::max(n, 1)))) return rc;
    if ((rc = ensure_buf(&m.d_res, &m.cap_res, (size_t)std::max(n, 1)))) return rc;
    if ((rc = ensure_buf(&m.d_top, &m.cap_top, (size_t)std::max(n, 1) * kTopK))) return rc;
    if (n > 0) {
        CandArgs ca{};
        ca.mode = 1; ca.nq = n; ca.F = CF; ca.LF = LF; ca.cs = m.cur_cs; ca.cl = m.cur_cl; ca.lfp = lfp;
        ca.th = th; ca.mono = mono; ca.cand = m.d_cand; ca.ncand = m.d_ncand; ca.top = m.d_top;
        ca.gate = gate; ca.gate_min = gate_min;
        hipLaunchKernelGGL(k_candidates<16>, dim3((n + 15) / 16), dim3(256), 0, m.ls(), ca);
    }
    GreedyArgs a{};
    a.mode = 1; a.nq = n; a.cand = m.d_cand; a.ncand = m.d_ncand; a.top = m.d_top; a.cap = cap; a.occ0 = occ0; a.F = CF;
    a.LF = LF;
    a.cs = m.cur_cs; a.cl = m.cur_cl; a.lfp = lfp; a.th = th; a.mono = mono; a.check_ori = check_ori;
    a.res = m.d_res; a.out = out; a.nmatches = nmatches; a.gate = gate; a.gate_min = gate_min;
    hipLaunchKernelGGL(k_greedy, dim3(1), dim3(kGreedyThreads), 0, m.ls(), a);
    return ORBMI_OK;
}

int launch_track_update(Matcher& m, const DevFrame& F, int stage, const uint8_t* outlier, int* match_lf,
                        const orbmi_lastframe_point* lfp, int n_lf, int* match_mp, const orbmi_mappoint* mps,
                        int n_mp, uint8_t* occ_out, int* counts) {
    hipLaunchKernelGGL(k_track_update, dim3(1), dim3(1024), 0, m.ls(), F, stage, outlier, match_lf, lfp, n_lf,
                       match_mp, mps, n_mp, occ_out, counts);
    return ORBMI_OK;
}

int launch_bow(Matcher& m, const DevFrame& KF, const uint8_t* kf_ok, const DevFV& kfv, const DevFrame& F,
               const DevFV& fv, float nnratio, int check_ori, int* match, int* nmatches) {
    int rc;
    if ((rc = ensure_buf(&m.d_bin_of, &m.cap_bin_of, (size_t)std::max(F.n, 1)))) return rc;
    if ((rc = ensure_buf(&m.d_hist, &m.cap_hist, (size_t)HISTO_LENGTH))) return rc;
    ORBMI_HIP(hipMemsetAsync(m.d_hist, 0, HISTO_LENGTH * sizeof(int), m.ls()));
    ORBMI_HIP(hipMemsetAsync(match, 0xFF, (size_t)std::max(F.n, 1) * sizeof(int), m.ls()));
    if (kfv.nnodes > 0)
        hipLaunchKernelGGL(k_bow_match, dim3((kfv.nnodes + 3) / 4), dim3(256), 0, m.ls(), KF, kf_ok, kfv, F, fv,
                           nnratio, check_ori, match, m.d_bin_of, m.d_hist);
    hipLaunchKernelGGL(k_bow_finalize, dim3(1), dim3(1024), 0, m.ls(), F, check_ori, m.d_hist, m.d_bin_of, match,
                       nmatches);
    return ORBMI_OK;
}

// ------------------------------------------------------------- SearchForTriangulation
// ORBmatcher::SearchForTriangulation (src/ORBmatcher.cc:783-975).  The reference keeps no
// exclusion state (vbMatched2 is never set), so KF1 features are independent: a wave takes one
// slice of a KF1 vocabulary node's features (`splits` slices per node, so that a keyframe pair
// with a few large nodes -- a coarse vocabulary level -- still fills the chip), finds the node in
// KF2 by lower_bound, and for each of its features in order scans the node's KF2 features across
// the lanes.  The scan `if (dist > bestDist) continue; ... if (CheckDistEpipolarLine) {bestIdx2 =
// idx2; bestDist = dist;}` ends on the smallest distance <= TH_LOW among the candidates that
// pass, the LAST one on ties: key (dist << 32 | ~pos), min.  CheckDistEpipolarLine (:173-196)
// compares in double (3.84 * sigma2); the epipole and the keyframe-1 centre follow the P10 float
// order.  The rotation histogram is k_bow_finalize's.

struct TriNode {  // one wave's work: KF1 features feat1[0..n1) against KF2 node features f0..f0+nf
    const int* feat1;
    int n1, f0, nf;
    float ex, ey;  // the epipole (KF1's centre in KF2)
};

__device__ inline void tri_record(const TriPair& P, int check_ori, int idx1, int i2, float angle1) {
    P.match[idx1] = i2;
    if (check_ori) {
        const int bin = rot_bin(angle1, P.KF2.keys[i2].angle);
        P.bin_of[idx1] = bin;
        atomicAdd(&P.hist[bin], 1);
    }
}

// the node's KF2 candidates in registers (lane p holds candidates p, p + 64, ..., H of them), the
// KF1 features in chunks of 64 (lane p holds feature p of the chunk), each loaded in one round;
// the KF1 features are then visited in order by broadcasting lane i's (readlane), so the inner
// loop issues no memory access
template <int H>
__device__ void tri_node_regs(const DevFrame& KF1, const uint8_t* __restrict__ has_mp1, const TriPair& P,
                              const TriNode& T, int only_stereo, int check_ori, int lane) {
    const DevFrame& KF2 = P.KF2;
    const DevFV& fv2 = P.fv2;
    const Mat3f F12 = P.F12;
    bool okc[H], stc[H];
    int idxc[H];
    uint4 e0[H], e1[H];
    float kx[H], ky[H], sc2[H];
#pragma unroll
    for (int h = 0; h < H; h++) {
        const int pos = lane + 64 * h;
        okc[h] = pos < T.nf;
        stc[h] = false;
        idxc[h] = 0;
        e0[h] = make_uint4(0, 0, 0, 0);
        e1[h] = e0[h];
        kx[h] = ky[h] = 0.f;
        sc2[h] = 1.f;
        if (okc[h]) {
            const int i2 = fv2.feat[T.f0 + pos];
            idxc[h] = i2;
            stc[h] = KF2.u_right[i2] >= 0;
            okc[h] = !P.has_mp2[i2] && !(only_stereo && !stc[h]);
            const uint4* d2 = reinterpret_cast<const uint4*>(KF2.desc + 32 * (long long)i2);
            e0[h] = d2[0];
            e1[h] = d2[1];
            const orbmi_keypoint k2 = KF2.keys[i2];
            kx[h] = k2.x;
            ky[h] = k2.y;
            sc2[h] = KF2.scale[min(max(k2.octave, 0), kMaxLevels - 1)];
        }
    }
    for (int c1 = 0; c1 < T.n1; c1 += 64) {
        bool ok1 = c1 + lane < T.n1;
        int idx1l = 0;
        uint4 g0 = make_uint4(0, 0, 0, 0), g1 = g0;
        orbmi_keypoint kp1l{};
        bool st1l = false;
        if (ok1) {
            idx1l = T.feat1[c1 + lane];
            st1l = KF1.u_right[idx1l] >= 0;
            ok1 = !has_mp1[idx1l] && !(only_stereo && !st1l);
            const uint4* d1 = reinterpret_cast<const uint4*>(KF1.desc + 32 * (long long)idx1l);
            g0 = d1[0];
            g1 = d1[1];
            kp1l = KF1.keys[idx1l];
        }
        unsigned long long todo = __ballot(ok1);
        while (todo) {
            const int i = __ffsll((long long)todo) - 1;
            todo &= todo - 1;
            const int idx1 = __builtin_amdgcn_readlane(idx1l, i);
            const bool st1 = __builtin_amdgcn_readlane((int)st1l, i) != 0;
            const float k1x = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(kp1l.x), i));
            const float k1y = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(kp1l.y), i));
            const uint4 d0 = make_uint4(__builtin_amdgcn_readlane(g0.x, i), __builtin_amdgcn_readlane(g0.y, i),
                                        __builtin_amdgcn_readlane(g0.z, i), __builtin_amdgcn_readlane(g0.w, i));
            const uint4 d1 = make_uint4(__builtin_amdgcn_readlane(g1.x, i), __builtin_amdgcn_readlane(g1.y, i),
                                        __builtin_amdgcn_readlane(g1.z, i), __builtin_amdgcn_readlane(g1.w, i));
            // epipolar line of kp1 in KF2: l = x1' F12
            const float la = k1x * F12.m[0] + k1y * F12.m[3] + F12.m[6];
            const float lb = k1x * F12.m[1] + k1y * F12.m[4] + F12.m[7];
            const float lc = k1x * F12.m[2] + k1y * F12.m[5] + F12.m[8];
            unsigned long long key = ~0ull;
#pragma unroll
            for (int h = 0; h < H; h++) {
                if (!okc[h]) continue;
                const int dist = popc256(d0, d1, e0[h], e1[h]);
                bool pass = dist <= TH_LOW;
                if (pass && !st1 && !stc[h]) {
                    const float distex = T.ex - kx[h];
                    const float distey = T.ey - ky[h];
                    pass = !(distex * distex + distey * distey < 100 * sc2[h]);
                }
                if (pass) {
                    const float num = la * kx[h] + lb * ky[h] + lc;
                    const float den = la * la + lb * lb;
                    if (den == 0) pass = false;
                    else {
                        const float dsqr = num * num / den;
                        const float sigma2 = sc2[h] * sc2[h];
                        pass = (double)dsqr < 3.84 * (double)sigma2;
                    }
                }
                const unsigned long long k =
                    (unsigned long long)dist << 32 | (unsigned)(0xFFFFFFFFu - (unsigned)(lane + 64 * h));
                if (pass && k < key) key = k;
            }
            key = wave_min_u64_dpp(key);
            if (key != ~0ull) {
                const int pos = __builtin_amdgcn_readfirstlane((int)(0xFFFFFFFFu - (unsigned)(key & 0xFFFFFFFFu)));
                int i2 = 0;
#pragma unroll
                for (int h = 0; h < H; h++)
                    if ((pos >> 6) == h) i2 = __builtin_amdgcn_readlane(idxc[h], pos & 63);
                const float a1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(kp1l.angle), i));
                if (lane == 0) tri_record(P, check_ori, idx1, i2, a1);
            }
        }
    }
}

// nodes with more than 256 KF2 features: the candidates are read from memory per KF1 feature
__device__ void tri_node_mem(const DevFrame& KF1, const uint8_t* __restrict__ has_mp1, const TriPair& P,
                             const TriNode& T, int only_stereo, int check_ori, int lane) {
    const DevFrame& KF2 = P.KF2;
    const DevFV& fv2 = P.fv2;
    const Mat3f F12 = P.F12;
    for (int ia = 0; ia < T.n1; ia++) {
        const int idx1 = T.feat1[ia];
        if (has_mp1[idx1]) continue;
        const bool st1 = KF1.u_right[idx1] >= 0;
        if (only_stereo && !st1) continue;
        const orbmi_keypoint kp1 = KF1.keys[idx1];
        const uint8_t* d1 = KF1.desc + 32 * (long long)idx1;
        const float la = kp1.x * F12.m[0] + kp1.y * F12.m[3] + F12.m[6];
        const float lb = kp1.x * F12.m[1] + kp1.y * F12.m[4] + F12.m[7];
        const float lc = kp1.x * F12.m[2] + kp1.y * F12.m[5] + F12.m[8];
        unsigned long long key = ~0ull;
        for (int pos = lane; pos < T.nf; pos += 64) {
            const int idx2 = fv2.feat[T.f0 + pos];
            if (P.has_mp2[idx2]) continue;
            const bool st2 = KF2.u_right[idx2] >= 0;
            if (only_stereo && !st2) continue;
            const int dist = popc_desc(d1, KF2.desc + 32 * (long long)idx2);
            if (dist > TH_LOW) continue;
            const orbmi_keypoint kp2 = KF2.keys[idx2];
            if (!st1 && !st2) {
                const float distex = T.ex - kp2.x;
                const float distey = T.ey - kp2.y;
                if (distex * distex + distey * distey < 100 * KF2.scale[kp2.octave]) continue;
            }
            const float num = la * kp2.x + lb * kp2.y + lc;
            const float den = la * la + lb * lb;
            if (den == 0) continue;
            const float dsqr = num * num / den;
            const float sigma2 = KF2.scale[kp2.octave] * KF2.scale[kp2.octave];
            if (!((double)dsqr < 3.84 * (double)sigma2)) continue;
            const unsigned long long k = (unsigned long long)dist << 32 | (unsigned)(0xFFFFFFFFu - (unsigned)pos);
            key = k < key ? k : key;
        }
        key = wave_min_u64(key);
        if (key != ~0ull && lane == 0) {
            const int pos = (int)(0xFFFFFFFFu - (unsigned)(key & 0xFFFFFFFFu));
            tri_record(P, check_ori, idx1, fv2.feat[T.f0 + pos], kp1.angle);
        }
    }
}

__global__ __launch_bounds__(256) void k_tri_match(DevFrame KF1, const uint8_t* __restrict__ has_mp1, DevFV fv1,
                                                   const TriPair* __restrict__ pairs, int only_stereo, int check_ori,
                                                   int splits) {
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int w = blockIdx.x * 4 + wid;
    const int a = w / splits, sl = w - a * splits;
    if (a >= fv1.nnodes) return;
    const TriPair& P = pairs[blockIdx.y];  // the pair (KF1, KF2 = P.KF2) of this grid row
    const DevFV fv2 = P.fv2;
    const int A0 = fv1.off[a], N1 = fv1.off[a + 1] - A0;
    const int lo1 = A0 + (int)(((long long)N1 * sl) / splits), hi1 = A0 + (int)(((long long)N1 * (sl + 1)) / splits);
    if (lo1 >= hi1) return;
    const unsigned id = fv1.node_id[a];
    int lo = 0, hi = fv2.nnodes;  // lower_bound
    while (lo < hi) { const int mid = (lo + hi) >> 1; if (fv2.node_id[mid] < id) lo = mid + 1; else hi = mid; }
    if (lo >= fv2.nnodes || fv2.node_id[lo] != id) return;
    const DevFrame& KF2 = P.KF2;
    TriNode T;
    T.feat1 = fv1.feat + lo1;
    T.n1 = hi1 - lo1;
    T.f0 = fv2.off[lo];
    T.nf = fv2.off[lo + 1] - T.f0;
    // epipole of KF1's centre in KF2
    const Pose34 T1 = frame_pose(KF1), T2 = frame_pose(KF2);
    float Ow[3], C2[3];
#pragma unroll
    for (int i = 0; i < 3; i++) Ow[i] = -(((T1.m[0 * 4 + i] * T1.m[3]) + T1.m[1 * 4 + i] * T1.m[7]) + T1.m[2 * 4 + i] * T1.m[11]);
#pragma unroll
    for (int i = 0; i < 3; i++)
        C2[i] = (((T2.m[i * 4 + 0] * Ow[0]) + T2.m[i * 4 + 1] * Ow[1]) + T2.m[i * 4 + 2] * Ow[2]) + T2.m[i * 4 + 3];
    const float invz = 1.0f / C2[2];
    T.ex = KF2.fx * C2[0] * invz + KF2.cx;
    T.ey = KF2.fy * C2[1] * invz + KF2.cy;
    if (T.nf <= 128) tri_node_regs<2>(KF1, has_mp1, P, T, only_stereo, check_ori, lane);
    else if (T.nf <= 256) tri_node_regs<4>(KF1, has_mp1, P, T, only_stereo, check_ori, lane);
    else tri_node_mem(KF1, has_mp1, P, T, only_stereo, check_ori, lane);
}

// one workgroup per pair: the rotation histogram and the count of SearchForTriangulation
__global__ __launch_bounds__(1024) void k_tri_finalize(int n1, const TriPair* __restrict__ pairs, int check_ori) {
    const TriPair& P = pairs[blockIdx.x];
    finalize_block(n1, check_ori, P.hist, P.bin_of, P.match, P.nmatches);
}

// slices per node: enough waves for the chip (~4096 over all pairs) while a slice keeps ~16 KF1
// features to amortise loading the node's KF2 candidates
static int tri_splits(const DevFrame& KF1, const DevFV& fv1, int npairs) {
    const int nodes = std::max(fv1.nnodes, 1);
    const int by_chip = 4096 / std::max(nodes * npairs, 1);
    const int by_size = std::max(KF1.n / nodes / 16, 1);
    return std::max(1, std::min(std::min(by_chip, by_size), 64));
}

// per-pair scratch and outputs of the search: match rows are consecutive (pair j at
// match + j * KF1.n)
int tri_pairs_prepare(Matcher& m, const DevFrame& KF1, int npairs, TriPair* pairs_host, int* match) {
    const size_t n1 = (size_t)std::max(KF1.n, 1);
    int rc;
    if ((rc = ensure_buf(&m.d_bin_of, &m.cap_bin_of, n1 * npairs))) return rc;
    if ((rc = ensure_buf(&m.d_hist, &m.cap_hist, (size_t)HISTO_LENGTH * npairs))) return rc;
    for (int j = 0; j < npairs; j++) {
        pairs_host[j].match = match + (size_t)j * KF1.n;
        pairs_host[j].bin_of = m.d_bin_of + (size_t)j * n1;
        pairs_host[j].hist = m.d_hist + (size_t)j * HISTO_LENGTH;
    }
    return ORBMI_OK;
}

// pairs_host == nullptr: the caller prepared and uploaded the pair table (tri_pairs_prepare)
static int launch_tri_search(Matcher& m, const DevFrame& KF1, const uint8_t* has_mp1, const DevFV& fv1, int npairs,
                             TriPair* pairs_host, TriPair* pairs_dev, int only_stereo, int check_ori, int* match,
                             bool counts) {
    int rc;
    if (pairs_host) {
        if ((rc = tri_pairs_prepare(m, KF1, npairs, pairs_host, match))) return rc;
        ORBMI_HIP(m.h2d(pairs_dev, pairs_host, sizeof(TriPair) * npairs));
    }
    // the histogram is read only by the orientation check
    if (check_ori) ORBMI_HIP(hipMemsetAsync(m.d_hist, 0, (size_t)HISTO_LENGTH * npairs * sizeof(int), m.ls()));
    if (KF1.n > 0) ORBMI_HIP(hipMemsetAsync(match, 0xFF, (size_t)KF1.n * npairs * sizeof(int), m.ls()));
    if (fv1.nnodes > 0) {
        const int splits = tri_splits(KF1, fv1, npairs);
        const int waves = fv1.nnodes * splits;
        hipLaunchKernelGGL(k_tri_match, dim3((waves + 3) / 4, npairs), dim3(256), 0, m.ls(), KF1, has_mp1, fv1,
                           pairs_dev, only_stereo, check_ori, splits);
    }
    // without the orientation check and counts the finalize pass has nothing to do
    if (check_ori || counts)
        hipLaunchKernelGGL(k_tri_finalize, dim3(npairs), dim3(1024), 0, m.ls(), KF1.n, pairs_dev, check_ori);
    return ORBMI_OK;
}

int launch_triangulation(Matcher& m, const DevFrame& KF1, const uint8_t* has_mp1, const DevFV& fv1, int npairs,
                         TriPair* pairs_host, TriPair* pairs_dev, int only_stereo, int check_ori, int* match) {
    if (npairs <= 0) return ORBMI_OK;
    int rc;
    bool counts = false;
    for (int j = 0; j < npairs; j++) counts |= pairs_host[j].nmatches != nullptr;
    if ((rc = launch_tri_search(m, KF1, has_mp1, fv1, npairs, pairs_host, pairs_dev, only_stereo, check_ori, match,
                                counts)))
        return rc;
    return hipGetLastError() == hipSuccess ? ORBMI_OK : ORBMI_E_HIP;
}

// CreateNewMapPoints' triangulation on the device (tri_geom.h's tests, the code the host runs):
// thread per KF1 keypoint, visiting the pairs in the reference's order.  A keypoint whose match
// an earlier pair accepted has a map point from then on, so the reference's search of the later
// pairs skips it (`if (pMP1) continue;`): its later matches are dropped -- the searches, which
// are independent per KF1 keypoint, ran for all pairs at once on the entry flags.
__global__ __launch_bounds__(256) void k_triangulate(tri::Side K1, const tri::Side* __restrict__ K2s, int npairs,
                                                     int* __restrict__ match, int n1, uint8_t* __restrict__ ok,
                                                     float* __restrict__ x3d) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n1) return;
    bool claimed = false;
    const float cps1 = K1.ur[i] >= 0 ? K1.cos_stereo[i] : 0.f;
    for (int j = 0; j < npairs; j++) {
        const size_t r = (size_t)j * n1 + i;
        const int i2 = match[r];
        uint8_t o = 0;
        if (i2 >= 0) {
            if (claimed) {
                match[r] = -1;
            } else {
                const tri::Side& K2 = K2s[j];
                const float cps2 = K2.ur[i2] >= 0 ? K2.cos_stereo[i2] : 0.f;
                float x[3];
                if (tri::triangulate_one(K1, K2, i, i2, cps1, cps2, x)) {
                    o = 1;
                    claimed = true;
                    x3d[3 * r] = x[0];
                    x3d[3 * r + 1] = x[1];
                    x3d[3 * r + 2] = x[2];
                }
            }
        }
        ok[r] = o;
    }
}

// The same outcome with every (keypoint, pair) geometry evaluated at once: G >= npairs lanes per
// KF1 keypoint (lane j = pair j, G a power of two dividing 64), each running triangulate_one for
// its match; the first pair (in the reference's order) whose geometry accepts owns the keypoint
// -- a wave ballot -- and the later pairs' matches of it are dropped, exactly as the sequential
// loop would (an accepted point makes pKF1's keypoint taken for the searches after it, and the
// KF1 keypoints of SearchForTriangulation are independent of each other).
template <int G>
__global__ __launch_bounds__(256) void k_triangulate_par(tri::Side K1, const tri::Side* __restrict__ K2s, int npairs,
                                                         int* __restrict__ match, int n1, uint8_t* __restrict__ ok,
                                                         float* __restrict__ x3d) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    const int i = t / G, j = t % G, lane = threadIdx.x & 63;
    const bool live = i < n1 && j < npairs;
    const size_t r = (size_t)j * n1 + i;
    const int i2 = live ? match[r] : -1;
    bool acc = false;
    float x[3];
    if (i2 >= 0) {
        const tri::Side& K2 = K2s[j];
        const float cps1 = K1.ur[i] >= 0 ? K1.cos_stereo[i] : 0.f;
        const float cps2 = K2.ur[i2] >= 0 ? K2.cos_stereo[i2] : 0.f;
        acc = tri::triangulate_one(K1, K2, i, i2, cps1, cps2, x);
    }
    const unsigned long long bits = __ballot(acc);
    const unsigned long long mine = G == 64 ? bits : (bits >> (lane & ~(G - 1))) & ((1ull << G) - 1);
    const int first = mine ? __builtin_ctzll(mine) : G;  // the pair that owns keypoint i
    if (!live) return;
    if (i2 >= 0 && j > first) match[r] = -1;
    ok[r] = j == first ? 1 : 0;
    if (j == first) {
        x3d[3 * r] = x[0];
        x3d[3 * r + 1] = x[1];
        x3d[3 * r + 2] = x[2];
    }
}

int launch_create_points(Matcher& m, const DevFrame& KF1, const uint8_t* has1, const DevFV& fv1, int npairs,
                         TriPair* pairs_host, TriPair* pairs_dev, const tri::Side& S1, const tri::Side* S2_dev,
                         int* match, uint8_t* ok, float* x3d) {
    if (npairs <= 0) return ORBMI_OK;
    int rc;
    if ((rc = launch_tri_search(m, KF1, has1, fv1, npairs, pairs_host, pairs_dev, 0, 0, match, false))) return rc;
    auto par = [&](auto kern, int G) {
        const long long nt = (long long)KF1.n * G;
        hipLaunchKernelGGL(kern, dim3((unsigned)((nt + 255) / 256)), dim3(256), 0, m.ls(), S1, S2_dev, npairs, match,
                           KF1.n, ok, x3d);
    };
    if (KF1.n <= 0) {
    } else if (npairs <= 4) {
        par(k_triangulate_par<4>, 4);
    } else if (npairs <= 8) {
        par(k_triangulate_par<8>, 8);
    } else if (npairs <= 16) {
        par(k_triangulate_par<16>, 16);
    } else if (npairs <= 32) {
        par(k_triangulate_par<32>, 32);
    } else if (npairs <= 64) {
        par(k_triangulate_par<64>, 64);
    } else {
        hipLaunchKernelGGL(k_triangulate, dim3((KF1.n + 255) / 256), dim3(256), 0, m.ls(), S1, S2_dev, npairs, match,
                           KF1.n, ok, x3d);
    }
    return hipGetLastError() == hipSuccess ? ORBMI_OK : ORBMI_E_HIP;
}

// -------------------------------------------------------------------------- Fuse
// ORBmatcher::Fuse(KeyFrame*, const vector<MapPoint*>&, th) (src/ORBmatcher.cc:977-1127), the
// search: thread per candidate map point.  Projection (P10 order), KeyFrame::IsInImage, the
// scale-invariance and 60-degree viewing tests, PredictScale, KeyFrame::GetFeaturesInArea
// without level limits, the level window [pred - 1, pred], the chi2 gates on the reprojection
// error (double compares against 7.8 / 5.99) and the descriptor distance; the first keypoint of
// the reference's grid order wins ties (key dist << 40 | cell << 20 | idx).  The map updates
// (Replace / AddObservation) are the caller's sequential replay of (best_idx, best_dist) in
// list order (include/orbmi.h).
// minimum over the G lanes of a group (G = 1 or 8, groups aligned inside a DPP row)
template <int G>
__device__ inline unsigned long long group_min_u64(unsigned long long v) {
    if constexpr (G == 8) {
        unsigned long long w;
        w = dpp_mov_u64<kDppXor1>(v); v = w < v ? w : v;
        w = dpp_mov_u64<kDppXor2>(v); v = w < v ? w : v;
        w = dpp_mov_u64<kDppHalfMirror>(v); v = w < v ? w : v;
    }
    return v;
}

// candidate i of Fuse on G lanes: every lane runs the projection and the tests, the window's
// grid cells are shared out among the G lanes (cell ci on lane ci mod G), the keys meet in a
// group minimum; lane 0 of the group writes.  valid = false: the lanes only take part in the
// group minimum.
template <int G>
__device__ inline void fuse_one(const DevFrame& F, const int* __restrict__ cs, const int* __restrict__ cl,
                                const orbmi_mappoint* __restrict__ mps, const uint8_t* __restrict__ in_kf, int i,
                                bool valid, int glane, float th, int* __restrict__ best_idx,
                                int* __restrict__ best_dist, int* __restrict__ ncand) {
    int bi = -1, bd = 256;
    const orbmi_mappoint mp = mps[valid ? i : 0];
    const Pose34 T = frame_pose(F);
    float Pc[3];
    bool ok = valid && !(mp.flags & ORBMI_MP_BAD) && !(in_kf && in_kf[i]);
    if (ok) {
        transform(T.m, mp.pos, Pc);
        ok = !(Pc[2] < 0.0f);
    }
    float u = 0, v = 0, invz = 0, dist3D = 0;
    if (ok) {
        invz = 1.0f / Pc[2];
        const float x = Pc[0] * invz, y = Pc[1] * invz;
        u = F.fx * x + F.cx;
        v = F.fy * y + F.cy;
        ok = u >= F.min_x && u < F.max_x && v >= F.min_y && v < F.max_y;  // KeyFrame::IsInImage
    }
    if (ok) {
        float Ow[3];
        camera_center(T.m, Ow);
        const float maxDistance = 1.2f * mp.max_distance, minDistance = 0.8f * mp.min_distance;
        const float PO[3] = {mp.pos[0] - Ow[0], mp.pos[1] - Ow[1], mp.pos[2] - Ow[2]};
        dist3D = (float)sqrt((double)PO[0] * PO[0] + (double)PO[1] * PO[1] + (double)PO[2] * PO[2]);
        ok = !(dist3D < minDistance || dist3D > maxDistance);
        if (ok) {
            const double dot = (double)PO[0] * mp.normal[0] + (double)PO[1] * mp.normal[1] + (double)PO[2] * mp.normal[2];
            ok = !(dot < 0.5 * (double)dist3D);
        }
    }
    unsigned long long best = ~0ull;
    if (ok) {
        const float ratio = mp.max_distance / dist3D;  // MapPoint::PredictScale(dist, KeyFrame*)
        int nPredictedLevel = (int)ceilf((float)log((double)ratio) / F.log_scale_factor);
        if (nPredictedLevel < 0) nPredictedLevel = 0;
        else if (nPredictedLevel >= F.nlevels) nPredictedLevel = F.nlevels - 1;
        const float radius = th * F.scale[nPredictedLevel];
        const float ur = u - F.bf * invz;
        for_features_in_area<G>(F, cs, cl, u, v, radius, -1, -1, glane, [&](int idx, int cell) {
            const orbmi_keypoint kp = F.keys[idx];
            const int kpLevel = kp.octave;
            if (kpLevel < nPredictedLevel - 1 || kpLevel > nPredictedLevel) return;
            const float inv = 1.0f / (F.scale[kpLevel] * F.scale[kpLevel]);  // mvInvLevelSigma2
            const float ex = u - kp.x, ey = v - kp.y;
            if (F.u_right && F.u_right[idx] >= 0) {
                const float er = ur - F.u_right[idx];
                const float e2 = ex * ex + ey * ey + er * er;
                if ((double)(e2 * inv) > 7.8) return;
            } else {
                const float e2 = ex * ex + ey * ey;
                if ((double)(e2 * inv) > 5.99) return;
            }
            const unsigned long long e = cand_entry(popc_desc(mp.desc, F.desc + 32 * (long long)idx), cell, idx);
            best = e < best ? e : best;
        });
    }
    best = group_min_u64<G>(best);
    if (!valid || glane != 0) return;
    if (best != ~0ull) {
        bd = (int)(best >> 40);
        bi = (int)(best & 0xFFFFF);
    }
    const bool fused = bi >= 0 && bd <= TH_LOW;
    best_idx[i] = fused ? bi : -1;
    best_dist[i] = bi >= 0 ? bd : 256;
    // one atomic per wave: a counter shared by the whole grid serialises per-thread atomics
    const unsigned long long m = __ballot(fused);
    if (ncand && fused && (threadIdx.x & 63) == __ffsll((long long)m) - 1) atomicAdd(ncand, (int)__popcll(m));
}

constexpr int kFuseLanes = 8;  // lanes per candidate map point (a window spans a few grid cells)

__global__ __launch_bounds__(256) void k_fuse(DevFrame F, const int* __restrict__ cs, const int* __restrict__ cl,
                                              const orbmi_mappoint* __restrict__ mps, const uint8_t* __restrict__ in_kf,
                                              int n, float th, int* __restrict__ best_idx, int* __restrict__ best_dist,
                                              int* __restrict__ ncand) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x, i = t / kFuseLanes;
    fuse_one<kFuseLanes>(F, cs, cl, mps, in_kf, i, i < n, t % kFuseLanes, th, best_idx, best_dist, ncand);
}

// the same candidate list against several keyframes (grid row = keyframe)
__global__ __launch_bounds__(256) void k_fuse_multi(const FuseKF* __restrict__ kfs, const orbmi_mappoint* __restrict__ mps,
                                                    int n, float th) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x, i = t / kFuseLanes;
    const FuseKF& K = kfs[blockIdx.y];
    fuse_one<kFuseLanes>(K.F, K.cs, K.cl, mps, K.in_kf, i, i < n, t % kFuseLanes, th, K.best_idx, K.best_dist, K.ncand);
}

int launch_fuse(Matcher& m, const DevFrame& F, const orbmi_mappoint* mps, const uint8_t* in_kf, int n, float th,
                int* best_idx, int* best_dist, int* ncand) {
    int rc;
    if ((rc = grid_for(m, F))) return rc;
    if (n > 0)
        hipLaunchKernelGGL(k_fuse, dim3((n * kFuseLanes + 255) / 256), dim3(256), 0, m.ls(), F, m.cur_cs, m.cur_cl,
                           mps, in_kf, n, th, best_idx, best_dist, ncand);
    return hipGetLastError() == hipSuccess ? ORBMI_OK : ORBMI_E_HIP;
}

int launch_fuse_multi(Matcher& m, int nkf, FuseKF* kfs_host, FuseKF* kfs_dev, const orbmi_mappoint* mps, int n,
                      float th, int* best_idx, int* best_dist, int* ncand) {
    if (nkf <= 0) return ORBMI_OK;
    int ncap = 1;
    for (int k = 0; k < nkf; k++) {
        if (kfs_host[k].F.n > kGreedyMaxKp) return ORBMI_E_UNSUPPORTED;
        ncap = std::max(ncap, kfs_host[k].F.n);
    }
    int rc;
    if ((rc = ensure_buf(&m.d_mcell_start, &m.cap_mcell_start, (size_t)(kGridCells + 1) * nkf))) return rc;
    if ((rc = ensure_buf(&m.d_mcell_list, &m.cap_mcell_list, (size_t)ncap * nkf))) return rc;
    if ((rc = ensure_buf(&m.d_mkp_cell, &m.cap_mkp_cell, (size_t)ncap * nkf))) return rc;
    for (int k = 0; k < nkf; k++) {
        FuseKF& K = kfs_host[k];
        K.cs = m.d_mcell_start + (size_t)k * (kGridCells + 1);
        K.cl = m.d_mcell_list + (size_t)k * ncap;
        K.best_idx = best_idx + (size_t)k * n;
        K.best_dist = best_dist + (size_t)k * n;
        K.ncand = ncand + k;
    }
    ORBMI_HIP(m.h2d(kfs_dev, kfs_host, sizeof(FuseKF) * nkf));
    hipLaunchKernelGGL(k_grid_build_multi, dim3(nkf), dim3(1024), 0, m.ls(), kfs_dev, m.d_mkp_cell, ncap);
    if (n > 0)
        hipLaunchKernelGGL(k_fuse_multi, dim3((n * kFuseLanes + 255) / 256, nkf), dim3(256), 0, m.ls(), kfs_dev, mps, n,
                           th);
    return hipGetLastError() == hipSuccess ? ORBMI_OK : ORBMI_E_HIP;
}

// records whose descriptor was just recomputed (desc_from[i] >= 0: row of `desc`) take it
__global__ __launch_bounds__(256) void k_patch_desc(orbmi_mappoint* __restrict__ mps, const int* __restrict__ desc_from,
                                                    const uint8_t* __restrict__ desc, int n) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;  // 8 threads per record, 4 bytes each
    const int i = t >> 3, w = t & 7;
    if (i >= n) return;
    const int r = desc_from[i];
    if (r < 0) return;
    reinterpret_cast<uint32_t*>(mps[i].desc)[w] = reinterpret_cast<const uint32_t*>(desc + 32 * (size_t)r)[w];
}

int launch_patch_desc(Matcher& m, orbmi_mappoint* mps, const int* desc_from, const uint8_t* desc, int n) {
    if (n > 0) hipLaunchKernelGGL(k_patch_desc, dim3((8 * n + 255) / 256), dim3(256), 0, m.ls(), mps, desc_from, desc, n);
    return hipGetLastError() == hipSuccess ? ORBMI_OK : ORBMI_E_HIP;
}

// ---------------------------------------------------------------- MapPoint descriptor
// MapPoint::ComputeDistinctiveDescriptors (src/MapPoint.cc:247-316): one wave per map point,
// lane = row i of the N x N distance matrix (rows in chunks of 64).  The row's median
// (vDists[0.5 (N - 1)] of the sorted row, self-distance 0 included) is found by a binary search
// on the value: the smallest v with #{j : d_ij <= v} > (N - 1) / 2, 9 steps over [0, 256].  The
// best row is the minimum of (median << 16 | i): least median, first index on ties, as the
// reference's strict `median < BestMedian` scan.  The point's descriptors are read from L1/L2.
__global__ __launch_bounds__(256) void k_distinctive(const uint4* __restrict__ desc, const int* __restrict__ off,
                                                     int np, int* __restrict__ best, uint4* __restrict__ out) {
    const int p = (blockIdx.x * blockDim.x + threadIdx.x) >> 6, lane = threadIdx.x & 63;
    if (p >= np) return;  // whole waves
    const int b = off[p], N = off[p + 1] - b;
    if (N <= 0) {
        if (lane == 0) best[p] = -1;
        return;
    }
    const int k = (N - 1) / 2;  // (size_t)(0.5 * (N - 1))
    unsigned long long bestkey = ~0ull;
    for (int i0 = 0; i0 < N; i0 += 64) {
        const int i = i0 + lane;
        unsigned long long key = ~0ull;
        if (i < N) {
            const uint4 a0 = desc[2 * (b + i)], a1 = desc[2 * (b + i) + 1];
            int lo = 0, hi = 256;  // answer in [lo, hi]
            while (lo < hi) {
                const int mid = (lo + hi) >> 1;
                int c = 0;
                for (int j = 0; j < N; j++) c += popc256(a0, a1, desc[2 * (b + j)], desc[2 * (b + j) + 1]) <= mid;
                if (c > k) hi = mid;
                else lo = mid + 1;
            }
            key = (unsigned long long)lo << 32 | (unsigned)i;
        }
        key = wave_min_u64(key);
        bestkey = key < bestkey ? key : bestkey;
    }
    const int bi = (int)(unsigned)bestkey;
    if (lane == 0) best[p] = bi;
    if (lane < 2) out[2 * p + lane] = desc[2 * (b + bi) + lane];
}

int launch_distinctive(Matcher& m, const uint8_t* desc, const int* off, int np, int* best, uint8_t* out) {
    if (np <= 0) return ORBMI_OK;
    hipLaunchKernelGGL(k_distinctive, dim3((np + 3) / 4), dim3(256), 0, m.ls(), (const uint4*)desc, off, np, best,
                       (uint4*)out);
    return hipGetLastError() == hipSuccess ? ORBMI_OK : ORBMI_E_HIP;
}

}  // namespace orbmi
