// Frame::ComputeStereoMatches (src/Frame.cc:501-675) on MI355X:
//   k_stereo_rows    row table of right keypoints (:514-527)             one workgroup
//   k_stereo_match   Hamming row search + 11x11 SAD over 11 shifts + parabola (:539-659)
//                    one wave per left keypoint
//   k_stereo_filter  median(SAD) * 2.1 outlier cull (:661-674)          one workgroup
#include <algorithm>

#include "extractor.h"

namespace orbmi {

constexpr int kStereoRowsMax = 4096;

// Row lists: best match = lexicographic min (Hamming, iR) over the row's candidates, which
// is what the reference's ascending-iR scan with strict '<' yields, so the fill order inside
// a row does not matter.
__global__ __launch_bounds__(1024) void k_stereo_rows(const orbmi_keypoint* __restrict__ kpsR,
                                                      const int* __restrict__ countR, int capR,
                                                      const float* __restrict__ scale, int nrows,
                                                      int* __restrict__ row_start, int* __restrict__ row_list,
                                                      int list_cap) {
    __shared__ int cnt[kStereoRowsMax];
    __shared__ int scratch[20];
    constexpr int kRegs = 4;  // right keypoints per thread kept in registers (4096)
    const int tid = threadIdx.x;
    const int nR = min(*countR, capR);
    for (int i = tid; i < nrows; i += blockDim.x) cnt[i] = 0;
    // the row band of each right keypoint, loaded once (:514-527)
    int lo[kRegs], hi[kRegs];
#pragma unroll
    for (int k = 0; k < kRegs; k++) {
        const int i = tid + k * 1024;
        lo[k] = 0;
        hi[k] = -1;
        if (i < nR) {
            const orbmi_keypoint kp = kpsR[i];
            const float r = 2.0f * scale[kp.octave];
            lo[k] = max((int)floorf(kp.y - r), 0);
            hi[k] = min((int)ceilf(kp.y + r), nrows - 1);
        }
    }
    auto band = [&](int k, int i, int& a, int& b) {
        if (k < kRegs) { a = lo[k]; b = hi[k]; return; }
        const orbmi_keypoint kp = kpsR[i];
        const float r = 2.0f * scale[kp.octave];
        a = max((int)floorf(kp.y - r), 0);
        b = min((int)ceilf(kp.y + r), nrows - 1);
    };
    __syncthreads();
    for (int i = tid, k = 0; i < nR; i += blockDim.x, k++) {
        int a, b;
        band(k, i, a, b);
        for (int yi = a; yi <= b; yi++) atomicAdd(&cnt[yi], 1);
    }
    __syncthreads();
    // exclusive scan of cnt (4 rows per thread)
    int v[4], s = 0;
    for (int k = 0; k < 4; k++) { const int i = tid * 4 + k; v[k] = i < nrows ? cnt[i] : 0; s += v[k]; }
    int total;
    int e = block_excl_scan(s, scratch, &total);
    for (int k = 0; k < 4; k++) {
        const int i = tid * 4 + k;
        if (i < nrows) { row_start[i] = e; cnt[i] = e; }
        e += v[k];
    }
    if (tid == 0) row_start[nrows] = total;
    __syncthreads();
    for (int i = tid, k = 0; i < nR; i += blockDim.x, k++) {
        int a, b;
        band(k, i, a, b);
        for (int yi = a; yi <= b; yi++) {
            const int p = atomicAdd(&cnt[yi], 1);
            if (p < list_cap) row_list[p] = i;
        }
    }
}

struct StereoArgs {
    const orbmi_keypoint* kpsL;
    const uint8_t* descL;
    const int* countL;
    const orbmi_keypoint* kpsR;
    const uint8_t* descR;
    const uint8_t* pyrL;
    const uint8_t* pyrR;
    const LevelGeom* levels;
    const float* scale;
    const float* inv_scale;
    const int* row_start;
    const int* row_list;
    float* u_right;
    float* depth;
    int* sad;
    int capL;
    float bf, minD, maxD;
};

__global__ __launch_bounds__(256) void k_stereo_match(StereoArgs a) {
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int iL = blockIdx.x * 4 + wid;
    const int nL = min(*a.countL, a.capL);
    if (iL >= nL) return;
    const orbmi_keypoint kpL = a.kpsL[iL];
    float outU = -1.0f, outD = -1.0f;
    int outSad = -1;
    const int levelL = kpL.octave;
    const float vL = kpL.y, uL = kpL.x;
    const int row = (int)vL;
    const int c0 = a.row_start[row], c1 = a.row_start[row + 1];
    const float minU = uL - a.maxD, maxU = uL - a.minD;
    if (c1 > c0 && !(maxU < 0)) {
        const uint4* dl = reinterpret_cast<const uint4*>(a.descL + (long long)iL * 32);
        const uint4 l0 = dl[0], l1 = dl[1];
        unsigned long long best = ~0ull;
        for (int c = c0 + lane; c < c1; c += 64) {
            const int iR = a.row_list[c];
            const orbmi_keypoint kpR = a.kpsR[iR];
            if (kpR.octave < levelL - 1 || kpR.octave > levelL + 1) continue;
            const float uR = kpR.x;
            if (uR >= minU && uR <= maxU) {
                const uint4* dr = reinterpret_cast<const uint4*>(a.descR + (long long)iR * 32);
                const int dist = popc256(l0, l1, dr[0], dr[1]);
                const unsigned long long k = ((unsigned long long)dist << 32) | (unsigned)iR;
                best = k < best ? k : best;
            }
        }
        best = wave_min_u64(best);
        const int bestDist = best == ~0ull ? 100 : min(100, (int)(best >> 32));
        const int thOrbDist = (100 + 50) / 2;
        if (bestDist < thOrbDist) {
            const int bestIdxR = (int)(best & 0xFFFFFFFFu);
            const float uR0 = a.kpsR[bestIdxR].x;
            const float sf = a.inv_scale[levelL];
            const float scaleduL = roundf(kpL.x * sf);
            const float scaledvL = roundf(kpL.y * sf);
            const float scaleduR0 = roundf(uR0 * sf);
            const int w = 5, L = 5;
            const LevelGeom g = a.levels[levelL];
            const float iniu = scaleduR0 + L - w;
            const float endu = scaleduR0 + L + w + 1;
            if (!(iniu < 0 || endu >= g.W)) {
                const uint8_t* il = a.pyrL + g.off + (long long)kEdge * g.stride + kEdge;
                const uint8_t* ir = a.pyrR + g.off + (long long)kEdge * g.stride + kEdge;
                const int yl0 = (int)scaledvL - w, xl0 = (int)scaleduL - w, xr0 = (int)scaleduR0 - w;
                const int cL = il[(long long)(yl0 + w) * g.stride + xl0 + w];
                int vl[2], pr[2], pc[2];
                for (int k = 0; k < 2; k++) {
                    const int p = lane + 64 * k;
                    pr[k] = p < 121 ? p / 11 : 0;
                    pc[k] = p < 121 ? p % 11 : 0;
                    vl[k] = p < 121 ? il[(long long)(yl0 + pr[k]) * g.stride + xl0 + pc[k]] - cL : 0;
                }
                float dists[2 * 5 + 1];
                int bestincR = 0;
                int bestSad = 0x7FFFFFFF;
                for (int inc = -L; inc <= L; inc++) {
                    const int cR = ir[(long long)(yl0 + w) * g.stride + xr0 + inc + w];
                    int part = 0;
                    for (int k = 0; k < 2; k++) {
                        const int p = lane + 64 * k;
                        if (p < 121) {
                            const int vr = ir[(long long)(yl0 + pr[k]) * g.stride + xr0 + inc + pc[k]] - cR;
                            part += abs(vl[k] - vr);
                        }
                    }
                    const int dist = wave_sum_i32(part);
                    dists[L + inc] = (float)dist;
                    if ((float)dist < (float)bestSad) { bestSad = dist; bestincR = inc; }
                }
                if (bestincR != -L && bestincR != L) {
                    const float dist1 = dists[L + bestincR - 1];
                    const float dist2 = dists[L + bestincR];
                    const float dist3 = dists[L + bestincR + 1];
                    const float deltaR = (dist1 - dist3) / (2.0f * (dist1 + dist3 - 2.0f * dist2));
                    if (!(deltaR < -1 || deltaR > 1)) {
                        float bestuR = a.scale[levelL] * ((float)scaleduR0 + (float)bestincR + deltaR);
                        float disparity = uL - bestuR;
                        if (disparity >= a.minD && disparity < a.maxD) {
                            if (disparity <= 0) {
                                disparity = 0.01f;
                                bestuR = (float)((double)uL - 0.01);
                            }
                            outD = a.bf / disparity;
                            outU = bestuR;
                            outSad = bestSad;
                        }
                    }
                }
            }
        }
    }
    if (lane == 0) {
        a.u_right[iL] = outU;
        a.depth[iL] = outD;
        a.sad[iL] = outSad;
    }
}

// sort(vDistIdx); median = vDistIdx[size/2].first; drop dist >= 1.5f*1.4f*median
// The median is a two-pass radix select over the SAD values (0 <= SAD <= 121 * 255 < 2^15):
// a 256-bin histogram of v >> 7 finds the bin holding rank size/2, a 128-bin histogram of the
// low bits inside it finds the value.  The values stay in registers between the passes.
constexpr int kFilterRegs = 8;  // values per thread held in registers (8192 keypoints)
__global__ __launch_bounds__(1024) void k_stereo_filter(const int* __restrict__ countL, int capL,
                                                        const int* __restrict__ sad, float* __restrict__ u_right,
                                                        float* __restrict__ depth) {
    __shared__ int h1[256], h2[128], sel[2];
    const int tid = threadIdx.x;
    const int n = min(*countL, capL);
    int v[kFilterRegs];
#pragma unroll
    for (int k = 0; k < kFilterRegs; k++) {
        const int i = tid + k * 1024;
        v[k] = i < n ? sad[i] : -1;
    }
    auto for_values = [&](auto&& f) {
#pragma unroll
        for (int k = 0; k < kFilterRegs; k++) f(tid + k * 1024, v[k]);
        for (int i = tid + kFilterRegs * 1024; i < n; i += 1024) f(i, sad[i]);
    };
    if (tid < 256) h1[tid] = 0;
    if (tid < 128) h2[tid] = 0;
    __syncthreads();
    for_values([&](int, int x) { if (x >= 0) atomicAdd(&h1[min(x >> 7, 255)], 1); });
    __syncthreads();
    auto select = [&](const int* h, int nb, int rank_in, int* bin, int* rest, int* total) {
        // wave 0: bins in lane order (nb / 64 per lane), prefix, the bin holding rank_in
        const int per = nb / 64;
        int c[4], s = 0;
        for (int j = 0; j < per; j++) { c[j] = h[tid * per + j]; s += c[j]; }
        const int incl = wave_incl_scan(s);
        *total = __builtin_amdgcn_readlane(incl, 63);
        const int rank = rank_in < 0 ? *total / 2 : rank_in;
        int before = incl - s;
        for (int j = 0; j < per; j++) {
            if (rank >= before && rank < before + c[j]) { *bin = tid * per + j; *rest = rank - before; }
            before += c[j];
        }
    };
    if (tid < 64) {
        int bin = -1, rest = 0, M = 0;
        select(h1, 256, -1, &bin, &rest, &M);
        if (M == 0 && tid == 0) sel[0] = -1;  // reference: median of an empty vector (UB); "no filter"
        if (bin >= 0) { sel[0] = bin; sel[1] = rest; }
    }
    __syncthreads();
    const int b1 = sel[0], r1 = sel[1];
    if (b1 < 0) return;
    for_values([&](int, int x) { if (x >= 0 && (x >> 7) == b1) atomicAdd(&h2[x & 127], 1); });
    __syncthreads();
    if (tid < 64) {
        int bin = -1, rest = 0, M = 0;
        select(h2, 128, r1, &bin, &rest, &M);
        if (bin >= 0) sel[0] = (b1 << 7) | bin;
    }
    __syncthreads();
    const float median = (float)sel[0];
    const float thDist = 1.5f * 1.4f * median;
    for_values([&](int i, int x) {
        if (i < n && x >= 0 && !((float)x < thDist)) { u_right[i] = -1; depth[i] = -1; }
    });
}

int stereo_run(Extractor& Lx, int itemL, Extractor& Rx, int itemR, float bf, float fx, float* d_u,
               float* d_depth, int cap) {
    ORBMI_HIP(hipSetDevice(Lx.device));
    const int nrows = Lx.levels[0].H;
    if (nrows + 1 > kStereoRowsMax) return ORBMI_E_UNSUPPORTED;
    const int capR = Rx.last_capacity, capL = Lx.last_capacity;
    const int list_cap = capR * 24;  // rows per right keypoint <= 2*ceil(2*scale)+2
    int rc;
    if ((rc = ensure_buf(&Lx.d_row_start, &Lx.row_cap, (size_t)nrows + 1))) return rc;
    if ((rc = ensure_buf(&Lx.d_row_list, &Lx.row_list_cap, (size_t)list_cap))) return rc;
    if ((rc = ensure_buf(&Lx.d_sad, &Lx.sad_cap, (size_t)capL))) return rc;
    const orbmi_keypoint* kpsR = Rx.last_kps + (long long)itemR * capR;
    hipEvent_t ev = Lx.prof_begin(ORBMI_STAGE_STEREO_ROWS);
    hipLaunchKernelGGL(k_stereo_rows, dim3(1), dim3(1024), 0, Lx.stream, kpsR, Rx.last_counts + itemR, capR,
                       Lx.d_scale_tab, nrows, Lx.d_row_start, Lx.d_row_list, list_cap);
    Lx.prof_end(ORBMI_STAGE_STEREO_ROWS, ev);
    StereoArgs a;
    a.kpsL = Lx.last_kps + (long long)itemL * capL;
    a.descL = Lx.last_desc + (long long)itemL * capL * 32;
    a.countL = Lx.last_counts + itemL;
    a.kpsR = kpsR;
    a.descR = Rx.last_desc + (long long)itemR * capR * 32;
    a.pyrL = Lx.d_pyr + (long long)itemL * Lx.pimg;
    a.pyrR = Rx.d_pyr + (long long)itemR * Rx.pimg;
    a.levels = Lx.d_levels;
    a.scale = Lx.d_scale_tab;
    a.inv_scale = Lx.d_scale_tab + Lx.nlevels;
    a.row_start = Lx.d_row_start;
    a.row_list = Lx.d_row_list;
    a.u_right = d_u;
    a.depth = d_depth;
    a.sad = Lx.d_sad;
    a.capL = std::min(cap, capL);
    a.bf = bf;
    const float mb = bf / fx;  // Frame::mb
    a.minD = 0;                // minD = 0           (src/Frame.cc:532)
    a.maxD = bf / mb;          // maxD = mbf / minZ  (src/Frame.cc:533)
    ev = Lx.prof_begin(ORBMI_STAGE_STEREO_MATCH);
    hipLaunchKernelGGL(k_stereo_match, dim3((a.capL + 3) / 4), dim3(256), 0, Lx.stream, a);
    Lx.prof_end(ORBMI_STAGE_STEREO_MATCH, ev);
    ev = Lx.prof_begin(ORBMI_STAGE_STEREO_FILTER);
    hipLaunchKernelGGL(k_stereo_filter, dim3(1), dim3(1024), 0, Lx.stream, a.countL, a.capL, Lx.d_sad, d_u,
                       d_depth);
    Lx.prof_end(ORBMI_STAGE_STEREO_FILTER, ev);
    ORBMI_HIP(hipGetLastError());
    return ORBMI_OK;
}

}  // namespace orbmi
