// MI355X (gfx950) ORB extractor: ORBextractor::operator() (src/ORBextractor.cc:1043-1105)
// as five kernel stages over a batch of images resident in HBM:
//   k_pyr_level0 / k_pyr_resize   ComputePyramid            (:1107-1132)    one launch/level
//   k_fast                        cell FAST + NMS + fallback (:778-829)      one WG per cell
//   k_octree                      DistributeOctTree          (:539-763)      one WG per level
//   k_describe                    IC_Angle + GaussianBlur + computeOrbDescriptor (:77-147,
//                                 :1076-1104)                               one wave per keypoint
// Results are bit-exact with the pinned CPU restatement (oracle/, DESIGN.md "Pinned semantics").
#include <algorithm>
#include <cmath>
#include <cstring>

#include "../../include/orbmi_pattern.h"
#include "extractor.h"

namespace orbmi {

__constant__ signed char c_pattern[256][4];
__constant__ signed char c_circle[768][2];  // (u, v) of the 749 IC_Angle patch pixels
__constant__ int c_ncircle;

// ------------------------------------------------------------------------------ pyramid
// Level 0: copyMakeBorder(image, 19, BORDER_REFLECT_101) (src/ORBextractor.cc:1128-1129).
__global__ void k_pyr_level0(const uint8_t* __restrict__ img, size_t step, size_t img_stride,
                             uint8_t* __restrict__ pyr, long long pimg, LevelGeom g) {
    const int xp = blockIdx.x * blockDim.x + threadIdx.x, yp = blockIdx.y, b = blockIdx.z;
    if (xp >= g.W + 2 * kEdge) return;
    const int ix = reflect101(xp - kEdge, g.W), iy = reflect101(yp - kEdge, g.H);
    pyr[b * pimg + g.off + (long long)yp * g.stride + xp] = img[b * img_stride + (size_t)iy * step + ix];
}

// Level l: resize(level l-1, INTER_LINEAR) then copyMakeBorder(REFLECT_101|ISOLATED)
// (src/ORBextractor.cc:1118-1124).  Border pixels recompute the interior pixel they mirror.
__global__ void k_pyr_resize(uint8_t* __restrict__ pyr, long long pimg, LevelGeom s, LevelGeom d,
                             const XTab* __restrict__ xt, const YTab* __restrict__ yt) {
    const int xp = blockIdx.x * blockDim.x + threadIdx.x, yp = blockIdx.y, b = blockIdx.z;
    if (xp >= d.W + 2 * kEdge) return;
    const int ix = reflect101(xp - kEdge, d.W), iy = reflect101(yp - kEdge, d.H);
    const uint8_t* src = pyr + b * pimg + s.off + (long long)kEdge * s.stride + kEdge;
    const XTab x = xt[ix];
    const YTab y = yt[iy];
    const uint8_t* r0 = src + (long long)y.y0 * s.stride;
    const uint8_t* r1 = src + (long long)y.y1 * s.stride;
    const int h0 = r0[x.sx0] * x.a0 + r0[x.sx1] * x.a1;
    const int h1 = r1[x.sx0] * x.a0 + r1[x.sx1] * x.a1;
    int v;
    if (ix < d.resize_xv)  // VResizeLinearVec_32s8u (SSE2) lanes
        v = ((((h0 >> 4) * y.b0) >> 16) + (((h1 >> 4) * y.b1) >> 16) + 2) >> 2;
    else
        v = (h0 * y.b0 + h1 * y.b1 + (1 << 21)) >> 22;
    v = v < 0 ? 0 : (v > 255 ? 255 : v);
    pyr[b * pimg + d.off + (long long)yp * d.stride + xp] = (uint8_t)v;
}

// ------------------------------------------------------------------------------ FAST
constexpr int kTile = 64;  // max cell ROI edge (wCell+6, hCell+6)

// LDS writes of this wave visible to its own later reads (wave-private LDS regions)
__device__ inline void wave_sync_lds_ex() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ inline int fast_score16_p(const uint8_t* t, int pitch, int x, int y, int th) {
    // OpenCV offsets16: (dx,dy) of the radius-3 Bresenham circle.
    const int o[16][2] = {{0, 3}, {1, 3}, {2, 2}, {3, 1}, {3, 0}, {3, -1}, {2, -2}, {1, -3},
                          {0, -3}, {-1, -3}, {-2, -2}, {-3, -1}, {-3, 0}, {-3, 1}, {-2, 2}, {-1, 3}};
    const int v = t[y * pitch + x];
    int p[16];
    unsigned bright = 0, dark = 0;
#pragma unroll
    for (int k = 0; k < 16; k++) {
        p[k] = t[(y + o[k][1]) * pitch + x + o[k][0]];
        bright |= (unsigned)(p[k] > v + th) << k;
        dark |= (unsigned)(p[k] < v - th) << k;
    }
    auto arc9 = [](unsigned m) {
        unsigned m2 = m | (m << 16), r = m2;
#pragma unroll
        for (int s = 1; s <= 8; s++) r &= m2 >> s;
        return (r & 0xFFFFu) != 0;
    };
    if (!arc9(bright) && !arc9(dark)) return 0;
    // cornerScore<16>  (OpenCV fast_score.cpp), d[k] = v - p[k mod 16], k < 25
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
    return (-b0 - 1) & 0xFF;  // stored as uchar (FAST_t: curr[j] = (uchar)cornerScore)
}

__device__ inline bool nms_keep(const uint8_t* sc, int x, int y) {
    const int s = sc[y * kTile + x];
    if (!s) return false;
    return s > sc[(y - 1) * kTile + x - 1] && s > sc[(y - 1) * kTile + x] && s > sc[(y - 1) * kTile + x + 1] &&
           s > sc[y * kTile + x - 1] && s > sc[y * kTile + x + 1] &&
           s > sc[(y + 1) * kTile + x - 1] && s > sc[(y + 1) * kTile + x] && s > sc[(y + 1) * kTile + x + 1];
}

// One wave per (image, cell), four cells per workgroup, so every step syncs at wave level only.
// The cell ROI (<= 64 x 64) is staged in the wave's LDS as aligned dwords (its first byte at a
// per-cell offset 0..3); scores, strict 3x3 NMS, and a ballot compaction that emits the
// survivors row-major (FAST_t emission order) as x | y << 12 | score << 24 with x, y relative to
// minBorder (:820-825).  A cell retries with min_th when ini_th finds nothing (:804-817).
constexpr int kFastCells = 4;           // waves (cells) per workgroup
constexpr int kTileS = 68;              // LDS row pitch of a staged ROI row (17 dwords)
__global__ __launch_bounds__(64 * kFastCells) void k_fast(const uint8_t* __restrict__ pyr, long long pimg,
                                                          const LevelGeom* __restrict__ levels,
                                                          const CellGeom* __restrict__ cells, int ncells,
                                                          uint32_t* __restrict__ slots, int nslots,
                                                          int* __restrict__ cell_counts, int ini_th, int min_th) {
    __shared__ unsigned tiles[kFastCells][kTile * kTileS / 4];
    __shared__ uint8_t scores[kFastCells][kTile * kTile];
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int c = blockIdx.x * kFastCells + wid, b = blockIdx.y;
    if (c >= ncells) return;
    const CellGeom cg = cells[c];
    if (cg.w == 0) {
        if (lane == 0) cell_counts[b * ncells + c] = 0;
        return;
    }
    const LevelGeom lg = levels[cg.level];
    const long long a = b * pimg + lg.off + (long long)(kEdge + cg.y0) * lg.stride + kEdge + cg.x0;
    const int o = (int)(a & 3);  // stride is a multiple of 64: the same offset on every row
    const unsigned* src = reinterpret_cast<const unsigned*>(pyr + (a - o));
    const int w = cg.w, h = cg.h, nd = (w + o + 3) >> 2, s4 = lg.stride >> 2;
    unsigned* t4 = tiles[wid];
    {
        unsigned v[(kTile * 17 + 63) / 64];
#pragma unroll
        for (int k = 0; k < (kTile * 17 + 63) / 64; k++) {
            const int i = lane + 64 * k, r = i / nd, d = i - r * nd;
            v[k] = r < h ? src[(long long)r * s4 + d] : 0u;
        }
#pragma unroll
        for (int k = 0; k < (kTile * 17 + 63) / 64; k++) {
            const int i = lane + 64 * k, r = i / nd, d = i - r * nd;
            if (r < h) t4[r * (kTileS / 4) + d] = v[k];
        }
    }
    // fast_score16 / nms_keep address a kTile-pitched tile: re-pack the staged rows
    uint8_t* sc = scores[wid];
    wave_sync_lds_ex();
    const uint8_t* tb = reinterpret_cast<const uint8_t*>(t4) + o;  // tb[y * kTileS + x]
    const int dw = w - 6, dh = h - 6, npix = dw > 0 && dh > 0 ? dw * dh : 0;
    int total = 0;
    for (int pass = 0; pass < 2; pass++) {
        int th = pass == 0 ? ini_th : min_th;
        th = min(max(th, 0), 255);
        for (int i = lane; i < kTile * h; i += 64) sc[i] = 0;
        wave_sync_lds_ex();
        for (int p = lane; p < npix; p += 64) {
            const int y = 3 + p / dw, x = 3 + p % dw;
            sc[y * kTile + x] = (uint8_t)fast_score16_p(tb, kTileS, x, y, th);
        }
        wave_sync_lds_ex();
        total = 0;
        for (int p0 = 0; p0 < npix; p0 += 64) {
            const int p = p0 + lane;
            const bool k = p < npix && nms_keep(sc, 3 + p % dw, 3 + p / dw);
            total += __popcll(__ballot(k));
        }
        if (total > 0) break;
    }
    if (total > 0) {
        uint32_t* out = slots + (long long)b * nslots + cg.slot_base;
        int r = 0;
        for (int p0 = 0; p0 < npix; p0 += 64) {
            const int p = p0 + lane;
            const int y = 3 + p / dw, x = 3 + p % dw;
            const bool k = p < npix && nms_keep(sc, x, y);
            const unsigned long long m = __ballot(k);
            if (k)
                out[r + __popcll(m & ((1ull << lane) - 1))] =
                    (uint32_t)(x + cg.sx) | ((uint32_t)(y + cg.sy) << 12) | ((uint32_t)sc[y * kTile + x] << 24);
            r += __popcll(m);
        }
    }
    if (lane == 0) cell_counts[b * ncells + c] = total;
}

// ------------------------------------------------------------------------------ octree
// DistributeOctTree (src/ORBextractor.cc:539-763) as data-parallel passes inside one
// workgroup per (image, level).  The std::list of nodes is kept as arrays in list order:
// a pass that divides D nodes pushes their non-empty children to the list front in visit
// order, so the new list is [children in reverse push order] ++ [undivided nodes in order]
// -- two prefix scans.  Keys never move: each key carries the index of its node, remapped
// after every pass through the parent's (node, quadrant) -> child table.
constexpr int kOctThreads = 1024;
constexpr int kOctRegKeys = 16;  // candidates per thread held in registers (16,384 per level)
#ifdef ORBMI_OCT_TRACE  // tools/octree_trace.hip: s_memtime stamps of (level 0, image 0)
__device__ unsigned long long g_oct_trace[256];
#define OCT_STAMP(i, v)                                                                      \
    do {                                                                                     \
        if (threadIdx.x == 0 && blockIdx.x == 0 && blockIdx.y == 0) g_oct_trace[i] = (v);    \
    } while (0)
#define OCT_SUB(it, j) do { if ((it) < 15) OCT_STAMP(100 + 10 * (it) + (j), __builtin_amdgcn_s_memtime()); } while (0)
#else
#define OCT_STAMP(i, v) do {} while (0)
#define OCT_SUB(it, j) do {} while (0)
#endif

struct OctShared {
    short4 box[2][kOctNodeCap];          // x0, y0, x1, y1 (UL = (x0,y0), BR = (x1,y1))
    int cnt[2][kOctNodeCap];
    int ccnt[kOctNodeCap][4];            // child key counts; reused as best-key words
    short remap[kOctNodeCap][4];         // (old node, quadrant) -> new index
    unsigned long long skey[kOctNodeCap];
    int tmp[kOctNodeCap];
    int newpos[kOctNodeCap];
    unsigned char dflag[kOctNodeCap];
    int scratch[kOctThreads / 64 + 2];
    int misc[8];
};

__device__ inline int quadrant(short4 bx, int x, int y) {
    const int halfX = (int)ceilf((float)(bx.z - bx.x) / 2);
    const int halfY = (int)ceilf((float)(bx.w - bx.y) / 2);
    return (x >= bx.x + halfX ? 1 : 0) | (y >= bx.y + halfY ? 2 : 0);
}

__device__ inline short4 child_box(short4 bx, int q) {
    const short mx = (short)(bx.x + (int)ceilf((float)(bx.z - bx.x) / 2));
    const short my = (short)(bx.y + (int)ceilf((float)(bx.w - bx.y) / 2));
    switch (q) {
        case 0: return make_short4(bx.x, bx.y, mx, my);
        case 1: return make_short4(mx, bx.y, bx.z, my);
        case 2: return make_short4(bx.x, my, mx, bx.w);
        default: return make_short4(mx, my, bx.z, bx.w);
    }
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

__global__ __launch_bounds__(kOctThreads) void k_octree(const LevelGeom* __restrict__ levels,
                                                         int nlevels, int ncells,
                                                         const int* __restrict__ cell_counts,
                                                         const CellGeom* __restrict__ cells,
                                                         const uint32_t* __restrict__ slots, int nslots,
                                                         uint32_t* __restrict__ keys,
                                                         uint16_t* __restrict__ node_of, int keys_cap,
                                                         uint2* __restrict__ oct_out, int out_cap,
                                                         int* __restrict__ oct_count) {
    __shared__ OctShared S;
    const int level = blockIdx.x, b = blockIdx.y, tid = threadIdx.x;
    const LevelGeom g = levels[level];
    const int c0 = g.cell_begin, nc = g.cell_end - g.cell_begin;
    const int* cnts = cell_counts + b * ncells + c0;
    uint32_t* K = keys + (long long)b * keys_cap + g.key_base;
    uint16_t* NO = node_of + (long long)b * keys_cap + g.key_base;

    OCT_STAMP(0, __builtin_amdgcn_s_memtime());
    // ---- gather candidates in original order (cells row-major, FAST order inside a cell):
    // thread t holds keys t R .. t R + R - 1 in registers (R = kOctRegKeys, neighbours in the
    // image, so a thread's increments mostly hit one counter); keys from kOctThreads R on
    // spill to K / NO in global memory.  A key finds its cell by a binary search over
    // the prefix of the cell counts, so every load of the gather is in flight at once.
    uint32_t kreg[kOctRegKeys];
    int nreg[kOctRegKeys];
#pragma unroll
    for (int r = 0; r < kOctRegKeys; r++) { kreg[r] = 0; nreg[r] = 0; }
    int nkeys = 0;
    for (int base = 0; base < nc; base += kOctNodeCap) {
        const int n = min(kOctNodeCap, nc - base);
        for (int i = tid; i < n; i += blockDim.x) {
            S.tmp[i] = cnts[base + i];
            S.newpos[i] = cells[c0 + base + i].slot_base;
        }
        __syncthreads();
        const int tot = block_scan_array(S.tmp, n, S.scratch);
        auto cell_of = [&](int kk) {  // kk in [0, tot): upper_bound over the prefix, minus one
            int lo = 0, hi = n;
            while (hi - lo > 1) {
                const int mid = (lo + hi) >> 1;
                if (S.tmp[mid] <= kk) lo = mid;
                else hi = mid;
            }
            return lo;
        };
        auto fetch = [&](int kk) -> uint32_t {
            const int lo = cell_of(kk);
            return slots[(long long)b * nslots + S.newpos[lo] + (kk - S.tmp[lo])];
        };
        {
            // one search for the thread's first key, then walk the cells forward; all slot
            // addresses first, then the loads
            const int k0 = tid * kOctRegKeys;
            const int kk0 = max(k0 - nkeys, 0);
            int lo = kk0 < tot ? cell_of(kk0) : 0;
            long long addr[kOctRegKeys];
#pragma unroll
            for (int r = 0; r < kOctRegKeys; r++) {
                const int kk = k0 + r - nkeys;
                addr[r] = -1;
                if (kk >= 0 && kk < tot) {
                    while (lo + 1 < n && S.tmp[lo + 1] <= kk) lo++;
                    addr[r] = (long long)b * nslots + S.newpos[lo] + (kk - S.tmp[lo]);
                }
            }
#pragma unroll
            for (int r = 0; r < kOctRegKeys; r++)
                if (addr[r] >= 0) kreg[r] = slots[addr[r]];
        }
        for (int k = tid + kOctThreads * kOctRegKeys; k < nkeys + tot; k += kOctThreads)
            if (k >= nkeys) K[k] = fetch(k - nkeys);
        nkeys += tot;
        __syncthreads();
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
            int no = NO[k];
            f(k, K[k], no);
            NO[k] = (uint16_t)no;
        }
    };

    OCT_STAMP(1, __builtin_amdgcn_s_memtime());
    OCT_STAMP(62, nkeys);
    // ---- initial nodes (:543-579)
    const int nIni = g.nIni;
    int cur = 0;
    for (int i = tid; i < nIni; i += blockDim.x) {
        S.box[cur][i] = make_short4((short)(int)(g.hX * (float)i), 0, (short)(int)(g.hX * (float)(i + 1)),
                                    (short)g.height);
        S.cnt[cur][i] = 0;
    }
    __syncthreads();
    {
        int run = -1, rc = 0;  // consecutive keys of a thread share a node: one atomic per run
        for_keys([&](int, uint32_t key, int& no) {
            int n = (int)((float)(key & 0xFFF) / g.hX);
            n = min(n, nIni - 1);
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
    // drop empty initial nodes (:581-593)
    for (int i = tid; i < nIni; i += blockDim.x) S.tmp[i] = S.cnt[cur][i] > 0;
    __syncthreads();
    int L = block_scan_array(S.tmp, nIni, S.scratch);
    for (int i = tid; i < nIni; i += blockDim.x) {
        const short ni = S.cnt[cur][i] > 0 ? (short)S.tmp[i] : (short)-1;
        S.remap[i][0] = S.remap[i][1] = S.remap[i][2] = S.remap[i][3] = ni;
        if (ni >= 0) { S.box[cur ^ 1][ni] = S.box[cur][i]; S.cnt[cur ^ 1][ni] = S.cnt[cur][i]; }
    }
    cur ^= 1;
    __syncthreads();

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
        __syncthreads();
        OCT_SUB(iter, 0);
        // keys: apply the previous pass's remap, then histogram children of nodes with >1 key
        {
            // register keys: every LDS read of the pass first (independent across keys), then
            // one atomic per run of equal (node, quadrant) -- atomics would serialise the reads
            // branch-free (absent keys read node 0 and are masked), so the compiler can
            // interleave the LDS round trips of all kOctRegKeys keys
            // staged: all box reads, then all remap reads, then all child reads (absent keys
            // carry key 0 / node 0 and are masked at the end)
            int tgt[kOctRegKeys];
            short4 bx[kOctRegKeys];
#pragma unroll
            for (int r = 0; r < kOctRegKeys; r++) bx[r] = S.box[prv][nreg[r]];
#pragma unroll
            for (int r = 0; r < kOctRegKeys; r++)
                tgt[r] = S.remap[nreg[r]][quadrant(bx[r], kreg[r] & 0xFFF, (kreg[r] >> 12) & 0xFFF)];
            int cn[kOctRegKeys];
#pragma unroll
            for (int r = 0; r < kOctRegKeys; r++) {
                nreg[r] = max(tgt[r], 0);
                bx[r] = S.box[cur][nreg[r]];
                cn[r] = S.cnt[cur][nreg[r]];
            }
#pragma unroll
            for (int r = 0; r < kOctRegKeys; r++) {
                const bool v = tid * kOctRegKeys + r < nkeys;
                const int t = 4 * nreg[r] + quadrant(bx[r], kreg[r] & 0xFFF, (kreg[r] >> 12) & 0xFFF);
                tgt[r] = (v && cn[r] >= 2) ? t : -1;
            }
            OCT_SUB(iter, 6);
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
                const uint32_t key = K[k];
                const int x = key & 0xFFF, y = (key >> 12) & 0xFFF;
                const int o = NO[k];
                const int n = S.remap[o][quadrant(S.box[prv][o], x, y)];
                NO[k] = (uint16_t)n;
                if (S.cnt[cur][n] >= 2) atomicAdd(&S.ccnt[n][quadrant(S.box[cur][n], x, y)], 1);
            }
            OCT_SUB(iter, 8);
        }
        __syncthreads();
        OCT_SUB(iter, 1);
        // which nodes divide, and in which push order
        int ncand = 0, kdiv = 0;
        if (!careful) {
            for (int i = tid; i < L; i += blockDim.x) {
                const bool d = S.cnt[cur][i] >= 2;
                S.dflag[i] = d;
                S.tmp[i] = d ? (S.ccnt[i][0] > 0) + (S.ccnt[i][1] > 0) + (S.ccnt[i][2] > 0) + (S.ccnt[i][3] > 0) : 0;
            }
            __syncthreads();
            block_scan_array(S.tmp, L, S.scratch);  // push base in list order
            for (int i = tid; i < L; i += blockDim.x) S.newpos[i] = S.tmp[i];
        } else {
            // vSizeAndPointerToNode sorted by (size, creation); divided largest first (:681-733)
            {
                int np2 = 2;
                while (np2 < L) np2 <<= 1;
                for (int i = tid; i < np2; i += blockDim.x) {
                    unsigned long long key = ~0ull;
                    if (i < L && S.cnt[cur][i] >= 2)
                        key = ((unsigned long long)(0xFFFFFFFFu - (unsigned)S.cnt[cur][i]) << 32) | (unsigned)i;
                    S.skey[i] = key;
                }
                if (tid == 0) S.misc[0] = 0;
                __syncthreads();
                for (int i = tid; i < L; i += blockDim.x)
                    if (S.cnt[cur][i] >= 2) atomicAdd(&S.misc[0], 1);
                bitonic_sort(S.skey, np2);
                ncand = S.misc[0];
            }
            for (int r = tid; r < ncand; r += blockDim.x) {
                const int n = (int)(S.skey[r] & 0xFFFFFFFFu);
                S.tmp[r] = (S.ccnt[n][0] > 0) + (S.ccnt[n][1] > 0) + (S.ccnt[n][2] > 0) + (S.ccnt[n][3] > 0) - 1;
            }
            if (tid == 0) S.misc[1] = ncand;
            __syncthreads();
            block_scan_array(S.tmp, ncand, S.scratch);  // exclusive prefix of (m - 1)
            for (int r = tid; r < ncand; r += blockDim.x) {
                const int n = (int)(S.skey[r] & 0xFFFFFFFFu);
                const int m = (S.ccnt[n][0] > 0) + (S.ccnt[n][1] > 0) + (S.ccnt[n][2] > 0) + (S.ccnt[n][3] > 0);
                if (L + S.tmp[r] + m - 1 >= N) atomicMin(&S.misc[1], r + 1);
            }
            __syncthreads();
            kdiv = S.misc[1];
            for (int i = tid; i < L; i += blockDim.x) S.dflag[i] = 0;
            __syncthreads();
            for (int r = tid; r < ncand; r += blockDim.x) {
                const int n = (int)(S.skey[r] & 0xFFFFFFFFu);
                const int m = (S.ccnt[n][0] > 0) + (S.ccnt[n][1] > 0) + (S.ccnt[n][2] > 0) + (S.ccnt[n][3] > 0);
                S.tmp[r] = r < kdiv ? m : 0;
                if (r < kdiv) S.dflag[n] = 1;
            }
            __syncthreads();
            block_scan_array(S.tmp, ncand, S.scratch);
            for (int r = tid; r < kdiv; r += blockDim.x) S.newpos[(int)(S.skey[r] & 0xFFFFFFFFu)] = S.tmp[r];
        }
        __syncthreads();
        OCT_SUB(iter, 2);
        // P = total pushes; survivors ranked in list order
        int P = 0;
        {
            int local = 0;
            for (int i = tid; i < L; i += blockDim.x)
                if (S.dflag[i]) local += (S.ccnt[i][0] > 0) + (S.ccnt[i][1] > 0) + (S.ccnt[i][2] > 0) + (S.ccnt[i][3] > 0);
            block_excl_scan(local, S.scratch, &P);
        }
        for (int i = tid; i < L; i += blockDim.x) S.tmp[i] = !S.dflag[i];
        __syncthreads();
        const int nsurv = block_scan_array(S.tmp, L, S.scratch);
        OCT_SUB(iter, 3);
        int nexp_local = 0;
        for (int i = tid; i < L; i += blockDim.x) {
            if (S.dflag[i]) {
                int p = S.newpos[i];
                const short4 bx = S.box[cur][i];
                for (int q = 0; q < 4; q++) {
                    const int c = S.ccnt[i][q];
                    if (c > 0) {
                        const int ni = P - 1 - p++;
                        if (ni < kOctNodeCap) {  // bound proven in DESIGN.md; guard LDS anyway
                            S.box[prv][ni] = child_box(bx, q);
                            S.cnt[prv][ni] = c;
                        }
                        S.remap[i][q] = (short)min(ni, kOctNodeCap - 1);
                        nexp_local += c > 1;
                    } else {
                        S.remap[i][q] = -1;
                    }
                }
            } else {
                const int ni = min(P + S.tmp[i], kOctNodeCap - 1);
                S.box[prv][ni] = S.box[cur][i];
                S.cnt[prv][ni] = S.cnt[cur][i];
                S.remap[i][0] = S.remap[i][1] = S.remap[i][2] = S.remap[i][3] = (short)ni;
            }
        }
        OCT_SUB(iter, 4);
        int nToExpand = 0;
        block_excl_scan(nexp_local, S.scratch, &nToExpand);
        OCT_SUB(iter, 5);
        const int newL = min(P + nsurv, kOctNodeCap);
        // the remap just written refers to the boxes of list `cur`; keys apply it next pass
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
    // one 64-bit max per node over score << 56 | (2^20 - 1 - k) << 24 | (y << 12 | x)
    const int prv = cur ^ 1;
    unsigned long long* best = reinterpret_cast<unsigned long long*>(&S.ccnt[0][0]);  // 2 per row
    for (int i = tid; i < L; i += blockDim.x) best[2 * i] = 0;
    __syncthreads();
    {
        int fn[kOctRegKeys];  // final node of each register key, all reads first
        short4 bx[kOctRegKeys];
#pragma unroll
        for (int r = 0; r < kOctRegKeys; r++) bx[r] = S.box[prv][nreg[r]];
#pragma unroll
        for (int r = 0; r < kOctRegKeys; r++) {
            const bool v = tid * kOctRegKeys + r < nkeys;
            const int n = S.remap[nreg[r]][quadrant(bx[r], kreg[r] & 0xFFF, (kreg[r] >> 12) & 0xFFF)];
            fn[r] = v ? n : -1;
        }
#pragma unroll
        for (int r = 0; r < kOctRegKeys; r++) {
            const int k = tid * kOctRegKeys + r;
            const uint32_t key = kreg[r];
            if (fn[r] >= 0)
                atomicMax(&best[2 * fn[r]], ((unsigned long long)(key >> 24) << 56) |
                                                ((unsigned long long)(0xFFFFFu - (unsigned)k) << 24) | (key & 0xFFFFFFu));
        }
        for (int k = tid + kOctThreads * kOctRegKeys; k < nkeys; k += kOctThreads) {
            const uint32_t key = K[k];
            const int o = NO[k];
            const int n = S.remap[o][quadrant(S.box[prv][o], key & 0xFFF, (key >> 12) & 0xFFF)];
            atomicMax(&best[2 * n], ((unsigned long long)(key >> 24) << 56) |
                                        ((unsigned long long)(0xFFFFFu - (unsigned)k) << 24) | (key & 0xFFFFFFu));
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
// x0 - 3 sits at a 16-B boundary), row sums in LDS, 4x4 outputs per thread stored as dwords
// into the interior-only blurred layout.
constexpr int kBlurInH = kBlurTH + 6, kBlurChunks = (kBlurTW + 6 + 15) / 16;  // 38 rows x 9 x 16 B
constexpr int kBlurInS = 16 * kBlurChunks;                                     // 144
__global__ __launch_bounds__(256) void k_blur(const uint8_t* __restrict__ pyr, uint8_t* __restrict__ blur,
                                              long long pimg, long long bimg, const LevelGeom* __restrict__ levels,
                                              const int2* __restrict__ tiles) {
    __shared__ uint4 in4[kBlurInH * kBlurChunks];
    __shared__ int rs[kBlurInH][kBlurTW];
    const uint8_t* in = reinterpret_cast<const uint8_t*>(in4);
    const int2 t = tiles[blockIdx.x];
    const int b = blockIdx.y, tid = threadIdx.x;
    const LevelGeom g = levels[t.x];
    const int x0 = t.y & 0xFFFF, y0 = t.y >> 16;
    const uint8_t* lvl = pyr + b * pimg + g.off + kEdge - 3 + x0;  // column x0 - 3 of padded row 0
    for (int i = tid; i < kBlurInH * kBlurChunks; i += 256) {
        const int r = i / kBlurChunks, ch = i - r * kBlurChunks;
        const int yy = min(y0 - 3 + r, g.H + 2);  // rows past H + 2 feed only discarded outputs
        in4[i] = *reinterpret_cast<const uint4*>(lvl + (long long)(kEdge + yy) * g.stride + 16 * ch);
    }
    __syncthreads();
    // row sums: one (row, 16 columns) run per task
    for (int task = tid; task < kBlurInH * (kBlurTW / 16); task += 256) {
        const int r = task / (kBlurTW / 16), c0 = 16 * (task - r * (kBlurTW / 16));
        const uint8_t* q = in + r * kBlurInS + c0;  // q[k] = input column c0 + k - 3
        int v[22];
#pragma unroll
        for (int k = 0; k < 22; k++) v[k] = q[k];
#pragma unroll
        for (int c = 0; c < 16; c++)
            rs[r][c0 + c] = 55 * v[c + 3] + 49 * (v[c + 2] + v[c + 4]) + 34 * (v[c + 1] + v[c + 5]) +
                            18 * (v[c] + v[c + 6]);
    }
    __syncthreads();
    const int cq = 4 * (tid & 31), rb = 4 * (tid >> 5);  // 4 columns x 4 rows per thread
    uint8_t* dst = blur + b * bimg + g.boff;
#pragma unroll
    for (int rr = 0; rr < 4; rr++) {
        const int y = y0 + rb + rr;
        if (y >= g.H) break;
        unsigned packedv = 0;
#pragma unroll
        for (int cc = 0; cc < 4; cc++) {
            const int c = cq + cc, x = x0 + c, r = rb + rr;
            const int c3 = rs[r + 3][c], p1 = rs[r + 2][c] + rs[r + 4][c], p2 = rs[r + 1][c] + rs[r + 5][c],
                      p3 = rs[r][c] + rs[r + 6][c];
            int v;
            if (x < g.blur_xv) {  // SymmColumnVec_32s8u float path
                float sacc = (float)c3 * (55.f / 65536.f) + 0.0f;
                sacc = sacc + (float)p1 * (49.f / 65536.f);
                sacc = sacc + (float)p2 * (34.f / 65536.f);
                sacc = sacc + (float)p3 * (18.f / 65536.f);
                v = (int)__builtin_rintf(sacc);
            } else {
                v = (c3 * 55 + p1 * 49 + p2 * 34 + p3 * 18 + (1 << 15)) >> 16;
            }
            packedv |= (unsigned)(v < 0 ? 0 : (v > 255 ? 255 : v)) << (8 * cc);
        }
        if (x0 + cq < g.bstride)
            *reinterpret_cast<unsigned*>(dst + (long long)y * g.bstride + x0 + cq) = packedv;
    }
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
    const float ca = (float)cos((double)ang), sa = (float)sin((double)ang);
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
        if (wCell + 6 > 64 || hCell + 6 > 64) return ORBMI_E_UNSUPPORTED;
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
                    cg.slot_base = slot;
                    slot += cap;
                    key += cap;
                }
                cells.push_back(cg);
            }
        }
        g.cell_end = (int)cells.size();
        g.key_cap = key - g.key_base;
        if (g.key_cap > (1 << 20)) return ORBMI_E_UNSUPPORTED;
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
    pimg = off;
    bimg = boff;
    btiles.clear();
    for (int l = 0; l < nlevels; l++)
        for (int y0 = 0; y0 < levels[l].H; y0 += kBlurTH)
            for (int x0 = 0; x0 < levels[l].W; x0 += kBlurTW) btiles.push_back(make_int2(l, x0 | (y0 << 16)));
    nbtiles = (int)btiles.size();
    nslots = slot;
    keys_cap = key;
    out_cap = outb;
    rows = r; cols = c;
    int rc;
    if ((rc = dev_alloc(&d_levels, levels.size()))) return rc;
    if ((rc = dev_alloc(&d_cells, cells.size()))) return rc;
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
        if ((rc = dev_alloc(&d_cell_counts, (size_t)batch * cells.size()))) return rc;
        if ((rc = dev_alloc(&d_slots, (size_t)batch * nslots))) return rc;
        if ((rc = dev_alloc(&d_keys, (size_t)batch * keys_cap))) return rc;
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

int Extractor::run(const uint8_t* d_images, int batch, size_t step, size_t image_stride,
                   orbmi_keypoint* kps, uint8_t* desc, int* counts, int capacity) {
    ORBMI_HIP(hipSetDevice(device));
    const int ncells = (int)cells.size();
    for (int l = 0; l < nlevels; l++) {
        const LevelGeom& g = levels[l];
        dim3 grid((g.W + 2 * kEdge + 255) / 256, g.ph, batch);
        if (l == 0) {
            hipEvent_t ev = prof_begin(ORBMI_STAGE_PYR_LEVEL0);
            hipLaunchKernelGGL(k_pyr_level0, grid, dim3(256), 0, stream, d_images, step, image_stride, d_pyr, pimg, g);
            prof_end(ORBMI_STAGE_PYR_LEVEL0, ev);
        } else {
            hipEvent_t ev = prof_begin(ORBMI_STAGE_PYR_RESIZE);
            hipLaunchKernelGGL(k_pyr_resize, grid, dim3(256), 0, stream, d_pyr, pimg, levels[l - 1], g,
                               d_xtab + g.xtab_off, d_ytab + g.ytab_off);
            prof_end(ORBMI_STAGE_PYR_RESIZE, ev);
        }
    }
    hipEvent_t ev = prof_begin(ORBMI_STAGE_FAST);
    hipLaunchKernelGGL(k_fast, dim3((ncells + kFastCells - 1) / kFastCells, batch), dim3(64 * kFastCells), 0, stream,
                       d_pyr, pimg, d_levels, d_cells,
                       ncells, d_slots, nslots, d_cell_counts, ini_th, min_th);
    prof_end(ORBMI_STAGE_FAST, ev);
    ev = prof_begin(ORBMI_STAGE_OCTREE);
    hipLaunchKernelGGL(k_octree, dim3(nlevels, batch), dim3(kOctThreads), 0, stream, d_levels, nlevels, ncells,
                       d_cell_counts, d_cells, d_slots, nslots, d_keys, d_node_of, keys_cap, d_oct, out_cap,
                       d_oct_count);
    prof_end(ORBMI_STAGE_OCTREE, ev);
    ev = prof_begin(ORBMI_STAGE_BLUR);
    hipLaunchKernelGGL(k_blur, dim3(nbtiles, batch), dim3(256), 0, stream, d_pyr, d_blur, pimg, bimg, d_levels,
                       d_btiles);
    prof_end(ORBMI_STAGE_BLUR, ev);
    ev = prof_begin(ORBMI_STAGE_DESCRIBE);
    hipLaunchKernelGGL(k_describe, dim3((out_cap + 3) / 4, batch), dim3(256), 0, stream, d_pyr, d_blur, pimg, bimg,
                       d_levels, nlevels, d_oct, out_cap, d_oct_count, kps, desc, counts, capacity);
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

hipEvent_t Extractor::prof_begin(int stage) {
    if (!(prof_mask >> stage & 1u)) return nullptr;
    hipEvent_t a = prof_event();
    if (a) (void)hipEventRecord(a, stream);
    return a;
}

void Extractor::prof_end(int stage, hipEvent_t a) {
    if (!a) return;
    hipEvent_t b = prof_event();
    if (!b) return;
    (void)hipEventRecord(b, stream);
    prof_pending.push_back(ProfPair{stage, a, b});
}

void Extractor::release() {
    for (auto& p : prof_pending) { (void)hipEventDestroy(p.a); (void)hipEventDestroy(p.b); }
    for (auto e : prof_pool) (void)hipEventDestroy(e);
    prof_pending.clear();
    prof_pool.clear();
    if (device >= 0) (void)hipSetDevice(device);
    void* ptrs[] = {d_levels, d_cells, d_btiles, d_blur, d_xtab, d_ytab, d_pyr, d_cell_counts, d_slots, d_keys, d_node_of,
                    d_oct, d_oct_count, d_kps, d_desc, d_counts, d_image, d_scale_tab, d_row_start,
                    d_row_list, d_sad, d_stereo_u, d_stereo_d};
    for (void* p : ptrs)
        if (p) (void)hipFree(p);
    if (stream) (void)hipStreamDestroy(stream);
    stream = nullptr;
}

}  // namespace orbmi
