// DBoW2 TemplatedVocabulary::transform on MI355X: Frame::ComputeBoW / KeyFrame::ComputeBoW
// (src/Frame.cc:425-432, src/KeyFrame.cc:59), SURVEY.md §8(f) rank 2.
//   TemplatedVocabulary::transform(features, BowVector&, FeatureVector&, levelsup)
//                                               Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h:1126-1194
//   per-feature descent                         :1217-1259 (FORB::distance, strict < : first child wins)
//   BowVector::addWeight / addIfNotExist / normalize   Thirdparty/DBoW2/DBoW2/BowVector.cpp:34-86
//   FeatureVector::addFeature                   Thirdparty/DBoW2/DBoW2/FeatureVector.cpp:31-45
// Two kernels:
//   k_bow_descend16  16 lanes (one DPP row) per descriptor, lane j on child j: per level one load
//                  of the children's 32-B descriptors, stored again in CSR order at upload (cdesc)
//                  so a node's children are contiguous, and a DPP min; fan-out > 16 falls back to
//                  k_bow_descend (thread per descriptor).  Outputs (word, weight, node at level
//                  L - levelsup).
//   k_bow_build    two 1024-thread workgroups side by side.  Block 0: sort of (word << 32 |
//                  feature) keys in LDS (bitonic, stages of stride < 128 inside a wave), segment
//                  heads -> BowVector entries in word order with the per-word weight accumulated
//                  sequentially in feature order (as addWeight does), the L1 / L2 norm summed
//                  sequentially in word order (as normalize does).  Block 1: the same sort on
//                  (node << 32 | feature) -> FeatureVector CSR.  Every sum has the reference's
//                  order, so the BowVector values are bit-exact, not merely close.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <mutex>
#include <new>
#include <vector>

#include "orbmi_common.h"

namespace orbmi {

constexpr int kBowMaxFeatures = 8192;
constexpr int kBowBuildThreads = 1024;
constexpr unsigned long long kNoKey = ~0ull;

struct VocDev {
    int k, L, scoring, weighting, nnodes, max_fanout;
    const uint4* desc;       // nnodes x 2
    const uint4* cdesc;      // child_off[nnodes] x 2: descriptor of children[j] at j (CSR order)
    const int* child_off;
    const int* children;
    const int* word_id;
    const double* weight;
};

// DBoW2 ScoringObject::mustNormalize (ScoringObject.h:60-92): L1 for L1 / chi-square / KL /
// Bhattacharyya, L2 for L2, none for the dot product.  norm: 1 = L1, 2 = L2.
__host__ __device__ inline bool must_normalize(int scoring, int* norm) {
    if (scoring == 1) { *norm = 2; return true; }
    *norm = 1;
    return scoring != 5;
}

__global__ __launch_bounds__(256) void k_bow_descend(VocDev v, const uint4* __restrict__ feats, int n,
                                                     const int* __restrict__ n_dev, int nid_level,
                                                     unsigned long long* __restrict__ key_w,
                                                     unsigned long long* __restrict__ key_n, double* __restrict__ wv) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const int nn = n_dev ? min(*n_dev, n) : n;
    if (i >= n) return;
    if (i >= nn) { key_w[i] = kNoKey; key_n[i] = kNoKey; return; }
    const uint4 a0 = feats[2 * i], a1 = feats[2 * i + 1];
    int node = 0, level = 0, nid = 0;
    for (;;) {
        const int c0 = v.child_off[node], c1 = v.child_off[node + 1];
        if (c0 == c1) break;  // leaf
        level++;
        int best = v.children[c0];
        int bd = popc256(a0, a1, v.desc[2 * best], v.desc[2 * best + 1]);
        for (int j = c0 + 1; j < c1; j++) {
            const int id = v.children[j];
            const int d = popc256(a0, a1, v.desc[2 * id], v.desc[2 * id + 1]);
            if (d < bd) { bd = d; best = id; }
        }
        node = best;
        if (level == nid_level) nid = node;
    }
    const double w = v.weight[node];
    const int word = v.word_id[node];
    const bool keep = w > 0;  // "not stopped"
    key_w[i] = keep ? ((unsigned long long)(unsigned)word << 32 | (unsigned)i) : kNoKey;
    key_n[i] = keep ? ((unsigned long long)(unsigned)nid << 32 | (unsigned)i) : kNoKey;
    wv[i] = w;
}

// 16 lanes per descriptor (one DPP row): lane j of the row takes child j of the current node
// (fan-out <= 16), so a level costs one load of the children's descriptors (contiguous in CSR
// order, cdesc) and a 4-step DPP min over (distance << 8 | child position) -- the lowest
// position wins ties, as the reference's strict `d < best_d` scan does.
__device__ inline unsigned row_min_u32(unsigned v) {
    v = min(v, (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xf, 0xf, false));   // xor 1
    v = min(v, (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xf, 0xf, false));   // xor 2
    v = min(v, (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x141, 0xf, 0xf, false));  // mirror 8
    v = min(v, (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x128, 0xf, 0xf, false));  // ror 8
    return v;
}

__global__ __launch_bounds__(256) void k_bow_descend16(VocDev v, const uint4* __restrict__ feats, int n,
                                                       const int* __restrict__ n_dev, int nid_level,
                                                       unsigned long long* __restrict__ key_w,
                                                       unsigned long long* __restrict__ key_n, double* __restrict__ wv) {
    const int g = (blockIdx.x * blockDim.x + threadIdx.x) >> 4, lane = threadIdx.x & 15;
    const int nn = n_dev ? min(*n_dev, n) : n;
    const bool valid = g < nn;
    const int i = valid ? g : 0;  // lanes of invalid groups run along (uniform DPP rows), write nothing
    const uint4 a0 = feats[2 * i], a1 = feats[2 * i + 1];
    int node = 0, level = 0, nid = 0;
    for (;;) {
        const int c0 = v.child_off[node], c1 = v.child_off[node + 1];
        if (c0 == c1) break;  // leaf (uniform in the row)
        level++;
        const int j = c0 + lane;
        unsigned key = 0xFFFFFFFFu;
        if (j < c1) key = (unsigned)popc256(a0, a1, v.cdesc[2 * j], v.cdesc[2 * j + 1]) << 8 | (unsigned)lane;
        key = row_min_u32(key);
        node = v.children[c0 + (int)(key & 0xFF)];
        if (level == nid_level) nid = node;
    }
    if (!valid || lane != 0) {
        if (lane == 0 && g < n) { key_w[g] = kNoKey; key_n[g] = kNoKey; }
        return;
    }
    const double w = v.weight[node];
    const int word = v.word_id[node];
    const bool keep = w > 0;  // "not stopped"
    key_w[i] = keep ? ((unsigned long long)(unsigned)word << 32 | (unsigned)i) : kNoKey;
    key_n[i] = keep ? ((unsigned long long)(unsigned)nid << 32 | (unsigned)i) : kNoKey;
    wv[i] = w;
}

// ---- sort of m (power of two, 64 <= m <= kBowMaxFeatures) u64 keys in LDS, ascending: bitonic,
// with every stage of stride < 128 done inside a wave on a 128-key chunk held 2 keys per lane
// (lane l: chunk positions 2l, 2l + 1; the partner of a stride-s pair sits in lane l ^ s/2), and
// only the stages of stride >= 128 through LDS with a barrier: for 2048 keys 10 barriered stages
// instead of 66
__device__ inline unsigned long long shfl_xor_u64(unsigned long long v, int m) {
    const int lo = __shfl_xor((int)(unsigned)v, m, 64), hi = __shfl_xor((int)(unsigned)(v >> 32), m, 64);
    return (unsigned long long)(unsigned)hi << 32 | (unsigned)lo;
}

// stages of bitonic level `size` with strides smax .. 1 on the lane's two keys (global index g0 of x0)
__device__ inline void chunk_stages(unsigned long long& x0, unsigned long long& x1, int g0, int size, int smax) {
    const int lane = threadIdx.x & 63;
    const bool up = (g0 & size) == 0;
    for (int stride = smax; stride >= 2; stride >>= 1) {
        const int lm = stride >> 1;
        const unsigned long long y0 = shfl_xor_u64(x0, lm), y1 = shfl_xor_u64(x1, lm);
        const bool keep_min = ((lane & lm) == 0) == up;
        x0 = keep_min ? (x0 < y0 ? x0 : y0) : (x0 < y0 ? y0 : x0);
        x1 = keep_min ? (x1 < y1 ? x1 : y1) : (x1 < y1 ? y1 : x1);
    }
    if ((x0 > x1) == up) { const unsigned long long t = x0; x0 = x1; x1 = t; }  // stride 1
}

__device__ void sort_keys(unsigned long long* s, int m) {
    const int C = m < 128 ? m : 128, lanes = C / 2, nchunks = m / C;
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63, nwv = blockDim.x >> 6;
    // levels 2 .. C entirely inside chunks
    for (int c = wid; c < nchunks; c += nwv) {
        if (lane < lanes) {
            const int g0 = c * C + 2 * lane;
            unsigned long long x0 = s[g0], x1 = s[g0 + 1];
            for (int size = 2; size <= C; size <<= 1) chunk_stages(x0, x1, g0, size, size >> 1);
            s[g0] = x0;
            s[g0 + 1] = x1;
        }
    }
    __syncthreads();
    for (int size = 2 * C; size <= m; size <<= 1) {
        for (int stride = size >> 1; stride >= C; stride >>= 1) {  // across chunks: LDS
            for (int t = threadIdx.x; t < (m >> 1); t += blockDim.x) {
                const int lo = 2 * stride * (t / stride) + (t % stride), hi = lo + stride;
                const bool up = (lo & size) == 0;
                const unsigned long long a = s[lo], b = s[hi];
                if ((a > b) == up) { s[lo] = b; s[hi] = a; }
            }
            __syncthreads();
        }
        for (int c = wid; c < nchunks; c += nwv) {  // strides C / 2 .. 1 inside chunks
            if (lane < lanes) {
                const int g0 = c * C + 2 * lane;
                unsigned long long x0 = s[g0], x1 = s[g0 + 1];
                chunk_stages(x0, x1, g0, size, C >> 1);
                s[g0] = x0;
                s[g0 + 1] = x1;
            }
        }
        __syncthreads();
    }
}

// heads[j] = 1 where sorted key j starts a new segment (same high 32 bits); returns the exclusive
// prefix of heads per element in pos[] and the number of segments
__device__ int segment_heads(const unsigned long long* s, int m, int* pos, int* scratch) {
    constexpr int PER = kBowMaxFeatures / kBowBuildThreads;  // 8 keys per thread
    const int base = threadIdx.x * PER;
    int h[PER], cnt = 0;
#pragma unroll
    for (int q = 0; q < PER; q++) {
        const int j = base + q;
        const bool valid = j < m && s[j] != kNoKey;
        h[q] = valid && (j == 0 || (s[j] >> 32) != (s[j - 1] >> 32));
        cnt += h[q];
    }
    int total;
    int run = block_excl_scan(cnt, scratch, &total);
#pragma unroll
    for (int q = 0; q < PER; q++) {
        const int j = base + q;
        if (j < m) pos[j] = h[q] ? run : -1;
        run += h[q];
    }
    __syncthreads();
    return total;
}

// Two workgroups that run side by side: block 0 builds the BowVector (sort of the word keys,
// per-word weights summed in feature order, the norm), block 1 the FeatureVector (sort of the
// node keys, CSR).  The norm is the one sequential chain (bit-exact: the reference's order).
__global__ __launch_bounds__(kBowBuildThreads) void k_bow_build(
    const unsigned long long* __restrict__ key_w, const unsigned long long* __restrict__ key_n,
    const double* __restrict__ wv, int n, int weighting, int scoring, unsigned* __restrict__ bow_word,
    double* __restrict__ bow_value, unsigned* __restrict__ fv_node, int* __restrict__ fv_off, int* __restrict__ fv_feat,
    int* __restrict__ counts) {
    __shared__ unsigned long long s[kBowMaxFeatures];
    __shared__ int pos[kBowMaxFeatures];
    __shared__ int scratch[kBowBuildThreads / 64 + 1];
    __shared__ double norm_s;
    int m = 64;
    while (m < n) m <<= 1;
    constexpr int PER = kBowMaxFeatures / kBowBuildThreads;
    if (blockIdx.x == 1) {  // ---- FeatureVector
        for (int j = threadIdx.x; j < m; j += blockDim.x) s[j] = j < n ? key_n[j] : kNoKey;
        __syncthreads();
        sort_keys(s, m);
        const int nnod = segment_heads(s, m, pos, scratch);
        for (int j = threadIdx.x; j < m; j += blockDim.x) {
            if (s[j] == kNoKey) continue;
            fv_feat[j] = (int)(unsigned)s[j];  // valid keys sort first: j is the CSR position
            const int k = pos[j];
            if (k >= 0) {
                fv_node[k] = (unsigned)(s[j] >> 32);
                fv_off[k] = j;
            }
            if (j + 1 == m || s[j + 1] == kNoKey) fv_off[nnod] = j + 1;
        }
        if (threadIdx.x == 0) {
            if (nnod == 0) fv_off[0] = 0;
            counts[1] = nnod;
        }
        return;
    }
    // ---- BowVector
    for (int j = threadIdx.x; j < m; j += blockDim.x) s[j] = j < n ? key_w[j] : kNoKey;
    __syncthreads();
    sort_keys(s, m);
    const int nw = segment_heads(s, m, pos, scratch);
    const bool tf = weighting == 0 || weighting == 1;  // TF_IDF, TF: addWeight; IDF, BINARY: addIfNotExist
    int nrm = 1;
    const bool must = must_normalize(scoring, &nrm);
    // every element's weight gathered once (in parallel), then kept in LDS in sorted order
    double w[PER];
    int nvalid = 0;  // valid keys sort first
#pragma unroll
    for (int q = 0; q < PER; q++) {
        const int j = threadIdx.x + q * kBowBuildThreads;
        w[q] = 0;
        if (j < m && s[j] != kNoKey) {
            w[q] = wv[(unsigned)s[j]];
            nvalid = j + 1;
            if (pos[j] >= 0) bow_word[pos[j]] = (unsigned)(s[j] >> 32);
        }
    }
    __shared__ int nvalid_s;
    if (threadIdx.x == 0) nvalid_s = 0;
    __syncthreads();
    atomicMax(&nvalid_s, nvalid);
    double* ws = reinterpret_cast<double*>(s);  // the keys are dead once words and weights are out
#pragma unroll
    for (int q = 0; q < PER; q++) {
        const int j = threadIdx.x + q * kBowBuildThreads;
        if (j < m) ws[j] = w[q];
    }
    __syncthreads();
    const int nv = nvalid_s;
    double val[PER];
    int slot[PER];
#pragma unroll
    for (int q = 0; q < PER; q++) {  // segment heads: one BowVector entry each, summed in feature order
        const int j = threadIdx.x + q * kBowBuildThreads;
        slot[q] = (j < m) ? pos[j] : -1;
        val[q] = 0;
        if (slot[q] < 0) continue;
        double x = ws[j];
        if (tf)
            for (int r = j + 1; r < nv && pos[r] < 0; r++) x += ws[r];
        if (tf && !must) x /= (double)nw;  // "unnecessary when normalizing": divide by v.size()
        val[q] = x;
    }
    __syncthreads();  // the weights are dead: the LDS holds the values, in word order
#pragma unroll
    for (int q = 0; q < PER; q++)
        if (slot[q] >= 0) ws[slot[q]] = val[q];
    __syncthreads();
    if (must && threadIdx.x == 0) {  // BowVector::normalize: sequential in word order
        double norm = 0.0;
        int k = 0;
        if (nrm == 1) {
            for (; k + 4 <= nw; k += 4) {
                const double a0 = ws[k], a1 = ws[k + 1], a2 = ws[k + 2], a3 = ws[k + 3];
                norm += fabs(a0);
                norm += fabs(a1);
                norm += fabs(a2);
                norm += fabs(a3);
            }
            for (; k < nw; k++) norm += fabs(ws[k]);
        } else {
            for (; k + 4 <= nw; k += 4) {
                const double a0 = ws[k], a1 = ws[k + 1], a2 = ws[k + 2], a3 = ws[k + 3];
                norm += a0 * a0;
                norm += a1 * a1;
                norm += a2 * a2;
                norm += a3 * a3;
            }
            for (; k < nw; k++) norm += ws[k] * ws[k];
            norm = sqrt(norm);
        }
        norm_s = norm;
    }
    __syncthreads();
    const double norm = must ? norm_s : 0.0;
    for (int k = threadIdx.x; k < nw; k += blockDim.x) bow_value[k] = norm > 0.0 ? ws[k] / norm : ws[k];
    if (threadIdx.x == 0) counts[0] = nw;
}

}  // namespace orbmi

// ---------------------------------------------------------------- host
struct orbmi_vocabulary {
    int device = 0;
    hipStream_t stream = nullptr;
    bool own_stream = true;           // false after orbmi_vocabulary_share_stream
    orbmi::VocDev v{};
    void* d_vocab = nullptr;          // one allocation for all vocabulary arrays
    uint8_t* d_work = nullptr;        // keys, weights and staging of one transform
    size_t cap_work = 0;
    // one transform at a time: d_work is the call's staging, and Tracking (TrackReferenceKeyFrame)
    // and LocalMapping (ProcessNewKeyFrame, run with the map lock released) may both transform
    // on one handle -- the reference's Vocabulary::transform is const, safe from both threads
    std::mutex mtx;
    // pinned host mirror of d_work: host descriptors go up from it, host outputs come back into it
    // in one copy; in_ev marks the last upload from it (an asynchronous call may still be reading)
    uint8_t* h_work = nullptr;
    hipEvent_t in_ev = nullptr;
    bool in_pending = false;
};

namespace {

bool on_device(const void* p) {
    if (!p) return false;
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return a.type == hipMemoryTypeDevice;
}

size_t align256(size_t b) { return (b + 255) & ~(size_t)255; }

}  // namespace

extern "C" {

int orbmi_vocabulary_create(int device, const orbmi_vocabulary_desc* d, orbmi_vocabulary** out) {
    if (!out || !d) return ORBMI_E_ARG;
    *out = nullptr;
    if (d->nnodes < 1 || !d->desc || !d->child_off || !d->word_id || !d->weight) return ORBMI_E_ARG;
    const int nch = d->child_off[d->nnodes];
    if (d->child_off[0] != 0 || nch < 0 || (nch > 0 && !d->children)) return ORBMI_E_ARG;
    for (int i = 0; i < d->nnodes; i++)  // CSR sanity: children ids in range, offsets monotone
        if (d->child_off[i + 1] < d->child_off[i]) return ORBMI_E_ARG;
    for (int j = 0; j < nch; j++)
        if (d->children[j] <= 0 || d->children[j] >= d->nnodes) return ORBMI_E_ARG;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return ORBMI_E_HIP;
    orbmi_vocabulary* h = new (std::nothrow) orbmi_vocabulary();
    if (!h) return ORBMI_E_ARG;
    h->device = device;
    const size_t nn = (size_t)d->nnodes;
    const size_t b_desc = align256(nn * 32), b_off = align256((nn + 1) * 4), b_ch = align256((size_t)std::max(nch, 1) * 4),
                 b_word = align256(nn * 4), b_w = align256(nn * 8), b_cdesc = align256((size_t)std::max(nch, 1) * 32);
    int max_fanout = 0;
    for (int i = 0; i < d->nnodes; i++) max_fanout = std::max(max_fanout, d->child_off[i + 1] - d->child_off[i]);
    std::vector<uint8_t> cdesc((size_t)std::max(nch, 1) * 32);
    for (int j = 0; j < nch; j++) memcpy(&cdesc[(size_t)j * 32], d->desc + (size_t)d->children[j] * 32, 32);
    auto fail = [&](int rc) { orbmi_vocabulary_destroy(h); return rc; };
    if (hipSetDevice(device) != hipSuccess || orbmi::stream_create(&h->stream, "VOCAB") != hipSuccess)
        return fail(ORBMI_E_HIP);
    if (hipMalloc(&h->d_vocab, b_desc + b_off + b_ch + b_word + b_w + b_cdesc) != hipSuccess) return fail(ORBMI_E_HIP);
    uint8_t* base = (uint8_t*)h->d_vocab;
    uint8_t* p_desc = base;
    int* p_off = (int*)(base + b_desc);
    int* p_ch = (int*)(base + b_desc + b_off);
    int* p_word = (int*)(base + b_desc + b_off + b_ch);
    double* p_w = (double*)(base + b_desc + b_off + b_ch + b_word);
    uint8_t* p_cdesc = base + b_desc + b_off + b_ch + b_word + b_w;
    if (hipMemcpy(p_desc, d->desc, nn * 32, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(p_off, d->child_off, (nn + 1) * 4, hipMemcpyHostToDevice) != hipSuccess ||
        (nch > 0 && hipMemcpy(p_ch, d->children, (size_t)nch * 4, hipMemcpyHostToDevice) != hipSuccess) ||
        hipMemcpy(p_word, d->word_id, nn * 4, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(p_w, d->weight, nn * 8, hipMemcpyHostToDevice) != hipSuccess ||
        (nch > 0 && hipMemcpy(p_cdesc, cdesc.data(), (size_t)nch * 32, hipMemcpyHostToDevice) != hipSuccess))
        return fail(ORBMI_E_HIP);
    h->v = orbmi::VocDev{d->k, d->L, d->scoring, d->weighting, d->nnodes, max_fanout, (const uint4*)p_desc,
                         (const uint4*)p_cdesc, p_off, p_ch, p_word, p_w};
    *out = h;
    return ORBMI_OK;
}

void orbmi_vocabulary_destroy(orbmi_vocabulary* h) {
    if (!h) return;
    (void)hipSetDevice(h->device);
    if (h->stream) (void)hipStreamSynchronize(h->stream);
    if (h->d_vocab) (void)hipFree(h->d_vocab);
    if (h->d_work) (void)hipFree(h->d_work);
    if (h->h_work) (void)hipHostFree(h->h_work);
    if (h->in_ev) (void)hipEventDestroy(h->in_ev);
    if (h->stream && h->own_stream) (void)hipStreamDestroy(h->stream);
    delete h;
}

int orbmi_vocabulary_get_stream(orbmi_vocabulary* h, void** stream) {
    if (!h || !stream) return ORBMI_E_ARG;
    *stream = (void*)h->stream;
    return ORBMI_OK;
}

int orbmi_vocabulary_share_stream(orbmi_vocabulary* h, orbmi_extractor* ex) {
    if (!h || !ex) return ORBMI_E_ARG;
    void* s = nullptr;
    int rc = orbmi_extractor_get_stream(ex, &s);
    if (rc) return rc;
    ORBMI_HIP(hipSetDevice(h->device));
    ORBMI_HIP(hipStreamSynchronize(h->stream));
    if (h->own_stream) ORBMI_HIP(hipStreamDestroy(h->stream));
    h->stream = (hipStream_t)s;
    h->own_stream = false;
    return ORBMI_OK;
}

int orbmi_vocabulary_set_stream(orbmi_vocabulary* h, void* stream) {
    if (!h) return ORBMI_E_ARG;
    ORBMI_HIP(hipSetDevice(h->device));
    ORBMI_HIP(hipStreamSynchronize(h->stream));
    hipStream_t s = (hipStream_t)stream;
    if (!s) ORBMI_HIP(orbmi::stream_create(&s, "VOCAB"));
    if (h->own_stream) ORBMI_HIP(hipStreamDestroy(h->stream));
    h->stream = s;
    h->own_stream = stream == nullptr;
    return ORBMI_OK;
}

int orbmi_vocabulary_synchronize(orbmi_vocabulary* h) {
    if (!h) return ORBMI_E_ARG;
    ORBMI_HIP(hipStreamSynchronize(h->stream));
    return ORBMI_OK;
}

int orbmi_transform(orbmi_vocabulary* h, const uint8_t* desc, int n, const int* n_device, int levelsup,
                    uint32_t* bow_word, double* bow_value, uint32_t* fv_node, int32_t* fv_off, int32_t* fv_feat,
                    int* counts) {
    using namespace orbmi;
    if (!h || n < 0 || (n > 0 && !desc) || !bow_word || !bow_value || !fv_node || !fv_off || !fv_feat || !counts)
        return ORBMI_E_ARG;
    if (n > kBowMaxFeatures) return ORBMI_E_UNSUPPORTED;
    if (n_device && !on_device(n_device)) return ORBMI_E_ARG;
    std::lock_guard<std::mutex> lock(h->mtx);
    ORBMI_HIP(hipSetDevice(h->device));
    const size_t nn = (size_t)std::max(n, 1);
    // work: keys (2 x 8 n), weights (8 n), staged input (32 n), staged outputs
    const size_t b_key = align256(nn * 8), b_w = align256(nn * 8), b_in = align256(nn * 32), b_u = align256(nn * 4),
                 b_d = align256(nn * 8), b_off = align256((nn + 1) * 4), b_cnt = 256;
    const size_t need = 2 * b_key + b_w + b_in + b_u + b_d + b_u + b_off + b_u + b_cnt;
    if (need > h->cap_work) {
        ORBMI_HIP(hipStreamSynchronize(h->stream));
        if (h->d_work) (void)hipFree(h->d_work);
        if (h->h_work) (void)hipHostFree(h->h_work);
        h->d_work = nullptr;
        h->h_work = nullptr;
        h->cap_work = 0;
        h->in_pending = false;
        ORBMI_HIP(hipMalloc((void**)&h->d_work, need));
        ORBMI_HIP(hipHostMalloc((void**)&h->h_work, need, hipHostMallocDefault));
        h->cap_work = need;
    }
    if (!h->in_ev) ORBMI_HIP(hipEventCreateWithFlags(&h->in_ev, hipEventDisableTiming));
    auto mirror = [&](const void* d) { return h->h_work + ((const uint8_t*)d - h->d_work); };
    uint8_t* w = h->d_work;
    unsigned long long* key_w = (unsigned long long*)w; w += b_key;
    unsigned long long* key_n = (unsigned long long*)w; w += b_key;
    double* wv = (double*)w; w += b_w;
    uint8_t* in_stage = w; w += b_in;
    uint32_t* s_word = (uint32_t*)w; w += b_u;
    double* s_value = (double*)w; w += b_d;
    uint32_t* s_node = (uint32_t*)w; w += b_u;
    int32_t* s_off = (int32_t*)w; w += b_off;
    int32_t* s_feat = (int32_t*)w; w += b_u;
    int* s_cnt = (int*)w;
    const uint8_t* d_in = desc;
    if (n > 0 && !on_device(desc)) {
        if (h->in_pending) ORBMI_HIP(hipEventSynchronize(h->in_ev));  // the mirror's last upload
        memcpy(mirror(in_stage), desc, (size_t)n * 32);
        ORBMI_HIP(hipMemcpyAsync(in_stage, mirror(in_stage), (size_t)n * 32, hipMemcpyHostToDevice, h->stream));
        ORBMI_HIP(hipEventRecord(h->in_ev, h->stream));
        h->in_pending = true;
        d_in = in_stage;
    }
    bool host_out = false;
    auto dev_out = [&](auto* p, auto* stage) {
        if (on_device(p)) return p;
        host_out = true;
        return stage;
    };
    uint32_t* o_word = dev_out(bow_word, s_word);
    double* o_value = dev_out(bow_value, s_value);
    uint32_t* o_node = dev_out(fv_node, s_node);
    int32_t* o_off = dev_out(fv_off, s_off);
    int32_t* o_feat = dev_out(fv_feat, s_feat);
    int* o_cnt = dev_out(counts, s_cnt);
    const int nid_level = h->v.L - levelsup;  // <= 0: the root (node 0)
    if (n > 0) {
        if (h->v.max_fanout <= 16)  // one DPP row per descriptor
            hipLaunchKernelGGL(k_bow_descend16, dim3((16 * n + 255) / 256), dim3(256), 0, h->stream, h->v,
                               (const uint4*)d_in, n, n_device, nid_level, key_w, key_n, wv);
        else
            hipLaunchKernelGGL(k_bow_descend, dim3((n + 255) / 256), dim3(256), 0, h->stream, h->v, (const uint4*)d_in,
                               n, n_device, nid_level, key_w, key_n, wv);
        ORBMI_HIP(hipGetLastError());
    }
    hipLaunchKernelGGL(k_bow_build, dim3(2), dim3(kBowBuildThreads), 0, h->stream, key_w, key_n, wv, n,
                       h->v.weighting, h->v.scoring, (unsigned*)o_word, o_value, (unsigned*)o_node, (int*)o_off,
                       (int*)o_feat, o_cnt);
    ORBMI_HIP(hipGetLastError());
    if (!host_out) return ORBMI_OK;
    if (o_word == s_word && o_value == s_value && o_node == s_node && o_off == s_off && o_feat == s_feat &&
        o_cnt == s_cnt) {
        // every output on the host: the staged outputs (contiguous, s_word .. s_cnt) come back in
        // one copy into the mirror and one wait, then the used parts are copied out
        const uint8_t* lo = (const uint8_t*)s_word;
        const size_t span = (size_t)((const uint8_t*)(s_cnt + 2) - lo);
        ORBMI_HIP(hipMemcpyAsync(mirror(lo), lo, span, hipMemcpyDeviceToHost, h->stream));
        ORBMI_HIP(hipStreamSynchronize(h->stream));
        h->in_pending = false;
        const int* hc = (const int*)mirror(s_cnt);
        const size_t nwd = (size_t)hc[0], nnd = (size_t)hc[1];
        const size_t nfeat = nnd > 0 ? (size_t)((const int32_t*)mirror(s_off))[nnd] : 0;
        memcpy(bow_word, mirror(s_word), nwd * 4);
        memcpy(bow_value, mirror(s_value), nwd * 8);
        memcpy(fv_node, mirror(s_node), nnd * 4);
        memcpy(fv_off, mirror(s_off), (nnd + 1) * 4);
        memcpy(fv_feat, mirror(s_feat), nfeat * 4);
        memcpy(counts, hc, 2 * sizeof(int));
        return ORBMI_OK;
    }
    int hc[2] = {0, 0};
    ORBMI_HIP(hipMemcpyAsync(hc, o_cnt, 2 * sizeof(int), hipMemcpyDeviceToHost, h->stream));
    ORBMI_HIP(hipStreamSynchronize(h->stream));
    const size_t nwd = (size_t)hc[0], nnd = (size_t)hc[1];
    size_t nfeat = 0;
    if (nnd > 0) {
        int last = 0;
        ORBMI_HIP(hipMemcpy(&last, o_off + nnd, sizeof(int), hipMemcpyDeviceToHost));
        nfeat = (size_t)last;
    }
    auto back = [&](void* user, const void* dev, size_t bytes) -> int {
        if (user != dev && bytes) ORBMI_HIP(hipMemcpyAsync(user, dev, bytes, hipMemcpyDeviceToHost, h->stream));
        return ORBMI_OK;
    };
    int rc = ORBMI_OK;
    rc |= back(bow_word, o_word, nwd * 4);
    rc |= back(bow_value, o_value, nwd * 8);
    rc |= back(fv_node, o_node, nnd * 4);
    rc |= back(fv_off, o_off, (nnd + 1) * 4);
    rc |= back(fv_feat, o_feat, nfeat * 4);
    rc |= back(counts, o_cnt, 2 * sizeof(int));
    if (rc) return ORBMI_E_HIP;
    ORBMI_HIP(hipStreamSynchronize(h->stream));
    return ORBMI_OK;
}

}  // extern "C"
