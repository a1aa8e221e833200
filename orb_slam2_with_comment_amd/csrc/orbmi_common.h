// Shared device/host helpers for the MI355X (gfx950) ORB front-end kernels.
// Compiled with -ffp-contract=off on host and device: every float expression below is
// evaluated with one IEEE rounding per operation, in source order (pinned semantics P7).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/orbmi.h"

#define ORBMI_HIP(call)                                                                 \
    do {                                                                                \
        hipError_t e_ = (call);                                                         \
        if (e_ != hipSuccess) {                                                         \
            fprintf(stderr, "orbmi: %s failed: %s (%s:%d)\n", #call, hipGetErrorString(e_), \
                    __FILE__, __LINE__);                                                \
            return ORBMI_E_HIP;                                                         \
        }                                                                               \
    } while (0)

namespace orbmi {

constexpr int kEdge = 19;        // EDGE_THRESHOLD  src/ORBextractor.cc:74
constexpr int kHalfPatch = 15;   // HALF_PATCH_SIZE src/ORBextractor.cc:73
constexpr int kPatch = 31;       // PATCH_SIZE      src/ORBextractor.cc:72
constexpr int kMaxLevels = 16;
constexpr int kWave = 64;

__host__ __device__ inline int reflect101(int p, int len) {
    if ((unsigned)p < (unsigned)len) return p;
    if (len == 1) return 0;
    do {
        if (p < 0) p = -p;
        else p = 2 * len - 2 - p;
    } while ((unsigned)p >= (unsigned)len);
    return p;
}

__host__ __device__ inline int cv_floor_f(float v) { int i = (int)v; return i - (i > v); }

// cvRound(float): round-half-even (v_rndne_f32 on device, rint under the default mode on host)
__host__ __device__ inline int cv_round_f(float v) { return (int)__builtin_rintf(v); }

// ---- wave-level reductions (wave64) --------------------------------------------------
__device__ inline int wave_sum_i32(int v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ inline unsigned long long wave_min_u64(unsigned long long v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        unsigned long long w = __shfl_xor(v, o, 64);
        v = w < v ? w : v;
    }
    return v;
}
__device__ inline unsigned long long wave_max_u64(unsigned long long v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        unsigned long long w = __shfl_xor(v, o, 64);
        v = w > v ? w : v;
    }
    return v;
}
// Inclusive prefix sum across the 64 lanes.
__device__ inline int wave_incl_scan(int v) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        int w = __shfl_up(v, o, 64);
        if (lane >= o) v += w;
    }
    return v;
}

// Block-wide exclusive scan of one int per thread; `scratch` holds >= blockDim/64 + 1 ints.
// Returns the exclusive prefix; *total receives the block sum.  Contains __syncthreads().
__device__ inline int block_excl_scan(int v, int* scratch, int* total) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
    const int incl = wave_incl_scan(v);
    if (lane == 63) scratch[wid] = incl;
    __syncthreads();
    // every thread adds up the wave totals itself (broadcast LDS reads, no serial pass)
    int before = 0, all = 0;
    for (int w = 0; w < nw; w++) {
        const int t = scratch[w];
        before += w < wid ? t : 0;
        all += t;
    }
    *total = all;
    __syncthreads();  // scratch may be rewritten by the next scan
    return before + incl - v;
}

__device__ inline int popc256(const uint4& a0, const uint4& a1, const uint4& b0, const uint4& b1) {
    return __popc(a0.x ^ b0.x) + __popc(a0.y ^ b0.y) + __popc(a0.z ^ b0.z) + __popc(a0.w ^ b0.w) +
           __popc(a1.x ^ b1.x) + __popc(a1.y ^ b1.y) + __popc(a1.z ^ b1.z) + __popc(a1.w ^ b1.w);
}

// Non-blocking stream of one handle.  ORBMI_PRIO_<ROLE>=high|low (ROLE = MATCHER, POSE, BA,
// VOCAB, EXTRACTOR) selects the device's greatest / least stream priority, else the default.
inline hipError_t stream_create(hipStream_t* s, const char* role) {
    char key[64];
    snprintf(key, sizeof(key), "ORBMI_PRIO_%s", role);
    const char* v = getenv(key);
    if (v && (!strcmp(v, "high") || !strcmp(v, "low"))) {
        int least = 0, greatest = 0;
        hipError_t e = hipDeviceGetStreamPriorityRange(&least, &greatest);
        if (e != hipSuccess) return e;
        return hipStreamCreateWithPriority(s, hipStreamNonBlocking, !strcmp(v, "high") ? greatest : least);
    }
    return hipStreamCreateWithFlags(s, hipStreamNonBlocking);
}

}  // namespace orbmi
