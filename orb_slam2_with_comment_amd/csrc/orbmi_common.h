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
// DPP moves inside each row of 16 lanes (quad perms, half-row mirror, row rotate by 8) and
// v_permlane16/32_swap across rows: no LDS round trip (a __shfl_xor butterfly is one
// ds_bpermute per step and dword); every lane ends with the result.  The reductions are
// integer / min / max, so their order does not matter.
namespace wave_detail {
template <int CTRL>
__device__ inline int dpp(int v) { return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xf, 0xf, false); }
template <int W>  // the value of lane ^ W (W = 16 or 32)
__device__ inline int partner(int v) {
    const auto r = W == 32 ? __builtin_amdgcn_permlane32_swap(v, v, false, false)
                           : __builtin_amdgcn_permlane16_swap(v, v, false, false);
    // one of the pair is the own value, the other the partner's (equal values: either)
    return (int)r[0] == v ? (int)r[1] : (int)r[0];
}
__device__ inline unsigned long long dpp64(unsigned long long u, int which) {
    const int lo = (int)(unsigned)u, hi = (int)(unsigned)(u >> 32);
    int l, h;
    switch (which) {
        case 0: l = dpp<0xB1>(lo); h = dpp<0xB1>(hi); break;    // quad_perm [1,0,3,2]: lane ^ 1
        case 1: l = dpp<0x4E>(lo); h = dpp<0x4E>(hi); break;    // quad_perm [2,3,0,1]: lane ^ 2
        case 2: l = dpp<0x141>(lo); h = dpp<0x141>(hi); break;  // row_half_mirror: 7 - i within 8
        case 3: l = dpp<0x128>(lo); h = dpp<0x128>(hi); break;  // row_ror:8: lane ^ 8 within 16
        case 4: l = partner<16>(lo); h = partner<16>(hi); break;
        default: l = partner<32>(lo); h = partner<32>(hi); break;
    }
    return (unsigned long long)(unsigned)h << 32 | (unsigned)l;
}
}  // namespace wave_detail

__device__ inline int wave_sum_i32(int v) {
    using namespace wave_detail;
    v += dpp<0xB1>(v);
    v += dpp<0x4E>(v);
    v += dpp<0x141>(v);
    v += dpp<0x128>(v);
    v += partner<16>(v);
    return v + partner<32>(v);
}
__device__ inline unsigned long long wave_min_u64(unsigned long long v) {
#pragma unroll
    for (int k = 0; k < 6; k++) {
        // the permlane swaps pair a lane with lane ^ 16 / ^ 32 only through the own value test
        // above, which is exact for distinct keys and harmless for equal ones
        const unsigned long long w = wave_detail::dpp64(v, k);
        v = w < v ? w : v;
    }
    return v;
}
__device__ inline unsigned long long wave_max_u64(unsigned long long v) {
#pragma unroll
    for (int k = 0; k < 6; k++) {
        const unsigned long long w = wave_detail::dpp64(v, k);
        v = w > v ? w : v;
    }
    return v;
}
// Inclusive prefix sum across the 64 lanes.
// Inside each row of 16 lanes by DPP row shifts (a lane without a source adds 0), then the
// totals of the rows before by readlane: no LDS round trip.
__device__ inline int wave_incl_scan(int v) {
    const int lane = threadIdx.x & 63;
    v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, true);  // row_shr:1
    v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, true);  // row_shr:2
    v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, true);  // row_shr:4
    v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, true);  // row_shr:8
    const int t0 = __builtin_amdgcn_readlane(v, 15), t1 = __builtin_amdgcn_readlane(v, 31);
    const int t2 = __builtin_amdgcn_readlane(v, 47);
    const int row = lane >> 4;
    return v + (row > 0 ? t0 : 0) + (row > 1 ? t1 : 0) + (row > 2 ? t2 : 0);
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
