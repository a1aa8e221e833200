// Wave-level cross-lane primitives for gfx950 (wave64): DPP moves inside a row of 16 lanes and
// v_permlane16/32_swap across rows, so reductions need no LDS round trip.  Shared by the
// PoseOptimization and LocalBundleAdjustment kernels; every sum has a fixed order.
#pragma once
#include <hip/hip_runtime.h>

namespace orbmi {

template <int CTRL>
__device__ inline double dpp_mov(double v) {
    const unsigned long long u = (unsigned long long)__double_as_longlong(v);
    const unsigned lo = __builtin_amdgcn_update_dpp(0u, (unsigned)u, CTRL, 0xf, 0xf, false);
    const unsigned hi = __builtin_amdgcn_update_dpp(0u, (unsigned)(u >> 32), CTRL, 0xf, 0xf, false);
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
constexpr int kDppXor1 = 0xB1;         // quad_perm [1,0,3,2]
constexpr int kDppXor2 = 0x4E;         // quad_perm [2,3,0,1]
constexpr int kDppHalfMirror = 0x141;  // lane i <-> 7-i within 8 (pairs lane bit 2 clear/set)
constexpr int kDppRor8 = 0x128;        // row_ror:8 = lane i <-> i^8 within 16

// v_permlane{16,32}_swap on (a, b): lanes with the bit clear end with a_own + a_partner, lanes
// with it set with b_partner + b_own (partner = lane ^ 16 or ^ 32)
template <int W>
__device__ inline double swap_combine(double a, double b) {
    const unsigned long long ua = (unsigned long long)__double_as_longlong(a);
    const unsigned long long ub = (unsigned long long)__double_as_longlong(b);
    unsigned xl = (unsigned)ua, xh = (unsigned)(ua >> 32), yl = (unsigned)ub, yh = (unsigned)(ub >> 32);
    if constexpr (W == 32) {
        auto l = __builtin_amdgcn_permlane32_swap(xl, yl, false, false);
        auto h = __builtin_amdgcn_permlane32_swap(xh, yh, false, false);
        xl = l[0]; yl = l[1]; xh = h[0]; yh = h[1];
    } else {
        auto l = __builtin_amdgcn_permlane16_swap(xl, yl, false, false);
        auto h = __builtin_amdgcn_permlane16_swap(xh, yh, false, false);
        xl = l[0]; yl = l[1]; xh = h[0]; yh = h[1];
    }
    const double nx = __longlong_as_double((long long)(((unsigned long long)xh << 32) | xl));
    const double ny = __longlong_as_double((long long)(((unsigned long long)yh << 32) | yl));
    return nx + ny;
}

// one reduce-scatter step inside a row: lanes with `upper` keep b, the others a, each adding
// the partner's copy of what it keeps
template <int CTRL>
__device__ inline double dpp_combine(double a, double b, bool upper) {
    const double recv = dpp_mov<CTRL>(upper ? a : b);
    return (upper ? b : a) + recv;
}

// Reduce-scatter of 32 per-lane values over the wave: afterwards lane l holds the wave sum of
// value l >> 1 (32 exchanges instead of 6 per value)
__device__ inline double wave_reduce_scatter32(double (&v)[32]) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int j = 0; j < 16; j++) v[j] = swap_combine<32>(v[j], v[16 + j]);
#pragma unroll
    for (int j = 0; j < 8; j++) v[j] = swap_combine<16>(v[j], v[8 + j]);
#pragma unroll
    for (int j = 0; j < 4; j++) v[j] = dpp_combine<kDppRor8>(v[j], v[4 + j], lane & 8);
#pragma unroll
    for (int j = 0; j < 2; j++) v[j] = dpp_combine<kDppHalfMirror>(v[j], v[2 + j], lane & 4);
    v[0] = dpp_combine<kDppXor2>(v[0], v[1], lane & 2);
    return v[0] + dpp_mov<kDppXor1>(v[0]);
}

// u64 DPP move inside a row of 16 lanes (both halves with the same control)
template <int CTRL>
__device__ inline unsigned long long dpp_mov_u64(unsigned long long u) {
    const unsigned lo = __builtin_amdgcn_update_dpp(0u, (unsigned)u, CTRL, 0xf, 0xf, false);
    const unsigned hi = __builtin_amdgcn_update_dpp(0u, (unsigned)(u >> 32), CTRL, 0xf, 0xf, false);
    return (unsigned long long)hi << 32 | lo;
}

// the partner's value across rows (lane ^ 16 for W = 16, lane ^ 32 for W = 32)
template <int W>
__device__ inline unsigned long long swap_partner_u64(unsigned long long u) {
    unsigned xl = (unsigned)u, xh = (unsigned)(u >> 32), yl = xl, yh = xh;
    if constexpr (W == 32) {
        auto l = __builtin_amdgcn_permlane32_swap(xl, yl, false, false);
        auto h = __builtin_amdgcn_permlane32_swap(xh, yh, false, false);
        xl = l[0]; yl = l[1]; xh = h[0]; yh = h[1];
    } else {
        auto l = __builtin_amdgcn_permlane16_swap(xl, yl, false, false);
        auto h = __builtin_amdgcn_permlane16_swap(xh, yh, false, false);
        xl = l[0]; yl = l[1]; xh = h[0]; yh = h[1];
    }
    // one of the pair is the own value, the other the partner's: min / max need no order
    const unsigned long long a = (unsigned long long)xh << 32 | xl, b = (unsigned long long)yh << 32 | yl;
    return a == u ? b : a;
}

// wave minimum of a u64 key (every lane ends with it) by DPP and permlane swaps: no LDS
// round trip (a __shfl_xor butterfly is 12 ds_bpermute)
__device__ inline unsigned long long wave_min_u64_dpp(unsigned long long v) {
    unsigned long long w;
    w = dpp_mov_u64<kDppXor1>(v); v = w < v ? w : v;
    w = dpp_mov_u64<kDppXor2>(v); v = w < v ? w : v;
    w = dpp_mov_u64<kDppHalfMirror>(v); v = w < v ? w : v;
    w = dpp_mov_u64<kDppRor8>(v); v = w < v ? w : v;
    w = swap_partner_u64<16>(v); v = w < v ? w : v;
    w = swap_partner_u64<32>(v); v = w < v ? w : v;
    return v;
}

// wave maximum of a u32 key (every lane ends with it), the same exchange pattern
__device__ inline unsigned wave_max_u32_dpp(unsigned v) {
    unsigned w;
    w = __builtin_amdgcn_update_dpp(0u, v, kDppXor1, 0xf, 0xf, false); v = w > v ? w : v;
    w = __builtin_amdgcn_update_dpp(0u, v, kDppXor2, 0xf, 0xf, false); v = w > v ? w : v;
    w = __builtin_amdgcn_update_dpp(0u, v, kDppHalfMirror, 0xf, 0xf, false); v = w > v ? w : v;
    w = __builtin_amdgcn_update_dpp(0u, v, kDppRor8, 0xf, 0xf, false); v = w > v ? w : v;
    auto s16 = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    w = s16[0] == v ? s16[1] : s16[0]; v = w > v ? w : v;
    auto s32 = __builtin_amdgcn_permlane32_swap(v, v, false, false);
    w = s32[0] == v ? s32[1] : s32[0]; v = w > v ? w : v;
    return v;
}

// all-reduce of one value over the wave (every lane ends with the same sum: each step adds the
// partner's value, and a + b == b + a)
__device__ inline double wave_sum(double v) {
    v += dpp_mov<kDppXor1>(v);
    v += dpp_mov<kDppXor2>(v);
    v += dpp_mov<kDppHalfMirror>(v);
    v += dpp_mov<kDppRor8>(v);
    v = swap_combine<16>(v, v);
    return swap_combine<32>(v, v);
}

__device__ inline double readlane_d(double v, int l) {
    const unsigned long long u = (unsigned long long)__double_as_longlong(v);
    const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)u, l);
    const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(u >> 32), l);
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

}  // namespace orbmi
