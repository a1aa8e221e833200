// FAST's arc strength on packed 16-bit pairs (host + device, so tests/cpp/fast_score_check.cpp
// can check it against the scalar restatement on the CPU).
//
// OpenCV's cornerScore<16> (fast_score.cpp, called by FAST_t at src/ORBextractor.cc:809-816)
// with d[k] = v - p[k mod 16] runs two scans:
//   a0 = max(th, max over even k of min(m_k, d[k]), min(m_k, d[k + 9])),  m_k = min d[k+1 .. k+8]
//   b0 = min(-a0, min over even k of max(M_k, d[k]), max(M_k, d[k + 9])),  M_k = max d[k+1 .. k+8]
// and returns -b0 - 1.  The even-k windows with one neighbour on either side are every 9-arc of
// the circle, so with e = (d, -d):
//   -b0 = max(th, A, B),  A = max over 9-arcs of min d,  B = max over 9-arcs of min(-d)
// (the scans' early `continue`s skip only updates that cannot change a0 / b0).  A > t is exactly
// "some 9-arc all darker than v - t", B > t "all brighter than v + t": the pixel passes FAST's
// segment test at t >= th exactly when S = max(th, A, B) > t, and its score is S - 1 whatever th
// it was scored at.  One pass of S over the compass survivors is therefore the segment test at
// both thresholds and the score (k_fast2).  Both maxima run at once on (d, -d) pairs: the
// 8-windows' minima from pair minima shared between windows, 47 packed min/max in all.
#pragma once
#include <hip/hip_runtime.h>

namespace orbmi {

typedef short s16x2_t __attribute__((ext_vector_type(2)));

__host__ __device__ inline s16x2_t pk_min16(s16x2_t a, s16x2_t b) { return __builtin_elementwise_min(a, b); }
__host__ __device__ inline s16x2_t pk_max16(s16x2_t a, s16x2_t b) { return __builtin_elementwise_max(a, b); }

// S = max(th, A, B) for centre v and circle p[0..15] (FAST's order, pixels 0..255), th >= 0
__host__ __device__ inline int fast_arc_strength(int v, const int p[16], int th) {
    s16x2_t e[16];
    const s16x2_t vv = {(short)v, (short)-v}, sg = {-1, 1};
#pragma unroll
    for (int k = 0; k < 16; k++) {
        const s16x2_t pp = {(short)p[k], (short)p[k]};
        e[k] = pp * sg + vv;  // (v - p, p - v)
    }
    s16x2_t q[8], r[8];  // q[i] = min e[2i+1 .. 2i+2], r[i] = min e[2i+1 .. 2i+4] (indices mod 16)
#pragma unroll
    for (int i = 0; i < 8; i++) q[i] = pk_min16(e[(2 * i + 1) & 15], e[(2 * i + 2) & 15]);
#pragma unroll
    for (int i = 0; i < 8; i++) r[i] = pk_min16(q[i], q[(i + 1) & 7]);
    s16x2_t c[8];  // k = 2 i: the window k+1 .. k+8 with either neighbour, min(m, max(e[k], e[k+9]))
#pragma unroll
    for (int i = 0; i < 8; i++)
        c[i] = pk_min16(pk_min16(r[i], r[(i + 2) & 7]), pk_max16(e[2 * i], e[(2 * i + 9) & 15]));
#pragma unroll
    for (int w = 4; w >= 1; w >>= 1)  // a tree, so no packed op waits on the one before it
#pragma unroll
        for (int i = 0; i < w; i++) c[i] = pk_max16(c[i], c[i + w]);
    const int s = c[0].x > c[0].y ? c[0].x : c[0].y;
    return s > th ? s : th;
}

}  // namespace orbmi
