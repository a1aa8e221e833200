// Optimizer::LocalBundleAdjustment (src/Optimizer.cc:483-808) on MI355X, fp64.
//
// The g2o schedule -- optimize(5), outlier levels, optimize(10), erase list -- runs as a chain
// of chip-wide kernels on one stream, with the Levenberg control (g2o/core/
// optimization_algorithm_levenberg.cpp:61-164) on the device.  Once per optimize():
//   k_ba_linearize     thread / edge   computeActiveErrors + robust chi2, Jacobians
//                                      (types_six_dof_expmap.cpp), Huber weights, the edge's
//                                      Hpl block and its Hll / b_l, Hpp / b_p contributions
//   k_ba_reduce        thread / point  Hll, b_l (sum over the point's edges, g2o order)
//                      block / pose    max |diag H| for computeLambdaInit
// per trial (lambda), three launches:
//   k_ba_schur         block / (pose i <= pose j)  H_schur(i,j) = Hpp + lambda I - sum_points
//                                      B_i D^-1 B_j^T over observation pairs (lists built once),
//                                      Hpp / b_p summed over the keyframe's edges in the diagonal
//                                      blocks, b_schur = b_p - sum B D^-1 b_l
//   k_ba_solve         one block       blocked (6x6) LDL^T of the 6K x 6K reduced system with the
//                                      right-hand side carried through, back substitution,
//                                      trial poses exp(dx) * T, poses' part of computeScale
//   k_ba_update_errors thread / point  back substitution x + dx, trial errors, computeScale, and
//                                      the linearisation at the trial state into the second
//                                      linear-system buffer (an accepted trial's next iteration
//                                      starts with computeActiveErrors + buildSystem at exactly
//                                      that state, so the buffers swap; a rejected trial keeps
//                                      the current system); its last block runs the Levenberg
//                                      decision (k_ba_control_body)
// The g2o semantics kept: lambda init tau = 1e-5, rho test with computeScale + 1e-3, the
// ORB-SLAM "3 bad iterations" stop, stale edge errors after a rejected trial, push/pop of
// the estimates (pointer swap of current / trial buffers), Huber kernels removed for the
// second pass.  Every reduction has a fixed order (deterministic).  Parity with the oracle: 1e-4.
#include <algorithm>
#include <cfloat>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <cstring>
#include <new>
#include <thread>
#include <vector>

#include "extractor.h"
#include "se3_device.h"
#include "wave_ops.h"

// The fan-ins between workgroups (k_ba_update_errors, k_ba_errors, the keyframe halves of
// k_ba_schur) hand partial sums over without __threadfence: agent-scope relaxed (sc1) stores
// drained by s_waitcnt vmcnt(0) before a relaxed arrival atomicAdd, read back by sc1 loads.
// That is ordered on gfx9's memory system (the store completes at L2 before the counter moves;
// sc1 loads bypass the non-coherent L1), not by the HIP/LLVM memory model, so the file builds
// only for the target it was validated on (MI355X_MICROARCH.md, inter-workgroup hand-offs).
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__gfx950__)
#error "lba.hip's fence-free fan-ins are validated on gfx950 only"
#endif

// fp64 solver with a 1e-4 parity tolerance: multiply-add contraction allowed here (the
// bit-exact extractor / matcher sources keep -ffp-contract=off)
#pragma clang fp contract(fast)

namespace orbmi {

constexpr int kBaMaxPoses = 30;                        // 6*30 = 180 unknowns
constexpr int kBaMaxN = 6 * kBaMaxPoses;
constexpr int kBaPacked = kBaMaxN * (kBaMaxN + 1) / 2;  // 16290 doubles = 127 KiB
constexpr int kBaMaxKf = 1024;
constexpr int kBaBlock = 256;

// Levenberg state of one SparseOptimizer::optimize(n) call, kept on the device so that the
// trials run back to back without a host round trip (optimization_algorithm_levenberg.cpp:61-164).
struct BaCtl {
    int cur;          // which of the two estimate buffers (Tb, Xb) holds the current state
    int it, max_it;   // iterations finished / requested
    int trial;        // qmax of the current iteration
    int need_lin;     // the next step starts an iteration (computeActiveErrors + linearize)
    int done;         // optimize() has returned (iterations exhausted, terminate, stop)
    int nbad;         // ORB-SLAM2's consecutive iterations without a 1e-3 relative decrease
    int np, nl;       // free poses / active points of the index mapping
    int unsupported;  // more than kBaMaxPoses active poses
    int steps;        // trial steps executed (diagnostics)
    int lin;          // which of the two linear-system buffers holds the current system
    unsigned arrive;  // blocks of k_ba_update_errors finished (the last one runs the control)
    unsigned arrive_s;  // blocks of k_ba_schur_solve finished (the last one solves)
    unsigned arrive_e;  // blocks of k_ba_activate_edges / k_ba_errors finished (the last one
                        // runs the one-wave tail: the LM state set-up / activeRobustChi2)
    double lambda, ni, currentChi, iniChi;
    double chi_out[2];  // activeRobustChi2 after optimize(5) / optimize(10)
    int it_out[2];      // iterations of optimize(5) / optimize(10); -1 with an empty mapping
    // The whole call is enqueued at once (Runner); these gate each kernel to its optimize():
    int gen;          // the optimize() the LM state belongs to (1: optimize(5), 2: optimize(10))
    int phases_done;  // optimize() calls finished (k_ba_errors' tail)
    int do_more;      // optimize(10) runs: pbStopFlag was clear after optimize(5) (:689-692)
    int checks;       // pbStopFlag checks made so far (#0 is the host's, src/Optimizer.cc:685)
    int stop_seen;    // the first check that found the flag raised (-1: none)
};

struct BaDev {
    int run_gen;                    // the optimize() (BaCtl::gen) a launch belongs to
    int nkf, npt, nedge, nblk, nf;  // nf = non-fixed keyframes (nblk = nf (nf + 1) / 2)
    int nb_e, nb_p, nb_q;           // blocks: edges (256), points (256), points (kBaUpdPts per block)
    BaCtl* ctl;
    const volatile int* stop;  // host-mapped mirror of pbStopFlag (may be null)
    int stop_at;               // orbmi_ba_set_stop_at_check: the flag reads raised from this check on (< 0: off)
    double* Tb[2];             // poses: SE3Quat (x, y, z, w, tx, ty, tz, -), current / trial
    double* Xb[2];             // points (x, y, z, -), current / trial
    double* part_lin;          // nb_e: robust chi2 at linearisation
    double* part_tchi;         // nb_q: trial robust chi2
    double* part_tscale;       // nb_q: trial computeScale (points)
    double* part_max;          // nb_p + kBaMaxPoses: max |diag H|
    const orbmi_ba_keyframe* kfs;
    const orbmi_ba_point* pts;
    const orbmi_ba_edge* edges;
    const int* kf_order;       // keyframe indices sorted by id (vertex order)
    const int* free_kf;        // nf: the non-fixed keyframes in id order (the b_schur blocks')
    double* part_kf;           // kBaMaxPoses x kSchurKfSplit x 64: the keyframe blocks' half sums
    unsigned* arrive_kf;       // kBaMaxPoses: halves of a keyframe's sums arrived (k_ba_setup zeroes)
    const int* pt_start;       // edges of point p: [pt_start[p], pt_start[p+1])
    const int* kf_start;       // CSR by keyframe over edge indices
    const int* kf_edges;
    const int* kf_pos;         // position of edge e in the keyframe CSR (kf_edges[kf_pos[e]] == e)
    const int* kf_pt;          // point of the edge at keyframe-CSR position j
    const int* blk_kf;         // nblk x 2: keyframes (a, b), id(a) <= id(b), both not fixed
    int* blk_cnt;              // nblk: pairs per block (k_ba_pairs_count)
    int* blk_start;            // nblk + 1 (k_ba_pairs_fill)
    int2* blk_pairs;           // (e_a, e_b): edges of one point into keyframes a and b
    int* blk_pt;               // the pair's point (so k_ba_schur's loads of a pair go out together)
    double* err;               // nedge x 3 (stale semantics)
    unsigned char* eflag;      // bit0 level-1, bit1 no robust kernel, bit2 active
    int* pose_idx;             // nkf
    int* pose_kf;              // kBaMaxPoses
    int* e_pi;                 // nedge: pose index of the edge's keyframe (-1 fixed / inactive)
    int* kf_act;               // nkf: activation generation that saw an active edge of the keyframe
    // the linear system: Hplb[L] etc. with L = ctl->lin is the current one (ba_sys selects it)
    double* Hpl;               // nedge x 18 (pose rows x point cols)
    double* Hle;               // nedge x 9: edge's Hll upper (6) + b_l (3)
    double* Hpe;               // nedge x 27 in keyframe-CSR order: edge's Hpp upper (21) + b_p (6)
    double* Hll;               // npt x 9
    double* bl;                // npt x 3
    double* Hplb[2];
    double* Hleb[2];
    double* Hpeb[2];
    double* Hllb[2];
    double* blb[2];
    double* Hpp;               // kBaMaxPoses x 36
    double* bp;                // kBaMaxPoses x 6 (k_ba_schur, read by the solve)
    double* S;                 // reduced system: packed upper (kBaPacked), or in k_ba_solve_mfma's
                               // tile layout when mfma_T > 0 (mfma_tile_pos)
    int mfma_T;                // tiles per dimension of the MFMA solve (0: the VALU solves)
    double* bs;                // kBaMaxN
    double* xp;                // kBaMaxN
    double* scal;              // [1] poses' computeScale part, [2] solve ok, [3] lambda used
    int* istat;                // [0] np, [1] nl, [2] too many poses, [3] solve ok
};

// the linear system of buffer L (kernels select ctl->lin on entry)
struct BaSys { double *Hpl, *Hle, *Hpe, *Hll, *bl; };
__device__ inline BaSys ba_sys(const BaDev& a, int L) {
    return BaSys{L ? a.Hplb[1] : a.Hplb[0], L ? a.Hleb[1] : a.Hleb[0], L ? a.Hpeb[1] : a.Hpeb[0],
                 L ? a.Hllb[1] : a.Hllb[0], L ? a.blb[1] : a.blb[0]};
}
__device__ inline void ba_use(BaDev& a, int L) {
    const BaSys y = ba_sys(a, L);
    a.Hpl = y.Hpl; a.Hle = y.Hle; a.Hpe = y.Hpe; a.Hll = y.Hll; a.bl = y.bl;
}

// ---------------------------------------------------------------- edges
__device__ inline bool edge_stereo(const orbmi_ba_edge& e) { return !(e.ur < 0); }

// The edge math works on values (the edge record, its keyframe's camera, the pose Tk) so that a
// kernel can load them once, early, and keep them in registers; the a-based helpers below load
// them from the arrays.
struct BaCam { float fx, fy, cx, cy, bf; };
__device__ inline BaCam ba_cam(const orbmi_ba_keyframe& k) { return BaCam{k.fx, k.fy, k.cx, k.cy, k.bf}; }

// error of edge e with the point's position at Xp (3 doubles)
__device__ inline void edge_err_math(const orbmi_ba_edge& e, const BaCam& kf, const double* Tk, const double* Xp,
                                     double* err) {
    double p[3];
    se3_map(Tk, Xp, p);
    if (!edge_stereo(e)) {
        const double px = p[0] / p[2], py = p[1] / p[2];
        err[0] = (double)e.u - (px * (double)kf.fx + (double)kf.cx);
        err[1] = (double)e.v - (py * (double)kf.fy + (double)kf.cy);
        err[2] = 0;
    } else {
        const float invz = (float)(1.0f / p[2]);  // float invz (types_six_dof_expmap.cpp:151)
        const double r0 = p[0] * invz * (double)kf.fx + (double)kf.cx;
        const double r1 = p[1] * invz * (double)kf.fy + (double)kf.cy;
        const double r2 = r0 - (double)(kf.bf * invz);
        err[0] = (double)e.u - r0;
        err[1] = (double)e.v - r1;
        err[2] = (double)e.ur - r2;
    }
}

__device__ inline double edge_chi2_math(const orbmi_ba_edge& e, const double* r) {
    const double info = (double)e.inv_sigma2;
    return r[0] * (info * r[0]) + r[1] * (info * r[1]) + (edge_stereo(e) ? r[2] * (info * r[2]) : 0.0);
}

__device__ inline double huber_delta(const orbmi_ba_edge& e) {
    // const float thHuberMono = sqrt(5.991), thHuberStereo = sqrt(7.815) (src/Optimizer.cc:599-600)
    const float th = edge_stereo(e) ? (float)sqrt(7.815) : (float)sqrt(5.991);
    return (double)th;
}

// robustified chi2 and weight rho' (RobustKernelHuber::robustify); fl = the edge's eflag
__device__ inline void edge_robust_math(unsigned char fl, const orbmi_ba_edge& e, double c, double* rho0, double* rho1) {
    if (fl & 2) { *rho0 = c; *rho1 = 1.0; return; }
    const double d = huber_delta(e), dsqr = d * d;
    if (c <= dsqr) { *rho0 = c; *rho1 = 1.0; }
    else { const double s = sqrt(c); *rho0 = 2 * s * d - dsqr; *rho1 = d / s; }
}

// Jacobians (types_six_dof_expmap.cpp:103-134, :188-234)
__device__ inline void edge_jac_math(const orbmi_ba_edge& e, const BaCam& kf, const double* Tk, const double* Xp,
                                     double Jl[3][3], double Jp[3][6]) {
    double p[3], R[3][3];
    se3_map(Tk, Xp, p);
    q_to_matrix(load_q(Tk), R);
    // one reciprocal per edge (fast_rcp: within an ulp of 1 / z) instead of the reference's
    // divisions; the Jacobians only steer the Levenberg steps (parity 1e-4), the errors and
    // chi2 keep the exact divisions
    const double x = p[0], y = p[1], z = p[2], iz = fast_rcp(z), iz2 = iz * iz;
    const double fx = kf.fx, fy = kf.fy, bf = kf.bf;
    if (!edge_stereo(e)) {
        const double t02 = -x * iz * fx, t12 = -y * iz * fy;
        for (int c = 0; c < 3; c++) {
            Jl[0][c] = -iz * (fx * R[0][c] + t02 * R[2][c]);
            Jl[1][c] = -iz * (fy * R[1][c] + t12 * R[2][c]);
            Jl[2][c] = 0;
        }
    } else {
        for (int c = 0; c < 3; c++) {
            Jl[0][c] = -fx * R[0][c] * iz + fx * x * R[2][c] * iz2;
            Jl[1][c] = -fy * R[1][c] * iz + fy * y * R[2][c] * iz2;
            Jl[2][c] = Jl[0][c] - bf * R[2][c] * iz2;
        }
    }
    Jp[0][0] = x * y * iz2 * fx; Jp[0][1] = -(1 + (x * x * iz2)) * fx; Jp[0][2] = y * iz * fx;
    Jp[0][3] = -iz * fx; Jp[0][4] = 0; Jp[0][5] = x * iz2 * fx;
    Jp[1][0] = (1 + y * y * iz2) * fy; Jp[1][1] = -x * y * iz2 * fy; Jp[1][2] = -x * iz * fy;
    Jp[1][3] = 0; Jp[1][4] = -iz * fy; Jp[1][5] = y * iz2 * fy;
    if (edge_stereo(e)) {
        Jp[2][0] = Jp[0][0] - bf * y * iz2; Jp[2][1] = Jp[0][1] + bf * x * iz2; Jp[2][2] = Jp[0][2];
        Jp[2][3] = Jp[0][3]; Jp[2][4] = 0; Jp[2][5] = Jp[0][5] - bf * iz2;
    } else {
        for (int c = 0; c < 6; c++) Jp[2][c] = 0;
    }
}

// weight W = rho' * info and omega_r = -info * e * rho' (constructQuadraticForm), err = the
// edge's current error
__device__ inline void edge_weights_math(unsigned char fl, const orbmi_ba_edge& ed, const double* err, double* w,
                                         double om[3]) {
    const double info = (double)ed.inv_sigma2;
    double r0, r1;
    edge_robust_math(fl, ed, edge_chi2_math(ed, err), &r0, &r1);
    *w = (fl & 2) ? info : r1 * info;
    const double s = (fl & 2) ? 1.0 : r1;
    for (int k = 0; k < 3; k++) om[k] = -(info * err[k]) * s;
}

// the a-based forms (they load the edge, its keyframe and pose from the arrays)
__device__ inline void edge_error_at(const BaDev& a, int i, const double* T, const double* Xp, double* err) {
    const orbmi_ba_edge e = a.edges[i];
    edge_err_math(e, ba_cam(a.kfs[e.kf]), T + 8 * e.kf, Xp, err);
}

__device__ inline void edge_error(const BaDev& a, int i, const double* T, const double* X, double* err) {
    edge_error_at(a, i, T, X + 4 * a.edges[i].point, err);
}

__device__ inline double edge_chi2(const BaDev& a, int i) { return edge_chi2_math(a.edges[i], a.err + 3 * i); }

__device__ inline void edge_robust(const BaDev& a, int i, double c, double* rho0, double* rho1) {
    edge_robust_math(a.eflag[i], a.edges[i], c, rho0, rho1);
}

// ---------------------------------------------------------------- block helpers
template <int NT>
__device__ inline double block_sum(double v, double* red) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    double t = 0;
    for (int w = 0; w < NT / 64; w++) t += red[w];
    __syncthreads();
    return t;
}

// two block sums in one pass, the results in thread 0 only: the same butterfly per wave and the
// same wave order as block_sum (bit-identical sums), one barrier instead of four
template <int NT>
__device__ inline void block_sum2_t0(double& x, double& y, double* red /* 2 NT / 64 */) {
    for (int o = 32; o > 0; o >>= 1) {
        x += __shfl_xor(x, o, 64);
        y += __shfl_xor(y, o, 64);
    }
    if ((threadIdx.x & 63) == 0) {
        red[threadIdx.x >> 6] = x;
        red[NT / 64 + (threadIdx.x >> 6)] = y;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        x = 0;
        y = 0;
        for (int w = 0; w < NT / 64; w++) x += red[w];
        for (int w = 0; w < NT / 64; w++) y += red[NT / 64 + w];
    }
}

template <int NT>
__device__ inline double block_max(double v, double* red) {
    for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, 64));
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    double t = 0;
    for (int w = 0; w < NT / 64; w++) t = fmax(t, red[w]);
    __syncthreads();
    return t;
}

__device__ inline int packed(int r, int c, int N) { return r * N - r * (r - 1) / 2 + (c - r); }  // r <= c

// position of element (R, C) of the reduced system in the MFMA solve's tile layout (k_ba_schur
// writes it, k_ba_solve_mfma loads it with one coalesced read per tile register): tile
// (R >> 4, C >> 4) of the upper triangle numbered row by row with the right-hand side as tile
// column T (C = 16 T), MFMA C layout inside the tile.  Diagonal tiles hold both triangles.
__host__ __device__ inline int mfma_tile_pos(int T, int R, int C) {
    const int i = R >> 4, j = C >> 4, rr = R & 15;
    return (i * (T + 1) - i * (i - 1) / 2 + (j - i)) * 256 + (rr >> 2) * 64 + 16 * (rr & 3) + (C & 15);
}


__device__ inline bool point_active(const BaDev& a, int p) {
    for (int i = a.pt_start[p]; i < a.pt_start[p + 1]; i++)
        if (a.eflag[i] & 4) return true;
    return false;
}

// ---------------------------------------------------------------- setup / activation
// vertices: SE3Quat from float Tcw (Converter::toSE3Quat), points to double
// One read of pbStopFlag (the caller's flag through its host-mapped mirror, or the deterministic
// stop_at hook), numbered in the order the reference evaluates them (orbmi_ba_set_stop_at_check);
// one lane.  The reads are where g2o reads _forceStopFlag: SparseOptimizer::optimize's loop
// condition (sparse_optimizer.cpp:376), the LM inner loop's (levenberg.cpp:149), and
// src/Optimizer.cc:689.
__device__ inline bool ba_check_stop(const BaDev& a, BaCtl& c) {
    const int idx = c.checks++;
    const bool s = (a.stop && *a.stop) || (a.stop_at >= 0 && idx >= a.stop_at);
    if (s && c.stop_seen < 0) c.stop_seen = idx;
    return s;
}

__global__ __launch_bounds__(kBaBlock) void k_ba_setup(BaDev a, double* __restrict__ T, double* __restrict__ X,
                                                       unsigned char* __restrict__ out_erase) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i == 0) {  // the control block and the index statistics start cleared; check #0
                   // (src/Optimizer.cc:685) was the host's, and found the flag clear
        BaCtl c = {};
        c.checks = 1;
        c.stop_seen = -1;
        *a.ctl = c;
        for (int k = 0; k < 8; k++) a.istat[k] = 0;
    }
    if (i < a.nkf) {
        const float* t = a.kfs[i].tcw;
        double R[3][3];
        for (int r = 0; r < 3; r++)
            for (int c = 0; c < 3; c++) R[r][c] = t[4 * r + c];
        Q q = q_from_matrix(R);
        q_normalize(q);
        double* Ti = T + 8 * i;
        Ti[0] = q.x; Ti[1] = q.y; Ti[2] = q.z; Ti[3] = q.w; Ti[4] = t[3]; Ti[5] = t[7]; Ti[6] = t[11]; Ti[7] = 0;
        a.kf_act[i] = 0;
    }
    if (i < a.nf) a.arrive_kf[i] = 0;
    if (i < a.npt) {
        for (int r = 0; r < 3; r++) X[4 * i + r] = a.pts[i].pos[r];
        X[4 * i + 3] = 0;
    }
    if (i < a.nedge) {
        a.eflag[i] = 0;
        out_erase[i] = 0;
        a.err[3 * i] = a.err[3 * i + 1] = a.err[3 * i + 2] = 0;
    }
}

// outlier levels, kernels off before the second optimisation (src/Optimizer.cc:701-732);
// chi2 from the stale errors, depth from the current estimate
__global__ __launch_bounds__(kBaBlock) void k_ba_levels(BaDev a) {
    if (!(a.ctl->phases_done >= 1 && a.ctl->do_more)) return;  // optimize(5) pending or no optimize(10)
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const double* T = a.Tb[a.ctl->cur];
    const double* X = a.Xb[a.ctl->cur];
    if (i >= a.nedge) return;
    const orbmi_ba_edge e = a.edges[i];
    if (a.pts[e.point].bad) return;
    double p[3];
    se3_map(T + 8 * e.kf, X + 4 * e.point, p);
    const double th = edge_stereo(e) ? 7.815 : 5.991;
    unsigned char f = a.eflag[i] & 3;
    if (edge_chi2(a, i) > th || !(p[2] > 0.0)) f |= 1;
    f |= 2;
    a.eflag[i] = f;
}

// SparseOptimizer::initializeOptimization(level 0) + buildIndexMapping, in two launches.
// Grid part: edges of level 0 become active (bit 2), their keyframes are marked (kf_act = gen)
// and each block counts the points whose first active edge it holds (partials in part_lin,
// which the next linearisation overwrites).  Bit 0 is never rewritten, so reading it from the
// point's other edges while they are updated is safe.
__device__ inline void activate_ctl_body(const BaDev& a, int max_it, int gen);
__global__ __launch_bounds__(kBaBlock) void k_ba_activate_edges(BaDev a, int max_it, int gen) {
    if (gen > 1 && !(a.ctl->phases_done >= gen - 1 && a.ctl->do_more)) return;
    __shared__ double red[kBaBlock / 64];
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    int first = 0;
    if (i < a.nedge) {
        unsigned char f = a.eflag[i] & 3;
        if (!(f & 1)) {
            f |= 4;
            const orbmi_ba_edge e = a.edges[i];
            a.kf_act[e.kf] = gen;
            first = 1;
            for (int j = a.pt_start[e.point]; j < i; j++)
                if (!(a.eflag[j] & 1)) { first = 0; break; }
        }
        a.eflag[i] = f;
    }
    const double n = block_sum<kBaBlock>((double)first, red);
    __shared__ bool last;
    if (threadIdx.x == 0) {
        a.part_lin[blockIdx.x] = n;
        __threadfence();
        last = atomicAdd(&a.ctl->arrive_e, 1u) == gridDim.x - 1;
    }
    __syncthreads();
    if (!last) return;
    __threadfence();  // every block's eflag / kf_act / part_lin
    if (threadIdx.x < 64) activate_ctl_body(a, max_it, gen);  // one wave: the LM state
    if (threadIdx.x == 0) a.ctl->arrive_e = 0;
}

// One wave: the number of active points, pose indices in vertex-id order (poses first) by a
// ballot scan over the id-ordered keyframes, and the LM state of levenberg.cpp:61-70.  The
// edges' pose indices (e_pi) are written by the next k_ba_linearize.
__device__ inline void activate_ctl_body(const BaDev& a, int max_it, int gen) {
    const int lane = threadIdx.x;
    double c = 0;
    for (int b = lane; b < a.nb_e; b += 64) c += a.part_lin[b];
    const int nl = (int)wave_sum(c);
    int n = 0;
    for (int o0 = 0; o0 < a.nkf; o0 += 64) {
        const int oi = o0 + lane;
        int k = -1;
        bool take = false;
        if (oi < a.nkf) {
            k = a.kf_order[oi];
            take = !a.kfs[k].fixed && a.kf_act[k] == gen;
        }
        const unsigned long long m = __ballot(take);
        const int idx = n + __popcll(m & ((1ull << lane) - 1));
        if (k >= 0) {
            a.pose_idx[k] = take && idx < kBaMaxPoses ? idx : -1;
            if (take && idx < kBaMaxPoses) a.pose_kf[idx] = k;
        }
        n += __popcll(m);
    }
    if (lane == 0) {
        a.istat[0] = n;
        a.istat[1] = nl;
        a.istat[2] = n > kBaMaxPoses;
        BaCtl& c2 = *a.ctl;
        c2.np = min(n, kBaMaxPoses);
        c2.nl = nl;
        c2.unsupported |= n > kBaMaxPoses;
        c2.it = 0;
        c2.max_it = max_it;
        c2.trial = 0;
        c2.need_lin = 1;
        c2.nbad = 0;
        c2.lambda = 0;
        c2.ni = 2;
        // SparseOptimizer::optimize: no vertex -> return -1 before the loop; else the loop
        // condition `i < iterations && !terminate()` before iteration 0
        const bool empty = n + nl == 0;
        const bool stopped = !empty && max_it > 0 && ba_check_stop(a, c2);
        c2.done = empty || c2.unsupported || max_it <= 0 || stopped;
        c2.gen = gen;
    }
}

// ---------------------------------------------------------------- Schur pair lists
// Block (a, b) of the reduced system sums over the points keyframes a and b both observe: the
// pairs (e_a, e_b) of their edges, ordered by point, then edge (the order the points' edges
// are inserted).  A keyframe's CSR lists its edges in edge order, hence by point: each edge of
// a looks its point up in b's list by binary search (staged in LDS when it fits).
constexpr int kPairThreads = 256;
constexpr int kPairLdsPts = 4096;

// [lo, hi) of point p in the sorted list l[0..n)
__device__ inline int2 pair_range(const int* __restrict__ l, int n, int p) {
    int lo = 0, hi = n;
    while (lo < hi) {
        const int m = (lo + hi) >> 1;
        if (l[m] < p) lo = m + 1; else hi = m;
    }
    int e = lo;
    hi = n;
    while (e < hi) {
        const int m = (e + hi) >> 1;
        if (l[m] <= p) e = m + 1; else hi = m;
    }
    return make_int2(lo, e);
}

// stages b's point list; returns the list to search (LDS or global)
__device__ inline const int* pair_list_b(const BaDev& a, int kb, int* lds, int* nb) {
    const int b0 = a.kf_start[kb];
    *nb = a.kf_start[kb + 1] - b0;
    if (*nb > kPairLdsPts) return a.kf_pt + b0;
    for (int j = threadIdx.x; j < *nb; j += blockDim.x) lds[j] = a.kf_pt[b0 + j];
    __syncthreads();
    return lds;
}

__global__ __launch_bounds__(kPairThreads) void k_ba_pairs_count(BaDev a) {
    __shared__ int lb[kPairLdsPts];
    __shared__ int scratch[kPairThreads / 64];
    const int b = blockIdx.x, ka = a.blk_kf[2 * b], kb = a.blk_kf[2 * b + 1];
    int nb;
    const int* L = pair_list_b(a, kb, lb, &nb);
    int cnt = 0;
    for (int j = a.kf_start[ka] + threadIdx.x; j < a.kf_start[ka + 1]; j += blockDim.x) {
        const int2 r = pair_range(L, nb, a.kf_pt[j]);
        cnt += r.y - r.x;
    }
    int total;
    block_excl_scan(cnt, scratch, &total);
    if (threadIdx.x == 0) a.blk_cnt[b] = total;
}

__global__ __launch_bounds__(kPairThreads) void k_ba_pairs_fill(BaDev a) {
    __shared__ int lb[kPairLdsPts];
    __shared__ int scratch[kPairThreads / 64];
    const int b = blockIdx.x, ka = a.blk_kf[2 * b], kb = a.blk_kf[2 * b + 1];
    int before = 0;  // pairs of the blocks before b
    for (int q = threadIdx.x; q < b; q += blockDim.x) before += a.blk_cnt[q];
    int off;
    block_excl_scan(before, scratch, &off);
    if (threadIdx.x == 0) {
        a.blk_start[b] = off;
        if (b == a.nblk - 1) a.blk_start[a.nblk] = off + a.blk_cnt[b];
    }
    int nb;
    const int* L = pair_list_b(a, kb, lb, &nb);
    const int b0 = a.kf_start[kb], a0 = a.kf_start[ka], a1 = a.kf_start[ka + 1];
    for (int c = a0; c < a1; c += blockDim.x) {  // chunks of a's list, in order
        const int j = c + threadIdx.x;
        int2 r = make_int2(0, 0);
        if (j < a1) r = pair_range(L, nb, a.kf_pt[j]);
        int total;
        const int o = off + block_excl_scan(r.y - r.x, scratch, &total);
        if (j < a1) {
            const int ea = a.kf_edges[j];
            const int pt = a.kf_pt[j];
            for (int t = r.x; t < r.y; t++) {
                a.blk_pairs[o + t - r.x] = make_int2(ea, a.kf_edges[b0 + t]);
                a.blk_pt[o + t - r.x] = pt;
            }
        }
        off += total;
    }
}

// ---------------------------------------------------------------- errors
// computeActiveErrors (recompute = 1) + activeRobustChi2; per-block partial sums
// activeRobustChi2 on the stored (possibly stale) errors; per-block partial sums
__device__ inline void chi_body(const BaDev& a, int phase);
__global__ __launch_bounds__(kBaBlock) void k_ba_errors(BaDev a, int phase) {
    if (!(a.ctl->done && a.ctl->gen == a.run_gen)) return;  // its optimize() still running
    __shared__ double red[kBaBlock / 64];
    double* part = a.part_lin;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    double s = 0;
    if (i < a.nedge && (a.eflag[i] & 4)) {
        double r0, r1;
        edge_robust(a, i, edge_chi2(a, i), &r0, &r1);
        s = r0;
    }
    s = block_sum<kBaBlock>(s, red);
    __shared__ bool last;
    if (threadIdx.x == 0) {  // the fan-in as k_ba_update_errors': sc1 store drained before the add
        __hip_atomic_store(&part[blockIdx.x], s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        last = atomicAdd(&a.ctl->arrive_e, 1u) == gridDim.x - 1;
    }
    __syncthreads();
    if (!last) return;
    if (threadIdx.x < 64) chi_body(a, phase);  // one wave: the partials in a fixed order (sc1 loads)
    if (threadIdx.x == 0) a.ctl->arrive_e = 0;
}

// ---------------------------------------------------------------- linear system
// D^-1 of the point's damped 3x3 block, Hll + lambda I (cofactors)
__device__ inline void point_dinv(const double* Hll, int p, double lam, double Di[9]) {
    double D[3][3];
    for (int r = 0; r < 3; r++)
        for (int c = 0; c < 3; c++) D[r][c] = Hll[9 * p + 3 * r + c] + (r == c ? lam : 0.0);
    const double c00 = D[1][1] * D[2][2] - D[1][2] * D[2][1];
    const double c10 = D[1][2] * D[2][0] - D[1][0] * D[2][2];
    const double c20 = D[1][0] * D[2][1] - D[1][1] * D[2][0];
    const double det = D[0][0] * c00 + D[0][1] * c10 + D[0][2] * c20;
    const double id = 1.0 / det;
    Di[0] = c00 * id; Di[3] = c10 * id; Di[6] = c20 * id;
    Di[1] = (D[0][2] * D[2][1] - D[0][1] * D[2][2]) * id;
    Di[4] = (D[0][0] * D[2][2] - D[0][2] * D[2][0]) * id;
    Di[7] = (D[0][1] * D[2][0] - D[0][0] * D[2][1]) * id;
    Di[2] = (D[0][1] * D[1][2] - D[0][2] * D[1][1]) * id;
    Di[5] = (D[0][2] * D[1][0] - D[0][0] * D[1][2]) * id;
    Di[8] = (D[0][0] * D[1][1] - D[0][1] * D[1][0]) * id;
}

// thread per edge: computeActiveErrors + robust chi2 (block partials), then
// BaseBinaryEdge::constructQuadraticForm (base_binary_edge.hpp:55-120): Hpl block, the
// edge's Hll / b_l and Hpp / b_p contributions.  Inactive edges into free poses write zeros,
// so the reductions and the Schur products need no activity tests.
// BaseBinaryEdge::constructQuadraticForm of edge i at (T, point position Xp) into a's linear
// system (errors already in a.err): Hpl block, the edge's Hll / b_l and Hpp / b_p contributions.
// Inactive edges into free poses write zeros, so the reductions and the Schur products need no
// activity tests.  Returns nothing; pi = pose index of the edge's keyframe (-1 fixed).
__device__ inline void edge_linearize_math(const BaSys& y, int i, int pi, int kpos, bool active, const orbmi_ba_edge& ed,
                                           const BaCam& kf, const double* Tk, unsigned char fl, const double* err,
                                           const double* Xp, double* He_out) {
    const bool free_pose = pi >= 0;
    double* Hp = y.Hpe + 27 * (long long)kpos;
    double* B = y.Hpl + 18 * (long long)i;
    if (!active) {
        if (free_pose) {
            for (int q = 0; q < 27; q++) Hp[q] = 0;
            for (int q = 0; q < 18; q++) B[q] = 0;
        }
        return;
    }
    double Jl[3][3], Jp[3][6], w, om[3];
    edge_jac_math(ed, kf, Tk, Xp, Jl, Jp);
    edge_weights_math(fl, ed, err, &w, om);
    double* He = He_out ? He_out : y.Hle + 9 * (long long)i;
    int q = 0;
    for (int r = 0; r < 3; r++)
        for (int c = r; c < 3; c++, q++)
            He[q] = Jl[0][r] * w * Jl[0][c] + Jl[1][r] * w * Jl[1][c] + Jl[2][r] * w * Jl[2][c];
    for (int r = 0; r < 3; r++) He[6 + r] = Jl[0][r] * om[0] + Jl[1][r] * om[1] + Jl[2][r] * om[2];
    if (free_pose) {
        for (int r = 0; r < 6; r++)
            for (int c = 0; c < 3; c++)
                B[r * 3 + c] = Jp[0][r] * w * Jl[0][c] + Jp[1][r] * w * Jl[1][c] + Jp[2][r] * w * Jl[2][c];
        q = 0;
        for (int r = 0; r < 6; r++)
            for (int c = r; c < 6; c++, q++)
                Hp[q] = Jp[0][r] * w * Jp[0][c] + Jp[1][r] * w * Jp[1][c] + Jp[2][r] * w * Jp[2][c];
        for (int r = 0; r < 6; r++) Hp[21 + r] = Jp[0][r] * om[0] + Jp[1][r] * om[1] + Jp[2][r] * om[2];
    }
}

__device__ inline void edge_linearize(const BaDev& a, const BaSys& y, int i, int pi, bool active, const double* T,
                                      const double* Xp, double* He_out = nullptr) {
    const orbmi_ba_edge ed = a.edges[i];
    edge_linearize_math(y, i, pi, a.kf_pos[i], active, ed, ba_cam(a.kfs[ed.kf]), T + 8 * ed.kf, a.eflag[i], a.err + 3 * i,
                        Xp, He_out);
}

// An edge of k_ba_update_errors with everything its trial pass reads except the point position,
// loaded in one round (the keyframe's camera and trial pose right behind the record)
struct EdgeIn {
    orbmi_ba_edge e;
    BaCam cam;
    double T[8];
    int pi, kpos;
    unsigned char fl;
};
__device__ inline void edge_in_static(const BaDev& a, int i, EdgeIn& s) {  // fixed within an optimize()
    s.e = a.edges[i];
    s.fl = a.eflag[i];
    s.pi = a.e_pi[i];
    s.kpos = a.kf_pos[i];
    s.cam = ba_cam(a.kfs[s.e.kf]);
}
__device__ inline void edge_in_pose(const double* T, EdgeIn& s) {
#pragma unroll
    for (int q = 0; q < 8; q++) s.T[q] = T[8 * s.e.kf + q];
}
__device__ inline void edge_in(const BaDev& a, int i, const double* T, EdgeIn& s) {
    edge_in_static(a, i, s);
    edge_in_pose(T, s);
}

// computeActiveErrors + robust chi2 + the linearisation of one edge at the trial state from
// registers (the error goes to a.err and stays in registers for the weights)
__device__ inline double edge_trial(const BaDev& a, const BaSys& t, int i, const EdgeIn& s, const double* Xp,
                                    double* He_out) {
    const bool active = s.fl & 4;
    double err[3] = {0, 0, 0}, r0 = 0;
    if (active) {
        edge_err_math(s.e, s.cam, s.T, Xp, err);
        double* eo = a.err + 3 * i;
        eo[0] = err[0]; eo[1] = err[1]; eo[2] = err[2];
        double r1;
        edge_robust_math(s.fl, s.e, edge_chi2_math(s.e, err), &r0, &r1);
    }
    edge_linearize_math(t, i, s.pi, s.kpos, active, s.e, s.cam, s.T, s.fl, err, Xp, He_out);
    return r0;
}

// thread per edge, the first linearisation of an optimize(): computeActiveErrors + robust chi2
// (block partials), then the edge's blocks (edge_linearize) into the current linear system
__global__ __launch_bounds__(kBaBlock) void k_ba_linearize(BaDev a) {
    const BaCtl& ctl = *a.ctl;
    if (ctl.done || !ctl.need_lin || ctl.gen != a.run_gen) return;
    const BaSys y = ba_sys(a, ctl.lin);
    const double* T = a.Tb[ctl.cur];
    const double* X = a.Xb[ctl.cur];
    double* part = a.part_lin;
    __shared__ double red[kBaBlock / 64];
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    double chi = 0;
    if (i < a.nedge) {
        const int pi = a.pose_idx[a.edges[i].kf];
        a.e_pi[i] = pi;  // for k_ba_update_errors (set by the first linearisation of optimize())
        const bool active = a.eflag[i] & 4;
        if (active) {
            edge_error(a, i, T, X, a.err + 3 * i);
            double r0, r1;
            edge_robust(a, i, edge_chi2(a, i), &r0, &r1);
            chi = r0;
        }
        edge_linearize(a, y, i, pi, active, T, X + 4 * a.edges[i].point);
    }
    chi = block_sum<kBaBlock>(chi, red);
    if (threadIdx.x == 0) part[blockIdx.x] = chi;
}

// blocks [0, nb_p): thread per point, Hll / b_l summed over its active edges in edge order;
// blocks [nb_p, nb_p + np): one per free pose, Hpp / b_p over its contiguous keyframe-CSR
// rows (thread = value x edge lane, fixed-order sum).  part_max = max |diag| per block
// (computeLambdaInit, optimization_algorithm_levenberg.cpp:166-180).
constexpr int kBaPoseLanes = kBaBlock / 27;  // 9
__global__ __launch_bounds__(kBaBlock) void k_ba_reduce(BaDev a) {
    const BaCtl& ctl = *a.ctl;
    if (ctl.done || !ctl.need_lin || ctl.gen != a.run_gen) return;
    ba_use(a, ctl.lin);
    const int nb_p = a.nb_p;
    double* part_max = a.part_max;
    __shared__ double red[kBaPoseLanes][27];
    __shared__ double redm[kBaBlock / 64];
    if ((int)blockIdx.x < nb_p) {
        const int p = blockIdx.x * blockDim.x + threadIdx.x;
        double m = 0;
        if (p < a.npt) {
            double h[6] = {0, 0, 0, 0, 0, 0}, b[3] = {0, 0, 0};
            for (int i = a.pt_start[p]; i < a.pt_start[p + 1]; i++) {
                if (!(a.eflag[i] & 4)) continue;
                const double* He = a.Hle + 9 * (long long)i;
                for (int k = 0; k < 6; k++) h[k] += He[k];
                for (int k = 0; k < 3; k++) b[k] += He[6 + k];
            }
            double* H = a.Hll + 9 * p;
            H[0] = h[0]; H[1] = h[1]; H[2] = h[2];
            H[3] = h[1]; H[4] = h[3]; H[5] = h[4];
            H[6] = h[2]; H[7] = h[4]; H[8] = h[5];
            for (int k = 0; k < 3; k++) a.bl[3 * p + k] = b[k];
            m = fmax(fabs(h[0]), fmax(fabs(h[3]), fabs(h[5])));
        }
        m = block_max<kBaBlock>(m, redm);
        if (threadIdx.x == 0) part_max[blockIdx.x] = m;
        return;
    }
    const int pi = blockIdx.x - nb_p;
    if (pi >= ctl.np) return;
    const int k = a.pose_kf[pi];
    const int q = threadIdx.x % 27, el = threadIdx.x / 27;
    if (el < kBaPoseLanes) {
        double v = 0;
        const double* base = a.Hpe + 27 * (long long)a.kf_start[k] + q;
        const int n = a.kf_start[k + 1] - a.kf_start[k];
        double v1 = 0, v2 = 0, v3 = 0;  // four loads in flight per lane
        int m = el;
        for (; m + 3 * kBaPoseLanes < n; m += 4 * kBaPoseLanes) {
            v += base[27 * (long long)m];
            v1 += base[27 * (long long)(m + kBaPoseLanes)];
            v2 += base[27 * (long long)(m + 2 * kBaPoseLanes)];
            v3 += base[27 * (long long)(m + 3 * kBaPoseLanes)];
        }
        for (; m < n; m += kBaPoseLanes) v += base[27 * (long long)m];
        red[el][q] = (v + v1) + (v2 + v3);
    }
    __syncthreads();
    if (threadIdx.x < 27) {
        double t = 0;
        for (int w = 0; w < kBaPoseLanes; w++) t += red[w][threadIdx.x];
        red[0][threadIdx.x] = t;  // row 0 is only re-read after the barrier below
        const int qq = threadIdx.x;
        if (qq < 21) {
            int r = 0, c = qq;
            while (c >= 6 - r) { c -= 6 - r; r++; }
            c += r;
            a.Hpp[36 * pi + r * 6 + c] = t;
            a.Hpp[36 * pi + c * 6 + r] = t;
        } else {
            a.bp[6 * pi + qq - 21] = t;
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) {  // diagonal of the packed upper 6x6: q = 0, 6, 11, 15, 18, 20
        double m = 0;
        const int dq[6] = {0, 6, 11, 15, 18, 20};
        for (int j = 0; j < 6; j++) m = fmax(m, fabs(red[0][dq[j]]));
        part_max[nb_p + pi] = m;
    }
}

// ---------------------------------------------------------------- Schur complement
// one block per pose pair (i < j): H_schur(i,j) = - sum_points B_i D^-1 B_j^T with D^-1
// recomputed per observation pair; one block per free keyframe i for the diagonal block
// [Hpp_i + lambda I] - sum_edges B D^-1 B^T and b_schur(i) = b_p - sum B D^-1 b_l (the (i, i)
// pair blocks return at once).  lam < 0: lambda = 1e-5 max|diag H| (every block reduces
// the same partials in the same order; block 0 publishes it in scal[3]).  512 threads (two
// waves per SIMD hide the dependent loads of a pair); the 36 block sums are reduced per wave
// by DPP / permlane reduce-scatter (wave_ops.h) and across waves in wave order.
constexpr int kSchurThreads = 512;
constexpr int kSchurWaves = kSchurThreads / 64;
constexpr int kSchurKfSplit = 2;  // blocks per free keyframe for its diagonal block and b_schur

// What block b of a k_ba_schur launch over nblk pose-pair blocks and nf free keyframes does
// (host and device: the CPU test orbmi_debug_ba_schur_blocks checks every index it leads to):
// b < nblk: pose-pair block b (blk_kf[2b], blk_kf[2b + 1], blk_start[b..b+1]); then kSchurKfSplit
// blocks per free keyframe r (free_kf[r], part_kf / arrive_kf[r]); then the MFMA padding block.
struct SchurRole {
    int kind;  // 0 pair block, 1 keyframe block, 2 MFMA padding, 3 past the launch
    int r, h;  // kind 1: free keyframe rank, half
};
__host__ __device__ inline SchurRole schur_role(int b, int nblk, int nf) {
    if (b < nblk) return SchurRole{0, b, 0};
    const int rb = b - nblk;
    if (rb < kSchurKfSplit * nf) return SchurRole{1, rb / kSchurKfSplit, rb % kSchurKfSplit};
    return SchurRole{rb == kSchurKfSplit * nf ? 2 : 3, 0, 0};
}

// sum over keyframe k's edges (keyframe-CSR rows of Hpe) of values [q0, q0 + NQ) of the 27,
// fixed order: thread t takes edges t, t + 512, ... (a config-3 keyframe has ~830: two per
// thread, every load of both in flight at once), then a per-wave reduce-scatter (DPP /
// permlane, wave_ops.h) and the waves' sums in wave order; tot[q] for q < NQ in LDS after the
// call (LDS scratch red, >= kSchurWaves x 32 doubles).  The diagonal blocks' Hpp sum was the
// Schur kernel's tail as value-per-lane loops (~35 dependent-batched loads per lane).
template <int NQ>
__device__ __attribute__((always_inline)) inline void pose_rows_sum(const BaDev& a, int k, int q0, double* red,
                                                                     double* tot) {
    static_assert(NQ <= 32, "one reduce-scatter");
    const int js = a.kf_start[k], n = a.kf_start[k + 1] - js;
    double v[32];
#pragma unroll
    for (int q = 0; q < 32; q++) v[q] = 0;
    for (int m0 = threadIdx.x; m0 < n; m0 += 2 * kSchurThreads) {
        double x[2][NQ];
#pragma unroll
        for (int u = 0; u < 2; u++) {
            const int m = min(m0 + u * kSchurThreads, n - 1);
            const double* rec = a.Hpe + 27 * (long long)(js + m) + q0;
#pragma unroll
            for (int q = 0; q < NQ; q++) x[u][q] = rec[q];
        }
#pragma unroll
        for (int u = 0; u < 2; u++)
            if (m0 + u * kSchurThreads < n) {
#pragma unroll
                for (int q = 0; q < NQ; q++) v[q] += x[u][q];
            }
    }
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const double r = wave_reduce_scatter32(v);  // lane l: value l >> 1 (even lanes)
    if (!(lane & 1) && (lane >> 1) < NQ) red[wid * 32 + (lane >> 1)] = r;
    __syncthreads();
    if ((int)threadIdx.x < NQ) {
        double t = 0;
        for (int w = 0; w < kSchurWaves; w++) t += red[w * 32 + threadIdx.x];
        tot[threadIdx.x] = t;
    }
    __syncthreads();
}

// (always_inline here and on pose_rows_sum: called from two kernels, the compiler otherwise
// outlines pose_rows_sum<21> into a function call with a 144-byte stack frame, and k_ba_schur
// went 16.5 -> 23.3 us)
__device__ __attribute__((always_inline)) inline void schur_body(BaDev a) {
    // the block's pair structure (static within an optimize()) is loaded before the LM state, so
    // that its two dependent loads overlap the control block's instead of following it
    const int b = blockIdx.x;
    int pka = 0, pkb = 0, pi1 = -1, pi2 = -1, pjs = 0, pje = 0, ppt = 0;
    int2 ppr = make_int2(0, 0);
    if (b < a.nblk) {
        pka = a.blk_kf[2 * b];
        pkb = a.blk_kf[2 * b + 1];
        pjs = a.blk_start[b];
        pje = a.blk_start[b + 1];
        pi1 = a.pose_idx[pka];
        pi2 = a.pose_idx[pkb];
        if (pjs + (int)threadIdx.x < pje) {
            ppr = a.blk_pairs[pjs + threadIdx.x];
            ppt = a.blk_pt[pjs + threadIdx.x];
        }
    }
    const BaCtl& ctl = *a.ctl;
    if (ctl.done || ctl.gen != a.run_gen) return;
    ba_use(a, ctl.lin);
    __shared__ double rows[kSchurThreads];
    const int N = 6 * ctl.np, nmax = a.nb_p + ctl.np;
    const double* part_max = a.part_max;
    // lambda: computeLambdaInit on the first trial of iteration 0, the LM state otherwise
    double lam = (ctl.it == 0 && ctl.trial == 0) ? -1.0 : ctl.lambda;
    __shared__ double red[kSchurWaves][36];
    __shared__ double lam_s;
    if (lam < 0) {
        if (threadIdx.x == 0) {
            double m = 0;
            for (int k = 0; k < nmax; k++) m = fmax(m, part_max[k]);
            lam_s = 1e-5 * m;
        }
        __syncthreads();
        lam = lam_s;
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) a.scal[3] = lam;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const SchurRole role = schur_role(blockIdx.x, a.nblk, a.nf);
    if (role.kind == 2) {  // the MFMA solve's padding: identity rows / columns
        // beyond N, zero columns 1..15 of the right-hand-side tiles.  Static within an optimize()
        // (N fixed, the solve only reads S): written on its first trial only
        if (!(ctl.it == 0 && ctl.trial == 0)) return;
        const int T = a.mfma_T, NT = T * (T + 3) / 2;
        for (int e = threadIdx.x; e < NT * 256; e += blockDim.x) {
            int t = e >> 8, i = 0;
            while (t >= T + 1 - i) { t -= T + 1 - i; i++; }
            const int j = i + t, rr = ((e >> 6) & 3) * 4 + ((e >> 4) & 3), cc = e & 15;
            const int R = 16 * i + rr, C = 16 * j + cc;
            if (j == T) {
                if (cc != 0 || R >= N) a.S[e] = 0.0;
            } else if (R >= N || C >= N) {
                a.S[e] = R == C ? 1.0 : 0.0;
            }
        }
        return;
    }
    if (role.kind == 1) {
        // blocks nblk + 2 r + h: half h of the r-th free keyframe's edges (CSR order) for its
        // diagonal block and b_schur: Hpp and b_p (the edges' Hpe rows), and per edge e of point l
        // with B = Hpl_e the diagonal pair product B D_l^-1 B^T and B D_l^-1 b_l -- the diagonal
        // pose pair's observation pairs are exactly the keyframe's edges, so the (i, i) pair
        // blocks return at once.  The two halves' 54 sums meet through sc1 partials and an
        // arrival counter (the second to arrive combines them in half order and writes)
        const int r = role.r, h = role.h;
        const int ka = a.free_kf[r];
        const int i1 = a.pose_idx[ka];
        if (i1 < 0) return;
        double vh[32], vp[32];
#pragma unroll
        for (int q = 0; q < 32; q++) vh[q] = vp[q] = 0;
        const int js = a.kf_start[ka], je = a.kf_start[ka + 1];
        for (int j = js + h * kSchurThreads + threadIdx.x; j < je; j += kSchurKfSplit * kSchurThreads) {
            const int e = a.kf_edges[j];
            const int p = a.kf_pt[j];
            const double* he = a.Hpe + 27 * (long long)j;  // keyframe-CSR rows
            double hx[27];
#pragma unroll
            for (int q = 0; q < 27; q++) hx[q] = he[q];
            double Di[9];
            point_dinv(a.Hll, p, lam, Di);
            const double* blp = a.bl + 3 * p;
            const double* B = a.Hpl + 18 * (long long)e;
            double bb[18], BD[18];
#pragma unroll
            for (int q = 0; q < 18; q++) bb[q] = B[q];
#pragma unroll
            for (int q = 0; q < 27; q++) vh[q] += hx[q];
#pragma unroll
            for (int rr = 0; rr < 6; rr++)
#pragma unroll
                for (int c = 0; c < 3; c++) BD[rr * 3 + c] = bb[rr * 3] * Di[c] + bb[rr * 3 + 1] * Di[3 + c] + bb[rr * 3 + 2] * Di[6 + c];
            int q = 0;
#pragma unroll
            for (int rr = 0; rr < 6; rr++)
#pragma unroll
                for (int c = rr; c < 6; c++, q++)
                    vp[q] += BD[rr * 3] * bb[c * 3] + BD[rr * 3 + 1] * bb[c * 3 + 1] + BD[rr * 3 + 2] * bb[c * 3 + 2];
#pragma unroll
            for (int rr = 0; rr < 6; rr++) vp[21 + rr] += BD[rr * 3] * blp[0] + BD[rr * 3 + 1] * blp[1] + BD[rr * 3 + 2] * blp[2];
        }
        {  // per wave: 27 + 27 sums by two reduce-scatters (lane l: value l >> 1), then across waves
            const double x = wave_reduce_scatter32(vh), y = wave_reduce_scatter32(vp);
            if (!(lane & 1) && (lane >> 1) < 27) {
                rows[wid * 64 + (lane >> 1)] = x;
                rows[wid * 64 + 32 + (lane >> 1)] = y;
            }
        }
        __syncthreads();
        if (wid != 0) return;
        double* part = a.part_kf + (size_t)(r * kSchurKfSplit + h) * 64;
        {  // this half's sums out as sc1 stores, drained, then the arrival (wave 0 only)
            double t = 0;
            for (int w = 0; w < kSchurWaves; w++) t += rows[w * 64 + lane];
            if ((lane & 31) < 27) __hip_atomic_store(part + lane, t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        int arrived = 0;
        if (lane == 0) arrived = (int)atomicAdd(&a.arrive_kf[r], 1u);
        arrived = __shfl(arrived, 0, 64);
        if (arrived != kSchurKfSplit - 1) return;
        if (lane == 0) a.arrive_kf[r] = 0;
        const int q = lane;
        if (q < 27) {
            double th = 0, tp = 0;  // halves in order
            for (int hh = 0; hh < kSchurKfSplit; hh++) {
                const double* ph = a.part_kf + (size_t)(r * kSchurKfSplit + hh) * 64;
                th += __hip_atomic_load(ph + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                tp += __hip_atomic_load(ph + 32 + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            if (q >= 21) {  // b_schur
                const int k = q - 21;
                a.bp[6 * i1 + k] = th;  // the solve's computeScale reads it
                a.bs[6 * i1 + k] = th - tp;
                if (a.mfma_T) a.S[mfma_tile_pos(a.mfma_T, 6 * i1 + k, 16 * a.mfma_T)] = th - tp;
            } else {  // diagonal block entry (rr, c), c >= rr: Hpp + lambda I - sum
                int rr = 0, c = q;
                while (c >= 6 - rr) { c -= 6 - rr; rr++; }
                c += rr;
                const double val = (th + (rr == c ? lam : 0.0)) - tp;
                const int R = 6 * i1 + rr, Cc = 6 * i1 + c;
                if (a.mfma_T) {  // the MFMA solve's tiles: diagonal tiles hold both triangles
                    a.S[mfma_tile_pos(a.mfma_T, R, Cc)] = val;
                    if ((R >> 4) == (Cc >> 4) && R != Cc) a.S[mfma_tile_pos(a.mfma_T, Cc, R)] = val;
                } else {
                    a.S[packed(R, Cc, N)] = val;
                }
            }
        }
        return;
    }
    const int ka = pka, kb = pkb;
    const int i1 = pi1, i2 = pi2;
    if (i1 < 0 || i2 < 0) return;
    const bool diag = ka == kb;
    if (diag) return;  // the keyframe's block nblk + r forms it (above)
    double acc[36];
#pragma unroll
    for (int q = 0; q < 36; q++) acc[q] = 0;
    for (int j = pjs + threadIdx.x; j < pje; j += blockDim.x) {
        const bool first = j == pjs + (int)threadIdx.x;  // the prefetched pair
        const int2 pr = first ? ppr : a.blk_pairs[j];  // inactive edges carry a zero Hpl block
        double Di[9];
        point_dinv(a.Hll, first ? ppt : a.blk_pt[j], lam, Di);
        const double* B1 = a.Hpl + 18 * (long long)pr.x;
        const double* B2 = a.Hpl + 18 * (long long)pr.y;
        double BD[18];
#pragma unroll
        for (int r = 0; r < 6; r++)
#pragma unroll
            for (int c = 0; c < 3; c++) BD[r * 3 + c] = B1[r * 3] * Di[c] + B1[r * 3 + 1] * Di[3 + c] + B1[r * 3 + 2] * Di[6 + c];
        double b2[18];
#pragma unroll
        for (int q = 0; q < 18; q++) b2[q] = B2[q];
#pragma unroll
        for (int r = 0; r < 6; r++)
#pragma unroll
            for (int c = 0; c < 6; c++)
                acc[r * 6 + c] += BD[r * 3] * b2[c * 3] + BD[r * 3 + 1] * b2[c * 3 + 1] + BD[r * 3 + 2] * b2[c * 3 + 2];
    }
    {  // values 0..31: reduce-scatter (lane l holds value l >> 1); 32..35: all-reduce
        double v[32];
#pragma unroll
        for (int q = 0; q < 32; q++) v[q] = acc[q];
        const double s = wave_reduce_scatter32(v);
        if (!(lane & 1)) red[wid][lane >> 1] = s;
#pragma unroll
        for (int q = 32; q < 36; q++) {
            const double x = wave_sum(acc[q]);
            if (lane == 0) red[wid][q] = x;
        }
    }
    __syncthreads();
    const int q = threadIdx.x;
    if (q < 36) {
        double t = 0;
        for (int w = 0; w < kSchurWaves; w++) t += red[w][q];
        const int r = q / 6, c = q % 6;  // an off-diagonal pose pair: -sum
        if (a.mfma_T) {  // the MFMA solve's tiles: diagonal tiles hold both triangles
            const int R = 6 * i1 + r, Cc = 6 * i2 + c;
            a.S[mfma_tile_pos(a.mfma_T, R, Cc)] = -t;
            if ((R >> 4) == (Cc >> 4)) a.S[mfma_tile_pos(a.mfma_T, Cc, R)] = -t;
        } else {
            a.S[packed(6 * i1 + r, 6 * i2 + c, N)] = -t;
        }
    }
}

__global__ __launch_bounds__(kSchurThreads) void k_ba_schur(BaDev a) { schur_body(a); }

// ---------------------------------------------------------------- reduced system solve
// Block Gauss-Jordan on the LDL^T = U^T D U factorisation of the reduced camera system,
// blocked by the 6x6 pose blocks and held in registers: TPT threads own tile (i, j), i <= j, of
// the upper triangle, or block i of the right-hand side carried as an extra tile column.  Block
// step k has two phases and two barriers:
//   B(k)  owners of (k, j > k) form W = U_kk^-T A_kj, U_kj = D_k^-1 W and the normalised pivot
//         row R_kj = U_kk^-1 U_kj (= A_kk^-1 A_kj) and publish W, U, R (LDS); the right-hand
//         side tile gives y_k = D_k^-1 U_kk^-T z_k and r_k = U_kk^-1 y_k.  Owners of the
//         column-k tiles above the pivot, (i < k, k), publish M_ik and drop the tile.
//   A(k)  rows below the pivot (i > k): A_ij -= W_ki^T U_kj (the LDL^T trailing update; the
//         owner of (k+1, k+1) then factors its tile at once, lookahead); rows above (i < k),
//         already normalised: M_ij -= M_ik R_kj, right-hand side r_i -= M_ik r_k.
// After the last step the right-hand side column holds x: no back substitution.  Same solution
// as LinearSolverEigen's SimplicialLDLT up to the rounding order.
constexpr int kBaSolveThreads = 512;  // >= TPT x tiles: 2 x (231 + 21) at np <= 21, 465 + 30 at np <= 30
#ifdef ORBMI_SOLVE_TRACE  // tools/solve_trace.hip: s_memtime stamps kept in LDS, copied out at the end
__device__ unsigned long long g_solve_trace[256];
#define SOLVE_STAMP_DECL __shared__ unsigned long long tstamp[256]
#define SOLVE_STAMP(cond, i)                                                                 \
    do {                                                                                     \
        if (cond) tstamp[i] = __builtin_amdgcn_s_memtime();                                  \
    } while (0)
#define SOLVE_STAMP_FLUSH()                                                                  \
    do {                                                                                     \
        if (threadIdx.x == 0)                                                                \
            for (int i_ = 0; i_ < 256; i_++) g_solve_trace[i_] = tstamp[i_];                 \
    } while (0)
#define SOLVE_STAMP_TO(ts, cond, i)                                                          \
    do {                                                                                     \
        if (cond) (ts)[i] = __builtin_amdgcn_s_memtime();                                    \
    } while (0)
#define SOLVE_STAMP_PTR tstamp
#else
#define SOLVE_STAMP_DECL
#define SOLVE_STAMP(cond, i) do {} while (0)
#define SOLVE_STAMP_FLUSH() do {} while (0)
#define SOLVE_STAMP_TO(ts, cond, i) do {} while (0)
#define SOLVE_STAMP_PTR nullptr
#endif

__device__ inline void wave_sync_lds() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// value of the neighbouring lane (lane ^ 1) through DPP quad_perm [1,0,3,2] (no LDS round trip)
__device__ inline double dpp_xor1(double v) {
    const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), 0xB1, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), 0xB1, 0xF, 0xF, false);
    return __hiloint2double(hi, lo);
}

// 1 / d: v_rcp_f64 and two Newton steps (the pivots of the reduced system)
__device__ inline double rcp_f64(double d) {
    double r = __builtin_amdgcn_rcp(d);
    double e = fma(-d, r, 1.0);
    r = fma(r, e, r);
    e = fma(-d, r, 1.0);
    return fma(r, e, r);
}

// LDL^T of a 6x6 tile (full row-major, upper triangle used): on return F[j][c] = U_jc (c > j),
// F[j][j] = d_j, inv6 = 1 / d.  False on a zero or non-finite pivot.
__device__ inline bool ldl6(double F[36], double inv6[6]) {
    bool bad = false;
#pragma unroll
    for (int j = 0; j < 6; j++) {
        const double d = F[j * 7];
        bad |= !(fabs(d) > 0) || !isfinite(d);
        const double inv = rcp_f64(d);
        inv6[j] = inv;
#pragma unroll
        for (int c = j + 1; c < 6; c++) {
            const double u = F[j * 6 + c] * inv;  // u_jc
#pragma unroll
            for (int r = j + 1; r <= c; r++) F[r * 6 + c] -= F[j * 6 + r] * u;
        }
#pragma unroll
        for (int c = j + 1; c < 6; c++) F[j * 6 + c] *= inv;
    }
    return !bad;
}

template <int TPT>  // threads per tile: 2 (np <= 21) or 1 (np <= kBaMaxPoses)
__global__ __launch_bounds__(kBaSolveThreads) void k_ba_solve(BaDev a) {
    const BaCtl& ctl = *a.ctl;
    if (ctl.done || ctl.gen != a.run_gen) return;
    const int np = ctl.np;
    double lam = a.scal[3];
    const double* __restrict__ T = a.Tb[ctl.cur];
    double* __restrict__ Tt = a.Tb[ctl.cur ^ 1];
    constexpr int CPT = 6 / TPT;  // tile columns per thread
    SOLVE_STAMP_DECL;
    SOLVE_STAMP(threadIdx.x == 0, 250);
    constexpr int kSlot = 37;  // odd stride in doubles: conflict-free LDS rows
    __shared__ double Wp[(kBaMaxPoses + 1) * kSlot], Up[(kBaMaxPoses + 1) * kSlot], Rp[(kBaMaxPoses + 1) * kSlot];
    __shared__ double Mp[kBaMaxPoses * kSlot];
    __shared__ double Ud[36], Dinv6[6];
    __shared__ double bs[kBaMaxN];
    __shared__ int fail;
    const int N = 6 * np, nblk = np * (np + 1) / 2;
    const int tid = threadIdx.x;
    // TPT adjacent threads -> tile (bi, bj) of the upper triangle, or (bi, np) = block bi of
    // the right-hand side.  Thread h of the tile owns its columns CPT h .. CPT h + CPT - 1.
    const int tile = tid / TPT, h = tid % TPT, c0 = CPT * h;
    const bool own = tile < nblk + np;
    const bool rhs = own && tile >= nblk;
    int bi = 0, bj = 0;
    if (rhs) {
        bi = tile - nblk;
        bj = np;
    } else if (own) {
        int t = tile;
        while (t >= np - bi) { t -= np - bi; bi++; }
        bj = bi + t;
    }
    const bool dg = !rhs && bi == bj;
    double A[6 * CPT];  // A[r * CPT + cc] = element (r, c0 + cc) of the tile
    // branch-free loads (clamped addresses, then a select) so that all of them are in flight
#pragma unroll
    for (int q = 0; q < 6 * CPT; q++) {
        const int r = q / CPT, c = c0 + q % CPT;
        const bool mat = own && !rhs && (!dg || c >= r), vec = rhs && c == 0;
        const double* src = vec ? a.bs + 6 * bi + r : a.S + (mat ? packed(6 * bi + r, 6 * bj + c, N) : 0);
        const double v = *src;
        A[q] = (mat || vec) ? v : 0.0;
    }
    if (tid == 0) fail = 0;
    // the owner of a diagonal tile factors it and publishes U_kk, 1 / D_k
    auto factor_diag = [&]() {
        double F[36];
        if constexpr (TPT == 2) {
#pragma unroll
            for (int q = 0; q < 18; q++) {
                const double o = dpp_xor1(A[q]);
                const int r = q / 3, cc = q % 3;
                F[r * 6 + cc] = h == 0 ? A[q] : o;
                F[r * 6 + 3 + cc] = h == 0 ? o : A[q];
            }
        } else {
#pragma unroll
            for (int q = 0; q < 36; q++) F[q] = A[q];
        }
        double inv6[6];
        const bool ok = ldl6(F, inv6);
        if (h == 0) {
#pragma unroll
            for (int q = 0; q < 36; q++) Ud[q] = F[q];
#pragma unroll
            for (int j = 0; j < 6; j++) Dinv6[j] = inv6[j];
            if (!ok) fail = 1;
        }
    };
    __syncthreads();
    if (own && dg && bi == 0) factor_diag();
    __syncthreads();
    SOLVE_STAMP(tid == 0, 251);
    for (int k = 0; k < np; k++) {
        if (fail) break;
        // ---- B(k): pivot row k; column k above the pivot
        if (own && bi == k && bj > k) {
            double ud[6][6];  // strict upper of U_kk (static indices only)
#pragma unroll
            for (int t = 0; t < 6; t++)
#pragma unroll
                for (int s2 = t + 1; s2 < 6; s2++) ud[t][s2] = Ud[t * 6 + s2];
#pragma unroll
            for (int cc = 0; cc < CPT; cc++)  // W = U_kk^-T A (unit lower solve)
#pragma unroll
                for (int t = 1; t < 6; t++)
#pragma unroll
                    for (int s2 = 0; s2 < t; s2++) A[t * CPT + cc] -= ud[s2][t] * A[s2 * CPT + cc];
#pragma unroll
            for (int q = 0; q < 6 * CPT; q++) {
                const int r = q / CPT, c = c0 + q % CPT;
                Wp[bj * kSlot + r * 6 + c] = A[q];
                A[q] *= Dinv6[r];
                Up[bj * kSlot + r * 6 + c] = A[q];
            }
#pragma unroll
            for (int cc = 0; cc < CPT; cc++)  // R = U_kk^-1 U (unit upper solve, bottom up)
#pragma unroll
                for (int t = 4; t >= 0; t--)
#pragma unroll
                    for (int s2 = t + 1; s2 < 6; s2++) A[t * CPT + cc] -= ud[t][s2] * A[s2 * CPT + cc];
#pragma unroll
            for (int q = 0; q < 6 * CPT; q++) Rp[bj * kSlot + (q / CPT) * 6 + c0 + q % CPT] = A[q];
            SOLVE_STAMP(bj == k + 1 && h == 0, 4 * k);
        }
        if (own && !rhs && bj == k && bi < k) {  // M_ik, stored transposed like W_ki
#pragma unroll
            for (int q = 0; q < 6 * CPT; q++) Mp[bi * kSlot + (c0 + q % CPT) * 6 + q / CPT] = A[q];
        }
        __syncthreads();
        // ---- A(k): eliminate column k from every other row
        if (own && bj > k && bi != k) {
            // A -= L^T P with L(t, r) = W_ki(t, r) below the pivot or M_ik(r, t) above it, and P =
            // U_kj or R_kj: 6 CPT independent accumulation chains (the unused lower part of a
            // diagonal tile and the zero columns of a right-hand-side tile stay harmless)
            const bool below = bi > k;
            const double* Pp = below ? Up : Rp;
            const double* Lp = below ? Wp : Mp;
            double u[6 * CPT], w[36];
#pragma unroll
            for (int q = 0; q < 6 * CPT; q++) u[q] = Pp[bj * kSlot + (q / CPT) * 6 + c0 + q % CPT];
#pragma unroll
            for (int q = 0; q < 36; q++) w[q] = Lp[bi * kSlot + q];  // w[t * 6 + r] = L(t, r)
#pragma unroll
            for (int t = 0; t < 6; t++)
#pragma unroll
                for (int r = 0; r < 6; r++)
#pragma unroll
                    for (int cc = 0; cc < CPT; cc++) A[r * CPT + cc] -= w[t * 6 + r] * u[t * CPT + cc];
            SOLVE_STAMP(dg && bi == k + 1 && h == 0, 4 * k + 1);
            if (dg && bi == k + 1) factor_diag();
            SOLVE_STAMP(dg && bi == k + 1 && h == 0, 4 * k + 2);
        }
        __syncthreads();
        SOLVE_STAMP(tid == 0, 4 * k + 3);
    }
    if (fail) {  // pop: trial poses = current ones, computeScale = 0
        for (int k = tid; k < a.nkf; k += blockDim.x)
            for (int q = 0; q < 8; q++) Tt[8 * k + q] = T[8 * k + q];
        if (tid == 0) { a.istat[3] = 0; a.scal[1] = 0; a.scal[2] = 0; }
        return;
    }
    if (rhs && h == 0) {  // x = the right-hand side column
#pragma unroll
        for (int r = 0; r < 6; r++) {
            bs[6 * bi + r] = A[r * CPT];
            a.xp[6 * bi + r] = A[r * CPT];
        }
    }
    __syncthreads();
    if (tid >= 64) return;
    const int lane = tid;
    SOLVE_STAMP(lane == 0, 252);
    // trial poses T_t = exp(x_p) * T (VertexSE3Expmap::oplusImpl) and the poses' part of
    // computeScale, sum x_p (lambda x_p + b_p) in index order
    for (int k = lane; k < a.nkf; k += 64) {
        const int pi = a.pose_idx[k];
        if (pi >= 0) {
            double u[6];
#pragma unroll
            for (int q = 0; q < 6; q++) u[q] = bs[6 * pi + q];
            se3_oplus(u, T + 8 * k, Tt + 8 * k);
        } else {
            for (int q = 0; q < 8; q++) Tt[8 * k + q] = T[8 * k + q];
        }
    }
    if (lane == 0) {
        double sc = 0;
        for (int q = 0; q < N; q++) sc += bs[q] * (lam * bs[q] + a.bp[q]);
        a.scal[1] = sc;
        a.scal[2] = 1;
        a.istat[3] = 1;
    }
    SOLVE_STAMP(lane == 0, 253);
    SOLVE_STAMP_FLUSH();
}

// The same elimination with the tiles laid out by row pairs, 3 threads per tile (2 tile columns
// each) and 1 thread per right-hand-side block: wave 0 owns tile row 0, wave w >= 1 rows w and
// np - w (3 np + 2 <= 64 lanes), so a pivot row, its diagonal tile and its right-hand side sit in
// one wave.  The pivot row publishes its tiles as they are (A_kj) and normalised (R_kj =
// A_kk^-1 A_kj, through the LDL^T of A_kk); since W_ki^T U_kj = A_ki^T A_kk^-1 A_kj, every other
// row then applies the same update A_ij -= L^T R_kj with L = A_ki below the pivot and M_ik above.
// Step k is one phase and one barrier: every tile applies pivot k; the wave of row k + 1 then
// publishes its updated diagonal tile, every lane of that wave factors it redundantly (no
// broadcast of the factor) and the row forms pivot row k + 1, synchronised within the wave only,
// at raised issue priority; the owners of column k + 1 above the pivot publish M.  The pivot-row
// and M buffers alternate by parity of k (the readers of step k and the writers for step k + 1
// overlap).  np <= kBaSolveRowsMaxPoses; larger systems use k_ba_solve<1>.
constexpr int kBaSolveRowsMaxPoses = 20;
constexpr int kBaSolveRowsThreads = 64 * (1 + kBaSolveRowsMaxPoses / 2);
static_assert(3 * kBaSolveRowsMaxPoses + 2 <= 64, "a row pair must fit one wave");
__device__ inline int solve_rows_wave(int row, int np) { return row <= np - row ? row : np - row; }
__global__ __launch_bounds__(kBaSolveRowsThreads) void k_ba_solve_rows(BaDev a) {
    const BaCtl& ctl = *a.ctl;
    if (ctl.done || ctl.gen != a.run_gen) return;
    const int np = ctl.np;
    double lam = a.scal[3];
    const double* __restrict__ T = a.Tb[ctl.cur];
    double* __restrict__ Tt = a.Tb[ctl.cur ^ 1];
    constexpr int CPT = 2;
    constexpr int kSlot = 38;  // doubles; 16-B aligned rows for b128 access
    constexpr int kRowSlots = kBaSolveRowsMaxPoses + 1;
    SOLVE_STAMP_DECL;
    SOLVE_STAMP(threadIdx.x == 0, 250);
    __shared__ __attribute__((aligned(16))) double Ap[2][kRowSlots * kSlot], Rp[2][kRowSlots * kSlot];
    __shared__ __attribute__((aligned(16))) double Mp[2][kBaSolveRowsMaxPoses * kSlot];
    __shared__ double bs[6 * kBaSolveRowsMaxPoses];
    __shared__ int fail;
    const int N = 6 * np;
    const int tid = threadIdx.x;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
    // lane -> (bi, bj, h); bj = np is the right-hand side (h = 0 only)
    const int ra = wv, rb = np - wv;  // rows of this wave (rb only for wv >= 1, rb > ra)
    const int na = 3 * (np - ra) + 1;
    int bi = -1, bj = 0, h = 0;
    if (ra < np && (wv == 0 || ra <= rb)) {
        int l = lane, r = ra;
        if (l >= na && wv > 0 && rb > ra) { l -= na; r = rb; }
        if (l < 3 * (np - r) + 1) {
            bi = r;
            bj = l < 3 * (np - r) ? r + l / 3 : np;
            h = l < 3 * (np - r) ? l % 3 : 0;
        }
    }
    const int c0 = CPT * h;
    const bool own = bi >= 0;
    const bool rhs = own && bj == np;
    const bool dg = own && !rhs && bi == bj;
    double A[6 * CPT];  // A[r * CPT + cc] = element (r, c0 + cc) of the tile
#pragma unroll
    for (int q = 0; q < 6 * CPT; q++) {
        const int r = q / CPT, c = c0 + q % CPT;
        const bool mat = own && !rhs && (!dg || c >= r), vec = rhs && c == 0;
        const double* src = vec ? a.bs + 6 * bi + r : a.S + (mat ? packed(6 * bi + r, 6 * bj + c, N) : 0);
        const double v = *src;
        A[q] = (mat || vec) ? v : 0.0;
    }
    if (tid == 0) fail = 0;
    // pivot row k: the diagonal tile's owners publish it, every lane of the wave factors it, then
    // tiles (k, j > k) and the right-hand side publish A_kj and R_kj into buffer k & 1
    auto pivot_row = [&](int k) {
        // the diagonal tile from its three owner lanes (lane base + h holds columns 2h, 2h + 1)
        // by readlane: no LDS round trip on the elimination's critical path
        const int base = __builtin_amdgcn_readfirstlane(k == ra ? 0 : na);
        double F[36], inv6[6];
#pragma unroll
        for (int r = 0; r < 6; r++)
#pragma unroll
            for (int c = r; c < 6; c++) F[r * 6 + c] = readlane_d(A[r * CPT + c % 2], base + c / 2);
        const bool ok = ldl6(F, inv6);
        if (dg && bi == k && h == 0 && !ok) fail = 1;
        if (!(own && bi == k && bj > k)) return;
        double* __restrict__ Ao = Ap[k & 1];
        double* __restrict__ R = Rp[k & 1];
#pragma unroll
        for (int q = 0; q < 6 * CPT; q++) Ao[bj * kSlot + (q / CPT) * 6 + c0 + q % CPT] = A[q];
#pragma unroll
        for (int cc = 0; cc < CPT; cc++)  // U_kk^-T A (unit lower solve)
#pragma unroll
            for (int t = 1; t < 6; t++)
#pragma unroll
                for (int s2 = 0; s2 < t; s2++) A[t * CPT + cc] -= F[s2 * 6 + t] * A[s2 * CPT + cc];
#pragma unroll
        for (int q = 0; q < 6 * CPT; q++) A[q] *= inv6[q / CPT];  // D^-1
#pragma unroll
        for (int cc = 0; cc < CPT; cc++)  // R = U_kk^-1 (unit upper solve, bottom up)
#pragma unroll
            for (int t = 4; t >= 0; t--)
#pragma unroll
                for (int s2 = t + 1; s2 < 6; s2++) A[t * CPT + cc] -= F[t * 6 + s2] * A[s2 * CPT + cc];
#pragma unroll
        for (int q = 0; q < 6 * CPT; q++) R[bj * kSlot + (q / CPT) * 6 + c0 + q % CPT] = A[q];
    };
    __syncthreads();
    if (wv == 0) pivot_row(0);  // prologue: pivot row 0
    __syncthreads();
    SOLVE_STAMP(tid == 0, 251);
    // a failed pivot (fail) is acted on after the loop: the remaining steps then only carry
    // non-finite values, and no step waits on an LDS read of the flag
    for (int k = 0; k < np; k++) {
        const bool crit = k + 1 < np && wv == solve_rows_wave(k + 1, np);  // wave-uniform
        if (crit) __builtin_amdgcn_s_setprio(3);
        // ---- A(k): eliminate column k from every other row
        if (own && bj > k && bi != k) {
            const double* Lp = bi > k ? Ap[k & 1] : Mp[k & 1];
            double u[6 * CPT], w[36];
#pragma unroll
            for (int q = 0; q < 6 * CPT; q++) u[q] = Rp[k & 1][bj * kSlot + (q / CPT) * 6 + c0 + q % CPT];
#pragma unroll
            for (int q = 0; q < 36; q++) w[q] = Lp[bi * kSlot + q];  // w[t * 6 + r] = L(t, r)
            __builtin_amdgcn_sched_barrier(0);  // all 24 LDS reads in flight before the first FMA
#pragma unroll
            for (int t = 0; t < 6; t++)
#pragma unroll
                for (int r = 0; r < 6; r++)
#pragma unroll
                    for (int cc = 0; cc < CPT; cc++) A[r * CPT + cc] -= w[t * 6 + r] * u[t * CPT + cc];
        }
        if (k + 1 < np) {
            // M_i,k+1 (column k + 1 above its pivot, final after A(k)), stored transposed
            if (own && !rhs && bj == k + 1 && bi <= k) {
#pragma unroll
                for (int q = 0; q < 6 * CPT; q++) Mp[(k + 1) & 1][bi * kSlot + (c0 + q % CPT) * 6 + q / CPT] = A[q];
            }
            if (crit) {
                SOLVE_STAMP(dg && bi == k + 1 && h == 0, 4 * k);
                pivot_row(k + 1);
                SOLVE_STAMP(own && bi == k + 1 && rhs, 4 * k + 2);
                __builtin_amdgcn_s_setprio(0);
            }
        }
        __syncthreads();
        SOLVE_STAMP(tid == 0, 4 * k + 3);
    }
    if (fail) {  // pop: trial poses = current ones, computeScale = 0
        for (int k = tid; k < a.nkf; k += blockDim.x)
            for (int q = 0; q < 8; q++) Tt[8 * k + q] = T[8 * k + q];
        if (tid == 0) { a.istat[3] = 0; a.scal[1] = 0; a.scal[2] = 0; }
        return;
    }
    if (rhs) {  // x = the right-hand side column
#pragma unroll
        for (int r = 0; r < 6; r++) {
            bs[6 * bi + r] = A[r * CPT];
            a.xp[6 * bi + r] = A[r * CPT];
        }
    }
    __syncthreads();
    if (tid >= 64) return;
    SOLVE_STAMP(lane == 0, 252);
    // trial poses T_t = exp(x_p) * T (VertexSE3Expmap::oplusImpl) and the poses' part of
    // computeScale, sum x_p (lambda x_p + b_p) in index order
    for (int k = lane; k < a.nkf; k += 64) {
        const int pi = a.pose_idx[k];
        if (pi >= 0) {
            double u[6];
#pragma unroll
            for (int q = 0; q < 6; q++) u[q] = bs[6 * pi + q];
            se3_oplus(u, T + 8 * k, Tt + 8 * k);
        } else {
            for (int q = 0; q < 8; q++) Tt[8 * k + q] = T[8 * k + q];
        }
    }
    double sc = 0;  // lane partials in index order, then a fixed-order wave sum
    for (int q = lane; q < N; q += 64) sc += bs[q] * (lam * bs[q] + a.bp[q]);
    sc = wave_sum(sc);
    if (lane == 0) {
        a.scal[1] = sc;
        a.scal[2] = 1;
        a.istat[3] = 1;
    }
    SOLVE_STAMP(lane == 0, 253);
    SOLVE_STAMP_FLUSH();
}

// k_ba_solve_rows' elimination with the pivot rows formed by a dedicated wave P (the last one),
// so that the chain from pivot row k to pivot row k + 1 holds no LDS round trip of the update and
// no wave switch.  P's lanes are column slices (lane 3 j + h: tile column j, columns 2h, 2h + 1;
// lane 3 np: the right-hand side) and hold, during step k, row k + 1:
//   step k, P:    A_{k+1,j} -= A_{k,k+1}^T R_{k,j} with R_k kept in P's registers from step k - 1
//                 and A_{k,k+1} read back from the pivot-row buffer P wrote; then the LDL^T of the
//                 updated diagonal tile (readlane) and pivot row k + 1 (A and R) into buffer
//                 (k + 1) & 1; row k + 2 arrives from its owner through LDS at the start of step
//                 k + 1 (its owner writes it during step k, after applying pivot k).
//   step k, bulk: the owners of row k load R_k (the pivot row, now normalised) into their
//                 registers; every other row except k + 1 (P's) applies pivot k as before.
// One barrier per step.  np <= kBaSolveRowsMaxPoses.
constexpr int kBaSolvePipeThreads = kBaSolveRowsThreads + 64;
__global__ __launch_bounds__(kBaSolvePipeThreads) void k_ba_solve_pipe(BaDev a) {
    const BaCtl& ctl = *a.ctl;
    if (ctl.done || ctl.gen != a.run_gen) return;
    const int np = ctl.np;
    double lam = a.scal[3];
    const double* __restrict__ T = a.Tb[ctl.cur];
    double* __restrict__ Tt = a.Tb[ctl.cur ^ 1];
    constexpr int CPT = 2;
    constexpr int kSlot = 38;
    constexpr int kRowSlots = kBaSolveRowsMaxPoses + 1;
    constexpr int kPivotWave = kBaSolveRowsThreads / 64;
    SOLVE_STAMP_DECL;
    SOLVE_STAMP(threadIdx.x == 0, 250);
    __shared__ __attribute__((aligned(16))) double Ap[2][kRowSlots * kSlot], Rp[2][kRowSlots * kSlot];
    __shared__ __attribute__((aligned(16))) double Nx[2][kRowSlots * kSlot];  // row k + 2 for P
    __shared__ __attribute__((aligned(16))) double Mp[2][kBaSolveRowsMaxPoses * kSlot];
    __shared__ double bs[6 * kBaSolveRowsMaxPoses];
    __shared__ int fail;
    const int N = 6 * np;
    const int tid = threadIdx.x;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
    const bool P = wv == kPivotWave;
    // bulk lanes: the row-pair layout of k_ba_solve_rows; P lanes: column slices
    int bi = -1, bj = 0, h = 0;
    const int ra = wv, rb = np - wv, na = 3 * (np - ra) + 1;
    if (P) {
        if (lane <= 3 * np) {
            bj = lane < 3 * np ? lane / 3 : np;
            h = lane < 3 * np ? lane % 3 : 0;
        }
    } else if (ra < np && (wv == 0 || ra <= rb)) {
        int l = lane, r = ra;
        if (l >= na && wv > 0 && rb > ra) { l -= na; r = rb; }
        if (l < 3 * (np - r) + 1) {
            bi = r;
            bj = l < 3 * (np - r) ? r + l / 3 : np;
            h = l < 3 * (np - r) ? l % 3 : 0;
        }
    }
    const int c0 = CPT * h;
    const bool own = bi >= 0;
    const bool rhs = bj == np;
    const bool plane = P && lane <= 3 * np;  // a P lane with a column slice
    // element (r, c0 + cc) of tile (row, bj) from the packed system (upper part of a diagonal tile)
    auto load_tile = [&](int row, double* A) {
        const bool dg = !rhs && row == bj;
#pragma unroll
        for (int q = 0; q < 6 * CPT; q++) {
            const int r = q / CPT, c = c0 + q % CPT;
            const bool mat = !rhs && bj >= row && (!dg || c >= r), vec = rhs && c == 0;
            const double* src = vec ? a.bs + 6 * row + r : a.S + (mat ? packed(6 * row + r, 6 * bj + c, N) : 0);
            const double v = *src;
            A[q] = (mat || vec) ? v : 0.0;
        }
    };
    double A[6 * CPT];   // bulk: its tile slice; P: row k + 1's slice
    double Rk[6 * CPT];  // P: R_{k,bj} slice (pivot row k, normalised)
#pragma unroll
    for (int q = 0; q < 6 * CPT; q++) { A[q] = 0.0; Rk[q] = 0.0; }
    if (own) load_tile(bi, A);
    if (tid == 0) fail = 0;
    // P: factor the diagonal tile of the row it holds (row k), publish A_k and R_k into buffer
    // k & 1, keep R_k in Rk
    auto pivot = [&](int k) {
        const int base = 3 * k;
        double F[36], inv6[6];
#pragma unroll
        for (int r = 0; r < 6; r++)
#pragma unroll
            for (int c = r; c < 6; c++) F[r * 6 + c] = readlane_d(A[r * CPT + c % 2], base + c / 2);
        const bool ok = ldl6(F, inv6);
        if (lane == 0 && !ok) fail = 1;
        double R[6 * CPT];
#pragma unroll
        for (int q = 0; q < 6 * CPT; q++) R[q] = A[q];
#pragma unroll
        for (int cc = 0; cc < CPT; cc++)
#pragma unroll
            for (int t = 1; t < 6; t++)
#pragma unroll
                for (int s2 = 0; s2 < t; s2++) R[t * CPT + cc] -= F[s2 * 6 + t] * R[s2 * CPT + cc];
#pragma unroll
        for (int q = 0; q < 6 * CPT; q++) R[q] *= inv6[q / CPT];
#pragma unroll
        for (int cc = 0; cc < CPT; cc++)
#pragma unroll
            for (int t = 4; t >= 0; t--)
#pragma unroll
                for (int s2 = t + 1; s2 < 6; s2++) R[t * CPT + cc] -= F[t * 6 + s2] * R[s2 * CPT + cc];
        if (plane && bj > k) {
            double* __restrict__ Ao = Ap[k & 1];
            double* __restrict__ Ro = Rp[k & 1];
#pragma unroll
            for (int q = 0; q < 6 * CPT; q++) {
                Ao[bj * kSlot + (q / CPT) * 6 + c0 + q % CPT] = A[q];
                Ro[bj * kSlot + (q / CPT) * 6 + c0 + q % CPT] = R[q];
            }
        }
#pragma unroll
        for (int q = 0; q < 6 * CPT; q++) Rk[q] = R[q];
    };
    __syncthreads();
    if (P && np > 0) {  // prologue: row 0 -> pivot row 0; row 1 stays in A for step 0
        __builtin_amdgcn_s_setprio(3);
        if (plane) load_tile(0, A);
        pivot(0);
        if (np > 1 && plane) load_tile(1, A);
    }
    __syncthreads();
    SOLVE_STAMP(tid == 0, 251);
    for (int k = 0; k < np; k++) {
        if (P) {
            if (k + 1 < np) {
                if (k >= 1 && plane) {  // row k + 1 with pivots < k applied, from its owner
#pragma unroll
                    for (int q = 0; q < 6 * CPT; q++) A[q] = Nx[(k - 1) & 1][bj * kSlot + (q / CPT) * 6 + c0 + q % CPT];
                }
                double w[36];  // L = A_{k,k+1} (w[t * 6 + r] = L(t, r)), as P published it
#pragma unroll
                for (int q = 0; q < 36; q++) w[q] = Ap[k & 1][(k + 1) * kSlot + q];
                __builtin_amdgcn_sched_barrier(0);
                if (plane && bj > k) {
#pragma unroll
                    for (int t = 0; t < 6; t++)
#pragma unroll
                        for (int r = 0; r < 6; r++)
#pragma unroll
                            for (int cc = 0; cc < CPT; cc++) A[r * CPT + cc] -= w[t * 6 + r] * Rk[t * CPT + cc];
                }
                SOLVE_STAMP(lane == 0, 4 * k);
                pivot(k + 1);
                SOLVE_STAMP(lane == 0, 4 * k + 2);
            }
        } else if (own) {
            if (bi == k) {  // pivot row k: its normalised tiles
                if (bj > k) {
#pragma unroll
                    for (int q = 0; q < 6 * CPT; q++) A[q] = Rp[k & 1][bj * kSlot + (q / CPT) * 6 + c0 + q % CPT];
                }
            } else if (bj > k && bi != k + 1) {
                const double* Lp = bi > k ? Ap[k & 1] : Mp[k & 1];
                double u[6 * CPT], w[36];
#pragma unroll
                for (int q = 0; q < 6 * CPT; q++) u[q] = Rp[k & 1][bj * kSlot + (q / CPT) * 6 + c0 + q % CPT];
#pragma unroll
                for (int q = 0; q < 36; q++) w[q] = Lp[bi * kSlot + q];
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int t = 0; t < 6; t++)
#pragma unroll
                    for (int r = 0; r < 6; r++)
#pragma unroll
                        for (int cc = 0; cc < CPT; cc++) A[r * CPT + cc] -= w[t * 6 + r] * u[t * CPT + cc];
                if (bi == k + 2) {  // P's row at step k + 1
#pragma unroll
                    for (int q = 0; q < 6 * CPT; q++) Nx[k & 1][bj * kSlot + (q / CPT) * 6 + c0 + q % CPT] = A[q];
                }
            }
            if (k + 1 < np && !rhs && bj == k + 1 && bi <= k) {  // M_{i,k+1}, stored transposed
#pragma unroll
                for (int q = 0; q < 6 * CPT; q++) Mp[(k + 1) & 1][bi * kSlot + (c0 + q % CPT) * 6 + q / CPT] = A[q];
            }
        }
        __syncthreads();
        SOLVE_STAMP(tid == 0, 4 * k + 3);
    }
    if (P) __builtin_amdgcn_s_setprio(0);
    if (fail) {  // pop: trial poses = current ones, computeScale = 0
        for (int k = tid; k < a.nkf; k += blockDim.x)
            for (int q = 0; q < 8; q++) Tt[8 * k + q] = T[8 * k + q];
        if (tid == 0) { a.istat[3] = 0; a.scal[1] = 0; a.scal[2] = 0; }
        return;
    }
    if (own && rhs) {  // x = the right-hand side column
#pragma unroll
        for (int r = 0; r < 6; r++) {
            bs[6 * bi + r] = A[r * CPT];
            a.xp[6 * bi + r] = A[r * CPT];
        }
    }
    __syncthreads();
    if (tid >= 64) return;
    SOLVE_STAMP(lane == 0, 252);
    for (int k = lane; k < a.nkf; k += 64) {
        const int pi = a.pose_idx[k];
        if (pi >= 0) {
            double u[6];
#pragma unroll
            for (int q = 0; q < 6; q++) u[q] = bs[6 * pi + q];
            se3_oplus(u, T + 8 * k, Tt + 8 * k);
        } else {
            for (int q = 0; q < 8; q++) Tt[8 * k + q] = T[8 * k + q];
        }
    }
    double sc = 0;
    for (int q = lane; q < N; q += 64) sc += bs[q] * (lam * bs[q] + a.bp[q]);
    sc = wave_sum(sc);
    if (lane == 0) {
        a.scal[1] = sc;
        a.scal[2] = 1;
        a.istat[3] = 1;
    }
    SOLVE_STAMP(lane == 0, 253);
    SOLVE_STAMP_FLUSH();
}

// ---------------------------------------------------------------- MFMA reduced-system solve
// The reduced camera system (g2o's BlockSolver::solve -> LinearSolverEigen, SimplicialLDLT:
// Thirdparty/g2o/g2o/core/block_solver.hpp:354-486, solvers/linear_solver_eigen.h:94-124) as a
// blocked right-looking LDL^T in 16 x 16 tiles, the tile products on v_mfma_f64_16x16x4f64.
// N = 6 np unknowns are padded to 16 T (identity rows); the right-hand side rides as tile column
// T (its column 0).  Every tile (i <= j, upper triangle, and (i, T)) lives in one wave's
// registers in the MFMA C layout (lane l, register s: row (l >> 4) + 4 s, column l & 15) for the
// whole solve.  Panel p:
//   factor  every wave factors the diagonal tile A_pp (staged in LDS) redundantly, one row per
//           lane (the four 16-lane rows alike): Gaussian elimination on [A_pp | I] with the
//           pivot row broadcast by DPP row_newbcast gives D_p and E_p = L_pp^-1 (no sync);
//   row     owners of (p, j > p): W^T_jp = E_p A_pj (4 MFMAs; a C-layout tile is exactly the
//           B operand), L^T_jp = D_p^-1 W^T_jp, both to LDS;
//   update  owners of (i, j), p < i <= j: A_ij -= (L^T_ip)^T W^T_jp (4 MFMAs; both operands are
//           C-layout tiles read lane for lane), the next diagonal tile to LDS.
// Three barriers per panel.  Then one wave back-substitutes L^T x = D^-1 E b with the stored
// L^T_jp and E_p.  Same solution as the LDL^T of the reference up to the rounding order.
using double4_t = __attribute__((ext_vector_type(4))) double;
constexpr int kBaMfmaThreads = 256;  // one wave per SIMD: critical tiles, two bulk waves, factor
constexpr int kBaSolveMfmaMaxPoses = 21;  // 126 unknowns in 8 tiles

template <int J>
__device__ inline double bcast16(double v) {  // lane J of this lane's row of 16 (DPP64 row_newbcast)
    const long long x = __double_as_longlong(v);
    return __longlong_as_double(__builtin_amdgcn_update_dpp(0ll, x, 0x150 + J, 0xF, 0xF, false));
}

// fused broadcast multiply-add, v_fmac_f64 with a DPP64 row_newbcast source (one instruction):
//   fmac_self<J>(acc, m)   acc += m * acc[lane J of the row]
//   fmac_bc<J>(acc, s, m)  acc += s[lane J of the row] * m
// Callers keep every lane active and issue `s_nop 1` between a VALU write of the broadcast
// register and its first DPP read (the DPP read-after-write hazard; hipcc pads nothing in asm).
template <int J> __device__ inline void fmac_self(double& acc, double m);
template <int J> __device__ inline void fmac_bc(double& acc, double s, double m);
#define ORBMI_FMAC_DPP(J)                                                                                        \
    template <> __device__ inline void fmac_self<J>(double& acc, double m) {                                     \
        asm volatile("v_fmac_f64_dpp %0, %0, %1 row_newbcast:" #J " row_mask:0xf bank_mask:0xf" : "+v"(acc) : "v"(m)); \
    }                                                                                                            \
    template <> __device__ inline void fmac_bc<J>(double& acc, double s, double m) {                             \
        asm volatile("v_fmac_f64_dpp %0, %1, %2 row_newbcast:" #J " row_mask:0xf bank_mask:0xf"                   \
                     : "+v"(acc) : "v"(s), "v"(m));                                                              \
    }
ORBMI_FMAC_DPP(0) ORBMI_FMAC_DPP(1) ORBMI_FMAC_DPP(2) ORBMI_FMAC_DPP(3) ORBMI_FMAC_DPP(4) ORBMI_FMAC_DPP(5)
ORBMI_FMAC_DPP(6) ORBMI_FMAC_DPP(7) ORBMI_FMAC_DPP(8) ORBMI_FMAC_DPP(9) ORBMI_FMAC_DPP(10) ORBMI_FMAC_DPP(11)
ORBMI_FMAC_DPP(12) ORBMI_FMAC_DPP(13) ORBMI_FMAC_DPP(14) ORBMI_FMAC_DPP(15)
#undef ORBMI_FMAC_DPP

// The elimination step's dependent chain as single instructions in asm volatile statements:
// volatile asm keeps its program order, so the chain stays interleaved with the step's bulk
// FMAs (as plain builtins the scheduler sank the whole chain below them, exposing every latency).
template <int J> __device__ inline double bcast16_asm(double v);
#define ORBMI_BCAST_DPP(J)                                                                               \
    template <> __device__ inline double bcast16_asm<J>(double v) {                                     \
        double d;                                                                                        \
        asm volatile("v_mov_b64_dpp %0, %1 row_newbcast:" #J " row_mask:0xf bank_mask:0xf" : "=v"(d) : "v"(v)); \
        return d;                                                                                        \
    }
ORBMI_BCAST_DPP(1) ORBMI_BCAST_DPP(2) ORBMI_BCAST_DPP(3) ORBMI_BCAST_DPP(4) ORBMI_BCAST_DPP(5)
ORBMI_BCAST_DPP(6) ORBMI_BCAST_DPP(7) ORBMI_BCAST_DPP(8) ORBMI_BCAST_DPP(9) ORBMI_BCAST_DPP(10)
ORBMI_BCAST_DPP(11) ORBMI_BCAST_DPP(12) ORBMI_BCAST_DPP(13) ORBMI_BCAST_DPP(14) ORBMI_BCAST_DPP(15)
#undef ORBMI_BCAST_DPP
__device__ inline double rcp_asm(double d) {  // v_rcp_f64 (a transcendental: one wait state before a use)
    double r;
    asm volatile("v_rcp_f64 %0, %1" : "=v"(r) : "v"(d));
    return r;
}
__device__ inline double newton_err_asm(double d, double r) {  // 1 - d r
    double e;
    asm volatile("v_fma_f64 %0, -%1, %2, 1.0" : "=v"(e) : "v"(d), "v"(r));
    return e;
}
__device__ inline double fma_asm(double a, double b, double c) {
    double o;
    asm volatile("v_fma_f64 %0, %1, %2, %3" : "=v"(o) : "v"(a), "v"(b), "v"(c));
    return o;
}
__device__ inline double negmul_asm(double a, double b) {  // -(a b)
    double o;
    asm volatile("v_mul_f64 %0, -%1, %2" : "=v"(o) : "v"(a), "v"(b));
    return o;
}
__device__ inline double select_asm(double v, unsigned long long lanes) {  // lanes set: v, else +0
    const unsigned long long x = __double_as_longlong(v);
    unsigned lo, hi;
    asm volatile("v_cndmask_b32_e64 %0, 0, %2, %4\n\tv_cndmask_b32_e64 %1, 0, %3, %4"
                 : "=&v"(lo), "=&v"(hi) : "v"((unsigned)x), "v"((unsigned)(x >> 32)), "s"(lanes));
    return __longlong_as_double(((unsigned long long)hi << 32) | lo);
}

// 1 / d: v_rcp_f64 (2^-24.4 relative, tools/ubench/dpp64.hip) and one Newton step (2^-48)
__device__ inline double rcp1_f64(double d) {
    const double r = __builtin_amdgcn_rcp(d);
    return fma(r, fma(-d, r, 1.0), r);
}

// Panel factorisation: Gaussian elimination on [A_pp | I] for D_p and E_p = L_pp^-1, one row r of
// the tile per lane.  A is replicated in the four 16-lane groups; E is split by strided columns:
// lane (g, r) holds E[r][g + 4 k], k = 0..3 (so a step's E update is J / 4 + 1 FMAs, not J + 1;
// Eg[k] is also the MFMA A operand of k-chunk k).
// Item I of elimination step J's bulk FMAs: A[J + 2 ..] (14 - J items), then the E columns.
template <int J, int I0, int I1>
__device__ inline void ldl_bulk(double (&A)[16], double (&Eg)[4], double nl) {
    if constexpr (I0 < I1) {
        constexpr int NA = 14 - J;
        if constexpr (I0 < NA) fmac_self<J>(A[J + 2 + I0], nl);
        else fmac_self<J>(Eg[I0 - NA], nl);
        ldl_bulk<J, I0 + 1, I1>(A, Eg, nl);
    }
}
__device__ inline double mul_asm(double a, double b) {
    double o;
    asm volatile("v_mul_f64 %0, %1, %2" : "=v"(o) : "v"(a), "v"(b));
    return o;
}

// Elimination step J, software-pipelined: nl = -l_rJ (0 for rows r <= J) comes from the previous
// step.  Rows r > J subtract l_rJ times pivot row J (A[J + 1 ..] and the E columns <= J of lane J,
// broadcast inside the fused FMAs).  The next pivot column A[J + 1] goes first; step J + 1's
// multiplier is a short chain -- pivot broadcast, reciprocal, then the Newton-corrected quotient
// nl' = a0 + a0 (1 - d r0) with a0 = -A[J + 1] r0 masked to the rows below the pivot (the mask
// folded into a multiply, no select on the chain) -- interleaved with this step's bulk FMAs.
// Step 15 has no row below its pivot: nothing to do.  inv[J] = 1 / d_J.  Each step is one asm
// statement generated by tools/gen_ldl16.py (ldl16_steps.inc): the order and the DPP wait states
// inside a step are fixed there, and the statement's leading s_nop 1 covers whatever the
// compiler put in front of it (tools/check_dpp_hazards.py checks the built code).
template <int J>
__device__ inline void ldl16_step(double (&A)[16], double (&Eg)[4], double (&inv)[16], int r, double nl);
#include "ldl16_steps.inc"

__device__ inline void ldl16(double (&A)[16], double (&Eg)[4], double (&inv)[16], int r) {
    inv[0] = rcp1_f64(bcast16<0>(A[0]));
    const double nl0 = r > 0 ? -(A[0] * inv[0]) : 0.0;
    ldl16_step<0>(A, Eg, inv, r, nl0);
}

// LDS flag hand-offs between the waves of one workgroup (release after the data, acquire after
// the flag)
__device__ inline void lds_publish(int* f, int v) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    *(volatile int*)f = v;
}
__device__ inline void lds_wait_ge(const int* f, int v) {
    while (*(const volatile int*)f < v) __builtin_amdgcn_s_sleep(1);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// tile (i, j) of the upper triangle plus the right-hand-side column (j == T), row-major numbering
template <int T>
__host__ __device__ constexpr int mfma_tile_index(int i, int j) { return i * (T + 1) - i * (i - 1) / 2 + (j - i); }
// the m-th tile (i, j) with j >= i + 2 (the bulk waves' tiles), row-major
template <int T>
__host__ __device__ constexpr int mfma_bulk_i(int m) {
    for (int i = 0; i < T; i++) {
        if (m < T - i - 1) return i;
        m -= T - i - 1;
    }
    return -1;
}
template <int T>
__host__ __device__ constexpr int mfma_bulk_j(int m) {
    for (int i = 0; i < T; i++) {
        if (m < T - i - 1) return i + 2 + m;
        m -= T - i - 1;
    }
    return -1;
}

template <int T>
struct MfmaSolveLds {
    static constexpr int NL = T * (T - 1) / 2;  // L^T_jp tiles, p < j < T
    double dg[16 * 17];                  // the next panel's diagonal tile (row-major)
    double Es[2][16 * 17];               // E_p rows, buffer p & 1 (the MFMA A operands are read here)
    double dvs[2][16];                   // 1 / d of the panel's rows
    double Eall[T][256];                 // E_p for the back substitution (row-major)
    double Wt[2][T + 1][4][64];          // -W^T_jp, buffer p & 1 (C layout)
    double Lt[NL > 0 ? NL : 1][4][64];   // L^T_jp (C layout: row t contiguous at [t >> 2][16 (t & 3)])
    double ys[16 * T], xs[16 * T];
    int flag_dg, flag_e, row_cnt[T], fail;
    __device__ static int lt_index(int p, int j) { return p * (2 * T - p - 1) / 2 + (j - p - 1); }
};

constexpr int kMfmaBulkWaves = 2;  // waves 1, 2; wave 0 = critical tiles, wave 3 = factor

// row panel product of one tile X = A_pj (C layout, registers) with E_p: z = W^T_jp = E_p X;
// -W^T to LDS, L^T = D^-1 W^T to LDS (or y_p = D^-1 E_p b_p for the right-hand side); returns z
template <int T>
__device__ inline double4_t mfma_row_tile(MfmaSolveLds<T>& L, int p, int j, const double4_t& X, const double (&e)[4],
                                          const double (&dv)[4], int lane) {
    double4_t z = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int s = 0; s < 4; s++) z = __builtin_amdgcn_mfma_f64_16x16x4f64(e[s], X[s], z, 0, 0, 0);
    const int q = lane >> 4, n = lane & 15;
#pragma unroll
    for (int s = 0; s < 4; s++) {
        L.Wt[p & 1][j][s][lane] = -z[s];
        const double lt = z[s] * dv[s];
        if (j < T) L.Lt[MfmaSolveLds<T>::lt_index(p, j)][s][lane] = lt;
        else if (n == 0) L.ys[16 * p + q + 4 * s] = lt;
    }
    return z;
}

// trailing update of tile (i, j) by panel p: X -= (L^T_ip)^T W^T_jp, both operands from LDS
template <int T>
__device__ inline void mfma_update_tile(MfmaSolveLds<T>& L, int p, int i, int j, double4_t& X, int lane) {
    const double* lp = &L.Lt[MfmaSolveLds<T>::lt_index(p, i)][0][lane];
    const double* wp = &L.Wt[p & 1][j][0][lane];
    double lo[4], wo[4];
#pragma unroll
    for (int s = 0; s < 4; s++) { lo[s] = lp[64 * s]; wo[s] = wp[64 * s]; }
#pragma unroll
    for (int s = 0; s < 4; s++) X = __builtin_amdgcn_mfma_f64_16x16x4f64(lo[s], wo[s], X, 0, 0, 0);
}

template <int T>
__device__ inline void mfma_load_tile(const BaDev& a, int i, int j, double4_t& X, int lane) {
    const double* src = a.S + (size_t)mfma_tile_index<T>(i, j) * 256 + lane;  // padding written by k_ba_schur
#pragma unroll
    for (int s = 0; s < 4; s++) X[s] = src[64 * s];
}

template <int T>
__device__ inline void mfma_operands(const MfmaSolveLds<T>& L, int p, int lane, double (&e)[4], double (&dv)[4]) {
    const int q = lane >> 4, n = lane & 15;
#pragma unroll
    for (int s = 0; s < 4; s++) {
        e[s] = L.Es[p & 1][n * 17 + 4 * s + q];  // A operand: E[n][4 s + q]
        dv[s] = L.dvs[p & 1][q + 4 * s];         // 1 / d of C-layout row q + 4 s
    }
}

template <int T>
__device__ inline void mfma_put_dg(MfmaSolveLds<T>& L, const double4_t& X, int lane) {
    const int q = lane >> 4, n = lane & 15;
#pragma unroll
    for (int s = 0; s < 4; s++) L.dg[(q + 4 * s) * 17 + n] = X[s];
}

// wave 0: the critical tiles, diagonal (i, i) and first off-diagonal (i, i + 1) (the last one the
// right-hand side's).  Per panel: as soon as E_p is published, row tile (p, p + 1), then the next
// diagonal tile's update from registers and its hand-off to the factor wave; then the bulk of its
// updates of this panel
template <int T>
__device__ inline void mfma_critical_wave(const BaDev& a, MfmaSolveLds<T>& L, int lane,
                                          unsigned long long* ts) {
    double4_t D[T], F1[T];
#pragma unroll
    for (int i = 0; i < T; i++) {
        mfma_load_tile<T>(a, i, i, D[i], lane);
        mfma_load_tile<T>(a, i, i + 1, F1[i], lane);
    }
    mfma_put_dg<T>(L, D[0], lane);
    if (lane == 0) lds_publish(&L.flag_dg, 0);
    SOLVE_STAMP_TO(ts, lane == 0, 251);
#pragma unroll
    for (int p = 0; p < T; p++) {
        lds_wait_ge(&L.flag_e, p);
        SOLVE_STAMP_TO(ts, lane == 0, 8 * p + 2);
        double e[4], dv[4];
        mfma_operands<T>(L, p, lane, e, dv);
        const double4_t z = mfma_row_tile<T>(L, p, p + 1, F1[p], e, dv, lane);
        if (p == T - 1) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            if (lane == 0) atomicAdd(&L.row_cnt[p], 1);
            break;
        }
        // A_{p+1,p+1} -= (L^T)^T W^T with this tile's L^T = D^-1 z and W^T = z, in registers
#pragma unroll
        for (int s = 0; s < 4; s++)
            D[p + 1] = __builtin_amdgcn_mfma_f64_16x16x4f64(z[s] * dv[s], -z[s], D[p + 1], 0, 0, 0);
        mfma_put_dg<T>(L, D[p + 1], lane);
        if (lane == 0) lds_publish(&L.flag_dg, p + 1);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        if (lane == 0) atomicAdd(&L.row_cnt[p], 1);
        SOLVE_STAMP_TO(ts, lane == 0, 8 * p + 3);
        lds_wait_ge(&L.row_cnt[p], 1 + kMfmaBulkWaves);
        SOLVE_STAMP_TO(ts, lane == 0, 8 * p + 4);
#pragma unroll
        for (int i = p + 1; i < T; i++) mfma_update_tile<T>(L, p, i, i + 1, F1[i], lane);
#pragma unroll
        for (int i = p + 2; i < T; i++) mfma_update_tile<T>(L, p, i, i, D[i], lane);
        SOLVE_STAMP_TO(ts, lane == 0, 8 * p + 5);
    }
}

// waves 1, 2: the tiles (i, j >= i + 2), round-robin
template <int T, int O>
__device__ inline void mfma_bulk_wave(const BaDev& a, MfmaSolveLds<T>& L, int lane) {
    constexpr int NB = T * (T - 1) / 2;
    constexpr int KB = (NB + kMfmaBulkWaves - 1 - O) / kMfmaBulkWaves;
    double4_t X[KB > 0 ? KB : 1];
#pragma unroll
    for (int k = 0; k < KB; k++)
        mfma_load_tile<T>(a, mfma_bulk_i<T>(O + kMfmaBulkWaves * k), mfma_bulk_j<T>(O + kMfmaBulkWaves * k), X[k], lane);
    for (int p = 0; p < T; p++) {
        lds_wait_ge(&L.flag_e, p);
        double e[4], dv[4];
        mfma_operands<T>(L, p, lane, e, dv);
#pragma unroll
        for (int k = 0; k < KB; k++) {
            const int i = mfma_bulk_i<T>(O + kMfmaBulkWaves * k), j = mfma_bulk_j<T>(O + kMfmaBulkWaves * k);
            if (i == p) mfma_row_tile<T>(L, p, j, X[k], e, dv, lane);
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        if (lane == 0) atomicAdd(&L.row_cnt[p], 1);
        if (p == T - 1) break;
        lds_wait_ge(&L.row_cnt[p], 1 + kMfmaBulkWaves);
#pragma unroll
        for (int k = 0; k < KB; k++) {
            const int i = mfma_bulk_i<T>(O + kMfmaBulkWaves * k), j = mfma_bulk_j<T>(O + kMfmaBulkWaves * k);
            if (i > p) mfma_update_tile<T>(L, p, i, j, X[k], lane);
        }
    }
}

template <int T>
__device__ __attribute__((always_inline)) inline void solve_mfma_body(const BaDev& a) {
    const BaCtl& ctl = *a.ctl;
    if (ctl.done || ctl.gen != a.run_gen) return;
    const int np = ctl.np, N = 6 * np;
    __shared__ MfmaSolveLds<T> L;
    const int tid = threadIdx.x, lane = tid & 63, q = lane >> 4, n = lane & 15;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    SOLVE_STAMP_DECL;
    SOLVE_STAMP(tid == 0, 250);
    if (tid == 0) {
        L.flag_dg = L.flag_e = -1;
        L.fail = 0;
    }
    if (tid < T) L.row_cnt[tid] = 0;
    __syncthreads();
    if (w == 0) { mfma_critical_wave<T>(a, L, lane, SOLVE_STAMP_PTR); return; }
    if (w == 1) { mfma_bulk_wave<T, 0>(a, L, lane); return; }
    if (w == 2) { mfma_bulk_wave<T, 1>(a, L, lane); return; }
    // ---- wave 3: A_pp -> E_p = L_pp^-1, D_p^-1 as soon as A_pp is final
    for (int p = 0; p < T; p++) {
        lds_wait_ge(&L.flag_dg, p);
        SOLVE_STAMP(lane == 0, 8 * p);
        double A[16], Eg[4], inv[16];
#pragma unroll
        for (int k = 0; k < 16; k++) A[k] = L.dg[n * 17 + k];
#pragma unroll
        for (int k = 0; k < 4; k++) Eg[k] = q + 4 * k == n ? 1.0 : 0.0;
        ldl16(A, Eg, inv, n);
#pragma unroll
        for (int k = 0; k < 4; k++) {  // lane (q, n): E[n][q + 4 k]
            L.Es[p & 1][n * 17 + q + 4 * k] = Eg[k];
            L.Eall[p][n * 16 + q + 4 * k] = Eg[k];
        }
        if (lane == 0) {
            bool bad = false;
#pragma unroll
            for (int k = 0; k < 16; k++) {
                L.dvs[p & 1][k] = inv[k];
                bad |= !isfinite(inv[k]) || inv[k] == 0.0;  // d zero, inf or NaN
            }
            if (bad) L.fail = 1;
        }
        if (lane == 0) lds_publish(&L.flag_e, p);
        SOLVE_STAMP(lane == 0, 8 * p + 1);
    }
    // ---- after every row panel: back substitution and the trial poses
    lds_wait_ge(&L.row_cnt[T - 1], 1 + kMfmaBulkWaves);
    SOLVE_STAMP(lane == 0, 252);
    const double* __restrict__ Tc = a.Tb[ctl.cur];
    double* __restrict__ Tt = a.Tb[ctl.cur ^ 1];
    if (L.fail) {  // pop: trial poses = current ones, computeScale = 0
        for (int k = lane; k < a.nkf; k += 64)
            for (int qq = 0; qq < 8; qq++) Tt[8 * k + qq] = Tc[8 * k + qq];
        if (lane == 0) { a.istat[3] = 0; a.scal[1] = 0; a.scal[2] = 0; }
        return;
    }
    // x_p = E_p^T (y_p - sum_{j > p} L^T_jp x_j).  Lane (g, t), g = lane >> 4: the copies xr[j]
    // are rotated by 4 g (lane (g, c) holds x_j[(c + 4 g) & 15]), so group g covers columns
    // 4 g .. 4 g + 3 of every tile with four fused DPP FMAs reading x from lanes 0..3 of its row;
    // the groups' partial sums meet by permlane swaps.  x_p comes out rotated: lane (g, c) forms
    // column (c + 4 g) & 15 of E_p^T r (four partial sums over t).  Software-pipelined: panel
    // p - 1's LDS operands (L^T rows, y, E column) are loaded while panel p computes, so each
    // panel waits on its dependent FMAs only, not on three LDS round trips.
    {
        const int g = q, t = n, rot = (n + 4 * g) & 15;
        double xr[T];
        double ltb[2][T][4], e4b[2][16], ysb[2];
        auto load = [&](int p, int b) {
#pragma unroll
            for (int j = p + 1; j < T; j++) {
                const double* row = &L.Lt[MfmaSolveLds<T>::lt_index(p, j)][t >> 2][16 * (t & 3) + 4 * g];
#pragma unroll
                for (int u = 0; u < 4; u++) ltb[b][j][u] = row[u];
            }
            ysb[b] = L.ys[16 * p + t];
            const double* Ec = &L.Eall[p][rot];
#pragma unroll
            for (int u = 0; u < 16; u++) e4b[b][u] = Ec[16 * u];
        };
        load(T - 1, (T - 1) & 1);
#pragma unroll
        for (int p = T - 1; p >= 0; p--) {
            const int b = p & 1;
            if (p > 0) load(p - 1, b ^ 1);
            double acc[4] = {0.0, 0.0, 0.0, 0.0};
            // (each DPP group is one asm statement opening with s_nop 1: the broadcast sources
            // xr[j] and r may have been written, or copied, right in front of it)
#pragma unroll
            for (int j = p + 1; j < T; j++) {
                double& a0 = acc[(j - p) & 3];
                asm volatile("s_nop 1\n\t"
                             "v_fmac_f64_dpp %0, %1, %2 row_newbcast:0 row_mask:0xf bank_mask:0xf\n\t"
                             "v_fmac_f64_dpp %0, %1, %3 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
                             "v_fmac_f64_dpp %0, %1, %4 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
                             "v_fmac_f64_dpp %0, %1, %5 row_newbcast:3 row_mask:0xf bank_mask:0xf"
                             : "+v"(a0)
                             : "v"(xr[j]), "v"(ltb[b][j][0]), "v"(ltb[b][j][1]), "v"(ltb[b][j][2]), "v"(ltb[b][j][3]));
            }
            double s = (acc[0] + acc[1]) + (acc[2] + acc[3]);
            s = swap_combine<16>(s, s);
            s = swap_combine<32>(s, s);
            const double r = ysb[b] - s;
            const double* e4 = e4b[b];
            double x0 = 0.0, x1 = 0.0, x2 = 0.0, x3 = 0.0;
            asm volatile("s_nop 1\n\t"
                         "v_fmac_f64_dpp %0, %4, %5 row_newbcast:0 row_mask:0xf bank_mask:0xf\n\t"
                         "v_fmac_f64_dpp %1, %4, %6 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
                         "v_fmac_f64_dpp %2, %4, %7 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
                         "v_fmac_f64_dpp %3, %4, %8 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
                         "v_fmac_f64_dpp %0, %4, %9 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
                         "v_fmac_f64_dpp %1, %4, %10 row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
                         "v_fmac_f64_dpp %2, %4, %11 row_newbcast:6 row_mask:0xf bank_mask:0xf\n\t"
                         "v_fmac_f64_dpp %3, %4, %12 row_newbcast:7 row_mask:0xf bank_mask:0xf\n\t"
                         "v_fmac_f64_dpp %0, %4, %13 row_newbcast:8 row_mask:0xf bank_mask:0xf\n\t"
                         "v_fmac_f64_dpp %1, %4, %14 row_newbcast:9 row_mask:0xf bank_mask:0xf\n\t"
                         "v_fmac_f64_dpp %2, %4, %15 row_newbcast:10 row_mask:0xf bank_mask:0xf\n\t"
                         "v_fmac_f64_dpp %3, %4, %16 row_newbcast:11 row_mask:0xf bank_mask:0xf\n\t"
                         "v_fmac_f64_dpp %0, %4, %17 row_newbcast:12 row_mask:0xf bank_mask:0xf\n\t"
                         "v_fmac_f64_dpp %1, %4, %18 row_newbcast:13 row_mask:0xf bank_mask:0xf\n\t"
                         "v_fmac_f64_dpp %2, %4, %19 row_newbcast:14 row_mask:0xf bank_mask:0xf\n\t"
                         "v_fmac_f64_dpp %3, %4, %20 row_newbcast:15 row_mask:0xf bank_mask:0xf"
                         : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3)
                         : "v"(r), "v"(e4[0]), "v"(e4[1]), "v"(e4[2]), "v"(e4[3]), "v"(e4[4]), "v"(e4[5]), "v"(e4[6]),
                           "v"(e4[7]), "v"(e4[8]), "v"(e4[9]), "v"(e4[10]), "v"(e4[11]), "v"(e4[12]), "v"(e4[13]),
                           "v"(e4[14]), "v"(e4[15]));
            const double x = (x0 + x1) + (x2 + x3);
            xr[p] = x;
            if (lane < 16) L.xs[16 * p + t] = x;  // group 0: unrotated
        }
        wave_sync_lds();
    }
    SOLVE_STAMP(lane == 0, 254);
    const double lam = a.scal[3];
    for (int qq = lane; qq < N; qq += 64) a.xp[qq] = L.xs[qq];
    for (int k = lane; k < a.nkf; k += 64) {
        const int pi = a.pose_idx[k];
        if (pi >= 0) {
            double u[6];
#pragma unroll
            for (int qq = 0; qq < 6; qq++) u[qq] = L.xs[6 * pi + qq];
            se3_oplus(u, Tc + 8 * k, Tt + 8 * k);
        } else {
            for (int qq = 0; qq < 8; qq++) Tt[8 * k + qq] = Tc[8 * k + qq];
        }
    }
    double sc = 0;
    for (int qq = lane; qq < N; qq += 64) sc += L.xs[qq] * (lam * L.xs[qq] + a.bp[qq]);
    sc = wave_sum(sc);
    if (lane == 0) {
        a.scal[1] = sc;
        a.scal[2] = 1;
        a.istat[3] = 1;
    }
    SOLVE_STAMP(lane == 0, 253);
#ifdef ORBMI_SOLVE_TRACE
    if (lane == 0)
        for (int i_ = 0; i_ < 256; i_++) g_solve_trace[i_] = tstamp[i_];
#endif
}

template <int T>
__global__ __launch_bounds__(kBaMfmaThreads) void k_ba_solve_mfma(BaDev a) { solve_mfma_body<T>(a); }

// The Schur complement and the MFMA solve in one launch: the Schur blocks as k_ba_schur, then the
// last block to finish (arrival counter; device-scope release / acquire, so every block's tiles
// are visible to it) runs the solve with its first four waves.  One launch per trial fewer.
template <int T>
__global__ __launch_bounds__(kSchurThreads) void k_ba_schur_solve(BaDev a) {
    {
        const BaCtl& ctl = *a.ctl;
        if (ctl.done || ctl.gen != a.run_gen) return;  // the same for every block
    }
    schur_body(a);
    __shared__ int last;
    __syncthreads();
    if (threadIdx.x == 0) {
        __threadfence();
        last = atomicAdd(&a.ctl->arrive_s, 1u) == gridDim.x - 1;
    }
    __syncthreads();
    if (!last) return;
    __threadfence();
    if (threadIdx.x == 0) a.ctl->arrive_s = 0;
    if (threadIdx.x >= kBaMfmaThreads) return;
    solve_mfma_body<T>(a);
}

// ---------------------------------------------------------------- Levenberg control
// fixed-order sum of n partials by one wave (lane l: l, l + 64, ...; then a fixed xor tree,
// lane 0's value broadcast): deterministic run to run
// the same over partials other workgroups of this launch wrote with sc1 stores (sc1 loads)
__device__ inline double wave_sum_fixed_sc1(const double* p, int n) {
    double s = 0;
    for (int k = threadIdx.x; k < n; k += 64) s += __hip_atomic_load(p + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    return __shfl(s, 0, 64);
}
__device__ inline double wave_sum_fixed(const double* p, int n) {
    double s = 0;
    for (int k = threadIdx.x; k < n; k += 64) s += p[k];
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    return __shfl(s, 0, 64);
}

// one wave, after each trial: OptimizationAlgorithmLevenberg::solve's decision
// (levenberg.cpp:104-164) and SparseOptimizer::optimize's loop (sparse_optimizer.cpp:354-419)
// with ORB-SLAM2's 3-bad-iterations stop; pbStopFlag is read through the host-mapped mirror.
// currentChi of an iteration's computeActiveErrors: the first linearisation's chi2 at
// iteration 0, the accepted trial's chi2 afterwards (the same errors; an iteration that ends
// on a rejection keeps the estimate, hence the chi2 and the linear system).
__device__ inline void k_ba_control_body(const BaDev& a) {
    BaCtl& c = *a.ctl;
    // the three fixed-order sums of wave_sum_fixed with their loads issued together (one memory
    // latency on the trial chain instead of three); the linearisation's chi2 only where it is read
    const bool need_lin = c.trial == 0 && c.it == 0;
    double l = 0, t = 0, sc = 0;
    const int lane = threadIdx.x, nmax = max(need_lin ? a.nb_e : 0, a.nb_q);
    for (int k = lane; k < nmax; k += 64) {
        if (need_lin && k < a.nb_e) l += a.part_lin[k];
        if (k < a.nb_q) {  // (this launch's blocks wrote them: sc1 loads, see k_ba_update_errors)
            t += __hip_atomic_load(&a.part_tchi[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            sc += __hip_atomic_load(&a.part_tscale[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    for (int o = 32; o > 0; o >>= 1) {
        l += __shfl_xor(l, o, 64);
        t += __shfl_xor(t, o, 64);
        sc += __shfl_xor(sc, o, 64);
    }
    const double lin = __shfl(l, 0, 64), tchi = __shfl(t, 0, 64), tsc = __shfl(sc, 0, 64);
    if (threadIdx.x != 0) return;
    if (c.trial == 0) {
        if (c.it == 0) c.currentChi = lin;
        c.iniChi = c.currentChi;
    }
    if (c.it == 0 && c.trial == 0) c.lambda = a.scal[3];  // computeLambdaInit (k_ba_schur)
    const bool ok2 = a.scal[2] != 0;
    const double tempChi = ok2 ? tchi : DBL_MAX;
    const double scale = ok2 ? tsc + a.scal[1] : 0.0;
    const double rho = (c.currentChi - tempChi) / (scale + 1e-3);
    if (rho > 0 && isfinite(tempChi)) {  // accept: the trial estimate and its linear system become current
        const double t = 2 * rho - 1;
        double alpha = 1. - t * t * t;
        alpha = fmin(alpha, 2. / 3.);
        c.lambda *= fmax(1. / 3., alpha);
        c.ni = 2;
        c.currentChi = tempChi;
        c.cur ^= 1;
        c.lin ^= 1;
    } else {  // reject: pop (the trial buffers are not adopted)
        c.lambda *= c.ni;
        c.ni *= 2;
    }
    c.trial++;
    c.steps++;
    // the inner loop's `while (rho < 0 && qmax < 10 && !terminate())`: the flag is read only
    // when the first two hold; raised, the iteration ends on the rejected trial
    if (rho < 0 && c.trial < 10 && !ba_check_stop(a, c)) return;  // next trial of the same iteration
    c.it++;
    bool term;
    if (c.trial == 10 || rho == 0) {
        term = true;
    } else {
        if ((c.iniChi - c.currentChi) * 1e3 < c.iniChi) c.nbad++;
        else c.nbad = 0;
        term = c.nbad >= 3;
    }
    c.trial = 0;
    // the outer loop's `i < iterations && !terminate() && ok`: the flag is read while i < iterations
    const bool stop = c.it < c.max_it && ba_check_stop(a, c);
    if (term || c.it >= c.max_it || stop) c.done = 1;
}

// ---------------------------------------------------------------- update + trial errors
// block = kBaUpdPts points, 8 lanes each: x_l = D^-1 (b_l - Hpl^T x_p), X_t = X + x_l (computeScale
// part); then every thread takes edges of the block's points: computeActiveErrors on the trial
// state (T_t from the solve) and the edge's linearisation at that state into the other
// linear-system buffer; threads 0..31 then sum the points' Hll / b_l there.  Block partials:
// robust chi2 and scale; the last block to finish runs the Levenberg decision.
#ifndef ORBMI_UPD_PTS
#define ORBMI_UPD_PTS 32
#endif
constexpr int kBaUpdPts = ORBMI_UPD_PTS;          // (16 per block, 188 blocks for config 3, measured slower)
constexpr int kBaUpdLanes = 8;                     // threads per point
constexpr int kBaUpdThreads = kBaUpdPts * kBaUpdLanes;
constexpr int kBaUpdLdsEdges = 512;                // a block's edges whose Hll / b_l terms stay in LDS
static_assert(kBaUpdLanes == 8, "8-lane segmented sums");

// sum over the 8 lanes of an aligned group (DPP quad xor steps, then the half-row mirror); every
// lane of the group ends with the same value
__device__ inline double sum8(double v) {
    v += dpp_mov<kDppXor1>(v);
    v += dpp_mov<kDppXor2>(v);
    return v + dpp_mov<kDppHalfMirror>(v);
}

__global__ __launch_bounds__(kBaUpdThreads) void k_ba_update_errors(BaDev a) {
    // the graph's part of what the block reads (static within an optimize()) is requested before
    // the LM state, so that its dependent loads overlap the control block's
    const int p0 = blockIdx.x * kBaUpdPts, p1 = min(p0 + kBaUpdPts, a.npt);
    const int tid = threadIdx.x, ps = tid / kBaUpdLanes, j = tid % kBaUpdLanes;
    const int p = p0 + ps;
    const bool own = p < p1;
    const int pe0 = own ? a.pt_start[p] : 0, pe1 = own ? a.pt_start[p + 1] : 0;
    const int be0 = p0 < p1 ? a.pt_start[p0] : 0, be1 = p0 < p1 ? a.pt_start[p1] : 0;
    const int e_pre = be0 + tid;
    EdgeIn pre;
    if (e_pre < be1) edge_in_static(a, e_pre, pre);
    BaCtl& ctl = *a.ctl;
    if (ctl.done || ctl.gen != a.run_gen) return;
    const int L = ctl.lin;
    const BaSys y = ba_sys(a, L);      // current linear system
    const BaSys t = ba_sys(a, L ^ 1);  // trial state's linear system (adopted if accepted)
    const double lam = a.scal[3];
    const double* __restrict__ X = a.Xb[ctl.cur];
    const double* __restrict__ Tt = a.Tb[ctl.cur ^ 1];
    double* __restrict__ Xt = a.Xb[ctl.cur ^ 1];
    double* __restrict__ part_chi = a.part_tchi;
    double* __restrict__ part_scale = a.part_tscale;
    __shared__ double red[2 * kBaUpdThreads / 64];
    __shared__ double xs[kBaUpdPts][4];
    __shared__ double sHe[kBaUpdLdsEdges * 9];
    __shared__ bool last;
    const bool ok = a.istat[3] != 0;
    // the block's edges (thread per edge in the trial pass): the first one's trial pose is loaded
    // now, under the back substitution's loads (its record and camera came before the LM state)
    if (e_pre < be1) edge_in_pose(Tt, pre);
    double sc = 0, chi = 0;
    {  // back substitution x_l = D^-1 (b_l - sum_e Hpl_e^T x_p), 8 lanes per point
        double c0 = 0, c1 = 0, c2 = 0, act = 0;
        for (int e = pe0 + j; e < pe1; e += kBaUpdLanes) {
            act += (a.eflag[e] & 4) ? 1.0 : 0.0;
            const int i1 = a.e_pi[e];
            if (i1 < 0) continue;  // inactive edges into free poses carry a zero block
            const double* B = y.Hpl + 18 * (long long)e;
            const double* xp = a.xp + 6 * i1;
#pragma unroll
            for (int r = 0; r < 6; r++) {
                c0 += B[r * 3] * xp[r];
                c1 += B[r * 3 + 1] * xp[r];
                c2 += B[r * 3 + 2] * xp[r];
            }
        }
        c0 = sum8(c0); c1 = sum8(c1); c2 = sum8(c2); act = sum8(act);
        if (own && j == 0) {
            double xl[3] = {0, 0, 0};
            if (ok && act > 0) {  // point_active
                const double cl[3] = {y.bl[3 * p] - c0, y.bl[3 * p + 1] - c1, y.bl[3 * p + 2] - c2};
                double Di[9];
                point_dinv(y.Hll, p, lam, Di);
                for (int r = 0; r < 3; r++) xl[r] = Di[r * 3] * cl[0] + Di[r * 3 + 1] * cl[1] + Di[r * 3 + 2] * cl[2];
            }
            for (int r = 0; r < 3; r++) {
                const double x = X[4 * p + r] + xl[r];
                Xt[4 * p + r] = x;
                xs[ps][r] = x;
                if (ok) sc += xl[r] * (lam * xl[r] + y.bl[3 * p + r]);
            }
        }
    }
    __syncthreads();
    // trial errors (computeActiveErrors) and the trial state's linearisation, thread per edge;
    // the edges' Hll / b_l terms go to LDS when the block's edges fit
    const bool lds = be1 - be0 <= kBaUpdLdsEdges;
    for (int e = e_pre; e < be1; e += blockDim.x) {
        EdgeIn s;
        if (e == e_pre) s = pre;
        else edge_in(a, e, Tt, s);
        chi += edge_trial(a, t, e, s, &xs[s.e.point - p0][0], lds ? sHe + 9 * (e - be0) : nullptr);
    }
    __syncthreads();
    {  // Hll / b_l at the trial state, 8 lanes per point, edges in order within a lane
        double h[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
        for (int e = pe0 + j; e < pe1; e += kBaUpdLanes) {
            if (!(a.eflag[e] & 4)) continue;
            const double* He = lds ? sHe + 9 * (e - be0) : t.Hle + 9 * (long long)e;
#pragma unroll
            for (int k = 0; k < 9; k++) h[k] += He[k];
        }
#pragma unroll
        for (int k = 0; k < 9; k++) h[k] = sum8(h[k]);
        if (own && j == 0) {
            double* H = t.Hll + 9 * p;
            H[0] = h[0]; H[1] = h[1]; H[2] = h[2];
            H[3] = h[1]; H[4] = h[3]; H[5] = h[4];
            H[6] = h[2]; H[7] = h[4]; H[8] = h[5];
            for (int k = 0; k < 3; k++) t.bl[3 * p + k] = h[6 + k];
        }
    }
    block_sum2_t0<kBaUpdThreads>(chi, sc, red);  // thread 0 holds both
    // the fan-in to the last block without __threadfence (an L2 write-back + L1 invalidate,
    // ~3.5 us on gfx950, twice per trial): the two partials go out as agent-scope (sc1) stores,
    // drained before the arrival add; the last block reads them with sc1 loads
    // (MI355X_MICROARCH.md, inter-workgroup hand-offs, row 1).  What else the blocks wrote is
    // read by the next launches only.
    if (tid == 0) {
        __hip_atomic_store(&part_chi[blockIdx.x], chi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&part_scale[blockIdx.x], sc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        last = atomicAdd(&ctl.arrive, 1u) == gridDim.x - 1;
    }
    __syncthreads();
    if (!last) return;
    if (tid < 64) k_ba_control_body(a);
    if (tid == 0) ctl.arrive = 0;
}

// activeRobustChi2 after optimize() (k_ba_errors partials) and the iteration count
__device__ inline void chi_body(const BaDev& a, int phase) {
    const double chi = wave_sum_fixed_sc1(a.part_lin, a.nb_e);
    if (threadIdx.x == 0) {
        BaCtl& c = *a.ctl;
        c.chi_out[phase] = chi;
        c.it_out[phase] = (c.np + c.nl == 0) ? -1 : c.it;
        c.phases_done = phase + 1;
        if (phase == 0) c.do_more = !ba_check_stop(a, c);  // src/Optimizer.cc:689-692 (bDoMore)
    }
}

// vToErase (src/Optimizer.cc:741-773) + write back (Converter::toCvMat)
__global__ __launch_bounds__(kBaBlock) void k_ba_finish(BaDev a, float* __restrict__ out_tcw,
                                                        float* __restrict__ out_pos,
                                                        unsigned char* __restrict__ out_erase) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const double* T = a.Tb[a.ctl->cur];
    const double* X = a.Xb[a.ctl->cur];
    if (i < a.nedge) {
        const orbmi_ba_edge e = a.edges[i];
        if (!a.pts[e.point].bad) {
            double p[3];
            se3_map(T + 8 * e.kf, X + 4 * e.point, p);
            const double th = edge_stereo(e) ? 7.815 : 5.991;
            out_erase[i] = (edge_chi2(a, i) > th || !(p[2] > 0.0)) ? 1 : 0;
        }
    }
    if (i < a.nkf) {
        const double* Ti = T + 8 * i;
        double R[3][3];
        q_to_matrix(load_q(Ti), R);
        float* o = out_tcw + 16 * i;
        for (int r = 0; r < 3; r++) {
            for (int c = 0; c < 3; c++) o[4 * r + c] = (float)R[r][c];
            o[4 * r + 3] = (float)Ti[4 + r];
        }
        o[12] = 0; o[13] = 0; o[14] = 0; o[15] = 1;
    }
    if (i < a.npt)
        for (int r = 0; r < 3; r++) out_pos[3 * i + r] = (float)X[4 * i + r];
}

}  // namespace orbmi

// ---------------------------------------------------------------- host
struct orbmi_ba {
    int device = 0;
    hipStream_t stream = nullptr;
    bool own_stream = true;  // false after orbmi_ba_set_stream(b, s != NULL)
    hipEvent_t done = nullptr;
    uint8_t* d_buf = nullptr;
    size_t cap = 0;
    uint8_t* h_stage = nullptr;  // pinned staging of the uploaded graph (one H2D copy)
    size_t cap_stage = 0;
    hipEvent_t up_done = nullptr;  // the last upload from h_stage has been read
    uint8_t* h_out = nullptr;      // pinned staging of the results (poses, positions, erase flags)
    size_t cap_out = 0;
    orbmi::BaCtl* h_ctl = nullptr;  // pinned readback of the LM control block
    int* h_stop = nullptr;          // host-mapped mirror of the caller's stop flag
    int* d_stop = nullptr;          //   (its device address)
    int stop_at = -1;               // orbmi_ba_set_stop_at_check
    void (*enqueued)(void*) = nullptr;  // orbmi_ba_set_enqueued_hook
    void* enqueued_arg = nullptr;
};

namespace {

using namespace orbmi;

// ORBMI_BA_TRACE=1: host wall time of the phases of one call on stderr (development aid)
struct BaTrace {
    bool on = getenv("ORBMI_BA_TRACE") != nullptr;
    std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now(), last = t0;
    char buf[512];
    int n = 0;
    void mark(const char* what) {
        if (!on) return;
        const auto t = std::chrono::steady_clock::now();
        n += snprintf(buf + n, sizeof(buf) - n > 0 ? sizeof(buf) - n : 0, " %s %.1f", what,
                      std::chrono::duration<double, std::micro>(t - last).count());
        last = t;
    }
    ~BaTrace() {
        if (on) fprintf(stderr, "[ba] total %.1f us:%s\n",
                        std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count(), buf);
    }
};

// the caller's stop flag (bool* pbStopFlag, src/Optimizer.cc:483), written by other threads:
// read with an atomic load
inline bool stop_set(const volatile int* stop) { return stop && __atomic_load_n(stop, __ATOMIC_ACQUIRE) != 0; }

// The pose-pair blocks' ids.  Pair l = (ra, rb >= ra) in row-major order (l = ra nf - ra (ra - 1)
// / 2 + rb - ra) runs as block blk_id[l] of k_ba_schur.  Placed by row: the blocks of row ra
// (which all read the Hpl blocks of keyframe ra's edges) go to ids of one residue mod 8 -- one XCD
// under the round-robin dispatch, so their re-reads of those blocks hit one L2 (speed only).
// Rows are dealt to the 8 residues largest first onto the least loaded; pairs beyond a residue's
// ids take the ids left over, in increasing order.  rowmajor: blk_id[l] = l (A/B runs).
// Every block id in [0, nblk) must name exactly one pair: an id no pair took would leave its
// blk_kf entry to whatever the pinned staging buffer last held, and the pair kernels index
// pose_idx / kf_start with it (the round-4 r04x illegal address, from a work-in-progress form of
// this table, on the first call that reused a larger graph's staging buffer).  So the table is
// checked before it is used: false = not a permutation (never, by construction; tested for
// every nf by tests/test_capi_exports.py through orbmi_debug_ba_schur_blocks).
bool ba_block_table(int nf, bool rowmajor, std::vector<int>& blk_id) {
    const int nblk = nf * (nf + 1) / 2;
    blk_id.assign(std::max(nblk, 1), -1);
    if (rowmajor) {
        for (int x = 0; x < nblk; x++) blk_id[x] = x;
    } else {
        const int R = 8;
        std::vector<int> load(R, 0), grp(std::max(nf, 1));
        for (int r = 0; r < nf; r++) {  // row r holds nf - r pairs: already largest first
            const int g = (int)(std::min_element(load.begin(), load.end()) - load.begin());
            grp[r] = g;
            load[g] += nf - r;
        }
        std::vector<int> next(R);
        for (int g = 0; g < R; g++) next[g] = g;
        std::vector<char> used(std::max(nblk, 1), 0);
        std::vector<int> spill;
        int l = 0;
        for (int ra = 0; ra < nf; ra++)
            for (int rb = ra; rb < nf; rb++, l++) {
                const int g = grp[ra];
                if (next[g] < nblk) { blk_id[l] = next[g]; used[next[g]] = 1; next[g] += R; }
                else spill.push_back(l);
            }
        int free_id = 0;
        for (int x : spill) {
            while (free_id < nblk && used[free_id]) free_id++;
            if (free_id >= nblk) return false;
            blk_id[x] = free_id;
            used[free_id] = 1;
        }
    }
    std::vector<char> hit(std::max(nblk, 1), 0);
    for (int x = 0; x < nblk; x++) {
        const int id = blk_id[x];
        if (id < 0 || id >= nblk || hit[id]) return false;
        hit[id] = 1;
    }
    return true;
}

// Trial steps enqueued beyond the iterations still to run: a rejected trial consumes one step
// without finishing an iteration, so the steps enqueued up front usually finish optimize().
constexpr int kBaStepSlack = 1;

// The whole g2o schedule -- optimize(5), levels, optimize(10), write-back -- is enqueued at once
// and read back once: every kernel checks on the device that its optimize() is the current one
// (BaCtl::gen, phases_done), so launches past an optimize() that ran out of enqueued trials do
// nothing, and the host resumes from there (more trials, then the rest of the schedule).
struct Runner {
    orbmi_ba& h;
    BaDev a;
    const volatile int* stop;
    bool solve_rows;  // nf <= kBaSolveRowsMaxPoses: k_ba_solve_rows, else k_ba_solve<1>
    bool solve_pipe;  // k_ba_solve_pipe (a dedicated pivot wave) in place of k_ba_solve_rows
                      // (ORBMI_BA_SOLVE=rows selects the latter, for A/B runs)
    int mfma_tiles;   // > 0: k_ba_solve_mfma<mfma_tiles> (nf <= kBaSolveMfmaMaxPoses, the default)

    bool fuse_schur = false;  // k_ba_schur_solve (ORBMI_BA_FUSE=1; measured slower than two launches)
    void launch_mfma() {
        const dim3 gs(a.nblk + kSchurKfSplit * a.nf + 1);
        switch (mfma_tiles) {
#define ORBMI_MFMA_CASE(T_)                                                                                      \
    case T_:                                                                                                     \
        if (fuse_schur) hipLaunchKernelGGL(k_ba_schur_solve<T_>, gs, dim3(kSchurThreads), 0, h.stream, a);       \
        else hipLaunchKernelGGL(k_ba_solve_mfma<T_>, dim3(1), dim3(kBaMfmaThreads), 0, h.stream, a);             \
        break;
            ORBMI_MFMA_CASE(1) ORBMI_MFMA_CASE(2) ORBMI_MFMA_CASE(3) ORBMI_MFMA_CASE(4)
            ORBMI_MFMA_CASE(5) ORBMI_MFMA_CASE(6) ORBMI_MFMA_CASE(7) ORBMI_MFMA_CASE(8)
#undef ORBMI_MFMA_CASE
            default: break;
        }
    }

    // wait for the stream; meanwhile mirror the caller's stop flag to the device, yielding the
    // core between polls (the caller's other threads, e.g. tracking, run on the host meanwhile)
    int wait() {
        ORBMI_HIP(hipEventRecord(h.done, h.stream));
        if (!stop) {
            ORBMI_HIP(hipEventSynchronize(h.done));
            return ORBMI_OK;
        }
        for (;;) {
            *(volatile int*)h.h_stop = stop_set(stop) ? 1 : 0;
            const hipError_t e = hipEventQuery(h.done);
            if (e == hipSuccess) return ORBMI_OK;
            if (e != hipErrorNotReady) return ORBMI_E_HIP;
            std::this_thread::yield();
        }
    }

    int read_ctl() {
        ORBMI_HIP(hipMemcpyAsync(h.h_ctl, a.ctl, sizeof(BaCtl), hipMemcpyDeviceToHost, h.stream));
        return wait();
    }

    // one LM trial of optimize() gen: Schur + solve + update (trial errors, the trial state's
    // linearisation and, in its last block, the Levenberg decision); every kernel returns at once
    // when that optimize() is done or not the current one
    void step(int gen) {
        a.run_gen = gen;
        if (a.nblk > 0 && !(mfma_tiles > 0 && fuse_schur))  // (+ the MFMA solve's padding block)
            hipLaunchKernelGGL(k_ba_schur, dim3(a.nblk + kSchurKfSplit * a.nf + (a.mfma_T > 0)), dim3(kSchurThreads), 0,
                               h.stream, a);
        if (mfma_tiles > 0)
            launch_mfma();
        else if (solve_rows && solve_pipe)
            hipLaunchKernelGGL(k_ba_solve_pipe, dim3(1), dim3(kBaSolvePipeThreads), 0, h.stream, a);
        else if (solve_rows) hipLaunchKernelGGL(k_ba_solve_rows, dim3(1), dim3(kBaSolveRowsThreads), 0, h.stream, a);
        else hipLaunchKernelGGL(k_ba_solve<1>, dim3(1), dim3(kBaSolveThreads), 0, h.stream, a);
        hipLaunchKernelGGL(k_ba_update_errors, dim3(a.nb_q), dim3(kBaUpdThreads), 0, h.stream, a);
    }

    // SparseOptimizer::initializeOptimization + the first linearisation of optimize() gen
    void prologue(int iterations, int gen) {
        a.run_gen = gen;
        if (gen == 2) hipLaunchKernelGGL(k_ba_levels, dim3(a.nb_e), dim3(kBaBlock), 0, h.stream, a);  // :694-737
        hipLaunchKernelGGL(k_ba_activate_edges, dim3(a.nb_e), dim3(kBaBlock), 0, h.stream, a, iterations, gen);
        // iteration 0's computeActiveErrors + buildSystem (later ones come with the trials)
        hipLaunchKernelGGL(k_ba_linearize, dim3(a.nb_e), dim3(kBaBlock), 0, h.stream, a);
        hipLaunchKernelGGL(k_ba_reduce, dim3(a.nb_p + std::max(a.nf, 1)), dim3(kBaBlock), 0, h.stream, a);
    }

    // activeRobustChi2 after optimize() gen
    void epilogue(int gen) {
        a.run_gen = gen;
        hipLaunchKernelGGL(k_ba_errors, dim3(a.nb_e), dim3(kBaBlock), 0, h.stream, a, gen - 1);
    }
};

}  // namespace

extern "C" {

int orbmi_ba_create(int device, orbmi_ba** out) {
    if (!out) return ORBMI_E_ARG;
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return ORBMI_E_HIP;
    orbmi_ba* b = new (std::nothrow) orbmi_ba();
    if (!b) return ORBMI_E_ARG;
    b->device = device;
    if (hipSetDevice(device) != hipSuccess || orbmi::stream_create(&b->stream, "BA") != hipSuccess ||
        hipEventCreateWithFlags(&b->done, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&b->up_done, hipEventDisableTiming) != hipSuccess ||
        hipHostMalloc((void**)&b->h_ctl, sizeof(BaCtl)) != hipSuccess ||
        hipHostMalloc((void**)&b->h_stop, 64, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
        hipHostGetDevicePointer((void**)&b->d_stop, b->h_stop, 0) != hipSuccess) {
        orbmi_ba_destroy(b);
        return ORBMI_E_HIP;
    }
    *b->h_stop = 0;
    *out = b;
    return ORBMI_OK;
}

void orbmi_ba_destroy(orbmi_ba* b) {
    if (!b) return;
    (void)hipSetDevice(b->device);
    if (b->stream) (void)hipStreamSynchronize(b->stream);
    if (b->d_buf) (void)hipFree(b->d_buf);
    if (b->h_stage) (void)hipHostFree(b->h_stage);
    if (b->h_ctl) (void)hipHostFree(b->h_ctl);
    if (b->h_stop) (void)hipHostFree(b->h_stop);
    if (b->done) (void)hipEventDestroy(b->done);
    if (b->up_done) (void)hipEventDestroy(b->up_done);
    if (b->h_out) (void)hipHostFree(b->h_out);
    if (b->stream && b->own_stream) (void)hipStreamDestroy(b->stream);
    delete b;
}

int orbmi_debug_ba_schur_blocks(int nf, int* table, int cap, int* n_out) {
    if (nf < 0 || nf > kBaMaxPoses || !n_out) return ORBMI_E_ARG;
    const int nblk = nf * (nf + 1) / 2, nb = nblk + kSchurKfSplit * nf + 1;
    *n_out = nb;
    if (cap < nb || !table) return ORBMI_E_CAP;
    std::vector<int> blk_id;
    if (!ba_block_table(nf, false, blk_id)) return ORBMI_E_UNSUPPORTED;
    std::vector<int> ra_of(std::max(nblk, 1)), rb_of(std::max(nblk, 1)), l_of(std::max(nblk, 1));
    for (int ra = 0, l = 0; ra < nf; ra++)
        for (int rb = ra; rb < nf; rb++, l++) { ra_of[blk_id[l]] = ra; rb_of[blk_id[l]] = rb; l_of[blk_id[l]] = l; }
    for (int b = 0; b < nb; b++) {
        const SchurRole role = schur_role(b, nblk, nf);
        int* t = table + 4 * b;
        t[0] = role.kind;
        t[1] = role.kind == 0 ? ra_of[role.r] : role.kind == 1 ? role.r : -1;
        t[2] = role.kind == 0 ? rb_of[role.r] : role.kind == 1 ? role.h : -1;
        t[3] = role.kind == 0 ? l_of[role.r] : -1;
    }
    return ORBMI_OK;
}

int orbmi_ba_set_stop_at_check(orbmi_ba* b, int k) {
    if (!b) return ORBMI_E_ARG;
    b->stop_at = k < 0 ? -1 : k;
    return ORBMI_OK;
}

int orbmi_ba_set_enqueued_hook(orbmi_ba* b, void (*fn)(void*), void* arg) {
    if (!b) return ORBMI_E_ARG;
    b->enqueued = fn;
    b->enqueued_arg = arg;
    return ORBMI_OK;
}

int orbmi_ba_set_stream(orbmi_ba* b, void* stream) {
    if (!b) return ORBMI_E_ARG;
    ORBMI_HIP(hipSetDevice(b->device));
    ORBMI_HIP(hipStreamSynchronize(b->stream));
    hipStream_t s = (hipStream_t)stream;
    if (!s) ORBMI_HIP(orbmi::stream_create(&s, "BA"));
    if (b->own_stream) ORBMI_HIP(hipStreamDestroy(b->stream));
    b->stream = s;
    b->own_stream = stream == nullptr;
    return ORBMI_OK;
}

int orbmi_local_bundle_adjustment(orbmi_ba* b, const orbmi_ba_problem* P, orbmi_ba_result* R,
                                  const volatile int* stop) {
    if (!b || !P || !R || P->nkf < 0 || P->npt < 0 || P->nedge < 0) return ORBMI_E_ARG;
    if ((P->nkf && (!P->kfs || !R->tcw)) || (P->npt && (!P->pts || !R->pos)) || (P->nedge && (!P->edges || !R->erase)))
        return ORBMI_E_ARG;
    orbmi_ba& h = *b;
    BaTrace tr;
    ORBMI_HIP(hipSetDevice(h.device));
    R->aborted = 0;
    R->iterations[0] = R->iterations[1] = 0;
    R->chi2[0] = R->chi2[1] = 0;
    R->stop_check = -1;
    R->checks = 1;
    for (int i = 0; i < P->nedge; i++) R->erase[i] = 0;
    if (stop_set(stop) || h.stop_at == 0) {  // check #0, src/Optimizer.cc:685-687
        R->aborted = 1;
        R->stop_check = 0;
        return ORBMI_OK;
    }
    const int nkf = P->nkf, npt = P->npt, ne = P->nedge;
    if (nkf > kBaMaxKf) return ORBMI_E_UNSUPPORTED;
    // host-side graph indexing: edges grouped by point (the reference inserts them point by
    // point), CSR by keyframe, keyframes ordered by id (SparseOptimizer vertex order).  The index
    // arrays are written straight into the pinned staging buffer that goes up in one copy.
    {
        // one edge per (point, keyframe), as the reference builds the graph from a map point's
        // observations (a std::map per point): the per-keyframe Schur blocks sum each edge's
        // B D^-1 B^T with itself only, so a second edge of one pair would lose its cross terms
        std::vector<int> last_pt(std::max(nkf, 1), -1);
        for (int i = 0; i < ne; i++) {
            const orbmi_ba_edge& e = P->edges[i];
            if (e.point < 0 || e.point >= npt || e.kf < 0 || e.kf >= nkf) return ORBMI_E_ARG;
            if (i && e.point < P->edges[i - 1].point) return ORBMI_E_ARG;
            if (last_pt[e.kf] == e.point) return ORBMI_E_ARG;  // (edges come grouped by point)
            last_pt[e.kf] = e.point;
        }
    }
    std::vector<int> order(std::max(nkf, 1));
    for (int k = 0; k < nkf; k++) order[k] = k;
    std::stable_sort(order.begin(), order.begin() + nkf, [&](int x, int y) { return P->kfs[x].id < P->kfs[y].id; });
    // Schur pair lists: blocks = pairs of non-fixed keyframes (a, b) with rank(a) <= rank(b)
    // in id order; pairs (e_a, e_b) = two observations of one point (both orders inside a
    // keyframe).  Pose indices follow the same order, so block (a, b) is (i <= j).
    std::vector<int> rank(std::max(nkf, 1), -1), free_kf;
    for (int oi = 0; oi < nkf; oi++)
        if (!P->kfs[order[oi]].fixed) { rank[order[oi]] = (int)free_kf.size(); free_kf.push_back(order[oi]); }
    const int nf = (int)free_kf.size();
    const long long nblk_ll = (long long)nf * (nf + 1) / 2;
    if (nblk_ll > (1 << 20)) return ORBMI_E_UNSUPPORTED;
    const int nblk = (int)nblk_ll;
    std::vector<int> blk_id;
    if (!ba_block_table(nf, getenv("ORBMI_BA_SCHUR_ROWMAJOR") != nullptr, blk_id)) return ORBMI_E_UNSUPPORTED;
    auto blk_of = [nf, &blk_id](int ra, int rb) { return blk_id[ra * nf - ra * (ra - 1) / 2 + (rb - ra)]; };
    // ---- one device arena; the graph and its index arrays go up in one copy
    const int nb_e = std::max(1, (ne + kBaBlock - 1) / kBaBlock), nb_p = std::max(1, (npt + kBaBlock - 1) / kBaBlock);
    const int nb_q = std::max(1, (npt + kBaUpdPts - 1) / kBaUpdPts);
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    size_t off = 0;
    auto take = [&](size_t bytes) { size_t o = off; off += al(std::max(bytes, (size_t)8)); return o; };
    // uploaded region first (contiguous)
    const size_t o_kfs = take(sizeof(orbmi_ba_keyframe) * nkf), o_pts = take(sizeof(orbmi_ba_point) * npt),
                 o_edges = take(sizeof(orbmi_ba_edge) * ne), o_order = take(4 * nkf), o_pts_start = take(4 * (npt + 1)),
                 o_kfs_start = take(4 * (nkf + 1)), o_kf_edges = take(4 * (size_t)ne), o_kf_pos = take(4 * (size_t)ne),
                 o_kf_pt = take(4 * (size_t)ne), o_blk_kf = take(8 * (size_t)nblk), o_free = take(4 * (size_t)nf);
    const size_t up_bytes = off;
    hipStream_t s = h.stream;
    // the previous call's upload may still be reading the staging buffer (only that copy is
    // waited for: the stream's other work, e.g. the searches enqueued before this call on a
    // shared stream, keeps running while the graph is indexed)
    ORBMI_HIP(hipEventSynchronize(h.up_done));
    if (up_bytes > h.cap_stage) {
        if (h.h_stage) (void)hipHostFree(h.h_stage);
        h.h_stage = nullptr;
        h.cap_stage = 0;
        ORBMI_HIP(hipHostMalloc((void**)&h.h_stage, up_bytes));
        h.cap_stage = up_bytes;
    }
    uint8_t* S = h.h_stage;
    int* pt_start = (int*)(S + o_pts_start);
    int* kf_start = (int*)(S + o_kfs_start);
    int* kf_edges = (int*)(S + o_kf_edges);
    int* kf_pos = (int*)(S + o_kf_pos);
    int* kf_pt = (int*)(S + o_kf_pt);
    std::memset(pt_start, 0, 4 * (size_t)(npt + 1));
    std::memset(kf_start, 0, 4 * (size_t)(nkf + 1));
    for (int i = 0; i < ne; i++) { pt_start[P->edges[i].point + 1]++; kf_start[P->edges[i].kf + 1]++; }
    for (int p = 0; p < npt; p++) pt_start[p + 1] += pt_start[p];
    for (int k = 0; k < nkf; k++) kf_start[k + 1] += kf_start[k];
    // capacity of the pair lists (built on the device): sum over points of (free edges)^2
    long long npair_cap = 0;
    {
        std::vector<int> fill(kf_start, kf_start + nkf);
        int p = -1;
        long long m = 0;
        for (int i = 0; i < ne; i++) {
            const orbmi_ba_edge& e = P->edges[i];
            const int j = fill[e.kf]++;
            kf_pos[i] = j;
            kf_edges[j] = i;
            kf_pt[j] = e.point;
            if (e.point != p) { npair_cap += m * m; m = 0; p = e.point; }
            m += rank[e.kf] >= 0;
        }
        npair_cap += m * m;
    }
    if (npair_cap > (1LL << 28)) return ORBMI_E_UNSUPPORTED;
    const int npair = (int)npair_cap;
    if (nkf) std::memcpy(S + o_order, order.data(), 4 * (size_t)nkf);
    if (nf) std::memcpy(S + o_free, free_kf.data(), 4 * (size_t)nf);
    {
        int* bk = (int*)(S + o_blk_kf);
        for (int ra = 0; ra < nf; ra++)
            for (int rb = ra; rb < nf; rb++) { bk[2 * blk_of(ra, rb)] = free_kf[ra]; bk[2 * blk_of(ra, rb) + 1] = free_kf[rb]; }
    }
    auto put = [&](size_t o, const void* src, size_t bytes) { if (bytes) std::memcpy(S + o, src, bytes); };
    put(o_kfs, P->kfs, sizeof(orbmi_ba_keyframe) * nkf);
    put(o_pts, P->pts, sizeof(orbmi_ba_point) * npt);
    put(o_edges, P->edges, sizeof(orbmi_ba_edge) * ne);
    const size_t o_blk_cnt = take(4 * (size_t)nblk), o_blk_start = take(4 * ((size_t)nblk + 1)),
                 o_pairs = take(8 * (size_t)npair), o_pairpt = take(4 * (size_t)npair);
    const size_t o_e_pi = take(4 * (size_t)ne), o_T0 = take(64 * nkf), o_T1 = take(64 * nkf), o_X0 = take(32 * npt),
                 o_X1 = take(32 * npt), o_err = take(24 * (size_t)ne), o_eflag = take(ne), o_pidx = take(4 * nkf), o_kfact = take(4 * nkf),
                 o_pkf = take(4 * kBaMaxPoses), o_Hpl = take(2 * 144 * (size_t)ne), o_Hle = take(2 * 72 * (size_t)ne),
                 o_Hpe = take(2 * 216 * (size_t)ne), o_Hll = take(2 * 72 * npt), o_bl = take(2 * 24 * npt),
                 o_Hpp = take(288 * kBaMaxPoses), o_bp = take(48 * kBaMaxPoses), o_S = take(8 * (size_t)kBaPacked),
                 o_bs = take(8 * kBaMaxN), o_xp = take(8 * kBaMaxN), o_scal = take(64), o_plin = take(8 * (size_t)nb_e),
                 o_ptchi = take(8 * (size_t)nb_q), o_ptsc = take(8 * (size_t)nb_q),
                 o_pmax = take(8 * ((size_t)nb_p + kBaMaxPoses)), o_istat = take(32), o_ctl = take(sizeof(BaCtl)),
                 o_otcw = take(64 * nkf), o_opos = take(12 * npt), o_oerase = take(ne),
                 o_pkfs = take(8 * 64 * kSchurKfSplit * (size_t)kBaMaxPoses), o_arrkf = take(4 * kBaMaxPoses);
    if (off > h.cap) {
        if (h.d_buf) (void)hipFree(h.d_buf);
        h.d_buf = nullptr;
        h.cap = 0;
        ORBMI_HIP(hipMalloc((void**)&h.d_buf, off));
        h.cap = off;
    }
    uint8_t* B = h.d_buf;
    tr.mark("host_index");
    ORBMI_HIP(hipMemcpyAsync(B, S, up_bytes, hipMemcpyHostToDevice, s));
    ORBMI_HIP(hipEventRecord(h.up_done, s));
    const size_t out_bytes = o_oerase + (size_t)std::max(ne, 1) - o_otcw;  // tcw, pos, erase (aligned)
    if (out_bytes > h.cap_out) {
        if (h.h_out) (void)hipHostFree(h.h_out);
        h.h_out = nullptr;
        h.cap_out = 0;
        ORBMI_HIP(hipHostMalloc((void**)&h.h_out, out_bytes));
        h.cap_out = out_bytes;
    }
    uint8_t* const Ho = h.h_out;
    BaDev a;
    a.nkf = nkf; a.npt = npt; a.nedge = ne; a.nblk = nblk; a.nf = nf;
    a.nb_e = nb_e; a.nb_p = nb_p; a.nb_q = nb_q;
    a.ctl = (BaCtl*)(B + o_ctl);
    a.stop = stop ? h.d_stop : nullptr;
    a.stop_at = h.stop_at;
    // the mirror starts with the flag's value now; Runner::wait keeps it current (the device reads
    // it only at the checks)
    *(volatile int*)h.h_stop = stop_set(stop) ? 1 : 0;
    a.Tb[0] = (double*)(B + o_T0); a.Tb[1] = (double*)(B + o_T1);
    a.Xb[0] = (double*)(B + o_X0); a.Xb[1] = (double*)(B + o_X1);
    a.part_lin = (double*)(B + o_plin); a.part_tchi = (double*)(B + o_ptchi); a.part_tscale = (double*)(B + o_ptsc);
    a.part_max = (double*)(B + o_pmax);
    a.kfs = (const orbmi_ba_keyframe*)(B + o_kfs);
    a.pts = (const orbmi_ba_point*)(B + o_pts);
    a.edges = (const orbmi_ba_edge*)(B + o_edges);
    a.kf_order = (const int*)(B + o_order);
    a.free_kf = (const int*)(B + o_free);
    a.part_kf = (double*)(B + o_pkfs);
    a.arrive_kf = (unsigned*)(B + o_arrkf);
    a.pt_start = (const int*)(B + o_pts_start);
    a.kf_start = (const int*)(B + o_kfs_start);
    a.kf_edges = (const int*)(B + o_kf_edges);
    a.kf_pos = (const int*)(B + o_kf_pos);
    a.kf_pt = (const int*)(B + o_kf_pt);
    a.e_pi = (int*)(B + o_e_pi);
    a.blk_kf = (const int*)(B + o_blk_kf);
    a.blk_cnt = (int*)(B + o_blk_cnt);
    a.blk_start = (int*)(B + o_blk_start);
    a.blk_pairs = (int2*)(B + o_pairs);
    a.blk_pt = (int*)(B + o_pairpt);
    a.err = (double*)(B + o_err); a.eflag = B + o_eflag;
    a.pose_idx = (int*)(B + o_pidx); a.pose_kf = (int*)(B + o_pkf); a.kf_act = (int*)(B + o_kfact);
    for (int L = 0; L < 2; L++) {  // two linear-system buffers (ctl.lin selects the current one)
        a.Hplb[L] = (double*)(B + o_Hpl) + (size_t)L * 18 * ne;
        a.Hleb[L] = (double*)(B + o_Hle) + (size_t)L * 9 * ne;
        a.Hpeb[L] = (double*)(B + o_Hpe) + (size_t)L * 27 * ne;
        a.Hllb[L] = (double*)(B + o_Hll) + (size_t)L * 9 * npt;
        a.blb[L] = (double*)(B + o_bl) + (size_t)L * 3 * npt;
    }
    a.Hpl = a.Hplb[0]; a.Hle = a.Hleb[0]; a.Hpe = a.Hpeb[0]; a.Hll = a.Hllb[0]; a.bl = a.blb[0];
    a.Hpp = (double*)(B + o_Hpp); a.bp = (double*)(B + o_bp);
    a.S = (double*)(B + o_S); a.bs = (double*)(B + o_bs); a.xp = (double*)(B + o_xp);
    a.scal = (double*)(B + o_scal); a.istat = (int*)(B + o_istat);
    const char* sv = getenv("ORBMI_BA_SOLVE");
    // the MFMA solve for nf <= kBaSolveMfmaMaxPoses (ORBMI_BA_SOLVE=pipe / rows: the VALU solves)
    const bool valu_solve = sv && (!strcmp(sv, "pipe") || !strcmp(sv, "rows"));
    a.mfma_T = (!valu_solve && nf <= kBaSolveMfmaMaxPoses) ? std::max(1, (6 * nf + 15) / 16) : 0;
    Runner r{h, a, stop, nf <= kBaSolveRowsMaxPoses, !(sv && !strcmp(sv, "rows")), a.mfma_T};
    {
        const char* fz = getenv("ORBMI_BA_FUSE");
        r.fuse_schur = fz && !strcmp(fz, "1");
    }
    unsigned char* out_erase = B + o_oerase;
    const int nb_all = std::max(1, (std::max(std::max(nkf, npt), ne) + kBaBlock - 1) / kBaBlock);
    hipLaunchKernelGGL(k_ba_setup, dim3(nb_all), dim3(kBaBlock), 0, s, a, a.Tb[0], a.Xb[0], out_erase);
    if (nblk > 0) {
        hipLaunchKernelGGL(k_ba_pairs_count, dim3(nblk), dim3(kPairThreads), 0, s, a);
        hipLaunchKernelGGL(k_ba_pairs_fill, dim3(nblk), dim3(kPairThreads), 0, s, a);
    }
    ORBMI_HIP(hipGetLastError());
    tr.mark("enqueue_setup");
    // optimize(5), levels, optimize(10), write-back, enqueued at once (stages from `from` on:
    // 0 = optimize(5)'s prologue, 1 = more trials of optimize(5), 2 = more trials of optimize(10))
    const char* slack_env = getenv("ORBMI_BA_SLACK");  // test hook: 0 forces the resume path
    const int slack = slack_env ? std::max(0, atoi(slack_env)) : kBaStepSlack;
    auto enqueue = [&](int from, int more) {
        if (from == 0) r.prologue(5, 1);
        if (from <= 1) {
            for (int k = 0; k < (from == 0 ? 5 + slack : more); k++) r.step(1);
            r.epilogue(1);
            r.prologue(10, 2);
        }
        for (int k = 0; k < (from <= 1 ? 10 + slack : more); k++) r.step(2);
        r.epilogue(2);
        hipLaunchKernelGGL(k_ba_finish, dim3(nb_all), dim3(kBaBlock), 0, s, a, (float*)(B + o_otcw), (float*)(B + o_opos),
                           out_erase);
        hipError_t e = hipSuccess;
        // the outputs are contiguous in the arena (tcw, pos, erase): one copy into pinned memory
        if (e == hipSuccess) e = hipMemcpyAsync(Ho, B + o_otcw, o_oerase + ne - o_otcw, hipMemcpyDeviceToHost, s);
        return e;
    };
    int rc, from = 0, more = 0;
    for (;;) {
        ORBMI_HIP(enqueue(from, more));
        ORBMI_HIP(hipGetLastError());
        if (from == 0 && h.enqueued) h.enqueued(h.enqueued_arg);  // the caller's work beside the solve
        if ((rc = r.read_ctl())) return rc;
        const BaCtl& c = *h.h_ctl;
        if (c.unsupported) return ORBMI_E_UNSUPPORTED;
        if (c.phases_done >= 2 || (c.phases_done == 1 && !c.do_more)) break;
        // an optimize() ran out of enqueued trials (rejections beyond the slack): resume it
        from = c.phases_done == 0 ? 1 : 2;
        more = std::max(1, c.max_it - c.it);
        tr.mark(from == 1 ? "resume5" : "resume10");
    }
    tr.mark("optimize+finish");
    if (nkf) std::memcpy(R->tcw, Ho, 64 * (size_t)nkf);
    if (npt) std::memcpy(R->pos, Ho + (o_opos - o_otcw), 12 * (size_t)npt);
    if (ne) std::memcpy(R->erase, Ho + (o_oerase - o_otcw), (size_t)ne);
    const BaCtl& c = *h.h_ctl;
    const bool second = c.do_more != 0;
    R->iterations[0] = c.it_out[0];
    R->iterations[1] = second ? c.it_out[1] : 0;
    R->chi2[0] = c.chi_out[0];
    R->chi2[1] = second ? c.chi_out[1] : 0;
    R->stop_check = c.stop_seen;
    R->checks = c.checks;
    return ORBMI_OK;
}

}  // extern "C"
