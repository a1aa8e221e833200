// ORACLE — test infrastructure only (see orb_oracle.h).
// Optimizer::PoseOptimization (src/Optimizer.cc:257-481) restated with the vendored g2o's
// semantics, sequential fp64:
//   EdgeSE3ProjectXYZOnlyPose / EdgeStereoSE3ProjectXYZOnlyPose
//                      types/types_six_dof_expmap.h:142-205, .cpp:266-364 (float invz in the
//                      stereo cam_project, invz / invz^2 products in the Jacobians)
//   BaseUnaryEdge::constructQuadraticForm       core/base_unary_edge.hpp:43-75
//   RobustKernelHuber::robustify                core/robust_kernel_impl.cpp:78-91
//   OptimizationAlgorithmLevenberg::solve       core/optimization_algorithm_levenberg.cpp:61-189
//                      (incl. ORB-SLAM2's 3-bad-iterations stop)
//   BlockSolver_6_3 + LinearSolverDense         solvers/linear_solver_dense.h:65-110 (one 6x6
//                      pose block; a dense LDL^T stands in for Eigen's LDLT: rounding only)
// Stale-error rule: the classification after each optimize(10) reads chi2() of the errors
// from the LM's last computeActiveErrors (a rejected trial leaves its errors behind).
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <limits>
#include <vector>

#include "../include/orbmi.h"
#include "g2o_oracle.h"

namespace {

using namespace g2o_oracle;

// Parity diagnostics for tests/test_pose_gpu.py (orc_pose_set_diag): the float chi2 each
// observation was classified with in each of the 4 rounds (round-major, n_obs per round, NaN
// where a round did not run), and per round the smallest relative distance
// |(iniChi - currentChi) * 1e3 - iniChi| / iniChi of the 3-bad-iterations stop test
// (optimization_algorithm_levenberg.cpp:154-161) over the round's iterations, then per round the
// smallest |currentChi - tempChi| / currentChi over its trials (how close an accept / reject
// decision came to a tie: converged rounds decide on rounding noise, and 10 rejections in a row
// end the optimisation, :163).  Null = off.
thread_local float* g_diag_chi2 = nullptr;
thread_local double* g_diag_stop = nullptr;

struct UEdge {
    double Xw[3];
    double obs[3];
    bool stereo;
    double info;
    double delta, dsqr;
    bool robust = true;
    int level = 0;
    double err[3] = {0, 0, 0};
};

struct Cam { double fx, fy, cx, cy, bf; };

void compute_error(const SE3& T, const Cam& c, UEdge& e) {
    double p[3];
    se3_map(T, e.Xw, p);
    if (!e.stereo) {  // obs - cam_project(project2d(p))
        const double px = p[0] / p[2], py = p[1] / p[2];
        e.err[0] = e.obs[0] - (px * c.fx + c.cx);
        e.err[1] = e.obs[1] - (py * c.fy + c.cy);
        e.err[2] = 0;
    } else {
        const float invz = (float)(1.0f / p[2]);
        const double r0 = p[0] * invz * c.fx + c.cx;
        const double r1 = p[1] * invz * c.fy + c.cy;
        const double r2 = r0 - c.bf * invz;
        e.err[0] = e.obs[0] - r0;
        e.err[1] = e.obs[1] - r1;
        e.err[2] = e.obs[2] - r2;
    }
}

double chi2(const UEdge& e) {
    const int d = e.stereo ? 3 : 2;
    double s = 0;
    for (int i = 0; i < d; i++) s += e.err[i] * (e.info * e.err[i]);
    return s;
}

void robustify(const UEdge& e, double c, double rho[3]) {
    if (c <= e.dsqr) { rho[0] = c; rho[1] = 1.; rho[2] = 0.; }
    else {
        const double s = std::sqrt(c);
        rho[0] = 2 * s * e.delta - e.dsqr;
        rho[1] = e.delta / s;
        rho[2] = -0.5 * rho[1] / c;
    }
}

void jacobian(const SE3& T, const Cam& c, const UEdge& e, double J[3][6]) {  // linearizeOplus
    double p[3];
    se3_map(T, e.Xw, p);
    const double x = p[0], y = p[1], invz = 1.0 / p[2], invz_2 = invz * invz;
    J[0][0] = x * y * invz_2 * c.fx; J[0][1] = -(1 + (x * x * invz_2)) * c.fx; J[0][2] = y * invz * c.fx;
    J[0][3] = -invz * c.fx; J[0][4] = 0; J[0][5] = x * invz_2 * c.fx;
    J[1][0] = (1 + y * y * invz_2) * c.fy; J[1][1] = -x * y * invz_2 * c.fy; J[1][2] = -x * invz * c.fy;
    J[1][3] = 0; J[1][4] = -invz * c.fy; J[1][5] = y * invz_2 * c.fy;
    if (e.stereo) {
        J[2][0] = J[0][0] - c.bf * y * invz_2; J[2][1] = J[0][1] + c.bf * x * invz_2; J[2][2] = J[0][2];
        J[2][3] = J[0][3]; J[2][4] = 0; J[2][5] = J[0][5] - c.bf * invz_2;
    } else {
        for (int k = 0; k < 6; k++) J[2][k] = 0;
    }
}

struct PoseOpt {
    SE3 T;
    Cam cam;
    std::vector<UEdge>& E;
    std::vector<int> active;
    double H[36], b[6], x[6];
    double lambda = 0, ni = 2;
    int nBad = 0;
    int iters = 0;
    double* stop_margin = nullptr;

    explicit PoseOpt(std::vector<UEdge>& e) : E(e) {}

    void compute_active_errors() {
        for (int i : active) compute_error(T, cam, E[i]);
    }
    double active_robust_chi2() const {
        double s = 0;
        for (int i : active) {
            const double c = chi2(E[i]);
            if (E[i].robust) { double rho[3]; robustify(E[i], c, rho); s += rho[0]; }
            else s += c;
        }
        return s;
    }
    void build_system() {
        for (double& v : H) v = 0;
        for (double& v : b) v = 0;
        for (int i : active) {
            const UEdge& e = E[i];
            const int D = e.stereo ? 3 : 2;
            double J[3][6];
            jacobian(T, cam, e, J);
            double w = e.info, s = 1.0;
            if (e.robust) { double rho[3]; robustify(e, chi2(e), rho); w = rho[1] * e.info; s = rho[1]; }
            for (int r = 0; r < 6; r++) {
                double br = 0;
                for (int k = 0; k < D; k++) br += J[k][r] * (e.info * e.err[k]);
                b[r] -= s * br;
                for (int c = 0; c < 6; c++) {
                    double h = 0;
                    for (int k = 0; k < D; k++) h += J[k][r] * w * J[k][c];
                    H[r * 6 + c] += h;
                }
            }
        }
    }
    bool solve(double lam) {
        std::vector<double> A(H, H + 36), bb(b, b + 6);
        for (int j = 0; j < 6; j++) A[j * 7] += lam;
        if (!ldlt_solve(A, 6, bb)) return false;
        for (int j = 0; j < 6; j++) x[j] = bb[j];
        return true;
    }
    double compute_scale() const {
        double s = 0;
        for (int j = 0; j < 6; j++) s += x[j] * (lambda * x[j] + b[j]);
        return s;
    }
    // ORC_POSE_TRACE=1: the accept (A) / reject (R) sequence of the trials on stderr, '|' per
    // iteration (a measurement aid for the device kernel's trial schedule)
    static bool trace_trials() {
        static const bool on = std::getenv("ORC_POSE_TRACE") != nullptr;
        return on;
    }
    enum Result { OK, Terminate };
    Result lm_solve(int iteration) {  // OptimizationAlgorithmLevenberg::solve
        compute_active_errors();
        double currentChi = active_robust_chi2();
        const double iniChi = currentChi;
        build_system();
        if (iteration == 0) {
            double m = 0;
            for (int j = 0; j < 6; j++) m = std::max(m, std::fabs(H[j * 7]));
            lambda = 1e-5 * m;
            ni = 2;
            nBad = 0;
        }
        double rho = 0;
        int qmax = 0;
        do {
            const SE3 T0 = T;
            const bool ok2 = solve(lambda);
            if (ok2) T = se3_mul(se3_exp(x), T);
            else for (double& v : x) v = 0;
            compute_active_errors();
            double tempChi = active_robust_chi2();
            if (!ok2) tempChi = std::numeric_limits<double>::max();
            rho = (currentChi - tempChi) / (compute_scale() + 1e-3);
            if (stop_margin && currentChi > 0 && ok2)
                stop_margin[4] = std::min(stop_margin[4], std::fabs(currentChi - tempChi) / currentChi);
            if (rho > 0 && std::isfinite(tempChi)) {
                double alpha = 1. - std::pow((2 * rho - 1), 3);
                alpha = std::min(alpha, 2. / 3.);
                lambda *= std::max(1. / 3., alpha);
                ni = 2;
                currentChi = tempChi;
            } else {
                lambda *= ni;
                ni *= 2;
                T = T0;
            }
            qmax++;
            if (trace_trials()) std::fputc(rho > 0 && std::isfinite(tempChi) ? 'A' : 'R', stderr);
        } while (rho < 0 && qmax < 10);
        if (trace_trials()) std::fputc('|', stderr);
        if (qmax == 10 || rho == 0) return Terminate;
        if (stop_margin && iniChi > 0)
            *stop_margin = std::min(*stop_margin, std::fabs((iniChi - currentChi) * 1e3 - iniChi) / iniChi);
        if ((iniChi - currentChi) * 1e3 < iniChi) nBad++;
        else nBad = 0;
        return nBad >= 3 ? Terminate : OK;
    }
    void optimize(int iterations) {  // SparseOptimizer::optimize on the level-0 edges
        active.clear();
        for (int i = 0; i < (int)E.size(); i++)
            if (E[i].level == 0) active.push_back(i);
        if (active.empty()) return;  // no active vertex: nothing is optimised
        for (int i = 0; i < iterations; i++) {
            const Result r = lm_solve(i);
            iters++;
            if (r != OK) break;
        }
    }
};

}  // namespace

// One frame; `outlier` receives mvbOutlier of every observation.  Returns the inlier count.
extern "C" int orc_pose_optimization(orbmi_pose_frame* f, const orbmi_pose_obs* obs, uint8_t* outlier) {
    const int n = f->n_obs;
    const float deltaMono = std::sqrt(5.991f), deltaStereo = std::sqrt(7.815f);  // :290-291
    std::vector<UEdge> E(n);
    for (int k = 0; k < n; k++) {
        const orbmi_pose_obs& o = obs[f->obs_begin + k];
        UEdge& e = E[k];
        for (int r = 0; r < 3; r++) e.Xw[r] = o.Xw[r];
        e.stereo = !(o.ur < 0);
        e.obs[0] = o.u; e.obs[1] = o.v; e.obs[2] = e.stereo ? o.ur : 0.0;
        e.info = o.inv_sigma2;
        e.delta = e.stereo ? deltaStereo : deltaMono;
        e.dsqr = e.delta * e.delta;
        outlier[f->obs_begin + k] = 0;
    }
    f->iterations = 0;
    f->inliers = 0;
    if (n < 3) return 0;  // :378-379, pose untouched
    PoseOpt P(E);
    P.cam = Cam{f->fx, f->fy, f->cx, f->cy, f->bf};
    if (g_diag_chi2)
        for (int k = 0; k < 4 * n; k++) g_diag_chi2[k] = std::numeric_limits<float>::quiet_NaN();
    if (g_diag_stop)
        for (int r = 0; r < 8; r++) g_diag_stop[r] = std::numeric_limits<double>::infinity();
    const float chi2Mono[4] = {5.991f, 5.991f, 5.991f, 5.991f};
    const float chi2Stereo[4] = {7.815f, 7.815f, 7.815f, 7.815f};
    int nBad = 0;
    for (int it = 0; it < 4; it++) {
        P.T = se3_from_tcw(f->tcw);
        P.stop_margin = g_diag_stop ? &g_diag_stop[it] : nullptr;
        P.optimize(10);
        nBad = 0;
        // mono edges first, then stereo (the reference's two loops; order is immaterial here)
        for (int pass = 0; pass < 2; pass++)
            for (int k = 0; k < n; k++) {
                UEdge& e = E[k];
                if ((int)e.stereo != pass) continue;
                if (outlier[f->obs_begin + k]) compute_error(P.T, P.cam, e);
                const float c2 = (float)chi2(e);
                if (g_diag_chi2) g_diag_chi2[it * n + k] = c2;
                if (c2 > (e.stereo ? chi2Stereo[it] : chi2Mono[it])) {
                    outlier[f->obs_begin + k] = 1;
                    e.level = 1;
                    nBad++;
                } else {
                    outlier[f->obs_begin + k] = 0;
                    e.level = 0;
                }
                if (it == 2) e.robust = false;
            }
        if (n < 10) break;  // optimizer.edges().size() < 10
    }
    se3_to_tcw(P.T, f->tcw);
    f->iterations = P.iters;
    f->inliers = n - nBad;
    return f->inliers;
}

// Diagnostics on (buffers of 4 * n_obs floats and 8 doubles for the next frame) or off (nulls).
extern "C" void orc_pose_set_diag(float* chi2_rounds, double* stop_margin) {
    g_diag_chi2 = chi2_rounds;
    g_diag_stop = stop_margin;
}
