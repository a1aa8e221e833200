// ORACLE — test infrastructure only (see orb_oracle.h).
// Optimizer::LocalBundleAdjustment (src/Optimizer.cc:483-808) restated on the assembled graph
// with the vendored g2o's semantics, sequential fp64:
//   SparseOptimizer::initializeOptimization/optimize/update  core/sparse_optimizer.cpp:199-419
//   OptimizationAlgorithmLevenberg::solve                    core/optimization_algorithm_levenberg.cpp:61-189
//   BlockSolver<6,3> Schur build / solve / setLambda         core/block_solver.hpp:354-604
//   BaseBinaryEdge::constructQuadraticForm + Huber            core/base_binary_edge.hpp:55-120,
//                                                            core/robust_kernel_impl.cpp:78-91
//   EdgeSE3ProjectXYZ / EdgeStereoSE3ProjectXYZ              types/types_six_dof_expmap.{h,cpp}
//   SE3Quat (exp, *, map, normalizeRotation)                 types/se3quat.h
// The linear solve of the reduced camera system is a dense LDL^T (the reference uses Eigen's
// SimplicialLDLT on the same matrix); results agree to rounding, parity is 1e-4 (BASELINE).
#include <algorithm>
#include <array>
#include <cmath>
#include <cstring>
#include <limits>
#include <vector>

#include "../include/orbmi.h"
#include "g2o_oracle.h"

namespace {

using namespace g2o_oracle;

struct Edge {
    int pt, kf;
    bool stereo;
    double obs[3];
    double info;            // Omega = info * I
    double delta, dsqr;     // Huber
    bool robust = true;
    int level = 0;
    double err[3] = {0, 0, 0};
    double fx, fy, cx, cy, bf;
};

struct Graph {
    std::vector<SE3> T;
    std::vector<int> kf_fixed;
    std::vector<uint32_t> kf_id;
    std::vector<std::array<double, 3>> X;
    std::vector<uint32_t> pt_id;
    std::vector<Edge> E;
};

// computeError (types_six_dof_expmap.h:89-95, :121-127) incl. the float invz of the stereo edge
void compute_error(const Graph& g, Edge& e) {
    double p[3];
    se3_map(g.T[e.kf], g.X[e.pt].data(), p);
    if (!e.stereo) {
        const double px = p[0] / p[2], py = p[1] / p[2];
        e.err[0] = e.obs[0] - (px * e.fx + e.cx);
        e.err[1] = e.obs[1] - (py * e.fy + e.cy);
    } else {
        const float invz = (float)(1.0f / p[2]);  // float = 1.0f / double (types_six_dof_expmap.cpp:151)
        const double r0 = p[0] * invz * e.fx + e.cx;
        const double r1 = p[1] * invz * e.fy + e.cy;
        const float bf = (float)e.bf;
        const double r2 = r0 - (double)(bf * invz);
        e.err[0] = e.obs[0] - r0;
        e.err[1] = e.obs[1] - r1;
        e.err[2] = e.obs[2] - r2;
    }
}

double chi2(const Edge& e) {
    const int d = e.stereo ? 3 : 2;
    double s = 0;
    for (int i = 0; i < d; i++) s += e.err[i] * (e.info * e.err[i]);
    return s;
}

void robustify(const Edge& e, double c, double rho[3]) {  // RobustKernelHuber::robustify
    if (c <= e.dsqr) { rho[0] = c; rho[1] = 1.; rho[2] = 0.; }
    else {
        const double s = std::sqrt(c);
        rho[0] = 2 * s * e.delta - e.dsqr;
        rho[1] = e.delta / s;
        rho[2] = -0.5 * rho[1] / c;
    }
}

bool depth_positive(const Graph& g, const Edge& e) {
    double p[3];
    se3_map(g.T[e.kf], g.X[e.pt].data(), p);
    return p[2] > 0.0;
}

// linearizeOplus (types_six_dof_expmap.cpp:103-134, :188-234): Jl = d e/d X (D x 3),
// Jp = d e/d xi (D x 6)
void jacobians(const Graph& g, const Edge& e, double Jl[3][3], double Jp[3][6]) {
    const SE3& T = g.T[e.kf];
    double p[3];
    se3_map(T, g.X[e.pt].data(), p);
    double R[3][3];
    quat_to_matrix(T.r, R);
    const double x = p[0], y = p[1], z = p[2], z2 = z * z;
    const double fx = e.fx, fy = e.fy, bf = e.bf;
    if (!e.stereo) {
        const double tmp[2][3] = {{fx, 0, -x / z * fx}, {0, fy, -y / z * fy}};
        for (int r = 0; r < 2; r++)
            for (int c = 0; c < 3; c++)
                Jl[r][c] = -1. / z * (tmp[r][0] * R[0][c] + tmp[r][1] * R[1][c] + tmp[r][2] * R[2][c]);
    } else {
        for (int c = 0; c < 3; c++) {
            Jl[0][c] = -fx * R[0][c] / z + fx * x * R[2][c] / z2;
            Jl[1][c] = -fy * R[1][c] / z + fy * y * R[2][c] / z2;
            Jl[2][c] = Jl[0][c] - bf * R[2][c] / z2;
        }
    }
    Jp[0][0] = x * y / z2 * fx; Jp[0][1] = -(1 + (x * x / z2)) * fx; Jp[0][2] = y / z * fx;
    Jp[0][3] = -1. / z * fx; Jp[0][4] = 0; Jp[0][5] = x / z2 * fx;
    Jp[1][0] = (1 + y * y / z2) * fy; Jp[1][1] = -x * y / z2 * fy; Jp[1][2] = -x / z * fy;
    Jp[1][3] = 0; Jp[1][4] = -1. / z * fy; Jp[1][5] = y / z2 * fy;
    if (e.stereo) {
        Jp[2][0] = Jp[0][0] - bf * y / z2; Jp[2][1] = Jp[0][1] + bf * x / z2; Jp[2][2] = Jp[0][2];
        Jp[2][3] = Jp[0][3]; Jp[2][4] = 0; Jp[2][5] = Jp[0][5] - bf / z2;
    }
}

struct Optimizer {
    Graph& g;
    const volatile int* stop;
    std::vector<int> active_edges;
    std::vector<int> pose_idx, pt_idx;  // hessian index (-1 = not active / fixed)
    std::vector<int> poses, pts;        // active free vertices in index order
    int np = 0, nl = 0;
    // quadratic form
    std::vector<double> Hpp, Hll, bp, bl;                   // per vertex blocks
    std::vector<double> Hpl;                                // per active edge 6x3 (pose-point)
    std::vector<int> edge_pp;                               // active edge -> pose index or -1
    double lambda = 0, ni = 2;
    int nBad = 0;
    std::vector<double> x;

    int stop_at = -1;      // orbmi_ba_set_stop_at_check's hook: raised from this check on
    int checks = 0;        // pbStopFlag reads so far, numbered as orbmi_ba_set_stop_at_check's
    int stop_seen = -1;    // the first read that found it raised
    Optimizer(Graph& gr, const volatile int* s, int at) : g(gr), stop(s), stop_at(at) {}
    // every read of pbStopFlag (src/Optimizer.cc:685, :689; SparseOptimizer::terminate()) in the
    // order the reference's short-circuit conditions evaluate them
    bool terminate() {
        const int idx = checks++;
        const bool s = (stop && *stop) || (stop_at >= 0 && idx >= stop_at);
        if (s && stop_seen < 0) stop_seen = idx;
        return s;
    }

    bool initialize(int level) {  // initializeOptimization(level)
        active_edges.clear();
        if (g.E.empty()) { np = nl = 0; poses.clear(); pts.clear(); return false; }
        const int nk = (int)g.T.size(), npt = (int)g.X.size();
        std::vector<int> kf_act(nk, 0), pt_act(npt, 0);
        for (int i = 0; i < (int)g.E.size(); i++) {
            const Edge& e = g.E[i];
            if (e.level != level) continue;
            // allVerticesFixed: a point is never fixed
            active_edges.push_back(i);
            kf_act[e.kf] = 1;
            pt_act[e.pt] = 1;
        }
        // active vertices sorted by id; poses (ids <= maxKFid) before points
        poses.clear(); pts.clear();
        std::vector<int> ko(nk), po(npt);
        for (int i = 0; i < nk; i++) ko[i] = i;
        for (int i = 0; i < npt; i++) po[i] = i;
        std::sort(ko.begin(), ko.end(), [&](int a, int b) { return g.kf_id[a] < g.kf_id[b]; });
        std::sort(po.begin(), po.end(), [&](int a, int b) { return g.pt_id[a] < g.pt_id[b]; });
        pose_idx.assign(nk, -1);
        pt_idx.assign(npt, -1);
        for (int k : ko)
            if (kf_act[k] && !g.kf_fixed[k]) { pose_idx[k] = (int)poses.size(); poses.push_back(k); }
        for (int p : po)
            if (pt_act[p]) { pt_idx[p] = (int)pts.size(); pts.push_back(p); }
        np = (int)poses.size();
        nl = (int)pts.size();
        return np + nl > 0;
    }

    void compute_active_errors() {
        for (int i : active_edges) compute_error(g, g.E[i]);
    }

    double active_robust_chi2() const {
        double c = 0;
        for (int i : active_edges) {
            const Edge& e = g.E[i];
            const double c2 = chi2(e);
            if (e.robust) { double rho[3]; robustify(e, c2, rho); c += rho[0]; }
            else c += c2;
        }
        return c;
    }

    void build_system() {  // BlockSolver::buildSystem
        Hpp.assign((size_t)np * 36, 0); bp.assign((size_t)np * 6, 0);
        Hll.assign((size_t)nl * 9, 0); bl.assign((size_t)nl * 3, 0);
        Hpl.assign(active_edges.size() * 18, 0);
        edge_pp.assign(active_edges.size(), -1);
        for (size_t a = 0; a < active_edges.size(); a++) {
            const Edge& e = g.E[active_edges[a]];
            const int D = e.stereo ? 3 : 2;
            double Jl[3][3] = {}, Jp[3][6] = {};
            jacobians(g, e, Jl, Jp);
            double w = e.info, s = 1.0;  // W = rho' * Omega; omega_r = -Omega e * rho'
            if (e.robust) { double rho[3]; robustify(e, chi2(e), rho); w = rho[1] * e.info; s = rho[1]; }
            double om_r[3];
            for (int i = 0; i < D; i++) om_r[i] = -(e.info * e.err[i]) * s;
            const int li = pt_idx[e.pt], pi = pose_idx[e.kf];
            for (int r = 0; r < 3; r++) {
                for (int i = 0; i < D; i++) bl[li * 3 + r] += Jl[i][r] * om_r[i];
                for (int c = 0; c < 3; c++) {
                    double h = 0;
                    for (int i = 0; i < D; i++) h += Jl[i][r] * w * Jl[i][c];
                    Hll[li * 9 + r * 3 + c] += h;
                }
            }
            if (pi >= 0) {
                edge_pp[a] = pi;
                for (int r = 0; r < 6; r++) {
                    for (int i = 0; i < D; i++) bp[pi * 6 + r] += Jp[i][r] * om_r[i];
                    for (int c = 0; c < 6; c++) {
                        double h = 0;
                        for (int i = 0; i < D; i++) h += Jp[i][r] * w * Jp[i][c];
                        Hpp[pi * 36 + r * 6 + c] += h;
                    }
                    for (int c = 0; c < 3; c++) {
                        double h = 0;
                        for (int i = 0; i < D; i++) h += Jp[i][r] * w * Jl[i][c];
                        Hpl[a * 18 + r * 3 + c] = h;
                    }
                }
            }
        }
    }

    double lambda_init() const {  // computeLambdaInit, tau = 1e-5
        double m = 0;
        for (int i = 0; i < np; i++)
            for (int j = 0; j < 6; j++) m = std::max(m, std::fabs(Hpp[i * 36 + j * 7]));
        for (int i = 0; i < nl; i++)
            for (int j = 0; j < 3; j++) m = std::max(m, std::fabs(Hll[i * 9 + j * 4]));
        return 1e-5 * m;
    }

    // BlockSolver::setLambda + solve (Schur) ; x = [poses | points]
    bool solve(double lam) {
        const int N = 6 * np;
        std::vector<double> S((size_t)N * N, 0), bs(N);
        for (int i = 0; i < np; i++)
            for (int r = 0; r < 6; r++) {
                for (int c = 0; c < 6; c++) S[(size_t)(6 * i + r) * N + 6 * i + c] = Hpp[i * 36 + r * 6 + c];
                S[(size_t)(6 * i + r) * N + 6 * i + r] += lam;
                bs[6 * i + r] = bp[i * 6 + r];
            }
        // per landmark: its active edges with a free pose
        std::vector<std::vector<int>> obs(nl);
        for (size_t a = 0; a < active_edges.size(); a++)
            if (edge_pp[a] >= 0) obs[pt_idx[g.E[active_edges[a]].pt]].push_back((int)a);
        std::vector<double> Dinv((size_t)nl * 9);
        for (int l = 0; l < nl; l++) {
            double D[3][3];
            for (int r = 0; r < 3; r++)
                for (int c = 0; c < 3; c++) D[r][c] = Hll[l * 9 + r * 3 + c] + (r == c ? lam : 0);
            // Eigen 3x3 inverse (cofactors)
            const double c00 = D[1][1] * D[2][2] - D[1][2] * D[2][1];
            const double c10 = D[1][2] * D[2][0] - D[1][0] * D[2][2];
            const double c20 = D[1][0] * D[2][1] - D[1][1] * D[2][0];
            const double det = D[0][0] * c00 + D[0][1] * c10 + D[0][2] * c20;
            double* Di = &Dinv[l * 9];
            Di[0] = c00 / det; Di[3] = c10 / det; Di[6] = c20 / det;
            Di[1] = (D[0][2] * D[2][1] - D[0][1] * D[2][2]) / det;
            Di[4] = (D[0][0] * D[2][2] - D[0][2] * D[2][0]) / det;
            Di[7] = (D[0][1] * D[2][0] - D[0][0] * D[2][1]) / det;
            Di[2] = (D[0][1] * D[1][2] - D[0][2] * D[1][1]) / det;
            Di[5] = (D[0][2] * D[1][0] - D[0][0] * D[1][2]) / det;
            Di[8] = (D[0][0] * D[1][1] - D[0][1] * D[1][0]) / det;
            double db[3];
            for (int r = 0; r < 3; r++) db[r] = Di[r * 3] * bl[l * 3] + Di[r * 3 + 1] * bl[l * 3 + 1] + Di[r * 3 + 2] * bl[l * 3 + 2];
            for (int a1 : obs[l]) {
                const int i1 = edge_pp[a1];
                const double* B1 = &Hpl[a1 * 18];
                double BD[6][3];
                for (int r = 0; r < 6; r++)
                    for (int c = 0; c < 3; c++) BD[r][c] = B1[r * 3] * Di[c] + B1[r * 3 + 1] * Di[3 + c] + B1[r * 3 + 2] * Di[6 + c];
                for (int r = 0; r < 6; r++) bs[6 * i1 + r] -= B1[r * 3] * db[0] + B1[r * 3 + 1] * db[1] + B1[r * 3 + 2] * db[2];
                for (int a2 : obs[l]) {
                    const int i2 = edge_pp[a2];
                    const double* B2 = &Hpl[a2 * 18];
                    for (int r = 0; r < 6; r++)
                        for (int c = 0; c < 6; c++)
                            S[(size_t)(6 * i1 + r) * N + 6 * i2 + c] -= BD[r][0] * B2[c * 3] + BD[r][1] * B2[c * 3 + 1] + BD[r][2] * B2[c * 3 + 2];
                }
            }
        }
        x.assign((size_t)N + 3 * nl, 0);
        if (N > 0) {
            if (!ldlt_solve(S, N, bs)) return false;
            for (int i = 0; i < N; i++) x[i] = bs[i];
        }
        for (int l = 0; l < nl; l++) {
            double cl[3] = {bl[l * 3], bl[l * 3 + 1], bl[l * 3 + 2]};
            for (int a : obs[l]) {
                const int i = edge_pp[a];
                const double* B = &Hpl[a * 18];
                for (int c = 0; c < 3; c++)
                    for (int r = 0; r < 6; r++) cl[c] -= B[r * 3 + c] * x[6 * i + r];
            }
            const double* Di = &Dinv[l * 9];
            for (int r = 0; r < 3; r++) x[N + 3 * l + r] = Di[r * 3] * cl[0] + Di[r * 3 + 1] * cl[1] + Di[r * 3 + 2] * cl[2];
        }
        return true;
    }

    void update() {  // SparseOptimizer::update -> oplus in index order
        for (int i = 0; i < np; i++) g.T[poses[i]] = se3_mul(se3_exp(&x[6 * i]), g.T[poses[i]]);
        for (int l = 0; l < nl; l++)
            for (int r = 0; r < 3; r++) g.X[pts[l]][r] += x[6 * np + 3 * l + r];
    }

    double compute_scale() const {
        double s = 0;
        const int N = 6 * np;
        for (int j = 0; j < N; j++) s += x[j] * (lambda * x[j] + bp[j]);
        for (int j = 0; j < 3 * nl; j++) s += x[N + j] * (lambda * x[N + j] + bl[j]);
        return s;
    }

    enum Result { OK, Terminate, Fail };

    Result lm_solve(int iteration) {  // OptimizationAlgorithmLevenberg::solve
        compute_active_errors();
        double currentChi = active_robust_chi2();
        double tempChi = currentChi;
        const double iniChi = currentChi;
        build_system();
        if (iteration == 0) { lambda = lambda_init(); ni = 2; nBad = 0; }
        double rho = 0;
        int qmax = 0;
        do {
            std::vector<SE3> T0;
            std::vector<std::array<double, 3>> X0;
            for (int k : poses) T0.push_back(g.T[k]);
            for (int p : pts) X0.push_back(g.X[p]);
            const bool ok2 = solve(lambda);
            if (ok2) update();
            else x.assign(x.size(), 0);
            compute_active_errors();
            tempChi = active_robust_chi2();
            if (!ok2) tempChi = std::numeric_limits<double>::max();
            rho = currentChi - tempChi;
            double scale = compute_scale();
            scale += 1e-3;
            rho /= scale;
            if (rho > 0 && std::isfinite(tempChi)) {
                double alpha = 1. - std::pow((2 * rho - 1), 3);
                alpha = std::min(alpha, 2. / 3.);
                const double scaleFactor = std::max(1. / 3., alpha);
                lambda *= scaleFactor;
                ni = 2;
                currentChi = tempChi;
            } else {
                lambda *= ni;
                ni *= 2;
                for (size_t i = 0; i < poses.size(); i++) g.T[poses[i]] = T0[i];
                for (size_t i = 0; i < pts.size(); i++) g.X[pts[i]] = X0[i];
            }
            qmax++;
        } while (rho < 0 && qmax < 10 && !terminate());
        if (qmax == 10 || rho == 0) return Terminate;
        if ((iniChi - currentChi) * 1e3 < iniChi) nBad++;
        else nBad = 0;
        if (nBad >= 3) return Terminate;
        last_chi = currentChi;
        return OK;
    }
    double last_chi = 0;

    int optimize(int iterations) {  // SparseOptimizer::optimize
        if (np + nl == 0) return -1;
        int it = 0;
        bool ok = true;
        for (int i = 0; i < iterations && !terminate() && ok; i++) {
            const Result r = lm_solve(i);
            ok = r == OK;
            ++it;
        }
        return it;
    }
};

}  // namespace

static int local_ba(const orbmi_ba_problem* P, orbmi_ba_result* R, const volatile int* stop, int stop_at,
                    double* edge_chi2);

extern "C" int orc_local_ba(const orbmi_ba_problem* P, orbmi_ba_result* R, const volatile int* stop) {
    return local_ba(P, R, stop, -1, nullptr);
}

/* Same, and the chi2 every erase decision of src/Optimizer.cc:758-773 reads (per edge; -1 for
 * edges of bad points): lets the parity tests show that an erase flag that differs from the
 * GPU's sits on its threshold within the pose tolerance. */
extern "C" int orc_local_ba_edge_chi2(const orbmi_ba_problem* P, orbmi_ba_result* R, const volatile int* stop,
                                      double* edge_chi2) {
    return local_ba(P, R, stop, -1, edge_chi2);
}

/* Same with the deterministic pbStopFlag of orbmi_ba_set_stop_at_check (stop_at < 0: off);
 * result.stop_check / checks report the reads as the device does. */
extern "C" int orc_local_ba_ex(const orbmi_ba_problem* P, orbmi_ba_result* R, const volatile int* stop, int stop_at,
                               double* edge_chi2) {
    return local_ba(P, R, stop, stop_at, edge_chi2);
}

static int local_ba(const orbmi_ba_problem* P, orbmi_ba_result* R, const volatile int* stop, int stop_at,
                    double* edge_chi2) {
    Graph g;
    for (int k = 0; k < P->nkf; k++) {
        g.T.push_back(se3_from_tcw(P->kfs[k].tcw));
        g.kf_fixed.push_back(P->kfs[k].fixed != 0);
        g.kf_id.push_back(P->kfs[k].id);
    }
    for (int p = 0; p < P->npt; p++) {
        g.X.push_back({(double)P->pts[p].pos[0], (double)P->pts[p].pos[1], (double)P->pts[p].pos[2]});
        g.pt_id.push_back(P->pts[p].id);
    }
    const float thHuberMono = (float)std::sqrt(5.991), thHuberStereo = (float)std::sqrt(7.815);
    for (int i = 0; i < P->nedge; i++) {
        const orbmi_ba_edge& s = P->edges[i];
        const orbmi_ba_keyframe& kf = P->kfs[s.kf];
        Edge e;
        e.pt = s.point; e.kf = s.kf;
        e.stereo = !(s.ur < 0);
        e.obs[0] = s.u; e.obs[1] = s.v; e.obs[2] = e.stereo ? s.ur : 0;
        e.info = (double)s.inv_sigma2;
        e.delta = e.stereo ? (double)thHuberStereo : (double)thHuberMono;
        e.dsqr = e.delta * e.delta;  // RobustKernelHuber::setDelta
        e.fx = kf.fx; e.fy = kf.fy; e.cx = kf.cx; e.cy = kf.cy; e.bf = kf.bf;
        g.E.push_back(e);
    }
    R->aborted = 0;
    R->iterations[0] = R->iterations[1] = 0;
    R->chi2[0] = R->chi2[1] = 0;
    for (int i = 0; i < P->nedge; i++) R->erase[i] = 0;
    Optimizer opt(g, stop, stop_at);
    auto report = [&] {
        R->stop_check = opt.stop_seen;
        R->checks = opt.checks;
    };
    if (opt.terminate()) {  // src/Optimizer.cc:685-687: return before optimising, no write-back
        R->aborted = 1;
        report();
        return 0;
    }
    opt.initialize(0);
    R->iterations[0] = opt.optimize(5);
    R->chi2[0] = opt.active_robust_chi2();
    bool bDoMore = !opt.terminate();  // :689-692
    if (bDoMore) {
        for (Edge& e : g.E) {
            if (P->pts[e.pt].bad) continue;
            const double th = e.stereo ? 7.815 : 5.991;
            if (chi2(e) > th || !depth_positive(g, e)) e.level = 1;
            e.robust = false;
        }
        opt.initialize(0);
        R->iterations[1] = opt.optimize(10);
        R->chi2[1] = opt.active_robust_chi2();
    }
    for (int i = 0; i < P->nedge; i++) {
        const Edge& e = g.E[i];
        if (edge_chi2) edge_chi2[i] = -1.0;
        if (P->pts[e.pt].bad) continue;
        const double th = e.stereo ? 7.815 : 5.991;
        if (edge_chi2) edge_chi2[i] = depth_positive(g, e) ? chi2(e) : -2.0;
        if (chi2(e) > th || !depth_positive(g, e)) R->erase[i] = 1;
    }
    for (int k = 0; k < P->nkf; k++) se3_to_tcw(g.T[k], R->tcw + 16 * k);
    for (int p = 0; p < P->npt; p++)
        for (int r = 0; r < 3; r++) R->pos[3 * p + r] = (float)g.X[p][r];
    report();
    return 0;
}
