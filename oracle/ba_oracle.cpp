// ============================================================================
// ORACLE — TEST INFRASTRUCTURE ONLY (see orb_oracle.cpp header for the rules).
//
// CPU restatement of the reference bundle-adjustment hot path, fp64:
//   U:src/Optimizer.cc::Optimizer::LocalBundleAdjustment / BundleAdjustment — the g2o
//     problem: VertexSE3Expmap poses (fixed flags), marginalised VertexSBAPointXYZ points,
//     EdgeSE3ProjectXYZ mono edges, information I*invSigma2[octave], Huber(delta),
//     BlockSolver_6_3 + LinearSolverEigen + OptimizationAlgorithmLevenberg, optimize(n).
//   U:src/OptimizableTypes.cpp::EdgeSE3ProjectXYZ::{computeError, linearizeOplus,
//     isDepthPositive}; U:src/CameraModels/Pinhole.cpp::{project, projectJac}.
//   g2o (vendored in the fork, absent here): SE3Quat::{exp, map, operator*,
//     normalizeRotation}, VertexSE3Expmap::oplusImpl (T <- exp(d)*T), VertexSBAPointXYZ
//     (X += d), BaseBinaryEdge::constructQuadraticForm, RobustKernelHuber::robustify,
//     BlockSolver::{buildSystem, setLambda, restoreDiagonal, solve} (per-landmark Schur,
//     upper pose pairs, landmark back-substitution), OptimizationAlgorithmLevenberg::
//     {solve, computeLambdaInit, computeScale}, SparseOptimizer::{optimize,
//     activeRobustChi2, push/pop}. Eigen 3x3 inverse by cofactors; Eigen quaternion
//     from rotation matrix / product / vector rotation.
// The reduced camera system is solved by a dense LDL^T without pivoting in natural order
// (SimplicialLDLT uses an AMD permutation: identical in exact arithmetic, differs in
// rounding — the tolerance of the BA parity tests covers it).
// PARITY UNPINNED by the reference (submodule empty, no fixtures).
// ============================================================================
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <limits>
#include <vector>

namespace bao {

struct Q { double x, y, z, w; };
struct V3 { double x, y, z; };
struct SE3 { Q q; V3 t; };

static inline Q qmul(const Q& a, const Q& b) {
    return Q{a.w * b.x + a.x * b.w + a.y * b.z - a.z * b.y, a.w * b.y + a.y * b.w + a.z * b.x - a.x * b.z,
             a.w * b.z + a.z * b.w + a.x * b.y - a.y * b.x, a.w * b.w - a.x * b.x - a.y * b.y - a.z * b.z};
}
static inline V3 cross(const V3& a, const V3& b) {
    return V3{a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}
static inline V3 qrot(const Q& q, const V3& v) {   // Eigen _transformVector
    V3 u{q.x, q.y, q.z};
    V3 uv = cross(u, v);
    uv = V3{uv.x + uv.x, uv.y + uv.y, uv.z + uv.z};
    V3 c = cross(u, uv);
    return V3{v.x + q.w * uv.x + c.x, v.y + q.w * uv.y + c.y, v.z + q.w * uv.z + c.z};
}
static inline void normalize_rotation(Q& q) {     // SE3Quat::normalizeRotation
    if (q.w < 0) { q.x = -q.x; q.y = -q.y; q.z = -q.z; q.w = -q.w; }
    double n = std::sqrt(q.x * q.x + q.y * q.y + q.z * q.z + q.w * q.w);
    q.x /= n; q.y /= n; q.z /= n; q.w /= n;
}
static inline void qtomat(const Q& q, double R[9]) {   // Eigen toRotationMatrix
    const double tx = 2 * q.x, ty = 2 * q.y, tz = 2 * q.z;
    const double twx = tx * q.w, twy = ty * q.w, twz = tz * q.w;
    const double txx = tx * q.x, txy = ty * q.x, txz = tz * q.x;
    const double tyy = ty * q.y, tyz = tz * q.y, tzz = tz * q.z;
    R[0] = 1 - (tyy + tzz); R[1] = txy - twz;       R[2] = txz + twy;
    R[3] = txy + twz;       R[4] = 1 - (txx + tzz); R[5] = tyz - twx;
    R[6] = txz - twy;       R[7] = tyz + twx;       R[8] = 1 - (txx + tyy);
}
static inline Q mattoq(const double m[9]) {            // Eigen quaternion from matrix
    Q q;
    double t = m[0] + m[4] + m[8];
    if (t > 0) {
        t = std::sqrt(t + 1.0);
        q.w = 0.5 * t;
        t = 0.5 / t;
        q.x = (m[7] - m[5]) * t;
        q.y = (m[2] - m[6]) * t;
        q.z = (m[3] - m[1]) * t;
    } else {
        int i = 0;
        if (m[4] > m[0]) i = 1;
        if (m[8] > m[3 * i + i]) i = 2;
        int j = (i + 1) % 3, k = (j + 1) % 3;
        t = std::sqrt(m[3 * i + i] - m[3 * j + j] - m[3 * k + k] + 1.0);
        double c[3];
        c[i] = 0.5 * t;
        t = 0.5 / t;
        q.w = (m[3 * k + j] - m[3 * j + k]) * t;
        c[j] = (m[3 * j + i] + m[3 * i + j]) * t;
        c[k] = (m[3 * k + i] + m[3 * i + k]) * t;
        q.x = c[0]; q.y = c[1]; q.z = c[2];
    }
    return q;
}
static inline V3 se3_map(const SE3& T, const V3& p) {
    V3 r = qrot(T.q, p);
    return V3{r.x + T.t.x, r.y + T.t.y, r.z + T.t.z};
}
// SE3Quat::exp(update), update = [omega; upsilon]
static SE3 se3_exp(const double u[6]) {
    const double ox = u[0], oy = u[1], oz = u[2];
    const double theta = std::sqrt(ox * ox + oy * oy + oz * oz);
    const double O[9] = {0, -oz, oy, oz, 0, -ox, -oy, ox, 0};
    double O2[9];
    for (int r = 0; r < 3; r++)
        for (int c = 0; c < 3; c++) {
            double s = 0;
            for (int k = 0; k < 3; k++) s += O[3 * r + k] * O[3 * k + c];
            O2[3 * r + c] = s;
        }
    double R[9], V[9];
    if (theta < 0.00001) {
        for (int i = 0; i < 9; i++) R[i] = (i % 4 == 0 ? 1.0 : 0.0) + O[i] + O2[i];
        for (int i = 0; i < 9; i++) V[i] = R[i];
    } else {
        const double a = std::sin(theta) / theta, b = (1 - std::cos(theta)) / (theta * theta);
        const double c = (theta - std::sin(theta)) / std::pow(theta, 3);
        for (int i = 0; i < 9; i++) R[i] = (i % 4 == 0 ? 1.0 : 0.0) + a * O[i] + b * O2[i];
        for (int i = 0; i < 9; i++) V[i] = (i % 4 == 0 ? 1.0 : 0.0) + b * O[i] + c * O2[i];
    }
    SE3 T;
    T.q = mattoq(R);
    T.t = V3{V[0] * u[3] + V[1] * u[4] + V[2] * u[5], V[3] * u[3] + V[4] * u[4] + V[5] * u[5],
             V[6] * u[3] + V[7] * u[4] + V[8] * u[5]};
    normalize_rotation(T.q);
    return T;
}
static inline SE3 se3_mul(const SE3& a, const SE3& b) {   // SE3Quat::operator*
    SE3 r = a;
    V3 bt = qrot(a.q, b.t);
    r.t = V3{a.t.x + bt.x, a.t.y + bt.y, a.t.z + bt.z};
    r.q = qmul(a.q, b.q);
    normalize_rotation(r.q);
    return r;
}

struct Problem {
    int P, M, E;
    std::vector<SE3> pose;
    std::vector<uint8_t> fixed;
    std::vector<V3> pts;
    std::vector<int> ep, em;
    std::vector<double> eu, ev, einfo;
    double fx, fy, cx, cy;   // float parameters promoted
    double delta;            // Huber delta (float promoted); <= 0: no robust kernel
};

struct EdgeState {
    double e0, e1, chi2, rho0, rho1;
};

static void compute_error(const Problem& pr, int e, EdgeState& s) {
    const V3 Xc = se3_map(pr.pose[pr.ep[e]], pr.pts[pr.em[e]]);
    const double u = pr.fx * Xc.x / Xc.z + pr.cx, v = pr.fy * Xc.y / Xc.z + pr.cy;
    s.e0 = pr.eu[e] - u;
    s.e1 = pr.ev[e] - v;
    s.chi2 = pr.einfo[e] * (s.e0 * s.e0 + s.e1 * s.e1);
    if (pr.delta > 0) {
        const double dsqr = pr.delta * pr.delta;
        if (s.chi2 <= dsqr) { s.rho0 = s.chi2; s.rho1 = 1.0; }
        else {
            const double sq = std::sqrt(s.chi2);
            s.rho0 = 2 * sq * pr.delta - dsqr;
            s.rho1 = pr.delta / sq;
        }
    } else {
        s.rho0 = s.chi2; s.rho1 = 1.0;
    }
}

// Jacobians of the error: A (2x3) wrt the point, B (2x6) wrt the pose (omega, upsilon)
static void linearize(const Problem& pr, int e, double A[6], double B[12]) {
    const SE3& T = pr.pose[pr.ep[e]];
    const V3 Xc = se3_map(T, pr.pts[pr.em[e]]);
    const double x = Xc.x, y = Xc.y, z = Xc.z;
    double J[6];   // -projectJac
    J[0] = -(pr.fx / z); J[1] = -0.0; J[2] = -(-pr.fx * x / (z * z));
    J[3] = -0.0; J[4] = -(pr.fy / z); J[5] = -(-pr.fy * y / (z * z));
    double R[9];
    qtomat(T.q, R);
    for (int r = 0; r < 2; r++)
        for (int c = 0; c < 3; c++)
            A[3 * r + c] = J[3 * r] * R[c] + J[3 * r + 1] * R[3 + c] + J[3 * r + 2] * R[6 + c];
    const double D[18] = {0, z, -y, 1, 0, 0, -z, 0, x, 0, 1, 0, y, -x, 0, 0, 0, 1};
    for (int r = 0; r < 2; r++)
        for (int c = 0; c < 6; c++)
            B[6 * r + c] = J[3 * r] * D[c] + J[3 * r + 1] * D[6 + c] + J[3 * r + 2] * D[12 + c];
}

// ---- dense LDL^T (no pivoting) ----
static bool ldlt_solve(std::vector<double>& S, int n, const std::vector<double>& b, std::vector<double>& x) {
    std::vector<double> d(n);
    for (int j = 0; j < n; j++) {
        double dj = S[(size_t)j * n + j];
        for (int k = 0; k < j; k++) dj -= S[(size_t)j * n + k] * S[(size_t)j * n + k] * d[k];
        if (dj == 0.0 || !std::isfinite(dj)) return false;
        d[j] = dj;
        for (int i = j + 1; i < n; i++) {
            double s = S[(size_t)i * n + j];
            for (int k = 0; k < j; k++) s -= S[(size_t)i * n + k] * S[(size_t)j * n + k] * d[k];
            S[(size_t)i * n + j] = s / dj;
        }
    }
    x = b;
    for (int i = 0; i < n; i++)
        for (int k = 0; k < i; k++) x[i] -= S[(size_t)i * n + k] * x[k];
    for (int i = 0; i < n; i++) x[i] /= d[i];
    for (int i = n - 1; i >= 0; i--)
        for (int k = i + 1; k < n; k++) x[i] -= S[(size_t)k * n + i] * x[k];
    return true;
}

static inline void inv3(const double m[9], double r[9]) {   // Eigen compute_inverse<3x3> (cofactors)
    const double c0 = m[4] * m[8] - m[5] * m[7];
    const double c1 = m[5] * m[6] - m[3] * m[8];   // cofactor (1,0) pattern per Eigen col-0 cofactors
    const double c2 = m[3] * m[7] - m[4] * m[6];
    const double det = m[0] * c0 + m[1] * c1 + m[2] * c2;
    const double id = 1.0 / det;
    r[0] = c0 * id;
    r[3] = c1 * id;
    r[6] = c2 * id;
    r[1] = (m[2] * m[7] - m[1] * m[8]) * id;
    r[4] = (m[0] * m[8] - m[2] * m[6]) * id;
    r[7] = (m[1] * m[6] - m[0] * m[7]) * id;
    r[2] = (m[1] * m[5] - m[2] * m[4]) * id;
    r[5] = (m[2] * m[3] - m[0] * m[5]) * id;
    r[8] = (m[0] * m[4] - m[1] * m[3]) * id;
}

struct Result {
    double chi2_init = 0, chi2_final = 0;
    int iters = 0, trials = 0;
    std::vector<EdgeState> es;
};

static int solve(Problem& pr, int iterations, int early_stop, Result& res, const volatile int* stop) {
    const int P = pr.P, M = pr.M, E = pr.E;
    std::vector<int> opt(P, -1);
    int np = 0;
    for (int i = 0; i < P; i++)
        if (!pr.fixed[i]) opt[i] = np++;
    const int n = 6 * np;
    // landmark columns: edges per point sorted by pose optimisation index (HplCCS column order)
    std::vector<std::vector<int>> col(M);
    for (int e = 0; e < E; e++)
        if (opt[pr.ep[e]] >= 0) col[pr.em[e]].push_back(e);
    for (auto& c : col)
        std::stable_sort(c.begin(), c.end(), [&](int a, int b) { return opt[pr.ep[a]] < opt[pr.ep[b]]; });
    res.es.assign(E, EdgeState{});
    auto errors = [&]() {
        double chi = 0;
        for (int e = 0; e < E; e++) { compute_error(pr, e, res.es[e]); chi += res.es[e].rho0; }
        return chi;
    };
    std::vector<double> Hpp((size_t)np * 36), Hll((size_t)M * 9), Hpl((size_t)E * 18), b((size_t)n + 3 * M);
    std::vector<double> x((size_t)n + 3 * M), S((size_t)n * n), bs(n), xp(n), coeff(n), Dinv((size_t)M * 9);
    double lambda = 0, ni = 2;
    int nBad = 0;
    double currentChi = errors();
    res.chi2_init = currentChi;
    int it;
    for (it = 0; it < iterations && !(stop && *stop); it++) {
        if (it > 0) currentChi = errors();
        // ---- buildSystem ----
        std::fill(Hpp.begin(), Hpp.end(), 0.0);
        std::fill(Hll.begin(), Hll.end(), 0.0);
        std::fill(Hpl.begin(), Hpl.end(), 0.0);
        std::fill(b.begin(), b.end(), 0.0);
        for (int e = 0; e < E; e++) {
            double A[6], B[12];
            linearize(pr, e, A, B);
            const EdgeState& s = res.es[e];
            const double w = s.rho1 * pr.einfo[e];        // weighted information
            const double om0 = -pr.einfo[e] * s.e0 * s.rho1, om1 = -pr.einfo[e] * s.e1 * s.rho1;
            const int m = pr.em[e];
            for (int r = 0; r < 3; r++) {
                b[n + 3 * m + r] += A[r] * om0 + A[3 + r] * om1;
                for (int c = 0; c < 3; c++) Hll[9 * m + 3 * r + c] += w * (A[r] * A[c] + A[3 + r] * A[3 + c]);
            }
            const int oi = opt[pr.ep[e]];
            if (oi >= 0) {
                for (int r = 0; r < 6; r++) {
                    b[6 * oi + r] += B[r] * om0 + B[6 + r] * om1;
                    for (int c = 0; c < 6; c++) Hpp[36 * oi + 6 * r + c] += w * (B[r] * B[c] + B[6 + r] * B[6 + c]);
                    for (int c = 0; c < 3; c++) Hpl[18 * e + 3 * r + c] += w * (B[r] * A[c] + B[6 + r] * A[3 + c]);
                }
            }
        }
        if (it == 0) {
            double md = 0;
            for (int i = 0; i < np; i++)
                for (int j = 0; j < 6; j++) md = std::max(md, std::fabs(Hpp[36 * i + 7 * j]));
            for (int m = 0; m < M; m++)
                for (int j = 0; j < 3; j++) md = std::max(md, std::fabs(Hll[9 * m + 4 * j]));
            lambda = 1e-5 * md;
            ni = 2;
            nBad = 0;
        }
        // ---- Levenberg trials ----
        double rho = 0, tempChi = currentChi;
        int qmax = 0;
        std::vector<SE3> pose_bak = pr.pose;
        std::vector<V3> pts_bak = pr.pts;
        do {
            pose_bak = pr.pose;   // push
            pts_bak = pr.pts;
            // setLambda + BlockSolver::solve (Schur)
            std::fill(S.begin(), S.end(), 0.0);
            for (int i = 0; i < np; i++)
                for (int r = 0; r < 6; r++)
                    for (int c = 0; c < 6; c++)
                        S[(size_t)(6 * i + r) * n + 6 * i + c] = Hpp[36 * i + 6 * r + c] + (r == c ? lambda : 0.0);
            std::fill(coeff.begin(), coeff.end(), 0.0);
            for (int m = 0; m < M; m++) {
                double D[9];
                for (int k = 0; k < 9; k++) D[k] = Hll[9 * m + k] + (k % 4 == 0 ? lambda : 0.0);
                inv3(D, &Dinv[9 * m]);
                const double* Di = &Dinv[9 * m];
                double db[3];
                for (int r = 0; r < 3; r++)
                    db[r] = Di[3 * r] * b[n + 3 * m] + Di[3 * r + 1] * b[n + 3 * m + 1] + Di[3 * r + 2] * b[n + 3 * m + 2];
                const auto& cl = col[m];
                for (size_t a = 0; a < cl.size(); a++) {
                    const int e1 = cl[a], i1 = opt[pr.ep[e1]];
                    const double* B1 = &Hpl[18 * e1];
                    double BD[18];
                    for (int r = 0; r < 6; r++)
                        for (int c = 0; c < 3; c++)
                            BD[3 * r + c] = B1[3 * r] * Di[c] + B1[3 * r + 1] * Di[3 + c] + B1[3 * r + 2] * Di[6 + c];
                    for (int r = 0; r < 6; r++)
                        coeff[6 * i1 + r] += B1[3 * r] * db[0] + B1[3 * r + 1] * db[1] + B1[3 * r + 2] * db[2];
                    for (size_t bb = a; bb < cl.size(); bb++) {
                        const int e2 = cl[bb], i2 = opt[pr.ep[e2]];
                        const double* B2 = &Hpl[18 * e2];
                        for (int r = 0; r < 6; r++)
                            for (int c = 0; c < 6; c++) {
                                const double v = BD[3 * r] * B2[3 * c] + BD[3 * r + 1] * B2[3 * c + 1] +
                                                 BD[3 * r + 2] * B2[3 * c + 2];
                                S[(size_t)(6 * i1 + r) * n + 6 * i2 + c] -= v;
                                if (i1 != i2) S[(size_t)(6 * i2 + c) * n + 6 * i1 + r] -= v;
                            }
                    }
                }
            }
            // the block (i,i) received both (e1,e2) and (e2,e1) only once above; mirror within
            // diagonal blocks for pairs of distinct edges of the same pose
            for (int m = 0; m < M; m++) {
                const auto& cl = col[m];
                for (size_t a = 0; a < cl.size(); a++)
                    for (size_t bb = a + 1; bb < cl.size(); bb++) {
                        const int e1 = cl[a], e2 = cl[bb];
                        const int i1 = opt[pr.ep[e1]], i2 = opt[pr.ep[e2]];
                        if (i1 != i2) continue;
                        const double* Di = &Dinv[9 * m];
                        const double* B1 = &Hpl[18 * e1];
                        const double* B2 = &Hpl[18 * e2];
                        for (int r = 0; r < 6; r++)
                            for (int c = 0; c < 6; c++) {
                                double v = 0;
                                for (int k = 0; k < 3; k++)
                                    for (int l = 0; l < 3; l++) v += B2[3 * r + k] * Di[3 * k + l] * B1[3 * c + l];
                                S[(size_t)(6 * i1 + r) * n + 6 * i2 + c] -= v;
                            }
                    }
            }
            for (int i = 0; i < n; i++) bs[i] = b[i] - coeff[i];
            std::vector<double> L = S;
            bool ok2 = n == 0 ? true : ldlt_solve(L, n, bs, xp);
            if (!ok2) std::fill(xp.begin(), xp.end(), 0.0);
            for (int i = 0; i < n; i++) x[i] = xp[i];
            for (int m = 0; m < M; m++) {
                double cl3[3] = {b[n + 3 * m], b[n + 3 * m + 1], b[n + 3 * m + 2]};
                for (int e : col[m]) {
                    const int i1 = opt[pr.ep[e]];
                    const double* B1 = &Hpl[18 * e];
                    for (int c = 0; c < 3; c++)
                        for (int r = 0; r < 6; r++) cl3[c] -= B1[3 * r + c] * xp[6 * i1 + r];
                }
                const double* Di = &Dinv[9 * m];
                for (int r = 0; r < 3; r++)
                    x[n + 3 * m + r] = Di[3 * r] * cl3[0] + Di[3 * r + 1] * cl3[1] + Di[3 * r + 2] * cl3[2];
            }
            // update
            for (int i = 0; i < P; i++)
                if (opt[i] >= 0) pr.pose[i] = se3_mul(se3_exp(&x[6 * opt[i]]), pr.pose[i]);
            for (int m = 0; m < M; m++) {
                pr.pts[m].x += x[n + 3 * m];
                pr.pts[m].y += x[n + 3 * m + 1];
                pr.pts[m].z += x[n + 3 * m + 2];
            }
            tempChi = errors();
            if (!ok2) tempChi = std::numeric_limits<double>::max();
            rho = currentChi - tempChi;
            double scale = 0;
            for (int j = 0; j < n + 3 * M; j++) scale += x[j] * (lambda * x[j] + b[j]);
            scale += 1e-3;
            rho /= scale;
            if (rho > 0 && std::isfinite(tempChi)) {
                double alpha = 1. - std::pow((2 * rho - 1), 3);
                alpha = std::min(alpha, 2. / 3.);
                const double sf = std::max(1. / 3., alpha);
                lambda *= sf;
                ni = 2;
                // vendored-g2o stall counter (early_stop): relative chi2 gain < 1e-3
                if (early_stop) {
                    if ((currentChi - tempChi) < 1e-3 * currentChi) nBad++;
                    else nBad = 0;
                }
                currentChi = tempChi;
            } else {
                lambda *= ni;
                ni *= 2;
                pr.pose = pose_bak;   // pop
                pr.pts = pts_bak;
            }
            qmax++;
            res.trials++;
        } while (rho < 0 && qmax < 10 && !(stop && *stop));
        res.iters = it + 1;
        if (qmax == 10 || rho == 0) break;
        if (early_stop && nBad >= 3) break;
    }
    res.chi2_final = currentChi;
    return 0;
}


// ---------------------------------------------------------------------------------------------
// U:src/Optimizer.cc::Optimizer::PoseOptimization(Frame*), monocular edges (recalled upstream):
// one VertexSE3Expmap (Tcw) and EdgeSE3ProjectXYZOnlyPose per matched MapPoint
// (U:src/OptimizableTypes.cpp: error obs - project(T.map(Xw)), Jacobian -projectJac(Xc) *
// [[0,z,-y,1,0,0],[-z,0,x,0,1,0],[y,-x,0,0,0,1]]), information I*invSigma2[octave], Huber
// deltaMono = (float)sqrt(5.991); BlockSolver_6_3 + LinearSolverDense + Levenberg. Four rounds
// of optimize(10) (its[4] = {10,10,10,10}); EVERY round starts from the frame's initial pose (the
// reference re-reads pFrame->GetPose(), which is only written after the last round). After a
// round each edge is classified with chi2() (an outlier's error recomputed at the current
// estimate, an inlier's as left by the last trial) against chi2Mono = 5.991f: outliers go to
// level 1 (inactive next round), inliers back to level 0; after round 2 the robust kernel is
// removed from every edge; the loop stops after a round if the frame has < 10 edges. Returns
// nInitialCorrespondences - nBad (0 and the pose untouched when < 3 correspondences).
// ---------------------------------------------------------------------------------------------
struct PoseEdge { V3 Xw; double u, v, info; };

static inline void pose_edge_error(const SE3& T, const PoseEdge& pe, double fx, double fy, double cx, double cy,
                                   double& e0, double& e1, double& chi2) {
    const V3 Xc = se3_map(T, pe.Xw);
    e0 = pe.u - (fx * Xc.x / Xc.z + cx);
    e1 = pe.v - (fy * Xc.y / Xc.z + cy);
    chi2 = pe.info * (e0 * e0 + e1 * e1);
}

static inline void robustify(double chi2, double delta, bool robust, double& rho0, double& rho1) {
    if (!robust || delta <= 0) { rho0 = chi2; rho1 = 1.0; return; }
    const double dsqr = delta * delta;
    if (chi2 <= dsqr) { rho0 = chi2; rho1 = 1.0; }
    else { const double sq = std::sqrt(chi2); rho0 = 2 * sq * delta - dsqr; rho1 = delta / sq; }
}

// g2o optimize(iterations) on the active (level 0) edges; chi2_last[e] = chi2 of the last
// computeActiveErrors (stale after a rejected final trial, as in g2o)
static void pose_optimize(SE3& T, const std::vector<PoseEdge>& ed, const std::vector<uint8_t>& level,
                          bool robust, double delta, double fx, double fy, double cx, double cy, int iterations,
                          std::vector<double>& chi2_last, int& trials_out) {
    const int N = (int)ed.size();
    int nact = 0;
    for (int e = 0; e < N; e++) nact += level[e] == 0;
    if (nact == 0) return;   // no active vertex: optimize() does nothing
    auto errors = [&](const SE3& Tc) {
        double chi = 0;
        for (int e = 0; e < N; e++) {
            if (level[e]) continue;
            double e0, e1, c2, r0, r1;
            pose_edge_error(Tc, ed[e], fx, fy, cx, cy, e0, e1, c2);
            robustify(c2, delta, robust, r0, r1);
            chi2_last[e] = c2;
            chi += r0;
        }
        return chi;
    };
    double lambda = 0, ni = 2;
    for (int it = 0; it < iterations; it++) {
        double currentChi = errors(T);
        // buildSystem: H = sum rho' B^T Omega B, b = -sum rho' B^T Omega e
        double H[36] = {0}, b[6] = {0};
        for (int e = 0; e < N; e++) {
            if (level[e]) continue;
            double e0, e1, c2, r0, r1;
            pose_edge_error(T, ed[e], fx, fy, cx, cy, e0, e1, c2);
            robustify(c2, delta, robust, r0, r1);
            const V3 Xc = se3_map(T, ed[e].Xw);
            const double x = Xc.x, y = Xc.y, z = Xc.z;
            double J[6];
            J[0] = -(fx / z); J[1] = -0.0; J[2] = -(-fx * x / (z * z));
            J[3] = -0.0; J[4] = -(fy / z); J[5] = -(-fy * y / (z * z));
            const double D[18] = {0, z, -y, 1, 0, 0, -z, 0, x, 0, 1, 0, y, -x, 0, 0, 0, 1};
            double B[12];
            for (int r = 0; r < 2; r++)
                for (int c = 0; c < 6; c++)
                    B[6 * r + c] = J[3 * r] * D[c] + J[3 * r + 1] * D[6 + c] + J[3 * r + 2] * D[12 + c];
            const double w = r1 * ed[e].info;
            const double om0 = -ed[e].info * e0 * r1, om1 = -ed[e].info * e1 * r1;
            for (int r = 0; r < 6; r++) {
                b[r] += B[r] * om0 + B[6 + r] * om1;
                for (int c = 0; c < 6; c++) H[6 * r + c] += w * (B[r] * B[c] + B[6 + r] * B[6 + c]);
            }
        }
        if (it == 0) {
            double md = 0;
            for (int j = 0; j < 6; j++) md = std::max(md, std::fabs(H[7 * j]));
            lambda = 1e-5 * md;
            ni = 2;
        }
        double rho = 0;
        int qmax = 0;
        do {
            const SE3 Tbak = T;
            std::vector<double> S(36), xv(6), bv(b, b + 6);
            for (int k = 0; k < 36; k++) S[k] = H[k] + (k % 7 == 0 ? lambda : 0.0);
            const bool ok2 = ldlt_solve(S, 6, bv, xv);
            if (!ok2) std::fill(xv.begin(), xv.end(), 0.0);
            T = se3_mul(se3_exp(xv.data()), T);
            double tempChi = errors(T);
            if (!ok2) tempChi = std::numeric_limits<double>::max();
            double scale = 1e-3;
            for (int j = 0; j < 6; j++) scale += xv[j] * (lambda * xv[j] + b[j]);
            rho = (currentChi - tempChi) / scale;
            if (rho > 0 && std::isfinite(tempChi)) {
                double alpha = 1. - std::pow((2 * rho - 1), 3);
                alpha = std::min(alpha, 2. / 3.);
                lambda *= std::max(1. / 3., alpha);
                ni = 2;
                currentChi = tempChi;
            } else {
                lambda *= ni;
                ni *= 2;
                T = Tbak;   // pop
            }
            qmax++;
            trials_out++;
        } while (rho < 0 && qmax < 10);
        if (qmax == 10 || rho == 0) break;
    }
}

static int pose_optimization(SE3& Tout, const SE3& Tinit, const std::vector<PoseEdge>& ed, double delta,
                             double fx, double fy, double cx, double cy, std::vector<uint8_t>& outlier, int& trials) {
    const int N = (int)ed.size();
    outlier.assign(N, 0);
    Tout = Tinit;
    if (N < 3) return 0;
    const float chi2Mono[4] = {5.991f, 5.991f, 5.991f, 5.991f};
    std::vector<uint8_t> level(N, 0);
    std::vector<double> chi2_last(N, 0.0);
    bool robust = true;
    int nBad = 0;
    SE3 T = Tinit;
    for (int it = 0; it < 4; it++) {
        T = Tinit;   // vSE3->setEstimate(pFrame->GetPose())
        pose_optimize(T, ed, level, robust, delta, fx, fy, cx, cy, 10, chi2_last, trials);
        nBad = 0;
        for (int e = 0; e < N; e++) {
            if (outlier[e]) {   // level-1 edge: e->computeError() at the current estimate
                double e0, e1;
                pose_edge_error(T, ed[e], fx, fy, cx, cy, e0, e1, chi2_last[e]);
            }
            if (chi2_last[e] > chi2Mono[it]) { outlier[e] = 1; level[e] = 1; nBad++; }
            else { outlier[e] = 0; level[e] = 0; }
        }
        if (it == 2) robust = false;   // e->setRobustKernel(0)
        if (N < 10) break;             // optimizer.edges().size() < 10
    }
    Tout = T;
    return N - nBad;
}
}  // namespace bao

extern "C" {

// Same layout as orbhip_ba_problem (see include/orbhip.h); outputs as orbhip_ba_result.
int orc_ba_solve(int P, int M, int E, const float* pose_q, const float* pose_t, const uint8_t* pose_fixed,
                 const float* points, const int32_t* edge_pose, const int32_t* edge_point, const float* edge_uv,
                 const int32_t* edge_octave, const float* inv_sigma2, float fx, float fy, float cx, float cy,
                 float huber_delta, int iterations, int early_stop, float* out_q, float* out_t, float* out_pts,
                 float* out_chi2, uint8_t* out_depth_ok, double* out_stats /* chi2_init, chi2_final, iters, trials */) {
    bao::Problem pr;
    pr.P = P; pr.M = M; pr.E = E;
    pr.pose.resize(P);
    for (int i = 0; i < P; i++) {
        bao::SE3& T = pr.pose[i];
        T.q = bao::Q{pose_q[4 * i], pose_q[4 * i + 1], pose_q[4 * i + 2], pose_q[4 * i + 3]};
        bao::normalize_rotation(T.q);
        T.t = bao::V3{pose_t[3 * i], pose_t[3 * i + 1], pose_t[3 * i + 2]};
    }
    pr.fixed.assign(pose_fixed, pose_fixed + P);
    pr.pts.resize(M);
    for (int m = 0; m < M; m++) pr.pts[m] = bao::V3{points[3 * m], points[3 * m + 1], points[3 * m + 2]};
    pr.ep.assign(edge_pose, edge_pose + E);
    pr.em.assign(edge_point, edge_point + E);
    pr.eu.resize(E); pr.ev.resize(E); pr.einfo.resize(E);
    for (int e = 0; e < E; e++) {
        pr.eu[e] = edge_uv[2 * e];
        pr.ev[e] = edge_uv[2 * e + 1];
        pr.einfo[e] = inv_sigma2[edge_octave[e]];
    }
    pr.fx = fx; pr.fy = fy; pr.cx = cx; pr.cy = cy;
    pr.delta = huber_delta;
    bao::Result res;
    bao::solve(pr, iterations, early_stop, res, nullptr);
    for (int i = 0; i < P; i++) {
        out_q[4 * i] = (float)pr.pose[i].q.x; out_q[4 * i + 1] = (float)pr.pose[i].q.y;
        out_q[4 * i + 2] = (float)pr.pose[i].q.z; out_q[4 * i + 3] = (float)pr.pose[i].q.w;
        out_t[3 * i] = (float)pr.pose[i].t.x; out_t[3 * i + 1] = (float)pr.pose[i].t.y;
        out_t[3 * i + 2] = (float)pr.pose[i].t.z;
    }
    for (int m = 0; m < M; m++) {
        out_pts[3 * m] = (float)pr.pts[m].x; out_pts[3 * m + 1] = (float)pr.pts[m].y;
        out_pts[3 * m + 2] = (float)pr.pts[m].z;
    }
    for (int e = 0; e < E; e++) {
        out_chi2[e] = (float)res.es[e].chi2;
        const bao::V3 Xc = bao::se3_map(pr.pose[pr.ep[e]], pr.pts[pr.em[e]]);
        out_depth_ok[e] = Xc.z > 0.0 ? 1 : 0;
    }
    out_stats[0] = res.chi2_init;
    out_stats[1] = res.chi2_final;
    out_stats[2] = res.iters;
    out_stats[3] = res.trials;
    return 0;
}

// Optimizer::PoseOptimization(Frame*) on N monocular correspondences (see pose_optimization).
// Returns the inlier count; out_stats = {trials}.
int orc_pose_optimization(int N, const float* pose_q, const float* pose_t, const float* points, const float* uv,
                          const int32_t* octave, const float* inv_sigma2, float fx, float fy, float cx, float cy,
                          float huber_delta, float* out_q, float* out_t, uint8_t* out_outlier, double* out_stats) {
    bao::SE3 T0;
    T0.q = bao::Q{pose_q[0], pose_q[1], pose_q[2], pose_q[3]};
    bao::normalize_rotation(T0.q);
    T0.t = bao::V3{pose_t[0], pose_t[1], pose_t[2]};
    std::vector<bao::PoseEdge> ed(N);
    for (int e = 0; e < N; e++)
        ed[e] = bao::PoseEdge{bao::V3{points[3 * e], points[3 * e + 1], points[3 * e + 2]}, (double)uv[2 * e],
                              (double)uv[2 * e + 1], (double)inv_sigma2[octave[e]]};
    bao::SE3 T;
    std::vector<uint8_t> outl;
    int trials = 0;
    const int nin = bao::pose_optimization(T, T0, ed, huber_delta, fx, fy, cx, cy, outl, trials);
    out_q[0] = (float)T.q.x; out_q[1] = (float)T.q.y; out_q[2] = (float)T.q.z; out_q[3] = (float)T.q.w;
    out_t[0] = (float)T.t.x; out_t[1] = (float)T.t.y; out_t[2] = (float)T.t.z;
    for (int e = 0; e < N; e++) out_outlier[e] = outl[e];
    if (out_stats) out_stats[0] = trials;
    return nin;
}
}
