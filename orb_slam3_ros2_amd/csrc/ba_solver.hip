// gfx950 bundle adjustment: the g2o problem of Optimizer::LocalBundleAdjustment /
// BundleAdjustment (U:src/Optimizer.cc) solved with the Levenberg-Marquardt schedule of
// OptimizationAlgorithmLevenberg and the Schur complement of BlockSolver<6,3>.
//
// Batched: every kernel runs over grid.y = the problems (problem index from act[]), so B
// independent problems (SURVEY.md §8e "replicas": concurrent maps / agents, or a batch of local
// windows) share each launch. The device-driven solve advances every problem by one LM trial per
// slot with no host round trip (the g2o control flow on the device, LmCtl); the host-driven
// rounds of r01 remain for the sharded solves. fp64 throughout:
//   k_ba_errors        EdgeSE3ProjectXYZ::computeError + RobustKernelHuber::robustify; in a trial
//                      its last workgroup per problem runs the LM controller step (ctl_end_body)
//   k_ba_lin           linearizeOplus + constructQuadraticForm: landmark side (Hll, b_l, the
//                      edge records) and pose side (Hpp, b_p, one wave per pose) in one launch;
//                      its last workgroup per problem starts the trial (ctl_begin_body)
//                      (k_ba_lin_points / k_ba_lin_poses: the same bodies for host-driven rounds)
//   k_ba_schur_points  setLambda on Hll, Dinv (Eigen 3x3 cofactor inverse), db
//   k_ba_schur_items   S_ij = [i==j](Hpp_i + lambda I) - sum W_a Hpl_b^T over shared landmarks,
//                      matrix-free; its trailing workgroups compute b_schur = b_p - sum Hpl db
//                      (a block of several items: its last item adds their partials in order)
//   k_chol_dag / k_ba_chol_reg / k_ba_cholesky / k_cb_*   the reduced camera system (ba_chol_*)
//   k_ba_backsub       xl = Dinv (b_l - Hpl^T xp), X += xl (push: old X saved)
//                      and T <- exp(xp) * T (SE3Quat::exp, operator*)   (push: old T saved)
//   k_ba_reduce        activeRobustChi2, computeScale, max diag (host-driven rounds)
//   k_ba_pop           restore the pushed state of problems whose trial was rejected
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <cfloat>
#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <limits>
#include <thread>
#include <vector>

#include "orbhip_ba.h"
#include "dev_attr.h"
#include "ba_chol.h"
#include "ba_chol_blocked.h"
#include "ba_chol_dag.h"
#include "ba_nd.h"
#include "ba_args.h"
#include "ba_chol_reg.h"
#include "ba_se3.h"

namespace orbhip {


// struct BaArgs: ba_args.h


// Grid (X work-groups per problem, Y problems). Work-groups are dispatched round-robin over the
// 8 XCDs in linear order, so the plain (blockIdx.x, blockIdx.y) spreads every problem over all
// XCDs and each XCD's L2 streams every problem's arrays. Remapped, the X work-groups of problem p
// run on XCD p % 8 (for the first 8 floor(Y / 8) problems; the tail keeps the plain order), so a
// problem's Hpl / W / S stay in one L2. Speed only: correctness never depends on the placement.
__device__ __forceinline__ void ba_xcd_map(int& bx, int& by) {
    const int X = gridDim.x, Y = gridDim.y;
    const int id = blockIdx.x + X * blockIdx.y;
    const int Yf = Y & ~7;
    if (id < X * Yf) {
        const int k = id & 7, s = id >> 3;
        by = 8 * (s / X) + k;
        bx = s - (s / X) * X;
    } else {
        by = id / X;
        bx = id - by * X;
    }
}
#define BA_PROLOGUE                                 \
    int bx_, by_;                                   \
    ba_xcd_map(bx_, by_);                           \
    const BaArgs& a = args[act[by_]];

// Device-driven rounds: a kernel runs for a problem only in the phase it belongs to (build:
// linearisation; trial: Schur / solve / update / errors). Host-driven rounds (a.ctl == nullptr)
// select problems through act[] alone.
__device__ __forceinline__ bool in_phase(const BaArgs& a, int ph) { return !a.ctl || a.ctl->phase == ph; }
#define BA_PHASE(ph) \
    if (!in_phase(a, ph)) return;

// sum over the workgroup, the same value in every thread (fixed order)
__device__ double block_sum(double v, double* sh) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    __syncthreads();
    if (lane == 0) sh[wid] = v;
    __syncthreads();
    double s = 0;
    for (int i = 0; i < (int)(blockDim.x >> 6); i++) s += sh[i];
    return s;
}

// Last-arriver hand-off inside one launch (MI355X_MICROARCH.md visibility table, row 1): each
// workgroup of a problem's row stores its partial with an agent-scope (sc1) store, drains it, and
// bumps the problem's counter; the workgroup that arrives last reads every partial with sc1 loads
// and runs the controller step that used to be its own launch. Nobody waits for anybody.
typedef __attribute__((address_space(1))) int ba_gint;
typedef __attribute__((address_space(1))) double ba_gdbl;
__device__ __forceinline__ void st_agent(double* p, double v) {
    __hip_atomic_store((ba_gdbl*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ld_agent(const double* p) {
    return __hip_atomic_load((ba_gdbl*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// every workgroup of the row calls it once, after thread 0's partial store; true (uniform) in the
// last one, which also resets the counter for the next launch
__device__ __forceinline__ bool last_arrival(int* counter, int total, int* sh_flag) {
    if (threadIdx.x == 0) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const int old = __hip_atomic_fetch_add((ba_gint*)counter, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const int last = old == total - 1;
        if (last) __hip_atomic_store((ba_gint*)counter, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        *sh_flag = last;
    }
    __syncthreads();
    return *sh_flag != 0;
}
__device__ void ctl_end_body(const BaArgs& a, int prob, int* done_flags, double* sh);
__device__ void ctl_begin_body(const BaArgs& a, int nlin, int* done_flags, int prob, double* sh);

// ---------------------------------------------------------------------------
// errors (when: 0 always, 1 the build's stale-error refresh, 2 a trial's new state); a trial also
// writes each workgroup's sum of the robust chi2 terms to part[bx] (k_ba_ctl_end adds them)
// ---------------------------------------------------------------------------
// one edge: error, chi2, robust rho (EdgeSE3ProjectXYZ::computeError + RobustKernelHuber::robustify);
// returns rho0
// the error terms of edge e from its camera-frame point
__device__ __forceinline__ void edge_terms(const BaArgs& a, int e, double cx, double cy, double cz, double& e0,
                                           double& e1, double& chi2, double& r0, double& r1) {
    const double u = a.fx * cx / cz + a.cx, v = a.fy * cy / cz + a.cy;
    e0 = a.e_obs[2 * e] - u;
    e1 = a.e_obs[2 * e + 1] - v;
    chi2 = a.e_info[e] * (e0 * e0 + e1 * e1);
    r0 = chi2;
    r1 = 1.0;
    if (a.delta > 0) {
        const double dsqr = a.delta * a.delta;
        if (chi2 > dsqr) {
            const double sq = sqrt(chi2);
            r0 = 2 * sq * a.delta - dsqr;
            r1 = a.delta / sq;
        }
    }
}
__device__ __forceinline__ void store_terms(const BaArgs& a, int e, double e0, double e1, double chi2, double r0,
                                            double r1) {
    a.e_err[2 * e] = e0;
    a.e_err[2 * e + 1] = e1;
    a.e_chi2[e] = chi2;
    a.e_rho0[e] = r0;
    a.e_rho1[e] = r1;
}
// Plain stores: no launch rewrites these words after another workgroup of the same launch wrote
// them (a rejected small problem's refresh is done by the next build, k_ba_lin, not by the
// trial's last workgroup; r05: the agent-scope stores cost ~4 us per C4 trial)
__device__ __forceinline__ double edge_error_at(const BaArgs& a, int e, const double* T, const double* X) {
    double cx, cy, cz;
    qrot(load_q(T), X[0], X[1], X[2], cx, cy, cz);
    cx += T[4]; cy += T[5]; cz += T[6];
    double e0, e1, chi2, r0, r1;
    edge_terms(a, e, cx, cy, cz, e0, e1, chi2, r0, r1);
    store_terms(a, e, e0, e1, chi2, r0, r1);
    return r0;
}
__device__ __forceinline__ double edge_error(const BaArgs& a, int e) {
    return edge_error_at(a, e, a.pose + 8 * a.e_pose[e], a.pts + 3 * a.e_pt[e]);
}

// when == 2 (a trial) ends in the trial's controller step, run by the last workgroup of each
// problem to finish (ctl_end_body; done: the host-mapped done flags).
// when == 1 also opens the device-driven slot (the former k_ba_ctl_pre): workgroup 0 of each
// problem clears the pop request of the previous slot and, at an iteration start, ends the solve
// on the iteration budget or the (host-relayed) stop flag (done[b], host-mapped: the host stops
// queueing slots once every problem is done). Every workgroup derives the same effective phase
// from the controller's fields, so none depends on that transition's store.
// host-mapped words of a device-driven solve, reached through a device-resident pointer pair
// donep = {done, hstop}: done[prob] is set once when the problem's LM run ends (the host stops
// queueing slots once all are set); *hstop is the caller's stop flag as the host relays it while
// it waits (null for sharded solves, whose shards must take the same decisions: they get the
// stop between batches of slots). A store to host memory in every trial put ~5 us in front of
// the next kernel, so the done words are written once per solve and the stop word only read.
__device__ __forceinline__ void post_done(int* done, int prob) {
    if (done) __hip_atomic_store(done + prob, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ int* done_of(int* const* donep) { return donep ? donep[0] : nullptr; }
// The stop word is read over PCIe (~2 us) by an extra workgroup of k_ba_schur_items, off every
// critical path (a read in the controller's tail, or early in a working wave, delays the kernel:
// vmcnt waits in order), and copied into LmCtl::stop, which the controller checks at its trial end
// (this slot) and at the next iteration's start.
// One read per slot (problem row 0's extra workgroup), fanned out to every problem of the launch:
// a read per problem put 256 same-address PCIe reads into every batched slot.
__device__ __forceinline__ void relay_host_stop(const BaArgs* args, const int* act, int* const* donep) {
    const int* hstop = donep ? donep[1] : nullptr;
    if (!hstop || __hip_atomic_load(hstop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == 0) return;
    for (int b = 0; b < (int)gridDim.y; b++) {
        LmCtl* c = args[act[b]].ctl;
        if (c) c->stop = 1;
    }
}

__global__ __launch_bounds__(256) void k_ba_errors(const BaArgs* __restrict__ args, const int* __restrict__ act,
                                                   int when, int* const* donep) {
    BA_PROLOGUE
    int* const done = done_of(donep);
    if (when == 1) {
        LmCtl* c = a.ctl;
        const bool ends = c && c->phase == kPhBuild && (c->stop || c->it >= c->iterations);
        if (c && bx_ == 0 && threadIdx.x == 0) {
            c->pop = 0;
            if (ends) {
                c->phase = kPhDone;
                post_done(done, act[by_]);
            }
        }
        if (ends || !(in_phase(a, kPhBuild) && (!c || !c->errors_valid))) return;
    }
    if (when == 2 && !in_phase(a, kPhTrial)) return;
    const bool has = bx_ * (int)blockDim.x < a.E;   // uniform
    if (when != 2 && !has) return;
    const int e = bx_ * blockDim.x + threadIdx.x;
    const double r0 = (has && e < a.E) ? edge_error(a, e) : 0.0;
    if (when == 2) {   // uniform: every thread reaches the workgroup sum's barriers once
        __shared__ double sh[4];
        __shared__ int lastf;
        const double t = block_sum(r0, sh);
        if (threadIdx.x == 0 && has) st_agent(a.part + bx_, t);
        // the row's last workgroup runs the trial's controller step (the former k_ba_ctl_end)
        if (a.ctl && !a.sync && last_arrival(&a.ctl->arrive_t, gridDim.x, &lastf)) ctl_end_body(a, act[by_], done, sh);
    }
}

// Jacobians of EdgeSE3ProjectXYZ at the camera-frame point (x, y, z) of a pose with rotation R
// (row-major). The (negated) projection Jacobian J has rows (j00, 0, j02) and (0, j11, j12):
//   j00 = -fx / z, j02 = fx x / z^2, j11 = -fy / z, j12 = fy y / z^2
// A (2x3, landmark) = J R, B (2x6, pose [omega, upsilon]) = J [ -[Pc]x | I ]:
//   B = [[j02 y, j00 z - j02 x, -j00 y, j00, 0, j02], [j12 y - j11 z, -j12 x, j11 x, 0, j11, j12]].
// The linearisation stores (x, y, z, w) per edge; every consumer (Schur, back-substitution)
// rebuilds J, A and B from that record and the pose's R_lin, so Hpl_e = w B^T A (18 doubles per
// edge) is never stored. These consumers are bound by L2 traffic, not flops: storing J too (64
// instead of 32 bytes per edge) measured 20% slower at B = 256.
__device__ __forceinline__ void proj_jac(double fx, double fy, double x, double y, double z, double j[4]) {
    j[0] = -(fx / z);
    j[1] = fx * x / (z * z);
    j[2] = -(fy / z);
    j[3] = fy * y / (z * z);
}
__device__ __forceinline__ void jac_ab(const double j[4], double x, double y, double z, const double R[9],
                                       double A[6], double B[12]) {
#pragma unroll
    for (int c = 0; c < 3; c++) {
        A[c] = j[0] * R[c] + j[1] * R[6 + c];
        A[3 + c] = j[2] * R[3 + c] + j[3] * R[6 + c];
    }
    B[0] = j[1] * y; B[1] = j[0] * z - j[1] * x; B[2] = -j[0] * y; B[3] = j[0]; B[4] = 0.0; B[5] = j[1];
    B[6] = j[3] * y - j[2] * z; B[7] = -j[3] * x; B[8] = j[2] * x; B[9] = 0.0; B[10] = j[2]; B[11] = j[3];
}

// camera-frame point of edge e at the current state + the pose's rotation matrix
__device__ __forceinline__ void edge_pc(const BaArgs& a, int e, double& x, double& y, double& z, double R[9]) {
    const double* T = a.pose + 8 * a.e_pose[e];
    const double* X = a.pts + 3 * a.e_pt[e];
    const DQ q = load_q(T);
    qrot(q, X[0], X[1], X[2], x, y, z);
    x += T[4]; y += T[5]; z += T[6];
    qtomat(q, R);
}

// A, B of edge e from its stored linearisation (e_lin) and its pose's R_lin (optimised poses only)
__device__ __forceinline__ double lin_ab(const BaArgs& a, int e, int oi, double A[6], double B[12]) {
    const double4 l = ((const double4*)a.e_lin)[e];
    double j[4];
    proj_jac(a.fx, a.fy, l.x, l.y, l.z, j);
    double R[9];
#pragma unroll
    for (int k = 0; k < 9; k++) R[k] = a.R_lin[9 * oi + k];
    jac_ab(j, l.x, l.y, l.z, R, A, B);
    return l.w;
}

// ---------------------------------------------------------------------------
// buildSystem
// ---------------------------------------------------------------------------
// one thread per landmark: Hll, b_l over all its edges; stores each edge's linearisation (Pc, w)
// returns the largest |diagonal| of Hll (0 for m >= M)
// fresh: the stored errors belong to a rejected trial (an unsharded problem whose iteration ended
// on one): each edge's terms are taken from the restored state here, and stored, instead of read
__device__ __forceinline__ double lin_point(const BaArgs& a, int m, bool fresh = false) {
    if (m >= a.M) return 0.0;
    double H[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0}, bl[3] = {0, 0, 0};
    for (int k = a.pt_ptr[m]; k < a.pt_ptr[m + 1]; k++) {
        const int e = a.pt_edges[k];
        double x, y, z, R[9], j[4], A[6], B[12];
        edge_pc(a, e, x, y, z, R);
        proj_jac(a.fx, a.fy, x, y, z, j);
        jac_ab(j, x, y, z, R, A, B);
        double r1, er0, er1;
        if (fresh) {   // uniform
            double chi2, r0;
            edge_terms(a, e, x, y, z, er0, er1, chi2, r0, r1);
            store_terms(a, e, er0, er1, chi2, r0, r1);
        } else {
            r1 = a.e_rho1[e];
            er0 = a.e_err[2 * e];
            er1 = a.e_err[2 * e + 1];
        }
        const double info = a.e_info[e];
        const double w = r1 * info;
        const double om0 = -info * er0 * r1, om1 = -info * er1 * r1;
#pragma unroll
        for (int r = 0; r < 3; r++) {
            bl[r] += A[r] * om0 + A[3 + r] * om1;
#pragma unroll
            for (int c = 0; c < 3; c++) H[3 * r + c] += w * (A[r] * A[c] + A[3 + r] * A[3 + c]);
        }
        ((double4*)a.e_lin)[e] = make_double4(x, y, z, w);
    }
#pragma unroll
    for (int i = 0; i < 9; i++) a.Hll[9 * m + i] = H[i];
#pragma unroll
    for (int r = 0; r < 3; r++) a.b[a.n + 3 * m + r] = bl[r];
    return fmax(fmax(fabs(H[0]), fabs(H[4])), fabs(H[8]));
}
// the same with four lanes per landmark (k_ba_lin, r06): lane sub takes edges sub, sub + 4, ...
// of landmark m, the 12 sums are added over the quad (butterfly: the same bits in its lanes) and
// lane 0 stores them; returns the largest |diagonal| of Hll in every lane of the quad
constexpr int kLinL = 64;   // landmarks per workgroup of k_ba_lin
__device__ __forceinline__ double lin_point_quad(const BaArgs& a, int m, int sub, bool fresh) {
    if (m >= a.M) return 0.0;
    double H[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0}, bl[3] = {0, 0, 0};
    for (int k = a.pt_ptr[m] + sub; k < a.pt_ptr[m + 1]; k += 4) {
        const int e = a.pt_edges[k];
        double x, y, z, R[9], j[4], A[6], B[12];
        edge_pc(a, e, x, y, z, R);
        proj_jac(a.fx, a.fy, x, y, z, j);
        jac_ab(j, x, y, z, R, A, B);
        double r1, er0, er1;
        if (fresh) {   // uniform
            double chi2, r0;
            edge_terms(a, e, x, y, z, er0, er1, chi2, r0, r1);
            store_terms(a, e, er0, er1, chi2, r0, r1);
        } else {
            r1 = a.e_rho1[e];
            er0 = a.e_err[2 * e];
            er1 = a.e_err[2 * e + 1];
        }
        const double info = a.e_info[e];
        const double w = r1 * info;
        const double om0 = -info * er0 * r1, om1 = -info * er1 * r1;
#pragma unroll
        for (int r = 0; r < 3; r++) {
            bl[r] += A[r] * om0 + A[3 + r] * om1;
#pragma unroll
            for (int c = 0; c < 3; c++) H[3 * r + c] += w * (A[r] * A[c] + A[3 + r] * A[3 + c]);
        }
        ((double4*)a.e_lin)[e] = make_double4(x, y, z, w);
    }
#pragma unroll
    for (int o = 1; o <= 2; o <<= 1) {
#pragma unroll
        for (int i = 0; i < 9; i++) H[i] += __shfl_xor(H[i], o, 64);
#pragma unroll
        for (int r = 0; r < 3; r++) bl[r] += __shfl_xor(bl[r], o, 64);
    }
    if (sub == 0) {
#pragma unroll
        for (int i = 0; i < 9; i++) a.Hll[9 * m + i] = H[i];
#pragma unroll
        for (int r = 0; r < 3; r++) a.b[a.n + 3 * m + r] = bl[r];
    }
    return fmax(fmax(fabs(H[0]), fabs(H[4])), fabs(H[8]));
}
__global__ __launch_bounds__(256) void k_ba_lin_points(const BaArgs* __restrict__ args, const int* __restrict__ act) {
    BA_PROLOGUE
    BA_PHASE(kPhBuild)
    (void)lin_point(a, bx_ * blockDim.x + threadIdx.x);
}

// one wave per optimised pose: 21 upper Hpp terms + 6 b terms, lanes over the pose's edges; lane 0
// keeps the pose's rotation at the linearisation (R_lin)
// one halving step of a transpose-reduce: a lane with bit m clear keeps values [0, H), set keeps
// [H, 2H); each adds its partner's copy of the values it keeps; the kept values end in [0, H)
template <int H>
__device__ __forceinline__ void reduce_half(double* acc, int lane, int m) {
    const bool up = (lane & m) != 0;
#pragma unroll
    for (int i = 0; i < H; i++) {
        const double send = up ? acc[i] : acc[i + H];
        const double keep = up ? acc[i + H] : acc[i];
        acc[i] = keep + __shfl_xor(send, m, 64);
    }
}

// one wave per pose i; returns (in every lane) the largest |diagonal| of the pose's Hpp block
__device__ __forceinline__ double lin_pose(const BaArgs& a, int i, int lane, bool fresh = false) {
    if (i >= a.np) return 0.0;   // wave-uniform
    double acc[32];   // 27 sums (21 of the upper Hpp triangle, 6 of b_p), padded to 32
#pragma unroll
    for (int k = 0; k < 32; k++) acc[k] = 0;
    for (int k = a.ps_ptr[i] + lane; k < a.ps_ptr[i + 1]; k += 64) {
        const int e = a.ps_edges[k];
        double x, y, z, R[9], j[4], A[6], B[12];
        edge_pc(a, e, x, y, z, R);
        proj_jac(a.fx, a.fy, x, y, z, j);
        jac_ab(j, x, y, z, R, A, B);
        double r1, er0, er1;
        if (fresh) {   // uniform; the landmark side stores the same values
            double chi2, r0;
            edge_terms(a, e, x, y, z, er0, er1, chi2, r0, r1);
        } else {
            r1 = a.e_rho1[e];
            er0 = a.e_err[2 * e];
            er1 = a.e_err[2 * e + 1];
        }
        const double info = a.e_info[e];
        const double w = r1 * info;
        const double om0 = -info * er0 * r1, om1 = -info * er1 * r1;
        int t = 0;
#pragma unroll
        for (int r = 0; r < 6; r++)
#pragma unroll
            for (int c = r; c < 6; c++) acc[t++] += w * (B[r] * B[c] + B[6 + r] * B[6 + c]);
#pragma unroll
        for (int r = 0; r < 6; r++) acc[21 + r] += B[r] * om0 + B[6 + r] * om1;
    }
    // transpose-reduce over the 64 lanes: at each step a lane keeps half of its values and adds
    // its partner's copy of them (16 + 8 + 4 + 2 + 1 shuffles, then one for the last pair instead
    // of 27 x 6); lane 2k ends with sum k (k = the lane's bits 5..1, most significant first)
    reduce_half<16>(acc, lane, 32);
    reduce_half<8>(acc, lane, 16);
    reduce_half<4>(acc, lane, 8);
    reduce_half<2>(acc, lane, 4);
    reduce_half<1>(acc, lane, 2);
    const double tot = acc[0] + __shfl_xor(acc[0], 1, 64);
    const int k = ((lane >> 5) & 1) << 4 | ((lane >> 4) & 1) << 3 | ((lane >> 3) & 1) << 2 | ((lane >> 2) & 1) << 1 |
                  ((lane >> 1) & 1);
    double dmax = 0.0;
    if ((lane & 1) == 0 && k < 27) {
        double* H = a.Hpp + 36 * i;
        if (k < 21) {   // k-th entry of the upper triangle, row-major
            int r = 0, t = k;
            while (t >= 6 - r) { t -= 6 - r; r++; }
            const int c = r + t;
            H[6 * r + c] = tot;
            H[6 * c + r] = tot;
            if (r == c) dmax = fabs(tot);
        } else {
            a.b[6 * i + k - 21] = tot;
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) dmax = fmax(dmax, __shfl_xor(dmax, o, 64));
    if (lane < 9 && a.ps_ptr[i] < a.ps_ptr[i + 1]) {   // the pose's rotation, as its edges used it
        {
            const int p = a.e_pose[a.ps_edges[a.ps_ptr[i]]];
            double R[9];
            qtomat(load_q(a.pose + 8 * p), R);
            double r = R[0];
#pragma unroll
            for (int k = 1; k < 9; k++) r = lane == k ? R[k] : r;
            a.R_lin[9 * i + lane] = r;
        }
    }
    return dmax;
}
// the same with the whole work-group on pose i (r06, k_ba_lin with one pose per work-group): its
// four waves take edges lane, lane + 256, ... of the pose, each reduces its 27 sums as above, and
// wave 0 adds the four in wave order; returns the largest |diagonal| in wave 0 (0 in the others)
__device__ __forceinline__ double lin_pose_wg(const BaArgs& a, int i, bool fresh, double* sh27) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    if (i >= a.np) return 0.0;   // work-group-uniform
    double acc[32];
#pragma unroll
    for (int k = 0; k < 32; k++) acc[k] = 0;
    for (int k = a.ps_ptr[i] + (int)threadIdx.x; k < a.ps_ptr[i + 1]; k += blockDim.x) {
        const int e = a.ps_edges[k];
        double x, y, z, R[9], j[4], A[6], B[12];
        edge_pc(a, e, x, y, z, R);
        proj_jac(a.fx, a.fy, x, y, z, j);
        jac_ab(j, x, y, z, R, A, B);
        double r1, er0, er1;
        if (fresh) {
            double chi2, r0;
            edge_terms(a, e, x, y, z, er0, er1, chi2, r0, r1);
        } else {
            r1 = a.e_rho1[e];
            er0 = a.e_err[2 * e];
            er1 = a.e_err[2 * e + 1];
        }
        const double info = a.e_info[e];
        const double w = r1 * info;
        const double om0 = -info * er0 * r1, om1 = -info * er1 * r1;
        int t = 0;
#pragma unroll
        for (int r = 0; r < 6; r++)
#pragma unroll
            for (int c = r; c < 6; c++) acc[t++] += w * (B[r] * B[c] + B[6 + r] * B[6 + c]);
#pragma unroll
        for (int r = 0; r < 6; r++) acc[21 + r] += B[r] * om0 + B[6 + r] * om1;
    }
    reduce_half<16>(acc, lane, 32);
    reduce_half<8>(acc, lane, 16);
    reduce_half<4>(acc, lane, 8);
    reduce_half<2>(acc, lane, 4);
    reduce_half<1>(acc, lane, 2);
    const double tot = acc[0] + __shfl_xor(acc[0], 1, 64);
    const int k = ((lane >> 5) & 1) << 4 | ((lane >> 4) & 1) << 3 | ((lane >> 3) & 1) << 2 | ((lane >> 2) & 1) << 1 |
                  ((lane >> 1) & 1);
    if ((lane & 1) == 0 && k < 27) sh27[27 * wid + k] = tot;
    __syncthreads();
    double dmax = 0.0;
    if (wid == 0) {
        if (lane < 27) {
            const double v = (sh27[lane] + sh27[27 + lane]) + (sh27[54 + lane] + sh27[81 + lane]);
            double* H = a.Hpp + 36 * i;
            if (lane < 21) {   // lane-th entry of the upper triangle, row-major
                int r = 0, t = lane;
                while (t >= 6 - r) { t -= 6 - r; r++; }
                const int c = r + t;
                H[6 * r + c] = v;
                H[6 * c + r] = v;
                if (r == c) dmax = fabs(v);
            } else {
                a.b[6 * i + lane - 21] = v;
            }
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) dmax = fmax(dmax, __shfl_xor(dmax, o, 64));
        if (lane < 9 && a.ps_ptr[i] < a.ps_ptr[i + 1]) {   // the pose's rotation, as its edges used it
            const int p = a.e_pose[a.ps_edges[a.ps_ptr[i]]];
            double R[9];
            qtomat(load_q(a.pose + 8 * p), R);
            double r = R[0];
#pragma unroll
            for (int kk = 1; kk < 9; kk++) r = lane == kk ? R[kk] : r;
            a.R_lin[9 * i + lane] = r;
        }
    }
    return dmax;
}
__global__ __launch_bounds__(256) void k_ba_lin_poses(const BaArgs* __restrict__ args, const int* __restrict__ act) {
    BA_PROLOGUE
    BA_PHASE(kPhBuild)
    (void)lin_pose(a, bx_ * 4 + (threadIdx.x >> 6), threadIdx.x & 63);
}

// the device-driven build in one launch: workgroups [0, nbp) linearise landmarks (kLinL each,
// four lanes per landmark), the rest poses (one per wave); each stores its largest |diagonal| (sc1), and the
// problem's last workgroup runs the controller's trial start (ctl_begin_body: lambda from the
// maxima on the first iteration)
// ppw: poses per pose work-group, 4 (a wave each) or 1 (the whole work-group, lin_pose_wg)
__global__ __launch_bounds__(256) void k_ba_lin(const BaArgs* __restrict__ args, const int* __restrict__ act,
                                               int nbp, int ppw, int* const* donep) {
    BA_PROLOGUE
    BA_PHASE(kPhBuild)
    __shared__ double sh[4];
    __shared__ double sh27[4 * 27];
    __shared__ int lastf;
    const int mP = (a.M + kLinL - 1) / kLinL, nP = (a.np + ppw - 1) / ppw;
    // a problem whose iteration ended on a rejected trial: its stored errors are the trial's, so this
    // build takes them from the restored state (a small problem's restored in the trial's launch, a
    // larger one's by k_ba_pop). r06 (late): every unsharded problem, so the larger ones' slots lost
    // their k_ba_errors(1) launch (C5: one launch less per trial); the shards keep it
    const bool fresh = (a.small || !a.sync) && a.ctl && !a.ctl->errors_valid;
    double d;
    int slot;
    if (bx_ < nbp) {
        d = lin_point_quad(a, bx_ * kLinL + (threadIdx.x >> 2), threadIdx.x & 3, fresh);
        slot = bx_ < mP ? bx_ : -1;
    } else {
        const int q = bx_ - nbp;
        d = ppw == 1 ? lin_pose_wg(a, q, fresh, sh27) : lin_pose(a, q * 4 + (threadIdx.x >> 6), threadIdx.x & 63, fresh);
        slot = q < nP ? mP + q : -1;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) d = fmax(d, __shfl_xor(d, o, 64));
    __syncthreads();
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = d;
    __syncthreads();
    if (threadIdx.x == 0 && slot >= 0) {
        double m = 0.0;
        for (int w = 0; w < (int)(blockDim.x >> 6); w++) m = fmax(m, sh[w]);
        st_agent(a.part + slot, m);
    }
    if (!a.sync && last_arrival(&a.ctl->arrive_b, gridDim.x, &lastf))
        ctl_begin_body(a, mP + nP, done_of(donep), act[by_], sh);
}

// ---------------------------------------------------------------------------
// Schur complement
// ---------------------------------------------------------------------------
__device__ __forceinline__ void inv3(const double m[9], double r[9]) {
    const double c0 = m[4] * m[8] - m[5] * m[7];
    const double c1 = m[5] * m[6] - m[3] * m[8];
    const double c2 = m[3] * m[7] - m[4] * m[6];
    const double det = m[0] * c0 + m[1] * c1 + m[2] * c2;
    const double id = 1.0 / det;
    r[0] = c0 * id; r[3] = c1 * id; r[6] = c2 * id;
    r[1] = (m[2] * m[7] - m[1] * m[8]) * id;
    r[4] = (m[0] * m[8] - m[2] * m[6]) * id;
    r[7] = (m[1] * m[6] - m[0] * m[7]) * id;
    r[2] = (m[1] * m[5] - m[2] * m[4]) * id;
    r[5] = (m[2] * m[3] - m[0] * m[5]) * id;
    r[8] = (m[0] * m[4] - m[1] * m[3]) * id;
}

// Dinv of landmark m = (Hll + lambda I)^-1 (Eigen 3x3 cofactor inverse)
__device__ __forceinline__ void dinv_of(const BaArgs& a, int m, double Di[9]) {
    const double lambda = *a.lambda;
    double D[9];
#pragma unroll
    for (int k = 0; k < 9; k++) D[k] = a.Hll[9 * m + k] + (k % 4 == 0 ? lambda : 0.0);
    inv3(D, Di);
}

// one thread per landmark: setLambda on Hll, Dinv (Eigen 3x3 cofactor inverse), db = Dinv b_l.
// Fused trials (BaArgs::fused) skip this launch: every consumer forms Dinv (the same bits) itself
__global__ __launch_bounds__(256) void k_ba_schur_points(const BaArgs* __restrict__ args, const int* __restrict__ act) {
    BA_PROLOGUE
    BA_PHASE(kPhTrial)
    const int m = bx_ * blockDim.x + threadIdx.x;
    if (m >= a.M) return;
    const double lambda = *a.lambda;
    double D[9], Di[9];
#pragma unroll
    for (int k = 0; k < 9; k++) D[k] = a.Hll[9 * m + k] + (k % 4 == 0 ? lambda : 0.0);
    inv3(D, Di);
#pragma unroll
    for (int k = 0; k < 9; k++) a.Dinv[9 * m + k] = Di[k];
    const double* bl = a.b + a.n + 3 * m;
#pragma unroll
    for (int r = 0; r < 3; r++) a.db[3 * m + r] = Di[3 * r] * bl[0] + Di[3 * r + 1] * bl[1] + Di[3 * r + 2] * bl[2];
}

__global__ __launch_bounds__(256) void k_ba_zero_s(const BaArgs* __restrict__ args, const int* __restrict__ act,
                                                   int always) {
    BA_PROLOGUE
    if (!always) BA_PHASE(kPhTrial)
    const size_t nn = (size_t)a.n * a.n;
    double2* S2 = (double2*)a.S;
    for (size_t i = (size_t)bx_ * blockDim.x + threadIdx.x; i < nn / 2; i += (size_t)gridDim.x * blockDim.x)
        S2[i] = make_double2(0.0, 0.0);
    if (bx_ == 0 && threadIdx.x == 0 && (nn & 1)) a.S[nn - 1] = 0.0;
}

// Two LANES per Schur work item (a chunk of pairs of one 6x6 block (i, j)): lane half h owns rows
// 3h..3h+2 of the block, 18 sums in registers (the pair prologue is computed by both lanes: the
// register budget, not the flops, bounds this kernel). Matrix-free: for a pair (a, b) of edges of
// landmark m,
//   W_a Hpl_b^T = Hpl_a Dinv_m Hpl_b^T = w_a w_b B_a^T (A_a Dinv_m A_b^T) B_b
// with A, B rebuilt from the edges' stored (Pc, w) and the poses' R_lin: 17 doubles read per pair
// (edge records + Dinv) instead of the 36 of stored W / Hpl blocks, and no W written per trial.
constexpr int kItemsWg = 128;   // Schur work items per k_ba_schur_items work-group (two lanes each)
__device__ __forceinline__ void schur_b_pose(const BaArgs& a, int i, int lane);
// work-groups [nbi, gridDim.x) run k_ba_schur_b's poses instead (it reads only k_ba_schur_points'
// db and the linearisation: no dependence on the items, one launch less per trial)
__global__ __launch_bounds__(256) void k_ba_schur_items(const BaArgs* __restrict__ args, const int* __restrict__ act,
                                                        int nbi, int* const* donep) {
    BA_PROLOGUE
    if (donep && bx_ == (int)gridDim.x - 1) {   // the extra workgroup: the relayed stop flag
        if (by_ == 0 && threadIdx.x == 0) relay_host_stop(args, act, donep);
        return;
    }
    BA_PHASE(kPhTrial)
    if (bx_ >= nbi) {
        schur_b_pose(a, (bx_ - nbi) * 4 + (threadIdx.x >> 6), threadIdx.x & 63);
        return;
    }
    const int gt = bx_ * blockDim.x + threadIdx.x;
    const int it = gt >> 1, h = gt & 1;
    const int lane = threadIdx.x & 63;
    const bool valid = it < a.nitems;   // no early exit: the whole wave meets at the ballot below
    const int4 wi = valid ? ((const int4*)a.items)[it] : make_int4(0, 0, 0, -1);
    const int bi = valid && wi.z >= 0 ? a.blk_i[wi.z] : 0, bj = valid && wi.z >= 0 ? a.blk_j[wi.z] : 0;
    double Ri[9], Rj[9];
#pragma unroll
    for (int k = 0; k < 9; k++) { Ri[k] = a.R_lin[9 * bi + k]; Rj[k] = a.R_lin[9 * bj + k]; }
    double s[18];
#pragma unroll
    for (int k = 0; k < 18; k++) s[k] = 0.0;
    const double fx = a.fx, fy = a.fy;
    for (int k = wi.x; k < wi.y; k++) {
        const int2 pr = ((const int2*)a.blk_pairs)[k];
        const double4 la = ((const double4*)a.e_lin)[pr.x], lb = ((const double4*)a.e_lin)[pr.y];
        double Di[9];   // in registers either way (a pointer choice would put a local copy in scratch)
        if (a.fused) {
            dinv_of(a, a.e_pt[pr.x], Di);
        } else {
#pragma unroll
            for (int k = 0; k < 9; k++) Di[k] = a.Dinv[9 * a.e_pt[pr.x] + k];
        }
        // the projection Jacobians of both edges (proj_jac); A and B are used through their structure
        double ja[4], jb[4];
        proj_jac(fx, fy, la.x, la.y, la.z, ja);
        proj_jac(fx, fy, lb.x, lb.y, lb.z, jb);
        const double a00 = ja[0], a02 = ja[1], a11 = ja[2], a12 = ja[3];
        const double b00 = jb[0], b02 = jb[1], b11 = jb[2], b12 = jb[3];
        double T[6];   // A_a Dinv (2x3), A_a = [a00 Ri0 + a02 Ri2; a11 Ri1 + a12 Ri2]
#pragma unroll
        for (int c = 0; c < 3; c++) {
            const double d0 = Di[c], d1 = Di[3 + c], d2 = Di[6 + c];
            const double r0 = Ri[0] * d0 + Ri[1] * d1 + Ri[2] * d2;
            const double r1 = Ri[3] * d0 + Ri[4] * d1 + Ri[5] * d2;
            const double r2 = Ri[6] * d0 + Ri[7] * d1 + Ri[8] * d2;
            T[c] = a00 * r0 + a02 * r2;
            T[3 + c] = a11 * r1 + a12 * r2;
        }
        const double ww = la.w * lb.w;
        double C[4];   // w_a w_b A_a Dinv A_b^T (2x2)
#pragma unroll
        for (int c = 0; c < 2; c++) {
            const double jb0 = c == 0 ? b00 : b11, jb2 = c == 0 ? b02 : b12;
            double ab[3];
#pragma unroll
            for (int q = 0; q < 3; q++) ab[q] = jb0 * Rj[3 * c + q] + jb2 * Rj[6 + q];
#pragma unroll
            for (int r = 0; r < 2; r++) C[2 * r + c] = ww * (T[3 * r] * ab[0] + T[3 * r + 1] * ab[1] + T[3 * r + 2] * ab[2]);
        }
        // B_b rows: [b02 y, b00 z - b02 x, -b00 y, b00, 0, b02], [b12 y - b11 z, -b12 x, b11 x, 0, b11, b12]
        const double Bb0[6] = {b02 * lb.y, b00 * lb.z - b02 * lb.x, -b00 * lb.y, b00, 0.0, b02};
        const double Bb1[6] = {b12 * lb.y - b11 * lb.z, -b12 * lb.x, b11 * lb.x, 0.0, b11, b12};
        double CB0[6], CB1[6];   // C B_b (2x6)
#pragma unroll
        for (int c = 0; c < 6; c++) {
            CB0[c] = C[0] * Bb0[c] + C[1] * Bb1[c];
            CB1[c] = C[2] * Bb0[c] + C[3] * Bb1[c];
        }
        // this lane's rows of B_a^T: rows 3h..3h+2 of [a02 y, a00 z - a02 x, -a00 y, a00, 0, a02] and
        // [a12 y - a11 z, -a12 x, a11 x, 0, a11, a12]
        double u0[3], u1[3];
        if (h == 0) {
            u0[0] = a02 * la.y; u0[1] = a00 * la.z - a02 * la.x; u0[2] = -a00 * la.y;
            u1[0] = a12 * la.y - a11 * la.z; u1[1] = -a12 * la.x; u1[2] = a11 * la.x;
        } else {
            u0[0] = a00; u0[1] = 0.0; u0[2] = a02;
            u1[0] = 0.0; u1[1] = a11; u1[2] = a12;
        }
#pragma unroll
        for (int rr = 0; rr < 3; rr++)
#pragma unroll
            for (int cc = 0; cc < 6; cc++) s[6 * rr + cc] -= u0[rr] * CB0[cc] + u1[rr] * CB1[cc];
    }
    // r06: a block's chunks (consecutive items, all in this work-group: prepare pads) are summed
    // here, not by a finisher launch: every chunk's 36 values go to LDS at its item position and
    // the pair holding a block's first chunk lists the block (per wave, 32 slots); after the
    // barrier the work-group's threads take the listed blocks' entries, one (block, entry) each:
    // Hpp + lambda (diagonal, pose side), then the chunks in order (the r05 finisher's order),
    // into S. (r06 first tries: the partials handed over through global memory to the block's last
    // arrival, agent-scope stores, an atomic count and loads: 11 + 6 us (items + finisher) ->
    // 26-43 us per C4 trial; a segmented shuffle tree per wave run before an LDS hand-off: 16.5 us,
    // 3.5 of them the tree; each wave summing its own blocks, 36 lanes per block: 15.5 us.)
    __shared__ double parts[kItemsWg * 36];   // partial sums by item position in the work-group
    __shared__ int4 blist[4 * 32];            // per wave: {first item position, chunks, i, j}
    __shared__ int bcnt[4];
    const int li = it & (kItemsWg - 1), wv = threadIdx.x >> 6;
    const int myf = valid && wi.w >= 0 ? a.ifin[it] : -1;
    const bool first = myf >= 0 && h == 0 && wi.w == a.fin[3 * myf + 1];
    const int nch0 = first ? a.fin[3 * myf + 2] : 0;
    if (myf >= 0)
#pragma unroll
        for (int k = 0; k < 18; k++) parts[36 * li + 18 * h + k] = s[k];
    const unsigned long long om = __ballot(first);
    if (first) blist[32 * wv + __popcll(om & ((1ull << lane) - 1))] = make_int4(li, nch0, bi, bj);
    if (lane == 0) bcnt[wv] = __popcll(om);
    __syncthreads();
    if (valid && myf < 0 && wi.z >= 0) {   // a block of one chunk: straight into S (both triangles)
#pragma unroll
        for (int r = 0; r < 3; r++) {
            const int rr = 3 * h + r;
#pragma unroll
            for (int cc = 0; cc < 6; cc++) {
                a.S[(size_t)(6 * bi + rr) * a.n + 6 * bj + cc] = s[6 * r + cc];
                a.S[(size_t)(6 * bj + cc) * a.n + 6 * bi + rr] = s[6 * r + cc];
            }
        }
    }
    const int n0 = bcnt[0], n1 = n0 + bcnt[1], n2 = n1 + bcnt[2], nb = n2 + bcnt[3];
    if (nb == 0) return;
    const double lambda = *a.lambda;
    for (int q = threadIdx.x; q < 36 * nb; q += blockDim.x) {
        const int g = q / 36, e = q - 36 * g;   // block g of the work-group's list, entry e
        const int w = (g >= n0) + (g >= n1) + (g >= n2);
        const int4 B = blist[32 * w + g - (w == 0 ? 0 : w == 1 ? n0 : w == 2 ? n1 : n2)];
        const int i = B.z, j = B.w, rr = e / 6, cc = e - 6 * rr;
        double acc = i == j && (a.own ? a.own[i] != 0 : a.lead != 0)
                         ? a.Hpp_g[36 * i + 6 * rr + cc] + (rr == cc ? lambda : 0.0) : 0.0;
        const double* pp = parts + 36 * B.x + e;
        for (int c = 0; c < B.y; c++) acc += pp[36 * c];
        a.S[(size_t)(6 * i + rr) * a.n + 6 * j + cc] = acc;
        if (i != j) a.S[(size_t)(6 * j + cc) * a.n + 6 * i + rr] = acc;
    }
}

// one wave per optimised pose: b_schur = b_p - sum_e Hpl_e db, Hpl_e db = w B^T (A db)
__device__ __forceinline__ void schur_b_pose(const BaArgs& a, int i, int lane) {
    if (i >= a.np) return;
    double acc[6] = {0, 0, 0, 0, 0, 0};
    for (int k = a.ps_ptr[i] + lane; k < a.ps_ptr[i + 1]; k += 64) {
        const int e = a.ps_edges[k];
        double A[6], B[12];
        const double w = lin_ab(a, e, i, A, B);
        double d0, d1, d2;
        if (a.fused) {   // db = Dinv b_l, formed here
            const int m = a.e_pt[e];
            double Di[9];
            dinv_of(a, m, Di);
            const double* bl = a.b + a.n + 3 * m;
            d0 = Di[0] * bl[0] + Di[1] * bl[1] + Di[2] * bl[2];
            d1 = Di[3] * bl[0] + Di[4] * bl[1] + Di[5] * bl[2];
            d2 = Di[6] * bl[0] + Di[7] * bl[1] + Di[8] * bl[2];
        } else {
            const double* d = a.db + 3 * a.e_pt[e];
            d0 = d[0]; d1 = d[1]; d2 = d[2];
        }
        const double v0 = w * (A[0] * d0 + A[1] * d1 + A[2] * d2), v1 = w * (A[3] * d0 + A[4] * d1 + A[5] * d2);
#pragma unroll
        for (int r = 0; r < 6; r++) acc[r] += B[r] * v0 + B[6 + r] * v1;
    }
#pragma unroll
    for (int r = 0; r < 6; r++) {
        double v = acc[r];
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
        if (lane == 0) a.bs[6 * i + r] = a.b[6 * i + r] - v;
    }
}
__global__ __launch_bounds__(256) void k_ba_schur_b(const BaArgs* __restrict__ args, const int* __restrict__ act) {
    BA_PROLOGUE
    BA_PHASE(kPhTrial)
    schur_b_pose(a, bx_ * 4 + (threadIdx.x >> 6), threadIdx.x & 63);
}

// ---------------------------------------------------------------------------
// dense Cholesky of S (n x n, lower, in place) + solve S xp = bs; one workgroup (8 waves).
// Right-looking, 32-column panels:
//  (a) 32x32 diagonal block factored by ONE wavefront in registers (no block barrier per
//      pivot): lane = column c (+ row parity), 16 rows per lane, the block kept as a full
//      symmetric square so every cross-lane operand is one ds_bpermute. Gaussian elimination
//      on [D | I | y] gives L_u (unit LDL^T factor), L_u^{-1} and the forward-solve slice;
//      L11 = L_u diag(sqrt piv), L11^{-1} = diag(1/sqrt piv) L_u^{-1} at the panel end.
//  (b) the panel L21 = A21 Linv^T and the
//      trailing update C -= L21_I L21_J^T run on v_mfma_f64_16x16x4f64
//      (operand map: lane l holds A[l&15][k=l>>4], B[k=l>>4][l&15]; C/D col = l&15,
//      row = (l>>4) + 4*reg). Panel rows live in LDS (stride 34 doubles: conflict-free).
//  (c) backward solve panel by panel: x_p = Linv^T (y_p - L21^T x_below) (Linv saved per panel).
// ---------------------------------------------------------------------------
constexpr int kNB = 32;
constexpr int kSchurChunk = 16;    // pairs per Schur work item (one lane)
constexpr int kCholSmallN = 480;   // largest n of the single-workgroup solver (LDS envelope)
constexpr int kPS = 34;   // panel row stride in doubles

__host__ __device__ inline size_t chol_lds_doubles(int n) {
    const int np = (n + 31) & ~31;
    return (size_t)(2 + 32 * 33 + np + (size_t)np * kPS + 4 * 32 + 32 * 33);
}


__device__ __forceinline__ void chol_solve(double* __restrict__ S, const double* __restrict__ bs, double* __restrict__ x, int n,
                           int* __restrict__ flag, double* __restrict__ Lsave, unsigned long long* __restrict__ dbg) {
    extern __shared__ __attribute__((aligned(16))) double lds[];
    const int npad = (n + 31) & ~31;
    int& bad = *(int*)lds;                   // control word
    double* Li = lds + 2;                    // 32 x 33 L11^{-1}
    double* y = Li + 32 * 33;                // npad
    double* Pn = y + npad;                   // npad x kPS panel rows
    double* invp = Pn + (size_t)npad * kPS;  // 1/piv (raw pivot) per column of the panel
    double* dval = invp + 32;                // sqrt(piv)
    double* invd = dval + 32;                // 1/sqrt(piv)
    double* red = invd + 32;                 // 32 x 33 scratch (back-solve partial sums)
    const int tid = threadIdx.x, nt = blockDim.x;
    const int wid = tid >> 6, lane = tid & 63, nw = nt >> 6;
    unsigned long long tprev = 0;
    auto stamp = [&](int ph) {
        if (dbg && tid == 0) {
            const unsigned long long t = __builtin_amdgcn_s_memtime();
            if (ph >= 0) dbg[ph] += t - tprev;
            tprev = t;
        }
    };
    stamp(-1);
    if (tid == 0) bad = 0;
    for (int i = tid; i < npad; i += nt) y[i] = i < n ? bs[i] : 0.0;
    __syncthreads();
    for (int k0 = 0; k0 < n; k0 += kNB) {
        const int kb = min(kNB, n - k0);
        // ---- (a) diagonal block: wave 0, registers only ----
        if (wid == 0) chol_diag_wave(S, n, k0, kb, Li, Lsave, &bad);
        __syncthreads();
        // forward-solve slice y_p = L11^{-1} y_p (elimination applied to y)
        if (tid < 32) {
            double s2 = 0.0;
#pragma unroll 8
            for (int k = 0; k < 32; k++) s2 += Li[tid * 33 + k] * (k < kb ? y[k0 + k] : 0.0);
            invp[tid] = s2;
        }
        __syncthreads();
        if (tid < kb) y[k0 + tid] = invp[tid];
        stamp(0);
        if (bad) break;
        // ---- (b2) stage A21 rows into Pn ----
        const int r0 = k0 + kb;
        const int nr = n - r0;
        const int nr_pad = (nr + 15) & ~15;
        for (int t = tid; t < nr_pad * 32; t += nt) {
            const int rr = t >> 5, cI = t & 31;
            Pn[rr * kPS + cI] = (rr < nr && cI < kb) ? S[(size_t)(r0 + rr) * n + k0 + cI] : 0.0;
        }
        __syncthreads();
        // ---- (b3) L21 = A21 Linv^T on MFMA: one wave per 16-row block, both column halves ----
        const int cc = lane & 15, rq = lane >> 4;
        for (int R = wid; R < nr_pad / 16; R += nw) {
            double4_t acc0 = {0, 0, 0, 0}, acc1 = {0, 0, 0, 0};
#pragma unroll
            for (int kk = 0; kk < 8; kk++) {
                const double av = Pn[(16 * R + cc) * kPS + 4 * kk + rq];
                const double b0 = Li[cc * 33 + 4 * kk + rq];
                const double b1 = Li[(16 + cc) * 33 + 4 * kk + rq];
                acc0 = __builtin_amdgcn_mfma_f64_16x16x4f64(av, b0, acc0, 0, 0, 0);
                acc1 = __builtin_amdgcn_mfma_f64_16x16x4f64(av, b1, acc1, 0, 0, 0);
            }
            // all lanes' A reads of this row block are done before any write (wave-synchronous)
            __builtin_amdgcn_wave_barrier();
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const int rr = 16 * R + rq + 4 * q;
                Pn[rr * kPS + cc] = acc0[q];
                Pn[rr * kPS + 16 + cc] = acc1[q];
            }
        }
        __syncthreads();
        // ---- (b4) L21 back to S (coalesced rows); y_r -= L21[r] . y_panel (half-wave per row) ----
        for (int t = tid; t < nr * 32; t += nt) {
            const int rr = t >> 5, cI = t & 31;
            const double lv = Pn[rr * kPS + cI];
            if (cI < kb) S[(size_t)(r0 + rr) * n + k0 + cI] = lv;
            double dot = cI < kb ? lv * y[k0 + cI] : 0.0;
#pragma unroll
            for (int o = 16; o > 0; o >>= 1) dot += __shfl_xor(dot, o, 32);
            if (cI == 0) y[r0 + rr] -= dot;
        }
        stamp(1);
        // ---- (c) trailing update, lower 16x16 tiles, 4 tiles per wave per round ----
        const int T = nr_pad / 16;
        const int ntile = T * (T + 1) / 2;
        for (int base = wid; base < ntile; base += 4 * nw) {
            double4_t acc[4];
            int ti[4], tj[4];
            bool on[4];
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const int tile = base + u * nw;
                on[u] = tile < ntile;
                const int tt = on[u] ? tile : 0;
                int I = (int)((sqrtf(8.0f * (float)tt + 1.0f) - 1.0f) * 0.5f);
                while ((I + 1) * (I + 2) / 2 <= tt) I++;
                while (I * (I + 1) / 2 > tt) I--;
                ti[u] = I;
                tj[u] = tt - I * (I + 1) / 2;
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    const int rr = r0 + 16 * ti[u] + rq + 4 * q, col = r0 + 16 * tj[u] + cc;
                    acc[u][q] = (on[u] && rr < n && col < n) ? S[(size_t)rr * n + col] : 0.0;
                }
            }
#pragma unroll
            for (int u = 0; u < 4; u++) {
#pragma unroll
                for (int kk = 0; kk < kNB / 4; kk++) {
                    const double av = -Pn[(16 * ti[u] + cc) * kPS + 4 * kk + rq];
                    const double bv = Pn[(16 * tj[u] + cc) * kPS + 4 * kk + rq];
                    acc[u] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc[u], 0, 0, 0);
                }
            }
#pragma unroll
            for (int u = 0; u < 4; u++) {
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    const int rr = r0 + 16 * ti[u] + rq + 4 * q, col = r0 + 16 * tj[u] + cc;
                    if (on[u] && rr < n && col < n) S[(size_t)rr * n + col] = acc[u][q];
                }
            }
        }
        __syncthreads();
        stamp(2);
    }
    if (bad) {
        if (tid == 0) flag[0] = 0;
        for (int i = tid; i < n; i += nt) x[i] = 0.0;
        return;
    }
    // ---- (d) backward: x_p = Linv_p^T (y_p - L21_p^T x_below), panels from the last ----
    const int npan = (n + kNB - 1) / kNB;
    const int G = nt >> 5;
    for (int pb = npan - 1; pb >= 0; pb--) {
        const int k0 = pb * kNB, kb = min(kNB, n - k0);
        const int r0 = k0 + kb;
        {
            const int cI = tid & 31, g = tid >> 5;   // g = 0..G-1
            double s2 = 0.0;
            if (cI < kb)
                for (int r = r0 + g; r < n; r += G) s2 += S[(size_t)r * n + k0 + cI] * y[r];
            red[g * 33 + cI] = s2;
        }
        for (int t = tid; t < 32 * 32; t += nt) Li[(t >> 5) * 33 + (t & 31)] = Lsave[(size_t)pb * 1024 + t];
        __syncthreads();
        if (tid < 32) {
            double w = 0.0;
            if (tid < kb) {
                double s2 = 0.0;
                for (int g = 0; g < G; g++) s2 += red[g * 33 + tid];
                w = y[k0 + tid] - s2;
            }
            invp[tid] = w;                       // reuse as the 32-vector w
        }
        __syncthreads();
        if (tid < kb) {
            double s2 = 0.0;
#pragma unroll
            for (int k = 0; k < 32; k++) s2 += Li[k * 33 + tid] * invp[k];
            y[k0 + tid] = s2;
        }
        __syncthreads();
    }
    stamp(3);
    for (int i = tid; i < n; i += nt) x[i] = y[i];
    if (tid == 0) flag[0] = 1;
}

__global__ __launch_bounds__(512) void k_ba_cholesky(const BaArgs* __restrict__ args, const int* __restrict__ act) {
    const BaArgs& a = args[act[blockIdx.x]];
    BA_PHASE(kPhTrial)
    if (a.n == 0) {
        if (threadIdx.x == 0) a.flag[0] = 1;
        return;
    }
    chol_solve(a.S, a.bs, a.x, a.n, a.flag, a.Lsave, nullptr);
}

__global__ __launch_bounds__(512) void k_chol_test(double* S, const double* bs, double* x, int n, int* flag,
                                                   double* Lsave, unsigned long long* dbg) {
    chol_solve(S, bs, x, n, flag, Lsave, dbg);
}

// ---------------------------------------------------------------------------
// back-substitution + updates (push saves the old state)
// ---------------------------------------------------------------------------
// landmark m: xl = Dinv (b_l - Hpl^T xp), X += xl (old X saved); returns xl (lambda xl + b_l)
__device__ __forceinline__ double backsub_point(const BaArgs& a, int m) {
    const double* bl = a.b + a.n + 3 * m;
    double c[3] = {bl[0], bl[1], bl[2]};
    for (int k = a.pt_ptr[m]; k < a.pt_ptr[m + 1]; k++) {
        const int e = a.pt_edges[k];
        const int oi = a.opt[a.e_pose[e]];
        if (oi < 0) continue;
        double A[6], B[12];
        const double w = lin_ab(a, e, oi, A, B);   // Hpl_e^T xp = w A^T (B xp)
        const double* xp = a.x + 6 * oi;
        double u0 = 0.0, u1 = 0.0;
#pragma unroll
        for (int r = 0; r < 6; r++) { u0 += B[r] * xp[r]; u1 += B[6 + r] * xp[r]; }
        u0 *= w; u1 *= w;
#pragma unroll
        for (int cc = 0; cc < 3; cc++) c[cc] -= A[cc] * u0 + A[3 + cc] * u1;
    }
    double Di[9];
    if (a.fused) {
        dinv_of(a, m, Di);
    } else {
#pragma unroll
        for (int k = 0; k < 9; k++) Di[k] = a.Dinv[9 * m + k];
    }
    double* X = a.pts + 3 * m;
    const double lambda = *a.lambda;
    double sc = 0.0;
#pragma unroll
    for (int r = 0; r < 3; r++) {
        const double xl = Di[3 * r] * c[0] + Di[3 * r + 1] * c[1] + Di[3 * r + 2] * c[2];
        a.x[a.n + 3 * m + r] = xl;
        const double xo = X[r];
        // sc1 for a small problem: its trial's last workgroup may restore pts from pts_bak in
        // the same launch (ctl_end_body); the others' k_ba_pop runs in a launch of its own
        if (a.small) {
            st_agent(a.pts_bak + 3 * m + r, xo);
            st_agent(X + r, xo + xl);
        } else {
            a.pts_bak[3 * m + r] = xo;
            X[r] = xo + xl;
        }
        sc += xl * (lambda * xl + bl[r]);
    }
    return sc;
}

// one thread per landmark (back-substitution) and, in the first workgroups, one per pose
// (T <- exp(xp) T, the former k_ba_update_poses: it reads xp and writes the poses, which the
// landmarks' back-substitution does not touch)
__global__ __launch_bounds__(256) void k_ba_backsub(const BaArgs* __restrict__ args, const int* __restrict__ act) {
    BA_PROLOGUE
    BA_PHASE(kPhTrial)
    if (bx_ * (int)blockDim.x >= max(a.M, a.P)) return;   // uniform
    const int m = bx_ * blockDim.x + threadIdx.x;
    if (m < a.P) {
        double* T = a.pose + 8 * m;
#pragma unroll
        for (int k = 0; k < 8; k++) a.pose_bak[8 * m + k] = T[k];
        const int oi = a.opt[m];
        if (oi >= 0) se3_update(a.x + 6 * oi, T);
    }
    // the landmark part of computeScale, sum of xl (lambda xl + b_l), per workgroup (uniform: every
    // thread reaches the workgroup sum's barriers once)
    __shared__ double sh[4];
    const double t = block_sum(m < a.M ? backsub_point(a, m) : 0.0, sh);
    if (threadIdx.x == 0) a.part[a.npart_e + bx_] = t;
    if (bx_ == 0)   // the scale slots past this launch's workgroups (npart_m counts k_ba_backsub_errs')
        for (int i = (max(a.M, a.P) + 255) / 256 + (int)threadIdx.x; i < a.npart_m; i += blockDim.x)
            a.part[a.npart_e + i] = 0.0;
}

// the fused trial (BaArgs::fused; every unsharded problem since r06, small ones only before): the
// back-substitution and the trial's errors in ONE launch, no k_ba_schur_points before it and no
// k_ba_errors(2) after it. The trial's poses go to pose_bak (pose keeps the accepted state until
// the controller commits). Every workgroup forms all P new poses in LDS (P <= kFusedMaxP: a few
// se3 updates per thread, overlapping its landmark loads) and takes kBsL landmarks, four lanes per
// landmark (r06; one thread per landmark and 256 per workgroup before: 8 workgroups at C4): the
// lanes split the landmark's edges for Hpl^T xp (summed over the quad), each forms the new point
// (the same bits in all four) and then the errors of its own edges with it. chi2 and the landmark
// scale terms leave as workgroup partials and the problem's last workgroup runs the controller
// step (ctl_end_body: commit the poses or take the points back)
constexpr int kFusedMaxP = 512;
constexpr int kBsL = 64;   // landmarks per workgroup of k_ba_backsub_errs
__global__ __launch_bounds__(256) void k_ba_backsub_errs(const BaArgs* __restrict__ args, const int* __restrict__ act,
                                                         int* const* donep) {
    BA_PROLOGUE
    int* const done = done_of(donep);
    BA_PHASE(kPhTrial)
    __shared__ double Tn[8 * kFusedMaxP];   // the trial's poses
    __shared__ double sh[4];
    __shared__ int lastf;
    const int nwg = (max(a.M, a.P) + kBsL - 1) / kBsL;   // this problem's partial slots (<= npart_e, npart_m)
    const int m = bx_ * kBsL + (threadIdx.x >> 2), sub = threadIdx.x & 3;
    // this lane's edges of landmark m: its back-substitution terms (their loads go out first)
    int k0 = 0, k1 = 0;
    if (m < a.M) { k0 = a.pt_ptr[m]; k1 = a.pt_ptr[m + 1]; }
    // r06: the landmark's own words and this lane's first two edges' observation words are loaded
    // here, with the first loop's: after the barrier below everything would be loaded again, two
    // dependent round trips (edge list -> edge words) in front of the errors
    double Hm[9] = {}, blv[3] = {}, Xo[3] = {};
    if (m < a.M) {
#pragma unroll
        for (int k = 0; k < 9; k++) Hm[k] = a.Hll[9 * m + k];
#pragma unroll
        for (int r = 0; r < 3; r++) { blv[r] = a.b[a.n + 3 * m + r]; Xo[r] = a.pts[3 * m + r]; }
    }
    int ce[2] = {-1, -1}, cp[2] = {0, 0};
    double co0[2] = {0, 0}, co1[2] = {0, 0}, ci[2] = {0, 0};
    double c0 = 0.0, c1 = 0.0, c2 = 0.0;   // - sum_e Hpl_e^T xp over this lane's edges
    for (int k = k0 + sub, j = 0; k < k1; k += 4, j++) {
        const int e = a.pt_edges[k];
        const int pe = a.e_pose[e];
        if (j < 2) {
            ce[j] = e; cp[j] = pe;
            co0[j] = a.e_obs[2 * e]; co1[j] = a.e_obs[2 * e + 1]; ci[j] = a.e_info[e];
        }
        const int oi = a.opt[pe];
        if (oi < 0) continue;
        double A[6], B[12];
        const double w = lin_ab(a, e, oi, A, B);   // Hpl_e^T xp = w A^T (B xp)
        const double* xp = a.x + 6 * oi;
        double u0 = 0.0, u1 = 0.0;
#pragma unroll
        for (int r = 0; r < 6; r++) { u0 += B[r] * xp[r]; u1 += B[6 + r] * xp[r]; }
        u0 *= w; u1 *= w;
        c0 -= A[0] * u0 + A[3] * u1;
        c1 -= A[1] * u0 + A[4] * u1;
        c2 -= A[2] * u0 + A[5] * u1;
    }
    for (int p = threadIdx.x; p < a.P; p += blockDim.x) {
        double T[8];
#pragma unroll
        for (int k = 0; k < 8; k++) T[k] = a.pose[8 * p + k];
        const int oi = a.opt[p];
        if (oi >= 0) se3_update(a.x + 6 * oi, T);
#pragma unroll
        for (int k = 0; k < 8; k++) Tn[8 * p + k] = T[k];
        if (bx_ == 0) {   // sc1: read back by the problem's last workgroup in this launch
#pragma unroll
            for (int k = 0; k < 8; k++) st_agent(a.pose_bak + 8 * p + k, T[k]);
        }
    }
    // the quad's sum (butterfly: the same bits in its four lanes)
    c0 += __shfl_xor(c0, 1, 64); c1 += __shfl_xor(c1, 1, 64); c2 += __shfl_xor(c2, 1, 64);
    c0 += __shfl_xor(c0, 2, 64); c1 += __shfl_xor(c1, 2, 64); c2 += __shfl_xor(c2, 2, 64);
    double sc = 0.0, Xn[3] = {0.0, 0.0, 0.0};
    if (m < a.M) {   // xl = Dinv (b_l - Hpl^T xp), X += xl (old X saved): every lane of the quad
        const double cv[3] = {blv[0] + c0, blv[1] + c1, blv[2] + c2};
        const double lambda = *a.lambda;
        double D[9], Di[9];   // dinv_of's expressions on the preloaded Hll
#pragma unroll
        for (int k = 0; k < 9; k++) D[k] = Hm[k] + (k % 4 == 0 ? lambda : 0.0);
        inv3(D, Di);
        double* X = a.pts + 3 * m;
#pragma unroll
        for (int r = 0; r < 3; r++) {
            const double xl = Di[3 * r] * cv[0] + Di[3 * r + 1] * cv[1] + Di[3 * r + 2] * cv[2];
            const double xo = Xo[r];
            Xn[r] = xo + xl;
            if (sub == 0) {
                a.x[a.n + 3 * m + r] = xl;
                // sc1 for a small problem: its trial's last workgroup may restore pts from pts_bak
                // in this launch (ctl_end_body)
                st_agent(a.pts_bak + 3 * m + r, xo);
                st_agent(X + r, Xn[r]);
                sc += xl * (lambda * xl + blv[r]);
            }
        }
    }
    __syncthreads();   // the trial's poses in Tn
    double chi = 0.0;
    for (int k = k0 + sub, j = 0; k < k1; k += 4, j++) {
        if (j < 2) {   // from the preloaded words (edge_error_at's expressions)
            const int e = ce[j];
            const double* T = Tn + 8 * cp[j];
            double cx, cy, cz;
            qrot(load_q(T), Xn[0], Xn[1], Xn[2], cx, cy, cz);
            cx += T[4]; cy += T[5]; cz += T[6];
            const double u = a.fx * cx / cz + a.cx, v = a.fy * cy / cz + a.cy;
            const double e0 = co0[j] - u, e1 = co1[j] - v;
            const double chi2 = ci[j] * (e0 * e0 + e1 * e1);
            double r0 = chi2, r1 = 1.0;
            if (a.delta > 0) {
                const double dsqr = a.delta * a.delta;
                if (chi2 > dsqr) {
                    const double sq = sqrt(chi2);
                    r0 = 2 * sq * a.delta - dsqr;
                    r1 = a.delta / sq;
                }
            }
            store_terms(a, e, e0, e1, chi2, r0, r1);
            chi += r0;
        } else {
            const int e = a.pt_edges[k];
            chi += edge_error_at(a, e, Tn + 8 * a.e_pose[e], Xn);
        }
    }
    const double tc = block_sum(chi, sh);
    const double ts = block_sum(sc, sh);
    if (threadIdx.x == 0 && bx_ < nwg) {
        st_agent(a.part + bx_, tc);
        st_agent(a.part + a.npart_e + bx_, ts);
    }
    if (bx_ == 0) {   // the slots past this problem's workgroups
        for (int i = nwg + (int)threadIdx.x; i < a.npart_e; i += blockDim.x) st_agent(a.part + i, 0.0);
        for (int i = nwg + (int)threadIdx.x; i < a.npart_m; i += blockDim.x) st_agent(a.part + a.npart_e + i, 0.0);
    }
    if (last_arrival(&a.ctl->arrive_t, gridDim.x, &lastf)) ctl_end_body(a, act[by_], done, sh);
}

// restore the pushed state: host-driven rounds list the rejected problems in act[]; device-driven
// rounds restore every problem whose controller flagged its trial rejected (ctl->pop)
__global__ __launch_bounds__(256) void k_ba_pop(const BaArgs* __restrict__ args, const int* __restrict__ act) {
    BA_PROLOGUE
    if (a.ctl && !a.ctl->pop) return;
    const int i = bx_ * blockDim.x + threadIdx.x;
    // (a fused trial left the poses unmoved: pose_bak holds the rejected trial's)
    if (i < 8 * a.P && !a.fused) a.pose[i] = a.pose_bak[i];
    if (i < 3 * a.M) a.pts[i] = a.pts_bak[i];
}

// red[0..3] + flag of the active problems packed contiguously for ONE device->host copy
__global__ void k_ba_gather_red(const BaArgs* __restrict__ args, const int* __restrict__ act, int nact,
                                double* __restrict__ out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nact) return;
    const BaArgs& a = args[act[i]];
    for (int k = 0; k < 4; k++) out[5 * i + k] = a.red[k];
    out[5 * i + 4] = (double)a.flag[0];
}

// ---------------------------------------------------------------------------
// reductions (one workgroup per problem, fixed order): [0] sum rho0, [1] scale, [2] max diag
// ---------------------------------------------------------------------------
// In-batch model of the sharded solve: problems 0..B-1 are shards of one problem (same poses,
// disjoint landmarks); every shard's field[off .. off+count) becomes the sum (op 0) or max
// (op 1) over the shards, in shard order (deterministic). field: 0 Hpp, 1 S, 2 bs, 3 red.
__device__ __forceinline__ double* shard_field(const BaArgs& a, int field) {
    return field == 0 ? a.Hpp : (field == 1 ? a.S : (field == 2 ? a.bs : a.red));
}
__global__ __launch_bounds__(256) void k_ba_shard_reduce(const BaArgs* __restrict__ args, int B, int field, int off,
                                                         size_t count, int op) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < count; i += (size_t)gridDim.x * blockDim.x) {
        double acc = op ? -1.0e300 : 0.0;
        for (int b = 0; b < B; b++) {
            const double v = shard_field(args[b], field)[off + i];
            acc = op ? fmax(acc, v) : acc + v;
        }
        for (int b = 0; b < B; b++) shard_field(args[b], field)[off + i] = acc;
    }
}

// Envelope packing of S for the sharded all-reduce: 32-row tile R keeps columns [32 rf[R],
// 32 R + 32) (the lower envelope, which is all any Cholesky here reads; outside it every shard's
// S is zero), packed row-major per tile at toff[R]. pack (dir 0) S -> buf, unpack (dir 1) buf -> S.
__global__ __launch_bounds__(256) void k_ba_env_pack(double* __restrict__ S, int n, const int* __restrict__ rf,
                                                     const long long* __restrict__ toff, double* __restrict__ buf,
                                                     int dir) {
    const int R = blockIdx.y;
    const int c0 = 32 * rf[R], c1 = min(32 * R + 32, n), w = c1 - c0;
    const int rows = min(32, n - 32 * R);
    double* tb = buf + toff[R];
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < rows * w; i += gridDim.x * blockDim.x) {
        const int r = i / w, c = i - r * w;
        double* e = S + (size_t)(32 * R + r) * n + c0 + c;
        if (dir == 0) tb[i] = *e;
        else *e = tb[i];
    }
}

__device__ void ba_reduce_body(const BaArgs& a, int what, double* sh) {
    double v = 0;
    if (what & 1) {
        for (int e = threadIdx.x; e < a.E; e += blockDim.x) v += a.e_rho0[e];
        v = block_sum(v, sh);
        if (threadIdx.x == 0) a.red[0] = v;
    }
    if (what & 2) {
        const double lambda = *a.lambda;
        const double lam_pose = a.lead ? lambda : 0.0;   // pose x is replicated across shards
        v = 0;
        const int N = a.n + 3 * a.M;
        for (int j = threadIdx.x; j < N; j += blockDim.x) v += a.x[j] * ((j < a.n ? lam_pose : lambda) * a.x[j] + a.b[j]);
        v = block_sum(v, sh);
        if (threadIdx.x == 0) a.red[1] = v;
    }
    if (what & 4) {
        v = 0;
        for (int i = threadIdx.x; i < a.np * 6; i += blockDim.x) v = fmax(v, fabs(a.Hpp[36 * (i / 6) + 7 * (i % 6)]));
        for (int i = threadIdx.x; i < a.M * 3; i += blockDim.x) v = fmax(v, fabs(a.Hll[9 * (i / 3) + 4 * (i % 3)]));
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, 64));
        __syncthreads();
        if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
        __syncthreads();
        if (threadIdx.x == 0) {
            double m = 0;
            for (int i = 0; i < (int)(blockDim.x >> 6); i++) m = fmax(m, sh[i]);
            a.red[2] = m;
        }
    }
    if ((what & 8) && threadIdx.x == 0) a.red[3] = a.flag[0] ? 0.0 : 1.0;   // the solve failed (summed over ranks)
}

__global__ __launch_bounds__(1024) void k_ba_reduce(const BaArgs* __restrict__ args, const int* __restrict__ act,
                                                    int what) {
    __shared__ double sh[16];
    ba_reduce_body(args[act[blockIdx.x]], what, sh);
}

// ---------------------------------------------------------------------------
// device-driven Levenberg-Marquardt control: one slot = [pre] build kernels [begin] trial kernels
// [end] pop. The rules are those of the host-driven rounds in ba_solve_batch (g2o
// OptimizationAlgorithmLevenberg::solve + SparseOptimizer::optimize, U:Thirdparty/g2o), applied
// per problem on the device so that a whole solve needs no host round trip per trial.
// ---------------------------------------------------------------------------
// initial activeRobustChi2 (errors computed by the preceding k_ba_errors)
__global__ __launch_bounds__(1024) void k_ba_ctl_init(const BaArgs* __restrict__ args, const int* __restrict__ act) {
    __shared__ double sh[16];
    const BaArgs& a = args[act[blockIdx.x]];
    ba_reduce_body(a, 1, sh);
    if (threadIdx.x == 0) {
        LmCtl& c = *a.ctl;
        c.currentChi = a.red[0];
        c.initChi = a.red[0];
    }
}

// the host's stop request (LocalMapping mbAbortBA): a problem between iterations ends now, one in a
// trial at the end of its iteration (ctl_end_decide)
__global__ void k_ba_ctl_stop(LmCtl* __restrict__ ctl, int B, int* const* donep) {
    int* const done = done_of(donep);
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    ctl[b].stop = 1;
    if (ctl[b].phase == kPhBuild) {
        ctl[b].phase = kPhDone;
        post_done(done, b);
    }
}

// after the build: lambda initialisation on the first iteration (1e-5 max diagonal, from k_ba_lin's
// per-workgroup maxima: sc1 loads), then trials. Run by the last workgroup of k_ba_lin.
__device__ void ctl_begin_apply(const BaArgs& a, double maxdiag) {
    LmCtl& c = *a.ctl;
    if (c.it == 0) {
        *const_cast<double*>(a.lambda) = 1e-5 * maxdiag;
        c.ni = 2;
        c.nBad = 0;
    }
    c.qmax = 0;
    c.rho = 0;
    c.errors_valid = 1;   // the build just done used the current state's errors
    c.phase = kPhTrial;
}
// every thread of the work-group calls it: on the first iteration the largest diagonal over the
// build's nlin work-group maxima is a block reduction (r06: thread 0 alone read them one after
// another, 94 us of the first C5 build for its 712 partials)
__device__ void ctl_begin_body(const BaArgs& a, int nlin, int* done_flags, int prob, double* sh) {
    double m = 0.0;
    if (a.ctl->it == 0) {   // block-uniform: written by an earlier launch
        for (int i = threadIdx.x; i < nlin; i += blockDim.x) m = fmax(m, ld_agent(a.part + i));
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) m = fmax(m, __shfl_xor(m, o, 64));
        __syncthreads();
        if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = m;
        __syncthreads();
        for (int w = 0; w < (int)(blockDim.x >> 6); w++) m = fmax(m, sh[w]);
    }
    if (threadIdx.x != 0) return;
    if (a.ctl->stop) {   // a stop relayed before this iteration: g2o's terminate() check, no trial
        LmCtl& c = *a.ctl;
        c.phase = kPhDone;
        post_done(done_flags, prob);
        return;
    }
    ctl_begin_apply(a, m);
}

// after a trial: chi2 and scale, rho, accept (lambda shrink) or reject (lambda *= ni, pop), and
// the end-of-iteration rules. Run by the last workgroup of k_ba_errors(2) of the problem: the chi2
// partials are that launch's (sc1 loads), the scale partials k_ba_backsub's.
__device__ void ctl_end_sums(const BaArgs& a, double* sh) {
    {   // chi2 and the scale from the trial kernels' workgroup partials (k_ba_errors, k_ba_backsub)
        double v = 0.0;
        for (int i = threadIdx.x; i < a.npart_e; i += blockDim.x) v += ld_agent(a.part + i);
        v = block_sum(v, sh);
        if (threadIdx.x == 0) a.red[0] = v;
        const double lambda = *a.lambda, lam_pose = a.lead ? lambda : 0.0;
        v = 0.0;
        for (int j = threadIdx.x; j < a.n; j += blockDim.x) v += a.x[j] * (lam_pose * a.x[j] + a.b[j]);
        for (int i = threadIdx.x; i < a.npart_m; i += blockDim.x) v += ld_agent(a.part + a.npart_e + i);
        v = block_sum(v, sh);
        if (threadIdx.x == 0) a.red[1] = v;
    }
}
// thread 0: the g2o rules on red[0] (chi2) and red[1] (scale)
__device__ void ctl_end_decide(const BaArgs& a, int prob, int* done_flags) {
    LmCtl& c = *a.ctl;
    double* lambda = const_cast<double*>(a.lambda);
    const bool ok2 = a.flag[0] != 0;
    const double tempChi = ok2 ? a.red[0] : DBL_MAX;
    double rho = c.currentChi - tempChi;
    rho /= (a.red[1] + 1e-3);
    if (rho > 0 && isfinite(tempChi)) {
        double alpha = 1. - pow((2 * rho - 1), 3.0);
        alpha = fmin(alpha, 2. / 3.);
        *lambda *= fmax(1. / 3., alpha);
        c.ni = 2;
        if (c.early_stop) {
            if ((c.currentChi - tempChi) < 1e-3 * c.currentChi) c.nBad++;
            else c.nBad = 0;
        }
        c.currentChi = tempChi;
        c.pop = 0;
    } else {
        *lambda *= c.ni;
        c.ni *= 2;
        c.pop = 1;
    }
    c.rho = rho;
    c.qmax++;
    c.trials++;
    if (rho < 0 && c.qmax < 10 && !c.stop) return;   // another trial of this iteration
    c.it++;
    c.errors_valid = rho > 0;   // rejected: the device errors belong to the popped trial
    bool done = (c.qmax == 10 || rho == 0) || c.stop;   // stop: SparseOptimizer's force-stop, at the iteration end
    if (c.early_stop && c.nBad >= 3) done = true;
    if (c.it >= c.iterations) done = true;   // the budget (a sharded slot's k_ba_errors(1) checks it too), no idle slot
    c.phase = done ? kPhDone : kPhBuild;
    if (done) post_done(done_flags, prob);
}
__device__ void ctl_end_body(const BaArgs& a, int prob, int* done_flags, double* sh) {
    ctl_end_sums(a, sh);
    if (threadIdx.x == 0) ctl_end_decide(a, prob, done_flags);
    if (!a.small && !a.fused) return;
    // a small problem: this workgroup restores a rejected trial's state (k_ba_pop), so that needs
    // no launch of its own (the restored state's errors, g2o's computeActiveErrors at the next
    // iteration's start, come from the next k_ba_lin).
    // Fused trials (k_ba_backsub_errs) left the poses unmoved and the new ones in pose_bak: an
    // accepted trial commits them, a rejected one only takes the points back
    __syncthreads();
    // The backups and the trial's points / errors were stored by other workgroups of this launch
    // (other XCDs) with sc1 stores drained before their arrival: sc1 loads here see them, and the
    // sc1 stores below are the last writes of those words.
    const LmCtl& c = *a.ctl;
    if (a.fused) {
        if (!c.pop) {
            for (int i = threadIdx.x; i < 8 * a.P; i += blockDim.x) st_agent(a.pose + i, ld_agent(a.pose_bak + i));
            return;
        }
        // r06: larger problems take the fused trial too; their points come back in k_ba_pop (3M
        // words are too many for this one work-group)
        if (!a.small) return;
    } else {
        if (!c.pop) return;
        for (int i = threadIdx.x; i < 8 * a.P; i += blockDim.x) st_agent(a.pose + i, ld_agent(a.pose_bak + i));
    }
    for (int i = threadIdx.x; i < 3 * a.M; i += blockDim.x) st_agent(a.pts + i, ld_agent(a.pts_bak + i));
    // the restored state's errors, when the iteration ended here, are taken by the next build
    // (k_ba_lin's fresh terms): rewritten here, in this launch, they raced the other workgroups'
    // plain stores of the trial's errors
}

// ---- sharded device-driven rounds (BaArgs::sync): the controller's reductions, a collective
// over the shards, then its decisions, each a launch of one workgroup per problem ----
// build: red[2] = the largest |diagonal| (landmarks: k_ba_lin's workgroup maxima; poses: the
// summed Hpp_g, since a shard's own Hpp holds only its edges' terms)
__global__ __launch_bounds__(256) void k_ba_sh_maxdiag(const BaArgs* __restrict__ args, const int* __restrict__ act) {
    const BaArgs& a = args[act[blockIdx.x]];
    if (!in_phase(a, kPhBuild)) return;
    const int mP = (a.M + kLinL - 1) / kLinL;   // k_ba_lin's landmark workgroups
    double m = 0.0;
    for (int i = threadIdx.x; i < mP; i += blockDim.x) m = fmax(m, ld_agent(a.part + i));
    for (int i = threadIdx.x; i < 6 * a.np; i += blockDim.x) m = fmax(m, fabs(a.Hpp_g[36 * (i / 6) + 7 * (i % 6)]));
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = fmax(m, __shfl_xor(m, o, 64));
    __shared__ double sh[4];
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) a.red[2] = fmax(fmax(sh[0], sh[1]), fmax(sh[2], sh[3]));
}
__global__ void k_ba_sh_init(const BaArgs* __restrict__ args, const int* __restrict__ act) {
    const BaArgs& a = args[act[blockIdx.x]];
    if (threadIdx.x == 0) { a.ctl->currentChi = a.red[0]; a.ctl->initChi = a.red[0]; }
}
__global__ void k_ba_sh_begin(const BaArgs* __restrict__ args, const int* __restrict__ act) {
    const BaArgs& a = args[act[blockIdx.x]];
    if (threadIdx.x == 0 && in_phase(a, kPhBuild)) ctl_begin_apply(a, a.red[2]);
}
__global__ __launch_bounds__(1024) void k_ba_sh_sums(const BaArgs* __restrict__ args, const int* __restrict__ act) {
    __shared__ double sh[16];
    const BaArgs& a = args[act[blockIdx.x]];
    if (in_phase(a, kPhTrial)) ctl_end_sums(a, sh);
}
__global__ void k_ba_sh_end(const BaArgs* __restrict__ args, const int* __restrict__ act, int* const* donep) {
    int* const done = done_of(donep);
    const BaArgs& a = args[act[blockIdx.x]];
    if (threadIdx.x == 0 && in_phase(a, kPhTrial)) ctl_end_decide(a, act[blockIdx.x], done);
}
// the in-process form of a collective over B shards: dst[s][i] = sum (op 0) / max (op 1) over the
// shards of src[s'][i], in shard order (deterministic); dst may alias src
// sum (op 0) or max (op 1) of nsrc buffers into each of ndst buffers (a destination may alias a
// source: every element is read before it is written, by the same thread)
__global__ __launch_bounds__(256) void k_ba_multi_reduce(const double* const* __restrict__ src, int nsrc,
                                                         double* const* __restrict__ dst, int ndst, size_t count, int op) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < count; i += (size_t)gridDim.x * blockDim.x) {
        double acc = op ? -1.0e300 : 0.0;
        for (int b = 0; b < nsrc; b++) {
            const double v = src[b][i];
            acc = op ? fmax(acc, v) : acc + v;
        }
        for (int b = 0; b < ndst; b++) dst[b][i] = acc;
    }
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
#define BAOK(x)                                                                                    \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess) {                                                                    \
            std::fprintf(stderr, "orbhip ba: %s: %s\n", #x, hipGetErrorString(e_));                \
            return ORBHIP_ERR_DEVICE;                                                              \
        }                                                                                          \
    } while (0)

namespace {

// per-problem host preparation (O(E)): index mapping, CSRs, Schur pair lists by counting sort
struct Prep {
    int rc = 0;
    int P = 0, M = 0, E = 0, np = 0, n = 0, nblk = 0;
    std::vector<int> opt, pt_ptr, pt_edges, ps_ptr, ps_edges, blk_i, blk_j, blk_ptr, blk_pairs;
    std::vector<int> row_first;   // blocked Cholesky structure: first 32-col tile per 32-row tile
    std::vector<int> cb_tiles, cb_off;   // blocked Cholesky: envelope tiles per panel (cb_envelope_tiles)
    std::vector<int> items, fin;  // Schur work items {k0, k1, blk, slot} and finisher blocks {blk, slot0, n}
    std::vector<int> ifin;        // each item's finisher entry (-1: the block's only item)
    int nslot = 0;
    bool use_dag = false;         // the persistent tiled-DAG Cholesky (ba_chol_dag.hip)
    DagPlan dag;                  // its helper task lists
    bool use_nd = false;          // nested dissection over the DAG solver (ba_nd.hip): a lone banded GBA
    NdPlan nd;
    bool use_nd_sh = false;       // a shard of a sharded solve by keyframe segments (segment = shard)
    std::vector<unsigned char> own;   // ... the poses whose pose-side terms it adds
    size_t dag_task_cap = 0;      // ints reserved for the lists (RCCL shards: planned after the union envelope)
    size_t o_dag = 0, o_dagi = 0;
    size_t o_red2 = 0;            // workgroup partials of a trial's chi2 / scale (BaArgs::part)
    // offsets (elements) into the packed buffers; see the segment map in ba_solve_batch
    size_t o_chi2 = 0, o_state = 0, o_obs = 0, o_scr = 0, o_lin = 0, o_S = 0, o_L = 0, o_int = 0;
};

// fn(i) for i in [0, n) on up to `threads` host threads (problems are independent)
template <typename F>
void parallel_for(int n, int threads, F fn) {
    threads = std::max(1, std::min(threads, n));
    if (threads == 1) {
        for (int i = 0; i < n; i++) fn(i);
        return;
    }
    std::atomic<int> next{0};
    auto work = [&] {
        for (int i; (i = next.fetch_add(1)) < n;) fn(i);
    };
    std::vector<std::thread> pool;
    for (int t = 1; t < threads; t++) pool.emplace_back(work);
    work();
    for (auto& th : pool) th.join();
}

int host_threads() {
    static const int n = [] {
        const char* s = std::getenv("ORBHIP_BA_THREADS");
        if (s && std::atoi(s) > 0) return std::atoi(s);
        const unsigned hw = std::thread::hardware_concurrency();
        return (int)std::min<unsigned>(16, hw ? hw : 1);
    }();
    return n;
}

constexpr int kPrepParallelE = 20000;   // edges from which one problem's pair lists use host threads

// A persistent host worker pool for the preparation of one large problem: run(n, fn) calls fn(i)
// for i in [0, n) on the caller and the idle workers (indices claimed dynamically, so it completes
// on the caller alone if no worker is free), and returns when every call has returned. One run at a
// time: a concurrent caller (another context's thread) runs its loop alone.
// Created lazily, on the first large problem prepared with ORBHIP_PREP_THREADS > 1 (never
// otherwise), and deliberately leaked with detached workers: no destructor runs at process exit
// or library unload, so no join can meet a worker inside run() or a destroyed mutex.
class HostPool {
  public:
    static HostPool& get(int workers) {
        static HostPool* pool = new HostPool(workers);
        return *pool;
    }
    template <typename F>
    void run(int n, F&& fn) {
        std::unique_lock<std::mutex> busy(run_m_, std::try_to_lock);
        if (!busy.owns_lock() || workers_.empty()) {
            for (int i = 0; i < n; i++) fn(i);
            return;
        }
        std::function<void(int)> job(fn);
        {
            std::lock_guard<std::mutex> g(m_);
            job_ = &job;
            n_ = n;
            next_.store(0, std::memory_order_relaxed);
            active_ = (int)workers_.size();
            gen_++;
        }
        cv_.notify_all();
        for (int i; (i = next_.fetch_add(1)) < n;) job(i);
        std::unique_lock<std::mutex> g(m_);
        done_cv_.wait(g, [&] { return active_ == 0; });   // every worker has left this job
        job_ = nullptr;
    }

  private:
    explicit HostPool(int workers) {
        for (int w = 0; w < workers; w++) {
            std::thread t([this] { loop(); });
            t.detach();
            workers_.push_back(w);
        }
    }
    ~HostPool() = delete;   // leaked (see above)
    void loop() {
        unsigned long long seen = 0;
        for (;;) {
            std::function<void(int)>* job;
            int n;
            {
                std::unique_lock<std::mutex> g(m_);
                cv_.wait(g, [&] { return gen_ != seen; });
                seen = gen_;
                job = job_;
                n = n_;
            }
            if (job)
                for (int i; (i = next_.fetch_add(1)) < n;) (*job)(i);
            std::lock_guard<std::mutex> g(m_);
            if (--active_ == 0) done_cv_.notify_one();
        }
    }
    std::vector<int> workers_;   // the detached workers' indices (their count is what run() uses)
    std::mutex run_m_, m_;
    std::condition_variable cv_, done_cv_;
    std::function<void(int)>* job_ = nullptr;
    int n_ = 0, active_ = 0;
    std::atomic<int> next_{0};
    unsigned long long gen_ = 0;
};

// r06 (late): one large problem (E >= kPrepParallelE, a GBA) writes its outputs on the pool (C5
// 0.146 -> 0.05 ms; its pair lists and packing measured slower there, tools/r06/gpu_hostpool_ab.sh);
// ORBHIP_HOST_POOL=0 keeps every host loop on the calling thread
bool host_pool_on() {
    static const bool on = [] {
        const char* s = std::getenv("ORBHIP_HOST_POOL");
        return !(s && s[0] == '0') && host_threads() > 1;
    }();
    return on;
}

// The Schur pair lists of prepare() on host threads, identical to the serial build:
//   1. landmark chunk t (contiguous): its pairs counted per pose row ia;
//   2. the same chunk writes its pairs (ib, ea, eb) at its per-row cursors (rows in order, chunks
//      in order within a row: landmark order within a row);
//   3. rows in parallel: a stable counting sort by ib gives the row's blocks (j = i always, others
//      with pairs) and their pairs at the row's offset; then the blocks are listed row by row.
void schur_pairs_parallel(Prep& o, const int* eopt, int threads) {
    const int M = o.M, np = o.np;
    const int T = std::max(1, std::min(threads, M / 512 + 1));
    // scratch kept per calling thread across calls; the lambdas below run on the pool's threads, so
    // they must reach it through these references (a thread_local named inside them would be the
    // worker's own, empty instance)
    static thread_local std::vector<size_t> rc_s, roff_s;
    static thread_local std::vector<int> tj_s, tab_s;
    static thread_local std::vector<std::vector<int>> rb_s;
    std::vector<size_t>& rc = rc_s;
    std::vector<size_t>& roff = roff_s;
    std::vector<int>& tj = tj_s;
    std::vector<int>& tab = tab_s;
    std::vector<std::vector<int>>& rb = rb_s;
    std::vector<int> m0(T + 1);
    for (int t = 0; t <= T; t++) m0[t] = (int)((long long)M * t / T);
    rc.assign((size_t)T * np, 0);
    roff.assign(np + 1, 0);
    rb.resize(np);
    for (auto& v : rb) v.clear();
    HostPool& pool = HostPool::get(host_threads() - 1);
    pool.run(T, [&](int t) {
        size_t* c = rc.data() + (size_t)t * np;
        for (int m = m0[t]; m < m0[t + 1]; m++) {
            const int k0 = o.pt_ptr[m], k1 = o.pt_ptr[m + 1];
            for (int ka = k0; ka < k1; ka++) {
                const int ia = eopt[ka];
                if (ia < 0) continue;
                for (int kb = k0; kb < k1; kb++) c[ia] += eopt[kb] >= ia;
            }
        }
    });
    size_t total = 0;
    for (int i = 0; i < np; i++) {
        roff[i] = total;
        for (int t = 0; t < T; t++) {
            const size_t v = rc[(size_t)t * np + i];
            rc[(size_t)t * np + i] = total;
            total += v;
        }
    }
    roff[np] = total;
    tj.resize(total);
    tab.resize(2 * total);
    o.blk_pairs.resize(2 * total);
    pool.run(T, [&](int t) {
        size_t* c = rc.data() + (size_t)t * np;
        for (int m = m0[t]; m < m0[t + 1]; m++) {
            const int k0 = o.pt_ptr[m], k1 = o.pt_ptr[m + 1];
            for (int ka = k0; ka < k1; ka++) {
                const int ia = eopt[ka];
                if (ia < 0) continue;
                const int ea = o.pt_edges[ka];
                for (int kb = k0; kb < k1; kb++) {
                    const int ib = eopt[kb];
                    if (ib < ia) continue;
                    const size_t slot = c[ia]++;
                    tj[slot] = ib;
                    tab[2 * slot] = ea;
                    tab[2 * slot + 1] = o.pt_edges[kb];
                }
            }
        }
    });
    const int RB = 8;   // rows per task
    pool.run((np + RB - 1) / RB, [&](int task) {
        static thread_local std::vector<int> cj;
        cj.assign(np, 0);
        for (int i = task * RB; i < std::min(np, task * RB + RB); i++) {
            const size_t a = roff[i], b = roff[i + 1];
            for (size_t k = a; k < b; k++) cj[tj[k]]++;
            int s = 0;
            for (int j = i; j < np; j++) {
                const int cnt = cj[j];
                if (j == i || cnt > 0) { rb[i].push_back(j); rb[i].push_back(cnt); }
                cj[j] = s;   // from here on: the block's cursor within the row
                s += cnt;
            }
            for (size_t k = a; k < b; k++) {
                const size_t slot = a + (size_t)cj[tj[k]]++;
                o.blk_pairs[2 * slot] = tab[2 * k];
                o.blk_pairs[2 * slot + 1] = tab[2 * k + 1];
            }
            for (int j = i; j < np; j++) cj[j] = 0;
        }
    });
    o.blk_ptr.assign(1, 0);
    size_t s = 0;
    for (int i = 0; i < np; i++)
        for (size_t q = 0; q < rb[i].size(); q += 2) {
            o.blk_i.push_back(i);
            o.blk_j.push_back(rb[i][q]);
            s += (size_t)rb[i][q + 1];
            o.blk_ptr.push_back((int)s);
        }
}

// a Prep for the next call with its vectors' capacity kept (no allocation / first-touch page
// faults on the hot path: the C5 lists are a few MB)
void prep_reset(Prep& o) {
    o.rc = 0;
    o.P = o.M = o.E = o.np = o.n = o.nblk = 0;
    for (auto* v : {&o.opt, &o.pt_ptr, &o.pt_edges, &o.ps_ptr, &o.ps_edges, &o.blk_i, &o.blk_j, &o.blk_ptr,
                    &o.blk_pairs, &o.row_first, &o.cb_tiles, &o.cb_off, &o.items, &o.fin, &o.ifin})
        v->clear();
    o.own.clear();
    o.nslot = 0;
    o.use_dag = o.use_nd = o.use_nd_sh = false;
    o.dag = DagPlan{};
    o.nd = NdPlan{};
    o.dag_task_cap = 0;
    o.o_dag = o.o_dagi = o.o_red2 = 0;
    o.o_chi2 = o.o_state = o.o_obs = o.o_scr = o.o_lin = o.o_S = o.o_L = o.o_int = 0;
}

inline void se3_from_float(const float* q, const float* t, double* out) {
    double x = q[0], y = q[1], z = q[2], w = q[3];
    if (w < 0) { x = -x; y = -y; z = -z; w = -w; }
    const double nn = std::sqrt(x * x + y * y + z * z + w * w);
    out[0] = x / nn; out[1] = y / nn; out[2] = z / nn; out[3] = w / nn;
    out[4] = t[0]; out[5] = t[1]; out[6] = t[2]; out[7] = 0;
}

int prepare(const orbhip_ba_problem* pr, Prep& o, int chunk, int threads) {
    const int P = pr->n_poses, M = pr->n_points, E = pr->n_edges;
    if (P < 0 || M < 0 || E < 0 || (P && (!pr->pose_q || !pr->pose_t || !pr->pose_fixed)) || (M && !pr->points) ||
        (E && (!pr->edge_pose || !pr->edge_point || !pr->edge_uv || !pr->edge_octave || !pr->inv_sigma2)))
        return ORBHIP_ERR_ARG;
    for (int e = 0; e < E; e++)
        if (pr->edge_pose[e] < 0 || pr->edge_pose[e] >= P || pr->edge_point[e] < 0 || pr->edge_point[e] >= M ||
            pr->edge_octave[e] < 0 || pr->edge_octave[e] >= pr->n_octaves)
            return ORBHIP_ERR_ARG;
    static const bool pdbg = std::getenv("ORBHIP_PREP_DBG") != nullptr;
    auto tus = [] { return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count(); };
    double tp[8] = {tus()};
    o.P = P; o.M = M; o.E = E;
    o.opt.assign(P, -1);
    int np = 0;
    for (int i = 0; i < P; i++)
        if (!pr->pose_fixed[i]) o.opt[i] = np++;
    o.np = np;
    o.n = 6 * np;
    // n <= kCholSmallN: single-workgroup Cholesky (LDS-resident panel); larger: blocked solver
    if (o.n > kCbMaxN) return ORBHIP_ERR_UNSUPPORTED;
    const int* e_pose = pr->edge_pose;
    const int* e_pt = pr->edge_point;
    o.pt_ptr.assign(M + 1, 0);
    o.ps_ptr.assign(np + 1, 0);
    for (int e = 0; e < E; e++) {
        o.pt_ptr[e_pt[e] + 1]++;
        if (o.opt[e_pose[e]] >= 0) o.ps_ptr[o.opt[e_pose[e]] + 1]++;
    }
    for (int m = 0; m < M; m++) o.pt_ptr[m + 1] += o.pt_ptr[m];
    for (int i = 0; i < np; i++) o.ps_ptr[i + 1] += o.ps_ptr[i];
    o.pt_edges.resize(E);
    o.ps_edges.resize(o.ps_ptr[np]);
    // scratch kept per host thread across calls (no page faults on the hot path): eopt[k] = the opt
    // index of the pose of landmark-CSR slot k (one load per pair endpoint below), cnt = the dense
    // (i, j) pair counts, then the blocks' fill cursors
    static thread_local std::vector<int> eopt, cnt, fp, fq;   // (fp / fq: the fill cursors, no allocation per call)
    eopt.resize(E);
    {
        fp.assign(o.pt_ptr.begin(), o.pt_ptr.end() - 1);
        fq.assign(o.ps_ptr.begin(), o.ps_ptr.end() - 1);
        for (int e = 0; e < E; e++) {
            const int oi = o.opt[e_pose[e]];
            const int k = fp[e_pt[e]]++;
            o.pt_edges[k] = e;
            eopt[k] = oi;
            if (oi >= 0) o.ps_edges[fq[oi]++] = e;
        }
    }
    tp[1] = tus();
    // Schur pairs (a, b) of one landmark with opt(a) <= opt(b), grouped by block (i, j) (row-major
    // over i <= j, every diagonal block listed); within a block: landmark order (deterministic).
    // Large problems: schur_pairs_parallel (the same lists, built on host threads)
    if (threads > 1 && E >= kPrepParallelE) {
        schur_pairs_parallel(o, eopt.data(), threads);
    } else {
        // a counting sort on the dense block id i*np + j
        cnt.assign((size_t)np * np, 0);
        size_t npairs = 0;
        for (int m = 0; m < M; m++) {
            const int k0 = o.pt_ptr[m], k1 = o.pt_ptr[m + 1];
            for (int ka = k0; ka < k1; ka++) {
                const int ia = eopt[ka];
                if (ia < 0) continue;
                int* row = cnt.data() + (size_t)ia * np;
                for (int kb = k0; kb < k1; kb++) {
                    const int ib = eopt[kb];
                    if (ib < ia) continue;   // also drops the fixed poses (-1)
                    row[ib]++;
                    npairs++;
                }
            }
        }
        o.blk_ptr.assign(1, 0);
        {
            int s = 0;
            for (int i = 0; i < np; i++) {
                int* row = cnt.data() + (size_t)i * np;
                for (int j = i; j < np; j++) {
                    const int c = row[j];
                    if (i == j || c > 0) {
                        o.blk_i.push_back(i);
                        o.blk_j.push_back(j);
                        row[j] = s;   // from here on: the block's fill cursor
                        s += c;
                        o.blk_ptr.push_back(s);
                    }
                }
            }
        }
        o.blk_pairs.resize(2 * npairs);
        int* bp = o.blk_pairs.data();
        for (int m = 0; m < M; m++) {
            const int k0 = o.pt_ptr[m], k1 = o.pt_ptr[m + 1];
            for (int ka = k0; ka < k1; ka++) {
                const int ia = eopt[ka];
                if (ia < 0) continue;
                const int ea = o.pt_edges[ka];
                int* row = cnt.data() + (size_t)ia * np;
                for (int kb = k0; kb < k1; kb++) {
                    const int ib = eopt[kb];
                    if (ib < ia) continue;
                    const int slot = row[ib]++;
                    bp[2 * (size_t)slot] = ea;
                    bp[2 * (size_t)slot + 1] = o.pt_edges[kb];
                }
            }
        }
    }
    tp[2] = tus();
    o.nblk = (int)o.blk_i.size();
    {   // envelope of S: first pose column coupled to each pose row (blocks are stored i <= j)
        std::vector<int> fp(np);
        for (int i = 0; i < np; i++) fp[i] = i;
        for (int b = 0; b < o.nblk; b++) fp[o.blk_j[b]] = std::min(fp[o.blk_j[b]], o.blk_i[b]);
        const int nt = (o.n + 31) / 32;
        o.row_first.assign(nt, 0);
        for (int R = 0; R < nt; R++) {
            int f = R;
            for (int r = 32 * R; r < std::min(o.n, 32 * R + 32); r++) f = std::min(f, (6 * fp[r / 6]) / 32);
            o.row_first[R] = f;
        }
    }
    // Schur work items: chunks of at most `chunk` pairs; a block with one off-diagonal chunk is
    // written by its item, the others (and every diagonal block) are summed inside one work-group
    // of k_ba_schur_items (r06): at most kItemsWg chunks per block (a longer block takes longer
    // chunks), and a block that would straddle a work-group boundary starts the next work-group
    // (empty items, blk -1, pad the one before)
    // (two passes: the count, then direct stores into the sized arrays; per-item vector inserts
    // cost ~6 ns each, 0.3 ms at C5)
    size_t nit = 0, nfin = 0;
    for (int b = 0; b < o.nblk; b++) {
        const int k0 = o.blk_ptr[b], k1 = o.blk_ptr[b + 1];
        if (o.blk_i[b] != o.blk_j[b] && k1 - k0 <= chunk) { nit++; continue; }
        const int cb = std::max(chunk, (k1 - k0 + kItemsWg - 1) / kItemsWg);
        const int nch = std::max(1, (k1 - k0 + cb - 1) / cb);
        const int at = (int)(nit % kItemsWg);
        if (at + nch > kItemsWg) nit += kItemsWg - at;
        nit += nch;
        nfin++;
    }
    o.items.resize(4 * nit);
    o.ifin.resize(nit);
    o.fin.resize(3 * nfin);
    int* itp = o.items.data();
    int* ifp = o.ifin.data();
    int* fnp = o.fin.data();
    size_t it = 0;
    int f = 0;
    for (int b = 0; b < o.nblk; b++) {
        const int k0 = o.blk_ptr[b], k1 = o.blk_ptr[b + 1];
        const bool diag = o.blk_i[b] == o.blk_j[b];
        if (!diag && k1 - k0 <= chunk) {
            int* q = itp + 4 * it;
            q[0] = k0; q[1] = k1; q[2] = b; q[3] = -1;
            ifp[it++] = -1;
            continue;
        }
        const int cb = std::max(chunk, (k1 - k0 + kItemsWg - 1) / kItemsWg);
        const int nch = std::max(1, (k1 - k0 + cb - 1) / cb);
        const int at = (int)(it % kItemsWg);
        if (at + nch > kItemsWg)
            for (int q = at; q < kItemsWg; q++) {
                int* r = itp + 4 * it;
                r[0] = 0; r[1] = 0; r[2] = -1; r[3] = -1;
                ifp[it++] = -1;
            }
        fnp[3 * f] = b; fnp[3 * f + 1] = o.nslot; fnp[3 * f + 2] = nch;
        for (int c = 0; c < nch; c++) {
            int* r = itp + 4 * it;
            r[0] = k0 + c * cb; r[1] = std::min(k1, k0 + (c + 1) * cb); r[2] = b; r[3] = o.nslot + c;
            ifp[it++] = f;
        }
        o.nslot += nch;
        f++;
    }
    tp[3] = tus();
    if (pdbg) std::fprintf(stderr, "prepare E=%d: csr %.0f us, pairs %.0f us, envelope+items %.0f us\n", E, tp[1] - tp[0], tp[2] - tp[1], tp[3] - tp[2]);
    return ORBHIP_OK;
}

template <typename T>
struct DBuf {
    T* p = nullptr;
    size_t n = 0;
    ~DBuf() { if (p) (void)hipFree(p); }
    hipError_t ensure(size_t c) {
        if (p && c <= n) return hipSuccess;
        if (p) { (void)hipFree(p); p = nullptr; n = 0; }
        hipError_t e = hipMalloc((void**)&p, std::max<size_t>(c, 1) * sizeof(T));
        if (e == hipSuccess) n = c;
        return e;
    }
};

template <typename T>
struct HBuf {   // pinned host staging
    T* p = nullptr;
    size_t n = 0;
    ~HBuf() { if (p) (void)hipHostFree(p); }
    hipError_t ensure(size_t c) {
        if (p && c <= n) return hipSuccess;
        if (p) { (void)hipHostFree(p); p = nullptr; n = 0; }
        c = std::max<size_t>(c + c / 4, 64);   // grow geometrically: pinning is expensive
        hipError_t e = hipHostMalloc((void**)&p, c * sizeof(T), hipHostMallocDefault);
        if (e == hipSuccess) n = c;
        return e;
    }
};

}  // namespace

struct BaWorkspace {
    DBuf<double> dbl;      // all fp64 per-problem arrays, packed (segment map in ba_solve_batch)
    DBuf<int> act;         // active problem lists (several slots)
    DBuf<double> lam;      // per-problem lambda
    DBuf<double> gath;     // gathered red/flag of the active problems
    DBuf<LmCtl> ctl;       // device-driven rounds: per-problem LM state
    HBuf<LmCtl> hctl;      // its pinned staging (initial state up, final state down)
    HBuf<double> hdbl;     // staging: [e_chi2 | pose,pts | obs,info | the int arrays | BaArgs] of every problem
    double* h_gath = nullptr;  // pinned
    double* h_lam = nullptr;   // pinned
    double* h_red = nullptr;   // pinned: per problem red[4] + flag
    int* h_act = nullptr;      // pinned
    size_t h_cap = 0;
    // sharded solve over RCCL (orbhip_comm_init): landmarks partitioned, poses replicated
    ncclComm_t comm = nullptr;
    int nranks = 1, rank = 0;
    DBuf<int> dstop;           // stop-flag consensus (all-reduce max)
    DBuf<double> envbuf;       // S's union envelope, packed for the all-reduce (k_ba_env_pack)
    DBuf<long long> envoff;    // its per-32-row-tile offsets
    int* h_stop = nullptr;     // pinned
    int* h_done = nullptr;     // pinned, mapped: per problem, set by the device when its LM run ends
    int* d_done = nullptr;     // its device address
    DBuf<int*> d_donep;        // ... stored in device memory: what the kernels get
    size_t done_cap = 0;
    HBuf<int> hto;             // pinned: the persistent solver's hand-off timeout count per problem
    long long dag_timeouts = 0, dag_reruns = 0;
    std::vector<Prep> prep;    // the per-problem host preparations of the last call (capacity reused)
    NdWorkspace* nd = nullptr; // nested-dissection solves (created on first use)
    std::vector<NdWorkspace*> nds;   // sharded solves by segments: one per shard of this process
    DBuf<double*> ptab;        // in-process shards: the collectives' pointer tables
    DBuf<int> dint4;           // RCCL: small consensus all-reduces (plan, stop)
    DBuf<unsigned char> uadj;  // RCCL, replicated form: the union pose adjacency (all-reduce max)
    int* h_int4 = nullptr;     // pinned
};

BaWorkspace* ba_create() { return new BaWorkspace(); }

void ba_destroy(BaWorkspace* w) {
    if (!w) return;
    if (w->comm) (void)ncclCommDestroy(w->comm);
    if (w->nd) nd_destroy(w->nd);
    for (NdWorkspace* q : w->nds) nd_destroy(q);
    if (w->h_int4) (void)hipHostFree(w->h_int4);
    if (w->h_stop) (void)hipHostFree(w->h_stop);
    if (w->h_done) (void)hipHostFree(w->h_done);
    if (w->h_lam) (void)hipHostFree(w->h_lam);
    if (w->h_red) (void)hipHostFree(w->h_red);
    if (w->h_act) (void)hipHostFree(w->h_act);
    if (w->h_gath) (void)hipHostFree(w->h_gath);
    delete w;
}

struct LmState {
    double lambda = 0, ni = 2, currentChi = 0, rho = 0;
    int nBad = 0, it = 0, trials = 0, qmax = 0;
    bool done = false, errors_valid = true;
};

int ba_solve_batch(BaWorkspace* ws, const orbhip_ba_problem* const* probs, int B, orbhip_ba_result* const* res,
                   const volatile int* stop, hipStream_t st, int shard_mode, bool no_dag, bool no_nd) {
    if (B <= 0 || !probs || !res) return ORBHIP_ERR_ARG;
    // RCCL: this rank holds B consecutive shards (segments rank*B .. rank*B+B-1 of nranks*B), the
    // same B on every rank; the shards of one rank are summed on the device before the all-reduce
    if (shard_mode == kShardRccl && !ws->comm) return ORBHIP_ERR_ARG;
    for (int b = 0; b < B; b++)
        if (!probs[b] || !res[b]) return ORBHIP_ERR_ARG;
    static const bool timing = std::getenv("ORBHIP_BA_TIMING") != nullptr;
    // the state words (8 P + 3 M) up to which the trial's last work-group restores a rejected
    // trial itself ("small"); larger problems restore in k_ba_pop. ORBHIP_BA_SMALL_WORDS (read per
    // call) lowers it: the tests run the large-problem path on problems that reject trials
    const char* e_sw = std::getenv("ORBHIP_BA_SMALL_WORDS");
    const long small_words = e_sw ? std::atol(e_sw) : 32768;
    auto now = [] { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count(); };
    const double t_start = now();
    const int nth = host_threads();
    // the per-problem preparations, kept in the workspace across calls (their vectors' capacity:
    // no allocation on the hot path). A DAG-timeout re-run re-enters with the same workspace as a
    // tail call, after this frame's last use of them.
    if (ws->prep.size() < (size_t)B) ws->prep.resize(B);
    std::vector<Prep>& pp = ws->prep;
    for (int b = 0; b < B; b++) prep_reset(pp[b]);
    // Schur work-item size: a batch fills the chip with 16 pairs per lane; a few problems alone
    // would leave it mostly idle, so their items are cut to 4 pairs (4x the lanes), 3 for the
    // LBA sizes (r06, alternating runs, tools/r06/gpu_chunk.sh: C4 1.323 -> 1.309 ms with 3, 1.31-1.33 with 2, 1.34-1.35
    // with 1; the C5 GBA 5.18 -> 5.58 ms with 2)
    static const int chunk_env = std::getenv("ORBHIP_SCHUR_CHUNK") ? std::atoi(std::getenv("ORBHIP_SCHUR_CHUNK")) : 0;
    int maxE_in = 0;
    for (int b = 0; b < B; b++) maxE_in = std::max(maxE_in, probs[b]->n_edges);
    const int chunk = chunk_env > 0 ? chunk_env : (B >= 32 ? kSchurChunk : (maxE_in <= 32768 ? 3 : 4));
    // one problem: its Schur pair lists on the host threads; a batch: one problem per thread
    // (ORBHIP_PREP_THREADS=k: one large problem's pair lists on k host threads; off by default: on
    // the MI355X box's EPYC the C5 build went 0.62 -> 0.55 ms at 16 threads, 0.71 at 4 in r05, and
    // 0.63 -> 1.09-1.26 ms on the r06 tree (tools/r06/gpu_hostpool_ab.sh): its scattered fill does
    // not scale)
    static const int prep_par = std::getenv("ORBHIP_PREP_THREADS") ? std::atoi(std::getenv("ORBHIP_PREP_THREADS"))
                                                                   : 1;
    parallel_for(B, nth, [&](int b) { pp[b].rc = prepare(probs[b], pp[b], chunk, B == 1 ? prep_par : 1); });
    const double t_prepare = now();
    // RCCL shards: a rank whose shards are invalid must not return before the first collective
    // (the other ranks would wait in it forever); its verdict travels in that all-reduce and every
    // rank returns together
    int local_bad = 0;
    for (int b = 0; b < B && !local_bad; b++)
        if (pp[b].rc) {
            if (shard_mode != kShardRccl) return pp[b].rc;
            local_bad = pp[b].rc;
        }
    if (shard_mode != kShardNone && B > 1 && !local_bad) {
        for (int b = 1; b < B && !local_bad; b++)
            if (pp[b].P != pp[0].P || pp[b].np != pp[0].np) {
                if (shard_mode != kShardRccl) return ORBHIP_ERR_ARG;
                local_bad = ORBHIP_ERR_ARG;
            }
    }
    if (shard_mode != kShardNone && B > 1 && !local_bad) {
        // every shard factors the SUMMED S: the blocked Cholesky needs the union envelope
        for (int b = 1; b < B; b++)
            for (size_t R = 0; R < pp[0].row_first.size(); R++)
                pp[0].row_first[R] = std::min(pp[0].row_first[R], pp[b].row_first[R]);
        for (int b = 1; b < B; b++) pp[b].row_first = pp[0].row_first;
    }
    // Cholesky per problem: the persistent DAG solver for the GBA sizes and for a problem solved
    // alone (one LBA), the register / LDS single-workgroup solvers for batches of small problems;
    // ORBHIP_CHOL_BLOCKED=1 restores the one-launch-per-panel blocked solver for the large ones,
    // ORBHIP_CHOL_DAG_MIN sets the smallest n a lone problem takes the DAG solver at (default 128)
    static const bool force_blocked = std::getenv("ORBHIP_CHOL_BLOCKED") != nullptr;
    static const int dag_min = std::getenv("ORBHIP_CHOL_DAG_MIN") ? std::atoi(std::getenv("ORBHIP_CHOL_DAG_MIN")) : 128;
    const int dag_helpers = dag_max_helpers();
    for (int b = 0; b < B; b++)
        pp[b].use_dag = !no_dag && !force_blocked && pp[b].n > 0 && (pp[b].n > kCholSmallN || (B == 1 && pp[b].n >= dag_min));
    // a lone large problem whose S is a narrow (cyclic) block band (a GBA's keyframe loop): nested
    // dissection, when the plan's chain is shorter (ORBHIP_ND=0 disables it, ORBHIP_ND_K=k forces k
    // segments, ORBHIP_ND_MIN sets the smallest n considered)
    {
        const char* e_nd = std::getenv("ORBHIP_ND");
        const char* e_k = std::getenv("ORBHIP_ND_K");
        const char* e_min = std::getenv("ORBHIP_ND_MIN");
        const int nd_min = e_min ? std::atoi(e_min) : 960;
        if (shard_mode == kShardNone && B == 1 && !no_nd && pp[0].use_dag && pp[0].n >= nd_min &&
            !(e_nd && e_nd[0] == '0')) {
            Prep& p = pp[0];
            if (nd_plan(p.np, p.blk_i.data(), p.blk_j.data(), p.nblk, e_k ? std::atoi(e_k) : 0, p.nd)) {
                p.use_nd = true;
                p.use_dag = false;
            }
        }
    }
    // sharded solves by keyframe segments (the distributed form of the dissection):
    // shard r is segment r when every shard's landmarks lie inside its segment's matrix
    // (sharding.shard_problem_nd); then each shard eliminates its interior, the separator system is
    // summed over the shards, every shard solves it, and the shards' x are summed. Otherwise the
    // shards sum S itself and every shard solves it (replicated). The decision is agreed over the
    // ranks; ORBHIP_SHARD_ND=0 forces the replicated form.
    const int seg0 = shard_mode == kShardRccl ? ws->rank * B : 0;   // segment of problem 0
    NdPlan ndp;
    bool nd_sh = false;
    std::vector<int> ubi, ubj;   // the replicated form's union block structure (when dissected)
    if (shard_mode != kShardNone) {
        const char* e_snd = std::getenv("ORBHIP_SHARD_ND");
        const char* e_min = std::getenv("ORBHIP_ND_MIN");
        const int nd_min = e_min ? std::atoi(e_min) : 960;
        const int K = shard_mode == kShardLocal ? B : ws->nranks * B;
        int wl = 0, wc = 0;
        for (int b = 0; b < B && !local_bad; b++) {
            int l = 0, c = 0;
            nd_bandwidth(pp[b].np, pp[b].blk_i.data(), pp[b].blk_j.data(), pp[b].nblk, l, c);
            wl = std::max(wl, l);
            wc = std::max(wc, c);
        }
        const bool ok_base = !no_dag && !force_blocked && pp[0].n >= nd_min;
        int ok = (ok_base && !(e_snd && e_snd[0] == '0')) ? 1 : 0;
        if (shard_mode == kShardRccl) {   // the band over every rank's landmarks; the same B everywhere
            // words 3 / 4: the max of B and of -B agree only when every rank has the same B and
            // valid shards (an invalid rank sends INT_MAX)
            ws->h_int4[0] = wl; ws->h_int4[1] = wc; ws->h_int4[2] = -ok;
            ws->h_int4[3] = local_bad ? std::numeric_limits<int>::max() : B; ws->h_int4[4] = -B;
            if (hipMemcpyAsync(ws->dint4.p, ws->h_int4, 5 * sizeof(int), hipMemcpyHostToDevice, st) != hipSuccess ||
                ncclAllReduce(ws->dint4.p, ws->dint4.p, 5, ncclInt32, ncclMax, ws->comm, st) != ncclSuccess ||
                hipMemcpyAsync(ws->h_int4, ws->dint4.p, 5 * sizeof(int), hipMemcpyDeviceToHost, st) != hipSuccess ||
                hipStreamSynchronize(st) != hipSuccess)
                return ORBHIP_ERR_DEVICE;
            if (ws->h_int4[3] != B || -ws->h_int4[4] != B) return local_bad ? local_bad : ORBHIP_ERR_ARG;
            wl = ws->h_int4[0]; wc = ws->h_int4[1]; ok = -ws->h_int4[2];
        }
        ok = ok && nd_plan_band(pp[0].np, wl, wc, K, ndp);
        for (int b = 0; b < B && ok; b++)
            ok = nd_blocks_fit(ndp, seg0 + b, pp[b].blk_i.data(), pp[b].blk_j.data(), pp[b].nblk);
        if (shard_mode == kShardRccl) {   // every rank's landmarks fit its segment
            ws->h_int4[0] = ok ? 0 : 1;
            if (hipMemcpyAsync(ws->dint4.p, ws->h_int4, sizeof(int), hipMemcpyHostToDevice, st) != hipSuccess ||
                ncclAllReduce(ws->dint4.p, ws->dint4.p, 1, ncclInt32, ncclMax, ws->comm, st) != ncclSuccess ||
                hipMemcpyAsync(ws->h_int4, ws->dint4.p, sizeof(int), hipMemcpyDeviceToHost, st) != hipSuccess ||
                hipStreamSynchronize(st) != hipSuccess)
                return ORBHIP_ERR_DEVICE;
            ok = ws->h_int4[0] == 0;
        }
        nd_sh = ok != 0;
        if (nd_sh)
            for (int b = 0; b < B; b++) {
                Prep& p = pp[b];
                p.use_nd_sh = true;
                p.use_dag = false;
                const int r = seg0 + b;
                p.own.assign(p.np, 0);
                for (int q = ndp.seg[r]; q < ndp.seg[r + 1]; q++) p.own[q] = 1;   // interior + own separator
            }
        // r06: the replicated form (landmark shards, or segments whose landmarks cross) solves the
        // summed S by nested dissection too when that pays, planned on the union of the shards'
        // pose adjacencies (every rank derives the same plan from the same union); ORBHIP_ND=0
        // keeps the plain DAG solve on the union envelope
        const char* e_nd = std::getenv("ORBHIP_ND");
        if (!nd_sh && ok_base && !no_nd && !(e_nd && e_nd[0] == '0')) {
            const int np = pp[0].np;
            std::vector<unsigned char> adj((size_t)np * np, 0);   // [max(i, j)][min(i, j)]
            for (int b = 0; b < B; b++)
                for (int k = 0; k < pp[b].nblk; k++) {
                    const int i = pp[b].blk_i[k], j = pp[b].blk_j[k];
                    adj[(size_t)std::max(i, j) * np + std::min(i, j)] = 1;
                }
            if (shard_mode == kShardRccl) {
                BAOK(ws->uadj.ensure(adj.size()));
                if (hipMemcpyAsync(ws->uadj.p, adj.data(), adj.size(), hipMemcpyHostToDevice, st) != hipSuccess ||
                    ncclAllReduce(ws->uadj.p, ws->uadj.p, adj.size(), ncclUint8, ncclMax, ws->comm, st) != ncclSuccess ||
                    hipMemcpyAsync(adj.data(), ws->uadj.p, adj.size(), hipMemcpyDeviceToHost, st) != hipSuccess ||
                    hipStreamSynchronize(st) != hipSuccess)
                    return ORBHIP_ERR_DEVICE;
            }
            for (int i = 0; i < np; i++)
                for (int j = 0; j <= i; j++)
                    if (adj[(size_t)i * np + j]) { ubi.push_back(j); ubj.push_back(i); }
            NdPlan up;
            if (nd_plan(np, ubi.data(), ubj.data(), (int)ubi.size(), 0, up))
                for (int b = 0; b < B; b++) {
                    pp[b].nd = up;
                    pp[b].use_nd = true;
                    pp[b].use_dag = false;
                }
            else
                ubi.clear(), ubj.clear();
        }
    }
    const bool sharded = shard_mode != kShardNone;
    // the per-panel tile lists / the DAG plans (RCCL shards: the envelope is the union over the
    // ranks, known after a collective; their DAG plan is made then, into reserved space)
    parallel_for(B, nth, [&](int b) {
        Prep& p = pp[b];
        if (p.use_nd || p.use_nd_sh) {
            // planned above; its device data is set up with the problem's buffers (nd_setup)
        } else if (p.use_dag) {
            if (shard_mode == kShardRccl) {
                const size_t NT = (p.n + kDagTile - 1) / kDagTile;
                p.dag_task_cap = (size_t)dag_helpers + 1 + NT * (NT + 1) / 2 + 2 * NT;   // + the copy tasks, the column counts
            } else {
                dag_plan(p.row_first.data(), p.n, dag_helpers, p.dag);
                p.dag_task_cap = p.dag.toff.size() + p.dag.tasks.size();
            }
        } else if (p.n > kCholSmallN && shard_mode != kShardRccl) {
            cb_envelope_tiles(p.row_first.data(), p.n, p.cb_tiles, p.cb_off);
        }
    });
    const double t_prep = now();
    // ---- packed layout: fp64 segments, each contiguous over all problems ----
    //   C  e_chi2 (E)                 downloaded with A in one transfer
    //   A  pose (8P) + pts (3M)       uploaded, optimised in place, downloaded
    //   U  obs (2E) + info (E)        uploaded
    //   R  the rest (scratch), then the edge linearisations e_lin (32-byte aligned), S (n*n) and
    //      the panel inverses Lsave, 16-byte aligned
    size_t nC = 0, nA = 0, nU = 0, nR = 0, ni = 0;
    for (int b = 0; b < B; b++) {
        Prep& p = pp[b];
        const size_t P = p.P, M = p.M, E = p.E, np_ = p.np, n = p.n;
        p.o_chi2 = nC; nC += E;
        p.o_state = nA; nA += 8 * P + 3 * M;
        p.o_obs = nU; nU += 3 * E;
        p.o_scr = nR;
        nR += 8 * P + 3 * M                          // pose_bak, pts_bak
              + 2 * E + 3 * E                        // e_err, e_rho0, e_rho1 (+ pad)
              + 36 * np_ + 9 * np_ + 18 * M + 3 * M  // Hpp, R_lin, Hll, Dinv, db
              + (sharded ? 36 * np_ : 0)             // Hpp_g: Hpp summed over the shards
              + 2 * (n + 3 * M) + n + 4;             // b, x, bs, red
        nR = (nR + 3) & ~size_t(3);
        p.o_lin = nR; nR += 4 * E;
        p.o_S = nR; nR += n * n;
        nR = (nR + 1) & ~size_t(1);
        p.o_L = nR; nR += 1024 * ((n + 31) / 32);
        nR = (nR + 1) & ~size_t(1);
        p.o_red2 = nR;
        nR += std::max((E + 255) / 256 + (std::max(M, P) + kBsL - 1) / kBsL, (M + kLinL - 1) / kLinL + np_) + 2;
        if (p.use_dag) {   // 128-byte aligned
            nR = (nR + 15) & ~size_t(15);
            p.o_dag = nR; nR += dag_doubles(p.n);
        }
        p.o_int = ni;
        ni += (P + 4) + 2 * E + (M + 1) + E + (np_ + 1) + p.ps_edges.size() + 3 * p.nblk + 1 + p.blk_pairs.size() +
              p.row_first.size() + p.items.size() + p.fin.size() + p.ifin.size() + p.cb_tiles.size() + 8 +
              (p.use_dag ? dag_ints(p.n) + p.dag_task_cap + 4 : 0) + (p.own.size() + 3) / 4 + 1;
    }
    // r06: the int arrays and the BaArgs follow the uploaded doubles in the same device / pinned
    // buffers, so that ONE copy uploads all of it (three blit launches of ~4.4 us each before)
    const size_t sC = 0, sA = nC, sU = sA + nA;
    const size_t sI = (sU + nU + 1) & ~size_t(1);                            // 16-byte aligned
    const size_t sG = (sI + (ni * sizeof(int) + 7) / 8 + 1) & ~size_t(1);  // the BaArgs
    const size_t sR = (sG + (B * sizeof(BaArgs) + 7) / 8 + 15) & ~size_t(15);
    const size_t nd = sR + nR;
    BAOK(ws->dbl.ensure(nd));
    BAOK(ws->act.ensure(3 * (size_t)B));
    BAOK(ws->lam.ensure(B));
    BAOK(ws->gath.ensure(5 * (size_t)B));
    BAOK(ws->ctl.ensure(B));
    BAOK(ws->hctl.ensure(B));
    BAOK(ws->hdbl.ensure(sR));
    if (ws->h_cap < (size_t)B) {
        if (ws->h_lam) (void)hipHostFree(ws->h_lam);
        if (ws->h_red) (void)hipHostFree(ws->h_red);
        ws->h_red = nullptr;
        if (ws->h_act) (void)hipHostFree(ws->h_act);
        if (ws->h_gath) (void)hipHostFree(ws->h_gath);
        BAOK(hipHostMalloc((void**)&ws->h_gath, sizeof(double) * 5 * B, hipHostMallocDefault));
        BAOK(hipHostMalloc((void**)&ws->h_lam, sizeof(double) * B, hipHostMallocDefault));
        BAOK(hipHostMalloc((void**)&ws->h_red, sizeof(double) * 5 * B, hipHostMallocDefault));
        BAOK(hipHostMalloc((void**)&ws->h_act, sizeof(int) * 3 * B, hipHostMallocDefault));
        ws->h_cap = B;
    }
    double* D = ws->dbl.p;
    int* I = reinterpret_cast<int*>(D + sI);
    double* hd = ws->hdbl.p;
    int* hi = reinterpret_cast<int*>(hd + sI);
    BaArgs* ha = reinterpret_cast<BaArgs*>(hd + sG);
    BaArgs* const dArgs = reinterpret_cast<BaArgs*>(D + sG);
    std::vector<DagDev> dd(B, DagDev{nullptr, nullptr, nullptr, nullptr, 0, 0, 0});
    parallel_for(B, nth, [&](int b) {
        const Prep& p = pp[b];
        const orbhip_ba_problem* pr = probs[b];
        const size_t P = p.P, M = p.M, E = p.E;
        double* st_ = hd + sA + p.o_state;
        for (size_t i = 0; i < P; i++) se3_from_float(pr->pose_q + 4 * i, pr->pose_t + 3 * i, st_ + 8 * i);
        for (size_t k = 0; k < 3 * M; k++) st_[8 * P + k] = pr->points[k];
        double* ob = hd + sU + p.o_obs;
        // (on the host pool this loop measured slower: C5 pack + upload 0.11 -> 0.21 ms, r06 A/B)
        for (size_t e = 0; e < E; e++) {
            ob[2 * e] = pr->edge_uv[2 * e];
            ob[2 * e + 1] = pr->edge_uv[2 * e + 1];
            ob[2 * E + e] = (double)pr->inv_sigma2[pr->edge_octave[e]];
        }
        int* q = hi + p.o_int;
        auto put = [&](const int* src, size_t cnt) { int* at = q; std::memcpy(q, src, cnt * sizeof(int)); q += cnt; return at; };
        BaArgs& a = ha[b];
        int* d0 = I + p.o_int;
        auto dev = [&](const int* host_at) { return d0 + (host_at - (hi + p.o_int)); };
        a.opt = dev(put(p.opt.data(), P));
        a.flag = dev(q);   // [0] Cholesky ok, [1] blocked backward arrival counter (zero between uses)
        std::memset(q, 0, 4 * sizeof(int));
        q += 4;
        a.e_pose = dev(put(pr->edge_pose, E));
        a.e_pt = dev(put(pr->edge_point, E));
        a.pt_ptr = dev(put(p.pt_ptr.data(), M + 1));
        a.pt_edges = dev(put(p.pt_edges.data(), E));
        a.ps_ptr = dev(put(p.ps_ptr.data(), p.np + 1));
        a.ps_edges = dev(put(p.ps_edges.data(), p.ps_edges.size()));
        a.blk_i = dev(put(p.blk_i.data(), p.nblk));
        a.blk_j = dev(put(p.blk_j.data(), p.nblk));
        a.blk_ptr = dev(put(p.blk_ptr.data(), p.nblk + 1));
        if ((q - hi) & 1) q++;   // int2 alignment of the pair list
        a.blk_pairs = dev(put(p.blk_pairs.data(), p.blk_pairs.size()));
        while ((q - hi) & 3) q++;   // int4 alignment of the items
        a.items = dev(put(p.items.data(), p.items.size()));
        a.nitems = (int)(p.items.size() / 4);
        a.fin = dev(put(p.fin.data(), p.fin.size()));
        a.nfin = (int)(p.fin.size() / 3);
        a.ifin = dev(put(p.ifin.data(), p.ifin.size()));
        a.row_first = dev(put(p.row_first.data(), p.row_first.size()));
        a.cb_tiles = p.cb_tiles.empty() ? nullptr : dev(put(p.cb_tiles.data(), p.cb_tiles.size()));
        a.own = nullptr;
        if (!p.own.empty()) {   // bytes, in the int staging
            std::memcpy(q, p.own.data(), p.own.size());
            a.own = reinterpret_cast<const unsigned char*>(dev(q));
            q += (p.own.size() + 3) / 4;
        }
        if (p.use_dag) {   // flags + control words (zero), then the plan (or the space reserved for it)
            while ((q - hi) & 3) q++;
            dd[b].ints = dev(q);
            std::memset(q, 0, dag_ints(p.n) * sizeof(int));
            q += dag_ints(p.n);
            dd[b].toff = dev(q);
            if (!p.dag.toff.empty()) {
                put(p.dag.toff.data(), p.dag.toff.size());
                dd[b].tasks = dev(q);
                put(p.dag.tasks.data(), p.dag.tasks.size());
            } else {
                dd[b].tasks = dev(q + kDagMaxHelpers + 1);   // RCCL: planned after the union envelope
                q += p.dag_task_cap;
            }
            dd[b].G = p.dag.G;
            dd[b].pb = p.dag.pb;
            dd[b].need_off = p.dag.toff.empty() ? 0 : p.dag.toff[p.dag.G];
        }
        a.nblk = p.nblk;
        a.P = p.P; a.M = p.M; a.E = p.E; a.np = p.np; a.n = p.n;
        a.fx = pr->fx; a.fy = pr->fy; a.cx = pr->cx; a.cy = pr->cy; a.delta = pr->huber_delta;
        a.e_chi2 = D + sC + p.o_chi2;
        a.pose = D + sA + p.o_state; a.pts = a.pose + 8 * P;
        a.e_obs = D + sU + p.o_obs; a.e_info = a.e_obs + 2 * E;
        a.e_lin = D + sR + p.o_lin;
        double* r = D + sR + p.o_scr;
        a.pose_bak = r; r += 8 * P;
        a.pts_bak = r; r += 3 * M;
        a.e_err = r; r += 2 * E;
        a.e_rho0 = r; r += E;
        a.e_rho1 = r; r += 2 * E;
        a.Hpp = r; r += 36 * (size_t)p.np;
        a.R_lin = r; r += 9 * (size_t)p.np;
        a.Hll = r; r += 9 * M;
        a.Dinv = r; r += 9 * M;
        a.db = r; r += 3 * M;
        a.Hpp_g = a.Hpp;
        if (sharded) { a.Hpp_g = r; r += 36 * (size_t)p.np; }
        a.sync = sharded ? 1 : 0;
        a.small = (!sharded && 8 * P + 3 * M <= (size_t)small_words && E <= 65536) ? 1 : 0;
        a.fused = 0;   // set below once the batch's launch width is known
        a.b = r; r += p.n + 3 * M;
        a.x = r; r += p.n + 3 * M;
        a.bs = r; r += p.n;
        a.red = r;
        a.S = D + sR + p.o_S;
        a.Lsave = D + sR + p.o_L;
        a.part = D + sR + p.o_red2;
        a.npart_e = (int)((E + 255) / 256);
        a.npart_m = (int)((std::max(M, (size_t)P) + kBsL - 1) / kBsL);   // k_ba_backsub_errs' workgroups
        if (p.use_dag) dd[b].buf = D + sR + p.o_dag;
        a.lambda = ws->lam.p + b;
        a.lead = shard_mode == kShardLocal ? (b == 0) : (shard_mode == kShardRccl ? (ws->rank == 0 && b == 0) : 1);
        a.ctl = ws->ctl.p + b;
    });
    BAOK(hipMemcpyAsync(D + sA, hd + sA, sizeof(double) * (sR - sA), hipMemcpyHostToDevice, st));
    // RCCL shards solved by the blocked Cholesky (which reads only the lower triangle inside the
    // envelope; the one-workgroup solvers also read the mirrored upper triangle) all-reduce S
    // over its union envelope only: ~5 MB instead of n^2 doubles (46 MB) at C5
    size_t env_total = 0;
    if (shard_mode == kShardRccl && !nd_sh && !pp[0].row_first.empty()) {   // union envelope over the ranks
        int* rf = const_cast<int*>(ha[0].row_first);
        if (ncclAllReduce(rf, rf, pp[0].row_first.size(), ncclInt32, ncclMin, ws->comm, st) != ncclSuccess)
            return ORBHIP_ERR_DEVICE;
        const int nt = (int)pp[0].row_first.size(), n = pp[0].n;
        std::vector<int> urf(nt);
        if (n > kCholSmallN || pp[0].use_dag) {
            BAOK(hipMemcpyAsync(urf.data(), rf, nt * sizeof(int), hipMemcpyDeviceToHost, st));
            BAOK(hipStreamSynchronize(st));
        }
        for (int b = 1; b < B; b++)   // this rank's other shards: the same envelope
            BAOK(hipMemcpyAsync(const_cast<int*>(ha[b].row_first), rf, nt * sizeof(int), hipMemcpyDeviceToDevice, st));
        if (pp[0].use_dag) {   // the DAG plan of the union envelope, into the reserved space
            DagPlan& dp = pp[0].dag;
            dag_plan(urf.data(), n, dag_helpers, dp);
            for (int b = 0; b < B; b++) {
                if (dp.toff.size() + dp.tasks.size() > pp[b].dag_task_cap) return ORBHIP_ERR_DEVICE;
                BAOK(hipMemcpy(const_cast<int*>(dd[b].toff), dp.toff.data(), dp.toff.size() * sizeof(int),
                               hipMemcpyHostToDevice));
                dd[b].tasks = dd[b].toff + dp.toff.size();
                if (!dp.tasks.empty())
                    BAOK(hipMemcpy(const_cast<int*>(dd[b].tasks), dp.tasks.data(), dp.tasks.size() * sizeof(int),
                                   hipMemcpyHostToDevice));
                dd[b].G = dp.G;
                dd[b].pb = dp.pb;
                dd[b].need_off = dp.toff[dp.G];
            }
        }
        // one shard per rank: S all-reduced over its union envelope, packed; several: the full S
        // (summed on the device first, then the all-reduce, then copied to the other shards)
        if (B == 1 && n > kCholSmallN && !std::getenv("ORBHIP_SHARD_FULL_S")) {
        std::vector<long long> off(nt + 1, 0);
        for (int R = 0; R < nt; R++)
            off[R + 1] = off[R] + (long long)std::min(32, n - 32 * R) * (std::min(32 * R + 32, n) - 32 * urf[R]);
        env_total = (size_t)off[nt];
        BAOK(ws->envbuf.ensure(env_total));
        BAOK(ws->envoff.ensure(nt + 1));
        BAOK(hipMemcpyAsync(ws->envoff.p, off.data(), (nt + 1) * sizeof(long long), hipMemcpyHostToDevice, st));
        }
    }
    const double t_pack = now();
    static LdsAttrOnce chol_attr;   // per device, thread-safe (dev_attr.h)
    BAOK(chol_attr.ensure((const void*)k_ba_cholesky, 160 * 1024));
    int maxM = 0, maxE = 0, maxP = 0, maxNp = 0, maxBlk = 0, maxN = 0, maxItems = 0;
    bool s_written = false;
    // "large": solved on its own (DAG or blocked); the rest share one single-workgroup launch
    auto large = [&](int b) { return pp[b].use_nd || pp[b].use_nd_sh || pp[b].use_dag || pp[b].n > kCholSmallN; };
    for (int b = 0; b < B; b++) {
        const Prep& p = pp[b];
        maxM = std::max(maxM, p.M); maxE = std::max(maxE, p.E); maxP = std::max(maxP, p.P);
        maxNp = std::max(maxNp, p.np); maxBlk = std::max(maxBlk, p.nblk);
        maxItems = std::max(maxItems, (int)(p.items.size() / 4));
        if (!large(b)) maxN = std::max(maxN, p.n);
        if (!p.use_dag && !p.use_nd && !p.use_nd_sh && p.n > kCholRegMaxN) s_written = true;   // the LDS and blocked solvers factor S in place
    }
    const size_t chol_lds = sizeof(double) * chol_lds_doubles(maxN);
    // every problem on a solver that reads S and never writes it (register / DAG / dissection) and no
    // sum of S over the shards (the replicated form all-reduces S in place): S is zeroed once, the
    // Schur finisher overwrites its blocks every trial (r05: segment shards too, which saved a
    // 46 MB memset per shard and trial at C5)
    const bool s_readonly = !s_written && (shard_mode == kShardNone || nd_sh);
    auto large_solve = [&](int b, const int* gate) -> int {
        if (pp[b].use_nd) {
            (void)gate;   // set at nd_setup
            BAOK(nd_solve(B == 1 ? ws->nd : ws->nds[b], st));
        } else if (pp[b].use_dag) {
            BAOK(chol_dag_solve(ha[b].S, pp[b].n, ha[b].row_first, ha[b].bs, ha[b].x, ha[b].flag, dd[b], st, gate));
        } else {
            chol_blocked_solve(ha[b].S, pp[b].n, ha[b].Lsave, ha[b].bs, ha[b].x, ha[b].flag, ha[b].row_first, st, gate,
                               ha[b].cb_tiles, pp[b].cb_off.empty() ? nullptr : pp[b].cb_off.data());
        }
        return ORBHIP_OK;
    };
    auto gx = [](int n_, int b_) { return (unsigned)std::max(1, (n_ + b_ - 1) / b_); };
    (void)hipGetLastError();
    int* d_act = ws->act.p;
    int* h_act = ws->h_act;
    auto upload_act = [&](const std::vector<int>& v) -> int {
        for (size_t i = 0; i < v.size(); i++) h_act[i] = v[i];
        BAOK(hipMemcpyAsync(d_act, h_act, v.size() * sizeof(int), hipMemcpyHostToDevice, st));
        return ORBHIP_OK;
    };
    const BaArgs* dA = dArgs;
    // stop flag: one consistent decision across ranks (all-reduce max) per batch of slots
    auto stop_now = [&]() -> bool {
        const bool local = stop && *stop;
        if (shard_mode != kShardRccl) return local;
        *ws->h_stop = local ? 1 : 0;
        if (hipMemcpyAsync(ws->dstop.p, ws->h_stop, sizeof(int), hipMemcpyHostToDevice, st) != hipSuccess) return true;
        if (ncclAllReduce(ws->dstop.p, ws->dstop.p, 1, ncclInt32, ncclMax, ws->comm, st) != ncclSuccess) return true;
        if (hipMemcpyAsync(ws->h_stop, ws->dstop.p, sizeof(int), hipMemcpyDeviceToHost, st) != hipSuccess) return true;
        if (hipStreamSynchronize(st) != hipSuccess) return true;
        return *ws->h_stop != 0;
    };
    // ---- hand-off timeouts of the persistent solver: a timed-out solve fails its trial (flag 0),
    // which must never pass for a g2o rejection. Counted per problem (control word 3), read with
    // the outputs (no extra synchronisation), agreed over the ranks of a sharded solve. ----
    std::vector<const int*> tw;   // the timeout words of every persistent solve of this call
    int ndag = 0;
    // the outputs: the timeout words, e_chi2 of every problem + optimised poses/points (one
    // transfer); r06: enqueued behind the slots that may be the last ones, so a solve that ended
    // there needs no further host round trip (a wasted copy of ~115 KB at C4 otherwise)
    auto out_copies = [&]() -> int {
        for (int i = 0; i < ndag; i++) BAOK(hipMemcpyAsync(ws->hto.p + i, tw[i], sizeof(int), hipMemcpyDeviceToHost, st));
        BAOK(hipMemcpyAsync(hd, D, sizeof(double) * (nC + nA), hipMemcpyDeviceToHost, st));
        return ORBHIP_OK;
    };
    bool outputs_in = false;
    std::vector<LmState> L(B);
    bool ctl_with_outputs = false;   // the final LM state is read back with the outputs
    std::vector<int> all(B);
    for (int b = 0; b < B; b++) all[b] = b;
    if (upload_act(all)) return ORBHIP_ERR_DEVICE;
    {
        // ---- device-driven rounds: each slot advances every problem by one LM trial (with the
        // iteration's linearisation in front when it starts one); the k_ba_ctl_* kernels apply
        // the g2o rules per problem, so the host only enqueues slots and reads the state back once
        // per batch of slots. Sharded solves run the same slots with their collectives on the
        // stream between the kernels (RCCL across ranks, k_ba_multi_reduce across the shards of
        // this process) and the controller's reductions split from its decisions (BaArgs::sync):
        // every shard sees the same sums, so every shard takes the same decisions, and the host
        // decides nothing per trial. ----
        LmCtl* dctl = ws->ctl.p;
        for (int b = 0; b < B; b++) {
            LmCtl& c = ws->hctl.p[b];
            c = LmCtl{};
            c.ni = 2;
            c.phase = probs[b]->iterations > 0 ? kPhBuild : kPhDone;   // optimize(0): nothing to run
            c.errors_valid = 1;
            c.iterations = probs[b]->iterations;
            c.early_stop = probs[b]->early_stop;
        }
        BAOK(hipMemcpyAsync(dctl, ws->hctl.p, B * sizeof(LmCtl), hipMemcpyHostToDevice, st));
        if (B > 1)   // shards of the replicated form: each solves the summed S in its own workspace
            while (ws->nds.size() < (size_t)B) ws->nds.push_back(nd_create());
        for (int b = 0; b < B; b++)
            if (pp[b].use_nd) {
                if (!ws->nd) ws->nd = nd_create();
                const bool uni = !ubi.empty();
                const int rc = nd_setup(B == 1 ? ws->nd : ws->nds[b], pp[b].nd, uni ? ubi.data() : pp[b].blk_i.data(),
                                        uni ? ubj.data() : pp[b].blk_j.data(), uni ? (int)ubi.size() : pp[b].nblk,
                                        ha[b].S, ha[b].bs, ha[b].x, ha[b].flag, &dctl[b].phase, st);
                // a plan the device setup refuses (a segment beyond the back-substitution's LDS, a
                // separator system beyond the DAG solver; the planner rejects both, so this is a
                // guard): the same problem again on the plain DAG solve, nothing was run yet
                if (rc == -5) {
                    if (hipStreamSynchronize(st) != hipSuccess) return ORBHIP_ERR_DEVICE;
                    return ba_solve_batch(ws, probs, B, res, stop, st, shard_mode, no_dag, true);
                }
                if (rc != 0) return ORBHIP_ERR_DEVICE;
            }
        if (nd_sh) {   // one segment per shard
            while (ws->nds.size() < (size_t)B) ws->nds.push_back(nd_create());
            for (int b = 0; b < B; b++)
                if (nd_setup(ws->nds[b], ndp, pp[b].blk_i.data(), pp[b].blk_j.data(), pp[b].nblk, ha[b].S, ha[b].bs,
                             ha[b].x, ha[b].flag, &dctl[b].phase, st, seg0 + b) != 0)
                    return ORBHIP_ERR_DEVICE;
        }
        for (int b = 0; b < B; b++) {
            if (pp[b].use_dag) tw.push_back(dd[b].ints + 3);
            if (pp[b].use_nd) nd_timeout_words(B == 1 ? ws->nd : ws->nds[b], tw);
            if (pp[b].use_nd_sh) nd_timeout_words(ws->nds[b], tw);
        }
        ndag = (int)tw.size();
        if (ndag) BAOK(ws->hto.ensure(ndag));
        // ---- the collectives of a sharded slot: site s sums (or maxes) src[b] into dst[b] over the
        // shards; RCCL: one all-reduce of this rank's buffers ----
        enum { kHpp, kRed0, kRed2, kRed01, kRepS, kRepBs, kNdPack, kNdBz, kNdX, kSites };
        struct Site { std::vector<double*> src, dst; size_t count = 0; int op = 0; size_t tab = 0; };
        std::vector<Site> sites(sharded ? kSites : 0);
        if (sharded) {
            auto site = [&](int id, size_t count, int op, auto src, auto dst) {
                Site& t = sites[id];
                t.count = count; t.op = op;
                for (int b = 0; b < B; b++) { t.src.push_back(src(b)); t.dst.push_back(dst(b)); }
            };
            site(kHpp, 36 * (size_t)maxNp, 0, [&](int b) { return ha[b].Hpp; }, [&](int b) { return const_cast<double*>(ha[b].Hpp_g); });
            site(kRed0, 1, 0, [&](int b) { return ha[b].red; }, [&](int b) { return ha[b].red; });
            site(kRed2, 1, 1, [&](int b) { return ha[b].red + 2; }, [&](int b) { return ha[b].red + 2; });
            site(kRed01, 2, 0, [&](int b) { return ha[b].red; }, [&](int b) { return ha[b].red; });
            if (!nd_sh) {
                site(kRepS, (size_t)pp[0].n * pp[0].n, 0, [&](int b) { return ha[b].S; }, [&](int b) { return ha[b].S; });
                site(kRepBs, (size_t)pp[0].n, 0, [&](int b) { return ha[b].bs; }, [&](int b) { return ha[b].bs; });
            } else {
                const NdSepBufs q0 = nd_sep_bufs(ws->nds[0]);
                site(kNdPack, q0.pack_n, 0, [&](int b) { return nd_sep_bufs(ws->nds[b]).pack; },
                     [&](int b) { return nd_sep_bufs(ws->nds[b]).pack; });
                site(kNdBz, (size_t)q0.nZ, 0, [&](int b) { return nd_sep_bufs(ws->nds[b]).bZ; },
                     [&](int b) { return nd_sep_bufs(ws->nds[b]).bZ; });
                site(kNdX, (size_t)q0.n + 1, 0, [&](int b) { return nd_sep_bufs(ws->nds[b]).x_loc; },
                     [&](int b) { return nd_sep_bufs(ws->nds[b]).xg; });
            }
            if (shard_mode == kShardLocal || B > 1) {   // the pointer tables of the in-process sums, on the device once
                std::vector<double*> tab;
                for (Site& t : sites) {
                    t.tab = tab.size();
                    tab.insert(tab.end(), t.src.begin(), t.src.end());
                    tab.insert(tab.end(), t.dst.begin(), t.dst.end());
                }
                BAOK(ws->ptab.ensure(tab.size()));
                BAOK(hipMemcpy(ws->ptab.p, tab.data(), tab.size() * sizeof(double*), hipMemcpyHostToDevice));
            }
        }
        auto coll = [&](int id) -> int {
            const Site& t = sites[id];
            if (t.count == 0) return ORBHIP_OK;
            const dim3 gr((unsigned)std::min<size_t>(1024, (t.count + 255) / 256));
            double* const* tab = (shard_mode == kShardLocal || B > 1) ? ws->ptab.p + t.tab : nullptr;   // [src | dst]
            if (shard_mode == kShardLocal) {
                hipLaunchKernelGGL(k_ba_multi_reduce, gr, dim3(256), 0, st, (const double* const*)tab, B, tab + B, B,
                                   t.count, t.op);
                return ORBHIP_OK;
            }
            if (B > 1) {   // RCCL with several shards per rank: this rank's sum into dst[0] first
                hipLaunchKernelGGL(k_ba_multi_reduce, gr, dim3(256), 0, st, (const double* const*)tab, B, tab + B, 1,
                                   t.count, t.op);
                if (ncclAllReduce(t.dst[0], t.dst[0], t.count, ncclDouble, t.op ? ncclMax : ncclSum, ws->comm, st) !=
                    ncclSuccess)
                    return ORBHIP_ERR_DEVICE;
                hipLaunchKernelGGL(k_ba_multi_reduce, gr, dim3(256), 0, st, (const double* const*)(tab + B), 1,
                                   tab + B + 1, B - 1, t.count, t.op);
                return ORBHIP_OK;
            }
            if (id == kRepS && env_total) {   // RCCL, replicated: S over its union envelope, packed
                const BaArgs& a0 = ha[0];
                const dim3 g(8, (unsigned)pp[0].row_first.size());
                hipLaunchKernelGGL(k_ba_env_pack, g, dim3(256), 0, st, a0.S, a0.n, a0.row_first, ws->envoff.p,
                                   ws->envbuf.p, 0);
                if (ncclAllReduce(ws->envbuf.p, ws->envbuf.p, env_total, ncclDouble, ncclSum, ws->comm, st) != ncclSuccess)
                    return ORBHIP_ERR_DEVICE;
                hipLaunchKernelGGL(k_ba_env_pack, g, dim3(256), 0, st, a0.S, a0.n, a0.row_first, ws->envoff.p,
                                   ws->envbuf.p, 1);
                return ORBHIP_OK;
            }
            if (ncclAllReduce(t.src[0], t.dst[0], t.count, ncclDouble, t.op ? ncclMax : ncclSum, ws->comm, st) != ncclSuccess)
                return ORBHIP_ERR_DEVICE;
            return ORBHIP_OK;
        };
        int ns = 0;   // problems on the single-workgroup solvers (act slot 3)
        for (int b = 0; b < B; b++)
            if (!large(b)) h_act[2 * B + ns++] = b;
        if (ns) BAOK(hipMemcpyAsync(d_act + 2 * B, h_act + 2 * B, ns * sizeof(int), hipMemcpyHostToDevice, st));
        if (s_readonly) hipLaunchKernelGGL(k_ba_zero_s, dim3(64, B), dim3(256), 0, st, dA, d_act, 1);
        hipLaunchKernelGGL(k_ba_errors, dim3(gx(maxE, 256), B), dim3(256), 0, st, dA, d_act, 0, nullptr);
        if (!sharded) {
            hipLaunchKernelGGL(k_ba_ctl_init, dim3(B), dim3(1024), 0, st, dA, d_act);
        } else {   // the initial chi2 over every shard's edges
            hipLaunchKernelGGL(k_ba_reduce, dim3(B), dim3(1024), 0, st, dA, d_act, 1);
            if (coll(kRed0)) return ORBHIP_ERR_DEVICE;
            hipLaunchKernelGGL(k_ba_sh_init, dim3(B), dim3(64), 0, st, dA, d_act);
        }
        const dim3 gB((unsigned)((B + 255) / 256)), b256(256);
        bool all_small = true;   // every problem restores / refreshes in its trial's last workgroup
        for (int b = 0; b < B; b++) all_small = all_small && ha[b].small;
        // ... and takes its errors inside the back-substitution when its partial slots hold the
        // fused kernel's workgroups (ORBHIP_BA_FUSED=0 keeps the separate k_ba_errors(2))
        const unsigned gbs = gx(std::max(maxM, maxP), kBsL);
        // k_ba_lin's pose work-groups: one pose per work-group (its four waves on its edges) for a
        // lone problem, four (a wave each) for batches; ORBHIP_LIN_PPW=1/4 forces one
        const char* e_ppw = std::getenv("ORBHIP_LIN_PPW");
        const int lin_ppw = e_ppw ? (std::atoi(e_ppw) == 1 ? 1 : 4) : (B == 1 ? 1 : 4);
        const char* fz = std::getenv("ORBHIP_BA_FUSED");   // per call: the tests compare both forms
        const bool fuse_env = !(fz && fz[0] == '0');
        // (r06: every unsharded problem, small or not; a sharded trial ends in the split controller)
        bool fused = !sharded && fuse_env;
        for (int b = 0; b < B && fused; b++) fused = (int)gbs <= ha[b].npart_e && pp[b].P <= kFusedMaxP;
        if (fused) {
            for (int b = 0; b < B; b++) ha[b].fused = 1;
            BAOK(hipMemcpyAsync(dArgs, ha, B * sizeof(BaArgs), hipMemcpyHostToDevice, st));
        }
        // the host-mapped words (post_done): B done flags, then the relayed stop flag. The kernels
        // get them through a device-resident pointer pair: {done, stop} for a solve of its own,
        // {done, null} for a sharded one (its shards agree on the stop between batches)
        if (ws->done_cap < (size_t)B) {
            if (ws->h_done) (void)hipHostFree(ws->h_done);
            ws->h_done = nullptr; ws->d_done = nullptr; ws->done_cap = 0;
            BAOK(hipHostMalloc((void**)&ws->h_done, sizeof(int) * (B + 1), hipHostMallocMapped | hipHostMallocCoherent));
            BAOK(hipHostGetDevicePointer((void**)&ws->d_done, ws->h_done, 0));
            int* const ptrs[4] = {ws->d_done, ws->d_done + B, ws->d_done, nullptr};
            BAOK(ws->d_donep.ensure(4));
            BAOK(hipMemcpy(ws->d_donep.p, ptrs, sizeof(ptrs), hipMemcpyHostToDevice));
            ws->done_cap = B;
        }
        const bool relay = !sharded && stop;   // a caller's stop flag to relay mid-solve
        int* const* const donep = ws->d_donep.p + (relay ? 0 : 2);
        int* const h_stopw = relay ? ws->h_done + ws->done_cap : nullptr;
        for (int b = 0; b < B; b++) __atomic_store_n(ws->h_done + b, probs[b]->iterations > 0 ? 0 : 1, __ATOMIC_RELAXED);
        __atomic_store_n(ws->h_done + ws->done_cap, 0, __ATOMIC_RELAXED);
        auto slot = [&]() -> int {
            // the sharded slots' error refresh and budget check; an unsharded problem's iteration
            // ends in its controller (ctl_end_decide) and its stale errors are refreshed by k_ba_lin
            if (!all_small && sharded)
                hipLaunchKernelGGL(k_ba_errors, dim3(gx(maxE, 256), B), b256, 0, st, dA, d_act, 1, donep);
            hipLaunchKernelGGL(k_ba_lin, dim3(gx(maxM, kLinL) + gx(maxNp, lin_ppw), B), b256, 0, st, dA, d_act,
                               (int)gx(maxM, kLinL), lin_ppw, donep);
            if (sharded) {   // the trial start on the shards' sums: Hpp, then the largest diagonal
                if (coll(kHpp)) return ORBHIP_ERR_DEVICE;
                hipLaunchKernelGGL(k_ba_sh_maxdiag, dim3(B), b256, 0, st, dA, d_act);
                if (coll(kRed2)) return ORBHIP_ERR_DEVICE;
                hipLaunchKernelGGL(k_ba_sh_begin, dim3(B), dim3(64), 0, st, dA, d_act);
            }
            if (!s_readonly) hipLaunchKernelGGL(k_ba_zero_s, dim3(64, B), b256, 0, st, dA, d_act, 0);
            if (!fused) hipLaunchKernelGGL(k_ba_schur_points, dim3(gx(maxM, 256), B), b256, 0, st, dA, d_act);
            hipLaunchKernelGGL(k_ba_schur_items, dim3(gx(2 * maxItems, 256) + gx(maxNp, 4) + 1, B), b256, 0, st, dA,
                               d_act, (int)gx(2 * maxItems, 256), donep);
            if (nd_sh) {   // each shard its segment; the separator system and x summed over the shards
                for (int b = 0; b < B; b++) BAOK(nd_factor_assemble(ws->nds[b], st));
                for (int b = 0; b < B; b++) BAOK(nd_sep_pack(ws->nds[b], 0, st));
                if (coll(kNdPack) || coll(kNdBz)) return ORBHIP_ERR_DEVICE;
                for (int b = 0; b < B; b++) BAOK(nd_sep_pack(ws->nds[b], 1, st));
                for (int b = 0; b < B; b++) BAOK(nd_separator_backsolve(ws->nds[b], st));
                if (coll(kNdX)) return ORBHIP_ERR_DEVICE;
                for (int b = 0; b < B; b++) BAOK(nd_finish(ws->nds[b], st));
            } else {
                if (sharded && (coll(kRepS) || coll(kRepBs))) return ORBHIP_ERR_DEVICE;   // replicated solves
                if (ns) {
                    if (maxN <= kCholRegMaxN) BAOK(chol_reg_launch(maxN, ns, dA, d_act + 2 * B, st));
                    else hipLaunchKernelGGL(k_ba_cholesky, dim3(ns), dim3(512), chol_lds, st, dA, d_act + 2 * B);
                }
                for (int b = 0; b < B; b++)
                    if (large(b) && large_solve(b, &dctl[b].phase)) return ORBHIP_ERR_DEVICE;
            }
            if (fused) {
                hipLaunchKernelGGL(k_ba_backsub_errs, dim3(gbs, B), b256, 0, st, dA, d_act, donep);
            } else {
                hipLaunchKernelGGL(k_ba_backsub, dim3(gx(std::max(maxM, maxP), 256), B), b256, 0, st, dA, d_act);
                hipLaunchKernelGGL(k_ba_errors, dim3(gx(maxE, 256), B), b256, 0, st, dA, d_act, 2, donep);
            }
            if (sharded) {   // the trial's end on the shards' sums of chi2 and the scale
                hipLaunchKernelGGL(k_ba_sh_sums, dim3(B), dim3(1024), 0, st, dA, d_act);
                if (coll(kRed01)) return ORBHIP_ERR_DEVICE;
                hipLaunchKernelGGL(k_ba_sh_end, dim3(B), dim3(64), 0, st, dA, d_act, donep);
            }
            int maxPM = 0;
            for (int b = 0; b < B; b++) maxPM = std::max(maxPM, std::max(8 * pp[b].P, 3 * pp[b].M));
            if (!all_small) hipLaunchKernelGGL(k_ba_pop, dim3(gx(maxPM, 256), B), b256, 0, st, dA, d_act);
            BAOK(hipGetLastError());
            return ORBHIP_OK;
        };
        // Slots go out in chunks of kChunk behind one event each (at most two chunks in flight):
        // the host checks the done flags once per chunk, and while it waits it relays the caller's
        // stop flag into the mapped word that every trial's Schur launch copies into the controller
        // (relay_host_stop; checked at the trial's end and the next iteration's start: g2o's
        // force-stop checks), so a stop takes effect within a trial or two however many slots are
        // queued. r04: an event or a store to host memory between every two slots put a
        // ~5 us bubble in front of every trial (the queue drains for the marker; the kernel that
        // wrote host memory ends with a system-scope release).
        constexpr int kChunk = 8;
        int rc = ORBHIP_OK;
        bool stop_sent = false;
        hipEvent_t ev[2];
        const unsigned evf = hipEventDisableTiming | hipEventDisableSystemFence;
        BAOK(hipEventCreateWithFlags(&ev[0], evf));
        if (hipEventCreateWithFlags(&ev[1], evf) != hipSuccess) { (void)hipEventDestroy(ev[0]); return ORBHIP_ERR_DEVICE; }
        auto all_done = [&] {
            for (int b = 0; b < B; b++)
                if (!__atomic_load_n(ws->h_done + b, __ATOMIC_RELAXED)) return false;
            return true;
        };
        auto relay_stop = [&] {
            if (h_stopw && stop && *stop) __atomic_store_n(h_stopw, 1, __ATOMIC_RELAXED);
        };
        // with a stop flag to relay: polls, yielding the core between polls (the caller's Tracking
        // thread may need it); without one: blocks in the runtime
        auto wait_ev = [&](hipEvent_t e) -> int {
            if (!h_stopw) return hipEventSynchronize(e) == hipSuccess ? ORBHIP_OK : ORBHIP_ERR_DEVICE;
            for (;;) {
                std::this_thread::yield();
                const hipError_t q = hipEventQuery(e);
                if (q == hipSuccess) return ORBHIP_OK;
                if (q != hipErrorNotReady) return ORBHIP_ERR_DEVICE;
                relay_stop();
            }
        };
        int remaining = 0;   // slots every unfinished problem still needs at least
        for (int b = 0; b < B; b++) remaining = std::max(remaining, probs[b]->iterations);
        int nchunk = 0;
        // ranks of an RCCL solve must enqueue the same slots (their collectives pair up): they look
        // at the stop flag only between batches, agreed by an all-reduce, and never end a batch on
        // the asynchronous done flags; the batch length comes from the LM state read back, which
        // every rank holds identically
        const bool rccl = shard_mode == kShardRccl;
        bool last_ev_spec = false;   // the last event recorded follows the speculative copies
        while (remaining > 0 && rc == ORBHIP_OK) {
            if (rccl && !stop_sent && stop_now()) {
                hipLaunchKernelGGL(k_ba_ctl_stop, gB, b256, 0, st, dctl, B, donep);
                stop_sent = true;
            }
            // RCCL: at most kChunk slots per batch, so the agreed stop is looked at every few trials
            const int batch = rccl ? std::min(remaining, kChunk) : remaining;
            for (int k = 0; k < batch && rc == ORBHIP_OK;) {
                if (!rccl && !stop_sent && stop && *stop) {
                    hipLaunchKernelGGL(k_ba_ctl_stop, gB, b256, 0, st, dctl, B, donep);
                    stop_sent = true;
                }
                const int n = std::min(kChunk, batch - k);
                for (int j = 0; j < n && rc == ORBHIP_OK; j++) rc = slot();
                k += n;
                bool spec = false;   // this batch's last slots: the LM state and outputs behind them
                if (rc == ORBHIP_OK && !rccl && k == batch) {
                    spec = true;
                    if (hipMemcpyAsync(ws->hctl.p, dctl, B * sizeof(LmCtl), hipMemcpyDeviceToHost, st) != hipSuccess ||
                        out_copies() != ORBHIP_OK)
                        rc = ORBHIP_ERR_DEVICE;
                }
                if (rc == ORBHIP_OK && hipEventRecord(ev[nchunk & 1], st) != hipSuccess) rc = ORBHIP_ERR_DEVICE;
                if (rc != ORBHIP_OK) break;
                last_ev_spec = spec;
                if (nchunk++ >= 1) rc = wait_ev(ev[nchunk & 1]);   // the chunk before this one
                if (rc == ORBHIP_OK && !rccl && all_done()) break;
            }
            if (rc == ORBHIP_OK) rc = wait_ev(ev[(nchunk - 1) & 1]);
            if (rc != ORBHIP_OK) break;
            if (!rccl && all_done()) {   // every problem ended: its LM state comes with the outputs
                // (already in when the last event followed the speculative copies)
                outputs_in = !rccl && last_ev_spec;
                ctl_with_outputs = !outputs_in;
                break;
            }
            if (hipMemcpyAsync(ws->hctl.p, dctl, B * sizeof(LmCtl), hipMemcpyDeviceToHost, st) != hipSuccess ||
                hipStreamSynchronize(st) != hipSuccess) {
                rc = ORBHIP_ERR_DEVICE;
                break;
            }
            remaining = 0;
            for (int b = 0; b < B; b++) {
                const LmCtl& c = ws->hctl.p[b];
                if (c.phase == kPhDone) continue;
                remaining = std::max(remaining, stop_sent ? 1 : std::max(1, c.iterations - c.it));
            }
        }
        (void)hipEventDestroy(ev[0]);
        (void)hipEventDestroy(ev[1]);
        if (rc != ORBHIP_OK) return rc;
        // the LM state read back with the outputs below (one synchronisation for all of it: each
        // read-back + synchronisation of its own cost ~20-30 us of host round trip at C4)
        if (ctl_with_outputs) BAOK(hipMemcpyAsync(ws->hctl.p, dctl, B * sizeof(LmCtl), hipMemcpyDeviceToHost, st));
    }
    const double t_solve = now();
    if (!outputs_in) {   // (else the speculative copies below the last slots brought them)
        if (out_copies() != ORBHIP_OK) return ORBHIP_ERR_DEVICE;
        BAOK(hipStreamSynchronize(st));
    }
    {   // the LM state of every problem (read back in the loop, or just now with the outputs)
        for (int b = 0; b < B; b++) {
            const LmCtl& c = ws->hctl.p[b];
            L[b].currentChi = c.currentChi;
            L[b].it = c.it;
            L[b].trials = c.trials;
            res[b]->initial_chi2 = c.initChi;
        }
    }
    {
        int timeouts = 0;
        for (int i = 0; i < ndag; i++) timeouts += ws->hto.p[i];
        if (shard_mode == kShardRccl) {   // one decision for every rank
            *ws->h_stop = timeouts;
            if (hipMemcpyAsync(ws->dstop.p, ws->h_stop, sizeof(int), hipMemcpyHostToDevice, st) != hipSuccess ||
                ncclAllReduce(ws->dstop.p, ws->dstop.p, 1, ncclInt32, ncclMax, ws->comm, st) != ncclSuccess ||
                hipMemcpyAsync(ws->h_stop, ws->dstop.p, sizeof(int), hipMemcpyDeviceToHost, st) != hipSuccess ||
                hipStreamSynchronize(st) != hipSuccess)
                return ORBHIP_ERR_DEVICE;
            timeouts = *ws->h_stop;
        }
        if (timeouts > 0) {
            ws->dag_timeouts += timeouts;
            // default: solve again on the non-persistent solvers (blocked / single-workgroup), which
            // reproduce the schedule g2o would have run; ORBHIP_DAG_RERUN=0 reports the timeout
            const char* e = std::getenv("ORBHIP_DAG_RERUN");
            if (no_dag || (e && e[0] == '0')) return ORBHIP_ERR_TIMEOUT;
            ws->dag_reruns++;
            return ba_solve_batch(ws, probs, B, res, stop, st, shard_mode, true, no_nd);
        }
    }
    // the outputs of problem b, edges [e0, e1) (the poses, points and LM words with the first range)
    auto outputs = [&](int b, int e0, int e1) {
        const Prep& p = pp[b];
        const orbhip_ba_problem* pr = probs[b];
        orbhip_ba_result* r = res[b];
        const double* pose_o = hd + sA + p.o_state;
        const double* pts_o = pose_o + 8 * (size_t)p.P;
        const double* chi2_o = hd + sC + p.o_chi2;
        if (e0 == 0) {
            r->final_chi2 = L[b].currentChi;
            r->iterations_done = L[b].it;
            r->lm_trials = L[b].trials;
            for (int i = 0; i < p.P; i++) {
                if (r->pose_q) for (int k = 0; k < 4; k++) r->pose_q[4 * i + k] = (float)pose_o[8 * i + k];
                if (r->pose_t) for (int k = 0; k < 3; k++) r->pose_t[3 * i + k] = (float)pose_o[8 * i + 4 + k];
            }
            if (r->points) for (int k = 0; k < 3 * p.M; k++) r->points[k] = (float)pts_o[k];
        }
        for (int e = e0; e < e1; e++) {
            if (r->edge_chi2) r->edge_chi2[e] = (float)chi2_o[e];
            if (r->edge_depth_ok) {   // isDepthPositive: (T.map(X)).z > 0
                const double* T = &pose_o[8 * pr->edge_pose[e]];
                const double* X = &pts_o[3 * pr->edge_point[e]];
                double ux = T[1] * X[2] - T[2] * X[1], uy = T[2] * X[0] - T[0] * X[2];
                ux += ux; uy += uy;
                const double uz2 = 2 * (T[0] * X[1] - T[1] * X[0]);
                const double cz = T[0] * uy - T[1] * ux;
                const double z = X[2] + T[3] * uz2 + cz + T[6];
                r->edge_depth_ok[e] = z > 0.0 ? 1 : 0;
            }
        }
    };
    if (B == 1 && pp[0].E >= kPrepParallelE && host_pool_on()) {
        // one large problem (a GBA): its edges in chunks on the host pool (r06, late: the C5 loop's
        // 80k depth tests and conversions took ~0.2 ms on one core)
        const int E = pp[0].E, T = std::min(host_threads(), E / 4096 + 1);
        HostPool::get(host_threads() - 1).run(T, [&](int t) { outputs(0, (int)((long long)E * t / T), (int)((long long)E * (t + 1) / T)); });
    } else {
        parallel_for(B, nth, [&](int b) { outputs(b, 0, pp[b].E); });
    }
    if (timing)
        std::fprintf(stderr,
                     "orbhip ba timing B=%d: prep %.3f ms (problem structure %.3f), pack+upload %.3f ms, solve %.3f ms, "
                     "outputs %.3f ms\n",
                     B, t_prep - t_start, t_prepare - t_start, t_pack - t_prep, t_solve - t_pack, now() - t_solve);
    return ORBHIP_OK;
}

int ba_solve(BaWorkspace* ws, const orbhip_ba_problem* prob, orbhip_ba_result* res, const volatile int* stop,
             hipStream_t st) {
    const orbhip_ba_problem* pp[1] = {prob};
    orbhip_ba_result* rr[1] = {res};
    return ba_solve_batch(ws, pp, 1, rr, stop, st, kShardNone);
}

int ba_test_prepare(const orbhip_ba_problem* pr, int threads, double* out4) {
    Prep a, b;
    int rc = prepare(pr, a, kSchurChunk, 1);
    if (rc) return rc;
    auto ms_since = [](std::chrono::steady_clock::time_point t) {
        return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
    };
    // out4[3]: the threaded build (threads > 1) or the serial build into a reused Prep (threads = 1)
    if (threads == 1) {
        prep_reset(a);
        const auto t1 = std::chrono::steady_clock::now();
        rc = prepare(pr, a, kSchurChunk, 1);
        const double ms1 = ms_since(t1);
        if (rc) return rc;
        if (out4) out4[3] = ms1;
    }
    const auto t0 = std::chrono::steady_clock::now();
    rc = prepare(pr, b, kSchurChunk, threads);
    const double ms = ms_since(t0);
    if (rc) return rc;
    if (threads == 1) {
        if (out4) { out4[0] = b.nblk; out4[1] = (double)(b.blk_pairs.size() / 2); out4[2] = ms; }
        return a.blk_pairs == b.blk_pairs ? ORBHIP_OK : -1;
    }
    const bool same = a.opt == b.opt && a.pt_ptr == b.pt_ptr && a.pt_edges == b.pt_edges && a.ps_ptr == b.ps_ptr &&
                      a.ps_edges == b.ps_edges && a.blk_i == b.blk_i && a.blk_j == b.blk_j && a.blk_ptr == b.blk_ptr &&
                      a.blk_pairs == b.blk_pairs && a.row_first == b.row_first && a.items == b.items && a.fin == b.fin &&
                      a.nslot == b.nslot && a.nblk == b.nblk;
    if (out4) {
        out4[0] = b.nblk;
        out4[1] = (double)(b.blk_pairs.size() / 2);
        out4[2] = (double)(b.items.size() / 4);
        out4[3] = ms;
    }
    return same ? ORBHIP_OK : -1;
}

void ba_stats(BaWorkspace* ws, long long* timeouts, long long* reruns) {
    *timeouts = ws ? ws->dag_timeouts : 0;
    *reruns = ws ? ws->dag_reruns : 0;
}

int ba_comm_init(BaWorkspace* ws, int nranks, int rank, const void* id) {
    if (nranks < 1 || rank < 0 || rank >= nranks || !id) return ORBHIP_ERR_ARG;
    if (ws->comm) { (void)ncclCommDestroy(ws->comm); ws->comm = nullptr; }
    ncclUniqueId uid;
    std::memcpy(&uid, id, sizeof(uid));
    if (ncclCommInitRank(&ws->comm, nranks, uid, rank) != ncclSuccess) { ws->comm = nullptr; return ORBHIP_ERR_DEVICE; }
    ws->nranks = nranks;
    ws->rank = rank;
    BAOK(ws->dstop.ensure(1));
    BAOK(ws->dint4.ensure(8));
    if (!ws->h_int4) BAOK(hipHostMalloc((void**)&ws->h_int4, 8 * sizeof(int), hipHostMallocDefault));
    if (!ws->h_stop) BAOK(hipHostMalloc((void**)&ws->h_stop, sizeof(int), hipHostMallocDefault));
    return ORBHIP_OK;
}

int ba_comm_unique_id(void* id) {
    ncclUniqueId uid;
    if (ncclGetUniqueId(&uid) != ncclSuccess) return ORBHIP_ERR_DEVICE;
    std::memcpy(id, &uid, sizeof(uid));
    return ORBHIP_OK;
}

// Diagnostic: factor+solve one SPD system with per-phase cycle stamps (test hook).
// Diagnostic: the register-resident solver on one SPD system (test hook); reps launches timed.
int ba_test_cholesky_reg(const double* A, const double* b, double* x, int n, int reps, float* ms,
                         unsigned long long* phases5) {
    if (n <= 0 || n > kCholRegMaxN || reps < 1) return ORBHIP_ERR_ARG;
    double *dS = nullptr, *db_ = nullptr, *dx = nullptr;
    int *df = nullptr, *dact = nullptr;
    BaArgs* dargs = nullptr;
    BAOK(hipMalloc((void**)&dS, sizeof(double) * n * n));
    BAOK(hipMalloc((void**)&db_, sizeof(double) * n));
    BAOK(hipMalloc((void**)&dx, sizeof(double) * n));
    BAOK(hipMalloc((void**)&df, sizeof(int)));
    BAOK(hipMalloc((void**)&dact, sizeof(int)));
    BAOK(hipMalloc((void**)&dargs, sizeof(BaArgs)));
    BAOK(hipMemcpy(dS, A, sizeof(double) * n * n, hipMemcpyHostToDevice));
    BAOK(hipMemcpy(db_, b, sizeof(double) * n, hipMemcpyHostToDevice));
    BaArgs h{};
    h.n = n; h.S = dS; h.bs = db_; h.x = dx; h.flag = df;
    const int zero = 0;
    BAOK(hipMemcpy(dargs, &h, sizeof(BaArgs), hipMemcpyHostToDevice));
    BAOK(hipMemcpy(dact, &zero, sizeof(int), hipMemcpyHostToDevice));
    BAOK(chol_reg_launch(n, 1, dargs, dact, nullptr));   // warm-up (S is read-only)
    hipEvent_t e0, e1;
    BAOK(hipEventCreate(&e0)); BAOK(hipEventCreate(&e1));
    BAOK(hipEventRecord(e0, nullptr));
    for (int r = 0; r < reps; r++) BAOK(chol_reg_launch(n, 1, dargs, dact, nullptr));
    BAOK(hipEventRecord(e1, nullptr));
    BAOK(hipDeviceSynchronize());
    BAOK(hipEventElapsedTime(ms, e0, e1));
    *ms /= reps;
    if (phases5) {
        unsigned long long* dd = nullptr;
        BAOK(hipMalloc((void**)&dd, sizeof(unsigned long long) * 48));
        BAOK(hipMemset(dd, 0, 48 * 8));
        BAOK(chol_reg_probe(n, dargs, dd, nullptr));
        BAOK(hipMemcpy(phases5, dd, sizeof(unsigned long long) * 48, hipMemcpyDeviceToHost));
        (void)hipFree(dd);
    }
    int fl = 0;
    BAOK(hipMemcpy(&fl, df, sizeof(int), hipMemcpyDeviceToHost));
    BAOK(hipMemcpy(x, dx, sizeof(double) * n, hipMemcpyDeviceToHost));
    (void)hipFree(dS); (void)hipFree(db_); (void)hipFree(dx); (void)hipFree(df); (void)hipFree(dact);
    (void)hipFree(dargs);
    (void)hipEventDestroy(e0); (void)hipEventDestroy(e1);
    return fl ? ORBHIP_OK : ORBHIP_ERR_NOT_PD;
}

int ba_test_cholesky(const double* A, const double* b, double* x, int n, unsigned long long* phases5, float* ms) {
    double *dS = nullptr, *db_ = nullptr, *dx = nullptr;
    int* df = nullptr;
    unsigned long long* dd = nullptr;
    BAOK(hipMalloc((void**)&dS, sizeof(double) * n * n));
    BAOK(hipMalloc((void**)&db_, sizeof(double) * n));
    BAOK(hipMalloc((void**)&dx, sizeof(double) * n));
    BAOK(hipMalloc((void**)&df, sizeof(int)));
    BAOK(hipMalloc((void**)&dd, sizeof(unsigned long long) * 8));
    BAOK(hipMemcpy(dS, A, sizeof(double) * n * n, hipMemcpyHostToDevice));
    BAOK(hipMemcpy(db_, b, sizeof(double) * n, hipMemcpyHostToDevice));
    BAOK(hipMemset(dd, 0, 64));
    BAOK(hipFuncSetAttribute((const void*)k_chol_test, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    const size_t lds = sizeof(double) * chol_lds_doubles(n);
    double* dL = nullptr;
    BAOK(hipMalloc((void**)&dL, sizeof(double) * 1024 * ((n + 31) / 32)));
    hipEvent_t e0, e1;
    BAOK(hipEventCreate(&e0)); BAOK(hipEventCreate(&e1));
    BAOK(hipEventRecord(e0, nullptr));
    hipLaunchKernelGGL(k_chol_test, dim3(1), dim3(512), lds, nullptr, dS, db_, dx, n, df, dL, dd);
    BAOK(hipEventRecord(e1, nullptr));
    BAOK(hipDeviceSynchronize());
    BAOK(hipEventElapsedTime(ms, e0, e1));
    BAOK(hipMemcpy(x, dx, sizeof(double) * n, hipMemcpyDeviceToHost));
    BAOK(hipMemcpy(phases5, dd, sizeof(unsigned long long) * 5, hipMemcpyDeviceToHost));
    (void)hipFree(dS); (void)hipFree(db_); (void)hipFree(dx); (void)hipFree(df); (void)hipFree(dd);
    (void)hipFree(dL);
    (void)hipEventDestroy(e0); (void)hipEventDestroy(e1);
    return ORBHIP_OK;
}

}  // namespace orbhip
