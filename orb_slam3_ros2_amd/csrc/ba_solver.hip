// gfx950 bundle adjustment: the g2o problem of Optimizer::LocalBundleAdjustment /
// BundleAdjustment (U:src/Optimizer.cc) solved with the Levenberg-Marquardt schedule of
// OptimizationAlgorithmLevenberg and the Schur complement of BlockSolver<6,3>.
//
// The host drives the exact g2o control flow (iterations, trials, lambda schedule, push/pop,
// termination) with ONE device->host read per trial (chi2, scale, solve flag). All
// arithmetic is fp64 on the device:
//   k_ba_errors        EdgeSE3ProjectXYZ::computeError + RobustKernelHuber::robustify
//   k_ba_lin_points    linearizeOplus + constructQuadraticForm, landmark side (Hll, b_l,
//                      per-edge Hpl blocks)
//   k_ba_lin_poses     the pose side (Hpp, b_p), one wave per pose, deterministic tree
//   k_ba_schur_points  setLambda on Hll, Dinv (Eigen 3x3 cofactor inverse), db, W = Hpl Dinv
//   k_ba_schur_blocks  S_ij = [i==j](Hpp_i + lambda I) - sum W_a Hpl_b^T over shared
//                      landmarks (precomputed pair lists: deterministic gather, no atomics)
//   k_ba_schur_b       b_schur = b_p - sum Hpl db
//   k_ba_cholesky      dense LL^T of S + two triangular solves, one workgroup; the trailing
//                      update is v_mfma_f64_16x16x4f64 on 16x16 tiles
//   k_ba_backsub       xl = Dinv (b_l - Hpl^T xp), X += xl (push: old X saved)
//   k_ba_update_poses  T <- exp(xp) * T (SE3Quat::exp, operator*)   (push: old T saved)
//   k_ba_reduce        activeRobustChi2 and computeScale, fixed-order reductions
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <limits>
#include <map>
#include <vector>

#include "orbhip_ba.h"

namespace orbhip {

typedef double double4_t __attribute__((ext_vector_type(4)));

struct BaArgs {
    int P, M, E, np, n;
    double fx, fy, cx, cy, delta;
    double* pose;      // P*8: qx qy qz qw tx ty tz pad
    double* pose_bak;
    double* pts;       // M*3
    double* pts_bak;
    const int* opt;    // P
    const int* e_pose;
    const int* e_pt;
    const double* e_obs;   // E*2
    const double* e_info;  // E
    double* e_err;     // E*2
    double* e_chi2;    // E
    double* e_rho0;    // E
    double* e_rho1;    // E
    double* Hpp;       // np*36
    double* Hll;       // M*9
    double* Hpl;       // E*18 (zero for edges of fixed poses)
    double* b;         // n + 3M
    double* Dinv;      // M*9
    double* db;        // M*3
    double* W;         // E*18
    double* S;         // n*n
    double* bs;        // n
    double* x;         // n + 3M
    const int* pt_ptr; const int* pt_edges;     // CSR point -> edges (all edges)
    const int* ps_ptr; const int* ps_edges;     // CSR optimised pose -> edges
    const int* blk_i; const int* blk_j; const int* blk_ptr; const int* blk_pairs;  // Schur pair lists
    int nblk;
    double* red;       // [0] chi2, [1] scale, [2] maxdiag
    int* flag;         // [0] cholesky ok
};

// ---------------------------------------------------------------------------
// SE3Quat helpers (Eigen formulas)
// ---------------------------------------------------------------------------
struct DQ { double x, y, z, w; };

__device__ __forceinline__ void qrot(const DQ& q, double vx, double vy, double vz, double& ox, double& oy, double& oz) {
    double ux = q.y * vz - q.z * vy, uy = q.z * vx - q.x * vz, uz = q.x * vy - q.y * vx;
    ux += ux; uy += uy; uz += uz;
    const double cx = q.y * uz - q.z * uy, cy = q.z * ux - q.x * uz, cz = q.x * uy - q.y * ux;
    ox = vx + q.w * ux + cx;
    oy = vy + q.w * uy + cy;
    oz = vz + q.w * uz + cz;
}

__device__ __forceinline__ void qtomat(const DQ& q, double R[9]) {
    const double tx = 2 * q.x, ty = 2 * q.y, tz = 2 * q.z;
    const double twx = tx * q.w, twy = ty * q.w, twz = tz * q.w;
    const double txx = tx * q.x, txy = ty * q.x, txz = tz * q.x;
    const double tyy = ty * q.y, tyz = tz * q.y, tzz = tz * q.z;
    R[0] = 1 - (tyy + tzz); R[1] = txy - twz;       R[2] = txz + twy;
    R[3] = txy + twz;       R[4] = 1 - (txx + tzz); R[5] = tyz - twx;
    R[6] = txz - twy;       R[7] = tyz + twx;       R[8] = 1 - (txx + tyy);
}

__device__ __forceinline__ DQ mattoq(const double m[9]) {
    DQ q;
    double t = m[0] + m[4] + m[8];
    if (t > 0) {
        t = sqrt(t + 1.0);
        q.w = 0.5 * t;
        t = 0.5 / t;
        q.x = (m[7] - m[5]) * t;
        q.y = (m[2] - m[6]) * t;
        q.z = (m[3] - m[1]) * t;
    } else {
        int i = 0;
        if (m[4] > m[0]) i = 1;
        if (m[8] > m[3 * i + i]) i = 2;
        const int j = (i + 1) % 3, k = (j + 1) % 3;
        t = sqrt(m[3 * i + i] - m[3 * j + j] - m[3 * k + k] + 1.0);
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

__device__ __forceinline__ void qnormalize(DQ& q) {
    if (q.w < 0) { q.x = -q.x; q.y = -q.y; q.z = -q.z; q.w = -q.w; }
    const double n = sqrt(q.x * q.x + q.y * q.y + q.z * q.z + q.w * q.w);
    q.x /= n; q.y /= n; q.z /= n; q.w /= n;
}

__device__ __forceinline__ DQ load_q(const double* p) { return DQ{p[0], p[1], p[2], p[3]}; }

// ---------------------------------------------------------------------------
// errors
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_ba_errors(BaArgs a) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= a.E) return;
    const double* T = a.pose + 8 * a.e_pose[e];
    const double* X = a.pts + 3 * a.e_pt[e];
    double cx, cy, cz;
    qrot(load_q(T), X[0], X[1], X[2], cx, cy, cz);
    cx += T[4]; cy += T[5]; cz += T[6];
    const double u = a.fx * cx / cz + a.cx, v = a.fy * cy / cz + a.cy;
    const double e0 = a.e_obs[2 * e] - u, e1 = a.e_obs[2 * e + 1] - v;
    const double chi2 = a.e_info[e] * (e0 * e0 + e1 * e1);
    double r0 = chi2, r1 = 1.0;
    if (a.delta > 0) {
        const double dsqr = a.delta * a.delta;
        if (chi2 > dsqr) {
            const double sq = sqrt(chi2);
            r0 = 2 * sq * a.delta - dsqr;
            r1 = a.delta / sq;
        }
    }
    a.e_err[2 * e] = e0;
    a.e_err[2 * e + 1] = e1;
    a.e_chi2[e] = chi2;
    a.e_rho0[e] = r0;
    a.e_rho1[e] = r1;
}

// Jacobians of the error for edge e: A (2x3, point), B (2x6, pose [omega, upsilon])
__device__ __forceinline__ void edge_jac(const BaArgs& a, int e, double A[6], double B[12]) {
    const double* T = a.pose + 8 * a.e_pose[e];
    const double* X = a.pts + 3 * a.e_pt[e];
    const DQ q = load_q(T);
    double x, y, z;
    qrot(q, X[0], X[1], X[2], x, y, z);
    x += T[4]; y += T[5]; z += T[6];
    double J[6];
    J[0] = -(a.fx / z); J[1] = -0.0; J[2] = -(-a.fx * x / (z * z));
    J[3] = -0.0; J[4] = -(a.fy / z); J[5] = -(-a.fy * y / (z * z));
    double R[9];
    qtomat(q, R);
#pragma unroll
    for (int r = 0; r < 2; r++)
#pragma unroll
        for (int c = 0; c < 3; c++)
            A[3 * r + c] = J[3 * r] * R[c] + J[3 * r + 1] * R[3 + c] + J[3 * r + 2] * R[6 + c];
    const double D[18] = {0, z, -y, 1, 0, 0, -z, 0, x, 0, 1, 0, y, -x, 0, 0, 0, 1};
#pragma unroll
    for (int r = 0; r < 2; r++)
#pragma unroll
        for (int c = 0; c < 6; c++)
            B[6 * r + c] = J[3 * r] * D[c] + J[3 * r + 1] * D[6 + c] + J[3 * r + 2] * D[12 + c];
}

// ---------------------------------------------------------------------------
// buildSystem
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_ba_lin_points(BaArgs a) {
    const int m = blockIdx.x * blockDim.x + threadIdx.x;
    if (m >= a.M) return;
    double H[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0}, bl[3] = {0, 0, 0};
    for (int k = a.pt_ptr[m]; k < a.pt_ptr[m + 1]; k++) {
        const int e = a.pt_edges[k];
        double A[6], B[12];
        edge_jac(a, e, A, B);
        const double r1 = a.e_rho1[e], info = a.e_info[e];
        const double w = r1 * info;
        const double om0 = -info * a.e_err[2 * e] * r1, om1 = -info * a.e_err[2 * e + 1] * r1;
#pragma unroll
        for (int r = 0; r < 3; r++) {
            bl[r] += A[r] * om0 + A[3 + r] * om1;
#pragma unroll
            for (int c = 0; c < 3; c++) H[3 * r + c] += w * (A[r] * A[c] + A[3 + r] * A[3 + c]);
        }
        double* hp = a.Hpl + 18 * e;
        if (a.opt[a.e_pose[e]] >= 0) {
#pragma unroll
            for (int r = 0; r < 6; r++)
#pragma unroll
                for (int c = 0; c < 3; c++) hp[3 * r + c] = w * (B[r] * A[c] + B[6 + r] * A[3 + c]);
        }
    }
#pragma unroll
    for (int i = 0; i < 9; i++) a.Hll[9 * m + i] = H[i];
#pragma unroll
    for (int r = 0; r < 3; r++) a.b[a.n + 3 * m + r] = bl[r];
}

// one wave per optimised pose: 21 upper Hpp terms + 6 b terms, lanes over the pose's edges
__global__ __launch_bounds__(256) void k_ba_lin_poses(BaArgs a) {
    const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (i >= a.np) return;
    double acc[27];
#pragma unroll
    for (int k = 0; k < 27; k++) acc[k] = 0;
    for (int k = a.ps_ptr[i] + lane; k < a.ps_ptr[i + 1]; k += 64) {
        const int e = a.ps_edges[k];
        double A[6], B[12];
        edge_jac(a, e, A, B);
        const double r1 = a.e_rho1[e], info = a.e_info[e];
        const double w = r1 * info;
        const double om0 = -info * a.e_err[2 * e] * r1, om1 = -info * a.e_err[2 * e + 1] * r1;
        int t = 0;
#pragma unroll
        for (int r = 0; r < 6; r++)
#pragma unroll
            for (int c = r; c < 6; c++) acc[t++] += w * (B[r] * B[c] + B[6 + r] * B[6 + c]);
#pragma unroll
        for (int r = 0; r < 6; r++) acc[21 + r] += B[r] * om0 + B[6 + r] * om1;
    }
#pragma unroll
    for (int k = 0; k < 27; k++) {
        double v = acc[k];
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
        acc[k] = v;
    }
    if (lane == 0) {
        int t = 0;
        double* H = a.Hpp + 36 * i;
        for (int r = 0; r < 6; r++)
            for (int c = r; c < 6; c++) { H[6 * r + c] = acc[t]; H[6 * c + r] = acc[t]; t++; }
        for (int r = 0; r < 6; r++) a.b[6 * i + r] = acc[21 + r];
    }
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

__global__ __launch_bounds__(256) void k_ba_schur_points(BaArgs a, double lambda) {
    const int m = blockIdx.x * blockDim.x + threadIdx.x;
    if (m >= a.M) return;
    double D[9], Di[9];
#pragma unroll
    for (int k = 0; k < 9; k++) D[k] = a.Hll[9 * m + k] + (k % 4 == 0 ? lambda : 0.0);
    inv3(D, Di);
#pragma unroll
    for (int k = 0; k < 9; k++) a.Dinv[9 * m + k] = Di[k];
    const double* bl = a.b + a.n + 3 * m;
#pragma unroll
    for (int r = 0; r < 3; r++) a.db[3 * m + r] = Di[3 * r] * bl[0] + Di[3 * r + 1] * bl[1] + Di[3 * r + 2] * bl[2];
    for (int k = a.pt_ptr[m]; k < a.pt_ptr[m + 1]; k++) {
        const int e = a.pt_edges[k];
        if (a.opt[a.e_pose[e]] < 0) continue;
        const double* B1 = a.Hpl + 18 * e;
        double* w = a.W + 18 * e;
#pragma unroll
        for (int r = 0; r < 6; r++)
#pragma unroll
            for (int c = 0; c < 3; c++)
                w[3 * r + c] = B1[3 * r] * Di[c] + B1[3 * r + 1] * Di[3 + c] + B1[3 * r + 2] * Di[6 + c];
    }
}

// one wave per (i <= j) block of S; lanes 0..35 own one entry each
__global__ __launch_bounds__(256) void k_ba_schur_blocks(BaArgs a, double lambda) {
    const int blk = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (blk >= a.nblk || lane >= 36) return;
    const int i = a.blk_i[blk], j = a.blk_j[blk];
    const int r = lane / 6, c = lane - 6 * (lane / 6);
    double s = (i == j) ? a.Hpp[36 * i + 6 * r + c] + (r == c ? lambda : 0.0) : 0.0;
    for (int k = a.blk_ptr[blk]; k < a.blk_ptr[blk + 1]; k++) {
        const int ea = a.blk_pairs[2 * k], eb = a.blk_pairs[2 * k + 1];
        const double* w = a.W + 18 * ea + 3 * r;
        const double* h = a.Hpl + 18 * eb + 3 * c;
        s -= w[0] * h[0] + w[1] * h[1] + w[2] * h[2];
    }
    a.S[(size_t)(6 * i + r) * a.n + 6 * j + c] = s;
    if (i != j) a.S[(size_t)(6 * j + c) * a.n + 6 * i + r] = s;
}

__global__ __launch_bounds__(256) void k_ba_schur_b(BaArgs a) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= a.n) return;
    const int i = t / 6, r = t - 6 * i;
    double s = 0;
    for (int k = a.ps_ptr[i]; k < a.ps_ptr[i + 1]; k++) {
        const int e = a.ps_edges[k];
        const double* h = a.Hpl + 18 * e + 3 * r;
        const double* d = a.db + 3 * a.e_pt[e];
        s += h[0] * d[0] + h[1] * d[1] + h[2] * d[2];
    }
    a.bs[t] = a.b[t] - s;
}

// ---------------------------------------------------------------------------
// dense Cholesky of S (n x n, lower, in place) + solve S xp = bs; one workgroup.
// Panel width 16; the panel below the diagonal block is staged in LDS and the trailing
// update C -= P_I P_J^T runs as 4 x v_mfma_f64_16x16x4f64 per 16x16 tile.
//   f64 MFMA operand map: lane l holds A[l&15][k=l>>4], B[k=l>>4][l&15];
//   C/D: col = l&15, row = (l>>4) + 4*reg.
// ---------------------------------------------------------------------------
constexpr int kCholNB = 16;

__global__ __launch_bounds__(1024) void k_ba_cholesky(double* __restrict__ S, const double* __restrict__ bs,
                                                      double* __restrict__ x, int n, int* __restrict__ flag) {
    extern __shared__ __attribute__((aligned(16))) double lds[];
    int& bad = *(int*)lds;                   // control word (first 16 bytes)
    double* Dg = lds + 2;                    // 16 x 16 diagonal block
    double* y = Dg + 256;                    // n (solution vector)
    double* Pn = y + ((n + 15) & ~15);       // panel rows (n_pad x 16)
    const int tid = threadIdx.x, nt = blockDim.x;
    const int wid = tid >> 6, lane = tid & 63, nw = nt >> 6;
    if (tid == 0) bad = 0;
    __syncthreads();
    for (int k0 = 0; k0 < n; k0 += kCholNB) {
        const int kb = min(kCholNB, n - k0);
        // (a) diagonal block
        for (int t = tid; t < 256; t += nt) {
            const int r = t >> 4, c = t & 15;
            Dg[t] = (r < kb && c <= r) ? S[(size_t)(k0 + r) * n + k0 + c] : 0.0;
        }
        __syncthreads();
        // (b) factor it (wave 0, 4 entries per lane)
        if (wid == 0) {
            for (int j = 0; j < kb; j++) {
                if (lane == 0) {
                    const double p = Dg[17 * j];
                    if (!(p > 0.0)) bad = 1;
                    Dg[17 * j] = sqrt(p > 0.0 ? p : 1.0);
                }
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                const double d = Dg[17 * j];
                if (lane > j && lane < kb) Dg[16 * lane + j] /= d;
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                for (int t = lane; t < 256; t += 64) {
                    const int r = t >> 4, c = t & 15;
                    if (r > j && c > j && c <= r && r < kb) Dg[t] -= Dg[16 * r + j] * Dg[16 * c + j];
                }
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            }
        }
        __syncthreads();
        if (bad) break;
        for (int t = tid; t < 256; t += nt) {
            const int r = t >> 4, c = t & 15;
            if (r < kb && c <= r) S[(size_t)(k0 + r) * n + k0 + c] = Dg[t];
        }
        // (c) panel rows: L[r][0:kb] = A[r][k0:k0+kb] * Dg^{-T}
        const int r0 = k0 + kb;
        const int nr = n - r0;
        const int nr_pad = (nr + 15) & ~15;
        for (int rr = tid; rr < nr_pad; rr += nt) {
            double v[kCholNB];
            const int r = r0 + rr;
#pragma unroll
            for (int c = 0; c < kCholNB; c++) v[c] = (rr < nr && c < kb) ? S[(size_t)r * n + k0 + c] : 0.0;
#pragma unroll
            for (int c = 0; c < kCholNB; c++) {
                if (c < kb) {
                    double s = v[c];
                    for (int p = 0; p < c; p++) s -= v[p] * Dg[16 * c + p];
                    v[c] = s / Dg[17 * c];
                }
            }
#pragma unroll
            for (int c = 0; c < kCholNB; c++) {
                Pn[rr * 16 + c] = v[c];
                if (rr < nr && c < kb) S[(size_t)r * n + k0 + c] = v[c];
            }
        }
        __syncthreads();
        // (d) trailing update, lower tiles only
        const int T = nr_pad / 16;
        const int ntile = T * (T + 1) / 2;
        for (int tile = wid; tile < ntile; tile += nw) {
            int I = (int)((sqrt(8.0 * tile + 1.0) - 1.0) * 0.5);
            while ((I + 1) * (I + 2) / 2 <= tile) I++;
            while (I * (I + 1) / 2 > tile) I--;
            const int J = tile - I * (I + 1) / 2;
            const int row_base = r0 + 16 * I, col_base = r0 + 16 * J;
            double4_t acc;
            const int cc = lane & 15, rq = lane >> 4;
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const int rr = row_base + rq + 4 * q;
                acc[q] = (rr < n && col_base + cc < n) ? S[(size_t)rr * n + col_base + cc] : 0.0;
            }
#pragma unroll
            for (int kk = 0; kk < 4; kk++) {
                const double av = -Pn[(16 * I + cc) * 16 + 4 * kk + rq];
                const double bv = Pn[(16 * J + cc) * 16 + 4 * kk + rq];
                acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc, 0, 0, 0);
            }
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const int rr = row_base + rq + 4 * q;
                if (rr < n && col_base + cc < n) S[(size_t)rr * n + col_base + cc] = acc[q];
            }
        }
        __syncthreads();
    }
    if (bad) {
        if (tid == 0) flag[0] = 0;
        for (int i = tid; i < n; i += nt) x[i] = 0.0;
        return;
    }
    // forward: L y = bs
    for (int i = tid; i < n; i += nt) y[i] = bs[i];
    __syncthreads();
    for (int k0 = 0; k0 < n; k0 += 16) {
        const int kb = min(16, n - k0);
        if (wid == 0) {
            double v = lane < kb ? y[k0 + lane] : 0.0;
            for (int j = 0; j < kb; j++) {
                const double yj = __shfl(v, j, 64) / S[(size_t)(k0 + j) * n + k0 + j];
                if (lane == j) v = yj;
                if (lane > j && lane < kb) v -= S[(size_t)(k0 + lane) * n + k0 + j] * yj;
            }
            if (lane < kb) y[k0 + lane] = v;
        }
        __syncthreads();
        for (int r = k0 + kb + tid; r < n; r += nt) {
            double s = 0;
            for (int j = 0; j < kb; j++) s += S[(size_t)r * n + k0 + j] * y[k0 + j];
            y[r] -= s;
        }
        __syncthreads();
    }
    // backward: L^T x = y
    const int nb = (n + 15) / 16;
    for (int b = nb - 1; b >= 0; b--) {
        const int k0 = 16 * b, kb = min(16, n - k0);
        if (wid == 0) {
            double v = lane < kb ? y[k0 + lane] : 0.0;
            for (int j = kb - 1; j >= 0; j--) {
                const double xj = __shfl(v, j, 64) / S[(size_t)(k0 + j) * n + k0 + j];
                if (lane == j) v = xj;
                if (lane < j) v -= S[(size_t)(k0 + j) * n + k0 + lane] * xj;
            }
            if (lane < kb) y[k0 + lane] = v;
        }
        __syncthreads();
        for (int r = tid; r < k0; r += nt) {
            double s = 0;
            for (int j = 0; j < kb; j++) s += S[(size_t)(k0 + j) * n + r] * y[k0 + j];
            y[r] -= s;
        }
        __syncthreads();
    }
    for (int i = tid; i < n; i += nt) x[i] = y[i];
    if (tid == 0) flag[0] = 1;
}

// ---------------------------------------------------------------------------
// back-substitution + updates (push saves the old state)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_ba_backsub(BaArgs a) {
    const int m = blockIdx.x * blockDim.x + threadIdx.x;
    if (m >= a.M) return;
    const double* bl = a.b + a.n + 3 * m;
    double c[3] = {bl[0], bl[1], bl[2]};
    for (int k = a.pt_ptr[m]; k < a.pt_ptr[m + 1]; k++) {
        const int e = a.pt_edges[k];
        const int oi = a.opt[a.e_pose[e]];
        if (oi < 0) continue;
        const double* h = a.Hpl + 18 * e;
        const double* xp = a.x + 6 * oi;
#pragma unroll
        for (int cc = 0; cc < 3; cc++)
#pragma unroll
            for (int r = 0; r < 6; r++) c[cc] -= h[3 * r + cc] * xp[r];
    }
    const double* Di = a.Dinv + 9 * m;
    double* X = a.pts + 3 * m;
#pragma unroll
    for (int r = 0; r < 3; r++) {
        const double xl = Di[3 * r] * c[0] + Di[3 * r + 1] * c[1] + Di[3 * r + 2] * c[2];
        a.x[a.n + 3 * m + r] = xl;
        a.pts_bak[3 * m + r] = X[r];
        X[r] += xl;
    }
}

__global__ __launch_bounds__(256) void k_ba_update_poses(BaArgs a) {
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= a.P) return;
    double* T = a.pose + 8 * p;
#pragma unroll
    for (int k = 0; k < 8; k++) a.pose_bak[8 * p + k] = T[k];
    const int oi = a.opt[p];
    if (oi < 0) return;
    const double* u = a.x + 6 * oi;
    // SE3Quat::exp
    const double ox = u[0], oy = u[1], oz = u[2];
    const double theta = sqrt(ox * ox + oy * oy + oz * oz);
    const double O[9] = {0, -oz, oy, oz, 0, -ox, -oy, ox, 0};
    double O2[9];
#pragma unroll
    for (int r = 0; r < 3; r++)
#pragma unroll
        for (int c = 0; c < 3; c++) O2[3 * r + c] = O[3 * r] * O[c] + O[3 * r + 1] * O[3 + c] + O[3 * r + 2] * O[6 + c];
    double R[9], V[9];
    if (theta < 0.00001) {
#pragma unroll
        for (int i = 0; i < 9; i++) { R[i] = (i % 4 == 0 ? 1.0 : 0.0) + O[i] + O2[i]; V[i] = R[i]; }
    } else {
        const double sa = sin(theta) / theta, cb = (1 - cos(theta)) / (theta * theta);
        const double cc = (theta - sin(theta)) / (theta * theta * theta);
#pragma unroll
        for (int i = 0; i < 9; i++) {
            R[i] = (i % 4 == 0 ? 1.0 : 0.0) + sa * O[i] + cb * O2[i];
            V[i] = (i % 4 == 0 ? 1.0 : 0.0) + cb * O[i] + cc * O2[i];
        }
    }
    DQ qe = mattoq(R);
    qnormalize(qe);
    const double tex = V[0] * u[3] + V[1] * u[4] + V[2] * u[5];
    const double tey = V[3] * u[3] + V[4] * u[4] + V[5] * u[5];
    const double tez = V[6] * u[3] + V[7] * u[4] + V[8] * u[5];
    // exp(d) * T
    const DQ qt = load_q(T);
    double rx, ry, rz;
    qrot(qe, T[4], T[5], T[6], rx, ry, rz);
    DQ q{qe.w * qt.x + qe.x * qt.w + qe.y * qt.z - qe.z * qt.y, qe.w * qt.y + qe.y * qt.w + qe.z * qt.x - qe.x * qt.z,
         qe.w * qt.z + qe.z * qt.w + qe.x * qt.y - qe.y * qt.x, qe.w * qt.w - qe.x * qt.x - qe.y * qt.y - qe.z * qt.z};
    qnormalize(q);
    T[0] = q.x; T[1] = q.y; T[2] = q.z; T[3] = q.w;
    T[4] = tex + rx; T[5] = tey + ry; T[6] = tez + rz;
}

// ---------------------------------------------------------------------------
// reductions (one workgroup, fixed order): [0] sum rho0, [1] computeScale, [2] max diag
// ---------------------------------------------------------------------------
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

__global__ __launch_bounds__(1024) void k_ba_reduce(BaArgs a, double lambda, int what) {
    __shared__ double sh[16];
    double v = 0;
    if (what & 1) {
        for (int e = threadIdx.x; e < a.E; e += blockDim.x) v += a.e_rho0[e];
        v = block_sum(v, sh);
        if (threadIdx.x == 0) a.red[0] = v;
    }
    if (what & 2) {
        v = 0;
        const int N = a.n + 3 * a.M;
        for (int j = threadIdx.x; j < N; j += blockDim.x) v += a.x[j] * (lambda * a.x[j] + a.b[j]);
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
}

// ---------------------------------------------------------------------------
// host workspace
// ---------------------------------------------------------------------------
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
    hipError_t up(const std::vector<T>& v, hipStream_t st) {
        hipError_t e = ensure(v.size());
        if (e != hipSuccess || v.empty()) return e;
        return hipMemcpyAsync(p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice, st);
    }
};

struct BaWorkspace {
    DBuf<double> pose, pose_bak, pts, pts_bak, e_obs, e_info, e_err, e_chi2, e_rho0, e_rho1, Hpp, Hll, Hpl, b, Dinv, db,
        W, S, bs, x, red;
    DBuf<int> opt, e_pose, e_pt, pt_ptr, pt_edges, ps_ptr, ps_edges, blk_i, blk_j, blk_ptr, blk_pairs, flag;
    double* h_red = nullptr;   // pinned: red[3] + flag
};

BaWorkspace* ba_create() {
    BaWorkspace* w = new BaWorkspace();
    if (hipHostMalloc((void**)&w->h_red, 64, hipHostMallocDefault) != hipSuccess) { delete w; return nullptr; }
    return w;
}

void ba_destroy(BaWorkspace* w) {
    if (!w) return;
    if (w->h_red) (void)hipHostFree(w->h_red);
    delete w;
}

#define BAOK(x)                                                                                    \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess) {                                                                    \
            std::fprintf(stderr, "orbhip ba: %s: %s\n", #x, hipGetErrorString(e_));                \
            return ORBHIP_ERR_DEVICE;                                                              \
        }                                                                                          \
    } while (0)

static inline void se3_from_float(const float* q, const float* t, double out[8]) {
    double x = q[0], y = q[1], z = q[2], w = q[3];
    if (w < 0) { x = -x; y = -y; z = -z; w = -w; }
    const double n = std::sqrt(x * x + y * y + z * z + w * w);
    out[0] = x / n; out[1] = y / n; out[2] = z / n; out[3] = w / n;
    out[4] = t[0]; out[5] = t[1]; out[6] = t[2]; out[7] = 0;
}

int ba_solve(BaWorkspace* ws, const orbhip_ba_problem* pr, orbhip_ba_result* res, const volatile int* stop,
             hipStream_t st) {
    const int P = pr->n_poses, M = pr->n_points, E = pr->n_edges;
    if (P < 0 || M < 0 || E < 0 || (P && (!pr->pose_q || !pr->pose_t || !pr->pose_fixed)) || (M && !pr->points) ||
        (E && (!pr->edge_pose || !pr->edge_point || !pr->edge_uv || !pr->edge_octave || !pr->inv_sigma2)))
        return ORBHIP_ERR_ARG;
    for (int e = 0; e < E; e++)
        if (pr->edge_pose[e] < 0 || pr->edge_pose[e] >= P || pr->edge_point[e] < 0 || pr->edge_point[e] >= M ||
            pr->edge_octave[e] < 0 || pr->edge_octave[e] >= pr->n_octaves)
            return ORBHIP_ERR_ARG;
    // ---- host-side structure (index mapping, CSR, Schur pair lists) ----
    std::vector<int> opt(P, -1);
    int np = 0;
    for (int i = 0; i < P; i++)
        if (!pr->pose_fixed[i]) opt[i] = np++;
    const int n = 6 * np;
    if (n > 1024) return ORBHIP_ERR_UNSUPPORTED;   // single-workgroup Cholesky envelope (round 1)
    std::vector<double> pose((size_t)8 * P), pts((size_t)3 * M), obs((size_t)2 * E), info(E);
    for (int i = 0; i < P; i++) se3_from_float(pr->pose_q + 4 * i, pr->pose_t + 3 * i, &pose[8 * i]);
    for (int k = 0; k < 3 * M; k++) pts[k] = pr->points[k];
    for (int e = 0; e < E; e++) {
        obs[2 * e] = pr->edge_uv[2 * e];
        obs[2 * e + 1] = pr->edge_uv[2 * e + 1];
        info[e] = (double)pr->inv_sigma2[pr->edge_octave[e]];
    }
    std::vector<int> pt_ptr(M + 1, 0), ps_ptr(np + 1, 0);
    for (int e = 0; e < E; e++) {
        pt_ptr[pr->edge_point[e] + 1]++;
        if (opt[pr->edge_pose[e]] >= 0) ps_ptr[opt[pr->edge_pose[e]] + 1]++;
    }
    for (int m = 0; m < M; m++) pt_ptr[m + 1] += pt_ptr[m];
    for (int i = 0; i < np; i++) ps_ptr[i + 1] += ps_ptr[i];
    std::vector<int> pt_edges(E), ps_edges(ps_ptr[np]);
    {
        std::vector<int> fp(pt_ptr.begin(), pt_ptr.end() - 1), fq(ps_ptr.begin(), ps_ptr.end() - 1);
        for (int e = 0; e < E; e++) {
            pt_edges[fp[pr->edge_point[e]]++] = e;
            const int oi = opt[pr->edge_pose[e]];
            if (oi >= 0) ps_edges[fq[oi]++] = e;
        }
    }
    // Schur pairs: for every landmark, every (a, b) of its edges with opt(a) <= opt(b)
    std::map<std::pair<int, int>, std::vector<std::pair<int, int>>> blocks;
    for (int i = 0; i < np; i++) blocks[{i, i}];   // diagonal blocks always present
    for (int m = 0; m < M; m++) {
        for (int ka = pt_ptr[m]; ka < pt_ptr[m + 1]; ka++) {
            const int ea = pt_edges[ka], ia = opt[pr->edge_pose[ea]];
            if (ia < 0) continue;
            for (int kb = pt_ptr[m]; kb < pt_ptr[m + 1]; kb++) {
                const int eb = pt_edges[kb], ib = opt[pr->edge_pose[eb]];
                if (ib < 0 || ib < ia) continue;
                blocks[{ia, ib}].push_back({ea, eb});
            }
        }
    }
    std::vector<int> blk_i, blk_j, blk_ptr(1, 0), blk_pairs;
    for (auto& kv : blocks) {
        blk_i.push_back(kv.first.first);
        blk_j.push_back(kv.first.second);
        for (auto& pe : kv.second) { blk_pairs.push_back(pe.first); blk_pairs.push_back(pe.second); }
        blk_ptr.push_back((int)blk_pairs.size() / 2);
    }
    const int nblk = (int)blk_i.size();
    // ---- upload ----
    std::vector<int> ep(pr->edge_pose, pr->edge_pose + E), em(pr->edge_point, pr->edge_point + E);
    BAOK(ws->pose.up(pose, st)); BAOK(ws->pose_bak.ensure(pose.size()));
    BAOK(ws->pts.up(pts, st)); BAOK(ws->pts_bak.ensure(pts.size()));
    BAOK(ws->e_obs.up(obs, st)); BAOK(ws->e_info.up(info, st));
    BAOK(ws->opt.up(opt, st)); BAOK(ws->e_pose.up(ep, st)); BAOK(ws->e_pt.up(em, st));
    BAOK(ws->pt_ptr.up(pt_ptr, st)); BAOK(ws->pt_edges.up(pt_edges, st));
    BAOK(ws->ps_ptr.up(ps_ptr, st)); BAOK(ws->ps_edges.up(ps_edges, st));
    BAOK(ws->blk_i.up(blk_i, st)); BAOK(ws->blk_j.up(blk_j, st));
    BAOK(ws->blk_ptr.up(blk_ptr, st)); BAOK(ws->blk_pairs.up(blk_pairs, st));
    BAOK(ws->e_err.ensure(2 * (size_t)E)); BAOK(ws->e_chi2.ensure(E)); BAOK(ws->e_rho0.ensure(E));
    BAOK(ws->e_rho1.ensure(E));
    BAOK(ws->Hpp.ensure((size_t)36 * np)); BAOK(ws->Hll.ensure((size_t)9 * M));
    BAOK(ws->Hpl.ensure((size_t)18 * E)); BAOK(ws->b.ensure((size_t)n + 3 * M));
    BAOK(ws->Dinv.ensure((size_t)9 * M)); BAOK(ws->db.ensure((size_t)3 * M)); BAOK(ws->W.ensure((size_t)18 * E));
    BAOK(ws->S.ensure((size_t)n * n)); BAOK(ws->bs.ensure(n)); BAOK(ws->x.ensure((size_t)n + 3 * M));
    BAOK(ws->red.ensure(4)); BAOK(ws->flag.ensure(4));
    BAOK(hipMemsetAsync(ws->Hpl.p, 0, sizeof(double) * 18 * std::max(E, 1), st));
    BAOK(hipMemsetAsync(ws->W.p, 0, sizeof(double) * 18 * std::max(E, 1), st));
    BaArgs a;
    a.P = P; a.M = M; a.E = E; a.np = np; a.n = n;
    a.fx = pr->fx; a.fy = pr->fy; a.cx = pr->cx; a.cy = pr->cy; a.delta = pr->huber_delta;
    a.pose = ws->pose.p; a.pose_bak = ws->pose_bak.p; a.pts = ws->pts.p; a.pts_bak = ws->pts_bak.p;
    a.opt = ws->opt.p; a.e_pose = ws->e_pose.p; a.e_pt = ws->e_pt.p; a.e_obs = ws->e_obs.p; a.e_info = ws->e_info.p;
    a.e_err = ws->e_err.p; a.e_chi2 = ws->e_chi2.p; a.e_rho0 = ws->e_rho0.p; a.e_rho1 = ws->e_rho1.p;
    a.Hpp = ws->Hpp.p; a.Hll = ws->Hll.p; a.Hpl = ws->Hpl.p; a.b = ws->b.p; a.Dinv = ws->Dinv.p; a.db = ws->db.p;
    a.W = ws->W.p; a.S = ws->S.p; a.bs = ws->bs.p; a.x = ws->x.p;
    a.pt_ptr = ws->pt_ptr.p; a.pt_edges = ws->pt_edges.p; a.ps_ptr = ws->ps_ptr.p; a.ps_edges = ws->ps_edges.p;
    a.blk_i = ws->blk_i.p; a.blk_j = ws->blk_j.p; a.blk_ptr = ws->blk_ptr.p; a.blk_pairs = ws->blk_pairs.p;
    a.nblk = nblk; a.red = ws->red.p; a.flag = ws->flag.p;
    const size_t chol_lds = sizeof(double) * (2 + 256 + ((n + 15) & ~15) + (size_t)((n + 15) & ~15) * 16);
    if (chol_lds > 160 * 1024) return ORBHIP_ERR_UNSUPPORTED;
    static bool lds_set = false;
    if (!lds_set) {
        BAOK(hipFuncSetAttribute((const void*)k_ba_cholesky, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
        lds_set = true;
    }
    (void)hipGetLastError();   // clear any sticky error left by an earlier, already-reported call
    auto g = [](int n_, int b_) { return dim3((unsigned)std::max(1, (n_ + b_ - 1) / b_)); };
    auto read_red = [&](int what) -> int {
        BAOK(hipMemcpyAsync(ws->h_red, ws->red.p, 4 * sizeof(double), hipMemcpyDeviceToHost, st));
        if (what) BAOK(hipMemcpyAsync(ws->h_red + 4, ws->flag.p, sizeof(int), hipMemcpyDeviceToHost, st));
        BAOK(hipStreamSynchronize(st));
        return ORBHIP_OK;
    };
    // ---- optimize(iterations) ----
    if (E > 0) hipLaunchKernelGGL(k_ba_errors, g(E, 256), dim3(256), 0, st, a);
    hipLaunchKernelGGL(k_ba_reduce, dim3(1), dim3(1024), 0, st, a, 0.0, 1);
    BAOK(hipGetLastError());
    if (read_red(0)) return ORBHIP_ERR_DEVICE;
    double currentChi = ws->h_red[0];
    res->initial_chi2 = currentChi;
    double lambda = 0, ni = 2;
    int nBad = 0, it = 0, trials = 0;
    const double dmax = std::numeric_limits<double>::max();
    bool errors_valid = true;
    for (it = 0; it < pr->iterations && !(stop && *stop); it++) {
        if (!errors_valid && E > 0) hipLaunchKernelGGL(k_ba_errors, g(E, 256), dim3(256), 0, st, a);
        errors_valid = true;
        if (M > 0) hipLaunchKernelGGL(k_ba_lin_points, g(M, 256), dim3(256), 0, st, a);
        if (np > 0) hipLaunchKernelGGL(k_ba_lin_poses, g(np, 4), dim3(256), 0, st, a);
        if (it == 0) {
            hipLaunchKernelGGL(k_ba_reduce, dim3(1), dim3(1024), 0, st, a, 0.0, 4);
            if (read_red(0)) return ORBHIP_ERR_DEVICE;
            lambda = 1e-5 * ws->h_red[2];
            ni = 2;
            nBad = 0;
        }
        double rho = 0, tempChi = currentChi;
        int qmax = 0;
        do {
            // setLambda + Schur + solve + update (push happens inside the update kernels)
            if (n > 0) BAOK(hipMemsetAsync(a.S, 0, sizeof(double) * (size_t)n * n, st));
            if (M > 0) hipLaunchKernelGGL(k_ba_schur_points, g(M, 256), dim3(256), 0, st, a, lambda);
            if (nblk > 0) hipLaunchKernelGGL(k_ba_schur_blocks, g(nblk, 4), dim3(256), 0, st, a, lambda);
            if (n > 0) {
                hipLaunchKernelGGL(k_ba_schur_b, g(n, 256), dim3(256), 0, st, a);
                hipLaunchKernelGGL(k_ba_cholesky, dim3(1), dim3(1024), chol_lds, st, a.S, a.bs, a.x, n, a.flag);
            } else {
                BAOK(hipMemsetAsync(a.flag, 0xFF, sizeof(int), st));
            }
            if (M > 0) hipLaunchKernelGGL(k_ba_backsub, g(M, 256), dim3(256), 0, st, a);
            if (P > 0) hipLaunchKernelGGL(k_ba_update_poses, g(P, 256), dim3(256), 0, st, a);
            if (E > 0) hipLaunchKernelGGL(k_ba_errors, g(E, 256), dim3(256), 0, st, a);
            hipLaunchKernelGGL(k_ba_reduce, dim3(1), dim3(1024), 0, st, a, lambda, 3);
            BAOK(hipGetLastError());
            if (read_red(1)) return ORBHIP_ERR_DEVICE;
            const bool ok2 = *(int*)(ws->h_red + 4) != 0;
            tempChi = ws->h_red[0];
            if (!ok2) tempChi = dmax;
            rho = currentChi - tempChi;
            double scale = ws->h_red[1] + 1e-3;
            rho /= scale;
            if (rho > 0 && std::isfinite(tempChi)) {
                double alpha = 1. - std::pow((2 * rho - 1), 3);
                alpha = std::min(alpha, 2. / 3.);
                lambda *= std::max(1. / 3., alpha);
                ni = 2;
                if (pr->early_stop) {
                    if ((currentChi - tempChi) < 1e-3 * currentChi) nBad++;
                    else nBad = 0;
                }
                currentChi = tempChi;
            } else {
                lambda *= ni;
                ni *= 2;
                // pop: restore the pre-trial state
                BAOK(hipMemcpyAsync(a.pose, a.pose_bak, sizeof(double) * 8 * (size_t)P, hipMemcpyDeviceToDevice, st));
                BAOK(hipMemcpyAsync(a.pts, a.pts_bak, sizeof(double) * 3 * (size_t)M, hipMemcpyDeviceToDevice, st));
            }
            qmax++;
            trials++;
        } while (rho < 0 && qmax < 10 && !(stop && *stop));
        // g2o recomputes the active errors at the start of every iteration; after an accepted
        // trial the device already holds them, after a rejected one they belong to the popped
        // trial (left stale for e->chi2(), exactly like g2o) and are refreshed below if we go on.
        errors_valid = rho > 0;
        if (qmax == 10 || rho == 0) { it++; break; }
        if (pr->early_stop && nBad >= 3) { it++; break; }
    }
    res->final_chi2 = currentChi;
    res->iterations_done = it;
    res->lm_trials = trials;
    // ---- outputs ----
    std::vector<double> pose_o((size_t)8 * P), pts_o((size_t)3 * M), chi2_o(E);
    if (P) BAOK(hipMemcpyAsync(pose_o.data(), a.pose, sizeof(double) * 8 * P, hipMemcpyDeviceToHost, st));
    if (M) BAOK(hipMemcpyAsync(pts_o.data(), a.pts, sizeof(double) * 3 * M, hipMemcpyDeviceToHost, st));
    if (E) BAOK(hipMemcpyAsync(chi2_o.data(), a.e_chi2, sizeof(double) * E, hipMemcpyDeviceToHost, st));
    BAOK(hipStreamSynchronize(st));
    for (int i = 0; i < P; i++) {
        if (res->pose_q) for (int k = 0; k < 4; k++) res->pose_q[4 * i + k] = (float)pose_o[8 * i + k];
        if (res->pose_t) for (int k = 0; k < 3; k++) res->pose_t[3 * i + k] = (float)pose_o[8 * i + 4 + k];
    }
    if (res->points) for (int k = 0; k < 3 * M; k++) res->points[k] = (float)pts_o[k];
    for (int e = 0; e < E; e++) {
        if (res->edge_chi2) res->edge_chi2[e] = (float)chi2_o[e];
        if (res->edge_depth_ok) {   // isDepthPositive: (T.map(X)).z > 0
            const double* T = &pose_o[8 * pr->edge_pose[e]];
            const double* X = &pts_o[3 * pr->edge_point[e]];
            double ux = T[1] * X[2] - T[2] * X[1], uy = T[2] * X[0] - T[0] * X[2];
            ux += ux; uy += uy;
            const double uz2 = 2 * (T[0] * X[1] - T[1] * X[0]);
            const double cz = T[0] * uy - T[1] * ux;
            const double z = X[2] + T[3] * uz2 + cz + T[6];
            res->edge_depth_ok[e] = z > 0.0 ? 1 : 0;
        }
    }
    return ORBHIP_OK;
}

}  // namespace orbhip
