// Multi-workgroup dense Cholesky + solve of the reduced camera system S xp = bs for large
// problems (GlobalBundleAdjustment / BundleAdjustment, SURVEY.md §8 a20/a22: n = 6 * #optimised
// KFs, up to 4096), right-looking with 32-column panels:
//   k_cb_diag    one wavefront factors the 32x32 diagonal block in registers (chol_diag_wave):
//                L11 into S, L11^{-1} into Lsave (the solves reuse it)
//   k_cb_panel   L21 = A21 L11^{-T} on v_mfma_f64_16x16x4f64, one wave per 16-row block
//   k_cb_update  C -= L21_I L21_J^T over 64x64 lower tiles of the trailing matrix (MFMA)
//   k_cb_solve   forward / backward substitution, one 1024-thread workgroup, y in LDS
// Structure: row_first[R] = first 32-column tile with a structural non-zero in 32-row tile R of
// S. The envelope (profile) of a symmetric matrix is preserved by its Cholesky factor, so every
// tile left of row_first stays zero: the panel, update and solve kernels skip it. A banded or
// arrow-shaped S (a loop of keyframes with a co-visibility window) costs O(n b^2), not O(n^3).
// Only the lower triangle of S is read; the update writes lower tiles (diagonal tiles in full,
// their upper half is never read).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <vector>

#include "ba_chol.h"
#include "ba_chol_blocked.h"

namespace orbhip {

constexpr int kCT = 32;    // panel width / structure tile
constexpr int kUT = 64;    // trailing-update tile

__global__ __launch_bounds__(64) void k_cb_diag(double* __restrict__ S, int n, int k0, double* __restrict__ Lsave,
                                                int* __restrict__ flag) {
    __shared__ double Li[32 * 33];
    int bad = 0;
    chol_diag_wave(S, n, k0, min(kCT, n - k0), Li, Lsave, &bad);
    if (threadIdx.x == 0 && bad) flag[0] = 0;
}

__global__ __launch_bounds__(256) void k_cb_panel(double* __restrict__ S, int n, int k0,
                                                  const double* __restrict__ Lsave, const int* __restrict__ row_first) {
    __shared__ double Li[32 * 33];
    const int tid = threadIdx.x, wid = tid >> 6, lane = tid & 63;
    const double* Lp = Lsave + (size_t)(k0 / kCT) * 1024;
    for (int t = tid; t < 1024; t += 256) Li[(t >> 5) * 33 + (t & 31)] = Lp[t];
    __syncthreads();
    const int r0 = k0 + kCT + 16 * (blockIdx.x * 4 + wid);
    if (r0 >= n || row_first[r0 / kCT] > k0 / kCT) return;   // wave-uniform
    const int cc = lane & 15, rq = lane >> 4;
    double4_t acc0 = {0, 0, 0, 0}, acc1 = {0, 0, 0, 0};
    const bool rin = r0 + cc < n;
#pragma unroll
    for (int kk = 0; kk < 8; kk++) {
        const double av = rin ? S[(size_t)(r0 + cc) * n + k0 + 4 * kk + rq] : 0.0;
        const double b0 = Li[cc * 33 + 4 * kk + rq];
        const double b1 = Li[(16 + cc) * 33 + 4 * kk + rq];
        acc0 = __builtin_amdgcn_mfma_f64_16x16x4f64(av, b0, acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f64_16x16x4f64(av, b1, acc1, 0, 0, 0);
    }
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const int row = r0 + rq + 4 * q;
        if (row < n) {
            S[(size_t)row * n + k0 + cc] = acc0[q];
            S[(size_t)row * n + k0 + 16 + cc] = acc1[q];
        }
    }
}

// lower 64x64 tile (I, J), I >= J, of the trailing matrix starting at t0; wave w owns rows
// 16w..16w+15 of the tile against all 64 columns (4 MFMA accumulators, K = 32)
__global__ __launch_bounds__(256) void k_cb_update(double* __restrict__ S, int n, int k0,
                                                   const int* __restrict__ row_first) {
    __shared__ double Bt[kUT * 34];
    const int t0 = k0 + kCT;
    int tt = blockIdx.x;
    int I = (int)((sqrtf(8.0f * (float)tt + 1.0f) - 1.0f) * 0.5f);
    while ((I + 1) * (I + 2) / 2 <= tt) I++;
    while (I * (I + 1) / 2 > tt) I--;
    const int J = tt - I * (I + 1) / 2;
    const int ri = t0 + kUT * I, rj = t0 + kUT * J;
    const int kt = k0 / kCT;
    // structure: the 64-row tile is non-zero in this panel if either 32-row half is
    const int fi = min(row_first[ri / kCT], ri + kCT < n ? row_first[ri / kCT + 1] : 1 << 30);
    const int fj = min(row_first[rj / kCT], rj + kCT < n ? row_first[rj / kCT + 1] : 1 << 30);
    if (fi > kt || fj > kt) return;   // workgroup-uniform
    const int tid = threadIdx.x, wid = tid >> 6, lane = tid & 63;
    for (int t = tid; t < kUT * kCT; t += 256) {
        const int r = t >> 5, c = t & 31;
        Bt[r * 34 + c] = rj + r < n ? S[(size_t)(rj + r) * n + k0 + c] : 0.0;
    }
    const int cc = lane & 15, rq = lane >> 4;
    const int rowA = ri + 16 * wid + cc;
    double av[8];
#pragma unroll
    for (int kk = 0; kk < 8; kk++) av[kk] = rowA < n ? -S[(size_t)rowA * n + k0 + 4 * kk + rq] : 0.0;
    __syncthreads();
    double4_t acc[4];
#pragma unroll
    for (int u = 0; u < 4; u++) {
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const int row = ri + 16 * wid + rq + 4 * q, col = rj + 16 * u + cc;
            acc[u][q] = (row < n && col < n) ? S[(size_t)row * n + col] : 0.0;
        }
    }
#pragma unroll
    for (int u = 0; u < 4; u++) {
        if (I == J && u > wid) continue;   // strictly-upper 16x16 blocks of a diagonal tile
#pragma unroll
        for (int kk = 0; kk < 8; kk++) {
            const double bv = Bt[(16 * u + cc) * 34 + 4 * kk + rq];
            acc[u] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[kk], bv, acc[u], 0, 0, 0);
        }
    }
#pragma unroll
    for (int u = 0; u < 4; u++) {
        if (I == J && u > wid) continue;
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const int row = ri + 16 * wid + rq + 4 * q, col = rj + 16 * u + cc;
            if (row < n && col < n) S[(size_t)row * n + col] = acc[u][q];
        }
    }
}

// L y = bs, L^T x = y with the factor in the lower triangle of S and the panel inverses in
// Lsave; flag[0] == 0 (a non-positive pivot) -> x = 0. y lives in LDS (n <= kCbMaxN).
__global__ __launch_bounds__(1024) void k_cb_solve(const double* __restrict__ S, int n,
                                                   const double* __restrict__ Lsave, const double* __restrict__ bs,
                                                   double* __restrict__ x, const int* __restrict__ flag,
                                                   const int* __restrict__ row_first) {
    __shared__ double y[kCbMaxN];
    __shared__ double red[32 * 33];
    __shared__ double w[32];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    if (flag[0] == 0) {
        for (int i = tid; i < n; i += 1024) x[i] = 0.0;
        return;
    }
    for (int i = tid; i < n; i += 1024) y[i] = bs[i];
    __syncthreads();
    const int np_ = (n + kCT - 1) / kCT;
    // ---- forward: y_p = L11^{-1} y_p, then y_below -= L21 y_p ----
    for (int p = 0; p < np_; p++) {
        const int k0 = p * kCT, kb = min(kCT, n - k0);
        if (tid < kCT) {
            const double* Lp = Lsave + (size_t)p * 1024 + tid * 32;
            double s = 0.0;
            for (int k = 0; k < kb; k++) s += Lp[k] * y[k0 + k];
            w[tid] = tid < kb ? s : 0.0;
        }
        __syncthreads();
        if (tid < kb) y[k0 + tid] = w[tid];
        // 16 lanes per row, 2 columns per lane: 4 rows per wave, 64 rows per pass
        const int sub = lane >> 4, l16 = lane & 15;
        for (int r = k0 + kb + wid * 4 + sub; r < n; r += 64) {
            if (row_first[r / kCT] > p) continue;
            const double* Lr = S + (size_t)r * n + k0;
            double v = Lr[2 * l16] * w[2 * l16] + Lr[2 * l16 + 1] * w[2 * l16 + 1];
#pragma unroll
            for (int o = 8; o > 0; o >>= 1) v += __shfl_xor(v, o, 16);
            if (l16 == 0) y[r] -= v;
        }
        __syncthreads();
    }
    // ---- backward: x_p = L11^{-T} (y_p - L21^T x_below) ----
    for (int p = np_ - 1; p >= 0; p--) {
        const int k0 = p * kCT, kb = min(kCT, n - k0);
        {
            const int c = tid & 31, g = tid >> 5;   // 32 row groups
            double s2 = 0.0;
            if (c < kb)
                for (int r = k0 + kb + g; r < n; r += 32)
                    if (row_first[r / kCT] <= p) s2 += S[(size_t)r * n + k0 + c] * y[r];
            red[g * 33 + c] = s2;
        }
        __syncthreads();
        if (tid < kCT) {
            double s2 = 0.0;
            for (int g = 0; g < 32; g++) s2 += red[g * 33 + tid];
            w[tid] = tid < kb ? y[k0 + tid] - s2 : 0.0;
        }
        __syncthreads();
        if (tid < kb) {
            const double* Lp = Lsave + (size_t)p * 1024;
            double s2 = 0.0;
            for (int k = 0; k < kCT; k++) s2 += Lp[k * 32 + tid] * w[k];
            y[k0 + tid] = s2;   // x_p (y is overwritten from the end)
        }
        __syncthreads();
    }
    for (int i = tid; i < n; i += 1024) x[i] = y[i];
}

__global__ void k_cb_flag_set(int* flag) { flag[0] = 1; }

void chol_blocked_solve(double* S, int n, double* Lsave, const double* bs, double* x, int* flag,
                        const int* row_first, hipStream_t st) {
    hipLaunchKernelGGL(k_cb_flag_set, dim3(1), dim3(1), 0, st, flag);
    const int np_ = (n + kCT - 1) / kCT;
    for (int p = 0; p < np_; p++) {
        const int k0 = p * kCT;
        hipLaunchKernelGGL(k_cb_diag, dim3(1), dim3(64), 0, st, S, n, k0, Lsave, flag);
        const int rest = n - (k0 + kCT);
        if (rest <= 0) break;
        hipLaunchKernelGGL(k_cb_panel, dim3((unsigned)((rest + 63) / 64)), dim3(256), 0, st, S, n, k0, Lsave,
                           row_first);
        const int T = (rest + kUT - 1) / kUT;
        hipLaunchKernelGGL(k_cb_update, dim3((unsigned)(T * (T + 1) / 2)), dim3(256), 0, st, S, n, k0, row_first);
    }
    hipLaunchKernelGGL(k_cb_solve, dim3(1), dim3(1024), 0, st, S, n, Lsave, bs, x, flag, row_first);
}

// test hook: solve A x = b (A dense SPD, n <= kCbMaxN) through the blocked path; ms = device time
int chol_blocked_test(const double* A, const double* b, double* x, int n, float* ms) {
    if (n <= 0 || n > kCbMaxN) return -1;
    const int nt = (n + kCT - 1) / kCT;
    std::vector<int> rf(nt);
    row_first_from_dense(A, n, rf.data());
    double *dS = nullptr, *db = nullptr, *dx = nullptr, *dL = nullptr;
    int *df = nullptr, *drf = nullptr;
    int rc = 0;
    auto ok = [&](hipError_t e) { if (e != hipSuccess && rc == 0) rc = -3; return e == hipSuccess; };
    ok(hipMalloc((void**)&dS, sizeof(double) * n * n));
    ok(hipMalloc((void**)&db, sizeof(double) * n));
    ok(hipMalloc((void**)&dx, sizeof(double) * n));
    ok(hipMalloc((void**)&dL, sizeof(double) * 1024 * nt));
    ok(hipMalloc((void**)&df, sizeof(int)));
    ok(hipMalloc((void**)&drf, sizeof(int) * nt));
    if (rc == 0) {
        ok(hipMemcpy(dS, A, sizeof(double) * n * n, hipMemcpyHostToDevice));
        ok(hipMemcpy(db, b, sizeof(double) * n, hipMemcpyHostToDevice));
        ok(hipMemcpy(drf, rf.data(), sizeof(int) * nt, hipMemcpyHostToDevice));
        hipEvent_t e0, e1;
        ok(hipEventCreate(&e0)); ok(hipEventCreate(&e1));
        ok(hipEventRecord(e0, nullptr));
        chol_blocked_solve(dS, n, dL, db, dx, df, drf, nullptr);
        ok(hipEventRecord(e1, nullptr));
        ok(hipDeviceSynchronize());
        ok(hipGetLastError());
        ok(hipEventElapsedTime(ms, e0, e1));
        int f = 0;
        ok(hipMemcpy(&f, df, sizeof(int), hipMemcpyDeviceToHost));
        ok(hipMemcpy(x, dx, sizeof(double) * n, hipMemcpyDeviceToHost));
        if (rc == 0 && f == 0) rc = -4;
        (void)hipEventDestroy(e0); (void)hipEventDestroy(e1);
    }
    (void)hipFree(dS); (void)hipFree(db); (void)hipFree(dx); (void)hipFree(dL); (void)hipFree(df); (void)hipFree(drf);
    return rc;
}

}  // namespace orbhip
