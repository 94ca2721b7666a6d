// Multi-workgroup dense Cholesky + solve of the reduced camera system S xp = bs for large
// problems (GlobalBundleAdjustment / BundleAdjustment, SURVEY.md §8 a20/a22: n = 6 * #optimised
// KFs, up to 4096), right-looking with 32-column panels:
//   k_cb_diag    one wavefront factors the 32x32 diagonal block in registers (chol_diag_wave):
//                L11 into S, L11^{-1} into Lsave (the backward solve reuses it), and applies
//                y_p = L11^{-1} x_p (the forward substitution rides on the factorization: x holds
//                bs, and each panel subtracts L21 y_p from the rows below it)
//   k_cb_panel   L21 = A21 L11^{-T} on v_mfma_f64_16x16x4f64, one wave per 16-row block, and
//                x_r -= L21[r] y_p for its rows
//   k_cb_update  C -= L21_I L21_J^T over 64x64 lower tiles of the trailing matrix (MFMA); the
//                work-group of tile (0, 0) then factors the next diagonal block (no k_cb_diag
//                launch after the first panel)
//   k_cb_back    backward substitution, one 1024-thread workgroup, x in LDS: per panel the 32x32
//                factor tiles below it (its envelope), loaded one panel ahead into registers
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
#include "ba_args.h"
#include "ba_chol_blocked.h"
#include "wave_f64.h"

namespace orbhip {

constexpr int kCT = 32;    // panel width / structure tile
constexpr int kUT = 64;    // trailing-update tile

// factor the diagonal block at k0 (one wave) and apply the forward step y_p = L11^{-1} x_p in place;
// Li: 32 x 33 doubles of LDS, xs: 32
__device__ __forceinline__ void cb_diag_forward(double* __restrict__ S, int n, int k0, double* __restrict__ Li,
                                                double* __restrict__ xs, double* __restrict__ Lsave,
                                                double* __restrict__ x, int* __restrict__ flag) {
    const int lane = threadIdx.x & 63, kb = min(kCT, n - k0);
    int bad = 0;
    chol_diag_wave(S, n, k0, kb, Li, Lsave, &bad);
    if (lane < kCT) xs[lane] = lane < kb ? x[k0 + lane] : 0.0;
    wave_lds_sync();
    if (lane < kb) {
        double s = 0.0;
        for (int c = 0; c <= lane; c++) s += Li[lane * 33 + c] * xs[c];
        x[k0 + lane] = s;
    }
    if (lane == 0 && bad) flag[0] = 0;
}

// gate: the device-driven LM rounds (ba_solver.hip) run a problem's solve only in its trial phase
// (the phase word of its LmCtl); nullptr = always
#define CB_GATE \
    if (gate && *gate != kPhTrial) return;

__global__ __launch_bounds__(64) void k_cb_diag(double* __restrict__ S, int n, int k0, double* __restrict__ Lsave,
                                                double* __restrict__ x, int* __restrict__ flag, const int* __restrict__ gate) {
    CB_GATE
    __shared__ double Li[32 * 33 + 32];
    cb_diag_forward(S, n, k0, Li, Li + 32 * 33, Lsave, x, flag);
}

// x = bs (the forward substitution runs in x), flag = 1
__global__ __launch_bounds__(256) void k_cb_init(const double* __restrict__ bs, double* __restrict__ x, int n,
                                                 int* __restrict__ flag, const int* __restrict__ gate) {
    CB_GATE
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i < n) x[i] = bs[i];
    if (i == 0) flag[0] = 1;
}

__global__ __launch_bounds__(256) void k_cb_panel(double* __restrict__ S, int n, int k0,
                                                  const double* __restrict__ Lsave, const int* __restrict__ row_first,
                                                  double* __restrict__ x, const int* __restrict__ gate) {
    CB_GATE
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
    // forward substitution: x_row -= L21[row] y_p (y_p = x[k0, k0 + 32), final since its diagonal
    // block; every row belongs to one wave)
    const double y0 = x[k0 + cc], y1 = x[k0 + 16 + cc];
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const int row = r0 + rq + 4 * q;
        const double part = row16_sum(fma(acc0[q], y0, acc1[q] * y1));
        if (row < n) {
            S[(size_t)row * n + k0 + cc] = acc0[q];
            S[(size_t)row * n + k0 + 16 + cc] = acc1[q];
            if (cc == 0) x[row] -= part;
        }
    }
}

// C -= L21_I L21_J^T on the 64x64 lower tile (ri, rj) of the trailing matrix
__device__ __forceinline__ void update_tile(double* __restrict__ S, int n, int k0, int ri, int rj, bool diag,
                                            double* __restrict__ Bt) {
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
        if (diag && u > wid) continue;   // strictly-upper 16x16 blocks of a diagonal tile
#pragma unroll
        for (int kk = 0; kk < 8; kk++) {
            const double bv = Bt[(16 * u + cc) * 34 + 4 * kk + rq];
            acc[u] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[kk], bv, acc[u], 0, 0, 0);
        }
    }
#pragma unroll
    for (int u = 0; u < 4; u++) {
        if (diag && u > wid) continue;
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const int row = ri + 16 * wid + rq + 4 * q, col = rj + 16 * u + cc;
            if (row < n && col < n) S[(size_t)row * n + col] = acc[u][q];
        }
    }
}

// lower 64x64 tile (I, J), I >= J, of the trailing matrix starting at t0; wave w owns rows
// 16w..16w+15 of the tile against all 64 columns (4 MFMA accumulators, K = 32)
__global__ __launch_bounds__(256) void k_cb_update(double* __restrict__ S, int n, int k0,
                                                   const int* __restrict__ row_first, double* __restrict__ Lsave,
                                                   double* __restrict__ x, int* __restrict__ flag,
                                                   const int* __restrict__ gate, const int* __restrict__ tiles) {
    CB_GATE
    __shared__ double Bt[kUT * 34];   // the J rows of the panel; then the next diagonal block's scratch
    const int t0 = k0 + kCT;
    const int tt = blockIdx.x;
    int I, J;
    if (tiles) {   // this panel's envelope tiles (host-built, tile (0, 0) first): I << 16 | J
        I = tiles[tt] >> 16;
        J = tiles[tt] & 0xFFFF;
    } else {       // every lower tile of the trailing matrix, triangular index
        I = (int)((sqrtf(8.0f * (float)tt + 1.0f) - 1.0f) * 0.5f);
        while ((I + 1) * (I + 2) / 2 <= tt) I++;
        while (I * (I + 1) / 2 > tt) I--;
        J = tt - I * (I + 1) / 2;
    }
    const int ri = t0 + kUT * I, rj = t0 + kUT * J;
    const int kt = k0 / kCT;
    // structure: the 64-row tile is non-zero in this panel if either 32-row half is
    const int fi = min(row_first[ri / kCT], ri + kCT < n ? row_first[ri / kCT + 1] : 1 << 30);
    const int fj = min(row_first[rj / kCT], rj + kCT < n ? row_first[rj / kCT + 1] : 1 << 30);
    const int wid = threadIdx.x >> 6;
    if (fi <= kt && fj <= kt) {   // workgroup-uniform: the tile is inside the envelope
        update_tile(S, n, k0, ri, rj, I == J, Bt);
    }
    // tile (0, 0) holds the next diagonal block, now final: factor it here (its own stores, so a
    // workgroup barrier is the only ordering needed)
    if (tt == 0 && t0 < n) {
        __syncthreads();
        if (wid == 0) cb_diag_forward(S, n, t0, Bt, Bt + 32 * 33, Lsave, x, flag);
    }
}

// Backward substitution L^T x = y (y: the forward result in x; the factor in the lower triangle of
// S, the panel inverses in Lsave); flag[0] == 0 (a non-positive pivot) -> x = 0. One 1024-thread
// workgroup, x in LDS (n <= kCbMaxN). Panel p: s = sum over the factor tiles R > p of its envelope
// (row_first[R] <= p) of L_Rp^T x_R, then x_p = L11^{-T} (y_p - s). Thread t owns element
// (t >> 5, t & 31) of every 32x32 tile; the next panel's tiles (up to kBackPre) and its L11^{-1}
// are loaded into registers before this panel's reductions, so the panel chain waits on LDS and
// barriers, not on HBM.
constexpr int kBackPre = 12;
__global__ __launch_bounds__(1024) void k_cb_back(const double* __restrict__ S, int n,
                                                  const double* __restrict__ Lsave, double* __restrict__ x,
                                                  const int* __restrict__ flag, const int* __restrict__ row_first,
                                                  const int* __restrict__ gate) {
    CB_GATE
    __shared__ double y[kCbMaxN];
    __shared__ double red[16 * 32];
    __shared__ double Lt[32 * 33];
    __shared__ double w[32];
    __shared__ unsigned char lst[128 * 128];   // factor tiles below panel p: lst[128 p + j]
    __shared__ int cnt[128];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    if (flag[0] == 0) {
        for (int i = tid; i < n; i += 1024) x[i] = 0.0;
        return;
    }
    const int np_ = (n + kCT - 1) / kCT;
    for (int i = tid; i < n; i += 1024) y[i] = x[i];
    if (tid < np_) {
        int m = 0;
        for (int R = tid + 1; R < np_; R++)
            if (row_first[R] <= tid) lst[128 * tid + m++] = (unsigned char)R;
        cnt[tid] = m;
    }
    __syncthreads();
    const int ti = tid >> 5, tc = tid & 31;
    double cur[kBackPre], nxt[kBackPre];
    double lcur, lnxt = 0.0;
    auto load = [&](int p, double (&buf)[kBackPre], double& l) {
        const int m = cnt[p], col = kCT * p + tc;
#pragma unroll
        for (int j = 0; j < kBackPre; j++) {
            double v = 0.0;
            if (j < m) {
                const int r = kCT * lst[128 * p + j] + ti;
                if (r < n && col < n) v = S[(size_t)r * n + col];
            }
            buf[j] = v;
        }
        l = Lsave[(size_t)p * 1024 + tid];
    };
    load(np_ - 1, cur, lcur);
    for (int p = np_ - 1; p >= 0; p--) {
        const int k0 = p * kCT, m = cnt[p];
        if (p > 0) load(p - 1, nxt, lnxt);
        double s = 0.0;
#pragma unroll
        for (int j = 0; j < kBackPre; j++)
            if (j < m) s = fma(cur[j], y[kCT * lst[128 * p + j] + ti], s);   // x of tiles R > p: final
        for (int j = kBackPre; j < m; j++) {                                 // wide envelopes only
            const int r = kCT * lst[128 * p + j] + ti;
            if (r < n && k0 + tc < n) s = fma(S[(size_t)r * n + k0 + tc], y[r], s);
        }
        Lt[ti * 33 + tc] = lcur;   // L11^{-1}[ti][tc]
        s += __shfl_xor(s, 32);    // rows 2w and 2w + 1 of the wave
        if (lane < 32) red[wid * 32 + lane] = s;
        __syncthreads();
        if (wid == 0) {
            if (lane < kCT) {
                double t = 0.0;
#pragma unroll
                for (int g = 0; g < 16; g++) t += red[g * 32 + lane];
                w[lane] = k0 + lane < n ? y[k0 + lane] - t : 0.0;
            }
            wave_lds_sync();
            if (lane < kCT && k0 + lane < n) {
                double xj = 0.0;
                for (int c = lane; c < kCT; c++) xj = fma(Lt[c * 33 + lane], w[c], xj);   // (L11^{-T} w)_j
                y[k0 + lane] = xj;
            }
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < kBackPre; j++) cur[j] = nxt[j];
        lcur = lnxt;
    }
    for (int i = tid; i < n; i += 1024) x[i] = y[i];
}

void chol_blocked_solve(double* S, int n, double* Lsave, const double* bs, double* x, int* flag,
                        const int* row_first, hipStream_t st, const int* gate, const int* tiles,
                        const int* tile_off) {
    hipLaunchKernelGGL(k_cb_init, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, bs, x, n, flag, gate);
    hipLaunchKernelGGL(k_cb_diag, dim3(1), dim3(64), 0, st, S, n, 0, Lsave, x, flag, gate);
    const int np_ = (n + kCT - 1) / kCT;
    for (int p = 0; p < np_; p++) {
        const int k0 = p * kCT, rest = n - (k0 + kCT);
        if (rest <= 0) break;
        hipLaunchKernelGGL(k_cb_panel, dim3((unsigned)((rest + 63) / 64)), dim3(256), 0, st, S, n, k0, Lsave,
                           row_first, x, gate);
        const int T = (rest + kUT - 1) / kUT;
        // + the diagonal block of panel p + 1 (tile (0, 0)'s work-group)
        if (tiles && tile_off)
            hipLaunchKernelGGL(k_cb_update, dim3((unsigned)(tile_off[p + 1] - tile_off[p])), dim3(256), 0, st, S, n,
                               k0, row_first, Lsave, x, flag, gate, tiles + tile_off[p]);
        else
            hipLaunchKernelGGL(k_cb_update, dim3((unsigned)(T * (T + 1) / 2)), dim3(256), 0, st, S, n, k0, row_first,
                               Lsave, x, flag, gate, nullptr);
    }
    hipLaunchKernelGGL(k_cb_back, dim3(1), dim3(1024), 0, st, S, n, Lsave, x, flag, row_first, gate);
}

// host: the 64x64 trailing-update tiles of every panel inside the envelope (the ones k_cb_update
// would not skip), tile (0, 0) first in each panel (its work-group factors the next diagonal
// block). tiles = I << 16 | J, offsets per panel (np + 1 entries, panels with no trailing matrix
// empty). At C5 (n = 2394, a loop with a 20-KF window) 865 of the 18278 lower tiles.
void cb_envelope_tiles(const int* row_first, int n, std::vector<int>& tiles, std::vector<int>& off) {
    const int np_ = (n + kCT - 1) / kCT;
    tiles.clear();
    off.assign(np_ + 1, 0);
    auto rf = [&](int r) { return row_first[r / kCT]; };
    for (int p = 0; p < np_; p++) {
        off[p] = (int)tiles.size();
        const int k0 = p * kCT, t0 = k0 + kCT, rest = n - t0;
        if (rest <= 0) continue;
        const int T = (rest + kUT - 1) / kUT;
        tiles.push_back(0);   // (0, 0)
        for (int I = 0; I < T; I++)
            for (int J = 0; J <= I; J++) {
                if (I == 0 && J == 0) continue;
                const int ri = t0 + kUT * I, rj = t0 + kUT * J;
                const int fi = std::min(rf(ri), ri + kCT < n ? rf(ri + kCT) : 1 << 30);
                const int fj = std::min(rf(rj), rj + kCT < n ? rf(rj + kCT) : 1 << 30);
                if (fi <= p && fj <= p) tiles.push_back((I << 16) | J);
            }
    }
    off[np_] = (int)tiles.size();
}

// test hook: solve A x = b (A dense SPD, n <= kCbMaxN) through the blocked path; ms = device time
int chol_blocked_test(const double* A, const double* b, double* x, int n, float* ms) {
    if (n <= 0 || n > kCbMaxN) return -1;
    const int nt = (n + kCT - 1) / kCT;
    std::vector<int> rf(nt);
    row_first_from_dense(A, n, rf.data());
    double *dS = nullptr, *db = nullptr, *dx = nullptr, *dL = nullptr;
    int *df = nullptr, *drf = nullptr, *dtl = nullptr;
    std::vector<int> tl, toff;
    cb_envelope_tiles(rf.data(), n, tl, toff);
    int rc = 0;
    auto ok = [&](hipError_t e) { if (e != hipSuccess && rc == 0) rc = -3; return e == hipSuccess; };
    ok(hipMalloc((void**)&dS, sizeof(double) * n * n));
    ok(hipMalloc((void**)&db, sizeof(double) * n));
    ok(hipMalloc((void**)&dx, sizeof(double) * n));
    ok(hipMalloc((void**)&dL, sizeof(double) * 1024 * nt));
    ok(hipMalloc((void**)&df, sizeof(int)));
    ok(hipMalloc((void**)&drf, sizeof(int) * nt));
    ok(hipMalloc((void**)&dtl, sizeof(int) * std::max<size_t>(1, tl.size())));
    if (rc == 0) {
        if (!tl.empty()) ok(hipMemcpy(dtl, tl.data(), sizeof(int) * tl.size(), hipMemcpyHostToDevice));
        ok(hipMemcpy(dS, A, sizeof(double) * n * n, hipMemcpyHostToDevice));
        ok(hipMemcpy(db, b, sizeof(double) * n, hipMemcpyHostToDevice));
        ok(hipMemcpy(drf, rf.data(), sizeof(int) * nt, hipMemcpyHostToDevice));
        hipEvent_t e0, e1;
        ok(hipEventCreate(&e0)); ok(hipEventCreate(&e1));
        ok(hipEventRecord(e0, nullptr));
        chol_blocked_solve(dS, n, dL, db, dx, df, drf, nullptr, nullptr, dtl, toff.data());
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
    (void)hipFree(dtl);
    return rc;
}

}  // namespace orbhip
