// Multi-workgroup dense Cholesky + solve of the reduced camera system S xp = bs for large
// problems (GlobalBundleAdjustment / BundleAdjustment, SURVEY.md §8 a20/a22: n = 6 * #optimised
// KFs, up to 4096), right-looking with 32-column panels, ONE launch per panel:
//   k_cb_diag    one wavefront factors the first 32x32 diagonal block in registers
//                (chol_diag_wave): L11 into S, L11^{-1} into Lsave (the backward solve reuses it),
//                and applies y_p = L11^{-1} x_p (the forward substitution rides on the
//                factorization: x holds bs)
//   k_cb_update  per 64x64 lower tile (I, J) of the trailing matrix: the work-group computes the
//                panel rows it needs, L21_I = A21_I L11^{-T} and L21_J (v_mfma_f64_16x16x4f64,
//                from the raw panel column and Lsave), then C -= L21_I L21_J^T (MFMA). The
//                work-group of each diagonal tile (I, I) also stores L21_I, transposed, into
//                S's upper triangle (rows of the panel, columns below it: nothing reads that
//                region during the factorization, while the panel column itself is still read
//                by the other work-groups) and applies x_r -= L21[r] y_p to its rows. The
//                work-group of tile (0, 0) then factors the next diagonal block.
//   k_cb_back_last / k_cb_back_step  backward substitution by super-blocks of 8 panels: the
//                tiles left of each diagonal super-block applied by one workgroup per panel, the
//                diagonal super-block solved by the last of them (details at cb_back_block)
// Structure: row_first[R] = first 32-column tile with a structural non-zero in 32-row tile R of
// S. The envelope (profile) of a symmetric matrix is preserved by its Cholesky factor, so every
// tile left of row_first stays zero: the update and solve kernels skip it. A banded or
// arrow-shaped S (a loop of keyframes with a co-visibility window) costs O(n b^2), not O(n^3).
// The lower triangle of S is the input; the factor ends as L11 blocks on the diagonal (lower)
// and L21 panels transposed in the upper triangle.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <vector>

#include "ba_chol.h"
#include "ba_args.h"
#include "ba_chol_blocked.h"
#include "ba_diag16.h"
#include "wave_f64.h"

namespace orbhip {

constexpr int kCT = 32;    // panel width / structure tile
constexpr int kUT = 64;    // trailing-update tile

// factor the diagonal block at k0 (one wave, diag32_linv: two 16x16 tiles with 4x4 pivot blocks on
// MFMA) and apply the forward step y_p = L11^{-1} x_p in place; Li: 32 x 33 doubles of LDS, xs: 32,
// then 512 doubles of factorization scratch. Only L11^{-1} is kept (Lsave + Li): every later use
// of the diagonal block (the panel rows, both triangular solves) needs the inverse, not L11.
__device__ __forceinline__ void cb_diag_forward(double* __restrict__ S, int n, int k0, double* __restrict__ Li,
                                                double* __restrict__ xs, double* __restrict__ Lsave,
                                                double* __restrict__ x, int* __restrict__ flag) {
    const int lane = threadIdx.x & 63, kb = min(kCT, n - k0);
    double* Ls = Lsave + (size_t)(k0 / kCT) * 1024;
    const bool ok = diag32_linv(
        [&](int r, int c) {   // r >= c; identity outside the matrix
            return (r < kb && c < kb) ? S[(size_t)(k0 + r) * n + k0 + c] : (r == c ? 1.0 : 0.0);
        },
        xs + kCT,
        [&](int r, int c, double v) {
            Li[r * 33 + c] = v;
            Ls[r * 32 + c] = v;
        });
    if (lane < kCT) xs[lane] = lane < kb ? x[k0 + lane] : 0.0;
    wave_lds_sync();
    if (lane < kb) {
        double s = 0.0;
        for (int c = 0; c <= lane; c++) s += Li[lane * 33 + c] * xs[c];
        x[k0 + lane] = s;
    }
    if (lane == 0 && !ok) flag[0] = 0;
}

// gate: the device-driven LM rounds (ba_solver.hip) run a problem's solve only in its trial phase
// (the phase word of its LmCtl); nullptr = always
#define CB_GATE \
    if (gate && *gate != kPhTrial) return;

__global__ __launch_bounds__(64) void k_cb_diag(double* __restrict__ S, int n, int k0, double* __restrict__ Lsave,
                                                double* __restrict__ x, int* __restrict__ flag, const int* __restrict__ gate) {
    CB_GATE
    __shared__ double Li[32 * 33 + 32 + 512];
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

// L21 rows [r0, r0 + 64) of the panel at k0 into LDS Lt (64 x 34): L21 = A21 Li^T, Li = L11^{-1}
// (LDS, 32 x 33), A21 the panel column of S (final: every earlier panel's update is done). Wave w
// computes rows 16w..16w+15 on MFMA (lane (cc, rq): A row cc, k = 4kk + rq; C rows rq + 4q).
// Split in a load (av: issued with the tile's other loads) and the MFMA part.
__device__ __forceinline__ void panel_rows_load(const double* __restrict__ S, int n, int k0, int r0, double* av) {
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63, cc = lane & 15, rq = lane >> 4;
    const int rb = r0 + 16 * wid;
    const bool rin = rb + cc < n;
#pragma unroll
    for (int kk = 0; kk < 8; kk++) av[kk] = rin ? S[(size_t)(rb + cc) * n + k0 + 4 * kk + rq] : 0.0;
}
__device__ __forceinline__ void panel_rows_mfma(const double* av, const double* __restrict__ Li,
                                                double* __restrict__ Lt) {
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63, cc = lane & 15, rq = lane >> 4;
    double4_t acc0 = {0, 0, 0, 0}, acc1 = {0, 0, 0, 0};
#pragma unroll
    for (int kk = 0; kk < 8; kk++) {
        acc0 = __builtin_amdgcn_mfma_f64_16x16x4f64(av[kk], Li[cc * 33 + 4 * kk + rq], acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f64_16x16x4f64(av[kk], Li[(16 + cc) * 33 + 4 * kk + rq], acc1, 0, 0, 0);
    }
#pragma unroll
    for (int q = 0; q < 4; q++) {
        Lt[(16 * wid + rq + 4 * q) * 34 + cc] = acc0[q];
        Lt[(16 * wid + rq + 4 * q) * 34 + 16 + cc] = acc1[q];
    }
}

// the 64x64 lower tile (ri, rj) of the trailing matrix: wave w holds rows 16w..16w+15 against all
// 64 columns (4 MFMA accumulators in C layout)
__device__ __forceinline__ void tile_load(const double* __restrict__ S, int n, int ri, int rj, double4_t* acc) {
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int cc = lane & 15, rq = lane >> 4;
#pragma unroll
    for (int u = 0; u < 4; u++) {
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const int row = ri + 16 * wid + rq + 4 * q, col = rj + 16 * u + cc;
            acc[u][q] = (row < n && col < n) ? S[(size_t)row * n + col] : 0.0;
        }
    }
}

// C -= L21_I L21_J^T on the loaded tile; LI / LJ: the panel rows of both (LDS, 64 x 34)
__device__ __forceinline__ void update_tile(double* __restrict__ S, int n, int ri, int rj, bool diag, double4_t* acc,
                                            const double* __restrict__ LI, const double* __restrict__ LJ) {
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int cc = lane & 15, rq = lane >> 4;
    double av[8];
#pragma unroll
    for (int kk = 0; kk < 8; kk++) av[kk] = -LI[(16 * wid + cc) * 34 + 4 * kk + rq];
#pragma unroll
    for (int u = 0; u < 4; u++) {
        if (diag && u > wid) continue;   // strictly-upper 16x16 blocks of a diagonal tile
#pragma unroll
        for (int kk = 0; kk < 8; kk++) {
            const double bv = LJ[(16 * u + cc) * 34 + 4 * kk + rq];
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

// lower 64x64 tile (I, J), I >= J, of the trailing matrix starting at t0
__global__ __launch_bounds__(256) void k_cb_update(double* __restrict__ S, int n, int k0,
                                                   const int* __restrict__ row_first, double* __restrict__ Lsave,
                                                   double* __restrict__ x, int* __restrict__ flag,
                                                   const int* __restrict__ gate, const int* __restrict__ tiles) {
    CB_GATE
    __shared__ double Li[32 * 33];          // L11^{-1} of the panel
    __shared__ double LI[kUT * 34], LJ[kUT * 34];   // panel rows of tiles I and J; LI then the next
                                                    // diagonal block's scratch
    const int t0 = k0 + kCT;
    const int tt = blockIdx.x, tid = threadIdx.x;
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
    const int wid = tid >> 6;
    if (fi <= kt && fj <= kt) {   // workgroup-uniform: the tile is inside the envelope
        // every global load of the tile in one round trip: L11^{-1}, both panel row blocks, C
        const double* Lp = Lsave + (size_t)kt * 1024;
        double lv[4];
#pragma unroll
        for (int u = 0; u < 4; u++) lv[u] = Lp[tid + 256 * u];
        double avI[8], avJ[8];
        panel_rows_load(S, n, k0, ri, avI);
        if (I != J) panel_rows_load(S, n, k0, rj, avJ);
        double4_t acc[4];
        tile_load(S, n, ri, rj, acc);
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int t = tid + 256 * u;
            Li[(t >> 5) * 33 + (t & 31)] = lv[u];
        }
        __syncthreads();
        panel_rows_mfma(avI, Li, LI);
        if (I != J) panel_rows_mfma(avJ, Li, LJ);
        __syncthreads();
        update_tile(S, n, ri, rj, I == J, acc, LI, I == J ? LI : LJ);
        if (I == J) {
            // the factor's panel rows, transposed into the upper triangle (rows k0.., columns ri..)
            for (int i = tid; i < kUT * kCT; i += 256) {
                const int r = i & 63, c = i >> 6;
                if (ri + r < n) S[(size_t)(k0 + c) * n + ri + r] = LI[r * 34 + c];
            }
            // forward substitution: x_r -= L21[r] y_p (y_p = x[k0, k0 + 32), final)
            if (tid < kUT && ri + tid < n) {
                double s = 0.0;
#pragma unroll 8
                for (int c = 0; c < kCT; c++) s = fma(LI[tid * 34 + c], x[k0 + c], s);
                x[ri + tid] -= s;
            }
        }
    }
    // tile (0, 0) holds the next diagonal block, now final: factor it here (its own stores, so a
    // workgroup barrier is the only ordering needed)
    if (tt == 0 && t0 < n) {
        __syncthreads();
        if (wid == 0) cb_diag_forward(S, n, t0, LI, LI + 32 * 33, Lsave, x, flag);
    }
}

// Backward substitution L^T x = y (y: the forward result in x; the factor's panels transposed in
// the upper triangle of S, the panel inverses in Lsave) in SUPER-BLOCKS of kSB panels (256 rows),
// last to first. For super-block b:
//   diagonal solve  x_p = L11^{-T} (y_p - sum over R > p inside b of L_Rp^T x_R), p descending
//                   (one 1024-thread workgroup, y of the super-block in LDS);
//   step            y_i -= sum over R in b of L_Ri^T x_R for every panel i left of b (one
//                   workgroup per panel, envelope tiles only), then the LAST workgroup to finish
//                   runs the diagonal solve of super-block b - 1.
// So the chain is ceil(np / 8) launches, the tiles left of the diagonal blocks are read by many
// workgroups at once, and no workgroup ever waits for another: the step workgroups publish their
// y_i with sc1 (write-through) stores, drain them (vmcnt(0)), and count themselves in flag[1] by
// an agent-scope atomic; the workgroup whose add comes last reads the super-block's y back with
// sc1 loads (MI355X_MICROARCH.md, inter-workgroup visibility, the table's first row). flag[0] == 0
// (a non-positive pivot) -> x = 0.
constexpr int kSB = 8;        // panels per super-block
constexpr int kBackPre = kSB - 1;
// workgroup barrier ordering LDS only: __syncthreads() is a workgroup fence, which on gfx950 also
// drains vmcnt, i.e. would wait for the next panel's prefetch loads at every panel
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}
__device__ __forceinline__ void wait_vm_all() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// diagonal solve of super-block sb (panels [p0, p1)), 1024 threads; sc1: read y with sc1 loads
// (it was published by other workgroups of this launch)
__device__ __forceinline__ void cb_back_block(const double* __restrict__ S, int n, const double* __restrict__ Lsave,
                                              double* __restrict__ x, const int* __restrict__ row_first, int sb,
                                              bool sc1) {
    __shared__ double y[kSB * kCT];
    __shared__ double red[32];
    __shared__ double Lt[32 * 33];
    __shared__ double w[32];
    __shared__ unsigned char lst[kSB * kSB];   // factor tiles below panel p inside the super-block
    __shared__ int cnt[kSB];
    const int np_ = (n + kCT - 1) / kCT;
    const int p0 = sb * kSB, p1 = min(np_, p0 + kSB), r0 = p0 * kCT;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    if (tid < kSB * kCT)   // rows past n (or past the super-block) read as 0: their tiles are 0
        y[tid] = (tid < (p1 - p0) * kCT && r0 + tid < n)
                     ? (sc1 ? __hip_atomic_load(&x[r0 + tid], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : x[r0 + tid])
                     : 0.0;
    if (tid < p1 - p0) {
        const int p = p0 + tid;
        int m = 0;
        for (int R = p + 1; R < p1; R++)
            if (row_first[R] <= p) lst[kSB * tid + m++] = (unsigned char)(R - p0);
        cnt[tid] = m;
    }
    __syncthreads();
    const int ti = tid & 31, tc = tid >> 5;   // row and column inside a 32x32 tile
    auto load = [&](int p, double (&buf)[kBackPre], double& l) {
        const int m = cnt[p - p0], col = kCT * p + tc;
#pragma unroll
        for (int j = 0; j < kBackPre; j++) {
            double v = 0.0;
            if (j < m) {
                const int r = r0 + kCT * lst[kSB * (p - p0) + j] + ti;
                if (r < n && col < n) v = S[(size_t)col * n + r];   // L[r][col], transposed
            }
            buf[j] = v;
        }
        l = Lsave[(size_t)p * 1024 + tid];
    };
    auto panel = [&](int p, const double (&cur)[kBackPre], double lcur, double (&nxt)[kBackPre], double& lnxt) {
        const int k0 = p * kCT, m = cnt[p - p0];
        Lt[(tid >> 5) * 33 + (tid & 31)] = lcur;   // L11^{-1} (Lsave is row-major 32 x 32)
        double s = 0.0;
#pragma unroll
        for (int j = 0; j < kBackPre; j++)
            if (j < m) s = fma(cur[j], y[kCT * lst[kSB * (p - p0) + j] + ti], s);   // x of tiles R > p: final
        if (p > p0) load(p - 1, nxt, lnxt);   // in flight through the reductions and barriers below
#pragma unroll
        for (int o = 16; o > 0; o >>= 1) s += __shfl_xor(s, o);
        if ((lane & 31) == 0) red[tc] = s;
        lds_barrier();
        if (wid == 0) {
            if (lane < kCT) w[lane] = k0 + lane < n ? y[k0 - r0 + lane] - red[lane] : 0.0;
            wave_lds_sync();
            if (lane < kCT && k0 + lane < n) {
                double xj = 0.0;
                for (int c = lane; c < kCT; c++) xj = fma(Lt[c * 33 + lane], w[c], xj);   // (L11^{-T} w)_j
                y[k0 - r0 + lane] = xj;
            }
        }
        lds_barrier();
    };
    double bufA[kBackPre], bufB[kBackPre], lA = 0.0, lB = 0.0;
    load(p1 - 1, bufA, lA);
    for (int p = p1 - 1; p >= p0; p -= 2) {
        panel(p, bufA, lA, bufB, lB);
        if (p - 1 >= p0) panel(p - 1, bufB, lB, bufA, lA);
    }
    if (tid < (p1 - p0) * kCT && r0 + tid < n) x[r0 + tid] = y[tid];
}

// the last super-block's diagonal solve (or x = 0 after a non-positive pivot)
__global__ __launch_bounds__(1024) void k_cb_back_last(const double* __restrict__ S, int n,
                                                       const double* __restrict__ Lsave, double* __restrict__ x,
                                                       const int* __restrict__ flag, const int* __restrict__ row_first,
                                                       const int* __restrict__ gate) {
    CB_GATE
    if (flag[0] == 0) {
        for (int i = threadIdx.x; i < n; i += 1024) x[i] = 0.0;
        return;
    }
    const int np_ = (n + kCT - 1) / kCT;
    cb_back_block(S, n, Lsave, x, row_first, (np_ - 1) / kSB, false);
}

// step of super-block sb: workgroup = panel i (panels[blockIdx.x], or blockIdx.x without a list)
__global__ __launch_bounds__(1024) void k_cb_back_step(const double* __restrict__ S, int n,
                                                       const double* __restrict__ Lsave, double* __restrict__ x,
                                                       int* __restrict__ flag, const int* __restrict__ row_first,
                                                       const int* __restrict__ gate, int sb,
                                                       const int* __restrict__ panels) {
    CB_GATE
    if (flag[0] == 0) return;   // x = 0 already
    __shared__ int last;
    const int np_ = (n + kCT - 1) / kCT;
    const int i = panels ? panels[blockIdx.x] : blockIdx.x;
    const int tid = threadIdx.x, ti = tid & 31, tc = tid >> 5, col = kCT * i + tc;
    const int R0 = sb * kSB, R1 = min(np_, R0 + kSB);
    double s = 0.0;
    for (int R = R0; R < R1; R++) {
        if (row_first[R] > i) continue;   // uniform
        const int r = kCT * R + ti;
        if (r < n && col < n) s = fma(S[(size_t)col * n + r], x[r], s);   // L[r][col] x_R[r]
    }
#pragma unroll
    for (int o = 16; o > 0; o >>= 1) s += __shfl_xor(s, o);
    if (ti == 0 && col < n)
        __hip_atomic_store(&x[col], x[col] - s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // sc1
    wait_vm_all();
    __syncthreads();
    if (tid == 0) last = atomicAdd(&flag[1], 1) == (int)gridDim.x - 1;
    __syncthreads();
    if (!last) return;
    if (tid == 0) (void)atomicExch(&flag[1], 0);
    cb_back_block(S, n, Lsave, x, row_first, sb - 1, true);
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
        const int T = (rest + kUT - 1) / kUT;
        // + the diagonal block of panel p + 1 (tile (0, 0)'s work-group)
        if (tiles && tile_off)
            hipLaunchKernelGGL(k_cb_update, dim3((unsigned)(tile_off[p + 1] - tile_off[p])), dim3(256), 0, st, S, n,
                               k0, row_first, Lsave, x, flag, gate, tiles + tile_off[p]);
        else
            hipLaunchKernelGGL(k_cb_update, dim3((unsigned)(T * (T + 1) / 2)), dim3(256), 0, st, S, n, k0, row_first,
                               Lsave, x, flag, gate, nullptr);
    }
    hipLaunchKernelGGL(k_cb_back_last, dim3(1), dim3(1024), 0, st, S, n, Lsave, x, flag, row_first, gate);
    const int nsb = (np_ + kSB - 1) / kSB;
    for (int sb = nsb - 1; sb >= 1; sb--) {
        if (tiles && tile_off) {   // this super-block's step panels (cb_envelope_tiles)
            const int o0 = tile_off[np_ + (nsb - 1 - sb)], o1 = tile_off[np_ + 1 + (nsb - 1 - sb)];
            hipLaunchKernelGGL(k_cb_back_step, dim3((unsigned)(o1 - o0)), dim3(1024), 0, st, S, n, Lsave, x, flag,
                               row_first, gate, sb, tiles + o0);
        } else {
            hipLaunchKernelGGL(k_cb_back_step, dim3((unsigned)(sb * kSB)), dim3(1024), 0, st, S, n, Lsave, x, flag,
                               row_first, gate, sb, nullptr);
        }
    }
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
    // backward steps, super-block sb = nsb-1 .. 1: the panels i < kSB sb with an envelope tile in
    // the super-block, and every panel of super-block sb - 1 (their last workgroup solves it)
    const int nsb = (np_ + kSB - 1) / kSB;
    off.resize(np_ + nsb);
    for (int sb = nsb - 1; sb >= 1; sb--) {
        const int R0 = sb * kSB, R1 = std::min(np_, R0 + kSB);
        for (int i = 0; i < R0; i++) {
            bool any = i >= R0 - kSB;
            for (int R = R0; R < R1 && !any; R++) any = row_first[R] <= i;
            if (any) tiles.push_back(i);
        }
        off[np_ + 1 + (nsb - 1 - sb)] = (int)tiles.size();
    }
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
    ok(hipMalloc((void**)&df, 4 * sizeof(int)));
    ok(hipMemset(df, 0, 4 * sizeof(int)));
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
