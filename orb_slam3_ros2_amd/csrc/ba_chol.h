// Device pieces of the dense Cholesky shared by the single-workgroup solver (ba_solver.hip,
// k_ba_cholesky) and the multi-workgroup blocked solver (ba_chol_blocked.hip).
#pragma once
#include <hip/hip_runtime.h>

namespace orbhip {

typedef double double4_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ double readlane_f64(double v, int lane) {
    const unsigned long long u = __builtin_bit_cast(unsigned long long, v);
    const unsigned lo = __builtin_amdgcn_readlane((unsigned)u, lane);
    const unsigned hi = __builtin_amdgcn_readlane((unsigned)(u >> 32), lane);
    return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}

// (a) of chol_solve: factor the 32x32 diagonal block at (k0, k0) with one wavefront.
__device__ __forceinline__ void chol_diag_wave(double* __restrict__ S, int n, int k0, int kb, double* __restrict__ Li,
                                            double* __restrict__ Lsave, int* bad) {
    const int lane = threadIdx.x & 63;
    const int c = lane & 31, h = lane >> 5;
    double d[16], xi[16];
#pragma unroll
    for (int k = 0; k < 16; k++) {
        const int r = 2 * k + h;
        double v = (r == c) ? 1.0 : 0.0;
        if (r < kb && c < kb)
            v = r >= c ? S[(size_t)(k0 + r) * n + k0 + c] : S[(size_t)(k0 + c) * n + k0 + r];
        d[k] = v;
        xi[k] = (r == c) ? 1.0 : 0.0;
    }
    double myip = 1.0;
    bool nonpd = false;
#pragma unroll
    for (int j = 0; j < 32; j++) {
        const int jr = j >> 1, jh = 32 * (j & 1);
        // all cross-lane operands of this step first (one LDS wait), then the FMAs
        double colj[16];
#pragma unroll
        for (int k = 0; k < 16; k++)
            if (2 * k + 1 > j) colj[k] = __shfl(d[k], j + 32 * h, 64);   // D[r][j], r = 2k+h
        const double rowj = __shfl(d[jr], c + jh, 64);                   // D[j][c]
        const double xrow = __shfl(xi[jr], c + jh, 64);                  // X[j][c]
        const double piv = readlane_f64(d[jr], j + jh);                  // uniform
        nonpd |= !(piv > 0.0);
        const double ip = 1.0 / (piv > 0.0 ? piv : 1.0);
        if (c == j) myip = ip;
        const double rs = c > j ? rowj * ip : 0.0;      // trailing columns: D[r][c] -= D[r][j] D[j][c] / piv
        const double xs = c > j ? 0.0 : xrow * ip;      // eliminated columns: X[r][c] -= D[r][j] X[j][c] / piv
#pragma unroll
        for (int k = 0; k < 16; k++) {
            if (2 * k + 1 <= j) continue;                  // rows r <= j untouched
            const double m = (2 * k == j && h == 0) ? 0.0 : colj[k];   // row r == j itself
            d[k] = fma(-m, rs, d[k]);
            xi[k] = fma(-m, xs, xi[k]);
        }
    }
    const double dv = sqrt(1.0 / myip), idv = 1.0 / dv;
#pragma unroll
    for (int k = 0; k < 16; k++) {
        const int r = 2 * k + h;
        const double idr = __shfl(idv, r, 64);
        if (r < kb && c < kb && c <= r) S[(size_t)(k0 + r) * n + k0 + c] = r == c ? dv : d[k] * idv;
        const double li = (r < kb && c < kb) ? xi[k] * idr : 0.0;
        Li[r * 33 + c] = li;
        if (Lsave) Lsave[(size_t)(k0 / 32) * 1024 + r * 32 + c] = li;
    }
    if (lane == 0 && nonpd) *bad = 1;
}

}  // namespace orbhip
