// Multi-workgroup blocked Cholesky solve of the reduced camera system (ba_chol_blocked.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <vector>

namespace orbhip {

constexpr int kCbMaxN = 4096;   // largest n (6 x optimised keyframes) of the blocked solver

// S (n x n, row-major, lower triangle read; the factor is written in place: its 32x32 diagonal
// blocks in the lower triangle, its panels below them transposed into the upper triangle), Lsave (1024 x ceil(n/32)
// doubles), row_first (ceil(n/32) ints: first 32-column tile with a structural non-zero in each
// 32-row tile). flag[0] = 1 on success, 0 on a non-positive pivot (x = 0). Asynchronous on st.
// gate (device int, optional): every kernel returns unless *gate == kPhTrial (ba_args.h).
void chol_blocked_solve(double* S, int n, double* Lsave, const double* bs, double* x, int* flag,
                        const int* row_first, hipStream_t st, const int* gate = nullptr,
                        const int* tiles = nullptr, const int* tile_off = nullptr);
// tiles / tile_off (optional): the per-panel trailing-update tiles inside the envelope
// (cb_envelope_tiles; tiles on the device, tile_off on the host); nullptr = every lower tile,
// skipped in the kernel when outside the envelope.
void cb_envelope_tiles(const int* row_first, int n, std::vector<int>& tiles, std::vector<int>& off);

int chol_blocked_test(const double* A, const double* b, double* x, int n, float* ms);

// host: row_first of a dense symmetric matrix from its lower triangle (test hook helper)
inline void row_first_from_dense(const double* A, int n, int* rf) {
    const int nt = (n + 31) / 32;
    for (int R = 0; R < nt; R++) {
        int f = R;
        for (int r = 32 * R; r < 32 * R + 32 && r < n; r++)
            for (int c = 0; c < 32 * f && c <= r; c++)
                if (A[(size_t)r * n + c] != 0.0) { f = std::min(f, c / 32); break; }
        rf[R] = f;
    }
}

}  // namespace orbhip
