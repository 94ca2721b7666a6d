// Persistent tiled-DAG Cholesky solve of the reduced camera system (ba_chol_dag.hip): ONE launch
// per solve, 32x32 tiles, a chain workgroup on the diagonal critical path and helper workgroups
// owning the off-diagonal tiles, in-launch hand-offs by flags (a20 / a22: g2o LinearSolverEigen
// behind OptimizationAlgorithmLevenberg).
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <vector>

namespace orbhip {

constexpr int kDagTile = 32;
constexpr int kDagMaxN = 4096;
constexpr int kDagMaxHelpers = 255;   // helper workgroups (+ the chain workgroup: one per CU)

// host plan of one problem: the helper tasks (tile (R, C) as R << 16 | C) of each helper
// workgroup, in the order the workgroup runs them (dependency key order, deadlock-free)
struct DagPlan {
    int NT = 0, G = 0;
    int nti = 0;              // partial solve: tiles [0, nti) factored, the trailing block update-only
    int pb = 0;               // backward substitution over the helpers (long rows) or in the chain
    std::vector<int> toff;    // G + 1 offsets into tasks
    std::vector<int> tasks;
};
void dag_plan(const int* row_first, int n, int max_helpers, DagPlan& p, int nti = 0);
int dag_max_helpers();   // min(kDagMaxHelpers, CUs - 1) of the current device: the whole grid resident
// a stream about to be destroyed: no later solve of another stream may record an event on it
void dag_stream_retired(hipStream_t st);
// solves launched on the current device, and how many of them first waited for another stream's
void dag_device_stats(long long* launches, long long* handoffs);
// polls before a hand-off wait gives up (ORBHIP_DAG_SPIN_MAX, default 2^19); a timeout counts in the
// problem's control word 3 (DagDev::ints[3]) and fails the solve (flag 0)
unsigned dag_spin_max();

// device storage of one problem: doubles (L tiles NT x NT, the two partial-tile rows, the
// diagonal inverses, y, the right-hand-side partials) and ints (4 control words + flags; zero
// before the first solve, never reset between solves: every solve counts its own epoch)
size_t dag_doubles(int n);
size_t dag_ints(int n);
// dag_doubles for NT tiles per side: L (NT x NT tiles), the three partial rows and the diagonal
// inverses (4 NT tiles), y / rhs partials / x / s (4 NT x 32), the column-major copies of L and
// of the inverses (NT x NT + NT tiles) that the chain's backward reads
__host__ __device__ inline size_t dag_doubles_nt(size_t NT) {
    return (NT * NT + 4 * NT) * kDagTile * kDagTile + NT * 4 * kDagTile + (NT * NT + NT) * kDagTile * kDagTile;
}

struct DagDev {
    double* buf;         // dag_doubles(n)
    int* ints;           // dag_ints(n), zeroed once; [3] counts hand-off timeouts
    const int* toff;     // plan, on the device
    const int* tasks;
    int G;
    int pb;              // DagPlan::pb
    int need_off;        // toff[G]: the chain backward's column counts follow the tasks there
};

// S (n x n row-major, lower triangle read, never written), row_first (ceil(n/32): first 32-col
// tile with a structural non-zero per 32-row tile), bs -> x; flag[0] = 1 ok, 0 on a non-positive
// pivot (x = 0). gate (optional): returns unless *gate == kPhTrial. dbg (optional, kDbgWords
// u64): the chain's shader-clock cycles: [0] prologue, [1] forward, [2] backward, [4] diag32 sum,
// [5] total, then per interval k < 200 six words at 8 + 6k: the interval, phase 1, phase 2, and in
// phase 3 wave 0 (diag32), wave 1 (publish + next diagonal partial), waves 2/3 (the next tiles).
// Then, for intervals k < kDbgSubK, 16 sub-phase stamps at kDbgSubOff + 16k (cycles from the
// interval start): wave 0 [0] diag part A done, [1] wave 1's D(1,*) in, [2] part B done; waves 2/3
// (h = 0, 1) [4 + 4h] their global loads in, [5 + 4h] L(k+2, k) row formed, [6 + 4h] T / D' updates
// done, [7 + 4h] rows of L(k+1, k) in.
constexpr int kDbgSubK = 100;
constexpr int kDbgSubOff = 8 + 6 * 200;
// then the backward steps R (chain-only form, R < kDbgBackR): [3R] wave 0 step start, [3R+1] wave 0
// x_{R-1} formed, [3R+2] wave 1 row R subtracted (cycles from the backward's start)
constexpr int kDbgBackR = 128;
constexpr int kDbgBackOff = kDbgSubOff + 16 * kDbgSubK;
constexpr int kDbgWords = kDbgBackOff + 3 * kDbgBackR;
hipError_t chol_dag_solve(const double* S, int n, const int* row_first, const double* bs, double* x, int* flag,
                          const DagDev& d, hipStream_t st, const int* gate = nullptr,
                          unsigned long long* dbg = nullptr);

// One problem of a multi-problem launch (the interiors of a nested dissection, ba_nd.hip): the
// solved matrix is S (row stride ld) through perm (row / column i = S's perm[i], -1 = padding:
// identity), n x n. nti > 0: partial solve (n > 32 nti): tiles [0, nti) are factored (L, Linv, y
// in d.buf as a full solve leaves them), and each trailing tile (R, C >= nti) inside the envelope
// receives -sum_{p < nti} L_Rp L_Cp^T (stored where its L tile would be, the trailing rows' rhs
// -sum L_Rp y_p at the rhs-partial slot R); flag[0] = the factored block's pivots were positive.
struct DagProb {
    const double* S;
    int ld;
    const int* perm;
    int n, nti;
    const int* rf;
    const double* bs;
    double* x;
    int* flag;
    DagDev d;
};
size_t dag_k_bytes();   // bytes of one problem's launch record
// fills np launch records (host_ks: np * dag_k_bytes()) and host_wgoff (np + 1): returns the grid
int dag_multi_fill(const DagProb* probs, int np, void* host_ks, int* host_wgoff, const int* gate, size_t* lds);
// the records / offsets uploaded to the device: one launch, every problem's chain and helpers
hipError_t chol_dag_multi_launch(const void* d_ks, const int* d_wgoff, int np, int grid, size_t lds, hipStream_t st);
// offsets (doubles) of a problem's DAG buffer: tile (R, C) of L (quadrant layout), the rhs partial of
// tile row R, y of tile row R
__host__ __device__ inline size_t dag_off_L(int NT, int R, int C) { return ((size_t)R * NT + C) * kDagTile * kDagTile; }
__host__ __device__ inline size_t dag_off_Linv(int NT, int k) { return ((size_t)NT * NT + 3 * (size_t)NT + k) * kDagTile * kDagTile; }
__host__ __device__ inline size_t dag_off_y(int NT, int k) { return ((size_t)NT * NT + 4 * (size_t)NT) * kDagTile * kDagTile + (size_t)k * kDagTile; }
__host__ __device__ inline size_t dag_off_R(int NT, int k) { return dag_off_y(NT, 0) + ((size_t)NT + k) * kDagTile; }

// test hook: A dense SPD (its structure -> row_first), reps timed solves; ms = device ms per solve;
// dbg as above (optional); returns 0, -4 on a failed pivot, -5 on a hand-off timeout
int chol_dag_test(const double* A, const double* b, double* x, int n, int reps, int max_helpers, float* ms,
                  unsigned long long* dbg);

}  // namespace orbhip
