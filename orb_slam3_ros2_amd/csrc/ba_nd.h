// Nested dissection of the reduced camera system (a20 / a22: the linear solve behind g2o's
// OptimizationAlgorithmLevenberg in GlobalBundleAdjustment).
//
// The optimised poses of a GBA are coupled only within the co-visibility window, so S is a (cyclic)
// block band of half-bandwidth w poses. The poses are cut into K segments; segment r = an interior
// I_r followed by a separator Z_r of w poses. Interiors never couple to each other: I_r touches only
// Z_{r-1} and Z_r. One solve is then
//   1. K partial factorizations in ONE k_chol_dag_multi launch: segment r's matrix is
//      [[S_II, S_IZ], [S_ZI, 0]] over (I_r, Z_{r-1}, Z_r), read from S through a permutation; its
//      interior tiles are factored and the separator block receives -W^T W (W = L_II^-1 S_IZ) and
//      the rhs -W^T y_I;
//   2. k_nd_assemble: the separator system S_Z = S[Z][Z] + the contributions (cyclic block
//      tridiagonal over Z_0 .. Z_{K-1});
//   3. the separator solve (k_chol_dag);
//   4. k_nd_backsolve: each interior L_II^T x_I = y_I - L_ZI^T x_Z, every x scattered to S's order.
// The arithmetic is a symmetric permutation of the same LL^T: equal to the full solve to rounding.
#pragma once
#include <hip/hip_runtime.h>

#include <vector>

namespace orbhip {

struct NdPlan {
    int np = 0;                 // optimised poses (S is 6 np square)
    int K = 0;                  // segments
    int w = 0;                  // separator width (poses) = the band's half-bandwidth
    bool cyclic = false;        // the band wraps around (a loop)
    std::vector<int> seg;       // K + 1 segment starts (poses), seg[K] = np
    int est_intervals = 0;      // modelled chain length (max interior tiles + separator tiles)
    int full_intervals = 0;     // the unpermuted solve's (tiles of S)
};
// A dissection of the pose graph (blocks (bi, bj), bi <= bj, over np optimised poses) into K
// segments (K = 0: the K of the smallest modelled chain). false when S is not a narrow (cyclic) band
// or the model does not pay (then the plain solve is used).
bool nd_plan(int np, const int* bi, const int* bj, int nblk, int K, NdPlan& p);
// the band of a set of pose blocks: wl = largest |j - i|, wc = largest cyclic distance (the plan of a
// sharded solve takes both maxima over every shard's blocks)
void nd_bandwidth(int np, const int* bi, const int* bj, int nblk, int& wl, int& wc);
// the segmentation for a given band and K: seg[r] = floor(r np / K), separators of w poses; false
// when an interior would be narrower than the band
bool nd_plan_band(int np, int wl, int wc, int K, NdPlan& p);
// whether every block lies inside segment r's matrix (its interior and the separators around it):
// a shard's landmarks must touch only those poses
bool nd_blocks_fit(const NdPlan& p, int r, const int* bi, const int* bj, int nblk);

struct NdWorkspace;
NdWorkspace* nd_create();
void nd_destroy(NdWorkspace* w);
// Device data of one problem's dissection (permutations, envelopes, DAG plans, buffers), uploaded on
// st; S (n x n, lower triangle), bs, x, flag: the problem's arrays (flag[0] = the solve succeeded).
// gate (optional): the LM phase word, every launch returns unless it is kPhTrial.
// seg_sel >= 0: a shard of a distributed solve: only segment seg_sel is factored
// here, S / bs hold the shard's partial system (its interior rows complete), and the separator
// system this shard assembles is its part of the sum (nd_sep_* below: the caller sums it over the
// shards between nd_factor_assemble and nd_separator_backsolve); the back-substitution writes this
// segment's interior and own separator into x_loc (n + 1 doubles: the rest zero, [n] = 1 when a
// factorization failed), which the caller sums over the shards into xg before nd_finish.
int nd_setup(NdWorkspace* w, const NdPlan& p, const int* bi, const int* bj, int nblk, const double* S,
             const double* bs, double* x, int* flag, const int* gate, hipStream_t st, int seg_sel = -1);
hipError_t nd_solve(NdWorkspace* w, hipStream_t st);   // the whole solve (seg_sel < 0)
hipError_t nd_factor_assemble(NdWorkspace* w, hipStream_t st);
hipError_t nd_separator_backsolve(NdWorkspace* w, hipStream_t st);
// the separator system's lower envelope packed (dir 0) into / unpacked (dir 1) from sep_pack
hipError_t nd_sep_pack(NdWorkspace* w, int dir, hipStream_t st);
struct NdSepBufs {
    double* pack; size_t pack_n;   // the packed envelope of S_Z
    double* bZ; int nZ;            // its right-hand side
    double* x_loc; double* xg;     // n + 1 each
    int n;
};
NdSepBufs nd_sep_bufs(NdWorkspace* w);
// x = xg[0, n), flag[0] = (xg[n] == 0) && the separator system factored (shards: after the x sum)
hipError_t nd_finish(NdWorkspace* w, hipStream_t st);
// the control words [3] (hand-off timeouts) of every DAG problem of the dissection (device pointers)
void nd_timeout_words(const NdWorkspace* w, std::vector<const int*>& out);

// test hook: A (6 np dense SPD, structure given by the pose blocks), b -> x; reps timed solves
int nd_test(const double* A, const double* b, double* x, int np, const int* bi, const int* bj, int nblk, int K,
            int reps, float* ms, int* K_used, float* stage_ms = nullptr, int* seg_out = nullptr);

}  // namespace orbhip
