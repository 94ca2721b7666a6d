// Per-problem argument record of the batched bundle-adjustment kernels (ba_solver.hip) and the
// register-resident Cholesky (ba_chol_reg.hip). Device pointers into the packed workspace.
#pragma once

namespace orbhip {

// Per-problem Levenberg-Marquardt state of the device-driven solve (k_ba_ctl_*): the exact g2o
// OptimizationAlgorithmLevenberg control flow, advanced one trial per slot on the device.
enum : int { kPhBuild = 0, kPhTrial = 1, kPhDone = 2 };
struct LmCtl {
    double ni, currentChi, rho, initChi;
    int phase, it, trials, qmax;
    int nBad, errors_valid, pop, stop;
    int iterations, early_stop;
    int arrive_b, arrive_t;   // last-arriver counters of k_ba_lin (build) and k_ba_errors(2) (trial), 0 between launches
};

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
    double* e_lin;     // E*4: linearisation per edge: camera-frame point (x y z), robust weight w
    double* R_lin;     // np*9: rotation of each optimised pose at the linearisation (row-major)
    double* b;         // n + 3M
    double* Dinv;      // M*9
    double* db;        // M*3
    double* S;         // n*n
    double* bs;        // n
    double* x;         // n + 3M
    const int* pt_ptr; const int* pt_edges;     // CSR point -> edges (all edges)
    const int* ps_ptr; const int* ps_edges;     // CSR optimised pose -> edges
    const int* blk_i; const int* blk_j; const int* blk_ptr; const int* blk_pairs;  // Schur pair lists
    int nblk;
    double* red;       // [0] chi2, [1] scale, [2] maxdiag
    int* flag;         // [0] cholesky ok
    const double* lambda;   // current lambda of this problem (device copy)
    double* Lsave;     // ceil(n/32) x 1024: L11^{-1} of every Cholesky panel
    const int* row_first;   // ceil(n/32): envelope of S in 32x32 tiles (blocked solver)
    const int* cb_tiles;    // blocked solver: each panel's trailing-update tiles inside the envelope
    int lead;          // sharded solve: this shard adds lambda x_p^2 to the scale (once), and the
                       // pose-side Hpp + lambda terms to S when `own` is null
    const unsigned char* own;   // sharded solve by segments: 1 for the poses whose pose-side terms this shard adds
    const double* Hpp_g;        // the pose Hessians summed over the shards (== Hpp unsharded)
    int small;         // unsharded, small enough for the trial's last workgroup to restore a rejected state
                       // and refresh its stale errors itself (no k_ba_pop / k_ba_errors(1) launch per slot)
    int fused;         // small and unsharded: the back-substitution computes the trial's errors too
                       // (k_ba_backsub_errs): the trial's poses go to pose_bak until the controller commits
    int sync;          // sharded device-driven rounds: the controller's reductions and decisions run as their
                       // own launches (a collective between them), not in the last workgroup of k_ba_lin /
                       // k_ba_errors(2)
    // Schur work items (k_ba_schur_items): {k0, k1, blk, slot} over blk_pairs; slot -1 = the
    // block's only item (written to S directly), else the block's chunk `slot` (the chunks of a
    // block sit in one work-group of 128 items and are summed there, + Hpp + lambda on the
    // diagonal; blk -1 = padding). fin: {blk, first slot, count} per such block; ifin: each item's
    // fin entry (-1: none)
    const int* items; int nitems;
    const int* fin; int nfin;
    const int* ifin;
    LmCtl* ctl;        // device-driven solve: this problem's LM state (nullptr: host-driven rounds)
    double* part;      // workgroup partial sums of a trial: chi2 (npart_e = ceil(E / 256)), then the
    int npart_e, npart_m;   // landmark scale terms (npart_m = ceil(M / 256)); in the build phase
                            // k_ba_lin's per-workgroup max diagonal (ceil(M / 256) + ceil(np / 4))
};

}  // namespace orbhip
