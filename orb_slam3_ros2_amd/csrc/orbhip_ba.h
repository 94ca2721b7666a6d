// Bundle-adjustment back-end (Optimizer::LocalBundleAdjustment / BundleAdjustment) host driver.
#pragma once
#include <hip/hip_runtime.h>

#include "../../include/orbhip.h"

namespace orbhip {
struct BaWorkspace;
BaWorkspace* ba_create();
void ba_destroy(BaWorkspace* ws);
int ba_solve(BaWorkspace* ws, const orbhip_ba_problem* prob, orbhip_ba_result* res, const volatile int* stop,
             hipStream_t st);
// shard_mode: kShardNone = B independent problems; kShardLocal = B shards of ONE problem in this
// process (device-side sum across the batch); kShardRccl = this rank's shard (B == 1), the
// sums are RCCL all-reduces over the communicator of ba_comm_init.
constexpr int kShardNone = 0, kShardLocal = 1, kShardRccl = 2;
// no_dag: never the persistent DAG Cholesky (the re-run after a DAG hand-off timeout); no_nd: no
// nested dissection of a lone problem (the re-run when its device setup refuses the plan)
int ba_solve_batch(BaWorkspace* ws, const orbhip_ba_problem* const* probs, int B, orbhip_ba_result* const* res,
                   const volatile int* stop, hipStream_t st, int shard_mode, bool no_dag = false,
                   bool no_nd = false);
// DAG hand-off timeouts this workspace saw, and the solves it re-ran on the other solvers
void ba_stats(BaWorkspace* ws, long long* timeouts, long long* reruns);
int ba_comm_init(BaWorkspace* ws, int nranks, int rank, const void* id);
int ba_comm_unique_id(void* id);
int ba_test_cholesky_reg(const double* A, const double* b, double* x, int n, int reps, float* ms,
                         unsigned long long* phases5);
int ba_test_cholesky(const double* A, const double* b, double* x, int n, unsigned long long* phases5, float* ms);
// host only: the problem preparation serial and on `threads` host threads; 0 when every list is
// identical (out4: blocks, pairs, Schur items, host ms of the threaded build), -1 otherwise
int ba_test_prepare(const orbhip_ba_problem* pr, int threads, double* out4);
}  // namespace orbhip
