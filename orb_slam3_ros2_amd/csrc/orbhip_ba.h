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
int ba_solve_batch(BaWorkspace* ws, const orbhip_ba_problem* const* probs, int B, orbhip_ba_result* const* res,
                   const volatile int* stop, hipStream_t st);
int ba_test_cholesky(const double* A, const double* b, double* x, int n, unsigned long long* phases5, float* ms);
}  // namespace orbhip
