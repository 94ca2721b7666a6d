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
}  // namespace orbhip
