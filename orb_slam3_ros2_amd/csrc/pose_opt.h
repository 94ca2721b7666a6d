// Motion-only BA (Optimizer::PoseOptimization) on the device: one wavefront per frame.
#pragma once
#include <hip/hip_runtime.h>

#include "../../include/orbhip.h"

namespace orbhip {
struct PoseWorkspace;
PoseWorkspace* pose_ws_create();
void pose_ws_destroy(PoseWorkspace* w);
int pose_opt_batch(PoseWorkspace* ws, const orbhip_pose_problem* probs, int B, orbhip_pose_result* res,
                   hipStream_t st);
}  // namespace orbhip
