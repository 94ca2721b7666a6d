// Projection-guided matching on the device (proj_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>

#include "../../include/orbhip.h"

namespace orbhip {
struct ProjWorkspace;
ProjWorkspace* proj_ws_create();
void proj_ws_destroy(ProjWorkspace* w);
int proj_search_last(ProjWorkspace* ws, const orbhip_frame* F, const orbhip_proj_last* L, float th,
                     int check_orientation, int32_t* match, int* rounds_out, hipStream_t st);
int proj_search_local(ProjWorkspace* ws, const orbhip_frame* F, const orbhip_local_points* M, float view_cos_limit,
                      float th, float nnratio, int far_points, float th_far, uint8_t* in_view, int32_t* level,
                      int32_t* match, int* rounds_out, hipStream_t st);
int init_search(ProjWorkspace* ws, const orbhip_init_frame* F1, const orbhip_init_frame* F2, float* prev_matched,
                int window_size, float nnratio, int check_orientation, int32_t* matches12, hipStream_t st);
// Staged host inputs (pinned block h, its device alias hd) to device memory d by a shader copy
// (small blocks: no DMA-engine start-up); ORBHIP_PROJ_DMA=1 uses hipMemcpyAsync.
hipError_t upload_inputs(const void* hd, void* d, const void* h, size_t bytes, hipStream_t st);
}  // namespace orbhip
