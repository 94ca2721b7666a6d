// KeyFrameDatabase place-recognition queries on the device (kfdb_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>

#include "../../include/orbhip.h"

namespace orbhip {
struct KfDb;
KfDb* kfdb_create(int max_kf, hipStream_t st, int* rc);
void kfdb_destroy(KfDb* d);
int kfdb_add(KfDb* d, int kf, const int32_t* words, const double* values, int n);
int kfdb_erase(KfDb* d, int kf);
int kfdb_detect_relocalization(KfDb* d, const orbhip_kfdb_query* q, int32_t* out, int cap);
int kfdb_detect_nbest(KfDb* d, const orbhip_kfdb_query* q, const uint8_t* connected, int ncand, int32_t* loop_out,
                      int32_t* n_loop, int32_t* merge_out, int32_t* n_merge);
}  // namespace orbhip
