// Register-resident single-workgroup Cholesky solve (ba_chol_reg.hip) for the reduced camera
// system of the batched LM solver, n <= kCholRegMaxN.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>

namespace orbhip {
struct BaArgs;
constexpr int kCholRegMaxN = 304;   // 19 tiles of 16: 171 off-diagonal tiles, 22 per wave
size_t chol_reg_lds_bytes(int n);
int chol_reg_maxt(int n);   // tile slots per wave for n (0 = too large)
// one workgroup per problem args[act[b]], b < nprob; maxN = the largest n among them
hipError_t chol_reg_launch(int maxN, int nprob, const BaArgs* args, const int* act, hipStream_t st);
// diagnostics: one problem (args on the device), per-phase shader-clock cycles into dbg[5]
hipError_t chol_reg_probe(int n, const BaArgs* args, unsigned long long* dbg, hipStream_t st);
}  // namespace orbhip
