// Wave64 fp64 exchange helpers shared by the register Cholesky (ba_chol_reg.hip) and the pose
// optimizer (pose_opt.hip): DPP / permlane moves of both 32-bit halves of a double, and
// reductions whose result has the same bits in every lane.
#pragma once
#include <hip/hip_runtime.h>

namespace orbhip {
namespace {

__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ unsigned lo32(double v) { return (unsigned)__builtin_bit_cast(unsigned long long, v); }
__device__ __forceinline__ unsigned hi32(double v) { return (unsigned)(__builtin_bit_cast(unsigned long long, v) >> 32); }
__device__ __forceinline__ double mk64(unsigned lo, unsigned hi) {
    return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}

// DPP move of a double (both halves), e.g. row_newbcast:J = 0x150 + J (lane J of each 16-lane row)
template <int CTRL>
__device__ __forceinline__ double dpp64(double v) {
    return mk64((unsigned)__builtin_amdgcn_update_dpp(0, (int)lo32(v), CTRL, 0xF, 0xF, false),
                (unsigned)__builtin_amdgcn_update_dpp(0, (int)hi32(v), CTRL, 0xF, 0xF, false));
}

// the value of row group G (lanes 16G..16G+15) at the same lane position, in every row group:
// permlane16_swap(v, v) gives [r0 r0 r2 r2] / [r1 r1 r3 r3], permlane32_swap then [x_lo x_lo] / [x_hi x_hi]
template <int G>
__device__ __forceinline__ unsigned rowgroup_bcast32(unsigned v) {
    const auto s = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    const unsigned e = (G & 1) ? s[1] : s[0];
    const auto t = __builtin_amdgcn_permlane32_swap(e, e, false, false);
    return (G & 2) ? t[1] : t[0];
}
template <int G>
__device__ __forceinline__ double rowgroup_bcast(double v) {
    return mk64(rowgroup_bcast32<G>(lo32(v)), rowgroup_bcast32<G>(hi32(v)));
}

// sum over the 16 lanes of a row group, bit-identical in every lane (xor 1, xor 2, half-row
// mirror, row mirror: each level adds the same two partial sums)
__device__ __forceinline__ double row16_sum(double v) {
    v += dpp64<0xB1>(v);    // quad_perm [1,0,3,2]
    v += dpp64<0x4E>(v);    // quad_perm [2,3,0,1]
    v += dpp64<0x141>(v);   // row_half_mirror
    v += dpp64<0x140>(v);   // row_mirror
    return v;
}
// sum over the 4 row groups (same l & 15), bit-identical in every lane
__device__ __forceinline__ double col4_sum(double v) {
    const auto sl = __builtin_amdgcn_permlane16_swap(lo32(v), lo32(v), false, false);
    const auto sh = __builtin_amdgcn_permlane16_swap(hi32(v), hi32(v), false, false);
    const double w = mk64(sl[0], sh[0]) + mk64(sl[1], sh[1]);   // even rows + odd rows
    const auto tl = __builtin_amdgcn_permlane32_swap(lo32(w), lo32(w), false, false);
    const auto th = __builtin_amdgcn_permlane32_swap(hi32(w), hi32(w), false, false);
    return mk64(tl[0], th[0]) + mk64(tl[1], th[1]);              // low half + high half
}

}  // namespace
}  // namespace orbhip
