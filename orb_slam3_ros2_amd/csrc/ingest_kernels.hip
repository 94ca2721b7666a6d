// gfx950 ingest: cv_bridge::toCvShare(bgr8 -> MONO8) = OpenCV cvtColor(COLOR_BGR2GRAY) 8U,
// bit-exact fixed point Y = (B*1868 + G*9617 + R*4899 + 2^13) >> 14 (R:src/imu_mono_realsense.cpp:298,
// OCV imgproc color_rgb RGB2Gray<uchar>). HBM-bound streaming kernel: 3 B in + 1 B out per px.
//   k_bgr2gray   grid (row chunks, rows, frames); each lane converts 16 px: three 16-byte
//                loads (48 B of BGR) and one 16-byte store when the row segment is aligned and
//                whole, a byte-wise tail otherwise.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "orbhip_kernels.h"

namespace orbhip {

__device__ __forceinline__ uint32_t gray_px(uint32_t b, uint32_t g, uint32_t r) {
    return (b * 1868u + g * 9617u + r * 4899u + (1u << 13)) >> 14;
}

__global__ __launch_bounds__(256) void k_bgr2gray(const uint8_t* __restrict__ src, int w, int h, int sstride,
                                                  int64_t sfstride, uint8_t* __restrict__ dst, int dstride,
                                                  int64_t dfstride) {
    const int y = blockIdx.y, f = blockIdx.z;
    const int x0 = (blockIdx.x * blockDim.x + threadIdx.x) * 16;
    if (x0 >= w) return;
    const uint8_t* s = src + f * sfstride + (int64_t)y * sstride + 3 * x0;
    uint8_t* d = dst + f * dfstride + (int64_t)y * dstride + x0;
    const bool vec = x0 + 16 <= w && (((uintptr_t)s | (uintptr_t)d) & 15) == 0;
    if (vec) {
        const uint4 v0 = *(const uint4*)s, v1 = *(const uint4*)(s + 16), v2 = *(const uint4*)(s + 32);
        uint32_t in[12] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w, v2.x, v2.y, v2.z, v2.w};
        uint32_t out[4] = {0, 0, 0, 0};
#pragma unroll
        for (int i = 0; i < 16; i++) {
            const int o = 3 * i;
            const uint32_t b = (in[o >> 2] >> (8 * (o & 3))) & 255;
            const uint32_t g = (in[(o + 1) >> 2] >> (8 * ((o + 1) & 3))) & 255;
            const uint32_t r = (in[(o + 2) >> 2] >> (8 * ((o + 2) & 3))) & 255;
            out[i >> 2] |= gray_px(b, g, r) << (8 * (i & 3));
        }
        *(uint4*)d = make_uint4(out[0], out[1], out[2], out[3]);
    } else {
        const int n = min(16, w - x0);
        for (int i = 0; i < n; i++) d[i] = (uint8_t)gray_px(s[3 * i], s[3 * i + 1], s[3 * i + 2]);
    }
}

void launch_bgr2gray(const uint8_t* src, int B, int w, int h, int sstride, int64_t sfstride, uint8_t* dst, int dstride,
                     int64_t dfstride, hipStream_t st) {
    const int per_block = 256 * 16;
    dim3 grid((unsigned)((w + per_block - 1) / per_block), (unsigned)h, (unsigned)B);
    hipLaunchKernelGGL(k_bgr2gray, grid, dim3(256), 0, st, src, w, h, sstride, sfstride, dst, dstride, dfstride);
}

}  // namespace orbhip
