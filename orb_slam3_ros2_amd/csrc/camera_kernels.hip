// Distorted pinhole camera on the device (VERDICT r01 "distorted-camera
// path"): U:src/Frame.cc::Frame::UndistortKeyPoints and Frame::ComputeImageBounds, which call
// cv::undistortPoints(pts, pts, K, mDistCoef, cv::Mat(), mK) (OpenCV 4.5.4,
// imgproc/src/undistort.dispatch.cpp cvUndistortPointsInternal, TermCriteria(MAX_ITER, 5)).
// The node's camera is R:config/Monocular/MilkV.yaml:22-25 (k1 -0.35952, k2 0.080321, p1, p2).
// Arithmetic restated operation for operation in fp64 (built with -ffp-contract=off, so no FMA
// contraction changes a rounding): the result is bit-identical to the CPU path.
// One lane per keypoint; HBM-bound copy of the 24-byte keypoint records (the 5 fixed-point
// rounds are ~60 fp64 ops per point, far below the VALU roof).
#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../include/orbhip.h"
#include "orbhip_kernels.h"

namespace orbhip {

__device__ __forceinline__ void undistort_point(float u_f, float v_f, const orbhip_pinhole& c, float& xo, float& yo) {
    // cvConvert of the CV_32F K and mDistCoef: exact float -> double; k[5..13] = 0
    const double k0 = c.k1, k1 = c.k2, k2 = c.p1, k3 = c.p2, k4 = c.k3, kz = 0.0;
    const double fx = c.fx, fy = c.fy, cx = c.cx, cy = c.cy;
    const double ifx = 1. / fx, ify = 1. / fy;
    const double u = u_f, v = v_f;
    double x = (u - cx) * ifx, y = (v - cy) * ify;
    const double x0 = x, y0 = y;   // the identity tilt leaves them exact
    for (int j = 0; j < 5; j++) {
        const double r2 = x * x + y * y;
        const double icdist = (1 + ((kz * r2 + kz) * r2 + kz) * r2) / (1 + ((k4 * r2 + k1) * r2 + k0) * r2);
        if (icdist < 0) {
            x = (u - cx) * ifx;
            y = (v - cy) * ify;
            break;
        }
        const double deltaX = 2 * k2 * x * y + k3 * (r2 + 2 * x * x) + kz * r2 + kz * r2 * r2;
        const double deltaY = k2 * (r2 + 2 * y * y) + 2 * k3 * x * y + kz * r2 + kz * r2 * r2;
        x = (x0 - deltaX) * icdist;
        y = (y0 - deltaY) * icdist;
    }
    // RR = P * I with P = mK
    const double xx = fx * x + 0.0 * y + cx;
    const double yy = 0.0 * x + fy * y + cy;
    const double ww = 1. / (0.0 * x + 0.0 * y + 1.0);
    xo = (float)(xx * ww);
    yo = (float)(yy * ww);
}

// kps[b][cap] -> out[b][cap] for the first n[b] records (n_arr) or n_fixed; out may alias kps (so
// neither is __restrict__)
__global__ __launch_bounds__(256) void k_undistort_kps(const orbhip_kp* kps, const int32_t* __restrict__ n_arr,
                                                       int n_fixed, int cap, orbhip_pinhole cam, orbhip_kp* out) {
    const int b = blockIdx.y;
    const int i = blockIdx.x * 256 + threadIdx.x;
    const int n = n_arr ? n_arr[b] : n_fixed;
    if (i >= n || i >= cap) return;
    const int64_t o = (int64_t)b * cap + i;
    orbhip_kp k = kps[o];
    if (cam.k1 != 0.0f) undistort_point(k.x, k.y, cam, k.x, k.y);
    out[o] = k;
}

// the 4 image corners, Frame::ComputeImageBounds order
__global__ void k_image_bounds(int cols, int rows, orbhip_pinhole cam, float* __restrict__ bounds) {
    __shared__ float xs[4], ys[4];
    const int t = threadIdx.x;
    if (t < 4) {
        const float u = (t & 1) ? (float)cols : 0.0f, v = (t & 2) ? (float)rows : 0.0f;
        undistort_point(u, v, cam, xs[t], ys[t]);
    }
    __syncthreads();
    if (t == 0) {
        bounds[0] = fminf(xs[0], xs[2]);
        bounds[1] = fmaxf(xs[1], xs[3]);
        bounds[2] = fminf(ys[0], ys[1]);
        bounds[3] = fmaxf(ys[2], ys[3]);
    }
}

void launch_undistort_kps(const orbhip_kp* kps, const int32_t* n_arr, int n_fixed, int B, int cap,
                          const orbhip_pinhole& cam, orbhip_kp* out, hipStream_t st) {
    const int n = n_arr ? cap : n_fixed;
    if (B <= 0 || n <= 0) return;
    hipLaunchKernelGGL(k_undistort_kps, dim3((unsigned)((n + 255) / 256), (unsigned)B), dim3(256), 0, st, kps, n_arr,
                       n_fixed, cap, cam, out);
}

void launch_image_bounds(int cols, int rows, const orbhip_pinhole& cam, float* bounds, hipStream_t st) {
    hipLaunchKernelGGL(k_image_bounds, dim3(1), dim3(64), 0, st, cols, rows, cam, bounds);
}

}  // namespace orbhip
