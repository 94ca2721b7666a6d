// Floor of the C3 level-1 resize traffic (64 frames, 1280x720 -> 1067x600): a flat uint4 stream of
// the same bytes, and a dword gather with k_resize's row/column pattern but no arithmetic.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr int SW = 1280, SH = 720, DW = 1067, DH = 600, DP = 1088, NF = 64;

__global__ void k_stream(const uint4* __restrict__ s, uint4* __restrict__ d, int64_t ns, int64_t nd) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t st = (int64_t)gridDim.x * blockDim.x;
    uint4 acc = {0, 0, 0, 0};
    for (int64_t k = i; k < ns; k += st) { uint4 v = s[k]; acc.x ^= v.x; acc.y ^= v.y; acc.z ^= v.z; acc.w ^= v.w; }
    for (int64_t k = i; k < nd; k += st) d[k] = acc;
}

template <int R>
__global__ __launch_bounds__(256) void k_gather(const uint8_t* __restrict__ s, uint8_t* __restrict__ d) {
    const int f = blockIdx.z;
    const int dyb = (blockIdx.y * 4 + threadIdx.y) * R;
    const int dx0 = (blockIdx.x * 64 + threadIdx.x) * 4;
    if (dyb >= DH || dx0 >= DW) return;
    const int base = ((dx0 * 6) / 5) & ~3;
    uint32_t W[R + 2][3];
    const uint8_t* sf = s + (int64_t)f * SW * SH;
    const int rb = (dyb * 6) / 5;
#pragma unroll
    for (int i = 0; i < R + 2; i++) {
        const uint32_t* p = (const uint32_t*)(sf + (int64_t)min(rb + i, SH - 1) * SW + min(base, SW - 12));
        W[i][0] = p[0]; W[i][1] = p[1]; W[i][2] = p[2];
    }
#pragma unroll
    for (int j = 0; j < R; j++) {
        if (dyb + j >= DH) break;
        const uint32_t v = W[j][0] ^ W[j + 1][1] ^ W[j + 2][2];
        if (dx0 + 3 < DW) *(uint32_t*)(d + (int64_t)f * DP * DH + (int64_t)(dyb + j) * DP + dx0) = v;
    }
}

template <typename F>
static float timeit(F launch) {
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    for (int i = 0; i < 3; i++) launch();
    hipEventRecord(a);
    for (int i = 0; i < 20; i++) launch();
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    return ms * 1000.f / 20;
}

int main() {
    uint8_t *s, *d;
    const int64_t nsb = (int64_t)NF * SW * SH, ndb = (int64_t)NF * DP * DH;
    hipMalloc(&s, nsb); hipMalloc(&d, ndb);
    hipMemset(s, 7, nsb); hipMemset(d, 0, ndb);
    for (int g : {1024, 2048, 4096, 8192}) {
        float us = timeit([&] { hipLaunchKernelGGL(k_stream, dim3(g), dim3(256), 0, 0, (const uint4*)s, (uint4*)d, nsb / 16, ndb / 16); });
        printf("stream grid %5d: %7.1f us  %.2f TB/s\n", g, us, (nsb + ndb) / us / 1e6);
    }
    const float u1 = timeit([&] { hipLaunchKernelGGL(k_gather<1>, dim3(5, (DH + 3) / 4, NF), dim3(64, 4), 0, 0, s, d); });
    const float u4 = timeit([&] { hipLaunchKernelGGL(k_gather<4>, dim3(5, (DH + 15) / 16, NF), dim3(64, 4), 0, 0, s, d); });
    printf("gather R=1: %7.1f us   R=4: %7.1f us   (algorithmic %.1f MB)\n", u1, u4, (nsb + (double)NF * DW * DH) / 1e6);
    return 0;
}
