// Device-side numeric helpers shared by the gfx950 kernels.
// Every routine here reproduces a host libm / OpenCV result bit-for-bit; all
// translation units are compiled with -ffp-contract=off so no FMA is formed.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstdlib>

namespace orbhip {

// cvRound(float) on x86 (cvtss2si, MXCSR round-to-nearest-even)
__device__ __forceinline__ int cv_round(float v) { return (int)__builtin_rintf(v); }

// ---------------------------------------------------------------------------
// glibc 2.35 sinf/cosf (sysdeps/ieee754/flt-32/s_sinf.c, s_cosf.c, sincosf.h):
// double-precision polynomial after a 2^24-prescaled quadrant reduction. This
// restatement matches glibc bit-for-bit on every float in [0, 6.2832]
// (exhaustive host check, tests/test_sincosf.py; device check in the gpu tests),
// which is the whole domain the rBRIEF angle (fastAtan2 degrees * pi/180) spans.
// The reference calls std::cos/std::sin on a float (U:src/ORBextractor.cc::
// computeOrbDescriptor), i.e. glibc cosf/sinf.
// ---------------------------------------------------------------------------
struct SinCosTab {
    double sign[4];
    double hpi_inv, hpi, c0, c1, c2, c3, c4, s1, s2, s3;
};

static __constant__ SinCosTab kSinCosTab[2] = {
    {{1.0, -1.0, -1.0, 1.0}, 0x1.45F306DC9C883p+23, 0x1.921FB54442D18p0, 0x1p0, -0x1.ffffffd0c621cp-2,
     0x1.55553e1068f19p-5, -0x1.6c087e89a359dp-10, 0x1.99343027bf8c3p-16, -0x1.555545995a603p-3,
     0x1.1107605230bc4p-7, -0x1.994eb3774cf24p-13},
    {{1.0, -1.0, -1.0, 1.0}, 0x1.45F306DC9C883p+23, 0x1.921FB54442D18p0, -0x1p0, 0x1.ffffffd0c621cp-2,
     -0x1.55553e1068f19p-5, 0x1.6c087e89a359dp-10, -0x1.99343027bf8c3p-16, -0x1.555545995a603p-3,
     0x1.1107605230bc4p-7, -0x1.994eb3774cf24p-13}};

__device__ __forceinline__ const SinCosTab& sincos_tab(int i) { return kSinCosTab[i]; }

__device__ __forceinline__ uint32_t abstop12(float x) { return (__float_as_uint(x) >> 20) & 0x7ff; }

__device__ __forceinline__ float sincosf_poly(double x, double x2, const SinCosTab& p, int n) {
    if ((n & 1) == 0) {
        double x3 = x * x2;
        double s1 = p.s2 + x2 * p.s3;
        double x7 = x3 * x2;
        double s = x + x3 * p.s1;
        return (float)(s + x7 * s1);
    } else {
        double x4 = x2 * x2;
        double c2 = p.c3 + x2 * p.c4;
        double c1 = p.c0 + x2 * p.c1;
        double x6 = x4 * x2;
        double c = c1 + x4 * p.c2;
        return (float)(c + x6 * c2);
    }
}

__device__ __forceinline__ double sincosf_reduce(double x, const SinCosTab& p, int* np) {
    double r = x * p.hpi_inv;
    int n = ((int32_t)r + 0x800000) >> 24;
    *np = n;
    return x - n * p.hpi;
}

// Valid for |y| < 120 (the range-reduction branch glibc uses up to 120.0f).
__device__ __forceinline__ float glibc_sinf(float y) {
    double x = y;
    if (abstop12(y) < abstop12(0x1.921FB6p-1f)) {
        double s = x * x;
        if (abstop12(y) < abstop12(0x1p-12f)) return y;
        return sincosf_poly(x, s, sincos_tab(0), 0);
    }
    int n;
    x = sincosf_reduce(x, sincos_tab(0), &n);
    double s = sincos_tab(0).sign[n & 3];
    return sincosf_poly(x * s, x * x, sincos_tab((n & 2) ? 1 : 0), n);
}

__device__ __forceinline__ float glibc_cosf(float y) {
    double x = y;
    if (abstop12(y) < abstop12(0x1.921FB6p-1f)) {
        double x2 = x * x;
        if (abstop12(y) < abstop12(0x1p-12f)) return 1.0f;
        return sincosf_poly(x, x2, sincos_tab(0), 1);
    }
    int n;
    x = sincosf_reduce(x, sincos_tab(0), &n);
    double s = sincos_tab(0).sign[n & 3];
    return sincosf_poly(x * s, x * x, sincos_tab((n & 2) ? 1 : 0), n ^ 1);
}

// OCV:core mathfuncs_core atan_f32 == cv::fastAtan2(y, x), degrees in [0, 360)
__device__ __forceinline__ float fast_atan2(float y, float x) {
    const float p1 = 0.9997878412794807f * 57.295780181884765625f;   // (float)(180/CV_PI)
    const float p3 = -0.3258083974640975f * 57.295780181884765625f;
    const float p5 = 0.1555786518463281f * 57.295780181884765625f;
    const float p7 = -0.04432655554792128f * 57.295780181884765625f;
    const float eps = (float)2.220446049250313e-16;                  // (float)DBL_EPSILON
    float ax = fabsf(x), ay = fabsf(y);
    float a, c, c2;
    if (ax >= ay) {
        c = ay / (ax + eps);
        c2 = c * c;
        a = (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
    } else {
        c = ax / (ay + eps);
        c2 = c * c;
        a = 90.f - (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
    }
    if (x < 0) a = 180.f - a;
    if (y < 0) a = 360.f - a;
    return a;
}

// ---------------------------------------------------------------------------
// wave64 / block helpers
// ---------------------------------------------------------------------------
__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }


// inclusive prefix sum within a wave64: DPP row_shr 1/2/4/8 inside each 16-lane row, then
// row_bcast:15 / row_bcast:31 carry the row totals (VALU only, no LDS round trips)
__device__ __forceinline__ int wave_incl_scan(int v) {
    v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xF, 0xF, false);   // row_shr:1
    v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xF, 0xF, false);   // row_shr:2
    v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xF, 0xF, false);   // row_shr:4
    v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xF, 0xF, false);   // row_shr:8
    v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xA, 0xF, false);   // row_bcast:15 -> rows 1, 3
    v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xC, 0xF, false);   // row_bcast:31 -> rows 2, 3
    return v;
}

// Work-groups are dealt round-robin over the 8 XCDs (dispatch index b -> XCD b % 8; observed,
// speed only, never correctness). xcd_runs maps dispatch index b of a grid of n onto a logical
// index such that each XCD receives runs of g consecutive logical indices, the runs dealt
// round-robin: neighbouring tiles / cells / keypoints, whose image windows overlap, then share one
// XCD's L2 (fewer lines fetched by several L2s), while every XCD still gets a spread of the grid
// (balance: level-0 cells cost more than the others). Identity on the tail past the last full
// round of 8 runs, so a bijection on [0, n) for any n; g == 0 is the identity.
__device__ __forceinline__ int xcd_runs(int b, int n, int g) {
    if (g <= 0) return b;
    const int full = (n / (8 * g)) * (8 * g);
    if (b >= full) return b;
    const int k = b & 7, i = b >> 3;
    return ((i / g) * 8 + k) * g + (i % g);
}

__device__ __forceinline__ int wave_sum_i32(int v) {
    return __builtin_amdgcn_readlane(wave_incl_scan(v), 63);
}

// Exclusive block scan of one int per thread. `scratch` >= blockDim/64 + 1 ints of LDS.
// Returns the exclusive prefix; *total receives the block sum. Two barriers: every wave
// re-scans the per-wave partials itself (no serial thread-0 pass); the trailing barrier lets
// the caller reuse `scratch` immediately.
__device__ __forceinline__ int block_excl_scan(int v, int* scratch, int* total) {
    const int lane = lane_id(), wid = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
    const int inc = wave_incl_scan(v);
    if (lane == 63) scratch[wid] = inc;
    __syncthreads();
    const int ws = wave_incl_scan(lane < nw ? scratch[lane] : 0);
    const int before = __builtin_amdgcn_readlane(ws, wid > 0 ? wid - 1 : 0);   // wid is wave-uniform
    *total = __builtin_amdgcn_readlane(ws, nw - 1);
    __syncthreads();
    return (wid > 0 ? before : 0) + inc - v;
}

// ---------------------------------------------------------------------------
// Diagnostics: per-workgroup timing trace (test hooks orbhip_test_trace_*). g_trace is null
// unless enabled, so production launches pay one scalar load and a branch. Each translation
// unit owns its copy (no relocatable device code), set through trace_set_<unit>().
// Layout per kernel id k (stride kTraceStride u64): [2b], [2b+1] = s_memrealtime (100 MHz)
// at start / end of workgroup b (b < 4096); [8192 + ph] = s_memtime cycles of phase ph of
// workgroup 0 (last launch).
// ---------------------------------------------------------------------------

// The unit's trace words are external symbols of hidden visibility: an internal-linkage
// (static) __constant__ variable is addressed through the GOT, i.e. two dependent scalar loads at
// every kernel start (with cold caches, ~1 us) before the branch on tr_buf could resolve.
#define ORBHIP_TRACE_UNIT(unit)                                                                 \
    __constant__ __attribute__((visibility("hidden"))) unsigned long long* g_trace_##unit = nullptr; \
    __constant__ __attribute__((visibility("hidden"))) int g_trace_blk_##unit = 0;          \
    static __device__ __forceinline__ unsigned long long* tr_ptr() { return g_trace_##unit; } \
    static __device__ __forceinline__ int tr_blk_val() { return g_trace_blk_##unit; }       \
    void trace_set_##unit(unsigned long long* p) {                                          \
        (void)hipMemcpyToSymbol(HIP_SYMBOL(g_trace_##unit), &p, sizeof(p));                 \
        const char* e = std::getenv("ORBHIP_TRACE_BLOCK");                                  \
        const int b = e ? std::atoi(e) : 0;                                                 \
        (void)hipMemcpyToSymbol(HIP_SYMBOL(g_trace_blk_##unit), &b, sizeof(b));             \
    }

// (stamping every wave unconditionally, so that nothing waited on the trace word, cost 5% of the
// 16-camera C2 stream: the clock reads are not free when every wave of every launch takes them)
#define TR_BEGIN()                                                                          \
    unsigned long long tr_t0 = 0, tr_tp = 0;                                                \
    unsigned long long* const tr_buf = tr_ptr();                                            \
    const int tr_blk = tr_blk_val();                                                        \
    (void)tr_tp; (void)tr_blk;                                                              \
    if (tr_buf && threadIdx.x == 0) {                                                       \
        tr_t0 = __builtin_amdgcn_s_memrealtime();                                           \
        tr_tp = __builtin_amdgcn_s_memtime();                                               \
    }
#define TR_PHASE(kid, ph)                                                                   \
    if (tr_buf && threadIdx.x == 0 && (int)blockIdx.x == tr_blk && blockIdx.y == 0 && blockIdx.z == 0) { \
        const unsigned long long tr_t = __builtin_amdgcn_s_memtime();                       \
        tr_buf[(kid) * kTraceStride + 8192 + (ph)] = tr_t - tr_tp;                          \
        tr_tp = tr_t;                                                                       \
    }
#define TR_END(kid)                                                                         \
    if (tr_buf && threadIdx.x == 0) {                                                       \
        const unsigned tr_b = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z); \
        if (tr_b < 4096) {                                                                  \
            tr_buf[(kid) * kTraceStride + 2 * tr_b] = tr_t0;                                \
            tr_buf[(kid) * kTraceStride + 2 * tr_b + 1] = __builtin_amdgcn_s_memrealtime(); \
        }                                                                                   \
    }

}  // namespace orbhip
