// gfx950 kernels of the ORB front-end (ORBextractor::operator() restated for CDNA4).
//
//   k_resize      a3/a4  one pyramid level from the previous one (cascade), bit-exact
//                        OpenCV 8U INTER_LINEAR fixed point (H exact, V SIMD/scalar split)
//   k_fast_cells  a5/a6  per 35-px cell: FAST-9 strength map in LDS, window-local strict
//                        3x3 NMS at iniThFAST, fallback to minThFAST, row-major compaction
//   k_octree      a7     DistributeOctTree emulated with arrays: one 1024-thread workgroup
//                        per (frame, level); list order / creation-serial tie-break exact
//   k_desc        a8/a9  per keypoint (one wave): IC_Angle + glibc sinf/cosf + rBRIEF on
//                        the 7x7 bit-exact Gaussian sampled from an LDS patch; final
//                        operator() ordering (lapping area from the end)
//
// Everything is integer or reproduces host float rounding exactly (-ffp-contract=off).
#include <hip/hip_runtime.h>
#include <cstdlib>
#include <type_traits>

#include "../../include/orbhip.h"
#include "dev_attr.h"
#include "../../include/orbhip_pattern.h"
#include "orbhip_device.h"
#include "orbhip_kernels.h"
#include "orbhip_plan.h"

namespace orbhip {

// external, hidden: a static __constant__ table is addressed through the GOT (a dependent load)
__constant__ __attribute__((visibility("hidden"))) signed char kPattern[256 * 4] = ORBHIP_BIT_PATTERN_31_INIT;

ORBHIP_TRACE_UNIT(extract)

// ---------------------------------------------------------------------------
// image addressing: level 0 is the caller's frame, levels >= 1 live in the pyramid block
// ---------------------------------------------------------------------------
struct ImgRef {
    const uint8_t* p;
    int pitch;
};

__device__ __forceinline__ ImgRef level_img(const ExtractPlan* __restrict__ P, const FrameBufs& fb, int f, int l) {
    if (l == 0) return ImgRef{fb.in + (int64_t)f * fb.in_fstride, fb.in_stride};
    return ImgRef{fb.pyr + (int64_t)f * P->pyr_bytes + P->lv[l].pyr_off, P->lv[l].pitch};
}

// a wave's own LDS writes visible to its later LDS reads (no workgroup barrier)
// LDS-only form: waits for the wave's LDS operations alone (a seq_cst fence also waits vmcnt(0),
// i.e. for every outstanding global store)
__device__ __forceinline__ void wave_lds_only() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
}
__device__ __forceinline__ void wave_lds_fence() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

// ---------------------------------------------------------------------------
// k_resize: OCV resizeGeneric_ 8UC1 INTER_LINEAR; block (64,4), 4 output px x kRzRows output rows
// per thread. Latency-bound at one round trip per dependent load, so each thread keeps
// kRzRows x 4 output bytes in flight: after the column and row tables, every source row its
// output rows read (a 1.2x downscale: kRzRows + 2 rows) is loaded at once as 3 aligned dwords.
// ---------------------------------------------------------------------------
constexpr int kRzRows = 4;
constexpr int kRzSrc = kRzRows + 2;   // source rows held (more: the per-row path)

// one output pixel from its two source rows' byte pairs (p0x: row sy, p1x: row sy + 1)
__device__ __forceinline__ int rz_px(int p00, int p01, int p10, int p11, int aa, int b0, int b1,
                                     bool inx, bool vecy) {
    int h0, h1;
    if (inx) {
        const int a0 = (int)(short)(aa & 0xFFFF), a1 = (int)(short)(aa >> 16);
        h0 = p00 * a0 + p01 * a1;
        h1 = p10 * a0 + p11 * a1;
    } else {
        h0 = p00 * 2048;
        h1 = p10 * 2048;
    }
    int v;
    if (vecy) {   // VResizeLinearVec_32s8u lanes (128-bit baseline)
        const int s0 = min(max(h0 >> 4, -32768), 32767);
        const int s1 = min(max(h1 >> 4, -32768), 32767);
        int t = ((s0 * b0) >> 16) + ((s1 * b1) >> 16);
        t = min(max(t, -32768), 32767);
        v = (t + 2) >> 2;
    } else {      // FixedPtCast<int, uchar, 22>
        v = (h0 * b0 + h1 * b1 + (1 << 21)) >> 22;
    }
    return v < 0 ? 0 : (v > 255 ? 255 : v);
}

typedef __attribute__((address_space(1))) int ex_gint;
// the one-launch batch pyramid (k_pyr_flow) reads the levels it writes itself: 4-byte sc1 buffer
// loads (L2-served, never a stale L1 line; MI355X_MICROARCH.md visibility table, row 1)
__device__ __forceinline__ uint32_t pyr_ld4_sc1(__amdgpu_buffer_rsrc_t rs, const uint8_t* p, const uint8_t* pyr) {
    return __builtin_amdgcn_raw_buffer_load_b32(rs, (int)(p - pyr), 0, 16);
}

// one lane's 4 columns x kRzRows rows of level l of frame f: output rows [dyb, min(dyb + kRzRows,
// row_end)) (dyb wave-uniform), columns dx0..dx0+3 (dx0 < the level's width).
// FLOW (k_pyr_flow): the outputs go to the wave's LDS stage (row j at dwords [64 j, 64 j + 64), this
// lane's 4 bytes at dword lane) instead of the pyramid, and a source level >= 1 is read with sc1 loads.
template <bool FLOW>
__device__ __forceinline__ void resize_tile_g(const ExtractPlan* __restrict__ P, const FrameBufs& fb, int f, int l,
                                              int dyb, int dx0, int row_end, const int* __restrict__ xofs,
                                              const int* __restrict__ xalpha, const int* __restrict__ yofs,
                                              const int* __restrict__ ybeta, __amdgpu_buffer_rsrc_t prs,
                                              uint32_t* stage) {
    const bool sc1 = FLOW && l >= 2;   // wave-uniform
    // geometry copied to registers (the byte stores below may alias the plan for the compiler)
    const int Dw = P->lv[l].w, Dpitch = P->lv[l].pitch;
    const int xmax = P->lv[l].xmax, vend = P->lv[l].vend;
    const int xtab = P->lv[l].xtab_off, ytab = P->lv[l].ytab_off;
    const int Sw = P->lv[l - 1].w, Sh = P->lv[l - 1].h;
    const ImgRef src = level_img(P, fb, f, l - 1);
    uint8_t* const dst0 = fb.pyr + (int64_t)f * P->pyr_bytes + P->lv[l].pyr_off;
    // the 4 columns' tables as one int4 each (16-byte aligned per level), the rows' tables
    const int4 xo4 = *(const int4*)(xofs + xtab + dx0);
    const int4 xa4 = *(const int4*)(xalpha + xtab + dx0);
    const int nrow = min(kRzRows, row_end - dyb);
    int sy[kRzRows], bbv[kRzRows];
#pragma unroll
    for (int j = 0; j < kRzRows; j++) {
        const int dy = dyb + min(j, nrow - 1);
        sy[j] = __builtin_amdgcn_readfirstlane(yofs[ytab + dy]);   // dy is wave-uniform
        bbv[j] = __builtin_amdgcn_readfirstlane(ybeta[ytab + dy]);
    }
    const int sxa[4] = {xo4.x, xo4.y, xo4.z, xo4.w}, axa[4] = {xa4.x, xa4.y, xa4.z, xa4.w};
    const int base = sxa[0] & ~3;
    auto clampr = [&](int r) { return r < 0 ? 0 : (r < Sh ? r : Sh - 1); };
    const int rbase = clampr(sy[0]);
    // interior lanes: 4 full columns inside xmax / vend, the source span as 3 aligned dwords of
    // each row, every row the outputs read within kRzSrc rows of rbase
    const bool interior = ((src.pitch & 3) == 0) && ((((uintptr_t)src.p) & 3) == 0) && base + 12 <= Sw &&
                          sxa[3] - base <= 10 &&
                          dx0 + 3 < xmax && dx0 + 3 < vend && nrow == kRzRows &&
                          clampr(sy[kRzRows - 1] + 1) - rbase < kRzSrc;
    if (interior) {
        uint32_t W[kRzSrc][3];
#pragma unroll
        for (int i = 0; i < kRzSrc; i++) {
            const uint8_t* pb = src.p + (int64_t)min(rbase + i, Sh - 1) * src.pitch + base;
            if (sc1) {   // one 16-byte sc1 load (4-byte aligned) for the 12-byte span
                typedef unsigned int u32x4v __attribute__((ext_vector_type(4)));
                const u32x4v q = __builtin_amdgcn_raw_buffer_load_b128(prs, (int)(pb - fb.pyr), 0, 16);
                W[i][0] = q.x; W[i][1] = q.y; W[i][2] = q.z;
            } else {
                const uint32_t* p = (const uint32_t*)pb;
                W[i][0] = p[0]; W[i][1] = p[1]; W[i][2] = p[2];
            }
        }
        // horizontal pass once per source row: bytes o, o + 1 (o = sx - base <= 10) of the 12-byte
        // span picked by one v_perm from the dword pair (w1:w0) (o <= 6) or (w2:w1) into 16-bit
        // halves, times the (a0, a1) pair by one dot2. A column whose lanes all have o <= 6 (every
        // column but the last at 1.2x) needs no pair choice.
        typedef short short2v __attribute__((ext_vector_type(2)));
        int H[4][kRzSrc];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const int o = sxa[k] - base;
            const int oo = o > 6 ? o - 4 : o;
            const uint32_t sel = 0x0C000C00u | (uint32_t)oo | ((uint32_t)(oo + 1) << 16);
            const short2v av = __builtin_bit_cast(short2v, axa[k]);
            const uint64_t m = __builtin_amdgcn_ballot_w64(o > 6);
            if (m == 0) {
#pragma unroll
                for (int i = 0; i < kRzSrc; i++) {
                    const uint32_t pp = __builtin_amdgcn_perm(W[i][1], W[i][0], sel);
                    H[k][i] = __builtin_amdgcn_sdot2(__builtin_bit_cast(short2v, pp), av, 0, false);
                }
            } else {
                // lane-mask choice (a plain ?: over W lets the compiler turn it into an indexed
                // scratch load)
                auto pick = [](uint32_t f, uint32_t t, uint64_t mm) {
                    uint32_t r;
                    asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(f), "v"(t), "s"(mm));
                    return r;
                };
#pragma unroll
                for (int i = 0; i < kRzSrc; i++) {
                    const uint32_t pp = __builtin_amdgcn_perm(pick(W[i][1], W[i][2], m), pick(W[i][0], W[i][1], m), sel);
                    H[k][i] = __builtin_amdgcn_sdot2(__builtin_bit_cast(short2v, pp), av, 0, false);
                }
            }
        }
        // vertical pass (VResizeLinearVec_32s8u lanes, 128-bit baseline); with taps checked on the
        // host (rz_noclamp) its saturations cannot bind and are left out
        const bool noclamp = P->lv[l].rz_noclamp != 0;
#pragma unroll
        for (int j = 0; j < kRzRows; j++) {
            // wave-uniform; readfirstlane'd so the H[k][i] selects stay SGPR-indexed (s_set_gpr_idx)
            // in every caller: left in VGPRs (k_resize_bands, k_pyr_flow) they were lowered to
            // readlane / writelane loops, ~25k cycles per 4-row tile
            const int i0 = __builtin_amdgcn_readfirstlane(clampr(sy[j]) - rbase);
            const int i1 = __builtin_amdgcn_readfirstlane(clampr(sy[j] + 1) - rbase);
            const int b0 = (int)(short)(bbv[j] & 0xFFFF), b1 = (int)(short)(bbv[j] >> 16);
            uint32_t packed = 0;
            if (noclamp) {
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    const int t = (__mul24(H[k][i0] >> 4, b0) >> 16) + (__mul24(H[k][i1] >> 4, b1) >> 16);
                    packed |= (uint32_t)((t + 2) >> 2) << (8 * k);
                }
            } else {
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    const int s0 = min(max(H[k][i0] >> 4, -32768), 32767);
                    const int s1 = min(max(H[k][i1] >> 4, -32768), 32767);
                    int t = ((s0 * b0) >> 16) + ((s1 * b1) >> 16);
                    t = min(max(t, -32768), 32767);
                    int v = (t + 2) >> 2;
                    v = v < 0 ? 0 : (v > 255 ? 255 : v);
                    packed |= (uint32_t)v << (8 * k);
                }
            }
            if (FLOW) stage[j * 64 + (threadIdx.x & 63)] = packed;
            else *(uint32_t*)(dst0 + (int64_t)(dyb + j) * Dpitch + dx0) = packed;
        }
    } else {
        auto ld1 = [&](const uint8_t* q) -> int {
            if (!sc1) return *q;
            const uintptr_t a = (uintptr_t)q;
            return (int)((pyr_ld4_sc1(prs, (const uint8_t*)(a & ~(uintptr_t)3), fb.pyr) >> (8 * (a & 3))) & 0xFFu);
        };
        for (int j = 0; j < nrow; j++) {
            const int dy = dyb + j;
            uint8_t* dst = dst0 + (int64_t)dy * Dpitch;
            const uint8_t* S0 = src.p + (int64_t)clampr(sy[j]) * src.pitch;
            const uint8_t* S1 = src.p + (int64_t)clampr(sy[j] + 1) * src.pitch;
            const int b0 = (int)(short)(bbv[j] & 0xFFFF), b1 = (int)(short)(bbv[j] >> 16);
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const int dx = dx0 + k;
                if (dx >= Dw) break;
                const int sx = sxa[k];
                const bool inx = dx < xmax;
                const int p00 = ld1(S0 + sx), p10 = ld1(S1 + sx);
                const int p01 = inx ? ld1(S0 + sx + 1) : 0, p11 = inx ? ld1(S1 + sx + 1) : 0;
                const uint8_t v = (uint8_t)rz_px(p00, p01, p10, p11, axa[k], b0, b1, inx, dx < vend);
                if (FLOW) ((uint8_t*)stage)[j * 256 + (threadIdx.x & 63) * 4 + k] = v;
                else dst[dx] = v;
            }
        }
    }
}

__device__ __forceinline__ void resize_tile(const ExtractPlan* __restrict__ P, const FrameBufs& fb, int f, int l,
                                            int dyb, int dx0, int row_end, const int* __restrict__ xofs,
                                            const int* __restrict__ xalpha, const int* __restrict__ yofs,
                                            const int* __restrict__ ybeta) {
    resize_tile_g<false>(P, fb, f, l, dyb, dx0, row_end, xofs, xalpha, yofs, ybeta,
                         __builtin_amdgcn_make_buffer_rsrc(fb.pyr, 0, 0, 0x00020000), nullptr);
}

__global__ __launch_bounds__(256) void k_resize(const ExtractPlan* __restrict__ P, FrameBufs fb, int l,
                                                const int* __restrict__ xofs, const int* __restrict__ xalpha,
                                                const int* __restrict__ yofs, const int* __restrict__ ybeta) {
    TR_BEGIN()
    const int Dw = P->lv[l].w, Dh = P->lv[l].h;
    // row groups on blockIdx.x: consecutive work-groups (dealt round-robin to the XCDs) walk down
    // a column strip, so every XCD gets the same share of the light right-edge strip
    const int dyb = (blockIdx.x * 4 + threadIdx.y) * kRzRows;   // wave-uniform
    const int dx0 = (blockIdx.y * 64 + threadIdx.x) * 4;
    if (dyb >= Dh || dx0 >= Dw) return;
    resize_tile(P, fb, blockIdx.z, l, dyb, dx0, Dh, xofs, xalpha, yofs, ybeta);
    if (l == 1) { TR_END(0) }
}

// Levels s0+1 .. L-1 of every frame in ONE launch (batches: the small levels' k_resize launches
// are latency-bound, ~13-25 us each at C3 whatever their size). Work-group (band, frame) computes,
// level by level, the full-width output rows rows[band][l] = its band of level l plus the halo
// rows the next level's band rows read, from the level below in global memory (its own rows of
// the step before; level s0 from k_resize), and writes them to the pyramid. A halo row is
// computed by both neighbouring bands with identical bytes. Waves take (4-row group, 256-column
// strip) tiles in turn; one workgroup barrier per level; no work-group waits for another.
__global__ __launch_bounds__(256) void k_resize_bands(const ExtractPlan* __restrict__ P, FrameBufs fb, int s0,
                                                       const int2* __restrict__ rows, const int* __restrict__ xofs,
                                                       const int* __restrict__ xalpha,
                                                       const int* __restrict__ yofs,
                                                       const int* __restrict__ ybeta) {
    TR_BEGIN()
    const int band = blockIdx.x, f = blockIdx.y;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, nw = blockDim.x >> 6;
    const int L = P->n_levels;
    for (int l = s0 + 1; l < L; l++) {
        const int2 rr = rows[band * kMaxLevels + l];
        const int Dw = P->lv[l].w;
        const int ng = (rr.y - rr.x + kRzRows - 1) / kRzRows, ns = (Dw + 255) / 256;
        for (int t = wave; t < ng * ns; t += nw) {   // wave-uniform
            const int g = t / ns, sidx = t - g * ns;
            const int dx0 = sidx * 256 + lane * 4;
            if (dx0 < Dw) resize_tile(P, fb, f, l, rr.x + g * kRzRows, dx0, rr.y, xofs, xalpha, yofs, ybeta);
        }
        __syncthreads();   // the level's rows (this work-group's global stores) before the next level reads them
        TR_PHASE(6, l)
    }
    TR_END(6)
}

// k_pyr_flow: the whole batch cascade (levels 1..L-1 of every frame) in ONE launch, as a dataflow
// over row bands. A task = (level l, frame f, band b): output rows [16 b, 16 b + 16) of level l,
// full width; wave w computes rows 16 b + 4 w .. + 3 with k_resize's per-pixel code
// (resize_tile), strip by strip (256 columns), staged in LDS and written as 16-byte sc1 stores.
// The frames are dealt to kFlowQ queues (frame f to queue f mod kFlowQ, work-group g serves queue
// g mod kFlowQ); a queue's tasks are numbered level-major, frame-major, and taken kFlowChunk
// tickets at a time from the queue's counter. A task of level l >= 2 first waits (wave 0, bounded
// sc1 polls) for the flags of the level l-1 bands of its frame that its source rows lie in: tasks
// of the same queue with lower tickets, and a ticket is only taken by a running work-group that
// runs its tickets in order, so the launch cannot deadlock whatever the grid size, residency or
// dispatch order. Visibility (MI355X_MICROARCH.md, visibility table row 1): the payload is stored
// sc1, each wave drains vmcnt, the work-group barriers, one lane stores the band's flag (agent
// scope); the consumer polls the flag with sc1 loads and reads the bytes with sc1 loads only
// (16-byte). Flags hold the launch's generation (advanced with the ticket reset by the last
// work-group out), so nothing is cleared between launches. A spin that runs out counts in
// ctl[kFlowQ + 2] (never expected: the waits cannot deadlock) and the band proceeds.
// ---------------------------------------------------------------------------
constexpr int kFlowRows = 16;         // output rows per task (4 waves x kRzRows)
constexpr int kFlowSpin = 1 << 22;    // polls before a wait gives up (~0.5 s)

__global__ __launch_bounds__(256) void k_pyr_flow(const ExtractPlan* __restrict__ P, FrameBufs fb,
                                                   const int* __restrict__ xofs, const int* __restrict__ xalpha,
                                                   const int* __restrict__ yofs, const int* __restrict__ ybeta,
                                                   PyrFlow a) {
    __shared__ __attribute__((aligned(16))) uint32_t stage[4][kRzRows * 64];
    __shared__ int s_t;
    TR_BEGIN()
    int tr_k = 0;   // tasks run by this work-group (trace phases of work-group 0: wait, then compute)
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int L = P->n_levels;
    int* const ctl = a.ctl;
    const int gen = __hip_atomic_load((ex_gint*)(ctl + kFlowQ + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const __amdgpu_buffer_rsrc_t prs = __builtin_amdgcn_make_buffer_rsrc(fb.pyr, 0, a.pyr_limit, 0x00020000);
    const int q = blockIdx.x % kFlowQ;
    const int nfq = q < a.B ? (a.B - q + kFlowQ - 1) / kFlowQ : 0;   // frames q, q + Q, ...
    const int ntask = nfq * a.boff[L];
    for (;;) {
        if (tid == 0) s_t = atomicAdd(ctl + q, kFlowChunk);
        __syncthreads();
        const int t0 = s_t;
        if (t0 >= ntask) break;
        const int t1 = min(t0 + kFlowChunk, ntask);
        for (int t = t0; t < t1; t++) {
            int l = 1;
            while (l + 1 < L && nfq * a.boff[l + 1] <= t) l++;
            const int nb = a.boff[l + 1] - a.boff[l];
            const int loc = t - nfq * a.boff[l], fi = loc / nb, b = loc - fi * nb;
            const int f = q + kFlowQ * fi;
            int* const fl = a.flags + (int64_t)f * a.nbt;
            if (l >= 2 && wave == 0) {
                const int2 d = a.dep[a.boff[l] + b];   // level l-1 bands holding this band's source rows
                const int* w = fl + a.boff[l - 1];
                for (int it = 0;; it++) {
                    const bool mine = d.x + lane > d.y ||
                                      __hip_atomic_load((ex_gint*)(w + d.x + lane), __ATOMIC_RELAXED,
                                                        __HIP_MEMORY_SCOPE_AGENT) == gen + 1;
                    if (__ballot(!mine) == 0ull) break;
                    if (it >= kFlowSpin) {
                        if (lane == 0) atomicAdd(ctl + kFlowQ + 2, 1);
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                }
            }
            __syncthreads();
            if (tr_k < 32) { TR_PHASE(7, 2 * tr_k) }
            const int Dh = P->lv[l].h, Dw = P->lv[l].w, pitch = P->lv[l].pitch;
            const int row_end = min(b * kFlowRows + kFlowRows, Dh);
            const int dyb = b * kFlowRows + wave * kRzRows;   // wave-uniform
            if (dyb < row_end) {
                const int obase = (int)((int64_t)f * P->pyr_bytes + P->lv[l].pyr_off);
                for (int s0 = 0; s0 < Dw; s0 += 256) {
                    const int dx0 = s0 + lane * 4;
                    if (dx0 < Dw)
                        resize_tile_g<true>(P, fb, f, l, dyb, dx0, row_end, xofs, xalpha, yofs, ybeta, prs,
                                            stage[wave]);
                    wave_lds_only();   // the stage's LDS writes, not the strip's stores (no vmcnt wait)
                    const int r = lane >> 4, c = s0 + (lane & 15) * 16;
                    if (dyb + r < row_end && c < Dw) {
                        const uint4 v = *(const uint4*)&stage[wave][r * 64 + (lane & 15) * 4];
                        typedef unsigned int u32x4v __attribute__((ext_vector_type(4)));
                        const u32x4v u = {v.x, v.y, v.z, v.w};
                        __builtin_amdgcn_raw_buffer_store_b128(u, prs, obase + (dyb + r) * pitch + c, 0, 16);
                    }
                    wave_lds_only();
                }
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (tid == 0)
                __hip_atomic_store((ex_gint*)(fl + a.boff[l] + b), gen + 1, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
            if (tr_k < 32) { TR_PHASE(7, 2 * tr_k + 1) }
            tr_k++;
        }
    }
    TR_END(7)
    // the last work-group out resets the tickets and advances the generation for the next launch
    if (tid == 0 && atomicAdd(ctl + kFlowQ, 1) == (int)gridDim.x - 1) {
        for (int i = 0; i <= kFlowQ; i++)
            __hip_atomic_store((ex_gint*)(ctl + i), 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store((ex_gint*)(ctl + kFlowQ + 1), gen + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// quotient of i / d for 0 <= i < 2^16, d >= 1: the float reciprocal's error stays below the
// 0.5/d margin of (i + 0.5)/d to the next integer
__device__ __forceinline__ int small_div(int i, float inv_d) { return (int)(((float)i + 0.5f) * inv_d); }

// ---------------------------------------------------------------------------
// k_pyr_cone: the whole cascade (levels 1..L-1, or s0+1..L-1 behind s0 k_resize levels) in ONE launch. Each workgroup owns a tile of
// the last level and the matching slice of every level (a partition per level); it recomputes
// in LDS the cone of each level its slices need (bit-exact: the same per-pixel INTER_LINEAR as
// k_resize, from the level below held in LDS, level 0 staged from the frame) and writes only its
// owned pixels. The redundant cone overlap (~1.3x the pyramid) costs far less than the 6
// dependent launch gaps of the per-level cascade at batch 1. Tables: ConeRect per (tile, level).
// ---------------------------------------------------------------------------
// LDS: [level 0 stage | level 1 .. L-1 cones] bytes, then per level the column table
// (xofs, xalpha) of its need columns and the row table (clamped r0, r1, ybeta) of its rows: one
// global round trip loads every table entry and the level-0 cone, then the levels follow from LDS.
__device__ __forceinline__ void wait_vm_all() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
// work-group barrier that orders LDS only: __syncthreads() also waits for every outstanding global
// access (s_waitcnt vmcnt(0)), so a level's byte stores to the pyramid would hold the barrier for
// their write acknowledgements although nothing in the work-group reads them back
__device__ __forceinline__ void lds_only_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

__device__ __forceinline__ void pyr_cone_body(const ExtractPlan* __restrict__ P, const FrameBufs& fb,
                                              const ConeRect* __restrict__ rects, const int* __restrict__ ctab,
                                              int tab_stride, uint8_t* __restrict__ cone, int tile, int f, int s0) {
    TR_BEGIN()
    const int L = P->n_levels, tid = threadIdx.x, nt = blockDim.x;
    const ConeRect* R = rects + (size_t)tile * kMaxLevels;
    // the tile's level rectangles (kMaxLevels x 16 bytes) as one dword per lane, read back by
    // readlane (uniform level index): read as int16 fields they compiled to a chain of dependent
    // global loads, one per level (~5k cycles before the staging loads were issued)
    static_assert(sizeof(ConeRect) == 16 && kMaxLevels * 4 <= 64 && (kMaxLevels & (kMaxLevels - 1)) == 0, "4 dwords per level");
    const uint32_t rdw = ((const uint32_t*)R)[threadIdx.x & (4 * kMaxLevels - 1)];
    auto rect = [&](int l) -> ConeRect {   // l wave-uniform
        const uint32_t d0 = (uint32_t)__builtin_amdgcn_readlane((int)rdw, 4 * l),
                       d1 = (uint32_t)__builtin_amdgcn_readlane((int)rdw, 4 * l + 1),
                       d2 = (uint32_t)__builtin_amdgcn_readlane((int)rdw, 4 * l + 2),
                       d3 = (uint32_t)__builtin_amdgcn_readlane((int)rdw, 4 * l + 3);
        return ConeRect{(int16_t)(d0 & 0xFFFF), (int16_t)(d0 >> 16), (int16_t)(d1 & 0xFFFF), (int16_t)(d1 >> 16),
                        (int16_t)(d2 & 0xFFFF), (int16_t)(d2 >> 16), (int16_t)(d3 & 0xFFFF), (int16_t)(d3 >> 16)};
    };
    int boff[kMaxLevels], toff[kMaxLevels];
    int tot = 0;
    // the source level s0 (0: the frame; s0 >= 1: a pyramid level written by k_resize) is staged
    // as aligned dwords: rows of P0 = round_up(width + 3, 4) bytes, the region starting at byte
    // sh0 of its row (sh0: the address misalignment, 0 on the byte path)
    const ConeRect Rs0 = rect(s0);
    const int P0 = (Rs0.nx1 - Rs0.nx0 + 6) & ~3;
    for (int l = s0; l < L; l++) {
        const ConeRect r = rect(l);
        boff[l] = tot;
        tot += ((l == s0 ? P0 : (r.nx1 - r.nx0)) * (r.ny1 - r.ny0) + 15) & ~15;
    }
    int sh0 = 0;
    int* tab = (int*)(cone + tot);
    int ttot = 0;
    for (int l = s0 + 1; l < L; l++) {
        toff[l] = ttot;
        const ConeRect r = rect(l);
        ttot += 2 * (r.nx1 - r.nx0) + 3 * (r.ny1 - r.ny0);
    }
    // staged table entry i (LDS layout: per level l > s0, xofs[nw] | xalpha[nw] | (r0, r1, beta)[nh]):
    // the host's per-tile copy (r05: computing the tables in the kernel, bit-exact, cut the cone's
    // HBM bytes 2.44 -> 1.98 MB per 640x480 launch but took the launch 21 -> 35 us in the 16-camera
    // stream: the per-level double-precision coefficients cost more than the table round trip)
    const int* gt = ctab + (size_t)tile * tab_stride;
    auto tab_at = [&](int i) -> int { return gt[i]; };
    TR_PHASE(0, 20)
    // ---- one round trip: the tile's tables of every level and its level-0 cone, all loads issued
    // before any store ----
    {
        const ImgRef in0 = level_img(P, fb, f, s0);
        const ConeRect r = Rs0;
        const int nw = r.nx1 - r.nx0, nh = r.ny1 - r.ny0;
        const uint8_t* src0 = in0.p + (int64_t)r.ny0 * in0.pitch + r.nx0;
        const bool dw = ((in0.pitch & 3) == 0) && ((((uintptr_t)in0.p) & 3) == 0);
        if (dw) sh0 = (int)(((uintptr_t)src0) & 3);
        const int nwd = dw ? (nw + sh0 + 3) >> 2 : 0;   // dwords per row (<= P0 / 4)
        const int tot0 = dw ? nwd * nh : nw * nh;
        const float inv_n = 1.0f / (float)(dw ? nwd : nw);
        uint8_t* lv0 = cone + boff[s0];
        if (dw && tot0 <= 1024 && ttot <= 2 * 1024 && nt == 1024) {
            const uint32_t* s4 = (const uint32_t*)(src0 - sh0);
            const int p4 = in0.pitch >> 2;
            int tv[2];
#pragma unroll
            for (int u = 0; u < 2; u++) tv[u] = gt[min(tid + 1024 * u, ttot - 1)];
            const int i = min(tid, tot0 - 1);
            const int y = small_div(i, inv_n), x = i - y * nwd;
            const uint32_t v = s4[(int64_t)y * p4 + x];
#pragma unroll
            for (int u = 0; u < 2; u++)
                if (tid + 1024 * u < ttot) tab[tid + 1024 * u] = tv[u];
            if (tid < tot0) ((uint32_t*)lv0)[y * (P0 >> 2) + x] = v;
            TR_PHASE(0, 21)
        } else if (dw) {
            // 8 loads per thread in flight before their stores (a load-store loop waits out one
            // global round trip per step)
            const uint32_t* s4 = (const uint32_t*)(src0 - sh0);
            const int p4 = in0.pitch >> 2;
            constexpr int U = 8;
            for (int i0 = tid; i0 < ttot; i0 += U * nt) {
                int v[U];
#pragma unroll
                for (int u = 0; u < U; u++) v[u] = tab_at(min(i0 + u * nt, ttot - 1));
#pragma unroll
                for (int u = 0; u < U; u++)
                    if (i0 + u * nt < ttot) tab[i0 + u * nt] = v[u];
            }
            for (int i0 = tid; i0 < tot0; i0 += U * nt) {
                uint32_t v[U];
                int o[U];
#pragma unroll
                for (int u = 0; u < U; u++) {
                    const int i = min(i0 + u * nt, tot0 - 1);
                    const int y = small_div(i, inv_n), x = i - y * nwd;
                    v[u] = s4[(int64_t)y * p4 + x];
                    o[u] = y * (P0 >> 2) + x;
                }
#pragma unroll
                for (int u = 0; u < U; u++)
                    if (i0 + u * nt < tot0) ((uint32_t*)lv0)[o[u]] = v[u];
            }
        } else {
            for (int i = tid; i < ttot; i += nt) tab[i] = tab_at(i);
            for (int i = tid; i < tot0; i += nt) {
                const int y = small_div(i, inv_n), x = i - y * nw;
                lv0[y * P0 + x] = src0[(int64_t)y * in0.pitch + x];
            }
        }
    }
    __syncthreads();
    TR_PHASE(0, 0)
    for (int l = s0 + 1; l < L; l++) {
        const LevelGeom& D = P->lv[l];
        const ConeRect r = rect(l), rp = rect(l - 1);
        const int nw = r.nx1 - r.nx0, nh = r.ny1 - r.ny0, nwp = l == s0 + 1 ? P0 : rp.nx1 - rp.nx0;
        const int* t = tab + toff[l];
        const uint8_t* src = cone + boff[l - 1] + (l == s0 + 1 ? sh0 : 0);
        uint8_t* dst = fb.pyr + (int64_t)f * P->pyr_bytes + D.pyr_off;
        const float inv_nw = 1.0f / (float)nw;
        const bool noclamp = D.rz_noclamp != 0;
        for (int i = tid; i < nw * nh; i += nt) {
            const int yy = small_div(i, inv_nw), xx = i - yy * nw;
            const int x = r.nx0 + xx, y = r.ny0 + yy;
            const int sx = t[xx] - rp.nx0;
            const uint8_t* S0 = src + (t[2 * nw + 3 * yy] - rp.ny0) * nwp;
            const uint8_t* S1 = src + (t[2 * nw + 3 * yy + 1] - rp.ny0) * nwp;
            int h0, h1;
            if (x < D.xmax) {
                const int aa = t[nw + xx];
                const int a0 = (int)(short)(aa & 0xFFFF), a1 = (int)(short)(aa >> 16);
                h0 = S0[sx] * a0 + S0[sx + 1] * a1;
                h1 = S1[sx] * a0 + S1[sx + 1] * a1;
            } else {
                h0 = S0[sx] * 2048;
                h1 = S1[sx] * 2048;
            }
            const int bb = t[2 * nw + 3 * yy + 2];
            const int b0 = (int)(short)(bb & 0xFFFF), b1 = (int)(short)(bb >> 16);
            int v;
            if (x < D.vend && noclamp) {   // as below; taps checked on the host (k_resize notes)
                v = ((__mul24(h0 >> 4, b0) >> 16) + (__mul24(h1 >> 4, b1) >> 16) + 2) >> 2;
            } else if (x < D.vend) {   // VResizeLinearVec_32s8u lanes (128-bit baseline)
                int s0 = min(max(h0 >> 4, -32768), 32767);
                int s1 = min(max(h1 >> 4, -32768), 32767);
                int tt = ((s0 * b0) >> 16) + ((s1 * b1) >> 16);
                tt = min(max(tt, -32768), 32767);
                v = (tt + 2) >> 2;
            } else {            // FixedPtCast<int, uchar, 22>
                v = (h0 * b0 + h1 * b1 + (1 << 21)) >> 22;
            }
            const uint8_t u = (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v));
            cone[boff[l] + i] = u;
            if (x >= r.ox0 && x < r.ox1 && y >= r.oy0 && y < r.oy1) dst[(int64_t)y * D.pitch + x] = u;
        }
        lds_only_barrier();   // the next level reads this one's LDS cone; the stores stay in flight
        TR_PHASE(0, l)
    }
    TR_END(0)
}

__global__ __launch_bounds__(1024) void k_pyr_cone(const ExtractPlan* __restrict__ P, FrameBufs fb,
                                                   const ConeRect* __restrict__ rects, const int* __restrict__ ctab,
                                                   int tab_stride, int xrun, int s0) {
    extern __shared__ __attribute__((aligned(16))) uint8_t cone[];
    if (fb.stamp && threadIdx.x == 0) atomicMin(fb.stamp, (unsigned long long)__builtin_amdgcn_s_memrealtime());
    const int X = gridDim.x, lg = xcd_runs(blockIdx.x + X * blockIdx.y, X * gridDim.y, xrun < 0 ? X : xrun);
    pyr_cone_body(P, fb, rects, ctab, tab_stride, cone, lg % X, lg / X, s0);
    if (fb.stamp) {   // the workgroup's end: every wave's stores drained (the barrier waits on them)
        __syncthreads();
        if (threadIdx.x == 0) atomicMax(fb.stamp + kStampStride, (unsigned long long)__builtin_amdgcn_s_memrealtime());
    }
}

// ---------------------------------------------------------------------------
// k_fast_cells: one workgroup per (cell, frame)
// FAST strength m = max(A, B, 0): A = max over the 16 9-arcs of min(v - p), B the same for
// (p - v). cornerScore<16> == m - 1 for every detected corner and a pixel is a corner at
// threshold t iff m > t (derivation in DESIGN.md), so one map serves both thresholds.
//
// The window sits in LDS as a "pair window" of f16 pairs: dword (r, c) holds 1024 + the pixel of
// window row r (low half) and of row r + R (high half), R = ceil(dr / 2) the pixel rows of the
// cell's top half. One ds_read_b32 at a circle offset then gives the circle value of a top-half
// pixel and of the pixel R rows below it, already packed for the v_pk_*_f16 ops; the 3-input
// v_pk_minimum3 / v_pk_maximum3 halve the arc networks. 1024 + v (v = 0..255, sums with t up to
// 1534) is an exact f16 integer, so every min / max / difference is exact.
// ---------------------------------------------------------------------------
constexpr int kWinMax = 80;
#ifndef ORBHIP_OCT_W0_MAIN
#define ORBHIP_OCT_W0_MAIN 1   // r05: the octree's MAIN rounds of short lists in wave 0 alone (0: the block loop)
#endif
#ifndef ORBHIP_OCT_BLK_FINAL
// r05: FINAL passes of lists of <= threads nodes by the whole block (block scans) instead of wave 0.
// A/B (profiles/r05_octree_blkfinal_ab.log, three alternating runs): octree stage 13.84-14.08 against
// 14.01-14.16 us, the stream 43.3-44.2k against 42.8-44.2k frames/s: the block's barriers cost about
// what wave 0's serial LDS round trips did
#define ORBHIP_OCT_BLK_FINAL 1
#endif
typedef _Float16 h2 __attribute__((ext_vector_type(2)));   // two pixels, one per 16-bit half
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
constexpr uint32_t kPwBias = 0x64006400u;                   // f16(1024) in both halves

__device__ __forceinline__ h2 as_h2(uint32_t u) { return __builtin_bit_cast(h2, u); }
__device__ __forceinline__ h2 hmin(h2 a, h2 b) { return __builtin_elementwise_minimum(a, b); }
__device__ __forceinline__ h2 hmax(h2 a, h2 b) { return __builtin_elementwise_maximum(a, b); }

// circle offsets (dwords) from the circle's top-left corner (the pixel at (-3, -3)), row pitch P:
// the 16 points of OpenCV's pattern in its order, then the centre
template <int P>
struct Circle {
    static constexpr int o[17] = {6 * P + 3, 6 * P + 4, 5 * P + 5, 4 * P + 6, 3 * P + 6, 2 * P + 6,
                                  P + 5,     4,         3,         2,         P + 1,     2 * P,
                                  3 * P,     4 * P,     5 * P + 1, 6 * P + 2, 3 * P + 3};
};

// LDS of one FAST cell, sized for windows of up to WR rows. Compact variant (WR 50): windows of
// <= 50 rows and <= 45 columns (every level of 640x480 and 1280x720), ~9.7 KB, 16 work-groups
// of 128 threads per CU. Full variant: any cell (windows up to 80 x 80).
template <int WR>
struct FastShape {
    static constexpr bool full = WR >= kWinMax;
    static constexpr int wmax = full ? kWinMax : 45;        // window columns
    // pair-window row pitch (dwords): 48 / 84. (r06 A/B: 68, which is the cells' dc = 36 mod 32, so
    // that each half-wave of the pair test reads 32 consecutive banks, took k_fast_cells at C3 0.353
    // -> 0.41 ms: the larger window costs work-groups per CU)
    static constexpr int pwp = ((wmax + 3 + 3) / 4) * 4;
    static constexpr int pwr = (WR - 6 + 1) / 2 + 6;         // pair-window rows: 28 / 43
    static constexpr int mp = full ? 80 : 48;                // strength map row pitch (bytes) >= dc + 2
    static constexpr int mr = WR - 4;                        // strength map rows dr + 2
    static constexpr int nw = ((WR - 6) * (wmax - 6) + 63) / 64;   // mask words of the largest cell
    static constexpr int cap = full ? kClistCap : 768;       // survivor list entries
    static_assert(mp % 4 == 0 && mp >= wmax - 4, "strength map rows");
};
struct FastLds {
    uint32_t* pw;                   // pair window
    uint8_t* mv;                    // strength map (zero border)
    unsigned long long* bmask;      // [2][nw] NMS survivors per threshold, raster order
    int nw;
    int* woff;                      // [nw] output offset of each 64-px word
    int* wsel;
    int* wtot;
    uint16_t* clist;                // pair-test survivors (strength to compute), one region per wave
    int* ncand;
    int* ncw;                       // [NT / 64] survivors listed by each wave
    int cap;                        // clist entries in use: min(plan's clist_cap, the variant's)
};

template <int NT, int PWP, int MP, int PWR>
__device__ __forceinline__ void fast_cell_body(const ExtractPlan* __restrict__ P, const CellGeom* __restrict__ cells,
                                               const FrameBufs& fb, uint32_t* __restrict__ cand,
                                               int* __restrict__ cand_cnt, int* __restrict__ err, int cell, int f,
                                               const FastLds& LS, const CandPack& cp) {
    uint32_t* const pw = LS.pw;
    uint8_t* const mv = LS.mv;
    unsigned long long* const bm0 = LS.bmask;
    unsigned long long* const bm1 = LS.bmask + LS.nw;
    int* const woff = LS.woff;
    int& wsel = *LS.wsel;
    int& wtot = *LS.wtot;
    uint16_t* const clist = LS.clist;
    int& ncand = *LS.ncand;
    TR_BEGIN()
    const CellGeom cg = cells[cell];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wc = cg.wc, hc = cg.hc;
    int* cnt_out = cand_cnt + (int64_t)f * P->n_cells_total + cell;
    // the error words of the extraction: cleared here, set by the octree (next launch)
    if (cell == 0 && f == 0 && tid < 4) __hip_atomic_store(&err[tid], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (wc <= 6 || hc <= 6) {
        if (tid == 0) {
            *cnt_out = 0;
            if (cp.off) cp.off[(int64_t)f * P->n_cells_total + cell] = 0;
        }
        return;
    }
    const LevelGeom& G = P->lv[cg.level];
    ImgRef im = level_img(P, fb, f, cg.level);
    const uint8_t* base = im.p + (int64_t)cg.y0 * im.pitch + cg.x0;
    const int dc = wc - 6, dr = hc - 6, np = dc * dr;
    const int R = (dr + 1) >> 1;   // top-half pixel rows; pair-window rows R + 6
    const int RW = R + 6;
    // ---- window -> pair window: all loads of a thread issued back to back. When the rows are
    // 4-byte aligned (pyramid levels always; the caller's frame when its pointer and stride are),
    // a task moves one aligned dword of window rows r and r + R (4 pixels each) into 4 pair-window
    // dwords (one ds_write_b128), columns shifted by sh = base & 3 ----
    int sh = 0;
    {
        const bool dw = ((im.pitch & 3) == 0) && ((((uintptr_t)im.p) & 3) == 0);
        if (dw) {
            sh = (int)(((uintptr_t)base) & 3);
            const uint32_t* b4 = (const uint32_t*)(base - sh);
            const int nwd = (wc + sh + 3) >> 2;   // <= PWP / 4
            const int p4 = im.pitch >> 2;
            auto put = [&](int r, int j, uint32_t a, uint32_t b) {
                uint4 o;
                o.x = __builtin_amdgcn_perm(b, a, 0x0C040C00u) | kPwBias;
                o.y = __builtin_amdgcn_perm(b, a, 0x0C050C01u) | kPwBias;
                o.z = __builtin_amdgcn_perm(b, a, 0x0C060C02u) | kPwBias;
                o.w = __builtin_amdgcn_perm(b, a, 0x0C070C03u) | kPwBias;
                *(uint4*)(pw + r * PWP + 4 * j) = o;
            };
            // threads on a (row, dword column) grid, no division: JC columns per row (>= the
            // window's dwords), NT / JC rows per pass, every pass's loads in flight together
            constexpr int JC = (PWP / 4 <= 16) ? 16 : 32;
            constexpr int RP = NT / JC;
            constexpr int NP = (PWR + RP - 1) / RP;
            const int j = tid % JC, r0 = tid / JC;
            uint32_t va[NP], vb[NP];
#pragma unroll
            for (int u = 0; u < NP; u++) {
                const int r = r0 + RP * u;
                const bool ok = r < RW && j < nwd;
                va[u] = ok ? b4[(int64_t)r * p4 + j] : 0u;
                vb[u] = ok && r + R < hc ? b4[(int64_t)(r + R) * p4 + j] : 0u;
            }
#pragma unroll
            for (int u = 0; u < NP; u++) {
                const int r = r0 + RP * u;
                if (r < RW && j < nwd) put(r, j, va[u], vb[u]);
            }
        } else {
            const int tot = wc * RW;
            const float inv_wc = 1.0f / (float)wc;
            for (int i = tid; i < tot; i += NT) {
                const int r = small_div(i, inv_wc), c = i - r * wc;
                const uint32_t a = base[(int64_t)r * im.pitch + c];
                const uint32_t b = r + R < hc ? base[(int64_t)(r + R) * im.pitch + c] : 0u;
                pw[r * PWP + c] = kPwBias | a | (b << 16);
            }
        }
    }
    // the strength map starts all zero (border, and every pixel the pair test rejects)
    {
        uint32_t* m4 = (uint32_t*)mv;
        const int n4 = (dr + 2) * (MP / 4);
        for (int i = tid; i < n4; i += NT) m4[i] = 0u;
    }
    for (int i = tid; i < 2 * LS.nw; i += NT) LS.bmask[i] = 0ull;
    __syncthreads();
    TR_PHASE(1, 0)
    const int t_ini = P->ini_th, t_min = P->min_th;
    const int t_lo = min(t_ini, t_min);
    const float inv_dc = 1.0f / (float)dc;
    // a threshold >= 255 passes no pixel, as 255 does (|v - c| <= 255); keeps every sum exact
    const _Float16 th = (_Float16)max(min(t_lo, 255), -255);
    const h2 tv = {th, th};
    constexpr int MPc = MP;
    using C = Circle<PWP>;
    const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    const int clist_cap = LS.cap;
    // every pixel pair (q: top half, q + R dc: the pixel R rows below) runs the cheap
    // opposite-pair test; the ~5-10% that pass are compacted into clist, and the strength (the
    // expensive part) runs on the dense list, so no wave spends its issue slots on masked-off
    // lanes. In circle values c: bright iff min_k max(c_k, c_k+8) > v + t, dark iff
    // v > max_k min(c_k, c_k+8) + t.
    // Each wave lists its survivors in its own region of clist (capw entries) with a running
    // count, so no list position waits on an LDS atomic. q advances by NT per round: (y, x) are
    // stepped, not divided.
    constexpr int NW = NT / 64;
    const int capw = clist_cap / NW;
    uint16_t* const wlist = clist + wid * capw;
    int wcnt = 0;   // wave-uniform
    const int nq = R * dc, qb = R * dc;
    const int ystep = NT / dc, xstep = NT - ystep * dc;
    int y = small_div(tid, inv_dc), x = tid - y * dc;
    // r05: the round without a branch (a lane past the last pixel reads a clamped row and passes
    // nothing), the list positions by mbcnt, the capacity checked once per wave and round
    (void)lt;
    for (int q0 = 0; q0 < nq; q0 += NT) {
        const int q = q0 + tid;
        const bool in = q < nq;
        const uint32_t* c = pw + min(y, R - 1) * PWP + x + sh;
        h2 cc[16];
#pragma unroll
        for (int k = 0; k < 16; k++) cc[k] = as_h2(c[C::o[k]]);
        const h2 v = as_h2(c[C::o[16]]);
        h2 M1 = hmax(cc[0], cc[8]), M2 = hmin(cc[0], cc[8]);
#pragma unroll
        for (int k = 1; k < 8; k++) {
            M1 = hmin(M1, hmax(cc[k], cc[k + 8]));
            M2 = hmax(M2, hmin(cc[k], cc[k + 8]));
        }
        const h2 s = hmax(M1 - (v + tv), v - (M2 + tv));   // > 0: passes (exact integers)
        const bool pass0 = in & (s.x > (_Float16)0);
        const bool pass1 = in & (y + R < dr) & (s.y > (_Float16)0);
        // the compare masks as they are (HIP's __ballot(int) makes a lane value of each and compares
        // it again)
        const uint64_t b0 = __builtin_amdgcn_ballot_w64(pass0), b1 = __builtin_amdgcn_ballot_w64(pass1);
        const int n0 = __popcll(b0), n1 = __popcll(b1);
        const int ci0 = wcnt + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(b0 >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)b0, 0u));
        const int ci1 = wcnt + n0 + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(b1 >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)b1, 0u));
        if (wcnt + n0 + n1 <= capw) {   // wave-uniform: the round's survivors all fit
            if (pass0) wlist[ci0] = (uint16_t)q;
            if (pass1) wlist[ci1] = (uint16_t)(q + qb);
        } else {
            if (pass0 && ci0 < capw) wlist[ci0] = (uint16_t)q;
            if (pass1 && ci1 < capw) wlist[ci1] = (uint16_t)(q + qb);
        }
        wcnt += n0 + n1;
        x += xstep;
        y += ystep;
        if (x >= dc) { x -= dc; y++; }
    }
    if (lane == 0) LS.ncw[wid] = wcnt;
    __syncthreads();
    // dense: a wave's list overflowed, so the strength runs on every pixel instead (m <= t_lo for
    // every pixel the pair test rejects, so the map is the same) and the NMS walks every pixel.
    // Otherwise survivor i (in wave order) sits at i + the unused tails of the regions before it.
    int pre[NW], gap[NW];
    bool dense = false;
    int nc = 0;
#pragma unroll
    for (int w = 0; w < NW; w++) {
        const int cw = LS.ncw[w];
        pre[w] = nc;
        gap[w] = capw - cw;
        dense |= cw > capw;
        nc += cw;
    }
    if (dense) nc = np;
    auto surv = [&](int i) -> int {
        if (dense) return i;
        int o = i;
#pragma unroll
        for (int w = 1; w < NW; w++) o += i >= pre[w] ? gap[w - 1] : 0;
        return clist[o];
    };
    {
        // two pixels per lane (i and i + hn) as the halves of one f16 pair, each read from its
        // pair-window half and joined by one v_perm per circle point:
        // m = max(v - min over 9-arcs of the arc max, max over 9-arcs of the arc min - v, 0), the
        // 9-arc extrema as 3-input ops over 3-arcs
        const int hn = (nc + 1) >> 1;
        for (int i = tid; i < hn; i += NT) {
            const bool two = i + hn < nc;
            const int pa = surv(i);
            const int pb = two ? surv(i + hn) : pa;
            const int ya = small_div(pa, inv_dc), xa = pa - ya * dc;
            const int yb = small_div(pb, inv_dc), xb = pb - yb * dc;
            const bool ha = ya >= R, hb = yb >= R;
            const uint32_t* ca = pw + (ha ? ya - R : ya) * PWP + xa + sh;
            const uint32_t* cb = pw + (hb ? yb - R : yb) * PWP + xb + sh;
            const uint32_t sel = (ha ? 0x0302u : 0x0100u) | ((hb ? 0x0706u : 0x0504u) << 16);
            h2 c[16];
#pragma unroll
            for (int k = 0; k < 16; k++) c[k] = as_h2(__builtin_amdgcn_perm(cb[C::o[k]], ca[C::o[k]], sel));
            const h2 v = as_h2(__builtin_amdgcn_perm(cb[C::o[16]], ca[C::o[16]], sel));
            // one network at a time (mins, then maxes): 16 3-arc registers live
            auto arc9 = [&](auto op, auto fold) {
                h2 u[16];
#pragma unroll
                for (int k = 0; k < 16; k++) u[k] = op(op(c[k], c[(k + 1) & 15]), c[(k + 2) & 15]);   // 3-arcs
                h2 r = op(op(u[0], u[3]), u[6]);
#pragma unroll
                for (int k = 1; k < 16; k++) r = fold(r, op(op(u[k], u[(k + 3) & 15]), u[(k + 6) & 15]));   // 9-arcs
                return r;
            };
            const h2 Mm = arc9(hmin, hmax);   // max over arcs of the arc min
            const h2 MM = arc9(hmax, hmin);   // min over arcs of the arc max
            const h2 zero = {(_Float16)0, (_Float16)0};
            const h2 m2 = hmax(hmax(v - MM, Mm - v), zero);
            const int ma = (int)m2.x, mb = (int)m2.y;
            mv[(ya + 1) * MPc + xa + 1] = (uint8_t)(ma > t_lo ? ma : 0);
            if (two) mv[(yb + 1) * MPc + xb + 1] = (uint8_t)(mb > t_lo ? mb : 0);
        }
    }
    __syncthreads();
    TR_PHASE(1, 1)
    // ---- window-local strict 3x3 NMS at both thresholds, on the surviving pixels only; the
    // results are bits of a raster-order mask per threshold ----
    for (int i = tid; i < nc; i += NT) {
        const int p = surv(i);
        const int py = small_div(p, inv_dc), px = p - py * dc;
        const uint8_t* c = &mv[(py + 1) * MPc + px + 1];
        const int m = c[0];
        if (m == 0) continue;
        const int nb[8] = {c[-MPc - 1], c[-MPc], c[-MPc + 1], c[-1], c[1], c[MPc - 1], c[MPc], c[MPc + 1]};
        bool k_ini = m > t_ini, k_min = m > t_min;
#pragma unroll
        for (int k = 0; k < 8; k++) {
            const int mq = nb[k];
            k_ini &= (m - 1) > (mq > t_ini ? mq - 1 : 0);
            k_min &= (m - 1) > (mq > t_min ? mq - 1 : 0);
        }
        const unsigned long long bit = 1ull << (p & 63);
        if (k_ini) atomicOr(&bm0[p >> 6], bit);
        if (k_min) atomicOr(&bm1[p >> 6], bit);
    }
    __syncthreads();
    TR_PHASE(1, 2)
    // ---- per-cell fallback iniThFAST -> minThFAST, then the ordered compaction ----
    const int nwd = (np + 63) >> 6;
    if (wid == 0) {
        int ci = 0;
        for (int w = lane; w < nwd; w += 64) ci += __popcll(bm0[w]);
        const int tot_ini = wave_sum_i32(ci);
        const int sel = tot_ini > 0 ? 0 : 1;
        const unsigned long long* bs = sel ? bm1 : bm0;
        // exclusive scan of the selected mask's word popcounts (2 words per lane: nwd <= 128)
        const int w0 = 2 * lane, w1 = 2 * lane + 1;
        const int c0 = w0 < nwd ? __popcll(bs[w0]) : 0, c1 = w1 < nwd ? __popcll(bs[w1]) : 0;
        const int inc = wave_incl_scan(c0 + c1);
        if (w0 < nwd) woff[w0] = inc - c0 - c1;
        if (w1 < nwd) woff[w1] = inc - c1;
        if (lane == 63) { wsel = sel; wtot = inc; }
    }
    __syncthreads();
    const int sel = wsel;
    int slot = cg.slot_off;
    if (cp.off) {
        // packed candidates (batches): the cell's run goes to the next free range of its level's
        // region (one atomic per cell), so the octree's reads cover whole lines instead of a line
        // per sparse cell; the run's frame offset goes to cp.off. ncand is free again here
        if (tid == 0) {
            int b = wtot ? atomicAdd(&cp.fill[f * kMaxLevels + cg.level], wtot) : 0;
            if (b + wtot > G.n_slots) {   // never expected (a level's cells cannot exceed its slots)
                atomicOr(err, 4);
                b = -1;
            }
            ncand = b;
            cp.off[(int64_t)f * P->n_cells_total + cell] = b < 0 ? 0 : G.slot_base + b;
        }
        __syncthreads();
        if (ncand < 0) {
            if (tid == 0) *cnt_out = 0;
            return;
        }
        slot = G.slot_base + ncand;
    }
    uint32_t* out = cand + (int64_t)f * P->n_slots_total + slot;
    // primary slots (fixed ranges): the cell's first kCandPrim candidates sit next to the other
    // cells' (16 per cell, cell-major), so the octree reads them as whole lines
    uint32_t* const prim = (cp.prim && !cp.off) ? cp.prim + ((int64_t)f * P->n_cells_total + cell) * kCandPrim : nullptr;
    // one lane per mask word walks its set bits (a cell keeps a few corners: ~1 per word), in
    // raster order from the word's scanned offset
    for (int w = tid; w < nwd; w += NT) {
        uint64_t mk = (sel ? bm1 : bm0)[w];
        int o = woff[w];
        while (mk) {
            const int p = 64 * w + __builtin_ctzll(mk);
            mk &= mk - 1;
            const int py = small_div(p, inv_dc), px = p - py * dc;
            const int x = cg.x0 + 3 + px - G.min_bx, y = cg.y0 + 3 + py - G.min_by;
            const uint32_t v = pack_cand(x, y, (int)mv[(py + 1) * MPc + px + 1] - 1);
            if (prim && o < kCandPrim) prim[o] = v;
            else out[o] = v;
            o++;
        }
    }
    if (tid == 0) *cnt_out = wtot;
    TR_PHASE(1, 3)
    TR_END(1)
}

template <int NT, int WR>
__global__ __launch_bounds__(NT) void k_fast_cells(const ExtractPlan* __restrict__ P,
                                                    const CellGeom* __restrict__ cells, FrameBufs fb,
                                                    uint32_t* __restrict__ cand, int* __restrict__ cand_cnt,
                                                    int* __restrict__ err, int xrun, CandPack cp) {
    using SH = FastShape<WR>;
    __shared__ __attribute__((aligned(16))) uint32_t pw[SH::pwr * SH::pwp];
    __shared__ __attribute__((aligned(16))) uint8_t mv[SH::mr * SH::mp];
    __shared__ unsigned long long bmask[2 * SH::nw];
    __shared__ int woff[SH::nw];
    __shared__ int wsel, wtot;
    __shared__ uint16_t clist[SH::cap];
    __shared__ int ncand;
    __shared__ int ncw[NT / 64];
    const FastLds LS{pw, mv, bmask, SH::nw, woff, &wsel, &wtot, clist, &ncand, ncw, min(P->clist_cap, SH::cap)};
    const int X = gridDim.x, lg = xcd_runs(blockIdx.x + X * blockIdx.y, X * gridDim.y, xrun < 0 ? X : xrun);
    fast_cell_body<NT, SH::pwp, SH::mp, SH::pwr>(P, cells, fb, cand, cand_cnt, err, lg % X, lg / X, LS, cp);
}

// ---------------------------------------------------------------------------
// k_octree: DistributeOctTree for one (level, frame). All node state in LDS; keys in LDS
// when they fit (flat pointers otherwise point at per-level global scratch).
// ---------------------------------------------------------------------------
struct OctLds {
    int* ctl;          // 64 ints: scan scratch / control words
    uint64_t* rectA; uint32_t* cntA; uint32_t* bestA; uint32_t* serA;
    uint64_t* rectB; uint32_t* cntB; uint32_t* bestB; uint32_t* serB;
    uint32_t* ccount;  // node_cap*4 child counts
    uint32_t* cbest;   // node_cap*4 child best (score<<24 | 0xFFFFFF-key)
    uint16_t* map4;    // node_cap*4 remap old node/quadrant -> new node
    int* tA; int* tB; int* tC; int* tD;
    uint64_t* skey;    // sort keys (sort_cap)
    uint64_t* skey2;   // rank-sorted keys (sort_cap)
    int* cellstart;    // max_cells_level + 1
    int* cslot;        // max_cells_level + 1: candidate slot offset of each cell
    uint32_t* keys;    // key_cap (LDS) or null
    uint16_t* knode;
};

__device__ __forceinline__ uint64_t mk_rect(int x0, int y0, int x1, int y1) {
    return (uint64_t)(uint16_t)x0 | ((uint64_t)(uint16_t)y0 << 16) | ((uint64_t)(uint16_t)x1 << 32) |
           ((uint64_t)(uint16_t)y1 << 48);
}
__device__ __forceinline__ int rx0(uint64_t r) { return (int)(r & 0xFFFF); }
__device__ __forceinline__ int ry0(uint64_t r) { return (int)((r >> 16) & 0xFFFF); }
__device__ __forceinline__ int rx1(uint64_t r) { return (int)((r >> 32) & 0xFFFF); }
__device__ __forceinline__ int ry1(uint64_t r) { return (int)(r >> 48); }

// ExtractorNode::DivideNode split: halfX = ceil((UR.x-UL.x)/2.f), halfY = ceil((BR.y-UL.y)/2.f)
__device__ __forceinline__ void split_of(uint64_t r, int* sx, int* sy) {
    *sx = rx0(r) + (int)ceilf((float)(rx1(r) - rx0(r)) / 2);
    *sy = ry0(r) + (int)ceilf((float)(ry1(r) - ry0(r)) / 2);
}
__device__ __forceinline__ int quad_of(uint64_t r, int x, int y) {
    int sx, sy;
    split_of(r, &sx, &sy);
    return (x >= sx ? 1 : 0) + (y >= sy ? 2 : 0);
}
__device__ __forceinline__ uint64_t child_rect(uint64_t r, int q) {
    int sx, sy;
    split_of(r, &sx, &sy);
    const int x0 = rx0(r), y0 = ry0(r), x1 = rx1(r), y1 = ry1(r);
    switch (q) {
        case 0: return mk_rect(x0, y0, sx, sy);
        case 1: return mk_rect(sx, y0, x1, sy);
        case 2: return mk_rect(x0, sy, sx, y1);
        default: return mk_rect(sx, sy, x1, y1);
    }
}
__device__ __forceinline__ uint32_t pack_best(int score, int k) { return ((uint32_t)score << 24) | (0xFFFFFFu - (uint32_t)k); }

// In-place exclusive scan of arr[0..n) by the whole block; returns the total. arr in LDS.
__device__ int block_scan_array(int* arr, int n, int* ctl) {
    const int nt = blockDim.x, tid = threadIdx.x;
    const int per = (n + nt - 1) / nt;
    const int b = tid * per, e = min(b + per, n);
    int s = 0;
    for (int i = b; i < e; i++) s += arr[i];
    int tot;
    int off = block_excl_scan(s, ctl, &tot);
    for (int i = b; i < e; i++) { int v = arr[i]; arr[i] = off; off += v; }
    __syncthreads();
    return tot;
}
// Three exclusive scans in one pass (2 barriers): arrays a0..a2 of length n each; scratch =
// ctl[0..47] (16 waves x 3). Returns the totals.
__device__ void block_scan_array3(int* a0, int* a1, int* a2, int n, int* ctl, int* tot) {
    const int nt = blockDim.x, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, nw = nt >> 6;
    const int per = (n + nt - 1) / nt;
    const int b = tid * per, e = min(b + per, n);
    int* arr[3] = {a0, a1, a2};
    int s[3] = {0, 0, 0}, inc[3];
#pragma unroll
    for (int k = 0; k < 3; k++) {
        for (int i = b; i < e; i++) s[k] += arr[k][i];
        inc[k] = wave_incl_scan(s[k]);
        if (lane == 63) ctl[16 * k + wid] = inc[k];
    }
    __syncthreads();
    int off[3];
#pragma unroll
    for (int k = 0; k < 3; k++) {
        const int ws = wave_incl_scan(lane < nw ? ctl[16 * k + lane] : 0);
        const int before = __builtin_amdgcn_readlane(ws, wid > 0 ? wid - 1 : 0);
        tot[k] = __builtin_amdgcn_readlane(ws, nw - 1);
        off[k] = (wid > 0 ? before : 0) + inc[k] - s[k];
    }
#pragma unroll
    for (int k = 0; k < 3; k++)
        for (int i = b; i < e; i++) { const int v = arr[k][i]; arr[k][i] = off[k]; off[k] += v; }
    __syncthreads();
}
// Descending sort of n unique keys by rank: out[#greater] = key. Four threads per key (a quad)
// each count a quarter of the keys, two ds_read_b128 per step; the quad sums by DPP.
__device__ void block_rank_sort_desc(const uint64_t* __restrict__ a, uint64_t* __restrict__ out, int n) {
    const int q = threadIdx.x & 3, nq = blockDim.x >> 2;
    const int per = (((n + 3) >> 2) + 1) & ~1;   // even: pairs of keys per 16-byte read
    const int j0 = min(q * per, n), j1 = min(j0 + per, n);
    for (int i0 = 0; i0 < n; i0 += nq) {
        const int i = i0 + (threadIdx.x >> 2);
        const uint64_t x = i < n ? a[i] : ~0ull;
        int r = 0;
        int j = j0;
        for (; j + 1 < j1; j += 2) {
            const ulonglong2 v = *(const ulonglong2*)(a + j);
            r += (v.x > x ? 1 : 0) + (v.y > x ? 1 : 0);
        }
        if (j < j1) r += a[j] > x ? 1 : 0;
        r += __builtin_amdgcn_update_dpp(0, r, 0xB1, 0xF, 0xF, false);   // quad_perm [1,0,3,2]
        r += __builtin_amdgcn_update_dpp(0, r, 0x4E, 0xF, 0xF, false);   // quad_perm [2,3,0,1]
        if (q == 0 && i < n) out[r] = x;
    }
    __syncthreads();
}

// cnt[tgt] += 1 for every lane with tgt != ~0u. Lanes form runs of equal tgt (keys are
// cell-major, so neighbouring lanes mostly share a node); each run head adds the run length
// (distance to the next head, from one ballot) with ONE LDS atomic — same-address atomics
// would otherwise serialise lane by lane. The neighbour compare is a DPP wave_shr:1 move.
__device__ __forceinline__ void wave_aggregate_count(uint32_t tgt, uint32_t* cnt) {
    const int lane = threadIdx.x & 63;
    const uint32_t prev = (uint32_t)__builtin_amdgcn_update_dpp((int)~tgt, (int)tgt, 0x138, 0xF, 0xF, false);
    const bool head = prev != tgt;   // lane 0 receives ~tgt
    const uint64_t heads = __ballot(head);
    if (head && tgt != 0xFFFFFFFFu) {
        const uint64_t above = lane == 63 ? 0ull : (heads & (~0ull << (lane + 1)));
        const int next = above ? __ffsll((unsigned long long)above) - 1 : 64;
        atomicAdd(&cnt[tgt], (uint32_t)(next - lane));
    }
}

constexpr int kOctKR = 8;    // keys per thread kept in registers through the division (M <= 8 x 1024)


// In-place exclusive scan of arr[0..n) in LDS by ONE wave (a contiguous range per lane, DPP wave
// scan of the range sums). Returns the total (uniform). No block barrier.
__device__ int wave_scan_lds(int* arr, int n) {
    const int lane = threadIdx.x & 63;
    const int per = (n + 63) >> 6;
    const int b = min(lane * per, n), e = min(b + per, n);
    int s = 0;
    for (int i = b; i < e; i++) s += arr[i];
    const int inc = wave_incl_scan(s);
    const int tot = __builtin_amdgcn_readlane(inc, 63);
    int off = inc - s;
    for (int i = b; i < e; i++) { const int v = arr[i]; arr[i] = off; off += v; }
    wave_lds_fence();
    return tot;
}

__device__ __forceinline__ int nonempty4(const uint32_t* c) { return (c[0] > 0) + (c[1] > 0) + (c[2] > 0) + (c[3] > 0); }
__device__ __forceinline__ int multi4(const uint32_t* c) { return (c[0] > 1) + (c[1] > 1) + (c[2] > 1) + (c[3] > 1); }

// Two division engines, one node list logic (MAIN / FINAL passes in wave 0, the block rank sort):
//  - pyramid path (cfg.fast, tried first): every key's quadrant path is fixed by geometry alone (a
//    node's split lines depend only on its rectangle), so one pass over the keys histograms their
//    depth-Dh cells (count + max (response, -key index, key)) and a reduction builds the counts and
//    retained keys of every shallower cell. A node is (depth, path) and its children's counts are
//    pyramid reads, so a division round touches no key: no sweep and one block barrier. A node
//    with > 1 key at depth Dh (its children are deeper than the pyramid) sends the level to
//    the sweep path, from scratch.
//  - sweep path: nodes are rectangles, each round remaps every key to its node and counts the
//    children (run-aggregated LDS atomics), then wave 0 runs the node pass. A MAIN round is 2
//    block barriers, a FINAL round 4.
// Node pass work (children counts, positions, serials, the largest-first selection of the FINAL
// pass) runs in wave 0 alone with DPP wave scans over a few nodes per lane.
constexpr int kOctMaxDh = 6;

__global__ __launch_bounds__(1024) void k_octree(const ExtractPlan* __restrict__ P, const CellGeom* __restrict__ cells,
                                                 const uint16_t* __restrict__ otab, const uint32_t* __restrict__ cand,
                                                 const uint32_t* __restrict__ cprim, const int* __restrict__ cand_cnt,
                                                 const int* __restrict__ cand_off,
                                                 uint32_t* __restrict__ kscratch, uint16_t* __restrict__ nscratch,
                                                 LevelKp* __restrict__ lvl_kp, int* __restrict__ lvl_cnt,
                                                 int* __restrict__ lvl_nlap, OctreeCfg cfg, int* __restrict__ err,
                                                 unsigned long long* __restrict__ stamp) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    TR_BEGIN()
    // live timing (stage timer): the earliest workgroup start, the latest end (FrameBufs::stamp)
    if (stamp && threadIdx.x == 0) atomicMin(stamp, (unsigned long long)__builtin_amdgcn_s_memrealtime());
    auto stamp_end = [&]() {
        if (!stamp) return;
        __syncthreads();   // every wave's stores drained
        if (threadIdx.x == 0) atomicMax(stamp + kStampStride, (unsigned long long)__builtin_amdgcn_s_memrealtime());
    };
    // grid (frame, level): the level-0 work-groups (the longest) of every frame dispatch first
    const int f = blockIdx.x, l = blockIdx.y;
    const LevelGeom& G = P->lv[l];
    const int tid = threadIdx.x, nt = blockDim.x, lane = tid & 63;
    const bool w0 = tid < 64;
    const int NC = cfg.node_cap;
    // ---- carve LDS (every offset a multiple of 16 bytes) ----
    OctLds S;
    size_t off = 0;
    auto carve = [&](size_t bytes) { void* p = smem + off; off += (bytes + 15) & ~size_t(15); return p; };
    S.ctl = (int*)carve(64 * 4);
    S.rectA = (uint64_t*)carve(NC * 8); S.cntA = (uint32_t*)carve(NC * 4);
    S.bestA = (uint32_t*)carve(NC * 4); S.serA = (uint32_t*)carve(NC * 4);
    S.rectB = (uint64_t*)carve(NC * 8); S.cntB = (uint32_t*)carve(NC * 4);
    S.bestB = (uint32_t*)carve(NC * 4); S.serB = (uint32_t*)carve(NC * 4);
    S.ccount = (uint32_t*)carve(NC * 16); S.cbest = (uint32_t*)carve(NC * 16);
    S.map4 = (uint16_t*)carve(NC * 8);
    S.tA = (int*)carve(NC * 4); S.tB = (int*)carve(NC * 4); S.tC = (int*)carve(NC * 4);
    S.tD = (int*)carve(NC * 4);
    S.skey = (uint64_t*)carve(cfg.sort_cap * 8);
    S.skey2 = (uint64_t*)carve(cfg.sort_cap * 8);
    S.cellstart = (int*)carve((P->max_cells_level + 1) * 4);
    S.cslot = (int*)carve((P->max_cells_level + 1) * 4);
    uint32_t* keysL = (uint32_t*)carve(cfg.key_cap * 4);
    uint16_t* knodeL = (uint16_t*)carve(cfg.key_cap * 2);
    int* ctl = S.ctl;
    const int nIni = G.n_ini;

    // ---- pyramid (fast path) in the sweep path's key region: depth d holds nIni * 4^d cells at
    // poff(d); pbest = (response << 56 | (0xFFFFFF - key index) << 32 | key), the retained key ----
    const size_t preg_bytes = (((size_t)cfg.key_cap * 4 + 15) & ~size_t(15)) + (((size_t)cfg.key_cap * 2 + 15) & ~size_t(15));
    // level d starts at poff(d), a multiple of 4 cells (16-byte vector reads of 4 siblings)
    const int nIni4 = (nIni + 3) & ~3;
    auto poff = [&](int d) { return d == 0 ? 0 : nIni4 + nIni * ((1 << (2 * d)) - 4) / 3; };
    // behind the pyramid: the depth-Dh x interval of every level column (root << 8 | x path bits)
    // and y interval of every row, so that a key's cell is two table reads
    const int Wlev = G.max_bx - G.min_bx, Hroot = G.max_by - G.min_by;
    const size_t tab_bytes = 2 * (size_t)Wlev + (size_t)Hroot + 32;
    // depth: one level below the first with >= N cells (ceil(log4(N / nIni)) + 1), where the
    // final divisions of a typical level stop; a deeper division takes the sweep path
    int Dh = 0;
    if (cfg.fast) {
        int want = 1;
        while (want < kOctMaxDh && (nIni << (2 * want)) < G.n_feat) want++;
        want = min(want + 1, min(cfg.max_dh, kOctMaxDh));
        for (int d = want; d >= 1; d--)
            if ((size_t)poff(d + 1) * 12 + tab_bytes <= preg_bytes) { Dh = d; break; }
    }
    unsigned long long* pbest = (unsigned long long*)keysL;
    uint32_t* pcnt = (uint32_t*)(pbest + (Dh ? poff(Dh + 1) : 0));
    uint16_t* xtab = (uint16_t*)(pcnt + (Dh ? poff(Dh + 1) : 0));
    uint8_t* ytab = (uint8_t*)(xtab + Wlev);
    const float hX = G.hX;
    auto root_of_x = [&](int x) {
        const int r = (int)((float)x / hX);
        return r < 0 ? 0 : (r >= nIni ? nIni - 1 : r);
    };
    // the plan's interval tables (6 split levels) cut to Dh levels, copied to LDS; entries
    // tid and tid + nt are loaded with the cell counts, the rest (wide levels) on the way
    const int ntab = Dh ? Wlev + Hroot : 0;
    const uint16_t* otl = otab + G.oct_tab_off;
    auto tab_put = [&](int i, uint32_t v) {
        if (i < Wlev) xtab[i] = (uint16_t)((v & 0xFF00u) | ((v & 0xFFu) >> (kOctMaxDh - Dh)));
        else ytab[i - Wlev] = (uint8_t)(v >> (kOctMaxDh - Dh));
    };
    // ---- 1. candidate count per cell -> cell-major key order (wave 0 scans the cells) ----
    const int ncell = G.n_cells;
    const int* cc = cand_cnt + (int64_t)f * P->n_cells_total + G.cell_base;
    TR_PHASE(2, 51)
    // the pyramid's deepest level starts at zero (16-byte stores while the count loads fly)
    auto zero_pyramid = [&]() {
        if (Dh) {
            ulonglong2* b2 = (ulonglong2*)(pbest + poff(Dh));
            uint4* c4 = (uint4*)(pcnt + poff(Dh));
            const int n4 = (poff(Dh + 1) - poff(Dh)) >> 2;
            for (int i = tid; i < n4; i += nt) {
                b2[2 * i] = ulonglong2{0ull, 0ull};
                b2[2 * i + 1] = ulonglong2{0ull, 0ull};
                c4[i] = uint4{0u, 0u, 0u, 0u};
            }
        }
    };
    const uint32_t* cbase = cand + (int64_t)f * P->n_slots_total;
    // key j of level cell c: its primary slot (j < kCandPrim, fixed ranges) or its slot range
    const uint32_t* pbase = (cprim && !cand_off) ? cprim + ((int64_t)f * P->n_cells_total + G.cell_base) * kCandPrim
                                                 : nullptr;
    auto cand_at = [&](int c, int j) -> uint32_t {
        return (pbase && j < kCandPrim) ? pbase[c * kCandPrim + j] : cbase[S.cslot[c] + j];
    };
    if (ncell <= nt) {
        // one cell per thread: every count / slot load in flight at once, one block scan
        const int c = tid < ncell ? cc[tid] : 0;
        const int so = tid >= ncell ? 0 : (cand_off ? cand_off[(int64_t)f * P->n_cells_total + G.cell_base + tid]
                                                   : cells[G.cell_base + tid].slot_off);
        const uint32_t t0 = tid < ntab ? otl[tid] : 0u, t1 = tid + nt < ntab ? otl[tid + nt] : 0u;
        zero_pyramid();
        if (tid < ncell) S.cslot[tid] = so;
        TR_PHASE(2, 52)
        int M0;
        const int ex = block_excl_scan(c, ctl, &M0);
        if (tid < ncell) S.cellstart[tid] = ex;
        if (tid == 0) { S.cellstart[ncell] = M0; ctl[55] = M0; }
        for (int i = tid; i < nIni * 4; i += nt) S.ccount[i] = 0;
        if (tid < ntab) tab_put(tid, t0);
        if (tid + nt < ntab) tab_put(tid + nt, t1);
        for (int i = tid + 2 * nt; i < ntab; i += nt) tab_put(i, otl[i]);
    } else if (w0) {
        for (int i = lane; i < ncell; i += 64) {
            S.cellstart[i] = cc[i];
            S.cslot[i] = cand_off ? cand_off[(int64_t)f * P->n_cells_total + G.cell_base + i]
                                  : cells[G.cell_base + i].slot_off;
        }
        wave_lds_fence();
        const int M0 = wave_scan_lds(S.cellstart, ncell);
        if (lane == 0) { S.cellstart[ncell] = M0; ctl[55] = M0; }
        for (int i = lane; i < nIni * 4; i += 64) S.ccount[i] = 0;
    }
    if (ncell > nt) {
        zero_pyramid();
        for (int i = tid; i < ntab; i += nt) tab_put(i, otl[i]);
    }
    __syncthreads();
    TR_PHASE(2, 50)
    const int M = ctl[55];
    const int N = G.n_feat;

    auto run = [&](auto fastc) -> bool {
        constexpr bool FAST = decltype(fastc)::value;
        const bool keys_in_lds = M <= cfg.key_cap;
        uint32_t* keys = keys_in_lds ? keysL : kscratch + (int64_t)f * P->n_slots_total + G.slot_base;
        uint16_t* knode = keys_in_lds ? knodeL : nscratch + (int64_t)f * P->n_slots_total + G.slot_base;
        // flattened gather: key k belongs to the cell c with cellstart[c] <= k < cellstart[c+1]
        // (binary search in LDS); 4 keys per thread with their loads in flight together
        // the 4 searches step together (a uniform trip count), so their LDS reads overlap
        int top = 1;
        while (2 * top < ncell) top *= 2;
        auto gather4 = [&](int k0, uint32_t* kv) {
            int k[4], lo[4] = {0, 0, 0, 0};
#pragma unroll
            for (int u = 0; u < 4; u++) k[u] = min(k0 + tid + u * nt, M - 1);
            for (int step = top; step > 0; step >>= 1) {
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    const int c = lo[u] + step;
                    if (c < ncell && S.cellstart[c] <= k[u]) lo[u] = c;
                }
            }
#pragma unroll
            for (int u = 0; u < 4; u++) kv[u] = cand_at(lo[u], k[u] - S.cellstart[lo[u]]);
        };
        auto root_of = [&](uint32_t key) { return root_of_x(cand_x(key)); };
        auto root_rect = [&](int r) { return mk_rect((int)(hX * (float)r), 0, (int)(hX * (float)(r + 1)), Hroot); };
        // node of the division: a rectangle (sweep) or (depth << 32 | path) (pyramid)
        auto kid = [&](uint64_t r, int q) -> uint64_t {
            if constexpr (FAST) return ((r + (1ull << 32)) & 0xFFFFFFFF00000000ull) | (uint64_t)((uint32_t)r * 4u + (uint32_t)q);
            else return child_rect(r, q);
        };
        // With M <= kOctKR * nt (every C2/C3 level) the sweep path keeps each thread's keys
        // k = tid + u * nt and their current nodes in registers for the whole division (kreg/nreg)
        const bool kr = !FAST && M <= kOctKR * nt;
        uint32_t kreg[kOctKR];
        int nreg[kOctKR];
#pragma unroll
        for (int u = 0; u < kOctKR; u++) { kreg[u] = 0u; nreg[u] = 0; }
        if constexpr (FAST) {
            // ---- 2. histogram of the depth-Dh cells, then the pyramid (two levels per barrier) ----
            // key -> cell without a search: each cell writes its index over its key range into
            // cellof (u16), which borrows the node-pass scratch (ccount .. skey2: untouched until
            // the roots); a level with more keys than it holds searches instead
            uint16_t* cellof = (uint16_t*)S.ccount;
            const bool direct = M <= (int)(((unsigned char*)(S.skey2 + cfg.sort_cap) - (unsigned char*)S.ccount) / 2);
            if (direct) {
                for (int c = tid; c < ncell; c += nt)
                    for (int j = S.cellstart[c]; j < S.cellstart[c + 1]; j++) cellof[j] = (uint16_t)c;
                __syncthreads();
            }
            const int ob = poff(Dh);
            for (int k0 = 0; k0 < M; k0 += 4 * nt) {
                uint32_t kv[4];
                if (direct) {
#pragma unroll
                    for (int u = 0; u < 4; u++) {
                        const int k = min(k0 + tid + u * nt, M - 1);
                        const int c = cellof[k];
                        kv[u] = cand_at(c, k - S.cellstart[c]);
                    }
                } else {
                    gather4(k0, kv);
                }
                if (k0 == 0) { TR_PHASE(2, 55) }
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    const int k = k0 + tid + u * nt;
                    if (k < M) {
                        const uint32_t xb = xtab[cand_x(kv[u])], yb = ytab[cand_y(kv[u])];
                        // Morton interleave: quadrant digit d = x bit d + 2 * y bit d
                        auto spread = [](uint32_t v) {
                            v = (v | (v << 4)) & 0x0F0Fu;
                            v = (v | (v << 2)) & 0x3333u;
                            return (v | (v << 1)) & 0x5555u;
                        };
                        const uint32_t path = ((xb >> 8) << (2 * Dh)) | spread(xb & 0xFFu) | (spread(yb) << 1);
                        atomicAdd(&pcnt[ob + (int)path], 1u);
                        atomicMax(&pbest[ob + (int)path], ((unsigned long long)cand_s(kv[u]) << 56) |
                                                              ((unsigned long long)(0xFFFFFFu - (uint32_t)k) << 32) | kv[u]);
                    }
                }
            }
            TR_PHASE(2, 56)
            __syncthreads();
            TR_PHASE(2, 53)
            // the two deepest levels below Dh by the block (a thread per depth-(Dh-2) cell), the
            // rest by wave 0 level by level (no block barriers); the root counts feed the roots
            int d = Dh;
            if (d >= 2) {
                const int o0 = poff(d), o1 = poff(d - 1), o2 = poff(d - 2);
                for (int i = tid; i < (nIni << (2 * (d - 2))); i += nt) {
                    uint32_t c2 = 0;
                    unsigned long long b2 = 0;
#pragma unroll
                    for (int j = 0; j < 4; j++) {
                        const int i1 = 4 * i + j;
                        const uint4 c4 = *(const uint4*)&pcnt[o0 + 4 * i1];
                        const ulonglong2 ba = *(const ulonglong2*)&pbest[o0 + 4 * i1];
                        const ulonglong2 bb = *(const ulonglong2*)&pbest[o0 + 4 * i1 + 2];
                        const uint32_t c1 = c4.x + c4.y + c4.z + c4.w;
                        const unsigned long long b1 = max(max(ba.x, ba.y), max(bb.x, bb.y));
                        pcnt[o1 + i1] = c1;
                        pbest[o1 + i1] = b1;
                        c2 += c1;
                        b2 = max(b2, b1);
                    }
                    pcnt[o2 + i] = c2;
                    pbest[o2 + i] = b2;
                }
                d -= 2;
                __syncthreads();
            }
            if (w0) {
                for (d = d - 1; d >= 0; d--) {
                    const int o0 = poff(d + 1), o1 = poff(d);
                    for (int i = lane; i < (nIni << (2 * d)); i += 64) {
                        const uint4 c4 = *(const uint4*)&pcnt[o0 + 4 * i];
                        const ulonglong2 ba = *(const ulonglong2*)&pbest[o0 + 4 * i];
                        const ulonglong2 bb = *(const ulonglong2*)&pbest[o0 + 4 * i + 2];
                        pcnt[o1 + i] = c4.x + c4.y + c4.z + c4.w;
                        pbest[o1 + i] = max(max(ba.x, ba.y), max(bb.x, bb.y));
                    }
                    wave_lds_fence();
                }
                for (int i = lane; i < nIni; i += 64) S.ccount[i] = pcnt[i];   // root counts (poff(0) = 0)
            }
        } else {
            // ---- 2. gather + root classification (run-aggregated counts per root) ----
            auto root4 = [&](int k0, const uint32_t* kv, uint32_t* kr4, int* nr4) {
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    const int k = k0 + tid + u * nt;
                    uint32_t tgt = 0xFFFFFFFFu;
                    if (k < M) {
                        keys[k] = kv[u];
                        const int r = root_of(kv[u]);
                        tgt = (uint32_t)r;
                        if (kr4) { kr4[u] = kv[u]; nr4[u] = r; }
                        else knode[k] = (uint16_t)r;
                    }
                    wave_aggregate_count(tgt, S.ccount);
                }
            };
            if (kr) {
                // compile-time register slots: group g holds keys k = (4g + u) * nt + tid
#pragma unroll
                for (int g = 0; g < kOctKR / 4; g++) {
                    if (4 * g * nt < M) {   // block-uniform
                        uint32_t kv[4];
                        gather4(4 * g * nt, kv);
                        root4(4 * g * nt, kv, kreg + 4 * g, nreg + 4 * g);
                    }
                }
            } else {
                for (int k0 = 0; k0 < M; k0 += 4 * nt) {
                    uint32_t kv[4];
                    gather4(k0, kv);
                    root4(k0, kv, nullptr, nullptr);
                }
            }
        }
        __syncthreads();
        TR_PHASE(2, 54)
        // ---- 3. roots (nIni <= 64 enforced by the host) ----
        if (w0) {
            if (lane == 0) {
                int n = 0;
                for (int r = 0; r < nIni; r++) {
                    const uint64_t rr = FAST ? (uint64_t)r : root_rect(r);
                    S.rectB[r] = rr;   // OLD buffer = roots (remap source)
                    if (S.ccount[r] > 0) {
                        S.rectA[n] = rr; S.cntA[n] = S.ccount[r]; S.serA[n] = r;
                        S.map4[r * 4 + 0] = S.map4[r * 4 + 1] = S.map4[r * 4 + 2] = S.map4[r * 4 + 3] = (uint16_t)n;
                        n++;
                    }
                }
                ctl[56] = n;          // list size
                ctl[57] = nIni;       // next serial
                ctl[58] = 0;          // mode: 0 main, 1 final
                ctl[59] = 0;          // finished
                ctl[62] = 0;          // pyramid too shallow: back to the sweep path
            }
            wave_lds_fence();
            const int n = ctl[56];
            for (int i = lane; i < n * 4; i += 64) S.ccount[i] = 0;
        }
        __syncthreads();
        TR_PHASE(2, 0)
        // CUR = A, OLD = B
        uint64_t *rectC = S.rectA, *rectO = S.rectB;
        uint32_t *cntC = S.cntA, *serC = S.serA;
        uint32_t *cntO = S.cntB, *serO = S.serB;
#if ORBHIP_OCT_W0_MAIN
        if constexpr (FAST) {
            // MAIN rounds of lists of <= 64 nodes by wave 0 alone, one node per lane in registers and
            // no block barrier between rounds: the same pass as the loop below (children of the
            // dividing nodes pushed to the front, later parents first, n4..n1 inside a parent's
            // block, the undivided nodes behind them in order; serials in division order). The
            // loop below takes over at the first longer list or FINAL pass (ctl[61]: rounds run).
            if (w0) {
                uint64_t *rC = S.rectA, *rO = S.rectB;
                uint32_t *cC = S.cntA, *sC = S.serA, *cO = S.cntB, *sO = S.serB;
                int n = ctl[56], serial = ctl[57], rounds = 0;
                bool deep = false, fin = false, fmode = false;
                while (n <= 64 && rounds < 64) {
                    // loads from clamped addresses, no branch around them (a branch per load made
                    // the compiler wait out each one's round trip in turn)
                    const bool has = lane < n;
                    const int pl = has ? lane : 0;
                    const uint64_t cd0 = rC[pl];
                    const uint32_t cnt0 = cC[pl], ser0 = sC[pl];
                    const uint64_t cd = has ? cd0 : 0ull;
                    const uint32_t cnt = has ? cnt0 : 0u, ser = has ? ser0 : 0u;
                    const bool dv = has && cnt > 1;
                    const int d = (int)(cd >> 32);
                    if (__ballot(dv && d >= Dh)) {   // a node too deep for the pyramid
                        deep = true;
                        break;
                    }
                    const uint4 c4l = *(const uint4*)&pcnt[dv ? poff(d + 1) + 4 * (int)(uint32_t)cd : 0];
                    const uint4 c4 = dv ? c4l : uint4{0u, 0u, 0u, 0u};
                    const uint32_t cq[4] = {c4.x, c4.y, c4.z, c4.w};
                    const int c = dv ? nonempty4(cq) : 0, e = dv ? multi4(cq) : 0, u = (has && !dv) ? 1 : 0;
                    const int ic = wave_incl_scan(c), iu = wave_incl_scan(u), ie = wave_incl_scan(e);
                    const int T = __builtin_amdgcn_readlane(ic, 63), U = __builtin_amdgcn_readlane(iu, 63);
                    const int E = __builtin_amdgcn_readlane(ie, 63);
                    const int cb = ic - c;
                    if (dv) {
                        const int base = T - cb - c;
                        int r = 0;
#pragma unroll
                        for (int q = 0; q < 4; q++) {
                            if (cq[q] == 0) continue;
                            const int pos = base + (c - 1 - r);
                            rO[pos] = kid(cd, q);
                            cO[pos] = cq[q];
                            sO[pos] = (uint32_t)(serial + cb + r);
                            r++;
                        }
                    } else if (has) {
                        const int pos = T + iu - u;
                        rO[pos] = cd;
                        cO[pos] = cnt;
                        sO[pos] = ser;
                    }
                    wave_lds_fence();
                    const int newSize = T + U;
                    serial += T;
                    rounds++;
                    { uint64_t* t = rC; rC = rO; rO = t; }
                    { uint32_t* t = cC; cC = cO; cO = t; }
                    { uint32_t* t = sC; sC = sO; sO = t; }
                    const int prev = n;
                    n = newSize;
                    if (newSize >= N || newSize == prev) { fin = true; break; }
                    if (newSize + E * 3 > N) { fmode = true; break; }
                }
                if (lane == 0) {
                    ctl[56] = n;
                    ctl[57] = serial;
                    ctl[58] = fmode ? 1 : 0;
                    ctl[59] = fin ? 1 : 0;
                    ctl[61] = rounds;
                    ctl[62] = deep ? 1 : 0;
                }
            }
            __syncthreads();
            TR_PHASE(2, 40)
            if (ctl[62]) return false;   // every thread, after the barrier: the level goes to the sweep path
            if (ctl[61] & 1) {
                { uint64_t* t = rectC; rectC = rectO; rectO = t; }
                { uint32_t* t = cntC; cntC = cntO; cntO = t; }
                { uint32_t* t = serC; serC = serO; serO = t; }
            }
        }
#endif
        for (int iter = 0; !ctl[59]; iter++) {
            // read before the round's barrier: wave 0 rewrites the control words in its node pass
            const int n = ctl[56];
            const int mode = ctl[58];
            if (iter > 64 || n > NC) {   // runaway guard: never expected
                if (tid == 0) atomicOr(err, 1);
                break;
            }
            // a FINAL pass of a list the block covers with one node per thread: its fill, key
            // collection and node pass by the whole block (block scans) instead of wave 0 alone
            const bool blk_final = FAST && ORBHIP_OCT_BLK_FINAL && mode == 1 && n <= nt;   // block-uniform
            if constexpr (FAST) {
                if (blk_final) {
                    // node tid's children counts, and its (size, serial, node) key if it divides
                    const int p = tid, pc = p < n ? p : 0;
                    const uint32_t cn = cntC[pc], sr = serC[pc];
                    const uint64_t cd = rectC[pc];
                    const bool dvd = p < n && cn > 1;
                    const int d = (int)(cd >> 32);
                    const bool okd = dvd && d < Dh;
                    const uint4 c4 = *(const uint4*)&pcnt[okd ? poff(d + 1) + 4 * (int)(uint32_t)cd : 0];
                    if (dvd && d >= Dh) ctl[62] = 1;   // every writer stores 1; read after the scan's barriers
                    if (okd) *(uint4*)&S.ccount[4 * p] = c4;
                    int K;
                    const int pos = block_excl_scan(dvd ? 1 : 0, ctl, &K);
                    if (dvd) S.skey2[pos] = ((uint64_t)cn << 40) | ((uint64_t)sr << 16) | (uint64_t)p;
                    if (tid == 0) ctl[60] = K;
                }
                // ---- children counts of every node to divide, from the pyramid (wave 0) ----
                if (w0 && !blk_final) {
                    bool deep = false;
                    for (int p = lane; p < n; p += 64) {
                        if (cntC[p] > 1) {
                            const uint64_t cd = rectC[p];
                            const int d = (int)(cd >> 32);
                            if (d >= Dh) {
                                deep = true;
                            } else {
                                const uint4 c4 = *(const uint4*)&pcnt[poff(d + 1) + 4 * (int)(uint32_t)cd];
                                *(uint4*)&S.ccount[4 * p] = c4;
                            }
                        }
                    }
                
                    if (__ballot(deep) && lane == 0) ctl[62] = 1;
                    wave_lds_fence();
                }
            } else {
                // ---- sweep: remap keys through map4 (OLD rect split), classify into CUR children ----
                if (kr) {
#pragma unroll
                    for (int g = 0; g < kOctKR / 4; g++) {
                        if (4 * g * nt >= M) continue;   // block-uniform
                        uint32_t tg[4];
#pragma unroll
                        for (int v = 0; v < 4; v++) {
                            const int u = 4 * g + v;
                            const int k = tid + u * nt;
                            tg[v] = 0xFFFFFFFFu;
                            if (k < M) {
                                const int x = cand_x(kreg[u]), y = cand_y(kreg[u]);
                                const int o = nreg[u];
                                nreg[u] = S.map4[o * 4 + quad_of(rectO[o], x, y)];
                            }
                        }
#pragma unroll
                        for (int v = 0; v < 4; v++) {
                            const int u = 4 * g + v;
                            const int k = tid + u * nt;
                            if (k < M) {
                                const int nd = nreg[u];
                                if (cntC[nd] > 1)
                                    tg[v] = (uint32_t)(nd * 4 + quad_of(rectC[nd], cand_x(kreg[u]), cand_y(kreg[u])));
                            }
                        }
#pragma unroll
                        for (int v = 0; v < 4; v++) wave_aggregate_count(tg[v], S.ccount);
                    }
                } else {
                    for (int k0 = 0; k0 < M; k0 += nt) {
                        const int k = k0 + tid;
                        uint32_t tgt = 0xFFFFFFFFu;
                        if (k < M) {
                            const uint32_t key = keys[k];
                            const int x = cand_x(key), y = cand_y(key);
                            const int o = knode[k];
                            const int nd = S.map4[o * 4 + quad_of(rectO[o], x, y)];
                            knode[k] = (uint16_t)nd;
                            if (cntC[nd] > 1) tgt = (uint32_t)(nd * 4 + quad_of(rectC[nd], x, y));
                        }
                        wave_aggregate_count(tgt, S.ccount);
                    }
                }
                __syncthreads();
            }
            if (iter == 1) { TR_PHASE(2, 41) }
            // wave 0 only: after the fill, ctl[62] is final for this round
            const bool stop = FAST && w0 && ctl[62];
            if (mode == 0) {
                // ---- MAIN pass (wave 0): divide every node with > 1 key ----
                if (w0 && !stop) {
                    const int serial0 = ctl[57];
                    const int per = (n + 63) >> 6;
                    const int b = min(lane * per, n), e = min(b + per, n);
                    int sc = 0, su = 0, se = 0;
                    for (int p = b; p < e; p++) {
                        if (cntC[p] > 1) { sc += nonempty4(S.ccount + 4 * p); se += multi4(S.ccount + 4 * p); }
                        else su += 1;
                    }
                    const int ic = wave_incl_scan(sc), iu = wave_incl_scan(su), ie = wave_incl_scan(se);
                    const int T = __builtin_amdgcn_readlane(ic, 63), U = __builtin_amdgcn_readlane(iu, 63);
                    const int nToExpand = __builtin_amdgcn_readlane(ie, 63);
                    int cb = ic - sc, ub = iu - su;
                    for (int p = b; p < e; p++) {
                        if (cntC[p] > 1) {
                            const int c = nonempty4(S.ccount + 4 * p);
                            const int base = T - cb - c;          // pushed to the front: later parents first
                            int r = 0;
                            for (int q = 0; q < 4; q++) {
                                const uint32_t cq = S.ccount[p * 4 + q];
                                if (cq == 0) continue;
                                const int pos = base + (c - 1 - r);   // n4..n1 order inside the block
                                rectO[pos] = kid(rectC[p], q);
                                cntO[pos] = cq; serO[pos] = serial0 + cb + r;
                                S.map4[p * 4 + q] = (uint16_t)pos;
                                r++;
                            }
                            cb += c;
                        } else {
                            const int pos = T + ub;
                            rectO[pos] = rectC[p]; cntO[pos] = cntC[p]; serO[pos] = serC[p];
                            S.map4[p * 4 + 0] = S.map4[p * 4 + 1] = S.map4[p * 4 + 2] = S.map4[p * 4 + 3] = (uint16_t)pos;
                            ub++;
                        }
                    }
                    const int newSize = T + U;
                    wave_lds_fence();
                    if constexpr (!FAST)
                        for (int i = lane; i < min(newSize, NC) * 4; i += 64) S.ccount[i] = 0;
                    if (lane == 0) {
                        ctl[57] = serial0 + T;
                        ctl[56] = newSize;
                        if (newSize >= N || newSize == n) ctl[59] = 1;
                        else if (newSize + nToExpand * 3 > N) ctl[58] = 1;
                    }
                }
            } else {
                // ---- FINAL phase: divide largest (size, serial) first until >= N ----
                TR_PHASE(2, 48)
                if (w0 && !blk_final) {
                    const int per = (n + 63) >> 6;
                    const int b = min(lane * per, n), e = min(b + per, n);
                    int s = 0;
                    for (int p = b; p < e; p++) s += cntC[p] > 1;
                    const int inc = wave_incl_scan(s);
                    int pos = inc - s;
                    for (int p = b; p < e; p++)
                        if (cntC[p] > 1)
                            S.skey2[pos++] = ((uint64_t)cntC[p] << 40) | ((uint64_t)serC[p] << 16) | (uint64_t)p;
                    if (lane == 0) ctl[60] = __builtin_amdgcn_readlane(inc, 63);
                }
                TR_PHASE(2, 45)
                __syncthreads();
                TR_PHASE(2, 46)
                const int K = ctl[60];
                block_rank_sort_desc(S.skey2, S.skey, K);   // keys unique: (size, serial) order; ends in a barrier
                TR_PHASE(2, 47)
                if (blk_final) {
                    if (!ctl[62]) {   // block-uniform (after the sort's barrier)
                        // thread j: sorted entry j. run_j = n + sum_{i <= j} (c_i - 1) is
                        // non-decreasing (a divided node has a child), so jstar, the first division
                        // after which the list holds >= N nodes, is the count of divisions that
                        // leave it short (or K - 1 when none reaches N)
                        const int serial0 = ctl[57];
                        const int j = tid, jc = j < K ? j : 0;
                        const int pj = (int)(S.skey[jc] & 0xFFFF);
                        const uint4 c4 = *(const uint4*)&S.ccount[4 * pj];
                        const uint64_t rj = rectC[pj];
                        const uint32_t q4[4] = {c4.x, c4.y, c4.z, c4.w};
                        const int c = j < K ? nonempty4(q4) : 0;
                        // (counted with an LDS atomic on a control word: __syncthreads_count
                        // would add static LDS to a kernel whose dynamic LDS fills the CU)
                        if (tid == 0) ctl[53] = 0;
                        int gt;
                        const int gex = block_excl_scan(j < K ? c - 1 : 0, ctl, &gt);   // barriers
                        if (j < K && n + gex + c - 1 < N) atomicAdd(&ctl[53], 1);
                        __syncthreads();
                        const int nb = ctl[53];
                        const int jstar = min(nb, K - 1);
                        const bool dvj = j < K && j <= jstar;
                        int Ctot;
                        const int cb = block_excl_scan(dvj ? c : 0, ctl, &Ctot);
                        if (tid < n) S.tD[tid] = 1;
                        __syncthreads();
                        if (dvj) {   // children pushed to the front in division order, n4..n1 inside
                            const int base = Ctot - cb - c;
                            int r = 0;
#pragma unroll
                            for (int q = 0; q < 4; q++) {
                                if (q4[q] == 0) continue;
                                const int ps = base + (c - 1 - r);
                                rectO[ps] = kid(rj, q);
                                cntO[ps] = q4[q];
                                serO[ps] = serial0 + cb + r;
                                r++;
                            }
                            S.tD[pj] = 0;
                        }
                        __syncthreads();
                        // the other nodes keep their order behind the children
                        const int p = tid, pc = p < n ? p : 0;
                        const int keep = p < n ? S.tD[pc] : 0;
                        const uint64_t rv = rectC[pc];
                        const uint32_t cv = cntC[pc], sv = serC[pc];
                        int nk;
                        const int ex = block_excl_scan(keep, ctl, &nk);
                        if (keep) {
                            rectO[Ctot + ex] = rv;
                            cntO[Ctot + ex] = cv;
                            serO[Ctot + ex] = sv;
                        }
                        const int newSize = Ctot + (n - (jstar + 1));
                        if (tid == 0) {
                            ctl[57] = serial0 + Ctot;
                            ctl[56] = newSize;
                            if (newSize >= N || newSize == n) ctl[59] = 1;
                        }
                    }
                } else if (w0 && !stop) {
                    const int serial0 = ctl[57];
                    const int per = (K + 63) >> 6;
                    const int b = min(lane * per, K), e = min(b + per, K);
                    // jstar: the first division (sorted order) after which the list holds >= N nodes
                    int g = 0;
                    for (int j = b; j < e; j++) g += nonempty4(S.ccount + 4 * (int)(S.skey[j] & 0xFFFF)) - 1;
                    const int ig = wave_incl_scan(g);
                    int run = n + ig - g, cand_j = K - 1;
                    for (int j = b; j < e; j++) {
                        run += nonempty4(S.ccount + 4 * (int)(S.skey[j] & 0xFFFF)) - 1;
                        if (run >= N) { cand_j = j; break; }
                    }
                    int jstar = cand_j;
#pragma unroll
                    for (int o = 1; o < 64; o <<= 1) jstar = min(jstar, __shfl_xor(jstar, o, 64));
                    // children of the divisions 0..jstar, pushed to the front in division order
                    int sc = 0;
                    for (int j = b; j < min(e, jstar + 1); j++) sc += nonempty4(S.ccount + 4 * (int)(S.skey[j] & 0xFFFF));
                    const int ic = wave_incl_scan(sc);
                    const int Ctot = __builtin_amdgcn_readlane(ic, 63);
                    for (int p = lane; p < n; p += 64) S.tD[p] = 1;
                    wave_lds_fence();
                    int cb = ic - sc;
                    for (int j = b; j < min(e, jstar + 1); j++) {
                        const int p = (int)(S.skey[j] & 0xFFFF);
                        const int c = nonempty4(S.ccount + 4 * p);
                        const int base = Ctot - cb - c;
                        int r = 0;
                        for (int q = 0; q < 4; q++) {
                            const uint32_t cq = S.ccount[p * 4 + q];
                            if (cq == 0) continue;
                            const int ps = base + (c - 1 - r);
                            rectO[ps] = kid(rectC[p], q);
                            cntO[ps] = cq; serO[ps] = serial0 + cb + r;
                            S.map4[p * 4 + q] = (uint16_t)ps;
                            r++;
                        }
                        S.tD[p] = 0;
                        cb += c;
                    }
                    wave_lds_fence();
                    // the other nodes keep their order behind the children
                    const int pn = (n + 63) >> 6;
                    const int bn = min(lane * pn, n), en = min(bn + pn, n);
                    int st = 0;
                    for (int p = bn; p < en; p++) st += S.tD[p];
                    const int is = wave_incl_scan(st);
                    int sb = is - st;
                    for (int p = bn; p < en; p++) {
                        if (S.tD[p]) {
                            const int ps = Ctot + sb;
                            rectO[ps] = rectC[p]; cntO[ps] = cntC[p]; serO[ps] = serC[p];
                            S.map4[p * 4 + 0] = S.map4[p * 4 + 1] = S.map4[p * 4 + 2] = S.map4[p * 4 + 3] = (uint16_t)ps;
                            sb++;
                        }
                    }
                    const int newSize = Ctot + (n - (jstar + 1));
                    wave_lds_fence();
                    if constexpr (!FAST)
                        for (int i = lane; i < min(newSize, NC) * 4; i += 64) S.ccount[i] = 0;
                    if (lane == 0) {
                        ctl[57] = serial0 + Ctot;
                        ctl[56] = newSize;
                        if (newSize >= N || newSize == n) ctl[59] = 1;
                    }
                }
            }
            __syncthreads();
            if (iter == 1) { TR_PHASE(2, 44) }
            if constexpr (FAST) {
                if (ctl[62]) return false;   // every thread, after the barrier: the level goes to the sweep path
            }
            // swap: NEXT (written into the O buffers) becomes CUR, CUR becomes OLD
            { uint64_t* t = rectC; rectC = rectO; rectO = t; }
            { uint32_t* t = cntC; cntC = cntO; cntO = t; }
            { uint32_t* t = serC; serC = serO; serO = t; }
            TR_PHASE(2, 1 + (iter < 28 ? iter : 28) + (mode ? 32 : 0))
            if (ctl[59]) break;
        }
        const int n = ctl[56];
        if constexpr (!FAST) {
            // ---- retained key per final node: max (response, then lowest key index) over the
            // keys of the node; keys reach their final node through the last division's map4 ----
            for (int i = tid; i < n; i += nt) S.cbest[i] = 0;
            __syncthreads();
            TR_PHASE(2, 60)
            if (kr) {
#pragma unroll
                for (int u = 0; u < kOctKR; u++) {
                    const int k = tid + u * nt;
                    if (k < M) {
                        const uint32_t key = kreg[u];
                        const int o = nreg[u];
                        const int nd = S.map4[o * 4 + quad_of(rectO[o], cand_x(key), cand_y(key))];
                        atomicMax(&S.cbest[nd], pack_best(cand_s(key), k));
                    }
                }
            } else {
                for (int k = tid; k < M; k += nt) {
                    const uint32_t key = keys[k];
                    const int o = knode[k];
                    const int nd = S.map4[o * 4 + quad_of(rectO[o], cand_x(key), cand_y(key))];
                    atomicMax(&S.cbest[nd], pack_best(cand_s(key), k));
                }
            }
            __syncthreads();
        }
        TR_PHASE(2, 61)
        // ---- output in list order: retained key per node, lapping flag, and its rank among the
        // same-flag nodes from one block scan per 1024 nodes ----
        const int ncap = min(n, G.kp_cap);
        LevelKp* out = lvl_kp + (int64_t)f * P->kp_slots_total + G.kp_base;
        int lap_run = 0;
        for (int p0 = 0; p0 < ncap; p0 += nt) {
            const int p = p0 + tid;
            int lap = 0, x = 0, y = 0, sc = 0;
            if (p < ncap) {
                uint32_t key;
                if constexpr (FAST) {
                    const uint64_t cd = rectC[p];
                    key = (uint32_t)pbest[poff((int)(cd >> 32)) + (int)(uint32_t)cd];
                } else {
                    key = keys[(int)(0xFFFFFFu - (S.cbest[p] & 0xFFFFFFu))];
                }
                x = cand_x(key) + G.min_bx; y = cand_y(key) + G.min_by;
                sc = cand_s(key);
                const float xs = (l == 0) ? (float)x : (float)x * G.scale;
                lap = (xs >= (float)cfg.lap0 && xs <= (float)cfg.lap1) ? 1 : 0;
            }
            int tot;
            const int before = lap_run + block_excl_scan(lap, ctl, &tot);   // same-flag nodes before p
            if (p < ncap) {
                const int rank = lap ? before : p - before;
                LevelKp r;
                r.x = (int16_t)x; r.y = (int16_t)y;
                r.srl = (uint32_t)sc | ((uint32_t)lap << 8) | ((uint32_t)rank << 9);
                out[p] = r;
            }
            lap_run += tot;
        }
        if (tid == 0) {
            lvl_cnt[f * P->n_levels + l] = ncap;
            lvl_nlap[f * P->n_levels + l] = lap_run;
            if (n > G.kp_cap) atomicOr(err, 2);
        }
        return true;
    };
    if (Dh) {
        if (run(std::true_type{})) {
            TR_PHASE(2, 63)
            TR_END(2)
            stamp_end();
            return;
        }
        // a node too deep for the pyramid: the sweep path from the gather on
        for (int i = tid; i < nIni * 4; i += nt) S.ccount[i] = 0;
        __syncthreads();
    }
    run(std::false_type{});
    TR_PHASE(2, 63)
    TR_END(2)
    stamp_end();
}

// ---------------------------------------------------------------------------
// k_desc: one wave per kept keypoint. IC_Angle on the level, rBRIEF on the bit-exact
// GaussianBlur(7x7, 2, REFLECT_101) of the level computed at the 512 sample points from a
// 43x43 LDS patch (reflect-101 applied at load). Writes the final operator() slot.
// ---------------------------------------------------------------------------
// rBRIEF samples lie within +-18 px of the keypoint (max rotated pattern radius 18.38,
// rounded): the blurred region is 37 x 37, computed from the 43 x 43 patch (+-3 blur halo).
constexpr int kBlR = 18, kBlW = 2 * kBlR + 1;   // 37
constexpr int kDpP = 48;                         // k_desc patch row pitch (12 dwords)
constexpr int kHrP = 48;                         // k_desc transposed row-pass pitch (rows 0..42, read to 45)
// GaussianBlur(7x7, sigma 2) 8-bit fixed-point taps (the host checks its table equals these)
__device__ __forceinline__ constexpr uint32_t blur_tap(int i) {
    return i == 0 || i == 6 ? 18u : (i == 1 || i == 5 ? 34u : (i == 2 || i == 4 ? 48u : 56u));
}

__global__ __launch_bounds__(256) void k_desc(const ExtractPlan* __restrict__ P, FrameBufs fb,
                                              const LevelKp* __restrict__ lvl_kp, const int* __restrict__ lvl_cnt,
                                              const int* __restrict__ lvl_nlap, const int* __restrict__ disc,
                                              orbhip_kp* __restrict__ out_kps, uint8_t* __restrict__ out_desc,
                                              int cap, int* __restrict__ n_out, int* __restrict__ mono_out, int xrun) {
    // patch rows of kDpP bytes: a pixel at byte sh + x of its row (sh = the patch origin's byte
    // misalignment when the rows were copied as aligned dwords, 0 on the reflected border path)
    __shared__ __attribute__((aligned(16))) uint8_t patch[4][kPatchW * kDpP + 16];
    // row pass output TRANSPOSED (column c at c * kHrP): the column pass reads row pairs as dwords
    __shared__ __attribute__((aligned(16))) uint16_t hrow[4][kBlW * kHrP];
    TR_BEGIN()
    const int X = gridDim.x, lg = xcd_runs(blockIdx.x + X * blockIdx.y, X * gridDim.y, xrun < 0 ? X : xrun);
    const int f = lg / X;
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    int slot = (lg % X) * 4 + wid;
    const int L = P->n_levels;
    // frame totals (same in every lane / wave of the frame)
    int total = 0, nlap_tot = 0;
    for (int l = 0; l < L; l++) { total += lvl_cnt[f * L + l]; nlap_tot += lvl_nlap[f * L + l]; }
    if (lg % X == 0 && threadIdx.x == 0) {
        n_out[f] = total;
        mono_out[f] = total - nlap_tot;
    }
    int l = 0, mono_base = 0, lap_base = 0;
    while (l < L && slot >= P->lv[l].kp_cap) {
        slot -= P->lv[l].kp_cap;
        mono_base += lvl_cnt[f * L + l] - lvl_nlap[f * L + l];
        lap_base += lvl_nlap[f * L + l];
        l++;
    }
    const bool active = l < L && slot < lvl_cnt[f * L + l];   // wave-uniform
    uint8_t* pt = patch[wid];
    uint16_t* hr = hrow[wid];
    uint8_t* bl = patch[wid];   // blurred 37 x 37: the patch is dead once the row pass has run
    static_assert(kBlW * kBlW <= kPatchW * kDpP, "blurred region fits the patch");
    int cx = 0, cy = 0, sh = 0;
    LevelKp kp{};
    // the IC_Angle disc offsets (n_disc <= 31 x 31 < 16 x 64), loaded with the keypoint so that
    // they arrive with the patch instead of one dependent load per disc round; entries past
    // n_disc are (0, 0) and add nothing
    constexpr int kDiscU = 16;
    int dv[kDiscU];
    if (active) {
        const int nd = P->n_disc;
#pragma unroll
        for (int u = 0; u < kDiscU; u++) dv[u] = lane + 64 * u < nd ? disc[lane + 64 * u] : 0;
    }
    if (active) {
        const LevelGeom& G = P->lv[l];
        ImgRef im = level_img(P, fb, f, l);
        kp = lvl_kp[(int64_t)f * P->kp_slots_total + G.kp_base + slot];
        cx = kp.x; cy = kp.y;
        const int lw = G.w, lh = G.h;
        const bool inside = cx - kPatchR >= 0 && cy - kPatchR >= 0 && cx + kPatchR < lw && cy + kPatchR < lh;
        const bool dw = inside && ((im.pitch & 3) == 0) && ((((uintptr_t)im.p) & 3) == 0);
        if (dw) {
            // 43 rows x 12 aligned dwords (the 43 + sh <= 46 patch bytes of a row), 9 per lane
            const uint8_t* src = im.p + (int64_t)(cy - kPatchR) * im.pitch + (cx - kPatchR);
            sh = (int)(((uintptr_t)src) & 3);
            const uint32_t* s4 = (const uint32_t*)(src - sh);
            const int p4 = im.pitch >> 2;
            constexpr int kND = kPatchW * (kDpP / 4), kDU = (kND + 63) / 64;
            uint32_t v[kDU];
#pragma unroll
            for (int u = 0; u < kDU; u++) {
                const int i = min(lane + 64 * u, kND - 1);   // branch-free loads
                const int r = (i * 43691) >> 19, k = i - 12 * r;   // i / 12 for i < 98304
                v[u] = s4[(int64_t)r * p4 + k];
            }
            uint32_t* d4 = (uint32_t*)pt;
#pragma unroll
            for (int u = 0; u < kDU; u++) {
                const int i = lane + 64 * u;
                if (i < kND) d4[i] = v[u];
            }
        } else {
            // reflected border: byte loads in rounds of 8 (few keypoints; bounded registers)
            constexpr int kPU = (kPatchW * kPatchW + 63) / 64;   // 29 bytes per lane
            constexpr float kInvPW = 1.0f / kPatchW;
#pragma unroll 1
            for (int u0 = 0; u0 < kPU; u0 += 8) {
                uint8_t v[8];
                int li[8];
#pragma unroll
                for (int u = 0; u < 8; u++) {
                    const int i = min(lane + 64 * (u0 + u), kPatchW * kPatchW - 1);
                    const int py = (int)(((float)i + 0.5f) * kInvPW), px = i - py * kPatchW;
                    int yy = cy - kPatchR + py, xx = cx - kPatchR + px;
                    // BORDER_REFLECT_101 (levels are >= 43 px in both dims)
                    yy = yy < 0 ? -yy : (yy >= lh ? 2 * lh - 2 - yy : yy);
                    xx = xx < 0 ? -xx : (xx >= lw ? 2 * lw - 2 - xx : xx);
                    v[u] = (u0 + u < kPU) ? im.p[(int64_t)yy * im.pitch + xx] : 0;
                    li[u] = py * kDpP + px;
                }
#pragma unroll
                for (int u = 0; u < 8; u++)
                    if (u0 + u < kPU && lane + 64 * (u0 + u) < kPatchW * kPatchW) pt[li[u]] = v[u];
            }
        }
    }
    wave_lds_fence();   // each wave works on its own keypoint's LDS only
    TR_PHASE(3, 0)
    // ---- IC_Angle: m10 = sum u*I, m01 = sum v*I over the umax disc (unblurred level) ----
    float angle = 0.f;
    if (active) {
        int m10 = 0, m01 = 0;
#pragma unroll
        for (int k = 0; k < kDiscU; k++) {
            const int uv = dv[k];
            const int u = (int)(int16_t)(uv & 0xFFFF), vv = (int)(int16_t)(uv >> 16);
            const int val = pt[(kPatchR + vv) * kDpP + sh + kPatchR + u];
            m10 += u * val;
            m01 += vv * val;
        }
        m10 = wave_sum_i32(m10);
        m01 = wave_sum_i32(m01);
        angle = fast_atan2((float)m01, (float)m10);
        // ---- 7x7 blur, row pass: hr[r][c] = sum_i k_i pt[r][c + i], r < 43, c < 37 ----
        // lane task = 4 consecutive columns of one row: 4 dword reads, realigned by sh, and two
        // v_dot4_u32_u8 per output (taps 18 34 48 56 | 48 34 18 0 against bytes c..c+3 | c+4..c+7)
        const uint32_t K0 = 18u | 34u << 8 | 48u << 16 | 56u << 24, K1 = 48u | 34u << 8 | 18u << 16;
        const uint32_t* p4 = (const uint32_t*)pt;
#pragma unroll 1
        for (int t = lane; t < kPatchW * 10; t += 64) {
            const int r = (t * 6554) >> 16, c0 = 4 * (t - 10 * r);   // t / 10 for t < 16384
            const uint32_t* w = p4 + r * (kDpP / 4) + (c0 >> 2);
            const uint32_t w0 = w[0], w1 = w[1], w2 = w[2], w3 = w[3];
            const uint32_t x0 = __builtin_amdgcn_alignbyte(w1, w0, sh);   // pixels c0 .. c0+3
            const uint32_t x1 = __builtin_amdgcn_alignbyte(w2, w1, sh);   // c0+4 .. c0+7
            const uint32_t x2 = __builtin_amdgcn_alignbyte(w3, w2, sh);   // c0+8 .. c0+11
#pragma unroll
            for (int o = 0; o < 4; o++) {
                if (c0 + o >= kBlW) break;
                const uint32_t a = o == 0 ? x0 : __builtin_amdgcn_alignbyte(x1, x0, o);
                const uint32_t bq = o == 0 ? x1 : __builtin_amdgcn_alignbyte(x2, x1, o);
                const uint32_t h = __builtin_amdgcn_udot4(bq, K1, __builtin_amdgcn_udot4(a, K0, 0u, false), false);
                hr[(c0 + o) * kHrP + r] = (uint16_t)h;
            }
        }
    }
    wave_lds_fence();   // each wave works on its own keypoint's LDS only
    if (active) {
        // ---- column pass: bl[r][c] = (sum_j k_j hr[r + j][c] + 2^15) >> 16, 4 rows per task:
        // rows r0 .. r0+9 of column c as 5 dwords of row pairs, 4 v_dot2_u32_u16 per output
        // (even outputs against taps (k0,k1)(k2,k3)(k4,k5)(k6,0), odd ones (0,k0)(k1,k2)(k3,k4)(k5,k6)) ----
        const u16x2 E0 = {18, 34}, E1 = {48, 56}, E2 = {48, 34}, E3 = {18, 0};
        const u16x2 O0 = {0, 18}, O1 = {34, 48}, O2 = {56, 48}, O3 = {34, 18};
        auto d2 = [](uint32_t d, u16x2 k, uint32_t acc) {
            return __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2, d), k, acc, false);
        };
        for (int t = lane; t < kBlW * 10; t += 64) {
            const int rb = (int)(((float)t + 0.5f) * (1.0f / kBlW)), c = t - kBlW * rb, r0 = 4 * rb;
            const uint32_t* y2 = (const uint32_t*)(hr + c * kHrP + r0);
            const uint32_t q0 = y2[0], q1 = y2[1], q2 = y2[2], q3 = y2[3], q4 = y2[4];
            const uint32_t s0 = d2(q3, E3, d2(q2, E2, d2(q1, E1, d2(q0, E0, 0u))));
            const uint32_t s1 = d2(q3, O3, d2(q2, O2, d2(q1, O1, d2(q0, O0, 0u))));
            const uint32_t s2 = d2(q4, E3, d2(q3, E2, d2(q2, E1, d2(q1, E0, 0u))));
            const uint32_t s3 = d2(q4, O3, d2(q3, O2, d2(q2, O1, d2(q1, O0, 0u))));
            const uint32_t sv[4] = {s0, s1, s2, s3};
#pragma unroll
            for (int o = 0; o < 4; o++) {
                if (r0 + o >= kBlW) break;
                bl[(r0 + o) * kBlW + c] = (uint8_t)((sv[o] + (1u << 15)) >> 16);
            }
        }
    }
    wave_lds_fence();   // each wave works on its own keypoint's LDS only
    TR_PHASE(3, 1)
    if (!active) {
        TR_END(3)
        return;
    }
    const LevelGeom& G = P->lv[l];
    // ---- rBRIEF on the blurred region ----
    const float factorPI = (float)(3.14159265358979323846 / 180.f);
    const float ang = angle * factorPI;
    const float a = glibc_cosf(ang), b = glibc_sinf(ang);
    auto sample = [&](int idx) -> int {
        const float px = (float)kPattern[2 * idx], py = (float)kPattern[2 * idx + 1];
        const int oy = cv_round(px * b + py * a);
        const int ox = cv_round(px * a - py * b);
        return bl[(kBlR + oy) * kBlW + kBlR + ox];
    };
    // lane handles pairs 4*lane .. 4*lane+3  (byte lane>>1, bits (lane&1)*4 ..)
    int nib = 0;
#pragma unroll
    for (int t = 0; t < 4; t++) {
        const int pair = 4 * lane + t;
        const int t0 = sample(2 * pair), t1 = sample(2 * pair + 1);
        nib |= (t0 < t1) << t;
    }
    const int other = __shfl_xor(nib, 1, 64);
    TR_PHASE(3, 2)
    TR_END(3)
    const int lapflag = (kp.srl >> 8) & 1;
    const int rank = (int)(kp.srl >> 9);
    const int idx = lapflag ? (total - 1 - (lap_base + rank)) : (mono_base + rank);
    if (idx >= cap) return;
    if ((lane & 1) == 0) out_desc[((int64_t)f * cap + idx) * 32 + (lane >> 1)] = (uint8_t)(nib | (other << 4));
    if (lane == 0) {
        orbhip_kp o;
        const float sc = G.scale;
        o.x = (l == 0) ? (float)cx : (float)cx * sc;
        o.y = (l == 0) ? (float)cy : (float)cy * sc;
        o.size = (float)G.patch_size;
        o.angle = angle;
        o.response = (float)(kp.srl & 0xFF);
        o.octave = l;
        out_kps[(int64_t)f * cap + idx] = o;
    }
}

// k_desc_kp: the same computation with ONE KEYPOINT PER WORK-GROUP (4 waves). At small batches
// (C2: ~1000 keypoints, one frame) k_desc's single wave per keypoint is issue-bound on its own
// instruction stream while most of the chip idles; here the patch load, the IC_Angle disc, both
// blur passes and the 256 rBRIEF pairs are spread over 256 threads, and each wave's 64 pair bits
// leave as one ballot (bytes 8w..8w+7 of the descriptor).
__global__ __launch_bounds__(256) void k_desc_kp(const ExtractPlan* __restrict__ P, FrameBufs fb,
                                                 const LevelKp* __restrict__ lvl_kp, const int* __restrict__ lvl_cnt,
                                                 const int* __restrict__ lvl_nlap, const int* __restrict__ disc,
                                                 orbhip_kp* __restrict__ out_kps, uint8_t* __restrict__ out_desc,
                                                 int cap, int* __restrict__ n_out, int* __restrict__ mono_out, int xrun,
                                                 int nlev) {
    // the k_desc layouts: patch rows of kDpP bytes offset by sh, row-pass sums transposed, the
    // blurred region over the dead patch
    __shared__ __attribute__((aligned(16))) uint8_t pt[kPatchW * kDpP + 16];
    __shared__ __attribute__((aligned(16))) uint16_t hr[kBlW * kHrP];
    uint8_t* const bl = pt;
    __shared__ int msum[2][4];
    TR_BEGIN()
    const int X = gridDim.x, lg = xcd_runs(blockIdx.x + X * blockIdx.y, X * gridDim.y, xrun < 0 ? X : xrun);
    const int f = lg / X;
    const int tid = threadIdx.x, wid = tid >> 6, lane = tid & 63;
    // Every load that needs only the kernel arguments goes out first, together (one round trip
    // after the arguments instead of a chain of five): the keypoint record (slot lg % X of the
    // frame's kp_slots_total = X slots), the IC_Angle disc offsets (zero-padded to 4 x 256 entries
    // on the host: a (0, 0) entry adds nothing), the level capacities and the frame's counts
    // (L = nlev, a launch argument, so their addresses wait for nothing)
    constexpr int kDiscU = 4;
    const int slot0 = lg % X;
    const LevelKp kp = lvl_kp[(int64_t)f * X + slot0];
    int dv[kDiscU];
#pragma unroll
    for (int u = 0; u < kDiscU; u++) dv[u] = disc[tid + 256 * u];
    const int L = nlev;
    int slot = slot0, total = 0, nlap_tot = 0, l = 0, mono_base = 0, lap_base = 0, cnt_l = 0;
    constexpr int kDescL = 8;   // levels walked from registers (more: the loop below)
    if (L <= kDescL) {
        int capv[kDescL], cntv[kDescL], nlv[kDescL];
#pragma unroll
        for (int q = 0; q < kDescL; q++) {
            const int lc = min(q, L - 1);
            capv[q] = P->lv[lc].kp_cap;
            cntv[q] = lvl_cnt[f * L + lc];
            nlv[q] = lvl_nlap[f * L + lc];
        }
        bool go = true;
#pragma unroll
        for (int q = 0; q < kDescL; q++) {
            if (q < L) {
                total += cntv[q];
                nlap_tot += nlv[q];
                if (go && slot >= capv[q]) {
                    slot -= capv[q];
                    mono_base += cntv[q] - nlv[q];
                    lap_base += nlv[q];
                    l = q + 1;
                } else {
                    go = false;
                }
            }
        }
#pragma unroll
        for (int q = 0; q < kDescL; q++) cnt_l = q == l ? cntv[q] : cnt_l;
    } else {
        for (int q = 0; q < L; q++) { total += lvl_cnt[f * L + q]; nlap_tot += lvl_nlap[f * L + q]; }
        while (l < L && slot >= P->lv[l].kp_cap) {
            slot -= P->lv[l].kp_cap;
            mono_base += lvl_cnt[f * L + l] - lvl_nlap[f * L + l];
            lap_base += lvl_nlap[f * L + l];
            l++;
        }
        cnt_l = l < L ? lvl_cnt[f * L + l] : 0;
    }
    if (slot0 == 0 && tid == 0) {
        n_out[f] = total;
        mono_out[f] = total - nlap_tot;
    }
    if (!(l < L && slot < cnt_l)) return;   // block-uniform
    const LevelGeom& G = P->lv[l];
    const int cx = kp.x, cy = kp.y;
    int sh = 0;
    {
        ImgRef im = level_img(P, fb, f, l);
        const int lw = G.w, lh = G.h;
        const bool inside = cx - kPatchR >= 0 && cy - kPatchR >= 0 && cx + kPatchR < lw && cy + kPatchR < lh;
        if (inside && ((im.pitch & 3) == 0) && ((((uintptr_t)im.p) & 3) == 0)) {
            // 43 rows x 12 aligned dwords, 3 per thread
            const uint8_t* src = im.p + (int64_t)(cy - kPatchR) * im.pitch + (cx - kPatchR);
            sh = (int)(((uintptr_t)src) & 3);
            const uint32_t* s4 = (const uint32_t*)(src - sh);
            const int p4 = im.pitch >> 2;
            constexpr int kND = kPatchW * (kDpP / 4), kDU = (kND + 255) / 256;
            uint32_t v[kDU];
#pragma unroll
            for (int u = 0; u < kDU; u++) {
                const int i = min(tid + 256 * u, kND - 1);
                const int r = (i * 43691) >> 19, k = i - 12 * r;   // i / 12 for i < 98304
                v[u] = s4[(int64_t)r * p4 + k];
            }
#pragma unroll
            for (int u = 0; u < kDU; u++)
                if (tid + 256 * u < kND) ((uint32_t*)pt)[tid + 256 * u] = v[u];
        } else {
            constexpr int kPU = (kPatchW * kPatchW + 255) / 256;   // 8 bytes per thread
            constexpr float kInvPW = 1.0f / kPatchW;
            uint8_t v[kPU];
            int li[kPU];
#pragma unroll
            for (int u = 0; u < kPU; u++) {
                const int i = min(tid + 256 * u, kPatchW * kPatchW - 1);   // branch-free loads
                const int py = (int)(((float)i + 0.5f) * kInvPW), px = i - py * kPatchW;
                int yy = cy - kPatchR + py, xx = cx - kPatchR + px;
                // BORDER_REFLECT_101 (levels are >= 43 px in both dims)
                yy = yy < 0 ? -yy : (yy >= lh ? 2 * lh - 2 - yy : yy);
                xx = xx < 0 ? -xx : (xx >= lw ? 2 * lw - 2 - xx : xx);
                v[u] = im.p[(int64_t)yy * im.pitch + xx];
                li[u] = py * kDpP + px;
            }
#pragma unroll
            for (int u = 0; u < kPU; u++)
                if (tid + 256 * u < kPatchW * kPatchW) pt[li[u]] = v[u];
        }
    }
    __syncthreads();
    TR_PHASE(3, 0)
    // ---- IC_Angle partial moments over the umax disc (unblurred level) + blur row pass ----
    {
        int m10 = 0, m01 = 0;
#pragma unroll
        for (int q = 0; q < kDiscU; q++) {
            const int uv = dv[q];
            const int u = (int)(int16_t)(uv & 0xFFFF), vv = (int)(int16_t)(uv >> 16);
            const int val = pt[(kPatchR + vv) * kDpP + sh + kPatchR + u];
            m10 += u * val;
            m01 += vv * val;
        }
        m10 = wave_sum_i32(m10);
        m01 = wave_sum_i32(m01);
        if (lane == 0) { msum[0][wid] = m10; msum[1][wid] = m01; }
        // row pass as in k_desc: realigned dwords, two v_dot4_u32_u8 per output, stored transposed
        const uint32_t K0 = 18u | 34u << 8 | 48u << 16 | 56u << 24, K1 = 48u | 34u << 8 | 18u << 16;
        const uint32_t* p4 = (const uint32_t*)pt;
        for (int t = tid; t < kPatchW * 10; t += 256) {
            const int r = (t * 6554) >> 16, c0 = 4 * (t - 10 * r);   // t / 10 for t < 16384
            const uint32_t* w = p4 + r * (kDpP / 4) + (c0 >> 2);
            const uint32_t w0 = w[0], w1 = w[1], w2 = w[2], w3 = w[3];
            const uint32_t x0 = __builtin_amdgcn_alignbyte(w1, w0, sh);
            const uint32_t x1 = __builtin_amdgcn_alignbyte(w2, w1, sh);
            const uint32_t x2 = __builtin_amdgcn_alignbyte(w3, w2, sh);
#pragma unroll
            for (int o = 0; o < 4; o++) {
                if (c0 + o >= kBlW) break;
                const uint32_t aq = o == 0 ? x0 : __builtin_amdgcn_alignbyte(x1, x0, o);
                const uint32_t bq = o == 0 ? x1 : __builtin_amdgcn_alignbyte(x2, x1, o);
                const uint32_t h = __builtin_amdgcn_udot4(bq, K1, __builtin_amdgcn_udot4(aq, K0, 0u, false), false);
                hr[(c0 + o) * kHrP + r] = (uint16_t)h;
            }
        }
    }
    __syncthreads();
    // ---- column pass: bl[r][c] = (sum_j k_j hr[r + j][c] + 2^15) >> 16, 4 rows per task, as
    // in k_desc (row pairs as dwords, 4 v_dot2_u32_u16 per output) ----
    {
        const u16x2 E0 = {18, 34}, E1 = {48, 56}, E2 = {48, 34}, E3 = {18, 0};
        const u16x2 O0 = {0, 18}, O1 = {34, 48}, O2 = {56, 48}, O3 = {34, 18};
        auto d2 = [](uint32_t d, u16x2 k, uint32_t acc) {
            return __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2, d), k, acc, false);
        };
        for (int t = tid; t < kBlW * 10; t += 256) {
            const int rb = (int)(((float)t + 0.5f) * (1.0f / kBlW)), c = t - kBlW * rb, r0 = 4 * rb;
            const uint32_t* y2 = (const uint32_t*)(hr + c * kHrP + r0);
            const uint32_t q0 = y2[0], q1 = y2[1], q2 = y2[2], q3 = y2[3], q4 = y2[4];
            const uint32_t sv[4] = {d2(q3, E3, d2(q2, E2, d2(q1, E1, d2(q0, E0, 0u)))),
                                    d2(q3, O3, d2(q2, O2, d2(q1, O1, d2(q0, O0, 0u)))),
                                    d2(q4, E3, d2(q3, E2, d2(q2, E1, d2(q1, E0, 0u)))),
                                    d2(q4, O3, d2(q3, O2, d2(q2, O1, d2(q1, O0, 0u))))};
#pragma unroll
            for (int o = 0; o < 4; o++) {
                if (r0 + o >= kBlW) break;
                bl[(r0 + o) * kBlW + c] = (uint8_t)((sv[o] + (1u << 15)) >> 16);
            }
        }
    }
    __syncthreads();
    TR_PHASE(3, 1)
    // the moments in the reference's summation order do not matter (integers)
    const int m10 = msum[0][0] + msum[0][1] + msum[0][2] + msum[0][3];
    const int m01 = msum[1][0] + msum[1][1] + msum[1][2] + msum[1][3];
    const float angle = fast_atan2((float)m01, (float)m10);
    const float factorPI = (float)(3.14159265358979323846 / 180.f);
    const float ang = angle * factorPI;
    const float a = glibc_cosf(ang), b = glibc_sinf(ang);
    // pair tid: bit (tid & 7) of byte tid >> 3
    int bit;
    {
        const float px0 = (float)kPattern[4 * tid], py0 = (float)kPattern[4 * tid + 1];
        const float px1 = (float)kPattern[4 * tid + 2], py1 = (float)kPattern[4 * tid + 3];
        const int t0 = bl[(kBlR + cv_round(px0 * b + py0 * a)) * kBlW + kBlR + cv_round(px0 * a - py0 * b)];
        const int t1 = bl[(kBlR + cv_round(px1 * b + py1 * a)) * kBlW + kBlR + cv_round(px1 * a - py1 * b)];
        bit = t0 < t1;
    }
    const uint64_t word = __ballot(bit);
    TR_PHASE(3, 2)
    TR_END(3)
    const int lapflag = (kp.srl >> 8) & 1;
    const int rank = (int)(kp.srl >> 9);
    const int idx = lapflag ? (total - 1 - (lap_base + rank)) : (mono_base + rank);
    if (idx >= cap) return;
    if (lane == 0) *(uint64_t*)(out_desc + ((int64_t)f * cap + idx) * 32 + 8 * wid) = word;
    if (tid == 0) {
        orbhip_kp o;
        const float sc = G.scale;
        o.x = (l == 0) ? (float)cx : (float)cx * sc;
        o.y = (l == 0) ? (float)cy : (float)cy * sc;
        o.size = (float)G.patch_size;
        o.angle = angle;
        o.response = (float)(kp.srl & 0xFF);
        o.octave = l;
        out_kps[(int64_t)f * cap + idx] = o;
    }
}

// ---------------------------------------------------------------------------
// host-side launchers
// ---------------------------------------------------------------------------
// Run length of the XCD-aware work-group order (xcd_runs) of the cone / FAST / rBRIEF launches.
// Batches of 8+ frames: -1 = one frame's whole grid row per run, so every frame's tiles / cells /
// keypoints land on ONE XCD and its L2 fetches the frame once (C3 k_fast_cells 835 -> ~183 MB of
// HBM traffic per launch, against 183 MB algorithmic; the time is unchanged, the kernel is
// VALU-bound). Smaller batches: runs of 16. One frame: the plain round-robin order (grouping
// neighbours onto one XCD measured ~1% below it on the 16-camera C2 stream).
// XCD-grouped work-group order (xcd_runs): whole frames per XCD for big batches, runs of 16 for
// small ones, runs of 8 at one frame (r05: at one frame the grouped order measured the same
// 16-camera throughput as round-robin (38.9k / 38.8k frames/s on one box) and cut the PMC bytes
// per launch of k_pyr_cone by 0.7 MB, k_fast_cells 4.16 -> 1.69 MB, k_desc_kp 5.24 -> 3.57 MB:
// neighbouring tiles' shared lines stay in one L2; r02 had measured it ~1% slower)
static int xcd_run_for(int B) {
    static const int env = getenv("ORBHIP_XCD_RUN") ? atoi(getenv("ORBHIP_XCD_RUN")) : -2;
    return env >= -1 ? env : (B >= 8 ? -1 : (B > 1 ? 16 : 8));
}

void launch_resize(const ExtractPlan* dP, const ExtractPlan& hP, const FrameBufs& fb, int B, int l,
                   const int* xofs, const int* xalpha, const int* yofs, const int* ybeta, hipStream_t st) {
    const LevelGeom& D = hP.lv[l];
    dim3 blk(64, 4, 1);
    dim3 grd((D.h + 4 * kRzRows - 1) / (4 * kRzRows), (D.w + 255) / 256, B);
    ORBHIP_LAUNCH(k_resize, grd, blk, 0, st, dP, fb, l, xofs, xalpha, yofs, ybeta);
}

void launch_pyr_flow(const ExtractPlan* dP, const FrameBufs& fb, const int* xofs, const int* xalpha, const int* yofs,
                     const int* ybeta, const PyrFlow& a, hipStream_t st) {
    // persistent work-groups (4 per CU): any grid is deadlock-free (tickets), this one keeps the
    // dispatch short and every CU busy
    const int ntask = a.B * a.boff[kMaxLevels];
    const int grid = std::max(kFlowQ, std::min((ntask + kFlowChunk - 1) / kFlowChunk, 1024));
    ORBHIP_LAUNCH(k_pyr_flow, dim3(grid), dim3(256), 0, st, dP, fb, xofs, xalpha, yofs, ybeta, a);
}

void launch_resize_bands(const ExtractPlan* dP, int nbands, const FrameBufs& fb, int B, int s0, const int2* rows,
                         const int* xofs, const int* xalpha, const int* yofs, const int* ybeta, hipStream_t st) {
    ORBHIP_LAUNCH(k_resize_bands, dim3(nbands, B), dim3(256), 0, st, dP, fb, s0, rows, xofs, xalpha, yofs, ybeta);
}

void launch_pyr_cone(const ExtractPlan* dP, int ntiles, size_t lds, const FrameBufs& fb, int B, const ConeRect* rects,
                     const int* ctab, int tab_stride, hipStream_t st, int s0, int nthreads, const int* xofs,
                     const int* xalpha, const int* yofs, const int* ybeta) {
    static LdsAttrOnce attr;   // per device, thread-safe (dev_attr.h)
    (void)attr.ensure((const void*)k_pyr_cone, 64 * 1024);
    (void)xofs; (void)xalpha; (void)yofs; (void)ybeta;
    // the host's per-tile table copies (r05 also measured the plan's compact per-level tables: 130
    // KB fewer fetched bytes, but every staged entry waited on its level's ConeRect before its
    // table load: 20.8 -> 26.9 us; and in-kernel tables, see pyr_cone_body)
    ORBHIP_LAUNCH(k_pyr_cone, dim3(ntiles, B), dim3(nthreads), lds, st, dP, fb, rects, ctab, tab_stride,
                  xcd_run_for(B), s0);
}

void launch_fast(const ExtractPlan* dP, const ExtractPlan& hP, const CellGeom* cells, const FrameBufs& fb, int B,
                 uint32_t* cand, int* cand_cnt, int* err, hipStream_t st, int nt_hint, CandPack cp) {
    // more threads per cell while the cells alone cannot fill the chip (one frame: ~600 cells on
    // 256 CUs), as many as keep every work-group resident at once (8192 wave slots); 256 once
    // the batch fills the chip; 128 for big batches (C3: 127k cells), where fewer waves per cell
    // idle less at the phase barriers and the compact LDS variant keeps 16 work-groups per CU
    const int ncell = B * hP.n_cells_total;
    // (ORBHIP_FAST_NT pins it per plan; a caller's hint, e.g. the front-end with many cameras, next)
    const int nt = hP.fast_nt ? hP.fast_nt
                              : (nt_hint ? nt_hint
                                         : (ncell <= 512 ? 1024 : (ncell <= 1024 ? 512 : (ncell <= 32768 ? 256 : 128))));
    dim3 grd(hP.n_cells_total, B, 1);
    const int xr = xcd_run_for(B);
    const bool compact = hP.fast_win_rows <= 50 && hP.fast_win_cols <= 45;   // FastShape<50>
#define ORBHIP_FAST_LAUNCH(NTV, WRV) \
    ORBHIP_LAUNCH((k_fast_cells<NTV, WRV>), grd, dim3(NTV), 0, st, dP, cells, fb, cand, cand_cnt, err, xr, cp)
    if (nt == 1024 && compact)
        ORBHIP_FAST_LAUNCH(1024, 50);
    else if (nt == 1024)
        ORBHIP_FAST_LAUNCH(1024, kWinMax);
    else if (nt == 512 && compact)
        ORBHIP_FAST_LAUNCH(512, 50);
    else if (nt == 512)
        ORBHIP_FAST_LAUNCH(512, kWinMax);
    else if (nt == 128 && compact)
        ORBHIP_FAST_LAUNCH(128, 50);
    else if (nt == 128)
        ORBHIP_FAST_LAUNCH(128, kWinMax);
    else if (compact)
        ORBHIP_FAST_LAUNCH(256, 50);
    else
        ORBHIP_FAST_LAUNCH(256, kWinMax);
#undef ORBHIP_FAST_LAUNCH
}

size_t octree_lds_bytes(const ExtractPlan& hP, const OctreeCfg& cfg) {
    size_t off = 0;
    auto carve = [&](size_t bytes) { off += (bytes + 15) & ~size_t(15); };
    const size_t NC = cfg.node_cap;
    carve(64 * 4);
    for (int b = 0; b < 2; b++) { carve(NC * 8); carve(NC * 4); carve(NC * 4); carve(NC * 4); }
    carve(NC * 16); carve(NC * 16); carve(NC * 8);
    carve(NC * 4); carve(NC * 4); carve(NC * 4); carve(NC * 4);
    carve((size_t)cfg.sort_cap * 8);
    carve((size_t)cfg.sort_cap * 8);
    carve((size_t)(hP.max_cells_level + 1) * 4);
    carve((size_t)(hP.max_cells_level + 1) * 4);
    carve((size_t)cfg.key_cap * 4);
    carve((size_t)cfg.key_cap * 2);
    return off;
}

void launch_octree(const ExtractPlan* dP, const ExtractPlan& hP, const CellGeom* cells, const uint16_t* otab,
                   const uint32_t* cand, const uint32_t* cprim,
                   const int* cand_cnt, const int* cand_off, uint32_t* kscratch, uint16_t* nscratch, LevelKp* lvl_kp,
                   int* lvl_cnt, int* lvl_nlap, const OctreeCfg& cfg, int* err, int B, hipStream_t st,
                   unsigned long long* stamp) {
    const size_t lds = octree_lds_bytes(hP, cfg);
    dim3 grd(B, hP.n_levels, 1);
    // threads per level: 512 (r05, C2 alternating runs: level-0 work-group 13.3 us at 512 against
    // 14.0 at 1024 and 13.5 at 256, with the slowest at 15.6; ORBHIP_OCT_NT = 256 / 1024 for A/B)
    static const int nt = [] {
        const char* e = std::getenv("ORBHIP_OCT_NT");
        const int v = e ? std::atoi(e) : 512;
        return (v == 256 || v == 1024) ? v : 512;
    }();
    ORBHIP_LAUNCH(k_octree, grd, dim3(nt), lds, st, dP, cells, otab, cand, cprim, cand_cnt, cand_off, kscratch,
                  nscratch, lvl_kp, lvl_cnt, lvl_nlap, cfg, err, stamp);
}

constexpr int kDescKpMaxSlots = 16384;

void launch_desc(const ExtractPlan* dP, const ExtractPlan& hP, const FrameBufs& fb, const LevelKp* lvl_kp,
                 const int* lvl_cnt, const int* lvl_nlap, const int* disc, orbhip_kp* out_kps, uint8_t* out_desc,
                 int cap, int* n_out, int* mono_out, int B, hipStream_t st) {
    // a keypoint per work-group while the batch leaves the chip mostly idle; a keypoint per wave
    // (4 per work-group) once there are enough keypoints to fill it
    static const int mode = getenv("ORBHIP_DESC_MODE") ? atoi(getenv("ORBHIP_DESC_MODE")) : -1;
    const bool per_wg = mode >= 0 ? mode == 1 : B * hP.kp_slots_total <= kDescKpMaxSlots;
    if (per_wg) {
        ORBHIP_LAUNCH(k_desc_kp, dim3(hP.kp_slots_total, B, 1), dim3(256), 0, st, dP, fb, lvl_kp, lvl_cnt,
                           lvl_nlap, disc, out_kps, out_desc, cap, n_out, mono_out, xcd_run_for(B), hP.n_levels);
        return;
    }
    dim3 grd((hP.kp_slots_total + 3) / 4, B, 1);
    ORBHIP_LAUNCH(k_desc, grd, dim3(256), 0, st, dP, fb, lvl_kp, lvl_cnt, lvl_nlap, disc, out_kps, out_desc,
                       cap, n_out, mono_out, xcd_run_for(B));
}

bool octree_set_lds_limit(size_t bytes) {
    return hipFuncSetAttribute((const void*)k_octree, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes) ==
           hipSuccess;
}

}  // namespace orbhip
