// gfx950 Hamming matcher: U:src/ORBmatcher.cc DescriptorDistance + best/second + ratio +
// TH_LOW acceptance, then the HISTO_LENGTH=30 rotation-consistency filter
// (ComputeThreeMaxima). Order-free over the whole train set.
//
//   k_match_top2    grid (64-query blocks, 256- (64- for one pair) descriptor train chunks, pairs): lane = query
//                   (descriptor in VGPRs), the chunk is staged in LDS and read as broadcasts;
//                   per-lane best/second/index in train order (v_xor + v_bcnt), the 4 waves'
//                   quarter-chunks merged in order, one partial per (pair, chunk, query).
//                   (A 64-bit atomicCAS merge into one record per query was tried: the
//                   cross-XCD atomics cost more than the finish saves.)
//   k_match_finish  one workgroup per pair: merge the partials (lexicographic (best, index),
//                   multiset second), TH_LOW + ratio, 30-bin rotation histogram, three maxima
//                   (one wave), filter, match count.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>

#include "orbhip_device.h"
#include "orbhip_kernels.h"

namespace orbhip {

ORBHIP_TRACE_UNIT(match)

struct MatchView {
    const uint8_t* qd;
    const uint8_t* td;
    const float* qa;
    const float* ta;
    int angle_stride;          // floats between consecutive angles
    int64_t pair_desc_stride;  // bytes between pairs (query and train advance together)
    int64_t pair_angle_stride; // floats between pairs
    const int32_t* nq_arr;     // per pair (nullable)
    const int32_t* nt_arr;
    int nq, nt;
    int64_t out_stride;        // entries between pairs in the outputs
};

constexpr int kTC = 256;     // train descriptors per workgroup chunk (64 per wave): batches
constexpr int kTCSmall = 64; // 16 per wave: one pair (C2), where 256-chunks leave the chip idle
constexpr int kFusedMaxPairs = 4;   // k_match_fused up to this many pairs (the sync scratch holds 64 ints each)

// A chunk partial {best | second << 16, index} (8 B), or packed in 4 B while every train index
// fits 14 bits (pk): best | second << 9 | index << 18 (index 0x3FFF when there is no best), which
// halves the partials' traffic; unpacked to the 8-byte form on read
__device__ __forceinline__ void part_store(uint2* part, int64_t i, int pk, int b, int s, int bi) {
    if (pk) ((uint32_t*)part)[i] = (uint32_t)b | ((uint32_t)s << 9) | ((uint32_t)(b < 256 ? bi : 0x3FFF) << 18);
    else part[i] = make_uint2((uint32_t)b | ((uint32_t)s << 16), (uint32_t)bi);
}
__device__ __forceinline__ uint2 part_load(const uint2* part, int64_t i, int pk) {
    if (!pk) return part[i];
    const uint32_t x = ((const uint32_t*)part)[i];
    const uint32_t b = x & 511u, s = (x >> 9) & 511u;
    return make_uint2(b | (s << 16), b < 256u ? (x >> 18) : 0x7fffffffu);
}

__device__ __forceinline__ void top2_merge(int& b, int& i, int& s, int b2, int i2, int s2) {
    const int nb = (b2 < b || (b2 == b && i2 < i)) ? b2 : b;
    const int ni = (b2 < b || (b2 == b && i2 < i)) ? i2 : i;
    const int ns = min(max(b, b2), min(s, s2));
    b = nb; i = ni; s = ns;
}

// Partial top-2 of 64 queries (one per lane, descriptor in VGPRs) against one TC-descriptor
// train chunk broadcast from LDS; wave w scans its quarter of the chunk in index order (strict <:
// the first index wins), the 4 waves merge in index order. part[(pair, chunk, q)] =
// {best | second << 16, index}.
// xrun > 0 (batches): the dispatch order is remapped (xcd_runs) so that each XCD receives whole
// pairs: a pair's train chunk and query blocks are then read by ONE L2, not by all eight.
template <int TC>
__global__ __launch_bounds__(256) void k_match_top2(MatchView v, uint2* __restrict__ part, int nchunk_cap,
                                                     int part_stride, int xrun, int pk) {
    __shared__ __attribute__((aligned(16))) uint4 tile[TC * 2];
    __shared__ int mb[3][64], mi[3][64], ms[3][64];
    TR_BEGIN()
    const int X = gridDim.x, XY = gridDim.x * gridDim.y;
    const int lg = xcd_runs(blockIdx.x + X * (blockIdx.y + gridDim.y * blockIdx.z), XY * gridDim.z, xrun);
    const int p = lg / XY, bx = lg % X, by = (lg % XY) / X;
    const int nq = v.nq_arr ? v.nq_arr[p] : v.nq;
    const int nt = v.nt_arr ? v.nt_arr[p] : v.nt;
    const int q0 = bx * 64, t0 = by * TC;
    if (q0 >= nq || t0 >= nt) return;   // workgroup-uniform
    const int tid = threadIdx.x, wid = tid >> 6, lane = tid & 63;
    const int tn = min(TC, nt - t0);
    const uint8_t* td = v.td + (int64_t)p * v.pair_desc_stride;
    const uint4* src = (const uint4*)(td + (int64_t)t0 * 32);
    for (int i = tid; i < tn * 2; i += 256) tile[i] = src[i];
    const int q = q0 + lane;
    uint4 qa = make_uint4(0, 0, 0, 0), qb = qa;
    if (q < nq) {
        const uint4* qp = (const uint4*)(v.qd + (int64_t)p * v.pair_desc_stride + (int64_t)q * 32);
        qa = qp[0];
        qb = qp[1];
    }
    __syncthreads();
    int b = 256, bi = 0x7fffffff, s = 256;
    const int w0 = wid * (TC / 4), w1 = min(tn, w0 + TC / 4);
    for (int t = w0; t < w1; t++) {
        const uint4 x = tile[2 * t], y = tile[2 * t + 1];
        const int d = __popc(x.x ^ qa.x) + __popc(x.y ^ qa.y) + __popc(x.z ^ qa.z) + __popc(x.w ^ qa.w) +
                      __popc(y.x ^ qb.x) + __popc(y.y ^ qb.y) + __popc(y.z ^ qb.z) + __popc(y.w ^ qb.w);
        if (d < b) { s = b; b = d; bi = t0 + t; }
        else if (d < s) s = d;
    }
    if (wid > 0) { mb[wid - 1][lane] = b; mi[wid - 1][lane] = bi; ms[wid - 1][lane] = s; }
    __syncthreads();
    if (wid == 0 && q < nq) {
#pragma unroll
        for (int w = 0; w < 3; w++) top2_merge(b, bi, s, mb[w][lane], mi[w][lane], ms[w][lane]);
        part_store(part, ((int64_t)p * nchunk_cap + by) * part_stride + q, pk, b, s, bi);
    }
    TR_END(4)
}

// ComputeThreeMaxima over a 30-bin LDS histogram by one wave. The reference inserts bins in
// index order with strict '>' into a top-3 that starts at 0, so its order is value descending,
// ties by lower index, positive values only: three wave max-reductions of (value << 8 | 255 - i).
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
    v = max(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, true));    // quad_perm [1,0,3,2]
    v = max(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, true));    // quad_perm [2,3,0,1]
    v = max(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x141, 0xF, 0xF, true));   // row_half_mirror
    v = max(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x140, 0xF, 0xF, true));   // row_mirror
    const auto a = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    v = max(a[0], a[1]);
    const auto b = __builtin_amdgcn_permlane32_swap(v, v, false, false);
    return max(b[0], b[1]);
}
__device__ __forceinline__ void three_maxima_wave(const int* hist, int* keep) {
    const int lane = threadIdx.x & 63;
    const int h = lane < 30 ? hist[lane] : 0;
    uint32_t key = h > 0 ? ((uint32_t)h << 8) | (uint32_t)(255 - lane) : 0u;
    uint32_t k[3];
#pragma unroll
    for (int j = 0; j < 3; j++) {
        k[j] = wave_max_u32(key);
        if (key == k[j]) key = 0u;
    }
    const int max1 = (int)(k[0] >> 8), max2 = (int)(k[1] >> 8), max3 = (int)(k[2] >> 8);
    int ind1 = k[0] ? 255 - (int)(k[0] & 0xFF) : -1;
    int ind2 = k[1] ? 255 - (int)(k[1] & 0xFF) : -1;
    int ind3 = k[2] ? 255 - (int)(k[2] & 0xFF) : -1;
    if (max2 < 0.1f * (float)max1) { ind2 = -1; ind3 = -1; }
    else if (max3 < 0.1f * (float)max1) { ind3 = -1; }
    if (lane == 0) { keep[0] = ind1; keep[1] = ind2; keep[2] = ind3; }
}

// One workgroup per pair: merge the chunk partials, apply best <= TH_LOW and best < ratio *
// second, then the HISTO_LENGTH=30 rotation filter (ComputeThreeMaxima). The per-query match and
// bin stay in LDS between the two passes (queries beyond kFinQ re-read). The train angles are
// staged in LDS while the first query's partials and angle are already in flight: one global
// round trip before the merge in the common case (nq <= 1024, <= 16 chunks).
constexpr int kFinQ = 6144;
__global__ __launch_bounds__(1024) void k_match_finish(MatchView v, const uint2* __restrict__ part, int nchunk_cap,
                                                        int part_stride, int tc, int th_low, float ratio,
                                                        int check_orientation, int32_t* __restrict__ match,
                                                        int32_t* __restrict__ best_out, int32_t* __restrict__ second_out,
                                                        int32_t* __restrict__ nmatch, int pk) {
    __shared__ int hist[32];
    __shared__ int keep[3];
    __shared__ int cnt;
    __shared__ int mq[kFinQ];
    __shared__ int8_t bq[kFinQ];
    __shared__ float tang[kFinQ];
    TR_BEGIN()
    const int p = blockIdx.x, nt_ = blockDim.x, tid = threadIdx.x;
    const int nq = v.nq_arr ? v.nq_arr[p] : v.nq;
    const int nt = v.nt_arr ? v.nt_arr[p] : v.nt;
    const int nch = (nt + tc - 1) / tc;
    const float* qa = v.qa + (int64_t)p * v.pair_angle_stride;
    const float* ta = v.ta + (int64_t)p * v.pair_angle_stride;
    int32_t* m = match + (int64_t)p * v.out_stride;
    const float factor = 1.0f / 30;
    const bool tang_lds = nt <= kFinQ;
    uint2 u0[16];
    float qa0 = 0.f;
    if (tid < nq) {
#pragma unroll
        for (int j = 0; j < 16; j++)
            u0[j] = part_load(part, ((int64_t)p * nchunk_cap + min(j, max(nch - 1, 0))) * part_stride + tid, pk);
        qa0 = qa[(int64_t)tid * v.angle_stride];
    }
    if (tang_lds)
        for (int t = tid; t < nt; t += nt_) tang[t] = ta[(int64_t)t * v.angle_stride];
    if (tid < 32) hist[tid] = 0;
    if (tid == 0) cnt = 0;
    __syncthreads();
    auto tangle = [&](int t) { return tang_lds ? tang[t] : ta[(int64_t)t * v.angle_stride]; };
    for (int q = tid; q < nq; q += nt_) {
        int b = 256, bi = 0x7fffffff, s = 256;
        float aq;
        if (q == tid) {
#pragma unroll
            for (int j = 0; j < 16; j++)
                if (j < nch) top2_merge(b, bi, s, (int)(u0[j].x & 0xFFFF), (int)u0[j].y, (int)(u0[j].x >> 16));
            aq = qa0;
        } else {
            aq = qa[(int64_t)q * v.angle_stride];
        }
        for (int c0 = (q == tid ? 16 : 0); c0 < nch; c0 += 16) {
            uint2 u[16];
#pragma unroll
            for (int j = 0; j < 16; j++)
                u[j] = part_load(part, ((int64_t)p * nchunk_cap + min(c0 + j, nch - 1)) * part_stride + q, pk);
#pragma unroll
            for (int j = 0; j < 16; j++)
                if (c0 + j < nch) top2_merge(b, bi, s, (int)(u[j].x & 0xFFFF), (int)u[j].y, (int)(u[j].x >> 16));
        }
        const bool ok = b < 256 && b <= th_low && (float)b < ratio * (float)s;
        const int mt = ok ? bi : -1;
        const int64_t o = (int64_t)p * v.out_stride + q;
        best_out[o] = b;
        second_out[o] = s;
        int bin = -1;
        if (ok && check_orientation) {
            float rot = aq - tangle(bi);
            if (rot < 0.0) rot += 360.0f;
            bin = (int)roundf(rot * factor);
            if (bin == 30) bin = 0;
        }
        // one LDS atomic per distinct bin of the wave (matches crowd into 1-3 bins, and
        // same-address atomics would serialise lane by lane)
        {
            uint64_t todo = __ballot(bin >= 0);
            while (todo) {
                const int b0 = __builtin_amdgcn_readlane(bin, __ffsll((unsigned long long)todo) - 1);
                const uint64_t same = __ballot(bin == b0) & todo;
                if ((tid & 63) == __ffsll((unsigned long long)same) - 1) atomicAdd(&hist[b0], __popcll(same));
                todo &= ~same;
            }
        }
        if (q < kFinQ) { mq[q] = mt; bq[q] = (int8_t)bin; }
        else m[q] = mt;
    }
    TR_PHASE(5, 0)
    __syncthreads();
    TR_PHASE(5, 1)
    if (check_orientation) {
        if (tid < 64) three_maxima_wave(hist, keep);
        __syncthreads();
    }
    TR_PHASE(5, 2)
    int c = 0;
    for (int q = tid; q < nq; q += nt_) {
        int t, bin;
        if (q < kFinQ) { t = mq[q]; bin = bq[q]; }
        else {
            t = m[q];
            bin = -1;
            if (t >= 0 && check_orientation) {
                float rot = qa[(int64_t)q * v.angle_stride] - tangle(t);
                if (rot < 0.0) rot += 360.0f;
                bin = (int)roundf(rot * factor);
                if (bin == 30) bin = 0;
            }
        }
        if (t >= 0 && check_orientation && bin != keep[0] && bin != keep[1] && bin != keep[2]) t = -1;
        m[q] = t;
        c += t >= 0;
    }
    c = wave_sum_i32(c);
    if ((tid & 63) == 0) atomicAdd(&cnt, c);
    __syncthreads();
    if (tid == 0) nmatch[p] = cnt;
    TR_PHASE(5, 3)
    TR_END(5)
}

// ---------------------------------------------------------------------------
// k_match_fused: the whole matcher in one launch, for a few pairs (C2: one frame pair). A
// workgroup takes 16 queries against the pair's whole train set: lane (query = tid & 15,
// slice = tid >> 4) scans trains slice, slice + 64, ... of each 1024-descriptor LDS chunk in
// index order (strict <), the 64 slices merge lexicographically (shuffles inside the wave, then
// 16 wave partials in LDS), so every query's (best, index, second) is final inside its workgroup
// and no chunk partials travel between workgroups. TH_LOW + ratio and the rotation bin follow
// at once (train angles staged in LDS with the first chunk). The last workgroup of the pair
// takes ComputeThreeMaxima of the pair's histogram, filters every query and writes the count.
//
// Cross-workgroup hand-off without an agent-scope fence: on gfx950 a release fence at agent
// scope is a buffer_wbl2 of the whole XCD L2 (~14 us measured here, the L2 still holds the
// pyramid), so everything another workgroup reads goes through device-coherent forms instead
// (every match[o] as an sc1 write-through store, histogram and count by atomicAdd), a vmcnt(0)
// wait orders them before the done-counter increment, and the last workgroup reads them back
// with sc1 loads (MI355X_MICROARCH.md, inter-workgroup visibility, "Valid forms": every store
// of the handed-off words sc1 and drained before the counter, every load of them sc1). r01
// stored the non-tentative match[o] plainly; the last workgroup then read stale words (the
// previous frame's indices, or zeros) as bin-0 tentative matches.
// sync: 64 ints per pair, zero before the first launch: [0] done counter, [1..30] histogram,
// [31] match count; the last workgroup resets them.
// ---------------------------------------------------------------------------
constexpr int kFQ = 16, kFChunk = 1024;

__device__ __forceinline__ void wait_vm_all() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

__global__ __launch_bounds__(1024) void k_match_fused(MatchView v, int th_low, float ratio, int check_orientation,
                                                       int32_t* __restrict__ match, int32_t* __restrict__ best_out,
                                                       int32_t* __restrict__ second_out, int32_t* __restrict__ nmatch,
                                                       int* __restrict__ sync) {
    __shared__ __attribute__((aligned(16))) uint4 tile[kFChunk * 2];
    __shared__ float tang[kFChunk];
    __shared__ int rb[16][kFQ], ri[16][kFQ], rs[16][kFQ];
    __shared__ int hist[32], keep[3], cnt, last;
    TR_BEGIN()
    const int p = blockIdx.y;
    const int nq = v.nq_arr ? v.nq_arr[p] : v.nq;
    const int nt = v.nt_arr ? v.nt_arr[p] : v.nt;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int active = (nq + kFQ - 1) / kFQ;
    int* ps = sync + 64 * p;
    if (nq <= 0) {
        if (blockIdx.x == 0 && tid == 0) nmatch[p] = 0;
        return;
    }
    if ((int)blockIdx.x >= active) return;   // workgroup-uniform
    const int ql = tid & (kFQ - 1), slice = tid >> 4;
    const int q = blockIdx.x * kFQ + ql;
    const float* qa_p = v.qa + (int64_t)p * v.pair_angle_stride;
    const float* ta_p = v.ta + (int64_t)p * v.pair_angle_stride;
    const uint4* src = (const uint4*)(v.td + (int64_t)p * v.pair_desc_stride);
    const bool tang_lds = nt <= kFChunk;
    // every global read of the prologue in flight at once (the descriptors were written by other
    // XCDs a kernel ago: one memory round trip, not four)
    const int tn0 = min(kFChunk, nt);
    uint4 t0 = make_uint4(0, 0, 0, 0), t1 = t0;
    if (tid < tn0 * 2) t0 = src[tid];
    if (tid + 1024 < tn0 * 2) t1 = src[tid + 1024];
    uint4 qa = make_uint4(0, 0, 0, 0), qb = qa;
    float aq = 0.f, at = 0.f;
    if (q < nq) {
        const uint4* qp = (const uint4*)(v.qd + (int64_t)p * v.pair_desc_stride + (int64_t)q * 32);
        qa = qp[0];
        qb = qp[1];
        if (tid < kFQ) aq = qa_p[(int64_t)q * v.angle_stride];
    }
    if (tang_lds && tid < nt) at = ta_p[(int64_t)tid * v.angle_stride];
    if (tid < 32) hist[tid] = 0;
    if (tid == 0) cnt = 0;
    if (tid < tn0 * 2) tile[tid] = t0;
    if (tid + 1024 < tn0 * 2) tile[tid + 1024] = t1;
    if (tang_lds && tid < nt) tang[tid] = at;
    int b = 256, bi = 0x7fffffff, s = 256;
    TR_PHASE(5, 6)
    for (int c0 = 0; c0 < nt; c0 += kFChunk) {
        const int tn = min(kFChunk, nt - c0);
        if (c0) {
            __syncthreads();   // the previous chunk is read
            for (int i = tid; i < tn * 2; i += 1024) tile[i] = src[(int64_t)c0 * 2 + i];
        }
        __syncthreads();
        for (int t = slice; t < tn; t += 64) {
            const uint4 x = tile[2 * t], y = tile[2 * t + 1];
            const int d = __popc(x.x ^ qa.x) + __popc(x.y ^ qa.y) + __popc(x.z ^ qa.z) + __popc(x.w ^ qa.w) +
                          __popc(y.x ^ qb.x) + __popc(y.y ^ qb.y) + __popc(y.z ^ qb.z) + __popc(y.w ^ qb.w);
            if (d < b) { s = b; b = d; bi = c0 + t; }
            else if (d < s) s = d;
        }
    }
    TR_PHASE(5, 2)
    // slices 4w .. 4w+3 of a query sit in lanes ql, ql+16, ql+32, ql+48 of wave w
#pragma unroll
    for (int o = 16; o <= 32; o <<= 1) {
        const int b2 = __shfl_xor(b, o, 64), i2 = __shfl_xor(bi, o, 64), s2 = __shfl_xor(s, o, 64);
        top2_merge(b, bi, s, b2, i2, s2);
    }
    if (lane < kFQ) { rb[wid][lane] = b; ri[wid][lane] = bi; rs[wid][lane] = s; }
    __syncthreads();
    if (tid < 64) {
        // wave 0: lane ql + 16k merges waves k, k+4, k+8, k+12; then the four lanes of a query
        const int k = lane >> 4;
        b = rb[k][ql]; bi = ri[k][ql]; s = rs[k][ql];
#pragma unroll
        for (int w = k + 4; w < 16; w += 4) top2_merge(b, bi, s, rb[w][ql], ri[w][ql], rs[w][ql]);
#pragma unroll
        for (int o = 16; o <= 32; o <<= 1) {
            const int b2 = __shfl_xor(b, o, 64), i2 = __shfl_xor(bi, o, 64), s2 = __shfl_xor(s, o, 64);
            top2_merge(b, bi, s, b2, i2, s2);
        }
    }
    if (tid < kFQ) {
        if (q < nq) {
            const bool ok = b < 256 && b <= th_low && (float)b < ratio * (float)s;
            const int64_t o = (int64_t)p * v.out_stride + q;
            best_out[o] = b;
            second_out[o] = s;
            int mt = ok ? bi : -1;
            if (ok && check_orientation) {
                float rot = aq - (tang_lds ? tang[bi] : ta_p[(int64_t)bi * v.angle_stride]);
                if (rot < 0.0) rot += 360.0f;
                int bin = (int)roundf(rot * (1.0f / 30));
                if (bin == 30) bin = 0;
                atomicAdd(&hist[bin], 1);
                mt |= bin << 24;   // tentative: the last workgroup filters
            }
            // With the rotation filter on, the last workgroup reads back EVERY match[o] of the
            // pair, so every one of them (tentative, rejected -1 and all) leaves as an sc1
            // write-through store: a plain store could still sit dirty in this XCD's L2 while the
            // last workgroup, on another XCD, reads the buffer's previous contents. Without the
            // filter nobody in this launch reads match[], and a plain store is enough.
            if (check_orientation)
                __hip_atomic_store(&match[o], mt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            else
                match[o] = mt;
            if (ok) atomicAdd(&cnt, 1);
        }
    }
    // LDS only (hist, cnt): __syncthreads() would also drain every thread's global stores here,
    // one write-through round trip before the histogram atomics go out; wait_vm_all() below
    // orders them all before the done counter
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    TR_PHASE(5, 3)
    if (tid < 30 && hist[tid]) atomicAdd(&ps[1 + tid], hist[tid]);
    if (tid == 0 && cnt) atomicAdd(&ps[31], cnt);
    wait_vm_all();      // this thread's device atomics are performed
    __syncthreads();    // ... for every thread of the workgroup
    if (tid == 0) last = atomicAdd(&ps[0], 1) == active - 1;
    __syncthreads();
    TR_PHASE(5, 0)
    if (!last) {
        TR_END(5)
        return;
    }
    if (!check_orientation) {
        if (tid == 0) {
            nmatch[p] = atomicExch(&ps[31], 0);
            (void)atomicExch(&ps[0], 0);
        }
        return;
    }
    if (tid < 30) hist[tid] = atomicAdd(&ps[1 + tid], 0);
    if (tid == 0) cnt = 0;
    __syncthreads();
    if (tid < 64) three_maxima_wave(hist, keep);
    __syncthreads();
    int c = 0;
    for (int qq = tid; qq < nq; qq += 1024) {
        const int64_t o = (int64_t)p * v.out_stride + qq;
        int mt = __hip_atomic_load(&match[o], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // sc1: written sc1 above
        if (mt >= 0) {
            const int bin = mt >> 24;
            mt &= 0xFFFFFF;
            if (bin != keep[0] && bin != keep[1] && bin != keep[2]) mt = -1;
            match[o] = mt;
            c += mt >= 0;
        }
    }
    c = wave_sum_i32(c);
    if (lane == 0 && c) atomicAdd(&cnt, c);
    if (tid < 32) (void)atomicExch(&ps[tid], 0);   // counter + histogram + count for the next launch
    __syncthreads();
    if (tid == 0) nmatch[p] = cnt;
    TR_PHASE(5, 1)
    TR_END(5)
}

size_t match_part_entries(int npairs, int max_q, int max_t) {
    const int nch = std::max(1, (max_t + kTCSmall - 1) / kTCSmall);
    return (size_t)std::max(npairs, 1) * nch * std::max(max_q, 1);
}

static bool match_xcd_on() {
    const char* e = std::getenv("ORBHIP_MATCH_XCD");
    return !(e && e[0] == '0');
}

static void run_match(const MatchView& v, int npairs, int max_q, int max_t, int th_low, float ratio,
                      int check_orientation, int32_t* match, int32_t* best, int32_t* second, int32_t* nmatch,
                      uint2* part, hipStream_t st, StageTimer* timer = nullptr, int* sync = nullptr) {
    if (npairs <= 0) return;
    const char* unf = std::getenv("ORBHIP_MATCH_UNFUSED");   // A/B switch (read per call: tests flip it)
    if (sync && npairs <= kFusedMaxPairs && !(unf && unf[0] && unf[0] != '0')) {
        if (timer) timer->begin(5, st);
        ORBHIP_LAUNCH(k_match_fused, dim3((unsigned)std::max(1, (max_q + kFQ - 1) / kFQ), npairs), dim3(1024),
                           0, st, v, th_low, ratio, check_orientation, match, best, second, nmatch, sync);
        if (timer) timer->end(5, st);
        return;
    }
    const int qblocks = (max_q + 63) / 64;
    // 16 trains per wave while 64 per wave would leave most of the chip idle (one pair)
    const bool small = (int64_t)npairs * qblocks * ((max_t + kTC - 1) / kTC) < 512;
    // batches: trains per chunk (ORBHIP_MATCH_TC = 256 / 512 / 1024, read per call; A/B): bigger
    // chunks write fewer (query, chunk) partials
    const char* e_tc = std::getenv("ORBHIP_MATCH_TC");
    const int tcb = e_tc ? std::atoi(e_tc) : kTC;
    const int tc = small ? kTCSmall : (tcb == 512 || tcb == 1024 ? tcb : kTC);
    const int nch = std::max(1, (max_t + tc - 1) / tc);
    const int pk = max_t <= 0x3FFF ? 1 : 0;   // 4-byte partials while train indices fit 14 bits
    if (timer) timer->begin(5, st);
    if (qblocks > 0 && max_t > 0) {
        if (small)
            ORBHIP_LAUNCH(k_match_top2<kTCSmall>, dim3(qblocks, nch, npairs), dim3(256), 0, st, v, part, nch,
                               max_q, 0, pk);
        else if (tc == 1024)   // batches: whole pairs per XCD (ORBHIP_MATCH_XCD=0: the plain round-robin order)
            ORBHIP_LAUNCH(k_match_top2<1024>, dim3(qblocks, nch, npairs), dim3(256), 0, st, v, part, nch, max_q,
                          match_xcd_on() && npairs >= 8 ? qblocks * nch : 0, pk);
        else if (tc == 512)
            ORBHIP_LAUNCH(k_match_top2<512>, dim3(qblocks, nch, npairs), dim3(256), 0, st, v, part, nch, max_q,
                          match_xcd_on() && npairs >= 8 ? qblocks * nch : 0, pk);
        else
            ORBHIP_LAUNCH(k_match_top2<kTC>, dim3(qblocks, nch, npairs), dim3(256), 0, st, v, part, nch, max_q,
                          match_xcd_on() && npairs >= 8 ? qblocks * nch : 0, pk);
    }
    if (timer) { timer->end(5, st); timer->begin(6, st); }
    ORBHIP_LAUNCH(k_match_finish, dim3(npairs), dim3(1024), 0, st, v, part, nch, max_q, tc, th_low, ratio,
                       check_orientation, match, best, second, nmatch, pk);
    if (timer) timer->end(6, st);
}

void launch_match_pairs(const orbhip_kp* kps, const uint8_t* desc, const int32_t* n, int npairs, int cap,
                        int th_low, float ratio, int check_orientation, int32_t* match, int32_t* best,
                        int32_t* second, int32_t* nmatch, void* part, hipStream_t st, StageTimer* timer,
                        int* sync) {
    MatchView v;
    v.qd = desc;
    v.td = desc + (int64_t)cap * 32;
    v.qa = &kps[0].angle;
    v.ta = &kps[cap].angle;
    v.angle_stride = (int)(sizeof(orbhip_kp) / sizeof(float));
    v.pair_desc_stride = (int64_t)cap * 32;
    v.pair_angle_stride = (int64_t)cap * v.angle_stride;
    v.nq_arr = n;
    v.nt_arr = n + 1;
    v.nq = cap;
    v.nt = cap;
    v.out_stride = cap;
    run_match(v, npairs, cap, cap, th_low, ratio, check_orientation, match, best, second, nmatch, (uint2*)part, st,
              timer, sync);
}

void launch_match_frames(const orbhip_kp* q_kps, const uint8_t* q_desc, const int32_t* nq, const orbhip_kp* t_kps,
                         const uint8_t* t_desc, const int32_t* nt, int cap, int th_low, float ratio,
                         int check_orientation, int32_t* match, int32_t* best, int32_t* second, int32_t* nmatch,
                         void* part, hipStream_t st, StageTimer* timer, int* sync) {
    MatchView v;
    v.qd = q_desc;
    v.td = t_desc;
    v.qa = &q_kps[0].angle;
    v.ta = &t_kps[0].angle;
    v.angle_stride = (int)(sizeof(orbhip_kp) / sizeof(float));
    v.pair_desc_stride = 0;
    v.pair_angle_stride = 0;
    v.nq_arr = nq;
    v.nt_arr = nt;
    v.nq = cap;
    v.nt = cap;
    v.out_stride = 0;
    run_match(v, 1, cap, cap, th_low, ratio, check_orientation, match, best, second, nmatch, (uint2*)part, st, timer,
              sync);
}

void launch_match_bf(const uint8_t* q, const float* qa, int nq, const uint8_t* t, const float* ta, int nt,
                     int th_low, float ratio, int check_orientation, int32_t* match, int32_t* best,
                     int32_t* second, int32_t* nmatch, void* part, hipStream_t st, int* sync) {
    MatchView v;
    v.qd = q; v.td = t; v.qa = qa; v.ta = ta;
    v.angle_stride = 1;
    v.pair_desc_stride = 0;
    v.pair_angle_stride = 0;
    v.nq_arr = nullptr; v.nt_arr = nullptr;
    v.nq = nq; v.nt = nt;
    v.out_stride = 0;
    run_match(v, 1, nq, nt, th_low, ratio, check_orientation, match, best, second, nmatch, (uint2*)part, st, nullptr,
              sync);
}

// ---- test hooks: device glibc sinf/cosf restatement ----
__global__ void k_sincos_probe(const float* x, float* c, float* s, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) { c[i] = glibc_cosf(x[i]); s[i] = glibc_sinf(x[i]); }
}

void launch_sincos_probe(const float* x, float* c, float* s, int64_t n, hipStream_t st) {
    hipLaunchKernelGGL(k_sincos_probe, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, x, c, s, n);
}

__global__ void k_sincos_sweep(uint32_t lo, uint32_t hi, const float* rc, const float* rs, unsigned long long* mism) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t u = lo + i;
    if (u > hi) return;
    const float x = __uint_as_float(u);
    const bool bad = glibc_cosf(x) != rc[i] || glibc_sinf(x) != rs[i];
    if (bad) atomicAdd(mism, 1ull);
}

void launch_sincos_sweep(uint32_t lo_bits, uint32_t hi_bits, const float* ref_c, const float* ref_s,
                         unsigned long long* mismatches, hipStream_t st) {
    const uint64_t n = (uint64_t)hi_bits - lo_bits + 1;
    hipLaunchKernelGGL(k_sincos_sweep, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, lo_bits, hi_bits, ref_c,
                       ref_s, mismatches);
}

}  // namespace orbhip
