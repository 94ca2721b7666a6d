// Projection-guided matching:
//   U:src/ORBmatcher.cc::SearchByProjection(Frame& CurrentFrame, const Frame& LastFrame, th, bMono)
//   U:src/Frame.cc::Frame::isInFrustum + ORBmatcher::SearchByProjection(Frame& F,
//       const vector<MapPoint*>& vpMapPoints, th, bFarPoints, thFarPoints)
// with the frame grid of U:src/Frame.cc (AssignFeaturesToGrid, PosInGrid, GetFeaturesInArea).
//
// MI355X formulation. The grid walk "cells ix (outer), iy, then cell order" is a total order on
// the frame's keypoints: key = (cell = px * 48 + py) << 16 | index, and a keypoint is visited
// iff its cell lies in the query's cell rectangle. So instead of CSR cell lists, ONE WAVEFRONT
// PER QUERY scans the frame's keypoints (lanes over keypoints, the query descriptor in
// registers), applies the rectangle / level / |dx|,|dy| < r tests, and keeps the lexicographic
// (distance, key) top-2 with levels; a wave merge then gives exactly the reference's best and
// second best (strict <, first in walk order wins).
// The reference is greedy: a current keypoint matched by an earlier query is skipped by later
// ones. That sequential dependence is resolved by a fixed point over parallel rounds: every round
// recomputes all queries with the exclusion "claimed by an earlier query in the previous round's
// picks" (owner[k] < i, an atomicMin over the picks); query i is final once queries < i are, and
// a round that changes nothing is exactly the sequential result (each pick equals its greedy
// definition given the picks before it). Typically 2-3 rounds.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../include/orbhip.h"
#include "dev_attr.h"
#include "orbhip_device.h"
#include "orbhip_kernels.h"
#include "proj.h"

namespace orbhip {

ORBHIP_TRACE_UNIT(proj)   // kernel id 7: k_proj_lists (phases 1-3), its resolving work-group (16-20)

namespace {

constexpr int kGridCols = 64, kGridRows = 48, kThHigh = 100, kHisto = 30;

struct ProjFrame {     // the current Frame
    int n;
    float minx, maxx, miny, maxy, invw, invh;
    float q[4], t[3], fx, fy, cx, cy;
    float R[9], Ow[3];   // mRcw, mOw (isInFrustum)
};
struct Query {         // one projected MapPoint: GetFeaturesInArea(u, v, r, minL, maxL)
    float u, v, r;
    int minL, maxL, valid;
};

// Eigen QuaternionBase::_transformVector, float
__device__ __forceinline__ void qrotf(const float q[4], const float v[3], float o[3]) {
    float uv[3] = {q[1] * v[2] - q[2] * v[1], q[2] * v[0] - q[0] * v[2], q[0] * v[1] - q[1] * v[0]};
    uv[0] += uv[0]; uv[1] += uv[1]; uv[2] += uv[2];
    const float c[3] = {q[1] * uv[2] - q[2] * uv[1], q[2] * uv[0] - q[0] * uv[2], q[0] * uv[1] - q[1] * uv[0]};
    o[0] = v[0] + q[3] * uv[0] + c[0];
    o[1] = v[1] + q[3] * uv[1] + c[1];
    o[2] = v[2] + q[3] * uv[2] + c[2];
}

// PosInGrid: cell = px * 48 + py, -1 outside the grid
__global__ void k_proj_cells(ProjFrame f, const orbhip_kp* __restrict__ kps, int* __restrict__ cell) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= f.n) return;
    const int px = (int)roundf((kps[k].x - f.minx) * f.invw);
    const int py = (int)roundf((kps[k].y - f.miny) * f.invh);
    cell[k] = (px < 0 || px >= kGridCols || py < 0 || py >= kGridRows) ? -1 : px * kGridRows + py;
}

// SearchByProjection(CurrentFrame, LastFrame, th, bMono): window th * scale[lastOctave], levels
// lastOctave - 1 .. lastOctave + 1
struct PrepLast {
    const float* pts;
    const int* oct;
    const float* scale;
    float th;
};
__device__ __forceinline__ Query prep_last(const ProjFrame& f, const PrepLast& a, int i) {
    Query Q{0, 0, 0, 0, 0, 0};
    const float P[3] = {a.pts[3 * i], a.pts[3 * i + 1], a.pts[3 * i + 2]};
    float Xc[3];
    qrotf(f.q, P, Xc);
    Xc[0] += f.t[0]; Xc[1] += f.t[1]; Xc[2] += f.t[2];
    const float invzc = (float)(1.0 / (double)Xc[2]);
    if (!(invzc < 0)) {
        const float u = f.fx * Xc[0] / Xc[2] + f.cx, v = f.fy * Xc[1] / Xc[2] + f.cy;
        if (!(u < f.minx || u > f.maxx || v < f.miny || v > f.maxy)) {
            const int lo = a.oct[i];
            Q = Query{u, v, a.th * a.scale[lo], lo - 1, lo + 1, 1};
        }
    }
    return Q;
}
__global__ void k_proj_prep_last(ProjFrame f, int nq, PrepLast a, Query* __restrict__ qs) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nq) return;
    qs[i] = prep_last(f, a, i);
}

// Frame::isInFrustum(pMP, viewCosLimit) + the window of SearchByProjection(F, vpMapPoints, ...)
struct PrepLocal {
    const float *pts, *nrm, *mind, *maxd;
    const uint8_t* skip;
    const float* scale;
    int n_levels;
    float log_sf, view_cos_limit, th;
    int far_points;
    float th_far;
};
__device__ __forceinline__ Query prep_local(const ProjFrame& f, const PrepLocal& a, int m, uint8_t* iv_out,
                                            int* lvl_out) {
    Query Q{0, 0, 0, 0, 0, 0};
    uint8_t iv = 0;
    int lvl = -1;
    do {
        if (a.skip && a.skip[m]) break;
        const float* P = a.pts + 3 * m;
        const float* R = f.R;
        const float Pc[3] = {R[0] * P[0] + R[1] * P[1] + R[2] * P[2] + f.t[0],
                             R[3] * P[0] + R[4] * P[1] + R[5] * P[2] + f.t[1],
                             R[6] * P[0] + R[7] * P[1] + R[8] * P[2] + f.t[2]};
        const float Pc_dist = sqrtf(Pc[0] * Pc[0] + Pc[1] * Pc[1] + Pc[2] * Pc[2]);
        if (Pc[2] < 0.0f) break;
        const float u = f.fx * Pc[0] / Pc[2] + f.cx, v = f.fy * Pc[1] / Pc[2] + f.cy;
        if (u < f.minx || u > f.maxx) break;
        if (v < f.miny || v > f.maxy) break;
        const float PO[3] = {P[0] - f.Ow[0], P[1] - f.Ow[1], P[2] - f.Ow[2]};
        const float dist = sqrtf(PO[0] * PO[0] + PO[1] * PO[1] + PO[2] * PO[2]);
        const float maxDistance = 1.2f * a.maxd[m], minDistance = 0.8f * a.mind[m];
        if (dist < minDistance || dist > maxDistance) break;
        const float* Pn = a.nrm + 3 * m;
        const float viewCos = (PO[0] * Pn[0] + PO[1] * Pn[1] + PO[2] * Pn[2]) / dist;
        if (viewCos < a.view_cos_limit) break;
        const float ratio = a.maxd[m] / dist;
        int nScale = (int)ceilf(logf(ratio) / a.log_sf);   // MapPoint::PredictScale
        if (nScale < 0) nScale = 0;
        else if (nScale >= a.n_levels) nScale = a.n_levels - 1;
        iv = 1;
        lvl = nScale;
        if (a.far_points && Pc_dist > a.th_far) break;
        float r = viewCos > 0.998 ? 2.5f : 4.0f;   // RadiusByViewingCos
        if (a.th != 1.0f) r *= a.th;
        Q = Query{u, v, r * a.scale[nScale], nScale - 1, nScale, 1};
    } while (false);
    *iv_out = iv;
    *lvl_out = lvl;
    return Q;
}
__global__ void k_proj_prep_local(ProjFrame f, int nq, PrepLocal a, Query* __restrict__ qs,
                                  uint8_t* __restrict__ in_view, int* __restrict__ level) {
    const int m = blockIdx.x * blockDim.x + threadIdx.x;
    if (m >= nq) return;
    uint8_t iv;
    int lvl;
    qs[m] = prep_local(f, a, m, &iv, &lvl);
    in_view[m] = iv;
    level[m] = lvl;
}

// lexicographic (dist, key) top-2 with the level of each
struct Top2 { int d1, k1, l1, d2, k2, l2; };
__device__ __forceinline__ bool lt(int da, int ka, int db, int kb) { return da < db || (da == db && ka < kb); }
__device__ __forceinline__ void top2_add(Top2& a, int d, int k, int l) {
    if (lt(d, k, a.d1, a.k1)) { a.d2 = a.d1; a.k2 = a.k1; a.l2 = a.l1; a.d1 = d; a.k1 = k; a.l1 = l; }
    else if (lt(d, k, a.d2, a.k2)) { a.d2 = d; a.k2 = k; a.l2 = l; }
}

// Round r of the fixed point, one wave per query. mode 0: LastFrame (best <= TH_HIGH); mode 1:
// local points (best/second, ratio test when both on the same level). owner[k] < i excludes
// keypoints claimed earlier. The owner table rotates through three buffers: round r reads
// own[r % 3] (built from round r-1's picks), builds own[(r+1) % 3] by atomicMin, and clears
// own[(r+2) % 3] for round r+1, so a round is one launch. chg[r] = some pick changed in round r;
// a round whose predecessor changed nothing exits at once (the host launches rounds ahead).
__global__ __launch_bounds__(256) void k_proj_round(ProjFrame f, int nq, int mode, float nnratio, int r,
                                                    const Query* __restrict__ qs, const orbhip_kp* __restrict__ kps,
                                                    const uint8_t* __restrict__ kdesc, const int* __restrict__ cell,
                                                    const uint8_t* __restrict__ claimed, int* __restrict__ own3,
                                                    const uint8_t* __restrict__ qdesc, int* __restrict__ pick,
                                                    int* __restrict__ chg) {
    if (r > 0 && chg[r - 1] == 0) return;   // converged: uniform over the grid
    const int n = f.n;
    const int* __restrict__ owner = own3 + (size_t)(r % 3) * n;
    int* own_next = own3 + (size_t)((r + 1) % 3) * n;
    int* own_clear = own3 + (size_t)((r + 2) % 3) * n;
    for (int k = blockIdx.x * blockDim.x + threadIdx.x; k < n; k += gridDim.x * blockDim.x) own_clear[k] = INT_MAX;
    const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (i >= nq) return;
    const Query Q = qs[i];
    int p = -1;
    if (Q.valid) {
        const int nMinCellX = max(0, (int)floorf((Q.u - f.minx - Q.r) * f.invw));
        const int nMaxCellX = min(kGridCols - 1, (int)ceilf((Q.u - f.minx + Q.r) * f.invw));
        const int nMinCellY = max(0, (int)floorf((Q.v - f.miny - Q.r) * f.invh));
        const int nMaxCellY = min(kGridRows - 1, (int)ceilf((Q.v - f.miny + Q.r) * f.invh));
        const bool any = nMinCellX < kGridCols && nMaxCellX >= 0 && nMinCellY < kGridRows && nMaxCellY >= 0;
        const bool bCheckLevels = (Q.minL > 0) || (Q.maxL >= 0);
        const uint4* qd4 = (const uint4*)(qdesc + 32 * (size_t)i);
        const uint4 qa = qd4[0], qb = qd4[1];
        Top2 t{256, INT_MAX, -1, 256, INT_MAX, -1};
        if (any) {
            for (int k = lane; k < f.n; k += 64) {
                const int c = cell[k];
                if (c < 0) continue;
                const int px = c / kGridRows, py = c - px * kGridRows;
                if (px < nMinCellX || px > nMaxCellX || py < nMinCellY || py > nMaxCellY) continue;
                const orbhip_kp kp = kps[k];
                if (bCheckLevels) {
                    if (kp.octave < Q.minL) continue;
                    if (Q.maxL >= 0 && kp.octave > Q.maxL) continue;
                }
                if (!(fabsf(kp.x - Q.u) < Q.r && fabsf(kp.y - Q.v) < Q.r)) continue;
                if ((claimed && claimed[k]) || owner[k] < i) continue;
                const uint4* kd4 = (const uint4*)(kdesc + 32 * (size_t)k);
                const uint4 ka = kd4[0], kb = kd4[1];
                const int d = __popc(qa.x ^ ka.x) + __popc(qa.y ^ ka.y) + __popc(qa.z ^ ka.z) + __popc(qa.w ^ ka.w) +
                              __popc(qb.x ^ kb.x) + __popc(qb.y ^ kb.y) + __popc(qb.z ^ kb.z) + __popc(qb.w ^ kb.w);
                if (d == 256) continue;   // never best (dist < 256) nor second (dist < bestDist2 <= 256)
                top2_add(t, d, (c << 16) | k, kp.octave);
            }
        }
        // wave merge (lexicographic: the order of the merge does not matter)
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            const int d1 = __shfl_xor(t.d1, o, 64), k1 = __shfl_xor(t.k1, o, 64), l1 = __shfl_xor(t.l1, o, 64);
            const int d2 = __shfl_xor(t.d2, o, 64), k2 = __shfl_xor(t.k2, o, 64), l2 = __shfl_xor(t.l2, o, 64);
            top2_add(t, d1, k1, l1);
            top2_add(t, d2, k2, l2);
        }
        if (t.d1 <= kThHigh) {
            if (mode == 0) {
                p = t.k1 & 0xFFFF;
            } else {
                const bool same = t.l1 == t.l2;
                const bool reject = same && (float)t.d1 > nnratio * (float)t.d2;
                if (!reject && (!same || (float)t.d1 <= nnratio * (float)t.d2)) p = t.k1 & 0xFFFF;
            }
        }
    }
    if (lane == 0) {
        if (pick[i] != p) chg[r] = 1;
        pick[i] = p;
        if (p >= 0) atomicMin(&own_next[p], i);   // owner[k] = the first query whose pick is k
    }
}

// the rotation-consistency filter of SearchByProjection(CurrentFrame, LastFrame) and the count
__global__ __launch_bounds__(1024) void k_proj_finish(int nq, int check_orientation, const float* __restrict__ qangle,
                                                      const orbhip_kp* __restrict__ kps, const int* __restrict__ pick,
                                                      int* __restrict__ match, int* __restrict__ nmatch) {
    __shared__ int hist[32], keep[3], cnt;
    if (threadIdx.x < 32) hist[threadIdx.x] = 0;
    if (threadIdx.x == 0) cnt = 0;
    __syncthreads();
    const float factor = 1.0f / kHisto;
    auto bin_of = [&](int i, int k) {
        float rot = qangle[i] - kps[k].angle;
        if (rot < 0.0) rot += 360.0f;
        int b = (int)roundf(rot * factor);
        if (b == kHisto) b = 0;
        return b;
    };
    if (check_orientation) {
        for (int i = threadIdx.x; i < nq; i += blockDim.x)
            if (pick[i] >= 0) atomicAdd(&hist[bin_of(i, pick[i])], 1);
        __syncthreads();
        if (threadIdx.x == 0) {   // ComputeThreeMaxima
            int m1 = 0, m2 = 0, m3 = 0, i1 = -1, i2 = -1, i3 = -1;
            for (int b = 0; b < kHisto; b++) {
                const int s = hist[b];
                if (s > m1) { m3 = m2; m2 = m1; m1 = s; i3 = i2; i2 = i1; i1 = b; }
                else if (s > m2) { m3 = m2; m2 = s; i3 = i2; i2 = b; }
                else if (s > m3) { m3 = s; i3 = b; }
            }
            if (m2 < 0.1f * (float)m1) { i2 = -1; i3 = -1; }
            else if (m3 < 0.1f * (float)m1) { i3 = -1; }
            keep[0] = i1; keep[1] = i2; keep[2] = i3;
        }
        __syncthreads();
    }
    int c = 0;
    for (int i = threadIdx.x; i < nq; i += blockDim.x) {
        int k = pick[i];
        if (k >= 0 && check_orientation) {
            const int b = bin_of(i, k);
            if (b != keep[0] && b != keep[1] && b != keep[2]) k = -1;
        }
        match[i] = k;
        c += k >= 0;
    }
    atomicAdd(&cnt, c);
    __syncthreads();
    if (threadIdx.x == 0) *nmatch = cnt;
}


// ---------------------------------------------------------------------------
// Two-launch form (the default while every candidate list fits kProjCap entries):
//   k_proj_lists    one wave per query: the query's window (prep_last / prep_local), then the
//                   round kernel's tests (cell rectangle, levels, |dx|,|dy| < r, pre-claimed
//                   keypoints, distance < 256) over the frame's keypoints ONCE, the passing
//                   keypoints appended by ballot as (dist << 32 | key << 4 | octave), key =
//                   cell << 16 | index: a u64 compare is the (dist, key) walk order
//   k_proj_resolve  ONE work-group: the fixed point of k_proj_round over the lists (owner tables
//                   in LDS, one barrier per round: a round walks a few list entries per query
//                   instead of scanning the frame), then k_proj_finish's rotation filter / count
// so the search is one upload, two launches and one download. A longer list (status word) sends
// the search to the round kernels with the inputs already on the device.
// ---------------------------------------------------------------------------
constexpr int kProjCap = 128;     // list entries per query
constexpr int kProjMaxN = 8192;   // frame keypoints: staged in LDS (16 B each), 3 owner tables of n ints
constexpr int kProjMaxQ = 8192;   // queries: list offsets in LDS
// queries per k_proj_lists work-group (one per wave of its first kListQ waves; the other waves
// only help stage the frame): one query wave per SIMD, so the scans do not share issue slots
constexpr int kListQ = 4;
// resolve_body's LDS head: 3 owner tables (n), list offsets (nq + 1), picks (nq); the lists follow
__host__ __device__ inline size_t resolve_head_bytes(int n, int nq) {
    return ((size_t)(3 * n + 2 * nq + 1) * 4 + 15) & ~size_t(15);
}
constexpr int kRectCap = 512;   // keypoints in a query's cell rectangle listed per wave (more: every keypoint)
constexpr size_t kListIdxBytes = kListQ * (kProjCap + kRectCap) * 2;   // k_proj_lists' per-wave index lists (LDS)

typedef __attribute__((address_space(1))) int pj_gint;
typedef __attribute__((address_space(1))) unsigned long long pj_gull;
__device__ __forceinline__ void st_ag(uint64_t* p, uint64_t v) {
    __hip_atomic_store((pj_gull*)p, (unsigned long long)v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t ld_ag(const uint64_t* p) {
    return __hip_atomic_load((pj_gull*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_ag(int* p, int v) {
    __hip_atomic_store((pj_gint*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int ld_ag(const int* p) {
    return __hip_atomic_load((pj_gint*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ int proj_decide(const Top2& t, int mode, float nnratio) {
    if (t.d1 > kThHigh) return -1;
    if (mode == 0) return t.k1 & 0xFFFF;
    const bool same = t.l1 == t.l2;
    const bool reject = same && (float)t.d1 > nnratio * (float)t.d2;
    return (!reject && (!same || (float)t.d1 <= nnratio * (float)t.d2)) ? (t.k1 & 0xFFFF) : -1;
}

// the one-launch form: the last work-group of k_proj_lists runs resolve_body (arrive: a counter,
// 0 between launches; fuse 0: the resolve runs as its own launch)
struct ResolveArgs {
    int fuse, check_orientation, ent_cap;
    const float* qangle;
    int* match;
    int* res;
    int* arrive;
};
template <int MODE>
__device__ void resolve_body(unsigned char* rsm, int n, int nq, float nnratio, int check_orientation, int cap,
                             int ent_cap, const float* __restrict__ qangle, const orbhip_kp* __restrict__ kps,
                             const uint64_t* __restrict__ lists, const int* __restrict__ lcnt,
                             const int* __restrict__ pick0, int* __restrict__ match, int* __restrict__ res,
                             unsigned long long* tr = nullptr);

// the frame's keypoints are staged once per work-group in LDS as (x, y, cell << 16 | claimed << 8 |
// octave, 0): PosInGrid computed as k_proj_cells does, a 16-byte read per lane and keypoint. The
// query's window is computed first, so its loads overlap the staging. A list entry is written for
// every keypoint passing the window tests (distance 256 included, skipped by the rounds): the
// ballot does not wait on the descriptor load, so the loads of all the scan's steps overlap.
// Round 0 of the fixed point (no exclusions) is the wave's own top-2: pick0[i].
template <int MODE>
__global__ __launch_bounds__(1024) void k_proj_lists(ProjFrame f, int nq, PrepLast pl, PrepLocal pc, int cap,
                                                     float nnratio, const orbhip_kp* __restrict__ kps,
                                                     const uint8_t* __restrict__ kdesc,
                                                     const uint8_t* __restrict__ claimed,
                                                     const uint8_t* __restrict__ qdesc,
                                                     uint64_t* __restrict__ lists, int* __restrict__ lcnt,
                                                     int* __restrict__ pick0, uint8_t* __restrict__ in_view,
                                                     int* __restrict__ level, ResolveArgs ra) {
    extern __shared__ uint4 kl[];
    TR_BEGIN()
    const int n = f.n, nt = blockDim.x;
    const int w = threadIdx.x >> 6;
    const int i = w < kListQ ? blockIdx.x * kListQ + w : nq;   // nq: no query
    const int lane = threadIdx.x & 63;
    // LDS (list_lds_bytes): kl[n] | kc[n256] cells (u16, 0xFFFF past n) | per-wave index lists
    const int n256 = (n + 255) & ~255;
    uint16_t* kc = (uint16_t*)(kl + n);
    uint16_t* wl = kc + n256 + min(w, kListQ - 1) * kProjCap;
    uint16_t* wr = kc + n256 + kListQ * kProjCap + min(w, kListQ - 1) * kRectCap;
    Query Q{0, 0, 0, 0, 0, 0};
    uint4 qa{0u, 0u, 0u, 0u}, qb{0u, 0u, 0u, 0u};
    uint8_t iv = 0;
    int lvl = 0;
    if (i < nq) {
        if constexpr (MODE == 0) Q = prep_last(f, pl, i);
        else Q = prep_local(f, pc, i, &iv, &lvl);
        const uint4* qd4 = (const uint4*)(qdesc + 32 * (size_t)i);
        qa = qd4[0];
        qb = qd4[1];
    }
    // staging: two keypoints per thread with their loads in flight together (1250 keypoints: one
    // round trip); the cell of each keypoint also into kc
    for (int k0 = threadIdx.x; k0 < n; k0 += 2 * nt) {
        orbhip_kp kp[2];
        uint32_t cl[2];
#pragma unroll
        for (int u = 0; u < 2; u++) {
            const int k = min(k0 + u * nt, n - 1);
            kp[u] = kps[k];
            cl[u] = (claimed && claimed[k]) ? 1u : 0u;
        }
#pragma unroll
        for (int u = 0; u < 2; u++) {
            const int k = k0 + u * nt;
            if (k >= n) break;
            const int px = (int)roundf((kp[u].x - f.minx) * f.invw);
            const int py = (int)roundf((kp[u].y - f.miny) * f.invh);
            const int c = (px < 0 || px >= kGridCols || py < 0 || py >= kGridRows) ? 0xFFFF : px * kGridRows + py;
            kl[k] = uint4{__float_as_uint(kp[u].x), __float_as_uint(kp[u].y), ((uint32_t)c << 16) | (cl[u] << 8) |
                          (uint32_t)(kp[u].octave & 0xFF), 0u};
            kc[k] = (uint16_t)c;
        }
    }
    for (int k = n + threadIdx.x; k < n256; k += nt) kc[k] = 0xFFFF;
    __syncthreads();
    TR_PHASE(7, 1)
    int cnt = 0;
    Top2 t{256, INT_MAX, -1, 256, INT_MAX, -1};
    if (i < nq && Q.valid) {
        const int nMinCellX = max(0, (int)floorf((Q.u - f.minx - Q.r) * f.invw));
        const int nMaxCellX = min(kGridCols - 1, (int)ceilf((Q.u - f.minx + Q.r) * f.invw));
        const int nMinCellY = max(0, (int)floorf((Q.v - f.miny - Q.r) * f.invh));
        const int nMaxCellY = min(kGridRows - 1, (int)ceilf((Q.v - f.miny + Q.r) * f.invh));
        const bool any = nMinCellX < kGridCols && nMaxCellX >= 0 && nMinCellY < kGridRows && nMaxCellY >= 0;
        const bool bCheckLevels = (Q.minL > 0) || (Q.maxL >= 0);
        uint64_t* out = lists + (size_t)i * cap;
        // pass 1, LDS only: the indices of the keypoints passing the window tests into the wave's
        // slice of the index buffer (the first `cap`; the count goes on). Four keypoints per lane
        // and step: their cells are one 8-byte read, and only the few inside the cell rectangle
        // read their 16-byte record for the level / radius / claimed tests
        const uint64_t* kc8 = (const uint64_t*)kc;
        const uint64_t lt = (1ull << lane) - 1ull;
        TR_PHASE(7, 5)
        auto in_rect = [&](int c) {
            const int px = c / kGridRows, py = c - px * kGridRows;   // c = 0xFFFF: px = 1365, out
            return px >= nMinCellX && px <= nMaxCellX && py >= nMinCellY && py <= nMaxCellY;
        };
        // 1a: the cell rectangle alone, four cells per lane from one 8-byte read
        int nr = 0;
        for (int s0 = 0; any && s0 < n; s0 += 256) {
            const uint64_t v = kc8[(s0 >> 2) + lane];
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const bool r = in_rect((int)((v >> (16 * u)) & 0xFFFF));
                const uint64_t m = __ballot(r);
                const int pos = nr + __popcll(m & lt);
                if (r && pos < kRectCap) wr[pos] = (uint16_t)(s0 + 4 * lane + u);
                nr += __popcll(m);
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();
        // 1b: the level / radius / claimed tests on the rectangle's keypoints (every keypoint when
        // the rectangle held more than kRectCap), compacted into wl
        const bool all = nr > kRectCap;
        const int nb = all ? n : nr;
        for (int j0 = 0; any && j0 < nb; j0 += 64) {
            const int j = j0 + lane;
            bool ok = false;
            int k = 0;
            if (j < nb) {
                k = all ? j : (int)wr[j];
                const uint4 e = kl[k];
                const uint32_t oct = e.z & 0xFF;
                const float x = __uint_as_float(e.x), y = __uint_as_float(e.y);
                ok = !all || in_rect((int)(e.z >> 16));
                if (ok && bCheckLevels) ok = (int)oct >= Q.minL && !(Q.maxL >= 0 && (int)oct > Q.maxL);
                ok = ok && fabsf(x - Q.u) < Q.r && fabsf(y - Q.v) < Q.r && !((e.z >> 8) & 1u);
            }
            const uint64_t m = __ballot(ok);
            const int pos = cnt + __popcll(m & lt);
            if (ok && pos < cap) wl[pos] = (uint16_t)k;
            cnt += __popcll(m);
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();
        TR_PHASE(7, 2)
        // pass 2: the descriptor loads of every listed keypoint in flight at once (one round trip
        // instead of one per 64-keypoint step that had a passing lane)
        const int nl = min(cnt, cap);
        int kk[kProjCap / 64];
        uint4 ka[kProjCap / 64], kb[kProjCap / 64];
#pragma unroll
        for (int u = 0; u < kProjCap / 64; u++) {
            const int j = lane + 64 * u;
            kk[u] = j < nl ? (int)wl[j] : -1;
            if (kk[u] >= 0) {
                const uint4* kd4 = (const uint4*)(kdesc + 32 * (size_t)kk[u]);
                ka[u] = kd4[0];
                kb[u] = kd4[1];
            }
        }
#pragma unroll
        for (int u = 0; u < kProjCap / 64; u++) {
            if (kk[u] < 0) continue;
            const int k = kk[u];
            const uint32_t z = kl[k].z, oct = z & 0xFF, key = ((z >> 16) << 16) | (uint32_t)k;
            const int d = __popc(qa.x ^ ka[u].x) + __popc(qa.y ^ ka[u].y) + __popc(qa.z ^ ka[u].z) +
                          __popc(qa.w ^ ka[u].w) + __popc(qb.x ^ kb[u].x) + __popc(qb.y ^ kb[u].y) +
                          __popc(qb.z ^ kb[u].z) + __popc(qb.w ^ kb[u].w);
            st_ag(out + lane + 64 * u, ((uint64_t)d << 32) | (uint64_t)((key << 4) | (oct & 15u)));
            if (d != 256) top2_add(t, d, (int)key, (int)(oct & 15u));
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const int d1 = __shfl_xor(t.d1, o, 64), k1 = __shfl_xor(t.k1, o, 64), l1 = __shfl_xor(t.l1, o, 64);
        const int d2 = __shfl_xor(t.d2, o, 64), k2 = __shfl_xor(t.k2, o, 64), l2 = __shfl_xor(t.l2, o, 64);
        top2_add(t, d1, k1, l1);
        top2_add(t, d2, k2, l2);
    }
    if (lane == 0 && i < nq) {
        st_ag(lcnt + i, cnt);
        st_ag(pick0 + i, proj_decide(t, MODE, nnratio));
    }
    TR_PHASE(7, 3)
    // the in_view / level outputs live in host memory: stored after the arrival's vmcnt drain (and
    // after the resolve in the resolving work-group, whose barriers drain stores), not before it
    auto host_outputs = [&]() {
        if constexpr (MODE == 1)
            if (lane == 0 && i < nq) { in_view[i] = iv; level[i] = lvl; }
    };
    if (!ra.fuse) { host_outputs(); TR_END(7) return; }   // uniform
    // one launch: every wave's list stores drained, then the last work-group to arrive resolves
    __shared__ int lastf;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        const int old = __hip_atomic_fetch_add((pj_gint*)ra.arrive, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        lastf = old == (int)gridDim.x - 1;
        if (lastf) __hip_atomic_store((pj_gint*)ra.arrive, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    TR_PHASE(7, 4)
    if (lastf)
        resolve_body<MODE>((unsigned char*)kl, n, nq, nnratio, ra.check_orientation, cap, ra.ent_cap, ra.qangle, kps,
                           lists, lcnt, pick0, ra.match, ra.res,
                           tr_buf ? tr_buf + 7 * kTraceStride + 8192 + 16 : nullptr);
    host_outputs();
    TR_END(7)
}

// res[0] = matches, res[1] = status (1: a list overflowed, nothing else written), res[2] = rounds.
// LDS rsm: 3 owner tables (n ints), the list offsets (nq ints), then the lists themselves when
// they fit the rest (`ent_cap` entries; else the rounds read them from global memory). The lists,
// their counts and pick0 are read with agent-scope (sc1) loads: in the one-launch form they were
// written by the other work-groups of the same launch.
template <int MODE>
__device__ void resolve_body(unsigned char* rsm, int n, int nq, float nnratio, int check_orientation, int cap,
                             int ent_cap, const float* __restrict__ qangle, const orbhip_kp* __restrict__ kps,
                             const uint64_t* __restrict__ lists, const int* __restrict__ lcnt,
                             const int* __restrict__ pick0, int* __restrict__ match, int* __restrict__ res,
                             unsigned long long* tr) {
    // tr (diagnostics): s_memtime cycles of the resolve's phases, written by thread 0
    unsigned long long tr_p = tr && threadIdx.x == 0 ? __builtin_amdgcn_s_memtime() : 0ull;
    auto mark = [&](int ph) {
        if (tr && threadIdx.x == 0) {
            const unsigned long long t = __builtin_amdgcn_s_memtime();
            tr[ph] = t - tr_p;
            tr_p = t;
        }
    };
    int* own = (int*)rsm;                        // 3 x n
    int* qoff = own + 3 * n;                     // nq + 1: list i = entries [qoff[i], qoff[i + 1])
    int* pk = qoff + nq + 1;                     // nq: the current picks
    uint64_t* ent = (uint64_t*)(rsm + resolve_head_bytes(n, nq));
    __shared__ int flag[4], hist[32], keep[3], cnt, scan[16];
    const int tid = threadIdx.x, nt = blockDim.x;
    if (tid < 4) flag[tid] = 0;
    if (tid < 32) hist[tid] = 0;
    if (tid == 0) cnt = 0;
    for (int k = tid; k < 3 * n; k += nt) own[k] = INT_MAX;
    // list offsets (block scan of the counts, nt queries at a time)
    int over = 0, run = 0;
    for (int i0 = 0; i0 < nq; i0 += nt) {
        const int i = i0 + tid;
        const int c = i < nq ? ld_ag(lcnt + i) : 0;
        const int p0 = i < nq ? ld_ag(pick0 + i) : 0;
        over |= c > cap;
        int tot;
        const int ex = block_excl_scan(c, scan, &tot);
        if (i < nq) { qoff[i] = run + ex; pk[i] = p0; }
        run += tot;
    }
    if (tid == 0) qoff[nq] = run;
    if (over) flag[3] = 1;
    __syncthreads();
    mark(0);
    if (flag[3]) {
        if (tid == 0) res[1] = 1;
        return;
    }
    const bool in_lds = run <= ent_cap;
    // round 0 was k_proj_lists' (pick0): its claims build own[1]
    for (int i = tid; i < nq; i += nt) {
        const int p = pk[i];
        if (p >= 0) atomicMin(&own[n + p], i);
        if (in_lds) {   // 8 loads in flight before their stores (one round trip per 8 entries)
            const int o = qoff[i], c = qoff[i + 1] - o;
            const uint64_t* L = lists + (size_t)i * cap;
            for (int j0 = 0; j0 < c; j0 += 8) {
                uint64_t v[8];
#pragma unroll
                for (int u = 0; u < 8; u++) v[u] = j0 + u < c ? ld_ag(L + j0 + u) : 0ull;
#pragma unroll
                for (int u = 0; u < 8; u++)
                    if (j0 + u < c) ent[o + j0 + u] = v[u];
            }
        }
    }
    __syncthreads();
    mark(1);
    // round r >= 1: reads own[r % 3], builds own[(r+1) % 3], clears own[(r+2) % 3]; flag[r % 3] =
    // some pick changed, and flag[(r+1) % 3] (last read before round r-1's barrier) is reset here
    int r = 1;
    for (; r < nq + 2; r++) {
        const int* owner = own + (r % 3) * n;
        int* own_next = own + ((r + 1) % 3) * n;
        int* own_clear = own + ((r + 2) % 3) * n;
        for (int k = tid; k < n; k += nt) own_clear[k] = INT_MAX;
        if (tid == 0) flag[(r + 1) % 3] = 0;
        int ch = 0;
        for (int i = tid; i < nq; i += nt) {
            const int o = qoff[i], c = qoff[i + 1] - o;
            const uint64_t* L = in_lds ? ent + o : lists + (size_t)i * cap;
            Top2 t{256, INT_MAX, -1, 256, INT_MAX, -1};
            for (int j = 0; j < c; j++) {
                const uint64_t e = in_lds ? L[j] : ld_ag(L + j);
                const uint32_t lo = (uint32_t)e;
                const int d = (int)(e >> 32);
                if (d == 256 || owner[(lo >> 4) & 0xFFFF] < i) continue;
                top2_add(t, d, (int)(lo >> 4), (int)(lo & 15));
            }
            const int p = proj_decide(t, MODE, nnratio);
            ch |= p != pk[i];
            pk[i] = p;
            if (p >= 0) atomicMin(&own_next[p], i);
        }
        if (ch) flag[r % 3] = 1;
        __syncthreads();
        if (!flag[r % 3]) break;
    }
    mark(2);
    // ---- the rotation filter of SearchByProjection(CurrentFrame, LastFrame), the count ----
    const float factor = 1.0f / kHisto;
    auto bin_of = [&](int i, int k) {
        float rot = qangle[i] - kps[k].angle;
        if (rot < 0.0) rot += 360.0f;
        int b = (int)roundf(rot * factor);
        if (b == kHisto) b = 0;
        return b;
    };
    const bool rot = MODE == 0 && check_orientation;
    if (rot) {
        for (int i = tid; i < nq; i += nt)
            if (pk[i] >= 0) atomicAdd(&hist[bin_of(i, pk[i])], 1);
        __syncthreads();
        if (tid == 0) {   // ComputeThreeMaxima
            int m1 = 0, m2 = 0, m3 = 0, i1 = -1, i2 = -1, i3 = -1;
            for (int b = 0; b < kHisto; b++) {
                const int v = hist[b];
                if (v > m1) { m3 = m2; m2 = m1; m1 = v; i3 = i2; i2 = i1; i1 = b; }
                else if (v > m2) { m3 = m2; m2 = v; i3 = i2; i2 = b; }
                else if (v > m3) { m3 = v; i3 = b; }
            }
            if (m2 < 0.1f * (float)m1) { i2 = -1; i3 = -1; }
            else if (m3 < 0.1f * (float)m1) { i3 = -1; }
            keep[0] = i1; keep[1] = i2; keep[2] = i3;
        }
        __syncthreads();
        for (int i = tid; i < nq; i += nt)   // each thread rewrites only its own queries
            if (pk[i] >= 0) {
                const int b = bin_of(i, pk[i]);
                if (b != keep[0] && b != keep[1] && b != keep[2]) pk[i] = -1;
            }
    }
    // the count first, then the stores (match / res may be host memory: no barrier waits on them)
    int c = 0;
    for (int i = tid; i < nq; i += nt) c += pk[i] >= 0;
    c = wave_sum_i32(c);   // one LDS atomic per wave: 1024 same-address atomics serialise
    if ((tid & 63) == 0) atomicAdd(&cnt, c);
    __syncthreads();
    mark(4);
    for (int i = tid; i < nq; i += nt) match[i] = pk[i];
    if (tid == 0) {
        res[0] = cnt;
        res[1] = 0;
        res[2] = r + 1;
    }
    mark(5);
}

template <int MODE>
__global__ __launch_bounds__(1024) void k_proj_resolve(int n, int nq, float nnratio, int check_orientation, int cap,
                                                       int ent_cap, const float* __restrict__ qangle,
                                                       const orbhip_kp* __restrict__ kps,
                                                       const uint64_t* __restrict__ lists,
                                                       const int* __restrict__ lcnt, const int* __restrict__ pick0,
                                                       int* __restrict__ match, int* __restrict__ res) {
    extern __shared__ __attribute__((aligned(16))) unsigned char rsm_[];
    resolve_body<MODE>(rsm_, n, nq, nnratio, check_orientation, cap, ent_cap, qangle, kps, lists, lcnt, pick0, match,
                       res);
}

// ---------------------------------------------------------------------------
// SearchForInitialization(F1, F2, vbPrevMatched, vnMatches12, windowSize)
//   (U:src/ORBmatcher.cc; monocular initialisation, Tracking::MonocularInitialization)
//
// The reference walks the F1 keypoints of octave 0 in index order; each reads and writes the
// per-F2-keypoint state (vMatchedDistance, vnMatches21), so query i depends on every earlier
// query. The device splits that into the state-free part and the chain:
//   k_init_prep     one WG: F2 octave-0 keypoints with a grid cell, ranked in walk order
//                   (cell = px * 48 + py, then index); F1 octave-0 keypoints -> query slots
//   k_init_cands    one wave per query: GetFeaturesInArea(prev, windowSize, 0, 0) as a
//                   rectangle/level/|d| < r test over the ranked F2 keypoints, Hamming distance,
//                   ballot-compacted list of (dist << 21 | rank << 5 | rotation bin), and the
//                   list's 16 smallest entries (per-lane sorted top-4, 16 wave-min extractions)
//   k_init_greedy   one WG: wave 0 runs the chain with the state in LDS. Per query: the
//                   eligible entries (dist < vMatchedDistance[rank]) among its 16 smallest by one
//                   ballot; the first two set bits are the reference's best and second best
//                   whenever two are eligible or the list has <= 16 entries (else the whole list
//                   is scanned, a DPP/permlane top-2 butterfly); TH_LOW / ratio test; the steal
//                   update. Four queries share a 64-lane register, blocks of four are in flight.
//                   Then the whole WG applies the rotation histogram (ComputeThreeMaxima over the
//                   pushes, stale ones included) and writes vnMatches12 / vbPrevMatched.
// (dist, rank) order is the walk order tie-break of "dist < bestDist", and the second-best
// distance is the second element of the multiset, so the chain is exact. The bin of the pair
// (the rotHist push) rides in the low bits, so the chain never touches the keypoints.
// ---------------------------------------------------------------------------
constexpr int kInitCells = kGridCols * kGridRows;   // 3072
constexpr int kThLow = 50;
constexpr int kInitK = 16;   // smallest list entries per query handed to the chain
constexpr int kInitR = 4;    // ring of 4-query blocks in flight in the chain
constexpr int kInitMaxRounds = 64;   // parallel rounds before the chain takes over

// min over the wave, every lane gets it
__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) {
    v = min(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, true));    // quad_perm [1,0,3,2]
    v = min(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, true));    // quad_perm [2,3,0,1]
    v = min(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x141, 0xF, 0xF, true));   // row_half_mirror
    v = min(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x140, 0xF, 0xF, true));   // row_mirror
    const auto a = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    v = min(a[0], a[1]);
    const auto b = __builtin_amdgcn_permlane32_swap(v, v, false, false);
    return min(b[0], b[1]);
}

struct InitGeom {
    int n1, n2;
    float minx, maxx, miny, maxy, invw, invh, r;
    int list_cap;    // entries per query list (>= number of ranked F2 keypoints, multiple of 64)
};

__device__ __forceinline__ int init_cell(const InitGeom& g, float x, float y) {   // PosInGrid
    const int px = (int)roundf((x - g.minx) * g.invw);
    const int py = (int)roundf((y - g.miny) * g.invh);
    return (px < 0 || px >= kGridCols || py < 0 || py >= kGridRows) ? -1 : px * kGridRows + py;
}

// counts[0] = queries (F1 octave 0), counts[1] = ranked F2 keypoints, counts[2] = nmatches
__global__ __launch_bounds__(1024) void k_init_prep(InitGeom g, const orbhip_kp* __restrict__ kps1,
                                                    const orbhip_kp* __restrict__ kps2, int* __restrict__ slot,
                                                    int* __restrict__ qlist, int* __restrict__ counts,
                                                    int* __restrict__ cnt3, int* __restrict__ flags, int nflags) {
    __shared__ int cnt[kInitCells], start[kInitCells], scratch[20], tot;
    const int tid = threadIdx.x, nt = blockDim.x;
    for (int c = tid; c < kInitCells; c += nt) cnt[c] = 0;
    __syncthreads();
    for (int k = tid; k < g.n2; k += nt) {
        const orbhip_kp kp = kps2[k];
        const int c = kp.octave == 0 ? init_cell(g, kp.x, kp.y) : -1;
        if (c >= 0) atomicAdd(&cnt[c], 1);
    }
    __syncthreads();
    // exclusive scan of the 3072 cell counts (3 per thread, in order)
    {
        int v[3], s = 0;
        for (int j = 0; j < 3; j++) { const int c = tid * 3 + j; v[j] = c < kInitCells ? cnt[c] : 0; s += v[j]; }
        int total;
        int base = block_excl_scan(s, scratch, &total);
        for (int j = 0; j < 3; j++) { const int c = tid * 3 + j; if (c < kInitCells) start[c] = base; base += v[j]; }
        if (tid == 0) tot = total;
    }
    __syncthreads();
    for (int c = tid; c < kInitCells; c += nt) cnt[c] = 0;
    __syncthreads();
    for (int k = tid; k < g.n2; k += nt) {
        const orbhip_kp kp = kps2[k];
        const int c = kp.octave == 0 ? init_cell(g, kp.x, kp.y) : -1;
        if (c >= 0) slot[start[c] + atomicAdd(&cnt[c], 1)] = k;
    }
    __syncthreads();
    // index order inside each cell (cells hold a handful of keypoints)
    for (int c = tid; c < kInitCells; c += nt) {
        int* a = slot + start[c];
        const int m = cnt[c];
        for (int i = 1; i < m; i++) {
            const int v = a[i];
            int j = i - 1;
            while (j >= 0 && a[j] > v) { a[j + 1] = a[j]; j--; }
            a[j + 1] = v;
        }
    }
    // F1 octave-0 keypoints in index order
    int run = 0;
    for (int k0 = 0; k0 < g.n1; k0 += nt) {
        const int k = k0 + tid;
        const int f = (k < g.n1 && kps1[k].octave == 0) ? 1 : 0;   // level1 > 0 -> skipped
        int total;
        const int pos = block_excl_scan(f, scratch, &total);
        if (f) qlist[run + pos] = k;
        run += total;
    }
    if (tid == 0) { counts[0] = run; counts[1] = tot; }
    // the parallel rounds' first two claim tables and flags start empty
    for (int k = tid; k < 2 * tot; k += nt) cnt3[k] = 0;
    for (int k = tid; k < nflags; k += nt) flags[k] = 0;
}

// one wave per query slot: the candidate list of GetFeaturesInArea(prev[i1], r, 0, 0)
__global__ __launch_bounds__(256) void k_init_cands(InitGeom g, const orbhip_kp* __restrict__ kps1,
                                                    const uint8_t* __restrict__ desc1,
                                                    const orbhip_kp* __restrict__ kps2,
                                                    const uint8_t* __restrict__ desc2, const float* __restrict__ prev,
                                                    const int* __restrict__ slot, const int* __restrict__ qlist,
                                                    const int* __restrict__ counts, uint32_t* __restrict__ lists,
                                                    int* __restrict__ lens, uint32_t* __restrict__ topk,
                                                    int* __restrict__ need) {
    const int q = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int nq = counts[0], nr = counts[1];
    if (q >= nq) return;
    const int i1 = qlist[q];
    const float x = prev[2 * i1], y = prev[2 * i1 + 1], r = g.r;
    const int nMinCellX = max(0, (int)floorf((x - g.minx - r) * g.invw));
    const int nMaxCellX = min(kGridCols - 1, (int)ceilf((x - g.minx + r) * g.invw));
    const int nMinCellY = max(0, (int)floorf((y - g.miny - r) * g.invh));
    const int nMaxCellY = min(kGridRows - 1, (int)ceilf((y - g.miny + r) * g.invh));
    const bool any = nMinCellX < kGridCols && nMaxCellX >= 0 && nMinCellY < kGridRows && nMaxCellY >= 0;
    uint32_t* out = lists + (size_t)q * g.list_cap;
    const float a1 = kps1[i1].angle, factor = 1.0f / kHisto;
    int n = 0, seen = 0;
    uint32_t t0 = ~0u, t1 = ~0u, t2 = ~0u, t3 = ~0u;
    if (any) {
        const uint4* qd4 = (const uint4*)(desc1 + 32 * (size_t)i1);
        const uint4 qa = qd4[0], qb = qd4[1];
        for (int b = 0; b < nr; b += 64) {
            const int rk = b + lane;
            bool ok = false;
            uint32_t v = 0;
            if (rk < nr) {
                const int k = slot[rk];
                const orbhip_kp kp = kps2[k];
                const int c = init_cell(g, kp.x, kp.y);
                const int px = c / kGridRows, py = c - px * kGridRows;
                if (px >= nMinCellX && px <= nMaxCellX && py >= nMinCellY && py <= nMaxCellY &&
                    fabsf(kp.x - x) < r && fabsf(kp.y - y) < r) {
                    const uint4* kd4 = (const uint4*)(desc2 + 32 * (size_t)k);
                    const uint4 ka = kd4[0], kb = kd4[1];
                    const int d = __popc(qa.x ^ ka.x) + __popc(qa.y ^ ka.y) + __popc(qa.z ^ ka.z) +
                                  __popc(qa.w ^ ka.w) + __popc(qb.x ^ kb.x) + __popc(qb.y ^ kb.y) +
                                  __popc(qb.z ^ kb.z) + __popc(qb.w ^ kb.w);
                    float rot = a1 - kp.angle;
                    if (rot < 0.0) rot += 360.0f;
                    int bin = (int)roundf(rot * factor);
                    if (bin == kHisto) bin = 0;
                    v = ((uint32_t)d << 21) | ((uint32_t)rk << 5) | (uint32_t)bin;
                    ok = true;
                }
            }
            const uint64_t m = __ballot(ok);
            if (ok) out[n + __popcll(m & ((1ull << lane) - 1ull))] = v;
            n += __popcll(m);
            // per-lane sorted top-4 (branch-free insert)
            const uint32_t w = ok ? v : ~0u;
            t3 = min(t3, max(t2, w)); t2 = min(t2, max(t1, w)); t1 = min(t1, max(t0, w)); t0 = min(t0, w);
            seen += ok;
        }
    }
    // the list's 16 smallest entries: 16 rounds of wave-min over the lane heads, the winning lane
    // pops. A lane that pops all 4 of its kept entries while it had more may have lost one of
    // the 16: then the chain scans the whole list (need = 2).
    uint32_t mine = ~0u;
    int popped = 0;
#pragma unroll
    for (int j = 0; j < kInitK; j++) {
        const uint32_t mn = wave_min_u32(t0);
        if (lane == j) mine = mn;
        if (t0 == mn && mn != ~0u) { t0 = t1; t1 = t2; t2 = t3; t3 = ~0u; popped++; }
    }
    const bool lost = __ballot(popped == 4 && seen > 4) != 0;
    if (lane < kInitK) topk[(size_t)q * kInitK + lane] = mine;
    if (lane == 0) {
        lens[q] = n;
        need[q] = lost ? 2 : (n > kInitK ? 1 : 0);
    }
}

// (m1, m2) = the two smallest values of the multiset union of two disjoint lane sets
__device__ __forceinline__ void top2_merge(uint32_t& m1, uint32_t& m2, uint32_t o1, uint32_t o2) {
    const uint32_t hi = max(m1, o1);
    m1 = min(m1, o1);
    m2 = min(hi, min(m2, o2));
}
template <int CTRL>
__device__ __forceinline__ void top2_dpp(uint32_t& m1, uint32_t& m2) {
    const uint32_t o1 = (uint32_t)__builtin_amdgcn_mov_dpp((int)m1, CTRL, 0xF, 0xF, true);
    const uint32_t o2 = (uint32_t)__builtin_amdgcn_mov_dpp((int)m2, CTRL, 0xF, 0xF, true);
    top2_merge(m1, m2, o1, o2);
}
// butterfly over the wave: xor 1, xor 2, half-row mirror, row mirror (each pairs lanes whose
// sets are disjoint), then rows 0<->1, 2<->3 and halves by permlane swaps; every lane ends with
// the wave's top-2
__device__ __forceinline__ void wave_top2(uint32_t& m1, uint32_t& m2) {
    top2_dpp<0xB1>(m1, m2);
    top2_dpp<0x4E>(m1, m2);
    top2_dpp<0x141>(m1, m2);
    top2_dpp<0x140>(m1, m2);
    {
        const auto a = __builtin_amdgcn_permlane16_swap(m1, m1, false, false);
        const auto b = __builtin_amdgcn_permlane16_swap(m2, m2, false, false);
        m1 = a[0]; m2 = b[0];
        top2_merge(m1, m2, a[1], b[1]);
    }
    {
        const auto a = __builtin_amdgcn_permlane32_swap(m1, m1, false, false);
        const auto b = __builtin_amdgcn_permlane32_swap(m2, m2, false, false);
        m1 = a[0]; m2 = b[0];
        top2_merge(m1, m2, a[1], b[1]);
    }
}


// LDS: ST u32[nr] = vMatchedDistance (low 16 bits, 0xFFFF = INT_MAX) | vnMatches21 as a query
// slot (high 16, 0xFFFF none); CL u32[nq] = the rank query q claimed | its rotHist push bin << 16
// (~0u none). vnMatches12 is implied: the claim of q survives iff ST[rank].hi == q at the end (a
// steal only ever replaces it), so the chain never reads a match back.
__global__ __launch_bounds__(256) void k_init_greedy(InitGeom g, float nnratio, int check_orientation,
                                                     const orbhip_kp* __restrict__ kps2, const int* __restrict__ slot,
                                                     const int* __restrict__ qlist, const int* __restrict__ counts,
                                                     const uint32_t* __restrict__ lists, const int* __restrict__ lens,
                                                     const uint32_t* __restrict__ topk, const int* __restrict__ need,
                                                     int32_t* __restrict__ matches12, float* __restrict__ prev,
                                                     int* __restrict__ nmatch) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    __shared__ int hist[32], keep[3], cnt;
    const int nq = counts[0], nr = counts[1];
    uint32_t* ST = (uint32_t*)smem;
    uint32_t* CL = ST + nr;
    const int tid = threadIdx.x, nt = blockDim.x, lane = tid & 63;
    for (int k = tid; k < nr; k += nt) ST[k] = ~0u;
    for (int q = tid; q < nq; q += nt) CL[q] = ~0u;
    for (int i = tid; i < g.n1; i += nt) matches12[i] = -1;
    if (tid < 32) hist[tid] = 0;
    if (tid == 0) cnt = 0;
    __syncthreads();
    if (tid < 64 && nq > 0) {
        // blocks of 4 queries: lane 16j + e holds entry e of query 4b + j's top-16 (one 256-byte
        // row per block), and lane j < 4 its `need`. A ring of kInitR blocks is in flight; the
        // loads are unconditional (clamped block) so the waits count only the oldest block.
        // vMatchedDistance of a block's entries is read from LDS one block ahead (mdv) and kept
        // current by forwarding (the chain is the only writer, one rank per accepted query): a
        // block's own updates go into its mdv at once and into the next block's at its start.
        const int nb = (nq + 3) >> 2;
        uint32_t tk[kInitR];
        int nd[kInitR], mdv[kInitR];
        auto load = [&](int b, int r) {
            const int bb = min(b, nb - 1);
            tk[r] = topk[(size_t)bb * 64 + lane];
            nd[r] = need[min(4 * bb + (lane & 3), nq - 1)];
        };
        auto rank_of = [&](uint32_t v) { return v == ~0u ? 0 : (int)((v >> 5) & 0xFFFF); };
#pragma unroll
        for (int r = 0; r < kInitR; r++) load(r, r);
        mdv[0] = (int)(ST[rank_of(tk[0])] & 0xFFFF);
        for (int b0 = 0; b0 < nb; b0 += kInitR) {
#pragma unroll
            for (int r = 0; r < kInitR; r++) {
                const int b = b0 + r;
                const int rn = (r + 1) % kInitR;
                mdv[rn] = (int)(ST[rank_of(tk[rn])] & 0xFFFF);   // next block, before this block's writes
                const int rk_c = rank_of(tk[r]), rk_n = rank_of(tk[rn]);
                int upd_rk[4] = {-1, -1, -1, -1}, upd_d[4] = {0, 0, 0, 0};
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    const int q = 4 * b + j;
                    if (q < nq) {
                        const uint32_t v = tk[r];
                        const bool elig = v != ~0u && (int)(v >> 21) < mdv[r];
                        const uint32_t mask = (uint32_t)(__ballot(elig) >> (16 * j)) & 0xFFFFu;
                        const int nq_need = __builtin_amdgcn_readlane(nd[r], j);
                        uint32_t m1 = ~0u, m2 = ~0u;
                        if (nq_need == 0 || (nq_need == 1 && __popc(mask) >= 2)) {
                            // the two smallest eligible entries are among the list's 16 smallest
                            if (mask) m1 = (uint32_t)__builtin_amdgcn_readlane((int)v, 16 * j + __ffs(mask) - 1);
                            const uint32_t rest = mask & (mask - 1);
                            if (rest) m2 = (uint32_t)__builtin_amdgcn_readlane((int)v, 16 * j + __ffs(rest) - 1);
                        } else {
                            // whole-list scan (fewer than two eligible among the 16, or a lost entry)
                            const int lc = lens[q];
                            const uint32_t* lq = lists + (size_t)q * g.list_cap;
                            for (int e = lane; e < lc; e += 64) {
                                const uint32_t w0 = lq[e];
                                const uint32_t w = (w0 >> 21) < (ST[(w0 >> 5) & 0xFFFF] & 0xFFFF) ? w0 : ~0u;
                                m2 = min(m2, max(m1, w));
                                m1 = min(m1, w);
                            }
                            wave_top2(m1, m2);
                            m1 = (uint32_t)__builtin_amdgcn_readfirstlane((int)m1);
                            m2 = (uint32_t)__builtin_amdgcn_readfirstlane((int)m2);
                        }
                        if (m1 != ~0u) {
                            const int d1 = (int)(m1 >> 21);
                            const int d2 = m2 == ~0u ? INT_MAX : (int)(m2 >> 21);
                            if (d1 <= kThLow && (float)d1 < (float)d2 * nnratio) {
                                const int rk = (int)((m1 >> 5) & 0xFFFF);
                                if (lane == 0) {
                                    CL[q] = (uint32_t)rk | ((m1 & 31) << 16);
                                    ST[rk] = (uint32_t)d1 | ((uint32_t)q << 16);
                                }
                                // forward into this block's registers now, the next block's later
                                mdv[r] = rk_c == rk ? d1 : mdv[r];
                                upd_rk[j] = rk;
                                upd_d[j] = d1;
                                // a wave's LDS operations complete in order: only keep the compiler
                                // from moving later MD reads above these writes
                                asm volatile("" ::: "memory");
                            }
                        }
                    }
                }
#pragma unroll
                for (int j = 0; j < 4; j++) mdv[rn] = rk_n == upd_rk[j] ? upd_d[j] : mdv[rn];
                load(b + kInitR, r);
            }
        }
    }
    __syncthreads();
    if (check_orientation) {
        for (int q = tid; q < nq; q += nt)
            if (CL[q] != ~0u) atomicAdd(&hist[CL[q] >> 16], 1);   // every push, stolen ones included
        __syncthreads();
        if (tid == 0) {   // ComputeThreeMaxima
            int m1 = 0, m2 = 0, m3 = 0, i1 = -1, i2 = -1, i3 = -1;
            for (int b = 0; b < kHisto; b++) {
                const int s = hist[b];
                if (s > m1) { m3 = m2; m2 = m1; m1 = s; i3 = i2; i2 = i1; i1 = b; }
                else if (s > m2) { m3 = m2; m2 = s; i3 = i2; i2 = b; }
                else if (s > m3) { m3 = s; i3 = b; }
            }
            if (m2 < 0.1f * (float)m1) { i2 = -1; i3 = -1; }
            else if (m3 < 0.1f * (float)m1) { i3 = -1; }
            keep[0] = i1; keep[1] = i2; keep[2] = i3;
        }
        __syncthreads();
    }
    int c = 0;
    for (int q = tid; q < nq; q += nt) {
        int rk = CL[q] == ~0u ? -1 : (int)(CL[q] & 0xFFFF);
        if (rk >= 0 && (int)(ST[rk] >> 16) != q) rk = -1;   // stolen by a later query
        if (rk >= 0 && check_orientation) {
            const int b = (int)(CL[q] >> 16);
            if (b != keep[0] && b != keep[1] && b != keep[2]) rk = -1;
        }
        if (rk >= 0) {
            const int i1 = qlist[q], k = slot[rk];
            matches12[i1] = k;
            prev[2 * i1] = kps2[k].x;
            prev[2 * i1 + 1] = kps2[k].y;
            c++;
        }
    }
    atomicAdd(&cnt, c);
    __syncthreads();
    if (tid == 0) *nmatch = cnt;
}

// ---------------------------------------------------------------------------
// The same greedy pass as a parallel fixed point. Round r recomputes every query's pick from the
// picks of round r - 1: query q's vMatchedDistance of rank k is the smallest distance among the
// earlier queries (j < q) that picked k in round r - 1 (in the sequential pass each later claimant
// is strictly closer, so the last write is the minimum). Query 0 is right in round 0, and a query
// is right once every earlier one was right a round before, so a round that changes nothing ends
// at the sequential result. The claims of a round go to a per-rank table (kInitC slots of
// q << 9 | dist); three tables rotate (read r, fill r + 1, clear r + 2), as in k_proj_round. A
// rank with more than kInitC claimants in one round sets the overflow flag and the host runs the
// chain kernel instead. The 16-lane row of a query holds its 16 smallest entries; the selection
// is the chain's (first two eligible bits, or the whole-list scan reduced within the row).
// flags[0] = overflow, flags[1 + r] = "round r changed a pick".
// ---------------------------------------------------------------------------
constexpr int kInitC = 8;

__device__ __forceinline__ int init_md(const int* __restrict__ cnt, const uint32_t* __restrict__ ent, int rk, int q) {
    const int c = min(cnt[rk], kInitC);
    int md = INT_MAX;
    for (int t = 0; t < c; t++) {
        const uint32_t e = ent[(size_t)rk * kInitC + t];
        md = (int)(e >> 9) < q ? min(md, (int)(e & 511)) : md;
    }
    return md;
}

__global__ __launch_bounds__(256) void k_init_round(InitGeom g, float nnratio, int r, const int* __restrict__ counts,
                                                    const uint32_t* __restrict__ lists, const int* __restrict__ lens,
                                                    const uint32_t* __restrict__ topk, const int* __restrict__ need,
                                                    int* __restrict__ cnt3, uint32_t* __restrict__ ent3,
                                                    uint32_t* __restrict__ pick, int* __restrict__ flags) {
    if (flags[0] || (r > 0 && flags[r] == 0)) return;   // overflow, or converged a round ago
    const int nq = counts[0], nr = counts[1];
    const int* cc = cnt3 + (size_t)(r % 3) * nr;
    const uint32_t* ec = ent3 + (size_t)(r % 3) * nr * kInitC;
    int* cn = cnt3 + (size_t)((r + 1) % 3) * nr;
    uint32_t* en = ent3 + (size_t)((r + 1) % 3) * nr * kInitC;
    int* cz = cnt3 + (size_t)((r + 2) % 3) * nr;
    for (int k = blockIdx.x * blockDim.x + threadIdx.x; k < nr; k += gridDim.x * blockDim.x) cz[k] = 0;

    const int lane = threadIdx.x & 63, row = lane >> 4, e = lane & 15;
    const int q = (blockIdx.x * 4 + (threadIdx.x >> 6)) * 4 + row;
    const bool qv = q < nq;
    const uint32_t v = qv ? topk[(size_t)q * kInitK + e] : ~0u;
    const int nd = qv ? need[q] : 0;
    const int md = v != ~0u ? init_md(cc, ec, (int)((v >> 5) & 0xFFFF), q) : INT_MAX;
    const bool elig = v != ~0u && (int)(v >> 21) < md;
    const uint32_t mask = (uint32_t)(__ballot(elig) >> (16 * row)) & 0xFFFFu;
    const uint32_t rest = mask & (mask - 1);
    // first two eligible entries of the row (all lanes shuffle, so no source lane is inactive)
    const uint32_t a = (uint32_t)__shfl((int)v, 16 * row + (mask ? __ffs(mask) - 1 : 0));
    const uint32_t b = (uint32_t)__shfl((int)v, 16 * row + (rest ? __ffs(rest) - 1 : 0));
    const bool full = qv && (nd == 2 || (nd == 1 && __popc(mask) < 2));
    uint32_t f1 = ~0u, f2 = ~0u;
    if (full) {   // whole list, 16 lanes of the row
        const int lc = lens[q];
        const uint32_t* lq = lists + (size_t)q * g.list_cap;
        for (int t = e; t < lc; t += 16) {
            const uint32_t w0 = lq[t];
            const uint32_t w = (int)(w0 >> 21) < init_md(cc, ec, (int)((w0 >> 5) & 0xFFFF), q) ? w0 : ~0u;
            f2 = min(f2, max(f1, w));
            f1 = min(f1, w);
        }
    }
    // top-2 within each 16-lane row (rows that did not scan reduce ~0u)
    top2_dpp<0xB1>(f1, f2);
    top2_dpp<0x4E>(f1, f2);
    top2_dpp<0x141>(f1, f2);
    top2_dpp<0x140>(f1, f2);
    const uint32_t m1 = full ? f1 : (mask ? a : ~0u);
    const uint32_t m2 = full ? f2 : (rest ? b : ~0u);
    uint32_t np = ~0u;
    if (m1 != ~0u) {
        const int d1 = (int)(m1 >> 21);
        const int d2 = m2 == ~0u ? INT_MAX : (int)(m2 >> 21);
        if (d1 <= kThLow && (float)d1 < (float)d2 * nnratio) np = m1;
    }
    if (qv && e == 0) {
        const uint32_t was = r == 0 ? ~0u : pick[q];   // round 0 starts from "no picks"
        if (r == 0 || was != np) pick[q] = np;
        if (was != np) flags[1 + r] = 1;
        if (np != ~0u) {
            const int rk = (int)((np >> 5) & 0xFFFF);
            const int s = atomicAdd(&cn[rk], 1);
            if (s < kInitC) en[(size_t)rk * kInitC + s] = ((uint32_t)q << 9) | (np >> 21);
            else flags[0] = 1;
        }
    }
}

// Applies converged picks: the last claimant of each rank keeps it (the steals), the rotation
// histogram counts every pick, as k_init_greedy. Writes matches12 and prev_out for all of F1 (so
// a finish over a not yet converged round, which the host discards, leaves nothing behind).
__global__ __launch_bounds__(1024) void k_init_finish(InitGeom g, int check_orientation, const orbhip_kp* __restrict__ kps2,
                                                      const int* __restrict__ slot, const int* __restrict__ qlist,
                                                      const int* __restrict__ counts, const uint32_t* __restrict__ pick,
                                                      const float* __restrict__ prev_in, int32_t* __restrict__ matches12,
                                                      float* __restrict__ prev_out, int* __restrict__ nmatch) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    __shared__ int hist[32], keep[3], cnt;
    int* owner = (int*)smem;
    const int nq = counts[0], nr = counts[1];
    const int tid = threadIdx.x, nt = blockDim.x;
    for (int k = tid; k < nr; k += nt) owner[k] = -1;
    for (int i = tid; i < g.n1; i += nt) {
        matches12[i] = -1;
        prev_out[2 * i] = prev_in[2 * i];
        prev_out[2 * i + 1] = prev_in[2 * i + 1];
    }
    if (tid < 32) hist[tid] = 0;
    if (tid == 0) cnt = 0;
    __syncthreads();
    for (int q = tid; q < nq; q += nt) {
        const uint32_t p = pick[q];
        if (p != ~0u) {
            atomicMax(&owner[(p >> 5) & 0xFFFF], q);
            if (check_orientation) atomicAdd(&hist[p & 31], 1);
        }
    }
    __syncthreads();
    if (check_orientation) {
        if (tid == 0) {   // ComputeThreeMaxima
            int m1 = 0, m2 = 0, m3 = 0, i1 = -1, i2 = -1, i3 = -1;
            for (int b = 0; b < kHisto; b++) {
                const int s = hist[b];
                if (s > m1) { m3 = m2; m2 = m1; m1 = s; i3 = i2; i2 = i1; i1 = b; }
                else if (s > m2) { m3 = m2; m2 = s; i3 = i2; i2 = b; }
                else if (s > m3) { m3 = s; i3 = b; }
            }
            if (m2 < 0.1f * (float)m1) { i2 = -1; i3 = -1; }
            else if (m3 < 0.1f * (float)m1) { i3 = -1; }
            keep[0] = i1; keep[1] = i2; keep[2] = i3;
        }
        __syncthreads();
    }
    int c = 0;
    for (int q = tid; q < nq; q += nt) {
        const uint32_t p = pick[q];
        int rk = p == ~0u ? -1 : (int)((p >> 5) & 0xFFFF);
        if (rk >= 0 && owner[rk] != q) rk = -1;   // stolen by a later query
        if (rk >= 0 && check_orientation) {
            const int b = (int)(p & 31);
            if (b != keep[0] && b != keep[1] && b != keep[2]) rk = -1;
        }
        if (rk >= 0) {
            const int i1 = qlist[q], k = slot[rk];
            matches12[i1] = k;
            prev_out[2 * i1] = kps2[k].x;
            prev_out[2 * i1 + 1] = kps2[k].y;
            c++;
        }
    }
    atomicAdd(&cnt, c);
    __syncthreads();
    if (tid == 0) *nmatch = cnt;
}

}  // namespace

// ---------------------------------------------------------------------------
// host
// ---------------------------------------------------------------------------
struct ProjWorkspace {
    void* d = nullptr;
    size_t dcap = 0;
    void* h = nullptr;
    void* hd = nullptr;   // h as the device addresses it (kernels write results there: no download)
    int* arrive = nullptr;   // the one-launch search's arrival counter (0 between launches)
    size_t hcap = 0;
    int ahead = 4;   // rounds launched per host sync (adapts to the last search)
    int init_ahead = 6;   // the same for SearchForInitialization's rounds
    ~ProjWorkspace() {
        if (arrive) (void)hipFree(arrive);
        if (d) (void)hipFree(d);
        if (h) (void)hipHostFree(h);
    }
};
ProjWorkspace* proj_ws_create() { return new ProjWorkspace(); }
void proj_ws_destroy(ProjWorkspace* w) { delete w; }

#define PJOK(x)                                                                                    \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess) {                                                                    \
            std::fprintf(stderr, "orbhip proj: %s: %s\n", #x, hipGetErrorString(e_));              \
            return ORBHIP_ERR_DEVICE;                                                              \
        }                                                                                          \
    } while (0)

namespace {

// staging layout helper: consecutive 256-byte aligned segments
struct Layout {
    size_t off = 0;
    size_t add(size_t bytes) { const size_t o = off; off += (bytes + 255) & ~size_t(255); return o; }
};

ProjFrame make_frame(const orbhip_frame* F) {
    ProjFrame f{};
    f.n = F->n;
    f.minx = F->min_x; f.maxx = F->max_x; f.miny = F->min_y; f.maxy = F->max_y;
    f.invw = (float)kGridCols / (f.maxx - f.minx);
    f.invh = (float)kGridRows / (f.maxy - f.miny);
    for (int k = 0; k < 4; k++) f.q[k] = F->pose_q[k];
    for (int k = 0; k < 3; k++) f.t[k] = F->pose_t[k];
    f.fx = F->fx; f.fy = F->fy; f.cx = F->cx; f.cy = F->cy;
    // mRcw = q.toRotationMatrix(); mOw = conj(q)._transformVector(-t) (Sophus SE3f::inverse)
    const float* q = f.q;
    const float tx = 2 * q[0], ty = 2 * q[1], tz = 2 * q[2];
    const float twx = tx * q[3], twy = ty * q[3], twz = tz * q[3];
    const float txx = tx * q[0], txy = ty * q[0], txz = tz * q[0];
    const float tyy = ty * q[1], tyz = tz * q[1], tzz = tz * q[2];
    f.R[0] = 1 - (tyy + tzz); f.R[1] = txy - twz; f.R[2] = txz + twy;
    f.R[3] = txy + twz; f.R[4] = 1 - (txx + tzz); f.R[5] = tyz - twx;
    f.R[6] = txz - twy; f.R[7] = tyz + twx; f.R[8] = 1 - (txx + tyy);
    const float qc[4] = {-q[0], -q[1], -q[2], q[3]};
    const float v[3] = {f.t[0] * -1.0f, f.t[1] * -1.0f, f.t[2] * -1.0f};
    float uv[3] = {qc[1] * v[2] - qc[2] * v[1], qc[2] * v[0] - qc[0] * v[2], qc[0] * v[1] - qc[1] * v[0]};
    uv[0] += uv[0]; uv[1] += uv[1]; uv[2] += uv[2];
    const float c[3] = {qc[1] * uv[2] - qc[2] * uv[1], qc[2] * uv[0] - qc[0] * uv[2], qc[0] * uv[1] - qc[1] * uv[0]};
    f.Ow[0] = v[0] + qc[3] * uv[0] + c[0];
    f.Ow[1] = v[1] + qc[3] * uv[1] + c[1];
    f.Ow[2] = v[2] + qc[3] * uv[2] + c[2];
    return f;
}

// The staged inputs to device memory by the shader: every lane reads two 16-byte pieces of the
// pinned staging block over the bus (~140 KB per search: a few us) instead of a DMA-engine copy,
// whose start-up and ~15 GB/s rate cost ~12 us per call (rocprofv3 memory-copy trace, r03).
// ORBHIP_PROJ_DMA=1 restores hipMemcpyAsync (A/B, read per call). Also the pose solver's upload.
__global__ __launch_bounds__(256) void k_upload(const uint4* __restrict__ src, uint4* __restrict__ dst, int n16) {
    const int i = blockIdx.x * 512 + threadIdx.x;
    uint4 a{}, b{};
    if (i < n16) a = src[i];
    if (i + 256 < n16) b = src[i + 256];
    if (i < n16) dst[i] = a;
    if (i + 256 < n16) dst[i + 256] = b;
}
}  // namespace

hipError_t upload_inputs(const void* hd, void* d, const void* h, size_t bytes, hipStream_t st) {
    const char* e = std::getenv("ORBHIP_PROJ_DMA");
    if (e && e[0] == '1') return hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, st);
    const int n16 = (int)((bytes + 15) / 16);   // bytes: a multiple of 256 (Layout)
    if (n16 == 0) return hipSuccess;
    hipLaunchKernelGGL(k_upload, dim3((unsigned)((n16 + 511) / 512)), dim3(256), 0, st, (const uint4*)hd, (uint4*)d,
                       n16);
    return hipGetLastError();
}

namespace {

int ensure(ProjWorkspace* ws, size_t total) {
    if (!ws->arrive) {
        PJOK(hipMalloc((void**)&ws->arrive, sizeof(int)));
        PJOK(hipMemset(ws->arrive, 0, sizeof(int)));
    }
    if (ws->dcap < total) {
        if (ws->d) (void)hipFree(ws->d);
        ws->d = nullptr;
        ws->dcap = 0;
        PJOK(hipMalloc(&ws->d, total));
        ws->dcap = total;
    }
    if (ws->hcap < total) {
        if (ws->h) (void)hipHostFree(ws->h);
        ws->h = nullptr;
        ws->hcap = 0;
        PJOK(hipHostMalloc(&ws->h, total + total / 4, hipHostMallocDefault));
        ws->hcap = total + total / 4;
        PJOK(hipHostGetDevicePointer(&ws->hd, ws->h, 0));
    }
    return ORBHIP_OK;
}

// The fixed-point rounds, launched `ws->ahead` at a time with the finishing work (`tail`: the
// finish kernel and the result downloads) behind them and ONE host sync per batch: rounds after
// convergence exit on the device, so the common case is a single round trip. Returns the number
// of rounds that did work (< 0 on error).
template <typename Tail>
int run_rounds(ProjWorkspace* ws, const ProjFrame& f, int nq, int mode, float nnratio, char* D, size_t o_q,
               size_t o_kps, size_t o_kd, size_t o_cell, const uint8_t* claimed, size_t o_own, size_t o_qd,
               size_t o_pick, size_t o_chg, char* H, hipStream_t st, Tail&& tail) {
    const dim3 gq((unsigned)std::max(1, (nq + 3) / 4));
    const int cap = nq + 2;   // a fixed point is reached within nq + 1 rounds
    int* chg = (int*)(D + o_chg);
    const int* hchg = (const int*)(H + o_chg);
    PJOK(hipMemsetAsync(D + o_own, 0x7F, 3 * sizeof(int) * (size_t)std::max(f.n, 1), st));   // > any query
    PJOK(hipMemsetAsync(chg, 0, sizeof(int) * (size_t)cap, st));
    int r = 0;
    for (;;) {
        const int R = std::min(ws->ahead, cap - r);
        for (int j = 0; j < R; j++)
            hipLaunchKernelGGL(k_proj_round, gq, dim3(256), 0, st, f, nq, mode, nnratio, r + j,
                               (const Query*)(D + o_q), (const orbhip_kp*)(D + o_kps), (const uint8_t*)(D + o_kd),
                               (const int*)(D + o_cell), claimed, (int*)(D + o_own), (const uint8_t*)(D + o_qd),
                               (int*)(D + o_pick), chg);
        PJOK(hipGetLastError());
        if (int rc = tail()) return rc;
        PJOK(hipMemcpyAsync(H + o_chg + sizeof(int) * r, chg + r, sizeof(int) * R, hipMemcpyDeviceToHost, st));
        PJOK(hipStreamSynchronize(st));
        for (int j = 0; j < R; j++)
            if (hchg[r + j] == 0) {
                const int rounds = r + j + 1;
                ws->ahead = std::min(16, std::max(2, rounds + 1));
                return rounds;
            }
        r += R;
        if (r >= cap) return r;
        ws->ahead = std::min(16, 2 * ws->ahead);
    }
}

}  // namespace

namespace {

// the two-launch form applies: every octave fits the list entry's 4 bits, the owner tables fit LDS
constexpr size_t kResolveLds = 150 * 1024;   // k_proj_resolve's dynamic LDS
bool onepass_ok(const orbhip_frame* F, int nq) {
    const char* e = std::getenv("ORBHIP_PROJ_ROUNDS");   // A/B switch (read per call: tests flip it)
    if ((e && e[0] == '1') || F->n > kProjMaxN || nq > kProjMaxQ || resolve_head_bytes(F->n, nq) > kResolveLds)
        return false;
    for (int k = 0; k < F->n; k++)
        if (F->kps[k].octave < 0 || F->kps[k].octave > 15) return false;
    return true;
}
// k_proj_lists' LDS: keypoint records, cells (padded to 256), the waves' index lists
size_t list_lds_bytes(int n) { return 16 * (size_t)n + 2 * (size_t)((n + 255) & ~255) + kListIdxBytes; }
static_assert(18 * (size_t)kProjMaxN + kListIdxBytes <= kResolveLds, "k_proj_lists' staging exceeds its LDS");
hipError_t proj_lds_attr() {   // beyond the default 64 KiB of dynamic LDS; per device (dev_attr.h)
    static LdsAttrOnce attr;
    static const void* const fs[] = {(const void*)k_proj_resolve<0>, (const void*)k_proj_resolve<1>,
                                     (const void*)k_proj_lists<0>, (const void*)k_proj_lists<1>};
    return attr.ensure(fs, 4, kResolveLds);
}
// list entries the resolve kernel holds in LDS next to its owner tables and list offsets
int resolve_ent_cap(int n, int nq) {
    const size_t head = resolve_head_bytes(n, nq);
    return head >= kResolveLds ? 0 : (int)((kResolveLds - head) / 8);
}
// one launch (the list kernel's last work-group resolves) unless ORBHIP_PROJ_TWO=1 (read per call)
bool proj_fused() {
    const char* e = std::getenv("ORBHIP_PROJ_TWO");
    return !(e && e[0] == '1');
}
int proj_cap() {
    const char* e = std::getenv("ORBHIP_PROJ_CAP");   // tests shrink it to force the round path
    return e ? std::max(1, std::min(kProjCap, std::atoi(e))) : kProjCap;
}

// outputs in one block (one download): match (nq ints), level (nq ints), in_view (nq bytes), res
struct OutBlock {
    size_t match, lvl, iv, res, bytes;
    explicit OutBlock(int nq) {
        match = 0;
        lvl = 4 * (size_t)nq;
        iv = 8 * (size_t)nq;
        res = (iv + (size_t)nq + 15) & ~size_t(15);
        bytes = res + 16;
    }
};

}  // namespace

int proj_search_last(ProjWorkspace* ws, const orbhip_frame* F, const orbhip_proj_last* L, float th,
                     int check_orientation, int32_t* match, int* rounds_out, hipStream_t st) {
    if (!ws || !F || !L || !match || F->n < 0 || L->n < 0 || F->n > 65535 || !F->scale_factors ||
        (F->n && (!F->kps || !F->desc)) || (L->n && (!L->points || !L->desc || !L->octave || !L->angle)))
        return ORBHIP_ERR_ARG;
    for (int i = 0; i < L->n; i++)
        if (L->octave[i] < 0 || L->octave[i] >= F->n_levels) return ORBHIP_ERR_ARG;
    const int n = F->n, nq = L->n;
    if (nq == 0) return 0;
    const bool onepass = onepass_ok(F, nq);
    const int cap = proj_cap();
    if (onepass) PJOK(proj_lds_attr());
    const OutBlock ob(nq);
    Layout lay;
    const size_t o_kps = lay.add(sizeof(orbhip_kp) * n), o_kd = lay.add(32 * (size_t)n), o_cl = lay.add(n);
    const size_t o_scale = lay.add(sizeof(float) * F->n_levels);
    const size_t o_pts = lay.add(12 * (size_t)nq), o_qd = lay.add(32 * (size_t)nq), o_oct = lay.add(4 * (size_t)nq);
    const size_t o_ang = lay.add(4 * (size_t)nq), o_in_end = lay.off;
    const size_t o_cell = lay.add(4 * (size_t)n), o_own = lay.add(12 * (size_t)std::max(n, 1));
    const size_t o_q = lay.add(sizeof(Query) * nq), o_chg = lay.add(4 * ((size_t)nq + 2));
    const size_t o_pick = lay.add(4 * (size_t)nq), o_out = lay.add(ob.bytes);
    const size_t o_list = onepass ? lay.add(8 * (size_t)nq * cap) : 0, o_lcnt = lay.add(4 * (size_t)nq);
    const size_t o_pick0 = lay.add(4 * (size_t)nq);
    if (int rc = ensure(ws, lay.off)) return rc;
    char* H = (char*)ws->h;
    char* HD = (char*)ws->hd;   // the two-launch form writes its results straight into H
    char* D = (char*)ws->d;
    std::memcpy(H + o_kps, F->kps, sizeof(orbhip_kp) * n);
    std::memcpy(H + o_kd, F->desc, 32 * (size_t)n);
    if (F->claimed) std::memcpy(H + o_cl, F->claimed, n);
    std::memcpy(H + o_scale, F->scale_factors, sizeof(float) * F->n_levels);
    std::memcpy(H + o_pts, L->points, 12 * (size_t)nq);
    std::memcpy(H + o_qd, L->desc, 32 * (size_t)nq);
    std::memcpy(H + o_oct, L->octave, 4 * (size_t)nq);
    std::memcpy(H + o_ang, L->angle, 4 * (size_t)nq);
    PJOK(upload_inputs(ws->hd, D, H, o_in_end, st));
    const ProjFrame f = make_frame(F);
    const PrepLast pl{(const float*)(D + o_pts), (const int*)(D + o_oct), (const float*)(D + o_scale), th};
    const uint8_t* dcl = F->claimed ? (const uint8_t*)(D + o_cl) : nullptr;
    int* hres = (int*)(H + o_out + ob.res);
    if (onepass) {
        const bool fused = proj_fused();
        const ResolveArgs ra{fused ? 1 : 0, check_orientation, resolve_ent_cap(n, nq), (const float*)(D + o_ang),
                             (int*)(HD + o_out + ob.match), (int*)(HD + o_out + ob.res),
                             ws->arrive};
        hipLaunchKernelGGL(k_proj_lists<0>, dim3((unsigned)((nq + kListQ - 1) / kListQ)), dim3(1024),
                           fused ? kResolveLds : list_lds_bytes(n), st, f, nq, pl, PrepLocal{}, cap, 0.f,
                           (const orbhip_kp*)(D + o_kps), (const uint8_t*)(D + o_kd), dcl, (const uint8_t*)(D + o_qd),
                           (uint64_t*)(D + o_list), (int*)(D + o_lcnt), (int*)(D + o_pick0), nullptr, nullptr, ra);
        if (!fused)
            hipLaunchKernelGGL(k_proj_resolve<0>, dim3(1), dim3(1024), kResolveLds, st, n, nq, 0.f, check_orientation,
                               cap, ra.ent_cap, ra.qangle, (const orbhip_kp*)(D + o_kps), (const uint64_t*)(D + o_list),
                               (const int*)(D + o_lcnt), (const int*)(D + o_pick0), ra.match, ra.res);
        PJOK(hipGetLastError());
        PJOK(hipStreamSynchronize(st));
        if (hres[1] == 0) {
            std::memcpy(match, H + o_out + ob.match, 4 * (size_t)nq);
            if (rounds_out) *rounds_out = hres[2];
            return hres[0];
        }
    }
    PJOK(hipMemsetAsync(D + o_pick, 0xFF, 4 * (size_t)nq, st));   // -1: the first round always "changes"
    if (n) hipLaunchKernelGGL(k_proj_cells, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, f,
                              (const orbhip_kp*)(D + o_kps), (int*)(D + o_cell));
    hipLaunchKernelGGL(k_proj_prep_last, dim3((unsigned)((nq + 255) / 256)), dim3(256), 0, st, f, nq, pl,
                       (Query*)(D + o_q));
    auto tail = [&]() -> int {
        hipLaunchKernelGGL(k_proj_finish, dim3(1), dim3(1024), 0, st, nq, check_orientation,
                           (const float*)(D + o_ang), (const orbhip_kp*)(D + o_kps), (const int*)(D + o_pick),
                           (int*)(D + o_out + ob.match), (int*)(D + o_out + ob.res));
        PJOK(hipMemcpyAsync(H + o_out, D + o_out, ob.bytes, hipMemcpyDeviceToHost, st));
        return 0;
    };
    const int rounds = run_rounds(ws, f, nq, 0, 0.f, D, o_q, o_kps, o_kd, o_cell, dcl, o_own, o_qd, o_pick, o_chg, H,
                                  st, tail);
    if (rounds < 0) return rounds;
    std::memcpy(match, H + o_out + ob.match, 4 * (size_t)nq);
    if (rounds_out) *rounds_out = rounds;
    return hres[0];
}

int proj_search_local(ProjWorkspace* ws, const orbhip_frame* F, const orbhip_local_points* M, float view_cos_limit,
                      float th, float nnratio, int far_points, float th_far, uint8_t* in_view, int32_t* level,
                      int32_t* match, int* rounds_out, hipStream_t st) {
    if (!ws || !F || !M || !match || !in_view || !level || F->n < 0 || M->n < 0 || F->n > 65535 ||
        !F->scale_factors || (F->n && (!F->kps || !F->desc)) ||
        (M->n && (!M->points || !M->normals || !M->min_dist || !M->max_dist || !M->desc)))
        return ORBHIP_ERR_ARG;
    const int n = F->n, nq = M->n;
    if (nq == 0) return 0;
    const bool onepass = onepass_ok(F, nq);
    const int cap = proj_cap();
    if (onepass) PJOK(proj_lds_attr());
    const OutBlock ob(nq);
    Layout lay;
    const size_t o_kps = lay.add(sizeof(orbhip_kp) * n), o_kd = lay.add(32 * (size_t)n), o_cl = lay.add(n);
    const size_t o_scale = lay.add(sizeof(float) * F->n_levels);
    const size_t o_pts = lay.add(12 * (size_t)nq), o_nrm = lay.add(12 * (size_t)nq), o_mind = lay.add(4 * (size_t)nq);
    const size_t o_maxd = lay.add(4 * (size_t)nq), o_qd = lay.add(32 * (size_t)nq), o_skip = lay.add(nq);
    const size_t o_in_end = lay.off;
    const size_t o_cell = lay.add(4 * (size_t)n), o_own = lay.add(12 * (size_t)std::max(n, 1));
    const size_t o_q = lay.add(sizeof(Query) * nq), o_chg = lay.add(4 * ((size_t)nq + 2));
    const size_t o_pick = lay.add(4 * (size_t)nq), o_out = lay.add(ob.bytes);
    const size_t o_list = onepass ? lay.add(8 * (size_t)nq * cap) : 0, o_lcnt = lay.add(4 * (size_t)nq);
    const size_t o_pick0 = lay.add(4 * (size_t)nq);
    if (int rc = ensure(ws, lay.off)) return rc;
    char* H = (char*)ws->h;
    char* HD = (char*)ws->hd;   // the two-launch form writes its results straight into H
    char* D = (char*)ws->d;
    std::memcpy(H + o_kps, F->kps, sizeof(orbhip_kp) * n);
    std::memcpy(H + o_kd, F->desc, 32 * (size_t)n);
    if (F->claimed) std::memcpy(H + o_cl, F->claimed, n);
    std::memcpy(H + o_scale, F->scale_factors, sizeof(float) * F->n_levels);
    std::memcpy(H + o_pts, M->points, 12 * (size_t)nq);
    std::memcpy(H + o_nrm, M->normals, 12 * (size_t)nq);
    std::memcpy(H + o_mind, M->min_dist, 4 * (size_t)nq);
    std::memcpy(H + o_maxd, M->max_dist, 4 * (size_t)nq);
    std::memcpy(H + o_qd, M->desc, 32 * (size_t)nq);
    if (M->skip) std::memcpy(H + o_skip, M->skip, nq);
    PJOK(upload_inputs(ws->hd, D, H, o_in_end, st));
    const ProjFrame f = make_frame(F);
    const PrepLocal pc{(const float*)(D + o_pts), (const float*)(D + o_nrm), (const float*)(D + o_mind),
                       (const float*)(D + o_maxd), M->skip ? (const uint8_t*)(D + o_skip) : nullptr,
                       (const float*)(D + o_scale), F->n_levels, F->log_scale_factor, view_cos_limit, th, far_points,
                       th_far};
    const uint8_t* dcl = F->claimed ? (const uint8_t*)(D + o_cl) : nullptr;
    uint8_t* d_iv = (uint8_t*)(D + o_out + ob.iv);
    int* d_lvl = (int*)(D + o_out + ob.lvl);
    int* hres = (int*)(H + o_out + ob.res);
    auto outputs = [&]() {
        std::memcpy(match, H + o_out + ob.match, 4 * (size_t)nq);
        std::memcpy(level, H + o_out + ob.lvl, 4 * (size_t)nq);
        std::memcpy(in_view, H + o_out + ob.iv, nq);
    };
    if (onepass) {
        const bool fused = proj_fused();
        const ResolveArgs ra{fused ? 1 : 0, 0, resolve_ent_cap(n, nq), nullptr,
                             (int*)(HD + o_out + ob.match), (int*)(HD + o_out + ob.res), ws->arrive};
        hipLaunchKernelGGL(k_proj_lists<1>, dim3((unsigned)((nq + kListQ - 1) / kListQ)), dim3(1024),
                           fused ? kResolveLds : list_lds_bytes(n), st, f, nq, PrepLast{}, pc, cap, nnratio,
                           (const orbhip_kp*)(D + o_kps), (const uint8_t*)(D + o_kd), dcl, (const uint8_t*)(D + o_qd),
                           (uint64_t*)(D + o_list), (int*)(D + o_lcnt), (int*)(D + o_pick0),
                           (uint8_t*)(HD + o_out + ob.iv), (int*)(HD + o_out + ob.lvl), ra);
        if (!fused)
            hipLaunchKernelGGL(k_proj_resolve<1>, dim3(1), dim3(1024), kResolveLds, st, n, nq, nnratio, 0, cap,
                               ra.ent_cap, (const float*)nullptr, (const orbhip_kp*)(D + o_kps),
                               (const uint64_t*)(D + o_list), (const int*)(D + o_lcnt), (const int*)(D + o_pick0),
                               ra.match, ra.res);
        PJOK(hipGetLastError());
        PJOK(hipStreamSynchronize(st));
        if (hres[1] == 0) {
            outputs();
            if (rounds_out) *rounds_out = hres[2];
            return hres[0];
        }
    }
    PJOK(hipMemsetAsync(D + o_pick, 0xFF, 4 * (size_t)nq, st));
    if (n) hipLaunchKernelGGL(k_proj_cells, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, f,
                              (const orbhip_kp*)(D + o_kps), (int*)(D + o_cell));
    hipLaunchKernelGGL(k_proj_prep_local, dim3((unsigned)((nq + 255) / 256)), dim3(256), 0, st, f, nq, pc,
                       (Query*)(D + o_q), d_iv, d_lvl);
    auto tail = [&]() -> int {
        hipLaunchKernelGGL(k_proj_finish, dim3(1), dim3(1024), 0, st, nq, 0, (const float*)nullptr,
                           (const orbhip_kp*)(D + o_kps), (const int*)(D + o_pick), (int*)(D + o_out + ob.match),
                           (int*)(D + o_out + ob.res));
        PJOK(hipMemcpyAsync(H + o_out, D + o_out, ob.bytes, hipMemcpyDeviceToHost, st));
        return 0;
    };
    const int rounds = run_rounds(ws, f, nq, 1, nnratio, D, o_q, o_kps, o_kd, o_cell, dcl, o_own, o_qd, o_pick, o_chg,
                                  H, st, tail);
    if (rounds < 0) return rounds;
    outputs();
    if (rounds_out) *rounds_out = rounds;
    return hres[0];
}

int init_search(ProjWorkspace* ws, const orbhip_init_frame* F1, const orbhip_init_frame* F2, float* prev_matched,
                int window_size, float nnratio, int check_orientation, int32_t* matches12, hipStream_t st) {
    if (!ws || !F1 || !F2 || !prev_matched || !matches12 || F1->n < 0 || F2->n < 0 || F1->n > 65535 ||
        F2->n > 65535 || (F1->n && (!F1->kps || !F1->desc)) || (F2->n && (!F2->kps || !F2->desc)) ||
        !(F2->max_x > F2->min_x) || !(F2->max_y > F2->min_y))
        return ORBHIP_ERR_ARG;
    const int n1 = F1->n, n2 = F2->n;
    for (int i = 0; i < n1; i++) matches12[i] = -1;
    if (n1 == 0) return 0;
    // capacity from the octave-0 counts (bounds of the device-side queries / ranks)
    // (octaves are >= 0: ORBextractor levels; a negative octave would disable the level check)
    int nq0 = 0, nr0 = 0;
    for (int i = 0; i < n1; i++) {
        if (F1->kps[i].octave < 0) return ORBHIP_ERR_ARG;
        nq0 += F1->kps[i].octave == 0;
    }
    for (int k = 0; k < n2; k++) nr0 += F2->kps[k].octave == 0;
    const size_t lds = 4 * (size_t)nr0 + 4 * (size_t)nq0 + 16;
    if (lds > 150 * 1024) return ORBHIP_ERR_UNSUPPORTED;
    const int list_cap = std::max(64, (nr0 + 63) & ~63);
    if ((size_t)std::max(nq0, 1) * list_cap > ((size_t)1 << 28)) return ORBHIP_ERR_UNSUPPORTED;
    // the kernel's static LDS (histogram) comes on top of the dynamic 150 KiB envelope
    static LdsAttrOnce attr;   // per device, thread-safe (dev_attr.h)
    static const void* const fs[] = {(const void*)k_init_greedy, (const void*)k_init_finish};
    PJOK(attr.ensure(fs, 2, 152 * 1024));
    Layout lay;
    const size_t o_k1 = lay.add(sizeof(orbhip_kp) * n1), o_d1 = lay.add(32 * (size_t)n1);
    const size_t o_k2 = lay.add(sizeof(orbhip_kp) * std::max(n2, 1)), o_d2 = lay.add(32 * (size_t)std::max(n2, 1));
    const size_t o_prev = lay.add(8 * (size_t)n1), o_in_end = lay.off;
    const size_t o_match = lay.add(4 * (size_t)n1), o_cnt = lay.add(16), o_out_end = lay.off;
    const size_t o_slot = lay.add(4 * (size_t)std::max(n2, 1)), o_ql = lay.add(4 * (size_t)n1);
    const size_t o_len = lay.add(4 * ((size_t)n1 + 1)), o_list = lay.add(4 * (size_t)std::max(nq0, 1) * list_cap);
    const size_t o_topk = lay.add(4 * (size_t)kInitK * (((size_t)std::max(nq0, 1) + 3) & ~size_t(3)));
    const size_t o_need = lay.add(4 * (size_t)std::max(nq0, 1));
    const int cap = std::min(kInitMaxRounds, nq0 + 2);
    const size_t o_cnt3 = lay.add(4 * 3 * (size_t)std::max(nr0, 1));
    const size_t o_ent3 = lay.add(4 * 3 * (size_t)std::max(nr0, 1) * kInitC);
    const size_t o_pick = lay.add(4 * (size_t)std::max(nq0, 1));
    const size_t o_pout = lay.add(8 * (size_t)n1);
    const size_t o_flags = lay.add(4 * ((size_t)cap + 1));
    if (int rc = ensure(ws, lay.off)) return rc;
    char* H = (char*)ws->h;
    char* D = (char*)ws->d;
    std::memcpy(H + o_k1, F1->kps, sizeof(orbhip_kp) * n1);
    std::memcpy(H + o_d1, F1->desc, 32 * (size_t)n1);
    if (n2) {
        std::memcpy(H + o_k2, F2->kps, sizeof(orbhip_kp) * n2);
        std::memcpy(H + o_d2, F2->desc, 32 * (size_t)n2);
    }
    std::memcpy(H + o_prev, prev_matched, 8 * (size_t)n1);
    PJOK(upload_inputs(ws->hd, D, H, o_in_end, st));
    InitGeom g{};
    g.n1 = n1; g.n2 = n2;
    g.minx = F2->min_x; g.maxx = F2->max_x; g.miny = F2->min_y; g.maxy = F2->max_y;
    g.invw = (float)kGridCols / (g.maxx - g.minx);
    g.invh = (float)kGridRows / (g.maxy - g.miny);
    g.r = (float)window_size;
    g.list_cap = list_cap;
    const orbhip_kp* dk1 = (const orbhip_kp*)(D + o_k1);
    const orbhip_kp* dk2 = (const orbhip_kp*)(D + o_k2);
    int* counts = (int*)(D + o_cnt);
    int* flags = (int*)(D + o_flags);
    hipLaunchKernelGGL(k_init_prep, dim3(1), dim3(1024), 0, st, g, dk1, dk2, (int*)(D + o_slot), (int*)(D + o_ql),
                       counts, (int*)(D + o_cnt3), flags, cap + 1);
    hipLaunchKernelGGL(k_init_cands, dim3((unsigned)std::max(1, (nq0 + 3) / 4)), dim3(256), 0, st, g, dk1,
                       (const uint8_t*)(D + o_d1), dk2, (const uint8_t*)(D + o_d2), (const float*)(D + o_prev),
                       (const int*)(D + o_slot), (const int*)(D + o_ql), (const int*)counts, (uint32_t*)(D + o_list),
                       (int*)(D + o_len), (uint32_t*)(D + o_topk), (int*)(D + o_need));
    PJOK(hipGetLastError());
    // parallel rounds, launched init_ahead at a time with the finish and the read-back behind them
    const int* hflags = (const int*)(H + o_flags);
    const dim3 gq((unsigned)std::max(1, (nq0 + 15) / 16));
    bool done = false;
    for (int r = 0; r < cap && !done && std::getenv("ORBHIP_INIT_CHAIN") == nullptr;) {
        const int R = std::min(ws->init_ahead, cap - r);
        for (int j = 0; j < R; j++)
            hipLaunchKernelGGL(k_init_round, gq, dim3(256), 0, st, g, nnratio, r + j, (const int*)counts,
                               (const uint32_t*)(D + o_list), (const int*)(D + o_len),
                               (const uint32_t*)(D + o_topk), (const int*)(D + o_need), (int*)(D + o_cnt3),
                               (uint32_t*)(D + o_ent3), (uint32_t*)(D + o_pick), flags);
        hipLaunchKernelGGL(k_init_finish, dim3(1), dim3(1024), 4 * (size_t)std::max(nr0, 1), st, g,
                           check_orientation, dk2, (const int*)(D + o_slot), (const int*)(D + o_ql),
                           (const int*)counts, (const uint32_t*)(D + o_pick), (const float*)(D + o_prev),
                           (int32_t*)(D + o_match), (float*)(D + o_pout), counts + 2);
        PJOK(hipGetLastError());
        PJOK(hipMemcpyAsync(H + o_match, D + o_match, o_out_end - o_match, hipMemcpyDeviceToHost, st));
        PJOK(hipMemcpyAsync(H + o_pout, D + o_pout, 8 * (size_t)n1, hipMemcpyDeviceToHost, st));
        PJOK(hipMemcpyAsync(H + o_flags, flags, 4 * ((size_t)cap + 1), hipMemcpyDeviceToHost, st));
        PJOK(hipStreamSynchronize(st));
        if (hflags[0]) break;   // a rank overflowed its claim slots: the chain decides
        for (int j = 0; j < R && !done; j++)
            if (hflags[1 + r + j] == 0) {
                done = true;
                ws->init_ahead = std::min(16, std::max(3, r + j + 2));
            }
        r += R;
        if (!done) ws->init_ahead = std::min(16, 2 * ws->init_ahead);
    }
    if (done) {
        std::memcpy(matches12, H + o_match, 4 * (size_t)n1);
        std::memcpy(prev_matched, H + o_pout, 8 * (size_t)n1);
        return ((int*)(H + o_cnt))[2];
    }
    hipLaunchKernelGGL(k_init_greedy, dim3(1), dim3(256), lds, st, g, nnratio, check_orientation, dk2,
                       (const int*)(D + o_slot), (const int*)(D + o_ql), (const int*)counts,
                       (const uint32_t*)(D + o_list), (const int*)(D + o_len), (const uint32_t*)(D + o_topk),
                       (const int*)(D + o_need), (int32_t*)(D + o_match), (float*)(D + o_prev), counts + 2);
    PJOK(hipGetLastError());
    PJOK(hipMemcpyAsync(H + o_prev, D + o_prev, o_out_end - o_prev, hipMemcpyDeviceToHost, st));
    PJOK(hipStreamSynchronize(st));
    std::memcpy(matches12, H + o_match, 4 * (size_t)n1);
    std::memcpy(prev_matched, H + o_prev, 8 * (size_t)n1);
    return ((int*)(H + o_cnt))[2];
}

}  // namespace orbhip
