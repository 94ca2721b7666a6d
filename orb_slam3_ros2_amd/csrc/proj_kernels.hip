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
#include <cstring>
#include <vector>

#include "../../include/orbhip.h"
#include "proj.h"

namespace orbhip {

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
__global__ void k_proj_prep_last(ProjFrame f, int nq, const float* __restrict__ pts, const int* __restrict__ oct,
                                 const float* __restrict__ scale, float th, Query* __restrict__ qs) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nq) return;
    Query Q{0, 0, 0, 0, 0, 0};
    const float P[3] = {pts[3 * i], pts[3 * i + 1], pts[3 * i + 2]};
    float Xc[3];
    qrotf(f.q, P, Xc);
    Xc[0] += f.t[0]; Xc[1] += f.t[1]; Xc[2] += f.t[2];
    const float invzc = (float)(1.0 / (double)Xc[2]);
    if (!(invzc < 0)) {
        const float u = f.fx * Xc[0] / Xc[2] + f.cx, v = f.fy * Xc[1] / Xc[2] + f.cy;
        if (!(u < f.minx || u > f.maxx || v < f.miny || v > f.maxy)) {
            const int lo = oct[i];
            Q = Query{u, v, th * scale[lo], lo - 1, lo + 1, 1};
        }
    }
    qs[i] = Q;
}

// Frame::isInFrustum(pMP, viewCosLimit) + the window of SearchByProjection(F, vpMapPoints, ...)
__global__ void k_proj_prep_local(ProjFrame f, int nq, const float* __restrict__ pts, const float* __restrict__ nrm,
                                  const float* __restrict__ mind, const float* __restrict__ maxd,
                                  const uint8_t* __restrict__ skip, const float* __restrict__ scale, int n_levels,
                                  float log_sf, float view_cos_limit, float th, int far_points, float th_far,
                                  Query* __restrict__ qs, uint8_t* __restrict__ in_view, int* __restrict__ level) {
    const int m = blockIdx.x * blockDim.x + threadIdx.x;
    if (m >= nq) return;
    Query Q{0, 0, 0, 0, 0, 0};
    uint8_t iv = 0;
    int lvl = -1;
    do {
        if (skip && skip[m]) break;
        const float* P = pts + 3 * m;
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
        const float maxDistance = 1.2f * maxd[m], minDistance = 0.8f * mind[m];
        if (dist < minDistance || dist > maxDistance) break;
        const float* Pn = nrm + 3 * m;
        const float viewCos = (PO[0] * Pn[0] + PO[1] * Pn[1] + PO[2] * Pn[2]) / dist;
        if (viewCos < view_cos_limit) break;
        const float ratio = maxd[m] / dist;
        int nScale = (int)ceilf(logf(ratio) / log_sf);   // MapPoint::PredictScale
        if (nScale < 0) nScale = 0;
        else if (nScale >= n_levels) nScale = n_levels - 1;
        iv = 1;
        lvl = nScale;
        if (far_points && Pc_dist > th_far) break;
        float r = viewCos > 0.998 ? 2.5f : 4.0f;   // RadiusByViewingCos
        if (th != 1.0f) r *= th;
        Q = Query{u, v, r * scale[nScale], nScale - 1, nScale, 1};
    } while (false);
    qs[m] = Q;
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

}  // namespace

// ---------------------------------------------------------------------------
// host
// ---------------------------------------------------------------------------
struct ProjWorkspace {
    void* d = nullptr;
    size_t dcap = 0;
    void* h = nullptr;
    size_t hcap = 0;
    int ahead = 4;   // rounds launched per host sync (adapts to the last search)
    ~ProjWorkspace() {
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

int ensure(ProjWorkspace* ws, size_t total) {
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

int proj_search_last(ProjWorkspace* ws, const orbhip_frame* F, const orbhip_proj_last* L, float th,
                     int check_orientation, int32_t* match, int* rounds_out, hipStream_t st) {
    if (!ws || !F || !L || !match || F->n < 0 || L->n < 0 || F->n > 65535 || !F->scale_factors ||
        (F->n && (!F->kps || !F->desc)) || (L->n && (!L->points || !L->desc || !L->octave || !L->angle)))
        return ORBHIP_ERR_ARG;
    for (int i = 0; i < L->n; i++)
        if (L->octave[i] < 0 || L->octave[i] >= F->n_levels) return ORBHIP_ERR_ARG;
    const int n = F->n, nq = L->n;
    if (nq == 0) return 0;
    Layout lay;
    const size_t o_kps = lay.add(sizeof(orbhip_kp) * n), o_kd = lay.add(32 * (size_t)n), o_cl = lay.add(n);
    const size_t o_scale = lay.add(sizeof(float) * F->n_levels);
    const size_t o_pts = lay.add(12 * (size_t)nq), o_qd = lay.add(32 * (size_t)nq), o_oct = lay.add(4 * (size_t)nq);
    const size_t o_ang = lay.add(4 * (size_t)nq), o_in_end = lay.off;
    const size_t o_cell = lay.add(4 * (size_t)n), o_own = lay.add(12 * (size_t)std::max(n, 1));
    const size_t o_q = lay.add(sizeof(Query) * nq), o_chg = lay.add(4 * ((size_t)nq + 2));
    const size_t o_pick = lay.add(4 * (size_t)nq), o_match = lay.add(4 * (size_t)nq), o_flag = lay.add(8);
    if (int rc = ensure(ws, lay.off)) return rc;
    char* H = (char*)ws->h;
    char* D = (char*)ws->d;
    std::memcpy(H + o_kps, F->kps, sizeof(orbhip_kp) * n);
    std::memcpy(H + o_kd, F->desc, 32 * (size_t)n);
    if (F->claimed) std::memcpy(H + o_cl, F->claimed, n);
    std::memcpy(H + o_scale, F->scale_factors, sizeof(float) * F->n_levels);
    std::memcpy(H + o_pts, L->points, 12 * (size_t)nq);
    std::memcpy(H + o_qd, L->desc, 32 * (size_t)nq);
    std::memcpy(H + o_oct, L->octave, 4 * (size_t)nq);
    std::memcpy(H + o_ang, L->angle, 4 * (size_t)nq);
    PJOK(hipMemcpyAsync(D, H, o_in_end, hipMemcpyHostToDevice, st));
    PJOK(hipMemsetAsync(D + o_pick, 0xFF, 4 * (size_t)nq, st));   // -1: the first round always "changes"
    const ProjFrame f = make_frame(F);
    if (n) hipLaunchKernelGGL(k_proj_cells, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, f,
                              (const orbhip_kp*)(D + o_kps), (int*)(D + o_cell));
    hipLaunchKernelGGL(k_proj_prep_last, dim3((unsigned)((nq + 255) / 256)), dim3(256), 0, st, f, nq,
                       (const float*)(D + o_pts), (const int*)(D + o_oct), (const float*)(D + o_scale), th,
                       (Query*)(D + o_q));
    auto tail = [&]() -> int {
        hipLaunchKernelGGL(k_proj_finish, dim3(1), dim3(1024), 0, st, nq, check_orientation,
                           (const float*)(D + o_ang), (const orbhip_kp*)(D + o_kps), (const int*)(D + o_pick),
                           (int*)(D + o_match), (int*)(D + o_flag));
        PJOK(hipMemcpyAsync(H + o_match, D + o_match, 4 * (size_t)nq, hipMemcpyDeviceToHost, st));
        PJOK(hipMemcpyAsync(H + o_flag, D + o_flag, 4, hipMemcpyDeviceToHost, st));
        return 0;
    };
    const int rounds = run_rounds(ws, f, nq, 0, 0.f, D, o_q, o_kps, o_kd, o_cell,
                                  F->claimed ? (const uint8_t*)(D + o_cl) : nullptr, o_own, o_qd, o_pick, o_chg, H,
                                  st, tail);
    if (rounds < 0) return rounds;
    std::memcpy(match, H + o_match, 4 * (size_t)nq);
    if (rounds_out) *rounds_out = rounds;
    return *(int*)(H + o_flag);
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
    Layout lay;
    const size_t o_kps = lay.add(sizeof(orbhip_kp) * n), o_kd = lay.add(32 * (size_t)n), o_cl = lay.add(n);
    const size_t o_scale = lay.add(sizeof(float) * F->n_levels);
    const size_t o_pts = lay.add(12 * (size_t)nq), o_nrm = lay.add(12 * (size_t)nq), o_mind = lay.add(4 * (size_t)nq);
    const size_t o_maxd = lay.add(4 * (size_t)nq), o_qd = lay.add(32 * (size_t)nq), o_skip = lay.add(nq);
    const size_t o_in_end = lay.off;
    const size_t o_cell = lay.add(4 * (size_t)n), o_own = lay.add(12 * (size_t)std::max(n, 1));
    const size_t o_q = lay.add(sizeof(Query) * nq), o_chg = lay.add(4 * ((size_t)nq + 2));
    const size_t o_pick = lay.add(4 * (size_t)nq), o_lvl = lay.add(4 * (size_t)nq), o_iv = lay.add(nq);
    const size_t o_match = lay.add(4 * (size_t)nq), o_flag = lay.add(8);
    if (int rc = ensure(ws, lay.off)) return rc;
    char* H = (char*)ws->h;
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
    PJOK(hipMemcpyAsync(D, H, o_in_end, hipMemcpyHostToDevice, st));
    PJOK(hipMemsetAsync(D + o_pick, 0xFF, 4 * (size_t)nq, st));
    const ProjFrame f = make_frame(F);
    if (n) hipLaunchKernelGGL(k_proj_cells, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, f,
                              (const orbhip_kp*)(D + o_kps), (int*)(D + o_cell));
    hipLaunchKernelGGL(k_proj_prep_local, dim3((unsigned)((nq + 255) / 256)), dim3(256), 0, st, f, nq,
                       (const float*)(D + o_pts), (const float*)(D + o_nrm), (const float*)(D + o_mind),
                       (const float*)(D + o_maxd), M->skip ? (const uint8_t*)(D + o_skip) : nullptr,
                       (const float*)(D + o_scale), F->n_levels, F->log_scale_factor, view_cos_limit, th, far_points,
                       th_far, (Query*)(D + o_q), (uint8_t*)(D + o_iv), (int*)(D + o_lvl));
    auto tail = [&]() -> int {
        hipLaunchKernelGGL(k_proj_finish, dim3(1), dim3(1024), 0, st, nq, 0, (const float*)nullptr,
                           (const orbhip_kp*)(D + o_kps), (const int*)(D + o_pick), (int*)(D + o_match),
                           (int*)(D + o_flag));
        PJOK(hipMemcpyAsync(H + o_match, D + o_match, 4 * (size_t)nq, hipMemcpyDeviceToHost, st));
        PJOK(hipMemcpyAsync(H + o_lvl, D + o_lvl, 4 * (size_t)nq, hipMemcpyDeviceToHost, st));
        PJOK(hipMemcpyAsync(H + o_iv, D + o_iv, nq, hipMemcpyDeviceToHost, st));
        PJOK(hipMemcpyAsync(H + o_flag, D + o_flag, 4, hipMemcpyDeviceToHost, st));
        return 0;
    };
    const int rounds = run_rounds(ws, f, nq, 1, nnratio, D, o_q, o_kps, o_kd, o_cell,
                                  F->claimed ? (const uint8_t*)(D + o_cl) : nullptr, o_own, o_qd, o_pick, o_chg, H,
                                  st, tail);
    if (rounds < 0) return rounds;
    std::memcpy(match, H + o_match, 4 * (size_t)nq);
    std::memcpy(level, H + o_lvl, 4 * (size_t)nq);
    std::memcpy(in_view, H + o_iv, nq);
    if (rounds_out) *rounds_out = rounds;
    return *(int*)(H + o_flag);
}

}  // namespace orbhip
