// Motion-only bundle adjustment: U:src/Optimizer.cc::Optimizer::PoseOptimization(Frame*)
// (SURVEY.md §8f rank 2), monocular edges, batched: ONE WAVEFRONT PER FRAME runs the whole
// reference procedure on the device, with no host round trip:
//   4 rounds x optimize(10) of g2o's Levenberg (lambda0 = 1e-5 max diag H, rho with the 1e-3
//   scale term, up to 10 trials per iteration, push/pop), each round restarting from the
//   frame's initial pose; after a round chi2 > 5.991 edges become outliers (level 1, inactive),
//   the robust kernel is dropped after round 2, and a frame with < 10 edges stops after round 0.
// EdgeSE3ProjectXYZOnlyPose (U:src/OptimizableTypes.cpp): e = obs - project(T.map(Xw)),
// J = -projectJac(Xc) [[0,z,-y,1,0,0],[-z,0,x,0,1,0],[y,-x,0,0,0,1]], Omega = I invSigma2[oct],
// Huber deltaMono = (float)sqrt(5.991). The 6x6 system (H + lambda I) x = b is tiny: every lane
// solves it redundantly (dense LDL^T), so the lanes never exchange anything but the edge sums.
// Edge sums are fixed-order LDS reductions (partials -> strip sums -> totals) with the same bits in
// every lane, the per-trial chi2 a DPP/permlane wave sum then the W wave sums in order.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <vector>

#include "../../include/orbhip.h"
#include "ba_se3.h"
#include "pose_opt.h"
#include "proj.h"
#include "wave_f64.h"

namespace orbhip {

struct PoseHdr {
    double T0[8];            // initial Tcw (normalised quaternion, translation)
    double fx, fy, cx, cy, delta;
    int n, off;              // edges [off, off + n) of the packed edge arrays
};
struct PoseOut {
    double T[8];
    int n_inliers, trials, pad[2];
};
struct PoseEdgeIn {          // float inputs as the reference holds them
    float X[3], u, v, info;
};

namespace {

constexpr int kAcc = 28;   // 21 upper-triangle H + 6 b + chi2

// The W wavefronts that run one frame, and their LDS: partial table [kAcc][RS], strip sums
// [kAcc][S], totals [32], wave sums [2][W] (double-buffered: consecutive sum1 calls need no
// trailing barrier).
template <int W>
struct FrameGroup {
    static constexpr int T = 64 * W;
    static constexpr int S = W == 1 ? 2 : 8;
    static constexpr int RS = T + S;   // row stride: the S-lane groups of the strip pass hit distinct banks
    static constexpr int kDoubles = kAcc * RS + kAcc * S + 32 + 2 * W;
    double* L;
    int tid, par = 0;
    __device__ __forceinline__ void sync() const {
        if constexpr (W == 1) wave_lds_sync();
        else __syncthreads();
    }
    // acc[k] <- sum over the group's threads, same bits everywhere
    __device__ __forceinline__ void sum_acc(double* acc) {
        double* L2 = L + kAcc * RS;
        double* L3 = L2 + kAcc * S;
#pragma unroll
        for (int k = 0; k < kAcc; k++) L[k * RS + tid] = acc[k];
        sync();
        if (tid < kAcc * S) {
            const int k = tid / S, s = tid - k * S;
            const double* row = L + k * RS;
            double p0 = 0, p1 = 0;
#pragma unroll 4
            for (int j = s; j < T; j += 2 * S) { p0 += row[j]; p1 += row[j + S]; }
            L2[tid] = p0 + p1;
        }
        sync();
        if (tid < kAcc) {
            double p = 0;
#pragma unroll
            for (int s = 0; s < S; s++) p += L2[tid * S + s];
            L3[tid] = p;
        }
        sync();
#pragma unroll
        for (int k = 0; k < kAcc; k++) acc[k] = L3[k];
    }
    __device__ __forceinline__ double sum1(double v) {
        v = col4_sum(row16_sum(v));
        if constexpr (W == 1) return v;
        double* Lw = L + kAcc * RS + kAcc * S + 32 + par * W;
        if ((tid & 63) == 0) Lw[tid >> 6] = v;
        sync();
        double s = 0;
#pragma unroll
        for (int w = 0; w < W; w++) s += Lw[w];
        par ^= 1;
        return s;
    }
};

// e = obs - project(T.map(Xw)); chi2 = info |e|^2
__device__ __forceinline__ void edge_err(const double* T, const PoseEdgeIn& ed, const PoseHdr& h, double& e0,
                                         double& e1, double& chi2, double& x, double& y, double& z) {
    const DQ q = load_q(T);
    qrot(q, (double)ed.X[0], (double)ed.X[1], (double)ed.X[2], x, y, z);
    x += T[4]; y += T[5]; z += T[6];
    const double iz = 1.0 / z;
    e0 = (double)ed.u - (h.fx * x * iz + h.cx);
    e1 = (double)ed.v - (h.fy * y * iz + h.cy);
    chi2 = (double)ed.info * (e0 * e0 + e1 * e1);
}

__device__ __forceinline__ void huber(double chi2, double delta, bool robust, double& rho0, double& rho1) {
    rho0 = chi2; rho1 = 1.0;
    if (robust && delta > 0) {
        const double dsqr = delta * delta;
        if (chi2 > dsqr) {
            const double sq = sqrt(chi2);
            rho0 = 2 * sq * delta - dsqr;
            rho1 = delta / sq;
        }
    }
}

// dense LDL^T without pivoting (the oracle's ldlt_solve), uniform in every lane
__device__ __forceinline__ bool ldlt6(double S[36], const double b[6], double x[6]) {
    double d[6], id[6];   // pivots and their reciprocals (one division per pivot)
#pragma unroll
    for (int j = 0; j < 6; j++) {
        double dj = S[6 * j + j];
#pragma unroll
        for (int k = 0; k < j; k++) dj -= S[6 * j + k] * S[6 * j + k] * d[k];
        if (dj == 0.0 || !isfinite(dj)) return false;
        d[j] = dj;
        id[j] = 1.0 / dj;
#pragma unroll
        for (int i = j + 1; i < 6; i++) {
            double s = S[6 * i + j];
#pragma unroll
            for (int k = 0; k < j; k++) s -= S[6 * i + k] * S[6 * j + k] * d[k];
            S[6 * i + j] = s * id[j];
        }
    }
#pragma unroll
    for (int i = 0; i < 6; i++) x[i] = b[i];
#pragma unroll
    for (int i = 0; i < 6; i++)
#pragma unroll
        for (int k = 0; k < i; k++) x[i] -= S[6 * i + k] * x[k];
#pragma unroll
    for (int i = 0; i < 6; i++) x[i] *= id[i];
#pragma unroll
    for (int i = 5; i >= 0; i--)
#pragma unroll
        for (int k = i + 1; k < 6; k++) x[i] -= S[6 * k + i] * x[k];
    return true;
}

// g2o optimize(10) over the level-0 edges of one frame (one wave). chi2_last[e] = the chi2 of
// the last computeActiveErrors that saw edge e (stale after a rejected final trial, as g2o).
template <int W>
__device__ void pose_optimize(FrameGroup<W>& g, double* T, const PoseHdr& h, const PoseEdgeIn* __restrict__ ed,
                              const uint8_t* __restrict__ level, double* __restrict__ chi2_last, bool robust,
                              int& trials) {
    constexpr int NT = FrameGroup<W>::T;
    // the first EC edges of every thread stay in registers for all trials (their level is fixed
    // during optimize(): a bit mask); the rest are re-read each pass
    constexpr int EC = W == 1 ? 2 : 4;
    const int tid = g.tid, n = h.n;
    PoseEdgeIn ec[EC];
    unsigned act = 0;
    int na = 0;
#pragma unroll
    for (int c = 0; c < EC; c++) {
        const int e = tid + c * NT;
        if (e < n) {
            ec[c] = ed[e];
            if (!level[e]) act |= 1u << c;
        }
    }
    na = __builtin_popcount(act);
    for (int e = tid + EC * NT; e < n; e += NT) na += level[e] == 0;
    if (g.sum1((double)na) == 0.0) return;   // no active vertex: optimize() does nothing
    double lambda = 0, ni = 2;
    for (int it = 0; it < 10; it++) {
        // computeActiveErrors + buildSystem
        double acc[kAcc];
#pragma unroll
        for (int k = 0; k < kAcc; k++) acc[k] = 0.0;
        auto build = [&](const PoseEdgeIn& E, int e) {
            double e0, e1, c2, x, y, z, r0, r1;
            edge_err(T, E, h, e0, e1, c2, x, y, z);
            huber(c2, h.delta, robust, r0, r1);
            chi2_last[e] = c2;
            acc[27] += r0;
            double J[6];
            const double iz = 1.0 / z, iz2 = iz * iz;
            J[0] = -(h.fx * iz); J[1] = -0.0; J[2] = h.fx * x * iz2;
            J[3] = -0.0; J[4] = -(h.fy * iz); J[5] = h.fy * y * iz2;
            const double D[18] = {0, z, -y, 1, 0, 0, -z, 0, x, 0, 1, 0, y, -x, 0, 0, 0, 1};
            double B[12];
#pragma unroll
            for (int r = 0; r < 2; r++)
#pragma unroll
                for (int c = 0; c < 6; c++)
                    B[6 * r + c] = J[3 * r] * D[c] + J[3 * r + 1] * D[6 + c] + J[3 * r + 2] * D[12 + c];
            const double w = r1 * (double)E.info;
            const double om0 = -(double)E.info * e0 * r1, om1 = -(double)E.info * e1 * r1;
            int t = 0;
#pragma unroll
            for (int r = 0; r < 6; r++)
#pragma unroll
                for (int c = r; c < 6; c++) acc[t++] += w * (B[r] * B[c] + B[6 + r] * B[6 + c]);
#pragma unroll
            for (int r = 0; r < 6; r++) acc[21 + r] += B[r] * om0 + B[6 + r] * om1;
        };
#pragma unroll
        for (int c = 0; c < EC; c++)
            if (act >> c & 1) build(ec[c], tid + c * NT);
        for (int e = tid + EC * NT; e < n; e += NT)
            if (!level[e]) build(ed[e], e);
        g.sum_acc(acc);
        double H[36], b[6];
        {
            int t = 0;
#pragma unroll
            for (int r = 0; r < 6; r++)
#pragma unroll
                for (int c = r; c < 6; c++) { H[6 * r + c] = acc[t]; H[6 * c + r] = acc[t]; t++; }
#pragma unroll
            for (int r = 0; r < 6; r++) b[r] = acc[21 + r];
        }
        double currentChi = acc[27];
        if (it == 0) {
            double md = 0;
#pragma unroll
            for (int j = 0; j < 6; j++) md = fmax(md, fabs(H[7 * j]));
            lambda = 1e-5 * md;
            ni = 2;
        }
        double rho = 0;
        int qmax = 0;
        do {
            double S[36], x[6];
#pragma unroll
            for (int k = 0; k < 36; k++) S[k] = H[k] + (k % 7 == 0 ? lambda : 0.0);
            const bool ok = ldlt6(S, b, x);
            if (!ok) {
#pragma unroll
                for (int k = 0; k < 6; k++) x[k] = 0.0;
            }
            double Tn[8];
#pragma unroll
            for (int k = 0; k < 8; k++) Tn[k] = T[k];
            se3_update(x, Tn);
            double tc = 0;
            auto chi = [&](const PoseEdgeIn& E, int e) {
                double e0, e1, c2, px, py, pz, r0, r1;
                edge_err(Tn, E, h, e0, e1, c2, px, py, pz);
                huber(c2, h.delta, robust, r0, r1);
                chi2_last[e] = c2;
                tc += r0;
            };
#pragma unroll
            for (int c = 0; c < EC; c++)
                if (act >> c & 1) chi(ec[c], tid + c * NT);
            for (int e = tid + EC * NT; e < n; e += NT)
                if (!level[e]) chi(ed[e], e);
            double tempChi = g.sum1(tc);
            if (!ok) tempChi = DBL_MAX;
            double scale = 1e-3;
#pragma unroll
            for (int j = 0; j < 6; j++) scale += x[j] * (lambda * x[j] + b[j]);
            rho = (currentChi - tempChi) / scale;
            if (rho > 0 && isfinite(tempChi)) {
                const double t2 = 2 * rho - 1;
                double alpha = 1. - t2 * t2 * t2;
                alpha = fmin(alpha, 2. / 3.);
                lambda *= fmax(1. / 3., alpha);
                ni = 2;
                currentChi = tempChi;
#pragma unroll
                for (int k = 0; k < 8; k++) T[k] = Tn[k];
            } else {
                lambda *= ni;   // pop: T keeps the pushed state
                ni *= 2;
            }
            qmax++;
            trials++;
        } while (rho < 0 && qmax < 10);
        if (qmax == 10 || rho == 0) break;
    }
}

}  // namespace

// W wavefronts per frame, 4 / W frames per 256-thread work-group
template <int W>
__global__ __launch_bounds__(256) void k_pose_opt(const PoseHdr* __restrict__ hdr, const PoseEdgeIn* __restrict__ edges,
                                                   uint8_t* __restrict__ level, uint8_t* __restrict__ outlier,
                                                   double* __restrict__ chi2_last, PoseOut* __restrict__ out,
                                                   uint8_t* __restrict__ outlier_copy, int B) {
    constexpr int FPB = 4 / W, NT = FrameGroup<W>::T;
    __shared__ double sm[FPB * FrameGroup<W>::kDoubles];
    const int grp = threadIdx.x / NT;
    const int f = blockIdx.x * FPB + grp;
    if (f >= B) return;   // W == 1 only (the grid is exact for W > 1): a whole wave leaves
    FrameGroup<W> g;
    g.L = sm + grp * FrameGroup<W>::kDoubles;
    g.tid = threadIdx.x - grp * NT;
    const int tid = g.tid;
    const PoseHdr h = hdr[f];
    const PoseEdgeIn* ed = edges + h.off;
    uint8_t* lv = level + h.off;
    uint8_t* ol = outlier + h.off;
    double* c2 = chi2_last + h.off;
    double T[8];
#pragma unroll
    for (int k = 0; k < 8; k++) T[k] = h.T0[k];
    for (int e = tid; e < h.n; e += NT) { lv[e] = 0; ol[e] = 0; c2[e] = 0.0; }
    int trials = 0, nbad = 0;
    if (h.n >= 3) {
        bool robust = true;
        for (int round = 0; round < 4; round++) {
#pragma unroll
            for (int k = 0; k < 8; k++) T[k] = h.T0[k];   // vSE3->setEstimate(pFrame->GetPose())
            pose_optimize<W>(g, T, h, ed, lv, c2, robust, trials);
            int nb = 0;
            for (int e = tid; e < h.n; e += NT) {   // each thread only touches its own edges
                double chi = c2[e];
                if (ol[e]) {   // level-1 edge: e->computeError() at the current estimate
                    double e0, e1, x, y, z;
                    edge_err(T, ed[e], h, e0, e1, chi, x, y, z);
                }
                const bool bad = chi > (double)5.991f;
                ol[e] = bad; lv[e] = bad; nb += bad;
            }
            nbad = (int)g.sum1((double)nb);
            if (round == 2) robust = false;   // e->setRobustKernel(0)
            if (h.n < 10) break;              // optimizer.edges().size() < 10
        }
    }
    if (outlier_copy)   // zero-copy result: the flags also into the caller-visible block
        for (int e = tid; e < h.n; e += NT) outlier_copy[h.off + e] = ol[e];
    if (tid == 0) {
        PoseOut& o = out[f];
#pragma unroll
        for (int k = 0; k < 8; k++) o.T[k] = T[k];
        o.n_inliers = h.n >= 3 ? h.n - nbad : 0;
        o.trials = trials;
    }
}

// ---------------------------------------------------------------------------
// host
// ---------------------------------------------------------------------------
struct PoseWorkspace {
    void* d = nullptr;
    size_t dcap = 0;
    void* h = nullptr;
    void* hd = nullptr;   // device alias of h
    size_t hcap = 0;
    ~PoseWorkspace() {
        if (d) (void)hipFree(d);
        if (h) (void)hipHostFree(h);
    }
};

PoseWorkspace* pose_ws_create() { return new PoseWorkspace(); }
void pose_ws_destroy(PoseWorkspace* w) { delete w; }

#define PSOK(x)                                                                                    \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess) {                                                                    \
            std::fprintf(stderr, "orbhip pose: %s: %s\n", #x, hipGetErrorString(e_));              \
            return ORBHIP_ERR_DEVICE;                                                              \
        }                                                                                          \
    } while (0)

int pose_opt_batch(PoseWorkspace* ws, const orbhip_pose_problem* probs, int B, orbhip_pose_result* res,
                   hipStream_t st) {
    if (!ws || !probs || !res || B <= 0) return ORBHIP_ERR_ARG;
    size_t E = 0;
    for (int b = 0; b < B; b++) {
        const orbhip_pose_problem& p = probs[b];
        if (p.n < 0 || !p.pose_q || !p.pose_t || (p.n && (!p.points || !p.uv || !p.octave || !p.inv_sigma2)))
            return ORBHIP_ERR_ARG;
        for (int e = 0; e < p.n; e++)
            if (p.octave[e] < 0 || p.octave[e] >= p.n_octaves) return ORBHIP_ERR_ARG;
        E += p.n;
    }
    // packed: [hdr B][edges E] (one upload) [out B][outlier E] (one download) [chi2 E][level E]
    auto al = [](size_t x) { return (x + 255) & ~size_t(255); };
    const size_t o_hdr = 0, o_edge = al(sizeof(PoseHdr) * B), o_out = o_edge + al(sizeof(PoseEdgeIn) * E);
    const size_t o_ol = o_out + al(sizeof(PoseOut) * B), o_c2 = o_ol + al(E);
    const size_t o_lv = o_c2 + al(sizeof(double) * E), total = o_lv + al(E);
    if (ws->dcap < total) {
        if (ws->d) (void)hipFree(ws->d);
        ws->d = nullptr;
        ws->dcap = 0;
        PSOK(hipMalloc(&ws->d, total));
        ws->dcap = total;
    }
    if (ws->hcap < total) {
        if (ws->h) (void)hipHostFree(ws->h);
        ws->h = nullptr;
        ws->hcap = 0;
        PSOK(hipHostMalloc(&ws->h, total + total / 4, hipHostMallocDefault));
        ws->hcap = total + total / 4;
        PSOK(hipHostGetDevicePointer(&ws->hd, ws->h, 0));
    }
    char* H = (char*)ws->h;
    char* D = (char*)ws->d;
    PoseHdr* hh = (PoseHdr*)(H + o_hdr);
    PoseEdgeIn* he = (PoseEdgeIn*)(H + o_edge);
    const float deltaMono = (float)std::sqrt(5.991);
    size_t off = 0;
    for (int b = 0; b < B; b++) {
        const orbhip_pose_problem& p = probs[b];
        PoseHdr& h = hh[b];
        // g2o::SE3Quat(q.cast<double>(), t.cast<double>()) normalises the rotation
        double x = p.pose_q[0], y = p.pose_q[1], z = p.pose_q[2], w = p.pose_q[3];
        if (w < 0) { x = -x; y = -y; z = -z; w = -w; }
        const double nn = std::sqrt(x * x + y * y + z * z + w * w);
        h.T0[0] = x / nn; h.T0[1] = y / nn; h.T0[2] = z / nn; h.T0[3] = w / nn;
        h.T0[4] = p.pose_t[0]; h.T0[5] = p.pose_t[1]; h.T0[6] = p.pose_t[2]; h.T0[7] = 0;
        h.fx = p.fx; h.fy = p.fy; h.cx = p.cx; h.cy = p.cy; h.delta = deltaMono;
        h.n = p.n; h.off = (int)off;
        for (int e = 0; e < p.n; e++) {
            PoseEdgeIn& E_ = he[off + e];
            E_.X[0] = p.points[3 * e]; E_.X[1] = p.points[3 * e + 1]; E_.X[2] = p.points[3 * e + 2];
            E_.u = p.uv[2 * e]; E_.v = p.uv[2 * e + 1];
            E_.info = p.inv_sigma2[p.octave[e]];
        }
        off += p.n;
    }
    // small batches (one tracking frame): a shader upload and results written straight into the
    // pinned block (no DMA-engine copies); large batches: DMA both ways
    const size_t in_bytes = o_edge + sizeof(PoseEdgeIn) * E;
    const bool small = in_bytes <= ((size_t)1 << 20);
    if (small) PSOK(upload_inputs(ws->hd, D, H, in_bytes, st));
    else PSOK(hipMemcpyAsync(D, H, in_bytes, hipMemcpyHostToDevice, st));
    // W = 4 wavefronts per frame while that still fills the chip's SIMDs twice over, else one
    int W = B <= 512 ? 4 : 1;
    if (const char* s = std::getenv("ORBHIP_POSE_WAVES")) W = std::atoi(s) == 1 ? 1 : 4;
    const PoseHdr* dh = (const PoseHdr*)(D + o_hdr);
    const PoseEdgeIn* de = (const PoseEdgeIn*)(D + o_edge);
    uint8_t* dlv = (uint8_t*)(D + o_lv);
    uint8_t* dol = (uint8_t*)(D + o_ol);
    double* dc2 = (double*)(D + o_c2);
    PoseOut* dout = (PoseOut*)((small ? (char*)ws->hd : D) + o_out);
    uint8_t* olc = small ? (uint8_t*)ws->hd + o_ol : nullptr;
    if (W == 4)
        hipLaunchKernelGGL(k_pose_opt<4>, dim3((unsigned)B), dim3(256), 0, st, dh, de, dlv, dol, dc2, dout, olc, B);
    else
        hipLaunchKernelGGL(k_pose_opt<1>, dim3((unsigned)((B + 3) / 4)), dim3(256), 0, st, dh, de, dlv, dol, dc2,
                           dout, olc, B);
    PSOK(hipGetLastError());
    if (!small) PSOK(hipMemcpyAsync(H + o_out, D + o_out, o_ol - o_out + E, hipMemcpyDeviceToHost, st));
    PSOK(hipStreamSynchronize(st));
    const PoseOut* ho = (const PoseOut*)(H + o_out);
    const uint8_t* hol = (const uint8_t*)(H + o_ol);
    for (int b = 0; b < B; b++) {
        orbhip_pose_result& r = res[b];
        for (int k = 0; k < 4; k++) r.pose_q[k] = (float)ho[b].T[k];
        for (int k = 0; k < 3; k++) r.pose_t[k] = (float)ho[b].T[4 + k];
        r.n_inliers = ho[b].n_inliers;
        r.lm_trials = ho[b].trials;
        if (r.outlier) std::memcpy(r.outlier, hol + hh[b].off, probs[b].n);
    }
    return ORBHIP_OK;
}

}  // namespace orbhip
