// Persistent tiled-DAG Cholesky solve of the reduced camera system S xp = bs (a20 / a22: g2o
// LinearSolverEigen::solve behind OptimizationAlgorithmLevenberg; C4 single LBA, C5 GBA).
//
// ONE launch per solve. S is cut into 32x32 tiles inside its envelope (row_first); the launch has
// one CHAIN workgroup (blockIdx 0) and G HELPER workgroups, 256 threads each, one per CU.
//   helpers   own the off-diagonal tiles (R, C), R >= C + 2 ("full" tasks): acc = A_RC - sum over
//             p < C of L_Rp L_Cp^T, then L_RC = acc Linv_C^T (Linv_C from the chain). They also
//             build the PARTIAL diagonal tiles A_JJ - sum_{p <= J-3} L_Jp L_Jp^T (with the
//             right-hand-side partial b_J - sum L_Jp y_p) and partial sub-diagonal tiles
//             A_{C+1,C} - sum_{p <= C-3} L_{C+1,p} L_Cp^T.
//   chain     interval k: finishes tile (k+1, k) with columns k-2, k-1, forms L_{k+1,k} =
//             T Linv_k^T, finishes the diagonal tile k+1 with columns k-1, k (and its rhs), factors
//             it (diag32_linv: 4x4 pivot blocks on v_mfma_f64_16x16x4f64) into Linv_{k+1}, y_{k+1}.
//             Then the backward substitution L^T x = y, column by column, in the chain workgroup.
// Every tile is stored as 4 quadrants in the MFMA C layout of its TRANSPOSE (lane l, component q:
// T[16a + (l & 15)][16b + (l >> 4) + 4q]), which is also the A-operand order: a loaded quadrant is
// directly an MFMA operand (the ba_chol_reg.hip convention).
// Hand-offs (MI355X_MICROARCH.md, visibility table row 1): every published byte is stored sc1
// (buffer_store ... sc1 / agent-scope atomic stores), each storing wave drains vmcnt, the
// workgroup barriers, ONE lane stores the flag (agent-scope atomic); the consumer polls the flag
// with sc1 loads (one wave), barriers, then reads the bytes with sc1 loads only. Flags hold the
// solve's epoch (a per-problem counter advanced by the last workgroup to finish), so nothing is
// reset between solves. Every spin is bounded: a timeout sets the abort word (epoch), every
// waiter gives up, flag[0] = 0 and x = 0 (the LM rejects the trial).
// Deadlock freedom: each helper runs its tasks in key order (dependency order over the whole
// DAG, dag_plan) and every workgroup of the launch is resident (grid <= 256, one per CU by LDS).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <mutex>
#include <utility>
#include <vector>

#include "ba_args.h"
#include "ba_chol.h"
#include "ba_chol_dag.h"
#include "ba_diag16.h"
#include "wave_f64.h"

namespace orbhip {

namespace {

constexpr int kT = kDagTile;
constexpr int kTD = kT * kT;            // doubles per tile
constexpr unsigned kSpinMax = 1u << 19;   // default poll bound (ORBHIP_DAG_SPIN_MAX overrides)
constexpr size_t kMinLds = 84 * 1024;   // > 80 KB: one workgroup per CU
constexpr int kCopyTask = 0x7FFF;       // task code kCopyTask << 16 | k: the copies of interval k
#ifndef ORBHIP_DAG_NEWTON
#define ORBHIP_DAG_NEWTON 1
#endif
constexpr int kNewton = ORBHIP_DAG_NEWTON;   // Newton steps after v_rsq_f64 / v_rcp_f64 in the pivots
#ifndef ORBHIP_DAG_DIAG_DPP
#define ORBHIP_DAG_DIAG_DPP 1   // r05: the 16x16 diagonal factorizations by DPP elimination (diag16_dpp)
#endif
#ifndef ORBHIP_DAG_T_W1
// r05: wave 1 (idle after its publishes) applies T_{k+1}'s column-k term for waves 2 / 3: the
// interval 13.55k -> 12.8k cycles at n = 294 (every wave now ends within ~0.6k of the others)
#define ORBHIP_DAG_T_W1 1
#endif

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(1))) int gint;
typedef __attribute__((address_space(1))) double gdbl;

struct DagK {
    const double* S;
    const double* bs;
    double* x;
    int* flag;
    const int* rf;
    double* buf;
    int* ints;
    const int* toff;
    const int* tasks;
    int need_off;        // tasks[need_off ...]: the chain backward's column counts (DagDev::need_off)
    const int* gate;
    unsigned long long* dbg;
    int n, NT, G;
    int pb;       // backward over the helpers (dag_helper_backward) or in the chain alone
    int hsleep;   // helpers' poll back-off (units of s_sleep 1)
    unsigned smax;   // polls before a wait gives up (timeout: ctl[2] abort, ctl[3] counted)
    int ld;          // row stride of S
    const int* perm; // nullptr: S itself; else row / column i of the solved matrix is S's perm[i] (-1: padding)
    int nti;         // partial mode (> 0): tiles [0, nti) are factored; every tile (R, C >= nti) only receives
                     // the updates of columns < nti (A = 0 there: the eliminated block's Schur contribution)
};

__device__ __forceinline__ int ld_flag(const int* p) {
    return __hip_atomic_load((gint*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_flag(int* p, int v) {
    __hip_atomic_store((gint*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ld_sc1(const double* p) {
    return __hip_atomic_load((gdbl*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1(double* p, double v) {
    __hip_atomic_store((gdbl*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void drain_stores() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
// workgroup barrier ordering LDS only: __syncthreads() is a workgroup fence, which on gfx950 also
// drains vmcnt, i.e. would wait for every wave's outstanding global loads and stores
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

// one quadrant (256 doubles, 4 per lane) at dbl_off of the DAG buffer, sc1 (16-byte accesses)
__device__ __forceinline__ double4_t qload(__amdgpu_buffer_rsrc_t rs, int dbl_off) {
    const int off = (dbl_off + (int)(threadIdx.x & 63) * 4) * 8;
    const u32x4 u = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 16);
    const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, off + 16, 0, 16);
    return double4_t{mk64(u.x, u.y), mk64(u.z, u.w), mk64(v.x, v.y), mk64(v.z, v.w)};
}
__device__ __forceinline__ void qstore(__amdgpu_buffer_rsrc_t rs, int dbl_off, const double4_t& d) {
    const int off = (dbl_off + (int)(threadIdx.x & 63) * 4) * 8;
    const u32x4 u = {lo32(d[0]), hi32(d[0]), lo32(d[1]), hi32(d[1])};
    const u32x4 v = {lo32(d[2]), hi32(d[2]), lo32(d[3]), hi32(d[3])};
    __builtin_amdgcn_raw_buffer_store_b128(u, rs, off, 0, 16);
    __builtin_amdgcn_raw_buffer_store_b128(v, rs, off + 16, 0, 16);
}
// Column copies of a tile for the chain's backward: lane L = c + 32 hh (c = L & 31, hh = L >> 5)
// reads column c, rows 16 hh .. 16 hh + 15, as 8 pairs; pair i of every lane forms one contiguous
// 1 KB block, so each of a tile's 8 loads is fully coalesced. Element (r, c) sits at double
// 2 (64 i + L) + e, i = (r & 15) >> 1, e = r & 1, L = c + 32 (r >> 4).
__device__ __forceinline__ int cm_idx(int r, int c) {
    return 2 * (64 * ((r & 15) >> 1) + c + 32 * (r >> 4)) + (r & 1);
}
// quadrant `quad` (a = quad >> 1, b = quad & 1) of a tile held in the quadrant layout (lane l,
// component q: element (16 a + (l & 15), 16 b + 4 q + (l >> 4))) stored into its column copy
__device__ __forceinline__ void cmstore(__amdgpu_buffer_rsrc_t rs, int dbl_off, int quad, const double4_t& d) {
    const int lane = threadIdx.x & 63, a = quad >> 1, b = quad & 1;
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const u32x2 u = {lo32(d[q]), hi32(d[q])};
        const int i = dbl_off + cm_idx(16 * a + (lane & 15), 16 * b + 4 * q + (lane >> 4));
        __builtin_amdgcn_raw_buffer_store_b64(u, rs, i * 8, 0, 16);
    }
}
// this lane's column of a column copy (v[j] = element (16 hh + j, c)), sc1. The lane's part of the
// address is a VGPR that never changes, the tile's (wave-uniform) part and the block's go in the
// scalar offset: no VGPR is written per load. (r06, late: with the whole address per load in VGPRs
// the allocator took the other prefetch set's destination registers as address temporaries, so
// the backward waited for that set's loads, vmcnt(1) / vmcnt(0), at every step)
__device__ __forceinline__ void cmload(__amdgpu_buffer_rsrc_t rs, int dbl_off, double (&v)[16]) {
    const int voff = 16 * (int)(threadIdx.x & 63);
    const int soff = __builtin_amdgcn_readfirstlane(dbl_off * 8);
#pragma unroll
    for (int i = 0; i < 8; i++) {
        const u32x4 u = __builtin_amdgcn_raw_buffer_load_b128(rs, voff, soff + 1024 * i, 16);
        v[2 * i] = mk64(u.x, u.y);
        v[2 * i + 1] = mk64(u.z, u.w);
    }
}
// a quadrant held in LDS (same layout)
__device__ __forceinline__ double4_t lq(const double* base) {
    const double* p = base + (threadIdx.x & 63) * 4;
    return double4_t{p[0], p[1], p[2], p[3]};
}
__device__ __forceinline__ void sq(double* base, const double4_t& v) {
    double* p = base + (threadIdx.x & 63) * 4;
    p[0] = v[0]; p[1] = v[1]; p[2] = v[2]; p[3] = v[3];
}
// index of element (r, c) of a 32x32 tile in the quadrant layout
__device__ __forceinline__ int qidx(int r, int c) {
    return (((r >> 4) * 2 + (c >> 4)) * 256) + (((r & 15) + 16 * (c & 3)) * 4) + ((c & 15) >> 2);
}
// element (r, c) of the solved matrix (plain loads: S is written by earlier kernels only): the
// lower triangle of S is read (mirrored above the diagonal); identity outside the matrix and on
// padding rows of a permuted matrix; zero in the trailing block of a partial solve
__device__ __forceinline__ double s_elem(const DagK& k, int r, int c) {
    const bool in = r < k.n && c < k.n;
    int pr = r, pc = c;
    bool z = !in;
    if (k.perm && in) {
        pr = k.perm[r];
        pc = k.perm[c];
        z = pr < 0 || pc < 0;
    }
    if (k.nti && r >= kT * k.nti && c >= kT * k.nti) z = true;   // the separator block: contributions only
    const size_t off = z ? 0 : (pr >= pc ? (size_t)pr * k.ld + pc : (size_t)pc * k.ld + pr);
    const double s = k.S[off];
    return z ? (r == c && (!in || r < kT * k.nti || !k.nti) ? 1.0 : 0.0) : s;
}
// right-hand side entry i (zero on padding and in the trailing block of a partial solve)
__device__ __forceinline__ double s_rhs(const DagK& k, int i) {
    if (i >= k.n || (k.nti && i >= kT * k.nti)) return 0.0;
    const int pi = k.perm ? k.perm[i] : i;
    return pi < 0 ? 0.0 : k.bs[pi];
}
// quadrant (a, b) of tile (R, C) of the solved matrix, in the quadrant layout
__device__ __forceinline__ double4_t s_quad(const DagK& k, int R, int C, int a, int b) {
    const int lane = threadIdx.x & 63;
    const int r = kT * R + 16 * a + (lane & 15);
    double4_t v;
#pragma unroll
    for (int q = 0; q < 4; q++) v[q] = s_elem(k, r, kT * C + 16 * b + (lane >> 4) + 4 * q);
    return v;
}
// c4 -= A B^T in the transposed C layout (a: L_Jk quadrant, b: L_Ik quadrant -> C_IJ^T). (Splitting
// the 4-deep accumulation over two accumulators measured slower: the extra adds and AGPR moves
// cost more than the MFMA latency they hide.)
__device__ __forceinline__ void mfma_sub(double4_t& c4, const double4_t& a, const double4_t& b) {
    c4 = __builtin_amdgcn_mfma_f64_16x16x4f64(-a[0], b[0], c4, 0, 0, 0);
    c4 = __builtin_amdgcn_mfma_f64_16x16x4f64(-a[1], b[1], c4, 0, 0, 0);
    c4 = __builtin_amdgcn_mfma_f64_16x16x4f64(-a[2], b[2], c4, 0, 0, 0);
    c4 = __builtin_amdgcn_mfma_f64_16x16x4f64(-a[3], b[3], c4, 0, 0, 0);
}
// r += Linv_q A_q^T (Linv quadrant in operand order, tile quadrant t)
__device__ __forceinline__ void panel_add(double4_t& r, const double4_t& a, const double4_t& t) {
    r = __builtin_amdgcn_mfma_f64_16x16x4f64(a[0], t[0], r, 0, 0, 0);
    r = __builtin_amdgcn_mfma_f64_16x16x4f64(a[1], t[1], r, 0, 0, 0);
    r = __builtin_amdgcn_mfma_f64_16x16x4f64(a[2], t[2], r, 0, 0, 0);
    r = __builtin_amdgcn_mfma_f64_16x16x4f64(a[3], t[3], r, 0, 0, 0);
}
// (L y) of a quadrant for its row l & 15: y values of this lane's columns (rg + 4q), summed over
// the 4 row groups (identical in every row group)
__device__ __forceinline__ double lmul_y4(const double4_t& l, double y0, double y1, double y2, double y3) {
    return col4_sum(l[0] * y0 + l[1] * y1 + l[2] * y2 + l[3] * y3);
}
__device__ __forceinline__ double lmul_ylds(const double4_t& l, const double* y) {
    const int rg = (threadIdx.x & 63) >> 4;
    return lmul_y4(l, y[rg], y[rg + 4], y[rg + 8], y[rg + 12]);
}
// this lane's part of lmul_ylds before the cross-row sum: several quadrants' parts are added
// first and summed across the row groups once (col4_sum)
__device__ __forceinline__ double lmul_part(const double4_t& l, const double* y) {
    const int rg = (threadIdx.x & 63) >> 4;
    return l[0] * y[rg] + l[1] * y[rg + 4] + l[2] * y[rg + 8] + l[3] * y[rg + 12];
}

// every lane's flag (nullptr: none) equal to epoch; false on abort / timeout (wave-uniform)
__device__ bool wave_wait_all(const int* f, int epoch, int* ctl, unsigned smax) {
    for (unsigned spins = 0;; spins++) {
        const bool ok = !f || ld_flag(f) == epoch;
        if (__all(ok)) return true;
        if (ld_flag(ctl + 2) == epoch) return false;
        if (spins >= smax) {
            if ((threadIdx.x & 63) == 0) {
                st_flag(ctl + 2, epoch);
                __hip_atomic_fetch_add((gint*)(ctl + 3), 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            return false;
        }
        __builtin_amdgcn_s_sleep(2);
    }
}
// the number m >= 1 of leading entries i < cnt (<= 64) with fa[i] == fb[i] == fc[i] == epoch
// (fb / fc optional); 0 on abort / timeout (wave-uniform)
__device__ int wave_wait_prefix(const int* fa, const int* fb, const int* fc, int cnt, int epoch, int* ctl, int hsleep,
                                 unsigned smax) {
    const int lane = threadIdx.x & 63;
    for (unsigned spins = 0;; spins++) {
        bool ok = true;
        if (lane < cnt) {
            ok = ld_flag(fa + lane) == epoch;
            if (fb) ok = ok && ld_flag(fb + lane) == epoch;
            if (fc) ok = ok && ld_flag(fc + lane) == epoch;
        }
        const unsigned long long bad = __ballot(!ok);
        const int m = bad ? __builtin_ctzll(bad) : cnt;
        if (m > 0) return m;
        if (ld_flag(ctl + 2) == epoch) return 0;
        if (spins >= smax) {
            if (lane == 0) {
                st_flag(ctl + 2, epoch);
                __hip_atomic_fetch_add((gint*)(ctl + 3), 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            return 0;
        }
        for (int z = 0; z < hsleep; z++) __builtin_amdgcn_s_sleep(1);   // helpers back off
    }
}

struct Lay {   // offsets (doubles) into the DAG buffer, flags
    int oL, oP, oLi, oY, oR, oX, oS, oCM, oCI;
    int *ctl, *fL, *fP0, *fP1, *fP2, *fCh, *fX, *fS, *fCp;
    __device__ Lay(const DagK& a) {
        const int NT = a.NT;
        oL = 0;
        oP = NT * NT * kTD;
        oLi = oP + 3 * NT * kTD;
        oY = oLi + NT * kTD;
        oR = oY + NT * kT;
        oX = oR + NT * kT;   // backward: x_R published by the chain
        oS = oX + NT * kT;   // backward: the helpers' sums s_j = y_j - sum_{R >= j+2} L(R, j)^T x_R
        // the chain's backward (short rows, dag_chain): column-major copies of the L tiles (element
        // (r, c) at 32 c + r) and of the diagonal inverses, so that a lane's tile column is 16
        // contiguous doubles (the full tiles' copies by their helper tasks, the chain's own tiles
        // by the copy tasks, fCp)
        oCM = oS + NT * kT;
        oCI = oCM + NT * NT * kTD;
        ctl = a.ints;
        fL = ctl + 4;
        fP0 = fL + NT * NT;
        fP1 = fP0 + NT;
        fP2 = fP1 + NT;
        fCh = fP2 + NT;
        fX = fCh + NT;
        fS = fX + NT;
        fCp = fS + NT;
    }
};

// ---------------------------------------------------------------------------------------------
// helper backward: helper h owns the columns j = h, h + G, ... <= NT - 3, spread over its 4
// waves. A wave accumulates s_j = y_j - sum_{R >= j+2} L(R, j)^T x_R (in LDS) as the chain
// publishes x_R (sc1 data, flag fX[R]), from R = NT - 1 down, and publishes s_j (oS, fS[j]) once
// R = j + 2 is in; the chain adds the sub-diagonal term L(j+1, j)^T x_{j+1} itself. L is final
// once x_{NT-1} exists (the chain's forward is over), so a wave loads its tiles without flags.
// An aborted solve (ctl[2]) ends every wait.
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ void tile_lt_x(const double4_t* t, const double* x, double (&out)[2][4]);
__device__ void dag_helper_backward(const DagK& a, const Lay& L, __amdgpu_buffer_rsrc_t rs, int epoch, double* lds,
                                    int h) {
    const int NT = a.NT, G = a.G;
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63, cc = lane & 15, rg = lane >> 4;
    if (G <= 0 || !a.pb) return;
    // this wave's columns: j = h + G * (wid + 4 i)
    const int j_first = h + G * wid;
    if (j_first > NT - 3) return;
    double* acc = lds;                  // NT x 32 (a column's running sum, owned by one wave)
    double* xw = lds + 4096 + 64 * wid; // this wave's copy of x_R
    for (int R = NT - 1; R >= j_first + 2; R--) {
        if (!wave_wait_all(lane == 0 ? L.fX + R : nullptr, epoch, L.ctl, a.smax)) return;
        if (R == NT - 1) {   // the forward is over (x_{NT-1} exists): every y_j is published
            for (int j = j_first; j <= NT - 3; j += 4 * G)
                if (lane < kT) acc[j * kT + lane] = ld_sc1(a.buf + L.oY + j * kT + lane);
        }
        if (lane < kT) xw[lane] = ld_sc1(a.buf + L.oX + R * kT + lane);
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();
        const int rfR = a.rf[R];
        for (int j = j_first; j <= R - 2; j += 4 * G) {
            if (j >= rfR) {
                double4_t tl[4];
#pragma unroll
                for (int qd = 0; qd < 4; qd++) tl[qd] = qload(rs, L.oL + (R * NT + j) * kTD + qd * 256);
                double t[2][4];
                tile_lt_x(tl, xw, t);
                if (cc == 0) {
#pragma unroll
                    for (int b = 0; b < 2; b++)
#pragma unroll
                        for (int q = 0; q < 4; q++) acc[j * kT + 16 * b + rg + 4 * q] -= t[b][q];
                }
            }
            if (j == R - 2) {   // s_j complete: publish
                __builtin_amdgcn_wave_barrier();
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                if (lane < kT) st_sc1(a.buf + L.oS + j * kT + lane, acc[j * kT + lane]);
                drain_stores();
                if (lane == 0) st_flag(L.fS + j, epoch);
            }
        }
        __builtin_amdgcn_wave_barrier();
    }
}

// ---------------------------------------------------------------------------------------------
// helper workgroup: its tasks in order
// ---------------------------------------------------------------------------------------------
__device__ void dag_helper(const DagK& a, const Lay& L, __amdgpu_buffer_rsrc_t rs, int epoch, double* lds, int h) {
    const int tid = threadIdx.x, wid = tid >> 6, lane = tid & 63, cc = lane & 15, rg = lane >> 4;
    const int rq = wid >> 1, cq = wid & 1, quad = 2 * rq + cq;
    const int NT = a.NT;
    double* Tx = lds + 2048;
    int* word = (int*)(lds + 4096);
    const int t0 = a.toff[h], t1 = a.toff[h + 1];
    int wsel = 0;   // rotating LDS word of the poll results
    auto wg_prefix = [&](const int* fa, const int* fb, const int* fc, int cnt) -> int {
        if (wid == 0) {
            const int m = wave_wait_prefix(fa, fb, fc, cnt, epoch, L.ctl, a.hsleep, a.smax);
            if (lane == 0) word[wsel] = m;
        }
        __syncthreads();
        const int m = word[wsel];
        wsel = (wsel + 1) & 3;
        return m;
    };
    const bool copies = !a.pb && !a.nti;   // the chain's backward reads column-major copies
    for (int t = t0; t < t1; t++) {
        const int code = a.tasks[t];
        const int R = code >> 16, C = code & 0xFFFF;
        if (R == kCopyTask) {
            // copy task of interval k = C: column-major copies of the tiles the chain published in
            // it (L(k+1, k), L(k+1, k-1), Linv_k; one flag covers all three), then fCp[k]
            const int k = C;
            if (wg_prefix(L.fCh + k, nullptr, nullptr, 1) == 0) break;
            const int tA = L.oL + ((k + 1) * NT + k) * kTD, tI = L.oLi + k * kTD;
            const double4_t qa = qload(rs, tA + quad * 256), qi = qload(rs, tI + quad * 256);
            double4_t qb = {0, 0, 0, 0};
            if (k >= 1) qb = qload(rs, L.oL + ((k + 1) * NT + k - 1) * kTD + quad * 256);
            cmstore(rs, L.oCM + ((k + 1) * NT + k) * kTD, quad, qa);
            cmstore(rs, L.oCI + k * kTD, quad, qi);
            if (k >= 1) cmstore(rs, L.oCM + ((k + 1) * NT + k - 1) * kTD, quad, qb);
            drain_stores();
            __syncthreads();
            if (tid == 0) st_flag(L.fCp + k, epoch);
            continue;
        }
        // by R - C: 0 the diagonal partial (columns <= C-4), 1 the sub-diagonal partial (<= C-3), 2
        // the second sub-diagonal's partial (<= C-2), >= 3 a full tile (every column, then the TRSM);
        // 3: a tile of a partial solve's trailing block (C >= nti): every column < nti, no TRSM
        const int dRC = R - C;
        const bool upd = a.nti && C >= a.nti;
        const int type = upd ? 3 : (dRC >= 3 ? 2 : (dRC == 0 ? 0 : 1));
        const int ps = max(a.rf[R], a.rf[C]),
                  pe = upd ? a.nti : (dRC >= 3 ? C : (dRC == 2 ? C - 1 : (dRC == 1 ? C - 2 : C - 3)));
        double4_t acc = s_quad(a, R, C, rq, cq);
        const bool dg = type == 0 || (upd && dRC == 0);   // a diagonal tile: with its right-hand side
        const bool rhs = dg && cq == 0;
        const bool skip = dg && quad == 1;   // the upper quadrant of a diagonal tile: unused
        double rv = 0.0;
        if (rhs) {
            const int i = kT * R + 16 * rq + cc;
            rv = s_rhs(a, i);
        }
        bool fail = false;
        for (int p = ps; p < pe && !fail;) {
            const int cnt = min(64, pe - p);
            const int m = wg_prefix(L.fL + R * NT + p, R != C ? L.fL + C * NT + p : nullptr,
                                    dg ? L.fCh + p : nullptr, cnt);
            if (m == 0) {
                fail = true;
                break;
            }
            for (int i = p; i < p + m; i++) {
                const int tC = L.oL + (C * NT + i) * kTD, tR = L.oL + (R * NT + i) * kTD;
                const double4_t a0 = qload(rs, tC + (2 * cq) * 256), a1 = qload(rs, tC + (2 * cq + 1) * 256);
                const double4_t b0 = qload(rs, tR + (2 * rq) * 256), b1 = qload(rs, tR + (2 * rq + 1) * 256);
                if (!skip) {
                    mfma_sub(acc, a0, b0);
                    mfma_sub(acc, a1, b1);
                }
                if (rhs) {
                    const double* y = a.buf + L.oY + i * kT;
                    rv -= lmul_y4(b0, ld_sc1(y + rg), ld_sc1(y + rg + 4), ld_sc1(y + rg + 8), ld_sc1(y + rg + 12));
                    rv -= lmul_y4(b1, ld_sc1(y + 16 + rg), ld_sc1(y + 20 + rg), ld_sc1(y + 24 + rg),
                                  ld_sc1(y + 28 + rg));
                }
            }
            p += m;
        }
        if (fail) break;
        int* target;
        if (type == 2) {
            if (wg_prefix(L.fCh + C, nullptr, nullptr, 1) == 0) break;
            sq(Tx + quad * 256, acc);
            __syncthreads();
            const int li = L.oLi + C * kTD;
            double4_t out = {0, 0, 0, 0};
            panel_add(out, qload(rs, li + (2 * cq) * 256), lq(Tx + (2 * rq) * 256));
            if (cq == 1) panel_add(out, qload(rs, li + 3 * 256), lq(Tx + (2 * rq + 1) * 256));
            qstore(rs, L.oL + (R * NT + C) * kTD + quad * 256, out);
            if (copies) cmstore(rs, L.oCM + (R * NT + C) * kTD, quad, out);   // covered by the tile's flag
            target = L.fL + R * NT + C;
        } else if (type == 3) {   // the trailing block's contribution, where its L tile would be
            qstore(rs, L.oL + (R * NT + C) * kTD + quad * 256, acc);
            if (rhs && rg == 0) st_sc1(a.buf + L.oR + R * kT + 16 * rq + cc, rv);
            target = L.fL + R * NT + C;
        } else {
            qstore(rs, L.oP + (dRC * NT + C) * kTD + quad * 256, acc);
            if (rhs && rg == 0) st_sc1(a.buf + L.oR + C * kT + 16 * rq + cc, rv);
            target = L.fP0 + dRC * NT + C;   // fP0, fP1, fP2 are consecutive rows of NT
        }
        drain_stores();
        __syncthreads();
        if (tid == 0) st_flag(target, epoch);
    }
    dag_helper_backward(a, L, rs, epoch, lds, h);
}

// ---------------------------------------------------------------------------------------------
// chain workgroup: the diagonal critical path, then the backward substitution
// ---------------------------------------------------------------------------------------------
// wave 0: Linv of the diagonal tile in Dx into Lin, y = Linv r into y (32)
__device__ __forceinline__ bool chain_factor(const double* Dx, double* scr, double* Lin, const double* rvec,
                                             double* y) {
    const bool ok = diag32_linv<kNewton>([&](int r, int c) { return Dx[qidx(r, c)]; }, scr,
                                         [&](int r, int c, double v) { Lin[qidx(r, c)] = v; });
    wave_lds_sync();
    const int lane = threadIdx.x & 63, i = lane >> 1, hh = lane & 1;
    double s = 0.0;
#pragma unroll
    for (int c = 0; c < 16; c++) s = fma(Lin[qidx(i, 16 * hh + c)], rvec[16 * hh + c], s);
    s += dpp64<0xB1>(s);
    if (hh == 0) y[i] = s;
    wave_lds_sync();
    return ok;
}

// sum over the two half-waves (lane l and l ^ 32), the same bits in both
__device__ __forceinline__ double half32_sum(double v) {
    const auto tl = __builtin_amdgcn_permlane32_swap(lo32(v), lo32(v), false, false);
    const auto th = __builtin_amdgcn_permlane32_swap(hi32(v), hi32(v), false, false);
    return mk64(tl[0], th[0]) + mk64(tl[1], th[1]);
}
// (T^T x)[c] for a tile column held by cmload and x (32 doubles in LDS): every lane of column c
// returns it
__device__ __forceinline__ double bwd_col_dot(const double (&v)[16], const double* x) {
    const double* xh = x + 16 * ((threadIdx.x & 63) >> 5);
    double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
#pragma unroll
    for (int i = 0; i < 16; i += 4) {
        s0 = fma(v[i], xh[i], s0);
        s1 = fma(v[i + 1], xh[i + 1], s1);
        s2 = fma(v[i + 2], xh[i + 2], s2);
        s3 = fma(v[i + 3], xh[i + 3], s3);
    }
    return half32_sum((s0 + s1) + (s2 + s3));
}

// the contribution L^T x of one tile (4 quadrants q0..q3 of this lane) to the 32 columns: lanes with
// (lane & 15) == 0 receive column 16b + rg + 4q in out[b][q]
__device__ __forceinline__ void tile_lt_x(const double4_t* t, const double* x, double (&out)[2][4]) {
    const int cc = threadIdx.x & 15;
    const double x0 = x[cc], x1 = x[16 + cc];
#pragma unroll
    for (int b = 0; b < 2; b++)
#pragma unroll
        for (int q = 0; q < 4; q++) out[b][q] = row16_sum(fma(t[b][q], x0, t[2 + b][q] * x1));
}

// wave-level helpers of the chain's 32x32 diagonal factorization, split at its two 16x16 pivots
// (the diag32_linv steps of ba_diag16.h, with the second pivot's inputs handed in by wave 1):
// part A: Linv11 of D11 (registers, C layout) into quadrant 0 of Lq (and zeros into quadrant 1),
// returns Linv11 in the C layout (lin11)
#if ORBHIP_DAG_DIAG_DPP
// D (C layout) -> v (column lane & 15, rows 0..15) through a padded column-major scratch (stride
// 18 doubles: the 16 lanes' 16-byte reads start on distinct banks)
__device__ __forceinline__ void c_to_cols(const double4_t& d, double* scr, double (&v)[16]) {
    const int lane = threadIdx.x & 63, cc = lane & 15, rg = lane >> 4;
#pragma unroll
    for (int q = 0; q < 4; q++) scr[cc * 18 + rg + 4 * q] = d[q];
    wave_lds_sync();
    const double* p = scr + cc * 18;
#pragma unroll
    for (int i = 0; i < 16; i++) v[i] = p[i];
    wave_lds_sync();
}
#endif
// part A: Linv11 of D11 (registers, C layout) into quadrant 0 of Lq (and zeros into quadrant 1),
// returns Linv11 in the C layout (lin11). scr: 288 doubles of wave-private LDS scratch.
__device__ __forceinline__ bool diag_part_a(const double4_t& d11, double* Lq, double4_t& lin11, double* scr) {
#if ORBHIP_DAG_DIAG_DPP
    // DPP column elimination (ba_diag16.h, diag16_dpp), then the quadrant stores
    const int lane = threadIdx.x & 63, cc = lane & 15, rg = lane >> 4;
    double v[16];
    c_to_cols(d11, scr, v);
    const bool ok = diag16_dpp<kNewton>(v, scr, lin11);
#pragma unroll
    for (int q = 0; q < 4; q++) {
        Lq[qidx(rg + 4 * q, cc)] = lin11[q];
        Lq[qidx(rg + 4 * q, 16 + cc)] = 0.0;
    }
    return ok;
#else
    (void)scr;
    return diag16_linv<kNewton>(d11, [&](int r, int c, double v) {
        Lq[qidx(r, c)] = v;
        Lq[qidx(r, 16 + c)] = 0.0;
        lin11[r >> 2] = v;
    });
#endif
}
// part B: from D21^T (quadrant (1, 0) registers) and D22: L21 = D21 Linv11^T (returned as L21^T in
// the C layout), D22 -= L21 L21^T, Linv22 into quadrant 3, Linv21 = -Linv22 L21 Linv11 into
// quadrant 2
__device__ __forceinline__ bool diag_part_b(const double4_t& d21t, double4_t d22, const double4_t& lin11, double* Lq,
                                            double4_t& l21t, double* scr) {
    const int lane = threadIdx.x & 63, cc = lane & 15, rg = lane >> 4;
    const double* a11 = Lq + lane * 4;   // quadrant 0 in operand order
    l21t = double4_t{0, 0, 0, 0};
    panel_add(l21t, double4_t{a11[0], a11[1], a11[2], a11[3]}, d21t);
    mfma_sub(d22, l21t, l21t);
    double* op22 = Lq + 3 * 256;
#if ORBHIP_DAG_DIAG_DPP
    double4_t l22;
    double v[16];
    c_to_cols(d22, scr, v);
    const bool ok2 = diag16_dpp<kNewton>(v, scr, l22);
#pragma unroll
    for (int q = 0; q < 4; q++) op22[(rg + 4 * q + 16 * (cc & 3)) * 4 + (cc >> 2)] = l22[q];
#else
    (void)scr;
    const bool ok2 = diag16_linv<kNewton>(d22, [&](int r, int c, double v) { op22[(r + 16 * (c & 3)) * 4 + (c >> 2)] = v; });
#endif
    double4_t w = {0, 0, 0, 0};
    panel_add(w, l21t, lin11);
    wave_lds_sync();
    const double* a22 = op22 + lane * 4;
    double4_t l21i = {0, 0, 0, 0};
    mfma_sub(l21i, double4_t{a22[0], a22[1], a22[2], a22[3]}, w);
#pragma unroll
    for (int q = 0; q < 4; q++) Lq[qidx(16 + rg + 4 * q, cc)] = l21i[q];
    return ok2;
}
// y[i] = sum_c Li[i][c] r[c] over one 16x16 quadrant of Lq (rows and columns from 0); every lane
// returns the value of row lane & 15
__device__ __forceinline__ double quad_matvec(const double* Lq, int qd, const double* r) {
    const int lane = threadIdx.x & 63, i = lane & 15, g = lane >> 4;
    double s = 0.0;
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const int c = 4 * g + j;   // element (i, c) of the quadrant: lane i + 16 (c & 3), component c >> 2
        s = fma(Lq[qd * 256 + (i + 16 * (c & 3)) * 4 + (c >> 2)], r[c], s);
    }
    return col4_sum(s);
}
__device__ __forceinline__ void lds_signal(int* w, int v) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __hip_atomic_store(w, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_wait(int* w, int v) {
    while (__hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < v) __builtin_amdgcn_s_sleep(1);
    asm volatile("" ::: "memory");
}

// DBG: the debug build of the chain (the probe's per-interval cycle words); the product build
// carries no stamp code (the debug values would otherwise stay live through the whole loop)
template <bool DBG>
__device__ void dag_chain(const DagK& a, const Lay& L, __amdgpu_buffer_rsrc_t rs, int epoch, double* lds) {
    const int tid = threadIdx.x, wid = tid >> 6, lane = tid & 63, cc = lane & 15, rg = lane >> 4;
    const int rq = wid >> 1, cq = wid & 1, quad = 2 * rq + cq;
    const int NT = a.NT, n = a.n;
    // LDS (doubles), double buffers by base arithmetic (an array of LDS pointers selected at run
    // time loses the address space: flat accesses, which wait on vmcnt too):
    //   [0, 2048)      Linv_k by parity p = k & 1
    //   [2048, 4096)   L1: L(k, k-1) / the new L(k+1, k)        (c1)
    //   [4096, 6144)   L2: L(k+1, k-1) / the new L(k+2, k)      (c2)
    //   [6144, 8192)   Tp: T_k, tile (k+1, k) with every column < k applied (parity)
    //   [8192, 10240)  Dp: D'_{k+1} (quadrants 0, 3: columns <= k-1 applied; 2: <= k-2) (parity)
    //   [10240, 11264) Dq: D(1,0), D(1,1) of tile k+1, wave 1 -> wave 0 (quadrants 2, 3); its first
    //                  half: wave 0's transposition scratch [10240, 10528), debug stamps [10560, 10576)
    int* word = (int*)(lds + 11264);    // [4] abort, [5] row polls ok, [8] ok, [10..12] wave flags
    double* rvec = lds + 11280;         // 32: r0 (wave 0), r1 (wave 1 -> wave 0)
    double* rppB = rvec + 32;           // 2 x 32: rhs of D' (parity)
    double* ys = rppB + 64;             // NT x 32: y_k; in the backward the running sums s_k
    double* xs = ys + NT * kT;          // NT x 32
    int* rfl = (int*)(xs + NT * kT);    // row_first (NT ints)
    int* F1 = word + 10;                // wave 0: row 0 of L(k+1, k) ready (k + 2)
    int* F2 = word + 11;                // wave 1: D(1,0), D(1,1), r1 of tile k+1 ready
    int* F3 = word + 12;                // wave 1: row 1 of L(k+1, k) ready
    int* F4 = word + 13;                // wave 2 / 3: their rows of T_{k+1} up to column k-1 in TpN
    int* F5 = word + 14;
    unsigned long long* wts = (unsigned long long*)(lds + 11264 + 8);   // per-wave cycles (dbg)
    unsigned long long* stm = (unsigned long long*)(lds + 10560);       // sub-phase stamps (dbg), 16
#define DAG_STAMP(i) do { if (dbg && lane == 0) stm[i] = __builtin_amdgcn_s_memtime() - tk; } while (0)
    unsigned long long* dbg = DBG ? a.dbg : nullptr;
    const unsigned long long t_start = dbg ? __builtin_amdgcn_s_memtime() : 0;
    unsigned long long t_fact = 0;
    bool ok = true, aborted = false;
    if (tid == 0) {
        word[4] = 0;
        word[5] = 1;
        word[18] = NT < 3 ? 1 : 0;   // the backward's column copies ready (no copy task below NT = 3)
        *F1 = 0;
        *F2 = 0;
        *F3 = 0;
        *F4 = 0;
        *F5 = 0;
    }
    for (int i = tid; i < NT; i += blockDim.x) rfl[i] = a.rf[i];
    // the chain backward's per-column counts (dag_plan: rows R >= k + 2 whose envelope reaches
    // column k), after the helpers' task list
    int* need = rfl + NT;
    if (!a.pb && !a.nti)
        for (int i = tid; i < NT; i += blockDim.x) need[i] = a.tasks[a.need_off + i];   // (r06: not behind a load of toff[G])
    int c1 = 0, c2 = 0;
    // ---- prologue: wave 0 factors tile 0; T_0 = A(1, 0), D'_1 = A(1, 1), L1 = L2 = 0 ----
    // every prologue load in one round trip: wave 0's tile-0 quadrants with the others, and tile
    // (1, 0) loaded whatever row_first says (a load chosen by a.rf[1] waited for that load first:
    // r06, ~5.3k cycles to the prologue's barrier at n = 294)
    double4_t q00 = {0, 0, 0, 0}, q10 = {0, 0, 0, 0}, q11 = {0, 0, 0, 0};
    if (wid == 0) {
        q00 = s_quad(a, 0, 0, 0, 0);
        q10 = s_quad(a, 0, 0, 1, 0);
        q11 = s_quad(a, 0, 0, 1, 1);
    }
    sq(lds + 2048 + quad * 256, double4_t{0, 0, 0, 0});
    sq(lds + 4096 + quad * 256, double4_t{0, 0, 0, 0});
    if (NT > 1) {
        const double4_t t10 = s_quad(a, 1, 0, rq, cq), t11 = s_quad(a, 1, 1, rq, cq);
        sq(lds + 6144 + quad * 256, a.rf[1] <= 0 ? t10 : double4_t{0, 0, 0, 0});
        sq(lds + 8192 + quad * 256, t11);
        if (cq == 0 && rg == 0) {
            const int i = kT + 16 * rq + cc;
            rppB[16 * rq + cc] = s_rhs(a, i);
        }
    }
    if (tid < kT) rvec[tid] = s_rhs(a, tid);
    __syncthreads();
    if (dbg && tid == 0) dbg[6] = __builtin_amdgcn_s_memtime() - t_start;
    // a partial solve (nti > 0) runs intervals 0 .. nti-1: the last one forms the trailing block's
    // first tiles of L (rows of L(nti, nti-1) and L(nti+1, nti-1)) but factors no diagonal tile
    const int kEnd = a.nti ? a.nti : NT - 1;
    // waves 2/3: the helpers' flag this lane waits for in interval kk (nullptr: none), i.e. the
    // partials P2[kk], P1[kk+1], P0[kk+2] and the full tile L(kk+2, kk-1) the flags of that interval
    // (fl) select
    auto helper_flag = [&](int kk) -> const int* {
        const int kk1 = kk + 1, kk2 = kk + 2;
        if (kk2 >= NT || lane > 3) return nullptr;
        const bool zT = a.nti && kk1 >= a.nti, zD = a.nti && kk2 >= a.nti;
        const int ra = rfl[kk1], rb = rfl[kk], rc = rfl[kk2];
        if (lane == 0) return max(rc, rb) <= kk - 2 ? L.fP2 + kk : nullptr;
        if (lane == 1) {
            const bool uU = kk - 1 >= max(rc, rb), uT = !zT && kk - 1 >= max(rc, ra), uC = !zD && kk - 1 >= rc;
            return (uU || uT || uC) ? L.fL + kk2 * NT + kk - 1 : nullptr;
        }
        if (lane == 2) return (!zT && max(rc, ra) <= kk - 2) ? L.fP1 + kk1 : nullptr;
        return (!zD && rc <= kk2 - 4) ? L.fP0 + kk2 : nullptr;
    };
    // every per-interval flag of interval k packed in one word (fl), every LDS buffer pointer
    // derived from one parity word (par) where it is used: held across the role branches as separate
    // values they exceeded the SGPR budget and were spilled / reloaded by readlanes
    auto flags_of = [&](int k) -> unsigned {
        const int k1 = k + 1, K2 = k + 2;
        const bool last = a.nti && k1 >= a.nti;   // tile k+1 is in the trailing block: not factored
        const bool zT = last, zD = a.nti && K2 >= a.nti;   // T_{k+1} / D'_{k+2}: trailing-block tiles
        const int rfa = rfl[k1], rfb = rfl[k];
        const bool inEnv1 = rfa <= k;
        const bool useD2 = k - 1 >= rfa;
        const int rfc = K2 < NT ? rfl[K2] : 0;
        const bool inEnvU = K2 < NT && rfc <= k, inEnvT = K2 < NT && rfc <= k1;
        const bool needP2 = K2 < NT && max(rfc, rfb) <= k - 2, useU = K2 < NT && k - 1 >= max(rfc, rfb);
        const bool needP1 = !zT && K2 < NT && max(rfc, rfa) <= k - 2;
        const bool useTp = !zT && K2 < NT && k - 1 >= max(rfc, rfa);
        const bool useTk = !zT && inEnvU && inEnv1;   // T_{k+1} -= L(k+2, k) L(k+1, k)^T
        const bool needP0 = !zD && K2 < NT && rfc <= K2 - 4;   // the helpers' diagonal partial: columns <= k-2
        const bool useP0c = !zD && K2 < NT && k - 1 >= rfc;     // column k-1 of D'_{k+2}: applied here
        return (unsigned)last | (unsigned)inEnv1 << 1 | (unsigned)useD2 << 2 | (unsigned)inEnvU << 3 |
               (unsigned)inEnvT << 4 | (unsigned)needP2 << 5 | (unsigned)useU << 6 | (unsigned)needP1 << 7 |
               (unsigned)useTp << 8 | (unsigned)useTk << 9 | (unsigned)needP0 << 10 | (unsigned)useP0c << 11;
    };
    // waves 2/3: the global inputs of interval kk (the helpers' partial tiles / S, the full tile
    // L(kk+2, kk-1), the rhs partial) into the p* registers, issued once the interval's helper flags
    // are in. (r06: issuing them at the end of interval kk-1 whenever its flags were already in,
    // behind an early poll, took the n = 294 interval 12.5k -> 15.6k cycles on one box, two alternating
    // runs each: reverted)
    double4_t pd0 = {0, 0, 0, 0}, pd1 = {0, 0, 0, 0}, pe0 = {0, 0, 0, 0}, pe1 = {0, 0, 0, 0};
    double4_t pu[2] = {}, pt[2] = {}, pdd[2] = {};
    double prr = 0.0;
    // part: 1 the inputs read from S itself (no helper flag), 2 the helpers' tiles, 3 both. r06: the
    // S part of interval kk goes out in interval kk-1 (the first touch of S costs ~5-7k cycles: the
    // first two intervals took 17.8k / 19.7k cycles against ~12.6k at n = 294); its loads are old
    // by the next interval's flag poll, which waits for them in the in-order vmcnt queue
    auto fetch_in = [&](int kk, unsigned flk, int part) {
        const int h = wid - 2, kk1 = kk + 1, KK2 = kk + 2;
        auto F = [&](int b) { return ((flk >> b) & 1u) != 0u; };
        const bool ps = part & 1, ph = part & 2;
        if (ph) {
            const int tD = L.oL + (KK2 * NT + kk - 1) * kTD;
            pd0 = pd1 = pe0 = pe1 = double4_t{0, 0, 0, 0};
            if (F(6) || F(8) || F(11)) {   // useU || useTp || useP0c
                pd0 = qload(rs, tD + (2 * h) * 256);
                pd1 = qload(rs, tD + (2 * h + 1) * 256);
            }
            // quadrant (1, 0) of D'_{kk+2} needs both row halves of L(kk+2, kk-1): wave 3, which forms
            // that term, loads the other half
            if (F(11) && h == 1) {
                pe0 = qload(rs, tD);
                pe1 = qload(rs, tD + 256);
            }
        }
#pragma unroll
        for (int c = 0; c < 2; c++) {
            if (!F(3)) {
                if (ps) pu[c] = double4_t{0, 0, 0, 0};
            } else if (F(5)) {
                if (ph) pu[c] = qload(rs, L.oP + (2 * NT + kk) * kTD + (2 * h + c) * 256);
            } else if (ps) {
                pu[c] = s_quad(a, KK2, kk, h, c);
            }
            if (!F(4)) {
                if (ps) pt[c] = double4_t{0, 0, 0, 0};
            } else if (F(7)) {
                if (ph) pt[c] = qload(rs, L.oP + (NT + kk1) * kTD + (2 * h + c) * 256);
            } else if (ps) {
                pt[c] = s_quad(a, KK2, kk1, h, c);
            }
            const int qd = 2 * h + c;   // D' quadrants: wave 2 q0, wave 3 q2 and q3
            if (h == 0 && c == 1) {
                if (ps) pdd[c] = double4_t{0, 0, 0, 0};
            } else if (F(10)) {
                if (ph) pdd[c] = qload(rs, L.oP + KK2 * kTD + qd * 256);
            } else if (ps) {
                pdd[c] = s_quad(a, KK2, KK2, qd >> 1, qd & 1);
            }
        }
        if (F(10)) {
            if (ph) prr = ld_sc1(a.buf + L.oR + KK2 * kT + 16 * h + cc);
        } else if (ps) {
            prr = s_rhs(a, kT * KK2 + 16 * h + cc);
        }
    };
    // interval 0's inputs (all from S: no helper tile exists yet) go out now, under the prologue's
    // factorization of tile 0
    if (wid >= 2 && kEnd > 0 && 2 < NT) fetch_in(0, flags_of(0), 3);
    if (wid == 0) {
        double4_t lin11, l21t;
        ok = diag_part_a(q00, lds, lin11, lds + 10240);
        if (dbg && lane == 0) dbg[7] = __builtin_amdgcn_s_memtime() - t_start;
        wave_lds_sync();
        const double y0 = quad_matvec(lds, 0, rvec);
        if (rg == 0) ys[cc] = y0;
        ok = diag_part_b(q10, q11, lin11, lds, l21t, lds + 10240) && ok;
        wave_lds_sync();
        const double r1 = rvec[16 + cc] - lmul_ylds(l21t, ys);
        wave_lds_sync();
        if (rg == 0) rvec[16 + cc] = r1;
        wave_lds_sync();
        const double y1 = quad_matvec(lds, 3, rvec + 16);
        if (rg == 0) ys[16 + cc] = y1;
    }
    __syncthreads();
    if (dbg && tid == 0) dbg[0] = __builtin_amdgcn_s_memtime() - t_start;
    // ---- interval k: wave 0 the critical path (row 0 of L(k+1, k), D(0,0), its pivot, then D22's
    // after wave 1's row 1 / D(1,*)); wave 1 row 1 and the publishes; waves 2 / 3 row h of
    // L(k+2, k), of T_{k+1} and of D'_{k+2} ----
    for (int k = 0; k < kEnd; k++) {
        const unsigned long long tk = dbg ? __builtin_amdgcn_s_memtime() : 0;
        const int k1 = k + 1, K2 = k + 2;
        // every per-interval flag packed in one word (fl), every LDS buffer pointer derived from
        // one parity word (par) where it is used: held across the role branches as separate
        // values they exceeded the SGPR budget and were spilled / reloaded by readlanes
        const unsigned fl = flags_of(k);
#define DAG_FL(b) (((fl >> (b)) & 1u) != 0u)
#define last DAG_FL(0)
#define inEnv1 DAG_FL(1)
#define useD2 DAG_FL(2)
#define inEnvU DAG_FL(3)
#define inEnvT DAG_FL(4)
#define needP2 DAG_FL(5)
#define useU DAG_FL(6)
#define needP1 DAG_FL(7)
#define useTp DAG_FL(8)
#define useTk DAG_FL(9)
#define needP0 DAG_FL(10)
#define useP0c DAG_FL(11)
        const int par = (k & 1) | c1 << 1 | c2 << 2;
#define cur (par & 1)
#define nxt ((par & 1) ^ 1)
#define Lin (lds + 1024 * cur)
#define LinN (lds + 1024 * nxt)
#define L1 (lds + 2048 + 1024 * ((par >> 1) & 1))
#define L1n (lds + 2048 + 1024 * (((par >> 1) & 1) ^ 1))
#define L2 (lds + 4096 + 1024 * ((par >> 2) & 1))
#define L2n (lds + 4096 + 1024 * (((par >> 2) & 1) ^ 1))
#define Tp (lds + 6144 + 1024 * cur)
#define TpN (lds + 6144 + 1024 * nxt)
#define Dp (lds + 8192 + 1024 * cur)
#define DpN (lds + 8192 + 1024 * nxt)
#define rp (rppB + 32 * cur)
#define rpN (rppB + 32 * nxt)
        double* Dq = lds + 10240;
        const int* f3 = wid >= 2 ? helper_flag(k) : nullptr;
        const bool need3 = f3 != nullptr;
        const int fv = wid >= 2 ? ld_flag(need3 ? f3 : L.ctl) : epoch;
        if (wid == 0) {
            if (dbg && lane == 0) wts[6] = __builtin_amdgcn_s_memtime() - tk;
            // row 0 of L(k+1, k) = T Linv_k^T
            double4_t l0 = {0, 0, 0, 0}, l1 = {0, 0, 0, 0};
            if (inEnv1) {
                const double4_t t0 = lq(Tp), t1 = lq(Tp + 256);
                double4_t l1b = {0, 0, 0, 0};
                panel_add(l0, lq(Lin), t0);
                panel_add(l1, lq(Lin + 2 * 256), t0);
                panel_add(l1b, lq(Lin + 3 * 256), t1);
                l1 += l1b;
            }
            sq(L1n, l0);
            sq(L1n + 256, l1);
            lds_signal(F1, k + 2);
            if (!last) {
            // D(0,0) and r0 of tile k+1
            double4_t D = lq(Dp);
            double r0 = rp[cc];
            if (inEnv1) {
                double4_t Db = {0, 0, 0, 0};
                mfma_sub(D, l0, l0);
                mfma_sub(Db, l1, l1);
                D += Db;
                r0 -= col4_sum(lmul_part(l0, ys + k * kT) + lmul_part(l1, ys + k * kT + 16));
            }
            if (rg == 0) rvec[cc] = r0;
            const unsigned long long tf = dbg ? __builtin_amdgcn_s_memtime() : 0;
            if (dbg && lane == 0) wts[7] = tf - tk;
            double4_t lin11, l21t;
            ok = diag_part_a(D, LinN, lin11, Dq) && ok;
            DAG_STAMP(0);
            wave_lds_sync();
            const double y0 = quad_matvec(LinN, 0, rvec);
            if (rg == 0) ys[k1 * kT + cc] = y0;
            const unsigned long long tw0 = dbg ? __builtin_amdgcn_s_memtime() : 0;
            lds_wait(F2, k + 2);
            if (dbg && lane == 0) wts[5] = __builtin_amdgcn_s_memtime() - tw0;
            DAG_STAMP(1);
            ok = diag_part_b(lq(Dq + 2 * 256), lq(Dq + 3 * 256), lin11, LinN, l21t, Dq) && ok;
            DAG_STAMP(2);
            wave_lds_sync();
            const double r1 = rvec[16 + cc] - lmul_ylds(l21t, ys + k1 * kT);
            wave_lds_sync();
            if (rg == 0) rvec[16 + cc] = r1;
            wave_lds_sync();
            const double y1 = quad_matvec(LinN, 3, rvec + 16);
            if (rg == 0) ys[k1 * kT + 16 + cc] = y1;
            DAG_STAMP(3);
            if (dbg) t_fact += __builtin_amdgcn_s_memtime() - tf;
            }   // !last
        } else if (wid == 1) {
            // row 1 of L(k+1, k)
            double4_t l0 = {0, 0, 0, 0}, l1 = {0, 0, 0, 0};
            if (inEnv1) {
                const double4_t t0 = lq(Tp + 2 * 256), t1 = lq(Tp + 3 * 256);
                double4_t l1b = {0, 0, 0, 0};
                panel_add(l0, lq(Lin), t0);
                panel_add(l1, lq(Lin + 2 * 256), t0);
                panel_add(l1b, lq(Lin + 3 * 256), t1);
                l1 += l1b;
            }
            sq(L1n + 2 * 256, l0);
            sq(L1n + 3 * 256, l1);
            lds_signal(F3, k + 2);
            // D(1,0), D(1,1), r1 of tile k+1
            double4_t D10 = lq(Dp + 2 * 256), D11 = lq(Dp + 3 * 256);
            double r1 = rp[16 + cc];
            lds_wait(F1, k + 2);
            if (useD2) {   // the column k-1 term of D(1,0) (the other quadrants had theirs applied)
                double4_t Db = {0, 0, 0, 0};
                mfma_sub(D10, lq(L2), lq(L2 + 2 * 256));
                mfma_sub(Db, lq(L2 + 256), lq(L2 + 3 * 256));
                D10 += Db;
            }
            if (inEnv1) {
                double4_t Db = {0, 0, 0, 0}, Dc = {0, 0, 0, 0};
                mfma_sub(D10, lq(L1n), l0);
                mfma_sub(Db, lq(L1n + 256), l1);
                mfma_sub(D11, l0, l0);
                mfma_sub(Dc, l1, l1);
                D10 += Db;
                D11 += Dc;
                r1 -= col4_sum(lmul_part(l0, ys + k * kT) + lmul_part(l1, ys + k * kT + 16));
            }
            sq(Dq + 2 * 256, D10);
            sq(Dq + 3 * 256, D11);
            if (rg == 0) rvec[16 + cc] = r1;
            lds_signal(F2, k + 2);
            // publish L(k+1, k), L(k+1, k-1), Linv_k, y_k
#pragma unroll
            for (int qd = 0; qd < 4; qd++) qstore(rs, L.oL + (k1 * NT + k) * kTD + qd * 256, lq(L1n + qd * 256));
            if (k >= 1) {
#pragma unroll
                for (int qd = 0; qd < 4; qd++) qstore(rs, L.oL + (k1 * NT + k - 1) * kTD + qd * 256, lq(L2 + qd * 256));
            }
#pragma unroll
            for (int qd = 0; qd < 4; qd++) qstore(rs, L.oLi + k * kTD + qd * 256, lq(Lin + qd * 256));
            if (lane < kT) st_sc1(a.buf + L.oY + k * kT + lane, ys[k * kT + lane]);
            drain_stores();
            if (lane == 0) {
                st_flag(L.fCh + k, epoch);
                st_flag(L.fL + k1 * NT + k, epoch);
                if (k >= 1) st_flag(L.fL + k1 * NT + k - 1, epoch);
            }
#if ORBHIP_DAG_T_W1
            // T_{k+1} -= L(k+2, k) L(k+1, k)^T for both row halves of waves 2 / 3 (their partials
            // in TpN, their rows of L(k+2, k) in L2n): off their critical path, the same MFMAs
            // in the same order as theirs
            if (K2 < NT && useTk) {
                lds_wait(F4, k + 2);
                lds_wait(F5, k + 2);
                if (!word[4]) {
#pragma unroll
                    for (int h = 0; h < 2; h++) {
                        const double4_t o0 = lq(L2n + (2 * h) * 256), o1 = lq(L2n + (2 * h + 1) * 256);
#pragma unroll
                        for (int c = 0; c < 2; c++) {
                            double4_t tc = lq(TpN + (2 * h + c) * 256), tb = {0, 0, 0, 0};
                            mfma_sub(tc, lq(L1n + (2 * c) * 256), o0);
                            mfma_sub(tb, lq(L1n + (2 * c + 1) * 256), o1);
                            sq(TpN + (2 * h + c) * 256, tc + tb);
                        }
                    }
                }
            }
#endif
        } else if (K2 < NT) {
            // row h of L(k+2, k) = U Linv_k^T, U = A(k+2, k) - sum_{p <= k-1} L(k+2,p) L(k,p)^T (the
            // helpers' partial: p <= k-2; here p = k-1); row h of T_{k+1} = A(k+2, k+1) - sum_{p <= k}
            // L(k+2,p) L(k+1,p)^T (partial p <= k-2; p = k-1 and p = k here); D'_{k+2} (partial
            // p <= k-2; p = k-1 and k here, quadrant (1,0)'s column k by wave 1 in the next interval)
            // and its rhs
            const int h = wid - 2;
            const bool got = __all(!need3 || fv == epoch) || wave_wait_all(f3, epoch, L.ctl, a.smax);
            if (dbg && lane == 0 && h == 1) wts[4] = __builtin_amdgcn_s_memtime() - tk;   // helpers' flags in
            if (got) fetch_in(k, fl, 2);   // (the S part went out in the interval before / the prologue)
            if (dbg) {   // the loads in (diagnostics only)
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                DAG_STAMP(4 + 4 * h);
            }
            if (!got) {
                if (lane == 0) word[4] = 1;
                if (ORBHIP_DAG_T_W1) lds_signal(h ? F5 : F4, k + 2);
            } else {
                const double4_t d0 = pd0, d1 = pd1, e0 = pe0, e1 = pe1;
                double4_t u[2] = {pu[0], pu[1]}, t[2] = {pt[0], pt[1]}, dd[2] = {pdd[0], pdd[1]};
                double rr = prr;
                if (k + 1 < kEnd && k + 3 < NT) fetch_in(k + 1, flags_of(k + 1), 1);   // the next interval's S part
                // every LDS operand of this wave's MFMA work first (one LDS round trip), the MFMA
                // chains two deep per product, the rhs terms (LDS + cross-row sums) after the tiles
                const double4_t l1q[4] = {lq(L1), lq(L1 + 256), lq(L1 + 512), lq(L1 + 768)};
                const double4_t liq[3] = {lq(Lin), lq(Lin + 512), lq(Lin + 768)};
                const double4_t l2q[4] = {lq(L2), lq(L2 + 256), lq(L2 + 512), lq(L2 + 768)};
                double4_t o0 = {0, 0, 0, 0}, o1 = {0, 0, 0, 0};
                // D' column k-1 terms (da, db; dc, de: quadrant (1, 0), wave 3)
                double4_t da = {0, 0, 0, 0}, db = {0, 0, 0, 0}, dc = {0, 0, 0, 0}, de = {0, 0, 0, 0};
                // (U's, T's and D''s column k-1 chains in one basic block measured slower, r05: L(k+2, k)
                // is published first, wave 1 waits on it)
                if (inEnvU) {
                    if (useU) {
#pragma unroll
                        for (int c = 0; c < 2; c++) {
                            double4_t ub = {0, 0, 0, 0};
                            mfma_sub(u[c], l1q[2 * c], d0);
                            mfma_sub(ub, l1q[2 * c + 1], d1);
                            u[c] += ub;
                        }
                    }
                    double4_t o1b = {0, 0, 0, 0};
                    panel_add(o0, liq[0], u[0]);
                    panel_add(o1, liq[1], u[0]);
                    panel_add(o1b, liq[2], u[1]);
                    o1 += o1b;
                }
                sq(L2n + (2 * h) * 256, o0);
                sq(L2n + (2 * h + 1) * 256, o1);
                DAG_STAMP(5 + 4 * h);
                if (inEnvT && useTp) {
#pragma unroll
                    for (int c = 0; c < 2; c++) {
                        double4_t tb = {0, 0, 0, 0};
                        mfma_sub(t[c], l2q[2 * c], d0);
                        mfma_sub(tb, l2q[2 * c + 1], d1);
                        t[c] += tb;
                    }
                }
#if ORBHIP_DAG_T_W1
                sq(TpN + (2 * h) * 256, t[0]);
                sq(TpN + (2 * h + 1) * 256, t[1]);
                lds_signal(h ? F5 : F4, k + 2);
#endif
                DAG_STAMP(12 + 2 * h);
                {   // D'_{k+2}: column k-1 (L(k+2, k-1)) and column k (L(k+2, k)) in independent chains
                    if (useP0c) {
                        mfma_sub(da, d0, d0);
                        mfma_sub(db, d1, d1);
                        if (h == 1) {   // quadrant (1, 0): row half 1 against row half 0
                            mfma_sub(dc, e0, d0);
                            mfma_sub(de, e1, d1);
                        }
                    }
                    double4_t dg = {0, 0, 0, 0}, dh = {0, 0, 0, 0};
                    if (inEnvU) {
                        mfma_sub(dg, o0, o0);
                        mfma_sub(dh, o1, o1);
                    }
                    const double4_t dsum = (da + db) + (dg + dh);
                    if (h == 0) {   // constant indices only (a runtime index put dd in scratch)
                        dd[0] += dsum;
                    } else {
                        dd[1] += dsum;
                        dd[0] += dc + de;
                    }
                }
                if (h == 0) {
                    sq(DpN, dd[0]);
                } else {
                    sq(DpN + 2 * 256, dd[0]);
                    sq(DpN + 3 * 256, dd[1]);
                }
                DAG_STAMP(13 + 2 * h);
                {   // the rhs terms of columns k-1 and k, one cross-row sum
                    double part = 0.0;
                    if (useP0c) part += lmul_part(d0, ys + (k - 1) * kT) + lmul_part(d1, ys + (k - 1) * kT + 16);
                    if (inEnvU) part += lmul_part(o0, ys + k * kT) + lmul_part(o1, ys + k * kT + 16);
                    rr -= col4_sum(part);
                }
                if (rg == 0) rpN[16 * h + cc] = rr;
                DAG_STAMP(6 + 4 * h);
#if ORBHIP_DAG_T_W1
                DAG_STAMP(7 + 4 * h);
#else
                // the column k term of T_{k+1} needs both rows of L(k+1, k)
                lds_wait(F1, k + 2);
                lds_wait(F3, k + 2);
                DAG_STAMP(7 + 4 * h);
                if (useTk) {
#pragma unroll
                    for (int c = 0; c < 2; c++) {
                        double4_t tb = {0, 0, 0, 0};
                        mfma_sub(t[c], lq(L1n + (2 * c) * 256), o0);
                        mfma_sub(tb, lq(L1n + (2 * c + 1) * 256), o1);
                        t[c] += tb;
                    }
                }
                sq(TpN + (2 * h) * 256, t[0]);
                sq(TpN + (2 * h + 1) * 256, t[1]);
#endif
            }
        } else if (wid == 2 && k == kEnd - 1 && !a.pb && !a.nti && NT >= 3) {
            // the last interval, idle otherwise: every copy task's flag (intervals <= NT - 3) for
            // the backward (the last one was published one interval ago)
            bool got = true;
            for (int k0 = 0; k0 <= NT - 3 && got; k0 += 64)
                got = wave_wait_all(k0 + lane <= NT - 3 ? L.fCp + k0 + lane : nullptr, epoch, L.ctl, a.smax);
            if (lane == 0) {
                if (got) lds_signal(word + 18, 1);
                else word[4] = 1;
            }
        }
        if (dbg && lane == 0) wts[wid] = __builtin_amdgcn_s_memtime() - tk;
        lds_barrier();
#undef DAG_FL
#undef last
#undef inEnv1
#undef useD2
#undef inEnvU
#undef inEnvT
#undef needP2
#undef useU
#undef needP1
#undef useTp
#undef useTk
#undef needP0
#undef useP0c
#undef cur
#undef nxt
#undef Lin
#undef LinN
#undef L1
#undef L1n
#undef L2
#undef L2n
#undef Tp
#undef TpN
#undef Dp
#undef DpN
#undef rp
#undef rpN
        c1 ^= 1;
        c2 ^= 1;
        if (dbg && tid == 0 && k < 200) {
            unsigned long long* dk = dbg + 8 + 6 * k;
            dk[0] = __builtin_amdgcn_s_memtime() - tk;
            for (int w = 0; w < 4; w++) dk[1 + w] = wts[w];
            dk[2] |= wts[4] << 32;   // wave 3: the helpers' flags arrived
            dk[5] = wts[6] | (wts[7] << 32);
            if (k < kDbgSubK) {
                unsigned long long* ds = dbg + kDbgSubOff + 16 * k;
                for (int i = 0; i < 16; i++) ds[i] = stm[i];
            }
        }
        if (word[4]) {
            aborted = true;
            break;
        }
    }
    if (a.nti) {   // partial solve: L(nti+1, nti-1) (formed by waves 2/3 in the last interval), then done
        const int R = a.nti + 1, C = a.nti - 1;
        if (wid == 1 && R < NT && !aborted) {
            const double* L2c = lds + 4096 + 1024 * c2;
#pragma unroll
            for (int qd = 0; qd < 4; qd++) qstore(rs, L.oL + (R * NT + C) * kTD + qd * 256, lq(L2c + qd * 256));
            drain_stores();
            if (lane == 0) st_flag(L.fL + R * NT + C, epoch);
        }
        if (wid == 0 && lane == 0) word[8] = (ok && !aborted) ? 1 : 0;
        __syncthreads();
        if (tid == 0) a.flag[0] = word[8] != 0 ? 1 : 0;
        return;
    }
    const unsigned long long t_fwd = dbg ? __builtin_amdgcn_s_memtime() : 0;
    double* Lin = lds + 1024 * ((NT - 1) & 1);
    // ---- backward, right-looking by rows: at step R (x_R known) wave 0 forms x_{R-1} from the
    // sub-diagonal tile (R, R-1) and s_{R-1}; waves 1..3 subtract row R's other tiles from the
    // running sums s_j, j <= R-2. The helper tiles' flags are polled once, up front; the tiles
    // are loaded two steps ahead. ----
    auto apply_lt = [&](int k) {   // wave 0: xs_k = Linv^T rvec (Linv in Lin)
        const int c = lane >> 1, hh = lane & 1;
        double s = 0.0;
#pragma unroll
        for (int i = 0; i < 16; i++) s = fma(Lin[qidx(16 * hh + i, c)], rvec[16 * hh + i], s);
        s += dpp64<0xB1>(s);
        if (hh == 0) xs[k * kT + c] = s;
    };
    if (a.G > 0 && a.pb) {
        // with helpers: they accumulate s_j for j <= NT-3 (dag_helper_backward) from the x_R this
        // wave publishes; wave 0 alone walks the chain: x_{R-1} = Linv_{R-1}^T (s_{R-1} -
        // L(R, R-1)^T x_R), s_{R-1} from the helpers (fS) or, for R-1 = NT-2, y itself
        if (!aborted && wid == 0) {
            auto publish = [&](int k) {   // x_k to oX (sc1), then its flag
                wave_lds_sync();
                if (lane < kT) st_sc1(a.buf + L.oX + k * kT + lane, xs[k * kT + lane]);
                drain_stores();
                if (lane == 0) st_flag(L.fX + k, epoch);
            };
            if (lane < kT) rvec[lane] = ys[(NT - 1) * kT + lane];
            wave_lds_sync();
            apply_lt(NT - 1);
            publish(NT - 1);
            double4_t st[4], li[4];
            for (int R = NT - 1; R >= 1 && !aborted; R--) {
#pragma unroll
                for (int qd = 0; qd < 4; qd++) {
                    st[qd] = qload(rs, L.oL + (R * NT + R - 1) * kTD + qd * 256);
                    li[qd] = qload(rs, L.oLi + (R - 1) * kTD + qd * 256);
                }
                double sv = 0.0;
                if (R - 1 <= NT - 3) {
                    if (!wave_wait_all(lane == 0 ? L.fS + R - 1 : nullptr, epoch, L.ctl, a.smax)) {
                        aborted = true;
                        break;
                    }
                    if (lane < kT) sv = ld_sc1(a.buf + L.oS + (R - 1) * kT + lane);
                } else if (lane < kT) {
                    sv = ys[(R - 1) * kT + lane];
                }
                if (lane < kT) rvec[lane] = sv;
#pragma unroll
                for (int qd = 0; qd < 4; qd++) sq(Lin + qd * 256, li[qd]);
                wave_lds_sync();
                double t[2][4];
                tile_lt_x(st, xs + R * kT, t);
                if (cc == 0) {
#pragma unroll
                    for (int b = 0; b < 2; b++)
#pragma unroll
                        for (int q = 0; q < 4; q++) rvec[16 * b + rg + 4 * q] -= t[b][q];
                }
                wave_lds_sync();
                apply_lt(R - 1);
                if (R - 1 >= 2) publish(R - 1);
            }
            if (aborted && lane == 0) word[5] = 0;
        }
        __syncthreads();
        if (!word[5]) aborted = true;
    } else {   // short rows (or no helpers): the chain work-group alone
        // Right-looking, no barrier per step (r06). Wave 0 walks the chain: step t forms
        // x_{t-1} = Linv_{t-1}^T (s_{t-1} - L(t, t-1)^T x_t) (t = NT: Linv_{NT-1}^T s_{NT-1}) from
        // column-major copies (a lane's column: 16 contiguous doubles, a 16-FMA dot product and one
        // half-wave sum), its operands prefetched two steps ahead; the last two steps' operands are
        // still in this work-group's LDS. Waves 1..3 own the columns j = wid - 1 (mod 3) of every
        // row: as x_R appears (xcnt) they subtract L(R, j)^T x_R from s_j for j <= R - 2, tiles
        // streamed two ahead, and count each applied row (cnt[j]); step t waits until s_{t-1} has
        // every row R >= t + 1 of its envelope. LDS flags only (the forward's tile buffers are
        // free now): cnt at the T / D' buffers, xcnt / the abort word after the forward's flags.
        int* cnt = (int*)(lds + 6144);
        int* xcnt = word + 16;
        int* bab = word + 17;
        int* cpok = word + 18;   // every copy task's flag seen (wave 2, in the last interval)
        for (int i = tid; i < NT; i += blockDim.x) cnt[i] = 0;
        if (tid == 0) { *xcnt = 0; *bab = 0; }
        __syncthreads();
        const int c = lane & 31, hh = lane >> 5;
        // element (16 hh + i, c) of a quadrant-layout tile in LDS, i = 0..15
        auto lds_col = [&](const double* base, double (&v)[16]) {
#pragma unroll
            for (int i = 0; i < 16; i++) v[i] = base[qidx(16 * hh + i, c)];
        };
        // an LDS count reaching v; false on the abort word or after smax polls (then the solve fails:
        // the abort word and the problem's timeout count, as a global wait's timeout does)
        auto lwait = [&](const int* w, int v) -> bool {
            for (unsigned spins = 0; __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < v; spins++) {
                if (__hip_atomic_load(bab, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) return false;
                if (spins >= a.smax) {
                    if (lane == 0) {
                        st_flag(L.ctl + 2, epoch);
                        __hip_atomic_fetch_add((gint*)(L.ctl + 3), 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    }
                    return false;
                }
                __builtin_amdgcn_s_sleep(1);
            }
            asm volatile("" ::: "memory");
            return true;
        };
        if (!aborted && wid == 0) {
            bool good = true;
            double li[2][16], lt[2][16], liA[16], ltA[16];
            // operands of step t <= NT - 2 (copies). r06 (late): issued on every path, t < 1 (and
            // NT < 2) reading step 1's (an unused reload, in range of the buffer): with the loads
            // behind a branch, the waitcnt pass merged the paths that skip them and made each
            // step's dot wait for the loads issued just before it (vmcnt(7) .. vmcnt(0) after the
            // next step's 16 loads), so no step had its operands two steps ahead
            auto load = [&](auto setc, int t) {
                constexpr int S = decltype(setc)::value;
                const int tt = NT >= 2 ? max(t, 1) : 0;
                cmload(rs, L.oCI + max(tt - 1, 0) * kTD, li[S]);
                cmload(rs, L.oCM + (tt * NT + max(tt - 1, 0)) * kTD, lt[S]);
            };
            // x_{t-1} from the step's operands (lv: L(t, t-1) by columns, unused at t = NT; iv: Linv_{t-1})
            auto xstep = [&](const double (&lv)[16], const double (&iv)[16], int t) -> bool {
                const int k = t - 1;
                if (dbg && lane == 0 && t < kDbgBackR) dbg[kDbgBackOff + 3 * t] = __builtin_amdgcn_s_memtime() - t_fwd;
                double p = 0.0;
                if (t < NT) p = bwd_col_dot(lv, xs + t * kT);
                if (!lwait(cnt + k, need[k])) return false;
                if (dbg && lane == 0 && t < kDbgBackR) dbg[kDbgBackOff + 3 * t + 2] = __builtin_amdgcn_s_memtime() - t_fwd;
                const double r = ys[k * kT + c] - p;
                if (hh == 0) rvec[c] = r;
                wave_lds_sync();
                const double xv = bwd_col_dot(iv, rvec);
                if (hh == 0) xs[k * kT + c] = xv;
                lds_signal(xcnt, NT - k);
                if (dbg && lane == 0 && t < kDbgBackR) dbg[kDbgBackOff + 3 * t + 1] = __builtin_amdgcn_s_memtime() - t_fwd;
                return true;
            };
            {
                // the last two steps' operands are in LDS (Linv_{NT-1}; Linv_{NT-2} and L(NT-1, NT-2):
                // the last interval's buffers), the rest are copies (every copy task's flag was
                // polled by wave 2 in the last interval): their first two steps' loads go out first
                good = lwait(cpok, 1);
                // (every load below issues whatever `good` says: a failed wait fails the solve and
                // its loads go unused; the steps themselves are skipped)
                load(std::integral_constant<int, 0>{}, NT - 2);
                load(std::integral_constant<int, 1>{}, NT - 3);
                if (good) {
                    lds_col(lds + 1024 * ((NT - 1) & 1), liA);
                    good = xstep(ltA, liA, NT);
                }
                if (good && NT >= 2) {
                    lds_col(lds + 1024 * (NT & 1), liA);
                    lds_col(lds + 2048 + 1024 * ((NT - 1) & 1), ltA);
                    good = xstep(ltA, liA, NT - 1);
                }
                for (int t = NT - 2; t >= 1; t -= 2) {
                    if (good) good = xstep(lt[0], li[0], t);
                    load(std::integral_constant<int, 0>{}, t - 2);
                    if (good && t - 1 >= 1) good = xstep(lt[1], li[1], t - 1);
                    load(std::integral_constant<int, 1>{}, t - 3);
                }
            }
            if (!good && lane == 0) __hip_atomic_store(bab, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        } else if (!aborted) {
            const int own = wid - 1;
            // the largest j <= R - 2 of this wave's residue class
            auto jtop = [&](int R) { const int j = R - 2; return j - ((j - own) % 3 + 3) % 3; };
            // (R, j) moved to this wave's next tile in processing order: by urgency, i.e. columns
            // down (s_j is needed at step j + 1), rows down within a column (x_R appears in that
            // order); j < 0: none left. Tile (NT-1, NT-3) (the last interval's, no copy) is taken
            // first, from LDS
            auto norm = [&](int& R, int& j) {
                for (;;) {
                    if (j < 0) return;
                    if (R >= j + 2) {
                        if (!(R == NT - 1 && j == NT - 3) && rfl[R] <= j) return;
                        R--;
                        continue;
                    }
                    j -= 3;
                    R = NT - 1;
                }
            };
            // Flags: the full tiles (helpers, copies stored before the tile's flag) were consumed by
            // the forward, which is over; the special tile (NT-1, NT-3) is read from this
            // work-group's LDS; the copy tiles (R, R-2), R <= NT-2,
            // wait for wave 0's poll of the copy tasks' flags (cpok) before their loads are issued.
            bool good = true;
            if (NT >= 3 && (NT - 3) % 3 == own && rfl[NT - 1] <= NT - 3) {
                // L(NT-1, NT-3) is still in the last interval's L2 buffer (wave 1 published it from there)
                const double* L2last = lds + 4096 + 1024 * (NT & 1);
                const double4_t tl[4] = {lq(L2last), lq(L2last + 256), lq(L2last + 512), lq(L2last + 768)};
                good = lwait(xcnt, 1);
                if (good) {
                    double t[2][4];
                    tile_lt_x(tl, xs + (NT - 1) * kT, t);
                    if (cc == 0) {
#pragma unroll
                        for (int b = 0; b < 2; b++)
#pragma unroll
                            for (int q = 0; q < 4; q++) ys[(NT - 3) * kT + 16 * b + rg + 4 * q] -= t[b][q];
                    }
                    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                    if (lane == 0) __hip_atomic_store(cnt + NT - 3, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                }
            }
            if (good) {
                // a ring of kOwnAhead tiles in flight (a tile's load ~2k cycles, its product ~0.5k:
                // two in flight left the owners behind the chain on the C5 loop's corner rows)
                constexpr int kOwnAhead = 4;
                double v[kOwnAhead][16];
                int Rq[kOwnAhead], jq[kOwnAhead];
                int Rn = NT - 1, jn = jtop(NT - 1);   // the next tile to load
                norm(Rn, jn);
                bool cp = false;   // cpok seen
                // the next tile into ring slot S. r06 (late): its load issues on every path (an
                // exhausted ring, or a failed wait, reloads tile 0's copy, unused), so the waitcnt
                // pass counts the ring exactly: behind a branch, every slot's product waited for
                // the three loads fetched after it (vmcnt(7) .. vmcnt(0))
                auto fetch = [&](auto setc) {
                    constexpr int S = decltype(setc)::value;
                    Rq[S] = Rn;
                    jq[S] = jn;
                    const bool has = jn >= 0;
                    if (has && jn == Rn - 2 && !cp) cp = good = good && lwait(cpok, 1);
                    cmload(rs, L.oCM + (has && good ? Rn * NT + jn : 0) * kTD, v[S]);
                    if (has) {
                        Rn--;
                        norm(Rn, jn);
                    }
                };
                // a column's tiles come one after another: their products are summed in a register
                // and s_j is updated once, its count set to the column's total (need[j])
                double acc = 0.0;
                int jcur = -1, xseen = 0;
                auto flush = [&]() {
                    if (jcur < 0) return;
                    if (hh == 0) ys[jcur * kT + c] -= acc;
                    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                    if (lane == 0) __hip_atomic_store(cnt + jcur, need[jcur], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                };
                auto stepq = [&](auto setc) -> bool {   // L(R, j)^T x_R of slot S into acc, then refill the slot
                    constexpr int S = decltype(setc)::value;
                    const int R = Rq[S], j = jq[S];
                    if (j < 0 || !good) return false;
                    if (j != jcur) {
                        flush();
                        jcur = j;
                        acc = 0.0;
                    }
                    if (xseen < NT - R) {   // x_R not seen yet: wait for it (xcnt only grows)
                        if (!(good = lwait(xcnt, NT - R))) return false;
                        xseen = __hip_atomic_load(xcnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    }
                    acc += bwd_col_dot(v[S], xs + R * kT);
                    fetch(setc);
                    return true;
                };
                fetch(std::integral_constant<int, 0>{});
                fetch(std::integral_constant<int, 1>{});
                fetch(std::integral_constant<int, 2>{});
                fetch(std::integral_constant<int, 3>{});
                while (stepq(std::integral_constant<int, 0>{}) && stepq(std::integral_constant<int, 1>{}) &&
                       stepq(std::integral_constant<int, 2>{}) && stepq(std::integral_constant<int, 3>{})) {
                }
                if (good) flush();
            }
            if (!good && lane == 0) __hip_atomic_store(bab, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        __syncthreads();
        if (*bab) aborted = true;
    }
    if (wid == 0 && lane == 0) word[8] = (ok && !aborted) ? 1 : 0;
    __syncthreads();
    const bool good = word[8] != 0;
    for (int i = tid; i < n; i += blockDim.x) a.x[i] = good ? xs[i] : 0.0;
    if (tid == 0) a.flag[0] = good ? 1 : 0;
    if (dbg && tid == 0) {
        const unsigned long long te = __builtin_amdgcn_s_memtime();
        dbg[1] = t_fwd - t_start;
        dbg[2] = te - t_fwd;
        dbg[3] = 0;
        dbg[4] = t_fact;
        dbg[5] = te - t_start;
    }
}

// one problem's workgroup: role 0 the chain, role h + 1 helper h. ep: the epoch counter (read by
// the kernel together with the gate word: r06, one dependent round trip less at kernel start)
template <bool DBG>
__device__ __forceinline__ void dag_run(const DagK& a, int role, int ep) {
    extern __shared__ __attribute__((aligned(16))) double lds[];
    const Lay L(a);
    // epoch of this solve: the counter the last workgroup of the previous solve advanced
    const int epoch = ep + 1;
    const size_t bytes = dag_doubles_nt(a.NT) * 8;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(a.buf, 0, (int)bytes, 0x00020000);
    if (role == 0) dag_chain<DBG>(a, L, rs, epoch, lds);
    else dag_helper(a, L, rs, epoch, lds, role - 1);
    // the last workgroup of the problem out advances the epoch counter
    drain_stores();
    __syncthreads();
    if (threadIdx.x == 0) {
        const int old = __hip_atomic_fetch_add((gint*)(L.ctl + 1), 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (old == a.G) {
            st_flag(L.ctl + 1, 0);
            st_flag(L.ctl, epoch);
        }
    }
}

template <bool DBG>
__global__ __launch_bounds__(256) void k_chol_dag(DagK a) {
    // the epoch load goes out with the gate's (the previous solve of this workspace is over: stream
    // order; unused when the gate returns)
    const int ep = ld_flag(Lay(a).ctl);
    if (a.gate && *a.gate != kPhTrial) return;   // device-driven LM: not in a trial (uniform)
    dag_run<DBG>(a, blockIdx.x, ep);
}

// several independent problems in one launch (the interiors of a nested dissection): problem p
// owns workgroups [wg_off[p], wg_off[p + 1]); the whole grid is resident (one workgroup per CU)
__global__ __launch_bounds__(256) void k_chol_dag_multi(const DagK* __restrict__ ks, const int* __restrict__ wg_off,
                                                        int np) {
    int p = 0;
    while (p + 1 < np && (int)blockIdx.x >= wg_off[p + 1]) p++;
    const DagK a = ks[p];
    const int ep = ld_flag(Lay(a).ctl);
    if (a.gate && *a.gate != kPhTrial) return;
    dag_run<false>(a, blockIdx.x - wg_off[p], ep);
}

size_t dag_lds_bytes(int NT) {
    const size_t need = sizeof(double) * (11280 + 32 + 64 + 2 * (size_t)NT * kT + 256 + 1) + sizeof(int) * NT;
    return std::max(need, kMinLds);
}

// Per-device state of the persistent solver. Every k_chol_dag launch of a device, from any
// context / stream / host thread, goes through chol_dag_solve under its mutex:
//  - the grid size (CUs - 1 helpers + the chain) is the device's own (partitioned GPUs may differ);
//  - the LDS attribute is set once per device;
//  - launches are SERIALISED on the device: a launch on a stream other than the previous one first
//    waits (hipStreamWaitEvent) for an event recorded at the tail of that stream. Two solves whose
//    grids each assume the whole chip (LocalMapping's LBA and LoopClosing's GBA, on two contexts:
//    R:src/imu_mono_realsense.cpp:99-100 spawns both threads) then never hold parts of it at once,
//    which is the residency the no-deadlock argument rests on. One stream pays nothing.
struct DagDevState {
    std::mutex m;
    int helpers = -1;
    bool attr = false, attr_multi = false;
    bool has_last = false;          // `last` launched the device's most recent solve
    hipStream_t last = nullptr;
    hipEvent_t ev = nullptr;        // recorded at the tail of `last` when another stream launches
    // contended (a hand-off in the last kContendWindow launches): every launch records `after`
    // right behind itself, and the next launch from another stream waits on that instead of the
    // other stream's tail (which may hold a whole chunk of its queued LM slots). An event between
    // two slots costs ~5 us of queue drain (r04), so an uncontended solve records none.
    hipEvent_t after = nullptr;
    bool after_valid = false;       // `after` was recorded right behind `last`'s latest launch
    long long contended_until = 0;
    long long launches = 0, handoffs = 0;
};
constexpr long long kContendWindow = 64;
// the hand-off before a launch on st, and the bookkeeping after it (ds.m held)
hipError_t dag_handoff_before(DagDevState& ds, hipStream_t st) {
    if (!ds.has_last || ds.last == st) return hipSuccess;
    static const bool tail_only = std::getenv("ORBHIP_DAG_HANDOFF_TAIL") != nullptr;   // A/B: r04's form
    hipError_t e = hipSuccess;
    if (ds.after_valid && !tail_only) {
        e = hipStreamWaitEvent(st, ds.after, 0);
    } else {
        if (!ds.ev && (e = hipEventCreateWithFlags(&ds.ev, hipEventDisableTiming)) != hipSuccess) return e;
        e = hipEventRecord(ds.ev, ds.last);
        if (e == hipSuccess) e = hipStreamWaitEvent(st, ds.ev, 0);
    }
    if (e != hipSuccess) return e;
    ds.handoffs++;
    ds.contended_until = ds.launches + kContendWindow;
    return hipSuccess;
}
hipError_t dag_handoff_after(DagDevState& ds, hipStream_t st) {
    ds.has_last = true;
    ds.last = st;
    ds.launches++;
    ds.after_valid = false;
    if (ds.launches < ds.contended_until) {
        hipError_t e = hipSuccess;
        if (!ds.after && (e = hipEventCreateWithFlags(&ds.after, hipEventDisableTiming)) != hipSuccess) return e;
        if ((e = hipEventRecord(ds.after, st)) != hipSuccess) return e;
        ds.after_valid = true;
    }
    return hipSuccess;
}
constexpr int kMaxDagDevices = 64;
DagDevState& dag_dev(int dev) {
    static DagDevState s[kMaxDagDevices];
    return s[dev];
}
int dag_cur_dev() {
    int d = 0;
    if (hipGetDevice(&d) != hipSuccess || d < 0 || d >= kMaxDagDevices) d = 0;
    return d;
}
int helpers_locked(DagDevState& ds, int dev) {
    if (ds.helpers < 0) {
        int cus = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 2) cus = 64;
        ds.helpers = std::min(kDagMaxHelpers, cus - 1);   // every workgroup of the launch resident: one per CU
    }
    return ds.helpers;
}

}  // namespace

int dag_max_helpers() {
    const int dev = dag_cur_dev();
    DagDevState& ds = dag_dev(dev);
    std::lock_guard<std::mutex> g(ds.m);
    return helpers_locked(ds, dev);
}

void dag_stream_retired(hipStream_t st) {
    for (int d = 0; d < kMaxDagDevices; d++) {
        DagDevState& ds = dag_dev(d);
        std::lock_guard<std::mutex> g(ds.m);
        if (ds.has_last && ds.last == st) {
            ds.has_last = false;
            ds.after_valid = false;
        }
    }
}

void dag_device_stats(long long* launches, long long* handoffs) {
    DagDevState& ds = dag_dev(dag_cur_dev());
    std::lock_guard<std::mutex> g(ds.m);
    if (launches) *launches = ds.launches;
    if (handoffs) *handoffs = ds.handoffs;
}

unsigned dag_spin_max() {
    const char* e = std::getenv("ORBHIP_DAG_SPIN_MAX");   // read per call: tests force a timeout with it
    const long v = e ? std::atol(e) : 0;
    return v > 0 ? (unsigned)v : kSpinMax;
}

size_t dag_doubles(int n) { return dag_doubles_nt((n + kT - 1) / kT); }
size_t dag_ints(int n) {
    const size_t NT = (n + kT - 1) / kT;
    return (4 + NT * NT + 7 * NT + 3) & ~size_t(3);
}

void dag_plan(const int* rf, int n, int max_helpers, DagPlan& p, int nti) {
    const int NT = (n + kT - 1) / kT;
    p.NT = NT;
    p.nti = nti;
    // dependency keys (x20; the chain's interval k publishes at 20k + 6 and waits for the
    // helpers at 20k + 8): every task waits only on smaller keys, so each helper running its
    // tasks in key order with the whole grid resident cannot deadlock
    struct Task { int key, R, C; };
    std::vector<Task> ts;
    for (int R = 0; R < NT; R++)
        for (int C = rf[R]; C <= R; C++) {
            const int d = R - C;
            if (nti && C >= nti) {   // partial solve: the trailing block, after every column < nti
                ts.push_back({20 * nti + 7, R, C});
            } else if (d == 0) {
                // diagonal partial: columns <= C-4, so that its last full tile L(C, C-4) comes from the
                // Linv of four intervals back (one helper hop between two more); the chain applies C-3..C-1
                if (rf[R] <= C - 4) ts.push_back({20 * C - 70, R, C});
            } else if (d == 1) {
                if (std::max(rf[R], rf[C]) <= C - 3) ts.push_back({20 * C - 50, R, C});           // sub-diagonal partial
            } else if (d == 2) {
                if (std::max(rf[R], rf[C]) <= C - 2) ts.push_back({20 * C - 10, R, C});           // second sub-diagonal
            } else {
                ts.push_back({20 * C + 7, R, C});                                                  // full tile
            }
        }
    // backward substitution: over the helpers when the rows are long (the chain's own waves would
    // stream every tile of L through one CU: dense n = 2394 1.24 -> 0.69 ms), in the chain when
    // they are short (a band: the helpers' hand-off per step costs more than the tiles; the C5
    // loop and C4 systems). ORBHIP_DAG_PBACK=0/1 forces it.
    {
        long long off = 0;   // tiles the backward reads beyond the sub-diagonal
        for (int R = 0; R < NT; R++) off += std::max(0, R - 1 - rf[R]);
        const char* e = std::getenv("ORBHIP_DAG_PBACK");
        p.pb = e ? (e[0] == '1' ? 1 : 0) : (off >= 10LL * NT ? 1 : 0);
        if (nti) p.pb = 0;   // a partial solve has no backward substitution
    }
    // the chain's backward reads column-major copies: the full tiles' helper tasks write theirs, a
    // copy task per interval k <= NT - 3 those of the chain's own tiles (L(k+1, k), L(k+1, k-1),
    // Linv_k; the last interval's stay in the chain's LDS / are read in the quadrant layout). Key
    // 20k + 7: after the interval's publish (20k + 6); nothing but the backward waits on them
    if (!p.pb && !nti)
        for (int k = 0; k <= NT - 3; k++) ts.push_back({20 * k + 7, kCopyTask, k});
    std::sort(ts.begin(), ts.end(), [](const Task& x, const Task& y) {
        return x.key != y.key ? x.key < y.key : (x.R != y.R ? x.R < y.R : x.C < y.C);
    });
    const int G = std::min<int>(std::max(1, max_helpers), (int)ts.size());
    p.G = G;
    p.toff.assign(G + 1, 0);
    p.tasks.resize(ts.size());
    std::vector<int> cnt(G, 0);
    for (size_t i = 0; i < ts.size(); i++) cnt[i % G]++;
    for (int h = 0; h < G; h++) p.toff[h + 1] = p.toff[h] + cnt[h];
    std::vector<int> at(p.toff.begin(), p.toff.end() - 1);
    for (size_t i = 0; i < ts.size(); i++) p.tasks[at[i % G]++] = ts[i].R << 16 | ts[i].C;
    // the chain's backward: for each column k, the rows R >= k + 2 whose envelope reaches it (the
    // tiles its owner wave applies), after the task list (tasks[toff[G] + k])
    if (!p.pb && !nti)
        for (int k = 0; k < NT; k++) {
            int q = 0;
            for (int R = k + 2; R < NT; R++) q += rf[R] <= k ? 1 : 0;
            p.tasks.push_back(q);
        }
}

hipError_t chol_dag_solve(const double* S, int n, const int* row_first, const double* bs, double* x, int* flag,
                          const DagDev& d, hipStream_t st, const int* gate, unsigned long long* dbg) {
    if (n <= 0 || n > kDagMaxN) return hipErrorInvalidValue;
    DagK a;
    a.S = S; a.bs = bs; a.x = x; a.flag = flag; a.rf = row_first;
    a.buf = d.buf; a.ints = d.ints; a.toff = d.toff; a.tasks = d.tasks; a.need_off = d.need_off; a.gate = gate; a.dbg = dbg;
    a.n = n; a.NT = (n + kT - 1) / kT; a.G = d.G; a.pb = d.pb;
    static const int hs = std::getenv("ORBHIP_DAG_SLEEP") ? std::atoi(std::getenv("ORBHIP_DAG_SLEEP")) : 6;
    a.hsleep = hs;
    a.smax = dag_spin_max();
    a.ld = n; a.perm = nullptr; a.nti = 0;
    const int dev = dag_cur_dev();
    DagDevState& ds = dag_dev(dev);
    std::lock_guard<std::mutex> g(ds.m);
    if (d.G > helpers_locked(ds, dev)) return hipErrorInvalidValue;   // a plan made for a larger device
    if (!ds.attr) {
        for (const void* f : {(const void*)k_chol_dag<false>, (const void*)k_chol_dag<true>}) {
            const hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
            if (e != hipSuccess) return e;
        }
        ds.attr = true;
    }
    {   // device-wide order: after the other stream's last solve
        const hipError_t e = dag_handoff_before(ds, st);
        if (e != hipSuccess) return e;
    }
    if (dbg) hipLaunchKernelGGL(k_chol_dag<true>, dim3((unsigned)(d.G + 1)), dim3(256), dag_lds_bytes(a.NT), st, a);
    else hipLaunchKernelGGL(k_chol_dag<false>, dim3((unsigned)(d.G + 1)), dim3(256), dag_lds_bytes(a.NT), st, a);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? dag_handoff_after(ds, st) : e;
}

size_t dag_k_bytes() { return sizeof(DagK); }

int dag_multi_fill(const DagProb* probs, int np, void* host_ks, int* host_wgoff, const int* gate, size_t* lds) {
    DagK* ks = static_cast<DagK*>(host_ks);
    int g = 0;
    size_t l = 0;
    const unsigned smax = dag_spin_max();
    static const int hs = std::getenv("ORBHIP_DAG_SLEEP") ? std::atoi(std::getenv("ORBHIP_DAG_SLEEP")) : 6;
    for (int i = 0; i < np; i++) {
        const DagProb& q = probs[i];
        DagK& a = ks[i];
        a = DagK{};
        a.S = q.S; a.bs = q.bs; a.x = q.x; a.flag = q.flag; a.rf = q.rf;
        a.buf = q.d.buf; a.ints = q.d.ints; a.toff = q.d.toff; a.tasks = q.d.tasks; a.need_off = q.d.need_off;
        a.gate = gate; a.dbg = nullptr;
        a.n = q.n; a.NT = (q.n + kT - 1) / kT; a.G = q.d.G; a.pb = q.d.pb;
        a.hsleep = hs; a.smax = smax;
        a.ld = q.ld; a.perm = q.perm; a.nti = q.nti;
        host_wgoff[i] = g;
        g += q.d.G + 1;
        l = std::max(l, dag_lds_bytes(a.NT));
    }
    host_wgoff[np] = g;
    if (lds) *lds = l;
    return g;
}

hipError_t chol_dag_multi_launch(const void* d_ks, const int* d_wgoff, int np, int grid, size_t lds, hipStream_t st) {
    if (np <= 0 || grid <= 0) return hipErrorInvalidValue;
    const int dev = dag_cur_dev();
    DagDevState& ds = dag_dev(dev);
    std::lock_guard<std::mutex> g(ds.m);
    if (grid > helpers_locked(ds, dev) + 1) return hipErrorInvalidValue;   // one workgroup per CU
    if (!ds.attr_multi) {
        const hipError_t e = hipFuncSetAttribute((const void*)k_chol_dag_multi,
                                                 hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        if (e != hipSuccess) return e;
        ds.attr_multi = true;
    }
    {
        const hipError_t e = dag_handoff_before(ds, st);
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(k_chol_dag_multi, dim3((unsigned)grid), dim3(256), lds, st, (const DagK*)d_ks, d_wgoff, np);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? dag_handoff_after(ds, st) : e;
}

int chol_dag_test(const double* A, const double* b, double* x, int n, int reps, int max_helpers, float* ms,
                  unsigned long long* dbg) {
    if (n <= 0 || n > kDagMaxN || reps < 1) return -1;
    const int nt = (n + kT - 1) / kT;
    std::vector<int> rf(nt);
    for (int R = 0; R < nt; R++) {   // envelope of the dense input (lower triangle)
        int f = R;
        for (int r = kT * R; r < std::min(n, kT * R + kT); r++)
            for (int c = 0; c < kT * f && c <= r; c++)
                if (A[(size_t)r * n + c] != 0.0) {
                    f = std::min(f, c / kT);
                    break;
                }
        rf[R] = f;
    }
    DagPlan plan;
    dag_plan(rf.data(), n, max_helpers > 0 ? std::min(max_helpers, dag_max_helpers()) : dag_max_helpers(), plan);
    double *dS = nullptr, *db = nullptr, *dx = nullptr, *dbuf = nullptr;
    int *dints = nullptr, *dflag = nullptr, *drf = nullptr, *dtoff = nullptr, *dtasks = nullptr;
    unsigned long long* ddbg = nullptr;
    int rc = 0;
    auto ok = [&](hipError_t e) { if (e != hipSuccess && rc == 0) rc = -3; return e == hipSuccess; };
    ok(hipMalloc((void**)&dS, sizeof(double) * n * n));
    ok(hipMalloc((void**)&db, sizeof(double) * n));
    ok(hipMalloc((void**)&dx, sizeof(double) * n));
    ok(hipMalloc((void**)&dbuf, sizeof(double) * dag_doubles(n)));
    ok(hipMalloc((void**)&dints, sizeof(int) * dag_ints(n)));
    ok(hipMalloc((void**)&dflag, 4 * sizeof(int)));
    ok(hipMalloc((void**)&drf, sizeof(int) * nt));
    ok(hipMalloc((void**)&dtoff, sizeof(int) * plan.toff.size()));
    ok(hipMalloc((void**)&dtasks, sizeof(int) * std::max<size_t>(1, plan.tasks.size())));
    if (dbg) ok(hipMalloc((void**)&ddbg, sizeof(unsigned long long) * kDbgWords));
    if (rc == 0) {
        ok(hipMemset(dints, 0, sizeof(int) * dag_ints(n)));
        ok(hipMemset(dflag, 0, 4 * sizeof(int)));
        ok(hipMemcpy(dS, A, sizeof(double) * n * n, hipMemcpyHostToDevice));
        ok(hipMemcpy(db, b, sizeof(double) * n, hipMemcpyHostToDevice));
        ok(hipMemcpy(drf, rf.data(), sizeof(int) * nt, hipMemcpyHostToDevice));
        ok(hipMemcpy(dtoff, plan.toff.data(), sizeof(int) * plan.toff.size(), hipMemcpyHostToDevice));
        if (!plan.tasks.empty())
            ok(hipMemcpy(dtasks, plan.tasks.data(), sizeof(int) * plan.tasks.size(), hipMemcpyHostToDevice));
        if (ddbg) ok(hipMemset(ddbg, 0, sizeof(unsigned long long) * kDbgWords));
        const DagDev d{dbuf, dints, dtoff, dtasks, plan.G, plan.pb, plan.toff[plan.G]};
        ok(chol_dag_solve(dS, n, drf, db, dx, dflag, d, nullptr, nullptr, nullptr));   // warm-up
        ok(hipDeviceSynchronize());
        hipEvent_t e0, e1;
        ok(hipEventCreate(&e0));
        ok(hipEventCreate(&e1));
        ok(hipEventRecord(e0, nullptr));
        for (int r = 0; r < reps; r++) ok(chol_dag_solve(dS, n, drf, db, dx, dflag, d, nullptr, nullptr, ddbg));
        ok(hipEventRecord(e1, nullptr));
        ok(hipDeviceSynchronize());
        float t = 0;
        ok(hipEventElapsedTime(&t, e0, e1));
        if (ms) *ms = t / reps;
        int f = 0, ctl[4] = {0, 0, 0, 0};
        ok(hipMemcpy(&f, dflag, sizeof(int), hipMemcpyDeviceToHost));
        ok(hipMemcpy(ctl, dints, 4 * sizeof(int), hipMemcpyDeviceToHost));
        ok(hipMemcpy(x, dx, sizeof(double) * n, hipMemcpyDeviceToHost));
        if (ddbg) ok(hipMemcpy(dbg, ddbg, sizeof(unsigned long long) * kDbgWords, hipMemcpyDeviceToHost));
        if (rc == 0 && ctl[3] != 0) rc = -5;
        if (rc == 0 && f == 0) rc = -4;
        (void)hipEventDestroy(e0);
        (void)hipEventDestroy(e1);
    }
    (void)hipFree(dS); (void)hipFree(db); (void)hipFree(dx); (void)hipFree(dbuf); (void)hipFree(dints);
    (void)hipFree(dflag); (void)hipFree(drf); (void)hipFree(dtoff); (void)hipFree(dtasks);
    if (ddbg) (void)hipFree(ddbg);
    return rc;
}

}  // namespace orbhip
