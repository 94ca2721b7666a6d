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
constexpr unsigned kSpinMax = 1u << 19;
constexpr size_t kMinLds = 84 * 1024;   // > 80 KB: one workgroup per CU
#ifndef ORBHIP_DAG_NEWTON
#define ORBHIP_DAG_NEWTON 1
#endif
constexpr int kNewton = ORBHIP_DAG_NEWTON;   // Newton steps after v_rsq_f64 in the pivot blocks

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
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
    const int* gate;
    unsigned long long* dbg;
    int n, NT, G;
    int hsleep;   // helpers' poll back-off (units of s_sleep 1)
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
// quadrant (a, b) of tile (R, C) of S (plain loads: written by earlier kernels only); the lower
// triangle is read (mirrored above the diagonal), identity outside the matrix
__device__ __forceinline__ double4_t s_quad(const double* __restrict__ S, int n, int R, int C, int a, int b) {
    const int lane = threadIdx.x & 63;
    const int r = kT * R + 16 * a + (lane & 15);
    double4_t v;
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const int c = kT * C + 16 * b + (lane >> 4) + 4 * q;
        const bool in = r < n && c < n;
        const size_t off = !in ? 0 : (r >= c ? (size_t)r * n + c : (size_t)c * n + r);
        const double s = S[off];
        v[q] = in ? s : (r == c ? 1.0 : 0.0);
    }
    return v;
}
// c4 -= A B^T in the transposed C layout (a: L_Jk quadrant, b: L_Ik quadrant -> C_IJ^T)
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

// every lane's flag (nullptr: none) equal to epoch; false on abort / timeout (wave-uniform)
__device__ bool wave_wait_all(const int* f, int epoch, int* ctl) {
    for (unsigned spins = 0;; spins++) {
        const bool ok = !f || ld_flag(f) == epoch;
        if (__all(ok)) return true;
        if (ld_flag(ctl + 2) == epoch) return false;
        if (spins >= kSpinMax) {
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
__device__ int wave_wait_prefix(const int* fa, const int* fb, const int* fc, int cnt, int epoch, int* ctl, int hsleep) {
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
        if (spins >= kSpinMax) {
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
    int oL, oP, oLi, oY, oR;
    int *ctl, *fL, *fP0, *fP1, *fP2, *fCh;
    __device__ Lay(const DagK& a) {
        const int NT = a.NT;
        oL = 0;
        oP = NT * NT * kTD;
        oLi = oP + 3 * NT * kTD;
        oY = oLi + NT * kTD;
        oR = oY + NT * kT;
        ctl = a.ints;
        fL = ctl + 4;
        fP0 = fL + NT * NT;
        fP1 = fP0 + NT;
        fP2 = fP1 + NT;
        fCh = fP2 + NT;
    }
};

// ---------------------------------------------------------------------------------------------
// helper workgroup: its tasks in order
// ---------------------------------------------------------------------------------------------
__device__ void dag_helper(const DagK& a, const Lay& L, __amdgpu_buffer_rsrc_t rs, int epoch, double* lds) {
    const int tid = threadIdx.x, wid = tid >> 6, lane = tid & 63, cc = lane & 15, rg = lane >> 4;
    const int rq = wid >> 1, cq = wid & 1, quad = 2 * rq + cq;
    const int NT = a.NT;
    double* Tx = lds + 2048;
    int* word = (int*)(lds + 4096);
    const int h = blockIdx.x - 1;
    const int t0 = a.toff[h], t1 = a.toff[h + 1];
    int wsel = 0;   // rotating LDS word of the poll results
    auto wg_prefix = [&](const int* fa, const int* fb, const int* fc, int cnt) -> int {
        if (wid == 0) {
            const int m = wave_wait_prefix(fa, fb, fc, cnt, epoch, L.ctl, a.hsleep);
            if (lane == 0) word[wsel] = m;
        }
        __syncthreads();
        const int m = word[wsel];
        wsel = (wsel + 1) & 3;
        return m;
    };
    for (int t = t0; t < t1; t++) {
        const int code = a.tasks[t];
        const int R = code >> 16, C = code & 0xFFFF;
        // by R - C: 0 the diagonal partial (columns <= C-3), 1 the sub-diagonal partial (<= C-3), 2
        // the second sub-diagonal's partial (<= C-2), >= 3 a full tile (every column, then the TRSM)
        const int dRC = R - C;
        const int type = dRC >= 3 ? 2 : (dRC == 0 ? 0 : 1);
        const int ps = max(a.rf[R], a.rf[C]), pe = dRC >= 3 ? C : (dRC == 2 ? C - 1 : C - 2);
        double4_t acc = s_quad(a.S, a.n, R, C, rq, cq);
        const bool rhs = type == 0 && cq == 0;
        const bool skip = type == 0 && quad == 1;   // the upper quadrant of a diagonal tile: unused
        double rv = 0.0;
        if (rhs) {
            const int i = kT * R + 16 * rq + cc;
            rv = i < a.n ? a.bs[i] : 0.0;
        }
        bool fail = false;
        for (int p = ps; p < pe && !fail;) {
            const int cnt = min(64, pe - p);
            const int m = wg_prefix(L.fL + R * NT + p, R != C ? L.fL + C * NT + p : nullptr,
                                    type == 0 ? L.fCh + p : nullptr, cnt);
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
            target = L.fL + R * NT + C;
        } else {
            qstore(rs, L.oP + (dRC * NT + C) * kTD + quad * 256, acc);
            if (rhs && rg == 0) st_sc1(a.buf + L.oR + C * kT + 16 * rq + cc, rv);
            target = (dRC == 0 ? L.fP0 : (dRC == 1 ? L.fP1 : L.fP2)) + C;
        }
        drain_stores();
        __syncthreads();
        if (tid == 0) st_flag(target, epoch);
    }
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

__device__ void dag_chain(const DagK& a, const Lay& L, __amdgpu_buffer_rsrc_t rs, int epoch, double* lds) {
    const int tid = threadIdx.x, wid = tid >> 6, lane = tid & 63, cc = lane & 15, rg = lane >> 4;
    const int rq = wid >> 1, cq = wid & 1, quad = 2 * rq + cq;
    const int NT = a.NT, n = a.n;
    // double buffers by base arithmetic (an array of LDS pointers selected at run time loses the
    // address space: flat accesses, which wait on vmcnt too)
    //   lds + 1024 p: Linv_k (p = k & 1); lds + 2048 + 1024 c1: L(k, k-1) / the new L(k+1, k);
    //   lds + 4096 + 1024 c2: L(k+1, k-1) / the new L(k+2, k)
    double* Tp = lds + 6144;            // T'_k: tile (k+1, k) with columns <= k-2 applied
    double* Tx = lds + 7168;            // exchange tile
    double* Dp = lds + 8192;            // D'_{k+1}: diagonal tile k+1 with columns <= k-2 applied
    double* Dx = lds + 9216;            // the diagonal tile to factor
    int* word = (int*)(lds + 10240);    // [0..3] poll results, [4] abort, [5] row polls ok, [8] ok
    double* scr = lds + 10256;          // diag32 scratch (512)
    double* rvec = scr + 512;           // 32
    double* rpp = rvec + 32;            // 32: rhs of D'
    double* ys = rpp + 32;              // NT x 32: y_k; in the backward the running sums s_k
    double* xs = ys + NT * kT;          // NT x 32
    int* rfl = (int*)(xs + NT * kT);    // row_first (NT ints)
    unsigned long long* dbg = a.dbg;
    const unsigned long long t_start = dbg ? __builtin_amdgcn_s_memtime() : 0;
    unsigned long long t_fact = 0;
    bool ok = true, aborted = false;
    if (tid == 0) {
        word[4] = 0;
        word[5] = 1;
    }
    for (int i = tid; i < NT; i += blockDim.x) rfl[i] = a.rf[i];
    int c1 = 0, c2 = 0;   // current L1 / L2 buffers
    // ---- prologue: factor tile 0 (wave 0); T'_0 = A(1, 0), D'_1 = A(1, 1), L1 = L2 = 0 ----
    sq(Dx + quad * 256, s_quad(a.S, n, 0, 0, rq, cq));
    sq(lds + 2048 + quad * 256, double4_t{0, 0, 0, 0});
    sq(lds + 4096 + quad * 256, double4_t{0, 0, 0, 0});
    if (NT > 1) {
        sq(Tp + quad * 256, a.rf[1] <= 0 ? s_quad(a.S, n, 1, 0, rq, cq) : double4_t{0, 0, 0, 0});
        sq(Dp + quad * 256, s_quad(a.S, n, 1, 1, rq, cq));
        if (cq == 0 && rg == 0) {
            const int i = kT + 16 * rq + cc;
            rpp[16 * rq + cc] = i < n ? a.bs[i] : 0.0;
        }
    }
    if (tid < kT) rvec[tid] = tid < n ? a.bs[tid] : 0.0;
    __syncthreads();
    if (wid == 0) ok = chain_factor(Dx, scr, lds, rvec, ys);
    __syncthreads();
    if (dbg && tid == 0) dbg[0] = __builtin_amdgcn_s_memtime() - t_start;
    // ---- interval k: phase 1 L(k+1, k) = (T'_k - L(k+1,k-1) L(k,k-1)^T) Linv_k^T; phase 2 the
    // diagonal tile k+1's last two columns and its rhs; phase 3 wave 0 factors it, wave 1
    // publishes and loads D'_{k+2}, waves 2 / 3 form row 0 / 1 of L(k+2, k) and of T'_{k+1} ----
    for (int k = 0; k + 1 < NT; k++) {
        const unsigned long long tk = dbg ? __builtin_amdgcn_s_memtime() : 0;
        const int k1 = k + 1, K2 = k + 2;
        double* Lin = lds + 1024 * (k & 1);
        double* LinN = lds + 1024 * (k1 & 1);
        double* L1 = lds + 2048 + 1024 * c1;
        double* L1n = lds + 2048 + 1024 * (c1 ^ 1);
        double* L2 = lds + 4096 + 1024 * c2;
        double* L2n = lds + 4096 + 1024 * (c2 ^ 1);
        const int rfa = rfl[k1], rfb = rfl[k];
        const bool inEnv1 = rfa <= k;
        const bool useT2 = k - 1 >= max(rfa, rfb);
        const bool useD2 = k - 1 >= rfa;
        // the flags waves 2 / 3 need in phase 3, loaded now (in flight through phases 1 and 2)
        const int rfc = K2 < NT ? rfl[K2] : 0;
        const bool inEnvU = K2 < NT && rfc <= k, inEnvT = K2 < NT && rfc <= k1;
        const bool needP2 = K2 < NT && max(rfc, rfb) <= k - 2, useU = K2 < NT && k - 1 >= max(rfc, rfb);
        const bool needP1 = K2 < NT && max(rfc, rfa) <= k - 2, useTp = K2 < NT && k - 1 >= max(rfc, rfa);
        const bool needP0 = K2 < NT && rfc <= K2 - 3;
        const int* f3 = nullptr;
        if (wid >= 2) {
            if (lane == 0 && needP2) f3 = L.fP2 + k;
            if (lane == 1 && (useU || useTp)) f3 = L.fL + K2 * NT + k - 1;
            if (lane == 2 && needP1) f3 = L.fP1 + k1;
            if (lane == 3 && needP0) f3 = L.fP0 + K2;
        }
        const bool need3 = f3 != nullptr;
        const int fv = ld_flag(need3 ? f3 : L.ctl);   // unconditional: its wait lands at the use in phase 3
        // wave 1 issues the publish of L(k+1, k-1) and Linv_k, y_k (drained in phase 3)
        if (wid == 1) {
            if (k >= 1) {
#pragma unroll
                for (int qd = 0; qd < 4; qd++) qstore(rs, L.oL + (k1 * NT + k - 1) * kTD + qd * 256, lq(L2 + qd * 256));
            }
#pragma unroll
            for (int qd = 0; qd < 4; qd++) qstore(rs, L.oLi + k * kTD + qd * 256, lq(Lin + qd * 256));
            if (lane < kT) st_sc1(a.buf + L.oY + k * kT + lane, ys[k * kT + lane]);
        }
        // phase 1
        double4_t T = lq(Tp + quad * 256);
        if (useT2) {   // two independent MFMA chains
            double4_t T2 = {0, 0, 0, 0};
            mfma_sub(T, lq(L1 + (2 * cq) * 256), lq(L2 + (2 * rq) * 256));
            mfma_sub(T2, lq(L1 + (2 * cq + 1) * 256), lq(L2 + (2 * rq + 1) * 256));
            T += T2;
        }
        sq(Tx + quad * 256, T);
        lds_barrier();
        double4_t Ln = {0, 0, 0, 0};
        if (inEnv1) {
            panel_add(Ln, lq(Lin + (2 * cq) * 256), lq(Tx + (2 * rq) * 256));
            if (cq == 1) {
                double4_t L2c = {0, 0, 0, 0};
                panel_add(L2c, lq(Lin + 3 * 256), lq(Tx + (2 * rq + 1) * 256));
                Ln += L2c;
            }
        }
        sq(L1n + quad * 256, Ln);
        lds_barrier();
        const unsigned long long tp1 = dbg ? __builtin_amdgcn_s_memtime() : 0;
        // phase 2 (waves 0, 2, 3: the lower quadrants)
        if (wid != 1) {
            double4_t D = lq(Dp + quad * 256);
            double4_t D1 = {0, 0, 0, 0}, D2 = {0, 0, 0, 0}, D3 = {0, 0, 0, 0};   // independent chains
            double r = cq == 0 ? rpp[16 * rq + cc] : 0.0;
            if (useD2) {
                const double4_t l0 = lq(L2 + (2 * rq) * 256), l1 = lq(L2 + (2 * rq + 1) * 256);
                mfma_sub(D2, lq(L2 + (2 * cq) * 256), l0);
                mfma_sub(D3, lq(L2 + (2 * cq + 1) * 256), l1);
                if (cq == 0) r -= lmul_ylds(l0, ys + (k - 1) * kT) + lmul_ylds(l1, ys + (k - 1) * kT + 16);
            }
            if (inEnv1) {
                const double4_t l0 = lq(L1n + (2 * rq) * 256), l1 = lq(L1n + (2 * rq + 1) * 256);
                mfma_sub(D, lq(L1n + (2 * cq) * 256), l0);
                mfma_sub(D1, lq(L1n + (2 * cq + 1) * 256), l1);
                if (cq == 0) r -= lmul_ylds(l0, ys + k * kT) + lmul_ylds(l1, ys + k * kT + 16);
            }
            D += (D1 + D2) + D3;
            sq(Dx + quad * 256, D);
            if (cq == 0 && rg == 0) rvec[16 * rq + cc] = r;
        } else {   // wave 1: the publish of L(k+1, k)
#pragma unroll
            for (int qd = 0; qd < 4; qd++) qstore(rs, L.oL + (k1 * NT + k) * kTD + qd * 256, lq(L1n + qd * 256));
        }
        lds_barrier();
        // phase 3
        const unsigned long long tf = dbg ? __builtin_amdgcn_s_memtime() : 0;
        unsigned long long* wts = (unsigned long long*)word + 8;   // per-wave phase-3 cycles (dbg)
        if (wid == 0) {
            ok = chain_factor(Dx, scr, LinN, rvec, ys + k1 * kT) && ok;
            if (dbg) t_fact += __builtin_amdgcn_s_memtime() - tf;
        } else if (wid == 1) {   // the publishes of this interval complete: drain, then the flags
            drain_stores();
            if (lane == 0) {
                st_flag(L.fCh + k, epoch);
                st_flag(L.fL + k1 * NT + k, epoch);
                if (k >= 1) st_flag(L.fL + k1 * NT + k - 1, epoch);
            }
        } else if (K2 < NT) {
            // waves 2 / 3: row h of L(k+2, k) = U Linv_k^T, U = A(k+2, k) - sum_{p <= k-1}
            // L(k+2,p) L(k,p)^T (the helpers' partial: p <= k-2; here p = k-1), and row h of
            // T'_{k+1} = A(k+2, k+1) - sum_{p <= k-1} L(k+2,p) L(k+1,p)^T (partial p <= k-2)
            const int h = wid - 2;
            if (!__all(!need3 || fv == epoch) && !wave_wait_all(f3, epoch, L.ctl)) {
                if (lane == 0) word[4] = 1;
            } else {
                const int tD = L.oL + (K2 * NT + k - 1) * kTD;
                double4_t d0 = {0, 0, 0, 0}, d1 = {0, 0, 0, 0};
                if (useU || useTp) {
                    d0 = qload(rs, tD + (2 * h) * 256);
                    d1 = qload(rs, tD + (2 * h + 1) * 256);
                }
                // D'_{k+2}: the helpers' partial (columns <= k-1) or A(k+2, k+2), and its rhs; wave 2
                // the quadrant (0, 0) and rows 0..15, wave 3 (1, 0), (1, 1) and rows 16..31
#pragma unroll
                for (int qd = 2 * h; qd <= 2 * h + h; qd++)
                    if (qd != 1)
                        sq(Dp + qd * 256, needP0 ? qload(rs, L.oP + K2 * kTD + qd * 256) : s_quad(a.S, n, K2, K2, qd >> 1, qd & 1));
                if (lane < 16) {
                    const int i = kT * K2 + 16 * h + lane;
                    rpp[16 * h + lane] = needP0 ? ld_sc1(a.buf + L.oR + K2 * kT + 16 * h + lane) : (i < n ? a.bs[i] : 0.0);
                }
                double4_t u[2], t[2];
#pragma unroll
                for (int c = 0; c < 2; c++) {
                    u[c] = !inEnvU ? double4_t{0, 0, 0, 0}
                                   : (needP2 ? qload(rs, L.oP + (2 * NT + k) * kTD + (2 * h + c) * 256)
                                             : s_quad(a.S, n, K2, k, h, c));
                    t[c] = !inEnvT ? double4_t{0, 0, 0, 0}
                                   : (needP1 ? qload(rs, L.oP + (NT + k1) * kTD + (2 * h + c) * 256)
                                             : s_quad(a.S, n, K2, k1, h, c));
                }
                double4_t o0 = {0, 0, 0, 0}, o1 = {0, 0, 0, 0};
                if (inEnvU) {
                    if (useU) {
#pragma unroll
                        for (int c = 0; c < 2; c++) {
                            mfma_sub(u[c], lq(L1 + (2 * c) * 256), d0);
                            mfma_sub(u[c], lq(L1 + (2 * c + 1) * 256), d1);
                        }
                    }
                    panel_add(o0, lq(Lin), u[0]);
                    panel_add(o1, lq(Lin + 2 * 256), u[0]);
                    panel_add(o1, lq(Lin + 3 * 256), u[1]);
                }
                sq(L2n + (2 * h) * 256, o0);
                sq(L2n + (2 * h + 1) * 256, o1);
                if (inEnvT && useTp) {
#pragma unroll
                    for (int c = 0; c < 2; c++) {
                        mfma_sub(t[c], lq(L2 + (2 * c) * 256), d0);
                        mfma_sub(t[c], lq(L2 + (2 * c + 1) * 256), d1);
                    }
                }
                sq(Tp + (2 * h) * 256, t[0]);
                sq(Tp + (2 * h + 1) * 256, t[1]);
            }
        }
        if (dbg && lane == 0) wts[wid] = __builtin_amdgcn_s_memtime() - tf;
        lds_barrier();
        c1 ^= 1;
        c2 ^= 1;
        if (dbg && tid == 0 && k < 200) {
            unsigned long long* dk = dbg + 8 + 6 * k;
            dk[0] = __builtin_amdgcn_s_memtime() - tk;
            dk[1] = tp1 - tk;
            dk[2] = tf - tp1;
            dk[3] = wts[0];
            dk[4] = wts[1];
            dk[5] = std::max(wts[2], wts[3]);
        }
        if (word[4]) {
            aborted = true;
            break;
        }
    }
    const unsigned long long t_fwd = dbg ? __builtin_amdgcn_s_memtime() : 0;
    double* Lin = lds + 1024 * ((NT - 1) & 1);
    // ---- backward, right-looking by rows: at step R (x_R known) wave 0 forms x_{R-1} from the
    // sub-diagonal tile (R, R-1) and s_{R-1}; waves 1..3 subtract row R's other tiles from the
    // running sums s_j, j <= R-2. The helper tiles' flags are polled once, up front; wave 0's
    // inputs and the first tiles of each wave's next row are loaded a step ahead. ----
    auto apply_lt = [&](int k) {   // wave 0: xs_k = Linv^T rvec (Linv in Lin)
        const int c = lane >> 1, hh = lane & 1;
        double s = 0.0;
#pragma unroll
        for (int i = 0; i < 16; i++) s = fma(Lin[qidx(16 * hh + i, c)], rvec[16 * hh + i], s);
        s += dpp64<0xB1>(s);
        if (hh == 0) xs[k * kT + c] = s;
    };
    auto sub_tile = [&](const double4_t* tl, const double* xR, int j) {   // s_j -= L(R, j)^T x_R
        double t[2][4];
        tile_lt_x(tl, xR, t);
        if (cc == 0) {
#pragma unroll
            for (int b = 0; b < 2; b++)
#pragma unroll
                for (int q = 0; q < 4; q++) ys[j * kT + 16 * b + rg + 4 * q] -= t[b][q];
        }
    };
    double4_t st[4], sn[4], li[4];   // wave 0: tile (R, R-1) now / next, Linv_{R-1}
    constexpr int kPf = 3;           // waves 1..3: tiles of a row loaded a step ahead
    double4_t pf[kPf][4], pn[kPf][4];
    if (!aborted) {
        if (wid == 0) {
            if (lane < kT) rvec[lane] = ys[(NT - 1) * kT + lane];
            wave_lds_sync();
            apply_lt(NT - 1);
            if (NT >= 2) {
#pragma unroll
                for (int qd = 0; qd < 4; qd++) {
                    st[qd] = qload(rs, L.oL + ((NT - 1) * NT + NT - 2) * kTD + qd * 256);
                    li[qd] = qload(rs, L.oLi + (NT - 2) * kTD + qd * 256);
                }
            }
        } else {
            // every tile (R, j), j <= R-2, rows 2.. (16 rows of this wave per round: up to 32
            // flag loads in flight per lane)
            bool good = true;
            for (int R0 = 1 + wid; R0 < NT && good; R0 += 48) {
                for (unsigned spins = 0;; spins++) {
                    int okl = 1;
#pragma unroll
                    for (int u = 0; u < 16; u++) {
                        const int R = R0 + 3 * u;
                        if (R < NT) {
                            const int rfR = rfl[R];
#pragma unroll
                            for (int hh = 0; hh < 2; hh++) {
                                const int j = rfR + 64 * hh + lane;
                                if (j <= R - 2) okl &= ld_flag(L.fL + R * NT + j) == epoch ? 1 : 0;
                            }
                        }
                    }
                    if (__all(okl)) break;
                    if (ld_flag(L.ctl + 2) == epoch || spins >= kSpinMax) {
                        if (spins >= kSpinMax && lane == 0) {
                            st_flag(L.ctl + 2, epoch);
                            __hip_atomic_fetch_add((gint*)(L.ctl + 3), 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        }
                        good = false;
                        break;
                    }
                    __builtin_amdgcn_s_sleep(2);
                }
            }
            if (!good && lane == 0) word[5] = 0;
        }
        __syncthreads();
        if (!word[5]) aborted = true;
        if (wid != 0 && !aborted && NT >= 2) {   // row NT-1's first tiles
            const int R = NT - 1, jn = rfl[R] + (wid - 1);
#pragma unroll
            for (int u = 0; u < kPf; u++)
                if (jn + 3 * u <= R - 2) {
#pragma unroll
                    for (int qd = 0; qd < 4; qd++) pf[u][qd] = qload(rs, L.oL + (R * NT + jn + 3 * u) * kTD + qd * 256);
                }
        }
    }
    for (int R = NT - 1; R >= 1 && !aborted; R--) {
        const double* xR = xs + R * kT;
        if (wid == 0) {
            // x_{R-1} = Linv_{R-1}^T (s_{R-1} - L(R, R-1)^T x_R)
#pragma unroll
            for (int qd = 0; qd < 4; qd++) sq(Lin + qd * 256, li[qd]);
            double t[2][4];
            tile_lt_x(st, xR, t);
            if (cc == 0) {
#pragma unroll
                for (int b = 0; b < 2; b++)
#pragma unroll
                    for (int q = 0; q < 4; q++) {
                        const int c = 16 * b + rg + 4 * q;
                        rvec[c] = ys[(R - 1) * kT + c] - t[b][q];
                    }
            }
            if (R >= 2) {   // step R-1's inputs
#pragma unroll
                for (int qd = 0; qd < 4; qd++) {
                    sn[qd] = qload(rs, L.oL + ((R - 1) * NT + R - 2) * kTD + qd * 256);
                    li[qd] = qload(rs, L.oLi + (R - 2) * kTD + qd * 256);
                }
            }
            wave_lds_sync();
            apply_lt(R - 1);
#pragma unroll
            for (int qd = 0; qd < 4; qd++) st[qd] = sn[qd];
        } else {
            // row R's tiles (R, j), j in [rf[R], R-2], j = rf[R] + wid - 1 + 3 i: the first kPf
            // came a step ahead, the next row's are issued now, the rest four at a time
            const int j0 = rfl[R] + (wid - 1);
            if (R >= 2) {
                const int jn = rfl[R - 1] + (wid - 1);
#pragma unroll
                for (int u = 0; u < kPf; u++)
                    if (jn + 3 * u <= R - 3) {
#pragma unroll
                        for (int qd = 0; qd < 4; qd++) pn[u][qd] = qload(rs, L.oL + ((R - 1) * NT + jn + 3 * u) * kTD + qd * 256);
                    }
            }
#pragma unroll
            for (int u = 0; u < kPf; u++) {
                const int j = j0 + 3 * u;
                if (j > R - 2) break;
                sub_tile(pf[u], xR, j);
            }
            for (int jb = j0 + 3 * kPf; jb <= R - 2; jb += 12) {
                double4_t tl[4][4];
#pragma unroll
                for (int u = 0; u < 4; u++)
                    if (jb + 3 * u <= R - 2) {
#pragma unroll
                        for (int qd = 0; qd < 4; qd++) tl[u][qd] = qload(rs, L.oL + (R * NT + jb + 3 * u) * kTD + qd * 256);
                    }
#pragma unroll
                for (int u = 0; u < 4; u++)
                    if (jb + 3 * u <= R - 2) sub_tile(tl[u], xR, jb + 3 * u);
            }
#pragma unroll
            for (int u = 0; u < kPf; u++)
#pragma unroll
                for (int qd = 0; qd < 4; qd++) pf[u][qd] = pn[u][qd];
        }
        lds_barrier();   // LDS only: the next step's tiles stay in flight
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

__global__ __launch_bounds__(256) void k_chol_dag(DagK a) {
    if (a.gate && *a.gate != kPhTrial) return;   // device-driven LM: not in a trial (uniform)
    extern __shared__ __attribute__((aligned(16))) double lds[];
    const Lay L(a);
    // epoch of this solve: the counter the last workgroup of the previous solve advanced
    const int epoch = ld_flag(L.ctl) + 1;
    const size_t bytes = ((size_t)a.NT * a.NT + 4 * (size_t)a.NT) * kTD * 8 + (size_t)a.NT * 64 * 8;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(a.buf, 0, (int)bytes, 0x00020000);
    if (blockIdx.x == 0) dag_chain(a, L, rs, epoch, lds);
    else dag_helper(a, L, rs, epoch, lds);
    // the last workgroup out advances the epoch counter
    drain_stores();
    __syncthreads();
    if (threadIdx.x == 0) {
        const int old = __hip_atomic_fetch_add((gint*)(L.ctl + 1), 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (old == (int)gridDim.x - 1) {
            st_flag(L.ctl + 1, 0);
            st_flag(L.ctl, epoch);
        }
    }
}

size_t dag_lds_bytes(int NT) {
    const size_t need = sizeof(double) * (10256 + 512 + 64 + 2 * (size_t)NT * kT) + sizeof(int) * NT;
    return std::max(need, kMinLds);
}

}  // namespace

int dag_max_helpers() {
    static int g = -1;
    if (g < 0) {
        int dev = 0, cus = 0;
        if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) !=
                                                    hipSuccess || cus < 2)
            cus = 64;
        g = std::min(kDagMaxHelpers, cus - 1);   // every workgroup of the launch resident: one per CU
    }
    return g;
}

size_t dag_doubles(int n) {
    const size_t NT = (n + kT - 1) / kT;
    return (NT * NT + 4 * NT) * kTD + NT * 64;
}
size_t dag_ints(int n) {
    const size_t NT = (n + kT - 1) / kT;
    return (4 + NT * NT + 4 * NT + 3) & ~size_t(3);
}

void dag_plan(const int* rf, int n, int max_helpers, DagPlan& p) {
    const int NT = (n + kT - 1) / kT;
    p.NT = NT;
    // dependency keys (x20; the chain's interval k publishes at 20k + 6 and waits for the
    // helpers at 20k + 8): every task waits only on smaller keys, so each helper running its
    // tasks in key order with the whole grid resident cannot deadlock
    struct Task { int key, R, C; };
    std::vector<Task> ts;
    for (int R = 0; R < NT; R++)
        for (int C = rf[R]; C <= R; C++) {
            const int d = R - C;
            if (d == 0) {
                if (rf[R] <= C - 3) ts.push_back({20 * C - 50, R, C});                            // diagonal partial
            } else if (d == 1) {
                if (std::max(rf[R], rf[C]) <= C - 3) ts.push_back({20 * C - 50, R, C});           // sub-diagonal partial
            } else if (d == 2) {
                if (std::max(rf[R], rf[C]) <= C - 2) ts.push_back({20 * C - 10, R, C});           // second sub-diagonal
            } else {
                ts.push_back({20 * C + 7, R, C});                                                  // full tile
            }
        }
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
}

hipError_t chol_dag_solve(const double* S, int n, const int* row_first, const double* bs, double* x, int* flag,
                          const DagDev& d, hipStream_t st, const int* gate, unsigned long long* dbg) {
    if (n <= 0 || n > kDagMaxN) return hipErrorInvalidValue;
    static bool attr = false;
    if (!attr) {
        const hipError_t e = hipFuncSetAttribute((const void*)k_chol_dag, hipFuncAttributeMaxDynamicSharedMemorySize,
                                                 160 * 1024);
        if (e != hipSuccess) return e;
        attr = true;
    }
    DagK a;
    a.S = S; a.bs = bs; a.x = x; a.flag = flag; a.rf = row_first;
    a.buf = d.buf; a.ints = d.ints; a.toff = d.toff; a.tasks = d.tasks; a.gate = gate; a.dbg = dbg;
    a.n = n; a.NT = (n + kT - 1) / kT; a.G = d.G;
    static const int hs = std::getenv("ORBHIP_DAG_SLEEP") ? std::atoi(std::getenv("ORBHIP_DAG_SLEEP")) : 6;
    a.hsleep = hs;
    hipLaunchKernelGGL(k_chol_dag, dim3((unsigned)(d.G + 1)), dim3(256), dag_lds_bytes(a.NT), st, a);
    return hipGetLastError();
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
        const DagDev d{dbuf, dints, dtoff, dtasks, plan.G};
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
