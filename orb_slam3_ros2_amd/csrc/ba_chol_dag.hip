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
__device__ int wave_wait_prefix(const int* fa, const int* fb, const int* fc, int cnt, int epoch, int* ctl) {
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
        __builtin_amdgcn_s_sleep(2);
    }
}

struct Lay {   // offsets (doubles) into the DAG buffer, flags
    int oL, oP, oLi, oY, oR;
    int *ctl, *fL, *fP0, *fP1, *fCh;
    __device__ Lay(const DagK& a) {
        const int NT = a.NT;
        oL = 0;
        oP = NT * NT * kTD;
        oLi = oP + 2 * NT * kTD;
        oY = oLi + NT * kTD;
        oR = oY + NT * kT;
        ctl = a.ints;
        fL = ctl + 4;
        fP0 = fL + NT * NT;
        fP1 = fP0 + NT;
        fCh = fP1 + NT;
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
            const int m = wave_wait_prefix(fa, fb, fc, cnt, epoch, L.ctl);
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
        const int type = R == C ? 0 : (R == C + 1 ? 1 : 2);   // diag partial, sub-diag partial, full
        const int ps = max(a.rf[R], a.rf[C]), pe = type == 2 ? C : C - 2;
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
            qstore(rs, L.oP + (type == 0 ? C : NT + C) * kTD + quad * 256, acc);
            if (rhs && rg == 0) st_sc1(a.buf + L.oR + C * kT + 16 * rq + cc, rv);
            target = (type == 0 ? L.fP0 : L.fP1) + C;
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
    const bool ok = diag32_linv([&](int r, int c) { return Dx[qidx(r, c)]; }, scr,
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
    double* Lin = lds;                  // Linv_k (quadrant layout)
    double* Lsub = lds + 2048;          // L(k+1, k)
    double* Tx = lds + 3072;            // the sub-diagonal tile of the next TRSM
    double* Dx = lds + 4096;            // the diagonal tile to factor
    double* Dp = lds + 5120;            // the next diagonal tile, all but its last column
    int* word = (int*)(lds + 6144);     // [0..3] poll results, [4] prep abort, [5] row poll, [8] ok
    double* scr = lds + 6160;           // diag32 scratch (512)
    double* rvec = scr + 512;           // 32
    double* rpp = rvec + 32;            // 32: the next rhs, all but its last column
    double* ys = rpp + 32;              // NT x 32: y_k; in the backward the running sums s_k
    double* xs = ys + NT * kT;          // NT x 32
    unsigned long long* dbg = a.dbg;
    const unsigned long long t_start = dbg ? __builtin_amdgcn_s_memtime() : 0;
    unsigned long long t_fact = 0;
    bool ok = true, aborted = false;
    if (tid == 0) {
        word[4] = 0;
        word[5] = 1;
    }
    // Prep of interval K (waves 1..3, while wave 0 factors): the sub-diagonal tile (K+1, K) with
    // columns K-2 and K-1 (T, into Tx), the diagonal tile K+1 with column K-1 (into Dp) and its rhs
    // (rpp). Each wave polls the flags of the tiles it reads itself. False on abort.
    auto prep = [&](int K) -> bool {
        const int K1 = K + 1;
        const int rfa = a.rf[K1], rfb = a.rf[K];
        const bool inEnv = rfa <= K;
        const bool needP1 = inEnv && max(rfa, rfb) <= K - 3;
        const bool needP0 = rfa <= K - 2;
        const int pA = K - 2, pB = K - 1;
        const bool useA = inEnv && pA >= max(rfa, rfb);
        const bool useBs = inEnv && pB >= max(rfa, rfb);
        const bool useBd = pB >= rfa;
        const int* f = nullptr;
        if (lane == 0 && needP1) f = L.fP1 + K;
        if (lane == 1 && needP0) f = L.fP0 + K1;
        if (lane == 2 && useA) f = L.fL + K1 * NT + pA;
        if (lane == 3 && useA) f = L.fL + K * NT + pA;
        if (lane == 4 && useBd) f = L.fL + K1 * NT + pB;
        if (!wave_wait_all(f, epoch, L.ctl)) return false;
        const int tA1 = L.oL + (K1 * NT + pA) * kTD, tA0 = L.oL + (K * NT + pA) * kTD;
        const int tB = L.oL + (K1 * NT + pB) * kTD;
        auto tjob = [&](int qr, int qc) {
            double4_t T = {0, 0, 0, 0};
            if (inEnv) {
                T = needP1 ? qload(rs, L.oP + (NT + K) * kTD + (2 * qr + qc) * 256) : s_quad(a.S, n, K1, K, qr, qc);
                if (useA) {
                    mfma_sub(T, qload(rs, tA0 + (2 * qc) * 256), qload(rs, tA1 + (2 * qr) * 256));
                    mfma_sub(T, qload(rs, tA0 + (2 * qc + 1) * 256), qload(rs, tA1 + (2 * qr + 1) * 256));
                }
                if (useBs) {
                    mfma_sub(T, lq(Lsub + (2 * qc) * 256), qload(rs, tB + (2 * qr) * 256));
                    mfma_sub(T, lq(Lsub + (2 * qc + 1) * 256), qload(rs, tB + (2 * qr + 1) * 256));
                }
            }
            sq(Tx + (2 * qr + qc) * 256, T);
        };
        auto djob = [&](int qr, int qc) {
            double4_t D = needP0 ? qload(rs, L.oP + K1 * kTD + (2 * qr + qc) * 256) : s_quad(a.S, n, K1, K1, qr, qc);
            double r = 0.0;
            if (qc == 0) {
                const int i = kT * K1 + 16 * qr + cc;
                r = needP0 ? ld_sc1(a.buf + L.oR + K1 * kT + 16 * qr + cc) : (i < n ? a.bs[i] : 0.0);
            }
            if (useBd) {
                const double4_t l0 = qload(rs, tB + (2 * qr) * 256), l1 = qload(rs, tB + (2 * qr + 1) * 256);
                mfma_sub(D, qload(rs, tB + (2 * qc) * 256), l0);
                mfma_sub(D, qload(rs, tB + (2 * qc + 1) * 256), l1);
                if (qc == 0) r -= lmul_ylds(l0, ys + pB * kT) + lmul_ylds(l1, ys + pB * kT + 16);
            }
            sq(Dp + (2 * qr + qc) * 256, D);
            if (qc == 0 && rg == 0) rpp[16 * qr + cc] = r;
        };
        if (wid == 2) {
            tjob(0, 0);
            tjob(0, 1);
            djob(0, 0);
        } else if (wid == 3) {
            tjob(1, 0);
            tjob(1, 1);
            djob(1, 1);
        } else {
            djob(1, 0);
        }
        return true;
    };
    // ---- prologue: factor the diagonal tile 0 (wave 0) while waves 1..3 prepare interval 0 ----
    sq(Dx + quad * 256, s_quad(a.S, n, 0, 0, rq, cq));
    if (tid < kT) rvec[tid] = tid < n ? a.bs[tid] : 0.0;
    __syncthreads();
    if (wid == 0) ok = chain_factor(Dx, scr, Lin, rvec, ys);
    else if (NT > 1 && !prep(0) && lane == 0) word[4] = 1;
    __syncthreads();
    if (dbg && tid == 0) dbg[0] = __builtin_amdgcn_s_memtime() - t_start;
    // ---- intervals: TRSM | SYRK | diag32 (wave 0) beside the publish and the next prep ----
    for (int k = 0; k + 1 < NT; k++) {
        const unsigned long long tk = dbg ? __builtin_amdgcn_s_memtime() : 0;
        if (word[4]) {
            aborted = true;
            break;
        }
        const int k1 = k + 1;
        const bool inEnv = a.rf[k1] <= k;
        // phase 1: wave 1 issues the publish of Linv_k and y_k; every wave one quadrant of
        // L(k+1, k) = T Linv_k^T
        if (wid == 1) {
#pragma unroll
            for (int qd = 0; qd < 4; qd++) qstore(rs, L.oLi + k * kTD + qd * 256, lq(Lin + qd * 256));
            if (lane < kT) st_sc1(a.buf + L.oY + k * kT + lane, ys[k * kT + lane]);
        }
        double4_t Ln = {0, 0, 0, 0};
        if (inEnv) {
            panel_add(Ln, lq(Lin + (2 * cq) * 256), lq(Tx + (2 * rq) * 256));
            if (cq == 1) panel_add(Ln, lq(Lin + 3 * 256), lq(Tx + (2 * rq + 1) * 256));
        }
        sq(Lsub + quad * 256, Ln);
        __syncthreads();
        // phase 2: the diagonal tile's last column (waves 0, 2, 3: the lower quadrants)
        if (wid != 1) {
            double4_t D = lq(Dp + quad * 256);
            double r = cq == 0 ? rpp[16 * rq + cc] : 0.0;
            if (inEnv) {
                const double4_t l0 = lq(Lsub + (2 * rq) * 256), l1 = lq(Lsub + (2 * rq + 1) * 256);
                mfma_sub(D, lq(Lsub + (2 * cq) * 256), l0);
                mfma_sub(D, lq(Lsub + (2 * cq + 1) * 256), l1);
                if (cq == 0) r -= lmul_ylds(l0, ys + k * kT) + lmul_ylds(l1, ys + k * kT + 16);
            }
            sq(Dx + quad * 256, D);
            if (cq == 0 && rg == 0) rvec[16 * rq + cc] = r;
        }
        __syncthreads();
        // phase 3: wave 0 factors tile k+1; wave 1 publishes L(k+1, k), then waves 1..3 prepare
        // interval k+1
        const unsigned long long tf = dbg ? __builtin_amdgcn_s_memtime() : 0;
        if (wid == 0) {
            ok = chain_factor(Dx, scr, Lin, rvec, ys + k1 * kT) && ok;
            if (dbg) t_fact += __builtin_amdgcn_s_memtime() - tf;
        } else {
            if (wid == 1) {   // L(k+1, k); then both publishes are drained and flagged
#pragma unroll
                for (int qd = 0; qd < 4; qd++) qstore(rs, L.oL + (k1 * NT + k) * kTD + qd * 256, lq(Lsub + qd * 256));
                drain_stores();
                if (lane == 0) {
                    st_flag(L.fCh + k, epoch);
                    st_flag(L.fL + k1 * NT + k, epoch);
                }
            }
            if (k1 + 1 < NT && !prep(k1) && lane == 0) word[4] = 1;
        }
        __syncthreads();
        if (dbg && tid == 0 && k < 256) dbg[8 + k] = __builtin_amdgcn_s_memtime() - tk;
    }
    if (word[4]) aborted = true;
    const unsigned long long t_fwd = dbg ? __builtin_amdgcn_s_memtime() : 0;
    // ---- backward, right-looking by rows: at step R (x_R known) wave 0 forms x_{R-1} from the
    // sub-diagonal tile (R, R-1) and s_{R-1}; waves 1..3 subtract row R's other tiles from the
    // running sums s_j, j <= R-2. Wave 0's inputs (chain-published) and the first tiles of each
    // wave's next row are loaded a step ahead; wave 1 polls the helper tiles of row R-2 during
    // step R. ----
    auto apply_lt = [&](int k) {   // wave 0: xs_k = Linv^T rvec (Linv in Lin)
        const int c = lane >> 1, hh = lane & 1;
        double s = 0.0;
#pragma unroll
        for (int i = 0; i < 16; i++) s = fma(Lin[qidx(16 * hh + i, c)], rvec[16 * hh + i], s);
        s += dpp64<0xB1>(s);
        if (hh == 0) xs[k * kT + c] = s;
    };
    auto row_poll = [&](int R) -> bool {   // wave 1: the helper tiles (R, j), j <= R - 2
        bool good = true;
        for (int j0 = a.rf[R]; j0 <= R - 2 && good; j0 += 64) {
            const int j = j0 + lane;
            good = wave_wait_all(j <= R - 2 ? L.fL + R * NT + j : nullptr, epoch, L.ctl);
        }
        return good;
    };
    double4_t st[4], sn[4], li[4];   // wave 0: tile (R, R-1) now / next, Linv_{R-1}
    constexpr int kPf = 3;           // waves 1..3: tiles of a row prefetched a step ahead
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
        } else if (wid == 1 && NT >= 2) {
            const bool g = row_poll(NT - 1) && (NT < 3 || row_poll(NT - 2));
            if (lane == 0) word[5] = g ? 1 : 0;
        }
        __syncthreads();
        if (!word[5]) aborted = true;
        if (wid != 0 && !aborted && NT >= 2) {   // row NT-1's first tiles
            const int R = NT - 1, jn = a.rf[R] + (wid - 1);
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
            if (R >= 2) {   // prefetch step R-1's inputs
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
            // row R's helper tiles (R, j), j in [rf[R], R-2], dealt over waves 1..3 (j = rf[R] +
            // wid - 1 + 3 i); the first kPf of this wave were loaded during the previous step, the
            // next row's are issued now (their flags were polled two steps ahead)
            const int j0 = a.rf[R] + (wid - 1);
            if (R >= 2) {
                const int jn = a.rf[R - 1] + (wid - 1);
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
                double t[2][4];
                tile_lt_x(pf[u], xR, t);
                if (cc == 0) {
#pragma unroll
                    for (int b = 0; b < 2; b++)
#pragma unroll
                        for (int q = 0; q < 4; q++) ys[j * kT + 16 * b + rg + 4 * q] -= t[b][q];
                }
            }
            for (int j = j0 + 3 * kPf; j <= R - 2; j += 3) {   // long rows: the rest on demand
                double4_t tl[4];
#pragma unroll
                for (int qd = 0; qd < 4; qd++) tl[qd] = qload(rs, L.oL + (R * NT + j) * kTD + qd * 256);
                double t[2][4];
                tile_lt_x(tl, xR, t);
                if (cc == 0) {
#pragma unroll
                    for (int b = 0; b < 2; b++)
#pragma unroll
                        for (int q = 0; q < 4; q++) ys[j * kT + 16 * b + rg + 4 * q] -= t[b][q];
                }
            }
#pragma unroll
            for (int u = 0; u < kPf; u++)
#pragma unroll
                for (int qd = 0; qd < 4; qd++) pf[u][qd] = pn[u][qd];
            if (wid == 1 && R >= 3) {
                const bool g = row_poll(R - 2);
                if (lane == 0) word[5] = g ? 1 : 0;
            }
        }
        __syncthreads();
        if (!word[5]) aborted = true;
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
    const size_t bytes = ((size_t)a.NT * a.NT + 3 * (size_t)a.NT) * kTD * 8 + (size_t)a.NT * 64 * 8;
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
    const size_t need = sizeof(double) * (6160 + 512 + 64 + 2 * (size_t)NT * kT);
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
    return (NT * NT + 3 * NT) * kTD + NT * 64;
}
size_t dag_ints(int n) {
    const size_t NT = (n + kT - 1) / kT;
    return (4 + NT * NT + 3 * NT + 3) & ~size_t(3);
}

void dag_plan(const int* rf, int n, int max_helpers, DagPlan& p) {
    const int NT = (n + kT - 1) / kT;
    p.NT = NT;
    struct Task { int key, R, C; };
    std::vector<Task> ts;
    for (int R = 0; R < NT; R++)
        for (int C = rf[R]; C <= R; C++) {
            if (R == C) {
                if (rf[R] <= C - 3) ts.push_back({10 * C - 29, R, C});             // diagonal partial
            } else if (R == C + 1) {
                if (std::max(rf[R], rf[C]) <= C - 3) ts.push_back({10 * C - 29, R, C});   // sub-diagonal partial
            } else {
                ts.push_back({10 * C - 3, R, C});                                 // full tile
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
    if (dbg) ok(hipMalloc((void**)&ddbg, sizeof(unsigned long long) * (8 + 256)));
    if (rc == 0) {
        ok(hipMemset(dints, 0, sizeof(int) * dag_ints(n)));
        ok(hipMemset(dflag, 0, 4 * sizeof(int)));
        ok(hipMemcpy(dS, A, sizeof(double) * n * n, hipMemcpyHostToDevice));
        ok(hipMemcpy(db, b, sizeof(double) * n, hipMemcpyHostToDevice));
        ok(hipMemcpy(drf, rf.data(), sizeof(int) * nt, hipMemcpyHostToDevice));
        ok(hipMemcpy(dtoff, plan.toff.data(), sizeof(int) * plan.toff.size(), hipMemcpyHostToDevice));
        if (!plan.tasks.empty())
            ok(hipMemcpy(dtasks, plan.tasks.data(), sizeof(int) * plan.tasks.size(), hipMemcpyHostToDevice));
        if (ddbg) ok(hipMemset(ddbg, 0, sizeof(unsigned long long) * (8 + 256)));
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
        if (ddbg) ok(hipMemcpy(dbg, ddbg, sizeof(unsigned long long) * (8 + 256), hipMemcpyDeviceToHost));
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
