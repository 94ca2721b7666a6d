// Register-resident dense Cholesky + solve of the reduced camera system S xp = bs (a20:
// g2o LinearSolverEigen::solve behind OptimizationAlgorithmLevenberg), one 512-thread workgroup
// per problem, n <= kCholRegMaxN (C4: n = 294).
//
// The lower triangle of S is cut into 16x16 tiles; every off-diagonal tile is held TRANSPOSED in
// the v_mfma_f64_16x16x4f64 C/D layout (lane l: column l & 15, rows (l >> 4) + 4q), in which a
// tile's registers ARE the A/B operand of the next MFMA:
//   panel     L_Ik^T = Linv_k A_Ik^T      (A operand: Linv_k from LDS, B operand: the tile)
//   trailing  C_IJ^T -= L_Jk L_Ik^T       (both operands: panel tiles, published in LDS)
// Roles (r03): wave 0 is the CHAIN wave, waves 1..7 the workers.
//   - The chain wave owns the critical path: the diagonal tiles (LDS, Dt) and the sub-diagonal
//     tiles (k+1, k) (LDS, Sub). In interval k it applies column k-1 to tile (k+1, k), forms the
//     panel L_{k+1,k} = S_{k+1,k} Linv_k^T, applies columns k-1 and k to tile (k+1, k+1) and
//     factors it (diag16_linv: 4x4 pivot blocks on MFMA) into Linv_{k+1}, stored over Dt[k+1];
//     with the forward substitution y_{k+1} riding along.
//   - The workers own the tiles (I, J), I >= J + 2, in registers (column-major order, dealt
//     round-robin). In interval k they apply column k - 1 (one interval behind the chain: its
//     panels are published by then) to their tiles and to the diagonal tiles J >= k + 2 and the
//     sub-diagonal tiles (J+1, J), J >= k + 1, then form their panel tiles of column k. Panel
//     tiles of two consecutive columns live at once (Lp, double-buffered by column parity).
//   One workgroup barrier per interval; the chain's diagonal factorization overlaps the workers'
//   trailing updates instead of following them.
// Backward L^T x = y, one barrier per tile row: the chain wave finishes x_k from y_k, the
// sub-diagonal tile and Linv_k^T; the workers apply x_{k+1} to the y_J of their row-(k+1) tiles.
// S is read from HBM once and never written. Numerics: fp64 throughout; LL^T with 4x4 pivot
// blocks instead of Eigen's SimplicialLDLT (the same solution to rounding; parity is the LM result
// within 1e-4).
#include <hip/hip_runtime.h>

#include <utility>

#include "ba_args.h"
#include "dev_attr.h"
#include "ba_chol.h"
#include "ba_chol_reg.h"
#include "ba_diag16.h"
#include "wave_f64.h"

namespace orbhip {

namespace {

constexpr int kRegWaves = 8;
constexpr int kWorkers = kRegWaves - 1;

// Register tiles need compile-time slot indices (unrolled code). run_slots(t0, t1, f) runs f(t)
// for the slots in [t0, t1) (one scalar compare per skipped slot, no tile walking).
template <int MAXT, int T0, typename F>
__device__ __forceinline__ void run_slots_from(int t0, int t1, F&& f) {
    if constexpr (T0 < MAXT) {
        if (T0 >= t0 && T0 < t1) f(std::integral_constant<int, T0>{});
        run_slots_from<MAXT, T0 + 1>(t0, t1, f);
    }
}
template <int MAXT, typename F>
__device__ __forceinline__ void run_slots(int t0, int t1, F&& f) {
    run_slots_from<MAXT, 0>(t0, t1, f);
}

__device__ __forceinline__ double4_t load4(const double* p) { return double4_t{p[0], p[1], p[2], p[3]}; }
__device__ __forceinline__ void store4(double* p, const double4_t& v) {
    p[0] = v[0]; p[1] = v[1]; p[2] = v[2]; p[3] = v[3];
}
// c4 -= A B^T on two tiles in the transposed C layout (A, B: L_Jk^T and L_Ik^T -> c4 = C_IJ^T)
__device__ __forceinline__ void mfma_sub(double4_t& c4, const double4_t& a, const double4_t& b) {
    c4 = __builtin_amdgcn_mfma_f64_16x16x4f64(-a[0], b[0], c4, 0, 0, 0);
    c4 = __builtin_amdgcn_mfma_f64_16x16x4f64(-a[1], b[1], c4, 0, 0, 0);
    c4 = __builtin_amdgcn_mfma_f64_16x16x4f64(-a[2], b[2], c4, 0, 0, 0);
    c4 = __builtin_amdgcn_mfma_f64_16x16x4f64(-a[3], b[3], c4, 0, 0, 0);
}
// L^T of a panel tile: Linv (operand order in LDS) times the tile A^T (C layout, own registers)
__device__ __forceinline__ double4_t panel4(const double4_t& a, const double4_t& t) {
    double4_t r = {0, 0, 0, 0};
    r = __builtin_amdgcn_mfma_f64_16x16x4f64(a[0], t[0], r, 0, 0, 0);
    r = __builtin_amdgcn_mfma_f64_16x16x4f64(a[1], t[1], r, 0, 0, 0);
    r = __builtin_amdgcn_mfma_f64_16x16x4f64(a[2], t[2], r, 0, 0, 0);
    r = __builtin_amdgcn_mfma_f64_16x16x4f64(a[3], t[3], r, 0, 0, 0);
    return r;
}
// (L y_k) of a tile L_Ik held as L_Ik^T in the C layout (lane holds L_Ik[cc][rg + 4q]), summed over
// the 4 row groups: the result for row cc, identical in every row group
__device__ __forceinline__ double lmul_y(const double4_t& l, const double* yk) {
    const int rg = (threadIdx.x & 63) >> 4;
    const double sv = l[0] * yk[rg] + l[1] * yk[rg + 4] + l[2] * yk[rg + 8] + l[3] * yk[rg + 12];
    return col4_sum(sv);
}
// y_J -= L_IJ^T x_I for a tile held as L_IJ^T (lane (cc, rg) holds L_IJ[cc][rg + 4q])
__device__ __forceinline__ void lt_apply(const double4_t& l, const double* xi, double* yj) {
    const int lane = threadIdx.x & 63, cc = lane & 15, rg = lane >> 4;
    const double xv = xi[cc];
    double sq[4];
#pragma unroll
    for (int q = 0; q < 4; q++) sq[q] = row16_sum(l[q] * xv);
    if (cc == 0) {
#pragma unroll
        for (int q = 0; q < 4; q++) yj[rg + 4 * q] -= sq[q];
    }
}
// x_k <- Linv_k^T y_k in place (one wave)
__device__ __forceinline__ void apply_linv_t(const double* __restrict__ Linv_k, double* __restrict__ yk) {
    const int lane = threadIdx.x & 63, c = lane & 15, rg = lane >> 4;
    double s = 0.0;
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const int r = rg + 4 * q;
        s += Linv_k[(r + 16 * (c & 3)) * 4 + (c >> 2)] * yk[r];
    }
    s = col4_sum(s);
    wave_lds_sync();
    if (rg == 0) yk[c] = s;
    wave_lds_sync();
}
// factor the diagonal tile dt (chain wave): Linv_k in operand order over its own LDS slot
// (element (r, c) at ((r + 16 (c & 3)) * 4 + (c >> 2))), then y_k <- Linv_k y_k
__device__ __forceinline__ bool chain_diag(const double4_t& dt, double* __restrict__ Linv_k, double* __restrict__ yk) {
    const bool ok = diag16_linv(dt, [&](int r, int c, double v) { Linv_k[(r + 16 * (c & 3)) * 4 + (c >> 2)] = v; });
    wave_lds_sync();
    const int lane = threadIdx.x & 63, r = lane >> 2, h = lane & 3;
    double sv = 0.0;
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const int c = 4 * h + j;
        sv = fma(Linv_k[(r + 16 * (c & 3)) * 4 + (c >> 2)], yk[c], sv);
    }
    sv += dpp64<0xB1>(sv);   // quad_perm [1,0,3,2]
    sv += dpp64<0x4E>(sv);   // quad_perm [2,3,0,1]
    wave_lds_sync();
    if (h == 0) yk[r] = sv;
    wave_lds_sync();
    return ok;
}

}  // namespace

size_t chol_reg_lds_bytes(int n) {
    const int T = (n + 15) / 16;
    return sizeof(double) * (4 * (size_t)T * 256 + 16 * (size_t)T + 8);
}

// shared LDS layout and element loads of one problem
typedef __attribute__((address_space(1))) const double gdouble;   // global loads, not flat
struct RegCtx {
    gdouble* S;
    int n, T, lane, cc, rg;
    double *Dt, *Sub, *Lp0, *y;
    int* bad;
    __device__ double* Lp(int k, int I) const { return Lp0 + ((size_t)(k & 1) * T + I) * 256 + lane * 4; }
    __device__ double* tileD(int J) const { return Dt + (size_t)J * 256 + lane * 4; }
    __device__ double* tileS(int J) const { return Sub + (size_t)J * 256 + lane * 4; }
    // element (a = rg + 4q, b = cc) of C_IJ^T = S[16I + b][16J + a]; inside a 6x6 diagonal block
    // the two triangles are separate sums (read the lower one), elsewhere S is an exact mirror
    // (read the coalesced row c)
    __device__ double s_elem(int I, int J, int q, bool valid) const {
        const int r = 16 * I + cc, c = 16 * J + rg + 4 * q;
        const bool in = valid && r < n && c < n;
        const size_t off = !in ? 0 : (r / 6 == c / 6) ? (size_t)max(r, c) * n + min(r, c) : (size_t)c * n + r;
        const double v = S[off];
        return in ? v : (r == c ? 1.0 : 0.0);
    }
    __device__ double4_t s_tile(int I, int J) const {
        double4_t v;
#pragma unroll
        for (int q = 0; q < 4; q++) v[q] = s_elem(I, J, q, true);
        return v;
    }
};

// The chain wave (wave 0). Barriers: 1 (prologue) + (T - 1) intervals + 1 + (T - 1) backward rows,
// the same count as worker_wave.
__device__ __forceinline__ void chain_wave(const RegCtx& R, unsigned long long* dbg) {
    const int T = R.T, cc = R.cc, rg = R.rg, lane = R.lane;
    double* y = R.y;
    unsigned long long t_start = dbg ? __builtin_amdgcn_s_memtime() : 0, t_busy = 0, t_diag = 0;
    __builtin_amdgcn_s_setprio(3);   // the chain wave issues first on its SIMD
    const double4_t d0 = R.s_tile(0, 0);
    for (int J = 1; J < T; J += kRegWaves) store4(R.tileD(J), R.s_tile(J, J));
    for (int J = 0; J < T - 1; J += kRegWaves) store4(R.tileS(J), R.s_tile(J + 1, J));
    wave_lds_sync();   // y[0..63] are this wave's own stores
    bool ok = chain_diag(d0, R.Dt, y);
    __syncthreads();
    if (dbg && lane == 0) dbg[0] = __builtin_amdgcn_s_memtime() - t_start;
    const unsigned long long t_fact = dbg ? __builtin_amdgcn_s_memtime() : 0;
    for (int k = 0; k < T - 1; k++) {
        const unsigned long long tb = dbg ? __builtin_amdgcn_s_memtime() : 0;
        // (a) column k-1 into the sub-diagonal tile (k+1, k); (b) its panel L_{k+1,k}
        double4_t s4 = load4(R.tileS(k));
        double4_t lkm{0, 0, 0, 0};   // L_{k+1,k-1}^T
        if (k >= 1) {
            lkm = load4(R.Lp(k - 1, k + 1));
            mfma_sub(s4, load4(R.tileS(k - 1)), lkm);
        }
        const double4_t l4 = panel4(load4(R.tileD(k)), s4);
        store4(R.tileS(k), l4);
        // (c) columns k-1 and k into the diagonal tile (k+1, k+1) and y_{k+1}
        double4_t dt = load4(R.tileD(k + 1));
        double ys = lmul_y(l4, y + 16 * k);
        if (k >= 1) {
            mfma_sub(dt, lkm, lkm);
            ys += lmul_y(lkm, y + 16 * (k - 1));
        }
        mfma_sub(dt, l4, l4);
        if (rg == 0) y[16 * (k + 1) + cc] -= ys;
        wave_lds_sync();
        // (d) factor it: Linv_{k+1} over Dt[k+1], y_{k+1} <- Linv_{k+1} y_{k+1}
        const unsigned long long td = dbg ? __builtin_amdgcn_s_memtime() : 0;
        ok = chain_diag(dt, R.Dt + (size_t)(k + 1) * 256, y + 16 * (k + 1)) && ok;
        if (dbg) {
            const unsigned long long te = __builtin_amdgcn_s_memtime();
            t_diag += te - td;
            t_busy += te - tb;
        }
        __syncthreads();
    }
    if (!ok) *R.bad = 1;
    else if (lane == 0) *R.bad = 0;
    apply_linv_t(R.Dt + (size_t)(T - 1) * 256, y + 16 * (T - 1));   // x_{T-1}
    __syncthreads();
    const unsigned long long t_back = dbg ? __builtin_amdgcn_s_memtime() : 0;
    for (int k = T - 2; k >= 0; k--) {
        lt_apply(load4(R.tileS(k)), y + 16 * (k + 1), y + 16 * k);
        wave_lds_sync();
        apply_linv_t(R.Dt + (size_t)k * 256, y + 16 * k);
        __syncthreads();
    }
    if (dbg && lane == 0) {
        const unsigned long long te = __builtin_amdgcn_s_memtime();
        dbg[1] = t_back - t_fact;
        dbg[2] = te - t_back;
        dbg[3] = t_busy;
        dbg[4] = t_diag;
    }
}

// A worker wave (1..7): its tiles (I, J), I >= J + 2, in registers (column-major index g, tile g
// in slot g / 7 of worker 1 + g % 7).
template <int MAXT>
__device__ __forceinline__ void worker_wave(const RegCtx& R, int wid) {
    const int T = R.T, cc = R.cc, rg = R.rg;
    double* y = R.y;
    const int NW = (T - 1) * (T - 2) / 2;
    const int wi = wid - 1;
    const int nslots = wi < NW ? (NW - wi + kWorkers - 1) / kWorkers : 0;
    auto offw = [&](int J) { return J * (T - 2) - J * (J - 1) / 2; };   // worker tiles in columns < J
    auto slot_at = [&](int G) { return min(nslots, G > wi ? (G - wi + kWorkers - 1) / kWorkers : 0); };
    int rIJ[MAXT];   // I | J << 8 of each slot (wave-uniform)
    double4_t acc[MAXT];
    {
        int I = 2 + wi, J = 0;
        while (I >= T && J < T - 2) { I = I - T + J + 3; J++; }
#pragma unroll
        for (int t = 0; t < MAXT; t++) {
            const bool v = t < nslots;
            rIJ[t] = (v ? I : 255) | J << 8;
#pragma unroll
            for (int q = 0; q < 4; q++) acc[t][q] = R.s_elem(I, J, q, v);
            I += kWorkers;
            while (I >= T && J < T - 2) { I = I - T + J + 3; J++; }
        }
    }
    for (int J = 1 + wid; J < T; J += kRegWaves) store4(R.tileD(J), R.s_tile(J, J));
    for (int J = wid; J < T - 1; J += kRegWaves) store4(R.tileS(J), R.s_tile(J + 1, J));
    __syncthreads();
    for (int k = 0; k < T - 1; k++) {
        if (k >= 1) {
            const int c = k - 1;
            // column c into this worker's tiles of columns >= k
            run_slots<MAXT>(slot_at(offw(k)), nslots, [&](auto tc) {
                constexpr int t = decltype(tc)::value;
                const int I = rIJ[t] & 0xFF, J = rIJ[t] >> 8;
                mfma_sub(acc[t], load4(J == k ? R.tileS(c) : R.Lp(c, J)), load4(R.Lp(c, I)));
            });
            // column c into the diagonal tiles J >= k + 2 (with y_J) and the sub-diagonal tiles
            // (J + 1, J), J >= k + 1: items dealt round-robin over the workers
            const int nd = T - k - 2;   // diagonal items J = k + 2 + i; sub-diagonal J = k + 1 + i
            for (int it = wi; it < 2 * nd; it += kWorkers) {
                if (it < nd) {
                    const int J = k + 2 + it;
                    const double4_t l = load4(R.Lp(c, J));
                    double4_t d4 = load4(R.tileD(J));
                    mfma_sub(d4, l, l);
                    store4(R.tileD(J), d4);
                    const double ys = lmul_y(l, y + 16 * c);
                    if (rg == 0) y[16 * J + cc] -= ys;
                } else {
                    const int J = k + 1 + (it - nd);
                    double4_t s4 = load4(R.tileS(J));
                    mfma_sub(s4, load4(R.Lp(c, J)), load4(R.Lp(c, J + 1)));
                    store4(R.tileS(J), s4);
                }
            }
        }
        // panel k: this worker's tiles of column k
        const double4_t a = load4(R.tileD(k));   // Linv_k in operand order
        run_slots<MAXT>(slot_at(offw(k)), slot_at(offw(k + 1)), [&](auto tc) {
            constexpr int t = decltype(tc)::value;
            acc[t] = panel4(a, acc[t]);
            store4(R.Lp(k, rIJ[t] & 0xFF), acc[t]);
        });
        __syncthreads();
    }
    __syncthreads();   // the chain wave's x_{T-1}
    for (int k = T - 2; k >= 0; k--) {
        run_slots<MAXT>(0, nslots, [&](auto tc) {
            constexpr int t = decltype(tc)::value;
            if ((rIJ[t] & 0xFF) == k + 1) lt_apply(acc[t], y + 16 * (k + 1), y + 16 * (rIJ[t] >> 8));
        });
        __syncthreads();
    }
}

template <int MAXT>
__device__ __forceinline__ void chol_reg_solve(const double* __restrict__ S, const double* __restrict__ bs,
                                               double* __restrict__ x, int n, int* __restrict__ flag,
                                               unsigned long long* __restrict__ dbg = nullptr) {
    // dbg (diagnostics, chain wave): [0] prologue (loads + diag 0), [1] factorization intervals,
    // [2] backward, [3] chain-wave busy cycles in the intervals, [4] diag16 cycles summed
    extern __shared__ __attribute__((aligned(16))) double lds[];
    RegCtx R;
    R.S = (gdouble*)S;
    R.n = n;
    R.T = (n + 15) >> 4;
    const int tid = threadIdx.x;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    R.lane = tid & 63; R.cc = R.lane & 15; R.rg = R.lane >> 4;
    R.Dt = lds;                                 // T x 256: diagonal tiles (C layout), then Linv_k (operand order)
    R.Sub = R.Dt + (size_t)R.T * 256;           // T x 256: S_{J+1,J}^T, then L_{J+1,J}^T (C layout)
    R.Lp0 = R.Sub + (size_t)R.T * 256;          // 2 x T x 256: workers' panel tiles L_{I,k}^T by column parity
    R.y = R.Lp0 + 2 * (size_t)R.T * 256;        // 16 T: y, then x in place
    R.bad = (int*)(R.y + 16 * R.T);
    for (int i = tid; i < 16 * R.T; i += blockDim.x) R.y[i] = i < n ? bs[i] : 0.0;
    if (wid == 0) chain_wave(R, dbg);
    else worker_wave<MAXT>(R, wid);
    const int nb = *R.bad;
    for (int i = tid; i < n; i += blockDim.x) x[i] = nb ? 0.0 : R.y[i];
    if (tid == 0) flag[0] = nb ? 0 : 1;
}

template <int MT>
__global__ __launch_bounds__(512) void k_ba_chol_reg(const BaArgs* __restrict__ args, const int* __restrict__ act) {
    const BaArgs& a = args[act[blockIdx.x]];
    if (a.ctl && a.ctl->phase != kPhTrial) return;   // device-driven rounds: not in a trial
    if (a.n == 0) {
        if (threadIdx.x == 0) a.flag[0] = 1;
        return;
    }
    chol_reg_solve<MT>(a.S, a.bs, a.x, a.n, a.flag);
}

template <int MT>
__global__ __launch_bounds__(512) void k_chol_reg_probe(const BaArgs* __restrict__ args, unsigned long long* dbg) {
    chol_reg_solve<MT>(args->S, args->bs, args->x, args->n, args->flag, dbg);
}

hipError_t chol_reg_probe(int n, const BaArgs* args, unsigned long long* dbg, hipStream_t st) {
    const size_t lds = chol_reg_lds_bytes(n);
    const dim3 g(1), b(512);
    switch (chol_reg_maxt(n)) {
        case 4: hipLaunchKernelGGL(k_chol_reg_probe<4>, g, b, lds, st, args, dbg); break;
        case 8: hipLaunchKernelGGL(k_chol_reg_probe<8>, g, b, lds, st, args, dbg); break;
        case 12: hipLaunchKernelGGL(k_chol_reg_probe<12>, g, b, lds, st, args, dbg); break;
        case 16: hipLaunchKernelGGL(k_chol_reg_probe<16>, g, b, lds, st, args, dbg); break;
        case 20: hipLaunchKernelGGL(k_chol_reg_probe<20>, g, b, lds, st, args, dbg); break;
        case 22: hipLaunchKernelGGL(k_chol_reg_probe<22>, g, b, lds, st, args, dbg); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

int chol_reg_maxt(int n) {
    const int T = (n + 15) / 16, nt = T >= 2 ? (T - 1) * (T - 2) / 2 : 0;
    const int need = (nt + kWorkers - 1) / kWorkers;
    return need <= 4 ? 4 : need <= 8 ? 8 : need <= 12 ? 12 : need <= 16 ? 16 : need <= 20 ? 20 : need <= 22 ? 22 : 0;
}

hipError_t chol_reg_launch(int maxN, int nprob, const BaArgs* args, const int* act, hipStream_t st) {
    const int mt = chol_reg_maxt(maxN);
    if (!mt) return hipErrorInvalidValue;
    static LdsAttrOnce attr;   // per device, thread-safe (dev_attr.h)
    static const void* const fs[] = {(const void*)k_ba_chol_reg<4>, (const void*)k_ba_chol_reg<8>,
                                     (const void*)k_ba_chol_reg<12>, (const void*)k_ba_chol_reg<16>,
                                     (const void*)k_ba_chol_reg<20>, (const void*)k_ba_chol_reg<22>,
                                     (const void*)k_chol_reg_probe<4>, (const void*)k_chol_reg_probe<8>,
                                     (const void*)k_chol_reg_probe<12>, (const void*)k_chol_reg_probe<16>,
                                     (const void*)k_chol_reg_probe<20>, (const void*)k_chol_reg_probe<22>};
    {
        const hipError_t e = attr.ensure(fs, 12, 160 * 1024);
        if (e != hipSuccess) return e;
    }
    const size_t lds = chol_reg_lds_bytes(maxN);
    const dim3 g((unsigned)nprob), b(512);
    switch (mt) {
        case 4: hipLaunchKernelGGL(k_ba_chol_reg<4>, g, b, lds, st, args, act); break;
        case 8: hipLaunchKernelGGL(k_ba_chol_reg<8>, g, b, lds, st, args, act); break;
        case 12: hipLaunchKernelGGL(k_ba_chol_reg<12>, g, b, lds, st, args, act); break;
        case 16: hipLaunchKernelGGL(k_ba_chol_reg<16>, g, b, lds, st, args, act); break;
        case 20: hipLaunchKernelGGL(k_ba_chol_reg<20>, g, b, lds, st, args, act); break;
        default: hipLaunchKernelGGL(k_ba_chol_reg<22>, g, b, lds, st, args, act); break;
    }
    return hipGetLastError();
}

}  // namespace orbhip
