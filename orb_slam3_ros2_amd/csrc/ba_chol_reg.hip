// Register-resident dense Cholesky + solve of the reduced camera system S xp = bs (a20:
// g2o LinearSolverEigen::solve behind OptimizationAlgorithmLevenberg), one 512-thread workgroup
// per problem, n <= kCholRegMaxN (C4: n = 294).
//
// The lower triangle of S is cut into 16x16 tiles. The off-diagonal tile (I, J), I > J, column-
// major index g, lives for the whole factorization in the registers of wave g % 8 (slot g / 8),
// stored TRANSPOSED in the v_mfma_f64_16x16x4f64 C/D layout (lane l: column l & 15, rows
// (l >> 4) + 4q). In that form a tile's registers ARE the A/B operand of the next MFMA (lane l:
// row l & 15, k = (l >> 4) + 4kk), so nothing is ever re-laid out:
//   panel     L_Ik^T = Linv_k A_Ik^T      (A operand: Linv_k from LDS, B operand: own registers)
//   trailing  C_IJ^T -= L_Jk L_Ik^T       (both operands: the panel tiles, published in LDS)
// The diagonal tiles live in LDS and are updated by compact code; S is read from HBM once and
// never written back. One step k is
//   [panel k] barrier [wave (k+1)%8: finish tile (k+1, k+1), y_{k+1} -= L y_k, factor it
//   (look-ahead) | others: diagonal-tile and y updates, then their trailing register tiles] barrier
// so the diagonal chain overlaps the trailing work of the other waves.
// Diagonal factorization: 2x2-block Gaussian elimination on [D | I] in one wave (rows through a
// small LDS scratch, columns by DPP row_newbcast, pivot blocks by readlane, rsq/rcp + Newton steps
// instead of IEEE div/sqrt sequences), giving Linv = Lp^-1 X. L itself is never formed: the panel
// needs Linv, and both triangular solves use Linv_k (kept in LDS) and the L_Ik register tiles.
// Code-size note: the whole step loop must stay inside the instruction cache, so per-slot code is
// minimal and the passes enter the unrolled slot code at their first live slot (run_slots).
// Numerics: fp64 throughout; LL^T with 2x2 pivot blocks instead of Eigen's SimplicialLDLT (the same
// solution to rounding; parity is the LM result within 1e-4).
#include <hip/hip_runtime.h>

#include <utility>

#include "ba_args.h"
#include "ba_chol.h"
#include "ba_chol_reg.h"
#include "wave_f64.h"

namespace orbhip {

namespace {

constexpr int kRegWaves = 8;

// Register tiles need compile-time slot indices (unrolled code). run_slots(t0, t1, f) runs f(t)
// for the slots in [t0, t1) (one scalar compare per skipped slot, no tile walking); at_slot(t, f)
// runs one slot through a binary dispatch.
template <int MAXT, int T0, typename F>
__device__ __forceinline__ void run_slots_from(int t0, int t1, F&& f) {
    if constexpr (T0 < MAXT) {
        // t0, t1 wave-uniform: a skipped slot costs two scalar compares (flat control flow)
        if (T0 >= t0 && T0 < t1) f(std::integral_constant<int, T0>{});
        run_slots_from<MAXT, T0 + 1>(t0, t1, f);
    }
}
template <int MAXT, typename F>
__device__ __forceinline__ void run_slots(int t0, int t1, F&& f) {
    run_slots_from<MAXT, 0>(t0, t1, f);
}
template <int MAXT, int LO, int HI, typename F>
__device__ __forceinline__ void at_slot_bs(int t, F&& f) {
    if constexpr (HI - LO == 1) {
        f(std::integral_constant<int, LO>{});
    } else {
        constexpr int MID = (LO + HI) / 2;
        if (t < MID) at_slot_bs<MAXT, LO, MID>(t, f);
        else at_slot_bs<MAXT, MID, HI>(t, f);
    }
}
template <int MAXT, typename F>
__device__ __forceinline__ void at_slot(int t, F&& f) {
    at_slot_bs<MAXT, 0, MAXT>(t, f);
}

// DPP row_newbcast without the init move of update_dpp (every lane of a row is a valid source)
template <int CTRL>
__device__ __forceinline__ double bcast64(double v) {
    return mk64((unsigned)__builtin_amdgcn_mov_dpp((int)lo32(v), CTRL, 0xF, 0xF, true),
                (unsigned)__builtin_amdgcn_mov_dpp((int)hi32(v), CTRL, 0xF, 0xF, true));
}

// One 2x2-block Gaussian-elimination step on [D | X] (C layout: lane (cc, rg) holds D[rg + 4q][cc]
// and X[rg + 4q][cc]), pivots J0 = 2P and J1 = 2P + 1: with the pivot block B = D[J0..J1][J0..J1],
// rows r > J1 get [D | X][r] -= [D[r][J0] D[r][J1]] B^-1 [D | X][J0..J1]. Half the sequential steps
// of scalar pivoting, same Schur complements. Rows J0, J1 cross lanes through LDS (abd + 24, two
// alternating 64-double buffers); columns J0, J1 come by DPP row_newbcast; the block by readlane. The D entries left of /
// above the trailing block are not masked: they only feed other such entries, never a later pivot
// or X. abd[3P..3P+2] receives the block's (a, b, det) for block_params; *ok is cleared on a
// non-positive-definite block.
template <int P>
__device__ __forceinline__ void elim_block(double4_t& d, double4_t& xv, int rg, int cc, double* abd, bool& ok) {
    constexpr int J0 = 2 * P, J1 = 2 * P + 1, jq = J0 >> 2, r0 = J0 & 3, r1 = J1 & 3;
    // rows J0, J1 of [D | X] cross lanes through LDS (lane cc reads its 4 values with two 16-byte
    // loads); measured faster than permlane16/32 broadcasts here (n = 294: 180 vs 198 us)
    double* buf = abd + 24 + 64 * (P & 1);
    if (rg == r0) { buf[cc * 4 + 0] = d[jq]; buf[cc * 4 + 1] = xv[jq]; }
    if (rg == r1) { buf[cc * 4 + 2] = d[jq]; buf[cc * 4 + 3] = xv[jq]; }
    double u0[4], u1[4];
#pragma unroll
    for (int q = 0; q < 4; q++) {
        u0[q] = bcast64<0x150 + J0>(d[q]);   // D[rg + 4q][J0]
        u1[q] = bcast64<0x150 + J1>(d[q]);   // D[rg + 4q][J1]
    }
    const double a = readlane_f64(d[jq], J0 + 16 * r0);   // D[J0][J0]
    const double b = readlane_f64(d[jq], J0 + 16 * r1);   // D[J1][J0]
    const double c = readlane_f64(d[jq], J1 + 16 * r1);   // D[J1][J1]
    const double det = a * c - b * b;
    double id = __builtin_amdgcn_rcp(det);
    id = fma(id, fma(-det, id, 1.0), id);
    id = fma(id, fma(-det, id, 1.0), id);
    const double i00 = c * id, i01 = -b * id, i11 = a * id;
    wave_lds_sync();
    const double d0 = buf[cc * 4 + 0], x0 = buf[cc * 4 + 1], d1 = buf[cc * 4 + 2], x1 = buf[cc * 4 + 3];
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const bool below = rg + 4 * q > J1;
        const double m0 = below ? fma(u0[q], i00, u1[q] * i01) : 0.0;
        const double m1 = below ? fma(u0[q], i01, u1[q] * i11) : 0.0;
        d[q] = fma(-m1, d1, fma(-m0, d0, d[q]));
        xv[q] = fma(-m1, x1, fma(-m0, x0, xv[q]));
    }
    ok = ok && a > 0.0 && det > 0.0;
    // the block's Cholesky-inverse parameters are computed for all 8 blocks together after the
    // elimination (block_params): only (a, b, det) leave the chain here
    if ((threadIdx.x & 63) == 0) {
        abd[3 * P] = a;
        abd[3 * P + 1] = b;
        abd[3 * P + 2] = det;
    }
    __builtin_amdgcn_sched_barrier(0);   // keep each step's live range local (register budget)
}

// prm[3P..3P+2] = Cholesky inverse [[s0, 0], [s1, s2]] of pivot block P from its (a, b, det):
// s0 = 1/sqrt(a), s2 = 1/sqrt(det/a), s1 = -b s0^2 s2; rsq + 2 Newton steps, one lane per block
__device__ __forceinline__ void block_params(const double* abd, double* prm) {
    const int lane = threadIdx.x & 63;
    if (lane < 8) {
        const double a = abd[3 * lane], b = abd[3 * lane + 1], det = abd[3 * lane + 2];
        double s0 = __builtin_amdgcn_rsq(a);
        s0 = s0 * fma(-0.5 * a * s0, s0, 1.5);
        s0 = s0 * fma(-0.5 * a * s0, s0, 1.5);
        const double sc2 = det * s0 * s0;              // det / a
        double s2 = __builtin_amdgcn_rsq(sc2);
        s2 = s2 * fma(-0.5 * sc2 * s2, s2, 1.5);
        s2 = s2 * fma(-0.5 * sc2 * s2, s2, 1.5);
        prm[3 * lane] = s0;
        prm[3 * lane + 1] = -b * s0 * s0 * s2;
        prm[3 * lane + 2] = s2;
    }
}

template <int... P>
__device__ __forceinline__ void elim_all(double4_t& d, double4_t& xv, int rg, int cc, double* abd, bool& ok,
                                         std::integer_sequence<int, P...>) {
    (elim_block<P>(d, xv, rg, cc, abd, ok), ...);
}

// Factor the diagonal tile held in d (C layout) with LDS scratch sc (128 doubles) and prm (24).
// Writes Linv_k = Lp^-1 X (Lp: the block-diagonal Cholesky factor of the 2x2 pivots) into LDS in
// operand order (element (r, c) at ((r + 16 (c & 3)) * 4 + (c >> 2))), applies y_k <- Linv_k y_k,
// and sets *bad on a non-positive-definite pivot block.
__device__ __forceinline__ void diag_tile(double4_t d, double* __restrict__ Linv_k, double* __restrict__ yk,
                                          double* __restrict__ sc, double* __restrict__ prm, int* bad,
                                          unsigned long long* tel = nullptr) {
    const int lane = threadIdx.x & 63, cc = lane & 15, rg = lane >> 4;
    const unsigned long long te0 = tel ? __builtin_amdgcn_s_memtime() : 0;
    double4_t xv;
#pragma unroll
    for (int q = 0; q < 4; q++) xv[q] = (rg + 4 * q == cc) ? 1.0 : 0.0;
    bool ok = true;
    elim_all(d, xv, rg, cc, sc, ok, std::make_integer_sequence<int, 8>{});
    if (tel) tel[0] += __builtin_amdgcn_s_memtime() - te0;
    wave_lds_sync();
    block_params(sc, prm);
    wave_lds_sync();
#pragma unroll
    for (int q = 0; q < 4; q++) {
        // row r = rg + 4q is row J0 (rg even) or J1 (rg odd) of block r / 2; an odd row needs X of
        // row r - 1: the even row group of the same q (permlane16_swap)
        const int P = (rg + 4 * q) >> 1;
        const auto sl = __builtin_amdgcn_permlane16_swap(lo32(xv[q]), lo32(xv[q]), false, false);
        const auto sh = __builtin_amdgcn_permlane16_swap(hi32(xv[q]), hi32(xv[q]), false, false);
        const double xprev = mk64(sl[0], sh[0]);
        const double l = (rg & 1) ? fma(xv[q], prm[3 * P + 2], xprev * prm[3 * P + 1]) : xv[q] * prm[3 * P];
        Linv_k[(rg + 4 * q + 16 * (cc & 3)) * 4 + (cc >> 2)] = l;
    }
    wave_lds_sync();
    // y_k <- Linv_k y_k: lane (r, h) sums columns 4h..4h+3 of row r from LDS, then two DPP levels
    {
        const int r = lane >> 2, h = lane & 3;
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
    }
    if (lane == 0 && !ok) *bad = 1;
    wave_lds_sync();
    if (tel) tel[1] += __builtin_amdgcn_s_memtime() - te0;
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

}  // namespace

size_t chol_reg_lds_bytes(int n) {
    const int T = (n + 15) / 16;
    return sizeof(double) * (3 * (size_t)T * 256 + 16 * (size_t)T + 176 + 8);
}

template <int MAXT>
__device__ __forceinline__ void chol_reg_solve(const double* __restrict__ S, const double* __restrict__ bs,
                                               double* __restrict__ x, int n, int* __restrict__ flag,
                                               unsigned long long* __restrict__ dbg = nullptr) {
    // dbg (diagnostics): [0] load+diag0, [1] panels, [2] trailing, [3] backward, [4] diagonal
    // factorizations (summed over waves); accumulated in registers, written once at the end
    unsigned long long tprev = 0, ph_acc[5] = {0, 0, 0, 0, 0}, tel[3] = {0, 0, 0};
    auto stamp = [&](int ph) {
        if (dbg) {
            const unsigned long long t = __builtin_amdgcn_s_memtime();
            if (ph >= 0) ph_acc[ph] += t - tprev;
            tprev = t;
        }
    };
    stamp(-1);
    extern __shared__ __attribute__((aligned(16))) double lds[];
    const int T = (n + 15) >> 4;
    const int noff = T * (T - 1) / 2;          // off-diagonal lower tiles (register-resident)
    const int tid = threadIdx.x;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int lane = tid & 63, cc = lane & 15, rg = lane >> 4;
    double* Lpan = lds;                        // T x 256: panel tiles L_Ik^T, lane-contiguous
    double* Linv = Lpan + (size_t)T * 256;     // T x 256: Linv_k in operand order
    double* Dt = Linv + (size_t)T * 256;       // T x 256: diagonal tiles C_JJ (C layout, lane-contiguous)
    double* y = Dt + (size_t)T * 256;          // 16 T: y, then x in place
    double* dsc = y + 16 * T;                  // diagonal-factorization scratch (24 + 128) + block params (24)
    int* bad = (int*)(dsc + 176);
    // Off-diagonal tile (I > J), column-major index g, lives in slot g / 8 of wave g % 8. (I, J)
    // are walked incrementally in scalar registers: +8 rows, wrapping into the next columns
    // (column J holds rows J+1 .. T-1).
    const int nslots = wid < noff ? (noff - wid + kRegWaves - 1) / kRegWaves : 0;
    int I0 = 1 + wid, J0 = 0;
    while (I0 >= T && J0 < T - 1) { I0 = I0 - T + J0 + 2; J0++; }
    // off(J): off-diagonal tiles in columns < J; slot_at(G): this wave's first slot with g >= G
    auto off = [&](int J) { return J * (T - 1) - J * (J - 1) / 2; };
    auto slot_at = [&](int G) { return min(nslots, G > wid ? (G - wid + kRegWaves - 1) / kRegWaves : 0); };
    // element (a = rg + 4q, b = cc) of C_IJ^T = S[16I + b][16J + a]; inside a 6x6 diagonal block
    // the two triangles are separate sums (read the lower one), elsewhere S is an exact mirror
    // (read the coalesced row c)
    auto s_elem = [&](int I, int J, int q, bool valid) {
        const int r = 16 * I + cc, c = 16 * J + rg + 4 * q;
        const bool in = valid && r < n && c < n;
        const size_t off = !in ? 0 : (r / 6 == c / 6) ? (size_t)max(r, c) * n + min(r, c) : (size_t)c * n + r;
        const double v = S[off];
        return in ? v : (r == c ? 1.0 : 0.0);
    };

    // ---- load: off-diagonal tiles into registers (all loads in flight together), diagonal
    // tiles J = wid (mod 8) into LDS ----
    double4_t acc[MAXT];
    {
        int I = I0, J = J0;
#pragma unroll
        for (int t = 0; t < MAXT; t++) {
#pragma unroll
            for (int q = 0; q < 4; q++) acc[t][q] = s_elem(I, J, q, t < nslots);
            I += kRegWaves;
            while (I >= T && J < T - 1) { I = I - T + J + 2; J++; }
        }
    }
    for (int J = wid; J < T; J += kRegWaves) {
        double* dst = Dt + (size_t)J * 256 + lane * 4;
#pragma unroll
        for (int q = 0; q < 4; q++) dst[q] = s_elem(J, J, q, true);
    }
    for (int i = tid; i < 16 * T; i += blockDim.x) y[i] = i < n ? bs[i] : 0.0;
    if (tid == 0) *bad = 0;
    __syncthreads();

    // C -= L_Jk L_Ik^T on the operands published in Lpan (the tile in C layout, transposed)
    auto tile_update = [&](double4_t& c4, int I, int J) {
        const double* pa = Lpan + (size_t)J * 256 + lane * 4;
        const double* pb = Lpan + (size_t)I * 256 + lane * 4;
        c4 = __builtin_amdgcn_mfma_f64_16x16x4f64(-pa[0], pb[0], c4, 0, 0, 0);
        c4 = __builtin_amdgcn_mfma_f64_16x16x4f64(-pa[1], pb[1], c4, 0, 0, 0);
        c4 = __builtin_amdgcn_mfma_f64_16x16x4f64(-pa[2], pb[2], c4, 0, 0, 0);
        c4 = __builtin_amdgcn_mfma_f64_16x16x4f64(-pa[3], pb[3], c4, 0, 0, 0);
    };
    auto load4 = [&](const double* p) { return double4_t{p[0], p[1], p[2], p[3]}; };
    // y_I -= L_Ik y_k (lane holds L_Ik[cc][rg + 4q] in the published panel tile)
    auto y_update = [&](int I, int k) {
        const double4_t l = load4(Lpan + (size_t)I * 256 + lane * 4);
        double sv = l[0] * y[16 * k + rg] + l[1] * y[16 * k + rg + 4] + l[2] * y[16 * k + rg + 8] +
                    l[3] * y[16 * k + rg + 12];
        sv = col4_sum(sv);
        if (rg == 0) y[16 * I + cc] -= sv;
    };

    // the (I, J) of every slot, walked once (wave-uniform: scalar registers), so that the trailing
    // updates and the backward steps read a slot's tile coordinates instead of re-walking the
    // column-major order
    int rIJ[MAXT];   // I | J << 8 (I = 255: no tile)
    {
        int I = I0, J = J0;
#pragma unroll
        for (int t = 0; t < MAXT; t++) {
            rIJ[t] = (t < nslots ? I : 255) | J << 8;
            I += kRegWaves;
            while (I >= T && J < T - 1) { I = I - T + J + 2; J++; }
        }
    }
    // step k = -1 .. T-2: [panel k] barrier [diag k+1 | diagonal-tile and y updates | trailing k]
    // barrier. The look-ahead wave (k+1) % 8 finishes tile (k+1, k+1) and factors it first.
    for (int k = -1; k < T - 1; k++) {
        if (k >= 0) {
            const double4_t a = load4(Linv + (size_t)k * 256 + lane * 4);
            const int ta = slot_at(off(k)), tb = slot_at(off(k + 1));
            const int Ia = k + 1 + (wid + kRegWaves * ta - off(k));   // row of slot ta (column k)
            run_slots<MAXT>(ta, tb, [&](auto tc) {
                constexpr int t = decltype(tc)::value;   // L_Ik^T = Linv_k A_Ik^T (B operand: own registers)
                const int I = Ia + kRegWaves * (t - ta);
                double4_t r4 = {0, 0, 0, 0};
                r4 = __builtin_amdgcn_mfma_f64_16x16x4f64(a[0], acc[t][0], r4, 0, 0, 0);
                r4 = __builtin_amdgcn_mfma_f64_16x16x4f64(a[1], acc[t][1], r4, 0, 0, 0);
                r4 = __builtin_amdgcn_mfma_f64_16x16x4f64(a[2], acc[t][2], r4, 0, 0, 0);
                r4 = __builtin_amdgcn_mfma_f64_16x16x4f64(a[3], acc[t][3], r4, 0, 0, 0);
                acc[t] = r4;
                double* dst = Lpan + (size_t)I * 256 + lane * 4;
                dst[0] = r4[0]; dst[1] = r4[1]; dst[2] = r4[2]; dst[3] = r4[3];
            });
            __syncthreads();
            stamp(1);
        }
        const int d1 = k + 1;
        if (wid == d1 % kRegWaves) {
            const unsigned long long t0 = dbg ? __builtin_amdgcn_s_memtime() : 0;
            double4_t dt = load4(Dt + (size_t)d1 * 256 + lane * 4);
            if (k >= 0) {
                tile_update(dt, d1, d1);
                y_update(d1, k);
                wave_lds_sync();
            }
            if (dbg) tel[2] += __builtin_amdgcn_s_memtime() - t0;
            diag_tile(dt, Linv + (size_t)d1 * 256, y + 16 * d1, dsc, dsc + 152, bad, dbg ? tel : nullptr);
            if (dbg) ph_acc[4] += __builtin_amdgcn_s_memtime() - t0;
        }
        if (k >= 0) {
            for (int J = d1 + 1 + ((wid - d1 - 1) % kRegWaves + kRegWaves) % kRegWaves; J < T; J += kRegWaves) {
                double4_t c4 = load4(Dt + (size_t)J * 256 + lane * 4);
                tile_update(c4, J, J);
                double* dst = Dt + (size_t)J * 256 + lane * 4;
                dst[0] = c4[0]; dst[1] = c4[1]; dst[2] = c4[2]; dst[3] = c4[3];
                y_update(J, k);
            }
            // slots of columns > k: a suffix of this wave's slots, walked from its first tile
            const int tb = slot_at(off(k + 1));
            run_slots<MAXT>(tb, nslots, [&](auto tc) {
                constexpr int t = decltype(tc)::value;
                tile_update(acc[t], rIJ[t] & 0xFF, rIJ[t] >> 8);
            });
        }
        __syncthreads();
        stamp(k >= 0 ? 2 : 0);
    }
    // ---- backward: x_{T-1} = Linv^T y_{T-1}; then per k: y_J -= L_kJ^T x_k (J < k), and the
    // owner of (k, k-1) (its update of y_{k-1} is the last one) finishes x_{k-1} ----
    if (wid == (T - 1) % kRegWaves) apply_linv_t(Linv + (size_t)(T - 1) * 256, y + 16 * (T - 1));
    __syncthreads();
    for (int k = T - 1; k >= 1; k--) {
        const double xk = y[16 * k + cc];
        bool own = false;
        // tiles (k, J), J < k
        run_slots<MAXT>(0, nslots, [&](auto tc) {
            constexpr int t = decltype(tc)::value;
            if ((rIJ[t] & 0xFF) == k) {
                const int J = rIJ[t] >> 8;
                // lane holds L_kJ[cc][rg + 4q]: (L_kJ^T x_k)[rg + 4q] = sum over cc
                double sq[4];
#pragma unroll
                for (int q = 0; q < 4; q++) sq[q] = row16_sum(acc[t][q] * xk);
                if (cc == 0) {
#pragma unroll
                    for (int q = 0; q < 4; q++) y[16 * J + rg + 4 * q] -= sq[q];
                }
                own |= (J == k - 1);
            }
        });
        if (own) {
            wave_lds_sync();
            apply_linv_t(Linv + (size_t)(k - 1) * 256, y + 16 * (k - 1));
        }
        __syncthreads();
    }
    stamp(3);
    if (dbg && lane == 0) {   // per wave: [8 + 5 w + i]; wave 0's phase totals also in [0..3], diag sum in [4]
        if (wid == 0)
            for (int i = 0; i < 4; i++) dbg[i] = ph_acc[i];
        atomicAdd(&dbg[4], ph_acc[4]);
        atomicAdd(&dbg[5], tel[2]);   // diag wave: tile update + y update before the factorization
        atomicAdd(&dbg[6], tel[0]);   // elimination
        atomicAdd(&dbg[7], tel[1] - tel[0]);   // parameters + Linv + y epilogue
        for (int i = 0; i < 5; i++) dbg[8 + 5 * wid + i] = ph_acc[i];
    }
    const int nb = *bad;
    for (int i = tid; i < n; i += blockDim.x) x[i] = nb ? 0.0 : y[i];
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
    const int T = (n + 15) / 16, nt = T * (T - 1) / 2;
    const int need = (nt + kRegWaves - 1) / kRegWaves;
    return need <= 4 ? 4 : need <= 8 ? 8 : need <= 12 ? 12 : need <= 16 ? 16 : need <= 20 ? 20 : need <= 22 ? 22 : 0;
}

hipError_t chol_reg_launch(int maxN, int nprob, const BaArgs* args, const int* act, hipStream_t st) {
    const int mt = chol_reg_maxt(maxN);
    if (!mt) return hipErrorInvalidValue;
    static bool attr = false;
    if (!attr) {
        for (const void* f : {(const void*)k_ba_chol_reg<4>, (const void*)k_ba_chol_reg<8>,
                              (const void*)k_ba_chol_reg<12>, (const void*)k_ba_chol_reg<16>,
                              (const void*)k_ba_chol_reg<20>, (const void*)k_ba_chol_reg<22>, (const void*)k_chol_reg_probe<4>,
                              (const void*)k_chol_reg_probe<8>, (const void*)k_chol_reg_probe<12>,
                              (const void*)k_chol_reg_probe<16>, (const void*)k_chol_reg_probe<20>,
                              (const void*)k_chol_reg_probe<22>}) {
            hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
            if (e != hipSuccess) return e;
        }
        attr = true;
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
