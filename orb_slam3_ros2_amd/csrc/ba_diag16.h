// One-wave factorization of a 16x16 SPD tile into the inverse of its Cholesky factor (a20: the
// diagonal-tile step of the dense reduced-camera-system Cholesky, g2o LinearSolverEigen behind
// OptimizationAlgorithmLevenberg). Shared by the register-resident solver (ba_chol_reg.hip) and
// the blocked solver (ba_chol_blocked.hip).
//
// Block LDL^T with 4x4 pivot blocks, every rank-4 step on v_mfma_f64_16x16x4f64:
//   D = L~ Dg L~^T (L~ unit block-lower, Dg = blockdiag(B_p)), B_p = C_p C_p^T (4x4 Cholesky),
//   so L = L~ C and Linv = L^-1 = C^-1 X with X = L~^-1 from the Gaussian elimination of [D | I].
// Pivot step p (rows J = 4p .. J+3), with the tile in the MFMA C layout (lane l = cc + 16 rg holds
// D[rg + 4q][cc] in component q):
//   - the 10 entries of B_p come by readlane (component p of lanes (J+b) + 16a); C_p^-1 is
//     computed in every lane (4x4 Cholesky, rsq + Newton steps, forward substitution);
//   - rows J..J+3 of D are component p of every lane, which IS the B operand R (lane (cc, k):
//     R[k][cc]); a 4x16 operand built from C_p^-1 goes in as A (rows 4..15 zero):
//       Y  = C^-1 R           (MFMA 1)        -> component 0 is again a B operand (Y[rg][cc])
//       M^T = C^-T Y = B^-1 R (MFMA 2)        -> lane (cc, rg) holds M[cc][rg] = an A operand
//       D -= M R, X -= M X_p  (MFMAs 3, 4; M masked to the rows below the pivot block)
//       Linv[J..J+3] = C^-1 X_p (MFMA 5; rows J..J+3 of X are final once step p starts)
// Four dependent pivot steps instead of sixteen column steps, no LDS round trip inside a step.
// The entries of D left of the trailing block are not masked: they only feed other such entries,
// never a later pivot block, Y's used columns or X.
#pragma once
#include <hip/hip_runtime.h>

#include "ba_chol.h"
#include "ba_dpp16.h"
#include "ba_dpp16f.h"

#ifndef ORBHIP_DPP16_FUSED
#define ORBHIP_DPP16_FUSED 1
#endif

namespace orbhip {

template <int NR = 2>
__device__ __forceinline__ double rsq_nr(double a) {   // 1/sqrt(a): rsq + NR Newton steps
    double s = __builtin_amdgcn_rsq(a);
#pragma unroll
    for (int i = 0; i < NR; i++) s = s * fma(-0.5 * a * s, s, 1.5);
    return s;
}

// Factor the tile d (C layout, both triangles) of one wave: writes Linv row by row through
// store(r, c, v) (r = J + rg, c = cc: lane (cc, rg) stores Linv[J + rg][cc] once per pivot step,
// every lane every step) and returns false in every lane on a non-positive-definite pivot block.
template <int NR = 2, typename Store>
__device__ __forceinline__ bool diag16_linv(double4_t d, Store&& store) {
    const int lane = threadIdx.x & 63, cc = lane & 15, rg = lane >> 4;
    double4_t xv;
#pragma unroll
    for (int q = 0; q < 4; q++) xv[q] = (rg + 4 * q == cc) ? 1.0 : 0.0;
    // operand-selection index of this lane: entry (max(cc,rg), min(cc,rg)) of a lower 4x4
    const int mi = cc > rg ? cc : rg, ni = cc > rg ? rg : cc;
    const int sel = mi * (mi + 1) / 2 + ni;   // 0..9 for cc < 4
    const bool a1 = cc < 4 && rg <= cc;       // A1[cc][rg] = Ci[cc][rg]
    const bool a2 = cc < 4 && cc <= rg;       // A2[cc][rg] = Ci[rg][cc]
    bool ok = true;
#pragma unroll
    for (int p = 0; p < 4; p++) {
        const int J = 4 * p;
        // pivot block B[a][b] = D[J+a][J+b] (a >= b): component p of lane (J + b) + 16 a
        const double b00 = readlane_f64(d[p], J + 0), b10 = readlane_f64(d[p], J + 16), b20 = readlane_f64(d[p], J + 32),
                     b30 = readlane_f64(d[p], J + 48), b11 = readlane_f64(d[p], J + 17), b21 = readlane_f64(d[p], J + 33),
                     b31 = readlane_f64(d[p], J + 49), b22 = readlane_f64(d[p], J + 34), b32 = readlane_f64(d[p], J + 50),
                     b33 = readlane_f64(d[p], J + 51);
        // C = chol(B), r_i = 1 / C_ii
        ok = ok && b00 > 0.0;
        const double r0 = rsq_nr<NR>(b00 > 0.0 ? b00 : 1.0);
        const double l10 = b10 * r0, l20 = b20 * r0, l30 = b30 * r0;
        const double s11 = fma(-l10, l10, b11);
        ok = ok && s11 > 0.0;
        const double r1 = rsq_nr<NR>(s11 > 0.0 ? s11 : 1.0);
        const double t21 = fma(-l20, l10, b21), t31 = fma(-l30, l10, b31);
        const double u22 = fma(-l20, l20, b22), u32 = fma(-l30, l20, b32), u33 = fma(-l30, l30, b33);
        const double l21 = t21 * r1, l31 = t31 * r1;
        const double s22 = fma(-l21, l21, u22);
        ok = ok && s22 > 0.0;
        const double r2 = rsq_nr<NR>(s22 > 0.0 ? s22 : 1.0);
        const double v33 = fma(-l31, l31, u33);
        const double l32 = fma(-l31, l21, u32) * r2;
        const double s33 = fma(-l32, l32, v33);
        ok = ok && s33 > 0.0;
        const double r3 = rsq_nr<NR>(s33 > 0.0 ? s33 : 1.0);
        // Ci = C^-1 (lower): Ci_ii = r_i, Ci_ij = -r_i sum_{j<=k<i} l_ik Ci_kj
        const double c10 = -r1 * (l10 * r0);
        const double c21 = -r2 * (l21 * r1);
        const double c20 = -r2 * fma(l21, c10, l20 * r0);
        const double c32 = -r3 * (l32 * r2);
        const double c31 = -r3 * fma(l32, c21, l31 * r1);
        const double c30 = -r3 * fma(l32, c20, fma(l31, c10, l30 * r0));
        // this lane's entry (sel) of Ci
        double e = r0;
        e = sel == 1 ? c10 : e;
        e = sel == 2 ? r1 : e;
        e = sel == 3 ? c20 : e;
        e = sel == 4 ? c21 : e;
        e = sel == 5 ? r2 : e;
        e = sel == 6 ? c30 : e;
        e = sel == 7 ? c31 : e;
        e = sel == 8 ? c32 : e;
        e = sel == 9 ? r3 : e;
        const double A1 = a1 ? e : 0.0, A2 = a2 ? e : 0.0;
        const double4_t z = {0.0, 0.0, 0.0, 0.0};
        // Linv rows J..J+3 (X rows J..J+3 are final)
        const double4_t lr = __builtin_amdgcn_mfma_f64_16x16x4f64(A1, xv[p], z, 0, 0, 0);
        store(J + rg, cc, lr[0]);
        if (p == 3) break;
        const double4_t y = __builtin_amdgcn_mfma_f64_16x16x4f64(A1, d[p], z, 0, 0, 0);
        const double4_t mt = __builtin_amdgcn_mfma_f64_16x16x4f64(A2, y[0], z, 0, 0, 0);
        const double mneg = cc > J + 3 ? -mt[0] : 0.0;   // -M[cc][rg], rows below the pivot block
        const double rp = d[p], xp = xv[p];
        d = __builtin_amdgcn_mfma_f64_16x16x4f64(mneg, rp, d, 0, 0, 0);
        xv = __builtin_amdgcn_mfma_f64_16x16x4f64(mneg, xp, xv, 0, 0, 0);
    }
    return ok;
}

// ---------------------------------------------------------------------------------------------
// DPP column elimination (r05): the same Linv of a 16x16 SPD tile with no MFMA and no readlane on
// its critical path. Lane c (= lane & 15, every 16-lane row holds the same copy) keeps column c
// of the tile in v[0..15]. Step j eliminates column j from rows j+1..15 (row ops on [D | I], the
// LDL^T of D): row i -= m_ij row j, m_ij = D[i][j] / d_j, where D[i][j] is lane j's v[i], read by
// v_fmac_f64_dpp row_newbcast:j as part of the update itself (one instruction per row and step).
// A lane's column is a column of D until its own step and a column of X = L~^-1 after it: at step
// j lane j keeps D's column j, which is -d_j times X's column j (X[i][j] = -m_ij, and later row ops
// act linearly on it), and every lane's multiplier operand is its own row-j entry, so D columns
// (c > j) and X columns (c < j) take the same update. At the end Linv = Dg^-1/2 X:
//   Linv[i][c] = -v[i] s_i / d_c (i > c),  s_c (i = c),  0 (i < c),  s_i = 1/sqrt(d_i).
// Critical path per step: the pivot broadcast, v_rcp_f64 + Newton, one multiply and the update of
// row j+1; the other rows' updates (rest()) fill the reciprocal's latency.
// ---------------------------------------------------------------------------------------------
template <int J>
__device__ __forceinline__ double bcast16(double v) {   // lane J of this lane's 16-lane row
    double r;
    asm("s_nop 1\n\tv_mov_b64_dpp %0, %1 row_newbcast:%2 row_mask:0xf bank_mask:0xf" : "=v"(r) : "v"(v), "n"(J));
    return r;
}
template <int NR = 1>
__device__ __forceinline__ double rcp_nr(double a) {   // 1/a: v_rcp_f64 + NR Newton steps
    double r = __builtin_amdgcn_rcp(a);
#pragma unroll
    for (int i = 0; i < NR; i++) r = fma(r, fma(-a, r, 1.0), r);
    return r;
}
// in lane J of each 16-lane row (and only there): t = 0, pown = piv. One opaque asm block per step:
// as plain selects, the compiler hoisted the 16 loop-invariant lane masks (32 SGPRs) out of the
// solve loop and spilled them. (Lane J cannot be left out by EXEC instead: it is the DPP source.)
template <int J>
__device__ __forceinline__ void lane_j_pick(double& t, double& pown, double piv, int c) {
    const unsigned long long tb = __builtin_bit_cast(unsigned long long, t), pb = __builtin_bit_cast(unsigned long long, pown),
                             vb = __builtin_bit_cast(unsigned long long, piv);
    unsigned tl = (unsigned)tb, th = (unsigned)(tb >> 32), pl = (unsigned)pb, ph = (unsigned)(pb >> 32);
    unsigned long long m;
    asm("v_cmp_eq_u32 %[m], %[j], %[c]\n\t"
        "v_cndmask_b32 %[tl], %[tl], 0, %[m]\n\t"
        "v_cndmask_b32 %[th], %[th], 0, %[m]\n\t"
        "v_cndmask_b32 %[pl], %[pl], %[vl], %[m]\n\t"
        "v_cndmask_b32 %[ph], %[ph], %[vh], %[m]"
        : [tl] "+v"(tl), [th] "+v"(th), [pl] "+v"(pl), [ph] "+v"(ph), [m] "=&s"(m)
        : [vl] "v"((unsigned)vb), [vh] "v"((unsigned)(vb >> 32)), [c] "v"(c), [j] "n"(J));
    t = __builtin_bit_cast(double, (unsigned long long)th << 32 | tl);
    pown = __builtin_bit_cast(double, (unsigned long long)ph << 32 | pl);
}
template <int J, int NR>
__device__ __forceinline__ void dpp16_step(double (&v)[16], double& pown, int c) {
    if constexpr (J < 16) {
        const double piv = bcast16<J>(v[J]);
        const double r = rcp_nr<NR>(piv);
        double t = -v[J] * r;
        lane_j_pick<J>(t, pown, piv, c);   // lane J: t = 0 (its column stays), pown = its pivot
        Dpp16Step<J>::first(v, t);
        Dpp16Step<J>::rest(v, t);
        dpp16_step<J + 1, NR>(v, pown, c);
    }
}
// v: column lane & 15 of the tile (rows 0..15, every 16-lane row the same); lv: Linv in the MFMA C
// layout (lane (c, g), component q: Linv[g + 4q][c]). False in every lane on a non-positive (or
// NaN) pivot. The raw columns go through scr (272 doubles of LDS, this wave's) into the C layout,
// where each lane scales its four rows: selecting register g + 4q per lane in registers made the
// compiler index the column array, i.e. put it in scratch memory.
// Fused form (r05, ORBHIP_DPP16_FUSED, one Newton step only): one asm block per step from
// tools/gen_dpp16.py (ba_dpp16f.h) issues the next pivot's reciprocal, Newton step and multiplier
// between the current step's row updates instead of after all of them, and broadcasts the pivot
// inside v_rcp_f64_dpp / v_fmac_f64_dpp; lane p's zero multiplier and own pivot come from bit p
// of a one-hot column mask. Critical path per step: row update -> rcp -> e -> multiplier.
template <int J>
__device__ __forceinline__ void dpp16f_steps(double (&v)[16], double t, double& pown, unsigned oh, unsigned nh) {
    if constexpr (J < 15) {
        double tn;
        Dpp16F<J>::step(v, t, tn, pown, oh, nh);
        dpp16f_steps<J + 1>(v, tn, pown, oh, nh);
    }
}
template <int NR = 1>
__device__ __forceinline__ bool diag16_dpp(double (&v)[16], double* __restrict__ scr, double4_t& lv) {
    const int lane = threadIdx.x & 63, c = lane & 15, g = lane >> 4;
#if ORBHIP_DPP16_FUSED
    double pown;
    if constexpr (NR == 1) {
        pown = 0.0;
        const unsigned oh = 1u << c;
        dpp16f_steps<-1>(v, 0.0, pown, oh, ~oh);
    } else {
        pown = 1.0;
        dpp16_step<0, NR>(v, pown, c);
    }
#else
    double pown = 1.0;
    dpp16_step<0, NR>(v, pown, c);
#endif
    const bool bad = __any(!(pown > 0.0));
    const double rown = rcp_nr<NR>(pown), sown = rsq_nr<NR>(pown);
    if (g == 0) {
#pragma unroll
        for (int i = 0; i < 16; i++) scr[16 * i + c] = v[i];
        scr[256 + c] = sown;
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    const double nr = -rown;
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const int i = g + 4 * q;
        const double x = scr[16 * i + c], si = scr[256 + i];
        const double p = x * nr * si;
        double o = i == c ? sown : 0.0;
        o = i > c ? p : o;
        lv[q] = o;
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    return !bad;
}

// One wave: the 32x32 SPD block read by elem(r, c) (r >= c, both < 32; the caller pads) into Linv
// (32x32, the inverse of its Cholesky factor) as 2x2 tiles of 16: Linv11 = diag16(D11), L21 =
// D21 Linv11^T, D22 -= L21 L21^T, Linv22 = diag16(D22), Linv21 = -Linv22 L21 Linv11 (MFMA).
// store(r, c, v) receives every entry of Linv once (the zero upper blocks included); scratch: 512
// doubles of LDS. Returns false on a non-positive-definite pivot block.
template <int NR = 2, typename Elem, typename Store>
__device__ __forceinline__ bool diag32_linv(Elem&& elem, double* __restrict__ scratch, Store&& store) {
    const int lane = threadIdx.x & 63, cc = lane & 15, rg = lane >> 4;
    double4_t d11, d21t, d22;
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const int r = rg + 4 * q;
        d11[q] = r >= cc ? elem(r, cc) : elem(cc, r);
        d21t[q] = elem(16 + cc, r);   // D21^T in the C layout: lane holds D21[cc][rg + 4q]
        d22[q] = r >= cc ? elem(16 + r, 16 + cc) : elem(16 + cc, 16 + r);
    }
    double* op11 = scratch;         // Linv11, operand order
    double* op22 = scratch + 256;   // Linv22, operand order
    double4_t lin11;                // Linv11 in the C layout
    const bool ok1 = diag16_linv<NR>(d11, [&](int r, int c, double v) {
        op11[(r + 16 * (c & 3)) * 4 + (c >> 2)] = v;
        lin11[r >> 2] = v;
        store(r, c, v);
        store(r, 16 + c, 0.0);
    });
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    const double* a11 = op11 + lane * 4;
    double4_t l21t = {0, 0, 0, 0};   // L21^T = Linv11 D21^T (C layout)
#pragma unroll
    for (int kk = 0; kk < 4; kk++) l21t = __builtin_amdgcn_mfma_f64_16x16x4f64(a11[kk], d21t[kk], l21t, 0, 0, 0);
#pragma unroll
    for (int kk = 0; kk < 4; kk++) d22 = __builtin_amdgcn_mfma_f64_16x16x4f64(-l21t[kk], l21t[kk], d22, 0, 0, 0);
    const bool ok2 = diag16_linv<NR>(d22, [&](int r, int c, double v) {
        op22[(r + 16 * (c & 3)) * 4 + (c >> 2)] = v;
        store(16 + r, 16 + c, v);
    });
    // W = L21 Linv11 (A: L21 from its transposed C layout, B: Linv11 in the C layout)
    double4_t w = {0, 0, 0, 0};
#pragma unroll
    for (int kk = 0; kk < 4; kk++) w = __builtin_amdgcn_mfma_f64_16x16x4f64(l21t[kk], lin11[kk], w, 0, 0, 0);
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    const double* a22 = op22 + lane * 4;
    double4_t l21i = {0, 0, 0, 0};   // Linv21 = -Linv22 W (C layout)
#pragma unroll
    for (int kk = 0; kk < 4; kk++) l21i = __builtin_amdgcn_mfma_f64_16x16x4f64(-a22[kk], w[kk], l21i, 0, 0, 0);
#pragma unroll
    for (int q = 0; q < 4; q++) store(16 + rg + 4 * q, cc, l21i[q]);
    return ok1 && ok2;
}

}  // namespace orbhip
