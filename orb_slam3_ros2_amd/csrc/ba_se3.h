// SE3Quat arithmetic of g2o (Eigen formulas), fp64, shared by the BA solver (ba_solver.hip) and
// the pose-only optimizer (pose_opt.hip). A pose is double[8] = (qx qy qz qw tx ty tz pad).
#pragma once
#include <hip/hip_runtime.h>

#include <type_traits>

namespace orbhip {

struct DQ { double x, y, z, w; };

__device__ __forceinline__ void qrot(const DQ& q, double vx, double vy, double vz, double& ox, double& oy, double& oz) {
    double ux = q.y * vz - q.z * vy, uy = q.z * vx - q.x * vz, uz = q.x * vy - q.y * vx;
    ux += ux; uy += uy; uz += uz;
    const double cx = q.y * uz - q.z * uy, cy = q.z * ux - q.x * uz, cz = q.x * uy - q.y * ux;
    ox = vx + q.w * ux + cx;
    oy = vy + q.w * uy + cy;
    oz = vz + q.w * uz + cz;
}

__device__ __forceinline__ void qtomat(const DQ& q, double R[9]) {
    const double tx = 2 * q.x, ty = 2 * q.y, tz = 2 * q.z;
    const double twx = tx * q.w, twy = ty * q.w, twz = tz * q.w;
    const double txx = tx * q.x, txy = ty * q.x, txz = tz * q.x;
    const double tyy = ty * q.y, tyz = tz * q.y, tzz = tz * q.z;
    R[0] = 1 - (tyy + tzz); R[1] = txy - twz;       R[2] = txz + twy;
    R[3] = txy + twz;       R[4] = 1 - (txx + tzz); R[5] = tyz - twx;
    R[6] = txz - twy;       R[7] = tyz + twx;       R[8] = 1 - (txx + tyy);
}

__device__ __forceinline__ DQ mattoq(const double m[9]) {
    DQ q;
    double t = m[0] + m[4] + m[8];
    if (t > 0) {
        t = sqrt(t + 1.0);
        q.w = 0.5 * t;
        t = 0.5 / t;
        q.x = (m[7] - m[5]) * t;
        q.y = (m[2] - m[6]) * t;
        q.z = (m[3] - m[1]) * t;
    } else {
        int i = 0;
        if (m[4] > m[0]) i = 1;
        if (m[8] > m[3 * i + i]) i = 2;
        // the three cases with static indices (a runtime-indexed c[3] / m[] goes to scratch)
        auto branch = [&](auto I) {
            constexpr int ii = decltype(I)::value, j = (ii + 1) % 3, k = (j + 1) % 3;
            double s = sqrt(m[3 * ii + ii] - m[3 * j + j] - m[3 * k + k] + 1.0);
            double c[3];
            c[ii] = 0.5 * s;
            s = 0.5 / s;
            q.w = (m[3 * k + j] - m[3 * j + k]) * s;
            c[j] = (m[3 * j + ii] + m[3 * ii + j]) * s;
            c[k] = (m[3 * k + ii] + m[3 * ii + k]) * s;
            q.x = c[0]; q.y = c[1]; q.z = c[2];
        };
        if (i == 0) branch(std::integral_constant<int, 0>{});
        else if (i == 1) branch(std::integral_constant<int, 1>{});
        else branch(std::integral_constant<int, 2>{});
    }
    return q;
}

__device__ __forceinline__ void qnormalize(DQ& q) {
    if (q.w < 0) { q.x = -q.x; q.y = -q.y; q.z = -q.z; q.w = -q.w; }
    const double in = 1.0 / sqrt(q.x * q.x + q.y * q.y + q.z * q.z + q.w * q.w);
    q.x *= in; q.y *= in; q.z *= in; q.w *= in;
}

__device__ __forceinline__ DQ load_q(const double* p) { return DQ{p[0], p[1], p[2], p[3]}; }



// VertexSE3Expmap::oplusImpl: T <- SE3Quat::exp(u) * T, u = [omega; upsilon]
__device__ __forceinline__ void se3_update(const double* u, double* T) {
    const double ox = u[0], oy = u[1], oz = u[2];
    const double theta = sqrt(ox * ox + oy * oy + oz * oz);
    const double O[9] = {0, -oz, oy, oz, 0, -ox, -oy, ox, 0};
    double O2[9];
#pragma unroll
    for (int r = 0; r < 3; r++)
#pragma unroll
        for (int c = 0; c < 3; c++) O2[3 * r + c] = O[3 * r] * O[c] + O[3 * r + 1] * O[3 + c] + O[3 * r + 2] * O[6 + c];
    double R[9], V[9];
    if (theta < 0.00001) {
#pragma unroll
        for (int i = 0; i < 9; i++) { R[i] = (i % 4 == 0 ? 1.0 : 0.0) + O[i] + O2[i]; V[i] = R[i]; }
    } else {
        double st, ct;
        sincos(theta, &st, &ct);
        const double it = 1.0 / theta, it2 = it * it;
        const double sa = st * it, cb = (1 - ct) * it2, cc = (theta - st) * it2 * it;
#pragma unroll
        for (int i = 0; i < 9; i++) {
            R[i] = (i % 4 == 0 ? 1.0 : 0.0) + sa * O[i] + cb * O2[i];
            V[i] = (i % 4 == 0 ? 1.0 : 0.0) + cb * O[i] + cc * O2[i];
        }
    }
    DQ qe = mattoq(R);
    qnormalize(qe);
    const double tex = V[0] * u[3] + V[1] * u[4] + V[2] * u[5];
    const double tey = V[3] * u[3] + V[4] * u[4] + V[5] * u[5];
    const double tez = V[6] * u[3] + V[7] * u[4] + V[8] * u[5];
    const DQ qt = load_q(T);
    double rx, ry, rz;
    qrot(qe, T[4], T[5], T[6], rx, ry, rz);
    DQ q{qe.w * qt.x + qe.x * qt.w + qe.y * qt.z - qe.z * qt.y, qe.w * qt.y + qe.y * qt.w + qe.z * qt.x - qe.x * qt.z,
         qe.w * qt.z + qe.z * qt.w + qe.x * qt.y - qe.y * qt.x, qe.w * qt.w - qe.x * qt.x - qe.y * qt.y - qe.z * qt.z};
    qnormalize(q);
    T[0] = q.x; T[1] = q.y; T[2] = q.z; T[3] = q.w;
    T[4] = tex + rx; T[5] = tey + ry; T[6] = tez + rz;
}

}  // namespace orbhip
