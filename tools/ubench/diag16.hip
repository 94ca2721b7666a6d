// Microbenchmark + check of diag16_linv (csrc/ba_diag16.h): one wave factors a 16x16 SPD tile into
// the inverse of its Cholesky factor. Prints the max relative error against a long-double host
// reference over well- and ill-conditioned tiles, and the s_memtime cycles of the routine.
//   hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -I../../orb_slam3_ros2_amd/csrc diag16.hip -o diag16
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <random>
#include <vector>

#include "ba_diag16.h"

using namespace orbhip;

__global__ __launch_bounds__(64) void k_diag16(const double* __restrict__ A, double* __restrict__ Linv,
                                               unsigned long long* cyc, int* okf) {
    const int lane = threadIdx.x, cc = lane & 15, rg = lane >> 4;
    const double* a = A + (size_t)blockIdx.x * 256;
    double* L = Linv + (size_t)blockIdx.x * 256;
    double4_t d;
#pragma unroll
    for (int q = 0; q < 4; q++) d[q] = a[(rg + 4 * q) * 16 + cc];
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_sched_barrier(0);
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    double lv[4];
    const bool ok = diag16_linv(d, [&](int r, int c, double v) { lv[r >> 2] = v; });
    __builtin_amdgcn_sched_barrier(0);
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
#pragma unroll
    for (int q = 0; q < 4; q++) L[(rg + 4 * q) * 16 + cc] = lv[q];
    if (lane == 0) {
        cyc[blockIdx.x] = t1 - t0;
        okf[blockIdx.x] = ok;
    }
}

__global__ __launch_bounds__(64) void k_diag16_loop(const double* __restrict__ A, double* __restrict__ Linv, int reps) {
    const int lane = threadIdx.x, cc = lane & 15, rg = lane >> 4;
    double4_t d;
#pragma unroll
    for (int q = 0; q < 4; q++) d[q] = A[(rg + 4 * q) * 16 + cc];
    double lv[4] = {0, 0, 0, 0};
    for (int r = 0; r < reps; r++) {
        double4_t dd;
#pragma unroll
        for (int q = 0; q < 4; q++) dd[q] = fma(0.0, lv[q], d[q]);   // a dependency on the previous result
        diag16_linv(dd, [&](int rr, int c, double v) { lv[rr >> 2] = v; });
    }
#pragma unroll
    for (int q = 0; q < 4; q++) Linv[(rg + 4 * q) * 16 + cc] = lv[q];
}

// the DPP column elimination (diag16_dpp): lane c holds column c, Linv comes in the C layout
__global__ __launch_bounds__(64) void k_dpp16(const double* __restrict__ A, double* __restrict__ Linv, int* okf) {
    const int lane = threadIdx.x, c = lane & 15, rg = lane >> 4;
    const double* a = A + (size_t)blockIdx.x * 256;
    double* L = Linv + (size_t)blockIdx.x * 256;
    __shared__ double scr[272];
    double v[16];
    double4_t lv;
#pragma unroll
    for (int i = 0; i < 16; i++) v[i] = a[i * 16 + c];
    const bool ok = diag16_dpp(v, scr, lv);
#pragma unroll
    for (int q = 0; q < 4; q++) L[(rg + 4 * q) * 16 + c] = lv[q];
    if (lane == 0) okf[blockIdx.x] = ok;
}
__global__ __launch_bounds__(64) void k_dpp16_loop(const double* __restrict__ A, double* __restrict__ Linv, int reps) {
    const int lane = threadIdx.x, c = lane & 15, rg = lane >> 4;
    __shared__ double scr[272];
    double v0[16];
    double4_t lv = {0, 0, 0, 0};
#pragma unroll
    for (int i = 0; i < 16; i++) v0[i] = A[i * 16 + c];
    for (int r = 0; r < reps; r++) {
        double v[16];
        const double z = lv[0] + lv[1] + lv[2] + lv[3];
#pragma unroll
        for (int i = 0; i < 16; i++) v[i] = fma(0.0, z, v0[i]);   // a dependency on the previous result
        diag16_dpp(v, scr, lv);
    }
#pragma unroll
    for (int q = 0; q < 4; q++) Linv[(rg + 4 * q) * 16 + c] = lv[q];
}

static void ref_linv(const double* A, double* Li) {
    long double L[16][16] = {}, X[16][16] = {};
    for (int j = 0; j < 16; j++) {
        long double s = A[j * 16 + j];
        for (int k = 0; k < j; k++) s -= L[j][k] * L[j][k];
        L[j][j] = sqrtl(s);
        for (int i = j + 1; i < 16; i++) {
            long double t = A[i * 16 + j];
            for (int k = 0; k < j; k++) t -= L[i][k] * L[j][k];
            L[i][j] = t / L[j][j];
        }
    }
    for (int c = 0; c < 16; c++)
        for (int r = 0; r < 16; r++) {
            long double t = r == c ? 1.0L : 0.0L;
            for (int k = 0; k < r; k++) t -= L[r][k] * X[k][c];
            X[r][c] = t / L[r][r];
        }
    for (int i = 0; i < 256; i++) Li[i] = (double)X[i / 16][i % 16];
}

int main() {
    const int NB = 64;
    std::mt19937_64 rng(7);
    std::normal_distribution<double> nd;
    std::vector<double> A(NB * 256), Lg(NB * 256), Lr(NB * 256);
    for (int b = 0; b < NB; b++) {
        double M[16][16];
        for (auto& r : M)
            for (auto& v : r) v = nd(rng);
        // condition: 1e0 .. 1e-(b % 12) spread on the diagonal of M M^T + eps I
        const double eps = std::pow(10.0, -(double)(b % 12));
        for (int i = 0; i < 16; i++)
            for (int j = 0; j < 16; j++) {
                double s = 0;
                for (int k = 0; k < 16; k++) s += M[i][k] * M[j][k] * (k < 8 ? 1.0 : eps);
                A[b * 256 + i * 16 + j] = s + (i == j ? eps : 0.0);
            }
        ref_linv(&A[b * 256], &Lr[b * 256]);
    }
    double *dA, *dL;
    unsigned long long* dc;
    int* dok;
    hipMalloc(&dA, sizeof(double) * A.size());
    hipMalloc(&dL, sizeof(double) * A.size());
    hipMalloc(&dc, sizeof(unsigned long long) * NB);
    hipMalloc(&dok, sizeof(int) * NB);
    hipMemcpy(dA, A.data(), sizeof(double) * A.size(), hipMemcpyHostToDevice);
    for (int it = 0; it < 3; it++) hipLaunchKernelGGL(k_diag16, dim3(NB), dim3(64), 0, nullptr, dA, dL, dc, dok);
    hipDeviceSynchronize();
    std::vector<unsigned long long> cyc(NB);
    std::vector<int> ok(NB);
    hipMemcpy(Lg.data(), dL, sizeof(double) * A.size(), hipMemcpyDeviceToHost);
    hipMemcpy(cyc.data(), dc, sizeof(unsigned long long) * NB, hipMemcpyDeviceToHost);
    hipMemcpy(ok.data(), dok, sizeof(int) * NB, hipMemcpyDeviceToHost);
    double worst = 0;
    unsigned long long cmin = ~0ull, cmax = 0, csum = 0;
    int nok = 0;
    for (int b = 0; b < NB; b++) {
        double num = 0, den = 0;
        for (int i = 0; i < 256; i++) {
            num = std::fmax(num, std::fabs(Lg[b * 256 + i] - Lr[b * 256 + i]));
            den = std::fmax(den, std::fabs(Lr[b * 256 + i]));
        }
        worst = std::fmax(worst, num / den);
        cmin = std::min(cmin, cyc[b]); cmax = std::max(cmax, cyc[b]); csum += cyc[b];
        nok += ok[b];
    }
    printf("diag16: %d/%d pd, max rel err %.3e, cycles min %llu avg %llu max %llu\n", nok, NB, worst, cmin, csum / NB, cmax);
    for (int b = 0; b < 12; b++) {
        double num = 0, den = 0;
        int wi = 0;
        for (int i = 0; i < 256; i++) {
            const double e = std::fabs(Lg[b * 256 + i] - Lr[b * 256 + i]);
            if (e > num) { num = e; wi = i; }
            den = std::fmax(den, std::fabs(Lr[b * 256 + i]));
        }
        // quality of the inverse factor: max |Linv A Linv^T - I| (GPU, and a plain fp64 host Cholesky)
        auto resid = [&](const double* Li) {
            double worst_r = 0;
            for (int i = 0; i < 16; i++)
                for (int j = 0; j < 16; j++) {
                    long double t = 0;
                    for (int k = 0; k < 16; k++)
                        for (int l = 0; l < 16; l++) t += (long double)Li[i * 16 + k] * A[b * 256 + k * 16 + l] * Li[j * 16 + l];
                    worst_r = std::fmax(worst_r, std::fabs((double)(t - (i == j ? 1.0L : 0.0L))));
                }
            return worst_r;
        };
        double Lf[256];
        {
            double L[16][16] = {}, X[16][16] = {};
            const double* Ab = &A[b * 256];
            for (int j = 0; j < 16; j++) {
                double sj = Ab[j * 16 + j];
                for (int k = 0; k < j; k++) sj -= L[j][k] * L[j][k];
                L[j][j] = std::sqrt(sj);
                for (int i = j + 1; i < 16; i++) {
                    double t = Ab[i * 16 + j];
                    for (int k = 0; k < j; k++) t -= L[i][k] * L[j][k];
                    L[i][j] = t / L[j][j];
                }
            }
            for (int c = 0; c < 16; c++)
                for (int r = 0; r < 16; r++) {
                    double t = r == c ? 1.0 : 0.0;
                    for (int k = 0; k < r; k++) t -= L[r][k] * X[k][c];
                    X[r][c] = t / L[r][r];
                }
            for (int i = 0; i < 256; i++) Lf[i] = X[i / 16][i % 16];
        }
        double numf = 0;
        for (int i = 0; i < 256; i++) numf = std::fmax(numf, std::fabs(Lf[i] - Lr[b * 256 + i]));
        printf("  tile %d (eps 1e-%d): rel err %.3e (host fp64 %.3e) at (%d,%d); |Linv A Linv^T - I| gpu %.2e host fp64 %.2e\n",
               b, b % 12, num / den, numf / den, wi / 16, wi % 16, resid(&Lg[b * 256]), resid(Lf));
    }
    // timing: R dependent factorizations in one wave
    {
        hipEvent_t e0, e1;
        hipEventCreate(&e0); hipEventCreate(&e1);
        hipLaunchKernelGGL(k_diag16_loop, dim3(1), dim3(64), 0, nullptr, dA, dL, 10);
        hipEventRecord(e0, nullptr);
        hipLaunchKernelGGL(k_diag16_loop, dim3(1), dim3(64), 0, nullptr, dA, dL, 1000);
        hipEventRecord(e1, nullptr);
        hipEventSynchronize(e1);
        float ms1 = 0;
        hipEventElapsedTime(&ms1, e0, e1);
        hipEventRecord(e0, nullptr);
        hipLaunchKernelGGL(k_diag16_loop, dim3(1), dim3(64), 0, nullptr, dA, dL, 11000);
        hipEventRecord(e1, nullptr);
        hipEventSynchronize(e1);
        float ms2 = 0;
        hipEventElapsedTime(&ms2, e0, e1);
        printf("diag16 chain: %.3f us per factorization (1000: %.3f ms, 11000: %.3f ms)\n", (ms2 - ms1) * 1e3 / 10000, ms1, ms2);
    }
    // the DPP forms: accuracy against the long-double reference and the dependent-chain time
    auto check = [&](const char* nm, void (*kone)(const double*, double*, int*), void (*kloop)(const double*, double*, int)) -> bool {
        hipLaunchKernelGGL(kone, dim3(NB), dim3(64), 0, nullptr, dA, dL, dok);
        hipDeviceSynchronize();
        hipMemcpy(Lg.data(), dL, sizeof(double) * A.size(), hipMemcpyDeviceToHost);
        hipMemcpy(ok.data(), dok, sizeof(int) * NB, hipMemcpyDeviceToHost);
        double w2 = 0;
        int nok2 = 0;
        for (int b = 0; b < NB; b++) {
            double num = 0, den = 0;
            for (int i = 0; i < 256; i++) {
                num = std::fmax(num, std::fabs(Lg[b * 256 + i] - Lr[b * 256 + i]));
                den = std::fmax(den, std::fabs(Lr[b * 256 + i]));
            }
            w2 = std::fmax(w2, num / den);
            nok2 += ok[b];
            if (b < 12) printf("  %s tile %d (eps 1e-%d): rel err %.3e\n", nm, b, b % 12, num / den);
        }
        printf("%s: %d/%d pd, max rel err %.3e\n", nm, nok2, NB, w2);
        std::vector<double> Bn(A.begin(), A.begin() + 256);
        Bn[5 * 16 + 5] = -1.0;
        hipMemcpy(dA, Bn.data(), sizeof(double) * 256, hipMemcpyHostToDevice);
        hipLaunchKernelGGL(kone, dim3(1), dim3(64), 0, nullptr, dA, dL, dok);
        int okn = 1;
        hipMemcpy(&okn, dok, sizeof(int), hipMemcpyDeviceToHost);
        printf("%s non-PD tile reported: %s\n", nm, okn ? "NO" : "yes");
        hipMemcpy(dA, A.data(), sizeof(double) * A.size(), hipMemcpyHostToDevice);
        hipEvent_t e0, e1;
        hipEventCreate(&e0); hipEventCreate(&e1);
        hipLaunchKernelGGL(kloop, dim3(1), dim3(64), 0, nullptr, dA, dL, 10);
        hipEventRecord(e0, nullptr);
        hipLaunchKernelGGL(kloop, dim3(1), dim3(64), 0, nullptr, dA, dL, 1000);
        hipEventRecord(e1, nullptr);
        hipEventSynchronize(e1);
        float ms1 = 0;
        hipEventElapsedTime(&ms1, e0, e1);
        hipEventRecord(e0, nullptr);
        hipLaunchKernelGGL(kloop, dim3(1), dim3(64), 0, nullptr, dA, dL, 11000);
        hipEventRecord(e1, nullptr);
        hipEventSynchronize(e1);
        float ms2 = 0;
        hipEventElapsedTime(&ms2, e0, e1);
        printf("%s chain: %.3f us per factorization\n", nm, (ms2 - ms1) * 1e3 / 10000);
        return !okn && nok2 == NB && w2 <= 1e-6;
    };
    if (!check("dpp16", k_dpp16, k_dpp16_loop)) return 1;
    return worst < 1e-6 && nok == NB ? 0 : 1;
}
