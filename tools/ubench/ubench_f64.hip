// Micro-benchmarks (shader-clock cycles from s_memtime, one wave unless noted) for the fp64
// pieces of the register-resident Cholesky: MFMA f64 chains, DPP / permlane exchanges, fp64
// division, LDS round trips and workgroup barriers.  hipcc --offload-arch=gfx950 -O3
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double d4 __attribute__((ext_vector_type(4)));
#define N 64
__global__ void k(double* out, unsigned long long* cyc, double a, double b) {
    extern __shared__ double lds[];
    const int lane = threadIdx.x & 63;
    d4 c0 = {a, a, a, a}, c1 = c0, c2 = c0, c3 = c0;
    double av = a + lane, bv = b - lane;
    unsigned long long t0, t1;
    __syncthreads();
    // 1: dependent MFMA chain
    t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < N; i++) c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, c0, 0, 0, 0);
    __builtin_amdgcn_s_waitcnt(0);
    out[0] += c0[0];
    t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) cyc[0] = (t1 - t0);
    // 2: 4 independent chains
    t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < N / 4; i++) {
        c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, c1, 0, 0, 0);
        c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, c2, 0, 0, 0);
        c3 = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, c3, 0, 0, 0);
    }
    out[1] += c0[1] + c1[1] + c2[1] + c3[1];
    t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) cyc[1] = (t1 - t0);
    // 3: dependent fp64 division chain
    double x = av;
    t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < N; i++) x = 1.0 / (x + 1.5);
    out[2] += x;
    t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) cyc[2] = (t1 - t0);
    // 4: dependent fp64 fma chain
    x = av;
    t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < N; i++) x = fma(x, bv, 0.5);
    out[3] += x;
    t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) cyc[3] = (t1 - t0);
    // 5: dependent DPP row_newbcast chain (32-bit)
    int iv = (int)lane;
    t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < N; i++) iv = __builtin_amdgcn_update_dpp(0, iv + 1, 0x153, 0xF, 0xF, false);
    out[4] += iv;
    t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) cyc[4] = (t1 - t0);
    // 6: dependent permlane16_swap chain
    unsigned uv = lane;
    t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < N; i++) {
        auto s = __builtin_amdgcn_permlane16_swap(uv, uv + 1, false, false);
        uv = s[0] + s[1];
    }
    out[5] += uv;
    t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) cyc[5] = (t1 - t0);
    // 7: dependent LDS write -> read round trip (other lane's value)
    double lv = av;
    t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < N; i++) {
        lds[lane] = lv;
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();
        lv = lds[(lane + 1) & 63] + 1.0;
    }
    out[6] += lv;
    t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) cyc[6] = (t1 - t0);
    // 8: __syncthreads chain (all waves of the block)
    t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < N; i++) __syncthreads();
    t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) cyc[7] = (t1 - t0);
    // 9: __shfl (bpermute) dependent chain on doubles
    x = av;
    t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < N; i++) x = __shfl_xor(x, 16, 64) + 1.0;
    out[7] += x;
    t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) cyc[8] = (t1 - t0);
}
int main() {
    double* o; unsigned long long* c;
    hipMalloc(&o, 64 * 8); hipMalloc(&c, 16 * 8);
    hipMemset(o, 0, 512);
    for (int threads : {64, 512}) {
        for (int rep = 0; rep < 2; rep++) hipLaunchKernelGGL(k, dim3(1), dim3(threads), 4096, 0, o, c, 1.0, 2.0);
        hipDeviceSynchronize();
        unsigned long long h[16];
        hipMemcpy(h, c, 16 * 8, hipMemcpyDeviceToHost);
        const char* nm[] = {"mfma_f64 16x16x4 dependent", "mfma_f64 16x16x4 4 chains", "fp64 div dependent",
                            "fp64 fma dependent", "dpp row_newbcast dependent", "permlane16_swap dependent",
                            "lds write->read roundtrip", "__syncthreads", "shfl_xor f64 dependent"};
        printf("block of %d threads (per op, cycles):\n", threads);
        for (int i = 0; i < 9; i++) printf("  %-32s %8.1f\n", nm[i], (double)h[i] / N);
    }
    return 0;
}
