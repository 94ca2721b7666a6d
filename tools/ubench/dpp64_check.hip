// r06: which 64-bit DPP forms of the fused pivot step (tools/gen_dpp16.py, RCP_DPP) compute what
// their non-DPP equivalents compute on gfx950. One wave; lane l holds v = 1.5 + l (distinct per
// lane); row_newbcast:P takes lane P of each 16-lane row. Printed: per form, the lanes whose
// result differs from the reference (v_mov_b64_dpp broadcast, then the plain VALU op).
//   A  v_rcp_f64_dpp r, v row_newbcast:P            vs  v_rcp_f64 r, bcast(v)
//   B  v_fmac_f64_dpp e, -v, r row_newbcast:P (e=1)  vs  v_fma_f64 e, -bcast(v), r, 1.0
//   C  v_fmac_f64_dpp e, v, r row_newbcast:P (e=1)   vs  v_fma_f64 e, bcast(v), r, 1.0
// Build: hipcc --offload-arch=gfx950 -O2 tools/ubench/dpp64_check.hip -o tools/ubench/dpp64_check
#include <hip/hip_runtime.h>

#include <cstdio>

template <int P>
__global__ void k_check(double* out) {
    const int l = threadIdx.x;
    double v = 1.5 + l, pv, rr, ra, eb, er, ec, erc;
    // (s_nop 1 first: 2 wait states between the VALU write of v and its DPP read)
    asm volatile("s_nop 1\n v_mov_b64_dpp %0, %1 row_newbcast:%2 row_mask:0xf bank_mask:0xf\n s_nop 1" : "=v"(pv) : "v"(v), "i"(P));
    asm volatile("v_rcp_f64 %0, %1\n s_nop 1" : "=v"(rr) : "v"(pv));
    asm volatile("s_nop 1\n v_rcp_f64_dpp %0, %1 row_newbcast:%2 row_mask:0xf bank_mask:0xf\n s_nop 1"
                 : "=v"(ra) : "v"(v), "i"(P));
    er = __builtin_fma(-pv, rr, 1.0);
    eb = 1.0;
    asm volatile("s_nop 1\n v_fmac_f64_dpp %0, -%1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf\n s_nop 1"
                 : "+v"(eb) : "v"(v), "v"(rr), "i"(P));
    erc = __builtin_fma(pv, rr, 1.0);
    ec = 1.0;
    asm volatile("s_nop 1\n v_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf\n s_nop 1"
                 : "+v"(ec) : "v"(v), "v"(rr), "i"(P));
    if (pv != 1.5 + 16 * (l >> 4) + P) rr = -1.0;   // the broadcast itself wrong: flag the reference
    out[6 * l + 0] = rr;
    out[6 * l + 1] = ra;
    out[6 * l + 2] = er;
    out[6 * l + 3] = eb;
    out[6 * l + 4] = erc;
    out[6 * l + 5] = ec;
}

int main() {
    double* d = nullptr;
    double h[6 * 64];
    if (hipMalloc(&d, sizeof(h)) != hipSuccess) return 1;
    auto run = [&](auto kern, int P) {
        hipLaunchKernelGGL(kern, dim3(1), dim3(64), 0, nullptr, d);
        if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return;
        int bad[3] = {0, 0, 0}, first[3] = {-1, -1, -1};
        for (int l = 0; l < 64; l++)
            for (int f = 0; f < 3; f++)
                if (h[6 * l + 2 * f] != h[6 * l + 2 * f + 1]) {
                    if (first[f] < 0) first[f] = l;
                    bad[f]++;
                }
        std::printf("P=%2d  A rcp_dpp: %2d lanes differ", P, bad[0]);
        if (first[0] >= 0) std::printf(" (lane %d: %.17g vs %.17g)", first[0], h[6 * first[0] + 1], h[6 * first[0]]);
        std::printf(" | B fmac_dpp -src0: %2d", bad[1]);
        if (first[1] >= 0) std::printf(" (lane %d: %.17g vs %.17g)", first[1], h[6 * first[1] + 3], h[6 * first[1] + 2]);
        std::printf(" | C fmac_dpp +src0: %2d", bad[2]);
        if (first[2] >= 0) std::printf(" (lane %d: %.17g vs %.17g)", first[2], h[6 * first[2] + 5], h[6 * first[2] + 4]);
        std::printf("\n");
    };
    run(k_check<0>, 0);
    run(k_check<3>, 3);
    run(k_check<9>, 9);
    run(k_check<15>, 15);
    (void)hipFree(d);
    return 0;
}
