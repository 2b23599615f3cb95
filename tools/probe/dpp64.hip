// Probe: semantics of 64-bit DPP FMA (v_fmac_f64_dpp row_newbcast + bank mask) on gfx950.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(double *out, int mode) {
    const int l = threadIdx.x;
    double g = 1000.0 * l, d = l + 1.0, c = 1.0;
    if (mode == 0)
        asm volatile("s_nop 4\n\tv_fmac_f64_dpp %0, %1, %2 row_newbcast:1 row_mask:0xf bank_mask:0x3" : "+v"(g) : "v"(d), "v"(c));
    else if (mode == 1)
        asm volatile("s_nop 4\n\tv_fmac_f64_dpp %0, %1, %2 row_newbcast:1 row_mask:0xf bank_mask:0xf" : "+v"(g) : "v"(d), "v"(c));
    else if (mode == 2)
        asm volatile("s_nop 4\n\tv_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0x3\n\t"
                     "v_fmac_f64_dpp %0, %1, %2 row_newbcast:%4 row_mask:0xf bank_mask:0xc" : "+v"(g) : "v"(d), "v"(c), "i"(2), "i"(10));
    else if (mode == 4)
        asm volatile("s_nop 4\n\tv_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0x3\n\ts_nop 1\n\t"
                     "v_fmac_f64_dpp %0, %1, %2 row_newbcast:%4 row_mask:0xf bank_mask:0xc" : "+v"(g) : "v"(d), "v"(c), "i"(2), "i"(10));
    else if (mode == 5)
        asm volatile("s_nop 4\n\tv_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0x3\n\ts_nop 4\n\t"
                     "v_fmac_f64_dpp %0, %1, %2 row_newbcast:%4 row_mask:0xf bank_mask:0xc" : "+v"(g) : "v"(d), "v"(c), "i"(2), "i"(10));
    else if (mode == 6) {
        double g2 = g;
        asm volatile("s_nop 4\n\tv_fmac_f64_dpp %0, %2, %3 row_newbcast:%4 row_mask:0xf bank_mask:0x3\n\t"
                     "v_fmac_f64_dpp %1, %2, %3 row_newbcast:%5 row_mask:0xf bank_mask:0xc" : "+v"(g), "+v"(g2) : "v"(d), "v"(c), "i"(2), "i"(10));
        g = (l & 8) ? g2 : g;
    } else if (mode == 7) {
        // single-instruction with d premasked: lane 16r+J and 16r+8+J hold values, shift-free?
        asm volatile("s_nop 4\n\tv_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0x3\n\t"
                     "v_nop\n\tv_nop\n\t"
                     "v_fmac_f64_dpp %0, %1, %2 row_newbcast:%4 row_mask:0xf bank_mask:0xc" : "+v"(g) : "v"(d), "v"(c), "i"(2), "i"(10));
    } else {
        double r;
        asm volatile("s_nop 4\n\tv_mov_b64_dpp %0, %1 row_newbcast:3 row_mask:0xf bank_mask:0xf" : "=v"(r) : "v"(d));
        g = r;
    }
    out[mode * 64 + l] = g;
}
int main() {
    double *o; hipMalloc(&o, 9 * 64 * sizeof(double));
    for (int m = 0; m < 9; ++m) hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, o, m);
    double h[576]; hipMemcpy(h, o, sizeof h, hipMemcpyDeviceToHost);
    for (int m = 0; m < 9; ++m) {
        printf("mode %d:", m);
        for (int l = 0; l < 32; ++l) printf(" %g", h[m * 64 + l]);
        printf("\n");
    }
    return 0;
}
