// Developer probe: the lane / register layout of v_mfma_f64_16x16x4f64 on gfx950.
// Prints, for one wave, D = A x B with A[i][k] = 100 i + k + 1 supplied by lane i + 16 k (the
// assumed A layout) and B = all ones (so D[i][j] = sum_k A[i][k] identifies the row i), then
// A = all ones and B[k][j] = 100 j + k + 1 from lane j + 16 k (identifies the column j).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double d4 __attribute__((ext_vector_type(4)));
__global__ void probe(double *out) {
    const int l = threadIdx.x;
    const int i = l % 16, k = l / 16;
    d4 acc = {0, 0, 0, 0};
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(100.0 * i + k + 1, 1.0, acc, 0, 0, 0);
    for (int v = 0; v < 4; ++v) out[l * 4 + v] = acc[v];
    d4 acc2 = {0, 0, 0, 0};
    acc2 = __builtin_amdgcn_mfma_f64_16x16x4f64(1.0, 100.0 * i + k + 1, acc2, 0, 0, 0);
    for (int v = 0; v < 4; ++v) out[256 + l * 4 + v] = acc2[v];
}
int main() {
    double *d;
    hipMalloc(&d, 512 * sizeof(double));
    probe<<<1, 64>>>(d);
    double h[512];
    hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    for (int t = 0; t < 2; ++t) {
        printf("%s\n", t == 0 ? "rows: (sum_k A[i][k] - 10)/400 per lane, reg" : "cols: (sum_k B[k][j] - 10)/400 per lane, reg");
        for (int l = 0; l < 64; ++l) {
            printf("l%02d:", l);
            for (int v = 0; v < 4; ++v) printf(" %5.2f", (h[t * 256 + l * 4 + v] - 10.0) / 400.0);
            printf("%s", (l % 4 == 3) ? "\n" : "  ");
        }
    }
    return 0;
}
