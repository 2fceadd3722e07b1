// Probe (gfx950): operand/result lane map of v_mfma_f64_4x4x4_4b_f64 with CBSZ/ABID broadcast, and
// the 16x16x4 f64 layout, from one-hot A operands.  Build: hipcc --offload-arch=gfx950 -O3 -o
// tools/probe_mfma_bcast tools/probe_mfma_bcast.hip
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double f64x4 __attribute__((ext_vector_type(4)));
template <int CB, int AB>
__global__ void k4(int L, double* out) {
    const int l = threadIdx.x;
    const double a = (l == L) ? 1.0 : 0.0, b = 100.0 + l;
    out[l] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, 0.0, CB, AB, 0);
}
__global__ void k16(int L, double* out) {
    const int l = threadIdx.x;
    const double a = (l == L) ? 1.0 : 0.0, b = 100.0 + l;
    f64x4 d = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, f64x4{0, 0, 0, 0}, 0, 0, 0);
    for (int r = 0; r < 4; ++r) out[r * 64 + l] = d[r];
}
template <typename K>
void show(const char* name, K kern, int L, int nreg) {
    double* d; hipMalloc(&d, 256 * sizeof(double)); hipMemset(d, 0, 256 * sizeof(double));
    hipLaunchKernelGGL(kern, dim3(1), dim3(64), 0, 0, L, d);
    double h[256]; hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    printf("%s A one-hot lane %2d:", name, L);
    for (int r = 0; r < nreg; ++r) for (int l = 0; l < 64; ++l) if (h[r * 64 + l] != 0.0) printf(" r%d:l%d=%g", r, l, h[r * 64 + l] - 100);
    printf("\n");
    hipFree(d);
}
int main() {
    for (int L : {0, 1, 4, 5, 16, 21, 37}) {
        show("16x16x4      ", k16, L, 4);
        show("4x4x4 cb0 ab0", k4<0, 0>, L, 1);
        show("4x4x4 cb2 ab0", k4<2, 0>, L, 1);
        show("4x4x4 cb2 ab1", k4<2, 1>, L, 1);
        show("4x4x4 cb2 ab3", k4<2, 3>, L, 1);
        show("4x4x4 cb1 ab1", k4<1, 1>, L, 1);
    }
    return 0;
}
