// Layout probe for v_mfma_f64_4x4x4_4b_f64 (diagnostic only): wave w uses A = one-hot at lane w,
// B[l] = l + 1, C = 0; prints for every wave the output lanes and values (which B lane pairs
// with A lane w and lands in which D lane).
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/probe_mfma4x4 tools/probe_mfma4x4.hip
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void probe(double* out) {
    const int l = threadIdx.x, w = blockIdx.x;
    const double a = (l == w) ? 1.0 : 0.0;
    const double b = (double)(l + 1);
    const double d = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, 0.0, 0, 0, 0);
    out[w * 64 + l] = d;
}

int main() {
    double* d;
    (void)hipMalloc(&d, 64 * 64 * sizeof(double));
    probe<<<64, 64>>>(d);
    static double h[64 * 64];
    (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    for (int w = 0; w < 64; ++w) {
        printf("A%02d:", w);
        for (int l = 0; l < 64; ++l)
            if (h[w * 64 + l] != 0.0) printf(" D%d=B%d", l, (int)h[w * 64 + l] - 1);
        printf("\n");
    }
    return 0;
}
