// DPP wave-shift direction probe (gfx950): prints which source lane each lane reads under
// wave_shr:1 (0x138) and wave_shl:1 (0x130).  Build: hipcc --offload-arch=gfx950 -O3 -o tools/probe_dpp_wave tools/probe_dpp_wave.hip
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(int* o) {
    const int v = threadIdx.x;
    o[threadIdx.x] = __builtin_amdgcn_update_dpp(-1, v, 0x138, 0xf, 0xf, false);
    o[64 + threadIdx.x] = __builtin_amdgcn_update_dpp(-1, v, 0x130, 0xf, 0xf, false);
}
int main() {
    int* d;
    int h[128];
    (void)hipMalloc(&d, sizeof(h));
    k<<<1, 64>>>(d);
    (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    printf("wave_shr:1 lanes 0,1,31,32,63 read %d %d %d %d %d\n", h[0], h[1], h[31], h[32], h[63]);
    printf("wave_shl:1 lanes 0,1,31,32,63 read %d %d %d %d %d\n", h[64], h[65], h[95], h[96], h[127]);
    return 0;
}
