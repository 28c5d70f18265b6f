#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(int *o) {
    if (threadIdx.x == 0) o[blockIdx.x] = __builtin_amdgcn_s_getreg(20 | (0 << 6) | (3 << 11));
}
int main() {
    int *d, h[64];
    hipMalloc(&d, 64 * 4);
    hipLaunchKernelGGL(k, dim3(64), dim3(64), 0, 0, d);
    hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
    for (int i = 0; i < 64; ++i) printf("%d%c", h[i], i % 16 == 15 ? '\n' : ' ');
    return 0;
}
