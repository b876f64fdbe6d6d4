// Minimal HIP library for the launch-blocking probe (scripts/launch_probe3.py):
// one spin kernel launched on a caller stream through a C entry point.
#include <hip/hip_runtime.h>

__global__ void k_spin2(float *x, int n, int iters) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float v = x[i];
    for (int k = 0; k < iters; k++) v = v * 1.0000001f + 1e-7f;
    x[i] = v;
}
__global__ void __launch_bounds__(256) k_lds64(float *x, int n) {
    __shared__ float l[16384];  // 64 KB static LDS
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    l[threadIdx.x * 64 % 16384] = i < n ? x[i] : 0.f;
    __syncthreads();
    if (i < n) x[i] = l[(threadIdx.x * 64 + 1) % 16384] + 1.f;
}
extern "C" int spin_launch(void *x, int n, int iters, void *stream) {
    hipLaunchKernelGGL(k_spin2, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, (float *)x, n, iters);
    return (int)hipGetLastError();
}
extern "C" int lds64_launch(void *x, int n, void *stream) {
    hipLaunchKernelGGL(k_lds64, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, (float *)x, n);
    return (int)hipGetLastError();
}
