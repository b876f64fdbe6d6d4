// Microbenchmark: the split kernel's register IFFT-32 (run_split, LDS tables)
// on register-resident data, no global memory, 4 waves per SIMD.  Reports
// kernel time and SIMD cycles per op pair.  Variants via -D (see gpu script).
#include "../../reedsolomon16_amd/csrc/kernels.hip"
#include <cstdio>

namespace rs {
namespace {
#ifndef NOSWAP
#define NOSWAP 0
#endif
template <int LOGM>
__global__ void __launch_bounds__(256, 4) kb(uint32_t *out, int iters) {
    typedef F16<1> F;
    constexpr int HM = (1 << LOGM) / 2;
    __shared__ __attribute__((aligned(16))) uint8_t tabs[2 * 20 * 96 + 36 * 1024];
    for (int i = threadIdx.x; i < 2 * 20 * 96 / 4; i += blockDim.x) ((uint32_t *)tabs)[i] = i * 0x9E3779B9u;
    __syncthreads();
    F::Vec w[HM];
    for (int r = 0; r < HM; r++) { w[r].l[0] = threadIdx.x * 7 + r; w[r].h[0] = threadIdx.x * 13 + r * 3; }
    const int half = (threadIdx.x & 63) >> 5;
    for (int it = 0; it < iters; it++)
        run_split<IfftSplit<LOGM>>(w, vgpr_lds_addr(tabs) + half * 16 * 96);
    uint32_t r = 0;
    for (int i = 0; i < HM; i++) r ^= w[i].l[0] ^ w[i].h[0];
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}
}  // namespace
}  // namespace rs

int main() {
    uint32_t *out;
    (void)hipMalloc(&out, 1024 * 256 * 4);
    const int iters = 64;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int rep = 0; rep < 2; rep++) {
        (void)hipEventRecord(e0);
        hipLaunchKernelGGL(rs::kb<5>, dim3(1024), dim3(256), 0, 0, out, iters);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
    }
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    // 1024 blocks x 4 waves = 4 waves per SIMD; 40 op pairs per IFFT per wave
    const double cyc = ms * 1e-3 * 2.2e9;
    printf("%s: %.1f us, %.1f SIMD-cycles per op pair @2.2GHz (4 waves/SIMD)\n", VNAME, ms * 1e3,
           cyc / (iters * 40.0 * 4));
    return 0;
}
