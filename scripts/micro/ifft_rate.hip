// Microbenchmark: the fused kernel's register IFFT-32 (op list, LDS tables)
// on register-resident data, no global memory.  Reports SIMD-cycles per
// butterfly at 1/2/4 waves per SIMD.
#include "../../reedsolomon16_amd/csrc/kernels.hip"
#include <cstdio>

namespace rs {
namespace {
template <int LOGM>
__global__ void __launch_bounds__(256) kb(uint32_t *out, unsigned long long *cyc, int iters) {
    typedef F16<1> F;
    constexpr int M = 1 << LOGM;
    __shared__ __attribute__((aligned(16))) uint8_t tabs[64 * 96];
    for (int i = threadIdx.x; i < 64 * 96 / 4; i += blockDim.x) ((uint32_t *)tabs)[i] = i * 0x9E3779B9u;
    __syncthreads();
    F::Vec w[M];
    for (int r = 0; r < M; r++) { w[r].l[0] = threadIdx.x * 7 + r; w[r].h[0] = threadIdx.x * 13 + r * 3; }
    unsigned long long c0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; it++) ifft_reg<F, LOGM>(w, vgpr_lds_addr(tabs));
    unsigned long long c1 = __builtin_amdgcn_s_memtime();
    uint32_t r = 0;
    for (int i = 0; i < M; i++) r ^= w[i].l[0] ^ w[i].h[0];
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
    if (threadIdx.x % 64 == 0) cyc[blockIdx.x * 4 + threadIdx.x / 64] = c1 - c0;
}
}  // namespace
}  // namespace rs

int main() {
    uint32_t *out;
    unsigned long long *cyc;
    (void)hipMalloc(&out, 256 * 16 * 256 * 4);
    (void)hipMalloc(&cyc, 256 * 16 * 4 * 8);
    static unsigned long long h[256 * 16 * 4];
    const int iters = 32;
    for (int wps = 1; wps <= 2; wps *= 2) {
        dim3 grid(256 * wps), block(256);
        hipLaunchKernelGGL(rs::kb<5>, grid, block, 0, 0, out, cyc, iters);
        (void)hipDeviceSynchronize();
        hipLaunchKernelGGL(rs::kb<5>, grid, block, 0, 0, out, cyc, iters);
        (void)hipDeviceSynchronize();
        const int nw = 256 * wps * 4;
        (void)hipMemcpy(h, cyc, nw * 8, hipMemcpyDeviceToHost);
        double avg = 0;
        for (int i = 0; i < nw; i++) avg += (double)h[i];
        avg /= nw;
        printf("IFFT-32 reg: waves/SIMD=%d  %.1f SIMD-cycles per butterfly (80 per IFFT)\n", wps, avg / (iters * 80.0) / wps);
    }
    return 0;
}
