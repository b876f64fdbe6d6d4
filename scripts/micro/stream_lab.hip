// Memory-side lab for the C3 encode access pattern (128 data rows + 32 parity
// rows of 1 MiB): no GF arithmetic, only the loads/stores the encode kernels
// issue.  Diagnostic only.
//   seq   : each wave streams a contiguous 16 KiB piece via LDS-DMA (upper bound)
//   pat   : split-kernel pattern: wave = 256 B column span; per chunk 32 rows x 256 B
//           by 8 buffer_load...lds; 4 chunks; then 32 rows x 256 B of dword stores
//   patx  : pat with an XCD-aware block order (blocks on one XCD take adjacent spans)
//   patw  : pat with 512 B spans per wave (2 units per lane; 16 DMA per chunk)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

typedef __attribute__((address_space(3))) void lvoid_t;
constexpr int K = 128, P = 32;
constexpr size_t S = 1 << 20;

__device__ __forceinline__ void wait_vm0() { __builtin_amdgcn_s_waitcnt(0x0F70); }

template <int SPAN, bool XCD, bool SPLITST = false>
__global__ void __launch_bounds__(256) k_pat(uint8_t *base, size_t stride, uint32_t *sink) {
    constexpr int M = 32, NDMA = M * SPAN / 1024, PPR = SPAN / 16;
    __shared__ __attribute__((aligned(16))) uint8_t lds[4 * M * SPAN];
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    unsigned b = blockIdx.x;
    if (XCD) {  // dispatch order b -> XCD b % 8; give each XCD a contiguous range of spans
        const unsigned nb = gridDim.x, per = nb / 8;
        b = (b % 8) * per + b / 8;
    }
    const uint32_t span = (b * 4 + wave) * SPAN;
    uint8_t *img = lds + wave * M * SPAN;
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(base, 0, (int)((K - 1) * stride + S), 0x00020000);
    const uint32_t loff = (lane / PPR) * (uint32_t)stride + (lane % PPR) * 16 + span;
    uint32_t acc = 0;
    for (int c = 0; c < K / M; c++) {
#pragma unroll
        for (int j = 0; j < NDMA; j++)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lvoid_t *)(img + j * 1024), 16, loff,
                                                     (uint32_t)((c * M + j * (64 / PPR)) * stride), 0, 0);
        wait_vm0();
        __syncthreads();
        acc ^= *(const __attribute__((address_space(3))) uint32_t *)(img + lane * 4);
    }
    uint8_t *par = base + K * stride + span;
    if (SPLITST) {
        // the encode kernels' store pattern: lane (cu, half) writes the lo dword of
        // unit cu at (cu/8)*64 + (cu%8)*4 and the hi dword 32 bytes later, for
        // rows r (lower half) and r + 16 (upper half)
        const int cu = lane & 31, hf = lane >> 5;
        const uint32_t colb = (cu >> 3) * 64 + (cu & 7) * 4;
        for (int row = 0; row < P / 2; row++) {
            uint8_t *q = par + (size_t)(row + 16 * hf) * stride + colb;
            *(__attribute__((address_space(1))) uint32_t *)q = acc + row;
            *(__attribute__((address_space(1))) uint32_t *)(q + 32) = acc ^ row;
        }
    } else {
        // parity: 32 rows x SPAN bytes, contiguous 4-byte-per-lane stores
        for (int row = 0; row < P; row++)
            for (int q = 0; q < SPAN / 256; q++)
                *(__attribute__((address_space(1))) uint32_t *)(par + row * stride + q * 256 + lane * 4) = acc + row;
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

__global__ void __launch_bounds__(256) k_seq(uint8_t *base, size_t total_rd, uint32_t *sink) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[4 * 16384];
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const size_t w = (size_t)blockIdx.x * 4 + wave;
    const size_t off = w * 16384;
    uint8_t *img = lds + wave * 16384;
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(base + off, 0, 16384, 0x00020000);
#pragma unroll
    for (int j = 0; j < 16; j++)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lvoid_t *)(img + j * 1024), 16, lane * 16, j * 1024, 0, 0);
    wait_vm0();
    uint32_t v = *(const __attribute__((address_space(3))) uint32_t *)(img + lane * 4);
    // writes: 1/4 of the read volume, contiguous
    uint8_t *out = base + total_rd + w * 4096;
    for (int q = 0; q < 16; q++) *(__attribute__((address_space(1))) uint32_t *)(out + q * 256 + lane * 4) = v + q;
    if (v == 0x12345678u) sink[0] = v;
}

template <class F>
float timeit(F f, int n = 20) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    for (int i = 0; i < 3; i++) f();
    (void)hipEventRecord(a);
    for (int i = 0; i < n; i++) f();
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms;
    (void)hipEventElapsedTime(&ms, a, b);
    return ms * 1e3f / n;
}

int main() {
    uint8_t *base;
    uint32_t *sink;
    const size_t bytes = (K + P) * S;
    (void)hipMalloc(&base, bytes + (64 << 20));
    (void)hipMalloc(&sink, 64);
    (void)hipMemset(base, 0x5A, bytes);
    const double alg = (double)bytes;
    auto rep = [&](const char *n, float us) { printf("%-6s %8.2f us  %7.1f GB/s (of (k+p)*S)\n", n, us, alg / us / 1e3); };
    const int nb256 = S / 256 / 4, nb512 = S / 512 / 4;
    rep("seq", timeit([&] { hipLaunchKernelGGL(k_seq, dim3(K * S / 16384 / 4), dim3(256), 0, 0, base, K * S, sink); }));
    rep("pat", timeit([&] { hipLaunchKernelGGL((k_pat<256, false>), dim3(nb256), dim3(256), 0, 0, base, S, sink); }));
    rep("patx", timeit([&] { hipLaunchKernelGGL((k_pat<256, true>), dim3(nb256), dim3(256), 0, 0, base, S, sink); }));
    rep("patS", timeit([&] { hipLaunchKernelGGL((k_pat<256, false, true>), dim3(nb256), dim3(256), 0, 0, base, S, sink); }));
    rep("patw", timeit([&] { hipLaunchKernelGGL((k_pat<512, false>), dim3(nb512), dim3(256), 0, 0, base, S, sink); }));
    rep("patwx", timeit([&] { hipLaunchKernelGGL((k_pat<512, true>), dim3(nb512), dim3(256), 0, 0, base, S, sink); }));
    return hipDeviceSynchronize() != hipSuccess;
}
