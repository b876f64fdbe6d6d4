// LDS read-cost lab: ds_read_b128 with a wave-uniform address (every lane
// reads the same 16 bytes: the twiddle-table pattern) vs per-lane addresses,
// at 16 waves per CU.  Prints LDS cycles per wave-instruction per CU.
#include <hip/hip_runtime.h>

#include <cstdio>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int MODE>  // 0 uniform address, 1 per-lane 16-B stride, 2 uniform but lane-half split (2 addresses)
__global__ void __launch_bounds__(256) k_lds(uint32_t *out, int iters, unsigned long long *cyc) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[32768];
    const int lane = threadIdx.x & 63;
    for (int i = threadIdx.x; i < 32768 / 4; i += 256) ((uint32_t *)lds)[i] = i * 2654435761u;
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    u32x4 acc = {0, 0, 0, 0};
    uint32_t base = (threadIdx.x >> 6) * 4096;
    if (MODE == 1) base += lane * 16;
    if (MODE == 2) base += (lane >> 5) * 2048;
    for (int it = 0; it < iters; it++) {
        const uint32_t a = base + (it & 15) * 96;
#pragma unroll
        for (int q = 0; q < 5; q++) {
            const u32x4 x = *(const volatile __attribute__((address_space(3))) u32x4 *)(uintptr_t)(a + 16 * q);
            acc ^= x;
        }
    }
    __syncthreads();
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) atomicMax(cyc, t1 - t0);
    if (acc.x == 0x1234567u) out[0] = acc.y;
}

int main() {
    uint32_t *out;
    unsigned long long *cyc;
    (void)hipMalloc(&out, 64);
    (void)hipMalloc(&cyc, 8);
    int cus = 256;
    const int iters = 2000;
    for (int mode = 0; mode < 3; mode++) {
        (void)hipMemset(cyc, 0, 8);
        // 4 blocks x 4 waves per CU
        if (mode == 0) hipLaunchKernelGGL(k_lds<0>, dim3(cus * 4), dim3(256), 0, 0, out, iters, cyc);
        if (mode == 1) hipLaunchKernelGGL(k_lds<1>, dim3(cus * 4), dim3(256), 0, 0, out, iters, cyc);
        if (mode == 2) hipLaunchKernelGGL(k_lds<2>, dim3(cus * 4), dim3(256), 0, 0, out, iters, cyc);
        (void)hipDeviceSynchronize();
        unsigned long long c;
        (void)hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
        // per CU: 16 waves x iters x 5 instructions
        printf("mode %d (%s): %.2f cycles per ds_read_b128 per CU (max over blocks %llu cycles)\n", mode,
               mode == 0 ? "uniform address" : mode == 1 ? "per-lane 16B" : "two addresses (lane halves)",
               (double)c / (16.0 * iters * 5), c);
    }
    return 0;
}
