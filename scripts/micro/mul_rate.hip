// Microbenchmark: cycles per GF(2^16) v_perm multiply-accumulate (4 symbols)
// with NI independent mul_adds interleaved, VGPR-resident tables, at 1/2/4
// waves per SIMD (s_memtime).
#include <hip/hip_runtime.h>
#include <cstdio>

__device__ __forceinline__ uint32_t perm(uint32_t a, uint32_t b, uint32_t s) { return __builtin_amdgcn_perm(a, b, s); }
__device__ __forceinline__ uint32_t x3(uint32_t a, uint32_t b, uint32_t c) { return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96); }

__device__ __forceinline__ void mul_add(uint32_t &xl, uint32_t &xh, uint32_t lo, uint32_t hi, const uint32_t *t) {
    const uint32_t a0 = lo & 0x07070707u, a1 = (lo >> 3) & 0x07070707u, a2 = (lo >> 6) & 0x03030303u;
    const uint32_t b0 = hi & 0x07070707u, b1 = (hi >> 3) & 0x07070707u, b2 = (hi >> 6) & 0x03030303u;
    xl = x3(x3(x3(xl, perm(t[1], t[0], a0), perm(t[5], t[4], a1)), perm(t[8], t[8], a2), perm(t[11], t[10], b0)),
            perm(t[15], t[14], b1), perm(t[18], t[18], b2));
    xh = x3(x3(x3(xh, perm(t[3], t[2], a0), perm(t[7], t[6], a1)), perm(t[9], t[9], a2), perm(t[13], t[12], b0)),
            perm(t[17], t[16], b1), perm(t[19], t[19], b2));
}

template <int NI>
__global__ void k(uint32_t *out, unsigned long long *cyc, const uint32_t *tab, int iters) {
    uint32_t t[20];
    for (int j = 0; j < 20; j++) t[j] = tab[j] + threadIdx.x * 0;  // VGPR tables
    for (int j = 0; j < 20; j++) asm volatile("" : "+v"(t[j]));
    uint32_t xl[NI], xh[NI], yl[NI], yh[NI];
    for (int i = 0; i < NI; i++) { xl[i] = threadIdx.x + i; xh[i] = xl[i] * 3; yl[i] = xl[i] * 5; yh[i] = xl[i] * 7; }
    unsigned long long c0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int s = 0; s < 8; s++) {
#pragma unroll
            for (int i = 0; i < NI; i++) {
                // IFFT butterfly: y ^= x; x ^= y * m
                yl[i] ^= xl[i]; yh[i] ^= xh[i];
                mul_add(xl[i], xh[i], yl[i], yh[i], t);
            }
        }
    }
    unsigned long long c1 = __builtin_amdgcn_s_memtime();
    uint32_t r = 0;
    for (int i = 0; i < NI; i++) r ^= xl[i] ^ xh[i] ^ yl[i] ^ yh[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
    if (threadIdx.x % 64 == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = c1 - c0;
}

int main() {
    uint32_t *out, *tab;
    unsigned long long *cyc;
    (void)hipMalloc(&out, 256 * 16 * 1024 * 4);
    (void)hipMalloc(&cyc, 256 * 16 * 16 * 8);
    (void)hipMalloc(&tab, 128);
    uint32_t ht[32];
    for (int i = 0; i < 32; i++) ht[i] = 0x01020304u * (i + 1);
    (void)hipMemcpy(tab, ht, 128, hipMemcpyHostToDevice);
    static unsigned long long h[256 * 16 * 16];
    const int iters = 128;
    for (int wps = 1; wps <= 4; wps *= 2) {
        for (int ni = 1; ni <= 4; ni *= 2) {
            dim3 grid(256 * wps), block(256);
            auto launch = [&]() {
                if (ni == 1) hipLaunchKernelGGL(k<1>, grid, block, 0, 0, out, cyc, tab, iters);
                if (ni == 2) hipLaunchKernelGGL(k<2>, grid, block, 0, 0, out, cyc, tab, iters);
                if (ni == 4) hipLaunchKernelGGL(k<4>, grid, block, 0, 0, out, cyc, tab, iters);
            };
            launch();
            (void)hipDeviceSynchronize();
            launch();
            (void)hipDeviceSynchronize();
            const int nw = 256 * wps * 4;
            (void)hipMemcpy(h, cyc, nw * 8, hipMemcpyDeviceToHost);
            double avg = 0;
            for (int i = 0; i < nw; i++) avg += (double)h[i];
            avg /= nw;
            const double muls = (double)iters * 8 * ni;
            printf("waves/SIMD=%d NI=%d: %.1f SIMD-cycles per butterfly (%.2f per VALU instr at 28 instr/butterfly)\n", wps,
                   ni, avg / muls / wps, avg / muls / wps / 28.0);
        }
    }
    return 0;
}
