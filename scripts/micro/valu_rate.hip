// Microbenchmark: VALU issue rate of the instructions the GF kernels use
// (v_perm_b32, v_bitop3_b32, v_and/v_lshrrev, v_xor) on gfx950, measured with
// s_memtime (shader clock) inside the kernel.  8 independent chains x 16
// unrolled steps per loop iteration.  Reports SIMD cycles per wave-instruction.
#include <hip/hip_runtime.h>
#include <cstdio>

template <int OP>
__global__ void k(uint32_t *out, unsigned long long *cyc, uint32_t seed, int iters) {
    uint32_t a[8];
    for (int i = 0; i < 8; i++) a[i] = seed + threadIdx.x * 8 + i;
    uint32_t t0 = seed * 3, t1 = seed * 7;
    unsigned long long c0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int s = 0; s < 16; s++) {
#pragma unroll
            for (int i = 0; i < 8; i++) {
                if (OP == 0) a[i] = __builtin_amdgcn_perm(t0, a[i], a[i] ^ t1);
                if (OP == 1) a[i] = __builtin_amdgcn_perm(t0, t1, a[i]);
                if (OP == 2) a[i] = __builtin_amdgcn_bitop3_b32(a[i], t0 + s, t1, 0x96);
                if (OP == 3) a[i] = (a[i] >> 3) & 0x07070707u;
                if (OP == 4) a[i] = a[i] ^ (t0 + s);
                if (OP == 5) a[i] = __builtin_amdgcn_perm(a[(i + 1) & 7], a[i], t1 + s);
            }
        }
    }
    unsigned long long c1 = __builtin_amdgcn_s_memtime();
    uint32_t r = 0;
    for (int i = 0; i < 8; i++) r ^= a[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
    if (threadIdx.x % 64 == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = c1 - c0;
}

int main() {
    uint32_t *out;
    unsigned long long *cyc;
    (void)hipMalloc(&out, 256 * 16 * 1024 * 4);
    (void)hipMalloc(&cyc, 256 * 16 * 16 * 8);
    static unsigned long long h[256 * 16 * 16];
    const char *names[] = {"perm(v,v,v)", "perm(s,s,v)", "bitop3", "lshr+and", "xor", "perm(v,v,s)"};
    const int iters = 256;
    for (int wps = 1; wps <= 4; wps *= 2) {
        for (int op = 0; op < 6; op++) {
            dim3 grid(256 * wps), block(256);
            auto launch = [&]() {
                switch (op) {
                    case 0: hipLaunchKernelGGL(k<0>, grid, block, 0, 0, out, cyc, 1u, iters); break;
                    case 1: hipLaunchKernelGGL(k<1>, grid, block, 0, 0, out, cyc, 1u, iters); break;
                    case 2: hipLaunchKernelGGL(k<2>, grid, block, 0, 0, out, cyc, 1u, iters); break;
                    case 3: hipLaunchKernelGGL(k<3>, grid, block, 0, 0, out, cyc, 1u, iters); break;
                    case 4: hipLaunchKernelGGL(k<4>, grid, block, 0, 0, out, cyc, 1u, iters); break;
                    case 5: hipLaunchKernelGGL(k<5>, grid, block, 0, 0, out, cyc, 1u, iters); break;
                }
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
            const double per_wave_instr = (double)iters * 16 * 8 * (op == 3 ? 2 : 1);
            // s_memtime ticks at the shader clock; wps waves share a SIMD
            printf("waves/SIMD=%d %-12s %.2f cycles per wave-instr per SIMD (wave alone: %.2f)\n", wps, names[op],
                   avg / per_wave_instr / wps, avg / per_wave_instr);
        }
    }
    return 0;
}
