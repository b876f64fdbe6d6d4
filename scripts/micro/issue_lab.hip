// VALU issue-cost calibration on gfx950: whole-kernel time (HIP events) at 8
// waves per SIMD, 8 independent chains per lane, long unrolled streams of one
// instruction kind.  SIMD cycles per wave-instruction = kernel time x clock /
// (wave-instructions per SIMD).  (Per-wave s_memtime brackets over-credit
// concurrency when a SIMD runs its waves one after another.)
#include <hip/hip_runtime.h>

#include <cstdio>

__device__ __forceinline__ uint32_t perm(uint32_t a, uint32_t b, uint32_t s) { return __builtin_amdgcn_perm(a, b, s); }
__device__ __forceinline__ uint32_t x3(uint32_t a, uint32_t b, uint32_t c) { return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96); }

constexpr int ITERS = 256, STEPS = 16, CH = 8;

template <int OP>
__global__ void __launch_bounds__(256) k(uint32_t *out, uint32_t seed, unsigned long long *clk) {
    uint32_t a[CH];
#pragma unroll
    for (int i = 0; i < CH; i++) a[i] = seed + threadIdx.x * 8 + i;
    uint32_t t0 = seed * 3 + threadIdx.x, t1 = seed * 7 + threadIdx.x, t2 = seed * 11 + threadIdx.x;
    asm volatile("" : "+v"(t0), "+v"(t1), "+v"(t2));
    const uint32_t s0 = __builtin_amdgcn_readfirstlane(seed * 5);
    const unsigned long long c0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < ITERS; it++) {
#pragma unroll
        for (int s = 0; s < STEPS; s++) {
#pragma unroll
            for (int i = 0; i < CH; i++) {
                if (OP == 0) a[i] = perm(t0, t1, a[i]);           // v_perm_b32, 3 VGPR sources
                if (OP == 1) a[i] = perm(s0, t1, a[i]);           // v_perm_b32, one SGPR table operand
                if (OP == 2) a[i] = x3(a[i], t0, t1);             // v_bitop3_b32
                if (OP == 3) a[i] = a[i] ^ t0;                    // v_xor_b32 (VOP2)
                if (OP == 4) a[i] = a[i] & 0x07070707u;           // v_and_b32 with a literal
                if (OP == 5) a[i] = a[i] >> 3;                    // v_lshrrev_b32
                if (OP == 6) a[i] = a[i] + t0;                    // v_add_u32
                if (OP < 7) asm volatile("" : "+v"(a[i]));        // no algebraic folding across steps
            }
            if (OP == 8) {  // v_permlane32_swap pairs
#pragma unroll
                for (int i = 0; i < CH; i += 2) {
                    const auto r = __builtin_amdgcn_permlane32_swap(a[i], a[i + 1], false, false);
                    a[i] = r[0];
                    a[i + 1] = r[1];
                }
            }
            if (OP == 7) {  // the GF(2^16) multiply-accumulate mix: CH/2 independent (x, y) pairs
#pragma unroll
                for (int i = 0; i < CH; i += 2) {
                    const uint32_t lo = a[i + 1], hi = a[i + 1] ^ t2;
                    const uint32_t a0 = lo & 0x07070707u, a1 = (lo >> 3) & 0x07070707u, a2 = (lo >> 6) & 0x03030303u;
                    const uint32_t b0 = hi & 0x07070707u, b1 = (hi >> 3) & 0x07070707u, b2 = (hi >> 6) & 0x03030303u;
                    a[i] = x3(x3(x3(a[i], perm(t1, t0, a0), perm(t2, t1, a1)), perm(t0, t0, a2), perm(t1, t2, b0)),
                              perm(t0, t2, b1), perm(t1, t1, b2));
                    a[i + 1] ^= a[i];
                }
            }
        }
    }
    const unsigned long long c1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    uint32_t r = 0;
#pragma unroll
    for (int i = 0; i < CH; i++) r ^= a[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        clk[0] = c1 - c0;
        clk[1] = r1 - r0;
    }
}


// I-cache sensitivity: the multiply mix with an unrolled body of NSTEP steps
// (about 27 x 4 x 8 bytes of code per step), total work held constant.
template <int NSTEP, int NCH = CH>
__global__ void __launch_bounds__(256) kmix(uint32_t *out, uint32_t seed, int iters) {
    constexpr int CH = NCH;
    uint32_t a[CH];
#pragma unroll
    for (int i = 0; i < CH; i++) a[i] = seed + threadIdx.x * 8 + i;
    uint32_t t0 = seed * 3 + threadIdx.x, t1 = seed * 7 + threadIdx.x, t2 = seed * 11 + threadIdx.x;
    asm volatile("" : "+v"(t0), "+v"(t1), "+v"(t2));
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int s = 0; s < NSTEP; s++) {
#pragma unroll
            for (int i = 0; i < CH; i += 2) {
                const uint32_t lo = a[i + 1], hi = a[i + 1] ^ t2;
                const uint32_t a0 = lo & 0x07070707u, a1 = (lo >> 3) & 0x07070707u, a2 = (lo >> 6) & 0x03030303u;
                const uint32_t b0 = hi & 0x07070707u, b1 = (hi >> 3) & 0x07070707u, b2 = (hi >> 6) & 0x03030303u;
                a[i] = x3(x3(x3(a[i], perm(t1, t0, a0), perm(t2, t1, a1)), perm(t0, t0, a2), perm(t1, t2, b0)),
                          perm(t0, t2, b1), perm(t1, t1, b2));
                a[i + 1] ^= a[i];
                asm volatile("" : "+v"(a[i]), "+v"(a[i + 1]));
            }
        }
    }
    uint32_t r = 0;
#pragma unroll
    for (int i = 0; i < CH; i++) r ^= a[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

int main() {
    uint32_t *out;
    unsigned long long *clk;
    const int cus = 256, wps = 8;
    const int blocks = cus * wps;  // 256-thread blocks: 1 wave per SIMD per block
    (void)hipMalloc(&out, (size_t)blocks * 256 * 4);
    (void)hipMalloc(&clk, 16);
    const char *names[] = {"v_perm vvv", "v_perm svv", "v_bitop3", "v_xor", "v_and lit", "v_lshrrev", "v_add", "mul_add mix",
                           "permlane32sw"};
    // wave-instructions per wave for each op (mix: per pair 10 extract + 12 perm + 3 bitop3 + 1 xor(hi) + 1 xor = 27)
    const double per_wave[] = {ITERS * STEPS * CH * 1.0, ITERS * STEPS * CH * 1.0, ITERS * STEPS * CH * 1.0,
                               ITERS * STEPS * CH * 1.0, ITERS * STEPS * CH * 1.0, ITERS * STEPS * CH * 1.0,
                               ITERS * STEPS * CH * 1.0, ITERS * STEPS * (CH / 2) * 27.0, ITERS * STEPS * (CH / 2) * 1.0};
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int op = 0; op < 9; op++) {
        auto launch = [&]() {
            switch (op) {
                case 0: hipLaunchKernelGGL(k<0>, dim3(blocks), dim3(256), 0, 0, out, 1u, clk); break;
                case 1: hipLaunchKernelGGL(k<1>, dim3(blocks), dim3(256), 0, 0, out, 1u, clk); break;
                case 2: hipLaunchKernelGGL(k<2>, dim3(blocks), dim3(256), 0, 0, out, 1u, clk); break;
                case 3: hipLaunchKernelGGL(k<3>, dim3(blocks), dim3(256), 0, 0, out, 1u, clk); break;
                case 4: hipLaunchKernelGGL(k<4>, dim3(blocks), dim3(256), 0, 0, out, 1u, clk); break;
                case 5: hipLaunchKernelGGL(k<5>, dim3(blocks), dim3(256), 0, 0, out, 1u, clk); break;
                case 6: hipLaunchKernelGGL(k<6>, dim3(blocks), dim3(256), 0, 0, out, 1u, clk); break;
                case 7: hipLaunchKernelGGL(k<7>, dim3(blocks), dim3(256), 0, 0, out, 1u, clk); break;
                case 8: hipLaunchKernelGGL(k<8>, dim3(blocks), dim3(256), 0, 0, out, 1u, clk); break;
            }
        };
        launch();
        (void)hipDeviceSynchronize();
        (void)hipEventRecord(e0);
        launch();
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        unsigned long long h[2];
        (void)hipMemcpy(h, clk, 16, hipMemcpyDeviceToHost);
        const double ghz = (double)h[0] / ((double)h[1] / 100.0) / 1e3;  // shader cycles per us / 1e3
        const double instr_per_simd = per_wave[op] * wps;
        printf("%-12s %.2f SIMD cycles per wave-instruction (kernel %.1f us, clock %.2f GHz)\n", names[op],
               ms * 1e3 * ghz * 1e3 / instr_per_simd, ms * 1e3, ghz);
    }
    // I-cache sweep: same total multiply count (4096 steps per wave), growing body
    {
        const int total = 4096;
        auto run = [&](const char *nm, auto launch, int body) {
            launch();
            (void)hipDeviceSynchronize();
            (void)hipEventRecord(e0);
            launch();
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            float ms;
            (void)hipEventElapsedTime(&ms, e0, e1);
            const double instr_per_simd = (double)total * (CH / 2) * 27.0 * wps;
            printf("mix body %-5s (%3d steps ~%5.1f KB) %.2f SIMD cycles/instr at 2.2 GHz (kernel %.1f us)\n", nm, body,
                   body * 4 * 27 * 8 / 1024.0, ms * 1e3 * 2.2e3 / instr_per_simd, ms * 1e3);
        };
        run("16", [&] { hipLaunchKernelGGL(kmix<16>, dim3(blocks), dim3(256), 0, 0, out, 1u, total / 16); }, 16);
        run("64", [&] { hipLaunchKernelGGL(kmix<64>, dim3(blocks), dim3(256), 0, 0, out, 1u, total / 64); }, 64);
        run("128", [&] { hipLaunchKernelGGL(kmix<128>, dim3(blocks), dim3(256), 0, 0, out, 1u, total / 128); }, 128);
        run("256", [&] { hipLaunchKernelGGL(kmix<256>, dim3(blocks), dim3(256), 0, 0, out, 1u, total / 256); }, 256);
    }
    // dependency / occupancy sweep: 1 or 4 independent (x, y) pairs per lane, 4 or 8 waves per SIMD
    for (int w = 4; w <= 8; w += 4) {
        for (int ch = 2; ch <= 8; ch += 6) {
            const int total = 4096, nb = cus * w;
            auto launch = [&]() {
                if (ch == 2) hipLaunchKernelGGL((kmix<16, 2>), dim3(nb), dim3(256), 0, 0, out, 1u, total / 16);
                else hipLaunchKernelGGL((kmix<16, 8>), dim3(nb), dim3(256), 0, 0, out, 1u, total / 16);
            };
            launch();
            (void)hipDeviceSynchronize();
            (void)hipEventRecord(e0);
            launch();
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            float ms;
            (void)hipEventElapsedTime(&ms, e0, e1);
            const double instr_per_simd = (double)total * (ch / 2) * 27.0 * w;
            printf("mix %d pair(s)/lane, %d waves/SIMD: %.2f SIMD cycles/instr at 2.2 GHz\n", ch / 2, w,
                   ms * 1e3 * 2.2e3 / instr_per_simd);
        }
    }
    return 0;
}
