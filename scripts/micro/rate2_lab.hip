// Issue-rate lab for the wave-independent bit-sliced encode design (round 2):
// SIMD cycles per wave-instruction at 1, 2 and 4 waves per SIMD for the
// instruction kinds that design uses -- v_bitop3_b32, v_xor_b32, v_cndmask_b32
// with a DPP source (lane-bit <-> register-bit swaps for lane bits 0-3),
// v_permlane16_swap / v_permlane32_swap (lane bits 4, 5) -- and a dependent
// bitop3 chain (latency).  Whole-kernel time (HIP events) x in-kernel clock.
// Diagnostic only.
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int ITERS = 256, STEPS = 16, CH = 8;

__device__ __forceinline__ uint32_t x3(uint32_t a, uint32_t b, uint32_t c) { return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96); }

template <int OP>
__global__ void k(uint32_t *out, uint32_t seed, unsigned long long *clk) {
    uint32_t a[CH];
#pragma unroll
    for (int i = 0; i < CH; i++) a[i] = seed + threadIdx.x * 8 + i;
    uint32_t t0 = seed * 3 + threadIdx.x, t1 = seed * 7 + threadIdx.x;
    asm volatile("" : "+v"(t0), "+v"(t1));
    const uint64_t lomask = 0x00FF00FF00FF00FFull;  // lanes with bit 3 clear
    const unsigned long long c0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < ITERS; it++) {
#pragma unroll
        for (int s = 0; s < STEPS; s++) {
            if constexpr (OP == 0) {
#pragma unroll
                for (int i = 0; i < CH; i++) { a[i] = x3(a[i], t0, t1); asm volatile("" : "+v"(a[i])); }
            } else if constexpr (OP == 1) {
#pragma unroll
                for (int i = 0; i < CH; i++) { a[i] = a[i] ^ t0; asm volatile("" : "+v"(a[i])); }
            } else if constexpr (OP == 2) {  // swap of lane bit 3 with a register bit: 1 cndmask_dpp per dword
                uint32_t n0, n1, n2, n3, n4, n5, n6, n7;
                asm volatile(
                    "s_mov_b64 vcc, %16\n\ts_nop 1\n\t"
                    "v_cndmask_b32_dpp %0, %9, %8, vcc row_ror:8 row_mask:0xf bank_mask:0xf\n\t"
                    "v_cndmask_b32_dpp %2, %11, %10, vcc row_ror:8 row_mask:0xf bank_mask:0xf\n\t"
                    "v_cndmask_b32_dpp %4, %13, %12, vcc row_ror:8 row_mask:0xf bank_mask:0xf\n\t"
                    "v_cndmask_b32_dpp %6, %15, %14, vcc row_ror:8 row_mask:0xf bank_mask:0xf\n\t"
                    "s_not_b64 vcc, vcc\n\t"
                    "v_cndmask_b32_dpp %1, %8, %9, vcc row_ror:8 row_mask:0xf bank_mask:0xf\n\t"
                    "v_cndmask_b32_dpp %3, %10, %11, vcc row_ror:8 row_mask:0xf bank_mask:0xf\n\t"
                    "v_cndmask_b32_dpp %5, %12, %13, vcc row_ror:8 row_mask:0xf bank_mask:0xf\n\t"
                    "v_cndmask_b32_dpp %7, %14, %15, vcc row_ror:8 row_mask:0xf bank_mask:0xf"
                    : "=&v"(n0), "=&v"(n1), "=&v"(n2), "=&v"(n3), "=&v"(n4), "=&v"(n5), "=&v"(n6), "=&v"(n7)
                    : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3]), "v"(a[4]), "v"(a[5]), "v"(a[6]), "v"(a[7]), "s"(lomask)
                    : "vcc");
                a[0] = n0; a[1] = n1; a[2] = n2; a[3] = n3; a[4] = n4; a[5] = n5; a[6] = n6; a[7] = n7;
            } else if constexpr (OP == 3) {
#pragma unroll
                for (int i = 0; i < CH; i += 2) {
                    const auto r = __builtin_amdgcn_permlane32_swap(a[i], a[i + 1], false, false);
                    a[i] = r[0];
                    a[i + 1] = r[1];
                    asm volatile("" : "+v"(a[i]), "+v"(a[i + 1]));
                }
            } else if constexpr (OP == 4) {
#pragma unroll
                for (int i = 0; i < CH; i += 2) {
                    const auto r = __builtin_amdgcn_permlane16_swap(a[i], a[i + 1], false, false);
                    a[i] = r[0];
                    a[i + 1] = r[1];
                    asm volatile("" : "+v"(a[i]), "+v"(a[i + 1]));
                }
            } else if constexpr (OP == 5) {  // one dependent chain
                a[0] = x3(a[0], t0, t1);
                asm volatile("" : "+v"(a[0]));
            } else if constexpr (OP == 6) {  // delta swap (transpose step): 2 shifts + 2 bitop3 per pair
#pragma unroll
                for (int i = 0; i < CH; i += 2) {
                    const uint32_t as = a[i] >> 4, bs = a[i + 1] << 4;
                    a[i] = __builtin_amdgcn_bitop3_b32(a[i], bs, 0x0F0F0F0Fu, 0xE4);      // (a&M)|(bs&~M)
                    a[i + 1] = __builtin_amdgcn_bitop3_b32(a[i + 1], as, 0x0F0F0F0Fu, 0xB8);  // (b&~M)|(as&M)
                    asm volatile("" : "+v"(a[i]), "+v"(a[i + 1]));
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

int main() {
    setvbuf(stdout, nullptr, _IONBF, 0);
    uint32_t *out;
    unsigned long long *clk;
    const int cus = 256;
    (void)hipMalloc(&out, (size_t)cus * 1024 * 4);
    (void)hipMalloc(&clk, 16);
    const char *names[] = {"v_bitop3", "v_xor", "cndmask_dpp swap", "permlane32_swap", "permlane16_swap", "bitop3 dep chain",
                           "delta swap"};
    // wave-instructions per wave per launch
    const double per_wave[] = {ITERS * STEPS * CH * 1.0, ITERS * STEPS * CH * 1.0, ITERS * STEPS * CH * 1.0,
                               ITERS * STEPS * CH / 2.0, ITERS * STEPS * CH / 2.0, ITERS * STEPS * 1.0,
                               ITERS * STEPS * CH * 2.0};
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int op = 0; op < 7; op++) {
        for (int wps = 1; wps <= 4; wps *= 2) {
            const int threads = 256 * wps;  // one block per CU, wps waves per SIMD
            auto launch = [&]() {
                switch (op) {
                    case 0: hipLaunchKernelGGL(k<0>, dim3(cus), dim3(threads), 0, 0, out, 1u, clk); break;
                    case 1: hipLaunchKernelGGL(k<1>, dim3(cus), dim3(threads), 0, 0, out, 1u, clk); break;
                    case 2: hipLaunchKernelGGL(k<2>, dim3(cus), dim3(threads), 0, 0, out, 1u, clk); break;
                    case 3: hipLaunchKernelGGL(k<3>, dim3(cus), dim3(threads), 0, 0, out, 1u, clk); break;
                    case 4: hipLaunchKernelGGL(k<4>, dim3(cus), dim3(threads), 0, 0, out, 1u, clk); break;
                    case 5: hipLaunchKernelGGL(k<5>, dim3(cus), dim3(threads), 0, 0, out, 1u, clk); break;
                    case 6: hipLaunchKernelGGL(k<6>, dim3(cus), dim3(threads), 0, 0, out, 1u, clk); break;
                }
            };
            fprintf(stderr, "op %d wps %d\n", op, wps);
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
            const double ghz = (double)h[0] / ((double)h[1] / 100.0) / 1e3;
            const double instr_per_simd = per_wave[op] * wps;
            printf("%-18s %d wave/SIMD: %.2f SIMD cycles per wave-instruction (kernel %.1f us, clock %.2f GHz)\n", names[op],
                   wps, ms * 1e3 * ghz * 1e3 / instr_per_simd, ms * 1e3, ghz);
        }
    }
    return 0;
}
