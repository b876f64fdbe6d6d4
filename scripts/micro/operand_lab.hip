// VGPR operand-read lab (gfx950): independent v_perm_b32 / v_bitop3_b32 whose
// source registers rotate over many VGPRs ("fresh" operands, as in the encode
// kernel where every perm reads a new table pair) vs a fixed operand set, and
// with one operand an SGPR.  Whole-kernel time at 8 waves/SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <string>

#define R4(a,b,c,d) a b c d
// fresh: sources walk v40..v63 (24 regs), banks mixed but distinct per instr
#define PF(d,s0,s1,s2) "v_perm_b32 v" #d ", v" #s0 ", v" #s1 ", v" #s2 "\n"
#define BF(d,s0,s1,s2) "v_bitop3_b32 v" #d ", v" #s0 ", v" #s1 ", v" #s2 " bitop3:0x96\n"
#define PS(d,s1,s2) "v_perm_b32 v" #d ", s8, v" #s1 ", v" #s2 "\n"
#define FRESH_P PF(32,41,40,50) PF(33,43,42,51) PF(34,45,44,52) PF(35,47,46,53) PF(36,49,48,54) PF(37,57,56,55) \
                PF(38,59,58,50) PF(39,61,60,51) PF(32,63,62,52) PF(33,41,44,53) PF(34,43,46,54) PF(35,45,48,55)
#define FIXED_P PF(32,41,42,43) PF(33,41,42,43) PF(34,41,42,43) PF(35,41,42,43) PF(36,41,42,43) PF(37,41,42,43) \
                PF(38,41,42,43) PF(39,41,42,43) PF(32,41,42,43) PF(33,41,42,43) PF(34,41,42,43) PF(35,41,42,43)
#define SGPR_P PS(32,40,50) PS(33,42,51) PS(34,44,52) PS(35,46,53) PS(36,48,54) PS(37,56,55) \
               PS(38,58,50) PS(39,60,51) PS(32,62,52) PS(33,44,53) PS(34,46,54) PS(35,48,55)
#define FRESH_B BF(32,41,42,51) BF(33,43,44,53) BF(34,45,46,55) BF(35,47,48,57) BF(36,49,50,59) BF(37,61,62,63) \
                BF(38,41,46,51) BF(39,43,48,53) BF(32,45,50,55) BF(33,47,58,57) BF(34,49,54,59) BF(35,61,42,63)
// bank probes: a fixed operand set whose registers share one bank (index mod 4),
// span three banks, or repeat one register as both table operands
#define FIX(s0,s1,s2) PF(32,s0,s1,s2) PF(33,s0,s1,s2) PF(34,s0,s1,s2) PF(35,s0,s1,s2) PF(36,s0,s1,s2) PF(37,s0,s1,s2) \
                PF(38,s0,s1,s2) PF(39,s0,s1,s2) PF(32,s0,s1,s2) PF(33,s0,s1,s2) PF(34,s0,s1,s2) PF(35,s0,s1,s2)
#define FIXB(s0,s1,s2) BF(32,s0,s1,s2) BF(33,s0,s1,s2) BF(34,s0,s1,s2) BF(35,s0,s1,s2) BF(36,s0,s1,s2) BF(37,s0,s1,s2) \
                BF(38,s0,s1,s2) BF(39,s0,s1,s2) BF(32,s0,s1,s2) BF(33,s0,s1,s2) BF(34,s0,s1,s2) BF(35,s0,s1,s2)
#define XF(d,s0,s1) "v_xor_b32 v" #d ", v" #s0 ", v" #s1 "\n"
#define FIXX(s0,s1) XF(32,s0,s1) XF(33,s0,s1) XF(34,s0,s1) XF(35,s0,s1) XF(36,s0,s1) XF(37,s0,s1) \
                XF(38,s0,s1) XF(39,s0,s1) XF(32,s0,s1) XF(33,s0,s1) XF(34,s0,s1) XF(35,s0,s1)
#define MIX PF(32,41,40,50) BF(20,21,22,32) PF(33,43,42,51) BF(23,24,25,33) PF(34,45,44,52) BF(26,27,28,34) \
            PF(35,47,46,53) BF(20,21,22,35) PF(36,49,48,54) BF(23,24,25,36) PF(37,57,56,55) BF(26,27,28,37)

template <int V>
__global__ void __launch_bounds__(256) k(uint32_t *out, int iters) {
    asm volatile("s_mov_b32 s8, 0x01020304" ::: "s8");
    for (int it = 0; it < iters; it++) {
        if (V == 0) asm volatile(FRESH_P FRESH_P FRESH_P FRESH_P ::: "v32","v33","v34","v35","v36","v37","v38","v39");
        if (V == 1) asm volatile(FIXED_P FIXED_P FIXED_P FIXED_P ::: "v32","v33","v34","v35","v36","v37","v38","v39");
        if (V == 2) asm volatile(SGPR_P SGPR_P SGPR_P SGPR_P ::: "v32","v33","v34","v35","v36","v37","v38","v39");
        if (V == 3) asm volatile(FRESH_B FRESH_B FRESH_B FRESH_B ::: "v32","v33","v34","v35","v36","v37","v38","v39");
        if (V == 4) asm volatile(MIX MIX MIX MIX ::: "v20","v23","v26","v32","v33","v34","v35","v36","v37");
        if (V == 5) asm volatile(FIX(40,44,48) FIX(40,44,48) FIX(40,44,48) FIX(40,44,48) ::: "v32","v33","v34","v35","v36","v37","v38","v39");
        if (V == 6) asm volatile(FIX(40,41,42) FIX(40,41,42) FIX(40,41,42) FIX(40,41,42) ::: "v32","v33","v34","v35","v36","v37","v38","v39");
        if (V == 7) asm volatile(FIX(40,40,42) FIX(40,40,42) FIX(40,40,42) FIX(40,40,42) ::: "v32","v33","v34","v35","v36","v37","v38","v39");
        if (V == 8) asm volatile(FIX(40,44,41) FIX(40,44,41) FIX(40,44,41) FIX(40,44,41) ::: "v32","v33","v34","v35","v36","v37","v38","v39");
        if (V == 9) asm volatile(FIXB(40,44,48) FIXB(40,44,48) FIXB(40,44,48) FIXB(40,44,48) ::: "v32","v33","v34","v35","v36","v37","v38","v39");
        if (V == 11) asm volatile(FIXB(40,44,41) FIXB(40,44,41) FIXB(40,44,41) FIXB(40,44,41) ::: "v32","v33","v34","v35","v36","v37","v38","v39");
        if (V == 12) asm volatile(FIXX(40,44) FIXX(40,44) FIXX(40,44) FIXX(40,44) ::: "v32","v33","v34","v35","v36","v37","v38","v39");
        if (V == 13) asm volatile(FIXX(40,41) FIXX(40,41) FIXX(40,41) FIXX(40,41) ::: "v32","v33","v34","v35","v36","v37","v38","v39");
        if (V == 14) asm volatile(FIXB(40,40,41) FIXB(40,40,41) FIXB(40,40,41) FIXB(40,40,41) ::: "v32","v33","v34","v35","v36","v37","v38","v39");
        if (V == 10) asm volatile(FIXB(40,41,42) FIXB(40,41,42) FIXB(40,41,42) FIXB(40,41,42) ::: "v32","v33","v34","v35","v36","v37","v38","v39");
    }
    uint32_t r;
    asm volatile("v_xor_b32 %0, v32, v35" : "=v"(r));
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

int main() {
    uint32_t *out;
    const int cus = 256, wps = 8, blocks = cus * wps, iters = 256;
    (void)hipMalloc(&out, (size_t)blocks * 256 * 4);
    const char *names[] = {"perm fresh vvv", "perm fixed vvv", "perm fresh svv", "bitop3 fresh", "perm+bitop3 mix",
                           "perm 1 bank", "perm 3 banks", "perm s0=s1", "perm 2 banks", "bitop3 1 bank", "bitop3 3 banks",
                           "bitop3 2 banks", "xor 1 bank", "xor 2 banks", "bitop3 a,a,b"};
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int v = 0; v < 15; v++) {
        auto launch = [&]() {
            switch (v) {
                case 0: hipLaunchKernelGGL(k<0>, dim3(blocks), dim3(256), 0, 0, out, iters); break;
                case 1: hipLaunchKernelGGL(k<1>, dim3(blocks), dim3(256), 0, 0, out, iters); break;
                case 2: hipLaunchKernelGGL(k<2>, dim3(blocks), dim3(256), 0, 0, out, iters); break;
                case 3: hipLaunchKernelGGL(k<3>, dim3(blocks), dim3(256), 0, 0, out, iters); break;
                case 4: hipLaunchKernelGGL(k<4>, dim3(blocks), dim3(256), 0, 0, out, iters); break;
                case 5: hipLaunchKernelGGL(k<5>, dim3(blocks), dim3(256), 0, 0, out, iters); break;
                case 6: hipLaunchKernelGGL(k<6>, dim3(blocks), dim3(256), 0, 0, out, iters); break;
                case 7: hipLaunchKernelGGL(k<7>, dim3(blocks), dim3(256), 0, 0, out, iters); break;
                case 8: hipLaunchKernelGGL(k<8>, dim3(blocks), dim3(256), 0, 0, out, iters); break;
                case 9: hipLaunchKernelGGL(k<9>, dim3(blocks), dim3(256), 0, 0, out, iters); break;
                case 10: hipLaunchKernelGGL(k<10>, dim3(blocks), dim3(256), 0, 0, out, iters); break;
                case 11: hipLaunchKernelGGL(k<11>, dim3(blocks), dim3(256), 0, 0, out, iters); break;
                case 12: hipLaunchKernelGGL(k<12>, dim3(blocks), dim3(256), 0, 0, out, iters); break;
                case 13: hipLaunchKernelGGL(k<13>, dim3(blocks), dim3(256), 0, 0, out, iters); break;
                case 14: hipLaunchKernelGGL(k<14>, dim3(blocks), dim3(256), 0, 0, out, iters); break;
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
        const double instr_per_simd = (double)iters * 48 * wps;
        printf("%-18s %.2f SIMD cycles/instr at 2.2 GHz (kernel %.1f us)\n", names[v], ms * 1e3 * 2.2e3 / instr_per_simd, ms * 1e3);
    }
    return 0;
}
