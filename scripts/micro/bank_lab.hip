// VGPR bank-conflict lab (gfx950): streams of independent v_perm_b32 /
// v_bitop3_b32 with fixed physical registers whose source operands sit in
// distinct banks (reg % 4) or collide.  Whole-kernel time at 8 waves/SIMD.
#include <hip/hip_runtime.h>

#include <cstdio>

#define REP8(x) x x x x x x x x
#define REP32(x) REP8(x) REP8(x) REP8(x) REP8(x)

template <int V>
__global__ void __launch_bounds__(256) k(uint32_t *out, int iters) {
    asm volatile("v_mov_b32 v40, %0\n v_mov_b32 v41, 3\n v_mov_b32 v42, 5\n v_mov_b32 v43, 7\n"
                 "v_mov_b32 v45, 11\n v_mov_b32 v46, 13\n v_mov_b32 v49, 17\n v_mov_b32 v47, 19\n v_mov_b32 v53, 23" ::"v"(threadIdx.x)
                 : "v40", "v41", "v42", "v43", "v45", "v46", "v47", "v49", "v53");
    for (int it = 0; it < iters; it++) {
        // destinations rotate over v32..v39 (distinct from the sources), so the ops are independent
        if (V == 0)  // v_perm, sources in banks 1, 2, 3
            asm volatile(REP32("v_perm_b32 v32, v41, v42, v43\n v_perm_b32 v33, v41, v42, v43\n v_perm_b32 v34, v41, v42, v43\n v_perm_b32 v35, v41, v42, v43\n")
                         ::: "v32", "v33", "v34", "v35");
        if (V == 1)  // v_perm, src0 and src2 in bank 1
            asm volatile(REP32("v_perm_b32 v32, v41, v42, v45\n v_perm_b32 v33, v41, v42, v45\n v_perm_b32 v34, v41, v42, v45\n v_perm_b32 v35, v41, v42, v45\n")
                         ::: "v32", "v33", "v34", "v35");
        if (V == 2)  // v_perm, all three sources in bank 1
            asm volatile(REP32("v_perm_b32 v32, v41, v45, v49\n v_perm_b32 v33, v41, v45, v49\n v_perm_b32 v34, v41, v45, v49\n v_perm_b32 v35, v41, v45, v49\n")
                         ::: "v32", "v33", "v34", "v35");
        if (V == 3)  // v_bitop3, banks 1, 2, 3
            asm volatile(REP32("v_bitop3_b32 v32, v41, v42, v43 bitop3:0x96\n v_bitop3_b32 v33, v41, v42, v43 bitop3:0x96\n v_bitop3_b32 v34, v41, v42, v43 bitop3:0x96\n v_bitop3_b32 v35, v41, v42, v43 bitop3:0x96\n")
                         ::: "v32", "v33", "v34", "v35");
        if (V == 4)  // v_bitop3, all in bank 1
            asm volatile(REP32("v_bitop3_b32 v32, v41, v45, v49 bitop3:0x96\n v_bitop3_b32 v33, v41, v45, v49 bitop3:0x96\n v_bitop3_b32 v34, v41, v45, v49 bitop3:0x96\n v_bitop3_b32 v35, v41, v45, v49 bitop3:0x96\n")
                         ::: "v32", "v33", "v34", "v35");
        if (V == 5)  // v_perm, src0/src1 consecutive (a table pair), selector in bank 0 (v40)
            asm volatile(REP32("v_perm_b32 v32, v42, v41, v40\n v_perm_b32 v33, v42, v41, v40\n v_perm_b32 v34, v42, v41, v40\n v_perm_b32 v35, v42, v41, v40\n")
                         ::: "v32", "v33", "v34", "v35");
        if (V == 6)  // v_perm with the same register as src0 and src1 (2-bit group table), selector other bank
            asm volatile(REP32("v_perm_b32 v32, v41, v41, v42\n v_perm_b32 v33, v41, v41, v42\n v_perm_b32 v34, v41, v41, v42\n v_perm_b32 v35, v41, v41, v42\n")
                         ::: "v32", "v33", "v34", "v35");
        if (V == 7)  // v_xor_b32 VOP2, banks 1, 2
            asm volatile(REP32("v_xor_b32 v32, v41, v42\n v_xor_b32 v33, v41, v42\n v_xor_b32 v34, v41, v42\n v_xor_b32 v35, v41, v42\n")
                         ::: "v32", "v33", "v34", "v35");
    }
    uint32_t r;
    asm volatile("v_xor_b32 %0, v32, v35" : "=v"(r));
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

int main() {
    uint32_t *out;
    const int cus = 256, wps = 8, blocks = cus * wps, iters = 64;
    (void)hipMalloc(&out, (size_t)blocks * 256 * 4);
    const char *names[] = {"perm banks 1,2,3", "perm src0/src2 same bank", "perm all same bank", "bitop3 banks 1,2,3",
                           "bitop3 all same bank", "perm table pair + sel", "perm same-reg table", "xor VOP2"};
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const double clk_ghz = 2.2;  // nominal; relative comparisons only
    for (int v = 0; v < 8; v++) {
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
        const double instr_per_simd = (double)iters * 128 * wps;
        printf("%-26s %.2f SIMD cycles/instr at %.1f GHz (kernel %.1f us)\n", names[v],
               ms * 1e3 * clk_ghz * 1e3 / instr_per_simd, clk_ghz, ms * 1e3);
    }
    return 0;
}
