// Issue cost of the byte-permute multiply's index extraction on gfx950:
// v_lshrrev_b32 / v_and_b32 (today: two 32-bit shifts per lo/hi dword pair)
// against one v_lshrrev_b64 over the pair, at 8 waves per SIMD, independent
// destinations.  Whole-kernel time -> SIMD cycles per wave64 instruction.
#include <hip/hip_runtime.h>
#include <cstdio>

#define S32(d, s) "v_lshrrev_b32 v" #d ", 3, v" #s "\n"
#define A32(d, s) "v_and_b32 v" #d ", 0x7070707, v" #s "\n"
#define S64(d, s) "v_lshrrev_b64 v[" #d ":" #d "+1], 3, v[" #s ":" #s "+1]\n"
#define B32 S32(32, 40) S32(33, 41) S32(34, 42) S32(35, 43) S32(36, 44) S32(37, 45) S32(38, 46) S32(39, 47) \
            S32(32, 48) S32(33, 49) S32(34, 50) S32(35, 51)
#define BAND A32(32, 40) A32(33, 41) A32(34, 42) A32(35, 43) A32(36, 44) A32(37, 45) A32(38, 46) A32(39, 47) \
             A32(32, 48) A32(33, 49) A32(34, 50) A32(35, 51)
#define B64 S64(32, 40) S64(34, 42) S64(36, 44) S64(38, 46) S64(32, 48) S64(34, 50) S64(36, 52) S64(38, 54) \
            S64(32, 56) S64(34, 58) S64(36, 60) S64(38, 62)

template <int V>
__global__ void __launch_bounds__(256) k(uint32_t *out, int iters) {
    for (int it = 0; it < iters; it++) {
        if (V == 0) asm volatile(B32 B32 B32 B32 ::: "v32", "v33", "v34", "v35", "v36", "v37", "v38", "v39");
        if (V == 1) asm volatile(BAND BAND BAND BAND ::: "v32", "v33", "v34", "v35", "v36", "v37", "v38", "v39");
        if (V == 2) asm volatile(B64 B64 B64 B64 ::: "v32", "v33", "v34", "v35", "v36", "v37", "v38", "v39");
    }
    uint32_t r;
    asm volatile("v_xor_b32 %0, v32, v35" : "=v"(r));
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

int main() {
    uint32_t *out;
    const int cus = 256, wps = 8, blocks = cus * wps, iters = 512;
    if (hipMalloc(&out, (size_t)blocks * 256 * 4) != hipSuccess) return 1;
    const char *names[] = {"v_lshrrev_b32", "v_and_b32", "v_lshrrev_b64"};
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int pass = 0; pass < 2; pass++)
        for (int v = 0; v < 3; v++) {
            auto launch = [&]() {
                if (v == 0) hipLaunchKernelGGL(k<0>, dim3(blocks), dim3(256), 0, 0, out, iters);
                if (v == 1) hipLaunchKernelGGL(k<1>, dim3(blocks), dim3(256), 0, 0, out, iters);
                if (v == 2) hipLaunchKernelGGL(k<2>, dim3(blocks), dim3(256), 0, 0, out, iters);
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
            printf("%-16s %.2f SIMD cycles/instr at 2.2 GHz (kernel %.1f us)\n", names[v], ms * 1e3 * 2.2e3 / instr_per_simd,
                   ms * 1e3);
        }
    return 0;
}
