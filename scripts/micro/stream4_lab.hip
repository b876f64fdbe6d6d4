// Memory-side lab for the C3 encode, round 3, part 2: does separating the
// read and write streams in time lift the 128-read / 32-write row pattern?
//
// stream3_lab measured on one box: the C3 pattern with loads only 357 us, with
// stores only 99 us, both at once 528 us (0.635 of 8 TB/s), i.e. mixing costs
// ~70 us over running the two halves back to back (456 us, 0.735).  Here the
// same XOR-fold kernel gates its loads and stores on the chip-wide realtime
// clock (s_memrealtime, 100 MHz, the same counter on every CU): a period of P
// ticks is split into a read window [0, R) and a write window [R, P); a wave
// issues parity stores only inside a write window and chunk loads only inside
// a read window.  Every wait ends within P ticks (the modulo always comes
// round), so the kernel cannot hang.
//
// 16 stripes of 160 rows (rows staggered by 3 KiB), 2 KB column tiles, 2.68 GB
// per launch.  Diagnostic only.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

constexpr int K = 128, P = 32, NST = 16;
constexpr uint32_t S = 1 << 20;
constexpr int TW = 2048, TPS = S / TW, NT = TPS * NST;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t phase_of(uint32_t period) {
    return (uint32_t)(__builtin_amdgcn_s_memrealtime() % period);
}
// wait until the clock is inside [lo, hi) of the period
__device__ __forceinline__ void wait_window(uint32_t period, uint32_t lo, uint32_t hi) {
    if (period == 0) return;
    for (;;) {
        const uint32_t ph = phase_of(period);
        if (ph >= lo && ph < hi) break;
        __builtin_amdgcn_s_sleep(2);
    }
}

// GATE: 0 none, 1 stores only gated, 2 stores and loads gated
// NP: one tile per workgroup (grid = tiles), else persistent over tiles
template <int GATE, bool NP>
__global__ void __launch_bounds__(256, 2) k_c3p(uint8_t *base, uint32_t RS, uint64_t SS, uint32_t period, uint32_t rwin) {
    constexpr int RPW = 8, RSTEP = 32, NSTEP = K / RSTEP;
    const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint32_t St[64], acc[64];
    auto stage = [&](int t, int c) {
        const int stripe = t / TPS, ct = t - stripe * TPS;
        const bool live = t < NT;
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            base + (live ? (size_t)stripe * SS : 0), 0, live ? (int)(K * RS) : 0, 0x00020000);
        uint32_t voff = (uint32_t)ct * TW + (uint32_t)lane * 16;
        asm volatile("" : "+v"(voff));
#pragma unroll
        for (int q = 0; q < 16; q++) {
            const int j = q / 2, pc = q % 2;
            const uint32_t so = (uint32_t)(RSTEP * c + RPW * w + j) * RS;
            const u32x4 x = __builtin_amdgcn_raw_buffer_load_b128(rs, voff + pc * 1024, so, 0);
            St[4 * q] = x[0], St[4 * q + 1] = x[1], St[4 * q + 2] = x[2], St[4 * q + 3] = x[3];
        }
    };
    auto tile_body = [&](int t, int tnext) {
#pragma unroll
        for (int c = 0; c < NSTEP; c++) {
#pragma unroll
            for (int j = 0; j < 64; j++) acc[j] = c == 0 ? St[j] : acc[j] ^ St[j];
#pragma unroll
            for (int j = 0; j < 64; j++) asm volatile("" : "+v"(acc[j])::"memory");
            if (c < NSTEP - 1) stage(t, c + 1);
            else if (tnext >= 0 && GATE < 2) stage(tnext, 0);
        }
        const int stripe = t / TPS, ct = t - stripe * TPS;
        const __amdgpu_buffer_rsrc_t ps = __builtin_amdgcn_make_buffer_rsrc(
            base + (size_t)stripe * SS + (size_t)K * RS, 0, (int)(P * RS), 0x00020000);
        if (GATE >= 1) wait_window(period, rwin, period);
        const uint32_t voff = (uint32_t)ct * TW + (uint32_t)lane * 16;
#pragma unroll
        for (int q = 0; q < 16; q++) {
            const int j = q / 2, pc = q % 2;
            const u32x4 v = u32x4{acc[4 * q], acc[4 * q + 1], acc[4 * q + 2], acc[4 * q + 3]};
            __builtin_amdgcn_raw_buffer_store_b128(v, ps, voff + pc * 1024, (uint32_t)(8 * w + j) * RS, 0);
        }
        if (GATE >= 2 && tnext >= 0) {
            wait_window(period, 0, rwin);
            stage(tnext, 0);
        }
    };
    if (NP) {
        const int t = blockIdx.x;
        if (t >= NT) return;
        if (GATE >= 2) wait_window(period, 0, rwin);
        stage(t, 0);
        tile_body(t, -1);
        return;
    }
    int t = blockIdx.x;
    if (GATE >= 2) wait_window(period, 0, rwin);
    stage(t, 0);
    for (; t < NT; t += gridDim.x) tile_body(t, t + (int)gridDim.x < NT ? t + (int)gridDim.x : -1);
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
    setvbuf(stdout, nullptr, _IONBF, 0);
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const uint32_t RS = S + 3072;
    const uint64_t SS = (uint64_t)(K + P) * RS;
    uint8_t *base;
    const size_t bytes = (size_t)NST * SS;
    if (hipMalloc(&base, bytes + (64 << 20)) != hipSuccess) return 1;
    (void)hipMemset(base, 0x5A, bytes);
    const double alg = (double)NST * (K + P) * S;
    auto rep = [&](const char *n, float us) {
        printf("%-44s %8.1f us  %7.1f GB/s  frac %.3f\n", n, us, alg / us / 1e3, alg / us / 1e3 / 8000.0);
    };
    char nm[96];
    for (int pass = 0; pass < 2; pass++) {
        printf("# pass %d\n", pass);
        rep("ungated persistent", timeit([&] { hipLaunchKernelGGL((k_c3p<0, false>), dim3(2 * cus), dim3(256), 0, 0, base, RS, SS, 0u, 0u); }));
        rep("ungated one tile per wg", timeit([&] { hipLaunchKernelGGL((k_c3p<0, true>), dim3(NT), dim3(256), 0, 0, base, RS, SS, 0u, 0u); }));
        for (uint32_t per : {200u, 500u, 1000u, 2000u, 3000u, 5000u}) {
            for (int rpct : {70, 78, 85}) {
                const uint32_t rw = per * rpct / 100;
                snprintf(nm, sizeof nm, "pers gate=st+ld P=%u R=%d%%", per, rpct);
                rep(nm, timeit([&] { hipLaunchKernelGGL((k_c3p<2, false>), dim3(2 * cus), dim3(256), 0, 0, base, RS, SS, per, rw); }));
                snprintf(nm, sizeof nm, "pers gate=st P=%u R=%d%%", per, rpct);
                rep(nm, timeit([&] { hipLaunchKernelGGL((k_c3p<1, false>), dim3(2 * cus), dim3(256), 0, 0, base, RS, SS, per, rw); }));
                snprintf(nm, sizeof nm, "np gate=st+ld P=%u R=%d%%", per, rpct);
                rep(nm, timeit([&] { hipLaunchKernelGGL((k_c3p<2, true>), dim3(NT), dim3(256), 0, 0, base, RS, SS, per, rw); }));
            }
        }
    }
    return hipDeviceSynchronize() != hipSuccess;
}
