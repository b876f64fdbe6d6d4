// Memory-side lab for the half-plane C3 encode (round 2): 16 stripes of 128
// data rows read + 32 parity rows written (1 MiB rows), 2 KB column tiles per
// 256-thread workgroup, 512 persistent workgroups (2 per CU), and only an XOR
// fold for compute.  Varies what the real kernel fixes:
//   LAYOUT 0: the kernel's lane layout (lane = (block, half): 64 B of one row
//             block per lane, four dwordx4 per row at stride 64 B)
//   LAYOUT 1: same bytes, lane-contiguous (each dwordx4 instruction 1 KB contiguous)
//   DEPTH   : chunks of 32 rows in flight per wave (register staging)
//   BAR     : two s_barrier per chunk (the kernel's exchange structure)
// Diagnostic only.
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int K = 128, P = 32, NST = 16;
constexpr size_t S = 1 << 20;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int LAYOUT, int DEPTH, bool BAR, bool SPLIT = false>
__global__ void __launch_bounds__(256, 2) k_stream(uint8_t *base, uint32_t *sink, uint32_t RS, uint32_t TS, uint64_t SS) {
    const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int h = lane >> 5, blk = lane & 31;
    constexpr int TPS = S / 2048, NT = TPS * NST;
    uint32_t St[DEPTH][64];
    uint32_t acc[64];
    auto stage = [&](int tile, int c, uint32_t (&d)[64], int i0 = 0, int i1 = 4) {
        const int stripe = tile / TPS, ct = tile % TPS;
        const bool live = tile < NT;
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            base + (live ? (size_t)stripe * SS : 0), 0, live ? (int)(K * RS + TPS * TS) : 0, 0x00020000);
        uint32_t voff;
        if (LAYOUT == 0) voff = ct * TS + blk * 64 + 4 * h * RS;
        else voff = ct * TS + lane * 16;
        asm volatile("" : "+v"(voff));
#pragma unroll
        for (int i = 0; i < 4; i++)
#pragma unroll
            for (int q = 0; q < 4; q++) {
                if (i < i0 || i >= i1) continue;
                uint32_t so, vo;
                if (LAYOUT == 0) { so = (uint32_t)(32 * c + 8 * w + i) * RS; vo = voff + q * 16; }
                else { so = (uint32_t)(32 * c + 8 * w + i + 4 * (q >> 1)) * RS; vo = voff + (q & 1) * 1024; }
                const u32x4 x = __builtin_amdgcn_raw_buffer_load_b128(rs, vo, so, 0);
                d[16 * i + 4 * q] = x[0], d[16 * i + 4 * q + 1] = x[1], d[16 * i + 4 * q + 2] = x[2], d[16 * i + 4 * q + 3] = x[3];
            }
    };
    int tile = blockIdx.x;
#pragma unroll
    for (int d = 0; d < DEPTH; d++) stage(d < 4 ? tile : tile + gridDim.x, d % 4, St[d]);
    for (; tile < NT; tile += gridDim.x) {
#pragma unroll
        for (int c = 0; c < 4; c++) {
            constexpr int dummy = 0;
            (void)dummy;
            uint32_t(&cur)[64] = St[c % DEPTH];
#pragma unroll
            for (int j = 0; j < 64; j++) {
                if (c == 0) acc[j] = cur[j];
                else acc[j] ^= cur[j];
            }
#pragma unroll
            for (int j = 0; j < 64; j++) asm volatile("" : "+v"(acc[j])::"memory");
            const int nc = c + DEPTH;  // chunk index that reuses this slot
            if (SPLIT) {
                stage(nc < 4 ? tile : tile + gridDim.x, nc % 4, cur, 0, 2);
                __builtin_amdgcn_s_barrier();
                __builtin_amdgcn_s_barrier();
                stage(nc < 4 ? tile : tile + gridDim.x, nc % 4, cur, 2, 4);
            } else {
                stage(nc < 4 ? tile : tile + gridDim.x, nc % 4, cur);
            }
            if (BAR) {
                __builtin_amdgcn_s_barrier();
                __builtin_amdgcn_s_barrier();
            }
        }
        const int stripe = tile / TPS, ct = tile % TPS;
        const __amdgpu_buffer_rsrc_t ps = __builtin_amdgcn_make_buffer_rsrc(
            base + (size_t)stripe * SS + (size_t)K * RS, 0, (int)(P * RS + TPS * TS), 0x00020000);
        uint32_t voff;
        if (LAYOUT == 0) voff = ct * TS + blk * 64 + 4 * h * RS;
        else voff = ct * TS + lane * 16;
#pragma unroll
        for (int i = 0; i < 4; i++)
#pragma unroll
            for (int q = 0; q < 4; q++) {
                uint32_t so, vo;
                if (LAYOUT == 0) { so = (uint32_t)(8 * w + i) * RS; vo = voff + q * 16; }
                else { so = (uint32_t)(8 * w + i + 4 * (q >> 1)) * RS; vo = voff + (q & 1) * 1024; }
                const u32x4 v = u32x4{acc[16 * i + 4 * q], acc[16 * i + 4 * q + 1], acc[16 * i + 4 * q + 2], acc[16 * i + 4 * q + 3]};
                __builtin_amdgcn_raw_buffer_store_b128(v, ps, vo, so, 0);
            }
    }
    (void)sink;
}



// Deferred parity stores: tile t's 16 parity stores are issued 4 per chunk
// during tile t + grid's chunk loop (pend holds them), instead of as one burst
// at the end of tile t.  LAYOUT 0, DEPTH 1.
__global__ void __launch_bounds__(256, 2) k_stream_defer(uint8_t *base, uint32_t *sink, uint32_t RS, uint32_t TS, uint64_t SS) {
    const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int h = lane >> 5, blk = lane & 31;
    constexpr int TPS = S / 2048, NT = TPS * NST;
    uint32_t St[64], acc[64], pend[64];
    auto stage = [&](int tile, int c) {
        const int stripe = tile / TPS, ct = tile % TPS;
        const bool live = tile < NT;
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            base + (live ? (size_t)stripe * SS : 0), 0, live ? (int)(K * RS + TPS * TS) : 0, 0x00020000);
        uint32_t voff = ct * TS + blk * 64 + 4 * h * RS;
        asm volatile("" : "+v"(voff));
#pragma unroll
        for (int i = 0; i < 4; i++)
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const u32x4 x = __builtin_amdgcn_raw_buffer_load_b128(rs, voff + q * 16, (uint32_t)(32 * c + 8 * w + i) * RS, 0);
                St[16 * i + 4 * q] = x[0], St[16 * i + 4 * q + 1] = x[1], St[16 * i + 4 * q + 2] = x[2], St[16 * i + 4 * q + 3] = x[3];
            }
    };
    auto store_part = [&](int ptile, int i) {  // parity row 8w + i of tile ptile from pend
        if (ptile < 0) return;
        const int stripe = ptile / TPS, ct = ptile % TPS;
        const __amdgpu_buffer_rsrc_t ps = __builtin_amdgcn_make_buffer_rsrc(
            base + (size_t)stripe * SS + (size_t)K * RS, 0, (int)(P * RS + TPS * TS), 0x00020000);
        const uint32_t voff = ct * TS + blk * 64 + 4 * h * RS;
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const u32x4 v = u32x4{pend[16 * i + 4 * q], pend[16 * i + 4 * q + 1], pend[16 * i + 4 * q + 2], pend[16 * i + 4 * q + 3]};
            __builtin_amdgcn_raw_buffer_store_b128(v, ps, voff + q * 16, (uint32_t)(8 * w + i) * RS, 0);
        }
    };
    int tile = blockIdx.x, ptile = -1;
    stage(tile, 0);
    for (; tile < NT; tile += gridDim.x) {
#pragma unroll
        for (int c = 0; c < 4; c++) {
#pragma unroll
            for (int j = 0; j < 64; j++) {
                if (c == 0) acc[j] = St[j];
                else acc[j] ^= St[j];
            }
#pragma unroll
            for (int j = 0; j < 64; j++) asm volatile("" : "+v"(acc[j])::"memory");
            const int nc = c + 1;
            stage(nc < 4 ? tile : tile + gridDim.x, nc % 4);
            store_part(ptile, c);
        }
#pragma unroll
        for (int j = 0; j < 64; j++) pend[j] = acc[j];
        ptile = tile;
    }
#pragma unroll
    for (int i = 0; i < 4; i++) store_part(ptile, i);
    (void)sink;
}

typedef __attribute__((address_space(3))) void lvoid_t;
typedef __attribute__((address_space(3))) u32x4 lds_u4;
// LDS-DMA staging: each wave streams its 16 KB chunk (4 rows x 2 KB... as 16
// 1-KB pieces) into its own LDS slot, then reads it back with ds_read_b128.
template <int AUX, int SLOTS>
__global__ void __launch_bounds__(256, 2) k_dma(uint8_t *base, uint32_t *sink, uint32_t RS, uint32_t TS, uint64_t SS) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[4 * SLOTS * 16384];
    const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    constexpr int TPS = S / 2048, NT = TPS * NST;
    uint32_t acc[64];
    auto stage = [&](int tile, int c, int slot) {
        const int stripe = tile / TPS, ct = tile % TPS;
        const bool live = tile < NT;
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            base + (live ? (size_t)stripe * SS : 0), 0, live ? (int)(K * RS + TPS * TS) : 0, 0x00020000);
        uint32_t voff = ct * TS + lane * 16;
        asm volatile("" : "+v"(voff));
        uint8_t *img = lds + (w * SLOTS + slot) * 16384;
#pragma unroll
        for (int j = 0; j < 16; j++)  // piece j: row 32c + 8w + j/2, half j%2 of the 2 KB
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lvoid_t *)(img + j * 1024), 16, voff + (j & 1) * 1024,
                                                     (uint32_t)(32 * c + 8 * w + (j >> 1)) * RS, 0, AUX);
    };
    int tile = blockIdx.x;
#pragma unroll
    for (int d = 0; d < SLOTS; d++) stage(tile, d, d);
    for (; tile < NT; tile += gridDim.x) {
#pragma unroll
        for (int c = 0; c < 4; c++) {
            const int slot = c % SLOTS;
            // wait for this slot's 16 DMA (the younger slots' DMA stay in flight)
            if (SLOTS == 1) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
            const uint8_t *img = lds + (w * SLOTS + slot) * 16384;
#pragma unroll
            for (int j = 0; j < 16; j++) {
                const u32x4 x = *(const lds_u4 *)(uintptr_t)(img + j * 1024 + lane * 16);
                if (c == 0) { acc[4 * j] = x[0]; acc[4 * j + 1] = x[1]; acc[4 * j + 2] = x[2]; acc[4 * j + 3] = x[3]; }
                else { acc[4 * j] ^= x[0]; acc[4 * j + 1] ^= x[1]; acc[4 * j + 2] ^= x[2]; acc[4 * j + 3] ^= x[3]; }
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
            for (int j = 0; j < 64; j++) asm volatile("" : "+v"(acc[j])::"memory");
            const int nc = c + SLOTS;
            stage(nc < 4 ? tile : tile + gridDim.x, nc % 4, slot);
        }
        const int stripe = tile / TPS, ct = tile % TPS;
        const __amdgpu_buffer_rsrc_t ps = __builtin_amdgcn_make_buffer_rsrc(
            base + (size_t)stripe * SS + (size_t)K * RS, 0, (int)(P * RS + TPS * TS), 0x00020000);
        const uint32_t voff = ct * TS + lane * 16;
#pragma unroll
        for (int j = 0; j < 16; j++) {
            const u32x4 v = u32x4{acc[4 * j], acc[4 * j + 1], acc[4 * j + 2], acc[4 * j + 3]};
            __builtin_amdgcn_raw_buffer_store_b128(v, ps, voff + (j & 1) * 1024, (uint32_t)(8 * w + (j >> 1)) * RS, 0);
        }
    }
    (void)sink;
}


// Calibration: plain grid-stride float4 copy (read n bytes, write n bytes).
__global__ void __launch_bounds__(256) k_copy(const u32x4 *src, u32x4 *dst, size_t n16) {
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n16; i += (size_t)gridDim.x * 256) dst[i] = src[i];
}
// Calibration: copy with U float4 per thread per iteration (a wave moves
// U KiB per step, each lane's U pieces 1 KiB apart), half the bytes read
// and half written, as the guide's "float4 copy" figure.
template <int U>
__global__ void __launch_bounds__(256) k_copyu(const u32x4 *src, u32x4 *dst, size_t n16) {
    const size_t step = (size_t)gridDim.x * 256 * U;
    for (size_t i = (size_t)blockIdx.x * 256 * U + threadIdx.x; i < n16; i += step) {
        u32x4 v[U];
#pragma unroll
        for (int j = 0; j < U; j++) v[j] = i + 256 * j < n16 ? src[i + 256 * j] : u32x4{0, 0, 0, 0};
#pragma unroll
        for (int j = 0; j < U; j++)
            if (i + 256 * j < n16) dst[i + 256 * j] = v[j];
    }
}
// Calibration: plain grid-stride float4 read (XOR fold, one store per thread).
__global__ void __launch_bounds__(256) k_read(const u32x4 *src, uint32_t *sink, size_t n16) {
    u32x4 a = {0, 0, 0, 0};
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n16; i += (size_t)gridDim.x * 256) a ^= src[i];
    if ((a[0] ^ a[1] ^ a[2] ^ a[3]) == 0x12345678u) sink[0] = 1;
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
    uint8_t *base;
    uint32_t *sink;
    const size_t bytes = (size_t)NST * (K + P) * S;
    (void)hipMalloc(&base, (size_t)NST * (K + P) * (S + 65536));
    (void)hipMalloc(&sink, 64);
    (void)hipMemset(base, 0x5A, bytes);
    const double alg = (double)bytes;
    auto rep = [&](const char *n, float us) {
        printf("%-22s %8.1f us  %7.1f GB/s  frac %.3f\n", n, us, alg / us / 1e3, alg / us / 1e3 / 8000.0);
    };
    const uint32_t RS = (uint32_t)S, TS = 2048;
    const uint64_t SS = (K + P) * S;
    rep("regs d1", timeit([&] { hipLaunchKernelGGL((k_stream<0, 1, false>), dim3(512), dim3(256), 0, 0, base, sink, RS, TS, SS); }));
    rep("regs d1 bar", timeit([&] { hipLaunchKernelGGL((k_stream<0, 1, true>), dim3(512), dim3(256), 0, 0, base, sink, RS, TS, SS); }));
    rep("regs d1 split", timeit([&] { hipLaunchKernelGGL((k_stream<0, 1, false, true>), dim3(512), dim3(256), 0, 0, base, sink, RS, TS, SS); }));
    rep("regs d2", timeit([&] { hipLaunchKernelGGL((k_stream<0, 2, false>), dim3(512), dim3(256), 0, 0, base, sink, RS, TS, SS); }));
    rep("contig d1", timeit([&] { hipLaunchKernelGGL((k_stream<1, 1, false>), dim3(512), dim3(256), 0, 0, base, sink, RS, TS, SS); }));
    rep("contig d1 bar", timeit([&] { hipLaunchKernelGGL((k_stream<1, 1, true>), dim3(512), dim3(256), 0, 0, base, sink, RS, TS, SS); }));
    rep("regs d1 grid1024", timeit([&] { hipLaunchKernelGGL((k_stream<0, 1, false>), dim3(1024), dim3(256), 0, 0, base, sink, RS, TS, SS); }));
    rep("defer d1", timeit([&] { hipLaunchKernelGGL(k_stream_defer, dim3(512), dim3(256), 0, 0, base, sink, RS, TS, SS); }));
    {
        const uint32_t RSp = (uint32_t)S + 3072;
        const uint64_t SSp = (uint64_t)(K + P) * RSp;
        rep("regs d1 rowpad 3072", timeit([&] { hipLaunchKernelGGL((k_stream<0, 1, false>), dim3(512), dim3(256), 0, 0, base, sink, RSp, TS, SSp); }));
        rep("defer d1 rowpad 3072", timeit([&] { hipLaunchKernelGGL(k_stream_defer, dim3(512), dim3(256), 0, 0, base, sink, RSp, TS, SSp); }));
    }
    // row stride padding: rows exactly 1 MiB apart alias in the low 20 address bits
    for (uint32_t pad : {256u, 2048u, 4096u, 8192u, 65536u}) {
        char nm[64];
        snprintf(nm, sizeof nm, "regs d1 rowpad %u", pad);
        const uint32_t RSp = (uint32_t)S + pad;
        const uint64_t SSp = (uint64_t)(K + P) * RSp;
        rep(nm, timeit([&] { hipLaunchKernelGGL((k_stream<0, 1, false>), dim3(512), dim3(256), 0, 0, base, sink, RSp, TS, SSp); }));
    }
    {
        const size_t half = bytes / 2, n16 = half / 16;
        for (int g : {2048, 4096, 8192, 16384}) {
            char nm[64];
            snprintf(nm, sizeof nm, "copy grid %d", g);
            rep(nm, timeit([&] { hipLaunchKernelGGL(k_copy, dim3(g), dim3(256), 0, 0, (const u32x4 *)base, (u32x4 *)(base + half), n16); }));
        }
        for (int g : {1024, 2048, 4096}) {
            char nm[64];
            snprintf(nm, sizeof nm, "copy x4 grid %d", g);
            rep(nm, timeit([&] { hipLaunchKernelGGL(k_copyu<4>, dim3(g), dim3(256), 0, 0, (const u32x4 *)base, (u32x4 *)(base + half), n16); }));
            snprintf(nm, sizeof nm, "copy x8 grid %d", g);
            rep(nm, timeit([&] { hipLaunchKernelGGL(k_copyu<8>, dim3(g), dim3(256), 0, 0, (const u32x4 *)base, (u32x4 *)(base + half), n16); }));
        }
        for (int g : {2048, 8192}) {
            char nm[64];
            snprintf(nm, sizeof nm, "read-only grid %d", g);
            const float us = timeit([&] { hipLaunchKernelGGL(k_read, dim3(g), dim3(256), 0, 0, (const u32x4 *)base, sink, bytes / 16); });
            rep(nm, us);
        }
    }
    return hipDeviceSynchronize() != hipSuccess;
}
