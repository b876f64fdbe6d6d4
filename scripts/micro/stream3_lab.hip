// Memory-side lab for the C3 encode, round 3: what the 128-read / 32-write
// row pattern of one 1 MiB stripe can reach on MI355X, with an XOR fold in
// place of the transform.  16 stripes of 160 rows (rows staggered by 3 KiB, as
// the bench lays them out), 2.68 GB per launch.
//
// Varied (the round-2 lab fixed all of these):
//   TW      contiguous bytes of each row per tile: 2, 4 or 8 KB (a wave still
//           stages 16 KB per chunk: 8 rows x 2 KB, 4 x 4 KB or 2 x 8 KB)
//   ORDER   0: tile t = stripe * tiles_per_stripe + column tile (round 2: all
//           workgroups sweep one stripe together); 1: stripe-interleaved
//           (t % 16 = stripe): concurrent workgroups spread over 16 stripes
//   WGCU    workgroups per CU (persistent grid = WGCU * 256), with the
//           accumulator halved (32 dwords, stored twice) at 4 per CU so the
//           kernel fits 128 VGPRs
//   PST     parity stores: 0 = the kernel's lane layout (lane = 64-byte
//           block, 4 x 16 B per row); 1 = lane-contiguous (1 KB per store
//           instruction)
//   NP      1: one tile per workgroup, not persistent (grid = tiles)
// plus streaming calibrations with the same 4:1 read/write byte ratio.
// Diagnostic only.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

constexpr int K = 128, P = 32, NST = 16;
constexpr uint32_t S = 1 << 20;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int TW, int ORDER, int WGCU, int PST, bool NP, int IO = 0>
__global__ void __launch_bounds__(256, WGCU) k_c3(uint8_t *base, uint32_t RS, uint64_t SS) {
    constexpr int TPS = S / TW, NT = TPS * NST;
    constexpr int RPW = 16384 / TW;   // rows a wave stages per step (8, 4, 2): 16 KB
    constexpr int RSTEP = 4 * RPW;    // rows a workgroup stages per step
    constexpr int NSTEP = K / RSTEP;  // steps per tile (4, 8, 16)
    constexpr int PPR = TW / 1024;    // 1 KB pieces per row (2, 4, 8)
    constexpr int ACC = WGCU >= 4 ? 32 : 64;
    const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint32_t St[64], acc[ACC];
    auto loc = [&](int t, int &stripe, int &ct) {
        if (ORDER == 0) { stripe = t / TPS; ct = t - stripe * TPS; }
        else { stripe = t % NST; ct = t / NST; }
    };
    // step c of tile t: rows RSTEP*c + RPW*w + j (j < RPW), 16 pieces per lane
    auto stage = [&](int t, int c) {
        if (IO == 2) {  // stores only: registers stay as they are
#pragma unroll
            for (int j = 0; j < 64; j++) asm volatile("" : "+v"(St[j]));
            return;
        }
        int stripe, ct;
        loc(t, stripe, ct);
        const bool live = t < NT;
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            base + (live ? (size_t)stripe * SS : 0), 0, live ? (int)(K * RS) : 0, 0x00020000);
        uint32_t voff = (uint32_t)ct * TW + (uint32_t)lane * 16;
        asm volatile("" : "+v"(voff));
#pragma unroll
        for (int q = 0; q < 16; q++) {
            const int j = q / PPR, pc = q % PPR;
            const uint32_t so = (uint32_t)(RSTEP * c + RPW * w + j) * RS;
            const u32x4 x = __builtin_amdgcn_raw_buffer_load_b128(rs, voff + pc * 1024, so, 0);
            St[4 * q] = x[0], St[4 * q + 1] = x[1], St[4 * q + 2] = x[2], St[4 * q + 3] = x[3];
        }
    };
    auto tile_body = [&](int t, int tnext) {
#pragma unroll
        for (int c = 0; c < NSTEP; c++) {
#pragma unroll
            for (int j = 0; j < 64; j++) {
                if (c == 0 && j < ACC) acc[j] = St[j];
                else acc[j % ACC] ^= St[j];
            }
#pragma unroll
            for (int j = 0; j < ACC; j++) asm volatile("" : "+v"(acc[j])::"memory");
            if (c < NSTEP - 1) stage(t, c + 1);
            else if (tnext >= 0) stage(tnext, 0);
        }
        // parity: 32 rows x TW bytes per tile; wave w stores rows 8w..8w+7
        int stripe, ct;
        loc(t, stripe, ct);
        const __amdgpu_buffer_rsrc_t ps = __builtin_amdgcn_make_buffer_rsrc(
            base + (size_t)stripe * SS + (size_t)K * RS, 0, (int)(P * RS), 0x00020000);
        if (IO == 1) {  // loads only: one conditional store keeps the fold alive
            uint32_t f = 0;
#pragma unroll
            for (int j = 0; j < ACC; j++) f ^= acc[j];
            if (f == 0x9E3779B9u) base[0] = 1;
        } else if (PST == 1 || TW != 2048) {
            const uint32_t voff = (uint32_t)ct * TW + (uint32_t)lane * 16;
#pragma unroll
            for (int q = 0; q < 8 * PPR; q++) {
                const int j = q / PPR, pc = q % PPR;
                const u32x4 v = u32x4{acc[(4 * q) % ACC], acc[(4 * q + 1) % ACC], acc[(4 * q + 2) % ACC], acc[(4 * q + 3) % ACC]};
                __builtin_amdgcn_raw_buffer_store_b128(v, ps, voff + pc * 1024, (uint32_t)(8 * w + j) * RS, 0);
            }
        } else {
            // the kernel's layout: lane (block b = lane & 31, half h = lane >> 5), rows 8w + 4h + i, 4 x 16 B
            const int h = lane >> 5, b = lane & 31;
            const uint32_t voff = (uint32_t)ct * TW + (uint32_t)b * 64 + (uint32_t)(4 * h) * RS;
#pragma unroll
            for (int i = 0; i < 4; i++)
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    const int z = 16 * i + 4 * q;
                    const u32x4 v = u32x4{acc[z % ACC], acc[(z + 1) % ACC], acc[(z + 2) % ACC], acc[(z + 3) % ACC]};
                    __builtin_amdgcn_raw_buffer_store_b128(v, ps, voff + q * 16, (uint32_t)(8 * w + i) * RS, 0);
                }
        }
    };
    if (NP) {
        const int t = blockIdx.x;
        if (t >= NT) return;
        stage(t, 0);
        tile_body(t, -1);
        return;
    }
    int t = blockIdx.x;
    stage(t, 0);
    for (; t < NT; t += gridDim.x) tile_body(t, t + (int)gridDim.x);
}

// The round-2 kernel's own load layout (lane = 64-byte block, 4 x 16 B per
// row, rows 8w + 4h + i), 2 KB tiles, for reference; ORDER as above.
template <int ORDER>
__global__ void __launch_bounds__(256, 2) k_c3_r2(uint8_t *base, uint32_t RS, uint64_t SS) {
    constexpr int TW = 2048, TPS = S / TW, NT = TPS * NST;
    const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int h = lane >> 5, b = lane & 31;
    uint32_t St[64], acc[64];
    auto loc = [&](int t, int &stripe, int &ct) {
        if (ORDER == 0) { stripe = t / TPS; ct = t - stripe * TPS; }
        else { stripe = t % NST; ct = t / NST; }
    };
    auto stage = [&](int t, int c) {
        int stripe, ct;
        loc(t, stripe, ct);
        const bool live = t < NT;
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            base + (live ? (size_t)stripe * SS : 0), 0, live ? (int)(K * RS) : 0, 0x00020000);
        uint32_t voff = (uint32_t)ct * TW + (uint32_t)b * 64 + (uint32_t)(4 * h) * RS;
        asm volatile("" : "+v"(voff));
#pragma unroll
        for (int i = 0; i < 4; i++)
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const u32x4 x = __builtin_amdgcn_raw_buffer_load_b128(rs, voff + q * 16, (uint32_t)(32 * c + 8 * w + i) * RS, 0);
                St[16 * i + 4 * q] = x[0], St[16 * i + 4 * q + 1] = x[1], St[16 * i + 4 * q + 2] = x[2], St[16 * i + 4 * q + 3] = x[3];
            }
    };
    int t = blockIdx.x;
    stage(t, 0);
    for (; t < NT; t += gridDim.x) {
#pragma unroll
        for (int c = 0; c < 4; c++) {
#pragma unroll
            for (int j = 0; j < 64; j++) acc[j] = c == 0 ? St[j] : acc[j] ^ St[j];
#pragma unroll
            for (int j = 0; j < 64; j++) asm volatile("" : "+v"(acc[j])::"memory");
            stage(c < 3 ? t : t + (int)gridDim.x, (c + 1) & 3);
        }
        int stripe, ct;
        loc(t, stripe, ct);
        const __amdgpu_buffer_rsrc_t ps = __builtin_amdgcn_make_buffer_rsrc(
            base + (size_t)stripe * SS + (size_t)K * RS, 0, (int)(P * RS), 0x00020000);
        const uint32_t voff = (uint32_t)ct * TW + (uint32_t)b * 64 + (uint32_t)(4 * h) * RS;
#pragma unroll
        for (int i = 0; i < 4; i++)
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const u32x4 v = u32x4{acc[16 * i + 4 * q], acc[16 * i + 4 * q + 1], acc[16 * i + 4 * q + 2], acc[16 * i + 4 * q + 3]};
                __builtin_amdgcn_raw_buffer_store_b128(v, ps, voff + q * 16, (uint32_t)(8 * w + i) * RS, 0);
            }
    }
}

// Calibration: 4:1 streaming.  Each thread reads U float4 from 4 input
// streams (each 1/5 of the bytes) and writes their XOR to the output stream.
template <int U>
__global__ void __launch_bounds__(256) k_mix41(const u32x4 *in, u32x4 *out, size_t n16) {
    const size_t step = (size_t)gridDim.x * 256 * U;
    for (size_t i = (size_t)blockIdx.x * 256 * U + threadIdx.x; i < n16; i += step) {
        u32x4 v[U];
#pragma unroll
        for (int j = 0; j < U; j++) {
            const size_t e = i + 256 * j;
            v[j] = e < n16 ? in[e] ^ in[e + n16] ^ in[e + 2 * n16] ^ in[e + 3 * n16] : u32x4{0, 0, 0, 0};
        }
#pragma unroll
        for (int j = 0; j < U; j++)
            if (i + 256 * j < n16) out[i + 256 * j] = v[j];
    }
}
// Calibration: R read streams + 1 write stream, each of n16 float4, streams
// spaced `gap` float4 apart.
template <int U, int R>
__global__ void __launch_bounds__(256) k_mixr(const u32x4 *in, u32x4 *out, size_t n16, size_t gap) {
    const size_t step = (size_t)gridDim.x * 256 * U;
    for (size_t i = (size_t)blockIdx.x * 256 * U + threadIdx.x; i < n16; i += step) {
        u32x4 v[U];
#pragma unroll
        for (int j = 0; j < U; j++) {
            const size_t e = i + 256 * j;
            u32x4 a = {0, 0, 0, 0};
#pragma unroll
            for (int r = 0; r < R; r++) a ^= e < n16 ? in[e + r * gap] : u32x4{0, 0, 0, 0};
            v[j] = a;
        }
#pragma unroll
        for (int j = 0; j < U; j++)
            if (i + 256 * j < n16) out[i + 256 * j] = v[j];
    }
}
// Calibration: one read stream and one write stream at 4:1 (each thread reads
// 4U float4 of a contiguous 4U KB block and writes U).
template <int U>
__global__ void __launch_bounds__(256) k_mix1(const u32x4 *in, u32x4 *out, size_t n16w) {
    const size_t step = (size_t)gridDim.x * 256 * U;
    for (size_t i = (size_t)blockIdx.x * 256 * U + threadIdx.x; i < n16w; i += step) {
        const size_t blk = i / (256 * U), o = i % (256 * U);
        u32x4 v[U];
#pragma unroll
        for (int j = 0; j < U; j++) v[j] = u32x4{0, 0, 0, 0};
#pragma unroll
        for (int q = 0; q < 4; q++)
#pragma unroll
            for (int j = 0; j < U; j++) {
                const size_t e = blk * 1024 * U + q * 256 * U + o + 256 * j;
                if (i + 256 * j < n16w) v[j] ^= in[e];
            }
#pragma unroll
        for (int j = 0; j < U; j++)
            if (i + 256 * j < n16w) out[i + 256 * j] = v[j];
    }
}
// Calibration: write-only stream.
template <int U>
__global__ void __launch_bounds__(256) k_writeu(u32x4 *dst, size_t n16) {
    const size_t step = (size_t)gridDim.x * 256 * U;
    for (size_t i = (size_t)blockIdx.x * 256 * U + threadIdx.x; i < n16; i += step)
#pragma unroll
        for (int j = 0; j < U; j++)
            if (i + 256 * j < n16) dst[i + 256 * j] = u32x4{(uint32_t)i, 1, 2, 3};
}
// Calibration: plain float4 copy with U in flight per thread (50/50).
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
// Calibration: read-only (XOR fold).
template <int U>
__global__ void __launch_bounds__(256) k_readu(const u32x4 *src, uint32_t *sink, size_t n16) {
    u32x4 a = {0, 0, 0, 0};
    const size_t step = (size_t)gridDim.x * 256 * U;
    for (size_t i = (size_t)blockIdx.x * 256 * U + threadIdx.x; i < n16; i += step) {
#pragma unroll
        for (int j = 0; j < U; j++)
            if (i + 256 * j < n16) a ^= src[i + 256 * j];
    }
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

int main(int argc, char **argv) {
    const int mode = argc > 1 ? atoi(argv[1]) : 0;
    setvbuf(stdout, nullptr, _IONBF, 0);
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const uint32_t RS = S + 3072;
    const uint64_t SS = (uint64_t)(K + P) * RS;
    uint8_t *base;
    uint32_t *sink;
    const size_t bytes = (size_t)NST * SS;
    if (hipMalloc(&base, bytes + (64 << 20)) != hipSuccess || hipMalloc(&sink, 64) != hipSuccess) return 1;
    (void)hipMemset(base, 0x5A, bytes);
    const double alg = (double)NST * (K + P) * S;
    auto rep = [&](const char *n, float us, double by) {
        printf("%-34s %8.1f us  %7.1f GB/s  frac %.3f\n", n, us, by / us / 1e3, by / us / 1e3 / 8000.0);
    };
#define C3(TW, ORD, WG, PST, NP, name)                                                                             \
    do {                                                                                                            \
        const int nt = (int)(S / TW) * NST;                                                                         \
        const int g = NP ? nt : WG * cus;                                                                          \
        rep(name, timeit([&] { hipLaunchKernelGGL((k_c3<TW, ORD, WG, PST, NP>), dim3(g), dim3(256), 0, 0, base, RS, SS); }), alg); \
    } while (0)
    if (mode == 1) {
        const double rd = (double)NST * K * S, wr = (double)NST * P * S;
        for (int r = 0; r < 2; r++) {
            C3(2048, 0, 2, 1, false, "c3 contig 2K both");
            rep("c3 contig 2K loads only", timeit([&] { hipLaunchKernelGGL((k_c3<2048, 0, 2, 1, false, 1>), dim3(2 * cus), dim3(256), 0, 0, base, RS, SS); }), rd);
            rep("c3 contig 2K stores only", timeit([&] { hipLaunchKernelGGL((k_c3<2048, 0, 2, 1, false, 2>), dim3(2 * cus), dim3(256), 0, 0, base, RS, SS); }), wr);
            rep("c3 contig 8K loads only", timeit([&] { hipLaunchKernelGGL((k_c3<8192, 0, 2, 1, false, 1>), dim3(2 * cus), dim3(256), 0, 0, base, RS, SS); }), rd);
            rep("c3 contig 2K NP loads only", timeit([&] { hipLaunchKernelGGL((k_c3<2048, 0, 2, 1, true, 1>), dim3((S / 2048) * NST), dim3(256), 0, 0, base, RS, SS); }), rd);
            rep("c3 contig 2K NP both", timeit([&] { hipLaunchKernelGGL((k_c3<2048, 0, 2, 1, true, 0>), dim3((S / 2048) * NST), dim3(256), 0, 0, base, RS, SS); }), alg);
        }
        const size_t n16 = (size_t)(bytes / 6) / 16 / 4096 * 4096;
        const u32x4 *in = (const u32x4 *)base;
        for (size_t gapx : {(size_t)0, (size_t)192}) {  // streams n16 apart, plus a 3 KB stagger per stream
            const size_t gap = n16 + gapx;
            u32x4 *out = (u32x4 *)(base + (size_t)(5 * gap) * 16);
            char nm[80];
            for (int g : {2048, 4096}) {
                snprintf(nm, sizeof nm, "mix R=4 x4 grid %d gap+%zu", g, gapx * 16);
                rep(nm, timeit([&] { hipLaunchKernelGGL((k_mixr<4, 4>), dim3(g), dim3(256), 0, 0, in, out, n16, gap); }), (double)n16 * 16 * 5);
                snprintf(nm, sizeof nm, "mix R=1 x4 grid %d gap+%zu", g, gapx * 16);
                rep(nm, timeit([&] { hipLaunchKernelGGL((k_mixr<4, 1>), dim3(g), dim3(256), 0, 0, in, out, n16, gap); }), (double)n16 * 16 * 2);
            }
        }
        {
            const size_t n16w = (size_t)(bytes / 5) / 16 / 4096 * 4096;
            u32x4 *out = (u32x4 *)(base + n16w * 16 * 4 + 3072);
            for (int g : {1024, 2048, 4096}) {
                char nm[80];
                snprintf(nm, sizeof nm, "mix1 4:1 x2 grid %d", g);
                rep(nm, timeit([&] { hipLaunchKernelGGL(k_mix1<2>, dim3(g), dim3(256), 0, 0, in, out, n16w); }), (double)n16w * 16 * 5);
                snprintf(nm, sizeof nm, "mix1 4:1 x4 grid %d", g);
                rep(nm, timeit([&] { hipLaunchKernelGGL(k_mix1<4>, dim3(g), dim3(256), 0, 0, in, out, n16w); }), (double)n16w * 16 * 5);
            }
            for (int g : {2048, 8192}) {
                char nm[80];
                snprintf(nm, sizeof nm, "write-only x4 grid %d", g);
                rep(nm, timeit([&] { hipLaunchKernelGGL(k_writeu<4>, dim3(g), dim3(256), 0, 0, (u32x4 *)base, bytes / 16); }), (double)bytes);
            }
        }
        return hipDeviceSynchronize() != hipSuccess;
    }
    for (int rep_i = 0; rep_i < 2; rep_i++) {
        printf("# pass %d\n", rep_i);
        rep("r2 layout, stripe-major", timeit([&] { hipLaunchKernelGGL((k_c3_r2<0>), dim3(2 * cus), dim3(256), 0, 0, base, RS, SS); }), alg);
        rep("r2 layout, stripe-interleaved", timeit([&] { hipLaunchKernelGGL((k_c3_r2<1>), dim3(2 * cus), dim3(256), 0, 0, base, RS, SS); }), alg);
        C3(2048, 0, 2, 1, false, "contig 2K ord0 wg2");
        C3(2048, 1, 2, 1, false, "contig 2K ord1 wg2");
        C3(4096, 0, 2, 1, false, "contig 4K ord0 wg2");
        C3(4096, 1, 2, 1, false, "contig 4K ord1 wg2");
        C3(8192, 0, 2, 1, false, "contig 8K ord0 wg2");
        C3(8192, 1, 2, 1, false, "contig 8K ord1 wg2");
        C3(2048, 0, 2, 0, false, "contig 2K ord0 wg2 r2-stores");
        C3(2048, 0, 3, 1, false, "contig 2K ord0 wg3");
        C3(2048, 1, 3, 1, false, "contig 2K ord1 wg3");
        C3(2048, 0, 4, 1, false, "contig 2K ord0 wg4");
        C3(2048, 1, 4, 1, false, "contig 2K ord1 wg4");
        C3(4096, 1, 4, 1, false, "contig 4K ord1 wg4");
        C3(2048, 0, 2, 1, true, "contig 2K ord0 one-tile-per-wg");
        C3(4096, 0, 2, 1, true, "contig 4K ord0 one-tile-per-wg");
    }
    {
        const size_t n16 = (size_t)(bytes / 5) / 16 / 256 * 256;
        const double by = (double)n16 * 16 * 5;
        const u32x4 *in = (const u32x4 *)base;
        u32x4 *out = (u32x4 *)(base + n16 * 16 * 4);
        for (int g : {1024, 2048, 4096}) {
            char nm[64];
            snprintf(nm, sizeof nm, "mix 4:1 x2 grid %d", g);
            rep(nm, timeit([&] { hipLaunchKernelGGL(k_mix41<2>, dim3(g), dim3(256), 0, 0, in, out, n16); }), by);
            snprintf(nm, sizeof nm, "mix 4:1 x4 grid %d", g);
            rep(nm, timeit([&] { hipLaunchKernelGGL(k_mix41<4>, dim3(g), dim3(256), 0, 0, in, out, n16); }), by);
        }
        const size_t h16 = bytes / 2 / 16;
        for (int g : {2048, 4096}) {
            char nm[64];
            snprintf(nm, sizeof nm, "copy x8 grid %d", g);
            rep(nm, timeit([&] { hipLaunchKernelGGL(k_copyu<8>, dim3(g), dim3(256), 0, 0, (const u32x4 *)base, (u32x4 *)(base + h16 * 16), h16); }), (double)h16 * 32);
            snprintf(nm, sizeof nm, "read x4 grid %d", g);
            rep(nm, timeit([&] { hipLaunchKernelGGL(k_readu<4>, dim3(g), dim3(256), 0, 0, (const u32x4 *)base, sink, bytes / 16); }), (double)bytes / 16 * 16);
        }
    }
    return hipDeviceSynchronize() != hipSuccess;
}
