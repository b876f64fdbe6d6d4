// Memory-side lab, round 4: why the C3 row pattern (128 reads / 32 writes of
// 1 MiB rows per stripe) streams at ~0.65 of 8 TB/s while a one-shot float4
// copy on the same box reaches ~0.78 (stream5_lab) and a grid-stride copy
// ~0.65.  Here the C3 byte pattern is moved by one-shot grids of small tiles:
// a workgroup takes TW contiguous bytes of every row of one stripe and writes
// out row j = XOR of in rows 4j..4j+3 (the 4:1 byte ratio of C3, no
// transform).  Loads are lane-contiguous (each instruction covers whole
// 128-byte lines), optionally non-temporal.  Also a plain 4:1 stream in the
// one-shot style (4 source regions, 1 destination).
//
//   ./stream6_lab [stripes]     (default 16: 2.7 GB moved per launch)
//
// Diagnostic only.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                      \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                  \
        }                                                                             \
    } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
constexpr int K = 128, P = 32;
constexpr uint32_t S = 1u << 20;

template <bool NT>
__device__ __forceinline__ u32x4 ldx(const __amdgpu_buffer_rsrc_t &rs, uint32_t voff, uint32_t soff) {
    return __builtin_amdgcn_raw_buffer_load_b128(rs, voff, soff, NT ? 2 : 0);
}

// One tile per workgroup: TW bytes of each of the 160 rows of one stripe.
// BS threads; each thread owns 16 bytes of a (row group, column) and walks
// the 128 input rows as 32 groups of 4 (XOR), storing one output row per group.
// ORDER 0: tile = stripe * tiles_per_stripe + column; 1: column-major over stripes.
template <int TW, int BS, bool NT, int ORDER>
__global__ void __launch_bounds__(BS) k_tile(uint8_t *base, uint32_t RS, uint64_t SS, int nst) {
    constexpr int LPR = TW / 16;           // lanes per row piece
    constexpr int RPI = BS / LPR;          // output rows handled per pass
    const int tps = S / TW;
    int stripe, ct;
    if (ORDER == 0) {
        stripe = blockIdx.x / tps;
        ct = blockIdx.x - stripe * tps;
    } else {
        stripe = blockIdx.x % nst;
        ct = blockIdx.x / nst;
    }
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(base + (size_t)stripe * SS, 0, (int)((K + P) * RS), 0x00020000);
    const int t = threadIdx.x;
    const uint32_t col = (uint32_t)ct * TW + (uint32_t)(t % LPR) * 16;
    const int r0 = t / LPR;
#pragma unroll
    for (int j = r0; j < P; j += RPI) {
        u32x4 a[4];
#pragma unroll
        for (int q = 0; q < 4; q++) a[q] = ldx<NT>(rs, col, (uint32_t)(4 * j + q) * RS);
        const u32x4 o = a[0] ^ a[1] ^ a[2] ^ a[3];
        __builtin_amdgcn_raw_buffer_store_b128(o, rs, col, (uint32_t)(K + j) * RS, 0);
    }
}

// All 128 reads first (held in registers), then the 32 writes: the encode's
// real order (every output depends on every input).  TW = 512 with 256
// threads: 32 lanes per row, 8 rows per instruction, 16 instructions of loads.
template <bool NT>
__global__ void __launch_bounds__(256) k_tile_allfirst(uint8_t *base, uint32_t RS, uint64_t SS) {
    constexpr int TW = 512, LPR = 32, RPI = 8;
    const int tps = S / TW;
    const int stripe = blockIdx.x / tps, ct = blockIdx.x - stripe * tps;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(base + (size_t)stripe * SS, 0, (int)((K + P) * RS), 0x00020000);
    const int t = threadIdx.x;
    const uint32_t col = (uint32_t)ct * TW + (uint32_t)(t % LPR) * 16;
    const int r0 = t / LPR;
    u32x4 acc[P / RPI] = {};
    u32x4 v[K / RPI];
#pragma unroll
    for (int i = 0; i < K / RPI; i++) v[i] = ldx<NT>(rs, col, (uint32_t)(r0 + RPI * i) * RS);
#pragma unroll
    for (int i = 0; i < K / RPI; i++) acc[i & 3] ^= v[i];
#pragma unroll
    for (int j = 0; j < P / RPI; j++)
        __builtin_amdgcn_raw_buffer_store_b128(acc[j], rs, col, (uint32_t)(K + r0 + RPI * j) * RS, 0);
}

// 2 KB tiles whose 32 blocks come from NP pieces of 2048 / NP contiguous bytes
// spread over the row (piece p at p * S / NP): concurrently running tiles then
// cover consecutive narrow pieces, as narrow tiles do, while a workgroup
// keeps k_encode_hp's 2 KB per row.  KL: the kernel's lane layout (lane =
// 64-byte block, four 16-byte loads per row at 64-byte stride, rows r and
// r + 4 in the two wave halves) instead of lane-contiguous loads.
template <int NP, bool KL>
__global__ void __launch_bounds__(256) k_tile_pieces(uint8_t *base, uint32_t RS, uint64_t SS) {
    constexpr int PW = 2048 / NP;  // bytes per piece
    const int tps = S / 2048;
    const int stripe = blockIdx.x / tps, ct = blockIdx.x - stripe * tps;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(base + (size_t)stripe * SS, 0, (int)((K + P) * RS), 0x00020000);
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    if (!KL) {
        // lane-contiguous: 128 lanes per row (2 KB), 2 rows per pass
        const int c16 = t & 127;                  // 16-byte unit of the tile row
        const int pc = (c16 * 16) / PW, within = (c16 * 16) % PW;
        const uint32_t col = (uint32_t)pc * (S / NP) + (uint32_t)ct * PW + within;
        const int r0 = t >> 7;
#pragma unroll
        for (int j = r0; j < P; j += 2) {
            u32x4 a[4];
#pragma unroll
            for (int q = 0; q < 4; q++) a[q] = ldx<false>(rs, col, (uint32_t)(4 * j + q) * RS);
            __builtin_amdgcn_raw_buffer_store_b128(a[0] ^ a[1] ^ a[2] ^ a[3], rs, col, (uint32_t)(K + j) * RS, 0);
        }
    } else {
        // kernel layout: lane (b = lane & 31, h = lane >> 5) owns block b of rows
        // 8w + 4h + i; each row is four 16-byte loads at 64-byte lane stride
        const int b = lane & 31, h = lane >> 5;
        const int pc = (b * 64) / PW, within = (b * 64) % PW;
        const uint32_t col = (uint32_t)pc * (S / NP) + (uint32_t)ct * PW + within;
#pragma unroll
        for (int s = 0; s < 4; s++) {  // 4 steps of 32 input rows: 8 per wave, 4 per lane
            u32x4 acc[4] = {};
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const uint32_t row = (uint32_t)(32 * s + 8 * w + 4 * h + i);
#pragma unroll
                for (int q = 0; q < 4; q++) acc[q] ^= ldx<false>(rs, col + 16 * q, row * RS);
            }
            // output row 8 s + 2 w + h (32 rows over the 4 steps)
            const uint32_t orow = (uint32_t)(K + 8 * s + 2 * w + h);
#pragma unroll
            for (int q = 0; q < 4; q++) __builtin_amdgcn_raw_buffer_store_b128(acc[q], rs, col + 16 * q, orow * RS, 0);
        }
    }
}

// The engine's memory schedule in isolation (k_encode_hp, m = 32): a 2 KB tile
// per 256-thread workgroup, every lane owning 64-byte block b = lane & 31 of
// rows 4h + i of its wave's 8-row group (h = lane >> 5); four chunks of 32
// rows, each chunk's 16 row loads per lane (4 rows x 4 x 16 B) in registers
// before they are folded into the accumulator, then 32 parity rows stored
// per tile.  KL = 1: the engine's lane layout (each load instruction touches
// 16 B of every 64-byte block: 16 bytes at a 64-byte lane stride); KL = 0:
// the same bytes per lane group but each instruction lane-contiguous (a lane
// takes 16-byte piece l of a 1 KB run).  Occupancy fixed by dynamic LDS.
template <bool KL, bool KLS = KL>
__global__ void __launch_bounds__(256) k_engine_mem(uint8_t *base, uint32_t RS, uint64_t SS) {
    const int tps = S / 2048;
    const int stripe = blockIdx.x / tps, ct = blockIdx.x - stripe * tps;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(base + (size_t)stripe * SS, 0, (int)((K + P) * RS), 0x00020000);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, h = lane >> 5, b = lane & 31;
    u32x4 acc[4][4] = {};
    for (int c = 0; c < 4; c++) {
        u32x4 v[4][4];
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const uint32_t row = (uint32_t)(32 * c + 8 * w + 4 * h + i);
#pragma unroll
            for (int q = 0; q < 4; q++) {
                // KL: lane b, piece q of its block; else: piece (lane & 31) of 1 KB run (q & 1) of row-pair half
                const uint32_t col = KL ? (uint32_t)ct * 2048 + b * 64 + q * 16 : (uint32_t)ct * 2048 + (q >> 1) * 1024 + (q & 1) * 512 + b * 16;
                v[i][q] = ldx<false>(rs, col, row * RS);
            }
        }
#pragma unroll
        for (int i = 0; i < 4; i++)
#pragma unroll
            for (int q = 0; q < 4; q++) acc[i][q] ^= v[i][q];
    }
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const uint32_t row = (uint32_t)(K + 8 * w + 4 * h + i);
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const uint32_t col = KLS ? (uint32_t)ct * 2048 + b * 64 + q * 16 : (uint32_t)ct * 2048 + (q >> 1) * 1024 + (q & 1) * 512 + b * 16;
            __builtin_amdgcn_raw_buffer_store_b128(acc[i][q], rs, col, row * RS, 0);
        }
    }
}

// Plain 4:1 one-shot stream: block b reads U float4 per lane from each of 4
// regions and writes their XOR to the destination.
template <int U, bool NT>
__global__ void __launch_bounds__(256) k_mix41_once(const u32x4 *src, u32x4 *dst, size_t n16) {
    const size_t base = (size_t)blockIdx.x * U * 256 + threadIdx.x;
    u32x4 v[U];
#pragma unroll
    for (int j = 0; j < U; j++) {
        const u32x4 *p = src + base + 256 * j;
        if (NT)
            v[j] = __builtin_nontemporal_load(p) ^ __builtin_nontemporal_load(p + n16) ^ __builtin_nontemporal_load(p + 2 * n16) ^
                   __builtin_nontemporal_load(p + 3 * n16);
        else
            v[j] = p[0] ^ p[n16] ^ p[2 * n16] ^ p[3 * n16];
    }
#pragma unroll
    for (int j = 0; j < U; j++) dst[base + 256 * j] = v[j];
}

template <class F>
float timeit(F f, int n = 20) {
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    for (int i = 0; i < 3; i++) f();
    CHECK(hipEventRecord(a));
    for (int i = 0; i < n; i++) f();
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms;
    CHECK(hipEventElapsedTime(&ms, a, b));
    return ms * 1e3f / n;
}

static void rep(const char *n, float us, double by) {
    printf("%-48s %9.1f us  %7.1f GB/s  frac %.3f\n", n, us, by / us / 1e3, by / us / 1e3 / 8000.0);
}

int main(int argc, char **argv) {
    setvbuf(stdout, nullptr, _IONBF, 0);
    const int nst = argc > 1 ? atoi(argv[1]) : 16;
    const uint32_t RS = S + 3072;
    const uint64_t SS = (uint64_t)(K + P) * RS;
    uint8_t *slab;
    CHECK(hipMalloc(&slab, nst * SS));
    CHECK(hipMemset(slab, 0x5A, nst * SS));
    const double alg = (double)nst * (K + P) * S;
    char nm[96];
    printf("# %d stripes of 128 + 32 x 1 MiB rows (stride 1 MiB + 3 KiB), %.2f GB per launch\n", nst, alg / 1e9);
    for (int pass = 0; pass < 2; pass++) {
        printf("# pass %d\n", pass);
#define TILE(TW, BS, NT, ORD)                                                                                       \
    do {                                                                                                            \
        const unsigned g = (unsigned)((uint64_t)nst * (S / TW));                                                    \
        snprintf(nm, sizeof nm, "C3 tile %dB bs%d%s%s", TW, BS, NT ? " nt" : "", ORD ? " col-major" : "");       \
        rep(nm, timeit([&] { hipLaunchKernelGGL((k_tile<TW, BS, NT, ORD>), dim3(g), dim3(BS), 0, 0, slab, RS, SS, nst); }), alg); \
    } while (0)
        TILE(256, 64, false, 0);
        TILE(256, 64, true, 0);
        TILE(512, 128, false, 0);
        TILE(512, 128, true, 0);
        TILE(512, 256, false, 0);
        TILE(512, 256, true, 0);
        TILE(1024, 256, false, 0);
        TILE(1024, 256, true, 0);
        TILE(2048, 256, false, 0);
        TILE(2048, 256, true, 0);
        TILE(2048, 512, false, 0);
        // occupancy held to the engine's (2 x 4 waves per CU at 64 KB LDS) by
        // dynamic LDS that the kernel never touches
#define TILEO(TW, BS, LDSKB)                                                                                        \
    do {                                                                                                            \
        const unsigned g = (unsigned)((uint64_t)nst * (S / TW));                                                    \
        snprintf(nm, sizeof nm, "C3 tile %dB bs%d, %d KB LDS per WG", TW, BS, LDSKB);                             \
        rep(nm, timeit([&] { hipLaunchKernelGGL((k_tile<TW, BS, false, 0>), dim3(g), dim3(BS), LDSKB << 10, 0, slab, RS, SS, nst); }), alg); \
    } while (0)
        TILEO(2048, 256, 64);
        TILEO(512, 64, 20);
        TILEO(512, 64, 40);
        TILEO(512, 128, 40);
        TILEO(512, 256, 64);
        {
            const unsigned g = (unsigned)((uint64_t)nst * (S / 2048));
            rep("engine memory schedule, KL loads/stores, 64 KB LDS", timeit([&] { hipLaunchKernelGGL((k_engine_mem<true>), dim3(g), dim3(256), 64 << 10, 0, slab, RS, SS); }), alg);
            rep("engine memory schedule, contiguous, 64 KB LDS", timeit([&] { hipLaunchKernelGGL((k_engine_mem<false>), dim3(g), dim3(256), 64 << 10, 0, slab, RS, SS); }), alg);
            rep("engine memory schedule, KL loads, contiguous stores", timeit([&] { hipLaunchKernelGGL((k_engine_mem<true, false>), dim3(g), dim3(256), 64 << 10, 0, slab, RS, SS); }), alg);
            rep("engine memory schedule, contiguous loads, KL stores", timeit([&] { hipLaunchKernelGGL((k_engine_mem<false, true>), dim3(g), dim3(256), 64 << 10, 0, slab, RS, SS); }), alg);
            rep("engine memory schedule, KL loads/stores, no LDS", timeit([&] { hipLaunchKernelGGL((k_engine_mem<true>), dim3(g), dim3(256), 0, 0, slab, RS, SS); }), alg);
        }
        TILE(512, 256, false, 1);
        TILE(512, 256, true, 1);
        {
            const unsigned g = (unsigned)((uint64_t)nst * (S / 2048));
#define PIECES(NPC, KL)                                                                                          \
    do {                                                                                                       \
        snprintf(nm, sizeof nm, "C3 tile 2KB = %d x %dB pieces%s", NPC, 2048 / NPC, KL ? " kernel-layout" : ""); \
        rep(nm, timeit([&] { hipLaunchKernelGGL((k_tile_pieces<NPC, KL>), dim3(g), dim3(256), 0, 0, slab, RS, SS); }), alg); \
    } while (0)
            PIECES(1, false);
            PIECES(4, false);
            PIECES(8, false);
            PIECES(1, true);
            PIECES(4, true);
            PIECES(8, true);
            PIECES(32, true);
        }
        {
            const unsigned g = (unsigned)((uint64_t)nst * (S / 512));
            rep("C3 tile 512B all-loads-first", timeit([&] { hipLaunchKernelGGL((k_tile_allfirst<false>), dim3(g), dim3(256), 0, 0, slab, RS, SS); }), alg);
            rep("C3 tile 512B all-loads-first nt", timeit([&] { hipLaunchKernelGGL((k_tile_allfirst<true>), dim3(g), dim3(256), 0, 0, slab, RS, SS); }), alg);
        }
        {
            // 4:1 stream over the same slab: 4 regions of n16 float4 in, one out
            const size_t n16 = (size_t)nst * SS / 16 / 5;
            const u32x4 *src = (const u32x4 *)slab;
            u32x4 *dst = (u32x4 *)slab + 4 * n16;
            const double by = 5.0 * n16 * 16;
            rep("mix 4:1 once U1", timeit([&] { hipLaunchKernelGGL((k_mix41_once<1, false>), dim3((unsigned)(n16 / 256)), dim3(256), 0, 0, src, dst, n16); }), by);
            rep("mix 4:1 once U1 nt", timeit([&] { hipLaunchKernelGGL((k_mix41_once<1, true>), dim3((unsigned)(n16 / 256)), dim3(256), 0, 0, src, dst, n16); }), by);
            rep("mix 4:1 once U2", timeit([&] { hipLaunchKernelGGL((k_mix41_once<2, false>), dim3((unsigned)(n16 / 512)), dim3(256), 0, 0, src, dst, n16); }), by);
            rep("mix 4:1 once U2 nt", timeit([&] { hipLaunchKernelGGL((k_mix41_once<2, true>), dim3((unsigned)(n16 / 512)), dim3(256), 0, 0, src, dst, n16); }), by);
        }
    }
    CHECK(hipFree(slab));
    return 0;
}
