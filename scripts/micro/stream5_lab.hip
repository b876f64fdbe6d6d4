// Copy-rate calibration against MI355X_MICROARCH.md's "6.29 TB/s measured
// (float4 copy, 79 %)", with the engine's C3 encode timed in the same process
// (lab only).  Every line is bytes moved (read + write)
// per second against 8 TB/s.
//
//   ./stream5_lab [MiB per buffer]      (default 2048: far past the 256 MiB Infinity Cache)
//
// Variants: grid-stride vs one-shot grids, float4 per lane in flight (U),
// block size, non-temporal loads / stores, buffer separation, and an XCD-aware
// block -> chunk map (consecutive chunks on one XCD).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../include/rs_mi355x.h"

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

#define CHECK(x)                                                                      \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                  \
        }                                                                             \
    } while (0)

template <bool NTL>
__device__ __forceinline__ u32x4 ld(const u32x4 *p) {
    if constexpr (NTL) return __builtin_nontemporal_load(p);
    return *p;
}
template <bool NTS>
__device__ __forceinline__ void st(u32x4 *p, u32x4 v) {
    if constexpr (NTS) __builtin_nontemporal_store(v, p);
    else *p = v;
}

// One-shot grid: block b copies U * BS float4 starting at chunk(b) * U * BS.
// XCD: blocks are dispatched round-robin over the 8 XCDs; XCD = 1 gives each
// XCD a contiguous range of chunks.
template <int U, int BS, bool NTL, bool NTS, bool XCD>
__global__ void __launch_bounds__(BS) k_copy_once(const u32x4 *__restrict__ src, u32x4 *__restrict__ dst, size_t n16) {
    size_t b = blockIdx.x;
    if (XCD) {
        const size_t nb = gridDim.x, per = nb / 8;
        if (b < per * 8) b = (b & 7) * per + (b >> 3);
    }
    const size_t base = b * (size_t)U * BS + threadIdx.x;
    u32x4 v[U];
#pragma unroll
    for (int j = 0; j < U; j++) v[j] = base + BS * j < n16 ? ld<NTL>(src + base + BS * j) : u32x4{0, 0, 0, 0};
#pragma unroll
    for (int j = 0; j < U; j++)
        if (base + BS * j < n16) st<NTS>(dst + base + BS * j, v[j]);
}

template <int U, int BS, bool NTL, bool NTS>
__global__ void __launch_bounds__(BS) k_copy_stride(const u32x4 *__restrict__ src, u32x4 *__restrict__ dst, size_t n16) {
    const size_t step = (size_t)gridDim.x * BS * U;
    for (size_t i = (size_t)blockIdx.x * BS * U + threadIdx.x; i < n16; i += step) {
        u32x4 v[U];
#pragma unroll
        for (int j = 0; j < U; j++) v[j] = i + BS * j < n16 ? ld<NTL>(src + i + BS * j) : u32x4{0, 0, 0, 0};
#pragma unroll
        for (int j = 0; j < U; j++)
            if (i + BS * j < n16) st<NTS>(dst + i + BS * j, v[j]);
    }
}

template <int U, bool NTL>
__global__ void __launch_bounds__(256) k_read_once(const u32x4 *__restrict__ src, uint32_t *sink, size_t n16) {
    const size_t base = (size_t)blockIdx.x * U * 256 + threadIdx.x;
    u32x4 a = {0, 0, 0, 0};
#pragma unroll
    for (int j = 0; j < U; j++)
        if (base + 256 * j < n16) a ^= ld<NTL>(src + base + 256 * j);
    if ((a[0] ^ a[1] ^ a[2] ^ a[3]) == 0x12345678u) sink[0] = 1;
}

template <int U, bool NTS>
__global__ void __launch_bounds__(256) k_write_once(u32x4 *dst, size_t n16) {
    const size_t base = (size_t)blockIdx.x * U * 256 + threadIdx.x;
#pragma unroll
    for (int j = 0; j < U; j++)
        if (base + 256 * j < n16) st<NTS>(dst + base + 256 * j, u32x4{(uint32_t)base, 1, 2, 3});
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
    printf("%-44s %9.1f us  %7.1f GB/s  frac %.3f\n", n, us, by / us / 1e3, by / us / 1e3 / 8000.0);
}

int main(int argc, char **argv) {
    setvbuf(stdout, nullptr, _IONBF, 0);
    const size_t mib = argc > 1 ? (size_t)atol(argv[1]) : 2048;
    const size_t bytes = mib << 20, n16 = bytes / 16;
    int cus = 0;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    u32x4 *a, *b, *one;
    uint32_t *sink;
    CHECK(hipMalloc(&a, bytes));
    CHECK(hipMalloc(&b, bytes));
    CHECK(hipMalloc(&one, 2 * bytes + (3 << 10)));  // both buffers of one allocation, 3 KB apart
    CHECK(hipMalloc(&sink, 64));
    CHECK(hipMemset(a, 0x5A, bytes));
    CHECK(hipMemset(b, 0, bytes));
    CHECK(hipMemset(one, 0x33, 2 * bytes + (3 << 10)));
    u32x4 *one_dst = (u32x4 *)((uint8_t *)one + bytes + (3 << 10));
    const double cb = 2.0 * bytes;
    char nm[96];
    printf("# %zu MiB per buffer, %d CUs\n", mib, cus);
    for (int pass = 0; pass < 2; pass++) {
        printf("# pass %d\n", pass);
#define ONCE(U, BS, NTL, NTS, XCD, SRC, DST, tag)                                                              \
    do {                                                                                                     \
        const unsigned g = (unsigned)((n16 + (size_t)(U) * (BS)-1) / ((size_t)(U) * (BS)));                  \
        snprintf(nm, sizeof nm, "copy once U%d bs%d%s%s%s %s", U, BS, NTL ? " ntl" : "", NTS ? " nts" : "", \
                 XCD ? " xcd" : "", tag);                                                                    \
        rep(nm, timeit([&] { hipLaunchKernelGGL((k_copy_once<U, BS, NTL, NTS, XCD>), dim3(g), dim3(BS), 0, 0, SRC, DST, n16); }), cb); \
    } while (0)
        ONCE(1, 256, false, false, false, a, b, "sep");
        ONCE(2, 256, false, false, false, a, b, "sep");
        ONCE(4, 256, false, false, false, a, b, "sep");
        ONCE(8, 256, false, false, false, a, b, "sep");
        ONCE(4, 512, false, false, false, a, b, "sep");
        ONCE(4, 1024, false, false, false, a, b, "sep");
        ONCE(4, 256, true, false, false, a, b, "sep");
        ONCE(4, 256, false, true, false, a, b, "sep");
        ONCE(4, 256, true, true, false, a, b, "sep");
        ONCE(4, 256, false, false, true, a, b, "sep");
        ONCE(8, 256, false, false, true, a, b, "sep");
        ONCE(4, 256, false, false, false, (const u32x4 *)one, one_dst, "one-alloc");
#define STRIDE(U, BS, NTL, NTS, G)                                                                              \
    do {                                                                                                        \
        snprintf(nm, sizeof nm, "copy stride U%d bs%d%s%s grid %d", U, BS, NTL ? " ntl" : "", NTS ? " nts" : "", G); \
        rep(nm, timeit([&] { hipLaunchKernelGGL((k_copy_stride<U, BS, NTL, NTS>), dim3(G), dim3(BS), 0, 0, a, b, n16); }), cb); \
    } while (0)
        STRIDE(4, 256, false, false, 4 * cus);
        STRIDE(4, 256, false, false, 8 * cus);
        STRIDE(4, 256, false, false, 16 * cus);
        STRIDE(8, 256, false, false, 8 * cus);
        STRIDE(2, 256, false, false, 32 * cus);
        STRIDE(4, 256, false, true, 8 * cus);
        {
            const unsigned g = (unsigned)(n16 / (4 * 256));
            rep("read once U4", timeit([&] { hipLaunchKernelGGL((k_read_once<4, false>), dim3(g), dim3(256), 0, 0, a, sink, n16); }), (double)bytes);
            rep("read once U4 ntl", timeit([&] { hipLaunchKernelGGL((k_read_once<4, true>), dim3(g), dim3(256), 0, 0, a, sink, n16); }), (double)bytes);
            rep("write once U4", timeit([&] { hipLaunchKernelGGL((k_write_once<4, false>), dim3(g), dim3(256), 0, 0, b, n16); }), (double)bytes);
            rep("write once U4 nts", timeit([&] { hipLaunchKernelGGL((k_write_once<4, true>), dim3(g), dim3(256), 0, 0, b, n16); }), (double)bytes);
        }
    }
    CHECK(hipFree(a));
    CHECK(hipFree(b));
    CHECK(hipFree(one));

    // The engine's C3 encode (128 + 32 x 1 MiB, 128 stripes, rows 3 KB staggered)
    // in the same process: rs_encode_dev_batch on the null stream.
    const int K = 128, P = 32, NST = argc > 2 ? atoi(argv[2]) : 128;
    const size_t S = 1 << 20, RS = S + 3072, SS = (K + P) * RS;
    uint8_t *slab;
    CHECK(hipMalloc(&slab, NST * SS));
    CHECK(hipMemset(slab, 0x77, NST * SS));
    rs_codec *c = nullptr;
    if (rs_new(16, K, P, 0, &c) != 0) return 2;
    const double alg = (double)NST * (K + P) * S;
    for (int pass = 0; pass < 2; pass++) {
        snprintf(nm, sizeof nm, "engine C3 encode x%d (%s)", NST, rs_encode_path(c));
        rep(nm, timeit([&] { (void)rs_encode_dev_batch(c, slab, RS, SS, NST, S, RS_NULL_STREAM); }, 10), alg);
    }
    rs_free(c);
    CHECK(hipFree(slab));
    return 0;
}
