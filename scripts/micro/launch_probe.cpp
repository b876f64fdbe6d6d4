// Host time vs GPU time of back-to-back rs_encode_dev_batch calls on one
// stream, from C (no Python): does a call return before its kernel finishes?
// Also a plain kernel of the same duration class launched from this program.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>

#include "../../include/rs_mi355x.h"

__global__ void k_spin(float *x, int n, int iters) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float v = x[i];
    for (int k = 0; k < iters; k++) v = v * 1.0000001f + 1e-7f;
    x[i] = v;
}

int main() {
    rs_codec *c = nullptr;
    if (rs_new(16, 1024, 256, 0, &c)) return 1;
    const size_t S = 256 << 10, rows = 1280;
    uint8_t *slab;
    if (hipMalloc(&slab, rows * S)) return 1;
    (void)hipMemset(slab, 0x5A, rows * S);
    float *x;
    (void)hipMalloc(&x, (64 << 20) * sizeof(float));
    hipStream_t s;
    (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    auto probe = [&](const char *name, auto fn) {
        for (int i = 0; i < 3; i++) fn();
        (void)hipStreamSynchronize(s);
        (void)hipEventRecord(e0, s);
        auto t0 = std::chrono::steady_clock::now();
        for (int i = 0; i < 50; i++) fn();
        auto t1 = std::chrono::steady_clock::now();
        (void)hipEventRecord(e1, s);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        printf("%-28s host %8.1f us/call  gpu %8.1f us/call\n", name,
               std::chrono::duration<double, std::micro>(t1 - t0).count() / 50, ms * 1e3 / 50);
    };
    probe("rs_encode_dev_batch C5", [&] { rs_encode_dev_batch(c, slab, S, rows * S, 1, S, s); });
    // C2 (GF(2^8) 10 + 4 x 1 MiB), one stripe per call: the shape every
    // New(10, 4).Encode of a device-resident stripe produces
    rs_codec *c2 = nullptr;
    if (rs_new(8, 10, 4, 0, &c2)) return 1;
    const size_t S2 = 1 << 20;
    probe("rs_encode_dev_batch C2 x1", [&] { rs_encode_dev_batch(c2, slab, S2, 14 * S2, 1, S2, s); });
    probe("rs_encode_dev_batch C2 x16", [&] { rs_encode_dev_batch(c2, slab, S2, 14 * S2, 16, S2, s); });
    uint8_t *rows2[14];
    for (int i = 0; i < 14; i++) rows2[i] = slab + i * S2;
    probe("rs_encode_dev C2 x1 (rows)", [&] { rs_encode_dev(c2, rows2, S2, s); });
    rs_free(c2);
    probe("k_spin", [&] { hipLaunchKernelGGL(k_spin, dim3((64 << 20) / 256), dim3(256), 0, s, x, 64 << 20, 20); });
    rs_free(c);
    return 0;
}
