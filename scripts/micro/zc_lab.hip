// Lab: host <-> device row copies for the host-resident reconstruct.
// (a) hipMemcpyAsync per row (the pipeline's copy_rows for scattered rows),
// (b) one kernel that reads the rows straight from pinned host memory (zero
//     copy over PCIe) into a device slab, (c) one kernel that writes device
//     rows straight into pinned host rows.  Rows are scattered (every other
//     row of a pinned slab), 128 in and 32 out of a 160-row stripe.
// Build: hipcc --offload-arch=gfx950 -O3 zc_lab.hip -o zc_lab
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdint>
#include <vector>

#define CK(x)                                                                       \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) {                                                     \
            std::printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            return 1;                                                               \
        }                                                                           \
    } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// rows[r] (host-mapped) bytes [0, w) -> dst + r * pitch; w a multiple of 16
__global__ void __launch_bounds__(256) k_gather(uint8_t *dst, uint64_t pitch, const uint8_t *const *rows, int nrows,
                                                uint64_t w) {
    const uint64_t per_row = w / 16;
    const uint64_t n = per_row * (uint64_t)nrows;
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
        const uint64_t r = i / per_row, c = i - r * per_row;
        const u32x4 v = *(const u32x4 *)(rows[r] + c * 16);
        *(u32x4 *)(dst + r * pitch + c * 16) = v;
    }
}
__global__ void __launch_bounds__(256) k_scatter(uint8_t *const *rows, const uint8_t *src, uint64_t pitch, int nrows,
                                                 uint64_t w) {
    const uint64_t per_row = w / 16;
    const uint64_t n = per_row * (uint64_t)nrows;
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
        const uint64_t r = i / per_row, c = i - r * per_row;
        *(u32x4 *)(rows[r] + c * 16) = *(const u32x4 *)(src + r * pitch + c * 16);
    }
}

int main() {
    const uint64_t W = 1 << 20;  // bytes per row per call
    const int nin = 128, nout = 32, stride_rows = 2;
    uint8_t *host = nullptr, *dev = nullptr;
    CK(hipHostMalloc((void **)&host, (uint64_t)(nin + nout) * stride_rows * W, hipHostMallocDefault));
    CK(hipMalloc((void **)&dev, (uint64_t)(nin + nout) * W));
    for (uint64_t i = 0; i < (uint64_t)(nin + nout) * stride_rows * W; i += 4096) host[i] = (uint8_t)i;
    std::vector<uint8_t *> hin(nin), hout(nout), kin(nin), kout(nout);
    for (int r = 0; r < nin; r++) hin[r] = host + (uint64_t)r * stride_rows * W;
    for (int r = 0; r < nout; r++) hout[r] = host + (uint64_t)(nin + r) * stride_rows * W;
    // the kernels address the pinned rows through the device's mapping of them
    uint8_t *hdev = nullptr;
    CK(hipHostGetDevicePointer((void **)&hdev, host, 0));
    std::printf("{\"host\": \"%p\", \"device_view\": \"%p\"}\n", (void *)host, (void *)hdev);
    for (int r = 0; r < nin; r++) kin[r] = hdev + (hin[r] - host);
    for (int r = 0; r < nout; r++) kout[r] = hdev + (hout[r] - host);
    uint8_t **din = nullptr, **dout = nullptr;
    CK(hipMalloc((void **)&din, nin * sizeof(void *)));
    CK(hipMalloc((void **)&dout, nout * sizeof(void *)));
    CK(hipMemcpy(din, kin.data(), nin * sizeof(void *), hipMemcpyHostToDevice));
    CK(hipMemcpy(dout, kout.data(), nout * sizeof(void *), hipMemcpyHostToDevice));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    auto now = [] { return std::chrono::steady_clock::now(); };
    auto secs = [](auto a, auto b) { return std::chrono::duration<double>(b - a).count(); };
    for (uint64_t seg : {W, W / 8, W / 16}) {
        const int reps = 5;
        // (a) per-row copies of `seg` bytes, as many segments as fit W
        CK(hipStreamSynchronize(s));
        auto t0 = now();
        for (int k = 0; k < reps; k++)
            for (uint64_t off = 0; off < W; off += seg) {
                for (int r = 0; r < nin; r++)
                    CK(hipMemcpyAsync(dev + (uint64_t)r * W + off, hin[r] + off, seg, hipMemcpyHostToDevice, s));
                for (int r = 0; r < nout; r++)
                    CK(hipMemcpyAsync(hout[r] + off, dev + (uint64_t)(nin + r) * W + off, seg, hipMemcpyDeviceToHost, s));
            }
        CK(hipStreamSynchronize(s));
        auto t1 = now();
        // (b)+(c) one gather and one scatter kernel per segment
        for (int k = 0; k < reps; k++)
            for (uint64_t off = 0; off < W; off += seg) {
                hipLaunchKernelGGL(k_gather, dim3(1024), dim3(256), 0, s, dev + off, W, (const uint8_t *const *)din, nin, seg);
                hipLaunchKernelGGL(k_scatter, dim3(256), dim3(256), 0, s, (uint8_t *const *)dout, dev + (uint64_t)nin * W + off,
                                   W, nout, seg);
            }
        CK(hipGetLastError());
        CK(hipStreamSynchronize(s));
        auto t2 = now();
        // gather only / scatter only, whole rows
        for (int k = 0; k < reps; k++)
            hipLaunchKernelGGL(k_gather, dim3(1024), dim3(256), 0, s, dev, W, (const uint8_t *const *)din, nin, W);
        CK(hipStreamSynchronize(s));
        auto t3 = now();
        for (int k = 0; k < reps; k++)
            hipLaunchKernelGGL(k_scatter, dim3(256), dim3(256), 0, s, (uint8_t *const *)dout, dev + (uint64_t)nin * W, W,
                               nout, W);
        CK(hipStreamSynchronize(s));
        auto t4 = now();
        const double bytes = (double)(nin + nout) * W * reps;
        std::printf("{\"seg\": %llu, \"memcpy_GBps\": %.1f, \"kernels_GBps\": %.1f, \"gather_GBps\": %.1f, \"scatter_GBps\": %.1f}\n",
                    (unsigned long long)seg, bytes / secs(t0, t1) / 1e9, bytes / secs(t1, t2) / 1e9,
                    (double)nin * W * reps / secs(t2, t3) / 1e9, (double)nout * W * reps / secs(t3, t4) / 1e9);
    }
    return 0;
}
