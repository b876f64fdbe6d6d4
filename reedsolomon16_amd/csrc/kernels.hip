// HIP kernels (gfx950 / CDNA4) for the Leopard-FFT Reed-Solomon codec.
//
// Arithmetic: GF(2^16) / GF(2^8) multiply-by-constant as byte permutes.
// A twiddle (multiply by exp(log_m)) is shipped as byte tables (gf_host.cpp,
// make_twiddle); the symbol is split into bit groups of <= 3 bits and each
// group is looked up for 4 symbols at once with one v_perm_b32 per output
// byte plane.  Tables are wave-uniform (SGPR operands).  No MFMA: the work is
// GF(2) XOR / table lookup, not a dense float contraction.
//
// Data layout (reference-compatible): GF(2^16) shards are 64-byte blocks of
// 32 symbols, low bytes [0,32) and high bytes [32,64) (leopard16.go:778-792).
// A lane "unit" is W dwords of the low half plus the same W dwords of the
// high half of one block (4*W symbols).  GF(2^8): a unit is W dwords (4*W
// byte symbols).  Consecutive lanes touch consecutive addresses.
//
// Butterflies (reference semantics, galois_noasm.go:58-76, leopard16.go:660-772):
//   IFFT: y ^= x; x ^= y*m        FFT: x ^= y*m; y ^= x
//   log_m == modulus means a zero twiddle: XOR only (wave-uniform branch).
#include "kernels.hpp"

namespace rs {
namespace {

template <int W> struct VecOf;
template <> struct VecOf<1> { typedef uint32_t T; };
template <> struct VecOf<2> { typedef uint32_t T __attribute__((ext_vector_type(2))); };
template <> struct VecOf<4> { typedef uint32_t T __attribute__((ext_vector_type(4))); };

template <int W>
__device__ __forceinline__ void ldw(const uint8_t *p, uint32_t (&v)[W]) {
    typedef typename VecOf<W>::T T;
    const T x = *reinterpret_cast<const T *>(p);
    if constexpr (W == 1) {
        v[0] = x;
    } else {
#pragma unroll
        for (int i = 0; i < W; i++) v[i] = x[i];
    }
}
template <int W>
__device__ __forceinline__ void stw(uint8_t *p, const uint32_t (&v)[W]) {
    typedef typename VecOf<W>::T T;
    T x;
    if constexpr (W == 1) {
        x = v[0];
    } else {
#pragma unroll
        for (int i = 0; i < W; i++) x[i] = v[i];
    }
    *reinterpret_cast<T *>(p) = x;
}

__device__ __forceinline__ uint32_t perm(uint32_t s0, uint32_t s1, uint32_t sel) {
    return __builtin_amdgcn_perm(s0, s1, sel);
}

// ---------------------------------------------------------------- GF(2^16)
template <int W_>
struct F16 {
    static constexpr int W = W_;
    static constexpr int TWD = 24;     // dwords per twiddle table
    static constexpr int LOGIDX = 20;  // dword holding log_m
    static constexpr uint32_t MOD = 65535;
    static constexpr int UPB = 8 / W;  // units per 64-byte block
    struct Vec {
        uint32_t l[W], h[W];
    };
    __device__ static uint64_t units(uint64_t S) { return (S >> 6) * UPB; }
    __device__ static uint64_t off(uint64_t u) { return (u / UPB) * 64 + (u % UPB) * (4 * W); }
    __device__ static Vec load(const uint8_t *row, uint64_t u) {
        Vec v;
        const uint8_t *p = row + off(u);
        ldw<W>(p, v.l);
        ldw<W>(p + 32, v.h);
        return v;
    }
    __device__ static void store(uint8_t *row, uint64_t u, const Vec &v) {
        uint8_t *p = row + off(u);
        stw<W>(p, v.l);
        stw<W>(p + 32, v.h);
    }
    __device__ static Vec zero() {
        Vec v;
#pragma unroll
        for (int i = 0; i < W; i++) v.l[i] = v.h[i] = 0;
        return v;
    }
    __device__ static void xor_into(Vec &a, const Vec &b) {
#pragma unroll
        for (int i = 0; i < W; i++) {
            a.l[i] ^= b.l[i];
            a.h[i] ^= b.h[i];
        }
    }
    __device__ static uint32_t diff(const Vec &a, const Vec &b) {
        uint32_t d = 0;
#pragma unroll
        for (int i = 0; i < W; i++) d |= (a.l[i] ^ b.l[i]) | (a.h[i] ^ b.h[i]);
        return d;
    }
    // x ^= y * exp(log_m); t = twiddle table (wave-uniform).
    __device__ static void mul_add(Vec &x, const Vec &y, const uint32_t *__restrict__ t) {
#pragma unroll
        for (int i = 0; i < W; i++) {
            const uint32_t lo = y.l[i], hi = y.h[i];
            const uint32_t a0 = lo & 0x07070707u, a1 = (lo >> 3) & 0x07070707u, a2 = (lo >> 6) & 0x03030303u;
            const uint32_t b0 = hi & 0x07070707u, b1 = (hi >> 3) & 0x07070707u, b2 = (hi >> 6) & 0x03030303u;
            x.l[i] ^= perm(t[1], t[0], a0) ^ perm(t[5], t[4], a1) ^ perm(t[8], t[8], a2) ^ perm(t[11], t[10], b0) ^
                      perm(t[15], t[14], b1) ^ perm(t[18], t[18], b2);
            x.h[i] ^= perm(t[3], t[2], a0) ^ perm(t[7], t[6], a1) ^ perm(t[9], t[9], a2) ^ perm(t[13], t[12], b0) ^
                      perm(t[17], t[16], b1) ^ perm(t[19], t[19], b2);
        }
    }
};

// ---------------------------------------------------------------- GF(2^8)
template <int W_>
struct F8 {
    static constexpr int W = W_;
    static constexpr int TWD = 8;
    static constexpr int LOGIDX = 5;
    static constexpr uint32_t MOD = 255;
    struct Vec {
        uint32_t b[W];
    };
    __device__ static uint64_t units(uint64_t S) { return S / (4 * W); }
    __device__ static uint64_t off(uint64_t u) { return u * (4 * W); }
    __device__ static Vec load(const uint8_t *row, uint64_t u) {
        Vec v;
        ldw<W>(row + off(u), v.b);
        return v;
    }
    __device__ static void store(uint8_t *row, uint64_t u, const Vec &v) { stw<W>(row + off(u), v.b); }
    __device__ static Vec zero() {
        Vec v;
#pragma unroll
        for (int i = 0; i < W; i++) v.b[i] = 0;
        return v;
    }
    __device__ static void xor_into(Vec &a, const Vec &b) {
#pragma unroll
        for (int i = 0; i < W; i++) a.b[i] ^= b.b[i];
    }
    __device__ static uint32_t diff(const Vec &a, const Vec &b) {
        uint32_t d = 0;
#pragma unroll
        for (int i = 0; i < W; i++) d |= a.b[i] ^ b.b[i];
        return d;
    }
    __device__ static void mul_add(Vec &x, const Vec &y, const uint32_t *__restrict__ t) {
#pragma unroll
        for (int i = 0; i < W; i++) {
            const uint32_t v = y.b[i];
            const uint32_t a0 = v & 0x07070707u, a1 = (v >> 3) & 0x07070707u, a2 = (v >> 6) & 0x03030303u;
            x.b[i] ^= perm(t[1], t[0], a0) ^ perm(t[3], t[2], a1) ^ perm(t[4], t[4], a2);
        }
    }
};

// ---------------------------------------------------------------- butterflies
template <class F>
__device__ __forceinline__ void ifft2(typename F::Vec &x, typename F::Vec &y, const uint32_t *__restrict__ t) {
    F::xor_into(y, x);
    if (t[F::LOGIDX] != F::MOD) F::mul_add(x, y, t);
}
template <class F>
__device__ __forceinline__ void fft2(typename F::Vec &x, typename F::Vec &y, const uint32_t *__restrict__ t) {
    if (t[F::LOGIDX] != F::MOD) F::mul_add(x, y, t);
    F::xor_into(y, x);
}
// Slot order of a radix-4 group: t[0] = m01, t[1] = m02, t[2] = m23 (each F::TWD dwords).
template <class F>
__device__ __forceinline__ void ifft4(typename F::Vec &x0, typename F::Vec &x1, typename F::Vec &x2,
                                      typename F::Vec &x3, const uint32_t *__restrict__ t) {
    ifft2<F>(x0, x1, t);               // m01
    ifft2<F>(x2, x3, t + 2 * F::TWD);  // m23
    ifft2<F>(x0, x2, t + F::TWD);      // m02
    ifft2<F>(x1, x3, t + F::TWD);
}
template <class F>
__device__ __forceinline__ void fft4(typename F::Vec &x0, typename F::Vec &x1, typename F::Vec &x2, typename F::Vec &x3,
                                     const uint32_t *__restrict__ t) {
    fft2<F>(x0, x2, t + F::TWD);  // m02
    fft2<F>(x1, x3, t + F::TWD);
    fft2<F>(x0, x1, t);               // m01
    fft2<F>(x2, x3, t + 2 * F::TWD);  // m23
}

// Twiddle slots of an IFFT of size 2^logm (must match gf_host.cpp ifft_passes).
constexpr int ifft_slot_count(int logm) {
    int M = 1 << logm, s = 0, dist = 1;
    for (; dist * 4 <= M; dist *= 4) s += 3 * (M / (4 * dist));
    if (dist < M) s += 1;
    return s;
}

__device__ __forceinline__ uint8_t *row_ptr(const RowSet &rs, int i) {
    return rs.table ? rs.table[i] : rs.base + (uint64_t)i * rs.stride;
}

// ---------------------------------------------------------------- register transforms (M <= 32)
// ifftDITEncoder transform (leopard16.go:694-741): radix-4 pairs at dist 1,4,16,
// then a radix-2 layer at M/2 when log2(M) is odd.  Groups with r >= mtrunc
// hold only zero rows and are skipped (uniform branch), as in the reference.
template <class F, int LOGM>
__device__ __forceinline__ void ifft_reg(typename F::Vec (&w)[1 << LOGM], const uint32_t *__restrict__ tw, int mtrunc) {
    constexpr int M = 1 << LOGM;
    int slot = 0;
#pragma unroll
    for (int dist = 1; dist * 4 <= M; dist *= 4) {
#pragma unroll
        for (int r = 0; r < M; r += 4 * dist) {
            const uint32_t *t = tw + slot * F::TWD;
            slot += 3;
            if (r < mtrunc) {
#pragma unroll
                for (int i = r; i < r + dist; i++) ifft4<F>(w[i], w[i + dist], w[i + 2 * dist], w[i + 3 * dist], t);
            }
        }
    }
    if constexpr (LOGM & 1) {
        constexpr int d = M / 2;
        const uint32_t *t = tw + slot * F::TWD;
#pragma unroll
        for (int i = 0; i < d; i++) ifft2<F>(w[i], w[i + d], t);
    }
}

// fftDIT (leopard16.go:618-657): radix-4 pairs at dist M/4, M/16, ..., then a
// radix-2 layer at dist 1 when log2(M) is odd; groups with r >= mtrunc skipped.
template <class F, int LOGM>
__device__ __forceinline__ void fft_reg(typename F::Vec (&w)[1 << LOGM], const uint32_t *__restrict__ tw, int mtrunc) {
    constexpr int M = 1 << LOGM;
    int slot = 0;
#pragma unroll
    for (int dist = M / 4; dist != 0; dist /= 4) {
#pragma unroll
        for (int r = 0; r < M; r += 4 * dist) {
            const uint32_t *t = tw + slot * F::TWD;
            slot += 3;
            if (r < mtrunc) {
#pragma unroll
                for (int i = r; i < r + dist; i++) fft4<F>(w[i], w[i + dist], w[i + 2 * dist], w[i + 3 * dist], t);
            }
        }
    }
    if constexpr (LOGM & 1) {
#pragma unroll
        for (int r = 0; r < M; r += 2) {
            const uint32_t *t = tw + (slot + r / 2) * F::TWD;
            if (r < mtrunc) fft2<F>(w[r], w[r + 1], t);
        }
    }
}

template <class F, int M>
__device__ __forceinline__ void load_chunk(typename F::Vec (&w)[M], const EncodeArgs &a, int c, uint64_t soff,
                                           uint64_t u) {
    const int row0 = c * M;
    const int cnt = a.k - row0;
#pragma unroll
    for (int r = 0; r < M; r++) {
        if (r < cnt) w[r] = F::load(row_ptr(a.data, row0 + r) + soff, u);
        else w[r] = F::zero();
    }
}

// Fused encode (leopard16.go:128-224 / leopard8.go:153-277) for m = 2^LOGM <= 32.
// Every lane owns one column unit of all k+p rows; the m-row work set, the
// m-row accumulator and the prefetched next chunk live in VGPRs, so HBM sees
// exactly k reads and p writes (or p reads for verify) per unit.
template <class F, int LOGM, bool VERIFY>
__global__ void __launch_bounds__(256, 2) k_encode_reg(EncodeArgs a) {
    constexpr int M = 1 << LOGM;
    typedef typename F::Vec V;
    const uint64_t units = F::units(a.shard_size);
    const uint64_t u = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (u >= units) return;
    const uint64_t soff = (uint64_t)blockIdx.y * a.stripe_stride;
    V acc[M], cur[M];
    load_chunk<F, M>(cur, a, 0, soff, u);
    for (int c = 0; c < a.nchunks; ++c) {
        V nxt[M];
        const bool more = c + 1 < a.nchunks;
        if (more) load_chunk<F, M>(nxt, a, c + 1, soff, u);
        const int cnt = a.k - c * M;
        ifft_reg<F, LOGM>(cur, a.tw_ifft + (uint64_t)c * ifft_slot_count(LOGM) * F::TWD, cnt);
        if (c == 0) {
#pragma unroll
            for (int r = 0; r < M; r++) acc[r] = cur[r];
        } else {
#pragma unroll
            for (int r = 0; r < M; r++) F::xor_into(acc[r], cur[r]);
        }
        if (more) {
#pragma unroll
            for (int r = 0; r < M; r++) cur[r] = nxt[r];
        }
    }
    fft_reg<F, LOGM>(acc, a.tw_fft, a.p);
    if constexpr (VERIFY) {
        uint32_t bad = 0;
#pragma unroll
        for (int r = 0; r < M; r++)
            if (r < a.p) bad |= F::diff(acc[r], F::load(row_ptr(a.parity, r) + soff, u));
        if (bad) atomicOr(a.mismatch, 1);
    } else {
#pragma unroll
        for (int r = 0; r < M; r++)
            if (r < a.p) F::store(row_ptr(a.parity, r) + soff, u, acc[r]);
    }
}

// ---------------------------------------------------------------- multi-pass kernels (any m / n)
// Each thread owns one column unit of one butterfly; rows live in a
// contiguous work slab (row stride = S).  Used for m > 32 and for decode.
typedef F8<4> Bytes16;  // field-agnostic 16-byte-per-lane view for copies and XORs

template <class F, bool INV>
__global__ void __launch_bounds__(256) k_pass4(uint8_t *work, uint64_t S, int dist, const uint32_t *__restrict__ tw,
                                               int q_off) {
    typedef typename F::Vec V;
    const uint64_t u = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (u >= F::units(S)) return;
    const int q = blockIdx.y + q_off;
    const int g = q / dist;
    const int i = g * 4 * dist + (q - g * dist);
    const uint32_t *t = tw + (uint64_t)g * 3 * F::TWD;
    uint8_t *r0 = work + (uint64_t)i * S;
    uint8_t *r1 = r0 + (uint64_t)dist * S;
    uint8_t *r2 = r1 + (uint64_t)dist * S;
    uint8_t *r3 = r2 + (uint64_t)dist * S;
    V x0 = F::load(r0, u), x1 = F::load(r1, u), x2 = F::load(r2, u), x3 = F::load(r3, u);
    if constexpr (INV) ifft4<F>(x0, x1, x2, x3, t);
    else fft4<F>(x0, x1, x2, x3, t);
    F::store(r0, u, x0);
    F::store(r1, u, x1);
    F::store(r2, u, x2);
    F::store(r3, u, x3);
}

// Radix-2 layer.  Inverse: pairs (i, i+dist), one twiddle.  Forward: dist = 1,
// pairs (2g, 2g+1) with twiddle g.
template <class F, bool INV>
__global__ void __launch_bounds__(256) k_pass2(uint8_t *work, uint64_t S, int dist, const uint32_t *__restrict__ tw,
                                               int q_off) {
    typedef typename F::Vec V;
    const uint64_t u = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (u >= F::units(S)) return;
    const int q = blockIdx.y + q_off;
    uint8_t *rx, *ry;
    const uint32_t *t;
    if constexpr (INV) {
        rx = work + (uint64_t)q * S;
        ry = rx + (uint64_t)dist * S;
        t = tw;
    } else {
        rx = work + (uint64_t)(2 * q) * S;
        ry = rx + S;
        t = tw + (uint64_t)q * F::TWD;
    }
    V x = F::load(rx, u), y = F::load(ry, u);
    if constexpr (INV) ifft2<F>(x, y, t);
    else fft2<F>(x, y, t);
    F::store(rx, u, x);
    F::store(ry, u, y);
}

__global__ void __launch_bounds__(256) k_gather(uint8_t *work, uint64_t S, RowSet src, int row0, int cnt, int r_off) {
    const uint64_t u = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (u >= Bytes16::units(S)) return;
    const int r = blockIdx.y + r_off;
    Bytes16::Vec v = r < cnt ? Bytes16::load(row_ptr(src, row0 + r), u) : Bytes16::zero();
    Bytes16::store(work + (uint64_t)r * S, u, v);
}

__global__ void __launch_bounds__(256) k_xor_rows(uint8_t *dst, const uint8_t *src, uint64_t S, int r_off) {
    const uint64_t u = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (u >= Bytes16::units(S)) return;
    const uint64_t r = blockIdx.y + r_off;
    Bytes16::Vec a = Bytes16::load(dst + r * S, u);
    Bytes16::xor_into(a, Bytes16::load(src + r * S, u));
    Bytes16::store(dst + r * S, u, a);
}

template <bool VERIFY>
__global__ void __launch_bounds__(256) k_copy_out(RowSet out, const uint8_t *work, uint64_t S, int *mismatch,
                                                  int r_off) {
    const uint64_t u = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (u >= Bytes16::units(S)) return;
    const int r = blockIdx.y + r_off;
    Bytes16::Vec v = Bytes16::load(work + (uint64_t)r * S, u);
    if constexpr (VERIFY) {
        if (Bytes16::diff(v, Bytes16::load(row_ptr(out, r), u))) atomicOr(mismatch, 1);
    } else {
        Bytes16::store(row_ptr(out, r), u, v);
    }
}

// mulgf16 (leopard16.go:492-514): always through the table (log 65535 is the
// identity there, unlike a butterfly twiddle).
template <class F>
__global__ void __launch_bounds__(256) k_scale_in(uint8_t *work, uint64_t S, const uint8_t *const *src,
                                                  const uint32_t *__restrict__ tw, int r_off) {
    const uint64_t u = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (u >= F::units(S)) return;
    const int r = blockIdx.y + r_off;
    const uint8_t *s = src[r];
    typename F::Vec v = F::zero();
    if (s) F::mul_add(v, F::load(s, u), tw + (uint64_t)r * F::TWD);
    F::store(work + (uint64_t)r * S, u, v);
}

// Formal derivative (leopard16.go:527-530) in closed form:
//   out[r] = in[r] ^ XOR_{b : bit b of r is 0} in[r | 2^b].
// Rows are visited in increasing order, so every row read is still original.
__global__ void __launch_bounds__(256) k_formal_derivative(uint8_t *work, uint64_t S, int n) {
    const uint64_t u = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (u >= Bytes16::units(S)) return;
    for (int r = 0; r < n; r++) {
        Bytes16::Vec v = Bytes16::load(work + (uint64_t)r * S, u);
        for (int b = 1; b < n; b <<= 1)
            if (!(r & b)) Bytes16::xor_into(v, Bytes16::load(work + (uint64_t)(r | b) * S, u));
        Bytes16::store(work + (uint64_t)r * S, u, v);
    }
}

template <class F>
__global__ void __launch_bounds__(256) k_reveal(uint8_t *const *dst, const uint8_t *work, uint64_t S, const int *pos,
                                                const uint32_t *__restrict__ tw, int i_off) {
    const uint64_t u = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (u >= F::units(S)) return;
    const int i = blockIdx.y + i_off;
    typename F::Vec v = F::zero();
    F::mul_add(v, F::load(work + (uint64_t)pos[i] * S, u), tw + (uint64_t)i * F::TWD);
    F::store(dst[i], u, v);
}

constexpr int kMaxGridY = 32768;
inline dim3 grid_x(uint64_t units) { return dim3((unsigned)((units + 255) / 256)); }

// Launch `body(y0, ny)` over y in [0, total) in slices of kMaxGridY.
template <class Fn>
hipError_t for_y(int total, Fn body) {
    for (int y0 = 0; y0 < total; y0 += kMaxGridY) {
        const int ny = total - y0 < kMaxGridY ? total - y0 : kMaxGridY;
        body(y0, ny);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

template <class F, int LOGM>
hipError_t enc_reg(bool verify, const EncodeArgs &a, hipStream_t s) {
    uint64_t nunits;
    if constexpr (F::TWD == 24) nunits = (a.shard_size >> 6) * (8 / F::W);
    else nunits = a.shard_size / (4 * F::W);
    dim3 grid((unsigned)((nunits + 255) / 256), (unsigned)a.nstripes);
    if (verify) hipLaunchKernelGGL((k_encode_reg<F, LOGM, true>), grid, dim3(256), 0, s, a);
    else hipLaunchKernelGGL((k_encode_reg<F, LOGM, false>), grid, dim3(256), 0, s, a);
    return hipGetLastError();
}

}  // namespace

// Lane width per (field, log2 m): keep acc + work + prefetch <= ~192 VGPRs
// (2 waves/SIMD) while using the widest coalesced access that fits.
hipError_t launch_encode_reg(int bits, int logm, bool verify, const EncodeArgs &a, hipStream_t s) {
    if (bits == 16) {
        switch (logm) {
            case 0: return enc_reg<F16<4>, 0>(verify, a, s);
            case 1: return enc_reg<F16<4>, 1>(verify, a, s);
            case 2: return enc_reg<F16<4>, 2>(verify, a, s);
            case 3: return enc_reg<F16<4>, 3>(verify, a, s);
            case 4: return enc_reg<F16<2>, 4>(verify, a, s);
            case 5: return enc_reg<F16<1>, 5>(verify, a, s);
        }
    } else {
        switch (logm) {
            case 0: return enc_reg<F8<4>, 0>(verify, a, s);
            case 1: return enc_reg<F8<4>, 1>(verify, a, s);
            case 2: return enc_reg<F8<4>, 2>(verify, a, s);
            case 3: return enc_reg<F8<4>, 3>(verify, a, s);
            case 4: return enc_reg<F8<4>, 4>(verify, a, s);
            case 5: return enc_reg<F8<2>, 5>(verify, a, s);
        }
    }
    return hipErrorInvalidValue;
}

const char *encode_reg_name(int bits, int logm) {
    static const char *n16[] = {"reg16-m1", "reg16-m2", "reg16-m4", "reg16-m8", "reg16-m16", "reg16-m32"};
    static const char *n8[] = {"reg8-m1", "reg8-m2", "reg8-m4", "reg8-m8", "reg8-m16", "reg8-m32"};
    if (logm < 0 || logm > 5) return "none";
    return bits == 16 ? n16[logm] : n8[logm];
}

hipError_t launch_gather(int bits, uint8_t *work, uint64_t S, RowSet src, int row0, int cnt, int rows, hipStream_t s) {
    (void)bits;
    return for_y(rows, [&](int y0, int ny) {
        hipLaunchKernelGGL(k_gather, dim3(grid_x(S / 16).x, ny), dim3(256), 0, s, work, S, src, row0, cnt, y0);
    });
}

hipError_t launch_pass(int bits, bool inverse, uint8_t *work, uint64_t S, int dist, int radix, int groups_active,
                       const uint32_t *tw, hipStream_t s) {
    if (groups_active <= 0) return hipSuccess;
    if (radix == 4) {
        const int quads = groups_active * dist;
        return for_y(quads, [&](int y0, int ny) {
            if (bits == 16) {
                dim3 g(grid_x((S >> 6) * 8).x, ny);
                if (inverse) hipLaunchKernelGGL((k_pass4<F16<1>, true>), g, dim3(256), 0, s, work, S, dist, tw, y0);
                else hipLaunchKernelGGL((k_pass4<F16<1>, false>), g, dim3(256), 0, s, work, S, dist, tw, y0);
            } else {
                dim3 g(grid_x(S / 16).x, ny);
                if (inverse) hipLaunchKernelGGL((k_pass4<F8<4>, true>), g, dim3(256), 0, s, work, S, dist, tw, y0);
                else hipLaunchKernelGGL((k_pass4<F8<4>, false>), g, dim3(256), 0, s, work, S, dist, tw, y0);
            }
        });
    }
    const int pairs = inverse ? dist : groups_active;
    return for_y(pairs, [&](int y0, int ny) {
        if (bits == 16) {
            dim3 g(grid_x((S >> 6) * 8).x, ny);
            if (inverse) hipLaunchKernelGGL((k_pass2<F16<1>, true>), g, dim3(256), 0, s, work, S, dist, tw, y0);
            else hipLaunchKernelGGL((k_pass2<F16<1>, false>), g, dim3(256), 0, s, work, S, dist, tw, y0);
        } else {
            dim3 g(grid_x(S / 16).x, ny);
            if (inverse) hipLaunchKernelGGL((k_pass2<F8<4>, true>), g, dim3(256), 0, s, work, S, dist, tw, y0);
            else hipLaunchKernelGGL((k_pass2<F8<4>, false>), g, dim3(256), 0, s, work, S, dist, tw, y0);
        }
    });
}

hipError_t launch_xor_rows(int bits, uint8_t *dst, const uint8_t *src, uint64_t S, int rows, hipStream_t s) {
    (void)bits;
    return for_y(rows, [&](int y0, int ny) {
        hipLaunchKernelGGL(k_xor_rows, dim3(grid_x(S / 16).x, ny), dim3(256), 0, s, dst, src, S, y0);
    });
}

hipError_t launch_copy_out(int bits, RowSet out, const uint8_t *work, uint64_t S, int rows, int *mismatch,
                           hipStream_t s) {
    (void)bits;
    return for_y(rows, [&](int y0, int ny) {
        if (mismatch)
            hipLaunchKernelGGL(k_copy_out<true>, dim3(grid_x(S / 16).x, ny), dim3(256), 0, s, out, work, S, mismatch, y0);
        else
            hipLaunchKernelGGL(k_copy_out<false>, dim3(grid_x(S / 16).x, ny), dim3(256), 0, s, out, work, S, mismatch,
                               y0);
    });
}

hipError_t launch_scale_in(int bits, uint8_t *work, uint64_t S, const uint8_t *const *src, const uint32_t *tw, int rows,
                           hipStream_t s) {
    return for_y(rows, [&](int y0, int ny) {
        if (bits == 16)
            hipLaunchKernelGGL(k_scale_in<F16<1>>, dim3(grid_x((S >> 6) * 8).x, ny), dim3(256), 0, s, work, S, src, tw, y0);
        else
            hipLaunchKernelGGL(k_scale_in<F8<4>>, dim3(grid_x(S / 16).x, ny), dim3(256), 0, s, work, S, src, tw, y0);
    });
}

hipError_t launch_formal_derivative(int bits, uint8_t *work, uint64_t S, int n, hipStream_t s) {
    (void)bits;
    hipLaunchKernelGGL(k_formal_derivative, grid_x(S / 16), dim3(256), 0, s, work, S, n);
    return hipGetLastError();
}

hipError_t launch_reveal(int bits, uint8_t *const *dst, const uint8_t *work, uint64_t S, const int *pos,
                         const uint32_t *tw, int count, hipStream_t s) {
    return for_y(count, [&](int y0, int ny) {
        if (bits == 16)
            hipLaunchKernelGGL(k_reveal<F16<1>>, dim3(grid_x((S >> 6) * 8).x, ny), dim3(256), 0, s, dst, work, S, pos, tw,
                               y0);
        else
            hipLaunchKernelGGL(k_reveal<F8<4>>, dim3(grid_x(S / 16).x, ny), dim3(256), 0, s, dst, work, S, pos, tw, y0);
    });
}

}  // namespace rs
