// Bit-sliced GF(2^16) encode for m = 32 (gfx950), specialized per geometry.
//
// Why: multiplying by a twiddle with v_perm_b32 byte tables costs ~115 SIMD
// cycles per 4 symbols (12 half-rate v_perm_b32 + extraction + XOR folding,
// scripts/micro/split_rate.hip), which caps the table-driven kernels at ~45 us
// of pure VALU for C3.  In bit-sliced form (a 32-bit word holds one bit of 32
// symbols) a multiply by a *known* constant is a fixed XOR network: output
// plane i = XOR of the input planes in row i of the twiddle's 16x16 GF(2)
// matrix -- about 50 full-rate v_bitop3_b32 per 32 symbols.  The matrices
// are generated at build time for the geometries listed in the Makefile
// (tools/gen_bs_tables.cpp -> build/bs_tables.h), so every twiddle is an
// instruction-stream constant.
//
// Work split (one 512-thread workgroup per CU, persistent over tiles): a tile
// is 64 adjacent 64-byte blocks (4 KB) of every row of one stripe; lane l owns
// block l (32 symbols) in every wave.  The 8 waves split the 32 rows of a
// transform; each radix-4 pass runs in registers on the 4 rows a wave holds,
// and the passes exchange rows through a 32-row bit-sliced LDS image (128 KB).
// A wave's role (which rows, hence which twiddles) is its wave index, a
// wave-uniform value: every role has its own instruction stream.
//
//   chunk IFFT (leopard16.go:694-741):  pass 1 rows 4w+{0..3} (dist 1, 2)
//                                        pass 2 rows 16h+j+{0,4,8,12} (dist 4, 8)
//                                        pass 3 rows w+{0,8,16,24} (dist 16)
//   accumulator rows w+{0,8,16} stay in registers across chunks, row w+24 in
//   a private LDS row of the wave;
//   final FFT (leopard16.go:618-657):   pass A rows w+{0,8,16,24} (dist 16, 8)
//                                        pass B rows 8g+j+{0,2,4,6} (dist 4, 2)
//                                        pass C rows 4w+{0..3} (dist 1)
// HBM: each data row read once, each parity row written once; the next
// chunk's rows are prefetched into registers during the current chunk.
//
// Register budget (2 waves per SIMD -> 256 VGPRs): 64 staged + 64 working +
// 48 accumulator.  The XOR networks are written as in-place inline asm so the
// compiler cannot rename their intermediates into fresh registers, and every
// butterfly and chunk is a scheduling region of its own.
#include <algorithm>
#include <cstdlib>
#include <utility>

#include "bs_tables.h"
#include "kernels.hpp"

namespace rs {
// RS_BS_STAMP (diagnostic builds only, scripts/bs_stamps.py): per wave,
// s_memtime totals of the load wait at each chunk start, the LDS barriers,
// the final FFT + stores, and the whole run, written once per launch.
#ifndef RS_BS_STAMP
#define RS_BS_STAMP 0
#endif
#if RS_BS_STAMP
__device__ unsigned long long g_bs_stamps[1024 * 8 * 4];
#endif
namespace {

typedef uint32_t Planes[16];
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// v ^= a  /  v ^= a ^ b, in place (v_bitop3_b32 truth table 0x96 = 3-input XOR).
__device__ __forceinline__ void ixor(uint32_t &v, uint32_t a) { asm("v_xor_b32 %0, %1, %0" : "+v"(v) : "v"(a)); }
__device__ __forceinline__ void ixor3(uint32_t &v, uint32_t a, uint32_t b) {
    asm("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(v) : "v"(a), "v"(b));
}

// Delta swap of word-index bit k with bit-position bit k (s = 2^k, M = positions with bit k clear).
__device__ __forceinline__ void bs_xchg(uint32_t &a, uint32_t &b, int s, uint32_t M) {
    const uint32_t as = a >> s, bsh = b << s;
    a = (a & M) | (bsh & ~M);
    b = (b & ~M) | (as & M);
}
// A 64-byte block (dwords 0-7: low bytes of symbols 4w+j at byte j of dword w;
// dwords 8-15: high bytes) <-> 16 bit-planes (plane b bit 8j+w = bit b of symbol
// 4w+j; planes 8-15 from the high bytes).  An involution.
__device__ __forceinline__ void bs_transpose(Planes &w) {
#ifdef RS_BS_ABL_NOTRANS
    return;
#endif
#pragma unroll
    for (int h = 0; h < 16; h += 8)
#pragma unroll
        for (int k = 0; k < 3; k++) {
            const int s = 1 << k;
            const uint32_t M = k == 0 ? 0x55555555u : k == 1 ? 0x33333333u : 0x0F0F0F0Fu;
#pragma unroll
            for (int a = 0; a < 8; a++)
                if (!(a & s)) bs_xchg(w[h + a], w[h + a + s], s, M);
        }
}

__device__ __forceinline__ void xor16(Planes &y, const Planes &x) {
#pragma unroll
    for (int i = 0; i < 16; i++) ixor(y[i], x[i]);
}

// x ^= y * twiddle (C >= 0: chunk C's IFFT slot; C < 0: FFT slot).
// Each output plane is a chain of 3-input XORs over the input planes its
// matrix row selects.
// out ^= XOR of y[B + j] over the set bits j of mask (3-input XOR pairs).
__device__ __forceinline__ void xor_rows(uint32_t &out, const Planes &y, int B, uint32_t mask, int nbits) {
    int pend = -1;
#pragma unroll
    for (int j = 0; j < nbits; j++) {
        if ((mask >> j) & 1) {
            if (pend < 0) {
                pend = j;
            } else {
                ixor3(out, y[B + pend], y[B + j]);
                pend = -1;
            }
        }
    }
    if (pend >= 0) ixor(out, y[B + pend]);
}
// Subfield coordinates (gf_host.hpp SubCoords): planes 0-7 ^= D(planes 8-15).
// An involution; applied after the load transpose and before the store one.
template <class TW>
__device__ __forceinline__ void bs_psi(Planes &w) {
#pragma unroll
    for (int r = 0; r < 8; r++) xor_rows(w[r], w, 8, TW::dmat[r], 8);
}
template <class TW, int C, int SLOT>
__device__ __forceinline__ void bs_mul_add(Planes &x, const Planes &y) {
#ifdef RS_BS_ABL_NOMUL  // ablation (performance experiments only)
    return;
#endif
    if constexpr (TW::SUB) {
        // one 8x8 network per byte half
#pragma unroll
        for (int h = 0; h < 16; h += 8)
#pragma unroll
            for (int i = 0; i < 8; i++)
                xor_rows(x[h + i], y, h, C < 0 ? TW::fft8[SLOT][i] : TW::ifft8[C < 0 ? 0 : C][SLOT][i], 8);
        return;
    }
#pragma unroll
    for (int i = 0; i < 16; i++) {
        const uint32_t r = C < 0 ? TW::fft[SLOT][i] : TW::ifft[C < 0 ? 0 : C][SLOT][i];
        int pend = -1;
#pragma unroll
        for (int j = 0; j < 16; j++) {
            if ((r >> j) & 1) {
                if (pend < 0) {
                    pend = j;
                } else {
                    ixor3(x[i], y[pend], y[j]);
                    pend = -1;
                }
            }
        }
        if (pend >= 0) ixor(x[i], y[pend]);
    }
}
// IFFT butterfly: y ^= x; x ^= y * t.   FFT butterfly: x ^= y * t; y ^= x.
// Each butterfly is a scheduling region of its own (sched_barrier): the
// machine scheduler would otherwise interleave butterflies for ILP and run
// the kernel out of registers.
template <class TW, int C, int SLOT>
__device__ __forceinline__ void bs_ifft2(Planes &x, Planes &y) {
    xor16(y, x);
    bs_mul_add<TW, C, SLOT>(x, y);
    __builtin_amdgcn_sched_barrier(0);
}
template <class TW, int SLOT>
__device__ __forceinline__ void bs_fft2(Planes &x, Planes &y) {
    bs_mul_add<TW, -1, SLOT>(x, y);
    xor16(y, x);
    __builtin_amdgcn_sched_barrier(0);
}
// Radix-4 groups with slots (m01, m02, m23) = (S0, S0+1, S0+2).
template <class TW, int C, int S0>
__device__ __forceinline__ void bs_ifft4(Planes (&r)[4]) {
    bs_ifft2<TW, C, S0>(r[0], r[1]);
    bs_ifft2<TW, C, S0 + 2>(r[2], r[3]);
    bs_ifft2<TW, C, S0 + 1>(r[0], r[2]);
    bs_ifft2<TW, C, S0 + 1>(r[1], r[3]);
}
template <class TW, int S0>
__device__ __forceinline__ void bs_fft4(Planes (&r)[4]) {
    bs_fft2<TW, S0 + 1>(r[0], r[2]);
    bs_fft2<TW, S0 + 1>(r[1], r[3]);
    bs_fft2<TW, S0>(r[0], r[1]);
    bs_fft2<TW, S0 + 2>(r[2], r[3]);
}

// Wave-uniform dispatch of a role-specialized pass: f(std::integral_constant<int, R>) for R = role.
template <int N, class Fn, int... Is>
__device__ __forceinline__ void dispatch_impl(int role, Fn &&f, std::integer_sequence<int, Is...>) {
    ((role == Is ? (f(std::integral_constant<int, Is>{}), 0) : 0), ...);
}
template <int N, class Fn>
__device__ __forceinline__ void dispatch(int role, Fn &&f) {
    dispatch_impl<N>(role, f, std::make_integer_sequence<int, N>{});
}

// LDS image: row r, plane quad q of lane l at dword r*1024 + q*256 + l*4.
typedef __attribute__((address_space(3))) u32x4 lds_u4;
// The row address is rebuilt at every use from an opaque copy of the lane base
// (one v_add): otherwise the compiler hoists every row address out of the
// persistent tile loop and spills them.
__device__ __forceinline__ uint32_t row_addr(uint32_t lbase, int row) {
    uint32_t b = lbase;
    asm volatile("" : "+v"(b));
    return b + (uint32_t)row * 4096u;
}
__device__ __forceinline__ void lds_put(uint32_t lbase, int row, const Planes &v) {
#ifdef RS_BS_ABL_NOLDS
    return;
#endif
    const uint32_t ra = row_addr(lbase, row);
#pragma unroll
    for (int q = 0; q < 4; q++)
        *(lds_u4 *)(uintptr_t)(ra + q * 1024) = u32x4{v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]};
}
__device__ __forceinline__ void lds_get(uint32_t lbase, int row, Planes &v) {
#ifdef RS_BS_ABL_NOLDS
#pragma unroll
    for (int q = 0; q < 16; q++) asm volatile("" : "+v"(v[q]));
    return;
#endif
    const uint32_t ra = row_addr(lbase, row);
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const u32x4 x = *(const lds_u4 *)(uintptr_t)(ra + q * 1024);
        v[4 * q] = x[0];
        v[4 * q + 1] = x[1];
        v[4 * q + 2] = x[2];
        v[4 * q + 3] = x[3];
    }
}

// Workgroup barrier for the LDS image only.  __syncthreads() is also a
// release/acquire fence, which waits for every outstanding global load
// (vmcnt(0)) and so would drain the next chunk's prefetch at the first
// barrier of every chunk; this waits for LDS traffic alone.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

typedef __attribute__((address_space(1))) const u32x4 gc_u4;
typedef __attribute__((address_space(1))) u32x4 g_u4;

template <class TW, bool VERIFY>
struct BsEncoder {
    static constexpr int NCH = TW::NCH;
    const BsArgs &a;
    uint32_t lbase;  // this lane's LDS byte address of row 0, quad 0
    int lane, w;
    Planes St[4];    // staged data rows (64-byte blocks as loaded)
    Planes R[4];     // working rows (bit-planes)
    Planes A[3];     // accumulator rows w, w + 8, w + 16 (row w + 24's: LDS row 32 + w)
#if RS_BS_STAMP
    unsigned long long t_load = 0, t_bar = 0, t_fft = 0, t_total = 0;
#endif
    __device__ __forceinline__ void bar() {
#if RS_BS_STAMP
        const unsigned long long t0 = __builtin_amdgcn_s_memtime();
        lds_barrier();
        t_bar += __builtin_amdgcn_s_memtime() - t0;
#else
        lds_barrier();
#endif
    }

    // Load rows 32c + 4w + i of `tile` (zero past k, past the row end, past the last tile).
    __device__ __forceinline__ void stage(int tile, int c) {
        const int tps = a.tiles_per_stripe;
        const int stripe = tile / tps, ct = tile - stripe * tps;
        const uint64_t col = (uint64_t)ct * 4096 + (uint64_t)lane * 64;
#ifdef RS_BS_ABL_NOLOAD
        const bool ok = false;
#else
        const bool ok = tile < a.ntiles && col < a.S;
#endif
        const uint8_t *base = a.data + (uint64_t)stripe * a.stripe_stride + col;
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const int row = 32 * c + 4 * w + i;
            if (ok && row < a.k) {
                gc_u4 *p = (gc_u4 *)(base + (uint64_t)row * a.row_stride);
#pragma unroll
                for (int q = 0; q < 4; q++) {
#ifdef RS_BS_ABL_COALESCED  // same bytes, lane-contiguous 16-byte pieces (wrong layout)
                    const u32x4 x = *(gc_u4 *)(base - (uint64_t)lane * 64 + (uint64_t)row * a.row_stride + q * 1024 + lane * 16);
#elif defined(RS_BS_NT_LOAD)  // streamed once: non-temporal policy
                    const u32x4 x = __builtin_nontemporal_load(p + q);
#else
                    const u32x4 x = p[q];
#endif
                    St[i][4 * q] = x[0];
                    St[i][4 * q + 1] = x[1];
                    St[i][4 * q + 2] = x[2];
                    St[i][4 * q + 3] = x[3];
                }
            } else {
#pragma unroll
                for (int q = 0; q < 16; q++) St[i][q] = 0;
            }
        }
    }

    template <int C>
    __device__ __forceinline__ void chunk(int tile) {
        __builtin_amdgcn_sched_barrier(0);
#if RS_BS_STAMP  // the compiler waits vmcnt(0) here anyway (chunk 0 included)
        {
            const unsigned long long t0 = __builtin_amdgcn_s_memtime();
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            t_load += __builtin_amdgcn_s_memtime() - t0;
        }
#endif
#pragma unroll
        for (int i = 0; i < 4; i++) {
#pragma unroll
            for (int q = 0; q < 16; q++) R[i][q] = St[i][q];
            bs_transpose(R[i]);
            if constexpr (TW::SUB) bs_psi<TW>(R[i]);
        }
        // The staged rows are consumed before the next chunk's loads are
        // issued: the memory clobber keeps IR passes from sinking the
        // transposes below those loads (which made the wait for the current
        // rows also wait for the prefetch, serializing HBM and compute).
#pragma unroll
        for (int i = 0; i < 4; i++)
#pragma unroll
            for (int q = 0; q < 16; q++) asm volatile("" : "+v"(R[i][q])::"memory");
        __builtin_amdgcn_sched_barrier(0);
        if (C + 1 < NCH) stage(tile, C + 1);
        else stage(tile + (int)gridDim.x, 0);
        __builtin_amdgcn_sched_barrier(0);
        // pass 1: rows 4w + i, radix-4 at dist 1 (group w, slots 3w..3w+2)
        dispatch<8>(w, [&](auto W) { bs_ifft4<TW, C, 3 * decltype(W)::value>(R); });
        bar();  // previous readers of the image are done
#pragma unroll
        for (int i = 0; i < 4; i++) lds_put(lbase, 4 * w + i, R[i]);
        bar();
        // pass 2: rows 16h + j + 4i, radix-4 at dist 4 (group h, slots 24 + 3h ..)
        const int h = w >> 2, j = w & 3;
#pragma unroll
        for (int i = 0; i < 4; i++) lds_get(lbase, 16 * h + j + 4 * i, R[i]);
        dispatch<2>(h, [&](auto H) { bs_ifft4<TW, C, 24 + 3 * decltype(H)::value>(R); });
#pragma unroll
        for (int i = 0; i < 4; i++) lds_put(lbase, 16 * h + j + 4 * i, R[i]);
        bar();
        // pass 3: rows w + 8i, radix-2 at dist 16 (slot 30): pairs (w, w+16), (w+8, w+24)
#pragma unroll
        for (int i = 0; i < 4; i++) lds_get(lbase, w + 8 * i, R[i]);
        bs_ifft2<TW, C, 30>(R[0], R[2]);
        bs_ifft2<TW, C, 30>(R[1], R[3]);
#pragma unroll
        for (int i = 0; i < 3; i++) {
            if (C == 0) {
#pragma unroll
                for (int q = 0; q < 16; q++) A[i][q] = R[i][q];
            } else {
                xor16(A[i], R[i]);
            }
        }
        // the fourth accumulator row lives in this wave's private LDS row
        if (C == 0) {
            lds_put(lbase, 32 + w, R[3]);
        } else {
            lds_get(lbase, 32 + w, R[0]);
            xor16(R[0], R[3]);
            lds_put(lbase, 32 + w, R[0]);
        }
        __builtin_amdgcn_sched_barrier(0);
    }

    template <int... Cs>
    __device__ __forceinline__ void chunks(int tile, std::integer_sequence<int, Cs...>) {
        (chunk<Cs>(tile), ...);
    }

    __device__ __forceinline__ void run() {
#if RS_BS_STAMP
        const unsigned long long t_start = __builtin_amdgcn_s_memtime();
#endif
        int tile = blockIdx.x;
        stage(tile, 0);
        for (; tile < a.ntiles; tile += gridDim.x) {
            chunks(tile, std::make_integer_sequence<int, NCH>{});
#if RS_BS_STAMP
            const unsigned long long t_f0 = __builtin_amdgcn_s_memtime();
#endif
            // FFT pass A: rows w + 8i (dist 16 then 8; the only group: slots 0..2)
#pragma unroll
            for (int i = 0; i < 3; i++)
#pragma unroll
                for (int q = 0; q < 16; q++) R[i][q] = A[i][q];
            lds_get(lbase, 32 + w, R[3]);
            bs_fft4<TW, 0>(R);
            bar();
#pragma unroll
            for (int i = 0; i < 4; i++) lds_put(lbase, w + 8 * i, R[i]);
            bar();
            // pass B: rows 8g + j + 2i (dist 4 then 2; group g, slots 3 + 3g ..)
            const int g = w >> 1, j = w & 1;
#pragma unroll
            for (int i = 0; i < 4; i++) lds_get(lbase, 8 * g + j + 2 * i, R[i]);
            dispatch<4>(g, [&](auto G) { bs_fft4<TW, 3 + 3 * decltype(G)::value>(R); });
#pragma unroll
            for (int i = 0; i < 4; i++) lds_put(lbase, 8 * g + j + 2 * i, R[i]);
            bar();
            // pass C: rows 4w + i, radix-2 at dist 1 (slots 15 + 2w, 16 + 2w)
#pragma unroll
            for (int i = 0; i < 4; i++) lds_get(lbase, 4 * w + i, R[i]);
            dispatch<8>(w, [&](auto W) {
                constexpr int s = 15 + 2 * decltype(W)::value;
                bs_fft2<TW, s>(R[0], R[1]);
                bs_fft2<TW, s + 1>(R[2], R[3]);
            });
            // parity rows 4w + i < p
            const int tps = a.tiles_per_stripe;
            const int stripe = tile / tps, ct = tile - stripe * tps;
            const uint64_t col = (uint64_t)ct * 4096 + (uint64_t)lane * 64;
            uint32_t bad = 0;
            if (col < a.S) {
                uint8_t *base = a.parity + (uint64_t)stripe * a.stripe_stride + col;
#pragma unroll
                for (int i = 0; i < 4; i++) {
                    const int row = 4 * w + i;
                    if (row >= a.p) continue;
                    if constexpr (TW::SUB) bs_psi<TW>(R[i]);
                    bs_transpose(R[i]);
#ifdef RS_BS_ABL_COALESCED
                    g_u4 *q = (g_u4 *)(base - (uint64_t)lane * 64 + (uint64_t)row * a.row_stride + lane * 16);
#else
                    g_u4 *q = (g_u4 *)(base + (uint64_t)row * a.row_stride);
#endif
#pragma unroll
                    for (int k = 0; k < 4; k++) {
#ifdef RS_BS_ABL_COALESCED
                        const int kq = k * 64;  // 1 KB apart
#else
                        const int kq = k;
#endif
                        const u32x4 v = u32x4{R[i][4 * k], R[i][4 * k + 1], R[i][4 * k + 2], R[i][4 * k + 3]};
                        if constexpr (VERIFY) {
                            const u32x4 o = q[kq];
                            bad |= (o[0] ^ v[0]) | (o[1] ^ v[1]) | (o[2] ^ v[2]) | (o[3] ^ v[3]);
                        } else {
#ifdef RS_BS_NT_STORE
                            __builtin_nontemporal_store(v, q + kq);
#else
                            q[kq] = v;
#endif
                        }
                    }
                }
            }
#if RS_BS_STAMP
            t_fft += __builtin_amdgcn_s_memtime() - t_f0;
#endif
            if constexpr (VERIFY) {
                // one store per wave, not per lane
                const uint64_t m = __ballot(bad != 0);
                if (m && lane == __ffsll((unsigned long long)m) - 1)
                    __hip_atomic_store(a.mismatch, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
#if RS_BS_STAMP
        t_total = __builtin_amdgcn_s_memtime() - t_start;
#endif
    }
};

template <class TW, bool VERIFY>
__global__ void __launch_bounds__(512, 2) k_encode_bs(BsArgs a) {
    // 32 image rows + 8 per-wave accumulator rows, each 64 blocks x 16 planes (160 KB)
    __shared__ __attribute__((aligned(16))) uint32_t lds[40 * 1024];
    BsEncoder<TW, VERIFY> e{a};
    e.lane = threadIdx.x & 63;
    e.w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    e.lbase = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) uint32_t *)lds + e.lane * 16;
    e.run();
#if RS_BS_STAMP
    if (e.lane == 0 && blockIdx.x < 1024) {
        unsigned long long *o = g_bs_stamps + (blockIdx.x * 8 + e.w) * 4;
        o[0] = e.t_load;
        o[1] = e.t_bar;
        o[2] = e.t_fft;
        o[3] = e.t_total;
    }
#endif
}

// ============================================================================
// Half-plane encode (k_encode_hp): subfield geometries (TW::SUB), two
// independent 256-thread workgroups per CU.
//
// In subfield coordinates every twiddle acts as the same 8x8 GF(2) map on
// both byte halves, so a lane can hold one half (8 bit-planes) of a 64-byte
// block, and the half becomes a lane bit.  A workgroup owns a 2 KB tile (32
// blocks) of every row of one stripe; lane l = (block l & 31, half l >> 5) in
// every wave, 4 waves.  The only lane-varying quantities are the block and the
// half, so every twiddle is wave-uniform:
//
//   chunk IFFT layers r0, r1, r2 (dist 1, 2, 4; leopard16.go:694-741): wave w
//     holds rows 8w + j (j = 0..7) of its half.  Their twiddles depend on the
//     row bits above the layer (r3, r4 = w), so the wave's role is w.
//   -> one LDS exchange (64 KB image: row x plane quad x lane) ->
//   chunk IFFT layers r3, r4 (dist 8, 16): wave w holds the cosets
//     co = 2w + u (u = 0, 1; row bits r0..r2) of rows co + 8t; twiddles
//     depend only on r4 (a register index), so every wave runs the same code.
//     XOR-accumulate into A (same layout, 64 VGPRs).
//   final FFT layers r4, r3 (fftDIT leopard16.go:618-657) in A's layout,
//   -> one exchange -> layers r2, r1, r0 on rows 8w + j, store.
//
// Loads/stores need whole 64-byte blocks (the bit-plane transpose and the
// coordinate change mix both halves): lane (b, h) loads rows 8w + 4h + i
// (i = 0..3) of block b, transposes them, and one v_permlane32_swap per plane
// pair moves the other half of each row to the partner lane (l ^ 32).
//
// One exchange per chunk (5 per tile), two barriers each, over 4 waves; the
// second workgroup on the CU computes while this one waits.  Registers: 64
// staged (next chunk, in flight) + 64 working + 64 accumulator.
typedef uint32_t Half[8];
#ifndef RS_HP_LOAD_AUX
#define RS_HP_LOAD_AUX 0     // cache policy of the data loads (2 = nt)
#endif

// out ^= XOR of y[j] over the set bits j of mask (3-input XOR pairs).
__device__ __forceinline__ void xor_net8(uint32_t &out, const Half &y, uint32_t mask) {
    int pend = -1;
#pragma unroll
    for (int j = 0; j < 8; j++) {
        if ((mask >> j) & 1) {
            if (pend < 0) {
                pend = j;
            } else {
                ixor3(out, y[pend], y[j]);
                pend = -1;
            }
        }
    }
    if (pend >= 0) ixor(out, y[pend]);
}
__device__ __forceinline__ void xor8(Half &y, const Half &x) {
#pragma unroll
    for (int i = 0; i < 8; i++) ixor(y[i], x[i]);
}
// x ^= y * twiddle (C >= 0: chunk C's IFFT slot; C < 0: FFT slot)
template <class TW, int C, int SLOT>
__device__ __forceinline__ void hp_mul_add(Half &x, const Half &y) {
#ifdef RS_BS_ABL_NOMUL
    return;
#endif
#pragma unroll
    for (int i = 0; i < 8; i++) xor_net8(x[i], y, C < 0 ? TW::fft8[SLOT][i] : TW::ifft8[C < 0 ? 0 : C][SLOT][i]);
}
template <class TW, int C, int SLOT>
__device__ __forceinline__ void hp_ifft2(Half &x, Half &y) {
    xor8(y, x);
    hp_mul_add<TW, C, SLOT>(x, y);
    __builtin_amdgcn_sched_barrier(0);
}
template <class TW, int SLOT>
__device__ __forceinline__ void hp_fft2(Half &x, Half &y) {
    hp_mul_add<TW, -1, SLOT>(x, y);
    xor8(y, x);
    __builtin_amdgcn_sched_barrier(0);
}
// One byte half of bs_transpose (8 dwords <-> 8 planes).
__device__ __forceinline__ void bs_transpose8(Half &w) {
#ifdef RS_BS_ABL_NOTRANS
    return;
#endif
#pragma unroll
    for (int k = 0; k < 3; k++) {
        const int s = 1 << k;
        const uint32_t M = k == 0 ? 0x55555555u : k == 1 ? 0x33333333u : 0x0F0F0F0Fu;
#pragma unroll
        for (int a = 0; a < 8; a++)
            if (!(a & s)) bs_xchg(w[a], w[a + s], s, M);
    }
}
// Subfield coordinates of a whole row held as (lo planes, hi planes).
template <class TW>
__device__ __forceinline__ void hp_psi(Half &lo, const Half &hi) {
#pragma unroll
    for (int r = 0; r < 8; r++) xor_net8(lo[r], hi, TW::dmat[r]);
}
// Rows i (lanes 0-31: lo half, lanes 32-63: hi half) <-> full rows: R[i] / R[4+i]
// hold the lo / hi planes of full row i on each lane, or the half rows i and
// 4 + i after the swap (an involution).
// In-place inline asm: the builtin's two results land in fresh registers, and
// 32 swaps in flight at once cost the kernel 64 VGPRs.  s_nop 1: two wait
// states between a VALU write of an operand and the swap that reads it.
__device__ __forceinline__ void hp_swap_halves(Half (&R)[8]) {
#pragma unroll
    for (int i = 0; i < 4; i++) {
        asm volatile(
            "s_nop 1\n\t"
            "v_permlane32_swap_b32 %0, %8\n\tv_permlane32_swap_b32 %1, %9\n\t"
            "v_permlane32_swap_b32 %2, %10\n\tv_permlane32_swap_b32 %3, %11\n\t"
            "v_permlane32_swap_b32 %4, %12\n\tv_permlane32_swap_b32 %5, %13\n\t"
            "v_permlane32_swap_b32 %6, %14\n\tv_permlane32_swap_b32 %7, %15"
            : "+v"(R[i][0]), "+v"(R[i][1]), "+v"(R[i][2]), "+v"(R[i][3]), "+v"(R[i][4]), "+v"(R[i][5]),
              "+v"(R[i][6]), "+v"(R[i][7]), "+v"(R[4 + i][0]), "+v"(R[4 + i][1]), "+v"(R[4 + i][2]),
              "+v"(R[4 + i][3]), "+v"(R[4 + i][4]), "+v"(R[4 + i][5]), "+v"(R[4 + i][6]), "+v"(R[4 + i][7]));
    }
}

// LDS image of the half-plane kernel: row r, plane quad qh of lane l at byte
// r * 2048 + qh * 1024 + l * 16 (every ds_*_b128 wave access is 1 KB contiguous).
__device__ __forceinline__ uint32_t hp_row_addr(uint32_t lbase, int row) {
    uint32_t b = lbase;
    asm volatile("" : "+v"(b));
    return b + (uint32_t)row * 2048u;
}
__device__ __forceinline__ void hp_put(uint32_t lbase, int row, const Half &v) {
#ifdef RS_BS_ABL_NOLDS
    return;
#endif
    const uint32_t ra = hp_row_addr(lbase, row);
    *(lds_u4 *)(uintptr_t)ra = u32x4{v[0], v[1], v[2], v[3]};
    *(lds_u4 *)(uintptr_t)(ra + 1024) = u32x4{v[4], v[5], v[6], v[7]};
}
__device__ __forceinline__ void hp_get(uint32_t lbase, int row, Half &v) {
#ifdef RS_BS_ABL_NOLDS
#pragma unroll
    for (int q = 0; q < 8; q++) asm volatile("" : "+v"(v[q]));
    return;
#endif
    const uint32_t ra = hp_row_addr(lbase, row);
    const u32x4 x = *(const lds_u4 *)(uintptr_t)ra;
    const u32x4 y = *(const lds_u4 *)(uintptr_t)(ra + 1024);
    v[0] = x[0], v[1] = x[1], v[2] = x[2], v[3] = x[3];
    v[4] = y[0], v[5] = y[1], v[6] = y[2], v[7] = y[3];
}

template <class TW, bool VERIFY>
struct HpEncoder {
    static_assert(TW::SUB, "the half-plane kernel needs every twiddle in the GF(2^8) subfield");
    static constexpr int NCH = TW::NCH;
    static constexpr int TILE = 2048;  // column bytes per tile (32 blocks)
    const BsArgs &a;
    uint32_t lbase;  // this lane's LDS byte address of row 0, quad 0
    int lane, w, h, blk;
    Half St[8];  // staged full rows i: St[i] = dwords 0-7 (low bytes), St[4+i] = dwords 8-15
    Half R[8];   // working rows
    Half A[8];   // accumulator: coset u = 0, 1 (co = 2w + u), rows co + 8t at A[4u + t]

    __device__ __forceinline__ void bar() { lds_barrier(); }

    // Load rows 32c + 8w + 4h + i of `tile` through a buffer descriptor over
    // the stripe's data rows: rows past k and bytes past the last row's end
    // read as zero (range check), a tile past the end has an empty range.
    // Lanes whose block lies past the row end read bytes of the next row;
    // their results are never stored.
    template <int I0, int I1>
    __device__ __forceinline__ void stage(int tile, int c) {
        const int tps = a.tiles_per_stripe;
        const int stripe = tile / tps, ct = tile - stripe * tps;
        const bool live = tile < a.ntiles;
#ifdef RS_BS_ABL_NOLOAD
        const uint32_t range = 0;
#else
        const uint32_t range = live ? a.span : 0u;
#endif
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            (void *)(a.data + (live ? (uint64_t)stripe * a.stripe_stride : 0)), 0, (int)range, 0x00020000);
        // lane part of the offset (block, half); opaque so that the compiler
        // does not precompute every chunk's offsets
        uint32_t voff = (uint32_t)ct * TILE + (uint32_t)blk * 64 + (uint32_t)(4 * h) * (uint32_t)a.row_stride;
        asm volatile("" : "+v"(voff));
#pragma unroll
        for (int i = I0; i < I1; i++) {
            // wave-uniform row of the h = 0 lanes (rows >= k are out of range: zeros)
            const uint32_t soff = (uint32_t)(32 * c + 8 * w + i) * (uint32_t)a.row_stride;
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const u32x4 x = __builtin_amdgcn_raw_buffer_load_b128(rs, voff + q * 16, soff, 0);
                uint32_t *d = q < 2 ? &St[i][q * 4] : &St[4 + i][(q - 2) * 4];
                d[0] = x[0], d[1] = x[1], d[2] = x[2], d[3] = x[3];
            }
        }
    }

    // IFFT layers r0, r1, r2 on rows 8W + j (pass-0 slots 3g.., g = 2W + j/4;
    // pass-1 slot 24 + 3 r4 + 2 r3 for layer r2).
    template <int C, int W>
    __device__ __forceinline__ void phase1() {
        hp_ifft2<TW, C, 3 * (2 * W)>(R[0], R[1]);
        hp_ifft2<TW, C, 3 * (2 * W) + 2>(R[2], R[3]);
        hp_ifft2<TW, C, 3 * (2 * W + 1)>(R[4], R[5]);
        hp_ifft2<TW, C, 3 * (2 * W + 1) + 2>(R[6], R[7]);
        hp_ifft2<TW, C, 3 * (2 * W) + 1>(R[0], R[2]);
        hp_ifft2<TW, C, 3 * (2 * W) + 1>(R[1], R[3]);
        hp_ifft2<TW, C, 3 * (2 * W + 1) + 1>(R[4], R[6]);
        hp_ifft2<TW, C, 3 * (2 * W + 1) + 1>(R[5], R[7]);
        constexpr int s2 = 24 + 3 * (W >> 1) + ((W & 1) ? 2 : 0);
        hp_ifft2<TW, C, s2>(R[0], R[4]);
        hp_ifft2<TW, C, s2>(R[1], R[5]);
        hp_ifft2<TW, C, s2>(R[2], R[6]);
        hp_ifft2<TW, C, s2>(R[3], R[7]);
    }

    // Next chunk's rows i in [I0, I1): chunk C + 1 of this tile, or chunk 0 of the next tile.
    template <int C, int I0, int I1>
    __device__ __forceinline__ void prefetch(int tile) {
        if (C + 1 < NCH) stage<I0, I1>(tile, C + 1);
        else stage<I0, I1>(tile + (int)gridDim.x, 0);
    }

    // The next chunk's loads go out in two halves so that at most 160 of the
    // 256 VGPRs hold data (A 64 + R 64 + half of St during the transposes and
    // layers r0-r2; A 64 + St 64 + one coset's 32 during layers r3-r4): rows
    // i = 0, 1 once the staged rows are transposed, rows 2, 3 once the
    // phase-1 rows are in the LDS image.  (Issuing all of them at the chunk
    // start, with 192 VGPRs of data live, spilled to scratch: +8 % HBM traffic.)
    template <int C>
    __device__ __forceinline__ void chunk(int tile) {
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < 8; i++)
#pragma unroll
            for (int q = 0; q < 8; q++) R[i][q] = St[i][q];
#pragma unroll
        for (int i = 0; i < 4; i++) {
            bs_transpose8(R[i]);
            bs_transpose8(R[4 + i]);
            hp_psi<TW>(R[i], R[4 + i]);
        }
        hp_swap_halves(R);
        // consume the staged rows before their registers are reloaded
#pragma unroll
        for (int i = 0; i < 8; i++)
#pragma unroll
            for (int q = 0; q < 8; q++) asm volatile("" : "+v"(R[i][q])::"memory");
        __builtin_amdgcn_sched_barrier(0);
        prefetch<C, 0, 2>(tile);
        __builtin_amdgcn_sched_barrier(0);
        dispatch<4>(w, [&](auto W) { phase1<C, decltype(W)::value>(); });
        bar();  // every wave has read the previous image
#pragma unroll
        for (int j = 0; j < 8; j++) hp_put(lbase, 8 * w + j, R[j]);
        bar();
        prefetch<C, 2, 4>(tile);
        __builtin_amdgcn_sched_barrier(0);
        // IFFT layers r3 (pass-1 m02: slot 25 for r4 = 0, 28 for r4 = 1) and r4
        // (slot 30), one coset u (rows 2w + u + 8t) at a time
#pragma unroll
        for (int u = 0; u < 2; u++) {
#pragma unroll
            for (int t = 0; t < 4; t++) hp_get(lbase, 2 * w + u + 8 * t, R[t]);
            hp_ifft2<TW, C, 25>(R[0], R[1]);
            hp_ifft2<TW, C, 28>(R[2], R[3]);
            hp_ifft2<TW, C, 30>(R[0], R[2]);
            hp_ifft2<TW, C, 30>(R[1], R[3]);
#pragma unroll
            for (int t = 0; t < 4; t++) {
                if (C == 0) {
#pragma unroll
                    for (int q = 0; q < 8; q++) A[4 * u + t][q] = R[t][q];
                } else {
                    xor8(A[4 * u + t], R[t]);
                }
            }
            __builtin_amdgcn_sched_barrier(0);
        }
    }

    template <int... Cs>
    __device__ __forceinline__ void chunks(int tile, std::integer_sequence<int, Cs...>) {
        (chunk<Cs>(tile), ...);
    }

    // FFT layers r2 (pass-1 m02), r1 (pass-1 m01/m23), r0 (pass-2 slot 15 + r/2) on rows 8W + j.
    template <int W>
    __device__ __forceinline__ void fft_b() {
        constexpr int s0 = 3 + 3 * W;
        hp_fft2<TW, s0 + 1>(R[0], R[4]);
        hp_fft2<TW, s0 + 1>(R[1], R[5]);
        hp_fft2<TW, s0 + 1>(R[2], R[6]);
        hp_fft2<TW, s0 + 1>(R[3], R[7]);
        hp_fft2<TW, s0>(R[0], R[2]);
        hp_fft2<TW, s0>(R[1], R[3]);
        hp_fft2<TW, s0 + 2>(R[4], R[6]);
        hp_fft2<TW, s0 + 2>(R[5], R[7]);
        hp_fft2<TW, 15 + 4 * W>(R[0], R[1]);
        hp_fft2<TW, 16 + 4 * W>(R[2], R[3]);
        hp_fft2<TW, 17 + 4 * W>(R[4], R[5]);
        hp_fft2<TW, 18 + 4 * W>(R[6], R[7]);
    }

    __device__ __forceinline__ void run() {
        int tile = blockIdx.x;
        stage<0, 4>(tile, 0);
        for (; tile < a.ntiles; tile += gridDim.x) {
            chunks(tile, std::make_integer_sequence<int, NCH>{});
            // FFT layers r4 (pass-0 m02, slot 1) and r3 (slot 0 for r4 = 0, 2 for r4 = 1) in A's layout
#pragma unroll
            for (int u = 0; u < 2; u++) {
                hp_fft2<TW, 1>(A[4 * u], A[4 * u + 2]);
                hp_fft2<TW, 1>(A[4 * u + 1], A[4 * u + 3]);
                hp_fft2<TW, 0>(A[4 * u], A[4 * u + 1]);
                hp_fft2<TW, 2>(A[4 * u + 2], A[4 * u + 3]);
            }
            bar();
#pragma unroll
            for (int u = 0; u < 2; u++)
#pragma unroll
                for (int t = 0; t < 4; t++) hp_put(lbase, 2 * w + u + 8 * t, A[4 * u + t]);
            bar();
#pragma unroll
            for (int j = 0; j < 8; j++) hp_get(lbase, 8 * w + j, R[j]);
            dispatch<4>(w, [&](auto W) { fft_b<decltype(W)::value>(); });
            hp_swap_halves(R);
            // parity rows 8w + 4h + i < p, through a descriptor over the stripe's
            // parity rows (lanes past the row end store nothing: exec mask)
            const int tps = a.tiles_per_stripe;
            const int stripe = tile / tps, ct = tile - stripe * tps;
            const uint32_t col = (uint32_t)ct * TILE + (uint32_t)blk * 64;
            const __amdgpu_buffer_rsrc_t ps = __builtin_amdgcn_make_buffer_rsrc(
                (void *)(a.parity + (uint64_t)stripe * a.stripe_stride), 0, (int)a.pspan, 0x00020000);
            uint32_t voff = col + (uint32_t)(4 * h) * (uint32_t)a.row_stride;
            asm volatile("" : "+v"(voff));
            uint32_t bad = 0;
            if (col < a.S) {
#pragma unroll
                for (int i = 0; i < 4; i++) {
                    const int row = 8 * w + 4 * h + i;
                    if (row >= TW::P) continue;
                    hp_psi<TW>(R[i], R[4 + i]);
                    bs_transpose8(R[i]);
                    bs_transpose8(R[4 + i]);
                    const uint32_t soff = (uint32_t)(8 * w + i) * (uint32_t)a.row_stride;
#pragma unroll
                    for (int k = 0; k < 4; k++) {
                        const int o = (k & 1) * 4;
                        const u32x4 v = k < 2 ? u32x4{R[i][o], R[i][o + 1], R[i][o + 2], R[i][o + 3]}
                                              : u32x4{R[4 + i][o], R[4 + i][o + 1], R[4 + i][o + 2], R[4 + i][o + 3]};
                        if constexpr (VERIFY) {
                            const u32x4 old = __builtin_amdgcn_raw_buffer_load_b128(ps, voff + k * 16, soff, 0);
                            bad |= (old[0] ^ v[0]) | (old[1] ^ v[1]) | (old[2] ^ v[2]) | (old[3] ^ v[3]);
                        } else {
#if defined(RS_BS_ABL_NOSTORE)
                            asm volatile("" ::"v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]));
#elif defined(RS_BS_NT_STORE)
                            __builtin_amdgcn_raw_buffer_store_b128(v, ps, voff + k * 16, soff, 2);
#else
                            __builtin_amdgcn_raw_buffer_store_b128(v, ps, voff + k * 16, soff, 0);
#endif
                        }
                    }
                }
            }
            if constexpr (VERIFY) {
                const uint64_t m = __ballot(bad != 0);
                if (m && lane == __ffsll((unsigned long long)m) - 1)
                    __hip_atomic_store(a.mismatch, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
    }
};

template <class TW, bool VERIFY>
__global__ void __launch_bounds__(256, 2) k_encode_hp(BsArgs a) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[16 * 1024];  // 32 rows x 2 KB
    HpEncoder<TW, VERIFY> e{a};
    e.lane = threadIdx.x & 63;
    e.w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    e.h = e.lane >> 5;
    e.blk = e.lane & 31;
    e.lbase = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) uint32_t *)lds + e.lane * 16;
    e.run();
}

// RS_BS_KERNEL=1 selects the round-1 512-thread kernel for subfield
// geometries too (A/B experiments only).
bool hp_enabled() {
    const char *e = getenv("RS_BS_KERNEL");
    return !(e && e[0] == '1');
}

template <class TW>
hipError_t launch_bs_t(bool verify, BsArgs a, int cus, hipStream_t s) {
    if constexpr (TW::SUB) {
        // buffer offsets are 32-bit: the data rows of one stripe must span < 4 GiB
        if (hp_enabled() && (uint64_t)(a.k - 1) * a.row_stride + a.S < (1ull << 32)) {
            a.tiles_per_stripe = (int)((a.S + 2047) / 2048);
            a.ntiles = a.tiles_per_stripe * a.nstripes;
            a.span = (uint32_t)((uint64_t)(a.k - 1) * a.row_stride + a.S);
            a.pspan = (uint32_t)((uint64_t)(a.p - 1) * a.row_stride + a.S);
            const int grid = std::min(a.ntiles, 2 * cus);
            if (verify) hipLaunchKernelGGL((k_encode_hp<TW, true>), dim3(grid), dim3(256), 0, s, a);
            else hipLaunchKernelGGL((k_encode_hp<TW, false>), dim3(grid), dim3(256), 0, s, a);
            return hipGetLastError();
        }
    }
    a.tiles_per_stripe = (int)((a.S + 4095) / 4096);
    a.ntiles = a.tiles_per_stripe * a.nstripes;
    const int grid = std::min(a.ntiles, cus);
    if (verify) hipLaunchKernelGGL((k_encode_bs<TW, true>), dim3(grid), dim3(512), 0, s, a);
    else hipLaunchKernelGGL((k_encode_bs<TW, false>), dim3(grid), dim3(512), 0, s, a);
    return hipGetLastError();
}

}  // namespace

bool encode_bs_available(int k, int p) {
#define RS_BS_HAS(K, P) \
    if (k == K && p == P) return true;
    RS_BS_CONFIGS(RS_BS_HAS)
#undef RS_BS_HAS
    return false;
}

hipError_t launch_encode_bs(bool verify, const BsArgs &a, int cus, hipStream_t s) {
#define RS_BS_LAUNCH(K, P) \
    if (a.k == K && a.p == P) return launch_bs_t<BsTw<K, P>>(verify, a, cus, s);
    RS_BS_CONFIGS(RS_BS_LAUNCH)
#undef RS_BS_LAUNCH
    return hipErrorNotSupported;
}

#if RS_BS_STAMP
extern "C" int rs_debug_bs_stamps(unsigned long long *out, size_t n) {
    return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_bs_stamps), n * sizeof(unsigned long long));
}
#endif

}  // namespace rs
