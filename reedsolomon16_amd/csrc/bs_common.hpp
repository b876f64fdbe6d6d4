// Bit-plane helpers shared by the bit-sliced kernels (csrc/bitslice.hip:
// encode; csrc/bitslice_dec.hip: the n = 256 decode).  A 32-bit word holds
// one bit of 32 symbols (a bit-plane); a multiply by a known GF(2^8)
// subfield constant is a fixed XOR network over 8 planes.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <utility>

namespace rs {
namespace bs {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) u32x4 lds_u4;
typedef uint32_t Half[8];

// ---- compile-time loops ----
template <int V> using ic = std::integral_constant<int, V>;
template <class Fn, int... Is>
__device__ __forceinline__ void sfor_impl(Fn &&f, std::integer_sequence<int, Is...>) {
    (f(ic<Is>{}), ...);
}
template <int N, class Fn>
__device__ __forceinline__ void sfor(Fn &&f) {
    sfor_impl(f, std::make_integer_sequence<int, N>{});
}
// Wave-uniform dispatch of a role-specialized pass: f(ic<R>) for R = role.
template <class Fn, int... Is>
__device__ __forceinline__ void dispatch_impl(int role, Fn &&f, std::integer_sequence<int, Is...>) {
    ((role == Is ? (f(ic<Is>{}), 0) : 0), ...);
}
template <int N, class Fn>
__device__ __forceinline__ void dispatch(int role, Fn &&f) {
    dispatch_impl(role, f, std::make_integer_sequence<int, N>{});
}

// ---- bit-plane arithmetic ----
// v ^= a  /  v ^= a ^ b, in place (v_bitop3_b32 truth table 0x96 = 3-input XOR).
__device__ __forceinline__ void ixor(uint32_t &v, uint32_t a) { asm("v_xor_b32 %0, %1, %0" : "+v"(v) : "v"(a)); }
__device__ __forceinline__ void ixor3(uint32_t &v, uint32_t a, uint32_t b) {
    asm("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(v) : "v"(a), "v"(b));
}
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
// The same with a compile-time mask (the pairing is resolved in the
// front end: no runtime value ever selects a register).
template <uint32_t MASK, int J = 0, int PEND = -1>
__device__ __forceinline__ void xor_net8c(uint32_t &out, const Half &y) {
    if constexpr (J == 8) {
        if constexpr (PEND >= 0) ixor(out, y[PEND]);
    } else if constexpr (!((MASK >> J) & 1)) {
        xor_net8c<MASK, J + 1, PEND>(out, y);
    } else if constexpr (PEND < 0) {
        xor_net8c<MASK, J + 1, J>(out, y);
    } else {
        ixor3(out, y[PEND], y[J]);
        xor_net8c<MASK, J + 1, -1>(out, y);
    }
}
// out = in ^ XOR of y[j] over the set bits j of MASK: the first operation
// writes a fresh register (no tied operand), the rest go in place.
template <uint32_t MASK, int J = 0, int PEND = -1, bool FRESH = true>
__device__ __forceinline__ void xor_net8f(uint32_t &out, uint32_t in, const Half &y) {
    if constexpr (J == 8) {
        if constexpr (PEND >= 0) {
            if constexpr (FRESH) asm("v_xor_b32 %0, %1, %2" : "=v"(out) : "v"(y[PEND]), "v"(in));
            else ixor(out, y[PEND]);
        } else if constexpr (FRESH) {
            out = in;
        }
    } else if constexpr (!((MASK >> J) & 1)) {
        xor_net8f<MASK, J + 1, PEND, FRESH>(out, in, y);
    } else if constexpr (PEND < 0) {
        xor_net8f<MASK, J + 1, J, FRESH>(out, in, y);
    } else if constexpr (FRESH) {
        asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(out) : "v"(in), "v"(y[PEND]), "v"(y[J]));
        xor_net8f<MASK, J + 1, -1, false>(out, in, y);
    } else {
        ixor3(out, y[PEND], y[J]);
        xor_net8f<MASK, J + 1, -1, false>(out, in, y);
    }
}
__device__ __forceinline__ void xor8(Half &y, const Half &x) {
#pragma unroll
    for (int i = 0; i < 8; i++) ixor(y[i], x[i]);
}
// Delta swap of word-index bit k with bit-position bit k (s = 2^k, M = positions with bit k clear).
__device__ __forceinline__ void bs_xchg(uint32_t &a, uint32_t &b, int s, uint32_t M) {
    const uint32_t as = a >> s, bsh = b << s;
    a = (a & M) | (bsh & ~M);
    b = (b & ~M) | (as & M);
}
// One byte half of a 64-byte block (8 dwords: byte j of dword w = that byte
// of symbol 4w + j) <-> 8 bit-planes (plane b bit 8j + w = bit b of symbol
// 4w + j).  Three delta-swap stages; an involution.
__device__ __forceinline__ void bs_transpose8(Half &w) {
#pragma unroll
    for (int k = 0; k < 3; k++) {
        const int s = 1 << k;
        const uint32_t M = k == 0 ? 0x55555555u : k == 1 ? 0x33333333u : 0x0F0F0F0Fu;
#pragma unroll
        for (int a = 0; a < 8; a++)
            if (!(a & s)) bs_xchg(w[a], w[a + s], s, M);
    }
}

// In-place lane-half swaps (gfx950).  permlane32: lane l < 32 of b trades with
// lane l + 32 of a (a's upper half <-> b's lower half); permlane16: the same
// between 16-lane rows (a's rows 1, 3 <-> b's rows 0, 2).  s_nop 1: two wait
// states between a VALU write of an operand and the swap that reads it.
__device__ __forceinline__ void swap32(uint32_t &a, uint32_t &b) {
    asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1" : "+v"(a), "+v"(b));
}
__device__ __forceinline__ void swap16(uint32_t &a, uint32_t &b) {
    asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1" : "+v"(a), "+v"(b));
}
// Workgroup barrier for LDS traffic only (global loads stay in flight).
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }


// ---- byte form: products by runtime twiddles with v_perm_b32 tables held in SGPRs
// Tables, shard maps and row pointers are read through the constant address
// space: read-only for the launch, so wave-uniform addresses become scalar loads.
typedef __attribute__((address_space(4))) const uint32_t cu32_t;
__device__ __forceinline__ cu32_t *ctab(const uint32_t *t) { return (cu32_t *)t; }

__device__ __forceinline__ uint32_t perm(uint32_t s0, uint32_t s1, uint32_t sel) {
    return __builtin_amdgcn_perm(s0, s1, sel);
}
__device__ __forceinline__ uint32_t xor3v(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// A table's leading dwords held in SGPRs (loaded one row ahead of its use).
template <int N>
struct Tab {
    uint32_t v[N];
    __device__ __forceinline__ uint32_t operator[](int i) const { return v[i]; }
};
// Tab<N> of the table at p; p passes an empty volatile asm first, which fixes
// where (in the sequence of volatile steps) the loads are issued.
template <int N>
__device__ __forceinline__ Tab<N> tab_at(cu32_t *p) {
    asm volatile("" : "+s"(p));
    Tab<N> t;
#pragma unroll
    for (int i = 0; i < N; i++) t.v[i] = p[i];
    return t;
}

// x = y * table (full-field table, make_twiddle / make_linear_image layout).
template <class T>
__device__ __forceinline__ void mul16(uint32_t (&x)[4], const uint32_t (&y)[4], const T &t) {
#pragma unroll
    for (int d = 0; d < 2; d++) {
        const uint32_t lo = y[d], hi = y[2 + d];
        const uint32_t a0 = lo & 0x07070707u, a1 = (lo >> 3) & 0x07070707u, a2 = (lo >> 6) & 0x03030303u;
        const uint32_t b0 = hi & 0x07070707u, b1 = (hi >> 3) & 0x07070707u, b2 = (hi >> 6) & 0x03030303u;
        x[d] = xor3v(xor3v(perm(t[1], t[0], a0), perm(t[5], t[4], a1), perm(t[8], t[8], a2)), perm(t[11], t[10], b0),
                     perm(t[15], t[14], b1)) ^ perm(t[18], t[18], b2);
        x[2 + d] = xor3v(xor3v(perm(t[3], t[2], a0), perm(t[7], t[6], a1), perm(t[9], t[9], a2)), perm(t[13], t[12], b0),
                         perm(t[17], t[16], b1)) ^ perm(t[19], t[19], b2);
    }
}
// x ^= y * table (subfield table, make_sub_twiddle layout: the same byte map on c0 and c1;
// a zero twiddle's table is all zero).
template <class T>
__device__ __forceinline__ void mul8_add(uint32_t *x, const uint32_t *y, const T &t) {
#pragma unroll
    for (int d = 0; d < 4; d++) {
        const uint32_t v = y[d];
        x[d] = xor3v(x[d] ^ perm(t[1], t[0], v & 0x07070707u), perm(t[3], t[2], (v >> 3) & 0x07070707u),
                     perm(t[4], t[4], (v >> 6) & 0x03030303u));
    }
}

// x ^= y * table for one (lo, hi) dword pair: 4 symbols (full-field table)
template <class T>
__device__ __forceinline__ void mul16_add1(uint32_t &xl, uint32_t &xh, uint32_t lo, uint32_t hi, const T &t) {
    const uint32_t a0 = lo & 0x07070707u, a1 = (lo >> 3) & 0x07070707u, a2 = (lo >> 6) & 0x03030303u;
    const uint32_t b0 = hi & 0x07070707u, b1 = (hi >> 3) & 0x07070707u, b2 = (hi >> 6) & 0x03030303u;
    xl = xor3v(xor3v(xl, perm(t[1], t[0], a0), perm(t[5], t[4], a1)), xor3v(perm(t[8], t[8], a2), perm(t[11], t[10], b0),
                                                                      perm(t[15], t[14], b1)), perm(t[18], t[18], b2));
    xh = xor3v(xor3v(xh, perm(t[3], t[2], a0), perm(t[7], t[6], a1)), xor3v(perm(t[9], t[9], a2), perm(t[13], t[12], b0),
                                                                      perm(t[17], t[16], b1)), perm(t[19], t[19], b2));
}

}  // namespace bs
}  // namespace rs
