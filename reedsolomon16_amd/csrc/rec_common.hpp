// Revealed-row mask helpers shared by the reconstruct kernels
// (kernels.hip k_rec_lds, bitslice_dec.hip k_rec_bs256).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace rs {
namespace rec {

// Rows [lo, lo + cnt) (cnt a power of two, lo a multiple of cnt) hold a set
// bit of the 256-bit row mask (wave-uniform words, lane-varying lo).  Passed
// by value (Need / NoNeed) so that the words stay in registers: a pointer to
// a local array through the pass functors left it on the stack (32 B of
// scratch stores per lane: +67 MB of HBM writes per C4 launch).
struct Need {
    uint32_t w[8];
};
struct NoNeed {};
__device__ __forceinline__ bool rows_needed(const Need &n, int lo, int cnt) {
    if (cnt >= 32) {
        uint32_t acc = 0;
#pragma unroll
        for (int k = 0; k < 8; k++)
            if (k * 32 >= lo && k * 32 < lo + cnt) acc |= n.w[k];
        return acc != 0;
    }
    // a select chain; the opaque step keeps the compiler from turning it into
    // a lane-indexed load of the words spilled to a stack array
    const int idx = lo >> 5;
    uint32_t word = n.w[0];
#pragma unroll
    for (int k = 1; k < 8; k++) {
        asm volatile("" : "+v"(word));
        word = idx == k ? n.w[k] : word;
    }
    return ((word >> (lo & 31)) & ((1u << cnt) - 1)) != 0;
}
__device__ __forceinline__ bool rows_needed(const NoNeed &, int, int) { return true; }
// n > 256: the mask's words in HBM (constant address space: wave-uniform
// indices become scalar loads)
struct NeedMem {
    const __attribute__((address_space(4))) uint32_t *w;
};
__device__ __forceinline__ bool rows_needed(const NeedMem &n, int lo, int cnt) {
    if (cnt >= 32) {
        uint32_t acc = 0;
        for (int k = lo >> 5; k < (lo + cnt) >> 5; k++) acc |= n.w[k];
        return acc != 0;
    }
    return ((((const uint32_t *)n.w)[lo >> 5] >> (lo & 31)) & ((1u << cnt) - 1)) != 0;
}
__device__ __forceinline__ Need load_need(const uint32_t (&src)[8]) {
    Need n;
#pragma unroll
    for (int k = 0; k < 8; k++) n.w[k] = __builtin_amdgcn_readfirstlane(src[k]);
    return n;
}
__device__ __forceinline__ Need load_need(const __attribute__((address_space(4))) uint32_t (&src)[8]) {
    Need n;
#pragma unroll
    for (int k = 0; k < 8; k++) n.w[k] = src[k];  // constant address space: scalar loads
    return n;
}

// Output index of revealed work row r, or -1: outputs are numbered as the
// reconstruct plan lists them (codec.cpp: erased data shards = work rows
// m.. first, then erased parity shards = rows 0..m-1), i.e. the rank of r
// among the set bits of the revealed-row mask in the rotated order [m, n),
// [0, m).  Replaces an LDS row -> output table (k_rec_lds then needs no LDS
// beyond its 32 KB tile at n = 256).
__device__ __forceinline__ int reveal_index(const Need &n, int m, int r) {
    int below = 0, below_m = 0, total = 0;
    const int wr = r >> 5;
    uint32_t word = n.w[0];
#pragma unroll
    for (int k = 0; k < 8; k++) {
        const int c = __builtin_popcount(n.w[k]);  // wave-uniform words: scalar counts
        total += c;
        if (k * 32 + 32 <= m) below_m += c;
        else if (k * 32 < m) below_m += __builtin_popcount(n.w[k] & ((1u << (m & 31)) - 1));
        below += k < wr ? c : 0;
        if (k > 0) {
            asm volatile("" : "+v"(word));  // a select chain, not a stack array (see rows_needed)
            word = wr == k ? n.w[k] : word;
        }
    }
    const uint32_t bit = 1u << (r & 31);
    if (!(word & bit)) return -1;
    below += __builtin_popcount(word & (bit - 1));
    return r >= m ? below - below_m : total - below_m + below;
}

}  // namespace rec
}  // namespace rs
