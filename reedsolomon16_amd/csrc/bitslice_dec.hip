// Bit-sliced GF(2^16) reconstruct for n = 256 work rows (gfx950):
// k_rec_bs256, the C4 path (128 data + 32 parity, any erasure pattern).
//
// Reference: reconstruct leopard16.go:390-570 -- scale the present shards by
// their error locators (mulgf16 :492-514), ifftDITDecoder over n rows
// (:573-615), the formal derivative (:527-530), fftDIT truncated to m + k
// (:534-540, errorBitfield pruning :1076-1252), reveal (:545-566).
//
// Why bit-sliced: the byte-permute LDS kernel (kernels.hip k_rec_lds) spends
// ~80 % of its VALU on v_perm_b32 multiplies.  Every decoder
// twiddle for n = 256 is fftSkew[< 255], an element of GF(2^8), and it is a
// constant of n: the butterfly of layer L on rows (a, a + 2^L) uses
// fftSkew[(a & ~(2^(L+1) - 1)) + 2^L - 1] in both transforms
// (tools/gen_bs_tables.cpp DecTab256).  In subfield coordinates
// (gf_host.hpp SubCoords) a product with such a twiddle is the same 8x8
// GF(2) map on both byte halves, i.e. a fixed XOR network over 8 bit-planes.
//
// Tile: 1 KB of columns (16 blocks of 64 bytes) of every row of one stripe.
// Lane l = (block b = l & 15, half h = (l >> 4) & 1, row bit 0 z = l >> 5);
// a lane holds 16 rows x 8 planes (128 VGPRs).  One workgroup per CU (the LDS
// image below takes all 160 KB), persistent over tiles, 12 waves (three per
// SIMD, <= 168 VGPRs): 8 run phase 2, and the phase-1 / phase-3 units of a
// tile go one per wave (make_plan), phase 3 of a tile overlapping phase 1 of
// the next one.
//
//   A layout: wave w = row bits 5-7, registers i = row bits 1-4.
//   B layout: wave v = row bits 1-3, registers q = row bits 4-7.
//
// Phase 1 (A, one wave per 32-row group below mtrunc): load each row as one 1 KB wave
// access (row-uniform, so the error-locator scaling reads its table from
// SGPRs), scale into subfield coordinates, IFFT layer 0 in byte form (rows
// 2i, 2i+1 of a lane are both in registers; wave-uniform tables), then
// permlane32 / permlane16 swaps and an in-lane bit transpose into planes, and
// IFFT layers 1-4 as constant XOR networks (one code path per wave role).
// Phase 2 (B, waves 0-7, one code path): IFFT layers 5-7, the formal
// derivative, FFT layers 7-5.  The derivative D = I + sum_b N_b (N_b: row r
// gets in[r | 2^b] when bit b of r is clear) splits into H = N_4..N_7, local
// in B, and Lo = N_0..N_3, which acts on row bits the B layers neither touch
// nor read their twiddles from, so it commutes with them:
//   B_F D B_I u = B_F (I + H) B_I u + Lo (B_F B_I) u = B_F (I + H) B_I u + Lo u,
// since the FFT layers invert the IFFT layers (same twiddles, inverse
// butterflies).  Lo u needs rows of other waves: they come from the LDS image
// of u, which phase 2 still holds.
// Phase 3 (A, one wave per group with a revealed row): FFT layers 4-1 (constant networks,
// pruned by the revealed-row mask), back to bytes, FFT layer 0 in byte form,
// reveal (error-locator scaling out of subfield coordinates), 1 KB stores.
//
// The LDS image holds rows < 160 (1 KB each): the kernel serves n = 256 codecs
// with m + k <= 160 (C4: 160).  Rows >= mtrunc of the decoder IFFT input are
// zero, rows >= 160 feed no output row < m + k.
#include <algorithm>
#include <atomic>
#include <climits>
#include <map>
#include <mutex>
#include <cstdio>
#include <vector>

#include "bs_common.hpp"
#include "bs_tables.h"
#include "kernels.hpp"
#include "rec_common.hpp"
#include "schedule.hpp"

namespace rs {
namespace {
using namespace bs;
using namespace rec;

typedef DecTab256 DT;
constexpr int kTile = 1024;      // column bytes per workgroup
constexpr int kImgRows = 160;    // LDS image rows
constexpr int kTw8 = 8;          // dwords per subfield twiddle table (kTwDwords8)
constexpr int kTw16 = 24;        // dwords per full-field table (kTwDwords16)
constexpr uint32_t kMod = 65535;

// Tables, shard maps and row pointers are read through the constant address
// space: read-only for the launch, so wave-uniform addresses become scalar loads.
typedef __attribute__((address_space(4))) const uint32_t cu32_t;
typedef __attribute__((address_space(4))) const int ci32_t;
typedef uint8_t *gptr_t;
typedef __attribute__((address_space(4))) const gptr_t cptr_t;  // a row pointer held in read-only memory
__device__ __forceinline__ cu32_t *ctab(const uint32_t *t) { return (cu32_t *)t; }

__device__ __forceinline__ uint32_t perm(uint32_t s0, uint32_t s1, uint32_t sel) {
    return __builtin_amdgcn_perm(s0, s1, sel);
}
__device__ __forceinline__ uint32_t xor3v(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// Byte form of a row in a lane: 8 symbols as (lo dwords l0, l1; hi dwords h0, h1),
// or in subfield coordinates (c0 dwords; c1 dwords).
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

// x ^= M * y over 8 planes (M row i: bit j set when plane j feeds plane i).
template <int L, int G>
__device__ __forceinline__ void net_add(Half &x, const Half &y) {
    sfor<8>([&](auto I) __attribute__((always_inline)) {
        constexpr int i = decltype(I)::value;
        xor_net8c<DT::m8[L][G][i]>(x[i], y);
    });
}
template <int L, int G> constexpr bool tw_zero() { return DT::logs[L][G] == kMod; }

template <int L, int G>
__device__ __forceinline__ void bs_ifft2(Half &x, Half &y) {
    xor8(y, x);
    if constexpr (!tw_zero<L, G>()) net_add<L, G>(x, y);
    __builtin_amdgcn_sched_barrier(0);
}
// FFT butterfly; Y = false: only x is needed afterwards.
template <int L, int G, bool Y = true>
__device__ __forceinline__ void bs_fft2(Half &x, Half &y) {
    if constexpr (!tw_zero<L, G>()) net_add<L, G>(x, y);
    if constexpr (Y) xor8(y, x);
    __builtin_amdgcn_sched_barrier(0);
}

// Layer-0 twiddle slot of rows (r, r + 1), r even: the radix-4 pass at dist 1
// holds (m01, m02, m23) per group of 4 rows; layer 0 uses m01 for rows 4g,
// 4g + 1 and m23 for 4g + 2, 4g + 3 (schedule.hpp ifft_slot / fft_slot).
constexpr __host__ __device__ int slot0(int r) { return 3 * (r >> 2) + ((r & 2) ? 2 : 0); }
constexpr int kFft0Slot = fft_slot(8, 0, 0);
static_assert(ifft_slot(8, 0, 6) == slot0(6) && ifft_slot(8, 0, 132) == slot0(132) &&
                  fft_slot(8, 0, 6) == kFft0Slot + slot0(6) && fft_slot(8, 0, 158) == kFft0Slot + slot0(158),
              "layer-0 slots");
// Rows (bit q of the mask) still zero after an IFFT layer on register-row bit qb.
constexpr uint32_t z_after(uint32_t z, int qb) {
    uint32_t r = 0;
    for (int q = 0; q < 16; q++) {
        const int x = q & ~(1 << qb), y = q | (1 << qb);
        if (((z >> x) & 1) && ((z >> y) & 1)) r |= 1u << q;
    }
    return r;
}

// The launch arguments, read through an opaque pointer into the kernarg
// segment at each use: the persistent loop would otherwise keep every field
// it touches in SGPRs for the whole loop (hundreds of SGPR spills).
typedef __attribute__((address_space(4))) const RecArgs cargs_t;

template <bool STRIDED>
struct Dec {
    cargs_t *ap;        // the kernel's RecArgs (first kernel argument, kernarg offset 0)
    uint32_t V[16][8];  // A layout: V[i] = row 32w + 2i + z (byte form: row 32w + t at V[t >> 1][4 (t & 1) ..])
    int w;
    uint32_t lds0;      // LDS address of the image
    int grp;            // phase 1 / phase 3 row group: rows 32 grp .. 32 grp + 31 (A layout)
    uint64_t col;       // first column byte of the tile
    uint8_t *sbase;     // this stripe (strided shards), or nullptr

    __device__ __forceinline__ cargs_t &args() const {
        cargs_t *p = ap;
        asm volatile("" : "+s"(p));
        return *p;
    }

    __device__ __forceinline__ uint32_t *bytes(int t) { return &V[t >> 1][4 * (t & 1)]; }
    // The lane index and what derives from it, recomputed where used: at three
    // waves per SIMD (<= 168 VGPRs) every long-lived lane constant is a spill.
    __device__ __forceinline__ uint32_t lane() const {
        uint32_t t = __builtin_amdgcn_workitem_id_x();
        asm volatile("" : "+v"(t));
        return t & 63u;
    }
    // LDS byte offset of this lane's 16 bytes in row 0, plane quad 0 (+ z rows)
    __device__ __forceinline__ uint32_t lbase() const {
        const uint32_t l = lane();
        return lds0 + (l & 31u) * 16u + (l >> 5) * 1024u;
    }
    // work row r's source shard (src_idx / src: -1 / nullptr for a zero row),
    // as a buffer descriptor over this tile with an empty range for zero rows
    __device__ __forceinline__ __amdgpu_buffer_rsrc_t src_rsrc(cargs_t &a, int r) const {
        const uint8_t *row;
        bool live;
        if constexpr (STRIDED) {
            const int i = ((ci32_t *)a.src_idx)[r];
            live = i >= 0;
            row = sbase + (uint64_t)(live ? i : 0) * a.stride;
        } else {
            row = ((cptr_t *)a.src)[r];
            live = row != nullptr;
            row = live ? row : (const uint8_t *)a.tw_in;
        }
        return row_rsrc(a, row, live ? 0u : 1u);
    }
    __device__ __forceinline__ uint8_t *dst_row(cargs_t &a, int j) const {
        if constexpr (STRIDED) return sbase + (uint64_t)((ci32_t *)a.dst_idx)[j] * a.stride;
        else return ((cptr_t *)a.dst)[j];
    }
    // one row's 1 KB through a buffer descriptor whose range ends at the row end
    // (empty = true: a descriptor with no range, every load reads zero)
    __device__ __forceinline__ __amdgpu_buffer_rsrc_t row_rsrc(cargs_t &a, const void *row, uint32_t empty = 0) const {
        const uint32_t n = empty ? 0u : (uint32_t)std::min<uint64_t>(a.S - col, kTile);
        return __builtin_amdgcn_make_buffer_rsrc((void *)((const uint8_t *)row + col), 0, (int)n, 0x00020000);
    }
    // lane (b, g, p) holds bytes [b*64 + p*32 + g*16, +16) of a row: lo (p = 0)
    // or hi (p = 1) bytes of symbols 16g .. 16g + 15 of block b
    __device__ __forceinline__ uint32_t lane_off() const {
        const uint32_t l = lane();
        return (l & 15u) * 64u + (l >> 5) * 32u + ((l >> 4) & 1u) * 16u;
    }

    // ---------------- phase 1: rows 32 grp .. 32 grp + 31
    // all 32 row loads in flight at once, straight into the row registers
    // (the wave's 32 KB; missing rows read as zero through an empty range)
    __device__ __forceinline__ void load_rows() {
        cargs_t &a = args();
        const uint32_t off = lane_off();
        sfor<32>([&](auto T) __attribute__((always_inline)) {
            constexpr int t = decltype(T)::value;
            const u32x4 x = __builtin_amdgcn_raw_buffer_load_b128(src_rsrc(a, 32 * grp + t), off, 0, 0);
#pragma unroll
            for (int d = 0; d < 4; d++) V[t >> 1][4 * (t & 1) + d] = x[d];
        });
        __builtin_amdgcn_sched_barrier(0);
    }
    // Rows into subfield coordinates, each times its errLocs factor: row t's
    // table is loaded while row t - 1 is multiplied (one table in flight; all
    // 32 at once would not fit the SGPRs).
    __device__ __forceinline__ void scale() {
        cargs_t &a = args();
        cu32_t *base = ctab(a.tw_in) + (uint64_t)(32 * grp) * kTw16;
        Tab<20> cur = tab_at<20>(base);
        sfor<32>([&](auto T) __attribute__((always_inline)) {
            constexpr int t = decltype(T)::value;
            Tab<20> nxt;
            if constexpr (t + 1 < 32) nxt = tab_at<20>(base + (t + 1) * kTw16);
            uint32_t(&v)[8] = V[t >> 1];
            constexpr int o = 4 * (t & 1);
            // pair each lane's lo bytes with the hi bytes of the same symbols:
            // p = 0 keeps symbols 16g + 0..7, p = 1 symbols 16g + 8..15
            swap32(v[o + 0], v[o + 2]);
            swap32(v[o + 1], v[o + 3]);
            uint32_t y[4] = {v[o], v[o + 1], v[o + 2], v[o + 3]}, s[4];
            mul16(s, y, cur);
            // the product is due before the next row's steps (volatile, ordered):
            // otherwise the multiplies sink below every row's table loads
            asm volatile("" : "+v"(s[0]), "+v"(s[1]), "+v"(s[2]), "+v"(s[3]));
#pragma unroll
            for (int d = 0; d < 4; d++) v[o + d] = s[d];
            if constexpr (t + 1 < 32) cur = nxt;
            __builtin_amdgcn_sched_barrier(0);
        });
    }
    // IFFT layer 0 (rows 2i, 2i + 1) in byte form: y ^= x; x ^= y * t
    // (pair i + 1's table loads while pair i multiplies)
    __device__ __forceinline__ void ifft0_bytes() {
        cargs_t &a = args();
        cu32_t *tw = ctab(a.tw_ifft) + (uint64_t)slot0(32 * grp) * kTw8;  // slot0(32w + 2i) = slot0(32w) + slot0(2i)
        Tab<5> cur = tab_at<5>(tw);
        sfor<16>([&](auto I) __attribute__((always_inline)) {
            constexpr int i = decltype(I)::value;
            Tab<5> nxt;
            if constexpr (i + 1 < 16) nxt = tab_at<5>(tw + slot0(2 * i + 2) * kTw8);
            uint32_t *x = bytes(2 * i), *y = bytes(2 * i + 1);
#pragma unroll
            for (int d = 0; d < 4; d++) y[d] ^= x[d];
            mul8_add(x, y, cur);
            asm volatile("" : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]));
            if constexpr (i + 1 < 16) cur = nxt;
            __builtin_amdgcn_sched_barrier(0);
        });
    }
    // FFT layer 0 in byte form: x ^= y * t; y ^= x (pairs with a revealed row)
    __device__ __forceinline__ void fft0_bytes(uint32_t nw) {
        cargs_t &a = args();
        cu32_t *tw = ctab(a.tw_fft) + (uint64_t)(kFft0Slot + slot0(32 * grp)) * kTw8;
        sfor<16>([&](auto I) __attribute__((always_inline)) {
            constexpr int i = decltype(I)::value;
            if ((nw >> (2 * i)) & 3u) {
                uint32_t *x = bytes(2 * i), *y = bytes(2 * i + 1);
                mul8_add(x, y, tab_at<5>(tw + slot0(2 * i) * kTw8));
#pragma unroll
                for (int d = 0; d < 4; d++) y[d] ^= x[d];
            }
            __builtin_amdgcn_sched_barrier(0);
        });
    }
    // byte form (rows t in lanes (b, g, p)) <-> planes (register rows i in lanes (b, h, z));
    // mask: register rows to convert (bit i)
    __device__ __forceinline__ void to_planes(uint32_t mask) {
#pragma unroll
        for (int i = 0; i < 16; i++) {
            if (!((mask >> i) & 1)) continue;
            // lane bit 5: symbol group p <-> row bit 0
#pragma unroll
            for (int d = 0; d < 4; d++) swap32(V[i][d], V[i][4 + d]);
            // lane bit 4: symbol group g <-> half h
            swap16(V[i][0], V[i][2]);
            swap16(V[i][1], V[i][3]);
            swap16(V[i][4], V[i][6]);
            swap16(V[i][5], V[i][7]);
            bs_transpose8(V[i]);
            __builtin_amdgcn_sched_barrier(0);  // one row at a time: the transposes are not in place
        }
    }
    __device__ __forceinline__ void to_bytes(uint32_t mask) {
#pragma unroll
        for (int i = 0; i < 16; i++) {
            if (!((mask >> i) & 1)) continue;
            bs_transpose8(V[i]);
            swap16(V[i][0], V[i][2]);
            swap16(V[i][1], V[i][3]);
            swap16(V[i][4], V[i][6]);
            swap16(V[i][5], V[i][7]);
#pragma unroll
            for (int d = 0; d < 4; d++) swap32(V[i][d], V[i][4 + d]);
            __builtin_amdgcn_sched_barrier(0);
        }
    }
    // IFFT layers 1-4 of role W (rows 32 W ..): register rows i, i + 2^(L-1) (row bit L)
    template <int W>
    __device__ __forceinline__ void ifft_a() {
        sfor<4>([&](auto LI) __attribute__((always_inline)) {
            constexpr int L = 1 + decltype(LI)::value, s = 1 << (L - 1);
            sfor<8>([&](auto Q) __attribute__((always_inline)) {
                constexpr int q = decltype(Q)::value;
                constexpr int i = ((q >> (L - 1)) << L) | (q & (s - 1));
                bs_ifft2<L, ((32 * W + 2 * i) >> (L + 1))>(V[i], V[i + s]);
            });
        });
    }
    // IFFT layers 1-4 with the role grp chosen per butterfly: V is live into
    // the role choice here, and a branch per role around the whole pass left
    // the allocator holding two copies of the rows.  Each role writes
    // x ^ M y into fresh registers (no tied operands) and the result moves into x.
    template <int L, int I>
    __device__ __forceinline__ void ifft_bf_a() {
        constexpr int s = 1 << (L - 1);
        Half &x = V[I], &y = V[I + s];
        xor8(y, x);
        Half nx;
        dispatch<5>(grp, [&](auto W) __attribute__((always_inline)) {
            constexpr int g = (32 * decltype(W)::value + 2 * I) >> (L + 1);
            sfor<8>([&](auto K) __attribute__((always_inline)) {
                constexpr int k = decltype(K)::value;
                xor_net8f<DT::m8[L][g][k]>(nx[k], x[k], y);
            });
        });
#pragma unroll
        for (int k = 0; k < 8; k++) x[k] = nx[k];
        __builtin_amdgcn_sched_barrier(0);
    }
    // FFT butterfly of layer L (1-4) on register rows I, I + 2^(L-1), the role
    // grp chosen per butterfly as in ifft_bf_a: x ^= M y; y ^= x
    template <int L, int I>
    __device__ __forceinline__ void fft_bf_a() {
        constexpr int s = 1 << (L - 1);
        Half &x = V[I], &y = V[I + s];
        Half nx;
        dispatch<5>(grp, [&](auto W) __attribute__((always_inline)) {
            constexpr int g = (32 * decltype(W)::value + 2 * I) >> (L + 1);
            sfor<8>([&](auto K) __attribute__((always_inline)) {
                constexpr int k = decltype(K)::value;
                xor_net8f<DT::m8[L][g][k]>(nx[k], x[k], y);
            });
        });
#pragma unroll
        for (int k = 0; k < 8; k++) x[k] = nx[k];
        xor8(y, x);
        __builtin_amdgcn_sched_barrier(0);
    }
    __device__ __forceinline__ void fft_a_rt() {
        sfor<4>([&](auto LI) __attribute__((always_inline)) {
            constexpr int L = 4 - decltype(LI)::value, s = 1 << (L - 1);
            sfor<8>([&](auto Q) __attribute__((always_inline)) {
                constexpr int q = decltype(Q)::value;
                fft_bf_a<L, ((q >> (L - 1)) << L) | (q & (s - 1))>();
            });
        });
    }
    __device__ __forceinline__ void ifft_a_rt() {
        sfor<4>([&](auto LI) __attribute__((always_inline)) {
            constexpr int L = 1 + decltype(LI)::value, s = 1 << (L - 1);
            sfor<8>([&](auto Q) __attribute__((always_inline)) {
                constexpr int q = decltype(Q)::value;
                ifft_bf_a<L, ((q >> (L - 1)) << L) | (q & (s - 1))>();
            });
        });
    }
    // ---------------- LDS image: row r at r * 1024, plane quad pq at + pq * 512, lane at + (lane & 31) * 16
    __device__ __forceinline__ void img_put(int row_nz, const Half &v) {  // row_nz: row without the lane's z
        uint32_t o = lbase();
        asm volatile("" : "+v"(o));
        o += (uint32_t)row_nz * 1024u;
        *(lds_u4 *)(uintptr_t)o = u32x4{v[0], v[1], v[2], v[3]};
        *(lds_u4 *)(uintptr_t)(o + 512) = u32x4{v[4], v[5], v[6], v[7]};
    }
    __device__ __forceinline__ void img_get(int row_nz, Half &v) const {
        uint32_t o = lbase();
        asm volatile("" : "+v"(o));
        o += (uint32_t)row_nz * 1024u;
        const u32x4 x = *(const lds_u4 *)(uintptr_t)o;
        const u32x4 y = *(const lds_u4 *)(uintptr_t)(o + 512);
        v[0] = x[0], v[1] = x[1], v[2] = x[2], v[3] = x[3];
        v[4] = y[0], v[5] = y[1], v[6] = y[2], v[7] = y[3];
    }
    // v ^= image row row_nz (+ the lane's z); ONLY_Z0: v ^= image row `row_nz`
    // itself in lanes with z = 0 (zmask all ones there), nothing in z = 1 lanes
    template <bool ONLY_Z0>
    __device__ __forceinline__ void img_xor(int row_nz, Half &v) const {
        Half p;
        const uint32_t l = lane();
        const uint32_t zmask = l < 32 ? ~0u : 0u;
        img_get(ONLY_Z0 ? row_nz - (int)(l >> 5) : row_nz, p);
#pragma unroll
        for (int k = 0; k < 8; k++) {
            if constexpr (ONLY_Z0) asm("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x78" : "+v"(v[k]) : "v"(p[k]), "v"(zmask));  // v ^= p & m (truth table over S0 = 0xF0, S1 = 0xCC, S2 = 0xAA)
            else ixor(v[k], p[k]);
        }
    }

    // ---------------- phase 2: rows z + 2v + 16q, q = 0..15 (rows >= 160 are zero)
    static constexpr int NQ = kImgRows / 16;  // 10 rows per lane below 160
    __device__ __forceinline__ void phase2() {
        int v = w;
        asm volatile("" : "+s"(v));  // per tile: keeps the image offsets from being hoisted out of the tile loop
#pragma unroll
        for (int q = 0; q < 16; q++) {
            if (q < NQ) img_get(2 * v + 16 * q, V[q]);
            else
#pragma unroll
                for (int k = 0; k < 8; k++) V[q][k] = 0;
        }
        // IFFT layers 5, 6, 7 (row bits 5-7 = q bits 1-3); rows q >= NQ start at zero
        constexpr uint32_t Z0 = ~((1u << NQ) - 1u) & 0xFFFFu;
        ifft_b<5, Z0>();
        constexpr uint32_t Z1 = z_after(Z0, 1);
        ifft_b<6, Z1>();
        constexpr uint32_t Z2 = z_after(Z1, 2);
        ifft_b<7, Z2>();
        // (I + H): out[q] ^= in[q | 2^b] for clear bits b of q (row bits 4-7); ascending q reads unmodified partners
#pragma unroll
        for (int q = 0; q < 16; q++)
#pragma unroll
            for (int b = 0; b < 4; b++)
                if (!((q >> b) & 1)) xor8(V[q], V[q | (1 << b)]);
        // FFT layers 7, 6, 5; outputs only rows q < NQ
        fft_b<7, 0xFFFFu>();
        fft_b<6, 0x0FFFu>();  // layer 5 reads rows 0..11
        fft_b<5, (1u << NQ) - 1u>();
        // + Lo u: rows r | 2^b for clear bits b of r among row bits 0-3, read from the image of u
#pragma unroll
        for (int q = 0; q < NQ; q++) {
            const int r = 2 * v + 16 * q;  // without z
            img_xor<true>(r + 1, V[q]);  // bit 0 (z = 0 lanes only)
            if (!(v & 1)) img_xor<false>(r + 2, V[q]);
            if (!(v & 2)) img_xor<false>(r + 4, V[q]);
            if (!(v & 4)) img_xor<false>(r + 8, V[q]);
        }
    }
    template <int L, uint32_t Z>
    __device__ __forceinline__ void ifft_b() {
        constexpr int qb = L - 4, s = 1 << qb;
        sfor<8>([&](auto Q) __attribute__((always_inline)) {
            constexpr int qq = decltype(Q)::value;
            constexpr int q = ((qq >> qb) << (qb + 1)) | (qq & (s - 1));
            if constexpr (!(((Z >> q) & 1) && ((Z >> (q + s)) & 1))) bs_ifft2<L, ((16 * q) >> (L + 1))>(V[q], V[q + s]);
        });
    }
    // OUT: rows q whose result is needed
    template <int L, uint32_t OUT>
    __device__ __forceinline__ void fft_b() {
        constexpr int qb = L - 4, s = 1 << qb;
        sfor<8>([&](auto Q) __attribute__((always_inline)) {
            constexpr int qq = decltype(Q)::value;
            constexpr int q = ((qq >> qb) << (qb + 1)) | (qq & (s - 1));
            constexpr bool nx = (OUT >> q) & 1, ny = (OUT >> (q + s)) & 1;
            constexpr int g = (16 * q) >> (L + 1);
            if constexpr (ny) bs_fft2<L, g, true>(V[q], V[q + s]);
            else if constexpr (nx) bs_fft2<L, g, false>(V[q], V[q + s]);
        });
    }

    // ---------------- phase 3 reveal: rows 32 grp + t revealed (nw), out = work * (mod - errLocs)
    __device__ __forceinline__ void reveal(uint32_t nw) {
        cargs_t &a = args();
        const Need need = load_need(a.need);
        // output index of revealed row r = 32 grp + t (rec_common.hpp reveal_index):
        // its rank among the revealed rows in the rotated order [m, n), [0, m)
        int below = 0, below_m = 0, total = 0;
#pragma unroll
        for (int k = 0; k < 8; k++) {
            const int c = __builtin_popcount(need.w[k]);
            total += c;
            if (k * 32 + 32 <= a.m) below_m += c;
            else if (k * 32 < a.m) below_m += __builtin_popcount(need.w[k] & ((1u << (a.m & 31)) - 1));
            below += k < grp ? c : 0;
        }
        const int j_hi = below - below_m, j_lo = total - below_m + below;
        const uint32_t off = lane_off();
        sfor<32>([&](auto T) __attribute__((always_inline)) {
            constexpr int t = decltype(T)::value;
            if ((nw >> t) & 1u) {
                const int r = 32 * grp + t;
                const int j = (r >= a.m ? j_hi : j_lo) + __builtin_popcount(nw & ((1u << t) - 1u));
                uint32_t o[4];
                uint32_t y[4] = {bytes(t)[0], bytes(t)[1], bytes(t)[2], bytes(t)[3]};
                mul16(o, y, tab_at<20>(ctab(a.tw_out) + (uint64_t)j * kTw16));
                swap32(o[0], o[2]);  // back to lo bytes (p = 0) / hi bytes (p = 1) of symbols 16g..16g+15
                swap32(o[1], o[3]);
                __builtin_amdgcn_raw_buffer_store_b128(u32x4{o[0], o[1], o[2], o[3]}, row_rsrc(a, dst_row(a, j)), off, 0, 0);
            }
            __builtin_amdgcn_sched_barrier(0);
        });
    }
};

// A role branch starts and ends with a volatile marker of its own: the
// branches' first and last instructions (the image stores) are identical
// across roles, and the CFG simplifier would otherwise sink them into a shared
// block that has to merge every row value of every role.
template <int W>
__device__ __forceinline__ void role_mark() {
    asm volatile("; role %0" ::"n"(W));
}

// RS_DEC_ABL: bitmask of steps left out (build experiments only; wrong results):
// 1 row loads, 2 phase-1 transform, 4 phase 2, 8 phase-3 transform, 16 reveal
#ifndef RS_DEC_ABL
#define RS_DEC_ABL 0
#endif
#define ABL(b) ((RS_DEC_ABL >> (b)) & 1)
// RS_DEC_STAMP (diagnostic builds only): per-wave cycle sums of the loop's
// segments, written to DecPlan::stamps and printed by the launcher.
#ifdef RS_DEC_STAMP
#define STAMP(k)                                          \
    do {                                                  \
        const uint64_t now_ = __builtin_amdgcn_s_memtime(); \
        seg[k] += now_ - last_;                           \
        last_ = now_;                                     \
    } while (0)
#else
#define STAMP(k) \
    do {         \
    } while (0)
#endif
[[maybe_unused]] constexpr int kSegs = 16;

// Waves per workgroup: 8 run phase 2 (B layout: wave = row bits 1-3); all of
// them take phase-1 / phase-3 units.  12 = three waves per SIMD, one unit each.
#ifndef RS_DEC_WAVES
#define RS_DEC_WAVES 12
#endif
constexpr int kWaves = RS_DEC_WAVES;
static_assert(kWaves >= 8 && kWaves <= 12, "wave count");

// Work plan of a workgroup's waves (host-made, the same for every tile:
// launch_rec_bs256).  Phase 1 (load, scale, IFFT layers 0-4 of a 32-row group)
// and phase 3 (FFT layers 4-0 and reveal of a group with revealed rows) run
// only on the groups below mtrunc, 5 at C4; each is a unit of one wave.  The
// units go to waves so that the four SIMDs carry about the same VALU work
// (wave w runs on SIMD w & 3), and phase 3 of tile t overlaps phase 1 of the
// next tile, whose row loads the phase-1-only waves issue early.
struct DecPlan {
    uint64_t p3;   // 4 bits per wave: phase-3 group + 1 (0: none)
    uint64_t p1;   // 5 bits per wave: mask of phase-1 groups
    int ntx;       // column tiles per stripe
    int ntiles;    // column tiles x stripes
    uint64_t *stamps;  // RS_DEC_STAMP builds: kSegs cycle sums per wave
};

// Persistent over tiles t = blockIdx.x + i * gridDim.x (column tile t % ntx of
// stripe t / ntx).  Iteration i runs phases 2 and 3 of tile t_(i-1) and phase
// 1 of tile t_i:
//   phase 2 (all waves) -> Y into the image -> phase-3 waves read their rows ->
//   barrier (image free) -> phase 3 of t_(i-1) || phase 1 of t_i into the image.
template <bool STRIDED>
__global__ void __launch_bounds__(64 * kWaves, kWaves / 4) k_rec_bs256(RecArgs a, DecPlan pl) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[kImgRows * kTile / 4];
    Dec<STRIDED> d;
    d.ap = (cargs_t *)__builtin_amdgcn_kernarg_segment_ptr();
    d.lds0 = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) uint32_t *)lds;
    d.w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int w = d.w;
    const int p3g = (int)((pl.p3 >> (4 * w)) & 15u) - 1;
    const uint32_t p1m = (uint32_t)(pl.p1 >> (5 * w)) & 31u;
    const int first = p1m ? __builtin_ctz(p1m) : -1;
    uint32_t nw = 0;  // revealed rows of the phase-3 group
    if (p3g >= 0) {
        const Need need = load_need(a.need);
        nw = need.w[0];
#pragma unroll
        for (int k = 1; k < 8; k++) nw = p3g == k ? need.w[k] : nw;  // wave-uniform word select
    }
    auto set_tile = [&](int t) {
        const int y = t / pl.ntx;
        d.col = (uint64_t)(t - y * pl.ntx) * kTile;
        if constexpr (STRIDED) {
            cargs_t &ar = d.args();
            d.sbase = ar.base + (uint64_t)y * ar.stripe_stride;
        } else {
            d.sbase = nullptr;
        }
    };
    int t = -1, tn = blockIdx.x;  // tile in phases 2-3, tile in phase 1
    if (tn >= pl.ntiles) return;
#ifdef RS_DEC_STAMP
    uint64_t seg[kSegs] = {};
    uint64_t last_ = __builtin_amdgcn_s_memtime();
#endif
    for (;;) {
        const bool cur = t >= 0, more = tn < pl.ntiles;
        if (cur) {
            // ---- phase 2: Y = B_F (I + H) B_I u + Lo u (B layout)
            if (w < 8)
                if constexpr (!ABL(2)) d.phase2();
            STAMP(0);
            lds_barrier();  // every wave has read u
            STAMP(1);
            if (w < 8) {
                int wt = w;
                asm volatile("" : "+s"(wt));
#pragma unroll
                for (int q = 0; q < Dec<STRIDED>::NQ; q++) d.img_put(2 * wt + 16 * q, d.V[q]);
            }
            lds_barrier();
            STAMP(2);
        }
        const bool early = more && first >= 0 && (p3g < 0 || !cur);
        if (early) {  // a phase-1-only wave: its first group's rows are on the way during the exchange
            set_tile(tn);
            d.grp = first;
            if constexpr (!ABL(0)) d.load_rows();
        }
        if (cur) {
            if (p3g >= 0) {
                int g = p3g;
                asm volatile("" : "+s"(g));
                d.grp = g;
#pragma unroll
                for (int i = 0; i < 16; i++) d.img_get(32 * g + 2 * i, d.V[i]);
            }
            lds_barrier();  // the image is free for phase 1 of the next tile
            STAMP(3);
            // ---- phase 3: FFT layers 4-0 and reveal of the revealed rows of group p3g
            if (p3g >= 0) {
                set_tile(t);
                if constexpr (!ABL(3)) d.fft_a_rt();
                STAMP(13);
                // opaque per tile: the loop-invariant row tests would otherwise be
                // hoisted out of the tile loop as 48 live 64-bit masks (SGPR spills)
                uint32_t nwt = nw;
                asm volatile("" : "+s"(nwt));
                uint32_t pairs = 0;  // register rows holding a revealed row (either z)
#pragma unroll
                for (int i = 0; i < 16; i++) pairs |= ((nwt >> (2 * i)) & 3u) ? 1u << i : 0u;
                d.to_bytes(pairs);
                d.fft0_bytes(nwt);
                STAMP(14);
                if constexpr (!ABL(4)) d.reveal(nwt);
            }
            STAMP(4);
        }
        if (more) {
            // ---- phase 1: u = IFFT layers 0-4 of the scaled rows (A layout), into the image
            set_tile(tn);
            for (uint32_t m = p1m; m; m &= m - 1) {
                const int g = __builtin_ctz(m);
                d.grp = g;
                if (!(early && g == first))
                    if constexpr (!ABL(0)) d.load_rows();
                STAMP(7);
                d.scale();
                STAMP(8);
                if constexpr (!ABL(1)) d.ifft0_bytes();
                STAMP(9);
                d.to_planes(0xFFFFu);
                STAMP(10);
                // one code path per role: the rows leave for the image inside
                // it, so no row value is merged from the role branches
#ifdef RS_DEC_ROLE_PASS
                dispatch<5>(g, [&](auto W) __attribute__((always_inline)) {
                    constexpr int gw = decltype(W)::value;
                    role_mark<gw>();
                    if constexpr (!ABL(1)) d.template ifft_a<gw>();
#pragma unroll
                    for (int i = 0; i < 16; i++) d.img_put(32 * gw + 2 * i, d.V[i]);
                    role_mark<gw>();
                });
#else
                if constexpr (!ABL(1)) d.ifft_a_rt();
#pragma unroll
                for (int i = 0; i < 16; i++) d.img_put(32 * g + 2 * i, d.V[i]);
#endif
                STAMP(12);
            }
        }
        STAMP(5);
        if (!more) break;
        lds_barrier();  // u of tile tn is in the image
        STAMP(6);
        t = tn;
        tn += gridDim.x;
    }
#ifdef RS_DEC_STAMP
    if (d.lane() == 0)
        for (int k = 0; k < kSegs; k++) pl.stamps[((uint64_t)blockIdx.x * kWaves + w) * kSegs + k] = seg[k];
#endif
}

// Unit placement (see DecPlan).  Costs in VALU work: a phase-3 unit 2, a
// phase-1 unit 4 (load, scale and byte-form layer 0 of 32 rows on top of
// the plane layers).  A wave runs its units one after the other; wave w runs
// on SIMD w & 3.  Alone on its SIMD a wave issues a VALU instruction every
// ~4.3 cycles; SIMDs shared by two / three waves issue one every ~3.15 / ~2.8
// cycles between them (scripts/micro/valu_rate.hip).  The plan minimises
// max(chain x 4.3, SIMD load x 3.0) over every placement with at most one
// phase-3 unit per wave (it is read from the image before phase 1 of the
// next tile may overwrite it), and one unit per wave when there are enough
// waves; searched once per (groups, revealed groups) and cached.
DecPlan make_plan(const RecArgs &a) {
    const int G = (a.mtrunc + 31) / 32;
    uint32_t rmask = 0;  // groups with revealed rows
    for (int g = 0; g < G; g++)
        if (a.need[g]) rmask |= 1u << g;
    static std::mutex mu;
    static std::map<uint32_t, DecPlan> cache;
    const uint32_t key = (uint32_t)G << 8 | rmask;
    {
        std::lock_guard<std::mutex> lk(mu);
        auto it = cache.find(key);
        if (it != cache.end()) return it->second;
    }
    int r3[5], n3 = 0;
    for (int g = 0; g < G; g++)
        if ((rmask >> g) & 1) r3[n3++] = g;
    constexpr int C3 = 2, C1 = 4;
    double best = 1e30;
    DecPlan bp{};
    auto score = [&](const int *load) {
        double sc = 0;
        for (int w = 0; w < kWaves; w++) sc = std::max(sc, load[w] * 4.3);
        for (int q = 0; q < 4; q++) {
            int sl = 0;
            for (int w = q; w < kWaves; w += 4) sl += load[w];
            sc = std::max(sc, sl * 3.0);
        }
        return sc;
    };
    const bool one_each = n3 + G <= kWaves;
    for (uint32_t s3 = 0; s3 < (1u << kWaves); s3++) {
        if (__builtin_popcount(s3) != n3) continue;
        if (one_each) {
            const uint32_t comp = ((1u << kWaves) - 1) & ~s3;
            for (uint32_t s1 = comp;; s1 = (s1 - 1) & comp) {  // phase-1 waves: G of the others
                if (!s1) break;
                if (__builtin_popcount(s1) != G) continue;
                int load[kWaves] = {0};
                for (int w = 0; w < kWaves; w++) load[w] = ((s3 >> w) & 1) * C3 + ((s1 >> w) & 1) * C1;
                const double sc = score(load);
                if (sc < best - 1e-9) {
                    best = sc;
                    bp = DecPlan{};
                    int j = 0, g = 0;
                    for (int w = 0; w < kWaves; w++) {
                        if ((s3 >> w) & 1) bp.p3 |= (uint64_t)(r3[j++] + 1) << (4 * w);
                        if ((s1 >> w) & 1) bp.p1 |= 1ull << (5 * w + g++);
                    }
                }
            }
            continue;
        }
        int w1[5] = {0, 0, 0, 0, 0};
        for (;;) {  // non-decreasing wave indices w1[0..G-1]
            int load[kWaves] = {0};
            for (int w = 0; w < kWaves; w++)
                if ((s3 >> w) & 1) load[w] += C3;
            for (int g = 0; g < G; g++) load[w1[g]] += C1;
            const double sc = score(load);
            if (sc < best - 1e-9) {
                best = sc;
                bp = DecPlan{};
                int j = 0;
                for (int w = 0; w < kWaves; w++)
                    if ((s3 >> w) & 1) bp.p3 |= (uint64_t)(r3[j++] + 1) << (4 * w);
                for (int g = 0; g < G; g++) bp.p1 |= 1ull << (5 * w1[g] + g);
            }
            int g = G - 1;
            while (g >= 0 && w1[g] == kWaves - 1) g--;
            if (g < 0) break;
            w1[g]++;
            for (int h = g + 1; h < G; h++) w1[h] = w1[g];
        }
    }
    std::lock_guard<std::mutex> lk(mu);
    cache[key] = bp;
    return bp;
}

}  // namespace

bool rec_bs256_available(int bits, int logn, bool sub, int mtrunc) {
    return bits == 16 && logn == 8 && sub && mtrunc <= kImgRows;
}

hipError_t launch_rec_bs256(const RecArgs &a, hipStream_t s) {
    if (a.mtrunc > kImgRows) return hipErrorNotSupported;
    static std::atomic<int> cus_of[64];
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    int cus = dev < 64 ? cus_of[dev].load() : 0;
    if (!cus) {
        e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        if (e != hipSuccess) return e;
        if (dev < 64) cus_of[dev].store(cus);
    }
    DecPlan pl = make_plan(a);
    pl.ntx = (int)((a.S + kTile - 1) / kTile);
    const uint64_t ny = a.base && a.nstripes > 1 ? (uint64_t)a.nstripes : 1;
    if ((uint64_t)pl.ntx * ny > (uint64_t)INT32_MAX) return hipErrorInvalidValue;
    pl.ntiles = (int)(pl.ntx * ny);
    const unsigned grid = (unsigned)std::min<int>(pl.ntiles, std::max(cus, 1));
#ifdef RS_DEC_STAMP
    static uint64_t *dstamps = nullptr;
    static int nprint = 0;
    const size_t nst = (size_t)grid * kWaves * kSegs;
    if (!dstamps && hipMalloc(&dstamps, 4096 * 16 * kSegs * sizeof(uint64_t)) != hipSuccess) return hipErrorOutOfMemory;
    (void)hipMemsetAsync(dstamps, 0, nst * sizeof(uint64_t), s);
    pl.stamps = dstamps;
#endif
    if (a.base) hipLaunchKernelGGL(k_rec_bs256<true>, dim3(grid), dim3(64 * kWaves), 0, s, a, pl);
    else hipLaunchKernelGGL(k_rec_bs256<false>, dim3(grid), dim3(64 * kWaves), 0, s, a, pl);
#ifdef RS_DEC_STAMP
    if (nprint < 4 && pl.ntiles >= 1024) {
        nprint++;
        std::vector<uint64_t> h(nst);
        (void)hipStreamSynchronize(s);
        (void)hipMemcpy(h.data(), dstamps, nst * sizeof(uint64_t), hipMemcpyDeviceToHost);
        std::fprintf(stderr, "stamps: grid %u tiles %d plan p3 %012llx p1 %015llx (mean cycles per workgroup)\n", grid,
                     pl.ntiles, (unsigned long long)pl.p3, (unsigned long long)pl.p1);
        for (int w = 0; w < kWaves; w++) {
            std::fprintf(stderr, "  wave %d:", w);
            for (int k = 0; k < kSegs; k++) {
                double m = 0;
                for (unsigned b = 0; b < grid; b++) m += (double)h[((size_t)b * kWaves + w) * kSegs + k];
                std::fprintf(stderr, " %7.0f", m / grid);
            }
            std::fprintf(stderr, "\n");
        }
    }
#endif
    return hipGetLastError();
}

}  // namespace rs
