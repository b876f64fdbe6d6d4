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
// Lane l = (block b = l & 15, half h = (l >> 4) & 1, row bit 0 z = l >> 5).
// One workgroup per CU (the LDS image below takes all 160 KB), persistent
// over tiles, 12 waves (three per SIMD, <= 168 VGPRs): 8 run phase 2; the
// phase-1 / phase-3 units of a tile are 16-row units spread over the waves
// (make_plan).  Waves 8-11 take no part in phase 2: they run phase 1 of the
// next tile while waves 0-7 run phase 2 of the current one.
//
//   A layout: unit u = row bits 4-7, registers i = row bits 1-3 (8 rows x 8 planes).
//   B layout: wave v = row bits 1-3, registers q = row bits 4-7 (16 rows x 8 planes).
//
// Phase 1 (A, one 16-row unit below mtrunc at a time): load each row as one
// 1 KB wave access (row-uniform, so the error-locator scaling reads its table
// from SGPRs), scale into subfield coordinates, IFFT layer 0 in byte form
// (rows 2i, 2i+1 of a lane are both in registers; wave-uniform tables), then
// permlane32 / permlane16 swaps and an in-lane bit transpose into planes, and
// IFFT layers 1-3 as constant XOR networks (the unit's code path chosen per
// butterfly).
// Phase 2 (B, waves 0-7, one code path): IFFT layers 4-7, the formal
// derivative, FFT layers 7-4.  The derivative D = I + sum_b N_b (N_b: row r
// gets in[r | 2^b] when bit b of r is clear) splits into H = N_4..N_7, local
// in B, and Lo = N_0..N_3, which acts on row bits the B layers neither touch
// nor read their twiddles from, so it commutes with them:
//   B_F D B_I u = B_F (I + H) B_I u + Lo (B_F B_I) u = B_F (I + H) B_I u + Lo u,
// since the FFT layers invert the IFFT layers (same twiddles, inverse
// butterflies).  Lo u needs rows of other waves: they come from the LDS image
// of u, which phase 2 still holds.
// Phase 3 (A, one 16-row unit with a revealed row at a time): FFT layers 3-1
// (constant networks), back to bytes, FFT layer 0 in byte form, reveal
// (error-locator scaling out of subfield coordinates), 1 KB stores.
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
#include <cstring>
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
typedef __attribute__((address_space(4))) const int ci32_t;
typedef uint8_t *gptr_t;
typedef __attribute__((address_space(4))) const gptr_t cptr_t;  // a row pointer held in read-only memory

constexpr int kTile = 1024;      // column bytes per workgroup
constexpr int kImgRows = 160;    // LDS image rows
constexpr int kTw8 = 8;          // dwords per subfield twiddle table (kTwDwords8)
constexpr int kTw16 = 24;        // dwords per full-field table (kTwDwords16)
constexpr uint32_t kMod = 65535;

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
    // A layout: V[i] (i < 8) = row 16u + 2i + z of the unit being worked on
    // (byte form: row 16u + t at V[t >> 1][4 (t & 1) ..]); V[8..15] park a
    // second unit.  B layout (phase 2): V[q] = row z + 2v + 16q.
    uint32_t V[16][8];
    int w;
    uint32_t lds0;      // LDS address of the image
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

    // ---------------- phase 1: rows 16 u .. 16 u + 15 into V[0..7]
    // all 16 row loads in flight at once, straight into the row registers
    // (missing rows read as zero through an empty range)
    // (RO = 8: into V[8..15], the registers phase 3 leaves alone)
    template <int RO = 0>
    __device__ __forceinline__ void load_rows(int u) {
        cargs_t &a = args();
        const uint32_t off = lane_off();
        sfor<16>([&](auto T) __attribute__((always_inline)) {
            constexpr int t = decltype(T)::value;
            const u32x4 x = __builtin_amdgcn_raw_buffer_load_b128(src_rsrc(a, 16 * u + t), off, 0, 0);
#pragma unroll
            for (int d = 0; d < 4; d++) V[RO + (t >> 1)][4 * (t & 1) + d] = x[d];
        });
        __builtin_amdgcn_sched_barrier(0);
    }
    // Rows into subfield coordinates, each times its errLocs factor: row t's
    // table is loaded while row t - 1 is multiplied (one table in flight; all
    // 16 at once would not fit the SGPRs).
    __device__ __forceinline__ void scale(int u) {
        cargs_t &a = args();
        cu32_t *base = ctab(a.tw_in) + (uint64_t)(16 * u) * kTw16;
        Tab<20> cur = tab_at<20>(base);
        sfor<16>([&](auto T) __attribute__((always_inline)) {
            constexpr int t = decltype(T)::value;
            Tab<20> nxt;
            if constexpr (t + 1 < 16) nxt = tab_at<20>(base + (t + 1) * kTw16);
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
            if constexpr (t + 1 < 16) cur = nxt;
            __builtin_amdgcn_sched_barrier(0);
        });
    }
    // IFFT layer 0 (rows 2i, 2i + 1) in byte form: y ^= x; x ^= y * t
    // (pair i + 1's table loads while pair i multiplies)
    __device__ __forceinline__ void ifft0_bytes(int u) {
        cargs_t &a = args();
        cu32_t *tw = ctab(a.tw_ifft) + (uint64_t)slot0(16 * u) * kTw8;  // slot0(16u + 2i) = slot0(16u) + slot0(2i)
        Tab<5> cur = tab_at<5>(tw);
        sfor<8>([&](auto I) __attribute__((always_inline)) {
            constexpr int i = decltype(I)::value;
            Tab<5> nxt;
            if constexpr (i + 1 < 8) nxt = tab_at<5>(tw + slot0(2 * i + 2) * kTw8);
            uint32_t *x = bytes(2 * i), *y = bytes(2 * i + 1);
#pragma unroll
            for (int d = 0; d < 4; d++) y[d] ^= x[d];
            mul8_add(x, y, cur);
            asm volatile("" : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]));
            if constexpr (i + 1 < 8) cur = nxt;
            __builtin_amdgcn_sched_barrier(0);
        });
    }
    // FFT layer 0 in byte form: x ^= y * t; y ^= x (pairs with a revealed row)
    __device__ __forceinline__ void fft0_bytes(int u, uint32_t nw) {
        cargs_t &a = args();
        cu32_t *tw = ctab(a.tw_fft) + (uint64_t)(kFft0Slot + slot0(16 * u)) * kTw8;
        sfor<8>([&](auto I) __attribute__((always_inline)) {
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
        for (int i = 0; i < 8; i++) {
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
        for (int i = 0; i < 8; i++) {
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
    // IFFT butterfly of layer L (1-3) on register rows I, I + 2^(L-1), the
    // unit's twiddle chosen per butterfly: V is live into the choice here, and
    // a branch per unit around the whole pass left the allocator holding two
    // copies of the rows.  Each branch writes x ^ M y into fresh registers (no
    // tied operands) and the result moves into x.
    template <int L, int I>
    __device__ __forceinline__ void ifft_bf_a(int u) {
        constexpr int s = 1 << (L - 1);
        Half &x = V[I], &y = V[I + s];
        xor8(y, x);
        Half nx;
        dispatch<kImgRows / 16>(u, [&](auto U) __attribute__((always_inline)) {
            constexpr int g = (16 * decltype(U)::value + 2 * I) >> (L + 1);
            sfor<8>([&](auto K) __attribute__((always_inline)) {
                constexpr int k = decltype(K)::value;
                xor_net8f<DT::m8[L][g][k]>(nx[k], x[k], y);
            });
        });
#pragma unroll
        for (int k = 0; k < 8; k++) x[k] = nx[k];
        __builtin_amdgcn_sched_barrier(0);
    }
    // FFT butterfly of layer L (1-3) on register rows I, I + 2^(L-1): x ^= M y; y ^= x
    template <int L, int I>
    __device__ __forceinline__ void fft_bf_a(int u) {
        constexpr int s = 1 << (L - 1);
        Half &x = V[I], &y = V[I + s];
        Half nx;
        dispatch<kImgRows / 16>(u, [&](auto U) __attribute__((always_inline)) {
            constexpr int g = (16 * decltype(U)::value + 2 * I) >> (L + 1);
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
    __device__ __forceinline__ void fft_a(int u) {
        sfor<3>([&](auto LI) __attribute__((always_inline)) {
            constexpr int L = 3 - decltype(LI)::value, s = 1 << (L - 1);
            sfor<4>([&](auto Q) __attribute__((always_inline)) {
                constexpr int q = decltype(Q)::value;
                fft_bf_a<L, ((q >> (L - 1)) << L) | (q & (s - 1))>(u);
            });
        });
    }
    __device__ __forceinline__ void ifft_a(int u) {
        sfor<3>([&](auto LI) __attribute__((always_inline)) {
            constexpr int L = 1 + decltype(LI)::value, s = 1 << (L - 1);
            sfor<4>([&](auto Q) __attribute__((always_inline)) {
                constexpr int q = decltype(Q)::value;
                ifft_bf_a<L, ((q >> (L - 1)) << L) | (q & (s - 1))>(u);
            });
        });
    }
    // the phase-1 transform of unit u, from its rows in HBM to planes in V[0..7].
    // nbar: workgroup barriers to pass after IFFT layer 0 (an early wave passes
    // phase 2's two barriers there, so it does not hold phase 2 back; after the
    // scaling / after the transpose measured 1753 / 1704 against 1690 us per
    // 16 C4 stripes, profiles/r03_c4_bsdec_units_ab.txt)
    // pre: the unit's rows are already loaded into V[0..7] (load_rows issued earlier)
    __device__ __forceinline__ void phase1(int u, int nbar = 0, bool pre = false) {
        if (16 * u >= args().mtrunc) {  // rows past mtrunc: zero (the image rows still have to be written)
#pragma unroll
            for (int i = 0; i < 8; i++)
#pragma unroll
                for (int k = 0; k < 8; k++) V[i][k] = 0;
            for (int b = 0; b < nbar; b++) lds_barrier();
            return;
        }
        if (pre) {  // rows preloaded into V[8..15] (late waves, lab bit 8)
#pragma unroll
            for (int i = 0; i < 8; i++)
#pragma unroll
                for (int k = 0; k < 8; k++) V[i][k] = V[8 + i][k];
        } else {
            load_rows(u);
        }
        scale(u);
        ifft0_bytes(u);
        for (int b = 0; b < nbar; b++) lds_barrier();
        to_planes(0xFFu);
        ifft_a(u);
    }
    // V[0..7] <-> V[8..15] (the parked unit)
    __device__ __forceinline__ void park_swap() {
#pragma unroll
        for (int i = 0; i < 8; i++)
#pragma unroll
            for (int k = 0; k < 8; k++) {
                const uint32_t t = V[i][k];
                V[i][k] = V[8 + i][k];
                V[8 + i][k] = t;
            }
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
    // unit u's 8 register rows from / to V[RO..RO+7]
    template <int RO>
    __device__ __forceinline__ void unit_put(int u) {
#pragma unroll
        for (int i = 0; i < 8; i++) img_put(16 * u + 2 * i, V[RO + i]);
    }
    template <int RO>
    __device__ __forceinline__ void unit_get(int u) {
#pragma unroll
        for (int i = 0; i < 8; i++) img_get(16 * u + 2 * i, V[RO + i]);
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
        // IFFT layers 4-7 (row bits 4-7 = q bits 0-3); rows q >= NQ start at zero
        constexpr uint32_t Z0 = ~((1u << NQ) - 1u) & 0xFFFFu;
        ifft_b<4, Z0>();
        constexpr uint32_t Z1 = z_after(Z0, 0);
        ifft_b<5, Z1>();
        constexpr uint32_t Z2 = z_after(Z1, 1);
        ifft_b<6, Z2>();
        constexpr uint32_t Z3 = z_after(Z2, 2);
        ifft_b<7, Z3>();
        // (I + H): out[q] ^= in[q | 2^b] for clear bits b of q (row bits 4-7); ascending q reads unmodified partners
#pragma unroll
        for (int q = 0; q < 16; q++)
#pragma unroll
            for (int b = 0; b < 4; b++)
                if (!((q >> b) & 1)) xor8(V[q], V[q | (1 << b)]);
        // FFT layers 7-4; outputs only rows q < NQ
        fft_b<7, 0xFFFFu>();
        fft_b<6, 0x0FFFu>();         // layer 5 reads rows 0..11
        fft_b<5, (1u << NQ) - 1u>();  // layer 4 reads rows 0..9
        fft_b<4, (1u << NQ) - 1u>();
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

    // ---------------- phase 3: FFT layers 3-0 and the reveal of unit u's rows (V[0..7])
    // revealed rows of unit u (bit t: row 16u + t)
    __device__ __forceinline__ static uint32_t unit_need(const Need &need, int u) {
        uint32_t word = need.w[0];
#pragma unroll
        for (int k = 1; k < 8; k++) {
            asm volatile("" : "+s"(word));  // a select chain, not a stack array (rec_common.hpp rows_needed)
            word = (u >> 1) == k ? need.w[k] : word;
        }
        return (word >> (16 * (u & 1))) & 0xFFFFu;
    }
    __device__ __forceinline__ void phase3(int u) {
        cargs_t &a = args();
        const Need need = load_need(a.need);
        const uint32_t nw = __builtin_amdgcn_readfirstlane(unit_need(need, u));
        fft_a(u);
        uint32_t pairs = 0;  // register rows holding a revealed row (either z)
#pragma unroll
        for (int i = 0; i < 8; i++) pairs |= ((nw >> (2 * i)) & 3u) ? 1u << i : 0u;
        to_bytes(pairs);
        fft0_bytes(u, nw);
        reveal(u, nw, need);
    }
    // out = work * (mod - errLocs) for the revealed rows 16u + t (bit t of nw)
    __device__ __forceinline__ void reveal(int u, uint32_t nw, const Need &need) {
        cargs_t &a = args();
        // output index of revealed row r = 16 u + t (rec_common.hpp reveal_index):
        // its rank among the revealed rows in the rotated order [m, n), [0, m)
        int below = 0, below_m = 0, total = 0;
        uint32_t word = need.w[0];
#pragma unroll
        for (int k = 0; k < 8; k++) {
            const int c = __builtin_popcount(need.w[k]);
            total += c;
            if (k * 32 + 32 <= a.m) below_m += c;
            else if (k * 32 < a.m) below_m += __builtin_popcount(need.w[k] & ((1u << (a.m & 31)) - 1));
            below += k < (u >> 1) ? c : 0;
            if (k > 0) {
                asm volatile("" : "+s"(word));
                word = (u >> 1) == k ? need.w[k] : word;
            }
        }
        if (u & 1) below += __builtin_popcount(word & 0xFFFFu);
        const int j_hi = below - below_m, j_lo = total - below_m + below;
        const uint32_t off = lane_off();
        // The unit's byte-form rows go to its own 16 image rows, which no other
        // wave reads between this wave's unit_get and the image-free barrier;
        // one rolled loop then reveals the rows of nw.  Unrolled over the 16
        // rows the reveal was 14 KB of the kernel's code (the
        // instruction cache); the LDS round trip costs 16 ds_write_b128 per unit
        // and one ds_read_b128 per revealed row.
        const uint32_t sb = lds0 + (uint32_t)u * (16u * 1024u) + lane() * 16u;
#pragma unroll
        for (int i = 0; i < 8; i++) {
            *(lds_u4 *)(uintptr_t)(sb + i * 2048u) = u32x4{V[i][0], V[i][1], V[i][2], V[i][3]};
            *(lds_u4 *)(uintptr_t)(sb + i * 2048u + 1024u) = u32x4{V[i][4], V[i][5], V[i][6], V[i][7]};
        }
        uint32_t rem = nw;
        // (loading the next revealed row's table and output row while this one
        // is multiplied measured no faster: C4 x 16 1648 vs 1657-1666 us, same box)
#pragma nounroll
        while (rem) {
            const int t = __builtin_ctz(rem);
            rem &= rem - 1u;
            const int r = 16 * u + t;
            const int j = (r >= a.m ? j_hi : j_lo) + __builtin_popcount(nw & ((1u << t) - 1u));
            const u32x4 x = *(const lds_u4 *)(uintptr_t)(sb + (uint32_t)(t >> 1) * 2048u + (uint32_t)(t & 1) * 1024u);
            uint32_t o[4];
            const uint32_t y[4] = {x[0], x[1], x[2], x[3]};
            mul16(o, y, tab_at<20>(ctab(a.tw_out) + (uint64_t)j * kTw16));
            swap32(o[0], o[2]);  // back to lo bytes (p = 0) / hi bytes (p = 1) of symbols 16g..16g+15
            swap32(o[1], o[3]);
            __builtin_amdgcn_raw_buffer_store_b128(u32x4{o[0], o[1], o[2], o[3]}, row_rsrc(a, dst_row(a, j)), off, 0, 0);
        }
    }
};

// Waves per workgroup: 8 run phase 2 (B layout: wave = row bits 1-3); waves
// 8 .. kWaves-1 run phase 1 of the next tile meanwhile.  12 = three waves per SIMD.
constexpr int kWaves = 12;
static_assert(kWaves > 8 && kWaves <= 12, "wave count");
constexpr int kUnits = kImgRows / 16;  // 16-row units below the image end

// Work plan of a workgroup's waves (host-made, the same for every tile:
// launch_rec_bs256).  Phase 1 (load, scale, IFFT layers 0-3 of a 16-row unit)
// runs on the units below mtrunc (10 at C4) and phase 3 (FFT layers 3-0 and
// reveal) on the units with a revealed row.  Per wave, four 4-bit fields
// (unit + 1, 0: none): phase-3 units 0 and 1, phase-1 units 0 and 1.  Waves
// >= 8 hold phase-1 units only and run them before phase 2 of the previous
// tile ("early"); waves < 8 run theirs after phase 3.
struct DecPlan {
    uint64_t code[3];  // 16 bits per wave, waves 4j .. 4j+3 in code[j]
    int ntx;           // column tiles per stripe
    int ntiles;        // column tiles x stripes
};

// Persistent over tiles t = blockIdx.x + i * gridDim.x (column tile t % ntx of
// stripe t / ntx).  Iteration i runs phases 2 and 3 of tile t_(i-1) and phase
// 1 of tile t_i:
//   early phase 1 of t_i (waves >= 8, registers only) || phase 2 of t_(i-1)
//   (waves < 8) -> Y into the image -> phase-3 waves read their rows ->
//   barrier (image free) -> early units into the image; phase 3 of t_(i-1);
//   late phase-1 units of t_i -> barrier (u of t_i in the image).
template <bool STRIDED>
__global__ void __launch_bounds__(64 * kWaves, kWaves / 4) k_rec_bs256(RecArgs a, DecPlan pl) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[kImgRows * kTile / 4];
    Dec<STRIDED> d;
    d.ap = (cargs_t *)__builtin_amdgcn_kernarg_segment_ptr();
    d.lds0 = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) uint32_t *)lds;
    d.w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int w = d.w;
    const uint64_t cw = w < 4 ? pl.code[0] : w < 8 ? pl.code[1] : pl.code[2];
    const uint32_t code = (uint32_t)(cw >> (16 * (w & 3))) & 0xFFFFu;
    const int u3a = (int)(code & 15u) - 1, u3b = (int)((code >> 4) & 15u) - 1;
    const int u1a = (int)((code >> 8) & 15u) - 1, u1b = (int)((code >> 12) & 15u) - 1;
    const bool early = w >= 8;
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
    for (;;) {
        const bool cur = t >= 0, more = tn < pl.ntiles;
        // The first iteration has no phase 2 / 3: every wave is free, so
        // wave w takes phase-1 unit w (one each) instead of the plan's split.
        const bool first = t < 0;
        const int p1a = first ? (w < kUnits ? w : -1) : u1a, p1b = first ? -1 : u1b;
        const bool early_p1 = early && more && p1a >= 0;  // passes phase 2's barriers inside its first unit
        // The last iteration has no phase 1: waves 8.. take the second phase-3
        // units of waves 0.. (so every phase-3 unit runs on a wave of its own).
        int p3a = u3a, p3b = u3b;
        bool pre = false;  // a late wave's phase-1 rows already in flight (lab bit 8)
        if (!more) {
            if (early) {
                p3a = (int)((uint32_t)(pl.code[0] >> (16 * (w - 8))) >> 4 & 15u) - 1;
                p3b = -1;
            } else if (w + 8 < kWaves) {
                p3b = -1;
            }
        }
        // Two slots, one copy of the phase-1 code: slot 0 runs the early
        // waves' phase 1 of tile tn (before phase 2), slot 1 phases 2 and 3 of
        // tile t and then the late waves' phase 1 of tile tn.  Two call sites
        // of phase1() put its code (scale-in, IFFT layers 0-3 of every unit)
        // into the kernel twice: 112 KB against a 64 KB instruction cache
        // (one instruction-cache-sized build measured 9 % faster).
#pragma nounroll
        for (int slot = 0; slot < 2; slot++) {
            if (slot == 1 && cur) {
                // ---- phase 2: Y = B_F (I + H) B_I u + Lo u (B layout)
                if (!early)
                    d.phase2();
                if (!early_p1) lds_barrier();  // every wave has read u
                if (!early) {
                    int wt = w;
                    asm volatile("" : "+s"(wt));
#pragma unroll
                    for (int q = 0; q < Dec<STRIDED>::NQ; q++) d.img_put(2 * wt + 16 * q, d.V[q]);
                    // lab bit 8: a late wave with no phase-3 unit issues its phase-1
                    // unit's row loads now, so they are in flight across the Y barrier
                    if ((d.args().lab & 8) && more && p1a >= 0 && p3a < 0 && 16 * p1a < d.args().mtrunc) {
                        set_tile(tn);
                        d.template load_rows<8>(p1a);
                        pre = true;
                    }
                }
                if (!early_p1) lds_barrier();  // Y is in the image
                if (p3a >= 0) {
                    // ---- phase 3 of tile t, one unit at a time (each read from the
                    // image before the barrier below frees it)
                    set_tile(t);
                    const int n3 = p3b >= 0 ? 2 : 1;
#pragma nounroll
                    for (int s = 0; s < n3; s++) {
                        const int u = s ? p3b : p3a;
                        d.template unit_get<0>(u);
                        d.phase3(u);
                    }
                }
            }
            // ---- phase 1 of tile tn (registers only): the early waves in slot 0,
            // a first unit parked in V[8..15]; the late waves in slot 1
            const bool run_p1 = slot == 0 ? early_p1 : !early && more && p1a >= 0;
            if (run_p1) {
                // The early waves' chain is the critical path: it issues ahead of
                // the phase-2 / phase-3 waves sharing its SIMD (C4 x 16 1692 ->
                // 1637 us, one stripe 124 -> 121 us; raising the phase-3 waves too
                // gained nothing, profiles/r03_c4_prio_ab.txt).
                const int lab = d.args().lab;
                if (slot == 0) __builtin_amdgcn_s_setprio(3);
                else if (lab & 4) __builtin_amdgcn_s_setprio(1);
                set_tile(tn);
                const int n1 = slot == 0 && p1b >= 0 ? 2 : 1;
                // (loading unit b's rows into V[8..15] up front measured slower:
                // 1950 vs 1694 us per 16 C4 stripes)
#pragma nounroll
                for (int s = 0; s < n1; s++) {
                    if (s) {
                        d.park_swap();
                        // lab: an early wave's second unit is off the critical path
                        // (the early waves wait at the image-free barrier): drop its priority
                        if (lab & 1) __builtin_amdgcn_s_setprio(0);
                        else if (lab & 2) __builtin_amdgcn_s_setprio(1);
                    }
                    d.phase1(s ? p1b : p1a, slot == 0 && s == 0 && cur ? 2 : 0, slot == 1 && pre);
                }
                __builtin_amdgcn_s_setprio(0);
            }
        }
        if (!more) break;
        lds_barrier();  // the image is free for phase 1 of tile tn
        if (p1a >= 0) {
            if (early) {
                d.template unit_put<0>(p1b >= 0 ? p1b : p1a);
                if (p1b >= 0) d.template unit_put<8>(p1a);
            } else {
                d.template unit_put<0>(p1a);
            }
        }
        lds_barrier();  // u of tile tn is in the image
        t = tn;
        tn += gridDim.x;
    }
}

// Unit placement (see DecPlan).  VALU cost: a phase-1 unit 2, a phase-3 unit
// 1; phase 2 and the exchange cost the waves < 8 about 2 before their phase 3
// / late phase 1 starts, while the early waves' phase-1 units overlap it.  So
// the early waves take two phase-1 units each first, the rest of phase 1 goes
// one unit per wave to waves < 8 from the top (7, 6, ...), and the phase-3
// units go round-robin, at most two per wave (run one after the other), to
// the waves < 8 without phase 1: about 4 per wave everywhere at C4.
// Wave w runs on SIMD w & 3: waves 8-11 land one per SIMD.
DecPlan make_plan(const RecArgs &a) {
    // phase 1 writes every image row: units past mtrunc write zeros (Dec::phase1)
    const int G = kUnits;
    uint32_t rmask = 0;  // units with revealed rows
    for (int u = 0; u < G; u++)
        if ((a.need[u >> 1] >> (16 * (u & 1))) & 0xFFFFu) rmask |= 1u << u;
    static std::mutex mu;
    static std::map<uint32_t, DecPlan> cache;
    const uint32_t key = (uint32_t)a.mtrunc << 16 | rmask;  // the costs depend on which units lie past mtrunc
    {
        std::lock_guard<std::mutex> lk(mu);
        auto it = cache.find(key);
        if (it != cache.end()) return it->second;
    }
    // Cost model (cycles per tile, from per-wave s_memtime stamps of lab builds at C4, scripts/lab): a phase-1
    // unit 27 k (a unit past mtrunc only writes zeros: 1 k), a phase-3 unit
    // 14 k, phase 2 plus the exchange 17 k before a wave < 8 starts its units;
    // the early waves start at once.  E phase-1 units go to the early waves
    // (at most two each), the rest one per wave < 8 from wave 7 down, and the
    // phase-3 units one by one to the cheapest wave < 8 (at most two each);
    // the E with the smallest maximum wins (ties: the larger E).  C4 with 32
    // erasures (ten phase-3 units) gets E = 8; few-erasure repairs get E = 4,
    // spreading phase 1 over the waves phase 3 leaves idle.
    const int ne = kWaves - 8;
    auto c1 = [&](int uu) { return 16 * uu < a.mtrunc ? 27 : 1; };
    int u1[kWaves][2], u3[kWaves][2];
    int best = INT_MAX;
    for (int E = std::min(G, 2 * ne); E >= 0; E--) {
        if (G - E > 8) break;
        int t1[kWaves][2], t3[kWaves][2], cost[kWaves] = {0};
        for (int w = 0; w < kWaves; w++) t1[w][0] = t1[w][1] = t3[w][0] = t3[w][1] = -1;
        for (int i = 0; i < E; i++) {
            t1[8 + i % ne][i / ne] = i;
            cost[8 + i % ne] += c1(i);
        }
        for (int w = 0; w < 8; w++) cost[w] = 17;
        for (int i = E, w = 7; i < G; i++, w--) {
            t1[w][0] = i;
            cost[w] += c1(i);
        }
        bool ok = true;
        for (int g = 0; g < G && ok; g++) {
            if (!((rmask >> g) & 1)) continue;
            int bw = -1;
            for (int w = 0; w < 8; w++)
                if (t3[w][1] < 0 && (bw < 0 || cost[w] < cost[bw])) bw = w;
            if (bw < 0) {
                ok = false;
                break;
            }
            t3[bw][t3[bw][0] < 0 ? 0 : 1] = g;
            cost[bw] += 14;
        }
        if (!ok) continue;
        int mx = 0;
        for (int w = 0; w < kWaves; w++) mx = std::max(mx, cost[w]);
        if (mx < best) {
            best = mx;
            std::memcpy(u1, t1, sizeof u1);
            std::memcpy(u3, t3, sizeof u3);
        }
    }
    if (best == INT_MAX) {  // cannot happen for G <= 10 units
        DecPlan bad{};
        bad.ntiles = -1;
        return bad;
    }
    DecPlan bp{};
    for (int w = 0; w < kWaves; w++) {
        const uint64_t c = (uint64_t)(u3[w][0] + 1) | (uint64_t)(u3[w][1] + 1) << 4 | (uint64_t)(u1[w][0] + 1) << 8 |
                           (uint64_t)(u1[w][1] + 1) << 12;
        bp.code[w >> 2] |= c << (16 * (w & 3));
    }
    std::lock_guard<std::mutex> lk(mu);
    cache[key] = bp;
    return bp;
}

}  // namespace

extern "C" int rs_debug_dec_plan(int mtrunc, const uint32_t *need, uint64_t *code) {
    if (mtrunc < 1 || mtrunc > kImgRows || !need || !code) return -1;
    RecArgs a{};
    a.mtrunc = mtrunc;
    for (int k = 0; k < 8; k++) a.need[k] = need[k];
    const DecPlan pl = make_plan(a);
    if (pl.ntiles < 0) return -1;
    for (int j = 0; j < 3; j++) code[j] = pl.code[j];
    return 0;
}

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
    if (pl.ntiles < 0) return hipErrorNotSupported;  // cannot happen for mtrunc <= kImgRows
    pl.ntx = (int)((a.S + kTile - 1) / kTile);
    const uint64_t ny = a.base && a.nstripes > 1 ? (uint64_t)a.nstripes : 1;
    if ((uint64_t)pl.ntx * ny > (uint64_t)INT32_MAX) return hipErrorInvalidValue;
    pl.ntiles = (int)(pl.ntx * ny);
    const unsigned grid = (unsigned)std::min<int>(pl.ntiles, std::max(cus, 1));
    if (a.base) hipLaunchKernelGGL(k_rec_bs256<true>, dim3(grid), dim3(64 * kWaves), 0, s, a, pl);
    else hipLaunchKernelGGL(k_rec_bs256<false>, dim3(grid), dim3(64 * kWaves), 0, s, a, pl);
    return hipGetLastError();
}

}  // namespace rs
