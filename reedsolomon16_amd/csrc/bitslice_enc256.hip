// Bit-sliced GF(2^16) encode for m = 256 (gfx950): k_enc_bs256, the C5 path
// (1024 data + 256 parity; any k <= 1024 with 129 <= p <= 256).
//
// Reference: encode leopard16.go:128-224 -- four chunk IFFTs
// (ifftDITEncoder :685-747, skewLUT = fftSkew[(c+1)m - 1:]) XOR-accumulated,
// then fftDIT (:618-657) over fftSkew, rows < p stored.
//
// Why this shape.  The byte-permute LDS kernel (kernels.hip k_enc_lds) is
// VALU-bound: every product costs ~6 VALU per symbol.  In
// subfield coordinates (gf_host.hpp SubCoords) a product by a twiddle in
// GF(2^8) is a fixed XOR network over 8 bit-planes, ~0.7 VALU per symbol.
// With raw twiddle values (Cantor coordinates) the encoder's layer-L twiddle
// of chunk c, group g is the element 2 (g + (c+1) (128 >> L)): it lies in the
// subfield for every FFT butterfly and every chunk butterfly of layers >= 3
// (layer 2 for c < 3); layers 0 and 1 (2 for c = 3) are full-field.
//
// A plane-form lane cannot own a row pair of layer 0 or 1 together with
// uniform twiddles (the 512-byte tile leaves only 8 blocks for 64 lanes), so
// those layers run in byte form, where a lane holds 8 bytes of a row and every
// row of the wave's 32-row unit: products by runtime tables (v_perm_b32, tables
// in SGPRs; bitslice_dec.hip uses the same for its layer 0).  Everything else
// is bit-sliced.
//
// Tile: 512 bytes of columns (8 blocks) of every row of one stripe; one
// 8-wave workgroup per CU (128 KB LDS exchange image), persistent over tiles.
//   byte form (BF): wave w = row bits 5-7, registers t = row bits 0-4 (32 rows
//     x 2 dwords).  Lane l: bit 0 = dq0, bits 1-3 = block, bit 4 = dq1, bit 5 =
//     p: the lane holds bytes [block*64 + p*32 + (2 dq1 + dq0)*8, +8) of each
//     row (p = 0: low bytes, 1: high bytes of 8 symbols).  "Paired" (one
//     permlane32 swap per row): lane bit 5 = symbol quad, dwords = (lo, hi).
//   planes (P1): lane bit 0 = row bit 0, bit 4 = row bit 1, bit 5 = subfield
//     half h; registers i = row bits 2-4 (8 rows x 8 planes); wave = rows 5-7.
//   planes (P2): registers = row bits 5-7, wave = row bits 2-4 (the LDS
//     exchange transposes wave and register indices; each wave access is 1 KB
//     contiguous).
//
// Per chunk: 32 row loads (prefetched during the previous chunk), pair, BF
// IFFT layers 0, 1 (2 for c = 3), coordinate change, unpair, BF -> P1
// (permlane16 swap, DPP swap, bit transpose), IFFT layers 2-4 (networks chosen
// by chunk and wave), exchange, layers 5-7, XOR into the accumulator (P2).
// Then the FFT: layers 7-5 (P2), exchange, layers 4-2 (P1), P1 -> BF, BF
// layers 1, 0, coordinate change back, stores of rows < p.
#include <algorithm>
#include <atomic>

#include "bs_common.hpp"
#include "bs_tables.h"
#include "gf_host.hpp"
#include "kernels.hpp"
#include "schedule.hpp"

namespace rs {
namespace {
using namespace bs;

typedef EncTab256 ET;
typedef DecTab256 DT;
constexpr int kTile = 512;  // column bytes per tile
constexpr int kWaves = 8;
constexpr int kTw16 = 24, kTw8 = 8;
constexpr int kBfTabs = 224;  // byte-form IFFT tables per chunk: layer 0 (128 groups), 1 (64), 2 (32)
constexpr uint32_t kMod = 65535;
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(4))) const E256Args cargs_t;

constexpr uint64_t pack8(const uint8_t (&m)[8]) {
    uint64_t r = 0;
    for (int k = 0; k < 8; k++) r |= (uint64_t)m[k] << (8 * k);
    return r;
}

// ---- compile-time binary dispatch (log2 N scalar compares)
template <int LO, int HI, class Fn>
__device__ __forceinline__ void bdispatch(int role, Fn &&f) {
    if constexpr (HI - LO == 1) {
        f(ic<LO>{});
    } else {
        constexpr int MID = (LO + HI) / 2;
        if (role < MID) bdispatch<LO, MID>(role, f);
        else bdispatch<MID, HI>(role, f);
    }
}

// x ^= y * table (subfield table, one dword of c0 or c1 bytes)
template <class T>
__device__ __forceinline__ void mul8_add1(uint32_t &x, uint32_t v, const T &t) {
    x = xor3v(x ^ perm(t[1], t[0], v & 0x07070707u), perm(t[3], t[2], (v >> 3) & 0x07070707u),
              perm(t[4], t[4], (v >> 6) & 0x03030303u));
}

// lane bit 0 <-> the register pair (a, b): a holds the bit-0 = 0 element, b the bit-0 = 1 one
__device__ __forceinline__ void swap_lb0(uint32_t &a, uint32_t &b, bool odd) {
    const uint32_t pa = __builtin_amdgcn_mov_dpp(a, 0xB1, 0xF, 0xF, false);  // quad_perm [1,0,3,2]: lane ^ 1
    const uint32_t pb = __builtin_amdgcn_mov_dpp(b, 0xB1, 0xF, 0xF, false);
    const uint32_t na = odd ? pb : a, nb = odd ? b : pa;
    a = na;
    b = nb;
}

struct Enc256 {
    cargs_t *ap;
    int w;
    uint32_t lds0;
    // BF row t (0..31) dword s at V[t >> 2][(t & 3) * 2 + s]; P1/P2: V[i] = 8 planes of register row i
    uint32_t V[8][8];
    uint32_t A[8][8];   // accumulator, P2
    uint32_t St[4][8];  // rows 0-15 of the next chunk as loaded (BF layout)

    __device__ __forceinline__ cargs_t &args() const {
        cargs_t *p = ap;
        asm volatile("" : "+s"(p));
        return *p;
    }
    __device__ __forceinline__ uint32_t lane() const {
        uint32_t t = __builtin_amdgcn_workitem_id_x();
        asm volatile("" : "+v"(t));
        return t & 63u;
    }
    // lane byte offset within the tile's row piece
    __device__ __forceinline__ uint32_t lane_off() const {
        const uint32_t l = lane();
        return ((l >> 1) & 7u) * 64u + (l >> 5) * 32u + ((((l >> 4) & 1u) << 1) | (l & 1u)) * 8u;
    }
    __device__ __forceinline__ uint32_t &bf(uint32_t (&R)[8][8], int t, int s) { return R[t >> 2][(t & 3) * 2 + s]; }

    struct Loc {
        int stripe, ct;
        bool live;
    };
    __device__ __forceinline__ Loc locate(int tile) const {
        cargs_t &a = args();
        const int tps = a.tiles_per_stripe;
        const int stripe = tile / tps;
        return Loc{stripe, tile - stripe * tps, tile < a.ntiles};
    }

    // rows c*256 + 32w + t, t in [T0, T0 + 16), of tile L into R (BF layout,
    // R's row t - R0); rows >= k and tiles past the end read zero
    template <int T0, int R0, int NR>
    __device__ __forceinline__ void stage(uint32_t (&R)[NR][8], const Loc &L, int c) {
        cargs_t &a = args();
        const uint32_t range = L.live ? a.span : 0u;
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            (void *)(a.data + (L.live ? (uint64_t)L.stripe * a.stripe_stride : 0)), 0, (int)range, 0x00020000);
        uint32_t voff = (uint32_t)L.ct * kTile + lane_off();
        asm volatile("" : "+v"(voff));
        const uint32_t rs0 = (uint32_t)a.row_stride;
        __builtin_amdgcn_s_setprio(2);
#pragma unroll
        for (int t = T0; t < T0 + 16; t++) {
            const uint32_t soff = (uint32_t)(256 * c + 32 * w + t) * rs0;
            const u32x2 x = __builtin_amdgcn_raw_buffer_load_b64(rs, voff, soff, 0);
            R[(t - R0) >> 2][((t - R0) & 3) * 2 + 0] = x[0];
            R[(t - R0) >> 2][((t - R0) & 3) * 2 + 1] = x[1];
        }
        __builtin_amdgcn_s_setprio(0);
    }

    // ---------------- byte form
    // lane bit 5 (p / symbol quad) <-> dword index (s) of each row
    template <int T0, int NT = 16>
    __device__ __forceinline__ void pair_rows() {
#pragma unroll
        for (int t = T0; t < T0 + NT; t++) swap32(bf(V, t, 0), bf(V, t, 1));
    }
    // IFFT layer L (0..2) in byte form on rows [T0, T0 + 16), paired (lo, hi):
    // y ^= x; x ^= y * t.  Rows (base + j, base + j + 2^L); group g = (32 w + base) >> (L + 1).
    template <int L, int T0>
    __device__ __forceinline__ void bf_ifft(int c) {
        cargs_t &a = args();
        constexpr int s = 1 << L, off = L == 0 ? 0 : L == 1 ? 128 : 192;
        constexpr int NG = 8 >> L;  // groups in the 16 rows
        cu32_t *tw = ctab(a.tw_bf) + ((uint64_t)c * kBfTabs + off + (uint64_t)w * (16 >> L) + (T0 >> (L + 1))) * kTw16;
        Tab<20> cur = tab_at<20>(tw);
        sfor<NG>([&](auto G) __attribute__((always_inline)) {
            constexpr int gi = decltype(G)::value, base = T0 + gi * 2 * s;
            Tab<20> nxt;
            if constexpr (gi + 1 < NG) nxt = tab_at<20>(tw + (gi + 1) * kTw16);
            sfor<s>([&](auto J) __attribute__((always_inline)) {
                constexpr int x = base + decltype(J)::value, y = x + s;
                bf(V, y, 0) ^= bf(V, x, 0);
                bf(V, y, 1) ^= bf(V, x, 1);
                mul16_add1(bf(V, x, 0), bf(V, x, 1), bf(V, y, 0), bf(V, y, 1), cur);
            });
            asm volatile("" ::: "memory");
            if constexpr (gi + 1 < NG) cur = nxt;
            __builtin_amdgcn_sched_barrier(0);
        });
    }
    // FFT layer L (1, 0) in byte form on rows [T0, T0 + 16), unpaired, subfield
    // coordinates: x ^= y * t; y ^= x
    template <int L, int T0>
    __device__ __forceinline__ void bf_fft() {
        cargs_t &a = args();
        constexpr int s = 1 << L, off = L == 0 ? 0 : 128;
        constexpr int NG = 8 >> L;
        cu32_t *tw = ctab(a.tw_bf_fft) + (off + (uint64_t)w * (16 >> L) + (T0 >> (L + 1))) * kTw8;
        Tab<5> cur = tab_at<5>(tw);
        sfor<NG>([&](auto G) __attribute__((always_inline)) {
            constexpr int gi = decltype(G)::value, base = T0 + gi * 2 * s;
            Tab<5> nxt;
            if constexpr (gi + 1 < NG) nxt = tab_at<5>(tw + (gi + 1) * kTw8);
            sfor<s>([&](auto J) __attribute__((always_inline)) {
                constexpr int x = base + decltype(J)::value, y = x + s;
#pragma unroll
                for (int d = 0; d < 2; d++) {
                    mul8_add1(bf(V, x, d), bf(V, y, d), cur);
                    bf(V, y, d) ^= bf(V, x, d);
                }
            });
            asm volatile("" ::: "memory");
            if constexpr (gi + 1 < NG) cur = nxt;
            __builtin_amdgcn_sched_barrier(0);
        });
    }
    // paired rows: lo ^= D(hi) (to / from subfield coordinates; an involution)
    template <int T0, int NT = 16>
    __device__ __forceinline__ void psi_rows(const Tab<5> &dt) {
#pragma unroll
        for (int t = T0; t < T0 + NT; t++) mul8_add1(bf(V, t, 0), bf(V, t, 1), dt);
    }
    // unpaired BF <-> P1 for register rows [I0, I0 + 4) (BF rows 4 I0 ..)
    template <int I0>
    __device__ __forceinline__ void bf_to_p1() {
        const bool odd = lane() & 1u;
#pragma unroll
        for (int i = I0; i < I0 + 4; i++) {
            // lane bit 4 (dq1) <-> row bit 1: rows 4i + z, 4i + z + 2
#pragma unroll
            for (int z = 0; z < 2; z++)
#pragma unroll
                for (int s = 0; s < 2; s++) swap16(V[i][z * 2 + s], V[i][(z + 2) * 2 + s]);
            // lane bit 0 (dq0) <-> row bit 0: rows 4i + 2q, 4i + 2q + 1
#pragma unroll
            for (int q = 0; q < 2; q++)
#pragma unroll
                for (int s = 0; s < 2; s++) swap_lb0(V[i][(2 * q) * 2 + s], V[i][(2 * q + 1) * 2 + s], odd);
            bs_transpose8(V[i]);
            __builtin_amdgcn_sched_barrier(0);
        }
    }
    template <int I0>
    __device__ __forceinline__ void p1_to_bf() {
        const bool odd = lane() & 1u;
#pragma unroll
        for (int i = I0; i < I0 + 4; i++) {
            bs_transpose8(V[i]);
#pragma unroll
            for (int q = 0; q < 2; q++)
#pragma unroll
                for (int s = 0; s < 2; s++) swap_lb0(V[i][(2 * q) * 2 + s], V[i][(2 * q + 1) * 2 + s], odd);
#pragma unroll
            for (int z = 0; z < 2; z++)
#pragma unroll
                for (int s = 0; s < 2; s++) swap16(V[i][z * 2 + s], V[i][(z + 2) * 2 + s]);
            __builtin_amdgcn_sched_barrier(0);
        }
    }

    // ---------------- plane form: networks
    // x ^= M y (M: 8 rows of input-plane masks packed a byte each), written to fresh registers
    template <uint64_t M>
    __device__ __forceinline__ void net(Half &x, const Half &y) {
        Half nx;
        net_to<M>(nx, x, y);
#pragma unroll
        for (int k = 0; k < 8; k++) x[k] = nx[k];
    }
    // nx = x ^ M y
    template <uint64_t M>
    __device__ __forceinline__ static void net_to(Half &nx, const Half &x, const Half &y) {
        sfor<8>([&](auto K) __attribute__((always_inline)) {
            constexpr int k = decltype(K)::value;
            xor_net8f<(uint32_t)((M >> (8 * k)) & 0xFFu)>(nx[k], x[k], y);
        });
    }
    // IFFT layers 2-4 in P1 (register rows i = row bits 2-4, wave = row bits 5-7):
    // the network of each butterfly is chosen by (chunk, wave) -- a wave-uniform
    // branch around the network alone, whose result goes to fresh registers (a
    // branch around whole layers made the allocator keep two copies of the rows)
    __device__ __forceinline__ void ifft_p1(int c) {
        const int cw = c * kWaves + w;
        sfor<3>([&](auto LI) __attribute__((always_inline)) {
            constexpr int L = 2 + decltype(LI)::value, s = 1 << (L - 2);
            if (L == 2 && c == 3) return;  // c = 3, layer 2: full-field, done in byte form
            sfor<4>([&](auto Q) __attribute__((always_inline)) {
                constexpr int q = decltype(Q)::value;
                constexpr int i = ((q >> (L - 2)) << (L - 1)) | (q & (s - 1));
                xor8(V[i + s], V[i]);
                Half nx;
                bdispatch<0, 4 * kWaves>(cw, [&](auto CW) __attribute__((always_inline)) {
                    constexpr int C = decltype(CW)::value / kWaves, W = decltype(CW)::value % kWaves;
                    constexpr int g = (32 * W + 4 * i) >> (L + 1);
                    net_to<pack8(ET::m8[C][L][g])>(nx, V[i], V[i + s]);
                });
#pragma unroll
                for (int k = 0; k < 8; k++) V[i][k] = nx[k];
                __builtin_amdgcn_sched_barrier(0);
            });
        });
    }
    // IFFT layers 5-7 in P2 (register rows i = row bits 5-7): networks chosen by chunk
    __device__ __forceinline__ void ifft_p2(int c) {
        sfor<3>([&](auto LI) __attribute__((always_inline)) {
            constexpr int L = 5 + decltype(LI)::value, s = 1 << (L - 5);
            sfor<4>([&](auto Q) __attribute__((always_inline)) {
                constexpr int q = decltype(Q)::value;
                constexpr int i = ((q >> (L - 5)) << (L - 4)) | (q & (s - 1));
                constexpr int g = (32 * i) >> (L + 1);
                xor8(V[i + s], V[i]);
                Half nx;
                bdispatch<0, 4>(c, [&](auto C) __attribute__((always_inline)) {
                    net_to<pack8(ET::m8[decltype(C)::value][L][g])>(nx, V[i], V[i + s]);
                });
#pragma unroll
                for (int k = 0; k < 8; k++) V[i][k] = nx[k];
                __builtin_amdgcn_sched_barrier(0);
            });
        });
    }
    // FFT layers 7-5 on the accumulator (P2): x ^= M y; y ^= x
    __device__ __forceinline__ void fft_p2() {
        sfor<3>([&](auto LI) __attribute__((always_inline)) {
            constexpr int L = 7 - decltype(LI)::value, s = 1 << (L - 5);
            sfor<4>([&](auto Q) __attribute__((always_inline)) {
                constexpr int q = decltype(Q)::value;
                constexpr int i = ((q >> (L - 5)) << (L - 4)) | (q & (s - 1));
                constexpr int g = (32 * i) >> (L + 1);
                if constexpr (DT::logs[L][g] != kMod) net<pack8(DT::m8[L][g])>(A[i], A[i + s]);
                xor8(A[i + s], A[i]);
                __builtin_amdgcn_sched_barrier(0);
            });
        });
    }
    // FFT layers 4-2 in P1: networks chosen by wave
    __device__ __forceinline__ void fft_p1() {
        sfor<3>([&](auto LI) __attribute__((always_inline)) {
            constexpr int L = 4 - decltype(LI)::value, s = 1 << (L - 2);
            sfor<4>([&](auto Q) __attribute__((always_inline)) {
                constexpr int q = decltype(Q)::value;
                constexpr int i = ((q >> (L - 2)) << (L - 1)) | (q & (s - 1));
                Half nx;
                bdispatch<0, kWaves>(w, [&](auto W) __attribute__((always_inline)) {
                    constexpr int g = (32 * decltype(W)::value + 4 * i) >> (L + 1);
                    net_to<pack8(DT::m8[L][g])>(nx, V[i], V[i + s]);  // a zero twiddle's matrix is zero: nx = x
                });
#pragma unroll
                for (int k = 0; k < 8; k++) V[i][k] = nx[k];
                xor8(V[i + s], V[i]);
                __builtin_amdgcn_sched_barrier(0);
            });
        });
    }

    // ---------------- LDS exchange: writer (wave w, register i) at slot 8w + i,
    // reader (wave w, register i) from slot 8i + w; 2 KB per slot (two plane quads)
    __device__ __forceinline__ uint32_t slot_addr(int slot, int q) const {
        uint32_t b = lds0 + lane() * 16u;
        asm volatile("" : "+v"(b));
        return b + (uint32_t)(slot * 2 + q) * 1024u;
    }
    __device__ __forceinline__ void exchange(uint32_t (&src)[8][8], uint32_t (&dst)[8][8]) {
        lds_barrier();  // every wave has read the previous exchange
#pragma unroll
        for (int i = 0; i < 8; i++) {
            const Half &v = src[i];
            *(lds_u4 *)(uintptr_t)slot_addr(8 * w + i, 0) = u32x4{v[0], v[1], v[2], v[3]};
            *(lds_u4 *)(uintptr_t)slot_addr(8 * w + i, 1) = u32x4{v[4], v[5], v[6], v[7]};
        }
        lds_barrier();
#pragma unroll
        for (int i = 0; i < 8; i++) {
            const u32x4 x = *(const lds_u4 *)(uintptr_t)slot_addr(8 * i + w, 0);
            const u32x4 y = *(const lds_u4 *)(uintptr_t)slot_addr(8 * i + w, 1);
            Half &v = dst[i];
            v[0] = x[0], v[1] = x[1], v[2] = x[2], v[3] = x[3];
            v[4] = y[0], v[5] = y[1], v[6] = y[2], v[7] = y[3];
        }
    }

    // ---------------- one chunk: St (rows 0-15) + rows 16-31 -> IFFT -> accumulator
    // Rows 16-31 of the chunk are loaded at its start, straight into V, and
    // stay in flight while rows 0-15 go through the byte-form layers; only
    // rows 0-15 of the next chunk are prefetched (V + A + St = 160 VGPRs).
    template <int T0>
    __device__ __forceinline__ void bf_half(int c) {
        pair_rows<T0>();
        bf_ifft<0, T0>(c);
        bf_ifft<1, T0>(c);
        if (c == 3) bf_ifft<2, T0>(c);
        psi_rows<T0>(tab_at<5>(ctab(args().dmap)));
        pair_rows<T0>();  // unpair
        bf_to_p1<T0 / 4>();
    }
    __device__ __forceinline__ void chunk(int c, const Loc &cur, const Loc &nxt, int nch) {
#pragma unroll
        for (int i = 0; i < 4; i++)
#pragma unroll
            for (int k = 0; k < 8; k++) V[i][k] = St[i][k];
        __builtin_amdgcn_sched_barrier(0);
        stage<16, 0>(V, cur, c);
        {
            const bool more = c + 1 < nch;  // wave-uniform
            stage<0, 0>(St, more ? cur : nxt, more ? c + 1 : 0);
        }
        __builtin_amdgcn_sched_barrier(0);
        bf_half<0>(c);
        bf_half<16>(c);
        ifft_p1(c);
        exchange(V, V);
        ifft_p2(c);
        if (c == 0) {
#pragma unroll
            for (int i = 0; i < 8; i++)
#pragma unroll
                for (int k = 0; k < 8; k++) A[i][k] = V[i][k];
        } else {
#pragma unroll
            for (int i = 0; i < 8; i++) xor8(A[i], V[i]);
        }
        __builtin_amdgcn_sched_barrier(0);
    }

    template <bool VERIFY>
    __device__ __forceinline__ void finish(const Loc &cur) {
        fft_p2();
        exchange(A, V);
        fft_p1();
        p1_to_bf<0>();
        p1_to_bf<4>();
        bf_fft<1, 0>();
        bf_fft<1, 16>();
        bf_fft<0, 0>();
        bf_fft<0, 16>();
        pair_rows<0, 32>();
        psi_rows<0, 32>(tab_at<5>(ctab(args().dmap)));
        pair_rows<0, 32>();
        cargs_t &a = args();
        const uint32_t col = (uint32_t)cur.ct * kTile + lane_off();
        const __amdgpu_buffer_rsrc_t ps = __builtin_amdgcn_make_buffer_rsrc(
            (void *)(a.parity + (uint64_t)cur.stripe * a.stripe_stride), 0, (int)a.pspan, 0x00020000);
        uint32_t voff = col;
        asm volatile("" : "+v"(voff));
        const int p = a.p;
        const uint32_t rs0 = (uint32_t)a.row_stride;
        uint32_t bad = 0;
        if (col < a.S) {
#pragma unroll
            for (int t = 0; t < 32; t++) {
                const int row = 32 * w + t;
                if (row >= p) break;  // wave-uniform
                const u32x2 v = u32x2{bf(V, t, 0), bf(V, t, 1)};
                if constexpr (VERIFY) {
                    const u32x2 old = __builtin_amdgcn_raw_buffer_load_b64(ps, voff, (uint32_t)row * rs0, 0);
                    bad |= (old[0] ^ v[0]) | (old[1] ^ v[1]);
                } else {
                    __builtin_amdgcn_raw_buffer_store_b64(v, ps, voff, (uint32_t)row * rs0, 0);
                }
            }
        }
        if constexpr (VERIFY) {
            const uint64_t m = __ballot(bad != 0);
            if (m && lane() == (uint32_t)(__ffsll((unsigned long long)m) - 1) &&
                __hip_atomic_load(a.mismatch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0)
                __hip_atomic_store(a.mismatch, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
};

template <bool VERIFY>
__global__ void __launch_bounds__(64 * kWaves, 1) k_enc_bs256(E256Args a) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[kWaves * 8 * 2 * 256];  // 128 slots x 1 KB
    Enc256 e;
    e.ap = (cargs_t *)__builtin_amdgcn_kernarg_segment_ptr();
    e.w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    e.lds0 = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) uint32_t *)lds;
    int tile = blockIdx.x;
    const int ntiles = e.args().ntiles, nch = e.args().nch;
    if (tile >= ntiles) return;
    Enc256::Loc cur = e.locate(tile);
    e.stage<0, 0>(e.St, cur, 0);
    for (; tile < ntiles; tile += gridDim.x) {
        const Enc256::Loc nxt = e.locate(tile + (int)gridDim.x);
#pragma nounroll
        for (int c = 0; c < nch; c++) e.chunk(c, cur, nxt, nch);
        e.template finish<VERIFY>(cur);
        cur = nxt;
    }
}

}  // namespace

bool encode_bs256_available(int k, int p, const uint32_t *ifft_logs, const uint32_t *fft_logs, uint32_t mod) {
    if (k < 1 || p < 129 || p > 256) return false;
    const int nch = (k + 255) / 256;
    if (nch > ET::NCH) return false;
    const int is = ifft_slots(8);
    // the compiled networks (layers >= 2) against the geometry's own schedule
    for (int c = 0; c < nch; c++)
        for (int L = 2; L < 8; L++)
            for (int g = 0; g < (128 >> L); g++) {
                const uint32_t l = ifft_logs[(size_t)c * is + ifft_slot(8, L, g * (2 << L))];
                if (l != mod && l != ET::logs[c][L][g]) return false;
            }
    for (int L = 2; L < 8; L++)
        for (int g = 0; g < (128 >> L); g++) {
            const uint32_t l = fft_logs[fft_slot(8, L, g * (2 << L))];
            if (l != mod && l != DT::logs[L][g]) return false;
        }
    return true;
}

bool encode_bs256_fits(int k, uint64_t row_stride, uint64_t S) {
    const uint64_t rows = (uint64_t)(k + 255) / 256 * 256;   // the last chunk's padding rows are addressed too
    const uint64_t cols = (S + kTile - 1) / kTile * kTile;  // lanes of the last tile past the row end
    return k >= 1 && (rows - 1) * row_stride + cols < (1ull << 32);
}

hipError_t launch_encode_bs256(bool verify, E256Args a, int cus, hipStream_t s) {
    if (a.k < 1 || a.p < 129 || a.p > 256 || a.nch < 1 || a.nch > ET::NCH) return hipErrorNotSupported;
    if (!encode_bs256_fits(a.k, a.row_stride, a.S)) return hipErrorNotSupported;
    a.tiles_per_stripe = (int)((a.S + kTile - 1) / kTile);
    a.ntiles = a.tiles_per_stripe * a.nstripes;
    a.span = (uint32_t)((uint64_t)(a.k - 1) * a.row_stride + a.S);
    a.pspan = (uint32_t)((uint64_t)(a.p - 1) * a.row_stride + a.S);
    const int grid = std::min(a.ntiles, std::max(cus, 1));
    if (verify) hipLaunchKernelGGL(k_enc_bs256<true>, dim3(grid), dim3(64 * kWaves), 0, s, a);
    else hipLaunchKernelGGL(k_enc_bs256<false>, dim3(grid), dim3(64 * kWaves), 0, s, a);
    return hipGetLastError();
}

}  // namespace rs
