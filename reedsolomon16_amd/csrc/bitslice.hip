// Bit-sliced GF(2^16) encode (gfx950): the half-plane kernel k_encode_hp for
// m = 16 and m = 32, any k up to HpTab<LOGM>::NCH chunks.
//
// Why bit-sliced: multiplying by a twiddle with v_perm_b32 byte tables costs
// ~115 SIMD cycles per 4 symbols (12 half-rate v_perm_b32 + extraction + XOR
// folding, scripts/micro/split_rate.hip).  In bit-sliced form (a 32-bit word
// holds one bit of 32 symbols) a multiply by a *known* constant is a fixed
// XOR network over the bit-planes -- a few full-rate v_bitop3_b32 per plane.
//
// Why one kernel serves every geometry of an m: the reference's twiddles
// depend only on m and the chunk index (leopard16.go:128-224: chunk c runs
// ifftDITEncoder over fftSkew[(c+1)m - 1:], the final fftDIT over
// fftSkew[0:]); k and p only truncate.  tools/gen_bs_tables.cpp writes the
// per-m tables (build/bs_tables.h, HpTab<LOGM>) and every twiddle is an
// instruction-stream constant; k and p are kernel arguments.
//
// Subfield coordinates (gf_host.hpp SubCoords): every twiddle of chunks
// c < NCH lies in GF(2^8), and in the coordinates lo ^= D(hi) it acts as the
// same 8x8 GF(2) map on both byte halves of a symbol.  So a lane holds one
// half (8 bit-planes) of a 64-byte block, and the half becomes a lane bit.
//
// Work split: one 2 KB tile (32 blocks of every row of one stripe) per
// 256-thread workgroup, two (m = 32) or four (m = 16) workgroups resident per
// CU; lane l = (block l & 31, half l >> 5) in each of
// the 4 waves.  With RW = m/4 rows per wave and LR = LOGM - 2:
//
//   chunk IFFT layers r0 .. r(LR-1) (leopard16.go:694-741): wave w holds rows
//     RW*w + j.  Their twiddles depend on the row bits above the layer (= w),
//     so the wave's role is w (a wave-uniform dispatch).
//   -> one LDS exchange (m x 2 KB image: row x plane quad x lane) ->
//   chunk IFFT layers r(LR), r(LR+1): wave w holds the cosets co = U*w + u
//     (U = m/16 cosets, row bits below LR) of rows co + RW*t (t = 0..3);
//     twiddles depend only on t, so every wave runs the same code.
//     XOR-accumulate into A (same layout).
//   final FFT layers r(LR+1), r(LR) (fftDIT leopard16.go:618-657) in A's
//   layout -> one exchange -> layers r(LR-1) .. r0 on rows RW*w + j, store.
//
// Loads/stores need whole 64-byte blocks (the bit-plane transpose and the
// coordinate change mix both halves): lane (b, h) loads rows RW*w + HR*h + i
// (HR = RW/2, i < HR) of block b, transposes them, and one v_permlane32_swap
// per plane pair moves the other half of each row to the partner lane.
// HBM: each data row read once (buffer loads, range-checked: rows >= k read
// as zero), each parity row < p written once; the next chunk's rows are
// prefetched into registers during the current chunk.
//
// Registers (m = 32, 2 waves per SIMD): 64 staged + 64 working + 64
// accumulator; m = 16 (4 waves per SIMD): 32 + 32 + 32.  The XOR networks
// are in-place inline asm so the compiler cannot rename their intermediates
// into fresh registers, and every butterfly is a scheduling region.
#include <algorithm>
#include <array>
#include <cstdlib>
#include <map>
#include <mutex>
#include <utility>

#include "bs_common.hpp"
#include "bs_tables.h"
#include "kernels.hpp"
#include "schedule.hpp"

namespace rs {
namespace {
using namespace bs;

// ---- slot indexing: schedule.hpp ifft_slot / fft_slot
// The slots the round-2 m = 32 kernel hard-coded.
static_assert(ifft_slot(5, 0, 8) == 6 && ifft_slot(5, 0, 10) == 8 && ifft_slot(5, 1, 12) == 10, "ifft r0/r1");
static_assert(ifft_slot(5, 2, 8) == 26 && ifft_slot(5, 2, 16) == 27 && ifft_slot(5, 3, 0) == 25 &&
                  ifft_slot(5, 3, 16) == 28 && ifft_slot(5, 4, 3) == 30, "ifft r2-r4");
static_assert(fft_slot(5, 4, 0) == 1 && fft_slot(5, 3, 0) == 0 && fft_slot(5, 3, 16) == 2, "fft r4/r3");
static_assert(fft_slot(5, 2, 8) == 7 && fft_slot(5, 1, 8) == 6 && fft_slot(5, 1, 12) == 8 &&
                  fft_slot(5, 0, 10) == 20 && fft_slot(5, 0, 30) == 30, "fft r2-r0");
static_assert(ifft_slot(4, 2, 0) == 12 && ifft_slot(4, 2, 8) == 14 && ifft_slot(4, 3, 0) == 13, "m16 ifft");
static_assert(fft_slot(4, 3, 0) == 1 && fft_slot(4, 2, 8) == 2 && fft_slot(4, 0, 6) == 8, "m16 fft");

// x ^= y * twiddle (C >= 0: chunk C's IFFT slot; C < 0: FFT slot)
template <class TW, int C, int SLOT>
__device__ __forceinline__ void hp_mul_add(Half &x, const Half &y) {
#pragma unroll
    for (int i = 0; i < 8; i++) xor_net8(x[i], y, C < 0 ? TW::fft8[SLOT][i] : TW::ifft8[C < 0 ? 0 : C][SLOT][i]);
}
// IFFT butterfly: y ^= x; x ^= y * t.   FFT butterfly: x ^= y * t; y ^= x.
// Each butterfly is a scheduling region of its own (sched_barrier): the
// machine scheduler would otherwise interleave butterflies for ILP and run
// the kernel out of registers.
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

// Subfield coordinates of a whole row held as (lo planes, hi planes): lo ^= D(hi).
template <class TW>
__device__ __forceinline__ void hp_psi(Half &lo, const Half &hi) {
#pragma unroll
    for (int r = 0; r < 8; r++) xor_net8(lo[r], hi, TW::dmat[r]);
}
// Full rows i (i < HR: R[i] lo planes, R[HR + i] hi planes) <-> half rows
// (lanes 0-31: lo half, lanes 32-63: hi half; R[i] = row i, R[HR + i] = row
// HR + i of the lane's half).  An involution.
// In-place inline asm: the builtin's two results land in fresh registers, and
// all swaps in flight at once cost the kernel 64 VGPRs.  s_nop 1: two wait
// states between a VALU write of an operand and the swap that reads it.
template <int HR>
__device__ __forceinline__ void hp_swap_halves(Half (&R)[2 * HR]) {
#pragma unroll
    for (int i = 0; i < HR; i++) {
        asm volatile(
            "s_nop 1\n\t"
            "v_permlane32_swap_b32 %0, %8\n\tv_permlane32_swap_b32 %1, %9\n\t"
            "v_permlane32_swap_b32 %2, %10\n\tv_permlane32_swap_b32 %3, %11\n\t"
            "v_permlane32_swap_b32 %4, %12\n\tv_permlane32_swap_b32 %5, %13\n\t"
            "v_permlane32_swap_b32 %6, %14\n\tv_permlane32_swap_b32 %7, %15"
            : "+v"(R[i][0]), "+v"(R[i][1]), "+v"(R[i][2]), "+v"(R[i][3]), "+v"(R[i][4]), "+v"(R[i][5]),
              "+v"(R[i][6]), "+v"(R[i][7]), "+v"(R[HR + i][0]), "+v"(R[HR + i][1]), "+v"(R[HR + i][2]),
              "+v"(R[HR + i][3]), "+v"(R[HR + i][4]), "+v"(R[HR + i][5]), "+v"(R[HR + i][6]), "+v"(R[HR + i][7]));
    }
}

// ---- LDS image: row r, plane quad qh of lane l at byte r * 2048 + qh * 1024 + l * 16
// (every ds_*_b128 wave access is 1 KB contiguous).
// The row address is rebuilt at every use from an opaque copy of the lane
// base (one v_add): otherwise the compiler hoists every row address out of
// the persistent tile loop and spills them.
__device__ __forceinline__ uint32_t hp_row_addr(uint32_t lbase, int row) {
    uint32_t b = lbase;
    asm volatile("" : "+v"(b));
    return b + (uint32_t)row * 2048u;
}
__device__ __forceinline__ void hp_put(uint32_t lbase, int row, const Half &v) {
    const uint32_t ra = hp_row_addr(lbase, row);
    *(lds_u4 *)(uintptr_t)ra = u32x4{v[0], v[1], v[2], v[3]};
    *(lds_u4 *)(uintptr_t)(ra + 1024) = u32x4{v[4], v[5], v[6], v[7]};
}
__device__ __forceinline__ void hp_get(uint32_t lbase, int row, Half &v) {
    const uint32_t ra = hp_row_addr(lbase, row);
    const u32x4 x = *(const lds_u4 *)(uintptr_t)ra;
    const u32x4 y = *(const lds_u4 *)(uintptr_t)(ra + 1024);
    v[0] = x[0], v[1] = x[1], v[2] = x[2], v[3] = x[3];
    v[4] = y[0], v[5] = y[1], v[6] = y[2], v[7] = y[3];
}
// Workgroup barrier for the LDS image only.  __syncthreads() is also a
// release/acquire fence, which waits for every outstanding global load
// (vmcnt(0)) and so would drain the next chunk's prefetch at the first
// barrier of every chunk; this waits for LDS traffic alone.

template <int LOGM, bool VERIFY>
struct HpEncoder {
    using TW = HpTab<LOGM>;
    static constexpr int M = 1 << LOGM;
    static constexpr int RW = M / 4;       // rows per wave in the row-group phases
    static constexpr int HR = RW / 2;      // full rows loaded (and stored) per lane
    static constexpr int LR = LOGM - 2;    // layers within a wave's rows
    static constexpr int U = M / 16;       // cosets per wave
    static constexpr int NCH = TW::NCH;    // chunks compiled in (k <= NCH * m)
    static constexpr int TILE = 2048;      // column bytes per tile (32 blocks)
    static constexpr int PF1 = LOGM == 5 ? 2 : HR / 2;  // rows of the next chunk issued before phase 1
    static_assert(LOGM == 4 || LOGM == 5, "m = 16 or 32");
    const BsArgs &a;
    uint32_t lbase;  // this lane's LDS byte address of row 0, quad 0
    int lane, w, h, blk, nch;
    Half St[RW];  // staged full rows i < HR: St[i] = dwords 0-7 (low bytes), St[HR+i] = dwords 8-15
    Half R[RW];   // working rows
    Half A[RW];   // accumulator: coset u (co = U*w + u), rows co + RW*t at A[4u + t]

    // A tile's stripe and column tile (wave-uniform), decomposed once per tile:
    // a scalar division costs ~40 instructions of the wave's issue slots.
    struct Loc {
        int stripe, ct;
        bool live;
    };
    __device__ __forceinline__ Loc locate(int tile) const {
        const int tps = a.tiles_per_stripe;
        const int stripe = tile / tps;
        return Loc{stripe, tile - stripe * tps, tile < a.ntiles};
    }

    // Load rows M*c + RW*w + HR*h + i, i in [I0, I1), of tile L through a
    // buffer descriptor over the stripe's data rows: rows past k and bytes past
    // the last row's end read as zero (range check), a tile past the end has
    // an empty range.  Lanes whose block lies past the row end read bytes of
    // the next row; their results are never stored.
    template <int I0, int I1>
    __device__ __forceinline__ void stage(const Loc &L, int c) {
        const uint32_t range = L.live ? a.span : 0u;
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            (void *)(a.data + (L.live ? (uint64_t)L.stripe * a.stripe_stride : 0)), 0, (int)range, 0x00020000);
        // lane part of the offset (block, half); opaque so that the compiler
        // does not precompute every chunk's offsets
        uint32_t voff = (uint32_t)L.ct * TILE + (uint32_t)blk * 64 + (uint32_t)(HR * h) * (uint32_t)a.row_stride;
        constexpr uint32_t QS = 16;
        asm volatile("" : "+v"(voff));
        // the loads issue at raised wave priority, ahead of the other waves'
        // VALU: one stripe per launch 0.524-0.527 -> 0.547-0.552 of the
        // roofline, 128 stripes unchanged (same box, profiles/r03_c3_prio_ab.txt;
        // raising it around the parity stores too gained nothing)
        __builtin_amdgcn_s_setprio(2);
#pragma unroll
        for (int i = I0; i < I1; i++) {
            // wave-uniform row of the h = 0 lanes (rows >= k are out of range: zeros)
            const uint32_t soff = (uint32_t)(M * c + RW * w + i) * (uint32_t)a.row_stride;
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const u32x4 x = __builtin_amdgcn_raw_buffer_load_b128(rs, voff + q * QS, soff, 0);
                uint32_t *d = q < 2 ? &St[i][q * 4] : &St[HR + i][(q - 2) * 4];
                d[0] = x[0], d[1] = x[1], d[2] = x[2], d[3] = x[3];
            }
        }
        __builtin_amdgcn_s_setprio(0);
    }

    // IFFT layers r0 .. r(LR-1) on rows RW*W + j.
    template <int C, int W>
    __device__ __forceinline__ void phase1() {
        sfor<LR>([&](auto L) {
            constexpr int l = decltype(L)::value;
            sfor<RW / 2>([&](auto Q) {
                constexpr int q = decltype(Q)::value;
                constexpr int j = ((q >> l) << (l + 1)) | (q & ((1 << l) - 1));
                hp_ifft2<TW, C, ifft_slot(LOGM, l, RW * W + j)>(R[j], R[j + (1 << l)]);
            });
        });
    }

    // Next chunk's rows i in [I0, I1): chunk C + 1 of this tile, or chunk 0 of the next tile.
    template <int C, int I0, int I1>
    __device__ __forceinline__ void prefetch(const Loc &cur, const Loc &nxt) {
        const bool more = C + 1 < nch;  // wave-uniform: one load sequence, no branch
        stage<I0, I1>(more ? cur : nxt, more ? C + 1 : 0);
    }

    // The next chunk's loads go out in two halves so that (m = 32) at most
    // 160 of the 256 VGPRs hold data (A 64 + R 64 + half of St during the
    // transposes and the row-group layers; A 64 + St 64 + one coset's 32
    // during the coset layers): rows i < HR/2 once the staged rows are
    // transposed, the rest once the row-group rows are in the LDS image.
    // (Issuing all of them at the chunk start, with 192 VGPRs of data live,
    // spilled to scratch: +8 % HBM traffic.)
    template <int C>
    __device__ __forceinline__ void chunk(const Loc &cur, const Loc &nxt) {
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < RW; i++)
#pragma unroll
            for (int q = 0; q < 8; q++) R[i][q] = St[i][q];
#pragma unroll
        for (int i = 0; i < HR; i++) {
            bs_transpose8(R[i]);
            bs_transpose8(R[HR + i]);
            hp_psi<TW>(R[i], R[HR + i]);
        }
        hp_swap_halves<HR>(R);
        // consume the staged rows before their registers are reloaded
#pragma unroll
        for (int i = 0; i < RW; i++)
#pragma unroll
            for (int q = 0; q < 8; q++) asm volatile("" : "+v"(R[i][q])::"memory");
        __builtin_amdgcn_sched_barrier(0);
        prefetch<C, 0, PF1>(cur, nxt);
        __builtin_amdgcn_sched_barrier(0);
        dispatch<4>(w, [&](auto W) { phase1<C, decltype(W)::value>(); });
        lds_barrier();  // every wave has read the previous image
#pragma unroll
        for (int j = 0; j < RW; j++) hp_put(lbase, RW * w + j, R[j]);
        lds_barrier();
        prefetch<C, PF1, HR>(cur, nxt);
        __builtin_amdgcn_sched_barrier(0);
        // IFFT layers r(LR), r(LR+1), one coset at a time
#pragma unroll
        for (int u = 0; u < U; u++) {
#pragma unroll
            for (int t = 0; t < 4; t++) hp_get(lbase, U * w + u + RW * t, R[t]);
            hp_ifft2<TW, C, ifft_slot(LOGM, LR, 0)>(R[0], R[1]);
            hp_ifft2<TW, C, ifft_slot(LOGM, LR, 2 * RW)>(R[2], R[3]);
            hp_ifft2<TW, C, ifft_slot(LOGM, LR + 1, 0)>(R[0], R[2]);
            hp_ifft2<TW, C, ifft_slot(LOGM, LR + 1, RW)>(R[1], R[3]);
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

    // Chunks C < nch (wave-uniform branches; the code of a geometry's unused
    // chunks is never fetched).  Chunk 0 unconditionally: with a branch
    // around it too, the allocator spilled 11-14 VGPRs.
    template <int... Cs>
    __device__ __forceinline__ void chunks(const Loc &cur, const Loc &nxt, std::integer_sequence<int, Cs...>) {
        ((Cs == 0 || Cs < nch ? (chunk<Cs>(cur, nxt), 0) : 0), ...);
    }

    // FFT layers r(LR-1) .. r0 on rows RW*W + j.
    template <int W>
    __device__ __forceinline__ void fft_b() {
        sfor<LR>([&](auto L) {
            constexpr int l = LR - 1 - decltype(L)::value;
            sfor<RW / 2>([&](auto Q) {
                constexpr int q = decltype(Q)::value;
                constexpr int j = ((q >> l) << (l + 1)) | (q & ((1 << l) - 1));
                hp_fft2<TW, fft_slot(LOGM, l, RW * W + j)>(R[j], R[j + (1 << l)]);
            });
        });
    }

    // Workgroup b runs tiles t0 + i * step, i < tpw (launch_hp_t): t0 =
    // (b / step) * step * tpw + b % step, so the tiles of the grid are each run once.
    __device__ __forceinline__ void run() {
        const int b = blockIdx.x, step = a.tile_step;
        int tile = (b / step) * step * a.tpw + b % step;
        const int tend = min(a.ntiles, tile + step * a.tpw);
        Loc cur = locate(tile);
        stage<0, HR>(cur, 0);
        for (; tile < tend; tile += step) {
            const Loc nxt = locate(tile + step < tend ? tile + step : a.ntiles);
            chunks(cur, nxt, std::make_integer_sequence<int, NCH>{});
            // FFT layers r(LR+1), r(LR) in A's layout
#pragma unroll
            for (int u = 0; u < U; u++) {
                hp_fft2<TW, fft_slot(LOGM, LR + 1, 0)>(A[4 * u], A[4 * u + 2]);
                hp_fft2<TW, fft_slot(LOGM, LR + 1, RW)>(A[4 * u + 1], A[4 * u + 3]);
                hp_fft2<TW, fft_slot(LOGM, LR, 0)>(A[4 * u], A[4 * u + 1]);
                hp_fft2<TW, fft_slot(LOGM, LR, 2 * RW)>(A[4 * u + 2], A[4 * u + 3]);
            }
            lds_barrier();
#pragma unroll
            for (int u = 0; u < U; u++)
#pragma unroll
                for (int t = 0; t < 4; t++) hp_put(lbase, U * w + u + RW * t, A[4 * u + t]);
            lds_barrier();
#pragma unroll
            for (int j = 0; j < RW; j++) hp_get(lbase, RW * w + j, R[j]);
            dispatch<4>(w, [&](auto W) { fft_b<decltype(W)::value>(); });
            hp_swap_halves<HR>(R);
            // parity rows RW*w + HR*h + i < p, through a descriptor over the
            // stripe's parity rows (lanes past the row end store nothing: exec mask)
            const uint32_t col = (uint32_t)cur.ct * TILE + (uint32_t)blk * 64;
            const __amdgpu_buffer_rsrc_t ps = __builtin_amdgcn_make_buffer_rsrc(
                (void *)(a.parity + (uint64_t)cur.stripe * a.stripe_stride), 0, (int)a.pspan, 0x00020000);
            uint32_t voff = col + (uint32_t)(HR * h) * (uint32_t)a.row_stride;
            constexpr uint32_t QS = 16;
            asm volatile("" : "+v"(voff));
            uint32_t bad = 0;
            if (col < a.S) {
#pragma unroll
                for (int i = 0; i < HR; i++) {
                    const int row = RW * w + HR * h + i;
                    if (row >= a.p) continue;
                    hp_psi<TW>(R[i], R[HR + i]);
                    bs_transpose8(R[i]);
                    bs_transpose8(R[HR + i]);
                    const uint32_t soff = (uint32_t)(RW * w + i) * (uint32_t)a.row_stride;
#pragma unroll
                    for (int k = 0; k < 4; k++) {
                        const int o = (k & 1) * 4;
                        const u32x4 v = k < 2 ? u32x4{R[i][o], R[i][o + 1], R[i][o + 2], R[i][o + 3]}
                                              : u32x4{R[HR + i][o], R[HR + i][o + 1], R[HR + i][o + 2], R[HR + i][o + 3]};
                        if constexpr (VERIFY) {
                            const u32x4 old = __builtin_amdgcn_raw_buffer_load_b128(ps, voff + k * QS, soff, 0);
                            bad |= (old[0] ^ v[0]) | (old[1] ^ v[1]) | (old[2] ^ v[2]) | (old[3] ^ v[3]);
                        } else {
                            __builtin_amdgcn_raw_buffer_store_b128(v, ps, voff + k * QS, soff, 0);
                        }
                    }
                }
            }
            if constexpr (VERIFY) {
                // one store per wave, not per lane
                const uint64_t m = __ballot(bad != 0);
                // a set flag stays set: skip the store (a failing verify would
                // otherwise store once per wave per tile into one contended word)
                if (m && lane == __ffsll((unsigned long long)m) - 1 &&
                    __hip_atomic_load(a.mismatch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0)
                    __hip_atomic_store(a.mismatch, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            cur = nxt;
        }
    }
};

// Workgroups per CU: LDS m x 2 KB and the register budget above.
template <int LOGM> constexpr int kHpWgPerCu = LOGM == 5 ? 2 : 4;

template <int LOGM, bool VERIFY>
__global__ void __launch_bounds__(256, kHpWgPerCu<LOGM>) k_encode_hp(BsArgs a) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[(1 << LOGM) * 512];  // m rows x 2 KB
    HpEncoder<LOGM, VERIFY> e{a};
    e.lane = threadIdx.x & 63;
    e.w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    e.h = e.lane >> 5;
    e.blk = e.lane & 31;
    e.nch = (a.k + (1 << LOGM) - 1) >> LOGM;
    e.lbase = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) uint32_t *)lds + e.lane * 16;
    e.run();
}

// Run-time choice of the tile map for launches where both maps are candidates
// (four tiles per workgroup a grid apart, or one).  Which one wins depends on
// the box: four tiles gave 0.684-0.686 against 0.655 for one on two boxes
// of round 6, and 0.634-0.640 against 0.653-0.657 on two others (full 1 MiB
// rows, 256 stripes; the 8-rank slice moves the other way on some boxes:
// profiles/r06_c3_tile_map_boxes.txt), with the same code and launch.  So the first launches of a shape alternate the two maps under
// events on the launch stream, and once kTrials of them have completed the
// shape keeps the map with the smaller median (the first pair, cold, is
// dropped).  Until then, and after a tie, the static rule's four tiles run.
// Both maps compute the same bytes (test_bs_tiles_per_workgroup).
class HpTuner {
  public:
    static constexpr int kTrials = 8;
    typedef std::array<int64_t, 8> Key;  // device, logm, verify, ntiles, tiles per stripe, strides, S
    // tpw for this launch; *e0 / *e1 events to record around it (trial launches only)
    int choose(const Key &key, hipEvent_t *e0, hipEvent_t *e1) {
        std::lock_guard<std::mutex> lk(mu_);
        Entry &t = m_[key];
        if (t.pick) return t.pick;
        if (t.n < kTrials) {
            if (hipEventCreate(&t.ev[t.n][0]) != hipSuccess || hipEventCreate(&t.ev[t.n][1]) != hipSuccess) {
                t.pick = kMany;  // no events: keep the static rule
                return t.pick;
            }
            *e0 = t.ev[t.n][0];
            *e1 = t.ev[t.n][1];
            return t.n++ % 2 ? 1 : kMany;
        }
        if (hipEventQuery(t.ev[kTrials - 1][1]) != hipSuccess) return kMany;  // trials still running
        float ms[2][kTrials / 2 - 1];
        bool ok = true;
        for (int i = 2; i < kTrials; i++)
            ok = ok && hipEventElapsedTime(&ms[i % 2][i / 2 - 1], t.ev[i][0], t.ev[i][1]) == hipSuccess;
        for (auto &e : t.ev) {
            (void)hipEventDestroy(e[0]);
            (void)hipEventDestroy(e[1]);
        }
        auto med = [](float *x) {
            std::sort(x, x + kTrials / 2 - 1);
            return x[(kTrials / 2 - 1) / 2];
        };
        const int pick = ok && med(ms[1]) < med(ms[0]) ? 1 : kMany;
        t.pick = pick;
        if (m_.size() > 256) {  // shapes of a long-lived process: re-tune rather than grow
            for (auto &kv : m_)
                if (!kv.second.pick)
                    for (int i = 0; i < kv.second.n; i++) {  // (a pending event is released once it completes)
                        (void)hipEventDestroy(kv.second.ev[i][0]);
                        (void)hipEventDestroy(kv.second.ev[i][1]);
                    }
            m_.clear();
        }
        return pick;
    }
    static constexpr int kMany = 4;

  private:
    struct Entry {
        int n = 0, pick = 0;
        hipEvent_t ev[kTrials][2] = {};
    };
    std::mutex mu_;
    std::map<Key, Entry> m_;
};
HpTuner g_hp_tuner;

template <int LOGM>
hipError_t launch_hp_t(bool verify, BsArgs a, int cus, hipStream_t s) {
    a.tiles_per_stripe = (int)((a.S + 2047) / 2048);
    a.ntiles = a.tiles_per_stripe * a.nstripes;
    a.span = (uint32_t)((uint64_t)(a.k - 1) * a.row_stride + a.S);
    a.pspan = (uint32_t)((uint64_t)(a.p - 1) * a.row_stride + a.S);
    // Tiles per workgroup: workgroup b runs tiles t0, t0 + step, ... (run()),
    // and each tile's last chunk prefetches the next tile's first (HpEncoder::
    // prefetch), so only its first tile pays the load latency with nothing to
    // overlap.  A fully persistent grid (one generation of workgroups) ran in
    // lockstep and lost (round 3: 0.611 against 0.631 for one tile per
    // workgroup, profiles/r03_c3_grid_ab.txt).  Round 5 (profiles/
    // r05_c3_tiles_per_wg.txt): four tiles per workgroup, a grid size apart,
    // take C3 launches of 224-512 full-row stripes from 0.65 to 0.69-0.71 on
    // five of six boxes (one lost 0.01); adjacent tiles or a one- to
    // sixteen-stripe distance lose (0.64-0.667).  Launches under ~200 tiles
    // per workgroup slot of full 1 MiB rows (<= 192 stripes) lose 0.01-0.02
    // with several tiles, so they keep one.  Rows of a byte-range slice
    // (<= 512 KiB: the per-rank shape of a 2-8 rank split, 256 stripes) never
    // lost on three boxes with four tiles and gained 0.002-0.06 (profiles/
    // r05_c3_tiles_per_wg.txt, calls r5h, r5k, r5m).
    const int slots = std::max(cus, 1) * kHpWgPerCu<LOGM>;
    int tpw = hp_tiles_override();
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (tpw <= 0) {
        tpw = (a.ntiles >= 224 * slots || (a.tiles_per_stripe <= 256 && a.ntiles >= 32 * slots)) ? HpTuner::kMany : 1;
        int dev = 0;
        if (tpw > 1 && hp_tune_enabled() && hipGetDevice(&dev) == hipSuccess)
            tpw = g_hp_tuner.choose({dev, LOGM, verify ? 1 : 0, a.ntiles, a.tiles_per_stripe, (int64_t)a.row_stride,
                                     a.nstripes > 1 ? (int64_t)a.stripe_stride : 0, (int64_t)a.S},
                                    &e0, &e1);
    }
    int step = hp_step_override();
    if (step <= 0) step = (a.ntiles + tpw - 1) / tpw;
    step = std::min(step, a.ntiles);
    // workgroups: full blocks of step * tpw tiles, then the remainder
    const int blocks = a.ntiles / (step * tpw), rem = a.ntiles - blocks * step * tpw;
    const int grid = blocks * step + std::min(rem, step);
    a.tpw = tpw;
    a.tile_step = step;
    if (e0) (void)hipEventRecord(e0, s);
    if (verify) hipLaunchKernelGGL((k_encode_hp<LOGM, true>), dim3(grid), dim3(256), 0, s, a);
    else hipLaunchKernelGGL((k_encode_hp<LOGM, false>), dim3(grid), dim3(256), 0, s, a);
    const hipError_t le = hipGetLastError();
    if (e1) (void)hipEventRecord(e1, s);
    return le;
}

int hp_logm(int p) { return p > 16 ? 5 : 4; }

template <int LOGM>
bool hp_tables_match(int k, const uint32_t *il, const uint32_t *fl, uint32_t mod) {
    using TW = HpTab<LOGM>;
    const int nch = (k + TW::M - 1) / TW::M;
    if (nch > TW::NCH) return false;
    for (int c = 0; c < nch; c++)
        for (int s = 0; s < TW::IS; s++)
            if (il[c * TW::IS + s] != mod && il[c * TW::IS + s] != TW::ifft_log[c][s]) return false;
    for (int s = 0; s < TW::FS; s++)
        if (fl[s] != mod && fl[s] != TW::fft_log[s]) return false;
    return true;
}

}  // namespace

bool encode_bs_available(int k, int p, const uint32_t *ifft_logs, const uint32_t *fft_logs, uint32_t mod) {
    if (k < 1 || p < 9 || p > 32) return false;
    return hp_logm(p) == 5 ? hp_tables_match<5>(k, ifft_logs, fft_logs, mod)
                           : hp_tables_match<4>(k, ifft_logs, fft_logs, mod);
}

bool encode_bs_fits(int k, int p, uint64_t row_stride, uint64_t S) {
    if (k < 1 || p < 9 || p > 32) return false;
    const int m = 1 << hp_logm(p);
    const uint64_t rows = (uint64_t)(k + m - 1) / m * m;  // padding rows of the last chunk are loaded too
    const uint64_t cols = (S + 2047) / 2048 * 2048;       // lanes of the last tile past the row end
    return (rows - 1) * row_stride + cols < (1ull << 32);
}

hipError_t launch_encode_bs(bool verify, const BsArgs &a, int cus, hipStream_t s) {
    if (a.k < 1 || a.p < 9 || a.p > 32) return hipErrorNotSupported;
    const int logm = hp_logm(a.p);
    if ((a.k + (1 << logm) - 1) >> logm > (logm == 5 ? HpTab<5>::NCH : HpTab<4>::NCH)) return hipErrorNotSupported;
    if (!encode_bs_fits(a.k, a.p, a.row_stride, a.S)) return hipErrorNotSupported;
    return logm == 5 ? launch_hp_t<5>(verify, a, cus, s) : launch_hp_t<4>(verify, a, cus, s);
}

}  // namespace rs
