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
#include <type_traits>
#include <cstdlib>
#include <utility>

#include "kernels.hpp"
#include "rec_common.hpp"
#include "schedule.hpp"


namespace rs {
namespace {
using namespace rec;

typedef __attribute__((address_space(1))) void gvoid_t;
typedef __attribute__((address_space(3))) void lvoid_t;

template <int W> struct VecOf;
template <> struct VecOf<1> { typedef uint32_t T; };
template <> struct VecOf<2> { typedef uint32_t T __attribute__((ext_vector_type(2))); };
template <> struct VecOf<4> { typedef uint32_t T __attribute__((ext_vector_type(4))); };

template <int W>
__device__ __forceinline__ void ldw(const uint8_t *p, uint32_t (&v)[W]) {
    typedef typename VecOf<W>::T T;
    const T x = *(const __attribute__((address_space(1))) T *)(p);
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
    *(__attribute__((address_space(1))) T *)(p) = x;
}
// LDS (address space 3) loads of W dwords.
template <int W>
__device__ __forceinline__ void ldw_lds(const uint8_t *p, uint32_t (&v)[W]) {
    typedef typename VecOf<W>::T T;
    const T x = *(const __attribute__((address_space(3))) T *)(p);
    if constexpr (W == 1) {
        v[0] = x;
    } else {
#pragma unroll
        for (int i = 0; i < W; i++) v[i] = x[i];
    }
}

// Verify's mismatch word is a device word the host reads back after the
// launch (codec.cpp): every writer stores the same 1, so a plain store
// suffices.  One lane per wave stores.
__device__ __forceinline__ void flag_mismatch(int *f, bool bad) {
    const uint64_t m = __ballot(bad);
    if (m && __lane_id() == (unsigned)(__ffsll((unsigned long long)m) - 1) &&
        __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0)  // set stays set: no contended store
        __hip_atomic_store(f, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ uint32_t perm(uint32_t s0, uint32_t s1, uint32_t sel) {
    return __builtin_amdgcn_perm(s0, s1, sel);
}
// a ^ b ^ c in one VALU op (gfx950 v_bitop3_b32, truth table 0x96).
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// ---------------------------------------------------------------- GF(2^16)
template <int W_>
struct F16 {
    static constexpr int W = W_;
    static constexpr bool SYM16 = true;  // 16-bit symbols (lo/hi halves of 64-byte blocks)
    static constexpr int TWD = 24;     // dwords per twiddle table
    static constexpr int TWU = 20;     // dwords used by mul_add
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
    // ---- LDS staging of one wave's 64 units of a row (512*W bytes).
    // Row image: [lo halves of blocks 0..4W) [hi halves of blocks 0..4W)
    //            [lo halves of blocks 4W..8W) [hi halves of blocks 4W..8W)
    // so lane l reads its lo dwords at (l/32)*256W + (l%32)*4W and its hi dwords
    // 128W bytes later: consecutive lanes hit consecutive banks (conflict-free).
    static constexpr int ROWB = 512 * W;
    __device__ static uint64_t span_off(uint64_t u0) { return (u0 / UPB) * 64; }
    // Global byte offset (within the wave span) of the 16-byte LDS piece s.
    __device__ static uint32_t piece_goff(uint32_t s) {
        const uint32_t G = s / (8 * W), t = s % (8 * W);
        return ((G >> 1) * 4 * W + (t >> 1)) * 64 + (G & 1) * 32 + (t & 1) * 16;
    }
    __device__ static Vec lds_load(const uint8_t *img, int lane) {
        Vec v;
        const uint8_t *p = img + (lane >> 5) * (256 * W) + (lane & 31) * (4 * W);
        ldw_lds<W>(p, v.l);
        ldw_lds<W>(p + 128 * W, v.h);
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
    // Empty asm that "redefines" the registers: chains the op that produced
    // them ahead of this point (bounds code motion in the unrolled op lists).
    __device__ static void pin(Vec &v) {
#pragma unroll
        for (int i = 0; i < W; i++) asm volatile("" : "+v"(v.l[i]), "+v"(v.h[i]));
    }
    // x ^= y * exp(log_m); t = twiddle table (wave-uniform).
    __device__ static void mul_add(Vec &x, const Vec &y, const uint32_t *__restrict__ t) {
#pragma unroll
        for (int i = 0; i < W; i++) {
            const uint32_t lo = y.l[i], hi = y.h[i];
            const uint32_t a0 = lo & 0x07070707u, a1 = (lo >> 3) & 0x07070707u, a2 = (lo >> 6) & 0x03030303u;
            const uint32_t b0 = hi & 0x07070707u, b1 = (hi >> 3) & 0x07070707u, b2 = (hi >> 6) & 0x03030303u;
            x.l[i] = xor3(xor3(xor3(x.l[i], perm(t[1], t[0], a0), perm(t[5], t[4], a1)), perm(t[8], t[8], a2),
                               perm(t[11], t[10], b0)),
                          perm(t[15], t[14], b1), perm(t[18], t[18], b2));
            x.h[i] = xor3(xor3(xor3(x.h[i], perm(t[3], t[2], a0), perm(t[7], t[6], a1)), perm(t[9], t[9], a2),
                               perm(t[13], t[12], b0)),
                          perm(t[17], t[16], b1), perm(t[19], t[19], b2));
        }
    }
};

// ---------------------------------------------------------------- GF(2^8)
template <int W_>
struct F8 {
    static constexpr int W = W_;
    static constexpr bool SYM16 = false;
    static constexpr int TWD = 8;
    static constexpr int TWU = 5;
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
    // LDS staging: natural layout, lane l at l*4W (conflict-free).
    static constexpr int ROWB = 256 * W;
    __device__ static uint64_t span_off(uint64_t u0) { return u0 * (4 * W); }
    __device__ static uint32_t piece_goff(uint32_t s) { return s * 16; }
    __device__ static Vec lds_load(const uint8_t *img, int lane) {
        Vec v;
        ldw_lds<W>(img + lane * (4 * W), v.b);
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
    __device__ static void pin(Vec &v) {
#pragma unroll
        for (int i = 0; i < W; i++) asm volatile("" : "+v"(v.b[i]));
    }
    __device__ static void mul_add(Vec &x, const Vec &y, const uint32_t *__restrict__ t) {
#pragma unroll
        for (int i = 0; i < W; i++) {
            const uint32_t v = y.b[i];
            const uint32_t a0 = v & 0x07070707u, a1 = (v >> 3) & 0x07070707u, a2 = (v >> 6) & 0x03030303u;
            x.b[i] = xor3(x.b[i] ^ perm(t[1], t[0], a0), perm(t[3], t[2], a1), perm(t[4], t[4], a2));
        }
    }
};

// ---------------------------------------------------------------- GF(2^16) in subfield coordinates
// Transforms whose twiddles all lie in GF(2^8) (fftSkew indices < 255, e.g. the
// n = 256 reconstruct of C4) run on symbols held as (x0, x1) = (lo ^ D(hi), hi)
// (gf_host.hpp SubCoords): a product with a subfield element is the same 8x8
// map on both bytes, 6 v_perm_b32 per 4 symbols with one GF(2^8)-layout table
// instead of 12.  Loads/stores are F16's; the coordinate change is folded into
// the full-field tables that scale the rows in and out.
template <int W_>
struct F16S : F16<W_> {
    static constexpr int TWD = 8, TWU = 5, LOGIDX = 5;
    typedef typename F16<W_>::Vec Vec;
    __device__ static void mul_add(Vec &x, const Vec &y, const uint32_t *__restrict__ t) {
#pragma unroll
        for (int i = 0; i < W_; i++) {
            const uint32_t lo = y.l[i], hi = y.h[i];
            x.l[i] = xor3(x.l[i] ^ perm(t[1], t[0], lo & 0x07070707u), perm(t[3], t[2], (lo >> 3) & 0x07070707u),
                          perm(t[4], t[4], (lo >> 6) & 0x03030303u));
            x.h[i] = xor3(x.h[i] ^ perm(t[1], t[0], hi & 0x07070707u), perm(t[3], t[2], (hi >> 3) & 0x07070707u),
                          perm(t[4], t[4], (hi >> 6) & 0x03030303u));
        }
    }
};

// v if keep, else zero (per lane: selects, no branch)
template <class F>
__device__ __forceinline__ void keep_if(typename F::Vec &v, bool keep) {
    if constexpr (F::SYM16) {
#pragma unroll
        for (int i = 0; i < F::W; i++) v.l[i] = keep ? v.l[i] : 0u, v.h[i] = keep ? v.h[i] : 0u;
    } else {
#pragma unroll
        for (int i = 0; i < F::W; i++) v.b[i] = keep ? v.b[i] : 0u;
    }
}

// A row unit's address for the reconstruct's scale-in (live = false: a
// readable stand-in whose product is dropped), and the unit as loaded.
struct RowLoc {
    const uint8_t *p;
    int u;
    bool live;
};
template <class F>
struct RawRow {
    typename F::Vec y;
    bool live;
};
template <class F>
__device__ __forceinline__ typename F::Vec scale_row(const RawRow<F> &y, const uint32_t *__restrict__ t) {
    typename F::Vec v = F::zero();
    F::mul_add(v, y.y, t);
    keep_if<F>(v, y.live);
    return v;
}
// Row sources with a split load (raw / scale): the first pass issues an item's row loads together.
template <class T, class = void> struct HasRaw : std::false_type {};
template <class T> struct HasRaw<T, std::void_t<decltype(&T::locate)>> : std::true_type {};

// ---------------------------------------------------------------- butterflies
#define RS_TW_LIVE(t) ((t)[F::LOGIDX] != F::MOD)
template <class F>
__device__ __forceinline__ void ifft2(typename F::Vec &x, typename F::Vec &y, const uint32_t *__restrict__ t) {
    F::xor_into(y, x);
    if (RS_TW_LIVE(t)) F::mul_add(x, y, t);
}
template <class F>
__device__ __forceinline__ void fft2(typename F::Vec &x, typename F::Vec &y, const uint32_t *__restrict__ t) {
    if (RS_TW_LIVE(t)) F::mul_add(x, y, t);
    F::xor_into(y, x);
}
// Branch-free forms for the fused register kernels: a zero twiddle is shipped
// as an all-zero table (product 0), so every multiply is straight-line code
// and the scalar table loads can be hoisted.  XOR-only (X) forms are used
// where the twiddle is zero by construction.
template <class F>
__device__ __forceinline__ void ifft2m(typename F::Vec &x, typename F::Vec &y, const uint32_t *__restrict__ t) {
    F::xor_into(y, x);
    F::mul_add(x, y, t);
}
template <class F>
__device__ __forceinline__ void fft2m(typename F::Vec &x, typename F::Vec &y, const uint32_t *__restrict__ t) {
    F::mul_add(x, y, t);
    F::xor_into(y, x);
}
template <class F>
__device__ __forceinline__ void fft2x(typename F::Vec &x, typename F::Vec &y) {
    F::xor_into(y, x);
}

// Slot order of a radix-4 group: t[0] = m01, t[1] = m02, t[2] = m23 (each F::TWD dwords).
// BF: branch-free multiplies (a zero twiddle's table is all zeros), for
// lane-varying tables, where a per-lane zero test would make every multiply
// wait for its table load.
template <class F, bool BF = false>
__device__ __forceinline__ void ifft4(typename F::Vec &x0, typename F::Vec &x1, typename F::Vec &x2,
                                      typename F::Vec &x3, const uint32_t *__restrict__ t) {
    if constexpr (BF) {
        ifft2m<F>(x0, x1, t);
        ifft2m<F>(x2, x3, t + 2 * F::TWD);
        ifft2m<F>(x0, x2, t + F::TWD);
        ifft2m<F>(x1, x3, t + F::TWD);
    } else {
        ifft2<F>(x0, x1, t);               // m01
        ifft2<F>(x2, x3, t + 2 * F::TWD);  // m23
        ifft2<F>(x0, x2, t + F::TWD);      // m02
        ifft2<F>(x1, x3, t + F::TWD);
    }
}
template <class F, bool BF = false>
__device__ __forceinline__ void fft4(typename F::Vec &x0, typename F::Vec &x1, typename F::Vec &x2, typename F::Vec &x3,
                                     const uint32_t *__restrict__ t) {
    if constexpr (BF) {
        fft2m<F>(x0, x2, t + F::TWD);
        fft2m<F>(x1, x3, t + F::TWD);
        fft2m<F>(x0, x1, t);
        fft2m<F>(x2, x3, t + 2 * F::TWD);
    } else {
        fft2<F>(x0, x2, t + F::TWD);  // m02
        fft2<F>(x1, x3, t + F::TWD);
        fft2<F>(x0, x1, t);               // m01
        fft2<F>(x2, x3, t + 2 * F::TWD);  // m23
    }
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
// Op lists (IfftOps / FftOps) and the half-wave split schedules live in
// schedule.hpp, shared with the host.

// Twiddle table held in registers (wave-uniform -> SGPRs).
template <class F>
struct Tab {
    uint32_t v[F::TWU];
};
// LDS-resident table (uniform address: every lane reads the same 16-byte
// slots, a broadcast); lands in VGPRs so both v_perm table operands are
// VGPRs and no SGPR->VGPR copies are needed.
template <class F>
__device__ __forceinline__ Tab<F> lds_tab(uint32_t vaddr, int byte_off) {
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    Tab<F> r;
#pragma unroll
    for (int q = 0; q < (F::TWU + 3) / 4; q++) {
        // volatile: keeps IR passes from hoisting all table reads of the unrolled
        // op list together (sched_barrier only constrains the machine scheduler).
        // vaddr lives in a VGPR, so byte_off folds into the ds_read offset field.
        const u32x4 x = *(const volatile __attribute__((address_space(3))) u32x4 *)(uintptr_t)(vaddr + byte_off + 16 * q);
#pragma unroll
        for (int j = 0; j < 4; j++)
            if (4 * q + j < F::TWU) r.v[4 * q + j] = x[j];
    }
    return r;
}

// Quads [qb, qe) of a table (16 bytes each) into r.
template <class F>
__device__ __forceinline__ void lds_tab_part(Tab<F> &r, uint32_t vaddr, int byte_off, int qb, int qe) {
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
#pragma unroll
    for (int q = qb; q < qe; q++) {
        const u32x4 x = *(const volatile __attribute__((address_space(3))) u32x4 *)(uintptr_t)(vaddr + byte_off + 16 * q);
#pragma unroll
        for (int j = 0; j < 4; j++)
            if (4 * q + j < F::TWU) r.v[4 * q + j] = x[j];
    }
}

// Loaded through the constant address space: read-only for the whole launch,
// so the wave-uniform address turns into s_load_dwordx* (scalar cache).
typedef __attribute__((address_space(4))) const uint32_t cu32_t;
template <class F>
__device__ __forceinline__ Tab<F> load_tab(const uint32_t *__restrict__ t) {
    Tab<F> r;
    cu32_t *ct = (cu32_t *)t;
#pragma unroll
    for (int j = 0; j < F::TWU; j++) r.v[j] = ct[j];
    return r;
}

// Multiplying ops of a list, in order, each with the slot it reads; XOR-only
// ops need no table.  A table is loaded once per run of equal slots.
template <class OPS>
struct TabRuns {
    static constexpr int N = OPS::N;
    int slot[N > 0 ? N : 1];  // slot of the k-th table load
    int load_at[N > 0 ? N : 1];  // op index whose table is load k (or -1)
    int first_use[N > 0 ? N : 1];  // table index used by op i (-1: XOR-only)
    int count;
    constexpr TabRuns() : slot(), load_at(), first_use(), count(0) {
        constexpr OPS ops{};
        int last = -1;
        for (int i = 0; i < N; i++) {
            if (ops.op[i].kind == OP_FFTX) { first_use[i] = -1; continue; }
            if (ops.op[i].slot != last) {
                slot[count] = ops.op[i].slot;
                count++;
                last = ops.op[i].slot;
            }
            first_use[i] = count - 1;
        }
    }
};

// Runs the op list.  Twiddle tables are wave-uniform scalar loads issued two
// tables ahead of use; scheduling fences keep each load at the top of its
// region (the machine scheduler would otherwise sink it next to its wait)
// and bound the VGPR pressure of the fully unrolled code.
struct NoHook {
    __device__ __forceinline__ void operator()(int) const {}
};

// hook(i) runs before op i (i is a constant after unrolling): lets the caller
// spread other issue work, e.g. the next chunk's LDS-DMAs, through the ops.
template <class F, class OPS, class Hook = NoHook>
__device__ __forceinline__ void run_ops(typename F::Vec *w, uint32_t ltab, const Hook &hook = Hook{}) {
    constexpr OPS ops{};
    constexpr TabRuns<OPS> runs{};
    constexpr int N = OPS::N;
    constexpr int NT = runs.count;
    constexpr int TB = F::TWD * 4;  // bytes per table slot
    Tab<F> t0, t1;
    if constexpr (NT > 0) t0 = lds_tab<F>(ltab, runs.slot[0] * TB);
    int have = 0;  // index of the table in t0
#pragma unroll
    for (int i = 0; i < N; i++) {
        const BOp o = ops.op[i];
        const int need = runs.first_use[i];
        hook(i);
        if (need >= 0 && need != have) {  // next run: its table was prefetched into t1
            t0 = t1;
            have = need;
        }
        if (need >= 0 && (i == 0 || runs.first_use[i - 1] != need)) {
            if (have + 1 < NT) t1 = lds_tab<F>(ltab, runs.slot[have + 1 < NT ? have + 1 : 0] * TB);
            __builtin_amdgcn_sched_barrier(0);
        }
        if (o.kind == OP_IFFT) {
            F::xor_into(w[o.y], w[o.x]);
            F::mul_add(w[o.x], w[o.y], t0.v);
        } else if (o.kind == OP_FFT) {
            F::mul_add(w[o.x], w[o.y], t0.v);
            F::xor_into(w[o.y], w[o.x]);
        } else {
            F::xor_into(w[o.y], w[o.x]);
        }
        F::pin(w[o.x]);  // chain every op's outputs: bounds code motion
        F::pin(w[o.y]);
    }
}

template <class F, int LOGM, class Hook = NoHook>
__device__ __forceinline__ void ifft_reg(typename F::Vec (&w)[1 << LOGM], uint32_t ltab, const Hook &hook = Hook{}) {
    if constexpr (LOGM > 0) run_ops<F, IfftOps<LOGM>, Hook>(w, ltab, hook);
}
template <int LOGM>
constexpr int ifft_op_count() {
    if constexpr (LOGM > 0) return IfftOps<LOGM>::N;
    return 0;
}
template <class F, int LOGM>
__device__ __forceinline__ void fft_reg(typename F::Vec (&w)[1 << LOGM], uint32_t ltab) {
    if constexpr (LOGM > 0) run_ops<F, FftOps<LOGM>>(w, ltab);
}
constexpr int fft_slot_count(int logm) {
    int M = 1 << logm, s = 0, dist4 = M, dist = M >> 2;
    for (; dist != 0; dist4 = dist, dist >>= 2) s += 3 * (M / dist4);
    if (dist4 == 2) s += M / 2;
    return s;
}

// 32-bit LDS address of p (wave-uniform: it passes through an SGPR),
// materialized in a VGPR (opaque to the compiler) so
// that constant offsets from it use the DS instruction's offset field instead
// of one SGPR add + v_mov per access.
__device__ __forceinline__ uint32_t vgpr_lds_addr(const uint8_t *p) {
    const uint32_t a = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) uint8_t *)p;
    uint32_t v;
    asm volatile("v_mov_b32 %0, %1" : "=v"(v) : "s"(a));
    return v;
}

// Waits through the builtin, not inline asm: the waitcnt-insertion pass sees
// them and resets its model, so later LDS table reads get graded
// lgkmcnt(N) waits (prefetch kept in flight) instead of lgkmcnt(0).
// gfx9 encoding: vmcnt [3:0]+[15:14], expcnt [6:4], lgkmcnt [11:8].
__device__ __forceinline__ void wait_vm0() { __builtin_amdgcn_s_waitcnt(0x0F70); }
__device__ __forceinline__ void wait_lgkm0() { __builtin_amdgcn_s_waitcnt(0xC07F); }

template <bool ROWTAB>
__device__ __forceinline__ uint8_t *rowp(const RowSet &rs, int i, uint64_t soff) {
    if constexpr (ROWTAB) return rs.table[i];
    else return rs.base + (uint64_t)i * rs.stride + soff;
}

// Fused encode (leopard16.go:128-224 / leopard8.go:153-277) for m = 2^LOGM <= 32.
// Every lane owns one column unit of all k+p rows; the m-row accumulator and
// the current chunk live in VGPRs.  While chunk c is transformed, chunk c+1's
// rows stream HBM -> LDS (global_load_lds_dwordx4, 16 B/lane, no VGPRs) into
// the wave's private image, and its twiddle tables into the block's other
// table buffer.  HBM sees exactly k row reads and p row writes (p reads for
// verify) per unit.
template <class F, int LOGM, bool VERIFY, bool ROWTAB>
__global__ void __launch_bounds__(256, 2) k_encode_reg(EncodeArgs a) {
    constexpr int M = 1 << LOGM;
    constexpr int ROWB = F::ROWB;          // bytes of a row covered by one wave
    constexpr int PPR = ROWB / 16;         // 16-byte pieces per row
    constexpr int NDMA = M * PPR / 64;     // DMA wave-instructions per chunk
    static_assert(NDMA * 64 == M * PPR, "chunk must be whole DMA instructions");
    constexpr int IS = ifft_slot_count(LOGM), FS = fft_slot_count(LOGM);
    constexpr int TB = F::TWD * 4;                      // bytes per twiddle table
    constexpr int TABB = ((IS > FS ? IS : FS) * TB + 15) / 16 * 16;  // bytes per table buffer
    typedef typename F::Vec V;
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    __shared__ __attribute__((aligned(16))) uint8_t lds[4 * M * ROWB + 2 * TABB];
    uint8_t *ltab = lds + 4 * M * ROWB;

    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform (SGPR)
    const uint64_t units = F::units(a.shard_size);
    const uint64_t u0 = (uint64_t)blockIdx.x * 256 + wave * 64;
    const bool wave_live = u0 < units;  // waves past the row end still join the barriers
    const uint64_t u = u0 + lane;
    const uint64_t soff = (uint64_t)blockIdx.y * a.stripe_stride;
    const uint64_t span = F::span_off(u0);
    uint8_t *img = lds + wave * (M * ROWB);

    // Stage chunk c's rows: rows past the chunk's count and pieces past the
    // row end are zero-filled.
    // Buffer descriptor over this stripe's data rows (strided mode; the host
    // guarantees (k-1)*stride + shard_size < 2^32).
    const __amdgpu_buffer_rsrc_t drsrc = __builtin_amdgcn_make_buffer_rsrc(
        ROWTAB ? nullptr : (void *)(a.data.base + soff), 0,
        ROWTAB ? 0 : (int)(uint32_t)((uint64_t)(a.k - 1) * a.data.stride + a.shard_size), 0x00020000);
    // One DMA wave-instruction (piece group j) of chunk c's rows.
    auto stage_one = [&](int c, int j) {
        const int row0 = c * M, cnt = a.k - row0;
        {
            const int P = j * 64 + lane;
            const int r = P / PPR;
            const uint64_t go = span + F::piece_goff(P % PPR);
            if (wave_live && r < cnt && go < a.shard_size) {
                if constexpr (ROWTAB) {
                    const uint8_t *src = rowp<ROWTAB>(a.data, row0 + r, soff) + go;
                    __builtin_amdgcn_global_load_lds((gvoid_t *)src, (lvoid_t *)(img + j * 1024), 16, 0, 0);
                } else {
                    // MUBUF LDS-DMA: with a FLAT global_load_lds in flight the compiler's
                    // waitcnt model turns every LDS table wait into lgkmcnt(0).
                    const uint32_t voff = (uint32_t)((uint64_t)(row0 + r) * a.data.stride + go);
                    __builtin_amdgcn_raw_ptr_buffer_load_lds(drsrc, (lvoid_t *)(img + j * 1024), 16, voff, 0, 0, 0);
                }
            } else {
                *(__attribute__((address_space(3))) u32x4 *)(img + j * 1024 + lane * 16) = u32x4{0, 0, 0, 0};
            }
        }
    };
    auto stage = [&](int c) {
#pragma unroll
        for (int j = 0; j < NDMA; j++) stage_one(c, j);
    };

    // Stage `nslot` twiddle tables into table buffer b (waves split the pieces).
    auto stage_tab = [&](const uint32_t *src, int nslot, int b) {
        const int npieces = nslot * TB / 16;
        const int P = wave * 64 + lane;
        const __amdgpu_buffer_rsrc_t trsrc = __builtin_amdgcn_make_buffer_rsrc((void *)src, 0, npieces * 16, 0x00020000);
        for (int base = 0; base < npieces; base += 256) {
            if (base + P < npieces)
                __builtin_amdgcn_raw_ptr_buffer_load_lds(trsrc, (lvoid_t *)(ltab + b * TABB + base * 16 + wave * 1024),
                                                         16, (base + P) * 16, 0, 0, 0);
        }
    };

    V acc[M];
    stage(0);
    stage_tab(a.tw_ifft, IS, 0);
    for (int c = 0; c < a.nchunks; ++c) {
        wait_vm0();  // this wave's DMAs for chunk c have landed
        __syncthreads();  // every wave's table pieces landed; buffer (c+1)&1 is no longer read
        V cur[M];
#pragma unroll
        for (int r = 0; r < M; r++) cur[r] = F::lds_load(img + r * ROWB, lane);
        wait_lgkm0();  // reads done before the image is overwritten
        const bool more = c + 1 < a.nchunks;
        if (more) stage_tab(a.tw_ifft + (uint64_t)(c + 1) * IS * F::TWD, IS, (c + 1) & 1);
        else stage_tab(a.tw_fft, FS, (c + 1) & 1);
        // The next chunk's row DMAs are issued spread through the IFFT (one
        // every SPREAD ops): issued back to back while the whole GPU streams,
        // they stall the wave at issue before any butterfly starts.
        constexpr int NOPS = ifft_op_count<LOGM>();
        constexpr int SPREAD = NOPS >= NDMA ? NOPS / NDMA : 0;
        if (!SPREAD && more) stage(c + 1);
        ifft_reg<F, LOGM>(cur, vgpr_lds_addr(ltab + (c & 1) * TABB), [&](int i) {
            if (SPREAD && i % SPREAD == 0 && i / SPREAD < NDMA && more) stage_one(c + 1, i / SPREAD);
        });
        if (c == 0) {
#pragma unroll
            for (int r = 0; r < M; r++) acc[r] = cur[r];
        } else {
#pragma unroll
            for (int r = 0; r < M; r++) F::xor_into(acc[r], cur[r]);
        }
    }
    wait_vm0();
    __syncthreads();
    fft_reg<F, LOGM>(acc, vgpr_lds_addr(ltab + (a.nchunks & 1) * TABB));
    if (!wave_live || u >= units) return;
    if constexpr (VERIFY) {
        uint32_t bad = 0;
#pragma unroll
        for (int r = 0; r < M; r++)
            if (r < a.p) bad |= F::diff(acc[r], F::load(rowp<ROWTAB>(a.parity, r, soff), u));
        flag_mismatch(a.mismatch, bad != 0);
    } else {
#pragma unroll
        for (int r = 0; r < M; r++)
            if (r < a.p) F::store(rowp<ROWTAB>(a.parity, r, soff), u, acc[r]);
    }
}

// ---------------------------------------------------------------- half-wave split encode (GF(2^16), 4 <= m <= 32)
// Same algorithm as k_encode_reg, but the M rows of a column unit are split
// over lanes L and L+32 (schedule.hpp, SplitSched): per lane M/2 rows of the
// chunk and of the accumulator, so the kernel fits 128 VGPRs and runs 4 waves
// per SIMD (k_encode_reg needs ~240 VGPRs at m = 32: 2 waves per SIMD, and
// its twiddle-table reads stay exposed).  A wave covers 32 column units
// (256 bytes of every row).  Each half-wave reads its own twiddle table: the
// host lays out each transform's table loads as [lower half | upper half].
// Rows are staged HBM -> LDS by MUBUF LDS-DMA (next chunk during this one).
template <int L>
struct IfftSplit {
    static constexpr auto s = EncodeSplit<L>::ifft;
};
template <int L>
struct FftSplit {
    static constexpr auto s = EncodeSplit<L>::fft;
};

template <class SRC>
__device__ __forceinline__ void run_split(F16<1>::Vec *w, uint32_t ltab) {
    typedef F16<1> F;
    constexpr auto sch = SRC::s;
    constexpr int NS = sch.nsteps;
    constexpr int NT = sch.ntab;
    constexpr int TB = F::TWD * 4;
    constexpr int NQ = (F::TWU + 3) / 4;              // quads per table
    constexpr int PQ = 3 < NQ ? 3 : NQ;  // quads (of 5) of the next table prefetched
    Tab<F> t0, t1;
    if constexpr (NT > 0) lds_tab_part<F>(t0, ltab, 0, 0, NQ);
    int have = 0;
#pragma unroll
    for (int i = 0; i < NS; i++) {
        const SStep st = sch.step[i];
        if (st.type == ST_SWAP) {
            const auto rl = __builtin_amdgcn_permlane32_swap(w[st.a].l[0], w[st.b].l[0], false, false);
            const auto rh = __builtin_amdgcn_permlane32_swap(w[st.a].h[0], w[st.b].h[0], false, false);
            w[st.a].l[0] = rl[0];
            w[st.b].l[0] = rl[1];
            w[st.a].h[0] = rh[0];
            w[st.b].h[0] = rh[1];
            continue;
        }
        const int need = st.tab;
        if (need >= 0 && need != have) {  // next table run: its first PQ quads were prefetched into t1
#pragma unroll
            for (int j = 0; j < 4 * PQ && j < F::TWU; j++) t0.v[j] = t1.v[j];
            lds_tab_part<F>(t0, ltab, need * TB, PQ, NQ);
            have = need;
        }
        bool first = need >= 0;
        if (first) {
            for (int j = 0; j < i; j++)
                if (sch.step[j].type == ST_OP && sch.step[j].tab == need) first = false;
        }
        if (first) {
            if (have + 1 < NT) lds_tab_part<F>(t1, ltab, (have + 1) * TB, 0, PQ);
            __builtin_amdgcn_sched_barrier(0);
        }
        typename F::Vec &x = w[st.a], &y = w[st.b];
        if (st.kind == OP_IFFT) {
            F::xor_into(y, x);
            F::mul_add(x, y, t0.v);
        } else if (st.kind == OP_FFT) {
            F::mul_add(x, y, t0.v);
            F::xor_into(y, x);
        } else {
            F::xor_into(y, x);
        }
        // pin every op: bounds code motion (VGPRs)
        F::pin(x);
        F::pin(y);
    }
}

template <int LOGM>
struct SplitGeom {
    typedef EncodeSplit<LOGM> ES;
    static constexpr int M = 1 << LOGM, HM = M / 2;
    static constexpr int ROWB = 256;                 // bytes of a row per wave (32 units x 8 B)
    static constexpr int NDMA = M * ROWB / 1024;     // LDS-DMA wave-instructions per chunk
    static constexpr int TB = F16<1>::TWD * 4;
    static constexpr int NTI = ES::ifft.ntab, NTF = ES::fft.ntab;
    static constexpr int TABB = 2 * (NTI > NTF ? NTI : NTF) * TB;  // one table buffer
    static constexpr int LDS = 4 * M * ROWB + 2 * TABB;
};

template <int LOGM, bool VERIFY>
__global__ void __launch_bounds__(256, 4) k_encode_split(EncodeArgs a) {
    typedef F16<1> F;
    typedef typename F::Vec V;
    typedef SplitGeom<LOGM> G;
    typedef typename G::ES ES;
    constexpr int M = G::M, HM = G::HM, ROWB = G::ROWB, NDMA = G::NDMA, TB = G::TB;
    constexpr int NTI = G::NTI, NTF = G::NTF, TABB = G::TABB;
    constexpr auto SI = ES::ifft;
    constexpr auto SF = ES::fft;
    constexpr int H0 = SI.h0, HF = SF.hend;
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    __shared__ __attribute__((aligned(16))) uint8_t lds[G::LDS];
    uint8_t *ltab = lds + 4 * M * ROWB;

    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int cu = lane & 31, half = lane >> 5;
    const uint64_t units = a.shard_size >> 3;  // 8-byte column units (4 symbols)
    const uint64_t u0 = ((uint64_t)blockIdx.x * 4 + wave) * 32;
    const bool wave_live = u0 < units;
    const bool lane_live = u0 + cu < units;
    const uint64_t soff = (uint64_t)blockIdx.y * a.stripe_stride;
    const uint32_t span = (uint32_t)(u0 * 8);                      // wave's byte offset in a row
    const uint32_t colb = (cu >> 3) * 64 + (cu & 7) * 4;           // lane's lo dword within the wave's 256 B
    uint8_t *img = lds + wave * (M * ROWB);

    const __amdgpu_buffer_rsrc_t drsrc = __builtin_amdgcn_make_buffer_rsrc(
        (void *)(a.data.base + soff), 0, (int)(uint32_t)((uint64_t)(a.k - 1) * a.data.stride + a.shard_size), 0x00020000);
    // chunk c's rows: piece P = 16 bytes; row P / 16, piece P % 16 of the wave's 256 B.
    // Full chunks of full-width waves: per-lane offset fixed, row base in soffset
    // (no per-lane predicates to keep live across the loop).
    const bool wave_full = (uint64_t)span + ROWB <= a.shard_size;
    const uint32_t lane_off = (uint32_t)((lane >> 4) * a.data.stride) + (lane & 15) * 16 + span;
    auto stage_one = [&](int c, int j) {
        const int row0 = c * M, cnt = a.k - row0;
        if (wave_full && cnt >= M) {
            const uint32_t so = (uint32_t)((uint64_t)(row0 + 4 * j) * a.data.stride);
            __builtin_amdgcn_raw_ptr_buffer_load_lds(drsrc, (lvoid_t *)(img + j * 1024), 16, lane_off, so, 0, 0);
            return;
        }
        const int P = j * 64 + lane;
        const int r = P >> 4;
        const uint32_t go = span + (P & 15) * 16;
        if (wave_live && r < cnt && go < a.shard_size) {
            const uint32_t voff = (uint32_t)((uint64_t)(row0 + r) * a.data.stride + go);
            __builtin_amdgcn_raw_ptr_buffer_load_lds(drsrc, (lvoid_t *)(img + j * 1024), 16, voff, 0, 0, 0);
        } else {
            *(__attribute__((address_space(3))) u32x4 *)(img + j * 1024 + lane * 16) = u32x4{0, 0, 0, 0};
        }
    };
    auto stage_tab = [&](const uint32_t *src, int nbytes, int b) {
        const int npieces = nbytes / 16;
        const int P = wave * 64 + lane;
        const __amdgpu_buffer_rsrc_t trsrc = __builtin_amdgcn_make_buffer_rsrc((void *)src, 0, nbytes, 0x00020000);
        for (int base = 0; base < npieces; base += 256)
            if (base + P < npieces)
                __builtin_amdgcn_raw_ptr_buffer_load_lds(trsrc, (lvoid_t *)(ltab + b * TABB + base * 16 + wave * 1024),
                                                         16, (base + P) * 16, 0, 0, 0);
    };
    constexpr int IMGB = 2 * NTI * TB, FMGB = 2 * NTF * TB;  // bytes of one chunk's / the FFT's table image

    V acc[HM];
#pragma unroll
    for (int j = 0; j < NDMA; j++) stage_one(0, j);
    stage_tab(a.tw_ifft, IMGB, 0);
    // lane's LDS read base: register k holds row row0[k] (lower) / row0[k] | 1 << H0 (upper)
    const uint8_t *rd = img + half * ((1 << H0) * ROWB) + colb;
    for (int c = 0; c < a.nchunks; ++c) {
        wait_vm0();
        __syncthreads();
        V cur[HM];
#pragma unroll
        for (int k = 0; k < HM; k++) {
            const uint8_t *p = rd + SI.row0[k] * ROWB;
            cur[k].l[0] = *(const __attribute__((address_space(3))) uint32_t *)p;
            cur[k].h[0] = *(const __attribute__((address_space(3))) uint32_t *)(p + 32);
        }
        wait_lgkm0();  // reads done before the image is overwritten
        const bool more = c + 1 < a.nchunks;
        if (more) stage_tab(a.tw_ifft + (uint64_t)(c + 1) * (IMGB / 4), IMGB, (c + 1) & 1);
        else stage_tab(a.tw_fft, FMGB, (c + 1) & 1);
        if (more) {
#pragma unroll
            for (int j = 0; j < NDMA; j++) stage_one(c + 1, j);
        }
        run_split<IfftSplit<LOGM>>(cur, vgpr_lds_addr(ltab + (c & 1) * TABB) + (uint32_t)half * (NTI * TB));
        if (c == 0) {
#pragma unroll
            for (int k = 0; k < HM; k++) acc[k] = cur[k];
        } else {
#pragma unroll
            for (int k = 0; k < HM; k++) F::xor_into(acc[k], cur[k]);
        }
    }
    wait_vm0();
    __syncthreads();
    run_split<FftSplit<LOGM>>(acc, vgpr_lds_addr(ltab + (a.nchunks & 1) * TABB) + (uint32_t)half * (NTF * TB));
    if (!lane_live) return;
    // register k, half h holds parity row fin_row[h][k]; the two halves' rows differ by 1 << HF
    const uint64_t prow_step = (uint64_t)a.parity.stride;
    uint8_t *pbase = a.parity.base + soff + span + colb + (uint64_t)half * ((uint64_t)(1 << HF) * prow_step);
    uint32_t bad = 0;
#pragma unroll
    for (int k = 0; k < HM; k++) {
        const int row = SF.fin_row[0][k] + half * (1 << HF);
        if (row < a.p) {
            uint8_t *q = pbase + (uint64_t)SF.fin_row[0][k] * prow_step;
            if constexpr (VERIFY) {
                bad |= (*(const __attribute__((address_space(1))) uint32_t *)q ^ acc[k].l[0]) |
                       (*(const __attribute__((address_space(1))) uint32_t *)(q + 32) ^ acc[k].h[0]);
            } else {
                *(__attribute__((address_space(1))) uint32_t *)q = acc[k].l[0];
                *(__attribute__((address_space(1))) uint32_t *)(q + 32) = acc[k].h[0];
            }
        }
    }
    if constexpr (VERIFY) {
        flag_mismatch(a.mismatch, bad != 0);
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
        flag_mismatch(mismatch, Bytes16::diff(v, Bytes16::load(row_ptr(out, r), u)) != 0);
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
    if constexpr (F::SYM16) nunits = (a.shard_size >> 6) * (8 / F::W);
    else nunits = a.shard_size / (4 * F::W);
    dim3 grid((unsigned)((nunits + 255) / 256), (unsigned)a.nstripes);
    const bool table = a.data.table != nullptr || a.parity.table != nullptr;
    if (table) {
        if (verify) hipLaunchKernelGGL((k_encode_reg<F, LOGM, true, true>), grid, dim3(256), 0, s, a);
        else hipLaunchKernelGGL((k_encode_reg<F, LOGM, false, true>), grid, dim3(256), 0, s, a);
    } else {
        if (verify) hipLaunchKernelGGL((k_encode_reg<F, LOGM, true, false>), grid, dim3(256), 0, s, a);
        else hipLaunchKernelGGL((k_encode_reg<F, LOGM, false, false>), grid, dim3(256), 0, s, a);
    }
    return hipGetLastError();
}


// ---------------------------------------------------------------- LDS-resident transforms (n <= 256)
// One workgroup owns a 32W-byte tile (W = 4: two 64-byte blocks) of every row and
// keeps all n rows of it in LDS for the whole operation, so HBM sees each
// input row once and each output row once (the multi-pass path above re-reads
// the n-row work slab on every radix-4 layer).  Used for reconstruct
// (leopard16.go:390-570 / leopard8.go:439-695: scale-in, IFFT over n rows,
// formal derivative, FFT, reveal) and for encode with 32 < m <= 256
// (leopard16.go:128-224: chunked IFFT-m + XOR + FFT-m).
// Lane work items are (row group, unit) pairs; units are F16<4> (16 symbols:
// 16 low bytes + the 16 high bytes 32 bytes later) or F8<4> (16 bytes).
// Twiddle tables come from global memory (identical for every workgroup, so
// they stay in L1/L2).
// Tile width per unit type: 4 units of F16<W> (8W bytes) or 8 of F8<W> (4W
// bytes), i.e. 32W bytes of each row per workgroup.  The launchers use
// 128-byte tiles (W = 4), or 64-byte tiles (W = 2) when 128-byte tiles would
// give fewer than kLdsMinGrid workgroups (C5's 32 KiB per-GPU byte range:
// 57.0 -> 52.8 us; full-size C4 / C5 are faster at 128 bytes).  A GF(2^16)
// tile must cover whole 64-byte blocks (low bytes [0,32), high bytes
// [32,64)), so W = 1 (32-byte tiles) is invalid: the parity tests reject it.
constexpr uint64_t kLdsMinGrid = 512;
// k_enc_lds keeps the accumulator in registers for even log m
constexpr bool enc_acc_regs(int logm) { return logm % 2 == 0 && logm >= 4; }
constexpr bool kLdsBranchFree = 1;  // lane-varying passes: branch-free multiplies

// rs_debug_set_path("unit_width", 0 / 1) forces the per-launch unit-width
// choices below (LDS tiles of 128 vs 64 bytes; GF(2^8) register units of 16
// vs 4 bytes) so the parity tests cover every variant at small sizes; -1 (the
// default) keeps the automatic choice.  Testing only.
bool pick_narrow(bool automatic) {
    const int o = unit_width_override();
    return o < 0 ? automatic : o == 1;
}

// PK (the reconstruct kernels, k_rec_lds): 64-byte GF(2^16) tiles (W = 2)
// keep a unit's 8 low and 8 high bytes together in one 16-byte LDS word,
// rows unpadded, so each unit access is one ds_read_b128 / ds_write_b128
// (256 B per LDS clock) instead of a ds_read2_b64 / ds_write2_b64 of the two
// halves 32 bytes apart (128 B per clock), and the lane groups of the
// n = 2048 passes fall on distinct banks but for a few stores
// (scripts/lds_bank_model.py: LDS-array cycles 53.2k -> 22.0k per tile;
// SQ_LDS_BANK_CONFLICT -95 %, profiles/r05_sq_counters.txt, r05_lds_pack_ab.txt).  Otherwise the halves keep their global
// (Leopard 64-byte block) order in rows padded by 16 bytes; the encoder keeps
// that layout (packed, its 64-byte-tile variant spills).
//
// PK = 2 (the n >= 1024 reconstruct, round 6): half tiles, 32 bytes of a row
// per workgroup (two 16-byte units: symbols 16j .. 16j + 15 of a 64-byte
// block, j = the tile's half), so the n x 32-byte image (64 KB at n = 2048)
// lets two workgroups share a CU.  The caller addresses a half tile from its
// block (tile = block * 64) and adds the half's unit offset (2j) to u.
// PK = 4 (n = 8192): quarter tiles, one 16-byte unit (symbols 8j .. 8j + 7)
// of a row per workgroup, the 8192 x 16-byte image 128 KB.
template <class F, int PK = 0>
struct LTile {
    static_assert(!F::SYM16 || F::W >= 2, "a GF(2^16) LDS tile must cover whole 64-byte blocks (W >= 2)");
    static_assert(PK < 2 || (F::SYM16 && F::W == 2), "half / quarter tiles: GF(2^16) 16-byte units");
    static constexpr bool W16 = F::SYM16;
    static constexpr int TB = (PK == 4 ? 8 : PK == 2 ? 16 : 32) * F::W;  // bytes of each row owned by a workgroup
    static constexpr bool PACK = PK != 0 && W16 && F::W == 2;
    static constexpr int ROW = PACK ? TB : TB + 16;  // LDS row stride
    static constexpr int UB = W16 ? 8 * F::W : 4 * F::W;  // global bytes per unit
    static constexpr int U = TB / UB;                     // units per tile
    typedef typename F::Vec V;
    // LDS byte offset of unit u's low (h = 0) or high (h = 1) half in `row`
    __device__ static uint32_t loff(int row, int u, int h) {
        if constexpr (PACK) return (uint32_t)(row * ROW + 16 * u + 8 * h);
        return (uint32_t)(row * ROW + F::off(u) + 32 * h);
    }
    __device__ static V get(const uint8_t *lds, int row, int u) {
        V v;
        if constexpr (PACK) {
            uint32_t x[4];
            ldw_lds<4>(lds + loff(row, u, 0), x);
            v.l[0] = x[0], v.l[1] = x[1], v.h[0] = x[2], v.h[1] = x[3];
        } else if constexpr (W16) {
            ldw_lds<F::W>(lds + loff(row, u, 0), v.l);
            ldw_lds<F::W>(lds + loff(row, u, 1), v.h);
        } else {
            ldw_lds<F::W>(lds + loff(row, u, 0), v.b);
        }
        return v;
    }
    __device__ static void put(uint8_t *lds, int row, int u, const V &v) {
        typedef typename VecOf<F::W>::T T;
        auto st = [](uint8_t *q, const uint32_t(&w)[F::W]) {
            T x;
            if constexpr (F::W == 1) x = w[0];
            else
#pragma unroll
                for (int i = 0; i < F::W; i++) x[i] = w[i];
            *(__attribute__((address_space(3))) T *)(q) = x;
        };
        if constexpr (PACK) {
            typedef typename VecOf<4>::T T4;
            const T4 x = {v.l[0], v.l[1], v.h[0], v.h[1]};
            *(__attribute__((address_space(3))) T4 *)(lds + loff(row, u, 0)) = x;
        } else if constexpr (W16) {
            st(lds + loff(row, u, 0), v.l);
            st(lds + loff(row, u, 1), v.h);
        } else {
            st(lds + loff(row, u, 0), v.b);
        }
    }
    // Unit u of the tile starting at byte `tile` exists in a row of S bytes.
    __device__ static bool valid(uint64_t tile, uint64_t S, int u) { return tile + (uint64_t)(F::off(u) & ~63) < S; }
};

// Row sources / sinks of a pass: the LDS image by default; the first pass of
// a transform may read its rows from HBM (LdsIn replaced by a loader) and the
// last may write them out (to HBM, or XOR them into the encoder's
// accumulator), so the tile is not staged through LDS an extra time.
template <class F, int PK = 0>
struct LdsIO {
    uint8_t *lds;
    __device__ typename F::Vec operator()(int row, int u) const { return LTile<F, PK>::get(lds, row, u); }
    __device__ void operator()(int row, int u, const typename F::Vec &v) const { LTile<F, PK>::put(lds, row, u, v); }
};

template <class T> struct IsLdsIO : std::false_type {};
template <class F, int PK> struct IsLdsIO<LdsIO<F, PK>> : std::true_type {};

template <class Fn, int... Is>
__device__ __forceinline__ void cfor_impl(Fn &&f, std::integer_sequence<int, Is...>) {
    (f(std::integral_constant<int, Is>{}), ...);
}
template <int N, class Fn>
__device__ __forceinline__ void cfor(Fn &&f) {
    cfor_impl(f, std::make_integer_sequence<int, N>{});
}

// Barrier between LDS passes: LDS-only (s_waitcnt lgkmcnt(0); s_barrier), so
// global loads a kernel has in flight (the encoder's next-chunk prefetch) are
// not drained at every pass as __syncthreads() would.  The passes communicate
// only through LDS; global stores are never read back inside a launch.
__device__ __forceinline__ void lds_sync() { __syncthreads(); }

// One radix-4 pass (rows i, i+d, i+2d, i+3d; twiddles m01, m02, m23 at
// tw + 3*g) over the active groups, or a radix-2 pass.  in(row, u) supplies
// the rows, out(row, u, v) takes the results.
// need (forward passes only): skip groups none of whose rows is read later --
// the pruning of errorBitfield.fftDIT (leopard16.go:1215-1252); the rows that
// are read come out identical.
template <class F, bool INV, class In, class Out, class NeedT, int NT = 256, int PK = 0>
__device__ __forceinline__ void lds_pass(int dist, int radix, int groups_active, const uint32_t *__restrict__ tw,
                                         NeedT need, const In &in, const Out &out) {
    typedef LTile<F, PK> L;
    typedef typename F::Vec V;
    constexpr int U = L::U;
    if (radix == 4) {
        const int items = groups_active * dist * U;
        const int ld = __builtin_ctz((unsigned)dist);  // dist is a power of two: no integer division
        auto group = [&](int it, int g, auto bf) {
            constexpr bool BF = decltype(bf)::value;
            const int q = it / U, u = it - q * U;
            const int j = q & (dist - 1);
            const int i = g * 4 * dist + j;
            if (!INV && !rows_needed(need, g * 4 * dist, 4 * dist)) return;
            const uint32_t *t = tw + (uint64_t)g * 3 * F::TWD;
            V x0, x1, x2, x3;
            if constexpr (HasRaw<In>::value) {
                // the four rows' addresses, then their loads, then their
                // scale tables: a load waits only for its own kind (with the
                // steps interleaved per row every row waited out the previous
                // row's HBM trip: the memory counter retires in order)
                const RowLoc l0 = in.locate(i, u), l1 = in.locate(i + dist, u), l2 = in.locate(i + 2 * dist, u),
                             l3 = in.locate(i + 3 * dist, u);
                __builtin_amdgcn_sched_barrier(0);
                const auto r0 = in.fetch(l0), r1 = in.fetch(l1), r2 = in.fetch(l2), r3 = in.fetch(l3);
                __builtin_amdgcn_sched_barrier(0);
                x0 = in.scale(i, r0), x1 = in.scale(i + dist, r1), x2 = in.scale(i + 2 * dist, r2), x3 = in.scale(i + 3 * dist, r3);
            } else {
                x0 = in(i, u), x1 = in(i + dist, u), x2 = in(i + 2 * dist, u), x3 = in(i + 3 * dist, u);
            }
            if constexpr (INV) ifft4<F, BF>(x0, x1, x2, x3, t);
            else fft4<F, BF>(x0, x1, x2, x3, t);
            out(i, u, x0);
            out(i + dist, u, x1);
            out(i + 2 * dist, u, x2);
            out(i + 3 * dist, u, x3);
        };
        if (dist * U >= 64) {
            // A wave's 64 items (aligned) lie in one group: the group index is
            // wave-uniform, so its twiddle tables come in by scalar loads and
            // the zero-twiddle test is a scalar branch.
            for (int it = threadIdx.x; it < items; it += NT)
                group(it, __builtin_amdgcn_readfirstlane((it / U) >> ld), std::false_type{});
        } else
        {
            for (int it = threadIdx.x; it < items; it += NT) group(it, (it / U) >> ld, std::bool_constant<kLdsBranchFree>{});
        }
    } else {
        // inverse: pairs (j, j + dist), j < dist, one twiddle; forward: dist 1, pairs (2g, 2g+1), twiddle g
        const int pairs = INV ? dist : groups_active;
        for (int it = threadIdx.x; it < pairs * U; it += NT) {
            const int q = it / U, u = it - q * U;
            const int rx = INV ? q : 2 * q, ry = INV ? q + dist : 2 * q + 1;
            if (!INV && !rows_needed(need, 2 * q, 2)) continue;
            const uint32_t *t = INV ? tw : tw + (uint64_t)q * F::TWD;
            V x = in(rx, u), y = in(ry, u);
            if constexpr (INV) ifft2<F>(x, y, t);
            else fft2<F>(x, y, t);
            out(rx, u, x);
            out(ry, u, y);
        }
    }
    lds_sync();
}

// Full transform over 2^LOGN LDS rows with the reference's pass structure
// (gf_host.cpp ifft_passes / fft_passes) and its mtrunc group skipping.  The
// first pass reads through `in`, the last writes through `out`.  A first pass
// that does not read the LDS image runs every group (rows past mtrunc come in
// as zero, and zero rows transform to zero rows): later passes read those rows.
// OUT_P1: pass P1 - 1 (the last this call runs) writes through `out` too.
template <class F, bool INV, int LOGN, class In, class Out, class NeedT = NoNeed, int P0 = 0, int P1 = 32, int NT = 256,
          bool OUT_P1 = false, int PK = 0>
__device__ __forceinline__ void lds_transform(uint8_t *lds, int mtrunc, const uint32_t *__restrict__ tw,
                                              NeedT need, const In &in, const Out &out) {
    constexpr int N = 1 << LOGN, NP4 = LOGN / 2, NP = NP4 + (LOGN & 1);
    const LdsIO<F, PK> lio{lds};
    cfor<NP>([=](auto PI) {  // by value: a captured reference to `need` kept it on the stack
        constexpr int p = decltype(PI)::value;
        if constexpr (p >= P0 && p < P1) {  // passes outside [P0, P1) are run by the caller (fused)
        constexpr bool radix4 = p < NP4;
        // IFFT: radix-4 passes at dist 4^p (groups N / (4 dist)), then radix-2 at dist N/2;
        // FFT: radix-4 passes at dist N / 4^(p+1) (groups 4^p), then radix-2 at dist 1
        constexpr int dist = INV ? (1 << (2 * p)) : (radix4 ? N >> (2 * (p + 1)) : 1);
        constexpr int groups = radix4 ? N / (4 * dist) : 1;
        constexpr int slot = [] {
            int sl = 0;
            for (int q = 0; q < p; q++) sl += 3 * (INV ? N / (4 << (2 * q)) : (1 << (2 * q)));
            return sl;
        }();
        constexpr bool from_hbm = p == 0 && !IsLdsIO<In>::value;  // every group (see above)
        int active;
        if constexpr (radix4) {
            active = (mtrunc + 4 * dist - 1) / (4 * dist);
            if (active > groups) active = groups;
            if constexpr (from_hbm && INV && p < NP - 1) {
                // groups past mtrunc hold zero rows: zero their LDS rows instead
                // of transforming them (the pass's barrier covers these stores)
                const int z0 = active * 4 * dist;
                for (int it = threadIdx.x; it < (N - z0) * LTile<F, PK>::U; it += NT)
                    lio(z0 + it / LTile<F, PK>::U, it % LTile<F, PK>::U, F::zero());
            } else if constexpr (from_hbm) {
                active = groups;
            }
        } else {
            active = INV ? 1 : (mtrunc + 1) / 2 < N / 2 && !from_hbm ? (mtrunc + 1) / 2 : N / 2;
        }
        const uint32_t *t = tw + (uint64_t)slot * F::TWD;
        auto run = [=](const auto &pin, const auto &pout) {
            if constexpr (INV) lds_pass<F, INV, std::decay_t<decltype(pin)>, std::decay_t<decltype(pout)>, NoNeed, NT, PK>(dist, radix4 ? 4 : 2, active, t, NoNeed{}, pin, pout);
            else lds_pass<F, INV, std::decay_t<decltype(pin)>, std::decay_t<decltype(pout)>, NeedT, NT, PK>(dist, radix4 ? 4 : 2, active, t, need, pin, pout);
        };
        constexpr bool to_out = p == NP - 1 || (OUT_P1 && p == P1 - 1);
        if constexpr (from_hbm) {
            if constexpr (to_out) run(in, out);
            else run(in, lio);
        } else if constexpr (to_out) {
            run(lio, out);
        } else {
            run(lio, lio);
        }
        }
    });
}
template <class F, bool INV, int LOGN>
__device__ __forceinline__ void lds_transform(uint8_t *lds, int mtrunc, const uint32_t *__restrict__ tw) {
    const LdsIO<F> lio{lds};
    lds_transform<F, INV, LOGN>(lds, mtrunc, tw, NoNeed{}, lio, lio);
}

// (lo, hi) <-> (lo ^ D(hi), hi) on every symbol of v (t: make_sub_dmap table).
template <class F>
__device__ __forceinline__ void sub_swap(typename F::Vec &v, const uint32_t *__restrict__ t) {
#pragma unroll
    for (int i = 0; i < F::W; i++) {
        const uint32_t h = v.h[i];
        v.l[i] = xor3(v.l[i] ^ perm(t[1], t[0], h & 0x07070707u), perm(t[3], t[2], (h >> 3) & 0x07070707u),
                      perm(t[4], t[4], (h >> 6) & 0x03030303u));
    }
}

// LDS sink that changes rows into subfield coordinates on their way in.
template <class F, int PK = 0>
struct LdsPsi {
    uint8_t *lds;
    const uint32_t *dmap;
    __device__ void operator()(int row, int u, const typename F::Vec &v0) const {
        typename F::Vec v = v0;
        sub_swap<F>(v, dmap);
        LTile<F, PK>::put(lds, row, u, v);
    }
};

// Reconstruct (leopard16.go:432-568) of one stripe, one 32W-byte tile (LTile) per workgroup.
// F scales rows in and out (full-field tables); FT runs the transforms (F, or
// F16S when every transform twiddle lies in GF(2^8)).  The scale-in feeds the
// IFFT's first pass straight from HBM and the FFT's last pass reveals straight
// to the output rows.
// Threads per workgroup: 256, and 1024 for n >= 1024 (the n x 64-byte image
// leaves room for one or two workgroups per CU: 16 waves keep the SIMDs fed).
template <int LOGN> constexpr int rec_lds_threads() { return LOGN >= 10 ? 1024 : 256; }
// PKV = 2 (half tiles, n >= 1024): two 512-thread workgroups per CU, so one
// workgroup's pass barriers are covered by the other's work.
// n = 4096 (round 6): half tiles only (the 4096 x 32-byte image is 128 KB),
// one 1024-thread workgroup per CU.
template <int LOGN, int PKV> constexpr int rec_threads() {
    return PKV == 4 ? 1024 : PKV == 2 ? (LOGN >= 12 ? 1024 : 512) : rec_lds_threads<LOGN>();
}

// n = 512..2048 with BSUB: the transforms in subfield coordinates wherever
// every twiddle of a pass lies in GF(2^8) (rec_big_sub_passes; RecArgs::tw_*_sub).
template <int LOGN> struct BigSub {
    static constexpr int NI = big_sub_ifft_first(LOGN);  // IFFT passes [NI, end) subfield
    static constexpr int FEND = big_sub_fft_end(LOGN);   // FFT passes [0, FEND) subfield
};

template <class F, class FT, int LOGN, bool BSUB = false, int PKV = 1>
__global__ void __launch_bounds__((rec_threads<LOGN, PKV>()), (PKV == 2 && LOGN < 12 ? 2 : 1)) k_rec_lds(RecArgs a) {
    typedef LTile<F, PKV> L;  // packed 64-byte tiles (LTile PK), or half / quarter tiles (PKV = 2 / 4)
    typedef typename F::Vec V;
    constexpr int N = 1 << LOGN, U = L::U, NT = rec_threads<LOGN, PKV>();
    constexpr int K = (N * U + NT - 1) / NT;  // derivative outputs per thread
    __shared__ __attribute__((aligned(16))) uint8_t lds[N * L::ROW];
    uint32_t bx = blockIdx.x;
    if constexpr (PKV >= 2) {
        // half (quarter) tiles: the T = 2 PKV tiles of a 128-byte line go to one
        // XCD: blocks 8Tq + x + 8j (j < T) take tiles 8Tq + Tx + j
        constexpr uint32_t T = 2 * PKV, G = 8 * T;
        if (bx < (gridDim.x & ~(G - 1))) bx = (bx & ~(G - 1)) | ((bx & 7u) * T) | ((bx >> 3) & (T - 1));
    } else if constexpr (LOGN > 8) {
        // 64-byte tiles: the two tiles of a 128-byte line go to one XCD
        // (workgroups are dealt round-robin over the 8 XCDs, each with its own
        // L2): blocks 16q + x and 16q + x + 8 take tiles 16q + 2x, 16q + 2x + 1
        if (bx < (gridDim.x & ~15u)) bx = (bx & ~15u) | ((bx & 7u) << 1) | ((bx >> 3) & 1u);
    }
    // a half tile is addressed from its 64-byte block, its units from uo on
    const uint64_t tile = PKV >= 2 ? (uint64_t)(bx / PKV) * 64 : (uint64_t)bx * L::TB;
    const int uo = PKV >= 2 ? L::U * (int)(bx % PKV) : 0;
    uint8_t *const sbase = a.base ? a.base + (uint64_t)blockIdx.y * a.stripe_stride : nullptr;  // this stripe
    // work row r = present shard * errLocs[r] (mulgf16 through the table), or 0.
    // Branch-free, so the four rows of a first-pass item issue their loads
    // together: a missing row (or a unit past the row end) loads from a
    // readable stand-in, the scale-in table, and its product is dropped.
    // (With a branch per row each row waited out its own HBM round trip.)
    // Two forms: rows at a stride from the stripe base (src_idx), or a row table.
    // locate(r, u): where the row's unit is; fetch: its load; scale: times
    // errLocs[r].  lds_pass runs each step for an item's four rows before the
    // next, so each kind of load waits for its own kind only.
    struct ScaleInStrided {
        const RecArgs &a;
        uint64_t tile;
        uint8_t *sbase;
        int uo;
        __device__ RowLoc locate(int r, int u) const {
            const int i = a.src_idx[r];
            const bool live = i >= 0 && L::valid(tile, a.S, u);
            return RowLoc{live ? sbase + (uint64_t)i * a.stride + tile : (const uint8_t *)a.tw_in, live ? u + uo : 0, live};
        }
        __device__ RawRow<F> fetch(const RowLoc &l) const { return RawRow<F>{F::load(l.p, l.u), l.live}; }
        __device__ V scale(int r, const RawRow<F> &y) const { return scale_row<F>(y, a.tw_in + (uint64_t)r * F::TWD); }
        __device__ V operator()(int r, int u) const { return scale(r, fetch(locate(r, u))); }
    };
    struct ScaleInTable {
        const RecArgs &a;
        uint64_t tile;
        int uo;
        __device__ RowLoc locate(int r, int u) const {
            const uint8_t *src = a.src[r];
            const bool live = src && L::valid(tile, a.S, u);
            return RowLoc{live ? src + tile : (const uint8_t *)a.tw_in, live ? u + uo : 0, live};
        }
        __device__ RawRow<F> fetch(const RowLoc &l) const { return RawRow<F>{F::load(l.p, l.u), l.live}; }
        __device__ V scale(int r, const RawRow<F> &y) const { return scale_row<F>(y, a.tw_in + (uint64_t)r * F::TWD); }
        __device__ V operator()(int r, int u) const { return scale(r, fetch(locate(r, u))); }
    };
    // n > 256: the revealed-row mask and the output indices come from HBM
    constexpr bool BIG = LOGN > 8;
    typedef typename std::conditional<BIG, NeedMem, Need>::type NeedT;
    auto need_of = [&]() {
        if constexpr (BIG) return NeedMem{(const __attribute__((address_space(4))) uint32_t *)a.need_w};
        else return load_need(a.need);
    };
    // reveal: shard = work[pos] * (modulus - errLocs[pos])
    struct Reveal {
        const RecArgs &a;
        uint64_t tile;
        uint8_t *sbase;
        NeedT nw;
        int uo;
        __device__ void operator()(int r, int u, const V &x) const {
            int j;  // output index of work row r (-1: not revealed)
            if constexpr (BIG) j = a.rev[r];
            else j = reveal_index(nw, a.m, r);  // from the revealed-row mask
            if (j < 0 || !L::valid(tile, a.S, u)) return;
            V v = F::zero();
            F::mul_add(v, x, a.tw_out + (uint64_t)j * F::TWD);
            uint8_t *dst = sbase ? sbase + (uint64_t)a.dst_idx[j] * a.stride : a.dst[j];
            F::store(dst + tile, u + uo, v);
        }
    };
    const LdsIO<FT, PKV> lio{lds};
    typedef F16S<F::W> FS;  // (BSUB only)
    if constexpr (BSUB) {
        // full-field passes, the last one writing subfield coordinates, then subfield passes
        if (sbase)
            lds_transform<F, true, LOGN, ScaleInStrided, LdsPsi<F, PKV>, NoNeed, 0, BigSub<LOGN>::NI, NT, true, PKV>(
                lds, a.mtrunc, a.tw_ifft, NoNeed{}, ScaleInStrided{a, tile, sbase, uo}, LdsPsi<F, PKV>{lds, a.tw_dmap});
        else
            lds_transform<F, true, LOGN, ScaleInTable, LdsPsi<F, PKV>, NoNeed, 0, BigSub<LOGN>::NI, NT, true, PKV>(
                lds, a.mtrunc, a.tw_ifft, NoNeed{}, ScaleInTable{a, tile, uo}, LdsPsi<F, PKV>{lds, a.tw_dmap});
        lds_transform<FS, true, LOGN, LdsIO<FS, PKV>, LdsIO<FS, PKV>, NoNeed, BigSub<LOGN>::NI, 32, NT, false, PKV>(
            lds, a.mtrunc, a.tw_ifft_sub, NoNeed{}, LdsIO<FS, PKV>{lds}, LdsIO<FS, PKV>{lds});
    } else {
        // the first pass (it reads the rows) per row form, then the rest
        if (sbase)
            lds_transform<FT, true, LOGN, ScaleInStrided, LdsIO<FT, PKV>, NoNeed, 0, 1, NT, false, PKV>(
                lds, a.mtrunc, a.tw_ifft, NoNeed{}, ScaleInStrided{a, tile, sbase, uo}, lio);
        else
            lds_transform<FT, true, LOGN, ScaleInTable, LdsIO<FT, PKV>, NoNeed, 0, 1, NT, false, PKV>(
                lds, a.mtrunc, a.tw_ifft, NoNeed{}, ScaleInTable{a, tile, uo}, lio);
        lds_transform<FT, true, LOGN, LdsIO<FT, PKV>, LdsIO<FT, PKV>, NoNeed, 1, 32, NT, false, PKV>(lds, a.mtrunc, a.tw_ifft, NoNeed{}, lio, lio);
    }
    const Reveal rv{a, tile, sbase, need_of(), uo};
    // formal derivative, closed form: out[r] = in[r] ^ XOR_{b: bit b of r clear} in[r | 2^b]
    if constexpr (LOGN >= 3) {
        // fused with the FFT's first pass (radix-4 at dist D = N/4, one group,
        // twiddle slot 0): a thread forms the derivative of its four rows
        // i + aD from the IFFT image (the a-bit terms from the rows it holds),
        // transforms them, and stores them after every thread has read.
        constexpr int D = N / 4;
        constexpr int KF = (D * U + NT - 1) / NT;  // fused items per thread
        V x[KF][4];
#pragma unroll
        for (int k = 0; k < KF; k++) {
            const int it = threadIdx.x + NT * k;
            if (it < D * U) {
                const int i = it / U, u = it - i * U;
                V X[4];
#pragma unroll
                for (int q = 0; q < 4; q++) X[q] = L::get(lds, i + q * D, u);
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    x[k][q] = X[q];
                    if (!(q & 1)) F::xor_into(x[k][q], X[q | 1]);
                    if (!(q & 2)) F::xor_into(x[k][q], X[q | 2]);
                    for (int b = 1; b < D; b <<= 1)
                        if (!(i & b)) F::xor_into(x[k][q], L::get(lds, (i | b) + q * D, u));
                }
                if constexpr (BSUB) fft4<FS>(x[k][0], x[k][1], x[k][2], x[k][3], a.tw_fft_sub);
                else fft4<FT>(x[k][0], x[k][1], x[k][2], x[k][3], a.tw_fft);
            }
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < KF; k++) {
            const int it = threadIdx.x + NT * k;
            if (it < D * U) {
                const int i = it / U, u = it - i * U;
#pragma unroll
                for (int q = 0; q < 4; q++) L::put(lds, i + q * D, u, x[k][q]);
            }
        }
        __syncthreads();
        if (a.prune) {
            if constexpr (BSUB) {
                // subfield passes up to FEND, the last one writing normal coordinates back, then full-field
                lds_transform<FS, false, LOGN, LdsIO<FS, PKV>, LdsPsi<F, PKV>, NeedT, 1, BigSub<LOGN>::FEND, NT, true, PKV>(
                    lds, a.mtrunc, a.tw_fft_sub, need_of(), LdsIO<FS, PKV>{lds}, LdsPsi<F, PKV>{lds, a.tw_dmap});
                lds_transform<F, false, LOGN, LdsIO<F, PKV>, Reveal, NeedT, BigSub<LOGN>::FEND, 32, NT, false, PKV>(
                    lds, a.mtrunc, a.tw_fft, need_of(), LdsIO<F, PKV>{lds}, rv);
            } else {
                lds_transform<FT, false, LOGN, LdsIO<FT, PKV>, Reveal, NeedT, 1, 32, NT, false, PKV>(lds, a.mtrunc, a.tw_fft, need_of(), lio, rv);
            }
        } else {
            if constexpr (BSUB) {
                lds_transform<FS, false, LOGN, LdsIO<FS, PKV>, LdsPsi<F, PKV>, NoNeed, 1, BigSub<LOGN>::FEND, NT, true, PKV>(
                    lds, a.mtrunc, a.tw_fft_sub, NoNeed{}, LdsIO<FS, PKV>{lds}, LdsPsi<F, PKV>{lds, a.tw_dmap});
                lds_transform<F, false, LOGN, LdsIO<F, PKV>, Reveal, NoNeed, BigSub<LOGN>::FEND, 32, NT, false, PKV>(
                    lds, a.mtrunc, a.tw_fft, NoNeed{}, LdsIO<F, PKV>{lds}, rv);
            } else {
                lds_transform<FT, false, LOGN, LdsIO<FT, PKV>, Reveal, NoNeed, 1, 32, NT, false, PKV>(lds, a.mtrunc, a.tw_fft, NoNeed{}, lio, rv);
            }
        }
        return;
    }
    {
        V o[K];
#pragma unroll
        for (int k = 0; k < K; k++) {
            const int it = threadIdx.x + NT * k;
            if (it < N * U) {
                const int r = it / U, u = it - r * U;
                o[k] = L::get(lds, r, u);
                for (int b = 1; b < N; b <<= 1)
                    if (!(r & b)) F::xor_into(o[k], L::get(lds, r | b, u));
            }
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < K; k++) {
            const int it = threadIdx.x + NT * k;
            if (it < N * U) {
                const int r = it / U, u = it - r * U;
                L::put(lds, r, u, o[k]);
            }
        }
        __syncthreads();
    }
    if (a.prune) {
        lds_transform<FT, false, LOGN, LdsIO<FT, PKV>, Reveal, NeedT, 0, 32, NT, false, PKV>(lds, a.mtrunc, a.tw_fft, need_of(), lio, rv);
    } else {
        lds_transform<FT, false, LOGN, LdsIO<FT, PKV>, Reveal, NoNeed, 0, 32, NT, false, PKV>(lds, a.mtrunc, a.tw_fft, NoNeed{}, lio, rv);
    }
}

// Encode for 32 < m <= 256 (leopard16.go:128-224 / leopard8.go:153-277):
// acc and the current chunk both live in LDS (2 x m rows of the tile).  Each
// chunk's first IFFT pass reads its rows from HBM, its last XORs the results
// into acc (chunk 0: writes acc), and the FFT's last pass writes the parity
// rows (or compares them, verify).
// FT: the field of the final FFT (F16S: subfield coordinates, EncodeArgs::tw_fft_sub).
// ISUB: the chunk IFFTs' subfield passes (EncodeArgs::tw_ifft_sub; needs FT = F16S).
// m = 512, 1024 (GF(2^16), round 6): 64-byte tiles (F16<2>) and one
// 1024-thread workgroup per CU, the m x 80-byte image(s) taking 80 KB of LDS
// (m = 1024: acc in registers, one image; m = 512: acc and chunk images);
// m = 2048: 32-byte half tiles (LTile PK = 2), acc and chunk images 128 KB;
// m = 4096: 16-byte quarter tiles (PK = 4), acc in registers, the image 64 KB.
template <int LOGM> constexpr int enc_threads() { return LOGM >= 9 ? 1024 : 256; }
template <int LOGM> constexpr int enc_pk() { return LOGM >= 12 ? 4 : LOGM >= 11 ? 2 : 0; }
template <class F, int LOGM, bool VERIFY, class FT = F, bool ISUB = false>
__global__ void __launch_bounds__((enc_threads<LOGM>()), (LOGM >= 9 ? 1 : 4)) k_enc_lds(EncodeArgs a) {
    constexpr int PK = enc_pk<LOGM>();
    typedef LTile<F, PK> L;
    typedef typename F::Vec V;
    constexpr int M = 1 << LOGM, NT = enc_threads<LOGM>();
    extern __shared__ __attribute__((aligned(16))) uint8_t lds_dyn[];
    constexpr bool ACCR = enc_acc_regs(LOGM);
    uint8_t *acc = lds_dyn, *cur = ACCR ? lds_dyn : lds_dyn + M * L::ROW;
    uint32_t bx = blockIdx.x;
    if constexpr (PK >= 2) {
        // half (quarter) tiles: the 2 PK tiles of a 128-byte line go to one XCD (as k_rec_lds)
        constexpr uint32_t T = 2 * PK, G = 8 * T;
        if (bx < (gridDim.x & ~(G - 1))) bx = (bx & ~(G - 1)) | ((bx & 7u) * T) | ((bx >> 3) & (T - 1));
    }
    // a half (quarter) tile is addressed from its 64-byte block, its units from uo on
    constexpr uint32_t PD = PK >= 2 ? PK : 1;  // tiles per 64-byte block
    const uint64_t tile = PK >= 2 ? (uint64_t)(bx / PD) * 64 : (uint64_t)bx * L::TB;
    const int uo = PK >= 2 ? L::U * (int)(bx % PD) : 0;
    const uint64_t soff = (uint64_t)blockIdx.y * a.stripe_stride;
    constexpr int its = ifft_slot_count(LOGM);
    struct ChunkIn {
        const EncodeArgs &a;
        int row0, cnt;
        uint64_t soff, tile;
        int uo;
        __device__ V operator()(int r, int u) const {
            if (r < cnt && L::valid(tile, a.shard_size, u)) return F::load(row_ptr(a.data, row0 + r) + soff + tile, u + uo);
            return F::zero();
        }
    };
    struct AccXor {
        uint8_t *acc;
        __device__ void operator()(int r, int u, const V &x) const {
            V v = L::get(acc, r, u);
            F::xor_into(v, x);
            L::put(acc, r, u, v);
        }
    };
    constexpr bool SUB = !std::is_same<F, FT>::value;
    struct ParityOut {
        const EncodeArgs &a;
        uint64_t soff, tile;
        int uo;
        uint32_t *bad;
        __device__ void operator()(int r, int u, const V &v0) const {
            if (r >= a.p || !L::valid(tile, a.shard_size, u)) return;
            V v = v0;
            if constexpr (SUB) sub_swap<F>(v, a.tw_dmap);  // back to (lo, hi)
            uint8_t *prow = row_ptr(a.parity, r) + soff + tile;
            if constexpr (VERIFY) *bad |= F::diff(v, F::load(prow, u + uo));
            else F::store(prow, u + uo, v);
        }
    };
    // m >= 512 (FSPLIT): the FFT's passes from FEND on are full-field, so its
    // subfield passes end by writing normal coordinates back (LdsPsi) and the
    // last pass stores through this sink, which converts nothing.
    struct ParityOutFull {
        const EncodeArgs &a;
        uint64_t soff, tile;
        int uo;
        uint32_t *bad;
        __device__ void operator()(int r, int u, const V &v) const {
            if (r >= a.p || !L::valid(tile, a.shard_size, u)) return;
            uint8_t *prow = row_ptr(a.parity, r) + soff + tile;
            if constexpr (VERIFY) *bad |= F::diff(v, F::load(prow, u + uo));
            else F::store(prow, u + uo, v);
        }
    };
    if constexpr (ACCR) {
        // acc in registers: the IFFT's last pass and the FFT's first are both
        // one radix-4 group at dist D = M/4 with the same item -> (rows, unit)
        // mapping, so a thread keeps acc rows i + qD of its items across the
        // chunks and the LDS holds only the current chunk.
        constexpr int NP = LOGM / 2, D = M / 4;
        constexpr int KF = (D * L::U + NT - 1) / NT;  // items per thread
        constexpr int last = [] {  // twiddle slot of the IFFT's last pass
            int sl = 0;
            for (int q = 0; q < NP - 1; q++) sl += 3 * (M / (4 << (2 * q)));
            return sl;
        }();
        V ar[KF][4];
        // chunk IFFT passes in subfield coordinates from ifft_nff[c] on
        // (6 v_perm_b32 per product instead of 12; EncodeArgs::tw_ifft_sub)
        constexpr bool isub = SUB && ISUB;
        for (int c = 0; c < a.nchunks; c++) {
            const int row0 = c * M, cnt = a.k - row0 < M ? a.k - row0 : M;
            const uint32_t *tw = a.tw_ifft + (uint64_t)c * its * F::TWD;
            const uint32_t *tws = isub ? a.tw_ifft_sub + (uint64_t)c * its * FT::TWD : nullptr;
            const LdsIO<F, PK> lio{cur};
            const ChunkIn in{a, row0, cnt, soff, tile, uo};
            if constexpr (isub) {
                // full-field passes, the last one writing subfield coordinates, then subfield passes
                const LdsPsi<F, PK> psi{cur, a.tw_dmap};
                const LdsIO<FT, PK> lios{cur};
                // 1 or 2, and up to 3 for m = 1024 (codec.cpp upload_ifft_sub)
                const int nff = a.ifft_nff[c];
                if (nff == 1) lds_transform<F, true, LOGM, ChunkIn, LdsPsi<F, PK>, NoNeed, 0, 1, NT, true, PK>(cur, cnt, tw, NoNeed{}, in, psi);
                else lds_transform<F, true, LOGM, ChunkIn, LdsIO<F, PK>, NoNeed, 0, 1, NT, false, PK>(cur, cnt, tw, NoNeed{}, in, lio);
                if constexpr (LOGM >= 10) {
                    if (nff == 2) lds_transform<F, true, LOGM, LdsIO<F, PK>, LdsPsi<F, PK>, NoNeed, 1, 2, NT, true, PK>(cur, cnt, tw, NoNeed{}, lio, psi);
                    else if (nff == 3) lds_transform<F, true, LOGM, LdsIO<F, PK>, LdsIO<F, PK>, NoNeed, 1, 2, NT, false, PK>(cur, cnt, tw, NoNeed{}, lio, lio);
                    else lds_transform<FT, true, LOGM, LdsIO<FT, PK>, LdsIO<FT, PK>, NoNeed, 1, 2, NT, false, PK>(cur, cnt, tws, NoNeed{}, lios, lios);
                    if (nff == 3) lds_transform<F, true, LOGM, LdsIO<F, PK>, LdsPsi<F, PK>, NoNeed, 2, 3, NT, true, PK>(cur, cnt, tw, NoNeed{}, lio, psi);
                    else lds_transform<FT, true, LOGM, LdsIO<FT, PK>, LdsIO<FT, PK>, NoNeed, 2, 3, NT, false, PK>(cur, cnt, tws, NoNeed{}, lios, lios);
                    lds_transform<FT, true, LOGM, LdsIO<FT, PK>, LdsIO<FT, PK>, NoNeed, 3, NP - 1, NT, false, PK>(cur, cnt, tws, NoNeed{}, lios, lios);
                } else {
                    if (nff == 2) lds_transform<F, true, LOGM, LdsIO<F, PK>, LdsPsi<F, PK>, NoNeed, 1, 2, NT, true, PK>(cur, cnt, tw, NoNeed{}, lio, psi);
                    else lds_transform<FT, true, LOGM, LdsIO<FT, PK>, LdsIO<FT, PK>, NoNeed, 1, 2, NT, false, PK>(cur, cnt, tws, NoNeed{}, lios, lios);
                    lds_transform<FT, true, LOGM, LdsIO<FT, PK>, LdsIO<FT, PK>, NoNeed, 2, NP - 1, NT, false, PK>(cur, cnt, tws, NoNeed{}, lios, lios);
                }
            } else {
                lds_transform<F, true, LOGM, ChunkIn, LdsIO<F, PK>, NoNeed, 0, NP - 1, NT, false, PK>(cur, cnt, tw, NoNeed{}, in, lio);
            }
#pragma unroll
            for (int k = 0; k < KF; k++) {
                const int it = threadIdx.x + NT * k;
                if (it < D * L::U) {
                    const int i = it / L::U, u = it - i * L::U;
                    V x[4];
#pragma unroll
                    for (int q = 0; q < 4; q++) x[q] = L::get(cur, i + q * D, u);
                    if constexpr (isub) ifft4<FT>(x[0], x[1], x[2], x[3], tws + (uint64_t)last * FT::TWD);
                    else ifft4<F>(x[0], x[1], x[2], x[3], tw + (uint64_t)last * F::TWD);
#pragma unroll
                    for (int q = 0; q < 4; q++) {
                        if (c == 0) ar[k][q] = x[q];
                        else F::xor_into(ar[k][q], x[q]);
                    }
                }
            }
            lds_sync();  // the next chunk's first pass overwrites cur
        }
        uint32_t bad = 0;
        const uint32_t *twf = SUB ? a.tw_fft_sub : a.tw_fft;
#pragma unroll
        for (int k = 0; k < KF; k++) {
            const int it = threadIdx.x + NT * k;
            if (it < D * L::U) {
                const int i = it / L::U, u = it - i * L::U;
                if constexpr (SUB && !isub)  // (a subfield IFFT leaves acc in subfield coordinates already)
#pragma unroll
                        for (int q = 0; q < 4; q++) sub_swap<F>(ar[k][q], a.tw_dmap);  // into subfield coordinates
                fft4<FT>(ar[k][0], ar[k][1], ar[k][2], ar[k][3], twf);
#pragma unroll
                for (int q = 0; q < 4; q++) L::put(cur, i + q * D, u, ar[k][q]);
            }
        }
        __syncthreads();
        if constexpr (SUB && LOGM > 8) {
            // FFT passes [1, FEND) in subfield coordinates, the last one writing
            // normal coordinates back, then the full-field passes
            constexpr int FEND = big_sub_fft_end(LOGM);
            lds_transform<FT, false, LOGM, LdsIO<FT, PK>, LdsPsi<F, PK>, NoNeed, 1, FEND, NT, true, PK>(
                cur, a.p, twf, NoNeed{}, LdsIO<FT, PK>{cur}, LdsPsi<F, PK>{cur, a.tw_dmap});
            lds_transform<F, false, LOGM, LdsIO<F, PK>, ParityOutFull, NoNeed, FEND, 32, NT, false, PK>(
                cur, a.p, a.tw_fft, NoNeed{}, LdsIO<F, PK>{cur}, ParityOutFull{a, soff, tile, uo, &bad});
        } else {
            lds_transform<FT, false, LOGM, LdsIO<FT, PK>, ParityOut, NoNeed, 1, 32, NT, false, PK>(cur, a.p, twf, NoNeed{}, LdsIO<FT, PK>{cur},
                                                                             ParityOut{a, soff, tile, uo, &bad});
        }
        if constexpr (VERIFY) flag_mismatch(a.mismatch, bad != 0);
        return;
    }
    for (int c = 0; c < a.nchunks; c++) {
        const int row0 = c * M, cnt = a.k - row0 < M ? a.k - row0 : M;
        const uint32_t *tw = a.tw_ifft + (uint64_t)c * its * F::TWD;
        const ChunkIn in{a, row0, cnt, soff, tile, uo};
        if (c == 0) lds_transform<F, true, LOGM, ChunkIn, LdsIO<F, PK>, NoNeed, 0, 32, NT, false, PK>(acc, cnt, tw, NoNeed{}, in, LdsIO<F, PK>{acc});
        else lds_transform<F, true, LOGM, ChunkIn, AccXor, NoNeed, 0, 32, NT, false, PK>(cur, cnt, tw, NoNeed{}, in, AccXor{acc});
    }
    uint32_t bad = 0;
    lds_transform<F, false, LOGM, LdsIO<F, PK>, ParityOut, NoNeed, 0, 32, NT, false, PK>(acc, a.p, a.tw_fft, NoNeed{}, LdsIO<F, PK>{acc},
                                                                    ParityOut{a, soff, tile, uo, &bad});
    if constexpr (VERIFY) {
        flag_mismatch(a.mismatch, bad != 0);
    }
}

template <class F, class FT, int LOGN, bool BSUB, int PKV = 1>
hipError_t rec_lds_tb(const RecArgs &a, hipStream_t s) {
    constexpr int TB = LTile<F, PKV>::TB, NT = rec_threads<LOGN, PKV>();
    const unsigned gx = (unsigned)((a.S + TB - 1) / TB);
    if (!a.base || a.nstripes <= 1) {
        hipLaunchKernelGGL((k_rec_lds<F, FT, LOGN, BSUB, PKV>), dim3(gx), dim3(NT), 0, s, a);
        return hipGetLastError();
    }
    return for_y(a.nstripes, [&](int y0, int ny) {  // batched strided stripes: grid.y = stripe
        RecArgs b = a;
        b.base = a.base + (uint64_t)y0 * a.stripe_stride;
        hipLaunchKernelGGL((k_rec_lds<F, FT, LOGN, BSUB, PKV>), dim3(gx, (unsigned)ny), dim3(NT), 0, s, b);
    });
}
template <class F, class FT, int LOGN>
hipError_t rec_lds_t(const RecArgs &a, hipStream_t s) {
    if constexpr (LOGN >= 13 && std::is_same<F, F16<2>>::value) {  // n = 8192: quarter tiles
        if (a.tw_ifft_sub && a.tw_fft_sub && a.tw_dmap) return rec_lds_tb<F, FT, LOGN, true, 4>(a, s);
        return rec_lds_tb<F, FT, LOGN, false, 4>(a, s);
    }
    if constexpr (LOGN >= 10 && LOGN < 13 && std::is_same<F, F16<2>>::value) {
        // n = 1024, 2048: half tiles, two workgroups per CU (rs_debug_set_path "rec_half");
        // n = 4096: half tiles always
        if (LOGN >= 12 || rec_half_enabled()) {
            if (a.tw_ifft_sub && a.tw_fft_sub && a.tw_dmap) return rec_lds_tb<F, FT, LOGN, true, 2>(a, s);
            return rec_lds_tb<F, FT, LOGN, false, 2>(a, s);
        }
    }
    if constexpr (LOGN >= 12) {
        return hipErrorInvalidValue;  // (unreachable: half tiles above)
    } else {
        if constexpr (LOGN > 8)
            if (a.tw_ifft_sub && a.tw_fft_sub && a.tw_dmap) return rec_lds_tb<F, FT, LOGN, true>(a, s);
        return rec_lds_tb<F, FT, LOGN, false>(a, s);
    }
}
template <class F, class FT = F>
hipError_t rec_lds_f(int logn, const RecArgs &a, hipStream_t s) {
    switch (logn) {
        case 1: return rec_lds_t<F, FT, 1>(a, s);
        case 2: return rec_lds_t<F, FT, 2>(a, s);
        case 3: return rec_lds_t<F, FT, 3>(a, s);
        case 4: return rec_lds_t<F, FT, 4>(a, s);
        case 5: return rec_lds_t<F, FT, 5>(a, s);
        case 6: return rec_lds_t<F, FT, 6>(a, s);
        case 7: return rec_lds_t<F, FT, 7>(a, s);
        case 8: return rec_lds_t<F, FT, 8>(a, s);
    }
    // n = 512 .. 2048: GF(2^16), 64-byte tiles (the packed n x 64-byte image
    // takes 128 KB at n = 2048); n = 4096: 32-byte half tiles (128 KB);
    // n = 8192: 16-byte quarter tiles (128 KB)
    if constexpr (std::is_same<F, F16<2>>::value && std::is_same<FT, F>::value) {
        switch (logn) {
            case 9: return rec_lds_t<F, FT, 9>(a, s);
            case 10: return rec_lds_t<F, FT, 10>(a, s);
            case 11: return rec_lds_t<F, FT, 11>(a, s);
            case 12: return rec_lds_t<F, FT, 12>(a, s);
            case 13: return rec_lds_t<F, FT, 13>(a, s);
        }
    }
    return hipErrorInvalidValue;
}

template <class F, int LOGM, class FT>
hipError_t enc_lds_tt(bool verify, const EncodeArgs &a, hipStream_t s) {
    typedef LTile<F, enc_pk<LOGM>()> L;
    const dim3 grid((unsigned)((a.shard_size + L::TB - 1) / L::TB), (unsigned)a.nstripes), block(enc_threads<LOGM>());
    const size_t lds = (size_t)(enc_acc_regs(LOGM) ? 1 : 2) * (1 << LOGM) * L::ROW;
    auto go = [&](auto vf, auto sf) {
        constexpr bool V = decltype(vf)::value, IS = decltype(sf)::value;
        (void)hipFuncSetAttribute((const void *)k_enc_lds<F, LOGM, V, FT, IS>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        hipLaunchKernelGGL((k_enc_lds<F, LOGM, V, FT, IS>), grid, block, lds, s, a);
    };
    const bool isub = !std::is_same<F, FT>::value && a.tw_ifft_sub && a.ifft_nff;
    if constexpr (!std::is_same<F, FT>::value) {
        if (isub) {
            if (verify) go(std::true_type{}, std::true_type{});
            else go(std::false_type{}, std::true_type{});
            return hipGetLastError();
        }
    }
    if (verify) go(std::true_type{}, std::false_type{});
    else go(std::false_type{}, std::false_type{});
    return hipGetLastError();
}
template <class F>
struct SubOf {
    typedef F type;
};
template <int W>
struct SubOf<F16<W>> {
    typedef F16S<W> type;
};
template <class F, int LOGM>
hipError_t enc_lds_t(bool verify, const EncodeArgs &a, hipStream_t s) {
    if constexpr (F::SYM16 && enc_acc_regs(LOGM)) {
        if (a.tw_fft_sub && a.tw_dmap) return enc_lds_tt<F, LOGM, typename SubOf<F>::type>(verify, a, s);
    }
    return enc_lds_tt<F, LOGM, F>(verify, a, s);
}
template <class F>
hipError_t enc_lds_f(int logm, bool verify, const EncodeArgs &a, hipStream_t s) {
    switch (logm) {
        case 2: return enc_lds_t<F, 2>(verify, a, s);
        case 3: return enc_lds_t<F, 3>(verify, a, s);
        case 4: return enc_lds_t<F, 4>(verify, a, s);
        case 5: return enc_lds_t<F, 5>(verify, a, s);
        case 6: return enc_lds_t<F, 6>(verify, a, s);
        case 7: return enc_lds_t<F, 7>(verify, a, s);
        case 8: return enc_lds_t<F, 8>(verify, a, s);
    }
    if constexpr (std::is_same<F, F16<2>>::value) {  // m = 512, 1024: 64-byte tiles; 2048: half, 4096: quarter tiles
        switch (logm) {
            case 9: return enc_lds_t<F, 9>(verify, a, s);
            case 10: return enc_lds_t<F, 10>(verify, a, s);
            case 11: return enc_lds_t<F, 11>(verify, a, s);
            case 12: return enc_lds_t<F, 12>(verify, a, s);
        }
    }
    return hipErrorInvalidValue;
}

}  // namespace

// Lane width per (field, log2 m): keep acc + work + prefetch <= ~192 VGPRs
// (2 waves/SIMD) while using the widest coalesced access that fits.
template <int LOGM>
hipError_t launch_split_t(bool verify, const EncodeArgs &a, hipStream_t s) {
    const uint64_t units = a.shard_size >> 3;
    dim3 grid((unsigned)((units + 127) / 128), (unsigned)a.nstripes);
    if (verify) hipLaunchKernelGGL((k_encode_split<LOGM, true>), grid, dim3(256), 0, s, a);
    else hipLaunchKernelGGL((k_encode_split<LOGM, false>), grid, dim3(256), 0, s, a);
    return hipGetLastError();
}

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
        // Small GF(2^8) stripes (C2: 10+4 x 1 MiB is 256 workgroups of 16-byte
        // units, one per CU, latency-bound): 4-byte units give 4x the
        // workgroups and 4x the loads in flight per CU.
#ifndef RS_F8_NARROW
#define RS_F8_NARROW 1
#endif
        const bool narrow = pick_narrow(RS_F8_NARROW && (a.shard_size / 16 + 255) / 256 * (uint64_t)a.nstripes < 1024);
        switch (logm) {
            case 0: return enc_reg<F8<4>, 0>(verify, a, s);
            case 1: return enc_reg<F8<4>, 1>(verify, a, s);
            case 2: return narrow ? enc_reg<F8<1>, 2>(verify, a, s) : enc_reg<F8<4>, 2>(verify, a, s);
            case 3: return narrow ? enc_reg<F8<1>, 3>(verify, a, s) : enc_reg<F8<4>, 3>(verify, a, s);
            case 4: return narrow ? enc_reg<F8<1>, 4>(verify, a, s) : enc_reg<F8<4>, 4>(verify, a, s);
            case 5: return enc_reg<F8<2>, 5>(verify, a, s);
        }
    }
    return hipErrorInvalidValue;
}

hipError_t launch_encode_split(int logm, bool verify, const EncodeArgs &a, hipStream_t s) {
    switch (logm) {
        case 2: return launch_split_t<2>(verify, a, s);
        case 3: return launch_split_t<3>(verify, a, s);
        case 4: return launch_split_t<4>(verify, a, s);
        case 5: return launch_split_t<5>(verify, a, s);
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

// Host-resident pipeline, zero copy: one launch moves every scattered row of a
// segment over PCIe (the device reads or writes the mapped pinned rows), where
// hipMemcpy*Async took one copy per run of rows at ~10-15 us each
// (profiles/r05_host_zero_copy.txt: 54-57 GB/s for 128 rows in and 32 out at
// any segment width, against 6-20 GB/s for per-row copies).  Block (x, y):
// 16 KB of columns of entry y.
template <bool TO_HOST>
__global__ void __launch_bounds__(256) k_zc_copy(ZcRows r, uint8_t *slab, uint64_t pitch, uint64_t off, uint64_t w) {
    const int e = blockIdx.y;
    uint8_t *h = r.host[e] + off;
    uint8_t *d = slab + (uint64_t)r.slab_row[e] * pitch;
    const uint64_t c0 = (uint64_t)blockIdx.x * 16384;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const uint64_t c = c0 + (uint64_t)k * 4096 + (uint64_t)threadIdx.x * 16;
        if (c < w) {
            if constexpr (TO_HOST) *(uint4 *)(h + c) = *(const uint4 *)(d + c);
            else *(uint4 *)(d + c) = *(const uint4 *)(h + c);
        }
    }
}

hipError_t launch_zc_copy(const ZcRows &r, uint8_t *slab, uint64_t pitch, uint64_t off, uint64_t w, bool to_host,
                          hipStream_t s) {
    if (r.n <= 0) return hipSuccess;
    if (r.n > kZcMax || (w & 15)) return hipErrorInvalidValue;
    const dim3 grid((unsigned)((w + 16383) / 16384), (unsigned)r.n);
    if (to_host) hipLaunchKernelGGL(k_zc_copy<true>, grid, dim3(256), 0, s, r, slab, pitch, off, w);
    else hipLaunchKernelGGL(k_zc_copy<false>, grid, dim3(256), 0, s, r, slab, pitch, off, w);
    return hipGetLastError();
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


template <int W>
hipError_t rec_lds_w(int bits, int logn, bool sub, const RecArgs &a, hipStream_t s) {
    if (bits != 16) return rec_lds_f<F8<W>>(logn, a, s);
    return sub ? rec_lds_f<F16<W>, F16S<W>>(logn, a, s) : rec_lds_f<F16<W>>(logn, a, s);
}
hipError_t launch_rec_lds(int bits, int logn, bool sub, const RecArgs &a, hipStream_t s) {
    if (rec_bs256_available(bits, logn, sub, a.mtrunc)) return launch_rec_bs256(a, s);
    if (logn > 8) {
        if (bits != 16 || sub || logn > kMaxLdsRecLogN16 || !a.need_w || !a.rev) return hipErrorInvalidValue;
        return rec_lds_f<F16<2>>(logn, a, s);
    }
    const uint64_t ns = a.base && a.nstripes > 1 ? (uint64_t)a.nstripes : 1;
    const bool narrow = pick_narrow((a.S + 127) / 128 * ns < kLdsMinGrid);
    return narrow ? rec_lds_w<2>(bits, logn, sub, a, s) : rec_lds_w<4>(bits, logn, sub, a, s);
}

hipError_t launch_encode_lds(int bits, int logm, bool verify, const EncodeArgs &a, hipStream_t s) {
    if (logm > 8) return bits == 16 ? enc_lds_f<F16<2>>(logm, verify, a, s) : hipErrorInvalidValue;
    const bool narrow = pick_narrow((a.shard_size + 127) / 128 * (uint64_t)a.nstripes < kLdsMinGrid);
    if (narrow) return bits == 16 ? enc_lds_f<F16<2>>(logm, verify, a, s) : enc_lds_f<F8<2>>(logm, verify, a, s);
    return bits == 16 ? enc_lds_f<F16<4>>(logm, verify, a, s) : enc_lds_f<F8<4>>(logm, verify, a, s);
}

}  // namespace rs
