// Host-side finite-field tables and GPU twiddle-table construction.
//
// Field construction follows the reference exactly:
//   GF(2^16): initLUTs / initFFTSkew  leopard16.go:940-1031 (poly 0x1002D, Cantor basis)
//   GF(2^8):  initLUTs8 / initFFTSkew8 leopard8.go:1034-1122 (poly 0x11D)
// The GPU never sees log/exp tables: every multiply by a constant (a "twiddle",
// given as its log) is shipped as a small set of byte-permute tables that the
// kernels evaluate with v_perm_b32 (see kernels.hip, mul_add).
#pragma once
#include <cstddef>
#include <cstdint>
#include <vector>

namespace rs {

constexpr int kTwDwords16 = 24;  // per-twiddle table size in dwords (GF(2^16))
constexpr int kTwDwords8 = 8;    // per-twiddle table size in dwords (GF(2^8))

struct Field {
    int bits = 0;       // 8 or 16
    uint32_t order = 0; // 2^bits
    uint32_t mod = 0;   // 2^bits - 1 ("modulus": a log value meaning "multiply by zero")
    std::vector<uint16_t> log, exp, skew, walsh;

    uint32_t add_mod(uint32_t a, uint32_t b) const {  // leopard16.go:840-845
        uint32_t s = a + b;
        return (s + (s >> bits)) & mod;
    }
    uint32_t sub_mod(uint32_t a, uint32_t b) const {  // leopard16.go:847-851
        uint32_t d = a - b;
        return (d + (d >> bits)) & mod;
    }
    uint32_t mul_log(uint32_t a, uint32_t log_b) const {  // leopard16.go:828-838
        if (a == 0) return 0;
        return exp[add_mod(log[a], log_b)];
    }
    void fwht(uint32_t *data, int mtrunc) const;  // leopard16.go:865-900
};

const Field &field(int bits);  // built once, thread-safe

// Perm-table image of "multiply by exp(log_m)" for the GPU (kTwDwords* dwords).
// Butterfly twiddles (zero_if_mod = true): log_m == mod is the zero twiddle of
// the reference's XOR-only butterflies, shipped as an all-zero table.
// mulgf16 scalings (zero_if_mod = false): log 65535 is the identity there
// (refMul through mul16LUTs[65535], leopard16.go:810-825).
void make_twiddle(const Field &F, uint32_t log_m, uint32_t *out, bool zero_if_mod = false);
inline int tw_dwords(int bits) { return bits == 16 ? kTwDwords16 : kTwDwords8; }

// ---- GF(2^8) inside GF(2^16) ("subfield coordinates").
// The Cantor-basis integers < 256 (the span of the first 8 basis vectors,
// leopard16.go:941-946) form the subfield GF(2^8), and every fftSkew entry
// with index < 255 lies in it (initFFTSkew :986-1031 builds them from
// 2, 4, ..., 128 by field operations).  Write the element 1 << (8+i) as
// d_i + beta8 * c_i (beta8 = the element 256, c_i, d_i < 256).  Holding a
// symbol as (x0, x1) = (lo ^ D(hi), hi), D(h) = XOR of d_i over the set bits
// of h, a product with a subfield element t is (t*x0, t*x1): one 8x8 GF(2)
// map on both bytes.  to_sub is an involution (it is its own inverse).
struct SubCoords {
    bool ok = false;  // the block structure was verified for every subfield element
    uint8_t d[8] = {};
    uint32_t D(uint32_t hi) const {
        uint32_t r = 0;
        for (int i = 0; i < 8; i++)
            if ((hi >> i) & 1) r ^= d[i];
        return r;
    }
    uint32_t to_sub(uint32_t x) const { return x ^ D(x >> 8); }
};
const SubCoords &sub_coords();  // GF(2^16); built once, thread-safe
// log_m is the zero twiddle (== mod) or exp(log_m) lies in the subfield.
inline bool in_subfield(const Field &F, uint32_t log_m) { return log_m == F.mod || F.exp[log_m] < 256; }
// GF(2^8)-layout (kTwDwords8) table of "multiply by exp(log_m)" on one byte of
// subfield coordinates; log_m == mod gives the all-zero table.  log_m at dword 5.
void make_sub_twiddle(const Field &F, uint32_t log_m, uint32_t *out);
// The same layout for the byte map D of the coordinate change (lo, hi) ->
// (lo ^ D(hi), hi); applying it twice is the identity.
void make_sub_dmap(uint32_t *out);
// GF(2^16)-layout (kTwDwords16) table of an arbitrary GF(2)-linear map f on
// 16-bit symbols (same group/byte layout as make_twiddle; dword 20 = 0).
template <class Fn>
void make_linear_image(Fn f, uint32_t *out) {
    static const int off[6] = {0, 3, 6, 8, 11, 14}, wid[6] = {3, 3, 2, 3, 3, 2};
    int d = 0;
    for (int g = 0; g < 6; g++)
        for (int o = 0; o < 2; o++) {
            uint8_t e[8] = {0};
            for (int x = 0; x < (1 << wid[g]); x++) e[x] = (uint8_t)(f((uint32_t)x << off[g]) >> (8 * o));
            out[d++] = e[0] | (e[1] << 8) | (e[2] << 16) | ((uint32_t)e[3] << 24);
            if (wid[g] == 3) out[d++] = e[4] | (e[5] << 8) | (e[6] << 16) | ((uint32_t)e[7] << 24);
        }
    while (d < kTwDwords16) out[d++] = 0;
}

inline int ceil_pow2(int n) { return n <= 1 ? 1 : 1 << (64 - __builtin_clzll((unsigned long long)(n - 1))); }
inline int ilog2(int n) { return 31 - __builtin_clz((unsigned)n); }

// Twiddle slot schedules.  A transform of size M = 2^L is a sequence of
// passes; radix-4 passes hold 3 slots per butterfly group in the order
// (m01, m02, m23); the radix-2 pass of an odd L holds 1 slot (IFFT) or one
// slot per row pair (FFT).  Kernels and host use the same offsets.
struct PassInfo {
    int dist;      // butterfly distance
    int radix;     // 4 or 2
    int groups;    // butterfly groups in the pass (radix-4: M/(4*dist); radix-2 IFFT: 1; radix-2 FFT: M/2)
    int slot_off;  // first slot of the pass
};
std::vector<PassInfo> ifft_passes(int logm);  // dist = 1, 4, 16, ... then radix-2 at M/2
std::vector<PassInfo> fft_passes(int logm);   // dist = M/4, M/16, ... then radix-2 at 1
int ifft_slots(int logm);
int fft_slots(int logm);

// Twiddle LOG values for the reference's encode schedule (leopard16.go:128-224):
// chunk c's IFFT (skew base m-1+c*m, indices skewLUT[iend], [iend+dist],
// [iend+2*dist], radix-2 [dist]) and the final FFT (fftSkew[iEnd-1]...).
// Groups the reference skips (r >= mtrunc) get `mod` (they act on zero rows).
// Returns false when the reference would panic (skew index out of range).
bool encode_schedule(const Field &F, int k, int p, std::vector<uint32_t> &ifft_logs, std::vector<uint32_t> &fft_logs,
                     int &nchunks);

// Decoder schedules over n = ceilPow2(m+k) rows (leopard16.go:573-657).
bool decode_schedule(const Field &F, int k, int p, std::vector<uint32_t> &ifft_logs, std::vector<uint32_t> &fft_logs);

// Error locators (log domain) for an erasure pattern, leopard16.go:433-470
// (GF(2^8): leopard8.go:478-531).  erased[i] for i in [0, k+p), data first.
// Returns false when the reference would panic (GF(2^8) with m+k > 256).
bool error_locators(const Field &F, int k, int p, const uint8_t *erased, std::vector<uint32_t> &err_locs);

}  // namespace rs
