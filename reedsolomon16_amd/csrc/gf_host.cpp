// Host-side finite-field tables and GPU twiddle-table construction (see gf_host.hpp).
#include "gf_host.hpp"

#include <mutex>

namespace rs {

namespace {

// initLUTs (leopard16.go:940-983) / initLUTs8 (leopard8.go:1034-1074).
void build_luts(Field &F, uint32_t poly, const uint16_t *cantor) {
    const uint32_t order = F.order, mod = F.mod;
    F.log.assign(order, 0);
    F.exp.assign(order, 0);
    // LFSR pass: exp[] temporarily holds state -> exponent.
    uint32_t state = 1;
    for (uint32_t i = 0; i < mod; i++) {
        F.exp[state] = (uint16_t)i;
        state <<= 1;
        if (state >= order) state ^= poly;
    }
    F.exp[0] = (uint16_t)mod;
    // Cantor-basis span, then log[] = exponent of the spanned element.
    F.log[0] = 0;
    for (int i = 0; i < F.bits; i++) {
        const uint32_t width = 1u << i;
        for (uint32_t j = 0; j < width; j++) F.log[j + width] = F.log[j] ^ cantor[i];
    }
    for (uint32_t i = 0; i < order; i++) F.log[i] = F.exp[F.log[i]];
    for (uint32_t i = 0; i < order; i++) F.exp[F.log[i]] = (uint16_t)i;
    F.exp[mod] = F.exp[0];
}

// initFFTSkew (leopard16.go:986-1031) / initFFTSkew8 (leopard8.go:1077-1122).
void build_skew(Field &F) {
    const int bits = F.bits;
    const uint32_t mod = F.mod;
    std::vector<uint32_t> temp(bits - 1);
    for (int i = 1; i < bits; i++) temp[i - 1] = 1u << i;
    std::vector<uint32_t> skew(mod, 0);
    for (int m = 0; m < bits - 1; m++) {
        const int step = 1 << (m + 1);
        skew[(1u << m) - 1] = 0;
        for (int i = m; i < bits - 1; i++) {
            const int s = 1 << (i + 1);
            for (int j = (1 << m) - 1; j < s; j += step) skew[j + s] = skew[j] ^ temp[i];
        }
        temp[m] = (mod - F.log[F.mul_log(temp[m], F.log[temp[m] ^ 1])]) & mod;
        for (int i = m + 1; i < bits - 1; i++) {
            const uint32_t sum = F.add_mod(F.log[temp[i] ^ 1], temp[m]);
            temp[i] = F.mul_log(temp[i], sum);
        }
    }
    F.skew.assign(mod, 0);
    for (uint32_t i = 0; i < mod; i++) F.skew[i] = F.log[skew[i]];
    std::vector<uint32_t> w(F.order);
    for (uint32_t i = 0; i < F.order; i++) w[i] = F.log[i];
    w[0] = 0;
    F.fwht(w.data(), (int)F.order);
    F.walsh.assign(F.order, 0);
    for (uint32_t i = 0; i < F.order; i++) F.walsh[i] = (uint16_t)w[i];
}

Field make_field(int bits) {
    Field F;
    F.bits = bits;
    F.order = 1u << bits;
    F.mod = F.order - 1;
    if (bits == 16) {
        static const uint16_t cantor[16] = {0x0001, 0xACCA, 0x3C0E, 0x163E, 0xC582, 0xED2E, 0x914C, 0x4012,
                                            0x6C98, 0x10D8, 0x6A72, 0xB900, 0xFDB8, 0xFB34, 0xFF38, 0x991E};
        build_luts(F, 0x1002D, cantor);
    } else {
        static const uint16_t cantor[8] = {1, 214, 152, 146, 86, 200, 88, 230};
        build_luts(F, 0x11D, cantor);
    }
    build_skew(F);
    return F;
}

}  // namespace

void Field::fwht(uint32_t *data, int mtrunc) const {
    // Decimation in time, two layers per step (leopard16.go:865-900).  Callers
    // guarantee mtrunc <= order, so the uint16 index wrap of the Go code never occurs.
    for (uint32_t dist = 1, dist4 = 4; dist4 <= order; dist = dist4, dist4 <<= 2) {
        for (uint32_t r = 0; r < (uint32_t)mtrunc; r += dist4) {
            for (uint32_t i = r; i < r + dist; i++) {
                uint32_t t0 = data[i], t1 = data[i + dist], t2 = data[i + 2 * dist], t3 = data[i + 3 * dist];
                uint32_t a = add_mod(t0, t1), b = sub_mod(t0, t1);
                t0 = a; t1 = b;
                a = add_mod(t2, t3); b = sub_mod(t2, t3);
                t2 = a; t3 = b;
                a = add_mod(t0, t2); b = sub_mod(t0, t2);
                t0 = a; t2 = b;
                a = add_mod(t1, t3); b = sub_mod(t1, t3);
                t1 = a; t3 = b;
                data[i] = t0; data[i + dist] = t1; data[i + 2 * dist] = t2; data[i + 3 * dist] = t3;
            }
        }
    }
}

const Field &field(int bits) {
    static std::once_flag o16, o8;
    static Field f16, f8;
    if (bits == 16) {
        std::call_once(o16, [] { f16 = make_field(16); });
        return f16;
    }
    std::call_once(o8, [] { f8 = make_field(8); });
    return f8;
}

// Byte-permute tables for y -> y * exp(log_m).
// A symbol is split into bit groups of <= 3 bits; each group indexes an
// 8-entry (or 4-entry) byte table per output byte, evaluated by one
// v_perm_b32 for 4 symbols at once.  By linearity of multiplication over
// GF(2), the product is the XOR of the group lookups.
//   GF(2^16) groups (bit offset, width): (0,3) (3,3) (6,2) (8,3) (11,3) (14,2)
//   dword layout: [g0 lo-out: e0-3, e4-7][g0 hi-out][g1 lo][g1 hi][g2 lo][g2 hi]
//                 [g3 lo][g3 hi][g4 lo][g4 hi][g5 lo][g5 hi][log_m][pad x3]
//   GF(2^8) groups: (0,3) (3,3) (6,2); layout [g0: e0-3, e4-7][g1][g2][log_m][pad x2]
void make_twiddle(const Field &F, uint32_t log_m, uint32_t *out, bool zero_if_mod) {
    static const int off16[6] = {0, 3, 6, 8, 11, 14}, wid16[6] = {3, 3, 2, 3, 3, 2};
    static const int off8[3] = {0, 3, 6}, wid8[3] = {3, 3, 2};
    const int ng = F.bits == 16 ? 6 : 3;
    const int *off = F.bits == 16 ? off16 : off8;
    const int *wid = F.bits == 16 ? wid16 : wid8;
    const int nout = F.bits == 16 ? 2 : 1;  // output bytes per symbol
    int d = 0;
    for (int g = 0; g < ng; g++) {
        for (int o = 0; o < nout; o++) {
            uint8_t e[8] = {0};
            if (!(zero_if_mod && log_m == F.mod))
                for (int x = 0; x < (1 << wid[g]); x++) e[x] = (uint8_t)(F.mul_log((uint32_t)x << off[g], log_m) >> (8 * o));
            out[d++] = e[0] | (e[1] << 8) | (e[2] << 16) | ((uint32_t)e[3] << 24);
            if (wid[g] == 3) out[d++] = e[4] | (e[5] << 8) | (e[6] << 16) | ((uint32_t)e[7] << 24);
        }
    }
    out[d++] = log_m;
    const int n = tw_dwords(F.bits);
    while (d < n) out[d++] = 0;
}

const SubCoords &sub_coords() {
    static std::once_flag once;
    static SubCoords sc;
    std::call_once(once, [] {
        const Field &F = field(16);
        const uint32_t lb8 = F.log[256];
        for (int i = 0; i < 8; i++) {
            bool found = false;
            for (uint32_t c = 1; c < 256 && !found; c++) {
                const uint32_t dd = F.mul_log(c, lb8) ^ (1u << (8 + i));  // 1<<(8+i) = dd + beta8*c
                if (dd < 256) {
                    sc.d[i] = (uint8_t)dd;
                    found = true;
                }
            }
            if (!found) return;
        }
        // multiply-by-t in coordinates == (t*x0, t*x1), checked on the basis for every subfield t
        for (uint32_t t = 1; t < 256; t++) {
            const uint32_t lt = F.log[t];
            for (int j = 0; j < 16; j++) {
                const uint32_t got = sc.to_sub(F.mul_log(sc.to_sub(1u << j), lt));
                const uint32_t want = j < 8 ? F.mul_log(1u << j, lt) : F.mul_log(1u << (j - 8), lt) << 8;
                if (got != want) return;
            }
        }
        sc.ok = true;
    });
    return sc;
}

void make_sub_twiddle(const Field &F, uint32_t log_m, uint32_t *out) {
    static const int off[3] = {0, 3, 6}, wid[3] = {3, 3, 2};
    int d = 0;
    for (int g = 0; g < 3; g++) {
        uint8_t e[8] = {0};
        if (log_m != F.mod)
            for (int x = 0; x < (1 << wid[g]); x++) e[x] = (uint8_t)F.mul_log((uint32_t)x << off[g], log_m);
        out[d++] = e[0] | (e[1] << 8) | (e[2] << 16) | ((uint32_t)e[3] << 24);
        if (wid[g] == 3) out[d++] = e[4] | (e[5] << 8) | (e[6] << 16) | ((uint32_t)e[7] << 24);
    }
    out[d++] = log_m;
    while (d < kTwDwords8) out[d++] = 0;
}

void make_sub_dmap(uint32_t *out) {
    static const int off[3] = {0, 3, 6}, wid[3] = {3, 3, 2};
    const SubCoords &sc = sub_coords();
    int d = 0;
    for (int g = 0; g < 3; g++) {
        uint8_t e[8] = {0};
        for (int x = 0; x < (1 << wid[g]); x++) e[x] = (uint8_t)sc.D((uint32_t)x << off[g]);
        out[d++] = e[0] | (e[1] << 8) | (e[2] << 16) | ((uint32_t)e[3] << 24);
        if (wid[g] == 3) out[d++] = e[4] | (e[5] << 8) | (e[6] << 16) | ((uint32_t)e[7] << 24);
    }
    while (d < kTwDwords8) out[d++] = 0;
}

std::vector<PassInfo> ifft_passes(int logm) {
    std::vector<PassInfo> v;
    const int M = 1 << logm;
    int slot = 0, dist = 1;
    for (; dist * 4 <= M; dist *= 4) {
        PassInfo p{dist, 4, M / (4 * dist), slot};
        slot += 3 * p.groups;
        v.push_back(p);
    }
    if (dist < M) v.push_back(PassInfo{dist, 2, 1, slot});
    return v;
}

std::vector<PassInfo> fft_passes(int logm) {
    std::vector<PassInfo> v;
    const int M = 1 << logm;
    int slot = 0, dist4 = M, dist = M >> 2;
    for (; dist != 0; dist4 = dist, dist >>= 2) {
        PassInfo p{dist, 4, M / dist4, slot};
        slot += 3 * p.groups;
        v.push_back(p);
    }
    if (dist4 == 2) v.push_back(PassInfo{1, 2, M / 2, slot});
    return v;
}

static int count_slots(const std::vector<PassInfo> &ps) {
    int s = 0;
    for (auto &p : ps) s += p.radix == 4 ? 3 * p.groups : p.groups;
    return s;
}
int ifft_slots(int logm) { return count_slots(ifft_passes(logm)); }
int fft_slots(int logm) { return count_slots(fft_passes(logm)); }

namespace {
// Bounds-checked reads of fftSkew as the Go slices do them.
struct SkewView {
    const Field &F;
    long off;
    bool ok = true;
    uint32_t at(long i) {
        if (off + i < 0 || off + i >= (long)F.mod) { ok = false; return F.mod; }
        return F.skew[off + i];
    }
};

// IFFT twiddles of one encoder chunk (ifftDITEncoder leopard16.go:694-741)
// or of the decoder (ifftDITDecoder :573-615, bias -1).
void ifft_logs(SkewView &sv, int logm, int mtrunc, int bias, uint32_t *dst) {
    for (const PassInfo &p : ifft_passes(logm)) {
        if (p.radix == 4) {
            for (int g = 0; g < p.groups; g++) {
                const int r = g * 4 * p.dist;
                uint32_t *s = dst + p.slot_off + 3 * g;
                if (r < mtrunc) {
                    const int iend = r + p.dist;
                    s[0] = sv.at(iend + bias);
                    s[1] = sv.at(iend + p.dist + bias);
                    s[2] = sv.at(iend + 2 * p.dist + bias);
                } else {
                    s[0] = s[1] = s[2] = sv.F.mod;  // group skipped by the reference: rows are zero
                }
            }
        } else {
            dst[p.slot_off] = sv.at(p.dist + bias);
        }
    }
}

// FFT twiddles (fftDIT leopard16.go:618-657).
void fft_logs(SkewView &sv, int logm, int mtrunc, uint32_t *dst) {
    for (const PassInfo &p : fft_passes(logm)) {
        if (p.radix == 4) {
            for (int g = 0; g < p.groups; g++) {
                const int r = g * 4 * p.dist;
                uint32_t *s = dst + p.slot_off + 3 * g;
                if (r < mtrunc) {
                    const int iend = r + p.dist;
                    s[0] = sv.at(iend - 1);
                    s[1] = sv.at(iend + p.dist - 1);
                    s[2] = sv.at(iend + 2 * p.dist - 1);
                } else {
                    s[0] = s[1] = s[2] = sv.F.mod;  // outputs not needed
                }
            }
        } else {
            for (int g = 0; g < p.groups; g++) dst[p.slot_off + g] = (2 * g < mtrunc) ? sv.at(2 * g) : sv.F.mod;
        }
    }
}
}  // namespace

bool encode_schedule(const Field &F, int k, int p, std::vector<uint32_t> &ifft, std::vector<uint32_t> &fft,
                     int &nchunks) {
    const int m = ceil_pow2(p), logm = ilog2(m);
    const int is = ifft_slots(logm);
    nchunks = (k + m - 1) / m;
    ifft.assign((size_t)nchunks * is, F.mod);
    fft.assign(fft_slots(logm), F.mod);
    // skewLUT := fftSkew[m-1:]  (slice bound: m-1 <= len)
    long off = m - 1;
    if (off > (long)F.mod) return false;
    for (int c = 0; c < nchunks; c++) {
        if (c > 0) {  // skewLUT = skewLUT[m:]
            off += m;
            if (off > (long)F.mod) return false;
        }
        const int cnt = (k - c * m) < m ? (k - c * m) : m;
        SkewView sv{F, off};
        ifft_logs(sv, logm, cnt, 0, ifft.data() + (size_t)c * is);
        if (!sv.ok) return false;
    }
    SkewView sv{F, 0};
    fft_logs(sv, logm, p, fft.data());
    // The fused kernels hard-code the r = 0 group's m01/m02 (and the radix-2
    // r = 0 twiddle) as XOR-only: fftSkew[2^j - 1] == log(0).
    for (const PassInfo &ps : fft_passes(logm)) {
        if (ps.radix == 4 && (fft[ps.slot_off] != F.mod || fft[ps.slot_off + 1] != F.mod)) return false;
        if (ps.radix == 2 && fft[ps.slot_off] != F.mod) return false;
    }
    return sv.ok;
}

bool decode_schedule(const Field &F, int k, int p, std::vector<uint32_t> &ifft, std::vector<uint32_t> &fft) {
    const int m = ceil_pow2(p);
    if ((long)m + k > (long)F.order) return false;  // the Go code panics (see error_locators)
    const int n = ceil_pow2(m + k), logn = ilog2(n);
    ifft.assign(ifft_slots(logn), F.mod);
    fft.assign(fft_slots(logn), F.mod);
    SkewView a{F, 0};
    ifft_logs(a, logn, m + k, -1, ifft.data());
    SkewView b{F, 0};
    fft_logs(b, logn, m + k, fft.data());
    return a.ok && b.ok;
}

bool error_locators(const Field &F, int k, int p, const uint8_t *erased, std::vector<uint32_t> &e) {
    const int m = ceil_pow2(p);
    // errLocs is a [order] array; the Go code panics for an index >= order and
    // fwht(&errLocs, m+k) with m+k > order reads out of range.
    if ((long)m + k > (long)F.order) return false;
    e.assign(F.order, 0);
    for (int i = 0; i < p; i++)
        if (erased[k + i]) e[i] = 1;
    for (int i = p; i < m; i++) e[i] = 1;
    for (int i = 0; i < k; i++)
        if (erased[i]) e[i + m] = 1;
    F.fwht(e.data(), m + k);
    for (uint32_t i = 0; i < F.order; i++) e[i] = (uint32_t)(((uint64_t)e[i] * F.walsh[i]) % F.mod);
    F.fwht(e.data(), (int)F.order);
    return true;
}

}  // namespace rs
