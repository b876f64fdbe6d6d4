/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.  Not part of the product.
 *
 * A scalar C restatement of the reference's portable ("Ref") Leopard-FFT
 * Reed-Solomon path, used by tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg as the checker.  The product library
 * (reedsolomon16_amd/csrc) never links, loads or calls anything in oracle/.
 *
 * Parity status: the reference (Go) cannot be built or run here (no Go
 * toolchain; the amd64 build is also broken) and ships no
 * golden vectors or known-answer tests.  This oracle is
 * therefore "parity unpinned" against reference OUTPUTS; it is pinned by
 *   (1) line-by-line restatement of the reference functions cited below,
 *   (2) an independent numpy restatement (oracle/leopard_np.py) that must agree
 *       bit-for-bit, and
 *   (3) the reference tests' own properties (encode->erase->reconstruct round
 *       trips, Verify true/false, MDS for every erasure class).
 *
 * Every function cites the reference file:line it follows.
 * GF(2^16): leopard16.go; GF(2^8): leopard8.go; butterflies: galois_noasm.go.
 */
#include <setjmp.h>
#include <stddef.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* Error codes: identical numbering to include/rs_mi355x.h (checked by tests). */
enum {
    ORC_OK = 0,
    ORC_ERR_INV_SHARD_NUM = 1,     /* ErrInvShardNum       reedsolomon.go:16 */
    ORC_ERR_MAX_SHARD_NUM = 2,     /* ErrMaxShardNum       reedsolomon.go:17 */
    ORC_ERR_TOO_FEW_SHARDS = 3,    /* ErrTooFewShards      reedsolomon.go:18 */
    ORC_ERR_SHARD_NO_DATA = 4,     /* ErrShardNoData       reedsolomon.go:19 */
    ORC_ERR_SHARD_SIZE = 5,        /* ErrShardSize         reedsolomon.go:20 */
    ORC_ERR_INVALID_SHARD_SIZE = 6,/* ErrInvalidShardSize  reedsolomon.go:25 */
    ORC_ERR_NOT_SUPPORTED = 7,     /* ErrNotSupported      reedsolomon.go:27 */
    ORC_ERR_SHORT_DATA = 8,        /* ErrShortData         reedsolomon.go:26 */
    ORC_ERR_RECONSTRUCT_REQUIRED = 9, /* ErrReconstructRequired reedsolomon.go:24 */
    ORC_ERR_PANIC = 50,            /* reference would panic (index out of range) */
    ORC_ERR_NOMEM = 51,
};

/* A Go panic (slice index out of range) is modelled as a longjmp back to the
 * API entry point, which returns ORC_ERR_PANIC. */
static jmp_buf g_panic;
#define GO_PANIC() longjmp(g_panic, 1)

/* Bounds-checked view of the skew table (Go slices are bounds-checked). */
typedef struct { const uint16_t *p; long len; } skew16_t;
typedef struct { const uint8_t *p; long len; } skew8_t;

static inline uint16_t sk16(skew16_t s, long i) { if (i < 0 || i >= s.len) GO_PANIC(); return s.p[i]; }
static inline skew16_t sk16_slice(skew16_t s, long off) { if (off < 0 || off > s.len) GO_PANIC(); skew16_t r = {s.p + off, s.len - off}; return r; }
static inline uint8_t sk8(skew8_t s, long i) { if (i < 0 || i >= s.len) GO_PANIC(); return s.p[i]; }
static inline skew8_t sk8_slice(skew8_t s, long off) { if (off < 0 || off > s.len) GO_PANIC(); skew8_t r = {s.p + off, s.len - off}; return r; }

/* ceilPow2: leopard16.go:853-856 */
static int ceil_pow2(int n) {
    if (n <= 1) return 1;
    return 1 << (64 - __builtin_clzll((unsigned long long)(n - 1)));
}

/* sliceXor(in, out): out ^= in — galois.go:963-980 (sliceXorGo) */
static void slice_xor(const uint8_t *in, uint8_t *out, size_t n) {
    for (size_t i = 0; i < n; i++) out[i] ^= in[i];
}

/* ===================================================================== */
/*                              GF(2^16)                                  */
/* ===================================================================== */
#define ORDER16 65536
#define MOD16 65535
#define POLY16 0x1002D

static uint16_t logLUT[ORDER16], expLUT[ORDER16];
static uint16_t fftSkew[MOD16], logWalsh[ORDER16];
typedef struct { uint16_t Lo[256], Hi[256]; } mul16lut_t;
static mul16lut_t *mul16LUTs; /* 64 MiB, leopard16.go:103-110 */

/* addMod / subMod with partial reduction: leopard16.go:840-850 */
static inline uint16_t add_mod16(uint16_t a, uint16_t b) {
    unsigned sum = (unsigned)a + (unsigned)b;
    return (uint16_t)(sum + (sum >> 16));
}
static inline uint16_t sub_mod16(uint16_t a, uint16_t b) {
    unsigned dif = (unsigned)a - (unsigned)b;
    return (uint16_t)(dif + (dif >> 16));
}
/* mulLog: leopard16.go:828-838 */
static inline uint16_t mul_log16(uint16_t a, uint16_t log_b) {
    if (a == 0) return 0;
    return expLUT[add_mod16(logLUT[a], log_b)];
}

/* fwht: leopard16.go:865-900 (uint16 index arithmetic as in the Go code) */
static void fwht16(uint16_t *data, int mtrunc) {
    int dist = 1, dist4 = 4;
    while (dist4 <= ORDER16) {
        for (int r = 0; r < mtrunc; r += dist4) {
            uint16_t d = (uint16_t)dist, off = (uint16_t)r;
            for (uint16_t i = 0; i < d; i++) {
                uint16_t t0 = data[off], t1 = data[(uint16_t)(off + d)];
                uint16_t t2 = data[(uint16_t)(off + d * 2)], t3 = data[(uint16_t)(off + d * 3)];
                uint16_t a, b;
                a = add_mod16(t0, t1); b = sub_mod16(t0, t1); t0 = a; t1 = b;
                a = add_mod16(t2, t3); b = sub_mod16(t2, t3); t2 = a; t3 = b;
                a = add_mod16(t0, t2); b = sub_mod16(t0, t2); t0 = a; t2 = b;
                a = add_mod16(t1, t3); b = sub_mod16(t1, t3); t1 = a; t3 = b;
                data[off] = t0; data[(uint16_t)(off + d)] = t1;
                data[(uint16_t)(off + d * 2)] = t2; data[(uint16_t)(off + d * 3)] = t3;
                off++;
            }
        }
        dist = dist4;
        dist4 <<= 2;
    }
}

/* initLUTs: leopard16.go:940-983 */
static void init_luts16(void) {
    static const uint16_t cantor[16] = {
        0x0001, 0xACCA, 0x3C0E, 0x163E, 0xC582, 0xED2E, 0x914C, 0x4012,
        0x6C98, 0x10D8, 0x6A72, 0xB900, 0xFDB8, 0xFB34, 0xFF38, 0x991E};
    unsigned state = 1;
    for (unsigned i = 0; i < MOD16; i++) {
        expLUT[state] = (uint16_t)i;
        state <<= 1;
        if (state >= ORDER16) state ^= POLY16;
    }
    expLUT[0] = MOD16;
    logLUT[0] = 0;
    for (int i = 0; i < 16; i++) {
        uint16_t basis = cantor[i];
        int width = 1 << i;
        for (int j = 0; j < width; j++) logLUT[j + width] = logLUT[j] ^ basis;
    }
    for (int i = 0; i < ORDER16; i++) logLUT[i] = expLUT[logLUT[i]];
    for (int i = 0; i < ORDER16; i++) expLUT[logLUT[i]] = (uint16_t)i;
    expLUT[MOD16] = expLUT[0];
}

/* initFFTSkew: leopard16.go:986-1031 */
static void init_fft_skew16(void) {
    uint16_t temp[15];
    for (int i = 1; i < 16; i++) temp[i - 1] = (uint16_t)(1u << i);
    for (int m = 0; m < 15; m++) {
        int step = 1 << (m + 1);
        fftSkew[(1 << m) - 1] = 0;
        for (int i = m; i < 15; i++) {
            int s = 1 << (i + 1);
            for (int j = (1 << m) - 1; j < s; j += step) fftSkew[j + s] = fftSkew[j] ^ temp[i];
        }
        temp[m] = (uint16_t)(MOD16 - logLUT[mul_log16(temp[m], logLUT[temp[m] ^ 1])]);
        for (int i = m + 1; i < 15; i++) {
            uint16_t sum = add_mod16(logLUT[temp[i] ^ 1], temp[m]);
            temp[i] = mul_log16(temp[i], sum);
        }
    }
    for (int i = 0; i < MOD16; i++) fftSkew[i] = logLUT[fftSkew[i]];
    for (int i = 0; i < ORDER16; i++) logWalsh[i] = logLUT[i];
    logWalsh[0] = 0;
    fwht16(logWalsh, ORDER16);
}

/* initMul16LUT (Ref tables only): leopard16.go:1033-1053 */
static int init_mul16(void) {
    mul16LUTs = (mul16lut_t *)malloc(sizeof(mul16lut_t) * ORDER16);
    if (!mul16LUTs) return -1;
    for (int log_m = 0; log_m < ORDER16; log_m++) {
        uint16_t tmp[64];
        for (int nibble = 0, shift = 0; nibble < 4; nibble++, shift += 4)
            for (int x = 0; x < 16; x++) tmp[nibble * 16 + x] = mul_log16((uint16_t)(x << shift), (uint16_t)log_m);
        mul16lut_t *lut = &mul16LUTs[log_m];
        for (int i = 0; i < 256; i++) {
            lut->Lo[i] = tmp[i & 15] ^ tmp[(i >> 4) + 16];
            lut->Hi[i] = tmp[(i & 15) + 32] ^ tmp[(i >> 4) + 48];
        }
    }
    return 0;
}

/* refMulAdd: x[] ^= y[] * log_m — leopard16.go:775-793 (64-byte lo/hi blocks) */
static void ref_mul_add16(uint8_t *x, const uint8_t *y, uint16_t log_m, size_t n) {
    const mul16lut_t *lut = &mul16LUTs[log_m];
    for (size_t off = 0; off + 64 <= n; off += 64) {
        for (int i = 0; i < 32; i++) {
            uint16_t prod = lut->Lo[y[off + i]] ^ lut->Hi[y[off + 32 + i]];
            x[off + i] ^= (uint8_t)prod;
            x[off + i + 32] ^= (uint8_t)(prod >> 8);
        }
    }
}
/* refMul: x[] = y[] * log_m — leopard16.go:810-825 */
static void ref_mul16(uint8_t *x, const uint8_t *y, uint16_t log_m, size_t n) {
    const mul16lut_t *lut = &mul16LUTs[log_m];
    for (size_t off = 0; off < n; off += 64) {
        for (int i = 0; i < 32; i++) {
            uint16_t prod = lut->Lo[y[off + i]] ^ lut->Hi[y[off + 32 + i]];
            x[off + i] = (uint8_t)prod;
            x[off + i + 32] = (uint8_t)(prod >> 8);
        }
    }
}
/* ifftDIT2 (Ref): y ^= x; x ^= y*m — galois_noasm.go:72-76 */
static void ifft_dit2_16(uint8_t *x, uint8_t *y, uint16_t log_m, size_t n) {
    slice_xor(x, y, n);
    ref_mul_add16(x, y, log_m, n);
}
/* fftDIT2 (Ref): x ^= y*m; y ^= x — galois_noasm.go:58-62 */
static void fft_dit2_16(uint8_t *x, uint8_t *y, uint16_t log_m, size_t n) {
    ref_mul_add16(x, y, log_m, n);
    slice_xor(x, y, n);
}

/* ifftDIT4Ref: leopard16.go:750-772 */
static void ifft_dit4_16(uint8_t **w, int dist, uint16_t m01, uint16_t m23, uint16_t m02, size_t n) {
    if (m01 == MOD16) slice_xor(w[0], w[dist], n); else ifft_dit2_16(w[0], w[dist], m01, n);
    if (m23 == MOD16) slice_xor(w[dist * 2], w[dist * 3], n); else ifft_dit2_16(w[dist * 2], w[dist * 3], m23, n);
    if (m02 == MOD16) {
        slice_xor(w[0], w[dist * 2], n);
        slice_xor(w[dist], w[dist * 3], n);
    } else {
        ifft_dit2_16(w[0], w[dist * 2], m02, n);
        ifft_dit2_16(w[dist], w[dist * 3], m02, n);
    }
}
/* fftDIT4Ref: leopard16.go:660-682 */
static void fft_dit4_16(uint8_t **w, int dist, uint16_t m01, uint16_t m23, uint16_t m02, size_t n) {
    if (m02 == MOD16) {
        slice_xor(w[0], w[dist * 2], n);
        slice_xor(w[dist], w[dist * 3], n);
    } else {
        fft_dit2_16(w[0], w[dist * 2], m02, n);
        fft_dit2_16(w[dist], w[dist * 3], m02, n);
    }
    if (m01 == MOD16) slice_xor(w[0], w[dist], n); else fft_dit2_16(w[0], w[dist], m01, n);
    if (m23 == MOD16) slice_xor(w[dist * 2], w[dist * 3], n); else fft_dit2_16(w[dist * 2], w[dist * 3], m23, n);
}

/* ifftDITEncoder: leopard16.go:685-747 */
static void ifft_dit_encoder16(uint8_t *const *data, int mtrunc, uint8_t **work, uint8_t **xor_res,
                               int m, skew16_t skew, size_t n) {
    for (int i = 0; i < mtrunc; i++) memcpy(work[i], data[i], n);
    for (int i = mtrunc; i < m; i++) memset(work[i], 0, n);
    int dist = 1, dist4 = 4;
    while (dist4 <= m) {
        for (int r = 0; r < mtrunc; r += dist4) {
            int iend = r + dist;
            uint16_t m01 = sk16(skew, iend), m02 = sk16(skew, iend + dist), m23 = sk16(skew, iend + dist * 2);
            for (int i = r; i < iend; i++) ifft_dit4_16(work + i, dist, m01, m23, m02, n);
        }
        dist = dist4;
        dist4 <<= 2;
    }
    if (dist < m) {
        uint16_t logm = sk16(skew, dist);
        if (logm == MOD16) {
            for (int i = 0; i < dist; i++) slice_xor(work[i], work[dist + i], n);
        } else {
            for (int i = 0; i < dist; i++) ifft_dit2_16(work[i], work[i + dist], logm, n);
        }
    }
    if (xor_res)
        for (int i = 0; i < m; i++) slice_xor(work[i], xor_res[i], n);
}

/* ifftDITDecoder: leopard16.go:573-615 */
static void ifft_dit_decoder16(int mtrunc, uint8_t **work, int m, skew16_t skew, size_t n) {
    int dist = 1, dist4 = 4;
    while (dist4 <= m) {
        for (int r = 0; r < mtrunc; r += dist4) {
            int iend = r + dist;
            uint16_t m01 = sk16(skew, iend - 1), m02 = sk16(skew, iend + dist - 1), m23 = sk16(skew, iend + dist * 2 - 1);
            for (int i = r; i < iend; i++) ifft_dit4_16(work + i, dist, m01, m23, m02, n);
        }
        dist = dist4;
        dist4 <<= 2;
    }
    if (dist < m) {
        uint16_t logm = sk16(skew, dist - 1);
        if (logm == MOD16) {
            for (int i = 0; i < dist; i++) slice_xor(work[i], work[dist + i], n);
        } else {
            for (int i = 0; i < dist; i++) ifft_dit2_16(work[i], work[i + dist], logm, n);
        }
    }
}

/* errorBitfield (16-bit): leopard16.go:1076-1252 */
#define KWORDMIPS 5
#define KWORDS (ORDER16 / 64)
#define KBIGMIPS 6
#define KBIGWORDS ((KWORDS + 63) / 64)
#define KBIGGESTMIPS 4
typedef struct {
    uint64_t Words[KWORDMIPS][KWORDS];
    uint64_t BigWords[KBIGMIPS][KBIGWORDS];
    uint64_t BiggestWords[KBIGGESTMIPS];
} errbits16_t;
static const uint64_t kHiMasks[5] = {0xAAAAAAAAAAAAAAAAull, 0xCCCCCCCCCCCCCCCCull, 0xF0F0F0F0F0F0F0F0ull,
                                     0xFF00FF00FF00FF00ull, 0xFFFF0000FFFF0000ull};
static void eb16_set(errbits16_t *e, int i) { e->Words[0][i / 64] |= 1ull << (i & 63); }
static int eb16_needed(const errbits16_t *e, int mip, int bit) { /* isNeededFn: :1104-1132 */
    if (mip >= 16) return 1;
    if (mip >= 12) { bit /= 4096; return 0 != (e->BiggestWords[mip - 12] & (1ull << bit)); }
    if (mip >= 6) { bit /= 64; return 0 != (e->BigWords[mip - 6][bit / 64] & (1ull << (bit & 63))); }
    if (mip > 0) return 0 != (e->Words[mip - 1][bit / 64] & (1ull << (bit & 63)));
    GO_PANIC(); /* nil func call */
    return 0;
}
static void eb16_prepare(errbits16_t *e) { /* :1157-1213 */
    for (int i = 0; i < KWORDS; i++) {
        uint64_t w = e->Words[0][i];
        uint64_t hi2lo0 = w | ((w & kHiMasks[0]) >> 1);
        uint64_t lo2hi0 = (w & (kHiMasks[0] >> 1)) << 1;
        w = hi2lo0 | lo2hi0;
        e->Words[0][i] = w;
        int bits = 2;
        for (int j = 1; j < KWORDMIPS; j++) {
            uint64_t hi2lo = w | ((w & kHiMasks[j]) >> bits);
            uint64_t lo2hi = (w & (kHiMasks[j] >> bits)) << bits;
            w = hi2lo | lo2hi;
            e->Words[j][i] = w;
            bits <<= 1;
        }
    }
    for (int i = 0; i < KBIGWORDS; i++) {
        uint64_t w_i = 0, bit = 1;
        const uint64_t *src = &e->Words[KWORDMIPS - 1][i * 64];
        for (int t = 0; t < 64; t++) {
            uint64_t w = src[t];
            w_i |= (w | (w >> 32) | (w << 32)) & bit;
            bit <<= 1;
        }
        e->BigWords[0][i] = w_i;
        int bits = 1;
        for (int j = 1; j < KBIGMIPS; j++) {
            uint64_t hi2lo = w_i | ((w_i & kHiMasks[j - 1]) >> bits);
            uint64_t lo2hi = (w_i & (kHiMasks[j - 1] >> bits)) << bits;
            w_i = hi2lo | lo2hi;
            e->BigWords[j][i] = w_i;
            bits <<= 1;
        }
    }
    uint64_t w_i = 0, bit = 1;
    for (int t = 0; t < KBIGWORDS; t++) {
        uint64_t w = e->BigWords[KBIGMIPS - 1][t];
        w_i |= (w | (w >> 32) | (w << 32)) & bit;
        bit <<= 1;
    }
    e->BiggestWords[0] = w_i;
    uint64_t bits = 1;
    for (int j = 1; j < KBIGGESTMIPS; j++) {
        uint64_t hi2lo = w_i | ((w_i & kHiMasks[j - 1]) >> bits);
        uint64_t lo2hi = (w_i & (kHiMasks[j - 1] >> bits)) << bits;
        w_i = hi2lo | lo2hi;
        e->BiggestWords[j] = w_i;
        bits <<= 1;
    }
}

/* fftDIT: leopard16.go:618-657; with errorBitfield pruning when eb != NULL (:1215-1252) */
static void fft_dit16(uint8_t **work, int mtrunc, int m, skew16_t skew, const errbits16_t *eb, size_t n) {
    int mip = 0;
    if (eb) mip = 31 - __builtin_clz((unsigned)m); /* bits.Len32(m) - 1 */
    int dist4 = m, dist = m >> 2;
    while (dist != 0) {
        for (int r = 0; r < mtrunc; r += dist4) {
            if (eb && !eb16_needed(eb, mip, r)) continue;
            int iEnd = r + dist;
            uint16_t m01 = sk16(skew, iEnd - 1), m02 = sk16(skew, iEnd + dist - 1), m23 = sk16(skew, iEnd + dist * 2 - 1);
            for (int i = r; i < iEnd; i++) fft_dit4_16(work + i, dist, m01, m23, m02, n);
        }
        dist4 = dist;
        dist >>= 2;
        mip -= 2;
    }
    if (dist4 == 2) {
        for (int r = 0; r < mtrunc; r += 2) {
            if (eb && !eb16_needed(eb, mip, r)) continue;
            uint16_t logM = sk16(skew, r + 1 - 1);
            if (logM == MOD16) slice_xor(work[r], work[r + 1], n);
            else fft_dit2_16(work[r], work[r + 1], logM, n);
        }
    }
}

/* checkShards / shardSize: encoder.go:102-126 */
static size_t shard_size(const size_t *lens, int n) {
    for (int i = 0; i < n; i++) if (lens[i] != 0) return lens[i];
    return 0;
}
static int check_shards(const size_t *lens, int n, int nilok) {
    size_t size = shard_size(lens, n);
    if (size == 0) return ORC_ERR_SHARD_NO_DATA;
    for (int i = 0; i < n; i++)
        if (lens[i] != size && (lens[i] != 0 || !nilok)) return ORC_ERR_SHARD_SIZE;
    return ORC_OK;
}

static int g_inited = 0;
int orc_init(void) {
    if (g_inited) return 0;
    init_luts16();
    init_fft_skew16();
    if (init_mul16() != 0) return -1;
    extern void orc_init8(void);
    orc_init8();
    g_inited = 1;
    return 0;
}

static uint8_t **alloc_rows(int rows, size_t n) {
    uint8_t **w = (uint8_t **)calloc((size_t)rows, sizeof(uint8_t *));
    if (!w) return NULL;
    uint8_t *slab = (uint8_t *)calloc((size_t)rows * (n ? n : 1), 1);
    if (!slab) { free(w); return NULL; }
    for (int i = 0; i < rows; i++) w[i] = slab + (size_t)i * n;
    return w;
}
static void free_rows(uint8_t **w) { if (w) { free(w[0]); free(w); } }

/* newFF16 validation: leopard16.go:36-54 */
int orc16_check_new(int k, int p) {
    if (k <= 0 || p <= 0) return ORC_ERR_INV_SHARD_NUM;
    if (k + p > 65536) return ORC_ERR_MAX_SHARD_NUM;
    return ORC_OK;
}

/* encode: leopard16.go:128-224 (parity written into shards[k..k+p)) */
static int encode16_body(int k, int p, uint8_t *const *shards, size_t S) {
    int m = ceil_pow2(p);
    uint8_t **volatile work = alloc_rows(m * 2, S);
    if (!work) return ORC_ERR_NOMEM;
    if (setjmp(g_panic)) { free_rows(work); return ORC_ERR_PANIC; }
    int mtrunc = m < k ? m : k;
    skew16_t full = {fftSkew, MOD16};
    skew16_t skewLUT = sk16_slice(full, m - 1);
    uint8_t *const *sh = shards;
    ifft_dit_encoder16(sh, mtrunc, work, NULL, m, skewLUT, S);
    int lastCount = k % m;
    if (m < k) {
        for (int i = m; i + m <= k; i += m) {
            sh += m;
            skewLUT = sk16_slice(skewLUT, m);
            ifft_dit_encoder16(sh, m, work + m, work, m, skewLUT, S);
        }
        if (lastCount != 0) {
            sh += m;
            skewLUT = sk16_slice(skewLUT, m);
            ifft_dit_encoder16(sh, lastCount, work + m, work, m, skewLUT, S);
        }
    }
    fft_dit16(work, p, m, full, NULL, S);
    for (int i = 0; i < p; i++) memcpy(shards[k + i], work[i], S);
    free_rows(work);
    return ORC_OK;
}

/* Encode: leopard16.go:116-125 */
int orc16_encode(int k, int p, uint8_t *const *shards, const size_t *lens, int nshards) {
    int e = orc16_check_new(k, p);
    if (e) return e;
    if (nshards != k + p) return ORC_ERR_TOO_FEW_SHARDS;
    if ((e = check_shards(lens, nshards, 0))) return e;
    size_t S = shard_size(lens, nshards);
    if (S % 64 != 0) return ORC_ERR_INVALID_SHARD_SIZE;
    return encode16_body(k, p, shards, S);
}

/* Verify: leopard16.go:361-387 */
int orc16_verify(int k, int p, uint8_t *const *shards, const size_t *lens, int nshards, int *ok) {
    *ok = 0;
    int e = orc16_check_new(k, p);
    if (e) return e;
    if (nshards != k + p) return ORC_ERR_TOO_FEW_SHARDS;
    if ((e = check_shards(lens, nshards, 0))) return e;
    size_t S = lens[0];
    if (S % 64 != 0) return ORC_ERR_INVALID_SHARD_SIZE;
    uint8_t **par = alloc_rows(p, S);
    uint8_t **outs = (uint8_t **)calloc((size_t)(k + p), sizeof(uint8_t *));
    if (!par || !outs) { free_rows(par); free(outs); return ORC_ERR_NOMEM; }
    for (int i = 0; i < k; i++) outs[i] = shards[i];
    for (int i = 0; i < p; i++) outs[k + i] = par[i];
    e = encode16_body(k, p, outs, S);
    if (e == ORC_OK) {
        *ok = 1;
        for (int i = 0; i < p; i++)
            if (memcmp(par[i], shards[k + i], S) != 0) { *ok = 0; break; }
    }
    free_rows(par);
    free(outs);
    return e;
}

/* reconstruct: leopard16.go:390-570.
 * lens[i]==0 marks shard i missing.  For every missing shard that gets
 * reconstructed, shards[i] must point at >= S writable bytes; lens[i] is set
 * to S on return (the Go code resizes/allocates the slice, :556-560). */
int orc16_reconstruct(int k, int p, uint8_t *const *shards, size_t *lens, int nshards, int recover_all) {
    int e = orc16_check_new(k, p);
    if (e) return e;
    int total = k + p;
    if (nshards != total) return ORC_ERR_TOO_FEW_SHARDS;
    if ((e = check_shards(lens, nshards, 1))) return e;
    int numberPresent = 0, dataPresent = 0;
    for (int i = 0; i < total; i++)
        if (lens[i] != 0) { numberPresent++; if (i < k) dataPresent++; }
    if (numberPresent == total || (!recover_all && dataPresent == k)) return ORC_OK;
    int useBits = (total - numberPresent) <= p / 4;
    if (numberPresent < k) return ORC_ERR_TOO_FEW_SHARDS;
    size_t S = shard_size(lens, nshards);
    if (S % 64 != 0) return ORC_ERR_INVALID_SHARD_SIZE;

    int m = ceil_pow2(p);
    int n = ceil_pow2(m + k);
    errbits16_t *volatile eb = (errbits16_t *)calloc(1, sizeof(errbits16_t));
    uint16_t *volatile errLocs = (uint16_t *)calloc(ORDER16, sizeof(uint16_t));
    uint8_t **volatile work = alloc_rows(n, S);
    if (!eb || !errLocs || !work) { free(eb); free(errLocs); free_rows(work); return ORC_ERR_NOMEM; }
    if (setjmp(g_panic)) { free(eb); free(errLocs); free_rows(work); return ORC_ERR_PANIC; }

    for (int i = 0; i < p; i++)
        if (lens[i + k] == 0) { errLocs[i] = 1; if (recover_all) eb16_set(eb, i); }
    for (int i = p; i < m; i++) { errLocs[i] = 1; if (recover_all) eb16_set(eb, i); }
    for (int i = 0; i < k; i++)
        if (lens[i] == 0) { errLocs[i + m] = 1; eb16_set(eb, i + m); }
    if (useBits) eb16_prepare(eb);

    fwht16(errLocs, m + k);
    for (int i = 0; i < ORDER16; i++)
        errLocs[i] = (uint16_t)(((unsigned long long)errLocs[i] * (unsigned long long)logWalsh[i]) % MOD16);
    fwht16(errLocs, ORDER16);

    for (int i = 0; i < p; i++) {
        if (lens[i + k] != 0) ref_mul16(work[i], shards[i + k], errLocs[i], S);
        else memset(work[i], 0, S);
    }
    for (int i = p; i < m; i++) memset(work[i], 0, S);
    for (int i = 0; i < k; i++) {
        if (lens[i] != 0) ref_mul16(work[m + i], shards[i], errLocs[m + i], S);
        else memset(work[m + i], 0, S);
    }
    for (int i = m + k; i < n; i++) memset(work[i], 0, S);

    skew16_t full = {fftSkew, MOD16};
    ifft_dit_decoder16(m + k, work, n, full, S);

    for (int i = 1; i < n; i++) { /* formal derivative :527-530 */
        int width = ((i ^ (i - 1)) + 1) >> 1;
        for (int j = 0; j < width; j++) slice_xor(work[i + j], work[i - width + j], S);
    }

    fft_dit16(work, m + k, n, full, useBits ? eb : NULL, S);

    int end = recover_all ? total : k;
    for (int i = 0; i < end; i++) {
        if (lens[i] != 0) continue;
        lens[i] = S;
        if (i >= k) ref_mul16(shards[i], work[i - k], (uint16_t)(MOD16 - errLocs[i - k]), S);
        else ref_mul16(shards[i], work[i + m], (uint16_t)(MOD16 - errLocs[i + m]), S);
    }
    free(eb);
    free(errLocs);
    free_rows(work);
    return ORC_OK;
}

/* Table accessors for cross-checks. */
void orc16_tables(uint16_t *log_out, uint16_t *exp_out, uint16_t *skew_out, uint16_t *walsh_out) {
    if (log_out) memcpy(log_out, logLUT, sizeof(logLUT));
    if (exp_out) memcpy(exp_out, expLUT, sizeof(expLUT));
    if (skew_out) memcpy(skew_out, fftSkew, sizeof(fftSkew));
    if (walsh_out) memcpy(walsh_out, logWalsh, sizeof(logWalsh));
}
/* x = y * exp(log_m) over a whole shard (refMul), exposed for kernel unit tests. */
void orc16_mul(uint8_t *x, const uint8_t *y, uint16_t log_m, size_t n) { ref_mul16(x, y, log_m, n); }
uint16_t orc16_mul_log(uint16_t a, uint16_t log_b) { return mul_log16(a, log_b); }

/* ===================================================================== */
/*                              GF(2^8)                                   */
/* ===================================================================== */
#define ORDER8 256
#define MOD8 255
#define POLY8 0x11D
#define WORKSIZE8 (32 << 10) /* leopard8.go:113 */

static uint8_t logLUT8[ORDER8], expLUT8[ORDER8], fftSkew8[MOD8], logWalsh8[ORDER8];
static uint8_t mul8LUTs[ORDER8][256];

static inline uint8_t add_mod8(uint8_t a, uint8_t b) { unsigned s = (unsigned)a + b; return (uint8_t)(s + (s >> 8)); }
static inline uint8_t sub_mod8(uint8_t a, uint8_t b) { unsigned d = (unsigned)a - (unsigned)b; return (uint8_t)(d + (d >> 8)); }
static inline uint8_t mul_log8(uint8_t a, uint8_t log_b) { return a == 0 ? 0 : expLUT8[add_mod8(logLUT8[a], log_b)]; }

/* fwht8: leopard8.go:959-994.  data is a [256]ffe8 indexed with uint16
 * offsets, so an index >= 256 is a Go bounds-check panic. */
static void fwht8(uint8_t *data, int mtrunc) {
    int dist = 1, dist4 = 4;
    while (dist4 <= ORDER8) {
        for (int r = 0; r < mtrunc; r += dist4) {
            uint16_t d = (uint16_t)dist, off = (uint16_t)r;
            for (uint16_t i = 0; i < d; i++) {
                if ((unsigned)off + 3u * d >= ORDER8) GO_PANIC();
                uint8_t t0 = data[off], t1 = data[off + d], t2 = data[off + d * 2], t3 = data[off + d * 3];
                uint8_t a, b;
                a = add_mod8(t0, t1); b = sub_mod8(t0, t1); t0 = a; t1 = b;
                a = add_mod8(t2, t3); b = sub_mod8(t2, t3); t2 = a; t3 = b;
                a = add_mod8(t0, t2); b = sub_mod8(t0, t2); t0 = a; t2 = b;
                a = add_mod8(t1, t3); b = sub_mod8(t1, t3); t1 = a; t3 = b;
                data[off] = t0; data[off + d] = t1; data[off + d * 2] = t2; data[off + d * 3] = t3;
                off++;
            }
        }
        dist = dist4;
        dist4 <<= 2;
    }
}

/* initLUTs8 / initFFTSkew8 / initMul8LUT: leopard8.go:1034-1163 */
void orc_init8(void) {
    static const uint8_t cantor[8] = {1, 214, 152, 146, 86, 200, 88, 230};
    unsigned state = 1;
    for (unsigned i = 0; i < MOD8; i++) {
        expLUT8[state] = (uint8_t)i;
        state <<= 1;
        if (state >= ORDER8) state ^= POLY8;
    }
    expLUT8[0] = MOD8;
    logLUT8[0] = 0;
    for (int i = 0; i < 8; i++) {
        int width = 1 << i;
        for (int j = 0; j < width; j++) logLUT8[j + width] = logLUT8[j] ^ cantor[i];
    }
    for (int i = 0; i < ORDER8; i++) logLUT8[i] = expLUT8[logLUT8[i]];
    for (int i = 0; i < ORDER8; i++) expLUT8[logLUT8[i]] = (uint8_t)i;
    expLUT8[MOD8] = expLUT8[0];

    uint8_t temp[7];
    for (int i = 1; i < 8; i++) temp[i - 1] = (uint8_t)(1u << i);
    for (int m = 0; m < 7; m++) {
        int step = 1 << (m + 1);
        fftSkew8[(1 << m) - 1] = 0;
        for (int i = m; i < 7; i++) {
            int s = 1 << (i + 1);
            for (int j = (1 << m) - 1; j < s; j += step) fftSkew8[j + s] = fftSkew8[j] ^ temp[i];
        }
        temp[m] = (uint8_t)(MOD8 - logLUT8[mul_log8(temp[m], logLUT8[temp[m] ^ 1])]);
        for (int i = m + 1; i < 7; i++) {
            uint8_t sum = add_mod8(logLUT8[temp[i] ^ 1], temp[m]);
            temp[i] = mul_log8(temp[i], sum);
        }
    }
    for (int i = 0; i < MOD8; i++) fftSkew8[i] = logLUT8[fftSkew8[i]];
    for (int i = 0; i < ORDER8; i++) logWalsh8[i] = logLUT8[i];
    logWalsh8[0] = 0;
    fwht8(logWalsh8, ORDER8);

    for (int log_m = 0; log_m < ORDER8; log_m++) {
        uint8_t tmp[64];
        for (int nibble = 0, shift = 0; nibble < 4; nibble++, shift += 4)
            for (int x = 0; x < 16; x++) tmp[nibble * 16 + x] = mul_log8((uint8_t)(x << shift), (uint8_t)log_m);
        for (int i = 0; i < 256; i++) mul8LUTs[log_m][i] = tmp[i & 15] ^ tmp[(i >> 4) + 16];
    }
}

/* refMulAdd8 / refMul8: leopard8.go:899-924 (64-byte blocks) */
static void ref_mul_add8(uint8_t *x, const uint8_t *y, uint8_t log_m, size_t n) {
    const uint8_t *lut = mul8LUTs[log_m];
    for (size_t off = 0; off + 64 <= n; off += 64)
        for (int i = 0; i < 64; i++) x[off + i] ^= lut[y[off + i]];
}
static void ref_mul8(uint8_t *x, const uint8_t *y, uint8_t log_m, size_t n) {
    const uint8_t *lut = mul8LUTs[log_m];
    for (size_t off = 0; off < n; off += 64)
        for (int i = 0; i < 64; i++) x[off + i] = lut[y[off + i]];
}
static void ifft_dit2_8(uint8_t *x, uint8_t *y, uint8_t m, size_t n) { slice_xor(x, y, n); ref_mul_add8(x, y, m, n); }
static void fft_dit2_8(uint8_t *x, uint8_t *y, uint8_t m, size_t n) { ref_mul_add8(x, y, m, n); slice_xor(x, y, n); }

/* ifftDIT4Ref8: leopard8.go:876-896 */
static void ifft_dit4_8(uint8_t **w, int d, uint8_t m01, uint8_t m23, uint8_t m02, size_t n) {
    if (m01 == MOD8) slice_xor(w[0], w[d], n); else ifft_dit2_8(w[0], w[d], m01, n);
    if (m23 == MOD8) slice_xor(w[d * 2], w[d * 3], n); else ifft_dit2_8(w[d * 2], w[d * 3], m23, n);
    if (m02 == MOD8) { slice_xor(w[0], w[d * 2], n); slice_xor(w[d], w[d * 3], n); }
    else { ifft_dit2_8(w[0], w[d * 2], m02, n); ifft_dit2_8(w[d], w[d * 3], m02, n); }
}
/* fftDIT4Ref8: leopard8.go:786-807 */
static void fft_dit4_8(uint8_t **w, int d, uint8_t m01, uint8_t m23, uint8_t m02, size_t n) {
    if (m02 == MOD8) { slice_xor(w[0], w[d * 2], n); slice_xor(w[d], w[d * 3], n); }
    else { fft_dit2_8(w[0], w[d * 2], m02, n); fft_dit2_8(w[d], w[d * 3], m02, n); }
    if (m01 == MOD8) slice_xor(w[0], w[d], n); else fft_dit2_8(w[0], w[d], m01, n);
    if (m23 == MOD8) slice_xor(w[d * 2], w[d * 3], n); else fft_dit2_8(w[d * 2], w[d * 3], m23, n);
}
/* ifftDITEncoder8: leopard8.go:810-872 */
static void ifft_dit_encoder8(uint8_t *const *data, int mtrunc, uint8_t **work, uint8_t **xor_res, int m,
                              skew8_t skew, size_t n) {
    for (int i = 0; i < mtrunc; i++) memcpy(work[i], data[i], n);
    for (int i = mtrunc; i < m; i++) memset(work[i], 0, n);
    int dist = 1, dist4 = 4;
    while (dist4 <= m) {
        for (int r = 0; r < mtrunc; r += dist4) {
            int iend = r + dist;
            uint8_t m01 = sk8(skew, iend), m02 = sk8(skew, iend + dist), m23 = sk8(skew, iend + dist * 2);
            for (int i = r; i < iend; i++) ifft_dit4_8(work + i, dist, m01, m23, m02, n);
        }
        dist = dist4;
        dist4 <<= 2;
    }
    if (dist < m) {
        uint8_t logm = sk8(skew, dist);
        if (logm == MOD8) { for (int i = 0; i < dist; i++) slice_xor(work[i], work[dist + i], n); }
        else { for (int i = 0; i < dist; i++) ifft_dit2_8(work[i], work[i + dist], logm, n); }
    }
    if (xor_res)
        for (int i = 0; i < m; i++) slice_xor(work[i], xor_res[i], n);
}
/* ifftDITDecoder8: leopard8.go:698-740 */
static void ifft_dit_decoder8(int mtrunc, uint8_t **work, int m, skew8_t skew, size_t n) {
    int dist = 1, dist4 = 4;
    while (dist4 <= m) {
        for (int r = 0; r < mtrunc; r += dist4) {
            int iend = r + dist;
            uint8_t m01 = sk8(skew, iend - 1), m02 = sk8(skew, iend + dist - 1), m23 = sk8(skew, iend + dist * 2 - 1);
            for (int i = r; i < iend; i++) ifft_dit4_8(work + i, dist, m01, m23, m02, n);
        }
        dist = dist4;
        dist4 <<= 2;
    }
    if (dist < m) {
        uint8_t logm = sk8(skew, dist - 1);
        if (logm == MOD8) { for (int i = 0; i < dist; i++) slice_xor(work[i], work[dist + i], n); }
        else { for (int i = 0; i < dist; i++) ifft_dit2_8(work[i], work[i + dist], logm, n); }
    }
}

/* errorBitfield8: leopard8.go:1165-1273 */
typedef struct { uint64_t Words[7][4]; } errbits8_t;
static void eb8_set(errbits8_t *e, int i) { e->Words[0][(i / 64) & 3] |= 1ull << (i & 63); }
static void eb8_cache_id(const errbits8_t *e, uint8_t out[32]) {
    for (int w = 0; w < 4; w++)
        for (int b = 0; b < 8; b++) out[w * 8 + b] = (uint8_t)(e->Words[0][w] >> (8 * b));
}
static int eb8_needed(const errbits8_t *e, int mip, int bit) {
    if (mip >= 8 || mip <= 0) return 1;
    return 0 != (e->Words[mip - 1][bit / 64] & (1ull << (bit & 63)));
}
static void eb8_prepare(errbits8_t *e) {
    for (int i = 0; i < 4; i++) {
        uint64_t w = e->Words[0][i];
        uint64_t hi2lo0 = w | ((w & kHiMasks[0]) >> 1);
        uint64_t lo2hi0 = (w & (kHiMasks[0] >> 1)) << 1;
        w = hi2lo0 | lo2hi0;
        e->Words[0][i] = w;
        int bits = 2;
        for (int j = 1; j < 5; j++) {
            uint64_t hi2lo = w | ((w & kHiMasks[j]) >> bits);
            uint64_t lo2hi = (w & (kHiMasks[j] >> bits)) << bits;
            w = hi2lo | lo2hi;
            e->Words[j][i] = w;
            bits <<= 1;
        }
    }
    for (int i = 0; i < 4; i++) {
        uint64_t w = e->Words[4][i];
        w |= w >> 32;
        w |= w << 32;
        e->Words[5][i] = w;
    }
    for (int i = 0; i < 4; i += 2) {
        uint64_t t = e->Words[5][i] | e->Words[5][i + 1];
        e->Words[6][i] = t;
        e->Words[6][i + 1] = t;
    }
}
/* fftDIT8 (+ errorBitfield8.fftDIT8): leopard8.go:743-782, 1222-1273 */
static void fft_dit8(uint8_t **work, int mtrunc, int m, skew8_t skew, const errbits8_t *eb, size_t n) {
    int mip = 31 - __builtin_clz((unsigned)m);
    int dist4 = m, dist = m >> 2;
    while (dist != 0) {
        for (int r = 0; r < mtrunc; r += dist4) {
            if (eb && !eb8_needed(eb, mip, r)) continue;
            int iend = r + dist;
            uint8_t m01 = sk8(skew, iend - 1), m02 = sk8(skew, iend + dist - 1), m23 = sk8(skew, iend + dist * 2 - 1);
            for (int i = r; i < iend; i++) fft_dit4_8(work + i, dist, m01, m23, m02, n);
        }
        dist4 = dist;
        dist >>= 2;
        mip -= 2;
    }
    if (dist4 == 2) {
        for (int r = 0; r < mtrunc; r += 2) {
            if (eb && !eb8_needed(eb, mip, r)) continue;
            uint8_t logm = sk8(skew, r + 1 - 1);
            if (logm == MOD8) slice_xor(work[r], work[r + 1], n);
            else fft_dit2_8(work[r], work[r + 1], logm, n);
        }
    }
}

/* leopardFF8 state incl. the inversion cache (leopard8.go:20-29, 67-71). */
typedef struct { uint8_t key[32]; uint8_t errLocs[256]; int has_bits; errbits8_t bits; } inv8_entry_t;
typedef struct {
    int k, p, total;
    int cache_on;
    inv8_entry_t *cache;
    int ncache, capcache;
} orc8_t;

void *orc8_new(int k, int p, int *err) {
    *err = ORC_OK;
    if (k <= 0 || p <= 0) { *err = ORC_ERR_INV_SHARD_NUM; return NULL; }
    if (k + p > 65536) { *err = ORC_ERR_MAX_SHARD_NUM; return NULL; }
    orc8_t *h = (orc8_t *)calloc(1, sizeof(orc8_t));
    h->k = k; h->p = p; h->total = k + p;
    h->cache_on = (h->total <= 64);
    return h;
}
void orc8_free(void *hv) {
    orc8_t *h = (orc8_t *)hv;
    if (!h) return;
    free(h->cache);
    free(h);
}

/* encode (leopard8.go:153-277): processed in 32 KiB column chunks, parity in place. */
static int encode8_body(orc8_t *h, uint8_t *const *shards, size_t S) {
    int k = h->k, p = h->p;
    int m = ceil_pow2(p);
    uint8_t **volatile wbuf = alloc_rows(m * 2, WORKSIZE8);
    uint8_t **volatile work = (uint8_t **)calloc((size_t)m * 2, sizeof(uint8_t *));
    uint8_t **volatile sh = (uint8_t **)calloc((size_t)(k + p), sizeof(uint8_t *));
    if (!wbuf || !work || !sh) { free_rows(wbuf); free(work); free(sh); return ORC_ERR_NOMEM; }
    if (setjmp(g_panic)) { free_rows(wbuf); free(work); free(sh); return ORC_ERR_PANIC; }
    int mtrunc = m < k ? m : k;
    skew8_t full = {fftSkew8, MOD8};
    skew8_t skewLUT = sk8_slice(full, m - 1);
    for (size_t off = 0; off < S; off += WORKSIZE8) {
        size_t end = off + WORKSIZE8 < S ? off + WORKSIZE8 : S;
        size_t n = end - off;
        for (int i = 0; i < m * 2; i++) work[i] = wbuf[i];
        for (int i = 0; i < k + p; i++) sh[i] = shards[i] + off;
        for (int i = 0; i < p; i++) work[i] = shards[k + i] + off; /* parity rows are work[0..p) */
        uint8_t **s = sh;
        ifft_dit_encoder8(s, mtrunc, work, NULL, m, skewLUT, n);
        int lastCount = k % m;
        skew8_t skew2 = skewLUT;
        if (m < k) {
            for (int i = m; i + m <= k; i += m) {
                s += m;
                skew2 = sk8_slice(skew2, m);
                ifft_dit_encoder8(s, m, work + m, work, m, skew2, n);
            }
            if (lastCount != 0) {
                s += m;
                skew2 = sk8_slice(skew2, m);
                ifft_dit_encoder8(s, lastCount, work + m, work, m, skew2, n);
            }
        }
        fft_dit8(work, p, m, full, NULL, n);
    }
    free_rows(wbuf);
    free(work);
    free(sh);
    return ORC_OK;
}

int orc8_encode(void *hv, uint8_t *const *shards, const size_t *lens, int nshards) {
    orc8_t *h = (orc8_t *)hv;
    if (nshards != h->total) return ORC_ERR_TOO_FEW_SHARDS;
    int e = check_shards(lens, nshards, 0);
    if (e) return e;
    size_t S = shard_size(lens, nshards);
    if (S % 64 != 0) return ORC_ERR_INVALID_SHARD_SIZE;
    return encode8_body(h, shards, S);
}

/* Verify: leopard8.go:415-436 */
int orc8_verify(void *hv, uint8_t *const *shards, const size_t *lens, int nshards, int *ok) {
    orc8_t *h = (orc8_t *)hv;
    *ok = 0;
    if (nshards != h->total) return ORC_ERR_TOO_FEW_SHARDS;
    int e = check_shards(lens, nshards, 0);
    if (e) return e;
    size_t S = lens[0];
    if (S % 64 != 0) return ORC_ERR_INVALID_SHARD_SIZE;
    int k = h->k, p = h->p;
    uint8_t **par = alloc_rows(p, S);
    uint8_t **outs = (uint8_t **)calloc((size_t)(k + p), sizeof(uint8_t *));
    if (!par || !outs) { free_rows(par); free(outs); return ORC_ERR_NOMEM; }
    for (int i = 0; i < k; i++) outs[i] = shards[i];
    for (int i = 0; i < p; i++) outs[k + i] = par[i];
    e = encode8_body(h, outs, S);
    if (e == ORC_OK) {
        *ok = 1;
        for (int i = 0; i < p; i++)
            if (memcmp(par[i], shards[k + i], S) != 0) { *ok = 0; break; }
    }
    free_rows(par);
    free(outs);
    return e;
}

static inv8_entry_t *cache_find(orc8_t *h, const uint8_t key[32]) {
    for (int i = 0; i < h->ncache; i++)
        if (memcmp(h->cache[i].key, key, 32) == 0) return &h->cache[i];
    return NULL;
}
static void cache_put(orc8_t *h, const uint8_t key[32], const uint8_t *errLocs, const errbits8_t *bits) {
    inv8_entry_t *ent = cache_find(h, key);
    if (!ent) {
        if (h->ncache == h->capcache) {
            h->capcache = h->capcache ? h->capcache * 2 : 8;
            h->cache = (inv8_entry_t *)realloc(h->cache, sizeof(inv8_entry_t) * (size_t)h->capcache);
        }
        ent = &h->cache[h->ncache++];
    }
    memcpy(ent->key, key, 32);
    memcpy(ent->errLocs, errLocs, 256);
    ent->has_bits = bits != NULL;
    if (bits) ent->bits = *bits; else memset(&ent->bits, 0, sizeof(ent->bits));
}

/* reconstruct: leopard8.go:439-695 (incl. the inversion cache exactly as written:
 * lookup key = raw erasure bitmap; store key = bitmap after prepare() when useBits). */
int orc8_reconstruct(void *hv, uint8_t *const *shards, size_t *lens, int nshards, int recover_all) {
    orc8_t *h = (orc8_t *)hv;
    int k = h->k, p = h->p, total = h->total;
    if (nshards != total) return ORC_ERR_TOO_FEW_SHARDS;
    int e = check_shards(lens, nshards, 1);
    if (e) return e;
    int numberPresent = 0, dataPresent = 0;
    for (int i = 0; i < total; i++)
        if (lens[i] != 0) { numberPresent++; if (i < k) dataPresent++; }
    if (numberPresent == total || (!recover_all && dataPresent == k)) return ORC_OK;
    if (numberPresent < k) return ORC_ERR_TOO_FEW_SHARDS;
    size_t S = shard_size(lens, nshards);
    if (S % 64 != 0) return ORC_ERR_INVALID_SHARD_SIZE;
    int useBits = (total - numberPresent) <= p / 4 && S * (size_t)total >= (64u << 10);
    int m = ceil_pow2(p);
    int n = ceil_pow2(m + k);

    errbits8_t eb;
    memset(&eb, 0, sizeof(eb));
    uint8_t errLocs[256];
    memset(errLocs, 0, sizeof(errLocs));
    uint8_t **volatile wbuf = NULL;
    uint8_t **volatile work = NULL;
    uint8_t **volatile sh = NULL;
    if (setjmp(g_panic)) { free_rows(wbuf); free(work); free(sh); return ORC_ERR_PANIC; }
#define EL(i) do { if ((i) < 0 || (i) >= 256) GO_PANIC(); } while (0)
    for (int i = 0; i < p; i++)
        if (lens[i + k] == 0) { EL(i); errLocs[i] = 1; if (recover_all) eb8_set(&eb, i); }
    for (int i = p; i < m; i++) { EL(i); errLocs[i] = 1; if (recover_all) eb8_set(&eb, i); }
    for (int i = 0; i < k; i++)
        if (lens[i] == 0) { EL(i + m); errLocs[i + m] = 1; eb8_set(&eb, i + m); }

    int gotInversion = 0;
    if (h->cache_on) {
        uint8_t key[32];
        eb8_cache_id(&eb, key);
        inv8_entry_t *ent = cache_find(h, key);
        if (ent) {
            memcpy(errLocs, ent->errLocs, 256);
            if (ent->has_bits && useBits) { eb = ent->bits; useBits = 1; }
            else useBits = 0;
            gotInversion = 1;
        }
    }
    if (!gotInversion) {
        if (useBits) eb8_prepare(&eb);
        fwht8(errLocs, m + k);
        for (int i = 0; i < ORDER8; i++) errLocs[i] = (uint8_t)(((unsigned)errLocs[i] * (unsigned)logWalsh8[i]) % MOD8);
        fwht8(errLocs, ORDER8);
        if (h->cache_on) {
            uint8_t key[32];
            eb8_cache_id(&eb, key);
            cache_put(h, key, errLocs, useBits ? &eb : NULL);
        }
    }

    wbuf = alloc_rows(n, WORKSIZE8);
    work = (uint8_t **)calloc((size_t)n, sizeof(uint8_t *));
    sh = (uint8_t **)calloc((size_t)total, sizeof(uint8_t *));
    if (!wbuf || !work || !sh) { free_rows(wbuf); free(work); free(sh); return ORC_ERR_NOMEM; }
    /* which shards were present on entry (sh[i] non-nil) */
    int *present = (int *)calloc((size_t)total, sizeof(int));
    for (int i = 0; i < total; i++) present[i] = lens[i] != 0;
    for (int i = 0; i < total; i++) {
        if (!recover_all && i >= k) continue;
        if (lens[i] == 0) lens[i] = S;
    }
    skew8_t full = {fftSkew8, MOD8};
    for (size_t off = 0; off < S; off += WORKSIZE8) {
        size_t end = off + WORKSIZE8 < S ? off + WORKSIZE8 : S;
        size_t sz = end - off;
        for (int i = 0; i < n; i++) work[i] = wbuf[i];
        for (int i = 0; i < total; i++) sh[i] = shards[i] + off;
        for (int i = 0; i < p; i++) {
            if (present[i + k]) ref_mul8(work[i], sh[i + k], errLocs[i], sz);
            else memset(work[i], 0, sz);
        }
        for (int i = p; i < m; i++) memset(work[i], 0, sz);
        for (int i = 0; i < k; i++) {
            if (present[i]) ref_mul8(work[m + i], sh[i], errLocs[m + i], sz);
            else memset(work[m + i], 0, sz);
        }
        for (int i = m + k; i < n; i++) memset(work[i], 0, sz);
        ifft_dit_decoder8(m + k, work, n, full, sz);
        for (int i = 1; i < n; i++) {
            int width = ((i ^ (i - 1)) + 1) >> 1;
            for (int j = 0; j < width; j++) slice_xor(work[i + j], work[i - width + j], sz);
        }
        fft_dit8(work, m + k, n, full, useBits ? &eb : NULL, sz);
        int endi = recover_all ? total : k;
        for (int i = 0; i < endi; i++) {
            if (present[i]) continue;
            if (i >= k) ref_mul8(sh[i], work[i - k], (uint8_t)(MOD8 - errLocs[i - k]), sz);
            else ref_mul8(sh[i], work[i + m], (uint8_t)(MOD8 - errLocs[i + m]), sz);
        }
    }
#undef EL
    free(present);
    free_rows(wbuf);
    free(work);
    free(sh);
    return ORC_OK;
}

void orc8_tables(uint8_t *log_out, uint8_t *exp_out, uint8_t *skew_out, uint8_t *walsh_out) {
    if (log_out) memcpy(log_out, logLUT8, sizeof(logLUT8));
    if (exp_out) memcpy(exp_out, expLUT8, sizeof(expLUT8));
    if (skew_out) memcpy(skew_out, fftSkew8, sizeof(fftSkew8));
    if (walsh_out) memcpy(walsh_out, logWalsh8, sizeof(logWalsh8));
}
void orc8_mul(uint8_t *x, const uint8_t *y, uint8_t log_m, size_t n) { ref_mul8(x, y, log_m, n); }
uint8_t orc8_mul_log(uint8_t a, uint8_t log_b) { return mul_log8(a, log_b); }

/* ===================================================================== */
/*   Reference-equivalent SIMD port of the GF(2^16) encode (CPU baseline) */
/* ===================================================================== */
/*
 * bench.py's cpu_baseline times this, not the scalar Ref path above: it is
 * the closest stand-in for the reference's own amd64 speed that can run here
 * (no Go toolchain).  It follows the reference's AVX2 path:
 *   - multiply256LUT nibble tables (leopard16.go:1056-1072): for nibble i of a
 *     symbol, 16 low-byte and 16 high-byte products of x << 4i;
 *   - mulgf16 / ifftDIT2 / fftDIT2 / ifftDIT4 / fftDIT4 as VPSHUFB nibble
 *     lookups on 64-byte lo/hi blocks, the radix-4 butterflies fused per
 *     block like ifftDIT4_avx2 / fftDIT4_avx2 (galois_gen_amd64.s:123870-125661),
 *     XOR-only where a twiddle is modulus (the _N variants, galois_amd64.go:184-256);
 *   - the same encode schedule (leopard16.go:128-224, ifftDITEncoder :685-747,
 *     fftDIT :618-657) over whole rows.
 * threads > 1 splits the shard bytes into 64-byte-aligned ranges, one per
 * thread (column independence, leopard16.go:778-792); the reference itself is
 * single-threaded per call.  Checked against the scalar oracle by
 * tests/test_oracle.py.  Test / bench infrastructure only.
 */
#include <immintrin.h>
#include <pthread.h>

static uint8_t (*mul256)[128]; /* [log_m][128]: lo tables [i*16+x], hi tables [64+i*16+x] */

static int init_mul256(void) {
    if (mul256) return 0;
    mul256 = (uint8_t (*)[128])malloc((size_t)ORDER16 * 128);
    if (!mul256) return -1;
    for (int log_m = 0; log_m < ORDER16; log_m++)
        for (int i = 0, shift = 0; i < 4; i++, shift += 4)
            for (int x = 0; x < 16; x++) {
                uint16_t prod = mul_log16((uint16_t)(x << shift), (uint16_t)log_m);
                mul256[log_m][i * 16 + x] = (uint8_t)prod;
                mul256[log_m][64 + i * 16 + x] = (uint8_t)(prod >> 8);
            }
    return 0;
}

typedef struct { __m256i lo[4], hi[4]; } tab256_t;
typedef struct { __m256i lo, hi; } blk_t;
typedef struct { int k, p; uint8_t *const *shards; size_t lo, hi; uint8_t **work; } simd_job_t;

/* The kernels once per ISA (leopard_simd.inc): AVX2 like ifftDIT4_avx2 /
 * fftDIT4_avx2 (galois_gen_amd64.s:123870-125661), and AVX-512 like
 * ifftDIT4_avx512_* / fftDIT4_avx512_* (:121966-123869), which keep the
 * 256-bit nibble-table form but hold the tables in the 16 extra registers
 * AVX-512VL gives and fold each 3-input XOR into one VPTERNLOGD 0x96. */
#define SIMD_NAME(f) f##_avx2
#define SIMD_FN __attribute__((target("avx2")))
#define XOR3(a, b, c) _mm256_xor_si256(_mm256_xor_si256(a, b), c)
#include "leopard_simd.inc"
#undef SIMD_NAME
#undef SIMD_FN
#undef XOR3
#define SIMD_NAME(f) f##_avx512
#define SIMD_FN __attribute__((target("avx2,avx512f,avx512vl,avx512bw")))
#define XOR3(a, b, c) _mm256_ternarylogic_epi32(a, b, c, 0x96)
#include "leopard_simd.inc"
#undef SIMD_NAME
#undef SIMD_FN
#undef XOR3

/* ISAs the CPU runs: bit 0 AVX2, bit 1 AVX-512 (F + VL + BW, what the
 * reference's avx512 path needs, galois_amd64.go:192). */
int orc16_simd_available(void) {
    __builtin_cpu_init();
    int m = __builtin_cpu_supports("avx2") ? 1 : 0;
    if (m && __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512vl") && __builtin_cpu_supports("avx512bw"))
        m |= 2;
    return m;
}

/* Encode with the SIMD port: same contract as orc16_encode (all rows present,
 * S % 64 == 0), geometries whose encode schedule stays inside fftSkew.
 * isa: 1 AVX2, 2 AVX-512, 0 the widest the CPU runs (the reference's own
 * choice, reedsolomon.go option defaults). */
int orc16_encode_simd_isa(int isa, int k, int p, uint8_t *const *shards, size_t S, int threads) {
    const int have = orc16_simd_available();
    if (isa == 0) isa = (have & 2) ? 2 : 1;
    if ((isa != 1 && isa != 2) || !(have & isa)) return ORC_ERR_NOT_SUPPORTED;
    if (k <= 0 || p <= 0 || k + p > ORDER16) return ORC_ERR_INV_SHARD_NUM;
    if (S == 0 || S % 64) return ORC_ERR_INVALID_SHARD_SIZE;
    if (init_mul256()) return ORC_ERR_NOMEM;
    const int m = ceil_pow2(p), nch = (k + m - 1) / m;
    /* every skew index the schedule reads: < (m-1) + nch*m + 3m (chunks), < m (fft) */
    if ((long)(m - 1) + (long)nch * m + m > MOD16) return ORC_ERR_PANIC;
    if (threads < 1) threads = 1;
    const size_t blocks = S / 64;
    if ((size_t)threads > blocks) threads = (int)blocks;
    void *(*job)(void *) = isa == 2 ? simd_encode_job_avx512 : simd_encode_job_avx2;
    simd_job_t *jobs = (simd_job_t *)calloc((size_t)threads, sizeof(simd_job_t));
    pthread_t *tid = (pthread_t *)calloc((size_t)threads, sizeof(pthread_t));
    uint8_t **work = alloc_rows(2 * m, S);  /* one work slab; threads own disjoint byte ranges of it */
    int e = (jobs && tid && work) ? ORC_OK : ORC_ERR_NOMEM;
    for (int t = 0; t < threads && e == ORC_OK; t++)
        jobs[t] = (simd_job_t){k, p, shards, (blocks * t / threads) * 64, (blocks * (t + 1) / threads) * 64, work};
    if (e == ORC_OK) {
        for (int t = 1; t < threads; t++) pthread_create(&tid[t], NULL, job, &jobs[t]);
        job(&jobs[0]);
        for (int t = 1; t < threads; t++) pthread_join(tid[t], NULL);
    }
    free_rows(work);
    free(jobs);
    free(tid);
    return e;
}
int orc16_encode_simd(int k, int p, uint8_t *const *shards, size_t S, int threads) {
    return orc16_encode_simd_isa(0, k, p, shards, S, threads);
}
