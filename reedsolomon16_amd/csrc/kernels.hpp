// Launcher interface between the host codec (codec.cpp) and the HIP kernels
// (kernels.hip).  Only plain pointers and sizes cross this boundary.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

namespace rs {

// A set of shard rows in device memory: either an explicit device array of
// row pointers, or base + i*stride.
struct RowSet {
    uint8_t *const *table;  // device array (nullable)
    uint8_t *base;
    uint64_t stride;
    // strided only: nstripes stripes at base + y * stripe_stride (grid.y), one erasure pattern
    uint64_t stripe_stride;
    int nstripes;
};

// Fused register-resident encode (m <= 32): one lane owns a column unit of
// every row; chunked IFFT + XOR-accumulate + FFT stay in VGPRs.
struct EncodeArgs {
    RowSet data;            // k rows
    RowSet parity;          // p rows
    int k, p, nchunks;
    uint64_t shard_size;    // bytes per row
    uint64_t stripe_stride; // batched: byte offset between stripes (applied to both RowSets' base)
    int nstripes;
    const uint32_t *tw_ifft;  // nchunks * ifft_slots(logm) twiddle tables
    const uint32_t *tw_fft;   // fft_slots(logm) twiddle tables
    int *mismatch;            // verify: set to 1 on any parity mismatch
    // Optional (GF(2^16), LDS kernel, even log m): the final FFT in subfield
    // coordinates.  Every fftDIT twiddle of an m <= 256 encode is fftSkew[< 255],
    // an element of GF(2^8) (leopard16.go:218-221), so the transform runs on
    // (lo ^ D(hi), hi) with kTwDwords8 subfield tables (6 v_perm_b32 per product
    // instead of 12); tw_dmap is the byte map D (make_sub_dmap).  nullptr: full field.
    // m = 1024, 4096: the FFT passes before big_sub_fft_end only (zero tables after them).
    const uint32_t *tw_fft_sub;
    const uint32_t *tw_dmap;
    // Optional (with tw_fft_sub): chunk c's IFFT passes from ifft_nff[c] on in
    // subfield coordinates too (tw_ifft_sub: nchunks x ifft_slots(logm)
    // kTwDwords8 tables, zero where a slot is full-field): the passes before it
    // run full-field and the last of them changes coordinates on its way into
    // the LDS image.  Every later slot of the chunk lies in GF(2^8).
    const uint32_t *tw_ifft_sub;
    const int *ifft_nff;
};

// Returns hipSuccess or the launch error.  logm in [0, 5].
// Subfield passes of the n = 512..2048 LDS reconstruct (k_rec_lds BigSub):
// the IFFT's radix-4 passes from big_sub_ifft_first(logn) on and the FFT's
// passes before big_sub_fft_end(logn) run in GF(2^8)-subfield coordinates.
// The host (codec.cpp upload_big_sub) checks every twiddle slot of exactly
// these passes against the schedule, so both sides share these definitions.
constexpr int big_sub_ifft_first(int logn) { return logn >= 13 ? 3 : logn >= 11 ? 2 : 1; }
constexpr int big_sub_fft_end(int logn) { return (void)logn, 4; }

// Test-only kernel-path overrides (rs_debug_set_path, codec.cpp): the LDS /
// register unit width, -1 = automatic, 0 = wide, 1 = narrow.
int unit_width_override();
// The bit-sliced encode's tiles per workgroup: 0 = automatic, n >= 1 forces n;
// and the distance in tiles between a workgroup's tiles, 0 = the grid size.
int hp_tiles_override();
int hp_step_override();
bool hp_tune_enabled();
bool rec_half_enabled();

hipError_t launch_encode_reg(int bits, int logm, bool verify, const EncodeArgs &a, hipStream_t s);
// Half-wave split encode (GF(2^16), logm 2..5, strided rows only: data.table ==
// nullptr, and (k-1)*stride + shard_size < 2^32).  tw_ifft = nchunks images of
// split_image_dwords(logm, false) dwords, tw_fft = one image of
// split_image_dwords(logm, true) dwords (codec.cpp lays them out from
// schedule.hpp's EncodeSplit<logm>).
hipError_t launch_encode_split(int logm, bool verify, const EncodeArgs &a, hipStream_t s);
// Name of the register-kernel variant (for diagnostics / profiles).
const char *encode_reg_name(int bits, int logm);

// ---- Multi-pass building blocks (any m / n; work rows contiguous, stride = shard_size) ----
// work[dst0 + r] = r < cnt ? src.row(row0 + r) : 0, for r in [0, rows)
hipError_t launch_gather(int bits, uint8_t *work, uint64_t S, RowSet src, int row0, int cnt, int rows, hipStream_t s);
// One radix-4 (or radix-2) pass over rows [0, M) of work (inverse or forward).
// groups_active: butterfly groups whose first row < mtrunc (the rest are skipped).
hipError_t launch_pass(int bits, bool inverse, uint8_t *work, uint64_t S, int dist, int radix, int groups_active,
                       const uint32_t *tw_pass, hipStream_t s);
// dst[r] ^= src[r] for r in [0, rows)
// Zero-copy row moves between a device staging slab and pinned host rows the
// device maps (codec.cpp host_pipeline): entry i is host row host[i] (device
// view) <-> slab row slab_row[i].  Passed by value (kernel arguments).
constexpr int kZcMax = 256;
struct ZcRows {
    uint8_t *host[kZcMax];
    uint16_t slab_row[kZcMax];
    int n;
};
// bytes [off, off + w) of every host row <-> the same bytes' slab row at
// slab + slab_row * pitch (column 0 = off); w a multiple of 16
hipError_t launch_zc_copy(const ZcRows &r, uint8_t *slab, uint64_t pitch, uint64_t off, uint64_t w, bool to_host,
                          hipStream_t s);
hipError_t launch_xor_rows(int bits, uint8_t *dst, const uint8_t *src, uint64_t S, int rows, hipStream_t s);
// out.row(r) = work[r]  (verify: compare, set *mismatch)
hipError_t launch_copy_out(int bits, RowSet out, const uint8_t *work, uint64_t S, int rows, int *mismatch,
                           hipStream_t s);
// work[r] = src[r] ? src[r] * tw[r] : 0 for r in [0, rows); src: device array of row pointers
hipError_t launch_scale_in(int bits, uint8_t *work, uint64_t S, const uint8_t *const *src, const uint32_t *tw, int rows,
                           hipStream_t s);
// In-place formal derivative over n rows (leopard16.go:527-530, closed form).
hipError_t launch_formal_derivative(int bits, uint8_t *work, uint64_t S, int n, hipStream_t s);
// dst[i] = work[pos[i]] * tw[i] for i in [0, count)
hipError_t launch_reveal(int bits, uint8_t *const *dst, const uint8_t *work, uint64_t S, const int *pos,
                         const uint32_t *tw, int count, hipStream_t s);


// ---- LDS-resident paths: one workgroup per 128-byte tile of every row ----
// Reconstruct of one stripe over n = 2^logn <= 2048 work rows.
struct RecArgs {
    const uint8_t *const *src;  // n device row pointers (nullptr: zero row)
    uint8_t *const *dst;        // nd output rows
    // strided shards (base != nullptr, LDS-resident kernel only): shard i at
    // base + i*stride; work row r reads shard src_idx[r] (-1: zero row),
    // output j is shard dst_idx[j]; src / dst are then unused
    uint8_t *base;
    uint64_t stride;
    // strided only: nstripes stripes at base + y * stripe_stride (grid.y), one erasure pattern
    uint64_t stripe_stride;
    int nstripes;
    const int *src_idx, *dst_idx;
    const int *pos;             // work row of each output
    const uint32_t *tw_in;      // n tables: errLocs scalings (mulgf16 semantics)
    const uint32_t *tw_out;     // nd tables: modulus - errLocs[pos]
    const uint32_t *tw_ifft;    // decoder IFFT schedule (ifft_slots(logn) tables)
    const uint32_t *tw_fft;     // decoder FFT schedule (fft_slots(logn) tables)
    uint64_t S;
    int mtrunc;                 // m + k
    int m;                      // work rows before the data rows (outputs: data rows m.., then parity rows 0..)
    int nd;
    // errorBitfield analog (leopard16.go:1076-1252): bit r set when work row r
    // is revealed; FFT groups whose rows are all unset are skipped.
    int prune;
    uint32_t need[8];           // n <= 256 rows
    // n = 512 .. 8192 (GF(2^16)): the revealed-row mask as n / 32
    // words and each work row's output index (-1: not revealed), both in HBM
    const uint32_t *need_w;
    const int *rev;
    // n = 512 .. 8192, optional: subfield tables (kTwDwords8, zero where a slot
    // is full-field) of the passes kernels.hip BigSub<logn> runs in subfield
    // coordinates, and the coordinate-change map; nullptr: full field throughout
    const uint32_t *tw_ifft_sub, *tw_fft_sub, *tw_dmap;
    // schedule variants of the bit-sliced n = 256 decoder (rs_debug_set_path
    // "dec_lab"; 0 = the product schedule; lab A/B only)
    int lab;
};
// sub: GF(2^16) transforms in subfield coordinates (tw_ifft/tw_fft are
// kTwDwords8 subfield tables; tw_in/tw_out fold in the coordinate change).
// logn <= 8, or GF(2^16) with logn <= kMaxLdsRecLogN16 (full field, need_w / rev set;
// n = 4096 / 8192 in 32-byte half / 16-byte quarter tiles, 1024 threads).
constexpr int kMaxLdsRecLogN16 = 13;
hipError_t launch_rec_lds(int bits, int logn, bool sub, const RecArgs &a, hipStream_t s);
// Bit-sliced reconstruct (csrc/bitslice_dec.hip): GF(2^16), n = 256, transforms
// in subfield coordinates (tw_ifft / tw_fft: kTwDwords8 subfield tables,
// tw_in / tw_out: full-field images that fold in the coordinate change), and
// m + k <= 160 (its LDS image).
bool rec_bs256_available(int bits, int logn, bool sub, int mtrunc);
hipError_t launch_rec_bs256(const RecArgs &a, hipStream_t s);
// Encode (or verify) for 2 <= logm <= 8, and GF(2^16) up to kMaxLdsEncLogM16
// (64-byte tiles, 32-byte half tiles at m = 2048, 16-byte quarter tiles at
// m = 4096), twiddles as for launch_encode_reg.
constexpr int kMaxLdsEncLogM16 = 12;
hipError_t launch_encode_lds(int bits, int logm, bool verify, const EncodeArgs &a, hipStream_t s);


// ---- Bit-sliced encode (csrc/bitslice.hip): GF(2^16), m = 16 or 32
// (9 <= p <= 32), k up to the chunk count compiled into the per-m tables
// (Makefile BS_CHUNKS).  Strided rows, one row stride for data and parity.
struct BsArgs {
    const uint8_t *data;    // stripe 0, data row 0
    uint8_t *parity;        // stripe 0, parity row 0
    uint64_t row_stride, stripe_stride, S;
    int k, p, nstripes;
    int tiles_per_stripe, ntiles;  // set by the launcher
    int tpw, tile_step;            // set by the launcher: tiles per workgroup, tile distance between them
    uint32_t span, pspan;          // set by the launcher: (k-1)*row_stride + S, (p-1)*row_stride + S
    int *mismatch;          // verify
};
// True when the tables cover (k, p) and agree with the geometry's own
// schedule (encode_schedule: nchunks * ifft_slots(logm) IFFT logs, then
// fft_slots(logm) FFT logs; entries == mod are truncated groups).
bool encode_bs_available(int k, int p, const uint32_t *ifft_logs, const uint32_t *fft_logs, uint32_t mod);
// Buffer offsets are 32-bit: every row the kernel addresses -- the padding
// rows of the last chunk (read as zeros by the range check only while their
// offset does not wrap) and the lanes of the last tile past the row end --
// must lie below 4 GiB from the stripe's first data row.
bool encode_bs_fits(int k, int p, uint64_t row_stride, uint64_t S);
// cus: compute units of the device (the launcher sizes its persistent grid).
// hipErrorNotSupported when the rows of one stripe span >= 4 GiB (32-bit buffer offsets).
hipError_t launch_encode_bs(bool verify, const BsArgs &a, int cus, hipStream_t s);


}  // namespace rs
