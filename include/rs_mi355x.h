/*
 * rs_mi355x.h — C-ABI of the MI355X-native Leopard-FFT Reed-Solomon engine.
 *
 * This is the drop-in boundary for the hot path of bpfs/reedsolomon16: the
 * Go methods leopardFF16/leopardFF8 {Encode, Verify, Reconstruct,
 * ReconstructData, ReconstructSome} are replaced by calls into this library
 * through a thin cgo shim.  Every entry point cites the
 * reference interface it replaces.  Plain pointers and sizes only; no torch
 * or HIP types appear in the signatures (a stream is passed as void*).
 *
 * Shard model (identical to the Go [][]byte model):
 *   shards[0..k)   data shards,  shards[k..k+p) parity shards;
 *   lens[i]        length of shard i; 0 means "missing" (Go: len(shards[i])==0).
 * Encode/Verify require every len equal (checkShards(shards,false),
 * encoder.go:102-115) and a multiple of 64 (leopard16.go:130).
 * GF(2^16) symbol layout: each 64-byte block holds 32 symbols, low bytes in
 * [0,32) and high bytes in [32,64) (leopard16.go:778-792).
 *
 * All calls are thread-safe (one mutex per codec, like the Go encoder's
 * sync.Pool/sync.Once design allows concurrent callers, leopard16.go:25).
 */
#ifndef RS_MI355X_H
#define RS_MI355X_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Error codes: 1:1 with the reference's sentinel errors (reedsolomon.go:15-33). */
#define RS_OK                       0
#define RS_ERR_INV_SHARD_NUM        1  /* ErrInvShardNum        reedsolomon.go:16 */
#define RS_ERR_MAX_SHARD_NUM        2  /* ErrMaxShardNum        reedsolomon.go:17 */
#define RS_ERR_TOO_FEW_SHARDS       3  /* ErrTooFewShards       reedsolomon.go:18 */
#define RS_ERR_SHARD_NO_DATA        4  /* ErrShardNoData        reedsolomon.go:19 */
#define RS_ERR_SHARD_SIZE           5  /* ErrShardSize          reedsolomon.go:20 */
#define RS_ERR_INVALID_SHARD_SIZE   6  /* ErrInvalidShardSize   reedsolomon.go:26 */
#define RS_ERR_NOT_SUPPORTED        7  /* ErrNotSupported       reedsolomon.go:28 */
#define RS_ERR_SHORT_DATA           8  /* ErrShortData          reedsolomon.go:27 */
#define RS_ERR_RECONSTRUCT_REQUIRED 9  /* ErrReconstructRequired reedsolomon.go:25 */
/* Conditions that have no sentinel in the reference: */
#define RS_ERR_PANIC               50  /* the Go code panics (slice index out of range) for this geometry */
#define RS_ERR_NOMEM               51  /* host or device allocation failed */
#define RS_ERR_DEVICE              52  /* HIP runtime / kernel launch failure */
#define RS_ERR_INVALID_ARG         53  /* NULL codec / pointer arguments */

typedef struct rs_codec rs_codec;

/* Construction.  field_bits: 16 -> New16 (reedsolomon.go:90-93, newFF16
 * leopard16.go:36-54); 8 -> New8 (reedsolomon.go:84-87, newFF8
 * leopard8.go:53-75); 0 -> New (reedsolomon.go:69-81: GF(2^8) iff k+p<=256).
 * device: HIP device ordinal the codec's kernels run on.
 * Returns RS_ERR_INV_SHARD_NUM / RS_ERR_MAX_SHARD_NUM like the Go constructors. */
int rs_new(int field_bits, int data_shards, int parity_shards, int device, rs_codec **out);
void rs_free(rs_codec *codec);

/* ---------------- Multi-device codec (the byte-range split) ----------------
 * rs_new_multi: one Encoder (reedsolomon.go:90-93) over `ndevices` GPUs.  Every
 * Leopard operation is column-local (leopard16.go:778-792), so device g owns
 * bytes [lo_g, hi_g) of EVERY shard (rs_byte_range: 64-byte blocks dealt as
 * evenly as possible) and works on them with no data exchange.  The host-
 * memory entry points (rs_encode / rs_verify / rs_reconstruct, their _async
 * forms, rs_ticket_wait / _query, rs_verify_result, rs_set_host_segment,
 * rs_split / rs_join) take the same arguments as for a one-device codec and
 * give the same results: each device's share runs on a host worker thread of
 * its own, over that device's streams and PCIe link; verify ANDs the devices'
 * verdicts on the host; a reconstruct's error locators are computed once and
 * handed to every device (for GF(2^8) with the reference's inversion-cache
 * keying on the full shard size, so the call sequence semantics of
 * rs_set_reference_inversion_cache are unchanged).  devices[] may repeat an
 * ordinal (several parts on one GPU).  ndevices == 1 returns a plain codec.
 * The device-resident entry points (rs_*_dev*) return RS_ERR_INVALID_ARG on a
 * multi-device codec (their rows live on one device): use rs_device_part for
 * device g's own codec, which the multi-device codec owns (never rs_free it). */
#define RS_MAX_DEVICES 64
int rs_new_multi(int field_bits, int data_shards, int parity_shards, const int *devices, int ndevices,
                 rs_codec **out);
/* Number of devices (parts) of a codec: 1 for rs_new. */
int rs_device_count(const rs_codec *codec);
/* Part `index` of a codec (the codec itself for a one-device codec) and its device ordinal. */
int rs_device_part(rs_codec *codec, int index, rs_codec **part, int *device);
/* [*lo, *hi) of the shard bytes part `index` of `nparts` owns; RS_ERR_INVALID_SHARD_SIZE if shard_size % 64. */
int rs_byte_range(size_t shard_size, int index, int nparts, size_t *lo, size_t *hi);

/* Extensions interface (reedsolomon.go:358-375). */
int rs_field_bits(const rs_codec *codec);
int rs_data_shards(const rs_codec *codec);
int rs_parity_shards(const rs_codec *codec);
int rs_total_shards(const rs_codec *codec);
int rs_shard_size_multiple(const rs_codec *codec); /* 64: leopard16.go:58-60 */

/* ---------------- Host-memory entry points (Go [][]byte semantics) ---------------- */

/* Encode: leopardFF16.Encode leopard16.go:116-125 / leopardFF8.Encode
 * leopard8.go:141-150.  Writes parity into shards[k..k+p). */
int rs_encode(rs_codec *codec, uint8_t *const *shards, const size_t *lens, int nshards);

/* Asynchronous Encode for stream pipelining (the analog of rsStream16.encode's
 * per-block loop, streaming16.go:1229-1318): queues the stripe's copy-in,
 * kernels and copy-out behind the codec's previous calls and returns; block
 * j+1's host-to-device copies overlap block j's kernels and device-to-host
 * copies.  The shards must stay valid (and the data rows unmodified) until the
 * ticket completes.  Parity rows in pageable memory make the call synchronous
 * (they go through the pinned bounce slab); pin them (rs_host_alloc /
 * rs_host_register) for overlap.  Same validation and errors as rs_encode. */
int rs_encode_async(rs_codec *codec, uint8_t *const *shards, const size_t *lens, int nshards, uint64_t *ticket);
/* Block until the encode behind `ticket` has written its parity rows. */
int rs_encode_wait(rs_codec *codec, uint64_t ticket);
/* *done = 1 when it has, 0 otherwise (no blocking). */
int rs_encode_query(rs_codec *codec, uint64_t ticket, int *done);

/* Verify: leopard16.go:361-387 / leopard8.go:415-436.  *ok = 1 iff parity matches. */
int rs_verify(rs_codec *codec, uint8_t *const *shards, const size_t *lens, int nshards, int *ok);

/* Asynchronous Verify and Reconstruct for stream pipelining (rsStream16.verify
 * streaming16.go:200-317 and reconstruct :320-468 call r.rs.Verify /
 * r.rs.Reconstruct once per 4 MiB block): queued like rs_encode_async, so block
 * j+1's copies overlap block j's kernels.  One ticket counter serves all three
 * operations; the shard memory must stay valid until the ticket completes.
 * rs_ticket_wait / rs_ticket_query work on any ticket (rs_encode_wait /
 * rs_encode_query are the same functions).  Same validation and errors as the
 * synchronous calls.  rs_reconstruct_async sets lens[i] = S for the shards it
 * will rebuild at call time; when nothing is missing it returns RS_OK with
 * *ticket = 0 (no work queued), which rs_ticket_wait / rs_ticket_query report
 * as complete.  Rebuilt rows in pageable memory make the call
 * synchronous (bounce slab), as for encode. */
int rs_verify_async(rs_codec *codec, uint8_t *const *shards, const size_t *lens, int nshards, uint64_t *ticket);
/* Waits for a verify ticket and reports *ok = 1 iff its parity matched.
 * RS_ERR_INVALID_ARG for a ticket that is not a verify, or older than the last
 * 64 tickets of the codec (its result slot has been reused). */
int rs_verify_result(rs_codec *codec, uint64_t ticket, int *ok);
int rs_reconstruct_async(rs_codec *codec, uint8_t *const *shards, size_t *lens, int nshards, int recover_all,
                         uint64_t *ticket);
int rs_ticket_wait(rs_codec *codec, uint64_t ticket);
int rs_ticket_query(rs_codec *codec, uint64_t ticket, int *done);

/* Reconstruct / ReconstructData / ReconstructSome: leopard16.go:343-358
 * (reconstruct :390-570), leopard8.go:392-407 (reconstruct :439-695).
 * recover_all = 1 (Reconstruct, or ReconstructSome with len(required)==total)
 * or 0 (ReconstructData).  Missing shards have lens[i]==0; for each one that
 * is rebuilt, shards[i] must point at >= S writable bytes (the cgo shim does
 * the Go slice resize, :556-560) and lens[i] is set to S on return. */
int rs_reconstruct(rs_codec *codec, uint8_t *const *shards, size_t *lens, int nshards, int recover_all);

/* EncodeIdx / Update: return RS_ERR_NOT_SUPPORTED (leopard16.go:227-229, 273-275). */
int rs_encode_idx(rs_codec *codec, const uint8_t *data_shard, size_t len, int idx, uint8_t *const *parity,
                  const size_t *parity_lens, int nparity);
int rs_update(rs_codec *codec, uint8_t *const *shards, const size_t *lens, int nshards,
              uint8_t *const *new_data, const size_t *new_lens, int nnew);

/* ---------------- Split / Join (leopard16.go:232-340) ---------------- */
/* Shard size Split would produce for `len` bytes of data: ceil(len/k) rounded
 * up to 64 (leopard16.go:283-288; len when total == 1 and len % 64 == 0).
 * RS_ERR_SHORT_DATA for len == 0. */
int rs_split_shard_size(const rs_codec *codec, size_t len, size_t *per_shard);
/* Split (leopard16.go:277-340) into a caller slab: shard i is written at
 * dst + i*dst_stride (per_shard bytes): data rows get the data, the rest of
 * the last one and every parity row are zeroed (the reference's padding).
 * data and dst may each be host memory (pageable or pinned) or device memory
 * (HBM), so the data can land directly in the device slab the encode reads;
 * device copies run on `stream` (NULL: the codec's stream, synchronous). */
int rs_split(rs_codec *codec, const uint8_t *data, size_t len, uint8_t *dst, size_t dst_stride, void *stream);
/* Join (leopard16.go:231-269): the first out_size bytes of the data shards,
 * in order, into dst.  ErrTooFewShards / ErrReconstructRequired (a missing
 * data shard: lens[i] == 0) / ErrShortData as the reference.  Shards and dst
 * may be host or device memory. */
int rs_join(rs_codec *codec, uint8_t *const *shards, const size_t *lens, int nshards, uint8_t *dst,
            size_t out_size, void *stream);

/* ---------------- Host-resident pipeline controls ---------------- */
/* rs_encode / rs_verify / rs_reconstruct stream the stripe through the GPU in
 * column segments (H2D, kernel and D2H on three streams, 3 staging slabs).
 * Pinned host rows (rs_host_alloc / rs_host_register) make the copies true
 * DMA; pageable rows work but are staged by the runtime.  Rows that are
 * equally spaced (one AllocAligned-style slab) are copied with one 2-D copy
 * per segment.  Segment width per row: `bytes` (multiple of 64) or 0 for
 * automatic (about 8 MiB copied in per segment). */
int rs_set_host_segment(rs_codec *codec, size_t bytes);

/* WARNING -- default behaviour that returns WRONG DATA for some call
 * sequences, exactly as the reference does: every GF(2^8) codec of at most 64
 * shards keeps the reference's inversion cache (below), so a reconstruct whose
 * erasure pattern shares the reference's cache key with an earlier call's
 * rebuilds its shards with that call's locators.  rs_set_reference_inversion_cache
 * (codec, 0) turns it off (always-correct exact keying).
 *
 * GF(2^8) reconstruct with the reference's inversion cache semantics
 * (leopard8.go:508-555, codecs of at most 64 shards: :67-71).  The reference
 * looks its cached errLocs up by the raw erasure bitfield, which leaves out
 * parity erasures unless recoverAll, and stores them under the bitfield after
 * prepare(); a later call whose erasures differ only in ways the key does not
 * see then reuses errLocs computed for another pattern, and rebuilds wrong
 * data.  By default (on = 1) the engine keeps this cache as the reference
 * does, per codec, and reproduces the reference's output call for call, stale
 * results included; on = 0 keys the locators on the exact erasure pattern and
 * always rebuilds the right data.  Each call of this function clears the cache, as a fresh
 * newFF8 would.  No effect on GF(2^16) codecs or above 64 shards. */
int rs_set_reference_inversion_cache(rs_codec *codec, int on);
/* Pinned, 64-byte-aligned host memory: AllocAligned (unsafe.go:17-41) for
 * shards that are to cross PCIe at full rate. */
int rs_host_alloc(size_t bytes, void **out);
void rs_host_free(void *ptr);
/* Pin existing host memory (e.g. a Go slab held by runtime.Pinner). */
int rs_host_register(void *ptr, size_t bytes);
int rs_host_unregister(void *ptr);

/* ---------------- Device-resident entry points (HBM in, HBM out) ---------------- */
/* Streams: a hipStream_t (asynchronous on it), NULL (the codec's own stream;
 * the call completes before it returns), or RS_NULL_STREAM: HIP's null
 * (legacy default) stream, asynchronous -- the handle 0 a caller's default
 * stream has (torch.cuda.default_stream().cuda_stream == 0), which NULL
 * cannot express. */
#define RS_NULL_STREAM ((void *)~(uintptr_t)0)
/* d_shards: HOST array of k+p DEVICE pointers, each to shard_size bytes
 * (4-byte aligned; 64-byte aligned recommended).  rs_encode_dev is
 * asynchronous on a caller stream when the rows are equally strided (the
 * common AllocAligned slab layout), rs_reconstruct_dev when n <= 256; the
 * other calls return after their work is complete. */
int rs_encode_dev(rs_codec *codec, uint8_t *const *d_shards, size_t shard_size, void *stream);
int rs_verify_dev(rs_codec *codec, uint8_t *const *d_shards, size_t shard_size, int *ok, void *stream);
/* present[i] != 0 marks shard i present; rebuilt rows are written into d_shards[i]. */
int rs_reconstruct_dev(rs_codec *codec, uint8_t *const *d_shards, const uint8_t *present, size_t shard_size,
                       int recover_all, void *stream);

/* Batched device reconstruct with ONE erasure pattern (the usual repair after
 * a lost device: every stripe misses the same shard indices): nstripes
 * stripes, shard i of stripe z at base + z*stripe_stride + i*row_stride, all
 * rebuilt in place in one launch (the LDS-resident kernel, grid.y = stripe)
 * for codecs whose decode transform has n <= 256, stripe by stripe otherwise.
 * Per stripe it is leopardFF16/FF8.Reconstruct (recover_all != 0) or
 * ReconstructData (leopard16.go:351-358, leopard8.go:392-407) on that
 * stripe's rows; present[] has k+p entries.  Same error rules and stream
 * semantics as rs_reconstruct_dev.  row_stride >= shard_size; stripe_stride
 * >= (k+p)*row_stride when nstripes > 1. */
int rs_reconstruct_dev_batch(rs_codec *codec, uint8_t *base, size_t row_stride, size_t stripe_stride, size_t nstripes,
                             const uint8_t *present, size_t shard_size, int recover_all, void *stream);

/* Batched device encode of `nstripes` independent stripes laid out as one slab
 * per stripe: stripe j, shard i at d_base + j*stripe_stride + i*row_stride.
 * Asynchronous on `stream`. */
int rs_encode_dev_batch(rs_codec *codec, uint8_t *d_base, size_t row_stride, size_t stripe_stride,
                        int nstripes, size_t shard_size, void *stream);
/* Verify (leopard16.go:361-387) of nstripes strided stripes in one launch
 * (rs_encode_dev_batch's layout): *ok = 1 when every stripe's parity matches
 * its data, 0 when any stripe differs.  Synchronous (the flag is read back). */
int rs_verify_dev_batch(rs_codec *codec, uint8_t *d_base, size_t row_stride, size_t stripe_stride, int nstripes,
                        size_t shard_size, int *ok, void *stream);

/* Name of the kernel path the codec uses for encode ("reg-m32", "lds", "multipass", ...). */
const char *rs_encode_path(const rs_codec *codec);

/* ---------------- Host-only diagnostics (no device calls; used by CPU tests) ---------------- */
/* Field tables as built by the engine (initLUTs/initFFTSkew, leopard16.go:940-1031). */
int rs_debug_field_tables(int field_bits, uint16_t *log_out, uint16_t *exp_out, uint16_t *skew_out,
                          uint16_t *walsh_out);
/* Byte-permute twiddle image of "multiply by exp(log_m)" (rs_debug_twiddle_dwords() dwords). */
int rs_debug_twiddle(int field_bits, uint32_t log_m, uint32_t *out);
int rs_debug_twiddle_dwords(int field_bits);
/* GF(2^8)-subfield coordinates of GF(2^16) (x0, x1) = (lo ^ D(hi), hi): 0 when the
 * engine verified that a subfield product acts as one 8x8 map on both bytes. */
int rs_debug_sub_check(void);
/* 8-dword subfield table of "multiply by exp(log_m)"; -1 if exp(log_m) is not in GF(2^8). */
int rs_debug_sub_twiddle(uint32_t log_m, uint32_t *out);
/* Symbol <-> subfield coordinates (an involution). */
uint32_t rs_debug_sub_swap(uint32_t x);
/* Error locators for an erasure pattern (leopard16.go:433-470); out has 2^field_bits entries.
 * Returns RS_ERR_PANIC where the reference panics. */
int rs_debug_error_locators(int field_bits, int data_shards, int parity_shards, const uint8_t *erased,
                            uint32_t *out);

/* Checks the half-wave split schedules of the GF(2^16) encode kernel
 * (logm 2..5) against the plain butterfly order on random symbols and
 * twiddles, on the host.  Returns the number of differing rows (0 = equal). */
int rs_debug_split_check(int logm, uint32_t seed);
/* Host emulation of the split encode kernel's data flow (same twiddle images,
 * byte-permute multiply and half-wave layout): data = k rows of S bytes,
 * parity = p rows of S bytes.  GF(2^16) codecs with 4 <= m <= 32 only. */
int rs_debug_split_emulate(rs_codec *codec, const uint8_t *data, uint8_t *parity, size_t shard_size);
/* The bit-sliced n = 256 reconstruct's wave plan (csrc/bitslice_dec.hip
 * make_plan) for work rows [0, mtrunc) with revealed-row mask need[8] (bit r:
 * work row r): per wave w, bits 16 (w % 4) .. of code[w / 4] hold four 4-bit
 * fields (unit + 1, 0 = none): phase-3 units 0, 1, phase-1 units 0, 1.
 * Returns 0, or -1 when the kernel does not serve mtrunc.  Host only. */
int rs_debug_dec_plan(int mtrunc, const uint32_t *need, uint64_t *code);

/* 1 when the host reconstruct would move these rows (S bytes each) with its
 * zero-copy kernels: every row 16-byte aligned and mapped for the device from
 * its first to its last byte, contiguously (codec.cpp zc_rows); 0 when it
 * would copy them.  Pointer queries only, nothing is launched. */
int rs_debug_zc_rows(uint8_t *const *rows, int nrows, size_t S);

/* Test-only kernel-path overrides (process-wide), so the parity tests can run
 * the variants other geometries select on the same small inputs:
 *   "bs" 0/1          bit-sliced GF(2^16) encode off / on (default 1; read by rs_new),
 *   "sub" 0/1         subfield-coordinate transforms off / on (default 1),
 *   "prune" 0/1       errorBitfield pruning of the reconstruct FFT off / on (default 1),
 *   "unit_width" -1/0/1  LDS and GF(2^8) register units automatic / wide / narrow (default -1),
 *   "hp_tiles" 0..64  bit-sliced encode tiles per workgroup, 0 = automatic (default 0),
 *   "hp_step" >= 0    distance in tiles between a workgroup's tiles, 0 = the grid size (default 0),
 *   "hp_tune" 0/1     run-time choice of the bit-sliced encode's tile map by timing both
 *                     on the first launches of a shape (default 1; 0: the static rule),
 *   "rec_half" 0/1    GF(2^16) reconstruct with n = 1024 / 2048 in 32-byte half tiles, two
 *                     workgroups per CU (1), or 64-byte tiles, one per CU (0),
 *   "dec_lab" 0..255  schedule variants of the bit-sliced n = 256 decoder (0: the product),
 *   "lds_big" 0/1     GF(2^16) encode with m = 512 .. 4096 and reconstruct with n = 4096 / 8192 in one
 *                     LDS-resident launch (1, default) or the multi-pass kernels (0),
 *   "zc"      0..3    host reconstruct over pinned mapped rows: zero-copy kernels move the
 *                     present rows in (bit 0) and the rebuilt rows out (bit 1) (default 3);
 *                     a cleared bit keeps that direction's per-run hipMemcpy copies.
 * Returns RS_ERR_INVALID_ARG for an unknown knob or value.  Host only. */
int rs_debug_set_path(const char *knob, int value);

/* Human-readable message for an error code. */
const char *rs_strerror(int code);

#ifdef __cplusplus
}
#endif
#endif /* RS_MI355X_H */
