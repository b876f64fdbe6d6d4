// Host side of the MI355X Reed-Solomon engine: the reference's codec
// interface (leopardFF16 / leopardFF8: Encode, Verify, Reconstruct,
// ReconstructData, ReconstructSome) over HIP kernels, exported as the C-ABI
// declared in include/rs_mi355x.h.
//
// Validation order and error codes follow the reference line by line:
//   Encode       leopard16.go:116-135   (checkShards encoder.go:102-115)
//   Verify       leopard16.go:361-387
//   reconstruct  leopard16.go:390-430
// GF(2^8) twins: leopard8.go:141-150, 415-436, 439-480.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <list>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/rs_mi355x.h"
#include "gf_host.hpp"
#include "kernels.hpp"
#include "multi.hpp"
#include "schedule.hpp"

using namespace rs;

namespace {

constexpr int kMaxRegLogM = 5;  // m <= 32: fused register kernel
constexpr int kMaxLdsLogN = 8;  // n (or m) <= 256: LDS-resident transform kernels
constexpr int kHostBufs = 3;    // staging slabs of the host-resident pipeline
constexpr uint64_t kHostSegTarget = 32ull << 20;  // bytes copied in per segment (scripts/host_seg_sweep.py: 256 KiB rows at 128+32)

template <class T>
struct DevBuf {
    T *p = nullptr;
    size_t n = 0;  // elements
    hipError_t ensure(size_t want) {
        if (want <= n) return hipSuccess;
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
        hipError_t e = hipMalloc(&p, want * sizeof(T));
        if (e == hipSuccess) n = want;
        return e;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
    }
};

// Scoped hipSetDevice that restores the caller's device.
struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev) {
        (void)hipGetDevice(&prev);
        if (prev != dev) (void)hipSetDevice(dev);
    }
    ~DeviceGuard() {
        int cur = -1;
        (void)hipGetDevice(&cur);
        if (prev >= 0 && cur != prev) (void)hipSetDevice(prev);
    }
};

#define HIP_TRY(x)                                   \
    do {                                             \
        hipError_t e_ = (x);                         \
        if (e_ != hipSuccess) return RS_ERR_DEVICE;  \
    } while (0)

// Host half of a reconstruct (leopard16.go:432-568) for one erasure pattern:
// which shard feeds each of the n work rows, the input scalings (errLocs),
// which shards are rebuilt from which work row, and their output scalings.
struct RecPlan {
    std::vector<int> src_shard;   // n entries: shard index feeding work row r, or -1 (zero row)
    std::vector<int> dst_shard;   // shards to rebuild, ascending
    std::vector<int> pos;         // work row each rebuilt shard is read from
    std::vector<uint32_t> tw_in, tw_out;
};

// A cached reconstruct plan with its per-pattern tables (scale-in / reveal
// images, rebuilt-row positions) resident in HBM: rs_reconstruct_dev of a
// pattern seen before uploads only its row pointers.
struct DevPlan {
    RecPlan pl;
    DevBuf<uint8_t> blob;
    const uint32_t *tw_in = nullptr, *tw_out = nullptr;
    const int *pos = nullptr;
    const int *src_idx = nullptr, *dst_idx = nullptr;  // pl.src_shard / pl.dst_shard (strided launches)
    uint32_t need[8] = {};
    const uint32_t *need_w = nullptr;  // the revealed-row mask, n / 32 words (kernels read it for n > 256)
    const int *rev = nullptr;          // output index of each work row, -1: not revealed (n > 256)
    // One event per stream that launched with this plan, recorded after each
    // such launch: an eviction frees blob only after the last launch on every
    // one of those streams (one event alone would cover only the latest).
    std::vector<std::pair<hipStream_t, hipEvent_t>> used;
    hipError_t mark_used(hipStream_t s) {
        for (auto &u : used)
            if (u.first == s) return hipEventRecord(u.second, s);
        // a new stream: first drop the streams whose last launch has finished
        // (short-lived caller streams would otherwise pile up events)
        for (size_t i = 0; i < used.size();) {
            if (hipEventQuery(used[i].second) == hipSuccess) {
                (void)hipEventDestroy(used[i].second);
                used[i] = used.back();
                used.pop_back();
            } else {
                i++;
            }
        }
        hipEvent_t ev = nullptr;
        hipError_t e = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
        if (e != hipSuccess) return e;
        used.emplace_back(s, ev);
        return hipEventRecord(ev, s);
    }
    ~DevPlan() {
        for (auto &u : used) {
            (void)hipEventSynchronize(u.second);
            (void)hipEventDestroy(u.second);
        }
        blob.release();
    }
};

}  // namespace

struct rs_codec {
    int bits = 16, k = 0, p = 0, total = 0, m = 1, logm = 0, device = 0;
    const Field *F = nullptr;
    int twd = kTwDwords16;
    std::mutex mu;
    hipStream_t stream = nullptr;

    // encode plan
    bool enc_ok = false, dev_ready = false;
    int nchunks = 0;
    std::vector<uint32_t> enc_ifft_logs, enc_fft_logs;
    DevBuf<uint32_t> tw_ifft, tw_fft;
    bool split_ok = false;            // half-wave split kernel available (GF(2^16), 4 <= m <= 32)
    bool bs_ok = false;               // bit-sliced kernel covers (k, p) (GF(2^16), m = 16 or 32)
    int cus = 0;                      // compute units of the device (persistent grids)
    DevBuf<uint32_t> tws_ifft, tws_fft;
    // LDS-kernel encode (GF(2^16), even log m): the final FFT's subfield tables
    // and the coordinate-change map (EncodeArgs::tw_fft_sub / tw_dmap)
    DevBuf<uint32_t> tw_fft_sub, tw_dmap;
    bool fft_sub = false;  // its twiddle images (schedule.hpp EncodeSplit)
    // ... and the chunk IFFT passes from ifft_nff[c] on (EncodeArgs::tw_ifft_sub)
    DevBuf<uint32_t> tw_ifft_sub;
    DevBuf<int> ifft_nff;
    bool ifft_sub = false;
    std::string path;

    // decode plan (built on first reconstruct)
    bool dec_built = false, dec_ok = false;
    bool dec_sub = false;  // LDS reconstruct runs its transforms in subfield coordinates
    int n = 0, logn = 0;
    DevBuf<uint32_t> dtw_ifft, dtw_fft;
    // n = 512..2048: subfield tables of the passes that run in subfield
    // coordinates (RecArgs::tw_ifft_sub / tw_fft_sub, kernels.hip BigSub)
    bool dec_big_sub = false;
    DevBuf<uint32_t> dtw_ifft_sub, dtw_fft_sub, dec_dmap;

    // scratch shared by the codec's calls (row table, multi-pass work rows,
    // reconstruct blob).  Calls may run on different caller streams and the
    // device-resident encodes return before their kernels finish, so every call
    // records scratch_ev after its last launch, and the next call orders itself
    // behind it (stream wait) before touching the scratch (host wait before a
    // host-side overwrite or a reallocation).
    hipEvent_t scratch_ev = nullptr;
    bool scratch_used = false;
    hipStream_t scratch_stream = nullptr;  // stream of the last scratch user
    DevBuf<uint8_t> work;
    DevBuf<uint8_t *> rows;         // row-pointer table (non-strided inputs)
    std::vector<uint8_t *> rows_host;
    int *hflag = nullptr, *dflag = nullptr;  // verify mismatch word: device word + pinned host readback
    // per-call reconstruct inputs, packed into one blob and uploaded with one copy
    DevBuf<uint8_t> rc_blob;
    uint8_t *rc_host = nullptr;  // pinned staging of the blob
    size_t rc_host_n = 0;
    const uint8_t **rc_src = nullptr;
    uint8_t **rc_dst = nullptr;
    uint32_t *rc_tw_in = nullptr, *rc_tw_out = nullptr;
    int *rc_pos = nullptr;

    // reconstruct plans keyed by (erasure pattern, recover_all) (bounded LRU)
    std::list<std::pair<std::vector<uint8_t>, RecPlan>> plan_cache;
    // device-resident plans of rs_reconstruct_dev (same key), and a ring of
    // per-call row-pointer slots (pinned host + HBM), each reusable once the
    // launch that read it has finished (ring_ev)
    std::list<std::pair<std::vector<uint8_t>, std::unique_ptr<DevPlan>>> dplan_cache;
    static constexpr int kRing = 8;
    DevBuf<uint8_t> ring_dev;
    uint8_t *ring_host = nullptr;
    size_t ring_slot = 0;  // bytes per slot
    hipEvent_t ring_ev[kRing] = {};
    bool ring_used[kRing] = {};
    int ring_next = 0;

    // error-locator cache keyed by erasure pattern (bounded LRU)
    std::list<std::pair<std::vector<uint8_t>, std::vector<uint32_t>>> el_cache;
    // rs_set_reference_inversion_cache: the GF(2^8) inversion cache exactly as
    // leopard8.go:508-555 keys it (raw erasure bits on lookup, bits after
    // prepare() on store), so the output is the reference's on every call
    // sequence; on by default (a drop-in returns the reference's bytes), off
    // keys the locators on the exact pattern
    bool ref_inv = true;
    std::map<std::array<uint64_t, 4>, std::vector<uint32_t>> ref_inv_cache;

    // host-resident pipeline (rs_encode / rs_verify / rs_reconstruct): copy-in,
    // compute and copy-out streams over kHostBufs rotating staging slabs
    hipStream_t s_in = nullptr, s_out = nullptr;
    hipEvent_t ev_in[kHostBufs] = {}, ev_k[kHostBufs] = {}, ev_free[kHostBufs] = {};
    DevBuf<uint8_t> stage;
    uint64_t host_seg_bytes = 0;  // 0: automatic
    // staging-slab rotation continues across calls, so the segments of an
    // asynchronous encode queue behind the previous call's (rs_encode_async)
    uint64_t pipe_seq = 0;
    // asynchronous calls (encode / verify / reconstruct): ticket t completes at
    // done_ev[t % kTickets]; a verify ticket's mismatch word is slot t % kTickets
    // of tk_dflag (device), copied to tk_hflag (pinned) by the ticket's own work
    static constexpr int kTickets = 64;
    hipEvent_t done_ev[kTickets] = {};
    uint64_t next_ticket = 1;
    int *tk_hflag = nullptr, *tk_dflag = nullptr;
    uint8_t tk_kind[kTickets] = {};  // HostOp of the slot's latest ticket, + 1
    // pinned bounce slabs for outputs in pageable host memory (kHostBufs x total x seg)
    uint8_t *bounce = nullptr;
    size_t bounce_n = 0;

    // rs_new_multi: the per-device parts (this codec then owns no device
    // resources of its own; its caches hold the reconstruct locators)
    Multi *multi = nullptr;

    ~rs_codec() {
        if (multi) multi_destroy(multi);  // joins the part workers, frees the parts
        multi = nullptr;
        if (!dev_ready && !stream) return;
        DeviceGuard g(device);
        if (stream) (void)hipStreamSynchronize(stream);
        if (scratch_ev) {
            (void)hipEventSynchronize(scratch_ev);
            (void)hipEventDestroy(scratch_ev);
        }
        tw_ifft.release(); tw_fft.release(); tws_ifft.release(); tws_fft.release(); tw_fft_sub.release(); tw_dmap.release(); tw_ifft_sub.release(); ifft_nff.release(); dtw_ifft.release(); dtw_fft.release(); dtw_ifft_sub.release(); dtw_fft_sub.release(); dec_dmap.release();
        work.release(); rows.release();
        if (hflag) (void)hipHostFree(hflag);
        if (dflag) (void)hipFree(dflag);
        rc_blob.release();
        if (rc_host) (void)hipHostFree(rc_host);
        dplan_cache.clear();  // each plan waits for its last launch
        for (int i = 0; i < kRing; i++)
            if (ring_ev[i]) {
                (void)hipEventSynchronize(ring_ev[i]);
                (void)hipEventDestroy(ring_ev[i]);
            }
        ring_dev.release();
        if (ring_host) (void)hipHostFree(ring_host);
        if (s_in) (void)hipStreamSynchronize(s_in);
        if (s_out) (void)hipStreamSynchronize(s_out);
        stage.release();
        if (bounce) (void)hipHostFree(bounce);
        for (int t = 0; t < kTickets; t++)
            if (done_ev[t]) (void)hipEventDestroy(done_ev[t]);
        if (tk_hflag) (void)hipHostFree(tk_hflag);
        if (tk_dflag) (void)hipFree(tk_dflag);
        for (int b = 0; b < kHostBufs; b++) {
            if (ev_in[b]) (void)hipEventDestroy(ev_in[b]);
            if (ev_k[b]) (void)hipEventDestroy(ev_k[b]);
            if (ev_free[b]) (void)hipEventDestroy(ev_free[b]);
        }
        if (s_in) (void)hipStreamDestroy(s_in);
        if (s_out) (void)hipStreamDestroy(s_out);
        if (stream) (void)hipStreamDestroy(stream);
    }
};

namespace {

// Butterfly twiddle tables (zero twiddles as all-zero tables).
int upload_twiddles(rs_codec *c, const std::vector<uint32_t> &logs, DevBuf<uint32_t> &dst) {
    std::vector<uint32_t> host(std::max<size_t>(logs.size(), 1) * c->twd, 0);
    for (size_t i = 0; i < logs.size(); i++) make_twiddle(*c->F, logs[i], host.data() + i * c->twd, true);
    HIP_TRY(dst.ensure(host.size()));
    HIP_TRY(hipMemcpy(dst.p, host.data(), host.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
    return RS_OK;
}

// ---- half-wave split kernel: table layout from the same compile-time schedule
struct SplitTabs {
    std::vector<int> lo, hi;  // twiddle slot per table load (-1: zero table)
};
template <class S>
void split_tabs_of(const S &s, SplitTabs &t) {
    t.lo.assign(s.tab_lo, s.tab_lo + s.ntab);
    t.hi.assign(s.tab_hi, s.tab_hi + s.ntab);
}
template <int L>
void split_tabs_t(bool fft, SplitTabs &t) {
    if (fft) split_tabs_of(EncodeSplit<L>::fft, t);
    else split_tabs_of(EncodeSplit<L>::ifft, t);
}
bool split_tabs(int logm, bool fft, SplitTabs &t) {
    switch (logm) {
        case 2: split_tabs_t<2>(fft, t); return true;
        case 3: split_tabs_t<3>(fft, t); return true;
        case 4: split_tabs_t<4>(fft, t); return true;
        case 5: split_tabs_t<5>(fft, t); return true;
    }
    return false;
}
// Image of one transform: [lower-half tables | upper-half tables], each table
// 24 dwords; logs[slot] are the reference's twiddle logs for that transform.
void split_image(const Field &F, const SplitTabs &t, const uint32_t *logs, uint32_t *out) {
    const size_t nt = t.lo.size();
    for (size_t i = 0; i < nt; i++) {
        make_twiddle(F, t.lo[i] < 0 ? F.mod : logs[t.lo[i]], out + i * kTwDwords16, true);
        make_twiddle(F, t.hi[i] < 0 ? F.mod : logs[t.hi[i]], out + (nt + i) * kTwDwords16, true);
    }
}
int upload_split(rs_codec *c) {
    SplitTabs ti, tf;
    if (!split_tabs(c->logm, false, ti) || !split_tabs(c->logm, true, tf)) return RS_OK;
    const int is = ifft_slots(c->logm);
    const size_t ni = 2 * ti.lo.size() * kTwDwords16, nf = 2 * tf.lo.size() * kTwDwords16;
    std::vector<uint32_t> hi((size_t)c->nchunks * ni), hf(std::max<size_t>(nf, 1));
    for (int ch = 0; ch < c->nchunks; ch++) split_image(*c->F, ti, c->enc_ifft_logs.data() + (size_t)ch * is, hi.data() + ch * ni);
    split_image(*c->F, tf, c->enc_fft_logs.data(), hf.data());
    HIP_TRY(c->tws_ifft.ensure(hi.size()));
    HIP_TRY(c->tws_fft.ensure(hf.size()));
    HIP_TRY(hipMemcpy(c->tws_ifft.p, hi.data(), hi.size() * 4, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(c->tws_fft.p, hf.data(), hf.size() * 4, hipMemcpyHostToDevice));
    c->split_ok = true;
    return RS_OK;
}

// Test-only path overrides, set through rs_debug_set_path (include/rs_mi355x.h).
// The parity tests use them to run the kernel variants that other geometries
// select (the bit-sliced encode off, the transforms in full-field coordinates,
// the reconstruct FFT unpruned, the narrow / wide LDS units) on the same small
// inputs.  Process-wide; read when a codec is created (bs) or at each launch.
std::atomic<int> g_path_bs{1}, g_path_sub{1}, g_path_prune{1}, g_path_unit_width{-1}, g_path_hp_tiles{0}, g_path_hp_step{0},
    g_path_zc{3}, g_path_hp_tune{1}, g_path_rec_half{0}, g_path_dec_lab{0}, g_path_lds_big{1};
bool bs_enabled() { return g_path_bs.load(std::memory_order_relaxed) != 0; }
bool sub_enabled() { return g_path_sub.load(std::memory_order_relaxed) != 0; }
bool prune_enabled() { return g_path_prune.load(std::memory_order_relaxed) != 0; }
int zc_mask() { return g_path_zc.load(std::memory_order_relaxed); }
}  // namespace
int rs::unit_width_override() { return g_path_unit_width.load(std::memory_order_relaxed); }
int rs::hp_tiles_override() { return g_path_hp_tiles.load(std::memory_order_relaxed); }
int rs::hp_step_override() { return g_path_hp_step.load(std::memory_order_relaxed); }
bool rs::hp_tune_enabled() { return g_path_hp_tune.load(std::memory_order_relaxed) != 0; }
bool rs::rec_half_enabled() { return g_path_rec_half.load(std::memory_order_relaxed) != 0; }
namespace {

// One LDS-resident encode launch covers m <= 256 (both fields) and, for
// GF(2^16), m up to 4096 (64-byte tiles, half tiles at 2048, quarter tiles at
// 4096, kernels.hpp kMaxLdsEncLogM16);
// larger m runs the multi-pass kernels.
bool enc_lds_ok(const rs_codec *c) {
    return c->logm <= kMaxLdsLogN ||
           (c->bits == 16 && c->logm <= kMaxLdsEncLogM16 && g_path_lds_big.load(std::memory_order_relaxed));
}

// Host half of the encode plan (no device calls): twiddle schedule and panic check.
void plan_encode_host(rs_codec *c) {
    c->enc_ok = encode_schedule(*c->F, c->k, c->p, c->enc_ifft_logs, c->enc_fft_logs, c->nchunks);
    c->path = !c->enc_ok ? "panic" : (c->logm <= kMaxRegLogM ? encode_reg_name(c->bits, c->logm)
                                                   : enc_lds_ok(c) ? "lds-m" + std::to_string(c->m) : "multipass");
    if (c->enc_ok && c->bits == 16 && c->logm >= 2 && c->logm <= 5)
        c->path = std::string("split16-m") + std::to_string(c->m);
    c->bs_ok = c->enc_ok && c->bits == 16 && (c->logm == 4 || c->logm == 5) && bs_enabled() &&
               encode_bs_available(c->k, c->p, c->enc_ifft_logs.data(), c->enc_fft_logs.data(), c->F->mod);
    if (c->bs_ok) c->path = std::string("bs16-m") + std::to_string(c->m);
}

// Chunk IFFT passes of the LDS encode in subfield coordinates (EncodeArgs::
// tw_ifft_sub): chunk c's twiddles are fftSkew[(c+1)m - 1 + ...]
// (ifftDITEncoder leopard16.go:699-741), full-field in the first layers and
// in GF(2^8) after them (C5, m = 256: layers 0-1 of every chunk and layer 2
// of chunk 3 are full-field; m = 1024: layers 0-2, 0-3, 0-3, 0-4).  ifft_nff[c] = the first radix-4 pass from which
// every slot of the chunk lies in the subfield; the kernel needs the last
// pass subfield (it is fused with the accumulator).
int upload_ifft_sub(rs_codec *c) {
    const auto passes = ifft_passes(c->logm);
    const int np = (int)passes.size(), is = ifft_slots(c->logm);
    for (const PassInfo &ps : passes)
        if (ps.radix != 4) return RS_OK;
    std::vector<int> nff(c->nchunks, 1);
    std::vector<uint32_t> ts((size_t)c->nchunks * is * kTwDwords8, 0);
    for (int ch = 0; ch < c->nchunks; ch++) {
        const uint32_t *lg = c->enc_ifft_logs.data() + (size_t)ch * is;
        for (int p = 0; p < np; p++)
            for (int sl = passes[p].slot_off; sl < passes[p].slot_off + 3 * passes[p].groups; sl++)
                if (lg[sl] != c->F->mod && !in_subfield(*c->F, lg[sl])) nff[ch] = std::max(nff[ch], p + 1);
        // the kernel compiles nff = 1 and 2 (and 3 for m >= 1024); the last pass is subfield
        if (nff[ch] > (c->logm >= 10 ? 3 : 2) || nff[ch] >= np) return RS_OK;
        for (int sl = passes[nff[ch]].slot_off; sl < is; sl++)
            make_sub_twiddle(*c->F, lg[sl], ts.data() + ((size_t)ch * is + sl) * kTwDwords8);
    }
    HIP_TRY(c->tw_ifft_sub.ensure(ts.size()));
    HIP_TRY(c->ifft_nff.ensure(nff.size()));
    HIP_TRY(hipMemcpy(c->tw_ifft_sub.p, ts.data(), ts.size() * 4, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(c->ifft_nff.p, nff.data(), nff.size() * sizeof(int), hipMemcpyHostToDevice));
    c->ifft_sub = true;
    return RS_OK;
}

// Device half, on first use: stream, flag word, encode twiddle tables.
int ensure_device(rs_codec *c) {
    if (c->dev_ready) return RS_OK;
    if (!c->stream) HIP_TRY(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    if (!c->hflag) {
        HIP_TRY(hipHostMalloc((void **)&c->hflag, sizeof(int), hipHostMallocDefault));
        HIP_TRY(hipMalloc((void **)&c->dflag, sizeof(int)));
    }
    if (c->enc_ok) {
        int e = upload_twiddles(c, c->enc_ifft_logs, c->tw_ifft);
        if (e) return e;
        e = upload_twiddles(c, c->enc_fft_logs, c->tw_fft);
        if (e) return e;
        if (c->bits == 16) {
            e = upload_split(c);
            if (e) return e;
        }
        // m <= 256: every fftDIT twiddle is fftSkew[< 255], in GF(2^8); m = 1024:
        // the FFT's passes before big_sub_fft_end (the rest, layers 0-1, are
        // full-field and keep zero subfield tables; the kernel runs them full)
        bool sub = c->bits == 16 && c->logm > kMaxRegLogM && c->logm <= kMaxLdsEncLogM16 && c->logm % 2 == 0 &&
                   sub_enabled() && sub_coords().ok;
        size_t fsub_end = c->enc_fft_logs.size();  // slots [0, fsub_end) subfield
        if (sub && c->logm > kMaxLdsLogN) {
            const auto fp = fft_passes(c->logm);
            const int fend = big_sub_fft_end(c->logm);
            sub = (int)fp.size() > fend;
            if (sub) fsub_end = fp[fend].slot_off;
        }
        for (size_t i = 0; i < fsub_end && sub; i++) sub = in_subfield(*c->F, c->enc_fft_logs[i]);
        if (sub) {
            std::vector<uint32_t> hf(std::max<size_t>(c->enc_fft_logs.size(), 1) * kTwDwords8, 0), dm(kTwDwords8, 0);
            for (size_t i = 0; i < fsub_end; i++) make_sub_twiddle(*c->F, c->enc_fft_logs[i], hf.data() + i * kTwDwords8);
            make_sub_dmap(dm.data());
            HIP_TRY(c->tw_fft_sub.ensure(hf.size()));
            HIP_TRY(c->tw_dmap.ensure(dm.size()));
            HIP_TRY(hipMemcpy(c->tw_fft_sub.p, hf.data(), hf.size() * 4, hipMemcpyHostToDevice));
            HIP_TRY(hipMemcpy(c->tw_dmap.p, dm.data(), dm.size() * 4, hipMemcpyHostToDevice));
            c->fft_sub = true;
            if (int e2 = upload_ifft_sub(c)) return e2;
        }
    }
    c->dev_ready = true;
    return RS_OK;
}

// n = 512..2048 (GF(2^16)): the decoder layers with a full-field twiddle are
// 0 (n = 512), 0-1 (1024) and 0-2 (2048), fftSkew indices >= 255 everywhere
// else lying in GF(2^8) all the same; so the IFFT runs its passes from NI on
// (NI = 2 at n = 2048, else 1) and the FFT its first FEND = 4 passes in
// subfield coordinates (kernels.hip BigSub).  Checked against the
// schedule's own logs: a codec whose slots do not fit stays full-field.
int upload_big_sub(rs_codec *c, const std::vector<uint32_t> &il, const std::vector<uint32_t> &fl) {
    if (c->bits != 16 || c->logn < 9 || c->logn > kMaxLdsRecLogN16 || !sub_enabled() || !sub_coords().ok) return RS_OK;
    const int ni = big_sub_ifft_first(c->logn), fend = big_sub_fft_end(c->logn);
    const auto ip = ifft_passes(c->logn), fp = fft_passes(c->logn);
    auto range = [](const std::vector<PassInfo> &ps, int p, size_t total) {
        return std::make_pair((size_t)ps[p].slot_off, p + 1 < (int)ps.size() ? (size_t)ps[p + 1].slot_off : total);
    };
    if ((int)fp.size() <= fend || (int)ip.size() <= ni) return RS_OK;
    std::vector<uint32_t> hi(il.size() * kTwDwords8, 0), hf(fl.size() * kTwDwords8, 0), dm(kTwDwords8, 0);
    for (int p = ni; p < (int)ip.size(); p++) {
        const auto r = range(ip, p, il.size());
        for (size_t sl = r.first; sl < r.second; sl++) {
            if (!in_subfield(*c->F, il[sl])) return RS_OK;
            make_sub_twiddle(*c->F, il[sl], hi.data() + sl * kTwDwords8);
        }
    }
    for (int p = 0; p < fend; p++) {
        const auto r = range(fp, p, fl.size());
        for (size_t sl = r.first; sl < r.second; sl++) {
            if (!in_subfield(*c->F, fl[sl])) return RS_OK;
            make_sub_twiddle(*c->F, fl[sl], hf.data() + sl * kTwDwords8);
        }
    }
    make_sub_dmap(dm.data());
    HIP_TRY(c->dtw_ifft_sub.ensure(hi.size()));
    HIP_TRY(c->dtw_fft_sub.ensure(hf.size()));
    HIP_TRY(c->dec_dmap.ensure(dm.size()));
    HIP_TRY(hipMemcpy(c->dtw_ifft_sub.p, hi.data(), hi.size() * 4, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(c->dtw_fft_sub.p, hf.data(), hf.size() * 4, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(c->dec_dmap.p, dm.data(), dm.size() * 4, hipMemcpyHostToDevice));
    c->dec_big_sub = true;
    return RS_OK;
}

int build_decode_plan(rs_codec *c) {
    if (c->dec_built) return RS_OK;
    std::vector<uint32_t> il, fl;
    c->dec_ok = decode_schedule(*c->F, c->k, c->p, il, fl);
    c->dec_built = true;
    if (!c->dec_ok) return RS_OK;
    c->n = ceil_pow2(c->m + c->k);
    c->logn = ilog2(c->n);
    // n <= 256: every decoder twiddle is fftSkew[< 255], an element of GF(2^8)
    bool sub = c->bits == 16 && c->logn <= kMaxLdsLogN && sub_enabled() && sub_coords().ok;
    for (uint32_t l : il) sub = sub && in_subfield(*c->F, l);
    for (uint32_t l : fl) sub = sub && in_subfield(*c->F, l);
    if (sub) {
        std::vector<uint32_t> hi(std::max<size_t>(il.size(), 1) * kTwDwords8, 0), hf(std::max<size_t>(fl.size(), 1) * kTwDwords8, 0);
        for (size_t i = 0; i < il.size(); i++) make_sub_twiddle(*c->F, il[i], hi.data() + i * kTwDwords8);
        for (size_t i = 0; i < fl.size(); i++) make_sub_twiddle(*c->F, fl[i], hf.data() + i * kTwDwords8);
        HIP_TRY(c->dtw_ifft.ensure(hi.size()));
        HIP_TRY(c->dtw_fft.ensure(hf.size()));
        HIP_TRY(hipMemcpy(c->dtw_ifft.p, hi.data(), hi.size() * 4, hipMemcpyHostToDevice));
        HIP_TRY(hipMemcpy(c->dtw_fft.p, hf.data(), hf.size() * 4, hipMemcpyHostToDevice));
        c->dec_sub = true;
        return RS_OK;
    }
    int e = upload_twiddles(c, il, c->dtw_ifft);
    if (e) return e;
    e = upload_twiddles(c, fl, c->dtw_fft);
    if (e) return e;
    return upload_big_sub(c, il, fl);
}

// One LDS-resident reconstruct launch covers n <= 256 (both fields) and, for
// GF(2^16), n up to 8192 (64-byte tiles to 2048, half tiles at 4096, quarter
// tiles at 8192, kernels.hpp kMaxLdsRecLogN16); larger n runs the multi-pass kernels.
bool rec_lds_ok(const rs_codec *c) {
    return c->logn <= kMaxLdsLogN ||
           (c->bits == 16 && (c->logn <= 11 || (c->logn <= kMaxLdsRecLogN16 && g_path_lds_big.load(std::memory_order_relaxed))));
}

hipStream_t pick_stream(rs_codec *c, void *s) {
    return s == RS_NULL_STREAM ? (hipStream_t)0 : s ? (hipStream_t)s : c->stream;
}

// Order this call's stream behind the previous user of the codec scratch
// (nothing to do when that was this stream: it is in order already, and an
// explicit wait would stop the next launch from being queued behind the
// previous one).
int scratch_acquire(rs_codec *c, hipStream_t s) {
    if (c->scratch_used && s != c->scratch_stream)
        HIP_TRY(hipStreamWaitEvent(s, c->scratch_ev, 0));
    return RS_OK;
}
// Host wait for the previous user of the scratch (before a host-side write or a reallocation).
int scratch_host_wait(rs_codec *c) {
    if (c->scratch_used) HIP_TRY(hipEventSynchronize(c->scratch_ev));
    return RS_OK;
}
// Does an encode launch over these row sets touch the codec scratch (the
// device row table, the multi-pass work rows)?  Launches that do not skip the
// scratch event: one hipEventRecord less per call (the single-stripe
// device-resident encode is host-bound).
bool encode_uses_scratch(const rs_codec *c, const RowSet &data, const RowSet &par) {
    return data.table || par.table || !enc_lds_ok(c);
}
// Mark the scratch as used by the work queued on `s` so far.
int scratch_release(rs_codec *c, hipStream_t s) {
    if (!c->scratch_ev) HIP_TRY(hipEventCreateWithFlags(&c->scratch_ev, hipEventDisableTiming));
    HIP_TRY(hipEventRecord(c->scratch_ev, s));
    c->scratch_used = true;
    c->scratch_stream = s;
    return RS_OK;
}
// DevBuf::ensure for codec scratch: a reallocation frees a buffer that a
// kernel of an earlier call (on another stream) may still read.
template <class T>
int scratch_ensure(rs_codec *c, DevBuf<T> &b, size_t want) {
    if (want <= b.n) return RS_OK;
    if (int e = scratch_host_wait(c)) return e;
    HIP_TRY(b.ensure(want));
    return RS_OK;
}

// Data rows [0,k) and parity rows [k,k+p) as RowSets: strided when both sets'
// pointers are equally spaced (AllocAligned slab), else both via a device
// table (one strided set and one table would reach a kernel whose ROWTAB
// parameter covers both: a null table dereference).
int make_rowsets(rs_codec *c, uint8_t *const *d, hipStream_t s, RowSet &data, RowSet &par) {
    auto strided = [&](int lo, int cnt, RowSet &rs) {
        if (cnt == 1) { rs = RowSet{nullptr, d[lo], 0}; return true; }
        const int64_t st = (int64_t)(d[lo + 1] - d[lo]);
        if (st <= 0) return false;
        for (int i = lo + 2; i < lo + cnt; i++)
            if ((int64_t)(d[i] - d[i - 1]) != st) return false;
        rs = RowSet{nullptr, d[lo], (uint64_t)st};
        return true;
    };
    bool ok_d = strided(0, c->k, data), ok_p = strided(c->k, c->p, par);
    if (ok_d && ok_p) return RS_OK;
    std::vector<uint8_t *> tbl(d, d + c->total);
    if (tbl != c->rows_host || c->rows.n < (size_t)c->total) {
        // previous users of the table are done: this call's stream and the last
        // scratch user (a device-resident encode may still run on another stream)
        HIP_TRY(hipStreamSynchronize(s));
        if (int e = scratch_host_wait(c)) return e;
        if (int e = scratch_ensure(c, c->rows, c->total)) return e;
        HIP_TRY(hipMemcpy(c->rows.p, tbl.data(), c->total * sizeof(uint8_t *), hipMemcpyHostToDevice));
        c->rows_host = tbl;
    }
    // both sets from the table: the kernels take one layout (template ROWTAB)
    // for data and parity rows alike
    data = RowSet{c->rows.p, nullptr, 0};
    par = RowSet{c->rows.p + c->k, nullptr, 0};
    return RS_OK;
}

// Multi-pass transform over `rows` rows of `work` (m or n rows).
int run_passes(rs_codec *c, bool inverse, uint8_t *work, uint64_t S, int logsz, int mtrunc, const uint32_t *tw,
               hipStream_t s) {
    const auto passes = inverse ? ifft_passes(logsz) : fft_passes(logsz);
    for (const PassInfo &ps : passes) {
        int active;
        if (ps.radix == 4) active = std::min(ps.groups, (mtrunc + 4 * ps.dist - 1) / (4 * ps.dist));
        else active = inverse ? 1 : std::min(ps.groups, (mtrunc + 1) / 2);
        HIP_TRY(launch_pass(c->bits, inverse, work, S, ps.dist, ps.radix, active, tw + (size_t)ps.slot_off * c->twd, s));
    }
    return RS_OK;
}

int encode_multipass(rs_codec *c, RowSet data, RowSet par, uint64_t S, int *mismatch, hipStream_t s) {
    const int m = c->m;
    if (int e = scratch_ensure(c, c->work, (size_t)2 * m * S)) return e;
    uint8_t *acc = c->work.p, *tmp = c->work.p + (size_t)m * S;
    const int is = ifft_slots(c->logm);
    for (int ch = 0; ch < c->nchunks; ch++) {
        uint8_t *dst = ch == 0 ? acc : tmp;
        const int cnt = std::min(m, c->k - ch * m);
        HIP_TRY(launch_gather(c->bits, dst, S, data, ch * m, cnt, m, s));
        int e = run_passes(c, true, dst, S, c->logm, cnt, c->tw_ifft.p + (size_t)ch * is * c->twd, s);
        if (e) return e;
        if (ch > 0) HIP_TRY(launch_xor_rows(c->bits, acc, tmp, S, m, s));
    }
    int e = run_passes(c, false, acc, S, c->logm, c->p, c->tw_fft.p, s);
    if (e) return e;
    HIP_TRY(launch_copy_out(c->bits, par, acc, S, c->p, mismatch, s));
    return RS_OK;
}

int encode_device(rs_codec *c, RowSet data, RowSet par, uint64_t S, uint64_t stripe_stride, int nstripes,
                  int *mismatch, hipStream_t s) {
    if (!c->enc_ok) return RS_ERR_PANIC;
    if (c->logm <= kMaxRegLogM) {
        EncodeArgs a{};
        a.data = data;
        a.parity = par;
        a.k = c->k;
        a.p = c->p;
        a.nchunks = c->nchunks;
        a.shard_size = S;
        a.stripe_stride = stripe_stride;
        a.nstripes = nstripes;
        a.tw_ifft = c->tw_ifft.p;
        a.tw_fft = c->tw_fft.p;
        a.mismatch = mismatch;
        // bit-sliced kernel: strided rows, one row stride for data and parity
        const uint64_t span = (uint64_t)(c->k - 1) * data.stride + S;
        if (c->bs_ok && !data.table && !par.table && data.stride == par.stride && data.stride >= S &&
            encode_bs_fits(c->k, c->p, data.stride, S)) {
            BsArgs b{};
            b.data = data.base;
            b.parity = par.base;
            b.row_stride = data.stride;
            b.stripe_stride = stripe_stride;
            b.S = S;
            b.k = c->k;
            b.p = c->p;
            b.nstripes = nstripes;
            b.mismatch = mismatch;
            if (!c->cus) HIP_TRY(hipDeviceGetAttribute(&c->cus, hipDeviceAttributeMultiprocessorCount, c->device));
            HIP_TRY(launch_encode_bs(mismatch != nullptr, b, c->cus, s));
            return RS_OK;
        }
        // split kernel: strided rows whose data span fits a 32-bit buffer offset
        if (c->split_ok && !data.table && !par.table && span < (1ull << 32)) {
            a.tw_ifft = c->tws_ifft.p;
            a.tw_fft = c->tws_fft.p;
            HIP_TRY(launch_encode_split(c->logm, mismatch != nullptr, a, s));
            return RS_OK;
        }
        HIP_TRY(launch_encode_reg(c->bits, c->logm, mismatch != nullptr, a, s));
        return RS_OK;
    }
    if (enc_lds_ok(c)) {  // m rows of accumulator + chunk LDS-resident
        EncodeArgs a{};
        a.data = data;
        a.parity = par;
        a.k = c->k;
        a.p = c->p;
        a.nchunks = c->nchunks;
        a.shard_size = S;
        a.stripe_stride = (data.table || par.table) ? 0 : stripe_stride;
        a.nstripes = (data.table || par.table) ? 1 : nstripes;
        a.tw_ifft = c->tw_ifft.p;
        a.tw_fft = c->tw_fft.p;
        if (c->fft_sub) {
            a.tw_fft_sub = c->tw_fft_sub.p;
            a.tw_dmap = c->tw_dmap.p;
            if (c->ifft_sub) {
                a.tw_ifft_sub = c->tw_ifft_sub.p;
                a.ifft_nff = c->ifft_nff.p;
            }
        }
        a.mismatch = mismatch;
        HIP_TRY(launch_encode_lds(c->bits, c->logm, mismatch != nullptr, a, s));
        return RS_OK;
    }
    for (int j = 0; j < nstripes; j++) {
        RowSet d = data, p = par;
        if (!d.table) d.base += (size_t)j * stripe_stride;
        if (!p.table) p.base += (size_t)j * stripe_stride;
        int e = encode_multipass(c, d, p, S, mismatch, s);
        if (e) return e;
    }
    return RS_OK;
}

// errLocs for an erasure pattern (cached: analog of leopard8.go:508-555, but
// keyed by the full pattern so a hit is always exact).
const std::vector<uint32_t> *error_locs_cached(rs_codec *c, const std::vector<uint8_t> &erased) {
    for (auto it = c->el_cache.begin(); it != c->el_cache.end(); ++it) {
        if (it->first == erased) {
            c->el_cache.splice(c->el_cache.begin(), c->el_cache, it);
            return &c->el_cache.front().second;
        }
    }
    std::vector<uint32_t> el;
    if (!error_locators(*c->F, c->k, c->p, erased.data(), el)) return nullptr;
    c->el_cache.emplace_front(erased, std::move(el));
    if (c->el_cache.size() > 64) c->el_cache.pop_back();
    return &c->el_cache.front().second;
}


// The reference-keyed GF(2^8) inversion cache (rs_set_reference_inversion_cache).
// leopard8.go:481-506 builds the error bitfield: parity erasures (and the
// padding rows p..m-1) only when recoverAll, data erasure i at bit i + m; the
// lookup (:509-524) uses those raw bits, a miss stores its errLocs (:542-554)
// under the bits after prepare() when useBits (:474), whose first level pairs
// bits 2i and 2i+1 (:1192-1199).  A hit hands back errLocs computed for
// whatever pattern stored them, which is the reference's output on that call.
// Pruning from a hit's stored bits covers every row the call rebuilds, so
// only errLocs decides the result.  Returns nullptr when the mode is off or
// the reference keeps no cache for this codec (GF(2^16), or total > 64: :67-71).
const std::vector<uint32_t> *ref_inv_errlocs(rs_codec *c, const std::vector<uint8_t> &present, bool recover_all,
                                             uint64_t S) {
    if (!c->ref_inv || c->bits != 8 || c->total > 64) return nullptr;
    const int k = c->k, p = c->p, m = c->m, total = c->total;
    std::array<uint64_t, 4> w{};
    auto set = [&](int b) { w[b >> 6] |= 1ull << (b & 63); };
    int npresent = 0;
    for (int i = 0; i < total; i++) npresent += present[i] ? 1 : 0;
    for (int i = 0; i < p; i++)
        if (!present[k + i] && recover_all) set(i);
    for (int i = p; i < m; i++)
        if (recover_all) set(i);
    for (int i = 0; i < k; i++)
        if (!present[i]) set(i + m);
    auto it = c->ref_inv_cache.find(w);
    if (it != c->ref_inv_cache.end()) return &it->second;
    std::vector<uint8_t> erased(total);
    for (int i = 0; i < total; i++) erased[i] = !present[i];
    std::vector<uint32_t> el;
    if (!error_locators(*c->F, k, p, erased.data(), el)) return nullptr;
    const bool use_bits = total - npresent <= p / 4 && S * (uint64_t)total >= (64u << 10);
    if (use_bits)
        for (uint64_t &x : w) x |= ((x & 0xAAAAAAAAAAAAAAAAull) >> 1) | ((x & 0x5555555555555555ull) << 1);
    auto &slot = c->ref_inv_cache[w];
    slot = std::move(el);
    return &slot;
}

int plan_reconstruct_new(rs_codec *c, const std::vector<uint8_t> &present, bool recover_all,
                         const std::vector<uint32_t> *el_ref, RecPlan &pl, const std::vector<uint32_t> *el_exact);

// Plan-cache key: (erasure pattern, recover_all), plus the errLocs a
// reference-keyed cache handed out, which can differ between calls with the
// same pattern.
std::vector<uint8_t> plan_key(const std::vector<uint8_t> &present, bool recover_all, const std::vector<uint32_t> *el_ref) {
    std::vector<uint8_t> key(present);
    key.push_back(recover_all ? 1 : 0);
    if (el_ref) {
        const uint8_t *b = (const uint8_t *)el_ref->data();
        key.insert(key.end(), b, b + el_ref->size() * sizeof(uint32_t));
    }
    return key;
}

// Plans are cached per (erasure pattern, recover_all): repeated repairs of
// the same pattern skip the table construction.  `el_ref` is the call's one
// reference-keyed cache answer (ref_inv_errlocs), looked up by the caller
// exactly once per reconstruct, as leopard8.go:509-554 looks up and stores once.
int plan_reconstruct_el(rs_codec *c, const std::vector<uint8_t> &present, bool recover_all,
                        const std::vector<uint32_t> *el_ref, RecPlan &pl, const std::vector<uint32_t> *el_exact = nullptr) {
    std::vector<uint8_t> key = plan_key(present, recover_all, el_ref);
    for (auto it = c->plan_cache.begin(); it != c->plan_cache.end(); ++it) {
        if (it->first == key) {
            c->plan_cache.splice(c->plan_cache.begin(), c->plan_cache, it);
            pl = c->plan_cache.front().second;
            return RS_OK;
        }
    }
    int e = plan_reconstruct_new(c, present, recover_all, el_ref, pl, el_exact);
    if (e) return e;
    c->plan_cache.emplace_front(std::move(key), pl);
    if (c->plan_cache.size() > 16) c->plan_cache.pop_back();
    return RS_OK;
}
// el_ext: locators handed in by a multi-device parent (computed once for all
// its parts) instead of this codec's own caches.
int plan_reconstruct(rs_codec *c, const std::vector<uint8_t> &present, bool recover_all, uint64_t S, RecPlan &pl,
                     const ElExt *el_ext = nullptr) {
    if (el_ext)
        return plan_reconstruct_el(c, present, recover_all, el_ext->ref ? el_ext->el : nullptr, pl,
                                   el_ext->ref ? nullptr : el_ext->el);
    return plan_reconstruct_el(c, present, recover_all, ref_inv_errlocs(c, present, recover_all, S), pl);
}

int plan_reconstruct_new(rs_codec *c, const std::vector<uint8_t> &present, bool recover_all,
                         const std::vector<uint32_t> *el_ref, RecPlan &pl, const std::vector<uint32_t> *el_exact) {
    int e = build_decode_plan(c);
    if (e) return e;
    if (!c->dec_ok) return RS_ERR_PANIC;
    const int k = c->k, p = c->p, m = c->m, n = c->n, total = c->total;
    std::vector<uint8_t> erased(total);
    for (int i = 0; i < total; i++) erased[i] = !present[i];
    const std::vector<uint32_t> *elp = el_ref ? el_ref : el_exact ? el_exact : error_locs_cached(c, erased);
    if (!elp) return RS_ERR_PANIC;
    const std::vector<uint32_t> &el = *elp;
    // work rows: [recovery m][original k][zero to n] (leopard16.go:547)
    pl.src_shard.assign(n, -1);
    for (int i = 0; i < p; i++)
        if (present[k + i]) pl.src_shard[i] = k + i;
    for (int i = 0; i < k; i++)
        if (present[i]) pl.src_shard[m + i] = i;
    pl.tw_in.assign((size_t)n * c->twd, 0);
    const Field &F = *c->F;
    const SubCoords &sc = sub_coords();
    for (int r = 0; r < m + k; r++) {
        if (pl.src_shard[r] < 0) continue;
        if (c->dec_sub)  // x -> subfield coordinates of x * errLocs[r]
            make_linear_image([&](uint32_t x) { return sc.to_sub(F.mul_log(x, el[r])); }, pl.tw_in.data() + (size_t)r * c->twd);
        else
            make_twiddle(F, el[r], pl.tw_in.data() + (size_t)r * c->twd);
    }
    pl.dst_shard.clear();
    pl.pos.clear();
    const int end = recover_all ? total : k;
    for (int i = 0; i < end; i++) {
        if (present[i]) continue;
        pl.dst_shard.push_back(i);
        pl.pos.push_back(i >= k ? i - k : i + m);
    }
    pl.tw_out.assign(std::max<size_t>(pl.dst_shard.size(), 1) * c->twd, 0);
    for (size_t j = 0; j < pl.dst_shard.size(); j++) {
        const uint32_t lg = (F.mod - el[pl.pos[j]]) & F.mod;
        if (c->dec_sub)  // subfield coordinates y -> symbol(y) * exp(lg)
            make_linear_image([&](uint32_t y) { return F.mul_log(sc.to_sub(y), lg); }, pl.tw_out.data() + j * c->twd);
        else
            make_twiddle(F, lg, pl.tw_out.data() + j * c->twd);
    }
    return RS_OK;
}

// Upload a plan for `nsets` row-pointer sets (set b: shard i at d[b][i]) as
// one packed blob: row pointers, scale tables, rebuilt-row positions.  The
// pinned staging buffer is reused by the next call; every caller synchronizes
// its stream before returning (calls are serialized by the codec mutex).
int upload_reconstruct(rs_codec *c, const RecPlan &pl, const std::vector<uint8_t *const *> &d, hipStream_t s) {
    const int n = c->n, nd = (int)pl.dst_shard.size(), ns = (int)d.size(), ndd = std::max(nd, 1);
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    const size_t s_src = (size_t)ns * n * sizeof(void *), s_dst = (size_t)ns * ndd * sizeof(void *);
    const size_t s_in = pl.tw_in.size() * 4, s_out = pl.tw_out.size() * 4, s_pos = std::max<size_t>(pl.pos.size(), 1) * 4;
    const size_t o_dst = al(s_src), o_in = o_dst + al(s_dst), o_out = o_in + al(s_in), o_pos = o_out + al(s_out);
    const size_t total = o_pos + al(s_pos);
    if (int e = scratch_ensure(c, c->rc_blob, total)) return e;
    if (c->rc_host_n < total) {
        if (c->rc_host) HIP_TRY(hipHostFree(c->rc_host));
        c->rc_host = nullptr;
        c->rc_host_n = 0;
        HIP_TRY(hipHostMalloc((void **)&c->rc_host, total, hipHostMallocDefault));
        c->rc_host_n = total;
    }
    uint8_t *h = c->rc_host;
    const uint8_t **src = (const uint8_t **)h;
    uint8_t **dst = (uint8_t **)(h + o_dst);
    for (int b = 0; b < ns; b++) {
        for (int r = 0; r < n; r++) src[(size_t)b * n + r] = pl.src_shard[r] >= 0 ? d[b][pl.src_shard[r]] : nullptr;
        for (int j = 0; j < ndd; j++) dst[(size_t)b * ndd + j] = j < nd ? d[b][pl.dst_shard[j]] : nullptr;
    }
    std::memcpy(h + o_in, pl.tw_in.data(), s_in);
    std::memcpy(h + o_out, pl.tw_out.data(), s_out);
    if (!pl.pos.empty()) std::memcpy(h + o_pos, pl.pos.data(), pl.pos.size() * 4);
    HIP_TRY(hipMemcpyAsync(c->rc_blob.p, h, total, hipMemcpyHostToDevice, s));
    uint8_t *g = c->rc_blob.p;
    c->rc_src = (const uint8_t **)g;
    c->rc_dst = (uint8_t **)(g + o_dst);
    c->rc_tw_in = (uint32_t *)(g + o_in);
    c->rc_tw_out = (uint32_t *)(g + o_out);
    c->rc_pos = (int *)(g + o_pos);
    return RS_OK;
}

// Device work of one reconstruct over row-pointer set `set` of the uploaded plan.
int launch_reconstruct(rs_codec *c, const RecPlan &pl, int set, uint64_t S, hipStream_t s) {
    const int n = c->n, nd = (int)pl.dst_shard.size();
    if (c->logn <= kMaxLdsLogN) {  // whole transform LDS-resident: one HBM read/write per row
        if (!nd) return RS_OK;
        RecArgs ra{};
        ra.src = c->rc_src + (size_t)set * n;
        ra.dst = c->rc_dst + (size_t)set * nd;
        ra.pos = c->rc_pos;
        ra.tw_in = c->rc_tw_in;
        ra.tw_out = c->rc_tw_out;
        ra.tw_ifft = c->dtw_ifft.p;
        ra.tw_fft = c->dtw_fft.p;
        ra.S = S;
        ra.mtrunc = c->m + c->k;
        ra.m = c->m;
        ra.nd = nd;
        ra.prune = prune_enabled() ? 1 : 0;
    ra.lab = g_path_dec_lab.load(std::memory_order_relaxed);
        for (int p : pl.pos) ra.need[p >> 5] |= 1u << (p & 31);
        HIP_TRY(launch_rec_lds(c->bits, c->logn, c->dec_sub, ra, s));
        return RS_OK;
    }
    if (int e = scratch_ensure(c, c->work, (size_t)n * S)) return e;
    uint8_t *w = c->work.p;
    HIP_TRY(launch_scale_in(c->bits, w, S, c->rc_src + (size_t)set * n, c->rc_tw_in, n, s));
    int e = run_passes(c, true, w, S, c->logn, c->m + c->k, c->dtw_ifft.p, s);
    if (e) return e;
    HIP_TRY(launch_formal_derivative(c->bits, w, S, n, s));
    e = run_passes(c, false, w, S, c->logn, c->m + c->k, c->dtw_fft.p, s);
    if (e) return e;
    if (nd) HIP_TRY(launch_reveal(c->bits, c->rc_dst + (size_t)set * nd, w, S, c->rc_pos, c->rc_tw_out, nd, s));
    return RS_OK;
}

void set_big_sub(const rs_codec *c, RecArgs &ra) {
    if (!c->dec_big_sub) return;
    ra.tw_ifft_sub = c->dtw_ifft_sub.p;
    ra.tw_fft_sub = c->dtw_fft_sub.p;
    ra.tw_dmap = c->dec_dmap.p;
}

// Device-resident plan for (present, recover_all), built and uploaded on first use.
int dev_plan(rs_codec *c, const std::vector<uint8_t> &present, bool recover_all, uint64_t S, DevPlan **out,
             const ElExt *el_ext = nullptr) {
    const std::vector<uint32_t> *el_ref =
        el_ext ? (el_ext->ref ? el_ext->el : nullptr) : ref_inv_errlocs(c, present, recover_all, S);
    const std::vector<uint32_t> *el_exact = el_ext && !el_ext->ref ? el_ext->el : nullptr;
    std::vector<uint8_t> key = plan_key(present, recover_all, el_ref);
    for (auto it = c->dplan_cache.begin(); it != c->dplan_cache.end(); ++it) {
        if (it->first == key) {
            c->dplan_cache.splice(c->dplan_cache.begin(), c->dplan_cache, it);
            *out = c->dplan_cache.front().second.get();
            return RS_OK;
        }
    }
    auto dp = std::make_unique<DevPlan>();
    if (int e = plan_reconstruct_el(c, present, recover_all, el_ref, dp->pl, el_exact)) return e;
    const RecPlan &pl = dp->pl;
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    const size_t s_in = pl.tw_in.size() * 4, s_out = pl.tw_out.size() * 4, s_pos = std::max<size_t>(pl.pos.size(), 1) * 4;
    const size_t s_si = pl.src_shard.size() * 4, s_di = std::max<size_t>(pl.dst_shard.size(), 1) * 4;
    const size_t s_nw = (size_t)std::max(c->n / 32, 1) * 4, s_rev = (size_t)c->n * 4;
    const size_t o_out = al(s_in), o_pos = o_out + al(s_out), o_si = o_pos + al(s_pos), o_di = o_si + al(s_si);
    const size_t o_nw = o_di + al(s_di), o_rev = o_nw + al(s_nw);
    const size_t total = o_rev + al(s_rev);
    std::vector<uint8_t> h(total, 0);
    {
        uint32_t *nw = (uint32_t *)(h.data() + o_nw);
        int *rev = (int *)(h.data() + o_rev);
        for (int r = 0; r < c->n; r++) rev[r] = -1;
        for (size_t j = 0; j < pl.pos.size(); j++) {
            nw[pl.pos[j] >> 5] |= 1u << (pl.pos[j] & 31);
            rev[pl.pos[j]] = (int)j;
        }
    }
    std::memcpy(h.data(), pl.tw_in.data(), s_in);
    std::memcpy(h.data() + o_out, pl.tw_out.data(), s_out);
    if (!pl.pos.empty()) std::memcpy(h.data() + o_pos, pl.pos.data(), pl.pos.size() * 4);
    std::memcpy(h.data() + o_si, pl.src_shard.data(), s_si);
    if (!pl.dst_shard.empty()) std::memcpy(h.data() + o_di, pl.dst_shard.data(), pl.dst_shard.size() * 4);
    HIP_TRY(dp->blob.ensure(total));
    HIP_TRY(hipMemcpy(dp->blob.p, h.data(), total, hipMemcpyHostToDevice));
    dp->tw_in = (const uint32_t *)dp->blob.p;
    dp->tw_out = (const uint32_t *)(dp->blob.p + o_out);
    dp->pos = (const int *)(dp->blob.p + o_pos);
    dp->src_idx = (const int *)(dp->blob.p + o_si);
    dp->dst_idx = (const int *)(dp->blob.p + o_di);
    dp->need_w = (const uint32_t *)(dp->blob.p + o_nw);
    dp->rev = (const int *)(dp->blob.p + o_rev);
    for (int p : pl.pos)
        if (p < 256) dp->need[p >> 5] |= 1u << (p & 31);
    c->dplan_cache.emplace_front(std::move(key), std::move(dp));
    if (c->dplan_cache.size() > 16) c->dplan_cache.pop_back();  // waits for the plan's last launch
    *out = c->dplan_cache.front().second.get();
    return RS_OK;
}

// One launch of the LDS-resident reconstruct (rec_lds_ok) with a cached device plan over
// strided shards (shard i of stripe y at base + y * stripe_stride + i * stride).
int launch_rec_plan(rs_codec *c, DevPlan *dpl, uint8_t *base, uint64_t stride, uint64_t stripe_stride, int nstripes,
                    uint64_t S, hipStream_t s) {
    const int nd = (int)dpl->pl.dst_shard.size();
    if (!nd) return RS_OK;
    RecArgs ra{};
    ra.pos = dpl->pos;
    ra.tw_in = dpl->tw_in;
    ra.tw_out = dpl->tw_out;
    ra.tw_ifft = c->dtw_ifft.p;
    ra.tw_fft = c->dtw_fft.p;
    ra.S = S;
    ra.mtrunc = c->m + c->k;
    ra.m = c->m;
    ra.nd = nd;
    ra.prune = prune_enabled() ? 1 : 0;
    ra.lab = g_path_dec_lab.load(std::memory_order_relaxed);
    std::memcpy(ra.need, dpl->need, sizeof(ra.need));
    ra.need_w = dpl->need_w;
    ra.rev = dpl->rev;
    set_big_sub(c, ra);
    ra.base = base;
    ra.stride = stride;
    ra.stripe_stride = stripe_stride;
    ra.nstripes = nstripes;
    ra.src_idx = dpl->src_idx;
    ra.dst_idx = dpl->dst_idx;
    HIP_TRY(launch_rec_lds(c->bits, c->logn, c->dec_sub, ra, s));
    HIP_TRY(dpl->mark_used(s));
    return RS_OK;
}

// rs_reconstruct_dev with rec_lds_ok (one LDS-resident launch): the plan's tables
// stay in HBM; equally strided shards (an AllocAligned slab, a torch 2-D
// tensor) go to the kernel as base + stride, other layouts' row pointers
// through a ring slot; nothing waits for the kernel -- the call is
// stream-ordered like the device encodes.
int reconstruct_device_lds(rs_codec *c, uint8_t *const *d, const std::vector<uint8_t> &present, uint64_t S,
                           bool recover_all, hipStream_t s) {
    DevPlan *dp = nullptr;
    if (int e = dev_plan(c, present, recover_all, S, &dp)) return e;
    const RecPlan &pl = dp->pl;
    const int n = c->n, nd = (int)pl.dst_shard.size();
    if (!nd) return RS_OK;
    RecArgs ra{};
    ra.pos = dp->pos;
    ra.tw_in = dp->tw_in;
    ra.tw_out = dp->tw_out;
    ra.tw_ifft = c->dtw_ifft.p;
    ra.tw_fft = c->dtw_fft.p;
    ra.S = S;
    ra.mtrunc = c->m + c->k;
    ra.m = c->m;
    ra.nd = nd;
    ra.prune = prune_enabled() ? 1 : 0;
    ra.lab = g_path_dec_lab.load(std::memory_order_relaxed);
    std::memcpy(ra.need, dp->need, sizeof(ra.need));
    ra.need_w = dp->need_w;
    ra.rev = dp->rev;
    set_big_sub(c, ra);
    {
        // strided: every shard the launch touches at d[0] + i * stride
        int i0 = -1, i1 = -1;
        for (int i = 0; i < c->total && i1 < 0; i++)
            if (d[i]) (i0 < 0 ? i0 : i1) = i;
        bool strided = i0 >= 0 && i1 >= 0 && d[i1] > d[i0] && (uint64_t)(d[i1] - d[i0]) % (uint64_t)(i1 - i0) == 0;
        const uint64_t stride = strided ? (uint64_t)(d[i1] - d[i0]) / (uint64_t)(i1 - i0) : 0;
        uint8_t *base = strided ? d[i0] - (uint64_t)i0 * stride : nullptr;
        strided = strided && stride >= S;
        for (int i = 0; i < c->total && strided; i++)
            if (d[i] && d[i] != base + (uint64_t)i * stride) strided = false;
        for (int r = 0; r < n && strided; r++)
            if (pl.src_shard[r] >= 0 && !d[pl.src_shard[r]]) strided = false;
        for (int j = 0; j < nd && strided; j++)
            if (!d[pl.dst_shard[j]]) strided = false;
        if (strided) {
            ra.base = base;
            ra.stride = stride;
            ra.src_idx = dp->src_idx;
            ra.dst_idx = dp->dst_idx;
            HIP_TRY(launch_rec_lds(c->bits, c->logn, c->dec_sub, ra, s));
            HIP_TRY(dp->mark_used(s));
            return RS_OK;
        }
    }
    const size_t bytes = ((size_t)(n + nd) * sizeof(void *) + 255) & ~(size_t)255;
    if (c->ring_slot < bytes) {
        for (int i = 0; i < rs_codec::kRing; i++)
            if (c->ring_used[i]) HIP_TRY(hipEventSynchronize(c->ring_ev[i]));
        if (c->ring_host) HIP_TRY(hipHostFree(c->ring_host));
        c->ring_host = nullptr;
        c->ring_slot = 0;
        HIP_TRY(c->ring_dev.ensure(bytes * rs_codec::kRing));
        HIP_TRY(hipHostMalloc((void **)&c->ring_host, bytes * rs_codec::kRing, hipHostMallocDefault));
        c->ring_slot = bytes;
    }
    const int i = c->ring_next;
    c->ring_next = (i + 1) % rs_codec::kRing;
    if (!c->ring_ev[i]) HIP_TRY(hipEventCreateWithFlags(&c->ring_ev[i], hipEventDisableTiming));
    if (c->ring_used[i]) HIP_TRY(hipEventSynchronize(c->ring_ev[i]));  // its copy and kernel are done
    uint8_t *h = c->ring_host + (size_t)i * c->ring_slot;
    uint8_t *g = c->ring_dev.p + (size_t)i * c->ring_slot;
    const uint8_t **src = (const uint8_t **)h;
    uint8_t **dst = (uint8_t **)h + n;
    for (int r = 0; r < n; r++) src[r] = pl.src_shard[r] >= 0 ? d[pl.src_shard[r]] : nullptr;
    for (int j = 0; j < nd; j++) dst[j] = d[pl.dst_shard[j]];
    HIP_TRY(hipMemcpyAsync(g, h, (size_t)(n + nd) * sizeof(void *), hipMemcpyHostToDevice, s));
    ra.src = (const uint8_t *const *)g;
    ra.dst = (uint8_t *const *)g + n;
    HIP_TRY(launch_rec_lds(c->bits, c->logn, c->dec_sub, ra, s));
    HIP_TRY(hipEventRecord(c->ring_ev[i], s));
    c->ring_used[i] = true;
    HIP_TRY(dp->mark_used(s));
    return RS_OK;
}

// Device reconstruct (leopard16.go:432-568) for already-validated input.
int reconstruct_device(rs_codec *c, uint8_t *const *d, const std::vector<uint8_t> &present, uint64_t S,
                       bool recover_all, hipStream_t s) {
    RecPlan pl;
    int e = plan_reconstruct(c, present, recover_all, S, pl);
    if (e) return e;
    e = scratch_acquire(c, s);
    if (e) return e;
    e = upload_reconstruct(c, pl, {d}, s);
    if (e) return e;
    e = launch_reconstruct(c, pl, 0, S, s);
    if (e) return e;
    e = scratch_release(c, s);
    if (e) return e;
    HIP_TRY(hipStreamSynchronize(s));  // the pinned staging of the upload is reused by the next call
    return RS_OK;
}

// checkShards / shardSize (encoder.go:102-126)
size_t shard_size_of(const size_t *lens, int n) {
    for (int i = 0; i < n; i++)
        if (lens[i]) return lens[i];
    return 0;
}
int check_shards(const size_t *lens, int n, bool nilok) {
    const size_t size = shard_size_of(lens, n);
    if (size == 0) return RS_ERR_SHARD_NO_DATA;
    for (int i = 0; i < n; i++)
        if (lens[i] != size && (lens[i] != 0 || !nilok)) return RS_ERR_SHARD_SIZE;
    return RS_OK;
}

// ---------------------------------------------------------------- host-resident pipeline
// Shards in host memory (the reference's own setting: Encode on [][]byte).
// The stripe is cut into column segments (every operation is column-local,
// leopard16.go:778-792); segment j is copied in on s_in, transformed on the
// codec stream and copied out on s_out, through staging slab j % kHostBufs,
// so PCIe copies in both directions overlap the kernels.

int ensure_host_pipe(rs_codec *c) {
    if (!c->s_in) HIP_TRY(hipStreamCreateWithFlags(&c->s_in, hipStreamNonBlocking));
    if (!c->s_out) HIP_TRY(hipStreamCreateWithFlags(&c->s_out, hipStreamNonBlocking));
    for (int b = 0; b < kHostBufs; b++) {
        if (!c->ev_in[b]) HIP_TRY(hipEventCreateWithFlags(&c->ev_in[b], hipEventDisableTiming));
        if (!c->ev_k[b]) HIP_TRY(hipEventCreateWithFlags(&c->ev_k[b], hipEventDisableTiming));
        if (!c->ev_free[b]) HIP_TRY(hipEventCreateWithFlags(&c->ev_free[b], hipEventDisableTiming));
    }
    return RS_OK;
}

uint64_t host_segment(const rs_codec *c, uint64_t S, size_t in_rows) {
    uint64_t seg = c->host_seg_bytes ? c->host_seg_bytes : kHostSegTarget / std::max<size_t>(in_rows, 1);
    seg = std::max<uint64_t>(seg / 64 * 64, 64);
    return std::min(seg, S);
}

// Copy bytes [off, off+w) of shards `rows` between host rows and a device slab
// (shard i at dev + i*dpitch).  Runs of consecutive shards whose host rows are
// equally spaced (an AllocAligned slab) go as one 2-D copy.  bridge (host to
// device only): a run also spans gaps of up to kBridgeRows shards that are not
// in `rows` but whose host rows exist on the same pitch (a reconstruct's
// missing shards that keep their memory, Go's shards[i][:0]); their bytes land
// in staging rows the kernel never reads, and each bridged gap saves a copy
// (each costs ~10-15 us in the pipeline against ~5 us to move a 256 KiB row).
constexpr int kBridgeRows = 3;
int copy_rows(uint8_t *dev, uint64_t dpitch, uint8_t *const *host, const std::vector<int> &rows, uint64_t off,
              uint64_t w, bool h2d, hipStream_t s, bool bridge = false) {
    size_t i = 0;
    while (i < rows.size()) {
        size_t j = i + 1;
        int64_t hp = 0;
        auto on_pitch = [&](int r0, int r1) {  // rows r0 < r1: every host row r0..r1 present and on pitch hp
            for (int r = r0 + 1; r <= r1; r++)
                if (!host[r] || (int64_t)(host[r] - host[r - 1]) != hp) return false;
            return true;
        };
        if (j < rows.size()) {
            const int gap = rows[j] - rows[i];
            if (gap == 1 || (bridge && gap <= kBridgeRows + 1)) {
                hp = (int64_t)(host[rows[i] + 1] ? host[rows[i] + 1] - host[rows[i]] : 0);
                if (hp >= (int64_t)w && on_pitch(rows[i], rows[j])) {
                    while (j < rows.size()) {
                        const int g = rows[j] - rows[j - 1];
                        if (!(g == 1 || (bridge && g <= kBridgeRows + 1)) || !on_pitch(rows[j - 1], rows[j])) break;
                        j++;
                    }
                } else {
                    j = i + 1;
                }
            }
        }
        uint8_t *d = dev + (uint64_t)rows[i] * dpitch;
        uint8_t *h = host[rows[i]] + off;
        const size_t nrows = (size_t)(rows[j - 1] - rows[i] + 1);
        if (nrows == 1) {
            HIP_TRY(hipMemcpyAsync(h2d ? (void *)d : (void *)h, h2d ? (const void *)h : (const void *)d, w,
                                   h2d ? hipMemcpyHostToDevice : hipMemcpyDeviceToHost, s));
        } else if (h2d) {
            HIP_TRY(hipMemcpy2DAsync(d, dpitch, h, (size_t)hp, w, nrows, hipMemcpyHostToDevice, s));
        } else {
            HIP_TRY(hipMemcpy2DAsync(h, (size_t)hp, d, dpitch, w, nrows, hipMemcpyDeviceToHost, s));
        }
        i = j;
    }
    return RS_OK;
}

// Device views of host rows for the zero-copy row moves (launch_zc_copy): true
// when every row of `rows` lies in pinned host memory the device maps
// (rs_host_alloc, hipHostMalloc), with its device address in z.host[i].  Rows
// in pageable memory, or registered without a device mapping, keep the copies.
// Both ends of each row are looked up: a row whose last byte (S - 1 past its
// start) is not mapped, or not mapped contiguously with its first (a region
// registered shorter than the row, or a row spanning two allocations), keeps
// the copies too, which report an error instead of faulting the GPU.
bool zc_rows(uint8_t *const *shards, const std::vector<int> &rows, uint64_t S, ZcRows &z) {
    if (rows.size() > (size_t)kZcMax || S == 0) return false;
    z.n = 0;
    auto dev_addr = [](const uint8_t *h, uint8_t *&d) {
        hipPointerAttribute_t at{};
        if (hipPointerGetAttributes(&at, h) != hipSuccess) {
            (void)hipGetLastError();
            return false;
        }
        if (at.type != hipMemoryTypeHost || !at.devicePointer || !at.hostPointer) return false;
        d = (uint8_t *)at.devicePointer + (h - (const uint8_t *)at.hostPointer);
        return true;
    };
    for (int r : rows) {
        if ((uintptr_t)shards[r] & 15) return false;  // the kernel moves 16-byte words
        uint8_t *d0 = nullptr, *d1 = nullptr;
        if (!dev_addr(shards[r], d0) || !dev_addr(shards[r] + (S - 1), d1) || d1 != d0 + (S - 1)) return false;
        z.host[z.n] = d0;
        z.slab_row[z.n] = (uint16_t)r;
        z.n++;
    }
    return true;
}

// True when `p` is ordinary pageable host memory (not hipHostMalloc'd or
// registered).  Device-to-host copies into such memory are staged by the
// driver one small copy at a time, which is what made the reconstruct of
// freshly allocated output shards (Go's make([]byte, S), leopard16.go:556-560)
// run at a few GB/s.
bool is_pageable(const void *p) {
    hipPointerAttribute_t at{};
    if (hipPointerGetAttributes(&at, p) != hipSuccess) {
        (void)hipGetLastError();
        return true;
    }
    return at.type != hipMemoryTypeHost && at.type != hipMemoryTypeDevice && at.type != hipMemoryTypeManaged;
}

// Drains the pipeline's three streams on every return path: on an error exit
// copies into or out of the caller's rows (or the bounce slab) may still be in
// flight, and the next call reuses the staging slabs.
struct PipeDrain {
    rs_codec *c;
    ~PipeDrain() {
        if (c->s_in) (void)hipStreamSynchronize(c->s_in);
        if (c->stream) (void)hipStreamSynchronize(c->stream);
        if (c->s_out) (void)hipStreamSynchronize(c->s_out);
    }
};


// Pointer kind for Split/Join: host memory (pageable, pinned or unknown to
// HIP) is copied with memcpy, device memory with hipMemcpy*Async.
bool is_device_ptr(const void *p) {
    hipPointerAttribute_t at{};
    if (hipPointerGetAttributes(&at, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return at.type == hipMemoryTypeDevice;
}

// Split's shard size (leopard16.go:283-288): ceil(len / k) rounded up to 64.
size_t split_per_shard(const rs_codec *c, size_t len) {
    if (c->total == 1 && (len & 63) == 0) return len;
    size_t per = (len + (size_t)c->k - 1) / (size_t)c->k;
    return (per + 63) / 64 * 64;
}

// Drains nothing on success when the call is asynchronous.
struct PipeDrainIf {
    rs_codec *c;
    bool armed = true;
    ~PipeDrainIf() {
        if (!armed) return;
        PipeDrain d{c};
    }
};

// ticket != nullptr: asynchronous encode (outputs in pinned or device memory):
// returns after queueing every segment; *ticket completes when the parity is
// in the caller's rows (rs_encode_wait).
int host_pipeline(rs_codec *c, uint8_t *const *shards, uint64_t S, HostOp op, const std::vector<uint8_t> &present,
                  bool recover_all, int *ok, uint64_t *ticket = nullptr, const ElExt *el_ext = nullptr) {
    int e = ensure_host_pipe(c);
    if (e) return e;
    PipeDrainIf drain_guard{c};
    hipStream_t sc = c->stream;
    e = scratch_acquire(c, sc);
    if (e) return e;
    const int k = c->k, total = c->total;
    std::vector<int> in_rows, out_rows;
    RecPlan pl;
    // LDS-resident reconstruct (rec_lds_ok): the pattern's tables stay in HBM (dev_plan)
    // and every staging slab is strided (shard i at slab + i * seg), so the
    // call uploads nothing and never waits for the previous one
    DevPlan *dpl = nullptr;
    if (op == HostOp::Reconstruct) {
        if (int be = build_decode_plan(c)) return be;
        if (c->dec_ok && rec_lds_ok(c)) {
            e = dev_plan(c, present, recover_all, S, &dpl, el_ext);
            if (e) return e;
            pl = dpl->pl;
        } else {
            e = plan_reconstruct(c, present, recover_all, S, pl, el_ext);
            if (e) return e;
        }
        for (int i = 0; i < total; i++)
            if (present[i]) in_rows.push_back(i);
        out_rows = pl.dst_shard;
    } else {
        for (int i = 0; i < (op == HostOp::Verify ? total : k); i++) in_rows.push_back(i);
        if (op == HostOp::Encode)
            for (int i = k; i < total; i++) out_rows.push_back(i);
    }
    const uint64_t seg = host_segment(c, S, in_rows.size());
    const uint64_t slab = (uint64_t)total * seg;
    const uint64_t slab_al = (slab + 255) / 256 * 256;
    if (c->stage.n / kHostBufs < slab_al) {  // a reallocation waits for queued segments
        HIP_TRY(hipStreamSynchronize(c->s_in));
        HIP_TRY(hipStreamSynchronize(sc));
        HIP_TRY(hipStreamSynchronize(c->s_out));
        HIP_TRY(c->stage.ensure((size_t)kHostBufs * slab_al));
        c->pipe_seq = 0;
    }
    // slabs keep their (kHostBufs) rotation across calls: each call starts at
    // pipe_seq.  Staging buffer b sits at a fixed address (b * stage_cap),
    // whatever this call's segment width: a call with a narrower slab (another
    // shard size, or verify's k+p rows after an encode) must not place its
    // buffer b inside a buffer b' that an earlier asynchronous call still
    // reads; it waits only on ev_free[b].
    const uint64_t stage_cap = (uint64_t)c->stage.n / kHostBufs;  // >= slab_al
    // scratch of the multi-pass paths, sized before any launch (no realloc mid-pipeline)
    // (the LDS-resident reconstruct plan and the m <= 256 LDS encode use none)
    if (op == HostOp::Reconstruct && !dpl) e = scratch_ensure(c, c->work, (size_t)c->n * seg);
    else if (op != HostOp::Reconstruct && !enc_lds_ok(c)) e = scratch_ensure(c, c->work, (size_t)2 * c->m * seg);
    if (e) return e;
    // outputs in pageable memory go D2H into a pinned bounce slab, and the host
    // copies segment j - 1 out while the device works on segment j
    bool use_bounce = false;
    for (int r : out_rows) use_bounce = use_bounce || is_pageable(shards[r]);
    const bool async = ticket && !use_bounce;  // pageable outputs need the host drain: synchronous
    // Reconstruct over pinned rows: one zero-copy kernel per segment and
    // direction instead of a copy per run of present rows and per rebuilt row
    // (30 runs and 32 single rows per segment at C4's random erasures)
    ZcRows zin{}, zout{};
    const int zm = op == HostOp::Reconstruct && !use_bounce ? zc_mask() : 0;
    const bool zc_in = (zm & 1) && zc_rows(shards, in_rows, S, zin);
    const bool zc_out = (zm & 2) && zc_rows(shards, out_rows, S, zout);
    std::vector<std::vector<uint8_t *>> btab(kHostBufs, std::vector<uint8_t *>(total));
    if (use_bounce) {
        const size_t need = (size_t)kHostBufs * slab;
        if (c->bounce_n < need) {
            if (c->bounce) HIP_TRY(hipHostFree(c->bounce));
            c->bounce = nullptr;
            c->bounce_n = 0;
            HIP_TRY(hipHostMalloc((void **)&c->bounce, need, hipHostMallocDefault));
            c->bounce_n = need;
        }
        for (int b = 0; b < kHostBufs; b++)
            for (int i = 0; i < total; i++) btab[b][i] = c->bounce + b * slab + (uint64_t)i * seg;
    }
    const uint64_t seq0 = c->pipe_seq;
    auto drain = [&](uint64_t j) -> int {  // host copy of segment j's outputs out of its bounce slab
        const int b = (int)((seq0 + j) % kHostBufs);
        const uint64_t off = j * seg, w = std::min(seg, S - off);
        HIP_TRY(hipEventSynchronize(c->ev_free[b]));
        for (int r : out_rows) std::memcpy(shards[r] + off, btab[b][r], w);
        return RS_OK;
    };
    std::vector<std::vector<uint8_t *>> sets(kHostBufs, std::vector<uint8_t *>(total));
    if (op == HostOp::Reconstruct && !dpl) {
        // the blob's per-set row tables point into the slabs; a reconstruct
        // waits for every queued segment before it rewrites the blob
        HIP_TRY(hipStreamSynchronize(c->s_out));
        HIP_TRY(hipStreamSynchronize(sc));
        std::vector<uint8_t *const *> d;
        for (int b = 0; b < kHostBufs; b++) {
            for (int i = 0; i < total; i++) sets[b][i] = c->stage.p + b * stage_cap + (uint64_t)i * seg;
            d.push_back(sets[b].data());
        }
        e = upload_reconstruct(c, pl, d, sc);
        if (e) return e;
    }
    // a ticket is numbered up front: a verify ticket owns a mismatch word
    const uint64_t tk = ticket ? c->next_ticket++ : 0;
    const int tslot = (int)(tk % rs_codec::kTickets);
    int *vflag_d = c->dflag, *vflag_h = c->hflag;
    if (ticket) {
        hipEvent_t &ev = c->done_ev[tslot];
        if (!ev) HIP_TRY(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        else if (tk > rs_codec::kTickets) HIP_TRY(hipEventSynchronize(ev));  // the slot's previous ticket is done
        c->tk_kind[tslot] = (uint8_t)((int)op + 1);
        if (op == HostOp::Verify) {
            if (!c->tk_hflag) {
                HIP_TRY(hipHostMalloc((void **)&c->tk_hflag, rs_codec::kTickets * sizeof(int), hipHostMallocDefault));
                HIP_TRY(hipMalloc((void **)&c->tk_dflag, rs_codec::kTickets * sizeof(int)));
            }
            vflag_d = c->tk_dflag + tslot;
            vflag_h = c->tk_hflag + tslot;
        }
    }
    if (op == HostOp::Verify) HIP_TRY(hipMemsetAsync(vflag_d, 0, sizeof(int), sc));
    // copies in must not start before this call's uploads on the compute
    // stream (the multi-pass reconstruct's row tables point into the slabs);
    // no other call has any, and waiting here would queue its copy-in behind
    // every kernel of the previous call
    if (op == HostOp::Reconstruct && !dpl) {
        HIP_TRY(hipEventRecord(c->ev_k[0], sc));
        HIP_TRY(hipStreamWaitEvent(c->s_in, c->ev_k[0], 0));
    }
    const uint64_t nseg = (S + seg - 1) / seg;
    for (uint64_t j = 0; j < nseg; j++) {
        const int b = (int)((seq0 + j) % kHostBufs);
        const uint64_t off = j * seg, w = std::min(seg, S - off);
        uint8_t *st = c->stage.p + b * stage_cap;
        if (seq0 + j >= (uint64_t)kHostBufs) HIP_TRY(hipStreamWaitEvent(c->s_in, c->ev_free[b], 0));
        if (zc_in) HIP_TRY(launch_zc_copy(zin, st, seg, off, w, false, c->s_in));
        else e = copy_rows(st, seg, shards, in_rows, off, w, true, c->s_in, op == HostOp::Reconstruct);
        if (e) return e;
        HIP_TRY(hipEventRecord(c->ev_in[b], c->s_in));
        HIP_TRY(hipStreamWaitEvent(sc, c->ev_in[b], 0));
        if (op == HostOp::Reconstruct && dpl) {
            e = launch_rec_plan(c, dpl, st, seg, 0, 1, w, sc);
        } else if (op == HostOp::Reconstruct) {
            e = launch_reconstruct(c, pl, b, w, sc);
        } else {
            RowSet data{nullptr, st, seg}, par{nullptr, st + (uint64_t)k * seg, seg};
            e = encode_device(c, data, par, w, 0, 1, op == HostOp::Verify ? vflag_d : nullptr, sc);
        }
        if (e) return e;
        HIP_TRY(hipEventRecord(c->ev_k[b], sc));
        if (!out_rows.empty()) {
            HIP_TRY(hipStreamWaitEvent(c->s_out, c->ev_k[b], 0));
            if (use_bounce) e = copy_rows(st, seg, btab[b].data(), out_rows, 0, w, false, c->s_out);
            else if (zc_out) e = launch_zc_copy(zout, st, seg, off, w, true, c->s_out) == hipSuccess ? RS_OK : RS_ERR_DEVICE;
            else e = copy_rows(st, seg, shards, out_rows, off, w, false, c->s_out);
            if (e) return e;
            HIP_TRY(hipEventRecord(c->ev_free[b], c->s_out));
            if (use_bounce && j > 0) {
                e = drain(j - 1);
                if (e) return e;
            }
        } else {
            HIP_TRY(hipEventRecord(c->ev_free[b], sc));
        }
    }
    c->pipe_seq = seq0 + nseg;
    if (op == HostOp::Verify) HIP_TRY(hipMemcpyAsync(vflag_h, vflag_d, sizeof(int), hipMemcpyDeviceToHost, sc));
    e = scratch_release(c, sc);
    if (e) return e;
    if (use_bounce && nseg) {
        e = drain(nseg - 1);
        if (e) return e;
    }
    if (ticket) {
        HIP_TRY(hipEventRecord(c->done_ev[tslot], out_rows.empty() ? sc : c->s_out));
        *ticket = tk;
        if (async) {
            drain_guard.armed = false;
            return RS_OK;
        }
    }
    HIP_TRY(hipStreamSynchronize(c->s_in));
    HIP_TRY(hipStreamSynchronize(sc));
    HIP_TRY(hipStreamSynchronize(c->s_out));
    if (op == HostOp::Verify && ok) {
        *ok = *(volatile int *)vflag_h == 0;
    }
    return RS_OK;
}

}  // namespace

// ---------------------------------------------------------------- multi-device parts (multi.hpp)
int rs::part_host_call(rs_codec *c, HostOp op, uint8_t *const *shards, uint64_t S, const std::vector<uint8_t> &present,
                       bool recover_all, int *ok, uint64_t *ticket, const ElExt *el) {
    std::lock_guard<std::mutex> lk(c->mu);
    DeviceGuard g(c->device);
    if (int ie = ensure_device(c)) return ie;
    return host_pipeline(c, shards, S, op, present, recover_all, ok, ticket, el);
}

// The locators a single-device codec would use for this call (its reference-
// keyed GF(2^8) cache, whose useBits key depends on the full S, else the exact
// ones), looked up once per call like leopard8.go:509-554.  The pointer stays
// valid while the parent's mutex is held, i.e. for the whole multi call.
int rs::parent_error_locators(rs_codec *c, const std::vector<uint8_t> &present, bool recover_all, uint64_t S,
                              ElExt &out) {
    out = ElExt{};
    if (const std::vector<uint32_t> *r = ref_inv_errlocs(c, present, recover_all, S)) {
        out.el = r;
        out.ref = true;
        return RS_OK;
    }
    std::vector<uint8_t> erased(c->total);
    for (int i = 0; i < c->total; i++) erased[i] = !present[i];
    out.el = error_locs_cached(c, erased);
    return out.el ? RS_OK : RS_ERR_PANIC;
}

// Host simulation of the split schedules against the plain op lists on random
// GF(2^16) symbols and random twiddle logs (modulus included): returns the
// number of differing rows over both transforms (0 = identical).
namespace {
template <class OPS, class SCH>
int split_sim_one(const Field &F, const SCH &s, uint32_t &seed) {
    constexpr OPS ops{};
    constexpr int M = SCH::M, HM = SCH::HM;
    auto rnd = [&]() { seed = seed * 1664525u + 1013904223u; return seed >> 8; };
    std::vector<uint32_t> logs(OPS::N + 1);
    for (auto &l : logs) l = (rnd() % 5 == 0) ? F.mod : rnd() % F.mod;
    std::vector<uint32_t> in(M), ref(M);
    for (int r = 0; r < M; r++) in[r] = ref[r] = rnd() & 0xFFFF;
    auto mul = [&](uint32_t v, uint32_t lg) -> uint32_t { return (v == 0 || lg == F.mod) ? 0 : F.mul_log(v, lg); };
    for (int i = 0; i < OPS::N; i++) {
        const BOp o = ops.op[i];
        uint32_t &x = ref[o.x], &y = ref[o.y];
        if (o.kind == OP_IFFT) { y ^= x; x ^= mul(y, logs[o.slot]); }
        else if (o.kind == OP_FFT) { x ^= mul(y, logs[o.slot]); y ^= x; }
        else y ^= x;
    }
    uint32_t reg[2][HM > 0 ? HM : 1];
    for (int r = 0; r < M; r++) {
        // initial layout: the schedule's row0 (lower) and its bit-h0 partner (upper)
        for (int k = 0; k < HM; k++) {
            if (s.row0[k] == r) reg[0][k] = in[r];
            if ((s.row0[k] | (1 << s.h0)) == r) reg[1][k] = in[r];
        }
    }
    for (int i = 0; i < s.nsteps; i++) {
        const SStep st = s.step[i];
        if (st.type == ST_SWAP) { std::swap(reg[1][st.a], reg[0][st.b]); continue; }
        for (int h = 0; h < 2; h++) {
            uint32_t &x = reg[h][st.a], &y = reg[h][st.b];
            const int slot = st.tab < 0 ? -1 : (h ? s.tab_hi[st.tab] : s.tab_lo[st.tab]);
            const uint32_t lg = slot < 0 ? F.mod : logs[slot];
            if (st.kind == OP_IFFT) { y ^= x; x ^= mul(y, lg); }
            else if (st.kind == OP_FFT) { x ^= mul(y, lg); y ^= x; }
            else y ^= x;
        }
    }
    int bad = 0;
    for (int h = 0; h < 2; h++)
        for (int k = 0; k < HM; k++) bad += reg[h][k] != ref[s.fin_row[h][k]];
    return bad;
}
template <int L>
int split_sim(const Field &F, uint32_t seed) {
    int bad = 0;
    for (int it = 0; it < 8; it++) {
        bad += split_sim_one<IfftOps<L>>(F, EncodeSplit<L>::ifft, seed);
        bad += split_sim_one<FftOps<L>>(F, EncodeSplit<L>::fft, seed);
    }
    // the chunk IFFT must end in the split bit the FFT starts from
    if (EncodeSplit<L>::ifft.hend != EncodeSplit<L>::fft.h0) bad += 1000;
    return bad;
}
}  // namespace

// Host emulation of k_encode_split (data flow of the kernel, bit for bit):
// twiddle images from split_image (as uploaded), the byte-permute multiply of
// F16::mul_add, the half-wave swaps and the row layouts of schedule.hpp.
namespace {
inline uint32_t emu_perm(uint32_t s0, uint32_t s1, uint32_t sel) {
    const uint64_t d = ((uint64_t)s0 << 32) | s1;
    uint32_t r = 0;
    for (int b = 0; b < 4; b++) r |= (uint32_t)((d >> (8 * ((sel >> (8 * b)) & 7))) & 0xFF) << (8 * b);
    return r;
}
inline void emu_mul_add(uint32_t &xl, uint32_t &xh, uint32_t lo, uint32_t hi, const uint32_t *t) {
    const uint32_t a0 = lo & 0x07070707u, a1 = (lo >> 3) & 0x07070707u, a2 = (lo >> 6) & 0x03030303u;
    const uint32_t b0 = hi & 0x07070707u, b1 = (hi >> 3) & 0x07070707u, b2 = (hi >> 6) & 0x03030303u;
    xl ^= emu_perm(t[1], t[0], a0) ^ emu_perm(t[5], t[4], a1) ^ emu_perm(t[8], t[8], a2) ^ emu_perm(t[11], t[10], b0) ^
          emu_perm(t[15], t[14], b1) ^ emu_perm(t[18], t[18], b2);
    xh ^= emu_perm(t[3], t[2], a0) ^ emu_perm(t[7], t[6], a1) ^ emu_perm(t[9], t[9], a2) ^ emu_perm(t[13], t[12], b0) ^
          emu_perm(t[17], t[16], b1) ^ emu_perm(t[19], t[19], b2);
}
template <class SCH>
void emu_run(const SCH &s, uint32_t (*rl)[16], uint32_t (*rh)[16], const uint32_t *img) {
    const int nt = s.ntab;
    for (int i = 0; i < s.nsteps; i++) {
        const SStep st = s.step[i];
        if (st.type == ST_SWAP) {
            std::swap(rl[1][st.a], rl[0][st.b]);
            std::swap(rh[1][st.a], rh[0][st.b]);
            continue;
        }
        for (int h = 0; h < 2; h++) {
            uint32_t &xl = rl[h][st.a], &xh = rh[h][st.a], &yl = rl[h][st.b], &yh = rh[h][st.b];
            const uint32_t *t = st.tab >= 0 ? img + (size_t)(h * nt + st.tab) * kTwDwords16 : nullptr;
            if (st.kind == OP_IFFT) {
                yl ^= xl; yh ^= xh;
                emu_mul_add(xl, xh, yl, yh, t);
            } else if (st.kind == OP_FFT) {
                emu_mul_add(xl, xh, yl, yh, t);
                yl ^= xl; yh ^= xh;
            } else {
                yl ^= xl; yh ^= xh;
            }
        }
    }
}
template <int L>
int emu_split(rs_codec *c, const uint8_t *data, uint8_t *parity, uint64_t S) {
    const auto &SI = EncodeSplit<L>::ifft;
    const auto &SF = EncodeSplit<L>::fft;
    constexpr int M = 1 << L, HM = M / 2;
    SplitTabs ti, tf;
    split_tabs(L, false, ti);
    split_tabs(L, true, tf);
    const int is = ifft_slots(L);
    const size_t ni = 2 * ti.lo.size() * kTwDwords16;
    std::vector<uint32_t> imi((size_t)c->nchunks * ni), imf(2 * tf.lo.size() * kTwDwords16 + 1);
    for (int ch = 0; ch < c->nchunks; ch++) split_image(*c->F, ti, c->enc_ifft_logs.data() + (size_t)ch * is, imi.data() + ch * ni);
    split_image(*c->F, tf, c->enc_fft_logs.data(), imf.data());
    auto dword = [&](const uint8_t *row, uint64_t off) { uint32_t v; std::memcpy(&v, row + off, 4); return v; };
    for (uint64_t u = 0; u < S / 8; u++) {
        const uint64_t lo_off = (u / 8) * 64 + (u % 8) * 4;
        uint32_t al[2][16] = {}, ah[2][16] = {};
        for (int ch = 0; ch < c->nchunks; ch++) {
            uint32_t cl[2][16] = {}, chh[2][16] = {};
            for (int h = 0; h < 2; h++)
                for (int k = 0; k < HM; k++) {
                    const int row = ch * M + SI.row0[k] + h * (1 << SI.h0);
                    if (row < c->k) {
                        cl[h][k] = dword(data + (size_t)row * S, lo_off);
                        chh[h][k] = dword(data + (size_t)row * S, lo_off + 32);
                    }
                }
            emu_run(SI, cl, chh, imi.data() + ch * ni);
            for (int h = 0; h < 2; h++)
                for (int k = 0; k < HM; k++) {
                    al[h][k] ^= cl[h][k];
                    ah[h][k] ^= chh[h][k];
                }
        }
        emu_run(SF, al, ah, imf.data());
        for (int h = 0; h < 2; h++)
            for (int k = 0; k < HM; k++) {
                const int row = SF.fin_row[h][k];
                if (row < c->p) {
                    std::memcpy(parity + (size_t)row * S + lo_off, &al[h][k], 4);
                    std::memcpy(parity + (size_t)row * S + lo_off + 32, &ah[h][k], 4);
                }
            }
    }
    return RS_OK;
}
}  // namespace

extern "C" {

int rs_new(int field_bits, int data_shards, int parity_shards, int device, rs_codec **out) {
    if (!out) return RS_ERR_INVALID_ARG;
    *out = nullptr;
    // New: reedsolomon.go:69-81; newFF16/newFF8 validation leopard16.go:39-45, leopard8.go:56-62.
    if (data_shards <= 0 || parity_shards <= 0) return RS_ERR_INV_SHARD_NUM;
    if (field_bits == 0) field_bits = data_shards + parity_shards <= 256 ? 8 : 16;
    if (field_bits != 8 && field_bits != 16) return RS_ERR_INVALID_ARG;
    if (data_shards + parity_shards > 65536) return RS_ERR_MAX_SHARD_NUM;
    rs_codec *c = new (std::nothrow) rs_codec();
    if (!c) return RS_ERR_NOMEM;
    c->bits = field_bits;
    c->k = data_shards;
    c->p = parity_shards;
    c->total = data_shards + parity_shards;
    c->m = ceil_pow2(parity_shards);
    c->logm = ilog2(c->m);
    c->device = device;
    c->F = &field(field_bits);
    c->twd = tw_dwords(field_bits);
    plan_encode_host(c);  // device resources are created on first use
    *out = c;
    return RS_OK;
}

void rs_free(rs_codec *c) { delete c; }

int rs_new_multi(int field_bits, int data_shards, int parity_shards, const int *devices, int ndevices, rs_codec **out) {
    if (!out) return RS_ERR_INVALID_ARG;
    *out = nullptr;
    if (!devices || ndevices < 1 || ndevices > RS_MAX_DEVICES) return RS_ERR_INVALID_ARG;
    rs_codec *c = nullptr;
    int e = rs_new(field_bits, data_shards, parity_shards, devices[0], &c);
    if (e) return e;
    if (ndevices == 1) {  // one device: the plain codec
        *out = c;
        return RS_OK;
    }
    std::vector<rs_codec *> parts;
    for (int g = 0; g < ndevices && !e; g++) {
        rs_codec *q = nullptr;
        e = rs_new(c->bits, data_shards, parity_shards, devices[g], &q);
        if (e) break;
        q->ref_inv = false;  // the parent hands every part its locators (parent_error_locators)
        parts.push_back(q);
    }
    if (!e) {
        c->multi = multi_create(parts, std::vector<int>(devices, devices + ndevices));
        if (!c->multi) e = RS_ERR_NOMEM;
    }
    if (e) {
        if (!c->multi)
            for (rs_codec *q : parts) delete q;
        delete c;
        return e;
    }
    *out = c;
    return RS_OK;
}

int rs_device_count(const rs_codec *c) { return !c ? 0 : c->multi ? multi_count(c->multi) : 1; }

int rs_device_part(rs_codec *c, int index, rs_codec **part, int *device) {
    if (!c || !part) return RS_ERR_INVALID_ARG;
    *part = nullptr;
    if (index < 0 || index >= rs_device_count(c)) return RS_ERR_INVALID_ARG;
    int dev = c->device;
    *part = c->multi ? multi_part(c->multi, index, &dev) : c;
    if (device) *device = dev;
    return RS_OK;
}

int rs_byte_range(size_t shard_size, int index, int nparts, size_t *lo, size_t *hi) {
    if (!lo || !hi || nparts < 1 || index < 0 || index >= nparts) return RS_ERR_INVALID_ARG;
    if (shard_size % 64) return RS_ERR_INVALID_SHARD_SIZE;
    uint64_t l = 0, h = 0;
    part_byte_range(shard_size, index, nparts, l, h);
    *lo = (size_t)l;
    *hi = (size_t)h;
    return RS_OK;
}

int rs_field_bits(const rs_codec *c) { return c ? c->bits : 0; }
int rs_data_shards(const rs_codec *c) { return c ? c->k : 0; }
int rs_parity_shards(const rs_codec *c) { return c ? c->p : 0; }
int rs_total_shards(const rs_codec *c) { return c ? c->total : 0; }
int rs_shard_size_multiple(const rs_codec *c) { return c ? 64 : 0; }
const char *rs_encode_path(const rs_codec *c) { return c ? c->path.c_str() : ""; }

int rs_encode_dev(rs_codec *c, uint8_t *const *d, size_t S, void *stream) {
    if (!c || !d) return RS_ERR_INVALID_ARG;
    if (c->multi) return RS_ERR_INVALID_ARG;  // device rows live on one device: use rs_device_part
    for (int i = 0; i < c->total; i++)
        if (!d[i]) return RS_ERR_INVALID_ARG;
    if (S == 0) return RS_ERR_SHARD_NO_DATA;
    if (S % 64) return RS_ERR_INVALID_SHARD_SIZE;
    std::lock_guard<std::mutex> lk(c->mu);
    DeviceGuard g(c->device);
    if (int ie = ensure_device(c)) return ie;
    hipStream_t s = pick_stream(c, stream);
    RowSet data, par;
    int e = make_rowsets(c, d, s, data, par);
    if (e) return e;
    const bool scr = encode_uses_scratch(c, data, par);
    if (scr && (e = scratch_acquire(c, s))) return e;
    e = encode_device(c, data, par, S, 0, 1, nullptr, s);
    if (e) return e;
    if (scr && (e = scratch_release(c, s))) return e;
    if (!stream) HIP_TRY(hipStreamSynchronize(s));
    return RS_OK;
}

int rs_encode_dev_batch(rs_codec *c, uint8_t *base, size_t row_stride, size_t stripe_stride, int nstripes, size_t S,
                        void *stream) {
    if (!c || !base || nstripes <= 0) return RS_ERR_INVALID_ARG;
    if (c->multi) return RS_ERR_INVALID_ARG;  // device rows live on one device: use rs_device_part
    if (S == 0) return RS_ERR_SHARD_NO_DATA;
    if (S % 64) return RS_ERR_INVALID_SHARD_SIZE;
    std::lock_guard<std::mutex> lk(c->mu);
    DeviceGuard g(c->device);
    if (int ie = ensure_device(c)) return ie;
    hipStream_t s = pick_stream(c, stream);
    RowSet data{nullptr, base, row_stride}, par{nullptr, base + (size_t)c->k * row_stride, row_stride};
    const bool scr = encode_uses_scratch(c, data, par);
    int e = scr ? scratch_acquire(c, s) : RS_OK;
    if (e) return e;
    e = encode_device(c, data, par, S, stripe_stride, nstripes, nullptr, s);
    if (e) return e;
    if (scr && (e = scratch_release(c, s))) return e;
    if (!stream) HIP_TRY(hipStreamSynchronize(s));
    return RS_OK;
}

int rs_verify_dev(rs_codec *c, uint8_t *const *d, size_t S, int *ok, void *stream) {
    if (!c || !d || !ok) return RS_ERR_INVALID_ARG;
    if (c->multi) return RS_ERR_INVALID_ARG;  // device rows live on one device: use rs_device_part
    *ok = 0;
    for (int i = 0; i < c->total; i++)
        if (!d[i]) return RS_ERR_INVALID_ARG;
    if (S == 0) return RS_ERR_SHARD_NO_DATA;
    if (S % 64) return RS_ERR_INVALID_SHARD_SIZE;
    std::lock_guard<std::mutex> lk(c->mu);
    DeviceGuard g(c->device);
    if (int ie = ensure_device(c)) return ie;
    hipStream_t s = pick_stream(c, stream);
    RowSet data, par;
    int e = make_rowsets(c, d, s, data, par);
    if (e) return e;
    e = scratch_acquire(c, s);
    if (e) return e;
    HIP_TRY(hipMemsetAsync(c->dflag, 0, sizeof(int), s));
    e = encode_device(c, data, par, S, 0, 1, c->dflag, s);
    if (e) return e;
    e = scratch_release(c, s);
    if (e) return e;
    HIP_TRY(hipMemcpyAsync(c->hflag, c->dflag, sizeof(int), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    *ok = *(volatile int *)c->hflag == 0;
    return RS_OK;
}

int rs_verify_dev_batch(rs_codec *c, uint8_t *base, size_t row_stride, size_t stripe_stride, int nstripes, size_t S,
                        int *ok, void *stream) {
    if (!c || !base || !ok || nstripes <= 0) return RS_ERR_INVALID_ARG;
    if (c->multi) return RS_ERR_INVALID_ARG;  // device rows live on one device: use rs_device_part
    *ok = 0;
    if (S == 0) return RS_ERR_SHARD_NO_DATA;
    if (S % 64) return RS_ERR_INVALID_SHARD_SIZE;
    std::lock_guard<std::mutex> lk(c->mu);
    DeviceGuard g(c->device);
    if (int ie = ensure_device(c)) return ie;
    hipStream_t s = pick_stream(c, stream);
    RowSet data{nullptr, base, row_stride}, par{nullptr, base + (size_t)c->k * row_stride, row_stride};
    int e = scratch_acquire(c, s);
    if (e) return e;
    HIP_TRY(hipMemsetAsync(c->dflag, 0, sizeof(int), s));
    e = encode_device(c, data, par, S, stripe_stride, nstripes, c->dflag, s);
    if (e) return e;
    e = scratch_release(c, s);
    if (e) return e;
    HIP_TRY(hipMemcpyAsync(c->hflag, c->dflag, sizeof(int), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    *ok = *(volatile int *)c->hflag == 0;
    return RS_OK;
}

int rs_reconstruct_dev_batch(rs_codec *c, uint8_t *base, size_t row_stride, size_t stripe_stride, size_t nstripes,
                             const uint8_t *present, size_t S, int recover_all, void *stream) {
    if (!c || !base || !present || nstripes == 0 || nstripes > (size_t)INT32_MAX) return RS_ERR_INVALID_ARG;
    if (c->multi) return RS_ERR_INVALID_ARG;  // device rows live on one device: use rs_device_part
    std::vector<uint8_t> pr(present, present + c->total);
    int np = 0, dp = 0;
    for (int i = 0; i < c->total; i++)
        if (pr[i]) {
            np++;
            if (i < c->k) dp++;
        }
    if (np == 0 || S == 0) return RS_ERR_SHARD_NO_DATA;
    if (np == c->total || (!recover_all && dp == c->k)) return RS_OK;
    if (np < c->k) return RS_ERR_TOO_FEW_SHARDS;
    if (S % 64) return RS_ERR_INVALID_SHARD_SIZE;
    if (row_stride < S || (nstripes > 1 && stripe_stride < (size_t)c->total * row_stride)) return RS_ERR_INVALID_ARG;
    std::lock_guard<std::mutex> lk(c->mu);
    DeviceGuard g(c->device);
    if (int ie = ensure_device(c)) return ie;
    const hipStream_t s = pick_stream(c, stream);
    if (int e = build_decode_plan(c)) return e;
    if (c->dec_ok && rec_lds_ok(c)) {
        // one launch: grid.y = stripe, the pattern's tables shared (dev_plan cache)
        DevPlan *dpl = nullptr;
        if (int e = dev_plan(c, pr, recover_all != 0, S, &dpl)) return e;
        if (int e = launch_rec_plan(c, dpl, base, row_stride, stripe_stride, (int)nstripes, S, s)) return e;
        if (!stream) HIP_TRY(hipStreamSynchronize(s));  // no caller stream: complete on return
        return RS_OK;
    }
    // multi-pass codecs (n > 256): stripe by stripe
    std::vector<uint8_t *> rows(c->total);
    for (size_t z = 0; z < nstripes; z++) {
        for (int i = 0; i < c->total; i++) rows[i] = base + z * stripe_stride + (uint64_t)i * row_stride;
        if (int e = reconstruct_device(c, rows.data(), pr, S, recover_all != 0, s)) return e;
    }
    return RS_OK;
}

int rs_reconstruct_dev(rs_codec *c, uint8_t *const *d, const uint8_t *present, size_t S, int recover_all,
                       void *stream) {
    if (!c || !d || !present) return RS_ERR_INVALID_ARG;
    if (c->multi) return RS_ERR_INVALID_ARG;  // device rows live on one device: use rs_device_part
    std::vector<uint8_t> pr(present, present + c->total);
    int np = 0, dp = 0;
    for (int i = 0; i < c->total; i++)
        if (pr[i]) {
            np++;
            if (i < c->k) dp++;
        }
    if (np == 0 || S == 0) return RS_ERR_SHARD_NO_DATA;
    if (np == c->total || (!recover_all && dp == c->k)) return RS_OK;
    if (np < c->k) return RS_ERR_TOO_FEW_SHARDS;
    if (S % 64) return RS_ERR_INVALID_SHARD_SIZE;
    const int end = recover_all ? c->total : c->k;
    for (int i = 0; i < c->total; i++)
        if ((pr[i] || i < end) && !d[i]) return RS_ERR_INVALID_ARG;
    std::lock_guard<std::mutex> lk(c->mu);
    DeviceGuard g(c->device);
    if (int ie = ensure_device(c)) return ie;
    const hipStream_t s = pick_stream(c, stream);
    if (int e = build_decode_plan(c)) return e;
    if (c->dec_ok && rec_lds_ok(c)) {
        if (int e = reconstruct_device_lds(c, d, pr, S, recover_all != 0, s)) return e;
        if (!stream) HIP_TRY(hipStreamSynchronize(s));  // no caller stream: complete on return
        return RS_OK;
    }
    return reconstruct_device(c, d, pr, S, recover_all != 0, s);
}

int rs_encode(rs_codec *c, uint8_t *const *shards, const size_t *lens, int nshards) {
    if (!c || !shards || !lens) return RS_ERR_INVALID_ARG;
    if (nshards != c->total) return RS_ERR_TOO_FEW_SHARDS;
    int e = check_shards(lens, nshards, false);
    if (e) return e;
    const uint64_t S = shard_size_of(lens, nshards);
    if (S % 64) return RS_ERR_INVALID_SHARD_SIZE;
    if (!c->enc_ok) return RS_ERR_PANIC;
    for (int i = 0; i < nshards; i++)
        if (!shards[i]) return RS_ERR_INVALID_ARG;
    std::lock_guard<std::mutex> lk(c->mu);
    if (c->multi) return multi_host(c->multi, c, HostOp::Encode, shards, S, {}, true, nullptr, nullptr);
    DeviceGuard g(c->device);
    if (int ie = ensure_device(c)) return ie;
    return host_pipeline(c, shards, S, HostOp::Encode, {}, true, nullptr);
}

int rs_encode_async(rs_codec *c, uint8_t *const *shards, const size_t *lens, int nshards, uint64_t *ticket) {
    if (!c || !shards || !lens || !ticket) return RS_ERR_INVALID_ARG;
    if (nshards != c->total) return RS_ERR_TOO_FEW_SHARDS;
    int e = check_shards(lens, nshards, false);
    if (e) return e;
    const uint64_t S = shard_size_of(lens, nshards);
    if (S % 64) return RS_ERR_INVALID_SHARD_SIZE;
    if (!c->enc_ok) return RS_ERR_PANIC;
    for (int i = 0; i < nshards; i++)
        if (!shards[i]) return RS_ERR_INVALID_ARG;
    std::lock_guard<std::mutex> lk(c->mu);
    if (c->multi) return multi_host(c->multi, c, HostOp::Encode, shards, S, {}, true, nullptr, ticket);
    DeviceGuard g(c->device);
    if (int ie = ensure_device(c)) return ie;
    return host_pipeline(c, shards, S, HostOp::Encode, {}, true, nullptr, ticket);
}

int rs_encode_query(rs_codec *c, uint64_t ticket, int *done) {
    if (!c || !done) return RS_ERR_INVALID_ARG;
    if (c->multi) return multi_ticket_query(c->multi, ticket, done);
    hipEvent_t ev;
    {
        std::lock_guard<std::mutex> lk(c->mu);
        if (ticket >= c->next_ticket) return RS_ERR_INVALID_ARG;
        if (ticket == 0) {  // no work was queued (rs_reconstruct_async with nothing missing)
            *done = 1;
            return RS_OK;
        }
        ev = c->done_ev[ticket % rs_codec::kTickets];
    }
    DeviceGuard g(c->device);
    const hipError_t q = hipEventQuery(ev);
    if (q == hipErrorNotReady) {
        *done = 0;
        return RS_OK;
    }
    HIP_TRY(q);
    *done = 1;
    return RS_OK;
}

int rs_encode_wait(rs_codec *c, uint64_t ticket) {
    if (!c) return RS_ERR_INVALID_ARG;
    if (c->multi) return multi_ticket_wait(c->multi, ticket);
    hipEvent_t ev;
    {
        std::lock_guard<std::mutex> lk(c->mu);
        if (ticket >= c->next_ticket) return RS_ERR_INVALID_ARG;
        if (ticket == 0) return RS_OK;  // no work was queued
        // an event slot reused by a later call completes after this ticket's
        // work (same streams, queue order): waiting on it is still correct
        ev = c->done_ev[ticket % rs_codec::kTickets];
    }
    DeviceGuard g(c->device);
    HIP_TRY(hipEventSynchronize(ev));
    return RS_OK;
}

int rs_ticket_query(rs_codec *c, uint64_t ticket, int *done) { return rs_encode_query(c, ticket, done); }
int rs_ticket_wait(rs_codec *c, uint64_t ticket) { return rs_encode_wait(c, ticket); }

int rs_verify_async(rs_codec *c, uint8_t *const *shards, const size_t *lens, int nshards, uint64_t *ticket) {
    if (!c || !shards || !lens || !ticket) return RS_ERR_INVALID_ARG;
    if (nshards != c->total) return RS_ERR_TOO_FEW_SHARDS;
    int e = check_shards(lens, nshards, false);
    if (e) return e;
    const uint64_t S = lens[0];
    if (S % 64) return RS_ERR_INVALID_SHARD_SIZE;
    if (!c->enc_ok) return RS_ERR_PANIC;
    for (int i = 0; i < nshards; i++)
        if (!shards[i]) return RS_ERR_INVALID_ARG;
    std::lock_guard<std::mutex> lk(c->mu);
    if (c->multi) return multi_host(c->multi, c, HostOp::Verify, shards, S, {}, true, nullptr, ticket);
    DeviceGuard g(c->device);
    if (int ie = ensure_device(c)) return ie;
    return host_pipeline(c, shards, S, HostOp::Verify, {}, true, nullptr, ticket);
}

int rs_verify_result(rs_codec *c, uint64_t ticket, int *ok) {
    if (!c || !ok) return RS_ERR_INVALID_ARG;
    *ok = 0;
    if (c->multi) return multi_verify_result(c->multi, ticket, ok);
    const int slot = (int)(ticket % rs_codec::kTickets);
    // the slot must still hold this verify ticket (not reused by a later call)
    auto owns_slot = [&] {
        return ticket != 0 && ticket < c->next_ticket && ticket + rs_codec::kTickets >= c->next_ticket &&
               c->tk_kind[slot] == (uint8_t)((int)HostOp::Verify + 1) && c->tk_hflag;
    };
    {
        std::lock_guard<std::mutex> lk(c->mu);
        if (!owns_slot()) return RS_ERR_INVALID_ARG;
    }
    if (int e = rs_encode_wait(c, ticket)) return e;
    // read the verdict under the lock, after checking again that no later call
    // (ticket + kTickets) has taken the slot and rewritten its flag meanwhile
    std::lock_guard<std::mutex> lk(c->mu);
    if (!owns_slot()) return RS_ERR_INVALID_ARG;
    *ok = *(volatile int *)(c->tk_hflag + slot) == 0;
    return RS_OK;
}

int rs_verify(rs_codec *c, uint8_t *const *shards, const size_t *lens, int nshards, int *ok) {
    if (!c || !shards || !lens || !ok) return RS_ERR_INVALID_ARG;
    *ok = 0;
    if (nshards != c->total) return RS_ERR_TOO_FEW_SHARDS;
    int e = check_shards(lens, nshards, false);
    if (e) return e;
    const uint64_t S = lens[0];
    if (S % 64) return RS_ERR_INVALID_SHARD_SIZE;
    if (!c->enc_ok) return RS_ERR_PANIC;
    for (int i = 0; i < nshards; i++)
        if (!shards[i]) return RS_ERR_INVALID_ARG;
    std::lock_guard<std::mutex> lk(c->mu);
    if (c->multi) return multi_host(c->multi, c, HostOp::Verify, shards, S, {}, true, ok, nullptr);
    DeviceGuard g(c->device);
    if (int ie = ensure_device(c)) return ie;
    return host_pipeline(c, shards, S, HostOp::Verify, {}, true, ok);
}

}  // extern "C"

namespace {
// rs_reconstruct / rs_reconstruct_async.  Nothing to rebuild: RS_OK with no
// ticket issued (*ticket stays 0, which rs_ticket_wait / query report as done).
int reconstruct_host(rs_codec *c, uint8_t *const *shards, size_t *lens, int nshards, int recover_all, uint64_t *ticket) {
    if (!c || !shards || !lens) return RS_ERR_INVALID_ARG;
    if (nshards != c->total) return RS_ERR_TOO_FEW_SHARDS;
    int e = check_shards(lens, nshards, true);
    if (e) return e;
    int np = 0, dp = 0;
    for (int i = 0; i < c->total; i++)
        if (lens[i]) {
            np++;
            if (i < c->k) dp++;
        }
    if (np == c->total || (!recover_all && dp == c->k)) return RS_OK;
    if (np < c->k) return RS_ERR_TOO_FEW_SHARDS;
    const uint64_t S = shard_size_of(lens, nshards);
    if (S % 64) return RS_ERR_INVALID_SHARD_SIZE;
    const int end = recover_all ? c->total : c->k;
    for (int i = 0; i < c->total; i++)
        if ((lens[i] || i < end) && !shards[i]) return RS_ERR_INVALID_ARG;
    std::lock_guard<std::mutex> lk(c->mu);
    std::vector<uint8_t> pr(c->total);
    for (int i = 0; i < c->total; i++) pr[i] = lens[i] != 0;
    if (c->multi) {
        e = multi_host(c->multi, c, HostOp::Reconstruct, shards, S, pr, recover_all != 0, nullptr, ticket);
    } else {
        DeviceGuard g(c->device);
        if (int ie = ensure_device(c)) return ie;
        e = host_pipeline(c, shards, S, HostOp::Reconstruct, pr, recover_all != 0, nullptr, ticket);
    }
    if (e) return e;
    for (int i = 0; i < end; i++)
        if (!pr[i]) lens[i] = S;
    return RS_OK;
}
}  // namespace

extern "C" {

int rs_reconstruct(rs_codec *c, uint8_t *const *shards, size_t *lens, int nshards, int recover_all) {
    return reconstruct_host(c, shards, lens, nshards, recover_all, nullptr);
}

int rs_reconstruct_async(rs_codec *c, uint8_t *const *shards, size_t *lens, int nshards, int recover_all,
                         uint64_t *ticket) {
    if (!ticket) return RS_ERR_INVALID_ARG;
    *ticket = 0;
    return reconstruct_host(c, shards, lens, nshards, recover_all, ticket);
}

int rs_split_shard_size(const rs_codec *c, size_t len, size_t *per_shard) {
    if (!c || !per_shard) return RS_ERR_INVALID_ARG;
    if (len == 0) return RS_ERR_SHORT_DATA;
    *per_shard = split_per_shard(c, len);
    return RS_OK;
}

int rs_split(rs_codec *c, const uint8_t *data, size_t len, uint8_t *dst, size_t dst_stride, void *stream) {
    if (!c || !data || !dst) return RS_ERR_INVALID_ARG;
    if (c->multi) c = multi_part(c->multi, 0, nullptr);  // same geometry; device copies on part 0's stream
    if (len == 0) return RS_ERR_SHORT_DATA;  // leopard16.go:279-281
    const size_t per = split_per_shard(c, len);
    if (dst_stride < per && c->total > 1) return RS_ERR_INVALID_ARG;
    const int total = c->total;
    const size_t nfull = std::min<size_t>(len / per, (size_t)total), rem = nfull < (size_t)total ? len - nfull * per : 0;
    const bool ddev = is_device_ptr(dst), sdev = is_device_ptr(data);
    if (!ddev && !sdev) {  // host -> host: plain copies, no device involved
        for (int i = 0; i < total; i++) {
            uint8_t *row = dst + (size_t)i * dst_stride;
            const size_t have = (size_t)i < nfull ? per : (size_t)i == nfull ? rem : 0;
            if (have) std::memcpy(row, data + (size_t)i * per, have);
            if (have < per) std::memset(row + have, 0, per - have);
        }
        return RS_OK;
    }
    std::lock_guard<std::mutex> lk(c->mu);
    DeviceGuard g(c->device);
    if (int ie = ensure_device(c)) return ie;
    hipStream_t s = pick_stream(c, stream);
    if (nfull) HIP_TRY(hipMemcpy2DAsync(dst, dst_stride, data, per, per, nfull, hipMemcpyDefault, s));
    if (rem) HIP_TRY(hipMemcpyAsync(dst + nfull * dst_stride, data + nfull * per, rem, hipMemcpyDefault, s));
    const size_t zrow = nfull + (rem ? 1 : 0);
    if (ddev) {
        if (rem) HIP_TRY(hipMemsetAsync(dst + nfull * dst_stride + rem, 0, per - rem, s));
        if (zrow < (size_t)total) HIP_TRY(hipMemset2DAsync(dst + zrow * dst_stride, dst_stride, 0, per, total - zrow, s));
    } else {
        HIP_TRY(hipStreamSynchronize(s));
        if (rem) std::memset(dst + nfull * dst_stride + rem, 0, per - rem);
        for (size_t i = zrow; i < (size_t)total; i++) std::memset(dst + i * dst_stride, 0, per);
    }
    if (!stream) HIP_TRY(hipStreamSynchronize(s));
    return RS_OK;
}

int rs_join(rs_codec *c, uint8_t *const *shards, const size_t *lens, int nshards, uint8_t *dst, size_t out_size,
            void *stream) {
    if (!c || !shards || !lens || (!dst && out_size)) return RS_ERR_INVALID_ARG;
    if (c->multi) c = multi_part(c->multi, 0, nullptr);
    if (nshards < c->k) return RS_ERR_TOO_FEW_SHARDS;  // leopard16.go:232-236
    size_t size = 0;
    int use = 0;
    for (int i = 0; i < c->k; i++) {  // :239-250
        if (!shards[i]) return RS_ERR_RECONSTRUCT_REQUIRED;  // nil; a zero-length shard counts 0 bytes
        size += lens[i];
        use = i + 1;
        if (size >= out_size) break;
    }
    if (size < out_size) return RS_ERR_SHORT_DATA;  // :251-253
    bool dev = is_device_ptr(dst);
    for (int i = 0; i < use && !dev; i++) dev = lens[i] && is_device_ptr(shards[i]);
    size_t written = 0;
    if (!dev) {
        for (int i = 0; i < use && written < out_size; i++) {  // :256-268
            const size_t n = std::min(lens[i], out_size - written);
            if (n) std::memcpy(dst + written, shards[i], n);
            written += n;
        }
        return RS_OK;
    }
    std::lock_guard<std::mutex> lk(c->mu);
    DeviceGuard g(c->device);
    if (int ie = ensure_device(c)) return ie;
    hipStream_t s = pick_stream(c, stream);
    for (int i = 0; i < use && written < out_size; i++) {
        const size_t n = std::min(lens[i], out_size - written);
        if (n) HIP_TRY(hipMemcpyAsync(dst + written, shards[i], n, hipMemcpyDefault, s));
        written += n;
    }
    if (!stream) HIP_TRY(hipStreamSynchronize(s));
    return RS_OK;
}

int rs_set_host_segment(rs_codec *c, size_t bytes) {
    if (!c || bytes % 64) return RS_ERR_INVALID_ARG;
    std::lock_guard<std::mutex> lk(c->mu);
    c->host_seg_bytes = bytes;
    if (c->multi) return multi_set_host_segment(c->multi, bytes);
    return RS_OK;
}

int rs_set_reference_inversion_cache(rs_codec *c, int on) {
    if (!c) return RS_ERR_INVALID_ARG;
    std::lock_guard<std::mutex> lk(c->mu);
    c->ref_inv = on != 0;
    c->ref_inv_cache.clear();
    return RS_OK;
}

int rs_host_alloc(size_t bytes, void **out) {
    if (!out || bytes == 0) return RS_ERR_INVALID_ARG;
    *out = nullptr;
    HIP_TRY(hipHostMalloc(out, bytes, hipHostMallocPortable));
    return RS_OK;
}

void rs_host_free(void *p) {
    if (p) (void)hipHostFree(p);
}

int rs_host_register(void *p, size_t bytes) {
    if (!p || bytes == 0) return RS_ERR_INVALID_ARG;
    // mapped: the host reconstruct's zero-copy kernels address the rows through the device's view (zc_rows)
    HIP_TRY(hipHostRegister(p, bytes, hipHostRegisterPortable | hipHostRegisterMapped));
    return RS_OK;
}

int rs_host_unregister(void *p) {
    if (!p) return RS_ERR_INVALID_ARG;
    HIP_TRY(hipHostUnregister(p));
    return RS_OK;
}

int rs_encode_idx(rs_codec *c, const uint8_t *, size_t, int, uint8_t *const *, const size_t *, int) {
    return c ? RS_ERR_NOT_SUPPORTED : RS_ERR_INVALID_ARG;
}
int rs_update(rs_codec *c, uint8_t *const *, const size_t *, int, uint8_t *const *, const size_t *, int) {
    return c ? RS_ERR_NOT_SUPPORTED : RS_ERR_INVALID_ARG;
}

int rs_debug_field_tables(int bits, uint16_t *log_out, uint16_t *exp_out, uint16_t *skew_out, uint16_t *walsh_out) {
    if (bits != 8 && bits != 16) return RS_ERR_INVALID_ARG;
    const Field &F = field(bits);
    for (uint32_t i = 0; i < F.order; i++) {
        if (log_out) log_out[i] = F.log[i];
        if (exp_out) exp_out[i] = F.exp[i];
        if (walsh_out) walsh_out[i] = F.walsh[i];
        if (skew_out && i < F.mod) skew_out[i] = F.skew[i];
    }
    return RS_OK;
}

int rs_debug_twiddle_dwords(int bits) { return (bits == 8 || bits == 16) ? tw_dwords(bits) : 0; }

int rs_debug_sub_check(void) { return sub_coords().ok ? 0 : -1; }

int rs_debug_sub_twiddle(uint32_t log_m, uint32_t *out) {
    const Field &F = field(16);
    if (!out || log_m > F.mod || !in_subfield(F, log_m)) return -1;
    make_sub_twiddle(F, log_m, out);
    return 0;
}

uint32_t rs_debug_sub_swap(uint32_t x) { return sub_coords().to_sub(x & 0xFFFF); }

int rs_debug_twiddle(int bits, uint32_t log_m, uint32_t *out) {
    if ((bits != 8 && bits != 16) || !out) return RS_ERR_INVALID_ARG;
    const Field &F = field(bits);
    make_twiddle(F, log_m & F.mod, out);
    return RS_OK;
}

int rs_debug_error_locators(int bits, int k, int p, const uint8_t *erased, uint32_t *out) {
    if ((bits != 8 && bits != 16) || !erased || !out || k <= 0 || p <= 0) return RS_ERR_INVALID_ARG;
    std::vector<uint32_t> el;
    if (!error_locators(field(bits), k, p, erased, el)) return RS_ERR_PANIC;
    std::copy(el.begin(), el.end(), out);
    return RS_OK;
}

int rs_debug_split_emulate(rs_codec *c, const uint8_t *data, uint8_t *parity, size_t S) {
    if (!c || !data || !parity || S % 64 || c->bits != 16 || !c->enc_ok) return RS_ERR_INVALID_ARG;
    switch (c->logm) {
        case 2: return emu_split<2>(c, data, parity, S);
        case 3: return emu_split<3>(c, data, parity, S);
        case 4: return emu_split<4>(c, data, parity, S);
        case 5: return emu_split<5>(c, data, parity, S);
    }
    return RS_ERR_INVALID_ARG;
}

int rs_debug_split_check(int logm, uint32_t seed) {
    const Field &F = field(16);
    switch (logm) {
        case 2: return split_sim<2>(F, seed);
        case 3: return split_sim<3>(F, seed);
        case 4: return split_sim<4>(F, seed);
        case 5: return split_sim<5>(F, seed);
    }
    return -1;
}

int rs_debug_zc_rows(uint8_t *const *rows, int nrows, size_t S) {
    if (!rows || nrows < 0) return -1;
    std::vector<int> idx(nrows);
    for (int i = 0; i < nrows; i++) idx[i] = i;
    ZcRows z{};
    return zc_rows(rows, idx, S, z) ? 1 : 0;
}

int rs_debug_set_path(const char *knob, int value) {
    if (!knob) return RS_ERR_INVALID_ARG;
    const std::string k(knob);
    if (k == "bs") g_path_bs = value != 0;
    else if (k == "sub") g_path_sub = value != 0;
    else if (k == "prune") g_path_prune = value != 0;
    else if (k == "unit_width" && value >= -1 && value <= 1) g_path_unit_width = value;
    else if (k == "hp_tiles" && value >= 0 && value <= 64) g_path_hp_tiles = value;
    else if (k == "hp_step" && value >= 0) g_path_hp_step = value;
    else if (k == "hp_tune" && value >= 0 && value <= 1) g_path_hp_tune = value;
    else if (k == "rec_half" && value >= 0 && value <= 1) g_path_rec_half = value;
    else if (k == "dec_lab" && value >= 0 && value <= 255) g_path_dec_lab = value;
    else if (k == "lds_big" && value >= 0 && value <= 1) g_path_lds_big = value;
    else if (k == "zc" && value >= 0 && value <= 3) g_path_zc = value;
    else return RS_ERR_INVALID_ARG;
    return RS_OK;
}

const char *rs_strerror(int code) {
    switch (code) {
        case RS_OK: return "ok";
        case RS_ERR_INV_SHARD_NUM: return "invalid number of data shards";  // ErrInvShardNum
        case RS_ERR_MAX_SHARD_NUM: return "too many shards";
        case RS_ERR_TOO_FEW_SHARDS: return "too few shards given";
        case RS_ERR_SHARD_NO_DATA: return "no shard data";
        case RS_ERR_SHARD_SIZE: return "shard sizes do not match";
        case RS_ERR_INVALID_SHARD_SIZE: return "shard size is not a multiple of 64";
        case RS_ERR_NOT_SUPPORTED: return "operation not supported";
        case RS_ERR_SHORT_DATA: return "not enough data to fill the number of requested shards";
        case RS_ERR_RECONSTRUCT_REQUIRED: return "reconstruction required as one or more required data shards are nil";
        case RS_ERR_PANIC: return "the reference implementation panics for this geometry (index out of range)";
        case RS_ERR_NOMEM: return "out of memory";
        case RS_ERR_DEVICE: return "HIP device error";
        case RS_ERR_INVALID_ARG: return "invalid argument";
    }
    return "unknown error";
}

}  // extern "C"
