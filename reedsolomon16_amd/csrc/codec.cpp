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
#include <cstring>
#include <list>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/rs_mi355x.h"
#include "gf_host.hpp"
#include "kernels.hpp"

using namespace rs;

namespace {

constexpr int kMaxRegLogM = 5;  // m <= 32: fused register kernel

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
    std::string path;

    // decode plan (built on first reconstruct)
    bool dec_built = false, dec_ok = false;
    int n = 0, logn = 0;
    DevBuf<uint32_t> dtw_ifft, dtw_fft;

    // scratch
    DevBuf<uint8_t> work, slab;
    DevBuf<uint8_t *> rows;         // row-pointer table (non-strided inputs)
    std::vector<uint8_t *> rows_host;
    DevBuf<int> flag;
    DevBuf<const uint8_t *> rc_src;
    DevBuf<uint8_t *> rc_dst;
    DevBuf<uint32_t> rc_tw_in, rc_tw_out;
    DevBuf<int> rc_pos;

    // error-locator cache keyed by erasure pattern (bounded LRU)
    std::list<std::pair<std::vector<uint8_t>, std::vector<uint32_t>>> el_cache;

    ~rs_codec() {
        if (!dev_ready && !stream) return;
        DeviceGuard g(device);
        if (stream) (void)hipStreamSynchronize(stream);
        tw_ifft.release(); tw_fft.release(); dtw_ifft.release(); dtw_fft.release();
        work.release(); slab.release(); rows.release(); flag.release();
        rc_src.release(); rc_dst.release(); rc_tw_in.release(); rc_tw_out.release(); rc_pos.release();
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

// Host half of the encode plan (no device calls): twiddle schedule and panic check.
void plan_encode_host(rs_codec *c) {
    c->enc_ok = encode_schedule(*c->F, c->k, c->p, c->enc_ifft_logs, c->enc_fft_logs, c->nchunks);
    c->path = !c->enc_ok ? "panic" : (c->logm <= kMaxRegLogM ? encode_reg_name(c->bits, c->logm) : "multipass");
}

// Device half, on first use: stream, flag word, encode twiddle tables.
int ensure_device(rs_codec *c) {
    if (c->dev_ready) return RS_OK;
    if (!c->stream) HIP_TRY(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    HIP_TRY(c->flag.ensure(1));
    if (c->enc_ok) {
        int e = upload_twiddles(c, c->enc_ifft_logs, c->tw_ifft);
        if (e) return e;
        e = upload_twiddles(c, c->enc_fft_logs, c->tw_fft);
        if (e) return e;
    }
    c->dev_ready = true;
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
    int e = upload_twiddles(c, il, c->dtw_ifft);
    if (e) return e;
    return upload_twiddles(c, fl, c->dtw_fft);
}

hipStream_t pick_stream(rs_codec *c, void *s) { return s ? (hipStream_t)s : c->stream; }

// Data rows [0,k) and parity rows [k,k+p) as RowSets: strided when the
// pointers are equally spaced (AllocAligned slab), else via a device table.
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
        HIP_TRY(hipStreamSynchronize(s));  // previous users of the table are done
        HIP_TRY(c->rows.ensure(c->total));
        HIP_TRY(hipMemcpy(c->rows.p, tbl.data(), c->total * sizeof(uint8_t *), hipMemcpyHostToDevice));
        c->rows_host = tbl;
    }
    if (!ok_d) data = RowSet{c->rows.p, nullptr, 0};
    if (!ok_p) par = RowSet{c->rows.p + c->k, nullptr, 0};
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
    HIP_TRY(c->work.ensure((size_t)2 * m * S));
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
        HIP_TRY(launch_encode_reg(c->bits, c->logm, mismatch != nullptr, a, s));
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

// Device reconstruct (leopard16.go:432-568) for already-validated input.
int reconstruct_device(rs_codec *c, uint8_t *const *d, const std::vector<uint8_t> &present, uint64_t S,
                       bool recover_all, hipStream_t s) {
    int e = build_decode_plan(c);
    if (e) return e;
    if (!c->dec_ok) return RS_ERR_PANIC;
    const int k = c->k, p = c->p, m = c->m, n = c->n, total = c->total;
    std::vector<uint8_t> erased(total);
    for (int i = 0; i < total; i++) erased[i] = !present[i];
    const std::vector<uint32_t> *elp = error_locs_cached(c, erased);
    if (!elp) return RS_ERR_PANIC;
    const std::vector<uint32_t> &el = *elp;

    // work rows: [recovery m][original k][zero to n] (leopard16.go:547)
    std::vector<const uint8_t *> src(n, nullptr);
    std::vector<uint32_t> tw_in((size_t)n * c->twd, 0);
    for (int i = 0; i < p; i++)
        if (present[k + i]) src[i] = d[k + i];
    for (int i = 0; i < k; i++)
        if (present[i]) src[m + i] = d[i];
    for (int r = 0; r < m + k; r++)
        if (src[r]) make_twiddle(*c->F, el[r], tw_in.data() + (size_t)r * c->twd);

    std::vector<uint8_t *> dst;
    std::vector<int> pos;
    const int end = recover_all ? total : k;
    for (int i = 0; i < end; i++) {
        if (present[i]) continue;
        dst.push_back(d[i]);
        pos.push_back(i >= k ? i - k : i + m);
    }
    std::vector<uint32_t> tw_out(std::max<size_t>(dst.size(), 1) * c->twd, 0);
    for (size_t j = 0; j < dst.size(); j++)
        make_twiddle(*c->F, (c->F->mod - el[pos[j]]) & c->F->mod, tw_out.data() + j * c->twd);

    HIP_TRY(c->work.ensure((size_t)n * S));
    HIP_TRY(c->rc_src.ensure(n));
    HIP_TRY(c->rc_tw_in.ensure(tw_in.size()));
    HIP_TRY(c->rc_dst.ensure(std::max<size_t>(dst.size(), 1)));
    HIP_TRY(c->rc_pos.ensure(std::max<size_t>(pos.size(), 1)));
    HIP_TRY(c->rc_tw_out.ensure(tw_out.size()));
    HIP_TRY(hipMemcpyAsync(c->rc_src.p, src.data(), n * sizeof(void *), hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(c->rc_tw_in.p, tw_in.data(), tw_in.size() * 4, hipMemcpyHostToDevice, s));
    if (!dst.empty()) {
        HIP_TRY(hipMemcpyAsync(c->rc_dst.p, dst.data(), dst.size() * sizeof(void *), hipMemcpyHostToDevice, s));
        HIP_TRY(hipMemcpyAsync(c->rc_pos.p, pos.data(), pos.size() * sizeof(int), hipMemcpyHostToDevice, s));
        HIP_TRY(hipMemcpyAsync(c->rc_tw_out.p, tw_out.data(), tw_out.size() * 4, hipMemcpyHostToDevice, s));
    }
    uint8_t *w = c->work.p;
    HIP_TRY(launch_scale_in(c->bits, w, S, c->rc_src.p, c->rc_tw_in.p, n, s));
    e = run_passes(c, true, w, S, c->logn, m + k, c->dtw_ifft.p, s);
    if (e) return e;
    HIP_TRY(launch_formal_derivative(c->bits, w, S, n, s));
    e = run_passes(c, false, w, S, c->logn, m + k, c->dtw_fft.p, s);
    if (e) return e;
    if (!dst.empty())
        HIP_TRY(launch_reveal(c->bits, c->rc_dst.p, w, S, c->rc_pos.p, c->rc_tw_out.p, (int)dst.size(), s));
    HIP_TRY(hipStreamSynchronize(s));  // host vectors above must outlive the async copies
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

int ensure_slab(rs_codec *c, uint64_t S, uint8_t **d) {
    HIP_TRY(c->slab.ensure((size_t)c->total * S));
    for (int i = 0; i < c->total; i++) d[i] = c->slab.p + (size_t)i * S;
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

int rs_field_bits(const rs_codec *c) { return c ? c->bits : 0; }
int rs_data_shards(const rs_codec *c) { return c ? c->k : 0; }
int rs_parity_shards(const rs_codec *c) { return c ? c->p : 0; }
int rs_total_shards(const rs_codec *c) { return c ? c->total : 0; }
int rs_shard_size_multiple(const rs_codec *c) { return c ? 64 : 0; }
const char *rs_encode_path(const rs_codec *c) { return c ? c->path.c_str() : ""; }

int rs_encode_dev(rs_codec *c, uint8_t *const *d, size_t S, void *stream) {
    if (!c || !d) return RS_ERR_INVALID_ARG;
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
    e = encode_device(c, data, par, S, 0, 1, nullptr, s);
    if (e) return e;
    if (!stream) HIP_TRY(hipStreamSynchronize(s));
    return RS_OK;
}

int rs_encode_dev_batch(rs_codec *c, uint8_t *base, size_t row_stride, size_t stripe_stride, int nstripes, size_t S,
                        void *stream) {
    if (!c || !base || nstripes <= 0) return RS_ERR_INVALID_ARG;
    if (S == 0) return RS_ERR_SHARD_NO_DATA;
    if (S % 64) return RS_ERR_INVALID_SHARD_SIZE;
    std::lock_guard<std::mutex> lk(c->mu);
    DeviceGuard g(c->device);
    if (int ie = ensure_device(c)) return ie;
    hipStream_t s = pick_stream(c, stream);
    RowSet data{nullptr, base, row_stride}, par{nullptr, base + (size_t)c->k * row_stride, row_stride};
    int e = encode_device(c, data, par, S, stripe_stride, nstripes, nullptr, s);
    if (e) return e;
    if (!stream) HIP_TRY(hipStreamSynchronize(s));
    return RS_OK;
}

int rs_verify_dev(rs_codec *c, uint8_t *const *d, size_t S, int *ok, void *stream) {
    if (!c || !d || !ok) return RS_ERR_INVALID_ARG;
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
    HIP_TRY(hipMemsetAsync(c->flag.p, 0, sizeof(int), s));
    e = encode_device(c, data, par, S, 0, 1, c->flag.p, s);
    if (e) return e;
    int h = 1;
    HIP_TRY(hipMemcpyAsync(&h, c->flag.p, sizeof(int), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    *ok = h == 0;
    return RS_OK;
}

int rs_reconstruct_dev(rs_codec *c, uint8_t *const *d, const uint8_t *present, size_t S, int recover_all,
                       void *stream) {
    if (!c || !d || !present) return RS_ERR_INVALID_ARG;
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
    return reconstruct_device(c, d, pr, S, recover_all != 0, pick_stream(c, stream));
}

int rs_encode(rs_codec *c, uint8_t *const *shards, const size_t *lens, int nshards) {
    if (!c || !shards || !lens) return RS_ERR_INVALID_ARG;
    if (nshards != c->total) return RS_ERR_TOO_FEW_SHARDS;
    int e = check_shards(lens, nshards, false);
    if (e) return e;
    const uint64_t S = shard_size_of(lens, nshards);
    if (S % 64) return RS_ERR_INVALID_SHARD_SIZE;
    if (!c->enc_ok) return RS_ERR_PANIC;
    std::lock_guard<std::mutex> lk(c->mu);
    DeviceGuard g(c->device);
    if (int ie = ensure_device(c)) return ie;
    hipStream_t s = c->stream;
    std::vector<uint8_t *> d(c->total);
    e = ensure_slab(c, S, d.data());
    if (e) return e;
    for (int i = 0; i < c->k; i++) HIP_TRY(hipMemcpyAsync(d[i], shards[i], S, hipMemcpyHostToDevice, s));
    RowSet data{nullptr, d[0], S}, par{nullptr, d[c->k], S};
    e = encode_device(c, data, par, S, 0, 1, nullptr, s);
    if (e) return e;
    for (int i = 0; i < c->p; i++)
        HIP_TRY(hipMemcpyAsync(shards[c->k + i], d[c->k + i], S, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
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
    std::lock_guard<std::mutex> lk(c->mu);
    DeviceGuard g(c->device);
    if (int ie = ensure_device(c)) return ie;
    hipStream_t s = c->stream;
    std::vector<uint8_t *> d(c->total);
    e = ensure_slab(c, S, d.data());
    if (e) return e;
    for (int i = 0; i < c->total; i++) HIP_TRY(hipMemcpyAsync(d[i], shards[i], S, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemsetAsync(c->flag.p, 0, sizeof(int), s));
    RowSet data{nullptr, d[0], S}, par{nullptr, d[c->k], S};
    e = encode_device(c, data, par, S, 0, 1, c->flag.p, s);
    if (e) return e;
    int h = 1;
    HIP_TRY(hipMemcpyAsync(&h, c->flag.p, sizeof(int), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    *ok = h == 0;
    return RS_OK;
}

int rs_reconstruct(rs_codec *c, uint8_t *const *shards, size_t *lens, int nshards, int recover_all) {
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
    for (int i = 0; i < end; i++)
        if (!lens[i] && !shards[i]) return RS_ERR_INVALID_ARG;
    std::lock_guard<std::mutex> lk(c->mu);
    DeviceGuard g(c->device);
    if (int ie = ensure_device(c)) return ie;
    hipStream_t s = c->stream;
    std::vector<uint8_t *> d(c->total);
    e = ensure_slab(c, S, d.data());
    if (e) return e;
    std::vector<uint8_t> pr(c->total);
    for (int i = 0; i < c->total; i++) {
        pr[i] = lens[i] != 0;
        if (pr[i]) HIP_TRY(hipMemcpyAsync(d[i], shards[i], S, hipMemcpyHostToDevice, s));
    }
    e = reconstruct_device(c, d.data(), pr, S, recover_all != 0, s);
    if (e) return e;
    for (int i = 0; i < end; i++) {
        if (pr[i]) continue;
        HIP_TRY(hipMemcpyAsync(shards[i], d[i], S, hipMemcpyDeviceToHost, s));
        lens[i] = S;
    }
    HIP_TRY(hipStreamSynchronize(s));
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
