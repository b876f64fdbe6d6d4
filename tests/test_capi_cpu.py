"""CPU tests of the product library's C-ABI (no device calls): it loads,
exports every function include/rs_mi355x.h declares, builds the same field
tables as the oracle, its byte-permute twiddle images multiply correctly
(emulating v_perm_b32 in numpy), its error locators match, and argument
validation mirrors the reference's error behaviour."""
import ctypes as C

import numpy as np
import pytest

import reedsolomon16_amd as rs
from oracle import leopard_np as lnp
from oracle import orc
from reedsolomon16_amd import _capi


def test_library_exports_header():
    L = rs.lib()
    names = _capi.header_functions()
    assert len(names) >= 20
    for n in names:
        assert hasattr(L, n), n


def test_error_codes_match_oracle_numbering():
    text = open(_capi.HEADER_PATH).read()
    want = {"RS_ERR_INV_SHARD_NUM": 1, "RS_ERR_MAX_SHARD_NUM": 2, "RS_ERR_TOO_FEW_SHARDS": 3,
            "RS_ERR_SHARD_NO_DATA": 4, "RS_ERR_SHARD_SIZE": 5, "RS_ERR_INVALID_SHARD_SIZE": 6,
            "RS_ERR_NOT_SUPPORTED": 7, "RS_ERR_PANIC": 50}
    for k, v in want.items():
        assert f"#define {k}" in text and str(v) in text.split(f"#define {k}")[1].split("\n")[0]


@pytest.mark.parametrize("bits", [16, 8])
def test_engine_tables_match_oracle(bits):
    n = 1 << bits
    bufs = [np.zeros(n, np.uint16), np.zeros(n, np.uint16), np.zeros(n - 1, np.uint16), np.zeros(n, np.uint16)]
    assert rs.lib().rs_debug_field_tables(bits, *[b.ctypes.data for b in bufs]) == 0
    ref = orc.tables16() if bits == 16 else orc.tables8()
    for a, b in zip(bufs, ref):
        assert np.array_equal(a.astype(np.int64), b.astype(np.int64))


def vperm(s0, s1, sel):
    """numpy model of v_perm_b32 (selector bytes 0..7 pick from {s0:s1}, s1 low)."""
    data = (np.uint64(s0) << np.uint64(32)) | np.uint64(s1)
    out = np.zeros_like(sel, dtype=np.uint32)
    for b in range(4):
        idx = (sel >> np.uint32(8 * b)) & np.uint32(0xFF)
        assert np.all(idx < 8)
        byte = (data >> (idx.astype(np.uint64) * np.uint64(8))) & np.uint64(0xFF)
        out |= byte.astype(np.uint32) << np.uint32(8 * b)
    return out


def twiddle(bits, log_m):
    L = rs.lib()
    n = L.rs_debug_twiddle_dwords(bits)
    t = np.zeros(n, np.uint32)
    assert L.rs_debug_twiddle(bits, log_m, t.ctypes.data) == 0
    return [np.uint32(x) for x in t]


def emulate_mul16(lo, hi, t):
    """The kernel's F16::mul_add on (lo, hi) dwords with x = 0."""
    m7, m3 = np.uint32(0x07070707), np.uint32(0x03030303)
    a0, a1, a2 = lo & m7, (lo >> np.uint32(3)) & m7, (lo >> np.uint32(6)) & m3
    b0, b1, b2 = hi & m7, (hi >> np.uint32(3)) & m7, (hi >> np.uint32(6)) & m3
    pl = vperm(t[1], t[0], a0) ^ vperm(t[5], t[4], a1) ^ vperm(t[8], t[8], a2) ^ vperm(t[11], t[10], b0) ^ \
        vperm(t[15], t[14], b1) ^ vperm(t[18], t[18], b2)
    ph = vperm(t[3], t[2], a0) ^ vperm(t[7], t[6], a1) ^ vperm(t[9], t[9], a2) ^ vperm(t[13], t[12], b0) ^ \
        vperm(t[17], t[16], b1) ^ vperm(t[19], t[19], b2)
    return pl, ph


def test_twiddle_image_multiplies_gf16():
    rng = np.random.default_rng(3)
    F = lnp.field(16)
    rows = rng.integers(0, 256, (1, 64 * 8), dtype=np.uint8)
    sym = lnp.to_symbols(rows, 16)[0]
    blk = rows.reshape(-1, 64)
    lo = blk[:, :32].copy().view(np.uint32).ravel()
    hi = blk[:, 32:].copy().view(np.uint32).ravel()
    for log_m in list(rng.integers(0, 65535, 30)) + [0, 1, 65534, 65535]:
        pl, ph = emulate_mul16(lo, hi, twiddle(16, int(log_m)))
        got_blk = np.concatenate([pl.reshape(-1, 8).view(np.uint8), ph.reshape(-1, 8).view(np.uint8)], axis=1)
        want = lnp.from_symbols(F.mul_log(sym, int(log_m))[None], 16)[0]
        assert np.array_equal(got_blk.ravel(), want), log_m


def test_twiddle_image_multiplies_gf8():
    rng = np.random.default_rng(4)
    F = lnp.field(8)
    data = rng.integers(0, 256, 256, dtype=np.uint8)
    d = data.view(np.uint32)
    m7, m3 = np.uint32(0x07070707), np.uint32(0x03030303)
    for log_m in range(256):
        t = twiddle(8, log_m)
        p = vperm(t[1], t[0], d & m7) ^ vperm(t[3], t[2], (d >> np.uint32(3)) & m7) ^ \
            vperm(t[4], t[4], (d >> np.uint32(6)) & m3)
        assert np.array_equal(p.view(np.uint8), F.mul_log(data.astype(np.int64), log_m).astype(np.uint8))


@pytest.mark.parametrize("bits,k,p", [(16, 10, 4), (16, 128, 32), (16, 1000, 300), (8, 10, 4), (8, 100, 28)])
def test_error_locators_match_numpy(bits, k, p):
    rng = np.random.default_rng(k)
    for _ in range(3):
        erased = np.zeros(k + p, np.uint8)
        erased[rng.choice(k + p, p, replace=False)] = 1
        out = np.zeros(1 << bits, np.uint32)
        assert rs.lib().rs_debug_error_locators(bits, k, p, erased.ctypes.data, out.ctypes.data) == 0
        assert np.array_equal(out.astype(np.int64), lnp.error_locators(bits, k, p, erased.astype(bool)))


def test_error_locators_panic_where_reference_panics():
    erased = np.zeros(240, np.uint8)
    out = np.zeros(256, np.uint32)
    assert rs.lib().rs_debug_error_locators(8, 200, 40, erased.ctypes.data, out.ctypes.data) == 50


def test_constructor_errors():
    with pytest.raises(rs.ErrInvShardNum):
        rs.New16(0, 4)
    with pytest.raises(rs.ErrInvShardNum):
        rs.New8(4, 0)
    with pytest.raises(rs.ErrMaxShardNum):
        rs.New16(60000, 6000)
    c = rs.New(10, 4)
    assert c.field_bits == 8 and c.total_shards() == 14 and c.shard_size_multiple() == 64
    assert rs.New(200, 100).field_bits == 16
    # bit-sliced kernel: one table per m covers every k <= chunks * m, 9 <= p <= 32
    assert rs.New16(128, 32).encode_path == "bs16-m32"
    assert rs.New16(130, 32).encode_path == "bs16-m32"
    assert rs.New16(192, 17).encode_path == "bs16-m32"
    assert rs.New16(64, 16).encode_path == "bs16-m16"
    assert rs.New16(192, 9).encode_path == "bs16-m16"
    assert rs.New16(193, 32).encode_path == "split16-m32"  # 7 chunks: past the m = 32 table
    assert rs.New16(193, 16).encode_path == "split16-m16"  # 13 chunks: past the m = 16 table
    assert rs.New16(64, 8).encode_path == "split16-m8"
    assert rs.New16(10, 1).encode_path == "reg16-m1"
    assert rs.New16(1024, 256).encode_path == "lds-m256"
    assert rs.New16(96, 100).encode_path == "lds-m128"
    # m = 512 .. 4096 (GF(2^16)): the LDS encode (64-byte tiles, half tiles at 2048, quarter
    # tiles at 4096); m = 8192: multi-pass
    assert rs.New16(1024, 300).encode_path == "lds-m512"
    assert rs.New16(4000, 1000).encode_path == "lds-m1024"
    assert rs.New16(3000, 1025).encode_path == "lds-m2048"
    assert rs.New16(3000, 2049).encode_path == "lds-m4096"
    assert rs.New16(1000, 5000).encode_path == "multipass"


def test_debug_set_path_knobs(paths):
    """rs_debug_set_path: the test-only kernel-path overrides (no environment
    variable reaches the product library)."""
    paths("bs", 0)
    assert rs.New16(128, 32).encode_path == "split16-m32"
    paths("bs", 1)
    assert rs.New16(128, 32).encode_path == "bs16-m32"
    for knob, value in (("sub", 0), ("prune", 0), ("unit_width", 1), ("unit_width", 0), ("unit_width", -1), ("zc", 0)):
        paths(knob, value)
    with pytest.raises(ValueError):
        paths("unit_width", 2)
    with pytest.raises(ValueError):
        paths("RS_BS", 0)


def test_host_validation_errors_without_device():
    """Validation happens before any device work (Encode leopard16.go:116-135,
    reconstruct :390-430)."""
    c = rs.New16(10, 4)
    S = 128
    good = [np.zeros(S, np.uint8) for _ in range(14)]
    with pytest.raises(rs.ErrTooFewShards):
        c.encode(good[:13])
    with pytest.raises(rs.ErrShardSize):
        c.encode(good[:13] + [np.zeros(64, np.uint8)])
    with pytest.raises(rs.ErrShardSize):
        c.encode(good[:13] + [None])
    with pytest.raises(rs.ErrInvalidShardSize):
        c.encode([np.zeros(100, np.uint8) for _ in range(14)])
    with pytest.raises(rs.ErrShardNoData):
        c.encode([None] * 14)
    with pytest.raises(rs.ErrTooFewShards):
        c.reconstruct([None] * 5 + good[5:])
    with pytest.raises(rs.ErrShardNoData):
        c.reconstruct([None] * 14)
    with pytest.raises(rs.ErrShardSize):
        c.reconstruct([np.zeros(64, np.uint8)] + good[1:])
    # nothing missing: no-op, no device needed
    assert c.reconstruct([g.copy() for g in good]) is not None
    with pytest.raises(rs.ErrNotSupported):
        c.encode_idx(good[0], 0, good[10:])
    with pytest.raises(rs.ErrNotSupported):
        c.update(good, good[:10])


def test_encode_panic_geometry_without_device():
    c = rs.New8(129, 127)
    assert c.encode_path == "panic"
    with pytest.raises(rs.ErrPanic):
        c.encode([np.zeros(64, np.uint8) for _ in range(256)])


def test_split_join_mirror_reference():
    """Split/Join (leopard16.go:232-340) as used by testEncodeDecode."""
    import io

    c = rs.New16(4, 2)
    data = (np.arange(1000) % 251).astype(np.uint8)
    shards = c.split(data)
    assert len(shards) == 6 and all(len(s) == 256 for s in shards)
    buf = io.BytesIO()
    c.join(buf, shards, len(data))
    assert buf.getvalue() == bytes(data)
    with pytest.raises(rs.ErrShortData):
        c.split(b"")
    with pytest.raises(rs.ErrReconstructRequired):
        c.join(io.BytesIO(), [None] + shards[1:], 10)
    with pytest.raises(rs.ErrShortData):
        c.join(io.BytesIO(), shards, 4 * 256 + 1)
    with pytest.raises(rs.ErrTooFewShards):
        c.join(io.BytesIO(), shards[:3], 10)
    # a zero-length (non-nil) data shard counts 0 bytes (leopard16.go:239-250):
    # the join reads on into the next shards, or is short
    empty = np.zeros(0, np.uint8)
    buf = io.BytesIO()
    c.join(buf, [shards[0], empty] + shards[2:], 3 * 256)
    assert buf.getvalue() == bytes(shards[0]) + bytes(shards[2]) + bytes(shards[3])
    with pytest.raises(rs.ErrShortData):
        c.join(io.BytesIO(), [shards[0], empty] + shards[2:], 3 * 256 + 1)


@pytest.mark.parametrize("logm", [2, 3, 4, 5])
def test_split_schedule_equals_plain_transform(logm):
    """The split kernel's compile-time schedules (schedule.hpp) compute the
    same IFFT / FFT as the reference butterfly order, simulated on the host."""
    for seed in (1, 2, 3):
        assert rs.lib().rs_debug_split_check(logm, seed) == 0
    assert rs.lib().rs_debug_split_check(6, 1) == -1


@pytest.mark.parametrize("k,p,S", [(10, 4, 1024), (10, 6, 128), (3, 7, 64), (37, 9, 64), (33, 17, 128), (128, 32, 256),
                                   (130, 32, 64)])
def test_split_kernel_emulation_matches_oracle(k, p, S):
    """Bit-level host emulation of the split kernel (images, v_perm multiply,
    half-wave swaps) against the oracle."""
    rng = np.random.default_rng(k * 31 + p)
    data = rng.integers(0, 256, (k, S), dtype=np.uint8)
    ref = orc.encode(16, k, p, data)
    c = rs.New16(k, p)
    out = np.zeros((p, S), np.uint8)
    assert rs.lib().rs_debug_split_emulate(c._h, data.ctypes.data, out.ctypes.data, S) == 0
    assert np.array_equal(out, ref)


def test_subfield_coordinates():
    """GF(2^8) inside GF(2^16): products of Cantor-basis integers < 256 stay
    below 256, every fftSkew entry below index 255 is such an element, and in
    the engine's coordinates (lo ^ D(hi), hi) the 8-dword subfield table
    (emulated v_perm_b32 on both bytes) multiplies exactly like the field."""
    F = lnp.field(16)
    a = np.arange(1, 256)
    for b in range(1, 256):
        assert (F.mul_log(a, int(F._log[b])) < 256).all()
    sk = F._skew[:255]
    assert ((sk == 65535) | (F._exp[sk] < 256)).all()
    L = rs.lib()
    assert L.rs_debug_sub_check() == 0
    rng = np.random.default_rng(9)
    x = rng.integers(0, 65536, 512).astype(np.int64)
    y = np.array([L.rs_debug_sub_swap(int(v)) for v in x], np.int64)
    assert np.array_equal(np.array([L.rs_debug_sub_swap(int(v)) for v in y], np.int64), x)
    m7, m3 = np.uint32(0x07070707), np.uint32(0x03030303)

    def sub_mul(t, bytes_):
        d = np.ascontiguousarray(bytes_.astype(np.uint8)).view(np.uint32)
        p = vperm(t[1], t[0], d & m7) ^ vperm(t[3], t[2], (d >> np.uint32(3)) & m7) ^ \
            vperm(t[4], t[4], (d >> np.uint32(6)) & m3)
        return p.view(np.uint8).astype(np.int64)

    t = np.zeros(8, np.uint32)
    for e in (1, 2, 3, 77, 200, 255):
        log_m = int(F._log[e])
        assert L.rs_debug_sub_twiddle(log_m, t.ctypes.data) == 0
        tt = [np.uint32(v) for v in t]
        z = sub_mul(tt, y & 0xFF) | (sub_mul(tt, y >> 8) << 8)
        back = np.array([L.rs_debug_sub_swap(int(v)) for v in z], np.int64)
        assert np.array_equal(back, F.mul_log(x, log_m)), e
    assert L.rs_debug_sub_twiddle(65535, t.ctypes.data) == 0 and not t[:5].any()
    assert L.rs_debug_sub_twiddle(int(F._log[300]), t.ctypes.data) == -1


@pytest.mark.parametrize("k,p,n", [(4, 2, 1), (4, 2, 63), (4, 2, 256), (4, 2, 1025), (10, 4, 64 * 10), (10, 4, 64 * 10 + 1),
                                   (128, 32, 1 << 16), (3, 1, 7)])
def test_split_c_abi_matches_go_model(k, p, n):
    """rs_split (host slab) against a transcription of leopard16.go:277-340:
    perShard = roundup64(ceil(n / k)); data rows hold the bytes, then zeros;
    parity rows zero."""
    c = rs.New16(k, p)
    data = np.random.default_rng(n + k).integers(0, 256, n, dtype=np.uint8)
    per = -(-n // k)
    per = -(-per // 64) * 64
    assert c.split_shard_size(n) == per
    want = np.zeros((k + p) * per, np.uint8)
    want[:n] = data
    got = c.split(data)
    assert len(got) == k + p and all(len(s) == per for s in got)
    assert np.array_equal(np.concatenate(got), want)
    import io

    buf = io.BytesIO()
    c.join(buf, got, n)
    assert buf.getvalue() == data.tobytes()


def _dec_plan(mtrunc, need):
    import ctypes as C

    L = rs._capi.lib()
    nd = (C.c_uint32 * 8)(*need)
    code = (C.c_uint64 * 3)()
    assert L.rs_debug_dec_plan(mtrunc, nd, code) == 0
    waves = []
    for w in range(12):
        c = (code[w // 4] >> (16 * (w % 4))) & 0xFFFF
        waves.append([((c >> (4 * f)) & 15) - 1 for f in range(4)])  # u3a, u3b, u1a, u1b
    return waves


@pytest.mark.parametrize("mtrunc", [160, 152, 129, 100, 33])
def test_bsdec_plan_covers_every_unit(mtrunc):
    """The bit-sliced decoder's host plan (bitslice_dec.hip make_plan): every
    16-row unit gets exactly one phase-1 slot, the units with a revealed row
    exactly one phase-3 slot, waves >= 8 (which run phase 1 during phase 2)
    hold no phase-3 unit, waves < 8 at most one phase-1 unit (the kernel's late
    path runs only the first), and the last iteration's remap (waves 8..11 take
    the second phase-3 unit of waves 0..3) still covers every phase-3 unit."""
    rng = np.random.default_rng(mtrunc)
    cases = [0, (1 << 10) - 1, 1, 1 << 9, 0b1010101010] + [int(x) for x in rng.integers(0, 1 << 10, 60)]
    units = (mtrunc + 15) // 16
    for mask in cases:
        need = [0] * 8
        rev = set()
        for u in range(units):
            if (mask >> u) & 1:
                r = min(16 * u + int(rng.integers(0, 16)), mtrunc - 1)
                need[r >> 5] |= 1 << (r & 31)
                rev.add(r // 16)
        waves = _dec_plan(mtrunc, need)
        p1 = sorted(u for w in waves for u in w[2:] if u >= 0)
        assert p1 == list(range(10)), (mask, waves)
        p3 = sorted(u for w in waves for u in w[:2] if u >= 0)
        assert p3 == sorted(rev), (mask, waves)
        for w, (u3a, u3b, u1a, u1b) in enumerate(waves):
            assert u3b < 0 or u3a >= 0
            assert u1b < 0 or u1a >= 0
            if w >= 8:
                assert u3a < 0 and u3b < 0
            else:
                assert u1b < 0
        last = [u for w in range(8) for u in (waves[w][:1] if w < 4 else waves[w][:2]) if u >= 0]
        last += [waves[w - 8][1] for w in range(8, 12) if waves[w - 8][1] >= 0]
        assert sorted(last) == sorted(rev)
