"""CPU checks of what the bit-sliced encode kernel (csrc/bitslice.hip) is
built from, no device calls:

* its 64-byte block <-> bit-plane transpose (three delta-swap stages per
  8-dword half, restated in numpy) puts bit b of symbol 4w+j at bit 8j+w of
  plane b, and is an involution;
* the per-m twiddle tables tools/gen_bs_tables.cpp writes into
  build/bs_tables.h (HpTab<LOGM>: 8x8 matrices in subfield coordinates, one
  table per m for every k and p), applied in the half-plane kernel's order
  (k_encode_hp: IFFT layers r0..r(LR-1) per row group, r(LR), r(LR+1) per
  coset, XOR-accumulate, FFT layers r(LR+1), r(LR) per coset, then
  r(LR-1)..r0 per row group) with its slot indexing (bitslice.hip
  ifft_slot / fft_slot, restated here), give the oracle's parity bit for bit
  (leopard16.go:128-224) for m = 16 and 32 and ragged k and p;
* the logs behind the matrices equal the geometry's own schedule wherever
  the reference does not truncate (the host check the codec runs).
"""
import os
import re

import numpy as np
import pytest

from oracle import orc

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "reedsolomon16_amd", "build", "bs_tables.h")
MASKS = (0x55555555, 0x33333333, 0x0F0F0F0F)


def bs_transpose(w):
    """bitslice.hip bs_transpose on 16 uint32 arrays."""
    w = [x.copy() for x in w]
    for h in (0, 8):
        for k, m in enumerate(MASKS):
            s, M = np.uint32(1 << k), np.uint32(m)
            for a in range(8):
                if a & (1 << k):
                    continue
                x, y = w[h + a], w[h + a + (1 << k)]
                w[h + a] = (x & M) | ((y << s) & ~M)
                w[h + a + (1 << k)] = (y & ~M) | ((x >> s) & M)
    return w


def test_transpose_layout_and_involution():
    rng = np.random.default_rng(1)
    blk = rng.integers(0, 256, (200, 64), dtype=np.uint8)
    words = blk.view("<u4")
    planes = bs_transpose([words[:, i].copy() for i in range(16)])
    sym = blk[:, :32].astype(np.uint32) | (blk[:, 32:].astype(np.uint32) << 8)
    for b in range(16):
        for w in range(8):
            for j in range(4):
                want = (sym[:, 4 * w + j] >> b) & 1
                got = (planes[b] >> np.uint32(8 * j + w)) & 1
                assert np.array_equal(got, want), (b, w, j)
    back = bs_transpose(planes)
    for i in range(16):
        assert np.array_equal(back[i], words[:, i])


def load_tables():
    if not os.path.exists(HDR):
        pytest.skip("build/bs_tables.h not generated (run __graft_entry__.build())")
    txt = open(HDR).read()
    out = {}
    for m in re.finditer(r"struct HpTab<(\d+)> \{(.*?)\n\};", txt, re.S):
        logm, body = int(m.group(1)), m.group(2)

        def num(name):
            return int(re.search(r"\b" + name + r" = (\d+)", body).group(1))

        def arr(name):
            blk = re.search(r"\b" + name + r"\[[^=]*= *(\{.*?\});", body, re.S).group(1)
            return np.array([int(x) for x in re.findall(r"\d+", blk)], np.uint64)

        nch, IS, FS = num("NCH"), num("IS"), num("FS")
        out[logm] = dict(nch=nch, dmat=arr("dmat").astype(np.uint32),
                         ifft8=arr("ifft8").astype(np.uint32).reshape(nch, IS, 8),
                         fft8=arr("fft8").astype(np.uint32).reshape(FS, 8),
                         ifft_log=arr("ifft_log").reshape(nch, IS), fft_log=arr("fft_log").reshape(FS))
    assert out, "no table in bs_tables.h"
    return out


def test_header_holds_makefile_tables():
    mk = open(os.path.join(ROOT, "reedsolomon16_amd", "Makefile")).read()
    req = dict(tuple(int(x) for x in c.split(":")) for c in re.search(r"BS_CHUNKS \?= (.*)", mk).group(1).split())
    tabs = load_tables()
    assert set(tabs) == set(req) == {4, 5}
    for logm, cap in req.items():
        assert tabs[logm]["nch"] == cap, "every requested chunk lies in the subfield"


def gf2_apply(rows, y):
    """Output bit i = parity(y & rows[i]) (the kernel's XOR network, per symbol)."""
    out = np.zeros_like(y)
    for i in range(16):
        out |= (np.bitwise_count(y & rows[i]) & 1).astype(np.uint32) << np.uint32(i)
    return out


def to_sub(dmat, sym):
    """Planes r < 8 ^= XOR of planes 8+i over the bits i of dmat[r] (an involution)."""
    out = sym.copy()
    hi = sym >> np.uint32(8)
    for r in range(8):
        out ^= (np.bitwise_count(hi & np.uint32(dmat[r])) & 1).astype(np.uint32) << np.uint32(r)
    return out


def widen(t):
    """8x8 rows -> the block-diagonal 16x16 rows (one map per byte half)."""
    return (t | (t << np.uint32(8)))[..., list(range(8)) * 2] & np.concatenate(
        [np.full(8, 0xFF, np.uint32), np.full(8, 0xFF00, np.uint32)])


def ifft_slot(logm, layer, row):
    """bitslice.hip ifft_slot (gf_host.cpp ifft_passes slot order)."""
    off, dist = 0, 1
    while dist * 4 <= (1 << logm):
        l0 = dist.bit_length() - 1
        g = row // (4 * dist)
        if layer == l0 + 1:
            return off + 3 * g + 1
        if layer == l0:
            return off + 3 * g + (2 if (row // dist) & 2 else 0)
        off += 3 * ((1 << logm) // (4 * dist))
        dist *= 4
    return off


def fft_slot(logm, layer, row):
    """bitslice.hip fft_slot (gf_host.cpp fft_passes slot order)."""
    M = 1 << logm
    off, dist4, dist = 0, M, M >> 2
    while dist:
        l0 = dist.bit_length() - 1
        g = row // dist4
        if layer == l0 + 1:
            return off + 3 * g + 1
        if layer == l0:
            return off + 3 * g + (2 if (row // dist) & 2 else 0)
        off += 3 * (M // dist4)
        dist4, dist = dist, dist >> 2
    return off + row // 2


def pairs(layer, rows):
    """Lower rows j of the pairs (j, j + 2^layer) among rows [0, rows)."""
    return [j for j in range(rows) if not (j >> layer) & 1]


def hp_encode(tab, logm, k, p, sym):
    """k_encode_hp's butterfly order and twiddle slots (bitslice.hip HpEncoder)."""
    M, RW, LR = 1 << logm, 1 << (logm - 2), logm - 2
    ifft, fft = widen(tab["ifft8"]), widen(tab["fft8"])

    def i2(X, a, b, Mx):
        X[b] ^= X[a]
        X[a] ^= gf2_apply(Mx, X[b])

    def f2(X, a, b, Mx):
        X[a] ^= gf2_apply(Mx, X[b])
        X[b] ^= X[a]

    nch = -(-k // M)
    assert nch <= tab["nch"]
    acc = None
    for c in range(nch):
        X = np.zeros((M, sym.shape[1]), np.uint32)
        n = min(M, k - M * c)
        X[:n] = sym[M * c:M * c + n]
        T = ifft[c]
        for w in range(4):  # row groups RW*w + j: layers r0 .. r(LR-1)
            for l in range(LR):
                for j in pairs(l, RW):
                    r = RW * w + j
                    i2(X, r, r + (1 << l), T[ifft_slot(logm, l, r)])
        for co in range(RW):  # cosets: rows co + RW*t, layers r(LR), r(LR+1)
            r = [co + RW * t for t in range(4)]
            i2(X, r[0], r[1], T[ifft_slot(logm, LR, 0)])
            i2(X, r[2], r[3], T[ifft_slot(logm, LR, 2 * RW)])
            i2(X, r[0], r[2], T[ifft_slot(logm, LR + 1, 0)])
            i2(X, r[1], r[3], T[ifft_slot(logm, LR + 1, RW)])
        acc = X if acc is None else acc ^ X
    for co in range(RW):
        r = [co + RW * t for t in range(4)]
        f2(acc, r[0], r[2], fft[fft_slot(logm, LR + 1, 0)])
        f2(acc, r[1], r[3], fft[fft_slot(logm, LR + 1, RW)])
        f2(acc, r[0], r[1], fft[fft_slot(logm, LR, 0)])
        f2(acc, r[2], r[3], fft[fft_slot(logm, LR, 2 * RW)])
    for w in range(4):
        for l in reversed(range(LR)):
            for j in pairs(l, RW):
                r = RW * w + j
                f2(acc, r, r + (1 << l), fft[fft_slot(logm, l, r)])
    return acc[:p]


GEOMS = [(128, 32), (32, 32), (100, 17), (130, 32), (192, 32), (1, 17), (64, 16), (9, 9), (192, 16), (33, 12),
         (1, 9), (177, 16)]


@pytest.mark.parametrize("k,p", GEOMS)
def test_half_plane_schedule_matches_oracle(k, p):
    """k_encode_hp's order in subfield coordinates (the only mode it runs in)."""
    tabs = load_tables()
    logm = 5 if p > 16 else 4
    tab = tabs[logm]
    rng = np.random.default_rng(3 * k + p)
    S = 128
    data = rng.integers(0, 256, (k, S), dtype=np.uint8)
    blk = data.reshape(k, -1, 64)
    sym = (blk[:, :, :32].astype(np.uint32) | (blk[:, :, 32:].astype(np.uint32) << 8)).reshape(k, -1)
    par = to_sub(tab["dmat"], hp_encode(tab, logm, k, p, to_sub(tab["dmat"], sym))).reshape(p, -1, 32)
    got = np.concatenate([(par & 0xFF).astype(np.uint8), (par >> 8).astype(np.uint8)], axis=2).reshape(p, S)
    assert np.array_equal(got, orc.encode(16, k, p, data)), (k, p)


def test_slot_functions_cover_every_slot():
    """Every IFFT/FFT slot of the schedule is used by exactly the butterflies
    gf_host.cpp assigns it: the kernel's (layer, row) -> slot maps hit every
    slot, and each slot sees one layer."""
    for logm in (4, 5):
        M = 1 << logm
        ifs, ffs = {}, {}
        for l in range(logm):
            for j in pairs(l, M):
                ifs.setdefault(ifft_slot(logm, l, j), set()).add(l)
                ffs.setdefault(fft_slot(logm, l, j), set()).add(l)
        n_if = {4: 15, 5: 31}[logm]
        assert sorted(ifs) == list(range(n_if)) and sorted(ffs) == list(range(n_if))
        assert all(len(v) == 1 for v in list(ifs.values()) + list(ffs.values()))


# ---------------------------------------------------------------- bit-sliced n = 256 decode (bitslice_dec.hip)
def load_dectab():
    if not os.path.exists(HDR):
        pytest.skip("build/bs_tables.h not generated (run __graft_entry__.build())")
    body = re.search(r"struct DecTab256 \{(.*?)\n\};", open(HDR).read(), re.S).group(1)

    def arr(name):
        blk = re.search(r"\b" + name + r"\[[^=]*= *(\{.*?\});", body, re.S).group(1)
        return np.array([int(x) for x in re.findall(r"\d+", blk)], np.int64)

    return arr("m8").reshape(8, 128, 8), arr("logs").reshape(8, 128)


def test_dectab_matches_decoder_twiddles():
    """DecTab256: layer L, group g holds fftSkew[g 2^(L+1) + 2^L - 1]
    (ifftDITDecoder / fftDIT indexing, leopard16.go:573-657) and its 8x8
    matrix in subfield coordinates (the product of each basis element < 256)."""
    from oracle import leopard_np as lnp

    F = lnp.field(16)
    m8, logs = load_dectab()
    for L in range(8):
        for g in range(128):
            if g >= 128 >> L:
                assert logs[L, g] == F.mod
                continue
            lg = int(F._skew[g * (2 << L) + (1 << L) - 1])
            assert logs[L, g] == lg, (L, g)
            for j in range(8):
                col = int(F.mul_log(1 << j, lg)) if lg != F.mod else 0
                assert col < 256, "decoder twiddles lie in the subfield"
                for i in range(8):
                    assert ((m8[L, g, i] >> j) & 1) == ((col >> i) & 1), (L, g, i, j)


def _layer(F, W, L, inverse):
    """One radix-2 layer of the decoder transform over all rows (twiddle of the pair (a, a + 2^L))."""
    n = W.shape[0]
    for a in range(n):
        if (a >> L) & 1:
            continue
        lg = int(F._skew[(a & ~((2 << L) - 1)) + (1 << L) - 1])
        x, y = W[a], W[a + (1 << L)]
        if inverse:
            y ^= x
            if lg != F.mod:
                x ^= F.mul_log(y, lg)
        else:
            if lg != F.mod:
                x ^= F.mul_log(y, lg)
            y ^= x


@pytest.mark.parametrize("mtrunc", [160, 129, 150])
def test_decode_split_equals_reference_chain(mtrunc):
    """The kernel's algebra (bitslice_dec.hip): IFFT layers 0-4, then
    B_F (I + H) B_I u + Lo u over layers 5-7 with the derivative split
    H = N_4..N_7 / Lo = N_0..N_3, then FFT layers 4-0, equals the reference
    chain ifftDITDecoder -> formal derivative -> fftDIT (leopard16.go:518-540)
    on every row < mtrunc, for zero rows past mtrunc."""
    from oracle import leopard_np as lnp

    F = lnp.field(16)
    n, cols = 256, 6
    rng = np.random.default_rng(mtrunc)
    x = np.zeros((n, cols), np.int64)
    x[:mtrunc] = rng.integers(0, 1 << 16, (mtrunc, cols))
    ref = x.copy()
    lnp.ifft_decoder(F, ref, mtrunc, n)
    ref = lnp.formal_derivative(ref, n)
    lnp.fft(F, ref, mtrunc, n)

    u = x.copy()
    for L in range(5):
        _layer(F, u, L, True)
    v = u.copy()
    for L in (5, 6, 7):
        _layer(F, v, L, True)
    h = v.copy()  # (I + H) v, H = N_4 .. N_7
    for r in range(n):
        for b in range(4, 8):
            if not (r >> b) & 1:
                h[r] ^= v[r | (1 << b)]
    for L in (7, 6, 5):
        _layer(F, h, L, False)
    for r in range(n):  # + Lo u
        for b in range(4):
            if not (r >> b) & 1:
                h[r] ^= u[r | (1 << b)]
    for L in (4, 3, 2, 1, 0):
        _layer(F, h, L, False)
    assert np.array_equal(h[:mtrunc], ref[:mtrunc])

