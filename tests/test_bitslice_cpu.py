"""CPU checks of what the bit-sliced encode kernel (csrc/bitslice.hip) is
built from, no device calls:

* its 64-byte block <-> bit-plane transpose (three delta-swap stages per
  8-dword half, restated in numpy) puts bit b of symbol 4w+j at bit 8j+w of
  plane b, and is an involution;
* the twiddle matrices tools/gen_bs_tables.cpp writes into build/bs_tables.h,
  applied as GF(2) matrices in the kernel's pass and butterfly order (chunk
  IFFT passes 1-3, XOR-accumulate, FFT passes A-C), give the oracle's parity
  bit for bit (leopard16.go:128-224) for every geometry compiled in;
* the same for the half-plane kernel's order (k_encode_hp: IFFT layers
  r0-r2 per 8-row group, layers r3-r4 per coset, FFT layers r4-r3 per coset,
  r2-r0 per group) and its slot indexing.
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
    for m in re.finditer(r"struct BsTw<(\d+), (\d+)> \{(.*?)\n\};", txt, re.S):
        k, p, body = int(m.group(1)), int(m.group(2)), m.group(3)
        nch = int(re.search(r"NCH = (\d+)", body).group(1))
        v = np.array([int(x, 16) for x in re.findall(r"0x([0-9a-fA-F]{4})", body)], np.uint32)
        assert v.size == (nch + 1) * 31 * 16, (k, p)
        sub = None
        if "SUB = true" in body:
            def nums(name):
                blk = re.search(r"\b" + name + r"\[[^=]*= *(\{.*?\});", body, re.S).group(1)
                return np.array([int(x) for x in re.findall(r"\d+", blk)], np.uint32)
            i8, f8 = nums("ifft8"), nums("fft8")
            assert i8.size == nch * 31 * 8 and f8.size == 31 * 8
            sub = (nums("dmat"), i8.reshape(nch, 31, 8), f8.reshape(31, 8))
        out[(k, p)] = (v[:nch * 496].reshape(nch, 31, 16), v[nch * 496:].reshape(31, 16), sub)
    assert out, "no geometry in bs_tables.h"
    return out


def test_header_holds_makefile_geometries():
    mk = open(os.path.join(ROOT, "reedsolomon16_amd", "Makefile")).read()
    cfg = re.search(r"BS_CONFIGS \?= (.*)", mk).group(1).split()
    assert {tuple(int(x) for x in c.split(":")) for c in cfg} == set(load_tables())


def gf2_apply(rows, y):
    """Output bit i = parity(y & rows[i]) (the kernel's XOR network, per symbol)."""
    out = np.zeros_like(y)
    for i in range(16):
        out |= (np.bitwise_count(y & rows[i]) & 1).astype(np.uint32) << np.uint32(i)
    return out


def bs_encode(tabs, k, p, sym):
    """The kernel's schedule on symbols (rows of uint32 symbol values)."""
    ifft, fft = tabs[0], tabs[1]

    def i2(X, a, b, M):
        X[b] ^= X[a]
        X[a] ^= gf2_apply(M, X[b])

    def f2(X, a, b, M):
        X[a] ^= gf2_apply(M, X[b])
        X[b] ^= X[a]

    def i4(X, r, T, s):
        i2(X, r[0], r[1], T[s])
        i2(X, r[2], r[3], T[s + 2])
        i2(X, r[0], r[2], T[s + 1])
        i2(X, r[1], r[3], T[s + 1])

    def f4(X, r, T, s):
        f2(X, r[0], r[2], T[s + 1])
        f2(X, r[1], r[3], T[s + 1])
        f2(X, r[0], r[1], T[s])
        f2(X, r[2], r[3], T[s + 2])

    acc = None
    for c in range(ifft.shape[0]):
        X = np.zeros((32, sym.shape[1]), np.uint32)
        n = min(32, k - 32 * c)
        X[:n] = sym[32 * c:32 * c + n]
        T = ifft[c]
        for w in range(8):  # pass 1
            i4(X, [4 * w + i for i in range(4)], T, 3 * w)
        for h in range(2):  # pass 2
            for j in range(4):
                i4(X, [16 * h + j + 4 * i for i in range(4)], T, 24 + 3 * h)
        for w in range(16):  # pass 3
            i2(X, w, w + 16, T[30])
        acc = X if acc is None else acc ^ X
    for j in range(8):  # pass A
        f4(acc, [j + 8 * i for i in range(4)], fft, 0)
    for g in range(4):  # pass B
        for j in range(2):
            f4(acc, [8 * g + j + 2 * i for i in range(4)], fft, 3 + 3 * g)
    for q in range(16):  # pass C
        f2(acc, 2 * q, 2 * q + 1, fft[15 + q])
    return acc[:p]


@pytest.mark.parametrize("S", [64, 192])
def test_tables_and_schedule_match_oracle(S):
    for (k, p), tabs in load_tables().items():
        rng = np.random.default_rng(k * 7 + p + S)
        data = rng.integers(0, 256, (k, S), dtype=np.uint8)
        blk = data.reshape(k, -1, 64)
        sym = (blk[:, :, :32].astype(np.uint32) | (blk[:, :, 32:].astype(np.uint32) << 8)).reshape(k, -1)
        par = bs_encode(tabs, k, p, sym).reshape(p, -1, 32)
        got = np.concatenate([(par & 0xFF).astype(np.uint8), (par >> 8).astype(np.uint8)], axis=2).reshape(p, S)
        assert np.array_equal(got, orc.encode(16, k, p, data)), (k, p)


def to_sub(dmat, sym):
    """Planes r < 8 ^= XOR of planes 8+i over the bits i of dmat[r] (an involution)."""
    out = sym.copy()
    hi = sym >> np.uint32(8)
    for r in range(8):
        out ^= (np.bitwise_count(hi & np.uint32(dmat[r])) & 1).astype(np.uint32) << np.uint32(r)
    return out


def test_subfield_tables_match_oracle():
    """SUB geometries: the same schedule with one 8x8 matrix on each byte half, in
    subfield coordinates, reproduces the oracle."""
    n = 0
    for (k, p), (_, _, sub) in load_tables().items():
        if sub is None:
            continue
        n += 1
        dmat, i8, f8 = sub
        # 8x8 rows -> the block-diagonal 16x16 rows the full-matrix emulation takes
        def widen(t):
            return (t | (t << np.uint32(8)))[..., list(range(8)) * 2] & np.concatenate(
                [np.full(8, 0xFF, np.uint32), np.full(8, 0xFF00, np.uint32)])
        tabs = (widen(i8), widen(f8))
        rng = np.random.default_rng(k + p)
        S = 128
        data = rng.integers(0, 256, (k, S), dtype=np.uint8)
        blk = data.reshape(k, -1, 64)
        sym = (blk[:, :, :32].astype(np.uint32) | (blk[:, :, 32:].astype(np.uint32) << 8)).reshape(k, -1)
        par = to_sub(dmat, bs_encode(tabs, k, p, to_sub(dmat, sym))).reshape(p, -1, 32)
        got = np.concatenate([(par & 0xFF).astype(np.uint8), (par >> 8).astype(np.uint8)], axis=2).reshape(p, S)
        assert np.array_equal(got, orc.encode(16, k, p, data)), (k, p)
    assert n >= 1


def hp_encode(tabs, k, p, sym):
    """k_encode_hp's butterfly order and twiddle slots (bitslice.hip HpEncoder)."""
    ifft, fft = tabs[0], tabs[1]

    def i2(X, a, b, M):
        X[b] ^= X[a]
        X[a] ^= gf2_apply(M, X[b])

    def f2(X, a, b, M):
        X[a] ^= gf2_apply(M, X[b])
        X[b] ^= X[a]

    acc = None
    for c in range(ifft.shape[0]):
        X = np.zeros((32, sym.shape[1]), np.uint32)
        n = min(32, k - 32 * c)
        X[:n] = sym[32 * c:32 * c + n]
        T = ifft[c]
        for w in range(4):  # phase 1: rows 8w + j, layers r0, r1, r2
            b = 8 * w
            for j in (0, 2, 4, 6):
                i2(X, b + j, b + j + 1, T[3 * (2 * w + (j >> 2)) + (2 if j & 2 else 0)])
            for j in (0, 1, 4, 5):
                i2(X, b + j, b + j + 2, T[3 * (2 * w + (j >> 2)) + 1])
            for j in range(4):
                i2(X, b + j, b + j + 4, T[24 + 3 * (w >> 1) + (2 if w & 1 else 0)])
        for co in range(8):  # phase 2: rows co + 8t, layers r3, r4
            r = [co + 8 * t for t in range(4)]
            i2(X, r[0], r[1], T[25])
            i2(X, r[2], r[3], T[28])
            i2(X, r[0], r[2], T[30])
            i2(X, r[1], r[3], T[30])
        acc = X if acc is None else acc ^ X
    for co in range(8):  # FFT layers r4, r3 per coset
        r = [co + 8 * t for t in range(4)]
        f2(acc, r[0], r[2], fft[1])
        f2(acc, r[1], r[3], fft[1])
        f2(acc, r[0], r[1], fft[0])
        f2(acc, r[2], r[3], fft[2])
    for w in range(4):  # FFT layers r2, r1, r0 per group
        b, s0 = 8 * w, 3 + 3 * w
        for j in range(4):
            f2(acc, b + j, b + j + 4, fft[s0 + 1])
        f2(acc, b, b + 2, fft[s0])
        f2(acc, b + 1, b + 3, fft[s0])
        f2(acc, b + 4, b + 6, fft[s0 + 2])
        f2(acc, b + 5, b + 7, fft[s0 + 2])
        for j in (0, 2, 4, 6):
            f2(acc, b + j, b + j + 1, fft[15 + 4 * w + (j >> 1)])
    return acc[:p]


def test_half_plane_schedule_matches_oracle():
    """k_encode_hp's order in subfield coordinates (the only mode it runs in)."""
    n = 0
    for (k, p), (_, _, sub) in load_tables().items():
        if sub is None:
            continue
        n += 1
        dmat, i8, f8 = sub

        def widen(t):
            return (t | (t << np.uint32(8)))[..., list(range(8)) * 2] & np.concatenate(
                [np.full(8, 0xFF, np.uint32), np.full(8, 0xFF00, np.uint32)])
        tabs = (widen(i8), widen(f8))
        rng = np.random.default_rng(3 * k + p)
        S = 128
        data = rng.integers(0, 256, (k, S), dtype=np.uint8)
        blk = data.reshape(k, -1, 64)
        sym = (blk[:, :, :32].astype(np.uint32) | (blk[:, :, 32:].astype(np.uint32) << 8)).reshape(k, -1)
        par = to_sub(dmat, hp_encode(tabs, k, p, to_sub(dmat, sym))).reshape(p, -1, 32)
        got = np.concatenate([(par & 0xFF).astype(np.uint8), (par >> 8).astype(np.uint8)], axis=2).reshape(p, S)
        assert np.array_equal(got, orc.encode(16, k, p, data)), (k, p)
    assert n >= 1
