"""CPU tests of the oracle (test infrastructure): the C restatement against the
independent numpy restatement, the golden fixtures, the survey's table
anchors, the reference tests' round-trip properties and the reference's
panic / error behaviour."""
import hashlib
import os

import numpy as np
import pytest

from oracle import leopard_np as lnp
from oracle import orc

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def test_table_anchors():
    """SURVEY.md §8c sanity anchors (fftSkew[0:8] for both fields)."""
    _, _, skew16, _ = orc.tables16()
    _, _, skew8, _ = orc.tables8()
    assert skew16[:8].tolist() == [65535, 65535, 21845, 65535, 17476, 21845, 34952, 65535]
    assert skew8[:8].tolist() == [255, 255, 85, 255, 17, 85, 34, 255]


@pytest.mark.parametrize("bits", [16, 8])
def test_tables_c_vs_numpy(bits):
    t = orc.tables16() if bits == 16 else orc.tables8()
    F = lnp.field(bits)
    for a, b in zip(t, (F.log, F.exp, F.skew, F.walsh)):
        assert np.array_equal(a.astype(np.int64), b.astype(np.int64))


@pytest.mark.parametrize("bits", [16, 8])
def test_field_is_a_field(bits):
    """exp/log are inverse bijections; mulLog distributes over XOR (linearity the kernels rely on)."""
    F = lnp.field(bits)
    n = F.order
    assert np.array_equal(np.sort(F._log[1:]), np.arange(n - 1))
    assert np.all(F._exp[F._log[1:]] == np.arange(1, n))
    rng = np.random.default_rng(bits)
    a = rng.integers(0, n, 2000)
    b = rng.integers(0, n, 2000)
    for lm in rng.integers(0, n, 20):
        assert np.array_equal(F.mul_log(a ^ b, lm), F.mul_log(a, lm) ^ F.mul_log(b, lm))
    # log 'modulus' is the identity for mulLog (leopard16.go:841-846)
    assert np.array_equal(F.mul_log(a, F.mod), a)


ENC = [(2, 1, 64), (4, 2, 128), (10, 4, 256), (5, 3, 64), (3, 7, 64), (16, 4, 192), (33, 17, 64),
       (128, 32, 64), (100, 28, 64), (200, 100, 64), (70, 40, 64), (1, 1, 64), (300, 64, 64)]


@pytest.mark.parametrize("bits", [16, 8])
@pytest.mark.parametrize("k,p,S", ENC)
def test_encode_c_vs_numpy(bits, k, p, S):
    if bits == 8 and k + p > 256:
        pytest.skip("GF(2^8) codec is for <= 256 shards")
    data = np.random.default_rng(k * 31 + p).integers(0, 256, (k, S), dtype=np.uint8)
    assert np.array_equal(orc.encode(bits, k, p, data), lnp.encode(bits, k, p, data))


@pytest.mark.parametrize("bits", [16, 8])
@pytest.mark.parametrize("k,p", [(4, 2), (10, 4), (16, 4), (20, 12), (33, 17), (128, 32), (5, 3)])
def test_reconstruct_round_trip_all_classes(bits, k, p):
    """testReconstruction (reedsolomon_test.go:195-310) over erasure classes:
    data only, parity only, mixed, maximum (p) erasures; ReconstructData."""
    S = 64
    rng = np.random.default_rng(k + p)
    data = rng.integers(0, 256, (k, S), dtype=np.uint8)
    par = orc.encode(bits, k, p, data)
    full = [data[i] for i in range(k)] + [par[i] for i in range(p)]
    patterns = [list(range(min(p, k))), list(range(k, k + p)), [0, k], rng.choice(k + p, p, replace=False).tolist()]
    for er in patterns:
        sh = [None if i in er else full[i].copy() for i in range(k + p)]
        e, got = orc.Oracle(bits, k, p).reconstruct(sh, True)
        assert e == 0
        assert all(np.array_equal(got[i], full[i]) for i in range(k + p))
        ref = lnp.reconstruct(bits, k, p, sh, True)
        assert all(np.array_equal(ref[i], full[i]) for i in er)
        e, got = orc.Oracle(bits, k, p).reconstruct([None if i in er else full[i].copy() for i in range(k + p)], False)
        assert e == 0
        for i in range(k + p):
            if i < k:
                assert np.array_equal(got[i], full[i])
            elif i in er:
                assert got[i] is None


@pytest.mark.parametrize("bits", [16, 8])
def test_verify_and_errors(bits):
    """testVerify (reedsolomon_test.go:313-411) and the sentinel errors."""
    k, p, S = 10, 4, 128
    data = np.random.default_rng(1).integers(0, 256, (k, S), dtype=np.uint8)
    par = orc.encode(bits, k, p, data)
    full = [data[i] for i in range(k)] + [par[i] for i in range(p)]
    o = orc.Oracle(bits, k, p)
    assert o.verify([x.copy() for x in full]) == (True, 0)
    bad = [x.copy() for x in full]
    bad[0][0] ^= 1
    assert o.verify(bad) == (False, 0)
    assert o.encode(full[:5]) == 3  # ErrTooFewShards
    assert o.encode([x.copy() for x in full[:-1]] + [np.zeros(64, np.uint8)]) == 5  # ErrShardSize
    odd = [np.zeros(65, np.uint8) for _ in range(k + p)]
    assert o.encode(odd) == 6  # ErrInvalidShardSize
    e, _ = o.reconstruct([None] * 5 + full[5:])
    assert e == 3  # ErrTooFewShards (5 missing > p)
    e, _ = o.reconstruct([None] * (k + p))
    assert e == 4  # ErrShardNoData


def test_reference_panics_are_modelled():
    """GF(2^8) geometries whose skew slice runs past fftSkew8 (leopard8.go:167-206)."""
    o = orc.Oracle(8, 129, 127)
    sh = [np.zeros(64, np.uint8) for _ in range(256)]
    assert o.encode(sh) == 50
    # m + k > 256: the last encode chunk runs past fftSkew8 and reconstruct's
    # errLocs[i+m] / fwht8 index past [256]ffe8.
    o = orc.Oracle(8, 200, 40)
    sh = [np.zeros(64, np.uint8) for _ in range(240)]
    assert o.encode(sh) == 50
    sh[0] = None
    e, _ = o.reconstruct(sh)
    assert e == 50
    # m + k == 256 is fine for both
    o = orc.Oracle(8, 128, 100)
    sh = [np.zeros(64, np.uint8) for _ in range(228)]
    assert o.encode(sh) == 0
    sh[0] = None
    e, _ = o.reconstruct(sh)
    assert e == 0


def test_gf8_inversion_cache_is_stateful():
    """leopard8.go:508-555: the cache key is the data-erasure bitmap (parity
    bits only when recoverAll), so a ReconstructData call can reuse error
    locators computed for a different parity-erasure pattern.  The oracle
    keeps that state per codec exactly as the reference does."""
    k, p, S = 10, 4, 64
    data = np.random.default_rng(2).integers(0, 256, (k, S), dtype=np.uint8)
    par = orc.encode(8, k, p, data)
    full = [data[i] for i in range(k)] + [par[i] for i in range(p)]
    fresh = orc.Oracle(8, k, p)
    e, ok = fresh.reconstruct([None if i in (0,) else full[i].copy() for i in range(k + p)], False)
    assert e == 0 and np.array_equal(ok[0], full[0])
    o = orc.Oracle(8, k, p)
    e, _ = o.reconstruct([None if i in (0, k) else full[i].copy() for i in range(k + p)], False)
    assert e == 0
    e, second = o.reconstruct([None if i in (0,) else full[i].copy() for i in range(k + p)], False)
    assert e == 0
    # Same key {data 0}: the cached locators were computed with parity 0 erased.
    assert not np.array_equal(second[0], full[0])


def _load(name):
    with np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False) as z:
        return {key: z[key] for key in z.files}


def golden_names():
    return sorted(f[:-4] for f in os.listdir(GOLDEN) if f.endswith(".npz"))


def test_golden_manifest():
    lines = open(os.path.join(GOLDEN, "MANIFEST.sha256")).read().split("\n")
    want = dict(reversed(l.split("  ")) for l in lines if l.strip())
    assert sorted(want) == sorted(n + ".npz" for n in golden_names())
    for fn, h in want.items():
        assert hashlib.sha256(open(os.path.join(GOLDEN, fn), "rb").read()).hexdigest() == h


@pytest.mark.parametrize("name", golden_names())
def test_golden_fixtures(name):
    g = _load(name)
    bits, k, p = int(g["bits"][0]), int(g["k"][0]), int(g["p"][0])
    assert np.array_equal(orc.encode(bits, k, p, g["data"]), g["parity"])
    full = [g["data"][i] for i in range(k)] + [g["parity"][i] for i in range(p)]
    for er in g["erasures"]:
        sh = [None if er[i] else full[i].copy() for i in range(k + p)]
        e, got = orc.Oracle(bits, k, p).reconstruct(sh, True)
        assert e == 0 and all(np.array_equal(got[i], full[i]) for i in range(k + p))


@pytest.mark.parametrize("k,p,S,threads", [(128, 32, 64 * 33, 1), (128, 32, 64 * 33, 4), (10, 4, 4096, 3),
                                           (37, 9, 640, 2), (1024, 256, 128, 2), (3, 7, 64, 1), (200, 100, 192, 8)])
@pytest.mark.parametrize("isa", ["avx2", "avx512"])
def test_simd_port_matches_scalar_oracle(k, p, S, threads, isa):
    """The SIMD ports bench.py times as the CPU baseline (AVX2, and AVX-512
    like the reference's ifftDIT4/fftDIT4_avx512_*) compute the oracle's parity."""
    if isa not in orc.simd_isas():
        pytest.skip(f"no {isa} on this CPU")
    rng = np.random.default_rng(k + p + S + threads)
    data = rng.integers(0, 256, (k, S), dtype=np.uint8)
    assert np.array_equal(orc.encode_simd(k, p, data, threads, isa=isa), orc.encode(16, k, p, data))


def test_c5_chunk_twiddles_are_chunk0_plus_layer_constant():
    """The structure behind a bit-sliced m = 256 encode:
    initFFTSkew builds fftSkew[j + 2^(i+1)] = fftSkew[j] ^ temp[i]
    (leopard16.go:986-1031), so the twiddles of chunk c's ifftDITEncoder
    (skewLUT advanced by m per chunk, leopard16.go:176-207) are chunk 0's XOR a
    constant per layer: 8 distinct differences per chunk at m = 256, i.e.
    one full-field constant network per (layer, chunk) on top of networks
    shared by every chunk."""
    log, exp, skew, _ = orc.tables16()
    raw = np.where(skew == 65535, 0, exp[np.minimum(skew, 65534)].astype(np.int64))
    m = 256
    j = np.arange(1, m)
    for c in range(1, 4):
        d = raw[(c + 1) * m - 1 + j] ^ raw[m - 1 + j]
        layer = np.floor(np.log2(j & -j)).astype(int)  # lowest set bit of j: the butterfly layer of slot j
        for L in range(8):
            assert len(set(d[layer == L].tolist())) == 1, (c, L)
        assert len(set(d.tolist())) == 8


def _is_sub(F, lg):
    return lg == F.mod or int(F.exp[lg]) < 256


def test_c5_chunk_subfield_passes():
    """What k_enc_lds's subfield chunk passes rely on (codec.cpp
    upload_ifft_sub): at m = 256 chunk c's IFFT twiddles
    fftSkew[(c+1) 256 - 1 + g 2^(L+1) + 2^L] (ifftDITEncoder leopard16.go:699-741)
    are full-field only in layers 0 (c = 0), 0-1 (c = 1, 2) and 0-2 (c = 3),
    so the first all-subfield radix-4 pass (layer pairs 0-1, 2-3, ...) is 1,
    1, 1, 2."""
    from oracle import leopard_np as lnp

    F = lnp.field(16)
    full = {}
    for c in range(4):
        full[c] = sorted({L for L in range(8) for g in range(128 >> L)
                          if not _is_sub(F, int(F._skew[(c + 1) * 256 - 1 + g * (2 << L) + (1 << L)]))})
    assert full == {0: [0], 1: [0, 1], 2: [0, 1], 3: [0, 1, 2]}
    assert [max(f) // 2 + 1 for f in full.values()] == [1, 1, 1, 2]


def test_big_n_decoder_subfield_layers():
    """What k_rec_lds's BigSub passes rely on (kernels.hip BigSub, codec.cpp
    upload_big_sub): the decoder twiddle of layer L, rows (a, a + 2^L) is
    fftSkew[(a & ~(2^(L+1) - 1)) + 2^L - 1] (ifftDITDecoder / fftDIT,
    leopard16.go:573-657); at n = 512, 1024, 2048 it is full-field only in
    layers 0, 0-1, 0-2, so the IFFT is subfield from radix-4 pass 1 (pass 2 at
    n = 2048) on and the FFT (passes from the top layer down) for its first
    four passes."""
    from oracle import leopard_np as lnp

    F = lnp.field(16)
    for logn, want in ((9, [0]), (10, [0, 1]), (11, [0, 1, 2])):
        n = 1 << logn
        full = sorted({L for L in range(logn) for g in range(n >> (L + 1))
                       if not _is_sub(F, int(F._skew[g * (2 << L) + (1 << L) - 1]))})
        assert full == want, logn
        ni = max(full) // 2 + 1
        assert ni == (2 if logn == 11 else 1)
        # FFT radix-4 passes cover layers (logn-1, logn-2), (logn-3, logn-4), ...:
        # the first four never reach a full-field layer
        assert logn - 8 > max(full)
