"""Parity pins through the HIP path (GPU, -m gpu):

* every committed golden fixture (tests/golden/*.npz, made by
  tests/golden/make_golden.py from the oracle) is replayed through the C-ABI:
  encode must reproduce the stored parity byte for byte, and for every stored
  erasure mask Reconstruct / ReconstructData must rebuild exactly the stored
  shards (host-pointer entry points rs_encode / rs_reconstruct, and the
  device-resident rs_encode_dev / rs_reconstruct_dev);
* rs_reconstruct_dev's output is compared directly with the oracle's
  reconstruct output (orc.Oracle.reconstruct, leopard16.go:390-570) for the C4
  erasure patterns (32 random erasures with the bench seed, the worst case
  "first 32 data shards", parity-only, data-only), at a window size the
  oracle finishes in seconds;
* the GF(2^8) inversion-cache sequence of leopard8.go:508-555 (a cached
  error-locator vector reused for a different parity-erasure pattern): by
  default the engine keeps the reference's cache and returns the reference's
  (stale) result, call for call against the oracle on random call sequences
  through the host and device entry points; rs_set_reference_inversion_cache(0)
  keys the cache on the exact pattern and returns the correct shard.
"""
import os

import numpy as np
import pytest

import reedsolomon16_amd as rs
from oracle import orc

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def golden_names():
    return sorted(f[:-4] for f in os.listdir(GOLDEN) if f.endswith(".npz"))


def load(name):
    with np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False) as z:
        return {key: z[key] for key in z.files}


@pytest.fixture(scope="module")
def torch():
    import torch as t

    return t


@pytest.mark.parametrize("name", golden_names())
def test_golden_replay_host(name):
    g = load(name)
    bits, k, p = int(g["bits"][0]), int(g["k"][0]), int(g["p"][0])
    S = g["data"].shape[1]
    c = rs.ReedSolomon(k, p, bits)
    shards = [np.ascontiguousarray(g["data"][i]) for i in range(k)] + [np.zeros(S, np.uint8) for _ in range(p)]
    c.encode(shards)
    assert np.array_equal(np.stack(shards[k:]), g["parity"])
    assert c.verify(shards)
    full = [g["data"][i] for i in range(k)] + [g["parity"][i] for i in range(p)]
    for er in g["erasures"]:
        # a codec per mask, as a fresh reference encoder would be: the GF(2^8)
        # inversion cache (leopard8.go:508-555, kept by default) does not carry
        # one mask's locators into another's
        c = rs.ReedSolomon(k, p, bits)
        sh = [None if er[i] else full[i].copy() for i in range(k + p)]
        c.reconstruct(sh)
        for i in range(k + p):
            assert np.array_equal(sh[i], full[i]), (name, i)
        sh = [None if er[i] else full[i].copy() for i in range(k + p)]
        c.reconstruct_data(sh)
        for i in range(k):
            assert np.array_equal(sh[i], full[i]), (name, i)


@pytest.mark.parametrize("name", golden_names())
def test_golden_replay_device(torch, name):
    g = load(name)
    bits, k, p = int(g["bits"][0]), int(g["k"][0]), int(g["p"][0])
    S = g["data"].shape[1]
    c = rs.ReedSolomon(k, p, bits)
    slab = torch.zeros((k + p, S), dtype=torch.uint8, device="cuda")
    slab[:k] = torch.from_numpy(g["data"]).cuda()
    c.encode_dev(slab)
    torch.cuda.synchronize()
    assert np.array_equal(slab[k:].cpu().numpy(), g["parity"])
    full = slab.clone()
    for er in g["erasures"]:
        c = rs.ReedSolomon(k, p, bits)  # a codec per mask (see test_golden_replay_host)
        present = er == 0
        broken = full.clone()
        broken[torch.from_numpy(np.flatnonzero(er)).cuda()] = 0
        c.reconstruct_dev(broken, present)
        torch.cuda.synchronize()
        assert torch.equal(broken, full), name


def c4_patterns(k, p):
    rng = np.random.default_rng(0x5EED)
    return {
        "random32": rng.choice(k + p, p, replace=False),
        "first32data": np.arange(p),
        "parity_only": np.arange(k, k + p),
        "mixed_few": np.array([0, 5, 64, 127, 128, 159]),
        "one": np.array([77]),
    }


@pytest.mark.parametrize("pattern", ["random32", "first32data", "parity_only", "mixed_few", "one"])
@pytest.mark.parametrize("recover_all", [True, False])
def test_reconstruct_dev_equals_oracle(torch, pattern, recover_all):
    """C4 geometry (128+32), oracle-sized window: the engine's rebuilt rows are
    the oracle's rebuilt rows (not just a round trip)."""
    k, p, S = 128, 32, 4096 + 640
    rng = np.random.default_rng(41)
    data = rng.integers(0, 256, (k, S), dtype=np.uint8)
    par = orc.encode(16, k, p, data)
    full = np.concatenate([data, par])
    er = c4_patterns(k, p)[pattern]
    mask = np.zeros(k + p, bool)
    mask[er] = True
    e, ref = orc.Oracle(16, k, p).reconstruct([None if mask[i] else full[i].copy() for i in range(k + p)], recover_all)
    assert e == 0
    c = rs.New16(k, p)
    slab = torch.from_numpy(full.copy()).cuda()
    slab[torch.from_numpy(np.flatnonzero(mask)).cuda()] = 0
    c.reconstruct_dev(slab, ~mask, recover_all=recover_all)
    torch.cuda.synchronize()
    got = slab.cpu().numpy()
    for i in range(k + p):
        if ref[i] is not None:
            assert np.array_equal(got[i], ref[i]), (pattern, i)


def test_gf8_inversion_cache_sequence_exact_mode():
    """leopard8.go:508-555 with total <= 64 (cache on): ReconstructData with
    data 0 + parity 0 erased, then with data 0 only.  The reference keys its
    cache on the data-erasure bitmap alone (parity bits only when recoverAll),
    so its second call reuses the first call's error locators and returns a
    wrong shard 0 (the oracle reproduces it).  With
    rs_set_reference_inversion_cache(0) the engine keys its cache on the exact
    pattern: shard 0 comes back correct."""
    k, p, S = 10, 4, 64
    data = np.random.default_rng(2).integers(0, 256, (k, S), dtype=np.uint8)
    par = orc.encode(8, k, p, data)
    full = [data[i] for i in range(k)] + [par[i] for i in range(p)]
    o = orc.Oracle(8, k, p)
    assert o.reconstruct([None if i in (0, k) else full[i].copy() for i in range(k + p)], False)[0] == 0
    e, stale = o.reconstruct([None if i == 0 else full[i].copy() for i in range(k + p)], False)
    assert e == 0 and not np.array_equal(stale[0], full[0])  # the reference's result
    c = rs.New8(k, p)
    c.set_reference_inversion_cache(False)
    sh = [None if i in (0, k) else full[i].copy() for i in range(k + p)]
    c.reconstruct_data(sh)
    assert np.array_equal(sh[0], full[0])
    sh = [None if i == 0 else full[i].copy() for i in range(k + p)]
    c.reconstruct_data(sh)
    assert np.array_equal(sh[0], full[0])  # the exact mode's (correct) result


def test_gf8_inversion_cache_sequence_default_is_reference():
    """By default the same sequence returns the reference's stale shard 0,
    byte for byte the oracle's; reset_inversion_cache() (a fresh newFF8)
    forgets it."""
    k, p, S = 10, 4, 64
    data = np.random.default_rng(2).integers(0, 256, (k, S), dtype=np.uint8)
    par = orc.encode(8, k, p, data)
    full = [data[i] for i in range(k)] + [par[i] for i in range(p)]
    o = orc.Oracle(8, k, p)
    c = rs.New8(k, p)
    for erased in ((0, k), (0,)):
        e, ref = o.reconstruct([None if i in erased else full[i].copy() for i in range(k + p)], False)
        assert e == 0
        sh = [None if i in erased else full[i].copy() for i in range(k + p)]
        c.reconstruct_data(sh)
        assert np.array_equal(sh[0], ref[0])
    assert not np.array_equal(sh[0], full[0])  # the stale result, as the reference returns it
    c.reset_inversion_cache()
    sh = [None if i == 0 else full[i].copy() for i in range(k + p)]
    c.reconstruct_data(sh)
    assert np.array_equal(sh[0], full[0])


@pytest.mark.parametrize("entry", ["host", "device"])
@pytest.mark.parametrize("S", [64, 2048])
def test_gf8_reference_inversion_cache_random_sequences(torch, entry, S):
    """60 reconstructs of one GF(2^8) codec (40 + 16: total <= 64, so the
    reference caches) over erasure sets drawn from a few shards, with random
    recoverAll, in reference mode: every rebuilt shard equals the oracle's on
    the same call sequence (the default mode).  At S = 2048 one-to-four erasures take the
    reference's useBits branch (leopard8.go:474), whose store key is the
    prepared bitfield (:1192-1199), so a later pattern with both bits of a
    pair erased reuses errLocs computed for one of them; at S = 64 only the
    parity bits left out of the key collide.  Both kinds of stale hit occur."""
    k, p = 40, 16
    rng = np.random.default_rng(S + (1 if entry == "device" else 0))
    data = rng.integers(0, 256, (k, S), dtype=np.uint8)
    par = orc.encode(8, k, p, data)
    full = np.concatenate([data, par])
    o = orc.Oracle(8, k, p)
    c = rs.New8(k, p)  # reference mode is the default
    pool = [0, 1, 2, 3, 6, 7, k, k + 1, k + 5]
    stale = 0
    for _ in range(60):
        er = sorted(set(int(x) for x in rng.choice(pool, int(rng.integers(1, 5)), replace=False)))
        ra = bool(rng.integers(0, 2))
        e, ref = o.reconstruct([None if i in er else full[i].copy() for i in range(k + p)], ra)
        assert e == 0
        if entry == "host":
            sh = [None if i in er else full[i].copy() for i in range(k + p)]
            (c.reconstruct if ra else c.reconstruct_data)(sh)
            got = sh
        else:
            present = np.ones(k + p, bool)
            present[er] = False
            slab = torch.from_numpy(full.copy()).cuda()
            slab[torch.tensor(er).cuda()] = 0
            c.reconstruct_dev(slab, present, recover_all=ra)
            torch.cuda.synchronize()
            got = slab.cpu().numpy()
        for i in er:
            if ref[i] is None:
                continue
            assert np.array_equal(got[i], ref[i]), (er, ra, i)
            stale += not np.array_equal(ref[i], full[i])
    assert stale > 0  # the sequence exercised the reference's stale hits


@pytest.mark.parametrize("bits,k,p", [(16, 128, 32), (8, 128, 32), (16, 100, 28), (8, 10, 4)])
@pytest.mark.parametrize("nerased", [1, 2, 3, 8])
def test_pruned_fft_equals_unpruned_and_oracle(torch, paths, bits, k, p, nerased):
    """The LDS reconstruct skips FFT groups whose rows are not revealed (the
    analog of errorBitfield, leopard16.go:1076-1252 / leopard8.go:1165-1273):
    the rebuilt rows equal the unpruned run (rs_debug_set_path("prune", 0)) and the oracle."""
    S = 4096 + 256
    rng = np.random.default_rng(k + p + nerased + bits)
    data = rng.integers(0, 256, (k, S), dtype=np.uint8)
    par = orc.encode(bits, k, p, data)
    full = np.concatenate([data, par])
    nerased = min(nerased, p)
    for trial in range(3):
        er = rng.choice(k + p, nerased, replace=False)
        mask = np.zeros(k + p, bool)
        mask[er] = True
        outs = []
        for noprune in ("0", "1"):
            paths("prune", int(noprune != "1"))
            c = rs.ReedSolomon(k, p, bits)
            slab = torch.from_numpy(full.copy()).cuda()
            slab[torch.from_numpy(np.flatnonzero(mask)).cuda()] = 0
            c.reconstruct_dev(slab, ~mask)
            torch.cuda.synchronize()
            outs.append(slab.cpu().numpy())
        assert np.array_equal(outs[0], full) and np.array_equal(outs[1], full), (trial, sorted(er))
