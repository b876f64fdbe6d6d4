"""GPU parity of the bit-sliced m = 256 encode (csrc/bitslice_enc256.hip,
k_enc_bs256; the C5 path) against the oracle: one to four chunks with full and
ragged last chunks (k = 1 .. 1024), p across 129 .. 256 (rows >= p not
stored), shard sizes below, at and past the 512-byte tile (a partial last
tile), several stripes per launch and more tiles than workgroups (the
persistent loop and its cross-tile prefetch), strided rows with guard bytes,
special inputs, and verify with tampering.  The byte-permute LDS kernel
(RS_BS=0) must give the same bytes."""
import numpy as np
import pytest

import reedsolomon16_amd as rs
from oracle import orc

pytestmark = pytest.mark.gpu

GEOMS = [(1024, 256), (1000, 200), (300, 129), (256, 256), (1, 129), (513, 255), (768, 256), (257, 130), (1023, 160)]


@pytest.fixture(scope="module")
def torch():
    import torch as t

    return t


@pytest.mark.parametrize("k,p", GEOMS)
def test_bs256_path_selected(k, p):
    assert rs.New16(k, p).encode_path == "bs16-m256"


def test_bs256_not_selected_outside_its_range():
    assert rs.New16(1025, 256).encode_path != "bs16-m256"  # five chunks
    assert rs.New16(1024, 128).encode_path != "bs16-m256"  # m = 128


@pytest.mark.parametrize("k,p,S,n", [(1024, 256, 512, 1), (1024, 256, 512 * 3 + 64, 2), (1000, 200, 64, 1),
                                     (300, 129, 512 * 2, 3), (256, 256, 192, 2), (1, 129, 512, 1),
                                     (513, 255, 512 + 128, 1), (768, 256, 1024, 2), (257, 130, 576, 1),
                                     (1023, 160, 512 * 4, 1)])
def test_bs256_batch_matches_oracle(torch, k, p, S, n):
    rng = np.random.default_rng(k * 7 + p + S + n)
    datas = [rng.integers(0, 256, (k, S), dtype=np.uint8) for _ in range(n)]
    slab = torch.zeros((n, k + p, S), dtype=torch.uint8, device="cuda")
    for j in range(n):
        slab[j, :k] = torch.from_numpy(datas[j]).cuda()
    c = rs.New16(k, p)
    assert c.encode_path == "bs16-m256"
    c.encode_dev_batch(slab)
    torch.cuda.synchronize()
    for j in range(n):
        got = slab[j, k:].cpu().numpy()
        ref = orc.encode(16, k, p, datas[j])
        bad = np.nonzero((got != ref).any(axis=1))[0]
        assert not len(bad), f"stripe {j}: parity rows {bad[:8]} differ"


def test_bs256_many_tiles_persistent(torch):
    """More tiles than workgroups: 1024 + 256 x 64 KiB x 3 stripes = 384 tiles."""
    k, p, S, n = 1024, 256, 64 << 10, 3
    g = torch.Generator(device="cuda")
    g.manual_seed(77)
    slab = torch.randint(0, 256, (n, k + p, S), dtype=torch.uint8, device="cuda", generator=g)
    c = rs.New16(k, p)
    c.encode_dev_batch(slab)
    torch.cuda.synchronize()
    for j in (0, n - 1):
        data = slab[j, :k].cpu().numpy()
        # the oracle over a few column windows (the whole stripe is slow in the scalar oracle)
        for lo in (0, S // 2 + 512, S - 1024):
            ref = orc.encode(16, k, p, np.ascontiguousarray(data[:, lo:lo + 1024]))
            assert np.array_equal(slab[j, k:, lo:lo + 1024].cpu().numpy(), ref), (j, lo)


@pytest.mark.parametrize("k,p", [(1024, 256), (300, 200)])
def test_bs256_special_inputs(torch, k, p):
    S = 1024
    c = rs.New16(k, p)
    cases = [np.zeros((k, S), np.uint8), np.full((k, S), 0xFF, np.uint8)]
    for r in (0, 1, 2, 31, 32, 255, 256, k // 2 + 13, k - 1):
        if r >= k:
            continue
        d = np.zeros((k, S), np.uint8)
        d[r, 5] = 1
        d[r, S - 1] = 0x80
        d[r, 37] = 0x41
        cases.append(d)
    for d in cases:
        slab = torch.zeros((k + p, S), dtype=torch.uint8, device="cuda")
        slab[:k] = torch.from_numpy(d).cuda()
        c.encode_dev(slab)
        torch.cuda.synchronize()
        assert np.array_equal(slab[k:].cpu().numpy(), orc.encode(16, k, p, d))


@pytest.mark.parametrize("k,p", [(1024, 256), (700, 150)])
def test_bs256_strided_rows_and_verify(torch, k, p):
    S = 512 * 2 + 192
    rng = np.random.default_rng(k + p)
    data = rng.integers(0, 256, (k, S), dtype=np.uint8)
    ref = orc.encode(16, k, p, data)
    big = torch.full((k + p, S + 320), 0xA5, dtype=torch.uint8, device="cuda")
    big[:k, :S] = torch.from_numpy(data).cuda()
    view = big[:, :S]
    c = rs.New16(k, p)
    assert c.encode_path == "bs16-m256"
    c.encode_dev(view)
    torch.cuda.synchronize()
    assert np.array_equal(view[k:].cpu().numpy(), ref)
    assert bool((big[:, S:] == 0xA5).all()), "wrote past the row end"
    assert c.verify_dev(view)
    for r, col in [(k, 0), (k + p - 1, S - 1), (k + p // 2, 512), (0, 0), (k - 1, S - 1), (k // 2, 700)]:
        view[r, col] ^= 1
        assert not c.verify_dev(view), (r, col)
        view[r, col] ^= 1
    assert c.verify_dev(view)
    view[k:] = torch.randint(0, 256, (p, S), dtype=torch.uint8, device="cuda")
    assert not c.verify_dev(view)


def test_bs256_equals_lds_kernel(torch, monkeypatch):
    """The byte-permute LDS kernel (RS_BS=0) and the bit-sliced kernel agree
    at the C5 shape's 8-rank slice width."""
    k, p, S = 1024, 256, 32 << 10
    g = torch.Generator(device="cuda")
    g.manual_seed(5)
    a = torch.randint(0, 256, (2, k + p, S), dtype=torch.uint8, device="cuda", generator=g)
    b = a.clone()
    rs.New16(k, p).encode_dev_batch(a)
    monkeypatch.setenv("RS_BS", "0")
    c = rs.New16(k, p)
    assert c.encode_path == "lds-m256"
    c.encode_dev_batch(b)
    torch.cuda.synchronize()
    assert torch.equal(a, b)
