"""GPU parity of the bit-sliced encode kernel (csrc/bitslice.hip) against the
oracle: every geometry compiled in (Makefile BS_CONFIGS), ragged shard sizes
(a partial last 4 KB tile, a single 64-byte block), several stripes per
launch, more tiles than workgroups (the persistent loop), strided rows with
guard bytes past the row end, and verify with tampering in the first and last
tile of data and parity rows."""
import numpy as np
import pytest

import reedsolomon16_amd as rs
from oracle import orc

pytestmark = pytest.mark.gpu

BS = [(128, 32), (32, 32), (100, 17)]


@pytest.fixture(scope="module")
def torch():
    import torch as t

    return t


@pytest.mark.parametrize("k,p", BS)
def test_bs_path_selected(k, p):
    assert rs.New16(k, p).encode_path == "bs16-m32"


@pytest.fixture(params=["hp", "bs"])
def kernel(request, monkeypatch):
    """Both bit-sliced kernels: the half-plane kernel (default for subfield
    geometries) and the round-1 512-thread kernel (RS_BS_KERNEL=1)."""
    monkeypatch.setenv("RS_BS_KERNEL", "2" if request.param == "hp" else "1")
    return request.param


@pytest.mark.parametrize("k,p,S,n", [(128, 32, 64, 1), (128, 32, 4096 * 3 + 64 * 5, 1), (128, 32, 8192, 3),
                                     (32, 32, 64 * 37, 2), (32, 32, 4096 * 64, 5), (100, 17, 4096 * 3 + 320, 2),
                                     (100, 17, 4096, 5), (128, 32, 2048 * 700 + 64 * 3, 2)])
def test_bs_batch_matches_oracle(torch, kernel, k, p, S, n):
    rng = np.random.default_rng(k * 131 + p * 7 + S + n)
    datas = [rng.integers(0, 256, (k, S), dtype=np.uint8) for _ in range(n)]
    slab = torch.zeros((n, k + p, S), dtype=torch.uint8, device="cuda")
    for j in range(n):
        slab[j, :k] = torch.from_numpy(datas[j]).cuda()
    c = rs.New16(k, p)
    assert c.encode_path == "bs16-m32"
    c.encode_dev_batch(slab)
    torch.cuda.synchronize()
    for j in range(n):
        assert np.array_equal(slab[j, k:].cpu().numpy(), orc.encode(16, k, p, datas[j])), f"stripe {j}"


def test_bs_special_inputs(torch):
    """All-zero, all-0xFF and single-symbol impulses in every chunk."""
    k, p, S = 128, 32, 4096
    c = rs.New16(k, p)
    cases = [np.zeros((k, S), np.uint8), np.full((k, S), 0xFF, np.uint8)]
    for r in (0, 31, 32, 77, 127):
        d = np.zeros((k, S), np.uint8)
        d[r, 5] = 1
        d[r, 4095] = 0x80
        cases.append(d)
    for d in cases:
        slab = torch.zeros((k + p, S), dtype=torch.uint8, device="cuda")
        slab[:k] = torch.from_numpy(d).cuda()
        c.encode_dev(slab)
        torch.cuda.synchronize()
        assert np.array_equal(slab[k:].cpu().numpy(), orc.encode(16, k, p, d))


@pytest.mark.parametrize("k,p", [(128, 32), (100, 17)])
def test_bs_strided_rows_and_verify(torch, k, p):
    S = 4096 * 2 + 192
    rng = np.random.default_rng(k + p)
    data = rng.integers(0, 256, (k, S), dtype=np.uint8)
    ref = orc.encode(16, k, p, data)
    big = torch.full((k + p, S + 256), 0xA5, dtype=torch.uint8, device="cuda")
    big[:k, :S] = torch.from_numpy(data).cuda()
    view = big[:, :S]
    c = rs.New16(k, p)
    c.encode_dev(view)
    torch.cuda.synchronize()
    assert np.array_equal(view[k:].cpu().numpy(), ref)
    assert bool((big[:, S:] == 0xA5).all()), "wrote past the row end"
    assert c.verify_dev(view)
    for r, col in [(k, 0), (k + p - 1, S - 1), (k + p // 2, 4096), (0, 0), (k - 1, S - 1)]:
        view[r, col] ^= 1
        assert not c.verify_dev(view), (r, col)
        view[r, col] ^= 1
    assert c.verify_dev(view)
    # every parity byte wrong: one flag store per wave, still correct
    view[k:] = torch.randint(0, 256, (p, S), dtype=torch.uint8, device="cuda")
    assert not c.verify_dev(view)
