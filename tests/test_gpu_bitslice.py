"""GPU parity of the bit-sliced encode kernel (csrc/bitslice.hip, k_encode_hp)
against the oracle: m = 32 and m = 16 geometries with full and ragged chunks
(the per-m tables serve every k up to the chunk cap and every p of the m),
ragged shard sizes (a partial last 2 KB tile, a single 64-byte block),
several stripes per launch, more tiles than workgroups (the persistent loop),
strided rows with guard bytes past the row end, and verify with tampering in
the first and last tile of data and parity rows."""
import numpy as np
import pytest

import reedsolomon16_amd as rs
from oracle import orc

pytestmark = pytest.mark.gpu

BS = [(128, 32), (32, 32), (100, 17), (130, 32), (192, 32), (1, 17), (64, 16), (9, 9), (192, 16), (33, 12)]


def path(p):
    return "bs16-m32" if p > 16 else "bs16-m16"


@pytest.fixture(scope="module")
def torch():
    import torch as t

    return t


@pytest.mark.parametrize("k,p", BS)
def test_bs_path_selected(k, p):
    assert rs.New16(k, p).encode_path == path(p)


@pytest.mark.parametrize("k,p,S,n", [(128, 32, 64, 1), (128, 32, 4096 * 3 + 64 * 5, 1), (128, 32, 8192, 3),
                                     (32, 32, 64 * 37, 2), (32, 32, 4096 * 64, 5), (100, 17, 4096 * 3 + 320, 2),
                                     (100, 17, 4096, 5), (128, 32, 2048 * 700 + 64 * 3, 2),
                                     (130, 32, 2048 * 5 + 64, 3), (192, 32, 4096, 2), (1, 17, 2048 * 3, 2),
                                     (64, 16, 64, 1), (64, 16, 2048 * 9 + 64 * 7, 3), (64, 16, 2048 * 1500, 1),
                                     (9, 9, 2048 * 2 + 192, 4), (192, 16, 4096 + 64, 2), (33, 12, 2048 * 4, 3)])
def test_bs_batch_matches_oracle(torch, k, p, S, n):
    rng = np.random.default_rng(k * 131 + p * 7 + S + n)
    datas = [rng.integers(0, 256, (k, S), dtype=np.uint8) for _ in range(n)]
    slab = torch.zeros((n, k + p, S), dtype=torch.uint8, device="cuda")
    for j in range(n):
        slab[j, :k] = torch.from_numpy(datas[j]).cuda()
    c = rs.New16(k, p)
    assert c.encode_path == path(p)
    c.encode_dev_batch(slab)
    torch.cuda.synchronize()
    for j in range(n):
        assert np.array_equal(slab[j, k:].cpu().numpy(), orc.encode(16, k, p, datas[j])), f"stripe {j}"


@pytest.mark.parametrize("tiles,step", [(2, 0), (3, 0), (4, 0), (4, 7), (3, 64), (8, 1), (5, 1000)])
@pytest.mark.parametrize("k,p,S,n", [(128, 32, 2048 * 20 + 64, 6), (100, 17, 2048 * 9 + 320, 5), (64, 16, 2048 * 33, 4)])
def test_bs_tiles_per_workgroup(torch, paths, tiles, step, k, p, S, n):
    """Several tiles per workgroup (launch_hp_t): workgroup b runs tiles
    t0 + i * step with the next tile's first chunk prefetched during the last
    chunk of the current one; every (tiles, step), the ragged last block of
    the grid included, gives the oracle's parity and verifies."""
    paths("hp_tiles", tiles)
    paths("hp_step", step)
    rng = np.random.default_rng(tiles * 31 + step + k + S)
    datas = [rng.integers(0, 256, (k, S), dtype=np.uint8) for _ in range(n)]
    slab = torch.zeros((n, k + p, S), dtype=torch.uint8, device="cuda")
    for j in range(n):
        slab[j, :k] = torch.from_numpy(datas[j]).cuda()
    c = rs.New16(k, p)
    assert c.encode_path == path(p)
    c.encode_dev_batch(slab)
    torch.cuda.synchronize()
    for j in range(n):
        assert np.array_equal(slab[j, k:].cpu().numpy(), orc.encode(16, k, p, datas[j])), f"stripe {j}"
    assert c.verify_dev_batch(slab)
    slab[n - 1, k + p - 1, S - 1] ^= 1
    assert not c.verify_dev_batch(slab)


def test_bs_tile_map_tuner(torch, paths):
    """The run-time tile-map choice (launch_hp_t HpTuner): the first launches
    of a candidate shape alternate four tiles per workgroup and one under
    events, later ones keep the faster map.  Every launch of the sequence --
    trials, the decision, the launches after it -- writes the parity one tile
    per workgroup writes (itself checked against the oracle on a window), and
    verify agrees.  Shape: the 8-rank slice of C3 (128 KiB of every row, 256
    stripes: 16384 tiles, both maps candidates)."""
    k, p, S, n = 128, 32, 128 << 10, 256
    g = torch.Generator(device="cuda")
    g.manual_seed(0x7A)
    slab = torch.randint(0, 256, (n, k + p, S), dtype=torch.uint8, device="cuda", generator=g)
    c = rs.New16(k, p)
    paths("hp_tiles", 1)
    c.encode_dev_batch(slab)
    torch.cuda.synchronize()
    ref = slab[:, k:].clone()
    for j in (0, n - 1):
        d = slab[j, :k, 4096:8192].cpu().numpy()
        assert np.array_equal(ref[j, :, 4096:8192].cpu().numpy(), orc.encode(16, k, p, np.ascontiguousarray(d)))
    paths("hp_tiles", 0)
    paths("hp_tune", 1)
    for it in range(14):
        slab[:, k:] = 0
        c.encode_dev_batch(slab)
        torch.cuda.synchronize()
        assert torch.equal(slab[:, k:], ref), f"launch {it}"
    assert c.verify_dev_batch(slab)


@pytest.mark.parametrize("k,p", [(128, 32), (64, 16)])
def test_bs_special_inputs(torch, k, p):
    """All-zero, all-0xFF and single-symbol impulses in every chunk."""
    S = 4096
    c = rs.New16(k, p)
    cases = [np.zeros((k, S), np.uint8), np.full((k, S), 0xFF, np.uint8)]
    m = 32 if p > 16 else 16
    for r in (0, m - 1, m, k // 2 + 13, k - 1):
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


@pytest.mark.parametrize("k,p", [(128, 32), (100, 17), (64, 16), (130, 32), (20, 10)])
def test_bs_strided_rows_and_verify(torch, k, p):
    S = 4096 * 2 + 192
    rng = np.random.default_rng(k + p)
    data = rng.integers(0, 256, (k, S), dtype=np.uint8)
    ref = orc.encode(16, k, p, data)
    big = torch.full((k + p, S + 256), 0xA5, dtype=torch.uint8, device="cuda")
    big[:k, :S] = torch.from_numpy(data).cuda()
    view = big[:, :S]
    c = rs.New16(k, p)
    assert c.encode_path == path(p)
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
