"""GPU parity of the LDS-resident reconstruct for n = 512 .. 8192 work rows
(kernels.hip k_rec_lds<F16<2>, F16<2>, 9..13>: 64-byte column tiles of all n
rows in LDS, 32-byte half tiles at n = 4096, 16-byte quarter tiles at n = 8192,
the revealed-row mask and output
indices from HBM), the C5 repair
geometry (1024 + 256, n = 2048) among them, against the oracle's
reconstruct (leopard16.go:390-570) bit for bit: erasure classes (random at
the limit, data only, parity only, a few rows, one row), recover_all on and
off, strided and row-list launches, batched stripes, the host-pointer path,
and the multi-pass kernels (rs_debug_set_path "lds_big" 0)."""
import numpy as np
import pytest

import reedsolomon16_amd as rs
from oracle import orc

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch():
    import torch as t

    return t


@pytest.fixture(params=[0, 1], ids=["tiles64", "half32"], autouse=True)
def tile_mode(request, paths):
    """Every test twice: 64-byte tiles, one workgroup per CU, and (round 6)
    32-byte half tiles, two workgroups per CU (rs_debug_set_path rec_half;
    n = 1024 and 2048 only)."""
    paths("rec_half", request.param)
    return request.param


def patterns(k, p, seed):
    rng = np.random.default_rng(seed)
    return {
        "random_p": rng.choice(k + p, p, replace=False),
        "first_data": np.arange(p),
        "parity_only": np.arange(k, k + p),
        "few": np.array(sorted({0, 5, k // 2, k - 1, k, k + p - 1})),
        "one": np.array([k // 3]),
    }


def encoded(k, p, S, seed):
    rng = np.random.default_rng(seed)
    data = rng.integers(0, 256, (k, S), dtype=np.uint8)
    return np.concatenate([data, orc.encode(16, k, p, data)])


def oracle_rec(k, p, full, mask, recover_all):
    e, ref = orc.Oracle(16, k, p).reconstruct([None if mask[i] else full[i].copy() for i in range(k + p)], recover_all)
    assert e == 0
    return ref


# (k, p, S): n = 512 (m = 128), n = 1024, n = 2048 (C5 geometry and a ragged
# one), n = 4096 (m = 1024, and m = 16 with 2100 data shards), n = 8192 (the
# reference's 4000 + 1000, reedsolomon_test.go:82, and m = 128)
GEOMS = [(300, 100, 192), (700, 200, 128), (1024, 256, 128), (1000, 200, 64), (3000, 1000, 64), (2100, 10, 128),
         (4000, 1000, 64), (5000, 100, 128)]


@pytest.mark.parametrize("k,p,S", GEOMS)
@pytest.mark.parametrize("pattern", ["random_p", "first_data", "parity_only", "few", "one"])
def test_big_n_reconstruct_dev_equals_oracle(torch, k, p, S, pattern):
    full = encoded(k, p, S, k + p)
    er = patterns(k, p, k)[pattern]
    mask = np.zeros(k + p, bool)
    mask[er] = True
    c = rs.New16(k, p)
    for recover_all in (True, False):
        ref = oracle_rec(k, p, full, mask, recover_all)
        slab = torch.from_numpy(full.copy()).cuda()
        slab[torch.from_numpy(np.flatnonzero(mask)).cuda()] = 0
        c.reconstruct_dev(slab, ~mask, recover_all=recover_all)
        torch.cuda.synchronize()
        got = slab.cpu().numpy()
        for i in range(k + p):
            if ref[i] is not None:
                assert np.array_equal(got[i], ref[i]), (pattern, recover_all, i)
            elif mask[i]:
                assert not got[i].any(), (pattern, recover_all, i)


@pytest.mark.parametrize("k,p,S,ns", [(1024, 256, 256, 3), (3000, 1000, 128, 2), (4000, 1000, 64, 2)])
def test_big_n_row_list_and_batch(torch, k, p, S, ns):
    """Row pointers that are not equally strided (the ring-slot launch), then
    several stripes at padded row / stripe strides in one launch (n = 2048, 4096, 8192)."""
    full = encoded(k, p, S, 5)
    er = patterns(k, p, 6)["random_p"]
    mask = np.zeros(k + p, bool)
    mask[er] = True
    ref = oracle_rec(k, p, full, mask, True)
    c = rs.New16(k, p)
    rows = [None] * (k + p)
    for i in reversed(range(k + p)):  # separate allocations, addresses falling with i: not one stride
        rows[i] = torch.from_numpy(full[i].copy()).cuda()
    for i in np.flatnonzero(mask):
        rows[i].zero_()
    c.reconstruct_dev(rows, ~mask)
    torch.cuda.synchronize()
    for i in np.flatnonzero(mask):
        assert np.array_equal(rows[i].cpu().numpy(), ref[i]), i
    RS, SS = S + 3072, (k + p) * (S + 3072) + 4096
    buf = torch.zeros(ns * SS, dtype=torch.uint8, device="cuda")
    slab = buf.as_strided((ns, k + p, S), (SS, RS, 1))
    fulls = [encoded(k, p, S, 50 + z) for z in range(ns)]
    for z in range(ns):
        slab[z] = torch.from_numpy(fulls[z]).cuda()
    slab[:, torch.from_numpy(er).cuda()] = 0
    c.reconstruct_dev_batch(slab, ~mask)
    torch.cuda.synchronize()
    for z in range(ns):
        assert np.array_equal(slab[z].cpu().numpy(), fulls[z]), z


@pytest.mark.parametrize("k,p,S", [(1024, 256, 4096), (2500, 900, 64 * 20)])
def test_big_n_host_reconstruct(torch, k, p, S):
    """Host shards (rs_reconstruct through the staging pipeline) with n = 2048 and 4096."""
    full = encoded(k, p, S, 9)
    er = patterns(k, p, 10)["random_p"]
    c = rs.New16(k, p)
    sh = [None if i in set(er.tolist()) else full[i].copy() for i in range(k + p)]
    c.reconstruct(sh)
    for i in range(k + p):
        assert np.array_equal(sh[i], full[i]), i


@pytest.mark.parametrize("k,p,lds", [(2100, 10, 1), (2100, 10, 0), (4000, 1000, 1), (4000, 1000, 0)])
def test_n4096_n8192_lds_and_multipass(torch, paths, k, p, lds):
    """n = 4096 (2100 + 10: m = 16) and n = 8192 (the reference's 4000 + 1000,
    reedsolomon_test.go:82) in one LDS launch and through the multi-pass
    kernels (rs_debug_set_path "lds_big" 0)."""
    S = 64
    paths("lds_big", lds)
    full = encoded(k, p, S, 11)
    er = np.array([0, 1, 700, 2099, 2100, k + p - 1, 1500, 33, 1024, 2048])
    mask = np.zeros(k + p, bool)
    mask[er] = True
    ref = oracle_rec(k, p, full, mask, True)
    c = rs.New16(k, p)
    slab = torch.from_numpy(full.copy()).cuda()
    slab[torch.from_numpy(er).cuda()] = 0
    c.reconstruct_dev(slab, ~mask)
    torch.cuda.synchronize()
    got = slab.cpu().numpy()
    for i in range(k + p):
        assert np.array_equal(got[i], ref[i] if ref[i] is not None else full[i]), i
