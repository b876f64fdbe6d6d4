"""The bit-sliced n = 256 reconstruct (csrc/bitslice_dec.hip, k_rec_bs256)
against the oracle (orc.Oracle.reconstruct, leopard16.go:390-570).

The kernel serves every GF(2^16) codec with 128 < m + k <= 160 (C4 is
128 + 32).  Covered: several (k, p) of that range, tile tails (S not a
multiple of its 1 KB column tile), every erasure class (data only, parity
only, mixed, one shard, the maximum p), the strided / row-table / batched
launch forms, guard bytes past a ragged row end, and random-count round trips.
"""
import numpy as np
import pytest

import reedsolomon16_amd as rs
from oracle import orc

pytestmark = pytest.mark.gpu

# (k, p, S): m + k in (128, 160]
GEOMS = [(128, 32, 4096), (128, 32, 1088), (96, 64, 2048), (120, 20, 1024 + 192), (144, 16, 640), (97, 32, 3072),
         (30, 100, 1024), (1, 128, 2048), (144, 9, 512)]


@pytest.fixture(params=[0, 8], ids=["product", "preload"], autouse=True)
def schedule(request, paths):
    """Every test under the product schedule and (round 6, rs_debug_set_path
    dec_lab bit 8) with the late phase-1 waves' row loads issued before the
    Y barrier, into V[8..15]."""
    paths("dec_lab", request.param)
    return request.param


def patterns(rng, k, p):
    n = k + p
    pats = [list(range(min(p, k))), list(range(k, k + p)), [0], [n - 1], [k - 1, k],
            rng.choice(n, p, replace=False).tolist(), rng.choice(n, max(1, p // 3), replace=False).tolist()]
    return [sorted(set(x)) for x in pats if len(set(x)) <= p]


@pytest.fixture(scope="module")
def torch():
    import torch as t

    return t


def encode_full(torch, k, p, S, seed):
    g = torch.Generator(device="cuda")
    g.manual_seed(seed)
    full = torch.randint(0, 256, (k + p, S), dtype=torch.uint8, device="cuda", generator=g)
    c = rs.New16(k, p)
    c.encode_dev(full)
    torch.cuda.synchronize()
    return c, full


@pytest.mark.parametrize("k,p,S", GEOMS)
def test_bsdec_equals_oracle(torch, k, p, S):
    c, full = encode_full(torch, k, p, S, k * 1000 + p + S)
    host = full.cpu().numpy()
    o = orc.Oracle(16, k, p)
    rng = np.random.default_rng(k + 7 * p)
    for er in patterns(rng, k, p):
        present = np.ones(k + p, bool)
        present[er] = False
        t = full.clone()
        t[torch.tensor(er, device="cuda")] = 0
        c.reconstruct_dev(t, present)
        torch.cuda.synchronize()
        e, ref = o.reconstruct([None if not present[i] else host[i].copy() for i in range(k + p)], True)
        assert e == 0
        got = t.cpu().numpy()
        for i in range(k + p):
            assert np.array_equal(got[i], ref[i]), f"{k}+{p} S={S} erased={er} shard {i}"
        assert torch.equal(t, full)


@pytest.mark.parametrize("recover_all", [True, False])
def test_bsdec_row_tables_and_data_only(torch, recover_all):
    """Separately allocated rows (the row-pointer form of the kernel) and
    ReconstructData (parity rows are not revealed)."""
    k, p, S = 128, 32, 2048 + 64
    c, full = encode_full(torch, k, p, S, 31)
    rng = np.random.default_rng(5)
    er = rng.choice(k + p, p, replace=False)
    present = np.ones(k + p, bool)
    present[er] = False
    rows = [full[i].clone() if present[i] else torch.zeros(S, dtype=torch.uint8, device="cuda") for i in range(k + p)]
    c.reconstruct_dev(rows, present, recover_all=recover_all)
    torch.cuda.synchronize()
    for i in range(k + p):
        if present[i] or recover_all or i < k:
            assert torch.equal(rows[i], full[i]), f"shard {i}"
        else:
            assert not rows[i].any(), f"parity shard {i} written by ReconstructData"


def test_bsdec_batched_stripes(torch):
    """rs_reconstruct_dev_batch: one pattern over 5 strided stripes (grid.y)."""
    k, p, S, B = 128, 32, 3072, 5
    g = torch.Generator(device="cuda")
    g.manual_seed(77)
    slab = torch.randint(0, 256, (B, k + p, S + 128), dtype=torch.uint8, device="cuda", generator=g)
    view = slab[:, :, :S]
    guard = slab[:, :, S:].clone()
    c = rs.New16(k, p)
    c.encode_dev_batch(view)
    torch.cuda.synchronize()
    ref = view.clone()
    rng = np.random.default_rng(77)
    er = rng.choice(k + p, p, replace=False)
    present = np.ones(k + p, bool)
    present[er] = False
    view[:, torch.from_numpy(er).cuda()] = 0
    c.reconstruct_dev_batch(view, present)
    torch.cuda.synchronize()
    assert torch.equal(view, ref)
    assert torch.equal(slab[:, :, S:], guard)


def test_bsdec_guard_bytes(torch):
    """A ragged last tile stores nothing past the row end: guard bytes after
    every row of a padded slab survive."""
    k, p, S = 128, 32, 1024 + 320
    g = torch.Generator(device="cuda")
    g.manual_seed(3)
    slab = torch.randint(0, 256, (k + p, S + 1024), dtype=torch.uint8, device="cuda", generator=g)
    guard = slab[:, S:].clone()
    view = slab[:, :S]
    c = rs.New16(k, p)
    c.encode_dev(view)
    torch.cuda.synchronize()
    ref = view.clone()
    er = list(range(0, k + p, 5))[:p]
    present = np.ones(k + p, bool)
    present[er] = False
    view[torch.tensor(er, device="cuda")] = 0
    c.reconstruct_dev(view, present)
    torch.cuda.synchronize()
    assert torch.equal(view, ref)
    assert torch.equal(slab[:, S:], guard)


def test_bsdec_random_pattern_round_trips(torch):
    """Random erasure counts 1..p at a larger width: rebuilt == encoded."""
    k, p, S = 128, 32, 8192
    c, full = encode_full(torch, k, p, S, 99)
    rng = np.random.default_rng(99)
    for _ in range(4):
        er = rng.choice(k + p, int(rng.integers(1, p + 1)), replace=False)
        present = np.ones(k + p, bool)
        present[er] = False
        t = full.clone()
        t[torch.from_numpy(er).cuda()] = 0
        c.reconstruct_dev(t, present)
        torch.cuda.synchronize()
        assert torch.equal(t, full)
