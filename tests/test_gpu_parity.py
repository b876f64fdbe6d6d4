"""GPU parity tests: the HIP engine (through the C-ABI) against the oracle.

Bit-exact comparison on seeded inputs at sizes the oracle finishes in
seconds; at the BASELINE configs' full sizes, size-independent properties
(encode -> erase -> reconstruct round trips, Verify, and column-window parity:
shard columns are independent, so any 64-byte-aligned byte window of the GPU
output must equal the oracle run on that window of the input).
"""
import os

import numpy as np
import pytest

import reedsolomon16_amd as rs
from oracle import orc

pytestmark = pytest.mark.gpu


def rand_data(rng, k, S):
    return rng.integers(0, 256, (k, S), dtype=np.uint8)


def gpu_encode(bits, k, p, data):
    c = rs.ReedSolomon(k, p, bits)
    S = data.shape[1]
    shards = [np.ascontiguousarray(data[i]) for i in range(k)] + [np.zeros(S, np.uint8) for _ in range(p)]
    c.encode(shards)
    return np.stack(shards[k:]), c


# (k, p, S): every register-kernel width (m = 1..32), tails (k % m != 0), k < m,
# the multi-pass path (m >= 64) and the reference tests' own configs
# (reedsolomon_test.go:33-131).
ENCODE_CASES = [
    (2, 1, 64), (3, 1, 128), (4, 2, 256), (10, 4, 1024), (5, 3, 64), (8, 4, 192), (16, 4, 320),
    (10, 6, 128), (20, 8, 64), (33, 17, 128), (100, 28, 64), (128, 32, 256), (130, 32, 64),
    (3, 7, 64), (1, 1, 64), (1, 5, 64), (37, 9, 64), (128, 128, 128), (200, 100, 64),
    (70, 40, 128), (300, 64, 64), (64, 65, 64), (100, 150, 128), (16, 200, 64),
]


@pytest.mark.parametrize("bits", [16, 8])
@pytest.mark.parametrize("k,p,S", ENCODE_CASES)
def test_encode_matches_oracle(bits, k, p, S):
    if bits == 8 and k + p > 256:
        pytest.skip("GF(2^8) codec is for <= 256 shards")
    rng = np.random.default_rng(k * 1000 + p * 7 + S + bits)
    data = rand_data(rng, k, S)
    o = orc.Oracle(bits, k, p)
    shards = [np.ascontiguousarray(data[i]) for i in range(k)] + [np.zeros(S, np.uint8) for _ in range(p)]
    eo = o.encode(shards)
    c = rs.ReedSolomon(k, p, bits)
    gs = [d.copy() for d in shards[:k]] + [np.zeros(S, np.uint8) for _ in range(p)]
    if eo == 50:
        with pytest.raises(rs.ErrPanic):
            c.encode(gs)
        return
    assert eo == 0
    c.encode(gs)
    for i in range(p):
        assert np.array_equal(gs[k + i], shards[k + i]), f"parity row {i} differs (path {c.encode_path})"


@pytest.mark.parametrize("bits", [16, 8])
def test_special_inputs(bits):
    """All-zero, all-0xFF and single-symbol impulses (BASELINE.md inputs)."""
    k, p, S = 12, 5, 128
    c = rs.ReedSolomon(k, p, bits)
    cases = [np.zeros((k, S), np.uint8), np.full((k, S), 0xFF, np.uint8)]
    for r in (0, 5, 11):
        d = np.zeros((k, S), np.uint8)
        d[r, 3] = 1
        d[r, 40] = 0x80
        cases.append(d)
    for d in cases:
        ref = orc.encode(bits, k, p, d)
        shards = [d[i].copy() for i in range(k)] + [np.zeros(S, np.uint8) for _ in range(p)]
        c.encode(shards)
        assert np.array_equal(np.stack(shards[k:]), ref)


@pytest.mark.parametrize("bits", [16, 8])
def test_verify(bits):
    """testVerify (reedsolomon_test.go:313-411)."""
    k, p, S = 10, 4, 1024
    rng = np.random.default_rng(5)
    data = rand_data(rng, k, S)
    par, c = gpu_encode(bits, k, p, data)
    shards = [data[i].copy() for i in range(k)] + [par[i].copy() for i in range(p)]
    assert c.verify(shards)
    shards[0][0] ^= 0xFF
    assert not c.verify(shards)
    shards[0][0] ^= 0xFF
    shards[k + p - 1][S - 1] ^= 1
    assert not c.verify(shards)


RECON_CASES = [(4, 2, 128), (10, 4, 256), (16, 4, 64), (128, 32, 128), (33, 17, 64), (200, 100, 64), (5, 3, 64),
               (2, 1, 64), (64, 65, 64)]


@pytest.mark.parametrize("bits", [16, 8])
@pytest.mark.parametrize("k,p,S", RECON_CASES)
def test_reconstruct_round_trip(bits, k, p, S):
    if bits == 8 and k + p > 256:
        pytest.skip("GF(2^8) codec is for <= 256 shards")
    rng = np.random.default_rng(k + 31 * p + bits)
    data = rand_data(rng, k, S)
    par, c = gpu_encode(bits, k, p, data)
    full = [data[i].copy() for i in range(k)] + [par[i].copy() for i in range(p)]
    # the reference's codec carries state across calls (the GF(2^8) inversion
    # cache, leopard8.go:508-555, kept by default): the same call sequence on
    # the stateful oracle gives the expected bytes, which are the encoded
    # shards except on a stale cache hit
    o = orc.Oracle(bits, k, p)
    for trial in range(4):
        ne = int(rng.integers(1, p + 1)) if trial else p
        er = set(rng.choice(k + p, ne, replace=False).tolist())
        for recover_all in (True, False):
            sh = [None if i in er else full[i].copy() for i in range(k + p)]
            (c.reconstruct if recover_all else c.reconstruct_data)(sh)
            e, ref = o.reconstruct([None if i in er else full[i].copy() for i in range(k + p)], recover_all)
            assert e == 0
            for i in range(k + p):
                if i < k or recover_all:
                    assert np.array_equal(sh[i], ref[i]), f"shard {i} (erased={i in er}, all={recover_all})"
                    if bits == 16 or k + p > 64:
                        assert np.array_equal(sh[i], full[i])
                elif i in er:
                    assert sh[i] is None  # ReconstructData leaves missing parity missing


def test_reconstruct_errors():
    c = rs.New16(10, 4)
    S = 64
    sh = [np.zeros(S, np.uint8) for _ in range(14)]
    c.encode(sh)
    bad = [None] * 5 + sh[5:]
    with pytest.raises(rs.ErrTooFewShards):
        c.reconstruct(bad)
    with pytest.raises(rs.ErrShardNoData):
        c.reconstruct([None] * 14)
    with pytest.raises(rs.ErrShardSize):
        c.reconstruct([np.zeros(128, np.uint8)] + [None] + sh[2:])
    # nothing missing: no-op
    c.reconstruct(sh)


@pytest.fixture(scope="module")
def torch_dev():
    import torch

    return torch


@pytest.mark.parametrize("bits,k,p,S", [(16, 128, 32, 4096), (8, 10, 4, 4096), (16, 20, 8, 1024), (16, 300, 64, 256)])
def test_device_encode_strided_and_table(torch_dev, bits, k, p, S):
    torch = torch_dev
    rng = np.random.default_rng(11)
    data = rand_data(rng, k, S)
    ref = orc.encode(bits, k, p, data)
    c = rs.ReedSolomon(k, p, bits)
    slab = torch.zeros((k + p, S), dtype=torch.uint8, device="cuda")
    slab[:k] = torch.from_numpy(data).cuda()
    c.encode_dev(slab)
    torch.cuda.synchronize()
    assert np.array_equal(slab[k:].cpu().numpy(), ref)
    # separately allocated rows (non-strided -> device row table)
    rows = [torch.from_numpy(data[i].copy()).cuda() for i in range(k)] + \
           [torch.zeros(S, dtype=torch.uint8, device="cuda") for _ in range(p)]
    c.encode_dev(rows)
    torch.cuda.synchronize()
    assert np.array_equal(np.stack([r.cpu().numpy() for r in rows[k:]]), ref)
    assert c.verify_dev(rows)
    rows[k][5] ^= 1
    assert not c.verify_dev(rows)


def test_device_batch(torch_dev):
    torch = torch_dev
    k, p, S, n = 16, 8, 2048, 5
    rng = np.random.default_rng(3)
    c = rs.New16(k, p)
    slab = torch.zeros((n, k + p, S), dtype=torch.uint8, device="cuda")
    datas = [rand_data(rng, k, S) for _ in range(n)]
    for j in range(n):
        slab[j, :k] = torch.from_numpy(datas[j]).cuda()
    c.encode_dev_batch(slab)
    torch.cuda.synchronize()
    for j in range(n):
        assert np.array_equal(slab[j, k:].cpu().numpy(), orc.encode(16, k, p, datas[j]))


def test_device_reconstruct(torch_dev):
    torch = torch_dev
    k, p, S = 128, 32, 8192
    rng = np.random.default_rng(9)
    data = rand_data(rng, k, S)
    c = rs.New16(k, p)
    slab = torch.zeros((k + p, S), dtype=torch.uint8, device="cuda")
    slab[:k] = torch.from_numpy(data).cuda()
    c.encode_dev(slab)
    torch.cuda.synchronize()
    full = slab.clone()
    er = rng.choice(k + p, p, replace=False)
    present = np.ones(k + p, bool)
    present[er] = False
    slab[torch.from_numpy(er).cuda()] = 0
    c.reconstruct_dev(slab, present)
    torch.cuda.synchronize()
    assert torch.equal(slab, full)


# ------------------------------------------------------------------ BASELINE configs at full size
def _window_check(bits, k, p, data_dev, par_dev, rng, width=4096, nwin=3):
    """GPU parity on random 64-B-aligned column windows == oracle on the window."""
    S = data_dev.shape[1]
    for _ in range(nwin):
        a = int(rng.integers(0, (S - width) // 64 + 1)) * 64
        d = data_dev[:, a:a + width].cpu().numpy()
        ref = orc.encode(bits, k, p, np.ascontiguousarray(d))
        assert np.array_equal(par_dev[:, a:a + width].cpu().numpy(), ref), f"window @{a}"


@pytest.mark.parametrize("bits,k,p,S", [(8, 10, 4, 1 << 20), (16, 128, 32, 1 << 20), (16, 1024, 256, 256 << 10)])
def test_baseline_config_encode(torch_dev, bits, k, p, S):
    """C2 / C3 / C5 encode at full size: column-window parity + verify."""
    torch = torch_dev
    g = torch.Generator(device="cuda")
    g.manual_seed(0x5EED)
    slab = torch.randint(0, 256, (k + p, S), dtype=torch.uint8, device="cuda", generator=g)
    c = rs.ReedSolomon(k, p, bits)
    c.encode_dev(slab)
    torch.cuda.synchronize()
    rng = np.random.default_rng(1)
    _window_check(bits, k, p, slab[:k], slab[k:], rng, width=2048 if k > 512 else 4096)
    assert c.verify_dev(slab)


def test_baseline_c3_full_oracle(torch_dev):
    """C3 (128+32 x 1 MiB) bit-exact against the oracle over the whole stripe."""
    torch = torch_dev
    k, p, S = 128, 32, 1 << 20
    rng = np.random.default_rng(0x5EED)
    data = rand_data(rng, k, S)
    ref = orc.encode(16, k, p, data)
    slab = torch.zeros((k + p, S), dtype=torch.uint8, device="cuda")
    slab[:k] = torch.from_numpy(data).cuda()
    rs.New16(k, p).encode_dev(slab)
    torch.cuda.synchronize()
    assert np.array_equal(slab[k:].cpu().numpy(), ref)


def test_baseline_c5_full_port(torch_dev):
    """C5 (1024+256 x 256 KiB, m = 256: the LDS-resident encode) bit-exact over
    the whole stripe against the AVX2 port of the reference encode, which
    tests/test_oracle.py pins to the scalar oracle (including 1024+256)."""
    if not orc.simd_available():
        pytest.skip("no AVX2 on this host")
    torch = torch_dev
    k, p, S = 1024, 256, 256 << 10
    rng = np.random.default_rng(0xC5)
    data = rand_data(rng, k, S)
    ref = orc.encode_simd(k, p, data, min(16, os.cpu_count() or 1))
    slab = torch.zeros((k + p, S), dtype=torch.uint8, device="cuda")
    slab[:k] = torch.from_numpy(data).cuda()
    c = rs.New16(k, p)
    c.encode_dev(slab)
    torch.cuda.synchronize()
    assert np.array_equal(slab[k:].cpu().numpy(), ref)
    assert c.verify_dev(slab)


def test_baseline_c4_reconstruct(torch_dev):
    """C4: 128+32 x 1 MiB, 32 random erasures (fixed seed) + worst case first 32 data shards."""
    torch = torch_dev
    k, p, S = 128, 32, 1 << 20
    g = torch.Generator(device="cuda")
    g.manual_seed(7)
    slab = torch.randint(0, 256, (k + p, S), dtype=torch.uint8, device="cuda", generator=g)
    c = rs.New16(k, p)
    c.encode_dev(slab)
    torch.cuda.synchronize()
    full = slab.clone()
    rng = np.random.default_rng(0x5EED)
    for er in (rng.choice(k + p, p, replace=False), np.arange(p)):
        present = np.ones(k + p, bool)
        present[er] = False
        slab[torch.from_numpy(np.asarray(er)).cuda()] = 0
        c.reconstruct_dev(slab, present)
        torch.cuda.synchronize()
        assert torch.equal(slab, full)


@pytest.mark.parametrize("bits,k,p,S,world", [(16, 128, 32, 256 << 10, 8), (16, 1024, 256, 32 << 10, 4), (8, 10, 4, 1 << 16, 2)])
def test_byte_range_sharding_on_gpu(torch_dev, bits, k, p, S, world):
    """C5-style byte-range split: every rank's slice encoded by the engine
    (all slices on this one GPU) reassembles to the whole-stripe parity."""
    torch = torch_dev
    from reedsolomon16_amd import dist as rsd

    g = torch.Generator(device="cuda")
    g.manual_seed(11)
    full = torch.randint(0, 256, (k + p, S), dtype=torch.uint8, device="cuda", generator=g)
    c = rs.ReedSolomon(k, p, bits)
    whole = full.clone()
    c.encode_dev(whole)
    sharded = full.clone()
    for r in range(world):
        rsd.encode_sharded(sharded, r, world, rsd.gpu_encode_fn(c))
    torch.cuda.synchronize()
    assert torch.equal(sharded, whole)
    present = np.ones(k + p, bool)
    er = np.random.default_rng(5).choice(k + p, p, replace=False)
    present[er] = False
    broken = whole.clone()
    broken[torch.from_numpy(er).cuda()] = 0
    for r in range(world):
        rsd.reconstruct_sharded(broken, present, r, world, rsd.gpu_reconstruct_fn(c))
    torch.cuda.synchronize()
    assert torch.equal(broken, whole)


def test_c5_shape_world8_byte_split(torch_dev):
    """The exact C5 configuration (1024 + 256 x 256 KiB, configs[4]) split over
    8 ranks by byte range, all ranks emulated on this GPU through the batched
    path bench.py --split bytes uses (dist.encode_sharded_batch: one strided
    launch per rank over 2 stripes): the reassembled parity equals the
    whole-stripe encode, and a 256-erasure reconstruct per rank slice restores
    every row (leopard16.go:778-792 column independence)."""
    torch = torch_dev
    from reedsolomon16_amd import dist as rsd

    k, p, S, world, B = 1024, 256, 256 << 10, 8, 2
    g = torch.Generator(device="cuda")
    g.manual_seed(0xC5)
    slab = torch.randint(0, 256, (B, k + p, S), dtype=torch.uint8, device="cuda", generator=g)
    c = rs.New16(k, p)
    whole = slab.clone()
    c.encode_dev_batch(whole)
    for r in range(world):
        lo, hi = rsd.byte_range(S, r, world)
        assert hi - lo == S // world
        rsd.encode_sharded_batch(slab, r, world, c)
    torch.cuda.synchronize()
    assert torch.equal(slab, whole)
    # one stripe, 256 random erasures, reconstructed slice by slice
    present = np.ones(k + p, bool)
    er = np.random.default_rng(0xC5).choice(k + p, p, replace=False)
    present[er] = False
    broken = whole[0].clone()
    broken[torch.from_numpy(er).cuda()] = 0
    for r in range(world):
        rsd.reconstruct_sharded(broken, present, r, world, rsd.gpu_reconstruct_fn(c))
    torch.cuda.synchronize()
    assert torch.equal(broken, whole[0])


# Host-resident pipeline (rs_encode / rs_verify / rs_reconstruct): small
# segment widths force many segments, a ragged last segment and reuse of every
# staging slab; rows as one slab (2-D copies) and as scattered arrays
# (per-row copies); pinned and pageable memory.
@pytest.mark.parametrize("bits,k,p,S,seg", [(16, 128, 32, 64 * 37, 256), (16, 10, 4, 64 * 50, 640),
                                            (8, 10, 4, 64 * 33, 128), (16, 300, 64, 64 * 9, 128),
                                            (8, 100, 28, 64 * 20, 64 * 7)])
@pytest.mark.parametrize("layout", ["slab", "scattered", "pinned"])
def test_host_pipeline_segments(bits, k, p, S, seg, layout):
    rng = np.random.default_rng(S + seg + k)
    data = rand_data(rng, k, S)
    ref = orc.encode(bits, k, p, data)
    c = rs.ReedSolomon(k, p, bits)
    c.set_host_segment(seg)
    if layout == "scattered":
        shards = [np.ascontiguousarray(data[i]) for i in range(k)] + [np.zeros(S, np.uint8) for _ in range(p)]
    else:
        shards = c.alloc_aligned(S, pinned=(layout == "pinned"))
        for i in range(k):
            shards[i][:] = data[i]
    c.encode(shards)
    assert np.array_equal(np.stack(shards[k:]), ref)
    assert c.verify(shards)
    shards[k + p - 1][S - 1] ^= 0x40  # last byte of the last segment
    assert not c.verify(shards)
    shards[k + p - 1][S - 1] ^= 0x40
    er = set(rng.choice(k + p, p, replace=False).tolist())
    # missing = nil (scattered) or an empty view (slab); rebuilt rows come back as fresh arrays
    gone = None if layout == "scattered" else np.zeros(0, np.uint8)
    broken = [gone if i in er else shards[i] for i in range(k + p)]
    out = c.reconstruct(broken)
    full = np.concatenate([data, ref])
    for i in range(k + p):
        assert np.array_equal(out[i], full[i]), i


def test_host_pipeline_c3_pinned_matches_device(torch_dev):
    torch = torch_dev
    k, p, S = 128, 32, 1 << 20
    c = rs.New16(k, p)
    shards = c.alloc_aligned(S, pinned=True)
    rng = np.random.default_rng(77)
    for i in range(k):
        shards[i][:] = rng.integers(0, 256, S, dtype=np.uint8)
    c.encode(shards)
    dev = torch.from_numpy(np.stack(shards[:k] + [np.zeros(S, np.uint8)] * p)).cuda()
    c.encode_dev(dev)
    torch.cuda.synchronize()
    assert np.array_equal(dev[k:].cpu().numpy(), np.stack(shards[k:]))
    assert c.verify(shards)


@pytest.mark.parametrize("k,p", [(128, 32), (100, 28), (10, 4), (300, 100), (700, 200), (1024, 256)])
def test_reconstruct_subfield_equals_full_field(torch_dev, paths, k, p):
    """The LDS reconstruct in GF(2^8)-subfield coordinates (every pass for
    n <= 256, all but the first passes of each transform at n = 512..2048:
    kernels.hip BigSub) and the full-field table path (rs_debug_set_path("sub", 0)) rebuild
    identical bytes."""
    torch = torch_dev
    S = 4096 + 192
    g = torch.Generator(device="cuda")
    g.manual_seed(k + p)
    full = torch.randint(0, 256, (k + p, S), dtype=torch.uint8, device="cuda", generator=g)
    rs.New16(k, p).encode_dev(full)
    torch.cuda.synchronize()
    present = np.ones(k + p, bool)
    present[np.random.default_rng(k).choice(k + p, p, replace=False)] = False
    out = []
    for nosub in ("0", "1"):
        paths("sub", int(nosub != "1"))
        c = rs.New16(k, p)
        broken = full.clone()
        broken[torch.from_numpy(np.flatnonzero(~present)).cuda()] = 0
        c.reconstruct_dev(broken, present)
        torch.cuda.synchronize()
        out.append(broken)
    assert torch.equal(out[0], full) and torch.equal(out[1], full)


def test_bitsliced_equals_split_kernel(torch_dev, paths):
    """C3 geometry: bit-sliced kernel (default) and the split perm kernel (rs_debug_set_path("bs", 0)) agree."""
    torch = torch_dev
    k, p, S = 128, 32, 4096 * 4
    g = torch.Generator(device="cuda")
    g.manual_seed(3)
    base = torch.randint(0, 256, (k + p, S), dtype=torch.uint8, device="cuda", generator=g)
    outs = []
    for bs in ("1", "0"):
        paths("bs", int(bs))
        c = rs.New16(k, p)
        assert c.encode_path == ("bs16-m32" if bs == "1" else "split16-m32")
        slab = base.clone()
        c.encode_dev(slab)
        torch.cuda.synchronize()
        outs.append(slab[k:].clone())
    assert torch.equal(outs[0], outs[1])


# Host reconstruct whose output rows are pinned (a C caller's preallocated
# rows): the rebuilt rows go device -> host directly; fresh pageable rows (the
# Python mirror, Go's make) go through the pinned bounce slab.  Both at C4's
# size with the default segment width (several segments).
@pytest.mark.parametrize("outputs", ["pinned", "pageable"])
def test_host_reconstruct_c4_output_memory(outputs):
    import ctypes as C

    from reedsolomon16_amd import codec as rc

    k, p, S = 128, 32, 1 << 20
    c = rs.New16(k, p)
    shards = c.alloc_aligned(S, pinned=True)
    rng = np.random.default_rng(4)
    for i in range(k):
        shards[i][:] = rng.integers(0, 256, S, dtype=np.uint8)
    c.encode(shards)
    full = [s.copy() for s in shards]
    er = sorted(rng.choice(k + p, p, replace=False).tolist())
    outs = {i: (rc.alloc_pinned(S) if outputs == "pinned" else np.empty(S, np.uint8)) for i in er}
    for o in outs.values():
        o[:] = 0xA5
    ptrs = (C.c_void_p * (k + p))(*[(outs[i] if i in outs else shards[i]).ctypes.data for i in range(k + p)])
    lens = (C.c_size_t * (k + p))(*[0 if i in outs else S for i in range(k + p)])
    assert c._L.rs_reconstruct(c._h, ptrs, lens, k + p, 1) == 0
    for i in er:
        assert lens[i] == S
        assert np.array_equal(outs[i], full[i]), i


# The Python mirror's Go-capacity form: a missing shard passed as
# EmptyShard(row) (Go: shards[i][:0] of an AllocAligned row) is rebuilt into
# that row -- pinned here, so the copy-out is direct -- and the list entry
# becomes that same memory; a plain empty array still gets a new array (Go's make).
def test_host_reconstruct_into_capacity():
    k, p, S = 128, 32, 1 << 18
    c = rs.New16(k, p)
    shards = c.alloc_aligned(S, pinned=True)
    rng = np.random.default_rng(5)
    for i in range(k):
        shards[i][:] = rng.integers(0, 256, S, dtype=np.uint8)
    c.encode(shards)
    full = [s.copy() for s in shards]
    er = sorted(rng.choice(k + p, p, replace=False).tolist())
    rows = {i: shards[i] for i in er}
    for i in er:
        rows[i][:] = 0x5A
    work = list(shards)
    for j, i in enumerate(er):
        work[i] = rs.EmptyShard(rows[i]) if j % 2 == 0 else np.zeros(0, np.uint8)
    c.reconstruct(work)
    for j, i in enumerate(er):
        assert np.array_equal(work[i], full[i]), i
        same = work[i].ctypes.data == rows[i].ctypes.data
        assert same == (j % 2 == 0), i
    # a capacity smaller than the shard size is not used (Go: make)
    work = [f.copy() for f in full]
    small = np.zeros(S // 2, np.uint8)
    work[er[0]] = rs.EmptyShard(small)
    c.reconstruct(work)
    assert np.array_equal(work[er[0]], full[er[0]]) and not np.any(small)


# Host reconstruct over pinned rows moves them with zero-copy kernels (one per
# segment and direction, the device reading / writing the mapped rows,
# codec.cpp zc_rows); rs_debug_set_path("zc", mask) picks the directions (bit 0 in,
# bit 1 out; 0 keeps the per-run copies).
# Both paths against the oracle: rows from one slab and from separate pinned
# allocations, a shard size of several segments with a ragged last one, both
# fields, and a pageable input row (no zero copy for that call).
@pytest.mark.parametrize("zc", [3, 1, 2, 0])
@pytest.mark.parametrize("bits,k,p,S", [(16, 128, 32, 3 * (1 << 18) + 192), (16, 100, 28, 1 << 16), (8, 10, 4, 1 << 17)])
@pytest.mark.parametrize("rows", ["slab", "separate", "one_pageable", "registered"])
def test_host_reconstruct_zero_copy(paths, zc, bits, k, p, S, rows):
    from reedsolomon16_amd import codec as rc

    paths("zc", zc)
    c = rs.ReedSolomon(k, p, bits)
    c.set_host_segment(1 << 16)  # several segments per call
    rng = np.random.default_rng(k + S + zc)
    data = rand_data(rng, k, S)
    reg = None
    if rows == "slab":
        shards = c.alloc_aligned(S, pinned=True)
    elif rows == "registered":
        # an ordinary host slab pinned in place (rs_host_register: Go's slab held by runtime.Pinner)
        raw = np.zeros((k + p) * S + 4096, np.uint8)
        o = (-raw.ctypes.data) % 4096
        reg = raw[o:o + (k + p) * S]
        assert c._L.rs_host_register(reg.ctypes.data, reg.nbytes) == 0
        shards = [reg[i * S:(i + 1) * S] for i in range(k + p)]
    else:
        shards = [rc.alloc_pinned(S) for _ in range(k + p)]
        if rows == "one_pageable":
            shards[3] = np.empty(S, np.uint8)
    for i in range(k):
        shards[i][:] = data[i]
    c.encode(shards)
    full = [np.array(s, copy=True) for s in shards]
    er = sorted(rng.choice(k + p, p, replace=False).tolist())
    if rows == "one_pageable" and 3 in er:
        er = [i for i in er if i != 3] + [min(set(range(k + p)) - set(er) - {3})]
    work = list(shards)
    for i in er:
        work[i][:] = 0xA5
        work[i] = rs.EmptyShard(work[i])
    c.reconstruct(work)
    ref = orc.Oracle(bits, k, p)
    e, out = ref.reconstruct([None if i in er else full[i] for i in range(k + p)], True)
    assert e == 0
    for i in er:
        assert np.array_equal(work[i], full[i]), i
        assert np.array_equal(out[i], full[i]), i
    if reg is not None:
        assert c._L.rs_host_unregister(reg.ctypes.data) == 0


def test_zero_copy_rows_checked_at_both_ends():
    """A row that starts in registered (mapped) host memory and runs past the
    registered range (advisor finding, round 5) must not go to the zero-copy
    kernels, which would read or write unmapped addresses: the codec checks
    both ends of every row (codec.cpp zc_rows, probed through
    rs_debug_zc_rows: pointer queries only, nothing touches the short row)."""
    import ctypes as C

    L = rs.lib()
    S, n = 1 << 16, 4
    raw = np.zeros(n * S + 8192, np.uint8)
    o = (-raw.ctypes.data) % 4096
    slab = raw[o:o + n * S]
    rows = (C.c_void_p * n)(*[slab.ctypes.data + i * S for i in range(n)])
    assert L.rs_debug_zc_rows(rows, n, S) == 0  # pageable
    assert L.rs_host_register(slab.ctypes.data, n * S) == 0
    try:
        assert L.rs_debug_zc_rows(rows, n, S) == 1  # every row mapped end to end
    finally:
        assert L.rs_host_unregister(slab.ctypes.data) == 0
    # registered up to the middle of the last row (a page-aligned cut)
    assert L.rs_host_register(slab.ctypes.data, (n - 1) * S + S // 2) == 0
    try:
        assert L.rs_debug_zc_rows(rows, n - 1, S) == 1
        assert L.rs_debug_zc_rows(rows, n, S) == 0
        one = (C.c_void_p * 1)(slab.ctypes.data + (n - 1) * S)
        assert L.rs_debug_zc_rows(one, 1, S // 2) == 1 and L.rs_debug_zc_rows(one, 1, S) == 0
    finally:
        assert L.rs_host_unregister(slab.ctypes.data) == 0
    # two separate pinned blocks: a "row" reaching from one into the next is refused
    a, b = rs.alloc_pinned(S), rs.alloc_pinned(S)
    r = (C.c_void_p * 1)(a.ctypes.data + S // 2)
    assert L.rs_debug_zc_rows(r, 1, S // 2) == 1
    if b.ctypes.data != a.ctypes.data + S:  # (adjacent only by chance)
        assert L.rs_debug_zc_rows(r, 1, S) == 0


# Batched device reconstruct (rs_reconstruct_dev_batch): one erasure pattern
# over many stripes in one launch, rows at a padded stride and stripes at a
# padded stripe stride; n <= 256 codecs run the LDS kernel with grid.y =
# stripe, n > 256 codecs go stripe by stripe.  Rebuilt bytes must equal the
# encoded stripes (data and parity erasures), and ReconstructData must leave
# erased parity rows untouched.
@pytest.mark.parametrize("bits,k,p,S,ns", [(16, 128, 32, 1 << 16, 5), (8, 10, 4, 1 << 14, 7), (16, 300, 100, 4096, 3),
                                           (16, 20, 10, 2048, 1)])
def test_reconstruct_dev_batch(torch_dev, bits, k, p, S, ns):
    torch = torch_dev
    RS, total = S + 3072, k + p
    SS = total * RS + 4096
    buf = torch.zeros(ns * SS, dtype=torch.uint8, device="cuda")
    slab = buf.as_strided((ns, total, S), (SS, RS, 1))
    g = torch.Generator(device="cuda")
    g.manual_seed(k + p + ns)
    slab[:, :k] = torch.randint(0, 256, (ns, k, S), dtype=torch.uint8, device="cuda", generator=g)
    c = rs.ReedSolomon(k, p, bits)
    c.encode_dev_batch(slab)
    torch.cuda.synchronize()
    full = slab.clone()
    rng = np.random.default_rng(k + p + S)
    er = rng.choice(total, p, replace=False)
    present = np.ones(total, bool)
    present[er] = False
    for recover_all in (True, False):
        slab[:, torch.from_numpy(er).cuda()] = 0
        c.reconstruct_dev_batch(slab, present, recover_all)
        torch.cuda.synchronize()
        for z in range(ns):
            for i in range(total):
                if i < k or recover_all:
                    assert torch.equal(slab[z, i], full[z, i]), (recover_all, z, i)
                elif not present[i]:
                    assert not torch.any(slab[z, i]), (z, i)


def test_reconstruct_sharded_batch_world8(torch_dev):
    """dist.reconstruct_sharded_batch: 8 byte-range slices of the same stripes,
    each rebuilt in one launch on its own, reassemble the encoded stripes."""
    from reedsolomon16_amd import dist as rsd
    torch = torch_dev
    k, p, S, ns, world = 128, 32, 1 << 15, 3, 8
    g = torch.Generator(device="cuda")
    g.manual_seed(88)
    slab = torch.zeros((ns, k + p, S), dtype=torch.uint8, device="cuda")
    slab[:, :k] = torch.randint(0, 256, (ns, k, S), dtype=torch.uint8, device="cuda", generator=g)
    c = rs.New16(k, p)
    c.encode_dev_batch(slab)
    torch.cuda.synchronize()
    full = slab.clone()
    er = np.random.default_rng(88).choice(k + p, p, replace=False)
    present = np.ones(k + p, bool)
    present[er] = False
    slab[:, torch.from_numpy(er).cuda()] = 0
    for r in range(world):
        rsd.reconstruct_sharded_batch(slab, present, r, world, c)
    torch.cuda.synchronize()
    assert torch.equal(slab, full)


@pytest.mark.parametrize("bits,k,p,S,ns", [(16, 128, 32, 1 << 16, 6), (8, 10, 4, 1 << 14, 5), (16, 1024, 256, 4096, 2)])
def test_verify_dev_batch(torch_dev, bits, k, p, S, ns):
    """rs_verify_dev_batch: all stripes clean -> True; one flipped byte in any
    one stripe (data or parity row) -> False; restored -> True."""
    torch = torch_dev
    RS = S + 3072
    SS = (k + p) * RS
    buf = torch.zeros(ns * SS, dtype=torch.uint8, device="cuda")
    slab = buf.as_strided((ns, k + p, S), (SS, RS, 1))
    g = torch.Generator(device="cuda")
    g.manual_seed(k + ns)
    slab[:, :k] = torch.randint(0, 256, (ns, k, S), dtype=torch.uint8, device="cuda", generator=g)
    c = rs.ReedSolomon(k, p, bits)
    c.encode_dev_batch(slab)
    assert c.verify_dev_batch(slab)
    rng = np.random.default_rng(ns)
    for z, row in ((ns - 1, 0), (0, k + p - 1), (ns // 2, k)):
        col = int(rng.integers(0, S))
        old = slab[z, row, col].item()
        slab[z, row, col] = old ^ 0x10
        assert not c.verify_dev_batch(slab), (z, row, col)
        slab[z, row, col] = old
        assert c.verify_dev_batch(slab)


# Codec scratch shared across caller streams: device-resident encodes return
# before their kernels finish, so a second call on another stream must not
# overwrite the row-pointer table (non-strided rows) or the multi-pass work
# rows (m > 256) the first call's kernels are still reading.
@pytest.mark.parametrize("bits,k,p,S,layout", [(16, 128, 32, 1 << 16, "table"), (8, 10, 4, 1 << 18, "table"),
                                               (16, 300, 300, 1 << 12, "slab")])
def test_device_encode_two_streams(torch_dev, bits, k, p, S, layout):
    torch = torch_dev
    rng = np.random.default_rng(k + p + S)
    datas = [rand_data(rng, k, S) for _ in range(2)]
    c = rs.ReedSolomon(k, p, bits)
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    outs = []
    for j in range(2):
        if layout == "table":
            rows = [torch.from_numpy(datas[j][i].copy()).cuda() for i in range(k)] + \
                   [torch.zeros(S, dtype=torch.uint8, device="cuda") for _ in range(p)]
        else:
            rows = torch.zeros((k + p, S), dtype=torch.uint8, device="cuda")
            rows[:k] = torch.from_numpy(datas[j]).cuda()
        outs.append(rows)
    torch.cuda.synchronize()
    for j in range(2):  # back to back, no synchronization in between
        c.encode_dev(outs[j], stream=streams[j])
    torch.cuda.synchronize()
    for j in range(2):
        got = np.stack([r.cpu().numpy() for r in outs[j][k:]])
        assert np.array_equal(got, orc.encode(bits, k, p, datas[j])), f"stream {j}"


# Unit-width variants (rs_debug_set_path("unit_width") forces the per-launch choice): the
# 64-byte and 128-byte LDS tiles of the LDS-resident encode / reconstruct
# (both fields, both coordinate systems), and the 4- and 16-byte GF(2^8)
# register units, at sizes the oracle finishes in seconds.
@pytest.mark.parametrize("width", ["narrow", "wide"])
@pytest.mark.parametrize("bits,k,p,S", [(8, 10, 4, 4096), (8, 100, 28, 4096 + 192), (16, 100, 28, 4096 + 192),
                                        (16, 70, 40, 2048), (8, 70, 40, 2048), (16, 128, 32, 4096 + 640),
                                        (16, 100, 100, 2048), (8, 100, 100, 2048), (16, 700, 200, 1024)])
def test_unit_width_variants(paths, width, bits, k, p, S):
    paths("unit_width", 1 if width == "narrow" else 0)
    paths("bs", 0)
    rng = np.random.default_rng(k + p + S + bits)
    data = rand_data(rng, k, S)
    ref = orc.encode(bits, k, p, data)
    c = rs.ReedSolomon(k, p, bits)
    shards = [np.ascontiguousarray(data[i]) for i in range(k)] + [np.zeros(S, np.uint8) for _ in range(p)]
    c.encode(shards)
    assert np.array_equal(np.stack(shards[k:]), ref), c.encode_path
    full = [data[i] for i in range(k)] + [ref[i] for i in range(p)]
    for nosub in (["0", "1"] if bits == 16 else ["0"]):
        paths("sub", int(nosub != "1"))
        c2 = rs.ReedSolomon(k, p, bits)
        er = set(rng.choice(k + p, p, replace=False).tolist())
        sh = [None if i in er else full[i].copy() for i in range(k + p)]
        c2.reconstruct(sh)
        for i in range(k + p):
            assert np.array_equal(sh[i], full[i]), (nosub, i)


@pytest.mark.parametrize("strided", ["data", "parity"])
def test_device_encode_mixed_layout(torch_dev, strided):
    """One row set equally spaced (a slab), the other scattered (rows of a
    buffer in permuted order): both must go through the row table (round 1
    passed a null table for the strided set)."""
    torch = torch_dev
    k, p, S = 16, 8, 4096
    rng = np.random.default_rng(7)
    data = rand_data(rng, k, S)
    ref = orc.encode(16, k, p, data)
    c = rs.New16(k, p)
    slab = torch.zeros((k + p, S), dtype=torch.uint8, device="cuda")
    slab[:k] = torch.from_numpy(data).cuda()
    rows = list(slab)
    lo, n = (k, p) if strided == "data" else (0, k)
    perm = np.r_[1, 0, 2:n][rng.permutation(n)] if n > 2 else np.arange(n)[::-1]
    scat = torch.zeros((n, S), dtype=torch.uint8, device="cuda")
    scat[torch.from_numpy(perm).cuda()] = slab[lo:lo + n]
    for i in range(n):
        rows[lo + i] = scat[int(perm[i])]
    c.encode_dev(rows)
    torch.cuda.synchronize()
    assert np.array_equal(np.stack([r.cpu().numpy() for r in rows[k:]]), ref)


@pytest.mark.parametrize("k,p,n", [(128, 32, (1 << 20) * 128 - 5), (10, 4, 1000), (4, 2, 64)])
def test_split_into_device_slab_encode_join(torch_dev, k, p, n):
    """rs_split straight into an HBM slab (host bytes -> device rows, padding and
    parity rows zeroed on the device), encode_dev on it, rs_join back (device
    rows -> host): the data round-trips and the parity is the oracle's."""
    torch = torch_dev
    c = rs.New16(k, p)
    data = np.random.default_rng(n).integers(0, 256, n, dtype=np.uint8)
    slab = c.split_dev(data)
    per = c.split_shard_size(n)
    assert slab.shape == (k + p, per)
    host = c.split(data)
    assert np.array_equal(slab.cpu().numpy(), np.stack(host))
    c.encode_dev(slab)
    torch.cuda.synchronize()
    if k * per <= (16 << 20):
        assert np.array_equal(slab[k:].cpu().numpy(), orc.encode(16, k, p, np.stack(host[:k])))
    assert np.array_equal(c.join_dev(slab, n), data)
    # device -> device split (data already in HBM)
    dd = torch.from_numpy(data).cuda()
    slab2 = c.split_dev(dd)
    assert torch.equal(slab2[:k], slab[:k])


def test_encode_async_stream_of_blocks():
    """rs_encode_async over a stream of blocks (the rsStream16.encode loop,
    streaming16.go:1229-1318): several stripes queued back to back through
    the three-stream pipeline, pinned rows, then waited; each equals the
    oracle.  Small segments force the slab rotation to continue across calls."""
    k, p, S, nblk = 20, 8, 64 * 40, 6
    c = rs.New16(k, p)
    c.set_host_segment(64 * 7)
    rng = np.random.default_rng(99)
    blocks, tickets = [], []
    for b in range(nblk):
        sh = c.alloc_aligned(S, pinned=True)
        for i in range(k):
            sh[i][:] = rng.integers(0, 256, S, dtype=np.uint8)
        blocks.append(sh)
        tickets.append(c.encode_async(sh))
    for t in tickets[::-1]:
        t.wait()
    assert all(t.done() for t in tickets)
    for sh in blocks:
        assert np.array_equal(np.stack(sh[k:]), orc.encode(16, k, p, np.stack(sh[:k])))
    # pageable parity rows: the call completes synchronously, same result
    sh = [rng.integers(0, 256, S, dtype=np.uint8) for _ in range(k)] + [np.zeros(S, np.uint8) for _ in range(p)]
    t = c.encode_async(sh)
    t.wait()
    assert np.array_equal(np.stack(sh[k:]), orc.encode(16, k, p, np.stack(sh[:k])))


def test_encode_async_mixed_sizes_then_sync_verify():
    """Async encodes of different shard sizes (a short last stripe) queued
    back to back, then a synchronous verify and encode before any ticket is
    waited on: the staging buffers sit at fixed addresses, so a narrower
    call's buffer never lands inside a buffer an earlier call still reads."""
    k, p = 20, 8
    c = rs.New16(k, p)
    c.set_host_segment(0)
    rng = np.random.default_rng(7)
    blocks, tickets = [], []
    for S in (64 * 4000, 64 * 37, 64 * 4000, 64 * 5, 64 * 1500):
        sh = c.alloc_aligned(S, pinned=True)
        for i in range(k):
            sh[i][:] = rng.integers(0, 256, S, dtype=np.uint8)
        blocks.append(sh)
        tickets.append(c.encode_async(sh))
    # sync calls while the async ones are in flight
    vsh = c.alloc_aligned(64 * 900, pinned=True)
    for i in range(k):
        vsh[i][:] = rng.integers(0, 256, 64 * 900, dtype=np.uint8)
    c.encode(vsh)
    assert c.verify(vsh)
    for t in tickets:
        t.wait()
    for sh in blocks:
        assert np.array_equal(np.stack(sh[k:]), orc.encode(16, k, p, np.stack(sh[:k])))
    assert np.array_equal(np.stack(vsh[k:]), orc.encode(16, k, p, np.stack(vsh[:k])))


# 256-point transforms: reconstruct with n = 256 and encode with m = 256
# against the oracle, over several erasure classes and ragged tiles.
@pytest.mark.parametrize("k,p,S", [(128, 32, 2048 + 64), (100, 100, 512), (190, 33, 256), (129, 64, 320)])
def test_n256_reconstruct(k, p, S):
    rng = np.random.default_rng(k * 3 + p + S)
    data = rand_data(rng, k, S)
    par, c = gpu_encode(16, k, p, data)
    full = [data[i].copy() for i in range(k)] + [par[i].copy() for i in range(p)]
    o = orc.Oracle(16, k, p)
    patterns = [list(range(p)), list(range(k, k + p)), [0], [k + p - 1], [3, k + 1],
                rng.choice(k + p, p, replace=False).tolist(), rng.choice(k + p, max(1, p // 4), replace=False).tolist()]
    for er in patterns:
        er = set(er)
        sh = [None if i in er else full[i].copy() for i in range(k + p)]
        c.reconstruct(sh)
        e, ref = o.reconstruct([None if i in er else full[i].copy() for i in range(k + p)])
        assert e == 0
        for i in range(k + p):
            assert np.array_equal(sh[i], full[i]), f"shard {i} (erased={i in er})"
            assert np.array_equal(sh[i], ref[i]), f"shard {i} vs oracle"


def test_n256_reconstruct_full_field(paths):
    """n = 256 reconstruct with transforms outside subfield coordinates (rs_debug_set_path("sub", 0))."""
    paths("sub", 0)
    k, p, S = 128, 32, 1024
    rng = np.random.default_rng(77)
    data = rand_data(rng, k, S)
    par, c = gpu_encode(16, k, p, data)
    full = [data[i].copy() for i in range(k)] + [par[i].copy() for i in range(p)]
    er = set(rng.choice(k + p, p, replace=False).tolist())
    sh = [None if i in er else full[i].copy() for i in range(k + p)]
    c.reconstruct(sh)
    for i in range(k + p):
        assert np.array_equal(sh[i], full[i])


@pytest.mark.parametrize("k,p,S", [(300, 256, 256 + 64), (257, 129, 256), (1024, 256, 512), (200, 200, 64)])
def test_m256_encode_verify(torch_dev, k, p, S):
    torch = torch_dev
    rng = np.random.default_rng(k + p * 5 + S)
    B = 3
    datas = [rand_data(rng, k, S) for _ in range(B)]
    slab = torch.zeros((B, k + p, S), dtype=torch.uint8, device="cuda")
    for j in range(B):
        slab[j, :k] = torch.from_numpy(datas[j]).cuda()
    c = rs.New16(k, p)
    assert c.encode_path == "lds-m256"
    c.encode_dev_batch(slab)
    torch.cuda.synchronize()
    for j in range(B):
        assert np.array_equal(slab[j, k:].cpu().numpy(), orc.encode(16, k, p, datas[j])), f"stripe {j}"
    one = slab[1].clone()
    assert c.verify_dev(one)
    one[k + p - 1, S - 1] ^= 1
    assert not c.verify_dev(one)


def test_reconstruct_dev_async_ring_and_plan_eviction(torch_dev):
    """rs_reconstruct_dev on a caller stream returns without waiting: 40 calls
    back to back over 20 erasure patterns (more than the 8 row-pointer ring
    slots and the 16 cached device plans, so slots are reused and plans
    evicted while launches are in flight), each on its own copy of the stripe,
    all checked after one synchronize."""
    torch = torch_dev
    k, p, S = 128, 32, 4096
    g = torch.Generator(device="cuda")
    g.manual_seed(21)
    full = torch.randint(0, 256, (k + p, S), dtype=torch.uint8, device="cuda", generator=g)
    c = rs.New16(k, p)
    c.encode_dev(full)
    torch.cuda.synchronize()
    rng = np.random.default_rng(21)
    pats = [rng.choice(k + p, int(rng.integers(1, p + 1)), replace=False) for _ in range(20)]
    st = torch.cuda.Stream()
    copies = []
    with torch.cuda.stream(st):
        for i in range(40):
            er = pats[i % 20]
            present = np.ones(k + p, bool)
            present[er] = False
            t = full.clone()
            t[torch.from_numpy(er).cuda()] = 0
            c.reconstruct_dev(t, present, stream=st)
            copies.append(t)
    st.synchronize()
    for i, t in enumerate(copies):
        assert torch.equal(t, full), f"call {i}"


def test_default_stream_is_stream_ordered(torch_dev):
    """torch's default stream (handle 0) goes to the C-ABI as RS_NULL_STREAM:
    the calls are asynchronous on it and ordered with torch's own work there
    (no synchronize between the encode / reconstruct and the reads)."""
    torch = torch_dev
    k, p, S = 128, 32, 1 << 16
    c = rs.New16(k, p)
    g = torch.Generator(device="cuda")
    g.manual_seed(5)
    slab = torch.randint(0, 256, (k + p, S), dtype=torch.uint8, device="cuda", generator=g)
    ref = slab.clone()
    c.encode_dev(ref)
    torch.cuda.synchronize()
    for _ in range(3):
        t = slab.clone()
        c.encode_dev(t)  # default stream
        par = t[k:].clone()  # torch kernel on the same stream, after the encode
        er = torch.tensor([0, 5, k + 1])
        t[er] = 0
        present = np.ones(k + p, bool)
        present[er.numpy()] = False
        c.reconstruct_dev(t, present)
        assert torch.equal(par, ref[k:]) and torch.equal(t, ref)


def test_reconstruct_dev_async_row_lists(torch_dev):
    """The pointer-ring path of rs_reconstruct_dev: shards as separately
    allocated rows (not equally strided), 24 calls over 12 patterns on a caller
    stream, checked after one synchronize."""
    torch = torch_dev
    k, p, S = 128, 32, 2048
    g = torch.Generator(device="cuda")
    g.manual_seed(22)
    full = torch.randint(0, 256, (k + p, S), dtype=torch.uint8, device="cuda", generator=g)
    c = rs.New16(k, p)
    c.encode_dev(full)
    torch.cuda.synchronize()
    rng = np.random.default_rng(22)
    pats = [rng.choice(k + p, int(rng.integers(1, p + 1)), replace=False) for _ in range(12)]
    st = torch.cuda.Stream()
    calls = []
    with torch.cuda.stream(st):
        for i in range(24):
            er = pats[i % 12]
            present = np.ones(k + p, bool)
            present[er] = False
            rows = [full[r].clone() if present[r] else torch.zeros(S, dtype=torch.uint8, device="cuda")
                    for r in range(k + p)]
            c.reconstruct_dev(rows, present, stream=st)
            calls.append(rows)
    st.synchronize()
    for i, rows in enumerate(calls):
        assert torch.equal(torch.stack(rows), full), f"call {i}"


@pytest.mark.parametrize("k,p,S", [(20, 8, 64 * 40), (128, 32, 64 * 96)])
def test_verify_and_reconstruct_async_stream_of_blocks(k, p, S):
    """rs_verify_async / rs_reconstruct_async over a stream of 6 blocks (the
    rsStream16.verify / reconstruct loops, streaming16.go:200-468): every
    block's verify and reconstruct are queued before any ticket is waited on,
    interleaved with encodes.  Missing shards are EmptyShard views of pinned
    rows (Go's cap() reuse), so the calls return early.  One corrupted block
    must verify False; every rebuilt block equals the oracle's."""
    nblk = 6
    c = rs.New16(k, p)
    c.set_host_segment(64 * 24)
    o = orc.Oracle(16, k, p)
    rng = np.random.default_rng(k + p)
    blocks = []
    for b in range(nblk):
        sh = c.alloc_aligned(S, pinned=True)
        for i in range(k):
            sh[i][:] = rng.integers(0, 256, S, dtype=np.uint8)
        par = orc.encode(16, k, p, np.stack(sh[:k]))
        for i in range(p):
            sh[k + i][:] = par[i]
        blocks.append(sh)
    bad = 3
    vtk = []
    for b, sh in enumerate(blocks):
        rows = list(sh)
        if b == bad:
            rows[k + 1] = rows[k + 1].copy()
            rows[k + 1][S // 2] ^= 0x5A
        vtk.append((c.verify_async(rows), rows))
    rtk, work, refs = [], [], []
    for b, sh in enumerate(blocks):
        pinned = c.alloc_aligned(S, pinned=True)
        er = sorted(rng.choice(k + p, int(rng.integers(1, p + 1)), replace=False).tolist())
        rows = [rs.EmptyShard(pinned[i]) if i in er else sh[i].copy() for i in range(k + p)]
        refs.append([None if i in er else sh[i].copy() for i in range(k + p)])
        rtk.append(c.reconstruct_async(rows, recover_all=(b % 2 == 0)))
        work.append((rows, er, b % 2 == 0))
    for b, (t, _) in enumerate(vtk):
        assert t.result() == (b != bad), f"block {b}"
    for t in rtk[::-1]:
        t.wait()
    assert all(t.done() for t in rtk)
    for b, (rows, er, all_) in enumerate(work):
        e, ref = o.reconstruct(refs[b], all_)
        assert e == 0
        for i in range(k + p):
            if i in er and not all_ and i >= k:
                continue
            assert np.array_equal(np.asarray(rows[i]), ref[i]), f"block {b} shard {i}"
            assert np.array_equal(np.asarray(rows[i]), blocks[b][i]), f"block {b} shard {i}"
    # a verify ticket older than the 64-slot result ring is refused
    old = vtk[0][0].ticket
    for _ in range(70):
        c.verify_async(list(blocks[0])).wait()
    with pytest.raises(rs.codec.RSError):
        rs.codec.VerifyTicket(c, old, None).result()


@pytest.mark.parametrize("k,p,S", [(1024, 256, 1024), (300, 200, 512), (100, 40, 256), (1000, 129, 128),
                                   (4000, 1000, 256), (3500, 600, 128), (1500, 1024, 64 * 3),
                                   (2000, 3000, 128), (13000, 2100, 64)])
def test_lds_encode_subfield_chunk_passes(torch_dev, paths, k, p, S):
    """k_enc_lds with the chunk IFFTs in subfield coordinates from their first
    all-subfield pass on (EncodeArgs::tw_ifft_sub, default) and the full-field
    chunk IFFTs (rs_debug_set_path("sub", 0)) both give the oracle's parity, and verify it.
    m = 1024, 4096 (round 6): chunk passes full-field up to pass 1, 2 or 3 (m = 1024
    chunk 3: layers 0-4) and the FFT's last passes full-field; at m = 4096 a
    fourth chunk (layers 0-6 full-field) keeps every chunk full-field and only
    the FFT in subfield coordinates."""
    torch = torch_dev
    rng = np.random.default_rng(k + p + S)
    data = rand_data(rng, k, S)
    ref = orc.encode(16, k, p, data)
    for nosub in ("0", "1"):
        paths("sub", int(nosub != "1"))
        c = rs.New16(k, p)
        assert c.encode_path.startswith("lds-m")
        slab = torch.zeros((2, k + p, S), dtype=torch.uint8, device="cuda")
        slab[:, :k] = torch.from_numpy(data).cuda()
        c.encode_dev_batch(slab)
        torch.cuda.synchronize()
        for z in range(2):
            assert np.array_equal(slab[z, k:].cpu().numpy(), ref), (nosub, z)
        assert c.verify_dev_batch(slab)
        slab[1, k + p - 1, 3] ^= 0x40
        assert not c.verify_dev_batch(slab)
