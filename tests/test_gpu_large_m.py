"""The LDS-resident encode for m = 512 .. 4096 (GF(2^16), kernels.hip
k_enc_lds with 64-byte tiles, 32-byte half tiles at m = 2048, 16-byte quarter
tiles at m = 4096, and 1024 threads): bit-exact against the oracle
on ragged geometries, batched / table / host-pipeline row layouts, verify, and
the reference's own large-shard-count tests replayed end to end
(reedsolomon_test.go:61-84 "500 / 1000 / 5000 Shards": testEncodeDecode
:133-190 and testLargeShardCount :414-516)."""
import io

import numpy as np
import pytest

import reedsolomon16_amd as rs
from oracle import orc

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch():
    import torch as t

    return t


def rand_data(rng, k, S):
    return rng.integers(0, 256, (k, S), dtype=np.uint8)


# (k, p, S): m = 512 and 1024, one chunk and several, ragged last chunk,
# p < m and p a power of two, one and several 64-byte blocks
GEOMS = [(300, 300, 64), (700, 300, 128), (512, 512, 192), (1100, 257, 64), (4000, 1000, 64),
         (1000, 600, 128), (2047, 1024, 64), (600, 700, 64 * 5), (3000, 1025, 64), (2048, 2048, 128),
         (5000, 1500, 64 * 3), (3000, 2049, 64), (5000, 4096, 128)]


@pytest.mark.parametrize("k,p,S", GEOMS)
def test_encode_matches_oracle(k, p, S):
    rng = np.random.default_rng(k * 3 + p + S)
    data = rand_data(rng, k, S)
    c = rs.New16(k, p)
    assert c.encode_path == "lds-m%d" % (1 << (p - 1).bit_length())
    shards = [data[i].copy() for i in range(k)] + [np.zeros(S, np.uint8) for _ in range(p)]
    c.encode(shards)
    ref = orc.encode(16, k, p, data)
    assert np.array_equal(np.stack(shards[k:]), ref)
    assert c.verify(shards)
    shards[k + p // 2][S - 1] ^= 0x10
    assert not c.verify(shards)
    shards[k + p // 2][S - 1] ^= 0x10
    shards[k - 1][0] ^= 1
    assert not c.verify(shards)


@pytest.mark.parametrize("k,p,S,B", [(700, 300, 4096 + 64, 3), (3000, 1000, 256, 2), (3000, 1500, 64 * 3, 2),
                                     (2000, 4000, 64 * 3, 2)])
def test_device_batch_and_table(torch, k, p, S, B):
    """Strided stripes in one launch (grid.y), and the same stripe through a row table."""
    rng = np.random.default_rng(k + p + B)
    datas = [rand_data(rng, k, S) for _ in range(B)]
    slab = torch.zeros((B, k + p, S), dtype=torch.uint8, device="cuda")
    for j in range(B):
        slab[j, :k] = torch.from_numpy(datas[j]).cuda()
    c = rs.New16(k, p)
    c.encode_dev_batch(slab)
    torch.cuda.synchronize()
    refs = [orc.encode(16, k, p, d) for d in datas]
    for j in range(B):
        assert np.array_equal(slab[j, k:].cpu().numpy(), refs[j]), f"stripe {j}"
    assert c.verify_dev_batch(slab)
    slab[B - 1, k, 5] ^= 0x80
    assert not c.verify_dev_batch(slab)
    # row table: rows in scattered allocations
    rows = [torch.from_numpy(datas[0][i]).cuda() for i in range(k)] + [torch.zeros(S, dtype=torch.uint8, device="cuda")
                                                                      for _ in range(p)]
    c.encode_dev(rows)
    torch.cuda.synchronize()
    assert np.array_equal(torch.stack(rows[k:]).cpu().numpy(), refs[0])


def test_host_pipeline_segments_large_m():
    """Host shards wider than one staging segment: the segment loop around the
    m = 1024 LDS encode (no multi-pass scratch)."""
    k, p, S = 2000, 600, 64 * 40
    rng = np.random.default_rng(9)
    data = rand_data(rng, k, S)
    c = rs.New16(k, p)
    c.set_host_segment(64 * 16)
    shards = [data[i].copy() for i in range(k)] + [np.zeros(S, np.uint8) for _ in range(p)]
    c.encode(shards)
    assert np.array_equal(np.stack(shards[k:]), orc.encode(16, k, p, data))
    assert c.verify(shards)


def _encode_decode(k, p, size):
    """testEncodeDecode (reedsolomon_test.go:133-190): Split, Encode, Verify, Join."""
    rng = np.random.default_rng(k + p)
    data = rng.integers(0, 256, size, dtype=np.uint8)
    r = rs.New16(k, p)
    shards = r.split(data)
    assert len(shards) == k + p
    r.encode(shards)
    assert r.verify(shards)
    buf = io.BytesIO()
    r.join(buf, shards, size)
    assert buf.getvalue() == data.tobytes()
    return r, shards


@pytest.mark.parametrize("k,p", [(350, 150), (700, 300)])
def test_reference_shard_counts(k, p):
    """reedsolomon_test.go:66-78: "500 Shards" (350 + 150) and "1000 Shards"
    (700 + 300, m = 512) at smallTestSize (1 KB, :16)."""
    r, shards = _encode_decode(k, p, 1 << 10)
    S = len(shards[0])
    data = np.stack([np.asarray(s) for s in shards[:k]])
    assert np.array_equal(np.stack([np.asarray(s) for s in shards[k:]]), orc.encode(16, k, p, np.ascontiguousarray(data)))


def test_reference_large_shard_count_5000():
    """testLargeShardCount(4000, 1000) (reedsolomon_test.go:80-83, :414-516):
    k * 64 bytes split into 4000 + 1000 shards (m = 1024, n = 8192), encode,
    verify, five data shards erased, ReconstructData, Join."""
    k, p = 4000, 1000
    size = k * 64
    rng = np.random.default_rng(5000)
    data = rng.integers(0, 256, size, dtype=np.uint8)
    r = rs.New16(k, p)
    assert r.encode_path == "lds-m1024"
    shards = r.split(data)
    assert len(shards) == k + p
    r.encode(shards)
    dmat = np.ascontiguousarray(np.stack([np.asarray(s) for s in shards[:k]]))
    assert np.array_equal(np.stack([np.asarray(s) for s in shards[k:]]), orc.encode(16, k, p, dmat))
    assert r.verify(shards)
    deleted = [i * (k // 5) for i in range(5)]
    orig = {i: np.asarray(shards[i]).copy() for i in deleted}
    sh = [None if i in orig else np.asarray(s).copy() for i, s in enumerate(shards)]
    r.reconstruct_data(sh)
    for i in deleted:
        assert sh[i] is not None and np.array_equal(sh[i], orig[i]), i
    buf = io.BytesIO()
    r.join(buf, sh, size)
    assert buf.getvalue() == data.tobytes()


def test_m8192_stays_multipass():
    """m = 8192 (p > 4096) keeps the multi-pass encode; still oracle-exact."""
    k, p, S = 1500, 4100, 64
    rng = np.random.default_rng(2048)
    data = rand_data(rng, k, S)
    c = rs.New16(k, p)
    assert c.encode_path == "multipass"
    shards = [data[i].copy() for i in range(k)] + [np.zeros(S, np.uint8) for _ in range(p)]
    c.encode(shards)
    assert np.array_equal(np.stack(shards[k:]), orc.encode(16, k, p, data))


@pytest.mark.parametrize("k,p,S", [(700, 300, 4096 + 64), (2500, 1000, 512), (3000, 1500, 64 * 7), (3000, 3000, 64 * 5)])
def test_lds_equals_multipass(torch, paths, k, p, S):
    """The one-launch LDS encode and the multi-pass kernels (rs_debug_set_path
    "lds_big" 0) write identical parity, two stripes per launch."""
    g = torch.Generator(device="cuda")
    g.manual_seed(k + p)
    base = torch.randint(0, 256, (2, k + p, S), dtype=torch.uint8, device="cuda", generator=g)
    out = []
    for big in (1, 0):
        paths("lds_big", big)
        c = rs.New16(k, p)
        assert c.encode_path == ("lds-m%d" % (1 << (p - 1).bit_length()) if big else "multipass")
        slab = base.clone()
        c.encode_dev_batch(slab)
        torch.cuda.synchronize()
        out.append(slab)
    assert torch.equal(out[0], out[1])
