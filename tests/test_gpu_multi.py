"""GPU tests of the multi-device codec (rs_new_multi): the north star's
byte-range split over GPUs, driven from ONE codec handle the way a cgo caller
holds one Encoder (reedsolomon.go:90-93).  The one-GPU box stands in for a
node: devices = [0, 0, 0, 0] makes four parts on device 0, each with its own
streams, staging slabs, tickets and host worker thread, exactly the code a
node with four GPUs runs (only the device ordinals differ).

Every result is checked against the oracle (or the oracle-pinned SIMD port at
C5), at the C3, C4 and C5 shapes of BASELINE.json: encode, verify with a
tampered byte in each part's range, 32-erasure reconstruct, the async tickets,
ragged splits, and the GF(2^8) inversion-cache call sequence (whose keying
depends on the FULL shard size, leopard8.go:475)."""
import os
import threading

import numpy as np
import pytest

import reedsolomon16_amd as rs
from oracle import orc

pytestmark = pytest.mark.gpu

DEV4 = [0, 0, 0, 0]


def host_rows(k, p, S, data, pinned):
    """k+p host rows: one pinned AllocAligned slab, or separate pageable arrays."""
    if pinned:
        c = rs.New16(1, 1)
        rows = c.alloc_aligned(S, k + p, pinned=True)
        c.close()
    else:
        rows = [np.zeros(S, np.uint8) for _ in range(k + p)]
    for i in range(k):
        rows[i][:] = data[i]
    return rows


@pytest.fixture(scope="module")
def c3():
    k, p, S = 128, 32, 1 << 20
    rng = np.random.default_rng(0x5EED)
    data = rng.integers(0, 256, (k, S), dtype=np.uint8)
    return k, p, S, data, orc.encode(16, k, p, data)


@pytest.mark.parametrize("pinned", [True, False])
def test_multi_c3_encode_verify_matches_oracle(c3, pinned):
    k, p, S, data, ref = c3
    c = rs.New16(k, p, devices=DEV4)
    assert c.device_count == 4
    rows = host_rows(k, p, S, data, pinned)
    c.encode(rows)
    assert np.array_equal(np.stack(rows[k:]), ref)
    assert c.verify(rows)
    # one flipped byte in each part's range (and the last byte) fails Verify
    for g in range(4):
        lo, hi = c.byte_range(S, g)
        for r, off in ((g * 37 % k, lo), (k + g, hi - 1)):
            rows[r][off] ^= 0x5A
            assert not c.verify(rows), (g, r, off)
            rows[r][off] ^= 0x5A
    assert c.verify(rows)
    c.close()


@pytest.mark.parametrize("pattern", ["random32", "first32", "one"])
def test_multi_c4_reconstruct(c3, pattern):
    """C4 through the multi-device codec: 32 erasures, pinned rows (zero-copy
    row moves per part) and Go's EmptyShard capacity semantics."""
    k, p, S, data, ref = c3
    full = [data[i] for i in range(k)] + [ref[i] for i in range(p)]
    c = rs.New16(k, p, devices=DEV4)
    rng = np.random.default_rng(7)
    er = {"random32": rng.choice(k + p, 32, replace=False).tolist(), "first32": list(range(32)), "one": [77]}[pattern]
    for recover_all in (True, False):
        rows = host_rows(k, p, S, data, True)
        for i in range(p):
            rows[k + i][:] = ref[i]
        sh = [rs.EmptyShard(rows[i]) if i in er else rows[i] for i in range(k + p)]
        for i in er:
            rows[i][:] = 0
        (c.reconstruct if recover_all else c.reconstruct_data)(sh)
        for i in range(k + p):
            if i < k or recover_all:
                assert np.array_equal(sh[i], full[i]), (pattern, recover_all, i)
    c.close()


def test_multi_c5_encode_verify_reconstruct():
    """C5 (1024 + 256 x 256 KiB) over four parts of 64 KiB of every row:
    encode bit-exact against the SIMD port over the whole stripe, verify,
    32-erasure reconstruct (n = 2048 decoder on every part)."""
    if not orc.simd_available():
        pytest.skip("no AVX2 on this host")
    k, p, S = 1024, 256, 256 << 10
    rng = np.random.default_rng(0xC5)
    data = rng.integers(0, 256, (k, S), dtype=np.uint8)
    ref = orc.encode_simd(k, p, data, min(16, os.cpu_count() or 1))
    c = rs.New16(k, p, devices=DEV4)
    rows = host_rows(k, p, S, data, True)
    c.encode(rows)
    assert np.array_equal(np.stack(rows[k:]), ref)
    assert c.verify(rows)
    lo, _ = c.byte_range(S, 3)
    rows[1000][lo + 5] ^= 1
    assert not c.verify(rows)
    rows[1000][lo + 5] ^= 1
    er = rng.choice(k + p, 32, replace=False).tolist()
    keep = {i: rows[i].copy() for i in er}
    sh = [rs.EmptyShard(rows[i]) if i in er else rows[i] for i in range(k + p)]
    for i in er:
        rows[i][:] = 0
    c.reconstruct(sh)
    for i in er:
        assert np.array_equal(sh[i], keep[i]), i
    c.close()


def test_multi_async_tickets_match_single_codec():
    """encode_async / verify_async / reconstruct_async on the multi-device
    codec: one parent ticket per call, waited and queried like a one-device
    codec's, same bytes and verdicts as the one-device codec."""
    k, p, S, nb = 128, 32, 64 * 1000, 4
    rng = np.random.default_rng(11)
    c1, c4 = rs.New16(k, p), rs.New16(k, p, devices=DEV4)
    blocks = [rng.integers(0, 256, (k, S), dtype=np.uint8) for _ in range(nb)]
    rows4 = [host_rows(k, p, S, d, True) for d in blocks]
    tks = [c4.encode_async(r) for r in rows4]
    for t in tks:
        t.wait()
        assert t.done()
    for d, r in zip(blocks, rows4):
        assert np.array_equal(np.stack(r[k:]), orc.encode(16, k, p, d))
    rows4[2][5][S - 7] ^= 3
    vt = [c4.verify_async(r) for r in rows4]
    assert [t.result() for t in vt] == [True, True, False, True]
    assert [c1.verify(r) for r in rows4] == [True, True, False, True]
    rows4[2][5][S - 7] ^= 3
    er = set(rng.choice(k + p, 20, replace=False).tolist())
    want = [[r[i].copy() for i in range(k + p)] for r in rows4]
    shs = [[None if i in er else r[i] for i in range(k + p)] for r in rows4]
    rt = [c4.reconstruct_async(sh) for sh in shs]
    for t in rt:
        t.wait()
    for sh, w in zip(shs, want):
        for i in er:
            assert np.array_equal(sh[i], w[i])
    c1.close()
    c4.close()


@pytest.mark.parametrize("bits,k,p,S,devs", [(16, 128, 32, 64 * 7, [0, 0, 0]), (16, 10, 4, 64, DEV4),
                                             (8, 10, 4, 64 * 5, [0] * 8), (16, 300, 100, 64 * 9, [0, 0]),
                                             (8, 100, 28, 64 * 33, DEV4),
                                             (16, 2000, 100, 64 * 3, [0, 0])])  # n = 4096: one LDS reconstruct (half tiles) on each part
def test_multi_ragged_splits(bits, k, p, S, devs):
    """Shard sizes the parts split unevenly, or that leave parts empty."""
    rng = np.random.default_rng(k + S)
    data = rng.integers(0, 256, (k, S), dtype=np.uint8)
    ref = orc.encode(bits, k, p, data)
    c = rs.ReedSolomon(k, p, bits, devices=devs)
    rows = [data[i].copy() for i in range(k)] + [np.zeros(S, np.uint8) for _ in range(p)]
    c.encode(rows)
    assert np.array_equal(np.stack(rows[k:]), ref)
    assert c.verify(rows)
    rows[k][S - 1] ^= 1
    assert not c.verify(rows)
    rows[k][S - 1] ^= 1
    er = set(rng.choice(k + p, p, replace=False).tolist())
    sh = [None if i in er else rows[i].copy() for i in range(k + p)]
    c.reconstruct(sh)
    o = orc.Oracle(bits, k, p)
    e, want = o.reconstruct([None if i in er else rows[i].copy() for i in range(k + p)], True)
    assert e == 0
    for i in range(k + p):
        assert np.array_equal(sh[i], want[i]), i
    c.close()


@pytest.mark.parametrize("S", [8192, 64 * 40])
def test_multi_gf8_reference_cache_sequence(S):
    """The reference-keyed GF(2^8) inversion cache (leopard8.go:508-555) on a
    multi-device codec: its store key depends on useBits, which depends on the
    FULL shard size (S * total >= 64 KiB, leopard8.go:475); at S = 8192 every
    part's own slice would key differently.  The parent keys once, so a call
    sequence returns the stateful oracle's bytes call for call, stale hits
    included, like a one-device codec."""
    k, p = 10, 4
    rng = np.random.default_rng(S)
    data = rng.integers(0, 256, (k, S), dtype=np.uint8)
    par = orc.encode(8, k, p, data)
    full = [data[i] for i in range(k)] + [par[i] for i in range(p)]
    c1, c4 = rs.New8(k, p), rs.New8(k, p, devices=DEV4)
    o = orc.Oracle(8, k, p)
    stale = 0
    for trial in range(40):
        ne = int(rng.integers(1, p + 1))
        er = set(rng.choice(k + p, ne, replace=False).tolist())
        recover_all = bool(rng.integers(0, 2))
        outs = []
        for cc in (c1, c4):
            sh = [None if i in er else full[i].copy() for i in range(k + p)]
            (cc.reconstruct if recover_all else cc.reconstruct_data)(sh)
            outs.append(sh)
        e, want = o.reconstruct([None if i in er else full[i].copy() for i in range(k + p)], recover_all)
        assert e == 0
        for i in range(k + p):
            if i < k or recover_all:
                assert np.array_equal(outs[0][i], want[i]) and np.array_equal(outs[1][i], want[i]), (trial, i)
                stale += int(not np.array_equal(want[i], full[i]))
    c1.close()
    c4.close()


def test_multi_concurrent_callers():
    """Two host threads on one multi-device codec (Go allows concurrent
    Encode calls on one Encoder): calls serialize on the codec, results exact."""
    k, p, S = 64, 16, 64 * 512
    c = rs.New16(k, p, devices=DEV4)
    rng = np.random.default_rng(3)
    jobs = [rng.integers(0, 256, (k, S), dtype=np.uint8) for _ in range(6)]
    outs = [None] * len(jobs)
    errs = []

    def run(idx):
        try:
            for j in idx:
                rows = [jobs[j][i].copy() for i in range(k)] + [np.zeros(S, np.uint8) for _ in range(p)]
                c.encode(rows)
                assert c.verify(rows)
                outs[j] = np.stack(rows[k:])
        except Exception as e:  # surfaced below
            errs.append(e)

    th = [threading.Thread(target=run, args=([0, 2, 4],)), threading.Thread(target=run, args=([1, 3, 5],))]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errs, errs
    for j, d in enumerate(jobs):
        assert np.array_equal(outs[j], orc.encode(16, k, p, d)), j
    c.close()


def test_multi_parts_device_resident():
    """rs_device_part: each part's own codec encodes its byte range of rows in
    HBM (the device-resident form of the split), the same bytes as one codec."""
    import torch

    k, p, S = 128, 32, 1 << 16
    g = torch.Generator(device="cuda")
    g.manual_seed(5)
    slab = torch.randint(0, 256, (3, k + p, S), dtype=torch.uint8, device="cuda", generator=g)
    ref = slab.clone()
    rs.New16(k, p).encode_dev_batch(ref)
    c = rs.New16(k, p, devices=DEV4)
    with pytest.raises(rs.RSError):
        c.encode_dev_batch(slab)
    for i in range(4):
        lo, hi = c.byte_range(S, i)
        c.part(i).encode_dev_batch(slab[:, :, lo:hi])
    torch.cuda.synchronize()
    assert torch.equal(slab, ref)
    c.close()


@pytest.mark.parametrize("bits", [16, 8])
def test_multi_stream_methods_match_single_codec(bits):
    """The interface's Stream* methods (rsStream16 / rsStreamFF8 loops over the
    async tickets, stream.py) on a multi-device codec: every 4 MiB block is
    split over the parts, and the writers get the same bytes as on one device."""
    import io

    k, p, n = 10, 4, (4 << 20) + 4160  # a full block, then a short one (64-byte multiple: no GF(2^16) verify panic)
    rng = np.random.default_rng(bits)
    data = rng.integers(0, 256, (k, n), dtype=np.uint8)
    outs = []
    for devs in (None, DEV4):
        c = rs.ReedSolomon(k, p, bits, devices=devs)
        par = [io.BytesIO() for _ in range(p)]
        c.stream_encode([io.BytesIO(data[i].tobytes()) for i in range(k)], par)
        pv = [x.getvalue() for x in par]
        ok = c.stream_verify([io.BytesIO(data[i].tobytes()) for i in range(k)] + [io.BytesIO(v) for v in pv])
        ins = [None if i in (1, 4) else io.BytesIO(data[i].tobytes()) for i in range(k)] + [io.BytesIO(v) for v in pv]
        rec = [io.BytesIO() if i in (1, 4) else None for i in range(k + p)]
        c.stream_reconstruct(ins, rec)
        outs.append((pv, ok, [r.getvalue() for r in rec if r is not None]))
        c.close()
    assert outs[0] == outs[1]
    assert outs[0][2] == [data[1].tobytes(), data[4].tobytes()]
