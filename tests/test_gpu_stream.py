"""The reference's stream loops (rsStream16, streaming16.go:200-632,
1229-1318, and rsStreamFF8, streaming8.go:109-766) replayed through the HIP
engine's asynchronous tickets (reedsolomon16_amd/stream.py: two pinned block
buffers, block j+1 queued while block j is in flight), each block's result
compared with the single-buffer restatement of the Go loop answered by the
oracle (tests/go_stream.py): 4 MiB blocks, a short odd-length last block
padded (to even and then) to 64, ragged shard lengths, verify with tampering
(and the GF(2^16) loop's panic after a zero-padded block verifies),
reconstruct and reconstructData."""
import io

import numpy as np
import pytest

from reedsolomon16_amd.codec import ErrPanic
from reedsolomon16_amd.stream import StreamEncoder8, StreamEncoder16
from tests.go_stream import GoPanic, GoStream8, GoStream16

pytestmark = pytest.mark.gpu

MiB = 1 << 20


def _streams(datas):
    return [None if d is None else io.BytesIO(d) for d in datas]


def _data(rng, lens):
    return [None if n is None else rng.integers(0, 256, n, dtype=np.uint8).tobytes() for n in lens]


def _outcome(fn, *args):
    try:
        return fn(*args)
    except (GoPanic, ErrPanic):
        return "panic"


# (k, p, block size, per-shard stream lengths): the default 4 MiB blocks with
# a bit-sliced m = 16 geometry, and the C3 geometry (128 + 32) on 256 KiB blocks
GEOMS = {
    "20p10_4MiB_odd_tail": (20, 10, 4 * MiB, [2 * 4 * MiB + 12345] * 20),
    "20p10_4MiB_ragged": (20, 10, 4 * MiB, [4 * MiB + 777] + [4 * MiB + 1000] * 9 + [5 * MiB] * 9 + [None]),
    "128p32_256KiB_odd_tail": (128, 32, 256 << 10, [2 * (256 << 10) + 4097] * 128),
}


@pytest.fixture(scope="module")
def encoded():
    out = {}
    for name, (k, p, blk, lens) in GEOMS.items():
        rng = np.random.default_rng(abs(hash(name)) % 2**32)
        datas = _data(rng, lens)
        go = GoStream16(k, p, blk)
        gout = [io.BytesIO() for _ in range(p)]
        go.encode(_streams(datas), gout)
        out[name] = (datas, [o.getvalue() for o in gout])
    return out


@pytest.fixture(scope="module")
def engines():
    return {name: StreamEncoder16(k, p, block_size=blk) for name, (k, p, blk, _) in GEOMS.items()}


@pytest.mark.parametrize("name", sorted(GEOMS))
def test_stream_encode_through_engine(name, encoded, engines):
    k, p, blk, _ = GEOMS[name]
    datas, ref = encoded[name]
    st = engines[name]
    assert st.rs.encode_path.startswith("bs16")
    out = [io.BytesIO() for _ in range(p)]
    st.encode(_streams(datas), out)
    for j in range(p):
        assert out[j].getvalue() == ref[j], f"parity {j} differs"


@pytest.mark.parametrize("tamper", [None, "data", "parity_last_block"])
def test_stream_verify_through_engine(tamper, encoded, engines):
    name = "20p10_4MiB_odd_tail"
    k, p, blk, _ = GEOMS[name]
    datas, par = encoded[name]
    shards = list(datas) + list(par)
    if tamper == "data":
        b = bytearray(shards[3])
        b[5 * MiB + 17] ^= 0x40
        shards[3] = bytes(b)
    elif tamper == "parity_last_block":
        b = bytearray(shards[k + 2])
        b[-3] ^= 1
        shards[k + 2] = bytes(b)
    go = GoStream16(k, p, blk)
    want = _outcome(go.verify, _streams(shards))
    # 20 + 10 has only GF(2^8) twiddles: the zero-padded odd tail verifies
    # and the reference then panics (streaming16.go:218, stream.py docstring)
    assert want == (False if tamper == "data" else "panic")
    assert _outcome(engines[name].verify, _streams(shards)) == want


def test_stream_verify_aligned_stream_true(engines):
    """A stream of whole 64-byte-aligned blocks verifies (no stale padding)."""
    name = "20p10_4MiB_odd_tail"
    k, p, blk, _ = GEOMS[name]
    rng = np.random.default_rng(5)
    datas = _data(rng, [blk + 64 * 1000] * k)
    go = GoStream16(k, p, blk)
    outs = [io.BytesIO() for _ in range(p)]
    go.encode(_streams(datas), outs)
    shards = list(datas) + [o.getvalue() for o in outs]
    assert engines[name].verify(_streams(shards)) is True
    assert go.verify(_streams(shards)) is True


@pytest.mark.parametrize("name,erase", [
    ("20p10_4MiB_odd_tail", (0, 7, 21, 29)),
    ("128p32_256KiB_odd_tail", tuple(range(0, 160, 5))),
])
def test_stream_reconstruct_through_engine(name, erase, encoded, engines):
    k, p, blk, _ = GEOMS[name]
    datas, par = encoded[name]
    shards = list(datas) + list(par)
    mk_in = lambda: [None if i in erase else io.BytesIO(shards[i]) for i in range(k + p)]
    go_out = [io.BytesIO() if i in erase else None for i in range(k + p)]
    GoStream16(k, p, blk).reconstruct(mk_in(), go_out)
    m_out = [io.BytesIO() if i in erase else None for i in range(k + p)]
    engines[name].reconstruct(mk_in(), m_out)
    for i in erase:
        assert m_out[i].getvalue() == go_out[i].getvalue(), f"shard {i}"
        if i < k:
            assert m_out[i].getvalue() == shards[i]


def test_stream_reconstruct_data_through_engine(encoded, engines):
    name = "20p10_4MiB_odd_tail"
    k, p, blk, _ = GEOMS[name]
    datas, par = encoded[name]
    shards = list(datas) + list(par)
    erase = (2, 11, 19)
    mk_in = lambda: [None if i in erase else io.BytesIO(shards[i]) for i in range(k + p)]
    go_out = [io.BytesIO() if i in erase else None for i in range(k + p)]
    GoStream16(k, p, blk).reconstruct_data(mk_in(), go_out)
    m_out = [io.BytesIO() if i in erase else None for i in range(k + p)]
    engines[name].reconstruct_data(mk_in(), m_out)
    for i in erase:
        assert m_out[i].getvalue() == go_out[i].getvalue() == shards[i]


# --------------------------------------------------------------------------- rsStreamFF8
GEOMS8 = {
    "10p4_4MiB_odd_tail": (10, 4, 4 * MiB, [2 * 4 * MiB + 12345] * 10),
    "100p28_4MiB_ragged_odd": (100, 28, 4 * MiB, [4 * MiB + 999] + [4 * MiB + 1001] * 98 + [None]),
}


@pytest.fixture(scope="module")
def encoded8():
    out = {}
    for name, (k, p, blk, lens) in GEOMS8.items():
        rng = np.random.default_rng(abs(hash(name)) % 2**32)
        datas = _data(rng, lens)
        go = GoStream8(k, p, blk)
        gout = [io.BytesIO() for _ in range(p)]
        go.encode(_streams(datas), gout)
        out[name] = (datas, [o.getvalue() for o in gout])
    return out


@pytest.fixture(scope="module")
def engines8():
    return {name: StreamEncoder8(k, p, block_size=blk) for name, (k, p, blk, _) in GEOMS8.items()}


@pytest.mark.parametrize("name", sorted(GEOMS8))
def test_stream8_encode_through_engine(name, encoded8, engines8):
    k, p, blk, _ = GEOMS8[name]
    datas, ref = encoded8[name]
    st = engines8[name]
    assert st.rs.field_bits == 8
    out = [io.BytesIO() for _ in range(p)]
    st.encode(_streams(datas), out)
    for j in range(p):
        assert out[j].getvalue() == ref[j], f"parity {j} differs"


@pytest.mark.parametrize("name", sorted(GEOMS8))
@pytest.mark.parametrize("tamper", [None, "data", "parity_last_block"])
def test_stream8_verify_through_engine(name, tamper, encoded8, engines8):
    k, p, blk, _ = GEOMS8[name]
    datas, par = encoded8[name]
    shards = list(datas) + list(par)
    if tamper == "data":
        b = bytearray(shards[3])
        b[4 * MiB + 17] ^= 0x40
        shards[3] = bytes(b)
    elif tamper == "parity_last_block":
        b = bytearray(shards[k + 2])
        b[-70] ^= 1
        shards[k + 2] = bytes(b)
    go = GoStream8(k, p, blk)
    want = go.verify(_streams(shards))
    assert want == (tamper is None)
    assert engines8[name].verify(_streams(shards)) == want


@pytest.mark.parametrize("name,erase", [
    ("10p4_4MiB_odd_tail", (0, 7, 9)),
    ("100p28_4MiB_ragged_odd", tuple(range(1, 100, 4))),
])
def test_stream8_reconstruct_data_through_engine(name, erase, encoded8, engines8):
    """streaming8.go:609-766, what StreamReconstruct runs for data outputs only."""
    k, p, blk, _ = GEOMS8[name]
    datas, par = encoded8[name]
    shards = list(datas) + list(par)
    mk_in = lambda: [None if i in erase else io.BytesIO(shards[i]) for i in range(k + p)]
    go_out = [io.BytesIO() if i in erase else None for i in range(k + p)]
    GoStream8(k, p, blk).reconstruct_data(mk_in(), go_out)
    m_out = [io.BytesIO() if i in erase else None for i in range(k + p)]
    engines8[name].reconstruct_data(mk_in(), m_out)
    for i in erase:
        assert m_out[i].getvalue() == go_out[i].getvalue(), f"shard {i}"
        if shards[i] is not None:
            assert m_out[i].getvalue()[:len(shards[i])] == shards[i][:len(m_out[i].getvalue())]


def test_stream8_reconstruct_through_engine(encoded8, engines8):
    """streaming8.go:447-606: the codec sees every shard present and the
    requested outputs receive zeros, as in the reference."""
    name = "10p4_4MiB_odd_tail"
    k, p, blk, _ = GEOMS8[name]
    datas, par = encoded8[name]
    shards = list(datas) + list(par)
    erase = (2, 11)
    mk_in = lambda: [None if i in erase else io.BytesIO(shards[i]) for i in range(k + p)]
    go_out = [io.BytesIO() if i in erase else None for i in range(k + p)]
    GoStream8(k, p, blk).reconstruct(mk_in(), go_out)
    m_out = [io.BytesIO() if i in erase else None for i in range(k + p)]
    engines8[name].reconstruct(mk_in(), m_out)
    for i in erase:
        assert m_out[i].getvalue() == go_out[i].getvalue()
        assert not any(m_out[i].getvalue())
