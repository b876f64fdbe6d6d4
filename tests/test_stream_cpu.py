"""The pipelined stream mirror (reedsolomon16_amd/stream.py) against the
single-buffer restatement of rsStream16 (tests/go_stream.py), on the CPU: the
codec behind the mirror is an oracle-backed stand-in with the engine's ticket
API, so these tests check the block logic (sizes, padding, truncation, the
verify loop's stale 64-byte pad, output sizes, block order, depth rotation).
The same comparisons run through the HIP engine in test_gpu_stream.py."""
import io

import numpy as np
import pytest

from oracle.orc import Oracle
from reedsolomon16_amd.stream import StreamEncoder16
from tests.go_stream import GoStream16


class _Ticket:
    def __init__(self, ok=True):
        self.ok = ok
        self.waited = False

    def wait(self):
        self.waited = True

    def done(self):
        return True

    def result(self):
        self.waited = True
        return self.ok


class OracleTicketCodec:
    """Oracle stand-in for reedsolomon16_amd.codec.ReedSolomon's ticket API
    (test infrastructure: records what the stream hands the codec)."""

    def __init__(self, k, p):
        self.k, self.p, self.total = k, p, k + p
        self.orc = Oracle(16, k, p)
        self.calls = []

    def alloc_aligned(self, each, shards=None, pinned=False):
        n = self.total if shards is None else shards
        slab = np.full(each * n, 0xA5, np.uint8)  # not zero: the mirror must not rely on fresh memory
        return [slab[i * each:(i + 1) * each] for i in range(n)]

    def encode_async(self, shards):
        rows = [np.asarray(s) for s in shards]
        assert self.orc.encode(rows) == 0
        self.calls.append(("encode", [bytes(r) for r in rows]))
        return _Ticket()

    def verify_async(self, shards):
        rows = [np.asarray(s) for s in shards]
        ok, e = self.orc.verify(rows)
        assert e == 0
        self.calls.append(("verify", [bytes(r) for r in rows]))
        return _Ticket(ok)

    def reconstruct_async(self, shards, recover_all=True):
        from reedsolomon16_amd.codec import EmptyShard

        rows = [None if (s is None or len(s) == 0) else np.asarray(s) for s in shards]
        self.calls.append(("reconstruct", [None if r is None else bytes(r) for r in rows]))
        e, out = self.orc.reconstruct(rows, recover_all)
        assert e == 0, e
        end = self.total if recover_all else self.k
        for i in range(end):
            if rows[i] is None and out[i] is not None:
                s = shards[i]
                buf = s.buf if isinstance(s, EmptyShard) else np.empty(len(out[i]), np.uint8)
                buf[:len(out[i])] = out[i]
                shards[i] = buf[:len(out[i])]
        return _Ticket()


BLOCK = 256


def _streams(datas):
    return [None if d is None else io.BytesIO(d) for d in datas]


def _mirror(k, p, depth=2):
    fake = OracleTicketCodec(k, p)
    return StreamEncoder16(k, p, block_size=BLOCK, depth=depth, codec=fake), fake


def _data(rng, lens):
    return [None if n is None else rng.integers(0, 256, n, dtype=np.uint8).tobytes() for n in lens]


ENC_CASES = {
    "aligned_3_blocks": [768] * 6,
    "odd_tail": [999] * 6,
    "one_short_block": [33] * 6,
    "ragged_truncate_extend": [999, 1200, 500, 1000, 999, 0],
    "nil_reader": [700, None, 700, 700, 700, 700],
    "first_shorter": [100, 900, 900, 900, 900, 900],
}


@pytest.mark.parametrize("depth", [1, 2, 3])
@pytest.mark.parametrize("case", sorted(ENC_CASES))
def test_stream_encode_matches_go_loop(case, depth):
    k, p = 6, 3
    rng = np.random.default_rng(len(case) * 7 + depth)
    datas = _data(rng, ENC_CASES[case])
    go = GoStream16(k, p, BLOCK)
    gout = [io.BytesIO() for _ in range(p)]
    go.encode(_streams(datas), gout)
    st, fake = _mirror(k, p, depth)
    mout = [io.BytesIO() for _ in range(p)]
    st.encode(_streams(datas), mout)
    assert [c[0] for c in fake.calls] == [c[0] for c in go.calls]
    assert fake.calls == go.calls  # the codec saw the same blocks, byte for byte
    assert [o.getvalue() for o in mout] == [o.getvalue() for o in gout]


def _encoded_stream(k, p, n, seed):
    rng = np.random.default_rng(seed)
    datas = _data(rng, [n] * k)
    go = GoStream16(k, p, BLOCK)
    outs = [io.BytesIO() for _ in range(p)]
    go.encode(_streams(datas), outs)
    return datas, [o.getvalue() for o in outs]


@pytest.mark.parametrize("n", [768, 999, 700, 62])
@pytest.mark.parametrize("tamper", [None, 0, 7])
def test_stream_verify_matches_go_loop(n, tamper):
    k, p = 5, 3
    datas, par = _encoded_stream(k, p, n, n)
    shards = list(datas) + list(par)
    if tamper is not None:
        b = bytearray(shards[tamper])
        b[min(300, len(b) - 1)] ^= 1
        shards[tamper] = bytes(b)
    go = GoStream16(k, p, BLOCK)
    gv = go.verify(_streams(shards))
    st, fake = _mirror(k, p)
    mv = st.verify(_streams(shards))
    assert mv == gv
    # every block the reference verified was verified with the same bytes
    # (the mirror may have queued one more block after a mismatch)
    assert fake.calls[:len(go.calls)] == go.calls


def test_stream_verify_stale_pad_is_reference_behaviour():
    """A multi-block stream whose last block is not 64-aligned: the reference's
    verify pads it with the previous block's bytes (streaming16.go:290-309),
    so it reports a mismatch for a stream its own encode produced."""
    k, p = 4, 2
    datas, par = _encoded_stream(k, p, BLOCK + 100, 3)
    go = GoStream16(k, p, BLOCK)
    assert go.verify(_streams(list(datas) + par)) is False
    st, fake = _mirror(k, p)
    assert st.verify(_streams(list(datas) + par)) is False
    assert fake.calls == go.calls
    # a single-block stream (fresh, zeroed buffer) verifies
    datas, par = _encoded_stream(k, p, 100, 4)
    assert GoStream16(k, p, BLOCK).verify(_streams(list(datas) + par)) is True
    assert _mirror(k, p)[0].verify(_streams(list(datas) + par)) is True


@pytest.mark.parametrize("n", [768, 999, 130])
@pytest.mark.parametrize("erase", [(0,), (1, 6), (0, 2, 5), (5, 6, 7)])
def test_stream_reconstruct_matches_go_loop(n, erase):
    k, p = 5, 3
    datas, par = _encoded_stream(k, p, n, n + len(erase))
    shards = list(datas) + list(par)
    inputs = [None if i in erase else io.BytesIO(shards[i]) for i in range(k + p)]
    go_out = [io.BytesIO() if i in erase else None for i in range(k + p)]
    go = GoStream16(k, p, BLOCK)
    go.reconstruct(inputs, go_out)
    inputs = [None if i in erase else io.BytesIO(shards[i]) for i in range(k + p)]
    m_out = [io.BytesIO() if i in erase else None for i in range(k + p)]
    st, fake = _mirror(k, p)
    st.reconstruct(inputs, m_out)
    assert fake.calls == go.calls
    for i in erase:
        assert m_out[i].getvalue() == go_out[i].getvalue()
        if i < k:
            assert m_out[i].getvalue() == shards[i]


@pytest.mark.parametrize("n", [768, 999])
def test_stream_reconstruct_data_matches_go_loop(n):
    k, p = 5, 3
    datas, par = _encoded_stream(k, p, n, 11)
    shards = list(datas) + list(par)
    erase = (1, 3)
    mk_in = lambda: [None if i in erase else io.BytesIO(shards[i]) for i in range(k + p)]
    go_out = [io.BytesIO() if i in erase else None for i in range(k + p)]
    go = GoStream16(k, p, BLOCK)
    go.reconstruct_data(mk_in(), go_out)
    m_out = [io.BytesIO() if i in erase else None for i in range(k + p)]
    st, fake = _mirror(k, p)
    st.reconstruct_data(mk_in(), m_out)
    assert fake.calls == go.calls
    for i in erase:
        assert m_out[i].getvalue() == go_out[i].getvalue() == shards[i]


def test_stream_errors():
    from reedsolomon16_amd.codec import ErrInvShardNum, ErrShardNoData, ErrTooFewShards
    from reedsolomon16_amd.stream import ErrReconstructMismatch, StreamReadError, StreamWriteError

    with pytest.raises(ErrInvShardNum):
        StreamEncoder16(0, 2, codec=OracleTicketCodec(1, 2))
    st, _ = _mirror(4, 2)
    with pytest.raises(ErrTooFewShards):
        st.encode(_streams([b"x"] * 3), [io.BytesIO()] * 2)
    with pytest.raises(ErrShardNoData):
        st.verify(_streams([b""] * 6))
    with pytest.raises(ErrReconstructMismatch):
        st.reconstruct(_streams([b"a"] * 6), [io.BytesIO()] + [None] * 5)

    class Bad:
        def read(self, n):
            raise OSError("disk")

    with pytest.raises(StreamReadError) as ei:
        st.encode([io.BytesIO(b"a" * 300), Bad(), io.BytesIO(b"a"), io.BytesIO(b"a")], [io.BytesIO(), io.BytesIO()])
    assert ei.value.stream == 1

    class Short:
        def write(self, b):
            return len(b) - 1

    with pytest.raises(StreamWriteError) as ei:
        st.encode(_streams([b"a" * 10] * 4), [io.BytesIO(), Short()])
    assert ei.value.stream == 5


def test_stream_write_order_and_read_error_after_blocks():
    """Blocks queued before a failing read are still written (the reference
    wrote them before it read the failing block)."""
    k, p = 4, 2
    rng = np.random.default_rng(9)
    datas = _data(rng, [3 * BLOCK] * k)

    class FailThird(io.BytesIO):
        def __init__(self, b):
            super().__init__(b)
            self.reads = 0

        def read(self, n=-1):
            if self.tell() >= 2 * BLOCK:
                raise OSError("late")
            return super().read(n)

        def readinto(self, b):
            if self.tell() >= 2 * BLOCK:
                raise OSError("late")
            return super().readinto(b)

    go = GoStream16(k, p, BLOCK)
    ref = [io.BytesIO() for _ in range(p)]
    go.encode(_streams([d[:2 * BLOCK] for d in datas]), ref)
    st, _ = _mirror(k, p)
    out = [io.BytesIO() for _ in range(p)]
    from reedsolomon16_amd.stream import StreamReadError

    with pytest.raises(StreamReadError):
        st.encode([io.BytesIO(datas[0])] + [FailThird(d) for d in datas[1:]], out)
    assert [o.getvalue() for o in out] == [o.getvalue() for o in ref]
