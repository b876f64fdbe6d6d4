"""The pipelined stream mirrors (reedsolomon16_amd/stream.py) against the
single-buffer restatements of rsStream16 and rsStreamFF8 (tests/go_stream.py),
on the CPU: the codec behind the mirror is an oracle-backed stand-in with the
engine's ticket API, so these tests check the block logic (sizes, padding,
truncation, the verify loop's zeroed 64-byte pad and the panic after it,
output sizes, block order, depth rotation).  The same comparisons run through
the HIP engine in test_gpu_stream.py."""
import io

import numpy as np
import pytest

from oracle.orc import Oracle
from reedsolomon16_amd.codec import ErrPanic
from reedsolomon16_amd.stream import StreamEncoder8, StreamEncoder16, StreamReadError
from tests.go_stream import GoPanic, GoStream8, GoStream16


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

    def __init__(self, k, p, bits=16):
        self.k, self.p, self.total = k, p, k + p
        self.orc = Oracle(bits, k, p)
        self.calls = []

    def reset_inversion_cache(self):
        """A fresh newFF8's empty inversion cache (stream.py _fresh_codec)."""
        self.orc = Oracle(self.orc.bits, self.k, self.p)

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


def _mirror(k, p, depth=2, bits=16):
    fake = OracleTicketCodec(k, p, bits)
    cls = StreamEncoder16 if bits == 16 else StreamEncoder8
    return cls(k, p, block_size=BLOCK, depth=depth, codec=fake), fake


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


def _outcome(fn, *args):
    """A verify verdict, or "panic" for the reference's Go panic / the
    mirror's ErrPanic."""
    try:
        return fn(*args)
    except (GoPanic, ErrPanic):
        return "panic"


@pytest.mark.parametrize("n", [768, 999, 700, 62, 20, 130])
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
    gv = _outcome(go.verify, _streams(shards))
    st, fake = _mirror(k, p)
    assert _outcome(st.verify, _streams(shards)) == gv
    # every block the reference verified was verified with the same bytes
    # (the mirror may have queued one more block after a mismatch)
    assert fake.calls[:len(go.calls)] == go.calls


@pytest.mark.parametrize("k,p,n,want", [
    # 4 + 2 has only GF(2^8) twiddles: a parity symbol's high byte depends on
    # the data's high bytes alone, the zero pad (which covers every high byte
    # the data lacks) drops zero parity, the block verifies, and the next
    # all[i][:r.blockSize] (:218) panics -- a single block as the tail of a
    # multi-block stream, whichever half the pad starts in
    (4, 2, BLOCK + 20, "panic"), (4, 2, 20, "panic"), (4, 2, 130, "panic"),
    (4, 2, BLOCK + 100, "panic"), (4, 2, 100, "panic"), (4, 2, 62, "panic"),
    # padded up to exactly blockSize: the capacity stays blockSize, no panic
    (4, 2, 2 * BLOCK - 10, True),
    # 300 + 4: chunk twiddles from fftSkew[255] on are full-field, so the pad
    # drops nonzero parity bytes and the block verifies False
    (300, 4, BLOCK + 20, False), (300, 4, 100, False), (300, 4, 62, False),
])
def test_stream_verify_unaligned_last_block_is_zero_padded(k, p, n, want):
    """streaming16.go:290-309: every row reaching :295 is `size` bytes long, so
    each becomes a fresh zeroed buffer of alignedSize; the parity rows' real
    bytes past `size` are replaced by zeros."""
    datas, par = _encoded_stream(k, p, n, n + k)
    go = GoStream16(k, p, BLOCK)
    assert _outcome(go.verify, _streams(list(datas) + par)) == want
    st, fake = _mirror(k, p)
    assert _outcome(st.verify, _streams(list(datas) + par)) == want
    assert fake.calls == go.calls
    # the codec saw zeros past `size` in every row, parity included
    size = (n - 1) % BLOCK + 1
    size += size % 2
    assert all(set(r[size:]) <= {0} for r in go.calls[-1][1])
    if want is not True:
        assert any(set(r[size:]) != {0} for r in par_blocks(par, len(go.calls) - 1)) == (want is False)


def par_blocks(par, blk):
    return [np.frombuffer(x, np.uint8)[blk * BLOCK:(blk + 1) * BLOCK] for x in par]


def test_stream_verify_true_on_unaligned_block_panics():
    """If the zero-padded block verifies (here: all-zero shards), the reference
    loops back to all[i][:r.blockSize] (streaming16.go:218) on a row whose
    capacity is now alignedSize, and panics; the mirror raises ErrPanic there.
    A tail whose alignedSize equals blockSize keeps the capacity and ends
    normally."""
    k, p = 4, 2
    shards = [bytes(100)] * k + [bytes(128)] * p
    with pytest.raises(GoPanic):
        GoStream16(k, p, BLOCK).verify(_streams(shards))
    st, fake = _mirror(k, p)
    with pytest.raises(ErrPanic):
        st.verify(_streams(shards))
    assert len(fake.calls) == 1
    # an aligned all-zero stream verifies and ends normally
    shards = [bytes(2 * BLOCK)] * k + [bytes(2 * BLOCK)] * p
    assert GoStream16(k, p, BLOCK).verify(_streams(shards)) is True
    assert _mirror(k, p)[0].verify(_streams(shards)) is True
    # a tail padded up to exactly blockSize
    shards = [bytes(2 * BLOCK - 10)] * k + [bytes(2 * BLOCK)] * p
    assert GoStream16(k, p, BLOCK).verify(_streams(shards)) is True
    assert _mirror(k, p)[0].verify(_streams(shards)) is True
    # a multi-block zero stream with an unaligned tail: full blocks verify,
    # the tail verifies, then the reference panics
    shards = [bytes(BLOCK + 70)] * k + [bytes(BLOCK + 128)] * p
    with pytest.raises(GoPanic):
        GoStream16(k, p, BLOCK).verify(_streams(shards))
    with pytest.raises(ErrPanic):
        _mirror(k, p, depth=3)[0].verify(_streams(shards))


# row-length classes at streaming16.go:295-302: the block size (aligned, odd,
# even and unaligned in the low / high half of a 64-byte block) and each
# row's own length (exact, short -> zero-extended, long -> truncated, nil)
VERIFY_ROW_CLASSES = {
    "aligned": (128, [128, 128, 128, 128, 128, 128]),
    "odd": (99, [99, 99, 50, 99, 99, 99]),
    "odd_to_64": (63, [63, 63, 63, 63, 63, 64]),
    "even_low_half": (20, [20, 7, 20, None, 20, 64]),
    "even_high_half": (52, [52, 52, 80, 52, 64, 64]),
    "two_blocks_tail_low": (BLOCK + 2, [BLOCK + 2] * 4 + [BLOCK + 64] * 2),
    "two_blocks_tail_high": (BLOCK + 90, [BLOCK + 90, BLOCK + 91, BLOCK + 1, BLOCK + 90, BLOCK + 128, BLOCK + 128]),
}


@pytest.mark.parametrize("case", sorted(VERIFY_ROW_CLASSES))
@pytest.mark.parametrize("zero", [False, True])
def test_stream_verify_row_length_classes(case, zero):
    k, p = 4, 2
    n, lens = VERIFY_ROW_CLASSES[case]
    rng = np.random.default_rng(len(case))
    if zero:
        shards = [None if m is None else bytes(m) for m in lens]
    else:
        datas, par = _encoded_stream(k, p, n, len(case))
        shards = [None if m is None else (d * 2)[:m] for d, m in zip(list(datas) + par, lens)]
    go = GoStream16(k, p, BLOCK)
    want = _outcome(go.verify, _streams(shards))
    st, fake = _mirror(k, p)
    assert _outcome(st.verify, _streams(shards)) == want
    assert fake.calls[:len(go.calls)] == go.calls
    if zero:
        assert want == ("panic" if (n + n % 2) % 64 else True)


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


# --------------------------------------------------------------------------- rsStreamFF8
def _encoded_stream8(k, p, n, seed):
    rng = np.random.default_rng(seed)
    datas = _data(rng, [n] * k)
    go = GoStream8(k, p, BLOCK)
    outs = [io.BytesIO() for _ in range(p)]
    go.encode(_streams(datas), outs)
    return datas, [o.getvalue() for o in outs]


@pytest.mark.parametrize("depth", [1, 2, 3])
@pytest.mark.parametrize("case", sorted(ENC_CASES))
def test_stream8_encode_matches_go_loop(case, depth):
    """streaming8.go:109-181: no even step, zero pad to 64, ceil64(size) parity bytes."""
    k, p = 6, 3
    rng = np.random.default_rng(len(case) * 11 + depth)
    datas = _data(rng, ENC_CASES[case])
    go = GoStream8(k, p, BLOCK)
    gout = [io.BytesIO() for _ in range(p)]
    go.encode(_streams(datas), gout)
    st, fake = _mirror(k, p, depth, bits=8)
    mout = [io.BytesIO() for _ in range(p)]
    st.encode(_streams(datas), mout)
    assert fake.calls == go.calls
    assert [o.getvalue() for o in mout] == [o.getvalue() for o in gout]


@pytest.mark.parametrize("n", [768, 999, 700, 62, 33])
@pytest.mark.parametrize("tamper", [None, 0, 7])
def test_stream8_verify_matches_go_loop(n, tamper):
    """streaming8.go:343-444: the block buffer keeps its capacity and the pad
    is zeroed, so an unaligned tail verifies (byte columns are independent)."""
    k, p = 5, 3
    datas, par = _encoded_stream8(k, p, n, n)
    shards = list(datas) + list(par)
    if tamper is not None:
        b = bytearray(shards[tamper])
        b[min(300, len(b) - 1)] ^= 1
        shards[tamper] = bytes(b)
    go = GoStream8(k, p, BLOCK)
    gv = go.verify(_streams(shards))
    st, fake = _mirror(k, p, bits=8)
    assert st.verify(_streams(shards)) == gv
    assert fake.calls[:len(go.calls)] == go.calls
    if tamper is None:
        assert gv is True


@pytest.mark.parametrize("n", [768, 999, 130])
@pytest.mark.parametrize("erase", [(0,), (1, 6), (0, 2, 5)])
def test_stream8_reconstruct_data_matches_go_loop(n, erase):
    """streaming8.go:609-766 (what StreamReconstruct runs when only data
    outputs are requested, reedsolomon.go:174-185): rebuilds the data shards."""
    k, p = 5, 3
    datas, par = _encoded_stream8(k, p, n, n + 3)
    shards = list(datas) + list(par)
    mk_in = lambda: [None if i in erase else io.BytesIO(shards[i]) for i in range(k + p)]
    go_out = [io.BytesIO() if i in erase and i < k else None for i in range(k + p)]
    go = GoStream8(k, p, BLOCK)
    go.reconstruct_data(mk_in(), go_out)
    m_out = [io.BytesIO() if i in erase and i < k else None for i in range(k + p)]
    st, fake = _mirror(k, p, bits=8)
    st.reconstruct_data(mk_in(), m_out)
    assert fake.calls == go.calls
    for i in erase:
        if i < k:
            assert m_out[i].getvalue() == go_out[i].getvalue()
            # a nil parity input is fed as a zero shard (:680-685), so the
            # rebuilt data is right only when every parity shard is read
            assert (go_out[i].getvalue() == shards[i]) == all(j < k for j in erase)


@pytest.mark.parametrize("n", [768, 130])
def test_stream8_reconstruct_writes_zeros_like_the_reference(n):
    """streaming8.go:447-606 zero-extends every nil input (:389-393), so the
    codec sees all shards present and returns at once (leopard8.go:459-462),
    and every requested output receives zeros: `size` bytes per data shard,
    ceil64(size) per parity shard."""
    k, p = 5, 3
    datas, par = _encoded_stream8(k, p, n, 21)
    shards = list(datas) + list(par)
    erase = (1, 6)
    mk_in = lambda: [None if i in erase else io.BytesIO(shards[i]) for i in range(k + p)]
    go_out = [io.BytesIO() if i in erase else None for i in range(k + p)]
    go = GoStream8(k, p, BLOCK)
    go.reconstruct(mk_in(), go_out)
    m_out = [io.BytesIO() if i in erase else None for i in range(k + p)]
    st, fake = _mirror(k, p, bits=8)
    st.reconstruct(mk_in(), m_out)
    assert [c[0] for c in fake.calls] == [c[0] for c in go.calls]
    assert all(None not in c[1] for c in go.calls)  # nothing missing in any call
    for i in erase:
        assert m_out[i].getvalue() == go_out[i].getvalue()
    assert go_out[1].getvalue() == bytes(n)
    assert go_out[6].getvalue() == bytes((n + 63) // 64 * 64)


def _mirror_threads(k, p, bits, threads, depth=2):
    fake = OracleTicketCodec(k, p, bits)
    cls = StreamEncoder16 if bits == 16 else StreamEncoder8
    return cls(k, p, block_size=BLOCK, depth=depth, codec=fake, threads=threads), fake


@pytest.mark.parametrize("bits", [16, 8])
@pytest.mark.parametrize("case", sorted(ENC_CASES))
def test_stream_threads_same_bytes_as_go_loop(case, bits):
    """threads > 1 (a pool reads a block's readers and writes its writers):
    the codec sees the same blocks and the writers the same bytes as the
    reference's sequential loops, for encode, verify and reconstruct."""
    k, p = 6, 3
    rng = np.random.default_rng(len(case) * 3 + bits)
    datas = _data(rng, ENC_CASES[case])
    go = (GoStream16 if bits == 16 else GoStream8)(k, p, BLOCK)
    gout = [io.BytesIO() for _ in range(p)]
    go.encode(_streams(datas), gout)
    st, fake = _mirror_threads(k, p, bits, 4)
    mout = [io.BytesIO() for _ in range(p)]
    st.encode(_streams(datas), mout)
    assert [o.getvalue() for o in mout] == [o.getvalue() for o in gout]
    if bits == 16:
        assert fake.calls == go.calls
    par = [o.getvalue() for o in gout]
    full = [d if d is not None else b"" for d in datas] + par
    assert _outcome(st.verify, _streams(full)) == _outcome(go.verify, _streams(full))
    # reconstruct two data shards into writers
    if all(d for d in datas):
        ins = [None if i in (0, 2) else full[i] for i in range(k + p)]
        outs_m = [io.BytesIO() if i in (0, 2) else None for i in range(k + p)]
        outs_g = [io.BytesIO() if i in (0, 2) else None for i in range(k + p)]
        st.reconstruct_data(_streams(ins), outs_m)
        go.reconstruct_data(_streams(ins), outs_g)
        assert [o.getvalue() if o else None for o in outs_m] == [o.getvalue() if o else None for o in outs_g]


class _Boom:
    def __init__(self, data, fail):
        self.b, self.fail = io.BytesIO(data), fail

    def readinto(self, mv):
        if self.fail:
            raise OSError("disk gone")
        return self.b.readinto(mv)


def test_stream_threads_report_the_lowest_failing_reader():
    k, p = 6, 3
    st, _ = _mirror_threads(k, p, 16, 4)
    rd = [_Boom(b"x" * 128, fail=i in (2, 5)) for i in range(k)]
    with pytest.raises(StreamReadError) as ei:
        st.encode(rd, [io.BytesIO() for _ in range(p)])
    assert ei.value.stream == 2


def test_stream_threads_aliased_reader_reads_in_order():
    """One reader object passed for several shards (advisor finding, round 5):
    with threads > 1 the mirror reads it in index order, as the reference's
    sequential loop does, so every shard gets the same bytes as threads = 1."""
    k, p = 6, 3
    payload = bytes(range(256)) * 40
    outs = []
    for threads in (1, 4):
        st, _ = _mirror_threads(k, p, 16, threads)
        shared = io.BytesIO(payload)
        mout = [io.BytesIO() for _ in range(p)]
        st.encode([shared] * k, mout)
        outs.append([o.getvalue() for o in mout])
        st.close()
    assert outs[0] == outs[1]


def test_stream_close_shuts_the_pool_down():
    st, _ = _mirror_threads(4, 2, 16, 4)
    pool = st._pool
    st.close()
    assert st._pool is None and pool._shutdown
