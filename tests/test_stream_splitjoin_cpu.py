"""StreamSplit / StreamJoin (reedsolomon16_amd.stream.stream_split /
stream_join; rsStream16.split/join streaming16.go:635-754, 882-1196 and the
identical rsStreamFF8 ones, streaming8.go:769-876, 1003-1320).

The layouts below are worked out by hand from the Go code, not by running
the transcription: shard sizes per (k, size), where the data ends up, and
which branch of join reads what."""
import io

import numpy as np
import pytest

from reedsolomon16_amd.codec import ErrNilWriter, ErrShortData, ErrSize, ErrTooFewShards
from reedsolomon16_amd.stream import stream_join, stream_split


def _data(n):
    return bytes(i % 256 for i in range(n))


def _split(k, data, size=None):
    dst = [io.BytesIO() for _ in range(k)]
    stream_split(k, io.BytesIO(data), dst, len(data) if size is None else size)
    return [d.getvalue() for d in dst]


# (k, size) -> shard lengths.  per = ceil64(ceil64(size) / k); when the last
# shard would get nothing, per = ceil64((size - 1) / (k - 1)) and the last
# shard at least one byte (streaming16.go:643-700)
LAYOUTS = {
    (4, 1): [0, 0, 0, 64],        # per 0: every byte in the last shard
    (4, 32): [64, 64, 64, 64],    # data ends in shard 0, the rest zero-filled at 64
    (4, 65): [64, 64, 64, 64],
    (4, 129): [64, 64, 64, 64],   # shard 2 holds one byte, shard 3 zero-filled
    (4, 1000): [256, 256, 256, 256],
    (3, 1000): [384, 384, 256],
    (4, 1024): [256] * 4,
    (2, 16384): [8192, 8192],
    (1, 1024): [1024],
    (100, 16384): [192] * 100,    # data ends in shard 85; 86..99 zero
    (200, 100): [0] * 199 + [128],
    (5, 6400): [1280] * 5,
}


@pytest.mark.parametrize("k,n", sorted(LAYOUTS))
def test_stream_split_layout(k, n):
    data = _data(n)
    got = _split(k, data)
    assert [len(s) for s in got] == LAYOUTS[(k, n)]
    # the data lies in order at the front of the shards, zeros after it
    flat, pos = b"", 0
    for s in got:
        take = min(len(s), n - pos)
        flat += s[:take]
        assert s[take:] == bytes(len(s) - take)
        pos += take
    assert flat == data


def test_stream_split_explicit_bytes():
    data = _data(1000)
    s = _split(4, data)
    assert s[3] == data[768:1000] + bytes(24)
    s = _split(4, _data(129))
    assert s[2] == data[128:129] + bytes(63) and s[3] == bytes(64)


def test_stream_split_errors_and_short_reader():
    with pytest.raises(ErrShortData):
        _split(4, b"", 0)
    with pytest.raises(ErrTooFewShards):
        stream_split(4, io.BytesIO(b"x"), [io.BytesIO()] * 3, 1)
    # 300 bytes for a declared 1024: shards 0 and 1 are written (1 padded),
    # then shard 2's read finds the end of the stream (streaming16.go:720-724)
    dst = [io.BytesIO() for _ in range(4)]
    data = _data(300)
    with pytest.raises(ErrShortData):
        stream_split(4, io.BytesIO(data), dst, 1024)
    assert dst[0].getvalue() == data[:256]
    assert dst[1].getvalue() == data[256:] + bytes(212)
    assert dst[2].getvalue() == b"" and dst[3].getvalue() == b""
    # a reader holding more than `size` is read no further than the layout
    rd = io.BytesIO(_data(5000))
    dst = [io.BytesIO() for _ in range(4)]
    stream_split(4, rd, dst, 1024)
    assert rd.tell() == 1024


class Chunky:
    """A reader that returns at most `chunk` bytes per Read and has no Seek."""

    def __init__(self, data, chunk):
        self.b, self.chunk = io.BytesIO(data), chunk

    def read(self, n=-1):
        return self.b.read(min(n, self.chunk) if n >= 0 else self.chunk)


class ChunkySeek(Chunky):
    def seek(self, *a):
        return self.b.seek(*a)


def _join(k, p, shards, n):
    out = io.BytesIO()
    stream_join(k, p, out, shards, n)
    return out.getvalue()


@pytest.mark.parametrize("k,n", sorted(LAYOUTS))
def test_stream_join_of_split_round_trips(k, n):
    data = _data(n)
    shards = _split(k, data)
    assert _join(k, 2, [io.BytesIO(s) for s in shards], n) == data
    # the same through the non-seekable (buffered) branch
    assert _join(k, 2, [Chunky(s, 1 << 20) for s in shards], n) == data


def test_stream_join_small_output_reads_every_reader_in_turn():
    # out_size <= k (streaming16.go:896-923): any non-nil reader, parity
    # readers of a k + p list included, feeds the output
    par = [b"\x11" * 64, b"\x22" * 64]
    assert _join(4, 2, [io.BytesIO(b"")] * 4 + [io.BytesIO(x) for x in par], 3) == b"\x11\x11\x11"
    assert _join(4, 2, [None, io.BytesIO(b"ab"), io.BytesIO(b"cd")], 3) == b"abc"
    with pytest.raises(ErrShortData):
        _join(4, 2, [io.BytesIO(b"a"), None], 2)


def test_stream_join_reader_count_rules():
    d = [_data(256)] * 4
    # k + p readers: only the first k are joined (:927-929); a nil among them fails
    assert _join(4, 2, [io.BytesIO(x) for x in d] + [None, None], 1024) == b"".join(d)
    with pytest.raises(ErrTooFewShards):
        _join(4, 2, [None] + [io.BytesIO(x) for x in d[1:]] + [io.BytesIO(x) for x in d[:2]], 1024)
    with pytest.raises(ErrTooFewShards):
        _join(4, 2, [io.BytesIO(x) for x in d[:3]], 1024)
    with pytest.raises(ErrNilWriter):
        stream_join(4, 2, None, [io.BytesIO(x) for x in d], 10)
    with pytest.raises(ErrTooFewShards):
        _join(4, 2, [], 10)
    with pytest.raises(ErrSize):
        _join(4, 2, [io.BytesIO(x) for x in d], 0)


def test_stream_join_under_1000_bytes_reads_each_shard_once():
    # one Read per shard (:976-1010): a reader handing out 10 bytes per Read
    # leaves the join short
    pieces = [_data(100)[i * 25:(i + 1) * 25] for i in range(4)]
    assert _join(4, 2, [io.BytesIO(x) for x in pieces], 100) == _data(100)
    with pytest.raises(ErrShortData):
        _join(4, 2, [ChunkySeek(x, 10) for x in pieces], 100)
    # the seekable >= 1000 branch reads each shard to its limit instead
    big = [_data(2000)[i * 512:(i + 1) * 512] for i in range(4)]
    assert _join(4, 2, [ChunkySeek(x, 10) for x in big], 2000) == _data(2000)


def test_stream_join_branches_differ_on_a_long_middle_shard():
    # k = 2 with three readers (not k + p, so all are kept), the last one nil;
    # per = ceil64(1250) = 1280
    a, b = b"A" * 1024, bytes(range(256)) * 8  # 1024 and 2048 bytes
    # seekable: shard 0 to its end (1024), shard 1 to per (1280): 2304 < 2500,
    # written, then ErrShortData (joinWithMultiReader :1022-1072)
    out = io.BytesIO()
    with pytest.raises(ErrShortData):
        stream_join(2, 2, out, [io.BytesIO(a), io.BytesIO(b), None], 2500)
    assert out.getvalue() == a + b[:1280]
    # buffered: the last non-nil reader is read on to the end of the output
    # (joinWithBufferedReads :1158-1188)
    assert _join(2, 2, [Chunky(a, 4096), Chunky(b, 4096), None], 2500) == a + b[:1476]


def test_stream_join_above_10_mib_takes_the_buffered_branch():
    n = 10 * 1024 * 1024 + 64
    rng = np.random.default_rng(3)
    data = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
    shards = _split(2, data)
    assert [len(s) for s in shards] == [5 * 1024 * 1024 + 64, 5 * 1024 * 1024]  # per = ceil64(5 MiB + 32)
    assert _join(2, 1, [io.BytesIO(s) for s in shards], n) == data


def _hypothesis():
    try:
        import hypothesis  # noqa: F401
        return True
    except ImportError:
        return False


@pytest.mark.skipif(not _hypothesis(), reason="hypothesis not installed")
def test_stream_split_join_properties():
    """Random (k, size): StreamJoin(StreamSplit(x)) == x through every join
    branch, every shard a multiple of 64 bytes, at most one shard's worth of
    zero padding past the data in the non-empty shards."""
    from hypothesis import given, settings, strategies as st

    @settings(max_examples=300, deadline=None)
    @given(st.integers(1, 300), st.integers(1, 40000), st.booleans())
    def check(k, n, seekable):
        data = bytes((i * 7 + k) % 256 for i in range(n))
        shards = _split(k, data)
        assert len(shards) == k
        assert all(len(s) % 64 == 0 for s in shards)
        assert sum(len(s) for s in shards) >= n
        rd = [io.BytesIO(s) if seekable else Chunky(s, 1 << 16) for s in shards]
        if seekable and _split_per(k, n) != _join_per(k, n):
            # the reference's own split and seekable join disagree on the
            # shard size here (test_reference_split_join_size_mismatch)
            return
        assert _join(k, 3, rd, n) == data

    check()


def _split_per(k, n):
    """rsStream16.split's shard size (streaming16.go:645-676): floor of the
    64-aligned size over k, rounded up to 64; recomputed from (size - 1) /
    (k - 1) when the last shard would get nothing."""
    aligned = -(-(n + (n & 1)) // 64) * 64
    per = -(-(aligned // k) // 64) * 64
    if n - per * (k - 1) <= 0 and k > 1:
        per = -(-((n - 1) // (k - 1)) // 64) * 64
    return per


def _join_per(k, n):
    """joinWithMultiReader's shard size (streaming16.go:1022-1031): the
    ceiling of size over k, rounded up to 64."""
    per = -(-n // k)
    return -(-per // 64) * 64 if per % 64 else per


def test_reference_split_join_size_mismatch():
    """k = 70, 4536 bytes: split writes 64-byte shards (4544 // 70 = 64) but
    the seekable join expects ceil(4536 / 70) -> 128 per shard, so its last
    shard's limit goes negative, the multi-reader stops one shard short and
    the join reports short data -- the reference's behaviour, restated; the
    buffered (non-seekable) branch reads the last shard to the end and
    round-trips."""
    k, n = 70, 4536
    assert (_split_per(k, n), _join_per(k, n)) == (64, 128)
    data = bytes((i * 7 + k) % 256 for i in range(n))
    shards = _split(k, data)
    with pytest.raises(ErrShortData):
        _join(k, 3, [io.BytesIO(s) for s in shards], n)
    assert _join(k, 3, [Chunky(s, 1 << 16) for s in shards], n) == data
