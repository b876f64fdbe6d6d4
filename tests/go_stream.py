"""Test helper: a line-by-line, single-buffer, synchronous restatement of the
reference's rsStream16 loops (streaming16.go:84-170 readInputs, :173-197
writeOutputs, :200-317 verify, :320-468 reconstruct, :471-632 reconstructData,
:1229-1318 encode), with r.rs.* calls answered by the oracle.  It is the
checker for reedsolomon16_amd/stream.py (the pipelined product mirror): both
must hand the codec the same bytes and write the same outputs.

Go slices are modelled as (buffer, length); the buffer's length is the
slice's capacity.  Re-slicing past it is the Go runtime panic (``GoPanic``),
and the ``make([]byte, n)`` branches allocate a fresh zeroed buffer of
capacity n -- the verify loop's 64-byte padding takes that branch for every
row (streaming16.go:295-299), which caps the row at alignedSize.

``GoStream8`` restates the GF(2^8) loops of streaming8.go the same way
(:109-181 encode, :242-316 readInputs, :318-340 writeOutputs, :343-444 verify,
:447-606 reconstruct, :609-766 reconstructData).
"""
from __future__ import annotations

import numpy as np

from oracle.orc import Oracle


class GoPanic(Exception):
    """A Go runtime panic (slice bounds out of range)."""


class GoSlice:
    __slots__ = ("buf", "n")

    def __init__(self, buf, n):
        self.buf, self.n = buf, n

    def view(self):
        return self.buf[:self.n]

    def cap(self):
        return len(self.buf)

    def reslice(self, n):
        """s = s[:n]"""
        if n > len(self.buf):
            raise GoPanic("slice bounds out of range [:%d] with capacity %d" % (n, len(self.buf)))
        self.n = n

    def full(self, n):
        """s[:n] as a writable view (io.ReadFull's destination)."""
        if n > len(self.buf):
            raise GoPanic("slice bounds out of range [:%d] with capacity %d" % (n, len(self.buf)))
        return self.buf[:n]

    def grow_copy(self, n):
        """newBuf := make([]byte, n); copy(newBuf, s); s = newBuf"""
        nb = np.zeros(n, np.uint8)
        m = min(self.n, n)
        nb[:m] = self.buf[:m]
        self.buf, self.n = nb, n


def _read_full(rd, view) -> int:
    n = 0
    while n < len(view):
        b = rd.read(len(view) - n)
        if not b:
            break
        view[n:n + len(b)] = np.frombuffer(b, np.uint8)
        n += len(b)
    return n


def _alloc(total, block):
    return [GoSlice(np.zeros(block, np.uint8), block) for _ in range(total)]


class GoStream16:
    def __init__(self, k, p, block=4 << 20):
        self.k, self.p, self.total, self.block = k, p, k + p, block
        self.orc = Oracle(16, k, p)
        self.calls = []  # (op, list of the shard byte strings the codec saw)

    # readInputs streaming16.go:84-170
    def _read_inputs(self, readers, dst):
        size = -1
        for i, rd in enumerate(readers):
            if rd is None:
                dst[i].n = 0
                continue
            n = _read_full(rd, dst[i].full(self.block))
            if n > 0 and size == -1:
                size = n
            dst[i].n = n
        if size == -1:
            return -1
        if size % 2:
            size += 1
        for s in dst:
            cur = s.n
            if cur == 0:
                s.n = size
                s.buf[:size] = 0
            elif cur < size:
                s.n = size
                s.buf[cur:size] = 0
            elif cur > size:
                s.n = size
        padded = size
        if padded % 64 or padded % 2:
            padded = (padded + 63) // 64 * 64
            for s in dst:
                if s.n == size:
                    s.n = padded
                    s.buf[size:padded] = 0
        return size

    def encode(self, inputs, outputs):
        shards = _alloc(self.total, self.block)
        while True:
            size = self._read_inputs(inputs, shards[:self.k])
            if size < 0:
                return
            al = size + (2 - size % 2) if size % 2 else size
            if al % 64:
                al = (al + 63) // 64 * 64
            for i, s in enumerate(shards):
                s.n = al
                if i < self.k and al > size:
                    s.buf[size:al] = 0
            rows = [s.view() for s in shards]
            assert self.orc.encode(rows) == 0
            self.calls.append(("encode", [bytes(r) for r in rows]))
            wal = (size + 63) // 64 * 64  # writeOutputs
            for j, w in enumerate(outputs):
                if w is not None:
                    w.write(bytes(shards[self.k + j].buf[:wal]))

    def verify(self, readers):
        """streaming16.go:200-317."""
        all_ = _alloc(self.total, self.block)
        read = 0
        while True:
            size = -1
            for i, rd in enumerate(readers):
                if rd is None:
                    all_[i].reslice(0)
                    continue
                n = _read_full(rd, all_[i].full(self.block))  # :218 panics past the capacity
                if size == -1 and n > 0:
                    size = n
                all_[i].reslice(n)
            if size in (-1, 0):
                if read == 0:
                    raise ValueError("ErrShardNoData")
                return True
            for s in all_:  # :245-270
                cur = s.n
                if cur == 0:
                    s.reslice(size)
                    s.buf[:size] = 0
                elif cur < size:
                    if s.cap() < size:
                        s.grow_copy(size)
                    else:
                        s.reslice(size)
                    s.buf[cur:size] = 0
                elif cur > size:
                    s.reslice(size)
            if size % 2:  # :274-287
                ps = size + 1
                for s in all_:
                    if s.n == size:
                        s.reslice(ps)
                        s.buf[size:ps] = 0
                size = ps
            al = size
            if size % 64:  # :290-309
                al = (size + 63) // 64 * 64
                for s in all_:
                    if s.n > 0:
                        if s.n < al:
                            s.grow_copy(al)  # every row: len == size < alignedSize
                        else:
                            s.reslice(al)
                        s.buf[s.n:al] = 0  # :304 starts at len(all[i]) == alignedSize: no-op
            read += size
            rows = [s.view() for s in all_]
            ok, e = self.orc.verify(rows)
            assert e == 0
            self.calls.append(("verify", [bytes(r) for r in rows]))
            if not ok:
                return False

    def _rebuild(self, all_, recover_all):
        rows = [s.view() if s.n else None for s in all_]
        self.calls.append(("reconstruct", [None if r is None else bytes(r) for r in rows]))
        e, out = self.orc.reconstruct(rows, recover_all)
        assert e == 0, e
        end = self.total if recover_all else self.k
        for i in range(end):
            if rows[i] is None:
                S = len(out[i])
                all_[i].buf[:S] = out[i]
                all_[i].n = S

    def reconstruct(self, inputs, outputs):
        all_ = _alloc(self.total, self.block)
        data_only = True
        for i in range(self.total):
            if inputs[i] is not None and outputs[i] is not None:
                raise ValueError("ErrReconstructMismatch")
            if i >= self.k and outputs[i] is not None:
                data_only = False
        missing = {i for i in range(self.total) if inputs[i] is None and outputs[i] is not None}
        if not missing:
            return
        read = 0
        while True:
            size = 0
            for i, rd in enumerate(inputs):
                if rd is None:
                    all_[i].n = 0
                    continue
                n = _read_full(rd, all_[i].full(self.block))
                all_[i].n = n
                if n > 0 and size == 0:
                    size = n
            if size == 0:
                if read == 0:
                    raise ValueError("ErrShardNoData")
                return
            orig = size
            al = (size + 63) // 64 * 64
            for i, s in enumerate(all_):
                if i in missing:
                    s.n = 0
                elif s.n == 0:
                    raise ValueError("ErrShardNoData")
                elif s.n < al:
                    cur = s.n
                    s.n = al
                    s.buf[cur:al] = 0
                elif s.n > al:
                    s.n = al
            self._rebuild(all_, not data_only)
            for i, w in enumerate(outputs):
                if w is None or i not in missing:
                    continue
                ws = orig if i < self.k else al
                w.write(bytes(all_[i].buf[:ws]))
            read += orig

    def reconstruct_data(self, inputs, outputs):
        all_ = _alloc(self.total, self.block)
        for i in range(self.total):
            if inputs[i] is not None and outputs[i] is not None:
                raise ValueError("ErrReconstructMismatch")
        missing = [i < self.k and inputs[i] is None and outputs[i] is not None for i in range(self.total)]
        read = 0
        while True:
            size = -1
            for i, rd in enumerate(inputs):
                if rd is None:
                    all_[i].n = 0
                    continue
                n = _read_full(rd, all_[i].full(self.block))
                if size == -1 and n > 0:
                    size = n
                all_[i].n = n
            if size in (-1, 0):
                if read == 0:
                    raise ValueError("ErrShardNoData")
                return
            for i, s in enumerate(all_):
                if missing[i]:
                    continue
                cur = s.n
                if cur == 0:
                    s.n = size
                    s.buf[:size] = 0
                elif cur < size:
                    s.n = size
                    s.buf[cur:size] = 0
                elif cur > size:
                    s.n = size
            al = (size + 63) // 64 * 64 if size % 64 else size
            for i, s in enumerate(all_):
                if missing[i]:
                    continue
                if s.n > 0:
                    s.n = al
                    s.buf[size:al] = 0
            read += size
            for i in range(self.total):
                if missing[i]:
                    all_[i].n = 0
            self._rebuild(all_, False)
            for i in range(self.k):
                if outputs[i] is None:
                    continue
                outputs[i].write(bytes(all_[i].buf[:size]))


class GoStream8:
    """rsStreamFF8 (streaming8.go), single buffer, r.rs.* answered by the
    GF(2^8) oracle.  A fresh encoder per call, as every rsFF8 Stream* method
    builds one (reedsolomon.go:132,147,169): `self.orc` is replaced per call so
    the leopard8 inversion cache starts empty, as newFF8's does."""

    def __init__(self, k, p, block=4 << 20):
        self.k, self.p, self.total, self.block = k, p, k + p, block
        self.calls = []

    def _fresh(self):
        self.orc = Oracle(8, self.k, self.p)

    def _read(self, readers, dst):
        """The read loop (:246-270, :355-379, :473-497, :639-663): first
        non-empty length, -1 if none."""
        size = -1
        for i, rd in enumerate(readers):
            if rd is None:
                dst[i].reslice(0)
                continue
            n = _read_full(rd, dst[i].full(self.block))
            if size == -1 and n > 0:
                size = n
            dst[i].reslice(n)
        return size

    @staticmethod
    def _uniform(all_, size, skip=()):
        """:276-296 / :388-414 / :506-532 / :672-703"""
        for i, s in enumerate(all_):
            if i in skip:
                continue
            cur = s.n
            if cur == 0:
                s.reslice(size)
                s.buf[:size] = 0
            elif cur < size:
                if s.cap() < size:
                    s.grow_copy(size)
                else:
                    s.reslice(size)
                s.buf[cur:size] = 0
            elif cur > size:
                s.reslice(size)

    @staticmethod
    def _align(all_, size, skip=()):
        """:416-436 / :534-554 / :705-730: zero pad to a multiple of 64."""
        al = size
        if size % 64:
            al = (size + 63) // 64 * 64
            for i, s in enumerate(all_):
                if i in skip or s.n == 0:
                    continue
                if s.cap() < al:
                    s.grow_copy(al)
                else:
                    s.reslice(al)
                s.buf[size:al] = 0
        return al

    def encode(self, inputs, outputs):
        """:109-181 with readInputs :242-316 and writeOutputs :318-340."""
        self._fresh()
        shards = _alloc(self.total, self.block)
        for s in shards:
            s.reslice(self.block)
        while True:
            data = shards[:self.k]
            size = self._read(inputs, data)
            if size == -1:
                return
            self._uniform(data, size)
            if size % 64:
                padded = (size + 63) // 64 * 64
                for s in data:
                    if s.n == size:
                        s.reslice(padded)
                        s.buf[size:padded] = 0
            al = (size + 63) // 64 * 64  # :155-164
            for s in shards:
                if s.n < al:
                    s.grow_copy(al)
                s.reslice(al)
            rows = [s.view() for s in shards]
            assert self.orc.encode(rows) == 0
            self.calls.append(("encode", [bytes(r) for r in rows]))
            for j, w in enumerate(outputs):
                if w is not None:
                    w.write(bytes(shards[self.k + j].buf[:al]))

    def verify(self, readers):
        """:343-444"""
        self._fresh()
        all_ = _alloc(self.total, self.block)
        read = 0
        while True:
            size = self._read(readers, all_)
            if size in (-1, 0):
                if read == 0:
                    raise ValueError("ErrShardNoData")
                return True
            self._uniform(all_, size)
            self._align(all_, size)
            read += size
            rows = [s.view() for s in all_]
            ok, e = self.orc.verify(rows)
            assert e == 0
            self.calls.append(("verify", [bytes(r) for r in rows]))
            if not ok:
                return False

    def _rebuild(self, all_, recover_all):
        rows = [s.view() if s.n else None for s in all_]
        self.calls.append(("reconstruct", [None if r is None else bytes(r) for r in rows]))
        e, out = self.orc.reconstruct(rows, recover_all)
        assert e == 0, e
        end = self.total if recover_all else self.k
        for i in range(end):
            if rows[i] is None and out[i] is not None:
                S = len(out[i])
                all_[i].buf[:S] = out[i]  # cap >= S: leopard8.go rebuilds in place
                all_[i].n = S

    def reconstruct(self, inputs, outputs):
        """:447-606: every nil input is zero-extended with the rest (:389-393),
        so the codec sees all shards present."""
        self._fresh()
        all_ = _alloc(self.total, self.block)
        data_only = True
        for i in range(self.total):
            if inputs[i] is not None and outputs[i] is not None:
                raise ValueError("ErrReconstructMismatch")
            if i >= self.k and outputs[i] is not None:
                data_only = False
        read = 0
        while True:
            size = self._read(inputs, all_)
            if size in (-1, 0):
                if read == 0:
                    raise ValueError("ErrShardNoData")
                return
            self._uniform(all_, size)
            al = self._align(all_, size)
            read += size
            for s in all_:  # :559-573
                if s.n not in (al, 0):
                    if s.cap() < al:
                        s.grow_copy(al)
                    else:
                        s.reslice(al)
            self._rebuild(all_, not data_only)
            for i, w in enumerate(outputs):
                if w is None:
                    continue
                ws = size if i < self.k else al
                w.write(bytes(all_[i].buf[:ws]))

    def reconstruct_data(self, inputs, outputs):
        """:609-766"""
        self._fresh()
        all_ = _alloc(self.total, self.block)
        for i in range(self.total):
            if inputs[i] is not None and outputs[i] is not None:
                raise ValueError("ErrReconstructMismatch")
        missing = {i for i in range(self.k) if inputs[i] is None and outputs[i] is not None}
        read = 0
        while True:
            size = self._read(inputs, all_)
            if size in (-1, 0):
                if read == 0:
                    raise ValueError("ErrShardNoData")
                return
            self._uniform(all_, size, skip=missing)
            al = self._align(all_, size, skip=missing)
            read += size
            for i in missing:  # :734-744
                if all_[i].cap() < al:
                    all_[i] = GoSlice(np.zeros(al, np.uint8), 0)
                else:
                    all_[i].reslice(0)
            self._rebuild(all_, False)
            for i in range(self.k):
                if outputs[i] is None:
                    continue
                outputs[i].write(bytes(all_[i].buf[:size]))
