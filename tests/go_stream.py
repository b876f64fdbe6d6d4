"""Test helper: a line-by-line, single-buffer, synchronous restatement of the
reference's rsStream16 loops (streaming16.go:84-170 readInputs, :173-197
writeOutputs, :200-317 verify, :320-468 reconstruct, :471-632 reconstructData,
:1229-1318 encode), with r.rs.* calls answered by the oracle.  It is the
checker for reedsolomon16_amd/stream.py (the pipelined product mirror): both
must hand the codec the same bytes and write the same outputs.

Go slices are modelled as (buffer, length) with the buffer's capacity fixed,
so re-slicing exposes whatever the buffer held -- the property the verify
loop's padding depends on.
"""
from __future__ import annotations

import numpy as np

from oracle.orc import Oracle


class GoSlice:
    __slots__ = ("buf", "n")

    def __init__(self, buf, n):
        self.buf, self.n = buf, n

    def view(self):
        return self.buf[:self.n]


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
            n = _read_full(rd, dst[i].buf[:self.block])
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
        all_ = _alloc(self.total, self.block)
        read = 0
        while True:
            size = -1
            for i, rd in enumerate(readers):
                if rd is None:
                    all_[i].n = 0
                    continue
                n = _read_full(rd, all_[i].buf[:self.block])
                if size == -1 and n > 0:
                    size = n
                all_[i].n = n
            if size in (-1, 0):
                if read == 0:
                    raise ValueError("ErrShardNoData")
                return True
            for s in all_:
                cur = s.n
                if cur == 0:
                    s.n = size
                    s.buf[:size] = 0
                elif cur < size:
                    s.n = size
                    s.buf[cur:size] = 0
                elif cur > size:
                    s.n = size
            if size % 2:
                ps = size + 1
                for s in all_:
                    if s.n == size:
                        s.n = ps
                        s.buf[size:ps] = 0
                size = ps
            al = size
            if size % 64:
                al = (size + 63) // 64 * 64
                for s in all_:
                    if s.n > 0:
                        s.n = al  # streaming16.go:301; the fill loop below it starts at len == al
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
                n = _read_full(rd, all_[i].buf[:self.block])
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
                n = _read_full(rd, all_[i].buf[:self.block])
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
