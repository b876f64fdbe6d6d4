"""Pipelined mirror of the reference's GF(2^16) stream codec ``rsStream16``
(bpfs/reedsolomon16 streaming16.go:16-71, 200-632, 1229-1318), with its
``r.rs.Encode / Verify / Reconstruct / ReconstructData`` calls bound to the
MI355X engine's asynchronous tickets.

This is the edit INTEGRATION.md describes for the Go side: the reference reads
one 4 MiB block per shard, calls the codec, writes the block out, and only then
reads the next block.  Here ``depth`` pinned block buffers rotate, so block j+1
is read (and its host->device copies run) while block j's kernels and copies
are in flight; outputs are still written in block order.

Block semantics follow the Go loops byte for byte (they decide which bytes the
codec sees, so parity and verdicts match the reference's for the same readers):

* the block size is the first non-empty shard's read (``readInputs``
  streaming16.go:84-170); other shards are zero-extended or truncated to it;
* encode pads the block to an even size and then to a multiple of 64 with
  zeros and writes ``ceil64(size)`` parity bytes (:1274-1318, :173-197);
* verify pads to even with zeros, then to 64 *without* zero-filling: its fill
  loop starts at ``len(all[i])`` after the reslice (:304-306), so those bytes
  are whatever the single Go block buffer last held there.  The mirror
  reproduces that content (``_GoBufferHistory``);
* reconstruct zero-pads present shards to 64 and writes ``origSize`` bytes of
  rebuilt data shards and ``ceil64(size)`` of rebuilt parity (:320-468);
  reconstructData (:471-632) feeds a nil parity input as a zero shard.

One observable difference: a pipelined verify reads block j+1 before it learns
that block j mismatched, so on a ``False`` result the readers have advanced one
block further than the reference's would have.
"""
from __future__ import annotations

from collections import deque
from typing import List, Optional, Sequence

import numpy as np

from .codec import EmptyShard, New16, RSError, ErrInvShardNum, ErrShardNoData, ErrTooFewShards

BLOCK_SIZE = 4 * 1024 * 1024  # streaming16.go:48


class ErrReconstructMismatch(RSError):
    """reedsolomon.go:30: a shard cannot be both an input and an output."""


class StreamReadError(RSError):
    """streaming8.go:24-31: error reading stream `stream`."""

    def __init__(self, err, stream: int):
        super().__init__("error reading stream %d: %r" % (stream, err))
        self.err, self.stream = err, stream


class StreamWriteError(RSError):
    """streaming8.go:34-41: error writing stream `stream`."""

    def __init__(self, err, stream: int):
        super().__init__("error writing to stream %d: %r" % (stream, err))
        self.err, self.stream = err, stream


def _ceil64(n: int) -> int:
    return (n + 63) // 64 * 64


def _read_full(reader, view: np.ndarray) -> int:
    """io.ReadFull into `view`: bytes read (< len(view) only at end of stream)."""
    want = len(view)
    n = 0
    readinto = getattr(reader, "readinto", None)
    mv = memoryview(view)
    while n < want:
        if readinto is not None:
            got = readinto(mv[n:])
            if not got:
                break
            n += got
        else:
            b = reader.read(want - n)
            if not b:
                break
            view[n:n + len(b)] = np.frombuffer(b, dtype=np.uint8)
            n += len(b)
    return n


def _write(writer, buf: np.ndarray, stream: int) -> None:
    try:
        n = writer.write(memoryview(buf))
    except Exception as e:  # the writer's own error, wrapped like the reference
        raise StreamWriteError(e, stream) from e
    if n is not None and n != len(buf):
        raise StreamWriteError("short write", stream)


class _GoBufferHistory:
    """What the reference's single block buffer holds past a row's current
    write extent.  Row i's buffer byte x is the byte the latest block that wrote
    x put there (ReadFull writes [0, n); zero padding writes up to the padded
    size), or 0 if no block did (AllocAligned zeroes it).  The mirror keeps
    `depth` buffers, so a byte last written by a block held in another buffer
    is copied over when a verify block reads it (streaming16.go:290-309)."""

    def __init__(self, total: int):
        self.ext: List[List[int]] = [[] for _ in range(total)]  # per row: write extent of each block

    def record(self, extents: Sequence[int]) -> None:
        for i, e in enumerate(extents):
            self.ext[i].append(e)

    def fill(self, blk: int, bufs, lo: int, hi: int) -> None:
        """Give bytes [lo, hi) of every row of block `blk` (already recorded)
        the reference buffer's content."""
        depth = len(bufs)
        cur = bufs[blk % depth]
        for i, ext in enumerate(self.ext):
            for x in range(lo, hi):
                t = blk
                while t >= 0 and x >= ext[t]:
                    t -= 1
                if t < 0:
                    cur[i][x] = 0
                elif t % depth != blk % depth:
                    cur[i][x] = bufs[t % depth][i][x]
                # else: the byte is still in this buffer from block t


class StreamEncoder16:
    """rsStream16 (streaming16.go:16-71) over the MI355X engine.

    ``encode(inputs, outputs)``, ``verify(shards)``, ``reconstruct(inputs,
    outputs)`` and ``reconstruct_data(inputs, outputs)`` take file-like readers
    (``readinto`` or ``read``; None = a nil reader) and writers (``write``;
    None = nil), like the Go io.Reader / io.Writer slices."""

    def __init__(self, data_shards: int, parity_shards: int, device: Optional[int] = None,
                 block_size: int = BLOCK_SIZE, depth: int = 2, codec=None):
        if data_shards <= 0 or parity_shards <= 0:  # streaming16.go:36-41
            raise ErrInvShardNum("invalid number of shards")
        if block_size % 2:  # streaming16.go:54-56
            block_size += 1
        if block_size % 64 or depth < 1:
            raise ValueError("block_size must be a multiple of 64 and depth >= 1")
        # newFF16 (streaming16.go:59-63); `codec` substitutes an object with the
        # same encode_async / verify_async / reconstruct_async / alloc_aligned
        # methods (the CPU tests drive the block logic with one)
        self.rs = codec if codec is not None else New16(data_shards, parity_shards, device)
        self.k, self.p = data_shards, parity_shards
        self.total = data_shards + parity_shards
        self.block_size = block_size
        self.depth = depth
        self._bufs = None

    def _buffers(self):
        # AllocAligned(totalShards, blockSize) (streaming16.go:66-76), pinned so
        # the queued copies run as DMA and the tickets return at once
        if self._bufs is None:
            self._bufs = [self.rs.alloc_aligned(self.block_size, pinned=True) for _ in range(self.depth)]
        return self._bufs

    # ------------------------------------------------------------------ encode
    def _read_inputs(self, readers, rows) -> int:
        """readInputs (streaming16.go:84-170) into `rows` (numpy row views of
        block_size bytes): returns the (even) block size, -1 at end of stream."""
        size = -1
        lens = []
        for i, rd in enumerate(readers):
            if rd is None:
                lens.append(0)
                continue
            try:
                n = _read_full(rd, rows[i][:self.block_size])
            except Exception as e:
                raise StreamReadError(e, i) from e
            if n > 0 and size == -1:
                size = n
            lens.append(n)
        if size == -1:
            return -1
        if size % 2:
            size += 1
        padded = _ceil64(size)
        for i, n in enumerate(lens):
            # short rows are zero-extended to size, long ones truncated to it,
            # and every row is zero-padded from size to the 64-byte pad
            rows[i][min(n, size):padded] = 0
        return size

    def encode(self, inputs: Sequence, outputs: Sequence) -> None:
        """rsStream16.encode (streaming16.go:1229-1318)."""
        if len(inputs) != self.k or len(outputs) != self.p:
            raise ErrTooFewShards("too few shards given")
        bufs = self._buffers()
        pending = deque()  # (ticket, buffer set, size)

        def drain_one():
            t, rows, size = pending.popleft()
            t.wait()
            al = _ceil64(size)  # writeOutputs (streaming16.go:173-197)
            for j, w in enumerate(outputs):
                if w is not None:
                    _write(w, rows[self.k + j][:al], self.k + j)

        blk = 0
        try:
            while True:
                if len(pending) == self.depth:
                    drain_one()
                rows = bufs[blk % self.depth]
                size = self._read_inputs(inputs, rows)
                if size < 0:
                    break
                al = _ceil64(size)
                pending.append((self.rs.encode_async([r[:al] for r in rows]), rows, size))
                blk += 1
        finally:
            # earlier blocks are written before an error surfaces, as the
            # reference wrote them before reading the failing block
            while pending:
                drain_one()

    # ------------------------------------------------------------------ verify
    def verify(self, shards: Sequence) -> bool:
        """rsStream16.verify (streaming16.go:200-317)."""
        if len(shards) != self.total:
            raise ErrTooFewShards("too few shards given")
        bufs = self._buffers()
        hist = _GoBufferHistory(self.total)
        pending = deque()
        verdict = [True]

        def drain_one():
            t = pending.popleft()
            if not t.result():
                verdict[0] = False

        blk, read = 0, 0
        try:
            while verdict[0]:
                if len(pending) == self.depth:
                    drain_one()
                    if not verdict[0]:
                        break
                rows = bufs[blk % self.depth]
                size, lens = -1, []
                for i, rd in enumerate(shards):
                    if rd is None:
                        lens.append(0)
                        continue
                    try:
                        n = _read_full(rd, rows[i][:self.block_size])
                    except Exception as e:
                        while pending and verdict[0]:  # the reference returns an earlier mismatch first
                            drain_one()
                        if not verdict[0]:
                            return False
                        raise StreamReadError(e, i) from e
                    if size == -1 and n > 0:
                        size = n
                    lens.append(n)
                if size <= 0:
                    while pending and verdict[0]:
                        drain_one()
                    if not verdict[0]:
                        return False
                    if read == 0:
                        raise ErrShardNoData("no shard data")
                    return True
                for i, n in enumerate(lens):  # zero-extend short rows (:245-270)
                    if n < size:
                        rows[i][n:size] = 0
                if size % 2:  # pad to even with a zero (:274-287)
                    rows_pad = size + 1
                    for r in rows:
                        r[size] = 0
                    size = rows_pad
                hist.record([max(n, size) for n in lens])
                al = _ceil64(size)
                if al > size:  # the 64-byte pad keeps the buffer's old bytes (:290-309)
                    hist.fill(blk, bufs, size, al)
                read += size
                pending.append(self.rs.verify_async([r[:al] for r in rows]))
                blk += 1
            return False
        finally:
            while pending:
                pending.popleft().wait()

    # ------------------------------------------------------------------ reconstruct
    def reconstruct(self, inputs: Sequence, outputs: Sequence) -> None:
        """rsStream16.reconstruct (streaming16.go:320-468)."""
        if len(inputs) != self.total or len(outputs) != self.total:
            raise ErrTooFewShards("too few shards given")
        data_only = True
        for i in range(self.total):
            if inputs[i] is not None and outputs[i] is not None:
                raise ErrReconstructMismatch("a shard cannot be both an input and an output")
            if i >= self.k and outputs[i] is not None:
                data_only = False
        missing = [inputs[i] is None and outputs[i] is not None for i in range(self.total)]
        if not any(missing):
            return
        self._reconstruct_loop(inputs, outputs, missing, recover_all=not data_only, data_loop=False)

    def reconstruct_data(self, inputs: Sequence, outputs: Sequence) -> None:
        """rsStream16.reconstructData (streaming16.go:471-632): rebuilds only
        missing data shards; a nil parity input is fed as a zero shard."""
        if len(inputs) != self.total or len(outputs) != self.total:
            raise ErrTooFewShards("too few shards given")
        for i in range(self.total):
            if inputs[i] is not None and outputs[i] is not None:
                raise ErrReconstructMismatch("a shard cannot be both an input and an output")
        missing = [i < self.k and inputs[i] is None and outputs[i] is not None for i in range(self.total)]
        self._reconstruct_loop(inputs, outputs, missing, recover_all=False, data_loop=True)

    def _reconstruct_loop(self, inputs, outputs, missing, recover_all: bool, data_loop: bool) -> None:
        bufs = self._buffers()
        pending = deque()  # (ticket, shards list, size, aligned)

        def drain_one():
            t, blk_shards, size, al = pending.popleft()
            t.wait()
            for i, w in enumerate(outputs):
                if w is None or not missing[i]:
                    continue
                if data_loop:
                    if i >= self.k:
                        continue
                    ws = size  # streaming16.go:618-630
                else:
                    ws = size if i < self.k else al  # streaming16.go:445-464
                _write(w, np.asarray(blk_shards[i])[:ws], i)

        blk, read = 0, 0
        try:
            while True:
                if len(pending) == self.depth:
                    drain_one()
                rows = bufs[blk % self.depth]
                size, lens = (-1 if data_loop else 0), []
                for i, rd in enumerate(inputs):
                    if rd is None:
                        lens.append(0)
                        continue
                    try:
                        n = _read_full(rd, rows[i][:self.block_size])
                    except Exception as e:
                        raise StreamReadError(e, i) from e
                    if n > 0 and size <= 0:
                        size = n
                    lens.append(n)
                if size <= 0:
                    if read == 0:
                        raise ErrShardNoData("no shard data")
                    return
                al = _ceil64(size)
                shards = []
                for i in range(self.total):
                    if missing[i]:
                        shards.append(EmptyShard(rows[i]))  # all[i][:0], cap blockSize: rebuilt in place
                        continue
                    n = lens[i]
                    if data_loop:
                        # to size (short rows, nil parity included, zero-extended;
                        # long ones truncated), then zeros from size to 64 (:534-596)
                        rows[i][min(n, size):al] = 0
                    else:
                        if n == 0:  # a nil input with a nil output (:410-412)
                            raise ErrShardNoData("no shard data")
                        if n < al:
                            rows[i][n:al] = 0
                    shards.append(rows[i][:al])
                t = self.rs.reconstruct_async(shards, recover_all)
                pending.append((t, shards, size, al))
                read += size
                blk += 1
        finally:
            while pending:
                drain_one()
