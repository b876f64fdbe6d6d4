"""Pipelined mirrors of the reference's stream codecs, with their
``r.rs.Encode / Verify / Reconstruct / ReconstructData`` calls bound to the
MI355X engine's asynchronous tickets:

* ``StreamEncoder16`` -- ``rsStream16`` (bpfs/reedsolomon16
  streaming16.go:16-71, 84-632, 1229-1318), the GF(2^16) stream codec that
  ``New16`` hands out;
* ``StreamEncoder8`` -- ``rsStreamFF8`` (streaming8.go:50-101, 109-181,
  242-340, 343-766), the GF(2^8) stream codec behind ``New`` for every
  k + p <= 256 (reedsolomon.go:77-80, 124-202).

This is the edit INTEGRATION.md describes for the Go side: the reference reads
one 4 MiB block per shard, calls the codec, writes the block out, and only then
reads the next block.  Here ``depth`` pinned block buffers rotate, so block j+1
is read (and its host->device copies run) while block j's kernels and copies
are in flight; outputs are still written in block order.

Block semantics follow the Go loops byte for byte (they decide which bytes the
codec sees, so parity and verdicts match the reference's for the same readers):

* the block size is the first non-empty shard's read (``readInputs``
  streaming16.go:84-170, streaming8.go:242-316); other shards are
  zero-extended or truncated to it;
* encode pads the block with zeros -- to an even size first in GF(2^16) --
  then to a multiple of 64, and writes ``ceil64(size)`` parity bytes
  (streaming16.go:1274-1318, :173-197; streaming8.go:155-181, :318-340);
* verify zero-pads the same way (streaming16.go:245-309, streaming8.go:388-436).
  In GF(2^16) every row reaching :295 is exactly ``size`` bytes long, so each
  one is replaced by a fresh zeroed ``make([]byte, alignedSize)`` (:297-299;
  the reslice at :301 never runs).  The parity rows' real bytes past ``size``
  are therefore replaced by zeros.  Whether the block still verifies depends
  on which bytes the pad covers: where every twiddle of the geometry lies in
  GF(2^8) (e.g. 128 + 32) a parity symbol's high byte depends only on the
  data's high bytes, so a pad inside the high half (size mod 64 >= 32) holds
  zero parity and verifies True; a pad reaching into the low half, or a
  full-field geometry, verifies False.  After a True verdict the loop's next
  ``all[i][:r.blockSize]`` (:218) slices past the new buffer's capacity
  (alignedSize < blockSize) and the reference panics; the mirror raises
  ``ErrPanic`` there.  GF(2^8) keeps the block buffer (capacity blockSize) and
  never panics; its byte columns are independent, so the zero pad verifies;
* GF(2^16) reconstruct zero-pads present shards to 64 and writes ``origSize``
  bytes of rebuilt data shards and ``ceil64(size)`` of rebuilt parity
  (streaming16.go:320-468); reconstructData (streaming16.go:471-632,
  streaming8.go:609-766) feeds a nil parity input as a zero shard;
* GF(2^8) reconstruct (streaming8.go:447-606) has no missing-shard map: its
  uniform-size loop (:389-393) zero-extends *every* nil input, the missing
  shards included, so ``r.rs.Reconstruct`` sees every shard present and does
  nothing (leopard8.go:459-462), and the loop writes zeros for every requested
  output (``size`` bytes per data shard, ``ceil64(size)`` per parity shard).
  ``StreamReconstruct`` takes this loop whenever a parity output is requested
  (reedsolomon.go:174-188); with data outputs only it takes reconstructData,
  which rebuilds.  The mirror reproduces both.

One observable difference: a pipelined verify reads block j+1 before it learns
that block j mismatched, so on a ``False`` result the readers have advanced one
block further than the reference's would have.
"""
from __future__ import annotations

from collections import deque
from typing import Optional, Sequence

import numpy as np

from .codec import (EmptyShard, New8, New16, RSError, ErrInvShardNum, ErrNilWriter, ErrPanic,
                    ErrShardNoData, ErrShortData, ErrSize, ErrTooFewShards)

BLOCK_SIZE = 4 * 1024 * 1024  # streaming16.go:48, streaming8.go:83


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


def _read_once(reader, n: int) -> bytes:
    """One io.Reader.Read of at most `n` bytes (b"" = io.EOF)."""
    return bytes(reader.read(n)) if n > 0 else b""


def stream_split(data_shards: int, data, dst: Sequence, size: int) -> None:
    """StreamSplit: rsStream16.split (streaming16.go:635-754) and
    rsStreamFF8.split (streaming8.go:769-876), which compute the same layout
    (GF(2^16)'s extra rounding to an even size is absorbed by the 64-byte one).

    Shards 0..k-2 get ``per`` bytes and the last one the remainder, each written
    zero-padded to a multiple of 64.  ``per`` is ceil64(ceil64(size) / k); when
    that leaves the last shard nothing, ``per`` becomes ceil64((size - 1) /
    (k - 1)) and the last shard at least 1 byte.  ``per`` can be 0 (k > 64 with
    a small size): the first k - 1 writers then receive empty writes and the
    last shard all the data.  A reader that ends inside the data: the partial
    shard is written padded, then the next shard's read finds end of stream and
    the call returns ErrShortData with the earlier shards already written.  A
    reader that ends after all ``size`` bytes while shards remain fills them
    with zeros of the current shard's padded length (:720-728).  Reader and
    writer errors pass through unwrapped, as in the Go code."""
    if len(dst) != data_shards:
        raise ErrTooFewShards("too few shards given")
    if size <= 0:
        raise ErrShortData("not enough data to fill the number of requested shards")
    k = data_shards
    per = _ceil64(_ceil64(size) // k)
    last = size - per * (k - 1)
    if last <= 0:  # :668-681
        per = _ceil64((size - 1) // (k - 1))
        last = size - per * (k - 1)
        if last <= 0:
            last = 1
    last_al = _ceil64(last)
    buf = np.zeros(max(per, last_al), dtype=np.uint8)
    total = 0
    for s in range(k):
        to_write, want = (last_al, last) if s == k - 1 else (per, per)
        n = _read_full(data, buf[:want])
        if n == 0 and want > 0:  # io.ReadFull's io.EOF: nothing read
            if total < size:
                raise ErrShortData("not enough data to fill the number of requested shards")
            zeros = np.zeros(to_write, dtype=np.uint8)
            for i in range(s, k):
                dst[i].write(memoryview(zeros))
            return
        total += n
        out = np.zeros(to_write, dtype=np.uint8)
        out[:n] = buf[:n]
        dst[s].write(memoryview(out))


def stream_join(data_shards: int, parity_shards: int, dst, shards: Sequence, out_size: int) -> None:
    """StreamJoin: rsStream16.join (streaming16.go:882-1196) and rsStreamFF8.join
    (streaming8.go:1003-1320, the same code): writes `out_size` bytes of the
    data shards' concatenation to `dst`.  Readers are file-like (``read``;
    None = nil); every branch of the Go code is kept, since each reads the
    shards differently:

    * ``out_size <= k``: io.ReadFull from each non-nil reader in turn (parity
      readers included) until ``out_size`` bytes are in;
    * given k + p readers, only the first k are used; fewer than k non-nil
      ones is ErrTooFewShards;
    * ``out_size < 1000``: ONE Read per non-nil shard of the bytes still
      missing (a short read is not retried: ErrShortData);
    * every reader seekable (``seek``, the io.Seeker assertion) and
      ``out_size <= 10 MiB``: each shard read up to ``per`` = ceil64(ceil(out_size
      / k)) bytes, the last slot up to what is still missing, copied through
      (joinWithMultiReader :1022-1072; bytes are written before a short result
      is reported);
    * otherwise per-shard reads of up to ``per`` bytes in 64 KiB pieces, the
      last slot's reader (or, when that slot is nil, the last non-nil one)
      read on to end of stream (joinWithBufferedReads :1074-1196)."""
    if dst is None:
        raise ErrNilWriter("the destination writer must not be nil")
    if len(shards) == 0:
        raise ErrTooFewShards("too few shards given")
    if out_size <= 0:
        raise ErrSize("invalid size")
    k = data_shards
    if out_size <= k:  # :896-923
        got = bytearray()
        for rd in shards:
            if rd is None:
                continue
            view = np.zeros(out_size - len(got), dtype=np.uint8)
            n = _read_full(rd, view)
            got += view[:n].tobytes()
            if len(got) >= out_size:
                break
        if len(got) < out_size:
            raise ErrShortData("not enough data to fill the number of requested shards")
        dst.write(bytes(got))
        return
    if len(shards) == data_shards + parity_shards:  # :927-929
        shards = shards[:k]
    if sum(rd is not None for rd in shards) < k:  # :932-941
        raise ErrTooFewShards("too few shards given")
    if out_size < 1000:  # :976-1010
        got = bytearray()
        for rd in shards:
            if rd is None:
                continue
            left = out_size - len(got)
            if left <= 0:
                break
            got += _read_once(rd, left)
            if len(got) >= out_size:
                break
        if len(got) < out_size:
            raise ErrShortData("not enough data to fill the number of requested shards")
        dst.write(bytes(got[:out_size]))
        return
    per = _ceil64(-(-out_size // k))
    if out_size <= 10 * 1024 * 1024 and all(rd is None or hasattr(rd, "seek") for rd in shards):
        limits = []
        for i, rd in enumerate(shards):  # :1036-1057
            if rd is None:
                continue
            want = per
            if i == len(shards) - 1:
                want = out_size - len(limits) * per
                if want <= 0:
                    break
            limits.append((rd, want))
        written = 0
        for rd, want in limits:
            view = np.zeros(min(want, out_size - written), dtype=np.uint8)
            n = _read_full(rd, view)
            if n:
                dst.write(view[:n].tobytes())
            written += n
            if written >= out_size:
                break
        if written < out_size:
            raise ErrShortData("not enough data to fill the number of requested shards")
        return
    piece = 64 * 1024
    written = 0
    last_i, last_rd = -1, None
    for i, rd in enumerate(shards):  # :1098-1155
        if rd is None:
            continue
        last_i, last_rd = i, rd
        if i == len(shards) - 1 and written < out_size:
            continue
        got = 0
        while got < per and written < out_size:
            want = min(piece, per - got, out_size - written)
            if want == 0:
                break
            b = _read_once(rd, want)
            if not b:
                break
            dst.write(b)
            got += len(b)
            written += len(b)
    if last_i >= 0 and written < out_size:  # :1158-1188
        while written < out_size:
            b = _read_once(last_rd, min(piece, out_size - written))
            if not b:
                break
            dst.write(b)
            written += len(b)
    if written < out_size:
        raise ErrShortData("not enough data to fill the number of requested shards")


class _StreamCodec:
    """The block loops shared by both fields; the subclasses set the field and
    the places where streaming16.go and streaming8.go differ."""

    FIELD = 16
    EVEN = True  # GF(2^16) pads an odd block to even first (streaming16.go:122-125, :274-287)

    def __init__(self, data_shards: int, parity_shards: int, device: Optional[int] = None,
                 block_size: int = BLOCK_SIZE, depth: int = 2, codec=None, threads: int = 1):
        if data_shards <= 0 or parity_shards <= 0:  # streaming16.go:36-41, streaming8.go:71-76
            raise ErrInvShardNum("invalid number of shards")
        if self.EVEN and block_size % 2:  # streaming16.go:54-56
            block_size += 1
        if block_size % 64 or depth < 1:
            raise ValueError("block_size must be a multiple of 64 and depth >= 1")
        # newFF16 / newFF8 (streaming16.go:59-63, streaming8.go:89-93); `codec`
        # substitutes an object with the same encode_async / verify_async /
        # reconstruct_async / alloc_aligned methods (the CPU tests drive the
        # block logic with one)
        if codec is None:
            codec = (New16 if self.FIELD == 16 else New8)(data_shards, parity_shards, device)
        self.rs = codec
        self.k, self.p = data_shards, parity_shards
        self.total = data_shards + parity_shards
        self.block_size = block_size
        self.depth = depth
        self._bufs = None
        # threads > 1: a block's readers are read, and its writers written,
        # on a pool of that many threads (file readers release the GIL in
        # readinto).  The bytes every reader and writer sees are the same as
        # the reference's sequential loops; what differs is only that a
        # failing reader no longer stops the reads of the readers after it
        # (the error reported is still the lowest-index one).
        self._pool = None
        if threads > 1:
            from concurrent.futures import ThreadPoolExecutor

            self._pool = ThreadPoolExecutor(max_workers=threads)

    def close(self) -> None:
        """Shut the read/write thread pool down and drop the block buffers."""
        pool, self._pool = self._pool, None
        if pool is not None:
            pool.shutdown(wait=True)
        self._bufs = None

    def _each(self, jobs, objs=None) -> None:
        """Run every job; re-raise the lowest-index job's exception.  `objs`
        are the readers / writers the jobs use: when one object appears twice
        (an aliased reader), the jobs run one after another in index order, so
        it sees its bytes in the order of the reference's sequential loop."""
        if objs is not None and len({id(o) for o in objs}) < len(objs):
            for j in jobs:
                j()
            return
        if self._pool is None or len(jobs) < 2:
            for j in jobs:
                j()
            return
        from concurrent.futures import wait

        futs = [self._pool.submit(j) for j in jobs]
        wait(futs)  # every job is done with the block buffers before anything is raised
        for f in futs:
            e = f.exception()
            if e is not None:
                raise e

    def _buffers(self):
        # AllocAligned(totalShards, blockSize) (streaming16.go:66-76,
        # streaming8.go:96-98), pinned so the queued copies run as DMA and the
        # tickets return at once
        if self._bufs is None:
            self._bufs = [self.rs.alloc_aligned(self.block_size, pinned=True) for _ in range(self.depth)]
        return self._bufs

    def _read_rows(self, readers, rows, lens) -> int:
        """The read loop every stream operation opens with: io.ReadFull of up
        to blockSize bytes per non-nil reader into its row; returns the first
        non-empty read's length (-1 if none), appends every row's length."""
        got = [0] * len(readers)

        def job(i, rd):
            def run():
                try:
                    got[i] = _read_full(rd, rows[i][:self.block_size])
                except Exception as e:
                    raise StreamReadError(e, i) from e
            return run

        self._each([job(i, rd) for i, rd in enumerate(readers) if rd is not None], [rd for rd in readers if rd is not None])
        lens.extend(got)
        return next((n for n in got if n > 0), -1)

    # ------------------------------------------------------------------ encode
    def _read_inputs(self, readers, rows) -> int:
        """readInputs (streaming16.go:84-170, streaming8.go:242-316) into
        `rows` (numpy row views of block_size bytes): returns the block size
        (made even in GF(2^16)), -1 at end of stream."""
        lens = []
        size = self._read_rows(readers, rows, lens)
        if size == -1:
            return -1
        if self.EVEN and size % 2:
            size += 1
        padded = _ceil64(size)
        for i, n in enumerate(lens):
            # short rows are zero-extended to size, long ones truncated to it,
            # and every row is zero-padded from size to the 64-byte pad
            rows[i][min(n, size):padded] = 0
        return size

    def encode(self, inputs: Sequence, outputs: Sequence) -> None:
        """rsStream16.encode (streaming16.go:1229-1318) / rsStreamFF8.encode
        (streaming8.go:109-181)."""
        if len(inputs) != self.k or len(outputs) != self.p:
            raise ErrTooFewShards("too few shards given")
        bufs = self._buffers()
        pending = deque()  # (ticket, buffer set, size)

        def drain_one():
            t, rows, size = pending.popleft()
            t.wait()
            al = _ceil64(size)  # writeOutputs (streaming16.go:173-197, streaming8.go:318-340)
            self._each([(lambda w=w, j=j: _write(w, rows[self.k + j][:al], self.k + j))
                        for j, w in enumerate(outputs) if w is not None], [w for w in outputs if w is not None])

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
        """rsStream16.verify (streaming16.go:200-317) / rsStreamFF8.verify
        (streaming8.go:343-444)."""
        if len(shards) != self.total:
            raise ErrTooFewShards("too few shards given")
        bufs = self._buffers()
        pending = deque()
        verdict = [True]

        def drain_one():
            t = pending.popleft()
            if not t.result():
                verdict[0] = False

        def settle() -> bool:
            # the reference returns an earlier block's mismatch before anything later
            while pending and verdict[0]:
                drain_one()
            return verdict[0]

        blk, read = 0, 0
        try:
            while verdict[0]:
                if len(pending) == self.depth:
                    drain_one()
                    if not verdict[0]:
                        break
                rows = bufs[blk % self.depth]
                lens = []
                try:
                    size = self._read_rows(shards, rows, lens)
                except StreamReadError:
                    if not settle():
                        return False
                    raise
                if size <= 0:
                    if not settle():
                        return False
                    if read == 0:
                        raise ErrShardNoData("no shard data")
                    return True
                for i, n in enumerate(lens):  # zero-extend short rows, truncate long ones
                    if n < size:
                        rows[i][n:size] = 0
                if self.EVEN and size % 2:  # pad to even with a zero (streaming16.go:274-287)
                    for r in rows:
                        r[size] = 0
                    size += 1
                al = _ceil64(size)
                for r in rows:  # zero pad to 64 (streaming16.go:297-305, streaming8.go:420-434)
                    r[size:al] = 0
                read += size
                pending.append(self.rs.verify_async([r[:al] for r in rows]))
                blk += 1
                if self.EVEN and size < al < self.block_size:
                    # every row is now a zeroed buffer of capacity alignedSize
                    # (streaming16.go:297): a True verdict sends the reference
                    # into all[i][:r.blockSize] (:218), which panics
                    if not settle():
                        return False
                    raise ErrPanic("streaming16.go:218: slice bounds out of range [:%d] with capacity %d "
                                   "(the verify loop continues past a block of %d bytes)"
                                   % (self.block_size, al, size))
            return False
        finally:
            while pending:
                pending.popleft().wait()

    # ------------------------------------------------------------------ reconstruct
    def _check_io(self, inputs, outputs) -> None:
        if len(inputs) != self.total or len(outputs) != self.total:
            raise ErrTooFewShards("too few shards given")
        for i in range(self.total):
            if inputs[i] is not None and outputs[i] is not None:
                raise ErrReconstructMismatch("a shard cannot be both an input and an output")

    # ------------------------------------------------------------------ split / join
    def split(self, data, dst: Sequence, size: int) -> None:
        """StreamSplit (reedsolomon.go:204-215, :312-323): see stream_split."""
        stream_split(self.k, data, dst, size)

    def join(self, dst, shards: Sequence, out_size: int) -> None:
        """StreamJoin (reedsolomon.go:217-228, :325-336): see stream_join."""
        stream_join(self.k, self.p, dst, shards, out_size)

    def _fresh_codec(self) -> None:
        """Every rsFF8 Stream* call builds its own rsStreamFF8 and newFF8
        (reedsolomon.go:132,147,169), whose inversion cache starts empty
        (leopard8.go:67-71): clear the engine's before each stream operation."""
        reset = getattr(self.rs, "reset_inversion_cache", None)
        if self.FIELD == 8 and reset is not None:
            reset()

    def reconstruct_data(self, inputs: Sequence, outputs: Sequence) -> None:
        """rsStream16.reconstructData (streaming16.go:471-632) /
        rsStreamFF8.reconstructData (streaming8.go:609-766): rebuilds only
        missing data shards; a nil parity input is fed as a zero shard."""
        self._check_io(inputs, outputs)
        self._fresh_codec()
        missing = [i < self.k and inputs[i] is None and outputs[i] is not None for i in range(self.total)]
        self._reconstruct_loop(inputs, outputs, missing, recover_all=False, data_loop=True)

    def _reconstruct_loop(self, inputs, outputs, missing, recover_all: bool, data_loop: bool) -> None:
        bufs = self._buffers()
        pending = deque()  # (ticket, shards list, size, aligned)

        def drain_one():
            t, blk_shards, size, al = pending.popleft()
            t.wait()
            jobs, objs = [], []
            for i, w in enumerate(outputs):
                if w is None or not missing[i]:
                    continue
                if data_loop:
                    if i >= self.k:
                        continue
                    ws = size  # streaming16.go:618-630, streaming8.go:752-764
                else:
                    ws = size if i < self.k else al  # streaming16.go:445-464
                jobs.append(lambda w=w, i=i, ws=ws: _write(w, np.asarray(blk_shards[i])[:ws], i))
                objs.append(w)
            self._each(jobs, objs)

        blk, read = 0, 0
        try:
            while True:
                if len(pending) == self.depth:
                    drain_one()
                rows = bufs[blk % self.depth]
                lens = []
                size = self._read_rows(inputs, rows, lens)
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


class StreamEncoder16(_StreamCodec):
    """rsStream16 (streaming16.go:16-71) over the MI355X engine.

    ``encode(inputs, outputs)``, ``verify(shards)``, ``reconstruct(inputs,
    outputs)`` and ``reconstruct_data(inputs, outputs)`` take file-like readers
    (``readinto`` or ``read``; None = a nil reader) and writers (``write``;
    None = nil), like the Go io.Reader / io.Writer slices."""

    FIELD = 16
    EVEN = True

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


class StreamEncoder8(_StreamCodec):
    """rsStreamFF8 (streaming8.go:50-101) over the MI355X engine: the stream
    codec ``New`` selects for k + p <= 256.  Same methods as StreamEncoder16."""

    FIELD = 8
    EVEN = False

    def reconstruct(self, inputs: Sequence, outputs: Sequence) -> None:
        """rsStreamFF8.reconstruct (streaming8.go:447-606).  Every nil input,
        the requested outputs included, becomes a zero row of the block size
        (:389-393, :507-532), so ``r.rs.Reconstruct`` finds every shard
        present and returns at once (leopard8.go:459-462): each requested
        output receives zeros, ``size`` bytes per data shard and
        ``ceil64(size)`` per parity shard (:586-604)."""
        self._check_io(inputs, outputs)
        self._fresh_codec()
        recover_all = any(outputs[i] is not None for i in range(self.k, self.total))  # :459-467
        bufs = self._buffers()
        blk, read = 0, 0
        while True:
            rows = bufs[blk % self.depth]
            lens = []
            size = self._read_rows(inputs, rows, lens)
            if size <= 0:
                if read == 0:
                    raise ErrShardNoData("no shard data")
                return
            al = _ceil64(size)
            for i, n in enumerate(lens):
                rows[i][min(n, size):al] = 0
            t = self.rs.reconstruct_async([r[:al] for r in rows], recover_all)  # all present: a no-op
            t.wait()
            read += size
            self._each([(lambda w=w, i=i: _write(w, rows[i][:size if i < self.k else al], i))
                        for i, w in enumerate(outputs) if w is not None], [w for w in outputs if w is not None])
            blk += 1
