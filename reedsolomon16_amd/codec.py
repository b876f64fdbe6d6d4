"""Python mirror of the reference's ``ReedSolomon`` codec interface for the hot
path (bpfs/reedsolomon16 reedsolomon.go:37-93, leopard16.go:36-387,
leopard8.go:53-436), running on the MI355X engine through the C-ABI.

Names, argument meaning and error behaviour follow the Go API:

* ``New(k, p)`` picks GF(2^8) when k+p <= 256, else GF(2^16) (reedsolomon.go:69-81);
  ``New8`` / ``New16`` force the field.
* ``encode(shards)`` fills ``shards[k:]`` in place; ``verify`` returns bool;
  ``reconstruct`` / ``reconstruct_data`` / ``reconstruct_some`` replace missing
  entries (``None`` or empty) with rebuilt arrays, like the Go slice resize.
* Errors raise the sentinel exception classes below (``ErrTooFewShards`` ...).

Host shards are numpy ``uint8`` arrays.  Device-resident variants take torch
CUDA tensors (one per shard, or a 2-D ``[k+p, S]`` tensor) and run on the
current torch stream.
"""
from __future__ import annotations

import contextlib
import ctypes as C
import io
import sys
import threading
from typing import Optional, Sequence

import numpy as np

from . import _capi


# --------------------------------------------------------------------------- errors
class RSError(Exception):
    code = -1


def _mk(name: str, code: int, doc: str):
    cls = type(name, (RSError,), {"code": code, "__doc__": doc})
    globals()[name] = cls
    return cls


_ERRORS = {
    1: _mk("ErrInvShardNum", 1, "reedsolomon.go:16"),
    2: _mk("ErrMaxShardNum", 2, "reedsolomon.go:17"),
    3: _mk("ErrTooFewShards", 3, "reedsolomon.go:18"),
    4: _mk("ErrShardNoData", 4, "reedsolomon.go:19"),
    5: _mk("ErrShardSize", 5, "reedsolomon.go:20"),
    6: _mk("ErrInvalidShardSize", 6, "reedsolomon.go:26"),
    7: _mk("ErrNotSupported", 7, "reedsolomon.go:28"),
    8: _mk("ErrShortData", 8, "reedsolomon.go:27"),
    9: _mk("ErrReconstructRequired", 9, "reedsolomon.go:25"),
    # host-side only (StreamJoin, stream.py); the C-ABI never returns these
    10: _mk("ErrNilWriter", 10, "reedsolomon.go:31"),
    11: _mk("ErrSize", 11, "reedsolomon.go:32"),
    50: _mk("ErrPanic", 50, "the Go reference panics (index out of range) for this geometry"),
    51: _mk("ErrNoMem", 51, "allocation failed"),
    52: _mk("ErrDevice", 52, "HIP device error"),
    53: _mk("ErrInvalidArg", 53, "invalid argument"),
}
ErrInvShardNum = _ERRORS[1]
ErrMaxShardNum = _ERRORS[2]
ErrTooFewShards = _ERRORS[3]
ErrShardNoData = _ERRORS[4]
ErrShardSize = _ERRORS[5]
ErrInvalidShardSize = _ERRORS[6]
ErrNotSupported = _ERRORS[7]
ErrShortData = _ERRORS[8]
ErrReconstructRequired = _ERRORS[9]
ErrNilWriter = _ERRORS[10]
ErrSize = _ERRORS[11]
ErrPanic = _ERRORS[50]
ErrDevice = _ERRORS[52]


def _check(code: int) -> None:
    if code != 0:
        cls = _ERRORS.get(code, RSError)
        raise cls(_capi.lib().rs_strerror(code).decode())


# --------------------------------------------------------------------------- helpers
class _PinnedBlock:
    """Owner of one rs_host_alloc block; freed when the last view dies."""

    def __init__(self, nbytes: int):
        self.ptr = None
        L = _capi.lib()
        p = C.c_void_p()
        _check(L.rs_host_alloc(nbytes, C.byref(p)))
        self.ptr, self._free = p.value, L.rs_host_free

    def __del__(self):
        if self.ptr:
            self._free(self.ptr)
            self.ptr = None


def alloc_pinned(nbytes: int) -> np.ndarray:
    """Page-locked, 64-byte-aligned host bytes (zeroed) as a numpy uint8 array."""
    blk = _PinnedBlock(nbytes)
    cbuf = (C.c_uint8 * nbytes).from_address(blk.ptr)
    cbuf._owner = blk  # the ctypes buffer keeps the block alive; numpy keeps the buffer
    a = np.frombuffer(cbuf, dtype=np.uint8)
    a[:] = 0
    return a


class _PinnedArena:
    """Sub-allocates pinned rows from 64 MiB rs_host_alloc blocks, so a
    reconstruct ticket's fresh output rows do not each pay for a page-locking
    allocation.  A block is freed when the last row cut from it is gone."""

    BLOCK = 64 << 20

    def __init__(self):
        self._cur, self._off = None, 0
        self._lock = threading.Lock()  # tickets may be queued from several threads

    def take(self, nbytes: int) -> np.ndarray:
        need = (nbytes + 63) // 64 * 64
        if nbytes > self.BLOCK // 4:
            return alloc_pinned(nbytes)
        with self._lock:
            if self._cur is None or self._off + need > len(self._cur):
                self._cur, self._off = alloc_pinned(self.BLOCK), 0
            row = self._cur[self._off:self._off + nbytes]
            self._off += need
        return row


class EmptyShard:
    """A missing shard that keeps its memory, like Go's ``shards[i][:0]``:
    length 0 (so Reconstruct treats it as missing) and capacity ``len(buf)``.
    When the capacity holds the shard size, Reconstruct writes the rebuilt
    shard into ``buf`` (leopard16.go:556-560, ``shards[i][0:shardSize]``) --
    e.g. straight into an alloc_aligned(pinned=True) row -- instead of
    allocating a new array."""

    __slots__ = ("buf",)

    def __init__(self, buf):
        self.buf = buf

    def __len__(self) -> int:
        return 0


def _capacity_view(s, S: int):
    """Go's cap() check for a missing shard: the EmptyShard's buffer, if it is
    a C-contiguous uint8 array of at least S bytes; None otherwise."""
    if not isinstance(s, EmptyShard):
        return None
    b = s.buf
    if not isinstance(b, np.ndarray) or b.dtype != np.uint8 or not b.flags["C_CONTIGUOUS"] or b.nbytes < S:
        return None
    return b.reshape(-1)[:S]


def _host_rows(shards: Sequence):
    n = len(shards)
    ptrs = (C.c_void_p * n)()
    lens = (C.c_size_t * n)()
    keep = []
    for i, s in enumerate(shards):
        if s is None or len(s) == 0:
            ptrs[i] = None
            lens[i] = 0
            continue
        a = np.asarray(s)
        if a.dtype != np.uint8 or not a.flags["C_CONTIGUOUS"]:
            raise TypeError("host shards must be C-contiguous numpy uint8 arrays")
        keep.append(a)
        ptrs[i] = a.ctypes.data
        lens[i] = a.nbytes
    return ptrs, lens, keep


def _dev_rows(rows, total: int):
    """torch CUDA tensors -> (ptr array, shard size).  A 2-D [total, S] tensor
    (rows contiguous) is turned into row pointers arithmetically: no per-row
    tensor objects on the host path."""
    if hasattr(rows, "dim") and rows.dim() == 2:
        if rows.shape[0] != total:
            raise ErrTooFewShards("need %d shards, got %d" % (total, rows.shape[0]))
        if not rows.is_cuda or rows.dtype.itemsize != 1 or rows.stride(1) != 1:
            raise TypeError("device shards must be a uint8 CUDA tensor with contiguous rows")
        base, stride = rows.data_ptr(), rows.stride(0)
        return (C.c_void_p * total)(*range(base, base + total * stride, stride)), rows.shape[1]
    if len(rows) != total:
        raise ErrTooFewShards("need %d shards, got %d" % (total, len(rows)))
    ptrs = (C.c_void_p * total)()
    S = None
    for i, t in enumerate(rows):
        if t is None:
            ptrs[i] = None
            continue
        if not t.is_cuda or t.dtype.itemsize != 1 or not t.is_contiguous():
            raise TypeError("device shards must be contiguous uint8 CUDA tensors")
        ptrs[i] = t.data_ptr()
        S = t.numel() if S is None else S
    return ptrs, S or 0


RS_NULL_STREAM = C.c_void_p(-1).value  # include/rs_mi355x.h: HIP's null stream, asynchronous


def _stream_handle(stream):
    """torch stream (default: the current one) -> the C-ABI stream argument.
    torch's default stream has handle 0, which the C-ABI reads as "the codec's
    own stream, synchronous": pass it as RS_NULL_STREAM so calls on it stay
    asynchronous and ordered with torch's work."""
    if stream is None:
        import torch

        stream = torch.cuda.current_stream()
    h = getattr(stream, "cuda_stream", stream)
    return RS_NULL_STREAM if h in (0, None) and stream is not None and hasattr(stream, "cuda_stream") else h


# --------------------------------------------------------------------------- codec
class ReedSolomon:
    """One encoder instance (leopardFF16 / leopardFF8 behind the ReedSolomon interface)."""

    def __init__(self, data_shards: int, parity_shards: int, field_bits: int = 0, device: Optional[int] = None,
                 devices: Optional[Sequence[int]] = None):
        """devices: a list of device ordinals (repeats allowed) makes one
        multi-device codec (rs_new_multi): the host-memory operations split
        every shard by 64-byte byte ranges over them (include/rs_mi355x.h)."""
        L = _capi.lib()
        if devices is not None:
            devs = [int(d) for d in devices]
            if not devs:
                raise ValueError("devices must name at least one device")
            device = devs[0]
        if device is None:
            device = 0
            # follow torch's current device only when the caller already uses
            # torch: importing it here, after this library has loaded the HIP
            # runtime, made the first pinned allocation of a torch-free process fail
            torch = sys.modules.get("torch")
            if torch is not None and torch.cuda.is_available():
                device = torch.cuda.current_device()
        h = C.c_void_p()
        if devices is not None:
            arr = (C.c_int * len(devs))(*devs)
            _check(L.rs_new_multi(field_bits, data_shards, parity_shards, arr, len(devs), C.byref(h)))
        else:
            _check(L.rs_new(field_bits, data_shards, parity_shards, device, C.byref(h)))
        self._h = h
        self._L = L
        self.device = device
        self.devices = list(devs) if devices is not None else [device]
        self._arena = _PinnedArena()
        self._ref_inv = True  # rs_set_reference_inversion_cache default
        self._streamer = None
        self._stream_lock = threading.Lock()

    def close(self):
        st, self._streamer = getattr(self, "_streamer", None), None
        if st is not None:
            st.close()
            if st.rs is not self:
                st.rs.close()
        if getattr(self, "_h", None):
            if not getattr(self, "_borrowed", False):  # a part() belongs to its multi-device codec
                self._L.rs_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # Extensions (reedsolomon.go:358-375)
    def data_shards(self) -> int:
        return self._L.rs_data_shards(self._h)

    def parity_shards(self) -> int:
        return self._L.rs_parity_shards(self._h)

    def total_shards(self) -> int:
        return self._L.rs_total_shards(self._h)

    def with_concurrency(self, n: int) -> "ReedSolomon":
        """WithConcurrency (reedsolomon.go:415-427): the reference's rsFF8 and
        rsFF16 return themselves unchanged; so does the engine (its concurrency
        is the GPU's)."""
        return self

    def shard_size_multiple(self) -> int:
        return self._L.rs_shard_size_multiple(self._h)

    @property
    def field_bits(self) -> int:
        return self._L.rs_field_bits(self._h)

    @property
    def device_count(self) -> int:
        """Devices the codec splits its host-memory calls over (rs_device_count)."""
        return self._L.rs_device_count(self._h)

    def part(self, index: int) -> "ReedSolomon":
        """Device `index`'s own codec (rs_device_part): the codec itself on
        one device.  For device-resident calls on that device's byte range
        (byte_range) of rows in its HBM.  Owned by this codec: valid while it
        is open, never freed on its own."""
        h, dev = C.c_void_p(), C.c_int(0)
        _check(self._L.rs_device_part(self._h, index, C.byref(h), C.byref(dev)))
        if h.value == self._h.value:
            return self
        q = ReedSolomon.__new__(ReedSolomon)
        q._h, q._L, q.device, q.devices = h, self._L, dev.value, [dev.value]
        q._arena, q._ref_inv, q._streamer, q._stream_lock = _PinnedArena(), False, None, threading.Lock()
        q._borrowed, q._owner = True, self
        return q

    def byte_range(self, shard_size: int, index: int):
        """[lo, hi) of the shard bytes device `index` of this codec owns (rs_byte_range)."""
        lo, hi = C.c_size_t(0), C.c_size_t(0)
        _check(self._L.rs_byte_range(shard_size, index, self.device_count, C.byref(lo), C.byref(hi)))
        return lo.value, hi.value

    @property
    def encode_path(self) -> str:
        return self._L.rs_encode_path(self._h).decode()

    def alloc_aligned(self, each: int, shards: Optional[int] = None, pinned: bool = False):
        """AllocAligned (unsafe.go:17-41): one 64-byte-aligned slab, rows of `each` bytes.
        pinned=True allocates page-locked memory (rs_host_alloc) so the host
        pipeline's PCIe copies are DMA at full rate."""
        n = self.total_shards() if shards is None else shards
        each_al = (each + 63) // 64 * 64
        slab = alloc_pinned(each_al * n) if pinned else None
        if slab is None:
            raw = np.zeros(each_al * n + 64, dtype=np.uint8)
            off = (-raw.ctypes.data) % 64
            slab = raw[off:off + each_al * n]
        return [slab[i * each_al:i * each_al + each] for i in range(n)]

    def set_host_segment(self, nbytes: int) -> None:
        """Column-segment width of the host pipeline (0 = automatic)."""
        _check(self._L.rs_set_host_segment(self._h, nbytes))

    def set_reference_inversion_cache(self, on: bool) -> None:
        """GF(2^8): reproduce leopard8.go:508-555's inversion cache call for
        call, including the stale errLocs it hands out when two erasure
        patterns share its key (include/rs_mi355x.h).  On by default, as the
        reference keeps it; off keys the locators on the exact pattern.
        Clears the cache, as a fresh newFF8 would."""
        _check(self._L.rs_set_reference_inversion_cache(self._h, 1 if on else 0))
        self._ref_inv = bool(on)

    def reset_inversion_cache(self) -> None:
        """Empty the GF(2^8) inversion cache, keeping the mode: the state of a
        fresh newFF8 (the reference's stream wrappers build one per call)."""
        self.set_reference_inversion_cache(self._ref_inv)

    # ---------------- host-memory operations (Go [][]byte semantics)
    def encode(self, shards: list) -> None:
        """Encode (leopard16.go:116-125): parity written into shards[k:]."""
        ptrs, lens, _keep = _host_rows(shards)
        _check(self._L.rs_encode(self._h, ptrs, lens, len(shards)))

    def encode_async(self, shards: list) -> "EncodeTicket":
        """Queue an Encode behind the codec's previous calls (rs_encode_async):
        the copies and kernels of consecutive stripes overlap.  Keep `shards`
        alive and unmodified until the ticket's wait() returns; pinned parity
        rows (alloc_aligned(pinned=True)) are needed for the call to return early."""
        ptrs, lens, keep = _host_rows(shards)
        t = C.c_uint64(0)
        _check(self._L.rs_encode_async(self._h, ptrs, lens, len(shards), C.byref(t)))
        return EncodeTicket(self, t.value, keep)

    def verify(self, shards: list) -> bool:
        """Verify (leopard16.go:361-387)."""
        ptrs, lens, _keep = _host_rows(shards)
        ok = C.c_int(0)
        _check(self._L.rs_verify(self._h, ptrs, lens, len(shards), C.byref(ok)))
        return bool(ok.value)

    def verify_async(self, shards: list) -> "VerifyTicket":
        """Queue a Verify behind the codec's previous calls (rs_verify_async);
        the ticket's result() waits and returns the verdict.  Keep `shards`
        alive and unmodified until then."""
        ptrs, lens, keep = _host_rows(shards)
        t = C.c_uint64(0)
        _check(self._L.rs_verify_async(self._h, ptrs, lens, len(shards), C.byref(t)))
        return VerifyTicket(self, t.value, keep)

    def reconstruct_async(self, shards: list, recover_all: bool = True) -> "EncodeTicket":
        """Queue a Reconstruct (rs_reconstruct_async).  Missing entries of
        `shards` are replaced at call time by the buffers the rebuilt shards
        will land in (the EmptyShard's own row, else a fresh pinned row); their
        bytes are final once the ticket's wait() returns.  A stripe with nothing
        to rebuild gets ticket 0, which is done at once."""
        keep = []
        t = self._reconstruct(shards, recover_all, ticket=True, keep=keep)
        return EncodeTicket(self, t, keep)

    def _reconstruct(self, shards: list, recover_all: bool, ticket: bool = False, keep=None):
        total = len(shards)
        S = next((len(s) for s in shards if s is not None and len(s)), 0)
        k = self.data_shards()
        end = total if recover_all else min(k, total)
        bufs = list(shards)
        for i in range(min(end, total)):
            if bufs[i] is None or len(bufs[i]) == 0:
                # Go: shards[i][0:shardSize] when cap(shards[i]) >= shardSize, else
                # make([]byte, shardSize) (leopard16.go:556-560); fully overwritten
                bufs[i] = _capacity_view(bufs[i], S)
                if bufs[i] is None:
                    # a ticket's rebuilt rows go into pinned memory: pageable
                    # outputs would make the queued call synchronous (bounce slab).
                    # Callers that loop over stripes pass EmptyShard(row) of their
                    # own pinned rows instead (stream.py does); otherwise the rows
                    # come from the codec's pinned arena
                    bufs[i] = self._arena.take(S) if ticket else np.empty(S, dtype=np.uint8)
        ptrs = (C.c_void_p * total)()
        lens = (C.c_size_t * total)()
        for i, s in enumerate(shards):
            present = s is not None and len(s) > 0
            b = bufs[i]
            if b is not None and len(b):
                b = np.asarray(b)
                if b.dtype != np.uint8 or not b.flags["C_CONTIGUOUS"]:
                    raise TypeError("host shards must be C-contiguous numpy uint8 arrays")
                bufs[i] = b
                ptrs[i] = b.ctypes.data
            lens[i] = len(s) if present else 0
        if ticket:
            t = C.c_uint64(0)
            _check(self._L.rs_reconstruct_async(self._h, ptrs, lens, total, int(recover_all), C.byref(t)))
            keep.extend(bufs)
        else:
            _check(self._L.rs_reconstruct(self._h, ptrs, lens, total, int(recover_all)))
        for i in range(total):
            if lens[i] and (shards[i] is None or len(shards[i]) == 0):
                shards[i] = bufs[i]
        return t.value if ticket else shards

    def reconstruct(self, shards: list) -> list:
        """Reconstruct (leopard16.go:351-353): rebuild every missing shard."""
        return self._reconstruct(shards, True)

    def reconstruct_data(self, shards: list) -> list:
        """ReconstructData (leopard16.go:356-358): rebuild missing data shards only."""
        return self._reconstruct(shards, False)

    def reconstruct_some(self, shards: list, required: Sequence[bool]) -> list:
        """ReconstructSome (leopard16.go:343-348): only len(required) matters."""
        return self._reconstruct(shards, len(required) == self.total_shards())

    def encode_idx(self, data_shard, idx: int, parity: list) -> None:
        """EncodeIdx (leopard16.go:227-229): not supported."""
        _check(self._L.rs_encode_idx(self._h, None, 0, idx, None, None, 0))

    def update(self, shards: list, new_datashards: list) -> None:
        """Update (leopard16.go:273-275): not supported."""
        _check(self._L.rs_update(self._h, None, None, 0, None, None, 0))

    # ---------------- Split / Join (leopard16.go:232-340) through the C-ABI (rs_split / rs_join)
    def split_shard_size(self, length: int) -> int:
        """Bytes per shard Split produces for `length` bytes (leopard16.go:283-288)."""
        per = C.c_size_t(0)
        _check(self._L.rs_split_shard_size(self._h, length, C.byref(per)))
        return per.value

    def split(self, data) -> list:
        """Split (leopard16.go:277-340): k+p equal shards of one 64-byte-aligned
        host slab; data rows carry the data, the padding and parity rows are zero."""
        data = np.frombuffer(bytes(data), dtype=np.uint8) if not isinstance(data, np.ndarray) else data
        data = np.ascontiguousarray(data, dtype=np.uint8)
        if len(data) == 0:
            raise ErrShortData("not enough data to fill the number of requested shards")
        per = self.split_shard_size(len(data))
        total = self.total_shards()
        if total == 1 and len(data) & 63 == 0:
            return [data]
        raw = np.empty(per * total + 64, dtype=np.uint8)
        off = (-raw.ctypes.data) % 64
        slab = raw[off:off + per * total]
        _check(self._L.rs_split(self._h, data.ctypes.data, len(data), slab.ctypes.data, per, None))
        return [slab[i * per:(i + 1) * per] for i in range(total)]

    def split_dev(self, data, out=None, stream=None):
        """Split into a device slab: returns a [k+p, per_shard] uint8 CUDA tensor
        (or fills `out`, rows contiguous); `data` is host bytes/ndarray or a
        device tensor.  The shards land in HBM in the layout encode_dev reads."""
        import torch

        if isinstance(data, torch.Tensor):
            src, n = data.data_ptr(), data.numel()
            keep = data
        else:
            keep = np.ascontiguousarray(np.frombuffer(bytes(data), dtype=np.uint8) if not isinstance(data, np.ndarray)
                                        else data, dtype=np.uint8)
            src, n = keep.ctypes.data, keep.nbytes
        if n == 0:
            raise ErrShortData("not enough data to fill the number of requested shards")
        per = self.split_shard_size(n)
        if out is None:
            out = torch.empty((self.total_shards(), per), dtype=torch.uint8, device="cuda")
        _check(self._L.rs_split(self._h, src, n, out.data_ptr(), out.stride(0), _stream_handle(stream)))
        if stream is None:
            torch.cuda.current_stream().synchronize()
        del keep
        return out

    def join(self, dst, shards: list, out_size: int) -> None:
        """Join (leopard16.go:231-269): write the first out_size data bytes to dst
        (a file-like object with .write)."""
        k = self.data_shards()
        if len(shards) < k:
            raise ErrTooFewShards("too few shards given")
        ptrs = (C.c_void_p * k)()
        lens = (C.c_size_t * k)()
        keep = []
        empty = np.zeros(1, dtype=np.uint8)  # a non-nil zero-length shard (Go: counts 0 bytes, leopard16.go:239-250)
        for i in range(k):
            s = shards[i]
            if s is None:  # nil: ErrReconstructRequired
                ptrs[i], lens[i] = None, 0
                continue
            if len(s) == 0:
                ptrs[i], lens[i] = empty.ctypes.data, 0
                continue
            a = np.ascontiguousarray(s, dtype=np.uint8)
            keep.append(a)
            ptrs[i], lens[i] = a.ctypes.data, a.nbytes
        out = np.empty(out_size, dtype=np.uint8)
        _check(self._L.rs_join(self._h, ptrs, lens, k, out.ctypes.data if out_size else None, out_size, None))
        dst.write(out.tobytes())

    def join_dev(self, rows, out_size: int) -> np.ndarray:
        """Join from device-resident shards (a [k+p, S] tensor or a list): the
        first out_size bytes as a host array (device -> host copies)."""
        k = self.data_shards()
        if hasattr(rows, "dim"):
            ptrs = (C.c_void_p * k)(*[rows[i].data_ptr() for i in range(k)])
            lens = (C.c_size_t * k)(*([rows.shape[1]] * k))
        else:
            if len(rows) < k:
                raise ErrTooFewShards("too few shards given")
            ptrs = (C.c_void_p * k)(*[None if r is None else r.data_ptr() for r in rows[:k]])
            lens = (C.c_size_t * k)(*[0 if r is None else r.numel() for r in rows[:k]])
        out = np.empty(out_size, dtype=np.uint8)
        _check(self._L.rs_join(self._h, ptrs, lens, k, out.ctypes.data if out_size else None, out_size, None))
        return out

    # ---------------- Stream* methods of the ReedSolomon interface
    # (reedsolomon.go:52-58; rsFF8 :123-228, rsFF16 :231-336)
    # pinned block buffers a codec keeps between Stream* calls (depth x
    # total x 4 MiB: 1.25 GiB at 128 + 32); larger sets are freed per call
    STREAM_KEEP_BYTES = 2 << 30

    def _new_streamer(self):
        """The stream codec each Stream* call of the reference builds
        (newStreamEncoderFF16 / newStreamEncoderFF8).  GF(2^16) streams run on
        this codec.  GF(2^8) ones get a codec of their own, as in the
        reference (newFF8, reedsolomon.go:132), whose inversion cache
        stream.py clears per call, so the caller's cache is left as it was."""
        from . import stream

        if self.field_bits == 16:
            return stream.StreamEncoder16(self.data_shards(), self.parity_shards(), codec=self)
        own = ReedSolomon(self.data_shards(), self.parity_shards(), 8, self.device,
                          devices=self.devices if len(self.devices) > 1 else None)
        return stream.StreamEncoder8(self.data_shards(), self.parity_shards(), codec=own)

    @contextlib.contextmanager
    def _stream(self):
        """A stream codec for one Stream* call.  The codec keeps one and reuses
        its pinned block buffers across calls (up to STREAM_KEEP_BYTES); a call
        made while another thread's Stream* call holds it gets a fresh one of
        its own, so concurrent calls never share block buffers (the reference
        builds a fresh encoder per call, reedsolomon.go:132,240)."""
        if self._stream_lock.acquire(blocking=False):
            try:
                if self._streamer is None:
                    self._streamer = self._new_streamer()
                st = self._streamer
                yield st
            finally:
                if st.depth * st.total * st.block_size > self.STREAM_KEEP_BYTES:
                    st._bufs = None
                self._stream_lock.release()
            return
        st = self._new_streamer()
        try:
            yield st
        finally:
            st.close()
            if st.rs is not self:
                st.rs.close()

    def stream_encode(self, inputs: Sequence, outputs: Sequence) -> None:
        """StreamEncode (reedsolomon.go:124-138, :232-247)."""
        if len(inputs) != self.data_shards() or len(outputs) != self.parity_shards():
            raise ErrTooFewShards("too few shards given")
        with self._stream() as st:
            st.encode(inputs, outputs)

    def stream_verify(self, shards: Sequence) -> bool:
        """StreamVerify (reedsolomon.go:141-154, :250-263)."""
        if len(shards) != self.total_shards():
            raise ErrTooFewShards("too few shards given")
        with self._stream() as st:
            return st.verify(shards)

    def stream_reconstruct(self, inputs: Sequence, outputs: Sequence) -> None:
        """StreamReconstruct (reedsolomon.go:156-189, :265-298): the stream's
        reconstructData when no parity output is requested, else its
        reconstruct."""
        with self._stream() as st:
            st._check_io(inputs, outputs)
            if all(outputs[i] is None for i in range(self.data_shards(), self.total_shards())):
                st.reconstruct_data(inputs, outputs)
            else:
                st.reconstruct(inputs, outputs)

    def stream_reconstruct_data(self, inputs: Sequence, outputs: Sequence) -> None:
        """StreamReconstructData (reedsolomon.go:191-202, :300-310): the data
        outputs only, through StreamReconstruct."""
        k = self.data_shards()
        masked = [outputs[i] if i < k else None for i in range(self.total_shards())]
        self.stream_reconstruct(inputs, masked)

    def stream_split(self, data, dst: Sequence, size: int) -> None:
        """StreamSplit (reedsolomon.go:204-215, :312-323)."""
        from .stream import stream_split

        stream_split(self.data_shards(), data, dst, size)

    def stream_join(self, dst, shards: Sequence, out_size: int) -> None:
        """StreamJoin (reedsolomon.go:217-228, :325-336)."""
        from .stream import stream_join

        stream_join(self.data_shards(), self.parity_shards(), dst, shards, out_size)

    # ---------------- device-resident operations (torch CUDA tensors)
    def encode_dev(self, rows, stream=None) -> None:
        """Encode shards already in HBM; asynchronous on `stream` (default: current torch stream)."""
        ptrs, S = _dev_rows(rows, self.total_shards())
        _check(self._L.rs_encode_dev(self._h, ptrs, S, _stream_handle(stream)))

    def verify_dev(self, rows, stream=None) -> bool:
        ptrs, S = _dev_rows(rows, self.total_shards())
        ok = C.c_int(0)
        _check(self._L.rs_verify_dev(self._h, ptrs, S, C.byref(ok), _stream_handle(stream)))
        return bool(ok.value)

    def reconstruct_dev(self, rows, present: Sequence[bool], recover_all: bool = True, stream=None) -> None:
        """Rebuild rows whose `present` flag is False, in place in HBM."""
        ptrs, S = _dev_rows(rows, self.total_shards())
        pr = (C.c_uint8 * self.total_shards())(*[1 if x else 0 for x in present])
        _check(self._L.rs_reconstruct_dev(self._h, ptrs, pr, S, int(recover_all), _stream_handle(stream)))

    def verify_dev_batch(self, slab, stream=None) -> bool:
        """Verify every stripe of a [nstripes, k+p, S] uint8 CUDA tensor in one
        launch (rs_verify_dev_batch): True when all stripes verify."""
        if slab.dim() != 3 or slab.shape[1] != self.total_shards():
            raise TypeError("slab must be a [nstripes, k+p, S] uint8 CUDA tensor")
        if not slab.is_cuda or slab.dtype.itemsize != 1 or slab.stride(2) != 1:
            raise TypeError("slab rows must be contiguous uint8 on a CUDA device")
        n, _, S = slab.shape
        ok = C.c_int(0)
        _check(self._L.rs_verify_dev_batch(self._h, slab.data_ptr(), slab.stride(1), slab.stride(0), n, S, C.byref(ok),
                                           _stream_handle(stream)))
        return bool(ok.value)

    def reconstruct_dev_batch(self, slab, present: Sequence[bool], recover_all: bool = True, stream=None) -> None:
        """Rebuild the missing shards of every stripe of a [nstripes, k+p, S]
        uint8 CUDA tensor in place, all with the same erasure pattern
        (`present`, k+p flags), in one launch (rs_reconstruct_dev_batch).  Any
        view with contiguous rows works; stripe and row strides come from the
        tensor."""
        if slab.dim() != 3 or slab.shape[1] != self.total_shards():
            raise TypeError("slab must be a [nstripes, k+p, S] uint8 CUDA tensor")
        if not slab.is_cuda or slab.dtype.itemsize != 1 or slab.stride(2) != 1:
            raise TypeError("slab rows must be contiguous uint8 on a CUDA device")
        if len(present) != self.total_shards():
            raise ErrTooFewShards("need %d present flags, got %d" % (self.total_shards(), len(present)))
        n, _, S = slab.shape
        pr = (C.c_uint8 * len(present))(*[1 if x else 0 for x in present])
        _check(self._L.rs_reconstruct_dev_batch(self._h, slab.data_ptr(), slab.stride(1), slab.stride(0), n, pr, S,
                                                int(recover_all), _stream_handle(stream)))

    def encode_dev_batch(self, slab, stream=None) -> None:
        """Encode a [nstripes, k+p, S] uint8 CUDA tensor in one launch.  Any
        view whose rows are contiguous works (stride(2) == 1): stripe and row
        strides come from the tensor, so a byte-range slice slab[:, :, lo:hi]
        of a resident slab is encoded in place."""
        if slab.dim() != 3 or slab.shape[1] != self.total_shards():
            raise TypeError("slab must be a [nstripes, k+p, S] uint8 CUDA tensor")
        if not slab.is_cuda or slab.dtype.itemsize != 1 or slab.stride(2) != 1:
            raise TypeError("slab rows must be contiguous uint8 on a CUDA device")
        n, _, S = slab.shape
        _check(self._L.rs_encode_dev_batch(self._h, slab.data_ptr(), slab.stride(1), slab.stride(0), n, S,
                                           _stream_handle(stream)))


class EncodeTicket:
    """Completion handle of ReedSolomon.encode_async / reconstruct_async (holds
    the shard arrays alive).  Ticket 0 means no work was queued."""

    def __init__(self, codec: ReedSolomon, ticket: int, keep):
        self.codec, self.ticket, self._keep = codec, ticket, keep

    def done(self) -> bool:
        if self.ticket == 0:
            return True
        d = C.c_int(0)
        _check(self.codec._L.rs_ticket_query(self.codec._h, self.ticket, C.byref(d)))
        return bool(d.value)

    def wait(self) -> None:
        if self.ticket:
            _check(self.codec._L.rs_ticket_wait(self.codec._h, self.ticket))
        self._keep = None


class VerifyTicket(EncodeTicket):
    """Completion handle of ReedSolomon.verify_async."""

    def result(self) -> bool:
        ok = C.c_int(0)
        _check(self.codec._L.rs_verify_result(self.codec._h, self.ticket, C.byref(ok)))
        self._keep = None
        return bool(ok.value)


def New(data_shards: int, parity_shards: int, device: Optional[int] = None,
        devices: Optional[Sequence[int]] = None) -> ReedSolomon:
    """New (reedsolomon.go:69-81): GF(2^8) when data+parity <= 256, else GF(2^16)."""
    return ReedSolomon(data_shards, parity_shards, 0, device, devices)


def New8(data_shards: int, parity_shards: int, device: Optional[int] = None,
         devices: Optional[Sequence[int]] = None) -> ReedSolomon:
    """New8 (reedsolomon.go:84-87)."""
    return ReedSolomon(data_shards, parity_shards, 8, device, devices)


def New16(data_shards: int, parity_shards: int, device: Optional[int] = None,
          devices: Optional[Sequence[int]] = None) -> ReedSolomon:
    """New16 (reedsolomon.go:90-93)."""
    return ReedSolomon(data_shards, parity_shards, 16, device, devices)
