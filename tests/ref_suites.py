"""Test helper: the reference's own test functions, replayed step for step
over any object with the ReedSolomon interface's stream and memory methods.

Each scenario follows one Go test function (cited per function) and returns
a log of everything a caller can observe: the bytes every writer received,
verify verdicts, join output and error names.  The tests run a scenario twice
-- on ``GoRS`` (the reference's loops restated in tests/go_stream.py, r.rs.*
answered by the oracle) and on the system under test (the stream mirror on an
oracle codec on the CPU, the HIP engine on the GPU) -- and require equal logs.
They then check the Go test's own assertions on the log (``checks``), so a
case where the reference's test itself would fail shows up as such instead
of being silently "matched".

Inputs are the Go tests' deterministic ``data[i] = byte(i % 256)``
(reedsolomon_test.go:1095-1098, hybrid_test.go:23-26,
mode_comparison_test.go:47-50, alignment_test.go:55-58), so no randomness is
involved.
"""
from __future__ import annotations

import io

import numpy as np

from oracle.orc import Oracle
from reedsolomon16_amd.codec import ErrPanic, ErrReconstructRequired, ErrShortData, ErrTooFewShards, RSError
from reedsolomon16_amd.stream import stream_join, stream_split
from tests.go_stream import GoPanic, GoStream8, GoStream16


def ref_data(n: int) -> bytes:
    return bytes(i % 256 for i in range(n))


def err_name(e: BaseException) -> str:
    if isinstance(e, (GoPanic, ErrPanic)):
        return "panic"
    if isinstance(e, RSError):
        return type(e).__name__
    if isinstance(e, ValueError) and str(e).startswith("Err"):
        return str(e)  # go_stream.py's sentinels
    raise e


def memory_join(k: int, dst, shards, out_size: int) -> None:
    """leopardFF16.Join (leopard16.go:232-269; leopardFF8.Join leopard8.go
    the same), for the model side."""
    if len(shards) < k:
        raise ErrTooFewShards("too few shards given")
    shards = shards[:k]
    size = 0
    for s in shards:
        if s is None:
            raise ErrReconstructRequired("reconstruction required")
        size += len(s)
        if size >= out_size:
            break
    if size < out_size:
        raise ErrShortData("short data")
    left = out_size
    for s in shards:
        if left < len(s):
            dst.write(bytes(s[:left]))
            return
        dst.write(bytes(s))
        left -= len(s)


class GoRS:
    """The reference's rsFF16 / rsFF8 (reedsolomon.go:101-336) over the Go-loop
    models: Stream* through GoStream16 / GoStream8 (a fresh one per call, as
    every Stream* method builds one), StreamSplit/StreamJoin through the
    package's transcription (stream_split / stream_join; their layout is pinned
    by hand-derived cases in test_stream_splitjoin_cpu.py), memory Reconstruct
    and Join through the oracle."""

    def __init__(self, k: int, p: int, bits: int, block: int):
        self.k, self.p, self.total, self.bits, self.block = k, p, k + p, bits, block
        self.orc = Oracle(bits, k, p)

    def _st(self):
        return (GoStream16 if self.bits == 16 else GoStream8)(self.k, self.p, self.block)

    def stream_encode(self, inputs, outputs):
        self._st().encode(inputs, outputs)

    def stream_verify(self, shards):
        return self._st().verify(shards)

    def stream_reconstruct(self, inputs, outputs):
        st = self._st()
        if all(outputs[i] is None for i in range(self.k, self.total)):  # reedsolomon.go:174-188
            st.reconstruct_data(inputs, outputs)
        else:
            st.reconstruct(inputs, outputs)

    def stream_reconstruct_data(self, inputs, outputs):
        self.stream_reconstruct(inputs, [outputs[i] if i < self.k else None for i in range(self.total)])

    def stream_split(self, data, dst, size):
        stream_split(self.k, data, dst, size)

    def stream_join(self, dst, shards, out_size):
        stream_join(self.k, self.p, dst, shards, out_size)

    def reconstruct(self, shards):
        rows = [None if s is None or len(s) == 0 else np.frombuffer(bytes(s), np.uint8) for s in shards]
        e, out = self.orc.reconstruct(rows, True)
        if e:
            raise RSError("oracle error %d" % e)
        return [bytes(out[i]) if rows[i] is None else shards[i] for i in range(self.total)]

    def join(self, dst, shards, out_size):
        memory_join(self.k, dst, shards, out_size)


def _readers(bufs):
    return [None if b is None else io.BytesIO(b) for b in bufs]


def _writers(n):
    return [io.BytesIO() for _ in range(n)]


class Log(list):
    def step(self, name, fn, *args):
        """Run one interface call; log its result (bytes / verdict) or error."""
        try:
            r = fn(*args)
        except Exception as e:  # noqa: BLE001 -- every error is part of the log
            self.append((name, "error", err_name(e)))
            return None
        self.append((name, "ok", r if isinstance(r, (bool, type(None))) else "value"))
        return r


def _split_encode(rs, log, k, p, data):
    dw = _writers(k)
    log.step("StreamSplit", rs.stream_split, io.BytesIO(data), dw, len(data))
    dshards = [w.getvalue() for w in dw]
    log.append(("data shards", dshards))
    pw = _writers(p)
    log.step("StreamEncode", rs.stream_encode, _readers(dshards), pw)
    pshards = [w.getvalue() for w in pw]
    log.append(("parity shards", pshards))
    return dshards, pshards


def _stream_join(rs, log, readers_bytes, n, name="StreamJoin"):
    out = io.BytesIO()
    log.step(name, rs.stream_join, out, _readers(readers_bytes), n)
    log.append((name + " output", out.getvalue()))
    return out.getvalue()


def _stream_rebuild(rs, log, k, p, dshards, pshards, lost, name="StreamReconstruct", method="stream_reconstruct"):
    everything = dshards + pshards
    inputs = [None if i in lost else everything[i] for i in range(k + p)]
    outs = [io.BytesIO() if i in lost else None for i in range(k + p)]
    log.step(name, getattr(rs, method), _readers(inputs), outs)
    rebuilt = {i: outs[i].getvalue() for i in lost}
    log.append((name + " output", [rebuilt[i] for i in sorted(lost)]))
    return rebuilt


# --------------------------------------------------------------------------- scenarios
# each returns (log, checks): checks = [(description, holds)] for the Go test's assertions


def stream_encode_decode(rs, k, p, n):
    """testStreamEncodeDecodeNew (reedsolomon_test.go:1081-1182)."""
    log, data = Log(), ref_data(n)
    d, par = _split_encode(rs, log, k, p, data)
    ok = log.step("StreamVerify", rs.stream_verify, _readers(d + par))
    out = _stream_join(rs, log, d, n)
    return log, [("verify true", ok is True), ("join == data", out == data)]


def stream_reconstruction(rs, k, p, n):
    """testStreamReconstructionNew (reedsolomon_test.go:1214-1368): shards 0
    and k-1 lost, StreamReconstruct into their writers, StreamJoin."""
    log, data = Log(), ref_data(n)
    d, par = _split_encode(rs, log, k, p, data)
    lost = [0, k - 1]
    rebuilt = _stream_rebuild(rs, log, k, p, d, par, lost)
    merge = [rebuilt[i] if i in rebuilt else d[i] for i in range(k)]
    out = _stream_join(rs, log, merge, n)
    return log, [("rebuilt == original", all(rebuilt[i] == d[i] for i in lost)), ("join == data", out == data)]


def stream_reconstruct_data(rs, k, p, n):
    """testStreamReconstructDataNew (reedsolomon_test.go:783-925): shards 0 and
    2 lost, StreamReconstructData, StreamJoin."""
    log, data = Log(), ref_data(n)
    d, par = _split_encode(rs, log, k, p, data)
    lost = [0, 2]
    rebuilt = _stream_rebuild(rs, log, k, p, d, par, lost, "StreamReconstructData", "stream_reconstruct_data")
    merge = [rebuilt[i] if i in rebuilt else d[i] for i in range(k)]
    out = _stream_join(rs, log, merge, n)
    return log, [("rebuilt == original", all(rebuilt[i] == d[i] for i in lost)), ("join == data", out == data)]


def stream_verify(rs, k, p, n):
    """testStreamVerifyNew (reedsolomon_test.go:1400-1496): true on the
    encoded shards, false after flipping byte 0 of shard 0."""
    log, data = Log(), ref_data(n)
    d, par = _split_encode(rs, log, k, p, data)
    ok = log.step("StreamVerify", rs.stream_verify, _readers(d + par))
    bad = bytearray(d[0])
    if bad:
        bad[0] ^= 0xFF
    ok2 = log.step("StreamVerify tampered", rs.stream_verify, _readers([bytes(bad)] + d[1:] + par))
    return log, [("verify true", ok is True), ("tampered verify not true", ok2 is not True)]


def stream_non_uniform(rs, k, p, n):
    """testStreamNonUniformShards (reedsolomon_test.go:683-780): the data cut
    by hand into k pieces (the first n % k one byte longer), StreamEncode,
    StreamJoin of the pieces."""
    log, data = Log(), ref_data(n)
    per, rem = divmod(n, k)
    pieces, pos = [], 0
    for i in range(k):
        ln = per + (1 if i < rem else 0)
        pieces.append(data[pos:pos + ln])
        pos += ln
    pw = _writers(p)
    log.step("StreamEncode", rs.stream_encode, _readers(pieces), pw)
    log.append(("parity shards", [w.getvalue() for w in pw]))
    out = _stream_join(rs, log, pieces, n)
    return log, [("join == data", out == data)]


def hybrid(rs, k, p, n):
    """TestHybridReconstruction (hybrid_test.go:10-181): memory Reconstruct
    and StreamReconstruct of shard 0 from the same stream-made shards."""
    log, data = Log(), ref_data(n)
    d, par = _split_encode(rs, log, k, p, data)
    mem = [None] + [bytearray(s) for s in (d + par)[1:]]
    got = log.step("Reconstruct", rs.reconstruct, mem)
    mem0 = bytes(got[0]) if got is not None and got[0] is not None else None
    log.append(("Reconstruct output", mem0))
    rebuilt = _stream_rebuild(rs, log, k, p, d, par, [0])
    return log, [("memory rebuild == original", mem0 == d[0]), ("stream rebuild == original", rebuilt[0] == d[0])]


def mode_comparison(rs, k, p, n):
    """testModeComparisonWithSize (mode_comparison_test.go:40-323): stream
    and memory Join, then memory Reconstruct + Join and StreamReconstruct +
    StreamJoin of shard 0."""
    log, data = Log(), ref_data(n)
    d, par = _split_encode(rs, log, k, p, data)
    ok = log.step("StreamVerify", rs.stream_verify, _readers(d + par))
    mj = io.BytesIO()
    log.step("Join", rs.join, mj, [bytearray(s) for s in d], n)
    log.append(("Join output", mj.getvalue()))
    sj = _stream_join(rs, log, d, n)
    mem = [None] + [bytearray(s) for s in (d + par)[1:]]
    got = log.step("Reconstruct", rs.reconstruct, mem)
    mem0 = bytes(got[0]) if got is not None and got[0] is not None else None
    log.append(("Reconstruct output", mem0))
    mrj = io.BytesIO()
    if got is not None:
        log.step("Join rebuilt", rs.join, mrj, [bytearray(s) for s in got[:k]], n)
    log.append(("Join rebuilt output", mrj.getvalue()))
    rebuilt = _stream_rebuild(rs, log, k, p, d, par, [0])
    srj = _stream_join(rs, log, [rebuilt[0]] + d[1:], n, "StreamJoin rebuilt")
    return log, [("verify true", ok is True), ("memory join == data", mj.getvalue() == data),
                 ("stream join == data", sj == data), ("memory rebuilt join == data", mrj.getvalue() == data),
                 ("stream rebuilt join == data", srj == data)]


def alignment(rs, k, p, n):
    """testAlignmentReconstruction (alignment_test.go:37-212): StreamVerify,
    StreamReconstruct of shard 0, StreamVerify with it, StreamJoin."""
    log, data = Log(), ref_data(n)
    d, par = _split_encode(rs, log, k, p, data)
    ok = log.step("StreamVerify", rs.stream_verify, _readers(d + par))
    rebuilt = _stream_rebuild(rs, log, k, p, d, par, [0])
    ok2 = log.step("StreamVerify rebuilt", rs.stream_verify, _readers([rebuilt[0]] + d[1:] + par))
    out = _stream_join(rs, log, [rebuilt[0]] + d[1:], n)
    return log, [("verify true", ok is True), ("rebuilt == original", rebuilt[0] == d[0]),
                 ("verify rebuilt true", ok2 is True), ("join == data", out == data)]


SCENARIOS = {
    "encode_decode": stream_encode_decode,
    "reconstruction": stream_reconstruction,
    "reconstruct_data": stream_reconstruct_data,
    "verify": stream_verify,
    "non_uniform": stream_non_uniform,
    "hybrid": hybrid,
    "mode_comparison": mode_comparison,
    "alignment": alignment,
}

_SIZES = [1, 32, 63, 64, 65, 127, 128, 129, 1024, 32768, 65536]
_REC_SIZES = [63, 64, 65, 127, 128, 32768]

# (scenario, k, p, size, bits), named after the Go test that runs it
CASES = {}
for _bits in (8, 16):
    _f = "FF%d" % _bits
    CASES["StreamBasicEncodeDecode/%s" % _f] = ("encode_decode", 4, 2, 16384, _bits)  # :521-534
    for _k, _p in [(2, 1), (4, 2), (8, 4), (16, 8), (100, 50)]:  # :537-562
        CASES["StreamDifferentShardSizes/%s_ds%d_ps%d" % (_f, _k, _p)] = ("encode_decode", _k, _p, 16384, _bits)
    for _n in _SIZES:  # :565-604 (size 0 skipped there for both fields)
        CASES["StreamDifferentDataSizes/%s_Size_%d" % (_f, _n)] = ("encode_decode", 4, 2, _n, _bits)
    for _k, _p in [(10, 4), (20, 8), (50, 20), (100, 40), (120, 50)]:  # :607-638
        if _bits == 8 or _k + _p <= 128:
            CASES["StreamLargeShardCount/%s_ds%d_ps%d" % (_f, _k, _p)] = ("encode_decode", _k, _p, 8192, _bits)
    CASES["StreamEdgeCases/%s_non_uniform" % _f] = ("non_uniform", 4, 2, 100, _bits)  # :641-657
    for _n in [63, 64, 65, 32768]:  # :660-680
        CASES["StreamReconstructData/%s_Size_%d" % (_f, _n)] = ("reconstruct_data", 4, 2, _n, _bits)
    for _n in _REC_SIZES:  # :1185-1211, :1371-1397
        CASES["StreamReconstruction/%s_Size_%d" % (_f, _n)] = ("reconstruction", 4, 2, _n, _bits)
        CASES["StreamVerify/%s_Size_%d" % (_f, _n)] = ("verify", 4, 2, _n, _bits)
CASES["StreamEdgeCases/single_shard"] = ("encode_decode", 1, 1, 1024, 8)  # :642-644
CASES["StreamEdgeCases/minimal_data"] = ("encode_decode", 4, 2, 1, 8)  # :646-648
CASES["HybridReconstruction"] = ("hybrid", 4, 2, 1024, 16)
for _n in _REC_SIZES:
    CASES["ModeComparison/Size_%d" % _n] = ("mode_comparison", 4, 2, _n, 16)
for _n in [63, 64, 65, 127, 128, 129, 32768]:  # alignment_test.go:13-34: New8
    CASES["AlignmentStreamReconstruction/%d" % _n] = ("alignment", 4, 2, _n, 8)

# Go tests whose own assertions the restated reference loops do not satisfy:
# {case: [failing check descriptions]} -- filled from the model runs
# (test_stream_suites_cpu.py prints the list when it changes).
REFERENCE_FAILS: dict = {}


def run(rs, case):
    scen, k, p, n, bits = CASES[case]
    return SCENARIOS[scen](rs, k, p, n)
