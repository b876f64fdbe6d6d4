"""The reference's stream test suites (reedsolomon_test.go:521-1496,
hybrid_test.go, mode_comparison_test.go, alignment_test.go; replayed by
tests/ref_suites.py) through the MI355X engine: the ReedSolomon interface's
Stream* methods (New16 / New / New8 codecs, each stream call on the HIP
kernels) against the restated Go loops answered by the oracle.  Every byte a
writer receives, every verdict and error must match, and the Go test's own
assertions must hold."""
import pytest

import reedsolomon16_amd as rs
from tests import ref_suites

pytestmark = pytest.mark.gpu


def _codec(case, k, p, bits):
    # the constructor each Go test uses: New16 for FF16, New (GF(2^8) for
    # k + p <= 256) for FF8, New8 in alignment_test.go:45
    if bits == 16:
        return rs.New16(k, p)
    return rs.New8(k, p) if case.startswith("Alignment") else rs.New(k, p)


@pytest.mark.parametrize("case", sorted(ref_suites.CASES))
def test_gpu_reference_stream_suite_case(case):
    _, k, p, _, bits = ref_suites.CASES[case]
    want, want_checks = ref_suites.run(ref_suites.GoRS(k, p, bits, 64 * 1024), case)
    c = _codec(case, k, p, bits)
    assert c.field_bits == bits
    try:
        got, got_checks = ref_suites.run(c, case)
    finally:
        c.close()
    assert got == want
    assert got_checks == want_checks
    assert [d for d, ok in got_checks if not ok] == ref_suites.REFERENCE_FAILS.get(case, [])


def test_gpu_stream_methods_reuse_one_stream_codec():
    """Stream* calls on one codec reuse its pinned block buffers; a GF(2^8)
    codec's streams run on a codec of their own (fresh inversion cache per
    call, reedsolomon.go:132), a GF(2^16) codec's on itself."""
    c16 = rs.New16(4, 2)
    c8 = rs.New(4, 2)
    try:
        case = "StreamVerify/FF16_Size_32768"
        ref_suites.run(c16, case)
        with c16._stream() as s:
            pass
        ref_suites.run(c16, case)
        with c16._stream() as s2:
            assert s2 is s and s.rs is c16
            # a call while the kept one is busy gets a fresh stream codec
            with c16._stream() as s3:
                assert s3 is not s and s3.rs is c16
        ref_suites.run(c8, "StreamVerify/FF8_Size_32768")
        with c8._stream() as s8:
            assert s8.rs is not c8 and s8.rs.field_bits == 8
    finally:
        c16.close()
        c8.close()


def test_gpu_stream_calls_from_two_threads():
    """Concurrent StreamEncode calls on one codec (advisor finding, round 5):
    each call has block buffers of its own, so both streams' parity is exact."""
    import io
    import threading

    import numpy as np

    from oracle import orc

    k, p, n = 6, 3, (4 << 20) * 2 + 4096  # two 4 MiB blocks and a short one per shard
    c = rs.New16(k, p)
    rng = np.random.default_rng(9)
    datas = [rng.integers(0, 256, (k, n), dtype=np.uint8) for _ in range(2)]
    outs = [[io.BytesIO() for _ in range(p)] for _ in range(2)]
    errs = []

    def run(j):
        try:
            for _ in range(2):
                for o in outs[j]:
                    o.seek(0)
                    o.truncate()
                c.stream_encode([io.BytesIO(datas[j][i].tobytes()) for i in range(k)], outs[j])
        except Exception as e:
            errs.append(e)

    th = [threading.Thread(target=run, args=(j,)) for j in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errs, errs
    try:
        for j in range(2):
            for off in (0, 4 << 20, 8 << 20):
                w = min(4 << 20, n - off)
                al = (w + 63) // 64 * 64
                blk = np.zeros((k, al), np.uint8)
                blk[:, :w] = datas[j][:, off:off + w]
                ref = orc.encode(16, k, p, blk)
                for i in range(p):
                    got = np.frombuffer(outs[j][i].getvalue(), np.uint8)
                    assert np.array_equal(got[off:off + al], ref[i]), (j, off, i)
    finally:
        c.close()


def test_gpu_with_concurrency_returns_the_codec():
    """WithConcurrency (reedsolomon.go:415-427) is a no-op returning the codec."""
    c = rs.New16(4, 2)
    try:
        assert c.with_concurrency(8) is c and c.with_concurrency(0) is c
    finally:
        c.close()
