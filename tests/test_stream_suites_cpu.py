"""The reference's stream test suites (reedsolomon_test.go:521-1496,
hybrid_test.go, mode_comparison_test.go, alignment_test.go; replayed by
tests/ref_suites.py) on the CPU: the package's stream mirrors, driving an
oracle-backed stand-in codec, against the restated Go loops.  The same cases
run through the HIP engine in test_gpu_stream_suites.py."""
import pytest

from reedsolomon16_amd.stream import StreamEncoder8, StreamEncoder16
from tests import ref_suites
from tests.test_stream_cpu import OracleTicketCodec

# the suites' shards are at most 64 KiB / 4 bytes and 1024 bytes (1 + 1): one
# block of 64 KiB behaves as the reference's 4 MiB one for all of them
BLOCK = 64 * 1024


class MirrorRS(ref_suites.GoRS):
    """The stream calls through the package's StreamEncoder16 / StreamEncoder8
    (one per codec, kept across calls like ReedSolomon._stream) over the
    oracle stand-in; the rest as GoRS."""

    def __init__(self, k, p, bits, block=BLOCK, depth=2):
        super().__init__(k, p, bits, block)
        cls = StreamEncoder16 if bits == 16 else StreamEncoder8
        self.st = cls(k, p, block_size=block, depth=depth, codec=OracleTicketCodec(k, p, bits))

    def stream_encode(self, inputs, outputs):
        self.st.encode(inputs, outputs)

    def stream_verify(self, shards):
        return self.st.verify(shards)

    def stream_reconstruct(self, inputs, outputs):
        self.st._check_io(inputs, outputs)
        if all(outputs[i] is None for i in range(self.k, self.total)):
            self.st.reconstruct_data(inputs, outputs)
        else:
            self.st.reconstruct(inputs, outputs)

    def stream_split(self, data, dst, size):
        self.st.split(data, dst, size)

    def stream_join(self, dst, shards, out_size):
        self.st.join(dst, shards, out_size)


@pytest.mark.parametrize("case", sorted(ref_suites.CASES))
def test_reference_stream_suite_case(case):
    _, k, p, _, bits = ref_suites.CASES[case]
    want, want_checks = ref_suites.run(ref_suites.GoRS(k, p, bits, BLOCK), case)
    got, got_checks = ref_suites.run(MirrorRS(k, p, bits), case)
    assert got == want
    assert got_checks == want_checks
    failing = [d for d, ok in want_checks if not ok]
    assert failing == ref_suites.REFERENCE_FAILS.get(case, []), (case, failing)
