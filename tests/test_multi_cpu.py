"""CPU tests of the multi-device codec's host side (rs_new_multi, no device
calls): construction and its errors, the part accessors, the byte ranges
(identical to dist.byte_range, the torch layer's split), and the argument
validation a multi-device call shares with a one-device codec.  The calls
that move data run on the GPU (tests/test_gpu_multi.py)."""
import ctypes as C

import numpy as np
import pytest

import reedsolomon16_amd as rs
from reedsolomon16_amd import _capi
from reedsolomon16_amd import dist as rsd

RS_ERR_INVALID_ARG = 53


def multi(bits, k, p, devices):
    L = _capi.lib()
    h = C.c_void_p()
    arr = (C.c_int * len(devices))(*devices)
    e = L.rs_new_multi(bits, k, p, arr, len(devices), C.byref(h))
    return e, h


def test_new_multi_parts_and_free():
    L = _capi.lib()
    e, h = multi(16, 128, 32, [0, 0, 0, 0])
    assert e == 0 and h.value
    assert L.rs_device_count(h) == 4
    assert L.rs_data_shards(h) == 128 and L.rs_parity_shards(h) == 32 and L.rs_field_bits(h) == 16
    seen = set()
    for g in range(4):
        part, dev = C.c_void_p(), C.c_int(-1)
        assert L.rs_device_part(h, g, C.byref(part), C.byref(dev)) == 0
        assert part.value and part.value != h.value and dev.value == 0
        assert L.rs_device_count(part) == 1 and L.rs_total_shards(part) == 160
        seen.add(part.value)
    assert len(seen) == 4
    part = C.c_void_p()
    assert L.rs_device_part(h, 4, C.byref(part), None) == RS_ERR_INVALID_ARG
    assert L.rs_device_part(h, -1, C.byref(part), None) == RS_ERR_INVALID_ARG
    L.rs_free(h)


def test_new_multi_one_device_is_plain_codec():
    L = _capi.lib()
    e, h = multi(8, 10, 4, [3])
    assert e == 0 and L.rs_device_count(h) == 1
    part, dev = C.c_void_p(), C.c_int(-1)
    assert L.rs_device_part(h, 0, C.byref(part), C.byref(dev)) == 0
    assert part.value == h.value and dev.value == 3
    L.rs_free(h)


@pytest.mark.parametrize("args,want", [
    ((16, 0, 4, [0, 0]), 1),            # ErrInvShardNum, as rs_new
    ((16, 65530, 10, [0, 0]), 2),       # ErrMaxShardNum
    ((16, 4, 2, []), RS_ERR_INVALID_ARG),
    ((16, 4, 2, [0] * 65), RS_ERR_INVALID_ARG),  # RS_MAX_DEVICES
    ((12, 4, 2, [0, 0]), RS_ERR_INVALID_ARG),
])
def test_new_multi_errors(args, want):
    e, h = multi(*args)
    assert e == want and not h.value


def test_new_multi_field_dispatch():
    """field_bits 0 is New (reedsolomon.go:69-81) for every part."""
    L = _capi.lib()
    for k, p, bits in ((10, 4, 8), (200, 100, 16)):
        e, h = multi(0, k, p, [0, 0, 0])
        assert e == 0 and L.rs_field_bits(h) == bits
        for g in range(3):
            part = C.c_void_p()
            assert L.rs_device_part(h, g, C.byref(part), None) == 0
            assert L.rs_field_bits(part) == bits
        L.rs_free(h)


@pytest.mark.parametrize("S", [64, 128, 640, 4096, 1 << 20, 256 << 10, 64 * 1001])
@pytest.mark.parametrize("n", [1, 2, 3, 4, 8, 13])
def test_byte_range_matches_dist(S, n):
    L = _capi.lib()
    lo, hi = C.c_size_t(), C.c_size_t()
    prev = 0
    for g in range(n):
        assert L.rs_byte_range(S, g, n, C.byref(lo), C.byref(hi)) == 0
        assert (lo.value, hi.value) == rsd.byte_range(S, g, n)
        assert lo.value == prev and lo.value % 64 == 0 and hi.value % 64 == 0
        prev = hi.value
    assert prev == S


def test_byte_range_errors():
    L = _capi.lib()
    lo, hi = C.c_size_t(), C.c_size_t()
    assert L.rs_byte_range(100, 0, 2, C.byref(lo), C.byref(hi)) == 6  # ErrInvalidShardSize
    assert L.rs_byte_range(128, 2, 2, C.byref(lo), C.byref(hi)) == RS_ERR_INVALID_ARG
    assert L.rs_byte_range(128, 0, 0, C.byref(lo), C.byref(hi)) == RS_ERR_INVALID_ARG


def test_multi_validation_matches_single_codec():
    """Validation runs on the parent before any part is called, with the
    reference's order and codes (encoder.go:102-126, leopard16.go:116-135)."""
    c = rs.New16(4, 2, devices=[0, 0])
    assert c.device_count == 2 and c.devices == [0, 0]
    good = [np.zeros(64, np.uint8) for _ in range(6)]
    with pytest.raises(rs.ErrTooFewShards):
        c.encode(good[:5])
    with pytest.raises(rs.ErrShardSize):
        c.encode(good[:5] + [np.zeros(128, np.uint8)])
    with pytest.raises(rs.ErrShardNoData):
        c.encode([np.zeros(0, np.uint8)] * 6)
    with pytest.raises(rs.ErrInvalidShardSize):
        c.encode([np.zeros(100, np.uint8)] * 6)
    with pytest.raises(rs.ErrShardSize):
        c.verify(good[:5] + [np.zeros(128, np.uint8)])
    # a reconstruct with nothing missing returns before any device work
    assert c.reconstruct(list(good)) is not None
    shards = list(good)
    shards[0] = shards[1] = shards[2] = None
    with pytest.raises(rs.ErrTooFewShards):
        c.reconstruct(shards)
    with pytest.raises(rs.ErrNotSupported):
        c.update([], [])
    assert c.byte_range(4096, 1) == rsd.byte_range(4096, 1, 2)
    c.close()


def test_multi_refuses_device_entry_points():
    L = _capi.lib()
    e, h = multi(16, 4, 2, [0, 0])
    assert e == 0
    rows = (C.c_void_p * 6)(*([0x1000] * 6))
    ok = C.c_int()
    assert L.rs_encode_dev(h, rows, 64, None) == RS_ERR_INVALID_ARG
    assert L.rs_verify_dev(h, rows, 64, C.byref(ok), None) == RS_ERR_INVALID_ARG
    assert L.rs_encode_dev_batch(h, 0x1000, 64, 64 * 6, 1, 64, None) == RS_ERR_INVALID_ARG
    pr = (C.c_uint8 * 6)(0, 1, 1, 1, 1, 1)
    assert L.rs_reconstruct_dev(h, rows, pr, 64, 1, None) == RS_ERR_INVALID_ARG
    assert L.rs_reconstruct_dev_batch(h, 0x1000, 64, 64 * 6, 1, pr, 64, 1, None) == RS_ERR_INVALID_ARG
    assert L.rs_verify_dev_batch(h, 0x1000, 64, 64 * 6, 1, 64, C.byref(ok), None) == RS_ERR_INVALID_ARG
    # unknown tickets on the parent's ticket space
    d = C.c_int()
    assert L.rs_ticket_wait(h, 0) == 0
    assert L.rs_ticket_query(h, 0, C.byref(d)) == 0 and d.value == 1
    assert L.rs_ticket_wait(h, 5) == RS_ERR_INVALID_ARG
    assert L.rs_verify_result(h, 1, C.byref(ok)) == RS_ERR_INVALID_ARG
    L.rs_free(h)


def test_multi_split_join_host():
    """Split / Join of host slabs need no device, multi-device or not (leopard16.go:232-340)."""
    c1, c4 = rs.New16(5, 3), rs.New16(5, 3, devices=[0, 0, 0, 0])
    data = np.arange(1000, dtype=np.uint32).astype(np.uint8)
    a, b = c1.split(data), c4.split(data)
    assert len(a) == len(b) == 8 and all(np.array_equal(x, y) for x, y in zip(a, b))
    import io

    out = io.BytesIO()
    c4.join(out, b, 1000)
    assert out.getvalue() == data.tobytes()
    c1.close()
    c4.close()
