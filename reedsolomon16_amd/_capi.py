"""ctypes binding for the product library ``librs_mi355x.so`` (the C-ABI in
include/rs_mi355x.h).  The library is built in-tree by ``make -C
reedsolomon16_amd`` (or ``__graft_entry__.build()``).  There is no fallback:
if the library is missing, importing the codec raises."""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# RS_MI355X_LIB overrides the library path (used by scripts/ablate.sh experiment builds).
LIB_PATH = os.environ.get("RS_MI355X_LIB") or os.path.join(_HERE, "librs_mi355x.so")
HEADER_PATH = os.path.join(os.path.dirname(_HERE), "include", "rs_mi355x.h")

_lib = None


def lib() -> C.CDLL:
    """Load the engine library (raises OSError if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise OSError(f"{LIB_PATH} not found: build it with `make -C {_HERE}` (no CPU fallback exists)")
    L = C.CDLL(LIB_PATH)
    P, vp, sz, i32 = C.POINTER, C.c_void_p, C.c_size_t, C.c_int
    L.rs_new.argtypes = [i32, i32, i32, i32, P(vp)]
    L.rs_free.argtypes = [vp]
    L.rs_free.restype = None
    L.rs_new_multi.argtypes = [i32, i32, i32, P(i32), i32, P(vp)]
    L.rs_device_count.argtypes = [vp]
    L.rs_device_part.argtypes = [vp, i32, P(vp), P(i32)]
    L.rs_byte_range.argtypes = [sz, i32, i32, P(sz), P(sz)]
    for fn in ("rs_field_bits", "rs_data_shards", "rs_parity_shards", "rs_total_shards", "rs_shard_size_multiple"):
        getattr(L, fn).argtypes = [vp]
    L.rs_encode.argtypes = [vp, P(vp), P(sz), i32]
    L.rs_encode_async.argtypes = [vp, P(vp), P(sz), i32, P(C.c_uint64)]
    L.rs_encode_wait.argtypes = [vp, C.c_uint64]
    L.rs_encode_query.argtypes = [vp, C.c_uint64, P(i32)]
    L.rs_verify.argtypes = [vp, P(vp), P(sz), i32, P(i32)]
    L.rs_verify_async.argtypes = [vp, P(vp), P(sz), i32, P(C.c_uint64)]
    L.rs_verify_result.argtypes = [vp, C.c_uint64, P(i32)]
    L.rs_reconstruct_async.argtypes = [vp, P(vp), P(sz), i32, i32, P(C.c_uint64)]
    L.rs_ticket_wait.argtypes = [vp, C.c_uint64]
    L.rs_ticket_query.argtypes = [vp, C.c_uint64, P(i32)]
    L.rs_reconstruct.argtypes = [vp, P(vp), P(sz), i32, i32]
    L.rs_encode_idx.argtypes = [vp, vp, sz, i32, P(vp), P(sz), i32]
    L.rs_update.argtypes = [vp, P(vp), P(sz), i32, P(vp), P(sz), i32]
    L.rs_encode_dev.argtypes = [vp, P(vp), sz, vp]
    L.rs_verify_dev.argtypes = [vp, P(vp), sz, P(i32), vp]
    L.rs_reconstruct_dev.argtypes = [vp, P(vp), P(C.c_uint8), sz, i32, vp]
    L.rs_reconstruct_dev_batch.argtypes = [vp, vp, sz, sz, sz, P(C.c_uint8), sz, i32, vp]
    L.rs_verify_dev_batch.argtypes = [vp, vp, sz, sz, i32, sz, P(i32), vp]
    L.rs_encode_dev_batch.argtypes = [vp, vp, sz, sz, i32, sz, vp]
    L.rs_set_host_segment.argtypes = [vp, sz]
    L.rs_set_reference_inversion_cache.argtypes = [vp, i32]
    L.rs_split_shard_size.argtypes = [vp, sz, P(sz)]
    L.rs_split.argtypes = [vp, vp, sz, vp, sz, vp]
    L.rs_join.argtypes = [vp, P(vp), P(sz), i32, vp, sz, vp]
    L.rs_host_alloc.argtypes = [sz, P(vp)]
    L.rs_host_free.argtypes = [vp]
    L.rs_host_free.restype = None
    L.rs_host_register.argtypes = [vp, sz]
    L.rs_host_unregister.argtypes = [vp]
    L.rs_encode_path.argtypes = [vp]
    L.rs_encode_path.restype = C.c_char_p
    L.rs_strerror.argtypes = [i32]
    L.rs_strerror.restype = C.c_char_p
    L.rs_debug_field_tables.argtypes = [i32, vp, vp, vp, vp]
    L.rs_debug_twiddle.argtypes = [i32, C.c_uint32, vp]
    L.rs_debug_twiddle_dwords.argtypes = [i32]
    L.rs_debug_error_locators.argtypes = [i32, i32, i32, vp, vp]
    L.rs_debug_split_check.argtypes = [i32, C.c_uint32]
    L.rs_debug_split_emulate.argtypes = [vp, vp, vp, sz]
    L.rs_debug_sub_check.argtypes = []
    L.rs_debug_sub_twiddle.argtypes = [C.c_uint32, vp]
    L.rs_debug_sub_swap.argtypes = [C.c_uint32]
    L.rs_debug_sub_swap.restype = C.c_uint32
    L.rs_debug_dec_plan.argtypes = [i32, vp, vp]
    L.rs_debug_set_path.argtypes = [C.c_char_p, i32]
    L.rs_debug_zc_rows.argtypes = [P(vp), i32, sz]
    _lib = L
    return L


_PATH_DEFAULTS = {"bs": 1, "sub": 1, "prune": 1, "unit_width": -1, "hp_tiles": 0, "hp_step": 0, "zc": 3, "hp_tune": 1, "rec_half": 0, "dec_lab": 0, "lds_big": 1}


def set_path(knob: str, value: int) -> None:
    """rs_debug_set_path: a test-only kernel-path override (include/rs_mi355x.h)."""
    if lib().rs_debug_set_path(knob.encode(), int(value)) != 0:
        raise ValueError("unknown path knob %r = %r" % (knob, value))


def reset_paths() -> None:
    for k, v in _PATH_DEFAULTS.items():
        set_path(k, v)


def header_functions() -> list[str]:
    """Function names declared in include/rs_mi355x.h."""
    import re

    text = open(HEADER_PATH).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(rs_[a-z0-9_]+)\s*\(", text)))
