"""ORACLE — TEST INFRASTRUCTURE ONLY.  ctypes binding for oracle/_build/liboracle.so.

Used by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg only.
The library is the scalar C restatement in oracle/leopard_ref.c.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "_build", "liboracle.so")
_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _SO


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_SO):
            build()
        L = C.CDLL(_SO)
        P = C.POINTER
        L.orc_init.restype = C.c_int
        L.orc16_encode.argtypes = [C.c_int, C.c_int, P(C.c_void_p), P(C.c_size_t), C.c_int]
        L.orc16_verify.argtypes = [C.c_int, C.c_int, P(C.c_void_p), P(C.c_size_t), C.c_int, P(C.c_int)]
        L.orc16_reconstruct.argtypes = [C.c_int, C.c_int, P(C.c_void_p), P(C.c_size_t), C.c_int, C.c_int]
        L.orc16_tables.argtypes = [C.c_void_p] * 4
        L.orc16_mul.argtypes = [C.c_void_p, C.c_void_p, C.c_uint16, C.c_size_t]
        L.orc16_mul_log.argtypes = [C.c_uint16, C.c_uint16]
        L.orc16_mul_log.restype = C.c_uint16
        L.orc8_new.argtypes = [C.c_int, C.c_int, P(C.c_int)]
        L.orc8_new.restype = C.c_void_p
        L.orc8_free.argtypes = [C.c_void_p]
        L.orc8_encode.argtypes = [C.c_void_p, P(C.c_void_p), P(C.c_size_t), C.c_int]
        L.orc8_verify.argtypes = [C.c_void_p, P(C.c_void_p), P(C.c_size_t), C.c_int, P(C.c_int)]
        L.orc8_reconstruct.argtypes = [C.c_void_p, P(C.c_void_p), P(C.c_size_t), C.c_int, C.c_int]
        L.orc8_tables.argtypes = [C.c_void_p] * 4
        L.orc8_mul.argtypes = [C.c_void_p, C.c_void_p, C.c_uint8, C.c_size_t]
        L.orc8_mul_log.argtypes = [C.c_uint8, C.c_uint8]
        L.orc8_mul_log.restype = C.c_uint8
        L.orc16_encode_simd.argtypes = [C.c_int, C.c_int, P(C.c_void_p), C.c_size_t, C.c_int]
        L.orc16_encode_simd_isa.argtypes = [C.c_int, C.c_int, C.c_int, P(C.c_void_p), C.c_size_t, C.c_int]
        L.orc16_simd_available.restype = C.c_int
        if L.orc_init() != 0:
            raise MemoryError("oracle table init failed")
        _lib = L
    return _lib


def _ptrs(shards):
    arr = (C.c_void_p * len(shards))()
    lens = (C.c_size_t * len(shards))()
    for i, s in enumerate(shards):
        if s is None:
            arr[i] = None
            lens[i] = 0
        else:
            arr[i] = s.ctypes.data
            lens[i] = s.nbytes
    return arr, lens


class Oracle:
    """Reference-shaped codec over numpy uint8 shards (oracle, not product)."""

    def __init__(self, bits: int, k: int, p: int):
        self.bits, self.k, self.p = bits, k, p
        self._h = None
        L = lib()
        if bits == 8:
            err = C.c_int(0)
            self._h = L.orc8_new(k, p, C.byref(err))
            self.err = err.value
        else:
            self.err = 0 if (k > 0 and p > 0 and k + p <= 65536) else (1 if (k <= 0 or p <= 0) else 2)

    def __del__(self):
        if self._h and _lib is not None:
            _lib.orc8_free(self._h)
            self._h = None

    def encode(self, shards) -> int:
        """Writes parity into shards[k:] in place; returns the error code."""
        arr, lens = _ptrs(shards)
        L = lib()
        if self.bits == 8:
            return L.orc8_encode(self._h, arr, lens, len(shards))
        return L.orc16_encode(self.k, self.p, arr, lens, len(shards))

    def verify(self, shards):
        arr, lens = _ptrs(shards)
        ok = C.c_int(0)
        L = lib()
        if self.bits == 8:
            e = L.orc8_verify(self._h, arr, lens, len(shards), C.byref(ok))
        else:
            e = L.orc16_verify(self.k, self.p, arr, lens, len(shards), C.byref(ok))
        return bool(ok.value), e

    def reconstruct(self, shards, recover_all: bool = True):
        """shards: list of uint8 arrays or None.  Returns (err, shards) with
        recovered shards filled in (new arrays) like the Go slice resize."""
        S = next((s.nbytes for s in shards if s is not None), 0)
        bufs = [s if s is not None else np.zeros(S, dtype=np.uint8) for s in shards]
        arr = (C.c_void_p * len(shards))()
        lens = (C.c_size_t * len(shards))()
        for i, s in enumerate(shards):
            arr[i] = bufs[i].ctypes.data if bufs[i].nbytes else None
            lens[i] = 0 if s is None else s.nbytes
        L = lib()
        if self.bits == 8:
            e = L.orc8_reconstruct(self._h, arr, lens, len(shards), int(recover_all))
        else:
            e = L.orc16_reconstruct(self.k, self.p, arr, lens, len(shards), int(recover_all))
        out = [bufs[i] if lens[i] else None for i in range(len(shards))]
        return e, out


def tables16():
    L = lib()
    log = np.zeros(65536, np.uint16)
    exp = np.zeros(65536, np.uint16)
    skew = np.zeros(65535, np.uint16)
    walsh = np.zeros(65536, np.uint16)
    L.orc16_tables(log.ctypes.data, exp.ctypes.data, skew.ctypes.data, walsh.ctypes.data)
    return log, exp, skew, walsh


def tables8():
    L = lib()
    log = np.zeros(256, np.uint8)
    exp = np.zeros(256, np.uint8)
    skew = np.zeros(255, np.uint8)
    walsh = np.zeros(256, np.uint8)
    L.orc8_tables(log.ctypes.data, exp.ctypes.data, skew.ctypes.data, walsh.ctypes.data)
    return log, exp, skew, walsh


def encode(bits: int, k: int, p: int, data: np.ndarray) -> np.ndarray:
    """Convenience: data (k,S) uint8 -> parity (p,S) uint8 via the C oracle."""
    S = data.shape[1]
    shards = [np.ascontiguousarray(data[i]) for i in range(k)] + [np.zeros(S, np.uint8) for _ in range(p)]
    o = Oracle(bits, k, p)
    e = o.encode(shards)
    if e != 0:
        raise RuntimeError(f"oracle encode error {e}")
    return np.stack(shards[k:])


SIMD_ISAS = {"avx2": 1, "avx512": 2}


def simd_available() -> bool:
    return bool(lib().orc16_simd_available())


def simd_isas() -> list:
    """ISAs of the SIMD port this CPU runs ("avx2", "avx512")."""
    m = lib().orc16_simd_available()
    return [n for n, b in SIMD_ISAS.items() if m & b]


def encode_simd(k: int, p: int, data: np.ndarray, threads: int = 1, parity: np.ndarray = None, isa: str = None) -> np.ndarray:
    """GF(2^16) encode with the reference-equivalent SIMD port (leopard_ref.c,
    CPU baseline only): data (k,S) uint8 -> parity (p,S); `threads` byte
    ranges; isa "avx2" / "avx512" (None: the widest the CPU runs)."""
    S = data.shape[1]
    if parity is None:
        parity = np.zeros((p, S), np.uint8)
    arr = (C.c_void_p * (k + p))(*([data[i].ctypes.data for i in range(k)] + [parity[i].ctypes.data for i in range(p)]))
    e = lib().orc16_encode_simd_isa(SIMD_ISAS[isa] if isa else 0, k, p, arr, S, threads)
    if e != 0:
        raise RuntimeError(f"simd encode error {e}")
    return parity
