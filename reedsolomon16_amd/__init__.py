"""reedsolomon16_amd — MI355X-native Leopard-FFT Reed-Solomon engine.

Drop-in for the hot path of bpfs/reedsolomon16 (leopard16.go / leopard8.go):
hand-written CDNA4 HIP kernels behind the C-ABI in include/rs_mi355x.h, with
this package as the host-side mirror of the reference's ReedSolomon interface.
"""
from .codec import (  # noqa: F401
    New,
    New8,
    New16,
    ReedSolomon,
    RSError,
    ErrInvShardNum,
    ErrMaxShardNum,
    ErrTooFewShards,
    ErrShardNoData,
    ErrShardSize,
    ErrInvalidShardSize,
    ErrNotSupported,
    ErrShortData,
    ErrReconstructRequired,
    ErrNilWriter,
    ErrSize,
    ErrPanic,
    ErrDevice,
    alloc_pinned,
    EmptyShard,
)
from ._capi import LIB_PATH, lib  # noqa: F401

__all__ = [
    "New", "New8", "New16", "ReedSolomon", "RSError", "ErrInvShardNum", "ErrMaxShardNum", "ErrTooFewShards",
    "ErrShardNoData", "ErrShardSize", "ErrInvalidShardSize", "ErrNotSupported", "ErrShortData",
    "ErrReconstructRequired", "ErrNilWriter", "ErrSize", "ErrPanic", "ErrDevice", "LIB_PATH", "lib", "alloc_pinned",
    "EmptyShard",
]
