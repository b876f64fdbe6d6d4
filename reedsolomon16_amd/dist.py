"""Multi-GPU layout: byte-range sharding of a stripe.

Every GF(2^w) operation of the Leopard codec acts independently on each
64-byte column block of the shards (leopard16.go:778-792; the GF(2^8) path
even processes 32 KiB column chunks independently, leopard8.go:198-274).  So
GPU g of G owns bytes [lo_g, hi_g) of *every* shard (64-byte granular) and
encodes / verifies / reconstructs its slice with no data exchange.  The only
collective is a one-word MIN over ranks for Verify (control plane).

One process per GPU (torch.distributed, RCCL backend "nccl" on ROCm, or gloo
on CPU for tests).  The per-rank codec call is injectable so the partition
logic is testable without a GPU; on the GPU it is the engine's device entry
point (``ReedSolomon.encode_dev`` etc.).
"""
from __future__ import annotations

from typing import Callable, Optional, Sequence, Tuple

BLOCK = 64  # GF(2^16) symbol block: 32 low bytes + 32 high bytes (leopard16.go:778-792)


def byte_range(shard_size: int, rank: int, world: int, align: int = BLOCK) -> Tuple[int, int]:
    """[lo, hi) of the shard bytes owned by `rank`: 64-byte blocks dealt as
    evenly as possible (the first `blocks % world` ranks get one extra)."""
    if shard_size % align:
        raise ValueError("shard size must be a multiple of %d" % align)
    if not 0 <= rank < world:
        raise ValueError("bad rank")
    blocks = shard_size // align
    base, extra = divmod(blocks, world)
    lo = rank * base + min(rank, extra)
    hi = lo + base + (1 if rank < extra else 0)
    return lo * align, hi * align


def local_rows(rows, rank: int, world: int):
    """Column slice [lo, hi) of every row of a [k+p, S] array/tensor (views)."""
    S = rows.shape[1]
    lo, hi = byte_range(S, rank, world)
    return rows[:, lo:hi]


def encode_sharded(rows, rank: int, world: int, encode_fn: Callable) -> None:
    """Encode this rank's byte range of the stripe in place (no collective).
    encode_fn(local_rows) fills the parity rows of the slice."""
    loc = local_rows(rows, rank, world)
    if loc.shape[1]:
        encode_fn(loc)


def reconstruct_sharded(rows, present: Sequence[bool], rank: int, world: int, reconstruct_fn: Callable) -> None:
    """Rebuild missing rows of this rank's byte range (same erasure pattern on every rank)."""
    loc = local_rows(rows, rank, world)
    if loc.shape[1]:
        reconstruct_fn(loc, present)


def verify_sharded(rows, rank: int, world: int, verify_fn: Callable, group=None, device: Optional[str] = None) -> bool:
    """Verify this rank's slice and AND the answers of all ranks (one-word MIN)."""
    import torch
    import torch.distributed as dist

    loc = local_rows(rows, rank, world)
    ok = bool(verify_fn(loc)) if loc.shape[1] else True
    if world > 1:
        t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=device or "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
        ok = bool(t.item())
    return ok


def gpu_encode_fn(codec, stream=None):
    """Per-rank encode through the engine: the [k+p, hi-lo] slice view goes to
    the C-ABI as base + row stride (no per-row host objects)."""
    def fn(loc):
        codec.encode_dev(loc, stream)
    return fn


def gpu_verify_fn(codec, stream=None):
    def fn(loc):
        return codec.verify_dev(loc, stream)
    return fn


def gpu_reconstruct_fn(codec, recover_all: bool = True, stream=None):
    def fn(loc, present):
        codec.reconstruct_dev(loc, present, recover_all, stream)
    return fn


def local_stripes(slab, rank: int, world: int):
    """Column slice [lo, hi) of every row of every stripe of a [n, k+p, S] slab (a view)."""
    lo, hi = byte_range(slab.shape[2], rank, world)
    return slab[:, :, lo:hi]


def encode_sharded_batch(slab, rank: int, world: int, codec, stream=None) -> None:
    """Encode this rank's byte range of n stripes in one launch
    (rs_encode_dev_batch over the strided view; no collective)."""
    loc = local_stripes(slab, rank, world)
    if loc.shape[2]:
        codec.encode_dev_batch(loc, stream)


def reconstruct_sharded_batch(slab, present: Sequence[bool], rank: int, world: int, codec, recover_all: bool = True,
                              stream=None) -> None:
    """Rebuild this rank's byte range of the missing shards of n stripes with
    one erasure pattern (a lost device) in one launch (rs_reconstruct_dev_batch
    over the strided view; no collective: every rank holds the same pattern)."""
    loc = local_stripes(slab, rank, world)
    if loc.shape[2]:
        codec.reconstruct_dev_batch(loc, present, recover_all, stream)
