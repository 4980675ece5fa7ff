"""Element-range sharding across the GPUs of one node.

Every element of the secagg path depends only on its global index: LOM element i uses
ChaCha20 block i // 8 and (i + tau); JL ciphertext k uses t_k = (k << 512) | tau.  So
the vector is cut into contiguous stripes -- on 8-element boundaries for LOM, on
ciphertext (cr-element) boundaries for JL -- one per rank (one process per GPU), each
stripe processed with its global offset and no data-path collective.  The concatenation
of the stripes' results is bit-identical to the unsharded result.
"""

from __future__ import annotations

import os
from typing import Tuple


def shard_range(n_total: int, world: int, rank: int, align: int) -> Tuple[int, int]:
    """[start, stop) of rank's stripe; start is a multiple of `align`, stripes tile [0, n)."""
    if world < 1 or not 0 <= rank < world or align < 1:
        raise ValueError("bad shard arguments")
    units = (n_total + align - 1) // align
    per, extra = divmod(units, world)
    u0 = rank * per + min(rank, extra)
    u1 = u0 + per + (1 if rank < extra else 0)
    return min(u0 * align, n_total), min(u1 * align, n_total)


def lom_shard(n_total: int, world: int, rank: int) -> Tuple[int, int]:
    return shard_range(n_total, world, rank, 8)


def jl_shard(n_total: int, world: int, rank: int, cr: int) -> Tuple[int, int]:
    """Element stripe on ciphertext boundaries; the stripe's first ciphertext index is start // cr."""
    return shard_range(n_total, world, rank, cr)


def env_rank() -> Tuple[int, int, int]:
    """(rank, world_size, local_rank) from the torch.distributed.run environment."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def init(backend: str = "nccl"):
    """One process per GPU; backend "nccl" is RCCL on ROCm (gloo for CPU tests)."""
    import torch
    import torch.distributed as dist

    rank, world, local = env_rank()
    if world > 1 and not dist.is_initialized():
        if backend == "nccl":
            torch.cuda.set_device(local)
        dist.init_process_group(backend=backend, rank=rank, world_size=world)
    return rank, world, local
