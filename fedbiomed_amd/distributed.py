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
from typing import Optional, Tuple


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


DEFAULT_TIMEOUT_S = 120.0


def pg_timeout():
    """The process group's collective timeout: FBM_DIST_TIMEOUT_S seconds (default 120).  torch's
    default for NCCL is 10 min -- as long as the driver's whole bench limit, so a collective stuck in
    an 8-GPU run would be killed at that limit with no line written.  Bounded, a stuck collective
    raises (gloo) or is aborted by the NCCL watchdog, and the rank exits non-zero well inside it."""
    from datetime import timedelta

    return timedelta(seconds=float(os.environ.get("FBM_DIST_TIMEOUT_S", DEFAULT_TIMEOUT_S)))


def init(backend: str = "nccl", device: Optional[int] = None):
    """One process per GPU; backend "nccl" is RCCL on ROCm (gloo for CPU tests).
    `device` overrides LOCAL_RANK as the rank's GPU (rehearsals with shared devices).
    Collectives time out after pg_timeout()."""
    import torch
    import torch.distributed as dist

    rank, world, local = env_rank()
    if device is not None:
        local = device
    if world > 1 and not dist.is_initialized():
        if backend == "nccl":
            torch.cuda.set_device(local)
            # a timed-out RCCL collective tears the process down instead of hanging in it
            os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
        dist.init_process_group(backend=backend, rank=rank, world_size=world, timeout=pg_timeout())
    return rank, world, local


def run_rank(fn, *args, **kw):
    """Runs one rank's body; if it raises, prints the traceback and ends the PROCESS at once with
    status 1 (os._exit: no interpreter shutdown, which could wait on a collective or the process
    group's teardown).  Its peers then fail their next collective within pg_timeout() and exit
    non-zero too; under torch.distributed.run the elastic agent stops them as soon as this rank
    exits, under bench.py's own spawn_ranks the parent does."""
    import sys
    import traceback

    try:
        return fn(*args, **kw)
    except SystemExit:  # a deliberate exit keeps its status
        raise
    except BaseException:  # noqa: BLE001 -- any failure of a rank ends the run
        traceback.print_exc()
        sys.stderr.flush()
        sys.stdout.flush()
        os._exit(1)


# ------------------------------------------------------------------------------------------
# party-per-rank exchange (the one real collective of the path)
#
# In a deployment each party's update is encrypted on its own node; when several parties'
# encrypted updates sit on different GPUs of one node (one rank each), the aggregate needs
# every party's value at every index.  The exchange is then:
#   LOM: sum the local parties' masked u64 vectors on the device (the LOM aggregate is a
#        plain sum mod 2^64), then ONE reduce-scatter over ranks (u64 sum == int64 sum mod
#        2^64, two's complement) leaves rank r with the global masked sum of stripe r ->
#        average + dequantise locally -> all-gather the float64 stripes.
#   JL:  the ciphertext product is not an RCCL reduction, so ranks all-to-all their
#        parties' ciphertexts by ciphertext stripe (256 B each), then each rank aggregates
#        its stripe with ct_offset and the float64 stripes are all-gathered.
# Backend "nccl" is RCCL over xGMI on the GPU box; the same code runs on gloo (CPU tensors)
# in the tests.  gloo lacks reduce_scatter, so it takes all-reduce + slice.
# ------------------------------------------------------------------------------------------
def _dist():
    import torch.distributed as dist

    return dist


def stripe_bounds(n_total: int, world: int, align: int):
    """Equal-capacity stripes for collectives: (per_rank_capacity, [(lo, hi) per rank])."""
    per = -(-n_total // world)
    per = -(-per // align) * align
    return per, [(min(r * per, n_total), min((r + 1) * per, n_total)) for r in range(world)]


def reduce_scatter_u64(local_sum, n_total: int):
    """Global mod-2^64 sum of every rank's `local_sum` (int64 [n_total], u64 bit patterns);
    returns this rank's stripe (8-aligned, see stripe_bounds)."""
    import torch

    dist = _dist()
    world, rank = dist.get_world_size(), dist.get_rank()
    per, bounds = stripe_bounds(n_total, world, 8)
    lo, hi = bounds[rank]
    if dist.get_backend() == "nccl":
        buf = torch.zeros(per * world, dtype=torch.int64, device=local_sum.device)
        buf[:n_total] = local_sum
        out = torch.empty(per, dtype=torch.int64, device=local_sum.device)
        dist.reduce_scatter_tensor(out, buf, op=dist.ReduceOp.SUM)
        return out[: hi - lo]
    buf = torch.zeros(per * world, dtype=torch.int64)  # gloo: host tensors, all-reduce + slice
    buf[:n_total] = local_sum.cpu()
    dist.all_reduce(buf, op=dist.ReduceOp.SUM)
    return buf[lo:hi].clone().to(local_sum.device)


def all_gather_stripes(stripe, n_total: int, align: int):
    """Inverse of the stripe split: every rank gets the full [n_total] vector."""
    import torch

    dist = _dist()
    world, rank = dist.get_world_size(), dist.get_rank()
    per, bounds = stripe_bounds(n_total, world, align)
    host = dist.get_backend() != "nccl"  # gloo: host tensors
    buf = torch.zeros(per, dtype=stripe.dtype, device="cpu" if host else stripe.device)
    buf[: stripe.numel()] = stripe.cpu() if host else stripe
    out = torch.empty(per * world, dtype=stripe.dtype, device=buf.device)
    dist.all_gather_into_tensor(out, buf)
    full = torch.cat([out[r * per: r * per + (hi - lo)] for r, (lo, hi) in enumerate(bounds)])
    return full.to(stripe.device) if host else full


def all_gather_shards(stripe, n_total: int, align: int):
    """The element-range split's final gather: every rank's output stripe (its
    shard_range(n_total, world, rank, align) elements) -> the whole [n_total] vector on every
    rank, one all-gather (RCCL over xGMI with "nccl"; host tensors with gloo)."""
    import torch

    dist = _dist()
    world = dist.get_world_size()
    bounds = [shard_range(n_total, world, r, align) for r in range(world)]
    per = max(hi - lo for lo, hi in bounds)
    dev = stripe.device
    host = dist.get_backend() != "nccl"
    buf = torch.zeros(per, dtype=stripe.dtype, device="cpu" if host else dev)
    buf[: stripe.numel()] = stripe.cpu() if host else stripe
    out = torch.empty(per * world, dtype=stripe.dtype, device=buf.device)
    dist.all_gather_into_tensor(out, buf)
    full = torch.cat([out[r * per: r * per + (hi - lo)] for r, (lo, hi) in enumerate(bounds)])
    return full.to(dev) if host else full


def all_to_all_ciphertexts(cts_local, parties_per_rank: int):
    """cts_local: [P_local, n_ct, 64] int32 limbs of this rank's parties (whole vector).
    Returns ([P_total, stripe_ct, 64] int32, ct_offset) = every party's ciphertexts for this
    rank's ciphertext stripe; party order = rank-major (rank 0's parties first)."""
    import torch

    dist = _dist()
    world, rank = dist.get_world_size(), dist.get_rank()
    P_local, n_ct, W = cts_local.shape
    if P_local != parties_per_rank:
        raise ValueError("every rank must hold the same number of parties")
    per, bounds = stripe_bounds(n_ct, world, 1)
    host = dist.get_backend() != "nccl"  # gloo: host tensors
    # ct-major, padded to equal stripes: rows [r*per, (r+1)*per) go to rank r
    send = torch.zeros((per * world, P_local, W), dtype=cts_local.dtype, device="cpu" if host else cts_local.device)
    send[:n_ct] = (cts_local.cpu() if host else cts_local).permute(1, 0, 2)
    recv = torch.empty_like(send)
    dist.all_to_all_single(recv, send)
    lo, hi = bounds[rank]
    # recv block s = source rank s's parties for my stripe: [per, P_local, W]
    recv = recv.view(world, per, P_local, W)[:, : hi - lo]
    out = recv.permute(0, 2, 1, 3).reshape(world * P_local, hi - lo, W).contiguous()
    return (out.to(cts_local.device) if host else out), lo
