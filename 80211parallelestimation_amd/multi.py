"""Multi-GPU plumbing: frame sharding and the single shared-state broadcast.

Frames are independent, so a batch is partitioned over ranks (one process
per GPU) with no data-path collective.  The only exchange is one broadcast
of the packed shared state (wce::State: C, H_LT, tx_pre, sinc table, MMSE
coefficients, per-frame covariance operators; ~260 KB) from the rank that built it -- the analogue of the
reference's MPI_Bcast of F/Ryy (main_mpi.c:687-688, 727-728).  With the
"nccl" backend torch.distributed is RCCL over xGMI; "gloo" is used by the
CPU tests.
"""
from __future__ import annotations

import numpy as np


def shard(total: int, world: int, rank: int):
    """Contiguous frame range [first, first + count) of `rank` (strong scaling:
    the first total % world ranks take one extra frame)."""
    if world <= 0 or not 0 <= rank < world or total < 0:
        raise ValueError("bad shard arguments")
    base, extra = divmod(total, world)
    first = rank * base + min(rank, extra)
    return first, base + (1 if rank < extra else 0)


def weak_shard(per_rank: int, rank: int):
    """Weak scaling: every rank owns per_rank frames, global index offset."""
    return rank * per_rank, per_rank


def broadcast_state_host(dist, blob, nbytes: int, src: int = 0, group=None):
    """Broadcast a host state blob (numpy uint8, only needed on src) with a
    CPU-tensor backend (gloo).  Returns the blob on every rank."""
    import torch

    t = torch.empty(nbytes, dtype=torch.uint8)
    if dist.get_rank(group) == src:
        t.copy_(torch.from_numpy(np.ascontiguousarray(blob, dtype=np.uint8)))
    dist.broadcast(t, src=src, group=group)
    return t.numpy().copy()


def state_to_buffer(wce, ctx, buf=None):
    """Copy ctx's device-resident state into a torch uint8 CUDA tensor (the
    buffer RCCL sends).  Device to device."""
    import torch

    ptr, nbytes = ctx.state()
    if buf is None:
        buf = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    if buf.numel() != nbytes or not buf.is_cuda:
        raise ValueError("broadcast buffer must be a CUDA uint8 tensor of wce_state_size() bytes")
    torch.cuda.synchronize()
    if wce.load().wce_memcpy_dtod(buf.data_ptr(), ptr, nbytes, None) != 0:
        raise wce.WceError(-2, "state -> broadcast buffer")
    return buf


def buffer_to_state(wce, buf, ctx):
    """Install a received state buffer into ctx (an empty context is fine)
    and mark it ready.  Device to device."""
    import torch

    ptr, nbytes = ctx.state()
    if buf.numel() != nbytes or not buf.is_cuda:
        raise ValueError("broadcast buffer must be a CUDA uint8 tensor of wce_state_size() bytes")
    torch.cuda.synchronize()
    if wce.load().wce_memcpy_dtod(ptr, buf.data_ptr(), nbytes, None) != 0:
        raise wce.WceError(-2, "broadcast buffer -> state")
    ctx.mark_ready()


def broadcast_state_device(dist, wce, ctx, src: int = 0, group=None):
    """ONE RCCL broadcast of ctx's device-resident state from src into every
    other rank's context (which may be an empty context).  Device to device:
    the state never goes back through the host."""
    import torch

    rank = dist.get_rank(group)
    if rank == src:
        buf = state_to_buffer(wce, ctx)
    else:
        buf = torch.empty(ctx.state()[1], dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    dist.broadcast(buf, src=src, group=group)
    torch.cuda.synchronize()
    if rank != src:
        buffer_to_state(wce, buf, ctx)
    return buf.numel()
