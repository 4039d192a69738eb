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


# ---- native C-ABI path (include/wce.h wce_comm_*): RCCL driven from libwce
# itself, for hosts without torch.distributed (the MPI model of main_mpi.c).
COMM_ID_BYTES = 128


def native_shard(wce, total: int, world: int, rank: int):
    """wce_shard through the C ABI (same partition as shard())."""
    import ctypes

    first, count = ctypes.c_int64(), ctypes.c_int64()
    rc = wce.load().wce_shard(total, world, rank, ctypes.byref(first), ctypes.byref(count))
    if rc != 0:
        raise wce.WceError(rc, "wce_shard")
    return first.value, count.value


class NativeComm:
    """One RCCL communicator owned by libwce (wce_comm).  Rank 0 makes the
    unique id with unique_id(); the host hands its bytes to every rank (any
    channel: MPI, a file, a socket, a torch.distributed broadcast)."""

    def __init__(self, wce, uid: bytes, nranks: int, rank: int, device: int = 0, handle=None):
        import ctypes

        self._wce = wce
        self.handle = ctypes.c_void_p(handle)
        if handle is None:
            if len(uid) != COMM_ID_BYTES:
                raise ValueError("unique id must be %d bytes" % COMM_ID_BYTES)
            buf = ctypes.create_string_buffer(uid, COMM_ID_BYTES)
            rc = wce.load().wce_comm_init_rank(ctypes.byref(self.handle), buf, nranks, rank, device)
            if rc != 0:
                raise wce.WceError(rc, "wce_comm_init_rank")

    @staticmethod
    def unique_id(wce) -> bytes:
        import ctypes

        buf = ctypes.create_string_buffer(COMM_ID_BYTES)
        rc = wce.load().wce_comm_unique_id(buf)
        if rc != 0:
            raise wce.WceError(rc, "wce_comm_unique_id")
        return buf.raw

    @classmethod
    def init_all(cls, wce, devices):
        """One communicator per listed device, all in this process."""
        import ctypes

        n = len(devices)
        hs = (ctypes.c_void_p * n)()
        devs = (ctypes.c_int * n)(*devices)
        rc = wce.load().wce_comm_init_all(hs, n, devs)
        if rc != 0:
            raise wce.WceError(rc, "wce_comm_init_all")
        return [cls(wce, b"", n, i, devices[i], handle=hs[i]) for i in range(n)]

    def info(self):
        import ctypes

        r, n, d = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        rc = self._wce.load().wce_comm_info(self.handle, ctypes.byref(r), ctypes.byref(n), ctypes.byref(d))
        if rc != 0:
            raise self._wce.WceError(rc, "wce_comm_info")
        return r.value, n.value, d.value

    def broadcast_state(self, ctx, root: int = 0, stream=None):
        """ONE in-place RCCL broadcast of ctx's state from root (ctx may be
        empty on the other ranks); returns once ctx is valid."""
        rc = self._wce.load().wce_ctx_broadcast_state(ctx.handle, self.handle, root, stream)
        if rc != 0:
            raise self._wce.WceError(rc, "wce_ctx_broadcast_state")

    def max_f64(self, value: float, stream=None) -> float:
        import ctypes

        v = ctypes.c_double(value)
        rc = self._wce.load().wce_comm_max_f64(self.handle, ctypes.byref(v), stream)
        if rc != 0:
            raise self._wce.WceError(rc, "wce_comm_max_f64")
        return v.value

    def close(self):
        if self.handle is not None and self.handle.value:
            self._wce.load().wce_comm_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def broadcast_state_all(wce, ctxs, comms, root: int = 0):
    """The grouped broadcast for one process driving several GPUs."""
    import ctypes

    n = len(ctxs)
    cs = (ctypes.c_void_p * n)(*[c.handle.value for c in ctxs])
    ms = (ctypes.c_void_p * n)(*[m.handle.value for m in comms])
    rc = wce.load().wce_ctx_broadcast_state_all(cs, ms, n, root, None)
    if rc != 0:
        raise wce.WceError(rc, "wce_ctx_broadcast_state_all")
