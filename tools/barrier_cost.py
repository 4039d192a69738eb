"""Cost of the barrier that closes bench.py's timed region, per form, in a
process group launched like the bench (RCCL backend, any world size):
  nccl_barrier   dist.barrier(device_ids=[local])      (round-2 bench)
  nccl_allreduce all_reduce of a preallocated 1-element device tensor + sync
  gloo_barrier   barrier of a gloo side group (host TCP) after the stream sync
usage: WCE-style env (RANK/WORLD_SIZE/LOCAL_RANK/MASTER_*) python tools/barrier_cost.py"""
import os
import time

import torch
import torch.distributed as dist

local = int(os.environ.get("LOCAL_RANK", "0"))
torch.cuda.set_device(local)
dist.init_process_group("nccl", device_id=torch.device("cuda", local))
g = dist.new_group(backend="gloo")
t = torch.zeros(1, device="cuda")


def nccl_barrier():
    dist.barrier(device_ids=[local])


def nccl_allreduce():
    dist.all_reduce(t)
    torch.cuda.synchronize()


def gloo_barrier():
    dist.barrier(group=g)


for name, fn in (("nccl_barrier", nccl_barrier), ("nccl_allreduce", nccl_allreduce), ("gloo_barrier", gloo_barrier)):
    for _ in range(5):
        fn()
    xs = []
    for _ in range(50):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        xs.append(time.perf_counter() - t0)
    xs.sort()
    if dist.get_rank() == 0:
        print(f"world {dist.get_world_size()} {name:15s} median {xs[25] * 1e6:8.1f} us  min {xs[0] * 1e6:8.1f}  "
              f"max {xs[-1] * 1e6:8.1f}", flush=True)
dist.destroy_process_group()
