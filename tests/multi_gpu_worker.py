"""Worker for tests/test_multi_gpu.py (run as its own process, so torch's HIP
runtime is loaded before libwce, as in bench.py's distributed path).

Runs the RCCL ("nccl" backend) state broadcast in a one-rank group on one
GPU and checks that a context filled from the broadcast buffer estimates
bit-identically to the context that built the state.  Prints one JSON line.
"""
import importlib
import json
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    wce = importlib.import_module("80211parallelestimation_amd")
    multi = importlib.import_module("80211parallelestimation_amd.multi")
    inp = dict(np.load(os.path.join(REPO, "tests", "golden", "inputs_h.npz")))
    res = {}
    try:
        for name, mode in (("textbook", wce.MMSE_TEXTBOOK), ("ref", wce.MMSE_REF)):
            src = wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], mode, device=0)
            nb = multi.broadcast_state_device(dist, wce, src, src=0)      # the src side of bench.py's call
            buf = multi.state_to_buffer(wce, src)
            dist.broadcast(buf, src=0)
            dst = wce.Context(empty=True, device=0)
            multi.buffer_to_state(wce, buf, dst)
            B = 96
            tx = np.repeat(inp["tx_symb"][None], B, axis=0)
            rx = np.repeat(inp["rx_symb"][None], B, axis=0) * (1.0 + 0.01 * np.arange(B))[:, None, None]
            a = src.estimate_host(tx, rx, mask=wce.ALL)
            b = dst.estimate_host(tx, rx, mask=wce.ALL)
            same = all(np.array_equal(a[k], b[k]) for k in a)
            res[name] = {"bytes": nb, "bit_identical": bool(same),
                         "finite": bool(all(np.isfinite(a[k]).all() for k in a))}
        t = torch.tensor([3.5], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dist.barrier(device_ids=[0])
        res["allreduce_max"] = float(t.item())
    finally:
        dist.destroy_process_group()
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
