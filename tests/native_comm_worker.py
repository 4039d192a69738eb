"""Worker for tests/test_multi_gpu.py::test_native_rccl_path: the C-ABI
multi-GPU path (include/wce.h wce_comm_*) with no torch in the process --
libwce loads RCCL itself, as a C or MPI host would use it.

One GPU holds one RCCL rank, so this runs the one-rank forms of both launch
models: wce_comm_unique_id + wce_comm_init_rank (process per GPU) and
wce_comm_init_all (one process, several GPUs).  Each broadcasts a built
context's state in place; its estimates must be bit-identical.
Prints one JSON line."""
import importlib
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def run_case(wce, inp, mode, bcast):
    """A one-rank group's broadcast is the root side only (its buffer is the
    only buffer): the state must come through byte-identical and the context
    must estimate exactly as before it.  The bytes reaching other ranks are
    the multi-rank case (gloo on CPU, the driver's 2/4/8-GPU runs)."""
    ctx = wce.Context(inp["tx_pre"], inp["rx_pre"], inp["ow2"], mode, device=0)
    ptr, nb = ctx.state()
    blob = np.empty(nb, np.uint8)
    assert wce.load().wce_memcpy_dtoh(blob.ctypes.data, ptr, nb) == 0
    B = 64
    tx = np.repeat(inp["tx_symb"][None], B, axis=0)
    rx = np.repeat(inp["rx_symb"][None], B, axis=0) * (1.0 + 0.01 * np.arange(B))[:, None, None]
    a = ctx.estimate_host(tx, rx, mask=wce.ALL)
    bcast(ctx)
    b = ctx.estimate_host(tx, rx, mask=wce.ALL)
    after = np.empty(nb, np.uint8)
    assert wce.load().wce_memcpy_dtoh(after.ctypes.data, ptr, nb) == 0
    return {"bytes": int(nb), "root_unchanged": bool(np.array_equal(after, blob)),
            "bit_identical": bool(all(np.array_equal(a[k], b[k]) for k in a)),
            "finite": bool(all(np.isfinite(a[k]).all() for k in a))}


def main():
    wce = importlib.import_module("80211parallelestimation_amd")
    multi = importlib.import_module("80211parallelestimation_amd.multi")
    inp = dict(np.load(os.path.join(REPO, "tests", "golden", "inputs_h.npz")))
    res = {}
    uid = multi.NativeComm.unique_id(wce)
    comm = multi.NativeComm(wce, uid, 1, 0, 0)
    res["info"] = list(comm.info())
    for name, mode in (("textbook", wce.MMSE_TEXTBOOK), ("ref", wce.MMSE_REF)):
        res["rank_" + name] = run_case(wce, inp, mode, lambda c: comm.broadcast_state(c, 0))
    res["max"] = comm.max_f64(3.5)
    # root with no valid state is refused
    empty = wce.Context(empty=True, device=0)
    try:
        comm.broadcast_state(empty, 0)
        res["empty_root_refused"] = False
    except wce.WceError:
        res["empty_root_refused"] = True
    comm.close()
    comms = multi.NativeComm.init_all(wce, [0])
    res["all_info"] = list(comms[0].info())
    res["all_ref"] = run_case(wce, inp, wce.MMSE_REF,
                              lambda c: multi.broadcast_state_all(wce, [c], comms, 0))
    for c in comms:
        c.close()
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
