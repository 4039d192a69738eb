"""bench.py --gpus N without a launcher starts N ranks itself (CPU: gloo, the
--dry-run control path that never touches a device).  The driver's N-GPU
command may or may not wrap bench.py in torch.distributed.run; either way the
line must span N ranks or the run must fail (main_mpi.c:16-27, 687-688: the
reference's mpirun world is what its timing covers)."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, timeout=240, **env):
    e = dict(os.environ, WCE_DIST_BACKEND="gloo", OMP_NUM_THREADS="1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env)
    return subprocess.run([sys.executable, os.path.join(REPO, "bench.py")] + args, capture_output=True, text=True,
                          timeout=timeout, env=e, cwd=REPO)


def _line(p):
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    assert p.stdout.rstrip().endswith(lines[0])        # the line is the last thing on stdout
    return json.loads(lines[0])


@pytest.mark.parametrize("n", [2, 3])
def test_gpus_n_spawns_n_ranks(n):
    p = _run(["--gpus", str(n), "--dry-run", "--steps", "7", "--warmup", "2"])
    assert p.returncode == 0, p.stderr[-3000:]
    r = _line(p)
    assert r["n_gpus"] == n and r["dry_run"] is True
    assert r["dist_check"] == {"backend": "gloo", "world_size_env": n, "group_size": n, "all_ranks_agree": True}
    assert r["steps"] == 7 and r["warmup"] == 2
    assert r["config"]["global_frames"] == n * r["config"]["frames_per_gpu"]
    assert "launching %d ranks" % n in p.stderr
    assert r["launcher"] == "bench.py --gpus %d" % n


def test_rank_failure_fails_the_run():
    p = _run(["--gpus", "2", "--dry-run"], WCE_DRY_FAIL_RANK="1")
    assert p.returncode != 0
    assert not [ln for ln in p.stdout.splitlines() if ln.startswith("{")]


def test_world_size_must_equal_gpus():
    p = _run(["--gpus", "1", "--dry-run"], WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    assert p.returncode == 2 and "WORLD_SIZE=2 but --gpus 1" in p.stderr
    p = _run(["--gpus", "8", "--dry-run"], WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    assert p.returncode == 2


def test_single_rank_dry_run_needs_no_launcher():
    p = _run(["--dry-run"])
    assert p.returncode == 0, p.stderr[-2000:]
    r = _line(p)
    assert r["n_gpus"] == 1 and r["dist_check"]["group_size"] == 1
    assert "launching" not in p.stderr and r["launcher"] is None


def test_launcher_parent_never_imports_torch():
    """The parent must not initialise a GPU before its children start (an exec
    or fork after HIP init is forbidden on the pool): check_world runs before
    anything imports torch."""
    src = open(os.path.join(REPO, "bench.py")).read()
    main = src[src.index("def main():"):]
    assert main.index("check_world(") < main.index("Dist()")
    head = src[:src.index("def main():")]
    assert "\nimport torch" not in head and "\nfrom torch" not in head


@pytest.mark.gpu
def test_gpus_2_without_launcher_runs_the_headline_on_the_device():
    """The launcher path end to end on the GPU: `bench.py --gpus 2` with no
    torch.distributed.run starts two ranks (gloo, both on device 0 of a
    one-GPU box), each estimates its shard of the headline batch on the
    device, and the relayed line spans both ranks with a measured value."""
    p = _run(["--gpus", "2", "--steps", "3", "--warmup", "1", "--prewarm-s", "0.05", "--no-extras",
              "--no-cpu-baseline", "--frames-per-gpu", "4096", "--extras-out", ""], timeout=600)
    assert p.returncode == 0, p.stderr[-3000:]
    r = _line(p)
    assert r["n_gpus"] == 2 and r["launcher"] == "bench.py --gpus 2"
    assert r["dist_check"]["group_size"] == 2 and r["dist_check"]["all_ranks_agree"]
    assert r["config"]["global_frames"] == 2 * 4096
    assert r["value"] > 0 and r["nonfinite_frames"] == 0


def test_sigterm_to_the_parent_reaches_the_ranks():
    """A driver that stops the parent with SIGTERM must not leave ranks
    behind: the parent forwards the signal to torch.distributed.run, which
    stops its workers, and the parent exits non-zero."""
    import signal
    import time
    e = dict(os.environ, WCE_DIST_BACKEND="gloo", OMP_NUM_THREADS="1", WCE_DRY_HOLD_S="60")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    p = subprocess.Popen([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--dry-run"],
                         stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=e, cwd=REPO)
    t0, seen = time.time(), 0
    while time.time() - t0 < 60 and p.poll() is None:   # wait until both ranks run
        time.sleep(1)
        seen = _ranks_of(p.pid)
        if seen >= 2:
            break
    assert seen == 2, "the two ranks never started"
    time.sleep(3)                      # past the process group's formation
    p.send_signal(signal.SIGTERM)
    out, err = p.communicate(timeout=120)
    assert p.returncode != 0
    assert _ranks_of(p.pid) == 0


def _ranks_of(ppid):
    """live bench.py rank processes below ppid (via /proc)"""
    import glob
    kids = {ppid}
    found = 0
    changed = True
    procs = {}
    for d in glob.glob("/proc/[0-9]*"):
        try:
            st = open(d + "/stat").read()
            pid = int(d.rsplit("/", 1)[1])
            procs[pid] = (int(st.rsplit(")", 1)[1].split()[1]), open(d + "/cmdline").read())
        except (OSError, ValueError, IndexError):
            continue
    while changed:
        changed = False
        for pid, (pp, _) in procs.items():
            if pp in kids and pid not in kids:
                kids.add(pid)
                changed = True
    for pid in kids - {ppid}:
        cmd = procs[pid][1]
        if "bench.py" in cmd and "torch.distributed.run" not in cmd:
            found += 1
    return found
