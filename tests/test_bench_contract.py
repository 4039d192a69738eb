"""The committed bench line (profiles/<round>_bench.json) keeps the driver's
contract and agrees with the committed rocprofv3 summary of the same command
(CPU-only: reads the evidence files, runs nothing on a GPU)."""
import csv
import glob
import json
import os

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BASELINE = json.load(open(os.path.join(REPO, "BASELINE.json")))


def _latest(pattern):
    files = sorted(glob.glob(os.path.join(REPO, "profiles", pattern)))
    if not files:
        pytest.skip(f"no profiles/{pattern}")
    return files[-1]


@pytest.fixture(scope="module")
def line():
    """The driver-facing line: bench.py prints it LAST, compact (round 5+)."""
    return json.load(open(_latest("r*_bench.json")))


@pytest.fixture(scope="module")
def full(line):
    """The full per-leg record (bench.py --extras-out, committed as
    profiles/<round>_bench_extras.json); rounds <= 4 printed it as the line."""
    path = _latest("r*_bench.json").replace("_bench.json", "_bench_extras.json")
    return json.load(open(path)) if os.path.exists(path) else line


def test_line_fits_driver_tail():
    """The driver keeps the last 8 KB of stdout and parses the final line:
    the committed line must fit whole (BENCH_r04.json parsed null at 20 KB)."""
    path = _latest("r*_bench.json")
    if os.path.basename(path) < "r05":
        pytest.skip("round <= 4 line predates the compact form")
    text = open(path).read().strip()
    assert "\n" not in text and len(text.encode()) <= 8192, len(text)


def test_compact_line_bounded_and_faithful():
    """bench.compact() of any full record (the largest committed one) stays
    under the limit and carries the headline numbers unchanged."""
    import sys
    sys.path.insert(0, REPO)
    import bench
    fulls = sorted(glob.glob(os.path.join(REPO, "profiles", "r*_bench_extras.json"))) or \
        [f for f in sorted(glob.glob(os.path.join(REPO, "profiles", "r*_bench.json")))]
    src = json.load(open(max(fulls, key=os.path.getsize)))
    c = bench.compact(src, "x.json")
    text = json.dumps(c, separators=(",", ":"))
    assert len(text) <= bench.COMPACT_LIMIT
    for k in ("metric", "value", "ms_per_step", "n_gpus", "dtype"):
        assert c[k] == src[k]
    assert c["roofline"]["frac"] == src["roofline"]["frac"]
    assert c["cpu_baseline"]["value"] == src["cpu_baseline"]["value"]


def test_contract_keys(line):
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in line, k
    assert line["metric"] == BASELINE["metric"]
    assert line["n_gpus"] == 1 and line["scaling"] == "weak" and line["higher_is_better"] is True
    assert line["vs_baseline"] is None          # BASELINE.md publishes no number for this metric
    assert "workload" in line["config"] and "model" not in line["config"]
    # value = frames of all ranks / timed wall
    B = line["config"]["frames_per_gpu"] * line["n_gpus"]
    assert abs(line["value"] - B / (line["ms_per_step"] * 1e-3)) / line["value"] < 1e-6


def test_timed_region_breakdown(line):
    """enqueue + stream wait + closing barrier = the timed wall of rank 0
    (at N=1 it is the whole timed region; the closing barrier is a no-op)."""
    t = line["timed_region_ms"]
    total = t["enqueue"] + t["stream_sync"] + t["barrier"]
    assert abs(total - line["ms_per_step"] * line["steps"]) / total < 1e-3
    assert t["stream_sync"] > t["enqueue"]       # the launches queue ahead of the GPU


def test_roofline_consistent(line):
    r = line["roofline"]
    assert r["bound"] in ("hbm", "mfma", "fp64-valu") and r["unit"] == "TFLOP/s"
    assert abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-9
    ach = r["flop_per_frame"] * r["frames_per_launch"] / (r["avg_launch_ms"] * 1e-3) / 1e12
    assert abs(ach - r["achieved"]) / ach < 1e-9
    assert r["traffic"] is None or r["traffic"] > 0.9 * r["algorithmic_bytes"]


def test_cpu_baseline_fields(line):
    c = line["cpu_baseline"]
    assert c["kind"] in ("port", "reference") and c["cores"] >= 1 and c["value"] > 0 and c["sample"]
    if "max_normrel_err_vs_gpu" in c:        # the port's H against the GPU's, same frames
        assert c["max_normrel_err_vs_gpu"] < 1e-10


def test_leg_rooflines(full):
    """Legs that carry a roofline keep its arithmetic; counters come from
    same-size launches (pmc_source names the legs file, not a refusal)."""
    line = full
    ref = line.get("ref_mode", {}).get("b1048576")
    if ref:
        r = ref["roofline"]
        assert r["bound"] == "hbm" and abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-9
        assert abs(r["achieved"] - r["algorithmic_bytes"] / (ref["avg_launch_ms"] * 1e-3) / 1e9) / r["achieved"] < 1e-9
        assert ref["nonfinite_frames"] == 0
        if r["traffic"] is not None:
            assert r["traffic"] > 0.95 * r["sector_floor_bytes"]
    app = line.get("apply_kernel")
    if app and "waves" in app:   # rounds <= 4: matvec_kernel, one 16-frame tile per wave
        # 3M form: 4 row blocks x 14 k-steps x 3 chains of v_mfma_f64_16x16x4 per 16-frame tile
        assert app["waves"] == 4096 and abs(app["mfma_insts_per_wave"] - 168) < 1e-6
        # executed MFMA flops vs the contract's 8 n^2 per frame: 168 x 2,048 per tile against 16 x 8 x 53^2
        ratio = 168 * 2048 / (16 * 8 * 53 * 53)
        assert abs(app["executed_tflops"] / app["achieved_tflops"] - ratio) < 0.05 * ratio
    elif app and "tiles" in app:   # round 5+: apply_kernel at every size
        # rows 0..47: 3 x 14 x 3 v_mfma_f64_16x16x4; rows 48..52: 14 x 6 v_mfma_f64_4x4x4_4b
        assert app["tiles"] == 4096 and abs(app["mfma_insts_per_tile"] - (126 + 84)) < 1e-6
        ratio = (126 * 2048 + 84 * 512) / (16 * 8 * 53 * 53)
        assert abs(app["executed_tflops"] / app["achieved_tflops"] - ratio) < 0.05 * ratio


def test_rocprof_headline_average_agrees(line):
    """The headline kernel's average duration in the committed headline-only
    rocprofv3 --stats summary is the bench's event-timed launch (within 10%:
    the profiled run includes the clock ramp)."""
    rows = list(csv.DictReader(open(_latest("r*_kernel_stats_headline.csv"))))
    k = [r for r in rows if "mmse_solve_fc_kernel" in r["Name"]]
    assert k, "headline kernel missing from the rocprof summary"
    avg_ms = float(k[0]["AverageNs"]) * 1e-6
    assert abs(avg_ms - line["roofline"]["avg_launch_ms"]) / avg_ms < 0.10, (avg_ms, line["roofline"]["avg_launch_ms"])


def test_extra_legs_consistent(line, full):
    """The extra legs that carry their own arithmetic agree with it: configs[3]
    (strong scaling over 1,048,576 frames), the PCIe-inclusive host pipeline,
    and the non-finite check of the headline output."""
    c4 = full.get("config4")
    if c4:
        assert c4["global_frames"] == 1 << 20 and c4["scaling"] == "strong"
        assert abs(c4["frames_per_s"] - c4["global_frames"] / (c4["ms_per_step"] * 1e-3)) / c4["frames_per_s"] < 1e-6
    hp = full.get("host_pipeline")
    if hp:
        assert hp["bit_identical_to_device_path"] is True
        assert hp["frames_per_s"] < line["value"]          # PCIe-bound, never the headline
    if "nonfinite_frames" in line:
        assert line["nonfinite_frames"] == 0


def test_config5_sharded_consistent(full):
    c5 = full.get("config5_sharded")
    if c5:
        if "nonfinite_outputs" in c5:
            assert c5["nonfinite_outputs"] == 0
        assert c5["global_frames"] == 1 << 20 and c5["scaling"] == "strong"
        assert abs(c5["frames_per_s"] - c5["global_frames"] / (c5["ms_per_step"] * 1e-3)) / c5["frames_per_s"] < 1e-6


def test_multirank_rehearsal_self_explaining():
    """The world-2 rehearsal of the N>1 line (gloo, two ranks on one GPU box:
    the driver's torch.distributed.run launch with WCE_DIST_BACKEND=gloo)
    carries the fields an N=8 reader needs: every rank's process group spans
    WORLD_SIZE (dist_check, min over ranks) and configs[3]'s strong-scaling
    rate per GPU beside its whole-job rate."""
    lines = [ln for ln in open(_latest("r*_bench_2rank_gloo_rehearsal.json")) if ln.startswith("{")]
    reh = json.loads(lines[-1])      # the rank-0 JSON line (gloo prints its own chatter first)
    assert reh["n_gpus"] == 2
    dc = reh.get("dist_check")
    if dc is None:
        pytest.skip("rehearsal predates dist_check (round < 3)")
    assert dc["all_ranks_agree"] is True and dc["group_size"] == 2 == dc["world_size_env"]
    c4 = reh["legs"]["config4"] if "legs" in reh else reh["config4"]   # round 5+: the compact line
    assert c4["n_gpus"] == 2 and c4["scaling"] == "strong"
    # round 6+: leg summaries carry 5 significant digits (full values in the extras file)
    assert abs(c4["frames_per_s_per_gpu"] * 2 - c4["frames_per_s"]) / c4["frames_per_s"] < 1e-4


def test_launcherless_rehearsal_spans_two_ranks():
    """Round 6: `python3 bench.py --gpus 2` with NO torch.distributed.run
    (gloo, both ranks on the one GPU of a gpurun box) -- bench.py started the
    two ranks itself (launch_ranks), and the line it relayed spans them."""
    path = _latest("r*_bench_2rank_gloo_rehearsal.json")
    if os.path.basename(path) < "r06":
        pytest.skip("rehearsal predates the launcher (round < 6)")
    reh = json.loads(open(path).read().strip().splitlines()[-1])
    assert reh["launcher"] == "bench.py --gpus 2"
    assert reh["n_gpus"] == 2 and reh["dist_check"]["group_size"] == 2 and reh["dist_check"]["all_ranks_agree"]
    assert reh["config"]["global_frames"] == 2 * reh["config"]["frames_per_gpu"]
    assert abs(reh["value"] - reh["config"]["global_frames"] / (reh["ms_per_step"] * 1e-3)) / reh["value"] < 1e-6


def test_dist_check_in_headline_line(line):
    dc = line.get("dist_check")
    if dc is None:
        pytest.skip("bench line predates dist_check (round < 3)")
    assert dc["all_ranks_agree"] is True and dc["group_size"] == line["n_gpus"]
