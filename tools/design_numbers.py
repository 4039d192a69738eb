"""Regenerate DESIGN.md's measurement table (section 6) from profiles/<round>_bench.json
and profiles/<round>_pmc_summary.json, so the document never drifts from the
committed evidence.  usage: python tools/design_numbers.py [r01]"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
rnd = sys.argv[1] if len(sys.argv) > 1 else "r01"
d = json.load(open(os.path.join(REPO, "profiles", f"{rnd}_bench.json")))
pm = json.load(open(os.path.join(REPO, "profiles", f"{rnd}_pmc_headline.json")))
r = d["roofline"]
refc = d["cpu_baseline"].get("reference_code", {})
hp = d.get("host_pipeline")
host_row = (f"| headline from pinned HOST memory (PCIe-inclusive; never `value`) | {hp['frames_per_s']:.3g} frames/s, "
            f"{hp['pcie_GBs']:.0f} GB/s over PCIe ({hp['pcie_bytes_per_frame']} B per frame: tx, rx block 0 in, H out), "
            f"{hp['ms_per_batch']:.2f} ms per 65,536 frames; bit-identical to the device-resident path: {hp['bit_identical_to_device_path']} |"
            if hp else "| headline from pinned host memory | not measured in this bench line |")
c4, c5s = d.get("config4"), d.get("config5_sharded")
c4_row = ""
if c4:
    c4_row += (f"| BASELINE configs[3] batch (1,048,576 frames, sharded over {c4['n_gpus']} GPU(s), strong scaling) | "
               f"{c4['frames_per_s']:.3g} frames/s |")
if c5s:
    c4_row += ("\n" if c4_row else "") + (f"| BASELINE configs[4] as named (1,048,576 frames, all 5 + eq fused, fp64 solve / fp32 LS, "
               f"sharded over {c5s['n_gpus']} GPU(s)) | {c5s['frames_per_s']:.3g} frames/s |")
sb = d["small_batch"]
mlsb = (f"; MATLAB + FRAME_COV (several kernels): {sb['matlab_frame_cov_direct']['us_per_call']:.0f} µs direct, "
        f"{sb['matlab_frame_cov_plan']['us_per_call']:.0f} µs as a plan" if "matlab_frame_cov_plan" in sb else "")
table = f"""| Quantity | Value |
|---|---|
| MMSE frames/s, TEXTBOOK (headline) | **{d['value']:.3g}** (target ≥1e7) |
| `mmse_solve_fc_kernel` (the whole step: one launch) | {r['avg_launch_ms']:.3f} ms per 65,536 frames. **{r['achieved']:.1f} TFLOP/s = {100 * r['frac']:.1f}%** of FP64 spec peak by SURVEY's F_alg. Executed flops: {r['achieved_executed']:.1f} TFLOP/s = {100 * r['achieved_executed'] / 78.6:.1f}% |
{c4_row}
| MMSE frames/s, REF (diagonal Ryy: no factorisation) | {d['ref_mode']['frames_per_s_per_gpu']:.3g} |
| MMSE with a dense model covariance (COV: back-substitution + MFMA GEMM) | {d['cov_mode']['frames_per_s_per_gpu']:.3g} frames/s; solve {d['cov_mode']['solve_tflops']:.1f} TFLOP/s |
| `matvec_kernel` as `H = C·W` (MFMA, COV mode) | {d['apply_kernel']['achieved_tflops']:.0f} TFLOP/s = {100 * d['apply_kernel']['frac_fp64_peak']:.0f}% of FP64 peak |
| per-frame covariance MMSE (`FRAME_COV`) | {d['frame_cov']['textbook']['frames_per_s']:.3g} frames/s TEXTBOOK, {d['frame_cov']['ref']['frames_per_s']:.3g} REF |
| config 5 (131,072 frames, all 5 + equalization, fused) | {d['config5']['fp64']['frames_per_s']:.3g} frames/s fp64; {d['config5']['mixed_fp64_solve_fp32_ls']['frames_per_s']:.3g} with fp32 LS outputs |
| LS config 2 (LT_LS + PS_Linear), 1,048,576 frames | {d['ls_config2']['b1048576']['achieved_GBs'] / 1000:.2f} TB/s algorithmic = {100 * d['ls_config2']['b1048576']['frac']:.0f}% of 8 TB/s; {d['ls_config2']['b1048576'].get('real_GBs', 0) / 1000:.2f} TB/s of PMC-measured HBM traffic (pilot sectors counted); {d['ls_config2']['b1048576']['frames_per_s']:.2g} frames/s |
| LS config 2, 65,536 frames (MALL-resident) | {d['ls_config2']['b65536']['achieved_GBs'] / 1000:.2f} TB/s, {d['ls_config2']['b65536']['frames_per_s']:.2g} frames/s |
| front end, 65,536 frames × 15 blocks | {d['front_end']['blocks']['achieved_GBs'] / 1000:.2f} TB/s = {100 * d['front_end']['blocks']['frac']:.1f}% of 8 TB/s (PMC traffic = algorithmic bytes to 1e-4); LTF {d['front_end']['preamble']['achieved_GBs'] / 1000:.2f} TB/s |
| non-finite guard (`wce_nonfinite_scan`), 1,048,576 LT_LS outputs | {d['ls_config2']['nonfinite_scan']['achieved_GBs'] / 1000:.2f} TB/s = {100 * d['ls_config2']['nonfinite_scan']['frac']:.1f}% of 8 TB/s; headline output non-finite frames: {d['nonfinite_frames']} |
| small batches (1,024 frames, all 5 + eq) | {d['small_batch']['direct']['us_per_call']:.0f} µs per call direct, {d['small_batch']['plan']['us_per_call']:.0f} µs as a replayed HIP-graph plan{mlsb} |
{host_row}
| CPU baseline (oracle fp64 port, 16 host cores, dense path) | {d['cpu_baseline']['value']:.2g} MMSE frames/s (4–6e5, host-load dependent) |
"""
if refc:
    table += (f"| the reference's own code (`oracle/_ref`, 1 core) | LT_LS + PS_Linear {refc['ls_config2']['value']:.2g} frames/s; "
              f"REF-mode PS_MMSE through its matrix routines {refc['mmse_ref_mode']['value']:.0f} frames/s "
              f"(NaN inverse repaired, per-frame 4-s `inverse(F)` hoisted) |\n")
    if "ls_config2_omp" in refc:
        table += (f"| the reference's own functions, frames-parallel OpenMP loop ({refc['ls_config2_omp']['cores']} host cores; "
                  f"its own OpenMP driver crashes) | LT_LS + PS_Linear {refc['ls_config2_omp']['value']:.2g} frames/s; "
                  f"REF-mode PS_MMSE {refc['mmse_ref_mode_omp']['value']:.0f} frames/s |\n")
table += "| reference `main.c` MMSE as written | ~0.004 frames/s, 1 core, NaN output; best published number 0.18 frames/s over 20 MPI ranks |\n"
k = [x for x in pm if x.endswith("mmse_solve_fc_kernel")]
pmc = ""
if k:
    v = {c: x / 65536 for c, x in pm[k[0]].items()}
    busy = 3 * v["SQ_ACTIVE_INST_VALU"] / v["SQ_WAVE_CYCLES"]
    traffic = (2 * pm[k[0]]["FETCH_SIZE"] + pm[k[0]]["WRITE_SIZE"]) * 1024 / 1e6
    pmc = f"""**PMC**, `mmse_solve_fc_kernel`, headline run only (TEXTBOOK), per frame (= per wave). Source: `profiles/{rnd}_pmc_headline.json`, collected with `tools/refresh_profiles.sh`, one pass per counter group.
- {v['SQ_INSTS_VALU']:,.0f} VALU instructions, of which {v['SQ_INSTS_VALU_FMA_F64']:,.0f} are `FMA_F64` and {v['SQ_INSTS_VALU_MUL_F64']:,.0f} `MUL_F64`.
- {v['SQ_INSTS_LDS']:,.0f} LDS instructions with {v['SQ_LDS_BANK_CONFLICT']:.0f} bank conflicts.
- VALU active {v['SQ_ACTIVE_INST_VALU']:,.0f} of {v['SQ_WAVE_CYCLES']:,.0f} quad-cycles per wave. Over 3 co-resident waves that is ≈{100 * busy:.0f}% of SIMD time.
- HBM: FETCH_SIZE×2 + WRITE_SIZE = {traffic:.0f} MB per 65,536-frame launch, against 167 MB algorithmic.
"""
p = os.path.join(REPO, "DESIGN.md")
s = open(p).read()
a = s.index("| Quantity | Value |")
b = s.index("The bench brings the GPU to its steady clock")
s = s[:a] + table + "\n" + s[b:]
a = s.index("**PMC**, `mmse_solve")
b = s.index("**What limits it now**")
s = s[:a] + pmc + "\n" + s[b:]
open(p, "w").write(s)
print(table)
