"""Regenerate DESIGN.md's measurement table (section 6) and its PMC
paragraph from profiles/<round>_bench.json and profiles/<round>_pmc_legs.json,
so the document never drifts from the committed evidence.
usage: python tools/design_numbers.py [r02]"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
rnd = sys.argv[1] if len(sys.argv) > 1 else "r02"
# round 5+: the full record is the extras file beside the compact bench line
_full = os.path.join(REPO, "profiles", f"{rnd}_bench_extras.json")
d = json.load(open(_full if os.path.exists(_full) else os.path.join(REPO, "profiles", f"{rnd}_bench.json")))
# PMC legs: the newest profile of each leg up to this round (a round re-profiles only the legs it changed)
import glob  # noqa: E402
legs, leg_src = {}, {}
for _f in sorted(glob.glob(os.path.join(REPO, "profiles", "r*_pmc_legs.json"))):
    if os.path.basename(_f)[:3] <= rnd:
        _l = json.load(open(_f))
        legs.update(_l)
        leg_src.update({k: os.path.basename(_f) for k in _l})
r = d["roofline"]
refc = d["cpu_baseline"].get("reference_code", {})
rows = []   # (quantity, value); None entries are skipped (never a blank table line)


def row(q, v):
    rows.append((q, v))


row("MMSE frames/s, TEXTBOOK (headline)", f"**{d['value']:.3g}** (target ≥1e7)")
row("`mmse_solve_fc_kernel` (the whole step: one launch)",
    f"{r['avg_launch_ms']:.3f} ms per 65,536 frames. **{r['achieved']:.1f} TFLOP/s = {100 * r['frac']:.1f}%** of the FP64 "
    f"spec peak by SURVEY's F_alg; executed flops {r['achieved_executed']:.1f} TFLOP/s = {100 * r['frac_executed']:.1f}%")
if r.get("board"):
    b = r["board"]
    row("board during the headline (`amd-smi`, untimed, back-to-back launches)",
        f"{b['socket_power_W']:.0f} W, shader clock {b['gfx_clock_MHz']:.0f} MHz (spec peak assumes 2,400): "
        f"{100 * r['frac'] * 2400 / b['gfx_clock_MHz']:.1f}% of the FP64 peak at that clock")
c4, c5s = d.get("config4"), d.get("config5_sharded")
if c4:
    row(f"BASELINE configs[3] batch (1,048,576 frames, sharded over {c4['n_gpus']} GPU(s), strong scaling)",
        f"{c4['frames_per_s']:.3g} frames/s")
if c5s:
    extra = ""
    if c5s.get("solve_only_ms"):
        extra = f"; {c5s['ms_per_step']:.2f} ms per step, PS_MMSE alone on the same frames {c5s['solve_only_ms']:.2f} ms"
        bf, bs = c5s.get("board_fused"), c5s.get("board_solve_only")
        if bf and bs:
            extra += (f"; board {bf['socket_power_W']:.0f} W / {bf['gfx_clock_MHz']:.0f} MHz fused, "
                      f"{bs['socket_power_W']:.0f} W / {bs['gfx_clock_MHz']:.0f} MHz solve alone")
    row(f"BASELINE configs[4] as named (1,048,576 frames, all 5 + eq fused, fp64 solve / fp32 LS, sharded over "
        f"{c5s['n_gpus']} GPU(s))",
        f"{c5s['frames_per_s']:.3g} frames/s; non-finite outputs: {c5s.get('nonfinite_outputs')}" + extra)
row("MMSE frames/s, REF (diagonal Ryy: no factorisation), 65,536 frames (MALL-resident)",
    f"{d['ref_mode']['frames_per_s_per_gpu']:.3g}")
rb = d["ref_mode"].get("b1048576")
if rb:
    rr = rb["roofline"]
    row("REF, 1,048,576 frames (past the MALL), `mmse_ref_elem_kernel` (round 6: one element per thread)",
        f"{rb['frames_per_s']:.3g} frames/s; {rr['achieved'] / 1000:.2f} TB/s algorithmic (976 B/frame) = "
        f"{100 * rr['frac']:.0f}% of 8 TB/s; {rr['achieved_sector_GBs'] / 1000:.2f} TB/s on the 1,360-B sector floor = "
        f"{100 * rr['frac_sector']:.0f}%; PMC traffic {rr['traffic'] / rb['frames']:.0f} B/frame")
cv = d["cov_mode"]
row("MMSE with a dense model covariance (COV: Cholesky keeping L + back-substitution, then MFMA `C·W`)",
    f"{cv['frames_per_s_per_gpu']:.3g} frames/s; solve {cv['solve_tflops']:.1f} TFLOP/s = "
    f"{100 * cv['solve_frac_fp64_peak']:.0f}% of FP64 peak")
cm = cv.get("constant_modulus")
if cm:
    row("the same on constant-modulus frames (`wce_ctx_set_modulus`: K = (a C P + b I)⁻¹ C once, H = K (x̄ ∘ rx) on "
        "f64 MFMA; never the headline)",
        f"{cm['frames_per_s_per_gpu']:.3g} frames/s ({cm['speedup_vs_per_frame']:.1f}× the per-frame path), "
        f"{cm['achieved_GBs'] / 1000:.2f} TB/s of the 2,544 B a frame moves")
lr = d.get("cov_lowrank")
if lr:
    parts = []
    for L in ("L4", "L8", "L16", "L24", "L53"):
        if L in lr:
            x = lr[L]
            parts.append(f"{L[1:]} taps `{x['kernel']}` {x['ms_per_step']:.3f} ms ({x['frames_per_s']:.3g} frames/s)"
                         + (f", product Gram {x['product_gram_ms_per_step']:.3f} ms" if "product_gram_ms_per_step" in x
                            else "")
                         + (f", {100 * x['roofline']['frac']:.0f}% of FP64 peak by its algorithmic flops"
                            if "roofline" in x else ""))
    row("MMSE with an L-tap power-delay profile (COV low-rank paths, 65,536 frames)", "; ".join(parts))
    for L in ("L16", "L53"):
        c = lr.get(L, {}).get("constant_modulus")
        if c:
            row(f"the same, {L[1:]} taps, constant-modulus frames (operator path)",
                f"{c['ms_per_step']:.3f} ms ({c['frames_per_s']:.3g} frames/s, {c['speedup_vs_per_frame']:.1f}× "
                f"the per-frame path; {100 * c['roofline']['frac']:.0f}% of HBM)")
    b8 = lr.get("L8", {}).get("frames_1048576")
    if b8:
        row("rank 8 at 1,048,576 frames (two-workgroups-per-CU build)",
            f"{b8['ms_per_step']:.3f} ms ({b8['frames_per_s']:.3g} frames/s, {100 * b8['roofline']['frac']:.0f}% of HBM)")
ap = d["apply_kernel"]
row("`apply_kernel` as `H = C·W` (f64 MFMA, COV mode, 65,536 frames = 4,096 16-frame tiles; persistent since round 5)",
    f"{ap['achieved_tflops']:.1f} TFLOP/s algorithmic = {100 * ap['frac_fp64_peak']:.0f}% of FP64 peak; "
    + (f"{ap['executed_tflops']:.1f} TFLOP/s executed; MFMA pipe busy {100 * ap['mfma_busy_frac_pmc']:.0f}% (PMC of "
       f"same-size launches); traffic {ap['traffic'] / 1e6:.0f} MB vs {ap['algorithmic_bytes'] / 1e6:.0f} MB algorithmic"
       if "executed_tflops" in ap else "no same-size PMC"))
if "frames_1M" in ap:
    ab = ap["frames_1M"]
    row("`apply_kernel` as `H = C·W`, 1,048,576 frames (streaming: C in LDS, next tile's W loaded under the MFMAs; "
        "3M form, three real MFMA products per complex one)",
        f"{ab['avg_launch_ms'] * 1e3:.0f} µs; {ab['achieved_GBs'] / 1000:.2f} TB/s of W in + H out"
        + (f" = {100 * ab['frac_hbm_peak']:.0f}% of 8 TB/s (its load/store stream alone: 380 µs)" if "frac_hbm_peak" in ab else "")
        + f"; {ab['achieved_tflops']:.1f} TFLOP/s algorithmic (8 n² per frame) = "
        f"{100 * ab['frac_fp64_peak']:.0f}% of FP64 peak"
        + (f"; {ab['executed_tflops']:.1f} TFLOP/s executed, MFMA pipe busy {100 * ab['mfma_busy_frac_pmc']:.0f}% (PMC of "
           f"same-size launches); traffic {ab['traffic'] / 1e6:.0f} MB vs {ab['algorithmic_bytes'] / 1e6:.0f} MB"
           if "executed_tflops" in ab else ""))
row("per-frame covariance MMSE (`FRAME_COV`)",
    f"{d['frame_cov']['textbook']['frames_per_s']:.3g} frames/s TEXTBOOK, {d['frame_cov']['ref']['frames_per_s']:.3g} REF")
c5r = d.get("config5_ref")
if c5r:
    txt = []
    for k, lab in (("fp64", "fp64"), ("mixed_fp64_solve_fp32_ls", "fp32 LS / eq"),
                   ("frame_cov_fp64", "FRAME_COV fp64"), ("frame_cov_mixed_fp32_ls", "FRAME_COV fp32 LS / eq")):
        if k in c5r:
            x = c5r[k]
            txt.append(f"{lab} {x['frames_per_s']:.3g} frames/s ({x['roofline']['achieved'] / 1000:.2f} TB/s)")
    row("configs[4] in `main.c` semantics (REF + LS family + eq, 1,048,576 frames; FRAME_COV: each frame's PS_MMSE "
        "on its own LT_LS, as main.c:37-53)", "; ".join(txt))
row("config 5 share (131,072 frames, all 5 + equalization, fused)",
    f"{d['config5']['fp64']['frames_per_s']:.3g} frames/s fp64; "
    f"{d['config5']['mixed_fp64_solve_fp32_ls']['frames_per_s']:.3g} with fp32 LS outputs")
ls = d["ls_config2"]["b1048576"]
row("LS config 2 (LT_LS + PS_Linear), 1,048,576 frames",
    f"{ls['achieved_GBs'] / 1000:.2f} TB/s algorithmic = {100 * ls['frac']:.0f}% of 8 TB/s; "
    + (f"{ls['real_GBs'] / 1000:.2f} TB/s of PMC-measured HBM traffic ({ls['traffic_bytes_per_frame']:.0f} B/frame); "
       if "real_GBs" in ls else "") + f"{ls['frames_per_s']:.2g} frames/s")
l65 = d["ls_config2"]["b65536"]
row("LS config 2, 65,536 frames (MALL-resident)", f"{l65['achieved_GBs'] / 1000:.2f} TB/s, {l65['frames_per_s']:.2g} frames/s")
fe = d["front_end"]
row("front end, 65,536 frames × 15 blocks",
    f"{fe['blocks']['achieved_GBs'] / 1000:.2f} TB/s = {100 * fe['blocks']['frac']:.1f}% of 8 TB/s; "
    f"LTF {fe['preamble']['achieved_GBs'] / 1000:.2f} TB/s")
ns = d["ls_config2"]["nonfinite_scan"]
row("non-finite guard (`wce_nonfinite_scan`), 1,048,576 LT_LS outputs",
    f"{ns['achieved_GBs'] / 1000:.2f} TB/s = {100 * ns['frac']:.1f}% of 8 TB/s; headline output non-finite frames: "
    f"{d['nonfinite_frames']}")
if "ldc_convert" in d:
    lc = d["ldc_convert"]
    row("reference-format conversion (`wce_ldc_to_complex` / `wce_complex_to_ldc`), 65,536 frames × 795 values",
        f"{lc['to_complex']['achieved_GBs'] / 1000:.2f} / {lc['to_ldc']['achieved_GBs'] / 1000:.2f} TB/s = "
        f"{100 * lc['to_complex']['frac']:.0f}% / {100 * lc['to_ldc']['frac']:.0f}% of 8 TB/s (48 B per value)")
sb = d["small_batch"]
row("small batches (1,024 frames, all 5 + eq)",
    f"{sb['direct']['us_per_call']:.0f} µs per call direct, {sb['plan']['us_per_call']:.0f} µs as a replayed "
    f"HIP-graph plan; MATLAB + FRAME_COV (several kernels): {sb['matlab_frame_cov_direct']['us_per_call']:.0f} µs "
    f"direct, {sb['matlab_frame_cov_plan']['us_per_call']:.0f} µs as a plan")
hp = d.get("host_pipeline")
if hp:
    row("headline from pinned HOST memory (PCIe-inclusive; never `value`)",
        f"{hp['frames_per_s']:.3g} frames/s, {hp['pcie_GBs']:.0f} GB/s over PCIe ({hp['pcie_bytes_per_frame']} B per "
        f"frame), {100 * hp['frac_of_h2d_bound']:.0f}% of the H2D copy bound; bit-identical to the device-resident "
        f"path: {hp['bit_identical_to_device_path']}")
cb = d["cpu_baseline"]
row(f"CPU baseline (oracle fp64 port, {cb['cores']} host cores, dense path)",
    f"{cb['value']:.2g} MMSE frames/s; its H vs the GPU's on the same {cb.get('err_frames', 0)} frames: max "
    f"{cb.get('max_normrel_err_vs_gpu', float('nan')):.1e} norm-relative")
if refc:
    row("the reference's own code (`oracle/_ref`, 1 core)",
        f"LT_LS + PS_Linear {refc['ls_config2']['value']:.2g} frames/s; REF-mode PS_MMSE through its matrix routines "
        f"{refc['mmse_ref_mode']['value']:.0f} frames/s (NaN inverse repaired, per-frame 4-s `inverse(F)` hoisted)")
    if "mmse_textbook" in refc:
        mt = refc["mmse_textbook"]
        fp = mt.get("frames_parallel", {})
        row("the reference's own routines composing the TEXTBOOK (headline) formula (`multiply()` + cofactor "
            "`inverse()`, `refh_mmse_formula`)",
            f"{mt['value']:.3g} frames/s on 1 core ({mt['sample']})"
            + (f"; {fp['value']:.3g} frames/s frames-parallel on {fp['cores']} cores" if fp else ""))
    if "ls_config2_omp" in refc:
        row(f"the reference's own functions, frames-parallel OpenMP loop ({refc['ls_config2_omp']['cores']} host "
            f"cores; its own OpenMP driver crashes)",
            f"LT_LS + PS_Linear {refc['ls_config2_omp']['value']:.2g} frames/s; REF-mode PS_MMSE "
            f"{refc['mmse_ref_mode_omp']['value']:.0f} frames/s")
row("reference `main.c` MMSE as written", "~0.004 frames/s, 1 core, NaN output; best published number 0.18 frames/s "
    "over 20 MPI ranks")
table = "| Quantity | Value |\n|---|---|\n" + "".join(f"| {q} | {v} |\n" for q, v in rows if q)

h = legs.get("headline")
pmc = ""
if h:
    n = h["frames"]
    v = {c: x / n for c, x in h["counters"].items()}
    busy = 3 * v["SQ_ACTIVE_INST_VALU"] / v["SQ_WAVE_CYCLES"]
    traffic = (2 * h["counters"]["FETCH_SIZE"] + h["counters"]["WRITE_SIZE"]) * 1024 / 1e6
    pmc = (f"**PMC**, `mmse_solve_fc_kernel` alone at the bench's launch size (65,536 frames, {h['dispatches']} "
           f"dispatches per pass), per frame (= per wave). Source: `profiles/{leg_src.get('headline', rnd + '_pmc_legs.json')}` "
           f"(`tools/pmc_legs.sh`, one pass per counter group).\n"
           f"- {v['SQ_INSTS_VALU']:,.0f} VALU instructions, of which {v['SQ_INSTS_VALU_FMA_F64']:,.0f} are `FMA_F64` and "
           f"{v['SQ_INSTS_VALU_MUL_F64']:,.0f} `MUL_F64`.\n"
           f"- {v['SQ_INSTS_LDS']:,.0f} LDS instructions with {v['SQ_LDS_BANK_CONFLICT']:.0f} bank conflicts.\n"
           f"- VALU active {v['SQ_ACTIVE_INST_VALU']:,.0f} of {v['SQ_WAVE_CYCLES']:,.0f} quad-cycles per wave. Over 3 "
           f"co-resident waves that is ≈{100 * busy:.0f}% of SIMD time.\n"
           f"- HBM: FETCH_SIZE×2 + WRITE_SIZE = {traffic:.0f} MB per 65,536-frame launch, against 167 MB algorithmic.\n")
    for leg, what, prev in (
            ("lowrank24", "`mmse_lr_quad2_kernel<24>` (leg `lowrank24`)",
             "The wave kernel it replaces at rank 24 issued 2,105 VALU and 432 LDS instructions per frame "
             "(`r04_pmc_legs.json`). Its LDS tables at odd 16-B-slot row pitches: 227 → 168 conflict cycles, "
             "164.5 → 160.2 µs (`r06_ab_lowrank_pad.txt`); what is left is the E[k d] gathers of the DFTs (16 lanes, "
             "16 different entries). The forward substitution as DPP64 FMAs over zeroed upper entries: 1,196 → "
             "1,100 VALU per frame, 153 → 135 µs (`r06_ab_lowrank_solves.txt`)."),
            ("lowrank16", "`mmse_lr_quad_kernel<16, true>` (leg `lowrank16`)",
             "Odd row pitches: 178 → 100 conflict cycles, 92.0 → 88.1 µs; the forward substitution as DPP64 FMAs: "
             "590 → 543 VALU per frame, 83.0 → 77.7 µs; the Gram tables in place (22.5 KB of LDS per "
             "workgroup, 4 workgroups per CU): 82.1 → 76.2 µs.")):
        q = legs.get(leg)
        if not q:
            continue
        u = {c: x / q["frames"] for c, x in q["counters"].items()}
        pmc += (f"- Round 6, {what}, per frame (4 frames per wave): {u['SQ_INSTS_VALU']:,.0f} VALU instructions, "
                f"{u['SQ_INSTS_VALU_FMA_F64']:,.0f} of them `FMA_F64`; {u['SQ_INSTS_LDS']:,.0f} LDS instructions, "
                f"{u['SQ_LDS_BANK_CONFLICT']:,.0f} bank-conflict cycles; `SQ_WAIT_INST_LDS` "
                f"{u['SQ_WAIT_INST_LDS']:,.0f}. {prev}\n")
    q = legs.get("ref")
    if q:
        fb, wb = (q["counters"][c] * 1024 / q["frames"] for c in ("FETCH_SIZE", "WRITE_SIZE"))
        pmc += (f"- Round 6, `mmse_ref_elem_kernel` (leg `ref`, {q['frames']:,} frames): FETCH_SIZE {fb:.0f} B and "
                f"WRITE_SIZE {wb:.0f} B per frame ({fb + wb:,.0f} B against the 1,360-B sector floor; the pilot "
                f"sectors of a frame that straddles two waves are read by both).\n")
p = os.path.join(REPO, "DESIGN.md")
s = open(p).read()
a = s.index("| Quantity | Value |")
b = s.index("The bench brings the GPU to its steady clock")
s = s[:a] + table + "\n" + s[b:]
if pmc:
    a = s.index("**PMC**, `mmse_solve")
    b = s.index("**What limits it now**")
    s = s[:a] + pmc + "\n" + s[b:]
open(p, "w").write(s)
print(table)
print(pmc)
