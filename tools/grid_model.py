"""Issue-count model of the headline solve's trailing update on two lane grids
(round-2 review item 5: the 4x16 lane grid of DESIGN.md s8).

Per pivot step k of the row-panel Cholesky (pivots 1..52 after the exact
first step; rows 0..54 = Ryy + the two bordered rows), the trailing update
A[i][j] -= c_i conj(c_j) over i >= j beyond the current 8-column panel is
issued block by block: one complex FMA group (4 v_fma_f64) per register block
that holds any live element, whatever fraction of its lanes is live.  Operand
reads per step: the 8x8 grid reads one row operand per live block row and one
column operand per live block column (ds_read_b128 each); the 4x16 grid reads
ONE register of row operands (row_newbcast DPP hands lane a of each 16-lane
row to the row) plus one column operand per live 16-wide block column.
Round 6 (review item 5, "one new lane mapping, measured before it is built"):
the same count for mappings that put 2 or 4 frames in one wave (each frame on
a 32- or 16-lane part of the wave, every FMA instruction updating the same
block of each), with the register budget that decides occupancy: the matrix
blocks plus the product kernel's other 56 VGPRs (168 - 112 at 3 waves/SIMD,
512 VGPRs per SIMD lane on gfx950) -> waves and frames per SIMD.
usage: python tools/grid_model.py"""

NR, NC = 55, 53   # rows incl. the bordered rows 53, 54; columns of Ryy


def blocks(bh, bw, jmin):
    """Register blocks (bh rows x bw columns) holding an element i >= j, j >= jmin."""
    out = []
    for a in range((NR + bh - 1) // bh):
        for b in range((NC + bw - 1) // bw):
            if any(i >= j and j >= jmin for i in range(a * bh, min(a * bh + bh, NR))
                   for j in range(b * bw, min(b * bw + bw, NC))):
                out.append((a, b))
    return out


def model():
    res = {}
    for name, bh, bw in (("8x8", 8, 8), ("4x16", 4, 16)):
        fma = reads = 0
        for k in range(1, NC):
            jmin = (k // 8) * 8 + 8          # trailing columns start after the current 8-column panel
            bl = blocks(bh, bw, jmin)
            fma += 4 * len(bl)
            rows = {a for a, _ in bl}
            cols = {b for _, b in bl}
            reads += (len(rows) + len(cols)) if name == "8x8" else (1 + len(cols)) if bl else 0
        res[name] = (fma, reads)
    return res


OTHER_VGPRS = 56   # the headline kernel's non-matrix registers (168 total at 3 waves/SIMD, 112 of them the 8x8 blocks)


def multi_frame():
    """(name, trailing FMA issues per frame, operand LDS reads per frame, VGPRs, waves/SIMD, frames/SIMD)"""
    out = []
    for name, bh, bw, fpw in (("8x8", 8, 8, 1), ("4x16", 4, 16, 1), ("2x(4x8)", 4, 8, 2), ("2x(8x4)", 8, 4, 2),
                              ("4x(4x4)", 4, 4, 4)):
        fma = reads = 0
        for k in range(1, NC):
            jmin = (k // 8) * 8 + 8
            bl = blocks(bh, bw, jmin)
            fma += 4 * len(bl)
            reads += len({a for a, _ in bl}) + len({b for _, b in bl})
        vg = 4 * len(blocks(bh, bw, 0)) + OTHER_VGPRS
        waves = 512 // vg
        out.append((name, fma / fpw, reads / fpw, vg, waves, waves * fpw))
    return out


if __name__ == "__main__":
    r = model()
    for name, (fma, reads) in r.items():
        print(f"{name:5s} grid: {fma:5d} trailing v_fma_f64 issued per frame, {reads:4d} operand ds_reads per frame")
    d_fma = r["4x16"][0] - r["8x8"][0]
    d_rd = r["8x8"][1] - r["4x16"][1]
    print(f"4x16 - 8x8: +{d_fma} FMA issues (+{100 * d_fma / 2615:.0f}% of the headline's 2,615 FMA_F64 per frame), "
          f"-{d_rd} LDS reads (-{100 * d_rd / 549:.0f}% of its 549 LDS instructions)")
    print()
    print("frames per wave (round 6): per frame   FMA issues  operand reads  VGPRs  waves/SIMD  frames/SIMD")
    for name, fma, rd, vg, w, fs in multi_frame():
        print(f"  {name:9s}                      {fma:7.0f}      {rd:7.1f}     {vg:4d}     {w:3d}        {fs:3d}")
