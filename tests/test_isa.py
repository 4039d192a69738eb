"""Static checks on the compiled gfx950 code (CPU: hipcc cross-compiles).

The rank-1 solve issues DPP64 FMAs from inline asm (wce_kernels.hip
cmsub_bc), and so does the rank 17..32 Cholesky (wce_lr_quad2.hip cmsub_dpp,
round 6); the compiler's hazard recognizer does not look inside them, so
the emitted code is checked for a VALU write of a DPP source VGPR within the
2 wait states the hardware needs (tools/isa_check.py)."""
import os
import shutil
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools"))


@pytest.fixture(scope="module")
def asm_text():
    if not shutil.which("/opt/rocm/bin/hipcc"):
        pytest.skip("hipcc not installed")
    import isa_check
    return isa_check.compile_asm()


def test_no_dpp_source_hazards(asm_text):
    import isa_check
    text = asm_text
    n = sum(1 for i in isa_check.instructions(text) if "_dpp" in i.split()[0])
    assert n > 600, "the headline's DPP in-panel FMAs are missing"
    assert isa_check.dpp_hazards(text) == []


def test_checker_flags_a_hazard():
    import isa_check
    bad = "v_mov_b32 v122, v1\nv_fmac_f64_dpp v[78:79], -v[122:123], v[90:91] row_newbcast:1\n"
    assert len(isa_check.dpp_hazards(bad)) == 1
    ok = "v_mov_b32 v122, v1\ns_nop 1\nv_fmac_f64_dpp v[78:79], -v[122:123], v[90:91] row_newbcast:1\n"
    assert isa_check.dpp_hazards(ok) == []


def test_checker_flags_dpp_after_a_label():
    """A DPP instruction at a branch target / loop header has predecessors the
    straight-line scan cannot see: flagged unless 2 wait states follow the label."""
    import isa_check
    asm = "v_fmac_f64_dpp v[78:79], -v[122:123], v[90:91] row_newbcast:1"
    bad = f"v_mov_b32 v1, v2\n.LBB0_3:\n\t;;#ASMSTART\n{asm}\n\t;;#ASMEND\n"
    assert [p for _, p in isa_check.dpp_hazards(bad)] == [isa_check.LABEL]
    ok = f".LBB0_3:\n\t;;#ASMSTART\ns_nop 1\n{asm}\n\t;;#ASMEND\n"
    assert isa_check.dpp_hazards(ok) == []


def test_compiler_dpp_after_a_label_is_the_compilers():
    """A compiler-emitted DPP (no ;;#ASMSTART) at a label: the compiler's hazard
    recognizer sees its predecessors, so only the straight-line rule applies."""
    import isa_check
    dpp = "v_mov_b32_dpp v30, v24 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf bound_ctrl:1"
    assert isa_check.dpp_hazards(f"s_or_b64 exec, exec, s[0:1]\n.LBB0_3:\n{dpp}\n") == []
    assert len(isa_check.dpp_hazards(f"v_mov_b32 v24, v2\n{dpp}\n")) == 1


def test_streaming_kernels_issue_their_loads_together(asm_text):
    """Round 5 found two streaming MFMA kernels whose per-tile loads sat under
    per-element branches, each waited before the next was issued (14 memory
    round trips per tile instead of one): a regression guard on the compiled
    code (tools/isa_check.py --rounds; profiles/r05_ab_lat.txt)."""
    import isa_check
    bodies = isa_check.kernel_bodies(asm_text)
    rounds = {n: isa_check.load_rounds(b) for n, b in bodies.items()}
    cm = [r for n, r in rounds.items() if "cm_real_kernel" in n]
    cc = [r for n, r in rounds.items() if "cm_cplx_kernel" in n]   # K / C fragments stay L2 reads per k-step
    fc = [r for n, r in rounds.items() if "ref_fc_kernel" in n]
    assert cm and cc and fc
    assert max(cm) <= 3, rounds
    assert max(cc) <= 65, rounds   # 90 with the per-subcarrier loads
    assert max(fc) <= 6, rounds


def test_load_rounds_counts_serialized_loads():
    import isa_check
    serial = ["global_load_dwordx4 v[0:3], v[0:1], off", "s_waitcnt vmcnt(0)"] * 3
    together = ["global_load_dwordx4 v[0:3], v[0:1], off"] * 3 + ["s_waitcnt vmcnt(0)"]
    assert isa_check.load_rounds(serial) == 2
    assert isa_check.load_rounds(together) == 0
