"""Static checks on the compiled gfx950 assembly of the kernels.

The solve kernels issue DPP64 FMAs from inline asm (row_newbcast operands,
wce_kernels.hip cmsub_bc).  The hardware needs 2 wait states between a VALU
write of a VGPR and a DPP instruction reading it through the DPP crossbar;
the compiler cannot see into inline asm, so this checks the emitted code:
no VALU instruction in the 2 wait states before a DPP instruction writes
that instruction's DPP source (src0).  A DPP instruction at a branch target
whose predecessors the straight-line scan cannot see is flagged only when it
comes from inline asm (;;#ASMSTART .. ;;#ASMEND): the compiler's own hazard
recognizer covers every predecessor of the DPP instructions it emits
(__builtin_amdgcn_mov_dpp, the quad kernel's row broadcasts).
usage: python tools/isa_check.py [file.s]   (default: compile wce_kernels.hip)"""
import os
import re
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(REPO, "80211parallelestimation_amd", "csrc", "wce_kernels.hip")
# every translation unit with DPP64 FMAs from inline asm (round 6: the quad2 Cholesky)
SRCS = (SRC, os.path.join(REPO, "80211parallelestimation_amd", "csrc", "wce_lr_quad2.hip"))
REG = re.compile(r"v\[(\d+):(\d+)\]|v(\d+)\b")


def regs(tok: str):
    m = REG.search(tok)
    if not m:
        return set()
    if m.group(3) is not None:
        return {int(m.group(3))}
    return set(range(int(m.group(1)), int(m.group(2)) + 1))


LABEL = "<label>"


def _lines(text: str):
    """(instruction or LABEL, inside inline asm) for every instruction and label."""
    in_asm = False
    for line in text.splitlines():
        c = line.strip()
        if c.startswith(";;#ASMSTART"):
            in_asm = True
        elif c.startswith(";;#ASMEND"):
            in_asm = False
        t = line.split(";")[0].strip()
        if t.endswith(":"):   # labels (".LBB0_3:", "kernel:") before directives (".p2align")
            yield LABEL, in_asm
            continue
        if not t or t.startswith("."):
            continue
        yield t, in_asm


def instructions(text: str, labels=False):
    """Instruction lines; with labels=True also the basic-block labels (as LABEL)."""
    for t, _ in _lines(text):
        if t != LABEL or labels:
            yield t


def dpp_hazards(text: str):
    """List of (dpp instruction, offending earlier instruction).  A label is a
    branch target or loop header whose predecessors this straight-line scan
    cannot see: a DPP instruction fewer than 2 wait states after one is
    reported (offender LABEL) unless those wait states come after the label --
    for inline-asm DPP only (module docstring)."""
    out, prev = [], []   # prev: (wait states the instruction provides, text)
    for ins, in_asm in _lines(text):
        if ins == LABEL:
            prev.append((0, LABEL))
            prev = prev[-8:]
            continue
        op = ins.split()[0]
        if "_dpp" in op:
            ops = [o.strip() for o in ins[len(op):].split(",")]
            src0 = regs(ops[1].lstrip("-|")) if len(ops) > 1 else set()
            ws = 0
            for w, p in reversed(prev):
                if ws >= 2:
                    break
                if p == LABEL:
                    if in_asm:
                        out.append((ins, LABEL))
                    break
                pop = p.split()[0]
                if pop.startswith("v_") and not pop.startswith(("v_readlane", "v_readfirstlane", "v_cmp")):
                    dst = regs(p[len(pop):].split(",")[0])
                    if dst & src0:
                        out.append((ins, p))
                ws += w
        ws_self = 1
        if op == "s_nop":
            ws_self = int(ins.split()[1], 0) + 1
        prev.append((ws_self, ins))
        prev = prev[-8:]
    return out


def compile_asm(flags=(), srcs=SRCS):
    """gfx950 assembly of the kernel sources, concatenated"""
    out = []
    for src in srcs:
        fd, path = tempfile.mkstemp(suffix=".s")
        os.close(fd)
        cmd = ["/opt/rocm/bin/hipcc", "-O3", "--offload-arch=gfx950", "-std=c++17", "-I" + os.path.join(REPO, "include"),
               "--cuda-device-only", "-S", src, "-o", path, *flags]
        subprocess.run(cmd, check=True, capture_output=True)
        out.append(open(path).read())
        os.unlink(path)
    return "\n".join(out)


def kernel_bodies(text: str):
    """{mangled kernel name: its instruction lines} of a compiled .s file."""
    out, name, buf = {}, None, []
    for line in text.splitlines():
        m = re.match(r"^(_Z[A-Za-z0-9_]+):", line)
        if m:
            name, buf = m.group(1), []
            continue
        if name:
            buf.append(line)
            if "s_endpgm" in line:
                out[name] = buf
                name = None
    return out


def load_rounds(body) -> int:
    """Serialized global-memory round trips, counted statically: the number of
    global loads issued after a vmcnt wait that itself followed a load (a load
    that could not be issued with the ones before it).  A kernel whose loads sit
    under per-element branches, each waited before the next is issued, scores
    one per load (round 5: cm_real_kernel 14 -> 2, ref_fc_kernel 16 -> 5).
    Branch-guarded cold paths count too: compare a kernel with itself."""
    state, n = None, 0
    for line in body:
        t = line.strip().split(";")[0].strip()
        if t.startswith("global_load") or t.startswith("buffer_load"):
            if state == "W":
                n += 1
            state = "L"
        elif "vmcnt(" in t and state == "L":
            state = "W"
    return n


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "--rounds":   # serialized load round trips per kernel
        text = open(sys.argv[2]).read() if len(sys.argv) > 2 else compile_asm()
        for name, body in sorted(kernel_bodies(text).items()):
            print(f"{load_rounds(body):4d}  {name}")
        return
    text = open(sys.argv[1]).read() if len(sys.argv) > 1 else compile_asm()
    n_dpp = sum(1 for i in instructions(text) if "_dpp" in i.split()[0])
    bad = dpp_hazards(text)
    print(f"{n_dpp} DPP instructions, {len(bad)} hazards")
    for d, p in bad[:20]:
        print("  ", p, "->", d)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
