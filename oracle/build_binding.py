#!/usr/bin/env python3
"""TEST INFRASTRUCTURE: build the reference-side binding INTEGRATION.md s1
documents, exactly as a maintainer would, and nothing more.

1. copy the reference's main.c into a temporary directory (never into this
   repository: the copy is deleted when the build ends);
2. apply INTEGRATION.md's diff: delete the five prototypes (main.c:4-8) and
   the five estimator bodies (main.c:66-211), and #include "wce_compat.h";
   the call sites (main.c:37-54) stay as they are;
3. compile it as the reference does, with g++ -std=gnu++98 -w (compile.c:26-29
   builds main.c with g++: C++ linkage everywhere except what wce_compat.h
   declares extern "C"), against include/wce_compat.h, together with the
   reference's own utils.c where it lies;
4. link it against libwce.so and the MPI library utils.h needs.

A second translation unit (probe) prints wce_compat_last_status() at exit,
so a run shows whether the shims reached the device (0) or reported its
absence (WCE_ENODEV = -5).  Output: oracle/_ref/main_wce (git-ignored; it
travels to the GPU box with the rest of oracle/_ref).

usage: build_binding.py [--ref /root/reference] [--out oracle/_ref/main_wce]
"""
import argparse
import os
import re
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
MPI_DIR = os.environ.get("MPI_DIR", "/opt/conda")

PROBE = r'''
#include <stdio.h>
#include "wce_compat.h"
/* runs after main() returns: the status of the last compat call */
__attribute__((destructor)) static void wce_binding_report(void)
{
    printf("wce_compat_last_status=%d\n", wce_compat_last_status());
    fflush(stdout);
}
'''


def patch_main(src: str) -> str:
    """INTEGRATION.md s1's diff, applied to main.c's text."""
    lines = src.split("\n")
    # main.c:4-8: the five prototypes (C++ linkage) -- now from wce_compat.h (C linkage)
    protos = [i for i, l in enumerate(lines[:12]) if re.match(r"\s*void WiFi_channel_estimation_\w+\(.*\);\s*$", l)]
    if len(protos) != 5:
        raise SystemExit(f"expected the 5 estimator prototypes near main.c:4-8, found {len(protos)}")
    # main.c:66-211: the five bodies, from the first definition to the end of the file
    defs = [i for i, l in enumerate(lines) if re.match(r"void WiFi_channel_estimation_\w+\(.*\)\s*\{\s*$", l)]
    if len(defs) != 5:
        raise SystemExit(f"expected the 5 estimator definitions (main.c:66-212), found {len(defs)}")
    out = lines[:defs[0]]
    out = [l for i, l in enumerate(out) if i not in protos]
    inc = next(i for i, l in enumerate(out) if l.startswith('#include "utils.h"'))
    out.insert(inc + 1, '#include "wce_compat.h"          /* prototypes of main.c:4-8, extern "C", from libwce */')
    return "\n".join(out) + "\n"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default=os.environ.get("WCE_REFERENCE", "/root/reference"))
    ap.add_argument("--out", default=os.path.join(HERE, "_ref", "main_wce"))
    args = ap.parse_args()
    ref = os.path.abspath(args.ref)
    if not os.path.exists(os.path.join(ref, "main.c")):
        raise SystemExit(f"no reference main.c under {ref}")
    os.makedirs(os.path.dirname(os.path.abspath(args.out)), exist_ok=True)
    lib_dir = os.path.join(REPO, "80211parallelestimation_amd")
    if not os.path.exists(os.path.join(lib_dir, "libwce.so")):
        raise SystemExit("libwce.so not built")
    rpath = os.path.relpath(lib_dir, os.path.dirname(os.path.abspath(args.out)))
    with tempfile.TemporaryDirectory(prefix="wce_binding_") as tmp:
        with open(os.path.join(ref, "main.c")) as f:
            patched = patch_main(f.read())
        with open(os.path.join(tmp, "main.c"), "w") as f:
            f.write(patched)
        with open(os.path.join(tmp, "probe.cpp"), "w") as f:
            f.write(PROBE)
        cmd = ["g++", "-std=gnu++98", "-O2", "-DMPICH_SKIP_MPICXX", "-I" + os.path.join(REPO, "include"),
               "-I" + ref, "-I" + os.path.join(MPI_DIR, "include"),
               os.path.join(tmp, "main.c"), os.path.join(tmp, "probe.cpp"), os.path.join(ref, "utils.c"),
               "-L" + lib_dir, "-lwce", os.path.join(MPI_DIR, "lib", "libmpi.so"),
               # RUNPATH order: libwce first, the system libstdc++ before the image's
               # older MPI-side copy in /opt/conda/lib (libamdhip64 needs GLIBCXX_3.4.30)
               "-Wl,-rpath,$ORIGIN/" + rpath + ":/usr/lib/x86_64-linux-gnu:" + os.path.join(MPI_DIR, "lib"),
               "-w", "-o", args.out]
        print(" ".join(cmd), flush=True)
        subprocess.check_call(cmd)
    print(f"built {args.out}")


if __name__ == "__main__":
    sys.exit(main())
