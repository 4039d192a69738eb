"""Content hash of libwce.so's sources.  The csrc Makefile writes it next to
the library (libwce.so.srchash) when it links; tests/conftest.py recomputes it
and rebuilds when they differ, so a stale library is never tested silently."""
import glob
import hashlib
import os

PKG = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(PKG)


def sources():
    files = []
    for pat in ("csrc/*.hip", "csrc/*.cpp", "csrc/*.h", "csrc/Makefile"):
        files += glob.glob(os.path.join(PKG, pat))
    files += glob.glob(os.path.join(REPO, "include", "*.h"))
    return sorted(files, key=lambda p: os.path.relpath(p, REPO))


def source_hash() -> str:
    h = hashlib.sha256()
    for p in sources():
        h.update(os.path.relpath(p, REPO).encode() + b"\0")
        with open(p, "rb") as f:
            h.update(f.read())
    return h.hexdigest()


if __name__ == "__main__":
    print(source_hash())
