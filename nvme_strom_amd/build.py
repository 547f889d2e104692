"""Build libstrom.so (engine + gfx950 kernels) and the CLI tools in-tree,
then check what was built.

``python -m nvme_strom_amd.build [-j N] [--clean]`` drives the top-level
Makefile (the same build runs here, cross-compiling for gfx950 without a
GPU, and on the GPU box) and then ``check()``s the result: every entry
point the ctypes binding declares (``_native._SIGS``) must be exported by
the library, and the library must carry a gfx950 code object — a missing
kernel or a stale build fails here, not at the first call on a GPU box.
``__graft_entry__.build()`` is this function.
"""
from __future__ import annotations

import argparse
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def build(jobs: int = 0, clean: bool = False, target: str = "all") -> None:
    jobs = jobs or min(16, os.cpu_count() or 4)
    env = dict(os.environ)
    env.setdefault("PYTORCH_ROCM_ARCH", "gfx950")
    if clean:
        subprocess.run(["make", "-C", ROOT, "clean"], check=True, env=env)
    subprocess.run(["make", "-C", ROOT, f"-j{jobs}", target], check=True, env=env)


def check() -> dict:
    """Exported symbols and the offload target of the built libstrom.so."""
    import ctypes as C

    from . import _native
    path = _native.LIB_PATH
    if not os.path.exists(path):
        raise RuntimeError(f"{path} missing: the build produced no library")
    lib = C.CDLL(path)
    missing = [n for n in _native._SIGS if not hasattr(lib, n)]
    if missing:
        raise RuntimeError(f"{path} lacks entry points the binding declares: {missing}")
    with open(path, "rb") as f:
        blob = f.read()
    if b"gfx950" not in blob:
        raise RuntimeError(f"{path} carries no gfx950 code object")
    return dict(library=path, entry_points=len(_native._SIGS), target="gfx950",
                bytes=len(blob))


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("-j", "--jobs", type=int, default=0)
    ap.add_argument("--clean", action="store_true")
    ap.add_argument("target", nargs="?", default="all")
    a = ap.parse_args(argv)
    build(a.jobs, a.clean, a.target)
    print(check())
    return 0


if __name__ == "__main__":
    sys.exit(main())
