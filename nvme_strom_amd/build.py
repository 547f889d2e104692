"""Build libstrom.so (engine + gfx950 kernels) and the CLI tools in-tree.

``python -m nvme_strom_amd.build [-j N] [--clean]`` — a thin driver over the
top-level Makefile so the same build runs here (cross-compiling for gfx950
without a GPU) and on the GPU box.
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


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("-j", "--jobs", type=int, default=0)
    ap.add_argument("--clean", action="store_true")
    ap.add_argument("target", nargs="?", default="all")
    a = ap.parse_args(argv)
    build(a.jobs, a.clean, a.target)
    return 0


if __name__ == "__main__":
    sys.exit(main())
