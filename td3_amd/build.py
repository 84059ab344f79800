"""Build libtd3hip.so in-tree with hipcc for gfx950 (MI355X).

    python -m td3_amd.build          # incremental (skips when up to date)
    python -m td3_amd.build --force
"""
from __future__ import annotations

import argparse
import glob
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
OUT = os.path.join(HERE, "libtd3hip.so")
SOURCES = ["csrc/replay.hip", "csrc/kernels.hip", "csrc/encoder.hip", "csrc/td3.hip"]
ARCH = os.environ.get("TD3_OFFLOAD_ARCH", "gfx950")
FLAGS = ["-O3", "-std=c++17", f"--offload-arch={ARCH}", "-fPIC", "-shared",
         "-ffp-contract=off", "-Wall", "-Wno-unused-function", "-Wno-unused-value",
         # the GEMM stages' problem directory (first 6 int kernel arguments) arrives in SGPRs
         "-mllvm", "-amdgpu-kernarg-preload-count=6"]


def _hipcc():
    for cand in (os.environ.get("HIPCC"), shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found (ROCm toolchain required)")


def _stale() -> bool:
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    deps = [os.path.join(HERE, s) for s in SOURCES]
    deps += glob.glob(os.path.join(HERE, "csrc", "*.h"))
    deps += glob.glob(os.path.join(ROOT, "include", "*.h"))
    return any(os.path.getmtime(d) > t for d in deps)


def build_library(force: bool = False, verbose: bool = False) -> str:
    if not force and not _stale():
        return OUT
    tmp = OUT + ".tmp"
    cmd = [_hipcc(), *FLAGS, *[os.path.join(HERE, s) for s in SOURCES], "-o", tmp, "-lrccl"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    r = subprocess.run(cmd, cwd=HERE, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed ({r.returncode}):\n{r.stderr[-6000:]}")
    if "warning:" in r.stderr:                      # the build is expected to be warning-free
        print(r.stderr[-6000:], file=sys.stderr)
    os.replace(tmp, OUT)
    return OUT


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    args = ap.parse_args()
    print(build_library(force=args.force, verbose=True))


if __name__ == "__main__":
    main()
