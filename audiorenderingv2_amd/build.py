"""Build libarx.so (HIP, gfx950) in-tree.

    python -m audiorenderingv2_amd.build          # incremental
    python -m audiorenderingv2_amd.build --force

Every translation unit is compiled by hipcc for --offload-arch=gfx950 with IEEE f32
semantics (-ffp-contract=off, correctly rounded f32 div/sqrt) so the trace kernel is
bit-compatible with the CPU oracle; objects are linked into
audiorenderingv2_amd/libarx.so, which travels with the repo snapshot to the GPU box.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import shutil
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
OBJDIR = os.path.join(PKG, "_obj")
LIB = os.path.join(PKG, "libarx.so")
ARCH = os.environ.get("ARX_OFFLOAD_ARCH", "gfx950")

SOURCES = ["arx_trace.hip", "arx_conv.hip", "arx_capi.cpp", "arx_bvh.cpp", "arx_io.cpp"]
HEADERS = ["arx_layout.hpp", "arx_kernels.hpp", "arx_bvh.hpp"]

COMMON = [
    "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-fno-fast-math",
    "-fhip-fp32-correctly-rounded-divide-sqrt", "-Wall", "-Wno-unused-function",
    f"--offload-arch={ARCH}", "-I", os.path.join(REPO, "include"),
]


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found (ROCm is required to build libarx.so)")


def _newest(paths: list[str]) -> float:
    return max(os.path.getmtime(p) for p in paths)


def _compile(src: str) -> str:
    obj = os.path.join(OBJDIR, os.path.basename(src) + ".o")
    deps = [src] + [os.path.join(CSRC, h) for h in HEADERS] + [os.path.join(REPO, "include", "arx.h")]
    if os.path.exists(obj) and os.path.getmtime(obj) >= _newest(deps):
        return obj
    lang = ["-x", "hip"]  # host-only TUs too: they use the HIP runtime headers
    cmd = [hipcc(), *lang, *COMMON, "-c", src, "-o", obj]
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{res.stdout}\n{res.stderr}")
    return obj


def build(force: bool = False, verbose: bool = False) -> str:
    os.makedirs(OBJDIR, exist_ok=True)
    srcs = [os.path.join(CSRC, s) for s in SOURCES]
    if force:
        for f in os.listdir(OBJDIR):
            os.remove(os.path.join(OBJDIR, f))
    with cf.ThreadPoolExecutor(max_workers=min(4, len(srcs))) as ex:
        objs = list(ex.map(_compile, srcs))
    if not force and os.path.exists(LIB) and os.path.getmtime(LIB) >= _newest(objs):
        return LIB
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", LIB + ".tmp", *objs, "-Wl,--no-undefined"]
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        raise RuntimeError(f"link failed: {' '.join(cmd)}\n{res.stdout}\n{res.stderr}")
    os.replace(LIB + ".tmp", LIB)
    if verbose:
        print("built", LIB)
    return LIB


def main(argv: list[str] | None = None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    args = ap.parse_args(argv)
    build(force=args.force, verbose=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
