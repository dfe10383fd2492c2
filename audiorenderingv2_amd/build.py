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
import hashlib
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

SOURCES = ["arx_trace.hip", "arx_receiver.hip", "arx_conv.hip", "arx_capi.cpp", "arx_group.cpp", "arx_bvh.cpp", "arx_io.cpp",
           "arx_wide.cpp"]
HEADERS = ["arx_layout.hpp", "arx_kernels.hpp", "arx_bvh.hpp", "arx_internal.hpp", "arx_wide.hpp", "arx_scene_share.hpp"]

COMMON = [
    "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-fno-fast-math",
    "-fhip-fp32-correctly-rounded-divide-sqrt", "-Wall", "-Wno-unused-function",
    f"--offload-arch={ARCH}", "-I", os.path.join(REPO, "include"),
]


# Per-file flags.  arx_trace.hip: no SLP vectorisation -- packed f32 VALU (v_pk_add/mul/fma_f32,
# which the SLP vectoriser forms from the triangle test's and shading's scalar arithmetic) costs more
# issue cycles than the scalar pairs it replaces (MI355X_MICROARCH.md); C3 trace -2 %, C2 -4 %
# (profiles/r03/ab_leaf2_noslp.txt).  Same arithmetic, bit-identical results.
FILE_FLAGS = {"arx_trace.hip": ["-fno-slp-vectorize"]}


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found (ROCm is required to build libarx.so)")


def _newest(paths: list[str]) -> float:
    return max(os.path.getmtime(p) for p in paths)


# Measurement-only macros: they add counters / per-wave records to the trace kernel but leave its
# traversal and arithmetic alone, so they do not change the kernel's identity (trace_source_id).
MEASUREMENT_MACROS = ("ARX_TRACE_COUNT", "ARX_TRACE_PROF")


def _source_id(files: tuple[str, ...], defines: tuple[str, ...]) -> str:
    h = hashlib.sha1()
    for f in files:
        with open(os.path.join(CSRC, f), "rb") as fh:
            h.update(fh.read())
    for d in sorted(d for d in defines if d.split("=")[0] not in MEASUREMENT_MACROS):
        h.update(b"\0" + d.encode())
    return "0x" + h.hexdigest()[:16] + "ull"


def trace_source_id(defines: tuple[str, ...] = ()) -> str:
    """64-bit identity of the trace kernel a build compiles: a hash of its source files and of the
    experiment macros (not the measurement-only ones).  Compiled into the library
    (arx_trace_kernel_id) and stored in every PMC profile's guard, so bench.py uses a stored
    profile only for the kernel it was taken of."""
    # arx_kernels.hpp (host launcher declarations) is not part of it: its edits do not change the kernel
    return _source_id(("arx_trace.hip", "arx_layout.hpp"), defines)


def conv_source_id(defines: tuple[str, ...] = ()) -> str:
    """The same identity for the file convolution's kernels (arx_conv.hip; arx_conv_kernel_id): the
    guard of the stored convolution traffic profile."""
    return _source_id(("arx_conv.hip",), defines)


SOURCE_IDS = {"arx_trace.hip": ("ARX_TRACE_SRC_ID", trace_source_id), "arx_conv.hip": ("ARX_CONV_SRC_ID", conv_source_id)}


def _compile(src: str, objdir: str = OBJDIR, defines: tuple[str, ...] = (), flags: tuple[str, ...] = ()) -> str:
    obj = os.path.join(objdir, os.path.basename(src) + ".o")
    deps = [src, os.path.abspath(__file__)] + [os.path.join(CSRC, h) for h in HEADERS] + [os.path.join(REPO, "include", "arx.h")]
    if os.path.exists(obj) and os.path.getmtime(obj) >= _newest(deps):
        return obj
    lang = ["-x", "hip"]  # host-only TUs too: they use the HIP runtime headers
    sid = SOURCE_IDS.get(os.path.basename(src))
    extra = [f"-D{sid[0]}={sid[1](defines)}"] if sid else []
    cmd = [hipcc(), *lang, *COMMON, *FILE_FLAGS.get(os.path.basename(src), []), *[f"-D{d}" for d in defines], *extra,
           *flags, "-c", src, "-o", obj]
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{res.stdout}\n{res.stderr}")
    return obj


def build(force: bool = False, verbose: bool = False, exp: str | None = None, defines: tuple[str, ...] = (),
          flags: tuple[str, ...] = ()) -> str:
    """The product libarx.so; with exp="<tag>", a design-experiment library
    tools/experiments/lib/libarx_<tag>.so built with the given -D macros (ARX_TRACE_*,
    ARX_LDS_STACK) and extra compiler flags, loaded by tools through ARX_LIB.  The product build
    takes neither."""
    objdir, lib = OBJDIR, LIB
    if exp:
        objdir = os.path.join(REPO, "tools", "experiments", "obj", exp)
        lib = os.path.join(REPO, "tools", "experiments", "lib", f"libarx_{exp}.so")
        os.makedirs(os.path.dirname(lib), exist_ok=True)
        force = True
    os.makedirs(objdir, exist_ok=True)
    srcs = [os.path.join(CSRC, s) for s in SOURCES]
    if force:
        for f in os.listdir(objdir):
            os.remove(os.path.join(objdir, f))
    with cf.ThreadPoolExecutor(max_workers=min(4, len(srcs))) as ex:
        objs = list(ex.map(lambda s: _compile(s, objdir, tuple(defines), tuple(flags)), srcs))
    if not force and os.path.exists(lib) and os.path.getmtime(lib) >= _newest(objs):
        return lib
    # RCCL for the multi-GPU groups' IR all-reduce (arx_group.cpp), from the ROCm install
    rocm_lib = os.path.join(os.path.dirname(os.path.dirname(hipcc())), "lib")
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", lib + ".tmp", *objs, "-Wl,--no-undefined",
           f"-L{rocm_lib}", "-lrccl", f"-Wl,-rpath,{rocm_lib}"]
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        raise RuntimeError(f"link failed: {' '.join(cmd)}\n{res.stdout}\n{res.stderr}")
    os.replace(lib + ".tmp", lib)
    if verbose:
        print("built", lib)
    return lib


def main(argv: list[str] | None = None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--exp", help="design-experiment library tag (tools/experiments/lib/libarx_<tag>.so)")
    ap.add_argument("-D", dest="defines", action="append", default=[], help="macro for --exp builds")
    ap.add_argument("--flag", dest="flags", action="append", default=[], help="compiler flag for --exp builds")
    args = ap.parse_args(argv)
    if (args.defines or args.flags) and not args.exp:
        ap.error("-D / --flag are only for --exp builds")
    build(force=args.force, verbose=True, exp=args.exp, defines=tuple(args.defines), flags=tuple(args.flags))
    return 0


if __name__ == "__main__":
    sys.exit(main())
