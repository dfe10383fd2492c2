#!/usr/bin/env python3
"""Render the C3 bench workload a few times (for profilers and A/B runs).

    python tools/trace_once.py [n_renders]      # library: ARX_LIB (default: the product libarx.so)
Prints the median trace-kernel time (HIP events) over the renders after the first; with
ARX_GUARD_OUT=path it also writes the run's profile guard (workload, tree hash, trace kernel VGPRs:
bench.py only uses a stored profile whose guard matches its own run)."""
import json
import os
import sys

import numpy as np

# ARX_PKG_ROOT: import the package from another tree (e.g. a build of an older commit, A/B only)
sys.path.insert(0, os.environ.get("ARX_PKG_ROOT") or os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from audiorenderingv2_amd import AudioRenderer, RenderSettings, conference_standin, receiver_local  # noqa: E402
from audiorenderingv2_amd.scene import CONFERENCE_EMITTER, CONFERENCE_LISTENER  # noqa: E402
from audiorenderingv2_amd._lib import lib, use_library  # noqa: E402

if os.environ.get("ARX_LIB"):  # a design-experiment build (tools only)
    use_library(os.environ["ARX_LIB"])

n = int(sys.argv[1]) if len(sys.argv) > 1 else 3
rays = tuple(int(v) for v in os.environ.get("RAYS", "100,100,100").split(","))
s = RenderSettings(rays=rays, sample_rate=48000, base_power=3.62, max_bounces=int(os.environ.get("BOUNCES", "16")))
r = AudioRenderer(s, scene=conference_standin(), receiver=receiver_local())
r.setEmitterPosInOptix(CONFERENCE_EMITTER)
r.setSphereCenterInOptix(CONFERENCE_LISTENER, 0.0)
if os.environ.get("TRACE_PATH"):  # arx_debug_set_trace_path: 0 BVH2 16-bit (default), 8 CW4, 1 BVH2 f32
    r.set_trace_path(int(os.environ["TRACE_PATH"]))
ms = [r.render() for _ in range(n)]
st = r.stats()
irl, irr = r.get_ir()
chk = int(np.frombuffer(irl.tobytes() + irr.tobytes(), np.uint32).astype(np.uint64).sum())
med = float(np.median(ms[1:] if n > 1 else ms))
if os.environ.get("ARX_GUARD_OUT"):
    with open(os.environ["ARX_GUARD_OUT"], "w") as fh:
        json.dump({"workload": "c3" if rays == (100, 100, 100) and s.max_bounces == 16 else f"rays{rays}",
                   "tree_hash": f"{int(st['tree_hash']):016x}", "trace_vgprs": int(st["trace_vgprs"]),
                   "trace_format": int(st["trace_format"]),
                   "trace_kernel_id": f"{int(lib().arx_trace_kernel_id()):016x}"}, fh)
print(f"trace {med:.3f} ms (median of {max(n - 1, 1)}) queries {st['queries']} nodes {st['n_nodes']} "
      f"depth {st['bvh_depth']} format {st['trace_format']} vgprs {st['trace_vgprs']} ir_checksum {chk} lib {os.path.basename(os.environ.get('ARX_LIB', 'libarx.so'))}",
      flush=True)
