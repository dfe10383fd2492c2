#!/usr/bin/env python3
"""Does a second frame in flight hide the trace launch's tail?  One renderer rendering K frames back
to back on its stream, vs two renderers (sharing nothing but the device, each on its own stream)
alternating frames so that frame k+1's persistent waves fill the SIMDs frame k's finished waves
leave.  Reports wall ms per frame (host clock around K frames, synchronised) for both, and checks the
IRs are the single renderer's.

    python tools/overlap_probe.py [K] [c3|c2]
"""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from audiorenderingv2_amd._lib import use_library  # noqa: E402

if os.environ.get("ARX_LIB"):
    use_library(os.environ["ARX_LIB"])
from audiorenderingv2_amd import AudioRenderer, RenderSettings, conference_standin, receiver_local  # noqa: E402
from audiorenderingv2_amd.scene import CONFERENCE_EMITTER, CONFERENCE_LISTENER  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
shape = sys.argv[2] if len(sys.argv) > 2 else "c3"
rays, bounces, sr = ((100, 100, 100), 16, 48000) if shape == "c3" else ((100, 100, 10), 8, 16000)
s = RenderSettings(rays=rays, sample_rate=sr, base_power=3.62, max_bounces=bounces)
scene, recv = conference_standin(), receiver_local()
rs = []
for _ in range(2):
    r = AudioRenderer(s, scene=scene, receiver=recv)
    r.setEmitterPosInOptix(CONFERENCE_EMITTER)
    r.setSphereCenterInOptix(CONFERENCE_LISTENER, 0.0)
    r.render()
    rs.append(r)
n = int(np.prod(rays))


def frame(r):
    r.clear_histogram()
    r.trace_rays(0, n)
    r.finalize_ir()


def run(nr: int) -> float:
    for r in rs:
        r.stats()
    t0 = time.perf_counter()
    for k in range(K):
        frame(rs[k % nr])
    for r in rs:
        r.stats()  # synchronises each renderer's stream
    return (time.perf_counter() - t0) / K * 1e3


ref = rs[0].get_ir()
for rep in range(3):
    one = run(1)
    two = run(2)
    print(f"{shape} rep {rep}: one stream {one:.3f} ms/frame, two frames in flight {two:.3f} ms/frame "
          f"({(1 - two / one) * 100:+.1f} %)", flush=True)
for r in rs:
    a = r.get_ir()
    assert np.array_equal(a[0].view(np.uint32), ref[0].view(np.uint32))
print("IRs identical")
