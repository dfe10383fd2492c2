#!/usr/bin/env python3
"""Frames in flight with the convolution in the step: one renderer doing K full C3 steps (clear,
trace, finalize, file convolution of 807 498 frames) back to back, against two renderers (the
scene build shared through libarx's cache, each on its own stream) alternating steps, with and
without the convolution.  ms per frame on the host clock around K frames.

    python tools/pipeline_probe.py [K]
"""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from audiorenderingv2_amd import AudioRenderer, RenderSettings, conference_standin, receiver_local  # noqa: E402
from audiorenderingv2_amd.renderer import DeviceBuffer  # noqa: E402
from audiorenderingv2_amd.scene import CONFERENCE_EMITTER, CONFERENCE_LISTENER  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
FRAMES = 807498
s = RenderSettings(rays=(100, 100, 100), sample_rate=48000, base_power=3.62, max_bounces=16)
scene, recv = conference_standin(), receiver_local()
audio = np.random.default_rng(1).standard_normal(FRAMES)
rs, bufs = [], []
for _ in range(2):
    r = AudioRenderer(s, scene=scene, receiver=recv)
    r.setEmitterPosInOptix(CONFERENCE_EMITTER)
    r.setSphereCenterInOptix(CONFERENCE_LISTENER, 0.0)
    r.render()
    rs.append(r)
    bufs.append((DeviceBuffer.from_numpy(0, audio), DeviceBuffer(0, 4 * FRAMES), DeviceBuffer(0, 4 * FRAMES)))
n = int(np.prod(s.rays))


def frame(i, conv):
    r = rs[i]
    r.clear_histogram()
    r.trace_rays(0, n)
    r.finalize_ir()
    if conv:
        x, ol, orr = bufs[i]
        r.convolute_device(x.ptr, FRAMES, ol.ptr, orr.ptr)


def run(nr, conv):
    for r in rs:
        r.stats()
    t0 = time.perf_counter()
    for k in range(K):
        frame(k % nr, conv)
    for r in rs:
        r.stats()
    return (time.perf_counter() - t0) / K * 1e3


for rep in range(3):
    a, b = run(1, True), run(2, True)
    c, d = run(1, False), run(2, False)
    print(f"rep {rep}: with convolution one {a:.3f} / two in flight {b:.3f} ms ({(1 - b / a) * 100:+.1f} %); "
          f"trace only one {c:.3f} / two {d:.3f} ms ({(1 - d / c) * 100:+.1f} %)", flush=True)
