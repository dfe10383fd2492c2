#!/usr/bin/env python3
"""Trace time vs ray count for given variants (tail analysis): rays per wave = n / 5120 on a
256-CU MI355X at 5 waves/SIMD, so 983040 and 1310720 rays are whole rounds of 64 lanes."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from audiorenderingv2_amd import AudioRenderer, RenderSettings, conference_standin, receiver_local  # noqa: E402
from audiorenderingv2_amd.scene import CONFERENCE_EMITTER, CONFERENCE_LISTENER  # noqa: E402

variants = sys.argv[1].split(",")
sizes = [tuple(int(v) for v in x.split("x")) for x in sys.argv[2].split(",")]
scene, recv = conference_standin(), receiver_local()
for dims in sizes:
    s = RenderSettings(rays=dims, sample_rate=48000, base_power=3.62, max_bounces=16)
    r = AudioRenderer(s, scene=scene, receiver=recv)
    r.setEmitterPosInOptix(CONFERENCE_EMITTER)
    r.setSphereCenterInOptix(CONFERENCE_LISTENER, 0.0)
    n = dims[0] * dims[1] * dims[2]
    for v in variants:
        os.environ["ARX_TRACE_KERNEL"] = v
        r.render()
        ms = sorted(r.render() for _ in range(5))[2]
        print(f"variant {v} rays {n} ({n / 5120:.1f}/wave): {ms:.3f} ms  {n / ms / 1e3:.3f} Mrays/ms", flush=True)
