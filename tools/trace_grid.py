#!/usr/bin/env python3
"""Persistent-grid size sweep (ARX_GRID_PCT) for given variants on the bench workload."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from audiorenderingv2_amd import AudioRenderer, RenderSettings, conference_standin, receiver_local  # noqa: E402
from audiorenderingv2_amd.scene import CONFERENCE_EMITTER, CONFERENCE_LISTENER  # noqa: E402

variants = sys.argv[1].split(",")
pcts = [int(x) for x in sys.argv[2].split(",")]
s = RenderSettings(rays=(100, 100, 100), sample_rate=48000, base_power=3.62, max_bounces=16)
r = AudioRenderer(s, scene=conference_standin(), receiver=receiver_local())
r.setEmitterPosInOptix(CONFERENCE_EMITTER)
r.setSphereCenterInOptix(CONFERENCE_LISTENER, 0.0)
for v in variants:
    os.environ["ARX_TRACE_KERNEL"] = v
    for p in pcts:
        os.environ["ARX_GRID_PCT"] = str(p)
        r.render()
        ms = sorted(r.render() for _ in range(5))[2]
        print(f"variant {v} grid {p}%: {ms:.3f} ms", flush=True)
