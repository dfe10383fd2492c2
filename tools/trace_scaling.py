#!/usr/bin/env python3
"""Trace-kernel time vs ray count (steady-state throughput vs fixed tail) for given variants.

    python tools/trace_scaling.py 0,320 250000,500000,1000000,2000000,4000000
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from audiorenderingv2_amd import AudioRenderer, RenderSettings, conference_standin, receiver_local  # noqa: E402
from audiorenderingv2_amd.scene import CONFERENCE_EMITTER, CONFERENCE_LISTENER  # noqa: E402

variants = [int(v) for v in sys.argv[1].split(",")]
counts = [int(v) for v in sys.argv[2].split(",")]
scene, recv = conference_standin(), receiver_local()
for v in variants:
    os.environ["ARX_TRACE_KERNEL"] = str(v)
    prev = None
    for n in counts:
        s = RenderSettings(rays=(n // 10000, 100, 100), sample_rate=48000, base_power=3.62, max_bounces=16)
        r = AudioRenderer(s, scene=scene, receiver=recv)
        r.setEmitterPosInOptix(CONFERENCE_EMITTER)
        r.setSphereCenterInOptix(CONFERENCE_LISTENER, 0.0)
        r.render()
        ms = sorted(r.render() for _ in range(5))[2]
        q = r.stats()["queries"]
        extra = ""
        if prev:
            dq, dt = q - prev[0], ms - prev[1]
            extra = f"  marginal {dq / dt / 1e6:.3f} Gq/s  implied fixed {ms - q / (dq / dt):.3f} ms"
        print(f"variant {v} rays {n}: {ms:.3f} ms  {q / ms / 1e6:.3f} Gq/s{extra}", flush=True)
        prev = (q, ms)
        r.close()
