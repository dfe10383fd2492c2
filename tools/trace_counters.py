#!/usr/bin/env python3
"""Run one render of the bench workload with ARX_TRACE_KERNEL=$1 and print the raw 16
device counters (design tool for instrumented / self-check variants)."""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["ARX_TRACE_KERNEL"] = sys.argv[1]
from audiorenderingv2_amd import AudioRenderer, RenderSettings, conference_standin, receiver_local  # noqa: E402
from audiorenderingv2_amd._lib import check, lib  # noqa: E402
from audiorenderingv2_amd.scene import CONFERENCE_EMITTER, CONFERENCE_LISTENER  # noqa: E402

s = RenderSettings(rays=(100, 100, 100), sample_rate=48000, base_power=3.62, max_bounces=16)
r = AudioRenderer(s, scene=conference_standin(), receiver=receiver_local())
r.setEmitterPosInOptix(CONFERENCE_EMITTER)
r.setSphereCenterInOptix(CONFERENCE_LISTENER, 0.0)
ms = r.render()
c = (C.c_uint64 * 16)()
check(lib().arx_debug_trace_counters(r.handle, c, 16))
print(f"variant {sys.argv[1]}: {ms:.3f} ms counters", list(c))
