#!/usr/bin/env python3
"""Trace-kernel time of each of the first N C3 renders of a fresh process (HIP events), to see how
long the GPU takes to reach its sustained clock (bench.py's pre-roll).  Also the renders' wall clock
with and without a pause, to tell a clock ramp from a cache warm-up.

    python tools/trace_ramp.py [N]
"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from audiorenderingv2_amd import AudioRenderer, RenderSettings, conference_standin, receiver_local  # noqa: E402
from audiorenderingv2_amd.scene import CONFERENCE_EMITTER, CONFERENCE_LISTENER  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 40
s = RenderSettings(rays=(100, 100, 100), sample_rate=48000, base_power=3.62, max_bounces=16)
r = AudioRenderer(s, scene=conference_standin(), receiver=receiver_local())
r.setEmitterPosInOptix(CONFERENCE_EMITTER)
r.setSphereCenterInOptix(CONFERENCE_LISTENER, 0.0)
t0 = time.perf_counter()
first = [r.render() for _ in range(n)]
t1 = time.perf_counter()
time.sleep(2.0)  # idle: a clock ramp starts over, a warm cache does not
after_pause = [r.render() for _ in range(10)]
print(json.dumps({"renders_ms": [round(x, 3) for x in first], "wall_s": t1 - t0,
                  "after_2s_idle_ms": [round(x, 3) for x in after_pause]}))
r.close()
