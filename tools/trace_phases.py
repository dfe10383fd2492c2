#!/usr/bin/env python3
"""Phased-launch tail compaction sweep: ARX_PHASES x ARX_DRAIN_LOW on the bench workload.
Every setting must reproduce the single-phase IR bit for bit."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from audiorenderingv2_amd import AudioRenderer, RenderSettings, conference_standin, receiver_local  # noqa: E402
from audiorenderingv2_amd.scene import CONFERENCE_EMITTER, CONFERENCE_LISTENER  # noqa: E402

configs = [tuple(int(x) for x in c.split(":")) for c in sys.argv[1].split(",")]  # phases:low
s = RenderSettings(rays=(100, 100, 100), sample_rate=48000, base_power=3.62, max_bounces=16)
r = AudioRenderer(s, scene=conference_standin(), receiver=receiver_local())
r.setEmitterPosInOptix(CONFERENCE_EMITTER)
r.setSphereCenterInOptix(CONFERENCE_LISTENER, 0.0)
ref = None
for ph, low in configs:
    os.environ["ARX_PHASES"] = str(ph)
    os.environ["ARX_DRAIN_LOW"] = str(low)
    r.render()
    ms = sorted(r.render() for _ in range(7))[3]
    ir, q = r.get_ir(), r.stats()["queries"]
    if ref is None:
        ref = (ir, q)
    same = np.array_equal(ir[0], ref[0][0]) and np.array_equal(ir[1], ref[0][1]) and q == ref[1]
    print(f"phases {ph} low {low}: {ms:.3f} ms  {q / ms / 1e6:.3f} Gq/s identical={same}", flush=True)
    if not same:
        raise SystemExit("phased launch changed the result")
