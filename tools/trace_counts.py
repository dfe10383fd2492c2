#!/usr/bin/env python3
"""Node steps and leaf triangle tests per closest-hit query of the C3 trace launch, from a
counting build of the library (build.py --exp count -D ARX_TRACE_COUNT=1; counters[4..7]).
Feeds the vector-memory (TD) roofline of DESIGN.md section 6: a node step is two 16-B lane
loads (QNode2), a triangle test three (TriRec), shading three more and the direction one.

    ARX_LIB=tools/experiments/lib/libarx_count.so python tools/trace_counts.py
"""
import ctypes as C
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from audiorenderingv2_amd import AudioRenderer, RenderSettings, conference_standin, receiver_local  # noqa: E402
from audiorenderingv2_amd._lib import check, lib  # noqa: E402
from audiorenderingv2_amd._lib import use_library  # noqa: E402

if os.environ.get("ARX_LIB"):  # a design-experiment build (tools only)
    use_library(os.environ["ARX_LIB"])
from audiorenderingv2_amd.scene import CONFERENCE_EMITTER, CONFERENCE_LISTENER  # noqa: E402

s = RenderSettings(rays=(100, 100, 100), sample_rate=48000, base_power=3.62, max_bounces=16)
r = AudioRenderer(s, scene=conference_standin(), receiver=receiver_local())
r.setEmitterPosInOptix(CONFERENCE_EMITTER)
r.setSphereCenterInOptix(CONFERENCE_LISTENER, 0.0)
ms = r.render()
c = (C.c_uint64 * 8)()
check(lib().arx_debug_trace_counters(r.handle, c, 8))
q, steps, tris, leader, slots = c[0], c[4], c[5], c[6], c[7]
loads = 2 * steps + 3 * tris + 3 * q + 1 * 10**6
st = r.stats()
# guard: the same tree as the product run (the counting build's kernel differs, its tree does not)
print(json.dumps({"workload": "c3", "tree_hash": f"{int(st['tree_hash']):016x}",
                  "trace_kernel_id": f"{int(lib().arx_trace_kernel_id()):016x}", "queries": q, "node_steps": steps,
                  "tri_tests": tris, "steps_per_query": steps / q, "tri_tests_per_query": tris / q,
                  "lane_loads_16B_per_query": loads / q, "trace_ms_counting_build": ms,
                  # the scalar-fetch probe: node lane-steps on the wave leader's node
                  "leader_node_lane_steps": leader, "node_step_slots": slots,
                  "leader_node_fraction": leader / steps if steps else None,
                  "lanes_per_node_step_slot": steps / slots if slots else None}))
