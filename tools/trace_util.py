#!/usr/bin/env python3
"""Wave-utilisation report of the trace kernel (instrumented variant 98 = default v3 + counters).

Counters [8..14] + s_memtime cycles in [5] (node), [15] (leaf), [7] (outer).
Lane utilisation of a phase = lanes doing that phase's work / (iterations x 64)."""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["ARX_TRACE_KERNEL"] = os.environ.get("UTIL_VARIANT", "98")
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
q = c[0]
outer, nit, nl, lit, ll, sh, idle = c[8], c[9], c[10], c[11], c[12], c[13], c[14]
print(f"trace {ms:.3f} ms (instrumented), queries {q}")
print(f"outer iterations {outer}  (per query {outer / q:.3f}); shading lanes/outer {sh / max(outer, 1):.1f} of 64")
print(f"node steps: {nit} wave-iterations, {nl} lane-steps = {nl / q:.1f} per query, utilisation {nl / (64 * nit):.3f}")
print(f"leaf steps: {lit} wave-iterations, {ll} lane-steps = {ll / q:.1f} per query, utilisation {ll / (64 * max(lit, 1)):.3f}")
print(f"idle lanes per inner iteration {idle / max(nit + lit, 1):.1f} of 64")
print(f"wave-iterations per query: node {nit / q:.3f} leaf {lit / q:.3f} outer {outer / q:.3f}")
pend, inact = c[6] >> 32, c[6] & 0xffffffff
print(f"per node iteration: node lanes {nl / nit:.1f}, pending-leaf lanes {pend / nit:.1f}, "
      f"no-ray lanes {inact / nit:.1f} (approx., 32-bit packed) of 64")
cn, cl, co = c[5], c[15], c[7]
tot = cn + cl + co
print(f"wave cycles (s_memtime): node {cn / tot:.3f}  leaf {cl / tot:.3f}  outer/shade/refill {co / tot:.3f}")
print(f"cycles per wave-iteration: node {cn / max(nit, 1):.0f}  leaf {cl / max(lit, 1):.0f}  outer {co / max(outer, 1):.0f}")
