#!/usr/bin/env python3
"""The latency floor of a small launch: C2 (conference stand-in, 100 K rays x 8
bounces, 16 kHz) traced whole, then every wave's worth of its rays (64 consecutive ray ids, the
static range one wave of the launch owns) as a launch of its own on the otherwise idle GPU, then each
ray of the slowest such wave alone.  A launch cannot end before its slowest ray's chain of dependent
node steps has run, and a ray alone on the GPU runs that chain at the shortest step latency there is
(no other wave shares its SIMD, its CU's caches or the TD): the slowest solo ray is a floor for the
whole launch under any assignment of rays to lanes, waves or GPUs that keeps one ray's bounces on one
lane.  HIP-event times of the trace kernel (arx_trace_times).

    python tools/c2_floor.py [out.json]
"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from audiorenderingv2_amd import AudioRenderer, RenderSettings, conference_standin, receiver_local  # noqa: E402
from audiorenderingv2_amd._lib import use_library  # noqa: E402
from audiorenderingv2_amd.scene import CONFERENCE_EMITTER, CONFERENCE_LISTENER  # noqa: E402

if os.environ.get("ARX_LIB"):
    use_library(os.environ["ARX_LIB"])

RAYS = (100, 100, 10)
N = RAYS[0] * RAYS[1] * RAYS[2]
WAVE = 64


def timed(r: AudioRenderer, b: int, e: int, reps: int = 3) -> float:
    t = []
    for _ in range(reps):
        r.trace_rays(b, e)
        t.append(float(r.trace_times(1)[0]))
    return float(np.median(t))


def main() -> int:
    s = RenderSettings(rays=RAYS, sample_rate=16000, base_power=3.62, max_bounces=8)
    r = AudioRenderer(s, scene=conference_standin(), receiver=receiver_local())
    r.setEmitterPosInOptix(CONFERENCE_EMITTER)
    r.setSphereCenterInOptix(CONFERENCE_LISTENER, 0.0)
    full = float(np.median([r.render() for _ in range(11)][1:]))
    full_ev = float(np.median(r.trace_times(10)))
    waves = np.array([timed(r, b, min(b + WAVE, N), 1) for b in range(0, N, WAVE)])
    order = np.argsort(waves)[::-1]
    top = [(int(w), timed(r, int(w) * WAVE, min(int(w) * WAVE + WAVE, N))) for w in order[:8]]
    w_slow = max(top, key=lambda x: x[1])[0]
    rays = [(int(i), timed(r, i, i + 1)) for i in range(w_slow * WAVE, min(w_slow * WAVE + WAVE, N))]
    ray_slow = max(rays, key=lambda x: x[1])
    out = {
        "workload": "c2 (conference stand-in, 100K rays x 8 bounces, 16 kHz)",
        "full_launch_ms": {"render_median": full, "trace_kernel_events_median": full_ev},
        "one_wave_launches_ms": {"waves": int(len(waves)), "max": float(waves.max()), "p99": float(np.quantile(waves, 0.99)),
                                 "p50": float(np.median(waves)), "min": float(waves.min())},
        "slowest_waves_remeasured_ms": top,
        "slowest_wave": w_slow,
        "its_rays_alone_ms": {"max": ray_slow[1], "ray_id": ray_slow[0],
                              "p50": float(np.median([t for _, t in rays]))},
        "floor_over_full": ray_slow[1] / full_ev,
        "method": __doc__.strip().splitlines()[0],
    }
    txt = json.dumps(out, indent=1)
    print(txt)
    if len(sys.argv) > 1:
        with open(sys.argv[1], "w") as fh:
            fh.write(txt)
    r.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
