#!/usr/bin/env python3
"""Where a trace launch's time goes, per wave: a profiling build of the
library (build.py --exp prof -D ARX_TRACE_PROF=1) records for every persistent wave its start /
end shader clock, the rays and queries it ran, and how many lanes were busy in each phase (node
steps, leaf tests, shading).  This reports, for one workload:

  * the launch span vs the mean / median wave duration (the tail: waves that still run while others
    are done), and the time between a wave's ray range running out and the wave ending;
  * lane efficiency per phase: busy lanes / (64 x phase executions);
  * instruction-slot shares: node-step slots vs leaf and shade phases.

    ARX_LIB=tools/experiments/lib/libarx_prof.so python tools/trace_profile.py c2|c3|c5rank [out.json]
"""
import ctypes as C
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from audiorenderingv2_amd._lib import use_library  # noqa: E402

if os.environ.get("ARX_LIB"):
    use_library(os.environ["ARX_LIB"])
from audiorenderingv2_amd import AudioRenderer, RenderSettings, conference_standin, receiver_local  # noqa: E402
from audiorenderingv2_amd._lib import check, lib  # noqa: E402
from audiorenderingv2_amd.scene import CONFERENCE_EMITTER, CONFERENCE_LISTENER  # noqa: E402

SHAPES = {  # rays of the launch, rays traced, bounces, sample rate
    "c2": ((100, 100, 10), 100_000, 8, 16000),
    "c3": ((100, 100, 100), 1_000_000, 16, 48000),
    "c5rank": ((100, 100, 100), 125_000, 16, 48000),  # one 8-GPU rank's shard of a C5 frame
}
W = 16  # kProfWords


def per_xcd(a: np.ndarray) -> dict:
    """Start skew and end spread within each XCD (s_memtime is per XCD), in units of the longest
    wave, and how the wave duration depends on the wave's slot on its SIMD."""
    xcc = (a[:, 15].astype(np.uint64) >> np.uint64(32)).astype(np.int64) & 0xF
    hw = (a[:, 15].astype(np.uint64) & np.uint64(0xFFFFFFFF)).astype(np.int64)
    dur = a[:, 1] - a[:, 0]
    dmax = dur.max()
    out = {}
    for x in sorted(set(xcc.tolist())):
        m = xcc == x
        t0, t1 = a[m, 0], a[m, 1]
        out[str(x)] = {"waves": int(m.sum()), "start_skew": float((t0.max() - t0.min()) / dmax),
                       "end_spread": float((t1.max() - t1.min()) / dmax),
                       "span": float((t1.max() - t0.min()) / dmax), "mean_dur": float(dur[m].mean() / dmax)}
    out["by_wave_slot_mean_dur"] = {str(k): float(dur[(hw & 0xF) == k].mean() / dmax)
                                    for k in sorted(set((hw & 0xF).tolist()))}
    return out


def main() -> int:
    name = sys.argv[1] if len(sys.argv) > 1 else "c3"
    rays, traced, bounces, sr = SHAPES[name]
    s = RenderSettings(rays=rays, sample_rate=sr, base_power=3.62, max_bounces=bounces)
    r = AudioRenderer(s, scene=conference_standin(), receiver=receiver_local())
    r.setEmitterPosInOptix(CONFERENCE_EMITTER)
    r.setSphereCenterInOptix(CONFERENCE_LISTENER, 0.0)
    if os.environ.get("TRACE_PATH"):  # arx_debug_set_trace_path (0 BVH2 16-bit, 8 CW4)
        r.set_trace_path(int(os.environ["TRACE_PATH"]))
    for _ in range(3):  # warm-up, then the measured launch
        r.clear_histogram()
        r.trace_rays(0, traced)
    ms = float(r.trace_times(1)[0])
    n = 256 * 64 * W
    buf = (C.c_uint64 * n)()
    k = C.c_size_t()
    check(lib().arx_debug_trace_profile(r.handle, buf, n, C.byref(k)))
    a = np.frombuffer(buf, np.uint64).reshape(-1, W).astype(np.float64)
    a = a[a[:, 0] > 0]
    t0, t1 = a[:, 0], a[:, 1]
    dur = t1 - t0
    span = t1.max() - t0.min()
    exhaust = np.where(a[:, 12] > 0, a[:, 12], t0)
    slots = a[:, 4].sum()
    leaf_ph, shade_ph = a[:, 6].sum(), a[:, 8].sum()
    out = {
        "workload": name, "trace_path": int(os.environ.get("TRACE_PATH", "0")), "rays": traced, "bounces": bounces, "waves": int(a.shape[0]),
        "trace_ms_hip_events": ms,
        "clock_ticks_per_ms": span / ms,
        "span_ticks": span,
        "wave_duration": {"mean_over_span": float(dur.mean() / span), "median_over_span": float(np.median(dur) / span),
                          "min_over_span": float(dur.min() / span), "max_over_span": float(dur.max() / span),
                          "p10_over_span": float(np.percentile(dur, 10) / span)},
        # s_memtime counts per XCD (not comparable across waves): durations only
        "wave_duration_over_max": {"mean": float(dur.mean() / dur.max()), "median": float(np.median(dur) / dur.max()),
                                   "p10": float(np.percentile(dur, 10) / dur.max()),
                                   "p90": float(np.percentile(dur, 90) / dur.max()), "min": float(dur.min() / dur.max())},
        "max_wave_ticks": float(dur.max()),
        "per_xcd": per_xcd(a),
        "start_skew_over_span": float((t0.max() - t0.min()) / span),
        "after_range_ran_out_over_span": float(np.mean(t1 - exhaust) / span),
        "queries_per_wave": {"mean": float(a[:, 3].mean()), "min": float(a[:, 3].min()), "max": float(a[:, 3].max())},
        "lane_efficiency": {
            "node_steps": float(a[:, 5].sum() / (64 * slots)),
            "leaf_phases": float(a[:, 7].sum() / (64 * leaf_ph)) if leaf_ph else None,
            "shade_phases": float(a[:, 9].sum() / (64 * shade_ph)) if shade_ph else None,
        },
        "per_wave": {"node_step_slots": float(slots / a.shape[0]), "leaf_phases": float(leaf_ph / a.shape[0]),
                     "shade_phases": float(shade_ph / a.shape[0]), "refills": float(a[:, 14].sum() / a.shape[0]),
                     "outer_iterations": float(a[:, 10].sum() / a.shape[0]),
                     "inner_iterations": float(a[:, 11].sum() / a.shape[0])},
        "node_lane_steps_per_query": float(a[:, 5].sum() / a[:, 3].sum()),
    }
    js = json.dumps(out, indent=1)
    print(js)
    if len(sys.argv) > 2:
        with open(sys.argv[2], "w") as fh:
            fh.write(js)
    return 0


if __name__ == "__main__":
    sys.exit(main())
