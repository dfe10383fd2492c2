#!/usr/bin/env python3
"""Where a single-frame step's time goes between kernels (the launch gaps a HIP graph could at most
recover), from a rocprofv3 kernel trace.

    python tools/step_gaps.py run c2|c3 [steps]          # the steps, one frame in flight
                                                         # (STEP_GAPS_TIMING=0: timing events off)
    rocprofv3 --kernel-trace -d DIR -o run -- python3 tools/step_gaps.py run c2 40
    python tools/step_gaps.py analyze DIR/.../run_kernel_trace.csv [steps] > summary.json

A step = render (clear, direction pre-pass, trace, finalize) + the file convolution (IR spectra and
the three passes), all on the renderer's stream.  The analysis takes the last `steps` steps (each
begins with the direction pre-pass, or the histogram clear before it), and per step reports the wall span from the first kernel's start to
the last one's end, the kernels' summed durations and the difference: the time the stream spent
between kernels.
"""
import csv
import json
import os
import sys

import numpy as np


def run(workload: str, steps: int) -> None:
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from audiorenderingv2_amd import AudioRenderer, RenderSettings, conference_standin, receiver_local
    from audiorenderingv2_amd.renderer import DeviceBuffer
    from audiorenderingv2_amd.scene import CONFERENCE_EMITTER, CONFERENCE_LISTENER, reference_audio
    from audiorenderingv2_amd._lib import check, lib, use_library
    if os.environ.get("ARX_LIB"):  # a design-experiment build (tools only)
        use_library(os.environ["ARX_LIB"])

    rays, bounces, sr, audio = {"c2": ((100, 100, 10), 8, 16000, "experimento"),
                                "c3": ((100, 100, 100), 16, 48000, "clapper")}[workload]
    s = RenderSettings(rays=rays, sample_rate=sr, base_power=3.62, max_bounces=bounces, hrtf_absorption_rate=1.0,
                       ir_length_in_seconds=2)
    r = AudioRenderer(s, scene=conference_standin(), receiver=receiver_local())
    r.setEmitterPosInOptix(CONFERENCE_EMITTER)
    r.setSphereCenterInOptix(CONFERENCE_LISTENER, 0.0)
    if os.environ.get("STEP_GAPS_TIMING", "1") == "0":
        r.set_timing(False)  # no per-launch event markers (arx_set_timing)
    x, asr = reference_audio(audio)
    assert asr == sr
    dx = DeviceBuffer.from_numpy(0, x)
    ol, orr = DeviceBuffer(0, 4 * x.size), DeviceBuffer(0, 4 * x.size)
    try:
        for _ in range(steps + 10):  # 10 untimed steps first (clock ramp)
            check(lib().arx_render(r.handle, None))  # no host wait between the render and the convolution
            r.convolute_device(dx.ptr, x.size, ol.ptr, orr.ptr)
            r.stats()  # one frame at a time: the host waits for the step
        print(json.dumps({"workload": workload, "steps": steps}))
    finally:
        for b in (dx, ol, orr):
            b.close()
        r.close()


def analyze(trace_csv: str, steps: int) -> None:
    rows = [r for r in csv.DictReader(open(trace_csv)) if "arx::" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    # a step begins with its direction pre-pass, or with the histogram clear right before it (builds
    # whose render() still launches the clear separately)
    starts = []
    for i, r in enumerate(rows):
        if "dirs_kernel" in r["Kernel_Name"]:
            starts.append(i - 1 if i > 0 and "clear_kernel" in rows[i - 1]["Kernel_Name"] else i)
    starts = starts[-(steps + 1):]  # step k = [starts[k], starts[k + 1])
    spans, busy, per_kernel, gaps = [], [], {}, {}
    for a, b in zip(starts, starts[1:]):
        ks = rows[a:b]
        t0, t1 = int(ks[0]["Start_Timestamp"]), max(int(k["End_Timestamp"]) for k in ks)
        spans.append((t1 - t0) / 1e3)
        busy.append(sum(int(k["End_Timestamp"]) - int(k["Start_Timestamp"]) for k in ks) / 1e3)
        for k in ks:
            name = k["Kernel_Name"].replace("void ", "").replace("arx::(anonymous namespace)::", "").split("(")[0]
            per_kernel.setdefault(name, []).append((int(k["End_Timestamp"]) - int(k["Start_Timestamp"])) / 1e3)
        for j in range(1, len(ks)):  # the gap before each kernel, by the kernel's name
            name = ks[j]["Kernel_Name"].replace("void ", "").replace("arx::(anonymous namespace)::", "").split("(")[0]
            gaps.setdefault(name, []).append((int(ks[j]["Start_Timestamp"]) - int(ks[j - 1]["End_Timestamp"])) / 1e3)
    spans, busy = np.array(spans), np.array(busy)
    out = {"steps": len(spans), "launches_per_step": (starts[-1] - starts[0]) / max(1, len(spans)),
           "span_us_median": float(np.median(spans)), "kernels_us_median": float(np.median(busy)),
           "between_kernels_us_median": float(np.median(spans - busy)),
           "per_kernel_us_median": {k: float(np.median(v)) for k, v in per_kernel.items()},
           "gap_before_us_median": {k: float(np.median(v)) for k, v in gaps.items()}}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 40)
    else:
        analyze(sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 40)
