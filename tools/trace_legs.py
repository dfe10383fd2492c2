"""Per-leg trace-kernel durations from a rocprofv3 kernel trace of the default bench command.

The bench's timed loop runs frames in flight, whose trace launches start while the previous frame's
is still draining, so a launch's own duration there is not its time on the GPU; the per-launch time
and the roofline come from the kernel-times leg (W + K single-frame launches with the renderer's
timing events on, followed by the input-reuse and host-buffer legs' W + K each when those ran; one
stream, no overlap).  This prints both, for comparison with the line's phases_ms_rank0.trace_kernel.
usage: trace_legs.py run_kernel_trace.csv bench.json > summary.json
"""
import csv
import json
import sys


def main(trace_csv, bench_json):
    d = json.load(open(bench_json))
    wk = d["steps"] + d["warmup"]
    rows = [r for r in csv.DictReader(open(trace_csv)) if r["Kernel_Name"].startswith("void arx::(anonymous namespace)::trace_kernel<128")]
    iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Stream_Id"]) for r in rows)
    first = [iv[0]]  # the C3 frames: pre-roll, timed frames in flight, single-frame leg (before the C5 walk)
    for a in iv[1:]:
        if a[0] - first[-1][1] > 50_000_000:
            break
        first.append(a)
    after = (d.get("convolution_input_reuse") is not None) + (d.get("host_buffers") is not None)
    single = first[-wk * (after + 1):len(first) - wk * after]
    ms = [(e - b) / 1e6 for b, e, _ in single]
    assert all(single[i][0] >= single[i - 1][1] for i in range(1, len(single))), "kernel-times leg overlaps"
    allms = [(e - b) / 1e6 for b, e, _ in first]
    out = {
        "trace_launches_c3": len(first),
        "overlapping_launches": sum(1 for i in range(1, len(first)) if first[i][0] < first[i - 1][1]),
        "all_c3_avg_ms": sum(allms) / len(allms),
        "kernel_times_leg": {"launches": wk, "avg_ms": sum(ms) / len(ms), "min_ms": min(ms), "max_ms": max(ms)},
        "bench_hip_events_ms": d["phases_ms_rank0"]["trace_kernel"],
        "bench_value": d["value"],
        "frames_in_flight": d["config"]["frames_in_flight"],
    }
    out["agreement"] = out["kernel_times_leg"]["avg_ms"] / out["bench_hip_events_ms"] - 1.0
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
