"""The timed steps' trace launches in a rocprofv3 kernel trace of the default bench command (frames in
flight): how many run side by side, their durations and the period between launch starts.

With frames in flight a ray-pool launch is sized for half the CUs' wave slots (arx_stats.trace_grid_cus),
so two frames' launches should run concurrently for most of their length; this reads it off the trace.
usage: grid_overlap.py run_kernel_trace.csv bench.json > summary.json
"""
import csv
import json
import sys


def main(trace_csv, bench_json):
    d = json.loads(open(bench_json).read().strip().splitlines()[-1])
    rows = [r for r in csv.DictReader(open(trace_csv)) if r["Kernel_Name"].startswith("void arx::(anonymous namespace)::trace_kernel<128")]
    iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Grid_Size", r.get("Grid_Size_X", ""))) for r in rows)
    # the bench's first C3 segment: pre-roll, warmup, timed steps (frames in flight), then the
    # single-frame legs; the timed steps are the K launches before the single-frame leg's 2 (W + K)
    seg = [iv[0]]
    for a in iv[1:]:
        if a[0] - seg[-1][1] > 50_000_000:
            break
        seg.append(a)
    k, w = d["steps"], d["warmup"]
    single = 2 * (w + k)  # single_frame leg + kernel-times leg (one frame in flight)
    after = (d.get("convolution_input_reuse") is not None) + (d.get("host_buffers") is not None)
    end = len(seg) - single - after * (w + k)
    timed = seg[end - k:end]
    durs = [(e - b) / 1e6 for b, e, _ in timed]
    starts = [b for b, _, _ in timed]
    # launches running at once, averaged over the timed launches' span (sum of durations / span)
    span = max(e for _, e, _ in timed) - min(b for b, _, _ in timed)
    conc = sum(e - b for b, e, _ in timed) / span
    alone = seg[end:end + single]
    out = {
        "timed_launches": len(timed),
        "timed_grid": sorted(set(g for _, _, g in timed)),
        "single_frame_grid": sorted(set(g for _, _, g in alone)),
        "timed_avg_duration_ms": sum(durs) / len(durs),
        "timed_start_period_ms": (starts[-1] - starts[0]) / (len(starts) - 1) / 1e6,
        "timed_mean_concurrency": conc,
        "single_frame_avg_duration_ms": sum((e - b) / 1e6 for b, e, _ in alone) / len(alone),
        # the kernel-times leg (the last W + K of the single-frame launches) against the line's HIP events
        "kernel_times_leg_avg_ms": sum((e - b) / 1e6 for b, e, _ in alone[-k:]) / k,
        "bench_hip_events_ms": d["phases_ms_rank0"]["trace_kernel"],
        "all_trace_launches_avg_ms": sum((e - b) / 1e6 for b, e, _ in iv) / len(iv),
        "bench_ms_per_step": d["ms_per_step"],
        "bench_value": d["value"],
        "frames_in_flight": d["config"]["frames_in_flight"],
        "trace_grid_cus": d["config"].get("trace_grid_cus"),
    }
    out["agreement"] = out["kernel_times_leg_avg_ms"] / out["bench_hip_events_ms"] - 1.0
    json.dump(out, sys.stdout, indent=1)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
