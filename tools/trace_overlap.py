#!/usr/bin/env python3
"""From a rocprofv3 kernel trace (CSV) of bench.py: the trace kernel's launches in time order, each
one's duration, and the gap from the previous launch's end to its start (negative: the launches
overlap -- two frames in flight).  Summarised over the launches of the bench's timed and warmup
steps (the last n_launches).

    python tools/trace_overlap.py run_kernel_trace.csv [n_launches [skip_last]] > overlap.json
(skip_last: launches at the end to leave out, e.g. bench.py's single-frame leg after its timed steps)
"""
import csv
import json
import sys

import numpy as np

rows = [r for r in csv.DictReader(open(sys.argv[1])) if "trace_kernel<" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
n = int(sys.argv[2]) if len(sys.argv) > 2 else len(rows)
skip = int(sys.argv[3]) if len(sys.argv) > 3 else 0
rows = rows[len(rows) - skip - n:len(rows) - skip]
s = np.array([int(r["Start_Timestamp"]) for r in rows], np.float64) * 1e-6
e = np.array([int(r["End_Timestamp"]) for r in rows], np.float64) * 1e-6
dur = e - s
gap = s[1:] - e[:-1]
period = (e[-1] - e[0]) / (len(e) - 1) if len(e) > 1 else float("nan")
print(json.dumps({
    "launches": len(rows),
    "duration_ms": {"mean": float(dur.mean()), "min": float(dur.min()), "max": float(dur.max())},
    "gap_to_previous_end_ms": {"mean": float(gap.mean()), "min": float(gap.min()), "max": float(gap.max()),
                               "overlapping": int((gap < 0).sum())},
    "end_to_end_period_ms": period,
    "method": __doc__.strip().splitlines()[0],
}, indent=1))
