#!/usr/bin/env python3
"""profiles/r03/trace_traffic.json from rocprofv3 PMC passes of the bench workload (tools/trace_once.py).

HBM-side bytes per trace launch = corrected FETCH_SIZE + WRITE_SIZE, following
/opt/skills/guides/MI355X_MICROARCH.md (HBM / rocprofv3): on gfx950 FETCH_SIZE counts
TCC_EA0_RDREQ x 64 B while the requests are 128 B, so it is doubled; WRITE_SIZE is exact for
the histogram's one-dword atomics.  Infinity-Cache hits are included (the guide: they are
counted, not excluded), so this is an upper bound on HBM traffic.

    python tools/make_traffic.py gpurun_out/pmc_traffic [workload] [out.json] [guard.json]

guard.json (tools/trace_once.py ARX_GUARD_OUT) carries the profiled run's tree hash and trace kernel
VGPRs; bench.py reports the traffic only for a run that matches them.
"""
import csv
import glob
import json
import os
import sys


def per_launch(root: str) -> dict:
    vals = {}
    for f in glob.glob(os.path.join(root, "*", "p_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if "trace_kernel" not in r["Kernel_Name"]:
                continue
            vals.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
            vals.setdefault("_kernel", r["Kernel_Name"])
    return vals


def main() -> int:
    root = sys.argv[1]
    workload = sys.argv[2] if len(sys.argv) > 2 else "c3"
    v = per_launch(root)
    avg = {k: sum(x) / len(x) for k, x in v.items() if k != "_kernel"}
    fetch_kb = avg.get("FETCH_SIZE")
    write_kb = avg.get("WRITE_SIZE")
    if fetch_kb is None or write_kb is None:
        print("FETCH_SIZE / WRITE_SIZE missing", file=sys.stderr)
        return 1
    out = {
        "workload": workload,
        "kernel": v.get("_kernel"),
        "fetch_size_kb": fetch_kb,
        "write_size_kb": write_kb,
        "tcc_ea0_rdreq": avg.get("TCC_EA0_RDREQ_sum"),
        "bytes_per_launch": 2.0 * fetch_kb * 1024.0 + write_kb * 1024.0,
        "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes), FETCH_SIZE x2 (gfx950 128-B "
                  "requests tallied at 64 B), Infinity-Cache hits included: upper bound on HBM bytes",
    }
    if len(sys.argv) > 4:
        with open(sys.argv[4]) as fh:
            guard = json.load(fh)
        out.update({k: guard[k] for k in ("tree_hash", "trace_vgprs", "trace_kernel_id") if k in guard})
    path = sys.argv[3] if len(sys.argv) > 3 else os.path.join(
        os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles", "r03", "trace_traffic.json")
    with open(path, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out))
    return 0


if __name__ == "__main__":
    sys.exit(main())
