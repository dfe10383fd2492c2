#!/usr/bin/env python3
"""Vector-memory ceiling of the trace kernel, calibrated on this GPU.

    python tools/vmem_ceiling.py profiles/r02/td_microbench_sizes.txt profiles/r03/pmc_state_r03.txt \
        profiles/r03/trace_counts_c3.json [guard.json] > profiles/r03/trace_vmem_ceiling.json

guard.json (tools/trace_once.py ARX_GUARD_OUT of the PMC run) adds the tree hash and the trace
kernel's VGPRs, which bench.py checks against its own run.

The trace kernel's node and triangle fetches are divergent 16-B gathers (one 64-B block per lane).
tools/td_microbench.hip measures the rate of such gathers when they hit in L1 (16 KB table), in
L2 (2 MB table) and in the Infinity Cache (16 MB table).  The kernel's own mix comes from its PMC
counters: lane loads per launch (counting build), L1 -> L2 requests (TCP_TCC_READ_REQ) and L2
misses (TCC_MISS).  The ceiling is the mix's harmonic rate:
    1 / (f_L1 / R_L1 + f_L2 / R_L2 + f_MALL / R_MALL)  16-B lane loads per second.
"""
import json
import re
import sys


def rates(log):
    out, size = {}, None
    for line in open(log):
        m = re.match(r"-- table (\d+) KB", line)
        if m:
            size = int(m.group(1))
        m = re.match(r"64 distinct blocks/instr, 64 lanes.*\s([0-9.e+]+) 16-B lane loads/s", line)
        if m and size is not None:
            out[size] = float(m.group(1))
    return out


def pmc(path):
    vals = {}
    for line in open(path):
        parts = line.split()
        if len(parts) == 2 and parts[0] in ("TCP_TCC_READ_REQ_sum", "TCC_HIT_sum", "TCC_MISS_sum"):
            vals[parts[0]] = float(parts[1])
    return vals


def main():
    r = rates(sys.argv[1])
    p = pmc(sys.argv[2])
    c = json.load(open(sys.argv[3]))
    lane_loads = c["lane_loads_16B_per_query"] * c["queries"]
    f_l2 = p["TCP_TCC_READ_REQ_sum"] / lane_loads
    miss = p["TCC_MISS_sum"] / (p["TCC_HIT_sum"] + p["TCC_MISS_sum"])
    f_mall = f_l2 * miss
    f_l2hit = f_l2 - f_mall
    f_l1 = 1.0 - f_l2
    r1, r2, r3 = r[16], r[2048], r[16384]
    ceiling = 1.0 / (f_l1 / r1 + f_l2hit / r2 + f_mall / r3)
    guard = json.load(open(sys.argv[4])) if len(sys.argv) > 4 else {}
    print(json.dumps({
        "workload": c["workload"],
        **{k: guard[k] for k in ("tree_hash", "trace_vgprs", "trace_kernel_id") if k in guard},
        "lane_loads_per_launch": lane_loads,
        "fraction_l1": f_l1, "fraction_l2_hit": f_l2hit, "fraction_l2_miss": f_mall,
        "rate_l1_lane_loads_per_s": r1, "rate_l2_lane_loads_per_s": r2, "rate_mall_lane_loads_per_s": r3,
        "ceiling_lane_loads_per_s": ceiling,
        "sources": sys.argv[1:4],
    }, indent=1))


if __name__ == "__main__":
    main()
