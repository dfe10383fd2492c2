#!/usr/bin/env python3
"""Per-kernel duration summary (rocprofv3 --stats style CSV) from a rocprofv3 rocpd database.

    python tools/rocpd_stats.py gpurun_out/prof/run_results.db > profiles/xxx_kernel_stats.csv
"""
import sqlite3
import sys


def main(path: str) -> int:
    c = sqlite3.connect(path)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name_col = "kernel_name" if "kernel_name" in cols else "name"
    rows = c.execute(f"select {name_col}, start, end from kernels").fetchall()
    agg = {}
    for name, s, e in rows:
        d = int(e) - int(s)
        a = agg.setdefault(name, [0, 0, None, 0])
        a[0] += 1
        a[1] += d
        a[2] = d if a[2] is None else min(a[2], d)
        a[3] = max(a[3], d)
    total = sum(v[1] for v in agg.values()) or 1
    print('"Name","Calls","TotalDurationNs","AverageNs","Percentage","MinNs","MaxNs"')
    for name, (n, tot, mn, mx) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print(f'"{name}",{n},{tot},{tot / n:.1f},{100.0 * tot / total:.4f},{mn},{mx}')
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1]))
