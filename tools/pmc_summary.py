"""Summarise rocprofv3 --pmc csv output of the trace kernel (tools/gpu_pmc_state.sh).

    python tools/pmc_summary.py gpurun_out/pmcs [td.json guard.json]

Per variant: every counter averaged per trace-kernel dispatch, plus derived ratios
(per-CU busy fractions, VALU/SALU per wave-cycle, L2 hit rate, mean L2 read latency).
"""
import collections
import csv
import glob
import json
import os
import sys


def load(root):
    per = collections.defaultdict(dict)  # variant -> counter -> value per dispatch
    for f in glob.glob(os.path.join(root, "v*_*", "**", "*counter_collection.csv"), recursive=True):
        variant = os.path.relpath(f, root).split(os.sep)[0].split("_")[0]
        sums = collections.defaultdict(float)
        disp = set()
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if "trace_kernel" not in r.get("Kernel_Name", ""):
                    continue
                sums[r["Counter_Name"]] += float(r["Counter_Value"])
                disp.add(r["Dispatch_Id"])
        for k, v in sums.items():
            per[variant][k] = v / max(1, len(disp))
    return per


def main():
    root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmcs"
    cus = 256
    data = load(root)
    if len(sys.argv) > 3:  # --json: the product variant's TD / TA busy fractions + the run's guard
        c = data["vprod"]
        g = c["GRBM_GUI_ACTIVE"] / 8
        guard = json.load(open(sys.argv[3]))
        out = {"workload": guard.get("workload"), "tree_hash": guard.get("tree_hash"),
               "trace_vgprs": guard.get("trace_vgprs"), "trace_kernel_id": guard.get("trace_kernel_id"), "kernel": "trace_kernel (16-bit BVH2, LDS stack)",
               "td_busy_per_cu_cycle": c["TD_TD_BUSY_sum"] / cus / g, "ta_busy_per_cu_cycle": c["TA_TA_BUSY_sum"] / cus / g,
               "l2_hit_rate": c["TCC_HIT_sum"] / (c["TCC_HIT_sum"] + c["TCC_MISS_sum"]),
               "sq_wait_any_per_wave_cycle": c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"],
               "valu_active_per_wave_cycle": c["SQ_ACTIVE_INST_VALU"] / c["SQ_WAVE_CYCLES"],
               "valu_instructions": c["SQ_INSTS_VALU"],
               # a wave64 VALU instruction holds a 16-lane SIMD for 4 cycles: the SIMDs' VALU issue
               # fraction over the kernel's cycles (GRBM_GUI_ACTIVE / 8 = cycles per XCD)
               "kernel_cycles_per_xcd": g,
               "valu_busy_per_simd_cycle": c["SQ_INSTS_VALU"] * 4.0 / (cus * 4) / g,
               # the tracked copy bench.py reads (the tool writes under gpurun_out/ on the GPU box)
               "source": "profiles/" + sys.argv[2].split("gpurun_out/", 1)[-1]}
        with open(sys.argv[2], "w") as fh:
            json.dump(out, fh, indent=1)
    for variant, c in sorted(data.items()):
        print(f"== {variant}")
        for k in sorted(c):
            print(f"  {k:34s} {c[k]:.4g}")
        g = c.get("GRBM_GUI_ACTIVE", 0) / 8  # summed over 8 XCDs
        if g:
            print(f"  kernel cycles (per XCD)            {g:.4g}")
            for k in ("TA_TA_BUSY_sum", "TD_TD_BUSY_sum"):
                if k in c:
                    print(f"  {k} per CU / cycles        {c[k] / cus / g:.3f}")
        if "SQ_WAVE_CYCLES" in c:
            wc = c["SQ_WAVE_CYCLES"]
            for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
                      "SQ_ACTIVE_INST_SCA", "SQ_ACTIVE_INST_VMEM", "SQ_ACTIVE_INST_LDS", "SQ_WAIT_INST_LDS"):
                if k in c:
                    print(f"  {k:34s} / wave-cycles {c[k] / wc:.3f}")
        if "TCC_HIT_sum" in c and "TCC_MISS_sum" in c:
            print(f"  L2 hit rate                        {c['TCC_HIT_sum'] / (c['TCC_HIT_sum'] + c['TCC_MISS_sum']):.3f}")
        if "TCP_UTCL1_TRANSLATION_MISS_sum" in c and "TCP_UTCL1_REQUEST_sum" in c:
            print(f"  UTCL1 translation miss rate        {c['TCP_UTCL1_TRANSLATION_MISS_sum'] / max(1, c['TCP_UTCL1_REQUEST_sum']):.4f}")
        if "TCP_TCC_READ_REQ_sum" in c and "TCP_TCC_READ_REQ_LATENCY_sum" in c:
            print(f"  mean L2 read latency (cycles)      {c['TCP_TCC_READ_REQ_LATENCY_sum'] / c['TCP_TCC_READ_REQ_sum']:.1f}")


if __name__ == "__main__":
    main()
