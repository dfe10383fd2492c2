"""Per-kernel bytes of the convolution passes from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE
(tools/gpu_conv_pmc.sh), per call, FETCH_SIZE doubled (gfx950 tallies 128-B requests at 64 B,
MI355X_MICROARCH.md), against the reference algorithm's 52 B per stereo frame."""
import collections
import csv
import glob
import json
import os
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/conv_pmc"
per = collections.defaultdict(lambda: collections.defaultdict(list))
for grp in ("FETCH_SIZE", "WRITE_SIZE"):
    for f in glob.glob(os.path.join(root, grp, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                name = r["Kernel_Name"].replace("void ", "").replace("arx::(anonymous namespace)::", "").split("(")[0]
                if not any(k in name for k in ("pass_", "finalize")):
                    continue
                per[name][grp].append(float(r["Counter_Value"]) * 1024)  # KB -> B
out = {}
total = 0.0
for name, d in sorted(per.items()):
    fetch = 2 * sum(d["FETCH_SIZE"]) / max(1, len(d["FETCH_SIZE"]))
    write = sum(d["WRITE_SIZE"]) / max(1, len(d["WRITE_SIZE"]))
    out[name] = {"fetch_bytes": fetch, "write_bytes": write}
    total += fetch + write
frames = 807498
out["total_bytes_per_step"] = total
out["algorithmic_bytes_per_step"] = 52 * frames
out["ratio"] = total / (52 * frames)
# the guard bench.py checks (bench.conv_profile_guard): workload and the convolution kernels' identity
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from audiorenderingv2_amd._lib import lib  # noqa: E402

out["workload"] = "c3"
out["conv_kernel_id"] = f"{int(lib().arx_conv_kernel_id()):016x}"
out["method"] = ("tools/gpu_conv_pmc.sh: rocprofv3 --pmc FETCH_SIZE (x2, gfx950 128-B requests tallied at 64 B) and "
                 "WRITE_SIZE in separate passes, per pass of the C3 convolution (tools/conv_once.py, IR spectra "
                 "included)")
print(json.dumps(out, indent=1))
