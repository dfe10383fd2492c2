#!/usr/bin/env python3
"""Where the C3 file convolution's time goes, per workgroup: a measurement build
(build.py --exp cprof -D ARX_CONV_PROF=1) stamps every workgroup of passes A / B / C with the device's
100-MHz real-time counter at entry, once its loads are in LDS, after its FFT and after its last store.
The bench step is replayed (clear + trace of 1M x 16 + finalize + IR spectra + convolution of
A_Clapper_Board.wav ch0), so the caches hold what they hold in the bench; the records of the last
step's convolution are reported:

  * per pass: span (first entry -> last store), entry skew (last - first workgroup entry), the gap to
    the previous pass, and the median / max per-workgroup load, FFT and store phases.

    ARX_LIB=tools/experiments/lib/libarx_cprof.so python tools/conv_phases.py [steps] [out.json]
"""
import ctypes as C
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from audiorenderingv2_amd._lib import use_library  # noqa: E402

use_library(os.environ.get("ARX_LIB", os.path.join(REPO, "tools", "experiments", "lib", "libarx_cprof.so")))
from audiorenderingv2_amd import AudioRenderer, DeviceBuffer, RenderSettings, conference_standin, receiver_local  # noqa: E402
from audiorenderingv2_amd._lib import lib  # noqa: E402
from audiorenderingv2_amd.scene import CONFERENCE_EMITTER, CONFERENCE_LISTENER, reference_audio  # noqa: E402

SLOT, PASS = 8, 4096 * 8
TICK_US = 0.01  # s_memrealtime: 100 MHz


def phases(rec: np.ndarray) -> dict:
    t = rec[:, :4].astype(np.float64) * TICK_US
    t0 = t[:, 0].min()
    return {
        "workgroups": int(len(rec)),
        "first_entry_us": 0.0,
        "span_us": float(t[:, 3].max() - t0),
        "entry_skew_us": float(t[:, 0].max() - t0),
        "load_us": [float(np.median(t[:, 1] - t[:, 0])), float((t[:, 1] - t[:, 0]).max())],
        "fft_us": [float(np.median(t[:, 2] - t[:, 1])), float((t[:, 2] - t[:, 1]).max())],
        "store_us": [float(np.median(t[:, 3] - t[:, 2])), float((t[:, 3] - t[:, 2]).max())],
        "wg_total_us": [float(np.median(t[:, 3] - t[:, 0])), float((t[:, 3] - t[:, 0]).max())],
        "t0_abs_us": float(t0), "t_end_abs_us": float(t[:, 3].max()),
    }


def main() -> int:
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    f = lib().arx_exp_conv_profile
    f.argtypes = [C.POINTER(C.c_ulonglong), C.c_size_t]
    f.restype = C.c_int
    x, sr = reference_audio("clapper")
    s = RenderSettings(rays=(100, 100, 100), sample_rate=sr, base_power=3.62, max_bounces=16, hrtf_absorption_rate=1.0)
    r = AudioRenderer(s, scene=conference_standin(), receiver=receiver_local())
    r.setEmitterPosInOptix(CONFERENCE_EMITTER)
    r.setSphereCenterInOptix(CONFERENCE_LISTENER, 0.0)
    dx = DeviceBuffer.from_numpy(0, x)
    dl, dr = DeviceBuffer(0, 4 * x.size), DeviceBuffer(0, 4 * x.size)
    buf = np.zeros(3 * PASS, np.uint64)
    for k in range(steps):
        if k == steps - 1:
            r.stats()
            f(buf.ctypes.data_as(C.POINTER(C.c_ulonglong)), buf.size)  # clear
        r.render()
        r.convolute_device(dx.ptr, x.size, dl.ptr, dr.ptr)
    r.stats()
    f(buf.ctypes.data_as(C.POINTER(C.c_ulonglong)), buf.size)
    conv_ms = float(r.conv_times(1)[0])
    out = {"conv_window_us": conv_ms * 1e3, "plan": r.conv_plan(), "passes": {}}
    prev_end = None
    for k, name in enumerate(("A", "B", "C")):
        rec = buf[k * PASS:(k + 1) * PASS].reshape(-1, SLOT)
        rec = rec[rec[:, 0] != 0]
        if len(rec) == 0:
            continue
        ph = phases(rec)
        ph["xcds"] = int(len(set(rec[:, 4].tolist())))
        if prev_end is not None:
            ph["gap_from_previous_pass_us"] = ph["t0_abs_us"] - prev_end
        prev_end = ph["t_end_abs_us"]
        out["passes"][name] = ph
    t_first = min(p["t0_abs_us"] for p in out["passes"].values())
    for p in out["passes"].values():
        p["first_entry_us"] = p["t0_abs_us"] - t_first
        del p["t0_abs_us"], p["t_end_abs_us"]
    txt = json.dumps(out, indent=1)
    print(txt)
    if len(sys.argv) > 2:
        with open(sys.argv[2], "w") as fh:
            fh.write(txt)
    r.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
