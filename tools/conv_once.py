#!/usr/bin/env python3
"""Run the C3 file convolution a few times on device buffers (for profilers): A_Clapper_Board.wav
channel 0 (807 498 frames, 48 kHz) with a rendered-like sparse stereo IR of 96 000 bins; the IR
is re-set before every run, so each run includes the IR spectra, as in a bench step."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from audiorenderingv2_amd import AudioRenderer, DeviceBuffer, RenderSettings  # noqa: E402
from audiorenderingv2_amd.scene import reference_audio  # noqa: E402
from audiorenderingv2_amd._lib import use_library  # noqa: E402

if os.environ.get("ARX_LIB"):  # a design-experiment build (tools only)
    use_library(os.environ["ARX_LIB"])

n = int(sys.argv[1]) if len(sys.argv) > 1 else 3
x, sr = reference_audio("clapper")
if os.environ.get("CONV_FRAMES"):  # a shorter signal (fewer block pairs), for the per-pair scaling
    x = np.ascontiguousarray(x[:int(os.environ["CONV_FRAMES"])])
r = AudioRenderer(RenderSettings(rays=(1, 1, 1), sample_rate=sr, ir_length_in_seconds=2))
rng = np.random.default_rng(0)
irs = []
for _ in range(2):
    ir = np.zeros(2 * sr, np.float32)
    ir[rng.integers(0, 2 * sr, 20000)] = rng.exponential(1e-4, 20000).astype(np.float32)
    irs.append(ir)
# device buffers of libarx itself (no second GPU framework in the process)
dx = DeviceBuffer.from_numpy(0, x)
dl, dr = DeviceBuffer(0, x.nbytes), DeviceBuffer(0, x.nbytes)
ms = []
for _ in range(n):
    r.set_ir(*irs)
    r.convolute_device(dx.ptr, x.size, dl.ptr, dr.ptr)
    r.stats()  # synchronises the renderer's stream
    ms.append(r.conv_times(1)[0])
print(f"frames {x.size} conv {np.median(ms[1:] if n > 1 else ms) * 1e3:.1f} us (median of {max(n - 1, 1)}) "
      f"checksum {float(np.abs(dl.to_numpy(np.float32).astype(np.float64)).sum() + np.abs(dr.to_numpy(np.float32).astype(np.float64)).sum()):.9e} "
      f"lib {os.path.basename(os.environ.get('ARX_LIB', 'libarx.so'))}", flush=True)
