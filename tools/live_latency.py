#!/usr/bin/env python3
"""Latency of one live (mic) block convolution (convoluteLiveInput, AudioRenderer.cpp:593-661):
host path (H2D + passes A-D + D2H + sync) and device path (passes only, + sync), per call,
for 4096-sample blocks at 44.1 / 48 / 16 kHz with 2-s IRs."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from audiorenderingv2_amd import AudioRenderer, RenderSettings  # noqa: E402


def main():
    import torch

    for sr in (44100, 48000, 16000):
        r = AudioRenderer(RenderSettings(rays=(1, 1, 1), sample_rate=sr, ir_length_in_seconds=2))
        rng = np.random.default_rng(0)
        n = 2 * sr
        irs = [np.zeros(n, np.float32) for _ in range(2)]
        for ir in irs:
            ir[rng.integers(0, n, 500)] = rng.exponential(1e-3, 500).astype(np.float32)
        r.set_ir(*irs)
        x = rng.uniform(-1, 1, 4096)
        for _ in range(20):
            r.convoluteLiveInput(x)
        host = []
        for _ in range(200):
            t0 = time.perf_counter()
            r.convoluteLiveInput(x)
            host.append(time.perf_counter() - t0)
        dx = torch.from_numpy(x).cuda()
        dy = torch.empty(2 * n, dtype=torch.float64, device="cuda")
        torch.cuda.synchronize()
        stream = torch.cuda.ExternalStream(r.get_stream())
        dev = []
        for _ in range(200):
            t0 = time.perf_counter()
            r.convolute_live_device(dx.data_ptr(), x.size, dy.data_ptr())
            stream.synchronize()
            dev.append(time.perf_counter() - t0)
        host = np.sort(np.array(host)) * 1e6
        dev = np.sort(np.array(dev)) * 1e6
        print(f"sr {sr}: host path p50 {host[100]:.0f} us p99 {host[198]:.0f} us | "
              f"device path p50 {dev[100]:.0f} us p99 {dev[198]:.0f} us", flush=True)


if __name__ == "__main__":
    main()
