#!/usr/bin/env python3
"""A/B the trace-kernel variants (ARX_TRACE_KERNEL) on the bench workload; every variant
must reproduce variant 1's IR and query count bit for bit."""
import os
import sys
import time
import zlib

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from audiorenderingv2_amd import AudioRenderer, RenderSettings, conference_standin, receiver_local  # noqa: E402
from audiorenderingv2_amd.scene import CONFERENCE_EMITTER, CONFERENCE_LISTENER  # noqa: E402


def main():
    variants = [v if ":" in v else int(v) for v in (sys.argv[1].split(",") if len(sys.argv) > 1 else "1,2,3,4,5,6,7".split(","))]
    sr = int(os.environ.get("SR", "48000"))
    rays = tuple(int(x) for x in os.environ.get("RAYS", "100,100,100").split(","))
    bounces = int(os.environ.get("BOUNCES", "16"))
    s = RenderSettings(rays=rays, sample_rate=sr, base_power=3.62, max_bounces=bounces)
    r = AudioRenderer(s, scene=conference_standin(), receiver=receiver_local())
    r.setEmitterPosInOptix(CONFERENCE_EMITTER)
    r.setSphereCenterInOptix(CONFERENCE_LISTENER, 0.0)
    ref = None
    for v in variants:
        label = v
        if isinstance(v, str) and ":" in v:  # "variant:ENV=value"
            v, kv = v.split(":", 1)
            k, val = kv.split("=", 1)
            os.environ[k] = val
        os.environ["ARX_TRACE_KERNEL"] = str(v)
        for _ in range(2):
            r.render()
        ms = sorted(r.render() for _ in range(7))
        ir = r.get_ir()
        st = r.stats()
        if ref is None:
            ref = (ir, st["queries"])
        same = np.array_equal(ir[0], ref[0][0]) and np.array_equal(ir[1], ref[0][1]) and st["queries"] == ref[1]
        print(f"variant {label}: median {ms[3]:.3f} ms min {ms[0]:.3f} ms  {st['queries'] / ms[3] / 1e6:.3f} Gq/s  "
              f"identical={same}  ir_crc={zlib.crc32(ir[0].tobytes() + ir[1].tobytes()):08x}", flush=True)
        if not same:
            raise SystemExit(f"variant {v} differs from variant {variants[0]}")


if __name__ == "__main__":
    main()
