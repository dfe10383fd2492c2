"""Price the build's IEEE convention against the reference's compiled arithmetic.

For C2 (in full), C3 (the whole 1M x 16 launch) and C4 (a 1M-ray slice of the 10M x 32 launch, rays
5M..6M: rays 0..1M are C3's own rays, same ids, same directions) the CPU oracle traces the same Philox
rays four ways (arx_oracle.h `arith`):
  0  the build's IEEE convention (bit-exact with the GPU kernel),
  1  the reference's fast-math arithmetic (devicePrograms.cu as compiled: FMA, .approx div/sqrt),
  2  IEEE with the reflection about normalize(cr) as the reference writes it (devicePrograms.cu:77,
     173) -- the convention before round 3, to price the reflection about cr on its own,
  and mode 0 on seed 2: the Monte-Carlo spread between two runs of the clock-seeded reference.
Per ray it keeps the final record (its closest-hit triangle sequence hashed), so every ray is classed
as identical, same path with a bin flip (roundf((dist / 343) * sr) on the other side of a .5
boundary), or diverged (another path), and each class's share of the IR's per-bin relative RMS is
reported beside the bin-tolerant RMS of the same-path rays (oracle/pricing.py); the bars of DESIGN.md
section 3 are evaluated per config (round 5).

    python tools/arith_pricing.py [--out profiles/r05/ieee_vs_reference_arith.json]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle"))

import pyoracle as po  # noqa: E402
from pricing import BARS, BIN_FLIP_DX, OTHER_PATH_VS_REFERENCE_FORM, bars_met, compare, records  # noqa: E402
from audiorenderingv2_amd import place_receiver_vertices, receiver_local  # noqa: E402
from audiorenderingv2_amd.scene import CONFERENCE_EMITTER, CONFERENCE_LISTENER, conference_standin  # noqa: E402

CONFIGS = {  # BASELINE.json configs[1..3]; hrtf 0.5 so both ears carry a cross term
    "C2": dict(rays=(100, 100, 10), sr=16000, bounces=8),
    "C3": dict(rays=(100, 100, 100), sr=48000, bounces=16),
    "C4": dict(rays=(1000, 100, 100), sr=48000, bounces=32),
}
HRTF = 0.5


def world():
    sc = conference_standin()
    L, R = receiver_local()
    Lw = place_receiver_vertices(L.reshape(-1, 3), CONFERENCE_LISTENER, 0.0).reshape(-1, 9)
    Rw = place_receiver_vertices(R.reshape(-1, 3), CONFERENCE_LISTENER, 0.0).reshape(-1, 9)
    tv = np.concatenate([sc.tri_v, Lw, Rw]).astype(np.float32)
    ta = np.concatenate([sc.tri_abs, np.full(len(Lw), -1, np.float32), np.full(len(Rw), -2, np.float32)])
    return tv, ta


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(REPO, "profiles", "r05", "ieee_vs_reference_arith.json"))
    ap.add_argument("--c3-rays", type=int, default=1_000_000)
    ap.add_argument("--c4-begin", type=int, default=5_000_000)
    ap.add_argument("--c4-rays", type=int, default=1_000_000)
    ap.add_argument("--configs", default="C2,C3,C4")
    ap.add_argument("--threads", type=int, default=os.cpu_count() or 8)
    args = ap.parse_args(argv)
    tv, ta = world()
    osc = po.Scene(tv, ta, bvh=True)
    res = {"scene_triangles": int(len(ta)), "hrtf": HRTF, "seed": 1,
           "modes": {"0": "build IEEE (reflection about cr)", "1": "reference fast-math arithmetic",
                     "2": "IEEE, reflection about normalize(cr)", "seed2": "mode 0 on seed 2 (Monte-Carlo spread)"},
           "configs": {}}
    res["bars_defined"] = {"fixed": BARS, "bin_flip_dx": BIN_FLIP_DX,
                           "other_path_vs_reference_form": OTHER_PATH_VS_REFERENCE_FORM}
    if os.path.exists(args.out):  # keep the configs not re-run
        with open(args.out) as f:
            res["configs"] = json.load(f).get("configs", {})
    for name in args.configs.split(","):
        c = CONFIGS[name]
        n = c["rays"][0] * c["rays"][1] * c["rays"][2]
        begin = {"C4": args.c4_begin}.get(name, 0)
        end = {"C3": min(n, args.c3_rays), "C4": min(n, args.c4_begin + args.c4_rays)}.get(name, n)
        ir_len = 2 * c["sr"]
        recs = {}
        t0 = time.time()
        for key, arith, seed in ((0, 0, 1), (1, 1, 1), (2, 2, 1), ("seed2", 0, 2)):
            p = po.make_params(rays=c["rays"], sample_rate=c["sr"], base_power=3.62, max_bounces=c["bounces"],
                               hrtf=HRTF, emitter=CONFERENCE_EMITTER, listener=CONFERENCE_LISTENER, arith=arith,
                               seed=seed)
            recs[key] = records(osc, p, begin, end, args.threads)
        arith = {0: 0, 1: 1, 2: 2, "seed2": 0}
        cmp = lambda a, b: compare(recs[a], recs[b], ta, ir_len, c["sr"], HRTF, arith[a], arith[b])  # noqa: E731
        r = {"rays": [begin, end], "launch_rays": n, "bounces": c["bounces"], "sample_rate": c["sr"],
             "ieee_vs_reference": cmp(0, 1),
             "normalize_reflection_vs_reference": cmp(2, 1),
             "ieee_vs_normalize_reflection": cmp(0, 2),
             "seed1_vs_seed2": cmp(0, "seed2")}
        r["bars"] = bars_met(r["ieee_vs_reference"], r["seed1_vs_seed2"], r["normalize_reflection_vs_reference"])
        r["bars_normalize_reflection"] = bars_met(r["normalize_reflection_vs_reference"], r["seed1_vs_seed2"])
        r["cpu_s"] = round(time.time() - t0, 1)
        res["configs"][name] = r
        print(name, json.dumps(r["bars"]), flush=True)
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    with open(args.out, "w") as f:
        json.dump(res, f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
