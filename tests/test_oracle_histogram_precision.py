"""How far is the engine's int64 fixed-point IR histogram from the reference's f32 accumulation?

The reference adds every receiver hit's f32 energy into an f32 IR with atomicAdd
(devicePrograms.cu:135-165), in an order that changes from run to run.  The engine quantizes each
contribution to an integer number of units e0 * 2^-frac_bits (frac_bits = clamp(59 - ceil(log2 N),
8, 52)), sums exactly in int64 and converts the sum to f32 once (arx_frac_bits, finalize_ir).
orc_trace_float_sums traces the same rays once and accumulates every contribution three ways: the
int64 histogram, an f64 sum (the reference value), and an f32 sum in ray order (the reference's
arithmetic in one of its orders).  Bar: relative RMS < 1e-4 per ear for the int64
IR and for the reference's f32 accumulation, both against the f64 sum -- at C2 in full and on a ray
sample of C4, whose 10 M rays x 32 bounces give the coarsest units (frac_bits 35) and the most
late, weak contributions.  The numbers (profiles/r03/histogram_precision.json) are recorded in
DESIGN.md §3.
"""
import numpy as np
import pytest

import pyoracle as po
from audiorenderingv2_amd.scene import CONFERENCE_EMITTER, CONFERENCE_LISTENER, conference_standin
from conftest import world_scene

TOL = 1e-4


@pytest.fixture(scope="module")
def conference_oracle():
    tv, ta = world_scene(conference_standin(), CONFERENCE_LISTENER, 0.0)
    return po.Scene(tv, ta, bvh=True)


def rel_rms(a, ref):
    return float(np.linalg.norm(a - ref) / np.linalg.norm(ref))


CASES = [
    # name, rays (the launch: sets e0 and frac_bits), sample_rate, bounces, traced ray range
    ("C2", (100, 100, 10), 16000, 8, (0, 100_000)),
    ("C4 sample", (1000, 100, 100), 48000, 32, (0, 20_000)),
]


@pytest.mark.parametrize("name,rays,sr,bounces,span", CASES)
def test_int64_histogram_vs_float_accumulation(conference_oracle, name, rays, sr, bounces, span):
    p = po.make_params(rays=rays, sample_rate=sr, base_power=3.62, max_bounces=bounces, hrtf=0.5,
                       emitter=CONFERENCE_EMITTER, listener=CONFERENCE_LISTENER)
    (L, R), (dL, dR), (fL, fR), st = conference_oracle.float_sums(p, *span)
    assert st["receiver_hits"] > 200
    # the int64 path is the engine's: the same sums as orc_trace (and so the GPU, bit for bit)
    L2, R2, st2 = conference_oracle.trace(p, *span, threads=8)
    assert np.array_equal(L, L2) and np.array_equal(R, R2) and st == st2
    il, ir = po.finalize_ir(p, L, R)
    out = {"case": name, "rays": list(rays), "traced": list(span), "frac_bits": po.frac_bits(int(np.prod(rays))),
           "receiver_hits": st["receiver_hits"]}
    for ear, i64, d, f in (("left", il, dL, fL), ("right", ir, dR, fR)):
        e_int = rel_rms(i64.astype(np.float64), d)
        e_f32 = rel_rms(f.astype(np.float64), d)
        out[ear] = {"int64_vs_f64": e_int, "f32_sequential_vs_f64": e_f32,
                    "int64_vs_f32_sequential": rel_rms(i64.astype(np.float64), f.astype(np.float64))}
        assert e_int < TOL, (name, ear, e_int)
        assert e_f32 < TOL, (name, ear, e_f32)
