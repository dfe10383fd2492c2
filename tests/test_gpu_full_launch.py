"""GPU parity on WHOLE launches at the BASELINE configs (BASELINE.json configs[1..4]).

Every test traces the contract's own launch on the GPU and the same launch with the CPU oracle
(oracle/arx_oracle.c, every ray of it, on this host's cores) and asserts the bar of SURVEY.md §8c
for integer work: equal closest-hit query, receiver-hit and miss counts, and both f32 IRs equal bit
for bit (the IR is a deterministic function of the exact int64 histogram).  Reference: the raygen
loop over the whole launch, devicePrograms.cu:192-254.

  C2  conference stand-in, 100 K rays x 8 bounces, 16 kHz, whole launch; its audio
      (experimento_entrada_16KHz.wav, tests/golden/audio_experimento_16k_ch0.npz) convolved with the
      rendered IR within 1 ULP(max) of the f64 oracle (kernels.cu:382-438, AudioRenderer.cpp:706-711)
  C3  1 M rays x 16 bounces, 48 kHz, whole launch
  C4  10 M rays x 32 bounces, 48 kHz: the contiguous 1 M-ray slice [5 M, 6 M) of the launch, at the
      10 M launch's own energy and fixed-point scale (a rank's shard on 10 GPUs)
  C5  the moving-listener walk (0.05 m / frame along +x, yaw +1 deg / frame; bench.py
      moving_listener), 600 frames of 1 M x 16 through the device receiver refit; frames 0, 300 and
      599 against the oracle at those poses (the walk leaves the stand-in room at frame 100)

With ARX_PARITY_RECORD=<dir> each test also writes a JSON record of what it compared (profiles/r06/
keeps the GPU box's records; bench.py reads the C3 one, guarded by tree hash and kernel identity).
"""
import json
import os
import time

import numpy as np
import pytest

import pyoracle as po
from audiorenderingv2_amd import AudioRenderer, RenderSettings, receiver_local
from audiorenderingv2_amd._lib import lib
from audiorenderingv2_amd.scene import CONFERENCE_EMITTER, CONFERENCE_LISTENER
from conftest import oracle_threads, world_scene

pytestmark = pytest.mark.gpu

C2 = RenderSettings(rays=(100, 100, 10), sample_rate=16000, base_power=3.62, max_bounces=8, hrtf_absorption_rate=1.0)
C3 = RenderSettings(rays=(100, 100, 100), sample_rate=48000, base_power=3.62, max_bounces=16, hrtf_absorption_rate=1.0)
C4 = RenderSettings(rays=(1000, 100, 100), sample_rate=48000, base_power=3.62, max_bounces=32, hrtf_absorption_rate=1.0)
C5_FRAMES = (0, 300, 599)


def renderer(scene, s, listener=CONFERENCE_LISTENER, yaw=0.0):
    r = AudioRenderer(s, scene=scene, receiver=receiver_local())
    r.setEmitterPosInOptix(CONFERENCE_EMITTER)
    r.setSphereCenterInOptix(listener, yaw)
    return r


def oracle(scene, s, listener=CONFERENCE_LISTENER, yaw=0.0, begin=0, end=None):
    tv, ta = world_scene(scene, listener, yaw)
    osc = po.Scene(tv, ta, bvh=True)
    p = po.make_params(rays=s.rays, sample_rate=s.sample_rate, ir_seconds=s.ir_length_in_seconds,
                       base_power=s.base_power, energy_thres=s.energy_thres, max_bounces=s.max_bounces,
                       hrtf=s.hrtf_absorption_rate, mono=s.mono, seed=s.seed, emitter=CONFERENCE_EMITTER,
                       listener=listener)
    t0 = time.perf_counter()
    L, R, st = osc.trace(p, begin, end, threads=oracle_threads())
    st["oracle_s"] = time.perf_counter() - t0
    irl, irr = po.finalize_ir(p, L, R)
    return irl, irr, st


def check_same(name, gpu_ir, gst, ora_ir, ost, extra=None, require_hits=True):
    counts_g = (int(gst["queries"]), int(gst["receiver_hits"]), int(gst["misses"]))
    counts_o = (int(ost["queries"]), int(ost["receiver_hits"]), int(ost["misses"]))
    bits = [bool(np.array_equal(g.view(np.uint32), o.view(np.uint32))) for g, o in zip(gpu_ir, ora_ir)]
    rec = {"test": name, "queries_gpu": counts_g[0], "queries_oracle": counts_o[0], "receiver_hits_gpu": counts_g[1],
           "receiver_hits_oracle": counts_o[1], "misses_gpu": counts_g[2], "misses_oracle": counts_o[2],
           "ir_left_bit_exact": bits[0], "ir_right_bit_exact": bits[1], "ir_nonzero_bins": int(np.count_nonzero(gpu_ir[0])),
           "tree_hash": f"{int(gst['tree_hash']):016x}", "trace_kernel_id": f"{int(lib().arx_trace_kernel_id()):016x}",
           "oracle_threads": oracle_threads(), "oracle_s": round(float(ost["oracle_s"]), 2), **(extra or {})}
    out = os.environ.get("ARX_PARITY_RECORD")
    if out:
        os.makedirs(out, exist_ok=True)
        with open(os.path.join(out, f"{name}.json"), "w") as fh:
            json.dump(rec, fh, indent=1)
    assert counts_g == counts_o, rec
    assert all(bits), rec
    if require_hits:
        assert gst["receiver_hits"] > 0
    return rec


def test_c2_whole_launch_and_experimento_convolution(conference):
    from audiorenderingv2_amd.scene import reference_audio

    r = renderer(conference, C2)
    r.render()
    ir, st = r.get_ir(), r.stats()
    irl, irr, ost = oracle(conference, C2)
    check_same("c2_whole_launch", ir, st, (irl, irr), ost, {"rays": 100000, "max_bounces": 8, "sample_rate": 16000})
    x, sr = reference_audio("experimento")
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "audio_experimento_16k_ch0.npz"))
    assert sr == 16000 and x.size == 128000 and int(g["sample_rate"]) == 16000
    assert np.array_equal(x, g["pcm16"].astype(np.float32) / np.float32(32768.0))  # AudioFile's 16-bit decode
    L, R, _, _ = r.convoluteAudioFile(x)
    for got, h in ((L, ir[0]), (R, ir[1])):
        ref = po.convolute_audio(x, sr, h)
        assert ref.any()
        assert np.abs(got - ref).max() <= np.spacing(np.float32(np.abs(ref).max()))


def test_c3_whole_launch(conference):
    r = renderer(conference, C3)
    r.render()
    ir, st = r.get_ir(), r.stats()
    irl, irr, ost = oracle(conference, C3)
    assert 10 * 10**6 < ost["queries"] <= 16 * 10**6
    check_same("c3_whole_launch", ir, st, (irl, irr), ost, {"rays": 10**6, "max_bounces": 16, "sample_rate": 48000,
                                                             "workload": "c3"})


def test_c4_one_million_ray_slice(conference):
    b, e = 5 * 10**6, 6 * 10**6
    r = renderer(conference, C4)
    r.clear_histogram()
    r.trace_rays(b, e)
    r.finalize_ir()
    ir, st = r.get_ir(), r.stats()
    irl, irr, ost = oracle(conference, C4, begin=b, end=e)
    check_same("c4_slice_5M_6M", ir, st, (irl, irr), ost, {"rays": [b, e], "launch_rays": 10**7, "max_bounces": 32,
                                                            "sample_rate": 48000})


@pytest.fixture(scope="module")
def c5_walk(conference):
    """The C5 walk on one renderer: every frame re-places the listener through the device refit
    (no scene rebuild) and renders; the IRs and counters of the checked frames are kept."""
    x0, y0, z0 = CONFERENCE_LISTENER
    r = renderer(conference, C3)
    kept = {}
    for k in range(max(C5_FRAMES) + 1):
        r.setSphereCenterInOptix((x0 + 0.05 * k, y0, z0), float(k % 360))
        r.render()
        if k in C5_FRAMES:
            kept[k] = (r.get_ir(), r.stats())
    r.close()
    return kept


@pytest.mark.parametrize("frame", C5_FRAMES)
def test_c5_walk_frames(conference, c5_walk, frame):
    x0, y0, z0 = CONFERENCE_LISTENER
    pose = (x0 + 0.05 * frame, y0, z0)
    ir, st = c5_walk[frame]
    irl, irr, ost = oracle(conference, C3, listener=pose, yaw=float(frame % 360))
    # the walk leaves the 20 m room at frame 100 (x = 10 m): later frames see the room's outside wall
    # and almost no receiver hits, which the oracle must reproduce just the same
    check_same(f"c5_walk_frame{frame}", ir, st, (irl, irr), ost, {"pose": list(pose), "yaw": frame % 360},
               require_hits=frame == 0)
