"""GPU parity: the HIP path (through the C ABI) against the CPU oracle.

Bar (DESIGN.md "Parity"):
  * ray directions, per-ray paths and the i64 IR histogram: BIT-EXACT (integer work);
    the f32 IR is a deterministic function of the histogram, so it is bit-exact too;
  * convolution: max |gpu - oracle_f32| <= 1 ULP(max |oracle|) (the north star's
    "within 1 ULP", as a norm-wise bound);
  * full BASELINE sizes: size-independent properties (determinism, shard-sum
    exactness, inverse-square energy, linearity of the convolution).
"""
import math

import numpy as np
import pytest

import pyoracle as po
from audiorenderingv2_amd import AudioRenderer, RenderSettings, debug_ray_directions, receiver_local
from audiorenderingv2_amd.scene import CONFERENCE_EMITTER, CONFERENCE_LISTENER, Scene
from conftest import world_scene

pytestmark = pytest.mark.gpu


def make(scene, listener, yaw=0.0, emitter=(0.0, 0.0, 0.0), **kw):
    s = RenderSettings(**kw)
    r = AudioRenderer(s, scene=scene, receiver=receiver_local())
    r.setEmitterPosInOptix(emitter)
    r.setSphereCenterInOptix(listener, yaw)
    return r


def oracle_run(scene, listener, yaw, emitter, s: RenderSettings, threads=8, bvh=True):
    tv, ta = world_scene(scene, listener, yaw)
    osc = po.Scene(tv, ta, bvh=bvh)
    p = po.make_params(rays=s.rays, sample_rate=s.sample_rate, ir_seconds=s.ir_length_in_seconds,
                       base_power=s.base_power, energy_thres=s.energy_thres, max_bounces=s.max_bounces,
                       hrtf=s.hrtf_absorption_rate, mono=s.mono, seed=s.seed, emitter=emitter, listener=listener)
    L, R, st = osc.trace(p, threads=threads)
    irl, irr = po.finalize_ir(p, L, R)
    return irl, irr, st


def assert_same_render(r, scene, listener, yaw, emitter, s):
    r.render()
    gl, gr = r.get_ir()
    st = r.stats()
    ol, orr, ost = oracle_run(scene, listener, yaw, emitter, s)
    assert (st["queries"], st["receiver_hits"], st["misses"]) == (ost["queries"], ost["receiver_hits"], ost["misses"])
    assert np.array_equal(gl.view(np.uint32), ol.view(np.uint32))
    assert np.array_equal(gr.view(np.uint32), orr.view(np.uint32))
    return gl, gr, st


def test_ray_directions_bitwise():
    for first in (0, (1 << 32) - 50000):
        g = debug_ray_directions(5, first, 100000)
        o = po.ray_directions(5, first, 100000)
        assert np.array_equal(g.view(np.uint32), o.view(np.uint32)), first


def test_c1_reference_config(c1_scene):
    """BASELINE configs[0] with R/config.json's placement verbatim: test.obj, 1024 rays x 2
    bounces, 16 kHz.  Structural only: the config's emitter (0, 0, 0) sits inside test.obj's
    floor slab (y in [0, 0.1427]), so every ray hits the slab from inside and the IR is empty --
    as it is for the reference on this config.  The lifted variant below checks a non-empty IR."""
    s = RenderSettings(rays=(32, 32, 1), sample_rate=16000, base_power=3.62, max_bounces=2)
    r = make(c1_scene, (2.5, 9.9, 0.0), **s.__dict__)
    gl, gr, st = assert_same_render(r, c1_scene, (2.5, 9.9, 0.0), 0.0, (0.0, 0.0, 0.0), s)
    assert st["receiver_hits"] == 0 and not gl.any() and not gr.any()


def test_c1_lifted_emitter_with_guitar():
    """configs[0] at its own ray count (1024 rays x 2 bounces, 16 kHz) with the emitter lifted
    into the test.obj room: a non-empty IR bit-exact with the oracle, then convolved with
    guitar_sample_16k.wav channel 0 (399 569 samples = 24 one-second blocks + a 15 569-sample
    tail the reference never processes) within 1 ULP(max) of the oracle."""
    from audiorenderingv2_amd.scene import reference_audio, reference_config_materials, test_obj_scene

    scene = test_obj_scene(reference_config_materials())
    s = RenderSettings(rays=(32, 32, 1), sample_rate=16000, base_power=3.62, max_bounces=2, hrtf_absorption_rate=0.5)
    em = (0.5, 3.0, 1.0)
    r = make(scene, (2.5, 9.9, 0.0), emitter=em, **s.__dict__)
    gl, gr, st = assert_same_render(r, scene, (2.5, 9.9, 0.0), 0.0, em, s)
    assert st["receiver_hits"] > 0 and gl.any() and gr.any()
    x, sr = reference_audio("guitar")
    assert sr == 16000 and x.size == 399569
    L, R, _, _ = r.convoluteAudioFile(x)
    for got, ir in ((L, gl), (R, gr)):
        ref = po.convolute_audio(x, sr, ir)
        assert np.abs(got - ref).max() <= np.spacing(np.float32(np.abs(ref).max()))
    # the input tail (len mod sr) is never read (kernels.cu:413): zeroing it changes nothing
    xt = x.copy()
    xt[24 * sr:] = 0.0
    Lt, Rt, _, _ = r.convoluteAudioFile(xt)
    assert np.array_equal(Lt, L) and np.array_equal(Rt, R)


def test_c1_dense_bitwise(c1_scene):
    # R/config.json's emitter (0,0,0) sits inside test.obj's floor slab (y in [0, 0.1427]) so the
    # configs[0] IR is empty (test above); lift the emitter to get receiver hits.
    s = RenderSettings(rays=(64, 64, 8), sample_rate=16000, base_power=3.62, max_bounces=8, hrtf_absorption_rate=0.5)
    em = (0.5, 3.0, 1.0)
    r = make(c1_scene, (2.5, 9.9, 0.0), emitter=em, **s.__dict__)
    gl, gr, st = assert_same_render(r, c1_scene, (2.5, 9.9, 0.0), 0.0, em, s)
    assert st["receiver_hits"] > 0 and gl.any() and gr.any()


def test_conference_bitwise(conference):
    s = RenderSettings(rays=(40, 40, 10), sample_rate=16000, base_power=3.62, max_bounces=8)
    r = make(conference, CONFERENCE_LISTENER, emitter=CONFERENCE_EMITTER, **s.__dict__)
    gl, gr, st = assert_same_render(r, conference, CONFERENCE_LISTENER, 0.0, CONFERENCE_EMITTER, s)
    assert st["receiver_hits"] > 0


def test_conference_48k_rotated_mono_bitwise(conference):
    s = RenderSettings(rays=(30, 40, 10), sample_rate=48000, base_power=3.62, max_bounces=16, mono=True,
                       hrtf_absorption_rate=0.25, seed=99)
    lst, yaw = (3.0, 1.5, -1.0), 75.0
    r = make(conference, lst, yaw=yaw, emitter=CONFERENCE_EMITTER, **s.__dict__)
    gl, gr, _ = assert_same_render(r, conference, lst, yaw, CONFERENCE_EMITTER, s)
    assert np.array_equal(gl, gr)


def test_listener_move_equals_fresh_renderer(conference):
    s = RenderSettings(rays=(20, 20, 10), sample_rate=16000, base_power=3.62, max_bounces=8)
    r = make(conference, (0.0, 1.0, 0.0), emitter=CONFERENCE_EMITTER, **s.__dict__)
    r.render()
    r.setSphereCenterInOptix((4.0, 1.3, -2.0), 200.0)  # no scene rebuild: receiver sub-tree only
    r.render()
    a = r.get_ir()
    f = make(conference, (4.0, 1.3, -2.0), yaw=200.0, emitter=CONFERENCE_EMITTER, **s.__dict__)
    f.render()
    b = f.get_ir()
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])


def test_shards_sum_exactly(conference):
    s = RenderSettings(rays=(100, 100, 10), sample_rate=48000, base_power=3.62, max_bounces=16)
    r = make(conference, CONFERENCE_LISTENER, emitter=CONFERENCE_EMITTER, **s.__dict__)
    r.render()
    full = r.get_ir()
    q_full = r.stats()["queries"]
    r.clear_histogram()
    n = 100 * 100 * 10
    for b, e in ((0, 12345), (12345, 60000), (60000, n)):
        r.trace_rays(b, e)
    r.finalize_ir()
    parts = r.get_ir()
    assert r.stats()["queries"] == q_full
    assert np.array_equal(full[0], parts[0]) and np.array_equal(full[1], parts[1])


def test_full_size_c3_properties(conference):
    """configs[2] size: 1M rays x 16 bounces, 48 kHz -- determinism + shard exactness."""
    s = RenderSettings(rays=(100, 100, 100), sample_rate=48000, base_power=3.62, max_bounces=16)
    r = make(conference, CONFERENCE_LISTENER, emitter=CONFERENCE_EMITTER, **s.__dict__)
    r.render()
    a = r.get_ir()
    st = r.stats()
    r.render()
    b = r.get_ir()
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])
    assert st["queries"] <= 16 * 10**6 and st["queries"] > 10 * 10**6
    assert st["receiver_hits"] > 1000
    # an independent 4-way shard (as 4 GPUs would run it) gives the identical histogram
    r.clear_histogram()
    for k in range(4):
        r.trace_rays(k * 250000, (k + 1) * 250000)
    r.finalize_ir()
    c = r.get_ir()
    assert np.array_equal(a[0], c[0]) and np.array_equal(a[1], c[1])
    # and it matches the oracle on a ray sample of the same launch (ray ids 0..3999)
    r.clear_histogram()
    r.trace_rays(0, 4000)
    tv, ta = world_scene(conference, CONFERENCE_LISTENER, 0.0)
    osc = po.Scene(tv, ta, bvh=True)
    p = po.make_params(rays=s.rays, sample_rate=48000, base_power=3.62, max_bounces=16,
                       emitter=CONFERENCE_EMITTER, listener=CONFERENCE_LISTENER)
    L, R, ost = osc.trace(p, 0, 4000, threads=8)
    h_ptr, n = r.histogram_device_ptr()
    assert r.stats()["queries"] == ost["queries"]
    r.finalize_ir()
    ol, orr = po.finalize_ir(p, L, R)
    gl, gr = r.get_ir()
    assert np.array_equal(gl, ol) and np.array_equal(gr, orr)


# trace paths (arx_debug_set_trace_path): 0 = the default (16-bit quantized BVH2, LDS stack), 8 =
# the 4-wide compressed tree (CW4), 1 = f32 coded BVH2 nodes (taken while the emitter is off the
# quantization grid), 2 = the global-memory stack (taken by trees deeper than the LDS stack), 3 =
# both fallbacks
PATHS = ["0", "8", "1", "2", "3"]


@pytest.mark.parametrize("path", PATHS)
def test_trace_paths_match_oracle(c1_scene, conference, path):
    """Every trace path against the oracle: C1 dense, the conference stand-in, a listener move
    (receiver sub-tree only) and an empty scene."""
    s = RenderSettings(rays=(64, 64, 8), sample_rate=16000, base_power=3.62, max_bounces=8, hrtf_absorption_rate=0.5)
    em = (0.5, 3.0, 1.0)
    r = make(c1_scene, (2.5, 9.9, 0.0), emitter=em, **s.__dict__)
    r.set_trace_path(int(path))
    assert_same_render(r, c1_scene, (2.5, 9.9, 0.0), 0.0, em, s)
    s = RenderSettings(rays=(40, 40, 10), sample_rate=16000, base_power=3.62, max_bounces=8)
    r = make(conference, CONFERENCE_LISTENER, emitter=CONFERENCE_EMITTER, **s.__dict__)
    r.set_trace_path(int(path))
    assert_same_render(r, conference, CONFERENCE_LISTENER, 0.0, CONFERENCE_EMITTER, s)
    lst = (2.0, 1.4, -1.5)
    r.setSphereCenterInOptix(lst, 33.0)
    assert_same_render(r, conference, lst, 33.0, CONFERENCE_EMITTER, s)
    empty = Scene(np.zeros((0, 9), np.float32), np.zeros(0, np.float32), [])
    r = make(empty, (0.0, 0.0, 3.0), **s.__dict__)
    r.set_trace_path(int(path))
    gl, _, st = assert_same_render(r, empty, (0.0, 0.0, 3.0), 0.0, (0.0, 0.0, 0.0), s)
    assert st["receiver_hits"] > 0


@pytest.mark.parametrize("path", ["8", "1", "2", "3"])
def test_trace_paths_identical_at_c3_shape(conference, path):
    """The fallback paths produce the default path's histogram bit for bit on a 100 K-ray,
    16-bounce, 48 kHz launch."""
    s = RenderSettings(rays=(100, 100, 10), sample_rate=48000, base_power=3.62, max_bounces=16, hrtf_absorption_rate=0.5)
    r = make(conference, CONFERENCE_LISTENER, emitter=CONFERENCE_EMITTER, **s.__dict__)
    r.render()
    ref, q = r.get_ir(), r.stats()["queries"]
    r.set_trace_path(int(path))
    r.render()
    got = r.get_ir()
    assert r.stats()["queries"] == q
    assert np.array_equal(ref[0], got[0]) and np.array_equal(ref[1], got[1])


@pytest.mark.parametrize("path", ["0", "8", "2"])
def test_quantized_nodes_regrid_and_fallback(c1_scene, path):
    """16-bit quantized nodes (QNode2): the grid covers scene + receiver + emitter at scene load.
    A listener moved off the grid (outside the room) re-grids once (a wider grid, full
    re-quantization); an emitter off the grid makes the launches take the f32 coded nodes.
    Every case stays bit-exact with the oracle."""
    s = RenderSettings(rays=(64, 64, 4), sample_rate=16000, base_power=3.62, max_bounces=8, hrtf_absorption_rate=0.5)
    em = (0.5, 3.0, 1.0)
    r = make(c1_scene, (2.5, 9.9, 0.0), emitter=em, **s.__dict__)
    r.set_trace_path(int(path))
    assert_same_render(r, c1_scene, (2.5, 9.9, 0.0), 0.0, em, s)
    far = (40.0, 9.0, -25.0)  # well outside the test.obj room and its grid margin
    r.setSphereCenterInOptix(far, 10.0)
    assert_same_render(r, c1_scene, far, 10.0, em, s)
    r.setSphereCenterInOptix((2.5, 9.9, 0.0), 0.0)
    assert_same_render(r, c1_scene, (2.5, 9.9, 0.0), 0.0, em, s)
    em_far = (300.0, 5.0, 0.0)
    r.setEmitterPosInOptix(em_far)
    assert_same_render(r, c1_scene, (2.5, 9.9, 0.0), 0.0, em_far, s)


@pytest.mark.parametrize("path", ["0", "8", "1"])
@pytest.mark.parametrize("offset", [(1.0e4, -3.0e3, 5.0e3), (-2.5e5, 0.0, 1.0e5)])
def test_room_far_from_origin(c1_scene, offset, path):
    """The test.obj room, emitter and listener translated far from the origin: f32 slab and
    triangle arithmetic at large magnitudes (coarse ulps) and a quantization grid whose origin
    is far away.  Quantized (0) and f32 (1) nodes stay bit-exact with the oracle."""
    off = np.asarray(offset, np.float32)
    tv = (c1_scene.tri_v.reshape(-1, 3, 3) + off).reshape(-1, 9).astype(np.float32)
    far = Scene(tv, c1_scene.tri_abs, c1_scene.names)
    em = tuple(float(v) for v in np.float32([0.5, 3.0, 1.0]) + off)
    lst = tuple(float(v) for v in np.float32([2.5, 9.9, 0.0]) + off)
    s = RenderSettings(rays=(64, 64, 4), sample_rate=16000, base_power=3.62, max_bounces=8, hrtf_absorption_rate=0.5)
    r = make(far, lst, emitter=em, **s.__dict__)
    r.set_trace_path(int(path))
    _, _, st = assert_same_render(r, far, lst, 0.0, em, s)
    assert st["queries"] > 16384


@pytest.mark.parametrize("path", PATHS)
def test_random_soup_with_degenerate_triangles(path):
    """A closed room filled with a random triangle soup: zero-area triangles, a coplanar
    stack at y = 1, exact duplicates (equal-t ties -> lowest id), and triangles through the
    emitter's position.  Bit-exact with the oracle on every trace path."""
    from audiorenderingv2_amd.scene import _box_tris

    rng = np.random.default_rng(17)
    room = _box_tris(np.array([[-4, -4, -4]], np.float32), np.array([[4, 4, 4]], np.float32))
    soup = rng.uniform(-3.5, 3.5, (3000, 9)).astype(np.float32)
    soup[:60, 3:6] = soup[:60, 0:3]            # degenerate (two equal vertices)
    soup[60:120, 1::3] = 1.0                   # coplanar at y = 1
    soup[120:180] = soup[180:240]              # exact duplicates
    soup[240:260, 0:3] = 0.0                   # a vertex at the emitter
    tv = np.concatenate([room, soup]).astype(np.float32)
    ta = rng.uniform(0.0, 0.9, tv.shape[0]).astype(np.float32)
    sc = Scene(tv, ta, [])
    s = RenderSettings(rays=(64, 64, 4), sample_rate=16000, base_power=3.62, max_bounces=8, hrtf_absorption_rate=0.5)
    r = make(sc, (1.5, 1.2, -0.7), emitter=(0.0, 0.0, 0.0), **s.__dict__)
    r.set_trace_path(int(path))
    assert_same_render(r, sc, (1.5, 1.2, -0.7), 0.0, (0.0, 0.0, 0.0), s)


@pytest.mark.parametrize("path", PATHS)
def test_leaves_of_more_than_two_triangles(path):
    """Leaves of up to 8 triangles (builder leaf_max 8; production trees have them only below the
    depth cap): the leaf step tests two triangles and continues with the same leaf two triangles on
    (trace_kernel leaf_step), on every trace path.  Bit-exact with the oracle, whose tree differs."""
    from audiorenderingv2_amd._lib import check, lib
    from audiorenderingv2_amd.scene import _box_tris

    rng = np.random.default_rng(23)
    room = _box_tris(np.array([[-4, -4, -4]], np.float32), np.array([[4, 4, 4]], np.float32))
    soup = rng.uniform(-3.5, 3.5, (2000, 9)).astype(np.float32)  # large, overlapping: leaves stay fat
    tv = np.concatenate([room, soup]).astype(np.float32)
    ta = rng.uniform(0.0, 0.9, tv.shape[0]).astype(np.float32)
    sc = Scene(tv, ta, [])
    s = RenderSettings(rays=(64, 64, 4), sample_rate=16000, base_power=3.62, max_bounces=8, hrtf_absorption_rate=0.5)
    check(lib().arx_debug_set_leaf_max(8))
    try:
        r = make(sc, (1.5, 1.2, -0.7), emitter=(0.0, 0.0, 0.0), **s.__dict__)
        r.set_trace_path(int(path))
        assert_same_render(r, sc, (1.5, 1.2, -0.7), 0.0, (0.0, 0.0, 0.0), s)
        cn = r.node_images()["cnodes"].view(np.int32).reshape(-1, 16)
        codes = cn[:, 12:14].ravel()  # BvhNode d[0..1]: child codes
        counts = (~codes[codes < -1]) & 15
        assert counts.max() > 2, counts.max()
    finally:
        check(lib().arx_debug_set_leaf_max(2))


@pytest.mark.parametrize("max_bounces,thres,secs", [(0, 0.0, 2), (1, 0.0, 1), (3, 0.05, 1), (64, 1e-7, 3)])
def test_bounce_and_threshold_limits(c1_scene, max_bounces, thres, secs):
    """Reflection-count and energy-threshold cut-offs (devicePrograms.cu:147-175, 234-236)
    and IR lengths of 1-3 s: 0 bounces (direct sound only), early energy cut, long paths."""
    em = (0.5, 3.0, 1.0)
    s = RenderSettings(rays=(48, 48, 4), sample_rate=16000, ir_length_in_seconds=secs, base_power=3.62,
                       max_bounces=max_bounces, energy_thres=thres, hrtf_absorption_rate=0.5)
    r = make(c1_scene, (2.5, 9.9, 0.0), emitter=em, **s.__dict__)
    assert_same_render(r, c1_scene, (2.5, 9.9, 0.0), 0.0, em, s)


def test_inverse_square_on_gpu():
    # listener on the +z (ear) axis: rays arrive through the half-spheres' domes, not through
    # the 0.058 m slot between the two halves (|z| < 0.029 in the local frame), which a
    # listener on the x axis would look through (~5 % of the chord-weighted energy).
    d = 4.0
    empty = Scene(np.zeros((0, 9), np.float32), np.zeros(0, np.float32), [])
    s = RenderSettings(rays=(1000, 1000, 1), sample_rate=16000, base_power=3.62, max_bounces=4)
    r = make(empty, (0.0, 0.0, d), **s.__dict__)
    r.render()
    gl, gr = r.get_ir()
    total = gl.astype(np.float64).sum() + gr.astype(np.float64).sum()
    integral = 2 * math.pi * (1 - (d * d - 1) / (2 * d) * math.log((d + 1) / (d - 1)))
    expect = float(np.float32(3.62)) / (4 * math.pi * 4.18879020478) * integral
    assert abs(total / expect - 1) < 0.02


# ------------------------------------------------------------------ convolution ---
def ulp_of_max(y):
    return np.spacing(np.float32(np.abs(y).max()))


def conv_renderer(sr, secs=2):
    return AudioRenderer(RenderSettings(rays=(1, 1, 1), sample_rate=sr, ir_length_in_seconds=secs))


def sparse_ir(n, rng, k=300, scale=1e-4):
    ir = np.zeros(n, np.float32)
    ir[rng.integers(0, n, k)] = rng.exponential(scale, k).astype(np.float32)
    return ir


@pytest.mark.parametrize("sr,secs,length", [(1000, 2, 10555), (1000, 2, 999), (1000, 2, 4000), (800, 3, 7777),
                                            (16000, 2, 128000), (441, 2, 5000), (32000, 2, 70000),
                                            (22050, 1, 50000), (44100, 2, 100000), (1125, 2, 9000),
                                            (1100, 2, 6000), (48000, 1, 100000), (96000, 2, 250000),
                                            (77175, 2, 200000)])
def test_convolution_matches_oracle(sr, secs, length):
    rng = np.random.default_rng(sr + length)
    n = sr * secs
    irl, irr = sparse_ir(n, rng), sparse_ir(n, rng)
    x = (0.3 * rng.standard_normal(length)).astype(np.float32)
    r = conv_renderer(sr, secs)
    r.set_ir(irl, irr)
    L, R, _, _ = r.convoluteAudioFile(x)
    for got, ir in ((L, irl), (R, irr)):
        ref = po.convolute_audio(x, sr, ir)
        if not ref.any():
            assert not got.any()
        else:
            assert np.abs(got - ref).max() <= ulp_of_max(ref)


@pytest.mark.parametrize("sr,secs,live,expect", [
    (48000, 2, False, "mixed-radix direct circular: n=96000 sr=48000 (300x320)"),  # C3
    (16000, 2, False, "mixed-radix direct circular: n=32000 sr=16000 (160x200)"),  # C1 / C2
    (44100, 2, True, "mixed-radix direct circular: n=88200 sr=4096 (315x280)"),    # the mic path
    (1125, 2, False, "mixed-radix direct circular: n=2250 sr=1125"),               # ragged column tiles
    (1100, 2, False, "pow2 linear+fold: n=2200 sr=1100 M=4096"),                    # 11 | n
])
def test_convolution_plan_choice(sr, secs, live, expect):
    """FFT length = ir_len (the reference's own cuFFT length) whenever ir_len = N1 x N2 with 7-smooth
    factors <= 512; the power-of-two linear convolution + fold otherwise.  Both are checked
    against the oracle above."""
    assert conv_renderer(sr, secs).conv_plan(live=live).startswith(expect)


def test_convolution_c3_size_with_rendered_ir(conference):
    """configs[2] audio: A_Clapper_Board.wav channel 0 (807 498 frames @ 48 kHz), IR from a render."""
    from audiorenderingv2_amd.scene import reference_audio

    s = RenderSettings(rays=(100, 100, 20), sample_rate=48000, base_power=3.62, max_bounces=16)
    r = make(conference, CONFERENCE_LISTENER, emitter=CONFERENCE_EMITTER, **s.__dict__)
    r.render()
    irl, irr = r.get_ir()
    x, sr = reference_audio("clapper")
    assert sr == 48000 and x.size == 807498
    L, R, _, _ = r.convoluteAudioFile(x)
    for got, ir in ((L, irl), (R, irr)):
        ref = po.convolute_audio(x, 48000, ir)
        assert np.abs(got - ref).max() <= ulp_of_max(ref)
    # linearity (size-independent property): conv(2x) == 2 conv(x) up to rounding
    L2, _, _, _ = r.convoluteAudioFile(2 * x)
    assert np.abs(L2 - 2 * L).max() <= 2 * ulp_of_max(2 * L)


def test_convolution_device_api_equals_host_api():
    # device buffers of the package itself (arx_device_alloc), not another framework's: a second HIP
    # runtime in the process (torch's) also loads libamd_smi, whose globals interpose librocm_smi64's
    # (RCCL's) and are then destroyed twice at interpreter exit (double free, the whole suite aborts)
    from audiorenderingv2_amd import DeviceBuffer

    sr = 16000
    rng = np.random.default_rng(3)
    r = conv_renderer(sr)
    irl, irr = sparse_ir(2 * sr, rng), sparse_ir(2 * sr, rng)
    r.set_ir(irl, irr)
    x = rng.standard_normal(5 * sr + 17).astype(np.float32)
    L, R, _, _ = r.convoluteAudioFile(x)
    dx = DeviceBuffer.from_numpy(0, x)
    dl, dr = DeviceBuffer(0, x.nbytes), DeviceBuffer(0, x.nbytes)
    r.convolute_device(dx.ptr, x.size, dl.ptr, dr.ptr)
    import audiorenderingv2_amd._lib as L_
    L_.check(L_.lib().arx_copy_ir(r.handle, None, None, r.ir_length))  # syncs the renderer stream
    assert np.array_equal(dl.to_numpy(np.float32, x.size), L) and np.array_equal(dr.to_numpy(np.float32, x.size), R)
    for b in (dx, dl, dr):
        b.close()
    # one timing pair per convolution, host and device entry points alike (arx_conv_times)
    t = r.conv_times(8)
    assert len(t) == 2 and np.all(t > 0)


def test_rejects_absorption_and_hrtf_outside_unit_interval():
    """The int64 fixed-point histogram's headroom needs energies that never grow: absorption in
    [0, 1] (or the receiver marks -1 / -2) and hrtf_absorption_rate in [0, 1]."""
    from audiorenderingv2_amd import ArxError

    tv = np.zeros((2, 9), np.float32)
    tv[:, 3] = 1.0
    tv[:, 7] = 1.0
    r = AudioRenderer(RenderSettings(rays=(4, 4, 4), sample_rate=16000))
    for bad in (1.5, -0.25, float("nan")):
        with pytest.raises(ArxError):
            r.set_scene(Scene(tv, np.array([0.5, bad], np.float32), []))
    r.set_scene(Scene(tv, np.array([0.0, 1.0], np.float32), []))
    with pytest.raises(ArxError):
        r.set_hrtf_absorption_rate(1.25)


def test_set_ir_device_equals_set_ir():
    """arx_set_ir_device: another renderer's IR taken by a device copy convolves like the same IR
    set from the host."""
    sr = 16000
    rng = np.random.default_rng(11)
    a, b = conv_renderer(sr), conv_renderer(sr)
    irl, irr = sparse_ir(2 * sr, rng), sparse_ir(2 * sr, rng)
    a.set_ir(irl, irr)
    dl, dr, n = a.ir_device_ptrs()
    assert n == 2 * sr
    b.set_ir_device(dl, dr)
    x = rng.standard_normal(3 * sr + 5).astype(np.float32)
    La, Ra, _, _ = a.convoluteAudioFile(x)
    Lb, Rb, _, _ = b.convoluteAudioFile(x)
    assert np.array_equal(La, Lb) and np.array_equal(Ra, Rb)
    gl, gr = b.get_ir()
    assert np.array_equal(gl, irl) and np.array_equal(gr, irr)
