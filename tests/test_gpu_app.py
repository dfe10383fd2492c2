"""End-to-end app flow on the GPU: config.json + OBJ/MTL + WAV files -> native loaders ->
HIP render + convolution -> normalised WAV export (main.cpp export mode), and the IR / output
text dumps.  Inputs are written to a temp tree shaped like the reference's working directory
(build dir two levels below assets/models); expected results come from the CPU oracle fed with
the same loaded geometry.
"""
import json
import os

import numpy as np
import pytest

import pyoracle as po
from audiorenderingv2_amd import place_receiver_vertices
from audiorenderingv2_amd.app import Context, export_audio, experimentation, main
from audiorenderingv2_amd.formats import (load_receiver_half, load_scene, load_wav, normalize_to_range_minus_one_to_one,
                                          read_float_lines, save_wav)
from audiorenderingv2_amd.scene import load_meshes_npz
from conftest import GOLDEN

pytestmark = pytest.mark.gpu


def write_obj(path, meshes, mtl_name):
    lines = [f"mtllib {mtl_name}"]
    base = 1
    for k, m in enumerate(meshes):
        lines.append(f"o part{k}")
        lines += [f"v {x:.9g} {y:.9g} {z:.9g}" for x, y, z in m.vertices]
        lines.append(f"usemtl {m.name}")
        lines += [f"f {a + base} {b + base} {c + base}" for a, b, c in m.faces]
        base += len(m.vertices)
    path.write_text("\n".join(lines) + "\n")
    (path.parent / mtl_name).write_text("".join(f"newmtl {n}\nKd 1 1 1\n" for n in sorted({m.name for m in meshes})))


@pytest.fixture()
def app_tree(tmp_path):
    models = tmp_path / "assets" / "models"
    models.mkdir(parents=True)
    build = tmp_path / "prebuild" / "build"
    build.mkdir(parents=True)
    rec = load_meshes_npz(os.path.join(GOLDEN, "receiver_local.npz"))
    write_obj(models / "leftHalf.obj", [rec[0]], "leftHalf.mtl")
    write_obj(models / "rightHalf.obj", [rec[1]], "rightHalf.mtl")
    write_obj(models / "room.obj", load_meshes_npz(os.path.join(GOLDEN, "test_obj.npz")), "room.mtl")
    rng = np.random.default_rng(0)
    sr = 16000
    x = (0.5 * np.sin(np.arange(int(3.4 * sr)) * 0.03) + 0.1 * rng.standard_normal(int(3.4 * sr))).astype(np.float32)
    save_wav(str(models / "in.wav"), np.clip(x, -1, 1)[None, :], sr, 16)
    cfg = {
        "renderer_parameters": {"ir_length_in_seconds": 2, "write_first_ir_to_file": True},
        "scene_parameters": {"scene_file_path": "../../assets/models/room.obj",
                             "audio_file_path": "../../assets/models/in.wav",
                             "initial_receiver_pos": {"x": 2.5, "y": 9.9, "z": 0},
                             "initial_emitter_pos": {"x": 0.5, "y": 3.0, "z": 1.0}},
        "pathtracer_parameters": {"base_power": 3.62, "rays": {"x": 64, "y": 64, "z": 8}, "ray_max_bounces": 8,
                                  "hrtf_absorption_rate": 0.4,
                                  "materials": [{"name": "Amarillo", "mat_absorption": 0.2}]},
    }
    (build / "config.json").write_text(json.dumps(cfg))
    return build, models


def oracle_export(ctx, models):
    c = ctx.config
    scene = load_scene(str(models / "room.obj"), c.materials)
    halves = []
    for side, name in enumerate(("leftHalf.obj", "rightHalf.obj")):
        m = load_receiver_half(str(models / name), side)
        halves.append(place_receiver_vertices(m.vertices, c.initial_receiver_pos, 0.0)[m.faces].reshape(-1, 9))
    tv = np.concatenate([scene.tri_v, *halves]).astype(np.float32)
    ta = np.concatenate([scene.tri_abs, np.full(len(halves[0]), -1.0, np.float32),
                         np.full(len(halves[1]), -2.0, np.float32)])
    s = ctx.renderer.settings
    p = po.make_params(rays=s.rays, sample_rate=s.sample_rate, ir_seconds=s.ir_length_in_seconds,
                       base_power=s.base_power, energy_thres=s.energy_thres, max_bounces=s.max_bounces,
                       hrtf=s.hrtf_absorption_rate, mono=s.mono, seed=s.seed, emitter=c.initial_emitter_pos,
                       listener=c.initial_receiver_pos)
    L, R, _ = po.Scene(tv, ta, bvh=True).trace(p, threads=8)
    irl, irr = po.finalize_ir(p, L, R)
    x = ctx.audio.samples[0]
    return irl, irr, po.convolute_audio(x, s.sample_rate, irl), po.convolute_audio(x, s.sample_rate, irr)


def pcm16(v):
    return np.trunc(np.clip(v, -1, 1).astype(np.float64) * 32767).astype(np.int64)


def test_export_mode_matches_oracle(app_tree, monkeypatch):
    build, models = app_tree
    monkeypatch.chdir(build)
    ctx = Context.load("config.json")
    assert ctx.config.hrtf_absorption_rate == 0.0 and ctx.sample_rate == 16000
    L, R = export_audio(ctx, "Result.wav")
    assert not os.path.exists("output_ir_left.txt")  # export_audio clears the dump flags (main.cpp:680)
    irl, irr, yl, yr = oracle_export(ctx, models)
    gl, gr = ctx.renderer.get_ir()
    assert np.array_equal(gl.view(np.uint32), irl.view(np.uint32)) and gl.any()
    assert np.array_equal(gr.view(np.uint32), irr.view(np.uint32))
    w = load_wav("Result.wav")
    assert (w.channels, w.sample_rate, w.bit_depth, w.frames) == (2, 16000, 16, ctx.audio.frames)
    for got, ref in ((w.samples[0], yl), (w.samples[1], yr)):
        want = pcm16(normalize_to_range_minus_one_to_one(ref))
        have = np.round(got.astype(np.float64) * 32768).astype(np.int64)
        assert np.abs(have - want).max() <= 1


def test_cli_export_and_ir_dump(app_tree, monkeypatch):
    build, models = app_tree
    monkeypatch.chdir(build)
    assert main(["config.json", "export", "out.wav"]) == 0
    assert load_wav("out.wav").channels == 2
    assert main(["missing.json", "export"]) == 1
    # write_first_ir_to_file from the config dumps the first render only (AudioRenderer.cpp:525-567)
    ctx = Context.load("config.json")
    ctx.prepare()
    ctx.renderer.render()
    gl, gr = ctx.renderer.get_ir()
    np.testing.assert_allclose(read_float_lines("output_ir_left.txt"), gl, rtol=1e-5, atol=1e-30)
    np.testing.assert_allclose(read_float_lines("output_ir_right.txt"), gr, rtol=1e-5, atol=1e-30)
    assert not ctx.renderer.write_ir_to_file_flag
    ctx.renderer.set_write_output_to_file_flag(True)
    L, R, _, _ = ctx.renderer.convoluteAudioFile(ctx.audio.samples[0])
    np.testing.assert_allclose(read_float_lines("output_convolute_left.txt"), L, rtol=1e-5, atol=1e-30)
    stats = experimentation(ctx, rounds=3, log=lambda *_: None)
    assert stats["render"]["median_ms"] > 0
