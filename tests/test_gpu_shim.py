"""GPU: the C++ AudioRenderer shim (include/arx_audio_renderer.hpp) end to end.

tests/cpp/export_demo.cpp is a main.cpp-style caller built with g++ against the shim and
libarx.so: config.json -> OBJ scene + receiver halves -> WAV -> render (through libarx's group
API, RCCL) -> convoluteAudioFile -> one convoluteLiveInput callback into a CircularBuffer.  Its
raw outputs are compared with the CPU oracle:
  * IR: bit-exact (integer histogram, same Philox stream);
  * file convolution: max |gpu - oracle| <= 1 ULP(max |oracle|);
  * live block: relative error < 1e-12 (f64 path).
Run once on one GPU (a one-GPU RCCL group) and once sharded 4 ways on it; both must agree.
"""
import json
import os
import shutil
import subprocess

import numpy as np
import pytest

import pyoracle as po
from audiorenderingv2_amd import receiver_local
from audiorenderingv2_amd.formats import save_wav, write_float_lines
from audiorenderingv2_amd.live import CircularBuffer
from audiorenderingv2_amd.scene import load_meshes_npz, reference_config_materials, scene_from_meshes
from conftest import GOLDEN, REPO, world_scene

pytestmark = pytest.mark.gpu


def write_obj(path, meshes, mtl_name):
    lines = [f"mtllib {mtl_name}"]
    base = 1
    for k, m in enumerate(meshes):
        lines.append(f"o shape{k}")
        for v in m.vertices:
            lines.append("v " + " ".join(f"{float(c):.9g}" for c in v))
        lines.append(f"usemtl {m.name}")
        for f in m.faces:
            lines.append("f " + " ".join(str(int(i) + base) for i in f))
        base += len(m.vertices)
    with open(path, "w") as fh:
        fh.write("\n".join(lines) + "\n")
    with open(os.path.join(os.path.dirname(path), mtl_name), "w") as fh:
        fh.write("".join(f"newmtl {n}\n" for n in sorted({m.name for m in meshes})))


def write_receivers(d):
    from audiorenderingv2_amd.scene import Mesh

    L, R = receiver_local()
    for tris, fn in ((L, "leftHalf.obj"), (R, "rightHalf.obj")):
        v = tris.reshape(-1, 3)
        write_obj(str(d / fn), [Mesh("half", v, np.arange(v.shape[0], dtype=np.int32).reshape(-1, 3))], fn + ".mtl")


@pytest.fixture(scope="module")
def demo(tmp_path_factory):
    gxx = shutil.which("g++")
    if not gxx:
        pytest.skip("g++ not available")
    d = tmp_path_factory.mktemp("shim")
    exe = str(d / "export_demo")
    pkg = os.path.join(REPO, "audiorenderingv2_amd")
    subprocess.run([gxx, "-std=c++17", "-O2", "-I", os.path.join(REPO, "include"),
                    os.path.join(REPO, "tests", "cpp", "export_demo.cpp"), "-L", pkg, "-larx", f"-Wl,-rpath,{pkg}",
                    "-o", exe], check=True)
    return d, exe


def test_cpp_shim_export_flow_matches_oracle(demo):
    d, exe = demo
    meshes = load_meshes_npz(os.path.join(GOLDEN, "test_obj.npz"))  # R/test.obj as the reference's tinyobj read it
    write_obj(str(d / "room.obj"), meshes, "room.mtl")
    write_receivers(d)
    sr = 16000
    rng = np.random.default_rng(5)
    t = np.arange(3 * sr + 1234) / sr
    x = (0.4 * np.sin(2 * np.pi * 330 * t) + 0.05 * rng.standard_normal(t.size)).astype(np.float32)
    save_wav(str(d / "in.wav"), x, sr, 32)
    mats = reference_config_materials()
    emitter, listener = (0.5, 3.0, 1.0), (2.5, 9.9, 0.0)
    cfg = {
        "renderer_parameters": {"ir_length_in_seconds": 2},
        "scene_parameters": {"mono": False, "scene_file_path": str(d / "room.obj"), "audio_file_path": str(d / "in.wav"),
                             "initial_receiver_pos": dict(zip("xyz", listener)),
                             "initial_emitter_pos": dict(zip("xyz", emitter))},
        "pathtracer_parameters": {"base_power": 3.62, "rays": {"x": 64, "y": 64, "z": 8}, "ray_energy_threshold": 0.0,
                                  "ray_max_bounces": 8, "hrtf_absorption_rate": 0.25,
                                  "materials": [{"name": n, "mat_absorption": a} for n, a in mats]},
    }
    (d / "config.json").write_text(json.dumps(cfg))
    # oracle on the same inputs (scene as loaded by the reference's loader; hrtf round()ed by the config reader)
    scene = scene_from_meshes(meshes, mats)
    tv, ta = world_scene(scene, listener, 0.0)
    p = po.make_params(rays=(64, 64, 8), sample_rate=sr, base_power=float(np.float32(3.62)), max_bounces=8, hrtf=0.0,
                       emitter=emitter, listener=listener)
    hl, hr, ost = po.Scene(tv, ta, bvh=True).trace(p, threads=8)
    ol, orr = po.finalize_ir(p, hl, hr)
    assert ost["receiver_hits"] > 0
    results = []
    for devices in ("0", "0,0,0,0"):
        out = d / f"out_{devices.count(',') + 1}"
        out.mkdir()
        dumps = devices == "0"  # replay key P (main.cpp:317-322) on the one-GPU run
        run = subprocess.run([exe, str(d / "config.json"), str(d / "leftHalf.obj"), str(d / "rightHalf.obj"), str(out),
                              devices] + (["dumps"] if dumps else []), capture_output=True, text=True, timeout=120)
        assert run.returncode == 0, run.stderr
        if dumps:  # the reference's text dumps, byte for byte against the oracle written the same way
            assert "dumps ok" in run.stdout
            for name, data in (("output_ir_left", ol), ("output_ir_right", orr),
                               ("output_convolute_left", po.convolute_audio(x, sr, ol)),
                               ("output_convolute_right", po.convolute_audio(x, sr, orr))):
                write_float_lines(str(d / f"{name}.oracle"), data)
                got, want = (out / f"{name}.txt.first").read_bytes(), (d / f"{name}.oracle").read_bytes()
                if name.startswith("output_ir"):
                    assert got == want, name
                else:  # the convolution agrees to 1 ULP(max): compare the parsed values
                    g = np.array(got.split(), np.float64)
                    w = np.array(want.split(), np.float64)
                    assert g.size == w.size == x.size
                    # 1 ULP(max) plus the 6-significant-digit rounding of each printed value
                    tol = np.spacing(np.float32(np.abs(w).max())) + 1e-5 * np.abs(w)
                    assert np.all(np.abs(g - w) <= tol), name
        line = [ln for ln in run.stdout.splitlines() if ln.startswith("queries ")][-1]
        st = dict(zip(line.split()[::2], line.split()[1::2]))
        assert int(st["gpus"]) == devices.count(",") + 1
        assert (int(st["queries"]), int(st["receiver_hits"]), int(st["misses"])) == \
            (ost["queries"], ost["receiver_hits"], ost["misses"])
        gl = np.fromfile(out / "ir_left.f32", np.float32)
        gr = np.fromfile(out / "ir_right.f32", np.float32)
        assert np.array_equal(gl.view(np.uint32), ol.view(np.uint32))
        assert np.array_equal(gr.view(np.uint32), orr.view(np.uint32))
        for ch, ir in (("left", ol), ("right", orr)):
            got = np.fromfile(out / f"conv_{ch}.f32", np.float32)
            ref = po.convolute_audio(x, sr, ir)
            assert np.abs(got - ref).max() <= np.spacing(np.float32(np.abs(ref).max()))
        live = np.fromfile(out / "live.f64", np.float64)
        cb = CircularBuffer(44100 * 2)
        cb.add(po.convolute_live_block(x[np.arange(4096) % x.size].astype(np.float64), ol, orr))
        ref = cb.get_and_reset(2 * 4096)
        assert np.abs(live - ref).max() <= 1e-12 * np.abs(ref).max()
        results.append((gl, gr))
    assert np.array_equal(results[0][0], results[1][0]) and np.array_equal(results[0][1], results[1][1])


def test_cpp_shim_c4_sharded_equals_python_group(demo):
    """configs[3] through the C++ shim: the conference stand-in as an OBJ file, 10 M rays x 32
    bounces at 48 kHz, 8 ray shards on the one GPU (group API).  Its IR must be bit-identical to the
    Python RenderGroup's single-device render of the same OBJ (the configs[3] path that
    tests/test_gpu_group.py::test_c4_sharded_group checks against the oracle on ray samples)."""
    from audiorenderingv2_amd import RenderGroup, RenderSettings
    from audiorenderingv2_amd.formats import load_scene
    from audiorenderingv2_amd.scene import CONFERENCE_EMITTER, CONFERENCE_LISTENER, conference_standin

    d, exe = demo
    write_receivers(d)
    sc = conference_standin()
    lines = ["mtllib conf.mtl"]
    base = 1
    start = 0
    names = sc.names
    while start < sc.n_tris:  # one OBJ object per run of equal material names
        end = start
        while end < sc.n_tris and names[end] == names[start]:
            end += 1
        lines.append(f"o part{start}")
        v = sc.tri_v[start:end].reshape(-1, 3)
        lines.extend("v %.9g %.9g %.9g" % tuple(p) for p in v.tolist())
        lines.append(f"usemtl {names[start]}")
        lines.extend(f"f {base + 3 * k} {base + 3 * k + 1} {base + 3 * k + 2}" for k in range(end - start))
        base += v.shape[0]
        start = end
    (d / "conf.obj").write_text("\n".join(lines) + "\n")
    (d / "conf.mtl").write_text("".join(f"newmtl {n}\n" for n in sorted(set(names))))
    sr = 48000
    x = (0.3 * np.sin(2 * np.pi * 440 * np.arange(2 * sr + 777) / sr)).astype(np.float32)
    save_wav(str(d / "conf.wav"), x, sr, 32)
    cfg = {
        "renderer_parameters": {"ir_length_in_seconds": 2},
        "scene_parameters": {"mono": False, "scene_file_path": str(d / "conf.obj"), "audio_file_path": str(d / "conf.wav"),
                             "initial_receiver_pos": dict(zip("xyz", CONFERENCE_LISTENER)),
                             "initial_emitter_pos": dict(zip("xyz", CONFERENCE_EMITTER))},
        "pathtracer_parameters": {"base_power": 3.62, "rays": {"x": 1000, "y": 100, "z": 100},
                                  "ray_energy_threshold": 0.0, "ray_max_bounces": 32, "hrtf_absorption_rate": 1.0,
                                  "materials": []},
    }
    (d / "conf.json").write_text(json.dumps(cfg))
    out = d / "out_c4"
    out.mkdir()
    run = subprocess.run([exe, str(d / "conf.json"), str(d / "leftHalf.obj"), str(d / "rightHalf.obj"), str(out),
                          ",".join(["0"] * 8)], capture_output=True, text=True, timeout=200)
    assert run.returncode == 0, run.stderr
    line = [ln for ln in run.stdout.splitlines() if ln.startswith("queries ")][-1]
    st = dict(zip(line.split()[::2], line.split()[1::2]))
    assert int(st["gpus"]) == 8
    # the same OBJ through the Python loader (the same native tinyobj restatement) and a one-GPU group
    scene = load_scene(str(d / "conf.obj"))
    s = RenderSettings(rays=(1000, 100, 100), sample_rate=sr, base_power=3.62, max_bounces=32,
                       hrtf_absorption_rate=1.0, ir_length_in_seconds=2)
    g = RenderGroup(s, devices=[0], scene=scene, receiver=receiver_local())
    g.setEmitterPosInOptix(CONFERENCE_EMITTER)
    g.setSphereCenterInOptix(CONFERENCE_LISTENER, 0.0)
    g.render()
    gl, gr = g.get_ir()
    gst = g.stats()
    g.close()
    assert int(st["queries"]) == gst["queries"] and int(st["receiver_hits"]) == gst["receiver_hits"]
    assert 20 * 10_000_000 < gst["queries"] <= 32 * 10_000_000 and gst["receiver_hits"] > 10000
    assert np.array_equal(np.fromfile(out / "ir_left.f32", np.float32).view(np.uint32), gl.view(np.uint32))
    assert np.array_equal(np.fromfile(out / "ir_right.f32", np.float32).view(np.uint32), gr.view(np.uint32))


@pytest.mark.parametrize("frames", [1, 2])
def test_main_style_full_render_matches_oracle(demo, frames):
    """main.cpp:40-67's full_render, unchanged, over the shim (tests/cpp/main_style_demo.cpp): an
    OptixModel*, a Sphere of two HalfSpheres, a gdt::vec3f camera point and glm::vec3 setters.  The file
    branch (full_render_cycle under the caller's mutex) renders with the receiver placed at the camera
    and rotated by its angle, then convolves; the live branch (placeReceiver + setSphereCenterInOptix +
    render) follows a moved, turned camera.  Both IRs bit-exact vs the oracle at those poses, the
    convolution <= 1 ULP(max).  Also with two frames in flight (setFramesInFlight): the same results."""
    d, _ = demo
    d = d / f"main_fif{frames}"
    d.mkdir()
    exe = str(d / "main_style_demo")
    pkg = os.path.join(REPO, "audiorenderingv2_amd")
    subprocess.run([shutil.which("g++"), "-std=c++17", "-O2", "-I", os.path.join(REPO, "include"),
                    os.path.join(REPO, "tests", "cpp", "main_style_demo.cpp"), "-L", pkg, "-larx",
                    f"-Wl,-rpath,{pkg}", "-o", exe], check=True)
    meshes = load_meshes_npz(os.path.join(GOLDEN, "test_obj.npz"))
    write_obj(str(d / "room2.obj"), meshes, "room2.mtl")
    write_receivers(d)
    sr = 16000
    x = (0.3 * np.sin(2 * np.pi * 220 * np.arange(2 * sr + 99) / sr)).astype(np.float32)
    save_wav(str(d / "in2.wav"), x, sr, 32)
    mats = reference_config_materials()
    emitter, listener, angle = (0.5, 3.0, 1.0), (2.5, 9.9, 0.0), 40.0
    cfg = {
        "renderer_parameters": {"ir_length_in_seconds": 2},
        "scene_parameters": {"mono": False, "scene_file_path": str(d / "room2.obj"), "audio_file_path": str(d / "in2.wav"),
                             "initial_receiver_pos": dict(zip("xyz", listener)),
                             "initial_emitter_pos": dict(zip("xyz", emitter))},
        "pathtracer_parameters": {"base_power": 3.62, "rays": {"x": 64, "y": 64, "z": 8}, "ray_energy_threshold": 0.0,
                                  "ray_max_bounces": 8, "hrtf_absorption_rate": 0.25,
                                  "materials": [{"name": n, "mat_absorption": a} for n, a in mats]},
    }
    (d / "config2.json").write_text(json.dumps(cfg))
    out = d / "out_main"
    out.mkdir()
    run = subprocess.run([exe, str(d / "config2.json"), str(d / "leftHalf.obj"), str(d / "rightHalf.obj"), str(out),
                          str(angle), str(frames)], capture_output=True, text=True, timeout=120)
    assert run.returncode == 0, run.stderr
    scene = scene_from_meshes(meshes, mats)
    moved = (np.float32(listener[0]) + np.float32(0.5), listener[1], np.float32(listener[2]) - np.float32(0.25))
    for tag, pos, yaw in (("file", listener, angle), ("live", moved, angle + 30.0)):
        tv, ta = world_scene(scene, tuple(float(c) for c in pos), yaw)
        p = po.make_params(rays=(64, 64, 8), sample_rate=sr, base_power=float(np.float32(3.62)), max_bounces=8,
                           hrtf=0.0, emitter=emitter, listener=tuple(float(c) for c in pos))
        hl, hr, ost = po.Scene(tv, ta, bvh=True).trace(p, threads=8)
        ol, orr = po.finalize_ir(p, hl, hr)
        assert ost["receiver_hits"] > 0, tag
        gl = np.fromfile(out / f"ir_{tag}_left.f32", np.float32)
        gr = np.fromfile(out / f"ir_{tag}_right.f32", np.float32)
        assert np.array_equal(gl.view(np.uint32), ol.view(np.uint32)), tag
        assert np.array_equal(gr.view(np.uint32), orr.view(np.uint32)), tag
        if tag == "file":
            for ch, ir in (("left", ol), ("right", orr)):
                got = np.fromfile(out / f"conv_{ch}.f32", np.float32)
                ref = po.convolute_audio(x, sr, ir)
                assert np.abs(got - ref).max() <= np.spacing(np.float32(np.abs(ref).max()))
