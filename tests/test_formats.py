"""Native input-format loaders (csrc/arx_io.cpp) against the reference's own parsers.

Pinned three ways:
  * committed golden fixtures (tests/golden/, produced by the reference's tinyobj / AudioFile /
    cJSON through oracle/_ref/refdump) -- bit-exact vertices, indices, samples, config values;
  * a differential sweep over every OBJ / WAV in the reference checkout and over randomly
    generated OBJ, WAV and JSON inputs, run through refdump (the reference code compiled from
    /root/reference) -- skipped where /root/reference or refdump is absent (GPU box);
  * self-contained known-answer cases that need neither.
Host only: no device is touched.
"""
import json
import os
import struct
import subprocess
import sys

import numpy as np
import pytest

from audiorenderingv2_amd import ArxError
from audiorenderingv2_amd.formats import load_config, load_obj, load_receiver_half, load_scene, load_wav, parse_config
from audiorenderingv2_amd.renderer import place_receiver_vertices
from audiorenderingv2_amd.scene import load_meshes_npz
from conftest import REPO

REF = "/root/reference"
GOLDEN = os.path.join(REPO, "tests", "golden")
REFDUMP = os.path.join(REPO, "oracle", "_ref", "refdump")
MODELS = os.path.join(REF, "assets", "models")

sys.path.insert(0, GOLDEN)
import make_golden  # noqa: E402  (fixture-format parser shared with the generator)

need_ref = pytest.mark.skipif(not os.path.isdir(REF), reason="reference checkout absent (only in the build container)")
need_refdump = pytest.mark.skipif(not (os.path.isdir(REF) and os.path.exists(REFDUMP)),
                                  reason="oracle/_ref/refdump not built (make -C oracle ref)")


def bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


def assert_meshes_equal(got, ref_names, ref_v, ref_f):
    assert [m.name or "<none>" for m in got] == list(ref_names)
    for m, v, f in zip(got, ref_v, ref_f):
        assert m.vertices.shape == v.shape and m.faces.shape == f.shape
        np.testing.assert_array_equal(bits(m.vertices), bits(v))
        np.testing.assert_array_equal(m.faces, f)


# ------------------------------------------------------------------ fixtures --
OBJ_FIXTURES = [("test_obj.npz", "test.obj"), ("3D_U_obj.npz", "assets/models/3D_U.obj"),
                ("cajaConToro_obj.npz", "assets/models/cajaConToro.obj"),
                ("planaso2_obj.npz", "assets/models/planaso2.obj")]


@need_ref
@pytest.mark.parametrize("fixture,rel", OBJ_FIXTURES)
def test_obj_matches_golden(fixture, rel):
    d = np.load(os.path.join(GOLDEN, fixture))
    meshes, info = load_obj(os.path.join(REF, rel))
    k = len(d["names"])
    assert_meshes_equal(meshes, d["names"], [d[f"v{i}"] for i in range(k)], [d[f"f{i}"] for i in range(k)])
    assert [info.shapes, info.materials, info.vertices] == list(d["header"])


@need_ref
@pytest.mark.parametrize("fixture,pos,yaw", [("receiver_local.npz", (0, 0, 0), 0), ("receiver_c1.npz", (2.5, 9.9, 0), 0),
                                             ("receiver_rot.npz", (-1.25, 2.0, 3.5), 37.5)])
def test_receiver_halves_match_golden(fixture, pos, yaw):
    # HalfSphere load + place_receiver_half: the fixtures are placed meshes (even at the
    # origin, where "0 + vert" turns the model's -0.0 coordinates into +0.0)
    ref = load_meshes_npz(os.path.join(GOLDEN, fixture))
    for side, path in enumerate(("leftHalf.obj", "rightHalf.obj")):
        m = load_receiver_half(os.path.join(MODELS, path), side)
        assert m.name == ref[side].name
        placed = place_receiver_vertices(m.vertices, pos, yaw)
        np.testing.assert_array_equal(bits(placed), bits(ref[side].vertices))
        np.testing.assert_array_equal(m.faces, ref[side].faces)


@need_ref
def test_wav_matches_golden():
    with open(os.path.join(GOLDEN, "wav_decode.json")) as fh:
        fixtures = json.load(fh)
    for fx in fixtures:
        w = load_wav(os.path.join(REF, fx["file"]))
        assert (w.sample_rate, w.channels, w.frames, w.bit_depth) == (
            fx["sample_rate"], fx["channels"], fx["samples_per_channel"], fx["bit_depth"])
        for c in range(w.channels):
            np.testing.assert_array_equal(bits(w.samples[c, :256]), bits(np.array(fx["head"][c], np.float32)))
            np.testing.assert_array_equal(bits(w.samples[c, ::997]), bits(np.array(fx["strided_997"][c], np.float32)))
            assert float(np.sum(w.samples[c], dtype=np.float64)) == fx["sum"][c]
            assert float(np.sum(w.samples[c].astype(np.float64) ** 2)) == fx["sumsq"][c]


def test_reference_audio_fixtures_match_golden():
    """The full channel-0 fixtures (tests/golden/audio_*.npz, used by GPU tests and bench.py where
    the reference tree is absent) agree with the independent head / strided / sum records of the
    reference's AudioFile decode (wav_decode.json)."""
    from audiorenderingv2_amd.scene import reference_audio

    with open(os.path.join(GOLDEN, "wav_decode.json")) as fh:
        fixtures = {os.path.basename(fx["file"]): fx for fx in json.load(fh)}
    for name, fname in (("guitar", "guitar_sample_16k.wav"), ("experimento", "experimento_entrada_16KHz.wav"),
                        ("clapper", "A_Clapper_Board.wav")):
        x, sr = reference_audio(name)
        fx = fixtures[fname]
        assert sr == fx["sample_rate"] and x.size == fx["samples_per_channel"]
        np.testing.assert_array_equal(bits(x[:256]), bits(np.array(fx["head"][0], np.float32)))
        np.testing.assert_array_equal(bits(x[::997]), bits(np.array(fx["strided_997"][0], np.float32)))
        assert float(np.sum(x, dtype=np.float64)) == fx["sum"][0]


def config_as_fixture(c):
    d = {
        "initial_volume": c.initial_volume, "ir_length_in_seconds": c.ir_length_in_seconds, "width": c.width,
        "height": c.height, "write_first_ir_to_file": int(c.write_first_ir_to_file),
        "write_first_output_to_file": int(c.write_first_output_to_file),
        "re_render_distance_threshold": c.re_render_distance_threshold,
        "re_render_angle_threshold": c.re_render_angle_threshold, "mono": int(c.mono),
        "scene_file_path": c.scene_file_path, "audio_file_path": c.audio_file_path or "<none>",
        "materials_file_path": c.materials_file_path or "<none>",
        "initial_receiver_pos": list(c.initial_receiver_pos), "initial_emitter_pos": list(c.initial_emitter_pos),
        "base_power": c.base_power, "rays": list(c.rays), "ray_energy_threshold": c.ray_energy_threshold,
        "ray_max_bounces": c.ray_max_bounces, "hrtf_absorption_rate": c.hrtf_absorption_rate,
        "materials": [[n, a] for n, a in c.materials],
    }
    return d


@need_ref
def test_config_matches_golden():
    with open(os.path.join(GOLDEN, "config_parsed.json")) as fh:
        ref = json.load(fh)
    got = config_as_fixture(load_config(os.path.join(REF, "config.json")))
    assert got == ref


@need_ref
def test_load_scene_flattens_with_absorption():
    mats = [("low", 0.1), ("med", 0.3)]
    s = load_scene(os.path.join(REF, "test.obj"), mats)
    d = load_meshes_npz(os.path.join(GOLDEN, "test_obj.npz"))
    from audiorenderingv2_amd.scene import scene_from_meshes
    ref = scene_from_meshes(d, mats)
    np.testing.assert_array_equal(bits(s.tri_v), bits(ref.tri_v))
    np.testing.assert_array_equal(s.tri_abs, ref.tri_abs)


# ------------------------------------------------- differential vs refdump --
def refdump(*args):
    return subprocess.run([REFDUMP, *args], check=True, capture_output=True, text=True).stdout.splitlines()


def compare_obj_with_refdump(path):
    ref = make_golden.parse_meshes(refdump("obj", path))
    try:
        meshes, info = load_obj(path)
    except ArxError as e:
        # the reference's loadOBJ throws on models without materials; refdump does not check
        assert ref["header"]["materials"] == 0, e
        return
    assert_meshes_equal(meshes, ref["names"], ref["vertices"], ref["indices"])
    assert (info.shapes, info.materials, info.vertices) == (
        ref["header"]["shapes"], ref["header"]["materials"], ref["header"]["vertices"])


def all_reference_objs():
    if not os.path.isdir(REF):
        return []
    out = []
    for root, _, files in os.walk(REF):
        if "/." in root:
            continue
        out += [os.path.join(root, f) for f in files if f.endswith(".obj")]
    return sorted(out)


@need_refdump
@pytest.mark.parametrize("path", all_reference_objs(), ids=lambda p: os.path.relpath(p, REF))
def test_every_reference_obj_matches_tinyobj(path):
    if os.path.getsize(path) > 20_000_000:
        pytest.skip("large model")
    compare_obj_with_refdump(path)


def number(rng):
    kind = rng.integers(0, 7)
    x = rng.uniform(-50, 50)
    if kind == 0:
        return f"{x:.6f}"
    if kind == 1:
        return f"{x:.12f}"  # > 7 fraction digits: pow(10,-k) branch
    if kind == 2:
        return f"{x:.5e}"
    if kind == 3:
        return f"{int(x)}"
    if kind == 4:
        s = f"{abs(x) % 1:.4f}"[1:]  # leading dot
        return ("-" if x < 0 else "") + s
    if kind == 5:
        return f"{x:.3E}".replace("E+0", "E+").replace("E-0", "E-")
    return f"+{abs(x):.2f}"


def random_obj(rng, tmp_path, k):
    mtl = tmp_path / f"m{k}.mtl"
    mats = [f"mat{i}" for i in range(4)]
    mtl.write_text("".join(f"newmtl {m}\nKd 0.5 0.5 0.5\n" for m in mats))
    lines = [f"mtllib missing.mtl m{k}.mtl"]
    nv = nvn = 0
    for _ in range(int(rng.integers(1, 5))):
        head = rng.choice(["o", "g", "none"])
        if head != "none":
            lines.append(f"{head} part{int(rng.integers(0, 99))}")
        for _ in range(int(rng.integers(1, 6))):
            if rng.uniform() < 0.5:
                lines.append(f"usemtl {rng.choice(mats + ['unknown'])}")
            # a star / concave polygon in a random plane
            n = int(rng.integers(3, 9))
            ang = np.sort(rng.uniform(0, 2 * np.pi, n))
            rad = rng.uniform(0.3, 2.0, n)
            axes = rng.permutation(3)
            base = nv
            for a, r in zip(ang, rad):
                p = np.zeros(3)
                p[axes[0]] = r * np.cos(a)
                p[axes[1]] = r * np.sin(a)
                p[axes[2]] = rng.uniform(-0.01, 0.01) if rng.uniform() < 0.3 else 0.0
                lines.append("v " + " ".join(number(rng) if rng.uniform() < 0.2 else f"{c:.6f}" for c in p))
                nv += 1
            if rng.uniform() < 0.3:
                lines.append("vn 0 1 0")
                lines.append("vt 0.5 0.5")
                nvn += 1
            corners = []
            for i in range(n):
                if rng.uniform() < 0.2:
                    c = str(base + i - nv)  # relative index
                else:
                    c = str(base + i + 1)
                if nvn:  # i/j, i//k, i/j/k with distinct (v,n,t) keys for the dedup map
                    j = int(rng.integers(1, nvn + 1))
                    c += ["", f"/{j}", f"//{j}", f"/{j}/{j}"][int(rng.integers(0, 4))]
                corners.append(c)
            lines.append("f " + " ".join(corners))
    sep = "\r\n" if rng.uniform() < 0.3 else "\n"
    path = tmp_path / f"r{k}.obj"
    path.write_bytes((sep.join(lines) + sep).encode())
    return str(path)


@need_refdump
def test_random_objs_match_tinyobj(tmp_path):
    rng = np.random.default_rng(11)
    for k in range(60):
        compare_obj_with_refdump(random_obj(rng, tmp_path, k))


def write_wav(path, data, sr, bits_, fmt):
    """data: (ch, n) integer codes (PCM) or float32 (fmt 3)."""
    ch, n = data.shape
    inter = data.T.reshape(-1)
    if fmt == 3:
        payload = inter.astype("<f4").tobytes()
    elif bits_ == 8:
        payload = inter.astype(np.uint8).tobytes()
    elif bits_ == 16:
        payload = inter.astype("<i2").tobytes()
    elif bits_ == 24:
        v = inter.astype(np.int64) & 0xFFFFFF
        payload = np.stack([v & 0xFF, (v >> 8) & 0xFF, (v >> 16) & 0xFF], 1).astype(np.uint8).tobytes()
    else:
        payload = inter.astype("<i4").tobytes()
    block = ch * bits_ // 8
    fmt_chunk = struct.pack("<4sIHHIIHH", b"fmt ", 16, fmt, ch, sr, sr * block, block, bits_)
    junk = struct.pack("<4sI", b"LIST", 6) + b"abcdef"
    data_chunk = struct.pack("<4sI", b"data", len(payload)) + payload
    body = b"WAVE" + fmt_chunk + junk + data_chunk
    with open(path, "wb") as fh:
        fh.write(struct.pack("<4sI", b"RIFF", len(body)) + body)


def random_wav(rng, path):
    bits_, fmt = [(8, 1), (16, 1), (24, 1), (32, 1), (32, 3)][int(rng.integers(0, 5))]
    ch = int(rng.integers(1, 3))
    n = int(rng.integers(1, 3000))
    sr = int(rng.choice([8000, 16000, 44100, 48000]))
    if fmt == 3:
        data = rng.uniform(-1, 1, (ch, n)).astype(np.float32)
    else:
        hi = 1 << (bits_ - 1)
        data = rng.integers(-hi, hi, (ch, n))
        if bits_ == 8:
            data = data + 128
    write_wav(path, data, sr, bits_, fmt)
    return sr, ch, n, bits_


@need_refdump
def test_random_wavs_match_audiofile(tmp_path):
    rng = np.random.default_rng(5)
    for k in range(25):
        p = str(tmp_path / f"w{k}.wav")
        random_wav(rng, p)
        lines = refdump("wav", p)
        sr, ch, n, b = (int(x) for x in lines[0].split()[1:])
        ref = np.array([float.fromhex(x) for x in lines[1:]], np.float32).reshape(ch, n)
        w = load_wav(p)
        assert (w.sample_rate, w.channels, w.frames, w.bit_depth) == (sr, ch, n, b)
        np.testing.assert_array_equal(bits(w.samples), bits(ref))


def random_config(rng):
    def num():
        return float(rng.choice([rng.uniform(-3, 200), int(rng.integers(0, 500)), 2.5, 3.5, 0.49999]))

    def key(k):
        return k.upper() if rng.uniform() < 0.15 else k

    cfg = {}
    rp = {}
    for k in ("initial_volume", "ir_length_in_seconds", "width", "height", "re_render_distance_threshold",
              "re_render_angle_threshold"):
        if rng.uniform() < 0.7:
            rp[key(k)] = abs(num())
    for k in ("write_first_ir_to_file", "write_first_output_to_file"):
        if rng.uniform() < 0.6:
            rp[k] = bool(rng.uniform() < 0.5) if rng.uniform() < 0.8 else "yes"
    sp = {}
    if rng.uniform() < 0.6:
        sp["mono"] = bool(rng.uniform() < 0.5)
    for k in ("scene_file_path", "audio_file_path", "materials_file_path"):
        if rng.uniform() < 0.6:
            sp[k] = f"dir/{k}_{int(rng.integers(0, 9))}.x"
    for k in ("initial_receiver_pos", "initial_emitter_pos"):
        if rng.uniform() < 0.7:
            sp[k] = {"x": num(), "y": num(), "z": num() if rng.uniform() < 0.9 else "bad"}
    pp = {}
    for k in ("base_power", "ray_energy_threshold", "ray_max_bounces", "hrtf_absorption_rate"):
        if rng.uniform() < 0.7:
            pp[key(k)] = abs(num())
    if rng.uniform() < 0.7:
        pp["rays"] = {"x": float(rng.integers(1, 300)), "y": 10.7, "z": 3}
    pp["materials"] = [{"name": f"m{i}", "mat_absorption": float(rng.uniform(0, 1))} if rng.uniform() < 0.85 else
                       {"name": 5, "mat_absorption": 0.3} for i in range(int(rng.integers(0, 6)))]
    for name, sec in (("renderer_parameters", rp), ("scene_parameters", sp), ("pathtracer_parameters", pp)):
        if rng.uniform() < 0.9:
            cfg[name] = sec
    return cfg


def parse_refdump_config(lines):
    cfg, mats = {}, []
    for line in lines:
        k, _, rest = line.partition(" ")
        if k == "material":
            n, v = rest.split()
            mats.append([n, float.fromhex(v)])
            continue
        vals = []
        for t in rest.split():
            try:
                vals.append(float.fromhex(t) if "0x" in t else int(t))
            except ValueError:
                vals.append(t)
        cfg[k] = vals[0] if len(vals) == 1 else vals
    cfg["materials"] = mats
    return cfg


@need_refdump
def test_random_configs_match_cjson(tmp_path):
    rng = np.random.default_rng(3)
    for k in range(40):
        text = json.dumps(random_config(rng), indent=int(rng.integers(0, 3)))
        if rng.uniform() < 0.2:
            text += "\n trailing text ignored by cJSON_Parse"
        p = tmp_path / f"c{k}.json"
        p.write_text(text)
        ref = parse_refdump_config(refdump("config", str(p)))
        got = config_as_fixture(load_config(str(p)))
        for kk in ("rays", "initial_receiver_pos", "initial_emitter_pos"):
            got[kk] = [float(x) for x in got[kk]]
            ref[kk] = [float(x) for x in ref[kk]]
        assert got == ref, text


# ------------------------------------------------------- self-contained KATs --
def test_obj_known_answers(tmp_path):
    (tmp_path / "a.mtl").write_text("newmtl wood\nKd 1 1 1\nnewmtl stone  \n")
    (tmp_path / "a.obj").write_text(
        "mtllib a.mtl\n"
        "v 0 0 0\nv 1 0 0\nv 1 1 0\nv 0 1 0\n"
        "v .5 -2.5e-1 1e1\n"
        "usemtl wood\nf 1 2 3 4\n"           # quad -> 2 triangles
        "usemtl stone\nf -5 -4 -1\n"         # relative indices
        "usemtl wood\nf 1/1 2//1 5/1/1\n"
    )
    meshes, info = load_obj(str(tmp_path / "a.obj"))
    assert (info.shapes, info.materials, info.vertices) == (1, 2, 5)
    assert [m.name for m in meshes] == ["wood", "stone"]
    assert meshes[0].faces.shape == (3, 3) and meshes[1].faces.shape == (1, 3)
    np.testing.assert_array_equal(meshes[1].vertices, np.array([[0, 0, 0], [1, 0, 0], [0.5, -0.25, 10]], np.float32))
    # a model without materials is rejected like loadOBJ's throw
    (tmp_path / "b.obj").write_text("v 0 0 0\nv 1 0 0\nv 0 1 0\nf 1 2 3\n")
    with pytest.raises(ArxError):
        load_obj(str(tmp_path / "b.obj"))
    with pytest.raises(ArxError):
        load_obj(str(tmp_path / "missing.obj"))


def test_wav_known_answers(tmp_path):
    p = str(tmp_path / "x.wav")
    write_wav(p, np.array([[-32768, 0, 16384, 32767]]), 16000, 16, 1)
    w = load_wav(p)
    np.testing.assert_array_equal(w.samples[0], np.array([-1.0, 0.0, 0.5, 32767 / 32768], np.float32))
    write_wav(p, np.array([[0, 128, 255], [64, 192, 1]]), 8000, 8, 1)
    w = load_wav(p)
    assert w.samples.shape == (2, 3)
    np.testing.assert_array_equal(w.samples[0], np.array([-1.0, 0.0, 127 / 128], np.float32))
    write_wav(p, np.array([[-(1 << 23), (1 << 22)]]), 44100, 24, 1)
    np.testing.assert_array_equal(load_wav(p).samples[0], np.array([-1.0, 0.5], np.float32))
    with open(p, "wb") as fh:
        fh.write(b"RIFX0000WAVE")
    with pytest.raises(ArxError):
        load_wav(p)


def test_config_defaults_and_quirks():
    c = parse_config("{}")
    assert (c.ir_length_in_seconds, c.width, c.height, c.ray_max_bounces) == (2, 1366, 768, 10)
    assert c.scene_file_path == "../../assets/models/1D_U.obj" and c.live
    assert c.initial_receiver_pos == (-2.5, 10.0, 0.0)
    assert c.hrtf_absorption_rate == np.float32(0.9)
    c = parse_config('{"PathTracer_Parameters": {"HRTF_absorption_rate": 0.6, "ray_max_bounces": 2.5,'
                     ' "base_power": 1, "base_power": 7, "rays": {"x": 10.9, "y": 2, "z": 1},'
                     ' "materials": [{"name": "a", "mat_absorption": 0.25}, {"name": "b"}]}} junk')
    assert c.hrtf_absorption_rate == 1.0        # round()ed like Context.cpp:147
    assert c.ray_max_bounces == 3               # round half away from zero
    assert c.base_power == 1.0                  # first duplicate wins
    assert c.rays_per_dimension() == (10, 2, 1)
    assert c.materials == [("a", 0.25)]
    with pytest.raises(ArxError):
        parse_config('{"renderer_parameters": {')
