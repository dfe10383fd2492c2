"""Scene assembly for the C ABI: flat triangle soups with per-triangle absorption.

Mirrors the host-side data flow of the reference: loadOBJ splits a model into one
mesh per (shape, material) (R/prebuild/obj_raytracer/OptixModel.cpp:75-151),
getMaterialAbsorption maps mesh names to absorption (AudioRenderer.cpp:34-56), and
the two receiver half-spheres come from leftHalf.obj / rightHalf.obj
(Context.cpp:190-193).  Mesh data arrive here already triangulated (golden fixtures
produced by the reference's own tinyobj in tests/golden/, or the synthetic
conference stand-in below).
"""
from __future__ import annotations

import json
import os
from dataclasses import dataclass

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(REPO, "tests", "golden")


@dataclass
class Mesh:
    name: str
    vertices: np.ndarray  # (nv, 3) f32
    faces: np.ndarray     # (nt, 3) i32

    def triangles(self) -> np.ndarray:
        return self.vertices[self.faces].reshape(-1, 9).astype(np.float32)


@dataclass
class Scene:
    tri_v: np.ndarray    # (T, 9) f32, P1 P2 P3
    tri_abs: np.ndarray  # (T,) f32
    names: list

    @property
    def n_tris(self) -> int:
        return int(self.tri_v.shape[0])


def material_absorption(name: str, materials: dict[str, float] | list) -> float:
    """getMaterialAbsorption (AudioRenderer.cpp:34-56)."""
    if name == "receiver_left":
        return -1.0
    if name == "receiver_right":
        return -2.0
    items = materials.items() if isinstance(materials, dict) else materials
    for n, a in items:
        if n == name:
            return float(np.float32(a))
    return 0.5


def load_meshes_npz(path: str) -> list[Mesh]:
    d = np.load(path)
    names = [str(x) for x in d["names"]]
    return [Mesh(names[k], d[f"v{k}"].astype(np.float32), d[f"f{k}"].astype(np.int32)) for k in range(len(names))]


def scene_from_meshes(meshes: list[Mesh], materials=()) -> Scene:
    tv, ab, names = [], [], []
    for m in meshes:
        t = m.triangles()
        tv.append(t)
        ab.append(np.full(t.shape[0], material_absorption(m.name, materials), np.float32))
        names.append(m.name)
    if not tv:
        return Scene(np.zeros((0, 9), np.float32), np.zeros(0, np.float32), [])
    return Scene(np.concatenate(tv), np.concatenate(ab), names)


def receiver_local(path: str | None = None) -> tuple[np.ndarray, np.ndarray]:
    """Local-frame triangles (n,9) of the left / right receiver halves."""
    ms = load_meshes_npz(path or os.path.join(GOLDEN, "receiver_local.npz"))
    by = {m.name: m.triangles() for m in ms}
    return by["receiver_left"], by["receiver_right"]


def test_obj_scene(materials=()) -> Scene:
    """R/test.obj (C1 of BASELINE.json) as triangulated by the reference's tinyobj."""
    return scene_from_meshes(load_meshes_npz(os.path.join(GOLDEN, "test_obj.npz")), materials)


REFERENCE_AUDIO = {
    "guitar": "audio_guitar_16k_ch0.npz",           # R/guitar_sample_16k.wav (C1)
    "experimento": "audio_experimento_16k_ch0.npz",  # R/experimento_entrada_16KHz.wav (C2)
    "clapper": "audio_clapper_48k_ch0.npz",          # R/assets/sound_samples/A_Clapper_Board.wav (C3)
}


def reference_audio(name: str) -> tuple[np.ndarray, int]:
    """Channel 0 of a reference WAV as the reference's AudioFile decodes it (golden fixture made by
    tests/golden/make_golden.py through oracle/_ref/refdump): (f32 samples, sample rate)."""
    d = np.load(os.path.join(GOLDEN, REFERENCE_AUDIO[name]))
    if "pcm16" in d:
        x = d["pcm16"].astype(np.float32) / np.float32(32768.0)
    else:
        x = d["f32"].astype(np.float32)
    return x, int(d["sample_rate"])


def reference_config_materials() -> list:
    """pathtracer_parameters.materials of R/config.json (parsed by the reference's cJSON)."""
    with open(os.path.join(GOLDEN, "config_parsed.json")) as fh:
        return [tuple(x) for x in json.load(fh)["materials"]]


# ---------------------------------------------------------------------------------
# Synthetic stand-in for conference.obj (missing from the reference checkout,
# R/.MISSING_LARGE_BLOBS): a closed 20 x 4 x 12 m room (Y up) furnished with boxes
# (tables) and 32-segment cylinders (chairs / columns), material names drawn from
# R/conference.mtl.  Deterministic for a given seed (numpy PCG64).
CONFERENCE_EMITTER = (-5.0, 1.2, 0.0)
CONFERENCE_LISTENER = (5.0, 1.2, 2.0)
ROOM_LO = np.array([-10.0, 0.0, -6.0], np.float32)
ROOM_HI = np.array([10.0, 4.0, 6.0], np.float32)


def _box_tris(lo: np.ndarray, hi: np.ndarray) -> np.ndarray:
    """(k,3),(k,3) -> (k*12, 9) triangles of axis-aligned boxes."""
    x0, y0, z0 = lo[:, 0], lo[:, 1], lo[:, 2]
    x1, y1, z1 = hi[:, 0], hi[:, 1], hi[:, 2]
    c = np.stack([
        np.stack([x0, y0, z0], -1), np.stack([x1, y0, z0], -1), np.stack([x1, y1, z0], -1),
        np.stack([x0, y1, z0], -1), np.stack([x0, y0, z1], -1), np.stack([x1, y0, z1], -1),
        np.stack([x1, y1, z1], -1), np.stack([x0, y1, z1], -1)], 1)  # (k, 8, 3)
    quads = [(0, 1, 2, 3), (4, 7, 6, 5), (0, 4, 5, 1), (3, 2, 6, 7), (0, 3, 7, 4), (1, 5, 6, 2)]
    tris = []
    for a, b, cc, d in quads:
        tris.append(np.concatenate([c[:, a], c[:, b], c[:, cc]], -1))
        tris.append(np.concatenate([c[:, a], c[:, cc], c[:, d]], -1))
    return np.stack(tris, 1).reshape(-1, 9).astype(np.float32)


def _cyl_tris(center: np.ndarray, radius: np.ndarray, y0: np.ndarray, y1: np.ndarray, seg: int = 32) -> np.ndarray:
    k = center.shape[0]
    ang = np.arange(seg + 1) * (2.0 * np.pi / seg)
    cx = center[:, 0:1] + radius[:, None] * np.cos(ang)[None, :]
    cz = center[:, 1:2] + radius[:, None] * np.sin(ang)[None, :]
    bot = np.stack([cx, np.repeat(y0[:, None], seg + 1, 1), cz], -1)  # (k, seg+1, 3)
    top = np.stack([cx, np.repeat(y1[:, None], seg + 1, 1), cz], -1)
    b0, b1, t0, t1 = bot[:, :-1], bot[:, 1:], top[:, :-1], top[:, 1:]
    side0 = np.concatenate([b0, b1, t1], -1)
    side1 = np.concatenate([b0, t1, t0], -1)
    cb = np.stack([center[:, 0], y0, center[:, 1]], -1)[:, None, :].repeat(seg, 1)
    ct = np.stack([center[:, 0], y1, center[:, 1]], -1)[:, None, :].repeat(seg, 1)
    capb = np.concatenate([cb, b1, b0], -1)
    capt = np.concatenate([ct, t0, t1], -1)
    return np.concatenate([side0, side1, capb, capt], 1).reshape(k * 4 * seg, 9).astype(np.float32)


def conference_standin(seed: int = 42, n_boxes: int = 400, n_cylinders: int = 2540, materials=()) -> Scene:
    """~3.3e5-triangle deterministic stand-in for conference.obj."""
    rng = np.random.Generator(np.random.PCG64(seed))
    with open(os.path.join(GOLDEN, "conference_materials.json")) as fh:
        mat_names = json.load(fh)
    # room shell, material Material__0
    room = _box_tris(ROOM_LO[None, :], ROOM_HI[None, :])
    keep_out = np.array([[CONFERENCE_EMITTER[0], CONFERENCE_EMITTER[2]],
                         [CONFERENCE_LISTENER[0], CONFERENCE_LISTENER[2]]], np.float32)

    def place(n, margin):
        pts = np.empty((0, 2), np.float32)
        while pts.shape[0] < n:
            cand = rng.uniform([-9.3, -5.3], [9.3, 5.3], size=(2 * n, 2)).astype(np.float32)
            d = np.min(np.linalg.norm(cand[:, None, :] - keep_out[None], axis=-1), axis=1)
            pts = np.concatenate([pts, cand[d > margin]])
        return pts[:n]

    bc = place(n_boxes, 2.2)
    half = rng.uniform([0.25, 0.25], [0.7, 0.7], size=(n_boxes, 2)).astype(np.float32)
    h = rng.uniform(0.4, 1.1, size=n_boxes).astype(np.float32)
    lo = np.stack([bc[:, 0] - half[:, 0], np.zeros(n_boxes, np.float32), bc[:, 1] - half[:, 1]], -1)
    hi = np.stack([bc[:, 0] + half[:, 0], h, bc[:, 1] + half[:, 1]], -1)
    boxes = _box_tris(lo, hi)
    cc = place(n_cylinders, 1.6)
    rad = rng.uniform(0.12, 0.3, size=n_cylinders).astype(np.float32)
    y0 = rng.uniform(0.0, 0.2, size=n_cylinders).astype(np.float32)
    y1 = y0 + rng.uniform(0.4, 2.5, size=n_cylinders).astype(np.float32)
    cyl = _cyl_tris(cc, rad, y0, y1)
    box_mats = rng.integers(1, len(mat_names), size=n_boxes)
    cyl_mats = rng.integers(1, len(mat_names), size=n_cylinders)
    names = [mat_names[0]] * 12 + [mat_names[i] for i in np.repeat(box_mats, 12)] + \
            [mat_names[i] for i in np.repeat(cyl_mats, 128)]
    tri_v = np.concatenate([room, boxes, cyl]).astype(np.float32)
    lut = {n: material_absorption(n, materials) for n in mat_names}
    tri_abs = np.array([lut[n] for n in names], np.float32)
    return Scene(tri_v, tri_abs, names)
