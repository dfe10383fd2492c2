"""Input formats of the reference app, read by libarx.so's native loaders (csrc/arx_io.cpp).

    load_obj(path)                 -- loadOBJ (R/prebuild/obj_raytracer/OptixModel.cpp:75-151)
    load_receiver_half(path, side) -- HalfSphere + place_receiver_half (HalfSphere.cpp:3-31,
                                      OptixModel.cpp:197-220), local frame
    load_wav(path)                 -- AudioFile<float>::load (R/prebuild/obj_raytracer/AudioFile.h)
    load_config(path)              -- Context::loadContext parameters (Context.cpp:15-164)
    load_scene(path, materials)    -- loadOBJ + getMaterialAbsorption as one triangle soup

All parsing is native (C++); these are thin ctypes wrappers that copy results into numpy.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass, field

import numpy as np

from ._lib import ArxAppConfig, check, lib
from .scene import Mesh, Scene

RECEIVER_NAMES = ("receiver_left", "receiver_right")


@dataclass
class ObjInfo:
    shapes: int
    materials: int
    vertices: int


def _model_meshes(handle) -> list[Mesh]:
    L = lib()
    out = []
    for i in range(L.arx_model_mesh_count(handle)):
        name = C.c_char_p()
        v = C.POINTER(C.c_float)()
        idx = C.POINTER(C.c_int32)()
        nv = C.c_int64()
        nt = C.c_int64()
        check(L.arx_model_mesh(handle, i, C.byref(name), C.byref(v), C.byref(nv), C.byref(idx), C.byref(nt)))
        verts = np.ctypeslib.as_array(v, shape=(nv.value * 3,)).reshape(-1, 3).copy() if nv.value else \
            np.zeros((0, 3), np.float32)
        faces = np.ctypeslib.as_array(idx, shape=(nt.value * 3,)).reshape(-1, 3).copy() if nt.value else \
            np.zeros((0, 3), np.int32)
        out.append(Mesh((name.value or b"").decode(), verts, faces))
    return out


class _Model:
    def __init__(self, path: str, mtl_dir: str | None, first_shape_only: bool, forced_name: str | None):
        h = C.c_void_p()
        check(lib().arx_model_load_obj(os.fsencode(path), None if mtl_dir is None else os.fsencode(mtl_dir),
                                       int(first_shape_only), None if forced_name is None else forced_name.encode(),
                                       C.byref(h)))
        self.h = h

    def __enter__(self):
        return self.h

    def __exit__(self, *exc):
        lib().arx_model_free(self.h)


def load_obj(path: str, mtl_dir: str | None = None) -> tuple[list[Mesh], ObjInfo]:
    """Meshes of an OBJ scene: one per (shape, material id ascending), names = material names."""
    with _Model(path, mtl_dir, False, None) as h:
        s, m, v = C.c_int64(), C.c_int64(), C.c_int64()
        lib().arx_model_info(h, C.byref(s), C.byref(m), C.byref(v))
        return _model_meshes(h), ObjInfo(s.value, m.value, v.value)


def load_receiver_half(path: str, side: int) -> Mesh:
    """A receiver half in its local frame (shapes[0] only; mtlDir without the trailing '/')."""
    mtl_dir = path[:path.rfind("/")] if "/" in path else ""
    with _Model(path, mtl_dir, True, RECEIVER_NAMES[side]) as h:
        meshes = _model_meshes(h)
    if len(meshes) != 1:
        # place_receiver_half keeps the LAST mesh when shapes[0] spans several materials
        # (each push_back first erases the previous one, OptixModel.cpp:232-251)
        meshes = meshes[-1:]
    return meshes[0]


def _materials_arrays(materials):
    items = list(materials.items()) if isinstance(materials, dict) else list(materials)
    names = (C.c_char_p * max(1, len(items)))(*[n.encode() for n, _ in items])
    ab = np.array([a for _, a in items] or [0.0], np.float32)
    return names, ab, len(items)


def load_scene(path: str, materials=(), mtl_dir: str | None = None) -> Scene:
    """loadOBJ + getMaterialAbsorption per mesh, flattened natively (arx_model_flatten)."""
    L = lib()
    with _Model(path, mtl_dir, False, None) as h:
        n = L.arx_model_triangle_count(h)
        tv = np.zeros((n, 9), np.float32)
        ta = np.zeros(n, np.float32)
        names, ab, nm = _materials_arrays(materials)
        check(L.arx_model_flatten(h, names, ab.ctypes.data_as(C.POINTER(C.c_float)), nm,
                                  tv.ctypes.data_as(C.POINTER(C.c_float)), ta.ctypes.data_as(C.POINTER(C.c_float))))
        mesh_names = [m.name for m in _model_meshes(h)]
    return Scene(tv, ta, mesh_names)


@dataclass
class Wav:
    samples: np.ndarray  # (channels, frames) f32, AudioFile::samples layout
    sample_rate: int
    bit_depth: int

    @property
    def channels(self) -> int:
        return int(self.samples.shape[0])

    @property
    def frames(self) -> int:
        return int(self.samples.shape[1])


def load_wav(path: str) -> Wav:
    L = lib()
    p = C.POINTER(C.c_float)()
    ch, sr, bits = C.c_int32(), C.c_int32(), C.c_int32()
    n = C.c_int64()
    check(L.arx_wav_load(os.fsencode(path), C.byref(p), C.byref(ch), C.byref(n), C.byref(sr), C.byref(bits)))
    try:
        count = ch.value * n.value
        data = np.ctypeslib.as_array(p, shape=(count,)).copy() if count else np.zeros(0, np.float32)
    finally:
        L.arx_free(C.cast(p, C.c_void_p))
    return Wav(data.reshape(ch.value, n.value), sr.value, bits.value)


def save_wav(path: str, samples: np.ndarray, sample_rate: int, bit_depth: int = 16) -> None:
    """AudioFile<float>::save (AudioFile.h:842-955); samples (channels, frames) or (frames,)."""
    x = np.ascontiguousarray(np.atleast_2d(samples), np.float32)
    check(lib().arx_wav_save(os.fsencode(path), x.ctypes.data_as(C.POINTER(C.c_float)), x.shape[0], x.shape[1],
                             int(sample_rate), int(bit_depth)))


def normalize_to_range_minus_one_to_one(x: np.ndarray) -> np.ndarray:
    """normalizeToRangeMinusOneToOne (main.cpp:628-651) on a copy; raises on constant input."""
    y = np.array(x, np.float32, copy=True).reshape(-1)
    check(lib().arx_normalize_min_max(y.ctypes.data_as(C.POINTER(C.c_float)), y.size))
    return y


def write_float_lines(path: str, data: np.ndarray) -> None:
    """One value per line in std::ostream's default format (AudioRenderer.cpp:552-556)."""
    x = np.ascontiguousarray(data, np.float32).reshape(-1)
    check(lib().arx_write_float_lines(os.fsencode(path), x.ctypes.data_as(C.POINTER(C.c_float)), x.size))


def read_float_lines(path: str) -> np.ndarray:
    """Reader for the text dumps (what R/utils/*.py plot)."""
    return np.loadtxt(path, dtype=np.float64, ndmin=1).astype(np.float32)


@dataclass
class AppConfig:
    """Context::loadContext's parameters with the reference's defaults (Context.cpp:19-119)."""
    initial_volume: float = 1.0
    ir_length_in_seconds: int = 2
    width: int = 1366
    height: int = 768
    write_first_ir_to_file: bool = False
    write_first_output_to_file: bool = False
    re_render_distance_threshold: float = 3.0
    re_render_angle_threshold: float = 5.0
    mono: bool = False
    scene_file_path: str = "../../assets/models/1D_U.obj"
    audio_file_path: str = ""
    materials_file_path: str = ""
    initial_receiver_pos: tuple = (-2.5, 10.0, 0.0)
    initial_emitter_pos: tuple = (0.0, 0.0, 0.0)
    base_power: float = 100.0
    rays: tuple = (100.0, 100.0, 100.0)
    ray_energy_threshold: float = 0.0
    ray_max_bounces: int = 10
    hrtf_absorption_rate: float = float(np.float32(0.9))
    materials: list = field(default_factory=list)

    @property
    def live(self) -> bool:
        """No audio file -> live mic input at 44100 Hz (Context.cpp:218-222)."""
        return self.audio_file_path == ""

    @classmethod
    def _from_struct(cls, c: ArxAppConfig) -> "AppConfig":
        return cls(
            initial_volume=c.initial_volume, ir_length_in_seconds=c.ir_length_in_seconds, width=c.width,
            height=c.height, write_first_ir_to_file=bool(c.write_first_ir_to_file),
            write_first_output_to_file=bool(c.write_first_output_to_file),
            re_render_distance_threshold=c.re_render_distance_threshold,
            re_render_angle_threshold=c.re_render_angle_threshold, mono=bool(c.mono),
            scene_file_path=c.scene_file_path.decode(), audio_file_path=c.audio_file_path.decode(),
            materials_file_path=c.materials_file_path.decode(),
            initial_receiver_pos=tuple(c.initial_receiver_pos), initial_emitter_pos=tuple(c.initial_emitter_pos),
            base_power=c.base_power, rays=tuple(c.rays), ray_energy_threshold=c.ray_energy_threshold,
            ray_max_bounces=c.ray_max_bounces, hrtf_absorption_rate=c.hrtf_absorption_rate,
            materials=[(c.material_names[i].value.decode(), float(c.material_absorption[i]))
                       for i in range(c.n_materials)],
        )

    def rays_per_dimension(self) -> tuple[int, int, int]:
        """launchParams.size_{x,y,z} = int(rays) (AudioRenderer.cpp:73-75, LaunchParams.h:24)."""
        return tuple(int(r) for r in self.rays)


def parse_config(text: str | bytes) -> AppConfig:
    raw = text.encode() if isinstance(text, str) else text
    c = ArxAppConfig()
    check(lib().arx_parse_app_config(raw, len(raw), C.byref(c)))
    return AppConfig._from_struct(c)


def load_config(path: str) -> AppConfig:
    c = ArxAppConfig()
    check(lib().arx_load_app_config(os.fsencode(path), C.byref(c)))
    return AppConfig._from_struct(c)
