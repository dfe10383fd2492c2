"""ctypes front-end of the CPU oracle (oracle/liboracle.so) -- TEST INFRASTRUCTURE.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this
module, and only as the checker.  See arx_oracle.h for what it restates.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")


class OrcParams(C.Structure):
    _fields_ = [
        ("rays_x", C.c_int32), ("rays_y", C.c_int32), ("rays_z", C.c_int32),
        ("ir_length", C.c_int32), ("sample_rate", C.c_int32),
        ("base_power", C.c_float), ("energy_thres", C.c_float), ("max_bounces", C.c_uint32),
        ("hrtf_absorption_rate", C.c_float), ("is_mono", C.c_int32), ("seed", C.c_uint64),
        ("emitter", C.c_float * 3), ("sphere_center", C.c_float * 3), ("arith", C.c_int32),
    ]


class OrcScene(C.Structure):
    _fields_ = [("tri_v", C.POINTER(C.c_float)), ("tri_abs", C.POINTER(C.c_float)),
                ("n_tris", C.c_int64), ("bvh", C.c_void_p)]


class OrcStats(C.Structure):
    _fields_ = [("queries", C.c_uint64), ("receiver_hits", C.c_uint64), ("misses", C.c_uint64)]


class OrcRayRecord(C.Structure):
    _fields_ = [("energy", C.c_float), ("distance", C.c_float), ("depth", C.c_int32), ("bin", C.c_int32),
                ("queries", C.c_int32), ("last_tri", C.c_int32), ("path_hash", C.c_uint32)]


_lib = None


class OrcStream(C.Structure):
    _fields_ = [("block", C.c_int32), ("N", C.c_int32), ("P", C.c_int32), ("ir_len", C.c_int32),
                ("blocks", C.c_int64), ("hist", C.c_void_p), ("X", C.c_void_p), ("G", C.c_void_p)]


def use_library(path: str) -> None:
    """Load this build of the oracle instead of liboracle.so (bench.py's -march=native CPU baseline);
    must precede the first call into the oracle."""
    global LIB_PATH
    if _lib is not None:
        raise RuntimeError("the oracle library is already loaded")
    LIB_PATH = path


def build() -> str:
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        if LIB_PATH == os.path.join(HERE, "liboracle.so") and (not os.path.exists(LIB_PATH) or (
                os.path.getmtime(LIB_PATH) < os.path.getmtime(os.path.join(HERE, "arx_oracle.c")))):
            build()
        L = C.CDLL(LIB_PATH)
        F = C.POINTER(C.c_float)
        I64 = C.POINTER(C.c_int64)
        L.orc_philox4x32_10.argtypes = [C.POINTER(C.c_uint32), C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]
        L.orc_ray_direction.argtypes = [C.c_uint64, C.c_uint64, F]
        L.orc_ray_direction_reference.argtypes = [C.c_uint64, C.c_uint64, F]
        L.orc_initial_energy.argtypes = [C.POINTER(OrcParams)]
        L.orc_initial_energy.restype = C.c_float
        L.orc_frac_bits.argtypes = [C.c_uint64]
        L.orc_frac_bits.restype = C.c_int
        L.orc_closest_hit.argtypes = [C.POINTER(OrcScene), F, F, F]
        L.orc_closest_hit.restype = C.c_int64
        L.orc_build_bvh.argtypes = [C.POINTER(OrcScene)]
        L.orc_free_bvh.argtypes = [C.POINTER(OrcScene)]
        L.orc_trace.argtypes = [C.POINTER(OrcScene), C.POINTER(OrcParams), C.c_uint64, C.c_uint64, I64, I64,
                                C.POINTER(OrcStats), C.c_int]
        L.orc_trace_records.argtypes = [C.POINTER(OrcScene), C.POINTER(OrcParams), C.c_uint64, C.c_uint64,
                                        C.POINTER(OrcRayRecord)]
        L.orc_finalize_ir.argtypes = [C.POINTER(OrcParams), I64, I64, F, F]
        L.orc_convolute_audio.argtypes = [F, C.c_int64, C.c_int32, F, C.c_int32, F]
        L.orc_fft.argtypes = [C.POINTER(C.c_double), C.c_int64, C.c_int]
        L.orc_fft.restype = C.c_int
        L.orc_convolute_live_block.argtypes = [C.POINTER(C.c_double), C.c_int64, F, F, C.c_int32,
                                               C.POINTER(C.c_double)]
        L.orc_stream_init.argtypes = [C.POINTER(OrcStream), C.c_int32, F, F, C.c_int32]
        L.orc_stream_init.restype = C.c_int
        L.orc_stream_process.argtypes = [C.POINTER(OrcStream), C.POINTER(C.c_double), C.c_int64,
                                         C.POINTER(C.c_double)]
        L.orc_stream_free.argtypes = [C.POINTER(OrcStream)]
        _lib = L
    return _lib


def _f(a):
    return a.ctypes.data_as(C.POINTER(C.c_float))


def philox(ctr, key):
    c = (C.c_uint32 * 4)(*ctr)
    k = (C.c_uint32 * 2)(*key)
    o = (C.c_uint32 * 4)()
    lib().orc_philox4x32_10(c, k, o)
    return [int(x) for x in o]


def ray_directions(seed: int, first: int, count: int, reference_formula: bool = False) -> np.ndarray:
    fn = lib().orc_ray_direction_reference if reference_formula else lib().orc_ray_direction
    out = np.empty((count, 3), np.float32)
    row = (C.c_float * 3)()
    for i in range(count):
        fn(seed, first + i, row)
        out[i] = row[:]
    return out


def frac_bits(n: int) -> int:
    return int(lib().orc_frac_bits(n))


def make_params(*, rays=(32, 32, 1), sample_rate=16000, ir_seconds=2, base_power=3.62, energy_thres=0.0,
                max_bounces=2, hrtf=1.0, mono=False, seed=1, emitter=(0.0, 0.0, 0.0),
                listener=(2.5, 9.9, 0.0), arith: int = 0) -> OrcParams:
    p = OrcParams()
    p.rays_x, p.rays_y, p.rays_z = rays
    p.sample_rate = sample_rate
    p.ir_length = ir_seconds * sample_rate
    p.base_power = base_power
    p.energy_thres = energy_thres
    p.max_bounces = max_bounces
    p.hrtf_absorption_rate = hrtf
    p.is_mono = 1 if mono else 0
    p.seed = seed
    p.arith = int(arith)
    p.emitter[:] = list(emitter)
    p.sphere_center[:] = list(listener)
    return p


class Scene:
    """Flat triangle soup (T,9) f32 + absorption (T,) f32; global id = row."""

    def __init__(self, tri_v: np.ndarray, tri_abs: np.ndarray, bvh: bool = False):
        self.tri_v = np.ascontiguousarray(tri_v, dtype=np.float32).reshape(-1, 9)
        self.tri_abs = np.ascontiguousarray(tri_abs, dtype=np.float32).reshape(-1)
        assert self.tri_v.shape[0] == self.tri_abs.shape[0]
        self.s = OrcScene(_f(self.tri_v), _f(self.tri_abs), self.tri_v.shape[0], None)
        if bvh:
            lib().orc_build_bvh(C.byref(self.s))

    def __del__(self):
        try:
            lib().orc_free_bvh(C.byref(self.s))
        except Exception:
            pass

    def closest_hit(self, o, d):
        t = C.c_float()
        oo = (C.c_float * 3)(*o)
        dd = (C.c_float * 3)(*d)
        i = lib().orc_closest_hit(C.byref(self.s), oo, dd, C.byref(t))
        return int(i), float(t.value)

    def trace(self, p: OrcParams, ray_begin: int = 0, ray_end: int | None = None, threads: int = 1):
        n = p.rays_x * p.rays_y * p.rays_z
        if ray_end is None:
            ray_end = n
        L = np.zeros(p.ir_length, np.int64)
        R = np.zeros(p.ir_length, np.int64)
        st = OrcStats()
        I64 = C.POINTER(C.c_int64)
        lib().orc_trace(C.byref(self.s), C.byref(p), ray_begin, ray_end, L.ctypes.data_as(I64),
                        R.ctypes.data_as(I64), C.byref(st), threads)
        return L, R, {"queries": st.queries, "receiver_hits": st.receiver_hits, "misses": st.misses}

    def float_sums(self, p: OrcParams, ray_begin: int, ray_end: int):
        """orc_trace_float_sums: (int64 L, R), (f64 L, R), (f32 L, R), stats of the same rays."""
        n = p.ir_length
        L, R = np.zeros(n, np.int64), np.zeros(n, np.int64)
        dL, dR = np.zeros(n, np.float64), np.zeros(n, np.float64)
        fL, fR = np.zeros(n, np.float32), np.zeros(n, np.float32)
        st = OrcStats()
        I64, D, F = C.POINTER(C.c_int64), C.POINTER(C.c_double), C.POINTER(C.c_float)
        lib().orc_trace_float_sums(C.byref(self.s), C.byref(p), ray_begin, ray_end, L.ctypes.data_as(I64),
                                   R.ctypes.data_as(I64), dL.ctypes.data_as(D), dR.ctypes.data_as(D),
                                   fL.ctypes.data_as(F), fR.ctypes.data_as(F), C.byref(st))
        return (L, R), (dL, dR), (fL, fR), {"queries": st.queries, "receiver_hits": st.receiver_hits,
                                             "misses": st.misses}

    def records(self, p: OrcParams, first: int, count: int) -> np.ndarray:
        rec = (OrcRayRecord * count)()
        lib().orc_trace_records(C.byref(self.s), C.byref(p), first, count, rec)
        return np.array([(r.energy, r.distance, r.depth, r.bin, r.queries, r.last_tri, r.path_hash) for r in rec],
                        dtype=[("energy", np.float32), ("distance", np.float32), ("depth", np.int32),
                               ("bin", np.int32), ("queries", np.int32), ("last_tri", np.int32),
                               ("path_hash", np.uint32)])


def finalize_ir(p: OrcParams, L: np.ndarray, R: np.ndarray):
    I64 = C.POINTER(C.c_int64)
    irl = np.zeros(p.ir_length, np.float32)
    irr = np.zeros(p.ir_length, np.float32)
    lib().orc_finalize_ir(C.byref(p), np.ascontiguousarray(L, np.int64).ctypes.data_as(I64),
                          np.ascontiguousarray(R, np.int64).ctypes.data_as(I64), _f(irl), _f(irr))
    return irl, irr


def convolute_audio(x: np.ndarray, sample_rate: int, ir: np.ndarray) -> np.ndarray:
    x = np.ascontiguousarray(x, np.float32)
    ir = np.ascontiguousarray(ir, np.float32)
    out = np.zeros_like(x)
    lib().orc_convolute_audio(_f(x), x.size, sample_rate, _f(ir), ir.size, _f(out))
    return out


def fft(x: np.ndarray, sign: int = -1) -> np.ndarray:
    buf = np.ascontiguousarray(np.asarray(x, np.complex128)).copy()
    lib().orc_fft(buf.ctypes.data_as(C.POINTER(C.c_double)), buf.size, sign)
    return buf


def convolute_live_block(x: np.ndarray, ir_left: np.ndarray, ir_right: np.ndarray) -> np.ndarray:
    x = np.ascontiguousarray(x, np.float64)
    n = ir_left.size
    out = np.zeros(2 * n, np.float64)
    lib().orc_convolute_live_block(x.ctypes.data_as(C.POINTER(C.c_double)), x.size,
                                   _f(np.ascontiguousarray(ir_left, np.float32)),
                                   _f(np.ascontiguousarray(ir_right, np.float32)), n,
                                   out.ctypes.data_as(C.POINTER(C.c_double)))
    return out


class Stream:
    """orc_stream_*: the streaming convolution (uniformly partitioned overlap-save) restated."""

    def __init__(self, block: int, ir_left: np.ndarray, ir_right: np.ndarray):
        self._s = OrcStream()
        self._l = np.ascontiguousarray(ir_left, np.float32)
        self._r = np.ascontiguousarray(ir_right, np.float32)
        if lib().orc_stream_init(C.byref(self._s), int(block), _f(self._l), _f(self._r), self._l.size) != 0:
            raise RuntimeError("orc_stream_init failed")
        self.block = int(block)

    def process(self, x: np.ndarray) -> np.ndarray:
        x = np.ascontiguousarray(x, np.float64)
        out = np.zeros(2 * self.block, np.float64)
        lib().orc_stream_process(C.byref(self._s), x.ctypes.data_as(C.POINTER(C.c_double)), x.size,
                                 out.ctypes.data_as(C.POINTER(C.c_double)))
        return out

    def __del__(self):
        try:
            lib().orc_stream_free(C.byref(self._s))
        except Exception:
            pass
