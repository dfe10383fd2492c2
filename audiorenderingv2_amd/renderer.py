"""Python host mirror of the reference's AudioRenderer (R/prebuild/obj_raytracer/AudioRenderer.h:16-152).

Method names follow the reference so callers and tests read like the original:
render(), convoluteAudioFile(), setEmitterPosInOptix(), setSphereCenterInOptix(),
setThresholds(), set_hrtf_absorption_rate(), setBasePower(), setMonoOutput().  Every
call goes through libarx.so's C ABI (include/arx.h); there is no CPU fallback.
"""
from __future__ import annotations

import atexit
import ctypes as C
import dataclasses
import os
import time
import weakref
from dataclasses import dataclass

import numpy as np

from ._lib import ArxConfig, ArxStats, check, fptr, lib
from .formats import write_float_lines
from .scene import Scene

# Every live native object, released at interpreter exit (streams, then buffers, groups and
# renderers), while the HIP and RCCL runtimes are still whole: objects the interpreter would finalize
# only during its own teardown -- or never -- otherwise reach the runtimes' exit-time destructors
# still allocated (a double free inside HIP 7.2's teardown was the result).
_LIVE: "dict[str, weakref.WeakSet]" = {k: weakref.WeakSet() for k in ("stream", "buffer", "group", "renderer")}


@atexit.register
def _release_all() -> None:
    for kind in ("stream", "buffer", "group", "renderer"):
        for obj in list(_LIVE[kind]):
            try:
                obj.close()
            except Exception:
                pass


@dataclass
class RenderSettings:
    rays: tuple = (100, 100, 100)          # pathtracer_parameters.rays (Context.cpp:125-133)
    ir_length_in_seconds: int = 2          # renderer_parameters.ir_length_in_seconds
    sample_rate: int = 44100               # audio file rate (Context.cpp:197-224)
    base_power: float = 100.0
    energy_thres: float = 0.0
    max_bounces: int = 10
    hrtf_absorption_rate: float = 1.0      # round(0.9), Context.cpp:145
    mono: bool = False
    seed: int = 1
    device: int = 0

    def to_c(self) -> ArxConfig:
        c = ArxConfig()
        c.rays_x, c.rays_y, c.rays_z = (int(v) for v in self.rays)
        c.ir_length_in_seconds = int(self.ir_length_in_seconds)
        c.sample_rate = int(self.sample_rate)
        c.base_power = float(self.base_power)
        c.energy_thres = float(self.energy_thres)
        c.max_bounces = int(self.max_bounces)
        c.hrtf_absorption_rate = float(self.hrtf_absorption_rate)
        c.is_mono = 1 if self.mono else 0
        c.seed = int(self.seed)
        c.device = int(self.device)
        return c


class AudioRenderer:
    """AudioRenderer(model, ir_length_in_seconds, sample_rate, materials, rays) (AudioRenderer.h:24)."""

    def __init__(self, settings: RenderSettings, scene: Scene | None = None,
                 receiver: tuple[np.ndarray, np.ndarray] | None = None, _borrowed: C.c_void_p | None = None):
        self.settings = settings
        self._owned = _borrowed is None
        self._h = C.c_void_p()
        if _borrowed is not None:  # a RenderGroup member: the group owns the handle
            self._h = _borrowed
        else:
            cfg = settings.to_c()
            check(lib().arx_create(C.byref(cfg), C.byref(self._h)))
            _LIVE["renderer"].add(self)
        self.ir_length = settings.ir_length_in_seconds * settings.sample_rate
        if receiver is not None:
            self.set_receiver_model(*receiver)
        if scene is not None:
            self.set_scene(scene)

    # -- lifecycle ---------------------------------------------------------------
    def close(self) -> None:
        if self._h and self._owned:
            lib().arx_destroy(self._h)
        self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    @property
    def handle(self) -> C.c_void_p:
        return self._h

    # -- scene -------------------------------------------------------------------
    def set_scene(self, scene: Scene) -> None:
        self._scene_v = np.ascontiguousarray(scene.tri_v, np.float32)
        self._scene_a = np.ascontiguousarray(scene.tri_abs, np.float32)
        check(lib().arx_set_scene(self._h, fptr(self._scene_v), fptr(self._scene_a), scene.n_tris))

    def set_receiver_model(self, left: np.ndarray, right: np.ndarray) -> None:
        for side, t in enumerate((left, right)):
            t = np.ascontiguousarray(t, np.float32).reshape(-1, 9)
            check(lib().arx_set_receiver_model(self._h, side, fptr(t), t.shape[0]))

    def setEmitterPosInOptix(self, pos) -> None:  # AudioRenderer.cpp:752-756
        check(lib().arx_set_emitter(self._h, *(float(v) for v in pos)))

    def setSphereCenterInOptix(self, pos, yaw_deg: float = 0.0) -> None:
        """placeReceiver(...) + setSphereCenterInOptix (AudioRenderer.cpp:758-762)."""
        check(lib().arx_set_listener(self._h, *(float(v) for v in pos), float(yaw_deg)))

    place_listener = setSphereCenterInOptix

    def setThresholds(self, energy: float, max_bounces: int) -> None:
        check(lib().arx_set_thresholds(self._h, float(energy), int(max_bounces)))

    def set_hrtf_absorption_rate(self, rate: float) -> None:
        check(lib().arx_set_hrtf_absorption_rate(self._h, float(rate)))

    def setBasePower(self, p: float) -> None:
        check(lib().arx_set_base_power(self._h, float(p)))

    def setMonoOutput(self, mono: bool) -> None:
        check(lib().arx_set_mono_output(self._h, 1 if mono else 0))

    def normalizeAndMergeStereoOutput(self, left, right, mono_len: int, out) -> None:
        """Declared by the reference with an empty body (AudioRenderer.cpp:574-576): a no-op,
        kept so callers of that API keep working (the live path zips L/R on the device)."""

    def set_frames_in_flight(self, n: int) -> None:
        """1 to 3 (arx_set_frames_in_flight): with n > 1, consecutive render() calls rotate over n
        streams and buffer sets, so a render / convolute loop keeps the GPU full; every getter and
        convolution refers to the last frame started."""
        check(lib().arx_set_frames_in_flight(self._h, int(n)))

    def set_timing(self, on: bool) -> None:
        """arx_set_timing: per-launch timing events (trace_times / conv_times) on or off; a render()
        still times its trace."""
        check(lib().arx_set_timing(self._h, 1 if on else 0))

    def set_seed(self, seed: int) -> None:
        check(lib().arx_set_seed(self._h, int(seed)))

    def set_stream(self, stream_ptr: int | None) -> None:
        """Issue work on this hipStream_t (e.g. torch.cuda.Stream().cuda_stream); 0/None = null stream."""
        check(lib().arx_set_stream(self._h, C.c_void_p(stream_ptr or 0)))

    def get_stream(self) -> int:
        return int(lib().arx_get_stream(self._h) or 0)

    # -- render ------------------------------------------------------------------
    def render(self) -> float:
        """AudioRenderer::render (AudioRenderer.cpp:489-523); returns the trace kernel's ms.
        With the write-IR flag set, dumps the IR once like :525-567 and clears the flag."""
        ms = C.c_double()
        check(lib().arx_render(self._h, C.byref(ms)))
        if self.write_ir_to_file_flag:
            L, R = self.get_ir()
            lp, rp = "output_ir_left.txt", "output_ir_right.txt"
            if self.experimentation:
                stamp = time.time_ns()
                lp = os.path.join("experimentation", f"output_ir_left_{stamp}.txt")
                rp = os.path.join("experimentation", f"output_ir_right_{stamp}.txt")
            write_float_lines(os.path.join(self.output_dir, lp), L)
            write_float_lines(os.path.join(self.output_dir, rp), R)
            self.write_ir_to_file_flag = False
        return ms.value

    # -- text dumps (AudioRenderer.cpp:525-567, 720-744; setters :780-788) -----------
    write_ir_to_file_flag = False
    write_output_to_file_flag = False
    experimentation = False
    output_dir = "."

    def set_write_ir_to_file_flag(self, value: bool) -> None:
        self.write_ir_to_file_flag = bool(value)

    def set_write_output_to_file_flag(self, value: bool) -> None:
        self.write_output_to_file_flag = bool(value)

    def enable_experimentation(self) -> None:
        self.experimentation = True

    def set_trace_path(self, path: int) -> None:
        """Parity hook (arx_debug_set_trace_path): bit 0 forces the f32 nodes, bit 1 the
        global-memory traversal stack; 0 = automatic."""
        check(lib().arx_debug_set_trace_path(self.handle, int(path)))

    def node_images(self) -> dict:
        """Parity hook (arx_debug_node_images): the device's coded f32 nodes (n x 16 words), their
        device-made 16-bit quantized copy (n x 8 words), the grid and the re-quantization count."""
        n = int(self.stats()["n_nodes"])
        cn = np.empty((n, 16), np.uint32)
        qn = np.empty((n, 8), np.uint32)
        grid = np.empty(6, np.float32)
        rq = C.c_uint64()
        check(lib().arx_debug_node_images(self._h, cn.ctypes.data_as(C.c_void_p), qn.ctypes.data_as(C.c_void_p), n,
                                          fptr(grid), C.byref(rq)))
        return {"cnodes": cn, "qnodes": qn, "origin": grid[:3], "scale": grid[3:], "requants": int(rq.value)}

    def clear_histogram(self) -> None:
        check(lib().arx_clear_histogram(self._h))

    def trace_rays(self, ray_begin: int, ray_end: int) -> None:
        check(lib().arx_trace_rays(self._h, int(ray_begin), int(ray_end)))

    def finalize_ir(self) -> None:
        check(lib().arx_finalize_ir(self._h))

    def histogram_device_ptr(self) -> tuple[int, int]:
        p = C.c_void_p()
        n = C.c_size_t()
        check(lib().arx_histogram_device(self._h, C.byref(p), C.byref(n)))
        return int(p.value), int(n.value)

    def attach_histogram(self, d_ptr: int | None, n_elems: int = 0) -> None:
        check(lib().arx_attach_histogram(self._h, C.c_void_p(d_ptr or 0), int(n_elems)))

    def ir_device_ptrs(self) -> tuple[int, int, int]:
        l, r, n = C.c_void_p(), C.c_void_p(), C.c_size_t()
        check(lib().arx_ir_device(self._h, C.byref(l), C.byref(r), C.byref(n)))
        return int(l.value), int(r.value), int(n.value)

    def get_ir(self) -> tuple[np.ndarray, np.ndarray]:
        L = np.empty(self.ir_length, np.float32)
        R = np.empty(self.ir_length, np.float32)
        check(lib().arx_copy_ir(self._h, fptr(L), fptr(R), self.ir_length))
        return L, R

    def set_ir(self, left: np.ndarray, right: np.ndarray) -> None:
        L = np.ascontiguousarray(left, np.float32)
        R = np.ascontiguousarray(right, np.float32)
        check(lib().arx_set_ir(self._h, fptr(L), fptr(R), L.size))

    def trace_times(self, n: int = 64) -> np.ndarray:
        """Device ms of the last min(n, ring) trace launches, oldest first (arx_trace_times)."""
        out = np.zeros(n, np.float64)
        k = C.c_size_t()
        check(lib().arx_trace_times(self._h, out.ctypes.data_as(C.POINTER(C.c_double)), n, C.byref(k)))
        return out[:k.value]

    def conv_times(self, n: int = 64) -> np.ndarray:
        """Device ms of the last min(n, ring) file convolutions, oldest first (arx_conv_times)."""
        out = np.zeros(n, np.float64)
        k = C.c_size_t()
        check(lib().arx_conv_times(self._h, out.ctypes.data_as(C.POINTER(C.c_double)), n, C.byref(k)))
        return out[:k.value]

    def live_times(self, n: int = 64) -> np.ndarray:
        """Device ms of the last min(n, ring) live / streaming convolution blocks (arx_live_times)."""
        out = np.zeros(n, np.float64)
        k = C.c_size_t()
        check(lib().arx_live_times(self._h, out.ctypes.data_as(C.POINTER(C.c_double)), n, C.byref(k)))
        return out[:k.value]

    def stats(self) -> dict:
        s = ArxStats()
        check(lib().arx_get_stats(self._h, C.byref(s)))
        return {k: getattr(s, k) for k, _ in ArxStats._fields_}

    # -- convolution ---------------------------------------------------------------
    def convoluteAudioFile(self, samples: np.ndarray) -> tuple[np.ndarray, np.ndarray, float, float]:
        """AudioRenderer::convoluteAudioFile (AudioRenderer.cpp:663-750): host in, host out."""
        x = np.ascontiguousarray(samples, np.float32)
        L = np.zeros_like(x)
        R = np.zeros_like(x)
        cms, pms = C.c_double(), C.c_double()
        check(lib().arx_convolute_audio_file(self._h, fptr(x), x.nbytes, fptr(L), fptr(R), C.byref(cms),
                                             C.byref(pms)))
        if self.write_output_to_file_flag:
            write_float_lines(os.path.join(self.output_dir, "output_convolute_left.txt"), L)
            write_float_lines(os.path.join(self.output_dir, "output_convolute_right.txt"), R)
            self.write_output_to_file_flag = False
        return L, R, cms.value, pms.value

    def convoluteLiveInput(self, block: np.ndarray, circular_buffer=None) -> np.ndarray:
        """AudioRenderer::convoluteLiveInput (AudioRenderer.cpp:593-661): one f64 mic block ->
        2*ir_len interleaved doubles, added into circular_buffer (CircularBuffer::add) if given."""
        x = np.ascontiguousarray(block, np.float64)
        out = np.empty(2 * self.ir_length, np.float64)
        D = C.POINTER(C.c_double)
        check(lib().arx_convolute_live_block(self._h, x.ctypes.data_as(D), x.nbytes, out.ctypes.data_as(D), out.size))
        if circular_buffer is not None:
            circular_buffer.add(out)
        return out

    def prepare_ir_spectra(self, file: bool = True, live: bool = False) -> None:
        """Recompute the cached IR spectra now (async) rather than in the next convolution."""
        check(lib().arx_prepare_ir_spectra(self._h, (1 if file else 0) | (2 if live else 0)))

    def set_ir_device(self, d_left: int, d_right: int) -> None:
        """Take the IR from device memory (arx_set_ir_device), async on this renderer's stream."""
        check(lib().arx_set_ir_device(self._h, C.c_void_p(d_left), C.c_void_p(d_right), self.ir_length))

    def conv_plan(self, live: bool = False) -> str:
        """The convolution plan in use (arx_conv_describe): direct mixed-radix or power-of-two."""
        buf = C.create_string_buffer(256)
        check(lib().arx_conv_describe(self._h, 2 if live else 1, buf, len(buf)))
        return buf.value.decode()

    def convolute_live_device(self, d_in: int, n_in: int, d_out: int) -> None:
        check(lib().arx_convolute_live_device(self._h, C.c_void_p(d_in), n_in, C.c_void_p(d_out)))

    def convolute_device(self, d_in: int, n_frames: int, d_out_left: int, d_out_right: int) -> None:
        check(lib().arx_convolute_device(self._h, C.c_void_p(d_in), n_frames, C.c_void_p(d_out_left),
                                         C.c_void_p(d_out_right)))

    def convolute_prepare_input(self, d_in: int, n_frames: int) -> None:
        """arx_convolute_prepare_input: the file's blocks transformed once, for convolute_prepared
        (the reference re-convolves the same file with every new IR, AudioRenderer.cpp:790-798)."""
        check(lib().arx_convolute_prepare_input(self._h, C.c_void_p(d_in), n_frames))

    def convolute_prepared(self, d_out_left: int, d_out_right: int) -> int:
        """arx_convolute_prepared: the prepared file convolved with the current IR (bit-identical to
        convolute_device on the same input); returns the frame count."""
        n = C.c_size_t()
        check(lib().arx_convolute_prepared(self._h, C.c_void_p(d_out_left), C.c_void_p(d_out_right), C.byref(n)))
        return int(n.value)


class LiveStream:
    """Streaming convolution of a renderer's IR (arx_stream_*, uniformly partitioned overlap-save
    in f64): process(block) consumes one block of <= block_frames f64 frames and returns
    block_frames output frames zipped L/R -- the linear convolution of the input stream with the
    current IR at the reference live path's scale (ir_len / (ir_len/2)).  The drop-in successor of
    convoluteLiveInput + CircularBuffer (AudioRenderer.cpp:593-661, main.cpp:99-135), whose
    full-length circular result the reference's buffer wraps onto itself."""

    def __init__(self, renderer: AudioRenderer, block_frames: int = 4096):
        self.renderer = renderer
        self._s = C.c_void_p()
        check(lib().arx_stream_create(renderer.handle, int(block_frames), C.byref(self._s)))
        _LIVE["stream"].add(self)
        b, p, n = C.c_int32(), C.c_int32(), C.c_int32()
        check(lib().arx_stream_info(self._s, C.byref(b), C.byref(p), C.byref(n)))
        self.block_frames, self.partitions, self.fft_size = b.value, p.value, n.value

    def process(self, block: np.ndarray) -> np.ndarray:
        x = np.ascontiguousarray(block, np.float64)
        out = np.empty(2 * self.block_frames, np.float64)
        D = C.POINTER(C.c_double)
        check(lib().arx_stream_process(self._s, x.ctypes.data_as(D), x.size, out.ctypes.data_as(D), out.size))
        return out

    def process_device(self, d_in: int, n_frames: int, d_out: int) -> None:
        check(lib().arx_stream_process_device(self._s, C.c_void_p(d_in), int(n_frames), C.c_void_p(d_out)))

    def reset(self) -> None:
        check(lib().arx_stream_reset(self._s))

    def close(self) -> None:
        if self._s:
            lib().arx_stream_destroy(self._s)
            self._s = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class RenderGroup:
    """Ray-sharded multi-GPU rendering through libarx.so's native RCCL groups (arx_group_*).

    RenderGroup(settings, devices=[0, 1, ...]) drives several GPUs from this process
    (ncclCommInitAll); RenderGroup.rank(settings, n_ranks, rank, uid) joins a one-GPU-per-process
    group (ncclCommInitRank) with the id rank 0 got from RenderGroup.unique_id().  render() =
    every shard traced + one int64 all-reduce + the IR finalised on every member; member(i) is
    that member's AudioRenderer (convolution, IR access).  The reference has no equivalent (it
    renders on device 0, AudioRenderer.cpp:252)."""

    def __init__(self, settings: RenderSettings, devices=None, scene: Scene | None = None,
                 receiver: tuple[np.ndarray, np.ndarray] | None = None, _rank=None):
        self.settings = settings
        self._g = C.c_void_p()
        cfg = settings.to_c()
        if _rank is not None:
            n_ranks, rank, uid = _rank
            check(lib().arx_group_create_rank(C.byref(cfg), int(n_ranks), int(rank), uid, len(uid) if uid else 0,
                                              C.byref(self._g)))
        else:
            devs = list(devices if devices is not None else [settings.device])
            arr = (C.c_int32 * len(devs))(*devs)
            check(lib().arx_group_create(C.byref(cfg), arr, len(devs), C.byref(self._g)))
        _LIVE["group"].add(self)
        self.ir_length = settings.ir_length_in_seconds * settings.sample_rate
        self.members = []
        for i in range(lib().arx_group_members(self._g)):
            h = C.c_void_p(lib().arx_group_member(self._g, i))
            cfg = ArxConfig()
            check(lib().arx_get_config(h, C.byref(cfg)))
            self.members.append(AudioRenderer(dataclasses.replace(settings, device=int(cfg.device)), _borrowed=h))
        if receiver is not None:
            self.set_receiver_model(*receiver)
        if scene is not None:
            self.set_scene(scene)

    @staticmethod
    def unique_id() -> bytes:
        buf = C.create_string_buffer(128)
        check(lib().arx_group_unique_id(buf, 128))
        return buf.raw

    @classmethod
    def rank(cls, settings: RenderSettings, n_ranks: int, rank: int, uid: bytes | None, **kw) -> "RenderGroup":
        return cls(settings, _rank=(n_ranks, rank, uid), **kw)

    def close(self) -> None:
        for m in getattr(self, "members", []):
            m._h = C.c_void_p()
        if self._g:
            lib().arx_group_destroy(self._g)
            self._g = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    @property
    def handle(self) -> C.c_void_p:
        return self._g

    def member(self, i: int = 0) -> AudioRenderer:
        return self.members[i]

    @property
    def n_ranks(self) -> int:
        return int(lib().arx_group_ranks(self._g))

    def set_scene(self, scene: Scene) -> None:
        self._scene_v = np.ascontiguousarray(scene.tri_v, np.float32)
        self._scene_a = np.ascontiguousarray(scene.tri_abs, np.float32)
        check(lib().arx_group_set_scene(self._g, fptr(self._scene_v), fptr(self._scene_a), scene.n_tris))

    def set_receiver_model(self, left: np.ndarray, right: np.ndarray) -> None:
        for side, t in enumerate((left, right)):
            t = np.ascontiguousarray(t, np.float32).reshape(-1, 9)
            check(lib().arx_group_set_receiver_model(self._g, side, fptr(t), t.shape[0]))

    def setEmitterPosInOptix(self, pos) -> None:
        check(lib().arx_group_set_emitter(self._g, *(float(v) for v in pos)))

    def setSphereCenterInOptix(self, pos, yaw_deg: float = 0.0) -> None:
        check(lib().arx_group_set_listener(self._g, *(float(v) for v in pos), float(yaw_deg)))

    def setThresholds(self, energy: float, max_bounces: int) -> None:
        check(lib().arx_group_set_thresholds(self._g, float(energy), int(max_bounces)))

    def set_hrtf_absorption_rate(self, rate: float) -> None:
        check(lib().arx_group_set_hrtf_absorption_rate(self._g, float(rate)))

    def setBasePower(self, p: float) -> None:
        check(lib().arx_group_set_base_power(self._g, float(p)))

    def setMonoOutput(self, mono: bool) -> None:
        check(lib().arx_group_set_mono_output(self._g, 1 if mono else 0))

    def set_frames_in_flight(self, n: int) -> None:
        """arx_group_set_frames_in_flight: AudioRenderer.set_frames_in_flight on every member."""
        check(lib().arx_group_set_frames_in_flight(self._g, int(n)))

    def set_timing(self, on: bool) -> None:
        """arx_group_set_timing: AudioRenderer.set_timing on every member."""
        check(lib().arx_group_set_timing(self._g, 1 if on else 0))

    def set_seed(self, seed: int) -> None:
        check(lib().arx_group_set_seed(self._g, int(seed)))

    def render(self, timed: bool = True) -> float:
        """Trace all shards + all-reduce + finalize; returns the longest shard's trace ms (timed)
        or 0.0 without synchronising (timed=False)."""
        ms = C.c_double()
        check(lib().arx_group_render(self._g, C.byref(ms) if timed else None))
        return ms.value

    def synchronize(self) -> None:
        check(lib().arx_group_synchronize(self._g))

    def get_ir(self) -> tuple[np.ndarray, np.ndarray]:
        L = np.empty(self.ir_length, np.float32)
        R = np.empty(self.ir_length, np.float32)
        check(lib().arx_group_copy_ir(self._g, fptr(L), fptr(R), self.ir_length))
        return L, R

    def stats(self) -> dict:
        s = ArxStats()
        check(lib().arx_group_get_stats(self._g, C.byref(s)))
        return {k: getattr(s, k) for k, _ in ArxStats._fields_}

    def allreduce(self, values, op: str = "sum") -> np.ndarray:
        """This process's values combined over every process of the group (one RCCL all-reduce,
        synchronising: also a barrier); a group living in one process returns them unchanged."""
        v = np.ascontiguousarray(np.atleast_1d(values), np.float64).copy()
        check(lib().arx_group_allreduce_f64(self._g, v.ctypes.data_as(C.POINTER(C.c_double)), v.size,
                                            {"sum": 0, "max": 1}[op]))
        return v

    def allreduce_times(self, n: int = 64, member: int = 0) -> np.ndarray:
        """Device ms of member `member`'s last min(n, 256) timed histogram all-reduces, oldest first
        (arx_group_allreduce_times; recorded while the members' timing is on)."""
        out = np.zeros(n, np.float64)
        k = C.c_size_t()
        check(lib().arx_group_allreduce_times(self._g, int(member), out.ctypes.data_as(C.POINTER(C.c_double)), n,
                                              C.byref(k)))
        return out[:k.value]

    def convolute_device(self, d_in, n_frames: int, d_out_left, d_out_right) -> None:
        """Time-block sharded file convolution (arx_group_convolute_device): per local member i, the
        whole file at d_in[i] and full-length outputs d_out_left[i] / d_out_right[i] on its device; rank
        g writes the output frames conv_shard(g) owns."""
        k = len(self.members)
        P = C.c_void_p * k
        check(lib().arx_group_convolute_device(self._g, P(*d_in), int(n_frames), P(*d_out_left), P(*d_out_right)))

    def convoluteAudioFile(self, samples: np.ndarray) -> tuple[np.ndarray, np.ndarray, float, float]:
        """AudioRenderer::convoluteAudioFile over the group (arx_group_convolute_audio_file): host in,
        host out, every GPU of this process convolving its time-block shard; bit-identical to one
        renderer's convoluteAudioFile.  Returns (L, R, convolute_ms, process_ms)."""
        x = np.ascontiguousarray(samples, np.float32)
        L = np.zeros_like(x)
        R = np.zeros_like(x)
        cms, pms = C.c_double(), C.c_double()
        check(lib().arx_group_convolute_audio_file(self._g, fptr(x), x.nbytes, fptr(L), fptr(R), C.byref(cms),
                                                   C.byref(pms)))
        return L, R, cms.value, pms.value

    def conv_shard(self, n_frames: int, rank: int, n_ranks: int | None = None) -> tuple[int, int]:
        """Output frames [begin, end) rank `rank` owns in a sharded convolution (arx_group_conv_shard)."""
        b, e = C.c_uint64(), C.c_uint64()
        lib().arx_group_conv_shard(int(self.settings.sample_rate), int(n_frames), int(rank),
                                   int(self.n_ranks if n_ranks is None else n_ranks), C.byref(b), C.byref(e))
        return int(b.value), int(e.value)

    @property
    def conv_sharded(self) -> bool:
        """Whether the convolution plan shards by time blocks (else every rank convolves the whole file)."""
        v = int(lib().arx_group_conv_sharded(self._g))
        if v < 0:
            check(6)
        return v == 1

    def debug_force_collectives(self, on: bool = True, out_of_place: bool = False) -> None:
        """Tests only (arx_debug_group_force_collectives): every collective issued at one rank too,
        out of place into 0xFF-filled receive buffers if asked."""
        check(lib().arx_debug_group_force_collectives(self._g, 1 if on else 0, 1 if out_of_place else 0))

    def debug_collectives(self) -> dict:
        """Collectives the group has issued (arx_debug_group_collectives)."""
        out = (C.c_uint64 * 3)()
        check(lib().arx_debug_group_collectives(self._g, out))
        return {"histogram_allreduce": int(out[0]), "f64_allreduce": int(out[1]), "scene_broadcast": int(out[2])}


class DeviceBuffer:
    """Device memory allocated through libarx (arx_device_alloc), so that a caller such as
    bench.py needs no other GPU framework (and libarx runs on the HIP runtime it was built with)."""

    def __init__(self, device: int, nbytes: int):
        self.device = int(device)
        self.nbytes = int(nbytes)
        p = C.c_void_p()
        check(lib().arx_device_alloc(self.device, self.nbytes, C.byref(p)))
        self.ptr = int(p.value)
        _LIVE["buffer"].add(self)

    @classmethod
    def from_numpy(cls, device: int, a: np.ndarray) -> "DeviceBuffer":
        a = np.ascontiguousarray(a)
        b = cls(device, a.nbytes)
        check(lib().arx_memcpy(b.device, C.c_void_p(b.ptr), a.ctypes.data_as(C.c_void_p), a.nbytes))
        return b

    def to_numpy(self, dtype, count: int | None = None) -> np.ndarray:
        dt = np.dtype(dtype)
        n = self.nbytes // dt.itemsize if count is None else int(count)
        out = np.empty(n, dt)
        check(lib().arx_memcpy(self.device, out.ctypes.data_as(C.c_void_p), C.c_void_p(self.ptr), out.nbytes))
        return out

    def close(self) -> None:
        if self.ptr:
            lib().arx_device_free(self.device, C.c_void_p(self.ptr))
            self.ptr = 0

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def device_count() -> int:
    """HIP devices visible to this process (arx_device_count)."""
    return int(lib().arx_device_count())


def runtime_info() -> str:
    """Paths and versions of the HIP and RCCL runtimes libarx resolved (arx_runtime_info)."""
    buf = C.create_string_buffer(2048)
    check(lib().arx_runtime_info(buf, len(buf)))
    return buf.value.decode()


def scene_build_count() -> int:
    return int(lib().arx_scene_build_count())


def place_receiver_vertices(local_xyz: np.ndarray, pos, yaw_deg: float) -> np.ndarray:
    """place_receiver_half's transform (OptixModel.cpp:178-193), host-only."""
    v = np.ascontiguousarray(local_xyz, np.float32).reshape(-1, 3)
    out = np.empty_like(v)
    check(lib().arx_place_receiver_vertices(fptr(v), v.shape[0], *(float(p) for p in pos), float(yaw_deg),
                                            fptr(out)))
    return out


def debug_ray_directions(seed: int, first: int, count: int, device: int = 0) -> np.ndarray:
    out = np.empty((count, 3), np.float32)
    check(lib().arx_debug_ray_directions(seed, first, count, fptr(out), device))
    return out


def frac_bits(n_rays: int) -> int:
    return int(lib().arx_frac_bits(n_rays))
