"""Headless counterpart of the reference app's driver (R/prebuild/obj_raytracer/main.cpp + Context.cpp).

    python -m audiorenderingv2_amd.app <config.json> export [Result.wav]
    python -m audiorenderingv2_amd.app <config.json> experiment [rounds]

Context          -- Context::loadContext (Context.cpp:15-236): config -> scene, receiver halves,
                    audio file, renderer (paths are relative to the working directory, as in the
                    reference, whose receivers live at ../../assets/models/{left,right}Half.obj)
export_audio     -- main.cpp:653-718: render, convolve channel 0, min-max normalise, save WAV
experimentation  -- main.cpp:531-626: N rounds of render + convolution, avg / median times
ListenerTracker  -- the re-render trigger of the interactive loop (main.cpp:440-498)

The interactive "main" mode (GLFW window + RtAudio devices) is not part of this hot-path
framework; the RtAudio callbacks themselves are in live.py / include/arx_rtaudio.hpp.
"""
from __future__ import annotations

import argparse
import math
import os
import statistics
import sys
import time
from dataclasses import dataclass

import numpy as np

from .formats import AppConfig, load_config, load_receiver_half, load_scene, load_wav, \
    normalize_to_range_minus_one_to_one, save_wav
from .renderer import AudioRenderer, RenderSettings

LIVE_SAMPLE_RATE = 44100  # main.cpp:36 / Context.cpp:220


def global_angle(orientation) -> float:
    """Camera::calculate_global_angle (Camera.cpp:31-41): degrees(atan2(z, x)) in [0, 360)."""
    a = float(np.float32(math.degrees(math.atan2(float(orientation[2]), float(orientation[0])))))
    return a + 360.0 if a < 0 else a


@dataclass
class Context:
    config: AppConfig
    renderer: AudioRenderer
    audio: object | None          # formats.Wav or None in live mode
    sample_rate: int
    camera_position: tuple
    camera_angle: float = 0.0     # Camera::globalAngle starts at 0 (Camera.h:33)

    @classmethod
    def load(cls, config: AppConfig | str, cwd: str | None = None, receiver_dir: str | None = None,
             seed: int = 1, device: int = 0) -> "Context":
        cfg = load_config(config) if isinstance(config, str) else config
        base = cwd or os.getcwd()

        def resolve(p: str) -> str:
            return p if os.path.isabs(p) else os.path.join(base, p)

        rdir = receiver_dir or resolve(os.path.join("..", "..", "assets", "models"))
        left = load_receiver_half(os.path.join(rdir, "leftHalf.obj"), 0)
        right = load_receiver_half(os.path.join(rdir, "rightHalf.obj"), 1)
        scene = load_scene(resolve(cfg.scene_file_path), cfg.materials)
        audio = None
        sr = LIVE_SAMPLE_RATE
        if cfg.audio_file_path:
            audio = load_wav(resolve(cfg.audio_file_path))
            sr = audio.sample_rate
        settings = RenderSettings(rays=cfg.rays_per_dimension(), ir_length_in_seconds=cfg.ir_length_in_seconds,
                                  sample_rate=sr, base_power=cfg.base_power, energy_thres=cfg.ray_energy_threshold,
                                  max_bounces=cfg.ray_max_bounces, hrtf_absorption_rate=cfg.hrtf_absorption_rate,
                                  mono=cfg.mono, seed=seed, device=device)
        r = AudioRenderer(settings, scene, (left.triangles(), right.triangles()))
        r.set_write_ir_to_file_flag(cfg.write_first_ir_to_file)        # Context.cpp:229-230
        r.set_write_output_to_file_flag(cfg.write_first_output_to_file)
        return cls(cfg, r, audio, sr, tuple(cfg.initial_receiver_pos))

    def prepare(self) -> None:
        """The setter sequence of export_audio / experimentation_mode (main.cpp:541-552, 665-676)."""
        r, c = self.renderer, self.config
        r.setSphereCenterInOptix(self.camera_position, self.camera_angle)   # placeReceiver + center
        r.setMonoOutput(c.mono)
        r.setBasePower(c.base_power)
        r.setThresholds(c.ray_energy_threshold, c.ray_max_bounces)
        r.setEmitterPosInOptix(c.initial_emitter_pos)


def export_audio(ctx: Context, export_path: str = "Result.wav") -> tuple[np.ndarray, np.ndarray]:
    """export_audio (main.cpp:653-718)."""
    if ctx.audio is None:
        raise ValueError("export mode needs scene_parameters.audio_file_path")
    ctx.prepare()
    r = ctx.renderer
    r.set_write_ir_to_file_flag(False)
    r.set_write_output_to_file_flag(False)
    r.render()
    L, R, _, _ = r.convoluteAudioFile(ctx.audio.samples[0])
    L = normalize_to_range_minus_one_to_one(L)
    R = normalize_to_range_minus_one_to_one(R)
    save_wav(export_path, np.stack([L, R]), ctx.audio.sample_rate, ctx.audio.bit_depth)
    return L, R


def experimentation(ctx: Context, rounds: int = 100, log=print) -> dict:
    """experimentation_mode (main.cpp:531-626): per-round render / convolution times."""
    if ctx.audio is None:
        raise ValueError("experiment mode needs scene_parameters.audio_file_path")
    ctx.prepare()
    r = ctx.renderer
    r.enable_experimentation()
    render_ms, conv_ms, proc_ms = [], [], []
    for k in range(rounds):
        t0 = time.perf_counter()
        r.set_write_ir_to_file_flag(False)
        render_ms.append(r.render())
        r.set_write_output_to_file_flag(False)
        _, _, c, p = r.convoluteAudioFile(ctx.audio.samples[0])
        conv_ms.append(c)
        proc_ms.append(p)
        log(f"Round {k}: took {(time.perf_counter() - t0) * 1e3:.3f} ms")
    out = {}
    for name, v in (("render", render_ms), ("convolute", conv_ms), ("convolute process", proc_ms)):
        out[name] = {"average_ms": sum(v) / len(v), "median_ms": statistics.median(v)}
        log(f"\tAverage {name} time: {out[name]['average_ms']} ms")
        log(f"\tMedian {name} time: {out[name]['median_ms']} ms")
    return out


class ListenerTracker:
    """Re-render trigger of the interactive loop (main.cpp:440-498): moved farther than
    re_render_distance_threshold, turned more than re_render_angle_threshold (wrapped at 180),
    or moved at all more than one second ago.  `now` is injectable for tests."""

    def __init__(self, cfg: AppConfig, position, now=time.time):
        self.dist_thr = float(cfg.re_render_distance_threshold)
        self.ang_thr = float(cfg.re_render_angle_threshold)
        self.last_position = np.asarray(position, np.float32)
        self.last_angle = 0.0  # main.cpp:444
        self.now = now
        self.timer_set = False
        self.last_time = int(now())

    def update(self, position, angle: float, is_rendering: bool = False) -> bool:
        p = np.asarray(position, np.float32)
        # distanceP2P (Utils.cpp:29-32): f32 differences, std::pow -> f64 squares, f32 result
        diff3 = (p - self.last_position).astype(np.float64)
        d = float(np.float32(math.sqrt(diff3[0] ** 2 + diff3[1] ** 2 + diff3[2] ** 2)))
        if d > 0 and not self.timer_set:
            self.last_time = int(self.now())
            self.timer_set = True
        dist_trigger = d > self.dist_thr
        turn = abs(self.last_angle - angle)
        if turn > 180.0:
            turn = 360.0 - turn
        ang_trigger = turn > self.ang_thr
        time_trigger = self.timer_set and (int(self.now()) - self.last_time) > 1
        if (dist_trigger or ang_trigger or time_trigger) and not is_rendering:
            self.timer_set = False
            self.last_angle = float(angle)
            self.last_position = p
            return True
        return False


def main(argv: list[str] | None = None) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("config")
    ap.add_argument("mode", nargs="?", default="main")
    ap.add_argument("arg", nargs="?")
    ap.add_argument("--receiver-dir")
    ap.add_argument("--seed", type=int, default=1)
    a = ap.parse_args(argv)
    try:
        if a.mode == "main":
            raise SystemExit("interactive mode (GLFW window + RtAudio devices) is not provided; "
                             "use `export` or `experiment`")
        ctx = Context.load(a.config, receiver_dir=a.receiver_dir, seed=a.seed)
        if a.mode == "export":
            export_audio(ctx, a.arg or "Result.wav")
        else:
            experimentation(ctx, int(a.arg or 100))
    except (OSError, ValueError, RuntimeError) as e:
        print(f"Exception caught: {e}", file=sys.stderr)
        return 1
    return 0


if __name__ == "__main__":
    sys.exit(main())
