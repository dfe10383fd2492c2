#!/usr/bin/env python3
"""Headline benchmark: ray-bounces/s (+ convolved audio frames/s) on the conference scene.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload c3|c2]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N

One step = one pass of the hot path on every rank (BASELINE.json configs[2], per GPU):
  clear the int64 IR histogram -> trace this rank's 1M-ray shard x 16 bounces (fused HIP
  kernel) -> RCCL all-reduce (SUM int64) of the 2 x 96000-bin histogram -> finalize the
  stereo f32 IR -> IR spectra + file-mode FFT convolution of 807498 frames (48 kHz).
Inputs are resident in HBM before timing.  Rank 0 prints ONE JSON line.
Scaling is weak: every rank owns 1M rays of a W*1M-ray launch (energy normalised by the
total count, devicePrograms.cu:208) and convolves its own 807498-frame stream.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = "ray-bounces/s + convolved audio frames/s on conference.obj at 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec

WORKLOADS = {
    # configs[2]: conference, 1M rays x 16 bounces, 48 kHz IR + convolution (per GPU)
    "c3": dict(rays=(100, 100, 100), max_bounces=16, sample_rate=48000, frames=807498,
               desc="configs[2]: conference stand-in, 1M rays x 16 bounces per GPU, 48 kHz IR (96000 bins/ear), "
                    "file-mode FFT convolution of 807498 frames (A_Clapper_Board length) per GPU"),
    # configs[1]: conference, 100K rays x 8 bounces, 16 kHz
    "c2": dict(rays=(100, 100, 10), max_bounces=8, sample_rate=16000, frames=128000,
               desc="configs[1]: conference stand-in, 100K rays x 8 bounces per GPU, 16 kHz IR, "
                    "convolution of 128000 frames (experimento_entrada_16KHz length) per GPU"),
    # configs[3]: conference, 10M rays x 32 bounces in total, ray-sharded over the ranks (strong)
    "c4": dict(rays=(1000, 100, 100), max_bounces=32, sample_rate=48000, frames=807498, total=True,
               desc="configs[3]: conference stand-in, 10M rays x 32 bounces in total, ray-sharded across the "
                    "ranks, 48 kHz IR, RCCL IR all-reduce; convolution of 807498 frames per GPU"),
}


def bytes_per_bounce(n_tris: int) -> int:
    """SURVEY.md §8d / BASELINE.md: 32 + 32 + 64*ceil(log2 T) + 48."""
    return 32 + 32 + 64 * math.ceil(math.log2(max(n_tris, 2))) + 48


BYTES_PER_STEREO_FRAME = 52  # SURVEY.md §8d (reference algorithm n = 2*sr, hop = sr)


def synthetic_audio(frames: int, sr: int, seed: int = 0) -> np.ndarray:
    rng = np.random.default_rng(seed)
    t = np.arange(frames) / sr
    x = 0.5 * np.sin(2 * np.pi * 440.0 * t) * np.exp(-3.0 * (t % 1.0)) + 0.05 * rng.standard_normal(frames)
    return x.astype(np.float32)


def cpu_baseline(scene, receiver, wl, n_total_rays, budget_s: float) -> dict:
    """The CPU oracle (naive C ray loop + simple BVH) on this host's cores, bounded sample."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import pyoracle as po
    from audiorenderingv2_amd.renderer import place_receiver_vertices
    from audiorenderingv2_amd.scene import CONFERENCE_EMITTER, CONFERENCE_LISTENER

    L, R = receiver
    Lw = place_receiver_vertices(L.reshape(-1, 3), CONFERENCE_LISTENER, 0.0).reshape(-1, 9)
    Rw = place_receiver_vertices(R.reshape(-1, 3), CONFERENCE_LISTENER, 0.0).reshape(-1, 9)
    tv = np.concatenate([scene.tri_v, Lw, Rw])
    ta = np.concatenate([scene.tri_abs, np.full(len(Lw), -1, np.float32), np.full(len(Rw), -2, np.float32)])
    osc = po.Scene(tv, ta, bvh=True)
    p = po.make_params(rays=(n_total_rays, 1, 1), sample_rate=wl["sample_rate"], base_power=3.62,
                       max_bounces=wl["max_bounces"], emitter=CONFERENCE_EMITTER, listener=CONFERENCE_LISTENER)
    threads = max(1, min(16, os.cpu_count() or 1))  # the GPU box's CPU share is 16
    n = 4000
    t0 = time.perf_counter()
    _, _, st = osc.trace(p, 0, n, threads=threads)
    dt = time.perf_counter() - t0
    rate_rays = n / max(dt, 1e-6)
    n2 = int(min(max(rate_rays * budget_s, n), 4_000_000))
    t0 = time.perf_counter()
    _, _, st = osc.trace(p, 0, n2, threads=threads)
    dt = time.perf_counter() - t0
    # convolution leg: f64 oracle FFT block convolution of a bounded slice
    sr = wl["sample_rate"]
    ir = np.zeros(2 * sr, np.float32)
    ir[::97] = 1e-4
    x = synthetic_audio(min(wl["frames"], 8 * sr), sr)
    t1 = time.perf_counter()
    po.convolute_audio(x, sr, ir)
    po.convolute_audio(x, sr, ir)
    dtc = time.perf_counter() - t1
    return {
        "value": st["queries"] / dt, "unit": "ray-bounces/s", "cores": threads, "kind": "port",
        "sample": f"oracle/arx_oracle.c (-O3, median-split BVH, {threads} pthreads): rays 0..{n2} of the same "
                  f"launch ({st['queries']} closest-hit queries, {dt:.1f} s)",
        "convolved_frames_per_s": x.size / (dtc / 2),
        "convolution_sample": f"f64 oracle block convolution, 1 thread, {x.size} frames x 2 ears",
        "cpu_model": _cpu_model(),
    }


def _cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def moving_listener(r, D, dev, stream, hist, ray_begin, ray_end, frames: int) -> dict:
    """the listener moves 0.05 m/frame along +x with yaw += 1 deg/frame.
    Frame latency = host wall time of: receiver re-placement (host transform + sub-tree BVH
    rebuild + upload, no scene rebuild) -> clear -> trace this rank's shard -> RCCL all-reduce
    -> finalize IR -> new IR spectra for the file and live convolution paths, synchronised.
    The reference instead re-places the receiver and rebuilds the whole GAS and pipeline
    (OptixModel.cpp:153-257, AudioRenderer.cpp:466-486, 790-798).  p50/p99 are max over ranks."""
    import torch

    from audiorenderingv2_amd.scene import CONFERENCE_LISTENER

    x0, y0, z0 = CONFERENCE_LISTENER
    lat = []
    for k in range(frames + 3):
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        r.setSphereCenterInOptix((x0 + 0.05 * k, y0, z0), float(k % 360))
        r.clear_histogram()
        r.trace_rays(ray_begin, ray_end)
        D.allreduce_histogram(hist)
        r.finalize_ir()
        r.prepare_ir_spectra(file=True, live=True)
        stream.synchronize()
        if k >= 3:  # first frames warm the receiver rebuild path
            lat.append((time.perf_counter() - t0) * 1e3)
    a = np.array(lat)
    p50 = D.max_over_ranks(float(np.percentile(a, 50)), dev)
    p99 = D.max_over_ranks(float(np.percentile(a, 99)), dev)
    return {"frames": frames, "p50_ms": p50, "p99_ms": p99, "max_ms": D.max_over_ranks(float(a.max()), dev),
            "budget_ms": 1000.0 / 60.0,
            "per_frame": "listener re-place (+0.05 m x, +1 deg yaw) + trace + all-reduce + finalize + IR spectra"}


def load_traffic() -> dict | None:
    path = os.path.join(REPO, "profiles", "trace_traffic.json")
    if os.path.exists(path):
        with open(path) as fh:
            return json.load(fh)
    return None


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="c3")
    ap.add_argument("--cpu-baseline-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--c5-frames", type=int, default=600,
                    help="moving-listener frames after the timed steps (SURVEY C5); 0 disables")
    args = ap.parse_args(argv)

    import torch

    from audiorenderingv2_amd import AudioRenderer, RenderSettings, conference_standin, receiver_local
    from audiorenderingv2_amd import distributed as D
    from audiorenderingv2_amd.scene import CONFERENCE_EMITTER, CONFERENCE_LISTENER

    rank, world, local = D.init()
    if not torch.cuda.is_available():
        raise SystemExit("bench.py needs a GPU (HIP); there is no CPU fallback")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    wl = WORKLOADS[args.workload]
    rx, ry, rz = wl["rays"]
    if wl.get("total"):  # a fixed total split over the ranks (strong scaling)
        total_rays = rx * ry * rz
        rays_per_gpu = total_rays // world
        launch = (rx, ry, rz)
    else:  # a fixed shard per rank (weak scaling)
        rays_per_gpu = rx * ry * rz
        total_rays = rays_per_gpu * world
        launch = (rx * world, ry, rz)
    settings = RenderSettings(rays=launch, ir_length_in_seconds=2, sample_rate=wl["sample_rate"],
                              base_power=3.62, max_bounces=wl["max_bounces"], hrtf_absorption_rate=1.0, seed=1,
                              device=local)
    scene = conference_standin()
    receiver = receiver_local()
    r = AudioRenderer(settings, scene=scene, receiver=receiver)
    r.setEmitterPosInOptix(CONFERENCE_EMITTER)
    r.setSphereCenterInOptix(CONFERENCE_LISTENER, 0.0)
    # one dedicated (non-null) stream for the renderer AND torch/RCCL, so the trace kernel,
    # the all-reduce, the convolution and the timing events are ordered on it
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    r.set_stream(stream.cuda_stream)
    ir_len = r.ir_length
    hist = torch.zeros(2 * ir_len, dtype=torch.int64, device=dev)
    r.attach_histogram(hist.data_ptr(), hist.numel())
    frames = wl["frames"]
    audio = torch.from_numpy(synthetic_audio(frames, wl["sample_rate"], seed=rank)).to(dev)
    out_l = torch.empty_like(audio)
    out_r = torch.empty_like(audio)
    b, e = D.shard_range(total_rays, rank, world)

    ev = [[torch.cuda.Event(enable_timing=True) for _ in range(4)] for _ in range(args.steps)]

    def step(k: int | None):
        if k is not None:
            ev[k][0].record(stream)
        r.clear_histogram()
        r.trace_rays(b, e)
        if k is not None:
            ev[k][1].record(stream)
        D.allreduce_histogram(hist)
        r.finalize_ir()
        if k is not None:
            ev[k][2].record(stream)
        r.convolute_device(audio.data_ptr(), frames, out_l.data_ptr(), out_r.data_ptr())
        if k is not None:
            ev[k][3].record(stream)

    for _ in range(args.warmup):
        step(None)
    torch.cuda.synchronize(dev)
    stats = r.stats()  # also raises if the kernel flagged a stack overflow
    D.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(k)
    torch.cuda.synchronize(dev)
    D.barrier()
    t1 = time.perf_counter()
    elapsed = D.max_over_ranks(t1 - t0, dev)
    stats = r.stats()
    q_rank = int(stats["queries"])  # per step (counters cleared every step)
    q_all = D.sum_over_ranks(q_rank, dev)
    trace_ms = float(np.mean([ev[k][0].elapsed_time(ev[k][1]) for k in range(args.steps)]))
    reduce_ms = float(np.mean([ev[k][1].elapsed_time(ev[k][2]) for k in range(args.steps)]))
    conv_ms = float(np.mean([ev[k][2].elapsed_time(ev[k][3]) for k in range(args.steps)]))
    trace_ms_max = D.max_over_ranks(trace_ms, dev)
    conv_ms_max = D.max_over_ranks(conv_ms, dev)

    value = q_all * args.steps / elapsed
    n_tris = int(stats["n_scene_tris"] + stats["n_receiver_tris"])
    moving = moving_listener(r, D, dev, stream, hist, b, e, args.c5_frames) if args.c5_frames > 0 else None
    bpb = bytes_per_bounce(n_tris)
    achieved = q_rank * bpb / (trace_ms * 1e-3) / 1e9
    traffic = load_traffic()
    conv_frames_s = world * frames / (conv_ms_max * 1e-3)
    result = {
        "metric": METRIC,
        "value": value,
        "unit": "ray-bounces/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "strong" if wl.get("total") else "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic: deterministic conference.obj stand-in (seed 42; conference.obj is missing from the "
                "reference checkout) + synthetic 48 kHz audio",
        "config": {
            "workload": wl["desc"],
            "scene_triangles": n_tris,
            "rays_per_gpu": rays_per_gpu,
            "max_bounces": wl["max_bounces"],
            "sample_rate": wl["sample_rate"],
            "ir_len": ir_len,
            "audio_frames_per_gpu": frames,
            "parallelism": f"ray-shard x{world}, RCCL int64 IR all-reduce" if world > 1 else "1 GPU",
        },
        "ray_bounces_per_step": q_all,
        "nominal_ray_bounces_per_s": total_rays * wl["max_bounces"] * args.steps / elapsed,
        "receiver_hits_per_step_rank0": int(stats["receiver_hits"]),
        "convolved_frames_per_s": conv_frames_s,
        "phases_ms_rank0": {"trace": trace_ms, "allreduce_finalize": reduce_ms, "ir_spectra_and_convolution": conv_ms},
        "roofline": {
            "kernel": "trace_kernel",
            "bound": "hbm",
            "achieved": achieved,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS,
            "traffic": (traffic or {}).get("bytes_per_launch") if traffic and traffic.get("workload") == args.workload
            else None,
            "algorithmic_bytes_per_bounce": bpb,
        },
        "roofline_convolution": {
            "bound": "hbm",
            "achieved": frames * BYTES_PER_STEREO_FRAME / (conv_ms * 1e-3) / 1e9,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": frames * BYTES_PER_STEREO_FRAME / (conv_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
            "algorithmic_bytes_per_stereo_frame": BYTES_PER_STEREO_FRAME,
        },
    }
    if moving is not None:
        result["moving_listener"] = moving
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(scene, receiver, wl, total_rays, args.cpu_baseline_seconds)
    if rank == 0:
        print(json.dumps(result), flush=True)
    r.close()
    if world > 1:
        import torch.distributed as dist

        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
