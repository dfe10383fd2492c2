#!/usr/bin/env python3
"""Headline benchmark: ray-bounces/s (+ convolved audio frames/s) on the conference scene.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload c3|c2|c4]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N

One step = one pass of the hot path on every GPU (BASELINE.json configs[2], per GPU):
  trace this GPU's 1M-ray shard x 16 bounces (fused HIP kernel) -> one RCCL all-reduce (int64
  SUM) of the 2 x 96000-bin histogram -> finalize the stereo f32 IR (libarx's native group API,
  arx_group_render) -> IR spectra + file-mode FFT convolution of A_Clapper_Board.wav channel 0
  (807 498 frames, 48 kHz), time-block sharded over the GPUs (arx_group_convolute_device: each GPU
  convolves its share of the file's one-second block pairs; the union is the one-GPU output bit for
  bit, no collective).

How the N GPUs are driven (plan_ranks):
  * plain `python bench.py --gpus N`: ONE process drives N GPUs through one native group
    (arx_group_create over devices 0..N-1 -> ncclCommInitAll), the design of SURVEY.md §5 / §8e;
  * under torch.distributed.run (WORLD_SIZE = N > 1): one GPU per process (LOCAL_RANK), joined
    with ncclCommInitRank; rank 0's RCCL unique id reaches the other ranks through a file keyed by
    the launcher's process id and port (all ranks share one node), and barriers / max-over-ranks
    timing are RCCL all-reduces of the group itself (arx_group_allreduce_f64).
The process imports no other GPU framework: device buffers, streams and timing events come from
libarx (arx_device_alloc, the renderer's own stream and per-launch event rings), so libarx runs on
the /opt/rocm HIP / RCCL runtime it was built and tested against (`runtime` in the JSON line).
Asking for more GPUs than the box has fails loudly instead of printing a smaller line.
Inputs are resident in HBM before timing.  Rank 0 prints ONE JSON line.
Scaling is weak for the rays: every GPU owns 1M rays of an N*1M-ray launch (energy normalised by
the total count, devicePrograms.cu:208); the file's convolution is shared (strong) and counted once.
A watchdog ends a run whose steps stop completing with one {"status": "hang", ...} line (exit 3).
"""
from __future__ import annotations

import argparse
import contextlib
import hashlib
import json
import math
import os
import subprocess
import sys
import tempfile
import threading
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = "ray-bounces/s + convolved audio frames/s on conference.obj at 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec

WORKLOADS = {
    # configs[2]: conference, 1M rays x 16 bounces, 48 kHz IR + convolution (per GPU)
    # fif: frames in flight on one GPU.  C3 with 2: two half-grid launches side by side, +8 % (round 6,
    # profiles/r06/grid_ab_*.txt; +3 % on the full grid before); C2, whose single frame fills 1.5 waves
    # per SIMD, +62 % with 2 and +112 % with 3; the 46 ms C4 launch loses 7-13 % with 2
    # (profiles/r06/grid_ab_c4.txt; 5 % on the full grid, profiles/r04/bench_c4_r04m.json)
    "c3": dict(rays=(100, 100, 100), max_bounces=16, sample_rate=48000, audio="clapper", fif=2,
               desc="configs[2]: conference stand-in, 1M rays x 16 bounces per GPU, 48 kHz IR (96000 bins/ear), "
                    "file-mode FFT convolution of A_Clapper_Board.wav ch0 (807498 frames) per GPU"),
    # configs[1]: conference, 100K rays x 8 bounces, 16 kHz
    "c2": dict(rays=(100, 100, 10), max_bounces=8, sample_rate=16000, audio="experimento", fif=3,
               desc="configs[1]: conference stand-in, 100K rays x 8 bounces per GPU, 16 kHz IR, "
                    "convolution of experimento_entrada_16KHz.wav (128000 frames) per GPU"),
    # configs[3]: conference, 10M rays x 32 bounces in total, ray-sharded over the GPUs (strong)
    "c4": dict(rays=(1000, 100, 100), max_bounces=32, sample_rate=48000, audio="clapper", total=True, fif=1,
               desc="configs[3]: conference stand-in, 10M rays x 32 bounces in total, ray-sharded across the "
                    "GPUs, 48 kHz IR, RCCL IR all-reduce; convolution of A_Clapper_Board.wav ch0 per GPU"),
}


def bytes_per_bounce(n_tris: int) -> int:
    """SURVEY.md §8d / BASELINE.md: 32 + 32 + 64*ceil(log2 T) + 48."""
    return 32 + 32 + 64 * math.ceil(math.log2(max(n_tris, 2))) + 48


BYTES_PER_STEREO_FRAME = 52  # SURVEY.md §8d (reference algorithm n = 2*sr, hop = sr)
NODE_FORMATS = {0: "f32 BVH2", 1: "16-bit quantized BVH2", 2: "4-wide compressed (CW4)"}  # arx_stats.trace_format
PROFILES = "r06"  # profiles/<round>/: the guarded PMC-derived profiles of the current kernel and tree
# the C3 file convolution's PMC traffic (tools/gpu_conv_pmc.sh), guarded by arx_conv_kernel_id
CONV_TRAFFIC = "r06/conv_traffic.json"
# the GPU box's full-launch parity record of C3 (tests/test_gpu_full_launch.py with ARX_PARITY_RECORD),
# guarded by tree hash and trace kernel identity
FULL_LAUNCH_PARITY = "r06/full_launch_parity/c3_whole_launch.json"
HBM_ACHIEVABLE_GBS = 6300.0  # MI355X_MICROARCH.md: measured-achievable HBM read bandwidth


# ----------------------------------------------------------------------------- rank plumbing ---
def plan_ranks(gpus: int, env: dict, process_group: bool = False, oversubscribe: bool = False) -> dict:
    """--gpus N and the launcher's environment -> how this process takes part.

    mode "local": this process drives devices 0..N-1 itself (one native group, ncclCommInitAll);
    mode "rank": torch.distributed.run started one process per GPU (WORLD_SIZE > 1, or
    --process-group at one rank): this process is rank RANK of WORLD_SIZE on device LOCAL_RANK
    (ncclCommInitRank).  `world` is the GPU count of the whole job either way.  oversubscribe (tests
    only): mode "local" with device 0 listed N times -- the N-rank job's shards, sharded convolution
    and bookkeeping on one GPU (its histograms summed on the device, no RCCL)."""
    if gpus < 1:
        raise ValueError(f"--gpus must be >= 1 (got {gpus})")
    world = int(env.get("WORLD_SIZE", "1"))
    if world > 1 or process_group:
        if gpus not in (1, world) or (world == 1 and gpus != 1):
            raise ValueError(f"--gpus {gpus} but the launcher started WORLD_SIZE={world} processes "
                             "(one GPU per process: pass --gpus WORLD_SIZE)")
        rank, local = int(env.get("RANK", "0")), int(env.get("LOCAL_RANK", "0"))
        if not (0 <= rank < world) or local < 0:
            raise ValueError(f"bad RANK={rank} / LOCAL_RANK={local} for WORLD_SIZE={world}")
        return {"mode": "rank", "world": world, "rank": rank, "devices": [local], "local_gpus_needed": local + 1}
    if oversubscribe:
        return {"mode": "local", "world": gpus, "rank": 0, "devices": [0] * gpus, "local_gpus_needed": 1}
    return {"mode": "local", "world": gpus, "rank": 0, "devices": list(range(gpus)), "local_gpus_needed": gpus}


def uid_path(env: dict) -> str:
    """Where rank 0 leaves the RCCL unique id for the other ranks of this launch: keyed by the
    launcher (the ranks' common parent process), its rendezvous port and run id, so a file left by
    another launch is never read."""
    key = f"{os.getppid()}:{env.get('MASTER_ADDR', '')}:{env.get('MASTER_PORT', '')}:{env.get('TORCHELASTIC_RUN_ID', '')}"
    return os.path.join(tempfile.gettempdir(), "arx_uid_" + hashlib.sha1(key.encode()).hexdigest()[:16] + ".bin")


def share_unique_ids(rank: int, world: int, env: dict, make_uid, count: int = 1,
                     timeout_s: float = 300.0) -> list:
    """Rank 0's `count` RCCL unique ids (one per group: the headline group and the second group of
    the frames-in-flight leg) to every rank; a one-rank group needs none."""
    if world == 1:
        return [None] * count
    path = uid_path(env)
    if rank == 0:
        ids = [make_uid() for _ in range(count)]
        tmp = f"{path}.{os.getpid()}.tmp"
        with open(tmp, "wb") as fh:
            fh.write(b"".join(ids))
        os.replace(tmp, path)
        return ids
    t0 = time.monotonic()
    while time.monotonic() - t0 < timeout_s:
        try:
            with open(path, "rb") as fh:
                blob = fh.read()
            if len(blob) == 128 * count:
                return [blob[128 * i:128 * (i + 1)] for i in range(count)]
        except FileNotFoundError:
            pass
        time.sleep(0.05)
    raise SystemExit(f"rank {rank}: no RCCL unique id from rank 0 at {path} after {timeout_s:.0f} s")


def share_unique_id(rank: int, world: int, env: dict, make_uid, timeout_s: float = 300.0) -> bytes | None:
    """Rank 0's RCCL unique id to every rank (a one-rank group needs none)."""
    return share_unique_ids(rank, world, env, make_uid, 1, timeout_s)[0]


class Ranks:
    """Barrier / max / sum over the job's processes: RCCL all-reduces of the group itself (one
    process driving every GPU needs none)."""

    def __init__(self, group, mode: str, forced: bool = False):
        self.g = group
        # forced (--debug-force-collectives): the one-rank group issues them too (tests only)
        self.multi = (mode == "rank" and group.n_ranks > 1) or forced

    def barrier(self) -> None:
        if self.multi:
            self.g.allreduce([0.0])

    def max(self, v: float) -> float:
        return float(self.g.allreduce([v], "max")[0]) if self.multi else float(v)

    def sum(self, v: float) -> float:
        return float(self.g.allreduce([v], "sum")[0]) if self.multi else float(v)


class Watchdog:
    """A step that never completes (a cross-GPU ordering bug in the frames-in-flight all-reduce chain,
    a collective some rank skipped) must not leave the driver's run hung without a line: a daemon
    thread watches the time since the last progress beat and, past the armed limit, prints ONE JSON
    line {"status": "hang", "phase", "rank", ...} and ends the process (exit code 3; no re-exec, no
    retry).  The main thread's GPU waits are ctypes calls, which release the GIL, so the thread runs
    while they block."""

    def __init__(self, rank: int, world: int, out=None, on_hang=None, poll_s: float = 0.5):
        self.rank, self.world = rank, world
        self.out = out if out is not None else sys.stdout
        self.on_hang = on_hang if on_hang is not None else os._exit
        self.limit_s = None
        self.phase = "setup"
        self.steps_done = 0
        self.info = {}
        self.fired = False
        self._last = time.monotonic()
        self._lock = threading.Lock()
        self._poll = poll_s
        threading.Thread(target=self._run, name="bench-watchdog", daemon=True).start()

    def arm(self, limit_s: float, phase: str | None = None) -> None:
        with self._lock:
            self.limit_s = float(limit_s)
            self._last = time.monotonic()
            if phase:
                self.phase = phase

    def disarm(self) -> None:
        with self._lock:
            self.limit_s = None

    def beat(self, phase: str | None = None, step: bool = False) -> None:
        with self._lock:
            self._last = time.monotonic()
            if phase:
                self.phase = phase
            if step:
                self.steps_done += 1

    def _run(self) -> None:
        while not self.fired:
            time.sleep(self._poll)
            with self._lock:
                if self.limit_s is None or time.monotonic() - self._last <= self.limit_s:
                    continue
                self.fired = True
                line = {"status": "hang", "metric": METRIC, "phase": self.phase, "rank": self.rank,
                        "world": self.world, "steps_done": self.steps_done,
                        "seconds_since_progress": round(time.monotonic() - self._last, 2),
                        "limit_s": self.limit_s, **self.info}
            # stdout carries one line per job: rank 0's; the other ranks say it on stderr
            out = self.out if self.rank == 0 else sys.stderr
            out.write(json.dumps(line) + "\n")
            out.flush()
            self.on_hang(3)


# ------------------------------------------------------------------------------ CPU baseline ---
def cpu_baseline(scene, receiver, wl, n_total_rays, audio, budget_s: float) -> dict:
    """The CPU oracle (naive C ray loop + median-split BVH) on this host, bounded samples of the
    same launch: one thread, and every core this process may run on (sched_getaffinity)."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import pyoracle as po
    from audiorenderingv2_amd.renderer import place_receiver_vertices

    build_note = native_oracle(po)
    from audiorenderingv2_amd.scene import CONFERENCE_EMITTER, CONFERENCE_LISTENER

    L, R = receiver
    Lw = place_receiver_vertices(L.reshape(-1, 3), CONFERENCE_LISTENER, 0.0).reshape(-1, 9)
    Rw = place_receiver_vertices(R.reshape(-1, 3), CONFERENCE_LISTENER, 0.0).reshape(-1, 9)
    tv = np.concatenate([scene.tri_v, Lw, Rw])
    ta = np.concatenate([scene.tri_abs, np.full(len(Lw), -1, np.float32), np.full(len(Rw), -2, np.float32)])
    osc = po.Scene(tv, ta, bvh=True)
    p = po.make_params(rays=(n_total_rays, 1, 1), sample_rate=wl["sample_rate"], base_power=3.62,
                       max_bounces=wl["max_bounces"], emitter=CONFERENCE_EMITTER, listener=CONFERENCE_LISTENER)
    cores = available_cores()

    def timed(threads: int, seconds: float) -> tuple[float, int, float]:
        n = 500 * threads
        t0 = time.perf_counter()
        osc.trace(p, 0, n, threads=threads)
        rate = n / max(time.perf_counter() - t0, 1e-6)
        n2 = int(min(max(rate * seconds, n), 4_000_000))
        t0 = time.perf_counter()
        _, _, st = osc.trace(p, 0, n2, threads=threads)
        dt = time.perf_counter() - t0
        return st["queries"] / dt, n2, dt

    one, n1, d1 = timed(1, budget_s / 2)
    allc, n2, d2 = timed(cores, budget_s / 2)
    # convolution leg: the f64 oracle block convolution of a bounded slice of the same audio
    sr = wl["sample_rate"]
    ir = np.zeros(2 * sr, np.float32)
    ir[::97] = 1e-4
    x = audio[:min(audio.size, 8 * sr)]
    t1 = time.perf_counter()
    po.convolute_audio(x, sr, ir)
    po.convolute_audio(x, sr, ir)
    dtc = time.perf_counter() - t1
    return {
        "value": allc, "unit": "ray-bounces/s", "cores": cores, "kind": "port",
        "sample": f"oracle/arx_oracle.c ({build_note}, median-split BVH): rays 0..{n2} of the same launch on {cores} "
                  f"threads = the CPUs this process may use (affinity capped by the cgroup quota) ({d2:.1f} s); "
                  f"1 thread: rays 0..{n1} ({d1:.1f} s)",
        "single_thread_value": one,
        "convolved_frames_per_s": x.size / (dtc / 2),
        "convolution_sample": f"f64 oracle block convolution, 1 thread, {x.size} frames x 2 ears",
        "cpu_model": _cpu_model(),
    }


def native_oracle(po) -> str:
    """Build the oracle with -O3 -march=native for THIS host (`make -C oracle native` into
    a temporary directory, a few seconds) and load it; the portable liboracle.so if that fails."""
    out = os.path.join(tempfile.mkdtemp(prefix="arx_oracle_native_"), "liboracle_native.so")
    try:
        r = subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle"), "native", f"NATIVE_OUT={out}"],
                           capture_output=True, text=True, timeout=180)
        if r.returncode == 0 and os.path.exists(out):
            po.use_library(out)
            return "-O3 -march=native -ffp-contract=off, built on this host"
        why = (r.stderr or r.stdout).strip().splitlines()[-1:] or ["make failed"]
    except (OSError, subprocess.SubprocessError, RuntimeError) as e:
        why = [str(e)]
    return f"-O3 portable liboracle.so (the -march=native build failed: {why[0][:120]})"


def available_cores() -> int:
    """CPUs this process may use: its affinity mask, capped by a cgroup CPU quota (on the GPU box the
    mask lists the whole machine while the container's share is a fraction of it)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        with open("/sys/fs/cgroup/cpu.max") as fh:
            quota, period = fh.read().split()[:2]
        if quota != "max":
            n = min(n, max(1, math.ceil(int(quota) / int(period))))
    except (OSError, ValueError):
        pass
    return n


def _cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


# ------------------------------------------------------------------------------- extra legs ---
C5 = dict(rays=(100, 100, 100), max_bounces=16, sample_rate=48000)  # configs[4]: 1M rays x 16 per frame in total


def moving_listener(g, ranks: Ranks, frames: int, rays_per_gpu: int, wd: "Watchdog | None" = None) -> dict:
    """SURVEY.md §8d C5 (configs[4]): 1M rays x 16 bounces per frame in total, sharded over the job's
    GPUs (125K per GPU on 8), the listener moving 0.05 m/frame along +x with yaw += 1 deg/frame.
    Frame latency = host wall time of: receiver re-placement (receiver sub-tree only, no scene
    rebuild; a grid that grows is re-quantized on the device) -> trace every GPU's shard -> RCCL
    all-reduce -> finalize IR -> new IR spectra for the file and the live convolution paths on every
    GPU, synchronised.  The reference instead re-places the receiver and rebuilds the whole GAS
    and pipeline (OptixModel.cpp:153-257, AudioRenderer.cpp:466-486, 790-798).  p50/p99/max are
    max over ranks."""
    from audiorenderingv2_amd.scene import CONFERENCE_LISTENER

    x0, y0, z0 = CONFERENCE_LISTENER
    lat = []
    for k in range(frames + 3):
        g.synchronize()
        t0 = time.perf_counter()
        g.setSphereCenterInOptix((x0 + 0.05 * k, y0, z0), float(k % 360))
        g.render(timed=False)
        for m in g.members:
            m.prepare_ir_spectra(file=True, live=True)
        g.synchronize()
        if k >= 3:  # first frames warm the receiver rebuild path
            lat.append((time.perf_counter() - t0) * 1e3)
        if wd is not None:
            wd.beat()
    a = np.array(lat)
    out = {"frames": frames, "rays_per_frame": int(np.prod(C5["rays"])), "rays_per_gpu": rays_per_gpu,
           "gpus": g.n_ranks, "p50_ms": ranks.max(float(np.percentile(a, 50))),
           "p99_ms": ranks.max(float(np.percentile(a, 99))), "max_ms": ranks.max(float(a.max())),
           "budget_ms": 1000.0 / 60.0, "walk_m": 0.05 * (frames + 2),
           "per_frame": "listener re-place (+0.05 m x, +1 deg yaw) + trace + RCCL all-reduce (N > 1) + finalize + "
                        "IR spectra, on a C5 group of its own (1M rays x 16 per frame over all GPUs)"}
    # the frames' all-reduces, measured (HIP events around the collective on each member's stream;
    # recorded when the group times its launches, at N > 1 or with the collectives forced)
    n_ar = min(frames, 256)  # the group's all-reduce event ring: the last 256 frames
    ars = [g.allreduce_times(n_ar, i) for i in range(len(g.members))]
    if n_ar > 0 and all(len(x) == n_ar for x in ars):
        worst = np.max(np.stack(ars), axis=0)
        out["allreduce_p50_ms"] = ranks.max(float(np.percentile(worst, 50)))
        out["allreduce_p99_ms"] = ranks.max(float(np.percentile(worst, 99)))
        out["allreduce_source"] = (f"measured: arx_group_allreduce_times over the last {n_ar} frames, slowest member "
                                   "per frame, max over ranks")
    return out


def allreduce_model_us(n_ranks: int, nbytes: int, alpha_us: float = 3.0, link_gbs: float = 153.0) -> float:
    """Ring all-reduce over xGMI: 2 (G - 1) dependent steps of latency alpha plus 2 (G - 1) / G of the
    buffer through one link (ring collectives are per-link bound; one xGMI link ~153 GB/s).  A model
    for the one-GPU box; on an N-GPU node the moving-listener leg measures the real one."""
    if n_ranks <= 1:
        return 0.0
    return 2 * (n_ranks - 1) * alpha_us + 2 * (n_ranks - 1) / n_ranks * nbytes / (link_gbs * 1e9) * 1e6


def moving_listener_rank_shape(settings, scene, receiver, frames: int, shard: int) -> dict:
    """C5's per-GPU frame on 8 GPUs: 1M rays per frame split 8 ways is 125K rays per GPU.  One
    renderer traces rays [0, shard) of the 1M launch per frame (plus re-placement, finalize and
    IR spectra); the 8-GPU all-reduce of 768 kB adds ~10-20 us over xGMI."""
    from audiorenderingv2_amd import AudioRenderer
    from audiorenderingv2_amd.scene import CONFERENCE_EMITTER, CONFERENCE_LISTENER

    r = AudioRenderer(settings, scene=scene, receiver=receiver)
    r.setEmitterPosInOptix(CONFERENCE_EMITTER)
    r.set_timing(False)  # host wall clock per frame; no event markers in it
    x0, y0, z0 = CONFERENCE_LISTENER
    lat = []
    for k in range(frames + 3):
        t0 = time.perf_counter()
        r.setSphereCenterInOptix((x0 + 0.05 * k, y0, z0), float(k % 360))
        r.clear_histogram()
        r.trace_rays(0, shard)
        r.finalize_ir()
        r.prepare_ir_spectra(file=True, live=True)
        r.stats()  # synchronises the renderer's stream
        if k >= 3:
            lat.append((time.perf_counter() - t0) * 1e3)
    hist_bytes = 2 * r.ir_length * 8  # the int64 histogram the 8 ranks all-reduce
    r.close()
    a = np.array(lat)
    ar_ms = allreduce_model_us(8, hist_bytes) / 1e3
    return {"frames": frames, "rays_per_gpu": shard, "p50_ms": float(np.percentile(a, 50)),
            "p99_ms": float(np.percentile(a, 99)), "max_ms": float(a.max()), "budget_ms": 1000.0 / 60.0,
            "allreduce_ms_model": ar_ms,
            "allreduce_model": f"NOT MEASURED: ring over 8 GPUs, {hist_bytes} B int64 histogram, 14 steps x 3 us + "
                               "1.75 x bytes at 153 GB/s (one xGMI link); the latency fields above exclude it, the "
                               "8-GPU run's moving_listener measures the real one",
            "per_frame": "one GPU's 1/8 shard of a 1M-ray frame: re-place + trace + finalize + IR spectra, measured "
                         "(the 8-GPU rank's frame without its all-reduce)"}


def streaming_leg(m, audio, block: int) -> dict:
    """C3's streaming overlap-add leg: the same audio fed through the streaming convolution
    (arx_stream_*: uniformly partitioned overlap-save, f64) in 4096-frame blocks, device-resident
    (arx_stream_process_device): per-block device latency (the renderer's live event ring) and
    frames/s (host clock around the back-to-back blocks)."""
    from audiorenderingv2_amd import DeviceBuffer, LiveStream

    dev = m.settings.device
    s = LiveStream(m, block)
    x = DeviceBuffer.from_numpy(dev, audio.astype(np.float64))
    out = DeviceBuffer(dev, 2 * block * 8)
    nb = audio.size // block
    for b in range(8):  # warm-up
        s.process_device(x.ptr + 8 * b * block, block, out.ptr)
    m.stats()  # synchronises the renderer's stream
    t0 = time.perf_counter()
    for b in range(nb):
        s.process_device(x.ptr + 8 * b * block, block, out.ptr)
    m.stats()
    total_s = time.perf_counter() - t0
    per = m.live_times(nb)
    s.close()
    x.close()
    out.close()
    return {"block_frames": block, "blocks": nb, "partitions": s.partitions, "fft_size": s.fft_size,
            "frames_per_s": nb * block / total_s, "block_p50_ms": float(np.percentile(per, 50)),
            "block_p99_ms": float(np.percentile(per, 99)), "block_period_ms": 1e3 * block / 48000.0,
            "method": "device-resident, back-to-back blocks on the renderer stream; per-block HIP events "
                      "(arx_live_times), frames/s on the host clock around all blocks"}


# -------------------------------------------------------------------------- stored profiles ---
def load_profile(name: str) -> dict | None:
    path = os.path.join(REPO, "profiles", name)
    if os.path.exists(path):
        with open(path) as fh:
            return json.load(fh)
    return None


def profile_guard(prof: dict | None, workload: str, stats: dict,
                  keys: tuple = ("workload", "tree_hash", "trace_vgprs", "trace_kernel_id")) -> tuple[dict | None, str]:
    """A stored PMC-derived profile applies to this run only if it was taken on the same workload,
    the same scene tree (content hash) and the same trace kernel (source identity, arx_trace_kernel_id,
    and register allocation): the counters cannot be read inside this run, and a stale file must not
    pass as a measurement.  (Per-query lane counts come from a separate counting build of the same
    kernel source: they are guarded by the tree and the kernel identity.)"""
    from audiorenderingv2_amd._lib import lib
    if prof is None:
        return None, "missing"
    want = {"workload": workload, "tree_hash": f"{int(stats['tree_hash']):016x}",
            "trace_vgprs": int(stats["trace_vgprs"]), "trace_kernel_id": f"{int(lib().arx_trace_kernel_id()):016x}"}
    want = {k: want[k] for k in keys}
    bad = [k for k, v in want.items() if prof.get(k) != v]
    if bad:
        return None, "stale: " + ", ".join(f"{k} {prof.get(k)!r} != {want[k]!r}" for k in bad)
    return prof, "matches " + " / ".join(keys)


def conv_profile_guard(prof: dict | None, workload: str) -> tuple[dict | None, str]:
    """The stored convolution traffic applies only to the C3 workload and to the convolution kernels
    it was taken of (arx_conv_kernel_id, a hash of arx_conv.hip compiled into libarx)."""
    from audiorenderingv2_amd._lib import lib
    if prof is None:
        return None, "missing"
    want = {"workload": workload, "conv_kernel_id": f"{int(lib().arx_conv_kernel_id()):016x}"}
    bad = [k for k, v in want.items() if prof.get(k) != v]
    if bad:
        return None, "stale: " + ", ".join(f"{k} {prof.get(k)!r} != {want[k]!r}" for k in bad)
    return prof, "matches workload / conv_kernel_id"


@contextlib.contextmanager
def _stdout_to_stderr():
    """Send whatever native libraries write on fd 1 to fd 2 for the duration."""
    sys.stdout.flush()
    saved = os.dup(1)
    try:
        os.dup2(2, 1)
        yield
    finally:
        sys.stdout.flush()
        os.dup2(saved, 1)
        os.close(saved)


# -------------------------------------------------------------------------------------- main ---
def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--preroll-s", type=float, default=0.5,
                    help="untimed steps for this long before the warmup steps: a fresh process on an idle GPU "
                         "runs its first ~10 C3 launches 2.95 -> 2.67 ms while the clock ramps, and again after "
                         "2 s idle (tools/trace_ramp.py, profiles/r04/trace_ramp.json)")
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="c3")
    ap.add_argument("--cpu-baseline-seconds", type=float, default=16.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--c5-frames", type=int, default=600,
                    help="moving-listener frames after the timed steps (SURVEY C5); 0 disables")
    ap.add_argument("--no-streaming", action="store_true")
    ap.add_argument("--no-reuse", action="store_true", help="skip the input-reuse convolution leg")
    ap.add_argument("--frames-in-flight", type=int, choices=(1, 2, 3), default=None,
                    help="frames the group keeps in flight in the timed steps (arx_group_set_frames_in_flight): "
                         "with 2, step k+1's trace starts while step k finishes, and a single-frame leg is timed "
                         "too; a ray-pool launch then takes half the CUs' wave slots, so two frames trace side by "
                         "side (config.trace_grid_cus).  Default on one GPU: 3 for c2, 2 for c3, 1 for c4 (its 46 ms "
                         "launches have little tail to hide and lose 7-13 %% on half grids, "
                         "profiles/r06/grid_ab_c4.txt).  Default at N > 1: 1, until a multi-GPU run of the frames-in-flight "
                         "all-reduce chain is on record (each frame's all-reduce runs on its own frame stream after "
                         "the previous frame's; tests/test_gpu_collectives.py runs that chain with every "
                         "collective forced on one GPU only)")
    ap.add_argument("--replicated-convolution", action="store_true",
                    help="every GPU convolves the whole file (replicas) instead of its time-block shard "
                         "(arx_group_convolute_device); the convolved-frames rates then count every copy")
    ap.add_argument("--watchdog-s", type=float, default=None,
                    help="no progress for this long -> one JSON line {\"status\": \"hang\", ...} and exit 3 "
                         "(default: 180 s through the pre-roll, then max(30 s, 50 x the pre-roll step))")
    ap.add_argument("--debug-oversubscribe", action="store_true",
                    help="tests only: --gpus N as N ranks on device 0 (one process, an oversubscribed group: the "
                         "N-rank job's shards, sharded convolution and accounting rehearsed on one GPU)")
    ap.add_argument("--debug-hang-at-step", type=int, default=-1,
                    help="tests only: stall the host inside timed step K (a stand-in for a GPU wait that never "
                         "returns), so the watchdog fires")
    ap.add_argument("--no-pipelined", action="store_true",
                    help="no-op: the two-group pipelined leg (round 3) became --frames-in-flight")
    ap.add_argument("--timing-events", action="store_true",
                    help="keep the renderers' per-launch timing events on in the timed steps too (A/B of their cost; "
                         "the kernel-times leg records them either way)")
    ap.add_argument("--no-host-leg", action="store_true",
                    help="skip the host-buffer (PCIe-inclusive) leg: render + arx_convolute_audio_file from and to "
                         "host memory")
    ap.add_argument("--debug-force-collectives", action="store_true",
                    help="tests only: every group collective is issued even at one rank (the histogram all-reduce "
                         "with frames in flight, the barriers and max-over-ranks, the rank path's scene broadcast), "
                         "so a one-GPU box runs the multi-GPU job's collective path (arx_debug_group_force_collectives)")
    ap.add_argument("--process-group", action="store_true",
                    help="take the one-GPU-per-process (RCCL rank) path even at one rank: a rehearsal of the "
                         "torch.distributed.run path on a one-GPU box")
    args = ap.parse_args(argv)
    try:
        plan = plan_ranks(args.gpus, os.environ, args.process_group, args.debug_oversubscribe)
    except ValueError as e:
        raise SystemExit(f"bench.py: {e}")

    from audiorenderingv2_amd import (RenderGroup, RenderSettings, conference_standin, device_count, receiver_local,
                                      runtime_info)
    from audiorenderingv2_amd._lib import lib
    from audiorenderingv2_amd.renderer import DeviceBuffer
    from audiorenderingv2_amd.scene import CONFERENCE_EMITTER, CONFERENCE_LISTENER, reference_audio

    ring = int(lib().arx_timing_ring())
    if args.steps < 1 or args.steps > ring:
        raise SystemExit(f"bench.py: --steps must be in [1, {ring}] (the renderer's per-launch timing ring)")
    have = device_count()
    if have < plan["local_gpus_needed"]:
        raise SystemExit(f"bench.py: --gpus {args.gpus} needs {plan['local_gpus_needed']} visible GPU(s) in this "
                         f"process, the HIP runtime sees {have}; refusing to print a line for fewer GPUs")
    world, rank = plan["world"], plan["rank"]
    wd = Watchdog(rank, world)
    wl = WORKLOADS[args.workload]
    rx, ry, rz = wl["rays"]
    if wl.get("total"):  # a fixed total split over the GPUs (strong scaling)
        total_rays = rx * ry * rz
        launch = (rx, ry, rz)
    else:  # a fixed shard per GPU (weak scaling)
        total_rays = rx * ry * rz * world
        launch = (rx * world, ry, rz)
    settings = RenderSettings(rays=launch, ir_length_in_seconds=2, sample_rate=wl["sample_rate"],
                              base_power=3.62, max_bounces=wl["max_bounces"], hrtf_absorption_rate=1.0, seed=1,
                              device=plan["devices"][0])
    scene = conference_standin()
    receiver = receiver_local()
    t_setup = time.perf_counter()
    with _stdout_to_stderr():  # RCCL prints its version banner on stdout; stdout is the JSON line only
        if plan["mode"] == "rank":
            uids = share_unique_ids(rank, world, os.environ, RenderGroup.unique_id, 3)
            g = RenderGroup.rank(settings, world, rank, uids[0])
        else:
            uids = [None, None, None]
            g = RenderGroup(settings, devices=plan["devices"])
        if args.debug_force_collectives:
            g.debug_force_collectives(True, True)
        g.set_receiver_model(*receiver)
        g.set_scene(scene)  # the rank path: rank 0 builds, the tree reaches the other ranks over RCCL
    # the timed steps carry no per-launch event markers (each cost its stream ~4.5 us,
    # tools/step_gaps.py); the kernel times come from a leg of their own below
    g.set_timing(args.timing_events)
    ranks = Ranks(g, plan["mode"], args.debug_force_collectives)
    ranks.barrier()
    if plan["mode"] == "rank" and rank == 0 and world > 1:
        with contextlib.suppress(OSError):
            os.remove(uid_path(os.environ))
    if g.n_ranks != world:
        raise SystemExit(f"bench.py: the group has {g.n_ranks} ranks, --gpus asked for {world}")
    g.setEmitterPosInOptix(CONFERENCE_EMITTER)
    g.setSphereCenterInOptix(CONFERENCE_LISTENER, 0.0)
    members = g.members
    ir_len = members[0].ir_length
    audio_np, sr = reference_audio(wl["audio"])
    assert sr == wl["sample_rate"]
    frames = int(audio_np.size)
    bufs = []  # per member: the audio and both output channels, resident on its GPU
    for m in members:
        d = m.settings.device
        bufs.append((DeviceBuffer.from_numpy(d, audio_np), DeviceBuffer(d, 4 * frames), DeviceBuffer(d, 4 * frames)))
    # the convolution: each rank convolves its time-block shard of the file (arx_group_convolute_device;
    # the union is the one-GPU convolution bit for bit, tests/test_gpu_group_conv.py), or with
    # --replicated-convolution the whole file on every GPU
    sharded_conv = not args.replicated_convolution
    d_in, d_ol, d_or = [b[0].ptr for b in bufs], [b[1].ptr for b in bufs], [b[2].ptr for b in bufs]
    conv_plan_shards = g.conv_sharded
    own = [g.conv_shard(frames, rank + i) for i in range(len(members))]
    unique_frames = frames if (sharded_conv or world == 1) else world * frames

    # timing: the renderers' own HIP events around each trace launch and each convolution (on
    # their streams); no further markers in the timed loop -- each costs the stream a few us
    def step():
        g.render(timed=False)  # clear + trace + RCCL all-reduce + finalize, every GPU
        if sharded_conv:
            g.convolute_device(d_in, frames, d_ol, d_or)
        else:
            for m, (x, ol, orr) in zip(members, bufs):
                m.convolute_device(x.ptr, frames, ol.ptr, orr.ptr)
        wd.beat(step=True)

    def sync(phase=None):
        g.synchronize()
        wd.beat(phase)

    if args.frames_in_flight is None:
        args.frames_in_flight = wl["fif"] if world == 1 else 1
    wd.info["frames_in_flight"] = args.frames_in_flight
    g.set_frames_in_flight(args.frames_in_flight)
    # pre-roll: untimed steps until the GPU runs at its sustained clock, then the contract's W warmup
    # steps.  The ranks agree after every step whether to go on (max over ranks), so each takes the
    # same number of steps and their all-reduces stay paired.
    wd.arm(args.watchdog_s or 180.0, "preroll")
    t_pre, pre_steps = time.perf_counter(), 0
    while True:
        step()
        sync()
        pre_steps += 1
        if ranks.max(1.0 if time.perf_counter() - t_pre < args.preroll_s else 0.0) == 0.0:
            break
    preroll_s = time.perf_counter() - t_pre
    wd_limit = args.watchdog_s or max(30.0, 50.0 * preroll_s / pre_steps)
    wd.arm(wd_limit, "warmup")
    for _ in range(args.warmup):
        step()
    sync()
    g.stats()
    setup_s = time.perf_counter() - t_setup
    ranks.barrier()
    sync("timed")
    t0 = time.perf_counter()
    for k in range(args.steps):
        if k == args.debug_hang_at_step:
            time.sleep(2.0 * wd_limit + 5.0)  # tests only: the watchdog ends the process first
        step()
    sync()
    ranks.barrier()
    t1 = time.perf_counter()
    elapsed = ranks.max(t1 - t0)
    stats = g.stats()
    collectives = g.debug_collectives()  # the headline group's, up to the end of the timed steps
    q_proc = int(stats["queries"])  # this process's members, per step (counters cleared every step)
    q_all = int(round(ranks.sum(q_proc)))
    m0 = members[0]
    st0 = m0.stats()
    q_m0 = int(st0["queries"])
    value = q_all * args.steps / elapsed
    # With two frames in flight a launch's HIP-event window (on its stream) also holds the time it
    # queues behind the other frame's kernels, so the per-launch times (phases, rooflines) come from
    # a single-frame leg: the same group, W + K steps with one frame in flight.
    single_frame = None
    if args.frames_in_flight > 1:
        wd.beat("single_frame")
        g.set_frames_in_flight(1)
        for _ in range(args.warmup):
            step()
        sync()
        ranks.barrier()
        t0s = time.perf_counter()
        for _ in range(args.steps):
            step()
        sync()
        ranks.barrier()
        el1 = ranks.max(time.perf_counter() - t0s)
        q1 = int(round(ranks.sum(int(g.stats()["queries"]))))
        single_frame = {"value": q1 * args.steps / el1, "ms_per_step": el1 / args.steps * 1e3,
                        "why": "the same steps with one frame in flight (no per-launch timing events, as in the "
                               "timed steps)"}
    # The per-launch kernel times: W + K more single-frame steps with the timing events on (HIP
    # events on the renderer's stream around the direction pre-pass + trace kernel, and around the IR
    # spectra + convolution), the K timed launches of GPU 0 of this process.
    wd.beat("kernel_times")
    g.set_frames_in_flight(1)
    g.set_timing(True)
    for _ in range(args.warmup):
        step()
    sync()
    ranks.barrier()
    t0k = time.perf_counter()
    for _ in range(args.steps):
        step()
    sync()
    ranks.barrier()
    timed_leg_ms = ranks.max(time.perf_counter() - t0k) / args.steps * 1e3
    trace_list = m0.trace_times(args.steps)
    assert len(trace_list) == args.steps, (len(trace_list), args.steps)
    grid_cus_single = int(m0.stats()["trace_grid_cus"])
    trace_ms = float(np.mean(trace_list))
    # the histogram all-reduce's own window (HIP events on each member's stream around the RCCL call,
    # arx_group_allreduce_times), the slowest member, max over ranks; none at one rank unless forced
    ar_lists = [g.allreduce_times(args.steps, i) for i in range(len(members))]
    if all(len(a) == args.steps for a in ar_lists):
        allreduce_ms = ranks.max(max(float(np.mean(a)) for a in ar_lists))
        allreduce_why = (f"RCCL int64 all-reduce of 2 x {ir_len} bins over {world} rank(s): HIP events around the "
                         "collective on each member's stream (arx_group_allreduce_times), mean of the K timed "
                         "launches, slowest member, max over ranks")
    else:
        allreduce_ms = None
        allreduce_why = "one rank: arx_group_render skips the no-op all-reduce (--debug-force-collectives times it)"
    conv_ms_all = []
    for m in members:
        cl = m.conv_times(args.steps)
        assert len(cl) == args.steps, (len(cl), args.steps)
        conv_ms_all.append(float(np.mean(cl)))
    conv_ms = conv_ms_all[0]
    # the frames rank 0's convolution window covers: its shard, or the whole file
    conv_frames_rank0 = (own[0][1] - own[0][0]) if (sharded_conv and conv_plan_shards and world > 1) else frames
    conv_ms_max = ranks.max(max(conv_ms_all))
    # Input reuse (arx_convolute_prepare_input / _prepared): the reference re-convolves the same file
    # with every new IR (full_render_cycle, AudioRenderer.cpp:790-798), so the file's blocks can be
    # transformed once.  Its own leg, one frame in flight, never the headline's work: the same steps
    # with the convolution of the prepared input, its kernel window beside the full one.
    reuse = None
    if not args.no_reuse:
        wd.beat("input_reuse")
        g.set_frames_in_flight(1)
        for m, (x, _, _) in zip(members, bufs):
            m.convolute_prepare_input(x.ptr, frames)

        def step_reuse():
            g.render(timed=False)
            for m, (_, ol, orr) in zip(members, bufs):
                m.convolute_prepared(ol.ptr, orr.ptr)

        for _ in range(args.warmup):
            step_reuse()
        sync()
        ranks.barrier()
        t0r = time.perf_counter()
        for _ in range(args.steps):
            step_reuse()
            wd.beat()
        sync()
        ranks.barrier()
        elr = ranks.max(time.perf_counter() - t0r)
        reuse_ms = float(np.mean(m0.conv_times(args.steps)))
        reuse = {"conv_ms_rank0": reuse_ms, "ms_per_step": elr / args.steps * 1e3,
                 "convolved_frames_per_s_kernel_window": frames / (reuse_ms * 1e-3),
                 "why": "the reference's re-render pattern (the same file, a new IR every frame): the file's blocks "
                        "transformed once (arx_convolute_prepare_input), each step's convolution "
                        "(arx_convolute_prepared) = the new IR's spectra + products + inverse transforms, "
                        "bit-identical to the full one (tests/test_gpu_conv_reuse.py); not the headline's work"}
        g.set_frames_in_flight(args.frames_in_flight)
    # Host buffers (the PCIe-inclusive rate, never the value): the reference's full_render_cycle
    # shape through the C ABI's host-memory entry point -- render, then arx_convolute_audio_file with
    # the audio in host memory and both output channels back in host memory (AudioRenderer.cpp:663-750).
    host_leg = None
    if not args.no_host_leg:
        wd.beat("host_buffers")
        g.set_frames_in_flight(1)

        def step_host():
            g.render(timed=False)
            return [m.convoluteAudioFile(audio_np)[3] for m in members]

        for _ in range(args.warmup):
            step_host()
        sync()
        ranks.barrier()
        t0h = time.perf_counter()
        host_conv = []
        for _ in range(args.steps):
            host_conv.append(max(step_host()))
            wd.beat()
        sync()
        ranks.barrier()
        elh = ranks.max(time.perf_counter() - t0h)
        host_leg = {"ms_per_step": elh / args.steps * 1e3,
                    "ray_bounces_per_s": q_all * args.steps / elh,
                    "host_path_ms": float(ranks.max(np.median(host_conv))),
                    "host_bytes_per_gpu_per_step": 3 * 4 * frames,
                    "why": "the PCIe-inclusive rate, not the value: each step renders and then convolves the file "
                           "from host memory into host memory (arx_convolute_audio_file: f32 samples in, both "
                           "channels out), one frame in flight; host_path_ms = that call's median window on the renderer's stream "
                           "(HIP events: host-to-device copy, IR spectra + convolution, both device-to-host copies), "
                           "slowest GPU"}
        g.set_frames_in_flight(args.frames_in_flight)

    n_tris = int(stats["n_scene_tris"] + stats["n_receiver_tris"])
    moving = None
    if args.c5_frames > 0:  # C5 on a group of its own: 1M rays per frame in total, sharded over the GPUs
        s5 = RenderSettings(rays=C5["rays"], ir_length_in_seconds=2, sample_rate=C5["sample_rate"], base_power=3.62,
                            max_bounces=C5["max_bounces"], hrtf_absorption_rate=1.0, seed=1, device=plan["devices"][0])
        with _stdout_to_stderr():
            if plan["mode"] == "rank":
                g5 = RenderGroup.rank(s5, world, rank, uids[2])
            else:
                g5 = RenderGroup(s5, devices=plan["devices"])
            if args.debug_force_collectives:
                g5.debug_force_collectives(True, True)
            g5.set_receiver_model(*receiver)
            g5.set_scene(scene)
        g5.setEmitterPosInOptix(CONFERENCE_EMITTER)
        # host wall clock per frame; event markers only where there is an all-reduce to time
        g5.set_timing(world > 1 or args.debug_force_collectives)
        wd.beat("moving_listener")
        moving = moving_listener(g5, ranks, args.c5_frames, int(np.prod(C5["rays"])) // world, wd)
        g5.close()
    bpb = bytes_per_bounce(n_tris)
    achieved = q_m0 * bpb / (trace_ms * 1e-3) / 1e9
    traffic, traffic_why = profile_guard(load_profile(os.path.join(PROFILES, "trace_traffic.json")), args.workload, st0)
    counts, counts_why = profile_guard(load_profile(os.path.join(PROFILES, "trace_counts_c3.json")), args.workload, st0,
                                       ("workload", "tree_hash", "trace_kernel_id"))
    td, td_why = profile_guard(load_profile(os.path.join(PROFILES, "trace_td_c3.json")), args.workload, st0)
    vmem, vmem_why = profile_guard(load_profile(os.path.join(PROFILES, "trace_vmem_ceiling.json")), args.workload, st0)
    conv_traffic, conv_traffic_why = conv_profile_guard(load_profile(CONV_TRAFFIC), args.workload)
    parity, parity_why = profile_guard(load_profile(FULL_LAUNCH_PARITY), args.workload, st0,
                                       ("workload", "tree_hash", "trace_kernel_id"))
    # unique stereo frames: the file once per step when it is time-block sharded (or on one GPU), every
    # GPU's copy with --replicated-convolution
    conv_frames_s = unique_frames / (conv_ms_max * 1e-3)  # the convolution kernels' own window
    conv_frames_step = unique_frames * args.steps / elapsed  # the pipeline: frames convolved per timed step
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
                "reference checkout) + the reference's own audio (" + wl["audio"] + ", channel 0)",
        "config": {
            "workload": wl["desc"],
            "scene_triangles": n_tris,
            "rays_per_gpu": total_rays // world,
            "max_bounces": wl["max_bounces"],
            "sample_rate": wl["sample_rate"],
            "ir_len": ir_len,
            "audio_frames": frames,
            "convolution": ("one GPU: the whole file" if world == 1 else
                            (f"time-block sharded over {world} GPUs (arx_group_convolute_device): rank r owns the "
                             f"output frames of block pairs [r P/{world}, (r+1) P/{world}) and re-makes its seam pair, "
                             "no collective" if conv_plan_shards else
                             "this plan has no chained pass: every GPU convolves the whole file")
                            if sharded_conv else f"replicas: each of the {world} GPUs convolves the whole file"),
            "convolved_frames_per_step": unique_frames,
            "conv_frames_owned_rank0": [int(own[0][0]), int(own[0][1])],
            "frames_in_flight": args.frames_in_flight,
            # the persistent trace grid (arx_stats.trace_grid_cus): half the CUs' wave slots per launch
            # with frames in flight, so two frames' launches run side by side; the full device with one
            "trace_grid_cus": {"timed_steps": int(st0["trace_grid_cus"]), "kernel_times_leg": grid_cus_single},
            "parallelism": (f"ray-shard x{world}, "
                            + ("REHEARSAL (--debug-oversubscribe): the ranks' histograms summed on device 0, no RCCL"
                               if args.debug_oversubscribe else
                               "native RCCL int64 IR all-reduce per step" if world > 1 else
                               "one rank: the group's RCCL communicator exists but arx_group_render skips its no-op "
                               "IR all-reduce (arx_group.cpp; tests/test_gpu_collectives.py forces it on one GPU)")
                            + " (arx_group: "
                            + ("one process, ncclCommInitAll over devices " + ",".join(map(str, plan["devices"]))
                               if plan["mode"] == "local" and not args.debug_oversubscribe else
                               "one process, device 0 listed " + str(world) + " times" if args.debug_oversubscribe
                               else f"one process per GPU, ncclCommInitRank, rank {rank}")
                            + ")"),
        },
        "runtime": runtime_info(),
        "collectives_issued": dict(collectives, forced=bool(args.debug_force_collectives),
                                   note="RCCL collectives the headline group issued up to the end of the timed steps "
                                        "(a one-rank group skips them unless forced)"),
        "setup_s_rank0": setup_s,
        "single_frame": single_frame,
        "kernel_times_leg": {"steps": args.steps, "warmup": args.warmup, "frames_in_flight": 1,
                             "ms_per_step": timed_leg_ms,
                             "why": "W + K more single-frame steps with the renderer's per-launch HIP events on "
                                    "(arx_set_timing): phases_ms_rank0 and the rooflines are this leg's launches; "
                                    "its step time against single_frame's is what the four event markers cost a "
                                    "step"},
        "preroll": {"steps": pre_steps, "seconds_rank0": preroll_s,
                    "why": "untimed steps before the W warmup steps, until the GPU runs at its sustained clock "
                           "(a fresh or idle MI355X ramps over its first ~10 C3 launches, 2.95 -> 2.67 ms; "
                           "profiles/r04/trace_ramp.json)"},
        "ray_bounces_per_step": q_all,
        "nominal_ray_bounces_per_s": total_rays * wl["max_bounces"] * args.steps / elapsed,
        "receiver_hits_per_step_rank0": int(st0["receiver_hits"]),
        "convolved_frames_per_s": conv_frames_step,
        "convolved_frames_per_s_kernel_window": conv_frames_s,
        "convolved_frames_per_s_labels": {
            "convolved_frames_per_s": "whole job, per timed step: unique stereo frames convolved "
                                      "(config.convolved_frames_per_step: the file once when sharded or on one GPU, "
                                      "every copy with --replicated-convolution) x K / the K steps' wall time, trace "
                                      "included",
            "convolved_frames_per_s_kernel_window": "the same frames / the slowest GPU's IR-spectra + convolution "
                                                    "window alone (the renderer's HIP events, arx_conv_times)"},
        "phases_ms_rank0": {"trace_kernel": trace_ms, "ir_spectra_and_convolution": conv_ms, "allreduce": allreduce_ms},
        "phases_allreduce_why": allreduce_why,
        "convolution_input_reuse": reuse,
        "host_buffers": host_leg,
        "trace_kernel_build": {"vgprs": int(st0["trace_vgprs"]), "waves_per_simd": int(st0["trace_waves_per_simd"]),
                               "waves_target": int(st0["trace_waves_target"]),
                               "node_format": NODE_FORMATS.get(int(st0["trace_format"]), str(st0["trace_format"])),
                               "tree_hash": f"{int(st0['tree_hash']):016x}"},
        "roofline": {
            "kernel": "trace_kernel",
            # what binds the kernel (PMC: the vector-memory return path TD, VALU beside it); achieved /
            # peak / frac below are the contract's HBM byte convention, whose tree bytes
            # are L1 / L2 hits, so frac can pass what HBM can deliver
            "bound": "td",
            "convention_bound": "hbm",
            "convention_exceeds_achievable_hbm": achieved > HBM_ACHIEVABLE_GBS,
            "achievable_hbm_GBps": HBM_ACHIEVABLE_GBS,
            "queries_match_oracle_full_launch": (
                bool(parity["queries_gpu"] == parity["queries_oracle"] and parity["ir_left_bit_exact"]
                     and parity["ir_right_bit_exact"] and parity["queries_gpu"] == q_m0)
                if parity and world == 1 else None),
            "queries_oracle_full_launch": parity["queries_oracle"] if parity else None,
            "full_launch_parity_source": f"profiles/{FULL_LAUNCH_PARITY} (tests/test_gpu_full_launch.py on the GPU box: "
                                         "the oracle traced every ray of the launch): " + parity_why,
            "convention": "SURVEY.md §8d algorithmic bytes per ray-bounce (32 + 32 + 64 ceil(log2 T) + 48); the "
                          "tree is cache-resident, so this is a byte convention, not the binding unit: the "
                          "kernel is co-limited by the vector-memory return path and VALU issue (roofline_td, "
                          "roofline_valu)",
            "binding_units": "td+valu",
            "binding_unit": "td (the vector-memory return path, busy per CU-cycle; VALU issue per SIMD-cycle "
                            "beside it in roofline_valu)",
            "binding_frac": td["td_busy_per_cu_cycle"] if td else None,
            "achieved": achieved,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS,
            "traffic": traffic.get("bytes_per_launch") if traffic else None,
            "traffic_GBps": traffic["bytes_per_launch"] / (trace_ms * 1e-3) / 1e9 if traffic else None,
            "traffic_frac": traffic["bytes_per_launch"] / (trace_ms * 1e-3) / 1e9 / HBM_PEAK_GBS if traffic else None,
            "traffic_note": "the PMC-counted HBM bytes of one launch over its time, against the 8 TB/s peak: what "
                            "actually crosses HBM (the tree and triangles sit in L2 / Infinity Cache)",
            "traffic_source": f"profiles/{PROFILES}/trace_traffic.json (rocprofv3 --pmc FETCH_SIZE x2 + WRITE_SIZE, same kernel "
                              "build, tree and workload; PMC counters cannot be read inside this run): " + traffic_why,
            "algorithmic_bytes_per_bounce": bpb,
            "trace_launch_ms": trace_ms,
            # the timed steps' own rate by the same convention: with frames in flight two launches
            # run side by side on half the grid each (config.trace_grid_cus), one frame per step
            "timed_steps_achieved": q_m0 * bpb / (elapsed / args.steps) / 1e9,
            "launch_note": "trace_launch_ms / achieved / frac: one launch alone on the full grid (the kernel-times "
                           "leg); timed_steps_achieved: the same bytes per frame over the timed steps' ms_per_step, "
                           "where frames in flight overlap their launches",
        },
        "roofline_convolution": {
            "bound": "hbm",
            "achieved": conv_frames_rank0 * BYTES_PER_STEREO_FRAME / (conv_ms * 1e-3) / 1e9,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": conv_frames_rank0 * BYTES_PER_STEREO_FRAME / (conv_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
            "frames_rank0": conv_frames_rank0,
            "algorithmic_bytes_per_stereo_frame": BYTES_PER_STEREO_FRAME,
            "traffic": conv_traffic["total_bytes_per_step"] if conv_traffic and world == 1 else None,
            "traffic_over_algorithmic": conv_traffic["ratio"] if conv_traffic and world == 1 else None,
            "traffic_source": f"profiles/{CONV_TRAFFIC} (tools/gpu_conv_pmc.sh: rocprofv3 --pmc "
                              "FETCH_SIZE x2 + WRITE_SIZE per pass, the C3 convolution incl. IR spectra, one GPU): "
                              + conv_traffic_why,
        },
    }
    if vmem and counts:
        # the trace's divergent 16-B gathers against the rate a microbenchmark of independent
        # divergent gathers reaches at this kernel's L1 / L2 / Infinity-Cache hit mix
        # (tools/vmem_ceiling.py).  A reference rate, not a hard ceiling: lanes of a wave share the
        # top nodes and a node's two 16-B halves share one 64-B block, which the microbenchmark's
        # one-block-per-lane pattern does not model, so frac may pass 1.
        lane_rate = counts["lane_loads_16B_per_query"] * q_m0 / (trace_ms * 1e-3)
        result["roofline_vmem"] = {
            "kernel": "trace_kernel", "bound": "vector-memory gathers (L1/L2/Infinity-Cache mix), reference rate",
            "achieved": lane_rate, "peak": vmem["ceiling_lane_loads_per_s"], "unit": "16-B lane loads/s",
            "frac": lane_rate / vmem["ceiling_lane_loads_per_s"],
            "note": "peak = independent one-block-per-lane gathers at this hit mix (tools/td_microbench.hip); "
                    "shared nodes and same-block node halves let the kernel pass it",
            "mix": {"l1": vmem["fraction_l1"], "l2_hit": vmem["fraction_l2_hit"], "l2_miss": vmem["fraction_l2_miss"]},
            "source": f"profiles/{PROFILES}/trace_vmem_ceiling.json (tools/td_microbench.hip rates + PMC mix): " + vmem_why,
        }
    else:
        result["roofline_vmem"] = None
        result["roofline_vmem_why"] = f"vmem ceiling {vmem_why}; lane counts {counts_why}"
    if td:
        # the trace kernel's vector-memory return path (TD), busy fraction per CU-cycle
        result["roofline_td"] = {
            "kernel": "trace_kernel", "bound": "td", "achieved": td["td_busy_per_cu_cycle"], "peak": 1.0,
            "unit": "TD busy cycles per CU-cycle", "frac": td["td_busy_per_cu_cycle"],
            "ta_busy": td["ta_busy_per_cu_cycle"], "source": td["source"] + ": " + td_why,
        }
        if "valu_busy_per_simd_cycle" in td:
            # the second unit the trace kernel saturates: VALU issue (a wave64 instruction holds a
            # 16-lane SIMD 4 cycles), SQ_INSTS_VALU x 4 over the SIMDs' cycles in the PMC run
            result["roofline_valu"] = {
                "kernel": "trace_kernel", "bound": "valu issue", "achieved": td["valu_busy_per_simd_cycle"],
                "peak": 1.0, "unit": "VALU-busy cycles per SIMD-cycle", "frac": td["valu_busy_per_simd_cycle"],
                "valu_instructions_per_launch": td["valu_instructions"], "source": td["source"] + ": " + td_why,
            }
    else:
        result["roofline_td"] = None
        result["roofline_td_why"] = td_why
    if counts:
        lanes = counts["lane_loads_16B_per_query"] * q_m0
        result["vector_memory"] = {
            "node_steps_per_query": counts["steps_per_query"], "tri_tests_per_query": counts["tri_tests_per_query"],
            "lane_loads_16B_per_query": counts["lane_loads_16B_per_query"],
            "lane_loads_per_s": lanes / (trace_ms * 1e-3),
            "l1_side_GBps": 16 * lanes / (trace_ms * 1e-3) / 1e9,
            "source": f"profiles/{PROFILES}/trace_counts_c3.json (counting build, tools/trace_counts.py): " + counts_why,
        }
    if moving is not None:
        result["moving_listener"] = moving
        if rank == 0 and world == 1:
            s5 = RenderSettings(rays=C5["rays"], ir_length_in_seconds=2, sample_rate=C5["sample_rate"], base_power=3.62,
                                max_bounces=C5["max_bounces"], hrtf_absorption_rate=1.0, seed=1,
                                device=plan["devices"][0])
            result["moving_listener_rank_of_8"] = moving_listener_rank_shape(s5, scene, receiver, args.c5_frames,
                                                                             int(np.prod(C5["rays"])) // 8)
    if rank == 0 and not args.no_streaming and wl["sample_rate"] == 48000:
        result["streaming"] = streaming_leg(m0, audio_np, 4096)
    wd.disarm()  # the CPU baseline below runs no GPU work
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(scene, receiver, wl, total_rays, audio_np, args.cpu_baseline_seconds)
    if rank == 0:
        print(json.dumps(result), flush=True)
    for b in bufs:
        for x in b:
            x.close()
    ranks.barrier()
    g.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
