"""GPU, two or more distinct GPUs: the N>1 path as the driver's 8-GPU run takes it.

Skipped on a one-GPU box (every test checks `device_count() >= 2` first); there the same code runs
as a one-GPU RCCL group, a one-rank ncclCommInitRank group and oversubscribed groups
(tests/test_gpu_group.py), with every collective forced at one rank -- including both tests below at
the same shapes (tests/test_gpu_collectives.py: test_forced_group_equals_one_renderer_c4,
test_bench_forced_collectives_count_the_plain_launch) -- and its host side in real processes
(tests/test_distributed_gloo.py).

  * RenderGroup(devices=range(n)) -- one process, ncclCommInitAll, one int64 ncclAllReduce of the
    histogram -- at configs[3]'s shape (C4: 10 M rays x 32 bounces, 48 kHz): the IR on every member is
    bit-identical to one renderer's, for two back-to-back renders with different seeds;
  * bench.py --gpus n under torch.distributed.run (one process per GPU, ncclCommInitRank, rank 0's
    scene image broadcast over RCCL) and as one process (ncclCommInitAll): C4 is a fixed total launch
    (strong scaling), so both lines count exactly the 1-GPU line's ray-bounces per step.
The reference renders on one GPU (AudioRenderer.cpp:252); SURVEY.md §8e.
"""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from audiorenderingv2_amd import AudioRenderer, RenderGroup, RenderSettings, device_count, receiver_local
from audiorenderingv2_amd.scene import CONFERENCE_EMITTER, CONFERENCE_LISTENER
from conftest import REPO

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def n_gpus():
    n = device_count()
    if n < 2:
        pytest.skip(f"needs >= 2 GPUs (this box has {n}); the N>1 code's one-GPU shapes run in test_gpu_group.py")
    return n


def same(a, b):
    return np.array_equal(a[0].view(np.uint32), b[0].view(np.uint32)) and \
        np.array_equal(a[1].view(np.uint32), b[1].view(np.uint32))


C4 = dict(rays=(1000, 100, 100), sample_rate=48000, base_power=3.62, max_bounces=32, hrtf_absorption_rate=0.5)


def test_rccl_group_over_all_gpus_equals_one_renderer_c4(conference, n_gpus):
    s = RenderSettings(**C4)
    g = RenderGroup(s, devices=list(range(n_gpus)), scene=conference, receiver=receiver_local())
    r = AudioRenderer(s, scene=conference, receiver=receiver_local())
    try:
        assert g.n_ranks == n_gpus and len(g.members) == n_gpus
        for x in (g, r):
            x.setEmitterPosInOptix(CONFERENCE_EMITTER)
            x.setSphereCenterInOptix(CONFERENCE_LISTENER, 30.0)
        for seed in (1, 2):  # two back-to-back renders, the second on other rays
            g.set_seed(seed)
            r.set_seed(seed)
            g.render()
            r.render()
            ref = r.get_ir()
            assert ref[0].any()
            for m in g.members:  # every rank holds the reduced IR
                assert same(m.get_ir(), ref), (seed, m.settings.device)
            gs, rs = g.stats(), r.stats()
            assert (gs["queries"], gs["receiver_hits"], gs["misses"]) == (rs["queries"], rs["receiver_hits"],
                                                                          rs["misses"])
    finally:
        g.close()
        r.close()


def _bench(args, torchrun_ranks=0, timeout=600):
    cmd = [sys.executable]
    if torchrun_ranks:
        with socket.socket() as sk:
            sk.bind(("127.0.0.1", 0))
            port = sk.getsockname()[1]
        cmd += ["-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={torchrun_ranks}",
                "--master-addr=127.0.0.1", f"--master-port={port}"]
    cmd += [os.path.join(REPO, "bench.py"), *args, "--workload", "c4", "--steps", "2", "--warmup", "1",
            "--c5-frames", "0", "--no-cpu-baseline", "--no-streaming", "--no-pipelined"]
    res = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, cwd=REPO)
    assert res.returncode == 0, res.stderr[-4000:]
    lines = [ln for ln in res.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, res.stdout[-2000:]
    return json.loads(lines[0])


def test_bench_rank_path_and_local_group_count_the_one_gpu_launch(n_gpus):
    one = _bench(["--gpus", "1"])
    ranks = _bench(["--gpus", str(n_gpus)], torchrun_ranks=n_gpus)
    local = _bench(["--gpus", str(n_gpus)])
    assert one["n_gpus"] == 1 and ranks["n_gpus"] == n_gpus and local["n_gpus"] == n_gpus
    assert "ncclCommInitRank" in ranks["config"]["parallelism"]
    assert "ncclCommInitAll" in local["config"]["parallelism"]
    assert ranks["scaling"] == local["scaling"] == "strong"
    assert ranks["ray_bounces_per_step"] == local["ray_bounces_per_step"] == one["ray_bounces_per_step"]


def test_time_block_sharded_convolution_over_all_gpus(conference, n_gpus):
    """arx_group_convolute_device over distinct GPUs: every rank convolves its block pairs of the
    clapper file on its own device; the union of the ranks' frames is the one-GPU convolution."""
    from test_gpu_group_conv import assemble_and_check, one_gpu_conv, sharded
    from audiorenderingv2_amd.scene import reference_audio

    x, sr = reference_audio("clapper")
    s = RenderSettings(rays=(100, 100, 4), sample_rate=48000, base_power=3.62, max_bounces=16)
    g = RenderGroup(s, devices=list(range(n_gpus)), scene=conference, receiver=receiver_local())
    try:
        g.setEmitterPosInOptix(CONFERENCE_EMITTER)
        g.setSphereCenterInOptix(CONFERENCE_LISTENER, 0.0)
        g.render()
        assert g.conv_sharded
        ref = one_gpu_conv(g.get_ir(), sr, x)
        assemble_and_check(sharded(g, x), ref, x.size, whole_file=False)
    finally:
        g.close()
