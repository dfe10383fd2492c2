"""N>1 path on CPU: ray shards + exact int64 all-reduce (gloo, world size 2 and 3).

The per-rank partial histograms come from the CPU oracle (standing in for each GPU's
trace kernel, which is bit-identical to it -- tests/test_gpu_parity.py); what is under
test is the product's sharding (shard_range) and reduction (allreduce_histogram).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from audiorenderingv2_amd.distributed import allreduce_histogram, max_over_ranks, shard_range, sum_over_ranks


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_shard_range_partitions():
    for n in (0, 1, 7, 1000, 10**7):
        for w in (1, 2, 3, 8):
            parts = [shard_range(n, r, w) for r in range(w)]
            assert parts[0][0] == 0 and parts[-1][1] == n
            assert all(parts[i][1] == parts[i + 1][0] for i in range(w - 1))
            assert max(e - b for b, e in parts) - min(e - b for b, e in parts) <= 1
    with pytest.raises(ValueError):
        shard_range(10, 2, 2)


def _worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import sys

    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "oracle"))
    sys.path.insert(0, os.path.dirname(__file__))
    import pyoracle as po
    from audiorenderingv2_amd.scene import conference_standin
    from conftest import world_scene

    scene = conference_standin()
    tv, ta = world_scene(scene, (5.0, 1.2, 2.0))
    osc = po.Scene(tv, ta, bvh=True)
    p = po.make_params(rays=(30, 20, 5), sample_rate=16000, max_bounces=8, emitter=(-5, 1.2, 0),
                       listener=(5, 1.2, 2))
    n = 30 * 20 * 5
    b, e = shard_range(n, rank, world)
    L, R, st = osc.trace(p, b, e)
    hist = torch.from_numpy(np.concatenate([L, R]))
    allreduce_histogram(hist)
    q = sum_over_ranks(st["queries"])
    m = max_over_ranks(float(rank))
    if rank == 0:
        np.save(os.path.join(out_dir, f"hist_w{world}.npy"), hist.numpy())
        np.save(os.path.join(out_dir, f"q_w{world}.npy"), np.array([q, m]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_allreduce_is_exact(tmp_path, world):
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    import pyoracle as po
    from audiorenderingv2_amd.scene import conference_standin
    from conftest import world_scene

    tv, ta = world_scene(conference_standin(), (5.0, 1.2, 2.0))
    p = po.make_params(rays=(30, 20, 5), sample_rate=16000, max_bounces=8, emitter=(-5, 1.2, 0),
                       listener=(5, 1.2, 2))
    L, R, st = po.Scene(tv, ta, bvh=True).trace(p)
    got = np.load(tmp_path / f"hist_w{world}.npy")
    assert np.array_equal(got, np.concatenate([L, R]))
    q, m = np.load(tmp_path / f"q_w{world}.npy")
    assert q == st["queries"] and m == world - 1
