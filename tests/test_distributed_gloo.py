"""The N>1 path's host side in real processes (world size 2 and 3, gloo for the collectives).

torch.distributed.run starts one process per rank, as it does for bench.py --gpus N on a GPU node;
each runs tests/dist_rank_worker.py: bench.py's plan_ranks and share_unique_ids (the launch-keyed id
file), libarx's rank-path scene hand-over (arx_debug_share_scene = arx_group_set_scene's protocol
over gloo instead of RCCL) including a failing rank 0, and the product's shard formula
(arx_group_shard, which arx_group_render uses) with an exact int64 all-reduce of the oracle's
per-shard histograms.
"""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from audiorenderingv2_amd import _lib
from conftest import REPO, world_scene


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_group_shard_partitions():
    import ctypes as C

    def shard(n, r, w):
        b, e = C.c_uint64(0), C.c_uint64(0)
        _lib.lib().arx_group_shard(n, r, w, C.byref(b), C.byref(e))
        return b.value, e.value

    for n in (0, 1, 7, 1000, 10**7, 2**62 + 3):
        for w in (1, 2, 3, 8):
            parts = [shard(n, r, w) for r in range(w)]
            assert parts[0][0] == 0 and parts[-1][1] == n
            assert all(parts[i][1] == parts[i + 1][0] for i in range(w - 1))
            assert max(e - b for b, e in parts) - min(e - b for b, e in parts) <= 1


@pytest.mark.parametrize("world", [2, 3])
def test_rank_plumbing_in_real_processes(tmp_path, world):
    env = dict(os.environ, OMP_NUM_THREADS="1", PYTHONPATH=REPO)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}",
           os.path.join(REPO, "tests", "dist_rank_worker.py"), str(tmp_path)]
    res = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    assert res.returncode == 0, res.stdout[-3000:] + res.stderr[-3000:]
    outs = [json.load(open(tmp_path / f"rank{r}.json")) for r in range(world)]
    for r, o in enumerate(outs):
        assert o["plan"] == {"mode": "rank", "world": world, "rank": r, "devices": [r], "local_gpus_needed": r + 1}
    # one launch, one id file, the same two ids on every rank; rank 0 removed the file afterwards
    assert len({o["uid_path"] for o in outs}) == 1 and not os.path.exists(outs[0]["uid_path"])
    assert all(o["ids"] == outs[0]["ids"] for o in outs) and len(set(outs[0]["ids"])) == 2
    # the scene reaches every rank as rank 0 built it
    for o in outs:
        assert o["share_ok"]["status"] == 0
        assert o["share_ok"]["hash"] == o["share_ok"]["local_hash"] == outs[0]["share_ok"]["hash"]
    # rank 0's input check fails: every rank returns an error (none waits in a collective)
    assert outs[0]["share_bad_root"]["status"] == 1 and "absorption" in outs[0]["share_bad_root"]["error"]
    for o in outs[1:]:
        assert o["share_bad_root"]["status"] != 0 and "rank 0" in o["share_bad_root"]["error"]
    # shards cover the launch; the all-reduced histogram is the single-process one, exactly
    import pyoracle as po
    from audiorenderingv2_amd.scene import conference_standin

    assert [o["shard"] for o in outs] == [[3000 * r // world, 3000 * (r + 1) // world] for r in range(world)]
    tv, ta = world_scene(conference_standin(), (5.0, 1.2, 2.0))
    p = po.make_params(rays=(30, 20, 5), sample_rate=16000, max_bounces=8, emitter=(-5, 1.2, 0), listener=(5, 1.2, 2))
    L, R, st = po.Scene(tv, ta, bvh=True).trace(p)
    assert np.array_equal(np.load(tmp_path / "hist.npy"), np.concatenate([L, R]))
    assert outs[0]["queries_all"] == st["queries"]
