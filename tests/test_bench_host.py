"""bench.py's host-side plumbing (no GPU): how --gpus N and the launcher's environment map to one
process driving N devices or one rank per process, the RCCL-id hand-off between the ranks of one
launch, the stored-profile guard, and the loud failure when the GPUs asked for are not there."""
import os
import subprocess
import sys
import threading

import pytest

from conftest import REPO

sys.path.insert(0, REPO)
import bench  # noqa: E402


def test_plain_run_drives_all_gpus_from_one_process():
    for n in (1, 2, 4, 8):
        p = bench.plan_ranks(n, {})
        assert p["mode"] == "local" and p["world"] == n and p["rank"] == 0
        assert p["devices"] == list(range(n)) and p["local_gpus_needed"] == n


def test_torchrun_ranks_take_one_gpu_each():
    for r in range(4):
        env = {"WORLD_SIZE": "4", "RANK": str(r), "LOCAL_RANK": str(r)}
        p = bench.plan_ranks(4, env)
        assert p == {"mode": "rank", "world": 4, "rank": r, "devices": [r], "local_gpus_needed": r + 1}
    # --process-group rehearses the rank path at one rank
    p = bench.plan_ranks(1, {}, process_group=True)
    assert p["mode"] == "rank" and p["world"] == 1 and p["devices"] == [0]


def test_inconsistent_requests_are_rejected():
    with pytest.raises(ValueError):
        bench.plan_ranks(0, {})
    with pytest.raises(ValueError):
        bench.plan_ranks(4, {"WORLD_SIZE": "8", "RANK": "0", "LOCAL_RANK": "0"})
    with pytest.raises(ValueError):
        bench.plan_ranks(2, {}, process_group=True)
    with pytest.raises(ValueError):
        bench.plan_ranks(8, {"WORLD_SIZE": "8", "RANK": "9", "LOCAL_RANK": "0"})


def test_unique_id_reaches_every_rank_of_one_launch(tmp_path, monkeypatch):
    monkeypatch.setattr(bench.tempfile, "gettempdir", lambda: str(tmp_path))
    env = {"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": "29555", "TORCHELASTIC_RUN_ID": "t"}
    uid = bytes(range(128))
    got = {}

    def rank(r):
        got[r] = bench.share_unique_id(r, 4, env, lambda: uid, timeout_s=30)

    ts = [threading.Thread(target=rank, args=(r,)) for r in (3, 2, 1)]  # the others wait for rank 0
    for t in ts:
        t.start()
    rank(0)
    for t in ts:
        t.join()
    assert all(got[r] == uid for r in range(4))
    assert os.path.exists(bench.uid_path(env))
    # another launch (other port) never reads this one's id
    other = dict(env, MASTER_PORT="29556")
    assert bench.uid_path(other) != bench.uid_path(env)
    with pytest.raises(SystemExit):
        bench.share_unique_id(1, 2, other, lambda: uid, timeout_s=0.2)
    assert bench.share_unique_id(0, 1, env, lambda: uid) is None  # one rank needs no id


def test_profile_guard():
    from audiorenderingv2_amd._lib import lib
    kid = f"{int(lib().arx_trace_kernel_id()):016x}"
    st = {"tree_hash": 0xABC, "trace_vgprs": 88}
    good = {"workload": "c3", "tree_hash": "0000000000000abc", "trace_vgprs": 88, "trace_kernel_id": kid,
            "bytes_per_launch": 1.0}
    assert bench.profile_guard(good, "c3", st)[0] is good
    assert bench.profile_guard(good, "c2", st)[0] is None
    assert bench.profile_guard(dict(good, tree_hash="0000000000000abd"), "c3", st)[0] is None
    p, why = bench.profile_guard(dict(good, trace_vgprs=80), "c3", st)
    assert p is None and "trace_vgprs" in why
    p, why = bench.profile_guard(dict(good, trace_kernel_id="0123456789abcdef"), "c3", st)
    assert p is None and "trace_kernel_id" in why  # another kernel's counters, same tree and VGPRs
    assert bench.profile_guard(None, "c3", st) == (None, "missing")


def test_more_gpus_than_visible_fails_loudly():
    """On a box without the GPUs asked for, bench exits non-zero and prints no JSON line."""
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "64"], capture_output=True,
                       text=True, timeout=120, env=env)
    assert p.returncode != 0
    assert p.stdout.strip() == ""
    assert "--gpus 64" in p.stderr


def test_steps_beyond_the_timing_ring_are_refused():
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--steps", "100000"], capture_output=True,
                       text=True, timeout=120)
    assert p.returncode != 0 and "--steps" in p.stderr and p.stdout.strip() == ""


class _FakeGroup:
    """A group stand-in that records the f64 all-reduces bench.Ranks issues."""

    def __init__(self, n_ranks):
        self.n_ranks = n_ranks
        self.calls = []

    def allreduce(self, values, op="sum"):
        self.calls.append((list(values), op))
        return list(values)


def test_ranks_issue_collectives_only_across_processes_unless_forced():
    # one process (plain run, or one rank): barrier / max / sum stay local
    for mode, n in (("local", 1), ("local", 8), ("rank", 1)):
        g = _FakeGroup(n)
        r = bench.Ranks(g, mode)
        r.barrier()
        assert r.max(2.5) == 2.5 and r.sum(3.0) == 3.0 and g.calls == []
    # ranks of a multi-process launch, and any group with --debug-force-collectives, go through RCCL
    for mode, n, forced in (("rank", 2, False), ("local", 1, True), ("rank", 1, True)):
        g = _FakeGroup(n)
        r = bench.Ranks(g, mode, forced)
        r.barrier()
        r.max(1.0)
        r.sum(1.0)
        assert [op for _, op in g.calls] == ["sum", "max", "sum"]


def test_watchdog_fires_once_without_progress_and_not_while_beating():
    import io
    import json
    import time

    out, codes = io.StringIO(), []
    wd = bench.Watchdog(0, 8, out=out, on_hang=codes.append, poll_s=0.05)
    wd.info["frames_in_flight"] = 1
    wd.arm(0.4, "timed")
    for _ in range(12):  # beats keep it quiet
        time.sleep(0.1)
        wd.beat(step=True)
    assert codes == [] and out.getvalue() == ""
    wd.disarm()
    time.sleep(0.6)  # disarmed: quiet
    assert codes == []
    wd.arm(0.2, "moving_listener")
    time.sleep(0.8)
    assert codes == [3]
    d = json.loads(out.getvalue())
    assert d["status"] == "hang" and d["phase"] == "moving_listener" and d["rank"] == 0 and d["world"] == 8
    assert d["steps_done"] == 12 and d["frames_in_flight"] == 1 and d["seconds_since_progress"] >= 0.2


def test_oversubscribed_rehearsal_plan():
    p = bench.plan_ranks(4, {}, oversubscribe=True)
    assert p == {"mode": "local", "world": 4, "rank": 0, "devices": [0, 0, 0, 0], "local_gpus_needed": 1}


def test_watchdog_of_another_rank_reports_on_stderr(capsys):
    import io
    import time

    out, codes = io.StringIO(), []
    wd = bench.Watchdog(3, 8, out=out, on_hang=codes.append, poll_s=0.05)
    wd.arm(0.1, "timed")
    time.sleep(0.5)
    assert codes == [3] and out.getvalue() == ""  # stdout keeps rank 0's line alone
    assert '"rank": 3' in capsys.readouterr().err
