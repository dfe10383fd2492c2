"""GPU: ray-sharded multi-GPU groups through the C ABI (arx_group_*, native RCCL).

The single-GPU box runs every group shape the product supports on one MI355X:
  * a one-GPU RCCL group (ncclCommInitAll over [0]) and a one-rank ncclCommInitRank group -- the
    all-reduce path the 8-GPU node takes, at size 1;
  * oversubscribed groups (device 0 listed G times): G shards of the launch, summed on the device.
Bar: the group's IR is bit-identical to the single-renderer launch (and to the CPU oracle on
sampled ray ranges) -- the int64 histogram sum is exact, so the result cannot depend on G.

configs[3] (C4: conference, 10 M rays x 32 bounces, 48 kHz, ray-sharded over 8 GPUs with an
RCCL IR reduce) is run here as 8 shards on one GPU.
"""
import numpy as np
import pytest

import pyoracle as po
from audiorenderingv2_amd import AudioRenderer, RenderGroup, RenderSettings, receiver_local
from audiorenderingv2_amd.scene import CONFERENCE_EMITTER, CONFERENCE_LISTENER
from conftest import world_scene

pytestmark = pytest.mark.gpu


def make_group(scene, settings, devices, listener=CONFERENCE_LISTENER, emitter=CONFERENCE_EMITTER, yaw=0.0):
    g = RenderGroup(settings, devices=devices, scene=scene, receiver=receiver_local())
    g.setEmitterPosInOptix(emitter)
    g.setSphereCenterInOptix(listener, yaw)
    return g


def single(scene, settings, listener=CONFERENCE_LISTENER, emitter=CONFERENCE_EMITTER, yaw=0.0):
    r = AudioRenderer(settings, scene=scene, receiver=receiver_local())
    r.setEmitterPosInOptix(emitter)
    r.setSphereCenterInOptix(listener, yaw)
    return r


def same(a, b):
    return np.array_equal(a[0].view(np.uint32), b[0].view(np.uint32)) and \
        np.array_equal(a[1].view(np.uint32), b[1].view(np.uint32))


def test_rccl_group_of_one_gpu_equals_renderer(conference):
    s = RenderSettings(rays=(100, 100, 10), sample_rate=48000, base_power=3.62, max_bounces=16, hrtf_absorption_rate=0.5)
    r = single(conference, s)
    r.render()
    ref, st = r.get_ir(), r.stats()
    g = make_group(conference, s, [0])
    assert g.n_ranks == 1 and len(g.members) == 1
    ms = g.render()
    assert ms > 0
    assert same(g.get_ir(), ref)
    gst = g.stats()
    assert (gst["queries"], gst["receiver_hits"], gst["misses"]) == (st["queries"], st["receiver_hits"], st["misses"])
    # the member renderer is a full renderer: its IR is the group's
    assert same(g.member(0).get_ir(), ref)


def test_rank_group_single_process(conference):
    s = RenderSettings(rays=(40, 40, 10), sample_rate=16000, base_power=3.62, max_bounces=8)
    r = single(conference, s)
    r.render()
    ref = r.get_ir()
    uid = RenderGroup.unique_id()
    assert len(uid) == 128
    for u in (uid, None):  # a one-rank group needs no shared id
        g = RenderGroup.rank(s, 1, 0, u, scene=conference, receiver=receiver_local())
        g.setEmitterPosInOptix(CONFERENCE_EMITTER)
        g.setSphereCenterInOptix(CONFERENCE_LISTENER, 0.0)
        g.render()
        assert same(g.get_ir(), ref)
        g.close()


@pytest.mark.parametrize("n", [2, 3, 5])
def test_oversubscribed_group_shards_exact(conference, n):
    s = RenderSettings(rays=(50, 40, 10), sample_rate=16000, base_power=3.62, max_bounces=8, hrtf_absorption_rate=0.25)
    lst, yaw = (3.0, 1.5, -1.0), 40.0
    r = single(conference, s, listener=lst, yaw=yaw)
    r.render()
    ref = r.get_ir()
    g = make_group(conference, s, [0] * n, listener=lst, yaw=yaw)
    assert g.n_ranks == n
    g.render()
    assert same(g.get_ir(), ref)
    for m in g.members:  # every member holds the full IR after the reduce
        assert same(m.get_ir(), ref)
    # setters reach every member; a listener move re-renders identically to a fresh renderer
    g.setSphereCenterInOptix((1.0, 1.2, 0.5), 300.0)
    g.render()
    f = single(conference, s, listener=(1.0, 1.2, 0.5), yaw=300.0)
    f.render()
    assert same(g.get_ir(), f.get_ir())


def test_oversubscribed_group_back_to_back_renders(conference):
    """Two renders with different seeds issued without a host synchronisation in between: the
    second render's clears must not overtake the first one's histogram copies (every member
    must end with exactly the second launch's IR)."""
    s = RenderSettings(rays=(50, 40, 10), sample_rate=16000, base_power=3.62, max_bounces=8, hrtf_absorption_rate=0.25)
    refs = {}
    for seed in (11, 12):
        r = single(conference, RenderSettings(**{**s.__dict__, "seed": seed}))
        r.render()
        refs[seed] = r.get_ir()
        r.close()
    assert not same(refs[11], refs[12])
    g = make_group(conference, s, [0] * 4)
    for _ in range(3):
        g.set_seed(11)
        g.render(timed=False)
        g.set_seed(12)
        g.render(timed=False)
        g.synchronize()
        for m in g.members:
            assert same(m.get_ir(), refs[12])
    g.close()


def test_group_rejects_mixed_device_lists():
    from audiorenderingv2_amd import ArxError

    s = RenderSettings(rays=(4, 4, 4), sample_rate=16000)
    with pytest.raises(ArxError):
        RenderGroup(s, devices=[0, 0, 1])


C4 = RenderSettings(rays=(1000, 100, 100), sample_rate=48000, base_power=3.62, max_bounces=32, hrtf_absorption_rate=1.0)


def test_c4_sharded_group(conference):
    """configs[3]: 10 M rays x 32 bounces at 48 kHz, as 8 ray shards (device 0 x 8) summed on the
    device: bit-identical to the single launch, deterministic, bounded by the 32-bounce cap, and
    equal to the oracle on ray-id samples at the start and the end of the launch."""
    n = 1000 * 100 * 100
    r = single(conference, C4)
    r.render()
    ref, st = r.get_ir(), r.stats()
    assert 20 * n < st["queries"] <= 32 * n  # a query per reflection while depth < 32 (devicePrograms.cu:233-236)
    assert st["receiver_hits"] > 10000
    g = make_group(conference, C4, [0] * 8)
    g.render()
    a = g.get_ir()
    assert same(a, ref)
    assert g.stats()["queries"] == st["queries"]
    g.render()
    assert same(g.get_ir(), a)  # deterministic
    g.close()
    # oracle on sampled ray ranges of the same 10 M-ray launch
    tv, ta = world_scene(conference, CONFERENCE_LISTENER, 0.0)
    osc = po.Scene(tv, ta, bvh=True)
    p = po.make_params(rays=C4.rays, sample_rate=48000, base_power=3.62, max_bounces=32, hrtf=1.0,
                       emitter=CONFERENCE_EMITTER, listener=CONFERENCE_LISTENER)
    for b, e in ((0, 3000), (n - 3000, n)):
        r.clear_histogram()
        r.trace_rays(b, e)
        r.finalize_ir()
        L, R, ost = osc.trace(p, b, e, threads=8)
        ol, orr = po.finalize_ir(p, L, R)
        assert r.stats()["queries"] == ost["queries"]
        assert same(r.get_ir(), (ol, orr)), (b, e)
