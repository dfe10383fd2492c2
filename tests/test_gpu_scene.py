"""GPU: scene maintenance on the device and the guards around it.

  * the quantized node copy is made on the device (launch_requant16) from the coded f32 nodes and
    must equal quantize_nodes16's host arithmetic (restated here in numpy f64) word for word;
  * a listener walking off the quantization grid re-grids with one device re-quantization -- no
    host quantization or upload -- and the IR stays identical to a fresh renderer's;
  * a renderer group builds the scene tree once and shares it (arx_scene_build_count), with an IR
    bit-identical to a single renderer's;
  * the production trace kernel's register allocation admits exactly the waves per SIMD the
    persistent launch is sized for (hipFuncGetAttributes through arx_stats);
  * a streaming convolution outliving its renderer fails cleanly.
"""
import os
import re

import numpy as np
import pytest

from audiorenderingv2_amd import ArxError, AudioRenderer, LiveStream, RenderGroup, RenderSettings, receiver_local
from audiorenderingv2_amd import scene_build_count
from audiorenderingv2_amd.scene import CONFERENCE_EMITTER, CONFERENCE_LISTENER

pytestmark = pytest.mark.gpu

EMPTY_CODE = ~16  # kEmptyChildCode
# kQ16Margin, the outward rounding margin of QNode2 planes in grid steps (arx_layout.hpp)
Q16_MARGIN = float(re.search(r"constexpr double kQ16Margin = ([0-9.]+);",
                             open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                               "audiorenderingv2_amd", "csrc", "arx_layout.hpp")).read()).group(1))


def host_quantize(cn: np.ndarray, origin: np.ndarray, scale: np.ndarray) -> np.ndarray:
    """quantize_nodes16 (arx_bvh.cpp) over coded nodes given as n x 16 u32 words."""
    f = cn.view(np.float32)
    codes = cn[:, 12:14].view(np.int32)
    out = np.zeros((cn.shape[0], 8), np.uint32)
    o = origin.astype(np.float64)
    sc = scale.astype(np.float64)
    for c in range(2):
        ab = f[:, 0:4] if c == 0 else f[:, 4:8]
        lo = np.stack([ab[:, 0], ab[:, 2], f[:, 8 + 2 * c]], 1).astype(np.float64)
        hi = np.stack([ab[:, 1], ab[:, 3], f[:, 9 + 2 * c]], 1).astype(np.float64)
        ql = np.floor((lo - o) / sc - Q16_MARGIN)
        qh = np.ceil((hi - o) / sc + Q16_MARGIN)
        empty = (codes[:, c] == EMPTY_CODE)[:, None]
        ql = np.where(empty, 1, ql)
        qh = np.where(empty, 0, qh)
        assert (ql >= 0).all() and (qh <= 65535).all()
        out[:, 4 * c:4 * c + 3] = ql.astype(np.uint32) | (qh.astype(np.uint32) << 16)
        out[:, 4 * c + 3] = cn[:, 12 + c]
    return out


def renderer(scene, s, listener=CONFERENCE_LISTENER, yaw=0.0):
    r = AudioRenderer(s, scene=scene, receiver=receiver_local())
    r.setEmitterPosInOptix(CONFERENCE_EMITTER)
    r.setSphereCenterInOptix(listener, yaw)
    return r


S = RenderSettings(rays=(40, 40, 10), sample_rate=16000, base_power=3.62, max_bounces=8, hrtf_absorption_rate=0.5)


def test_device_requantization_equals_host_arithmetic(conference):
    r = renderer(conference, S)
    r.render()
    img = r.node_images()
    assert img["requants"] == 1
    ref = host_quantize(img["cnodes"], img["origin"], img["scale"])
    assert np.array_equal(img["qnodes"], ref)  # scene by the re-quantization, receiver by the refit
    r.close()


def test_walk_off_the_grid_requantizes_on_the_device(conference):
    """C5's walk: 0.05 m per frame along +x from the conference listener; once the receiver leaves
    the grid the grid grows, the quantized copy is re-made on the device, and every frame's IR
    equals a fresh renderer's at that pose."""
    r = renderer(conference, S)
    r.render()
    base = r.node_images()
    x0, y0, z0 = CONFERENCE_LISTENER
    grown_at = None
    for k in range(0, 1200, 25):
        pose = (x0 + 0.05 * k, y0, z0)
        r.setSphereCenterInOptix(pose, float(k % 360))
        r.render()
        img = r.node_images()
        if img["requants"] > base["requants"]:
            grown_at = k
            # the whole copy (scene re-quantized, receiver refit) follows the new grid, word for
            # word the host arithmetic
            assert not np.array_equal(img["origin"], base["origin"])
            ref = host_quantize(img["cnodes"], img["origin"], img["scale"])
            assert np.array_equal(img["qnodes"], ref)
            f = renderer(conference, S, listener=pose, yaw=float(k % 360))
            f.render()
            a, b = r.get_ir(), f.get_ir()
            assert np.array_equal(a[0].view(np.uint32), b[0].view(np.uint32))
            assert np.array_equal(a[1].view(np.uint32), b[1].view(np.uint32))
            f.close()
            break
    assert grown_at is not None, "the walk never left the grid"
    assert r.stats()["trace_format"] == 1  # still on the quantized nodes
    r.set_trace_path(8)  # and the CW4 copy, re-made for the new grid too, gives the same IR
    r.render()
    c = r.get_ir()
    assert r.stats()["trace_format"] == 2
    assert np.array_equal(c[0].view(np.uint32), a[0].view(np.uint32))
    assert np.array_equal(c[1].view(np.uint32), a[1].view(np.uint32))
    r.close()


def test_group_builds_the_scene_once(conference):
    """8 members, one build (none if an earlier test's renderer still holds this scene: the build
    cache); a renderer given the same geometry while the group holds it reuses the build too."""
    before = scene_build_count()
    g = RenderGroup(S, devices=[0] * 8, scene=conference, receiver=receiver_local())
    assert scene_build_count() - before <= 1
    after_group = scene_build_count()
    g.setEmitterPosInOptix(CONFERENCE_EMITTER)
    g.setSphereCenterInOptix(CONFERENCE_LISTENER, 0.0)
    g.render()
    hashes = {m.stats()["tree_hash"] for m in g.members}
    assert len(hashes) == 1
    r = renderer(conference, S)
    assert scene_build_count() == after_group
    r.render()
    a, b = g.get_ir(), r.get_ir()
    assert np.array_equal(a[0].view(np.uint32), b[0].view(np.uint32))
    assert np.array_equal(a[1].view(np.uint32), b[1].view(np.uint32))
    assert r.stats()["tree_hash"] in hashes  # the same deterministic build
    g.close()
    r.close()


def test_trace_kernel_occupancy_matches_launch_sizing(conference):
    r = renderer(conference, S)
    r.render()
    st = r.stats()
    assert st["trace_vgprs"] > 0
    assert st["trace_waves_per_simd"] == st["trace_waves_target"], (st["trace_vgprs"], st["trace_waves_per_simd"],
                                                                   st["trace_waves_target"])
    r.close()


def test_stream_outliving_its_renderer_fails_cleanly():
    s = RenderSettings(rays=(4, 4, 4), sample_rate=16000)
    r = AudioRenderer(s)
    st = LiveStream(r, 256)
    st.process(np.zeros(256))
    r.close()
    with pytest.raises(ArxError):
        st.process(np.zeros(256))
    st.close()  # detached: only the handle is freed
