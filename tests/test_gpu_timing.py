"""GPU: per-launch timing on and off (arx_set_timing / arx_group_set_timing).

Each timed launch puts two event markers on the renderer's stream (~4.5 us of stream time apiece on
MI355X, tools/step_gaps.py); with timing off the same launches go to the stream alone.  Off must
change nothing but the rings: the same IR and convolution output bit for bit, no new entries in
trace_times / conv_times, while a call that asks for its own time (render() with render_ms, the
host-buffer convolution with convolute_ms, a group render with timed=True) is still timed, as the
reference times render() only when render_ms is given (AudioRenderer.h:27)."""
import numpy as np
import pytest

from audiorenderingv2_amd import AudioRenderer, RenderGroup, RenderSettings, receiver_local
from audiorenderingv2_amd._lib import check, lib
from audiorenderingv2_amd.renderer import DeviceBuffer
from audiorenderingv2_amd.scene import CONFERENCE_EMITTER, CONFERENCE_LISTENER

pytestmark = pytest.mark.gpu

S = dict(rays=(60, 60, 10), sample_rate=16000, base_power=3.62, max_bounces=8, hrtf_absorption_rate=0.5)


def bits(a):
    return np.asarray(a).view(np.uint32)


def test_renderer_timing_off_changes_only_the_rings(conference):
    r = AudioRenderer(RenderSettings(**S), scene=conference, receiver=receiver_local())
    x = (0.3 * np.sin(np.arange(40000) * 0.01)).astype(np.float32)
    dx = DeviceBuffer.from_numpy(0, x)
    outs = [DeviceBuffer(0, x.nbytes) for _ in range(4)]
    try:
        r.setEmitterPosInOptix(CONFERENCE_EMITTER)
        r.setSphereCenterInOptix(CONFERENCE_LISTENER, 0.0)
        assert r.render() > 0.0  # timed (default on)
        ir_on = r.get_ir()
        r.convolute_device(dx.ptr, x.size, outs[0].ptr, outs[1].ptr)
        r.stats()
        n_trace, n_conv = len(r.trace_times(256)), len(r.conv_times(256))
        assert n_trace == 1 and n_conv == 1
        r.set_timing(False)
        check(lib().arx_render(r.handle, None))  # no time asked for: no events
        r.convolute_device(dx.ptr, x.size, outs[2].ptr, outs[3].ptr)
        r.stats()
        assert len(r.trace_times(256)) == n_trace and len(r.conv_times(256)) == n_conv
        ir_off = r.get_ir()
        assert np.array_equal(bits(ir_on[0]), bits(ir_off[0])) and np.array_equal(bits(ir_on[1]), bits(ir_off[1]))
        for a, b in ((outs[0], outs[2]), (outs[1], outs[3])):
            assert np.array_equal(bits(a.to_numpy(np.float32, x.size)), bits(b.to_numpy(np.float32, x.size)))
        # calls that ask for their time are timed either way
        assert r.render() > 0.0 and len(r.trace_times(256)) == n_trace + 1
        _, _, conv_ms, proc_ms = r.convoluteAudioFile(x)
        assert conv_ms > 0.0 and proc_ms >= conv_ms and len(r.conv_times(256)) == n_conv + 1
        r.set_timing(True)
        check(lib().arx_render(r.handle, None))
        r.stats()
        assert len(r.trace_times(256)) == n_trace + 2
    finally:
        for b in [dx, *outs]:
            b.close()
        r.close()


def test_group_timing_off(conference):
    g = RenderGroup(RenderSettings(**S), devices=[0], scene=conference, receiver=receiver_local())
    try:
        g.setEmitterPosInOptix(CONFERENCE_EMITTER)
        g.setSphereCenterInOptix(CONFERENCE_LISTENER, 0.0)
        g.set_timing(False)
        g.set_frames_in_flight(2)
        for _ in range(3):
            g.render(timed=False)
        g.synchronize()
        m = g.member(0)
        assert len(m.trace_times(256)) == 0
        assert g.render(timed=True) > 0.0 and len(m.trace_times(256)) == 1
    finally:
        g.close()
