"""GPU: time-block sharded file convolution over a group (arx_group_convolute_device, SURVEY.md §8e:
"time blocks sharded ... only the n - sr overlap is summed at shard seams"; the reference's block
loop is kernels.cu:404-430, one GPU).

Bar: the union of the ranks' output frames (arx_group_conv_shard) is bit-identical to the one-GPU
convolution (arx_convolute_device) of the same file with the same IR -- which is itself within
1 ULP(max) of the f64 oracle (tests/test_gpu_parity.py, tests/test_gpu_full_launch.py).  Shapes:
oversubscribed groups (device 0 listed G times, G shards), more ranks than block pairs (empty
shards), a forced one-rank RCCL group, and a plan without the chained pass (every rank convolves
the whole file).
"""
import ctypes as C

import numpy as np
import pytest

from audiorenderingv2_amd._lib import check, lib
from audiorenderingv2_amd import AudioRenderer, DeviceBuffer, RenderGroup, RenderSettings, receiver_local
from audiorenderingv2_amd.scene import CONFERENCE_EMITTER, CONFERENCE_LISTENER, reference_audio

pytestmark = pytest.mark.gpu


def rendered_group(conference, s, devices, force=False):
    g = RenderGroup(s, devices=devices, scene=conference, receiver=receiver_local())
    if force:
        g.debug_force_collectives(True, True)
    g.setEmitterPosInOptix(CONFERENCE_EMITTER)
    g.setSphereCenterInOptix(CONFERENCE_LISTENER, 0.0)
    g.render()
    return g


def one_gpu_conv(ir, sr, x):
    r = AudioRenderer(RenderSettings(rays=(1, 1, 1), sample_rate=sr, ir_length_in_seconds=2))
    r.set_ir(*ir)
    L, R, _, _ = r.convoluteAudioFile(x)
    r.close()
    return L, R


def sharded(g, x):
    """Run the group's sharded convolution; per rank: (begin, end, L, R) of its full-length outputs."""
    bufs = []
    for m in g.members:
        d = m.settings.device
        out_l, out_r = DeviceBuffer(d, 4 * x.size), DeviceBuffer(d, 4 * x.size)
        nan = np.full(x.size, np.nan, np.float32)
        for b in (out_l, out_r):  # frames a rank does not own must stay untouched
            check(lib().arx_memcpy(d, C.c_void_p(b.ptr), nan.ctypes.data_as(C.c_void_p), nan.nbytes))
        bufs.append((DeviceBuffer.from_numpy(d, x), out_l, out_r))
    g.convolute_device([b[0].ptr for b in bufs], x.size, [b[1].ptr for b in bufs], [b[2].ptr for b in bufs])
    g.synchronize()
    res = []
    for i, (xin, ol, orr) in enumerate(bufs):
        b, e = g.conv_shard(x.size, i)
        res.append((b, e, ol.to_numpy(np.float32, x.size), orr.to_numpy(np.float32, x.size)))
        for buf in (xin, ol, orr):
            buf.close()
    return res


def assemble_and_check(res, ref, x_size, whole_file):
    L, R = np.full(x_size, np.nan, np.float32), np.full(x_size, np.nan, np.float32)
    cursor = 0
    for b, e, ol, orr in res:
        assert b == cursor or (b == e), (b, e, cursor)  # the ranks' ranges tile [0, n) in rank order
        cursor = max(cursor, e)
        L[b:e], R[b:e] = ol[b:e], orr[b:e]
        if whole_file:  # a plan without the chained pass: every rank wrote the whole file
            assert np.array_equal(ol.view(np.uint32), ref[0].view(np.uint32))
        else:  # a rank writes exactly its frames
            outside = np.ones(x_size, bool)
            outside[b:e] = False
            assert np.isnan(ol[outside]).all() and np.isnan(orr[outside]).all()
    assert cursor == x_size
    assert np.array_equal(L.view(np.uint32), ref[0].view(np.uint32))
    assert np.array_equal(R.view(np.uint32), ref[1].view(np.uint32))


@pytest.mark.parametrize("n", [2, 3, 4, 8, 11])
def test_c3_clapper_sharded_bit_identical(conference, n):
    """C3's audio (A_Clapper_Board.wav ch 0, 807 498 frames at 48 kHz = 16 blocks = 8 pairs + a tail)
    over n oversubscribed ranks (11: three ranks own no pair)."""
    x, sr = reference_audio("clapper")
    s = RenderSettings(rays=(100, 100, 4), sample_rate=48000, base_power=3.62, max_bounces=16)
    g = rendered_group(conference, s, [0] * n)
    assert g.conv_sharded
    ref = one_gpu_conv(g.get_ir(), sr, x)
    res = sharded(g, x)
    assert sum(e - b for b, e, _, _ in res) == x.size
    assemble_and_check(res, ref, x.size, whole_file=False)
    g.close()


@pytest.mark.parametrize("n", [3, 4])
def test_c2_experimento_sharded_bit_identical(conference, n):
    """C2's audio (experimento_entrada_16KHz.wav, 128 000 frames at 16 kHz = 8 blocks = 4 pairs)."""
    x, sr = reference_audio("experimento")
    s = RenderSettings(rays=(100, 100, 4), sample_rate=16000, base_power=3.62, max_bounces=8)
    g = rendered_group(conference, s, [0] * n)
    ref = one_gpu_conv(g.get_ir(), sr, x)
    assemble_and_check(sharded(g, x), ref, x.size, whole_file=False)
    g.close()


def test_forced_one_rank_group_owns_the_whole_file(conference):
    x, sr = reference_audio("clapper")
    s = RenderSettings(rays=(100, 100, 4), sample_rate=48000, base_power=3.62, max_bounces=16)
    g = rendered_group(conference, s, [0], force=True)
    assert g.conv_shard(x.size, 0) == (0, x.size)
    ref = one_gpu_conv(g.get_ir(), sr, x)
    assemble_and_check(sharded(g, x), ref, x.size, whole_file=False)
    g.close()


def test_unsharded_plan_convolves_whole_file_on_every_rank(conference):
    """44.1 kHz: n = 88200 = 315 x 280 (N1 odd, no chained pass): every rank convolves the whole file."""
    rng = np.random.default_rng(5)
    x = (0.3 * rng.standard_normal(5 * 44100 + 99)).astype(np.float32)
    s = RenderSettings(rays=(40, 40, 4), sample_rate=44100, base_power=3.62, max_bounces=8)
    g = rendered_group(conference, s, [0] * 3)
    assert not g.conv_sharded
    ref = one_gpu_conv(g.get_ir(), 44100, x)
    assemble_and_check(sharded(g, x), ref, x.size, whole_file=True)
    g.close()


def test_short_file_and_ragged_tails(conference):
    """Files shorter than one block (the reference's output stays zero) and odd block counts."""
    s = RenderSettings(rays=(40, 40, 4), sample_rate=16000, base_power=3.62, max_bounces=8)
    g = rendered_group(conference, s, [0] * 3)
    rng = np.random.default_rng(9)
    for n_frames in (9000, 16000, 3 * 16000 + 5, 5 * 16000, 7 * 16000 + 15999):
        # a fresh IR on every member (the IR spectra are made with the first convolution after it, by
        # the same fused pass as the one-GPU reference's; a file shorter than a block makes them in a
        # pass of their own, whose rounding differs, and they are then kept)
        g.render()
        x = rng.standard_normal(n_frames).astype(np.float32)
        ref = one_gpu_conv(g.get_ir(), 16000, x)
        assemble_and_check(sharded(g, x), ref, x.size, whole_file=False)
    g.close()


def test_allreduce_times_forced_one_rank(conference):
    """The histogram all-reduce's own HIP-event window (arx_group_allreduce_times): recorded with
    timing on, on a forced one-rank RCCL group (the collective path a multi-GPU node takes)."""
    s = RenderSettings(rays=(40, 40, 4), sample_rate=48000, base_power=3.62, max_bounces=8)
    g = RenderGroup(s, devices=[0], scene=conference, receiver=receiver_local())
    g.setEmitterPosInOptix(CONFERENCE_EMITTER)
    g.setSphereCenterInOptix(CONFERENCE_LISTENER, 0.0)
    g.set_timing(False)
    g.render(timed=False)
    assert g.allreduce_times(8).size == 0  # one rank, not forced: no all-reduce
    g.debug_force_collectives(True, False)
    g.set_timing(True)
    for _ in range(5):
        g.render(timed=False)
    t = g.allreduce_times(16)
    assert t.size == 5 and np.all(t > 0) and np.all(t < 50.0)
    assert g.debug_collectives()["histogram_allreduce"] == 5
    g.close()


@pytest.mark.parametrize("devices,sr,audio", [([0] * 3, 48000, "clapper"), ([0] * 5, 16000, "experimento"),
                                              ([0], 48000, "clapper")])
def test_group_convolute_audio_file_equals_one_renderer(conference, devices, sr, audio):
    """arx_group_convolute_audio_file (the C++ shim's convoluteAudioFile on a group): host buffers in
    and out, each member convolving its shard; bit-identical to one renderer's convoluteAudioFile,
    for the reference's own recordings and for files shorter than a block or with a ragged tail."""
    x, xsr = reference_audio(audio)
    assert xsr == sr
    s = RenderSettings(rays=(100, 100, 4), sample_rate=sr, base_power=3.62, max_bounces=8)
    g = rendered_group(conference, s, devices)
    rng = np.random.default_rng(4)
    for sig in (x, x[: sr // 2], x[: 3 * sr + 17], rng.standard_normal(6 * sr).astype(np.float32)):
        g.render()  # a new IR: both sides make the spectra with their first convolution
        L, R, cms, pms = g.convoluteAudioFile(sig)
        ref = one_gpu_conv(g.get_ir(), sr, sig)
        assert np.array_equal(L.view(np.uint32), ref[0].view(np.uint32))
        assert np.array_equal(R.view(np.uint32), ref[1].view(np.uint32))
        assert pms > 0 and cms > 0
    g.close()
