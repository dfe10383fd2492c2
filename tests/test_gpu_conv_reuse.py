"""GPU: input reuse for the reference's re-render pattern (arx_convolute_prepare_input / _prepared).

The reference convolves the SAME audio file with every new IR (full_render_cycle,
AudioRenderer.cpp:790-798, driven by main.cpp:40-67 on each listener move).  Preparing the input
transforms its one-second blocks once; each later convolution then costs the new IR's spectra, the
products, the inverse rows and the inverse columns only.  The arithmetic is the same as
arx_convolute_device's, in the same order, so the bar is bit-identity with it (itself <= 1 ULP(max)
of the f64 oracle, test_gpu_parity.py) -- checked here for a sequence of IRs, with the IR changed
and unchanged between calls, at C3's size (the chained pass C) and on plans without it (the kept
copy of the input), and against the oracle once.
"""
import numpy as np
import pytest

import pyoracle as po
from audiorenderingv2_amd import ArxError, AudioRenderer, DeviceBuffer, RenderSettings

pytestmark = pytest.mark.gpu


def sparse_ir(n, rng, k=300, scale=1e-4):
    ir = np.zeros(n, np.float32)
    ir[rng.integers(0, n, k)] = rng.exponential(scale, k).astype(np.float32)
    return ir


def bits(a):
    return np.asarray(a).view(np.uint32)


def fetch(r, a, b, n):
    r.stats()  # synchronises the renderer's stream (the device buffers are read on the null stream)
    return a.to_numpy(np.float32, n), b.to_numpy(np.float32, n)


@pytest.mark.parametrize("sr,secs,length,plan", [
    (48000, 2, 807498, "direct"),      # C3: A_Clapper_Board's length, 300 x 320, chained pass C
    (16000, 2, 128000 + 77, "direct"),  # C2: experimento's length (+ a ragged tail)
    (16000, 1, 70000, "copy"),          # ir_len = sr: no chained pass C, the kept copy
    (1100, 2, 6000, "copy"),            # power-of-two plan
])
def test_prepared_equals_device_convolution(sr, secs, length, plan):
    rng = np.random.default_rng(sr + length)
    n = sr * secs
    x = (0.3 * rng.standard_normal(length)).astype(np.float32)
    r = AudioRenderer(RenderSettings(rays=(1, 1, 1), sample_rate=sr, ir_length_in_seconds=secs))
    dx = DeviceBuffer.from_numpy(0, x)
    bufs = [DeviceBuffer(0, x.nbytes) for _ in range(4)]
    try:
        irs = [(sparse_ir(n, rng), sparse_ir(n, rng)) for _ in range(3)]
        # reference outputs: convolute_device per IR
        want = []
        for irl, irr in irs:
            r.set_ir(irl, irr)
            r.convolute_device(dx.ptr, x.size, bufs[0].ptr, bufs[1].ptr)
            want.append(fetch(r, bufs[0], bufs[1], x.size))
        r.convolute_prepare_input(dx.ptr, x.size)
        r.stats()
        # the caller may overwrite its input once it is prepared
        import audiorenderingv2_amd._lib as L_
        z = np.zeros(x.size, np.float32)
        L_.check(L_.lib().arx_memcpy(0, dx.ptr, z.ctypes.data, z.nbytes))
        for k, (irl, irr) in enumerate(irs):
            r.set_ir(irl, irr)  # a new IR: its spectra folded into the prepared run
            assert r.convolute_prepared(bufs[2].ptr, bufs[3].ptr) == x.size
            got = fetch(r, bufs[2], bufs[3], x.size)
            assert np.array_equal(bits(got[0]), bits(want[k][0])) and np.array_equal(bits(got[1]), bits(want[k][1])), k
            # the same IR again: the stored spectra
            r.convolute_prepared(bufs[2].ptr, bufs[3].ptr)
            again = fetch(r, bufs[2], bufs[3], x.size)
            assert np.array_equal(bits(again[0]), bits(want[k][0])) and np.array_equal(bits(again[1]), bits(want[k][1]))
        assert want[0][0].any() and not np.array_equal(want[0][0], want[1][0])
        # against the oracle once (the last IR)
        for got, ir in ((again[0], irs[-1][0]), (again[1], irs[-1][1])):
            ref = po.convolute_audio(x, sr, ir)
            assert np.abs(got - ref).max() <= np.spacing(np.float32(np.abs(ref).max()))
        if plan == "direct":
            assert r.conv_plan().startswith("mixed-radix direct circular")
        # any other file convolution on the renderer discards the prepared input
        r.convolute_device(dx.ptr, x.size, bufs[0].ptr, bufs[1].ptr)
        with pytest.raises(ArxError):
            r.convolute_prepared(bufs[2].ptr, bufs[3].ptr)
    finally:
        for b in [dx, *bufs]:
            b.close()
        r.close()


def test_prepared_short_input_and_nothing_prepared():
    r = AudioRenderer(RenderSettings(rays=(1, 1, 1), sample_rate=16000))
    out = [DeviceBuffer(0, 4 * 1000) for _ in range(2)]
    x = DeviceBuffer.from_numpy(0, np.ones(1000, np.float32))
    try:
        with pytest.raises(ArxError):  # nothing prepared yet
            r.convolute_prepared(out[0].ptr, out[1].ptr)
        r.set_ir(np.ones(32000, np.float32), np.ones(32000, np.float32))
        r.convolute_prepare_input(x.ptr, 1000)  # shorter than one block: the output stays zero
        assert r.convolute_prepared(out[0].ptr, out[1].ptr) == 1000
        a, b = fetch(r, out[0], out[1], 1000)
        assert not a.any() and not b.any()
    finally:
        for b in [x, *out]:
            b.close()
        r.close()


@pytest.mark.parametrize("sr", [48000, 16000, 44100])
def test_ir_spectra_are_the_same_bits_whichever_call_made_them(sr):
    """The IR spectra come out of one route -- the packed IR through pass A's IR batch and pass B's
    mirror-row split -- whether a file convolution made them with its own first pass, a file shorter
    than one block made them alone, or arx_prepare_ir_spectra did: a convolution's output does not
    depend on the calls before it."""
    rng = np.random.default_rng(sr)
    n = 2 * sr
    irl, irr = sparse_ir(n, rng), sparse_ir(n, rng)
    x = (0.3 * rng.standard_normal(5 * sr + 321)).astype(np.float32)
    short = rng.standard_normal(sr // 3).astype(np.float32)
    outs = []
    for how in ("fresh", "short_file_first", "prepared_spectra"):
        r = AudioRenderer(RenderSettings(rays=(1, 1, 1), sample_rate=sr, ir_length_in_seconds=2))
        r.set_ir(irl, irr)
        if how == "short_file_first":
            r.convoluteAudioFile(short)  # no whole block: the spectra are made alone
        elif how == "prepared_spectra":
            r.prepare_ir_spectra(file=True, live=False)
        L, R, _, _ = r.convoluteAudioFile(x)
        outs.append((L, R))
        r.close()
    for L, R in outs[1:]:
        assert np.array_equal(bits(L), bits(outs[0][0])) and np.array_equal(bits(R), bits(outs[0][1]))
    for got, ir in zip(outs[0], (irl, irr)):
        ref = po.convolute_audio(x, sr, ir)
        assert np.abs(got - ref).max() <= np.spacing(np.float32(np.abs(ref).max()))
