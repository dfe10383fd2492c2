"""GPU parity of the live (mic) path: convoluteLiveInput (AudioRenderer.cpp:593-661) and the
duplex callback (main.cpp:99-135) against the f64 oracle (orc_convolute_live_block)."""
import numpy as np
import pytest

import pyoracle as po
from audiorenderingv2_amd import ArxError, AudioRenderer, RenderSettings
from audiorenderingv2_amd.live import CircularBuffer, audio_handler_with_mic

pytestmark = pytest.mark.gpu


def live_renderer(sr=44100, secs=2, seed=0):
    r = AudioRenderer(RenderSettings(rays=(1, 1, 1), sample_rate=sr, ir_length_in_seconds=secs))
    rng = np.random.default_rng(seed)
    n = sr * secs
    irs = []
    for _ in range(2):
        ir = np.zeros(n, np.float32)
        ir[rng.integers(0, n, 500)] = rng.exponential(1e-3, 500).astype(np.float32)
        irs.append(ir)
    r.set_ir(*irs)
    return r, irs


def rel_err(got, ref):
    return np.abs(got - ref).max() / max(np.abs(ref).max(), 1e-300)


@pytest.mark.parametrize("n_in", [4096, 1000, 5000, 0])
def test_live_block_matches_oracle(n_in):
    r, (irl, irr) = live_renderer()
    x = np.random.default_rng(n_in).uniform(-1, 1, n_in)
    got = r.convoluteLiveInput(x)
    ref = po.convolute_live_block(x, irl, irr)
    if n_in == 0:
        assert not got.any()
    else:
        assert rel_err(got, ref) < 1e-12


def test_prepared_spectra_follow_new_ir():
    r, (irl, irr) = live_renderer(seed=3)
    x = np.random.default_rng(4).uniform(-1, 1, 4096)
    r.prepare_ir_spectra(file=True, live=True)
    assert rel_err(r.convoluteLiveInput(x), po.convolute_live_block(x, irl, irr)) < 1e-12
    irl2, irr2 = irr * 0.5, irl * 2.0  # new IR -> spectra must be recomputed
    r.set_ir(irl2, irr2)
    r.prepare_ir_spectra(file=True, live=True)
    assert rel_err(r.convoluteLiveInput(x), po.convolute_live_block(x, irl2, irr2)) < 1e-12


@pytest.mark.parametrize("sr,secs", [(16000, 2), (22050, 1), (32000, 2)])
def test_live_block_256_point_plans(sr, secs):
    """Plans whose sub-FFTs are 256 points (M = 2^16: 16 kHz x 2 s, 22.05 kHz x 1 s) or mix
    256-point columns with 512-point rows (M = 2^17: 32 kHz x 2 s) -- the radix-4 wave FFTs."""
    r, (irl, irr) = live_renderer(sr=sr, secs=secs, seed=sr)
    x = np.random.default_rng(sr).uniform(-1, 1, min(4096, sr))
    assert rel_err(r.convoluteLiveInput(x), po.convolute_live_block(x, irl, irr)) < 1e-12


def test_live_block_48k_and_oversize():
    r, (irl, irr) = live_renderer(sr=48000)
    x = np.random.default_rng(1).uniform(-1, 1, 4096)
    assert rel_err(r.convoluteLiveInput(x), po.convolute_live_block(x, irl, irr)) < 1e-12
    with pytest.raises(ArxError):
        r.convoluteLiveInput(np.zeros(2 * 48000 + 1))


def test_mic_callback_sequence():
    r, (irl, irr) = live_renderer()
    rng = np.random.default_rng(7)
    gpu_cb = CircularBuffer(44100 * 2)
    ref_cb = CircularBuffer(44100 * 2)
    for k in range(6):
        block = rng.uniform(-0.5, 0.5, 4096)
        out = audio_handler_with_mic(r, gpu_cb, block, 4096, volume=0.7)
        ref_cb.add(po.convolute_live_block(block, irl, irr))
        ref = ref_cb.get_and_reset(2 * 4096) * 0.7
        assert rel_err(out, ref) < 1e-12, k
    silent = audio_handler_with_mic(r, gpu_cb, block, 4096, volume=0.7, is_rendering=True)
    assert not silent.any()
