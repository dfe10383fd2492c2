"""Pin the oracle's f64 FFT convolution against numpy (pocketfft) and direct sums.

Reference semantics (kernels.cu:382-438 + AudioRenderer.cpp:706-711): S = len // sr
one-second blocks, each zero padded to n = ir_len, circular length-n convolution with
the IR, unnormalised (x n), overlap-added at sr hops clipped to len, tail samples never
processed, then divided by (n // 2).
"""
import numpy as np
import pytest

import pyoracle as po


def numpy_reference(x, sr, ir):
    """Independent numpy restatement of convoluteFromAudioBuffer + host normalisation."""
    n = ir.size
    H = np.fft.fft(ir.astype(np.float64))
    acc = np.zeros(x.size, np.float64)
    for s in range(x.size // sr):
        seg = np.zeros(n)
        seg[:sr] = x[s * sr:(s + 1) * sr]
        y = np.fft.ifft(np.fft.fft(seg) * H).real * n
        cnt = n if s * sr + n < x.size else x.size - s * sr
        acc[s * sr:s * sr + cnt] += y[:cnt]
    return (acc / (n // 2)).astype(np.float32)


def direct_reference(x, sr, ir):
    n = ir.size
    acc = np.zeros(x.size, np.float64)
    for s in range(x.size // sr):
        seg = x[s * sr:(s + 1) * sr].astype(np.float64)
        cc = np.zeros(n)
        for i in range(sr):
            cc += seg[i] * np.roll(ir.astype(np.float64), i)
        cnt = min(n, x.size - s * sr)
        acc[s * sr:s * sr + cnt] += n * cc[:cnt]
    return (acc / (n // 2)).astype(np.float32)


@pytest.mark.parametrize("n", [1, 2, 3, 4, 5, 7, 12, 97, 1000, 4096, 32000])
def test_fft_matches_numpy(n):
    rng = np.random.default_rng(n)
    x = rng.normal(size=n) + 1j * rng.normal(size=n)
    ref = np.fft.fft(x)
    got = po.fft(x, -1)
    assert np.abs(got - ref).max() <= 1e-12 * max(1.0, np.abs(ref).max())
    back = po.fft(got, +1) / n
    assert np.abs(back - x).max() < 1e-12 * max(1.0, np.abs(x).max())


def ulp_of_max(y):
    return np.spacing(np.float32(np.abs(y).max()))


@pytest.mark.parametrize("sr,secs,length", [(50, 2, 537), (64, 3, 640), (31, 1, 200), (40, 2, 39)])
def test_conv_small_direct(sr, secs, length):
    rng = np.random.default_rng(sr + length)
    x = rng.uniform(-1, 1, length).astype(np.float32)
    ir = (rng.exponential(size=sr * secs) * (rng.uniform(size=sr * secs) < 0.2)).astype(np.float32)
    got = po.convolute_audio(x, sr, ir)
    ref = direct_reference(x, sr, ir)
    assert np.abs(got - ref).max() <= ulp_of_max(ref)


@pytest.mark.parametrize("sr,length", [(16000, 128000), (16000, 399569), (1000, 10555)])
def test_conv_matches_numpy(sr, length):
    rng = np.random.default_rng(length)
    x = (0.3 * rng.standard_normal(length)).astype(np.float32)
    n = 2 * sr
    ir = np.zeros(n, np.float32)
    k = rng.integers(0, n, 400)
    ir[k] = rng.exponential(1e-4, 400).astype(np.float32)
    got = po.convolute_audio(x, sr, ir)
    ref = numpy_reference(x, sr, ir)
    assert np.abs(got - ref).max() <= ulp_of_max(ref)


def test_conv_tail_and_short_input():
    sr = 100
    rng = np.random.default_rng(1)
    ir = rng.uniform(size=2 * sr).astype(np.float32)
    x = rng.uniform(-1, 1, 3 * sr + 57).astype(np.float32)
    y = po.convolute_audio(x, sr, ir)
    x2 = x.copy()
    x2[3 * sr:] = 5.0  # the unprocessed tail (kernels.cu:413) never reaches the output
    assert np.array_equal(po.convolute_audio(x2, sr, ir), y)
    short = x[:sr - 1]  # len < sr: zero blocks, output stays zero
    assert not po.convolute_audio(short, sr, ir).any()


def test_live_block_matches_numpy():
    n = 4410
    rng = np.random.default_rng(5)
    x = rng.uniform(-1, 1, 409)
    irl = rng.uniform(size=n).astype(np.float32)
    irr = rng.uniform(size=n).astype(np.float32)
    got = po.convolute_live_block(x, irl, irr)
    seg = np.zeros(n)
    seg[:x.size] = x
    for ch, ir in enumerate((irl, irr)):
        ref = np.fft.ifft(np.fft.fft(seg) * np.fft.fft(ir.astype(np.float64))).real * n / (n // 2)
        np.testing.assert_allclose(got[ch::2], ref, rtol=1e-10, atol=1e-10)


# ---- streaming convolution (uniformly partitioned overlap-save, orc_stream_*) -------------------
def stream_all(block, hl, hr, x, cuts=None):
    st = po.Stream(block, hl, hr)
    outs, pos = [], 0
    for n in cuts or [block] * (-(-x.size // block)):
        outs.append(st.process(x[pos:pos + n]))
        pos += n
    return np.concatenate(outs)


@pytest.mark.parametrize("ir_len,block", [(1000, 64), (1000, 100), (441, 441), (3000, 4096 // 8), (88200, 4096)])
def test_stream_oracle_equals_linear_convolution(ir_len, block):
    rng = np.random.default_rng(ir_len + block)
    hl = rng.standard_normal(ir_len).astype(np.float32)
    hr = (rng.standard_normal(ir_len) * (rng.random(ir_len) < 0.05)).astype(np.float32)
    nb = 6 if ir_len > 50000 else 25
    x = rng.uniform(-1, 1, block * nb)
    out = stream_all(block, hl, hr, x)
    scale = ir_len / (ir_len // 2)
    for ch, h in ((0, hl), (1, hr)):
        ref = np.convolve(x, h.astype(np.float64))[:x.size] * scale
        assert np.abs(out[ch::2] - ref).max() <= 1e-13 * np.abs(ref).max()


def test_stream_oracle_short_blocks_are_zero_padded():
    rng = np.random.default_rng(2)
    hl, hr = rng.standard_normal(500).astype(np.float32), rng.standard_normal(500).astype(np.float32)
    cuts = [64, 10, 64, 0, 37, 64]
    x = rng.uniform(-1, 1, sum(cuts))
    out = stream_all(64, hl, hr, x, cuts)
    padded = np.concatenate([np.pad(x[sum(cuts[:i]):sum(cuts[:i + 1])], (0, 64 - c)) for i, c in enumerate(cuts)])
    ref = np.convolve(padded, hl.astype(np.float64))[:padded.size] * (500 / 250)
    assert np.abs(out[0::2] - ref).max() <= 1e-13 * np.abs(ref).max()


def test_stream_equals_compat_path_when_tails_do_not_wrap():
    """The reference's live path (per block: full-length circular convolution, accumulated at
    the block's offset) equals the stream when the IR support leaves room for a block
    (support <= ir_len - block) and the accumulator does not wrap."""
    rng = np.random.default_rng(4)
    n, block, nb = 4000, 256, 12
    hl = np.zeros(n, np.float32)
    hr = np.zeros(n, np.float32)
    hl[:n - block] = rng.standard_normal(n - block)
    hr[rng.integers(0, n - block, 40)] = 1.0
    x = rng.uniform(-1, 1, block * nb)
    acc = np.zeros(2 * (block * nb + n))
    for b in range(nb):
        acc[2 * b * block:2 * b * block + 2 * n] += po.convolute_live_block(x[b * block:(b + 1) * block], hl, hr)
    out = stream_all(block, hl, hr, x)
    assert np.abs(out - acc[:out.size]).max() <= 1e-12 * np.abs(acc).max()


@pytest.mark.parametrize("N1,N2", [(300, 320), (315, 280), (160, 200), (45, 50)])
def test_four_step_packed_ir_mirror_rows(N1, N2):
    """The index algebra of pass_b_pair (arx_conv.hip), in numpy: the four-step spectrum of the
    packed IR g = h_L + i h_R (columns of length N1 * twiddle, then rows of length N2) puts
    X[k1 + N1 k2] at row k1, column k2; -k lies in row N1 - k1 at column N2 - 1 - k2 (row 0:
    column -k2 mod N2), and H_L = (G + conj G-) / 2, H_R = (G - conj G-) / 2i recover both IR
    spectra."""
    n = N1 * N2
    rng = np.random.default_rng(N1)
    hl, hr = rng.standard_normal(n), rng.standard_normal(n)
    g = (hl + 1j * hr).reshape(N1, N2)  # x[N2 n1 + n2] at [n1, n2]
    cols = np.fft.fft(g, axis=0)  # [k1, n2]
    k1 = np.arange(N1)[:, None]
    n2 = np.arange(N2)[None, :]
    cols = cols * np.exp(-2j * np.pi * k1 * n2 / n)
    G = np.fft.fft(cols, axis=1)  # [k1, k2] = X[k1 + N1 k2]
    ref = np.fft.fft(hl + 1j * hr)
    kk = (k1 + N1 * np.arange(N2)[None, :])
    assert np.allclose(G, ref[kk], atol=1e-9 * n)
    rows = np.where(np.arange(N1) == 0, 0, N1 - np.arange(N1))
    mir = np.empty_like(G)
    for r in range(N1):
        i = np.arange(N2)
        mi = np.where(i == 0, 0, N2 - i) if r == 0 else N2 - 1 - i
        mir[r] = G[rows[r], mi]
    HL = (G + np.conj(mir)) / 2
    HR = (G - np.conj(mir)) / 2j
    assert np.allclose(HL, np.fft.fft(hl)[kk], atol=1e-9 * n)
    assert np.allclose(HR, np.fft.fft(hr)[kk], atol=1e-9 * n)
