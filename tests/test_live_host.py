"""Host side of the RtAudio surface: CircularBuffer semantics (CircularBuffer.h:8-50), the
C++ headers compiling against libarx.so, and the C++ / Python CircularBuffer agreeing."""
import os
import subprocess

import numpy as np
import pytest

from audiorenderingv2_amd.live import CircularBuffer, audio_handler
from conftest import REPO


def reference_circular(size, ops):
    """Literal restatement of CircularBuffer<T> (CircularBuffer.h:13-36)."""
    buf = [0.0] * size
    index = 0
    outs = []
    for op, arg in ops:
        if op == "add":
            init = index
            for v in arg:
                buf[index] += v
                index = (index + 1) % size
            index = init
        else:
            res = []
            for i in range(arg):
                res.append(buf[(index + i) % size])
                buf[(index + i) % size] = 0.0
            index = (index + arg) % size
            outs.append(res)
    return outs


def random_ops(rng, size):
    ops = []
    for _ in range(12):
        if rng.uniform() < 0.5:
            ops.append(("add", list(rng.standard_normal(int(rng.integers(1, 3 * size))))))
        else:
            ops.append(("get", int(rng.integers(1, size + 1))))
    return ops


def test_circular_buffer_matches_reference():
    rng = np.random.default_rng(0)
    for size in (5, 64, 1000):
        ops = random_ops(rng, size)
        cb = CircularBuffer(size)
        outs = []
        for op, arg in ops:
            if op == "add":
                cb.add(np.array(arg))
            else:
                outs.append(list(cb.get_and_reset(arg)))
        ref = reference_circular(size, ops)
        assert len(outs) == len(ref)
        for a, b in zip(outs, ref):
            np.testing.assert_allclose(a, b, rtol=0, atol=1e-12)
    with pytest.raises(ValueError):
        CircularBuffer(4).get_and_reset(5)


def test_mic_path_wraps_like_reference():
    # 44100*ir_sec slots receive 2*ir_len values per callback (main.cpp:189-195, AudioRenderer.cpp:653)
    ir_len = 88200
    cb = CircularBuffer(44100 * 2)
    cb.add(np.ones(2 * ir_len))
    assert np.all(cb.get_and_reset(8192) == 2.0)


CPP = r"""
#include <cstdio>
#include <vector>
#include "arx_audio_renderer.hpp"
#include "arx_circular_buffer.hpp"
#include "arx_rtaudio.hpp"
int main(int argc, char** argv) {
    (void)argc;
    arx::CircularBuffer<double> cb(7);
    std::vector<double> a = {1, 2, 3, 4, 5, 6, 7, 8, 9, 10};
    cb.add(a.data(), a.size());
    auto x = cb.get_and_reset(3);
    cb.add(a.data(), 4);
    auto y = cb.get_and_reset(7);
    for (double v : x) std::printf("%g ", v);
    for (double v : y) std::printf("%g ", v);
    // file playback callback on host buffers
    std::vector<float> L = {1, 2, 3, 4}, R = {5, 6, 7, 8};
    arx::FileCallbackData fd;
    fd.out_left = L.data(); fd.out_right = R.data(); fd.len = 4; fd.sample_rate = 2; fd.volume = 0.5f;
    std::vector<double> out(6, -1.0);
    arx::audio_handler(out.data(), nullptr, 3, 0.5, 0, &fd);
    for (double v : out) std::printf("%g ", v);
    arx_config c; arx_default_config(&c);
    std::printf("%d\n", c.rays_x);
    // native formats through the shim (host only)
    auto meshes = arx::loadOBJ(argv[1]);
    std::printf("%zu %s %zu\n", meshes.size(), meshes[0].material_name.c_str(), meshes[0].index.size() / 3);
    arx::Wav w;
    w.samples = {{0.5f, -0.25f, 1.0f}};
    w.sample_rate = 8000;
    w.bit_depth = 32;
    arx::saveWav(argv[2], w);
    auto r = arx::loadWav(argv[2]);
    std::printf("%d %d %g %g\n", r.sample_rate, r.bit_depth, r.samples[0][1], arx::normalizeToRangeMinusOneToOne(r.samples[0])[0]);
    return 0;
}
"""


def test_cpp_headers_compile_and_agree(tmp_path):
    src = tmp_path / "t.cpp"
    src.write_text(CPP)
    exe = tmp_path / "t"
    pkg = os.path.join(REPO, "audiorenderingv2_amd")
    subprocess.run(["g++", "-std=c++17", "-O1", "-I", os.path.join(REPO, "include"), str(src), "-L", pkg, "-larx",
                    f"-Wl,-rpath,{pkg}", "-o", str(exe)], check=True)
    (tmp_path / "m.mtl").write_text("newmtl brick\n")
    (tmp_path / "m.obj").write_text("mtllib m.mtl\nv 0 0 0\nv 1 0 0\nv 1 1 0\nv 0 1 0\nusemtl brick\nf 1 2 3 4\n")
    lines = subprocess.run([str(exe), str(tmp_path / "m.obj"), str(tmp_path / "w.wav")], check=True,
                           capture_output=True, text=True).stdout.splitlines()
    assert lines[-2].split() == ["1", "brick", "2"]
    assert lines[-1].split() == ["8000", "32", "-0.25", "0.2"]
    out = " ".join(lines[:-2]).split()
    vals = [float(v) for v in out]
    ops = [("add", [1, 2, 3, 4, 5, 6, 7, 8, 9, 10]), ("get", 3), ("add", [1, 2, 3, 4]), ("get", 7)]
    ref = reference_circular(7, ops)
    assert vals[:10] == ref[0] + ref[1]
    py = audio_handler(np.array([1, 2, 3, 4], np.float32), np.array([5, 6, 7, 8], np.float32), 0.5, 2, 3, 0.5)
    assert vals[10:16] == list(py)
    assert vals[16] == 100
