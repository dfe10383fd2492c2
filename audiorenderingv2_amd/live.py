"""RtAudio-callback surface of the reference, host side (Python mirror; C++ in include/).

* CircularBuffer  -- R/prebuild/obj_raytracer/CircularBuffer.h:8-50 (same quirks: add()
  accumulates from the current index WITHOUT advancing it; get_and_reset(n) reads, zeroes
  and advances; the mic path's buffer holds 44100*ir_sec values but receives 2*ir_len per
  callback, so it wraps, main.cpp:189-195 / AudioRenderer.cpp:653).
* audio_handler_with_mic -- main.cpp:99-135 (duplex mic callback: convolve the input block
  unless a render is in progress, pop 2*nFrames interleaved samples, NaN -> 0, x volume).
* audio_handler -- main.cpp:69-97 (file playback from the convolved output buffers,
  interleaved by parity of the output index, x100 x volume, bound checked against the
  BYTE length of the buffers as in the reference).
"""
from __future__ import annotations

import numpy as np


class CircularBuffer:
    def __init__(self, size: int):
        self.size = int(size)
        self.buffer = np.zeros(self.size, np.float64)
        self.index = 0

    def add(self, values: np.ndarray) -> None:
        v = np.asarray(values, np.float64).ravel()
        idx = (self.index + np.arange(v.size)) % self.size
        np.add.at(self.buffer, idx, v)  # wraps; index is NOT advanced (CircularBuffer.h:13-20)

    def get_and_reset(self, n: int) -> np.ndarray:
        if n > self.size:
            raise ValueError("Requested more elements than present in the buffer")
        idx = (self.index + np.arange(n)) % self.size
        out = self.buffer[idx].copy()
        self.buffer[idx] = 0.0
        self.index = (self.index + n) % self.size
        return out


INPUT_SAMPLE_RATE = 44100  # main.cpp:36
INPUT_BUFFER_LENGTH = 4096  # main.cpp:37


def audio_handler_with_mic(renderer, circular_buffer: CircularBuffer, input_block: np.ndarray, n_frames: int,
                           volume: float, is_rendering: bool = False) -> np.ndarray:
    """One duplex callback (main.cpp:99-135); returns the 2*n_frames interleaved output."""
    if is_rendering:  # "Buffer is still being processed": silence
        return np.zeros(2 * n_frames, np.float64)
    # the reference always passes INPUT_BUFFER_LENGTH * sizeof(double) bytes (main.cpp:112)
    renderer.convoluteLiveInput(np.asarray(input_block, np.float64)[:INPUT_BUFFER_LENGTH], circular_buffer)
    out = circular_buffer.get_and_reset(2 * n_frames)
    out = np.where(np.isnan(out), 0.0, out * volume)
    return out


def audio_handler(out_left: np.ndarray, out_right: np.ndarray, stream_time: float, sample_rate: int,
                  n_frames: int, volume: float) -> np.ndarray:
    """File playback callback (main.cpp:69-97).  The bound check compares the interleaved
    index against the buffers' BYTE length (output_buffer_len = 4*len), as the reference does;
    reads past the float arrays are clipped to zero here instead of reading garbage."""
    n = out_left.size
    next_stream = int(stream_time * sample_rate) % n
    byte_len = 4 * n
    res = np.zeros(2 * n_frames, np.float64)
    for i in range(2 * n_frames):
        if i + next_stream >= byte_len:
            break
        j = i + next_stream
        src = out_left if i % 2 == 0 else out_right
        res[i] = (float(src[j]) if j < n else 0.0) * 100 * volume
    return res
