// arx_rtaudio.hpp -- RtAudio callbacks of the reference app over libarx.so.
//
// Signature of RtAudioCallback (R/RtAudio.h:222-226; C form rtaudio_c.h:107-109):
//   int cb(void* outputBuffer, void* inputBuffer, unsigned int nFrames, double streamTime,
//          RtAudioStreamStatus status, void* userData)
// with RtAudioStreamStatus an unsigned int.  Streams are opened with RTAUDIO_FLOAT64
// (main.cpp:157, 202), so both buffers are double.  No RtAudio header is needed here: the
// functions match the typedef and can be passed to RtAudio::openStream directly.
#pragma once

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstddef>
#include <mutex>
#include <vector>

#include "arx.h"
#include "arx_circular_buffer.hpp"

namespace arx {

constexpr unsigned kInputSampleRate = 44100;   // main.cpp:36
constexpr unsigned kInputBufferLength = 4096;  // main.cpp:37

// audioCallbackData (main.cpp:172-186) reduced to what the callback reads.  renderer_mutex (if
// set) is the lock the render thread holds around render() / full_render_cycle: the callback only
// try-locks it and outputs silence when the renderer is busy, so the two threads never drive the
// renderer at once (arx.h: one host thread per renderer).  The reference instead checks a plain
// bool is_rendering and then calls the renderer, a check-then-act race (main.cpp:104-112).
struct MicCallbackData {
    arx_renderer* renderer = nullptr;
    CircularBuffer<double>* samplesRecordBuffer = nullptr;  // size 44100 * ir_sec (main.cpp:189)
    float volume = 1.0f;                                     // Context::get_volume()
    std::atomic<bool>* is_rendering = nullptr;               // Context::get_is_rendering()
    std::mutex* renderer_mutex = nullptr;
    std::vector<double> scratch;                             // 2 * ir_len
    arx_stream* stream = nullptr;                            // audio_handler_with_mic_stream only
};

// audioHandlerWithMic (main.cpp:99-135), the reference-compatible path: one full-length circular
// convolution per callback added into the CircularBuffer.  At most min(nBufferFrames, 4096) input
// frames are read (the reference always passes 4096, over-reading a smaller buffer).
inline int audio_handler_with_mic(void* outputBuffer, void* inputBuffer, unsigned int nBufferFrames,
                                  double /*streamTime*/, unsigned int /*status*/, void* data) {
    MicCallbackData* d = static_cast<MicCallbackData*>(data);
    double* out = static_cast<double*>(outputBuffer);
    const double* in = static_cast<const double*>(inputBuffer);
    std::unique_lock<std::mutex> lock;
    if (d->renderer_mutex) lock = std::unique_lock<std::mutex>(*d->renderer_mutex, std::try_to_lock);
    if ((d->is_rendering && d->is_rendering->load()) || (d->renderer_mutex && !lock.owns_lock())) {
        for (unsigned i = 0; i < 2 * nBufferFrames; ++i) out[i] = 0.0;  // "Buffer is still being processed"
        return 0;
    }
    arx_config c;
    arx_get_config(d->renderer, &c);
    const size_t ir_len = (size_t)c.ir_length_in_seconds * (size_t)c.sample_rate;
    d->scratch.resize(2 * ir_len);
    const size_t n_in = std::min<size_t>(nBufferFrames, kInputBufferLength);
    if (arx_convolute_live_block(d->renderer, in, n_in * sizeof(double), d->scratch.data(), d->scratch.size()) != ARX_OK)
        return 1;  // abort the stream on device failure (the reference would exit())
    d->samplesRecordBuffer->add(d->scratch.data(), d->scratch.size());
    std::vector<double> v = d->samplesRecordBuffer->get_and_reset(2 * (size_t)nBufferFrames);
    for (unsigned i = 0; i < 2 * nBufferFrames; ++i) out[i] = (v[i] != v[i]) ? 0.0 : v[i] * d->volume;
    return 0;
}

// The same duplex callback over the streaming convolution (arx_stream_*, d->stream created with
// block_frames = the stream's nBufferFrames; any other buffer size aborts the stream): the output block is the linear convolution of the
// mic stream with the IR, one block of latency, no circular wrap and no CircularBuffer.
inline int audio_handler_with_mic_stream(void* outputBuffer, void* inputBuffer, unsigned int nBufferFrames,
                                         double /*streamTime*/, unsigned int /*status*/, void* data) {
    MicCallbackData* d = static_cast<MicCallbackData*>(data);
    double* out = static_cast<double*>(outputBuffer);
    const double* in = static_cast<const double*>(inputBuffer);
    std::unique_lock<std::mutex> lock;
    if (d->renderer_mutex) lock = std::unique_lock<std::mutex>(*d->renderer_mutex, std::try_to_lock);
    int32_t block = 0;
    // the stream consumes exactly one block per call: a shorter device buffer would be zero padded
    // to a full block (gaps in the input timeline) and lose the tail of every output block
    if (!d->stream || arx_stream_info(d->stream, &block, nullptr, nullptr) != ARX_OK || nBufferFrames != (unsigned)block)
        return 1;
    if ((d->is_rendering && d->is_rendering->load()) || (d->renderer_mutex && !lock.owns_lock())) {
        for (unsigned i = 0; i < 2 * nBufferFrames; ++i) out[i] = 0.0;
        return 0;
    }
    d->scratch.resize(2 * (size_t)block);
    if (arx_stream_process(d->stream, in, nBufferFrames, d->scratch.data(), d->scratch.size()) != ARX_OK) return 1;
    for (unsigned i = 0; i < 2 * nBufferFrames; ++i) {
        const double v = d->scratch[i];
        out[i] = (v != v) ? 0.0 : v * d->volume;
    }
    return 0;
}

// AudioInfo + output buffers for file playback (main.cpp:69-97, 137-161).
struct FileCallbackData {
    const float* out_left = nullptr;   // Context::get_output_buffer_left()
    const float* out_right = nullptr;
    size_t len = 0;                    // samples per channel
    unsigned sample_rate = 0;          // audio file rate
    float volume = 1.0f;
};

// audioHandler (main.cpp:69-97): interleaves by the parity of the output index, x100 x volume;
// the bound is checked against the BYTE length like the reference (output_buffer_len =
// sizeof(float) * len, Context.cpp:212), reads beyond the arrays yield 0 instead of garbage.
inline int audio_handler(void* outputBuffer, void* /*inputBuffer*/, unsigned int nBufferFrames, double streamTime,
                         unsigned int /*status*/, void* data) {
    FileCallbackData* d = static_cast<FileCallbackData*>(data);
    double* out = static_cast<double*>(outputBuffer);
    if (d->len == 0) return 0;
    const size_t next = (size_t)(int)(streamTime * d->sample_rate) % d->len;
    const size_t byte_len = sizeof(float) * d->len;
    for (unsigned i = 0; i < nBufferFrames * 2; ++i) {
        if (i + next >= byte_len) break;
        const size_t j = i + next;
        const float* src = (i % 2 == 0) ? d->out_left : d->out_right;
        *out++ = (j < d->len ? (double)src[j] : 0.0) * 100 * d->volume;
    }
    return 0;
}

}  // namespace arx
