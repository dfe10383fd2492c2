// arx_rtaudio.hpp -- RtAudio callbacks of the reference app over libarx.so.
//
// Signature of RtAudioCallback (R/RtAudio.h:222-226; C form rtaudio_c.h:107-109):
//   int cb(void* outputBuffer, void* inputBuffer, unsigned int nFrames, double streamTime,
//          RtAudioStreamStatus status, void* userData)
// with RtAudioStreamStatus an unsigned int.  Streams are opened with RTAUDIO_FLOAT64
// (main.cpp:157, 202), so both buffers are double.  No RtAudio header is needed here: the
// functions match the typedef and can be passed to RtAudio::openStream directly.
#pragma once

#include <atomic>
#include <cmath>
#include <cstddef>
#include <vector>

#include "arx.h"
#include "arx_circular_buffer.hpp"

namespace arx {

constexpr unsigned kInputSampleRate = 44100;   // main.cpp:36
constexpr unsigned kInputBufferLength = 4096;  // main.cpp:37

// audioCallbackData (main.cpp:172-186) reduced to what the callback reads.
struct MicCallbackData {
    arx_renderer* renderer = nullptr;
    CircularBuffer<double>* samplesRecordBuffer = nullptr;  // size 44100 * ir_sec (main.cpp:189)
    float volume = 1.0f;                                     // Context::get_volume()
    std::atomic<bool>* is_rendering = nullptr;               // Context::get_is_rendering()
    std::vector<double> scratch;                             // 2 * ir_len
};

// audioHandlerWithMic (main.cpp:99-135).
inline int audio_handler_with_mic(void* outputBuffer, void* inputBuffer, unsigned int nBufferFrames,
                                  double /*streamTime*/, unsigned int /*status*/, void* data) {
    MicCallbackData* d = static_cast<MicCallbackData*>(data);
    double* out = static_cast<double*>(outputBuffer);
    const double* in = static_cast<const double*>(inputBuffer);
    if (d->is_rendering && d->is_rendering->load()) {  // "Buffer is still being processed"
        for (unsigned i = 0; i < 2 * nBufferFrames; ++i) out[i] = 0.0;
        return 0;
    }
    arx_config c;
    arx_get_config(d->renderer, &c);
    const size_t ir_len = (size_t)c.ir_length_in_seconds * (size_t)c.sample_rate;
    d->scratch.resize(2 * ir_len);
    if (arx_convolute_live_block(d->renderer, in, kInputBufferLength * sizeof(double), d->scratch.data(),
                                 d->scratch.size()) != ARX_OK)
        return 1;  // abort the stream on device failure (the reference would exit())
    d->samplesRecordBuffer->add(d->scratch.data(), d->scratch.size());
    std::vector<double> v = d->samplesRecordBuffer->get_and_reset(2 * (size_t)nBufferFrames);
    for (unsigned i = 0; i < 2 * nBufferFrames; ++i) out[i] = (v[i] != v[i]) ? 0.0 : v[i] * d->volume;
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
