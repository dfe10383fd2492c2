// arx_circular_buffer.hpp -- the mic path's output accumulator with the reference's semantics
// (R/prebuild/obj_raytracer/CircularBuffer.h:8-50): add() accumulates from the current index
// without advancing it; get_and_reset(n) reads n values from the index, zeroes them and
// advances.  Host-side: it is consumed by the RtAudio thread (main.cpp:114-127).
#pragma once

#include <cstddef>
#include <stdexcept>
#include <vector>

namespace arx {

template <typename T>
class CircularBuffer {
  public:
    explicit CircularBuffer(size_t size) : size_(size), buffer_(size, T(0)), index_(0) {}

    void add(const T* values, size_t length) {
        size_t i = index_;
        for (size_t k = 0; k < length; ++k) {
            buffer_[i] += values[k];
            i = (i + 1) % size_;
        }
    }

    std::vector<T> get_and_reset(size_t n) {
        if (n > size_) throw std::invalid_argument("Requested more elements than present in the buffer");
        std::vector<T> out(n);
        for (size_t k = 0; k < n; ++k) {
            const size_t i = (index_ + k) % size_;
            out[k] = buffer_[i];
            buffer_[i] = T(0);
        }
        index_ = (index_ + n) % size_;
        return out;
    }

    size_t size() const { return size_; }
    size_t index() const { return index_; }

  private:
    size_t size_;
    std::vector<T> buffer_;
    size_t index_;
};

}  // namespace arx
