// ringbuffer.h -- the single-producer / single-consumer ring the reference's threads
// hand samples and display data through (includes/various/ringbuffer.h:127-319):
// RingBuffer<T>(elementCount) with a power-of-two capacity (anything else falls back
// to 32768 elements, as the reference does), putDataIntoBuffer / getDataFromBuffer
// returning the element count actually moved, GetRingBufferReadAvailable /
// GetRingBufferWriteAvailable (and their ReadSpace / WriteSpace aliases),
// skipDataInBuffer and FlushRingBuffer.  The drop-in ofdmProcessor / ofdmDecoder
// (dabgpu_dropin.h) fill the GUI's spectrum and constellation rings through it.
//
// Indices run modulo twice the capacity, so a full ring and an empty one differ;
// std::atomic acquire/release ordering stands in for the reference's explicit
// memory barriers (the producer publishes its copies before the write index, the
// consumer finishes its copies before it releases the space).
#pragma once
#include <atomic>
#include <cstdint>
#include <cstring>
#include <vector>

namespace dabgpu {

template <class elementtype>
class RingBuffer {
public:
    explicit RingBuffer(uint32_t elementCount) {
        if (elementCount == 0 || (elementCount & (elementCount - 1)) != 0) elementCount = 32768;
        size_ = elementCount;
        mask_ = elementCount - 1;
        wrap_ = 2 * elementCount - 1;
        buf_.resize(elementCount);
    }
    RingBuffer(const RingBuffer &) = delete;
    RingBuffer &operator=(const RingBuffer &) = delete;

    int32_t GetRingBufferReadAvailable() const {
        return (int32_t)((w_.load(std::memory_order_acquire) - r_.load(std::memory_order_acquire)) & wrap_);
    }
    int32_t GetRingBufferWriteAvailable() const { return (int32_t)size_ - GetRingBufferReadAvailable(); }
    int32_t ReadSpace() const { return GetRingBufferReadAvailable(); }
    int32_t WriteSpace() const { return GetRingBufferWriteAvailable(); }
    void FlushRingBuffer() {
        w_.store(0, std::memory_order_release);
        r_.store(0, std::memory_order_release);
    }

    // copies min(elementCount, free space) elements in; returns that count
    int32_t putDataIntoBuffer(const void *data, int32_t elementCount) {
        const int32_t room = GetRingBufferWriteAvailable();
        const uint32_t n = (uint32_t)(elementCount < room ? (elementCount > 0 ? elementCount : 0) : room);
        const uint32_t w = w_.load(std::memory_order_relaxed);
        copy_in((const elementtype *)data, w & mask_, n);
        w_.store((w + n) & wrap_, std::memory_order_release);
        return (int32_t)n;
    }
    // copies min(elementCount, available) elements out; returns that count
    int32_t getDataFromBuffer(void *data, int32_t elementCount) {
        const int32_t avail = GetRingBufferReadAvailable();
        const uint32_t n = (uint32_t)(elementCount < avail ? (elementCount > 0 ? elementCount : 0) : avail);
        const uint32_t r = r_.load(std::memory_order_relaxed);
        copy_out((elementtype *)data, r & mask_, n);
        r_.store((r + n) & wrap_, std::memory_order_release);
        return (int32_t)n;
    }
    int32_t skipDataInBuffer(uint32_t n_values) {
        const uint32_t avail = (uint32_t)GetRingBufferReadAvailable();
        if (n_values > avail) n_values = avail;
        r_.store((r_.load(std::memory_order_relaxed) + n_values) & wrap_, std::memory_order_release);
        return (int32_t)n_values;
    }

private:
    void copy_in(const elementtype *src, uint32_t at, uint32_t n) {
        const uint32_t first = n < size_ - at ? n : size_ - at;
        std::memcpy((void *)&buf_[at], (const void *)src, sizeof(elementtype) * first);
        if (n > first) std::memcpy((void *)&buf_[0], (const void *)(src + first), sizeof(elementtype) * (n - first));
    }
    void copy_out(elementtype *dst, uint32_t at, uint32_t n) const {
        const uint32_t first = n < size_ - at ? n : size_ - at;
        std::memcpy((void *)dst, (const void *)&buf_[at], sizeof(elementtype) * first);
        if (n > first) std::memcpy((void *)(dst + first), (const void *)&buf_[0], sizeof(elementtype) * (n - first));
    }
    uint32_t size_ = 0, mask_ = 0, wrap_ = 0;
    std::vector<elementtype> buf_;
    std::atomic<uint32_t> w_{0}, r_{0};
};

}  // namespace dabgpu
