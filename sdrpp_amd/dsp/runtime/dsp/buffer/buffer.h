// Mirror of dsp::buffer (core/src/dsp/buffer/buffer.h:6-17): aligned sample buffers.
// volk_malloc is replaced by 4 KiB-aligned allocation so a buffer can be registered with
// the GPU runtime (sdrgpu_host_register) for direct DMA.
#pragma once
#include <cstdlib>
#include <cstring>

namespace dsp::buffer {
template <class T>
inline T* alloc(int count) {
    size_t bytes = ((size_t)(count > 0 ? count : 1) * sizeof(T) + 4095) & ~(size_t)4095;
    return (T*)std::aligned_alloc(4096, bytes);
}
template <class T>
inline void clear(T* buffer, int count, int offset = 0) {
    std::memset(&buffer[offset], 0, (size_t)count * sizeof(T));
}
inline void free(void* buffer) { std::free(buffer); }
}  // namespace dsp::buffer
