// Mirror of dsp::buffer (core/src/dsp/buffer/buffer.h:6-17): aligned sample buffers.
// volk_malloc is replaced by 4 KiB-aligned allocation so a buffer can be registered with
// the GPU runtime (sdrgpu_host_register) for direct DMA. Built with SDRGPU_PIN_STREAMS, every
// buffer (so every dsp::stream buffer) is registered on alloc and unregistered on free, and the
// GPU blocks' process() then DMA straight from / into the stream buffers.
#pragma once
#include <cstdlib>
#include <cstring>
#ifdef SDRGPU_PIN_STREAMS
#include "sdrgpu.h"
#endif

namespace dsp::buffer {
template <class T>
inline T* alloc(int count) {
    size_t bytes = ((size_t)(count > 0 ? count : 1) * sizeof(T) + 4095) & ~(size_t)4095;
    T* p = (T*)std::aligned_alloc(4096, bytes);
#ifdef SDRGPU_PIN_STREAMS
    if (p) (void)sdrgpu_host_register(p, bytes);   // (without a GPU it stays pageable)
#endif
    return p;
}
template <class T>
inline void clear(T* buffer, int count, int offset = 0) {
    std::memset(&buffer[offset], 0, (size_t)count * sizeof(T));
}
inline void free(void* buffer) {
#ifdef SDRGPU_PIN_STREAMS
    if (buffer) (void)sdrgpu_host_unregister(buffer);
#endif
    std::free(buffer);
}
}  // namespace dsp::buffer
