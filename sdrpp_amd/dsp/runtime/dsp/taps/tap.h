// Mirror of dsp::tap<T> (core/src/dsp/taps/tap.h:6-30): borrowed {T* taps; unsigned size}.
#pragma once
#include "../buffer/buffer.h"

namespace dsp {
template <class T>
class tap {
public:
    T* taps = nullptr;
    unsigned int size = 0;
};
namespace taps {
template <class T>
inline tap<T> alloc(int count) {
    tap<T> t;
    t.size = count;
    t.taps = buffer::alloc<T>(count);
    return t;
}
template <class T>
inline void free(tap<T>& t) {
    if (!t.taps) return;
    buffer::free(t.taps);
    t.taps = nullptr;
    t.size = 0;
}
template <class T>
inline tap<T> fromArray(int count, const T* arr) {   // taps/from_array.h
    tap<T> t = alloc<T>(count);
    for (int i = 0; i < count; i++) t.taps[i] = arr[i];
    return t;
}
}  // namespace taps
}  // namespace dsp
