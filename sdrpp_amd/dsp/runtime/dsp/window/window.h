// Mirror of dsp::window::windowType (core/src/dsp/window/window.h:27-35); the window values
// themselves are made by the library (sdrgpu_create_window, bit-exact with createWindow).
#pragma once

namespace dsp::window {
enum windowType {
    RECTANGULAR,
    HAMMING,
    HANN,
    BLACKMAN,
    NUTTALL,
    BLACKMAN_HARRIS4,
    BLACKMAN_HARRIS7,
};
}  // namespace dsp::window
