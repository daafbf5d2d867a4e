// Reference probe (test infrastructure; built only where /root/reference exists, output in
// oracle/_ref/). Compiles the reference's OWN header-only hot-path code -- dsp/window/*.h,
// dsp/math/*.h, dsp/types.h (complex_t), dsp/taps/estimate_tap_count.h and the decimation
// plans -- straight from the reference tree (no VOLK/FFTW needed for these) and prints their
// outputs, so the oracle and libsdrgpu are pinned against reference code, not a restatement.
// Modes (binary float32 on stdout):
//   window <type> <size> <centered>      dsp::window::createWindow          (window.h:38-64)
//   lowpass <cutoff> <trans> <fs>        int32 count + taps: estimateTapCount + windowedSinc
//                                        body (windowed_sinc.h:16-27 composed of the reference's
//                                        math::sinc, window::nuttall, math::hzToRads)
//   quad <deviation_rad>                 stdin complex64 -> Quadrature::process arithmetic
//                                        (quadrature.h:41-56, complex_t ops of types.h), _din = 0
//   xlatordelta <offset_rad>             the float phaseDelta of frequency_xlator.h:17 (2 floats)
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include <dsp/types.h>
#include <dsp/window/window.h>
#include <dsp/math/hz_to_rads.h>
#include <dsp/math/sinc.h>
#include <dsp/taps/estimate_tap_count.h>

int main(int argc, char** argv) {
    if (argc < 2) return 2;
    if (!strcmp(argv[1], "window") && argc == 5) {
        int type = atoi(argv[2]), size = atoi(argv[3]), centered = atoi(argv[4]);
        std::vector<float> w(size + 1);   // +1: the reference writes w[size] for odd centred sizes
        dsp::window::createWindow((dsp::window::windowType)type, w.data(), size, centered != 0);
        fwrite(w.data(), sizeof(float), size, stdout);
        return 0;
    }
    if (!strcmp(argv[1], "lowpass") && argc == 5) {
        double cutoff = atof(argv[2]), tw = atof(argv[3]), fs = atof(argv[4]);
        int count = dsp::taps::estimateTapCount(tw, fs);
        double omega = dsp::math::hzToRads(cutoff, fs);
        double half = (double)count / 2.0;
        double corr = 1.0 * omega / DB_M_PI;
        std::vector<float> t(count);
        for (int i = 0; i < count; i++) {
            double tt = (double)i - half + 0.5;
            t[i] = dsp::math::sinc(tt * omega) * dsp::window::nuttall(tt - half, count) * corr;
        }
        fwrite(&count, sizeof(int), 1, stdout);
        fwrite(t.data(), sizeof(float), count, stdout);
        return 0;
    }
    if (!strcmp(argv[1], "quad") && argc == 3) {
        float inv = 1.0 / atof(argv[2]);              // float _invDeviation = 1.0 / deviation
        dsp::complex_t din = {0.0f, 0.0f}, y;
        float out;
        while (fread(&y, sizeof(y), 1, stdin) == 1) {
            out = (y * din.conj()).phase() * inv;
            din = y;
            fwrite(&out, sizeof(out), 1, stdout);
        }
        return 0;
    }
    if (!strcmp(argv[1], "xlatordelta") && argc == 3) {
        double off = atof(argv[2]);
        float d[2] = {(float)cos(off), (float)sin(off)};   // lv_cmake(cos(offset), sin(offset))
        fwrite(d, sizeof(float), 2, stdout);
        return 0;
    }
    return 2;
}
