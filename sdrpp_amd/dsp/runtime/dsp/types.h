// Stand-alone mirror of the reference's sample types (core/src/dsp/types.h:6-127): same
// layout ({float re, im}, {float l, r}) and member operators, so GPU blocks and their tests
// build without the reference tree. In an SDR++ build the reference's own header is used.
#pragma once
#include <cmath>

namespace dsp {
struct complex_t {
    float re, im;
    complex_t operator*(float b) const { return {re * b, im * b}; }
    complex_t operator*(double b) const { return {re * (float)b, im * (float)b}; }
    complex_t operator/(float b) const { return {re / b, im / b}; }
    complex_t operator*(const complex_t& b) const { return {re * b.re - im * b.im, im * b.re + re * b.im}; }
    complex_t operator+(const complex_t& b) const { return {re + b.re, im + b.im}; }
    complex_t operator-(const complex_t& b) const { return {re - b.re, im - b.im}; }
    complex_t& operator+=(const complex_t& b) { re += b.re; im += b.im; return *this; }
    complex_t& operator-=(const complex_t& b) { re -= b.re; im -= b.im; return *this; }
    complex_t& operator*=(const float& b) { re *= b; im *= b; return *this; }
    complex_t conj() const { return {re, -im}; }
    float phase() const { return atan2f(im, re); }
    float amplitude() const { return sqrtf(re * re + im * im); }
};
struct stereo_t {
    float l, r;
    stereo_t operator*(float b) const { return {l * b, r * b}; }
    stereo_t operator+(const stereo_t& b) const { return {l + b.l, r + b.r}; }
    stereo_t operator-(const stereo_t& b) const { return {l - b.l, r - b.r}; }
};
static_assert(sizeof(complex_t) == 8 && sizeof(stereo_t) == 8, "interleaved float pairs");
}  // namespace dsp
