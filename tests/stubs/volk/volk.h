// Declaration-only stand-in for VOLK's public header, used ONLY by tests/test_overlay_syntax.py to
// run `g++ -fsyntax-only` over the drop-in overlay placed into the reference tree (VOLK is not
// installed in this image). It declares the kernels the reference headers call with VOLK's
// published signatures (volk 2.x: volk_complex.h's lv_32fc_t = std::complex<float>); nothing here is
// defined, linked or executed, so it proves that the overlay and its callers type-check against the
// reference's block API -- never any arithmetic.
#pragma once
#include <complex>
#include <cstddef>
#include <cstdint>
typedef std::complex<float> lv_32fc_t;
inline lv_32fc_t lv_cmake(float r, float i) { return lv_32fc_t(r, i); }
size_t volk_get_alignment(void);
void* volk_malloc(size_t size, size_t alignment);
void volk_free(void* p);
void volk_32f_x2_dot_prod_32f(float* result, const float* input, const float* taps, unsigned int num_points);
void volk_32fc_32f_dot_prod_32fc(lv_32fc_t* result, const lv_32fc_t* input, const float* taps, unsigned int num_points);
void volk_32fc_x2_dot_prod_32fc(lv_32fc_t* result, const lv_32fc_t* input, const lv_32fc_t* taps, unsigned int num_points);
void volk_32fc_magnitude_32f(float* magnitudeVector, const lv_32fc_t* complexVector, unsigned int num_points);
void volk_32f_x2_interleave_32fc(lv_32fc_t* complexVector, const float* iBuffer, const float* qBuffer, unsigned int num_points);
void volk_32f_x2_subtract_32f(float* cVector, const float* aVector, const float* bVector, unsigned int num_points);
void volk_32f_x2_add_32f(float* cVector, const float* aVector, const float* bVector, unsigned int num_points);
void volk_32f_x2_multiply_32f(float* cVector, const float* aVector, const float* bVector, unsigned int num_points);
void volk_32f_s32f_multiply_32f(float* cVector, const float* aVector, const float scalar, unsigned int num_points);
void volk_32f_index_max_32u(uint32_t* target, const float* src0, uint32_t num_points);
void volk_8i_s32f_convert_32f(float* outputVector, const int8_t* inputVector, const float scalar, unsigned int num_points);
void volk_16i_s32f_convert_32f(float* outputVector, const int16_t* inputVector, const float scalar, unsigned int num_points);
void volk_32f_s32f_convert_8i(int8_t* outputVector, const float* inputVector, const float scalar, unsigned int num_points);
void volk_32f_s32f_convert_16i(int16_t* outputVector, const float* inputVector, const float scalar, unsigned int num_points);
void volk_32fc_x2_multiply_32fc(lv_32fc_t* cVector, const lv_32fc_t* aVector, const lv_32fc_t* bVector, unsigned int num_points);
void volk_32fc_32f_multiply_32fc(lv_32fc_t* cVector, const lv_32fc_t* aVector, const float* bVector, unsigned int num_points);
void volk_32fc_s32fc_x2_rotator_32fc(lv_32fc_t* outVector, const lv_32fc_t* inVector, const lv_32fc_t phase_inc, lv_32fc_t* phase,
                                     unsigned int num_points);
void volk_32fc_s32fc_x2_rotator2_32fc(lv_32fc_t* outVector, const lv_32fc_t* inVector, const lv_32fc_t* phase_inc, lv_32fc_t* phase,
                                      unsigned int num_points);
void volk_32fc_deinterleave_real_32f(float* iBuffer, const lv_32fc_t* complexVector, unsigned int num_points);
void volk_32fc_conjugate_32fc(lv_32fc_t* cVector, const lv_32fc_t* aVector, unsigned int num_points);
void volk_32f_accumulator_s32f(float* result, const float* inputBuffer, unsigned int num_points);
