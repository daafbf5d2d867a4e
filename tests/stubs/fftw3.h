// Declaration-only stand-in for FFTW3's single-precision API, used ONLY by
// tests/test_overlay_syntax.py (`g++ -fsyntax-only` of the overlay inside the reference tree; FFTW is
// not installed in this image). Published fftw3.h signatures; nothing is defined, linked or run.
#pragma once
#include <cstddef>
typedef float fftwf_complex[2];
typedef struct fftwf_plan_s* fftwf_plan;
#define FFTW_FORWARD (-1)
#define FFTW_BACKWARD (+1)
#define FFTW_ESTIMATE (1U << 6)
void* fftwf_malloc(size_t n);
void fftwf_free(void* p);
fftwf_plan fftwf_plan_dft_1d(int n, fftwf_complex* in, fftwf_complex* out, int sign, unsigned flags);
void fftwf_execute(const fftwf_plan p);
void fftwf_destroy_plan(fftwf_plan p);
