/*
 * sdr_oracle.h -- CPU restatement of SDR++'s streaming-DSP hot path.
 *
 * TEST INFRASTRUCTURE ONLY. This library is the parity checker and the CPU
 * baseline for bench.py's cpu_baseline leg; the product path (libsdrgpu.so)
 * never links or calls it. Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it.
 *
 * Every function cites the reference file:line it restates (paths relative to
 * the qrp73/SDRPP tree, core/src/...). Parity status: the reference hot path
 * cannot be compiled here (VOLK/FFTW/fmt absent) and ships no DSP
 * tests or golden vectors, so the arithmetic that lives in VOLK/FFTW is
 * restated from its published semantics and pinned by the known-answer
 * properties and committed fixtures described in DESIGN.md ("parity pinned by
 * known answers, reference binary unavailable").
 *
 * Two accumulation modes for every dot product:
 *   precise=1  fp64 accumulation, rounded once to float (the parity truth)
 *   precise=0  fp32, 8 independent accumulators (VOLK-class SIMD speed; used
 *              only for the CPU-baseline timing)
 */
#ifndef SDR_ORACLE_H
#define SDR_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- window (core/src/dsp/window/window.h:22-64, cosine.h:7-16) ---- */
enum { ORC_WIN_RECTANGULAR = 0, ORC_WIN_HAMMING, ORC_WIN_HANN, ORC_WIN_BLACKMAN,
       ORC_WIN_NUTTALL, ORC_WIN_BLACKMAN_HARRIS4, ORC_WIN_BLACKMAN_HARRIS7 };
double orc_window_value(int type, double n, double N);
void   orc_create_window(int type, float* buffer, int size, int centered);

/* ---- framing (core/src/signal_path/iq_frontend.h:56-60) ---- */
void orc_gen_reshape_params(double sampleRate, int size, double rate, int* skip, int* nz);

/* ---- taps (core/src/dsp/taps/ windowed_sinc, low_pass, high_pass, band_pass) ---- */
int orc_estimate_tap_count(double transWidth, double samplerate);
int orc_windowed_sinc(int count, double omega, double norm, float* out);          /* nuttall window */
int orc_low_pass(double cutoff, double transWidth, double sampleRate, int odd, float* out);
int orc_high_pass(double cutoff, double transWidth, double sampleRate, int odd, float* out);
int orc_band_pass_f(double start, double stop, double transWidth, double sampleRate, int odd, float* out);
int orc_band_pass_c(double start, double stop, double transWidth, double sampleRate, int odd, float* out /*2*count*/);
int orc_decim_plan(int ratio, int* decims, int* ntaps, const float** taps);        /* multirate/decim/plans.h */

/* ---- ingest converters (source_modules/file_source/src/main.cpp:361-542) ---- */
void orc_u8_to_f32(const uint8_t* in, float* out, long n);
void orc_i16_to_f32(const int16_t* in, float* out, long n);
void orc_i24_to_f32(const uint8_t* in, float* out, long n);
void orc_i32_to_f32(const int32_t* in, float* out, long n);
void orc_f64_to_f32(const double* in, float* out, long n);
void orc_i8_to_f32(const int8_t* in, float* out, long n);   /* hackrf_source main.cpp:386 */

/* ---- spectrum (core/src/signal_path/iq_frontend.cpp:230-249, 272-296) ---- */
void orc_fft_c2c(const float* in, float* out, int N);        /* fp32 forward DFT, radix-2 */
void orc_fft_c2c_f64(const double* in, double* out, int N);  /* fp64 forward DFT, radix-2 */
void orc_power_spectrum_db(const float* X, float* out, int N);
void orc_fft_logmag(const float* in, int nz, int N, const float* window, float* work, float* out_db);

/* ---- stateful blocks ---- */
enum { ORC_F32 = 0, ORC_C64 = 1 };
typedef struct orc_fir orc_fir;
orc_fir* orc_fir_create(int dtype, int ttype, const float* taps, int ntaps, int decim, int precise);
void     orc_fir_set_taps(orc_fir* f, const float* taps, int ntaps);
void     orc_fir_reset(orc_fir* f);
int      orc_fir_process(orc_fir* f, const float* in, int count, float* out);
void     orc_fir_destroy(orc_fir* f);

typedef struct orc_xlator orc_xlator;
orc_xlator* orc_xlator_create(double offset_rad);
orc_xlator* orc_xlator_create_fast(double offset_rad);
void orc_xlator_set_offset(orc_xlator* x, double offset_rad);
void orc_xlator_reset(orc_xlator* x);
int  orc_xlator_process(orc_xlator* x, const float* in, int count, float* out);
double orc_xlator_effective_omega(double offset_rad);
void orc_xlator_destroy(orc_xlator* x);

typedef struct orc_quad orc_quad;
orc_quad* orc_quad_create(double deviation_rad);
void orc_quad_reset(orc_quad* q);
int  orc_quad_process(orc_quad* q, const float* in, int count, float* out);
void orc_quad_destroy(orc_quad* q);

typedef struct orc_pdec orc_pdec;            /* multirate/power_decimator.h */
orc_pdec* orc_pdec_create(int dtype, int ratio, int precise);
int  orc_pdec_process(orc_pdec* p, const float* in, int count, float* out);
void orc_pdec_reset(orc_pdec* p);
void orc_pdec_destroy(orc_pdec* p);

typedef struct orc_poly orc_poly;            /* multirate/polyphase_resampler.h */
orc_poly* orc_poly_create(int dtype, int interp, int decim, const float* taps, int ntaps, int precise);
int  orc_poly_process(orc_poly* p, const float* in, int count, float* out);
void orc_poly_reset(orc_poly* p);
void orc_poly_destroy(orc_poly* p);

typedef struct orc_rres orc_rres;            /* multirate/rational_resampler.h */
orc_rres* orc_rres_create(int dtype, double inSr, double outSr, int precise);
int  orc_rres_process(orc_rres* r, const float* in, int count, float* out);
int  orc_rres_info(orc_rres* r, int* mode, int* predec, int* interp, int* decim, int* ntaps);
void orc_rres_destroy(orc_rres* r);

typedef struct orc_vfo orc_vfo;              /* channel/rx_vfo.h */
orc_vfo* orc_vfo_create(double inSr, double outSr, double bw, double offset, int precise);
int  orc_vfo_process(orc_vfo* v, const float* in, int count, float* out);
void orc_vfo_destroy(orc_vfo* v);

typedef struct orc_wfm orc_wfm;              /* demod/broadcast_fm.h (mono path) */
orc_wfm* orc_wfm_create(double deviation, double samplerate, int lowPass, int precise);
int  orc_wfm_process(orc_wfm* w, const float* in, int count, float* out_stereo);
void orc_wfm_destroy(orc_wfm* w);
typedef struct orc_wfms orc_wfms;            /* demod/broadcast_fm.h, stereo or mono (no RDS) */
orc_wfms* orc_wfms_create(double deviation, double samplerate, int stereo, int lowPass, int precise);
int  orc_wfms_process(orc_wfms* w, const float* in, int count, float* out_stereo);
void orc_wfms_destroy(orc_wfms* w);

typedef struct orc_fm orc_fm;                /* demod/fm.h */
orc_fm* orc_fm_create(double samplerate, double bandwidth, int lowPass, int highPass, int precise);
int  orc_fm_process(orc_fm* f, const float* in, int count, float* out_mono);
void orc_fm_destroy(orc_fm* f);

/* loops / IIRs: serial reference semantics */
typedef struct orc_agc orc_agc;              /* loop/agc.h */
orc_agc* orc_agc_create(int dtype, double setPoint, double attack, double decay, double maxGain, double maxOutputAmp, double initGain);
void orc_agc_set_enabled(orc_agc* a, int en);
void orc_agc_set_gain(orc_agc* a, float g);
float orc_agc_get_gain(orc_agc* a);
int  orc_agc_process(orc_agc* a, const float* in, int count, float* out);
void orc_agc_destroy(orc_agc* a);

typedef struct orc_dcb orc_dcb;              /* correction/dc_blocker.h */
orc_dcb* orc_dcb_create(int dtype, double rate);
int  orc_dcb_process(orc_dcb* d, const float* in, int count, float* out);
void orc_dcb_destroy(orc_dcb* d);

typedef struct orc_am orc_am;                /* demod/am.h (float output) */
orc_am* orc_am_create(int agcMode, double bandwidth, double agcAttack, double agcDecay, double dcBlockRate, double samplerate, int precise);
int  orc_am_process(orc_am* a, const float* in, int count, float* out);
void orc_am_destroy(orc_am* a);

typedef struct orc_ssb orc_ssb;              /* demod/ssb.h (float output) */
orc_ssb* orc_ssb_create(int mode, double bandwidth, double samplerate, int agcEnabled, double agcAttack, double agcDecay);
int  orc_ssb_process(orc_ssb* s, const float* in, int count, float* out);
void orc_ssb_destroy(orc_ssb* s);

/* compression (dsp/compression/sample_stream_{compressor,decompressor}.h) */
int orc_compress(int pcmType, const float* in, int count, uint8_t* out);
int orc_decompress(const uint8_t* in, int nbytes, float* out);

/* C4 channelizer definition: channel k = FrequencyXlator(-k fs/M) with an
 * EXACT NCO (angle 2 pi (k n mod M)/M) -> DecimatingFIR<complex_t, float>(h, M)
 * (frequency_xlator.h:43-50, decimating_fir.h:45-68), fp64 throughout, from reset.
 * out: [nchan][frames] complex (re, im doubles), frames = ceil(count / M). */
int orc_channelize(const float* in, long count, const float* h, int ntaps, int M, const int* chans, int nchan,
                   double* out);

typedef struct orc_deemp orc_deemp;          /* filter/deephasis.h, channels 1 (float) or 2 (stereo_t) */
orc_deemp* orc_deemp_create(int channels, double tau, double samplerate);
int  orc_deemp_process(orc_deemp* d, const float* in, int count, float* out);
void orc_deemp_destroy(orc_deemp* d);
/* gui/widgets/fft_scaler.h doZoom */
int orc_zoom(const float* data, int fftSize, double viewOffset, double viewBandwidth, double wholeBandwidth,
             int outSize, float* out);

/* WaterFall::pushFFT consumers (gui/widgets/waterfall.cpp) */
void orc_colormap(const float* in, long n, float wfMin, float wfMax, const unsigned* pallet, int res, unsigned* out);
void orc_fft_smooth_hold(float* rows, int nrows, int width, int smoothing, float alpha, float beta, float* smooth,
                         int holdOn, float holdSpeed, float* hold);
void orc_vfo_signal_info(const float* line, int fftSize, double wholeBandwidth, double centerOffset, double bandwidth,
                         float* strength, float* snr);

typedef struct orc_ddcfm orc_ddcfm;          /* C3: xlator -> DecimatingFIR -> Quadrature */
orc_ddcfm* orc_ddcfm_create(double offsetRad, const float* taps, int ntaps, int decim, double deviationRad, int precise);
int  orc_ddcfm_process(orc_ddcfm* d, const float* in, int count, float* out);
void orc_ddcfm_destroy(orc_ddcfm* d);

/* recorder WAV encoders (utils/wav.cpp:296-336): kind 0 u8, 1 i16, 2 i24, 3 i32, 4 f32 */
int orc_wav_encode(int kind, const float* in, int n, uint8_t* out);

/* C5 per-stream chain used as the CPU baseline: 64k BH7 spectrum (back-to-back
 * frames) + RxVFO(plan_256 + 91-tap LPF) + BroadcastFM mono. Returns audio pairs. */
typedef struct orc_chain orc_chain;
orc_chain* orc_chain_create(double fs, int fftSize, double vfoOffset, int precise);
long orc_chain_process(orc_chain* c, const float* in, long count, float* spectra, long maxFrames, float* audio);
void orc_chain_destroy(orc_chain* c);

#ifdef __cplusplus
}
#endif
#endif
