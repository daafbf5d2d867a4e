/*
 * sdrgpu.h -- C ABI of the MI355X (gfx950) streaming-DSP hot path of SDR++.
 *
 * Plain pointers and sizes only; no C++ or torch types. Two calling styles:
 *   *_process(...)      drop-in for the reference's host-buffer process(count, in, out)
 *                       (synchronous, host pointers; staged through pinned memory)
 *   *_process_dev(...)  device-resident batches on a caller stream (hipStream_t as void*,
 *                       NULL = the handle's own stream); asynchronous, host-side state
 *                       (decimation offsets, output counts) is updated at call time.
 * Every call returns >= 0 on success (an output count where meaningful) or a
 * negative SDRGPU_E* code; sdrgpu_last_error() gives the thread's last message.
 * A handle is used by one thread at a time (the reference's one-worker-per-block
 * model, core/src/dsp/block.h:70-76).
 *
 * Reference interfaces replaced (paths in qrp73/SDRPP, core/src/...):
 *   spectrum  : IQFrontEnd::handler + updateFFTSize, signal_path/iq_frontend.cpp:230-249,272-296
 *   windows   : dsp::window::createWindow, dsp/window/window.h:38-64
 *   taps      : dsp::taps::{lowPass,highPass,bandPass,windowedSinc}, dsp/taps/
 *   FIR       : dsp::filter::FIR::process, dsp/filter/fir.h:62-83
 *   decim FIR : dsp::filter::DecimatingFIR::process, dsp/filter/decimating_fir.h:45-68
 *   xlator    : dsp::channel::FrequencyXlator::process, dsp/channel/frequency_xlator.h:43-50
 *   power dec : dsp::multirate::PowerDecimator::process, dsp/multirate/power_decimator.h:51-70
 *   polyphase : dsp::multirate::PolyphaseResampler::process, dsp/multirate/polyphase_resampler.h:69-99
 *   rational  : dsp::multirate::RationalResampler, dsp/multirate/rational_resampler.h:83-167
 *   VFO       : dsp::channel::RxVFO::process, dsp/channel/rx_vfo.h:89-100
 *   quadrature: dsp::demod::Quadrature::process, dsp/demod/quadrature.h:41-56
 *   FM        : dsp::demod::FM<float>::process, dsp/demod/fm.h:86-103
 *   WFM       : dsp::demod::BroadcastFM::process (mono), dsp/demod/broadcast_fm.h:144-215
 *   ingest    : file_source converters, source_modules/file_source/src/main.cpp:361-542
 */
#ifndef SDRGPU_H
#define SDRGPU_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SDRGPU_VERSION 100

enum {
    SDRGPU_OK = 0,
    SDRGPU_EARG = -1,     /* invalid argument (reference: assert / std::runtime_error) */
    SDRGPU_EHIP = -2,     /* HIP runtime error (name in sdrgpu_last_error) */
    SDRGPU_ENOMEM = -3,
    SDRGPU_ESTATE = -4,   /* wrong handle kind / not initialised */
    SDRGPU_ENODEV = -5,
    SDRGPU_ETIMEOUT = -6  /* a peer rank did not answer within the deadline (gather: communicator aborted) */
};

/* element types (dsp::complex_t is {float re, im}, dsp/types.h:6; stereo_t {float l, r}) */
enum { SDRGPU_F32 = 0, SDRGPU_C64 = 1 };

/* window ids = dsp::window::windowType (dsp/window/window.h:27-35) */
enum { SDRGPU_WIN_RECTANGULAR = 0, SDRGPU_WIN_HAMMING, SDRGPU_WIN_HANN, SDRGPU_WIN_BLACKMAN,
       SDRGPU_WIN_NUTTALL, SDRGPU_WIN_BLACKMAN_HARRIS4, SDRGPU_WIN_BLACKMAN_HARRIS7 };

/* ----------------------------------------------------------- runtime ---- */
int         sdrgpu_version(void);
const char* sdrgpu_last_error(void);
int         sdrgpu_device_count(void);
int         sdrgpu_malloc(int device, void** dptr, size_t bytes);
int         sdrgpu_free(void* dptr);
int         sdrgpu_memcpy_h2d(void* dst, const void* src, size_t bytes, void* stream);
int         sdrgpu_memcpy_d2h(void* dst, const void* src, size_t bytes, void* stream);
int         sdrgpu_stream_create(int device, void** stream);
int         sdrgpu_stream_destroy(void* stream);
int         sdrgpu_stream_synchronize(void* stream);
int         sdrgpu_host_register(void* ptr, size_t bytes);   /* pin a dsp::stream buffer */
int         sdrgpu_host_unregister(void* ptr);
int         sdrgpu_host_alloc(void** ptr, size_t bytes);   /* pinned + registered (DMA'd directly) */
int         sdrgpu_host_free(void* ptr);

/* ------------------------------------------- host-side design (exact) ---- */
/* Bit-exact restatements evaluated on the host, as the reference does. */
int  sdrgpu_create_window(int type, float* buffer, int size, int centered);          /* window.h:38 */
void sdrgpu_gen_reshape_params(double sampleRate, int size, double rate, int* skip, int* nz); /* iq_frontend.h:56 */
int  sdrgpu_taps_estimate_count(double transWidth, double sampleRate);               /* estimate_tap_count.h:4 */
int  sdrgpu_taps_windowed_sinc(int count, double omega, double norm, float* out);   /* windowed_sinc.h:9 (window::nuttall) */
int  sdrgpu_taps_low_pass(double cutoff, double transWidth, double sampleRate, int odd, float* out); /* low_pass.h:7; out NULL -> count */
int  sdrgpu_taps_high_pass(double cutoff, double transWidth, double sampleRate, int odd, float* out); /* high_pass.h:7 */
int  sdrgpu_taps_band_pass_f(double start, double stop, double transWidth, double sampleRate, int odd, float* out); /* band_pass.h:11 */
int  sdrgpu_taps_band_pass_c(double start, double stop, double transWidth, double sampleRate, int odd, float* out);
int  sdrgpu_decim_plan(int ratio, int* decims, int* ntaps, const float** taps);      /* decim/plans.h */

/* --------------------------------------------------------- spectrum ---- */
/* Window * FFT(N, forward, unnormalised) * 10*log10(|X|^2) of nz <= N samples,
 * zero-padded to N (iq_frontend.cpp:230-249 + :295). N = 2^k, 64 <= N <= 2^20. */
typedef struct sdrgpu_fft sdrgpu_fft;
typedef struct sdrgpu_block sdrgpu_block;   /* stream blocks (below) */
int sdrgpu_fft_create(sdrgpu_fft** h, int device, int fftSize, int nz, int windowType);
int sdrgpu_fft_set_window(sdrgpu_fft* h, const float* window, int nz);   /* exact host floats */
int sdrgpu_fft_set_window_type(sdrgpu_fft* h, int windowType, int nz);
/* device batch: frame f starts at in + f*frameStride complex samples; out: frames x N floats */
int sdrgpu_fft_execute_dev(sdrgpu_fft* h, const void* in, long long frameStride, int frames, float* out, void* stream);
/* rows + the waterfall's full-span zoom rows (fft_scaler(0, bw, bw, N, zoomSize).doZoom of each
 * row, gui/widgets/fft_scaler.h:27-64) into zoomOut (frames x zoomSize floats). With N = 65536 and
 * zoomSize = 2048 the zoom is fused into the transform's last pass. */
int sdrgpu_fft_execute_zoom_dev(sdrgpu_fft* h, const void* in, long long frameStride, int frames, float* out,
                                float* zoomOut, int zoomSize, void* stream);
/* spectrum + one RxVFO over the same device batch of `frames` back-to-back frames (frame stride
 * N, nz = N: fftRate = fs / N), the VFO reading the batch in place as the front end's splitter
 * feeds both (iq_frontend.cpp:15-52, splitter.h:46-60), on one stream. Returns the VFO's output
 * count (vfoOut). On the 64k plan with an RxVFO whose first stage is the D = 32 row decimator
 * (61.44 MS/s -> 240 kHz) that stage runs inside the spectrum launches, so the batch is read from
 * HBM once; otherwise the spectrum and the VFO run as two launch groups. */
int sdrgpu_fft_execute_vfo_dev(sdrgpu_fft* h, const void* in, int frames, float* out, sdrgpu_block* vfo,
                               void* vfoOut, void* stream);
/* the same + the waterfall's full-span zoom rows (as sdrgpu_fft_execute_zoom_dev; zoomOut may be NULL) */
int sdrgpu_fft_execute_zoom_vfo_dev(sdrgpu_fft* h, const void* in, int frames, float* out, float* zoomOut,
                                    int zoomSize, sdrgpu_block* vfo, void* vfoOut, void* stream);
/* (not in the reference; its IQFrontEnd hands the spectrum and each VFO to blocks on their own
 * threads, iq_frontend.cpp:15-52) A second stream for sdrgpu_fft_execute_zoom_vfo_dev calls with zoom
 * rows: the VFO's later stages and the zoom fold run on `tailStream`, so they overlap the next call's
 * spectrum launch on the call's stream instead of following it. Then `out` (the dB rows) is complete
 * on the call's stream, while `vfoOut` and `zoomOut` are complete on `tailStream`: their consumers
 * (a demodulator, a gather) must run on, or wait for, `tailStream`. Results are bit-identical to the
 * one-stream calls. NULL turns it off (waiting for tails in flight). */
int sdrgpu_fft_set_tail_stream(sdrgpu_fft* h, void* tailStream);
/* (measurement, not in the reference) HIP events around each call's spectrum launch group -- the
 * fused VFO stage included, the VFO's later stages not; group_times returns the last
 * min(n, calls, 256) group times in ms, oldest first, waiting for them */
int sdrgpu_fft_set_timing(sdrgpu_fft* h, int on);
int sdrgpu_fft_group_times(sdrgpu_fft* h, float* ms, int n);
/* drop-in for IQFrontEnd::handler: in = host complex_t[nz]; out = host float[N] or NULL
 * (acquireFFTBuffer may return NULL; the spectrum is then computed but not written). */
int sdrgpu_fft_logmag(sdrgpu_fft* h, const void* in, float* out);
int sdrgpu_fft_size(sdrgpu_fft* h);
/* spectrum arithmetic (not in the reference: the north_star's <= 1 ulp parity mode):
 * 0 = fp32 kernels (default; FFTW-class accuracy), 1 = fp64 interior: the reference's fp32 window
 * product (volk_32fc_32f_multiply_32fc), then fp64 butterflies, twiddles, |X|^2 and 10 log10,
 * rounded once to fp32 -- the correctly rounded dB of the exact DFT up to ~1e-15. Waits for the
 * device; the zoom rows of sdrgpu_fft_execute_zoom_dev are then computed unfused. */
int sdrgpu_fft_set_precision(sdrgpu_fft* h, int mode);
int sdrgpu_fft_get_precision(sdrgpu_fft* h);
/* 64k transform form (not in the reference; FFTW picks its plan per size the same way). The 64k
 * plan has two fp32 kernels that round differently: the one-pass transform (one radix-4 DIF step
 * into four 16k sub-transforms, fft_1p_kernel) and the two-pass 256 x 256 four-step launches. Both
 * meet the spectrum parity bar against the exact DFT, but they are not bit-identical to each other:
 * rows of the same frame differ by at most 0.05 dB anywhere and 1e-3 dB within 40 dB of the frame's
 * peak (further down, each form's fp32 error is a growing fraction of the bin: 60 dB below a noise
 * frame's peak two rows were measured 5.4e-3 dB apart) (tests/test_gpu_parity.py::
 * test_spectrum_64k_rows_vs_call_size, test_spectrum_onepass_rows_and_zoom). mode 2 (the default) picks
 * per call: one-pass for calls of >= 64 frames, two-pass below (a reference-size block of 4.7
 * frames runs faster there), so a stream's 64k rows then depend on how it is batched into calls.
 * mode 1 (always one-pass) or 0 (always two-pass) pins the form per plan: rows then depend only on
 * the frame. Other sizes have one form and ignore the mode. The device front end
 * (sdrgpu_frontend_*) pins its plans to 0. Returns the previous mode. */
int sdrgpu_fft_set_kernel(sdrgpu_fft* h, int mode);
int sdrgpu_fft_destroy(sdrgpu_fft* h);

/* ---------------------------------------------------- stream blocks ---- */
/* FrequencyXlator (offset in rad/sample, like init(in, offset)) */
int sdrgpu_xlator_create(sdrgpu_block** h, int device, double offsetRad);
int sdrgpu_xlator_set_offset(sdrgpu_block* h, double offsetRad);
/* FIR<D,T> (decim = 1) and DecimatingFIR<D,T>: dtype/ttype SDRGPU_F32 or SDRGPU_C64 */
int sdrgpu_fir_create(sdrgpu_block** h, int device, int dtype, int ttype, const float* taps, int ntaps, int decim);
int sdrgpu_fir_set_taps(sdrgpu_block* h, const float* taps, int ntaps);
int sdrgpu_fir_set_decimation(sdrgpu_block* h, int decim);
/* Quadrature (deviation in rad/sample) */
int sdrgpu_quadrature_create(sdrgpu_block** h, int device, double deviationRad);
int sdrgpu_quadrature_set_deviation(sdrgpu_block* h, double deviationRad);
/* PowerDecimator<T> (ratio = 1 or 2^k <= 8192), PolyphaseResampler<T>, RationalResampler<T> */
int sdrgpu_power_decimator_create(sdrgpu_block** h, int device, int dtype, int ratio);
int sdrgpu_polyphase_resampler_create(sdrgpu_block** h, int device, int dtype, int interp, int decim, const float* taps, int ntaps);
int sdrgpu_rational_resampler_create(sdrgpu_block** h, int device, int dtype, double inSamplerate, double outSamplerate);
/* RxVFO: xlator(-offset) -> rational resampler -> LPF(bw/2) if bw != outSr */
int sdrgpu_rxvfo_create(sdrgpu_block** h, int device, double inSamplerate, double outSamplerate, double bandwidth, double offset);
int sdrgpu_rxvfo_set_offset(sdrgpu_block* h, double offset);
/* Fused DDC: xlator(offsetRad) -> DecimatingFIR<complex_t,float>(taps, decim); complex_t out
 * (frequency_xlator.h:43-50 + decimating_fir.h:45-68 in one kernel) */
int sdrgpu_ddc_create(sdrgpu_block** h, int device, double offsetRad, const float* taps, int ntaps, int decim);
/* Fused DDC: xlator(offsetRad) -> DecimatingFIR<complex_t,float>(taps, decim) -> Quadrature(deviationRad); float out */
int sdrgpu_ddc_fm_create(sdrgpu_block** h, int device, double offsetRad, const float* taps, int ntaps, int decim, double deviationRad);
/* FM<float> (demod/fm.h) and BroadcastFM mono (stereo_t out, broadcast_fm.h) */
int sdrgpu_fm_create(sdrgpu_block** h, int device, double samplerate, double bandwidth, int lowPass, int highPass);
int sdrgpu_wfm_create(sdrgpu_block** h, int device, double deviation, double samplerate, int lowPass);
/* Serial loops (one workgroup per stream; bit-identical to the reference arithmetic) */
/* loop::AGC<T> (loop/agc.h:13-147); dtype F32 or C64; setGain latched at the next process() */
int sdrgpu_agc_create(sdrgpu_block** h, int device, int dtype, double setPoint, double attack, double decay,
                      double maxGain, double maxOutputAmp, double initGain);
int sdrgpu_agc_set_params(sdrgpu_block* h, double setPoint, double attack, double decay, double maxGain,
                          double maxOutputAmp, double initGain);   /* agc.h:44-79 setters (state kept) */
int sdrgpu_agc_set_enabled(sdrgpu_block* h, int enabled);      /* agc.h:38 */
int sdrgpu_agc_set_gain(sdrgpu_block* h, float gain);          /* agc.h:31 */
int sdrgpu_agc_get_gain(sdrgpu_block* h, float* gain);         /* agc.h:28 (synchronises) */
/* correction::DCBlocker<T> (correction/dc_blocker.h:17-60); rate = rate_hz / samplerate */
int sdrgpu_dc_blocker_create(sdrgpu_block** h, int device, int dtype, double rate);
int sdrgpu_dc_blocker_set_rate(sdrgpu_block* h, double rate);   /* dc_blocker.h:30 (also on an AM handle) */
/* demod::AM<T> (demod/am.h:27-142): agcMode 0 OFF, 1 CARRIER, 2 AUDIO; stereo != 0 -> stereo_t out */
int sdrgpu_am_create(sdrgpu_block** h, int device, int agcMode, double bandwidth, double agcAttack, double agcDecay,
                     double dcBlockRate, double samplerate, int stereo);
/* demod::SSB<T> (demod/ssb.h:20-105): mode 0 USB, 1 LSB, 2 DSB; stereo != 0 -> stereo_t out */
int sdrgpu_ssb_create(sdrgpu_block** h, int device, int mode, double bandwidth, double samplerate, int agcEnabled,
                      double agcAttack, double agcDecay, int stereo);
/* AGC inside an AM / SSB handle: which 0 = first AGC (AM carrier AGC, SSB AGC), 1 = last (AM audio AGC);
 * am.h:63-97 setAGCGain/getAGCGain/setAGCAttack/setAGCDecay, ssb.h:62-84 */
int sdrgpu_demod_agc_set_gain(sdrgpu_block* h, int which, float gain);
int sdrgpu_demod_agc_get_gain(sdrgpu_block* h, int which, float* gain);
int sdrgpu_demod_agc_set_enabled(sdrgpu_block* h, int which, int enabled);
int sdrgpu_demod_agc_set_attack_decay(sdrgpu_block* h, double attack, double decay);
/* demod::BroadcastFM with the stereo decoder (broadcast_fm.h:34-60, 144-215): quadrature ->
 * pilot band-pass (complex taps) -> PLL (loop/pll.h) -> L+R / L-R matrix -> audio low-pass;
 * stereo_t out. stereo = 0 gives the mono path (= sdrgpu_wfm_create). */
int sdrgpu_broadcast_fm_create(sdrgpu_block** h, int device, double deviation, double samplerate, int stereo, int lowPass);
/* RDS branch (broadcast_fm.h:121-127, 164-171, 193-203): setRDSOut; when on, every process call
 * also produces complex_t RDS baseband = RationalResampler(fs -> 5 kHz)(FrequencyXlator(-57 kHz)(MPX)),
 * read with rds_dev (device pointer + count of the last call) or read_rds (host copy) */
int sdrgpu_broadcast_fm_set_rds(sdrgpu_block* h, int enabled);
int sdrgpu_broadcast_fm_rds_dev(sdrgpu_block* h, const void** out, int* n);
int sdrgpu_broadcast_fm_read_rds(sdrgpu_block* h, void* out, int max);
/* filter::Deemphasis<T> (filter/deephasis.h:57-93): dtype F32 (float) or C64 (stereo_t);
 * serial recurrence, bit-identical to the reference arithmetic */
int sdrgpu_deemphasis_create(sdrgpu_block** h, int device, int dtype, double tau, double samplerate);
int sdrgpu_deemphasis_set(sdrgpu_block* h, double tau, double samplerate);   /* setTau / setSamplerate */
/* M-channel critically sampled polyphase channelizer (BASELINE C4): channel k of output frame
 * m is FrequencyXlator(-k fs/M) -> DecimatingFIR<complex_t,float>(taps, M) (frequency_xlator.h:43,
 * decimating_fir.h:45) with an exact NCO; taps <= 16 M (bank layout polyphase_bank.h:32).
 * Output: frames x M complex, out[m*M + k]; out_count = frames * M. M in {256, 512, 1024}. */
int sdrgpu_channelizer_create(sdrgpu_block** h, int device, int channels, const float* taps, int ntaps);
/* The channelizer's per-frame M-point DFT (same definition as above): mode 0 = LDS FFT (default),
 * 1 = the polyphase filterbank "cast as batched MFMA GEMM" (BASELINE C4): 1024 = 32 x 32, two
 * complex 32x32 products per frame on v_mfma_f32_16x16x4_f32. M = 1024 only. */
int sdrgpu_channelizer_set_dft(sdrgpu_block* h, int mode);

int sdrgpu_block_process(sdrgpu_block* h, const void* in, int count, void* out);      /* host buffers */
int sdrgpu_block_process_dev(sdrgpu_block* h, const void* in, int count, void* out, void* stream);
int sdrgpu_block_out_count(sdrgpu_block* h, int count);   /* exact output count of the next call */
int sdrgpu_block_reset(sdrgpu_block* h);
int sdrgpu_block_destroy(sdrgpu_block* h);

/* ------------------------------------------------- device IQ front end ---- */
/* IQFrontEnd's data path on the device (signal_path/iq_frontend.cpp:15-52, 115-249; SURVEY
 * 8f rank 1): ingest conversion -> [PowerDecimator] -> [DCBlocker] -> [Conjugate] -> VFOs
 * (RxVFO, read in place) + spectrum frames (Reshaper keep = nz / skip from genReshapeParams,
 * window * FFT * log-power). Replaces the SampleFrameBuffer -> Splitter -> Reshaper memcpy
 * fan-out: one H2D per sample, every consumer reads the block from HBM.
 * kind: -1 complex float, else SDRGPU_CONV_* (interleaved IQ of that sample format). */
typedef struct sdrgpu_frontend sdrgpu_frontend;
int sdrgpu_frontend_create(sdrgpu_frontend** f, int device, double sampleRate, int decimRatio, int dcBlocking,
                           int fftSize, double fftRate, int windowType);                    /* IQFrontEnd::init */
int sdrgpu_frontend_destroy(sdrgpu_frontend* f);
int sdrgpu_frontend_configure(sdrgpu_frontend* f, double sampleRate, int decimRatio, int dcBlocking); /* setSampleRate/setDecimation/setDCBlocking */
int sdrgpu_frontend_set_invert_iq(sdrgpu_frontend* f, int enabled);                       /* setInvertIQ */
int sdrgpu_frontend_set_fft(sdrgpu_frontend* f, int fftSize, double fftRate, int windowType);  /* setFFTSize/Rate/Window */
int sdrgpu_frontend_framing(sdrgpu_frontend* f, int* nz, int* skip, double* effectiveSampleRate);
int sdrgpu_frontend_add_vfo(sdrgpu_frontend* f, int* id, double outSampleRate, double bandwidth, double offset); /* addVFO */
int sdrgpu_frontend_remove_vfo(sdrgpu_frontend* f, int id);                                /* removeVFO */
int sdrgpu_frontend_set_vfo_offset(sdrgpu_frontend* f, int id, double offset);
/* push a block; returns the number of spectrum rows completed by it */
int sdrgpu_frontend_push(sdrgpu_frontend* f, const void* in, int count, int kind);          /* host block (synchronous) */
int sdrgpu_frontend_push_dev(sdrgpu_frontend* f, const void* in, int count, int kind, void* stream); /* device block (async) */
int sdrgpu_frontend_spectra_dev(sdrgpu_frontend* f, const float** rows, int* nrows);       /* returns N */
int sdrgpu_frontend_read_spectra(sdrgpu_frontend* f, float* out, int maxRows);
int sdrgpu_frontend_vfo_dev(sdrgpu_frontend* f, int id, const void** out, int* n);
int sdrgpu_frontend_read_vfo(sdrgpu_frontend* f, int id, void* out, int max);
/* host copy of the last push's preprocessed IQ (what bound IQ streams receive, iq_frontend.cpp:114-120) */
int sdrgpu_frontend_read_iq(sdrgpu_frontend* f, void* out, int max);
/* Pipelined host call style (the IQFrontEnd drop-in's worker, round 3): submit enqueues a host
 * block's H2D on the front end's copy stream, its processing and the read-back of its rows, VFO
 * outputs and (flags & SDRGPU_FE_IQ) preprocessed IQ into pinned result slots, and returns a
 * ticket without waiting; block k + 1's H2D overlaps block k's kernels and read-back. collect
 * waits for a ticket and returns its row count with pinned host pointers to its results (valid
 * until release). At most two tickets are in flight: release(k) before submitting block k + 2.
 * A registered (sdrgpu_host_register / sdrgpu_host_alloc) `in` is DMA'd directly and must stay
 * untouched until its ticket is collected; any other `in` is staged and may be reused at once. */
#define SDRGPU_FE_IQ 1
int sdrgpu_frontend_submit(sdrgpu_frontend* f, const void* in, int count, int kind, int flags);
int sdrgpu_frontend_collect(sdrgpu_frontend* f, int ticket, const float** rows, const void** iq, int* niq);
int sdrgpu_frontend_collected_vfo(sdrgpu_frontend* f, int ticket, int id, const void** out, int* n);
int sdrgpu_frontend_release(sdrgpu_frontend* f, int ticket);

/* ------------------------------------------ spectra gather (multi-GPU) ---- */
/* Independent IQ streams run one per GPU; the only collective is a gather of their
 * spectrum rows to rank 0 (the display) over RCCL / xGMI. Rank 0 makes a communicator id, the
 * host hands it to every rank out of band, each rank creates its handle on its own GPU.
 * gather_rows: `count` device floats of this rank -> rank 0's out[r * count + i] (out: world x
 * count device floats, rank 0 only), asynchronous on `stream` (RCCL send/recv in one group).
 * RCCL is loaded at first use; without it these calls fail with SDRGPU_ESTATE. */
#define SDRGPU_GATHER_ID_BYTES 128
typedef struct sdrgpu_gather sdrgpu_gather;
int sdrgpu_gather_get_id(void* id /* SDRGPU_GATHER_ID_BYTES */);
/* Every wait on the peers has a deadline (SDRGPU_GATHER_TIMEOUT_S, default 120 s; set_timeout per
 * handle): create and rows poll the non-blocking communicator, wait polls `stream`; on expiry the
 * communicator is aborted and the call returns SDRGPU_ETIMEOUT naming the rank (the reference never
 * blocks forever on a stopped peer either: utils/threading.h:53-62, dsp/stream.h:94-116). After a
 * failure the handle accepts only destroy. create's device < 0: the thread's current device. */
int sdrgpu_gather_create(sdrgpu_gather** g, int device, int rank, int world, const void* id);
int sdrgpu_gather_set_timeout(sdrgpu_gather* g, double seconds);
int sdrgpu_gather_rows(sdrgpu_gather* g, const float* rows, long long count, float* out, void* stream);
int sdrgpu_gather_wait(sdrgpu_gather* g, void* stream, double timeoutS /* <= 0: the handle's */);
int sdrgpu_gather_destroy(sdrgpu_gather* g);

/* ---------------------------------------------- spectrum/IQ consumers ---- */
/* waterfall zoom, fft_scaler(viewOffset, viewBandwidth, wholeBandwidth, fftSize, outSize).doZoom
 * (gui/widgets/fft_scaler.h:27-64) on device dB rows: out[r][o] = max over the reference's bins */
typedef struct sdrgpu_zoom sdrgpu_zoom;
int sdrgpu_zoom_create(sdrgpu_zoom** z, int device, double viewOffset, double viewBandwidth, double wholeBandwidth,
                       int fftSize, int outSize);
int sdrgpu_zoom_execute_dev(sdrgpu_zoom* z, const float* rows, int nrows, float* out, void* stream);
int sdrgpu_zoom_destroy(sdrgpu_zoom* z);
/* SampleStreamCompressor::process (compression/sample_stream_compressor.h:26-60) of a device block:
 * pcmType 0 I8, 1 I16, 2 F32; `scratch` = 4 device bytes (I8/I16); returns bytes written */
int sdrgpu_compress_dev(int device, int pcmType, const float* in, int count, unsigned char* out, unsigned* scratch, void* stream);
/* SampleStreamDecompressor::process (sample_stream_decompressor.h:13-33): hdr = host copy of the
 * 8-byte header, payload = device bytes after it; returns complex samples written */
int sdrgpu_decompress_dev(int device, const unsigned char* hdr, const unsigned char* payload, int nbytes, float* out, void* stream);

/* WaterFall::pushFFT consumers (gui/widgets/waterfall.cpp), device buffers, bit-exact:
 *  colormap: zoomed dB -> waterfall pixels, pallet[(int)(((clamp(v) - min) / (max - min)) * (res - 1))] (:903-910);
 *  fft_smooth_hold: per column over nrows rows in order, smoothing (smooth = row*alpha + smooth*beta,
 *    row <- smooth; :918-925) then hold (hold[i] = max(row[i], hold[i] - speed), i >= 1; :952-957);
 *  vfo_signal_info: calculateVFOSignalInfo per raw row -> strength (in-band max) and snr (max minus
 *    side-band mean) (:563-601) */
int sdrgpu_colormap_dev(int device, const float* in, long long n, float wfMin, float wfMax, const unsigned* pallet, int res,
                        unsigned* out, void* stream);
int sdrgpu_fft_smooth_hold_dev(int device, float* rows, int nrows, int width, int smoothing, float alpha, float beta,
                               float* smooth, int holdOn, float holdSpeed, float* hold, void* stream);
int sdrgpu_vfo_signal_info_dev(int device, const float* rows, int nrows, int fftSize, double wholeBandwidth,
                               double centerOffset, double bandwidth, float* strength, float* snr, void* stream);

/* recorder WAV encoders (utils/wav.cpp:296-336) of n device floats: kind 0 u8, 1 i16, 2 i24
 * (packed LE), 3 i32, 4 f32; returns bytes written */
int sdrgpu_wav_encode_dev(int device, int kind, const float* in, long long n, unsigned char* out, void* stream);

/* ------------------------------------------------------------ ingest ---- */

/* file_source / rtl_sdr / hackrf sample converters (elementwise, n scalars):
 * kind 0 u8 (b-128+0.5f)/127.5f, 1 i16 (s+0.5f)/32767.5f, 2 i24 packed LE,
 * 3 i32 ((v+0.5)/(2^31-0.5) in double), 4 f64 -> f32, 5 i8 x*(1/128) */
enum { SDRGPU_CONV_U8 = 0, SDRGPU_CONV_I16, SDRGPU_CONV_I24, SDRGPU_CONV_I32, SDRGPU_CONV_F64, SDRGPU_CONV_I8,
       SDRGPU_CONV_F32 /* 32-bit IEEE float copied as it is (WAV IEEE_FLOAT 32) */ };
int sdrgpu_convert_dev(int device, int kind, const void* in, long long n, float* out, void* stream);
int sdrgpu_convert(int device, int kind, const void* in, long long n, float* out);      /* host buffers */
/* one-channel file_source WAV (main.cpp:294-430): n samples -> n complex_t with I = Q = the
 * converted sample (any SDRGPU_CONV_* kind) */
int sdrgpu_convert_mono_dev(int device, int kind, const void* in, long long n, void* out, void* stream);
int sdrgpu_convert_mono(int device, int kind, const void* in, long long n, void* out);   /* host buffers */

/* file_source WavReader (source_modules/file_source/src/wavreader.h:34-226): RIFF / RF64 WAVE,
 * fmt PCM / IEEE_FLOAT / EXTENSIBLE (by SubFormat), samples = [data offset, end of file) */
typedef struct sdrgpu_wav sdrgpu_wav;
int sdrgpu_wav_open(sdrgpu_wav** h, const char* path);
int sdrgpu_wav_info(sdrgpu_wav* h, int* format, int* channels, int* bits, double* sampleRate, long long* sampleCount);
/* converter kind (SDRGPU_CONV_*) for the file's (format, bits) as worker_1ch / worker_2ch pick it
 * (main.cpp:316-560); < 0 = unsupported (error) */
int sdrgpu_wav_kind(sdrgpu_wav* h);
int sdrgpu_wav_block_size(sdrgpu_wav* h);                      /* min(fs / 200, 1e6) frames */
int sdrgpu_wav_read(sdrgpu_wav* h, void* out, int maxFrames);   /* raw frames; 0 at the end */
int sdrgpu_wav_seek(sdrgpu_wav* h, long long frame);
int sdrgpu_wav_close(sdrgpu_wav* h);

#ifdef __cplusplus
}
#endif
#endif
