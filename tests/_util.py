"""Shared parity helpers (tolerances are stated here, once)."""
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

EPS32 = np.finfo(np.float32).eps


def fir_atol(taps, x):
    """fp32 FIR vs fp64-accumulated oracle: |err| <= 8*eps32*sqrt(ntaps)*sum|h|*max|x| (+tiny)."""
    h = np.abs(np.asarray(taps)).sum()
    xm = np.abs(np.asarray(x)).max() if np.size(x) else 1.0
    return 8 * EPS32 * np.sqrt(len(taps)) * h * xm + 1e-30


def assert_close_c(a, b, atol, what=""):
    a = np.asarray(a)
    b = np.asarray(b)
    assert a.shape == b.shape, f"{what}: shape {a.shape} vs {b.shape}"
    err = np.abs(a.astype(np.complex128) - b.astype(np.complex128)).max() if a.size else 0.0
    assert err <= atol, f"{what}: max abs err {err:.3e} > atol {atol:.3e}"
    return err


def db_check(db_gpu, power_true, N, ref32_db=None, floor_db=60.0):
    """Spectrum parity (DESIGN.md 'Parity bar'), on bins within `floor_db` of the frame peak:
    1. the GPU's dB error vs the fp64 truth is in the accuracy class of a reference-class fp32
       FFT (pocketfft single precision) on the same windowed input: rms <= 2x its rms (+ the
       rms of 1 ulp of the fp32 dB values) and max <= 8x its max (+2 ulp of the fp32 dB value).
       The max bar is a ratio of two single-bin maxima, a heavy-tailed statistic: over 504 random
       frames (4k / 16k / 64k, all 7 windows; profiles/r3/fft_cmul/) it reached 5.72x for the
       round-2 kernels and 6.63x with the packed-asm complex multiply (p99 3.2x / 3.6x), while the
       rms ratio stayed at 0.97 / 0.98 (mean). A 3x bar failed 9 / 10 of those frames for the two
       builds, so it was a coin toss at the 2% level; 8x sits above both tails, and the rms bar
       carries the accuracy class;
    2. normwise: || |X_gpu| - |X_true| ||_2 <= 4 * eps32 * log2(N) * ||X_true||_2 (all bins).
    Without a reference-class FFT the bound is 2e-4 dB.
    """
    db_true = 10.0 * np.log10(np.maximum(power_true, 1e-300))
    peak = db_true.max()
    sel = db_true >= peak - floor_db
    err = np.abs(db_gpu.astype(np.float64) - db_true)[sel]
    ulp = np.spacing(np.abs(db_gpu[sel]).astype(np.float32)).astype(np.float64)
    if ref32_db is not None:
        rerr = np.abs(ref32_db.astype(np.float64) - db_true)[sel]
        rms_g, rms_r = np.sqrt(np.mean(err ** 2)), np.sqrt(np.mean(rerr ** 2))
        # + the rms of 1 ulp of the fp32 dB value: the reference writes 10*log10f(re^2+im^2) in
        # fp32 (volk_32fc_s32f_power_spectrum_32f), i.e. the dB row itself carries ~1 ulp
        # (log10f + the x10 rounding); the scipy row here is rounded once from fp64
        ulp_rms = np.sqrt(np.mean(ulp ** 2))
        assert rms_g <= 2.0 * rms_r + ulp_rms + 1e-12, f"rms dB err {rms_g:.3e} > 2 x fp32-ref {rms_r:.3e} + ulp {ulp_rms:.3e}"
        assert np.all(err <= 8.0 * rerr.max() + 2.0 * ulp), f"max dB err {err.max():.3e} > 8 x fp32-ref {rerr.max():.3e}"
    else:
        assert np.all(err <= np.maximum(2e-4, 2.0 * ulp)), f"max dB err {err.max():.3e}"
    mag_gpu = np.sqrt(10.0 ** (db_gpu.astype(np.float64) / 10.0))
    mag_true = np.sqrt(power_true)
    nerr = np.linalg.norm(mag_gpu - mag_true) / np.linalg.norm(mag_true)
    assert nerr <= 4 * EPS32 * np.log2(N), f"normwise magnitude error {nerr:.3e}"
    return err.max(), nerr


def db_ulp_errors(db, power_true, floor_db=60.0):
    """|db - db_true| in units of the fp32 ulp of the true dB value (db_true = 10 log10 of the fp64
    power, rounded once to fp32), on bins within `floor_db` of the frame peak. This is the
    north_star's "<= 1 ulp on FFT magnitude" measured literally: a value of 1 means the dB row is
    one fp32 step from the correctly rounded dB of the exact DFT."""
    t64 = 10.0 * np.log10(np.maximum(np.asarray(power_true, np.float64), 1e-300))
    sel = t64 >= t64.max() - floor_db
    t32 = t64[sel].astype(np.float32)
    ulp = np.spacing(np.abs(t32)).astype(np.float64)
    return np.abs(np.asarray(db, np.float32)[sel].astype(np.float64) - t32.astype(np.float64)) / ulp


def ulp_summary(e):
    return {"bins": int(e.size), "p50": float(np.percentile(e, 50)), "p90": float(np.percentile(e, 90)),
            "p99": float(np.percentile(e, 99)), "max": float(e.max()), "frac_le_1ulp": float(np.mean(e <= 1.0))}


def write_report(name, obj):
    """Append a JSON line to $SDRGPU_REPORT_DIR/<name>.jsonl when that directory is set (GPU
    sessions copy these into profiles/)."""
    import json
    d = os.environ.get("SDRGPU_REPORT_DIR")
    if d:
        os.makedirs(d, exist_ok=True)
        with open(os.path.join(d, name + ".jsonl"), "a") as f:
            f.write(json.dumps(obj) + "\n")


def ref32_fft_db(x, nz, N, window):
    """A reference-class fp32 FFT (pocketfft single precision via scipy) on the windowed frame."""
    import scipy.fft
    buf = np.zeros(N, dtype=np.complex64)
    buf[:nz] = (np.asarray(x[:nz], dtype=np.complex64) * np.asarray(window, dtype=np.float32)).astype(np.complex64)
    X = scipy.fft.fft(buf, workers=1)
    assert X.dtype == np.complex64
    p = X.real.astype(np.float32) ** 2 + X.imag.astype(np.float32) ** 2
    with np.errstate(divide="ignore"):
        return (10.0 * np.log10(p.astype(np.float64))).astype(np.float32)


def iq(rng, n, scale=1.0):
    """SpeedTester-style uniform [-1,1) complex IQ (core/src/dsp/bench/speed_tester.h:37-41)."""
    return (rng.uniform(-1, 1, n) + 1j * rng.uniform(-1, 1, n)).astype(np.complex64) * np.float32(scale)
