"""Spectrum accuracy over a fixed-seed frame corpus, in fp32 ulps of the correctly rounded dB of the
fp64 DFT of the same float-windowed frame (bins within 60 dB of each frame's peak), for the library
under test (SDRGPU_LIB_PATH or the in-tree build) next to pocketfft single precision (scipy, the
FFTW-class CPU reference) on every frame, and the fp64-interior mode (sdrgpu_fft_set_precision).

Corpus: 4096 / 16384 / 65536 points x the 7 window types x FRAMES (default 24) random frames =
504 frames, plus F1M (default 6) 1M-point frames with nz = 1e6 (BH7). Seeds depend only on
(N, window, k), so every build sees the same frames.
Output: one JSON object: per-frame rows and the corpus aggregates the parity tests' bars use."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle  # noqa: E402  (checker)
from sdrpp_amd import dsp  # noqa: E402
from _util import db_ulp_errors, ref32_fft_db  # noqa: E402


def frame(N, nz, wt, k):
    rng = np.random.default_rng(1234 + wt + 100 * k + 7 * N)
    return (rng.uniform(-1, 1, nz) + 1j * rng.uniform(-1, 1, nz)).astype(np.complex64)


def stats(e):
    return {"frac_le_1ulp": float(np.mean(e <= 1.0)), "p999": float(np.percentile(e, 99.9)), "max": float(e.max())}


def main():
    frames = int(os.environ.get("FRAMES", "24"))
    f1m = int(os.environ.get("F1M", "6"))
    cases = [(N, N, wt, k) for N in (4096, 16384, 65536) for wt in range(7) for k in range(frames)]
    cases += [(1 << 20, 1000000, 6, k) for k in range(f1m)]
    plans = {}
    rows = []
    for N, nz, wt, k in cases:
        key = (N, nz, wt)
        if key not in plans:
            plans[key] = (dsp.FFTSpectrum(N, nz, wt), dsp.FFTSpectrum(N, nz, wt, precision="f64"))
        f32, f64 = plans[key]
        x = frame(N, nz, wt, k)
        w = oracle.create_window(wt, nz)
        truth = oracle.fft_truth_power(x, nz, N, w)
        e = db_ulp_errors(f32.logmag(x), truth)
        er = db_ulp_errors(ref32_fft_db(x, nz, N, w), truth)
        e64 = db_ulp_errors(f64.logmag(x), truth)
        g, r = stats(e), stats(er)
        rows.append({"N": N, "nz": nz, "w": wt, "k": k, "bins": int(e.size), "gpu": g, "pocketfft": r,
                     "max_ratio": g["max"] / max(r["max"], 1.0), "f64_max": float(e64.max()),
                     "f64_frac_exact": float(np.mean(e64 == 0))})
    agg = {}
    for N in sorted({r["N"] for r in rows}):
        rs = [r for r in rows if r["N"] == N]
        agg[str(N)] = {
            "frames": len(rs),
            "gpu_min_frac_le_1ulp": min(r["gpu"]["frac_le_1ulp"] for r in rs),
            "pocketfft_min_frac_le_1ulp": min(r["pocketfft"]["frac_le_1ulp"] for r in rs),
            "gpu_max_p999": max(r["gpu"]["p999"] for r in rs),
            "pocketfft_max_p999": max(r["pocketfft"]["p999"] for r in rs),
            "gpu_max": max(r["gpu"]["max"] for r in rs),
            "pocketfft_max": max(r["pocketfft"]["max"] for r in rs),
            "frames_max_ratio_gt_1.25": sum(r["max_ratio"] > 1.25 for r in rs),
            "worst_max_ratio": max(r["max_ratio"] for r in rs),
            "f64_max": max(r["f64_max"] for r in rs),
            "f64_min_frac_exact": min(r["f64_frac_exact"] for r in rs),
        }
    print(json.dumps({"lib": os.environ.get("SDRGPU_LIB_PATH", "in-tree"), "aggregate": agg, "rows": rows}))


if __name__ == "__main__":
    main()
