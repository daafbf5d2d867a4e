"""Max / rms dB error vs the fp64 truth, per window type, for the library at SDRGPU_LIB_PATH (or the
default), next to pocketfft f32 on the same frame (bins within 60 dB of the peak)."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
import oracle  # noqa: E402  (checker)
from sdrpp_amd import dsp  # noqa: E402
from _util import ref32_fft_db  # noqa: E402

out = []
frames = int(os.environ.get("FRAMES", "1"))
for N in (16384, 65536, 4096):
    for wt, k in [(wt, k) for wt in range(7) for k in range(frames)]:
        rng = np.random.default_rng(1234 + wt + 100 * k)
        x = (rng.uniform(-1, 1, N) + 1j * rng.uniform(-1, 1, N)).astype(np.complex64)
        w = oracle.create_window(wt, N)
        truth = oracle.fft_truth_power(x, N, N, w)
        t = 10 * np.log10(np.maximum(truth, 1e-300))
        sel = t >= t.max() - 60
        db = dsp.FFTSpectrum(N, N, wt).logmag(x)
        r = ref32_fft_db(x, N, N, w)
        e, er = np.abs(db.astype(np.float64) - t)[sel], np.abs(r.astype(np.float64) - t)[sel]
        out.append({"N": N, "w": wt, "k": k, "max": float(e.max()), "ref_max": float(er.max()), "ratio": float(e.max() / er.max()),
                    "rms": float(np.sqrt(np.mean(e ** 2))), "ref_rms": float(np.sqrt(np.mean(er ** 2)))})
print(json.dumps({"lib": os.environ.get("SDRGPU_LIB_PATH", "default"), "rows": out}))
