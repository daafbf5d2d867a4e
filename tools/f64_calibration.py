"""CPU calibration of the fp64-interior spectrum's exactness bar (tests/test_gpu_parity.py
test_spectrum_f64_within_1ulp): how often two independent fp64 evaluations of the same DFT round to
different fp32 dB values, by depth below the frame's peak. numpy's FFT (the test's truth) against a
four-step evaluation (256 x 256, dense fp64 DFT matrices: a larger rounding error than any fp64 FFT,
so an upper bound on the disagreement) on the AES17 golden frame. Prints one JSON object."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle  # noqa: E402

g = np.load(os.path.join(ROOT, "tests", "golden", "fft_aes17.npz"))
N = int(g["N"])
w = oracle.create_window(6, N)
xw = (g["x"].astype(np.complex64) * w.astype(np.float32)).astype(np.complex64).astype(np.complex128)
N1 = N2 = int(round(np.sqrt(N)))
A = xw.reshape(N1, N2)                                       # n = N2 n1 + n2
F1 = np.exp(-2j * np.pi * np.outer(np.arange(N1), np.arange(N1)) / N1)
B = (F1 @ A) * np.exp(-2j * np.pi * np.outer(np.arange(N1), np.arange(N2)) / N)
X = (B @ np.exp(-2j * np.pi * np.outer(np.arange(N2), np.arange(N2)) / N2).T).T.reshape(-1)   # X[k1 + N1 k2]
t64 = 10 * np.log10(np.maximum(g["power_f64"], 1e-300))
a64 = 10 * np.log10(np.maximum(X.real ** 2 + X.imag ** 2, 1e-300))
sel = t64 >= t64.max() - 200
diff = t64[sel].astype(np.float32) != a64[sel].astype(np.float32)
depth = t64.max() - t64[sel]
out = {"frame": "tests/golden/fft_aes17.npz", "bins_200dB": int(sel.sum()), "differ": int(diff.sum()),
       "by_depth_db": {str(d): {"bins": int((depth <= d).sum()), "differ": int(diff[depth <= d].sum())}
                       for d in (60, 100, 120, 140, 160, 180, 200)}}
print(json.dumps(out))
