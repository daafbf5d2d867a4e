"""Phase timestamps of the one-pass 64k kernel (measurement build: python sdrpp_amd/build.py --variant
t1p SDRGPU_1P_TIMING=1; run with SDRGPU_LIB_PATH=sdrpp_amd/lib_t1p/libsdrgpu.so SDRGPU_TUNING=1
SDRGPU_FFT_1P=1). Runs the C5 group on a 2^28-sample batch and reports, over the workgroups of the
last call, the mean cycles (wave 0, s_memtime) of: VFO quarter, load + combine, stage 1 (W, DFT32,
twiddle, LDS write), stage 2, stage 3 (+ dB stores), and the workgroup's total."""
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import sdrpp_amd  # noqa: E402
from sdrpp_amd import dsp  # noqa: E402

N, B = 65536, 1 << 28
frames = B // N
x = (torch.rand(2 * B, device="cuda") * 2 - 1)
fft = dsp.FFTSpectrum(N, N, 6)
vfo = dsp.RxVFO(61.44e6, 240000, 200000, 2.5e6)
spec = torch.empty(frames * N, device="cuda")
zoom = torch.empty(frames * 2048, device="cuda")
ifb = torch.empty(2 * (B // 256 + 64), device="cuda")
for _ in range(4):
    fft.execute_zoom_vfo_dev(x.data_ptr(), frames, spec.data_ptr(), zoom.data_ptr(), 2048, vfo, ifb.data_ptr())
torch.cuda.synchronize()
n = 16384 * 8
buf = (ctypes.c_ulonglong * n)()
assert sdrpp_amd.lib.sdrgpu_debug_1p_times(buf, n) == 0
t = np.frombuffer(buf, dtype=np.uint64).reshape(16384, 8).astype(np.int64)[:, :6]
d = np.diff(t, axis=1)
names = ["vfo", "loads", "stage1", "stage2", "stage3"]
start = t[:, 0] - t[:, 0].min()
out = {"workgroups": int(t.shape[0]), "mean_cycles": {k: float(d[:, i].mean()) for i, k in enumerate(names)},
       "mean_total": float((t[:, 5] - t[:, 0]).mean()),
       "p50_total": float(np.median(t[:, 5] - t[:, 0])),
       "span_cycles": float(t[:, 5].max() - t[:, 0].min()),
       "start_quantiles": [float(q) for q in np.quantile(start, [0.0, 0.25, 0.5, 0.75, 1.0])]}
print(json.dumps(out, indent=1))
