"""Phase stamps of the one-pass 64k kernel (measurement build: python sdrpp_amd/build.py
--variant t1p SDRGPU_1P_TIMING=1; run with SDRGPU_LIB_PATH=sdrpp_amd/lib_t1p/libsdrgpu.so
SDRGPU_TUNING=1 SDRGPU_FFT_1P=1). Runs the C5 group on a 2^28-sample batch and reports, over the
workgroups of the last call, the mean s_memtime units (wave 0) of each phase of a workgroup (one frame,
a quarter pair): the VFO half, the four-quarter loads + combine, and the two 16k transforms (stage-1
finish, stages 2 and 3, dB stores, zoom partials)."""
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
novfo = "--novfo" in sys.argv
for _ in range(4):
    if novfo:
        fft.execute_zoom_dev(x.data_ptr(), N, frames, spec.data_ptr(), zoom.data_ptr(), 2048)
    else:
        fft.execute_zoom_vfo_dev(x.data_ptr(), frames, spec.data_ptr(), zoom.data_ptr(), 2048, vfo, ifb.data_ptr())
torch.cuda.synchronize()
n = 16384 * 8
buf = (ctypes.c_ulonglong * n)()
assert sdrpp_amd.lib.sdrgpu_debug_1p_times(buf, n) == 0
wgs = 2 * frames
t8 = np.frombuffer(buf, dtype=np.uint64).reshape(16384, 8).astype(np.int64)[:wgs]
t = t8[:, :5]
d = np.diff(t, axis=1)
names = ["vfo", "loads", "transform_p", "transform_p2"]
# stamps 5-7 (after the first quarter's stage-1 finish, after each quarter's stage 2): the transforms by stage
o = t8[:, [2, 5, 6, 3, 7, 4]]
stages = ["q0_stage1", "q0_stage2", "q0_stage3_db", "q1_stage1_2", "q1_stage3_db_stores"]
out = {"workgroups": wgs, "vfo": not novfo, "mean_units": {k: round(float(d[:, i].mean())) for i, k in enumerate(names)},
       "transform_stages": {k: round(float(np.diff(o, axis=1)[:, i].mean())) for i, k in enumerate(stages)},
       "mean_total": round(float((t[:, 4] - t[:, 0]).mean())),
       "span": float(t[:, 4].max() - t[:, 0].min()),
       "note": "s_memtime units (clock64); ratios between phases are what matter"}
print(json.dumps(out, indent=1))
