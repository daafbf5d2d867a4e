"""C3 with and without the fused quadrature epilogue (DDCFM vs DDC: the same fir_mfma_kernel, complex
out instead of the FM quadrature): HIP-event time per 2^28-sample call, 3 interleaved rounds."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from sdrpp_amd import dsp  # noqa: E402

torch.cuda.set_device(0)
st = torch.cuda.Stream()
torch.cuda.set_stream(st)
B = 1 << 28
FS = 61.44e6
x = (torch.rand(2 * B, device="cuda") * 2 - 1)
taps = dsp.low_pass(3.0e6, 912000.0, FS)
w = 2 * np.pi * (-1.5e6 / FS)
fm = dsp.DDCFM(w, taps, 8, 2 * np.pi * 100e3 / (FS / 8))
dd = dsp.DDC(w, taps, 8)
out = torch.empty(2 * (B // 8 + 64), dtype=torch.float32, device="cuda")
s = st.cuda_stream


def t(blk, n=10):
    for _ in range(2):
        blk.process_dev(x.data_ptr(), B, out.data_ptr(), s)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        blk.process_dev(x.data_ptr(), B, out.data_ptr(), s)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n


res = {"ddcfm_ms": [], "ddc_ms": []}
for _ in range(3):
    res["ddcfm_ms"].append(round(t(fm), 4))
    res["ddc_ms"].append(round(t(dd), 4))
print(json.dumps(res))
