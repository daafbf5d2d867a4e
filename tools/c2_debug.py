"""1M spectrum debug: rows of batch / single-frame calls vs the fp64 truth, per variant (env set by
the caller), and batch-vs-batch determinism."""
import os, sys
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
from sdrpp_amd import dsp
import oracle
N, nz = 1 << 20, 1000000
frames = int(sys.argv[1]) if len(sys.argv) > 1 else 32
g = torch.Generator(device="cuda"); g.manual_seed(3)
x = (torch.rand(2 * nz * frames, device="cuda", generator=g) * 2 - 1).contiguous()
f = dsp.FFTSpectrum(N, nz, 6)
rows = torch.empty(frames * N, device="cuda"); rows2 = torch.empty_like(rows)
f.execute_dev(x.data_ptr(), nz, frames, rows.data_ptr()); f.execute_dev(x.data_ptr(), nz, frames, rows2.data_ptr())
torch.cuda.synchronize()
one = dsp.FFTSpectrum(N, nz, 6)
single = torch.empty(N, device="cuda")
w = oracle.create_window(6, nz)
xh = x.cpu().numpy().view(np.complex64)
print("batch-vs-batch equal", torch.equal(rows, rows2), "nbad", int((rows != rows2).sum()))
for j in (0, 1, 5, 15, 16, frames - 1):
    one.execute_dev(x.data_ptr() + 8 * j * nz, nz, 1, single.data_ptr()); torch.cuda.synchronize()
    truth = 10 * np.log10(oracle.fft_truth_power(xh[j * nz:(j + 1) * nz], nz, N, w))
    b = rows[j * N:(j + 1) * N].cpu().numpy(); s = single.cpu().numpy()
    sel = truth > truth.max() - 60
    eb, es = np.abs(b - truth)[sel], np.abs(s - truth)[sel]
    bad = np.nonzero(np.abs(b - truth) > 0.01)[0]
    print(j, "batch max", eb.max(), "single max", es.max(), "nbad batch", len(bad), "first", bad[:8].tolist(),
          "k1 set", sorted(set((bad % 1024).tolist()))[:16], "k2 set", sorted(set((bad // 1024).tolist()))[:16])
