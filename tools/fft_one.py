"""Run one FFT configuration (for profiling): python tools/fft_one.py N nz frames iters"""
import sys, os, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from sdrpp_amd import dsp
N, nz, frames, iters = (int(v) for v in sys.argv[1:5])
torch.cuda.set_stream(torch.cuda.Stream())
s = torch.cuda.current_stream()
x = torch.rand(2 * nz * frames, device="cuda") * 2 - 1
out = torch.empty(frames * N, device="cuda")
f = dsp.FFTSpectrum(N, nz, 6)
for _ in range(iters):
    f.execute_dev(x.data_ptr(), nz, frames, out.data_ptr(), s.cuda_stream)
torch.cuda.synchronize()
