"""Does the RxVFO's read of an IQ chunk get cheaper when the spectrum read the same chunk just
before (Infinity Cache reuse)? Times, over 2^28 device-resident samples in P chunks:
  A: VFO chain alone, P calls
  C: 64k spectrum alone, P calls
  B: spectrum(chunk c) then VFO(chunk c), P times
MALL benefit = (A + C) - B. Launch overheads are the same in A+C and B."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
from sdrpp_amd import dsp  # noqa: E402

N = 65536
B = 1 << 28
torch.cuda.set_stream(torch.cuda.Stream())
s = torch.cuda.current_stream()
x = (torch.rand(2 * B, device="cuda") * 2 - 1).contiguous()
spec = torch.empty(B, device="cuda")
ifb = torch.empty(2 * (B // 256 + 64), device="cuda")
fft = dsp.FFTSpectrum(N, N, 6)
vfo = dsp.RxVFO(61.44e6, 240000, 200000, 2.5e6)


def run(P, do_fft, do_vfo):
    fr = B // N // P
    m = 0
    for c in range(P):
        p = x.data_ptr() + 8 * c * fr * N
        if do_fft:
            fft.execute_dev(p, N, fr, spec.data_ptr() + 4 * c * fr * N, s.cuda_stream)
        if do_vfo:
            m += vfo.process_dev(p, fr * N, ifb.data_ptr() + 8 * m, s.cuda_stream)


def timeit(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(reps):
        fn()
    e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


for P in (1, 4, 8, 16, 32):
    a = timeit(lambda: run(P, False, True))
    c = timeit(lambda: run(P, True, False))
    b = timeit(lambda: run(P, True, True))
    print(f"P={P:3d} chunk={B // P * 8 >> 20} MB  vfo {a:.3f}  fft {c:.3f}  sum {a + c:.3f}  interleaved {b:.3f}  "
          f"gain {a + c - b:+.3f} ms", flush=True)
