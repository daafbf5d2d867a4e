"""Timing experiment: C5 with the VFO's full-rate first stage run per Infinity-Cache-sized
slice next to the spectrum of the same slice, the low-rate tail once per step."""
import sys, time, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from sdrpp_amd import dsp

N = 65536
B = 1 << 28
frames = B // N
torch.cuda.set_device(0)
torch.cuda.set_stream(torch.cuda.Stream())
st = torch.cuda.current_stream()
s = st.cuda_stream
x = (torch.rand(2 * B, device="cuda") * 2 - 1).contiguous()
spec = torch.empty(frames * N, device="cuda")
fft = dsp.FFTSpectrum(N, N, 6)
plan = dsp.decim_plan(256)
s1 = dsp.FIR(plan[0][1], plan[0][0])
s2 = dsp.FIR(plan[1][1], plan[1][0])
s3 = dsp.FIR(plan[2][1], plan[2][0])
lpf = dsp.FIR(dsp.low_pass(100000.0, 10000.0, 240000.0), 1)
wfm = dsp.BroadcastFM(100000, 240000, True)
vfo = dsp.RxVFO(61.44e6, 240000, 200000, 2.5e6)
h1 = torch.empty(2 * (B // 32 + 64), device="cuda")
h2 = torch.empty(2 * (B // 128 + 64), device="cuda")
h3 = torch.empty(2 * (B // 256 + 64), device="cuda")
h4 = torch.empty(2 * (B // 256 + 64), device="cuda")
au = torch.empty(2 * (B // 256 + 64), device="cuda")


def tail(m1):
    m2 = s2.process_dev(h1.data_ptr(), m1, h2.data_ptr(), s)
    m3 = s3.process_dev(h2.data_ptr(), m2, h3.data_ptr(), s)
    m4 = lpf.process_dev(h3.data_ptr(), m3, h4.data_ptr(), s)
    wfm.process_dev(h4.data_ptr(), m4, au.data_ptr(), s)


def step(sub, order):
    fr = frames // sub
    n = B // sub
    m1 = 0
    for i in range(sub):
        if order == "vf":
            m1 += s1.process_dev(x.data_ptr() + 8 * i * n, n, h1.data_ptr() + 8 * m1, s)
        fft.execute_dev(x.data_ptr() + 8 * i * n, N, fr, spec.data_ptr() + 4 * i * fr * N, s)
        if order == "fv":
            m1 += s1.process_dev(x.data_ptr() + 8 * i * n, n, h1.data_ptr() + 8 * m1, s)
    tail(m1)


def step_ref():
    fft.execute_dev(x.data_ptr(), N, frames, spec.data_ptr(), s)
    m = vfo.process_dev(x.data_ptr(), B, h4.data_ptr(), s)
    wfm.process_dev(h4.data_ptr(), m, au.data_ptr(), s)


def timeit(fn, reps=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps * 1e3


res = []
for rnd in range(2):
    res.append(("ref", timeit(step_ref)))
    for sub in (1, 8, 16, 32, 64):
        for order in ("vf", "fv"):
            res.append((f"sub{sub}_{order}", timeit(lambda: step(sub, order))))
for k, v in res:
    print(f"{k:14s} {v:.3f} ms  {B / v / 1e3:.0f} MS/s", flush=True)
