"""Sweep FFT tuning knobs (env vars read at plan creation) on the GPU; prints us per frame-chunk."""
import json, os, subprocess, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import sys, time, torch
sys.path.insert(0, %r)
from sdrpp_amd import dsp
N, nz, frames = %d, %d, %d
torch.cuda.set_stream(torch.cuda.Stream())
s = torch.cuda.current_stream()
x = torch.rand(2 * nz * frames, device="cuda") * 2 - 1
out = torch.empty(frames * N, device="cuda")
f = dsp.FFTSpectrum(N, nz, 6)
for _ in range(3): f.execute_dev(x.data_ptr(), nz, frames, out.data_ptr(), s.cuda_stream)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record(s)
for _ in range(10): f.execute_dev(x.data_ptr(), nz, frames, out.data_ptr(), s.cuda_stream)
e1.record(s); torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / 10
print(ms, nz * frames / ms / 1e6, 12 * nz * frames / ms / 1e6)
'''
res = []
for N, nz, frames in [(65536, 65536, 4096), (1 << 20, 1000000, 256)]:
    for env in json.loads(sys.argv[1]):
        e = dict(os.environ); e.update({k: str(v) for k, v in env.items()})
        r = subprocess.run([sys.executable, "-c", CHILD % (ROOT, N, nz, frames)], env=e, capture_output=True, text=True, timeout=300)
        line = r.stdout.strip().splitlines()[-1] if r.stdout.strip() else r.stderr[-300:]
        print(N, env, "ms/GSps/GBps:", line, flush=True)
