"""Parity at BASELINE's full sizes through size-independent properties (one bench step of
2^28 device-resident samples per config):

- C5 spectrum: rows of a 4096-frame batch (merged chunk launches) equal the same frames
  transformed one at a time, and a bin-centred tone reads 20 log10 A at bin N/2 + k0 in every
  row;
- C5 VFO, C3 fused DDC and C4 channelizer: one call over the whole batch equals the same stream
  pushed as ragged blocks (the state carried across calls: FIR history, decimation phase, NCO
  phase, quadrature sample, channelizer rotation). The channelizer (exact per-channel rotation
  by index) is bit-identical; the xlator paths agree to the NCO's last bits (each call rebuilds
  its coarse phasor table from the carried double-double phase, so a split moves the table's
  rounding).

The small-size tests compare against the oracle; these check that nothing changes with size."""
import numpy as np
import pytest
import torch

import sdrpp_amd
from sdrpp_amd import dsp

pytestmark = pytest.mark.gpu

B = 1 << 28


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    assert sdrpp_amd.lib.sdrgpu_device_count() > 0, "no HIP device visible: gpu tests need an MI355X"


@pytest.fixture(scope="module")
def batch():
    g = torch.Generator(device="cuda")
    g.manual_seed(0xACE1)
    return (torch.rand(2 * B, device="cuda", generator=g) * 2 - 1).contiguous()


def _split_calls(block, x, n, out_floats, out_bytes, cuts):
    """outputs of block over x[0:n] pushed in the ragged pieces given by `cuts` (out_bytes per
    output sample)"""
    out = torch.empty(out_floats, dtype=torch.float32, device="cuda")
    m = 0
    for a, b in zip([0] + cuts, cuts + [n]):
        m += block.process_dev(x.data_ptr() + 8 * a, b - a, out.data_ptr() + out_bytes * m)
    torch.cuda.synchronize()
    return out, m


def test_c5_spectrum_full_batch(batch):
    N = 65536
    frames = B // N
    f = dsp.FFTSpectrum(N, N, 6)
    rows = torch.empty(frames * N, device="cuda")
    f.execute_dev(batch.data_ptr(), N, frames, rows.data_ptr())
    torch.cuda.synchronize()
    one = dsp.FFTSpectrum(N, N, 6)
    single = torch.empty(N, device="cuda")
    for j in (0, 1, 255, 256, 1023, 2048, frames - 1):
        one.execute_dev(batch.data_ptr() + 8 * j * N, N, 1, single.data_ptr())
        torch.cuda.synchronize()
        a = rows[j * N:(j + 1) * N].cpu().numpy()
        b = single.cpu().numpy()
        near = b >= b.max() - 60.0
        d = np.abs(a - b)
        assert d[near].max() <= 1e-3 and d.max() <= 0.05, (j, d[near].max(), d.max())
    # a bin-centred tone in every frame of the batch (tone frames written over the random batch)
    k0, A = 777, 0.5
    n = torch.arange(N, device="cuda", dtype=torch.float64)
    tone = torch.stack([A * torch.cos(2 * np.pi * k0 * n / N), A * torch.sin(2 * np.pi * k0 * n / N)], 1).float().reshape(-1)
    xt = tone.repeat(frames)
    f.execute_dev(xt.data_ptr(), N, frames, rows.data_ptr())
    torch.cuda.synchronize()
    r = rows.view(frames, N)
    assert torch.all(torch.argmax(r, dim=1) == N // 2 + k0)
    assert float((r[:, N // 2 + k0] - 20 * np.log10(A)).abs().max()) < 0.01


def test_c5_vfo_full_batch_split_invariant(batch):
    a = dsp.RxVFO(61.44e6, 240000, 200000, 2.5e6)
    b = dsp.RxVFO(61.44e6, 240000, 200000, 2.5e6)
    cap = 2 * (B // 256 + 64)
    ya, ma = _split_calls(a, batch, B, cap, 8, [])
    yb, mb = _split_calls(b, batch, B, cap, 8, [1, 12345, 3 * 10 ** 7, 1 << 27, B - 999])
    assert ma == mb == B // 256
    d = (ya[:2 * ma] - yb[:2 * mb]).abs().max().item()
    assert d <= 1e-5 * ya[:2 * ma].abs().max().item(), d


def test_c3_ddc_full_batch_split_invariant(batch):
    fs = 61.44e6
    taps = dsp.low_pass(3.0e6, 912000.0, fs)
    args = (2 * np.pi * (-1.5e6 / fs), taps, 8, 2 * np.pi * 100e3 / (fs / 8))
    a, b = dsp.DDCFM(*args), dsp.DDCFM(*args)
    ya, ma = _split_calls(a, batch, B, B // 8 + 64, 4, [])
    yb, mb = _split_calls(b, batch, B, B // 8 + 64, 4, [7, 8192 * 1023 + 5, 1 << 27, B - 8])
    assert ma == mb == B // 8
    assert bool(torch.isfinite(ya[:ma]).all())
    # the quadrature of nearly equal FIR outputs: atan2 is ill-conditioned where |y| is tiny, so a
    # last-bit NCO difference moves a few outputs; the fraction measured 0.99990 and 0.99989 on
    # two boxes (torch's generator draws depend on the device's CU count), so the bar is 0.9995
    close = ((ya[:ma] - yb[:mb]).abs() <= 1e-4).float().mean().item()
    assert close >= 0.9995, close


def test_c4_channelizer_full_batch_split_invariant(batch):
    M = 1024
    taps = dsp.windowed_sinc(16 * M, np.pi / M)
    a, b = dsp.PolyphaseChannelizer(M, taps), dsp.PolyphaseChannelizer(M, taps)
    cap = 2 * (B + M)
    ya, ma = _split_calls(a, batch, B, cap, 8, [])
    yb, mb = _split_calls(b, batch, B, cap, 8, [M * 3 + 17, 1 << 27, B - 5 * M - 1])
    assert ma == mb == B
    assert torch.equal(ya[:2 * ma], yb[:2 * mb])
