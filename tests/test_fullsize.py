"""Parity at BASELINE's full sizes through size-independent properties (one bench step of
2^28 device-resident samples per config):

- C5 spectrum: rows of a 4096-frame batch (merged chunk launches) equal the same frames
  transformed one at a time, and a bin-centred tone reads 20 log10 A at bin N/2 + k0 in every
  row;
- C2 spectrum: rows of the 256-frame bench batch (16 chunks) equal single-frame transforms, and a
  tone reads 20 log10 A at its bin in every row;
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
    """C3 over one 2^28-sample call vs the same stream in ragged calls, every output checked.
    FIR stage (fused xlator + 256-tap FIR /8, complex out): a split moves only the NCO's last bits
    (each call rebuilds its coarse phasor table), so the outputs agree to a few ulps of the FIR's
    input scale. Quadrature: each output lies within the per-sample bound that FIR difference
    implies, |d| <= [2 (e/|y_i| + e/|y_i-1|) + 8 eps pi] / dev (wrap-aware), with |y| from the
    FIR stage itself -- a wrong output anywhere in the batch fails it."""
    fs = 61.44e6
    taps = dsp.low_pass(3.0e6, 912000.0, fs)
    w, dev = 2 * np.pi * (-1.5e6 / fs), 2 * np.pi * 100e3 / (fs / 8)
    cuts = [7, 8192 * 1023 + 5, 1 << 27, B - 8]
    fa, fb = dsp.DDC(w, taps, 8), dsp.DDC(w, taps, 8)
    ya, ma = _split_calls(fa, batch, B, 2 * (B // 8 + 64), 8, [])
    yb, mb = _split_calls(fb, batch, B, 2 * (B // 8 + 64), 8, cuts)
    assert ma == mb == B // 8
    ya = torch.view_as_complex(ya[:2 * ma].view(-1, 2))
    yb = torch.view_as_complex(yb[:2 * mb].view(-1, 2))
    e_fir = (ya - yb).abs().max().item()
    eps = float(np.finfo(np.float32).eps)
    hsum = float(np.abs(taps).sum())
    assert e_fir <= 8 * eps * hsum * np.sqrt(2.0), e_fir     # a few ulps of the input scale (|x| <= sqrt 2)
    a, b = dsp.DDCFM(w, taps, 8, dev), dsp.DDCFM(w, taps, 8, dev)
    qa, _ = _split_calls(a, batch, B, B // 8 + 64, 4, [])
    qb, _ = _split_calls(b, batch, B, B // 8 + 64, 4, cuts)
    qa, qb = qa[:ma].double(), qb[:mb].double()
    assert bool(torch.isfinite(qa).all())
    # the fused quadrature epilogue vs the fp64 quadrature of the FIR stage's own output, every
    # sample: the two kernels group an output's taps differently (1023- vs 1024-output tiles), so
    # their FIR values differ by a few ulps of the accumulation scale, e_b
    e_b = 8 * eps * hsum * np.sqrt(2.0)
    y64 = ya.to(torch.complex128)
    yp64 = torch.cat([torch.zeros(1, dtype=torch.complex128, device="cuda"), y64[:-1]])
    q64 = torch.angle(y64 * torch.conj(yp64)) / dev
    dq = (torch.remainder((qa - q64) * dev + np.pi, 2 * np.pi) - np.pi).abs()
    mag0 = y64.abs()
    bq = 2.0 * (e_b / mag0 + e_b / yp64.abs()) + 8 * eps * np.pi
    nbq = int((dq > bq).sum().item())
    assert nbq == 0, (nbq, torch.nonzero(dq > bq)[:5].flatten().tolist())
    e = max(e_fir, 1e-9)
    mag = ya.abs().double()
    magp = torch.cat([torch.zeros(1, dtype=torch.float64, device="cuda"), mag[:-1]])
    bound = (2.0 * (e / mag + e / magp) + 8 * eps * np.pi) / dev
    d = (qa - qb) * dev
    d = torch.remainder(d + np.pi, 2 * np.pi) - np.pi      # atan2 wrap
    err = d.abs() / dev
    nbad = int((err > bound).sum().item())
    assert nbad == 0, (nbad, torch.nonzero(err > bound)[:5].flatten().tolist())


def test_c2_spectrum_full_batch(batch):
    """C2's bench step (256 frames of nz = 1e6 at stride 1e6, 16 chunks, zero-padded to 2^20): rows of
    the batch equal the same frames transformed one at a time (same kernels; chunking changes only
    which launch a frame belongs to), and a bin-centred tone reads 20 log10 A in every row."""
    N, nz, frames = 1 << 20, 1000000, 256
    f = dsp.FFTSpectrum(N, nz, 6)
    rows = torch.empty(frames * N, device="cuda")
    f.execute_dev(batch.data_ptr(), nz, frames, rows.data_ptr())
    torch.cuda.synchronize()
    one = dsp.FFTSpectrum(N, nz, 6)
    single = torch.empty(N, device="cuda")
    for j in (0, 1, 15, 16, 17, 128, frames - 1):
        one.execute_dev(batch.data_ptr() + 8 * j * nz, nz, 1, single.data_ptr())
        torch.cuda.synchronize()
        assert torch.equal(rows[j * N:(j + 1) * N], single), j
    k0, A = 4321, 0.25
    n = torch.arange(nz, device="cuda", dtype=torch.float64)
    # bin-centred for the N-point transform of the zero-padded frame: exp(2 pi i k0 n / N)
    tone = torch.stack([A * torch.cos(2 * np.pi * k0 * n / N), A * torch.sin(2 * np.pi * k0 * n / N)], 1).float().reshape(-1)
    xt = tone.repeat(frames)
    f.execute_dev(xt.data_ptr(), nz, frames, rows.data_ptr())
    torch.cuda.synchronize()
    r = rows.view(frames, N)
    assert torch.all(torch.argmax(r, dim=1) == N // 2 + k0)
    # a window truncated to nz < N has coherent gain 1 over its own nz samples: the peak reads 20 log10 A
    assert float((r[:, N // 2 + k0] - 20 * np.log10(A)).abs().max()) < 0.01


def test_c4_channelizer_full_batch_split_invariant(batch):
    M = 1024
    taps = dsp.windowed_sinc(16 * M, np.pi / M)
    a, b = dsp.PolyphaseChannelizer(M, taps), dsp.PolyphaseChannelizer(M, taps)
    cap = 2 * (B + M)
    ya, ma = _split_calls(a, batch, B, cap, 8, [])
    yb, mb = _split_calls(b, batch, B, cap, 8, [M * 3 + 17, 1 << 27, B - 5 * M - 1])
    assert ma == mb == B
    assert torch.equal(ya[:2 * ma], yb[:2 * mb])
