"""C4 polyphase channelizer: libsdrgpu (HIP) vs the oracle's per-channel definition
(exact-NCO FrequencyXlator(-k fs/M) -> DecimatingFIR(h, M), fp64; oracle/sdr_oracle.c
orc_channelize) and vs the literal oracle xlator + FIR chain.

Tolerance (stated once, `chan_tol`): normwise per output frame over the tested channels,
||y_gpu - y_true||_2 <= 8 * eps32 * (log2 M + sqrt(Q)) * ||y_true||_2 (fp32 Q-tap branch
FIRs followed by an fp32 M-point FFT), and elementwise |err| <= the same bound scaled to the
frame's rms, so stopband channels are held to the frame's accuracy, not to their own size.
"""
import numpy as np
import pytest

import oracle
import sdrpp_amd
from sdrpp_amd import dsp
from _util import EPS32, iq

Q = 16


def chan_tol(M):
    return 8 * EPS32 * (np.log2(M) + np.sqrt(Q))


def check_frames(y, truth, M, what):
    """y, truth: [nchan, frames] complex."""
    assert y.shape == truth.shape, f"{what}: {y.shape} vs {truth.shape}"
    tol = chan_tol(M)
    for m in range(truth.shape[1]):
        t = truth[:, m]
        e = y[:, m].astype(np.complex128) - t
        nt = np.linalg.norm(t)
        if nt == 0:
            assert np.all(y[:, m] == 0), f"{what}: frame {m} nonzero on zero input"
            continue
        assert np.linalg.norm(e) <= tol * nt, f"{what}: frame {m} normwise {np.linalg.norm(e) / nt:.3e} > {tol:.3e}"
        rms = nt / np.sqrt(t.size)
        assert np.abs(e).max() <= tol * rms * np.sqrt(t.size), f"{what}: frame {m} max err {np.abs(e).max():.3e}"


# ---------------------------------------------------------------- host-only
def test_prototype_taps_match_oracle():
    """windowedSinc<float>(16384, pi/M, nuttall) -- the C4 prototype -- bit-exact host design."""
    for M in (256, 1024):
        assert np.array_equal(dsp.windowed_sinc(16 * M, np.pi / M), oracle.windowed_sinc(16 * M, np.pi / M))


def test_oracle_definition_equals_literal_chain():
    """The exact-NCO definition vs the oracle's literal FrequencyXlator (float-quantised phase
    increment, frequency_xlator.h:17) -> DecimatingFIR: they differ only by the xlator's
    phase-increment rounding: |dw| = |arg(float(cos w), float(sin w)) - w| per sample, so the
    bound is (n |dw| + 8 eps32) max|y| after n samples."""
    rng = np.random.default_rng(7)
    M = 64
    h = oracle.windowed_sinc(16 * M, np.pi / M)
    x = iq(rng, 40 * M + 17)
    chans = [0, 1, 7, 31, 32, 63]
    y = oracle.channelize(x, h, M, chans)
    for i, k in enumerate(chans):
        w = -2 * np.pi * k / M
        dw = abs(np.arctan2(np.float64(np.float32(np.sin(w))), np.float64(np.float32(np.cos(w)))) - w)
        dw = min(dw, abs(dw - 2 * np.pi))
        z = oracle.FIR(h, decim=M).process(oracle.Xlator(w).process(x))
        assert z.shape[0] == y.shape[1]
        assert np.abs(z - y[i]).max() <= (len(x) * dw + 8 * EPS32) * np.abs(y[i]).max()


# ---------------------------------------------------------------- GPU parity
@pytest.fixture(scope="module")
def _gpu():
    assert sdrpp_amd.lib.sdrgpu_device_count() > 0, "no HIP device visible: gpu tests need an MI355X"


def _frames(y, M):
    return y.reshape(-1, M).T        # [M channels, frames]


@pytest.mark.gpu
@pytest.mark.parametrize("M", [256, 512, 1024])
def test_channelizer_vs_definition(_gpu, M, rng):
    h = dsp.windowed_sinc(16 * M, np.pi / M)
    n = 48 * M + 333                                     # ragged tail
    x = iq(rng, n)
    ch = dsp.PolyphaseChannelizer(M, h)
    y = ch.process(x)
    frames = (n + M - 1) // M
    assert y.shape[0] == frames * M
    chans = sorted(set([0, 1, 2, M // 2 - 1, M // 2, M // 2 + 1, M - 2, M - 1] + list(rng.integers(0, M, 8))))
    truth = oracle.channelize(x, h, M, chans)
    check_frames(_frames(y, M)[chans], truth, M, f"M={M}")


@pytest.mark.gpu
def test_channelizer_all_channels_tone(_gpu):
    """Every channel: a complex tone at the centre of channel k0 lands in channel k0 (gain
    ~1 after the unity-DC prototype), every channel agrees with the definition normwise."""
    M = 1024
    h = dsp.windowed_sinc(16 * M, np.pi / M)
    k0 = 300
    n = 64 * M
    t = np.arange(n)
    x = (0.5 * np.exp(2j * np.pi * k0 * t / M)).astype(np.complex64)
    y = _frames(dsp.PolyphaseChannelizer(M, h).process(x), M)
    truth = oracle.channelize(x, h, M, list(range(M)))
    check_frames(y, truth, M, "tone")
    steady = y[:, 20:]
    assert np.allclose(np.abs(steady[k0]), 0.5 * h.sum(), rtol=1e-4)
    others = np.delete(np.abs(steady), k0, axis=0)
    assert others.max() < 1e-3 * 0.5


@pytest.mark.gpu
@pytest.mark.parametrize("M", [256, 1024])
def test_channelizer_block_split_invariance(_gpu, M, rng):
    """Ragged process() calls give the same output stream as one call, bit for bit (the
    history, decimation phase and NCO rotation are carried across calls)."""
    h = dsp.windowed_sinc(16 * M - 37, np.pi / M)       # tap count not a multiple of M
    x = iq(rng, 40 * M + 5)
    one = dsp.PolyphaseChannelizer(M, h).process(x)
    ch = dsp.PolyphaseChannelizer(M, h)
    parts, i = [], 0
    for c in [1, M - 1, 3 * M + 7, 0, 5 * M, 17, 2 * M]:
        parts.append(ch.process(x[i:i + c]))
        i += c
    parts.append(ch.process(x[i:]))
    cat = np.concatenate(parts)
    assert cat.shape == one.shape
    assert np.array_equal(cat, one)
    truth = oracle.channelize(x, h, M, [0, 3, M - 1])
    check_frames(_frames(one, M)[[0, 3, M - 1]], truth, M, "split")


@pytest.mark.gpu
def test_channelizer_reset_and_empty(_gpu, rng):
    M = 256
    h = dsp.windowed_sinc(16 * M, np.pi / M)
    x = iq(rng, 10 * M)
    ch = dsp.PolyphaseChannelizer(M, h)
    a = ch.process(x)
    assert ch.process(x[:0]).shape[0] == 0
    ch.reset()
    b = ch.process(x)
    assert np.array_equal(a, b)


# ---------------------------------------------------------------- MFMA DFT-GEMM form (C4)
@pytest.mark.gpu
@pytest.mark.parametrize("n", [48 * 1024 + 333, 700 * 1024 + 5])
def test_channelizer_gemm_vs_definition(_gpu, n, rng):
    """dft="gemm" (the filterbank's DFT as two complex 32x32 products per frame on the matrix
    cores): every channel of every frame against the fp64 definition at the same `chan_tol` bar
    as the FFT form; 700 frames span several workgroups (256 frames each) and a ragged last one."""
    M = 1024
    h = dsp.windowed_sinc(16 * M, np.pi / M)
    x = iq(rng, n)
    y = dsp.PolyphaseChannelizer(M, h, dft="gemm").process(x)
    frames = (n + M - 1) // M
    assert y.shape[0] == frames * M
    yf = _frames(y, M)
    if n < 100 * M:
        check_frames(yf, oracle.channelize(x, h, M, list(range(M))), M, "gemm all channels")
    else:
        chans = sorted(set([0, 1, 31, 32, 33, 511, 512, 1023] + list(rng.integers(0, M, 8))))
        check_frames(yf[chans], oracle.channelize(x, h, M, chans), M, "gemm multi-workgroup")
    # same branch FIRs as the FFT form: the two DFTs agree to the same bar
    yfft = _frames(dsp.PolyphaseChannelizer(M, h).process(x), M)
    check_frames(yf, yfft.astype(np.complex128), M, "gemm vs fft")


@pytest.mark.gpu
def test_channelizer_gemm_tone_and_split(_gpu, rng):
    """A tone at the centre of channel k0 lands in k0 only (gemm form), and ragged calls give
    the same output stream as one call, bit for bit."""
    M = 1024
    h = dsp.windowed_sinc(16 * M, np.pi / M)
    k0, n = 777, 64 * M
    t = np.arange(n)
    x = (0.5 * np.exp(2j * np.pi * k0 * t / M)).astype(np.complex64)
    y = _frames(dsp.PolyphaseChannelizer(M, h, dft="gemm").process(x), M)
    steady = y[:, 20:]
    assert np.allclose(np.abs(steady[k0]), 0.5 * h.sum(), rtol=1e-4)
    assert np.delete(np.abs(steady), k0, axis=0).max() < 1e-3 * 0.5
    xr = iq(rng, 40 * M + 5)
    one = dsp.PolyphaseChannelizer(M, h, dft="gemm").process(xr)
    ch = dsp.PolyphaseChannelizer(M, h, dft="gemm")
    parts, i = [], 0
    for c in [1, M - 1, 3 * M + 7, 0, 5 * M, 17, 2 * M]:
        parts.append(ch.process(xr[i:i + c]))
        i += c
    parts.append(ch.process(xr[i:]))
    assert np.array_equal(np.concatenate(parts), one)


@pytest.mark.gpu
def test_channelizer_gemm_needs_1024(_gpu):
    with pytest.raises(Exception):
        dsp.PolyphaseChannelizer(256, dsp.windowed_sinc(16 * 256, np.pi / 256), dft="gemm")
