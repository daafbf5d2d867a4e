"""Serial loops and the AM / SSB demodulators: libsdrgpu (HIP) vs the oracle restatement of
loop/agc.h, correction/dc_blocker.h, demod/am.h, demod/ssb.h.

Bar: the AGC and the DC blocker are BIT-EXACT (the GPU runs the reference recurrence in the
reference's operation order, compiled without FMA contraction, IEEE divide and sqrt). AM is bit-exact up to its
low-pass FIR, whose fp32 accumulation is held to tests/_util.py fir_atol against the oracle's
fp64-accumulating FIR. SSB's xlator is the GPU NCO (<= 2 ulp per sample vs the oracle's long
double NCO), after which the AGC is the same recurrence; its bound is stated in the test.
"""
import numpy as np
import pytest

import oracle
import sdrpp_amd
from sdrpp_amd import dsp
from _util import EPS32, fir_atol, iq

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    assert sdrpp_amd.lib.sdrgpu_device_count() > 0, "no HIP device visible: gpu tests need an MI355X"


def bursty(rng, n, complex_data):
    """Level steps over 60 dB, silent gaps (exact zeros) and single-sample spikes, so the
    attack/decay branches, the zero-amplitude branch and the clip look-ahead all run."""
    env = np.repeat(10.0 ** rng.uniform(-3, 0, n // 500 + 1), 500)[:n]
    x = iq(rng, n) if complex_data else rng.uniform(-1, 1, n).astype(np.float32)
    x = (x * env.astype(np.float32)).astype(x.dtype)
    x[n // 3:n // 3 + 700] = 0
    spikes = rng.integers(0, n, 12)
    x[spikes] *= 50
    return x


@pytest.mark.parametrize("complex_data", [False, True])
@pytest.mark.parametrize("blocks", [[48000], [1, 1023, 1024, 1025, 4000, 0, 37, 20000]])
def test_agc_bit_exact(complex_data, blocks, rng):
    n = sum(blocks) + 3000
    x = bursty(rng, n, complex_data)
    args = (1.0, 50.0 / 48000, 5.0 / 48000, 10e6, 10.0, float("inf"))
    g = dsp.AGC(*args, complex_data=complex_data)
    o = oracle.AGC(complex_data, *args)
    i = 0
    for b in blocks + [n - sum(blocks)]:
        yg, yo = g.process(x[i:i + b]), o.process(x[i:i + b])
        assert yg.shape == yo.shape
        assert np.array_equal(yg.view(np.uint32), yo.view(np.uint32)), f"block at {i}: max diff {np.abs(yg - yo).max()}"
        i += b
    assert g.get_gain() == o.get_gain()


@pytest.mark.parametrize("complex_data", [False, True])
def test_agc_disabled_and_set_gain(complex_data, rng):
    x = bursty(rng, 30000, complex_data)
    args = (1.0, 0.01, 0.001, 10e6, 10.0, float("inf"))
    g, o = dsp.AGC(*args, complex_data=complex_data), oracle.AGC(complex_data, *args)
    for obj in (g, o):
        obj.set_enabled(False)
        obj.set_gain(3.5)                  # AM::setAGCGain path: fixed gain, clip at maxOutputAmp
    a, b = g.process(x[:10000]), o.process(x[:10000])
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))
    for obj in (g, o):
        obj.set_enabled(True)
    a, b = g.process(x[10000:]), o.process(x[10000:])
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))


@pytest.mark.parametrize("complex_data", [False, True])
def test_dc_blocker_bit_exact(complex_data, rng):
    n = 50000
    x = (iq(rng, n) + (0.3 + 0.2j)).astype(np.complex64) if complex_data else (rng.uniform(-1, 1, n) + 0.25).astype(np.float32)
    rate = 10.0 / 48000
    g, o = dsp.DCBlocker(rate, complex_data), oracle.DCBlocker(rate, complex_data)
    for s, e in [(0, 1), (1, 3000), (3000, 3000), (3000, 50000)]:
        a, b = g.process(x[s:e]), o.process(x[s:e])
        assert np.array_equal(a.view(np.uint32), b.view(np.uint32))
    # the offset converges to the DC level (the block's purpose)
    tail = g.process(x[:20000])
    assert abs(np.mean(tail[-5000:])) < 0.02


@pytest.mark.parametrize("mode", [0, 1, 2])
def test_am_vs_oracle(mode, rng):
    fs = 48000.0
    n = 60000
    t = np.arange(n)
    carrier = (1.0 + 0.6 * np.sin(2 * np.pi * 700 * t / fs)) * np.exp(1j * (2 * np.pi * 300 * t / fs + 0.3))
    x = (0.05 * carrier + 0.001 * iq(rng, n)).astype(np.complex64)
    x[20000:21000] *= 40                                   # a burst: clip look-ahead
    args = (mode, 10000.0, 50.0 / fs, 5.0 / fs, 10.0 / fs, fs)
    g, o = dsp.AM(*args), oracle.AM(*args, precise=True)
    lpf = oracle.low_pass(5000.0, 500.0, fs)
    for s, e in [(0, 4800), (4800, 30000), (30000, n)]:
        a, b = g.process(x[s:e]), o.process(x[s:e])
        assert a.shape == b.shape
        # the FIR input is bit-identical (AGC/|x|/DC block exact), so the only difference is
        # the LPF's fp32 vs fp64 accumulation
        pre = np.abs(b).max() if b.size else 1.0
        assert np.abs(a - b).max() <= fir_atol(lpf, np.array([pre * 2])), f"mode {mode} block {s}"


def test_am_stereo_interleave(rng):
    fs = 48000.0
    x = (0.1 * iq(rng, 20000)).astype(np.complex64)
    args = (2, 8000.0, 50.0 / fs, 5.0 / fs, 10.0 / fs, fs)
    mono = dsp.AM(*args).process(x)
    st = dsp.AM(*args, stereo=True).process(x)
    assert np.array_equal(st["l"], mono) and np.array_equal(st["r"], mono)


@pytest.mark.parametrize("mode", [0, 1, 2])
@pytest.mark.parametrize("agc", [True, False])
def test_ssb_vs_oracle(mode, agc, rng):
    fs = 24000.0
    n = 48000
    t = np.arange(n)
    x = (0.2 * np.exp(2j * np.pi * 1100 * t / fs) + 0.05 * np.exp(-2j * np.pi * 700 * t / fs)).astype(np.complex64)
    x = (x + 0.002 * iq(rng, n)).astype(np.complex64)
    args = (mode, 2800.0, fs, agc, 50.0 / fs, 5.0 / fs)
    g, o = dsp.SSB(*args), oracle.SSB(*args)
    for s, e in [(0, 2400), (2400, n)]:
        a, b = g.process(x[s:e]), o.process(x[s:e])
        assert a.shape == b.shape
        scale = max(np.abs(b).max(), 1e-30)
        err = np.abs(a - b)
        if agc:
            # xlator: <= ~4 ulp relative per sample (GPU NCO vs long double); the AGC
            # recurrence carries such perturbations at the output scale: bound 1e-5 of it
            assert err.max() <= 1e-5 * scale + 16 * EPS32 * scale, f"mode {mode} agc {agc} block {s}"
        else:
            # AGC disabled (ssb.h:31): fixed gain min(initGain = inf, maxGain) = 1e7 with the
            # clip at 10 -- a hard limiter, which maps an ulp-level xlator difference at a
            # near-zero sample to a 1e7-times larger one. Clipped samples (|y| = 10) must agree
            # exactly in sign and value; the rare unclipped ones are the limiter's linear region.
            clipped = np.abs(b) >= 10.0 * (1 - 1e-6)
            assert clipped.mean() > 0.99
            assert np.all(np.abs(a[clipped] - b[clipped]) <= 16 * EPS32 * 10.0), f"mode {mode} block {s}"


def fm_stereo_iq(n, fs, left_hz=1000.0, right_hz=0.0, seed=3):
    """FM broadcast: mpx = 0.45 (L+R) + 0.45 (L-R) cos(2 th) + 0.1 cos(th), th = 19 kHz pilot
    phase, 75 kHz deviation, plus a little complex noise."""
    t = np.arange(n) / fs
    L = np.sin(2 * np.pi * left_hz * t) if left_hz else np.zeros(n)
    R = np.sin(2 * np.pi * right_hz * t) if right_hz else np.zeros(n)
    th = 2 * np.pi * 19000 * t
    mpx = 0.45 * (L + R) + 0.45 * (L - R) * np.cos(2 * th) + 0.1 * np.cos(th)
    ph = 2 * np.pi * 75000 * np.cumsum(mpx) / fs
    rng = np.random.default_rng(seed)
    return (0.5 * np.exp(1j * ph) + 1e-3 * (rng.standard_normal(n) + 1j * rng.standard_normal(n))).astype(np.complex64)


@pytest.mark.parametrize("low_pass", [True, False])
def test_broadcast_fm_stereo_vs_oracle(low_pass):
    """Stereo decoder (pilot band-pass -> PLL -> matrix -> low-pass) vs the oracle's float
    restatement of broadcast_fm.h / pll.h. The PLL uses cosf/sinf/atan2f, whose last bits
    differ between the GPU's and the host's libm: the loop filter keeps those differences at
    the ulp level of the phase, so the audio agrees to 2e-5 of full scale."""
    fs = 240000.0
    x = fm_stereo_iq(72000, fs)
    g = dsp.BroadcastFM(100000, fs, low_pass, stereo=True)
    o = oracle.BroadcastFMStereo(100000, fs, True, low_pass)
    for s, e in [(0, 7000), (7000, 40000), (40000, 72000)]:
        a, b = g.process(x[s:e]), o.process(x[s:e])
        assert a.shape == b.shape
        for ch in ("l", "r"):
            err = np.abs(a[ch].astype(np.float64) - b[ch]).max()
            assert err <= 2e-5 * max(np.abs(b[ch]).max(), 1.0), f"{ch} block {s}: {err:.3e}"


def test_broadcast_fm_stereo_mono_path_equals_wfm(rng):
    fs = 240000.0
    x = fm_stereo_iq(20000, fs)
    a = dsp.BroadcastFM(100000, fs, True, stereo=False).process(x)
    o = oracle.BroadcastFMStereo(100000, fs, False, True).process(x)
    assert np.abs(a["l"] - o["l"]).max() <= 2e-5 and np.array_equal(a["l"], a["r"])
