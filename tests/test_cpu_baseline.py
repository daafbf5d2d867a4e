"""The CPU baseline's fast kernels (oracle/cpu_fast.c: vectorised rotator, 8-outputs-per-pass
decimating FIR, polynomial-atan quadrature; the precise = 0 paths bench.py's cpu_baseline leg
times) compute the same chains as the parity oracle (precise = 1): a fast baseline that computed
something else would make every GPU / CPU ratio meaningless."""
import numpy as np

import oracle


def _x(n, seed=5):
    rng = np.random.default_rng(seed)
    return (rng.uniform(-1, 1, n) + 1j * rng.uniform(-1, 1, n)).astype(np.complex64)


def test_fast_decimating_fir_matches_precise():
    x = _x(200003)
    for ntaps, D in ((256, 8), (143, 32), (27, 4), (69, 2), (91, 1), (256, 3)):
        taps = (np.random.default_rng(ntaps).standard_normal(ntaps) / ntaps).astype(np.float32)
        f0, f1 = oracle.FIR(taps, D, True, precise=True), oracle.FIR(taps, D, True, precise=False)
        a = f0.process(x)
        parts = [f1.process(p) for p in np.split(x, [777, 50000, 50001, 130000])]   # ragged calls
        b = np.concatenate(parts)
        assert len(a) == len(b), (ntaps, D)
        assert np.abs(a - b).max() <= 1e-5 * (1 + np.abs(a).max()), (ntaps, D)


def test_fast_ddcfm_matches_precise():
    """C3 chain: xlator -> 256-tap FIR / 8 -> quadrature."""
    x = _x(400000, 7)
    taps = oracle.low_pass(3.0e6, 912000.0, 61.44e6)
    args = (2 * np.pi * (-1.5e6 / 61.44e6), taps, 8, 2 * np.pi * 100e3 / (61.44e6 / 8))
    a = oracle.DDCFM(*args, precise=True).process(x)
    d = oracle.DDCFM(*args, precise=False)
    b = np.concatenate([d.process(p) for p in np.split(x, [100001, 250000])])
    assert len(a) == len(b)
    err = np.abs(a - b)
    assert np.median(err) < 1e-4 and np.quantile(err, 0.999) < 1e-2, (np.median(err), err.max())


def test_fast_rxvfo_wfm_match_precise():
    """C5 VFO chain: RxVFO 61.44 MHz -> 240 kHz -> BroadcastFM mono."""
    x = _x(307200 * 3, 9)
    v0, v1 = oracle.RxVFO(61.44e6, 240000, 200000, 2.5e6, precise=True), oracle.RxVFO(61.44e6, 240000, 200000, 2.5e6, precise=False)
    w0, w1 = oracle.BroadcastFM(100000, 240000, True, precise=True), oracle.BroadcastFM(100000, 240000, True, precise=False)
    a = w0.process(v0.process(x))
    b = np.concatenate([w1.process(v1.process(p)) for p in np.split(x, [307200, 614400])])
    assert a.shape == b.shape
    a, b = a.view(np.float32), b.view(np.float32)
    assert np.abs(a - b).max() < 2e-3, np.abs(a - b).max()
