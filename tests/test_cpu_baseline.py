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


def test_fast_channelizer_branch_fir_matches_numpy():
    """C4's CPU leg: the C branch FIRs (cpu_fast.c cf_chan_fir) equal the numpy restatement
    u[f] = sum_q h[q] x[f + q] (fp32 sums in tap order up to the vector FMA contraction)."""
    M, Q, frames = 1024, 16, 70
    x = _x((frames + Q - 1) * M, 11).reshape(frames + Q - 1, M)
    h = oracle.windowed_sinc(Q * M, np.pi / M).reshape(Q, M).astype(np.float32)
    u = oracle.chan_branch_fir(np.ascontiguousarray(x), np.ascontiguousarray(h), frames)
    ref = np.zeros((frames, M), np.complex128)
    for q in range(Q):
        ref += h[q].astype(np.float64) * x[q:q + frames].astype(np.complex128)
    assert np.abs(u - ref).max() <= 1e-6 * (1 + np.abs(ref).max())


def test_spread_placement_one_stream_per_l3(monkeypatch):
    """The all-core CPU leg's spread placement: on a 2-socket host with 4 L3
    domains per socket and SMT siblings, 8 streams land one per L3 domain, alternating sockets, on
    first threads of distinct cores; 12 streams start a second core per domain only after every
    domain has one. The packed placement is the first CPUs in order."""
    import cpu_baseline as cb
    # cpu c: socket c // 32 (SMT sibling c + 64 on the same core), L3 domain (c % 64) // 8 within it
    cpus = list(range(128))

    def topo(cs):
        out = {}
        for c in cs:
            p = c % 64
            out[c] = (str(p // 32), f"l3-{p // 8}", f"core-{p}")
        return out
    monkeypatch.setattr(cb, "cpu_topology", topo)
    place, info = cb.placements(cpus, 8)
    assert info == {"sockets": 2, "l3_domains": 8}
    assert place["packed"] == list(range(8))
    sp = place["spread"]
    assert len(set((c % 64) // 8 for c in sp)) == 8            # one per L3 domain
    assert [(c % 64) // 32 for c in sp] == [0, 1] * 4           # sockets alternate
    assert all(c < 64 for c in sp)                               # first SMT thread of each core
    sp12 = cb.placements(cpus, 12)[0]["spread"]
    assert sp12[:8] == sp and len(set(sp12)) == 12 and all(c < 64 for c in sp12)


def test_measure_one_core_not_below_streams():
    """the 1-core figure is never below what a stream of the all-core leg reached,
    so the all-core aggregate is at most (stream count) x the 1-core figure and the whole-host bound
    bench.py builds on it is not understated."""
    import cpu_baseline as cb
    r = cb.measure("c3", 0.3, max_cores=2)
    assert r["value_1core"] >= r["value_1core_run"] and r["value_1core"] >= r["value_1core_spread_mean"]
    assert r["value_all_cores"] <= r["cores_all"] * r["value_1core"] * (1 + 1e-9), r
    assert r["value_1core_cpu"] in r["host"]["placement"]["cpus_spread"]
