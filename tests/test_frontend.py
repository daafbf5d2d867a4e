"""Device IQ front end (sdrgpu_frontend_*, the IQFrontEnd data path) vs the same stages run
one by one and vs the oracle.

- Framing follows the Reshaper (keep nz, skip; genReshapeParams): the rows a stream of
  ragged pushes produces are BIT-IDENTICAL to one spectrum batch over the whole stream with
  frame stride nz + skip (same kernels: the front end's plans run the 64k transform as the two-pass
  launches, _util.two_pass_fft; same frame data, including frames stitched across two pushes).
- VFO outputs equal a standalone RxVFO fed the same blocks, bit for bit.
- C1: file_source-style 2.4 MS/s blocks of fs/200 samples, 64k BH7, fftRate 15
  -> nz 65,536, skip 94,464; every row vs the fp64 truth (tests/_util.py db_check).
- Raw u8 / i16 ingest through the front end equals converting first.
"""
import numpy as np
import pytest

import oracle
import sdrpp_amd
from sdrpp_amd import dsp
from _util import db_check, iq, ref32_fft_db, two_pass_fft

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    assert sdrpp_amd.lib.sdrgpu_device_count() > 0, "no HIP device visible: gpu tests need an MI355X"


def multitone(n, fs, seed=0xACE1):
    """C1 input: tones + xorshift-like noise (test_source style), complex64."""
    rng = np.random.default_rng(seed)
    t = np.arange(n) / fs
    x = 0.3 * np.exp(2j * np.pi * 150e3 * t) + 0.05 * np.exp(-2j * np.pi * 431e3 * t + 0.7j) + 0.001 * np.exp(2j * np.pi * 7e3 * t)
    x = x + 1e-4 * (rng.standard_normal(n) + 1j * rng.standard_normal(n))
    return x.astype(np.complex64)


def pushes(x, sizes):
    i = 0
    k = 0
    while i < len(x):
        c = sizes[k % len(sizes)]
        yield x[i:i + c]
        i += c
        k += 1


def test_c1_framing_and_truth():
    fs, N, rate = 2.4e6, 65536, 15.0
    fe = dsp.IQFrontEnd(fs, fft_size=N, fft_rate=rate)
    nz, skip, sr = fe.framing()
    assert (nz, skip, sr) == (65536, 94464, fs)
    x = multitone(int(fs * 2.2), fs)                      # 2.2 s -> 33 frames
    rows = [fe.push(b) for b in pushes(x, [int(fs / 200)])]   # file_source block = fs/200
    rows = np.concatenate(rows)
    stride = nz + skip
    nframes = (len(x) - nz) // stride + 1
    assert rows.shape == (nframes, N)
    # bit-identical to one batch with the reshaper's stride
    sp = two_pass_fft(N, nz)
    w = oracle.create_window(6, nz)
    for j in (0, 1, nframes // 2, nframes - 1):
        frame = x[j * stride:j * stride + nz]
        db_check(rows[j], oracle.fft_truth_power(frame, nz, N, w), N, ref32_fft_db(frame, nz, N, w))
        assert np.array_equal(rows[j], sp.logmag(frame))


@pytest.mark.parametrize("sizes", [[1000, 77777, 3, 131072], [65535, 65537], [200000]])
def test_ragged_pushes_bit_identical(sizes, rng):
    fs, N = 10e6, 16384
    fe = dsp.IQFrontEnd(fs, fft_size=N, fft_rate=fs / 20000)     # interval 20000 -> nz 16384, skip 3616
    nz, skip, _ = fe.framing()
    assert (nz, skip) == (16384, 3616)
    x = iq(rng, 600000)
    rows = np.concatenate([fe.push(b) for b in pushes(x, sizes)])
    stride = nz + skip
    n = (len(x) - nz) // stride + 1
    assert rows.shape[0] == n
    sp = two_pass_fft(N, nz)
    for j in range(n):
        assert np.array_equal(rows[j], sp.logmag(x[j * stride:j * stride + nz])), f"frame {j}"


def test_zero_pad_framing(rng):
    """C2-style framing: interval < N -> nz = interval, skip 0, zero-padded FFT."""
    fs, N = 1e6, 65536
    fe = dsp.IQFrontEnd(fs, fft_size=N, fft_rate=25.0)           # interval 40000 < N
    nz, skip, _ = fe.framing()
    assert (nz, skip) == (40000, 0)
    x = iq(rng, 205000)
    rows = np.concatenate([fe.push(b) for b in pushes(x, [30011])])
    assert rows.shape[0] == len(x) // nz
    sp = two_pass_fft(N, nz)
    for j in range(rows.shape[0]):
        assert np.array_equal(rows[j], sp.logmag(x[j * nz:(j + 1) * nz]))


def test_vfos_match_standalone(rng):
    fs = 61.44e6
    fe = dsp.IQFrontEnd(fs, fft_size=65536, fft_rate=fs / 65536)
    a = fe.add_vfo(240000, 200000, 2.5e6)
    b = fe.add_vfo(48000, 12500, -7.3e6)
    va, vb = dsp.RxVFO(fs, 240000, 200000, 2.5e6), dsp.RxVFO(fs, 48000, 12500, -7.3e6)
    x = iq(rng, 5 * 307200)
    for blk in pushes(x, [307200]):
        fe.push(blk)
        assert np.array_equal(fe.vfo_output(a), va.process(blk))
        assert np.array_equal(fe.vfo_output(b), vb.process(blk))
    fe.remove_vfo(b)
    fe.push(x[:307200])


@pytest.mark.parametrize("kind,dtype", [(sdrpp_amd.CONV_U8, np.uint8), (sdrpp_amd.CONV_I16, np.int16)])
def test_raw_ingest(kind, dtype, rng):
    fs, N = 2.4e6, 8192
    raw = rng.integers(np.iinfo(dtype).min, np.iinfo(dtype).max, 2 * 100000, endpoint=True).astype(dtype)
    x = oracle.convert(kind, raw).view(np.complex64)
    fe_raw = dsp.IQFrontEnd(fs, fft_size=N, fft_rate=200.0)
    fe_f = dsp.IQFrontEnd(fs, fft_size=N, fft_rate=200.0)
    for r, f in zip(np.array_split(raw.reshape(-1, 2), 7), np.array_split(x, 7)):
        assert np.array_equal(fe_raw.push(r.reshape(-1), kind), fe_f.push(f))


def test_preproc_decim_dcblock_invert(rng):
    """decimation + DC blocking + IQ inversion (iq_frontend.cpp:29-39) vs the oracle stages."""
    fs = 8e6
    fe = dsp.IQFrontEnd(fs, decim=4, dc_blocking=True, fft_size=4096, fft_rate=100.0)
    fe.set_invert_iq(True)
    nz, skip, sr = fe.framing()
    assert sr == fs / 4
    vid = fe.add_vfo(sr, sr, 0.0)                  # identity VFO: observes the preprocessed stream
    x = (iq(rng, 400000) + (0.2 - 0.1j)).astype(np.complex64)
    dec = oracle.PowerDecimator(4)
    dcb = oracle.DCBlocker(50.0 / sr, complex_data=True)
    got, want = [], []
    for blk in pushes(x, [40000]):
        fe.push(blk)
        got.append(fe.vfo_output(vid))
        want.append(np.conj(dcb.process(dec.process(blk))))
    got, want = np.concatenate(got), np.concatenate(want)
    assert got.shape == want.shape
    assert np.abs(got - want).max() <= 2e-5 * np.abs(want).max()


def test_pipelined_submit_collect_matches_push():
    """sdrgpu_frontend_submit / collect (the drop-in worker's pipelined call style: H2D of block
    k + 1 on the copy stream while block k computes and reads back) gives, block for block, the
    rows, VFO outputs and preprocessed IQ of the synchronous push -- bit for bit -- for ragged
    blocks, with two tickets in flight, from pageable and from sdrgpu_host_alloc'ed memory."""
    import ctypes
    fs, N = 2.4e6, 8192
    x = multitone(int(fs * 0.4), fs, seed=11)
    sizes = [12000, 5000, 31000, 777, 12000]
    blocks = list(pushes(x, sizes))
    ref = dsp.IQFrontEnd(fs, fft_size=N, fft_rate=60.0)
    rv = ref.add_vfo(48000, 12500, 150e3)
    want = []
    for b in blocks:
        r = ref.push(b)
        want.append((r, ref.vfo_output(rv)))
    ref.close()
    # host_alloc'ed staging: DMA'd straight from the caller's buffer
    hp = ctypes.c_void_p()
    sdrpp_amd.check(sdrpp_amd.lib.sdrgpu_host_alloc(ctypes.byref(hp), 8 * max(sizes)))
    pinned = np.ctypeslib.as_array((ctypes.c_float * (2 * max(sizes))).from_address(hp.value)).view(np.complex64)
    try:
        for use_pinned in (False, True):
            fe = dsp.IQFrontEnd(fs, fft_size=N, fft_rate=60.0)
            vid = fe.add_vfo(48000, 12500, 150e3)
            got, pend = [], []
            for k, b in enumerate(blocks):
                if use_pinned:
                    if pend:   # the pinned buffer is reused: the previous H2D must be done -> collect first
                        got.append(fe.collect(pend.pop(0), vfos=[vid]))
                    pinned[:len(b)] = b
                    t = fe.submit(None, ptr=pinned.ctypes.data, count=len(b), want_iq=True)
                else:
                    t = fe.submit(b, want_iq=True)
                pend.append(t)
                if len(pend) == 2:
                    got.append(fe.collect(pend.pop(0), vfos=[vid]))
            while pend:
                got.append(fe.collect(pend.pop(0), vfos=[vid]))
            with pytest.raises(sdrpp_amd.SdrGpuError):
                fe.collect(12345)   # not in flight
            fe.close()
            assert len(got) == len(blocks)
            for k, ((r, o, iq_), (wr, wo), b) in enumerate(zip(got, want, blocks)):
                assert np.array_equal(r, wr), (use_pinned, k)
                assert np.array_equal(o[vid], wo), (use_pinned, k)
                assert np.array_equal(iq_, b), (use_pinned, k)
    finally:
        sdrpp_amd.lib.sdrgpu_host_free(hp)


def test_submit_refuses_a_third_ticket():
    fe = dsp.IQFrontEnd(2.4e6, fft_size=4096, fft_rate=60.0)
    b = multitone(12000, 2.4e6)
    t0 = fe.submit(b)
    t1 = fe.submit(b)
    with pytest.raises(sdrpp_amd.SdrGpuError):
        fe.submit(b)
    fe.collect(t0)
    t2 = fe.submit(b)
    fe.collect(t1)
    fe.collect(t2)
    fe.close()
