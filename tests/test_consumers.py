"""Consumers beside the hot path: de-emphasis (filter/deephasis.h), the waterfall zoom
(gui/widgets/fft_scaler.h doZoom) and the IQ wire codec (compression/sample_stream_*.h).
All three are BIT-EXACT against the oracle restatements."""
import ctypes

import numpy as np
import pytest
import torch

import oracle
import sdrpp_amd
from sdrpp_amd import dsp
from _util import iq

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    assert sdrpp_amd.lib.sdrgpu_device_count() > 0, "no HIP device visible: gpu tests need an MI355X"


def _bits(a):
    return np.ascontiguousarray(a).view(np.uint32)


@pytest.mark.parametrize("stereo", [False, True])
def test_deemphasis_bit_exact(stereo, rng):
    n = 50000
    if stereo:
        x = np.zeros(n, dsp.STEREO)
        x["l"], x["r"] = rng.uniform(-1, 1, n), rng.uniform(-1, 1, n)
    else:
        x = rng.uniform(-1, 1, n).astype(np.float32)
    g, o = dsp.Deemphasis(50e-6, 48000, stereo), oracle.Deemphasis(50e-6, 48000, stereo)
    for s, e in [(0, 1), (1, 1500), (1500, 1500), (1500, n)]:
        assert np.array_equal(_bits(g.process(x[s:e])), _bits(o.process(x[s:e])))


@pytest.mark.parametrize("view", [(0.0, 2.0e6), (0.0, 0.25e6), (-0.7e6, 0.5e6), (0.9e6, 0.3e6), (0.0, 10.0)])
@pytest.mark.parametrize("out_size", [1024, 4000])
def test_zoom_bit_exact(view, out_size, rng):
    N, whole = 65536, 2.0e6
    rows = (rng.standard_normal((8, N)) * 10 - 60).astype(np.float32)
    z = dsp.Zoom(view[0], view[1], whole, N, out_size)
    d_in = torch.from_numpy(rows).cuda()
    d_out = torch.empty((8, out_size), dtype=torch.float32, device="cuda")
    z.execute_dev(d_in.data_ptr(), 8, d_out.data_ptr())
    torch.cuda.synchronize()
    got = d_out.cpu().numpy()
    for r in range(8):
        assert np.array_equal(got[r], oracle.zoom(rows[r], view[0], view[1], whole, out_size))


@pytest.mark.parametrize("pcm", [0, 1, 2])
def test_codec_bit_exact(pcm, rng):
    lib = sdrpp_amd.lib
    x = iq(rng, 100000, 0.8)
    x[1234] = 0.95 + 0.1j                                   # the signed max (re part)
    ref = oracle.compress(pcm, x)
    d_x = torch.from_numpy(x.view(np.float32)).cuda()
    d_b = torch.zeros(len(ref) + 16, dtype=torch.uint8, device="cuda")
    scratch = torch.zeros(1, dtype=torch.int32, device="cuda")
    n = sdrpp_amd.check(lib.sdrgpu_compress_dev(0, pcm, ctypes.c_void_p(d_x.data_ptr()), len(x), ctypes.c_void_p(d_b.data_ptr()),
                                                ctypes.c_void_p(scratch.data_ptr()), None))
    torch.cuda.synchronize()
    got = d_b.cpu().numpy()[:n]
    assert n == len(ref)
    assert np.array_equal(got, ref)
    # decompress on the device from the same bytes
    hdr = np.ascontiguousarray(got[:8])
    d_out = torch.empty(2 * len(x), dtype=torch.float32, device="cuda")
    m = sdrpp_amd.check(lib.sdrgpu_decompress_dev(0, hdr.ctypes.data_as(ctypes.c_void_p), ctypes.c_void_p(d_b.data_ptr() + 8), n,
                                                  ctypes.c_void_p(d_out.data_ptr()), None))
    torch.cuda.synchronize()
    y = d_out.cpu().numpy().view(np.complex64)[:m]
    yo = oracle.decompress(ref)
    assert m == len(yo) == len(x)
    assert np.array_equal(_bits(y.view(np.float32)), _bits(yo.view(np.float32)))


@pytest.mark.parametrize("kind", [0, 1, 2, 3, 4])
def test_wav_encoders_bit_exact(kind, rng):
    """Recorder WAV encoders (utils/wav.cpp:296-336) incl. out-of-range and exact-code inputs."""
    x = np.concatenate([rng.uniform(-1.2, 1.2, 200000), [-1.0, 1.0, 0.0, -0.0, 0.5, -0.5, 1.5, -3.0],
                        (np.arange(-128, 128) + 0.5) / 127.5 - 0.0]).astype(np.float32)
    ref = oracle.wav_encode(kind, x)
    d_x = torch.from_numpy(x).cuda()
    d_o = torch.zeros(len(ref) + 16, dtype=torch.uint8, device="cuda")
    n = sdrpp_amd.check(sdrpp_amd.lib.sdrgpu_wav_encode_dev(0, kind, ctypes.c_void_p(d_x.data_ptr()), len(x),
                                                            ctypes.c_void_p(d_o.data_ptr()), None))
    torch.cuda.synchronize()
    assert n == len(ref)
    assert np.array_equal(d_o.cpu().numpy()[:n], ref)


# ------------------------------------------------ WaterFall::pushFFT consumers (§8f rank 3)
def _vp(t):
    return ctypes.c_void_p(t.data_ptr())


def test_waterfall_colormap_bit_exact(rng):
    """waterfall.cpp:903-910 on zoomed rows: clamped to [min, max], pallet index by truncation;
    values on, inside and outside the range, with the reference's 1e6-entry pallet size."""
    res = 1000000
    pallet = rng.integers(0, 2 ** 32, size=res, dtype=np.uint32)
    x = rng.uniform(-160, 20, 300 * 1024).astype(np.float32)
    x[:8] = [-150.0, 0.0, -150.0000001, 1e30, -1e30, -75.0, -0.0, 5.0]
    wf_min, wf_max = np.float32(-150.0), np.float32(0.0)
    d_x, d_p = torch.from_numpy(x).cuda(), torch.from_numpy(pallet.view(np.int32)).cuda()
    d_o = torch.empty(x.size, dtype=torch.int32, device="cuda")
    sdrpp_amd.check(sdrpp_amd.lib.sdrgpu_colormap_dev(0, _vp(d_x), x.size, float(wf_min), float(wf_max), _vp(d_p), res,
                                                      _vp(d_o), None))
    torch.cuda.synchronize()
    assert np.array_equal(d_o.cpu().numpy().view(np.uint32), oracle.colormap(x, wf_min, wf_max, pallet))


@pytest.mark.parametrize("smoothing,hold_on", [(True, True), (True, False), (False, True)])
def test_waterfall_smoothing_and_hold_bit_exact(smoothing, hold_on, rng):
    """waterfall.cpp:918-925, 952-957: per-column IIR smoothing across rows and FFT hold (from
    column 1), state carried across calls (two batches of rows)."""
    w = 2000
    alpha, beta, speed = np.float32(0.3), np.float32(0.7), np.float32(0.25)
    smooth0 = rng.uniform(-100, 0, w).astype(np.float32)
    hold0 = rng.uniform(-100, 0, w).astype(np.float32)
    rows = rng.uniform(-120, 10, (37, w)).astype(np.float32)
    ref_rows, ref_s, ref_h = oracle.fft_smooth_hold(rows, smoothing, alpha, beta, smooth0, hold_on, speed, hold0)
    d_rows = torch.from_numpy(rows.copy()).cuda()
    d_s, d_h = torch.from_numpy(smooth0.copy()).cuda(), torch.from_numpy(hold0.copy()).cuda()
    for a, b in [(0, 10), (10, 37)]:
        sdrpp_amd.check(sdrpp_amd.lib.sdrgpu_fft_smooth_hold_dev(
            0, ctypes.c_void_p(d_rows.data_ptr() + 4 * a * w), b - a, w, int(smoothing), float(alpha), float(beta), _vp(d_s),
            int(hold_on), float(speed), _vp(d_h), None))
    torch.cuda.synchronize()
    assert np.array_equal(_bits(d_rows.cpu().numpy()), _bits(ref_rows))
    if smoothing:
        assert np.array_equal(_bits(d_s.cpu().numpy()), _bits(ref_s))
    if hold_on:
        assert np.array_equal(_bits(d_h.cpu().numpy()), _bits(ref_h))


@pytest.mark.parametrize("vfo", [(100e3, 50e3), (-1.1e6, 200e3), (1.19e6, 40e3), (0.0, 1e3), (0.0, 2.4e6)])
def test_vfo_signal_info_matches_reference(vfo, rng):
    """WaterFall::calculateVFOSignalInfo (waterfall.cpp:563-601) per raw row: in-band max and SNR
    against the side-band mean, including VFOs at the band edge (clamped offsets) and a bandwidth
    with no side bins (mean 0/0 = NaN, as in the reference)."""
    fft, whole = 8192, 2.4e6
    rows = rng.uniform(-130, -20, (9, fft)).astype(np.float32)
    d_rows = torch.from_numpy(rows).cuda()
    d_st = torch.empty(9, device="cuda")
    d_sn = torch.empty(9, device="cuda")
    sdrpp_amd.check(sdrpp_amd.lib.sdrgpu_vfo_signal_info_dev(0, _vp(d_rows), 9, fft, whole, vfo[0], vfo[1], _vp(d_st),
                                                             _vp(d_sn), None))
    torch.cuda.synchronize()
    st, sn = d_st.cpu().numpy(), d_sn.cpu().numpy()
    for r in range(9):
        rs, rn = oracle.vfo_signal_info(rows[r], whole, vfo[0], vfo[1])
        assert np.array_equal(_bits(np.float32(st[r])), _bits(np.float32(rs)))
        assert (np.isnan(sn[r]) and np.isnan(rn)) or np.float32(sn[r]) == np.float32(rn), (r, sn[r], rn)
