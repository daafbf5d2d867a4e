"""file_source ingest: the WAV container reader (sdrgpu_wav_*, wavreader.h:34-226) on the host,
and on the GPU the worker's sample conversion (main.cpp:294-560) feeding the IQ front end (C1:
file_source WAV 2.4 MS/s -> 64k BH7 spectra)."""
import struct

import numpy as np
import pytest

import oracle
import sdrpp_amd
from sdrpp_amd import dsp

PCM, IEEE_FLOAT, EXTENSIBLE = 1, 3, 0xFFFE


def fmt_chunk(tag, ch, sr, bits, size=16, subformat=None, align=None):
    align = ch * bits // 8 if align is None else align
    body = struct.pack("<HHIIHH", tag, ch, sr, sr * align, align, bits)
    if size == 18:
        body += struct.pack("<H", 0)
    elif size == 40:
        body += struct.pack("<HHIIHHQ", 22, bits, 3, subformat, 0, 0x10, 0x719B3800AA000080)
    elif size != 16:
        body += b"\0" * (size - 16)
    return b"fmt " + struct.pack("<I", len(body)) + body


def write_wav(path, data, tag, ch, sr, bits, fmt_size=16, subformat=None, rf64=False, before=b"", after=b"",
              align=None):
    """A WAVE file: [ds64] fmt [extra chunk] data [trailing chunk]."""
    chunks = b""
    if rf64:
        chunks += b"ds64" + struct.pack("<I", 28) + struct.pack("<QQQI", 0, len(data), 0, 0)
    chunks += fmt_chunk(tag, ch, sr, bits, fmt_size, subformat, align) + before
    chunks += b"data" + struct.pack("<I", len(data)) + data + after
    head = (b"RF64" if rf64 else b"RIFF") + struct.pack("<I", 4 + len(chunks)) + b"WAVE"
    path.write_bytes(head + chunks)
    return path


@pytest.mark.parametrize("variant", ["plain", "fmt18", "extensible", "rf64", "extra_chunk"])
def test_wav_header_and_blocks(variant, tmp_path):
    rng = np.random.default_rng(5)
    sr = 48000                                   # block = fs / 200 = 240 frames
    x = rng.integers(-32768, 32767, size=(1000, 2), dtype=np.int16)
    kw = dict(tag=PCM, ch=2, sr=sr, bits=16)
    if variant == "fmt18":
        kw["fmt_size"] = 18
    if variant == "extensible":
        kw.update(tag=EXTENSIBLE, fmt_size=40, subformat=1)
    if variant == "rf64":
        kw["rf64"] = True
    if variant == "extra_chunk":
        kw["before"] = b"LIST" + struct.pack("<I", 6) + b"abcdef"
    w = dsp.WavFile(write_wav(tmp_path / "a.wav", x.tobytes(), **kw))
    assert (w.format, w.channels, w.bits, w.sample_rate, w.sample_count) == (PCM, 2, 16, sr, 1000)
    assert w.kind == sdrpp_amd.CONV_I16 and w.block_size == 240
    blocks = list(w.blocks())
    assert [b.size // 4 for b in blocks] == [240, 240, 240, 240, 40]
    assert np.array_equal(np.concatenate(blocks).view(np.int16).reshape(-1, 2), x)
    w.seek(990)
    assert np.array_equal(w.read().view(np.int16).reshape(-1, 2), x[990:])
    w.close()


def test_wav_samples_run_to_end_of_file(tmp_path):
    """The reference reads [data offset, EOF): a chunk after 'data' is read as samples; a partial
    frame at the end is dropped (getSampleCount / readSamples, wavreader.h:85-88, 207-221)."""
    x = np.arange(40, dtype=np.float32)            # 20 complex frames
    tail = b"LIST" + struct.pack("<I", 8) + b"12345678" + b"xyz"   # 19 bytes: 2 frames + 3 bytes
    w = dsp.WavFile(write_wav(tmp_path / "b.wav", x.tobytes(), IEEE_FLOAT, 2, 2400000, 32, after=tail))
    assert w.kind == sdrpp_amd.CONV_F32 and w.sample_count == 22 and w.block_size == 12000
    raw = w.read()
    assert raw.size == 22 * 8
    assert np.array_equal(raw[:160].view(np.float32), x)


def test_wav_rejects(tmp_path):
    x = np.zeros(16, np.int16).tobytes()
    bad = tmp_path / "bad.wav"
    bad.write_bytes(b"RIFX" + b"\0" * 40)
    with pytest.raises(sdrpp_amd.SdrGpuError):
        dsp.WavFile(bad)
    with pytest.raises(sdrpp_amd.SdrGpuError):        # fmt size 17 (wavreader.h:136)
        dsp.WavFile(write_wav(tmp_path / "c.wav", x, PCM, 2, 8000, 16, fmt_size=17))
    with pytest.raises(sdrpp_amd.SdrGpuError):        # EXTENSIBLE with an unknown SubFormat
        dsp.WavFile(write_wav(tmp_path / "d.wav", x, EXTENSIBLE, 2, 8000, 16, fmt_size=40, subformat=7))
    with pytest.raises(sdrpp_amd.SdrGpuError):        # 3 channels: no worker (main.cpp:301, 445)
        dsp.WavFile(write_wav(tmp_path / "e.wav", x[:12], PCM, 3, 8000, 16))
    with pytest.raises(sdrpp_amd.SdrGpuError):        # 12-bit PCM: not a supported sample format
        dsp.WavFile(write_wav(tmp_path / "f.wav", x, PCM, 2, 8000, 12))


@pytest.mark.parametrize("align", [8, 5, 2, 0])
def test_wav_rejects_block_align_mismatch(align, tmp_path):
    """wBlockAlign must equal channels x bits / 8: the reference workers read the sample region as
    a packed stream of such frames (main.cpp:320-537), so a padded or malformed block align is
    rejected at open instead of framing (or over-reading) the samples by it."""
    x = np.zeros(64, np.int16).tobytes()
    with pytest.raises(sdrpp_amd.SdrGpuError):
        dsp.WavFile(write_wav(tmp_path / "g.wav", x, PCM, 2, 8000, 16, align=align))
    ok = dsp.WavFile(write_wav(tmp_path / "h.wav", x, PCM, 2, 8000, 16, align=4))
    assert ok.sample_count == 32 and ok.read().size == 128


@pytest.mark.gpu
@pytest.mark.parametrize("ch,bits,tag", [(2, 8, PCM), (2, 16, PCM), (2, 24, PCM), (2, 32, PCM), (2, 64, IEEE_FLOAT),
                                         (1, 8, PCM), (1, 16, PCM), (1, 24, PCM), (1, 32, IEEE_FLOAT), (1, 64, IEEE_FLOAT)])
def test_wav_conversion_bit_exact(ch, bits, tag, tmp_path):
    """Every sample format of worker_1ch / worker_2ch through the GPU converter, bit for bit
    against the oracle's restatement (1 channel: I = Q = the converted sample)."""
    rng = np.random.default_rng(bits * 10 + ch)
    n = 5000 * ch
    if tag == IEEE_FLOAT:
        vals = rng.standard_normal(n).astype(np.float32 if bits == 32 else np.float64)
        raw = vals.tobytes()
    elif bits == 24:
        raw = rng.integers(0, 256, size=3 * n, dtype=np.uint8).tobytes()
    else:
        dt = {8: np.uint8, 16: np.int16, 32: np.int32}[bits]
        info = np.iinfo(dt)
        raw = rng.integers(info.min, info.max, size=n, dtype=dt, endpoint=True).tobytes()
    w = dsp.WavFile(write_wav(tmp_path / "s.wav", raw, tag, ch, 2400000, bits))
    got = np.concatenate([w.samples(b) for b in w.blocks()])
    assert got.size == 5000
    kind = w.kind
    if kind == sdrpp_amd.CONV_F32:
        ref = np.frombuffer(raw, np.float32)
    else:
        typed = np.frombuffer(raw, {0: np.uint8, 1: np.int16, 2: np.uint8, 3: np.int32, 4: np.float64}[kind])
        ref = oracle.convert(kind, typed)
    ref = np.repeat(ref, 2) if ch == 1 else ref
    assert np.array_equal(got.view(np.float32).view(np.uint32), ref.astype(np.float32).view(np.uint32))


@pytest.mark.gpu
def test_c1_wav_file_to_spectra(tmp_path):
    """C1 at SURVEY 8(d)'s size: 30 s of a 2-channel IEEE_FLOAT32 WAV at 2.4 MS/s (72 M samples,
    576 MB) read in file_source blocks (fs / 200) through the device front end (64k BH7, fftRate
    15 -> nz 65,536, skip 94,464, 450 frames): every row equals the front end fed the same samples
    directly in one push, and every 10th row (and the last) meets the spectrum parity bar against
    the fp64 truth."""
    from _util import db_check, ref32_fft_db
    fs, N, secs = 2400000, 65536, 30
    n = fs * secs
    rng = np.random.default_rng(0xACE1)
    x = np.empty(n, np.complex64)
    step = 1 << 22
    for a in range(0, n, step):                 # built in slices: fp64 phases without a 1 GB temp
        t = np.arange(a, min(a + step, n)) / fs
        x[a:a + t.size] = (0.3 * np.exp(2j * np.pi * 150e3 * t) + 0.05 * np.exp(-2j * np.pi * 431e3 * t)
                           + 1e-4 * (rng.standard_normal(t.size) + 1j * rng.standard_normal(t.size)))
    w = dsp.WavFile(write_wav(tmp_path / "c1.wav", x.tobytes(), IEEE_FLOAT, 2, fs, 32))
    assert w.block_size == fs // 200 and w.sample_count == n
    fe = dsp.IQFrontEnd(fs, fft_size=N, fft_rate=15.0)
    rows = np.concatenate([r for r in (fe.push(w.samples(b)) for b in w.blocks()) if r.shape[0]])
    w.close()
    nz, skip, _ = fe.framing()
    assert (nz, skip) == (65536, 94464)
    ref_fe = dsp.IQFrontEnd(fs, fft_size=N, fft_rate=15.0)
    ref_rows = ref_fe.push(x)
    assert rows.shape == ref_rows.shape == ((n - nz) // (nz + skip) + 1, N) == (450, N)
    assert np.array_equal(rows, ref_rows)
    win = oracle.create_window(6, nz)
    for j in sorted(set(range(0, rows.shape[0], 10)) | {rows.shape[0] - 1}):
        frame = x[j * (nz + skip):j * (nz + skip) + nz]
        db_check(rows[j], oracle.fft_truth_power(frame, nz, N, win), N, ref32_fft_db(frame, nz, N, win))
