"""Generate the committed golden fixtures under tests/golden/ (run in the dev container).

The reference ships no DSP tests or vectors and cannot be built here,
so fixtures are produced by INDEPENDENT numpy/fp64 evaluations of the reference's
formulas (file:line cited per fixture) and, where noted, by the oracle. They pin the
oracle (CPU suite) and the GPU path (gpu suite) to the same numbers.
"""
import hashlib
import math
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden")
os.makedirs(OUT, exist_ok=True)
PI = 3.14159265358979323846

COEFS = {  # window/*.h
    0: [1.0], 1: [0.53836, 0.46164], 2: [0.5, 0.5], 3: [0.42, 0.5, 0.08],
    4: [0.355768, 0.487396, 0.144232, 0.012604], 5: [0.35875, 0.48829, 0.14128, 0.01168],
    6: [0.27105140069342, 0.43329793923448, 0.21812299954311, 0.06592544638803, 0.01081174209837,
        0.00077658482522, 0.00001388721735],
}


def window_py(wtype, size, centered=True):
    """window/window.h:38-64 + cosine.h:7-16, evaluated with Python floats (IEEE double, libm cos)."""
    buf = np.empty(size, dtype=np.float32)
    c = COEFS[wtype]
    for n in range(size):
        if wtype == 0:
            v = 1.0
        else:
            v, sign = 0.0, 1.0
            for i, a in enumerate(c):
                v += sign * a * math.cos(float(i) * 2.0 * PI * n / size)
                sign = -sign
        buf[n] = np.float32(v)
    ws = 0.0
    for v in buf:
        ws += float(v)
    ws = 1.0 / ws
    out = np.empty_like(buf)
    for n in range(size):
        s = (-ws if (n % 2 == 0) else ws) if centered else ws
        out[n] = np.float32(float(buf[n]) * s)
    return out


def main():
    # 1. windows: bit-exact tables (all types at 4096, BH7 at 65536) + sha256 of BH7 at 1e6 / 2^20
    win = {f"w{t}_4096": window_py(t, 4096) for t in range(7)}
    win["w6_65536"] = window_py(6, 65536)
    np.savez_compressed(os.path.join(OUT, "windows.npz"), **win)
    sha = {}
    for n in (1000000, 1 << 20):
        sha[str(n)] = hashlib.sha256(oracle.create_window(6, n).tobytes()).hexdigest()
    with open(os.path.join(OUT, "windows_sha256.txt"), "w") as f:
        for k, v in sha.items():
            f.write(f"{k} {v}\n")

    # 2. converters (file_source/src/main.cpp:489,506,522-525): numpy float32 IEEE division
    u8 = np.arange(256, dtype=np.int32)
    i16 = np.arange(-32768, 32768, dtype=np.int32)
    conv_u8 = (((u8 - 128).astype(np.float32) + np.float32(0.5)) / np.float32(127.5)).astype(np.float32)
    conv_i16 = ((i16.astype(np.float32) + np.float32(0.5)) / np.float32(32767.5)).astype(np.float32)
    np.savez_compressed(os.path.join(OUT, "converters.npz"), u8=conv_u8, i16=conv_i16)

    # 3. taps used on the hot path (fp64 numpy restatement of taps/windowed_sinc.h + low_pass.h)
    def low_pass_np(cutoff, tw, fs):
        count = int(3.8 * fs / tw)
        omega = 2.0 * PI * (cutoff / fs)
        half = count / 2.0
        corr = omega / PI
        out = np.empty(count, dtype=np.float32)
        for i in range(count):
            t = i - half + 0.5
            s = 1.0 if t * omega == 0.0 else math.sin(t * omega) / (t * omega)
            n = t - half
            w, sign = 0.0, 1.0
            for k, a in enumerate(COEFS[4]):
                w += sign * a * math.cos(float(k) * 2.0 * PI * n / count)
                sign = -sign
            out[i] = np.float32(s * w * corr)
        return out
    taps = {
        "vfo_lpf_91": low_pass_np(100000.0, 10000.0, 240000.0),        # rx_vfo.h:117-121 (bw 200 kHz)
        "wfm_audio_228": low_pass_np(15000.0, 4000.0, 240000.0),       # broadcast_fm.h:40
        "c3_256": low_pass_np(3.0e6, 912000.0, 61.44e6),               # BASELINE C3
        "af_resamp_380": low_pass_np(24000.0, 2400.0, 240000.0) * np.float32(4),  # rational_resampler.h:152-155 (x interp)
    }
    np.savez_compressed(os.path.join(OUT, "taps.npz"), **taps)

    # 4. spectrum of the test_source AES17 0 dBFS 14-bit table (test_source/src/main.cpp:41-48, 82-93)
    tab = np.array([0x3fff, 0x0c3e, 0x16a0, 0x1d8f, 0x1fff, 0x1d8f, 0x16a0, 0x0c3e, 0x0000, 0x33c1, 0x295f, 0x2270,
                    0x2000, 0x2270, 0x295f, 0x33c1], dtype=np.int64)
    v = ((tab << 50) >> 50).astype(np.float64) * (1.0 / ((1 << 14) / 2 - 1))
    N = 65536
    xi = np.tile(v.astype(np.float32), N // 16)
    x = (xi + 0j).astype(np.complex64)   # TableSource::next(): I = table, Q = 0
    w = oracle.create_window(6, N)
    power = oracle.fft_truth_power(x, N, N, w)
    import scipy.fft
    buf = (x * w).astype(np.complex64)
    X = scipy.fft.fft(buf, workers=1)
    p32 = X.real.astype(np.float32) ** 2 + X.imag.astype(np.float32) ** 2
    with np.errstate(divide="ignore"):
        db32 = (10.0 * np.log10(p32.astype(np.float64))).astype(np.float32)
    np.savez_compressed(os.path.join(OUT, "fft_aes17.npz"), N=N, x=x, power_f64=power, db_ref32=db32)

    # 5. FIR known answer: C3 decimating FIR on a seeded stream, fp64-accumulated (oracle precise)
    rng = np.random.default_rng(0xACE1)
    xs = (rng.uniform(-1, 1, 20000) + 1j * rng.uniform(-1, 1, 20000)).astype(np.complex64)
    y = oracle.FIR(taps["c3_256"], 8).process(xs)
    np.savez_compressed(os.path.join(OUT, "fir_c3.npz"), x=xs, y=y)
    print("golden fixtures written to", OUT)


if __name__ == "__main__":
    main()
