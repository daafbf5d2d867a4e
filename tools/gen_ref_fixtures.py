"""Fixtures produced by the REFERENCE's own code (oracle/_ref/ref_probe, compiled from the
reference tree's header-only window/math/types/taps headers): run in the dev container where
/root/reference exists; the outputs are committed under tests/golden/ref_*.npz so the GPU box
(which has no reference tree) checks against them."""
import hashlib
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROBE = os.path.join(ROOT, "oracle", "_ref", "ref_probe")
OUT = os.path.join(ROOT, "tests", "golden")


def probe(*args, stdin=None):
    return subprocess.run([PROBE, *map(str, args)], input=stdin, capture_output=True, check=True).stdout


def main():
    subprocess.check_call(["make", "-C", os.path.join(ROOT, "oracle"), "-s", "ref"])
    w = {}
    for t in range(7):
        w[f"w{t}_4096_c"] = np.frombuffer(probe("window", t, 4096, 1), np.float32)
        w[f"w{t}_1000_n"] = np.frombuffer(probe("window", t, 1000, 0), np.float32)
    w["w6_65536_c"] = np.frombuffer(probe("window", 6, 65536, 1), np.float32)
    w["w6_4097_c"] = np.frombuffer(probe("window", 6, 4097, 1), np.float32)   # odd: reference writes w[size]
    np.savez_compressed(os.path.join(OUT, "ref_windows.npz"), **w)
    with open(os.path.join(OUT, "ref_windows_sha256.txt"), "w") as f:
        for n in (1000000, 1 << 20, 666667):
            f.write(f"{n} {hashlib.sha256(probe('window', 6, n, 1)).hexdigest()}\n")
    taps = {}
    for name, args in {"vfo_lpf": (100000.0, 10000.0, 240000.0), "wfm_audio": (15000.0, 4000.0, 240000.0),
                       "c3": (3.0e6, 912000.0, 61.44e6), "af_resamp": (24000.0, 2400.0, 240000.0),
                       "nfm_lpf": (6250.0, 625.0, 50000.0)}.items():
        raw = probe("lowpass", *args)
        n = int(np.frombuffer(raw[:4], np.int32)[0])
        taps[name] = np.frombuffer(raw[4:], np.float32)
        assert len(taps[name]) == n
    np.savez_compressed(os.path.join(OUT, "ref_taps.npz"), **taps)
    rng = np.random.default_rng(0xACE1)
    x = (rng.uniform(-1, 1, 50000) + 1j * rng.uniform(-1, 1, 50000)).astype(np.complex64)
    dev = 2 * np.pi * 100e3 / 7.68e6
    y = np.frombuffer(probe("quad", f"{float(dev):.17g}", stdin=x.tobytes()), np.float32)
    offs = np.array([2 * np.pi * (-1.5e6 / 61.44e6), 2 * np.pi * (-2.5e6 / 61.44e6), 2 * np.pi * (2.5e6 / 61.44e6)])
    deltas = np.stack([np.frombuffer(probe("xlatordelta", f"{float(o):.17g}"), np.float32) for o in offs])
    np.savez_compressed(os.path.join(OUT, "ref_quad.npz"), x=x, dev=dev, y=y, offs=offs, deltas=deltas)
    print("reference-code fixtures written")


if __name__ == "__main__":
    main()
