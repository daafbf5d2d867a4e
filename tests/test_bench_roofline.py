"""bench.py's roofline arithmetic on the CPU: the fp64 parity mode's entry (VERDICT r5 item 5 asks for a
`roofline` of the mode in the bench line) counts the fp32 op's algorithmic bytes and reports the two passes'
double2 intermediate separately."""
import bench


def test_f64_roofline_bytes_and_fraction():
    N, nz, frames, ms = 65536, 65536, 1024, 0.75
    r = bench.f64_roofline(N, nz, frames, ms)
    algo = 8 * nz * frames + 4 * N * frames            # 12 B per sample at nz = N
    assert r["algorithmic_bytes"] == algo
    assert r["moved_bytes"] == 8 * nz * frames + 36 * N * frames   # + 16 B written + 16 B read per element
    assert r["bound"] == "hbm" and r["unit"] == "GB/s" and r["peak"] == bench.HBM_PEAK_GBS
    assert abs(r["achieved"] - algo / (ms * 1e-3) / 1e9) < 0.1
    assert abs(r["frac"] - r["achieved"] / bench.HBM_PEAK_GBS) < 1e-4


def test_f64_roofline_zero_padded_frames():
    # the C2 plan: nz = 1e6 samples read per frame, N = 2^20 bins written
    r = bench.f64_roofline(1 << 20, 1000000, 32, 0.5)
    assert r["algorithmic_bytes"] == 8 * 1000000 * 32 + 4 * (1 << 20) * 32
    assert r["moved_bytes"] > r["algorithmic_bytes"]
