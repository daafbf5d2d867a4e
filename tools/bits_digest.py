"""Digest of the bits a build produces on fixed inputs (GPU): equal digests from two builds
(SDRGPU_LIB_PATH) show an A/B change kept every output bit.

  python tools/bits_digest.py            -> one JSON line {case: sha256[:16]}

Cases: RxVFO (C5: 61.44 MHz -> 240 kHz) over ragged host calls; BroadcastFM mono on one big call; the C5 launch group (spectrum rows,
zoom rows, VFO stage-1 + later stages) over 24 frames; the standalone spectrum over 24 frames; the fp64-interior
spectrum (64k over 300 frames, 1M over 3)."""
import hashlib
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    import torch
    from sdrpp_amd import dsp
    rng = np.random.default_rng(1234)
    out = {}

    def h(a):
        return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()[:16]

    x = (rng.uniform(-1, 1, 24 * 65536 + 4099) + 1j * rng.uniform(-1, 1, 24 * 65536 + 4099)).astype(np.complex64)
    v = dsp.RxVFO(61.44e6, 240000, 200000, 2.5e6)
    ys = [v.process(p) for p in np.split(x, [307200, 307201, 1000000])]
    out["rxvfo_host"] = h(np.concatenate(ys))

    N, F, ZW = 65536, 24, 2048
    d_x = torch.from_numpy(x[:F * N].view(np.float32)).cuda()
    rows = torch.empty(F * N, device="cuda")
    zoom = torch.empty(F * ZW, device="cuda")
    vo = torch.empty(2 * (F * N // 256 + 64), device="cuda")
    fft = dsp.FFTSpectrum(N, N, 6)
    vfo = dsp.RxVFO(61.44e6, 240000, 200000, 2.5e6)
    m = fft.execute_zoom_vfo_dev(d_x.data_ptr(), F, rows.data_ptr(), zoom.data_ptr(), ZW, vfo, vo.data_ptr())
    torch.cuda.synchronize()
    out["c5_rows"] = h(rows.cpu().numpy())
    out["c5_zoom"] = h(zoom.cpu().numpy())
    out["c5_vfo"] = h(vo[:2 * m].cpu().numpy())
    w = dsp.BroadcastFM(100000, 240000, True)   # a 1,048,576-sample call: wfm_big_kernel
    out["wfm_big"] = h(w.process(x[:1 << 20]).view(np.uint32))
    r2 = torch.empty(F * N, device="cuda")
    dsp.FFTSpectrum(N, N, 6).execute_dev(d_x.data_ptr(), N, F, r2.data_ptr())
    torch.cuda.synchronize()
    out["spectrum_rows"] = h(r2.cpu().numpy())
    # the fp64-interior mode: 300 64k frames (three chunks, several pass-B tiles per workgroup) and 3 1M frames
    g = torch.Generator(device="cuda")
    g.manual_seed(99)
    for n, nz, f in ((65536, 65536, 300), (1 << 20, 1000000, 3)):
        xs = torch.rand(2 * nz * f, device="cuda", generator=g) * 2 - 1
        r = torch.empty(n * f, device="cuda")
        dsp.FFTSpectrum(n, nz, 6, precision="f64").execute_dev(xs.data_ptr(), nz, f, r.data_ptr())
        torch.cuda.synchronize()
        out[f"spectrum_f64_{n}"] = h(r.cpu().numpy())
    print(json.dumps(out))


if __name__ == "__main__":
    main()
