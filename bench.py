"""Throughput bench for the MI355X streaming-DSP hot path (BASELINE.json metric).

Default workload (--config c5, one stream per GPU): BASELINE config C5's per-GPU slice,
i.e. a 61.44 MS/s-class IQ stream pushed as fast as the GPU takes it through
  * the IQ front end's spectrum: 65,536-point BH7 window * FFT * 10log10|X|^2, frames
    back to back (fftRate = fs/N -> skip 0), and
  * one VFO: RxVFO(61.44 MHz -> 240 kHz, bw 200 kHz, offset +2.5 MHz; plan_256 + 91-tap
    LPF) -> BroadcastFM mono (dev 100 kHz, 228-tap audio LPF) -> stereo_t,
with every rank's last 16 spectra gathered to rank 0 over RCCL each step (N > 1).
A step = one batch of B synthetic complex-float IQ samples resident in HBM
(uniform [-1, 1), SpeedTester distribution). Other configs: c2 (1M-point BH7 spectrum,
nz = 1e6, zero-padded), c3 (xlator + 256-tap FIR /8 + FM quadrature, fused), c4 (1024-channel
polyphase channelizer, 16384-tap prototype).

Launch: python bench.py [--gpus N --steps K --warmup W]; N > 1 under torch.distributed.run.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import sdrpp_amd  # noqa: E402
from sdrpp_amd import dsp  # noqa: E402
from sdrpp_amd.multistream import StreamShard  # noqa: E402

METRIC = "IQ Msamples/s through FFT+FIR+demod chain; % HBM roofline at 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md chip table (spec)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c5", choices=["c5", "c2", "c3", "c4"])
    ap.add_argument("--log2-batch", type=int, default=28, help="IQ samples per GPU per step = 2^k (c5/c3)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu", action="store_true")
    return ap.parse_args()


class C5:
    """FFT(64k BH7) spectra + RxVFO + BroadcastFM mono, one stream per GPU."""
    N = 65536
    FS = 61.44e6

    def __init__(self, B, shard, dev):
        self.B = (B // self.N) * self.N
        self.frames = self.B // self.N
        self.fft = dsp.FFTSpectrum(self.N, self.N, 6, device=dev)
        self.vfo = dsp.RxVFO(self.FS, 240000, 200000, shard.vfo_offset(), device=dev)
        self.wfm = dsp.BroadcastFM(100000, 240000, True, device=dev)
        self.spectra = torch.empty(self.frames * self.N, dtype=torch.float32, device="cuda")
        self.ifbuf = torch.empty(2 * (self.B // 256 + 64), dtype=torch.float32, device="cuda")
        self.audio = torch.empty(2 * (self.B // 256 + 64), dtype=torch.float32, device="cuda")
        self.bytes_per_sample = 8 + 4 + 8 / 256 + 8 / 256   # ~12.06 B
        self.kernel_bytes = 12.0 * self.B                   # spectrum pair: 8 B in + 4 B dB out per sample
        self.kernel_name = "spectrum (fft_passA + fft_passB, N=65536)"
        self.pieces = max(1, int(os.environ.get("BENCH_C5_PIECES", "1")))

    def run(self, x, s, timed_call):
        # the batch is pushed through the chain in `pieces` blocks, each through the spectrum and
        # then the VFO, as the reference's splitter feeds both paths block by block
        # (iq_frontend.cpp:15-52); pieces > 1 lets the VFO re-read a block the spectrum just read
        P = self.pieces
        fpp = self.frames // P
        m_if = m_au = 0
        for k in range(P):
            f0 = k * fpp
            nf = fpp if k < P - 1 else self.frames - f0
            xp = x.data_ptr() + 8 * f0 * self.N
            timed_call(lambda: self.fft.execute_dev(xp, self.N, nf, self.spectra.data_ptr() + 4 * f0 * self.N, s))
            m = self.vfo.process_dev(xp, nf * self.N, self.ifbuf.data_ptr() + 8 * m_if, s)
            a = self.wfm.process_dev(self.ifbuf.data_ptr() + 8 * m_if, m, self.audio.data_ptr() + 8 * m_au, s)
            m_if += m
            m_au += a

    def gather_src(self):
        return self.spectra[-16 * self.N:]


class C2:
    """1,048,576-point BH7 spectrum, fftRate 10 at 10 MS/s -> nz = 1e6, zero-padded."""
    N = 1 << 20
    NZ = 1000000

    def __init__(self, B, shard, dev):
        self.frames = max(1, B // self.NZ)
        self.B = self.frames * self.NZ
        self.fft = dsp.FFTSpectrum(self.N, self.NZ, 6, device=dev)
        self.spectra = torch.empty(self.frames * self.N, dtype=torch.float32, device="cuda")
        self.bytes_per_sample = 8 + 4 * self.N / self.NZ
        self.kernel_bytes = self.bytes_per_sample * self.B
        self.kernel_name = "spectrum (fft_passA + fft_passB, N=2^20, nz=1e6)"

    def dominant(self, x, s):
        self.fft.execute_dev(x.data_ptr(), self.NZ, self.frames, self.spectra.data_ptr(), s)

    def rest(self, x, s):
        pass

    def gather_src(self):
        return self.spectra[-2 * self.N:]


class C3:
    """FrequencyXlator(-1.5 MHz) -> 256-tap DecimatingFIR /8 -> Quadrature(100 kHz), fused kernel."""
    FS = 61.44e6

    def __init__(self, B, shard, dev):
        self.B = B
        taps = dsp.low_pass(3.0e6, 912000.0, self.FS)
        w = 2 * np.pi * (-1.5e6 / self.FS)
        self.ddc = dsp.DDCFM(w, taps, 8, 2 * np.pi * 100e3 / (self.FS / 8), device=dev)
        self.out = torch.empty(B // 8 + 64, dtype=torch.float32, device="cuda")
        self.bytes_per_sample = 8 + 4 / 8
        self.kernel_bytes = self.bytes_per_sample * B
        self.kernel_name = "fir_mfma_kernel<4,XL,QUAD> (xlator + 256-tap FIR /8 on f32 MFMA + quadrature)"

    def dominant(self, x, s):
        self.ddc.process_dev(x.data_ptr(), self.B, self.out.data_ptr(), s)

    def rest(self, x, s):
        pass

    def gather_src(self):
        return self.out[:65536]


class C4:
    """1024-channel critically sampled polyphase channelizer at 200 MS/s (prototype
    windowedSinc(16384, fs/(2M), fs, nuttall), 16 taps/branch), output [frame][channel]."""
    M = 1024

    def __init__(self, B, shard, dev):
        self.B = (B // self.M) * self.M
        taps = dsp.windowed_sinc(16 * self.M, np.pi / self.M)
        self.ch = dsp.PolyphaseChannelizer(self.M, taps, device=dev)
        self.out = torch.empty(2 * (self.B + self.M), dtype=torch.float32, device="cuda")
        self.bytes_per_sample = 16.0
        self.kernel_bytes = 16.0 * self.B
        self.kernel_name = "chan_kernel<1024> (16-tap branch FIRs + 1024-pt FFT per frame)"

    def dominant(self, x, s):
        self.ch.process_dev(x.data_ptr(), self.B, self.out.data_ptr(), s)

    def rest(self, x, s):
        pass

    def gather_src(self):
        return self.out[:2 * 16 * self.M]


def _run_generic(wl, x, s, timed_call):
    timed_call(lambda: wl.dominant(x, s))
    wl.rest(x, s)


def _timed(fn, blk, seconds):
    n, t0 = 0, time.perf_counter()
    while True:
        fn()
        n += blk
        dt = time.perf_counter() - t0
        if dt >= seconds:
            return n / dt / 1e6, n, dt


def cpu_baseline(config, seconds):
    """The reference CPU path for the config, time-bounded sample on the host (1 thread):
    the oracle's C port (VOLK-generic-equivalent fp32 loops) and, for the FFT configs, an
    optimized library FFT (torch.fft on CPU = pocketfft, 1 thread) -- the faster of the two
    is the baseline value (every speed-up claim uses the faster CPU number)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    rng = np.random.default_rng(0xACE1)
    torch.set_num_threads(1)
    if config == "c5":
        blk = 1 << 20
        x = (rng.uniform(-1, 1, blk) + 1j * rng.uniform(-1, 1, blk)).astype(np.complex64)
        chain = oracle.Chain(61.44e6, 65536, 2.5e6, precise=False)
        v, n, dt = _timed(lambda: chain.process(x), blk, seconds)
        return {"value": round(v, 3), "cores": 1, "kind": "port",
                "sample": f"oracle C port of the same C5 chain (64k BH7 spectra + RxVFO + WFM mono; fp32, VOLK-style "
                          f"rotator/dots), {n} samples in 1M blocks, {dt:.1f} s on 1 host core"}
    if config == "c2":
        N, nz = 1 << 20, 1000000
        x = (rng.uniform(-1, 1, nz) + 1j * rng.uniform(-1, 1, nz)).astype(np.complex64)
        w = oracle.create_window(6, nz)
        v1, n1, dt1 = _timed(lambda: oracle.fft_logmag(x, nz, N, w), nz, seconds / 2)
        xt, wt = torch.from_numpy(x), torch.from_numpy(w)

        def lib_fft():
            buf = torch.zeros(N, dtype=torch.complex64)
            buf[:nz] = xt * wt
            X = torch.fft.fft(buf)
            return 10.0 * torch.log10(X.real * X.real + X.imag * X.imag)
        v2, n2, dt2 = _timed(lib_fft, nz, seconds / 2)
        best = max(v1, v2)
        return {"value": round(best, 3), "cores": 1, "kind": "port",
                "sample": f"1M BH7 window*FFT*log-power of nz=1e6 frames, 1 thread: oracle C port {v1:.2f} MS/s "
                          f"({n1 // nz} frames, {dt1:.1f} s); torch.fft CPU (pocketfft) {v2:.2f} MS/s ({n2 // nz} frames, "
                          f"{dt2:.1f} s); value = the faster"}
    if config == "c3":
        blk = 1 << 20
        x = (rng.uniform(-1, 1, blk) + 1j * rng.uniform(-1, 1, blk)).astype(np.complex64)
        taps = oracle.low_pass(3.0e6, 912000.0, 61.44e6)
        d = oracle.DDCFM(2 * np.pi * (-1.5e6 / 61.44e6), taps, 8, 2 * np.pi * 100e3 / (61.44e6 / 8), precise=False)
        v, n, dt = _timed(lambda: d.process(x), blk, seconds)
        return {"value": round(v, 3), "cores": 1, "kind": "port",
                "sample": f"oracle C port: FrequencyXlator -> 256-tap DecimatingFIR /8 -> Quadrature (fp32, VOLK-style), "
                          f"{n} samples in 1M blocks, {dt:.1f} s on 1 host core"}
    if config == "c4":
        M, Q = 1024, 16
        h = oracle.windowed_sinc(Q * M, np.pi / M).reshape(Q, M)
        frames = 256
        x = (rng.uniform(-1, 1, (frames + Q) * M) + 1j * rng.uniform(-1, 1, (frames + Q) * M)).astype(np.complex64)
        xt = torch.from_numpy(x).reshape(frames + Q, M)
        ht = torch.from_numpy(h)

        def chan():   # same algorithm as the GPU (16-tap branch FIRs + M-point FFT per frame), vectorised
            u = torch.zeros((frames, M), dtype=torch.complex64)
            for q in range(Q):
                u += ht[q] * xt[q:q + frames]
            return torch.fft.fft(u, dim=1)
        v, n, dt = _timed(chan, frames * M, seconds)
        return {"value": round(v, 3), "cores": 1, "kind": "port",
                "sample": f"polyphase channelizer restated with torch CPU ops (branch FIR + pocketfft), 1 thread, "
                          f"{n} samples, {dt:.1f} s"}
    return None


def traffic_per_sample(config):
    """HBM bytes per input sample of the dominant launch group, from the committed rocprofv3
    PMC passes (FETCH_SIZE x2 gfx950 correction + WRITE_SIZE; tools/pmc_traffic.py)."""
    path = os.path.join(ROOT, "profiles", "r1", f"{config}_pmc_traffic.json")
    try:
        d = json.load(open(path))
        return float(d["bytes_per_sample"])
    except (OSError, KeyError, ValueError):
        return None


def main():
    a = parse()
    shard = StreamShard(backend="nccl")
    world, rank = shard.world, shard.rank
    if world == 1:
        torch.cuda.set_device(0)
    dev = torch.cuda.current_device()
    # one explicit non-default stream for every kernel of the step (libsdrgpu treats a NULL
    # stream as "the handle's own stream", which would split the chain over several queues)
    torch.cuda.set_stream(torch.cuda.Stream())
    B = 1 << a.log2_batch
    if a.config == "c2":
        B = 256 * 1000000
    wl = {"c5": C5, "c2": C2, "c3": C3, "c4": C4}[a.config](B, shard, dev)
    B = wl.B
    g = torch.Generator(device="cuda")
    g.manual_seed(shard.seed())
    x = (torch.rand(2 * B, device="cuda", generator=g) * 2 - 1).contiguous()   # complex_t interleaved
    stream = torch.cuda.current_stream()
    gather_bufs = None
    if world > 1 and rank == 0:
        gather_bufs = [torch.empty_like(wl.gather_src()) for _ in range(world)]
    gather_stage = torch.empty_like(wl.gather_src()) if world > 1 else None
    pending = [None]   # the in-flight gather (async work handle)

    ev = []
    # One stream for the whole step. Forking the spectrum and the VFO chain onto two streams
    # (the reference runs them on separate block threads, iq_frontend.cpp:49,115) was
    # measured twice: the step time does not change (2.95 vs 2.97 ms; with the MFMA VFO stage
    # 2.265 vs 2.261 ms; with the register-streaming VFO stage 1, 2.03-2.13 vs 2.01-2.04 ms)
    # but the spectrum's event/rocprof durations stretch by the overlap
    # (1.58 -> 1.89 ms), so the roofline numbers would stop describing the kernel.
    def step(timed):
        evs = []

        def timed_call(fn):   # HIP events around the dominant kernel's launches, on their stream
            if timed:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
            fn()
            if timed:
                e1.record(stream)
                evs.append((e0, e1))
        if hasattr(wl, "run"):
            wl.run(x, stream.cuda_stream, timed_call)
        else:
            _run_generic(wl, x, stream.cuda_stream, timed_call)
        if timed:
            ev.append(evs)
        if world > 1:
            # RCCL gather of this step's latest spectra, overlapped with the next step: the rows
            # are snapshotted into a staging buffer (the next step overwrites them) and the
            # collective runs on the process group's stream; it is waited on one step later
            if pending[0] is not None:
                pending[0].wait()
            gather_stage.copy_(wl.gather_src())
            pending[0], _ = shard.gather_spectra_async(gather_stage, gather_bufs)

    def drain():
        if pending[0] is not None:
            pending[0].wait()
            pending[0] = None

    for _ in range(a.warmup):
        step(False)
    drain()
    torch.cuda.synchronize()
    shard.barrier()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step(True)
    drain()   # the last step's gather is inside the timed region
    torch.cuda.synchronize()
    shard.barrier()
    elapsed = time.perf_counter() - t0
    kern_ms = sum(sum(e0.elapsed_time(e1) for e0, e1 in evs) for evs in ev) / max(len(ev), 1)
    elapsed, kern_ms = shard.max_over_ranks([elapsed, kern_ms], device="cuda")

    if rank == 0:
        total = world * B * a.steps
        value = total / elapsed / 1e6
        achieved = wl.kernel_bytes / (kern_ms * 1e-3) / 1e9
        tps = traffic_per_sample(a.config)
        out = {
            "metric": METRIC, "value": round(value, 3), "unit": "MS/s", "n_gpus": world, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": round(elapsed / a.steps * 1e3, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": "synthetic uniform[-1,1) complex IQ in HBM",
            "config": {"workload": {"c5": "C5 per-GPU slice: 64k BH7 FFT+log-mag (back-to-back) + RxVFO 61.44M->240k "
                                          "+ BroadcastFM mono; RCCL gather of 16 spectra/rank/step",
                                    "c2": "C2: 1M-point BH7 FFT + log-mag, nz=1e6 zero-padded",
                                    "c3": "C3: xlator + 256-tap FIR /8 + FM quadrature (fused)",
                                    "c4": "C4: 1024-channel polyphase channelizer (16384-tap prototype), 1 stream"}[a.config],
                       "samples_per_gpu_per_step": B, "parallelism": f"replica-streams x{world}",
                       "bytes_per_sample": round(wl.bytes_per_sample, 4)},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": round(tps * B) if tps else None,
                         "kernel": wl.kernel_name, "kernel_ms": round(kern_ms, 4)},
            "chain_hbm_GBs": round(wl.bytes_per_sample * value * 1e6 / world / 1e9, 1),
        }
        if world == 1 and not a.no_cpu:
            cb = cpu_baseline(a.config, a.cpu_seconds)
            if cb:
                out["cpu_baseline"] = {"value": cb["value"], "unit": "MS/s", "cores": cb["cores"], "kind": cb["kind"],
                                       "sample": cb["sample"]}
        print(json.dumps(out), flush=True)
    shard.close()


if __name__ == "__main__":
    main()
