"""CPU baseline for bench.py (TEST INFRASTRUCTURE: only bench.py's cpu_baseline leg runs this).

The reference's CPU dsp:: path cannot run on the GPU box (no VOLK/FFTW there, and the reference
tree does not travel), so the baseline is the oracle's C restatement of the same chain, built on
the host that runs it with -O3 -march=native (no fast-math; vectorised VOLK-class dot products),
plus the FFTW-class library FFT the
host has (pocketfft through scipy.fft, single precision, one worker) for the spectrum legs.
For every config the faster CPU variant is the reported value.

Harness: SpeedTester-style (core/src/dsp/bench/speed_tester.h:31-56): 1,000,000-sample blocks of
uniform [-1, 1) IQ pushed through the chain for a bounded time; MS/s = samples / duration.
  * 1 core: one stream on one thread (the reference's model: one worker thread per block, one
    single-threaded FFT);
  * all cores: one independent stream per core (separate processes, each pinned to a core),
    aggregate = sum of the per-stream rates (they run concurrently).

Usage (worker): python oracle/cpu_baseline.py --config c5 --seconds 8 --seed 3 [--cpu K]
prints one JSON line {"samples": n, "seconds": t, "variant": "..."}.
"""
import argparse
import json
import os
import subprocess
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
BLK = 1000000        # SpeedTester block (speed_tester.h:37: 1e6 samples)


def native_oracle():
    """Build the oracle with -march=native for the host this runs on (outside the repo tree)."""
    out_dir = os.path.join(os.environ.get("TMPDIR", "/tmp"), "sdrgpu_cpu_baseline")
    os.makedirs(out_dir, exist_ok=True)
    so = os.path.join(out_dir, "libsdr_oracle_native.so")
    src = os.path.join(HERE, "sdr_oracle.c")
    fast = os.path.join(HERE, "cpu_fast.c")
    if not os.path.exists(so) or os.path.getmtime(so) < max(os.path.getmtime(src), os.path.getmtime(fast)):
        # -ffp-contract=fast: the dot products use FMA like VOLK's *_avx2_fma kernels (this copy
        # is only timed; the in-tree checker build keeps -ffp-contract=off)
        cmd = ["gcc", "-O3", "-march=native", "-ffp-contract=fast", "-fno-fast-math", "-fPIC", "-shared",
               "-o", so, src, fast, "-lm"]
        try:
            subprocess.check_call(cmd, cwd=HERE, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
        except (OSError, subprocess.CalledProcessError):
            return None
    return so


def cgroup_cpu_quota():
    """CPUs this process may use per the cgroup v2 CPU controller (cpu.max "quota period"), or None
    when unlimited / not readable. The GPU box grants 16 (1600000 / 100000) of its 256 CPUs."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, p = f.read().split()[:2]
        if q == "max":
            return None
        return max(1, int(int(q) // int(p)))
    except (OSError, ValueError):
        return None


def core_peak_gflops():
    """fp32 FMA peak of one core: 2 FMA pipes x 16 lanes (AVX-512) x 2 flop x the max clock (lscpu
    'CPU max MHz', else /proc/cpuinfo 'cpu MHz'). Zen 5 (EPYC 9575F): 2 x 512-bit FMA per cycle."""
    mhz = None
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for line in out.splitlines():
            if line.startswith("CPU max MHz"):
                mhz = float(line.split(":", 1)[1])
    except (OSError, ValueError, subprocess.SubprocessError):
        pass
    if mhz is None:
        try:
            with open("/proc/cpuinfo") as f:
                for line in f:
                    if line.startswith("cpu MHz"):
                        mhz = float(line.split(":", 1)[1])
                        break
        except (OSError, ValueError):
            return None, None
    return (2 * 16 * 2 * mhz / 1e3 if mhz else None), mhz


def host_info():
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count()
    peak, mhz = core_peak_gflops()
    return {"nproc": os.cpu_count(), "affinity": aff, "model": model, "cgroup_cpu_quota": cgroup_cpu_quota(),
            "core_max_mhz": mhz, "core_fp32_peak_gflops": peak}


# DDR channels x MT/s per socket of the host CPUs the GPU boxes carry (vendor specifications): the
# DRAM ceiling of a whole host is sockets x channels x MT/s x 8 B
DRAM_PER_SOCKET = {"AMD EPYC 9575F": (12, 6400)}


def host_sockets():
    try:
        ids = set()
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("physical id"):
                    ids.add(line.split(":", 1)[1].strip())
        return max(1, len(ids))
    except OSError:
        return None


def host_dram_peak_gbs(model, sockets):
    for k, (ch, mts) in DRAM_PER_SOCKET.items():
        if model and k in model and sockets:
            return sockets * ch * mts * 8 / 1000.0
    return None


def _read(path):
    try:
        with open(path) as f:
            return f.read().strip()
    except OSError:
        return None


def cpu_topology(cpus):
    """{cpu: (socket, L3 domain, physical core)} from sysfs (L3 domain = index3 shared_cpu_list,
    core = thread_siblings_list); None where sysfs does not say."""
    topo = {}
    for c in cpus:
        base = f"/sys/devices/system/cpu/cpu{c}"
        topo[c] = (_read(f"{base}/topology/physical_package_id"), _read(f"{base}/cache/index3/shared_cpu_list"),
                   _read(f"{base}/topology/thread_siblings_list"))
    return topo


def placements(cpus, n):
    """Two placements of n single-threaded streams over the affinity CPUs:
      packed -- the first n CPUs in order (round 4's placement: on a 2 x 64-core EPYC the first 16
                CPUs are two 8-core CCDs of socket 0, sharing two L3s and one socket's DRAM channels);
      spread -- one stream per L3 domain, the domains dealt alternately from each socket, one CPU per
                physical core, before any domain takes a second stream.
    Returns ({name: [cpu]}, {"sockets": s, "l3_domains": d})."""
    cpus = sorted(cpus)
    topo = cpu_topology(cpus)
    doms = {}
    for c in cpus:
        sock, l3, core = topo[c]
        doms.setdefault((sock, l3 if l3 is not None else f"cpu{c}"), {}).setdefault(core or f"c{c}", []).append(c)
    by_sock = {}
    for (sock, l3), cores in sorted(doms.items(), key=lambda kv: min(min(v) for v in kv[1].values())):
        by_sock.setdefault(sock, []).append([sorted(v)[0] for v in sorted(cores.values())] +
                                            [c for v in sorted(cores.values()) for c in sorted(v)[1:]])
    order = []   # domains alternating sockets
    socks = list(by_sock)
    for i in range(max(len(v) for v in by_sock.values())):
        for s in socks:
            if i < len(by_sock[s]):
                order.append(by_sock[s][i])
    spread, k = [], 0
    while len(spread) < min(n, len(cpus)):
        for d in order:
            if k < len(d) and len(spread) < n:
                spread.append(d[k])
        k += 1
    return {"packed": cpus[:n], "spread": spread}, {"sockets": len(by_sock), "l3_domains": len(doms)}


def _stream_worker(seconds):
    """memcpy bandwidth of one process over 256 MB buffers (read + write bytes), GB/s"""
    import numpy as np
    a = np.ones(64 << 20, dtype=np.float32)
    b = np.empty_like(a)
    np.copyto(b, a)
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        np.copyto(b, a)
        n += 1
    return 2 * a.nbytes * n / (time.perf_counter() - t0) / 1e9


def stream_bw(ncores, cores, seconds=2.0):
    """Aggregate memcpy bandwidth of `ncores` concurrent single-threaded processes (one per core of
    the lease): what the lease's CPUs move to and from DRAM."""
    procs = [subprocess.Popen([sys.executable, os.path.abspath(__file__), "--stream", str(seconds), "--cpu", str(cores[k])],
                              stdout=subprocess.PIPE, stderr=subprocess.DEVNULL, text=True) for k in range(ncores)]
    tot = 0.0
    for p in procs:
        tot += float(p.communicate()[0].strip().splitlines()[-1])
    return tot


def _iq(rng, n):
    import numpy as np
    return (rng.uniform(-1, 1, n) + 1j * rng.uniform(-1, 1, n)).astype(np.complex64)


def _timed(fn, blk, seconds):
    n, t0 = 0, time.perf_counter()
    while True:
        fn()
        n += blk
        dt = time.perf_counter() - t0
        if dt >= seconds:
            return n, dt


def workloads(config, seed):
    """{variant: (step_fn, samples_per_step)} for the config's CPU restatements."""
    import numpy as np
    sys.path.insert(0, HERE)
    import oracle
    import scipy.fft
    rng = np.random.default_rng(0xACE1 + seed)
    out = {}
    if config == "c5":
        # 64k BH7 spectra back to back (fftRate = fs / N) + RxVFO(61.44 M -> 240 k) + WFM mono
        N = 65536
        blk = 16 * N                                      # ~1e6 samples, whole frames
        x = _iq(rng, blk)
        w = oracle.create_window(6, N)
        chain = oracle.Chain(61.44e6, N, 2.5e6, precise=False)
        out["oracle C chain (radix-2 FFT)"] = (lambda: chain.process(x), blk)
        vfo = oracle.RxVFO(61.44e6, 240000, 200000, 2.5e6, precise=False)
        wfm = oracle.BroadcastFM(100000, 240000, True, precise=False)
        frames = x.reshape(-1, N)

        def pocket():
            X = scipy.fft.fft(frames * w, axis=1, workers=1)
            p = X.real * X.real + X.imag * X.imag
            db = 10.0 * np.log10(p)
            wfm.process(vfo.process(x))
            return db
        out["pocketfft spectra + oracle C VFO/WFM"] = (pocket, blk)
    elif config == "c2":
        N, nz = 1 << 20, 1000000
        x = _iq(rng, nz)
        w = oracle.create_window(6, nz)
        out["oracle C radix-2 FFT"] = (lambda: oracle.fft_logmag(x, nz, N, w), nz)
        buf = np.zeros(N, dtype=np.complex64)

        def pocket():
            buf[:nz] = x * w
            X = scipy.fft.fft(buf, workers=1)
            return 10.0 * np.log10(X.real * X.real + X.imag * X.imag)
        out["pocketfft"] = (pocket, nz)
    elif config == "c3":
        x = _iq(rng, BLK)
        taps = oracle.low_pass(3.0e6, 912000.0, 61.44e6)
        d = oracle.DDCFM(2 * np.pi * (-1.5e6 / 61.44e6), taps, 8, 2 * np.pi * 100e3 / (61.44e6 / 8), precise=False)
        out["oracle C xlator + 256-tap FIR/8 + quadrature"] = (lambda: d.process(x), BLK)
    elif config == "c4":
        M, Q = 1024, 16
        h = oracle.windowed_sinc(Q * M, np.pi / M).reshape(Q, M).astype(np.float32)
        frames = 1024
        x = _iq(rng, (frames + Q) * M).reshape(frames + Q, M)

        def chan():    # 16-tap branch FIRs + M-point FFT per output frame (the GPU's algorithm)
            u = np.zeros((frames, M), dtype=np.complex64)
            for q in range(Q):
                u += h[q] * x[q:q + frames]
            return scipy.fft.fft(u, axis=1, workers=1)
        out["numpy branch FIR + pocketfft"] = (chan, frames * M)
        FB = 64    # frames per block: the block's FIR output (512 KB) is FFT'd while it is in L2
        ub = np.empty((FB, M), dtype=np.complex64)

        def chan_c():  # the branch FIRs in the oracle's C (cpu_fast.c: 8 complex lanes per vector)
            for f0 in range(0, frames, FB):
                oracle.chan_branch_fir(x[f0:f0 + FB + Q - 1], h, FB, ub)
                scipy.fft.fft(ub, axis=1, workers=1, overwrite_x=True)
        out["oracle C branch FIR + pocketfft"] = (chan_c, frames * M)
    return out


def worker(config, seconds, seed, variant=None):
    res = {}
    for name, (fn, blk) in workloads(config, seed).items():
        if variant is not None and name != variant:
            continue
        fn()   # warm
        n, dt = _timed(fn, blk, seconds)
        res[name] = {"samples": n, "seconds": dt}
    return res


def _spawn(config, seconds, seed, variant, cpu, lib):
    env = dict(os.environ)
    for k in ("OMP_NUM_THREADS", "OPENBLAS_NUM_THREADS", "MKL_NUM_THREADS"):
        env[k] = "1"
    if lib:
        env["ORACLE_LIB_PATH"] = lib
    cmd = [sys.executable, os.path.abspath(__file__), "--config", config, "--seconds", str(seconds), "--seed", str(seed),
           "--variant", variant]
    if cpu is not None:
        cmd += ["--cpu", str(cpu)]
    return subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.DEVNULL, text=True)


# fp32 flop per input sample of each config's CPU chain (for the FMA-peak fraction of the 1-core leg)
FLOP_PER_SAMPLE = {
    "c3": 2 * 256 * 2 / 8 + 6 + 40 / 8,   # 256 complex x real MACs per output / D, rotator, quadrature
}


_BW = None   # the lease's memcpy bandwidth, measured once per process


def measure(config, seconds=8.0, max_cores=None):
    """1-core figure of every variant (in turn), then the fastest variant on all cores this process
    may use: the cgroup CPU quota (16 on the GPU box), capped by the affinity mask."""
    lib = native_oracle()
    info = host_info()
    cores_avail = sorted(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else list(range(os.cpu_count()))
    quota = info["cgroup_cpu_quota"]
    ncores = len(cores_avail) if quota is None else min(quota, len(cores_avail))
    if max_cores is not None:
        ncores = min(ncores, max_cores)
    ncores = max(1, ncores)
    # the all-core leg's placements: the quota limits CPU time, not where the
    # streams run, so the streams are also spread one per L3 domain over both sockets
    place, topo = placements(cores_avail, ncores)
    # the 1-core leg runs on the spread placement's first CPU, not CPU 0 (CPU 0 sits
    # beside the bench parent and the system's own work, and measured 0.65x the spread streams' mean)
    cpu1 = place["spread"][0] if place["spread"] else cores_avail[0]
    one = {}
    for name in workloads_names(config):
        p = _spawn(config, seconds, 0, name, cpu1, lib)
        r = json.loads(p.communicate()[0].strip().splitlines()[-1])[name]
        one[name] = r["samples"] / r["seconds"] / 1e6
    best = max(one, key=one.get)
    agg, per_min, per_mean = {}, {}, {}
    for name, cpus in place.items():
        procs = [_spawn(config, seconds, k + 1, best, cpus[k], lib) for k in range(len(cpus))]
        rates = []
        for p in procs:
            r = json.loads(p.communicate()[0].strip().splitlines()[-1])[best]
            rates.append(r["samples"] / r["seconds"] / 1e6)
        agg[name], per_min[name], per_mean[name] = sum(rates), min(rates), sum(rates) / len(rates)
    faster = max(agg, key=agg.get)
    # one core's rate: the better of the 1-core run and the placements' per-stream means (a core of
    # the all-core leg cannot be slower alone than it was beside the others), so that every
    # aggregate / 1-core ratio stays <= the stream count and the whole-host bound built on it is not
    # understated
    one_run = one[best]
    one_core = max(one_run, *per_mean.values())
    global _BW
    if _BW is None:
        _BW = stream_bw(ncores, place["spread"])
    info["sockets"] = host_sockets()
    info["dram_peak_GBs"] = host_dram_peak_gbs(info["model"], info["sockets"])
    info["lease_memcpy_GBs"] = round(_BW, 1)
    info["placement"] = {"cpus_" + k: v for k, v in place.items()}
    info["placement"].update(topo)
    r = {"value_1core": one_core, "value_1core_run": one_run, "value_1core_cpu": cpu1,
         "value_1core_spread_mean": max(per_mean.values()), "variant": best, "variants_1core": one,
         "value_all_cores": agg[faster],
         "value_all_cores_packed": agg["packed"], "value_all_cores_spread": agg["spread"], "placement": faster,
         "cores_all": ncores, "cores_source": "cgroup cpu.max quota" if quota is not None else "affinity mask",
         "per_stream_min": per_min[faster], "host": info,
         "build": "oracle C -O3 -march=native (host-built)" if lib else "oracle C (in-tree build)"}
    if config in FLOP_PER_SAMPLE and info.get("core_fp32_peak_gflops"):
        gf = one_core * 1e6 * FLOP_PER_SAMPLE[config] / 1e9
        r["gflops_1core"] = round(gf, 1)
        r["fma_peak_frac_1core"] = round(gf / info["core_fp32_peak_gflops"], 3)
    return r


def workloads_names(config):
    return {"c5": ["oracle C chain (radix-2 FFT)", "pocketfft spectra + oracle C VFO/WFM"],
            "c2": ["oracle C radix-2 FFT", "pocketfft"],
            "c3": ["oracle C xlator + 256-tap FIR/8 + quadrature"],
            "c4": ["numpy branch FIR + pocketfft", "oracle C branch FIR + pocketfft"]}[config]


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default=None)
    ap.add_argument("--seconds", type=float, default=8.0)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--variant", default=None)
    ap.add_argument("--cpu", type=int, default=None)
    ap.add_argument("--measure", action="store_true", help="run the 1-core + all-core measurement")
    ap.add_argument("--stream", type=float, default=None, help="memcpy bandwidth worker (seconds)")
    a = ap.parse_args()
    if a.stream is not None:
        if a.cpu is not None and hasattr(os, "sched_setaffinity"):
            os.sched_setaffinity(0, {a.cpu})
        print(_stream_worker(a.stream))
        sys.exit(0)
    if a.measure:
        print(json.dumps(measure(a.config, a.seconds)))
        sys.exit(0)
    if a.cpu is not None and hasattr(os, "sched_setaffinity"):
        os.sched_setaffinity(0, {a.cpu})
    print(json.dumps(worker(a.config, a.seconds, a.seed, a.variant)))
