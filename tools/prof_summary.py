"""Reduce one session's rocprofv3 kernel traces to per-config roofline figures that can be checked
against the bench line of the SAME process (tools/session.sh `prof` step).

For each config: the dominant launch group's dispatches (GROUPS below, the kernels the bench line's
`roofline.kernel` names) are split into the warm-up steps and the timed steps by dispatch order
(with --no-sub --no-ulp every group dispatch of the run belongs to run_config: (warmup + steps) x
dispatches-per-step of them). Reported per step:
  * rocprof_ms_all    -- the rocprofv3 --stats view: every dispatch, warm-up included, / (warmup+steps)
  * rocprof_ms_timed  -- the timed steps only (what the bench's HIP events bracket)
  * event_ms          -- the bench line's roofline.kernel_ms from the same process
  * frac_*            -- algorithmic bytes / time / 8 TB/s for each of the three
Usage: python tools/prof_summary.py <gpurun_out dir> <TAG> <config> [config ...]
       python tools/prof_summary.py --combined <gpurun_out dir> <TAG>   (session step benchprof)"""
import csv
import json
import os
import re
import sys

PEAK = 8000.0
GROUPS = {
    "c5": r"fft_vfo_kernel<true|fft_passA_kernel<256, 32>|fft_merged_kernel<256, 32, 256, 32|fft_passB_kernel<256, 32, true>"
          r"|fft_1p_kernel<true, true|fft_1p_zoom_kernel",
    "c2": r"fft_passA_1m_kernel|fft_passB_1m_kernel",
    "c3": r"fir_mfma_kernel<4, true, true",
    "c4": r"chan2_kernel<1024, false>",
    "c4g": r"chan2_kernel<1024, true>",
}


def line_of(path):
    for ln in reversed(open(path).read().strip().splitlines()):
        if ln.startswith("{"):
            return json.loads(ln)
    raise ValueError(f"no JSON line in {path}")


def summarise(out, tag, cfg, pattern=None):
    d = os.path.join(out, f"{tag}_prof_{cfg}")
    trace = os.path.join(d, "run_kernel_trace.csv")
    line = line_of(os.path.join(out, f"{tag}_prof_{cfg}.json"))
    rx = re.compile(pattern or GROUPS[cfg])
    rows = [r for r in csv.DictReader(open(trace)) if rx.search(r["Kernel_Name"])]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    return reduce_rows(cfg, rows, line)


BENCH_ORDER = ["c5", "c2", "c3", "c4", "c4g"]   # bench.py main(): the head config, then the others in this order


def summarise_combined(out, tag):
    """`benchprof` step: ONE default bench process under rocprofv3; every config's group dispatches are
    taken from the window between its first dispatch and the next config's first dispatch (the live
    ulp report, the fp64-mode cost and the per-call runs come after all configs)."""
    trace = os.path.join(out, f"{tag}_benchprof", "run_kernel_trace.csv")
    line = line_of(os.path.join(out, f"{tag}_bench.json"))
    allrows = sorted(csv.DictReader(open(trace)), key=lambda r: int(r["Start_Timestamp"]))
    order = [line.get("config_key", "c5")] + [c for c in BENCH_ORDER if c in line.get("configs", {})]
    first = {}
    for c in order:
        rx = re.compile(GROUPS[c])
        ts = [int(r["Start_Timestamp"]) for r in allrows if rx.search(r["Kernel_Name"])]
        first[c] = ts[0] if ts else None
    res = {}
    for i, c in enumerate(order):
        rx = re.compile(GROUPS[c])
        lo = first[c]
        hi = next((first[n] for n in order[i + 1:] if first[n] is not None and first[n] > lo), None) if lo else None
        rows = [r for r in allrows if rx.search(r["Kernel_Name"]) and int(r["Start_Timestamp"]) >= (lo or 0)
                and (hi is None or int(r["Start_Timestamp"]) < hi)]
        sub = line if i == 0 else dict(line["configs"][c], steps=line["steps"], warmup=line["warmup"])
        try:
            res[c] = reduce_rows(c, rows, sub)
        except (ValueError, KeyError) as e:
            res[c] = {"error": str(e)}
    return res


def reduce_rows(cfg, rows, line):
    rx = re.compile(GROUPS[cfg])
    steps, warm = line["steps"], line["warmup"]
    n = len(rows)
    if n == 0:
        raise ValueError(f"{cfg}: no dispatch matches {rx.pattern}")
    if n % (steps + warm):
        raise ValueError(f"{cfg}: {n} group dispatches is not a multiple of {steps + warm} steps")
    dps = n // (steps + warm)
    dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6 for r in rows]   # ms
    timed = dur[warm * dps:]
    # per timed step: the group's span from its first start to its last end (launch gaps included,
    # as the events see it) next to the sum of the kernel durations
    spans = []
    for k in range(steps):
        grp = rows[(warm + k) * dps:(warm + k + 1) * dps]
        spans.append((int(grp[-1]["End_Timestamp"]) - int(grp[0]["Start_Timestamp"])) * 1e-6)
    alg = line["roofline"]["algorithmic_bytes"]
    ms_all = sum(dur) / (steps + warm)
    ms_timed = sum(timed) / steps
    span = sum(spans) / steps
    ev = line["roofline"]["kernel_ms"]

    def frac(ms):
        return round(alg / (ms * 1e-3) / 1e9 / PEAK, 4)
    return {"config": cfg, "kernels": sorted({r["Kernel_Name"][:110] for r in rows}), "dispatches_per_step": dps,
            "steps": steps, "warmup": warm, "algorithmic_bytes": alg,
            "rocprof_ms_all": round(ms_all, 4), "rocprof_ms_timed": round(ms_timed, 4),
            "rocprof_span_ms_timed": round(span, 4), "event_ms": ev,
            "frac_rocprof_all": frac(ms_all), "frac_rocprof_timed": frac(ms_timed), "frac_event": frac(ev),
            "line_frac": line["roofline"]["frac"], "event_vs_rocprof_timed": round(ev / ms_timed, 4),
            "min_dispatch_ms": round(min(timed), 4), "max_dispatch_ms": round(max(timed), 4),
            "line_value_MSps": line["value"], "line_ms_per_step": line["ms_per_step"]}


def main():
    if sys.argv[1] == "--combined":
        print(json.dumps(summarise_combined(sys.argv[2], sys.argv[3]), indent=1))
        return
    out, tag, cfgs = sys.argv[1], sys.argv[2], sys.argv[3:]
    res = {}
    for c in cfgs:
        try:
            res[c] = summarise(out, tag, c)
        except (OSError, ValueError, KeyError) as e:
            res[c] = {"error": str(e)}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
