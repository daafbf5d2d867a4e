"""HBM bytes per input sample of a launch group from rocprofv3 PMC passes over a whole bench run:
sum over every dispatch of the matching kernels of FETCH_SIZE x 2 (the gfx950 correction of
MI355X_MICROARCH.md's HBM section: FETCH_SIZE tallies 128-B requests at 64 B) + WRITE_SIZE (KB),
divided by the samples the run pushed through them.

  python tools/pmc_bytes_per_sample.py --config <c> <fetch_dir> <write_dir> <out.json>
      the group of tools/prof_summary.py GROUPS[c]; samples = (warmup + steps) x samples per step,
      read from the JSON line the profiled bench run printed (<fetch_dir>.json, run with
      --no-sub --no-ulp so every group dispatch belongs to the timed config)
  python tools/pmc_bytes_per_sample.py <fetch_dir> <write_dir> <substr>[,substr] <samples> <out.json> [algorithmic]"""
import csv
import json
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def total(d, match):
    s, names, n = 0.0, set(), 0
    for r in csv.DictReader(open(d + "/run_counter_collection.csv")):
        if match(r["Kernel_Name"]):
            s += float(r["Counter_Value"])
            names.add(r["Kernel_Name"])
            n += 1
    return s * 1024, sorted(names), n


def main():
    if sys.argv[1] == "--config":
        from prof_summary import GROUPS, line_of
        cfg, fdir, wdir, out = sys.argv[2:6]
        rx = re.compile(GROUPS[cfg])
        match = rx.search
        line = line_of(fdir.rstrip("/") + ".json")
        samples = float(line["config"]["samples_per_gpu_per_step"]) * (line["steps"] + line["warmup"])
        alg = line["roofline"]["algorithmic_bytes"] / line["config"]["samples_per_gpu_per_step"]
    else:
        fdir, wdir, keys, samples, out = sys.argv[1], sys.argv[2], sys.argv[3].split(","), float(sys.argv[4]), sys.argv[5]
        alg = float(sys.argv[6]) if len(sys.argv) > 6 else None
        match = lambda name: any(k in name for k in keys)   # noqa: E731
        cfg = None
    f, names, nf = total(fdir, match)
    w, _, nw = total(wdir, match)
    d = {"bytes_per_sample": (2 * f + w) / samples, "fetch_bytes_per_sample": 2 * f / samples,
         "write_bytes_per_sample": w / samples, "samples": samples, "dispatches": [nf, nw],
         "kernels": [n[:120] for n in names],
         "source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes ({fdir.rstrip('/').split('/')[-1]}, "
                   f"{wdir.rstrip('/').split('/')[-1]})"}
    if cfg:
        d["config"] = cfg
    if alg is not None:
        d["algorithmic_bytes_per_sample"] = alg
        d["traffic_over_algorithmic"] = round(d["bytes_per_sample"] / alg, 3)
    json.dump(d, open(out, "w"), indent=1)
    print(json.dumps(d, indent=1))


if __name__ == "__main__":
    main()
