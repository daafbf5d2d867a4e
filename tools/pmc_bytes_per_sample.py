"""HBM bytes per input sample of a launch group from rocprofv3 PMC passes over a whole bench run:
sum over every dispatch of the matching kernels of FETCH_SIZE x 2 (gfx950 correction, see
tools/pmc_traffic.py) + WRITE_SIZE (KB), divided by the samples the run pushed through them.
Usage: python tools/pmc_bytes_per_sample.py <fetch_dir> <write_dir> <substr>[,substr] <samples> <out.json> [algorithmic]"""
import csv
import json
import sys


def total(d, keys):
    s, names = 0.0, set()
    for r in csv.DictReader(open(d + "/run_counter_collection.csv")):
        if any(k in r["Kernel_Name"] for k in keys):
            s += float(r["Counter_Value"])
            names.add(r["Kernel_Name"])
    return s * 1024, sorted(names)


def main():
    fdir, wdir, keys, samples, out = sys.argv[1], sys.argv[2], sys.argv[3].split(","), float(sys.argv[4]), sys.argv[5]
    alg = float(sys.argv[6]) if len(sys.argv) > 6 else None
    f, names = total(fdir, keys)
    w, _ = total(wdir, keys)
    d = {"bytes_per_sample": (2 * f + w) / samples, "fetch_bytes_per_sample": 2 * f / samples,
         "write_bytes_per_sample": w / samples, "samples": samples, "kernels": [n[:120] for n in names],
         "source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes ({fdir.split('/')[-1]}, {wdir.split('/')[-1]})"}
    if alg is not None:
        d["algorithmic_bytes_per_sample"] = alg
    json.dump(d, open(out, "w"), indent=1)
    print(json.dumps(d, indent=1))


if __name__ == "__main__":
    main()
