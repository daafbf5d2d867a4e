"""HBM traffic per launch from rocprofv3 PMC passes (FETCH_SIZE and WRITE_SIZE in separate runs),
corrected as MI355X_MICROARCH.md prescribes: FETCH_SIZE reads half the bytes of a wide coalesced
stream on gfx950 (x2), WRITE_SIZE is exact for 16-B-per-lane streaming stores. Counters are in KB.
Usage: python tools/pmc_traffic.py <fetch_dir> <write_dir> <kernel-substring>[,<substring>...]"""
import collections
import csv
import json
import sys


def per_kernel(d):
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(d + "/run_counter_collection.csv")):
        acc[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}


def main():
    fdir, wdir, keys = sys.argv[1], sys.argv[2], sys.argv[3].split(",")
    f, w = per_kernel(fdir), per_kernel(wdir)
    out = {}
    total = 0.0
    for key in keys:
        names = [k for k in f if key in k]
        fk = sum(f[k] for k in names) * 1024 * 2
        wk = sum(w.get(k, 0.0) for k in names) * 1024
        out[key] = {"fetch_bytes_corrected": fk, "write_bytes": wk, "kernels": names}
        total += fk + wk
    out["total_bytes_per_launch_group"] = total
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
