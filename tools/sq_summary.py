"""Reduce tools/pmc_sets.sh SQ counter runs to per-kernel per-dispatch means and derived ratios.

  python tools/sq_summary.py gpurun_out/<TAG>   (reads <TAG>_1 .. <TAG>_5/run_counter_collection.csv)

Ratios (per dispatch, summed over its waves): VALU instructions per wave; busy fractions of the wave
cycles: SQ_ACTIVE_INST_VALU, SQ_ACTIVE_INST_ANY, SQ_WAIT_INST_ANY (waiting on a dependency or
waitcnt), SQ_WAIT_ANY, LDS busy and bank conflicts; the dispatch duration from the kernel trace."""
import csv
import glob
import json
import sys
from collections import defaultdict


def main():
    tag = sys.argv[1]
    acc = defaultdict(lambda: defaultdict(list))   # kernel -> counter -> per-dispatch values
    dur = defaultdict(list)
    for f in sorted(glob.glob(tag + "_[0-9]/run_counter_collection.csv")):
        per = defaultdict(lambda: defaultdict(float))
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")
            per[(k, r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
            per[(k, r["Dispatch_Id"])]["_ns"] = float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
        for (k, _), c in per.items():
            for name, v in c.items():
                if name == "_ns":
                    dur[k].append(v)
                else:
                    acc[k][name].append(v)
    out = {}
    for k, c in acc.items():
        m = {n: sum(v) / len(v) for n, v in c.items()}
        d = {"counters_mean_per_dispatch": {n: round(v, 1) for n, v in sorted(m.items())},
             "dispatch_us_mean": round(sum(dur[k]) / len(dur[k]) / 1e3, 2) if dur[k] else None}
        wc = m.get("SQ_WAVE_CYCLES")
        if wc:
            for n in ("SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY", "SQ_ACTIVE_INST_LDS",
                      "SQ_WAIT_INST_LDS", "SQ_INST_CYCLES_VMEM_RD", "SQ_ACTIVE_INST_SCA"):
                if n in m:
                    d[n + "_frac_of_wave_cycles"] = round(m[n] / wc, 3)
        if m.get("SQ_WAVES"):
            d["valu_insts_per_wave"] = round(m.get("SQ_INSTS_VALU", 0) / m["SQ_WAVES"], 1)
            d["vmem_rd_per_wave"] = round(m.get("SQ_INSTS_VMEM_RD", 0) / m["SQ_WAVES"], 1)
            d["lds_insts_per_wave"] = round(m.get("SQ_INSTS_LDS", 0) / m["SQ_WAVES"], 1)
        if m.get("SQ_INSTS_LDS"):
            d["lds_bank_conflict_cycles_per_lds_inst"] = round(m.get("SQ_LDS_BANK_CONFLICT", 0) / m["SQ_INSTS_LDS"], 3)
        out[k] = d
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
