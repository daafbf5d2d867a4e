"""C3 MFMA FIR issue picture from tools/pmc_r2b.sh counter CSVs (one pass per set):
python tools/sq_summary.py <dir with c3_mfma_counters.csv, c3_issue_counters.csv, c3_mfma_kernel_trace.csv>

SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* count quad-cycles, SQ_VALU_MFMA_BUSY_CYCLES cycles
per SIMD (summed), GRBM_GUI_ACTIVE cycles summed over the 8 XCDs (MI355X_MICROARCH.md)."""
import csv, json, sys

d = sys.argv[1]
m = {}
for f in ("c3_mfma_counters.csv", "c3_issue_counters.csv"):
    acc = {}
    for r in csv.DictReader(open(f"{d}/{f}")):
        if "fir_mfma_kernel" in r["Kernel_Name"]:
            acc.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    for k, v in acc.items():
        m.setdefault(k, sum(v) / len(v))
dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
       for r in csv.DictReader(open(f"{d}/c3_mfma_kernel_trace.csv")) if "fir_mfma_kernel" in r["Kernel_Name"]]
t = sum(dur) / len(dur)
SIMDS = 1024
cyc = m["GRBM_GUI_ACTIVE"] / 8
w = m["SQ_WAVE_CYCLES"]
out = {
    "kernel": "fir_mfma_kernel<4, XL, QUAD> (C3)", "kernel_us_profiled": round(t * 1e6, 1),
    "clock_ghz_effective": round(cyc / t / 1e9, 3),
    "mfma_busy_frac": round(m["SQ_VALU_MFMA_BUSY_CYCLES"] / SIMDS / cyc, 3),
    "mfma_cycles_per_instruction": round(m["SQ_VALU_MFMA_BUSY_CYCLES"] / m["SQ_INSTS_MFMA"], 2),
    "waves_per_simd_avg": round(w * 4 / SIMDS / cyc, 2),
    "wave_cycle_split": {k: round(m[k] / w, 3) for k in ("SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY")},
    "active_split": {k: round(m[k] / w, 3) for k in ("SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS", "SQ_WAIT_INST_LDS")},
    "lds_bank_conflict_per_lds_active": round(m["SQ_LDS_BANK_CONFLICT"] / m["SQ_ACTIVE_INST_LDS"], 2),
    "counters_avg_per_dispatch": {k: round(v) for k, v in sorted(m.items())},
}
print(json.dumps(out, indent=1))
