"""Per-kernel averages of rocprofv3 --pmc SQ_* / GRBM_* passes (run_counter_collection.csv), with the
derived shares used in DESIGN.md: wave-time split (issuing / issue-stalled / waiting), LDS-array and VALU
busy fractions per CU / SIMD against the kernel's duration in shader cycles (GRBM_GUI_ACTIVE / XCDs).
Usage: python tools/sq_summary.py OUT.json KERNEL_PREFIX DIR [DIR ...]"""
import collections
import csv
import json
import os
import sys

CUS, SIMDS, XCDS = 256, 1024, 8


def main():
    out, prefix, dirs = sys.argv[1], sys.argv[2], sys.argv[3:]
    tot = collections.defaultdict(float)
    disp = collections.defaultdict(set)
    for d in dirs:
        for r in csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))):
            if not r["Kernel_Name"].startswith(prefix):
                continue
            tot[r["Counter_Name"]] += float(r["Counter_Value"])
            disp[r["Counter_Name"]].add((d, r["Dispatch_Id"]))
    avg = {k: tot[k] / len(disp[k]) for k in tot}
    res = {"kernel_prefix": prefix, "sources": dirs, "per_dispatch": avg,
           "dispatches": {k: len(v) for k, v in disp.items()}}
    if "SQ_WAVE_CYCLES" in avg:
        w = avg["SQ_WAVE_CYCLES"]
        res["wave_time_split"] = {k: avg[k] / w for k in ("SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY",
                                                           "SQ_WAIT_INST_LDS") if k in avg}
    if "GRBM_GUI_ACTIVE" in avg:
        cyc = avg["GRBM_GUI_ACTIVE"] / XCDS
        res["kernel_cycles_per_xcd"] = cyc
        if "SQ_LDS_IDX_ACTIVE" in avg:
            res["lds_array_busy_per_cu"] = avg["SQ_LDS_IDX_ACTIVE"] / CUS / cyc
        if "SQ_LDS_BANK_CONFLICT" in avg and "SQ_LDS_IDX_ACTIVE" in avg:
            res["lds_bank_conflict_share"] = avg["SQ_LDS_BANK_CONFLICT"] / avg["SQ_LDS_IDX_ACTIVE"]
        if "SQ_INSTS_VALU" in avg:   # a wave64 VALU instruction occupies a 16-lane SIMD for 4 cycles
            res["valu_busy_per_simd"] = avg["SQ_INSTS_VALU"] * 4 / SIMDS / cyc
        if "SQ_WAVES" in avg:
            res["waves"] = avg["SQ_WAVES"]
            res["valu_insts_per_wave"] = avg.get("SQ_INSTS_VALU", 0) / avg["SQ_WAVES"]
            res["lds_insts_per_wave"] = avg.get("SQ_INSTS_LDS", 0) / avg["SQ_WAVES"]
    json.dump(res, open(out, "w"), indent=1, sort_keys=True)
    print(json.dumps({k: v for k, v in res.items() if k not in ("per_dispatch", "sources", "dispatches")},
                     indent=1))


if __name__ == "__main__":
    main()
