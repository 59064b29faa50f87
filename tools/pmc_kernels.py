#!/usr/bin/env python3
"""Per-kernel summary of the PMC passes of tools/pmc_kernels.sh: counters summed over every
dispatch of each kernel, and the derived wave-cycle split, VALU issue and lane utilisation
(MI355X_MICROARCH.md: SQ_* cycle counters in quad-cycles, FETCH_SIZE doubled on gfx950).

    python tools/pmc_kernels.py gpurun_out/<run>/pmc [kernel-substring ...]
"""
import collections
import csv
import glob
import json
import os
import sys


def load(d):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    time_ns = collections.defaultdict(float)
    calls = collections.defaultdict(int)
    for f in glob.glob(os.path.join(d, "*", "run_counter_collection.csv")):
        seen = set()
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            per[k][r["Counter_Name"]] += float(r["Counter_Value"])
            if "sqa" in f and (r["Dispatch_Id"], k) not in seen:
                seen.add((r["Dispatch_Id"], k))
                calls[k] += 1
    for f in glob.glob(os.path.join(d, "sqa", "run_kernel_trace.csv")):
        for r in csv.DictReader(open(f)):
            time_ns[r["Kernel_Name"]] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    return per, time_ns, calls


def main():
    d = sys.argv[1]
    keys = sys.argv[2:]
    per, time_ns, calls = load(d)
    out = {}
    for k, c in per.items():
        if keys and not any(s in k for s in keys):
            continue
        rec = {"calls": calls.get(k, 0), "time_ms": time_ns.get(k, 0) / 1e6, "counters": dict(c)}
        if c.get("SQ_WAVE_CYCLES"):
            rec["wave_cycle_split"] = {n: c[n] / c["SQ_WAVE_CYCLES"] for n in
                                       ("SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY") if n in c}
        if c.get("SQ_ACTIVE_INST_VALU") and "SQ_THREAD_CYCLES_VALU" in c:
            rec["valu_lane_utilisation"] = c["SQ_THREAD_CYCLES_VALU"] / (c["SQ_ACTIVE_INST_VALU"] * 64.0)
        t = time_ns.get(k, 0) / 1e9
        if t > 0 and "SQ_INSTS_VALU" in c:
            rec["valu_issue_frac"] = c["SQ_INSTS_VALU"] * 64 / t / 78.64e12
        if "FETCH_SIZE" in c and t > 0:
            rec["hbm_GBs"] = (c["FETCH_SIZE"] * 2 + c.get("WRITE_SIZE", 0)) * 1024 / t / 1e9
        if "TCC_HIT_sum" in c and c.get("TCC_MISS_sum") is not None:
            tot = c["TCC_HIT_sum"] + c["TCC_MISS_sum"]
            rec["tcc_hit_rate"] = c["TCC_HIT_sum"] / tot if tot else None
        if c.get("SQ_ACTIVE_INST_LDS"):
            rec["lds_bank_conflict_per_active_lds"] = c.get("SQ_LDS_BANK_CONFLICT", 0) / c["SQ_ACTIVE_INST_LDS"]
        out[k] = rec
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
