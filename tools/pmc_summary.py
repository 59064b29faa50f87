#!/usr/bin/env python3
"""Summarise the PMC passes of tools/pmc.sh into a record of profiles/pmc_records.json.

HBM traffic per launch of the path-tracing kernel, corrected as MI355X_MICROARCH.md
§HBM prescribes: FETCH_SIZE and WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports
half the bytes of a wide coalesced read, so the read side is doubled (our reads are
scene records served from L2, so the read side is tiny either way).  The SQ counters
give the VALU issue picture (SQ_* wave counters are quad-cycle units; GRBM_GUI_ACTIVE is
summed over the 8 XCDs).

    python tools/pmc_summary.py gpurun_out/<run>/pmc <workload> profiles/pmc_records.json [--launches=K] [--calls=N]

The record carries the sha256 of the libmcpt.so that was profiled; bench.py uses a record only
for that exact build (records of other builds are dropped from the file on merge).
"""
import collections
import csv
import glob
import hashlib
import json
import os
import sys

KERNEL = "render_kernel<false"
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(REPO, "montecarlo-pathtracing_amd", "mcpt", "libmcpt.so")


def merge_record(recs, rec):
    """The records file after adding `rec`: records of other builds are dropped, and there is one
    record per (workload, schedule) of this build — a record of another schedule stays beside the
    new one (bench.py uses the one of the schedule its run settled on); a record of mixed
    schedules (None) replaces, and is replaced by, every record of its workload."""
    def same_slot(r):
        if r.get("workload") != rec.get("workload"):
            return False
        a, b = r.get("schedule"), rec.get("schedule")
        return a is None or b is None or a == b
    return [r for r in recs if r.get("lib_sha256") == rec["lib_sha256"] and not same_slot(r)] + [rec]

def load(d, launches=1, calls=1):
    """Counters of the timed step's path-tracing launches in each pass, summed: the LAST
    `launches` dispatches (earlier ones are warm-up, including AUTO's timing trials).  A render
    call spanning more pass segments than the segment-sum budget holds runs as several
    sub-launches (C5 under the old 1 GiB partial budget: 4; one since the 4 GiB default), and
    bench.py times the whole call, so its record sums them."""
    out = {}
    for f in glob.glob(os.path.join(d, "*", "run_counter_collection.csv")):
        per_dispatch = collections.defaultdict(dict)
        names = {}
        for r in csv.DictReader(open(f)):
            if KERNEL in r["Kernel_Name"]:
                k = int(r["Dispatch_Id"])
                per_dispatch[k][r["Counter_Name"]] = per_dispatch[k].get(r["Counter_Name"], 0.0) + \
                    float(r["Counter_Value"])
                names[k] = r["Kernel_Name"]
        if per_dispatch:
            # the last `calls` timed calls of `launches` dispatches each, averaged per call (the
            # work-item order's tail pieces make a call's instruction count vary by a few %)
            last = sorted(per_dispatch)[-launches * calls:]
            summed = collections.defaultdict(float)
            for k in last:
                for n, v in per_dispatch[k].items():
                    summed[n] += v / calls
            out.update(summed)
            out["_kernel"] = names[last[-1]]
    return out


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    launches, calls = 1, 1
    for a in sys.argv[1:]:
        if a.startswith("--launches="):
            launches = int(a.split("=", 1)[1])
        if a.startswith("--calls="):
            calls = int(a.split("=", 1)[1])
    d, workload, out = args[0], args[1], args[2]
    c = load(d, launches, calls)
    kernel = c.pop("_kernel", "mcpt::render_kernel<false, *>")
    fetch_b = c["FETCH_SIZE"] * 1024 * 2          # gfx950: FETCH_SIZE = half the bytes
    write_b = c["WRITE_SIZE"] * 1024
    rec = {
        "workload": workload,
        "lib_sha256": hashlib.sha256(open(LIB, "rb").read()).hexdigest(),
        "kernel": kernel,
        "source": "rocprofv3 --pmc passes of tools/pmc.sh (session %s)" % "/".join(d.rstrip("/").split("/")[-2:]),
        "launches_summed": launches,
        "calls_averaged": calls,
        "hbm_bytes_per_launch": fetch_b + write_b,
        "fetch_bytes_per_launch_corrected": fetch_b,
        "write_bytes_per_launch": write_b,
        "counters_per_launch": c,
    }
    # the schedule AUTO settled on in each counter pass (each pass is its own bench process): a
    # record combines passes only when they all ran the same one (bench.py uses a record only for
    # its own settled schedule)
    scheds = {}
    for f in sorted(glob.glob(os.path.join(d, "*.log"))):
        try:
            line = [ln for ln in open(f) if ln.startswith("{")][-1]
            sc = json.loads(line)["kernel_ms"]["schedule_rank0"]
            scheds[os.path.basename(f)[:-4]] = {"traversal": sc["traversal"], "seg_per_item": sc["seg_per_item"]}
        except (IndexError, KeyError, ValueError, OSError):
            pass
    distinct = {json.dumps(v, sort_keys=True) for v in scheds.values()}
    rec["schedule"] = json.loads(distinct.pop()) if len(distinct) == 1 else None
    if len(scheds) and rec["schedule"] is None:
        rec["schedules_by_pass"] = scheds
    if "SQ_INSTS_VALU" in c and "GRBM_GUI_ACTIVE" in c:
        cycles = c["GRBM_GUI_ACTIVE"] / 8.0                     # per-XCD clock cycles of the launch
        simds = 256 * 4
        rec["valu_issue_busy_frac"] = c["SQ_INSTS_VALU"] * 2.0 / (simds * cycles)   # ≥2 cycles per wave64 VALU
        rec["wave_cycle_split"] = {k: c[k] / c["SQ_WAVE_CYCLES"] for k in
                                   ("SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY") if k in c}
    if "SQ_THREAD_CYCLES_VALU" in c and c.get("SQ_ACTIVE_INST_VALU"):
        # active lanes per issued VALU instruction: rocprof's VALUUtilization expression,
        # 100 * SQ_THREAD_CYCLES_VALU / (SQ_ACTIVE_INST_VALU * 64)
        rec["valu_lane_utilisation"] = c["SQ_THREAD_CYCLES_VALU"] / (c["SQ_ACTIVE_INST_VALU"] * 64.0)
    if "SQ_INSTS_VALU_FMA_F32" in c:
        # fp32 flop upper bound (every lane active): FMA = 2, MUL / ADD = 1
        rec["f32_flop_per_launch_upper"] = 64.0 * (2 * c["SQ_INSTS_VALU_FMA_F32"] + c["SQ_INSTS_VALU_MUL_F32"] +
                                                   c["SQ_INSTS_VALU_ADD_F32"])
    if c.get("TCP_TCC_READ_REQ_sum"):
        # the gathers' memory hierarchy (tools/pmc.sh PMC_MEM=1 passes): L1 -> L2 read requests per
        # VMEM read instruction, their mean latency (cycles), the L2 hit rate, fabric read requests
        # by size and the share of them that went to DRAM (the rest: Infinity Cache hits)
        m = {"l1_to_l2_reads": c["TCP_TCC_READ_REQ_sum"],
             "l1_to_l2_latency_cycles": c.get("TCP_TCC_READ_REQ_LATENCY_sum", 0.0) / c["TCP_TCC_READ_REQ_sum"]}
        if c.get("SQ_INSTS_VMEM_RD"):
            m["l1_to_l2_reads_per_vmem_rd"] = c["TCP_TCC_READ_REQ_sum"] / c["SQ_INSTS_VMEM_RD"]
        if c.get("TCP_TOTAL_CACHE_ACCESSES_sum"):
            m["l1_accesses"] = c["TCP_TOTAL_CACHE_ACCESSES_sum"]
        if c.get("TCC_HIT_sum") is not None and c.get("TCC_MISS_sum") is not None:
            m["l2_hit_rate"] = c["TCC_HIT_sum"] / max(c["TCC_HIT_sum"] + c["TCC_MISS_sum"], 1.0)
        if c.get("TCC_EA0_RDREQ_sum"):
            m["fabric_reads"] = c["TCC_EA0_RDREQ_sum"]
            m["fabric_reads_dram_frac"] = c.get("TCC_EA0_RDREQ_DRAM_sum", 0.0) / c["TCC_EA0_RDREQ_sum"]
        if c.get("TCC_EA0_RDREQ_128B_sum") is not None:
            m["fabric_reads_128B"] = c["TCC_EA0_RDREQ_128B_sum"]
            m["fabric_reads_64B"] = c.get("TCC_EA0_RDREQ_64B_sum")
            m["fabric_read_bytes_by_size"] = 128.0 * c["TCC_EA0_RDREQ_128B_sum"] + 64.0 * c.get("TCC_EA0_RDREQ_64B_sum", 0.0)
        if c.get("TA_TA_BUSY_sum") and c.get("GRBM_GUI_ACTIVE"):
            m["ta_busy_frac"] = c["TA_TA_BUSY_sum"] / (256 * c["GRBM_GUI_ACTIVE"] / 8.0)
        rec["memory"] = m
    try:
        with open(out) as f:
            recs = json.load(f)["records"]
    except (OSError, ValueError, KeyError):
        recs = []
    recs = merge_record(recs, rec)
    with open(out, "w") as f:
        json.dump({"records": recs}, f, indent=1)
    print(json.dumps(rec, indent=1))


if __name__ == "__main__":
    main()
