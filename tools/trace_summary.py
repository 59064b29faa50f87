#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace CSV: per dispatch duration and resources.

    python tools/trace_summary.py gpurun_out/<run>/prof/run_kernel_trace.csv [title]
"""
import csv
import sys


def main():
    path = sys.argv[1]
    title = sys.argv[2] if len(sys.argv) > 2 else path
    rows = list(csv.DictReader(open(path)))
    print(title)
    print("kernel, duration_ms, VGPR, SGPR, scratch, LDS, grid")
    for r in rows:
        name = r["Kernel_Name"]
        if name.startswith("__amd") or "at::native" in name:
            continue
        ms = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        print(f'{name}, {ms:.3f}, {r["VGPR_Count"]}, {r["SGPR_Count"]}, {r["Scratch_Size"]}, '
              f'{r["LDS_Block_Size"]}, {r["Grid_Size_X"]}')


if __name__ == "__main__":
    main()
