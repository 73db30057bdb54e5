#!/usr/bin/env python
"""Effective clock per kernel NAME (every template instance apart): GRBM_GUI_ACTIVE / 8 / average duration, from a
rocprofv3 --pmc GRBM_GUI_ACTIVE pass and a --kernel-trace pass of the same program (MI355X_MICROARCH.md 'DVFS
give-back'; reads high below ~0.3 ms per dispatch).

usage: tools/pmc_clock_kernels.py CLOCK_DIR TRACE_DIR [name substring]
"""
import csv
import sys
from collections import defaultdict


def main():
    cdir, tdir = sys.argv[1:3]
    sub = sys.argv[3] if len(sys.argv) > 3 else ""
    act, n = defaultdict(float), defaultdict(int)
    for r in csv.DictReader(open(cdir + "/run_counter_collection.csv")):
        if r["Counter_Name"] == "GRBM_GUI_ACTIVE" and sub in r["Kernel_Name"]:
            act[r["Kernel_Name"]] += float(r["Counter_Value"])
            n[r["Kernel_Name"]] += 1
    dur, m = defaultdict(float), defaultdict(int)
    for r in csv.DictReader(open(tdir + "/run_kernel_trace.csv")):
        if sub in r["Kernel_Name"]:
            dur[r["Kernel_Name"]] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
            m[r["Kernel_Name"]] += 1
    print("%-60s %8s %10s %10s" % ("kernel", "calls", "avg ms", "clock GHz"))
    for k in sorted(act):
        if not m.get(k):
            continue
        a, d = act[k] / n[k], dur[k] / m[k]
        print("%-60s %8d %10.4f %10.3f" % (k[:60], m[k], d * 1e3, a / 8.0 / d / 1e9))


if __name__ == "__main__":
    main()
