#!/usr/bin/env python
"""Effective clock per kernel class under load: GRBM_GUI_ACTIVE (summed over the 8 XCDs by rocprofv3) / 8 /
the class's average kernel duration from the kernel-trace pass (MI355X_MICROARCH.md 'DVFS give-back').
The quotient reads high on dispatches shorter than ~0.3 ms (6.8 GHz on the 9 us split_x3): only classes whose average
dispatch is at least MIN_MS are printed (the upconv classes, ~0.55 ms).

usage: tools/pmc_clock.py CLOCK_DIR TRACE_DIR
"""
import csv
import sys
from collections import defaultdict

from pmc_traffic import classify

MIN_MS = 0.3


def main():
    cdir, tdir = sys.argv[1:3]
    act, n = defaultdict(float), defaultdict(int)
    for r in csv.DictReader(open(cdir + "/run_counter_collection.csv")):
        if r["Counter_Name"] != "GRBM_GUI_ACTIVE":
            continue
        c = classify(r["Kernel_Name"])
        if c:
            act[c] += float(r["Counter_Value"])
            n[c] += 1
    dur, m = defaultdict(float), defaultdict(int)
    for r in csv.DictReader(open(tdir + "/run_kernel_trace.csv")):
        c = classify(r["Kernel_Name"])
        if c:
            dur[c] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
            m[c] += 1
    print("%-18s %12s %12s %10s" % ("class", "GUI_ACTIVE", "avg ms", "clock GHz"))
    for c in sorted(act):
        if not m.get(c) or dur[c] / m[c] * 1e3 < MIN_MS:  # GUI_ACTIVE / duration is not a clock on short dispatches
            continue
        a, d = act[c] / n[c], dur[c] / m[c]
        print("%-18s %12.0f %12.4f %10.3f" % (c, a, d * 1e3, a / 8.0 / d / 1e9))


if __name__ == "__main__":
    main()
