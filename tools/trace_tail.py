#!/usr/bin/env python
"""The dispatches of a rocprofv3 --kernel-trace CSV from the last one whose name matches PATTERN to the end (one call of
a multi-kernel entry point, e.g. the encoder's first-layer kernel), as start offset, duration, grid, workgroup, name.
usage: python tools/trace_tail.py run_kernel_trace.csv PATTERN ["title line"]"""
import csv
import re
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
hit = [i for i, r in enumerate(rows) if re.search(sys.argv[2], r["Kernel_Name"])]
if not hit:
    sys.exit("no dispatch matches %r" % sys.argv[2])
sel = rows[hit[-1]:]
t0 = int(sel[0]["Start_Timestamp"])
if len(sys.argv) > 3:
    print("# " + sys.argv[3])
print("# columns: start us, duration us, grid, workgroup, kernel")
busy = 0.0
for r in sel:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    busy += (e - s) / 1e3
    grid = "(%s,%s,%s)" % (r["Grid_Size_X"], r["Grid_Size_Y"], r["Grid_Size_Z"])
    print("%8.1f %7.1f  grid=%-18s wg=%-4s %s" % ((s - t0) / 1e3, (e - s) / 1e3, grid, r["Workgroup_Size_X"],
                                                 r["Kernel_Name"][:110]))
print("# span %.1f us, kernel time %.1f us, %d dispatches" % ((int(sel[-1]["End_Timestamp"]) - t0) / 1e3, busy, len(sel)))
