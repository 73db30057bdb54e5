#!/usr/bin/env python
"""One posterior Langevin step's dispatches from a rocprofv3 --kernel-trace CSV (run_kernel_trace.csv): the dispatches
after the second-to-last posterior update kernel (ebm_reg_kernel<1> / the MFMA update) up to and including the last
one, as start offset, duration, grid, workgroup size and kernel name, plus the step's span and kernel-time sum.
usage: python tools/dispatch_list.py run_kernel_trace.csv ["title line"]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
upd = [i for i, r in enumerate(rows) if "ebm_reg_kernel<1>" in r["Kernel_Name"] or "posterior_update" in r["Kernel_Name"]]
if len(upd) < 2:
    sys.exit("fewer than two posterior update dispatches in the trace")
sel = rows[upd[-2] + 1: upd[-1] + 1]
t0 = int(sel[0]["Start_Timestamp"])
if len(sys.argv) > 2:
    print("# " + sys.argv[2])
print("# columns: start us, duration us, grid, workgroup, kernel")
busy = 0.0
for r in sel:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    busy += (e - s) / 1e3
    grid = "(%s,%s,%s)" % (r["Grid_Size_X"], r["Grid_Size_Y"], r["Grid_Size_Z"])
    print("%8.1f %7.1f  grid=%-18s wg=%-4s %s" % ((s - t0) / 1e3, (e - s) / 1e3, grid, r["Workgroup_Size_X"],
                                                 r["Kernel_Name"][:100]))
span = (int(sel[-1]["End_Timestamp"]) - t0) / 1e3
print("# step span %.1f us, kernel time %.1f us, %d dispatches" % (span, busy, len(sel)))
