#!/usr/bin/env python
"""Per-block median duration of the reverse sweep's chain kernels from a rocprofv3 kernel trace."""
import collections
import csv
import sys

rows = [r for r in csv.DictReader(open(sys.argv[1])) if "chain_kernel" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
pat = None
per = collections.defaultdict(list)
gaps = []
for i, r in enumerate(rows):
    per[i % 7].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    if i:
        gaps.append(int(r["Start_Timestamp"]) - int(rows[i - 1]["End_Timestamp"]))
for k in sorted(per):
    v = sorted(per[k])
    print("block %d: n=%d median %.2f us  p10 %.2f  p90 %.2f" % (k, len(v), v[len(v) // 2] / 1e3, v[len(v) // 10] / 1e3,
                                                            v[9 * len(v) // 10] / 1e3))
g = sorted(gaps)
print("gap between chain kernels: median %.2f us  p10 %.2f  p90 %.2f" % (g[len(g) // 2] / 1e3, g[len(g) // 10] / 1e3,
                                                                      g[9 * len(g) // 10] / 1e3))
