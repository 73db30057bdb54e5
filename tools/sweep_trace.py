#!/usr/bin/env python
"""Per-stage timing of the one-launch reverse sweep from a DAMC_SWEEP_TRACE dump (100 MHz stamps per workgroup
and stage: wait begin, wait end, reduced, published).  Workgroup b belongs to team b % 8 (sweep_team_kernel); every
quantity is taken within a team, relative to that team's last publish of the previous stage, then the median
over teams and steps is printed per block."""
import sys

import numpy as np

raw = open(sys.argv[1], "rb").read()
P, n, G = np.frombuffer(raw[:12], dtype=np.int32)
t = np.frombuffer(raw[12:], dtype=np.uint64).reshape(P, 7 * n, 4).astype(np.int64)
base = t[t > 0].min()
t = np.where(t > 0, t - base, -1) * 10  # ns
S = 7 * n
rows = []
span = []
for team in range(min(8, G)):
    tt = t[team::8]
    pub = np.array([tt[:, s, 3][tt[:, s, 3] >= 0].max() if (tt[:, s, 3] >= 0).any() else -1 for s in range(S)])
    span.append(pub.max() - tt[:, :, 0][tt[:, :, 0] >= 0].min())
    for s in range(1, S):
        live = tt[:, s, 1] >= 0
        if not live.any() or pub[s - 1] < 0:
            continue
        wend, wbeg, red, p = tt[live, s, 1], tt[live, s, 0], tt[live, s, 2], tt[live, s, 3]
        rows.append((s % 7, pub[s] - pub[s - 1], wend.min() - pub[s - 1], wend.max() - pub[s - 1],
                     np.median(red - wend), np.median(p - red), np.median(wend - wbeg)))
r = np.array(rows, dtype=np.float64)
print("P=%d n=%d G=%d  team span median %.1f us (%.2f us/step)" % (P, n, G, np.median(span) / 1e3,
                                                                   np.median(span) / 1e3 / n))
print("block  stage(us)  first-wake  last-wake  ->reduced  ->published  wait(med)   [us after the team's previous publish]")
for j in range(7):
    q = r[r[:, 0] == j]
    print("%5d  %9.2f  %10.2f  %9.2f  %9.2f  %11.2f  %9.2f" % (j, *(np.median(q[:, i]) / 1e3 for i in range(1, 7))))
