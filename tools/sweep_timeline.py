#!/usr/bin/env python
"""Per-workgroup timeline of the one-launch reverse sweep from a DAMC_SWEEP_TRACE dump (data-driven hand-off:
stamps {task start, wake, reduced, published} per task): the median gaps of each slot of one team, in us:
publish -> next task start (loop overhead), start -> wake (task setup), wake -> reduced, reduced -> published.
usage: python tools/sweep_timeline.py trace.bin [team]"""
import sys

import numpy as np

raw = open(sys.argv[1], "rb").read()
P, n, G = np.frombuffer(raw[:12], dtype=np.int32)
t = np.frombuffer(raw[12:], dtype=np.uint64).reshape(P, 7 * n, 4).astype(np.int64)
t = np.where(t > 0, t, -1)
team = int(sys.argv[2]) if len(sys.argv) > 2 else 0
print("wg  slot tasks  per-step  pub->start start->wake wake->red red->pub   (us, medians over the slot's tasks)")
for b in range(team, P, 8):
    tt = t[b]
    live = [s for s in range(7 * n) if tt[s, 1] >= 0]
    if len(live) < 2:
        continue
    g = np.array([(tt[live[i + 1], 0] - tt[s, 3], tt[s, 1] - tt[s, 0], tt[s, 2] - tt[s, 1], tt[s, 3] - tt[s, 2])
                  for i, s in enumerate(live[:-1])], dtype=np.float64) / 100
    span = (tt[live[-1], 3] - tt[live[0], 0]) / 100
    print("%3d  %4d %5d  %8.2f  %9.2f %10.2f %9.2f %7.2f" % (b, b // 8, len(live), span / n,
                                                              *np.median(g, axis=0)))
