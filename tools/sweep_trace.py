#!/usr/bin/env python
"""Per-stage timing of the persistent reverse-sweep chain from a DAMC_SWEEP_TRACE dump (100 MHz stamps):
for every stage (step k, block j) the last publish of the previous stage, the first / last wait end and the
last publish, summarised as medians over the steps."""
import sys

import numpy as np

raw = open(sys.argv[1], "rb").read()
P, n, G = np.frombuffer(raw[:12], dtype=np.int32)
t = np.frombuffer(raw[12:], dtype=np.uint64).reshape(P, 7 * n, 3).astype(np.int64)
base = t[t > 0].min()
t = np.where(t > 0, t - base, -1) * 10  # ns
S = 7 * n
stage_pub = np.array([t[:, s, 2][t[:, s, 2] >= 0].max() if (t[:, s, 2] >= 0).any() else -1 for s in range(S)])
rows = []
for s in range(1, S):
    live = t[:, s, 1] >= 0
    if not live.any():
        continue
    wend = t[live, s, 1]
    wbeg = t[live, s, 0]
    pub = t[live, s, 2]
    rows.append((s % 7, stage_pub[s] - stage_pub[s - 1], wend.min() - stage_pub[s - 1], wend.max() - stage_pub[s - 1],
                 np.median(pub - wend), np.median(wend - wbeg)))
r = np.array(rows, dtype=np.float64)
print("P=%d n=%d G=%d  total %.1f us  (%.2f us/step)" % (P, n, G, (stage_pub.max()) / 1e3, stage_pub.max() / 1e3 / n))
print("block  stage(us)  first-wake  last-wake  compute(med)  wait(med)   [us after the previous stage's last publish]")
for j in range(7):
    q = r[r[:, 0] == j]
    print("%5d  %9.2f  %10.2f  %9.2f  %12.2f  %9.2f" % (j, *(np.median(q[:, i]) / 1e3 for i in range(1, 6))))
