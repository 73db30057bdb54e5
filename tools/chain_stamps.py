#!/usr/bin/env python
"""Breakdown of the launch-based reverse-sweep chain from a DAMC_CHAIN_TRACE dump (per launch, per workgroup
start / end stamps at 100 MHz): median over the steps, per block, of the workgroup start spread, workgroup
lifetime, launch span (first start -> last end) and the gap from the previous launch's last end to this
launch's first start."""
import sys

import numpy as np

raw = open(sys.argv[1], "rb").read()
rows = int(np.frombuffer(raw[:8], dtype=np.int64)[0])
T = np.frombuffer(raw[8:], dtype=np.uint64).reshape(rows, 512, 8).astype(np.int64)
t = T[:, :, :2]
live = (t[:, :, 0] > 0) & (t[:, :, 1] > 0)
res = []
prev_end = None
for li in range(rows):
    m = live[li]
    if not m.any():
        prev_end = None
        continue
    st, en = t[li, m, 0], t[li, m, 1]
    gap = (st.min() - prev_end) * 10 if prev_end is not None else np.nan
    res.append((li % 7, m.sum(), (st.max() - st.min()) * 10, np.median(en - st) * 10, (en.max() - en.min()) * 10,
                (en.max() - st.min()) * 10, gap))
    prev_end = en.max()
r = np.array(res, dtype=np.float64)
print("launches %d; ns medians over steps" % rows)
print("block  WGs  start-spread  WG-life(med)  end-spread  span  gap-from-prev-end")
for j in range(7):
    q = r[r[:, 0] == j]
    print("%5d %4d %13.0f %13.0f %11.0f %5.0f %18.0f" % (j, q[0, 1], *(np.nanmedian(q[:, i]) for i in range(2, 7))))
tot = r[:, 5].sum() + np.nansum(r[:, 6])
print("per step: spans %.2f us + gaps %.2f us" % (r[:, 5].sum() / 1e3 / (rows / 7), np.nansum(r[:, 6]) / 1e3 / (rows / 7)))

# shader-clock segments inside a workgroup (cycles): entry -> loads waited (dbg 1024 only), -> reduced, -> end
seg = []
for li in range(rows):
    m = live[li]
    if not m.any():
        continue
    c = T[li, m, 2:6]
    ld = np.median(c[:, 1] - c[:, 0]) if (c[:, 1] > 0).all() else np.nan
    red = np.median(c[:, 2] - (c[:, 1] if (c[:, 1] > 0).all() else c[:, 0]))
    seg.append((li % 7, ld, red, np.median(c[:, 3] - c[:, 2]), np.median(c[:, 3] - c[:, 0])))
g = np.array(seg, dtype=np.float64)
print("block  cycles: entry->loads  ->reduced  ->end  total")
for j in range(7):
    q = g[g[:, 0] == j]
    print("%5d  %18.0f %10.0f %6.0f %6.0f" % (j, *(np.nanmedian(q[:, i]) for i in range(1, 5))))

# wave launch skew inside a workgroup: waves 1 and 3 entry minus wave 0 entry (shader clock)
sk = []
for li in range(rows):
    m = live[li]
    if not m.any():
        continue
    c = T[li, m]
    sk.append((li % 7, np.median(c[:, 6] - c[:, 2]), np.median(c[:, 7] - c[:, 2]), np.max(c[:, 7] - c[:, 2])))
g = np.array(sk, dtype=np.float64)
print("block  wave1-wave0  wave3-wave0 (median, max) cycles")
for j in range(7):
    q = g[g[:, 0] == j]
    print("%5d  %11.0f  %11.0f %8.0f" % (j, *(np.median(q[:, i]) for i in range(1, 4))))
