#!/usr/bin/env python
"""Summarise a rocprofv3 kernel_stats.csv: name, calls, average us, share of total.  usage: kstats.py csv [n]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 30
tot = sum(float(x["TotalDurationNs"]) for x in rows)
print(f"total {tot / 1e6:.3f} ms")
for x in rows[:n]:
    print(f"{x['Name'][:96]:96s} {x['Calls']:>6} {float(x['AverageNs']) / 1e3:9.1f} us {float(x['TotalDurationNs']) / tot * 100:5.1f} %")
