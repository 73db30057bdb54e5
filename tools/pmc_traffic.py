#!/usr/bin/env python
"""Per-kernel-class HBM traffic from rocprofv3 --pmc passes (FETCH_SIZE and WRITE_SIZE collected in
SEPARATE runs, as MI355X_MICROARCH.md §HBM prescribes).  gfx950 corrections applied:
FETCH_SIZE counts exactly half of a wide coalesced streaming read -> x2; WRITE_SIZE is exact for
16-B streaming stores (our epilogues store 4 B/lane rows: uncalibrated, reported as read).
Units: both counters are KiB -> bytes x 1024.

usage: tools/pmc_traffic.py FETCH_DIR WRITE_DIR OUT_JSON
"""
import csv
import json
import re
import sys
from collections import defaultdict

CLASSES = [
    (r"gemm_x3_kernel<2, 0", "upconv_dgrad"),
    (r"gemm_x3_kernel<1, 1", "upconv_fwd"),
    (r"gemm_x3_kernel<1, 0", "proj_fwd"),
    (r"split_x3_kernel", "split_x3"),
    (r"gemm_km_kernel<2, 0", "upconv_dgrad"),
    (r"gemm_km_kernel<1, 1", "upconv_fwd"),
    (r"gemm_f32_kernel<1, 2, 0", "upconv_dgrad"),
    (r"gemm_f32_kernel<1, 1, 1", "upconv_fwd"),
    (r"gemm_f32_kernel<0, 1, 0", "proj_fwd"),
    (r"gemm_f32_kernel<0, 0, 0", "proj_dgrad"),
    (r"smallc_fwd", "smallc_fwd"),
    (r"smallc_dgrad", "smallc_dgrad"),
    (r"slab_sum_kernel", "slab_sum"),
    (r"posterior_update_kernel", "posterior_update"),
    (r"prior_chain_kernel", "prior_chain"),
]


def classify(name):
    for pat, cls in CLASSES:
        if re.search(pat, name):
            return cls
    return None


def per_class(path, counter):
    tot, n = defaultdict(float), defaultdict(int)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        c = classify(r["Kernel_Name"])
        if c:
            tot[c] += float(r["Counter_Value"])
            n[c] += 1
    return {c: tot[c] / n[c] for c in tot}


def main():
    fdir, wdir, out = sys.argv[1:4]
    f = per_class(fdir + "/run_counter_collection.csv", "FETCH_SIZE")
    w = per_class(wdir + "/run_counter_collection.csv", "WRITE_SIZE")
    res = {}
    for c in sorted(set(f) | set(w)):
        rd = 2.0 * f.get(c, 0.0) * 1024
        wr = w.get(c, 0.0) * 1024
        res[c] = dict(fetch_bytes_per_launch=rd, fetch_size_uncorrected_bytes=f.get(c, 0.0) * 1024,
                      write_bytes_per_launch=wr, hbm_bytes_per_launch=rd + wr,
                      correction="FETCH_SIZE x2 (gfx950 half-count), KiB->B")
    json.dump(res, open(out, "w"), indent=1)
    for c, v in res.items():
        print("%-18s read %8.1f MB (FETCH_SIZE %8.1f MB x2)  write %8.1f MB" % (
            c, v["fetch_bytes_per_launch"] / 1e6, v["fetch_size_uncorrected_bytes"] / 1e6,
            v["write_bytes_per_launch"] / 1e6))


if __name__ == "__main__":
    main()
