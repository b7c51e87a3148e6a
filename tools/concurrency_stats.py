#!/usr/bin/env python3
"""Do concurrent batches stretch each other's kernels?  From a rocprofv3
kernel trace of a C5 run (tools/r5aa_step.sh): for the latency form's
kernels, the duration percentiles grouped by how many other verify kernels
overlapped each one on the device.

    python tools/concurrency_stats.py DIR_WITH_KERNEL_TRACE_CSV
"""
import collections
import csv
import glob
import json
import os
import sys

import numpy as np

NAMES = ("prep16", "dsm16", "txn_stage", "pull", "combine")


def short(name):
    for n in NAMES:
        if n in name:
            return n
    return None


def main():
    rows = []
    for f in glob.glob(os.path.join(sys.argv[1], "**", "*kernel_trace.csv"), recursive=True):
        with open(f) as fh:
            rows += list(csv.DictReader(fh))
    ks = []
    for r in rows:
        n = short(r["Kernel_Name"])
        if n:
            ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), n, int(r["Grid_Size_X"])))
    ks.sort()
    starts = np.array([k[0] for k in ks])
    ends = np.array([k[1] for k in ks])
    out = collections.defaultdict(lambda: collections.defaultdict(list))
    for i, (s, e, n, g) in enumerate(ks):
        # kernels whose [start, end) intersects this one's
        lo = np.searchsorted(starts, s - 10_000_000)
        hi = np.searchsorted(starts, e)
        ov = int(np.sum(ends[lo:hi] > s)) - 1
        out[n][min(ov, 4)].append((e - s) / 1e3)
    res = {}
    for n, d in out.items():
        res[n] = {}
        for ov in sorted(d):
            a = np.array(d[ov])
            res[n]["overlap_%d%s" % (ov, "+" if ov == 4 else "")] = {
                "count": int(a.size), "p50_us": round(float(np.percentile(a, 50)), 1),
                "p90_us": round(float(np.percentile(a, 90)), 1), "p99_us": round(float(np.percentile(a, 99)), 1)}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
