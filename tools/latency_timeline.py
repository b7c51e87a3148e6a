#!/usr/bin/env python3
"""Per-batch GPU timeline of a C5 latency run from rocprofv3 CSV traces
(kernel_trace.csv, memory_copy_trace.csv): for each batch, the H2D copy,
each kernel and the D2H copy (a small one runs as the runtime's blit
kernel, __amd_rocclr_copyBuffer) in stream order, and the gaps between them
(where launch and dispatch overhead shows).

    python tools/latency_timeline.py DIR_WITH_CSVS
"""
import collections
import csv
import glob
import os
import sys

import numpy as np


def rows(pattern):
    out = []
    for f in glob.glob(pattern, recursive=True):
        with open(f) as fh:
            out += list(csv.DictReader(fh))
    return out


def main():
    d = sys.argv[1]
    ks = rows(os.path.join(d, "**", "*kernel_trace.csv"))
    cs = rows(os.path.join(d, "**", "*memory_copy_trace.csv"))
    ev = []
    for r in ks:
        name = r["Kernel_Name"].split("(")[0].replace("fd_ed25519_", "")
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name, r.get("Stream_Id", r.get("Queue_Id", ""))))
    for r in cs:
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Direction"], r.get("Stream_Id", "")))
    ev.sort()
    # a batch = H2D ... D2H on one stream
    by_stream = collections.defaultdict(list)
    for e in ev:
        by_stream[e[3]].append(e)
    seqs = collections.Counter()
    gaps = collections.defaultdict(list)
    durs = collections.defaultdict(list)
    spans = []
    for st, es in by_stream.items():
        cur = []
        for e in es:
            if "HOST_TO_DEVICE" in e[2] or "H2D" in e[2]:
                cur = [e]
                continue
            if not cur:
                continue
            cur.append(e)
            if "DEVICE_TO_HOST" in e[2] or "copyBuffer" in e[2]:   # small D2H copies run as a blit kernel
                names = tuple(x[2] for x in cur)
                seqs[names] += 1
                for a, b in zip(cur, cur[1:]):
                    gaps[(a[2], b[2])].append((b[0] - a[1]) / 1e3)
                for x in cur:
                    durs[x[2]].append((x[1] - x[0]) / 1e3)
                spans.append((cur[-1][1] - cur[0][0]) / 1e3)
                cur = []
    for s, c in seqs.most_common(3):
        print(c, "batches:", " -> ".join(s))
    print("durations (us, p50 / p90):")
    for k, v in durs.items():
        print(f"  {k:28s} {np.percentile(v, 50):8.1f} {np.percentile(v, 90):8.1f}  n={len(v)}")
    print("gaps (us, p50 / p90):")
    for k, v in gaps.items():
        print(f"  {k[0]:>24s} -> {k[1]:24s} {np.percentile(v, 50):8.1f} {np.percentile(v, 90):8.1f}")
    if spans:
        print(f"H2D start -> D2H end (us): p50 {np.percentile(spans, 50):.1f} p90 {np.percentile(spans, 90):.1f}")


if __name__ == "__main__":
    main()
