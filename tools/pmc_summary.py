#!/usr/bin/env python3
"""Summarize rocprofv3 --pmc CSV outputs (one directory per pass) into one
JSON per kernel: counters averaged per dispatch, plus derived numbers.

  python tools/pmc_summary.py OUT.json DIR [DIR ...] [--n SIGS_PER_DISPATCH]

FETCH_SIZE / WRITE_SIZE are in KB (rocprofv3).  On gfx950 FETCH_SIZE reads
half the bytes of a wide coalesced stream (MI355X_MICROARCH.md §HBM); both
the raw value and the x2 upper bound are reported."""
import collections
import csv
import glob
import json
import os
import re
import sys


def main():
    args = sys.argv[1:]
    n = None
    if "--n" in args:
        i = args.index("--n")
        n = int(args[i + 1])
        del args[i:i + 2]
    out, dirs = args[0], args[1:]
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(lambda: collections.defaultdict(set))
    meta = {}
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                # "void fd_ed25519_dsm_kernel<24>(...)" -> fd_ed25519_dsm_kernel
                # (the template argument is the base-table radix)
                k = re.sub(r"<[^>]*>$", "", re.sub(r"^void ", "", r["Kernel_Name"].split("(")[0]))
                c = r["Counter_Name"]
                agg[k][c] += float(r["Counter_Value"])
                disp[k][c].add((f, r["Dispatch_Id"]))
                meta[k] = {"vgpr": int(r["VGPR_Count"]), "agpr": int(r.get("Accum_VGPR_Count", 0) or 0),
                           "sgpr": int(r["SGPR_Count"]), "lds": int(r["LDS_Block_Size"]),
                           "scratch": int(r["Scratch_Size"]), "workgroup": int(r["Workgroup_Size"])}
    res = {}
    for k, cs in agg.items():
        per = {c: v / max(len(disp[k][c]), 1) for c, v in cs.items()}
        d = {"per_dispatch": per, "meta": meta.get(k)}
        if "FETCH_SIZE" in per:
            d["hbm_read_bytes"] = per["FETCH_SIZE"] * 1024
            d["hbm_read_bytes_x2_upper"] = per["FETCH_SIZE"] * 2048
        if "WRITE_SIZE" in per:
            d["hbm_write_bytes"] = per["WRITE_SIZE"] * 1024
        if n and k in ("fd_ed25519_dsm_kernel", "fd_ed25519_hash_kernel", "fd_ed25519_decode_kernel"):
            lanes = n
        else:
            lanes = None
        if lanes:
            d["signatures_per_dispatch"] = n
            for c in ("SQ_INSTS_VALU", "SQ_INSTS_VALU_INT32", "SQ_INSTS_VALU_INT64"):
                if c in per:
                    d[c + "_per_signature"] = per[c] * 64 / n
            if "hbm_read_bytes" in d:
                d["hbm_read_bytes_per_signature"] = d["hbm_read_bytes"] / n
            if "hbm_write_bytes" in d:
                d["hbm_write_bytes_per_signature"] = d["hbm_write_bytes"] / n
        res[k] = d
    with open(out, "w") as f:
        json.dump(res, f, indent=1, sort_keys=True)
    for k, d in sorted(res.items()):
        print(k, {x: round(y, 1) for x, y in d.items() if isinstance(y, float)})


if __name__ == "__main__":
    main()
