#!/usr/bin/env python3
"""Per-phase time of one verify launch at small batch sizes (the verify
tile's latency regime, C5): where a batch spends its time, over many
different batches (the share of batches holding a signature that needs the
longer dsm form shows up in the upper percentiles).

    python tools/small_batch_probe.py [--sizes 64,256,1024,4096,16384] [--batches 40] [--half extended|strict]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from firedancer_amd import ed25519  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="64,256,1024,4096,16384")
    ap.add_argument("--batches", type=int, default=40)
    ap.add_argument("--msg", type=int, default=200)
    ap.add_argument("--half", default="extended")
    ap.add_argument("--dsm", default="auto")
    ap.add_argument("--forms", default=None, help="quad_max,oct_max (0,0: the one-lane phase kernels)")
    args = ap.parse_args()
    forms = tuple(int(x) for x in args.forms.split(",")) if args.forms else None
    eng = ed25519.Engine(0, max_chunk=1 << 16, half=args.half, dsm=args.dsm, forms=forms)
    for n in [int(x) for x in args.sizes.split(",")]:
        wall, dsm, other, phases = [], [], [], []
        for b in range(args.batches):
            w = ed25519.DeviceWorkload(eng, n, args.msg, args.msg, 0, seed=1000 + b)
            w.verify()
            eng.sync()
            eng.timing(True)
            eng.timing_read()
            t0 = time.perf_counter()
            w.verify()
            eng.sync()
            wall.append((time.perf_counter() - t0) * 1e3)
            ph, cnt = eng.timing_read()
            eng.timing(False)
            dsm.append(ph["dsm"])
            phases.append(ph)
            other.append(ph["hash"] + ph["scalar"] + ph["decode"])
            w.free()
        pct = lambda a, q: float(np.percentile(np.array(a), q))  # noqa: E731
        print(json.dumps({"n": n, "half": args.half, "dsm": args.dsm, "batches": args.batches,
                          "wall_ms": {"p50": pct(wall, 50), "p90": pct(wall, 90), "max": max(wall)},
                          "dsm_ms": {"p50": pct(dsm, 50), "p90": pct(dsm, 90), "max": max(dsm)},
                          "hash_scalar_decode_ms_p50": pct(other, 50),
                          "phase_ms_p50": {k: pct([q[k] for q in phases], 50) for k in phases[0]}}), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
