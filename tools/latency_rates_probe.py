#!/usr/bin/env python3
"""The in-process latency mode (C5's vtile + ring, no processes or shared-
memory links) at fixed offered rates from the reference tile's load to the
GPU path's: p50 / p99 and the mean batch size at each, to separate the GPU
round trip from the deployed path's host chain (run on the box).

    python tools/latency_rates_probe.py [--rates 28000,57000,570000,2400000] [--txns 40000] [--slots 8]
"""
import argparse
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rates", default="28000,57000,570000,2400000")
    ap.add_argument("--txns", type=int, default=40000)
    ap.add_argument("--slots", type=int, default=8)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--runs", type=int, default=3)
    ap.add_argument("--host-scalars", default=None,
                    help="comma list of fd_ed25519_hip_pipe_set_host_scalars values to sweep (default: the library's)")
    ap.add_argument("--host-decode", default=None,
                    help="comma list of fd_ed25519_hip_pipe_set_host_decode values to sweep (default: the library's)")
    ap.add_argument("--split", type=int, default=None, help="fd_ed25519_hip_pipe_set_split_waves (A/B: 2, 4, 8)")
    ap.add_argument("--pin", action="store_true", help="producer and tile on two physical cores of the GPU's node")
    args = ap.parse_args()
    os.environ.setdefault("GPU_MAX_HW_QUEUES", str(args.slots))
    from firedancer_amd import ed25519, tile, workload
    eng = ed25519.Engine(0, max_chunk=1 << 16)
    pay, _ = workload.txn_payloads(eng, args.txns, 4242, msg_sz=200)
    if args.pin:
        cores = tile.physical_cores(tile.device_cpus(eng.info()))
        tile.latency_set_cpus(cores[0], cores[1])
    eng.close()
    if args.split is not None:
        tile.pipe_set_split_waves(args.split)
    hs_values = [None] if args.host_scalars is None else [int(x) for x in args.host_scalars.replace(":", ",").split(",")]
    hd_values = [None] if args.host_decode is None else [int(x) for x in args.host_decode.replace(":", ",").split(",")]
    for hs, hd, rate in [(h, d, float(r)) for h in hs_values for d in hd_values
                         for r in args.rates.replace(":", ",").split(",")]:
        if hs is not None:
            tile.pipe_set_host_scalars(hs)
        if hd is not None:
            tile.pipe_set_host_decode(hd)
        pooled, batches, achieved = [], 0, []
        for _ in range(args.runs):
            n = min(args.txns, max(2000, int(rate * 0.5))) if rate > 0 else args.txns
            lat, v, res = tile.latency_run(pay[:n] if isinstance(pay, list) else pay, rate, slot_cnt=args.slots,
                                           batch_sigs=args.batch, ring_depth=4096)
            pooled.append(lat * 1e3)
            batches += res["batches"]
            achieved.append(res["achieved_txn_per_s"])
        ms = np.concatenate(pooled)
        print(json.dumps({"host_scalars": hs, "host_decode": hd, "rate": rate, "txns": int(ms.size), "p50_ms": float(np.percentile(ms, 50)),
                          "p99_ms": float(np.percentile(ms, 99)), "mean_batch": ms.size / max(batches, 1),
                          "achieved_txn_per_s": float(np.mean(achieved))}), flush=True)


if __name__ == "__main__":
    main()
